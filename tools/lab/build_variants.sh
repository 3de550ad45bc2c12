#!/bin/bash
# Build libzgpu.so variants with different zstd kernel constants for A/B runs (ZGPU_LIB=<path>).
# Usage: tools/lab/build_variants.sh name:-DFLAG=V,-DFLAG2=V ...
set -e
cd "$(dirname "$0")/../../zarrs_amd/csrc"
make -s -j8
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}; flags=${flags//,/ }
  out=../lib_variants/$name; mkdir -p $out
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -munsafe-fp-atomics $flags -c kernels/${VFILE:-zstd}.hip -o $out/${VFILE:-zstd}.o
  objs=$(ls ../lib/obj/*.o | grep -v "/${VFILE:-zstd}.o$")
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $out/libzgpu.so $objs $out/${VFILE:-zstd}.o
  echo "built $out/libzgpu.so ($flags)"
done
