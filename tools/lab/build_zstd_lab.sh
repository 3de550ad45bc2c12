#!/bin/bash
# Builds the zstd lab harness (plain, ZG_PROFILE and ZG_LIT_STATS variants). Not product code.
cd "$(dirname "$0")"
F="--offload-arch=gfx950 -O3 -std=c++17 -fopenmp -I../../zarrs_amd/csrc -x hip zstd_lab.cpp -L../synth -lsynth -Wl,-rpath,\$ORIGIN/../synth -l:libzstd.so.1"
hipcc $F -o zstd_lab && hipcc -DZG_LIT_STATS $F -o zstd_lab_stats
