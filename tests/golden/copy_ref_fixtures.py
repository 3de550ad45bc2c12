"""Copy the reference's own golden fixture DATA (zarr.json/.zarray metadata + encoded chunk
files) from zarrs/tests/data into tests/golden/ref/. Run in the dev container only (the GPU box
has no /root/reference). These are data files, not source: zarr-python / zarrs wrote them and
zarrs' tests assert they decode to float32 0..99 (zarrs/src/array.rs:1684-1788) or to uint16
0..63 (zarrs/examples/sharded_array_write_read.rs)."""
import os
import shutil

SRC = "/root/reference/zarrs/tests/data"
DST = os.path.join(os.path.dirname(os.path.abspath(__file__)), "ref")
ARRAYS = [
    "v3/array_none.zarr", "v3/array_none_transpose.zarr", "v3/array_gzip.zarr",
    "v3/array_zstd.zarr",
    "v3_zarr_python/array_none.zarr", "v3_zarr_python/array_gzip.zarr",
    "v3_zarr_python/array_zstd.zarr",
    "v2/array_none_C.zarr", "v2/array_none_F.zarr", "v2/array_gzip_C.zarr",
    "v2/array_zstd_C.zarr",
    "sharded_array_write_read.zarr/group/array",
    # blosc (c-blosc 1.21 via blosc-src): zstd + bitshuffle, float32 0..99
    "v3/array_blosc.zarr", "v3/array_blosc_transpose.zarr", "v3_zarr_python/array_blosc.zarr",
    "v2/array_blosc_C.zarr", "v2/array_blosc_F.zarr",
]

if __name__ == "__main__":
    for a in ARRAYS:
        src = os.path.join(SRC, a)
        for root, _, files in os.walk(src):
            for f in files:
                if f == ".zattrs":
                    continue
                s = os.path.join(root, f)
                d = os.path.join(DST, os.path.relpath(s, SRC))
                os.makedirs(os.path.dirname(d), exist_ok=True)
                shutil.copyfile(s, d)
    print("copied to", DST)
