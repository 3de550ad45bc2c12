"""Load the committed reference fixtures (tests/golden/ref/, copied from zarrs/tests/data) into
(metadata, {chunk grid index: encoded bytes}). V2 metadata is converted to the equivalent V3
codec chain the way zarrs does (zarrs/src/array/array_metadata_v2_to_v3 conversion):
order "F" -> transpose(reversed axes), compressor gzip/zstd -> b2b codec."""
from __future__ import annotations

import itertools
import json
import os

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
REF = os.path.join(GOLDEN, "ref")

V2_DTYPES = {"<f4": "float32", "<u2": "uint16", "<f8": "float64", "<i4": "int32"}


def load_array(rel: str):
    path = os.path.join(REF, rel)
    if os.path.exists(os.path.join(path, "zarr.json")):
        meta = json.load(open(os.path.join(path, "zarr.json")))
        shape = meta["shape"]
        chunk_shape = meta["chunk_grid"]["configuration"]["chunk_shape"]
        kenc = meta["chunk_key_encoding"]
        sep = kenc.get("configuration", {}).get("separator", "/" if kenc["name"] == "default" else ".")
        prefix = "c" + sep if kenc["name"] == "default" else ""
        codecs = meta["codecs"]
        data_type = meta["data_type"]
        fill = meta["fill_value"]
    else:
        z = json.load(open(os.path.join(path, ".zarray")))
        shape, chunk_shape = z["shape"], z["chunks"]
        sep = z.get("dimension_separator", ".")
        prefix = ""
        data_type = V2_DTYPES[z["dtype"]]
        fill = z["fill_value"]
        codecs = []
        if z.get("order", "C") == "F":
            codecs.append({"name": "transpose",
                           "configuration": {"order": list(range(len(shape)))[::-1]}})
        codecs.append({"name": "bytes", "configuration": {"endian": "little"}})
        comp = z.get("compressor")
        if comp:
            if comp["id"] == "gzip":
                codecs.append({"name": "gzip", "configuration": {"level": comp.get("level", 5)}})
            elif comp["id"] == "zstd":
                codecs.append({"name": "zstd", "configuration": {"level": comp.get("level", 0),
                                                                 "checksum": False}})
            elif comp["id"] == "blosc":  # zarrs_metadata_ext v2->v3 blosc: shuffle 0/1/2, typesize = dtype
                codecs.append({"name": "blosc", "configuration": {
                    "cname": comp["cname"], "clevel": comp["clevel"],
                    "shuffle": ["noshuffle", "shuffle", "bitshuffle"][comp.get("shuffle", 1)],
                    "typesize": int(z["dtype"][2:]), "blocksize": comp.get("blocksize", 0)}})
            else:
                raise ValueError(comp)
    grid = [-(-s // c) for s, c in zip(shape, chunk_shape)]
    chunks = {}
    for idx in itertools.product(*[range(g) for g in grid]):
        key = prefix + sep.join(str(i) for i in idx)
        f = os.path.join(path, key)
        if os.path.exists(f):
            chunks[idx] = open(f, "rb").read()
    return dict(shape=shape, chunk_shape=chunk_shape, codecs=codecs, data_type=data_type,
                fill_value=fill), chunks


# (fixture, expected decoded array as (numpy dtype, arange count, shape))
FLOAT_0_99 = [
    "v3/array_none.zarr", "v3/array_none_transpose.zarr", "v3/array_gzip.zarr", "v3/array_zstd.zarr",
    "v3_zarr_python/array_none.zarr", "v3_zarr_python/array_gzip.zarr",
    "v3_zarr_python/array_zstd.zarr",
    "v2/array_none_C.zarr", "v2/array_none_F.zarr", "v2/array_gzip_C.zarr", "v2/array_zstd_C.zarr",
]
SHARDED = "sharded_array_write_read.zarr/group/array"
# blosc fixtures (zstd + bitshuffle, typesize 4), also float32 0..99 (zarrs/src/array.rs:1684-1788)
BLOSC = ["v3/array_blosc.zarr", "v3/array_blosc_transpose.zarr", "v3_zarr_python/array_blosc.zarr",
         "v2/array_blosc_C.zarr", "v2/array_blosc_F.zarr"]
