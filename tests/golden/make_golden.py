"""Generate the committed synthetic golden vectors (tests/golden/synthetic.npz + cases.json).

Encoded inputs are produced by independent encoders where one exists (Python's zlib for gzip,
numpy for transpose/byte order/shuffle, hand-built shard layouts), and by libzstd (through the
oracle) for zstd. Every expected decoded output is computed here with numpy/zlib, and is also
checked against the oracle before it is written — so the goldens pin BOTH the oracle and the GPU
path. Run from the repo root:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import json
import os
import struct
import sys
import zlib

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402

rng = np.random.default_rng(20240611)
cases = []
arrays = {}


def add(name, codecs, data_type, shape, enc: bytes, dec: np.ndarray | None, status=0, fill=0,
        sel=None):
    arrays[name + "/enc"] = np.frombuffer(enc, dtype=np.uint8).copy()
    if dec is not None:
        arrays[name + "/dec"] = np.ascontiguousarray(dec)
    cases.append(dict(name=name, codecs=codecs, data_type=data_type, shape=list(shape), status=status,
                      fill_value=fill, sel=sel))
    # self-check against the oracle
    try:
        ch = O.OracleChain.from_metadata(codecs, data_type, fill, len(shape))
        if sel is None:
            got = ch.decode(enc, shape)
        else:
            got = O.retrieve_array_subset(ch, shape, shape, {tuple([0] * len(shape)): enc}, sel[0], sel[1])
        assert status == 0, f"{name}: oracle decoded but status {status} expected"
        assert np.array_equal(got.view(np.uint8), np.ascontiguousarray(dec).view(np.uint8)), name
    except O.OracleError as e:
        assert e.status == status, f"{name}: oracle status {e.status} != {status}"


def gz(data: bytes, level: int) -> bytes:
    c = zlib.compressobj(level, zlib.DEFLATED, 31)
    return c.compress(data) + c.flush()


BYTES_LE = {"name": "bytes", "configuration": {"endian": "little"}}
BYTES_BE = {"name": "bytes", "configuration": {"endian": "big"}}

# 1. config-2 chain (transpose [2,1,0] + bytes big endian), f32
for shape in ([4, 5, 6], [16, 16, 16], [3, 64, 7]):
    dec = rng.standard_normal(shape).astype(np.float32)
    enc = np.ascontiguousarray(dec.transpose(2, 1, 0)).astype(">f4").tobytes()
    add("c2_%s" % "x".join(map(str, shape)),
        [{"name": "transpose", "configuration": {"order": [2, 1, 0]}}, BYTES_BE], "float32", shape, enc, dec)
# other permutations and dtypes
for order, dt, shape in (([1, 0], "uint16", [9, 70]), ([0, 2, 1], "float64", [3, 17, 5]),
                         ([1, 2, 0], "int32", [6, 7, 8]), ([2, 0, 1], "uint8", [5, 66, 3]),
                         ([3, 1, 0, 2], "float32", [2, 3, 4, 5])):
    npdt = np.dtype(O.DTYPES[dt][0])
    dec = rng.integers(0, 1 << min(30, 8 * npdt.itemsize - 1), size=shape).astype(npdt) if npdt.kind != "f" \
        else rng.standard_normal(shape).astype(npdt)
    for big in (False, True):
        enc = np.ascontiguousarray(dec.transpose(order)).astype(npdt.newbyteorder(">" if big else "<")).tobytes()
        add("tr_%s_%s_%s" % ("".join(map(str, order)), dt, "be" if big else "le"),
            [{"name": "transpose", "configuration": {"order": order}}, BYTES_BE if big else BYTES_LE],
            dt, shape, enc, dec)
# complex64 (component size 4): big endian swaps each 4-byte component
dec = (rng.standard_normal((5, 7)) + 1j * rng.standard_normal((5, 7))).astype(np.complex64)
add("complex64_be", [BYTES_BE], "complex64", [5, 7], dec.astype(">c8").tobytes(), dec)

# 2. crc32c
for n in (0, 6, 1000, 65536 + 13):
    data = bytes(((i * 31 + 7) & 255) for i in range(n)) if n != 6 else bytes(range(6))
    dec = np.frombuffer(data, dtype=np.uint8).copy()
    crc = O.crc32c(data)
    if n == 6:
        assert crc.to_bytes(4, "little") == bytes([20, 133, 9, 65])  # crc32c.rs:126 KAT
    add("crc32c_%d" % n, [BYTES_LE, {"name": "crc32c"}], "uint8", [n], data + crc.to_bytes(4, "little"),
        dec)
    add("crc32c_start_%d" % n, [BYTES_LE, {"name": "crc32c", "configuration": {"location": "start"}}],
        "uint8", [n], crc.to_bytes(4, "little") + data, dec)

# 3. gzip (python zlib encoder; decoded by zlib too)
mix = np.concatenate([rng.integers(0, 255, 20000, dtype=np.uint8),
                      np.repeat(rng.integers(0, 255, 300, dtype=np.uint8), 50),
                      np.frombuffer(b"zarrs chunk decode " * 1000, dtype=np.uint8)])
for level in (0, 1, 5, 9):
    data = mix.tobytes()
    enc = gz(data, level)
    assert zlib.decompress(enc, 31) == data
    add("gzip_l%d" % level, [BYTES_LE, {"name": "gzip", "configuration": {"level": level}}], "uint8",
        [len(data)], enc, mix)
f = (np.arange(32 * 32 * 32, dtype=np.float32) * 0.25).reshape(32, 32, 32)
for level in (1, 6):
    add("gzip_f32_l%d" % level, [BYTES_LE, {"name": "gzip", "configuration": {"level": level}}], "float32",
        [32, 32, 32], gz(f.tobytes(), level), f)
small = np.arange(10, dtype=np.uint8)
add("gzip_tiny", [BYTES_LE, {"name": "gzip", "configuration": {"level": 6}}], "uint8", [10],
    gz(small.tobytes(), 6), small)
# fixed-Huffman-only stream (zlib Z_FIXED strategy)
c = zlib.compressobj(6, zlib.DEFLATED, 31, 8, zlib.Z_FIXED)
add("gzip_fixed", [BYTES_LE, {"name": "gzip", "configuration": {"level": 6}}], "uint8", [len(mix)],
    c.compress(mix.tobytes()) + c.flush(), mix)

# 4. zstd (libzstd through the oracle encoder; expected output is the plaintext)
for level in (1, 3, 19):
    ch = O.OracleChain.from_metadata([BYTES_LE, {"name": "zstd", "configuration": {"level": level,
                                      "checksum": level == 19}}], "uint8", 0, 1)
    add("zstd_l%d" % level, ch.codecs if hasattr(ch, "codecs") else
        [BYTES_LE, {"name": "zstd", "configuration": {"level": level, "checksum": level == 19}}], "uint8",
        [len(mix)], ch.encode(mix), mix)
u16 = (100 + 40 * np.sin(np.arange(64 * 64) / 50.0)).astype(np.uint16).reshape(64, 64)
zc = [BYTES_LE, {"name": "numcodecs.shuffle", "configuration": {"elementsize": 2}},
      {"name": "zstd", "configuration": {"level": 3, "checksum": False}}]
add("shuffle_zstd_u16", zc, "uint16", [64, 64], O.OracleChain.from_metadata(zc, "uint16", 0, 2).encode(u16), u16)

# 5. shuffle (numpy encoder)
for es, dt in ((2, "uint16"), (4, "float32"), (8, "float64")):
    dec = rng.standard_normal(257).astype(np.dtype(O.DTYPES[dt][0])) if dt != "uint16" else \
        rng.integers(0, 65535, 257).astype(np.uint16)
    enc = dec.view(np.uint8).reshape(-1, es).T.copy().tobytes()
    add("shuffle_%s" % dt, [BYTES_LE, {"name": "numcodecs.shuffle", "configuration": {"elementsize": es}}],
        dt, [257], enc, dec)
# shuffle elementsize != dtype size (not fused: standalone unshuffle)
dec = rng.integers(0, 65535, 256).astype(np.uint16)
add("shuffle_es4_u16", [BYTES_LE, {"name": "numcodecs.shuffle", "configuration": {"elementsize": 4}}],
    "uint16", [256], dec.view(np.uint8).reshape(-1, 4).T.copy().tobytes(), dec)


# 6. hand-built shards: u16 [8,8], inner [4,4], inner codecs [bytes, crc32c]
def shard(dec, inner, order, empty, at_start, inner_codecs="crc"):
    cps = [s // i for s, i in zip(dec.shape, inner)]
    n = cps[0] * cps[1]
    idx_len = n * 16 + 4
    body, index = b"", [0] * (2 * n)
    base = idx_len if at_start else 0
    for k in order:
        if k in empty:
            index[2 * k] = index[2 * k + 1] = (1 << 64) - 1
            continue
        r, c = divmod(k, cps[1])
        blk = dec[r * inner[0]:(r + 1) * inner[0], c * inner[1]:(c + 1) * inner[1]].astype("<u2").tobytes()
        if inner_codecs == "crc":
            blk = blk + O.crc32c(blk).to_bytes(4, "little")
        index[2 * k], index[2 * k + 1] = base + len(body), len(blk)
        body += blk
    for k in empty:
        index[2 * k] = index[2 * k + 1] = (1 << 64) - 1
    ib = struct.pack("<%dQ" % (2 * n), *index)
    ib += O.crc32c(ib).to_bytes(4, "little")
    return (ib + body) if at_start else (body + ib)


sdec = np.arange(64, dtype=np.uint16).reshape(8, 8) + 1000
for at_start in (False, True):
    loc = "start" if at_start else "end"
    codecs = [{"name": "sharding_indexed", "configuration": {
        "chunk_shape": [4, 4], "codecs": [BYTES_LE, {"name": "crc32c"}],
        "index_codecs": [BYTES_LE, {"name": "crc32c"}], "index_location": loc}}]
    exp = sdec.copy()
    exp[0:4, 4:8] = 7  # inner chunk 1 is empty -> fill value 7
    enc = shard(sdec, [4, 4], [3, 1, 2, 0], {1}, at_start)
    add("shard_%s" % loc, codecs, "uint16", [8, 8], enc, exp, fill=7)
    # partial selection of the shard: rows 2..7, cols 1..6
    add("shard_%s_partial" % loc, codecs, "uint16", [8, 8], enc, exp[2:8, 1:7], fill=7,
        sel=[[2, 1], [6, 6]])
    # errors: corrupted inner-chunk checksum (full path verifies, partial path only strips)
    bad = bytearray(enc)
    off0 = struct.unpack_from("<Q", bytes(enc), (len(enc) - 68 if not at_start else 0) + 0)[0]
    bad[off0 + 3] ^= 0xFF  # inner chunk 0 data byte
    exp_bad = exp.copy()
    exp_bad.view(np.uint8).reshape(8, 16)[0, 3] ^= 0xFF
    add("shard_%s_badcrc" % loc, codecs, "uint16", [8, 8], bytes(bad), None, status=1, fill=7)
    add("shard_%s_badcrc_partial" % loc, codecs, "uint16", [8, 8], bytes(bad), exp_bad[0:2, 0:8], fill=7,
        sel=[[0, 0], [2, 8]])
# index offset past the end of the shard -> SHARD_INDEX_OOB
codecs = [{"name": "sharding_indexed", "configuration": {
    "chunk_shape": [4, 4], "codecs": [BYTES_LE], "index_codecs": [BYTES_LE, {"name": "crc32c"}]}}]
enc = bytearray(shard(sdec, [4, 4], [0, 1, 2, 3], set(), False, inner_codecs="none"))
n_idx = 4 * 16
ib = bytearray(enc[-(n_idx + 4):-4])
struct.pack_into("<Q", ib, 16, len(enc) + 100)  # inner chunk 1 offset
enc[-(n_idx + 4):] = bytes(ib) + O.crc32c(bytes(ib)).to_bytes(4, "little")
add("shard_oob", codecs, "uint16", [8, 8], bytes(enc), None, status=3)
add("shard_too_small", codecs, "uint16", [8, 8], b"\x00" * 20, None, status=8)
add("crc_too_short", [BYTES_LE, {"name": "crc32c"}], "uint8", [0], b"\x01\x02", None, status=7)
cor = bytearray(gz(mix.tobytes(), 6))
cor[len(cor) // 2] ^= 0x55
add("gzip_corrupt", [BYTES_LE, {"name": "gzip", "configuration": {"level": 6}}], "uint8", [len(mix)],
    bytes(cor), None, status=4)
trl = bytearray(gz(mix.tobytes(), 6))
trl[-6] ^= 0x01  # trailer CRC-32 byte
add("gzip_bad_trailer", [BYTES_LE, {"name": "gzip", "configuration": {"level": 6}}], "uint8", [len(mix)],
    bytes(trl), None, status=4)
add("shuffle_len", [BYTES_LE, {"name": "numcodecs.shuffle", "configuration": {"elementsize": 4}}],
    "uint16", [3], b"\x00" * 6, None, status=9)
add("size_mismatch", [BYTES_LE], "float32", [4], b"\x00" * 12, None, status=2)

# 7. CodecChain::from_metadata (codec_chain.rs:192-229): a codec that cannot be created is skipped when
# "must_understand": false, an error otherwise; entries are sorted by kind, not by position
dec = np.arange(50, dtype=np.uint16) * 3
raw = dec.tobytes()
crc_enc = raw + O.crc32c(raw).to_bytes(4, "little")
add("must_understand_false_skipped",
    [BYTES_LE, {"name": "example.unknown_codec", "configuration": {"x": 1}, "must_understand": False},
     {"name": "crc32c"}], "uint16", [50], crc_enc, dec)
add("must_understand_default_true", [BYTES_LE, {"name": "example.unknown_codec"}], "uint16", [50], raw, None,
    status=6)
add("codecs_sorted_by_kind", [{"name": "crc32c"}, BYTES_LE], "uint16", [50], crc_enc, dec)

if __name__ == "__main__":
    np.savez_compressed(os.path.join(HERE, "synthetic.npz"), **arrays)
    json.dump(cases, open(os.path.join(HERE, "cases.json"), "w"), indent=1)
    print(len(cases), "cases;", sum(a.nbytes for a in arrays.values()), "bytes")
