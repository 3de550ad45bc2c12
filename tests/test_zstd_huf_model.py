"""The zstd Huffman literal format the GPU encoder writes, pinned on the CPU: frames built by the
plain-Python model (tests/zstd_huf_model.py, RFC 8878 §3.1.1.3.1, §4.1.1, §4.2.1) decode with libzstd
(the oracle's zstd, zstd_codec.rs:113-130) to the exact bytes. CPU only."""
import numpy as np
import pytest

import oracle as O
import zstd_huf_model as M

ZS = [{"name": "bytes", "configuration": {"endian": "little"}}, {"name": "zstd", "configuration": {"level": 3}}]


def _decode(frame, n):
    return O.OracleChain.from_metadata(ZS, "uint8", 0, 1).decode(frame, [n]).tobytes()


def _cases():
    rng = np.random.default_rng(8)
    n = 20000
    geo = np.minimum(rng.geometric(0.08, n), 255).astype(np.uint8)           # skewed, < 128 mostly
    low = rng.integers(0, 100, n, dtype=np.uint8)                              # direct weights
    full = rng.integers(0, 256, n, dtype=np.uint8)                             # FSE weights, flat
    img = (128 + rng.normal(0, 18, n)).clip(0, 255).astype(np.uint8)          # FSE weights, bell
    fib = [1, 1]
    while len(fib) < 24:
        fib.append(fib[-1] + fib[-2])
    deep = rng.permutation(np.repeat(np.arange(24, dtype=np.uint8) * 11, fib))[:n]  # 11-bit limit
    two = rng.integers(0, 2, n, dtype=np.uint8) * 200                          # two symbols
    one = np.full(3000, 7, np.uint8)                                           # one symbol: raw
    mixed = np.concatenate([img[:5000], low[:3000], full[:4096], geo[:100]])   # treeless + not
    return {"geo": geo, "low": low, "full": full, "img": img, "deep": deep, "two": two, "one": one,
            "mixed": mixed}


@pytest.mark.parametrize("name", list(_cases()))
@pytest.mark.parametrize("block", [4096, 700, 64])
def test_literal_blocks_decode_with_libzstd(name, block):
    data = bytes(_cases()[name])
    frame = M.frame_of_literal_blocks(data, block)
    assert _decode(frame, len(data)) == data


def test_weight_descriptions_both_forms():
    """Both tree descriptions occur: direct 4-bit weights (max symbol <= 128) and FSE-compressed
    weights (a byte alphabet), and Huffman coding pays on skewed data."""
    c = _cases()
    small = np.repeat(np.arange(4, dtype=np.uint8), [900, 400, 200, 100])  # 3 weights: direct
    lens = M.huff_lengths(np.bincount(small, minlength=256).tolist(), M.HUF_MAX_BITS)
    assert M.huf_description(lens)[0] >= 128
    assert _decode(M.frame_of_literal_blocks(bytes(small)), len(small)) == bytes(small)
    lens = M.huff_lengths(np.bincount(c["img"], minlength=256).tolist(), M.HUF_MAX_BITS)
    d = M.huf_description(lens)
    assert d is not None and d[0] < 128
    frame = M.frame_of_literal_blocks(bytes(c["img"]))
    assert len(frame) < 0.8 * len(c["img"])


def test_huffman_lengths_are_complete_and_limited():
    rng = np.random.default_rng(1)
    for _ in range(300):
        n = int(rng.integers(2, 257))
        freq = (rng.pareto(0.7, n) * 10).astype(np.int64).tolist()
        freq[0] = max(freq[0], 1)
        freq[-1] = max(freq[-1], 1)
        lens = M.huff_lengths(freq, M.HUF_MAX_BITS)
        assert max(lens) <= M.HUF_MAX_BITS
        assert sum(2.0 ** -L for L in lens if L) == 1.0
