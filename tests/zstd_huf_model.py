"""Test infrastructure (not product code): a plain-Python model of the zstd Huffman literal sections
the GPU encoder writes (k_zstd_encode, zarrs_amd/csrc/kernels/zstd_enc.hip), restating RFC 8878
§3.1.1.3.1 (literals section header, Compressed / Treeless literal blocks, 1 or 4 streams with a jump
table), §4.2.1 (Huffman tree description: direct 4-bit weights or FSE-compressed weights) and §4.1.1
(FSE table description). tests/test_zstd_huf_model.py builds frames with it and decodes them with
libzstd (the oracle's zstd, the library zarrs' zstd codec wraps: zstd_codec.rs:113-130), so the
format the kernel follows is pinned on the CPU. Functions mirror the kernel's steps one to one."""
import numpy as np

HUF_MAX_BITS = 11  # Max_Number_of_Bits (RFC 8878 §4.2.1)
WEIGHT_LOG = 6     # FSE accuracy log of the weight table (libzstd HUF_compressWeights: <= 6)


class BitW:
    """Forward bit writer, LSB first (zstd's backward-read streams are written forward)."""

    def __init__(self):
        self.acc, self.n, self.out = 0, 0, bytearray()

    def put(self, v, k):
        self.acc |= (v & ((1 << k) - 1)) << self.n
        self.n += k
        while self.n >= 8:
            self.out.append(self.acc & 0xFF)
            self.acc >>= 8
            self.n -= 8

    def close_backward(self):
        """End mark for a backward-read stream: a 1 bit, then zero padding to the byte."""
        self.put(1, 1)
        if self.n:
            self.out.append(self.acc & 0xFF)
            self.acc, self.n = 0, 0
        return bytes(self.out)

    def close(self):
        if self.n:
            self.out.append(self.acc & 0xFF)
            self.acc, self.n = 0, 0
        return bytes(self.out)


def huff_lengths(freq, maxlen):
    """Length-limited Huffman code lengths (the kernels' huff_lengths, zlib gen_bitlen): two-queue
    merge over (frequency, symbol)-sorted leaves, depths clamped top-down with every clamped node an
    overflow, bl_count repaired, the least frequent leaves taking the longest codes."""
    n = len(freq)
    syms = [s for s in range(n) if freq[s]]
    m = len(syms)
    lens = [0] * n
    if m < 2:
        raise ValueError("a Huffman code needs two symbols")
    srt = sorted(syms, key=lambda s: (freq[s], s))
    weight, parent = [], [0] * (2 * m)
    li = ii = 0

    def wt(node):
        return freq[srt[node]] if node < m else weight[node - m]

    for _ in range(m - 1):
        pair = []
        for _ in range(2):
            if li < m and (ii >= len(weight) or wt(li) <= weight[ii]):
                pair.append(li)
                li += 1
            else:
                pair.append(m + ii)
                ii += 1
        weight.append(wt(pair[0]) + wt(pair[1]))
        parent[pair[0]] = parent[pair[1]] = m + len(weight) - 1
    root = 2 * m - 2
    depth, blc, ov = [0] * (2 * m), [0] * (maxlen + 2), 0
    for node in range(root - 1, -1, -1):
        d = depth[parent[node]] + 1
        if d > maxlen:
            d, ov = maxlen, ov + 1
        depth[node] = d
        if node < m:
            blc[d] += 1
    while ov > 0:
        bits = maxlen - 1
        while blc[bits] == 0:
            bits -= 1
        blc[bits] -= 1
        blc[bits + 1] += 2
        blc[maxlen] -= 1
        ov -= 2
    idx = 0
    for L in range(maxlen, 0, -1):
        for _ in range(blc[L]):
            lens[srt[idx]] = L
            idx += 1
    return lens


def huff_codes(lens):
    """zstd prefix codes (RFC 8878 §4.2.1.1 example): from the longest length up, consecutive values
    in symbol order; the value moves to the next shorter length as (value + count) >> 1."""
    maxb = max(lens)
    codes = [0] * len(lens)
    val = 0
    for L in range(maxb, 0, -1):
        for s in range(len(lens)):
            if lens[s] == L:
                codes[s] = val
                val += 1
        val >>= 1
    return codes


def fse_normalize(counts, tl):
    """Normalised counts summing to 2^tl, every present symbol >= 1 (no 'less than 1' entries)."""
    total, size = sum(counts), 1 << tl
    norm = [max(1, c * size // total) if c else 0 for c in counts]
    diff = size - sum(norm)
    while diff:
        s = max(range(len(norm)), key=lambda t: (norm[t], -t))
        if diff > 0:
            norm[s] += diff
            diff = 0
        else:
            cand = [t for t in range(len(norm)) if norm[t] > 1]
            s = max(cand, key=lambda t: (norm[t], -t))
            take = min(-diff, norm[s] - 1)
            norm[s] -= take
            diff += take
    return norm


def fse_write_ncount(norm, tl, w):
    """FSE table description (RFC 8878 §4.1.1; libzstd FSE_writeNCount): accuracy log - 5 in 4 bits,
    then value = count + 1 per symbol in a variable number of bits (small values one bit shorter),
    a zero count followed by 2-bit repeat flags for the zeros after it; stops when the probability
    points are spent. Byte-aligned at the end."""
    w.put(tl - 5, 4)
    remaining, threshold, nbits = (1 << tl) + 1, 1 << tl, tl + 1
    s, prev0, n = 0, False, len(norm)
    while s < n and remaining > 1:
        if prev0:
            start = s
            while s < n and norm[s] == 0:
                s += 1
            while s >= start + 3:
                start += 3
                w.put(3, 2)
            w.put(s - start, 2)
        count = norm[s]
        s += 1
        mx = (2 * threshold - 1) - remaining
        remaining -= count
        count += 1
        if count >= threshold:
            count += mx
        w.put(count, nbits - (1 if count < mx else 0))
        prev0 = count == 1
        while remaining < threshold:
            nbits -= 1
            threshold >>= 1
    assert remaining == 1
    return w.close()


def fse_tables(norm, tl):
    """FSE_buildDTable's symbol spread and per-state (symbol, nb, base), plus the first state of each
    symbol (its largest nb) and the encoding view enc[s][x] = the state of s whose range holds x."""
    size, mask = 1 << tl, (1 << tl) - 1
    sym = [0] * size
    step = (size >> 1) + (size >> 3) + 3
    pos = 0
    for s, c in enumerate(norm):
        for _ in range(c):
            sym[pos] = s
            pos = (pos + step) & mask
    nxt = list(norm)
    nb, base = [0] * size, [0] * size
    for u in range(size):
        s = sym[u]
        x = nxt[s]
        nxt[s] += 1
        nb[u] = tl - (x.bit_length() - 1)
        base[u] = (x << nb[u]) - size
    first = {}
    for u in range(size - 1, -1, -1):
        first[sym[u]] = u
    enc = {}
    for u in range(size):
        for x in range(base[u], base[u] + (1 << nb[u])):
            enc[(sym[u], x)] = u
    return sym, nb, base, first, enc


def fse_encode_2state(symbols, norm, tl, w):
    """Two interleaved FSE states (libzstd FSE_compress_usingCTable / FSE_decompress_usingDTable):
    state 1 decodes the even positions, state 2 the odd ones; the decoder stops after the update that
    follows the second-to-last symbol overflows the stream and emits the last one from the other
    state, so that symbol's state starts with its largest bit count (first[s], nb >= 1)."""
    sym, nb, base, first, enc = fse_tables(norm, tl)
    N = len(symbols)
    X = [None, None]  # current state of stream 0 (even positions) / 1 (odd positions)
    X[(N - 1) & 1] = first[symbols[N - 1]]
    X[(N - 2) & 1] = first[symbols[N - 2]]
    for k in range(N - 3, -1, -1):
        st = k & 1
        u = enc[(symbols[k], X[st])]
        w.put(X[st] - base[u], nb[u])
        X[st] = u
    w.put(X[1], tl)
    w.put(X[0], tl)
    return w.close_backward()


def huf_description(lens):
    """Huffman tree description (RFC 8878 §4.2.1): weights w = maxBits + 1 - len for symbols
    0..maxSym-1 (maxSym's is implied). Direct 4-bit weights when maxSym <= 128, else FSE-compressed
    weights (libzstd HUF_writeCTable); None when neither applies (one weight value only, or the
    compressed weights are not smaller than maxSym / 2 bytes)."""
    maxb = max(lens)
    max_sym = max(s for s in range(len(lens)) if lens[s])
    weights = [(maxb + 1 - lens[s]) if lens[s] else 0 for s in range(max_sym)]
    counts = [0] * 13
    for x in weights:
        counts[x] += 1
    if sum(1 for c in counts if c) > 1 and max(counts) < len(weights):
        norm = fse_normalize(counts[:max(i for i in range(13) if counts[i]) + 1], WEIGHT_LOG)
        hdr = fse_write_ncount(norm, WEIGHT_LOG, BitW())
        body = fse_encode_2state(weights, norm, WEIGHT_LOG, BitW())
        comp = hdr + body
        if 1 < len(comp) < max_sym // 2 and len(comp) < 128:
            return bytes([len(comp)]) + comp
    if max_sym <= 128:
        nib = weights + [0] * (len(weights) & 1)
        return bytes([127 + max_sym]) + bytes((nib[i] << 4) | nib[i + 1] for i in range(0, len(nib), 2))
    return None


def huf_stream(lits, lens, codes):
    """One Huffman stream: the last literal's code written first, so the backward reader meets the
    first literal first; end mark + padding."""
    w = BitW()
    for b in reversed(lits):
        w.put(codes[b], lens[b])
    return w.close_backward()


def literals_section(lits, table=None):
    """A Compressed_Literals_Block (type 2, with the tree description) or, with table=(lens, codes)
    from an earlier block, a Treeless_Literals_Block (type 3). Single stream for <= 1023 literals
    (Size_Format 00), else 4 streams with a 6-byte jump table (Size_Format 01 / 10). Returns
    (section bytes, (lens, codes)) or (None, None) when Huffman coding does not apply."""
    n = len(lits)
    if table is None:
        freq = np.bincount(np.frombuffer(bytes(lits), np.uint8), minlength=256).tolist()
        if sum(1 for f in freq if f) < 2:
            return None, None
        lens = huff_lengths(freq, HUF_MAX_BITS)
        desc = huf_description(lens)
        if desc is None:
            return None, None
        codes = huff_codes(lens)
        ltype = 2
    else:
        lens, codes = table
        desc, ltype = b"", 3
    if n <= 1023:
        streams = huf_stream(lits, lens, codes)
        comp = desc + streams
        if len(comp) > 1023:
            return None, None
        hdr = ltype | (0 << 2) | (n << 4) | (len(comp) << 14)
        return hdr.to_bytes(3, "little") + comp, (lens, codes)
    seg = (n + 3) // 4
    parts = [huf_stream(lits[i * seg:min(n, (i + 1) * seg)], lens, codes) for i in range(4)]
    jump = b"".join(len(p).to_bytes(2, "little") for p in parts[:3])
    comp = desc + jump + b"".join(parts)
    if n <= 1023 and len(comp) <= 1023:
        hdr = ltype | (1 << 2) | (n << 4) | (len(comp) << 14)
        return hdr.to_bytes(3, "little") + comp, (lens, codes)
    hdr = ltype | (2 << 2) | (n << 4) | (len(comp) << 18)
    return hdr.to_bytes(4, "little") + comp, (lens, codes)


def frame_of_literal_blocks(data, block=4096, treeless=True):
    """A single-segment zstd frame of compressed blocks holding only literals (no sequences): the
    first Huffman block of the frame carries the tree, later ones reuse it (treeless) when its
    symbols cover theirs; blocks Huffman coding does not help are raw-literal blocks."""
    out = bytearray(b"\x28\xb5\x2f\xfd")
    n = len(data)
    fcs = 2 if n > 65535 + 256 else (1 if n > 255 else 0)
    out.append((fcs << 6) | (1 << 5))
    out += (n - 256 if fcs == 1 else n).to_bytes([1, 2, 4][fcs], "little")
    table = None
    for b0 in range(0, max(n, 1), block):
        lits = data[b0:b0 + block]
        sec, t = None, None
        if table is not None and treeless and all(table[0][x] for x in set(lits)):
            sec, t = literals_section(lits, table)
        if sec is None:
            sec, t = literals_section(lits)
            if sec is not None:
                table = t
        if sec is None:  # raw literals: Size_Format 11 (20-bit size)
            sec = (0 | (3 << 2) | (len(lits) << 4)).to_bytes(3, "little") + bytes(lits)
        body = sec + b"\x00"  # Number_of_Sequences = 0
        last = b0 + block >= n
        out += (int(last) | (2 << 1) | (len(body) << 3)).to_bytes(3, "little") + body
    return bytes(out)
