"""CPU model of k_gzip's segmented symbol decode (kernels/inflate.hip, ZG_INFLATE_SEG): the check of
its synchronisation logic against zlib, and the source of its sync statistics.

A Huffman block is decoded in rounds. In a round starting at the true bit position r0, lane l owns
the stream region [r0 + l*SEGB, r0 + (l+1)*SEGB) and decodes serially from OVL bits before it (lane 0
from r0). Its symbols starting inside its region are its records; `mask` marks which of the region's
first 64 bit positions start a symbol on its chain. Lane l is right when lane l-1 is, ended normally
(its exit = the first symbol start past its region), and that exit starts a symbol on lane l's chain;
lane l's records before the exit are dropped. The first wrong lane is re-decoded from its
predecessor's exit (at most MAXREP times a round); the round ends at the last right lane.

Test infrastructure (tests/test_gzip_seg_model.py), not the product path.
"""
from __future__ import annotations

import zlib

LEN_BASE = [3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163,
            195, 227, 258]
LEN_EXTRA = [0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0]
DIST_BASE = [1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193, 257, 385, 513, 769, 1025, 1537, 2049, 3073,
             4097, 6145, 8193, 12289, 16385, 24577]
DIST_EXTRA = [0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13]
CLEN_ORDER = [16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15]
END, EOB, BAD, CAP, PAST = 0, 1, 2, 4, 5


class Bits:
    def __init__(self, data: bytes):
        self.v = int.from_bytes(data, "little")
        self.n = len(data) * 8

    def get(self, p: int, k: int) -> int:
        return (self.v >> p) & ((1 << k) - 1)


def table(lens):
    """{(length, reversed code): symbol} for an LSB-first bit reader (RFC 1951 3.2.2)."""
    mx = max(lens) if lens else 0
    cnt = [0] * (mx + 2)
    for ln in lens:
        if ln:
            cnt[ln] += 1
    code, nxt = 0, [0] * (mx + 2)
    for b in range(1, mx + 1):
        code = (code + cnt[b - 1]) << 1 if b > 1 else 0
        nxt[b] = code
    t = {}
    for s, ln in enumerate(lens):
        if ln:
            c = nxt[ln]
            nxt[ln] += 1
            t[(ln, int(format(c, "0%db" % ln)[::-1], 2))] = s
    return t, mx


def read_sym(B: Bits, p: int, t, mx):
    for ln in range(1, mx + 1):
        s = t.get((ln, B.get(p, ln)))
        if s is not None:
            return s, ln
    return None, 0


def symbol(B: Bits, p: int, lt, dt):
    """(kind, record, bits, out_len) of the symbol at p: kind 0 literal/match, EOB, BAD."""
    s, ln = read_sym(B, p, *lt)
    if s is None or s > 285:
        return BAD, 0, 0, 0
    if s < 256:
        return 0, s, ln, 1
    if s == 256:
        return EOB, 0, ln, 0
    i = s - 257
    q = p + ln
    length = LEN_BASE[i] + B.get(q, LEN_EXTRA[i])
    q += LEN_EXTRA[i]
    d, dl = read_sym(B, q, *dt)
    if d is None or d > 29:
        return BAD, 0, 0, 0
    q += dl
    dist = DIST_BASE[d] + B.get(q, DIST_EXTRA[d])
    q += DIST_EXTRA[d]
    return 0, (1 << 31) | (dist << 9) | length, q - p, length


def seg_decode(B, p, s_own, s_end, end_bits, lt, dt, cap):
    recs, mask = [], 0
    while p < s_end:
        if p >= end_bits:
            return PAST, p, recs, mask
        kind, rec, nb, _ = symbol(B, p, lt, dt)
        own = p >= s_own
        if own and p - s_own < 64:
            mask |= 1 << (p - s_own)
        if kind != 0:
            if not own:
                return PAST, p, recs, mask
            if kind == EOB:
                return EOB, p + nb, recs, mask
            return BAD, p, recs, mask
        if own:
            if len(recs) == cap:
                return CAP, p, recs, mask
            recs.append(rec)
        p += nb
    return END, p, recs, mask


def decode_block_seg(B, r0, end_bits, lt, dt, segb, ovl, cap, maxrep, stats):
    """Records of one Huffman block from r0 and the bit after its end-of-block code."""
    out = []
    while True:
        lanes = []
        for l in range(64):
            s_own = r0 + l * segb
            p = s_own - ovl if l else r0
            st, p, recs, mask = seg_decode(B, p, s_own, s_own + segb, end_bits, lt, dt, cap)
            lanes.append(dict(s_own=s_own, st=st, p=p, recs=recs, mask=mask, skip=0, ok=l == 0, rep=False))
        for rep in range(maxrep + 1):
            for l in range(1, 64):
                L, P = lanes[l], lanes[l - 1]
                if L["rep"]:
                    continue
                e, d = P["p"], P["p"] - L["s_own"]
                L["ok"] = P["st"] == END and 0 <= d < 64 and (L["mask"] >> d) & 1 == 1
                L["skip"] = bin(L["mask"] & ((1 << d) - 1)).count("1") if L["ok"] else 0
            j = next((l for l in range(64) if not all(lanes[k]["ok"] for k in range(l + 1))), 64)
            j = next((l for l in range(64) if not lanes[l]["ok"]), 64)
            if j == 64:
                break
            if lanes[j - 1]["st"] != END or rep >= maxrep:
                for l in range(j, 64):
                    lanes[l]["ok"] = False
                break
            e = lanes[j - 1]["p"]
            st, p, recs, mask = seg_decode(B, e, e, lanes[j]["s_own"] + segb, end_bits, lt, dt, cap)
            lanes[j].update(st=st, p=p, recs=recs, mask=mask, skip=0, ok=True, rep=True)
            stats["repairs"] += 1
        J = next((l for l in range(64) if not lanes[l]["ok"]), 64)
        stats["rounds"] += 1
        stats["valid_lanes"] += J
        for l in range(J):
            out.extend(lanes[l]["recs"][lanes[l]["skip"]:])
        last = lanes[J - 1]
        if last["st"] == EOB:
            return out, last["p"]
        if last["st"] in (END, CAP):
            r0 = last["p"]
            continue
        raise ValueError("corrupt stream (status %d)" % last["st"])


def inflate_seg(gz: bytes, segb=512, ovl=256, cap=64, maxrep=8, stats=None):
    """gzip member -> decoded bytes through the segmented decode (stored blocks copied directly)."""
    stats = stats if stats is not None else {}
    for k in ("rounds", "valid_lanes", "repairs", "blocks"):
        stats.setdefault(k, 0)
    assert gz[:3] == b"\x1f\x8b\x08"
    flg, hp = gz[3], 10
    if flg & 4:
        hp += 2 + int.from_bytes(gz[hp:hp + 2], "little")
    for f in (8, 16):
        if flg & f:
            hp = gz.index(b"\0", hp) + 1
    if flg & 2:
        hp += 2
    B = Bits(gz)
    end_bits = (len(gz) - 8) * 8
    p, out, last = hp * 8, bytearray(), False
    while not last:
        last, typ = B.get(p, 1), B.get(p + 1, 2)
        p += 3
        stats["blocks"] += 1
        if typ == 0:
            p = (p + 7) & ~7
            n = B.get(p, 16)
            p += 32
            out += gz[p // 8:p // 8 + n]
            p += 8 * n
            continue
        if typ == 1:
            lens = [8] * 144 + [9] * 112 + [7] * 24 + [8] * 8
            dl = [5] * 30
        else:
            hlit, hdist, hclen = B.get(p, 5) + 257, B.get(p + 5, 5) + 1, B.get(p + 10, 4) + 4
            p += 14
            cl = [0] * 19
            for i in range(hclen):
                cl[CLEN_ORDER[i]] = B.get(p, 3)
                p += 3
            ct = table(cl)
            ll = []
            while len(ll) < hlit + hdist:
                s, n = read_sym(B, p, *ct)
                p += n
                if s < 16:
                    ll.append(s)
                elif s == 16:
                    ll += [ll[-1]] * (3 + B.get(p, 2))
                    p += 2
                elif s == 17:
                    ll += [0] * (3 + B.get(p, 3))
                    p += 3
                else:
                    ll += [0] * (11 + B.get(p, 7))
                    p += 7
            lens, dl = ll[:hlit], ll[hlit:]
        recs, p = decode_block_seg(B, p, end_bits, table(lens), table(dl), segb, ovl, cap, maxrep, stats)
        for r in recs:  # LZ77
            if r >> 31:
                dist, ln = (r >> 9) & 0xFFFF, r & 511
                for _ in range(ln):
                    out.append(out[-dist])
            else:
                out.append(r)
    return bytes(out)


if __name__ == "__main__":
    import numpy as np
    rng = np.random.default_rng(7)
    x = np.arange(32, dtype=np.float32)
    for lvl in (1, 6, 9):
        a = np.rint(256 * (np.sin(0.05 * x)[:, None, None] + np.cos(0.03 * x)[None, :, None]
                           + 0.5 * np.sin(0.07 * x)[None, None, :]) + rng.standard_normal((32, 32, 32))) / 256
        raw = a.astype(np.float32).tobytes()
        co = zlib.compressobj(lvl, zlib.DEFLATED, 31)
        gz = co.compress(raw) + co.flush()
        st = {}
        assert inflate_seg(gz, stats=st) == raw
        print(f"level {lvl}: {len(gz)} B, {st['blocks']} blocks, {st['rounds']} rounds, "
              f"{st['valid_lanes'] / st['rounds']:.1f} valid lanes/round, {st['repairs']} repairs")
