#!/usr/bin/env python3
"""Generate tests/golden/inflate_edges.json: hand-built zlib streams that hit the decode edges of
k_inflate's fast loop, with the result the REAL zlib 1.2.8 (the reference's vendored copy, built by
oracle/build_ref.sh into oracle/_ref/libzref.so) gives for each, called the way the reference's scanner
calls it (ZlibWrapper.h:58-75, main.cpp:228-239: inflate(Z_SYNC_FLUSH) until the output buffer is not
filled).  Run in the build container only; the JSON (inputs + expected outputs) is committed.

Families (zlib 1.2.8's error points: Z/inffast.c:288 "invalid literal/length code", Z/inffast.c:303 /
Z/inflate.c:1100 "invalid distance code", Z/inflate.c:1064 the slow path's "invalid literal/length code",
Z/inflate.c:941 "too many length or distance symbols"):
  fixed_ll   fixed-Huffman block: literals, then lit/len symbol 286 or 287 (coded, but invalid), then
             trailing bytes; the symbol lands deep in the input or within its last 8 bytes
  fixed_dist fixed-Huffman block: literals, a length symbol, then distance symbol 30 or 31
  far        a distance past the output produced so far ("invalid distance too far back")
  dyn_dist   dynamic block with a one-code distance tree (incomplete, which zlib allows) whose
             unused code is read
  dyn_hdr    dynamic block header with HLIT 287/288 or HDIST 31/32
  overlap    valid streams of d literals and one match (length L, distance d) for every d in 1..258 and
             L in 3..258 (the fast loop's overlapping copies compute i % d with v_rcp_f32); the
             Adler-32 trailer makes any wrong output byte an error
"""
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import _libs  # noqa: E402


class Bits:
    """LSB-first bit writer (RFC 1951 s3.1.1): Huffman codes go in most significant bit first."""

    def __init__(self):
        self.out = bytearray()
        self.acc = 0
        self.n = 0

    def put(self, v, n):
        self.acc |= (v & ((1 << n) - 1)) << self.n
        self.n += n
        while self.n >= 8:
            self.out.append(self.acc & 255)
            self.acc >>= 8
            self.n -= 8

    def code(self, c, n):   # Huffman code of n bits, MSB first
        r = 0
        for i in range(n):
            r |= ((c >> i) & 1) << (n - 1 - i)
        self.put(r, n)

    def flush(self):
        if self.n:
            self.out.append(self.acc & 255)
        self.acc = 0
        self.n = 0
        return bytes(self.out)


def fixed_ll(b, sym):   # RFC 1951 s3.2.6
    if sym < 144:
        b.code(0x30 + sym, 8)
    elif sym < 256:
        b.code(0x190 + sym - 144, 9)
    elif sym < 280:
        b.code(sym - 256, 7)
    else:
        b.code(0xc0 + sym - 280, 8)


LBASE = [3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258]
LEXT = [0] * 8 + [1] * 4 + [2] * 4 + [3] * 4 + [4] * 4 + [5] * 4 + [0]
DBASE = [1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193, 257, 385, 513, 769, 1025, 1537, 2049, 3073,
         4097, 6145, 8193, 12289, 16385, 24577]
DEXT = [0, 0, 0, 0] + [i // 2 for i in range(2, 28)]


def put_len(b, L):
    s = max(i for i in range(29) if LBASE[i] <= L)
    if L == 258:
        s = 28
    fixed_ll(b, 257 + s)
    if LEXT[s]:
        b.put(L - LBASE[s], LEXT[s])


def put_dist(b, d):
    s = max(i for i in range(30) if DBASE[i] <= d)
    b.code(s, 5)
    if DEXT[s]:
        b.put(d - DBASE[s], DEXT[s])


def adler32(d):
    a, s = 1, 0
    for i in range(0, len(d), 5552):
        for x in d[i:i + 5552]:
            a += x
            s += a
        a %= 65521
        s %= 65521
    return (s << 16) | a


def zhdr():
    return bytearray([0x78, 0x01])


def case_fixed(r, nlit, tail, sym=None, dist_sym=None, far=False):
    b = Bits()
    for x in zhdr():
        b.put(x, 8)
    b.put(1, 1)   # BFINAL
    b.put(1, 2)   # BTYPE fixed
    lits = bytes(r.randrange(256) for _ in range(nlit))
    for x in lits:
        fixed_ll(b, x)
    if sym is not None:
        fixed_ll(b, sym)
    elif dist_sym is not None:
        put_len(b, r.randrange(3, 259))
        b.code(dist_sym, 5)
    elif far:
        put_len(b, r.randrange(3, 259))
        put_dist(b, nlit + 1 + r.randrange(0, 40))
    fixed_ll(b, 256)
    s = b.flush()
    return s + bytes(r.randrange(256) for _ in range(tail))


def case_dyn_dist(r, nlit, tail):
    """Dynamic block: literal/length code with literals 0-253 at 8 bits and 254-257 at 9 bits
    (254/256 + 4/512 = 1, complete), a distance tree of one 1-bit code (incomplete, which zlib allows
    for a single distance code), code-length code {1: 1 bit, 8: 2, 9: 2}; then literals and a length
    whose distance uses the unused code."""
    ll = [8] * 254 + [9] * 4
    dl = [1]
    lens = ll + dl
    clen = {1: 1, 8: 2, 9: 2}
    # canonical codes for the code length code
    def canon(lengths):
        maxb = max(lengths.values())
        bl_count = [0] * (maxb + 1)
        for v in lengths.values():
            bl_count[v] += 1
        code, nxt = 0, [0] * (maxb + 1)
        for bits in range(1, maxb + 1):
            code = (code + bl_count[bits - 1]) << 1
            nxt[bits] = code
        out = {}
        for sym in sorted(lengths):
            out[sym] = (nxt[lengths[sym]], lengths[sym])
            nxt[lengths[sym]] += 1
        return out
    cc = canon(clen)
    order = [16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15]
    hclen = max(i for i, s in enumerate(order) if s in clen) + 1
    lcodes = canon({i: v for i, v in enumerate(ll)})
    b = Bits()
    for x in zhdr():
        b.put(x, 8)
    b.put(1, 1)
    b.put(2, 2)            # dynamic
    b.put(len(ll) - 257, 5)
    b.put(len(dl) - 1, 5)
    b.put(hclen - 4, 4)
    for i in range(hclen):
        b.put(clen.get(order[i], 0), 3)
    for v in lens:
        c, n = cc[v]
        b.code(c, n)
    lits = [r.randrange(254) for _ in range(nlit)]
    for x in lits:
        c, n = lcodes[x]
        b.code(c, n)
    c, n = lcodes[257]     # length 3
    b.code(c, n)
    b.code(1, 1)           # the distance code nobody has: "invalid distance code"
    c, n = lcodes[256]
    b.code(c, n)
    return b.flush() + bytes(r.randrange(256) for _ in range(tail))


def case_dyn_hdr(r, hlit, hdist, tail):
    b = Bits()
    for x in zhdr():
        b.put(x, 8)
    b.put(1, 1)
    b.put(2, 2)
    b.put(hlit - 257, 5)
    b.put(hdist - 1, 5)
    b.put(15, 4)
    for _ in range(19):
        b.put(r.randrange(8), 3)
    return b.flush() + bytes(r.randrange(256) for _ in range(tail))


def case_overlap(d, r):
    """d literals, then matches (L, d) for L = 3..258, stored in one fixed block, zlib trailer."""
    b = Bits()
    for x in zhdr():
        b.put(x, 8)
    b.put(1, 1)
    b.put(1, 2)
    out = bytearray(r.randrange(256) for _ in range(d))
    for x in out:
        fixed_ll(b, x)
    for L in range(3, 259):
        put_len(b, L)
        put_dist(b, d)
        for i in range(L):
            out.append(out[-d])
    fixed_ll(b, 256)
    s = b.flush()
    a = adler32(bytes(out))
    return s + bytes([a >> 24, (a >> 16) & 255, (a >> 8) & 255, a & 255]) + bytes(r.randrange(256) for _ in range(8)), len(out)


def main():
    if not _libs.have_zref():
        sys.exit("oracle/_ref/libzref.so missing: run oracle/build_ref.sh first")
    r = random.Random(2024)
    cases = []

    def add(family, s):
        rf, tf, rl, ti, to, ai = _libs.zref_inflate_scan(s)
        st = 0 if rl == 1 else (1 if rl == -3 else 2)   # Z_STREAM_END / Z_DATA_ERROR / wants more input
        cases.append({"family": family, "hex": s.hex(), "status": st, "consumed": ti, "produced": to,
                      "zlib_ret": rl})

    for sym in (286, 287):
        for nlit in (0, 1, 7, 40, 300, 3000):
            for tail in (0, 1, 2, 3, 5, 8, 9, 16, 40):
                add("fixed_ll", case_fixed(r, nlit, tail, sym=sym))
    for ds in (30, 31):
        for nlit in (1, 7, 40, 300, 3000):
            for tail in (0, 1, 3, 5, 8, 16, 40):
                add("fixed_dist", case_fixed(r, nlit, tail, dist_sym=ds))
    for nlit in (0, 1, 5, 100, 2000):
        for tail in (0, 2, 8, 40):
            add("far", case_fixed(r, nlit, tail, far=True))
    for nlit in (0, 3, 60, 1500):
        for tail in (0, 1, 4, 8, 30):
            add("dyn_dist", case_dyn_dist(r, nlit, tail))
    for hlit, hdist in ((287, 1), (288, 1), (257, 31), (257, 32), (286, 30)):
        for tail in (0, 10, 60):
            add("dyn_hdr", case_dyn_hdr(r, hlit, hdist, tail))
    for d in range(1, 259):
        s, n = case_overlap(d, r)
        add("overlap", s)
        assert cases[-1]["status"] == 0 and cases[-1]["produced"] == n, cases[-1]
    # every case's expectation also holds for the plain-C restatement (oracle/ora_inflate.c)
    for c in cases:
        st, co, pr = _libs.ora_inflate(bytes.fromhex(c["hex"]))
        assert (st, co, pr) == (c["status"], c["consumed"], c["produced"]), (c["family"], st, co, pr)
    fam = {}
    for c in cases:
        fam.setdefault(c["family"], [0, 0, 0])[c["status"]] += 1
    out = {"source": "oracle/_ref/libzref.so (zlib 1.2.8 vendored by the reference), scanner call sequence "
                     "(ZlibWrapper.h:58-75, main.cpp:228-239); generated by tests/golden/make_inflate_edges.py",
           "status": "0 end of stream, 1 data error, 2 needs more input", "families": fam, "cases": cases}
    with open(os.path.join(HERE, "inflate_edges.json"), "w") as f:
        json.dump(out, f, indent=0)
    print(json.dumps(fam))


if __name__ == "__main__":
    main()
