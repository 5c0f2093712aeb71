"""Deterministic synthetic workloads for the zlib-stream precompressor (BASELINE.json configs).

Text comes from a seeded 20 000-word vocabulary (words of 2-10 lowercase letters, space-joined).  zlib
streams are produced with the interpreter's zlib, whose deflate output is byte-identical to the
reference's vendored zlib 1.2.8 for clevel 1-9 (tests/test_oracle.py pins this); clevel 0 is never
used by the generators.  Every config is generated from its seed alone, so the same bytes appear on
every machine; tests pin the SHA-256 of the small ones.

  C1  ~172 KB PDF-like file (FlateDecode objects, c in {6,6,6,6,9,1}, w15, m8)          seed 172
  C2  10 000 x zlib(c6, w15, m8) of 4096 B text, concatenated                           seed 2
  C3  ~100 MB mix: PDF-like c6/c9 50 %, PNG-like Z_FILTERED c9 30 %, JAR-like raw 20 %   seed 3
  C4  1 GB, 100 000 streams, c U{1..9}, m U{1..9}, w15, ~10 KB compressed, 0-64 B gaps    seed 4
  C5  C4 with w U{10..15}                                                                 seed 5
"""
import os
import struct
import zlib
from concurrent.futures import ProcessPoolExecutor

import numpy as np

_VOCAB = None


def _vocab():
    global _VOCAB
    if _VOCAB is None:
        rng = np.random.default_rng(12345)
        lens = rng.integers(2, 11, size=20000)
        letters = rng.integers(ord("a"), ord("z") + 1, size=int(lens.sum()), dtype=np.uint8)
        words, pos = [], 0
        for n in lens:
            words.append(letters[pos:pos + n].tobytes() + b" ")
            pos += n
        blob = b"".join(words)
        offs = np.zeros(len(words) + 1, dtype=np.int64)
        offs[1:] = np.cumsum([len(w) for w in words])
        _VOCAB = (np.frombuffer(blob, dtype=np.uint8), offs)
    return _VOCAB


def text(rng, nbytes):
    """nbytes of space-joined vocabulary words drawn by `rng` (a numpy Generator)."""
    blob, offs = _vocab()
    lens = offs[1:] - offs[:-1]
    avg = float(lens.mean())
    k = int(nbytes / avg * 1.1) + 8
    while True:
        idx = rng.integers(0, len(lens), size=k)
        wl = lens[idx]
        if wl.sum() >= nbytes:
            break
        k *= 2
    starts = offs[idx]
    total = int(wl.sum())
    # gather: position p of output maps to blob[starts[w] + (p - cum[w])]
    cum = np.zeros(len(idx) + 1, dtype=np.int64)
    cum[1:] = np.cumsum(wl)
    wid = np.repeat(np.arange(len(idx)), wl)
    src = starts[wid] + (np.arange(total) - cum[wid])
    return blob[src[:nbytes]].tobytes()


def zstream(data, c, w=15, m=8, strategy=zlib.Z_DEFAULT_STRATEGY):
    co = zlib.compressobj(c, zlib.DEFLATED, w, m, strategy)
    return co.compress(data) + co.flush()


def gen_c1(seed=172):
    rng = np.random.default_rng(seed)
    levels = [6, 6, 6, 6, 9, 1]
    out = [b"%PDF-1.4\n%\xe2\xe3\xcf\xd3\n"]
    size, k = len(out[0]), 1
    while size < 172 * 1024:
        c = levels[int(rng.integers(0, len(levels)))]
        s = zstream(text(rng, int(rng.integers(2048, 12289))), c)
        obj = b"%d 0 obj\n<< /Length %d /Filter /FlateDecode >>\nstream\n" % (k, len(s)) + s + \
              b"\nendstream\nendobj\n"
        out.append(obj)
        size += len(obj)
        k += 1
    out.append(b"trailer\n<< /Size %d >>\n%%%%EOF\n" % k)
    return b"".join(out)


def gen_c2(seed=2, n=10000, payload=4096):
    rng = np.random.default_rng(seed)
    return b"".join(zstream(text(rng, payload), 6) for _ in range(n))


def _png_like(rng, nbytes):
    """PNG-ish IDAT payload: filtered scanlines of a smooth random image, zlib c9 Z_FILTERED."""
    width = int(rng.integers(64, 512))
    rows = max(1, nbytes // (width * 3 + 1))
    img = np.cumsum(rng.integers(-3, 4, size=(rows, width * 3)), axis=1).astype(np.int64) % 256
    raw = bytearray()
    prev = np.zeros(width * 3, dtype=np.int64)
    for r in range(rows):
        f = int(rng.integers(0, 3))
        line = img[r]
        if f == 1:
            flt = (line - np.concatenate(([0, 0, 0], line[:-3]))) % 256
        elif f == 2:
            flt = (line - prev) % 256
        else:
            flt = line
        raw.append(f)
        raw += flt.astype(np.uint8).tobytes()
        prev = line
    return zstream(bytes(raw), 9, 15, 8, zlib.Z_FILTERED)


def _jar_entry(rng, k):
    data = text(rng, int(rng.integers(2000, 20000)))
    co = zlib.compressobj(6, zlib.DEFLATED, -15)
    raw = co.compress(data) + co.flush()
    name = b"org/example/C%06d.class" % k
    hdr = b"PK\x03\x04" + struct.pack("<HHHHHIIIHH", 20, 0, 8, 0, 0, zlib.crc32(data), len(raw),
                                        len(data), len(name), 0)
    return hdr + name + raw


def _c3_piece(args):
    seed, target = args
    rng = np.random.default_rng(seed)
    out, size, k = [], 0, 0
    while size < target:
        u = float(rng.random())
        if u < 0.5:
            s = zstream(text(rng, int(rng.integers(4096, 32769))), 6 if rng.random() < 0.7 else 9)
            piece = b"%d 0 obj\n<< /Length %d /Filter /FlateDecode >>\nstream\n" % (k, len(s)) + s + \
                    b"\nendstream\nendobj\n"
        elif u < 0.8:
            s = _png_like(rng, int(rng.integers(8192, 65537)))
            piece = struct.pack(">I", len(s)) + b"IDAT" + s + b"\0\0\0\0"
        else:
            piece = _jar_entry(rng, k)
        out.append(piece)
        size += len(piece)
        k += 1
    return b"".join(out)


def _c4_piece(args):
    seed, n, wrange = args
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        c = int(rng.integers(1, 10))
        m = int(rng.integers(1, 10))
        w = 15 if wrange is None else int(rng.integers(wrange[0], wrange[1] + 1))
        payload = int(rng.integers(12500, 18751))   # ~10 KB compressed, 100k streams ~ 1 GB
        gap = int(rng.integers(0, 65))
        out.append(rng.integers(0, 256, size=gap, dtype=np.uint8).tobytes())
        out.append(zstream(text(rng, payload), c, w, m))
    return b"".join(out)


def _parallel(fn, args, workers):
    if workers <= 1:
        return b"".join(fn(a) for a in args)
    with ProcessPoolExecutor(max_workers=workers) as ex:
        return b"".join(ex.map(fn, args))


def gen_c3(seed=3, total=100 * 1000 * 1000, workers=None):
    workers = workers or min(16, os.cpu_count() or 1)
    pieces = 64
    return _parallel(_c3_piece, [(seed * 1000003 + i, total // pieces) for i in range(pieces)], workers)


def gen_c4(seed=4, n_streams=100000, wrange=None, workers=None):
    workers = workers or min(16, os.cpu_count() or 1)
    per = 500
    args = []
    left, i = n_streams, 0
    while left > 0:
        k = min(per, left)
        args.append((seed * 1000003 + i, k, wrange))
        left -= k
        i += 1
    return _parallel(_c4_piece, args, workers)


def gen_c5(seed=5, n_streams=100000, workers=None):
    return gen_c4(seed, n_streams, (10, 15), workers)


def gen_c4c3(seed=4, n_streams=100000, c3_bytes=100 * 1000 * 1000, workers=None):
    """C4 followed by a C3 cluster (its PNG-like Z_FILTERED streams run their whole trial list): the
    multi-GPU split's balance test (bench.py --workload c4c3), not a BASELINE config."""
    return gen_c4(seed, n_streams, workers=workers) + gen_c3(seed=3, total=c3_bytes, workers=workers)


def _relevel(s, flevel):
    """The same zlib stream with its header's FLEVEL field set to `flevel` (FCHECK recomputed): it still
    inflates, but no trial can reproduce its second byte, so its best ident is at most C - 1."""
    cmf = s[0]
    flg = (flevel << 6) | (s[1] & 0x20)
    flg |= (31 - (cmf * 256 + flg) % 31) % 31
    return s[:1] + bytes([flg]) + s[2:]


def gen_near(seed=71, n_streams=600):
    """Small streams (mostly one deflate block) at c U{1..9}, m U{1..9}, w U{10..15}; half of them with
    their header's FLEVEL moved to another class, so their best trial misses the original by exactly one
    byte (ident = C - 1).  The mismatch-tolerance stop (main.cpp:700) and the brute-window phase
    (main.cpp:590) then decide them: the threshold-grid fixtures (tests/golden/threshold_grid.json)."""
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n_streams):
        c = int(rng.integers(1, 10))
        m = int(rng.integers(1, 10))
        w = int(rng.integers(10, 16))
        s = zstream(text(rng, int(rng.integers(300, 4097))), c, w, m)
        if rng.random() < 0.5:
            fl = (s[1] >> 6) & 3
            s = _relevel(s, (fl + 1 + int(rng.integers(0, 3))) % 4)
        out.append(rng.integers(0, 256, size=int(rng.integers(0, 33)), dtype=np.uint8).tobytes())
        out.append(s)
    return b"".join(out)


CONFIGS = {"c1": gen_c1, "c2": gen_c2, "c3": gen_c3, "c4": gen_c4, "c5": gen_c5, "c4c3": gen_c4c3,
           "near": gen_near}


def cached(name, cache_dir, **kw):
    """Generate config `name` (kwargs forwarded) once into cache_dir and return its path."""
    tag = "_".join("%s%s" % (k, v) for k, v in sorted(kw.items()))
    path = os.path.join(cache_dir, "%s%s.bin" % (name, ("_" + tag) if tag else ""))
    if not os.path.exists(path):
        os.makedirs(cache_dir, exist_ok=True)
        data = CONFIGS[name](**kw)
        tmp = path + ".tmp%d" % os.getpid()
        with open(tmp, "wb") as f:
            f.write(data)
        os.replace(tmp, path)
    return path
