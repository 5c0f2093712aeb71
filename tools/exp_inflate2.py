"""Diagnostic: k_inflate clocks per symbol on literal-only (Z_HUFFMAN_ONLY), normal (level 6) and
RLE streams -- run with ATZ_LIB=<diag build> ATZ_TIMING=1 (ATZ_INF_CLOCKS=1 prints per-launch clocks)."""
import os, sys, time, zlib
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import antiz_amd
from antiz_amd import datagen

rng = np.random.default_rng(7)
n = int(os.environ.get("EXP_N", "2000"))
kinds = {"huffman_only": zlib.Z_HUFFMAN_ONLY, "default_l6": zlib.Z_DEFAULT_STRATEGY, "rle": zlib.Z_RLE}
with antiz_amd.Context(device=0) as c:
    for name, strat in kinds.items():
        buf = bytearray()
        rng_ = []
        for i in range(n):
            t = datagen.text(rng, 25000)
            z = datagen.zstream(t, 6, 15, 8, strat)
            rng_.append((len(buf), len(z)))
            buf += z
            buf += bytes((-len(buf)) % 4)
        buf = bytes(buf) + bytes(4096)
        c.inflate_batch(buf, rng_[:8])
        t0 = time.perf_counter()
        r = c.inflate_batch(buf, rng_)
        dt = time.perf_counter() - t0
        print("%-14s n=%d  %.1f ms  out %.1f MB  ok=%d" % (name, n, dt * 1e3, sum(x[2] for x in r) / 1e6,
              sum(1 for x in r if x[0] == 0)), flush=True)
