"""Diagnostics (GPU box): randomized one-shot deflates through the library against the oracle, biased
to the cases with window slides and MAX_DIST edges (windowBits 9-13, streams of 1-8 windows).
usage: python3 tools/stress_deflate.py <seed> <cases> [levels]"""
import os
import random
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import _libs  # noqa: E402
import antiz_amd  # noqa: E402
from antiz_amd import datagen  # noqa: E402

seed, ncase = int(sys.argv[1]), int(sys.argv[2])
levels = [int(v) for v in sys.argv[3].split(",")] if len(sys.argv) > 3 else list(range(0, 10))
r = random.Random(seed)
rng = np.random.default_rng(seed)
buf = bytearray()
items = []
for k in range(ncase):
    w = r.choice([9, 10, 11, 12, 13, 14, 15])
    n = int((1 << w) * r.uniform(0.8, 8.0))
    kind = r.randrange(3)
    if kind == 0:
        d = datagen.text(rng, n)
    elif kind == 1:
        words = [bytes(r.choice(b"abcdefghij") for _ in range(r.randrange(2, 8))) for _ in range(r.choice([8, 30, 200]))]
        d = bytearray()
        while len(d) < n:
            d += r.choice(words) + b" "
        d = bytes(d[:n])
    else:
        d = datagen.text(rng, n // 2) + rng.integers(0, 256, size=n // 4, dtype=np.uint8).tobytes() + datagen.text(rng, n // 4)
    items.append((len(buf), len(d), r.choice(levels), w, r.randrange(1, 10)))
    buf += d
with antiz_amd.Context() as c:
    outs = []
    for i in range(0, len(items), 500):
        outs += c.deflate_batch(bytes(buf), items[i:i + 500])
bad = 0
for it, o in zip(items, outs):
    want, _ = _libs.ora_deflate(bytes(buf[it[0]:it[0] + it[1]]), it[2], it[3], it[4])
    if o != want:
        bad += 1
        if bad <= 20:
            first = next((i for i in range(min(len(o), len(want))) if o[i] != want[i]), min(len(o), len(want)))
            print("BAD", it[1:], len(o), len(want), "first diff byte", first, flush=True)
print("cases", len(items), "bad", bad, flush=True)
