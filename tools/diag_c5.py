"""Diagnostics (GPU box): the library's per-stream sweep results on the C5 cpu_baseline sample (8 000
streams, seed 5, --brute-window) against a stream table the oracle wrote in this container.
usage: python3 tools/diag_c5.py <oracle table json> <reference sha256 prefix> [warm]"""
import hashlib
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import antiz_amd  # noqa: E402
from antiz_amd import datagen  # noqa: E402

exp = json.load(open(sys.argv[1]))
data = datagen.gen_c5(seed=5, n_streams=8000, workers=8)
with antiz_amd.Context(brute_window=True) as c:
    if len(sys.argv) > 3:   # the bench's order: a larger file first on the same context
        c.precompress(datagen.gen_c5(seed=6, n_streams=20000, workers=8))
    out, st = c.precompress(data)
    print("sha", hashlib.sha256(out).hexdigest()[:16], "want", sys.argv[2], "stats", {k: st[k] for k in
          ("n_streams", "n_recomp", "n_trials", "n_trials_replayed", "n_trials_duplicate", "n_replay_checked")})
    recs = c.scan(data)
    res, _ = c.sweep()
    bad = 0
    for i, (rc, r, e) in enumerate(zip(recs, res, exp)):
        got = tuple(rc[:4]) + (r["clevel"], r["window"], r["memlevel"], r["ident"], r["recomp"])
        if got != tuple(e):
            bad += 1
            if bad <= 25:
                print("BAD", i, "got", got, "exp", tuple(e))
    print("streams", len(res), len(exp), "bad", bad)
