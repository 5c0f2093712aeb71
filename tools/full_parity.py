"""Parity at BASELINE.json's full sizes (GPU box): every config C1-C5 generated at full size, precompressed
by the library (C5 with --brute-window), and its ATZ1 SHA-256 compared with the real reference's, which
tests/golden/full_configs.json holds (oracle/_ref/uncomp run in the build container on the same
generated inputs; the input SHA-256 is checked too).  Reconstruct of each ATZ1 must give the input.
usage: python3 tools/full_parity.py [configs...]"""
import hashlib
import json
import os
import sys
import time

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
import antiz_amd  # noqa: E402
from antiz_amd import datagen  # noqa: E402

ref = json.load(open(os.path.join(ROOT, "tests", "golden", "full_configs.json")))
names = sys.argv[1:] or sorted(k for k in ref if not k.startswith("_"))
ok_all = True
for name in names:
    e = ref[name]
    t = time.time()
    p = datagen.cached(name, "/tmp/atz_full_cache", **e["gen"])
    data = open(p, "rb").read()
    in_ok = hashlib.sha256(data).hexdigest() == e["input_sha256"]
    with antiz_amd.Context(brute_window="--brute-window" in e["flags"]) as c:
        t1 = time.time()
        out, st = c.precompress(data)
        dt = time.time() - t1
        same = hashlib.sha256(out).hexdigest() == e["atz_sha256"]
        back = c.reconstruct(out) == data
    ok_all &= in_ok and same and back
    print("%s: input %s, atz %s (%d bytes, %d/%d recompressed), reconstruct %s, %.2f s (gen+load %.1f s)" %
          (name, "ok" if in_ok else "DIFFERS", "IDENTICAL to the reference" if same else "DIFFERS from the reference",
           len(out), st["n_recomp"], st["n_streams"], "ok" if back else "FAILED", dt, t1 - t), flush=True)
print("ALL IDENTICAL" if ok_all else "MISMATCH")
sys.exit(0 if ok_all else 1)
