"""Writes tests/golden/share_configs.json: the reference side of the per-rank share files that stand in for
one rank's part of the 1 GB C4 file at N = 2 / 4 / 8 (the same generator and seed with 50 000 / 25 000 /
12 500 streams), and the C4 + C3 cluster file of the split-balance runs (bench.py --workload c4c3).  Each
is generated, precompressed by the REAL reference (oracle/_ref/uncomp, 1 core) and its ATZ1 SHA-256 kept,
so bench.py can report atz_parity for --streams < 100000 and tests/test_gpu_full.py can check them.
Build container only (needs oracle/_ref).  Run: python3 tools/make_share_configs.py  (~10 min here)."""
import hashlib
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from antiz_amd import datagen  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden", "share_configs.json")
CASES = [("c4", 12500), ("c4", 25000), ("c4", 50000), ("c4c3", 100000)]


def main():
    res = json.load(open(OUT)) if os.path.exists(OUT) else {}
    os.makedirs("/tmp/share", exist_ok=True)
    for wl, n in CASES:
        key = "%s:%d" % (wl, n)
        if key in res:
            continue
        gen = {"seed": 4, "n_streams": n}
        p = datagen.cached(wl, "/tmp/atz_bench_cache", **gen)
        d = open(p, "rb").read()
        t = time.time()
        r = subprocess.run([os.path.join(ROOT, "oracle", "_ref", "uncomp"), "-i", p, "-o", "/tmp/share/o.atz", "--notest"],
                           capture_output=True, text=True)
        dt = time.time() - t
        a = open("/tmp/share/o.atz", "rb").read()
        res[key] = {"workload": wl, "gen": gen, "input_sha256": hashlib.sha256(d).hexdigest(), "input_bytes": len(d),
                    "flags": [], "atz_sha256": hashlib.sha256(a).hexdigest(), "atz_bytes": len(a), "ref_rc": r.returncode,
                    "ref_seconds": round(dt, 1), "ref_stdout_tail": r.stdout.strip().splitlines()[-2:]}
        print(key, res[key], flush=True)
        os.remove("/tmp/share/o.atz")
        json.dump(res, open(OUT, "w"), indent=1)


if __name__ == "__main__":
    main()
