"""Writes tests/golden/threshold_grid.json: the REAL reference's ATZ1 SHA-256 (oracle/_ref/uncomp, built from
/root/reference by oracle/build_ref.sh) on three seeded inputs under a grid of non-default thresholds.

The grid pins the rule-level shortcuts of the sweep (the eligibility floor, the device
stop flag, replays) where the defaults never take them:
  --mismatch-tol 0                        no tolerance stop (main.cpp:700)
  --mismatch-tol 200 --recomp-tresh 128   tol > recomp_tresh: the eligibility floor switches off
  --recomp-tresh 0                        only exact streams are recompressed (main.cpp:454)
  --sizediff-tresh 0                      every size difference fails the trial (main.cpp:671)
  --shortcut-len 64 --recomp-tresh 16     an early, strict shortcut (main.cpp:632-649)
  --brute-window --mismatch-tol 1         phase 1 on C - ident >= 1 (main.cpp:590)
Inputs: a 2 000-stream C4 slice (seed 61), a 1 000-stream C5 slice (seed 62, every grid point with
--brute-window) and `near` (antiz_amd.datagen.gen_near: small streams, half of them one byte from their best
trial, so the tolerance stop and phase 1 decide them).
Build container only.  Run: python3 tools/make_threshold_grid.py   (~5 min here, 6 processes)."""
import hashlib
import json
import os
import subprocess
import sys
import time
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from antiz_amd import datagen  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden", "threshold_grid.json")
CACHE = "/tmp/atz_bench_cache"
GRID = [["--mismatch-tol", "0"], ["--mismatch-tol", "200", "--recomp-tresh", "128"], ["--recomp-tresh", "0"],
        ["--sizediff-tresh", "0"], ["--shortcut-len", "64", "--recomp-tresh", "16"], ["--brute-window", "--mismatch-tol", "1"]]
NEAR = [[], ["--mismatch-tol", "0"], ["--mismatch-tol", "1"], ["--brute-window"], ["--brute-window", "--mismatch-tol", "0"],
        ["--brute-window", "--mismatch-tol", "1"], ["--mismatch-tol", "200", "--recomp-tresh", "128"],
        ["--brute-window", "--mismatch-tol", "200", "--recomp-tresh", "0"]]
INPUTS = [("c4", {"seed": 61, "n_streams": 2000}, GRID),
          ("c5", {"seed": 62, "n_streams": 1000}, [f if "--brute-window" in f else ["--brute-window"] + f for f in GRID]),
          ("near", {"seed": 71, "n_streams": 600}, NEAR)]


def run_ref(path, flags, tag):
    out = "/tmp/tgrid_%s.atz" % tag
    t = time.time()
    r = subprocess.run([os.path.join(ROOT, "oracle", "_ref", "uncomp"), "-i", path, "-o", out, "--notest"] + flags,
                       capture_output=True, text=True)
    dt = time.time() - t
    a = open(out, "rb").read()
    os.remove(out)
    return r, a, dt


def main():
    res = json.load(open(OUT)) if os.path.exists(OUT) else {}
    jobs = []
    for wl, gen, grid in INPUTS:
        path = datagen.cached(wl, CACHE, **gen)
        d = open(path, "rb").read()
        for flags in grid:
            key = "%s:%d %s" % (wl, gen["n_streams"], " ".join(flags))
            if key not in res:
                jobs.append((key, wl, gen, path, d, flags))

    def one(j):
        key, wl, gen, path, d, flags = j
        r, a, dt = run_ref(path, flags, hashlib.md5(key.encode()).hexdigest()[:10])
        return key, {"workload": wl, "gen": gen, "input_sha256": hashlib.sha256(d).hexdigest(), "input_bytes": len(d),
                     "flags": flags, "atz_sha256": hashlib.sha256(a).hexdigest(), "atz_bytes": len(a),
                     "ref_rc": r.returncode, "ref_seconds": round(dt, 1),
                     "ref_stdout_tail": r.stdout.strip().splitlines()[-2:]}

    with ThreadPoolExecutor(6) as ex:
        for key, e in ex.map(one, jobs):
            res[key] = e
            print(key, e["atz_sha256"][:16], e["ref_stdout_tail"], e["ref_seconds"], flush=True)
    json.dump(dict(sorted(res.items())), open(OUT, "w"), indent=1)


if __name__ == "__main__":
    main()
