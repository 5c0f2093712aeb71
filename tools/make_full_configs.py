"""Writes the reference side of tests/golden/full_configs.json: every BASELINE config generated at full size and
precompressed by the REAL reference (oracle/_ref/uncomp, 1 core). Build container only (needs oracle/_ref).
Run: python3 tools/make_full_configs.py  (≈25 min here: C4 and C5 take ≈10 min each)."""
import sys, time, subprocess, hashlib, json, os
sys.path.insert(0, '/root/repo')
from antiz_amd import datagen
res = {}
for name, kw, flags in (("c1", {}, []), ("c2", {}, []), ("c3", {}, []), ("c4", {"seed": 4, "n_streams": 100000}, []),
                        ("c5", {"seed": 5, "n_streams": 100000}, ["--brute-window"])):
    t = time.time()
    p = datagen.cached(name, "/tmp/atz_full_cache", **kw)
    tg = time.time() - t
    d = open(p, "rb").read()
    t = time.time()
    r = subprocess.run(["/root/repo/oracle/_ref/uncomp", "-i", p, "-o", "/tmp/full/o.atz", "--notest"] + flags,
                       capture_output=True, text=True)
    dt = time.time() - t
    a = open("/tmp/full/o.atz", "rb").read()
    res[name] = {"input_sha256": hashlib.sha256(d).hexdigest(), "input_bytes": len(d), "flags": flags, "gen": kw,
                 "atz_sha256": hashlib.sha256(a).hexdigest(), "atz_bytes": len(a), "ref_rc": r.returncode,
                 "ref_seconds": round(dt, 1), "ref_stdout_tail": r.stdout.strip().splitlines()[-2:]}
    print(name, res[name], "gen", round(tg, 1), flush=True)
    json.dump(res, open("/tmp/full/ref_full.json", "w"), indent=1)
    os.remove("/tmp/full/o.atz")
