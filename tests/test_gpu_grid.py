"""Non-default thresholds against the REAL reference, under the sweep policies of a big file.

tests/golden/threshold_grid.json holds oracle/_ref/uncomp's ATZ1 SHA-256 for a 2 000-stream C4 slice, a
1 000-stream C5 slice (--brute-window) and the `near` input (small streams one byte from their best
trial) under a grid of thresholds (tools/make_threshold_grid.py).  The sweep's rule-level shortcuts --
the eligibility floor (off when mismatch_tol > recomp_tresh), the device stop flag, symbol replay, the
multi-wave hand-over -- must leave every ATZ1 byte as the reference's rule (main.cpp:454, 590, 632-649,
671, 685-700) gives it.  Each setting of the library's schedule switches runs in its own process (they
are read once per process):
  big      ATZ_PIPES=3 ATZ_MHINT=1 ATZ_PREFIX_MIN=3072: the policies of a > 16 000-stream sweep
  default  the library's own choice for a file this size (6 pipes where the queues allow, 8192 target)
  mw4      ATZ_MW=4 ATZ_TARGET=16384 (near only): deep speculative rounds (K > 1) of multi-wave trials on
           single-block streams, where a stream that stops at C - mismatch_tol skips its later trials
"""
import hashlib
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GRID = json.load(open(os.path.join(ROOT, "tests", "golden", "threshold_grid.json")))
CACHE = os.environ.get("ATZ_BENCH_CACHE", "/tmp/atz_bench_cache")
ENVS = {"big": {"ATZ_PIPES": "3", "ATZ_MHINT": "1", "ATZ_PREFIX_MIN": "3072"}, "default": {},
        "mw4": {"ATZ_MW": "4", "ATZ_TARGET": "16384"}}

RUN = r"""
import hashlib, json, sys
sys.path.insert(0, %r)
import antiz_amd
data = open(sys.argv[1], "rb").read()
for flags in json.loads(sys.argv[2]):
    kw = {}
    i = 0
    while i < len(flags):
        f = flags[i]
        if f == "--brute-window":
            kw["brute_window"] = True
            i += 1
            continue
        kw[f[2:].replace("-", "_")] = int(flags[i + 1])
        i += 2
    with antiz_amd.Context(device=0, **kw) as c:
        out, st = c.precompress(data)
    print(json.dumps({"flags": flags, "sha": hashlib.sha256(out).hexdigest(), "n": len(out),
                      "tail": "recompressed:%%d/%%d" %% (st["n_recomp"], st["n_streams"])}), flush=True)
""" % ROOT


def _inputs():
    seen = {}
    for e in GRID.values():
        key = (e["workload"], json.dumps(e["gen"], sort_keys=True))
        seen.setdefault(key, []).append(e)
    return seen


CASES = [(wl, gen, env) for (wl, gen) in _inputs() for env in (("big", "default", "mw4") if wl == "near" else ("big", "default"))]


@pytest.mark.parametrize("wl,gen,env", CASES, ids=["%s-%s" % (c[0], c[2]) for c in CASES])
def test_threshold_grid_identical_to_reference(wl, gen, env):
    from antiz_amd import datagen
    entries = _inputs()[(wl, gen)]
    path = datagen.cached(wl, CACHE, **json.loads(gen))
    with open(path, "rb") as f:
        d = f.read()
    assert hashlib.sha256(d).hexdigest() == entries[0]["input_sha256"], "generator output changed"
    del d
    r = subprocess.run([sys.executable, "-u", "-c", RUN, path, json.dumps([e["flags"] for e in entries])],
                       env=dict(os.environ, **ENVS[env]), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    got = [json.loads(line) for line in r.stdout.splitlines() if line.startswith("{")]
    assert len(got) == len(entries)
    bad = []
    for e, g in zip(entries, got):
        assert g["flags"] == e["flags"]
        if g["sha"] != e["atz_sha256"] or g["n"] != e["atz_bytes"] or g["tail"] != e["ref_stdout_tail"][0]:
            bad.append((" ".join(e["flags"]), g["tail"], e["ref_stdout_tail"][0], g["n"], e["atz_bytes"]))
    assert not bad, "ATZ1 differs from the reference's under %s: %s" % (env, bad)
