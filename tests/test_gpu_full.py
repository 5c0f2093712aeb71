"""Parity at BASELINE.json's full sizes, in the -m gpu suite.

Every config is generated at full size from its seed (antiz_amd.datagen; the input SHA-256 is
checked), precompressed through the C ABI on the GPU (C5 with --brute-window) and its ATZ1 SHA-256
compared with the real reference's: tests/golden/full_configs.json holds oracle/_ref/uncomp's result
on the same generated inputs (tools/make_full_configs.py, run in the build container; the reference's
own end-to-end contract is the whole file, main.cpp:1216-1225).  The reconstruct of each ATZ1 must
give the input back (main.cpp:869-950).
"""
import hashlib
import json
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FULL = json.load(open(os.path.join(ROOT, "tests", "golden", "full_configs.json")))
CACHE = os.environ.get("ATZ_BENCH_CACHE", "/tmp/atz_bench_cache")   # shared with bench.py (same C4 file)


def sha(b):
    return hashlib.sha256(b).hexdigest()


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(k for k in FULL if not k.startswith("_")))
def test_full_size_config_identical_to_reference(name):
    import antiz_amd
    from antiz_amd import datagen
    e = FULL[name]
    path = datagen.cached(name, CACHE, **e["gen"])
    with open(path, "rb") as f:
        data = f.read()
    assert len(data) == e["input_bytes"] and sha(data) == e["input_sha256"], "generator output changed"
    with antiz_amd.Context(brute_window="--brute-window" in e["flags"]) as c:
        atz, st = c.precompress(data)
        assert len(atz) == e["atz_bytes"]
        assert sha(atz) == e["atz_sha256"], "%s: ATZ1 differs from the reference's" % name
        # the reference's stdout tail: recompressed:K/N
        assert e["ref_stdout_tail"][0] == "recompressed:%d/%d" % (st["n_recomp"], st["n_streams"])
        del data
        back = c.reconstruct(atz)
    assert sha(back) == e["input_sha256"]
