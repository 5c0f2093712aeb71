"""The library's remaining run-time switches change how the sweep is scheduled, never its result.

Each one is read once per process, so every setting runs in its own subprocess on the same input:
the ATZ1 bytes must equal the oracle's (the reference's algorithm, oracle/) for each of them.
  ATZ_REPLAY   0 no symbol replay, 2 save sequences but never replay, 3 replays between budget-free
               trials only (default 1: DESIGN.md s3.5)
  ATZ_DEDUP    0 launch duplicate trials anyway (default 1)
  ATZ_PIPES    sweep pipes, 1..8 (default 3; 6 for a sweep of <= 16 000 streams when
               GPU_MAX_HW_QUEUES >= 8, as bench.py sets it for small per-rank shares)
  ATZ_TARGET   trials per round and pipe (speculation depth; default 8192 for a sweep of at most 32 000
               streams, else 4096)
  ATZ_SPEC_CONT 0: the scan waits for the first chunk-boundary continuations (default 1: speculative)
  ATZ_MW       multi-wave trials up to this memLevel (default 2, 4 in rounds with at most 16 000 streams left;
               0: every trial on one wave)
  ATZ_MHINT    0 / 1: whole match tables for the first block's memLevel off / on (default: above 16 000
               streams, or on six or more pipes: atz_accel.cpp big_sweep)
  ATZ_PREFIX_MIN the match-table prefix floor in positions (default 3072 where big_sweep holds, else 1024)
  ATZ_ELIG     0: every trial keeps the reference's exact rule to its end (default 1: a trial stops once
               it cannot make its stream recompressible; atz_accel.cpp elig_floor)
  ATZ_DFIRST   0: a depth pass before every bucket table (default: only where a replay may spare it)
  ATZ_EARLY    0: every first-pass match table waits for the round's plan (default: tables of trials that
               cannot replay are launched before it)
  ATZ_STAGE    0: uploads straight from pageable memory (default: through a pinned staging buffer)
  ATZ_STOPFLAG 0: speculative trials run to their own end (default: a stream's stop ends its later trials)
  ATZ_CAP_DIV  every device-memory cap divided by this (test_memory_caps_bind_...): the paths past the caps
"""
import hashlib
import os
import subprocess
import sys

import pytest

import _libs

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SETTINGS = [{"ATZ_REPLAY": "0"}, {"ATZ_REPLAY": "2"}, {"ATZ_REPLAY": "3"}, {"ATZ_DEDUP": "0"},
            {"ATZ_PIPES": "1"}, {"ATZ_PIPES": "5"}, {"GPU_MAX_HW_QUEUES": "8"}, {"ATZ_TARGET": "256"}, {"ATZ_TARGET": "65536"},
            {"ATZ_SPEC_CONT": "0"}, {"ATZ_MW": "0"}, {"ATZ_MW": "2"}, {"ATZ_MW": "9"}, {"ATZ_REPLAY": "0", "ATZ_DEDUP": "0", "ATZ_PIPES": "2", "ATZ_SPEC_CONT": "0"},
            {"ATZ_PIPES": "8", "ATZ_TARGET": "256"}, {"ATZ_PIPES": "6", "ATZ_TARGET": "65536"},
            {"ATZ_MHINT": "1"}, {"ATZ_MHINT": "0"}, {"ATZ_PREFIX_MIN": "3072", "ATZ_MHINT": "1"},
            {"ATZ_ELIG": "0"}, {"ATZ_ELIG": "0", "ATZ_REPLAY": "0"},
            {"ATZ_DFIRST": "0"}, {"ATZ_EARLY": "0"}, {"ATZ_STAGE": "0"},
            {"ATZ_EARLY": "0", "ATZ_STAGE": "0"}, {"ATZ_STOPFLAG": "0"}, {"ATZ_TARGET": "16384"},
            {"ATZ_PIPES": "6", "GPU_MAX_HW_QUEUES": "8", "ATZ_TARGET": "65536"}]

RUN = r"""
import hashlib, sys
sys.path.insert(0, %r)
import antiz_amd
data = open(sys.argv[1], "rb").read()
with antiz_amd.Context(chunksize=int(sys.argv[2]), device=0) as c:
    out, st = c.precompress(data)
print(hashlib.sha256(out).hexdigest())
""" % ROOT


@pytest.fixture(scope="module")
def sample(tmp_path_factory):
    from antiz_amd import datagen
    data = datagen.gen_c4(seed=51, n_streams=700)   # ~7 MB, chunk-boundary streams at 65536
    path = str(tmp_path_factory.mktemp("knobs") / "c4k.bin")
    with open(path, "wb") as f:
        f.write(data)
    rc, ref, _ = _libs.ora_precompress(data, chunksize=65536)
    assert rc == 0
    return path, hashlib.sha256(ref).hexdigest()


@pytest.mark.parametrize("env", SETTINGS, ids=lambda e: ",".join("%s=%s" % kv for kv in e.items()))
def test_switch_keeps_the_atz_bytes(sample, env):
    path, want = sample
    r = subprocess.run([sys.executable, "-c", RUN, path, "65536"], env=dict(os.environ, **env),
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.strip().splitlines()[-1] == want


CAPS = r"""
import hashlib, sys
sys.path.insert(0, %r)
import antiz_amd
data = open(sys.argv[1], "rb").read()
with antiz_amd.Context(chunksize=int(sys.argv[2]), device=0, brute_window=sys.argv[3] == "1") as c:
    out, st = c.precompress(data)
    back = c.reconstruct(out)
print(st["n_inflate_retries"], int(back == data))
print(hashlib.sha256(out).hexdigest())
""" % ROOT


@pytest.mark.parametrize("div", ["4096", "1000000000"])
def test_memory_caps_bind_and_keep_the_atz_bytes(sample, div):
    """The caps on device memory (scan output arena, bucket cache, replay arena, round and reconstruct
    batch budgets: atz_accel.cpp cap_bytes) bind only on inputs of tens of GB. Divided down, they bind on
    this sample: candidates are re-inflated, rounds build their own tables and defer streams, replays go
    unsaved, reconstruct runs in batches. 1e9 puts every cap at its 4 KiB floor (one stream per round)."""
    path, want = sample
    r = subprocess.run([sys.executable, "-c", CAPS, path, "65536", "0"], env=dict(os.environ, ATZ_CAP_DIV=div),
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = r.stdout.strip().splitlines()
    retries, same = (int(v) for v in lines[-2].split())
    assert lines[-1] == want
    assert same == 1
    assert retries > 0   # the scan arena did overflow


@pytest.fixture(scope="module")
def sample_c5(tmp_path_factory):
    from antiz_amd import datagen
    data = datagen.gen_c5(seed=52, n_streams=400)   # windows 10-15: brute-window phases, sliding windows
    path = str(tmp_path_factory.mktemp("knobs5") / "c5k.bin")
    with open(path, "wb") as f:
        f.write(data)
    rc, ref, _ = _libs.ora_precompress(data, chunksize=65536, brute=1)
    assert rc == 0
    return path, hashlib.sha256(ref).hexdigest()


def test_memory_caps_bind_under_brute_window(sample_c5):
    """The same caps divided down on a --brute-window (C5-like) sample: the brute-window lists (main.cpp:590)
    run through deferred rounds, per-round tables and unsaved replays."""
    path, want = sample_c5
    r = subprocess.run([sys.executable, "-c", CAPS, path, "65536", "1"], env=dict(os.environ, ATZ_CAP_DIV="4096"),
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = r.stdout.strip().splitlines()
    assert lines[-1] == want
    assert lines[-2].split()[1] == "1"
