"""The oracle (CPU restatement, oracle/) pinned against the reference's golden vectors.

These run without a GPU.  They establish that oracle/ reproduces zlib 1.2.8 deflate bit-exactly
(G2, from the reference's vendored zlib) and the reference pipeline's .atz bytes (G1 = the
reference's own ZT vectors, G3-G5 = cases produced by the real reference binary).
"""
import hashlib
import json
import os
import random

import pytest

import _libs
import golden_cases as G

GOLD = G.GOLD


def sha(b):
    return hashlib.sha256(b).hexdigest()


def test_deflate_kats_full_bytes():
    full = json.load(open(os.path.join(GOLD, "deflate_kat_text4k_w15.json")))
    d = open(os.path.join(GOLD, "kat", "text4k.bin"), "rb").read()
    for key, hexs in full.items():
        c, m = map(int, key.split("/"))
        out, hazard = _libs.ora_deflate(d, c, 15, m)
        assert out.hex() == hexs, key
        assert hazard == 0


@pytest.mark.parametrize("name", ["asd", "text4k", "rand5k", "input8k"])
def test_deflate_kats_all_params(name):
    kat = json.load(open(os.path.join(GOLD, "deflate_kat.json")))
    d = open(os.path.join(GOLD, "kat", name + ".bin"), "rb").read()
    assert sha(d) == kat["inputs"][name]
    for c in range(10):
        for w in range(9, 16):
            for m in range(1, 10):
                out, _ = _libs.ora_deflate(d, c, w, m)
                n, h = kat["results"]["%s/%d/%d/%d" % (name, c, w, m)]
                assert (len(out), sha(out)) == (n, h), (name, c, w, m)


def test_zt_kat_pipeline():
    data, meta = G.zt_kat()
    rc, atz, st = _libs.ora_precompress(data)
    assert rc == 0
    assert sha(atz) == meta["atz_sha256"]
    got = [(s["offset"], s["clevel"], s["window"], s["memlevel"]) for s in st["streams"]]
    want = [(s["offset"], s["clevel"], s["window"], s["memlevel"]) for s in meta["streams"]]
    assert got == want
    rc, rec = _libs.ora_reconstruct(atz)
    assert rc == 0 and rec == data


@pytest.mark.parametrize("case", G.cases(), ids=lambda c: c["name"])
def test_golden_case_pipeline(case):
    data = G.case_input(case)
    rc, atz, st = _libs.ora_precompress(data, **G.opts_kwargs(case["opts"]))
    assert rc == 0
    assert sha(atz) == case["atz_sha256"], case["name"]
    assert st["hazard"] == 0
    rc, rec = _libs.ora_reconstruct(atz)
    assert rc == 0 and rec == data


def test_inflate_roundtrip_and_truncation():
    r = random.Random(5)
    for k in range(200):
        d = _libs.text(r, r.randrange(0, 5000))
        s, _ = _libs.ora_deflate(d, r.randrange(0, 10), r.randrange(9, 16), r.randrange(1, 10))
        st, c, p = _libs.ora_inflate(s + b"junk")
        assert (st, c, p) == (0, len(s), len(d))
        cut = r.randrange(1, len(s))
        st, c, p = _libs.ora_inflate(s[:cut])
        assert st in (1, 2)
        if st == 2:
            assert c == cut


@pytest.mark.skipif(not _libs.have_zref(), reason="reference build (oracle/_ref) absent")
def test_live_reference_deflate_inflate_sample():
    r = random.Random(11)
    for k in range(150):
        d = _libs.text(r, r.randrange(1, 20000))
        c, w, m = r.randrange(0, 10), r.randrange(9, 16), r.randrange(1, 10)
        a, _ = _libs.ora_deflate(d, c, w, m)
        assert a == _libs.zref_deflate(d, c, w, m), (c, w, m)
        s = bytearray(a)
        s[r.randrange(2, len(s))] ^= 1 << r.randrange(8)
        s = bytes(s[:r.randrange(2, len(s) + 1)])
        st, cons, prod = _libs.ora_inflate(s)
        rf, tf, rl, ti, to, ai = _libs.zref_inflate_scan(s)
        assert cons == ti and tf == ti
        assert (st == 0) == (rl == 1)
        if st == 0:
            assert prod == to


MAXDIST_EDGE_SHA = "d75a2a586f840cd037952b7289852f11c4702d92dbefef4b6112824d68680f32"


def test_maxdist_edge_fixture_pinned():
    """tests/golden/maxdist_edge.bin: 11 streams of the C5 workload (windowBits 11, 13, 14; longer than
    MAX_DIST) whose parses hinge on a hash head at distance exactly MAX_DIST (walked as a head, not as
    a chain successor: Z/deflate.c:1227, 1660, 1766).  The expected ATZ1 SHA-256 was produced by the
    real reference (oracle/_ref/uncomp, with and without --brute-window: the same bytes); the oracle
    must agree."""
    data = open(os.path.join(G.GOLD, "maxdist_edge.bin"), "rb").read()
    for brute in (0, 1):
        rc, out, _ = _libs.ora_precompress(data, brute=brute)
        assert rc == 0 and hashlib.sha256(out).hexdigest() == MAXDIST_EDGE_SHA


def test_inflate_edge_fixtures_pinned():
    """tests/golden/inflate_edges.json: the real zlib 1.2.8's results (make_inflate_edges.py) on hand-built
    streams at k_inflate's fast-loop edges (fixed-code 286/287 and distance 30/31, far distances,
    incomplete dynamic distance trees, oversized HLIT/HDIST, all overlapping copies); the oracle agrees."""
    cases = json.load(open(os.path.join(G.GOLD, "inflate_edges.json")))["cases"]
    assert len(cases) > 400
    for c in cases:
        got = _libs.ora_inflate(bytes.fromhex(c["hex"]))
        assert got == (c["status"], c["consumed"], c["produced"]), c["family"]


def test_threshold_grid_near_pins_the_oracle():
    """The oracle's rule (main.cpp:454, 590, 671, 685-700) under non-default thresholds equals the real
    reference's ATZ1 on the `near` input (tests/golden/threshold_grid.json, tools/make_threshold_grid.py)."""
    from antiz_amd import datagen
    grid = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "threshold_grid.json")))
    data = datagen.gen_near(seed=71, n_streams=600)
    for e in (e for e in grid.values() if e["workload"] == "near"):
        assert sha(data) == e["input_sha256"]
        f = e["flags"]
        kw = {"brute": int("--brute-window" in f)}
        for name, key in (("--mismatch-tol", "tol"), ("--recomp-tresh", "recomp"), ("--sizediff-tresh", "sizediff"),
                          ("--shortcut-len", "shortcut")):
            if name in f:
                kw[key] = int(f[f.index(name) + 1])
        rc, atz, _ = _libs.ora_precompress(data, **kw)
        assert rc == 0 and sha(atz) == e["atz_sha256"], f


def test_fuzz_small_files_pin_the_oracle():
    """The seeded fuzz cases (small files, chunk sizes from 2 bytes, threshold variants): the oracle's
    ATZ1 equals the real reference's (tests/golden/fuzz_small.json, tools/make_fuzz_golden.py) on every
    case the reference completes; where it crashes (empty input, main.cpp:406 reads rBuffer[-1]) the
    oracle reports undefined behaviour instead of bytes."""
    fx = json.load(open(os.path.join(GOLD, "fuzz_small.json")))
    checked = 0
    for i, data, cs, opts in G.fuzz_cases():
        f = fx[str(i)]
        if sha(data) != f["input_sha256"]:   # another zlib build made different input streams
            continue
        rc, atz, _ = _libs.ora_precompress(data, chunksize=cs, **G.opts_kwargs(opts))
        if "atz_sha256" in f:
            assert rc == 0 and sha(atz) == f["atz_sha256"], (i, cs, opts)
        else:
            assert f["rc"] != 0 and rc != 0, (i, cs, opts, f["rc"], rc)
        checked += 1
    assert checked >= 150
