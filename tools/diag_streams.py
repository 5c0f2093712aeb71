"""Diagnostics (GPU box): streams of diag/bad_streams.json -- (1) the library's one-shot deflate at every
(clevel, memLevel) of the stream's header window against the oracle; (2) each stream alone as a file,
precompressed with --brute-window, against the oracle's ATZ1.
usage: python3 tools/diag_streams.py diag/bad_streams.json"""
import hashlib
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import _libs  # noqa: E402
import antiz_amd  # noqa: E402

cases = json.load(open(sys.argv[1]))
with antiz_amd.Context(brute_window=True) as c:
    for cs in cases:
        d = bytes.fromhex(cs["data"])
        orig = bytes.fromhex(cs["orig"])
        w = cs["w"]
        bad = []
        for cl in range(0, 10):
            for m in range(1, 10):
                got = c.deflate(d, cl, w, m)
                want, _ = _libs.ora_deflate(d, cl, w, m)
                if got != want:
                    bad.append((cl, m))
        rc, ref, st = _libs.ora_precompress(orig, brute=1)
        out, st2 = c.precompress(orig)
        print("stream", cs["i"], "w", w, "exp", (cs["c"], cs["m"]), "deflate mismatches", bad,
              "alone:", "OK" if hashlib.sha256(out).digest() == hashlib.sha256(ref).digest() else "BAD", flush=True)
