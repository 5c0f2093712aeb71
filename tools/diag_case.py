"""Diagnostics: per-stream sweep results of one golden case against the oracle (GPU box).
usage: python3 tools/diag_case.py <case name>"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import _libs  # noqa: E402
import golden_cases as G  # noqa: E402
import antiz_amd  # noqa: E402

name = sys.argv[1]
case = [c for c in G.cases() if c["name"] == name][0]
data = G.case_input(case)
o = case["opts"]
rc, ref, st = _libs.ora_precompress(data, **G.opts_kwargs(o))
with antiz_amd.Context(recomp_tresh=o.get("recomp_tresh", 128), sizediff_tresh=o.get("sizediff_tresh", 128),
                       shortcut_len=o.get("shortcut_len", 512), mismatch_tol=o.get("mismatch_tol", 2),
                       chunksize=o.get("chunksize", 524288), brute_window=bool(o.get("brute_window", 0))) as c:
    c.scan(data)
    res, _ = c.sweep()
    for i, (r, s) in enumerate(zip(res, st["streams"])):
        got = (r["clevel"], r["window"], r["memlevel"], r["ident"], r["recomp"])
        exp = (s["clevel"], s["window"], s["memlevel"], s["ident"], s["recomp"])
        print(i, s["infl_len"], s["comp_len"], "OK " if got == exp else "BAD", got, exp)
