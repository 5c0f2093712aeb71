"""Diagnostics (GPU box): the library's one-shot deflate of stream i of diag/bad_streams.json at the
given (clevel, window, memLevel) list, written to gpurun_out/<dir>/s<i>_c<c>_w<w>_m<m>.bin.
usage: python3 tools/diag_dump.py <json> <i> <outdir> c,w,m [c,w,m ...]"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import antiz_amd  # noqa: E402

cases = {c["i"]: c for c in json.load(open(sys.argv[1]))}
cs = cases[int(sys.argv[2])]
d = bytes.fromhex(cs["data"])
os.makedirs(sys.argv[3], exist_ok=True)
with antiz_amd.Context() as c:
    for spec in sys.argv[4:]:
        cl, w, m = (int(v) for v in spec.split(","))
        with open(os.path.join(sys.argv[3], "s%s_c%d_w%d_m%d.bin" % (sys.argv[2], cl, w, m)), "wb") as f:
            f.write(c.deflate(d, cl, w, m))
print("ok")
