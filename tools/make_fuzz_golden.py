#!/usr/bin/env python3
"""Writes tests/golden/fuzz_small.json: the REAL reference's ATZ1 SHA-256 (oracle/_ref/uncomp, built from
/root/reference by oracle/build_ref.sh) for the seeded fuzz cases of tests/golden_cases.py fuzz_cases (small
files, chunk sizes from 2 bytes, threshold variants).  Cases where the reference exits non-zero or writes no
file (the oracle's reference-UB codes) are recorded as such.  usage: python3 tools/make_fuzz_golden.py"""
import hashlib
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)
import golden_cases as G  # noqa: E402

FLAG = {"mismatch_tol": "--mismatch-tol", "recomp_tresh": "--recomp-tresh", "shortcut_len": "--shortcut-len",
        "sizediff_tresh": "--sizediff-tresh"}


def main():
    out = {}
    for i, data, cs, opts in G.fuzz_cases():
        inp, atz = "/tmp/fuzz_%d.bin" % i, "/tmp/fuzz_%d.atz" % i
        with open(inp, "wb") as f:
            f.write(data)
        flags = ["--chunksize", str(cs)]
        for k, v in opts.items():
            flags += ["--brute-window"] if k == "brute_window" else [FLAG[k], str(v)]
        if os.path.exists(atz):
            os.remove(atz)
        r = subprocess.run([os.path.join(ROOT, "oracle", "_ref", "uncomp"), "-i", inp, "-o", atz, "--notest"] + flags,
                           capture_output=True, timeout=120)
        rec = {"input_sha256": hashlib.sha256(data).hexdigest(), "chunksize": cs, "opts": opts, "rc": r.returncode}
        if r.returncode == 0 and os.path.exists(atz):
            rec["atz_sha256"] = hashlib.sha256(open(atz, "rb").read()).hexdigest()
            os.remove(atz)
        os.remove(inp)
        out[str(i)] = rec
    with open(os.path.join(ROOT, "tests", "golden", "fuzz_small.json"), "w") as f:
        json.dump(out, f, indent=0, sort_keys=True)
    print(len(out), "cases,", sum("atz_sha256" in v for v in out.values()), "with an ATZ1")


if __name__ == "__main__":
    main()
