#!/usr/bin/env python3
"""Generate tests/golden/cli_cases.json from the REAL reference CLI (oracle/_ref/uncomp, main.cpp +
TCLAP 1.2.1 built by oracle/build_ref.sh).  Run in the build container only; the fixture is data
(argv, input files, expected stdout/stderr bytes and exit status), so the CLI tests need neither
/root/reference nor a GPU.

Every case here ends before any GPU work: help/version, TCLAP parse errors (unknown flags, missing
values, bad integers, repeated arguments, combined switches, "--"), a missing input file and the
-r header checks (main.cpp:1011-1030, 27-35).  The precompress/verify/-r paths that do GPU work are
compared live against the reference in tests/test_gpu.py::test_cli_matches_reference.
"""
import base64
import json
import os
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import _libs  # noqa: E402

LONG_PROG = "./a_rather_long_program_name_to_exercise_usage_wrapping/uncomp"

# (argv[0], args, {file name: bytes}); files are created in an empty working directory
CASES = [
    ("uncomp", ["-h"], {}),
    ("uncomp", ["--help"], {}),
    ("uncomp", ["--version"], {}),
    ("uncomp", [], {}),
    (LONG_PROG, [], {}),
    (LONG_PROG, ["-h"], {}),
    ("u", ["-h"], {}),
    ("uncomp", ["-i"], {}),
    ("uncomp", ["-o"], {}),
    ("uncomp", ["-i", "x", "--chunksize"], {}),
    ("uncomp", ["--bogus", "-i", "x"], {}),
    ("uncomp", ["-x"], {}),
    ("uncomp", ["-i", "x", "extra"], {}),
    ("uncomp", ["-i", "x", "--chunksize", "abc"], {}),
    ("uncomp", ["-i", "x", "--chunksize", "12abc"], {}),
    ("uncomp", ["-i", "x", "--chunksize", "12 13"], {}),
    ("uncomp", ["-i", "x", "--chunksize", "12 "], {}),
    ("uncomp", ["-i", "x", "--chunksize", "0x10"], {}),
    ("uncomp", ["-i", "x", "--chunksize", "1e3"], {}),
    ("uncomp", ["-i", "x", "--mismatch-tol", "99999999999999999999"], {}),
    ("uncomp", ["-i", "x", "--recomp-tresh", "-1"], {}),
    ("uncomp", ["-i", "x", "--shortcut-len", "+5"], {}),
    ("uncomp", ["-i", "x", "--chunksize", " 12"], {}),
    ("uncomp", ["-i", "x", "--sizediff-tresh", ""], {}),
    ("uncomp", ["-i", "x", "-i", "y"], {}),
    ("uncomp", ["-i", "x", "--notest", "--notest"], {}),
    ("uncomp", ["-r", "-r", "-i", "x"], {}),
    ("uncomp", ["-rh"], {}),
    ("uncomp", ["-hr"], {}),
    ("uncomp", ["-hh"], {}),
    ("uncomp", ["-rr", "-i", "x"], {}),
    ("uncomp", ["-ri", "x"], {}),
    ("uncomp", ["-ix"], {}),
    ("uncomp", ["-i x"], {}),
    ("uncomp", ["--input x"], {}),
    ("uncomp", ["--input=x"], {}),
    ("uncomp", ["--chunksize=5", "-i", "x"], {}),
    ("uncomp", ["-i", "x", "--brute-window=1"], {}),
    ("uncomp", ["---i", "x"], {}),
    ("uncomp", ["-", "-i", "x"], {}),
    ("uncomp", ["", "-i", "x"], {}),
    ("uncomp", ["-i", "x", "--", "-z", "--bogus"], {}),
    ("uncomp", ["--", "-i", "x"], {}),
    ("uncomp", ["-i", "x", "--ignore_rest", "--", "-h"], {}),
    ("uncomp", ["-h", "--bogus"], {}),
    ("uncomp", ["--bogus", "-h"], {}),
    ("uncomp", ["-i", "x", "--version"], {}),
    ("uncomp", ["--version", "--bogus"], {}),
    ("uncomp", ["--version", "-h"], {}),
    ("uncomp", ["-i", ""], {}),
    ("uncomp", ["-i", "x"], {}),
    ("uncomp", ["-i", "x", "-o", "y", "--notest", "--brute-window"], {}),
    ("uncomp", ["--input", "x", "--output", "y"], {}),
    ("uncomp", ["--reconstruct", "--input", "x"], {}),
    ("uncomp", ["-r", "-i", "x", "-o", "y"], {}),
    ("uncomp", ["-r", "-i", "bad.atz"], {"bad.atz": b"hello, not an atz file"}),
    ("uncomp", ["-r", "-i", "size.atz"], {"size.atz": b"ATZ\x01" + (99).to_bytes(8, "little") + bytes(20)}),
    ("uncomp", ["-i", "x", "-r", "--chunksize", "77"], {}),
]


def run(exe, prog, args, files):
    with tempfile.TemporaryDirectory() as d:
        for n, b in files.items():
            with open(os.path.join(d, n), "wb") as f:
                f.write(b)
        r = subprocess.run([prog] + args, executable=exe, cwd=d, capture_output=True, timeout=60)
        left = sorted(set(os.listdir(d)) - set(files))
    return {"rc": r.returncode, "stdout": r.stdout.decode("latin-1"), "stderr": r.stderr.decode("latin-1"),
            "files_left": left}


def main():
    out = []
    for prog, args, files in CASES:
        res = run(_libs.REF_UNCOMP, prog, args, files)
        out.append({"prog": prog, "args": args,
                    "files": {n: base64.b64encode(b).decode() for n, b in files.items()}, **res})
    with open(os.path.join(HERE, "cli_cases.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_cli_golden.py (oracle/_ref/uncomp)", "cases": out}, f, indent=1)
    print("wrote", len(out), "cases")


if __name__ == "__main__":
    main()
