"""Build the MI355X product: antiz_amd/_build/libatz_accel.so (HIP, gfx950) and antiz_amd/_build/uncomp (CLI).

Plain hipcc invocations (no cmake/ninja needed); outputs stay in-tree so they travel to the GPU box.
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "_build")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"
LIB = os.path.join(OUT, "libatz_accel.so")
CLI = os.path.join(OUT, "uncomp")


def _newer(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd):
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout + r.stderr)
        raise RuntimeError("build failed: " + " ".join(cmd))


def build(force=False, verbose=False):
    os.makedirs(OUT, exist_ok=True)
    srcs = [os.path.join(CSRC, f) for f in ("atz_accel.cpp", "k_inflate.hip", "k_deflate.hip", "atz_device.h")]
    srcs.append(os.path.join(os.path.dirname(HERE), "include", "atz_accel.h"))
    if force or _newer(LIB, srcs):
        cmd = [HIPCC, "--offload-arch=" + ARCH, "-O3", "-std=c++17", "-fPIC", "-shared", "-x", "hip",
               "-Wno-unused-result", "-Wno-unused-value", "-Xarch_host", "-gline-tables-only",
               os.path.join(CSRC, "atz_accel.cpp"), "-o", LIB] + os.environ.get("ATZ_HIPFLAGS", "").split()
        if verbose:
            print(" ".join(cmd))
        _run(cmd)
    cli_src = os.path.join(CSRC, "uncomp.cpp")
    if force or _newer(CLI, [cli_src, LIB]):
        cmd = ["g++", "-O2", "-std=c++17", cli_src, "-I" + os.path.join(os.path.dirname(HERE), "include"),
               "-L" + OUT, "-latz_accel", "-Wl,-rpath,$ORIGIN", "-o", CLI]
        if verbose:
            print(" ".join(cmd))
        _run(cmd)
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv, verbose=True)
    print("built", LIB, CLI)
