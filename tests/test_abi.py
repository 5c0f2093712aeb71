"""CPU-side checks of the drop-in boundary: the HIP library builds for gfx950, exports every entry point
include/atz_accel.h declares, and refuses to run (no CPU fallback) when no MI355X is present."""
import os
import re
import subprocess

import pytest

import antiz_amd
from antiz_amd import build as B

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def built():
    B.build()
    return B.LIB


def declared_functions():
    hdr = open(os.path.join(ROOT, "include", "atz_accel.h")).read()
    hdr = re.sub(r"/\*.*?\*/", "", hdr, flags=re.S)
    return sorted(set(re.findall(r"\b(atz_[a-z_]+)\s*\(", hdr)))


def test_exports_every_declared_symbol(built):
    out = subprocess.run(["nm", "-D", "--defined-only", built], capture_output=True, text=True).stdout
    exported = set(re.findall(r" T (atz_\w+)", out))
    decl = declared_functions()
    assert decl, "no declarations parsed"
    missing = [f for f in decl if f not in exported]
    assert not missing, missing
    assert set(antiz_amd.EXPORTS) <= set(decl)


def test_code_object_targets_gfx950(built, tmp_path):
    fb = str(tmp_path / "fatbin.bin")
    subprocess.run(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", built, fb], check=True)
    r = subprocess.run(["/opt/rocm/lib/llvm/bin/clang-offload-bundler", "--list", "--type=o", "--input=" + fb],
                       capture_output=True, text=True, check=True)
    assert "hipv4-amdgcn-amd-amdhsa--gfx950" in r.stdout


def test_cli_built(built):
    assert os.path.exists(B.CLI)


def test_no_cpu_fallback_without_gpu(built):
    import torch
    if torch.cuda.device_count() > 0:
        pytest.skip("GPU present")
    with pytest.raises(antiz_amd.AtzError):
        antiz_amd.Context()
