#!/usr/bin/env python3
"""Register, spill, scratch, LDS and occupancy figures of every kernel in libatz_accel, from the
compiler's own report (hipcc -Rpass-analysis=kernel-resource-usage, gfx950).
usage: python3 tools/kernel_resources.py [out.txt]   (compiles to a temporary .so; ~40 s; ATZ_HIPFLAGS: extra flags)"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIELDS = [("TotalSGPRs", "sgpr"), ("VGPRs", "vgpr"), ("AGPRs", "agpr"), ("ScratchSize [bytes/lane]", "scratch"),
          ("Occupancy [waves/SIMD]", "occ"), ("SGPRs Spill", "sgpr_spill"), ("VGPRs Spill", "vgpr_spill"),
          ("LDS Size [bytes/block]", "lds_static")]


def main():
    src = os.path.join(ROOT, "antiz_amd", "csrc", "atz_accel.cpp")
    with tempfile.TemporaryDirectory() as td:
        cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", "-x", "hip",
               "-Wno-unused-result", "-Wno-unused-value", "-Rpass-analysis=kernel-resource-usage", src,
               "-o", os.path.join(td, "lib.so")] + os.environ.get("ATZ_HIPFLAGS", "").split()
        r = subprocess.run(cmd, capture_output=True, text=True, check=True)
    rows, cur = [], None
    for line in r.stderr.splitlines():
        m = re.search(r"remark:\s+(Function Name|[A-Za-z ]+(?:\[[^\]]*\])?): (\S+)", line)
        if not m:
            continue
        k, v = m.group(1).strip(), m.group(2)
        if k == "Function Name":
            cur = {"name": v}
            rows.append(cur)
        elif cur is not None:
            cur[k] = v
    sha = subprocess.run(["git", "-C", ROOT, "rev-parse", "--short", "HEAD"], capture_output=True, text=True).stdout.strip()
    out = ["# kernel resources, hipcc -Rpass-analysis=kernel-resource-usage, gfx950, code at %s" % sha,
           "# lds_static excludes dynamic LDS (k_buckets_sort / k_match_lds size it per launch)",
           "%-64s " % "kernel" + " ".join("%10s" % s for _, s in FIELDS)]
    for row in rows:
        dem = subprocess.run(["c++filt", row["name"]], capture_output=True,
                             text=True).stdout.strip() or row["name"]
        dem = re.sub(r"\(.*\)$", "", dem.replace("(anonymous namespace)", "anon"))
        out.append("%-64s " % dem[:64] + " ".join("%10s" % row.get(f, "-") for f, _ in FIELDS))
    text = "\n".join(out) + "\n"
    if len(sys.argv) > 1:
        open(sys.argv[1], "w").write(text)
    sys.stdout.write(text)


if __name__ == "__main__":
    main()
