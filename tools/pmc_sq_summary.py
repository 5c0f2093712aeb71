#!/usr/bin/env python3
"""Issue utilisation per kernel family from two rocprofv3 SQ counter passes (tools/measure.sh ... sq):
   tools/pmc_sq_summary.py <sq1 dir> <sq2 dir> <out.json> [code sha]

rocprofv3 serialises the dispatches while it collects counters, so every figure describes a kernel
running alone on the GPU.  Units (MI355X guide, 'rocprofv3 PMC slots' and the cycle-constants table):
SQ_WAVE_CYCLES, SQ_WAIT_*, SQ_ACTIVE_INST_* and SQ_BUSY_CYCLES count quad-cycles; GRBM_GUI_ACTIVE
counts GPU cycles over the dispatch summed over the 8 XCDs (elapsed = GRBM_GUI_ACTIVE / 8: k_inflate's
one dispatch, 78 ms in the kernel trace, reads 1.46e9).  Capacities used for the fractions (gfx950: 256 CUs, one scalar
unit and 4 SIMD-32 per CU, the sequencer issuing for one SIMD per cycle):
  salu_issue_frac = SQ_INSTS_SALU / (256 CUs x elapsed)      (one SALU per CU per cycle)
  valu_issue_frac = 2 x SQ_INSTS_VALU / (4 x 256 x elapsed)  (wave64 on a SIMD-32: 2 cycles)
  lds_issue_frac  = SQ_INSTS_LDS / (256 x elapsed)           (one LDS instruction per CU per cycle)
  wait_frac       = SQ_WAIT_ANY / SQ_WAVE_CYCLES   (waves parked on s_waitcnt / barriers)
  stall_frac      = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES (waves ready but not issued: pipe busy, dependency)
  active_frac     = SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES
  waves_resident  = 4 x SQ_WAVE_CYCLES / elapsed (mean waves on the GPU while the kernel ran)
"""
import collections
import csv
import glob
import json
import os
import sys

FAMILIES = ("k_trial_fast_mw", "k_trial_slow_mw", "k_trial_fast", "k_trial_slow", "k_trial_stored", "k_match_lds",
            "k_match", "k_buckets_sort", "k_bucket_depth", "k_buckets", "k_inflate", "k_headers", "k_diffs", "k_gather",
            "copyBuffer", "fillBuffer")


def family(name):
    for f in FAMILIES:
        if f in name:
            return f
    return name[:40]


def load(d):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(f)):
        k = family(r["Kernel_Name"])
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
    for k in acc:
        acc[k]["dispatches"] = len(disp[k])
    return acc


def main():
    d1, d2, out = sys.argv[1:4]
    sha = sys.argv[4] if len(sys.argv) > 4 else None
    a, b = load(d1), load(d2)
    fam = {}
    for k in sorted(set(a) | set(b), key=lambda k: -a[k].get("SQ_WAVE_CYCLES", 0)):
        c = dict(a[k])
        for n, v in b[k].items():
            if n in ("GRBM_GUI_ACTIVE", "dispatches"):
                c[n + "_pass2"] = v
            else:
                c[n] = v
        g = (c.get("GRBM_GUI_ACTIVE", 0) or 8) / 8.0
        wc = c.get("SQ_WAVE_CYCLES", 0) or 1
        e = {"counters": {n: int(v) for n, v in c.items()}}
        e["salu_issue_frac"] = round(c.get("SQ_INSTS_SALU", 0) / (256 * g), 4)
        e["valu_issue_frac"] = round(2 * c.get("SQ_INSTS_VALU", 0) / (4 * 256 * g), 4)
        e["lds_issue_frac"] = round(c.get("SQ_INSTS_LDS", 0) / (256 * g), 4)
        e["wait_frac"] = round(c.get("SQ_WAIT_ANY", 0) / wc, 4)
        e["stall_frac"] = round(c.get("SQ_WAIT_INST_ANY", 0) / wc, 4)
        e["active_frac"] = round(c.get("SQ_ACTIVE_INST_ANY", 0) / wc, 4)
        e["scalar_active_frac"] = round(c.get("SQ_ACTIVE_INST_SCA", 0) / wc, 4)
        e["waves_resident"] = round(4 * wc / g, 1)
        e["salu_per_valu"] = round(c.get("SQ_INSTS_SALU", 0) / max(1, c.get("SQ_INSTS_VALU", 0)), 3)
        fam[k] = e
    tk = [k for k in fam if k.startswith("k_trial")]
    tot = collections.defaultdict(float)
    for k in tk:
        for n, v in fam[k]["counters"].items():
            tot[n] += v
    g = (tot.get("GRBM_GUI_ACTIVE", 0) or 8) / 8.0
    wc = tot.get("SQ_WAVE_CYCLES", 0) or 1
    trial = {"salu_issue_frac": round(tot["SQ_INSTS_SALU"] / (256 * g), 4),
             "valu_issue_frac": round(2 * tot["SQ_INSTS_VALU"] / (4 * 256 * g), 4),
             "lds_issue_frac": round(tot["SQ_INSTS_LDS"] / (256 * g), 4),
             "wait_frac": round(tot["SQ_WAIT_ANY"] / wc, 4), "stall_frac": round(tot["SQ_WAIT_INST_ANY"] / wc, 4),
             "active_frac": round(tot.get("SQ_ACTIVE_INST_ANY", 0) / wc, 4),
             "waves_resident": round(4 * wc / g, 1)}
    res = {"source": "rocprofv3 --pmc (two SQ passes + GRBM_GUI_ACTIVE) -- python3 bench.py --steps 1 --warmup 0 "
                     "--no-cpu --no-recon --no-h2h, full C4 (100 000 streams, 1.007 GB), one MI355X; dispatches "
                     "serialised by the profiler",
           "definitions": __doc__.split("Units")[1].strip(), "code_sha": sha, "k_trial": trial, "kernels": fam}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({"k_trial": trial}))
    for k in list(fam)[:8]:
        e = fam[k]
        print("%-16s salu %.3f valu %.3f lds %.3f wait %.3f stall %.3f active %.3f waves %.0f" % (
            k, e["salu_issue_frac"], e["valu_issue_frac"], e["lds_issue_frac"], e["wait_frac"], e["stall_frac"],
            e["active_frac"], e["waves_resident"]))


if __name__ == "__main__":
    main()
