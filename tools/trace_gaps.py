#!/usr/bin/env python3
"""Kernel timeline of a rocprofv3 --kernel-trace run (tools/trace_share.sh): for the last precompress step
(the run's last k_headers_ordered launch to its last kernel), per kernel class the launches, summed and
wall-clock busy time, and the time with no trial kernel / no kernel at all running; per hardware queue its
busy fraction.  usage: python3 tools/trace_gaps.py <rocprofv3 output dir>"""
import csv
import glob
import os
import re
import sys


def cls(name):
    for k in ("k_trial", "k_match", "k_buckets_sort", "k_bucket_depth", "k_buckets", "k_inflate", "k_headers",
              "k_gather", "k_diffs", "k_adler32", "copyBuffer", "fillBuffer"):
        if k in name:
            return k
    return "other"


def union(iv):
    iv = sorted(iv)
    tot, cs, ce = 0, None, None
    for s, e in iv:
        if cs is None or s > ce:
            if cs is not None:
                tot += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    if cs is not None:
        tot += ce - cs
    return tot


def main():
    files = glob.glob(os.path.join(sys.argv[1], "**", "*kernel_trace.csv"), recursive=True)
    rows = []
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r.get("Queue_Id", "?")))
    rows.sort()
    heads = [r for r in rows if "k_headers_ordered" in r[2]]
    t0 = heads[-2][0] if len(heads) >= 2 else rows[0][0]   # the last step's scan (two header passes)
    step = [r for r in rows if r[0] >= t0]
    t1 = max(r[1] for r in step)
    span = t1 - t0
    print("last step: %.2f ms, %d kernels" % (span / 1e6, len(step)))
    by = {}
    for s, e, n, q in step:
        by.setdefault(cls(n), []).append((s, e))
    print("%-16s %8s %12s %12s %8s" % ("class", "launches", "summed ms", "busy ms", "busy %"))
    for k, iv in sorted(by.items(), key=lambda kv: -union(kv[1])):
        print("%-16s %8d %12.2f %12.2f %7.1f%%" % (k, len(iv), sum(e - s for s, e in iv) / 1e6, union(iv) / 1e6,
                                               100.0 * union(iv) / span))
    allb = union([(s, e) for s, e, _, _ in step])
    trial = union(by.get("k_trial", []))
    print("any kernel running %.1f%%, a trial kernel running %.1f%%, idle %.2f ms" % (100.0 * allb / span, 100.0 * trial / span,
                                                                                    (span - allb) / 1e6))
    timeline(step, t0, t1)
    qs = {}
    for s, e, n, q in step:
        qs.setdefault(q, []).append((s, e))
    for q, iv in sorted(qs.items()):
        # overlap: summed minus union (0: the queue's kernels never ran at once); gaps between a kernel's
        # end and the next one's start on the same queue
        iv.sort()
        gaps = sorted(max(0, iv[i + 1][0] - iv[i][1]) for i in range(len(iv) - 1))
        med = gaps[len(gaps) // 2] / 1e3 if gaps else 0.0
        print("queue %s: %d kernels, busy %.1f%%, overlap %.2f ms, gap median %.1f us, gaps < 20 us %d" %
              (q, len(iv), 100.0 * union(iv) / span, (sum(e - s for s, e in iv) - union(iv)) / 1e6, med,
               sum(1 for g in gaps if g < 20000)))
    # concurrency of kernel classes over time, 2 ms bins
    nb = int(span // 2e6) + 1
    print("per 2 ms: running kernels by class (trial/match/buckets/other)")
    out = []
    for b in range(nb):
        lo, hi = t0 + b * 2e6, t0 + (b + 1) * 2e6
        cnt = [0, 0, 0, 0]
        for s, e, n, q in step:
            if s < hi and e > lo:
                c = cls(n)
                cnt[0 if c == "k_trial" else 1 if c == "k_match" else 2 if c.startswith("k_bucket") else 3] += 1
        out.append("%d/%d/%d/%d" % tuple(cnt))
    print(" ".join(out))


def timeline(step, t0, t1, bin_ms=10.0):
    """Per bin: the busy fraction of each kernel class (union of its launches within the bin)."""
    b = int(bin_ms * 1e6)
    classes = ("k_inflate", "k_buckets_sort", "k_match", "k_trial", "idle")
    print("%-10s" % "ms" + "".join("%15s" % c for c in classes))
    for a in range(t0, t1, b):
        e = min(a + b, t1)
        row = []
        allv = []
        for c in classes[:-1]:
            iv = [(max(s, a), min(en, e)) for s, en, n, _ in step if cls(n) == c and en > a and s < e]
            allv += iv
            row.append(union(iv) / (e - a))
        anyb = union([(max(s, a), min(en, e)) for s, en, n, _ in step if en > a and s < e])
        row.append(1.0 - anyb / (e - a))
        print("%-10.0f" % ((a - t0) / 1e6) + "".join("%14.0f%%" % (100 * v) for v in row))


if __name__ == "__main__":
    main()
