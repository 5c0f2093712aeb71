"""GPU occupancy over time from a rocprofv3 --kernel-trace CSV (one bench step): the union of kernel
intervals (busy time), time with 0/1/2/3+ kernels in flight, and per-kernel-family busy time, for the
last precompress call (the window from the first k_headers_ordered of it to the end).
usage: python3 tools/trace_busy.py <kernel_trace.csv>"""
import csv
import sys
from collections import defaultdict


def family(name):
    for k in ("k_trial_fast", "k_trial_slow", "k_trial_stored", "k_match_lds", "k_match", "k_buckets_sort",
              "k_bucket_depth", "k_buckets", "k_inflate", "k_headers", "k_diffs", "k_gather", "copyBuffer", "fillBuffer"):
        if k in name:
            return k
    return name[:40]


rows = list(csv.DictReader(open(sys.argv[1])))
ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), family(r["Kernel_Name"])) for r in rows]
ev.sort()
starts = [s for s, e, f in ev if f == "k_headers"]
t0 = starts[-2] if len(starts) >= 2 else ev[0][0]   # each precompress launches k_headers_ordered twice
ev = [x for x in ev if x[0] >= t0]
t1 = max(e for s, e, f in ev)
pts = []
for s, e, f in ev:
    pts.append((s, 1))
    pts.append((e, -1))
pts.sort()
conc = defaultdict(int)
cur, last = 0, t0
for t, d in pts:
    conc[min(cur, 3)] += t - last
    cur += d
    last = t
fam = defaultdict(int)
for s, e, f in ev:
    fam[f] += e - s
span = t1 - t0
print("window %.1f ms; busy %.1f ms (%.0f %%); idle %.1f ms" % (span / 1e6, (span - conc[0]) / 1e6,
      100 * (span - conc[0]) / span, conc[0] / 1e6))
for k in (1, 2, 3):
    print("  %s kernels in flight: %.1f ms" % (k if k < 3 else "3+", conc[k] / 1e6))
for f, v in sorted(fam.items(), key=lambda x: -x[1]):
    print("  %-16s %8.1f ms summed" % (f, v / 1e6))
# idle gaps over time (10 ms bins)
bins = defaultdict(int)
cur, last = 0, t0
for t, d in pts:
    if cur == 0:
        a = last
        while a < t:
            b = min(t, (a // 10_000_000 + 1) * 10_000_000)
            bins[(a - t0) // 10_000_000] += b - a
            a = b
    cur += d
    last = t
print("idle per 10 ms bin:", " ".join("%d" % (bins[i] / 1e6 * 10) for i in range(int(span // 10_000_000) + 1)), "(tenths of ms)")
