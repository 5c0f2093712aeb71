"""Diagnostic: k_inflate throughput on the C4 workload's real streams at several batch sizes."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import antiz_amd
from antiz_amd import datagen

path = datagen.cached("c4", "/tmp/atz_bench_cache", seed=4, n_streams=100000)
data = open(path, "rb").read()
with antiz_amd.Context(device=0) as c:
    t0 = time.perf_counter()
    recs = c.scan(data)
    print("scan %.1f ms, %d records" % ((time.perf_counter() - t0) * 1e3, len(recs)), flush=True)
    c._cands = None
    sizes = [int(x) for x in os.environ.get("EXP_N", "1000,4000,16000,0").split(",")]
    for n in [x or len(recs) for x in sizes]:
        sel = recs[:n]
        buf = bytearray()
        rng = []
        for (off, typ, cl, il, fl) in sel:
            rng.append((len(buf), cl))
            buf += data[off:off + cl]
            buf += bytes((-len(buf)) % 4)
        buf = bytes(buf) + bytes(4096)
        c.inflate_batch(buf, rng[:10])
        t0 = time.perf_counter()
        r = c.inflate_batch(buf, rng)
        dt = time.perf_counter() - t0
        tot_out = sum(x[2] for x in r)
        print("n=%6d  %.1f ms  out %.1f MB  -> %.1f MB/s  ok=%d" % (n, dt * 1e3, tot_out / 1e6, tot_out / 1e6 / dt,
              sum(1 for x in r if x[0] == 0)), flush=True)
