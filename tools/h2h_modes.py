"""atz_precompress (host buffer in, host ATZ1 out) under each ATZ_H2H_PREP mode, interleaved, against the
device-resident precompress of the same file: 0 = plain malloc after the sweep, 1 = buffer touched
during the sweep, 2 = touched and registered with HIP in 64 MB pieces (default).  Run on the GPU box."""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["ATZ_H2H_TIMING"] = "1"
import torch  # noqa: E402
import antiz_amd  # noqa: E402
from antiz_amd import datagen  # noqa: E402

data = open(datagen.cached("c4", "/tmp/atz_bench_cache", seed=4, n_streams=100000), "rb").read()
dev = torch.frombuffer(bytearray(data) + bytearray(4096), dtype=torch.uint8).to("cuda")
ctx = antiz_amd.Context(device=0)
L = antiz_amd.lib()
p, n, st = ctypes.POINTER(ctypes.c_uint8)(), ctypes.c_uint64(0), antiz_amd.Stats()
ctx.precompress_device(dev.data_ptr(), data)
for rep in range(2):
    for mode in ("dev", "0", "1", "2"):
        t0 = time.perf_counter()
        if mode == "dev":
            ctx.precompress_device(dev.data_ptr(), data)
        else:
            os.environ["ATZ_H2H_PREP"] = mode
            assert L.atz_precompress(ctx.h, data, len(data), ctypes.byref(p), ctypes.byref(n), ctypes.byref(st)) == 0
            L.atz_free(p)
        print("rep %d mode %-3s %7.1f ms" % (rep, mode, (time.perf_counter() - t0) * 1e3), flush=True)
