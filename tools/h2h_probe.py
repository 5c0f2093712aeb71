"""Where the host-buffer path's extra time goes: H2D of a 1 GB pageable buffer and
D2H of 1.56 GB (the C4 ATZ1 size) into fresh / reused / pinned host memory, one copy or split over
threads on their own streams.  Prints one line per case (ms, GB/s).  Run on the GPU box."""
import ctypes
import threading
import time

import numpy as np
import torch

hip = ctypes.CDLL("libamdhip64.so")
hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
hip.hipStreamCreate.argtypes = [ctypes.POINTER(ctypes.c_void_p)]
hip.hipStreamSynchronize.argtypes = [ctypes.c_void_p]
hip.hipHostMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
H2D, D2H = 1, 2

IN, OUT = 1_007_000_000, 1_558_434_085
dev_in = torch.empty(IN, dtype=torch.uint8, device="cuda")
dev_out = torch.randint(0, 255, (OUT,), dtype=torch.uint8, device="cuda")
host_in = np.random.default_rng(0).integers(0, 255, IN, dtype=np.uint8)
torch.cuda.synchronize()


def t(name, f, nbytes, reps=3):
    best = 1e9
    for _ in range(reps):
        t0 = time.perf_counter()
        f()
        dt = time.perf_counter() - t0
        best = min(best, dt)
    print("%-52s %8.1f ms %6.1f GB/s" % (name, best * 1e3, nbytes / best / 1e9), flush=True)


def copy(dst, src, n, kind):
    assert hip.hipMemcpy(dst, src, n, kind) == 0


def split(dst, src, n, kind, k):
    streams = []
    for _ in range(k):
        s = ctypes.c_void_p()
        hip.hipStreamCreate(ctypes.byref(s))
        streams.append(s)
    part = (n + k - 1) // k

    def run(i):
        a = i * part
        b = min(n, a + part)
        assert hip.hipMemcpyAsync(dst + a, src + a, b - a, kind, streams[i]) == 0
        hip.hipStreamSynchronize(streams[i])

    def go():
        th = [threading.Thread(target=run, args=(i,)) for i in range(k)]
        for x in th:
            x.start()
        for x in th:
            x.join()
    return go


t("H2D 1 GB pageable (one hipMemcpy)", lambda: copy(dev_in.data_ptr(), host_in.ctypes.data, IN, H2D), IN)
for k in (2, 4, 8):
    t("H2D 1 GB pageable, %d threads/streams" % k, split(dev_in.data_ptr(), host_in.ctypes.data, IN, H2D, k), IN)
reuse = np.empty(OUT, dtype=np.uint8)
reuse[::4096] = 1


def fresh_one():
    b = np.empty(OUT, dtype=np.uint8)
    copy(b.ctypes.data, dev_out.data_ptr(), OUT, D2H)


t("D2H 1.56 GB into fresh pageable (one hipMemcpy)", fresh_one, OUT)
t("D2H 1.56 GB into reused pageable (one hipMemcpy)", lambda: copy(reuse.ctypes.data, dev_out.data_ptr(), OUT, D2H), OUT)
for k in (2, 4, 8):
    def fresh_k(k=k):
        b = np.empty(OUT, dtype=np.uint8)
        split(b.ctypes.data, dev_out.data_ptr(), OUT, D2H, k)()
    t("D2H 1.56 GB into fresh pageable, %d threads/streams" % k, fresh_k, OUT)
    t("D2H 1.56 GB into reused pageable, %d threads/streams" % k,
      split(reuse.ctypes.data, dev_out.data_ptr(), OUT, D2H, k), OUT)
p = ctypes.c_void_p()
t0 = time.perf_counter()
assert hip.hipHostMalloc(ctypes.byref(p), OUT, 0) == 0
print("%-52s %8.1f ms" % ("hipHostMalloc 1.56 GB", (time.perf_counter() - t0) * 1e3), flush=True)
t("D2H 1.56 GB into pinned (one hipMemcpy)", lambda: copy(p.value, dev_out.data_ptr(), OUT, D2H), OUT)
t("memcpy 1.56 GB pinned -> fresh pageable (numpy)", lambda: np.frombuffer(
    (ctypes.c_uint8 * OUT).from_address(p.value), dtype=np.uint8).copy(), OUT)
