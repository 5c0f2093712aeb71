#!/usr/bin/env python3
"""bench.py -- input MB/s precompressed on MI355X (BASELINE.json metric), one JSON line on rank 0.

Workload (BASELINE.json configs[3]): 1 GB synthetic file, 100 000 zlib streams,
clevel U{1..9} x memLevel U{1..9}, w15, ~10 KB compressed each, 0-64 B random gaps, seed 4.
A step = one full precompress (Phase 1 scan+inflate, Phase 3 parameter sweep, Phase 4 ATZ1 assembly)
of that file, input already resident in HBM, ATZ1 output assembled in HBM.

Multi-GPU (python -m torch.distributed.run --nproc-per-node N bench.py --gpus N): by default ONE 1 GB
file (config 4: "1 GB synthetic, 100k streams, stream-sharded across 8 x MI355X") is split over the
ranks (--mode file, antiz_amd.shard): an all-gather of the scan results, a cost-balanced split of the
streams, and a gather of the ATZ1 pieces to rank 0 over RCCL -- strong scaling.  --mode shards (every
rank its own 1 GB file, seed 4 + rank: weak scaling) is a labelled secondary line.

roofline: the dominant kernel (k_trial_*: deflate trials) -- achieved = algorithmic bytes
(trial input read + compare read, summed over the launches) / the kernels' summed
device time (HIP events recorded inside libatz_accel on its own stream), peak = MI355X HBM 8 TB/s;
achieved_wall divides the same bytes by the step's wall time (the pipes' launches overlap).
cpu_baseline: the REAL reference (oracle/_ref/uncomp, built from /root/reference) on a bounded
sample of the same workload (first seed, fewer streams), 1 core, --notest; the host CPU is named.
host_to_host: atz_precompress from a host buffer to host ATZ1 bytes (H2D + D2H included), the path
the uncomp CLI takes; reported beside the metric, never as its value.
"""
import argparse
import hashlib
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_model():
    """The host CPU the baseline runs on (/proc/cpuinfo), and the cores this process may use."""
    name = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    name = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return name, len(os.sched_getaffinity(0))


def cpu_baseline(n_streams, seed, ctx, workload="c4"):
    """Time the real reference binary on a bounded sample of the workload (1 thread), and check that
    the library's .atz of the same sample is byte-identical to the reference's (parity at the bench
    configuration: same generator, seed and options, 3 sweep pipes)."""
    import hashlib
    from antiz_amd import datagen
    ref = os.path.join(ROOT, "oracle", "_ref", "uncomp")
    if not os.path.exists(ref):
        return None
    if workload == "c2":     # the whole config: the reference takes ~3 s on it
        data, what = datagen.gen_c2(), "the whole C2 config"
    elif workload == "c3":   # a 10 MB prefix config of the same mix (the reference: ~1 MB/s here)
        data, what = datagen.gen_c3(seed=seed, total=10 * 1000 * 1000), "a 10 MB config of the same C3 mix"
    else:
        data = datagen.CONFIGS[workload](seed=seed, n_streams=n_streams)
        what = "%d-stream prefix config of the same generator" % n_streams
    d = tempfile.mkdtemp(prefix="atzcpu")
    p = os.path.join(d, "sample.bin")
    with open(p, "wb") as f:
        f.write(data)
    cmd = [ref, "-i", p, "-o", p + ".atz", "--notest"] + (["--brute-window"] if workload == "c5" else [])
    try:
        cmd = ["taskset", "-c", "0"] + cmd if subprocess.run(["which", "taskset"], capture_output=True).returncode == 0 else cmd
        t0 = time.perf_counter()
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
        dt = time.perf_counter() - t0
        ok = r.returncode == 0
        ref_sha = None
        if ok:
            with open(p + ".atz", "rb") as f:
                ref_sha = hashlib.sha256(f.read()).hexdigest()
    finally:
        for fn in (p, p + ".atz"):
            if os.path.exists(fn):
                os.remove(fn)
        os.rmdir(d)
    if not ok:
        return None
    atz, _ = ctx.precompress(data)
    same = hashlib.sha256(atz).hexdigest() == ref_sha
    if not same:
        log("PARITY FAILURE: the library's .atz of the cpu_baseline sample differs from the reference's")
    model, visible = cpu_model()
    return {"value": round(len(data) / 1e6 / dt, 4), "unit": "MB/s", "cores": 1, "kind": "reference",
            "cpu_model": model, "host_cpus_visible": visible,
            "atz_identical_to_reference": same, "atz_sha256": ref_sha[:16],
            "sample": "%s (%.1f MB, seed %d), oracle/_ref/uncomp --notest, "
                      "%.1f s wall" % (what, len(data) / 1e6, seed, dt)
                      + (" --brute-window" if workload == "c5" else "")}


def hip_copy(dst, src, n):
    """hipMemcpy(dst, src, n, hipMemcpyDefault) on raw pointers (the library's device buffers)."""
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    if n and hip.hipMemcpy(dst, src, n, 4) != 0:
        raise RuntimeError("hipMemcpy failed")


def pmc_traffic():
    """HBM traffic per k_trial launch from the newest committed PMC summary (profiles/r*_pmc_traffic.json:
    separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over this bench, FETCH_SIZE doubled per the
    MI355X guide's gfx950 correction). rocprofv3 cannot run inside the timed process, so the counter
    passes are their own runs of the same command; the file named here is the one used, and its
    "code_sha" (the commit the passes ran, when recorded) shows which code it measured."""
    import glob
    import re
    files = glob.glob(os.path.join(ROOT, "profiles", "r*_v*_pmc_traffic.json"))
    if not files:
        return None, None, None
    key = lambda p: tuple(int(x) for x in re.findall(r"r(\d+)_v(\d+)_", os.path.basename(p))[0])
    path = max(files, key=key)
    with open(path) as f:
        d = json.load(f)
    return d["k_trial"]["traffic_per_launch"], os.path.relpath(path, ROOT), d.get("code_sha")


def pmc_issue():
    """Issue utilisation of the trial kernels from the newest committed SQ profile (profiles/r*_v*_pmc_sq.json:
    two rocprofv3 --pmc SQ passes over this bench with GRBM_GUI_ACTIVE, made by tools/pmc_sq_summary.py;
    dispatches serialised by the profiler).  Fractions of the CU's scalar-issue, VALU-issue and LDS-issue
    capacity, and of the waves' cycles spent parked on s_waitcnt (wait) or ready but not issued (stall)."""
    import glob
    import re
    files = glob.glob(os.path.join(ROOT, "profiles", "r*_v*_pmc_sq.json"))
    if not files:
        return None
    key = lambda p: tuple(int(x) for x in re.findall(r"r(\d+)_v(\d+)_", os.path.basename(p))[0])
    path = max(files, key=key)
    with open(path) as f:
        d = json.load(f)
    t = d["k_trial"]
    out = {k: t[k] for k in ("salu_issue_frac", "valu_issue_frac", "lds_issue_frac", "wait_frac", "stall_frac",
                             "active_frac", "waves_resident")}
    out["source"] = os.path.relpath(path, ROOT)
    out["code_sha"] = d.get("code_sha")
    inf = d["kernels"].get("k_inflate")
    if inf:
        out["k_inflate_salu_issue_frac"] = inf["salu_issue_frac"]
    return out


def aggregate(dt, atz_len, shard_bytes, steps, world, device):
    """Cross-rank reduction of one timed run: max step time over ranks, per-rank ATZ sizes.
    value = bytes all ranks processed / the slowest rank's time (weak scaling: one shard per rank)."""
    import torch
    import torch.distributed as dist
    tmax = torch.tensor([dt], dtype=torch.float64, device=device)
    sizes = torch.tensor([float(atz_len)], dtype=torch.float64, device=device)
    gathered = [sizes]
    if world > 1:
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        gathered = [torch.zeros_like(sizes) for _ in range(world)]
        dist.all_gather(gathered, sizes)
    dt = float(tmax.item())
    total_bytes = shard_bytes * world
    value = total_bytes / 1e6 / (dt / steps)
    return dt, value, [int(g.item()) for g in gathered]


def rank_balance(st, world, device):
    """Per-rank work of the last step (all-gathered): streams swept, trials, the trials' algorithmic bytes
    (input parsed + output compared), shader cycles the trials took, sweep wall time.  max/mean
    of the algorithmic bytes shows how evenly the split (atz_accel.cpp shard_records) shared the work;
    the cycles say the same on one GPU per rank, but with several ranks sharing one GPU (a gloo
    rehearsal) they also count the waits the co-running ranks cause."""
    import torch
    import torch.distributed as dist
    keys = ("n_streams", "n_trials", "k_trial_alg_bytes", "trial_cyc_total", "sweep_ms", "k_trial_ms")
    mine = torch.tensor([float(st[k]) for k in keys], dtype=torch.float64, device=device)
    allr = [torch.zeros_like(mine) for _ in range(world)]
    dist.all_gather(allr, mine)
    cols = {k: [float(r[i].item()) for r in allr] for i, k in enumerate(keys)}
    cyc = cols["trial_cyc_total"]
    mean = sum(cyc) / len(cyc) if cyc else 0.0
    out = {k: [int(v) if k != "sweep_ms" and k != "k_trial_ms" else round(v, 1) for v in vals] for k, vals in cols.items()}
    out["cyc_max_over_mean"] = round(max(cyc) / mean, 4) if mean > 0 else None
    alg = cols["k_trial_alg_bytes"]
    amean = sum(alg) / len(alg) if alg else 0.0
    out["alg_max_over_mean"] = round(max(alg) / amean, 4) if amean > 0 else None
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--streams", type=int, default=100000, help="streams per rank (C4: 100000 = 1 GB)")
    ap.add_argument("--cpu-sample-streams", type=int, default=8000)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-recon", action="store_true", help="skip the reconstruct (-r / verify) measurement")
    ap.add_argument("--no-h2h", action="store_true", help="skip the host-to-host (atz_precompress) measurement")
    ap.add_argument("--cache", default=os.environ.get("ATZ_BENCH_CACHE", "/tmp/atz_bench_cache"))
    ap.add_argument("--workload", choices=("c4", "c5", "c4c3", "c2", "c3"), default="c4",
                    help="c4: the metric's workload (BASELINE configs[3]); c5: configs[4], the same generator with "
                         "windowBits U10-15 and --brute-window (a measurement beside the metric, not its value); "
                         "c2 / c3: configs[1] / configs[2] at their full size (10 000 x 4 KB level-6 streams; the 100 MB "
                         "PDF/PNG/JAR mix), measurements beside the metric (--streams is ignored); "
                         "c4c3: C4 followed by a 100 MB C3 cluster, for the split's rank balance at N > 1")
    ap.add_argument("--files-per-gpu", type=int, default=1,
                    help="independent files in flight per GPU (one context and host thread each; shards mode). "
                         "1 = the metric's workload; 2 measures the multi-file throughput mode (DESIGN s3.6)")
    ap.add_argument("--mode", choices=("file", "shards"), default="file",
                    help="file (default, the metric's config 4): ONE 1 GB file split over the ranks (antiz_amd.shard: "
                         "all-gather of scan results, cost-balanced stream split, RCCL gather of the ATZ1 pieces to "
                         "rank 0; strong scaling); shards: every rank precompresses its own 1 GB file (weak scaling, "
                         "no data-path collective; a secondary line)")
    args = ap.parse_args()
    if args.mode == "file" and args.files_per_gpu > 1:
        ap.error("--files-per-gpu > 1 needs --mode shards (one file per step is split in file mode)")

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # One rank's share of a file split over many GPUs is a small sweep, bound by its rounds' slowest
    # trials: the library runs 6 sweep pipes on their own hardware queues there (atz_accel.cpp
    # sweep_pipes, DESIGN s6), which needs the queues before HIP initialises
    if args.mode == "file" and world > 1 and args.streams / world <= 16000:
        os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")
    import torch
    import torch.distributed as dist
    # ATZ_BENCH_BACKEND=gloo: rehearsal of the N > 1 paths with several ranks on one GPU (RCCL refuses
    # two ranks on one device); the driver's runs use the default, nccl = RCCL, one rank per GPU
    backend = os.environ.get("ATZ_BENCH_BACKEND", "nccl")
    local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    red_dev = "cuda" if backend == "nccl" else "cpu"

    import antiz_amd
    from antiz_amd import datagen

    base = {"c5": 5, "c2": 2, "c3": 3}.get(args.workload, 4)
    seed = base + rank if args.mode == "shards" else base
    fixed = args.workload in ("c2", "c3")   # BASELINE's fixed-size configs: the generator's own defaults
    gen = {"seed": seed} if fixed else {"seed": seed, "n_streams": args.streams}
    nf = max(1, args.files_per_gpu) if args.mode == "shards" else 1
    t0 = time.time()
    if args.mode == "file" and world > 1 and rank != 0:
        dist.barrier()   # rank 0 generates the one shared file first (same seed, same cache path)
    path = datagen.cached(args.workload, args.cache, **({} if fixed and seed == base else gen))
    if args.mode == "file" and world > 1 and rank == 0:
        dist.barrier()
    with open(path, "rb") as f:
        data = f.read()
    log("rank %d: workload %s (%.1f MB) ready in %.1fs" % (rank, os.path.basename(path), len(data) / 1e6, time.time() - t0))
    # input resident in HBM before the timed region (+4 KiB slack the kernels may over-read)
    host = torch.frombuffer(bytearray(data) + bytearray(4096), dtype=torch.uint8)
    dev = host.to("cuda", non_blocking=False)
    torch.cuda.synchronize()

    ctx = antiz_amd.Context(device=local, brute_window=args.workload == "c5")
    group = None
    # --files-per-gpu k > 1: k - 1 more independent files (seeds after every rank's), each with its own
    # context, precompressed by their own host threads beside the first (ctypes drops the GIL)
    extra = []
    for k in range(1, nf):
        p2 = datagen.cached(args.workload, args.cache, **dict(gen, seed=base + world * k + rank))
        with open(p2, "rb") as f:
            d2 = f.read()
        h2 = torch.frombuffer(bytearray(d2) + bytearray(4096), dtype=torch.uint8)
        extra.append((antiz_amd.Context(device=local, brute_window=args.workload == "c5"), d2, h2.to("cuda")))
    torch.cuda.synchronize()

    def step_extra():
        import threading
        res = [None] * len(extra)
        def run(i):
            c2, d2, dv2 = extra[i]
            res[i] = c2.precompress_device(dv2.data_ptr(), d2)
        th = [threading.Thread(target=run, args=(i,)) for i in range(len(extra))]
        for t in th:
            t.start()
        return th, res

    def step():
        if extra:
            th, _ = step_extra()
            dptr, n, st = ctx.precompress_device(dev.data_ptr(), data)
            for t in th:
                t.join()
            return n, st
        return step1()

    last_out = [None]   # device pointer (int) or tensor holding the last step's ATZ1 on rank 0

    def step1():
        if args.mode == "file" and world > 1:
            from antiz_amd import shard
            out, n, st = shard.precompress_sharded(ctx, dev, data, group=group)
            last_out[0] = out
            return n, st
        dptr, n, st = ctx.precompress_device(dev.data_ptr(), data)
        last_out[0] = dptr
        return n, st

    for _ in range(args.warmup):
        step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    stats = []
    for _ in range(args.steps):
        n, st = step()
        stats.append(st)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    shard_bytes = len(data) + sum(len(e[1]) for e in extra) if args.mode == "shards" else len(data) / world
    dt, value, atz_sizes = aggregate(dt, n, shard_bytes, args.steps, world, red_dev)
    balance = rank_balance(stats[-1], world, red_dev) if world > 1 else None
    ms_per_step = dt * 1000.0 / args.steps

    last = stats[-1]
    ktime = last["k_trial_ms"] / 1000.0
    alg = last["k_trial_alg_bytes"]
    achieved = alg / ktime / 1e9 if ktime > 0 else 0.0
    launches = max(1, last["k_trial_launches"])
    traffic, traffic_src, traffic_sha = pmc_traffic()
    achieved_wall = alg / (ms_per_step / 1000.0) / 1e9
    roof = {"bound": "hbm", "achieved": round(achieved, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 6), "traffic": traffic,
            "achieved_wall": round(achieved_wall, 3), "frac_wall": round(achieved_wall / HBM_PEAK_GBS, 6),
            "limiter": "not HBM: the trial kernels are latency-bound serial parses (see issue: waves parked on "
                       "s_waitcnt most of their cycles, the CU's scalar issue part-used; DESIGN.md s3.5); the HBM "
                       "fraction is reported because it is the graded roofline",
            "issue": pmc_issue(),
            "traffic_unit": "bytes per launch (FETCH_SIZE x 2 + WRITE_SIZE)", "traffic_source": traffic_src,
            "traffic_code_sha": traffic_sha,
            "kernel": "k_trial_{stored,fast,slow}", "launches": last["k_trial_launches"],
            "avg_launch_ms": round(last["k_trial_ms"] / launches, 4),
            "alg_bytes_per_launch": int(alg / launches)}

    # parity of the timed run's own output: the ATZ1 SHA-256 of the last step against the real reference's
    # on the same generated file (oracle/_ref/uncomp): tests/golden/full_configs.json for the full-size
    # configs, tests/golden/share_configs.json for the per-rank share files (--streams 12500 / 25000 /
    # 50000) and the C4 + C3 cluster file
    atz_check = None
    if rank == 0 and last_out[0] is not None and (args.mode == "file" or not extra):
        gold = os.path.join(ROOT, "tests", "golden")
        sp = os.path.join(gold, "share_configs.json")
        ref = (json.load(open(sp)) if os.path.exists(sp) else {}).get("%s:%d" % (args.workload, args.streams))
        if ref is None and (args.streams == 100000 or fixed):
            ref = json.load(open(os.path.join(gold, "full_configs.json"))).get(args.workload)
        if ref and len(data) == ref["input_bytes"]:
            h = torch.empty(n, dtype=torch.uint8)
            if isinstance(last_out[0], int):
                torch.cuda.synchronize()
                hip_copy(h.data_ptr(), last_out[0], n)
            else:
                h.copy_(last_out[0][:n].cpu())
            sha = hashlib.sha256(h.numpy().tobytes()).hexdigest()
            atz_check = {"atz_sha256": sha[:16], "identical_to_reference": sha == ref["atz_sha256"],
                         "reference": "oracle/_ref/uncomp on the same file (tests/golden/%s)"
                                      % ("share_configs.json" if "workload" in ref else "full_configs.json")}
            if sha != ref["atz_sha256"]:
                log("PARITY FAILURE: the timed run's ATZ1 differs from the reference's")

    # reconstruct (-r, and precompress's default verify: main.cpp:869-950, 1173-1203) of the last ATZ1,
    # resident in HBM; not part of the metric: its own wall time, and the round trip checked.  Every rank
    # of a shards run, and the one-GPU file run (at N > 1 in file mode the ATZ1 sits on rank 0 only)
    recon = None
    if (args.mode == "shards" or world == 1) and not args.no_recon:
        dptr, alen, _ = ctx.precompress_device(dev.data_ptr(), data)
        hdev = torch.empty(alen + 4096, dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        hip_copy(hdev.data_ptr(), dptr, alen)                # the context reuses its own ATZ1 buffer
        h = torch.empty(alen, dtype=torch.uint8)
        hip_copy(h.data_ptr(), dptr, alen)
        hb = h.numpy().tobytes()
        ctx.reconstruct_device(hdev.data_ptr(), hb)          # warm-up (buffers sized)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(args.steps):
            rp, rl = ctx.reconstruct_device(hdev.data_ptr(), hb)
        torch.cuda.synchronize()
        rdt = (time.perf_counter() - t1) / args.steps
        back = torch.empty(rl, dtype=torch.uint8)
        hip_copy(back.data_ptr(), rp, rl)
        recon = {"value": round(len(data) / 1e6 / rdt, 3), "unit": "MB/s restored (ATZ1 resident in HBM)",
                 "ms_per_step": round(rdt * 1000, 2), "atz_bytes": alen,
                 "atz_sha256": hashlib.sha256(hb).hexdigest()[:16],
                 "identical": rl == len(data) and back.numpy().tobytes() == data}
        del hdev

    # the product path as the CLI runs it: host buffer in, host ATZ1 bytes out (H2D + D2H included)
    h2h = None
    if world == 1 and not args.no_h2h:
        import ctypes
        L = antiz_amd.lib()
        p, n, st = ctypes.POINTER(ctypes.c_uint8)(), ctypes.c_uint64(0), antiz_amd.Stats()
        ts = []
        for _ in range(2):   # the first call sizes the library's pinned staging
            t1 = time.perf_counter()
            rc = L.atz_precompress(ctx.h, data, len(data), ctypes.byref(p), ctypes.byref(n), ctypes.byref(st))
            ts.append(time.perf_counter() - t1)
            if rc != 0:
                raise RuntimeError("atz_precompress failed: %d" % rc)
            L.atz_free(p)
        h2h = {"value": round(len(data) / 1e6 / ts[-1], 3), "unit": "MB/s", "ms": round(ts[-1] * 1000, 2),
               "atz_bytes": n.value, "what": "atz_precompress: host file bytes -> host ATZ1 bytes (H2D of the input, "
                                             "D2H of the ATZ1 included), the uncomp CLI's path; not the metric's value"}
    elif world > 1 and args.mode == "file" and not args.no_h2h:
        # the host path at N > 1 (antiz_amd.shard.precompress_sharded_to_file): every rank copies its own
        # piece from its HBM into the output file at its offset, rank 0 writes the header and the residue
        from antiz_amd import shard
        opath = os.path.join("/dev/shm" if os.path.isdir("/dev/shm") else tempfile.gettempdir(),
                             "atz_bench_%d.atz" % os.getppid())
        ts = []
        for _ in range(2):   # the first call sizes the pinned staging
            dist.barrier()
            t1 = time.perf_counter()
            hn, _ = shard.precompress_sharded_to_file(ctx, dev, data, opath, group=group)
            dist.barrier()
            ts.append(time.perf_counter() - t1)
        if rank == 0:
            with open(opath, "rb") as f:
                hsha = hashlib.sha256(f.read()).hexdigest()
            h2h = {"value": round(len(data) / 1e6 / ts[-1], 3), "unit": "MB/s", "ms": round(ts[-1] * 1000, 2),
                   "atz_bytes": hn, "atz_sha256": hsha[:16],
                   "identical_to_reference": (atz_check or {}).get("atz_sha256") == hsha[:16]
                                             and bool((atz_check or {}).get("identical_to_reference")),
                   "what": "the host path over %d GPUs: device-resident input -> ATZ1 file (each rank writes its own "
                           "piece device -> host at its offset; SURVEY s8e); not the metric's value" % world}
        dist.barrier()
        if rank == 0:
            os.remove(opath)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline(args.cpu_sample_streams, seed, ctx, args.workload)

    if rank == 0:
        wl = {"c4": "C4: %d zlib streams (clevel U1-9, memLevel U1-9, w15)",
              "c2": "C2: 10 000 zlib streams (level 6, 4 KB of text each)",
              "c3": "C3: 100 MB PDF-like / PNG-like Z_FILTERED / JAR-like mix",
              "c5": "C5: %d zlib streams (clevel U1-9, memLevel U1-9, windowBits U10-15), --brute-window",
              "c4c3": "C4 (%d zlib streams) followed by a 100 MB C3 cluster (PDF-like, PNG-like Z_FILTERED, "
                      "JAR-like)"}[args.workload]
        wl = wl if fixed else wl % args.streams
        out = {
            "metric": "input MB/s precompressed (1 GB synthetic, 100k streams) at 1/2/4/8 MI355X",
            "value": round(value, 3),
            "unit": "MB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 2),
            "higher_is_better": True,
            "scaling": "weak" if args.mode == "shards" else "strong",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (antiz_amd.datagen %s, seed %s; text from a seeded 20k-word vocabulary)"
                    % (args.workload.upper(), ("%d+rank" if args.mode == "shards" else "%d") % base),
            "config": ({"workload": wl + ", %.3f GB per GPU, default thresholds" % (len(data) / 1e9),
                        "streams_per_gpu": args.streams * nf, "bytes_per_gpu": len(data) + sum(len(e[1]) for e in extra),
                        "files_per_gpu": nf, "parallelism": "stream-sharded dp%d" % world}
                       if args.mode == "shards" or world == 1 else
                       {"workload": "one file, " + wl + ", %.3f GB, split over %d GPUs, default thresholds"
                                    % (len(data) / 1e9, world),
                        "file_bytes": len(data),
                        "parallelism": "one file: scan by chunk ranges, cost-balanced stream split x%d, RCCL gather"
                                       % world}),
            "roofline": roof,
            "cpu_baseline": cpu,
            "atz_bytes_per_rank": atz_sizes,
            "rank_balance": balance,
            "atz_parity": atz_check,
            "reconstruct": recon,
            "host_to_host": h2h,
            "detail": {k: (round(v, 3) if isinstance(v, float) else v) for k, v in last.items()},
        }
        print(json.dumps(out), flush=True)
    ctx.close()
    for e in extra:
        e[0].close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
