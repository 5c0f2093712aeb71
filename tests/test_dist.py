"""World-size-2 gloo rehearsal of bench.py's multi-GPU reduction (CPU only).

bench.py --gpus N runs one process per GPU, each precompressing its own shard; the only
collectives are the timing max-reduction and the all_gather of per-rank ATZ sizes (bench.aggregate).
"""
import os
import socket
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    dt = [2.0, 3.0][rank]                    # rank 1 is the slowest
    out = bench.aggregate(dt, atz_len=1000 + rank, shard_bytes=10_000_000, steps=2, world=world, device="cpu")
    q.put((rank, out))
    dist.barrier()
    dist.destroy_process_group()


def test_aggregate_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(2):
        dt, value, sizes = res[r]
        assert dt == 3.0                                   # max over ranks
        assert value == pytest.approx(2 * 10_000_000 / 1e6 / (3.0 / 2))   # whole-job bytes / slowest
        assert sizes == [1000, 1001]                        # per-rank ATZ sizes, rank order


def test_aggregate_world1():
    import bench
    dt, value, sizes = bench.aggregate(1.5, 77, 3_000_000, 3, 1, "cpu")
    assert dt == 1.5 and sizes == [77]
    assert value == pytest.approx(3.0 / 0.5)
