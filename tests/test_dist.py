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


# ---- antiz_amd.shard: one file over several ranks (host logic; the GPU test runs the real library) ----
class FakeShardCtx:
    """Stands in for a libatz_accel context: every shard_* call checks what the driver hands it and
    writes recognisable bytes, so the exchanges and the placement of the pieces can be checked on CPU."""

    def __init__(self, rank, world):
        self.rank, self.world = rank, world
        self.calls = []

    def piece_len(self, r):
        return [5, 0, 7, 3][r % 4]

    def flags(self, r):
        return bytes([1, 0, 1][: 1 + r % 3])

    def shard_scan(self, dptr, data, rank, world):
        assert (rank, world) == (self.rank, self.world)
        self.calls.append("scan")
        return b"blob-%d-" % rank + bytes(range(rank * 3))

    def shard_sweep(self, dptr, data, blobs):
        assert blobs == [b"blob-%d-" % q + bytes(range(q * 3)) for q in range(self.world)]
        self.calls.append("sweep")
        f = self.flags(self.rank)
        return self.piece_len(self.rank), f, sum(f), {"rank": self.rank}

    def shard_piece(self, dst):
        import ctypes
        n = self.piece_len(self.rank)
        ctypes.memmove(dst, bytes([0x10 + self.rank]) * n, n)

    def shard_assemble(self, dptr, flen, flags, n_recomp, pieces_len, d_atz, cap):
        import ctypes
        assert flags == b"".join(self.flags(q) for q in range(self.world))
        assert n_recomp == sum(sum(self.flags(q)) for q in range(self.world))
        assert pieces_len == sum(self.piece_len(q) for q in range(self.world))
        assert cap >= 28 + pieces_len + flen
        ctypes.memmove(d_atz, b"H" * 28, 28)
        ctypes.memmove(d_atz + 28 + pieces_len, b"R" * flen, flen)
        return 28 + pieces_len + flen


def _shard_worker(rank, world, port, q, path=None):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from antiz_amd import shard
    data = b"x" * 11
    fake = FakeShardCtx(rank, world)
    if path is None:
        out, n, st = shard.precompress_sharded(fake, torch.zeros(16, dtype=torch.uint8), data, out_device="cpu")
        q.put((rank, None if out is None else out[:n].numpy().tobytes(), n, st, fake.calls))
    else:   # the host path: every rank writes its piece into the file
        n, st = shard.precompress_sharded_to_file(fake, torch.zeros(16, dtype=torch.uint8), data, path, device="cpu")
        q.put((rank, open(path, "rb").read() if rank == 0 else None, n, st, fake.calls))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_precompress_sharded_exchanges(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_shard_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {r: (atz, n, st, calls) for r, atz, n, st, calls in (q.get(timeout=120) for _ in range(world))}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    fake = FakeShardCtx(0, world)
    want = b"H" * 28 + b"".join(bytes([0x10 + r]) * fake.piece_len(r) for r in range(world)) + b"R" * 11
    assert res[0][0] == want and res[0][1] == len(want)
    for r in range(world):
        assert res[r][2] == {"rank": r} and res[r][3] == ["scan", "sweep"]
        if r:
            assert res[r][0] is None and res[r][1] == 0


@pytest.mark.parametrize("world", [2, 3, 4])
def test_precompress_sharded_to_file(world, tmp_path):
    """The host path: each rank writes its own piece into the output file at its prefix
    offset; rank 0 writes the header and the residue around them.  The file equals rank 0's assembled ATZ1."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    path = str(tmp_path / "out.atz")
    procs = [ctx.Process(target=_shard_worker, args=(r, world, port, q, path)) for r in range(world)]
    for p in procs:
        p.start()
    res = {r: (atz, n, st, calls) for r, atz, n, st, calls in (q.get(timeout=120) for _ in range(world))}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    fake = FakeShardCtx(0, world)
    want = b"H" * 28 + b"".join(bytes([0x10 + r]) * fake.piece_len(r) for r in range(world)) + b"R" * 11
    assert res[0][0] == want
    for r in range(world):
        assert res[r][1] == len(want) and res[r][2] == {"rank": r} and res[r][3] == ["scan", "sweep"]


# ---- a rank that fails stops every rank (main.cpp:450-452, 663-665 abort the process) ----
class FailingShardCtx(FakeShardCtx):
    """FakeShardCtx whose `fail_at` call raises AtzError on `fail_rank` (as a library error would; rank 1
    has an empty piece, so its shard_piece is never called)."""

    def __init__(self, rank, world, fail_at, fail_rank=1):
        super().__init__(rank, world)
        self.fail_at, self.fail_rank = fail_at, fail_rank

    def _maybe_fail(self, what):
        if what == self.fail_at and self.rank == self.fail_rank:
            from antiz_amd import AtzError
            raise AtzError("atz error -7: injected %s failure" % what, -7)

    def shard_scan(self, *a):
        self._maybe_fail("scan")
        return super().shard_scan(*a)

    def shard_sweep(self, *a):
        self._maybe_fail("sweep")
        return super().shard_sweep(*a)

    def shard_piece(self, dst):
        self._maybe_fail("piece")
        return super().shard_piece(dst)

    def shard_assemble(self, *a):
        self._maybe_fail("assemble")
        return super().shard_assemble(*a)


def _failing_worker(rank, world, port, q, fail_at, fail_rank, path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from antiz_amd import AtzError, shard
    fake = FailingShardCtx(rank, world, fail_at, fail_rank)
    try:
        if path is None:
            shard.precompress_sharded(fake, torch.zeros(16, dtype=torch.uint8), b"x" * 11, out_device="cpu")
        else:
            shard.precompress_sharded_to_file(fake, torch.zeros(16, dtype=torch.uint8), b"x" * 11, path, device="cpu")
    except AtzError as e:
        q.put((rank, str(e), e.code))
        q.close()
        q.join_thread()
        os._exit(3)   # non-zero, like the reference's abort; no collective is left pending
    q.put((rank, None, 0))
    q.close()
    q.join_thread()
    os._exit(0)


@pytest.mark.parametrize("fail_at,fail_rank,host", [("scan", 1, False), ("sweep", 1, False), ("piece", 2, False),
                                                    ("piece", 0, False), ("sweep", 2, True), ("piece", 2, True),
                                                    ("assemble", 0, True)])
def test_rank_failure_stops_every_rank(fail_at, fail_rank, host, tmp_path):
    """A library error on one rank makes every rank raise the same AtzError within seconds (the status
    all-gather before each data collective), instead of the others blocking in the next collective."""
    import time
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    path = str(tmp_path / "out.atz") if host else None
    procs = [ctx.Process(target=_failing_worker, args=(r, world, port, q, fail_at, fail_rank, path)) for r in range(world)]
    t0 = time.time()
    for p in procs:
        p.start()
    res = {r: (msg, code) for r, msg, code in (q.get(timeout=60) for _ in range(world))}
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 3, "every rank exits non-zero"
    assert time.time() - t0 < 60
    for r in range(world):
        msg, code = res[r]
        assert msg is not None and "failed on rank(s) %d" % fail_rank in msg, msg
        assert code == -7
