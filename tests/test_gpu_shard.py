"""One file precompressed by several ranks (antiz_amd.shard over the atz_shard_* C ABI).

The GPU box has one MI355X, so the ranks share it (gloo carries the exchanges; on a node, bench.py
runs one rank per GPU over RCCL).  Rank 0's ATZ1 bytes must equal the one-GPU precompress and the
oracle's (the reference's algorithm restated in oracle/), for every world size, including chunk
ranges whose boundary a pending stream crosses.
"""
import hashlib
import os
import socket
import sys

import pytest

import _libs

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, path, chunksize, q):
    try:
        sys.path.insert(0, ROOT)
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import antiz_amd
        from antiz_amd import shard
        data = open(path, "rb").read()
        d = torch.frombuffer(bytearray(data) + bytearray(4096), dtype=torch.uint8).to("cuda")
        with antiz_amd.Context(chunksize=chunksize, device=0) as ctx:
            out, n, st = shard.precompress_sharded(ctx, d, data, out_device="cuda")
            atz = out[:n].cpu().numpy().tobytes() if out is not None else None
        q.put((rank, atz, st["n_streams"], st["n_recomp"], st["trial_cyc_total"], None))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:   # report instead of hanging the parent
        q.put((rank, None, 0, 0, 0, repr(e)))


def _run(world, path, chunksize):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, path, chunksize, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, atz, ns, nr, cyc, err = q.get(timeout=240)
        assert err is None, "rank %d: %s" % (r, err)
        res[r] = (atz, ns, nr, cyc)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


@pytest.fixture(scope="module")
def sample(tmp_path_factory):
    from antiz_amd import datagen
    data = datagen.gen_c4(seed=41, n_streams=1200)   # ~12 MB
    path = str(tmp_path_factory.mktemp("shard") / "c4s.bin")
    with open(path, "wb") as f:
        f.write(data)
    return path, data


@pytest.mark.parametrize("world,chunksize", [(1, 524288), (2, 524288), (3, 65536), (4, 65536)])
def test_sharded_equals_single_gpu_and_oracle(sample, world, chunksize):
    import antiz_amd
    path, data = sample
    with antiz_amd.Context(chunksize=chunksize, device=0) as c:
        one, st = c.precompress(data)
    rc, ref, _ = _libs.ora_precompress(data, chunksize=chunksize)
    assert rc == 0 and one == ref
    res = _run(world, path, chunksize)
    assert hashlib.sha256(res[0][0]).hexdigest() == hashlib.sha256(one).hexdigest()
    assert sum(v[1] for v in res.values()) == st["n_streams"]     # the ranks' records partition the file's
    assert sum(v[2] for v in res.values()) == st["n_recomp"]


@pytest.fixture(scope="module")
def clustered(tmp_path_factory):
    """C4 streams followed by a cluster of C3's PNG-like Z_FILTERED streams (they match no trial, so
    each runs its class's whole list): an equal split of the chunks would leave the ranks that hold the
    cluster with most of the sweep; the cost-balanced split gives them fewer records."""
    from antiz_amd import datagen
    data = datagen.gen_c4(seed=43, n_streams=500) + datagen.gen_c3(seed=44, total=3_000_000)
    path = str(tmp_path_factory.mktemp("shardc") / "mixed.bin")
    with open(path, "wb") as f:
        f.write(data)
    rc, ref, _ = _libs.ora_precompress(data)
    assert rc == 0
    return path, data, ref


@pytest.mark.parametrize("world", [2, 3, 4])
def test_sharded_cost_split_on_clustered_input(clustered, world):
    """The ranks' record ranges partition the file's records, and the split follows cost, not counts: the
    last rank, which holds the cluster of PNG-like streams (each runs its class's whole trial list), gets
    fewer records than an equal split would give it, and the ranks' trial cycles stay within 2x of their
    mean (the measured balance is reported by bench.py's rank_balance)."""
    import antiz_amd
    path, data, ref = clustered
    with antiz_amd.Context(device=0) as c:
        recs = c.scan(data)
    res = _run(world, path, 524288)
    assert hashlib.sha256(res[0][0]).hexdigest() == hashlib.sha256(ref).hexdigest()
    counts = [res[r][1] for r in range(world)]
    assert sum(counts) == len(recs) and all(n > 0 for n in counts)
    assert counts[-1] < len(recs) // world
    cyc = [res[r][3] for r in range(world)]
    assert max(cyc) <= 2.0 * sum(cyc) / world, cyc
