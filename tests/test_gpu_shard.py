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


def _worker(rank, world, port, path, chunksize, q, out_path=None, backend="gloo"):
    try:
        sys.path.insert(0, ROOT)
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(0)
        dist.init_process_group(backend, rank=rank, world_size=world)
        import antiz_amd
        from antiz_amd import shard
        data = open(path, "rb").read()
        d = torch.frombuffer(bytearray(data) + bytearray(4096), dtype=torch.uint8).to("cuda")
        with antiz_amd.Context(chunksize=chunksize, device=0) as ctx:
            if out_path is None:
                out, n, st = shard.precompress_sharded(ctx, d, data, out_device="cuda")
                atz = out[:n].cpu().numpy().tobytes() if out is not None else None
            else:   # the host path: each rank writes its piece into the file
                n, st = shard.precompress_sharded_to_file(ctx, d, data, out_path)
                atz = open(out_path, "rb").read() if rank == 0 else None
        q.put((rank, atz, st["n_streams"], st["n_recomp"], st["k_trial_alg_bytes"], None))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:   # report instead of hanging the parent
        q.put((rank, None, 0, 0, 0, repr(e)))


def _run(world, path, chunksize, out_path=None, backend="gloo"):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, path, chunksize, q, out_path, backend)) for r in range(world)]
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


def test_sharded_one_rank_over_rccl(sample, tmp_path):
    """The "nccl" (RCCL) branches of shard.py -- status and blob all-gathers on device tensors -- at one
    rank: RCCL refuses two ranks on one GPU, so this is as far as the one-GPU box goes (bench.py runs
    them at N > 1 on a node)."""
    path, data = sample
    rc, ref, _ = _libs.ora_precompress(data, chunksize=524288)
    assert rc == 0
    res = _run(1, path, 524288, backend="nccl")
    assert res[0][0] == ref
    res = _run(1, path, 524288, out_path=str(tmp_path / "out.atz"), backend="nccl")
    assert res[0][0] == ref


def test_sharded_with_memory_caps_bound(sample, monkeypatch):
    """Two ranks with every device-memory cap divided down (ATZ_CAP_DIV, inherited by the spawned ranks):
    the shard scan's arena overflows into re-inflates and the shard sweeps defer streams; rank 0's ATZ1
    bytes still equal the oracle's."""
    path, data = sample
    rc, ref, _ = _libs.ora_precompress(data, chunksize=65536)
    assert rc == 0
    monkeypatch.setenv("ATZ_CAP_DIV", "4096")
    res = _run(2, path, 65536)
    assert res[0][0] == ref


@pytest.mark.parametrize("k", range(4))
def test_sharded_fuzz_files_equal_oracle(k, tmp_path):
    """Fuzz files (tests/golden_cases.py fuzz_file, 40 of them joined: ~60 KB of streams, noise,
    truncated streams and bare headers) over three ranks with chunks of 64 B - 4 KiB, so the ranks'
    chunk ranges split pending streams and refills: rank 0's ATZ1 equals the oracle's."""
    import random
    import golden_cases as G
    r = random.Random(900 + k)
    data = b"".join(G.fuzz_file(r) for _ in range(40))
    cs = [64, 257, 1000, 4096][k]
    rc, ref, _ = _libs.ora_precompress(data, chunksize=cs)
    assert rc == 0
    path = str(tmp_path / "fz.bin")
    with open(path, "wb") as f:
        f.write(data)
    res = _run(3, path, cs)
    assert res[0][0] == ref


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


def _first_block_noshort(stream):
    """The split's cost hint restated (k_inflate.hip, INF_HINT_NOSHORT): the zlib stream's first block is
    dynamic (RFC 1951 3.2.7) and its literal/length code lengths give codes to some length symbol but to
    none of 257-259 (lengths 3-5), which zlib's Z_FILTERED never emits (Z/deflate.c:1774-1782)."""
    pos = [16]

    def bits(n):
        v = 0
        for i in range(n):
            p = pos[0] + i
            v |= ((stream[p >> 3] >> (p & 7)) & 1) << i
        pos[0] += n
        return v

    bits(1)
    if bits(2) != 2:
        return False
    nlen, ndist, ncode = bits(5) + 257, bits(5) + 1, bits(4) + 4
    order = [16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15]
    cl = [0] * 19
    for i in range(ncode):
        cl[order[i]] = bits(3)
    # canonical code -> symbol for the code-length alphabet
    table, code = {}, 0
    for length in range(1, 8):
        for sym in range(19):
            if cl[sym] == length:
                table[(length, code)] = sym
                code += 1
        code <<= 1
    lens = []
    while len(lens) < nlen + ndist:
        c, n = 0, 0
        while (n, c) not in table:
            c, n = (c << 1) | bits(1), n + 1
            assert n <= 7
        sym = table[(n, c)]
        if sym < 16:
            lens.append(sym)
        elif sym == 16:
            lens += [lens[-1]] * (3 + bits(2))
        elif sym == 17:
            lens += [0] * (3 + bits(3))
        else:
            lens += [0] * (11 + bits(7))
    m = [lens[257 + i] != 0 for i in range(nlen - 257)]
    return any(m) and not any(m[:3])


def test_split_hint_matches_first_block_headers(clustered):
    """Candidate flag bit1 (k_inflate's first-block test) equals the restatement above on every record,
    and it marks the PNG-like Z_FILTERED cluster: most of the C3 part's zlib streams run their whole
    trial list, while the C4 part's streams (default strategy) are almost never marked."""
    import antiz_amd
    path, data, _ = clustered
    with antiz_amd.Context(device=0) as c:
        recs = c.scan(data)
    got = [(r[4] >> 1) & 1 for r in recs]
    want = [int(_first_block_noshort(data[r[0]:r[0] + r[2]])) for r in recs]
    assert got == want
    c4_len = len(__import__("antiz_amd.datagen", fromlist=["x"]).gen_c4(seed=43, n_streams=500))
    c4 = [g for r, g in zip(recs, got) if r[0] < c4_len]
    c3 = [g for r, g in zip(recs, got) if r[0] >= c4_len]
    assert sum(c4) <= len(c4) // 50 and sum(c3) >= len(c3) // 5, (sum(c4), len(c4), sum(c3), len(c3))


@pytest.mark.parametrize("world", [2, 3, 4])
def test_sharded_cost_split_on_clustered_input(clustered, world):
    """The ranks' record ranges partition the file's records, and the split follows cost, not counts: the
    last rank, which holds the cluster of PNG-like streams (each runs its class's whole trial list), gets
    fewer records than an equal split would give it, and the ranks' trial work (algorithmic bytes: input
    parsed + output compared; shader cycles would also count the waits of ranks sharing the one GPU)
    stays within 2x of their mean (bench.py's rank_balance reports the measured balance)."""
    import antiz_amd
    path, data, ref = clustered
    with antiz_amd.Context(device=0) as c:
        recs = c.scan(data)
    res = _run(world, path, 524288)
    assert hashlib.sha256(res[0][0]).hexdigest() == hashlib.sha256(ref).hexdigest()
    counts = [res[r][1] for r in range(world)]
    assert sum(counts) == len(recs) and all(n > 0 for n in counts)
    assert counts[-1] < len(recs) // world
    work = [res[r][3] for r in range(world)]
    assert max(work) <= 2.0 * sum(work) / world, work


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_host_output_equals_oracle(sample, world, tmp_path):
    """The host path: every rank copies its own piece from its HBM into the output file at
    its offset, rank 0 writes the header and the residue; the file equals the oracle's ATZ1."""
    path, data = sample
    rc, ref, _ = _libs.ora_precompress(data, chunksize=65536)
    assert rc == 0
    res = _run(world, path, 65536, out_path=str(tmp_path / "out.atz"))
    assert hashlib.sha256(res[0][0]).hexdigest() == hashlib.sha256(ref).hexdigest()
