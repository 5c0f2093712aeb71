"""One file precompressed by several GPUs: one process and libatz_accel context per GPU,
launched by torch.distributed (backend "nccl" = RCCL over xGMI; "gloo" for CPU-side tests).

The reference is single-threaded (main.cpp has no threads); this is the build's own multi-GPU layer
over the C ABI's atz_shard_* calls (include/atz_accel.h).  The data path has two exchanges:
  1. all-gather of the scan-candidate results of every rank's chunk range (a few MB): each rank then
     replays the reference's greedy chunk scan (main.cpp:205-246) for the whole file;
  2. gather of the ATZ1 pieces (descriptors + inflated payloads of each rank's recompressed streams,
     main.cpp:805-831) to rank 0, one point-to-point transfer per rank, received in place at its
     offset in rank 0's output buffer; rank 0 then writes the header and the residue (main.cpp:764-801).
Failures follow the reference's abort (main.cpp:450-452, 663-665) on every rank: each library step is
followed by an all-gather of the ranks' status codes before the next data collective, so a rank whose
step raised makes every rank raise the same AtzError instead of leaving its peers blocked in a collective.
The ATZ1 bytes equal the one-GPU result.  precompress_sharded keeps the ATZ1 in rank 0's HBM (the
metric's device-resident output); precompress_sharded_to_file is the host path (the CLI's output file):
each rank copies its own piece device -> host into the file at its offset (payloads go to
the host per GPU, not over xGMI), and rank 0 writes only the header and the residue.
"""
import os

import torch
import torch.distributed as dist

from . import AtzError

HEADER = 28   # "ATZ\x01" + file length + original length + stream count (main.cpp:770-776)


def _device(group=None):
    return torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" else torch.device("cpu")


def allgather_bytes(b, group=None):
    """Every rank's byte string, in rank order (variable sizes: lengths first, then padded payloads)."""
    dev = _device(group)
    world = dist.get_world_size(group)
    n = torch.tensor([len(b)], dtype=torch.int64, device=dev)
    ns = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(ns, n, group=group)
    ns = [int(x.item()) for x in ns]
    m = max(max(ns), 1)
    t = torch.zeros(m, dtype=torch.uint8, device=dev)
    if b:
        t[:len(b)] = torch.frombuffer(bytearray(b), dtype=torch.uint8).to(dev)
    outs = [torch.empty(m, dtype=torch.uint8, device=dev) for _ in range(world)]
    dist.all_gather(outs, t, group=group)
    return [o[:k].cpu().numpy().tobytes() for o, k in zip(outs, ns)]


def allgather_ints(vals, group=None):
    """[[v0, v1, ...] of rank 0, of rank 1, ...] for a fixed-length list of ints per rank."""
    dev = _device(group)
    world = dist.get_world_size(group)
    t = torch.tensor(vals, dtype=torch.int64, device=dev)
    ts = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(ts, t, group=group)
    return [[int(x) for x in u.cpu().tolist()] for u in ts]


def _status(err):
    """A rank's status for the exchange: 0 ok, -ATZ_E_* for a library error, 1000 for anything else."""
    if err is None:
        return 0
    code = getattr(err, "code", 0)
    return -code if code < 0 else 1000


def agree(step, fn, group=None):
    """Run this rank's part of `step` (fn()), then exchange every rank's status (one small all-gather)
    before any data collective: if any rank failed, every rank raises AtzError naming the failed ranks
    and their codes (main.cpp:450-452 aborts the process; here the whole job stops, no rank is left
    waiting in a collective for a peer that is gone)."""
    err, val = None, None
    try:
        val = fn()
    except Exception as e:   # noqa: BLE001 -- any failure must reach the other ranks before we raise
        err = e
    codes = [c[0] for c in allgather_ints([_status(err)], group)]
    bad = [(q, c) for q, c in enumerate(codes) if c]
    if bad:
        msg = "%s failed on rank(s) %s" % (step, ", ".join("%d (%s)" % (q, "atz error %d" % -c if c != 1000 else "exception")
                                                           for q, c in bad))
        code = -bad[0][1] if bad[0][1] != 1000 else 0
        if err is not None:
            raise AtzError("%s: %s" % (msg, err), getattr(err, "code", 0)) from err
        raise AtzError(msg, code)
    return val


def gather_pieces(ctx, piece_lens, out, out_device="cuda", group=None):
    """Rank r's piece lands at out[HEADER + sum(piece_lens[:r])] on rank 0 (out: rank 0's output buffer;
    pieces are staged through the host when the backend is gloo).  Zero-length pieces are not sent."""
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    dev = _device(group)
    offs = [HEADER]
    for L in piece_lens[:-1]:
        offs.append(offs[-1] + L)
    piece = None

    def local():
        nonlocal piece
        if rank == 0 and piece_lens[0]:
            ctx.shard_piece(out.data_ptr() + offs[0])
        elif rank != 0 and piece_lens[rank]:
            piece = torch.empty(piece_lens[rank], dtype=torch.uint8, device=out_device)
            ctx.shard_piece(piece.data_ptr())
    agree("shard_piece", local, group)
    if rank == 0:
        ops, stage = [], []
        for q in range(1, world):
            if not piece_lens[q]:
                continue
            if out.device == dev:
                buf = out[offs[q]:offs[q] + piece_lens[q]]
            else:   # gloo: receive on the host, then copy into place
                buf = torch.empty(piece_lens[q], dtype=torch.uint8, device=dev)
                stage.append((q, buf))
            ops.append(dist.P2POp(dist.irecv, buf, q, group=group))
        for w in (dist.batch_isend_irecv(ops) if ops else []):
            w.wait()
        for q, buf in stage:
            out[offs[q]:offs[q] + piece_lens[q]].copy_(buf)
    elif piece_lens[rank]:
        if piece.device != dev:
            piece = piece.to(dev)
        for w in dist.batch_isend_irecv([dist.P2POp(dist.isend, piece, 0, group=group)]):
            w.wait()


def _scan_and_sweep(ctx, d_file, data, group):
    """Exchange 1 and the sweep of this rank's share: (piece_lens, all recomp flags, recompressed total, stats)."""
    dptr = d_file.data_ptr()
    blob = agree("shard_scan", lambda: ctx.shard_scan(dptr, data, dist.get_rank(group), dist.get_world_size(group)), group)
    blobs = allgather_bytes(blob, group)
    piece_len, flags, n_recomp, st = agree("shard_sweep", lambda: ctx.shard_sweep(dptr, data, blobs), group)
    meta = allgather_ints([piece_len, n_recomp, len(flags)], group)
    return [m[0] for m in meta], b"".join(allgather_bytes(flags, group)), sum(m[1] for m in meta), st


def precompress_sharded_to_file(ctx, d_file, data, path, group=None, device="cuda"):
    """Precompress `data` over every rank of `group` into the file `path` (one node: the ranks share the
    filesystem).  Rank r copies its piece (descriptors + payloads of its recompressed streams) from its
    own HBM into the file at 28 + the lengths of the pieces before it; rank 0 assembles the header and
    the residue in its HBM and writes just those two ranges.  Returns (atz_len, stats); atz_len on every
    rank once the file is complete.  (device: where the pieces are staged, "cpu" for the host-logic tests.)"""
    rank = dist.get_rank(group)
    piece_lens, flags, n_recomp, st = _scan_and_sweep(ctx, d_file, data, group)
    pieces = sum(piece_lens)

    def create():
        if rank == 0:
            with open(path, "wb"):
                pass
    agree("creating " + path, create, group)   # (also the barrier: the file exists before any rank opens it)

    def write_piece():
        if not piece_lens[rank]:
            return
        off = HEADER + sum(piece_lens[:rank])
        piece = torch.empty(piece_lens[rank], dtype=torch.uint8, device=device)
        ctx.shard_piece(piece.data_ptr())
        host = torch.empty(piece_lens[rank], dtype=torch.uint8, pin_memory=device != "cpu")
        host.copy_(piece)
        del piece
        fd = os.open(path, os.O_WRONLY)
        try:
            mv, done = memoryview(host.numpy()), 0
            while done < len(mv):
                done += os.pwrite(fd, mv[done:], off + done)
        finally:
            os.close(fd)
    agree("writing the pieces", write_piece, group)

    def assemble():
        if rank != 0:
            return 0
        # atz_shard_assemble writes the header at 0 and the residue at 28 + pieces of one buffer, so the
        # buffer spans the pieces too (never written here): rank 0's device peak holds 28 + pieces +
        # the residue (at most the file) + 4 KiB, e.g. ~2.8 GB for C4 + C3, freed before returning
        cap = HEADER + pieces + len(data) + 4096
        out = torch.empty(cap, dtype=torch.uint8, device=device)
        n = ctx.shard_assemble(d_file.data_ptr(), len(data), flags, n_recomp, pieces, out.data_ptr(), cap)
        head = out[:HEADER].cpu().numpy().tobytes()
        tail = out[HEADER + pieces:n].cpu().numpy().tobytes()
        del out
        fd = os.open(path, os.O_WRONLY)
        try:
            os.pwrite(fd, head, 0)
            done = 0
            while done < len(tail):
                done += os.pwrite(fd, memoryview(tail)[done:], HEADER + pieces + done)
            os.ftruncate(fd, n)
        finally:
            os.close(fd)
        return n
    n = agree("shard_assemble", assemble, group)
    n = allgather_ints([n], group)[0][0]
    return n, st


def precompress_sharded(ctx, d_file, data, group=None, out_device="cuda"):
    """Precompress `data` (host bytes; d_file: the same bytes resident on this rank's GPU, a uint8 tensor
    with >= 4096 bytes of slack) over every rank of `group`.  Returns (atz tensor, atz_len, stats) on
    rank 0 (ATZ1 bytes = atz[:atz_len], on out_device) and (None, 0, stats) elsewhere."""
    rank = dist.get_rank(group)
    dptr = d_file.data_ptr()
    piece_lens, flags, n_recomp, st = _scan_and_sweep(ctx, d_file, data, group)
    cap = HEADER + sum(piece_lens) + len(data) + 4096   # the residue is at most the whole file
    out = agree("output buffer", lambda: torch.empty(cap, dtype=torch.uint8, device=out_device) if rank == 0 else None,
                group)
    gather_pieces(ctx, piece_lens, out, out_device, group)
    if rank != 0:
        return None, 0, st
    n = ctx.shard_assemble(dptr, len(data), flags, n_recomp, sum(piece_lens), out.data_ptr(), out.numel())   # no collective follows
    return out, n, st
