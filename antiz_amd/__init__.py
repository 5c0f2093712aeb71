"""antiz_amd -- MI355X-native zlib-stream precompressor (drop-in for AntiZ's precompress/reconstruct path).

The product is the C ABI library antiz_amd/_build/libatz_accel.so (HIP kernels for gfx950, see
include/atz_accel.h) and the `uncomp` CLI built beside it.  This module is the thin Python host
mirror used by tests and bench.py: it loads that library and raises if it is missing -- there is
no CPU fallback.
"""
import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("ATZ_LIB") or os.path.join(HERE, "_build", "libatz_accel.so")   # ATZ_LIB: diagnostic builds
CLI_PATH = os.path.join(HERE, "_build", "uncomp")

u64 = C.c_uint64
u8p = C.POINTER(C.c_uint8)


class Opts(C.Structure):
    _fields_ = [("recomp_tresh", u64), ("sizediff_tresh", u64), ("shortcut_len", u64), ("mismatch_tol", u64),
                ("chunksize", u64), ("brute_window", C.c_int32), ("device", C.c_int32)]


class Cand(C.Structure):
    _fields_ = [("offset", u64), ("comp_len", u64), ("infl_len", u64), ("type", C.c_int32), ("flags", C.c_uint32)]


class Result(C.Structure):
    _fields_ = [("clevel", C.c_uint8), ("window", C.c_uint8), ("memlevel", C.c_uint8), ("recomp", C.c_uint8),
                ("n_trials", C.c_uint32), ("ident", u64), ("first_diff", C.c_int64), ("n_diff", u64),
                ("diff_index", u64)]


class Stats(C.Structure):
    _fields_ = [(k, u64) for k in ("file_bytes", "n_streams", "n_recomp", "n_trials", "n_trials_shortcut",
                                   "n_rounds", "atz_bytes", "n_candidates", "n_continuations", "n_hazard")] + \
               [(k, C.c_double) for k in ("scan_ms", "sweep_ms", "write_ms", "total_ms", "k_trial_ms",
                                          "k_inflate_ms", "k_chains_ms", "k_other_ms")] + \
               [(k, u64) for k in ("k_trial_launches", "k_inflate_launches", "k_chains_launches",
                                   "k_trial_alg_bytes", "k_inflate_alg_bytes", "k_chains_alg_bytes",
                                   "trial_parsed_bytes")] + \
               [("k_match_ms", C.c_double)] + \
               [(k, u64) for k in ("k_match_launches", "k_match_positions", "n_trials_rerun", "n_fast_fallbacks",
                                   "trial_cyc_total", "trial_cyc_tree", "trial_cyc_emit", "trial_blocks",
                                   "trial_cyc_heap", "trial_cyc_fallback", "trial_symbols",
                                   "n_trials_speculative", "n_reinflated", "n_inflate_retries", "n_trials_replayed", "n_replay_checked",
                                   "n_trials_duplicate", "n_fast_restarts", "dev_bytes_peak", "dev_bytes_held",
                                   "n_trials_skipped")]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


EXPORTS = ["atz_open", "atz_close", "atz_strerror", "atz_free", "atz_default_opts", "atz_scan", "atz_sweep",
           "atz_precompress", "atz_precompress_device", "atz_reconstruct", "atz_deflate", "atz_deflate_batch",
           "atz_inflate_batch", "atz_deflate_bound", "atz_shard_scan", "atz_shard_sweep", "atz_shard_piece",
           "atz_shard_assemble", "atz_reconstruct_device"]

_lib = None


class AtzError(RuntimeError):
    """A libatz_accel call failed; `code` is its negative ATZ_E_* value (include/atz_accel.h), 0 if none."""

    def __init__(self, msg, code=0):
        super().__init__(msg)
        self.code = code


def lib():
    """Load libatz_accel.so; raise if it was not built (never fall back to the CPU)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise AtzError("libatz_accel.so not built: run `python -m antiz_amd.build` (no CPU fallback)")
        L = C.CDLL(LIB_PATH)
        L.atz_open.argtypes = [C.POINTER(C.c_void_p), C.POINTER(Opts)]
        L.atz_close.argtypes = [C.c_void_p]
        L.atz_strerror.restype = C.c_char_p
        L.atz_strerror.argtypes = [C.c_int]
        L.atz_free.argtypes = [C.c_void_p]
        L.atz_default_opts.argtypes = [C.POINTER(Opts)]
        L.atz_scan.argtypes = [C.c_void_p, C.c_char_p, u64, C.POINTER(C.POINTER(Cand)), C.POINTER(u64)]
        L.atz_sweep.argtypes = [C.c_void_p, C.POINTER(Cand), u64, C.POINTER(Result), C.POINTER(C.POINTER(u64)),
                                C.POINTER(u8p), C.POINTER(u64)]
        L.atz_precompress.argtypes = [C.c_void_p, C.c_char_p, u64, C.POINTER(u8p), C.POINTER(u64), C.POINTER(Stats)]
        L.atz_precompress_device.argtypes = [C.c_void_p, C.c_void_p, C.c_char_p, u64, C.POINTER(C.c_void_p),
                                             C.POINTER(u64), C.POINTER(Stats)]
        L.atz_reconstruct.argtypes = [C.c_void_p, C.c_char_p, u64, C.POINTER(u8p), C.POINTER(u64)]
        L.atz_deflate.argtypes = [C.c_void_p, C.c_char_p, u64, C.c_int, C.c_int, C.c_int, C.c_char_p, u64,
                                  C.POINTER(u64)]
        L.atz_inflate_batch.argtypes = [C.c_void_p, C.c_char_p, u64, C.POINTER(u64), C.POINTER(u64), u64,
                                        C.POINTER(C.c_uint32), C.POINTER(u64), C.POINTER(u64)]
        L.atz_deflate_batch.argtypes = [C.c_void_p, C.c_char_p, u64, C.POINTER(u64), C.POINTER(u64),
                                        C.POINTER(C.c_uint32), u64, C.c_char_p, C.POINTER(u64), C.POINTER(u64),
                                        C.POINTER(u64)]
        L.atz_deflate_bound.restype = u64
        L.atz_deflate_bound.argtypes = [u64, C.c_int, C.c_int]
        L.atz_shard_scan.argtypes = [C.c_void_p, C.c_void_p, C.c_char_p, u64, C.c_int, C.c_int, C.POINTER(u8p),
                                     C.POINTER(u64)]
        L.atz_shard_sweep.argtypes = [C.c_void_p, C.c_void_p, C.c_char_p, u64, C.POINTER(C.c_char_p),
                                      C.POINTER(u64), C.c_int, C.POINTER(u64), C.POINTER(u8p), C.POINTER(u64),
                                      C.POINTER(u64), C.POINTER(Stats)]
        L.atz_shard_piece.argtypes = [C.c_void_p, C.c_void_p]
        L.atz_reconstruct_device.argtypes = [C.c_void_p, C.c_void_p, C.c_char_p, u64, C.POINTER(C.c_void_p),
                                             C.POINTER(u64)]
        L.atz_shard_assemble.argtypes = [C.c_void_p, C.c_void_p, u64, C.c_char_p, u64, u64, u64, C.c_void_p, u64,
                                         C.POINTER(u64)]
        _lib = L
    return _lib


def _check(rc):
    if rc != 0:
        raise AtzError("atz error %d: %s" % (rc, lib().atz_strerror(rc).decode()), rc)


class Context:
    """One libatz_accel context (one GPU).  Mirrors the reference's programOptions (ATZData.h:7-35)."""

    def __init__(self, recomp_tresh=128, sizediff_tresh=128, shortcut_len=512, mismatch_tol=2,
                 chunksize=524288, brute_window=False, device=-1):
        L = lib()
        self.o = Opts(recomp_tresh, sizediff_tresh, shortcut_len, mismatch_tol, chunksize, int(brute_window), device)
        self.h = C.c_void_p()
        _check(L.atz_open(C.byref(self.h), C.byref(self.o)))

    def close(self):
        if self.h:
            lib().atz_close(self.h)
            self.h = C.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def precompress(self, data):
        L = lib()
        p = u8p()
        n = u64(0)
        st = Stats()
        _check(L.atz_precompress(self.h, data, len(data), C.byref(p), C.byref(n), C.byref(st)))
        out = C.string_at(p, n.value)
        L.atz_free(p)
        return out, st.as_dict()

    def precompress_device(self, d_ptr, host_data):
        """Input already resident in HBM (d_ptr: device pointer, e.g. torch tensor.data_ptr())."""
        L = lib()
        dp = C.c_void_p()
        n = u64(0)
        st = Stats()
        _check(L.atz_precompress_device(self.h, C.c_void_p(d_ptr), host_data, len(host_data), C.byref(dp),
                                        C.byref(n), C.byref(st)))
        return dp.value, n.value, st.as_dict()

    # ---- one file over several GPUs (antiz_amd.shard drives these with torch.distributed) ----
    def shard_scan(self, d_ptr, host_data, rank, world):
        L = lib()
        p = u8p()
        n = u64(0)
        _check(L.atz_shard_scan(self.h, C.c_void_p(d_ptr), host_data, len(host_data), rank, world, C.byref(p),
                                C.byref(n)))
        out = C.string_at(p, n.value)
        L.atz_free(p)
        return out

    def shard_sweep(self, d_ptr, host_data, blobs):
        """-> (piece_len, recomp flags (bytes, one per record of this rank), n_recomp, stats)"""
        L = lib()
        k = len(blobs)
        bp = (C.c_char_p * k)(*blobs)
        bl = (u64 * k)(*[len(b) for b in blobs])
        pl, nf, nr = u64(0), u64(0), u64(0)
        fp = u8p()
        st = Stats()
        _check(L.atz_shard_sweep(self.h, C.c_void_p(d_ptr), host_data, len(host_data), bp, bl, k, C.byref(pl),
                                 C.byref(fp), C.byref(nf), C.byref(nr), C.byref(st)))
        flags = C.string_at(fp, nf.value)
        L.atz_free(fp)
        return pl.value, flags, nr.value, st.as_dict()

    def shard_piece(self, d_dst):
        _check(lib().atz_shard_piece(self.h, C.c_void_p(d_dst)))

    def shard_assemble(self, d_ptr, file_len, flags, n_recomp, pieces_len, d_atz, cap):
        n = u64(0)
        _check(lib().atz_shard_assemble(self.h, C.c_void_p(d_ptr), file_len, flags, len(flags), n_recomp,
                                        pieces_len, C.c_void_p(d_atz), cap, C.byref(n)))
        return n.value

    def reconstruct(self, atz):
        L = lib()
        p = u8p()
        n = u64(0)
        _check(L.atz_reconstruct(self.h, atz, len(atz), C.byref(p), C.byref(n)))
        out = C.string_at(p, n.value)
        L.atz_free(p)
        return out

    def reconstruct_device(self, d_atz, host_atz):
        """ATZ1 bytes already in HBM (d_atz: device pointer); returns (device pointer, length) of the original."""
        dp = C.c_void_p()
        n = u64(0)
        _check(lib().atz_reconstruct_device(self.h, C.c_void_p(d_atz), host_atz, len(host_atz), C.byref(dp),
                                            C.byref(n)))
        return dp.value, n.value

    def scan(self, data):
        L = lib()
        p = C.POINTER(Cand)()
        n = u64(0)
        _check(L.atz_scan(self.h, data, len(data), C.byref(p), C.byref(n)))
        recs = [(p[i].offset, p[i].type, p[i].comp_len, p[i].infl_len, p[i].flags) for i in range(n.value)]
        self._cands = (p, n.value)
        return recs

    def sweep(self):
        L = lib()
        p, n = self._cands
        res = (Result * max(n, 1))()
        do = C.POINTER(u64)()
        dv = u8p()
        nd = u64(0)
        _check(L.atz_sweep(self.h, p, n, res, C.byref(do), C.byref(dv), C.byref(nd)))
        out = [{k: getattr(res[i], k) for k, _ in Result._fields_} for i in range(n)]
        diffs = ([do[i] for i in range(nd.value)], bytes(dv[i] for i in range(nd.value)))
        L.atz_free(do)
        L.atz_free(dv)
        L.atz_free(p)
        self._cands = None
        return out, diffs

    def deflate(self, data, clevel, window, memlevel):
        L = lib()
        cap = L.atz_deflate_bound(len(data), 10, 1) + 1024
        out = C.create_string_buffer(cap)
        n = u64(0)
        _check(L.atz_deflate(self.h, data, len(data), clevel, window, memlevel, out, cap, C.byref(n)))
        return out.raw[:n.value]

    def deflate_batch(self, buf, items):
        """items: list of (offset, length, clevel, window, memlevel) over `buf`; returns list of bytes."""
        L = lib()
        k = len(items)
        offs = (u64 * max(k, 1))(*[it[0] for it in items])
        lens = (u64 * max(k, 1))(*[it[1] for it in items])
        prm = (C.c_uint32 * max(k, 1))(*[(it[2] << 16) | (it[3] << 8) | it[4] for it in items])
        caps = [L.atz_deflate_bound(it[1], 10, 1) + 64 for it in items]
        oo, tot = [], 0
        for cp in caps:
            oo.append(tot)
            tot += cp
        out = C.create_string_buffer(max(tot, 1))
        ooff = (u64 * max(k, 1))(*oo)
        ocap = (u64 * max(k, 1))(*caps)
        olen = (u64 * max(k, 1))()
        _check(L.atz_deflate_batch(self.h, buf, len(buf), offs, lens, prm, k, out, ooff, ocap, olen))
        raw = out.raw
        return [raw[oo[i]:oo[i] + olen[i]] for i in range(k)]

    def inflate_batch(self, buf, ranges):
        L = lib()
        k = len(ranges)
        offs = (u64 * max(k, 1))(*[a for a, _ in ranges])
        lens = (u64 * max(k, 1))(*[b for _, b in ranges])
        st = (C.c_uint32 * max(k, 1))()
        co = (u64 * max(k, 1))()
        pr = (u64 * max(k, 1))()
        _check(L.atz_inflate_batch(self.h, buf, len(buf), offs, lens, k, st, co, pr))
        return [(st[i], co[i], pr[i]) for i in range(k)]
