"""ctypes handles on the test-side libraries (oracle restatement, reference shim) and input generators.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module.
"""
import ctypes as C
import os
import random
import zlib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_SO = os.path.join(ROOT, "oracle", "_build", "libatz_oracle.so")
ZREF_SO = os.path.join(ROOT, "oracle", "_ref", "libzref.so")
REF_UNCOMP = os.path.join(ROOT, "oracle", "_ref", "uncomp")

u8p = C.POINTER(C.c_uint8)
u64 = C.c_uint64


class OraOpts(C.Structure):
    _fields_ = [("recomp_tresh", u64), ("sizediff_tresh", u64), ("shortcut_len", u64),
                ("mismatch_tol", u64), ("chunksize", u64), ("brute_window", C.c_int)]


class OraStream(C.Structure):
    _fields_ = [("offset", u64), ("type", C.c_int32), ("clevel", C.c_uint8), ("window", C.c_uint8),
                ("memlevel", C.c_uint8), ("recomp", C.c_uint8), ("comp_len", u64), ("infl_len", u64),
                ("ident", u64), ("first_diff", C.c_int64), ("n_diff", u64), ("diff_index", u64),
                ("n_trials", u64)]


class OraResult(C.Structure):
    _fields_ = [("streams", C.POINTER(OraStream)), ("n_streams", u64), ("diff_off", C.POINTER(u64)),
                ("diff_val", u8p), ("n_diffs", u64), ("n_trials", u64), ("n_shortcut_bailed", u64),
                ("n_hazard", u64)]


_ora = None
_zref = None


def ora():
    global _ora
    if _ora is None:
        L = C.CDLL(ORACLE_SO)
        L.ora_deflate.argtypes = [C.c_char_p, u64, C.c_int, C.c_int, C.c_int, C.c_char_p, u64,
                                  C.POINTER(u64), C.POINTER(C.c_int)]
        L.ora_deflate_bound.restype = u64
        L.ora_deflate_bound.argtypes = [u64, C.c_int, C.c_int]
        L.ora_inflate.argtypes = [C.c_char_p, u64, C.c_char_p, u64, C.POINTER(u64), C.POINTER(u64)]
        L.ora_scan.argtypes = [C.c_char_p, u64, u64, C.POINTER(OraResult)]
        L.ora_sweep.argtypes = [C.c_char_p, u64, C.POINTER(OraOpts), C.POINTER(OraResult)]
        L.ora_precompress.argtypes = [C.c_char_p, u64, C.POINTER(OraOpts), C.POINTER(u8p), C.POINTER(u64),
                                      C.POINTER(OraResult)]
        L.ora_reconstruct.argtypes = [C.c_char_p, u64, C.POINTER(u8p), C.POINTER(u64)]
        L.ora_result_free.argtypes = [C.POINTER(OraResult)]
        L.ora_free.argtypes = [C.c_void_p]
        _ora = L
    return _ora


def zref():
    global _zref
    if _zref is None:
        L = C.CDLL(ZREF_SO)
        L.zref_deflate.argtypes = [C.c_char_p, C.c_ulong, C.c_int, C.c_int, C.c_int, C.c_char_p,
                                   C.c_ulong, C.POINTER(C.c_ulong)]
        L.zref_deflate_bound.restype = C.c_ulong
        L.zref_deflate_bound.argtypes = [C.c_ulong, C.c_int, C.c_int, C.c_int]
        L.zref_deflate_shortcut.argtypes = [C.c_char_p, C.c_ulong, C.c_int, C.c_int, C.c_int, C.c_uint,
                                            C.c_char_p, C.POINTER(C.c_ulong), C.POINTER(C.c_ulong)]
        L.zref_inflate_scan.argtypes = [C.c_char_p, C.c_ulong, C.c_ulong, C.POINTER(C.c_int),
                                        C.POINTER(C.c_ulong), C.POINTER(C.c_int), C.POINTER(C.c_ulong),
                                        C.POINTER(C.c_ulong), C.POINTER(C.c_ulong)]
        L.zref_inflate.argtypes = [C.c_char_p, C.c_ulong, C.c_char_p, C.c_ulong, C.POINTER(C.c_ulong),
                                   C.POINTER(C.c_ulong)]
        _zref = L
    return _zref


def have_zref():
    return os.path.exists(ZREF_SO)


def ora_deflate(data, c, w, m):
    L = ora()
    cap = L.ora_deflate_bound(len(data), 10, 1) + 1024
    out = C.create_string_buffer(cap)
    n = u64(0)
    fl = C.c_int(0)
    r = L.ora_deflate(data, len(data), c, w, m, out, cap, C.byref(n), C.byref(fl))
    assert r == 0, r
    return out.raw[:n.value], fl.value


def zref_deflate(data, c, w, m):
    L = zref()
    cap = L.zref_deflate_bound(len(data), c, w, m) + 64
    out = C.create_string_buffer(cap)
    n = C.c_ulong(0)
    r = L.zref_deflate(data, len(data), c, w, m, out, cap, C.byref(n))
    assert r == 0, r
    return out.raw[:n.value]


def ora_inflate(data):
    L = ora()
    c = u64(0)
    p = u64(0)
    st = L.ora_inflate(data, len(data), None, 0, C.byref(c), C.byref(p))
    return st, c.value, p.value


def zref_inflate_scan(data, bufsz=524288):
    L = zref()
    rf = C.c_int()
    tf = C.c_ulong()
    rl = C.c_int()
    ti = C.c_ulong()
    to = C.c_ulong()
    ai = C.c_ulong()
    L.zref_inflate_scan(data, len(data), bufsz, C.byref(rf), C.byref(tf), C.byref(rl), C.byref(ti),
                        C.byref(to), C.byref(ai))
    return rf.value, tf.value, rl.value, ti.value, to.value, ai.value


def ora_precompress(data, chunksize=524288, recomp=128, sizediff=128, shortcut=512, tol=2, brute=0):
    L = ora()
    o = OraOpts(recomp, sizediff, shortcut, tol, chunksize, brute)
    p = u8p()
    n = u64(0)
    res = OraResult()
    r = L.ora_precompress(data, len(data), C.byref(o), C.byref(p), C.byref(n), C.byref(res))
    if r != 0:
        L.ora_result_free(C.byref(res))
        return r, None, None
    atz = C.string_at(p, n.value)
    L.ora_free(p)
    streams = [{k: getattr(res.streams[i], k) for k, _ in OraStream._fields_} for i in range(res.n_streams)]
    stats = dict(trials=res.n_trials, bailed=res.n_shortcut_bailed, hazard=res.n_hazard, streams=streams)
    L.ora_result_free(C.byref(res))
    return 0, atz, stats


def ora_reconstruct(atz):
    L = ora()
    p = u8p()
    n = u64(0)
    r = L.ora_reconstruct(atz, len(atz), C.byref(p), C.byref(n))
    if r != 0:
        return r, None
    out = C.string_at(p, n.value)
    L.ora_free(p)
    return 0, out


# ----------------------------------------------------------------------------------------------
# Deterministic synthetic inputs: seeded vocabulary text.
def vocab(seed=12345, n=20000):
    r = random.Random(seed)
    letters = "abcdefghijklmnopqrstuvwxyz"
    return ["".join(r.choice(letters) for _ in range(r.randint(2, 10))) for _ in range(n)]


_VOCAB = None


def text(r, nbytes):
    global _VOCAB
    if _VOCAB is None:
        _VOCAB = vocab()
    out = []
    size = 0
    while size < nbytes:
        w = r.choice(_VOCAB)
        out.append(w)
        size += len(w) + 1
    return (" ".join(out)).encode()[:nbytes]
