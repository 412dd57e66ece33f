"""ctypes view of oracle/_build/libmcoracle.so (the CPU checker; TEST INFRASTRUCTURE)."""
import ctypes as C
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.path.join(ROOT, "oracle", "_build", "libmcoracle.so")

MAXS, MAXC, MAXL = 8, 8, 4


class Classifier(C.Structure):
    _fields_ = [
        ("n_single", C.c_int32),
        ("lookup", C.c_uint16 * MAXS),
        ("is_sim", C.c_int32 * MAXS),
        ("mins", C.c_double * MAXS),
        ("maxs", C.c_double * MAXS),
        ("n_combo", C.c_int32),
        ("combo_kind", C.c_int32 * MAXC),
        ("combo_len", C.c_int32 * MAXC),
        ("combo_idx", (C.c_int32 * MAXL) * MAXC),
        ("weights", C.c_double * (MAXC + 1)),
    ]


def classifier_from_golden(g):
    """Build an mc_classifier from a train_*.npz golden (Feature + GLM weight dump)."""
    c = Classifier()
    c.n_single = len(g["lookup"])
    for i, v in enumerate(g["lookup"]):
        c.lookup[i] = int(v)
        c.is_sim[i] = int(g["is_sim"][i])
        c.mins[i] = float(g["mins"][i])
        c.maxs[i] = float(g["maxs"][i])
    combos = g["combos"]
    c.n_combo = len(combos)
    for i, row in enumerate(combos):
        idx = [int(x) for x in row[1:] if x >= 0]
        c.combo_kind[i] = int(row[0])
        c.combo_len[i] = len(idx)
        for j, x in enumerate(idx):
            c.combo_idx[i][j] = x
    for i, w in enumerate(g["weights"]):
        c.weights[i] = float(w)
    return c


_lib = None


def lib():
    global _lib
    if _lib is None:
        L = C.CDLL(LIB_PATH)
        u8p = np.ctypeslib.ndpointer(np.uint8, flags="C")
        L.mco_kmer_hist.argtypes = [u8p, C.c_int64, np.ctypeslib.ndpointer(np.int32, flags="C"),
                                    C.c_int, C.c_int, C.c_uint64,
                                    np.ctypeslib.ndpointer(np.uint64, flags="C")]
        L.mco_distance.restype = C.c_uint64
        L.mco_distance.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_uint64, C.c_uint64]
        L.mco_distance_d.restype = C.c_double
        L.mco_distance_d.argtypes = [C.c_void_p, C.c_int, C.c_int, np.ctypeslib.ndpointer(np.float64, flags="C")]
        L.mco_raw.argtypes = [C.c_uint16, C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_uint64,
                              C.c_uint64, C.c_uint64, C.c_uint64, C.POINTER(C.c_double)]
        L.mco_classify.argtypes = [C.POINTER(Classifier), np.ctypeslib.ndpointer(np.float64, flags="C"),
                                   C.POINTER(C.c_double), C.POINTER(C.c_double)]
        L.mco_nw.argtypes = [C.c_char_p, C.c_int, C.c_char_p, C.c_int, C.c_int, C.c_int, C.c_int,
                             C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_int),
                             C.POINTER(C.c_double)]
        _lib = L
    return _lib


def kmer_hist(codes, segments, k, init=1):
    codes = np.ascontiguousarray(codes, dtype=np.uint8)
    seg = np.ascontiguousarray(np.array(segments, dtype=np.int32).reshape(-1))
    out = np.zeros(4 ** k, dtype=np.uint64)
    rc = lib().mco_kmer_hist(codes, len(codes), seg if seg.size else np.zeros(1, np.int32),
                             len(segments), k, init, out)
    if rc:
        raise ValueError("mco_kmer_hist rc=%d" % rc)
    return out


def _ptr(a):
    return a.ctypes.data_as(C.c_void_p)


def distance(p, q):
    return lib().mco_distance(_ptr(p), _ptr(q), p.itemsize, p.size, int(p.sum(dtype=np.uint64)),
                              int(q.sum(dtype=np.uint64)))


def distance_d(p, mean):
    return lib().mco_distance_d(_ptr(p), p.itemsize, p.size, np.ascontiguousarray(mean, np.float64))


def raw(flag, p, q, lenp, lenq):
    out = C.c_double()
    rc = lib().mco_raw(flag, _ptr(p), _ptr(q), p.itemsize, p.size, int(p.sum(dtype=np.uint64)),
                       int(q.sum(dtype=np.uint64)), lenp, lenq, C.byref(out))
    if rc:
        raise ValueError("mco_raw rc=%d" % rc)
    return out.value


def classify(cls, raw_vals):
    s, c0 = C.c_double(), C.c_double()
    d = lib().mco_classify(C.byref(cls), np.ascontiguousarray(raw_vals, np.float64), C.byref(s), C.byref(c0))
    return d, s.value, c0.value


def nw(a, b, match=1, mismatch=-1, gap_open=2, gap_ext=1):
    sc, ln, ids, ident = C.c_int(), C.c_int(), C.c_int(), C.c_double()
    lib().mco_nw(bytes(a), len(a), bytes(b), len(b), match, mismatch, gap_open, gap_ext,
                 C.byref(sc), C.byref(ln), C.byref(ids), C.byref(ident))
    return ident.value, ln.value, ids.value, sc.value
