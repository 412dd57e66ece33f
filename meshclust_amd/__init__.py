"""meshclust_amd -- MI355X-native engine for MeShClust's data-parallel hot path.

The product is native code built in-tree by ``meshclust_amd/csrc/Makefile``:

* ``lib/libmcgpu.so``      gfx950 HIP kernels behind the C-ABI of ``include/meshclust_amd.h``
* ``lib/libmeshclust.so``  the host driver (reference control flow) + in-process C API
* ``bin/meshclust``        drop-in CLI for the reference's ``bin/meshclust``

This module is a thin ctypes view of those libraries for tests and ``bench.py``.  It never
computes anything itself: if the libraries are missing or no GPU is present, the calls fail
loudly (``ImportError`` / ``MCError``); there is no CPU fallback.
"""
import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
LIB_DIR = os.path.join(HERE, "lib")
BIN = os.path.join(HERE, "bin", "meshclust")
GPU_LIB = os.environ.get("MC_GPU_LIB", os.path.join(LIB_DIR, "libmcgpu.so"))
HOST_LIB = os.path.join(LIB_DIR, "libmeshclust.so")
HEADER = os.path.join(ROOT, "include", "meshclust_amd.h")

FEAT_ALIGN, FEAT_LD, FEAT_MANHATTAN = 1, 2, 4
FEAT_INTERSECTION, FEAT_PEARSON, FEAT_KULCZYNSKI2 = 16, 32, 1024
COMBO_SQUARED, COMBO_SELF = 1, 2
FAMILIES = ("kmer", "keys", "pairs", "scan", "finalize", "mean_shift", "nw", "layout")


class MCError(RuntimeError):
    pass


def build(jobs=8):
    """Compile libmcgpu / libmeshclust / bin/meshclust for gfx950 (hipcc cross-compiles)."""
    subprocess.run(["make", "-s", "-j%d" % jobs, "-C", os.path.join(HERE, "csrc")], check=True)


class Classifier(C.Structure):
    _fields_ = [
        ("n_single", C.c_int32),
        ("lookup", C.c_uint16 * 8),
        ("is_sim", C.c_int32 * 8),
        ("mins", C.c_double * 8),
        ("maxs", C.c_double * 8),
        ("n_combo", C.c_int32),
        ("combo_kind", C.c_int32 * 8),
        ("combo_len", C.c_int32 * 8),
        ("combo_idx", (C.c_int32 * 4) * 8),
        ("weights", C.c_double * 9),
    ]


class ScanResult(C.Structure):
    _fields_ = [
        ("is_min", C.c_int32),
        ("has_best", C.c_int32),
        ("best_pos", C.c_uint64),
        ("best_val", C.c_double),
        ("n_flagged", C.c_uint64),
        ("new_centre", C.c_uint32),
        ("n_members", C.c_uint32),
        ("nw_pairs", C.c_uint64),
        ("nw_cells", C.c_uint64),
    ]


_gpu = None
_host = None


def _p(a):
    return a.ctypes.data_as(C.c_void_p) if a is not None else None


def gpu_lib():
    global _gpu
    if _gpu is None:
        if not os.path.exists(GPU_LIB):
            raise ImportError("libmcgpu.so not built (run meshclust_amd.build()); no CPU fallback exists")
        lib = C.CDLL(GPU_LIB)
        lib.mc_last_error.restype = C.c_char_p
        lib.mc_ctx_create.argtypes = [C.c_int, C.POINTER(C.c_void_p)]
        lib.mc_ctx_destroy.argtypes = [C.c_void_p]
        for name in ("mc_load_sequences", "mc_load_packed", "mc_kmer_max", "mc_kmer_build", "mc_get_histograms", "mc_distance_keys",
                     "mc_pair_features", "mc_set_classifier", "mc_classify_pairs", "mc_nw_identity",
                     "mc_nw_identity_raw", "mc_set_order", "mc_kill", "mc_cluster_begin", "mc_scan",
                     "mc_mean_shift", "mc_update_iteration", "mc_timers", "mc_classify_values", "mc_mean_shift_select", "mc_accumulate",
                     "mc_scan_part", "mc_scan_commit", "mc_comm_unique_id", "mc_comm_create", "mc_comm_allgather",
                     "mc_comm_stats", "mc_comm_destroy", "mc_sync"):
            getattr(lib, name).restype = C.c_int
        lib.mc_comm_create.argtypes = [C.c_int, C.c_int, C.c_int, C.c_char_p, C.POINTER(C.c_void_p)]
        lib.mc_comm_allgather.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p]
        lib.mc_comm_stats.argtypes = [C.c_void_p, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
        lib.mc_comm_destroy.argtypes = [C.c_void_p, C.c_int]
        _gpu = lib
    return _gpu


def host_lib():
    global _host
    if _host is None:
        if not os.path.exists(HOST_LIB):
            raise ImportError("libmeshclust.so not built (run meshclust_amd.build())")
        gpu_lib()
        lib = C.CDLL(HOST_LIB)
        lib.mcl_parse.restype = C.c_void_p
        lib.mcl_parse.argtypes = [C.POINTER(C.c_char_p), C.c_int, C.c_int, C.c_char_p, C.c_int]
        lib.mcl_num_seqs.restype = C.c_uint64
        lib.mcl_num_seqs.argtypes = [C.c_void_p]
        lib.mcl_view.argtypes = [C.c_void_p] + [C.POINTER(C.c_void_p)] * 4
        lib.mcl_header.restype = C.c_char_p
        lib.mcl_header.argtypes = [C.c_void_p, C.c_uint64]
        lib.mcl_free.argtypes = [C.c_void_p]
        lib.mcl_run.restype = C.c_int
        lib.mcl_run.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.POINTER(C.c_char_p), C.c_int, C.c_char_p,
                                C.c_char_p, C.c_int]
        lib.mcl_run_sharded.restype = C.c_int
        lib.mcl_run_sharded.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.POINTER(C.c_char_p), C.c_int, C.c_char_p,
                                        C.c_char_p, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p]
        lib.mcl_tune_host_heap.restype = C.c_int
        _host = lib
    return _host


def tune_host_heap():
    """Opt in (process-global): keep large freed host blocks in the heap, so repeated parses and
    clusterings in this process touch no new pages (what bin/meshclust does for itself)."""
    return bool(host_lib().mcl_tune_host_heap())


def _check(rc, what):
    if rc != 0:
        raise MCError("%s failed (%d): %s" % (what, rc, gpu_lib().mc_last_error().decode()))


class Engine:
    """One libmcgpu context on one GPU (``mc_ctx``)."""

    def __init__(self, device=0):
        self.lib = gpu_lib()
        self.ctx = C.c_void_p()
        _check(self.lib.mc_ctx_create(device, C.byref(self.ctx)), "mc_ctx_create")
        self.n = 0
        self.width = 0
        self.B = 0

    def close(self):
        if self.ctx:
            self.lib.mc_ctx_destroy(self.ctx)
            self.ctx = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def load_sequences(self, codes, seq_off, seg, seg_off):
        codes = np.ascontiguousarray(codes, np.uint8)
        seq_off = np.ascontiguousarray(seq_off, np.uint64)
        seg = np.ascontiguousarray(seg, np.int32).reshape(-1)
        seg_off = np.ascontiguousarray(seg_off, np.uint64)
        if seg.size == 0:
            seg = np.zeros(2, np.int32)
        self.n = len(seq_off) - 1
        _check(self.lib.mc_load_sequences(self.ctx, _p(codes), _p(seq_off), C.c_uint64(self.n), _p(seg),
                                          _p(seg_off)), "mc_load_sequences")

    def load_packed(self, seqs, segs):
        """seqs: list of uint8 one-digit arrays; segs: per sequence [[s, e], ...].  Packs them the
        way the host parser does (2-bit words, records word-aligned, exception bytes) and loads
        them with mc_load_packed."""
        lens = [len(x) for x in seqs]
        seq_off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
        pk_off = np.concatenate([[0], np.cumsum([(l + 15) // 16 for l in lens])]).astype(np.uint64)
        packed = np.zeros(max(1, int(pk_off[-1])), np.uint32)
        exc_pos, exc_val = [], []
        for i, x in enumerate(seqs):
            x = np.asarray(x, np.uint8)
            pad = np.zeros((len(x) + 15) // 16 * 16, np.uint32)
            pad[:len(x)] = x & 3
            w = (pad.reshape(-1, 16) << (2 * np.arange(16, dtype=np.uint32))).sum(axis=1, dtype=np.uint64)
            packed[int(pk_off[i]):int(pk_off[i + 1])] = w.astype(np.uint32)
            bad = np.nonzero(x > 3)[0]
            exc_pos.extend((int(seq_off[i]) + bad).tolist())
            exc_val.extend(x[bad].tolist())
        seg = np.array([v for s in segs for pair in s for v in pair], np.int32)
        seg_off = np.concatenate([[0], np.cumsum([len(s) for s in segs])]).astype(np.uint64)
        if seg.size == 0:
            seg = np.zeros(2, np.int32)
        ep = np.array(exc_pos, np.uint64)
        ev = np.array(exc_val, np.uint8)
        self.n = len(seqs)
        _check(self.lib.mc_load_packed(self.ctx, _p(packed), _p(pk_off), _p(seq_off), C.c_uint64(self.n),
                                       _p(ep) if len(ep) else None, _p(ev) if len(ev) else None, C.c_uint64(len(ep)),
                                       _p(seg), _p(seg_off)), "mc_load_packed")

    def kmer_max(self, k):
        out = C.c_uint64()
        _check(self.lib.mc_kmer_max(self.ctx, k, C.byref(out)), "mc_kmer_max")
        return out.value

    def kmer_build(self, k, width):
        _check(self.lib.mc_kmer_build(self.ctx, k, width), "mc_kmer_build")
        self.width, self.B = width, 4 ** k

    def histograms(self):
        dt = {1: np.uint8, 2: np.uint16, 4: np.uint32, 8: np.uint64}[self.width]
        h = np.zeros((self.n, self.B), dt)
        m = np.zeros(self.n, np.uint64)
        _check(self.lib.mc_get_histograms(self.ctx, _p(h), _p(m)), "mc_get_histograms")
        return h, m

    def distance_keys(self, pivots, ids):
        pivots = np.ascontiguousarray(pivots, np.uint32)
        ids = np.ascontiguousarray(ids, np.uint32)
        keys = np.zeros((len(pivots), len(ids)), np.uint16)
        _check(self.lib.mc_distance_keys(self.ctx, _p(pivots), C.c_uint32(len(pivots)), _p(ids),
                                         C.c_uint64(len(ids)), _p(keys)), "mc_distance_keys")
        return keys

    def pair_features(self, a, b, flags):
        a = np.ascontiguousarray(a, np.uint32)
        b = np.ascontiguousarray(b, np.uint32)
        fl = np.ascontiguousarray(flags, np.uint16)
        raw = np.zeros((len(a), len(fl)), np.float64)
        _check(self.lib.mc_pair_features(self.ctx, _p(a), _p(b), C.c_uint64(len(a)), _p(fl), len(fl), _p(raw)),
               "mc_pair_features")
        return raw

    def set_classifier(self, cls):
        _check(self.lib.mc_set_classifier(self.ctx, C.byref(cls)), "mc_set_classifier")

    def classify_pairs(self, a, b):
        a = np.ascontiguousarray(a, np.uint32)
        b = np.ascontiguousarray(b, np.uint32)
        sim = np.zeros(len(a), np.uint8)
        c0 = np.zeros(len(a))
        s = np.zeros(len(a))
        _check(self.lib.mc_classify_pairs(self.ctx, _p(a), _p(b), C.c_uint64(len(a)), _p(sim), _p(c0), _p(s)),
               "mc_classify_pairs")
        return sim, c0, s

    def classify_values(self, raw):
        """raw: (m, n_single) precomputed single-feature values -> (similar, combo0, sum)."""
        raw = np.ascontiguousarray(raw, np.float64)
        m = raw.shape[0]
        sim = np.zeros(m, np.uint8)
        c0 = np.zeros(m)
        s = np.zeros(m)
        _check(self.lib.mc_classify_values(self.ctx, _p(raw), C.c_uint64(m), _p(sim), _p(c0), _p(s)),
               "mc_classify_values")
        return sim, c0, s

    def mean_shift(self, centres, member_off, members, delta):
        centres = np.ascontiguousarray(centres, np.uint32)
        member_off = np.ascontiguousarray(member_off, np.uint64)
        members = np.ascontiguousarray(members, np.uint32)
        out = np.zeros(len(centres), np.uint32)
        _check(self.lib.mc_mean_shift(self.ctx, _p(centres), len(centres), _p(member_off), _p(members), delta, _p(out)),
               "mc_mean_shift")
        return out

    def update_iteration(self, centres, member_off, members, delta):
        """mc_update_iteration: (new centres, merge pairs' similar flags, their combo 0 values)."""
        centres = np.ascontiguousarray(centres, np.uint32)
        member_off = np.ascontiguousarray(member_off, np.uint64)
        members = np.ascontiguousarray(members, np.uint32)
        C_ = len(centres)
        m = sum(min(delta, C_ - 1 - i) for i in range(C_))
        out = np.zeros(C_, np.uint32)
        sim = np.zeros(max(m, 1), np.uint8)
        c0 = np.zeros(max(m, 1))
        n = C.c_uint64(0)
        _check(self.lib.mc_update_iteration(self.ctx, _p(centres), C_, _p(member_off), _p(members), delta, _p(out),
                                            _p(sim), _p(c0), C.byref(n)), "mc_update_iteration")
        assert n.value == m
        return out, sim[:m], c0[:m]

    def mean_shift_select(self, centres, member_off, members, delta, keep):
        centres = np.ascontiguousarray(centres, np.uint32)
        member_off = np.ascontiguousarray(member_off, np.uint64)
        members = np.ascontiguousarray(members, np.uint32)
        keep = np.ascontiguousarray(keep, np.uint8)
        out = np.zeros(len(centres), np.uint32)
        _check(self.lib.mc_mean_shift_select(self.ctx, _p(centres), len(centres), _p(member_off), _p(members), delta,
                                             _p(keep), _p(out)), "mc_mean_shift_select")
        return out

    def nw_identity(self, a, b):
        a = np.ascontiguousarray(a, np.uint32)
        b = np.ascontiguousarray(b, np.uint32)
        ident = np.zeros(len(a))
        ln = np.zeros(len(a), np.int32)
        ids = np.zeros(len(a), np.int32)
        _check(self.lib.mc_nw_identity(self.ctx, _p(a), _p(b), C.c_uint64(len(a)), _p(ident), _p(ln), _p(ids)),
               "mc_nw_identity")
        return ident, ln, ids

    def nw_identity_raw(self, a_cat, a_off, b_cat, b_off):
        a_cat = np.ascontiguousarray(a_cat, np.uint8)
        b_cat = np.ascontiguousarray(b_cat, np.uint8)
        a_off = np.ascontiguousarray(a_off, np.uint64)
        b_off = np.ascontiguousarray(b_off, np.uint64)
        m = len(a_off) - 1
        ident = np.zeros(m)
        ln = np.zeros(m, np.int32)
        ids = np.zeros(m, np.int32)
        sc = np.zeros(m, np.int32)
        _check(self.lib.mc_nw_identity_raw(self.ctx, _p(a_cat), _p(a_off), _p(b_cat), _p(b_off), C.c_uint64(m),
                                           _p(ident), _p(ln), _p(ids), _p(sc)), "mc_nw_identity_raw")
        return ident, ln, ids, sc

    def sync(self):
        """Wait for all work on this context's GPU (mc_sync)."""
        _check(self.lib.mc_sync(self.ctx), "mc_sync")

    def timers(self, reset=False):
        out = np.zeros(2 * len(FAMILIES))
        _check(self.lib.mc_timers(self.ctx, _p(out), len(out), 1 if reset else 0), "mc_timers")
        return {f: (out[2 * i], int(out[2 * i + 1])) for i, f in enumerate(FAMILIES)}


class Dataset:
    """Parsed FASTA held by libmeshclust (one parse, many GPU runs)."""

    def __init__(self, files, threads=8):
        self.lib = host_lib()
        arr = (C.c_char_p * len(files))(*[f.encode() for f in files])
        err = C.create_string_buffer(1024)
        self.h = self.lib.mcl_parse(arr, len(files), threads, err, 1024)
        if not self.h:
            raise MCError("parse failed: " + err.value.decode())
        self.n = self.lib.mcl_num_seqs(self.h)

    def records(self):
        """[(header, codes uint8, [[start, end], ...])] as parsed (ChromListMaker +
        Chromosome::help + ChromosomeOneDigit encoding)."""
        ptr = [C.c_void_p() for _ in range(4)]
        self.lib.mcl_view(self.h, *[C.byref(p) for p in ptr])
        n = self.n

        def arr(p, ct, count):
            return np.ctypeslib.as_array(C.cast(p, C.POINTER(ct)), shape=(count,)) if count else np.zeros(0)

        seq_off = arr(ptr[1], C.c_uint64, n + 1).copy()
        seg_off = arr(ptr[3], C.c_uint64, n + 1).copy()
        codes = arr(ptr[0], C.c_uint8, int(seq_off[-1])).copy()
        seg = arr(ptr[2], C.c_int32, 2 * int(seg_off[-1])).copy()
        out = []
        for i in range(n):
            s = seg[2 * int(seg_off[i]):2 * int(seg_off[i + 1])]
            out.append((self.lib.mcl_header(self.h, i).decode(), codes[int(seq_off[i]):int(seq_off[i + 1])],
                        [[int(s[j]), int(s[j + 1])] for j in range(0, len(s), 2)]))
        return out

    def run(self, engine, args=(), upload=True, clstr=None, comm=None):
        """Run the full pipeline (reference options in ``args``); returns the stats dict.
        ``comm`` (meshclust_amd.dist.RcclShardComm or TorchShardComm) shares the clustering
        over its ranks."""
        import json
        argv = [b"meshclust"] + [a.encode() for a in args]
        arr = (C.c_char_p * len(argv))(*argv)
        buf = C.create_string_buffer(1 << 16)
        if comm is not None:
            rc = self.lib.mcl_run_sharded(self.h, engine.ctx, len(argv), arr, 1 if upload else 0,
                                          clstr.encode() if clstr else None, buf, len(buf), comm.rank, comm.world,
                                          C.cast(comm.callback, C.c_void_p), comm.user)
        else:
            rc = self.lib.mcl_run(self.h, engine.ctx, len(argv), arr, 1 if upload else 0,
                                  clstr.encode() if clstr else None, buf, len(buf))
        st = json.loads(buf.value.decode() or "{}")
        if rc != 0 or "error" in st:  # incl. the reference's exit(0) stops (no partition)
            raise MCError("mcl_run failed (%d): %s" % (rc, st))
        return st

    def __del__(self):
        try:
            self.lib.mcl_free(self.h)
        except Exception:
            pass
