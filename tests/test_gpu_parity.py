"""GPU parity: libmcgpu (through its C-ABI) against the reference goldens and the C oracle.

Bit-exact everywhere: integer histograms / sort keys / NW lengths and identity counts, and
the IEEE-double features, GLM sums and decisions compared with ==.  End to end, the shipped
bin/meshclust must reproduce the reference's --threads 1 .clstr byte for byte.
"""
import gzip
import os
import subprocess
import sys

import numpy as np
import pytest

import fixtures
import meshclust_amd as M
import oracle_lib as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng(built):
    M.build()
    e = M.Engine(0)
    yield e
    e.close()


def load_records(eng, recs):
    """recs: list of (codes uint8, segments [[s,e],...])."""
    codes = np.concatenate([c for c, _ in recs]).astype(np.uint8)
    seq_off = np.cumsum([0] + [len(c) for c, _ in recs]).astype(np.uint64)
    seg = np.array([x for _, s in recs for pair in s for x in pair], np.int32)
    seg_off = np.cumsum([0] + [len(s) for _, s in recs]).astype(np.uint64)
    eng.load_sequences(codes, seq_off, seg, seg_off)


@pytest.mark.parametrize("k", [1, 3, 4, 6])
def test_kmer_hist_edge(eng, k):
    recs = [(np.frombuffer(bytes.fromhex(r["data_hex"]), np.uint8), r["segments"]) for r in fixtures.edge_records()]
    g = np.load(fixtures.golden("edge_hist.npz"))
    load_records(eng, recs)
    assert eng.kmer_max(k) == int(g["k%d" % k].max())
    eng.kmer_build(k, 1 if g["k%d" % k].max() <= 255 else 2)
    h, mags = eng.histograms()
    assert np.array_equal(h.astype(np.uint64), g["k%d" % k])
    assert np.array_equal(mags, g["mag%d" % k])


def test_kmer_widths_match_oracle(eng):
    """u16/u32 histograms (forced widths) on long low-complexity sequences."""
    rng = np.random.default_rng(3)
    recs = []
    for i in range(40):
        L = int(rng.integers(300, 5000))
        c = rng.integers(0, 2 if i % 3 == 0 else 4, size=L).astype(np.uint8)
        recs.append((c, [[0, L - 1]]))
    load_records(eng, recs)
    for k in (2, 4):
        want = np.array([O.kmer_hist(c, s, k) for c, s in recs])
        assert eng.kmer_max(k) == int(want.max())
        for width, dt in ((2, np.uint16), (4, np.uint32), (8, np.uint64)):
            if want.max() > np.iinfo(dt).max:
                continue
            eng.kmer_build(k, width)
            h, _ = eng.histograms()
            assert h.dtype == dt and np.array_equal(h.astype(np.uint64), want)


@pytest.mark.parametrize("mean_len", [900, 9000])
def test_kmer_all_k_and_table_modes_vs_oracle(eng, mean_len):
    """K1's three table modes against the oracle: per-wave LDS tables (k <= 6), one shared LDS
    table (k = 7), per-wave global tables (k >= 8); one wave per sequence (short) and the
    waves of a workgroup sharing a sequence (mean length >= 4 kb).  Sequences with several
    segments, an 'N' outside segments (impure: byte path) and lengths not a multiple of 16."""
    rng = np.random.default_rng(11 + mean_len)
    recs = []
    for i in range(24):
        L = int(rng.integers(mean_len // 2, mean_len * 3 // 2)) + (i % 16)
        c = rng.integers(0, 4, size=L).astype(np.uint8)
        if i % 3 == 0:
            a = L // 3
            c[a:a + 30] = 78  # 'N' run outside the segments
            recs.append((c, [[0, a - 1], [a + 30, L - 1]]))
        else:
            recs.append((c, [[0, L - 1]]))
    load_records(eng, recs)
    for k in (1, 2, 5, 7, 8):
        want = np.array([O.kmer_hist(c, s, k) for c, s in recs])
        width = 1 if want.max() <= 255 else 2
        assert eng.kmer_max(k) == int(want.max()), k
        eng.kmer_build(k, width)
        h, mags = eng.histograms()
        assert np.array_equal(h.astype(np.uint64), want), k
        assert np.array_equal(mags, want.sum(axis=1)), k


@pytest.mark.parametrize("k", [4, 5, 6])
def test_kmer_stream_equals_general(eng, k, monkeypatch):
    """K1's streaming form (8-bit rows, k = 4..6: the next sequence's words in flight while the
    current one is counted, statistics stored per 64 sequences; k compiled in, and k at run time)
    against the general form
    (MC_KMER_NO_STREAM) and the oracle: several 64-sequence batches per wave, sequences longer
    than 64 16-start groups, several segments, 'N' bytes (impure), segments shorter than k.
    The PEARSON feature checks the sums of squares, the histograms and magnitudes the rest."""
    rng = np.random.default_rng(40 + k)
    recs = []
    for i in range(1500):
        L = int(rng.integers(20, 2600)) if i % 50 else int(rng.integers(1, 8))
        c = rng.integers(0, 4, size=L).astype(np.uint8)
        if i % 7 == 0 and L > 60:
            a = L // 2
            c[a:a + 9] = 78
            recs.append((c, [[0, a - 1], [a + 9, L - 1]]))
        else:
            recs.append((c, [[0, L - 1]]))
    recs = [r for r in recs if all(e - s + 1 >= k for s, e in r[1])]
    load_records(eng, recs)
    want = np.array([O.kmer_hist(c, s, k) for c, s in recs])
    assert want.max() <= 255
    ij = np.array([(i, (i * 7 + 3) % len(recs)) for i in range(len(recs))], np.uint32)
    flags = [(1 << 5), (1 << 4), (1 << 2)]  # PEARSON, INTERSECTION, MANHATTAN
    out = {}
    for mode in ("stream", "runtime_k", "general"):
        if mode == "runtime_k":  # the streaming form with k a run-time value (not K = 4 / 5 / 6)
            monkeypatch.setenv("MC_KMER_RUNTIME_K", "1")
        if mode == "general":
            monkeypatch.setenv("MC_KMER_NO_STREAM", "1")
        assert eng.kmer_max(k) == int(want.max())
        eng.kmer_build(k, 1)
        h, mags = eng.histograms()
        assert np.array_equal(h.astype(np.uint64), want), mode
        assert np.array_equal(mags, want.sum(axis=1)), mode
        out[mode] = eng.pair_features(ij[:, 0], ij[:, 1], flags)
    assert np.array_equal(out["stream"], out["general"])
    assert np.array_equal(out["runtime_k"], out["general"])


def test_load_packed_equals_bytes(eng):
    """mc_load_packed (2-bit words + exception bytes, the host parser's form) leaves the same
    sequences on the device as mc_load_sequences: same histograms, same NW identities."""
    rng = np.random.default_rng(12)
    recs = []
    for i in range(40):
        L = int(rng.integers(20, 700))
        c = rng.integers(0, 4, size=L).astype(np.uint8)
        if i % 4 == 0:
            c[L // 2:L // 2 + 12] = 78
        recs.append((c, [[0, L // 2 - 1]] if i % 4 == 0 else [[0, L - 1]]))
    load_records(eng, recs)
    eng.kmer_build(3, 1)
    h0, m0 = eng.histograms()
    a = np.arange(40, dtype=np.uint32)
    b = (a * 7 + 3) % 40
    id0 = eng.nw_identity(a, b)
    eng.load_packed([c for c, _ in recs], [s for _, s in recs])
    eng.kmer_build(3, 1)
    h1, m1 = eng.histograms()
    assert np.array_equal(h0, h1) and np.array_equal(m0, m1)
    id1 = eng.nw_identity(a, b)
    for x, y in zip(id0, id1):
        assert np.array_equal(x, y)


def test_nw_golden(eng):
    g = np.load(fixtures.golden("nw.npz"))
    ident, ln, ids, sc = eng.nw_identity_raw(g["a"], g["a_off"], g["b"], g["b_off"])
    assert np.array_equal(ln, g["length"])
    assert np.array_equal(ids, g["ids"])
    assert np.array_equal(sc, g["score"])
    assert np.array_equal(ident, g["identity"])


def test_nw_golden_batch_paths(eng):
    """The golden pairs through both launch forms: a small batch (one multi-wave workgroup per
    pair, DPP lane shifts, LDS ring between waves) and a batch of >= 1024 pairs (one wavefront
    per pair)."""
    g = np.load(fixtures.golden("nw.npz"))
    n = len(g["a_off"]) - 1
    for reps in (1, (1024 + n - 1) // n + 1):
        la = np.diff(g["a_off"])
        lb = np.diff(g["b_off"])
        a = np.tile(g["a"], reps)
        b = np.tile(g["b"], reps)
        a_off = np.concatenate([[0], np.cumsum(np.tile(la, reps))])
        b_off = np.concatenate([[0], np.cumsum(np.tile(lb, reps))])
        ident, ln, ids, sc = eng.nw_identity_raw(a, a_off, b, b_off)
        assert np.array_equal(ln, np.tile(g["length"], reps)), reps
        assert np.array_equal(ids, np.tile(g["ids"], reps)), reps
        assert np.array_equal(sc, np.tile(g["score"], reps)), reps


def test_nw_long_multiblock_vs_oracle(eng):
    """Pairs longer than one row block of either launch form (boundary row in scratch: the
    latency form's blocks are 64*R*W rows, 4096 at W = 8, 8192 at W = 16)."""
    rng = np.random.default_rng(9)
    pairs = []
    for la, lb in ((1500, 1400), (2100, 2500), (4000, 3900), (1025, 1030), (3000, 200), (5000, 4900),
                   (9000, 8500)):
        a = rng.integers(0, 4, size=la).astype(np.uint8)
        b = a[:lb].copy() if lb <= la else np.concatenate([a, rng.integers(0, 4, size=lb - la).astype(np.uint8)])
        flip = rng.random(len(b)) < 0.08
        b[flip] = rng.integers(0, 4, size=int(flip.sum()))
        pairs.append((a, b))
    a_cat = np.concatenate([a for a, _ in pairs])
    b_cat = np.concatenate([b for _, b in pairs])
    a_off = np.cumsum([0] + [len(a) for a, _ in pairs])
    b_off = np.cumsum([0] + [len(b) for _, b in pairs])
    ident, ln, ids, sc = eng.nw_identity_raw(a_cat, a_off, b_cat, b_off)
    for i, (a, b) in enumerate(pairs):
        w = O.nw(a.tobytes(), b.tobytes())
        assert (ident[i], ln[i], ids[i], sc[i]) == w, i
    # the same pairs in a batch of >= 1024 (one wavefront per pair, 1024-row blocks)
    reps = 1024 // len(pairs) + 1
    la = np.diff(a_off)
    lb = np.diff(b_off)
    big = eng.nw_identity_raw(np.tile(a_cat, reps), np.concatenate([[0], np.cumsum(np.tile(la, reps))]),
                              np.tile(b_cat, reps), np.concatenate([[0], np.cumsum(np.tile(lb, reps))]))
    for got, want in zip(big, (ident, ln, ids, sc)):
        assert np.array_equal(got, np.tile(want, reps))


_LONG_PAIRS_SCRIPT = r"""
import sys, numpy as np
sys.path[:0] = [sys.argv[1], __import__("os").path.dirname(sys.argv[1])]
import meshclust_amd as M, oracle_lib as O
rng = np.random.default_rng(11)
pairs = []
for la, lb in ((1500, 1400), (2100, 2500), (4000, 3900), (513, 700), (1025, 63), (3000, 200), (9000, 8500),
               (12000, 11000), (4100, 64), (2049, 1)):
    a = rng.integers(0, 4, size=la).astype(np.uint8)
    b = a[:lb].copy() if lb <= la else np.concatenate([a, rng.integers(0, 4, size=lb - la).astype(np.uint8)])
    flip = rng.random(len(b)) < 0.08
    b[flip] = rng.integers(0, 4, size=int(flip.sum()))
    pairs.append((a, b))
e = M.Engine(0)
a_off = np.cumsum([0] + [len(a) for a, _ in pairs])
b_off = np.cumsum([0] + [len(b) for _, b in pairs])
got = e.nw_identity_raw(np.concatenate([a for a, _ in pairs]), a_off, np.concatenate([b for _, b in pairs]), b_off)
for i, (a, b) in enumerate(pairs):
    w = O.nw(a.tobytes(), b.tobytes())
    assert tuple(x[i] for x in got) == w, (i, tuple(x[i] for x in got), w)
print("ok", len(pairs))
"""


@pytest.mark.parametrize("env", [{"MC_NW_CHAIN": "0"}, {"MC_NW_CHAIN_R": "8"}, {"MC_NW_CHAIN_R": "16"},
                                 {"MC_NW_CHAIN": "2", "MC_NW_MW_MAX": "0"}],
                         ids=["sequential", "chain_r8", "chain_r16", "chain_throughput"])
def test_nw_long_pairs_chain_forms_vs_oracle(built, env):
    """Long pairs (up to 12 kb: many row blocks) in every form of the row-block hand-off: the
    blocks of a pair in sequence inside one workgroup (MC_NW_CHAIN=0), chained single-wave
    blocks of 8 and of 16 rows per lane (the default takes 8 for batches averaging above 4 kb),
    and the throughput form's pairs chained too (MC_NW_CHAIN=2).  The settings are read once per
    process: a child process each."""
    here = os.path.dirname(os.path.abspath(__file__))
    r = subprocess.run([sys.executable, "-c", _LONG_PAIRS_SCRIPT, here], capture_output=True, text=True,
                       timeout=300, env=dict(os.environ, **env))
    assert r.returncode == 0 and "ok" in r.stdout, r.stderr[-2000:]


@pytest.fixture(scope="module")
def a1k(eng):
    g = np.load(fixtures.golden("train_a1k.npz"))
    man = fixtures.manifest()["e2e"]["a1k"]["generator"]
    recs = fixtures.synth_records(*man)
    load_records(eng, [(c, [[0, L - 1]]) for _, c, L in recs])
    k = int(g["k"])
    eng.kmer_build(k, 1)
    return g, recs


def test_distance_keys_golden(eng, a1k):
    g, recs = a1k
    ij = g["pair_ij"]
    n = 40
    keys = eng.distance_keys(np.arange(n), np.arange(n))  # keys[p, i] = distance(i, p)
    want = g["distance"].reshape(n, n)                     # row i, col j: points[i].distance(points[j])
    assert np.array_equal(keys.T.astype(np.uint64), want)
    assert ij[1][0] == 0 and ij[1][1] == 1


def test_distance_keys_many_pivots_vs_oracle(eng, a1k):
    g, recs = a1k
    h, mags = eng.histograms()
    rng = np.random.default_rng(1)
    piv = rng.choice(len(recs), size=150, replace=False)
    keys = eng.distance_keys(piv, np.arange(len(recs)))
    for pi in range(0, 150, 37):
        for i in range(0, len(recs), 53):
            assert keys[pi, i] == O.distance(h[i], h[piv[pi]])


def test_features_and_classify_golden(eng, a1k):
    g, recs = a1k
    ij = g["pair_ij"]
    flags = [2, 16, 4, 32, 1024]
    raw = eng.pair_features(ij[:, 0], ij[:, 1], flags)
    assert np.array_equal(raw, g["raw"])
    eng.set_classifier(O.classifier_from_golden(g))
    sim, c0, s = eng.classify_pairs(ij[:, 0], ij[:, 1])
    assert np.array_equal(s, g["sums"])
    assert np.array_equal(sim, g["decision"].astype(np.uint8))
    assert np.array_equal(c0, g["combo_vals"][:, 0])


def test_nw_loaded_sequences(eng, a1k):
    g, recs = a1k
    pos = g["pos"]
    a, b = pos[:64, 0].astype(np.uint32), pos[:64, 1].astype(np.uint32)
    ident, _, _ = eng.nw_identity(a, b)
    assert np.array_equal(ident, pos[:64, 2])


# every e2e golden, plus the ones only the GPU runs in reasonable time: config C's shape at
# 2,000 reads (--id 0.55 --align: one NW per centre x candidate, memoised, Feature.cpp:221-243)
E2E = sorted(fixtures.manifest()["e2e"]) + sorted(fixtures.manifest().get("e2e_gpu", {}))


@pytest.mark.parametrize("name", E2E)
def test_e2e_cli_byte_identical(eng, name, tmp_path):
    fa, flags = fixtures.e2e_input(name, tmp_path)
    out = tmp_path / (name + ".clstr")
    r = subprocess.run([M.BIN, fa] + flags + ["--output", str(out), "--quiet"], capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    with gzip.open(fixtures.golden("e2e_%s.clstr.gz" % name), "rb") as f:
        assert out.read_bytes() == f.read()


@pytest.mark.parametrize("env", [{"MC_NW_LOOKAHEAD": "1"}, {"MC_NW_LOOKAHEAD": "3"}, {"MC_NW_SPINE": "0"},
                                 {"MC_PAGEABLE_UPLOADS": "1"}, {"MC_NW_WAVES": "2"}, {"MC_NW_WAVES": "16"}],
                         ids=["lookahead1", "lookahead3", "nospine", "pageable", "nw2waves", "nw16waves"])
@pytest.mark.parametrize("name", ["b3k300", "fam2k_id85", "c2k_m15_al55"])
def test_e2e_cli_variants_byte_identical(eng, name, env, tmp_path):
    """The training search's speculation (Trainer.cpp:703-721: the left-spine round on or off,
    one level per round -- the reference's order -- or three), the upload path and the NW latency form's width (2 / 16
    waves per pair for every small batch; c2k_m15_al55: the --align window scans) do not change
    the output."""
    fa, flags = fixtures.e2e_input(name, tmp_path)
    out = tmp_path / (name + ".clstr")
    r = subprocess.run([M.BIN, fa] + flags + ["--output", str(out), "--quiet"], capture_output=True, text=True,
                       timeout=600, env=dict(os.environ, **env))
    assert r.returncode == 0, r.stderr[-3000:]
    with gzip.open(fixtures.golden("e2e_%s.clstr.gz" % name), "rb") as f:
        assert out.read_bytes() == f.read()


# ---------------------------------------------------------------- alignment mode
def align_classifier(cutoff):
    """The classifier Trainer::train installs for k == 0 (Trainer.cpp:570-577)."""
    c = O.Classifier()
    c.n_single = 1
    c.lookup[0] = 1  # FEAT_ALIGN
    c.is_sim[0] = 1
    c.mins[0], c.maxs[0] = 0.0, 1.0  # Feature::normalize (Feature.cpp:90-95)
    c.n_combo = 1
    c.combo_kind[0] = 2  # COMBO_SELF
    c.combo_len[0] = 1
    c.combo_idx[0][0] = 0
    c.weights[0], c.weights[1] = -cutoff, 1.0
    return c


def test_nw_empty_strings_vs_oracle(eng):
    """GlobAlignE with len1 or len2 == 1 (a Center clone carries no data string)."""
    rng = np.random.default_rng(4)
    pairs = [(b"", b""), (b"", bytes([1])), (bytes([2]), b""), (b"", bytes(rng.integers(0, 4, 700, np.uint8))),
             (bytes(rng.integers(0, 4, 1500, np.uint8)), b""), (bytes([0, 1, 2]), bytes([0, 1, 2]))]
    a_cat = np.frombuffer(b"".join(a for a, _ in pairs), np.uint8)
    b_cat = np.frombuffer(b"".join(b for _, b in pairs), np.uint8)
    a_off = np.cumsum([0] + [len(a) for a, _ in pairs])
    b_off = np.cumsum([0] + [len(b) for _, b in pairs])
    ident, ln, ids, sc = eng.nw_identity_raw(a_cat, a_off, b_cat, b_off)
    for i, (a, b) in enumerate(pairs):
        wi, wl, wd, ws = O.nw(a, b)
        assert (ln[i], ids[i], sc[i]) == (wl, wd, ws), i
        assert ident[i] == wi or (np.isnan(ident[i]) and np.isnan(wi)), i


@pytest.mark.parametrize("cutoff", [0.55, 0.8, 0.9])
def test_align_classify_values_vs_oracle(eng, a1k, cutoff):
    cls = align_classifier(cutoff)
    eng.set_classifier(cls)
    vals = np.array([0.0, 1.0, cutoff, np.nextafter(cutoff, 0), np.nextafter(cutoff, 1), np.nan, 0.5, 0.93, 1e-300])
    sim, c0, s = eng.classify_values(vals[:, None])
    for i, v in enumerate(vals):
        d, ws, wc0 = O.classify(cls, [v])
        assert sim[i] == d, (v, sim[i], d)
        assert (s[i] == ws or (np.isnan(s[i]) and np.isnan(ws))) and (c0[i] == wc0 or np.isnan(wc0)), v


def _mean_closest_py(h, ids):
    """get_mean / Trainer::closest restated with the oracle's distance_d (first minimum)."""
    mean = h[ids].astype(np.float64).sum(axis=0) / len(ids)
    best, bd = None, None
    for i in ids:
        d = O.distance_d(h[i], mean)
        if best is None or d < bd:
            best, bd = i, d
    return best


def test_mean_shift_select_vs_oracle(eng, a1k):
    g, recs = a1k
    h, _ = eng.histograms()
    rng = np.random.default_rng(8)
    C, delta = 12, 2
    sizes = rng.integers(1, 30, size=C)
    members = rng.choice(len(recs), size=int(sizes.sum()), replace=False).astype(np.uint32)
    off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint64)
    centres = members[off[:-1].astype(np.int64)]
    keep, want = [], []
    for j in range(C):
        b, e = max(0, j - delta), min(C - 1, j + delta)
        nb = members[int(off[b]):int(off[e + 1])]
        kj = (rng.random(len(nb)) < (0.0 if j == 3 else 0.4)).astype(np.uint8)
        keep.append(kj)
        kept = [int(x) for x, k in zip(nb, kj) if k]
        want.append(int(centres[j]) if not kept else _mean_closest_py(h, kept))
    eng.set_classifier(align_classifier(0.9))
    got = eng.mean_shift_select(centres, off, members, delta, np.concatenate(keep))
    assert list(got) == want


def test_update_iteration_equals_separate_calls(eng, a1k):
    """mc_update_iteration (mean shift + merge pairs in one round trip) == mc_mean_shift followed
    by mc_classify_pairs on the new centres (ClusterFactory.cpp:740-760); twice with the same
    member lists (the device copy is reused) and once after they change."""
    g, recs = a1k
    eng.set_classifier(O.classifier_from_golden(g))
    rng = np.random.default_rng(11)
    for it, delta in enumerate([3, 3, 2]):
        C = 20
        sizes = rng.integers(1, 40, size=C)
        if it == 1:
            sizes = prev_sizes
        members = prev_members if it == 1 else rng.choice(len(recs), size=int(sizes.sum()), replace=False).astype(np.uint32)
        off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint64)
        centres = members[off[:-1].astype(np.int64)]
        if it == 1:
            centres = centres[::-1].copy()
        prev_sizes, prev_members = sizes, members
        newc, sim, c0 = eng.update_iteration(centres, off, members, delta)
        want = eng.mean_shift(centres, off, members, delta)
        assert np.array_equal(newc, want)
        pa = [want[t] for i in range(C) for t in range(i + 1, min(C - 1, i + delta) + 1)]
        pb = [want[i] for i in range(C) for t in range(i + 1, min(C - 1, i + delta) + 1)]
        s2, c2, _ = eng.classify_pairs(np.array(pa), np.array(pb))
        assert np.array_equal(sim, s2) and np.array_equal(c0, c2)


# ---------------------------------------------------------------- device-resident accumulation
ACC_CASES = {
    "b20k": ((20000, 1000, 200, 0.03, 71), ["--id", "0.90"]),
    "mixed6k": (("mixed", 6000, 60, 0.06, 72), ["--id", "0.85"]),
    "fam5k": (("family", 5000, 80, 12, 0.10, 0.03, 73), ["--id", "0.90"]),
    "short3k_k3": ((3000, 300, 50, 0.05, 74), ["--id", "0.95", "--kmer", "3"]),
}


@pytest.mark.parametrize("name", sorted(ACC_CASES))
def test_device_accumulate_equals_step_path(eng, name, tmp_path):
    """mc_accumulate (persistent kernel, bvec on the device) and the host-driven mc_scan loop
    (whose bvec is the host restatement) give byte-identical .clstr on inputs larger than the
    reference goldens."""
    import importlib.util
    spec, flags = ACC_CASES[name]
    mg = importlib.util.spec_from_file_location("make_golden", fixtures.golden("make_golden.py"))
    mod = importlib.util.module_from_spec(mg)
    mg.loader.exec_module(mod)
    fa = str(tmp_path / (name + ".fa"))
    mod.make_input(spec, fa)
    outs = []
    for env_steps in (False, True):
        out = tmp_path / ("%s_%d.clstr" % (name, env_steps))
        env = dict(os.environ)
        if env_steps:
            env["MC_ACCUM_STEPS"] = "1"
        r = subprocess.run([M.BIN, fa] + flags + ["--output", str(out), "--quiet"], capture_output=True, text=True,
                           timeout=300, env=env)
        assert r.returncode == 0, r.stderr[-3000:]
        outs.append(out.read_bytes())
    assert outs[0] == outs[1]
