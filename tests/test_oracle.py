"""The CPU oracle (oracle/mc_oracle.c) pinned against the reference's own outputs.

Goldens come from oracle/ref_probe, which links the unmodified reference objects
(tests/golden/make_golden.py).  Everything here is bit-exact: integer histograms, keys,
NW length/identities, and the IEEE-double feature/GLM values compared with ==.
"""
import numpy as np
import pytest

import fixtures
import oracle_lib as O


@pytest.fixture(scope="module", autouse=True)
def _build(built):
    return built


@pytest.mark.parametrize("k", [1, 3, 4, 6])
def test_kmer_hist_edge(k):
    recs = fixtures.edge_records()
    g = np.load(fixtures.golden("edge_hist.npz"))
    for i, r in enumerate(recs):
        codes = np.frombuffer(bytes.fromhex(r["data_hex"]), np.uint8)
        h = O.kmer_hist(codes, r["segments"], k, init=1)
        assert np.array_equal(h, g["k%d" % k][i]), (k, i, r["header"])
        assert int(h.sum()) == int(g["mag%d" % k][i])


def test_nw_golden():
    g = np.load(fixtures.golden("nw.npz"))
    a, b = g["a"].tobytes(), g["b"].tobytes()
    for i in range(len(g["identity"])):
        sa = a[g["a_off"][i]:g["a_off"][i + 1]]
        sb = b[g["b_off"][i]:g["b_off"][i + 1]]
        ident, ln, ids, sc = O.nw(sa, sb)
        assert (ln, ids, sc) == (g["length"][i], g["ids"][i], g["score"][i]), i
        assert ident == g["identity"][i], i


@pytest.fixture(scope="module")
def train_a1k():
    g = np.load(fixtures.golden("train_a1k.npz"))
    man = fixtures.manifest()["e2e"]["a1k"]["generator"]
    recs = fixtures.synth_records(*man)
    k = int(g["k"])
    hists = [O.kmer_hist(c, [[0, L - 1]], k).astype(np.uint8) for _, c, L in recs[:40]]
    return g, recs, hists


def test_features_and_classifier(train_a1k):
    g, recs, hists = train_a1k
    cls = O.classifier_from_golden(g)
    flags = [2, 16, 4, 32, 1024]  # LD, INTERSECTION, MANHATTAN, PEARSON, KULCZYNSKI2
    for row, (i, j) in enumerate(g["pair_ij"]):
        p, q = hists[i], hists[j]
        raw = [O.raw(f, p, q, recs[i][2], recs[j][2]) for f in flags]
        assert raw == list(g["raw"][row]), (i, j)
        # the trained Feature's lookup order picks its singles out of the five
        order = {2: 0, 16: 1, 4: 2, 32: 3, 1024: 4}
        sel = [raw[order[int(f)]] for f in g["lookup"]]
        d, s, c0 = O.classify(cls, sel)
        assert s == g["sums"][row], (i, j)
        assert d == g["decision"][row], (i, j)
        assert c0 == g["combo_vals"][row][0]
        assert O.distance(p, q) == g["distance"][row]


def test_distance_d(train_a1k):
    g, recs, hists = train_a1k
    for m, row in enumerate(g["dist_d"], start=1):
        mean = np.sum([h.astype(np.float64) for h in hists[:m]], axis=0) / float(m)
        got = [O.distance_d(h, mean) for h in hists]
        assert got == list(row), m
