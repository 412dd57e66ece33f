"""GPU paths that the BASELINE configurations do not reach, each against an independent check.

* 32/64-bit histograms (Runner.cpp:75-89 picks them when a k-mer count exceeds 65,535):
  the raw features of Feature.cpp:117-339 at those widths, including the pearson trap of
  Feature.cpp:273-294 (for 32-bit T, p - ap is computed in unsigned 32-bit arithmetic and only
  then widened), against the C oracle; and the whole CLI with the histogram width forced
  (MC_FORCE_WIDTH): the device-resident accumulation does not take 32/64-bit rows
  (MC_ERR_UNSUPPORTED), so the host-driven get_close steps run, and their .clstr must equal the
  one the same host code produces on the CPU oracle engine (oracle/_build/meshclust_cpu).
* clusters of 1,500 members (tests/golden e2e_big2_3k, the reference's own output): past
  the accumulation kernel's LDS member cache, both loops byte-identical to the reference.
"""
import gzip
import json
import os
import subprocess

import numpy as np
import pytest

import fixtures
import meshclust_amd as M
import oracle_lib as O

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(fixtures.HERE)
HARNESS = os.path.join(ROOT, "oracle", "_build", "meshclust_cpu")


@pytest.fixture(scope="module")
def eng():
    M.build()
    e = M.Engine(0)
    yield e
    e.close()


@pytest.mark.parametrize("width,dt", [(4, np.uint32), (8, np.uint64)])
def test_wide_histogram_features_vs_oracle(eng, width, dt):
    rng = np.random.default_rng(21 + width)
    recs = []
    for i in range(48):
        L = int(rng.integers(200, 1500))
        c = rng.integers(0, 2 if i % 4 == 0 else 4, size=L).astype(np.uint8)  # some low-complexity rows
        recs.append((c, [[0, L - 1]]))
    codes = np.concatenate([c for c, _ in recs])
    seq_off = np.cumsum([0] + [len(c) for c, _ in recs]).astype(np.uint64)
    seg = np.array([x for _, s in recs for pair in s for x in pair], np.int32)
    seg_off = np.arange(len(recs) + 1, dtype=np.uint64)
    eng.load_sequences(codes, seq_off, seg, seg_off)
    k = 3
    eng.kmer_max(k)
    eng.kmer_build(k, width)
    h, _ = eng.histograms()
    assert h.dtype == dt
    a = rng.integers(0, len(recs), 200).astype(np.uint32)
    b = rng.integers(0, len(recs), 200).astype(np.uint32)
    flags = [M.FEAT_LD, M.FEAT_INTERSECTION, M.FEAT_MANHATTAN, M.FEAT_PEARSON, M.FEAT_KULCZYNSKI2]
    raw = eng.pair_features(a, b, flags)
    lens = np.diff(seq_off)
    traps = 0
    for i in range(len(a)):
        for f, flag in enumerate(flags):
            want = O.raw(flag, h[a[i]], h[b[i]], int(lens[a[i]]), int(lens[b[i]]))
            assert raw[i, f] == want or (np.isnan(raw[i, f]) and np.isnan(want)), (i, flag)
        if width == 4:  # a bin below the rounded mean: the unsigned 32-bit wrap of Feature.cpp:281
            ap = int(round(int(h[a[i]].astype(np.uint64).sum()) / h.shape[1]))
            traps += int((h[a[i]].astype(np.int64) < ap).any())
    assert width == 8 or traps > 0


def _harness_run(fa, flags, out, env):
    r = subprocess.run([HARNESS, fa] + flags + ["--output", out, "--quiet"], capture_output=True, text=True,
                       timeout=900, env=env)
    assert r.returncode == 0, r.stderr[-2000:]


@pytest.mark.timeout(900)
@pytest.mark.parametrize("width", [4, 8])
def test_forced_wide_histograms_cli_equals_cpu_engine(eng, tmp_path, width):
    if not os.path.exists(HARNESS):
        pytest.skip("oracle harness not built")
    fa, flags = fixtures.e2e_input("a1k", tmp_path)
    env = dict(os.environ, MC_FORCE_WIDTH=str(width))
    out_gpu = str(tmp_path / "gpu.clstr")
    st = str(tmp_path / "st.json")
    r = subprocess.run([M.BIN, fa] + flags + ["--output", out_gpu, "--stats-json", st, "--quiet"], capture_output=True,
                       text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    stats = json.load(open(st))
    assert stats["width"] == width
    assert stats["accum_path"].startswith("steps"), stats["accum_path"]  # MC_ERR_UNSUPPORTED -> get_close steps
    out_cpu = str(tmp_path / "cpu.clstr")
    _harness_run(fa, flags, out_cpu, env)
    assert open(out_gpu, "rb").read() == open(out_cpu, "rb").read()


@pytest.mark.parametrize("steps", [False, True])
def test_clusters_past_member_cache_equal_reference(eng, tmp_path, steps):
    if "big2_3k" not in fixtures.manifest()["e2e"]:
        pytest.skip("golden not generated")
    fa, flags = fixtures.e2e_input("big2_3k", tmp_path)
    out = str(tmp_path / "o.clstr")
    env = dict(os.environ)
    if steps:
        env["MC_ACCUM_STEPS"] = "1"
    r = subprocess.run([M.BIN, fa] + flags + ["--output", out, "--quiet"], capture_output=True, text=True, timeout=600,
                       env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    with gzip.open(fixtures.golden("e2e_big2_3k.clstr.gz"), "rb") as f:
        assert open(out, "rb").read() == f.read()


# The accumulation kernel's row variants (accum.hip): rows of >= 512 bytes take the wide form
# (a wave per candidate, NW-candidate tiles, column sums and closest member from the row-major
# copy); MC_ACCUM_NARROW keeps the lane-per-candidate form.  k = 5 at 8 bits (1 KiB rows) and
# k = 4 forced to 16 bits (512-byte rows: the same feature values as the reference's 8-bit
# ones, so the same output) against the reference's own .clstr; big2_3k's 1,500-member
# clusters flag more than the controller's 1,024-entry step list in one step.
@pytest.mark.parametrize("name,env,wide", [("s1k_k5", {}, True), ("s1k_k5", {"MC_ACCUM_NARROW": "1"}, False),
                                           ("big2_3k", {"MC_FORCE_WIDTH": "2"}, True),
                                           ("fam2k", {"MC_FORCE_WIDTH": "2"}, True),
                                           ("fam2k", {"MC_FORCE_WIDTH": "2", "MC_ACCUM_NARROW": "1"}, False)])
def test_accum_row_variants_equal_reference(eng, tmp_path, name, env, wide):
    fa, flags = fixtures.e2e_input(name, tmp_path)
    out = str(tmp_path / "o.clstr")
    st = str(tmp_path / "st.json")
    r = subprocess.run([M.BIN, fa] + flags + ["--output", out, "--stats-json", st, "--quiet"], capture_output=True,
                       text=True, timeout=600, env=dict(os.environ, MC_ACCUM_PROFILE="1", **env))
    assert r.returncode == 0, r.stderr[-3000:]
    assert json.load(open(st))["accum_path"] == "device"
    assert ("wide %d" % int(wide)) in r.stderr
    with gzip.open(fixtures.golden("e2e_%s.clstr.gz" % name), "rb") as f:
        assert open(out, "rb").read() == f.read()
