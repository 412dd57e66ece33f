"""Host restatement of the reference control flow, checked end to end on the CPU.

bin/meshclust's host objects are linked against the CPU oracle engine (oracle/_build/
meshclust_cpu; test-only) and must reproduce the reference's --threads 1 .clstr byte for
byte on every e2e golden.  The GPU run of the real product is checked against the same
goldens in test_gpu_parity.py.
"""
import gzip
import os
import subprocess

import pytest

import fixtures

ROOT = fixtures.HERE.rsplit(os.sep, 1)[0]
HARNESS = os.path.join(ROOT, "oracle", "_build", "meshclust_cpu")
NAMES = sorted(fixtures.manifest()["e2e"])


@pytest.fixture(scope="module")
def harness(built):
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "harness"], check=True)
    return HARNESS


@pytest.mark.parametrize("name", NAMES)
def test_e2e_byte_identical(harness, name, tmp_path):
    fa, flags = fixtures.e2e_input(name, tmp_path)
    out = tmp_path / (name + ".clstr")
    r = subprocess.run([harness, fa] + flags + ["--output", str(out), "--quiet"],
                       capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-2000:]
    with gzip.open(fixtures.golden("e2e_%s.clstr.gz" % name), "rb") as f:
        want = f.read()
    assert out.read_bytes() == want


@pytest.mark.parametrize("env", [{"MC_NW_LOOKAHEAD": "1"}, {"MC_NW_LOOKAHEAD": "3"}, {"MC_NW_SPINE": "0"},
                                 {"MC_NW_SPINE": "0", "MC_NW_LOOKAHEAD": "1"}, {"MC_NW_SPINE_LEVELS": "3"}],
                         ids=["look1", "look3", "nospine", "nospine_look1", "spine3"])
@pytest.mark.parametrize("name", ["a1k", "m2k_id80", "fam2k_id85"])
def test_e2e_nw_lookahead_depth(harness, name, env, tmp_path):
    """Trainer::split's binary search aligns, in its first round, every chain's left spine (the
    pivots visited while the identities stay below the cutoff, its first 2,048 / chains levels or
    MC_NW_SPINE_LEVELS; MC_NW_SPINE=0: off), then
    MC_NW_LOOKAHEAD levels of every chain's decision tree per dependent round (default 2; 1 for
    reads averaging above 4 kb).  One
    level per round without the spine is the reference's order; every form gives the same
    pivots, so the same .clstr (Trainer.cpp:703-721)."""
    fa, flags = fixtures.e2e_input(name, tmp_path)
    out = tmp_path / (name + ".clstr")
    r = subprocess.run([harness, fa] + flags + ["--output", str(out), "--quiet"], capture_output=True, text=True,
                       timeout=900, env=dict(os.environ, **env))
    assert r.returncode == 0, r.stderr[-2000:]
    with gzip.open(fixtures.golden("e2e_%s.clstr.gz" % name), "rb") as f:
        assert out.read_bytes() == f.read()


@pytest.mark.parametrize("name", ["fam2k", "noisy2k", "m2k_id80", "b3k300", "al300", "c2k_al55"])
def test_update_stops_at_fixed_point(harness, name, tmp_path):
    """The update loop (ClusterFactory.cpp:737-752) ends at a fixed point -- no centre moved and
    nothing merged, so every remaining iteration would find the same state -- and counts the
    iterations it leaves out: the .clstr (pinned to the reference above) and the evaluation
    counts equal a run of every iteration (MC_UPDATE_ALL_ITERATIONS=1)."""
    import json
    fa, flags = fixtures.e2e_input(name, tmp_path)
    got = {}
    for mode in ("fixed", "all"):
        env = dict(os.environ)
        env.pop("MC_UPDATE_ALL_ITERATIONS", None)
        if mode == "all":
            env["MC_UPDATE_ALL_ITERATIONS"] = "1"
        out, js = tmp_path / (mode + ".clstr"), tmp_path / (mode + ".json")
        r = subprocess.run([harness, fa] + flags + ["--output", str(out), "--stats-json", str(js), "--quiet"],
                           capture_output=True, text=True, timeout=900, env=env)
        assert r.returncode == 0, r.stderr[-2000:]
        got[mode] = (out.read_bytes(), json.load(open(js)))
    assert got["fixed"][0] == got["all"][0]
    for k in ("update_evals", "merge_evals", "clusters", "align_nw_pairs", "align_nw_cells"):
        assert got["fixed"][1][k] == got["all"][1][k], k
    assert got["all"][1]["update_iters_fixed"] == 0
    if not name.startswith(("al", "c2k")):  # (these k-mer inputs settle early; al300 never does)
        assert got["fixed"][1]["update_iters_fixed"] > 0
