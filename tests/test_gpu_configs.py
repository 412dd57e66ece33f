"""GPU parity at the BASELINE.json sizes: bin/meshclust on MI355X against the reference's own
partitions of the same synthetic inputs.

* config E (viral shape: 7 families x 13 genomes, 8-12 kb, k = 6, --id 0.80) against the
  reference's .clstr (tests/golden/cfg_E91.clstr.gz, canonical partition + centres);
* config B (100k x 1 kb, --id 0.90) against the reference's canonical partition
  (tests/golden/cfg_B100k.npz, written by make_big_golden.py from oracle/_ref/meshclust
  --threads 1), with the accumulation kernel's LDS-bitmap and global-bitmap variants;
* config D (1M x 1 kb, --id 0.90): property checks and device loop == host-driven steps (the
  reference needs hours at this size).

Reference loop: ClusterFactory.cpp:637-761 (accumulate, MS), Trainer.cpp:34-157, 334-365.
The inputs are regenerated here by meshclust_amd.synth (deterministic; SHA-256 checked).
"""
import hashlib
import json
import os
import subprocess
import sys

import numpy as np
import pytest

import clstr
import fixtures
import meshclust_amd as M
from meshclust_amd import synth

pytestmark = pytest.mark.gpu

sys.path.insert(0, fixtures.GOLDEN)
import make_big_golden as BG  # noqa: E402


def _cache_dir():
    d = os.environ.get("MC_TEST_CACHE", os.path.join("/tmp", "mc_test_cache_%d" % os.getuid()))
    os.makedirs(d, exist_ok=True)
    return d


def _run(fa, flags, out, timeout, env=None):
    st = out + ".stats.json"
    r = subprocess.run([M.BIN, fa] + flags + ["--output", out, "--stats-json", st, "--quiet", "--threads", "16"],
                       capture_output=True, text=True, timeout=timeout, env=dict(os.environ, **(env or {})))
    assert r.returncode == 0, r.stderr[-3000:]
    return json.load(open(st))


@pytest.fixture(scope="module")
def product():
    M.build()
    return M.BIN


@pytest.mark.parametrize("env", [{}, {"MC_ACCUM_NARROW": "1"}, {"MC_ACCUM_STEPS": "1"}, {"MC_ACCUM_NO_XFAST": "1"},
                                 {"MC_NW_SPINE": "1"}, {"MC_NW_LOOKAHEAD": "2", "MC_NW_CHAIN_R": "16"}])
def test_config_E91_partition_equals_reference(product, tmp_path, env):
    """k = 6 (4 KiB rows): the accumulation kernel's wide form (default), its lane-per-candidate
    form, the host-driven get_close steps and the controller's general window form (no
    nearest-alive queries for windows with an empty edge bin, MC_ACCUM_NO_XFAST), each against
    the reference's partition; and the sampler's left-spine round forced on (it is off by
    default above a mean length of 4 kb), and its search at two levels per round in chained
    blocks of 16 rows per lane (the short-read defaults; one level and 8 rows above 4 kb)."""
    fa = str(tmp_path / "E91.fa")
    synth.write_fasta(fa, synth.families(7, 13, 8000, 12000, 0.05, 0.15, 61))
    out = str(tmp_path / "E91.clstr")
    st = _run(fa, ["--id", "0.80"], out, 300, env)
    assert st["k"] == 6 and st["n"] == 91
    assert st["accum_path"] == ("device" if "MC_ACCUM_STEPS" not in env else "steps (MC_ACCUM_STEPS)")
    assert clstr.canonical(out) == clstr.canonical(fixtures.golden("cfg_E91.clstr.gz"))


def _input(name):
    gen, _ = BG.BIG[name]
    fa = os.path.join(_cache_dir(), "%s.fa" % name)
    if not os.path.exists(fa):
        BG.make_input(gen, fa + ".tmp")
        os.replace(fa + ".tmp", fa)
    return fa


def _big(name, product, timeout, env=None, tag=""):
    gen, flags = BG.BIG[name]
    gpath = fixtures.golden("cfg_%s.npz" % name)
    if not os.path.exists(gpath):
        pytest.skip("reference partition for %s not generated" % name)
    g = np.load(gpath)
    fa = _input(name)
    out = fa[:-3] + tag + ".clstr"
    st = _run(fa, flags, out, timeout, env)
    got = BG.clusters_of(out)
    assert sorted(c for c, _ in got) == [int(x) for x in g["centres"]], "centre sets differ"
    if "centre_of" in g:
        mine = np.full(int(g["n"]), 0xffffffff, np.uint32)
        for c, mem in got:
            mine[np.array(mem, np.int64)] = c
        diff = int((mine != g["centre_of"]).sum())
        assert diff == 0, "%d reads in a different cluster" % diff
    assert BG.canonical_digest(got) == str(g["digest"])
    assert st["clusters"] == int(g["clusters"])
    return st


def test_config_B100k_partition_equals_reference(product):
    st = _big("B100k", product, 300)
    assert st["accum_path"] == "device"


def test_config_B100k_global_bitmap_equals_reference(product):
    """The accumulation kernel's global-bitmap variant (the one N >~ 900k reads takes, config
    D) forced at config B, against the same reference partition."""
    st = _big("B100k", product, 300, env={"MC_ACCUM_GBITS": "1"}, tag=".gbits")
    assert st["accum_path"] == "device"


@pytest.mark.parametrize("env,tag", [({"MC_ACCUM_DBG": "3"}, ".dbg3"), ({"MC_CLASSIFY_EXACT": "1"}, ".exact"),
                                     ({"MC_CLASSIFY_NO_SMALL": "1"}, ".nosmall"), ({"MC_ACCUM_THIN": "0"}, ".nothin")])
def test_config_B100k_accum_variants_equal_reference(product, env, tag):
    """The accumulation kernel's opt-in forms (per-bin aggregated bvec kills and the
    quad-per-member closest search, MC_ACCUM_DBG=3; every new seed's record published whole,
    MC_ACCUM_THIN=0), the workers' exact classifier
    (MC_CLASSIFY_EXACT: classify_std everywhere, no division-light decision) and the
    division-light decision without the small-magnitude form (MC_CLASSIFY_NO_SMALL:
    classify_fast) at config B, against the reference's partition."""
    st = _big("B100k", product, 300, env=env, tag=tag)
    assert st["accum_path"] == "device"


@pytest.mark.parametrize("env,tag", [({"MC_ACCUM_GRID": "64"}, ".g64"), ({"MC_ACCUM_GRID": "32"}, ".g32"),
                                     ({"MC_ACCUM_GRID": "64", "MC_ACCUM_NO_DSTREAM": "1"}, ".g64chunks"),
                                     ({"MC_ACCUM_GRID": "64", "MC_ACCUM_DRES": "0"}, ".g64nores")])
def test_config_B100k_streaming_forms_equal_reference(product, env, tag):
    """The streaming accumulation forms config D takes on one to four GPUs, forced at config B by a
    small grid (more candidates per worker than one workgroup holds): the dense streaming workers
    (one position-ordered list per worker, rows in HBM, rebuilt as candidates die; each thread's
    first entry also in LDS) at 63 and 31 workers and with every row streamed (MC_ACCUM_DRES=0),
    and the 512-position-chunk streaming form (MC_ACCUM_NO_DSTREAM)."""
    st = _big("B100k", product, 300, env=env, tag=tag)
    assert st["accum_path"] == "device"


@pytest.mark.parametrize("env", [{}, {"MC_ACCUM_STEPS": "1"}, {"MC_ACCUM_GRID": "64"},
                                 {"MC_ACCUM_GRID": "64", "MC_ACCUM_THIN": "0"}])
def test_config_D100k_partition_equals_reference(product, env):
    """Config D's shape (10 reads per template, 10,000 clusters) at 100k reads: the device loop
    and the host-driven steps against the reference's own partition (tests/golden/cfg_D100k.npz,
    oracle/_ref/meshclust --threads 1, 48 min here); the dense streaming workers (grid 64) with
    thin and with whole new-seed records."""
    tag = "".join(".%s%s" % (k[9:].lower(), v) for k, v in sorted(env.items()))
    st = _big("D100k", product, 300, env=env, tag=tag)
    assert st["accum_path"] == ("steps (MC_ACCUM_STEPS)" if "MC_ACCUM_STEPS" in env else "device")


def _partition(path):
    got = BG.clusters_of(path)
    ids = np.concatenate([np.array(m, np.int64) for _, m in got])
    return got, ids


@pytest.mark.timeout(1200)
def test_config_D1M_properties():
    """Config D (1M x 1 kb, 10,000 templates, --id 0.90) on one GPU.  The reference needs hours
    here, so there is no reference partition at this size: every read must be
    in exactly one cluster, every centre a member of its own cluster, and the device-resident
    accumulation (global-bitmap variant) must give the same partition and centres as the
    host-driven get_close steps (ClusterFactory.cpp:637-730), whose exactness the smaller
    reference partitions pin."""
    M.build()
    gen, flags = BG.BIG["D1M"]
    fa = _input("D1M")
    out_dev, out_steps = fa[:-3] + ".dev.clstr", fa[:-3] + ".steps.clstr"
    st = _run(fa, flags, out_dev, 600)
    assert st["accum_path"] == "device", st["accum_path"]
    got, ids = _partition(out_dev)
    assert len(ids) == gen[0] and np.array_equal(np.sort(ids), np.arange(gen[0]))
    centres = [c for c, _ in got if c is not None]
    assert len(set(centres)) == len(centres)
    assert all(c in m for c, m in got if c is not None)
    assert st["clusters"] == len(got)
    print("config D: %d clusters (%d without their centre as a member), phases %s"
          % (len(got), len(got) - len(centres), json.dumps(st.get("phases_ms"))))
    st2 = _run(fa, flags, out_steps, 900, env={"MC_ACCUM_STEPS": "1"})
    got2, _ = _partition(out_steps)
    assert BG.canonical_digest(got2) == BG.canonical_digest(got)
    # the 512-position-chunk streaming form (the dense streaming workers are the default here)
    out_chk = fa[:-3] + ".chunks.clstr"
    st4 = _run(fa, flags, out_chk, 600, env={"MC_ACCUM_NO_DSTREAM": "1"})
    assert st4["accum_path"] == "device", st4["accum_path"]
    got4, _ = _partition(out_chk)
    assert BG.canonical_digest(got4) == BG.canonical_digest(got)
    # the streaming form's opt-in per-chunk compaction of alive rows (MC_ACCUM_COMPACT)
    out_cmp = fa[:-3] + ".compact.clstr"
    st3 = _run(fa, flags, out_cmp, 600, env={"MC_ACCUM_COMPACT": "1"})
    assert st3["accum_path"] == "device", st3["accum_path"]
    got3, _ = _partition(out_cmp)
    assert BG.canonical_digest(got3) == BG.canonical_digest(got)


def _properties(path, n):
    """Every read in exactly one cluster, every centre one of its own cluster's members."""
    got, ids = _partition(path)
    assert len(ids) == n and np.array_equal(np.sort(ids), np.arange(n))
    centres = [c for c, _ in got]
    assert None not in centres and len(set(centres)) == len(centres)
    assert all(c in m for c, m in got)
    return got


def _families_input(name, *gen):
    fa = os.path.join(_cache_dir(), "%s.fa" % name)
    if not os.path.exists(fa):
        synth.write_fasta(fa + ".tmp", synth.families(*gen))
        os.replace(fa + ".tmp", fa)
    return fa


@pytest.mark.timeout(900)
def test_config_E9100_properties(product):
    """Config E scaled (70 families x 130 genomes, 8-12 kb, k = 6, --id 0.80: the input that
    gives 8 GPUs work): the reference's partition (tests/golden/cfg_E9100.npz, when generated),
    a partition with member centres, and identical across the accumulation
    kernel's wide form, its lane-per-candidate form (MC_ACCUM_NARROW), the host-driven get_close
    steps, the controller's general window form (MC_ACCUM_NO_XFAST), and the NW kernels' forms (every batch in the throughput form / in the 8-wave latency
    form).  E91 pins these forms against the reference (test_config_E91_partition_equals_reference)."""
    fa = _families_input("E9100", 70, 130, 8000, 12000, 0.05, 0.15, 61)
    base = fa[:-3] + ".clstr"
    st = _run(fa, ["--id", "0.80"], base, 600)
    assert st["k"] == 6 and st["n"] == 9100 and st["accum_path"] == "device"
    want = BG.canonical_digest(_properties(base, 9100))
    gpath = fixtures.golden("cfg_E9100.npz")
    if os.path.exists(gpath):  # the reference's own partition (tests/golden/make_big_golden.py E9100)
        g = np.load(gpath)
        got = BG.clusters_of(base)
        assert sorted(c for c, _ in got) == [int(x) for x in g["centres"]], "centre sets differ"
        assert want == str(g["digest"])
    for tag, env in (("narrow", {"MC_ACCUM_NARROW": "1"}), ("steps", {"MC_ACCUM_STEPS": "1"}),
                     ("noxfast", {"MC_ACCUM_NO_XFAST": "1"}),
                     ("nwtp", {"MC_NW_MW_MAX": "0"}), ("nw8", {"MC_NW_MW_MAX": "100000000", "MC_NW_WAVES": "8"})):
        out = fa[:-3] + "." + tag + ".clstr"
        _run(fa, ["--id", "0.80"], out, 600, env)
        assert BG.canonical_digest(_properties(out, 9100)) == want, tag


@pytest.mark.timeout(900)
def test_config_C20k_align_properties(product):
    """Config C's shape at 20k reads (200 templates, --id 0.55 --align: one NW alignment per centre
    x candidate through the memo replay).  The reference needs days at 100k; its
    partitions at 2k reads of this shape are the e2e_c2k goldens.  Here: a partition with member
    centres, identical whether every NW batch runs in the one-wave throughput form
    (MC_NW_MW_MAX=0), in the 4-wave or the 8-wave latency form."""
    gen = (20000, 1000, 200, 0.03, 41)
    fa = os.path.join(_cache_dir(), "C20k.fa")
    if not os.path.exists(fa):
        synth.generate(fa + ".tmp", *gen)
        os.replace(fa + ".tmp", fa)
    flags = ["--id", "0.55", "--align"]
    base = fa[:-3] + ".clstr"
    st = _run(fa, flags, base, 600)
    assert st["accum_path"] == "steps (alignment mode)" and st["align_nw_pairs"] > 0
    want = BG.canonical_digest(_properties(base, gen[0]))
    for tag, env in (("tp", {"MC_NW_MW_MAX": "0"}), ("w4", {"MC_NW_MW_MAX": "100000000", "MC_NW_WAVES": "4"}),
                     ("w8", {"MC_NW_MW_MAX": "100000000", "MC_NW_WAVES": "8"})):
        out = fa[:-3] + "." + tag + ".clstr"
        _run(fa, flags, out, 600, env)
        assert BG.canonical_digest(_properties(out, gen[0])) == want, tag


@pytest.mark.timeout(1200)
def test_config_C100k_align_properties(product):
    """Config C at its BASELINE size (100k x 1 kb, 1,000 templates, --id 0.55 --align; the
    reference would need days on the CPU): every read in exactly one cluster,
    every centre a member of its cluster, and the same canonical partition whether the
    window scans' NW batches run in the one-wave throughput form (MC_NW_MW_MAX=0) or in the
    default mix of throughput and latency forms."""
    gen = (100000, 1000, 1000, 0.03, 41)
    fa = os.path.join(_cache_dir(), "C100k.fa")
    if not os.path.exists(fa):
        synth.generate(fa + ".tmp", *gen)
        os.replace(fa + ".tmp", fa)
    flags = ["--id", "0.55", "--align"]
    base = fa[:-3] + ".clstr"
    st = _run(fa, flags, base, 900)
    assert st["accum_path"] == "steps (alignment mode)" and st["align_nw_pairs"] > 0
    want = BG.canonical_digest(_properties(base, gen[0]))
    out = fa[:-3] + ".tp.clstr"
    _run(fa, flags, out, 900, {"MC_NW_MW_MAX": "0"})
    assert BG.canonical_digest(_properties(out, gen[0])) == want
