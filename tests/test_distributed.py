"""The multi-rank path: one clustering shared by several ranks over
torch.distributed (127.0.0.1).  Every get_close step is split over the ranks by record
(mc_scan_part on each rank's static blocks, one all-gather of the partial results, the same
mc_scan_commit everywhere), every mean-shift iteration by centre (all-gather of the new
centres); rank 0's .clstr must be byte-identical to the reference golden (= the one-rank run).

* CPU: the product's host code on the CPU oracle engine (test-only), gloo, world sizes 2 and 3
  (3 ranks own unequal shares of every window);
* GPU: two ranks of the product on cuda:0 with the gloo exchange, and one rank with libmcgpu's
  RCCL communicator forced through the sharded code path (MC_SHARD_FORCE; RCCL refuses two
  ranks on one GPU, and the test boxes have one)."""
import gzip
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

import fixtures

ROOT = fixtures.HERE.rsplit(os.sep, 1)[0]
WORKER = os.path.join(fixtures.HERE, "dist", "shard_worker.py")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _launch(fa, flags, out, gpu, world, rccl=False, env_extra=None, timeout=600, worker_args=()):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), WORKER]
    cmd += (["--gpu"] if gpu else []) + (["--rccl"] if rccl else []) + list(worker_args) + [fa, out, "--"] + flags
    # (MC_SHARD_ACCUM: split the accumulation over the ranks even where one GPU holds every row
    # resident -- the product replicates it there, cluster.cpp -- so the mailbox path is tested)
    env = dict(os.environ, OMP_NUM_THREADS="2", MC_SHARD_ACCUM="1")
    env.update(env_extra or {})
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    ranks = [json.load(open(out + ".rank%d.json" % i)) for i in range(world)]
    for rk in ranks:
        assert rk["clusters"] == ranks[0]["clusters"]
    return ranks


def _run_world(name, tmp_path, gpu, world=2, rccl=False, env_extra=None, worker_args=()):
    """Rank 0's .clstr against the reference golden.  The GPU ranks run ONE device-resident
    accumulation together (mailbox exchange between their kernels: "device xW"), unless
    MC_SHARD_HOST_STEPS asks for the host-driven sharded steps (one all-gather per step: the
    CPU engine's only form)."""
    fa, flags = fixtures.e2e_input(name, tmp_path)
    out = str(tmp_path / (name + ".clstr"))
    ranks = _launch(fa, flags, out, gpu, world, rccl, env_extra, worker_args=worker_args)
    with gzip.open(fixtures.golden("e2e_%s.clstr.gz" % name), "rb") as f:
        assert open(out, "rb").read() == f.read()
    host_steps = not gpu or "MC_SHARD_HOST_STEPS" in (env_extra or {})
    for rk in ranks:
        assert rk["accum_path"] == ("sharded steps x%d" if host_steps else "device x%d") % world, rk["accum_path"]
        assert rk["calls"] == ranks[0]["calls"]
        if host_steps:  # one exchange per get_close step (+ the long-list ones) and per iteration
            assert rk["calls"] >= rk["scan_steps"] > 0
    return ranks


@pytest.fixture(scope="module")
def cpu_lib(built):
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "harness"], check=True)


@pytest.mark.parametrize("name,world", [("a1k", 2), ("fam2k", 2), ("m2k_id80", 3)])
def test_sharded_gloo_cpu_byte_identical(cpu_lib, name, world, tmp_path):
    _run_world(name, tmp_path, gpu=False, world=world)


def _run_align_world(name, tmp_path, gpu, world):
    """Alignment mode shares the NW alignments of every get_close window over the ranks
    (cluster.cpp align_sharded_step: mc_align_part + identity all-gather + mc_scan_ident):
    rank 0's .clstr equals the reference golden and every rank reports the sharded path."""
    fa, flags = fixtures.e2e_input(name, tmp_path)
    out = str(tmp_path / (name + ".clstr"))
    ranks = _launch(fa, flags, out, gpu, world)
    with gzip.open(fixtures.golden("e2e_%s.clstr.gz" % name), "rb") as f:
        assert open(out, "rb").read() == f.read()
    for rk in ranks:
        assert rk["accum_path"] == "steps (alignment mode, NW sharded x%d)" % world, rk["accum_path"]
        assert rk["calls"] >= rk["scan_steps"] > 0  # one identity exchange per step
    return ranks


@pytest.mark.parametrize("name,world", [("al300", 2), ("al_mix300", 3)])
def test_align_sharded_gloo_cpu_byte_identical(cpu_lib, name, world, tmp_path):
    _run_align_world(name, tmp_path, gpu=False, world=world)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["al300", "al_mix300", "c2k_m15_al55"])
def test_align_sharded_gpu_byte_identical(name, tmp_path):
    """Two ranks on the GPU (each on half of the CUs) share every alignment window's NW."""
    _run_align_world(name, tmp_path, gpu=True, world=2)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["a1k", "fam2k", "m2k_id80", "big2_3k", "s1k_k5"])
def test_world2_gpu_byte_identical(name, tmp_path):
    """Two ranks' kernels on the one GPU of the test box (each takes half of the CUs), the
    step exchange through the shared host-memory mailbox, gloo for the mean-shift all-gather."""
    _run_world(name, tmp_path, gpu=True)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["fam2k", "big2_3k"])
def test_world2_gpu_host_steps_byte_identical(name, tmp_path):
    _run_world(name, tmp_path, gpu=True, env_extra={"MC_SHARD_HOST_STEPS": "1"})


@pytest.mark.gpu
@pytest.mark.parametrize("name,env", [("a1k", {}), ("fam2k", {}), ("fam2k", {"MC_SHARD_HOST_STEPS": "1"})])
def test_rccl_sharded_path_gpu_byte_identical(name, env, tmp_path):
    _run_world(name, tmp_path, gpu=True, world=1, rccl=True, env_extra=dict(env, MC_SHARD_FORCE="1"))


# ---- the sharded paths at the BASELINE sizes --------------------------------------------
sys.path.insert(0, fixtures.GOLDEN)
import make_big_golden as BG  # noqa: E402


def _big_input(name):
    from meshclust_amd import synth
    gen, _ = BG.BIG[name]
    d = os.environ.get("MC_TEST_CACHE", os.path.join("/tmp", "mc_test_cache_%d" % os.getuid()))
    os.makedirs(d, exist_ok=True)
    fa = os.path.join(d, "%s.fa" % name)
    if not os.path.exists(fa):
        synth.generate(fa + ".tmp", *gen)
        os.replace(fa + ".tmp", fa)
    return fa


@pytest.mark.gpu
@pytest.mark.timeout(900)
@pytest.mark.parametrize("world,rccl,env", [(1, True, {"MC_SHARD_FORCE": "1"}),
                                            (1, True, {"MC_SHARD_FORCE": "1", "MC_SHARD_HOST_STEPS": "1"}),
                                            (2, False, {})])
def test_sharded_B100k_equals_reference(world, rccl, env, tmp_path):
    """Config B (100k x 1 kb) through the sharded paths against the reference's partition."""
    g = np.load(fixtures.golden("cfg_B100k.npz"))
    fa = _big_input("B100k")
    out = str(tmp_path / "B100k.clstr")
    ranks = _launch(fa, ["--id", "0.90"], out, True, world, rccl, env, timeout=800)
    want = "sharded steps x%d" if "MC_SHARD_HOST_STEPS" in env else "device x%d"
    assert ranks[0]["accum_path"] == want % world
    assert BG.canonical_digest(BG.clusters_of(out)) == str(g["digest"])


@pytest.mark.gpu
@pytest.mark.timeout(900)
def test_sharded_D100k_equals_reference(tmp_path):
    """Config D's shape (10,000 clusters of 10 reads) at 100k reads: two ranks' kernels sharing
    the accumulation against the reference's partition (cfg_D100k.npz)."""
    g = np.load(fixtures.golden("cfg_D100k.npz"))
    fa = _big_input("D100k")
    out = str(tmp_path / "D100k.clstr")
    ranks = _launch(fa, ["--id", "0.90"], out, True, 2, False, {}, timeout=800)
    assert ranks[0]["accum_path"] == "device x2"
    got = BG.clusters_of(out)
    assert sorted(c for c, _ in got) == [int(x) for x in g["centres"]]
    assert BG.canonical_digest(got) == str(g["digest"])


@pytest.mark.gpu
@pytest.mark.parametrize("world,env", [(1, {"MC_SHARD_FORCE": "1"}), (2, {})])
def test_sharded_E91_equals_reference(world, env, tmp_path):
    """Config E (k = 6, the wide accumulation rows) through the sharded path."""
    import clstr
    from meshclust_amd import synth
    fa = str(tmp_path / "E91.fa")
    synth.write_fasta(fa, synth.families(7, 13, 8000, 12000, 0.05, 0.15, 61))
    out = str(tmp_path / "E91.clstr")
    ranks = _launch(fa, ["--id", "0.80"], out, True, world, world == 1, env)
    assert ranks[0]["accum_path"] == "device x%d" % world
    assert clstr.canonical(out) == clstr.canonical(fixtures.golden("cfg_E91.clstr.gz"))


@pytest.mark.gpu
@pytest.mark.timeout(1200)
def test_sharded_D1M_equals_single_gpu(tmp_path):
    """Config D (1M x 1 kb, 10,000 templates): two ranks' kernels sharing the accumulation
    give the single-GPU device loop's partition and centres (no reference partition exists at
    this size; tests/test_gpu_configs.py pins the device loop against the host-driven steps)."""
    import meshclust_amd as M
    M.build()
    fa = _big_input("D1M")
    one = str(tmp_path / "D1M.one.clstr")
    r = subprocess.run([M.BIN, fa, "--id", "0.90", "--output", one, "--quiet", "--threads", "16"],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    out = str(tmp_path / "D1M.two.clstr")
    ranks = _launch(fa, ["--id", "0.90"], out, True, 2, False, {}, timeout=900)
    assert ranks[0]["accum_path"] == "device x2"
    assert BG.canonical_digest(BG.clusters_of(out)) == BG.canonical_digest(BG.clusters_of(one))


@pytest.mark.gpu
@pytest.mark.timeout(900)
def test_sharded_uneven_grids_B100k_equals_reference(tmp_path):
    """Two ranks on one GPU whose own grids differ (MC_ACCUM_GRID 64 and 256: rank 0 alone would
    take 512-position tiles, rank 1 alone the dense 64-position tiles).  Tile t belongs to rank
    t mod 2, so the ranks must agree on the tile: attach_mailbox gives both the smaller grid and
    compares the plans (cluster.cpp).  The partition must be the reference's."""
    g = np.load(fixtures.golden("cfg_B100k.npz"))
    fa = _big_input("B100k")
    out = str(tmp_path / "B100k.clstr")
    ranks = _launch(fa, ["--id", "0.90"], out, True, 2, False, {}, timeout=800, worker_args=["--grid-per-rank", "64,256"])
    assert ranks[0]["accum_path"] == "device x2"
    assert BG.canonical_digest(BG.clusters_of(out)) == str(g["digest"])


def _bench_line(extra_env, args, timeout=900):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                       timeout=timeout, env={**os.environ, "MC_SHARD_ACCUM": "1", **extra_env})
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    return json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])


@pytest.mark.gpu
@pytest.mark.timeout(900)
def test_bench_two_ranks_one_gpu_D100k(tmp_path):
    """bench.py --gpus 2 spawns its two ranks itself (no launcher), and they share ONE config-D
    clustering; MC_BENCH_ONE_GPU=1 puts both on the box's one GPU.  The line reports two GPUs
    and the partition is the reference's (cfg_D100k: config D's shape at 100k reads)."""
    g = np.load(fixtures.golden("cfg_D100k.npz"))  # (bench.py --workload D --n 100000: the same generator and seed)
    keep = str(tmp_path / "bench_D100k.clstr")
    line = _bench_line({"MC_BENCH_ONE_GPU": "1", "OMP_NUM_THREADS": "4"},
                       ["--gpus", "2", "--workload", "D", "--n", "100000", "--steps", "1", "--warmup", "1",
                        "--no-cpu-baseline", "--keep-clstr", keep])
    assert line["n_gpus"] == 2 and line["config"]["mode"] == "shard" and line["config"]["workload_config"] == "D"
    assert line["extra"]["accum_path"] == "device x2"
    assert line["value"] > 0 and line["steps"] == 1
    got = BG.clusters_of(keep)
    assert sorted(c for c, _ in got) == [int(x) for x in g["centres"]]
    assert BG.canonical_digest(got) == str(g["digest"])


@pytest.mark.gpu
def test_world2_replicated_accumulation_byte_identical(tmp_path):
    """Without MC_SHARD_ACCUM the ranks replicate the accumulation when one GPU holds every row
    resident (here: 3k reads), sharding the training and the mean shift only."""
    fa, flags = fixtures.e2e_input("big2_3k", tmp_path)
    out = str(tmp_path / "big2_3k.clstr")
    ranks = _launch(fa, flags, out, True, 2, False, {"MC_SHARD_ACCUM": ""})
    assert ranks[0]["accum_path"] == "device (replicated x2)", ranks[0]["accum_path"]
    with gzip.open(fixtures.golden("e2e_big2_3k.clstr.gz"), "rb") as f:
        assert open(out, "rb").read() == f.read()


# ---- boxes with two or more GPUs (the driver's multi-GPU node): one rank per GPU ------------
def _gpu_count():
    try:
        import torch
        return torch.cuda.device_count()  # (does not initialise HIP on this image)
    except Exception:
        return 0


multi_gpu = pytest.mark.skipif(_gpu_count() < 2, reason="needs two GPUs")


@pytest.mark.gpu
@multi_gpu
@pytest.mark.parametrize("name", ["a1k", "fam2k", "big2_3k", "s1k_k5"])
def test_rccl_world2_two_gpus_byte_identical(name, tmp_path):
    """Two processes, one GPU each, RCCL over xGMI for the all-gathers and the mailbox between
    two devices' kernels: byte-identical to the reference golden."""
    _run_world(name, tmp_path, gpu=True, world=2, rccl=True, worker_args=["--per-rank-gpu"])


@pytest.mark.gpu
@multi_gpu
@pytest.mark.timeout(900)
def test_rccl_world2_two_gpus_B100k_equals_reference(tmp_path):
    g = np.load(fixtures.golden("cfg_B100k.npz"))
    fa = _big_input("B100k")
    out = str(tmp_path / "B100k.clstr")
    ranks = _launch(fa, ["--id", "0.90"], out, True, 2, True, {}, timeout=800, worker_args=["--per-rank-gpu"])
    assert ranks[0]["accum_path"] == "device x2"
    assert BG.canonical_digest(BG.clusters_of(out)) == str(g["digest"])


@pytest.mark.gpu
@multi_gpu
@pytest.mark.timeout(900)
def test_bench_two_gpus_D100k(tmp_path):
    g = np.load(fixtures.golden("cfg_D100k.npz"))
    keep = str(tmp_path / "bench_D100k.clstr")
    line = _bench_line({"OMP_NUM_THREADS": "4"}, ["--gpus", "2", "--workload", "D", "--n", "100000", "--steps", "1",
                                                  "--warmup", "1", "--no-cpu-baseline", "--keep-clstr", keep])
    assert line["n_gpus"] == 2 and line["extra"]["accum_path"] == "device x2"
    assert BG.canonical_digest(BG.clusters_of(keep)) == str(g["digest"])


# ---- one process, several ranks (bin/meshclust --devices): threads sharing a host exchange ----
HARNESS = os.path.join(ROOT, "oracle", "_build", "meshclust_cpu")


def _cli(binary, name, tmp_path, devices, env_extra=None, timeout=600, shard_accum=True):
    """bin/meshclust --devices.  Ranks that share a GPU run in the product's default environment:
    each rank's context takes a CU partition of its own (mc_ctx_partition: a CU-masked stream,
    a hardware queue per rank) and every rank allocates before any rank launches
    (mc_accum_reserve), so no rank's work waits behind another rank's persistent kernel."""
    fa, flags = fixtures.e2e_input(name, tmp_path)
    out = str(tmp_path / (name + ".clstr"))
    st = out + ".json"
    env = dict(os.environ)
    env.pop("GPU_MAX_HW_QUEUES", None)
    if shard_accum:
        env["MC_SHARD_ACCUM"] = "1"
    env["MC_PHASE_LOG"] = "1"  # (each rank's phases on stderr: a run past its limit shows where it stopped)
    env.update(env_extra or {})
    try:
        r = subprocess.run([binary, fa] + flags + ["--devices", devices, "--output", out, "--stats-json", st, "--quiet",
                            "--threads", "4"], capture_output=True, text=True, timeout=timeout, env=env)
    except subprocess.TimeoutExpired as e:
        err = e.stderr.decode() if isinstance(e.stderr, bytes) else (e.stderr or "")
        pytest.fail("--devices %s on %s still running after %d s; its phases so far:\n%s" % (devices, name, timeout, err[-4000:]))
    return r, out, st


@pytest.mark.parametrize("name", ["a1k", "fam2k"])
def test_devices_threads_cpu_byte_identical(cpu_lib, name, tmp_path):
    """--devices 0,1 on the CPU engine: two threads, the in-process exchange, host-driven
    sharded steps (the CPU engine has no device mailbox)."""
    r, out, st = _cli(HARNESS, name, tmp_path, "0,1")
    assert r.returncode == 0, r.stderr[-3000:]
    assert json.load(open(st))["accum_path"] == "sharded steps x2"
    with gzip.open(fixtures.golden("e2e_%s.clstr.gz" % name), "rb") as f:
        assert open(out, "rb").read() == f.read()


@pytest.mark.parametrize("stage", ["upload", "train", "accumulate", "update"])
def test_devices_threads_fault_stops_every_rank(cpu_lib, stage, tmp_path):
    """A failure on one rank at any stage ends the whole run with an error (no rank left
    waiting in an exchange): MC_FAULT injects it on rank 1."""
    import time
    t0 = time.time()
    r, _, _ = _cli(HARNESS, "a1k", tmp_path, "0,1", {"MC_FAULT": "1:" + stage}, timeout=120)
    assert r.returncode != 0
    assert "injected fault" in r.stderr, r.stderr[-2000:]
    assert time.time() - t0 < 60


def test_devices_threads_align_fault_stops_every_rank(cpu_lib, tmp_path):
    """Alignment mode's sharded NW part (cluster.cpp align_sharded_step): a rank whose part fails
    still joins the identity all-gather with its block marked failed, so both ranks stop."""
    import time
    t0 = time.time()
    r, _, _ = _cli(HARNESS, "al300", tmp_path, "0,1", {"MC_FAULT": "1:align_part"}, timeout=120)
    assert r.returncode != 0
    assert "injected fault" in r.stderr, r.stderr[-2000:]
    assert time.time() - t0 < 60


def test_processes_align_fault_stops_every_rank(cpu_lib, tmp_path):
    """The same with one process per rank (gloo): the run ends promptly with the failing rank's
    error, no rank waits out the exchange timeout."""
    import time
    fa, flags = fixtures.e2e_input("al300", tmp_path)
    out = str(tmp_path / "al300.clstr")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), WORKER, fa, out, "--"] + flags
    t0 = time.time()
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, OMP_NUM_THREADS="2", MC_FAULT="1:align_part", MC_DIST_TIMEOUT_S="120"))
    assert r.returncode != 0
    assert "injected fault" in r.stdout + r.stderr
    assert time.time() - t0 < 100  # (well inside the 120 s exchange timeout: no rank waited it out)


@pytest.mark.parametrize("stage", ["train", "update"])
def test_processes_fault_stops_every_rank(cpu_lib, stage, tmp_path):
    """The same with one process per rank (gloo): the surviving rank's exchange fails or the
    launcher stops it, and the job exits non-zero promptly."""
    import time
    fa, flags = fixtures.e2e_input("a1k", tmp_path)
    out = str(tmp_path / "a1k.clstr")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), WORKER, fa, out, "--"] + flags
    t0 = time.time()
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, OMP_NUM_THREADS="2", MC_FAULT="1:" + stage, MC_DIST_TIMEOUT_S="30"))
    assert r.returncode != 0
    assert time.time() - t0 < 200


@pytest.mark.gpu
@pytest.mark.parametrize("name,devices", [("fam2k", "0"), ("fam2k", "0,0"), ("big2_3k", "0,0"), ("s1k_k5", "0,0"),
                                          pytest.param("fam2k", "0,1", marks=multi_gpu),
                                          pytest.param("big2_3k", "0,1", marks=multi_gpu),
                                          pytest.param("s1k_k5", "0,0,1", marks=multi_gpu)])
def test_devices_cli_gpu_byte_identical(name, devices, tmp_path):
    """bin/meshclust --devices on the product: one GPU, or two ranks (threads, contexts) on the
    test box's one GPU sharing the accumulation through the mailbox (each kernel takes half of
    the CUs)."""
    import meshclust_amd as M
    M.build()
    r, out, st = _cli(M.BIN, name, tmp_path, devices, timeout=150)
    assert r.returncode == 0, r.stderr[-3000:]
    w = len(devices.split(","))
    assert json.load(open(st))["accum_path"] == ("device x%d" % w if w > 1 else "device")
    with gzip.open(fixtures.golden("e2e_%s.clstr.gz" % name), "rb") as f:
        assert open(out, "rb").read() == f.read()


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["fam2k", "big2_3k"])
def test_devices_cli_gpu_default_env_replicated(name, tmp_path):
    """--devices 0,0 with the product's defaults (no MC_SHARD_ACCUM): inputs this small fit one
    rank's CU partition in the dense resident form, so every rank runs the whole accumulation
    chain itself ("device (replicated x2)"), each on its own CUs; the comm timers are in the
    stats."""
    import meshclust_amd as M
    M.build()
    r, out, st = _cli(M.BIN, name, tmp_path, "0,0", shard_accum=False, timeout=150)
    assert r.returncode == 0, r.stderr[-3000:]
    stats = json.load(open(st))
    assert stats["accum_path"] == "device (replicated x2)", stats["accum_path"]
    assert stats["phases_ms"].get("gpu_share") == 2.0
    assert stats["phases_ms"]["comm.train.calls"] >= 1
    # (the update exchanges from its second iteration on; a loop that reached its fixed point in
    # the first, cluster.cpp, exchanged nothing there)
    if 15 - stats["update_iters_fixed"] > 1:
        assert stats["phases_ms"]["comm.update.calls"] >= 1
    with gzip.open(fixtures.golden("e2e_%s.clstr.gz" % name), "rb") as f:
        assert open(out, "rb").read() == f.read()
