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

import pytest

import fixtures

ROOT = fixtures.HERE.rsplit(os.sep, 1)[0]
WORKER = os.path.join(fixtures.HERE, "dist", "shard_worker.py")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run_world(name, tmp_path, gpu, world=2, rccl=False, env_extra=None):
    fa, flags = fixtures.e2e_input(name, tmp_path)
    out = str(tmp_path / (name + ".clstr"))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), WORKER]
    cmd += (["--gpu"] if gpu else []) + (["--rccl"] if rccl else []) + [fa, out, "--"] + flags
    env = dict(os.environ, OMP_NUM_THREADS="2", **(env_extra or {}))
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    with gzip.open(fixtures.golden("e2e_%s.clstr.gz" % name), "rb") as f:
        assert open(out, "rb").read() == f.read()
    ranks = [json.load(open(out + ".rank%d.json" % i)) for i in range(world)]
    for rk in ranks:
        assert rk["accum_path"] == "sharded steps x%d" % world, rk["accum_path"]
        # one exchange per get_close step (+ the long-list ones) and one per mean-shift iteration
        assert rk["calls"] >= rk["scan_steps"] > 0 and rk["calls"] == ranks[0]["calls"]
        assert rk["clusters"] == ranks[0]["clusters"]
    return ranks


@pytest.fixture(scope="module")
def cpu_lib(built):
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "harness"], check=True)


@pytest.mark.parametrize("name,world", [("a1k", 2), ("fam2k", 2), ("m2k_id80", 3)])
def test_sharded_gloo_cpu_byte_identical(cpu_lib, name, world, tmp_path):
    _run_world(name, tmp_path, gpu=False, world=world)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["a1k", "fam2k", "m2k_id80", "big2_3k"])
def test_world2_gpu_byte_identical(name, tmp_path):
    _run_world(name, tmp_path, gpu=True)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["a1k", "fam2k"])
def test_rccl_sharded_path_gpu_byte_identical(name, tmp_path):
    _run_world(name, tmp_path, gpu=True, world=1, rccl=True, env_extra={"MC_SHARD_FORCE": "1"})
