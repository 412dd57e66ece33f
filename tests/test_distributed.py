"""The multi-rank path: one clustering shared by two ranks over
torch.distributed (gloo, world size 2, 127.0.0.1).  Each rank runs the accumulation and its
share of every mean-shift iteration, the ranks all-gather the new centres, and rank 0's .clstr
must be byte-identical to the reference golden (i.e. to the one-rank run).

The CPU case drives the product's host code on the CPU oracle engine (test-only); the GPU case
runs two ranks of the product on cuda:0."""
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


def _run_world2(name, tmp_path, gpu):
    fa, flags = fixtures.e2e_input(name, tmp_path)
    out = str(tmp_path / (name + ".clstr"))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), WORKER]
    cmd += (["--gpu"] if gpu else []) + [fa, out, "--"] + flags
    env = dict(os.environ, OMP_NUM_THREADS="2")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    with gzip.open(fixtures.golden("e2e_%s.clstr.gz" % name), "rb") as f:
        assert open(out, "rb").read() == f.read()
    ranks = [json.load(open(out + ".rank%d.json" % i)) for i in range(2)]
    assert ranks[0]["calls"] > 0 and ranks[0]["calls"] == ranks[1]["calls"]  # the exchange ran
    assert ranks[0]["clusters"] == ranks[1]["clusters"]


@pytest.fixture(scope="module")
def cpu_lib(built):
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "harness"], check=True)


@pytest.mark.parametrize("name", ["a1k", "fam2k"])
def test_world2_gloo_cpu_byte_identical(cpu_lib, name, tmp_path):
    _run_world2(name, tmp_path, gpu=False)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["a1k", "fam2k", "m2k_id80"])
def test_world2_gpu_byte_identical(name, tmp_path):
    _run_world2(name, tmp_path, gpu=True)
