"""The C-ABI boundary: the libraries build for gfx950, load, and export every entry point
include/meshclust_amd.h declares (no compute calls: this runs without a GPU)."""
import ctypes
import os
import re
import subprocess

import pytest

import meshclust_amd as M


@pytest.fixture(scope="module")
def product():
    M.build()
    return M


def declared():
    text = open(M.HEADER).read()
    return sorted(set(re.findall(r"\b(mc_[a-z_0-9]+)\s*\(", text)))


def test_header_declares_api():
    names = declared()
    for n in ("mc_ctx_create", "mc_kmer_build", "mc_distance_keys", "mc_pair_features", "mc_classify_pairs",
              "mc_nw_identity", "mc_scan", "mc_mean_shift"):
        assert n in names


def test_libmcgpu_exports_every_symbol(product):
    out = subprocess.run(["nm", "-D", "--defined-only", M.GPU_LIB], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r" T (mc_[a-z_0-9]+)", out))
    missing = [n for n in declared() if n not in exported]
    assert not missing, missing


def test_libmcgpu_loads_and_has_gfx950_code(product):
    lib = ctypes.CDLL(M.GPU_LIB)
    assert lib.mc_abi_version() == 1
    # the bundled device code object targets gfx950
    import tempfile
    import shutil
    with tempfile.TemporaryDirectory() as td:  # (--offloading extracts the bundles next to its input)
        lib = os.path.join(td, "libmcgpu.so")
        shutil.copyfile(M.GPU_LIB, lib)
        r = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "--offloading", lib],
                           capture_output=True, text=True, cwd=td)
    assert "amdgcn-amd-amdhsa--gfx950" in r.stdout + r.stderr


def test_host_library_and_cli(product):
    out = subprocess.run(["nm", "-D", "--defined-only", M.HOST_LIB], capture_output=True, text=True, check=True).stdout
    for n in ("mcl_parse", "mcl_run", "mcl_run_sharded", "mcl_num_seqs", "mcl_free"):
        assert " T " + n in out
    assert os.access(M.BIN, os.X_OK)
    # the CLI links libmcgpu (the GPU engine), never the oracle
    ldd = subprocess.run(["ldd", M.BIN], capture_output=True, text=True).stdout
    assert "libmcgpu.so" in ldd and "oracle" not in ldd


def test_no_gpu_fails_loudly(product):
    """Without a GPU the engine refuses to run (no silent CPU path)."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(M.MCError):
        M.Engine(0)
