"""The closed-form bvec window logic of the device-resident accumulation kernel
(meshclust_amd/csrc/gpu/bvec_core.hpp) equals the host BVec restatement
(meshclust_amd/csrc/host/bvec.cpp: get_range, inner_index_of's binary search, the
bvec_iterator window incl. its error cases) on random length distributions and random
pop / erase / remove_available sequences."""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def test_bvec_core_matches_host_bvec(tmp_path):
    exe = str(tmp_path / "bvec_check")
    subprocess.run(["g++", "-O2", "-std=c++17", os.path.join(HERE, "native", "bvec_check.cpp"),
                    os.path.join(ROOT, "meshclust_amd", "csrc", "host", "bvec.cpp"), "-o", exe], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and r.stdout.startswith("OK"), r.stdout + r.stderr
