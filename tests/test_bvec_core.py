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


def test_bvec_begin_bounds_from_histogram(tmp_path):
    """BVec's begin bounds taken from a length histogram equal the sorted lengths at every bin
    start (bvec.cpp:9-24's sort), on random length distributions incl. lengths too large for the
    histogram, and the bins' contents after insert_finalize equal those of the earlier
    restatement."""
    exe = str(tmp_path / "bvec_insert_check")
    subprocess.run(["g++", "-O2", "-std=c++17", os.path.join(HERE, "native", "bvec_insert_check.cpp"),
                    os.path.join(ROOT, "meshclust_amd", "csrc", "host", "bvec.cpp"), "-o", exe], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and r.stdout.rstrip().endswith("OK"), r.stdout[-2000:]
    assert r.stdout.count("digest") == 60
    # the digests of the reference's construction as restated before these changes (a sort for
    # the bounds, a scan of the vectors' sizes per insert: tests/golden/bvec_insert_digests.txt)
    with open(os.path.join(HERE, "golden", "bvec_insert_digests.txt")) as f:
        assert r.stdout == f.read()
