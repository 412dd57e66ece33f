"""LazyIntroSort (meshclust_amd/csrc/host/lazysort.hpp) reproduces libstdc++'s std::sort
permutation -- including the order among equal keys and the heapsort fallback -- at every
position.  The check program compiles against the same libstdc++ the host build uses and
compares with std::sort and with std::__introsort_loop at forced depth limits."""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))


def test_lazy_introsort_matches_std_sort(tmp_path):
    exe = str(tmp_path / "lazysort_check")
    subprocess.run(["g++", "-O2", "-fopenmp", "-std=c++17", os.path.join(HERE, "native", "lazysort_check.cpp"), "-o", exe],
                   check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and r.stdout.startswith("OK"), r.stdout + r.stderr
