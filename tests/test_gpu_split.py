"""The device lazy introsort behind Trainer::split (split.hip, mc_split_*) equals libstdc++'s
std::sort -- ties, presorted / reversed inputs, the heapsort fallback at forced depth limits --
at queried positions (tests/native/select_check.cpp, linked against libmcgpu.so)."""
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


@pytest.mark.gpu
def test_device_split_select_matches_std_sort(tmp_path):
    lib = os.path.join(ROOT, "meshclust_amd", "lib")
    exe = str(tmp_path / "select_check")
    subprocess.run(["g++", "-O2", "-std=c++17", os.path.join(HERE, "native", "select_check.cpp"), "-o", exe,
                    "-L" + lib, "-lmcgpu", "-Wl,-rpath," + lib], check=True, timeout=120)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and r.stdout.startswith("OK"), r.stdout + r.stderr
