"""The accumulation workers' divisions by a constant (features.hpp mk_div / pterms_mk, used by
classify_small) are IEEE-exact: tests/native/mk_div_check.cpp compares them with `/`."""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))


def test_mk_div_equals_ieee_division(tmp_path):
    exe = str(tmp_path / "mk_div_check")
    subprocess.run(["g++", "-O2", "-std=c++17", os.path.join(HERE, "native", "mk_div_check.cpp"), "-o", exe],
                   check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and r.stdout.startswith("OK"), r.stdout + r.stderr
