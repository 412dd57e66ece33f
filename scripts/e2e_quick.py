#!/usr/bin/env python3
"""Run bin/meshclust on the named e2e goldens and report byte-identity (quick GPU check).

usage: e2e_quick.py NAME [NAME ...]
exit 0 all identical, 1 a mismatch or error, 3 a run hit its time limit (possible hang)
"""
import gzip
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)
import fixtures  # noqa: E402
import meshclust_amd as M  # noqa: E402


def main():
    td = tempfile.mkdtemp()
    for name in sys.argv[1:]:
        fa, flags = fixtures.e2e_input(name, td)
        out = os.path.join(td, name + ".clstr")
        r = subprocess.run(["timeout", "-k", "5", "90", M.BIN, fa] + flags + ["--output", out, "--quiet"],
                           capture_output=True, text=True)
        same = None
        if r.returncode == 0:
            with gzip.open(fixtures.golden("e2e_%s.clstr.gz" % name), "rb") as f:
                same = open(out, "rb").read() == f.read()
        print(name, "rc", r.returncode, "identical", same, r.stderr[-400:], flush=True)
        if r.returncode in (124, 137):
            sys.exit(3)
        if r.returncode != 0 or not same:
            sys.exit(1)


if __name__ == "__main__":
    main()
