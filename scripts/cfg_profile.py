#!/usr/bin/env python3
"""Run bin/meshclust on one scripts/configs.py input with extra environment (e.g.
MC_ACCUM_PROFILE=1) and keep its stderr: the accumulation kernel's phase profile for configs
other than bench.py's.   usage: cfg_profile.py NAME [VAR=VALUE ...]"""
import os
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import configs as C  # noqa: E402


def main():
    name = sys.argv[1]
    env = dict(os.environ)
    for kv in sys.argv[2:]:
        k, v = kv.split("=", 1)
        env[k] = v
    gen, flags, limit, _ = C.CONFIGS[name]
    d = os.path.join(tempfile.gettempdir(), "mc_cfg")
    os.makedirs(d, exist_ok=True)
    fa = C.make_input(gen, os.path.join(d, name + ".fa"))
    cmd = ["timeout", "-k", "10", str(limit), C.M.BIN, fa] + flags + ["--threads", "16", "--output",
                                                                      os.path.join(d, name + ".prof.clstr")]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True)
    out = os.path.join(C.ROOT, "gpurun_out", "cfg_profile_%s.log" % name)
    with open(out, "w") as f:
        f.write(r.stderr)
    print("\n".join(l for l in r.stderr.splitlines() if l.startswith("[accum")))
    sys.exit(r.returncode)


if __name__ == "__main__":
    main()
