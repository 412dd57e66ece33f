#!/usr/bin/env python3
"""Instructions of one candidate wave's scoring chain in the accumulation workers: compiles
scripts/microbench/score_count.hip (16 chunks of SAD / dot4 + classify_small, the dense
workers' per-candidate work) for gfx950 and counts its VALU / LDS / memory instructions.
bench.py prices the accumulation's step-latency floor with the VALU count."""
import json
import os
import re
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
src = os.path.join(HERE, "microbench", "score_count.hip")
with tempfile.TemporaryDirectory() as td:
    out = os.path.join(td, "s.s")
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "--offload-arch=gfx950", "-std=c++17", "-ffp-contract=off",
                    "--cuda-device-only", "-S", src, "-o", out], check=True)
    lines = open(out).read().split("\n")
body = []
inside = False
for l in lines:
    if re.match(r"^_Z\w*score_one\w*:", l):
        inside = True
        continue
    if inside and l.strip().startswith("s_endpgm"):
        break
    if inside:
        body.append(l.strip())
ins = [l.split()[0] for l in body if l and not l.startswith((";", ".")) and not l.endswith(":")]
cnt = {
    "valu": sum(1 for i in ins if i.startswith("v_")),
    "valu_f64": sum(1 for i in ins if i.startswith("v_") and "f64" in i),
    "sad_dot4": sum(1 for i in ins if i.startswith(("v_sad_u8", "v_dot4"))),
    "salu": sum(1 for i in ins if i.startswith("s_") and not i.startswith(("s_waitcnt", "s_load", "s_cbranch", "s_branch"))),
    "smem": sum(1 for i in ins if i.startswith("s_load")),
    "vmem": sum(1 for i in ins if i.startswith(("global_", "buffer_"))),
    "total": len(ins),
}
cnt["note"] = ("one candidate wave of worker_dense: 16 row chunks (its row loads are LDS reads in the kernel, global "
               "loads here) + 16 centre chunks, 64 v_sad_u8 + 64 v_dot4_u32_u8, classify_small")
json.dump(cnt, sys.stdout, indent=1)
print()
