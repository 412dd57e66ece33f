#!/usr/bin/env python3
"""One config-B step's kernel timeline from a rocprofv3 --kernel-trace CSV (scripts/trace_b.sh):
the span from the end of one accumulation kernel to the end of the next, every kernel with the
GPU-idle gap before it, and the idle gaps summed per phase (the gap is charged to the kernel
that follows it).   usage: step_timeline.py KERNEL_TRACE.csv OUT.json"""
import collections
import csv
import json
import re
import sys


def short(name):
    n = name.replace("mcg::(anonymous namespace)::", "").replace("mcg::", "").replace("void ", "")
    return re.sub(r"\(.*", "", n)[:80]


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    ends = [i for i, r in enumerate(rows) if "accum_kernel" in r["Kernel_Name"]]
    if len(ends) < 2:
        sys.exit("need two accumulation kernels in the trace")
    a, b = ends[-2], ends[-1]
    t0 = int(rows[a]["End_Timestamp"])
    ks, idle, last = [], 0.0, t0
    per = collections.defaultdict(float)
    for r in rows[a + 1:b + 1]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = max(0, s - last) / 1e3
        idle += gap
        per[short(r["Kernel_Name"])] += gap
        ks.append({"t_us": round((s - t0) / 1e3, 1), "gap_before_us": round(gap, 1), "dur_us": round((e - s) / 1e3, 1),
                   "kernel": short(r["Kernel_Name"])})
        last = max(last, e)
    out = {"note": "one timed config-B step (accumulation end to the next accumulation end) under rocprofv3 "
                   "--kernel-trace, scripts/trace_b.sh + scripts/step_timeline.py",
           "gpu_idle_us": round(idle, 1), "span_us": round((last - t0) / 1e3, 1),
           "idle_before_us": {k: round(v, 1) for k, v in sorted(per.items(), key=lambda kv: -kv[1]) if v >= 50},
           "kernels": ks}
    json.dump(out, open(sys.argv[2], "w"), indent=1)
    print("span %.1f us, GPU idle %.1f us" % (out["span_us"], out["gpu_idle_us"]))
    for k, v in list(out["idle_before_us"].items())[:12]:
        print("  idle before %-60s %8.1f us" % (k, v))


if __name__ == "__main__":
    main()
