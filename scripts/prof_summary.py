#!/usr/bin/env python3
"""Summaries of scripts/prof_round.sh output for profiles/ (one JSON per configuration).

  kernels   rocprofv3 --stats: per kernel calls, total / average duration
  sq        8 SQ counters per kernel (summed over dispatches and the counter's instances) and
            the derived fractions: VALU issue = SQ_INSTS_VALU x 4 cycles (a 64-lane VALU
            instruction occupies a 16-lane SIMD 4 cycles) over the SIMD-cycles of the kernel's
            duration (1,024 SIMDs at the measured clock); LDS array busy = SQ_LDS_IDX_ACTIVE
            (LDS-array cycles) over the CU-cycles of its duration (256 CUs); bank-conflict share
            = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE (MI355X_MICROARCH.md: extra cycles over all
            LDS-array cycles)
  hbm       FETCH_SIZE (x2 on gfx950, MI355X_MICROARCH.md) + WRITE_SIZE per dispatch

usage: prof_summary.py OUTDIR X [X ...]     (reads gpurun_out/{stats,pmc_sq,fetch,write}_X)
"""
import collections
import csv
import json
import os
import re
import sys

CLOCK_HZ = 2.4e9  # the accumulation controller measured 2.39-2.40 GHz (s_memtime vs s_memrealtime)
SIMDS, CUS = 1024, 256


def kname(s):
    s = s.replace("mcg::(anonymous namespace)::", "").replace("void ", "")
    return re.sub(r"\(.*", "", s)


def stats(d):
    p = os.path.join(d, "run_kernel_stats.csv")
    if not os.path.exists(p):
        return None
    out = {}
    for r in csv.DictReader(open(p)):
        out[kname(r["Name"])] = {"calls": int(r["Calls"]), "total_ms": float(r["TotalDurationNs"]) / 1e6,
                                 "avg_us": float(r["AverageNs"]) / 1e3, "percent": float(r["Percentage"])}
    return out


def counters(d):
    p = os.path.join(d, "run_counter_collection.csv")
    if not os.path.exists(p):
        return None
    val = collections.defaultdict(float)
    disp = collections.defaultdict(set)
    dur = {}
    for r in csv.DictReader(open(p)):
        k = kname(r["Kernel_Name"])
        val[(k, r["Counter_Name"])] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
    tp = os.path.join(d, "run_kernel_trace.csv")
    if os.path.exists(tp):
        for r in csv.DictReader(open(tp)):
            k = kname(r["Kernel_Name"])
            dur[k] = dur.get(k, 0.0) + (float(r["End_Timestamp"]) - float(r["Start_Timestamp"])) / 1e9
    out = {}
    for (k, c), v in val.items():
        e = out.setdefault(k, {"dispatches": len(disp[k]), "duration_s": dur.get(k)})
        e[c] = v
    return out


def derive_sq(e):
    t = e.get("duration_s")
    if not t:
        return
    if "SQ_INSTS_VALU" in e:
        e["valu_issue_frac"] = round(e["SQ_INSTS_VALU"] * 4 / (t * CLOCK_HZ * SIMDS), 4)
    if "SQ_LDS_IDX_ACTIVE" in e:
        e["lds_array_busy_frac"] = round(e["SQ_LDS_IDX_ACTIVE"] / (t * CLOCK_HZ * CUS), 4)
        if e["SQ_LDS_IDX_ACTIVE"]:
            e["lds_bank_conflict_share"] = round(e.get("SQ_LDS_BANK_CONFLICT", 0) / e["SQ_LDS_IDX_ACTIVE"], 4)


def main():
    outdir, names = sys.argv[1], sys.argv[2:]
    for x in names:
        res = {"kernels": stats("gpurun_out/stats_%s" % x)}
        sj = "gpurun_out/stats_%s.json" % x
        if os.path.exists(sj):
            res["run"] = json.load(open(sj))
        sq = counters("gpurun_out/pmc_sq_%s" % x)
        if sq:
            for e in sq.values():
                derive_sq(e)
            res["sq"] = sq
        f, w = counters("gpurun_out/fetch_%s" % x), counters("gpurun_out/write_%s" % x)
        if f or w:
            hbm = {}
            for k in set(f or {}) | set(w or {}):
                fe, we = (f or {}).get(k, {}), (w or {}).get(k, {})
                n = fe.get("dispatches") or we.get("dispatches") or 1
                fb = 2.0 * fe.get("FETCH_SIZE", 0.0) * 1024 / n
                wb = we.get("WRITE_SIZE", 0.0) * 1024 / n
                hbm[k] = {"dispatches": n, "fetch_bytes_corrected_per_dispatch": fb,
                          "write_bytes_per_dispatch": wb, "hbm_bytes_per_dispatch": fb + wb}
            res["hbm"] = hbm
        path = os.path.join(outdir, "config_%s.json" % x)
        json.dump(res, open(path, "w"), indent=1, sort_keys=True)
        print(path)


if __name__ == "__main__":
    main()
