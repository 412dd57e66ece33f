#!/usr/bin/env python3
"""profiles/nw_counters.json: the NW roofline inputs bench.py prices its nw_roofline with,
from this round's counter passes and the VALU microbenchmark.

  * per configuration (scripts/prof_round.sh pmc_sq_X + stats_X, summarised by
    scripts/prof_summary.py into PROFDIR/config_X.json): every nw_mw_kernel instance's
    SQ_INSTS_VALU, duration, VALU issue fraction (x 4 cycles per wave64 instruction over the
    SIMD-cycles of its duration), LDS-array busy fraction and bank-conflict share, and the
    configuration's VALU lane-instructions per DP cell (SQ_INSTS_VALU x 64 over the run's cells);
  * the issue rate of the cell update's instruction classes (scripts/microbench/valu_peak,
    gpurun_out/valu_peak.json): v_max_i32 / v_max3_i32 / v_add3_u32 / v_cndmask_b32_e64 ...

usage: nw_counters.py PROFDIR VALU_JSON OUT_JSON
"""
import json
import os
import sys

CLOCK_HZ = 2.4e9
SIMDS = 1024


def main():
    profdir, valu_path, out = sys.argv[1:4]
    valu = json.load(open(valu_path))
    rates = {}
    for r in valu["results"]:
        rates.setdefault(r["inst"], {})[r["waves_per_simd"]] = r["lane_insts_per_s"]
    # the NW kernels run 2 waves per SIMD (throughput form: 250 VGPRs) to 4 (latency form):
    # the cell update is max / compare / select / add, priced at v_max_i32's rate at 2 waves
    peak = rates["v_max_i32"][2]
    res = {"source": "rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_LDS "
                     "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES on bin/meshclust (scripts/prof_round.sh); "
                     "issue rates from scripts/microbench/valu_peak.hip",
           "valu_lane_ops_per_s": peak,
           "valu_peak_note": "v_max_i32 at 2 waves/SIMD, measured (valu_peak): the NW cell update's max / compare / "
                             "select class issues 16 lanes per clock per SIMD; v_add_u32 alone reaches 32",
           "issue_rates_lane_insts_per_s": {k: v for k, v in rates.items()},
           "configs": {}}
    for name, label in (("b", "config B (training: label batch + sampler rounds)"),
                        ("c", "config C20k (--align: window scans)"),
                        ("e", "config E9100 (training: 8-12 kb pairs)")):
        p = os.path.join(profdir, "config_%s.json" % name)
        if not os.path.exists(p):
            continue
        d = json.load(open(p))
        run = d.get("run", {})
        cells = (run.get("nw_cells") or 0) + (run.get("align_nw_cells") or 0)
        ks = {k: v for k, v in (d.get("sq") or {}).items() if k.startswith("nw_mw_kernel")}
        insts = sum(v.get("SQ_INSTS_VALU", 0.0) for v in ks.values())
        dur = sum(v.get("duration_s") or 0.0 for v in ks.values())
        c = {"label": label, "cells": cells, "nw_kernel_s": dur,
             "lane_insts_per_cell": round(insts * 64 / cells, 2) if cells else None,
             "cells_per_s": cells / dur if dur else None, "kernels": {}}
        for k, v in sorted(ks.items()):
            c["kernels"][k] = {f: v.get(f) for f in ("dispatches", "duration_s", "SQ_INSTS_VALU", "SQ_INSTS_LDS",
                                                      "valu_issue_frac", "lds_array_busy_frac",
                                                      "lds_bank_conflict_share", "SQ_WAVES")}
        res["configs"][name] = c
    b = res["configs"].get("b")
    if b and b["lane_insts_per_cell"]:
        res["lane_insts_per_cell"] = b["lane_insts_per_cell"]  # (the bench line's workload)
    json.dump(res, open(out, "w"), indent=1, sort_keys=True)
    print(json.dumps({k: (v["lane_insts_per_cell"], v["cells_per_s"]) for k, v in res["configs"].items()}))


if __name__ == "__main__":
    main()
