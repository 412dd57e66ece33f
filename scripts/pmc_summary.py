#!/usr/bin/env python3
"""Per-kernel PMC summary from rocprofv3 --pmc runs (FETCH_SIZE and WRITE_SIZE in separate
passes, as MI355X_MICROARCH.md's rocprofv3 section prescribes).

FETCH_SIZE/WRITE_SIZE are reported by rocprofv3 in KiB.  On gfx950 FETCH_SIZE counts exactly
half the bytes of a wide (16 B/lane) coalesced streaming read (MI355X_MICROARCH.md, HBM), so
`fetch_bytes_corrected` doubles it; WRITE_SIZE is exact for 16 B/lane stores.

usage: pmc_summary.py FETCH_DIR WRITE_DIR OUT.json
"""
import collections
import csv
import json
import os
import re
import sys


def load(d):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
        name = re.sub(r"\(.*", "", r["Kernel_Name"].replace("mcg::(anonymous namespace)::", "").replace("void ", ""))
        agg[(name, r["Counter_Name"])].append(float(r["Counter_Value"]) * 1024.0)
    return agg


def main():
    fetch, write, out = sys.argv[1:4]
    res = {}
    for src in (load(fetch), load(write)):
        for (k, c), v in src.items():
            e = res.setdefault(k, {"dispatches": len(v)})
            e[c.lower() + "_bytes_per_dispatch"] = sum(v) / len(v)
    for k, e in res.items():
        if "fetch_size_bytes_per_dispatch" in e:
            e["fetch_bytes_corrected"] = 2.0 * e["fetch_size_bytes_per_dispatch"]
            e["hbm_bytes_per_dispatch"] = e["fetch_bytes_corrected"] + e.get("write_size_bytes_per_dispatch", 0.0)
    json.dump(res, open(out, "w"), indent=1, sort_keys=True)
    for k, e in sorted(res.items()):
        print("%-60s %6d  fetch %.3e  write %.3e" % (k, e["dispatches"], e.get("fetch_bytes_corrected", 0),
                                                     e.get("write_size_bytes_per_dispatch", 0)))


if __name__ == "__main__":
    main()
