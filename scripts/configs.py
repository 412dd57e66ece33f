#!/usr/bin/env python3
"""Time bin/meshclust end to end (parse -> .clstr written) on the BASELINE.json configs that
are not bench.py's line: config C (--align, batched NW), config D on one GPU
(1M reads) and config E (the viral shape, mixed 8-12 kb genomes, k = 6).  One JSON line per run, also written to
gpurun_out/configs_<name>.json.

usage: configs.py NAME [NAME ...]      names: see CONFIGS below
A run that hits its time limit exits 3 (nothing further is started).
"""
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import meshclust_amd as M  # noqa: E402
from meshclust_amd import synth  # noqa: E402

# name -> (generator, flags, time limit s, description)
CONFIGS = {
    "C20k": (("reads", 20000, 1000, 200, 0.03, 41), ["--id", "0.55", "--align"], 600,
             "config C shape at 20k reads (200 templates): --id 0.55 --align"),
    "C100k": (("reads", 100000, 1000, 1000, 0.03, 41), ["--id", "0.55", "--align"], 900,
              "config C: 100k x 1 kb, 1000 templates, mut 0.03, --id 0.55 --align"),
    "C20k_m15": (("reads", 20000, 1000, 200, 0.15, 41), ["--id", "0.55", "--align"], 600,
                 "config C 0.15-mutation variant at 20k reads: --id 0.55 --align"),
    "E91": (("families", 7, 13, 8000, 12000, 0.05, 0.15, 61), ["--id", "0.80"], 300,
            "config E: 7 families x 13 genomes, 8-12 kb, 5-15% within-family mutation, --id 0.80"),
    "E9100": (("families", 70, 130, 8000, 12000, 0.05, 0.15, 61), ["--id", "0.80"], 900,
              "config E scaled: 70 families x 130 genomes, 8-12 kb, --id 0.80"),
    "D1M": (("reads", 1000000, 1000, 10000, 0.03, 51), ["--id", "0.90"], 900,
            "config D on one GPU: 1M x 1 kb, 10,000 templates, mut 0.03, --id 0.90"),
}


def make_input(gen, path):
    if os.path.exists(path):
        return path
    tmp = path + ".tmp%d" % os.getpid()
    if gen[0] == "reads":
        synth.generate(tmp, *gen[1:])
    else:
        synth.write_fasta(tmp, synth.families(*gen[1:]))
    os.replace(tmp, path)
    return path


def run(name, outdir):
    gen, flags, limit, desc = CONFIGS[name]
    d = os.path.join(tempfile.gettempdir(), "mc_cfg")
    os.makedirs(d, exist_ok=True)
    fa = make_input(gen, os.path.join(d, name + ".fa"))
    out = os.path.join(d, name + ".clstr")
    st = os.path.join(d, name + ".stats.json")
    cmd = ["timeout", "-k", "10", str(limit), M.BIN, fa] + flags + [
        "--threads", "16", "--output", out, "--stats-json", st, "--quiet"]
    t0 = time.perf_counter()
    r = subprocess.run(cmd, capture_output=True, text=True)
    wall = time.perf_counter() - t0
    line = {"config": name, "desc": desc, "rc": r.returncode, "wall_s": round(wall, 3)}
    if r.returncode == 0:
        s = json.load(open(st))
        cells = s.get("nw_cells", 0) + s.get("align_nw_cells", 0)
        line.update({"n": s["n"], "k": s["k"], "width": s["width"], "clusters": s["clusters"],
                     "sequences_per_s": round(s["n"] / wall, 1),
                     "nw_pairs": s.get("nw_pairs", 0) + s.get("align_nw_pairs", 0), "nw_cells": cells,
                     "nw_cells_per_s_wall": round(cells / wall, 1), "phases_ms": s.get("phases_ms")})
        if s.get("scan_candidates") and s.get("phases_ms", {}).get("accumulate"):
            # accumulation scan: algorithmic bytes (B*w + 17 per evaluation) over the phase's wall
            evb = (4 ** s["k"]) * s["width"] + 17
            line.update({"scan_evals": s["scan_candidates"], "scan_steps": s.get("scan_steps"),
                         "accum_scan_gbs": round(s["scan_candidates"] * evb / (s["phases_ms"]["accumulate"] / 1e3) / 1e9, 1)})
        g = os.path.join(ROOT, "tests", "golden", "cfg_%s.clstr.gz" % name)
        if os.path.exists(g):  # reference output on the same input: canonical partition
            import clstr
            line["partition_equals_reference"] = clstr.canonical(out) == clstr.canonical(g)
        os.makedirs(outdir, exist_ok=True)
        if s["n"] <= 200000:  # (large outputs are not copied back)
            os.replace(out, os.path.join(outdir, "configs_%s.clstr" % name))
        else:
            os.remove(out)
    else:
        line["stderr"] = r.stderr[-600:]
    print(json.dumps(line), flush=True)
    with open(os.path.join(outdir, "configs_%s.json" % name), "w") as f:
        json.dump(line, f, indent=1)
    return r.returncode


def main():
    outdir = os.path.join(ROOT, "gpurun_out")
    for name in sys.argv[1:]:
        rc = run(name, outdir)
        if rc in (124, 137):
            sys.exit(3)
        if rc != 0:
            sys.exit(1)


if __name__ == "__main__":
    main()
