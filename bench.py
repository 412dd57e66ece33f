#!/usr/bin/env python3
"""bench.py -- sequences clustered per second on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[1]): 100,000 synthetic 1 kb
reads, 1,000 templates, 3% per-base mutation, seed 41, --id 0.90 (auto k = 4, 8-bit
histograms).  One "step" = one full clustering of that batch by the GPU pipeline
(K1 histograms -> training: split sort keys, NW labels, GLM -> accumulation scans ->
15 mean-shift + merge iterations), starting from the encoded sequences already resident in
HBM (FASTA parse and the one-time upload are outside the timed region; their cost is
reported separately in "extra").

With --gpus N (torch.distributed, one rank per GPU) every rank clusters its own batch
(seed 41 + rank): replicas, weak scaling; no collective is on the data path.  With --shard the
ranks instead share ONE clustering of the seed-41 batch (meshclust_amd.dist): each runs the
accumulation chain, computes its share of every mean-shift iteration and the ranks all-gather
the new centres over RCCL (strong scaling).

Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec


def ensure_fasta(n, length, templates, mut, seed):
    from meshclust_amd import synth
    d = os.environ.get("MC_BENCH_CACHE", os.path.join(tempfile.gettempdir(), "mc_bench"))
    os.makedirs(d, exist_ok=True)
    path = os.path.join(d, "synth_%d_%d_%d_%g_%d.fa" % (n, length, templates, mut, seed))
    if not os.path.exists(path):
        tmp = path + ".tmp%d" % os.getpid()
        synth.generate(tmp, n, length, templates, mut, seed)
        os.replace(tmp, path)
    return path


def head_fasta(src, n_reads, dst):
    """First n_reads records of a FASTA (a bounded sample of the same workload)."""
    count = 0
    with open(src, "rb") as f, open(dst, "wb") as g:
        for line in f:
            if line.startswith(b">"):
                count += 1
                if count > n_reads:
                    break
            g.write(line)
    return dst


def cpu_baseline(fasta, args, sample_n, threads):
    """The reference itself (oracle/_ref/meshclust, compiled from /root/reference by
    oracle/Makefile) timed on this host on a bounded sample of the workload."""
    ref = os.path.join(ROOT, "oracle", "_ref", "meshclust")
    if not os.path.exists(ref):
        return None
    with tempfile.TemporaryDirectory() as td:
        sample = head_fasta(fasta, sample_n, os.path.join(td, "sample.fa"))
        out = os.path.join(td, "o.clstr")
        t0 = time.perf_counter()
        r = subprocess.run([ref, sample] + args + ["--threads", str(threads), "--output", out],
                           stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, timeout=900)
        dt = time.perf_counter() - t0
    if r.returncode != 0:
        return None
    return {"value": sample_n / dt, "unit": "sequences/s", "cores": threads, "kind": "reference",
            "sample": "first %d reads of the workload, reference meshclust --threads %d, wall %.2f s"
                      % (sample_n, threads, dt)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--n", type=int, default=100000)
    ap.add_argument("--len", type=int, default=1000)
    ap.add_argument("--templates", type=int, default=1000)
    ap.add_argument("--mut", type=float, default=0.03)
    ap.add_argument("--seed", type=int, default=41)
    ap.add_argument("--id", default="0.90")
    ap.add_argument("--cpu-sample", type=int, default=10000)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--stats-out", default=None)
    ap.add_argument("--shard", action="store_true", help="ranks share one clustering (strong scaling)")
    a = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist  # noqa: F811
        dist.init_process_group("gloo", init_method="env://")

    import meshclust_amd as M
    if rank == 0 and not os.path.exists(M.GPU_LIB):
        M.build()
    if dist:
        dist.barrier()
    shard = dist is not None and a.shard
    fasta = ensure_fasta(a.n, a.len, a.templates, a.mut, a.seed + (0 if shard else rank))
    t0 = time.perf_counter()
    ds = M.Dataset([fasta], threads=16)
    parse_s = time.perf_counter() - t0
    eng = M.Engine(local)
    args = ["--id", a.id, "--threads", "16"]
    comm = None
    if shard:
        import torch
        from meshclust_amd.dist import TorchShardComm
        if torch.cuda.is_available():
            torch.cuda.set_device(local)
            comm = TorchShardComm(dist.new_group(backend="nccl"))  # RCCL for the centre exchange
        else:
            comm = TorchShardComm()

    import torch
    if torch.cuda.is_available():
        torch.cuda.set_device(local)  # sync() below must wait on this rank's GPU, not cuda:0
    sync = torch.cuda.synchronize if torch.cuda.is_available() else (lambda: None)

    t0 = time.perf_counter()
    st = ds.run(eng, args, upload=True, comm=comm)  # one-time upload (+ first warm-up pass)
    first_s = time.perf_counter() - t0
    for _ in range(max(0, a.warmup - 1)):
        ds.run(eng, args, upload=False, comm=comm)
    eng.timers(reset=True)

    if dist:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    stats = []
    for _ in range(a.steps):
        stats.append(ds.run(eng, args, upload=False, comm=comm))
    sync()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    tim = eng.timers()
    if dist:
        import torch as _t
        t = _t.tensor([elapsed], dtype=_t.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    if rank != 0:
        eng.close()
        if dist:
            dist.destroy_process_group()
        return
    s0 = stats[-1]
    n_total = a.n * a.steps * (1 if shard else world)
    value = n_total / elapsed
    ms_step = elapsed / a.steps * 1000.0

    # roofline of the dominant kernel family
    fam_ms = {f: v[0] for f, v in tim.items()}
    fam_n = {f: v[1] for f, v in tim.items()}
    B = 4 ** s0["k"]
    width = s0["width"]
    eval_bytes = B * width + 17  # row + length + magnitude + flag per candidate
    scan_evals = sum(s["scan_candidates"] for s in stats)
    dominant = max(fam_ms, key=lambda f: fam_ms[f])
    roof = None
    if fam_n["scan"]:
        per_launch_bytes = scan_evals * eval_bytes / fam_n["scan"]
        avg_s = fam_ms["scan"] / fam_n["scan"] / 1e3
        ach = per_launch_bytes / avg_s / 1e9
        # one launch per clustering = the device-resident accumulation (accum.hip); otherwise
        # one fused scan launch per get_close step (scan.hip)
        device_loop = fam_n["scan"] <= a.steps
        kname = "accum_kernel<unsigned char>" if device_loop else "fused_scan_kernel<unsigned char>"
        roof = {"kernel": ("accum_kernel (whole accumulation phase, %d dependent get_close steps per launch)"
                           % s0["scan_steps"]) if device_loop else "fused_scan_kernel (Trainer::get_close step)",
                "bound": "hbm", "achieved": round(ach, 1),
                "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": None,
                "bytes_per_eval": eval_bytes, "evals_per_launch": round(scan_evals / fam_n["scan"], 1),
                "avg_launch_us": round(avg_s * 1e6, 2),
                "us_per_step": round(fam_ms["scan"] * 1e3 / sum(s["scan_steps"] for s in stats), 2)}
        pmc = os.path.join(ROOT, "profiles", "pmc_latest.json")
        if os.path.exists(pmc):  # rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (scripts/pmc_summary.py)
            e = json.load(open(pmc)).get(kname)
            if e and "hbm_bytes_per_dispatch" in e:
                roof["traffic"] = round(e["hbm_bytes_per_dispatch"])
                roof["traffic_unit"] = "bytes/launch (FETCH_SIZE x2 + WRITE_SIZE, profiles/pmc_latest.json)"
                roof["algorithmic_bytes_per_launch"] = round(per_launch_bytes)
    nw_cells = sum(s["nw_cells"] for s in stats)
    nw_rate = nw_cells / (fam_ms["nw"] / 1e3) if fam_ms["nw"] else None
    cpu = None
    if not a.no_cpu_baseline and world == 1:  # the reference is timed on rank 0 at N = 1 only
        cpu = cpu_baseline(fasta, ["--id", a.id], min(a.cpu_sample, a.n), min(16, os.cpu_count() or 1))
    line = {
        "metric": "sequences clustered/sec (+ NW cell-updates/sec) at 1/2/4/8 MI355X",
        "value": round(value, 1),
        "unit": "sequences/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(ms_step, 2),
        "higher_is_better": True,
        "scaling": "strong" if shard else "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (meshclust_amd.synth: %d reads x %d bp, %d templates, mut %.2f, seed %d+rank)"
                % (a.n, a.len, a.templates, a.mut, a.seed),
        "config": {"workload": "config B: 100k synthetic 1kb reads, --id %s k-mer mean-shift" % a.id,
                   "reads_per_gpu": a.n, "read_len": a.len, "k": s0["k"], "histogram_bits": 8 * width,
                   "parallelism": ("one clustering sharded x%d (centre all-gather over RCCL)" % world) if shard
                   else "replicas x%d" % world},
        "roofline": roof,
        "cpu_baseline": cpu,
        "extra": {"nw_cell_updates_per_s": nw_rate, "clusters": s0["clusters"], "dominant_family": dominant,
                  "device_ms_per_step": {f: round(v / a.steps, 3) for f, v in fam_ms.items()},
                  "launches_per_step": {f: round(v / a.steps, 1) for f, v in fam_n.items()},
                  "host_phases_ms": s0["phases_ms"], "parse_s": round(parse_s, 3),
                  "first_run_incl_upload_s": round(first_s, 3), "scan_steps": s0["scan_steps"]},
    }
    print(json.dumps(line))
    if a.stats_out:
        with open(a.stats_out, "w") as f:
            json.dump({"line": line, "stats": stats, "timers": tim}, f, indent=1)
    eng.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
