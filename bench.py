#!/usr/bin/env python3
"""bench.py -- sequences clustered per second on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[1]): 100,000 synthetic 1 kb
reads, 1,000 templates, 3% per-base mutation, seed 41, --id 0.90 (auto k = 4, 8-bit
histograms).  One "step" = one end-to-end run of meshclust on that FASTA, the BASELINE
metric's unit of work (N / wall from parse to .clstr written): parse +
encode + 2-bit pack on the host, upload, K1 histograms -> training (split sort keys, NW
labels, GLM) -> accumulation -> 15 mean-shift + merge iterations on the GPU, .clstr written.
The FASTA is read from the page cache (the file is generated before the timed region).  The
rate on sequences already resident in HBM (no parse / upload / write) is reported in
"extra" as resident_sequences_per_s.

With --gpus N > 1 (torch.distributed, one rank per GPU) the ranks share ONE clustering of
BASELINE.json configs[3] (config D: 1,000,000 reads x 1 kb, 10,000 templates, seed 51,
--id 0.90), sharded by record (strong scaling): every rank's persistent accumulation kernel
scans only its interleaved tiles of each get_close window and the kernels exchange each step's
{first maximum, flagged reads} through a host-memory mailbox they all map (no host round trip
per step); every mean-shift iteration is split by centre and the new centres all-gathered over
RCCL.  --mode replicas instead gives every rank its own config-B batch (seed 41 + rank: weak
scaling, no collective on the data path); --mode shard at N = 1 runs the sharded code path on
one rank.

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


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def host_threads():
    """Cores this process may use: the affinity mask, capped by OMP_NUM_THREADS when the
    environment sets it (the GPU box grants 16 cores per GPU and sets it to 16)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    env = os.environ.get("OMP_NUM_THREADS")
    return max(1, min(n, int(env))) if env and env.isdigit() else n


def cpu_baseline(fasta, args, n_reads, threads, repeats, limit_s=600):
    """The reference itself (oracle/_ref/meshclust, compiled from /root/reference by
    oracle/Makefile) on the same FASTA on this host's cores, end to end (process start to
    .clstr written), median of `repeats` runs."""
    ref = os.path.join(ROOT, "oracle", "_ref", "meshclust")
    if not os.path.exists(ref):
        return None
    walls = []
    with tempfile.TemporaryDirectory() as td:
        for i in range(repeats):
            out = os.path.join(td, "o%d.clstr" % i)  # (a new file per run, as the GPU steps)
            t0 = time.perf_counter()
            try:
                r = subprocess.run([ref, fasta] + args + ["--threads", str(threads), "--output", out],
                                   stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, timeout=limit_s)
            except subprocess.TimeoutExpired:
                return None
            if r.returncode != 0:
                return None
            walls.append(time.perf_counter() - t0)
    walls.sort()
    dt = walls[len(walls) // 2]
    return {"value": round(n_reads / dt, 1), "unit": "sequences/s", "cores": threads, "kind": "reference",
            "sample": "the full workload (%d reads, the same FASTA), reference meshclust %s --threads %d, "
                      "wall %s s (median of %d), parse to .clstr written"
                      % (n_reads, " ".join(args), threads, "/".join("%.2f" % w for w in walls), len(walls)),
            "cpu_model": cpu_model(), "host_cpus": os.cpu_count(), "threads": threads}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--mode", choices=["auto", "shard", "replicas"], default="auto",
                    help="auto: one GPU -> config B, several -> config D shared by the ranks")
    ap.add_argument("--n", type=int, default=None)
    ap.add_argument("--len", type=int, default=1000)
    ap.add_argument("--templates", type=int, default=None)
    ap.add_argument("--mut", type=float, default=0.03)
    ap.add_argument("--seed", type=int, default=None)
    ap.add_argument("--id", default="0.90")
    ap.add_argument("--cpu-repeats", type=int, default=3, help="reference runs (median)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--stats-out", default=None)
    a = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    shard = a.mode == "shard" or (a.mode == "auto" and world > 1)
    cfg_d = shard and a.n is None  # the sharded workload: config D unless a size is given
    a.n = a.n if a.n is not None else (1000000 if cfg_d else 100000)
    a.templates = a.templates if a.templates is not None else (10000 if cfg_d else 1000)
    a.seed = a.seed if a.seed is not None else (51 if cfg_d else 41)
    dist = None
    if world > 1 or shard:
        import torch.distributed as dist  # noqa: F811
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29517")
        dist.init_process_group("gloo", init_method="env://", rank=rank, world_size=world)

    import meshclust_amd as M
    if rank == 0 and not os.path.exists(M.GPU_LIB):
        M.build()
    M.tune_host_heap()  # this process runs many clusterings: keep large freed blocks
    if shard and world == 1:
        os.environ["MC_SHARD_FORCE"] = "1"  # the sharded code path with one rank
    if shard and rank == 0:  # one shared input: rank 0 writes it, the others wait
        ensure_fasta(a.n, a.len, a.templates, a.mut, a.seed)
    if dist:
        dist.barrier()
    fasta = ensure_fasta(a.n, a.len, a.templates, a.mut, a.seed + (0 if shard else rank))
    threads = min(16, host_threads())
    # MC_BENCH_ONE_GPU=1 (rehearsal on a one-GPU box): every rank on GPU 0, the ranks' kernels
    # splitting its CUs, gloo for the host-side all-gathers (RCCL takes one rank per GPU)
    one_gpu = os.environ.get("MC_BENCH_ONE_GPU") == "1"
    if one_gpu:
        local = 0
    eng = M.Engine(local)
    args = ["--id", a.id, "--threads", str(threads)]
    comm = None
    if shard:  # libmcgpu's RCCL communicator, called from C++ (torch.distributed only hands out its id)
        from meshclust_amd.dist import RcclShardComm, TorchShardComm
        comm = TorchShardComm() if one_gpu else RcclShardComm(local)
    # The GPU is driven by libmcgpu alone: torch's own HIP runtime (a second HIP/HSA runtime in
    # the process, from torch's bundled ROCm) is never initialised here -- two runtimes on one
    # GPU made the process fault in the system HSA runtime's exit handler under rocprofv3.
    sync = eng.sync  # hipDeviceSynchronize on this rank's GPU
    out_dir = tempfile.mkdtemp(prefix="mc_bench_out")
    nstep = [0]

    def one_step():
        """parse -> upload -> GPU pipeline -> .clstr written (the BASELINE metric's work).
        Every run writes a new output file, as a clustering run does (rewriting one path would
        time the kernel freeing the previous run's page-cache pages on O_TRUNC: 2.5 ms for
        4 MB); the files are removed after the timed region."""
        nstep[0] += 1
        clstr = os.path.join(out_dir, "bench_rank%d_%d.clstr" % (rank, nstep[0]))
        t = time.perf_counter()
        ds = M.Dataset([fasta], threads=threads)
        t1 = time.perf_counter()
        st = ds.run(eng, args, upload=True, clstr=clstr, comm=comm)
        t2 = time.perf_counter()
        del ds
        st["parse_s"] = t1 - t
        st["run_s"] = t2 - t1
        st["free_s"] = time.perf_counter() - t2
        return st

    # warm-up: end-to-end steps, then resident-data runs (sequences already in HBM)
    t0 = time.perf_counter()
    for _ in range(max(1, a.warmup)):
        one_step()
    first_s = time.perf_counter() - t0
    ds_res = M.Dataset([fasta], threads=threads)
    ds_res.run(eng, args, upload=True, comm=comm)
    res_t = []
    for _ in range(2):
        t = time.perf_counter()
        ds_res.run(eng, args, upload=False, comm=comm)
        res_t.append(time.perf_counter() - t)
    del ds_res
    eng.timers(reset=True)

    if dist:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    stats = []
    for _ in range(a.steps):
        stats.append(one_step())
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
        if comm is not None:
            comm.close()
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
        # (sharded: each rank's kernel scans its 1/world of every window)
        per_launch_bytes = scan_evals * eval_bytes / fam_n["scan"] / (world if shard else 1)
        avg_s = fam_ms["scan"] / fam_n["scan"] / 1e3
        ach = per_launch_bytes / avg_s / 1e9
        # one launch per clustering = the device-resident accumulation (accum.hip); otherwise
        # one fused scan launch per get_close step (scan.hip)
        device_loop = fam_n["scan"] <= a.steps
        kname = "accum_kernel<unsigned char" if device_loop else "fused_scan_kernel<unsigned char"
        roof = {"kernel": ("accum_kernel (whole accumulation phase, %d dependent get_close steps per launch)"
                           % s0["scan_steps"]) if device_loop else "fused_scan_kernel (Trainer::get_close step)",
                "bound": "hbm", "achieved": round(ach, 1),
                "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": None,
                "bytes_per_eval": eval_bytes, "evals_per_launch": round(scan_evals / fam_n["scan"], 1),
                "avg_launch_us": round(avg_s * 1e6, 2),
                "us_per_step": round(fam_ms["scan"] * 1e3 / sum(s["scan_steps"] for s in stats), 2)}
        pmc = os.path.join(ROOT, "profiles", "pmc_latest.json")
        if os.path.exists(pmc) and not shard:  # (counters of the config-B launch)  # rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (scripts/pmc_summary.py)
            e = next((v for k2, v in sorted(json.load(open(pmc)).items()) if k2.startswith(kname)), None)
            if e and "hbm_bytes_per_dispatch" in e:
                roof["traffic"] = round(e["hbm_bytes_per_dispatch"])
                roof["traffic_unit"] = "bytes/launch (FETCH_SIZE x2 + WRITE_SIZE, profiles/pmc_latest.json)"
                roof["algorithmic_bytes_per_launch"] = round(per_launch_bytes)
    nw_cells = sum(s["nw_cells"] for s in stats)
    nw_rate = nw_cells / (fam_ms["nw"] / 1e3) if fam_ms["nw"] else None
    # NW is VALU-bound: 26.5 VALU instructions per cell in the throughput form;
    # a wave64 VALU instruction holds its SIMD 4 cycles (MI355X_MICROARCH.md issue costs), so
    # the int32 issue peak is 256 CU x 4 SIMD x 16 lanes/clk x 2.4 GHz = 39.3e12 lane-ops/s
    # (SQ_INSTS_VALU agrees: profiles/r03_v4/config_c.json, 0.98 of it in the throughput form)
    nw_peak = 256 * 4 * 16 * 2.4e9 / 26.5
    nw_roof = {"bound": "valu", "achieved": nw_rate, "peak": nw_peak, "unit": "cells/s",
               "frac": round(nw_rate / nw_peak, 4) if nw_rate else None,
               "cells_per_step": nw_cells / a.steps, "ms_per_step": round(fam_ms["nw"] / a.steps, 3)}
    nwc = os.path.join(ROOT, "profiles", "nw_counters.json")
    if os.path.exists(nwc):  # rocprofv3 SQ counter pass on the NW kernels (scripts/prof_summary.py)
        nw_roof["counters"] = json.load(open(nwc))
    cpu = None
    if not a.no_cpu_baseline and world == 1 and not shard:  # the reference: rank 0 at N = 1 only
        cpu = cpu_baseline(fasta, ["--id", a.id], a.n, host_threads(), a.cpu_repeats)
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
        "data": "synthetic (meshclust_amd.synth: %d reads x %d bp, %d templates, mut %.2f, seed %d%s)"
                % (a.n, a.len, a.templates, a.mut, a.seed, "" if shard else "+rank"),
        "config": {"workload": ("config D: %dk synthetic 1kb reads (%d templates), --id %s k-mer mean-shift, "
                                "one clustering shared by %d GPU(s)" % (a.n // 1000, a.templates, a.id, world)) if shard
                   else "config B: %dk synthetic 1kb reads, --id %s k-mer mean-shift" % (a.n // 1000, a.id),
                   "reads": a.n if shard else a.n * world, "read_len": a.len, "k": s0["k"], "histogram_bits": 8 * width,
                   "parallelism": ("one clustering sharded by record x%d (device mailbox exchange per get_close "
                                   "step, RCCL all-gather per mean-shift iteration)" % world) if shard
                   else "replicas x%d" % world},
        "roofline": roof,
        "cpu_baseline": cpu,
        "extra": {"nw_cell_updates_per_s": nw_rate, "nw_roofline": nw_roof, "clusters": s0["clusters"],
                  "dominant_family": dominant,
                  "resident_sequences_per_s": round(a.n / min(res_t), 1),
                  "resident_ms_per_run": [round(x * 1e3, 2) for x in res_t],
                  "step_split_ms": {"parse": round(1e3 * sum(s["parse_s"] for s in stats) / a.steps, 2),
                                    "upload_to_partition": round(sum(s["phases_ms"]["total_pipeline"]
                                                                     for s in stats) / a.steps, 2),
                                    "write_clstr": round(sum(s["write_ms"] for s in stats) / a.steps, 2),
                                    "run_other": round(sum(1e3 * s["run_s"] - s["phases_ms"]["total_pipeline"] - s["write_ms"]
                                                           for s in stats) / a.steps, 2),
                                    "free_dataset": round(1e3 * sum(s["free_s"] for s in stats) / a.steps, 2)},
                  "device_ms_per_step": {f: round(v / a.steps, 3) for f, v in fam_ms.items()},
                  "launches_per_step": {f: round(v / a.steps, 1) for f, v in fam_n.items()},
                  "host_phases_ms": s0["phases_ms"], "accum_path": s0.get("accum_path"),
                  "warmup_s": round(first_s, 3), "scan_steps": s0["scan_steps"]},
    }
    print(json.dumps(line), flush=True)
    if a.stats_out:
        with open(a.stats_out, "w") as f:
            json.dump({"line": line, "stats": stats, "timers": tim}, f, indent=1)
    if comm is not None:
        comm.close()
    eng.close()
    if os.environ.get("MC_DUMP_MAPS"):  # diagnostics: the process map, to resolve exit-time PCs
        with open("/proc/self/maps") as f, open(os.environ["MC_DUMP_MAPS"], "w") as g:
            g.write(f.read())
    import shutil
    shutil.rmtree(out_dir, ignore_errors=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
