#!/usr/bin/env python3
"""bench.py -- sequences clustered per second on MI355X (BASELINE.json metric).

Workloads (synthetic reads from meshclust_amd.synth, generated before the
timed region and read from the page cache):

* ``--workload B`` (default; BASELINE.json configs[1]): 100,000 reads x 1 kb, 1,000
  templates, 3% per-base mutation, seed 41, ``--id 0.90`` (auto k = 4, 8-bit histograms);
* ``--workload D`` (configs[3]): 1,000,000 reads x 1 kb, 10,000 templates, seed 51.

One "step" = one end-to-end run of meshclust on that FASTA (N / wall from
parse to .clstr written): parse + encode + 2-bit pack on the host, upload, K1 histograms ->
training (split sort keys, NW labels, GLM) -> accumulation -> 15 mean-shift + merge
iterations on the GPU, .clstr written.  The rate on sequences already resident in HBM (no
parse / upload / write) is reported in "extra" as resident_sequences_per_s.

GPUs.  ``--gpus N`` runs N ranks, one process per GPU: launched by the driver through
torch.distributed.run, or -- when WORLD_SIZE is not set -- spawned here as N child processes
(RANK / WORLD_SIZE / MASTER_* as torch.distributed.run sets them, 127.0.0.1) before anything
touches a GPU; rank 0 prints the line.
The N ranks share ONE clustering of the same workload at every N, sharded by record (strong
scaling): every rank's persistent accumulation kernel scans its interleaved tiles of each
get_close window and the kernels exchange each step's {first maximum, flagged reads} through a
host-memory mailbox they all map (no host round trip per step); the training's pivots and label
alignments and every mean-shift iteration are split over the ranks and all-gathered (RCCL, the
centre reassignment).  ``--mode replicas`` instead gives every rank its own batch (seed +
rank: weak scaling, no collective on the data path); ``--mode shard`` at N = 1 runs the
sharded code path on one rank.  MC_BENCH_ONE_GPU=1 (rehearsal on a one-GPU box): every rank
on GPU 0, each kernel on its share of the CUs, gloo for the host-side all-gathers.

Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
WORKLOADS = {  # reads, templates, seed (length 1 kb, mutation 0.03)
    "B": (100000, 1000, 41),
    "D": (1000000, 10000, 51),
}


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


def cpu_baseline(fasta, args, n_reads, threads, repeats, limit_s=600, binary="meshclust", march="x86-64-v4"):
    """The reference itself (oracle/_ref/meshclust, compiled from /root/reference by
    oracle/Makefile with the reference's own flags, -march=native pinned to x86-64-v4: AVX-512)
    on the same FASTA on this host's cores, end to end (process start to .clstr written),
    median of `repeats` runs."""
    ref = os.path.join(ROOT, "oracle", "_ref", binary)
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
                      "wall %s s (median of %d), parse to .clstr written; built -O3 -march=%s -fopenmp "
                      "(src/cluster/Makefile's flags, -march=native pinned)"
                      % (n_reads, " ".join(args), threads, "/".join("%.2f" % w for w in walls), len(walls), march),
            "march": march,
            "cpu_model": cpu_model(), "host_cpus": os.cpu_count(), "threads": threads}


def spawn_ranks(n):
    """--gpus N without a launcher: N child processes of this script, one rank each (RANK,
    LOCAL_RANK, WORLD_SIZE and MASTER_* set as torch.distributed.run sets them, 127.0.0.1);
    this process never touches a GPU.  A rank that fails ends the others; the exit status is
    the first failure's."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            c = p.poll()
            if c is None:
                continue
            live.remove(p)
            if c != 0 and rc == 0:
                rc = c if c > 0 else 1
                for q in live:
                    q.terminate()
        time.sleep(0.05)
    return rc


NW_STEADY_INSTS_PER_CELL = 19.9
# The accumulation's step-latency floor ("The floor"): a get_close step cannot
# take less than two cross-CU hand-offs (the step record out to the workers, their partials
# back; MI355X_MICROARCH.md price list, handoff-1to1, idle, 8 B: 0.8 us each), one candidate
# wave's scoring chain at the VALU issue interval of one wave per SIMD (the ISA's instructions
# per candidate wave, scripts/isa_count.py -> profiles/r05/accum_isa_counts.json; 5.7 clocks per
# wave instruction at one wave per SIMD, profiles/r04/valu_peak.json, 2.4 GHz), and in a member
# step one dependent memory round trip for the new members' rows (half a hand-off, 0.4 us).
HOP_US = 0.8
SCORE_WAVE_INSTS = 324  # profiles/r05/accum_isa_counts.json "valu"
CLK_PER_WAVE_INST = 5.7
MEMBER_LOAD_US = 0.4


def latency_floor(achieved_us, stats):
    steps = sum(s["scan_steps"] for s in stats)
    clusters = sum(s["clusters"] for s in stats)
    member_frac = max(0.0, 1.0 - clusters / steps) if steps else 0.0  # (one is_min step per cluster)
    score = SCORE_WAVE_INSTS * CLK_PER_WAVE_INST / 2.4e3
    floor = 2 * HOP_US + score + member_frac * MEMBER_LOAD_US
    return {"floor_us_per_step": round(floor, 3), "achieved_us_per_step": achieved_us,
            "frac": round(floor / achieved_us, 4) if achieved_us else None,
            "hops_us": 2 * HOP_US, "score_us": round(score, 3), "member_load_us": round(member_frac * MEMBER_LOAD_US, 3),
            "member_step_frac": round(member_frac, 3),
            "model": "2 hand-offs (handoff-1to1 idle) + one candidate wave's VALU chain at 1 wave/SIMD + "
                     "a member step's dependent row load"}


def comm_summary(stats):
    """Per phase, ms per step of waiting for the last rank and of the exchange itself (the
    ranks' all-gathers are timed in C++, runner.cpp TimedComm), calls and KB."""
    out = {}
    for s in stats:
        for k, v in s["phases_ms"].items():
            if k.startswith("comm."):
                out[k[5:]] = out.get(k[5:], 0.0) + v / len(stats)
    return {k: round(v, 3) for k, v in sorted(out.items())} or None


def kernel_pmc(kname):
    """The FETCH_SIZE / WRITE_SIZE passes of a kernel (rocprofv3 --pmc, separate passes,
    scripts/pmc_summary.py): HBM bytes per launch, FETCH doubled per the gfx950 note."""
    pmc = os.path.join(ROOT, "profiles", "pmc_latest.json")
    if not os.path.exists(pmc):
        return None
    e = next((v for k, v in sorted(json.load(open(pmc)).items()) if k.startswith(kname)), None)
    return round(e["hbm_bytes_per_dispatch"]) if e and "hbm_bytes_per_dispatch" in e else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="B",
                    help="B: 100k x 1 kb (BASELINE configs[1]); D: 1M x 1 kb (configs[3])")
    ap.add_argument("--mode", choices=["auto", "shard", "replicas"], default="auto",
                    help="auto: one clustering (sharded by record over the ranks when N > 1)")
    ap.add_argument("--n", type=int, default=None)
    ap.add_argument("--len", type=int, default=1000)
    ap.add_argument("--templates", type=int, default=None)
    ap.add_argument("--mut", type=float, default=0.03)
    ap.add_argument("--seed", type=int, default=None)
    ap.add_argument("--id", default="0.90")
    ap.add_argument("--cpu-repeats", type=int, default=3, help="reference runs (median)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--stats-out", default=None)
    ap.add_argument("--keep-clstr", default=None, help="rank 0 keeps the last timed step's .clstr here")
    ap.add_argument("--config-d-steps", type=int, default=2,
                    help="with the config-B line: also time config D (1M reads, BASELINE configs[3], the workload "
                         "that shards) at the same N, reported in extra.config_d (0: skip)")
    ap.add_argument("--no-config-d", action="store_true", help="same as --config-d-steps 0")
    a = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        sys.exit(spawn_ranks(a.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    mode = "replicas" if a.mode == "replicas" else "shard" if (a.mode == "shard" or world > 1) else "single"
    shard = mode == "shard"
    n0, t0_, s0_ = WORKLOADS[a.workload]
    a.n = a.n if a.n is not None else n0
    a.templates = a.templates if a.templates is not None else t0_
    a.seed = a.seed if a.seed is not None else s0_
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
    replicas = mode == "replicas"
    if rank == 0:  # one shared input (rank 0 writes it, the others wait), or rank 0's replica
        ensure_fasta(a.n, a.len, a.templates, a.mut, a.seed)
    if dist:
        dist.barrier()
    fasta = ensure_fasta(a.n, a.len, a.templates, a.mut, a.seed + (rank if replicas else 0))
    threads = min(16, host_threads())
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
    last_clstr = [None]

    def one_step(fa):
        """parse -> upload -> GPU pipeline -> .clstr written (the BASELINE metric's work).
        Every run writes a new output file, as a clustering run does (rewriting one path would
        time the kernel freeing the previous run's page-cache pages on O_TRUNC: 2.5 ms for
        4 MB); the files are removed after the timed region."""
        nstep[0] += 1
        clstr = os.path.join(out_dir, "bench_rank%d_%d.clstr" % (rank, nstep[0]))
        last_clstr[0] = clstr
        t = time.perf_counter()
        ds = M.Dataset([fa], threads=threads)
        t1 = time.perf_counter()
        st = ds.run(eng, args, upload=True, clstr=clstr, comm=comm)
        t2 = time.perf_counter()
        del ds
        st["parse_s"] = t1 - t
        st["run_s"] = t2 - t1
        st["free_s"] = time.perf_counter() - t2
        return st

    def timed(fa, steps, warmup, resident_runs):
        """`warmup` untimed end-to-end steps (and `resident_runs` runs on sequences already in
        HBM), then exactly `steps` timed steps bracketed by a barrier + device sync on both sides;
        the elapsed time is the maximum over the ranks."""
        t0 = time.perf_counter()
        for _ in range(max(1, warmup)):
            one_step(fa)
        first = time.perf_counter() - t0
        res = []
        if resident_runs:
            ds_res = M.Dataset([fa], threads=threads)
            ds_res.run(eng, args, upload=True, comm=comm)
            for _ in range(resident_runs):
                t = time.perf_counter()
                ds_res.run(eng, args, upload=False, comm=comm)
                res.append(time.perf_counter() - t)
            del ds_res
        eng.timers(reset=True)
        if dist:
            dist.barrier()
        sync()
        t0 = time.perf_counter()
        st = [one_step(fa) for _ in range(steps)]
        sync()
        if dist:
            dist.barrier()
        el = time.perf_counter() - t0
        tm = eng.timers()
        if dist:
            import torch as _t
            t = _t.tensor([el], dtype=_t.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        return el, st, tm, first, res

    elapsed, stats, tim, first_s, res_t = timed(fasta, a.steps, a.warmup, 2)
    keep_src = last_clstr[0]

    # config D at the same N (the workload that shards by record: BASELINE configs[3]), so the
    # driver's 1 -> 8 GPU runs carry a config-D curve beside the config-B headline
    d_run = None
    d_steps = 0 if a.no_config_d or a.workload != "B" or replicas else a.config_d_steps
    if d_steps > 0:
        dn, dt_, ds_ = WORKLOADS["D"]
        if rank == 0:
            ensure_fasta(dn, a.len, dt_, a.mut, ds_)
        if dist:
            dist.barrier()
        d_fa = ensure_fasta(dn, a.len, dt_, a.mut, ds_)
        d_el, d_stats, d_tim, d_first, _ = timed(d_fa, d_steps, 1, 0)
        d_run = (dn, dt_, ds_, d_el, d_stats, d_tim, d_first)

    if rank != 0:
        if comm is not None:
            comm.close()
        eng.close()
        if dist:
            dist.destroy_process_group()
        return
    s0 = stats[-1]
    n_total = a.n * a.steps * (world if replicas else 1)
    value = n_total / elapsed
    ms_step = elapsed / a.steps * 1000.0

    # roofline of the dominant kernel (accumulation), and of the other HBM kernels
    fam_ms = {f: v[0] for f, v in tim.items()}
    fam_n = {f: v[1] for f, v in tim.items()}
    B = 4 ** s0["k"]
    width = s0["width"]
    dominant = max(fam_ms, key=lambda f: fam_ms[f])

    def scan_roofline(stats, tim, steps, workload):
        """accum_kernel's roofline: evaluations x (B*w + 17) algorithmic bytes per launch over
        the launch's duration by HIP events on the library's stream."""
        fms = {f: v[0] for f, v in tim.items()}
        fn = {f: v[1] for f, v in tim.items()}
        st0 = stats[-1]
        eval_bytes = 4 ** st0["k"] * st0["width"] + 17  # row + length + magnitude + flag per candidate
        scan_evals = sum(s["scan_candidates"] for s in stats)
        acc_split = shard and str(st0.get("accum_path", "")).startswith("device x")  # (vs replicated)
        if not fn["scan"]:
            return None, acc_split
        # (accumulation split over the ranks: each rank's kernel scans its 1/world of every window)
        per_launch_bytes = scan_evals * eval_bytes / fn["scan"] / (world if acc_split else 1)
        avg_s = fms["scan"] / fn["scan"] / 1e3
        ach = per_launch_bytes / avg_s / 1e9
        # one launch per clustering = the device-resident accumulation (accum.hip); otherwise
        # one fused scan launch per get_close step (scan.hip)
        device_loop = fn["scan"] <= steps
        kname = "accum_kernel<unsigned char" if device_loop else "fused_scan_kernel<unsigned char"
        r = {"kernel": ("accum_kernel (whole accumulation phase, %d dependent get_close steps per launch)"
                        % st0["scan_steps"]) if device_loop else "fused_scan_kernel (Trainer::get_close step)",
             "bound": "hbm", "achieved": round(ach, 1),
             "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": None,
             "bytes_per_eval": eval_bytes, "evals_per_launch": round(scan_evals / fn["scan"], 1),
             "avg_launch_us": round(avg_s * 1e6, 2),
             "us_per_step": round(fms["scan"] * 1e3 / sum(s["scan_steps"] for s in stats), 2),
             "note": ("priced against HBM by algorithmic bytes (SURVEY.md §8(d)); the rows stay in LDS, "
                      "so the kernel is bound by its dependent step chain, not by HBM (DESIGN.md §3.1)")
                     if workload == "B" else
                     ("priced against HBM by algorithmic bytes (SURVEY.md §8(d)); on one to four GPUs "
                      "the workers stream every window's rows from HBM (dense streaming form, DESIGN.md "
                      "§3.1c), except each thread's first list entry, kept in the launch's spare LDS (the "
                      "achieved figure counts those rows' bytes too: §5.0); at eight each rank's share of "
                      "the rows is LDS-resident (§6)")}
        if device_loop and workload == "B":
            r["latency_floor"] = latency_floor(r["us_per_step"], stats)
        if workload == "B" and not shard and world == 1:  # (the counters are of the config-B launch)
            tr = kernel_pmc(kname)
            if tr is not None:
                r["traffic"] = tr
                r["traffic_unit"] = "bytes/launch (FETCH_SIZE x2 + WRITE_SIZE, profiles/pmc_latest.json)"
                r["algorithmic_bytes_per_launch"] = round(per_launch_bytes)
        return r, acc_split

    roof, acc_split = scan_roofline(stats, tim, a.steps, a.workload)
    # K1 and the mean-shift update, the other two HBM-class kernels north_star names
    # (K1: ceil(L/4) packed bytes in + B*w row + 8 magnitude out per read; mean shift: one read
    # of each neighbourhood member's row and magnitudes per centre, update_evals of them)
    others = {}
    if fam_n["kmer"]:
        kb = a.n * (a.len / 4.0 + B * width + 8) * a.steps / fam_n["kmer"]
        ks = fam_ms["kmer"] / fam_n["kmer"] / 1e3
        others["kmer_kernel"] = {"bound": "hbm", "bytes_per_read": a.len / 4.0 + B * width + 8,
                                 "algorithmic_bytes_per_launch": round(kb), "avg_launch_us": round(ks * 1e6, 2),
                                 "achieved": round(kb / ks / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                 "frac": round(kb / ks / 1e9 / HBM_PEAK_GBS, 4),
                                 "traffic": kernel_pmc("kmer_kernel<unsigned char") if width == 1 and a.workload == "B" else None}
    if fam_n["mean_shift"]:
        # (the evaluations of the update iterations actually run: a fixed point ends the loop early)
        mb = sum(s.get("update_evals_run", s["update_evals"]) for s in stats) * (B * width + 16) / fam_n["mean_shift"] \
            / (world if shard else 1)
        ms = fam_ms["mean_shift"] / fam_n["mean_shift"] / 1e3
        others["mean_shift_kernel"] = {"bound": "hbm", "bytes_per_member": B * width + 16,
                                       "algorithmic_bytes_per_launch": round(mb), "avg_launch_us": round(ms * 1e6, 2),
                                       "achieved": round(mb / ms / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                       "frac": round(mb / ms / 1e9 / HBM_PEAK_GBS, 4),
                                       "traffic": kernel_pmc("mean_shift_kernel<unsigned char") if width == 1 and a.workload == "B" else None}
    nw_cells = sum(s["nw_cells"] for s in stats)
    nw_rate = nw_cells / (fam_ms["nw"] / 1e3) if fam_ms["nw"] else None
    # NW is VALU-bound: the peak is the int32 VALU issue rate (lane-instructions
    # per second, from the microbenchmark in profiles/) over the VALU instructions per cell that
    # the SQ_INSTS_VALU counter gives for the current kernels (profiles/nw_counters.json)
    nwc_path = os.path.join(ROOT, "profiles", "nw_counters.json")
    nwc = json.load(open(nwc_path)) if os.path.exists(nwc_path) else {}
    lane_ops = nwc.get("valu_lane_ops_per_s", 256 * 4 * 16 * 2.4e9)
    # priced at the throughput form's steady-state step, 19.9 lane-instructions per cell (the ISA
    # count): the latency form's hand-offs, ramps and barriers are overhead, not
    # work, so they count against the fraction (the kernels' own counter ratio is kept beside it)
    ipc = NW_STEADY_INSTS_PER_CELL
    nw_peak = lane_ops / ipc
    nw_roof = {"bound": "valu", "achieved": nw_rate, "peak": nw_peak, "unit": "cells/s",
               "frac": round(nw_rate / nw_peak, 4) if nw_rate else None,
               "lane_insts_per_cell": ipc, "kernel_lane_insts_per_cell": nwc.get("lane_insts_per_cell"),
               "valu_lane_ops_per_s": lane_ops,
               "cells_per_step": nw_cells / a.steps, "ms_per_step": round(fam_ms["nw"] / a.steps, 3)}
    if nwc:
        nw_roof["counters"] = nwc
    cpu = cpu_v3 = None
    if not a.no_cpu_baseline and world == 1 and mode == "single" and a.workload == "B":
        # the reference: rank 0 at N = 1 only, on the full config-B FASTA (~27 s a run)
        cpu = cpu_baseline(fasta, ["--id", a.id], a.n, host_threads(), a.cpu_repeats)
        # (rounds 1-5 timed an x86-64-v3 build: one run of it, for continuity)
        cpu_v3 = cpu_baseline(fasta, ["--id", a.id], a.n, host_threads(), 1, binary="meshclust_v3", march="x86-64-v3")
    wl = "config %s: %dk synthetic 1kb reads (%d templates), --id %s k-mer mean-shift" % (
        a.workload, a.n // 1000, a.templates, a.id)
    line = {
        "metric": "sequences clustered/sec (+ NW cell-updates/sec) at 1/2/4/8 MI355X",
        "value": round(value, 1),
        "unit": "sequences/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(ms_step, 2),
        "higher_is_better": True,
        "scaling": "weak" if replicas else "strong",
        "vs_baseline": None,
        "dtype": "u8" if width == 1 else "u%d" % (8 * width),
        "data": "synthetic (meshclust_amd.synth: %d reads x %d bp, %d templates, mut %.2f, seed %d%s)"
                % (a.n, a.len, a.templates, a.mut, a.seed, "+rank" if replicas else ""),
        "config": {"workload": wl + (", one clustering sharded by record over %d GPU(s)" % world if shard else
                                     ", %d independent replica(s)" % world if replicas else ", one GPU"),
                   "workload_config": a.workload, "mode": mode,
                   "reads": a.n * (world if replicas else 1), "read_len": a.len, "k": s0["k"],
                   "histogram_bits": 8 * width,
                   "parallelism": ("one clustering over %d GPUs: accumulation %s; training pivots / labels and "
                                   "every mean-shift iteration split by rank, RCCL all-gathers"
                                   % (world, "sharded by record (device mailbox exchange per get_close step)" if acc_split
                                      else "replicated (every row resident in one GPU's LDS: the per-step exchange "
                                           "would lengthen the chain)")) if shard
                   else "replicas x%d" % world if replicas else "single GPU"},
        "roofline": roof,
        "cpu_baseline": cpu,
        "extra": {"nw_cell_updates_per_s": nw_rate, "nw_roofline": nw_roof, "kernel_rooflines": others,
                  "clusters": s0["clusters"], "dominant_family": dominant,
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
                  "comm_ms_per_step": comm_summary(stats),
                  "warmup_s": round(first_s, 3), "scan_steps": s0["scan_steps"],
                  # (the reference's default --iterations 15; bench passes none)
                  "update_iterations": {"run": 15 - s0.get("update_iters_fixed", 0),
                                        "fixed_point_left_out": s0.get("update_iters_fixed", 0)},
                  "rehearsal_one_gpu": one_gpu},
    }
    if cpu_v3 is not None:
        line["extra"]["cpu_baseline_x86_64_v3"] = cpu_v3
    if cpu is None and world == 1 and a.workload != "B":
        line["extra"]["cpu_baseline_note"] = "the reference is timed on config B only (config D takes it hours)"
    if a.workload == "B" and world > 1 and not replicas:
        line["config"]["config_b_at_n_gt_1"] = (
            "config B's accumulation is replicated by design whenever one GPU's LDS holds its 100k rows (a "
            "per-step exchange would only lengthen the dependent chain: DESIGN.md §6) -- here: %s; the training "
            "and the mean shift split by rank.  extra.config_d is the workload that shards by record"
            % ("sharded (ranks sharing one GPU: each rank's CU share cannot hold the rows)" if acc_split
               else "replicated"))
    if d_run is not None:
        dn, dt_, ds_, d_el, d_stats, d_tim, d_first = d_run
        d0 = d_stats[-1]
        d_roof, d_split = scan_roofline(d_stats, d_tim, len(d_stats), "D")
        nd = len(d_stats)
        line["extra"]["config_d"] = {
            "workload": "config D: %dk synthetic 1kb reads (%d templates, seed %d), --id %s k-mer mean-shift, one "
                        "clustering%s" % (dn // 1000, dt_, ds_, a.id,
                                          " sharded by record over %d GPU(s)" % world if shard else " on one GPU"),
            "value": round(dn * nd / d_el, 1), "unit": "sequences/s", "n_gpus": world, "steps": nd, "warmup": 1,
            "ms_per_step": round(d_el / nd * 1e3, 2), "scaling": "strong", "roofline": d_roof,
            "accum_path": d0.get("accum_path"), "accum_sharded_by_record": d_split, "clusters": d0["clusters"],
            "scan_steps": d0["scan_steps"],
            "step_split_ms": {"parse": round(1e3 * sum(s["parse_s"] for s in d_stats) / nd, 2),
                              "upload_to_partition": round(sum(s["phases_ms"]["total_pipeline"] for s in d_stats) / nd, 2),
                              "write_clstr": round(sum(s["write_ms"] for s in d_stats) / nd, 2)},
            "device_ms_per_step": {f: round(v[0] / nd, 3) for f, v in d_tim.items()},
            "comm_ms_per_step": comm_summary(d_stats), "warmup_s": round(d_first, 3)}
    print(json.dumps(line), flush=True)
    if a.stats_out:
        with open(a.stats_out, "w") as f:
            json.dump({"line": line, "stats": stats, "timers": tim}, f, indent=1)
    if a.keep_clstr and keep_src:
        import shutil
        shutil.copyfile(keep_src, a.keep_clstr)
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
