"""One rank of a sharded clustering (launched by torch.distributed.run; see
tests/test_distributed.py).  Engine: the CPU oracle engine (test-only) or, with --gpu, the
product's libmcgpu on cuda:0 (every rank: the test boxes have one GPU), or with --per-rank-gpu
on the rank's own GPU (LOCAL_RANK; boxes with several GPUs).  Exchange: a gloo all-gather
through a Python callback, or with --rccl libmcgpu's RCCL communicator called from C++ (one
rank per GPU).  --grid-per-rank G0,G1,...: rank r caps its accumulation grid at G_r
(MC_ACCUM_GRID), so the ranks start from different plans."""
import argparse
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fasta")
    ap.add_argument("out")
    ap.add_argument("--gpu", action="store_true")
    ap.add_argument("--rccl", action="store_true")
    ap.add_argument("--per-rank-gpu", action="store_true")
    ap.add_argument("--grid-per-rank", default=None)
    ap.add_argument("flags", nargs="*")
    a = ap.parse_args()
    import datetime
    import torch.distributed as dist
    # a rank that fails (tests inject faults, MC_FAULT) never joins the next exchange: the others
    # give up after MC_DIST_TIMEOUT_S instead of gloo's 30 minutes
    dist.init_process_group("gloo", init_method="env://",
                            timeout=datetime.timedelta(seconds=float(os.environ.get("MC_DIST_TIMEOUT_S", "600"))))
    from meshclust_amd.dist import RcclShardComm, TorchShardComm
    if a.grid_per_rank:
        os.environ["MC_ACCUM_GRID"] = a.grid_per_rank.split(",")[dist.get_rank()]
    if a.gpu:
        import meshclust_amd as M
        dev = int(os.environ.get("LOCAL_RANK", "0")) if a.per_rank_gpu else 0
        eng = M.Engine(dev)
        comm = RcclShardComm(dev) if a.rccl else TorchShardComm()
        ds = M.Dataset([a.fasta], threads=4)
        st = ds.run(eng, a.flags + ["--threads", "4"], upload=True, clstr=a.out if comm.rank == 0 else None,
                    comm=comm)
        eng.close()
    else:
        comm = TorchShardComm()
        lib = C.CDLL(os.path.join(ROOT, "oracle", "_build", "libmeshclust_cpu.so"))
        lib.mcl_parse.restype = C.c_void_p
        lib.mcl_parse.argtypes = [C.POINTER(C.c_char_p), C.c_int, C.c_int, C.c_char_p, C.c_int]
        lib.mcl_run_sharded.restype = C.c_int
        lib.mcl_run_sharded.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.POINTER(C.c_char_p), C.c_int, C.c_char_p,
                                        C.c_char_p, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p]
        ctx = C.c_void_p()
        assert lib.mc_ctx_create(0, C.byref(ctx)) == 0
        err = C.create_string_buffer(512)
        ds = lib.mcl_parse((C.c_char_p * 1)(a.fasta.encode()), 1, 2, err, 512)
        assert ds, err.value
        argv = [b"meshclust"] + [f.encode() for f in a.flags] + [b"--threads", b"2"]
        buf = C.create_string_buffer(1 << 16)
        rc = lib.mcl_run_sharded(ds, ctx, len(argv), (C.c_char_p * len(argv))(*argv), 1,
                                 a.out.encode() if comm.rank == 0 else None, buf, len(buf), comm.rank, comm.world,
                                 C.cast(comm.callback, C.c_void_p), comm.user)
        assert rc == 0, buf.value
        st = json.loads(buf.value.decode())
    with open(a.out + ".rank%d.json" % comm.rank, "w") as f:
        json.dump({"calls": comm.calls, "clusters": st.get("clusters"), "accum_path": st.get("accum_path"),
                   "scan_steps": st.get("scan_steps")}, f)
    comm.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
