"""One clustering shared by several GPUs: one process per GPU over
torch.distributed.

MeShClust's accumulation is a chain of dependent steps (the next centre is the member closest
to the current mean), so every rank runs it -- on its own GPU, deterministically, with the
same result.  The mean-shift update that follows is independent per centre: each rank computes
the new centres of its share (``mc_mean_shift_range``) and the ranks all-gather them, the
centre-reassignment exchange, once per iteration.  The C++ driver calls back into Python for
that exchange (``mcl_run_sharded``); with the ``nccl`` backend (RCCL on ROCm) the blocks travel
as device tensors, with ``gloo`` as host tensors.

Results are identical to a single-rank run (tests/test_distributed.py).
"""
import ctypes as C

ALLGATHER = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p)


class TorchShardComm:
    """All-gather of equal byte blocks over a torch.distributed process group."""

    def __init__(self, group=None):
        import torch
        import torch.distributed as dist
        self.torch, self.dist, self.group = torch, dist, group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        nccl = dist.get_backend(group) == "nccl"
        self.device = torch.device("cuda", torch.cuda.current_device()) if nccl else torch.device("cpu")
        self.calls = 0
        self.bytes = 0
        self.callback = ALLGATHER(self._allgather)  # keep a reference: C holds the pointer

    def _allgather(self, _user, src, nbytes, dst):
        try:
            t = self.torch
            self.calls += 1
            self.bytes += nbytes * self.world
            if nbytes == 0:
                return 0
            host = t.empty(nbytes, dtype=t.uint8)
            C.memmove(host.data_ptr(), src, nbytes)
            x = host.to(self.device)
            parts = [t.empty(nbytes, dtype=t.uint8, device=self.device) for _ in range(self.world)]
            self.dist.all_gather(parts, x, group=self.group)
            out = t.cat(parts).cpu()
            C.memmove(dst, out.data_ptr(), nbytes * self.world)
            return 0
        except Exception:  # reported to the driver as a failed exchange (it raises)
            return 1
