"""One clustering shared by several GPUs: one process per GPU over
torch.distributed.

The C++ driver (csrc/host/cluster.cpp) splits every get_close step of the accumulation over the
ranks by record -- rank r scans the alive candidates of the window in its static bvec blocks
(mc_scan_part) -- and the ranks all-gather one 1 KiB block per step ({first maximum of combo 0,
is_min, flagged positions}) before every rank applies the same remove_available + get_mean
(mc_scan_commit).  Each mean-shift iteration is split by centre and the ranks all-gather the
new centres (the centre-reassignment exchange).  The exchange is a C callback
``allgather(user, in, bytes, out)``:

* ``RcclShardComm`` -- RCCL over xGMI, called from C++ (libmcgpu's mc_comm_allgather); torch
  only distributes the communicator id (the product path on GPUs);
* ``TorchShardComm`` -- a Python callback over a torch.distributed group (gloo on CPUs: the
  CPU tests, where no RCCL exists).

Results are identical to a single-rank run (tests/test_distributed.py).
"""
import ctypes as C

ALLGATHER = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p)


class RcclShardComm:
    """An RCCL communicator of libmcgpu (mc_comm) for this rank's GPU; rank 0's id is broadcast
    over the default torch.distributed group."""

    def __init__(self, device, group=None):
        import torch.distributed as dist
        from . import gpu_lib, MCError
        self.lib = gpu_lib()
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        uid = C.create_string_buffer(128)
        if self.rank == 0 and self.lib.mc_comm_unique_id(uid) != 0:
            raise MCError("mc_comm_unique_id: " + self.lib.mc_last_error().decode())
        box = [uid.raw]
        dist.broadcast_object_list(box, src=0, group=group)
        self.user = C.c_void_p()
        if self.lib.mc_comm_create(device, self.rank, self.world, box[0], C.byref(self.user)) != 0:
            raise MCError("mc_comm_create: " + self.lib.mc_last_error().decode())
        self.callback = C.cast(self.lib.mc_comm_allgather, C.c_void_p)  # called from C++ directly

    @property
    def calls(self):
        c, b = C.c_uint64(), C.c_uint64()
        self.lib.mc_comm_stats(self.user, C.byref(c), C.byref(b))
        return c.value

    def close(self, abort=False):
        if self.user:
            self.lib.mc_comm_destroy(self.user, 1 if abort else 0)
            self.user = C.c_void_p()


class TorchShardComm:
    """All-gather of equal byte blocks over a torch.distributed process group (Python callback)."""

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
        self.user = None
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

    def close(self, abort=False):
        pass
