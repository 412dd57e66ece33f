"""Probe: can two ranks share one GPU in an RCCL communicator? (1-GPU test boxes)"""
import os
import sys
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def work(rank, world):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT="29533")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=rank, world_size=world)
    x = torch.full((4,), rank, dtype=torch.int32, device="cuda")
    parts = [torch.empty_like(x) for _ in range(world)]
    dist.all_gather(parts, x)
    torch.cuda.synchronize()
    print("rank", rank, [p.tolist() for p in parts], flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    mp.spawn(work, args=(2,), nprocs=2)
