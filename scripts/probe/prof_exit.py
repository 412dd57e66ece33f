"""Probe (rocprofv3 exit-time SIGSEGV): load libmcgpu, run a small K1 + NW workload, close the
context, dump /proc/self/maps (to resolve the crash PCs), exit.  argv[1]: maps output path;
argv[2] (optional) 'torch' to import torch first, as bench.py does."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
if len(sys.argv) > 2 and sys.argv[2] == "torch":
    import torch  # noqa: F401
import numpy as np
import meshclust_amd as M

e = M.Engine(0)
rng = np.random.default_rng(1)
seqs = [rng.integers(0, 4, 500).astype(np.uint8) for _ in range(20)]
e.load_packed(seqs, [[[0, 499]] for _ in seqs])
e.kmer_max(4)
e.kmer_build(4, 1)
print("nw", e.nw_identity(np.arange(10), np.arange(10, 20))[0][:3], flush=True)
e.close()
with open("/proc/self/maps") as f, open(sys.argv[1], "w") as g:
    g.write(f.read())
print("done", flush=True)
