"""Deterministic synthetic read generator for the BASELINE.json configs.

SURVEY.md §8(d): T uniform-ACGT templates drawn with numpy ``default_rng(seed)``; read i
copies template ``i mod T`` and applies, per template base, a substitution, a deletion or
an insertion (a random base placed after the kept base) with probability ``mut/3`` each.
Headers are ``>read{i} template_{t}``, sequence lines are 60 columns.  The same generator
produced the CPU baselines quoted in BASELINE.md (config A: 1000 500 20 0.04 1; config B:
100000 1000 1000 0.03 41; config D: 1000000 1000 10000 0.03 51).

Usage: ``python -m meshclust_amd.synth N L T MUT SEED OUT.fa``
"""
import sys

import numpy as np

_ALPHA = np.frombuffer(b"ACGT", dtype=np.uint8)


def reads(n, length, n_templates, mut, seed):
    """Yield (header_bytes, sequence_bytes) for the configured synthetic set."""
    rng = np.random.default_rng(seed)
    temps = rng.integers(0, 4, size=(n_templates, length), dtype=np.uint8)
    p = mut / 3.0
    for i in range(n):
        t = i % n_templates
        s = temps[t]
        r = rng.random(length)
        sub = r < p
        dele = (r >= p) & (r < 2 * p)
        ins = (r >= 2 * p) & (r < mut)
        s2 = s.copy()
        s2[sub] = rng.integers(0, 4, size=int(sub.sum()), dtype=np.uint8)
        keep = ~dele
        reps = np.where(ins, 2, 1)[keep]
        base = np.repeat(s2[keep], reps)
        idx = np.cumsum(reps) - 1
        insm = reps == 2
        base[idx[insm]] = rng.integers(0, 4, size=int(insm.sum()), dtype=np.uint8)
        yield b"read%d template_%d" % (i, t), _ALPHA[base].tobytes()


def _mutate(rng, s, mut):
    p = mut / 3.0
    r = rng.random(len(s))
    sub = r < p
    dele = (r >= p) & (r < 2 * p)
    ins = (r >= 2 * p) & (r < mut)
    s2 = s.copy()
    s2[sub] = rng.integers(0, 4, size=int(sub.sum()), dtype=np.uint8)
    keep = ~dele
    reps = np.where(ins, 2, 1)[keep]
    base = np.repeat(s2[keep], reps)
    idx = np.cumsum(reps) - 1
    insm = reps == 2
    base[idx[insm]] = rng.integers(0, 4, size=int(insm.sum()), dtype=np.uint8)
    return base


def families(n_fam, per_fam, lmin, lmax, mut_lo, mut_hi, seed):
    """Viral-shape set (the shape of Tables/Viral.csv): n_fam
    family templates of uniform length in [lmin, lmax], each genome a copy of its family's
    template with a per-genome mutation rate uniform in [mut_lo, mut_hi].  Headers
    ``>genome{i} family_{f}``."""
    rng = np.random.default_rng(seed)
    temps = [rng.integers(0, 4, size=int(rng.integers(lmin, lmax + 1)), dtype=np.uint8)
             for _ in range(n_fam)]
    for i in range(n_fam * per_fam):
        f = i % n_fam
        base = _mutate(rng, temps[f], float(rng.uniform(mut_lo, mut_hi)))
        yield b"genome%d family_%d" % (i, f), _ALPHA[base].tobytes()


def write_fasta(path, records, width=60, newline=b"\n"):
    with open(path, "wb") as f:
        for hdr, seq in records:
            f.write(b">" + hdr + newline)
            for k in range(0, len(seq), width):
                f.write(seq[k:k + width] + newline)


def generate(path, n, length, n_templates, mut, seed):
    write_fasta(path, reads(n, length, n_templates, mut, seed))
    return path


if __name__ == "__main__":
    a = sys.argv[1:]
    generate(a[5], int(a[0]), int(a[1]), int(a[2]), float(a[3]), int(a[4]))
