"""Reference partitions at the BASELINE.json sizes (config B 100k, config D's shape at 100k,
config E scaled to 9,100 genomes).

Runs ONLY in the build container: the reference (oracle/_ref/meshclust, compiled from the
read-only sources by oracle/Makefile) clusters the synthetic input that meshclust_amd.synth
regenerates deterministically, and the canonical partition is stored compactly:

  cfg_<name>.npz   n, clusters, centres (sorted centre read ids), digest (SHA-256 of the
                   canonical partition, see canonical_digest), and for inputs up to
                   200k reads centre_of[i] = read id of the centre of read i's cluster.

The reference runs with --threads 1: its OpenMP reductions break ties between equal values
in thread-combine order (Trainer.cpp:38-40, 132-134; ClusterFactory.cpp:406-412), and at 100k
reads its 8-thread run differs from its 1-thread run in 3 centres and 2 memberships (measured
here).  The serial order is the reference's defined semantics (first maximum in get_close,
first minimum in get_mean / closest), and the product restates it.  Read ids
come from the synthetic headers (">read{i} template_{t}").

Usage: python tests/golden/make_big_golden.py NAME [--threads T] [--reuse WALL_S]      NAME in BIG
(--reuse: summarise an existing <workdir>/<NAME>.clstr of a reference run that took WALL_S)
"""
import argparse
import hashlib
import json
import os
import subprocess
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
from meshclust_amd import synth  # noqa: E402

REF = os.path.join(ROOT, "oracle", "_ref", "meshclust")

# name -> (synth.generate args (n, L, T, mut, seed), flags): SURVEY.md §8(d)
BIG = {
    "B100k": ((100000, 1000, 1000, 0.03, 41), ["--id", "0.90"]),
    "D1M": ((1000000, 1000, 10000, 0.03, 51), ["--id", "0.90"]),
    # config D's shape (10 reads per template, 10,000 clusters) at a size the serial
    # reference finishes in about an hour
    "D100k": ((100000, 1000, 10000, 0.03, 51), ["--id", "0.90"]),
    # config E scaled (scripts/configs.py E9100): 70 families x 130 genomes of 8-12 kb
    "E9100": (("families", 70, 130, 8000, 12000, 0.05, 0.15, 61), ["--id", "0.80"]),
}


def n_reads(gen):
    return gen[1] * gen[2] if gen[0] == "families" else gen[0]


def make_input(gen, path):
    if gen[0] == "families":
        synth.write_fasta(path, synth.families(*gen[1:]))
    else:
        synth.generate(path, *gen)


def read_id(header):
    """'>read123 template_4' -> 123 ('>genome5221 family_41' -> 5221: the first number)"""
    name = header[1:].split(" ", 1)[0]
    return int(name[len(name.rstrip("0123456789")):])


def clusters_of(clstr_path):
    """[(centre id, [member ids])] from a .clstr (ClusterFactory.cpp:495-520 format)."""
    out, cur = [], None
    with open(clstr_path) as f:
        for line in f:
            if line.startswith(">Cluster"):
                cur = [None, []]
                out.append(cur)
                continue
            if not line.strip():
                continue
            rest = line.split("\t", 1)[1].split("nt, ", 1)[1]
            hdr = rest.rsplit("... ", 1)[0]
            i = read_id(hdr)
            cur[1].append(i)
            if line.rstrip().endswith("*"):
                cur[0] = i
    return out


def canonical_digest(clusters):
    """SHA-256 over the clusters sorted by centre id, each as uint32 [centre, size, sorted
    member ids...]: equal digests <=> equal partitions with equal centres."""
    h = hashlib.sha256()
    # a cluster whose centre is not one of its members prints no '*' (ClusterFactory.cpp:511):
    # centre id 0xffffffff, ordered by its smallest member
    key = [(0xffffffff if c is None else c, min(mem)) for c, mem in clusters]
    for i in sorted(range(len(clusters)), key=lambda i: key[i]):
        c, mem = clusters[i]
        h.update(np.array([key[i][0], len(mem)] + sorted(mem), dtype=np.uint32).tobytes())
    return h.hexdigest()


def summary(clusters, n):
    centres = np.array(sorted(c for c, _ in clusters), dtype=np.uint32)
    out = {"n": n, "clusters": len(clusters), "centres": centres, "digest": canonical_digest(clusters)}
    if n <= 200000:
        centre_of = np.full(n, 0xffffffff, dtype=np.uint32)
        for c, mem in clusters:
            centre_of[np.array(mem, dtype=np.int64)] = c
        out["centre_of"] = centre_of
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("name", choices=sorted(BIG))
    ap.add_argument("--threads", type=int, default=1)
    ap.add_argument("--workdir", default="/tmp/mc_big")
    ap.add_argument("--reuse", type=float, default=None)
    a = ap.parse_args()
    gen, flags = BIG[a.name]
    os.makedirs(a.workdir, exist_ok=True)
    fa = os.path.join(a.workdir, a.name + ".fa")
    if not os.path.exists(fa):
        make_input(gen, fa + ".tmp")
        os.replace(fa + ".tmp", fa)
    out = os.path.join(a.workdir, a.name + ".clstr")
    if a.reuse is not None:
        wall = a.reuse
    else:
        t0 = time.time()
        subprocess.run([REF, fa] + flags + ["--threads", str(a.threads), "--output", out], check=True,
                       stdout=subprocess.DEVNULL)
        wall = time.time() - t0
    s = summary(clusters_of(out), n_reads(gen))
    np.savez_compressed(os.path.join(HERE, "cfg_%s.npz" % a.name), n=s["n"], clusters=s["clusters"],
                        centres=s["centres"], digest=s["digest"],
                        **({"centre_of": s["centre_of"]} if "centre_of" in s else {}))
    man_path = os.path.join(HERE, "manifest.json")
    man = json.load(open(man_path))
    man.setdefault("big", {})[a.name] = {"generator": list(gen), "flags": flags, "threads": a.threads,
                                         "reference_wall_s": round(wall, 1), "clusters": s["clusters"],
                                         "digest": s["digest"]}
    with open(man_path, "w") as f:
        json.dump(man, f, indent=1, sort_keys=True)
    print(json.dumps(man["big"][a.name]))


if __name__ == "__main__":
    main()
