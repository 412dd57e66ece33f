"""Regenerate the golden fixtures in tests/golden from the reference itself.

Runs ONLY in the build container (it needs oracle/_ref, which is compiled from the
read-only reference sources by oracle/Makefile).  Inputs are either the hand-written
edge-case FASTA committed here (edge.fa) or synthetic FASTA produced by
meshclust_amd.synth (deterministic, so only the generator arguments and a SHA-256 of the
generated file are committed, not the file).  Outputs:

  edge_parse.json          ChromListMaker/Chromosome/ChromosomeOneDigit per record
  edge_hist.npz            fill_table + KmerHashTable histograms (k = 1, 3, 4, 6)
  nw.npz                   GlobAlignE identity/length/matches/score for many pairs
  train_<name>.npz         Trainer split/labels/feature bounds/weights + per-pair vectors
  e2e_<name>.clstr.gz      meshclust --threads 1 output for the e2e configs
  manifest.json            generator arguments, flags, SHA-256 of generated inputs

Usage: python tests/golden/make_golden.py [--only NAME ...]
"""
import argparse
import gzip
import hashlib
import json
import os
import subprocess
import sys
import tempfile
from concurrent.futures import ThreadPoolExecutor

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
from meshclust_amd import synth  # noqa: E402

REF = os.path.join(ROOT, "oracle", "_ref", "meshclust")
PROBE = os.path.join(ROOT, "oracle", "_ref", "ref_probe")

# name -> (generator args (n, L, T, mut, seed) or variable-length spec, meshclust flags)
E2E = {
    "a1k": ((1000, 500, 20, 0.04, 1), ["--id", "0.90", "--kmer", "3"]),
    "b3k30": ((3000, 1000, 30, 0.03, 11), ["--id", "0.90"]),
    "b3k300": ((3000, 1000, 300, 0.03, 12), ["--id", "0.90"]),
    "m2k_id80": (("mixed", 2000, 40, 0.08, 21), ["--id", "0.80"]),
    "m2k_id95": (("mixed", 2000, 40, 0.02, 22), ["--id", "0.95", "--delta", "3", "--iterations", "5"]),
    "s1k_k5": ((1200, 400, 60, 0.05, 23), ["--id", "0.85", "--kmer", "5"]),
    # 16-bit histograms (k = 1: per-base counts > 255) through the whole pipeline
    "w16_k1": ((800, 1200, 20, 0.05, 24), ["--id", "0.90", "--kmer", "1"]),
    # related templates (families): ambiguous pairs, many merges
    "fam2k": (("family", 2000, 50, 10, 0.10, 0.03, 25), ["--id", "0.90"]),
    "fam2k_id85": (("family", 2000, 40, 8, 0.12, 0.04, 26), ["--id", "0.85", "--delta", "8"]),
    # two clusters of 1,500 members: past the accumulation kernel's member cache
    "big2_3k": ((3000, 1000, 2, 0.03, 75), ["--id", "0.90"]),
    # lower-case, IUPAC, N runs, records < 20 bp (the parser's edge cases end to end)
    "noisy2k": (("noisy", 2000, 40, 0.04, 27), ["--id", "0.90"]),
    # alignment mode (Feature::align classifier; --align, or --id < 0.6 switches it on)
    "al300": ((300, 500, 10, 0.03, 7), ["--align", "--id", "0.9"]),
    "al_fam400_id55": (("family", 400, 16, 4, 0.25, 0.05, 31), ["--id", "0.55"]),
    "al_mix300": (("mixed", 300, 10, 0.08, 32), ["--align", "--id", "0.8", "--delta", "3"]),
    # two input files given out of basename order, with different mean lengths: the basename
    # sort, find_k's per-file integer mean (k = 5 here; the pooled mean would give k = 4) and
    # the ids numbered across files (Runner.cpp:253-262, 265-292)
    "two_files": (("multi", [("zz_long", (300, 2000, 10, 0.03, 81)),
                             ("aa_short", (900, 300, 30, 0.03, 82))]), ["--id", "0.90"]),
}
# Goldens only the GPU tests use (the CPU harness would take as long as the reference):
# config C's shape (100 reads per template, 1 kb, --id 0.55 --align) at 2,000
# reads, and its 0.15-mutation variant whose identities straddle 0.55.
E2E_GPU = {
    "c2k_al55": ((2000, 1000, 20, 0.03, 41), ["--id", "0.55", "--align"]),
    "c2k_m15_al55": ((2000, 1000, 20, 0.15, 41), ["--id", "0.55", "--align"]),
}
TRAIN = {"a1k": ("a1k", 3, 0.90)}


def sha256(path):
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for chunk in iter(lambda: f.read(1 << 20), b""):
            h.update(chunk)
    return h.hexdigest()


def mixed_reads(n, n_templates, mut, seed):
    """Templates of uniform length 700..1300 (exercises many bvec length bins)."""
    rng = np.random.default_rng(seed)
    lens = rng.integers(700, 1301, size=n_templates)
    temps = [rng.integers(0, 4, size=int(l), dtype=np.uint8) for l in lens]
    alpha = np.frombuffer(b"ACGT", dtype=np.uint8)
    p = mut / 3.0
    for i in range(n):
        t = i % n_templates
        s = temps[t]
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
        yield b"read%d template_%d" % (i, t), alpha[base].tobytes()


def family_reads(n, n_templates, n_families, tmut, mut, seed, length=1000):
    """Templates derived from a few family roots (tmut divergence), reads mutated by mut."""
    rng = np.random.default_rng(seed)
    alpha = np.frombuffer(b"ACGT", dtype=np.uint8)
    roots = rng.integers(0, 4, size=(n_families, length), dtype=np.uint8)

    def mutate(s, m):
        p = m / 3.0
        r = rng.random(len(s))
        sub = r < p
        dele = (r >= p) & (r < 2 * p)
        ins = (r >= 2 * p) & (r < m)
        s2 = s.copy()
        s2[sub] = rng.integers(0, 4, size=int(sub.sum()), dtype=np.uint8)
        keep = ~dele
        reps = np.where(ins, 2, 1)[keep]
        base = np.repeat(s2[keep], reps)
        idx = np.cumsum(reps) - 1
        insm = reps == 2
        base[idx[insm]] = rng.integers(0, 4, size=int(insm.sum()), dtype=np.uint8)
        return base

    temps = [mutate(roots[t % n_families], tmut) for t in range(n_templates)]
    for i in range(n):
        t = i % n_templates
        yield b"read%d family_%d template_%d" % (i, t % n_families, t), alpha[mutate(temps[t], mut)].tobytes()


def noisy_reads(n, n_templates, mut, seed, length=1000):
    """Reads with what real FASTA carries: lower-case stretches, IUPAC ambiguity letters,
    short N runs (merged into the segment: N -> C) and long N runs (segment splits, 'N' kept),
    leading/trailing N, and a few records shorter than 20 bp (no segment)."""
    rng = np.random.default_rng(seed)
    base_reads = list(synth.reads(n, length, n_templates, mut, seed))
    iupac = np.frombuffer(b"RYMKSWHBVDX", np.uint8)
    for i, (hdr, seq) in enumerate(base_reads):
        s = bytearray(seq)
        L = len(s)
        if i % 7 == 0:  # lower-case stretch
            a = int(rng.integers(0, L - 50))
            s[a:a + 50] = bytes(s[a:a + 50]).lower()
        if i % 5 == 0:  # IUPAC letters
            for q in rng.integers(0, L, size=3):
                s[int(q)] = int(iupac[int(rng.integers(0, len(iupac)))])
        if i % 11 == 0:  # short N run (< 10: merged)
            a = int(rng.integers(30, L - 40))
            s[a:a + int(rng.integers(1, 9))] = b"N" * len(s[a:a + int(rng.integers(1, 9))])
        if i % 13 == 0:  # long N run (>= 10: split, 'N' kept outside segments)
            a = int(rng.integers(30, L - 60))
            s[a:a + 25] = b"N" * 25
        if i % 17 == 0:  # leading / trailing N
            s = bytearray(b"NNNN") + s + bytearray(b"nn")
        if i % 97 == 0:  # shorter than 20: no segment, pseudocount-only histogram
            s = s[:15]
        yield hdr, bytes(s)


def multi_paths(spec, path):
    """Files of a ("multi", [(basename, spec), ...]) input, in command-line order."""
    d = path[:-3] + "_files"
    return [os.path.join(d, b + ".fa") for b, _ in spec[1]]


def make_input(spec, path):
    if spec[0] == "multi":
        # one FASTA per part; headers prefixed with the part's basename so they stay unique
        h = hashlib.sha256()
        for (b, sub), fp in zip(spec[1], multi_paths(spec, path)):
            os.makedirs(os.path.dirname(fp), exist_ok=True)
            synth.write_fasta(fp, ((b.encode() + b"_" + hdr, seq) for hdr, seq in synth.reads(*sub)))
            h.update(sha256(fp).encode())
        return h.hexdigest()
    if spec[0] == "noisy":
        _, n, t, mut, seed = spec
        synth.write_fasta(path, noisy_reads(n, t, mut, seed))
        return sha256(path)
    if spec[0] == "family":
        _, n, t, f, tmut, mut, seed = spec
        synth.write_fasta(path, family_reads(n, t, f, tmut, mut, seed))
        return sha256(path)
    if spec[0] == "mixed":
        _, n, t, mut, seed = spec
        synth.write_fasta(path, mixed_reads(n, t, mut, seed))
    else:
        synth.generate(path, *spec)
    return sha256(path)


def run_probe(*args):
    with tempfile.NamedTemporaryFile("r", suffix=".txt", delete=False) as tf:
        out = tf.name
    subprocess.run([PROBE, out] + [str(a) for a in args], check=True,
                   stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    with open(out) as f:
        text = f.read()
    os.unlink(out)
    return text


def long_fasta():
    """One 2.5 Mb record with a run of N (a 2.3 Mb segment: two 1 Mb fragments) and a short one."""
    rng = np.random.default_rng(0)
    seq = bytearray(np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, 2_500_000)].tobytes())
    seq[2_300_000:2_300_050] = b"N" * 50
    return b">long\n" + bytes(seq) + b"\n>short\n" + bytes(seq[:100]) + b"\n"


def crlf_variant(src, dst):
    """edge.fa with mixed line ends: "\r\n", a lone "\r" and "\n" in turn (safe_getline,
    ChromListMaker.cpp:23-47), plus a blank "\r\n" line."""
    with open(src, "rb") as f:
        lines = f.read().split(b"\n")
    ends = (b"\r\n", b"\r", b"\n")
    out = b"".join(l + ends[i % 3] for i, l in enumerate(lines[:-1]) if l) + b"\r\n"
    with open(dst, "wb") as f:
        f.write(out)


def parse_records(fa):
    text = run_probe("parse", fa)
    recs = []
    cur = None
    for line in text.splitlines():
        tag, _, rest = line.partition(" ")
        if tag == "R":
            i, length, nseg = map(int, rest.split())
            cur = {"length": length, "nseg": nseg}
            recs.append(cur)
        elif tag == "H":
            cur["header"] = rest
        elif tag == "S":
            v = list(map(int, rest.split())) if rest.strip() else []
            cur["segments"] = [v[k:k + 2] for k in range(0, len(v), 2)]
        elif line.startswith("S"):
            cur["segments"] = []
        elif tag == "D":
            cur["data_hex"] = rest.strip()
    return recs


def golden_parse():
    recs = parse_records(os.path.join(HERE, "edge.fa"))
    with open(os.path.join(HERE, "edge_parse.json"), "w") as f:
        json.dump(recs, f, indent=1)
    # a 2.5 Mb record (makeSegmentList's 1 Mb fragments): segments and a digest of the codes
    with tempfile.TemporaryDirectory() as td:
        fa = os.path.join(td, "long.fa")
        with open(fa, "wb") as f:
            f.write(long_fasta())
        long_recs = parse_records(fa)
    for r in long_recs:
        r["codes_sha256"] = hashlib.sha256(bytes.fromhex(r.pop("data_hex"))).hexdigest()
    with open(os.path.join(HERE, "long_parse.json"), "w") as f:
        json.dump(long_recs, f, indent=1)
    crlf_variant(os.path.join(HERE, "edge.fa"), os.path.join(HERE, "edge_crlf.fa"))
    with open(os.path.join(HERE, "edge_crlf_parse.json"), "w") as f:
        json.dump(parse_records(os.path.join(HERE, "edge_crlf.fa")), f, indent=1)
    hist = {}
    for k in (1, 3, 4, 6):
        text = run_probe("hist", os.path.join(HERE, "edge.fa"), k)
        rows, mags = [], []
        for line in text.splitlines():
            if line.startswith("K "):
                v = list(map(int, line.split()[2:]))
                mags.append(v[0])
                rows.append(v[1:])
        hist["k%d" % k] = np.array(rows, dtype=np.uint64)
        hist["mag%d" % k] = np.array(mags, dtype=np.uint64)
    np.savez_compressed(os.path.join(HERE, "edge_hist.npz"), **hist)


# inputs the reference rejects while reading (Chromosome.cpp:162-258, ChromosomeOneDigit.cpp:95-144)
PARSE_ERRORS = {
    "invalid_nucleotide": b">a\nACGTACGTACGTACGTACGTACGTAC\n>b\nACGTQACGTACGTACGTACGTACGTACGT\n",
    "one_base": b">a\nACGTACGTACGTACGTACGTACGTAC\n>b\nA\n",
    "all_n": b">a\nACGTACGTACGTACGTACGTACGTAC\n>b\nNNNNNNNN\n",
}


def golden_parse_errors(tmp):
    """The reference's exit status and the message of what it throws, per error input."""
    out = {}
    for name, data in PARSE_ERRORS.items():
        fa = os.path.join(tmp, name + ".fa")
        with open(fa, "wb") as f:
            f.write(data)
        r = subprocess.run([REF, fa, "--id", "0.9", "--kmer", "3", "--threads", "1", "--output",
                            os.path.join(tmp, name + ".clstr")], capture_output=True, text=True)
        msg = [l for l in (r.stdout + r.stderr).splitlines() if "Invalid nucleotide" in l or "what():" in l]
        out[name] = {"fasta": data.decode(), "returncode": r.returncode,
                     "message": msg[-1].split("what():")[-1].strip() if msg else None}
    with open(os.path.join(HERE, "parse_errors.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)


def nw_pairs():
    """Pairs covering identical, near, distant, unequal-length, N-containing, tiny inputs."""
    rng = np.random.default_rng(5)
    pairs = []
    def mutate(s, mut):
        out = bytearray()
        for c in s:
            r = rng.random()
            if r < mut / 3:
                out.append(int(rng.integers(0, 4)))
            elif r < 2 * mut / 3:
                continue
            elif r < mut:
                out.append(c)
                out.append(int(rng.integers(0, 4)))
            else:
                out.append(c)
        return bytes(out)
    for length in (1, 2, 3, 5, 17, 64, 100, 257, 500, 1000):
        for mut in (0.0, 0.03, 0.1, 0.3, 0.6):
            a = bytes(rng.integers(0, 4, size=length, dtype=np.uint8))
            b = mutate(a, mut) or bytes([int(rng.integers(0, 4))])
            pairs.append((a, b))
            pairs.append((b, a))
    for _ in range(40):  # unrelated, unequal lengths
        la, lb = int(rng.integers(1, 700)), int(rng.integers(1, 700))
        pairs.append((bytes(rng.integers(0, 4, size=la, dtype=np.uint8)),
                      bytes(rng.integers(0, 4, size=lb, dtype=np.uint8))))
    for _ in range(20):  # 'N' (78) bytes outside segments and raw ASCII (no segments)
        a = bytearray(rng.integers(0, 4, size=int(rng.integers(20, 300)), dtype=np.uint8))
        b = bytearray(mutate(bytes(a), 0.1))
        for arr in (a, b):
            for _ in range(int(rng.integers(0, 6))):
                arr[int(rng.integers(0, len(arr)))] = 78
        pairs.append((bytes(a), bytes(b)))
    pairs.append((b"GACGCTGTCTGA", b"GACGCTGTCTGA"))
    pairs.append((b"ACGTACGT", bytes([0, 1, 2, 3, 0, 1, 2, 3])))
    a = bytes(rng.integers(0, 4, size=3000, dtype=np.uint8))
    pairs.append((a, mutate(a, 0.05)))
    with tempfile.NamedTemporaryFile("w", suffix=".txt", delete=False) as tf:
        for a, b in pairs:
            tf.write(a.hex() + " " + b.hex() + "\n")
        pf = tf.name
    text = run_probe("nw", pf)
    os.unlink(pf)
    ident, length, ids, score = [], [], [], []
    for line in text.splitlines():
        _, i, l, m, s = line.split()
        ident.append(float.fromhex(i))
        length.append(int(l))
        ids.append(int(m))
        score.append(int(s))
    a_cat = b"".join(a for a, _ in pairs)
    b_cat = b"".join(b for _, b in pairs)
    a_off = np.cumsum([0] + [len(a) for a, _ in pairs]).astype(np.int64)
    b_off = np.cumsum([0] + [len(b) for _, b in pairs]).astype(np.int64)
    np.savez_compressed(os.path.join(HERE, "nw.npz"),
                        a=np.frombuffer(a_cat, np.uint8), a_off=a_off,
                        b=np.frombuffer(b_cat, np.uint8), b_off=b_off,
                        identity=np.array(ident), length=np.array(length, np.int32),
                        ids=np.array(ids, np.int32), score=np.array(score, np.int32))


def golden_train(name, fa, k, ident, npts=40):
    text = run_probe("train", fa, k, ident, 3000, 20, npts)
    sp, lp, ln, fl, fs, fmin, fmax, fc, w, P, DD = [], [], [], [], [], [], [], [], [], [], []
    for line in text.splitlines():
        t = line.split()
        if not t:
            continue
        if t[0] == "SP":
            sp.append((int(t[1]), int(t[2])))
        elif t[0] in ("LP", "LN"):
            (lp if t[0] == "LP" else ln).append((int(t[1]), int(t[2]), float.fromhex(t[3])))
        elif t[0] == "FL":
            fl = [int(x) for x in t[1:]]
        elif t[0] == "FS":
            fs = [int(x) for x in t[1:]]
        elif t[0] == "FMIN":
            fmin = [float.fromhex(x) for x in t[1:]]
        elif t[0] == "FMAX":
            fmax = [float.fromhex(x) for x in t[1:]]
        elif t[0] == "FC":
            fc.append([int(x) for x in t[1:]])
        elif t[0] == "W":
            w = [float.fromhex(x) for x in t[1:]]
        elif t[0] == "P":
            parts = line.split("|")
            head = parts[0].split()
            raw = [float.fromhex(x) for x in head[3:]]
            cache = [float.fromhex(x) for x in parts[1].split()]
            combos = [float.fromhex(x) for x in parts[2].split()]
            tail = parts[3].split()
            P.append((int(head[1]), int(head[2]), raw, cache, combos,
                      float.fromhex(tail[0]), int(tail[1]), int(tail[2])))
        elif t[0] == "DD":
            DD.append([float.fromhex(x) for x in t[2:]])
    ncombo = max(len(c) for c in fc)
    combos_arr = np.full((len(fc), ncombo), -1, np.int32)
    for i, c in enumerate(fc):
        combos_arr[i, :len(c)] = c
    np.savez_compressed(
        os.path.join(HERE, "train_%s.npz" % name),
        split_pairs=np.array(sp, np.int64), pos=np.array(lp), neg=np.array(ln),
        lookup=np.array(fl, np.int32), is_sim=np.array(fs, np.int32),
        mins=np.array(fmin), maxs=np.array(fmax), combos=combos_arr, weights=np.array(w),
        pair_ij=np.array([(p[0], p[1]) for p in P], np.int32),
        raw=np.array([p[2] for p in P]), cache=np.array([p[3] for p in P]),
        combo_vals=np.array([p[4] for p in P]), sums=np.array([p[5] for p in P]),
        decision=np.array([p[6] for p in P], np.int8),
        distance=np.array([p[7] for p in P], np.uint64), dist_d=np.array(DD),
        k=k, identity=ident)


def golden_e2e(name, spec, flags, tmp):
    fa = os.path.join(tmp, name + ".fa")
    digest = make_input(spec, fa)
    files = multi_paths(spec, fa) if spec[0] == "multi" else [fa]
    out = os.path.join(tmp, name + ".clstr")
    log = subprocess.run([REF] + files + flags + ["--threads", "1", "--output", out],
                         capture_output=True, text=True)
    if log.returncode != 0:
        raise RuntimeError("reference failed on %s: %s" % (name, log.stderr[-2000:]))
    with open(out, "rb") as f, open(os.path.join(HERE, "e2e_%s.clstr.gz" % name), "wb") as raw, \
            gzip.GzipFile(fileobj=raw, mode="wb", mtime=0, filename="") as g:
        g.write(f.read())
    return name, {"generator": list(spec), "flags": flags, "sha256": digest}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", nargs="*")
    args = ap.parse_args()
    want = set(args.only) if args.only else None
    man_path = os.path.join(HERE, "manifest.json")
    manifest = json.load(open(man_path)) if os.path.exists(man_path) else {"e2e": {}}
    manifest["reference_flags"] = "g++ -O3 -march=x86-64-v3 -fopenmp -std=c++11 (oracle/Makefile)"
    with tempfile.TemporaryDirectory() as tmp:
        if want is None or "parse" in want:
            golden_parse()
            golden_parse_errors(tmp)
        if want is None or "nw" in want:
            nw_pairs()
        if want is None or "train" in want:
            for name, (e2e_name, k, ident) in TRAIN.items():
                fa = os.path.join(tmp, e2e_name + "_train.fa")
                make_input(E2E[e2e_name][0], fa)
                golden_train(name, fa, k, ident)
        todo = [("e2e", n, s, f) for n, (s, f) in E2E.items() if want is None or n in want]
        todo += [("e2e_gpu", n, s, f) for n, (s, f) in E2E_GPU.items() if want is not None and n in want]
        results = {}
        with ThreadPoolExecutor(max_workers=6) as ex:
            for (sec, *_), (name, meta) in zip(todo, ex.map(lambda a: golden_e2e(a[1], a[2], a[3], tmp), todo)):
                results.setdefault(sec, {})[name] = meta
    # re-read: make_big_golden.py may have updated the manifest while the reference ran
    fresh = json.load(open(man_path)) if os.path.exists(man_path) else {}
    for key in ("big", "configs"):
        if key in fresh:
            manifest[key] = fresh[key]
    for sec, metas in results.items():
        manifest.setdefault(sec, {}).update(metas)
    with open(man_path, "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
