"""Canonical form of a CD-HIT style .clstr file (ClusterFactory.cpp:495-520 writer).

Member order inside a cluster and cluster order are nondeterministic in the reference's
OpenMP build, so parity compares the partition as a set of clusters, each
cluster being (centre header, frozenset of member headers).  Lengths are checked too.
"""
import gzip


def parse(path_or_text):
    if "\n" in path_or_text:
        text = path_or_text
    else:
        op = gzip.open if path_or_text.endswith(".gz") else open
        with op(path_or_text, "rt") as f:
            text = f.read()
    clusters = []
    cur = None
    for line in text.splitlines():
        if line.startswith(">Cluster"):
            cur = {"centre": None, "members": []}
            clusters.append(cur)
        elif line.strip():
            idx, rest = line.split("\t", 1)
            length, rest = rest.split("nt, ", 1)
            hdr = rest.rsplit("... ", 1)[0] if "... " in rest else rest
            cur["members"].append((hdr, int(length)))
            if line.rstrip().endswith("*"):
                cur["centre"] = hdr
    return clusters


def canonical(path_or_text):
    cl = parse(path_or_text)
    return frozenset((c["centre"], frozenset(c["members"])) for c in cl)


def diff_summary(a, b):
    ca, cb = canonical(a), canonical(b)
    return {"n_a": len(ca), "n_b": len(cb), "only_a": len(ca - cb), "only_b": len(cb - ca)}
