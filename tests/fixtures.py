"""Shared helpers for the parity tests: golden loading, synthetic inputs, simple parsing."""
import functools
import json
import os

import numpy as np

from meshclust_amd import synth

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden")
_LUT = np.full(256, 255, dtype=np.uint8)
for _c, _v in zip(b"ACGT", range(4)):
    _LUT[_c] = _v


def golden(name):
    return os.path.join(GOLDEN, name)


@functools.lru_cache(None)
def manifest():
    with open(golden("manifest.json")) as f:
        return json.load(f)


def edge_records():
    with open(golden("edge_parse.json")) as f:
        return json.load(f)


def synth_records(n, length, n_templates, mut, seed):
    """(header, codes uint8, length) for pure-ACGT synthetic reads: one segment each."""
    out = []
    for hdr, seq in synth.reads(n, length, n_templates, mut, seed):
        out.append((b">" + hdr, _LUT[np.frombuffer(seq, np.uint8)], len(seq)))
    return out


def e2e_input(name, tmpdir):
    """Regenerate the FASTA of an e2e golden and check its SHA-256 against the manifest."""
    import hashlib
    import importlib.util
    man = manifest()
    spec = man["e2e"][name] if name in man["e2e"] else man["e2e_gpu"][name]
    path = os.path.join(str(tmpdir), name + ".fa")
    gen = spec["generator"]
    mg = importlib.util.spec_from_file_location("make_golden", golden("make_golden.py"))
    mod = importlib.util.module_from_spec(mg)
    mg.loader.exec_module(mod)
    if gen[0] == "multi":
        # several input files: the first is returned as the input, the others lead the flags
        gen = ("multi", [(b, tuple(s)) for b, s in gen[1]])
        h = mod.make_input(gen, path)
        files = mod.multi_paths(gen, path)
        assert h == spec["sha256"], "synthetic generator drifted for %s" % name
        return files[0], files[1:] + spec["flags"]
    mod.make_input(tuple(gen), path)
    h = hashlib.sha256(open(path, "rb").read()).hexdigest()
    assert h == spec["sha256"], "synthetic generator drifted for %s" % name
    return path, spec["flags"]
