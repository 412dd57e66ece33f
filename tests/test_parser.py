"""The product's FASTA ingest (meshclust_amd/csrc/host/fasta.cpp) against the reference's own
parse of the same files (tests/golden/edge_parse.json, edge_crlf_parse.json and
parse_errors.json, written by make_golden.py from oracle/_ref).

Reference behaviour covered: ChromListMaker::makeChromOneDigitList's record split with the
whole header line (ChromListMaker.cpp:92-120) and safe_getline's "\\n" / "\\r\\n" / lone "\\r"
line ends (:23-47); Chromosome::help's upper-casing, N-run segments, merging of gaps < 10,
dropping of segments < 20 and 1 Mb fragments (Chromosome.cpp:99-258); ChromosomeOneDigit's
IUPAC map, N -> C inside segments, 'N' kept outside (ChromosomeOneDigit.cpp:59-144); and
the reference's failures: an invalid nucleotide, a 1-base record and an all-N record.
No GPU is needed: only the host library's parser runs.
"""
import json

import numpy as np
import pytest

import fixtures
import meshclust_amd as M


@pytest.fixture(scope="module")
def host_built():
    M.build()


@pytest.mark.parametrize("fa,golden", [("edge.fa", "edge_parse.json"), ("edge_crlf.fa", "edge_crlf_parse.json")])
def test_parse_matches_reference(host_built, fa, golden):
    want = json.load(open(fixtures.golden(golden)))
    got = M.Dataset([fixtures.golden(fa)], threads=2).records()
    assert len(got) == len(want)
    for (hdr, codes, segs), w in zip(got, want):
        assert hdr == w["header"]
        assert len(codes) == w["length"]
        assert segs == w["segments"], hdr
        assert codes.tobytes().hex() == w["data_hex"], hdr


def test_parse_lengths_and_segment_counts(host_built):
    """The reference's segment counts (nseg) and lengths, incl. the record shorter than 20
    (no segment: its histogram is all pseudocounts) and the 1 Mb-free long record."""
    want = json.load(open(fixtures.golden("edge_parse.json")))
    got = M.Dataset([fixtures.golden("edge.fa")], threads=1).records()
    assert [len(s) for _, _, s in got] == [w["nseg"] for w in want]
    assert any(w["nseg"] == 0 for w in want)


def test_long_record_fragments(host_built, tmp_path):
    """makeSegmentList splits segments longer than 1,000,000 into 1 Mb fragments, the last
    one absorbing the remainder (Chromosome.cpp:235-247); reference segments and code digest
    in long_parse.json (make_golden.long_fasta)."""
    import hashlib
    import importlib.util
    mg = importlib.util.spec_from_file_location("make_golden", fixtures.golden("make_golden.py"))
    mod = importlib.util.module_from_spec(mg)
    mg.loader.exec_module(mod)
    p = tmp_path / "long.fa"
    p.write_bytes(mod.long_fasta())
    want = json.load(open(fixtures.golden("long_parse.json")))
    got = M.Dataset([str(p)], threads=2).records()
    assert len(got) == len(want) and len(want[0]["segments"]) >= 2
    for (hdr, codes, segs), w in zip(got, want):
        assert (hdr, len(codes), segs) == (w["header"], w["length"], w["segments"])
        assert hashlib.sha256(codes.tobytes()).hexdigest() == w["codes_sha256"]


@pytest.mark.parametrize("case", ["invalid_nucleotide", "one_base", "all_n"])
def test_parse_errors_match_reference(host_built, tmp_path, case):
    """Inputs the reference aborts on while reading: the product raises with the same message
    (the reference exits through std::terminate; the library reports the error instead)."""
    spec = json.load(open(fixtures.golden("parse_errors.json")))[case]
    assert spec["returncode"] != 0
    p = tmp_path / (case + ".fa")
    p.write_text(spec["fasta"])
    with pytest.raises(M.MCError) as ei:
        M.Dataset([str(p)], threads=1)
    assert spec["message"] in str(ei.value)


_DIFF_SCRIPT = r"""
import hashlib, sys
import meshclust_amd as M
h = hashlib.sha256()
for hdr, codes, segs in M.Dataset([sys.argv[1]], threads=int(sys.argv[2])).records():
    h.update(repr((hdr, segs)).encode()); h.update(codes.tobytes())
print(h.hexdigest())
"""


@pytest.mark.parametrize("seed", [1, 2])
def test_lf_fast_path_matches_line_path(host_built, tmp_path, seed):
    """parse_chunk_lf (records of a '\\r'-free chunk packed straight from the file bytes) gives
    the records of parse_chunk (lines gathered first; pinned by the goldens above, and forced by
    MC_PARSE_LINES=1): random multi-line records of mixed case, N runs, IUPAC codes, blank lines,
    records under 20 bases and line widths that straddle the 32-byte blocks, parsed in many
    chunks."""
    import os
    import subprocess
    import sys
    rng = np.random.default_rng(seed)
    out = []
    for r in range(3000):
        L = int(rng.choice([20, 21, 31, 32, 33, 64, 95, 150, 700, 2000]) + rng.integers(0, 3))
        s = rng.choice(list(b"ACGTacgt"), L).astype(np.uint8)
        kind = rng.integers(0, 8)
        if kind == 0:
            i = int(rng.integers(0, L - 5)); s[i:i + 5] = ord("N")
        elif kind == 1:
            s[int(rng.integers(0, L))] = ord(rng.choice(list("RYKMSWn")))
        seq = s.tobytes()
        w = int(rng.choice([10, 31, 32, 33, 60, 80, 1000]))
        lines = [seq[i:i + w] for i in range(0, len(seq), w)]
        if rng.integers(0, 10) == 0:
            lines.insert(int(rng.integers(0, len(lines) + 1)), b"")
        out.append(b">r%d some text\n" % r + b"\n".join(lines) + (b"\n" if rng.integers(0, 20) else b"\n\n"))
    if seed == 2:
        out[-1] = out[-1].rstrip(b"\n")
    p = tmp_path / "mix.fa"
    p.write_bytes(b"\n" + b"".join(out))
    digest = {}
    for mode in ("fast", "lines"):
        env = dict(os.environ)
        env.pop("MC_PARSE_LINES", None)
        if mode == "lines":
            env["MC_PARSE_LINES"] = "1"
        res = subprocess.run([sys.executable, "-c", _DIFF_SCRIPT, str(p), "8"], env=env, capture_output=True,
                             text=True, check=True, cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        digest[mode] = res.stdout.strip()
    assert digest["fast"] == digest["lines"]


def test_chunking_independent(host_built, tmp_path):
    """The file is cut at record starts into threads x MC_PARSE_CHUNKS_PER_THREAD chunks, each
    read by the thread that parses it: one chunk and 8 x 16 chunks give the same records, with
    records that span many chunks (300 kb among 1 kb ones), CRLF and LF records, and cut points
    that land inside headers, sequence lines and blank lines."""
    import os
    import subprocess
    import sys
    rng = np.random.default_rng(7)
    out = []
    for r in range(600):
        L = int(rng.choice([25, 999, 1000, 1001, 5000, 300000], p=[0.1, 0.3, 0.3, 0.2, 0.08, 0.02]))
        seq = rng.choice(list(b"ACGTN"), L, p=[0.24, 0.25, 0.25, 0.25, 0.01]).astype(np.uint8).tobytes()
        nl = b"\r\n" if r % 97 == 5 else b"\n"
        w = int(rng.choice([60, 61, 80]))
        lines = [seq[i:i + w] for i in range(0, len(seq), w)]
        out.append(b">rec%d %s" % (r, b"x" * int(rng.integers(0, 40))) + nl + nl.join(lines) + nl)
    p = tmp_path / "chunks.fa"
    p.write_bytes(b"".join(out))
    assert p.stat().st_size > 2 << 20
    digest = {}
    for threads, per in (("1", "1"), ("8", "16"), ("3", "5")):
        env = dict(os.environ, MC_PARSE_CHUNKS_PER_THREAD=per)
        res = subprocess.run([sys.executable, "-c", _DIFF_SCRIPT, str(p), threads], env=env, capture_output=True,
                             text=True, check=True, cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        digest[(threads, per)] = res.stdout.strip()
    assert len(set(digest.values())) == 1, digest
