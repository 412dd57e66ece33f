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
