// fasta.hpp -- multi-FASTA ingest with the exact semantics of the reference's
// ChromListMaker::makeChromOneDigitList (src/nonltr/ChromListMaker.cpp:92-120),
// Chromosome::help (src/nonltr/Chromosome.cpp:99-258) and
// ChromosomeOneDigit::encodeNucleotides (src/nonltr/ChromosomeOneDigit.cpp:95-144),
// done in one pass per file with 256-entry tables instead of std::map lookups.
#pragma once
#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

namespace mc {

struct Dataset {
  std::vector<std::string> headers;  // whole header line incl. '>' (ChromListMaker.cpp:100-109)
  std::vector<uint64_t> lengths;     // base.length() incl. N's (ClusterFactory.cpp:1007)
  std::vector<uint8_t> codes;        // one-digit strings, concatenated
  std::vector<uint64_t> seq_off;     // size n+1
  std::vector<int32_t> seg;          // [start,end] pairs, inclusive
  std::vector<uint64_t> seg_off;     // size n+1, in pairs
  std::vector<uint64_t> file_count;  // records per input file
  std::vector<uint64_t> file_len_sum;  // sum of base.size() per file (Runner::find_k)
  size_t size() const { return headers.size(); }
};

// Parses the files in the given order (the caller sorts by basename, Runner.cpp:253-262).
// Throws mc::Error where the reference throws or crashes.
void parse_fasta_files(const std::vector<std::string> &files, Dataset &ds, int threads);

// One record: upper-case, N-segmentation, merge, fragment, encode -- exposed for tests.
void process_record(std::string &base, std::vector<int32_t> &segs);

}  // namespace mc
