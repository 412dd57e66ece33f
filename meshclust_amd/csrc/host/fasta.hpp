// fasta.hpp -- multi-FASTA ingest with the exact semantics of the reference's
// ChromListMaker::makeChromOneDigitList (src/nonltr/ChromListMaker.cpp:92-120),
// Chromosome::help (src/nonltr/Chromosome.cpp:99-258) and
// ChromosomeOneDigit::encodeNucleotides (src/nonltr/ChromosomeOneDigit.cpp:95-144),
// done in one parallel pass per file with 256-entry tables instead of std::map lookups.
//
// The output is what the device consumes (mc_load_packed): 2-bit codes, 16 bases per 32-bit
// word, every record starting on a word; the bytes a record keeps outside {0..3} (the 'N'
// that encodeNucleotides leaves outside segments) as a sorted exception list.
#pragma once
#include <cstddef>
#include <cstdint>
#include <cstdlib>
#include <memory>
#include <string>
#include <string_view>
#include <vector>

namespace mc {

// Grow-only POD array without value initialisation (the parser fills every element).
template <typename T>
struct PodArray {
  std::unique_ptr<T[]> p;
  size_t n = 0;
  void resize(size_t m) {
    if (m > n || !p) {
      p.reset(new T[m ? m : 1]);
    }
    n = m;
  }
  T *data() { return p.get(); }
  const T *data() const { return p.get(); }
  size_t size() const { return n; }
  T &operator[](size_t i) { return p[i]; }
  const T &operator[](size_t i) const { return p[i]; }
};

// Every header in one buffer (each followed by a NUL): two allocations for any number of
// records, so a dataset is freed in microseconds (100k std::strings allocated by the parse's
// threads took milliseconds to free from another thread's arena).
struct Headers {
  std::string blob;
  std::vector<uint64_t> off{0};  // size n+1: header i is blob[off[i], off[i+1] - 1)
  size_t size() const { return off.size() - 1; }
  std::string_view operator[](size_t i) const { return std::string_view(blob.data() + off[i], off[i + 1] - off[i] - 1); }
  const char *c_str(size_t i) const { return blob.data() + off[i]; }
};

struct Dataset {
  Headers headers;                   // whole header line incl. '>' (ChromListMaker.cpp:100-109)
  std::vector<uint64_t> lengths;     // base.length() incl. N's (ClusterFactory.cpp:1007)
  std::vector<uint64_t> seq_off;     // size n+1: byte offsets of the concatenated one-digit strings
  PodArray<uint32_t> packed;         // 2-bit codes, base j of a record at bits 2*(j%16) of word j/16
  std::vector<uint64_t> pk_off;      // size n+1: first word of each record in `packed`
  std::vector<uint64_t> exc_pos;     // global byte positions whose one-digit byte is not 0..3
  std::vector<uint8_t> exc_val;      // ... and that byte (78, 'N', outside segments)
  std::vector<int32_t> seg;          // [start,end] pairs, inclusive
  std::vector<uint64_t> seg_off;     // size n+1, in pairs
  std::vector<uint64_t> file_count;  // records per input file
  std::vector<uint64_t> file_len_sum;  // sum of base.size() per file (Runner::find_k)
  std::vector<uint8_t> bytes_view;     // unpack_codes(), filled on demand (mcl_view)
  size_t size() const { return headers.size(); }
  uint64_t bases() const { return seq_off.empty() ? 0 : seq_off.back(); }
};

// Parses the files in the given order (the caller sorts by basename, Runner.cpp:253-262).
// Throws mc::Error where the reference throws or crashes.
void parse_fasta_files(const std::vector<std::string> &files, Dataset &ds, int threads);

// The one-digit bytes of every record, concatenated (what ChromosomeOneDigit::getBase holds):
// unpacked from `packed` + the exceptions.  For tests and the byte-level ABI.
std::vector<uint8_t> unpack_codes(const Dataset &ds);

// One record in place: upper-case, N-segmentation, merge, fragment, encode -- exposed for tests.
void process_record(uint8_t *base, size_t size, std::vector<int32_t> &segs);

}  // namespace mc
