// fasta.cpp -- see fasta.hpp.
//
// One pass per file, in parallel: the mapped file is cut into chunks at record starts (a '>'
// at the start of a line), each thread splits its chunk into records with safe_getline's
// line semantics, runs Chromosome::help + encodeNucleotides on every record in place and
// packs the codes; the chunks are then stitched together with prefix sums.
#include "fasta.hpp"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <immintrin.h>

#include <algorithm>
#include <string>
#include <mutex>
#include <memory>
#include <malloc.h>
#include <cerrno>
#include <atomic>
#include <chrono>
#include <cctype>
#include <cstring>
#include <exception>

#include "common.hpp"

namespace mc {

namespace {

// ChromosomeOneDigit::buildCodes (ChromosomeOneDigit.cpp:59-85): A0 C1 G2 T3 and the
// IUPAC ambiguity letters mapped onto one of them; 255 = not in the map.
struct CodeTable {
  uint8_t v[256];
  uint8_t up[256];  // toupper (Chromosome::toUpperCase, Chromosome.cpp:153-157)
  CodeTable() {
    memset(v, 255, sizeof v);
    v['A'] = 0; v['C'] = 1; v['G'] = 2; v['T'] = 3;
    v['R'] = 2; v['Y'] = 1; v['M'] = 0; v['K'] = 3; v['S'] = 2; v['W'] = 3;
    v['H'] = 1; v['B'] = 3; v['V'] = 0; v['D'] = 3; v['N'] = 1; v['X'] = 2;
    for (int c = 0; c < 256; c++) up[c] = (uint8_t)toupper(c);
  }
};
const CodeTable kCodes;

[[noreturn]] void invalid_nucleotide(uint8_t c) {
  throw Error(std::string("Invalid nucleotide: ") + (char)c, 1);
}

}  // namespace

// Chromosome::help(1000000, true) then ChromosomeOneDigit::help().
void process_record(uint8_t *base, size_t usize, std::vector<int32_t> &out) {
  const int size = (int)usize;
  // toUpperCase (Chromosome.cpp:153-157)
  for (int i = 0; i < size; i++) base[i] = kCodes.up[base[i]];
  // removeN (Chromosome.cpp:162-184): maximal non-N runs; a run that starts on the very last
  // character is never closed (the else-if chain at :166-182).
  std::vector<int32_t> seg;
  int start = -1;
  for (int i = 0; i < size; i++) {
    if (base[i] != 'N' && start == -1) {
      start = i;
    } else if (base[i] == 'N' && start != -1) {
      seg.push_back(start);
      seg.push_back(i - 1);
      start = -1;
    } else if (i == size - 1 && base[i] != 'N' && start != -1) {
      seg.push_back(start);
      seg.push_back(i);
      start = -1;
    }
  }
  // mergeSegments (Chromosome.cpp:190-226); segment->at(0) throws on an empty list
  // (a 1-base or all-N record has no closed run).
  if (seg.empty()) throw Error("vector::_M_range_check: __n (which is 0) >= this->size() (which is 0)", 1);
  std::vector<int32_t> merged;
  int s = seg[0], e = seg[1];
  for (size_t i = 2; i < seg.size(); i += 2) {
    int s1 = seg[i], e1 = seg[i + 1];
    if (s1 - e < 10) {
      e = e1;
    } else {
      if (e - s + 1 >= 20) { merged.push_back(s); merged.push_back(e); }
      s = s1;
      e = e1;
    }
  }
  if (e - s + 1 >= 20) { merged.push_back(s); merged.push_back(e); }
  // makeSegmentList (Chromosome.cpp:228-258), segLength = 1,000,000
  const int segLength = 1000000;
  out.clear();
  for (size_t i = 0; i < merged.size(); i += 2) {
    int ss = merged[i], ee = merged[i + 1];
    if (ee - ss + 1 > segLength) {
      int fragNum = (ee - ss + 1) / segLength;
      for (int h = 0; h < fragNum; h++) {
        int fs = ss + h * segLength;
        int fe = (h == fragNum - 1) ? ee : fs + segLength - 1;
        out.push_back(fs);
        out.push_back(fe);
      }
    } else {
      out.push_back(ss);
      out.push_back(ee);
    }
  }
  // encodeNucleotides (ChromosomeOneDigit.cpp:95-144)
  const int nseg = (int)out.size() / 2;
  for (int k = 0; k < nseg; k++) {
    for (int i = out[2 * k]; i <= out[2 * k + 1]; i++) {
      uint8_t v = kCodes.v[base[i]];
      if (v == 255) invalid_nucleotide(base[i]);
      base[i] = v;
    }
  }
  if (nseg > 0) {  // the skipped intervals: every non-'N' byte is encoded, 'N' stays
    auto outside = [&](int a, int b) {
      for (int i = a; i <= b; i++) {
        uint8_t c = base[i];
        if (c != 'N') {
          uint8_t v = kCodes.v[c];
          if (v == 255) invalid_nucleotide(c);
          base[i] = v;
        }
      }
    };
    outside(0, out[0] - 1);
    for (int k = 0; k + 1 < nseg; k++) outside(out[2 * k + 1] + 1, out[2 * k + 2] - 1);
    outside(out[2 * nseg - 1] + 1, size - 1);
  }
}

namespace {

// One chunk of a file: whole records, parsed, encoded and packed.
struct Chunk {
  struct Rec {
    size_t hdr, hdr_len;  // header line in the mapped file
    size_t off, len;      // chunk-local byte offset and length of the one-digit string
    uint64_t w_off;       // chunk-local first word in `pk`
    bool ready;           // isBaseReady: some line followed the header (or EOF did)
  };
  std::vector<Rec> recs;
  std::vector<uint32_t> pk;       // packed words, records word-aligned
  std::vector<int32_t> seg;
  std::vector<uint64_t> nseg;     // segment pairs per record
  std::vector<uint64_t> exc_pos;  // chunk-local byte positions
  std::vector<uint8_t> exc_val;
  uint64_t bytes = 0;
  std::string err;
};

// A/C/G/T in either case -> 0..3 (a record made only of these needs no segmentation work:
// one N-free run, encodeNucleotides maps every byte); everything else -> 255
struct FastTable {
  uint8_t v[256];
  FastTable() {
    memset(v, 255, sizeof v);
    v['A'] = v['a'] = 0;
    v['C'] = v['c'] = 1;
    v['G'] = v['g'] = 2;
    v['T'] = v['t'] = 3;
  }
};
const FastTable kFast;

// A record of plain bases (A/C/G/T in either case) -> 2-bit words appended to pk (base j of
// the record at bits 2*(j % 16) of word j / 16).  32 bases per AVX2 step: the code of a byte
// is ((c >> 1) ^ (c >> 2)) & 3 (A/a C/c G/g T/t -> 0 1 2 3); the byte is plain iff c | 0x20
// equals "acgt"[code]; pext gathers the 2-bit fields.  False (pk unchanged) if some byte is
// not plain.
bool encode_plain(const uint8_t *b, size_t L, std::vector<uint32_t> &pk) {
  const size_t w0 = pk.size();
  pk.resize(w0 + (L + 15) / 16);
  uint32_t *out = pk.data() + w0;
  const __m256i lower = _mm256_set1_epi8(0x20), three = _mm256_set1_epi8(3);
  const __m256i tbl = _mm256_setr_epi8('a', 'c', 'g', 't', 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,  //
                                       'a', 'c', 'g', 't', 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0);
  size_t i = 0;
  for (; i + 32 <= L; i += 32) {
    const __m256i v = _mm256_loadu_si256(reinterpret_cast<const __m256i *>(b + i));
    const __m256i c = _mm256_and_si256(_mm256_xor_si256(_mm256_srli_epi16(v, 1), _mm256_srli_epi16(v, 2)), three);
    const __m256i ok = _mm256_cmpeq_epi8(_mm256_shuffle_epi8(tbl, c), _mm256_or_si256(v, lower));
    if ((uint32_t)_mm256_movemask_epi8(ok) != 0xffffffffu) {
      pk.resize(w0);
      return false;
    }
    alignas(32) uint64_t q[4];
    _mm256_store_si256(reinterpret_cast<__m256i *>(q), c);
    const uint64_t m = 0x0303030303030303ull;
    out[i / 16] = (uint32_t)(_pext_u64(q[0], m) | (_pext_u64(q[1], m) << 16));
    out[i / 16 + 1] = (uint32_t)(_pext_u64(q[2], m) | (_pext_u64(q[3], m) << 16));
  }
  uint32_t acc = 0;
  int sh = 0;
  for (; i < L; i++) {
    const uint32_t v = kFast.v[b[i]];
    if (v > 3) {
      pk.resize(w0);
      return false;
    }
    acc |= v << sh;
    sh += 2;
    if (sh == 32) {
      out[i / 16] = acc;
      acc = 0;
      sh = 0;
    }
  }
  if (sh) out[(L - 1) / 16] = acc;
  return true;
}

inline bool line_start(const char *buf, size_t i) { return i == 0 || buf[i - 1] == '\n' || buf[i - 1] == '\r'; }

// Calls on_line(pos, len) for the lines of buf[a, z) with safe_getline's semantics
// (ChromListMaker.cpp:23-47): lines end at "\n", "\r\n", a lone "\r", or the end.
template <class F>
inline void for_lines(const char *buf, size_t a, size_t z, F &&on_line) {
  size_t pos = a;
  while (pos < z) {
    const char *p = buf + pos;
    const size_t rem = z - pos;
    const char *nl = (const char *)memchr(p, '\n', rem);
    const char *cr = (const char *)memchr(p, '\r', nl ? (size_t)(nl - p) : rem);
    if (cr) {
      on_line(pos, (size_t)(cr - p));
      pos = (size_t)(cr - buf) + 1;
      if (pos < z && buf[pos] == '\n') pos++;
    } else if (nl) {
      on_line(pos, (size_t)(nl - p));
      pos = (size_t)(nl - buf) + 1;
    } else {
      on_line(pos, rem);
      pos = z;
    }
  }
}

// Chromosome::help's segments for an N-free record of length L >= 20 (removeN: one run
// [0, L-1]; mergeSegments keeps it; makeSegmentList: 1 Mb fragments, Chromosome.cpp:228-258)
inline void plain_segments(int64_t L, std::vector<int32_t> &seg) {
  const int64_t segLength = 1000000;
  if (L > segLength) {
    const int64_t fragNum = L / segLength;
    for (int64_t h = 0; h < fragNum; h++) {
      seg.push_back((int32_t)(h * segLength));
      seg.push_back((int32_t)(h == fragNum - 1 ? L - 1 : h * segLength + segLength - 1));
    }
  } else {
    seg.push_back(0);
    seg.push_back((int32_t)(L - 1));
  }
}

// Records of buf[a, z): a line starting with '>' opens a record whose header is the whole
// line; other lines are appended to the current record.  `eof`: the chunk ends the file (the
// final empty read sets isBaseReady of the last record).  A record's lines are gathered, then
// plain records (A/C/G/T only, at least 20 bases: one N-free segment) are packed by
// encode_plain; any other record goes through process_record.  A chunk without '\r' splits
// lines at '\n' alone.
void parse_chunk(const char *buf, size_t a, size_t z, bool first, bool eof, const std::string &path, Chunk &ck) {
  Chunk::Rec *cur = nullptr;
  std::vector<uint8_t> tmp;
  std::vector<int32_t> segs;
  auto close = [&]() {
    if (!cur) return;
    auto &r = *cur;
    r.off = ck.bytes;
    r.len = tmp.size();
    ck.bytes += r.len;
    if (r.len >= 20 && encode_plain(tmp.data(), tmp.size(), ck.pk)) {
      const size_t s0 = ck.seg.size();
      plain_segments((int64_t)r.len, ck.seg);
      ck.nseg.push_back((ck.seg.size() - s0) / 2);
    } else {
      if (!r.ready) throw Error("The header and the sequence must be set before calling finalize", 1);
      process_record(tmp.data(), tmp.size(), segs);
      ck.seg.insert(ck.seg.end(), segs.begin(), segs.end());
      ck.nseg.push_back(segs.size() / 2);
      for (size_t j = 0; j < tmp.size(); j += 16) {
        uint32_t x = 0;
        for (size_t t = 0; t < 16 && j + t < tmp.size(); t++) {
          const uint8_t c = tmp[j + t];
          x |= (uint32_t)(c & 3) << (2 * t);
          if (c > 3) {
            ck.exc_pos.push_back(r.off + j + t);
            ck.exc_val.push_back(c);
          }
        }
        ck.pk.push_back(x);
      }
    }
    tmp.clear();
    cur = nullptr;
  };
  auto on_line = [&](size_t p, size_t len) {
    if (len > 0 && buf[p] == '>') {
      close();
      ck.recs.push_back({p, len, 0, 0, (uint64_t)ck.pk.size(), false});
      cur = &ck.recs.back();
      return;
    }
    if (!cur) {
      if (len == 0) return;  // blank lines before the first header
      if (first) throw Error("sequence data before the first '>' header in " + path, 1);
      throw Error("internal: chunk does not start at a record", 1);
    }
    tmp.insert(tmp.end(), buf + p, buf + p + len);
    cur->ready = true;
  };
  if (memchr(buf + a, '\r', z - a)) {
    for_lines(buf, a, z, on_line);
  } else {
    for (size_t pos = a; pos < z;) {
      const char *nl = (const char *)memchr(buf + pos, '\n', z - pos);
      const size_t e = nl ? (size_t)(nl - buf) : z;
      on_line(pos, e - pos);
      pos = e + 1;
    }
  }
  if (cur && eof) cur->ready = true;
  close();
}

// The same for a chunk with no '\r' (lines end at '\n' alone), without copying a plain record's
// lines into one buffer first: each record's sequence bytes are classified 32 at a time (the
// '\n' bytes dropped, every other byte A/C/G/T in either case) and their 2-bit codes gathered
// straight into the record's packed words (pext over each 8-byte group, the newline bytes left
// out of its mask).  A record with any other byte, or shorter than 20 bases, is handed to
// parse_chunk's path (its lines gathered, process_record).  Records, headers, lengths, segments
// and packed words are exactly parse_chunk's.
void parse_chunk_lf(const char *buf, size_t a, size_t z, bool first, bool eof, const std::string &path, Chunk &ck) {
  // ck.pk's words [0, np) are this chunk's so far; the vector is kept at least as long (and is
  // cut to np at the end), so the packed words of a plain record are stored without a bounds
  // check per word
  size_t np = ck.pk.size();
  ck.pk.resize(np + (z - a) / 16 + 64);
  std::vector<uint8_t> tmp;
  std::vector<uint32_t> fb;
  std::vector<int32_t> segs;
  const __m256i lower = _mm256_set1_epi8(0x20), three = _mm256_set1_epi8(3), nlv = _mm256_set1_epi8('\n'),
                gtv = _mm256_set1_epi8('>');
  const __m256i tbl = _mm256_setr_epi8('a', 'c', 'g', 't', 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,  //
                                       'a', 'c', 'g', 't', 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0);
  const uint64_t M8 = 0x0303030303030303ull;
  size_t pos = a;
  // lines before the first header: blank ones are skipped, anything else is an error
  while (pos < z && buf[pos] != '>') {
    const char *nl = (const char *)memchr(buf + pos, '\n', z - pos);
    const size_t e = nl ? (size_t)(nl - buf) : z;
    if (e > pos) {
      if (first) throw Error("sequence data before the first '>' header in " + path, 1);
      throw Error("internal: chunk does not start at a record", 1);
    }
    pos = e + 1;
  }
  while (pos < z) {
    // the header line [pos, he)
    const char *hn = (const char *)memchr(buf + pos, '\n', z - pos);
    const size_t he = hn ? (size_t)(hn - buf) : z;
    Chunk::Rec r{pos, he - pos, 0, 0, (uint64_t)np, false};
    // the record's lines are [s, t), t = the next '>' at the start of a line (or the chunk's
    // end); t is found in the same pass that classifies and packs the bytes
    const size_t s = he < z ? he + 1 : z;
    size_t t = z, i = s, o = np;
    bool plain = true, found = false;
    uint64_t acc = 0, nb = 0;
    uint32_t fill = 0, carry = 1;  // carry: the byte before block i is '\n' (buf[he] at first)
    for (; i < z; i += 32) {
      const __m256i v = _mm256_loadu_si256(reinterpret_cast<const __m256i *>(buf + i));  // (64 bytes of slack)
      const __m256i c = _mm256_and_si256(_mm256_xor_si256(_mm256_srli_epi16(v, 1), _mm256_srli_epi16(v, 2)), three);
      const uint32_t ok = (uint32_t)_mm256_movemask_epi8(_mm256_cmpeq_epi8(_mm256_shuffle_epi8(tbl, c), _mm256_or_si256(v, lower)));
      const uint32_t nl = (uint32_t)_mm256_movemask_epi8(_mm256_cmpeq_epi8(v, nlv));
      const uint32_t gt = (uint32_t)_mm256_movemask_epi8(_mm256_cmpeq_epi8(v, gtv));
      uint32_t live = z - i >= 32 ? 0xffffffffu : (1u << (z - i)) - 1u;
      const uint32_t st = gt & ((nl << 1) | carry) & live;
      if (st) {
        const uint32_t e = (uint32_t)__builtin_ctz(st);
        live = (1u << e) - 1u;
        t = i + e;
        found = true;
      }
      carry = nl >> 31;
      if (((ok | nl) & live) != live) {
        plain = false;
        break;
      }
      if (o + 4 > ck.pk.size()) ck.pk.resize(2 * ck.pk.size() + 64);
      uint32_t *out = ck.pk.data();
      const uint32_t keep = ok & ~nl & live;
      alignas(32) uint64_t q[4];
      _mm256_store_si256(reinterpret_cast<__m256i *>(q), c);
      // two 16-byte halves: their 2-bit codes (pext of each byte's two low bits), then the
      // kept bytes' codes (pext with the keep mask spread to 2-bit fields) appended to acc
#pragma GCC unroll 2
      for (int h = 0; h < 2; h++) {
        const uint64_t codes = _pext_u64(q[2 * h], M8) | (_pext_u64(q[2 * h + 1], M8) << 16);
        const uint32_t k16 = (keep >> (16 * h)) & 0xffffu;
        const uint64_t bits = _pext_u64(codes, _pdep_u64(k16, 0x55555555ull) * 3u);
        const uint32_t n = (uint32_t)__builtin_popcount(k16);
        acc |= bits << fill;
        fill += 2 * n;
        nb += n;
        out[o] = (uint32_t)acc;
        const uint32_t adv = fill >> 5;
        o += adv;
        acc >>= 32 * adv;
        fill &= 31;
      }
      if (found) break;
    }
    if (!found && i < z && !plain) {
      // a non-plain byte before the record's end was known: find the end as parse_chunk would
      for (t = i;;) {
        const char *g = t < z ? (const char *)memchr(buf + t, '>', z - t) : nullptr;
        if (!g) {
          t = z;
          break;
        }
        t = (size_t)(g - buf);
        if (buf[t - 1] == '\n') break;
        t++;
      }
    }
    r.ready = s < t || (t == z && eof);  // some line followed the header (or the file ended)
    if (plain && nb >= 20) {
      if (fill) ck.pk[o++] = (uint32_t)acc;
      np = o;
      r.off = ck.bytes;
      r.len = nb;
      ck.bytes += nb;
      const size_t s0 = ck.seg.size();
      plain_segments((int64_t)nb, ck.seg);
      ck.nseg.push_back((ck.seg.size() - s0) / 2);
      ck.recs.push_back(r);
    } else {
      // parse_chunk's path for this record: its lines gathered, then encode_plain or
      // process_record, packing into fb; fb is then copied to words [np, ...)
      tmp.clear();
      fb.clear();
      for (size_t u = s; u < t;) {
        const char *nl = (const char *)memchr(buf + u, '\n', t - u);
        const size_t e = nl ? (size_t)(nl - buf) : t;
        tmp.insert(tmp.end(), buf + u, buf + e);
        u = e + 1;
      }
      r.off = ck.bytes;
      r.len = tmp.size();
      ck.bytes += r.len;
      if (r.len >= 20 && encode_plain(tmp.data(), tmp.size(), fb)) {
        const size_t s0 = ck.seg.size();
        plain_segments((int64_t)r.len, ck.seg);
        ck.nseg.push_back((ck.seg.size() - s0) / 2);
      } else {
        if (!r.ready) throw Error("The header and the sequence must be set before calling finalize", 1);
        process_record(tmp.data(), tmp.size(), segs);
        ck.seg.insert(ck.seg.end(), segs.begin(), segs.end());
        ck.nseg.push_back(segs.size() / 2);
        for (size_t j = 0; j < tmp.size(); j += 16) {
          uint32_t x = 0;
          for (size_t u = 0; u < 16 && j + u < tmp.size(); u++) {
            const uint8_t cc = tmp[j + u];
            x |= (uint32_t)(cc & 3) << (2 * u);
            if (cc > 3) {
              ck.exc_pos.push_back(r.off + j + u);
              ck.exc_val.push_back(cc);
            }
          }
          fb.push_back(x);
        }
      }
      ck.recs.push_back(r);
      if (np + fb.size() + 4 > ck.pk.size()) ck.pk.resize(std::max(2 * ck.pk.size(), np + fb.size() + 64));
      if (!fb.empty()) memcpy(ck.pk.data() + np, fb.data(), fb.size() * sizeof(uint32_t));
      np += fb.size();
    }
    pos = t;
  }
  ck.pk.resize(np);
}

}  // namespace

void parse_fasta_files(const std::vector<std::string> &files, Dataset &ds, int threads) {
  if (threads < 1) threads = 1;
  if (ds.seq_off.empty()) {
    ds.seq_off.push_back(0);
    ds.seg_off.push_back(0);
    ds.pk_off.push_back(0);
  }
  for (const auto &path : files) {
    int fd = open(path.c_str(), O_RDONLY);
    if (fd < 0) throw Error("File \"" + path + "\" does not exist", 1);
    struct stat st;
    fstat(fd, &st);
    const size_t n = (size_t)st.st_size;
    if (n == 0) {
      close(fd);
      throw Error("input file " + path + " is empty", 1);
    }
    const bool prof = getenv("MC_PARSE_PROFILE") != nullptr;
    auto tp0 = std::chrono::steady_clock::now();
    auto lap = [&](const char *what) {
      if (!prof) return;
      const auto t = std::chrono::steady_clock::now();
      fprintf(stderr, "[parse] %s %.3f ms\n", what, std::chrono::duration<double, std::milli>(t - tp0).count());
      tp0 = t;
    };
    // The file is read into heap memory by parallel preads: the pages come from the page
    // cache as copies, and a repeated parse reuses the heap's already-touched pages (the
    // heap keeps large blocks, see keep_heap), where an mmap pays page-table population and
    // teardown for every file (MAP_POPULATE + munmap: 13 ms of a 30 ms parse of 100 MB).
    std::unique_ptr<char, void (*)(void *)> mem((char *)malloc(n + 64), free);
    if (!mem) {
      close(fd);
      throw Error("cannot allocate " + std::to_string(n) + " bytes for " + path, 1);
    }
    char *wbuf = mem.get();
    memset(wbuf + n, 0, 64);  // (the chunk parsers' 32-byte loads run up to 31 bytes past a chunk)
    const char *buf = wbuf;
    std::atomic<int> bad{0};
    auto read_at = [&](char *dst, size_t off, size_t end) {  // bytes [off, end) of the file
      while (off < end) {
        const ssize_t r = pread(fd, dst, end - off, (off_t)off);
        if (r < 0 && errno == EINTR) continue;
        if (r <= 0) {
          bad = 1;
          return;
        }
        off += (size_t)r;
        dst += r;
      }
    };
    // chunks: the first record start at or after t * n / T.  Each chunk is read by the thread
    // that then parses it, so the parse finds its bytes in that core's cache instead of reading
    // them back from memory after a separate read phase (the cut points come from small probe
    // reads around t * n / T first).
    static const int per_thread = [] {  // MC_PARSE_CHUNKS_PER_THREAD (default 8)
      const char *e = getenv("MC_PARSE_CHUNKS_PER_THREAD");
      const int v = e ? atoi(e) : 8;
      return v < 1 ? 1 : v > 64 ? 64 : v;
    }();
    const int T = (int)std::max<size_t>(1, std::min<size_t>((size_t)threads * per_thread, n / (1 << 16) + 1));
    std::vector<size_t> cut(T + 1, n);
    cut[0] = 0;
#pragma omp parallel for schedule(dynamic, 1) num_threads(threads)
    for (int t = 1; t < T; t++) {
      // first '>' at the start of a line at or after n * t / T (the byte before it read too)
      const size_t c0 = (size_t)((double)n * t / T);
      std::vector<char> win;
      size_t base = c0 - 1, got = 0, i = 1;  // window = file bytes [base, base + got)
      cut[t] = n;
      for (size_t want = 1 << 13; base + got < n; want *= 2) {
        const size_t end = std::min(n, base + got + want);
        win.resize(end - base);
        read_at(win.data() + got, base + got, end);
        if (bad) break;
        got = end - base;
        bool hit = false;
        for (; i < got; i++)
          if (win[i] == '>' && (win[i - 1] == '\n' || win[i - 1] == '\r')) {
            hit = true;
            break;
          }
        if (hit) {
          cut[t] = base + i;
          break;
        }
      }
    }
    if (bad) {
      close(fd);
      throw Error("cannot read " + path, 1);
    }
    lap("cut");
    std::vector<Chunk> ck(T);
    static const bool fast_lf = !getenv("MC_PARSE_LINES");  // (MC_PARSE_LINES=1: parse_chunk only)
#pragma omp parallel for schedule(dynamic, 1) num_threads(threads)
    for (int t = 0; t < T; t++) {
      try {
        if (cut[t] < cut[t + 1]) {
          read_at(wbuf + cut[t], cut[t], cut[t + 1]);
          if (bad) throw Error("cannot read " + path, 1);
          if (fast_lf && !memchr(buf + cut[t], '\r', cut[t + 1] - cut[t]))
            parse_chunk_lf(buf, cut[t], cut[t + 1], t == 0, cut[t + 1] == n, path, ck[t]);
          else
            parse_chunk(buf, cut[t], cut[t + 1], t == 0, cut[t + 1] == n, path, ck[t]);
        }
      } catch (const std::exception &e) {
        ck[t].err = e.what();
      }
    }
    close(fd);
    // the first failing record in file order reports (the reference stops there)
    for (int t = 0; t < T; t++)
      if (!ck[t].err.empty()) throw Error(ck[t].err, 1);
    lap("chunks");
    // stitch: prefix sums over chunks, then parallel copies
    std::vector<uint64_t> rec0(T + 1, ds.size()), byte0(T + 1, ds.bases()), word0(T + 1, ds.pk_off.back()),
        seg0(T + 1, ds.seg.size() / 2), exc0(T + 1, ds.exc_pos.size());
    uint64_t lsum = 0;
    for (int t = 0; t < T; t++) {
      rec0[t + 1] = rec0[t] + ck[t].recs.size();
      byte0[t + 1] = byte0[t] + ck[t].bytes;
      word0[t + 1] = word0[t] + ck[t].pk.size();
      seg0[t + 1] = seg0[t] + ck[t].seg.size() / 2;
      exc0[t + 1] = exc0[t] + ck[t].exc_pos.size();
      lsum += ck[t].bytes;
    }
    const uint64_t nr = rec0[T], nwords = word0[T];
    std::vector<uint64_t> hb0(T + 1, ds.headers.blob.size());  // header bytes (+ NUL) per chunk
    for (int t = 0; t < T; t++) {
      uint64_t b = 0;
      for (const auto &rec : ck[t].recs) b += rec.hdr_len + 1;
      hb0[t + 1] = hb0[t] + b;
    }
    ds.headers.blob.resize(hb0[T]);
    ds.headers.off.resize(nr + 1);
    ds.lengths.resize(nr);
    ds.seq_off.resize(nr + 1);
    ds.pk_off.resize(nr + 1);
    ds.seg_off.resize(nr + 1);
    ds.seg.resize(2 * seg0[T]);
    ds.exc_pos.resize(exc0[T]);
    ds.exc_val.resize(exc0[T]);
    {
      PodArray<uint32_t> grown;
      grown.resize(nwords);
      if (word0[0]) memcpy(grown.data(), ds.packed.data(), word0[0] * 4);
      ds.packed = std::move(grown);
    }
#pragma omp parallel for schedule(dynamic, 1) num_threads(threads)
    for (int t = 0; t < T; t++) {
      const Chunk &c = ck[t];
      uint64_t sg = seg0[t], hb = hb0[t];
      for (size_t r = 0; r < c.recs.size(); r++) {
        const auto &rec = c.recs[r];
        const uint64_t id = rec0[t] + r;
        memcpy(&ds.headers.blob[hb], buf + rec.hdr, rec.hdr_len);
        hb += rec.hdr_len;
        ds.headers.blob[hb++] = '\0';
        ds.headers.off[id + 1] = hb;
        ds.lengths[id] = rec.len;
        ds.seq_off[id + 1] = byte0[t] + rec.off + rec.len;
        ds.pk_off[id + 1] = word0[t] + (r + 1 < c.recs.size() ? c.recs[r + 1].w_off : c.pk.size());
        sg += c.nseg[r];
        ds.seg_off[id + 1] = sg;
      }
      if (!c.pk.empty()) memcpy(ds.packed.data() + word0[t], c.pk.data(), c.pk.size() * 4);
      std::copy(c.seg.begin(), c.seg.end(), ds.seg.begin() + 2 * seg0[t]);
      for (size_t q = 0; q < c.exc_pos.size(); q++) {
        ds.exc_pos[exc0[t] + q] = byte0[t] + c.exc_pos[q];
        ds.exc_val[exc0[t] + q] = c.exc_val[q];
      }
    }
    lap("stitch");
    ds.file_count.push_back(nr - rec0[0]);
    ds.file_len_sum.push_back(lsum);
  }
}

std::vector<uint8_t> unpack_codes(const Dataset &ds) {
  std::vector<uint8_t> out(ds.bases());
  for (size_t i = 0; i < ds.size(); i++) {
    const uint32_t *w = ds.packed.data() + ds.pk_off[i];
    for (uint64_t j = 0; j < ds.lengths[i]; j++) out[ds.seq_off[i] + j] = (uint8_t)((w[j / 16] >> (2 * (j % 16))) & 3);
  }
  for (size_t q = 0; q < ds.exc_pos.size(); q++) out[ds.exc_pos[q]] = ds.exc_val[q];
  return out;
}

}  // namespace mc
