// fasta.cpp -- see fasta.hpp.
#include "fasta.hpp"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cctype>
#include <cstring>

#include "common.hpp"

namespace mc {

namespace {

// ChromosomeOneDigit::buildCodes (ChromosomeOneDigit.cpp:59-85): A0 C1 G2 T3 and the
// IUPAC ambiguity letters mapped onto one of them; 255 = not in the map.
struct CodeTable {
  uint8_t v[256];
  CodeTable() {
    memset(v, 255, sizeof v);
    v['A'] = 0; v['C'] = 1; v['G'] = 2; v['T'] = 3;
    v['R'] = 2; v['Y'] = 1; v['M'] = 0; v['K'] = 3; v['S'] = 2; v['W'] = 3;
    v['H'] = 1; v['B'] = 3; v['V'] = 0; v['D'] = 3; v['N'] = 1; v['X'] = 2;
  }
};
const CodeTable kCodes;

[[noreturn]] void invalid_nucleotide(char c) {
  throw Error(std::string("Invalid nucleotide: ") + c, 1);
}

struct RawRecord {
  std::string header;
  std::string base;
  bool base_ready = false;
};

}  // namespace

// Chromosome::help(1000000, true) then ChromosomeOneDigit::help().
void process_record(std::string &base, std::vector<int32_t> &out) {
  // toUpperCase (Chromosome.cpp:153-157)
  for (auto &c : base) c = (char)toupper((unsigned char)c);
  // removeN (Chromosome.cpp:162-184): maximal non-N runs; a run that starts on the very last
  // character is never closed (the else-if chain at :166-182).
  std::vector<int32_t> seg;
  const int size = (int)base.size();
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
  // mergeSegments (Chromosome.cpp:190-226); segment->at(0) throws on an empty list.
  // (a 1-base or all-N record has no closed run)
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
      uint8_t v = kCodes.v[(unsigned char)base[i]];
      if (v == 255) invalid_nucleotide(base[i]);
      base[i] = (char)v;
    }
  }
  if (nseg > 0) {  // the skipped intervals: every non-'N' byte is encoded, 'N' stays
    auto outside = [&](int a, int b) {
      for (int i = a; i <= b; i++) {
        char c = base[i];
        if (c != 'N') {
          uint8_t v = kCodes.v[(unsigned char)c];
          if (v == 255) invalid_nucleotide(c);
          base[i] = (char)v;
        }
      }
    };
    outside(0, out[0] - 1);
    for (int k = 0; k + 1 < nseg; k++) outside(out[2 * k + 1] + 1, out[2 * k + 2] - 1);
    outside(out[2 * nseg - 1] + 1, size - 1);
  }
}

namespace {

// Splits a file into records with safe_getline's line semantics (ChromListMaker.cpp:23-47):
// lines end at "\n", "\r\n", a lone "\r", or EOF.
void read_records(const std::string &path, std::vector<RawRecord> &recs) {
  int fd = open(path.c_str(), O_RDONLY);
  if (fd < 0) throw Error("File \"" + path + "\" does not exist", 1);
  struct stat st;
  fstat(fd, &st);
  size_t n = (size_t)st.st_size;
  const char *buf = nullptr;
  if (n > 0) {
    void *m = mmap(nullptr, n, PROT_READ, MAP_PRIVATE, fd, 0);
    if (m == MAP_FAILED) {
      close(fd);
      throw Error("cannot map " + path, 1);
    }
    madvise(m, n, MADV_SEQUENTIAL);
    buf = (const char *)m;
  }
  close(fd);
  if (n == 0) throw Error("input file " + path + " is empty", 1);
  RawRecord *cur = nullptr;
  size_t pos = 0;
  auto on_line = [&](const char *p, size_t len) {
    if (len > 0 && p[0] == '>') {
      recs.emplace_back();
      cur = &recs.back();
      cur->header.assign(p, len);
    } else {
      if (!cur) {
        if (len == 0) return;  // blank lines before the first header
        throw Error("sequence data before the first '>' header in " + path, 1);
      }
      cur->base.append(p, len);
      cur->base_ready = true;
    }
  };
  while (pos < n) {
    const char *p = buf + pos;
    size_t rem = n - pos;
    const char *nl = (const char *)memchr(p, '\n', rem);
    const char *cr = (const char *)memchr(p, '\r', nl ? (size_t)(nl - p) : rem);
    if (cr) {
      on_line(p, (size_t)(cr - p));
      pos = (size_t)(cr - buf) + 1;
      if (pos < n && buf[pos] == '\n') pos++;
    } else if (nl) {
      on_line(p, (size_t)(nl - p));
      pos = (size_t)(nl - buf) + 1;
    } else {
      on_line(p, rem);
      pos = n;
    }
  }
  on_line(buf + n, 0);  // the final empty read at EOF (sets isBaseReady of the last record)
  munmap((void *)buf, n);
}

}  // namespace

void parse_fasta_files(const std::vector<std::string> &files, Dataset &ds, int threads) {
  for (const auto &f : files) {
    std::vector<RawRecord> recs;
    read_records(f, recs);
    const size_t nr = recs.size();
    std::vector<std::vector<int32_t>> segs(nr);
    std::vector<std::string> err(nr);
#pragma omp parallel for schedule(dynamic, 64) num_threads(threads)
    for (size_t i = 0; i < nr; i++) {
      try {
        if (!recs[i].base_ready)
          throw Error("The header and the sequence must be set before calling finalize", 1);
        process_record(recs[i].base, segs[i]);
      } catch (const std::exception &e) {
        err[i] = e.what();
      }
    }
    for (size_t i = 0; i < nr; i++)
      if (!err[i].empty()) throw Error(err[i] + " (record " + recs[i].header + ")", 1);
    uint64_t lsum = 0;
    size_t old = ds.codes.size();
    size_t add = 0;
    for (auto &r : recs) add += r.base.size();
    ds.codes.resize(old + add);
    if (ds.seq_off.empty()) ds.seq_off.push_back(0);
    if (ds.seg_off.empty()) ds.seg_off.push_back(0);
    std::vector<uint64_t> offs(nr + 1, old);
    for (size_t i = 0; i < nr; i++) offs[i + 1] = offs[i] + recs[i].base.size();
#pragma omp parallel for schedule(static) num_threads(threads)
    for (size_t i = 0; i < nr; i++)
      if (!recs[i].base.empty()) memcpy(&ds.codes[offs[i]], recs[i].base.data(), recs[i].base.size());
    for (size_t i = 0; i < nr; i++) {
      ds.headers.push_back(std::move(recs[i].header));
      ds.lengths.push_back(recs[i].base.size());
      lsum += recs[i].base.size();
      ds.seq_off.push_back(offs[i + 1]);
      ds.seg.insert(ds.seg.end(), segs[i].begin(), segs[i].end());
      ds.seg_off.push_back(ds.seg.size() / 2);
    }
    ds.file_count.push_back(nr);
    ds.file_len_sum.push_back(lsum);
  }
}

}  // namespace mc
