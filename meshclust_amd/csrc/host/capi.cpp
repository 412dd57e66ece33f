// capi.cpp -- in-process C API of libmeshclust.so (used by bench.py and the Python package):
// parse once, keep the dataset, run the GPU pipeline repeatedly on a resident context.
#include <chrono>
#include <cstring>
#include <string>
#include <vector>

#include "runner.hpp"

extern "C" {

void *mcl_parse(const char *const *files, int nfiles, int threads, char *err, int errcap) {
  try {
    auto *ds = new mc::Dataset();
    std::vector<std::string> f(files, files + nfiles);
    mc::parse_fasta_files(f, *ds, threads > 0 ? threads : 1);
    return ds;
  } catch (const std::exception &e) {
    if (err && errcap > 0) snprintf(err, errcap, "%s", e.what());
    return nullptr;
  }
}

uint64_t mcl_num_seqs(void *ds) { return ((mc::Dataset *)ds)->size(); }

// Opt-in for a host process that runs many clusterings: keep large freed blocks in the heap
// (runner.cpp tune_host_heap).  Process-global, so never done implicitly by the library.
int mcl_tune_host_heap(void) { return mc::tune_host_heap() ? 1 : 0; }

// Read-only view of a parsed dataset (what the reference's Chromosome objects hold after
// ChromListMaker::makeChromOneDigitList): the concatenated one-digit codes with per-record
// offsets, the [start, end] segment pairs with per-record pair offsets.  Pointers stay valid
// until mcl_free.  Used by the parser parity tests.
void mcl_view(void *dsv, const uint8_t **codes, const uint64_t **seq_off, const int32_t **seg,
              const uint64_t **seg_off) {
  auto *ds = (mc::Dataset *)dsv;
  if (ds->bytes_view.size() != ds->bases()) ds->bytes_view = mc::unpack_codes(*ds);
  *codes = ds->bytes_view.data();
  *seq_off = ds->seq_off.data();
  *seg = ds->seg.data();
  *seg_off = ds->seg_off.data();
}
const char *mcl_header(void *dsv, uint64_t i) {
  const auto *ds = (mc::Dataset *)dsv;
  return i < ds->size() ? ds->headers.c_str(i) : nullptr;
}
void mcl_free(void *ds) { delete (mc::Dataset *)ds; }

// Error text as a JSON string literal body (quotes, backslashes and control bytes escaped).
static std::string json_escape(const char *m) {
  std::string o;
  for (const char *c = m; *c; c++) {
    const unsigned char u = (unsigned char)*c;
    if (u == '"' || u == '\\') {
      o += '\\';
      o += (char)u;
    } else if (u < 0x20) {
      char b[8];
      snprintf(b, sizeof b, "\\u%04x", u);
      o += b;
    } else {
      o += (char)u;
    }
  }
  return o;
}

static void put_error(char *stats, int cap, const char *what, int code) {
  if (stats && cap > 0) snprintf(stats, cap, "{\"error\": \"%s\", \"exit_code\": %d}", json_escape(what).c_str(), code);
}

// argv: reference-style options without input files (e.g. {"prog","--id","0.90"}).
// upload != 0 re-uploads the sequences.  Writes the .clstr if clstr_path is non-NULL and
// the JSON run summary into stats (cap bytes).  Returns 0, or the driver's exit code; an
// error never ends the calling process.  The reference's exit(0) stops ("Identity value does
// not match sampled data", Trainer.cpp:306-315) return 0 with {"error": ..., "exit_code": 0}
// in stats and no partition, so a caller must check for "error" (Dataset.run raises).
static int run_common(void *dsv, mc_ctx *ctx, int argc, char **argv, int upload, const char *clstr_path, char *stats,
                      int cap, const mc::ShardComm *comm) {
  auto *ds = (mc::Dataset *)dsv;
  try {
    mc::Options opt = mc::parse_options(argc, argv, false);
    opt.quiet = true;
    mc::RunResult rr = mc::run_pipeline(*ds, ctx, opt, upload != 0, comm);
    const auto t1 = std::chrono::steady_clock::now();
    if (clstr_path) mc::write_clstr(clstr_path, *ds, rr.part, opt.threads > 0 ? opt.threads : 1);
    const double write_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t1).count();
    std::string js = mc::stats_json(rr, 0, write_ms);
    if (stats && cap > 0) snprintf(stats, cap, "%s", js.c_str());
    return 0;
  } catch (const mc::Error &e) {
    put_error(stats, cap, e.what(), e.code);
    return e.code;
  } catch (const std::exception &e) {
    put_error(stats, cap, e.what(), 1);
    return 1;
  }
}

int mcl_run(void *dsv, mc_ctx *ctx, int argc, char **argv, int upload, const char *clstr_path, char *stats,
            int cap) {
  return run_common(dsv, ctx, argc, argv, upload, clstr_path, stats, cap, nullptr);
}

// One clustering shared by `world` ranks: each rank calls this with the same
// input and options; `allgather(user, in, bytes, out)` exchanges equal blocks in rank order.
// Every rank ends with the same partition (rank 0 usually writes the .clstr).
int mcl_run_sharded(void *dsv, mc_ctx *ctx, int argc, char **argv, int upload, const char *clstr_path, char *stats,
                    int cap, int rank, int world, int (*allgather)(void *, const void *, uint64_t, void *),
                    void *user) {
  if (world < 1 || rank < 0 || rank >= world || (world > 1 && !allgather)) return 1;
  mc::ShardComm comm;
  comm.rank = rank;
  comm.world = world;
  comm.allgather = allgather;
  comm.user = user;
  return run_common(dsv, ctx, argc, argv, upload, clstr_path, stats, cap, &comm);
}
}
