// capi.cpp -- in-process C API of libmeshclust.so (used by bench.py and the Python package):
// parse once, keep the dataset, run the GPU pipeline repeatedly on a resident context.
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
void mcl_free(void *ds) { delete (mc::Dataset *)ds; }

// argv: reference-style options without input files (e.g. {"prog","--id","0.90"}).
// upload != 0 re-uploads the sequences.  Writes the .clstr if clstr_path is non-NULL and
// the JSON run summary into stats (cap bytes).  Returns 0, or the driver's exit code.
int mcl_run(void *dsv, mc_ctx *ctx, int argc, char **argv, int upload, const char *clstr_path, char *stats,
            int cap) {
  auto *ds = (mc::Dataset *)dsv;
  try {
    mc::Options opt = mc::parse_options(argc, argv, false);
    opt.quiet = true;
    mc::RunResult rr = mc::run_pipeline(*ds, ctx, opt, upload != 0);
    if (clstr_path) mc::write_clstr(clstr_path, *ds, rr.part);
    std::string js = mc::stats_json(rr, 0, 0);
    if (stats && cap > 0) snprintf(stats, cap, "%s", js.c_str());
    return 0;
  } catch (const mc::Error &e) {
    if (stats && cap > 0) snprintf(stats, cap, "{\"error\": \"%s\"}", e.what());
    return e.code ? e.code : 0;
  } catch (const std::exception &e) {
    if (stats && cap > 0) snprintf(stats, cap, "{\"error\": \"%s\"}", e.what());
    return 1;
  }
}
}
