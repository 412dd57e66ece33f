// oracle/ref_probe.cpp -- TEST INFRASTRUCTURE ONLY.
//
// Our own driver that links the unmodified MeShClust v1 reference objects (built by
// oracle/Makefile from /root/reference/src, never copied) and dumps per-function golden
// vectors for tests/golden.  It calls the reference's own functions:
//   parse : ChromListMaker::makeChromOneDigitList   (src/nonltr/ChromListMaker.cpp:92-120)
//   hist  : fill_table + KmerHashTable              (src/cluster/src/ClusterFactory.h:40-55)
//   train : Trainer<T>::split/get_labels/train      (src/cluster/src/Trainer.cpp:253-783)
//           then Feature::compute/operator(), DivergencePoint::distance/distance_d on pairs
//   nw    : utility::GlobAlignE(...).getIdentity()  (src/utility/GlobAlignE.cpp:22-305)
// Private members of the reference classes are read through the usual test-probe
// `#define private public` trick (no reference source is modified).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>
#include <fstream>
#include <sstream>
#include <iostream>
#include <algorithm>
#define private public
#define protected public
#include "nonltr/ChromListMaker.h"
#include "nonltr/ChromosomeOneDigit.h"
#include "nonltr/KmerHashTable.h"
#include "cluster/src/ClusterFactory.h"
#include "cluster/src/DivergencePoint.h"
#include "cluster/src/Trainer.h"
#include "cluster/src/Feature.h"
#include "utility/GlobAlignE.h"
#undef private
#undef protected

using namespace std;

static const char *hexd = "0123456789abcdef";
static string to_hex(const string &s) {
	string o;
	o.reserve(s.size() * 2);
	for (unsigned char c : s) { o.push_back(hexd[c >> 4]); o.push_back(hexd[c & 15]); }
	return o;
}
static string from_hex(const string &h) {
	string o;
	for (size_t i = 0; i + 1 < h.size(); i += 2) o.push_back((char)strtol(h.substr(i, 2).c_str(), NULL, 16));
	return o;
}

static int mode_parse(const char *fa, FILE *out) {
	ChromListMaker maker(fa);
	auto lst = maker.makeChromOneDigitList();
	for (size_t i = 0; i < lst->size(); i++) {
		ChromosomeOneDigit *c = dynamic_cast<ChromosomeOneDigit *>(lst->at(i));
		auto seg = c->getSegment();
		fprintf(out, "R %zu %zu %zu\n", i, c->getBase()->size(), seg->size());
		fprintf(out, "H %s\n", c->getHeader().c_str());
		fprintf(out, "S");
		for (auto v : *seg) fprintf(out, " %d %d", v->at(0), v->at(1));
		fprintf(out, "\nD %s\n", to_hex(*c->getBase()).c_str());
	}
	return 0;
}

static int mode_hist(const char *fa, int k, FILE *out) {
	ChromListMaker maker(fa);
	auto lst = maker.makeChromOneDigitList();
	uint64_t largest = 0;
	for (size_t i = 0; i < lst->size(); i++) {
		ChromosomeOneDigit *c = dynamic_cast<ChromosomeOneDigit *>(lst->at(i));
		KmerHashTable<unsigned long, uint64_t> table(k, 1);
		vector<uint64_t> values;
		fill_table<uint64_t>(table, c, values);
		uint64_t mag = 0, mx = 0;
		for (auto v : values) { mag += v; mx = std::max(mx, v); }
		largest = std::max(largest, mx);
		fprintf(out, "K %zu %llu", i, (unsigned long long)mag);
		for (auto v : values) fprintf(out, " %llu", (unsigned long long)v);
		fprintf(out, "\n");
	}
	fprintf(out, "M %llu\n", (unsigned long long)largest);
	return 0;
}

template<class T>
static void dump_feature(Feature<T> *f, FILE *out) {
	fprintf(out, "FL");
	for (auto l : f->lookup) fprintf(out, " %u", (unsigned)l);
	fprintf(out, "\nFS");
	for (size_t i = 0; i < f->is_sims.size(); i++) fprintf(out, " %d", (int)f->is_sims[i]);
	fprintf(out, "\nFMIN");
	for (auto m : f->mins) fprintf(out, " %a", m);
	fprintf(out, "\nFMAX");
	for (auto m : f->maxs) fprintf(out, " %a", m);
	fprintf(out, "\n");
	for (auto &c : f->combos) {
		fprintf(out, "FC %d", c.first);
		for (auto idx : c.second) fprintf(out, " %d", idx);
		fprintf(out, "\n");
	}
}

// train <fasta> <k> <id> <sample> <pivot> <npts>: replicate Runner::do_run<uint8_t> up to
// Trainer::train (Runner.cpp:321-333), then dump the trained classifier and per-pair vectors.
static int mode_train(const char *fa, int k, double id, int sample, int pivot, int npts, FILE *out) {
	typedef uint8_t T;
	ClusterFactory<T> factory(k);
	vector<string> files = {fa};
	auto points = factory.build_points(files, [&](nonltr::ChromosomeOneDigit *p) { return factory.get_divergence_point(p); });
	for (size_t i = 0; i < points.size(); i++) points[i]->set_id(i);
	double mat[4][4] = {{1, -1, -1, -1}, {-1, 1, -1, -1}, {-1, -1, 1, -1}, {-1, -1, -1, 1}};
	Trainer<T> tr(points, sample, 255, id, pivot, mat, -2, -1, k);
	auto pairs = tr.split();
	for (auto &p : pairs) fprintf(out, "SP %d %d\n", p.first->get_id(), p.second->get_id());
	auto both = tr.get_labels(pairs, id);
	for (auto &p : both.first) fprintf(out, "LP %d %d %a\n", p.first.first->get_id(), p.first.second->get_id(), p.second);
	for (auto &p : both.second) fprintf(out, "LN %d %d %a\n", p.first.first->get_id(), p.first.second->get_id(), p.second);
	tr.train();
	dump_feature(tr.feat, out);
	fprintf(out, "W");
	for (int r = 0; r < tr.weights.getNumRow(); r++) fprintf(out, " %a", tr.weights.get(r, 0));
	fprintf(out, "\n");
	int n = std::min<int>(npts, points.size());
	int ncols = tr.weights.getNumRow();
	// per-pair vectors: raw features (all five live ones), normalized cache, combos, GLM sum
	for (int i = 0; i < n; i++) {
		for (int j = 0; j < n; j++) {
			Point<T> &p = *points[i];
			Point<T> &q = *points[j];
			double ld = Feature<T>::length_difference(p, q);
			double in = Feature<T>::intersection(p, q);
			double ma = Feature<T>::manhattan(p, q);
			double pe = Feature<T>::pearson(p, q);
			double ku = Feature<T>::kulczynski2(p, q);
			auto cache = tr.feat->compute(p, q);
			double sum = tr.weights.get(0, 0);
			double c0 = 0;
			fprintf(out, "P %d %d %a %a %a %a %a", i, j, ld, in, ma, pe, ku);
			fprintf(out, " |");
			for (auto c : cache) fprintf(out, " %a", c);
			fprintf(out, " |");
			for (int col = 1; col < ncols; col++) {
				double v = (*tr.feat)(col - 1, cache);
				if (col == 1) c0 = v;
				sum += tr.weights.get(col, 0) * v;
				fprintf(out, " %a", v);
			}
			double res = round(1.0 / (1 + exp(-sum)));
			fprintf(out, " | %a %d %llu\n", sum, (int)(res == 1.0), (unsigned long long)p.distance(q));
			(void)c0;
		}
	}
	// distance_d against the mean of the first m points, m = 1..min(n,16)
	for (int m = 1; m <= std::min(n, 16); m++) {
		Point<double> *top = points[0]->create_double();
		top->zero();
		Point<double> *temp = top->clone();
		for (int i = 0; i < m; i++) { points[i]->set_arg_to_this_d(*temp); *top += *temp; }
		*top /= (double)m;
		fprintf(out, "DD %d", m);
		for (int i = 0; i < n; i++) fprintf(out, " %a", points[i]->distance_d(*top));
		fprintf(out, "\n");
		delete top;
		delete temp;
	}
	return 0;
}

// nw <pairs file>: each line "hexA hexB"; prints identity, length, matches of GlobAlignE(A,B).
static int mode_nw(const char *pf, FILE *out) {
	ifstream in(pf);
	string a, b;
	while (in >> a >> b) {
		string sa = from_hex(a), sb = from_hex(b);
		utility::GlobAlignE g(sa.c_str(), 0, (int)sa.size() - 1, sb.c_str(), 0, (int)sb.size() - 1, 1, -1, 2, 1);
		fprintf(out, "N %a %d %d %d\n", g.getIdentity(), g.alignmentLength, g.totalMatches, g.alignmentScore);
	}
	return 0;
}

int main(int argc, char **argv) {
	if (argc < 4) {
		fprintf(stderr, "usage: ref_probe <out> parse|hist|train|nw args...\n");
		return 2;
	}
	FILE *out = fopen(argv[1], "w");
	string mode = argv[2];
	int rc = 2;
	if (mode == "parse") rc = mode_parse(argv[3], out);
	else if (mode == "hist" && argc >= 5) rc = mode_hist(argv[3], atoi(argv[4]), out);
	else if (mode == "train" && argc >= 9)
		rc = mode_train(argv[3], atoi(argv[4]), atof(argv[5]), atoi(argv[6]), atoi(argv[7]), atoi(argv[8]), out);
	else if (mode == "nw") rc = mode_nw(argv[3], out);
	fclose(out);
	return rc;
}
