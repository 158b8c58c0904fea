// wis_ana.cc -- boda_hip_wis_ana: Boda's `wis-ana` (src/op-tuner.cc:204-330) for wisdom files
// that include runs of this backend (plat tag hip:MI355X...). For every op of the wisdom
// file(s) and every platform whose tag matches --s-plat: the per-op best run over all tunes
// ("pom", the reference's boda-autotuned column) and the run of the single tune that is best
// over all ops ("aom", boda-manual-tune: most ops handled, then least total time). Ops from
// several files (e.g. the reference's test/wisdom-merged.wis and an ops-prof --write-runs=1
// output of this backend) are matched by conv / sgemm shape, so the two op-line dialects mix.
//
//   boda_hip_wis_ana --wisdom-in-fn=A.wis [--wisdom-in-fn=B.wis ...] [--s-plat=REGEX]
//                    [--s-img=N] [--min-flops=F] [--csv-out-fn=F]
//
// Prints per platform: ops with a run, sum of flops / sum of per-op best times, and for each
// platform pair the geometric-mean per-op speedup on the ops both ran.
#include <cmath>
#include <cstdio>
#include <fstream>
#include <iostream>
#include <map>
#include <regex>
#include <set>
#include <sstream>

#include "nda_digest.H"
#include "op_desc.H"

using namespace boda_hip;

namespace {
struct op_rec_t {
  std::string key, line;
  double flops = 0;
  uint32_t img = 0;
  std::map<std::string, std::map<std::string, double>> plat_tune_secs;  // plat -> tune -> best secs
};

std::string shape_key(op_base_t const &op, double &flops, uint32_t &img) {
  op_work_t w = op_work(op);
  flops = w.flops;
  if (op.type == "Convolution") {
    conv_shape_t s = get_conv_shape(op);
    img = s.B;
    char b[160];
    snprintf(b, sizeof(b), "conv %u %u %u %u %u %u %u %u %u %u %u", s.B, s.IC, s.H, s.W, s.OC, s.KY, s.KX, s.sy, s.sx,
             s.py, s.px);
    return b;
  }
  sgemm_shape_t s = get_sgemm_shape(op);
  img = 0;
  return "sgemm " + std::to_string(s.M) + " " + std::to_string(s.N) + " " + std::to_string(s.K);
}
}  // namespace

int main(int argc, char **argv) {
  std::vector<std::string> ins;
  std::string s_plat = ".*", csv;
  uint32_t s_img = 0;
  double min_flops = 0;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto v = [&](char const *p) -> std::string { return a.substr(std::string(p).size()); };
    if (a.rfind("--wisdom-in-fn=", 0) == 0) ins.push_back(v("--wisdom-in-fn="));
    else if (a.rfind("--s-plat=", 0) == 0) s_plat = v("--s-plat=");
    else if (a.rfind("--s-img=", 0) == 0) s_img = (uint32_t)atoi(v("--s-img=").c_str());
    else if (a.rfind("--min-flops=", 0) == 0) min_flops = atof(v("--min-flops=").c_str());
    else if (a.rfind("--csv-out-fn=", 0) == 0) csv = v("--csv-out-fn=");
    else {
      fprintf(stderr, "usage: boda_hip_wis_ana --wisdom-in-fn=F [...] [--s-plat=RE] [--s-img=N] [--min-flops=F] "
                      "[--csv-out-fn=F]\n");
      return 2;
    }
  }
  if (ins.empty()) {
    fprintf(stderr, "boda_hip_wis_ana: need --wisdom-in-fn\n");
    return 2;
  }
  try {
    std::regex rp(s_plat);
    std::map<std::string, op_rec_t> ops;  // by shape key
    std::vector<std::string> order;
    std::set<std::string> plats;
    for (auto const &fn : ins) {
      std::ifstream in(fn);
      if (!in) rt_err("cannot open " + fn);
      op_wisdom_t w;
      while (read_next_wisdom(in, w)) {
        op_base_t op = parse_op_line(w.op_line);
        if (op.type != "Convolution" && op.type != "sgemm") continue;
        double flops;
        uint32_t img;
        std::string key = shape_key(op, flops, img);
        if ((s_img && img != s_img) || flops < min_flops) continue;
        op_rec_t &r = ops[key];
        if (r.key.empty()) {
          r.key = key;
          r.line = w.op_line;
          r.flops = flops;
          r.img = img;
          order.push_back(key);
        }
        for (auto const &t : w.tunes)
          for (auto const &run : t.second) {
            if (!run.err.empty() || !std::regex_search(run.plat_tag, rp)) continue;
            plats.insert(run.plat_tag);
            auto &m = r.plat_tune_secs[run.plat_tag];
            auto it = m.find(t.first);
            if (it == m.end() || run.rt_secs < it->second) m[t.first] = run.rt_secs;
          }
      }
    }
    // per platform: the overall best single tune (most ops handled, then least total time)
    std::map<std::string, std::string> aom_tune;
    for (auto const &p : plats) {
      std::map<std::string, std::pair<size_t, double>> score;
      for (auto const &k : order) {
        auto it = ops[k].plat_tune_secs.find(p);
        if (it == ops[k].plat_tune_secs.end()) continue;
        for (auto const &ts : it->second) {
          score[ts.first].first += 1;
          score[ts.first].second += ts.second;
        }
      }
      std::string best;
      std::pair<size_t, double> bs{0, 0};
      for (auto const &s : score)
        if (best.empty() || s.second.first > bs.first || (s.second.first == bs.first && s.second.second < bs.second)) {
          best = s.first;
          bs = s.second;
        }
      aom_tune[p] = best;
    }
    std::ofstream co;
    if (!csv.empty()) {
      co.open(csv);
      co << "OP FLOPS";
      for (auto const &p : plats) co << " \"pom:" << p << "\" \"aom:" << p << "\"";
      co << "\n";
    }
    std::map<std::string, double> sum_t, sum_f;
    std::map<std::string, size_t> n_ops;
    for (auto const &k : order) {
      op_rec_t &r = ops[k];
      if (co.is_open()) co << "\"" << k << "\" " << r.flops;
      for (auto const &p : plats) {
        double pom = NAN, aom = NAN;
        auto it = r.plat_tune_secs.find(p);
        if (it != r.plat_tune_secs.end()) {
          for (auto const &ts : it->second) pom = std::isnan(pom) ? ts.second : std::min(pom, ts.second);
          auto a = it->second.find(aom_tune[p]);
          if (a != it->second.end()) aom = a->second;
          sum_t[p] += pom;
          sum_f[p] += r.flops;
          n_ops[p] += 1;
        }
        if (co.is_open()) co << " " << pom << " " << aom;
      }
      if (co.is_open()) co << "\n";
    }
    printf("%-34s %5s %12s %12s\n", "platform", "ops", "sum_best_ms", "GFLOP/s");
    for (auto const &p : plats)
      printf("%-34s %5zu %12.3f %12.1f\n", p.c_str(), n_ops[p], sum_t[p] * 1e3, sum_f[p] / sum_t[p] / 1e9);
    // geometric-mean per-op speedup of each platform over each other, on the ops both ran
    for (auto const &a : plats)
      for (auto const &b : plats) {
        if (a >= b) continue;
        double lg = 0;
        size_t n = 0;
        for (auto const &k : order) {
          auto &m = ops[k].plat_tune_secs;
          if (!m.count(a) || !m.count(b)) continue;
          double ta = 1e30, tb = 1e30;
          for (auto const &ts : m[a]) ta = std::min(ta, ts.second);
          for (auto const &ts : m[b]) tb = std::min(tb, ts.second);
          lg += std::log(tb / ta);
          ++n;
        }
        if (n) printf("per-op geomean speedup %s over %s: %.2fx (%zu ops)\n", a.c_str(), b.c_str(), std::exp(lg / n), n);
      }
  } catch (std::exception const &e) {
    fprintf(stderr, "error: %s\n", e.what());
    return 1;
  }
  return 0;
}
