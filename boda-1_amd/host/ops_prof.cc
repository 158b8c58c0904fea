// ops_prof.cc -- boda_hip_ops_prof: Boda's per-op profiling sweep (ops-prof,
// src/rtc_prof.cc:139-371 with profile_rcg_call :44-126) over be=hip.
//
// For each op of an op list (either dialect) and each tune of --op-tunes (the known-good tune
// --kg-tune-tag first, then the others in tag order; default one tune, the tuning table's
// choice): annotate it for the hip backend with the tune (a kernel configuration, its K splits
// and store policy, forced through bh_tune_set), create its vars (zero-filled), fill the inputs
// with gen_data on the device, run the main kernel --run-iter times, take the event-timed
// duration of the last call; compare every output element-wise with the known-good tune's
// (comp_vars, src/rtc_prof.cc:276-321) at --mrd-toler, or the per-function --func-mrd-toler of
// the kernel variant the call ran (Winograd variants: 2e-3, the reference's Winograd widening,
// :314-319); digest it (seed = std::hash of the var name) and compare it with the known-good
// digest of --wisdom-in-fn using the reference's own mrd_comp at the same tolerance; write
// --wisdom-out-fn (the kg tune's digests, and every tune's runs with --write-runs=1) and print
// ***ALL IS WELL*** or ***MAD FAILS***, as the reference does.
// --shard=k/n runs only the ops a greedy LPT partition (by roofline time) gives
// to shard k of n, so n processes (one per GPU, --device=k) split a list with no
// communication at all.
// --selftest-wisdom=F needs no GPU: decodes every kg digest of F, re-encodes it and
// checks the hex round-trips byte-identically and the sample plan matches.
#include <algorithm>
#include <cstdio>
#include <fstream>
#include <iostream>
#include <map>
#include <sstream>

#include "boda_hip.h"
#include "lexp.H"
#include "nda_digest.H"
#include "op_desc.H"
#include "rtc_compute.H"

using namespace boda_hip;

namespace {

struct opts_t {
  std::map<std::string, std::string> kv;
  std::string get(std::string const &k, std::string const &d = "") const {
    auto it = kv.find(k);
    return it == kv.end() ? d : it->second;
  }
};

int selftest_wisdom(std::string const &fn) {
  std::ifstream in(fn);
  if (!in) rt_err("cannot open " + fn);
  std::string line, prev;
  size_t n = 0;
  while (std::getline(in, line)) {
    if (prev == "kg") {
      std::string vn = line, hex;
      std::getline(in, hex);
      nda_digest_t d = nda_digest_t::from_hex(hex);
      if (d.to_hex() != hex) rt_err("hex round trip differs for a digest of " + vn);
      if (d.plan().size() != d.samps.size()) rt_err("sample plan size differs for a digest of " + vn);
      ++n;
      line.clear();
    }
    prev = line;
  }
  std::ifstream in2(fn);
  op_wisdom_t w;
  size_t nops = 0;
  while (read_next_wisdom(in2, w)) {
    parse_op_line(w.op_line);
    ++nops;
  }
  std::cout << "selftest ok: " << n << " digests, " << nops << " op_wisdom blocks\n";
  return 0;
}

// structural op equality, as the reference's op_base_t comparison (src/rtc_prof.cc:238)
bool same_op(op_base_t const &a, op_base_t const &b) {
  if (a.type != b.type || a.str_vals != b.str_vals || a.scalars != b.scalars) return false;
  if (a.dims_vals.size() != b.dims_vals.size()) return false;
  for (auto const &kv : a.dims_vals) {
    auto it = b.dims_vals.find(kv.first);
    if (it == b.dims_vals.end() || it->second != kv.second) return false;
  }
  return true;
}

// Greedy LPT over the op list by roofline time (same algorithm as boda_hip.shard.lpt_partition):
// ops by descending cost (stable), each to the least-loaded shard (lowest index on ties).
std::vector<bool> lpt_mine(std::vector<std::string> const &lines, std::string const &spec) {
  size_t sl = spec.find('/');
  if (sl == std::string::npos) rt_err("--shard wants k/n");
  uint32_t k = parse_u32(spec.substr(0, sl), "shard index"), n = parse_u32(spec.substr(sl + 1), "shard count");
  if (!n || k >= n) rt_err("--shard: need 0 <= k < n");
  std::vector<std::pair<double, size_t>> cost;
  for (size_t i = 0; i < lines.size(); ++i) {
    op_base_t op = parse_op_line(lines[i]);
    double c = (op.type == "Convolution" || op.type == "sgemm") ? roofline_secs(op_work(op)) : 0.0;
    cost.emplace_back(c, i);
  }
  std::stable_sort(cost.begin(), cost.end(), [](auto const &x, auto const &y) { return x.first > y.first; });
  std::vector<double> load(n, 0.0);
  std::vector<bool> mine(lines.size(), false);
  for (auto const &c : cost) {
    size_t j = std::min_element(load.begin(), load.end()) - load.begin();
    load[j] += c.first;
    mine[c.second] = (j == k);
  }
  return mine;
}

std::vector<std::string> read_lines(std::string const &fn) {
  std::ifstream f(fn);
  if (!f) rt_err("cannot open " + fn);
  std::vector<std::string> lines;
  std::string l;
  while (std::getline(f, l))
    if (!l.empty()) lines.push_back(l);
  return lines;
}

std::vector<std::string> arg_vars(op_base_t const &op) {
  if (op.type == "Convolution") return {"in", "filts", "biases", "out"};
  return {"a", "b", "c"};
}
std::vector<std::string> in_vars(op_base_t const &op) {
  if (op.type == "Convolution") return {"in", "filts", "biases"};
  return {"a", "b"};
}
std::vector<std::string> out_vars(op_base_t const &op) {
  if (op.type == "Convolution") return {"out"};
  return {"c"};
}

}  // namespace

int main(int argc, char **argv) {
  opts_t o;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    if (a.rfind("--", 0) != 0) {
      std::cerr << "bad argument " << a << "\n";
      return 2;
    }
    size_t eq = a.find('=');
    o.kv[a.substr(2, eq == std::string::npos ? std::string::npos : eq - 2)] =
        eq == std::string::npos ? "1" : a.substr(eq + 1);
  }
  try {
    if (o.kv.count("selftest-wisdom")) return selftest_wisdom(o.get("selftest-wisdom"));
    if (o.kv.count("dump-ops")) {  // parse-only: one line per Convolution/sgemm op, no GPU needed
      size_t skipped = 0;
      for (auto const &op : read_op_list(o.get("dump-ops"), &skipped)) {
        op_work_t w = op_work(op);
        if (op.type == "Convolution") {
          conv_shape_t s = get_conv_shape(op);
          std::printf("Convolution %u %u %u %u %u %u %u %u %u %u %u %.0f %.0f\n", s.B, s.IC, s.H, s.W, s.OC, s.KY,
                      s.KX, s.sy, s.sx, s.py, s.px, w.flops, w.bytes);
        } else {
          sgemm_shape_t s = get_sgemm_shape(op);
          std::printf("sgemm %u %u %u %.0f %.0f\n", s.M, s.N, s.K, w.flops, w.bytes);
        }
      }
      std::printf("skipped %zu\n", skipped);
      return 0;
    }
    std::string ops_fn = o.get("ops-fn");
    if (o.kv.count("list-shard")) {  // GPU-free: the op indices shard k/n would run
      std::vector<bool> m = lpt_mine(read_lines(ops_fn), o.get("list-shard"));
      for (size_t i = 0; i < m.size(); ++i)
        if (m[i]) std::printf("%zu\n", i);
      return 0;
    }
    if (ops_fn.empty()) {
      std::cerr << "usage: boda_hip_ops_prof --ops-fn=F [--wisdom-in-fn=F] [--wisdom-out-fn=F] [--out-fn=F]\n"
                   "  [--op-tunes='(tag=(use_be=hip,cfg=NAME,splits=N,wt=W),...)'] [--kg-tune-tag=tag]\n"
                   "  [--func-mrd-toler='(variant-or-word=toler,...)'] [--wino-mrd-toler=2e-3] [--max-err=10]\n"
                   "  [--gen-data-mode=5] [--run-iter=1] [--mrd-toler=2e-4] [--device=0] [--write-runs=0]\n"
                   "  [--write-kg-digest=1] [--live-mrd-toler=0]\n"
                   "  [--skip-ops=0] [--shard=k/n] | --selftest-wisdom=F | --dump-ops=F | --list-shard=k/n --ops-fn=F\n";
      return 2;
    }
    const uint32_t mode = parse_u32(o.get("gen-data-mode", "5"), "--gen-data-mode");
    const uint32_t run_iter = std::max(1u, parse_u32(o.get("run-iter", "1"), "--run-iter"));
    const double mrd = parse_f64(o.get("mrd-toler", "2e-4"), "--mrd-toler");
    const uint32_t max_err = parse_u32(o.get("max-err", "10"), "--max-err");
    const bool write_runs = o.get("write-runs", "0") != "0";
    const bool write_kg_digest = o.get("write-kg-digest", "1") != "0";
    uint32_t skip = parse_u32(o.get("skip-ops", "0"), "--skip-ops");
    // --op-tunes (a tag -> op_tune map, iterated in tag order as the reference's map_str_op_tune_t)
    // and --kg-tune-tag (src/rtc_prof.cc:151,166): the kg tune runs first; its outputs are the lhs
    // of a full-data comp_vars against every tune, itself included (:276-321)
    std::map<std::string, hip_op_tune_t> tunes;
    {
      p_lexp_t l = parse_lexp(o.get("op-tunes", "(hip=(use_be=hip))"));
      if (!l->is_list || l->kids.empty()) rt_err("--op-tunes wants (tag=(k=v,...),...)");
      for (auto const &kv : l->kids) {
        if (tunes.count(kv.first)) rt_err("--op-tunes: duplicate tag " + kv.first);
        tunes[kv.first] = parse_hip_op_tune(kv.second->str());
      }
    }
    std::string kg_tag = o.get("kg-tune-tag");
    if (kg_tag.empty()) {
      if (tunes.size() != 1) rt_err("--kg-tune-tag is required with more than one tune");
      kg_tag = tunes.begin()->first;
    }
    if (!tunes.count(kg_tag)) rt_err("--kg-tune-tag=" + kg_tag + " names no tune of --op-tunes");
    std::vector<std::string> order{kg_tag};
    for (auto const &kv : tunes)
      if (kv.first != kg_tag) order.push_back(kv.first);
    // --func-mrd-toler=(key=toler,...): per-function tolerance (src/rtc_prof.cc:160,312). The
    // function is the kernel variant a call ran (bh_variant_name_ctx); a key applies when it equals
    // the variant or is one of its '_'-separated words (wino, dm, k1s, ...), the longest key wins.
    std::map<std::string, double> func_toler;
    {
      p_lexp_t l = parse_lexp(o.get("func-mrd-toler", "()"));
      for (auto const &kv : l->kids) func_toler[kv.first] = parse_f64(kv.second->leaf, "tolerance");
    }
    // Winograd routes widen to 2e-3, the reference's widening for cuDNN's 3x3 Winograd
    // (src/rtc_prof.cc:314-319), unless --func-mrd-toler names them
    const double wino_toler = parse_f64(o.get("wino-mrd-toler", "2e-3"), "--wino-mrd-toler");
    // --live-mrd-toler (MI355X extension, default 0: the reference's single tolerance): a floor for
    // the full-data compare only, the digest compare keeps the function's tolerance. Two fp32
    // routes summing K in different orders differ element-wise by about their error against the
    // exact sum, far above a digest's 2e-4 at K in the thousands
    const double live_floor = parse_f64(o.get("live-mrd-toler", "0"), "--live-mrd-toler");
    auto toler_of = [&](std::string const &variant) {
      double t = mrd;
      size_t best = 0;
      for (auto const &kv : func_toler) {
        const bool hit = variant == kv.first || ("_" + variant + "_").find("_" + kv.first + "_") != std::string::npos;
        if (hit && kv.first.size() > best) best = kv.first.size(), t = kv.second;
      }
      if (!best && variant.find("_wino_") != std::string::npos) t = wino_toler;
      return t;
    };
    std::ofstream fout;
    std::ostream *out = &std::cout;
    if (!o.get("out-fn").empty()) {
      fout.open(o.get("out-fn"));
      out = &fout;
    }
    std::ifstream win;
    if (!o.get("wisdom-in-fn").empty()) {
      win.open(o.get("wisdom-in-fn"));
      if (!win) rt_err("cannot open wisdom-in " + o.get("wisdom-in-fn"));
    }
    std::ofstream wout;
    if (!o.get("wisdom-out-fn").empty()) wout.open(o.get("wisdom-out-fn"));

    // every line of the list (the wisdom file has one block per line, whatever the type)
    std::vector<std::string> lines = read_lines(ops_fn);
    // optional LPT shard by roofline time
    std::vector<bool> mine(lines.size(), true);
    if (!o.get("shard").empty()) mine = lpt_mine(lines, o.get("shard"));

    p_rtc_compute_t rtc = make_hip_compute(parse_i32(o.get("device", "0"), "--device"));
    rtc->init();
    const std::string plat = rtc->get_plat_tag();
    uint32_t num_mad_fail = 0, n_unsup = 0;
    struct agg_t {
      uint32_t n = 0;
      double flops = 0, secs = 0, roof = 0;
    };
    std::map<std::string, agg_t> agg;
    for (size_t ix = 0; ix < lines.size(); ++ix) {
      op_wisdom_t wi;
      bool have_wi = win.is_open() && read_next_wisdom(win, wi);
      if (skip) {
        --skip;
        continue;
      }
      op_base_t op0 = parse_op_line(lines[ix]);
      if (have_wi && !same_op(parse_op_line(wi.op_line), op0)) rt_err("op mismatch between input wisdom and ops-list at op " + std::to_string(ix));
      if (!mine[ix]) continue;
      op_wisdom_t wo;
      wo.op_line = lines[ix];
      bool op_seen_errs = false;  // the op is printed once, before its first error (on_op_err)
      std::map<std::string, p_nda_t> vs_kg;
      bool have_kg = false;
      for (std::string const &tag : order) {
        hip_op_tune_t const &tune = tunes[tag];
        op_base_t op = op0;
        op_run_t run;
        run.plat_tag = plat;
        std::ostringstream err, err_extra;
        std::map<std::string, p_nda_t> outs;
        std::string variant;
        try {
          add_hip_annotations(op, tune);
          std::vector<rtc_func_info_t> fis{{op.func_name, "", {}, op}};
          for (auto const &vn : in_vars(op)) fis.push_back({"gen_data_" + op.type + "_" + vn, "", {}, op});
          rtc->compile(fis, rtc_compile_opts_t());
          for (auto const &vn : arg_vars(op)) rtc->create_var_with_dims(vn, op.get_dims(vn));
          for (auto const &vn : in_vars(op)) {
            rtc_func_call_t g;
            g.rtc_func_name = "gen_data_" + op.type + "_" + vn;
            g.arg_map[vn] = vn;
            g.arg_map["mode"] = rtc_arg_t::val(mode);
            g.arg_map["vi"] = rtc_arg_t::val(0.0);
            rtc->run(g);
          }
          rtc_func_call_t c;
          c.rtc_func_name = op.func_name;
          for (auto const &vn : arg_vars(op)) c.arg_map[vn] = vn;
          if (op.type == "Convolution") {
            // layout transform of the filters before the timed calls, as the reference's
            // xpose_filts (src/rtc_prof.cc:93-99; untimed)
            conv_shape_t s = get_conv_shape(op);
            rtc->compile({{"hip_xpose_filts", "", {}, op}}, rtc_compile_opts_t());
            const uint32_t nxp = (uint32_t)bh_conv_filts_packed_floats(s.OC, s.IC, s.KY, s.KX);
            rtc->create_var_with_dims("filts_xp", dims_t(std::vector<std::pair<std::string, uint32_t>>{{"x", nxp}}));
            rtc_func_call_t x;
            x.rtc_func_name = "hip_xpose_filts";
            x.arg_map["filts"] = "filts";
            x.arg_map["filts_xp"] = "filts_xp";
            rtc->run(x);
            c.arg_map["filts_xp"] = "filts_xp";
          }
          uint32_t call_id = 0;
          for (uint32_t r = 0; r < run_iter; ++r) call_id = rtc->run(c);
          rtc->finish_and_sync();
          run.rt_secs = rtc->get_dur(call_id, call_id) / 1000.0;
          variant = rtc->get_call_variant(call_id);
          for (auto const &vn : out_vars(op)) outs[vn] = rtc->create_nda_from_var(vn);
          run.op_line = op.line;
        } catch (unsup_exception const &e) {
          err << "profile call failure: " << e.what();
          ++n_unsup;  // recorded, not a MAD failure (src/rtc_prof.cc:287-296, :368-369)
        }
        for (auto const &vn : arg_vars(op))
          if (op.has_dims(vn)) {
            try {
              rtc->release_var(vn);
            } catch (rt_exception const &) {
            }
          }
        if (op.type == "Convolution") {
          try {
            rtc->release_var("filts_xp");
          } catch (rt_exception const &) {
          }
        }
        rtc->release_per_call_id_data();
        rtc->release_all_funcs();
        if (tag == kg_tag) {  // the known-good run: the lhs of the compares, and the digests
          if (!err.str().empty()) {
            err << " known-good op_tune (kg_tune_tag=" << kg_tag << ") failed. Can't write digests or do live comparisons.";
          } else {
            vs_kg = outs;
            have_kg = true;
            if (write_kg_digest)
              for (auto const &kv : outs)
                wo.kgs.emplace_back(kv.first, nda_digest_t::make(kv.second->elems(), kv.second->dims,
                                                                 digest_seed_for(kv.first)));
          }
        }
        std::string dstat = "n/a", cstat = "n/a";
        double worst_mrd = 0;
        if (err.str().empty()) {
          const double vmt = toler_of(variant), lvmt = std::max(vmt, live_floor);
          if (have_kg) {  // full-data compare against the known-good run
            cstat = "ok";
            for (auto const &kv : vs_kg) {
              auto it = outs.find(kv.first);
              if (it == outs.end()) rt_err("reg/comp out var set mismatch for tune " + tag);
              double m = 0;
              std::ostringstream cv;
              if (comp_var(cv, kv.first, kv.second->dims, *kv.second->data, *it->second->data, lvmt, max_err, &m)) {
                ++num_mad_fail;
                cstat = "FAIL";
                err << cv.str();
              }
              worst_mrd = std::max(worst_mrd, m);
            }
          }
          if (have_wi) {  // digest compare against the stored known-good digests
            dstat = "ok";
            for (auto const &kv : outs) {
              nda_digest_t d = nda_digest_t::make(kv.second->elems(), kv.second->dims, digest_seed_for(kv.first));
              for (auto const &kg : wi.kgs)
                if (kg.first == kv.first) {
                  double worst = 0;
                  std::string cr = kg.second.mrd_comp(d, vmt, &worst);
                  if (!cr.empty()) {
                    dstat = "FAIL";
                    err << kv.first << " digest mrd_comp() failure vs stored digest (worst rd/tol " << worst << ")";
                    err_extra << "comp_res:\n" << cr;
                  }
                }
            }
            if (dstat == "FAIL") ++num_mad_fail;
          }
          op_work_t w = op_work(op);
          agg_t &g = agg[tag];
          g.flops += w.flops;
          g.secs += run.rt_secs;
          g.roof += roofline_secs(w);
          ++g.n;
          char buf[640];
          std::snprintf(buf, sizeof(buf),
                        "op_ix=%zu tune=%s func=%s secs=%.6e gflops=%.1f roofline=%.1f%% mrd_vs_kg=%.3e toler=%.1e "
                        "comp=%s dtoler=%.1e digest=%s\n",
                        ix, tag.c_str(), variant.empty() ? op.func_name.c_str() : variant.c_str(), run.rt_secs,
                        w.flops / run.rt_secs / 1e9, 100.0 * roofline_secs(w) / run.rt_secs, worst_mrd, lvmt,
                        cstat.c_str(), vmt, dstat.c_str());
          *out << buf;
        }
        run.err = err.str();
        if (!run.err.empty()) {
          if (!op_seen_errs) *out << "-----\n errors for op_ix=" << ix << " op='" << lines[ix] << "'\n";
          op_seen_errs = true;
          *out << "--  comp fail for op_tune='" << tune.str() << "'\n" << run.err << "\n" << err_extra.str();
        }
        if (write_runs) wo.tunes.push_back({tune.str(), {run}});
      }
      if (!write_kg_digest && have_wi) wo.kgs = wi.kgs;
      if (wout.is_open()) {
        write_wisdom(wout, wo);
        wout.flush();
      }
      out->flush();
    }
    for (std::string const &tag : order) {
      agg_t const &g = agg[tag];
      if (!g.n) continue;
      char buf[320];
      std::snprintf(buf, sizeof(buf),
                    "summary: ops=%u sum_gflop=%.3f sum_kernel_ms=%.4f agg_gflops=%.1f roofline_frac=%.4f plat=%s "
                    "tune=%s\n",
                    g.n, g.flops / 1e9, g.secs * 1e3, g.flops / g.secs / 1e9, g.roof / g.secs, plat.c_str(), tag.c_str());
      *out << buf;
    }
    if (n_unsup) *out << "unsupported (recorded in wisdom, skipped): " << n_unsup << "\n";
    if (!num_mad_fail) *out << "***ALL IS WELL***\n";
    else *out << "***MAD FAILS*** num_mad_fail=" << num_mad_fail << "\n";
    return num_mad_fail ? 1 : 0;
  } catch (rt_exception const &e) {
    std::cerr << "error: " << e.what() << "\n";
    return 3;
  }
}
