// cnn_op_info.cc -- boda_hip_cnn_op_info: one tune against a comparator, per op, with Boda's
// efficiency rows (cnn_op_info_t::main, src/cnn-prof.cc:59-130).
//
// For each op line of --cnn-func-sigs-fn (either dialect, Convolution or sgemm):
//   * writes the op's info row to --op-info-tab-fn (conv_op_info_to_latex_t::info_row,
//     src/latex-util.H:59-68; never brief there, as the reference);
//   * runs the op on the hand-written MI355X kernels (be=hip, libboda_hip.so) on gen_data inputs,
//     --run-iter times, and takes the event time of the last call (profile_rcg_call,
//     src/rtc_prof.cc:44-126); --graph-reps=N instead captures N back-to-back calls in one hipGraph,
//     replays it and takes the per-call time (the bench's per-op convention) -- printed
//     to the log; with a comparator the eff row carries both sides in the reference's per-call
//     convention (the event pair of the last of --run-iter calls; the comparator's calls one by
//     one, each between its own event pair), so its columns compare like with like;
//   * with --comp=vendor (the default, the reference's use_culibs=1 comparator,
//     src/cnn-prof.cc:40,90-91 / src/culibs-wrap.cc:94-242), runs the same op through rocBLAS / MIOpen
//     (libboda_hip_vendor.so) on the SAME device inputs into its own output, prints
//     "vars_to_compare: <vars>" and compares the outputs as comp_vars does (src/comp_util.cc:21-57:
//     a MAD failure when the max min_sig_mag_rel_diff(1, v1, v2) >= --mrd-toler or a NaN; a failing
//     var prints its ssds summary and its first --max-err differing elements);
//   * writes the op's efficiency row to --op-eff-tab-fn (eff_row, src/latex-util.H:74-100: conv =
//     KSZ & stride & OC & dims(in) & type & runtime & GF/s & %peak; sgemm = MKN & bytes & flops &
//     F/B & comparator runtime & GF/s & runtime & GF/s & speedup; --eff-comp=1 appends the
//     comparator's runtime & GF/s & speedup to conv rows too, which the reference's drop);
// and prints ***ALL IS WELL*** or ***MAD FAILS*** num_mad_fail=N at the end (exit status 1 on
// failure). The comparator is never linked by the product library; this driver is the harness.
// --peak-flops defaults to the MI355X fp32 MFMA peak (op_desc.H), not the reference's 6600e9.
#include <cmath>
#include <cstdio>
#include <fstream>
#include <iostream>
#include <map>
#include <sstream>

#include "boda_hip.h"
#include "boda_hip_vendor.h"
#include "nda_digest.H"
#include "op_desc.H"
#include "rtc_compute.H"

using namespace boda_hip;

namespace {

std::string fmt(char const *f, double v) {
  char b[64];
  std::snprintf(b, sizeof b, f, v);
  return b;
}

// engineering-suffix printing, restated from src/str_util.cc:230-256 (pp_val_part / pp_val)
std::string pp_val_part(double v, bool force) {
  if (v < 10.0) return fmt("%.2f", v);
  if (v < 100.0) return fmt("%.1f", v);
  if (v < 1000.0 || force) return fmt("%.0f", v);
  return "***";
}
std::string raw_str(double v) {  // str(double) of the reference: a default ostream (src/str_util.H:107-111)
  std::ostringstream s;
  s << v;
  return s.str();
}
std::string pp_val(double orig) {
  if (std::isnan(orig)) return "NAN";
  if (orig < 0) rt_err("pp_val: negative value");
  double v = orig;
  int e = 0;
  while (v < 1.0) {
    v *= 1000.0;
    --e;
    if (e < -4) return raw_str(orig);
  }
  std::string r;
  while (true) {
    r = pp_val_part(v, false);
    if (r != pp_val_part(1e6, e == 5)) break;
    v /= 1000.0;
    ++e;
  }
  if (e < 0) return r + "munp"[-1 - e];
  if (e == 0) return r;
  return r + "KMGTP"[e - 1];
}

// conv_op_info_to_latex_t (src/latex-util.H:22-139), for one op
struct latex_rows_t {
  uint32_t print_format = 0;  // 0 pretty, 1 raw, 2 raw flops in info rows
  bool inc_op_info_in_eff = false;
  bool eff_comp = false;  // conv rows: append the comparator's runtime, GF/s and its time / ours
  bool is_conv = false;
  conv_shape_t cs{};
  uint64_t M = 0, N = 0, K = 0, B = 1;
  double fwd_bytes = 0, fwd_flops = 0;

  std::string pp(double v, char const *unit) const { return print_format == 0 ? pp_val(v) + unit : raw_str(v); }
  static std::string yxc(uint32_t y, uint32_t x, uint32_t c, int64_t img = -1) {  // dims_yxc_str
    std::string s = "$ ";
    if (img >= 0) s += std::to_string(img) + " \\dx";
    return s + " " + std::to_string(y) + " \\dx " + std::to_string(x) + " \\dx " + std::to_string(c) + " $";
  }
  static std::string mkn(uint64_t m, uint64_t k, uint64_t n) {  // mkn_str
    if (m == k && k == n) return "$ " + std::to_string(m) + " $";
    return "$ " + std::to_string(m) + " \\dx " + std::to_string(k) + " \\dx " + std::to_string(n) + " $";
  }

  void init(op_base_t const &op) {
    op_work_t w = op_work(op);  // the latex-util flop / byte model (src/latex-util.H:101-136)
    fwd_flops = w.flops;
    fwd_bytes = w.bytes;
    is_conv = op.type == "Convolution";
    if (is_conv) {
      cs = get_conv_shape(op);
      if (cs.KY != cs.KX || cs.sy != cs.sx) rt_err("cnn_op_info: non-square kernel or stride");  // base_info asserts
      B = cs.B;
      M = (uint64_t)cs.B * cs.OH * cs.OW;
      K = (uint64_t)cs.IC * cs.KY * cs.KX;
      N = cs.OC;
    } else {
      sgemm_shape_t s = get_sgemm_shape(op);
      M = s.M, N = s.N, K = s.K;
    }
  }
  std::string base_info() const {
    if (!is_conv) return "";
    return std::to_string(cs.KY) + " & " + std::to_string(cs.sy) + " & " + std::to_string(cs.OC);
  }
  std::string ai_mkn() const {  // show_bytes_and_ai = 1 (cnn-prof.cc passes 1)
    return " " + mkn(M, K, N) + " & " + pp(fwd_bytes, "B") + " & " + pp(fwd_flops, "F") + " & " +
           pp(fwd_flops / fwd_bytes, "") + " ";
  }
  std::string info_row() const {
    std::string r = base_info();
    if (is_conv) {
      r += " & " + std::to_string(B) + " & " + yxc(cs.H, cs.W, cs.IC) + " & ";
      r += yxc(cs.OH, cs.OW, cs.OC) + " & ";
    }
    return r + ai_mkn() + "\\\\ \n";
  }
  std::string eff_row(std::string const &type, double secs, double peak, double secs_comp) const {
    std::string r;
    if (!is_conv) {
      r = ai_mkn();
      r += " & " + pp(secs_comp, "s") + " & " + pp(fwd_flops / secs_comp, "F/s") + " ";
      r += " & " + pp(secs, "s") + " & " + pp(fwd_flops / secs, "F/s") + " ";
      r += fmt(" & %.2fx ", secs_comp / secs);
    } else {
      r = base_info() + " & " + yxc(cs.H, cs.W, cs.IC, B) + " & \\verb|" + type + "| & ";
      if (inc_op_info_in_eff) r += ai_mkn() + " & ";
      const double fps = fwd_flops / secs;
      r += " " + pp(secs, "s") + " & " + pp(fps, "F/s") + " & " + pp(fps / peak * 100.0, "") + " ";
      if (eff_comp) r += " & " + pp(secs_comp, "s") + " & " + pp(fwd_flops / secs_comp, "F/s") + fmt(" & %.2fx ", secs_comp / secs);
    }
    return r + "\\\\ \n";
  }
};

void vcheck(int rc, char const *what) {
  if (rc != BHV_OK) rt_err(std::string(what) + ": " + bhv_last_error());
}

struct opts_t {
  std::map<std::string, std::string> kv;
  std::string get(std::string const &k, std::string const &d = "") const {
    auto it = kv.find(k);
    return it == kv.end() ? d : it->second;
  }
};

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
  if (o.kv.count("pp-vals")) {  // GPU-free check of the number formatting: pp_val of a comma list
    std::stringstream ss(o.get("pp-vals"));
    std::string t;
    while (std::getline(ss, t, ',')) std::cout << pp_val(parse_f64(t, "value")) << "\n";
    return 0;
  }
  if (o.get("cnn-func-sigs-fn").empty()) {
    std::cerr << "usage: boda_hip_cnn_op_info --cnn-func-sigs-fn=F [--out-fn=F] [--op-info-tab-fn=F]\n"
                 "  [--op-eff-tab-fn=F] [--print-format=0|1|2] [--inc-op-info-in-eff=0] [--peak-flops=157.3e12]\n"
                 "  [--run-iter=1] [--graph-reps=0] [--gen-data-mode=5] [--comp=vendor|none] [--mrd-toler=2e-4]\n"
                 "  [--max-err=10] [--wino-mrd-toler=2e-3] [--show-mrd=1] [--device=0]\n"
                 "  [--eff-comp=1] [--no-run=1] | --pp-vals=v,v,...\n";
    return 2;
  }
  try {
    std::ofstream fout, oit, oet;
    std::ostream *out = &std::cout;
    if (!o.get("out-fn").empty()) {
      fout.open(o.get("out-fn"));
      out = &fout;
    }
    if (!o.get("op-info-tab-fn").empty()) oit.open(o.get("op-info-tab-fn"));
    if (!o.get("op-eff-tab-fn").empty()) oet.open(o.get("op-eff-tab-fn"));
    const uint32_t print_format = parse_u32(o.get("print-format", "0"), "--print-format");
    const bool inc_info = o.get("inc-op-info-in-eff", "0") != "0";
    // not in the reference (its conv eff rows drop the comparator's time, latex-util.H:90-97)
    const bool eff_comp = o.get("eff-comp", "0") != "0";
    const double peak = parse_f64(o.get("peak-flops", std::to_string(PEAK_FP32_FLOPS)), "--peak-flops");
    const uint32_t run_iter = std::max(1u, parse_u32(o.get("run-iter", "1"), "--run-iter"));
    const uint32_t graph_reps = parse_u32(o.get("graph-reps", "0"), "--graph-reps");
    const uint32_t mode = parse_u32(o.get("gen-data-mode", "5"), "--gen-data-mode");
    const double toler = parse_f64(o.get("mrd-toler", "2e-4"), "--mrd-toler");
    // Winograd routes (variant names *_wino_*) compare at the reference's Winograd tolerance, 2e-3
    // (ops-prof's widening for cuDNN's 3x3 Winograd, src/rtc_prof.cc:314-319): the input / output
    // transforms turn cancellation in the direct sum into element errors min_sig_mag_rel_diff sees
    // on near-zero outputs (measured per op with --show-mrd=1)
    const double wino_toler = parse_f64(o.get("wino-mrd-toler", "2e-3"), "--wino-mrd-toler");
    const bool show_mrd = o.get("show-mrd", "0") != "0";
    const uint32_t max_err = parse_u32(o.get("max-err", "10"), "--max-err");
    const std::string comp = o.get("comp", "vendor");
    if (comp != "vendor" && comp != "none") rt_err("--comp must be vendor or none");
    const int device = parse_i32(o.get("device", "0"), "--device");
    // --no-run: rows only, no device (runtimes NAN, as a failed profile call leaves them, cnn-prof.cc:95)
    const bool no_run = o.get("no-run", "0") != "0";

    size_t skipped = 0;
    std::vector<op_base_t> ops = read_op_list(o.get("cnn-func-sigs-fn"), &skipped);
    p_rtc_compute_t rtc;
    bhv_ctx *vctx = nullptr;
    if (!no_run) {
      rtc = make_hip_compute(device);
      rtc->init();
      if (comp == "vendor") vcheck(bhv_init(device, &vctx), "bhv_init");
    }

    uint32_t num_mad_fail = 0;
    for (op_base_t op : ops) {
      latex_rows_t lx;
      lx.print_format = print_format;
      lx.inc_op_info_in_eff = inc_info;
      lx.eff_comp = eff_comp;
      lx.init(op);
      if (oit.is_open()) oit << lx.info_row();
      if (no_run) {
        if (oet.is_open()) oet << lx.eff_row(op.type, NAN, peak, NAN);
        continue;
      }

      add_hip_annotations(op);
      const bool conv = op.type == "Convolution";
      const std::vector<std::string> ins = conv ? std::vector<std::string>{"in", "filts", "biases"}
                                                : std::vector<std::string>{"a", "b"};
      const std::string ovn = conv ? "out" : "c";
      std::vector<rtc_func_info_t> fis{{op.func_name, "", {}, op}};
      for (auto const &vn : ins) fis.push_back({"gen_data_" + op.type + "_" + vn, "", {}, op});
      rtc->compile(fis, rtc_compile_opts_t());
      for (auto const &vn : ins) rtc->create_var_with_dims(vn, op.get_dims(vn));
      rtc->create_var_with_dims(ovn, op.get_dims(ovn));
      for (auto const &vn : ins) {
        rtc_func_call_t g;
        g.rtc_func_name = "gen_data_" + op.type + "_" + vn;
        g.arg_map[vn] = vn;
        g.arg_map["mode"] = rtc_arg_t::val(mode);
        g.arg_map["vi"] = rtc_arg_t::val(0.0);
        rtc->run(g);
      }
      rtc_func_call_t c;
      c.rtc_func_name = op.func_name;
      for (auto const &vn : ins) c.arg_map[vn] = vn;
      c.arg_map[ovn] = ovn;
      if (conv) {  // filter layout transform outside the timed calls, as ops_prof.cc (src/rtc_prof.cc:93-99)
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
      // the reference's convention: the event pair of the last of run_iter calls (profile_rcg_call,
      // src/rtc_prof.cc:104-124); the comparator below is timed the same way
      const double secs_call = rtc->get_dur(call_id, call_id) / 1e3;
      double secs = secs_call;
      // graph_reps back-to-back calls captured in one graph, replayed 3 times: the per-call time
      if (graph_reps) {
        secs = rtc->time_graph([&] { for (uint32_t r = 0; r < graph_reps; ++r) rtc->run(c); }, 3) / graph_reps / 1e3;
        *out << "graph_amortized_secs=" << raw_str(secs) << " per_call_event_secs=" << raw_str(secs_call) << "\n";
      }
      p_nda_t o1 = rtc->create_nda_from_var(ovn);

      char vb[160] = "";
      {
        std::vector<uint32_t> dims;
        if (conv) {
          conv_shape_t s = get_conv_shape(op);
          dims = {s.B, s.IC, s.H, s.W, s.OC, s.KY, s.KX, s.sy, s.sx, s.py, s.px};
        } else {
          sgemm_shape_t s = get_sgemm_shape(op);
          dims = {s.M, s.N, s.K};
        }
        if (bh_variant_name(conv ? 1 : 0, dims.data(), vb, sizeof vb) != 0)
          std::snprintf(vb, sizeof vb, "%s", op.func_name.c_str());
      }
      const bool wino = std::string(vb).find("_wino_") != std::string::npos;
      double secs_comp = NAN;
      if (vctx) {
        // the comparator on the same device inputs, into a second output var
        rtc->create_var_with_dims("comp_" + ovn, op.get_dims(ovn));
        auto P = [&](std::string const &vn) { return (float *)rtc->get_var_raw_native_pointer(vn)->rp; };
        float ms = 0;
        if (conv) {
          conv_shape_t s = get_conv_shape(op);
          vcheck(bhv_conv2d_fwd_nchw(vctx, P("in"), P("filts"), P("biases"), P("comp_out"), s.B, s.IC, s.H, s.W,
                                     s.OC, s.KY, s.KX, s.sy, s.sx, s.py, s.px, (int)op.scalars["conv_has_relu"]),
                 "bhv_conv2d_fwd_nchw");
          vcheck(bhv_sync(vctx), "bhv_sync");
          // run_iter single calls, each between its own event pair; the last one's time (as ours)
          for (uint32_t r = 0; r < run_iter; ++r)
            vcheck(bhv_time_conv(vctx, s.B, s.IC, s.H, s.W, s.OC, s.KY, s.KX, s.sy, s.sx, s.py, s.px,
                                 (int)op.scalars["conv_has_relu"], 1, &ms, nullptr, nullptr, nullptr, 0),
                   "bhv_time_conv");
        } else {
          sgemm_shape_t s = get_sgemm_shape(op);
          vcheck(bhv_sgemm_kmajor(vctx, P("a"), P("b"), P("comp_c"), s.M, s.N, s.K), "bhv_sgemm_kmajor");
          vcheck(bhv_sync(vctx), "bhv_sync");
          for (uint32_t r = 0; r < run_iter; ++r) vcheck(bhv_time_sgemm(vctx, s.M, s.N, s.K, 1, &ms), "bhv_time_sgemm");
        }
        secs_comp = ms / 1e3;
        p_nda_t o2 = rtc->create_nda_from_var("comp_" + ovn);
        *out << "vars_to_compare: " << ovn << "\n";
        double mrd = 0;
        if (comp_var(*out, ovn, o1->dims, *o1->data, *o2->data, wino ? wino_toler : toler, max_err, &mrd))
          ++num_mad_fail;
        if (show_mrd) *out << ovn << ": max_rel_diff=" << raw_str(mrd) << " toler=" << (wino ? wino_toler : toler)
                           << " variant=" << vb << "\n";
        rtc->release_var("comp_" + ovn);
      }
      if (oet.is_open()) {
        // with a comparator every runtime on the row is a per-call event time (the comparator's
        // method: MIOpen / rocBLAS are not graph-captured); the graph-amortized time stays in the log
        oet << lx.eff_row(vb, vctx ? secs_call : secs, peak, secs_comp);
        oet.flush();
      }
      for (auto const &vn : ins) rtc->release_var(vn);
      rtc->release_var(ovn);
      if (conv) rtc->release_var("filts_xp");
      rtc->release_per_call_id_data();
      rtc->release_all_funcs();
      out->flush();
    }
    if (vctx) bhv_destroy(vctx);
    if (!num_mad_fail) *out << "***ALL IS WELL***\n";
    else *out << "***MAD FAILS*** num_mad_fail=" << num_mad_fail << "\n";
    out->flush();
    return num_mad_fail ? 1 : 0;
  } catch (rt_exception const &e) {
    std::cerr << "error: " << e.what() << "\n";
    return 3;
  }
}
