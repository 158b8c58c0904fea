// rtc_fwd_main.cc -- boda_hip_rtc_fwd: full-net forward of a Caffe prototxt on be=hip, the
// counterpart of Boda's `boda rtc_fwd` / test_compute net runs (src/rtc_fwd.cc:469-577) for the
// layers the MI355X backend executes. Parameters are synthetic (conv_pipe.H); the input is
// gen_data mode 5 (det_hash_rand(i + 234234567), the reference's Convolution `in` seed).
//
//   boda_hip_rtc_fwd --net nets/alexnet/train_val.prototxt [--img 20] [--out-node pool5]
//                    [--iters 5] [--plan | --plan-json] [--save DIR] [--device 0] [--no-pack] [--no-fold]
//
// --plan / --plan-json print the net plan without touching a GPU (host logic tests); --plan-exec
// the executor's BatchNorm/Scale folds and in-place Concat slabs;
// --no-fold runs BatchNorm / Scale as separate affine layers instead of folding them into the
// producing conv (conv_pipe_fwd_t::plan_folds); --no-inplace-concat copies every Concat input
// instead of letting its producing conv write the Concat's channel slab (plan_slabs).
// --no-resadd runs a ResNet shortcut Eltwise SUM as its own layer instead of in the epilogue
// of the conv producing one of its inputs (plan_resadds).
// --graph R also times the whole forward captured as one hipGraph, replayed R times (ms per
// forward with every launch seam; the per-layer list is event-timed per call).
// --save writes DIR/in.f32 and DIR/out.f32 (raw little-endian fp32) for the parity tests.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>

#include "conv_pipe.H"

using namespace boda_hip;

namespace {
std::string read_file(std::string const &fn) {
  std::ifstream f(fn, std::ios::binary);
  if (!f) rt_err("cannot read " + fn);
  std::stringstream ss;
  ss << f.rdbuf();
  return ss.str();
}
void write_f32(std::string const &fn, nda_t const &n) {
  FILE *f = fopen(fn.c_str(), "wb");
  if (!f) rt_err("cannot write " + fn);
  fwrite(n.elems(), 4, n.dims.elems(), f);
  fclose(f);
}
std::string jstr(std::string const &s) {
  std::string o = "\"";
  for (char c : s) {
    if (c == '"' || c == '\\') o += '\\';
    o += c;
  }
  return o + "\"";
}
std::string jdims(dims_t const &d) {
  std::string o = "[";
  for (size_t i = 0; i < d.d.size(); ++i) o += (i ? "," : "") + std::to_string(d.d[i].sz);
  return o + "]";
}
// machine-readable plan: the executed ops in order, for tests/oracle (oracle/net.py)
std::string plan_json(conv_pipe_t const &cp) {
  std::ostringstream o;
  o << "{\"name\":" << jstr(cp.name) << ",\"out_node\":" << jstr(cp.out_node) << ",\"inputs\":[";
  for (size_t i = 0; i < cp.inputs.size(); ++i)
    o << (i ? "," : "") << "{\"name\":" << jstr(cp.inputs[i]) << ",\"dims\":" << jdims(cp.node_dims.at(cp.inputs[i]))
      << "}";
  o << "],\"ops\":[";
  bool first = true;
  for (auto const &op : cp.ops) {
    if (op->fused) continue;
    o << (first ? "" : ",") << "{\"type\":" << jstr(op->type) << ",\"tag\":" << jstr(op->tag) << ",\"bots\":[";
    first = false;
    for (size_t i = 0; i < op->bots.size(); ++i) o << (i ? "," : "") << jstr(op->bots[i]);
    o << "],\"tops\":[";
    for (size_t i = 0; i < op->tops.size(); ++i) o << (i ? "," : "") << jstr(op->tops[i]);
    o << "],\"out_dims\":" << jdims(cp.node_dims.at(op->tops[0])) << ",\"k\":[" << op->ky << "," << op->kx
      << "],\"s\":[" << op->sy << "," << op->sx << "],\"p\":[" << op->py << "," << op->px
      << "],\"out_chans\":" << op->out_chans << ",\"bias\":" << (op->bias_term ? 1 : 0)
      << ",\"avg\":" << (op->avg_pool ? 1 : 0) << ",\"global\":" << (op->global_pool ? 1 : 0)
      << ",\"local_size\":" << op->local_size << ",\"alpha\":" << op->alpha << ",\"beta\":" << op->beta
      << ",\"kk\":" << op->k << ",\"eltwise\":" << jstr(op->eltwise_op) << ",\"relu\":" << (op->fused_relu ? 1 : 0)
      << "}";
  }
  o << "],\"ignored\":[";
  for (size_t i = 0; i < cp.ignored.size(); ++i) o << (i ? "," : "") << jstr(cp.ignored[i]);
  o << "]}";
  return o.str();
}
}  // namespace

int main(int argc, char **argv) {
  std::string net, out_node, save;
  uint32_t img = 0, iters = 3;
  int device = 0;
  bool plan = false, plan_js = false, plan_exec = false, pack = true, fold = true, inplace = true, resadd = true;
  uint32_t graph_reps = 0;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto val = [&]() -> std::string {
      if (i + 1 >= argc) {
        fprintf(stderr, "%s needs a value\n", a.c_str());
        exit(2);
      }
      return argv[++i];
    };
    if (a == "--net") net = val();
    else if (a == "--img") img = (uint32_t)atoi(val().c_str());
    else if (a == "--out-node") out_node = val();
    else if (a == "--iters") iters = (uint32_t)atoi(val().c_str());
    else if (a == "--device") device = atoi(val().c_str());
    else if (a == "--save") save = val();
    else if (a == "--plan") plan = true;
    else if (a == "--plan-json") plan_js = true;
    else if (a == "--plan-exec") plan_exec = true;
    else if (a == "--no-pack") pack = false;
    else if (a == "--no-fold") fold = false;
    else if (a == "--no-resadd") resadd = false;
    else if (a == "--graph") graph_reps = (uint32_t)atoi(val().c_str());
    else if (a == "--no-inplace-concat") inplace = false;
    else {
      fprintf(stderr, "unknown argument %s\n", a.c_str());
      return 2;
    }
  }
  if (net.empty()) {
    fprintf(stderr, "usage: boda_hip_rtc_fwd --net <prototxt> [--img N] [--out-node n] [--iters K] "
                    "[--plan|--plan-json|--plan-exec] [--save DIR] [--device d] [--no-pack] [--no-fold] [--no-inplace-concat] [--no-resadd] [--graph R]\n");
    return 2;
  }
  try {
    p_conv_pipe_t cp = create_pipe_from_prototxt(read_file(net), img, out_node);
    if (plan_exec) {  // the executor's folds / in-place Concat slabs (no GPU)
      conv_pipe_fwd_t fwd;
      fwd.cp = cp;
      if (fold) fwd.plan_folds();
      if (resadd) fwd.plan_resadds();
      if (inplace) fwd.plan_slabs();
      printf("%s", fwd.exec_plan_str().c_str());
      return 0;
    }
    if (plan || plan_js) {
      if (plan_js) printf("%s\n", plan_json(*cp).c_str());
      else {
        printf("%s", cp->plan_str().c_str());
        for (auto const &s : cp->ignored) printf("ignored %s\n", s.c_str());
      }
      return 0;
    }
    if (cp->inputs.size() != 1) rt_err("nets with one data input are supported");
    p_rtc_compute_t rtc = make_hip_compute(device);
    rtc->init();
    conv_pipe_fwd_t fwd;
    fwd.pack_filts = pack;
    fwd.fold_affines = fold;
    fwd.concat_in_place = inplace;
    fwd.fuse_residual = resadd;
    fwd.init(cp, rtc);
    auto in = std::make_shared<nda_t>(cp->node_dims.at(cp->inputs[0]));
    for (uint64_t i = 0; i < in->dims.elems(); ++i) in->elems()[i] = det_hash_rand((uint32_t)i + 234234567u);
    double best = 1e30;
    for (uint32_t it = 0; it < std::max(1u, iters); ++it) {
      fwd.run_fwd({{cp->inputs[0], in}});
      best = std::min(best, fwd.sum_ms());
    }
    double flops = 0;
    for (auto const &t : fwd.times) flops += t.flops;
    printf("net %s  plat %s  input %s  out %s %s\n", cp->name.c_str(), rtc->get_plat_tag().c_str(),
           cp->node_dims.at(cp->inputs[0]).str().c_str(), cp->out_node.c_str(),
           cp->node_dims.at(cp->out_node).str().c_str());
    for (auto const &t : fwd.times) {
      char rate[32] = "";
      if (t.flops > 0 && t.ms > 0) snprintf(rate, sizeof(rate), "%.1f GFLOP/s", t.flops / t.ms / 1e6);
      printf("  %-28s %-34s %9.4f ms %s\n", t.tag.c_str(), t.func.c_str(), t.ms, rate);
    }
    printf("total (best of %u) %.4f ms  conv GFLOP %.3f  %.1f GFLOP/s\n", std::max(1u, iters), best, flops / 1e9,
           flops / best / 1e6);
    if (graph_reps) {
      const double g = fwd.time_fwd_graph(graph_reps);
      printf("forward as one hipGraph (%zu calls, %u replays) %.4f ms  %.1f GFLOP/s\n", fwd.times.size(), graph_reps, g,
             flops / g / 1e6);
    }
    if (!save.empty()) {
      write_f32(save + "/in.f32", *in);
      write_f32(save + "/out.f32", *fwd.get(cp->out_node));
    }
  } catch (unsup_exception const &e) {
    fprintf(stderr, "unsupported: %s\n", e.what());
    return 3;
  } catch (std::exception const &e) {
    fprintf(stderr, "error: %s\n", e.what());
    return 1;
  }
  return 0;
}
