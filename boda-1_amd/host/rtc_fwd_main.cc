// rtc_fwd_main.cc -- boda_hip_rtc_fwd: full-net forward of a Caffe prototxt through Boda's net-level
// plugin surface, has_conv_fwd_t (src/has_conv_fwd.H:16-25), mode "rtc" over be=hip -- the
// counterpart of Boda's `boda rtc_fwd` / test_compute net runs (src/rtc_fwd.cc:469-577). The driver
// uses only that surface: make_p_has_conv_fwd_t("rtc"), init(cp, nia), set_det_drop_seed,
// run_fwd(to_set_vns, fwd, to_get_vns), get_info_log. Parameters are synthetic (conv_pipe.H); the
// input is gen_data mode 5 (det_hash_rand(i + 234234567), the reference's Convolution `in` seed).
//
//   boda_hip_rtc_fwd --net nets/alexnet/train_val.prototxt [--img 20] [--out-node pool5]
//                    [--iters 5] [--plan | --plan-json | --plan-exec] [--save DIR] [--save-blobs DIR
//                    [--blob-sample N]] [--device 0] [--no-pack] [--no-fold] [--no-inplace-concat]
//                    [--no-resadd] [--graph R] [--det-dropout SEED] [--mode-args "(k=v,...)"]
//
// --plan / --plan-json print the net plan without touching a GPU (host logic tests); --plan-exec
// the executor's BatchNorm/Scale folds and in-place Concat slabs. Mode options (nia): --no-pack
// pack_filts=0, --no-fold fold_affines=0 (BatchNorm / Scale as separate affine layers),
// --no-inplace-concat concat_in_place=0 (every Concat input copied), --no-resadd fuse_residual=0
// (ResNet shortcut Eltwise SUM as its own layer), --graph R graph_reps=R (the whole forward also
// timed as one hipGraph replayed R times), --device d rtc=(be=hip,device=d); --mode-args adds any
// other (e.g. "(enable_stats=1,per_call_fn=t.py)"). --det-dropout keeps in-place Dropout layers
// and runs them with the reference's deterministic mask seeded by set_det_drop_seed(SEED).
// --save writes DIR/in.f32 and DIR/out.f32 (raw little-endian fp32) for the parity tests;
// --save-blobs every blob of the net as DIR/blob_<blob>.f32 (names with '/' -> '_') with
// DIR/blobs.json (dims, sample stride): with --blob-sample N every ceil(elems/N)-th element. Every
// blob has a var only with the rewrites off (--no-fold is not needed: folds keep the blob names;
// --no-inplace-concat --no-resadd are): run_fwd raises for a blob a rewrite keeps only inside
// another op's output, as the reference's copy_vars_to_ndas does for a missing var.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <set>
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
      << ",\"kk\":" << op->k << ",\"ratio\":" << op->dropout_ratio << ",\"eltwise\":" << jstr(op->eltwise_op) << ",\"relu\":" << (op->fused_relu ? 1 : 0)
      << "}";
  }
  o << "],\"ignored\":[";
  for (size_t i = 0; i < cp.ignored.size(); ++i) o << (i ? "," : "") << jstr(cp.ignored[i]);
  o << "]}";
  return o.str();
}
}  // namespace

int main(int argc, char **argv) {
  std::string net, out_node, save, save_blobs, mode_args;
  uint32_t img = 0, iters = 3, blob_sample = 0;
  int device = 0;
  bool plan = false, plan_js = false, plan_exec = false, pack = true, fold = true, inplace = true, resadd = true;
  bool det_dropout = false;
  uint32_t graph_reps = 0, drop_seed = 0;
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
    else if (a == "--save-blobs") save_blobs = val();
    else if (a == "--blob-sample") blob_sample = (uint32_t)atoi(val().c_str());
    else if (a == "--plan") plan = true;
    else if (a == "--plan-json") plan_js = true;
    else if (a == "--plan-exec") plan_exec = true;
    else if (a == "--no-pack") pack = false;
    else if (a == "--no-fold") fold = false;
    else if (a == "--no-resadd") resadd = false;
    else if (a == "--graph") graph_reps = (uint32_t)atoi(val().c_str());
    else if (a == "--no-inplace-concat") inplace = false;
    else if (a == "--det-dropout") {
      det_dropout = true;
      drop_seed = (uint32_t)strtoul(val().c_str(), nullptr, 0);
    } else if (a == "--mode-args") mode_args = val();
    else {
      fprintf(stderr, "unknown argument %s\n", a.c_str());
      return 2;
    }
  }
  if (net.empty()) {
    fprintf(stderr, "usage: boda_hip_rtc_fwd --net <prototxt> [--img N] [--out-node n] [--iters K] "
                    "[--plan|--plan-json|--plan-exec] [--save DIR] [--save-blobs DIR [--blob-sample N]] [--device d] "
                    "[--no-pack] [--no-fold] [--no-inplace-concat] [--no-resadd] [--graph R] [--det-dropout SEED] "
                    "[--mode-args (k=v,...)]\n");
    return 2;
  }
  try {
    p_conv_pipe_t cp = create_pipe_from_prototxt(read_file(net), img, out_node, det_dropout);
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
    // the mode's init arguments (NESI's name -> lexp map)
    nesi_init_arg_t nia(mode_args.empty() ? nullptr : parse_lexp(mode_args));
    nia.set("rtc", "(be=hip,device=" + std::to_string(device) + ")");
    if (!pack) nia.set("pack_filts", "0");
    if (!fold) nia.set("fold_affines", "0");
    if (!inplace) nia.set("concat_in_place", "0");
    if (!resadd) nia.set("fuse_residual", "0");
    if (graph_reps) nia.set("graph_reps", std::to_string(graph_reps));
    p_has_conv_fwd_t fwd = make_p_has_conv_fwd_t("rtc");
    fwd->init(cp, &nia);
    if (det_dropout) fwd->set_det_drop_seed(drop_seed);

    std::string const in_vn = cp->inputs[0];
    auto in = std::make_shared<nda_t>(cp->node_dims.at(in_vn));
    for (uint64_t i = 0; i < in->dims.elems(); ++i) in->elems()[i] = det_hash_rand((uint32_t)i + 234234567u);
    // blobs fetched: the output, or every blob the forward holds (--save-blobs)
    vect_string gets{cp->out_node};
    if (!save_blobs.empty()) {
      gets.clear();
      std::set<std::string> seen;
      for (auto const &op : cp->ops)
        for (auto const &t : op->tops)
          if (seen.insert(t).second) gets.push_back(t);
    }
    p_map_str_p_nda_t fmap = std::make_shared<map_str_p_nda_t>();
    (*fmap)[in_vn] = in;
    std::string best_log;
    double best = 1e30;
    for (uint32_t it = 0; it < std::max(1u, iters); ++it) {
      fwd->run_fwd({in_vn}, fmap, gets);
      std::string log = fwd->get_info_log();
      // "forward <ms> ms" line of the info log: keep the fastest forward's log
      size_t p = log.find("\nforward ");
      const double ms = p == std::string::npos ? 0.0 : atof(log.c_str() + p + 9);
      if (ms < best || best_log.empty()) {
        best = ms;
        best_log = log;
      }
    }
    printf("net %s  input %s  out %s %s  (best of %u forwards)\n", cp->name.c_str(),
           cp->node_dims.at(in_vn).str().c_str(), cp->out_node.c_str(), cp->node_dims.at(cp->out_node).str().c_str(),
           std::max(1u, iters));
    printf("%s", best_log.c_str());
    if (!save.empty()) {
      write_f32(save + "/in.f32", *in);
      write_f32(save + "/out.f32", *fmap->at(cp->out_node));
    }
    if (!save_blobs.empty()) {
      std::string idx = "{\"blobs\":[";
      bool first = true;
      for (auto const &g : gets) {
        nda_t const &n = *fmap->at(g);
        const uint64_t ne = n.dims.elems();
        const uint64_t stride = blob_sample ? std::max<uint64_t>(1, (ne + blob_sample - 1) / blob_sample) : 1;
        std::string fn = g;
        for (auto &c : fn)
          if (c == '/') c = '_';
        fn = "blob_" + fn + ".f32";
        FILE *f = fopen((save_blobs + "/" + fn).c_str(), "wb");
        if (!f) rt_err("cannot write " + save_blobs + "/" + fn);
        for (uint64_t i = 0; i < ne; i += stride) fwrite(n.elems() + i, 4, 1, f);
        fclose(f);
        idx += std::string(first ? "" : ",") + "{\"name\":" + jstr(g) + ",\"file\":" + jstr(fn) +
               ",\"dims\":" + jdims(n.dims) + ",\"stride\":" + std::to_string(stride) + "}";
        first = false;
      }
      idx += "]}";
      FILE *f = fopen((save_blobs + "/blobs.json").c_str(), "w");
      if (!f) rt_err("cannot write " + save_blobs + "/blobs.json");
      fputs(idx.c_str(), f);
      fclose(f);
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
