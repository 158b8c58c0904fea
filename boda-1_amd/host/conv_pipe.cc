// conv_pipe.cc -- Caffe prototxt reader, net plan (dims, ReLU fusion) and the forward
// executor over rtc_compute_t (be=hip). See conv_pipe.H for the reference map.
#include "conv_pipe.H"

#include <algorithm>

#include <cmath>
#include <cstring>
#include <set>
#include <sstream>

#include "boda_hip.h"
#include "op_desc.H"

namespace boda_hip {

// ---------------------------------------------------------------------------
// protobuf text format (the subset prototxts use: `name: value`, `name { ... }`,
// `name: { ... }`, # comments, quoted strings)
namespace {
struct pt_lexer {
  std::string const &s;
  size_t i = 0;
  uint32_t line = 1;
  explicit pt_lexer(std::string const &t) : s(t) {}
  void skip() {
    while (i < s.size()) {
      char c = s[i];
      if (c == '\n') { ++line; ++i; }
      else if (isspace((unsigned char)c) || c == ',' || c == ';') ++i;
      else if (c == '#') { while (i < s.size() && s[i] != '\n') ++i; }
      else break;
    }
  }
  [[noreturn]] void err(std::string const &m) { rt_err("prototxt line " + std::to_string(line) + ": " + m); }
  bool at_end() { skip(); return i >= s.size(); }
  char peek() { skip(); return i < s.size() ? s[i] : 0; }
  std::string word() {
    skip();
    size_t b = i;
    while (i < s.size() && !isspace((unsigned char)s[i]) && !strchr("{}:\"'#,;", s[i])) ++i;
    if (b == i) err(std::string("expected a name or value, saw '") + (i < s.size() ? s[i] : '?') + "'");
    return s.substr(b, i - b);
  }
  std::string quoted() {
    char q = s[i++];
    std::string out;
    while (i < s.size() && s[i] != q) {
      if (s[i] == '\\' && i + 1 < s.size()) ++i;
      if (s[i] == '\n') ++line;
      out += s[i++];
    }
    if (i >= s.size()) err("unterminated string");
    ++i;
    return out;
  }
};

p_pt_msg parse_body(pt_lexer &lx, bool top) {
  auto m = std::make_shared<pt_msg>();
  while (true) {
    char c = lx.peek();
    if (c == 0) {
      if (!top) lx.err("unexpected end of file inside a message");
      return m;
    }
    if (c == '}') {
      if (top) lx.err("unbalanced '}'");
      ++lx.i;
      return m;
    }
    pt_field f;
    f.name = lx.word();
    if (lx.peek() == ':') ++lx.i;
    c = lx.peek();
    if (c == '{') {
      ++lx.i;
      f.msg = parse_body(lx, false);
    } else if (c == '"' || c == '\'') {
      f.scalar = lx.quoted();
    } else {
      f.scalar = lx.word();
    }
    m->fields.push_back(f);
  }
}
}  // namespace

p_pt_msg parse_prototxt(std::string const &text) {
  pt_lexer lx(text);
  return parse_body(lx, true);
}

std::string pt_msg::get(std::string const &n, std::string const &dflt) const {
  for (auto const &f : fields)
    if (f.name == n && !f.msg) return f.scalar;
  return dflt;
}
bool pt_msg::has(std::string const &n) const {
  for (auto const &f : fields)
    if (f.name == n) return true;
  return false;
}
std::vector<std::string> pt_msg::all(std::string const &n) const {
  std::vector<std::string> r;
  for (auto const &f : fields)
    if (f.name == n && !f.msg) r.push_back(f.scalar);
  return r;
}
p_pt_msg pt_msg::sub(std::string const &n) const {
  for (auto const &f : fields)
    if (f.name == n && f.msg) return f.msg;
  return nullptr;
}
std::vector<p_pt_msg> pt_msg::subs(std::string const &n) const {
  std::vector<p_pt_msg> r;
  for (auto const &f : fields)
    if (f.name == n && f.msg) r.push_back(f.msg);
  return r;
}

// ---------------------------------------------------------------------------
// net plan
namespace {
uint32_t u32(std::string const &s, std::string const &what) {
  char *e = nullptr;
  unsigned long v = strtoul(s.c_str(), &e, 10);
  if (s.empty() || *e) rt_err("bad integer '" + s + "' for " + what);
  return (uint32_t)v;
}
float f32(std::string const &s, std::string const &what) {
  char *e = nullptr;
  float v = strtof(s.c_str(), &e);
  if (s.empty() || *e) rt_err("bad number '" + s + "' for " + what);
  return v;
}
// V1 (`layers { type: CONVOLUTION }`) -> V2 type names (caffe upgrade_proto's table)
std::string v2_type(std::string const &t) {
  static const std::map<std::string, std::string> m = {
      {"CONVOLUTION", "Convolution"}, {"POOLING", "Pooling"},   {"RELU", "ReLU"},
      {"LRN", "LRN"},                 {"CONCAT", "Concat"},     {"DROPOUT", "Dropout"},
      {"INNER_PRODUCT", "InnerProduct"}, {"DATA", "Data"},      {"SOFTMAX", "Softmax"},
      {"SOFTMAX_LOSS", "SoftmaxWithLoss"}, {"ACCURACY", "Accuracy"}, {"ELTWISE", "Eltwise"},
      {"SPLIT", "Split"}};
  auto it = m.find(t);
  return it == m.end() ? t : it->second;
}
// caffe layer inclusion for the TEST phase (the forward net; caffe NetState default)
bool included_for_test(pt_msg const &lp) {
  auto phase_of = [](p_pt_msg const &r) { return r ? r->get("phase", "") : std::string(); };
  auto inc = lp.subs("include");
  auto exc = lp.subs("exclude");
  for (auto const &r : exc)
    if (phase_of(r) == "TEST") return false;
  if (inc.empty()) return true;
  for (auto const &r : inc)
    if (phase_of(r).empty() || phase_of(r) == "TEST") return true;
  return false;
}
// kernel / stride / pad (y, x) from a convolution_param / pooling_param
void geom(pt_msg const &p, conv_op_t &op, bool need_kernel) {
  auto pick = [&](char const *both, char const *h, char const *w, uint32_t dflt, uint32_t &y, uint32_t &x) {
    auto v = p.all(both);
    y = x = dflt;
    if (v.size() == 1) y = x = u32(v[0], both);
    else if (v.size() >= 2) { y = u32(v[0], both); x = u32(v[1], both); }
    if (p.has(h)) y = u32(p.get(h), h);
    if (p.has(w)) x = u32(p.get(w), w);
  };
  pick("kernel_size", "kernel_h", "kernel_w", 0, op.ky, op.kx);
  pick("stride", "stride_h", "stride_w", 1, op.sy, op.sx);
  pick("pad", "pad_h", "pad_w", 0, op.py, op.px);
  if (need_kernel && (!op.ky || !op.kx)) rt_err("layer '" + op.tag + "': no kernel size");
}
dims_t nchw(uint32_t b, uint32_t c, uint32_t y, uint32_t x) {
  return dims_t({{"img", b}, {"chan", c}, {"y", y}, {"x", x}});
}
}  // namespace

p_conv_pipe_t create_pipe_from_prototxt(std::string const &text, uint32_t img, std::string const &out_node,
                                        bool det_dropout) {
  p_pt_msg net = parse_prototxt(text);
  auto cp = std::make_shared<conv_pipe_t>();
  cp->name = net->get("name", "net");
  // old-style top-level inputs: input + 4 input_dim each, or input_shape { dim ... }
  auto ins = net->all("input");
  auto idims = net->all("input_dim");
  auto ishapes = net->subs("input_shape");
  for (size_t i = 0; i < ins.size(); ++i) {
    std::vector<uint32_t> d;
    if (ishapes.size() == ins.size()) {
      for (auto const &s : ishapes[i]->all("dim")) d.push_back(u32(s, "input_shape.dim"));
    } else if (idims.size() == 4 * ins.size()) {
      for (int j = 0; j < 4; ++j) d.push_back(u32(idims[4 * i + j], "input_dim"));
    } else {
      rt_err("net inputs: need 4 input_dim or one input_shape per input");
    }
    if (d.size() != 4) unsup_err("net input '" + ins[i] + "' is not 4-D");
    if (img) d[0] = img;
    cp->inputs.push_back(ins[i]);
    cp->node_dims[ins[i]] = nchw(d[0], d[1], d[2], d[3]);
  }
  auto layers = net->subs("layer");
  for (auto const &l : net->subs("layers")) layers.push_back(l);  // V1 nets use `layers`
  bool found_out = false;
  for (auto const &lp : layers) {
    if (!included_for_test(*lp)) continue;
    auto op = std::make_shared<conv_op_t>();
    op->tag = lp->get("name");
    op->type = v2_type(lp->get("type"));
    op->bots = lp->all("bottom");
    op->tops = lp->all("top");
    bool keep = true;
    std::string why;
    if (op->type == "Convolution") {
      p_pt_msg p = lp->sub("convolution_param");
      if (!p) rt_err("layer '" + op->tag + "': no convolution_param");
      geom(*p, *op, true);
      op->out_chans = u32(p->get("num_output", "0"), "num_output");
      op->bias_term = p->get("bias_term", "true") != "false";
      if (p->has("group") && p->get("group") != "1") unsup_err("layer '" + op->tag + "': grouped convolution");
    } else if (op->type == "InnerProduct") {
      p_pt_msg p = lp->sub("inner_product_param");
      if (!p) rt_err("layer '" + op->tag + "': no inner_product_param");
      op->out_chans = u32(p->get("num_output", "0"), "num_output");
      op->bias_term = p->get("bias_term", "true") != "false";
    } else if (op->type == "Pooling") {
      p_pt_msg p = lp->sub("pooling_param");
      if (!p) rt_err("layer '" + op->tag + "': no pooling_param");
      op->global_pool = p->get("global_pooling", "false") == "true";
      geom(*p, *op, !op->global_pool);
      std::string pool = p->get("pool", "MAX");
      if (pool == "AVE") op->avg_pool = true;
      else if (pool != "MAX") unsup_err("layer '" + op->tag + "': pooling method " + pool);
    } else if (op->type == "LRN") {
      p_pt_msg p = lp->sub("lrn_param");
      if (p) {
        op->local_size = u32(p->get("local_size", "5"), "local_size");
        op->alpha = f32(p->get("alpha", "1"), "alpha");
        op->beta = f32(p->get("beta", "0.75"), "beta");
        op->k = f32(p->get("k", "1"), "k");
        if (p->get("norm_region", "ACROSS_CHANNELS") != "ACROSS_CHANNELS") unsup_err("LRN within channel");
      }
    } else if (op->type == "Eltwise") {
      p_pt_msg p = lp->sub("eltwise_param");
      if (p) op->eltwise_op = p->get("operation", "SUM");
      if (p && p->has("coeff")) unsup_err("layer '" + op->tag + "': Eltwise coefficients");
    } else if (op->type == "BatchNorm") {
      p_pt_msg p = lp->sub("batch_norm_param");
      op->k = p ? f32(p->get("eps", "1e-5"), "eps") : 1e-5f;
    } else if (op->type == "Scale") {
      p_pt_msg p = lp->sub("scale_param");
      op->bias_term = p && p->get("bias_term", "false") == "true";
    } else if (op->type == "Dropout") {
      // the forward (TEST) net: identity; in place -> no op, else a copy. det_dropout: the rtc
      // mode's deterministic mask (an in-place op, src/rtc_fwd.cc:348-358)
      p_pt_msg p = lp->sub("dropout_param");
      op->dropout_ratio = p ? f32(p->get("dropout_ratio", "0.5"), "dropout_ratio") : 0.5f;
      if (op->tops != op->bots) {
        // the rtc mode's dropout is an in-place op (src/rtc_fwd.cc:349 asserts it); the TEST-phase
        // identity of an out-of-place one is a copy, which is only right without det_dropout
        if (det_dropout) rt_err("layer '" + op->tag + "': det_dropout needs an in-place Dropout");
        op->type = "Copy";
      } else if (!det_dropout) { keep = false; why = "Dropout in place (identity at test time)"; }
    } else if (op->type == "Data") {
      p_pt_msg tp = lp->sub("transform_param"), dp = lp->sub("data_param");
      if (!tp || !dp) rt_err("Data layer '" + op->tag + "' without transform_param / data_param");
      uint32_t crop = u32(tp->get("crop_size", "0"), "crop_size");
      uint32_t bs = u32(dp->get("batch_size", "1"), "batch_size");
      if (!crop) unsup_err("Data layer '" + op->tag + "' without crop_size");
      if (op->tops.empty()) rt_err("Data layer without outputs");
      cp->inputs.push_back(op->tops[0]);
      cp->node_dims[op->tops[0]] = nchw(img ? img : bs, 3, crop, crop);  // src/caffepb.cc: 3-channel crops
      keep = false;
      why = "Data layer (source node " + op->tops[0] + ")";
    } else if (op->type == "ReLU" || op->type == "Concat") {
    } else if (op->type == "Softmax" || op->type == "SoftmaxWithLoss" || op->type == "Accuracy") {
      keep = false;
      why = op->type + " (not part of the forward feature net, as in the reference)";
    } else {
      keep = false;
      why = "unhandled layer type " + op->type;
    }
    bool has_out = false;
    for (auto const &t : op->tops)
      if (t == out_node) has_out = found_out = true;
    if (found_out && !has_out) break;
    if (keep) cp->ops.push_back(op);
    else cp->ignored.push_back(op->tag + ": " + why);
  }
  if (!out_node.empty() && !found_out) rt_err("out node '" + out_node + "' is not produced by any layer");
  cp->calc_dims();
  cp->fuse_relus();
  cp->out_node = out_node;
  if (cp->out_node.empty() && !cp->ops.empty()) cp->out_node = cp->ops.back()->tops.at(0);
  return cp;
}

void conv_pipe_t::calc_dims() {
  for (auto const &op : ops) {
    if (op->bots.empty() || op->tops.empty()) rt_err("layer '" + op->tag + "' needs inputs and outputs");
    for (auto const &b : op->bots)
      if (!node_dims.count(b)) rt_err("layer '" + op->tag + "': input '" + b + "' has no producer");
    dims_t const in = node_dims.at(op->bots[0]);
    const uint32_t B = in.dsz("img"), C = in.dsz("chan"), H = in.dsz("y"), W = in.dsz("x");
    dims_t out = in;
    if (op->type == "Convolution") {
      const uint32_t pin_y = H + 2 * op->py, pin_x = W + 2 * op->px;
      if (pin_y < op->ky || pin_x < op->kx) rt_err("layer '" + op->tag + "': padded input smaller than the kernel");
      out = nchw(B, op->out_chans, conv_in_sz_to_out_sz(H, op->py, op->ky, op->sy),
                 conv_in_sz_to_out_sz(W, op->px, op->kx, op->sx));
    } else if (op->type == "InnerProduct") {
      out = nchw(B, op->out_chans, 1, 1);  // a convolution whose window is the whole input (ipconv)
    } else if (op->type == "Pooling") {
      if (op->global_pool) {
        op->ky = H; op->kx = W; op->sy = op->sx = 1; op->py = op->px = 0;
      }
      auto psz = [](uint32_t n, uint32_t k, uint32_t s, uint32_t p) -> uint32_t {  // src/conv_util.cc:198-204
        uint32_t pin = n + 2 * p;
        return pin < k ? 1 : (pin - k + s - 1) / s + 1;
      };
      if (op->py >= op->ky || op->px >= op->kx) unsup_err("layer '" + op->tag + "': pooling pad >= kernel");
      out = nchw(B, C, psz(H, op->ky, op->sy, op->py), psz(W, op->kx, op->sx, op->px));
    } else if (op->type == "Concat") {
      uint32_t ct = 0;
      for (auto const &b : op->bots) {
        dims_t const &d = node_dims.at(b);
        if (d.dsz("img") != B || d.dsz("y") != H || d.dsz("x") != W)
          rt_err("Concat '" + op->tag + "': inputs differ outside the channel dim");
        ct += d.dsz("chan");
      }
      out = nchw(B, ct, H, W);
    } else if (op->type == "Eltwise") {
      for (auto const &b : op->bots)
        if (node_dims.at(b) != in) rt_err("Eltwise '" + op->tag + "': input dims differ");
      if (op->eltwise_op != "SUM" && op->eltwise_op != "PROD" && op->eltwise_op != "MAX")
        unsup_err("Eltwise operation " + op->eltwise_op);
    } else if (op->type == "LRN") {
      if (op->local_size % 2 == 0 || op->local_size > 11) unsup_err("LRN local_size must be odd and <= 11");
    }
    if (op->type != "ReLU" && op->type != "BatchNorm" && op->type != "Scale" && op->type != "LRN" &&
        op->type != "Copy" && op->tops.size() != 1)
      unsup_err("layer '" + op->tag + "' with " + std::to_string(op->tops.size()) + " outputs");
    for (auto const &t : op->tops) {
      if (node_dims.count(t) && node_dims.at(t) != out)
        rt_err("layer '" + op->tag + "' changes the dims of blob '" + t + "' it writes in place");
      node_dims[t] = out;
    }
  }
}

// A ReLU running in place on the output of a Convolution / InnerProduct / Eltwise / affine
// (BatchNorm+Scale) that produced it just before is folded into that op (conv_has_relu,
// src/cnn_op.cc:335-337; the reference's rtc_fwd fuses conv + ReLU the same way).
void conv_pipe_t::fuse_relus() {
  for (size_t i = 1; i < ops.size(); ++i) {
    conv_op_t &r = *ops[i];
    if (r.type != "ReLU" || r.bots.size() != 1 || r.tops != r.bots) continue;
    conv_op_t &p = *ops[i - 1];
    if (p.tops.size() != 1 || p.tops[0] != r.bots[0]) continue;
    if (p.type == "Convolution" || p.type == "InnerProduct" || p.type == "Eltwise" || p.type == "Scale" ||
        p.type == "BatchNorm") {
      p.fused_relu = true;
      r.fused = true;
    }
  }
}

std::string conv_pipe_t::plan_str() const {
  std::ostringstream o;
  for (auto const &in : inputs) o << "input " << in << " " << node_dims.at(in).str() << "\n";
  for (auto const &op : ops) {
    if (op->fused) continue;
    o << op->type << " " << op->tag << " ";
    for (size_t i = 0; i < op->bots.size(); ++i) o << (i ? "," : "") << op->bots[i];
    o << " -> " << op->tops[0] << " " << node_dims.at(op->tops[0]).str();
    if (op->type == "Convolution" || op->type == "Pooling")
      o << " k=" << op->ky << "x" << op->kx << " s=" << op->sy << "x" << op->sx << " p=" << op->py << "x" << op->px;
    if (op->type == "Pooling") o << (op->avg_pool ? " avg" : " max");
    if (op->fused_relu) o << " +relu";
    o << "\n";
  }
  return o.str();
}

// ---------------------------------------------------------------------------
// synthetic parameters (no caffemodel ships with the reference)
float det_hash_rand(uint32_t r) {  // test/rtc/gen-util.h:1-9
  uint32_t h = r;
  h ^= h >> 16;
  h *= 0x85ebca6bu;
  h ^= h >> 13;
  h *= 0xc2b2ae35u;
  h ^= h >> 16;
  return std::fma((float)h, 10.0f / 4294967295.0f, -5.0f);
}
uint32_t param_seed(std::string const &layer, std::string const &which) {  // FNV-1a of "layer/which"
  uint32_t h = 2166136261u;
  for (char c : layer + "/" + which) {
    h ^= (uint8_t)c;
    h *= 16777619u;
  }
  return h;
}
void synth_param(std::vector<float> &v, uint32_t seed, float scale) {
  for (size_t i = 0; i < v.size(); ++i) v[i] = det_hash_rand((uint32_t)i + seed) * scale;
}

// ---------------------------------------------------------------------------
// forward executor
void conv_pipe_fwd_t::add_call(std::string const &fn, conv_op_t const &op,
                               std::map<std::string, rtc_arg_t> const &args, double flops) {
  call_t c;
  c.rfc.rtc_func_name = fn;
  c.rfc.arg_map = args;
  c.tag = op.tag;
  c.flops = flops;
  calls.push_back(c);
}

namespace {
dims_t vec_dims(std::string const &n, uint32_t sz) { return dims_t({{n, sz}}); }
}  // namespace

// Inference BatchNorm (mean, var, eps) or Scale (gamma, beta) as out = in * sc[c] + sh[c];
// synthetic statistics: mean ~ U(-0.1, 0.1), var ~ U(0.5, 1.5), gamma ~ 1 + U(-0.1, 0.1)
void affine_params(conv_op_t const &op, uint32_t C, std::vector<float> &sc, std::vector<float> &sh) {
  sc.assign(C, 0.0f);
  sh.assign(C, 0.0f);
  std::vector<float> a(C), b(C);
  if (op.type == "BatchNorm") {
    synth_param(a, param_seed(op.tag, "mean"), 0.1f / 5.0f);
    synth_param(b, param_seed(op.tag, "var"), 0.5f / 5.0f);
    for (uint32_t c = 0; c < C; ++c) {
      const float var = 1.0f + b[c];
      sc[c] = 1.0f / std::sqrt(var + op.k);
      sh[c] = -a[c] * sc[c];
    }
  } else {
    synth_param(a, param_seed(op.tag, "gamma"), 0.1f / 5.0f);
    synth_param(b, param_seed(op.tag, "beta"), 0.1f / 5.0f);
    for (uint32_t c = 0; c < C; ++c) {
      sc[c] = 1.0f + a[c];
      sh[c] = op.bias_term ? b[c] : 0.0f;
    }
  }
}

// Inference-time folding: a BatchNorm / Scale running in place on the output of the
// Convolution / InnerProduct just before it (and of nothing else: no ReLU in between) is a
// per-output-channel affine of that conv's result, so it is folded into the conv's bank and
// biases at init (w' = w * s, b' = b * s + t): one kernel and one HBM round trip of the
// activation less per affine (resnet-50: 106 of its 230 layer calls). A ReLU fused into the
// last folded affine moves to the conv.
void conv_pipe_fwd_t::plan_folds() {
  folds.clear();
  folded.clear();
  conv_op_t const *tgt = nullptr;
  for (auto const &p : cp->ops) {
    conv_op_t const &op = *p;
    if ((op.type == "Convolution" || op.type == "InnerProduct") && op.tops.size() == 1) {
      tgt = op.fused_relu ? nullptr : &op;
    } else if ((op.type == "BatchNorm" || op.type == "Scale") && tgt && !op.fused && op.bots.size() == 1 &&
               op.tops == op.bots && op.bots[0] == tgt->tops[0]) {
      folds[tgt->tag].push_back(&op);
      folded.insert(op.tag);
      if (op.fused_relu) tgt = nullptr;
    } else {
      tgt = nullptr;
    }
  }
}

bool conv_pipe_fwd_t::conv_relu(conv_op_t const &conv) const {
  auto f = folds.find(conv.tag);
  return conv.fused_relu || (f != folds.end() && !f->second.empty() && f->second.back()->fused_relu);
}

// Residual add in the conv epilogue: an Eltwise SUM of two blobs, one of them written by the
// Convolution that runs just before it (no ReLU of its own, read by nothing else), becomes
// that conv's epilogue out = relu?(conv + bias + other) (bh_conv2d_fwd_nchw_res; the same
// adds in the same order, so bit-identical). ResNet-50: its 16 shortcut sums, one activation
// write + two reads less each.
void conv_pipe_fwd_t::plan_resadds() {
  resadds.clear();
  res_fused.clear();
  std::map<std::string, uint32_t> readers;
  for (auto const &p : cp->ops) {
    if (p->fused || folded.count(p->tag)) continue;
    for (auto const &b : p->bots) ++readers[b];
  }
  conv_op_t const *prev = nullptr;
  for (auto const &p : cp->ops) {
    conv_op_t const &op = *p;
    if (op.fused || folded.count(op.tag)) continue;
    if (op.type == "Eltwise" && op.eltwise_op == "SUM" && op.bots.size() == 2 && op.tops.size() == 1 && prev &&
        prev->type == "Convolution" && prev->tops.size() == 1 && !conv_relu(*prev)) {
      std::string const &cv = prev->tops[0];
      const int w = op.bots[0] == cv ? 0 : (op.bots[1] == cv ? 1 : -1);
      if (w >= 0) {
        std::string const &other = op.bots[1 - w];
        if (other != cv && readers[cv] == 1 && op.tops[0] != other && cv != cp->out_node &&
            cp->node_dims.at(other) == cp->node_dims.at(cv) && cp->node_dims.at(op.tops[0]) == cp->node_dims.at(cv)) {
          resadds[prev->tag] = {op.tag, op.tops[0], other, op.fused_relu};
          res_fused.insert(op.tag);
        }
      }
    }
    prev = &op;
  }
}

std::string conv_pipe_fwd_t::exec_plan_str() const {
  std::ostringstream o;
  for (auto const &kv : resadds)
    o << "resadd " << kv.second.eltwise << " -> " << kv.first << (kv.second.relu ? " +relu" : "") << "\n";
  for (auto const &kv : folds)
    for (conv_op_t const *a : kv.second) o << "fold " << a->type << " " << a->tag << " -> " << kv.first << "\n";
  for (auto const &kv : slabs) o << "slab " << kv.first << " -> " << kv.second.first << " @" << kv.second.second << "\n";
  return o.str();
}

// Concat in place: a Concat input produced by a Convolution / InnerProduct (out of place) and
// read by nothing but that Concat is written by the conv straight into its channel slab of the
// Concat's output (bh_conv2d_fwd_nchw_slab); the Concat then copies only its other inputs.
// The reference copies every input (src/rtc_fwd.cc:267-280). googlenet: 36 of its 36 Concat
// inputs, one activation write + read less each.
void conv_pipe_fwd_t::plan_slabs() {
  slabs.clear();
  std::map<std::string, conv_op_t const *> producer;
  std::map<std::string, uint32_t> readers;  // ops that run and read the blob
  for (auto const &p : cp->ops) {
    conv_op_t const &op = *p;
    if (op.fused || folded.count(op.tag) || res_fused.count(op.tag)) continue;
    for (auto const &b : op.bots) ++readers[b];
    for (auto const &t : op.tops) producer[t] = &op;
  }
  for (auto const &p : cp->ops) {
    conv_op_t const &op = *p;
    if (op.type != "Concat" || op.fused) continue;
    uint32_t oc0 = 0;
    for (auto const &b : op.bots) {
      auto pr = producer.find(b);
      const uint32_t nc = cp->node_dims.at(b).dsz("chan");
      const bool conv = pr != producer.end() && (pr->second->type == "Convolution" || pr->second->type == "InnerProduct");
      const bool src = std::find(cp->inputs.begin(), cp->inputs.end(), b) != cp->inputs.end();
      if (conv && !src && readers[b] == 1 && b != cp->out_node && pr->second->bots[0] != b &&
          std::count(op.bots.begin(), op.bots.end(), b) == 1)
        slabs[b] = {op.tops[0], oc0};
      oc0 += nc;
    }
  }
}

void conv_pipe_fwd_t::gen_op(conv_op_t const &op) {
  if (op.fused) return;
  dims_t const &in = cp->node_dims.at(op.bots[0]);
  dims_t const &out = cp->node_dims.at(op.tops[0]);
  const uint32_t B = in.dsz("img"), C = in.dsz("chan"), H = in.dsz("y"), W = in.dsz("x");
  const std::string fn_base = op.tag;
  op_base_t fo;
  fo.type = op.type;
  std::vector<rtc_func_info_t> fis;
  auto ensure_out = [&](std::string const &vn) {
    if (!declared.count(vn)) {
      rtc->create_var_with_dims(vn, cp->node_dims.at(vn));
      declared.insert(vn);
    }
  };
  if (op.type == "Convolution" || op.type == "InnerProduct") {
    const bool ip = op.type == "InnerProduct";
    const uint32_t KY = ip ? H : op.ky, KX = ip ? W : op.kx;
    fo.type = "Convolution";
    fo.dims_vals["in"] = in;
    fo.dims_vals["filts"] = dims_t({{"out_chan", op.out_chans}, {"in_chan", C}, {"y", KY}, {"x", KX}});
    fo.dims_vals["kern_sz"] = dims_t({{"y", KY}, {"x", KX}}, "none");
    fo.dims_vals["stride"] = dims_t({{"y", ip ? 1u : op.sy}, {"x", ip ? 1u : op.sx}}, "none");
    fo.dims_vals["in_pad"] = dims_t({{"y", ip ? 0u : op.py}, {"x", ip ? 0u : op.px}}, "none");
    fo.scalars["out_chans"] = op.out_chans;
    fo.scalars["conv_has_relu"] = op.fused_relu ? 1 : 0;
    fo.line = op.tag;
    add_hip_annotations(fo);
    conv_shape_t s = get_conv_shape(fo);
    // weights: synthetic, uploaded once at init (Boda's rtc_fwd copies caffe weights into vars)
    std::string fv = op.tag + "_filts", bv = op.tag + "_biases";
    rtc->create_var_with_dims(fv, fo.dims_vals["filts"]);
    std::vector<float> w((size_t)s.OC * s.IC * s.KY * s.KX);
    synth_param(w, param_seed(op.tag, "filts"), std::sqrt(3.0f / (float)(s.IC * s.KY * s.KX)) / 5.0f);
    std::vector<float> b(s.OC, 0.0f);
    if (op.bias_term && !force_zero_bias) synth_param(b, param_seed(op.tag, "biases"), 0.1f / 5.0f);
    auto fit = folds.find(op.tag);
    const bool fold = fit != folds.end();
    if (fold) {
      const size_t kk = (size_t)s.IC * s.KY * s.KX;
      std::vector<float> sc, sh;
      for (conv_op_t const *a : fit->second) {
        affine_params(*a, s.OC, sc, sh);
        for (uint32_t oc = 0; oc < s.OC; ++oc) {
          for (size_t k = 0; k < kk; ++k) w[oc * kk + k] *= sc[oc];
          b[oc] = b[oc] * sc[oc] + sh[oc];
        }
        if (a->fused_relu) fo.scalars["conv_has_relu"] = 1;
      }
    }
    upload(fv, w);
    const bool bias = op.bias_term || fold;
    if (bias) {
      rtc->create_var_with_dims(bv, fo.dims_vals["biases"]);
      upload(bv, b);
    }
    std::string ov = op.tops[0];
    auto sl = slabs.find(ov);
    if (sl != slabs.end()) {  // write the channel slab of the Concat's output
      ov = sl->second.first;
      fo.scalars["out_chan_ofs"] = sl->second.second;
    }
    auto ra = resadds.find(op.tag);
    if (ra != resadds.end()) {  // the Eltwise SUM (+ ReLU) after this conv, in its epilogue
      ov = ra->second.out;
      fo.scalars["conv_has_relu"] = ra->second.relu ? 1 : 0;
    }
    ensure_out(ov);
    std::string fn = "hip_conv__" + op.tag;
    rtc->compile({{fn, "", {}, fo}}, rtc_compile_opts_t());
    std::map<std::string, rtc_arg_t> args{{"in", op.bots[0]}, {"filts", fv}, {"out", ov}};
    if (bias) args["biases"] = bv;
    if (ra != resadds.end()) args["res"] = ra->second.res;
    if (pack_filts && !ip) {
      // Boda's xpose_filts at init (src/rtc_fwd.cc:306-326): the k-major bank the ring kernels read,
      // + the Winograd bank the conv's route reads (bh_conv_route_banks; pack_all_banks: all of them)
      uint32_t banks = BH_BANKS_ALL;
      if (!pack_all_banks) {
        const uint32_t d[11] = {s.B, s.IC, s.H, s.W, s.OC, s.KY, s.KX, s.sy, s.sx, s.py, s.px};
        if (bh_conv_route_banks(nullptr, d, &banks) != BH_OK) rt_err("bh_conv_route_banks: " + std::string(bh_last_error()));
      }
      fo.str_vals["hip_pack_banks"] = std::to_string(banks);
      rtc->compile({{fn, "", {}, fo}}, rtc_compile_opts_t());  // the conv reads the same mask
      const size_t nxp = bh_conv_filts_packed_floats_banks(s.OC, s.IC, s.KY, s.KX, banks);
      pack_bytes += nxp * 4;
      filt_bytes += (uint64_t)s.OC * s.IC * s.KY * s.KX * 4;
      std::string xv = op.tag + "_filts_xp";
      rtc->create_var_with_dims(xv, vec_dims("v", (uint32_t)nxp));
      std::string xfn = "hip_xpose_filts__" + op.tag;
      rtc->compile({{xfn, "", {}, fo}}, rtc_compile_opts_t());
      rtc_func_call_t xc;
      xc.rtc_func_name = xfn;
      xc.arg_map = {{"filts", fv}, {"filts_xp", xv}};
      rtc->run(xc);
      args["filts_xp"] = xv;
    }
    add_call(fn, op, args, 2.0 * B * s.OH * s.OW * (double)s.OC * s.IC * s.KY * s.KX);
    return;
  }
  if (op.type == "ReLU") {
    if (op.tops[0] != op.bots[0]) {  // not in place: copy then rectify
      ensure_out(op.tops[0]);
      fo.scalars = {{"ic0", 0}, {"oc0", 0}, {"nc", C}};
      rtc->compile({{"hip_copy__" + op.tag, "", {}, fo}}, rtc_compile_opts_t());
      add_call("hip_copy__" + op.tag, op, {{"in", op.bots[0]}, {"out", op.tops[0]}});
    }
    rtc->compile({{"hip_relu__" + op.tag, "", {}, fo}}, rtc_compile_opts_t());
    add_call("hip_relu__" + op.tag, op, {{"x", op.tops[0]}});
    return;
  }
  if (op.type == "Dropout") {  // in place; the seed is a call argument (set_det_drop_seed)
    char buf[64];
    snprintf(buf, sizeof(buf), "%.9g", op.dropout_ratio);
    fo.str_vals = {{"dropout_ratio", buf}};
    rtc->compile({{"hip_dropout__" + op.tag, "", {}, fo}}, rtc_compile_opts_t());
    add_call("hip_dropout__" + op.tag, op, {{"inout", op.tops[0]}, {"det_drop_seed", rtc_arg_t::u32(det_drop_seed)}});
    dropout_cixs.push_back((uint32_t)calls.size() - 1);
    return;
  }
  if (op.type == "Pooling") {
    ensure_out(op.tops[0]);
    fo.scalars = {{"ky", op.ky}, {"kx", op.kx}, {"sy", op.sy}, {"sx", op.sx},
                  {"py", op.py}, {"px", op.px}, {"avg", op.avg_pool ? 1u : 0u}};
    rtc->compile({{"hip_pool__" + op.tag, "", {}, fo}}, rtc_compile_opts_t());
    add_call("hip_pool__" + op.tag, op, {{"in", op.bots[0]}, {"out", op.tops[0]}});
    return;
  }
  if (op.type == "LRN") {
    if (op.tops[0] == op.bots[0]) unsup_err("LRN in place");
    ensure_out(op.tops[0]);
    fo.scalars = {{"local_size", op.local_size}};
    fo.str_vals = {{"alpha", std::to_string(op.alpha)}, {"beta", std::to_string(op.beta)}, {"k", std::to_string(op.k)}};
    char buf[64];
    snprintf(buf, sizeof(buf), "%.9g", op.alpha); fo.str_vals["alpha"] = buf;
    snprintf(buf, sizeof(buf), "%.9g", op.beta); fo.str_vals["beta"] = buf;
    snprintf(buf, sizeof(buf), "%.9g", op.k); fo.str_vals["k"] = buf;
    rtc->compile({{"hip_lrn__" + op.tag, "", {}, fo}}, rtc_compile_opts_t());
    add_call("hip_lrn__" + op.tag, op, {{"in", op.bots[0]}, {"out", op.tops[0]}});
    return;
  }
  if (op.type == "Concat" || op.type == "Copy") {
    ensure_out(op.tops[0]);
    uint32_t oc0 = 0;
    for (size_t i = 0; i < op.bots.size(); ++i) {
      const uint32_t nc = cp->node_dims.at(op.bots[i]).dsz("chan");
      if (slabs.count(op.bots[i])) {  // its producer wrote the slab already
        oc0 += nc;
        continue;
      }
      op_base_t f2 = fo;
      f2.scalars = {{"ic0", 0}, {"oc0", oc0}, {"nc", nc}};
      std::string fn = "hip_copy__" + op.tag + "_" + std::to_string(i);
      rtc->compile({{fn, "", {}, f2}}, rtc_compile_opts_t());
      add_call(fn, op, {{"in", op.bots[i]}, {"out", op.tops[0]}});
      oc0 += nc;
    }
    return;
  }
  if (op.type == "BatchNorm" || op.type == "Scale") {
    if (folded.count(op.tag)) return;  // folded into the producing Convolution's bank and biases
    std::vector<float> sc, sh;
    affine_params(op, C, sc, sh);
    std::string sv = op.tag + "_scale", tv = op.tag + "_shift";
    rtc->create_var_with_dims(sv, vec_dims("chan", C));
    rtc->create_var_with_dims(tv, vec_dims("chan", C));
    upload(sv, sc);
    upload(tv, sh);
    if (op.tops[0] != op.bots[0]) ensure_out(op.tops[0]);
    fo.scalars = {{"relu", op.fused_relu ? 1u : 0u}};
    rtc->compile({{"hip_affine__" + op.tag, "", {}, fo}}, rtc_compile_opts_t());
    add_call("hip_affine__" + op.tag, op, {{"in", op.bots[0]}, {"out", op.tops[0]}, {"scale", sv}, {"shift", tv}});
    return;
  }
  if (op.type == "Eltwise") {
    if (res_fused.count(op.tag)) return;  // in its producing conv's epilogue
    if (op.bots.size() != 2) unsup_err("Eltwise '" + op.tag + "' with " + std::to_string(op.bots.size()) + " inputs");
    if (op.tops[0] != op.bots[0] && op.tops[0] != op.bots[1]) ensure_out(op.tops[0]);
    const uint32_t code = op.eltwise_op == "PROD" ? 0 : (op.eltwise_op == "SUM" ? 1 : 2);
    fo.scalars = {{"op", code}, {"relu", op.fused_relu ? 1u : 0u}};
    rtc->compile({{"hip_eltwise__" + op.tag, "", {}, fo}}, rtc_compile_opts_t());
    add_call("hip_eltwise__" + op.tag, op, {{"a", op.bots[0]}, {"b", op.bots[1]}, {"out", op.tops[0]}});
    return;
  }
  (void)out;
  unsup_err("conv_pipe_fwd: no executor for layer type " + op.type);
}

void conv_pipe_fwd_t::upload(std::string const &vn, std::vector<float> const &v) {
  auto n = std::make_shared<nda_t>(rtc->get_var_dims(vn));
  if (n->dims.elems() != v.size()) rt_err("upload: size mismatch for " + vn);
  std::copy(v.begin(), v.end(), n->elems());
  rtc->copy_nda_to_var(vn, n);
}

void conv_pipe_fwd_t::init_with_rtc(p_conv_pipe_t const &cp_, p_rtc_compute_t const &rtc_) {
  cp = cp_;
  rtc = rtc_;
  for (auto const &in : cp->inputs) {
    rtc->create_var_with_dims(in, cp->node_dims.at(in));
    declared.insert(in);
  }
  if (fold_affines) plan_folds();
  if (fuse_residual) plan_resadds();
  if (concat_in_place) plan_slabs();
  for (auto const &op : cp->ops) gen_op(*op);
  rtc->finish_and_sync();
}

// src/rtc_fwd.cc:469-533: the mode's options from nia, the backend (NESI "rtc", default be=hip
// on device 0; Boda picks nvrtc / ocl by enabled feature), then the executor
void conv_pipe_fwd_t::init(p_conv_pipe_t const &cp_, nesi_init_arg_t *const nia) {
  if (!cp_) rt_err("conv_pipe_fwd_t::init: null conv_pipe");
  nesi_init_arg_t none;
  nesi_init_arg_t &a = nia ? *nia : none;
  enable_prof = a.get_u32("enable_prof", 1);
  enable_double_run = a.get_u32("enable_double_run", 0);
  enable_stats = a.get_u32("enable_stats", 0);
  force_zero_bias = a.get_u32("force_zero_bias", 0);
  per_call_fn = a.get_str("per_call_fn", "");
  graph_reps = a.get_u32("graph_reps", 0);
  pack_filts = a.get_bool("pack_filts", true);
  pack_all_banks = a.get_bool("pack_all_banks", false);
  fold_affines = a.get_bool("fold_affines", true);
  concat_in_place = a.get_bool("concat_in_place", true);
  fuse_residual = a.get_bool("fuse_residual", true);
  dump_vars.clear();
  if (a.has("dump_vars")) {  // "(0=blob,1=blob,...)" or "blob:blob"
    p_lexp_t l = a.nvm.at("dump_vars");
    a.used.insert("dump_vars");
    if (l->is_list) {
      for (auto const &k : l->kids) dump_vars.push_back(k.second->leaf);
    } else {
      std::string v = l->leaf;
      for (size_t b = 0; b <= v.size();) {
        size_t e = v.find(':', b);
        if (e == std::string::npos) e = v.size();
        if (e > b) dump_vars.push_back(v.substr(b, e - b));
        b = e + 1;
      }
    }
  }
  p_lexp_t rl = parse_lexp(a.get_str("rtc", "(be=hip)"));
  nesi_init_arg_t ra(rl);
  const std::string be = ra.get_str("be", "hip");
  if (be != "hip") unsup_err("rtc mode: backend be=" + be + " is not built here (this backend provides be=hip)");
  const int device = (int)ra.get_u32("device", 0);
  ra.check_unused();
  a.check_unused();
  if (!rtc) {
    rtc = make_hip_compute(device);
    rtc->init();
  }
  init_with_rtc(cp_, rtc);
}

void conv_pipe_fwd_t::set_det_drop_seed(uint32_t const &det_drop_seed_) {  // src/rtc_fwd.cc:91-99
  det_drop_seed = det_drop_seed_;
  for (uint32_t i : dropout_cixs) {
    auto it = calls.at(i).rfc.arg_map.find("det_drop_seed");
    if (it == calls.at(i).rfc.arg_map.end()) rt_err("set_det_drop_seed: dropout call without a seed argument");
    it->second = rtc_arg_t::u32(det_drop_seed_);
  }
}

// src/rtc_fwd.cc:535-577
void conv_pipe_fwd_t::run_fwd(vect_string const &to_set_vns, p_map_str_p_nda_t const &fwd,
                              vect_string const &to_get_vns) {
  if (!rtc) rt_err("conv_pipe_fwd_t::run_fwd before init");
  if (!fwd) rt_err("conv_pipe_fwd_t::run_fwd: null fwd map");
  if (enable_double_run)
    for (auto const &c : calls) rtc->run(c.rfc);
  rtc->finish_and_sync();
  for (auto const &vn : to_set_vns) {  // copy sources in
    auto it = fwd->find(vn);
    if (it == fwd->end() || !it->second) rt_err("run_fwd: no input nda named '" + vn + "'");
    if (!declared.count(vn)) rt_err("run_fwd: '" + vn + "' is not a var of this net");
    rtc->copy_nda_to_var(vn, it->second);
  }
  rtc->finish_and_sync();
  rtc->release_per_call_id_data();
  std::vector<uint32_t> ids;
  for (auto const &c : calls) ids.push_back(rtc->run(c.rfc));
  rtc->finish_and_sync();
  for (auto const &vn : to_get_vns) {  // copy requested vars out
    if (!declared.count(vn))
      rt_err("run_fwd: blob '" + vn + "' has no var (a rewrite keeps it only inside another op's output)");
    (*fwd)[vn] = rtc->create_nda_from_var(vn);
  }
  times.clear();
  for (size_t i = 0; i < calls.size(); ++i) {
    layer_time_t t;
    t.tag = calls[i].tag;
    t.func = calls[i].rfc.rtc_func_name;
    t.ms = rtc->get_dur(ids[i], ids[i]);  // every call has its event pair (src/rtc_fwd.cc:563)
    t.flops = calls[i].flops;
    times.push_back(t);
  }
  if (!per_call_fn.empty()) {
    FILE *f = fopen(per_call_fn.c_str(), "w");
    if (!f) rt_err("cannot write per_call_fn " + per_call_fn);
    const double dur = ids.empty() ? 0.0 : rtc->get_dur(ids.front(), ids.back());
    fprintf(f, "net.args.runtime=%.9g\n", dur / 1000.0);
    for (auto const &t : times)
      fprintf(f, "per_layer_time['%s']=per_layer_time.get('%s',0.0) + %.9g # %s \n", t.tag.c_str(), t.tag.c_str(),
              t.ms / 1000.0, t.func.c_str());
    // (the reference also appends cp->dump_ops, its op-graph dump, src/rtc_fwd.cc:568: this
    // backend's equivalent is boda_hip_rtc_fwd --plan-exec, not written here)
    fclose(f);
  }
  stats_map.clear();
  if (enable_stats) {
    for (auto const &vn : to_get_vns) {
      nda_t const &n = *fwd->at(vn);
      double mn = 0, mx = 0, sum = 0;
      const uint64_t cnt = n.dims.elems();
      for (uint64_t i = 0; i < cnt; ++i) {
        const double v = n.elems()[i];
        mn = i ? std::min(mn, v) : v;
        mx = i ? std::max(mx, v) : v;
        sum += v;
      }
      stats_map[vn + "_min"] = mn;
      stats_map[vn + "_max"] = mx;
      stats_map[vn + "_sum"] = sum;
      stats_map[vn + "_cnt"] = (double)cnt;
    }
  }
  graph_ms = graph_reps ? time_fwd_graph(graph_reps) : 0.0;
  rtc->release_per_call_id_data();
  rtc->finish_and_sync();
}

// src/rtc_fwd.cc:140-161: dumped vars and stats; plus (enable_prof) the per-call times of the
// last forward and, with graph_reps, the forward as one replayed hipGraph
std::string conv_pipe_fwd_t::get_info_log(void) {
  std::string ret;
  char buf[512];
  if (enable_prof) {
    double flops = 0;
    for (auto const &t : times) {
      char rate[32] = "";
      if (t.flops > 0 && t.ms > 0) snprintf(rate, sizeof(rate), "%.1f GFLOP/s", t.flops / t.ms / 1e6);
      snprintf(buf, sizeof(buf), "  %-28s %-34s %9.4f ms %s\n", t.tag.c_str(), t.func.c_str(), t.ms, rate);
      ret += buf;
      flops += t.flops;
    }
    snprintf(buf, sizeof(buf), "forward %.4f ms  conv GFLOP %.3f  %.1f GFLOP/s\n", sum_ms(), flops / 1e9,
             sum_ms() > 0 ? flops / sum_ms() / 1e6 : 0.0);
    ret += buf;
    if (graph_reps) {
      snprintf(buf, sizeof(buf), "forward as one hipGraph (%zu calls, %u replays) %.4f ms  %.1f GFLOP/s\n",
               times.size(), graph_reps, graph_ms, graph_ms > 0 ? flops / graph_ms / 1e6 : 0.0);
      ret += buf;
    }
    snprintf(buf, sizeof(buf), "resident filter packs %.1f MB (%.2fx the %.1f MB of filters%s)\n", pack_bytes / 1e6,
             filt_bytes ? (double)pack_bytes / filt_bytes : 0.0, filt_bytes / 1e6,
             pack_all_banks ? ", every Winograd bank" : ", the banks each route reads");
    ret += buf;
  }
  for (auto const &vn : dump_vars) {
    p_nda_t n = rtc->create_nda_from_var(vn);
    ret += "dumping var '" + vn + "'\n";
    for (uint64_t i = 0; i < n->dims.elems(); ++i) {
      snprintf(buf, sizeof(buf), "[%llu]: %.9g\n", (unsigned long long)i, n->elems()[i]);
      ret += buf;
    }
  }
  for (auto const &kv : stats_map) {
    snprintf(buf, sizeof(buf), "%s=%.9g\n", kv.first.c_str(), kv.second);
    ret += buf;
  }
  return ret;
}

double conv_pipe_fwd_t::time_fwd_graph(uint32_t reps) {
  return rtc->time_graph([&] { for (auto const &c : calls) rtc->run(c.rfc); }, reps);
}

double conv_pipe_fwd_t::sum_ms() const {
  double s = 0;
  for (auto const &t : times) s += t.ms;
  return s;
}

}  // namespace boda_hip
