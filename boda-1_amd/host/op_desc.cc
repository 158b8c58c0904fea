// op_desc.cc -- see op_desc.H
#include "op_desc.H"

#include <algorithm>
#include <fstream>

#include "lexp.H"

namespace boda_hip {

std::string dims_t::str() const {
  std::string o = "(";
  if (tn != "float") o += "tn=" + tn + ",";
  o += "dims=(";
  for (size_t i = 0; i < d.size(); ++i) o += (i ? "," : "") + d[i].name + "=" + std::to_string(d[i].sz);
  return o + "))";
}

namespace {
dims_t dims_from_lexp(lexp_t const &l, std::string const &tn) {
  std::vector<std::pair<std::string, uint32_t>> nd;
  std::string t = tn;
  for (auto const &k : l.kids) {
    if (k.first == "__tn__") {
      t = k.second->leaf;
      continue;
    }
    if (k.second->is_list) rt_err("nested list where a dimension size was expected");
    nd.emplace_back(k.first, parse_u32(k.second->leaf, "dim size"));
  }
  return dims_t(nd, t);
}
}  // namespace

op_base_t parse_op_line(std::string const &line) {
  p_lexp_t t = parse_lexp(line);
  if (!t->is_list) rt_err("op line is not a list: " + line);
  op_base_t op;
  op.line = line;
  p_lexp_t sv = t->find("str_vals"), nv = t->find("nda_vals");
  if (nv || (sv && sv->is_list && sv->find("type"))) {  // current dialect
    for (auto const &k : t->kids)
      if (k.first != "str_vals" && k.first != "nda_vals") rt_err("unused input: " + k.first);
    if (!sv || !sv->find("type")) rt_err("op line without str_vals.type: " + line);
    for (auto const &k : sv->kids) {
      if (k.first == "type") op.type = k.second->leaf;
      else if (k.first == "func_name") op.func_name = k.second->leaf;
      else op.str_vals[k.first] = k.second->leaf;
    }
    if (nv)
      for (auto const &k : nv->kids) {
        lexp_t const &n = *k.second;
        p_lexp_t tn = n.find("tn"), dims = n.find("dims"), v = n.find("v");
        std::string tns = tn ? tn->leaf : "float";
        if (dims) op.dims_vals[k.first] = dims_from_lexp(*dims, tns);
        else if (v) op.scalars[k.first] = parse_u64(v->leaf, "scalar " + k.first);
        else rt_err("nda '" + k.first + "' has neither dims nor v");
      }
    return op;
  }
  p_lexp_t ty = t->find("type");  // legacy dialect
  if (!ty) rt_err("unrecognised op line: " + line);
  op.type = ty->leaf;
  for (auto const &k : t->kids) {
    if (k.first == "type") continue;
    if (k.first == "dims_vals") {
      for (auto const &d : k.second->kids) op.dims_vals[d.first] = dims_from_lexp(*d.second, "float");
    } else if (k.first == "str_vals") {
      for (auto const &s : k.second->kids) {
        std::string const &v = s.second->leaf;
        bool num = !v.empty() && std::all_of(v.begin(), v.end(), ::isdigit);
        if (num) op.scalars[s.first] = parse_u64(v, "scalar " + s.first);
        else op.str_vals[s.first] = v;
      }
    } else {
      rt_err("unused input: " + k.first);
    }
  }
  // legacy dims-only ndas carry no element type: kern_sz / stride / in_pad are 'none'
  for (char const *n : {"kern_sz", "stride", "in_pad"})
    if (op.dims_vals.count(n)) op.dims_vals[n].tn = "none";
  return op;
}

std::vector<op_base_t> read_op_list(std::string const &fn, size_t *skipped, std::vector<std::string> const &types) {
  std::ifstream f(fn);
  if (!f) rt_err("cannot open op list '" + fn + "'");
  std::vector<op_base_t> out;
  std::string line;
  size_t sk = 0;
  while (std::getline(f, line)) {
    while (!line.empty() && (line.back() == '\r' || line.back() == ' ')) line.pop_back();
    if (line.empty()) continue;
    op_base_t op = parse_op_line(line);
    if (std::find(types.begin(), types.end(), op.type) == types.end()) {
      ++sk;
      continue;
    }
    out.push_back(op);
  }
  if (skipped) *skipped = sk;
  return out;
}

uint32_t conv_in_sz_to_out_sz(uint32_t in, uint32_t pad, uint32_t k, uint32_t stride) {
  uint32_t p = in + 2 * pad;
  if (p < k) return 0;
  return (p - k) / stride + 1;
}

conv_shape_t get_conv_shape(op_base_t const &op) {
  if (op.type != "Convolution") rt_err("not a Convolution op: " + op.type);
  dims_t const &in = op.get_dims("in"), &f = op.get_dims("filts");
  dims_t const &ks = op.get_dims("kern_sz"), &st = op.get_dims("stride"), &pd = op.get_dims("in_pad");
  conv_shape_t s;
  s.B = in.dsz("img"); s.IC = in.dsz("chan"); s.H = in.dsz("y"); s.W = in.dsz("x");
  s.OC = f.dsz("out_chan"); s.KY = ks.dsz("y"); s.KX = ks.dsz("x");
  s.sy = st.dsz("y"); s.sx = st.dsz("x"); s.py = pd.dsz("y"); s.px = pd.dsz("x");
  s.OH = conv_in_sz_to_out_sz(s.H, s.py, s.KY, s.sy);
  s.OW = conv_in_sz_to_out_sz(s.W, s.px, s.KX, s.sx);
  if (f.dsz("in_chan") != s.IC || f.dsz("y") != s.KY || f.dsz("x") != s.KX)
    rt_err("filts dims inconsistent with in / kern_sz: " + op.line);
  if (op.has_dims("out")) {
    dims_t const &o = op.get_dims("out");
    if (o.dsz("img") != s.B || o.dsz("chan") != s.OC || o.dsz("y") != s.OH || o.dsz("x") != s.OW)
      rt_err("out dims inconsistent with conv_in_sz_to_out_sz: " + op.line);
  }
  auto oc = op.scalars.find("out_chans");
  if (oc != op.scalars.end() && oc->second != s.OC) rt_err("out_chans mismatch: " + op.line);
  return s;
}

sgemm_shape_t get_sgemm_shape(op_base_t const &op) {
  if (op.type != "sgemm") rt_err("not an sgemm op: " + op.type);
  dims_t const &a = op.get_dims("a"), &b = op.get_dims("b"), &c = op.get_dims("c");
  sgemm_shape_t s{a.dsz("M"), b.dsz("N"), a.dsz("K")};
  if (b.dsz("K") != s.K || c.dsz("M") != s.M || c.dsz("N") != s.N) rt_err("sgemm dims inconsistent: " + op.line);
  if (a.tn != "float" || b.tn != "float" || c.tn != "float")
    unsup_err("hip backend sgemm is fp32 only (half-storage sgemm is out of scope)");
  return s;
}

op_work_t op_work(op_base_t const &op) {
  op_work_t w;
  if (op.type == "Convolution") {
    conv_shape_t s = get_conv_shape(op);
    double M = (double)s.B * s.OH * s.OW, K = (double)s.IC * s.KY * s.KX, N = s.OC;
    w.flops = 2 * M * N * K;
    w.bytes = 4.0 * ((double)s.B * s.IC * s.H * s.W + (double)s.B * s.OC * s.OH * s.OW + N * K + N);
  } else if (op.type == "sgemm") {
    sgemm_shape_t s = get_sgemm_shape(op);
    w.flops = 2.0 * s.M * s.N * s.K;
    w.bytes = 4.0 * ((double)s.M * s.K + (double)s.K * s.N + (double)s.M * s.N);
  } else {
    rt_err("op_work: unhandled op type " + op.type);
  }
  return w;
}

double roofline_secs(op_work_t const &w) { return std::max(w.flops / PEAK_FP32_FLOPS, w.bytes / PEAK_HBM_BPS); }

void add_hip_annotations(op_base_t &op) {
  if (op.type == "Convolution") {
    conv_shape_t s = get_conv_shape(op);
    op.func_name = "hip_conv";
    op.dims_vals["in"] = dims_t({{"img", s.B}, {"chan", s.IC}, {"y", s.H}, {"x", s.W}});
    op.dims_vals["filts"] = dims_t({{"out_chan", s.OC}, {"in_chan", s.IC}, {"y", s.KY}, {"x", s.KX}});
    op.dims_vals["biases"] = dims_t({{"out_chan", s.OC}});
    op.dims_vals["out"] = dims_t({{"img", s.B}, {"chan", s.OC}, {"y", s.OH}, {"x", s.OW}});
    if (op.str_vals.count("conv_has_relu") == 0 && op.scalars.count("conv_has_relu") == 0)
      op.scalars["conv_has_relu"] = 1;  // ops-prof always fuses ReLU (src/cnn_op.cc:335-337)
    return;
  }
  if (op.type == "sgemm") {
    get_sgemm_shape(op);
    op.func_name = "hip_sgemm";
    return;
  }
  unsup_err("hip backend: no kernel for op type '" + op.type + "'");
}

std::string hip_op_tune_t::str() const {
  std::string r;
  auto add = [&](std::string const &k, std::string const &v) { r += (r.empty() ? "" : ",") + k + "=" + v; };
  if (!use_be.empty()) add("use_be", use_be);
  if (!cfg.empty()) add("cfg", cfg);
  if (splits) add("splits", std::to_string(splits));
  if (wt >= 0) add("wt", std::to_string(wt));
  return "(" + r + ")";
}

hip_op_tune_t parse_hip_op_tune(std::string const &s) {
  p_lexp_t l = parse_lexp(s);
  hip_op_tune_t t;
  if (!l->is_list) rt_err("op_tune: expected a (k=v,...) list, got '" + s + "'");
  for (auto const &kv : l->kids) {
    if (kv.second->is_list) rt_err("op_tune: field '" + kv.first + "' is a list");
    std::string const &v = kv.second->leaf;
    try {
      if (kv.first == "use_be") t.use_be = v;
      else if (kv.first == "cfg") t.cfg = v;
      else if (kv.first == "splits") t.splits = parse_i32(v, "splits");
      else if (kv.first == "wt") t.wt = parse_i32(v, "wt");
      else rt_err("op_tune: unknown field '" + kv.first + "' (use_be, cfg, splits, wt)");
    } catch (std::logic_error const &) {
      rt_err("op_tune: bad value '" + v + "' for " + kv.first);
    }
  }
  if (!t.use_be.empty() && t.use_be != "hip") unsup_err("op_tune: use_be=" + t.use_be + " is not this backend");
  if (t.wt < -1 || t.wt > 1) rt_err("op_tune: wt must be -1, 0 or 1");
  return t;
}

void add_hip_annotations(op_base_t &op, hip_op_tune_t const &tune) {
  add_hip_annotations(op);
  if (!tune.cfg.empty()) op.str_vals["hip_cfg"] = tune.cfg;
  if (tune.splits) op.str_vals["hip_splits"] = std::to_string(tune.splits);
  if (tune.wt >= 0) op.str_vals["hip_wt"] = std::to_string(tune.wt);
}

}  // namespace boda_hip
