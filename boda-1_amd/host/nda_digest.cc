// nda_digest.cc -- see nda_digest.H
#include "nda_digest.H"

#include <cmath>
#include <cstring>
#include <functional>
#include <istream>
#include <limits>
#include <ostream>
#include <random>
#include <set>
#include <sstream>

namespace boda_hip {

namespace {

uint32_t floor_log2_u64(uint64_t v) {
  uint32_t r = 0;
  while (v >>= 1) ++r;
  return r;
}

// boost::random::uniform_int_distribution<uint64_t>(0, range) over mt19937
// (32-bit engine range 0xFFFFFFFF): the bucket-rejection branch; range 0 draws nothing.
uint64_t boost_uniform(std::mt19937 &g, uint64_t range) {
  if (range == 0) return 0;
  const uint32_t brange = 0xFFFFFFFFu, r = (uint32_t)range;
  uint32_t bucket = brange / (r + 1u);
  if (brange % (r + 1u) == r) ++bucket;
  for (;;) {
    uint32_t res = (uint32_t)g() / bucket;
    if (res <= r) return res;
  }
}

// little-endian binary writer/reader for the bwrite/bread layout
struct bw_t {
  std::string b;
  template <typename T> void raw(T const &v) { b.append((char const *)&v, sizeof(T)); }
  void str(std::string const &s) {
    raw((uint32_t)s.size());
    b += s;
  }
};
struct br_t {
  std::string const &b;
  size_t o = 0;
  explicit br_t(std::string const &b_) : b(b_) {}
  template <typename T> T raw() {
    if (o + sizeof(T) > b.size()) rt_err("digest decode: truncated");
    T v;
    std::memcpy(&v, b.data() + o, sizeof(T));
    o += sizeof(T);
    return v;
  }
  std::string str() {
    uint32_t n = raw<uint32_t>();
    if (o + n > b.size()) rt_err("digest decode: truncated string");
    std::string s = b.substr(o, n);
    o += n;
    return s;
  }
};
const uint32_t NDD_VER1 = 0xdada0101u;

}  // namespace

uint64_t digest_seed_for(std::string const &var_name) { return (uint64_t)std::hash<std::string>()(var_name); }

double min_sig_mag_rel_diff(double min_sig_mag, double v1, double v2) {
  double a1 = std::fabs(v1), a2 = std::fabs(v2);
  double amax = std::max(min_sig_mag, std::max(a1, a2));
  return std::fabs(v2 - v1) / amax;
}

std::vector<digest_sample_t> nda_digest_t::plan() const {
  std::set<uint64_t> strides;
  for (uint64_t p : {1, 2, 3, 5, 7, 11, 13, 17, 19, 23, 29})
    if (p <= strides_sz) strides.insert(p);
  for (auto const &d : dims.d) strides.insert(d.stride);
  strides.insert(strides_sz);
  std::mt19937 gen((uint32_t)seed);
  std::vector<digest_sample_t> sis;
  for (uint64_t stride : strides) {
    if (!stride || stride > strides_sz) rt_err("digest: bad stride");
    uint32_t n = floor_log2_u64(stride + 1);
    std::set<uint64_t> seen;
    for (uint32_t i = 0; i < n; ++i) {
      uint64_t off = boost_uniform(gen, stride - 1);
      if (!seen.insert(off).second) continue;
      sis.push_back({stride, off, (strides_sz - off) / stride});
    }
  }
  return sis;
}

nda_digest_t nda_digest_t::make(float const *v, dims_t const &dims, uint64_t seed) {
  nda_digest_t d;
  d.dims = dims;
  d.dims.calc_strides();
  d.strides_sz = dims.elems();
  d.seed = seed;
  d.min_v = std::numeric_limits<float>::max();
  d.max_v = std::numeric_limits<float>::lowest();
  for (uint64_t i = 0; i < d.strides_sz; ++i) {
    d.min_v = std::min(d.min_v, v[i]);
    d.max_v = std::max(d.max_v, v[i]);
  }
  for (auto const &si : d.plan()) {
    float sv = 0.0f;  // sequential fp32 strided checksum
    for (uint64_t i = si.offset; i < d.strides_sz; i += si.stride) sv += v[i];
    d.samps.push_back(sv);
  }
  return d;
}

std::string nda_digest_t::mrd_comp(nda_digest_t const &o, double mrd, double *worst) const {
  if (dims != o.dims) return "nda_digest dims mismatch";
  if (seed != o.seed) return "nda_digest seed mismatch";
  std::vector<digest_sample_t> sis = plan();
  if (sis.size() != samps.size() || o.samps.size() != samps.size()) return "nda_digest sample count mismatch";
  std::string ret;
  double w = 0;
  auto check = [&](std::string const &tag, double v1, double v2, double tol) {
    double rd = min_sig_mag_rel_diff(1.0, v1, v2);
    w = std::max(w, rd / tol);
    if (rd > tol) ret += " [" + tag + "]: v1=" + std::to_string(v1) + " v2=" + std::to_string(v2) + "\n";
  };
  check("min_v", min_v, o.min_v, mrd);
  check("max_v", max_v, o.max_v, mrd);
  for (size_t i = 0; i < samps.size(); ++i) {
    double adj = mrd;
    if (sis[i].num_subsamps > 1000) adj *= std::sqrt(sis[i].num_subsamps / 1000.0);
    check("stride=" + std::to_string(sis[i].stride) + ",offset=" + std::to_string(sis[i].offset), samps[i],
          o.samps[i], adj);
  }
  if (worst) *worst = w;
  return ret;
}

std::string nda_digest_t::to_hex() const {
  bw_t w;
  w.raw((uint8_t)1);  // non-null shared_ptr
  w.str(dims.tn);
  w.raw(NDD_VER1);
  w.raw(self_cmp_mrd);
  w.raw((uint32_t)dims.d.size());
  for (auto const &d : dims.d) {
    w.raw(d.sz);
    w.raw(d.stride);
    w.str(d.name);
  }
  w.str(dims.tn);
  w.raw(strides_sz);
  w.raw((uint8_t)1);  // strides_valid
  w.raw(seed);
  w.raw(min_v);
  w.raw(max_v);
  w.raw((uint32_t)samps.size());
  for (float s : samps) w.raw(s);
  static const char *hx = "0123456789ABCDEF";
  std::string h;
  for (unsigned char c : w.b) {
    h += hx[c >> 4];
    h += hx[c & 15];
  }
  return h;
}

nda_digest_t nda_digest_t::from_hex(std::string const &h) {
  if (h.size() % 2) rt_err("digest hex: odd length");
  std::string b;
  for (size_t i = 0; i < h.size(); i += 2) b += (char)parse_u32(h.substr(i, 2), "hex byte", 16);
  br_t r(b);
  if (r.raw<uint8_t>() != 1) rt_err("digest hex: null digest");
  std::string tn = r.str();
  if (tn != "float") unsup_err("digest hex: element type " + tn + " (only float digests are used on this path)");
  if (r.raw<uint32_t>() != NDD_VER1) rt_err("digest hex: bad magic");
  nda_digest_t d;
  d.self_cmp_mrd = r.raw<double>();
  uint32_t nd = r.raw<uint32_t>();
  for (uint32_t i = 0; i < nd; ++i) {
    dim_t x;
    x.sz = r.raw<uint32_t>();
    x.stride = r.raw<uint32_t>();
    x.name = r.str();
    d.dims.d.push_back(x);
  }
  d.dims.tn = r.str();
  d.strides_sz = r.raw<uint64_t>();
  r.raw<uint8_t>();
  d.seed = r.raw<uint64_t>();
  d.min_v = r.raw<float>();
  d.max_v = r.raw<float>();
  uint32_t ns = r.raw<uint32_t>();
  for (uint32_t i = 0; i < ns; ++i) d.samps.push_back(r.raw<float>());
  if (r.o != b.size()) rt_err("digest hex: trailing bytes");
  return d;
}

namespace {
bool getline_nocr(std::istream &in, std::string &l) {
  if (!std::getline(in, l)) return false;
  if (!l.empty() && l.back() == '\r') l.pop_back();
  return true;
}
std::string must_getline(std::istream &in) {
  std::string l;
  if (!getline_nocr(in, l)) rt_err("wisdom: unexpected EOF");
  return l;
}
}  // namespace

bool read_next_wisdom(std::istream &in, op_wisdom_t &w) {
  std::string l;
  do {
    if (!getline_nocr(in, l)) return false;
  } while (l.empty());
  if (l != "op_wisdom_t") rt_err("wisdom: expected 'op_wisdom_t', saw '" + l + "'");
  w = op_wisdom_t();
  w.op_line = must_getline(in);
  while (true) {
    l = must_getline(in);
    if (l == "/op_wisdom_t") return true;
    if (l == "kg") {
      std::string vn = must_getline(in);
      w.kgs.emplace_back(vn, nda_digest_t::from_hex(must_getline(in)));
    } else if (l == "op_tune_wisdom_t") {
      std::pair<std::string, std::vector<op_run_t>> t;
      t.first = must_getline(in);
      while (true) {
        l = must_getline(in);
        if (l == "/op_tune_wisdom_t") break;
        if (l != "op_run_t") rt_err("wisdom: unknown op_tune_wisdom_t command '" + l + "'");
        op_run_t r;
        r.plat_tag = must_getline(in);
        r.rt_secs = parse_f64(must_getline(in), "run time");
        r.err = must_getline(in);
        if (r.err.empty()) r.op_line = must_getline(in);
        t.second.push_back(r);
      }
      w.tunes.push_back(t);
    } else {
      rt_err("wisdom: unknown op_wisdom_t command '" + l + "'");
    }
  }
}

void write_wisdom(std::ostream &out, op_wisdom_t const &w) {
  out << "op_wisdom_t\n" << w.op_line << "\n";
  for (auto const &k : w.kgs) out << "kg\n" << k.first << "\n" << k.second.to_hex() << "\n";
  for (auto const &t : w.tunes) {
    out << "op_tune_wisdom_t\n" << t.first << "\n";
    for (auto const &r : t.second) {
      out << "op_run_t\n" << r.plat_tag << "\n" << r.rt_secs << "\n" << r.err << "\n";
      if (r.err.empty()) out << r.op_line << "\n";
    }
    out << "/op_tune_wisdom_t\n";
  }
  out << "/op_wisdom_t\n";
}

namespace {
std::string num_str(double v) {  // str(double) of the reference: a default ostream (src/str_util.H:107-111)
  std::ostringstream s;
  s << v;
  return s.str();
}
}  // namespace

// comp_vars for one var pair (src/comp_util.cc:21-57 with ssds_diff_t, src/boda_base.cc:126-207)
bool comp_var(std::ostream &out, std::string const &vn, dims_t const &dims, std::vector<float> const &o1,
              std::vector<float> const &o2, double toler, uint32_t max_err, double *mrd_out) {
  double ssds = 0, sds = 0, mad = 0, mrd = 0, s1 = 0, s2 = 0;
  uint64_t ndiff = 0;
  const size_t n = o1.size();
  for (size_t i = 0; i < n; ++i) {
    s1 += o1[i];
    s2 += o2[i];
    const double d = double(o2[i]) - double(o1[i]);
    sds += d;
    ssds += d * d;
    mad = std::max(mad, std::fabs(d));
    mrd = std::max(mrd, min_sig_mag_rel_diff(1.0, o1[i], o2[i]));
    ndiff += o1[i] != o2[i];
  }
  const bool nan = std::isnan(ssds) || std::isnan(sds) || std::isnan(mad);
  *mrd_out = nan ? NAN : mrd;
  if (!(mrd >= toler || nan)) return false;
  out << vn << ": DIMS[" << dims.str() << "] ssds_str(out_batch_1,out_batch_2)=cnt=" << ndiff
      << " sum_squared_diffs=" << num_str(ssds) << " avg_abs_diff=" << num_str(std::sqrt(ssds / n))
      << " max_abs_diff=" << num_str(mad) << " sum_diffs=" << num_str(sds) << " avg_diff=" << num_str(sds / n)
      << " max_rel_diff=" << num_str(mrd) << " avg1=" << num_str(s1 / n) << " avg2=" << num_str(s2 / n) << "\n";
  uint32_t nerr = 0;
  for (size_t i = 0; i < n; ++i) {
    if (std::fabs(min_sig_mag_rel_diff(1.0, o1[i], o2[i])) < toler) continue;
    std::string ix;  // dims_t::ix_str: name=index per dim
    size_t r = i;
    for (size_t k = dims.d.size(); k-- > 0;) {
      ix = dims.d[k].name + "=" + std::to_string(r % dims.d[k].sz) + (ix.empty() ? "" : ":") + ix;
      r /= dims.d[k].sz;
    }
    out << "[" << ix << "]: v1=" << num_str(o1[i]) << " v2=" << num_str(o2[i]) << " \n";
    if (++nerr > max_err) break;
  }
  return true;
}

}  // namespace boda_hip
