// has_conv_fwd.cc -- the mode's init-argument map and the mode factory (has_conv_fwd.H).
#include "has_conv_fwd.H"

#include <cstdlib>

#include "conv_pipe.H"

namespace boda_hip {

lexp_name_val_map_t::lexp_name_val_map_t(p_lexp_t const &l) {
  if (!l) return;
  if (!l->is_list) {
    if (!l->leaf.empty()) rt_err("mode arguments must be a (name=value,...) list, not '" + l->leaf + "'");
    return;
  }
  for (auto const &k : l->kids) {
    if (nvm.count(k.first)) rt_err("mode argument '" + k.first + "' given twice");
    nvm[k.first] = k.second;
  }
}

void lexp_name_val_map_t::set(std::string const &n, std::string const &v) {
  auto l = std::make_shared<lexp_t>();
  l->leaf = v;
  nvm[n] = l;
}

std::string lexp_name_val_map_t::get_str(std::string const &n, std::string const &dflt) {
  auto it = nvm.find(n);
  if (it == nvm.end()) return dflt;
  used.insert(n);
  return it->second->is_list ? it->second->str() : it->second->leaf;
}

uint32_t lexp_name_val_map_t::get_u32(std::string const &n, uint32_t dflt) {
  auto it = nvm.find(n);
  if (it == nvm.end()) return dflt;
  used.insert(n);
  std::string const &v = it->second->leaf;
  char *e = nullptr;
  const unsigned long x = strtoul(v.c_str(), &e, 0);
  if (it->second->is_list || v.empty() || *e) rt_err("mode argument " + n + "='" + v + "' is not a uint32");
  return (uint32_t)x;
}

void lexp_name_val_map_t::check_unused() const {  // src/lexp.cc lexp_check_unused
  std::string bad;
  for (auto const &kv : nvm)
    if (!used.count(kv.first)) bad += (bad.empty() ? "" : ", ") + kv.first;
  if (!bad.empty()) rt_err("unused mode arguments: " + bad);
}

p_has_conv_fwd_t make_p_has_conv_fwd_t(std::string const &mode) {
  if (mode == "rtc") return std::make_shared<conv_pipe_fwd_t>();
  unsup_err("has_conv_fwd_t mode '" + mode + "' is not provided by this backend (modes: rtc)");
}

}  // namespace boda_hip
