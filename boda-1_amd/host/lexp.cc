// lexp.cc -- recursive-descent parser for Boda's list expressions (see lexp.H).
#include "lexp.H"

#include "boda_host.H"

namespace boda_hip {

namespace {
struct parser_t {
  std::string const &s;
  size_t pos = 0;
  explicit parser_t(std::string const &s_) : s(s_) {}

  [[noreturn]] void err(std::string const &m) { rt_err("lexp parse error at " + std::to_string(pos) + ": " + m + " in '" + s + "'"); }

  std::string leaf() {
    std::string out;
    int depth = 0;
    while (pos < s.size()) {
      char c = s[pos];
      if (c == '\\' && pos + 1 < s.size()) {
        out += s[pos + 1];
        pos += 2;
        continue;
      }
      if (c == '(') ++depth;
      else if (c == ')') {
        if (!depth) break;
        --depth;
      } else if (c == ',' && !depth) break;
      out += c;
      ++pos;
    }
    return out;
  }

  p_lexp_t node() {
    auto n = std::make_shared<lexp_t>();
    if (pos < s.size() && s[pos] == '(') {
      n->is_list = true;
      ++pos;
      if (pos < s.size() && s[pos] == ')') {
        ++pos;
        return n;
      }
      while (true) {
        size_t eq = s.find('=', pos);
        if (eq == std::string::npos) err("expected name=");
        std::string name = s.substr(pos, eq - pos);
        if (name.empty() || name.find_first_of("(),") != std::string::npos) err("bad name '" + name + "'");
        for (auto const &k : n->kids)
          if (k.first == name) err("duplicate key '" + name + "'");
        pos = eq + 1;
        n->kids.emplace_back(name, node());
        if (pos >= s.size()) err("unterminated list");
        if (s[pos] == ',') {
          ++pos;
          continue;
        }
        if (s[pos] == ')') {
          ++pos;
          return n;
        }
        err(std::string("unexpected '") + s[pos] + "'");
      }
    }
    n->leaf = leaf();
    return n;
  }
};
}  // namespace

p_lexp_t parse_lexp(std::string const &s) {
  parser_t p(s);
  p_lexp_t r = p.node();
  if (p.pos != s.size()) p.err("trailing text");
  return r;
}

std::string lexp_t::str() const {
  if (!is_list) return leaf;
  std::string o = "(";
  for (size_t i = 0; i < kids.size(); ++i) {
    if (i) o += ",";
    o += kids[i].first + "=" + kids[i].second->str();
  }
  return o + ")";
}

}  // namespace boda_hip
