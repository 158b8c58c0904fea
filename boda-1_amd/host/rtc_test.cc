// rtc_test.cc -- boda_hip_rtc_test: Boda's rtc_test mode (src/rtc_compute.cc:135-194), the
// minimal conformance test of an rtc_compute_t backend, on be=hip.
//
// Reads a CUCL program (--prog-fn), compiles it through the backend's compile() (for a
// function the backend does not intercept: hiprtc JIT with the CUCL prelude), creates vars a,
// b, c of --data-sz floats (a, b uniform in [2.5, 7.5), c = 123.456), runs --func-name with
// args (a, b, c, n) -- n by value: a uint32_t (my_dot) or a struct holding one (my_dot_struct),
// the same bytes -- at tpb 256, copies c back and checks c[i] == a[i] + b[i] within 1e-6.
// Writes "All is Well." (the reference's verdict, test/good_tr/test_rtc_nvrtc/rtc_test.txt) or
// the first bad element to --out-fn (default stdout), and exits 0 / 1.
#include <cmath>
#include <cstdio>
#include <fstream>
#include <iostream>
#include <map>
#include <random>
#include <sstream>

#include "rtc_compute.H"

using namespace boda_hip;

int main(int argc, char **argv) {
  std::map<std::string, std::string> kv;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    size_t eq = a.find('=');
    if (a.rfind("--", 0) != 0 || eq == std::string::npos) {
      std::cerr << "usage: boda_hip_rtc_test --prog-fn=F.cucl [--func-name=my_dot] [--data-sz=10000] "
                   "[--out-fn=F] [--device=0]\n";
      return 2;
    }
    kv[a.substr(2, eq - 2)] = a.substr(eq + 1);
  }
  try {
    std::ifstream pf(kv["prog-fn"]);
    if (!pf) rt_err("cannot read --prog-fn '" + kv["prog-fn"] + "'");
    std::stringstream ss;
    ss << pf.rdbuf();
    const std::string fn = kv.count("func-name") ? kv["func-name"] : "my_dot";
    const uint32_t n = kv.count("data-sz") ? parse_u32(kv["data-sz"], "data-sz") : 10000u;
    p_rtc_compute_t rtc = make_hip_compute(kv.count("device") ? parse_i32(kv["device"], "device") : 0);
    rtc->init();
    op_base_t dot;
    dot.func_name = fn;
    rtc->compile({rtc_func_info_t{fn, ss.str(), {"a", "b", "c", "n"}, dot}}, rtc_compile_opts_t());

    dims_t d({{"v", n}});
    std::mt19937 gen(0);
    std::uniform_real_distribution<float> u(2.5f, 7.5f);
    p_nda_t a = std::make_shared<nda_t>(d), b = std::make_shared<nda_t>(d), c = std::make_shared<nda_t>(d);
    for (uint32_t i = 0; i < n; ++i) {
      a->elems()[i] = u(gen);
      b->elems()[i] = u(gen);
      c->elems()[i] = 123.456f;
    }
    for (auto const &x : {std::make_pair("a", a), std::make_pair("b", b), std::make_pair("c", c)}) {
      rtc->create_var_with_dims(x.first, d);
      rtc->copy_nda_to_var(x.first, x.second);
    }
    rtc_func_call_t rfc;
    rfc.rtc_func_name = fn;
    rfc.arg_map["a"] = rtc_arg_t("a");
    rfc.arg_map["b"] = rtc_arg_t("b");
    rfc.arg_map["c"] = rtc_arg_t("c");
    rfc.arg_map["n"] = rtc_arg_t::u32(n);
    rfc.tpb = 256;
    rfc.blks = (n + rfc.tpb - 1) / rfc.tpb;
    rtc->run(rfc);
    rtc->finish_and_sync();
    rtc->copy_var_to_nda(c, "c");
    rtc->release_all_funcs();
    std::ofstream of;
    std::ostream *out = &std::cout;
    if (kv.count("out-fn")) {
      of.open(kv["out-fn"]);
      out = &of;
    }
    for (uint32_t i = 0; i < n; ++i) {
      const float x = a->elems()[i], y = b->elems()[i], z = c->elems()[i];
      if (std::fabs((x + y) - z) > 1e-6f) {
        *out << "bad res: i=" << i << " a[i]=" << x << " b[i]=" << y << " c[i]=" << z << "\n";
        return 1;
      }
    }
    *out << "All is Well.\n";
    return 0;
  } catch (rt_exception const &e) {
    std::cerr << "error: " << e.what() << "\n";
    return 3;
  }
}
