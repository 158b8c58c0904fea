// bh_jit.hip -- generic device functions compiled at run time through hiprtc: the rtc_compute_t
// contract for every function name the backend does not intercept (the reference JIT-compiles
// all CUCL through nvrtc: nvrtc_compute_t::compile / nvrtc_compile, src/nvrtc_util.cc:216-260,
// and launches them with cuLaunchKernel, :355-385). The hot ops never come here -- they are the
// precompiled gfx950 kernels of the other sources; this path serves Boda's helper CUCL (its
// rtc_test's dot.cucl, layout transforms, ...) so the backend is a complete rtc_compute_t.
//
// A module is one hiprtc program (the caller's full source, CUCL prelude included) built for
// gfx950 and loaded into the context's device; functions are looked up by name at compile time
// (a missing name fails the compile, as the reference's check_runnable does). Launches are 1-D
// blks x tpb on the context's stream; an event pair armed by bh_time_next_call is recorded on
// the launch itself (hipExtModuleLaunchKernel), so get_dur covers just the kernel.
#include "bh_common.h"
#include <hip/hiprtc.h>
#include <cstring>

namespace {

struct jit_module_t {
  hipModule_t mod = nullptr;
  std::map<std::string, hipFunction_t> funcs;
};

std::mutex g_jit_mu;
std::map<std::pair<bh_ctx *, int>, jit_module_t> g_modules;  // (context, module id)
int g_next_module = 0;

void put_log(char *log, size_t loglen, std::string const &s) {
  if (!log || !loglen) return;
  std::snprintf(log, loglen, "%s", s.c_str());
}

// hiprtc build for gfx950: code object bytes, or an error with the compiler log
int build(const char *src, const char *opts, std::vector<char> &code, std::string &log) {
  hiprtcProgram prog;
  if (hiprtcCreateProgram(&prog, src, "boda_cucl.cu", 0, nullptr, nullptr) != HIPRTC_SUCCESS)
    return bh::fail(BH_ERR, "hiprtcCreateProgram failed");
  std::vector<std::string> o = {"--offload-arch=gfx950", "-O3"};
  if (opts && *opts) {  // extra options, space separated
    std::string s(opts);
    size_t b = 0;
    while (b < s.size()) {
      size_t e = s.find(' ', b);
      if (e == std::string::npos) e = s.size();
      if (e > b) o.push_back(s.substr(b, e - b));
      b = e + 1;
    }
  }
  std::vector<const char *> ov;
  for (auto const &x : o) ov.push_back(x.c_str());
  const hiprtcResult r = hiprtcCompileProgram(prog, (int)ov.size(), ov.data());
  size_t ls = 0;
  if (hiprtcGetProgramLogSize(prog, &ls) == HIPRTC_SUCCESS && ls > 1) {
    log.resize(ls);
    hiprtcGetProgramLog(prog, &log[0]);
    log.resize(strlen(log.c_str()));
  }
  if (r != HIPRTC_SUCCESS) {
    hiprtcDestroyProgram(&prog);
    return bh::fail(BH_ERR, std::string("hiprtc compile failed: ") + hiprtcGetErrorString(r) + "\n" + log);
  }
  size_t cs = 0;
  hiprtcGetCodeSize(prog, &cs);
  code.resize(cs);
  hiprtcGetCode(prog, code.data());
  hiprtcDestroyProgram(&prog);
  return BH_OK;
}

}  // namespace

extern "C" {

int bh_jit_build(const char *src, const char *opts, char *log, size_t loglen, size_t *code_bytes) {
  if (!src) return bh::fail(BH_ERR, "null source");
  std::vector<char> code;
  std::string l;
  const int rc = build(src, opts, code, l);
  put_log(log, loglen, rc == BH_OK ? l : bh_last_error());
  if (code_bytes) *code_bytes = code.size();
  return rc;
}

int bh_jit_compile(bh_ctx *c, const char *src, const char *const *names, int n, const char *opts, int *module_id,
                   char *log, size_t loglen) {
  BH_ENTER(c);
  if (!src || !module_id || (n > 0 && !names)) return bh::fail(BH_ERR, "null argument");
  *module_id = -1;
  std::vector<char> code;
  std::string l;
  int rc = build(src, opts, code, l);
  put_log(log, loglen, rc == BH_OK ? l : bh_last_error());
  if (rc != BH_OK) return rc;
  jit_module_t m;
  BH_HIP(hipModuleLoadData(&m.mod, code.data()));
  for (int i = 0; i < n; ++i) {
    hipFunction_t f = nullptr;
    if (hipModuleGetFunction(&f, m.mod, names[i]) != hipSuccess) {
      (void)hipModuleUnload(m.mod);
      return bh::fail(BH_ERR, std::string("jit: no function '") + names[i] + "' in the compiled module");
    }
    m.funcs[names[i]] = f;
  }
  std::lock_guard<std::mutex> g(g_jit_mu);
  *module_id = g_next_module++;
  g_modules[{c, *module_id}] = m;
  return BH_OK;
}

int bh_jit_launch(bh_ctx *c, int module_id, const char *name, void **args, uint32_t blks, uint32_t tpb) {
  BH_ENTER_CALL(c);
  if (!name) return bh::fail(BH_ERR, "null function name");
  if (!blks || !tpb) return bh::fail(BH_ERR, std::string("jit launch of '") + name + "' with zero blks or tpb");
  if ((uint64_t)blks * tpb > 0xffffffffull) return bh::fail(BH_UNSUP, "jit launch: grid too large");
  // the lock is held until the launch is enqueued: a concurrent bh_jit_release then unloads the
  // module only after its stream has run this launch (it synchronises the stream after erasing)
  std::lock_guard<std::mutex> g(g_jit_mu);
  auto it = g_modules.find({c, module_id});
  if (it == g_modules.end()) return bh::fail(BH_ERR, "jit launch: unknown module");
  auto fit = it->second.funcs.find(name);
  if (fit == it->second.funcs.end())
    return bh::fail(BH_ERR, std::string("jit launch: '") + name + "' is not a function of the module");
  // global size in work-items (hipExtModuleLaunchKernel takes the grid in threads)
  BH_HIP(hipExtModuleLaunchKernel(fit->second, blks * tpb, 1, 1, tpb, 1, 1, 0, c->stream, args, nullptr, c->t_start,
                                  c->t_stop, 0));
  return BH_OK;
}

int bh_jit_release(bh_ctx *c, int module_id) {
  BH_ENTER(c);
  jit_module_t m;
  {
    std::lock_guard<std::mutex> g(g_jit_mu);
    auto it = g_modules.find({c, module_id});
    if (it == g_modules.end()) return bh::fail(BH_ERR, "jit release: unknown module");
    m = it->second;
    g_modules.erase(it);
  }
  BH_HIP(hipStreamSynchronize(c->stream));
  BH_HIP(hipModuleUnload(m.mod));
  return BH_OK;
}

}  // extern "C"

namespace bh {
// modules of a context being destroyed (bh_destroy)
void jit_release_all(bh_ctx *c) {
  std::lock_guard<std::mutex> g(g_jit_mu);
  for (auto it = g_modules.begin(); it != g_modules.end();) {
    if (it->first.first == c) {
      (void)hipModuleUnload(it->second.mod);
      it = g_modules.erase(it);
    } else {
      ++it;
    }
  }
}
}  // namespace bh
