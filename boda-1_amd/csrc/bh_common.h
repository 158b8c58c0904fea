// bh_common.h -- internal declarations shared by the libboda_hip.so sources.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdint.h>
#include <algorithm>
#include <dlfcn.h>
#include <map>
#include <mutex>
#include <string>
#include <vector>
#include "boda_hip.h"

struct bh_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  hipDeviceProp_t prop{};
  std::vector<hipEvent_t> events;  // pool; ids index into it
  int events_used = 0;
  void *ws = nullptr;  // split-K workspace, grown on demand
  size_t ws_bytes = 0;
  int ovr_cfg[2] = {-1, -1};  // tuning override per op (0 sgemm, 1 conv); -1 = table/heuristic
  uint32_t ovr_splits[2] = {0, 0};
  int ovr_red[2] = {0, 0};
  int ovr_wt[2] = {-1, -1};  // output store policy override (-1 = the table's / heuristic's)
  std::vector<hipGraphExec_t> graphs;  // captured launch sequences
  void *stamps = nullptr;              // device timestamp slots (bh_stamp)
  hipEvent_t t_start = nullptr;        // bh_time_next_call: events for the next call's
  hipEvent_t t_stop = nullptr;         //   first / last kernel dispatch
  double stamp_hz = 100e6;
  void *cnt = nullptr;  // split-K arrival tickets
  uint64_t cnt_n = 0;
  void *wpack = nullptr;  // k-major filter bank for the ring conv kernels, grown on demand
  size_t wpack_bytes = 0;
  // outgrown workspaces still referenced by captured graphs: freed with the last graph (or the context)
  // (a graph replays the pointers it was captured with)
  std::vector<void *> retired;
};

namespace bh {

int fail(int code, const std::string &msg);  // records thread-local message, returns code
int ok();                                    // clears nothing, returns BH_OK

// Kernel launch checks (hipGetLastError after each launch).
int check_launch(const char *what);

// Launch on the context's stream; when bh_time_next_call armed an event pair, the
// first dispatch of the call records the start event and the last one the stop
// event on the kernel's own dispatch (hipExtLaunchKernel).
int launch(bh_ctx *ctx, const void *kernel, dim3 grid, dim3 block, void **args, bool first, bool last,
           const char *what, uint32_t shmem = 0);

// Magic-number unsigned division for 0 <= n < 2^31, 1 <= d < 2^31:
// q = (umulhi(n, m) + n) >> s.
struct fastdiv {
  uint32_t d, m, s;
};
inline fastdiv make_fastdiv(uint32_t d) {
  fastdiv f{d, 0, 0};
  uint32_t s = 0;
  while ((1ull << s) < d) ++s;
  f.s = s;
  f.m = (uint32_t)(((1ull << 32) * ((1ull << s) - d)) / d + 1);
  return f;
}

}  // namespace bh

#define BH_HIP(x)                                                                      \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) return bh::fail(BH_ERR, std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)

#define BH_CHECK_CTX(c) \
  do { if (!(c)) return bh::fail(BH_ERR, "null bh_ctx"); } while (0)

namespace bh {
// Every C-ABI entry that allocates, creates events or launches runs with the context's
// device current (several contexts / host threads may drive several GPUs), restoring the
// caller's device on return.
struct device_scope {
  int prev = -1;
  explicit device_scope(const bh_ctx *c) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != c->device) (void)hipSetDevice(c->device);
  }
  ~device_scope() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};
// A hot-path call consumes the event pair bh_time_next_call armed, whether it launched or
// failed first: a pair left armed by a rejected call must not attach to an unrelated later
// launch.
struct call_scope : device_scope {
  bh_ctx *c;
  explicit call_scope(bh_ctx *ctx) : device_scope(ctx), c(ctx) {}
  ~call_scope() {
    c->t_start = nullptr;
    c->t_stop = nullptr;
  }
};
// Grow a per-context device buffer to at least `want` bytes (+25 % headroom). Refuses to
// allocate while the context's stream is capturing (a capture records no allocation: run the
// op once eagerly first). The outgrown buffer is kept until the context is destroyed when a
// captured graph may still reference it, freed otherwise.
int grow_buffer(bh_ctx *ctx, void *&buf, size_t &have, size_t want, bool zero, const char *what);
}  // namespace bh

#define BH_ENTER(c)  \
  BH_CHECK_CTX(c);   \
  bh::device_scope bh_dev_scope_(c)
#define BH_ENTER_CALL(c) \
  BH_CHECK_CTX(c);       \
  bh::call_scope bh_call_scope_(c)

// ---- internal entry points implemented in the kernel sources ----
namespace bh {
int launch_gen_data(bh_ctx *ctx, int kind, float *dst, const uint32_t dims[4], uint32_t mode, float vi);
int launch_sgemm(bh_ctx *ctx, const float *a, const float *b, float *c, uint32_t M, uint32_t N, uint32_t K);
int tune_set_wt(bh_ctx *ctx, int op, int wt);
int launch_conv(bh_ctx *ctx, const float *in, const float *filts, const float *packed, const float *biases,
                float *out, uint32_t B, uint32_t IC, uint32_t H, uint32_t W, uint32_t OC, uint32_t KY,
                uint32_t KX, uint32_t sy, uint32_t sx, uint32_t py, uint32_t px, int relu, uint32_t out_ctot = 0,
                const float *res = nullptr, bool no_dc = false, bool repacked = false,
                uint32_t pk_banks = 0xffffffffu);
// packs (bhk::launch_pack_banks): the k-major bank + the Winograd banks of `banks` (BH_BANK_*)
size_t conv_filts_packed_floats(uint32_t OC, uint32_t IC, uint32_t KY, uint32_t KX, uint32_t banks);
int launch_conv_filts_pack(bh_ctx *ctx, const float *filts, float *packed, uint32_t OC, uint32_t IC, uint32_t KY,
                           uint32_t KX, uint32_t banks);
// the Winograd bank (BH_BANK_*, 0: none) the shape's route on ctx reads
uint32_t conv_route_banks(bh_ctx *ctx, const uint32_t *d);
uint32_t pool_out_sz(uint32_t in, uint32_t k, uint32_t s, uint32_t p);
int launch_pool(bh_ctx *ctx, const float *in, float *out, float *out_in_yx, uint32_t B, uint32_t C, uint32_t H,
                uint32_t W, uint32_t KY, uint32_t KX, uint32_t sy, uint32_t sx, uint32_t py, uint32_t px, int avg);
int launch_lrn(bh_ctx *ctx, const float *in, float *out, float *out_scale_base, uint32_t B, uint32_t C, uint32_t H,
               uint32_t W, uint32_t local_size, float alpha, float beta, float k);
int launch_relu(bh_ctx *ctx, float *x, uint64_t n);
int launch_dropout(bh_ctx *ctx, float *x, uint64_t n, float ratio, uint32_t seed);
int launch_softmax(bh_ctx *ctx, const float *in, float *prob, uint32_t B, uint32_t C, uint32_t H, uint32_t W);
int launch_chan_copy(bh_ctx *ctx, const float *in, float *out, uint32_t B, uint32_t HW, uint32_t in_c, uint32_t ic0,
                     uint32_t out_c, uint32_t oc0, uint32_t nc);
int launch_chan_affine(bh_ctx *ctx, const float *in, float *out, const float *scale, const float *shift, uint32_t B,
                       uint32_t C, uint32_t HW, int relu);
int launch_eltwise(bh_ctx *ctx, const float *a, const float *b, float *out, uint64_t n, int op, int relu);
std::string sgemm_variant(uint32_t M, uint32_t N, uint32_t K);
std::string conv_variant(const uint32_t *d);
std::string sgemm_variant_ctx(bh_ctx *ctx, uint32_t M, uint32_t N, uint32_t K);  // with ctx's overrides
std::string conv_variant_ctx(bh_ctx *ctx, const uint32_t *d);
int tune_set(bh_ctx *ctx, int op, int cfg, int splits);
int tune_cfg_name(int op, int cfg, std::string &out);
void jit_release_all(bh_ctx *c);
}  // namespace bh
