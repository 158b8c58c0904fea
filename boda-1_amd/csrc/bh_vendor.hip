// bh_vendor.hip -- same-node comparator: the vendor libraries' SGEMM (rocBLAS) and convolution
// forward (MIOpen) on the op shapes the hand-written kernels run, for a per-op yardstick beside
// them. This is the role of the reference's culibs-wrap (cublas_sgemm / cudnn_conv intercepts,
// src/culibs-wrap.cc:94-242) as cnn_op_info's use_culibs comparator uses it
// (src/cnn-prof.cc:40,90-91). Context only: nothing in the product path (libboda_hip.so) calls
// it, and it is a library of its own (libboda_hip_vendor.so) so the product does not link
// rocBLAS/MIOpen.
//
// Timing convention: the same amortized one as bench.py's per-op graph time -- `reps` calls
// issued back to back on the context's stream, HIP events around the whole run, ms per call.
// The conv is MIOpen's Find choice (miopenFindConvolutionForwardAlgorithm, cached per shape)
// followed by MIOpen's own bias add (miopenOpTensor) and ReLU (miopenActivationForward), i.e.
// the work bh_conv2d_fwd_nchw does in one kernel; the conv-only time is reported beside it.
#include <hip/hip_runtime.h>
#include <miopen/miopen.h>
#include <rocblas/rocblas.h>

#include <cstdint>
#include <cstdio>
#include <map>
#include <string>
#include <tuple>
#include <vector>

#include "boda_hip_vendor.h"

namespace {

thread_local std::string g_err;

int fail(std::string const &m) {
  g_err = m;
  return BHV_ERR;
}

#define V_HIP(x)                                                                          \
  do {                                                                                    \
    hipError_t e_ = (x);                                                                  \
    if (e_ != hipSuccess) return fail(std::string(#x) + ": " + hipGetErrorString(e_));   \
  } while (0)
#define V_RB(x)                                                                           \
  do {                                                                                    \
    rocblas_status s_ = (x);                                                              \
    if (s_ != rocblas_status_success)                                                     \
      return fail(std::string(#x) + ": " + rocblas_status_to_string(s_));                 \
  } while (0)
#define V_MI(x)                                                                           \
  do {                                                                                    \
    miopenStatus_t s_ = (x);                                                              \
    if (s_ != miopenStatusSuccess) return fail(std::string(#x) + ": " + miopenGetErrorString(s_)); \
  } while (0)

struct conv_plan_t {
  miopenTensorDescriptor_t x = nullptr, w = nullptr, y = nullptr, b = nullptr;
  miopenConvolutionDescriptor_t conv = nullptr;
  miopenConvFwdAlgorithm_t algo = miopenConvolutionFwdAlgoGEMM;
  size_t ws = 0;
  float find_ms = 0.f;
};

using conv_key_t = std::tuple<uint32_t, uint32_t, uint32_t, uint32_t, uint32_t, uint32_t, uint32_t, uint32_t,
                              uint32_t, uint32_t, uint32_t>;

__global__ void fill_kernel(float *p, size_t n, uint32_t seed) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 15;
    h *= 2246822519u;
    h ^= h >> 13;
    p[i] = (float)(h & 0xffff) * (1.0f / 65536.0f) - 0.5f;  // [-0.5, 0.5)
  }
}

const char *algo_name(miopenConvFwdAlgorithm_t a) {
  switch (a) {
    case miopenConvolutionFwdAlgoGEMM: return "gemm";
    case miopenConvolutionFwdAlgoDirect: return "direct";
    case miopenConvolutionFwdAlgoFFT: return "fft";
    case miopenConvolutionFwdAlgoWinograd: return "winograd";
    case miopenConvolutionFwdAlgoImplicitGEMM: return "implicit_gemm";
  }
  return "?";
}

}  // namespace

struct bhv_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  rocblas_handle rb = nullptr;
  miopenHandle_t mi = nullptr;
  miopenActivationDescriptor_t relu = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  std::map<conv_key_t, conv_plan_t> plans;
  void *ws = nullptr;  // MIOpen workspace (grown, never shrunk)
  size_t ws_bytes = 0;
  float *scratch[4] = {nullptr, nullptr, nullptr, nullptr};  // timing operands (grown)
  size_t scratch_n[4] = {0, 0, 0, 0};
};

namespace {

struct dev_scope {
  int prev = -1;
  explicit dev_scope(bhv_ctx *c) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (c) (void)hipSetDevice(c->device);
  }
  ~dev_scope() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

int grow(bhv_ctx *c, int i, size_t n, uint32_t seed) {
  if (c->scratch_n[i] >= n) return BHV_OK;
  V_HIP(hipStreamSynchronize(c->stream));
  if (c->scratch[i]) V_HIP(hipFree(c->scratch[i]));
  c->scratch[i] = nullptr;
  c->scratch_n[i] = 0;
  V_HIP(hipMalloc(&c->scratch[i], n * sizeof(float)));
  c->scratch_n[i] = n;
  fill_kernel<<<1024, 256, 0, c->stream>>>(c->scratch[i], n, seed);
  V_HIP(hipGetLastError());
  return BHV_OK;
}

int ensure_ws(bhv_ctx *c, size_t bytes) {
  if (c->ws_bytes >= bytes) return BHV_OK;
  V_HIP(hipStreamSynchronize(c->stream));
  if (c->ws) V_HIP(hipFree(c->ws));
  c->ws = nullptr;
  c->ws_bytes = 0;
  V_HIP(hipMalloc(&c->ws, bytes));
  c->ws_bytes = bytes;
  return BHV_OK;
}

int sgemm(bhv_ctx *c, const float *a, const float *b, float *cc, uint32_t M, uint32_t N, uint32_t K) {
  // c (M x N, row-major) = a^T b with a K x M, b K x N row-major: in rocBLAS's column-major view
  // c^T (N x M, ld N) = b' (N x K, ld N) * (a' (M x K, ld M))^T
  const float one = 1.f, zero = 0.f;
  V_RB(rocblas_sgemm(c->rb, rocblas_operation_none, rocblas_operation_transpose, (rocblas_int)N, (rocblas_int)M,
                     (rocblas_int)K, &one, b, (rocblas_int)N, a, (rocblas_int)M, &zero, cc, (rocblas_int)N));
  return BHV_OK;
}

// the MIOpen descriptors and Find choice for one conv shape (Find runs once per shape, on the
// caller's buffers, as the API requires)
int plan_of(bhv_ctx *c, conv_key_t const &k, const float *in, const float *filts, float *out, conv_plan_t **pp) {
  auto it = c->plans.find(k);
  if (it != c->plans.end()) {
    *pp = &it->second;
    return BHV_OK;
  }
  uint32_t B, IC, H, W, OC, KY, KX, sy, sx, py, px;
  std::tie(B, IC, H, W, OC, KY, KX, sy, sx, py, px) = k;
  conv_plan_t p;
  V_MI(miopenCreateTensorDescriptor(&p.x));
  V_MI(miopenCreateTensorDescriptor(&p.w));
  V_MI(miopenCreateTensorDescriptor(&p.y));
  V_MI(miopenCreateTensorDescriptor(&p.b));
  V_MI(miopenCreateConvolutionDescriptor(&p.conv));
  V_MI(miopenSet4dTensorDescriptor(p.x, miopenFloat, (int)B, (int)IC, (int)H, (int)W));
  V_MI(miopenSet4dTensorDescriptor(p.w, miopenFloat, (int)OC, (int)IC, (int)KY, (int)KX));
  V_MI(miopenInitConvolutionDescriptor(p.conv, miopenConvolution, (int)py, (int)px, (int)sy, (int)sx, 1, 1));
  int n, ch, h, w;
  V_MI(miopenGetConvolutionForwardOutputDim(p.conv, p.x, p.w, &n, &ch, &h, &w));
  V_MI(miopenSet4dTensorDescriptor(p.y, miopenFloat, n, ch, h, w));
  V_MI(miopenSet4dTensorDescriptor(p.b, miopenFloat, 1, (int)OC, 1, 1));
  size_t ws = 0;
  V_MI(miopenConvolutionForwardGetWorkSpaceSize(c->mi, p.w, p.x, p.conv, p.y, &ws));
  if (ensure_ws(c, ws ? ws : 4) != BHV_OK) return BHV_ERR;
  miopenConvAlgoPerf_t perf[8];
  int got = 0;
  hipEvent_t a, e;
  V_HIP(hipEventCreate(&a));
  V_HIP(hipEventCreate(&e));
  V_HIP(hipEventRecord(a, c->stream));
  V_MI(miopenFindConvolutionForwardAlgorithm(c->mi, p.x, in, p.w, filts, p.conv, p.y, out, 8, &got, perf, c->ws,
                                             c->ws_bytes, false));
  V_HIP(hipEventRecord(e, c->stream));
  V_HIP(hipEventSynchronize(e));
  V_HIP(hipEventElapsedTime(&p.find_ms, a, e));
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(e);
  if (got < 1) return fail("MIOpen Find returned no forward algorithm");
  p.algo = perf[0].fwd_algo;
  p.ws = perf[0].memory;
  if (ensure_ws(c, p.ws ? p.ws : 4) != BHV_OK) return BHV_ERR;
  *pp = &(c->plans[k] = p);
  return BHV_OK;
}

int conv(bhv_ctx *c, conv_plan_t *p, const float *in, const float *filts, const float *biases, float *out,
         int relu) {
  const float one = 1.f, zero = 0.f;
  V_MI(miopenConvolutionForward(c->mi, &one, p->x, in, p->w, filts, p->conv, p->algo, &zero, p->y, out, c->ws,
                                p->ws));
  if (biases)
    V_MI(miopenOpTensor(c->mi, miopenTensorOpAdd, &one, p->y, out, &one, p->b, biases, &zero, p->y, out));
  if (relu) V_MI(miopenActivationForward(c->mi, c->relu, &one, p->y, out, &zero, p->y, out));
  return BHV_OK;
}

}  // namespace

extern "C" {

const char *bhv_last_error(void) { return g_err.c_str(); }

int bhv_init(int device, bhv_ctx **out) {
  if (!out) return fail("null ctx out-pointer");
  *out = nullptr;
  int n = 0;
  V_HIP(hipGetDeviceCount(&n));
  if (device < 0 || device >= n) return fail("no such device");
  auto *c = new bhv_ctx;
  c->device = device;
  dev_scope ds(c);
  int rc = BHV_OK;
  auto chk = [&](bool ok, const char *what) {
    if (!ok && rc == BHV_OK) rc = fail(what);
  };
  chk(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) == hipSuccess, "hipStreamCreate failed");
  chk(rc || rocblas_create_handle(&c->rb) == rocblas_status_success, "rocblas_create_handle failed");
  chk(rc || rocblas_set_stream(c->rb, c->stream) == rocblas_status_success, "rocblas_set_stream failed");
  chk(rc || miopenCreateWithStream(&c->mi, c->stream) == miopenStatusSuccess, "miopenCreateWithStream failed");
  chk(rc || miopenCreateActivationDescriptor(&c->relu) == miopenStatusSuccess, "miopenCreateActivationDescriptor");
  chk(rc || miopenSetActivationDescriptor(c->relu, miopenActivationRELU, 0., 0., 1.) == miopenStatusSuccess,
      "miopenSetActivationDescriptor failed");
  chk(rc || hipEventCreate(&c->e0) == hipSuccess, "hipEventCreate failed");
  chk(rc || hipEventCreate(&c->e1) == hipSuccess, "hipEventCreate failed");
  if (rc != BHV_OK) {
    std::string m = g_err;
    bhv_destroy(c);
    g_err = m;
    return rc;
  }
  *out = c;
  return BHV_OK;
}

int bhv_destroy(bhv_ctx *c) {
  if (!c) return BHV_OK;
  dev_scope ds(c);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  for (auto &kv : c->plans) {
    conv_plan_t &p = kv.second;
    (void)miopenDestroyTensorDescriptor(p.x);
    (void)miopenDestroyTensorDescriptor(p.w);
    (void)miopenDestroyTensorDescriptor(p.y);
    (void)miopenDestroyTensorDescriptor(p.b);
    (void)miopenDestroyConvolutionDescriptor(p.conv);
  }
  for (int i = 0; i < 4; ++i)
    if (c->scratch[i]) (void)hipFree(c->scratch[i]);
  if (c->ws) (void)hipFree(c->ws);
  if (c->relu) (void)miopenDestroyActivationDescriptor(c->relu);
  if (c->mi) (void)miopenDestroy(c->mi);
  if (c->rb) (void)rocblas_destroy_handle(c->rb);
  if (c->e0) (void)hipEventDestroy(c->e0);
  if (c->e1) (void)hipEventDestroy(c->e1);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
  return BHV_OK;
}

int bhv_sync(bhv_ctx *c) {
  if (!c) return fail("null ctx");
  dev_scope ds(c);
  V_HIP(hipStreamSynchronize(c->stream));
  return BHV_OK;
}

int bhv_sgemm_kmajor(bhv_ctx *c, const float *a, const float *b, float *cc, uint32_t M, uint32_t N, uint32_t K) {
  if (!c || !a || !b || !cc) return fail("null argument");
  if (!M || !N || !K || M > 0x7fffffffu || N > 0x7fffffffu || K > 0x7fffffffu) return fail("bad sgemm dims");
  dev_scope ds(c);
  return sgemm(c, a, b, cc, M, N, K);
}

int bhv_conv2d_fwd_nchw(bhv_ctx *c, const float *in, const float *filts, const float *biases, float *out, uint32_t B,
                        uint32_t IC, uint32_t H, uint32_t W, uint32_t OC, uint32_t KY, uint32_t KX, uint32_t sy,
                        uint32_t sx, uint32_t py, uint32_t px, int relu) {
  if (!c || !in || !filts || !out) return fail("null argument");
  if (!B || !IC || !H || !W || !OC || !KY || !KX || !sy || !sx) return fail("bad conv dims");
  dev_scope ds(c);
  conv_plan_t *p = nullptr;
  if (plan_of(c, conv_key_t(B, IC, H, W, OC, KY, KX, sy, sx, py, px), in, filts, out, &p) != BHV_OK) return BHV_ERR;
  return conv(c, p, in, filts, biases, out, relu);
}

int bhv_time_sgemm(bhv_ctx *c, uint32_t M, uint32_t N, uint32_t K, int reps, float *ms) {
  if (!c || !ms || reps < 1) return fail("bad argument");
  if (!M || !N || !K) return fail("bad sgemm dims");
  dev_scope ds(c);
  if (grow(c, 0, (size_t)K * M, 1) || grow(c, 1, (size_t)K * N, 2) || grow(c, 2, (size_t)M * N, 3)) return BHV_ERR;
  if (sgemm(c, c->scratch[0], c->scratch[1], c->scratch[2], M, N, K)) return BHV_ERR;  // warm
  V_HIP(hipEventRecord(c->e0, c->stream));
  for (int r = 0; r < reps; ++r)
    if (sgemm(c, c->scratch[0], c->scratch[1], c->scratch[2], M, N, K)) return BHV_ERR;
  V_HIP(hipEventRecord(c->e1, c->stream));
  V_HIP(hipEventSynchronize(c->e1));
  V_HIP(hipEventElapsedTime(ms, c->e0, c->e1));
  *ms /= reps;
  return BHV_OK;
}

int bhv_time_conv(bhv_ctx *c, uint32_t B, uint32_t IC, uint32_t H, uint32_t W, uint32_t OC, uint32_t KY,
                  uint32_t KX, uint32_t sy, uint32_t sx, uint32_t py, uint32_t px, int relu, int reps, float *ms,
                  float *conv_only_ms, float *find_ms, char *algo, size_t algolen) {
  if (!c || !ms || reps < 1) return fail("bad argument");
  if (!B || !IC || !H || !W || !OC || !KY || !KX || !sy || !sx) return fail("bad conv dims");
  if (H + 2 * py < KY || W + 2 * px < KX) return fail("kernel larger than padded input");
  dev_scope ds(c);
  const size_t OH = (H + 2 * py - KY) / sy + 1, OW = (W + 2 * px - KX) / sx + 1;
  if (grow(c, 0, (size_t)B * IC * H * W, 1) || grow(c, 1, (size_t)OC * IC * KY * KX, 2) ||
      grow(c, 2, (size_t)B * OC * OH * OW, 3) || grow(c, 3, OC, 4))
    return BHV_ERR;
  const float *in = c->scratch[0], *f = c->scratch[1], *b = c->scratch[3];
  float *out = c->scratch[2];
  conv_plan_t *p = nullptr;
  if (plan_of(c, conv_key_t(B, IC, H, W, OC, KY, KX, sy, sx, py, px), in, f, out, &p) != BHV_OK) return BHV_ERR;
  if (conv(c, p, in, f, b, out, relu)) return BHV_ERR;  // warm
  for (int pass = 0; pass < 2; ++pass) {
    if (pass == 1 && !conv_only_ms) break;
    V_HIP(hipEventRecord(c->e0, c->stream));
    for (int r = 0; r < reps; ++r)
      if (pass == 0 ? conv(c, p, in, f, b, out, relu) : conv(c, p, in, f, nullptr, out, 0)) return BHV_ERR;
    V_HIP(hipEventRecord(c->e1, c->stream));
    V_HIP(hipEventSynchronize(c->e1));
    float t = 0.f;
    V_HIP(hipEventElapsedTime(&t, c->e0, c->e1));
    *(pass == 0 ? ms : conv_only_ms) = t / reps;
  }
  if (find_ms) *find_ms = p->find_ms;
  if (algo && algolen) std::snprintf(algo, algolen, "%s", algo_name(p->algo));
  return BHV_OK;
}

}  // extern "C"
