// bh_runtime.hip -- device context, vars, copies, events and the extern "C"
// surface of libboda_hip.so (declared in include/boda_hip.h).
//
// Mirrors the contract of Boda's nvrtc_compute_t (src/nvrtc_util.cc:174-395):
// one device per context, zero-filled var allocation (:80-84), an event pair
// around every timed call (:289-298, :367-381), durations in milliseconds
// (src/rtc_compute.H:66-71). Unlike the reference (default stream 0), each
// context owns a non-blocking stream so several contexts / host threads can
// drive several GPUs of one node independently.
#include "bh_common.h"
#include <cstdio>
#include <cstring>

namespace {
thread_local std::string g_last_error;

// Device timestamp: one lane writes the constant-rate wall clock (s_memrealtime).
// Usable inside captured graphs, where HIP event timing is not available.
__global__ void stamp_kernel(unsigned long long *t, int slot) {
  if (threadIdx.x == 0) t[slot] = wall_clock64();
}
// bounded busy-wait on the 100 MHz constant clock (every wave exits after us µs)
__global__ void spin_kernel(unsigned long long ticks) {
  const unsigned long long t0 = wall_clock64();
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
}
constexpr int STAMP_SLOTS = 1 << 18;
}

namespace bh {
int fail(int code, const std::string &msg) {
  g_last_error = msg;
  return code;
}
int ok() { return BH_OK; }
int check_launch(const char *what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(BH_ERR, std::string("launch of ") + what + " failed: " + hipGetErrorString(e));
  return BH_OK;
}

int grow_buffer(bh_ctx *ctx, void *&buf, size_t &have, size_t want, bool zero, const char *what) {
  if (have >= want) return BH_OK;
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  BH_HIP(hipStreamIsCapturing(ctx->stream, &st));
  if (st != hipStreamCaptureStatusNone)
    return fail(BH_ERR, std::string(what) + ": the per-context workspace must grow (" + std::to_string(want) +
                            " bytes) while the stream is being captured; run this op once eagerly before capturing");
  if (buf) {
    bool live_graph = false;
    for (hipGraphExec_t g : ctx->graphs) live_graph |= g != nullptr;
    if (live_graph) {
      ctx->retired.push_back(buf);  // a captured graph may still replay this pointer
    } else {
      BH_HIP(hipStreamSynchronize(ctx->stream));
      BH_HIP(hipFree(buf));
    }
    buf = nullptr;
    have = 0;
  }
  const size_t sz = want + (want >> 2);
  BH_HIP(hipMalloc(&buf, sz));
  if (zero) BH_HIP(hipMemsetAsync(buf, 0, sz, ctx->stream));
  have = sz;
  return BH_OK;
}

int launch(bh_ctx *ctx, const void *kernel, dim3 grid, dim3 block, void **args, bool first, bool last,
           const char *what, uint32_t shmem) {
  hipEvent_t b = first ? ctx->t_start : nullptr, e = last ? ctx->t_stop : nullptr;
  hipError_t r = (b || e) ? hipExtLaunchKernel(kernel, grid, block, args, shmem, ctx->stream, b, e, 0)
                          : hipLaunchKernel(kernel, grid, block, args, shmem, ctx->stream);
  if (first) ctx->t_start = nullptr;
  if (last) ctx->t_stop = nullptr;
  if (r != hipSuccess) return fail(BH_ERR, std::string("launch of ") + what + " failed: " + hipGetErrorString(r));
  return check_launch(what);
}
}  // namespace bh

extern "C" {

int bh_abi_version(void) { return BH_ABI_VERSION; }

const char *bh_last_error(void) { return g_last_error.c_str(); }

int bh_device_count(int *count) {
  if (!count) return bh::fail(BH_ERR, "null count");
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess) n = 0;
  *count = n;
  return BH_OK;
}

int bh_init(int device, bh_ctx **out) {
  if (!out) return bh::fail(BH_ERR, "null ctx out-pointer");
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0)
    return bh::fail(BH_ERR, "no HIP device available (libboda_hip has no CPU fallback)");
  if (device < 0 || device >= n) return bh::fail(BH_ERR, "device index out of range");
  bh_ctx *c = new bh_ctx();
  c->device = device;
  hipError_t e = hipSetDevice(device);
  if (e == hipSuccess) e = hipGetDeviceProperties(&c->prop, device);
  if (e == hipSuccess && std::strncmp(c->prop.gcnArchName, "gfx950", 6) != 0) {
    std::string arch = c->prop.gcnArchName;
    delete c;
    return bh::fail(BH_ERR, "device is " + arch + "; libboda_hip is built for gfx950 (MI355X) only");
  }
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipMalloc(&c->stamps, STAMP_SLOTS * sizeof(unsigned long long));
  if (e == hipSuccess) {
    int khz = 0;
    e = hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device);
    c->stamp_hz = khz > 0 ? khz * 1000.0 : 100e6;
  }
  if (e != hipSuccess) {
    delete c;
    return bh::fail(BH_ERR, std::string("bh_init: ") + hipGetErrorString(e));
  }
  *out = c;
  return BH_OK;
}

int bh_destroy(bh_ctx *c) {
  BH_ENTER(c);
  (void)hipSetDevice(c->device);
  (void)hipStreamSynchronize(c->stream);
  for (hipEvent_t ev : c->events) (void)hipEventDestroy(ev);
  for (hipGraphExec_t g : c->graphs)
    if (g) (void)hipGraphExecDestroy(g);
  bh::jit_release_all(c);
  for (void *r : c->retired) (void)hipFree(r);
  if (c->ws) (void)hipFree(c->ws);
  if (c->wpack) (void)hipFree(c->wpack);
  if (c->stamps) (void)hipFree(c->stamps);
  if (c->cnt) (void)hipFree(c->cnt);
  (void)hipStreamDestroy(c->stream);
  delete c;
  return BH_OK;
}

int bh_plat_tag(bh_ctx *c, char *buf, size_t n) {
  BH_ENTER(c);
  if (!buf || !n) return bh::fail(BH_ERR, "null buffer");
  // the marketing name comes from libdrm's amdgpu.ids; where that table is missing (some
  // launch environments) HIP reports a generic "AMD Radeon Graphics": gfx950 is MI355X
  const bool named = std::strstr(c->prop.name, "MI3") != nullptr;
  std::snprintf(buf, n, "hip:%s:%s", named ? c->prop.name : "MI355X", c->prop.gcnArchName);
  return BH_OK;
}

int bh_get_stream(bh_ctx *c, void **s) {
  BH_ENTER(c);
  if (!s) return bh::fail(BH_ERR, "null out");
  *s = (void *)c->stream;
  return BH_OK;
}

int bh_alloc(bh_ctx *c, size_t bytes, void **p) {
  BH_ENTER(c);
  if (!p) return bh::fail(BH_ERR, "null out");
  *p = nullptr;
  void *d = nullptr;
  BH_HIP(hipMalloc(&d, bytes ? bytes : 16));
  hipError_t e = hipMemsetAsync(d, 0, bytes ? bytes : 16, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  if (e != hipSuccess) {
    (void)hipFree(d);
    return bh::fail(BH_ERR, std::string("bh_alloc zero-fill: ") + hipGetErrorString(e));
  }
  *p = d;
  return BH_OK;
}

int bh_free(bh_ctx *c, void *p) {
  BH_ENTER(c);
  BH_HIP(hipStreamSynchronize(c->stream));
  BH_HIP(hipFree(p));
  return BH_OK;
}

int bh_memset0(bh_ctx *c, void *p, size_t bytes) {
  BH_ENTER(c);
  BH_HIP(hipMemsetAsync(p, 0, bytes, c->stream));
  return BH_OK;
}

int bh_h2d(bh_ctx *c, void *d, const void *h, size_t bytes) {
  BH_ENTER(c);
  // synchronous w.r.t. the host buffer (caller may free it on return)
  BH_HIP(hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, c->stream));
  BH_HIP(hipStreamSynchronize(c->stream));
  return BH_OK;
}

int bh_d2h(bh_ctx *c, void *h, const void *d, size_t bytes) {
  BH_ENTER(c);
  BH_HIP(hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, c->stream));
  BH_HIP(hipStreamSynchronize(c->stream));
  return BH_OK;
}

int bh_sync(bh_ctx *c) {
  BH_ENTER(c);
  BH_HIP(hipStreamSynchronize(c->stream));
  return BH_OK;
}

int bh_event_record(bh_ctx *c, int *id) {
  BH_ENTER(c);
  if (!id) return bh::fail(BH_ERR, "null out");
  if (c->events_used == (int)c->events.size()) {
    hipEvent_t ev;
    BH_HIP(hipEventCreate(&ev));
    c->events.push_back(ev);
  }
  BH_HIP(hipEventRecord(c->events[c->events_used], c->stream));
  *id = c->events_used++;
  return BH_OK;
}

int bh_time_next_call(bh_ctx *c, int *begin_id, int *end_id) {
  BH_ENTER(c);
  if (!begin_id || !end_id) return bh::fail(BH_ERR, "null out");
  for (int k = 0; k < 2; ++k)
    if (c->events_used + k >= (int)c->events.size()) {
      hipEvent_t ev;
      BH_HIP(hipEventCreate(&ev));
      c->events.push_back(ev);
    }
  *begin_id = c->events_used++;
  *end_id = c->events_used++;
  c->t_start = c->events[*begin_id];
  c->t_stop = c->events[*end_id];
  return BH_OK;
}

int bh_elapsed_ms(bh_ctx *c, int b, int e, float *ms) {
  BH_ENTER(c);
  if (!ms) return bh::fail(BH_ERR, "null out");
  if (b < 0 || e < 0 || b >= c->events_used || e >= c->events_used) return bh::fail(BH_ERR, "bad event id");
  BH_HIP(hipEventSynchronize(c->events[e]));
  BH_HIP(hipEventElapsedTime(ms, c->events[b], c->events[e]));
  return BH_OK;
}

int bh_events_reset(bh_ctx *c) {
  BH_ENTER(c);
  c->events_used = 0;
  return BH_OK;
}

int bh_gen_data(bh_ctx *c, int kind, float *dst, const uint32_t dims[4], uint32_t mode, float vi) {
  BH_ENTER_CALL(c);
  if (!dst || !dims) return bh::fail(BH_ERR, "null argument");
  return bh::launch_gen_data(c, kind, dst, dims, mode, vi);
}

int bh_sgemm_kmajor(bh_ctx *c, const float *a, const float *b, float *cc, uint32_t M, uint32_t N, uint32_t K) {
  BH_ENTER_CALL(c);
  if (!a || !b || !cc) return bh::fail(BH_ERR, "null tensor");
  if (!M || !N || !K) return bh::fail(BH_UNSUP, "sgemm: zero-sized dimension");
  return bh::launch_sgemm(c, a, b, cc, M, N, K);
}

int bh_conv2d_fwd_nchw_pk(bh_ctx *c, const float *in, const float *filts, const float *packed, const float *biases,
                          float *out, uint32_t B, uint32_t IC, uint32_t H, uint32_t W, uint32_t OC, uint32_t KY,
                          uint32_t KX, uint32_t sy, uint32_t sx, uint32_t py, uint32_t px, int relu) {
  BH_ENTER_CALL(c);
  if (!in || !filts || !out) return bh::fail(BH_ERR, "null tensor");
  if (!B || !IC || !H || !W || !OC || !KY || !KX || !sy || !sx)
    return bh::fail(BH_UNSUP, "conv: zero-sized dimension or stride");
  if (H + 2 * py < KY || W + 2 * px < KX) return bh::fail(BH_UNSUP, "conv: padded input smaller than kernel");
  return bh::launch_conv(c, in, filts, packed, biases, out, B, IC, H, W, OC, KY, KX, sy, sx, py, px, relu);
}

int bh_conv2d_fwd_nchw_res(bh_ctx *c, const float *in, const float *filts, const float *packed, const float *biases,
                           const float *res, float *out, uint32_t B, uint32_t IC, uint32_t H, uint32_t W, uint32_t OC,
                           uint32_t KY, uint32_t KX, uint32_t sy, uint32_t sx, uint32_t py, uint32_t px, int relu) {
  BH_ENTER_CALL(c);
  if (!in || !filts || !out) return bh::fail(BH_ERR, "null tensor");
  if (!B || !IC || !H || !W || !OC || !KY || !KX || !sy || !sx)
    return bh::fail(BH_UNSUP, "conv: zero-sized dimension or stride");
  if (H + 2 * py < KY || W + 2 * px < KX) return bh::fail(BH_UNSUP, "conv: padded input smaller than kernel");
  return bh::launch_conv(c, in, filts, packed, biases, out, B, IC, H, W, OC, KY, KX, sy, sx, py, px, relu, 0, res);
}

int bh_conv2d_fwd_nchw_slab(bh_ctx *c, const float *in, const float *filts, const float *packed,
                            const float *biases, float *out, uint32_t out_chans_total, uint32_t out_chan_ofs,
                            uint32_t B, uint32_t IC, uint32_t H, uint32_t W, uint32_t OC, uint32_t KY, uint32_t KX,
                            uint32_t sy, uint32_t sx, uint32_t py, uint32_t px, int relu) {
  BH_ENTER_CALL(c);
  if (!in || !filts || !out) return bh::fail(BH_ERR, "null tensor");
  if (!B || !IC || !H || !W || !OC || !KY || !KX || !sy || !sx)
    return bh::fail(BH_UNSUP, "conv: zero-sized dimension or stride");
  if (H + 2 * py < KY || W + 2 * px < KX) return bh::fail(BH_UNSUP, "conv: padded input smaller than kernel");
  if ((uint64_t)out_chan_ofs + OC > out_chans_total) return bh::fail(BH_ERR, "conv: output channel slab out of range");
  const uint64_t ohw = (uint64_t)((H + 2 * py - KY) / sy + 1) * ((W + 2 * px - KX) / sx + 1);
  return bh::launch_conv(c, in, filts, packed, biases, out + out_chan_ofs * ohw, B, IC, H, W, OC, KY, KX, sy, sx,
                         py, px, relu, out_chans_total);
}

int bh_conv2d_fwd_nchw_pkb(bh_ctx *c, const float *in, const float *filts, const float *packed, uint32_t banks,
                           const float *biases, const float *res, float *out, uint32_t out_chans_total,
                           uint32_t out_chan_ofs, uint32_t B, uint32_t IC, uint32_t H, uint32_t W, uint32_t OC,
                           uint32_t KY, uint32_t KX, uint32_t sy, uint32_t sx, uint32_t py, uint32_t px, int relu) {
  BH_ENTER_CALL(c);
  if (!in || !filts || !out) return bh::fail(BH_ERR, "null tensor");
  if (!B || !IC || !H || !W || !OC || !KY || !KX || !sy || !sx)
    return bh::fail(BH_UNSUP, "conv: zero-sized dimension or stride");
  if (H + 2 * py < KY || W + 2 * px < KX) return bh::fail(BH_UNSUP, "conv: padded input smaller than kernel");
  if (!out_chans_total) out_chans_total = OC;
  if ((uint64_t)out_chan_ofs + OC > out_chans_total) return bh::fail(BH_ERR, "conv: output channel slab out of range");
  if (res && out_chans_total != OC) return bh::fail(BH_ERR, "conv: residual and channel slab together");
  const uint64_t ohw = (uint64_t)((H + 2 * py - KY) / sy + 1) * ((W + 2 * px - KX) / sx + 1);
  return bh::launch_conv(c, in, filts, packed, biases, out + out_chan_ofs * ohw, B, IC, H, W, OC, KY, KX, sy, sx, py,
                         px, relu, out_chans_total, res, false, false, banks);
}

int bh_conv2d_fwd_nchw(bh_ctx *c, const float *in, const float *filts, const float *biases, float *out,
                       uint32_t B, uint32_t IC, uint32_t H, uint32_t W, uint32_t OC, uint32_t KY, uint32_t KX,
                       uint32_t sy, uint32_t sx, uint32_t py, uint32_t px, int relu) {
  return bh_conv2d_fwd_nchw_pk(c, in, filts, nullptr, biases, out, B, IC, H, W, OC, KY, KX, sy, sx, py, px, relu);
}

int bh_pool_out_size(uint32_t in, uint32_t k, uint32_t stride, uint32_t pad) {
  if (!k || !stride) return 0;
  return (int)bh::pool_out_sz(in, k, stride, pad);
}

int bh_pool_fwd_nchw(bh_ctx *c, const float *in, float *out, float *out_in_yx, uint32_t B, uint32_t C, uint32_t H,
                     uint32_t W, uint32_t KY, uint32_t KX, uint32_t sy, uint32_t sx, uint32_t py, uint32_t px,
                     int avg) {
  BH_ENTER_CALL(c);
  if (!in || !out) return bh::fail(BH_ERR, "null tensor");
  if (!B || !C || !H || !W || !KY || !KX || !sy || !sx) return bh::fail(BH_UNSUP, "pool: zero-sized dimension");
  if (py >= KY || px >= KX) return bh::fail(BH_UNSUP, "pool: padding must be smaller than the window");
  return bh::launch_pool(c, in, out, out_in_yx, B, C, H, W, KY, KX, sy, sx, py, px, avg ? 1 : 0);
}

int bh_lrn_fwd_nchw(bh_ctx *c, const float *in, float *out, float *out_scale_base, uint32_t B, uint32_t C, uint32_t H,
                    uint32_t W, uint32_t local_size, float alpha, float beta, float k) {
  BH_ENTER_CALL(c);
  if (!in || !out) return bh::fail(BH_ERR, "null tensor");
  if (!B || !C || !H || !W) return bh::fail(BH_UNSUP, "lrn: zero-sized dimension");
  return bh::launch_lrn(c, in, out, out_scale_base, B, C, H, W, local_size, alpha, beta, k);
}

int bh_relu_inplace(bh_ctx *c, float *x, uint64_t n) {
  BH_ENTER_CALL(c);
  if (!x) return bh::fail(BH_ERR, "null tensor");
  if (!n) return BH_OK;
  return bh::launch_relu(c, x, n);
}

int bh_dropout_inplace(bh_ctx *c, float *x, uint64_t n, float ratio, uint32_t det_drop_seed) {
  BH_ENTER_CALL(c);
  if (!x) return bh::fail(BH_ERR, "null tensor");
  if (!n) return BH_OK;
  return bh::launch_dropout(c, x, n, ratio, det_drop_seed);
}

int bh_softmax_chans(bh_ctx *c, const float *in, float *prob, uint32_t B, uint32_t C, uint32_t H, uint32_t W) {
  BH_ENTER_CALL(c);
  if (!in || !prob) return bh::fail(BH_ERR, "null tensor");
  if (!B || !C || !H || !W) return bh::fail(BH_UNSUP, "softmax: zero-sized dimension");
  return bh::launch_softmax(c, in, prob, B, C, H, W);
}

int bh_chan_copy(bh_ctx *c, const float *in, float *out, uint32_t B, uint32_t HW, uint32_t in_c, uint32_t ic0,
                 uint32_t out_c, uint32_t oc0, uint32_t nc) {
  BH_ENTER_CALL(c);
  if (!in || !out) return bh::fail(BH_ERR, "null tensor");
  return bh::launch_chan_copy(c, in, out, B, HW, in_c, ic0, out_c, oc0, nc);
}

int bh_chan_affine(bh_ctx *c, const float *in, float *out, const float *scale, const float *shift, uint32_t B,
                   uint32_t C, uint32_t HW, int relu) {
  BH_ENTER_CALL(c);
  if (!in || !out || !scale || !shift) return bh::fail(BH_ERR, "null tensor");
  return bh::launch_chan_affine(c, in, out, scale, shift, B, C, HW, relu ? 1 : 0);
}

int bh_eltwise(bh_ctx *c, const float *a, const float *b, float *out, uint64_t n, int op, int relu) {
  BH_ENTER_CALL(c);
  if (!a || !b || !out) return bh::fail(BH_ERR, "null tensor");
  if (!n) return BH_OK;
  return bh::launch_eltwise(c, a, b, out, n, op, relu ? 1 : 0);
}

size_t bh_conv_filts_packed_floats(uint32_t OC, uint32_t IC, uint32_t KY, uint32_t KX) {
  return bh::conv_filts_packed_floats(OC, IC, KY, KX, BH_BANKS_ALL);
}

int bh_conv_filts_pack(bh_ctx *c, const float *filts, float *packed, uint32_t OC, uint32_t IC, uint32_t KY,
                       uint32_t KX) {
  return bh_conv_filts_pack_banks(c, filts, packed, OC, IC, KY, KX, BH_BANKS_ALL);
}

size_t bh_conv_filts_packed_floats_banks(uint32_t OC, uint32_t IC, uint32_t KY, uint32_t KX, uint32_t banks) {
  return bh::conv_filts_packed_floats(OC, IC, KY, KX, banks);
}

int bh_conv_filts_pack_banks(bh_ctx *c, const float *filts, float *packed, uint32_t OC, uint32_t IC, uint32_t KY,
                             uint32_t KX, uint32_t banks) {
  BH_ENTER_CALL(c);
  if (!filts || !packed) return bh::fail(BH_ERR, "null tensor");
  if (!OC || !IC || !KY || !KX) return bh::fail(BH_UNSUP, "conv_filts_pack: zero-sized dimension");
  return bh::launch_conv_filts_pack(c, filts, packed, OC, IC, KY, KX, banks);
}

int bh_conv_route_banks(bh_ctx *c, const uint32_t *dims, uint32_t *banks) {
  // c may be NULL: the tuning table's / heuristic's route (no device needed)
  if (!dims || !banks) return bh::fail(BH_ERR, "null argument");
  *banks = bh::conv_route_banks(c, dims);
  return BH_OK;
}

int bh_variant_name(int op, const uint32_t *dims, char *buf, size_t n) {
  if (!dims || !buf || !n) return bh::fail(BH_ERR, "null argument");
  std::string s;
  if (op == 0) s = bh::sgemm_variant(dims[0], dims[1], dims[2]);
  else if (op == 1) s = bh::conv_variant(dims);
  else return bh::fail(BH_ERR, "unknown op kind");
  std::snprintf(buf, n, "%s", s.c_str());
  return BH_OK;
}

int bh_variant_name_ctx(bh_ctx *c, int op, const uint32_t *dims, char *buf, size_t n) {
  BH_ENTER(c);
  if (!dims || !buf || !n) return bh::fail(BH_ERR, "null argument");
  std::string s;
  if (op == 0) s = bh::sgemm_variant_ctx(c, dims[0], dims[1], dims[2]);
  else if (op == 1) s = bh::conv_variant_ctx(c, dims);
  else return bh::fail(BH_ERR, "unknown op kind");
  std::snprintf(buf, n, "%s", s.c_str());
  return BH_OK;
}

int bh_stamp(bh_ctx *c, int slot) {
  BH_ENTER(c);
  if (slot < 0 || slot >= STAMP_SLOTS) return bh::fail(BH_ERR, "stamp slot out of range");
  unsigned long long *t = (unsigned long long *)c->stamps;
  void *args[] = {&t, &slot};
  BH_HIP(hipLaunchKernel((const void *)stamp_kernel, dim3(1), dim3(64), args, 0, c->stream));
  return bh::check_launch("stamp");
}

int bh_spin(bh_ctx *c, int us) {
  BH_ENTER(c);
  if (us < 1 || us > 100000) return bh::fail(BH_ERR, "bh_spin: us out of range 1..100000");
  unsigned long long ticks = (unsigned long long)us * (unsigned long long)(c->stamp_hz / 1e6);
  void *args[] = {&ticks};
  BH_HIP(hipLaunchKernel((const void *)spin_kernel, dim3(1), dim3(64), args, 0, c->stream));
  return bh::check_launch("spin");
}

int bh_stamps_read(bh_ctx *c, int first, int n, double *us) {
  BH_ENTER(c);
  if (!us || first < 0 || n < 0 || first + n > STAMP_SLOTS) return bh::fail(BH_ERR, "bad stamp range");
  std::vector<unsigned long long> t(n);
  BH_HIP(hipMemcpyAsync(t.data(), (unsigned long long *)c->stamps + first, n * sizeof(unsigned long long),
                        hipMemcpyDeviceToHost, c->stream));
  BH_HIP(hipStreamSynchronize(c->stream));
  for (int i = 0; i < n; ++i) us[i] = (double)(t[i] - t[0]) * 1e6 / c->stamp_hz;
  return BH_OK;
}

int bh_capture_begin(bh_ctx *c) {
  BH_ENTER(c);
  BH_HIP(hipStreamBeginCapture(c->stream, hipStreamCaptureModeThreadLocal));
  return BH_OK;
}

int bh_capture_end(bh_ctx *c, int *graph_id) {
  BH_ENTER(c);
  if (!graph_id) return bh::fail(BH_ERR, "null out");
  hipGraph_t g = nullptr;
  BH_HIP(hipStreamEndCapture(c->stream, &g));
  hipGraphExec_t ge = nullptr;
  hipError_t e = hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
  (void)hipGraphDestroy(g);
  if (e != hipSuccess) return bh::fail(BH_ERR, std::string("hipGraphInstantiate: ") + hipGetErrorString(e));
  c->graphs.push_back(ge);
  *graph_id = (int)c->graphs.size() - 1;
  return BH_OK;
}

int bh_graph_launch(bh_ctx *c, int graph_id) {
  BH_ENTER(c);
  if (graph_id < 0 || graph_id >= (int)c->graphs.size() || !c->graphs[graph_id]) return bh::fail(BH_ERR, "bad graph id");
  BH_HIP(hipGraphLaunch(c->graphs[graph_id], c->stream));
  return BH_OK;
}

int bh_graph_destroy(bh_ctx *c, int graph_id) {
  BH_ENTER(c);
  if (graph_id < 0 || graph_id >= (int)c->graphs.size() || !c->graphs[graph_id]) return bh::fail(BH_ERR, "bad graph id");
  BH_HIP(hipStreamSynchronize(c->stream));
  BH_HIP(hipGraphExecDestroy(c->graphs[graph_id]));
  c->graphs[graph_id] = nullptr;
  // outgrown workspaces were kept for the graphs that captured them: free them with the last one
  bool live_graph = false;
  for (hipGraphExec_t g : c->graphs) live_graph |= g != nullptr;
  if (!live_graph) {
    for (void *r : c->retired) BH_HIP(hipFree(r));
    c->retired.clear();
  }
  return BH_OK;
}

int bh_tune_set(bh_ctx *c, int op, int cfg_index, int splits) {
  BH_ENTER(c);
  return bh::tune_set(c, op, cfg_index, splits);
}

int bh_tune_set_policy(bh_ctx *c, int op, int wt) {
  BH_ENTER(c);
  return bh::tune_set_wt(c, op, wt);
}

int bh_tune_cfg_name(int op, int cfg_index, char *buf, size_t n) {
  if (!buf || !n) return bh::fail(BH_ERR, "null buffer");
  std::string s;
  int rc = bh::tune_cfg_name(op, cfg_index, s);
  if (rc == BH_OK) std::snprintf(buf, n, "%s", s.c_str());
  return rc;
}

}  // extern "C"
