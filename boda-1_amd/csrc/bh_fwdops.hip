// bh_fwdops.hip -- the non-conv forward layers of Boda's net executor (conv_pipe_fwd_t,
// src/rtc_fwd.cc:263-405) as gfx950 kernels: Pooling, LRN, ReLU, Softmax, and the channel
// copies behind Concat / Split. All are HBM-bound (a few flops per byte): one pass over the
// input, coalesced along x (or along the flat index), results as the reference kernels
// compute them (test/rtc/{pool,lrn,relu,softmax,copy,split_copy}.cucl).
#include "bh_common.h"

#include <cfloat>

namespace {

// Pooling (test/rtc/pool.cucl): one thread per output element; only non-padding pixels
// count, for max and for average (the average divides by the number of in-image taps).
// out_in_yx (may be null): for max pooling, the in_y*W + in_x of the winning input (-1 if
// none), stored as a float as the reference does.
// KY_/KX_ > 0: the window is a compile-time constant (3x3 and 2x2: every pooling layer of
// the reference nets but the global ones), so the loop unrolls and all taps' loads issue
// together instead of one guarded load per loop trip.
template <int KY_, int KX_>
__global__ __launch_bounds__(256) void pool_kernel(const float *__restrict__ in, float *__restrict__ out,
                                                   float *__restrict__ out_in_yx, uint32_t total, uint32_t C,
                                                   uint32_t H, uint32_t W, uint32_t OH, uint32_t OW, uint32_t KY_rt,
                                                   uint32_t KX_rt, uint32_t sy, uint32_t sx, uint32_t py, uint32_t px,
                                                   int avg, uint32_t ow_m, uint32_t ow_s, uint32_t oh_m, uint32_t oh_s) {
  const uint32_t KY = KY_ > 0 ? (uint32_t)KY_ : KY_rt, KX = KX_ > 0 ? (uint32_t)KX_ : KX_rt;
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  // i -> (nc, oy, ox) with multiply-shift division (nc = img * C + chan)
  const uint32_t t = (__umulhi(i, ow_m) + i) >> ow_s, ox = i - t * OW;
  const uint32_t nc = (__umulhi(t, oh_m) + t) >> oh_s, oy = t - nc * OH;
  const float *const src = in + (size_t)nc * H * W;
  float v = avg ? 0.0f : -FLT_MAX, cnt = 0.0f;
  int oyx = -1;
  // the reference's loop order (kx outer, ky inner) decides ties and the summation order; a
  // tap in the padding loads src[0] (always valid) and is then ignored, so no load is guarded
  auto tap = [&](uint32_t ky, uint32_t kx) {
    const int iy = (int)(oy * sy + ky) - (int)py, ix = (int)(ox * sx + kx) - (int)px;
    const bool ok = iy >= 0 && ix >= 0 && ix < (int)W && iy < (int)H;
    const float x = src[ok ? iy * (int)W + ix : 0];
    if (ok) {
      if (avg) {
        v += x;
        cnt += 1.0f;
      } else if (x > v) {
        v = x;
        oyx = iy * (int)W + ix;
      }
    }
  };
  if constexpr (KY_ > 0 && KX_ > 0) {
#pragma unroll
    for (int kx = 0; kx < KX_; ++kx)
#pragma unroll
      for (int ky = 0; ky < KY_; ++ky) tap(ky, kx);
  } else {
    for (uint32_t kx = 0; kx < KX; ++kx)
      for (uint32_t ky = 0; ky < KY; ++ky) tap(ky, kx);
  }
  if (avg) v /= cnt;
  out[i] = v;
  if (out_in_yx) out_in_yx[i] = (float)oyx;
  (void)C;
}

// Pooling staged through LDS (round 6), used for the windows pool_kernel loops over at run time
// (global pooling: 49 dependent-address taps per thread there). pool_kernel reads every tap
// straight from global memory: lanes S floats apart, KY*KX dword loads per output. Here a
// block copies a band of whole input rows -- or several whole planes when a plane is small -- into
// LDS with coalesced loads (each input float read once, plus KY - sy overlap rows per band), then
// computes the band's outputs from LDS in pool_kernel's tap order (kx outer, ky inner: the same
// max / argmax ties and the same average summation order, so the results are bitwise the same).
// Block = (plane group of PPB planes, output row band of RB rows); PPB > 1 only when RB covers OH.
constexpr int POOL_LDS = 8192;  // floats of input staged per block
__global__ __launch_bounds__(256) void pool_lds_kernel(const float *__restrict__ in, float *__restrict__ out,
                                                       float *__restrict__ out_in_yx, uint32_t NC, uint32_t H,
                                                       uint32_t W, uint32_t OH, uint32_t OW, uint32_t KY, uint32_t KX,
                                                       uint32_t sy, uint32_t sx, uint32_t py, uint32_t px, int avg,
                                                       uint32_t RB, uint32_t PPB, uint32_t nbands, uint32_t ow_m,
                                                       uint32_t ow_s, uint32_t oh_m, uint32_t oh_s) {
  __shared__ float t[POOL_LDS];
  const uint32_t band = blockIdx.x % nbands, nc0 = (blockIdx.x / nbands) * PPB;
  const uint32_t np = min(PPB, NC - nc0);
  const uint32_t oy0 = band * RB, oy1 = min(OH, oy0 + RB);
  // staged input rows [iy0, iy0 + rows): whole planes when PPB > 1 (then RB >= OH and the planes
  // are one contiguous run), else the rows the band's windows touch, clipped to the image
  int iy0 = 0, iy1 = (int)H;
  if (PPB == 1) {
    iy0 = max(0, (int)(oy0 * sy) - (int)py);
    iy1 = min((int)H, (int)((oy1 - 1) * sy + KY) - (int)py);
  }
  const uint32_t rows = iy1 > iy0 ? (uint32_t)(iy1 - iy0) : 0u, per = rows * W, total = np * per;
  const float *const src = in + (size_t)nc0 * H * W + (size_t)iy0 * W;
  // all of a thread's loads in flight together, then the LDS writes (total <= POOL_LDS)
  float r[POOL_LDS / 256];
#pragma unroll
  for (int j = 0; j < POOL_LDS / 256; ++j) {
    const uint32_t e = threadIdx.x + 256u * j;
    r[j] = e < total ? src[e] : 0.0f;
  }
#pragma unroll
  for (int j = 0; j < POOL_LDS / 256; ++j) {
    const uint32_t e = threadIdx.x + 256u * j;
    if (e < total) t[e] = r[j];
  }
  __syncthreads();
  const uint32_t nrow = oy1 - oy0, nout = np * nrow * OW;
  for (uint32_t o = threadIdx.x; o < nout; o += 256) {
    const uint32_t q = (__umulhi(o, ow_m) + o) >> ow_s, ox = o - q * OW;  // q = plane * nrow + row
    uint32_t pl = 0, ry = q;
    if (PPB > 1) {  // nrow == OH
      pl = (__umulhi(q, oh_m) + q) >> oh_s;
      ry = q - pl * OH;
    }
    const uint32_t oy = oy0 + ry;
    const float *const T = t + pl * per;
    float v = avg ? 0.0f : -FLT_MAX, cnt = 0.0f;
    int oyx = -1;
    auto tap = [&](uint32_t ky, uint32_t kx) {
      const int iy = (int)(oy * sy + ky) - (int)py, ix = (int)(ox * sx + kx) - (int)px;
      const bool ok = iy >= 0 && ix >= 0 && ix < (int)W && iy < (int)H;
      const float x = T[ok ? (iy - iy0) * (int)W + ix : 0];
      if (ok) {
        if (avg) {
          v += x;
          cnt += 1.0f;
        } else if (x > v) {
          v = x;
          oyx = iy * (int)W + ix;
        }
      }
    };
    for (uint32_t kx = 0; kx < KX; ++kx)
      for (uint32_t ky = 0; ky < KY; ++ky) tap(ky, kx);
    if (avg) v /= cnt;
    const size_t i = ((size_t)(nc0 + pl) * OH + oy) * OW + ox;
    out[i] = v;
    if (out_in_yx) out_in_yx[i] = (float)oyx;
  }
}

// LRN across channels (test/rtc/lrn.cucl, LRN_MATCH_CAFFE): a running sum of squares over a
// window of LS channels kept with a ring of the last LS inputs (+ new^2 - old^2, the
// reference's order), out = in * (k + alpha/LS * sum)^-beta.
// The reference gives each (img, y, x) one thread walking all C channels: a serial chain of C
// powf's and loads on only B*H*W threads (14580 for AlexNet norm2 at batch 20, < 1 wave per
// SIMD). Here a thread owns LRN_CH output channels of one pixel (threads of a wave: adjacent
// pixels, coalesced): it loads its LRN_CH + LS - 1 inputs up front and runs the same ring
// from channel c0 - LS/2 (zeros before channel 0, as the reference's ring starts). The first
// chunk is the reference's sequence exactly; later chunks start their running sum fresh (the
// window sum without the earlier channels' +/- residue: within 1 ulp-scale of it).
constexpr int LRN_CH = 16;
template <int LS>
__global__ __launch_bounds__(256) void lrn_kernel(const float *__restrict__ in, float *__restrict__ out,
                                                  float *__restrict__ out_scale_base, uint32_t npix, uint32_t C,
                                                  uint32_t HW, float alpha, float beta, float k, uint32_t total) {
  const uint32_t t = blockIdx.x * 256 + threadIdx.x;
  if (t >= total) return;
  const uint32_t chunk = t / npix, i = t - chunk * npix;
  const uint32_t img = i / HW, pix = i - img * HW;
  const size_t base = (size_t)img * C * HW + pix;
  constexpr int hls = LS >> 1, NI = LRN_CH + 2 * hls;
  const int c0 = (int)chunk * LRN_CH;  // first output channel
  const float alpha_over_ls = alpha / (float)LS;
  float x[NI];  // inputs c0 - hls .. c0 + LRN_CH + hls - 1
#pragma unroll
  for (int j = 0; j < NI; ++j) {
    const int c = c0 - hls + j;
    x[j] = (c >= 0 && c < (int)C) ? in[base + (size_t)c * HW] : 0.0f;
  }
  float sum = 0.0f;
#pragma unroll
  for (int j = 0; j < NI; ++j) {
    const float old = j >= LS ? x[j - LS] : 0.0f;  // the ring slot's previous occupant
    sum += x[j] * x[j];
    sum -= old * old;
    const int oc = c0 - hls + j - hls;
    if (j >= 2 * hls && oc < (int)C) {
      const float sb = k + sum * alpha_over_ls;
      if (out_scale_base) out_scale_base[base + (size_t)oc * HW] = sb;
      // sb^-beta as exp2(-beta * log2(sb)) on the hardware transcendentals (v_log_f32 /
      // v_exp_f32): what the reference's kernels get from nvrtc --use_fast_math (__powf,
      // src/nvrtc_util.cc:251); an accurate powf made this layer instruction-latency bound
      out[base + (size_t)oc * HW] = x[j - hls] * __builtin_amdgcn_exp2f(-beta * __builtin_amdgcn_logf(sb));
    }
  }
}

// ReLU in place (test/rtc/relu.cucl): x <= 0 -> 0.
__global__ __launch_bounds__(256) void relu_kernel(float *__restrict__ x, uint64_t n) {
  const uint64_t n4 = n / 4;
  float4 *const x4 = (float4 *)x;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (uint64_t)gridDim.x * 256) {
    float4 v = x4[i];
    v.x = v.x <= 0.0f ? 0.0f : v.x;
    v.y = v.y <= 0.0f ? 0.0f : v.y;
    v.z = v.z <= 0.0f ? 0.0f : v.z;
    v.w = v.w <= 0.0f ? 0.0f : v.w;
    x4[i] = v;
  }
  if (blockIdx.x == 0 && threadIdx.x < n - n4 * 4) {
    float &v = x[n4 * 4 + threadIdx.x];
    v = v <= 0.0f ? 0.0f : v;
  }
}

// Deterministic dropout in place (test/rtc/dropout.cucl, the rtc mode's Dropout with
// has_conv_fwd_t::set_det_drop_seed): element i is kept, scaled by 1 / (1 - ratio), iff the
// murmur3 finalizer of i + seed exceeds U32_MAX * ratio; else zeroed.
__global__ __launch_bounds__(256) void dropout_kernel(float *__restrict__ x, uint32_t n, uint32_t thresh, float scale,
                                                      uint32_t seed) {
  for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    uint32_t h = i + seed;
    h ^= h >> 16;
    h *= 0x85ebca6bu;
    h ^= h >> 13;
    h *= 0xc2b2ae35u;
    h ^= h >> 16;
    x[i] = h > thresh ? x[i] * scale : 0.0f;
  }
}

// Softmax over channels per pixel (test/rtc/softmax.cucl): max starts at 0 (as the reference),
// exp(x - max), then divide by the sum.
__global__ __launch_bounds__(256) void softmax_kernel(const float *__restrict__ in, float *__restrict__ prob,
                                                      uint32_t npix, uint32_t C, uint32_t HW) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= npix) return;
  const uint32_t img = i / HW, pix = i - img * HW;
  const size_t base = (size_t)img * C * HW + pix;
  float mx = 0.0f, sum = 0.0f;
  for (uint32_t c = 0; c < C; ++c) mx = fmaxf(mx, in[base + (size_t)c * HW]);
  for (uint32_t c = 0; c < C; ++c) {
    const float v = expf(in[base + (size_t)c * HW] - mx);
    prob[base + (size_t)c * HW] = v;
    sum += v;
  }
  for (uint32_t c = 0; c < C; ++c) prob[base + (size_t)c * HW] /= sum;
}

// Channel-slab copy between NCHW tensors of equal H x W: out[img][c + oc0] = in[img][c + ic0]
// for c < nc (Concat: copy.cucl with ocix; Split: split_copy.cucl with icix). Each image's
// slab is contiguous on both sides: float4 when both offsets are 16-B aligned.
__global__ __launch_bounds__(256) void chan_copy_kernel(const float *__restrict__ in, float *__restrict__ out,
                                                        uint32_t B, uint64_t slab, uint64_t in_img, uint64_t out_img,
                                                        uint64_t in_off, uint64_t out_off, int vec) {
  const uint32_t img = blockIdx.y;
  const float *const s = in + img * in_img + in_off;
  float *const d = out + img * out_img + out_off;
  if (vec) {
    const uint64_t n4 = slab / 4;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (uint64_t)gridDim.x * 256)
      ((float4 *)d)[i] = ((const float4 *)s)[i];
  } else {
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < slab; i += (uint64_t)gridDim.x * 256) d[i] = s[i];
  }
  (void)B;
}

// Per-channel affine y = x * scale[c] + shift[c] (+ ReLU): inference BatchNorm followed by
// Scale, folded (resnet prototxts; not in the reference's rtc_fwd). One block row
// per (img, chan) slab, float4 along the pixels when HW % 4 == 0.
__global__ __launch_bounds__(256) void chan_affine_kernel(const float *__restrict__ in, float *__restrict__ out,
                                                          const float *__restrict__ scale,
                                                          const float *__restrict__ shift, uint32_t C, uint32_t HW,
                                                          int relu) {
  const uint32_t nc = blockIdx.y, c = nc % C;
  const float a = scale[c], b = shift[c];
  const size_t base = (size_t)nc * HW;
  if (HW % 4 == 0) {
    const float4 *s = (const float4 *)(in + base);
    float4 *d = (float4 *)(out + base);
    for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < HW / 4; i += gridDim.x * 256) {
      float4 v = s[i];
      v.x = fmaf(v.x, a, b); v.y = fmaf(v.y, a, b); v.z = fmaf(v.z, a, b); v.w = fmaf(v.w, a, b);
      if (relu) {
        v.x = v.x <= 0.0f ? 0.0f : v.x; v.y = v.y <= 0.0f ? 0.0f : v.y;
        v.z = v.z <= 0.0f ? 0.0f : v.z; v.w = v.w <= 0.0f ? 0.0f : v.w;
      }
      d[i] = v;
    }
  } else {
    for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < HW; i += gridDim.x * 256) {
      float v = fmaf(in[base + i], a, b);
      out[base + i] = (relu && v <= 0.0f) ? 0.0f : v;
    }
  }
}

// Elementwise combine of two tensors (Caffe Eltwise: 0 PROD, 1 SUM, 2 MAX) (+ ReLU).
__global__ __launch_bounds__(256) void eltwise_kernel(const float *__restrict__ a, const float *__restrict__ b,
                                                      float *__restrict__ out, uint64_t n, int op, int relu) {
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
    const float x = a[i], y = b[i];
    float v = op == 0 ? x * y : (op == 1 ? x + y : fmaxf(x, y));
    out[i] = (relu && v <= 0.0f) ? 0.0f : v;
  }
}

uint32_t grid_for(uint64_t n, uint32_t cap = 16384) {
  return (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((n + 255) / 256, cap));
}

}  // namespace

namespace bh {

uint32_t pool_out_sz(uint32_t in, uint32_t k, uint32_t s, uint32_t p) {
  // Caffe pooling: a partial last window makes one more output (src/conv_util.cc:198-204)
  const uint32_t pin = in + 2 * p;
  if (pin < k) return 1;
  return (pin - k + s - 1) / s + 1;
}

int launch_pool(bh_ctx *ctx, const float *in, float *out, float *out_in_yx, uint32_t B, uint32_t C, uint32_t H,
                uint32_t W, uint32_t KY, uint32_t KX, uint32_t sy, uint32_t sx, uint32_t py, uint32_t px, int avg) {
  const uint32_t OH = pool_out_sz(H, KY, sy, py), OW = pool_out_sz(W, KX, sx, px);
  const uint64_t total = (uint64_t)B * C * OH * OW;
  if (total >= (1ull << 31) || (uint64_t)B * C * H * W >= (1ull << 31)) return fail(BH_UNSUP, "pool: tensor too large");
  uint32_t tot = (uint32_t)total;
  const fastdiv fow = make_fastdiv(OW), foh = make_fastdiv(OH);
  uint32_t ow_m = fow.m, ow_s = fow.s, oh_m = foh.m, oh_s = foh.s;
  // the LDS-staged form for the windows without a compile-time kernel (global / large windows: the
  // googlenet 7x7 average pool 10.7 -> 8.2 us at batch 20), where a band of at least one output row
  // fits POOL_LDS floats: whole planes (PPB of them, at least 512 blocks where there are enough
  // planes) when a plane fits, else bands of RB output rows of one plane. On the 3x3 and 2x2 pools
  // it measured slower than pool_kernel (googlenet pool1 31.7 -> 34.9 us, inception 3x3 s1 15.0 ->
  // 27.6 us, VGG pool2 37.0 -> 40.8 us; profiles/r06/layers/): those keep the global-memory form
  uint32_t NC = B * C, RB = 0, PPB = 1, nbands = 1;
  const bool fixed = (KY == 3 && KX == 3) || (KY == 2 && KX == 2);
  if (fixed) {
  } else if ((uint64_t)H * W <= (uint64_t)POOL_LDS) {
    RB = OH;
    PPB = std::max(1u, std::min<uint32_t>((uint32_t)POOL_LDS / (H * W), NC / 512));
  } else if (W <= (uint32_t)POOL_LDS && (uint32_t)POOL_LDS / W >= KY) {
    RB = std::min(OH, ((uint32_t)POOL_LDS / W - KY) / sy + 1);
    nbands = (OH + RB - 1) / RB;
  }
  if (RB) {
    const uint64_t blocks = (uint64_t)((NC + PPB - 1) / PPB) * nbands;
    if (blocks < (1ull << 31)) {
      void *la[] = {&in, &out, &out_in_yx, &NC, &H, &W, (void *)&OH, (void *)&OW, &KY, &KX, &sy, &sx, &py, &px,
                    &avg, &RB, &PPB, &nbands, &ow_m, &ow_s, &oh_m, &oh_s};
      return launch(ctx, (const void *)pool_lds_kernel, dim3((uint32_t)blocks), dim3(256), la, true, true, "pool");
    }
  }
  void *args[] = {&in,  &out, &out_in_yx, &tot, &C,   &H,   &W,   (void *)&OH, (void *)&OW, &KY,
                  &KX,  &sy,  &sx,        &py,  &px,  &avg, &ow_m, &ow_s,      &oh_m,       &oh_s};
  const void *kern = KY == 3 && KX == 3   ? (const void *)pool_kernel<3, 3>
                     : KY == 2 && KX == 2 ? (const void *)pool_kernel<2, 2>
                                          : (const void *)pool_kernel<0, 0>;
  return launch(ctx, kern, dim3((tot + 255) / 256), dim3(256), args, true, true, "pool");
}

int launch_lrn(bh_ctx *ctx, const float *in, float *out, float *out_scale_base, uint32_t B, uint32_t C, uint32_t H,
               uint32_t W, uint32_t local_size, float alpha, float beta, float k) {
  const uint64_t np = (uint64_t)B * H * W;
  if (np * C >= (1ull << 31)) return fail(BH_UNSUP, "lrn: tensor too large");
  const uint64_t tot64 = np * ((C + LRN_CH - 1) / LRN_CH);  // threads: pixels x channel chunks
  uint32_t npix = (uint32_t)np, HW = H * W, total = (uint32_t)tot64;
  void *args[] = {&in, &out, &out_scale_base, &npix, &C, &HW, &alpha, &beta, &k, &total};
  const void *kern = nullptr;
  switch (local_size) {
    case 1: kern = (const void *)lrn_kernel<1>; break;
    case 3: kern = (const void *)lrn_kernel<3>; break;
    case 5: kern = (const void *)lrn_kernel<5>; break;
    case 7: kern = (const void *)lrn_kernel<7>; break;
    case 9: kern = (const void *)lrn_kernel<9>; break;
    case 11: kern = (const void *)lrn_kernel<11>; break;
    default: return fail(BH_UNSUP, "lrn: local_size must be odd and <= 11");
  }
  return launch(ctx, kern, dim3((total + 255) / 256), dim3(256), args, true, true, "lrn");
}

int launch_relu(bh_ctx *ctx, float *x, uint64_t n) {
  if ((uintptr_t)x % 16) return fail(BH_UNSUP, "relu: pointer must be 16-byte aligned");
  void *args[] = {&x, &n};
  return launch(ctx, (const void *)relu_kernel, dim3(grid_for(n / 4 + 1)), dim3(256), args, true, true, "relu");
}

int launch_dropout(bh_ctx *ctx, float *x, uint64_t n, float ratio, uint32_t seed) {
  if (!(ratio > 0.0f && ratio < 1.0f)) return fail(BH_ERR, "dropout: ratio must be in (0, 1)");
  if (n >= (1ull << 32)) return fail(BH_UNSUP, "dropout: tensor too large");
  // the reference substitutes the ratio into its kernel text: double arithmetic on both
  uint32_t n32 = (uint32_t)n, thresh = (uint32_t)(4294967295.0 * (double)ratio);
  float scale = (float)(1.0 / (1.0 - (double)ratio));
  void *args[] = {&x, &n32, &thresh, &scale, &seed};
  return launch(ctx, (const void *)dropout_kernel, dim3(grid_for(n)), dim3(256), args, true, true, "dropout");
}

int launch_softmax(bh_ctx *ctx, const float *in, float *prob, uint32_t B, uint32_t C, uint32_t H, uint32_t W) {
  const uint64_t np = (uint64_t)B * H * W;
  if (np * C >= (1ull << 31)) return fail(BH_UNSUP, "softmax: tensor too large");
  uint32_t npix = (uint32_t)np, HW = H * W;
  void *args[] = {&in, &prob, &npix, &C, &HW};
  return launch(ctx, (const void *)softmax_kernel, dim3((npix + 255) / 256), dim3(256), args, true, true, "softmax");
}

int launch_chan_copy(bh_ctx *ctx, const float *in, float *out, uint32_t B, uint32_t HW, uint32_t in_c, uint32_t ic0,
                     uint32_t out_c, uint32_t oc0, uint32_t nc) {
  if (ic0 + nc > in_c || oc0 + nc > out_c) return fail(BH_ERR, "chan_copy: channel range out of bounds");
  uint64_t slab = (uint64_t)nc * HW, in_img = (uint64_t)in_c * HW, out_img = (uint64_t)out_c * HW;
  uint64_t in_off = (uint64_t)ic0 * HW, out_off = (uint64_t)oc0 * HW;
  int vec = (slab % 4 == 0 && in_img % 4 == 0 && out_img % 4 == 0 && in_off % 4 == 0 && out_off % 4 == 0 &&
             (uintptr_t)in % 16 == 0 && (uintptr_t)out % 16 == 0);
  if (!B || !slab) return BH_OK;
  void *args[] = {&in, &out, &B, &slab, &in_img, &out_img, &in_off, &out_off, &vec};
  uint32_t gx = grid_for(vec ? slab / 4 : slab, 4096);
  return launch(ctx, (const void *)chan_copy_kernel, dim3(gx, B), dim3(256), args, true, true, "chan_copy");
}

int launch_chan_affine(bh_ctx *ctx, const float *in, float *out, const float *scale, const float *shift, uint32_t B,
                       uint32_t C, uint32_t HW, int relu) {
  if ((uint64_t)B * C > 65535u * 1024u || !B || !C || !HW) return fail(BH_UNSUP, "chan_affine: bad extent");
  if (HW % 4 == 0 && ((uintptr_t)in % 16 || (uintptr_t)out % 16)) return fail(BH_UNSUP, "chan_affine: unaligned");
  uint32_t gx = grid_for(HW % 4 == 0 ? HW / 4 : HW, 64);
  void *args[] = {&in, &out, &scale, &shift, &C, &HW, &relu};
  return launch(ctx, (const void *)chan_affine_kernel, dim3(gx, B * C), dim3(256), args, true, true, "chan_affine");
}

int launch_eltwise(bh_ctx *ctx, const float *a, const float *b, float *out, uint64_t n, int op, int relu) {
  if (op < 0 || op > 2) return fail(BH_UNSUP, "eltwise: op must be 0 (PROD), 1 (SUM) or 2 (MAX)");
  void *args[] = {&a, &b, &out, &n, &op, &relu};
  return launch(ctx, (const void *)eltwise_kernel, dim3(grid_for(n)), dim3(256), args, true, true, "eltwise");
}

}  // namespace bh
