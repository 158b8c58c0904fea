// bh_gendata.hip -- deterministic test-pattern generation on the device.
//
// Same values as Boda's gen_data_* CUCL templates over the reference layout,
// flat index i: test/rtc/gen-util.h:1-9 (det_hash_rand), gen_data_sgemm_a.cucl:7-19,
// gen_data_sgemm_b.cucl:8-20, gen_data_Convolution_{in,filts,biases}.cucl.
// The hash's final multiply-subtract is written as one fmaf (the reference
// JIT contracts it under --use_fast_math), so data is bit-reproducible.
// HBM-bound: one dwordx4 store per lane, grid-stride.
#include "bh_common.h"

namespace {

__device__ __forceinline__ float det_hash_rand(uint32_t rv) {
  uint32_t h = rv;
  h ^= h >> 16;
  h *= 0x85ebca6bu;
  h ^= h >> 13;
  h *= 0xc2b2ae35u;
  h ^= h >> 16;
  return __builtin_fmaf((float)h, 10.0f / 4294967296.0f, -5.0f);
}

struct gen_args {
  float *dst;
  uint64_t n;
  uint32_t d[4];  // outermost first
  uint32_t mode;
  float vi;
  int kind;
};

__device__ __forceinline__ float gen_one(const gen_args &g, uint64_t i) {
  float v = g.vi;
  uint32_t mode = g.mode;
  switch (g.kind) {
    case BH_GEN_SGEMM_A: {  // a K:M
      uint32_t M = g.d[1], K = g.d[0];
      uint32_t m = (uint32_t)(i % M), k = (uint32_t)(i / M);
      uint32_t fin = mode >= 100 ? mode / 100 : mode;
      if (fin == 2) v += (float)m;
      if (fin == 3) v += (float)k;
      else if (fin == 4) { if (m == M / 2 && k == K / 2) v += 1.0f; }
      else if (fin == 5) v += det_hash_rand((uint32_t)i + 12738732u);
      else if (fin == 6) v += (float)(m * 1000u + k);
      break;
    }
    case BH_GEN_SGEMM_B: {  // b K:N
      uint32_t N = g.d[1], K = g.d[0];
      uint32_t n = (uint32_t)(i % N), k = (uint32_t)(i / N);
      if (mode == 2) v += (float)n;
      if (mode == 3) v += (float)k;
      else if (mode == 4) { if (n == N / 2 && k == K / 2) v += 1.0f; }
      else if (mode == 5) v += det_hash_rand((uint32_t)i + 12738732u);
      else if (mode >= 100) { if (n == k) v += 1.0f; }
      break;
    }
    case BH_GEN_CONV_IN:
    case BH_GEN_CONV_FILTS: {  // img:chan:y:x / out_chan:in_chan:y:x
      uint32_t X = g.d[3], Y = g.d[2];
      uint32_t x = (uint32_t)(i % X), y = (uint32_t)((i / X) % Y);
      uint32_t seed = g.kind == BH_GEN_CONV_IN ? 234234567u : 8753985u;
      if (mode == 2) v += (float)x;
      if (mode == 3) v += (float)y;
      else if (mode == 4) { if (x == X / 2 && y == Y / 2) v += 1.0f; }
      else if (mode == 5) v += det_hash_rand((uint32_t)i + seed);
      break;
    }
    case BH_GEN_CONV_BIASES:
      if (mode == 5) v += det_hash_rand((uint32_t)i + 39475612u);
      break;
  }
  return v;
}

__global__ __launch_bounds__(256) void gen_data_kernel(gen_args g) {
  uint64_t nvec = g.n / 4;
  uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  bool aligned = (((uintptr_t)g.dst) & 15) == 0;
  if (aligned) {
    float4 *d4 = (float4 *)g.dst;
    for (uint64_t v = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += stride) {
      uint64_t i = v * 4;
      d4[v] = make_float4(gen_one(g, i), gen_one(g, i + 1), gen_one(g, i + 2), gen_one(g, i + 3));
    }
    for (uint64_t i = nvec * 4 + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < g.n; i += stride)
      g.dst[i] = gen_one(g, i);
  } else {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < g.n; i += stride)
      g.dst[i] = gen_one(g, i);
  }
}

}  // namespace

namespace bh {
int launch_gen_data(bh_ctx *ctx, int kind, float *dst, const uint32_t dims[4], uint32_t mode, float vi) {
  gen_args g;
  g.dst = dst;
  g.kind = kind;
  g.mode = mode;
  g.vi = vi;
  switch (kind) {
    case BH_GEN_SGEMM_A:
    case BH_GEN_SGEMM_B:
      g.d[0] = dims[0]; g.d[1] = dims[1]; g.d[2] = 1; g.d[3] = 1;
      g.n = (uint64_t)dims[0] * dims[1];
      break;
    case BH_GEN_CONV_IN:
    case BH_GEN_CONV_FILTS:
      for (int i = 0; i < 4; ++i) g.d[i] = dims[i];
      g.n = (uint64_t)dims[0] * dims[1] * dims[2] * dims[3];
      break;
    case BH_GEN_CONV_BIASES:
      g.d[0] = dims[0]; g.d[1] = g.d[2] = g.d[3] = 1;
      g.n = dims[0];
      break;
    default:
      return fail(BH_ERR, "bh_gen_data: unknown kind");
  }
  for (int i = 0; i < 4; ++i)
    if (!g.d[i]) return fail(BH_UNSUP, "bh_gen_data: zero dim");
  if (!g.n) return BH_OK;
  uint64_t want = (g.n / 4 + 255) / 256;
  uint32_t grid = (uint32_t)(want < 2048 ? (want ? want : 1) : 2048);
  void *args[] = {&g};
  return launch(ctx, (const void *)gen_data_kernel, dim3(grid), dim3(256), args, true, true, "gen_data");
}
}  // namespace bh
