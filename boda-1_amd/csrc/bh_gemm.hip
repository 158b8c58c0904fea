// bh_gemm.hip -- fp32 MFMA GEMM core for gfx950 and the two hot-path ops built on it:
//
//   SGEMM   c[M][N] = sum_k a[k][m] b[k][n]           (test/rtc/sgemm.cucl:1-3)
//   conv    out[n][oc][p] = act(bias[oc] + sum_k W[oc][k] * im2col[k][n,p])
//           (implicit GEMM over M = OC, N = B*OH*OW, K = IC*KY*KX; Caffe
//            semantics of test/rtc/conv.cucl:25-44, bias+ReLU of
//            src/cnn_codegen.cc:35-42)
//
// Design (MI355X-first, not a translation of the CUCL register-tile codegen):
//  * v_mfma_f32_32x32x2_f32: exact fp32 products and accumulation, 64 FLOP/clk/SIMD
//    = the f32 vector peak, operands one VGPR each (A[i=l&31][k=l>>5], B[k=l>>5][j=l&31]).
//  * A and B tiles live in LDS as [BK][BM] / [BK][BN] (k-rows). A wave owns a
//    TM x TN grid of 32x32 MFMA tiles; tile t's row i maps to m = wm0 + TM*i + t,
//    so one ds_read_b64/b128 returns a lane's operands for all TM (TN) tiles, and
//    in the epilogue each lane holds TN adjacent output columns (vector stores).
//  * Global->LDS staging through registers with a double-buffered LDS ring and one
//    barrier per K-tile; all global reads are buffer loads whose out-of-range /
//    padding elements are steered to an out-of-bounds offset and come back as 0
//    (no branches around loads, zero padding for free).
//  * Block->tile mapping is XCD-aware (bijective remap so blocks sharing an XCD's
//    L2 get neighbouring tiles) and grouped (8 m-tiles share each B panel).
//  * The conv B operand is gathered straight from NCHW input (implicit im2col):
//    a thread's output column (image, pixel) is fixed for the whole K loop, its k
//    row is wave-uniform, so the (ic, ky, kx) decomposition is scalar work.
#include "bh_common.h"

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4v __attribute__((ext_vector_type(4)));
typedef float f32x2v __attribute__((ext_vector_type(2)));

enum { A_KVEC = 0, A_KSCALAR = 1, A_MVEC = 2, A_MSCALAR = 3 };
enum { B_KVEC = 0, B_KSCALAR = 1, B_IM2COL = 2, B_IM1X1 = 3 };

constexpr uint32_t OOB = 0x80000000u;  // buffer offset that always misses (extents < 2^31)

struct GemmArgs {
  const float *a, *b;
  float *c;
  const float *bias;
  uint32_t M, N, K;
  uint32_t lda, ldb, ldc;
  uint64_t b_bstride, c_bstride;  // per blockIdx.z, dense B/C only
  uint32_t a_bytes, b_bytes;      // buffer extents in bytes (reads beyond come back 0)
  uint32_t tiles_m, tiles_n;
  int relu;
  int cvec;  // dense C rows can take TN-wide vector stores
  // implicit im2col (B_IM2COL / B_IM1X1); N = B*OH*OW, K = IC*KY*KX
  uint32_t H, W, KX, KYX, sy, sx, py, px, OW, OHW, HW, ICHW, OCOHW;
  uint32_t kyx_m, kyx_s, kx_m, kx_s, ohw_m, ohw_s, ow_m, ow_s;  // fastdiv constants
};

__device__ __forceinline__ uint32_t fdiv(uint32_t n, uint32_t m, uint32_t s) {
  return (__umulhi(n, m) + n) >> s;
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void *p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ f32x4v ld4(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_bit_cast(f32x4v, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}
__device__ __forceinline__ float ld1(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0));
}

__device__ __forceinline__ void map_tile(uint32_t bid, uint32_t tiles_m, uint32_t tiles_n, uint32_t &tm,
                                         uint32_t &tn) {
  uint32_t nwg = tiles_m * tiles_n;
  uint32_t xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  uint32_t wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  const uint32_t G = 8;
  uint32_t per_group = G * tiles_n;
  uint32_t group = wgid / per_group;
  uint32_t first_m = group * G;
  uint32_t gsm = min(tiles_m - first_m, G);
  uint32_t rem = wgid - group * per_group;
  tm = first_m + rem % gsm;
  tn = rem / gsm;
}

template <int N>
struct fvec;
template <>
struct fvec<1> { typedef float t; };
template <>
struct fvec<2> { typedef f32x2v t; };
template <>
struct fvec<4> { typedef f32x4v t; };

template <int BM, int BN, int BK, int TM, int TN, int WAVES_M, int WAVES_N, int ALD, int BLD>
__global__ __launch_bounds__(WAVES_M *WAVES_N * 64) void gemm_kernel(GemmArgs p) {
  constexpr int NT = WAVES_M * WAVES_N * 64;
  constexpr int WM = TM * 32, WN = TN * 32;
  static_assert(BM == WM * WAVES_M && BN == WN * WAVES_N, "tile shape");
  static_assert(BK % 2 == 0, "BK");
  constexpr bool IM = (BLD == B_IM2COL || BLD == B_IM1X1);
  static_assert(!IM || (NT % BN == 0), "im2col loader needs NT % BN == 0");

  __shared__ __attribute__((aligned(16))) float smem[2 * BK * (BM + BN)];
  float *const As = smem;
  float *const Bs = smem + 2 * BK * BM;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WAVES_N, wn = wave % WAVES_N;

  uint32_t tile_m, tile_n;
  map_tile(blockIdx.x, p.tiles_m, p.tiles_n, tile_m, tile_n);
  const uint32_t bm0 = tile_m * BM, bn0 = tile_n * BN;
  const uint32_t z = blockIdx.z;

  const __amdgpu_buffer_rsrc_t rsa = make_rsrc(p.a, p.a_bytes);
  const __amdgpu_buffer_rsrc_t rsb = make_rsrc(IM ? p.b : p.b + z * p.b_bstride, p.b_bytes);

  // ---- per-thread constants of the im2col gather (column fixed over the K loop)
  int col_base = 0, iy0 = 0, ix0 = 0;
  bool col_ok = false;
  if constexpr (IM) {
    const uint32_t col = bn0 + (uint32_t)(tid % BN);
    col_ok = col < p.N;
    const uint32_t img = fdiv(col, p.ohw_m, p.ohw_s);
    const uint32_t pix = col - img * p.OHW;
    if constexpr (BLD == B_IM1X1) {
      col_base = (int)(img * p.ICHW + pix);
    } else {
      const uint32_t oy = fdiv(pix, p.ow_m, p.ow_s);
      const uint32_t ox = pix - oy * p.OW;
      iy0 = (int)(oy * p.sy) - (int)p.py;
      ix0 = (int)(ox * p.sx) - (int)p.px;
      col_base = (int)(img * p.ICHW) + iy0 * (int)p.W + ix0;
    }
  }

  // ---- staging registers
  constexpr bool AV = (ALD == A_KVEC || ALD == A_MVEC);
  constexpr bool BV = (BLD == B_KVEC);
  constexpr int A_TOT = AV ? BM * BK / 4 : BM * BK;
  constexpr int A_PER = (A_TOT + NT - 1) / NT;
  constexpr int B_TOT = BV ? BN * BK / 4 : BN * BK;
  constexpr int B_PER = (B_TOT + NT - 1) / NT;
  f32x4v sa4[AV ? A_PER : 1];
  float sa1[AV ? 1 : A_PER];
  f32x4v sb4[BV ? B_PER : 1];
  float sb1[BV ? 1 : B_PER];

  auto load_tiles = [&](uint32_t k0) {
#pragma unroll
    for (int j = 0; j < A_PER; ++j) {
      const int idx = tid + j * NT;
      if (A_TOT % NT == 0 || idx < A_TOT) {
        if constexpr (ALD == A_KVEC) {
          const int kr = idx / (BM / 4), mc = idx % (BM / 4);
          const uint32_t m = bm0 + 4 * mc, k = k0 + kr;
          sa4[j] = ld4(rsa, (m < p.M && k < p.K) ? (k * p.lda + m) * 4u : OOB);
        } else if constexpr (ALD == A_KSCALAR) {
          const int kr = idx / BM, mc = idx % BM;
          const uint32_t m = bm0 + mc, k = k0 + kr;
          sa1[j] = ld1(rsa, (m < p.M && k < p.K) ? (k * p.lda + m) * 4u : OOB);
        } else if constexpr (ALD == A_MVEC) {
          const int mr = idx % BM, kc = idx / BM;
          const uint32_t m = bm0 + mr, k = k0 + 4 * kc;
          sa4[j] = ld4(rsa, (m < p.M && k < p.K) ? (m * p.lda + k) * 4u : OOB);
        } else {
          const int mr = idx % BM, kr = idx / BM;
          const uint32_t m = bm0 + mr, k = k0 + kr;
          sa1[j] = ld1(rsa, (m < p.M && k < p.K) ? (m * p.lda + k) * 4u : OOB);
        }
      }
    }
#pragma unroll
    for (int j = 0; j < B_PER; ++j) {
      const int idx = tid + j * NT;
      if (B_TOT % NT == 0 || idx < B_TOT) {
        if constexpr (BLD == B_KVEC) {
          const int kr = idx / (BN / 4), ncol = idx % (BN / 4);
          const uint32_t n = bn0 + 4 * ncol, k = k0 + kr;
          sb4[j] = ld4(rsb, (n < p.N && k < p.K) ? (k * p.ldb + n) * 4u : OOB);
        } else if constexpr (BLD == B_KSCALAR) {
          const int kr = idx / BN, ncol = idx % BN;
          const uint32_t n = bn0 + ncol, k = k0 + kr;
          sb1[j] = ld1(rsb, (n < p.N && k < p.K) ? (k * p.ldb + n) * 4u : OOB);
        } else {
          // this thread's k row; wave-uniform when BN is a multiple of 64
          uint32_t kr = (uint32_t)(idx / BN);
          if constexpr (BN % 64 == 0) kr = __builtin_amdgcn_readfirstlane(kr);
          const uint32_t k = k0 + kr;
          if constexpr (BLD == B_IM1X1) {
            const bool ok = col_ok && k < p.K;
            sb1[j] = ld1(rsb, ok ? (uint32_t)(col_base + (int)(k * p.HW)) * 4u : OOB);
          } else {
            // k = (ic * KY + ky) * KX + kx
            const uint32_t ic = fdiv(k, p.kyx_m, p.kyx_s);
            const uint32_t rem = k - ic * p.KYX;
            const uint32_t ky = fdiv(rem, p.kx_m, p.kx_s);
            const uint32_t kx = rem - ky * p.KX;
            const int iy = iy0 + (int)ky, ix = ix0 + (int)kx;
            const bool ok = col_ok && k < p.K && (uint32_t)iy < p.H && (uint32_t)ix < p.W;
            const int off = col_base + (int)(ic * p.HW + ky * p.W + kx);
            sb1[j] = ld1(rsb, ok ? (uint32_t)off * 4u : OOB);
          }
        }
      }
    }
  };

  auto store_tiles = [&](int buf) {
    float *const Ab = As + buf * BK * BM;
    float *const Bb = Bs + buf * BK * BN;
#pragma unroll
    for (int j = 0; j < A_PER; ++j) {
      const int idx = tid + j * NT;
      if (A_TOT % NT == 0 || idx < A_TOT) {
        if constexpr (ALD == A_KVEC) {
          const int kr = idx / (BM / 4), mc = idx % (BM / 4);
          *(f32x4v *)&Ab[kr * BM + 4 * mc] = sa4[j];
        } else if constexpr (ALD == A_KSCALAR) {
          const int kr = idx / BM, mc = idx % BM;
          Ab[kr * BM + mc] = sa1[j];
        } else if constexpr (ALD == A_MVEC) {
          const int mr = idx % BM, kc = idx / BM;
          Ab[(4 * kc + 0) * BM + mr] = sa4[j][0];
          Ab[(4 * kc + 1) * BM + mr] = sa4[j][1];
          Ab[(4 * kc + 2) * BM + mr] = sa4[j][2];
          Ab[(4 * kc + 3) * BM + mr] = sa4[j][3];
        } else {
          const int mr = idx % BM, kr = idx / BM;
          Ab[kr * BM + mr] = sa1[j];
        }
      }
    }
#pragma unroll
    for (int j = 0; j < B_PER; ++j) {
      const int idx = tid + j * NT;
      if (B_TOT % NT == 0 || idx < B_TOT) {
        if constexpr (BLD == B_KVEC) {
          const int kr = idx / (BN / 4), ncol = idx % (BN / 4);
          *(f32x4v *)&Bb[kr * BN + 4 * ncol] = sb4[j];
        } else {
          const int kr = idx / BN, ncol = idx % BN;
          Bb[kr * BN + ncol] = sb1[j];
        }
      }
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;

  auto compute = [&](int buf) {
    const float *const Ab = As + buf * BK * BM + wm * WM + TM * (lane & 31);
    const float *const Bb = Bs + buf * BK * BN + wn * WN + TN * (lane & 31);
    const int kh = lane >> 5;
#pragma unroll
    for (int kk = 0; kk < BK / 2; ++kk) {
      const int kr = 2 * kk + kh;
      typename fvec<TM>::t av = *(const typename fvec<TM>::t *)&Ab[kr * BM];
      typename fvec<TN>::t bv = *(const typename fvec<TN>::t *)&Bb[kr * BN];
      float a[TM], b[TN];
      if constexpr (TM == 1) a[0] = av; else {
#pragma unroll
        for (int i = 0; i < TM; ++i) a[i] = av[i];
      }
      if constexpr (TN == 1) b[0] = bv; else {
#pragma unroll
        for (int j = 0; j < TN; ++j) b[j] = bv[j];
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i], b[j], acc[i][j], 0, 0, 0);
    }
  };

  // ---- main loop: register-staged, double-buffered LDS, one barrier per K tile
  const uint32_t nkt = (p.K + BK - 1) / BK;
  load_tiles(0);
  store_tiles(0);
  __syncthreads();
  int buf = 0;
  for (uint32_t kt = 0; kt < nkt; ++kt) {
    const bool more = kt + 1 < nkt;
    if (more) load_tiles((kt + 1) * BK);
    compute(buf);
    if (more) store_tiles(buf ^ 1);
    __syncthreads();
    buf ^= 1;
  }

  // ---- epilogue: bias, ReLU, stores
  const uint32_t n_base = bn0 + wn * WN + TN * (lane & 31);
  int cofs[TN];
  if constexpr (IM) {
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const uint32_t col = n_base + j;
      const uint32_t img = fdiv(col, p.ohw_m, p.ohw_s);
      const uint32_t pix = col - img * p.OHW;
      cofs[j] = col < p.N ? (int)(img * p.OCOHW + pix) : -1;
    }
  }
  float *const cz = IM ? p.c : p.c + z * p.c_bstride;
#pragma unroll
  for (int i = 0; i < TM; ++i) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      const uint32_t m = bm0 + wm * WM + TM * row + i;
      if (m >= p.M) continue;
      float v[TN];
      const float bv = p.bias ? p.bias[m] : 0.0f;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        float x = acc[i][j][r] + bv;
        v[j] = (p.relu && x < 0.0f) ? 0.0f : x;
      }
      if constexpr (IM) {
        float *const crow = cz + (size_t)m * p.OHW;
#pragma unroll
        for (int j = 0; j < TN; ++j)
          if (cofs[j] >= 0) crow[cofs[j]] = v[j];
      } else {
        float *const crow = cz + (size_t)m * p.ldc + n_base;
        if (p.cvec && n_base + TN <= p.N) {
          typename fvec<TN>::t w;
          if constexpr (TN == 1) w = v[0]; else {
#pragma unroll
            for (int j = 0; j < TN; ++j) w[j] = v[j];
          }
          *(typename fvec<TN>::t *)crow = w;
        } else {
#pragma unroll
          for (int j = 0; j < TN; ++j)
            if (n_base + j < p.N) crow[j] = v[j];
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------
// host side: tile configurations and dispatch
// ---------------------------------------------------------------------------

struct TileCfg {
  int BM, BN, BK, TM, TN, WAVES_M, WAVES_N;
  const char *name;
};

// Instantiated configurations (name used for reporting / wisdom).
#define CFG_L 128, 128, 16, 2, 2, 2, 2  // 4 waves, 64x64 per wave
#define CFG_M 64, 128, 16, 1, 2, 2, 2   // 4 waves, 32x64 per wave (OC <= 64)
#define CFG_S 32, 256, 16, 1, 2, 1, 4   // 4 waves, 32x64 per wave (OC <= 32)

template <int BM, int BN, int BK, int TM, int TN, int WM_, int WN_, int ALD, int BLD>
int launch_cfg(bh_ctx *ctx, GemmArgs &p, uint32_t batch, const char *what) {
  p.tiles_m = (p.M + BM - 1) / BM;
  p.tiles_n = (p.N + BN - 1) / BN;
  const uint64_t nblk = (uint64_t)p.tiles_m * p.tiles_n;
  if (nblk > 0x7fffffffu || batch > 65535) return bh::fail(BH_UNSUP, std::string(what) + ": grid too large");
  hipLaunchKernelGGL((gemm_kernel<BM, BN, BK, TM, TN, WM_, WN_, ALD, BLD>), dim3((uint32_t)nblk, 1, batch),
                     dim3(WM_ * WN_ * 64), 0, ctx->stream, p);
  return bh::check_launch(what);
}

bool fits_buffer(uint64_t bytes) { return bytes < (uint64_t)OOB - 64; }

void set_fd(uint32_t d, uint32_t &m, uint32_t &s) {
  bh::fastdiv f = bh::make_fastdiv(d ? d : 1);
  m = f.m;
  s = f.s;
}

}  // namespace

namespace bh {

std::string sgemm_variant(uint32_t M, uint32_t N, uint32_t K) {
  (void)K;
  bool vec = (M % 4 == 0) && (N % 4 == 0);
  return std::string("mfma32_sgemm_128x128x16") + (vec ? "_vec" : "_scalar");
}

int launch_sgemm(bh_ctx *ctx, const float *a, const float *b, float *c, uint32_t M, uint32_t N, uint32_t K) {
  if (!fits_buffer((uint64_t)K * M * 4) || !fits_buffer((uint64_t)K * N * 4))
    return fail(BH_UNSUP, "sgemm: operand larger than 2 GiB");
  GemmArgs p{};
  p.a = a; p.b = b; p.c = c; p.bias = nullptr;
  p.M = M; p.N = N; p.K = K;
  p.lda = M; p.ldb = N; p.ldc = N;
  p.a_bytes = (uint32_t)((uint64_t)K * M * 4);
  p.b_bytes = (uint32_t)((uint64_t)K * N * 4);
  p.relu = 0;
  const bool vec = (M % 4 == 0) && (N % 4 == 0) && ((uintptr_t)a % 16 == 0) && ((uintptr_t)b % 16 == 0);
  p.cvec = (N % 2 == 0) && ((uintptr_t)c % 8 == 0);
  if (vec) return launch_cfg<CFG_L, A_KVEC, B_KVEC>(ctx, p, 1, "sgemm");
  return launch_cfg<CFG_L, A_KSCALAR, B_KSCALAR>(ctx, p, 1, "sgemm");
}

namespace {
struct conv_shape {
  uint32_t B, IC, H, W, OC, KY, KX, sy, sx, py, px, OH, OW;
};
int pick_tile(uint32_t OC) { return OC <= 32 ? 2 : (OC <= 64 ? 1 : 0); }
}  // namespace

std::string conv_variant(const uint32_t *d) {
  uint32_t IC = d[1], OC = d[4], KY = d[5], KX = d[6], sy = d[7], sx = d[8], py = d[9], px = d[10];
  bool k1 = KY == 1 && KX == 1 && sy == 1 && sx == 1 && py == 0 && px == 0;
  uint32_t K = IC * KY * KX;
  static const char *tiles[3] = {"128x128x16", "64x128x16", "32x256x16"};
  std::string s = std::string("mfma32_conv_") + (k1 ? "1x1_" : "im2col_") + tiles[pick_tile(OC)];
  s += (K % 4 == 0) ? "_avec" : "_ascalar";
  return s;
}

int launch_conv(bh_ctx *ctx, const float *in, const float *filts, const float *biases, float *out, uint32_t B,
                uint32_t IC, uint32_t H, uint32_t W, uint32_t OC, uint32_t KY, uint32_t KX, uint32_t sy,
                uint32_t sx, uint32_t py, uint32_t px, int relu) {
  const uint32_t OH = (H + 2 * py - KY) / sy + 1, OW = (W + 2 * px - KX) / sx + 1;
  const uint64_t K = (uint64_t)IC * KY * KX, P = (uint64_t)B * OH * OW;
  const uint64_t in_bytes = (uint64_t)B * IC * H * W * 4, w_bytes = (uint64_t)OC * K * 4;
  if (!fits_buffer(in_bytes) || !fits_buffer(w_bytes) || !fits_buffer((uint64_t)B * OC * OH * OW * 4))
    return fail(BH_UNSUP, "conv: tensor larger than 2 GiB");
  if (K >= (1u << 31) || P >= (1u << 31)) return fail(BH_UNSUP, "conv: GEMM extent too large");
  GemmArgs p{};
  p.a = filts; p.b = in; p.c = out; p.bias = biases;
  p.M = OC; p.N = (uint32_t)P; p.K = (uint32_t)K;
  p.lda = (uint32_t)K; p.ldb = 0; p.ldc = 0;
  p.a_bytes = (uint32_t)w_bytes;
  p.b_bytes = (uint32_t)in_bytes;
  p.relu = relu;
  p.cvec = 0;
  p.H = H; p.W = W; p.KX = KX; p.KYX = KY * KX;
  p.sy = sy; p.sx = sx; p.py = py; p.px = px;
  p.OW = OW; p.OHW = OH * OW; p.HW = H * W; p.ICHW = IC * H * W; p.OCOHW = OC * OH * OW;
  set_fd(p.KYX, p.kyx_m, p.kyx_s);
  set_fd(KX, p.kx_m, p.kx_s);
  set_fd(p.OHW, p.ohw_m, p.ohw_s);
  set_fd(OW, p.ow_m, p.ow_s);
  const bool k1 = KY == 1 && KX == 1 && sy == 1 && sx == 1 && py == 0 && px == 0;
  const bool avec = (K % 4 == 0) && ((uintptr_t)filts % 16 == 0);
  const int t = pick_tile(OC);
#define DISPATCH(CFG)                                                                              \
  do {                                                                                             \
    if (k1) {                                                                                      \
      if (avec) return launch_cfg<CFG, A_MVEC, B_IM1X1>(ctx, p, 1, "conv");                        \
      return launch_cfg<CFG, A_MSCALAR, B_IM1X1>(ctx, p, 1, "conv");                               \
    }                                                                                              \
    if (avec) return launch_cfg<CFG, A_MVEC, B_IM2COL>(ctx, p, 1, "conv");                         \
    return launch_cfg<CFG, A_MSCALAR, B_IM2COL>(ctx, p, 1, "conv");                                \
  } while (0)
  if (t == 0) DISPATCH(CFG_L);
  if (t == 1) DISPATCH(CFG_M);
  DISPATCH(CFG_S);
#undef DISPATCH
}

}  // namespace bh
