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
//    The two lane halves carry different k; we assign half h the k rows
//    h*BK/2 .. h*BK/2+BK/2-1 of a K tile (any k order is a valid reduction order),
//    so an m-major A tile is read 4 k at a time with one ds_read_b128.
//  * LDS tiles: B [BK][BN] (k rows); A [BK][BM] when A is k-major (SGEMM's a),
//    [BM][BK+4] when A is m-major (conv weights OC x IC*KY*KX), so 8 lanes stream
//    one 128-B weight row segment with dwordx4 loads. A wave owns a TM x TN grid of
//    32x32 MFMA tiles; tile t's row i maps to m = wm0 + TM*i + t, so one vector LDS
//    read returns a lane's operands for all TM (TN) tiles, and in the epilogue each
//    lane holds TN adjacent output columns (vector stores).
//  * Register-staged double-buffered LDS ring, one barrier per K tile; every global
//    read is a buffer load whose out-of-range / padding elements are steered to an
//    out-of-bounds offset and come back as 0 (no branches around loads).
//  * Split-K for grids that cannot fill 256 CUs: split s writes raw partial sums to a
//    workspace slab; a second HBM-bound kernel sums the slabs in fixed order
//    (bitwise reproducible), adds bias, applies ReLU and scatters to NCHW.
//  * Block->tile mapping is XCD-aware (bijective remap so blocks sharing an XCD's
//    L2 get neighbouring tiles) and grouped (8 m-tiles share each B panel).
//  * The conv B operand is gathered straight from NCHW input (implicit im2col):
//    a thread's output column (image, pixel) is fixed for the whole K loop, its k
//    row is wave-uniform, so the (ic, ky, kx) decomposition is scalar work.
#include "bh_common.h"
#include "bh_gemm_dev.h"

namespace {

using namespace bhk;


// SPL: 0 = whole K per block; 1 = split-K, partial slabs combined by splitk_reduce_kernel;
//      2 = split-K, the last-arriving block of a tile combines the slabs in fixed order.
template <int BM, int BN, int BK, int TM, int TN, int WAVES_M, int WAVES_N, int ALD, int BLD, int SPL>
__global__ __launch_bounds__(WAVES_M *WAVES_N * 64) void gemm_kernel(GemmArgs p) {
  constexpr int NT = WAVES_M * WAVES_N * 64;
  constexpr int WM = TM * 32, WN = TN * 32;
  static_assert(BM == WM * WAVES_M && BN == WN * WAVES_N, "tile shape");
  static_assert(BK % 8 == 0, "BK must be a multiple of 8");
  constexpr bool IM = (BLD == B_IM2COL || BLD == B_IM1X1);
  constexpr bool AMM = (ALD == A_MVEC || ALD == A_MSCALAR);  // m-major A tile in LDS
  static_assert(!IM || (NT % BN == 0), "im2col loader needs NT % BN == 0");
  constexpr int A_LDS = AMM ? BM * (BK + APAD) : BK * BM;  // floats per A buffer
  constexpr int B_LDS = BK * BN;
  constexpr int AST = BK + APAD;  // m-major A row stride

  // conv (IM) kernels stage the block's BM biases in LDS behind the tiles
  __shared__ __attribute__((aligned(16))) float smem[2 * (A_LDS + B_LDS) + (IM ? BM : 0)];
  float *const As = smem;
  float *const Bs = smem + 2 * A_LDS;
  float *const Lbias = smem + 2 * (A_LDS + B_LDS);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WAVES_N, wn = wave % WAVES_N;
  KT(0);

  uint32_t tile_m, tile_n;
  map_tile(blockIdx.x, p.tiles_m, p.tiles_n, tile_m, tile_n);
  const uint32_t bm0 = tile_m * BM, bn0 = tile_n * BN;
  constexpr bool SPLIT = SPL != 0;
  const uint32_t split = SPLIT ? blockIdx.y : 0;
  const uint32_t kbeg = split * p.ks;
  const uint32_t kend = SPLIT ? min(p.K, kbeg + p.ks) : p.K;

  const __amdgpu_buffer_rsrc_t rsa = make_rsrc(p.a, p.a_bytes);
  const __amdgpu_buffer_rsrc_t rsb = make_rsrc(p.b, p.b_bytes);

  // ---- per-thread constants of the im2col gather (column fixed over the K loop)
  int col_base = 0, iy0 = 0, ix0 = 0;
  uint32_t col_oob = 0;  // OOB for a column past N: or-ed into every offset (no per-load branch)
  if constexpr (IM) {
    const uint32_t col = bn0 + (uint32_t)(tid % BN);
    col_oob = col < p.N ? 0u : OOB;
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
          sa4[j] = ld4(rsa, oob_unless((m < p.M) & (k < p.K), (k * p.lda + m) * 4u));
        } else if constexpr (ALD == A_KSCALAR) {
          const int kr = idx / BM, mc = idx % BM;
          const uint32_t m = bm0 + mc, k = k0 + kr;
          sa1[j] = ld1(rsa, oob_unless((m < p.M) & (k < p.K), (k * p.lda + m) * 4u));
        } else if constexpr (ALD == A_MVEC) {
          const int kc = idx % (BK / 4), mr = idx / (BK / 4);
          const uint32_t m = bm0 + mr, k = k0 + 4 * kc;
          sa4[j] = ld4(rsa, oob_unless((m < p.M) & (k < p.K), (m * p.lda + k) * 4u));
        } else {
          const int kr = idx % BK, mr = idx / BK;
          const uint32_t m = bm0 + mr, k = k0 + kr;
          sa1[j] = ld1(rsa, oob_unless((m < p.M) & (k < p.K), (m * p.lda + k) * 4u));
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
          sb4[j] = ld4(rsb, oob_unless((n < p.N) & (k < p.K), (k * p.ldb + n) * 4u));
        } else if constexpr (BLD == B_KSCALAR) {
          const int kr = idx / BN, ncol = idx % BN;
          const uint32_t n = bn0 + ncol, k = k0 + kr;
          sb1[j] = ld1(rsb, oob_unless((n < p.N) & (k < p.K), (k * p.ldb + n) * 4u));
        } else {
          // this thread's k row; wave-uniform when BN is a multiple of 64
          uint32_t kr = (uint32_t)(idx / BN);
          if constexpr (BN % 64 == 0) kr = __builtin_amdgcn_readfirstlane(kr);
          const uint32_t k = k0 + kr;
          if constexpr (BLD == B_IM1X1) {
            sb1[j] = ld1(rsb, oob_unless(k < p.K, (uint32_t)(col_base + (int)(k * p.HW)) * 4u) | col_oob);
          } else {
            // k = (ic * KY + ky) * KX + kx
            const uint32_t ic = fdiv(k, p.kyx_m, p.kyx_s);
            const uint32_t rem = k - ic * p.KYX;
            const uint32_t ky = fdiv(rem, p.kx_m, p.kx_s);
            const uint32_t kx = rem - ky * p.KX;
            const int iy = iy0 + (int)ky, ix = ix0 + (int)kx;
            const bool ok = (k < p.K) & ((uint32_t)iy < p.H) & ((uint32_t)ix < p.W);
            const int off = col_base + (int)(ic * p.HW + ky * p.W + kx);
            sb1[j] = ld1(rsb, oob_unless(ok, (uint32_t)off * 4u) | col_oob);
          }
        }
      }
    }
  };

  auto store_tiles = [&](int buf) {
    float *const Ab = As + buf * A_LDS;
    float *const Bb = Bs + buf * B_LDS;
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
          const int kc = idx % (BK / 4), mr = idx / (BK / 4);
          *(f32x4v *)&Ab[mr * AST + 4 * kc] = sa4[j];
        } else {
          const int kr = idx % BK, mr = idx / BK;
          Ab[mr * AST + kr] = sa1[j];
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

  const int kh = lane >> 5, li = lane & 31;
  auto compute = [&](int buf) {
    const float *const Ab = As + buf * A_LDS;
    const float *const Bb = Bs + buf * B_LDS + wn * WN + TN * li;
#pragma unroll
    for (int kq = 0; kq < BK / 8; ++kq) {
      f32x4v am[AMM ? TM : 1];
      if constexpr (AMM) {
#pragma unroll
        for (int t = 0; t < TM; ++t)
          am[t] = *(const f32x4v *)&Ab[(wm * WM + TM * li + t) * AST + kh * (BK / 2) + 4 * kq];
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int krow = kh * (BK / 2) + 4 * kq + q;
        float a[TM], b[TN];
        if constexpr (AMM) {
#pragma unroll
          for (int t = 0; t < TM; ++t) a[t] = am[t][q];
        } else {
          typename fvec<TM>::t av = *(const typename fvec<TM>::t *)&Ab[krow * BM + wm * WM + TM * li];
#pragma unroll
          for (int t = 0; t < TM; ++t) a[t] = vget<TM>(av, t);
        }
        typename fvec<TN>::t bv = *(const typename fvec<TN>::t *)&Bb[krow * BN];
#pragma unroll
        for (int j = 0; j < TN; ++j) b[j] = vget<TN>(bv, j);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i], b[j], acc[i][j], 0, 0, 0);
      }
    }
  };

  // ---- main loop: register-staged, double-buffered LDS, one barrier per K tile
  const uint32_t nkt = (kend - kbeg + BK - 1) / BK;
  if constexpr (IM && SPL != 1) {  // rows >= M and a null bias read 0 through the range check
    const __amdgpu_buffer_rsrc_t rsbias = make_rsrc(p.bias, p.bias ? p.M * 4u : 0u);
    for (int i = tid; i < BM; i += NT) Lbias[i] = ld1(rsbias, bm0 + i < p.M ? (bm0 + i) * 4u : OOB);
  }
  load_tiles(kbeg);
  store_tiles(0);
  __syncthreads();
  KT(1);
  int buf = 0;
  for (uint32_t kt = 0; kt < nkt; ++kt) {
    const bool more = kt + 1 < nkt;
    if (more) load_tiles(kbeg + (kt + 1) * BK);
    compute(buf);
    if (more) store_tiles(buf ^ 1);
    __syncthreads();
    buf ^= 1;
  }

  KT(2);
  // ---- epilogue
  const uint32_t n_base = bn0 + wn * WN + TN * li;
  if constexpr (SPLIT) {
    // raw partial sums -> this split's slab of this tile (tile-major, row-major BM x BN)
    const uint32_t tile = tile_m * p.tiles_n + tile_n;
    const size_t slab_off = ((size_t)split * p.tiles_m * p.tiles_n + tile) * (BM * BN);
    float *const wz = p.ws + slab_off;
    const __amdgpu_buffer_rsrc_t rw = make_rsrc(wz, BM * BN * 4);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = wm * WM + TM * ((r & 3) + 8 * (r >> 2) + 4 * kh) + i;
        const uint32_t off = row * BN + wn * WN + TN * li;
        typename fvec<TN>::t w;
        if constexpr (TN == 1) w = acc[i][0][r]; else {
#pragma unroll
          for (int j = 0; j < TN; ++j) w[j] = acc[i][j][r];
        }
        if constexpr (SPL == 1) {
          *(typename fvec<TN>::t *)&wz[off] = w;
        } else if constexpr (TN == 1) {  // write-through (sc1): handed off inside this launch
          __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, w), rw, off * 4, 0, AUX_SC1);
        } else if constexpr (TN == 2) {
          __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(__attribute__((ext_vector_type(2))) uint32_t, w),
                                                rw, off * 4, 0, AUX_SC1);
        } else {
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) uint32_t, w),
                                                 rw, off * 4, 0, AUX_SC1);
        }
      }
    if constexpr (SPL == 1) return;  // bias / ReLU / NCHW scatter happen in splitk_reduce_kernel
    // Publish the slab and count arrivals (cdna_hip_programming.md §5 split-K recipe, the
    // write-through form): sc1 slab stores, every storing wave drains them, barrier, one
    // lane takes a relaxed agent-scope ticket. The block drawing S-1 combines all S slabs
    // reading every one of them with sc1 loads -- no release / acquire fences needed.
    uint32_t *const flag = (uint32_t *)smem;  // the A/B tiles are dead after the loop's last barrier
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      const uint32_t old = __hip_atomic_fetch_add(&p.cnt[tile], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const uint32_t last = old == gridDim.y - 1 ? 1u : 0u;
      if (last) __hip_atomic_store(&p.cnt[tile], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // ready for the next call
      *flag = last;
    }
    __syncthreads();
    KT(3);
    if (!*flag) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // compiler-only: keep the loads below the ticket
    combine_tile<IM ? 1 : 0, NT, BM * BN / 4 / NT, (BM * BN / 4 / NT < 4 ? BM * BN / 4 / NT : 4)>(
        p, tile, tile_m, tile_n, gridDim.y, IM ? Lbias : nullptr, tid);
#ifdef BH_KTRACE
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    KT(4);
#endif
    return;
  }
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
#pragma unroll
  for (int i = 0; i < TM; ++i) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = (r & 3) + 8 * (r >> 2) + 4 * kh;
      const uint32_t m = bm0 + wm * WM + TM * row + i;
      if (m >= p.M) continue;
      float v[TN];
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        float x = acc[i][j][r];
        if constexpr (IM) {
          x += Lbias[wm * WM + TM * row + i];
          if (p.res && cofs[j] >= 0) x += p.res[(size_t)m * p.OHW + cofs[j]];  // residual (Eltwise SUM)
        }
        v[j] = (p.relu && x < 0.0f) ? 0.0f : x;
      }
      if constexpr (IM) {
        float *const crow = p.c + (size_t)m * p.OHW;
#pragma unroll
        for (int j = 0; j < TN; ++j)
          if (cofs[j] >= 0) crow[cofs[j]] = v[j];
      } else {
        float *const crow = p.c + (size_t)m * p.ldc + n_base;
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
#ifdef BH_KTRACE
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  KT(4);
#endif
}

// ---------------------------------------------------------------------------
// Latency kernel for small ops (few output tiles, short K): the regime where a
// call is a chain of memory round trips (~1 us each on a busy MI355X) rather
// than MFMA work.
//  * One block of 4 waves owns a small BM x BN tile and the waves split every
//    64-deep K tile four ways (wave w takes k rows 16w..16w+15), so all four SIMDs
//    work on one small tile and there are 4x more tiles than with one wave per
//    32x32 subtile; the four partial tiles are summed through LDS at the end.
//  * Operands go global -> LDS by LDS-DMA (buffer_load ... lds, per-lane source
//    offsets, out-of-range lanes read as 0) into a ring of D stages with D-1 tiles
//    in flight; one counted vmcnt + raw s_barrier per K tile (cdna_hip_programming.md
//    §5 "Pipelining across barriers"), so a K step costs max(MFMA, latency / (D-1)).
//  * 16-byte DMA wherever the layout allows (a dword DMA instruction costs about as
//    much CU time as a 16-byte one): the m-major weight tile lands as [BM][64] with
//    16-B chunk c of row m stored at c ^ (m & 15) (swizzled through the per-lane
//    source address), so the b128 A-fragment reads of 16 consecutive rows hit
//    distinct banks; 1x1 convs with OH*OW % 4 == 0 stream 4 pixels per lane.
// Same GemmArgs contract, slab layout and split-K modes as gemm_kernel.
// ---------------------------------------------------------------------------
template <int BM, int BN, int NW, int D, int ALD, int BLD, int SPL>
__global__ __launch_bounds__(NW * 64) void gemm_sk_kernel(GemmArgs p) {
  constexpr int NT = NW * 64, BK = 64, KW = BK / NW;  // KW: k rows per wave per stage
  static_assert(NW == 4 || NW == 8, "4 or 8 waves");
  constexpr int TM = BM / 32, TN = BN / 32;
  static_assert(BM % 32 == 0 && BN % 32 == 0 && D >= 2, "sk tile shape");
  constexpr bool IM = (BLD == B_IM2COL || BLD == B_IM1X1 || BLD == B_IM1X1V);
  constexpr bool AMM = (ALD == A_MVEC || ALD == A_MSCALAR);
  // m-major A: 16-B DMA into swizzled [BM][64] (A_MVEC) or dword DMA into rows padded
  // to 68 floats (A_MSCALAR: K % 4 != 0 or unaligned weights; one instruction per row)
  constexpr int AST = ALD == A_MSCALAR ? BK + APAD : BK;
  constexpr int A_LDS = AMM ? BM * AST : BK * BM;
  constexpr int B_LDS = BK * BN;
  constexpr int SLOT = A_LDS + B_LDS;
  constexpr bool AV16 = (ALD == A_KVEC || ALD == A_MVEC);
  constexpr bool BV16 = (BLD == B_KVEC || BLD == B_IM1X1V);
  // LDS-DMA wave instructions per wave per stage (64 lanes x 16 or 4 bytes each)
  constexpr int LA = AV16 ? BK * BM / (NW * 256) : BK * BM / (NW * 64);
  constexpr int LB = BV16 ? BK * BN / (NW * 256) : BK * BN / (NW * 64);
  static_assert(BK * BM % (NW * (AV16 ? 256 : 64)) == 0 && BK * BN % (NW * (BV16 ? 256 : 64)) == 0,
                "whole DMA instructions per wave");
  constexpr int LW = LA + LB;
  static_assert(LA >= 1 && LB >= 1 && (D - 2) * LW <= 63, "vmcnt range");
  constexpr int RED = NW * BM * BN;  // per-wave partial tiles, aliasing the ring after the loop
  constexpr int SMF = D * SLOT > RED ? D * SLOT : RED;
  constexpr int NCH = BM * BN / 4;           // float4 output chunks of the tile
  constexpr int CH = (NCH + NT - 1) / NT;    // per thread
  static_assert(NCH % NT == 0 || CH == 1, "sk epilogue chunking");
  static_assert(BM <= 64, "bias arrives by one 64-lane DMA");

  // one __shared__ array only (a second object makes hipcc wait vmcnt(0) at ds_reads)
  __shared__ __attribute__((aligned(16))) float smem[SMF + 64 + 4];
  float *const Lbias = smem + SMF;
  uint32_t *const flag = (uint32_t *)(smem + SMF + 64);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  KT(0);
  uint32_t tile_m, tile_n;
  map_tile(blockIdx.x, p.tiles_m, p.tiles_n, tile_m, tile_n);
  const uint32_t bm0 = tile_m * BM, bn0 = tile_n * BN;
  constexpr bool SPLIT = SPL != 0;
  const uint32_t split = SPLIT ? blockIdx.y : 0;
  const uint32_t kbeg = split * p.ks;
  const uint32_t kend = SPLIT ? min(p.K, kbeg + p.ks) : p.K;

  const __amdgpu_buffer_rsrc_t rsa = make_rsrc(p.a, p.a_bytes);
  const __amdgpu_buffer_rsrc_t rsb = make_rsrc(p.b, p.b_bytes);

  // B DMA: this lane's column is fixed (64 % BN == 0); its k row within a stage is
  // rb0 + j * (64 / BN) * NW... computed per instruction below
  int col_base = 0, iy0 = 0, ix0 = 0;
  uint32_t col_oob = 0;
  if constexpr (IM) {
    // this lane's (first) column is fixed: 64 % BN == 0 (dword), 64 % (BN / 4) == 0 (16 B)
    const uint32_t col = bn0 + (uint32_t)(BLD == B_IM1X1V ? 4 * (lane % (BN / 4)) : lane % BN);
    col_oob = col < p.N ? 0u : OOB;
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

  constexpr int RPI = BV16 ? 256 / BN : 64 / BN;  // B rows per DMA instruction
  const uint32_t lr = (uint32_t)(BV16 ? lane / (BN / 4) : lane / BN);  // this lane's row in it
  auto issue_stage = [&](int slot, uint32_t k0) {
    float *const Ab = smem + slot * SLOT;
    float *const Bb = Ab + A_LDS;
#pragma unroll
    for (int j = 0; j < LA; ++j) {
      const int ins = wave * LA + j;
      if constexpr (ALD == A_MVEC) {
        // 4 rows x 16 chunks per instruction; LDS chunk c of row m holds k chunk c ^ (m & 15)
        const int r = 4 * ins + (lane >> 4), c = lane & 15;
        const uint32_t m = bm0 + r, k = k0 + 4 * (c ^ (r & 15));
        dma16(rsa, Ab + ins * 256, oob_unless((m < p.M) & (k < kend), (m * p.lda + k) * 4u));
      } else if constexpr (ALD == A_MSCALAR) {
        const uint32_t m = bm0 + ins, k = k0 + lane;
        dma4(rsa, Ab + ins * AST, oob_unless((m < p.M) & (k < kend), (m * p.lda + k) * 4u));
      } else {
        constexpr int W = (ALD == A_KVEC) ? 4 : 1;
        const int e = ins * 64 * W + W * lane;  // element index in [BK][BM]
        const uint32_t m = bm0 + e % BM, k = k0 + e / BM;
        const uint32_t off = oob_unless((m < p.M) & (k < kend), (k * p.lda + m) * 4u);
        if constexpr (ALD == A_KVEC) dma16(rsa, Ab + ins * 256, off);
        else dma4(rsa, Ab + ins * 64, off);
      }
    }
    if constexpr (BLD == B_KVEC || BLD == B_KSCALAR) {
#pragma unroll
      for (int j = 0; j < LB; ++j) {
        constexpr int W = (BLD == B_KVEC) ? 4 : 1;
        const int e = (wave * LB + j) * 64 * W + W * lane;  // element index in [BK][BN]
        const uint32_t n = bn0 + e % BN, k = k0 + e / BN;
        const uint32_t off = oob_unless((n < p.N) & (k < kend), (k * p.ldb + n) * 4u);
        if constexpr (BLD == B_KVEC) dma16(rsb, Bb + (wave * LB + j) * 256, off);
        else dma4(rsb, Bb + (wave * LB + j) * 64, off);
      }
    } else if constexpr (BLD == B_IM1X1 || BLD == B_IM1X1V) {
      // k = k0 + RPI*i + lr with i = wave*LB + j: offset linear in i
      const uint32_t vb = (uint32_t)(col_base + (int)((k0 + lr + RPI * wave * LB) * p.HW)) * 4u;
      const int kl = (int)kend - (int)(k0 + lr + RPI * wave * LB);
#pragma unroll
      for (int j = 0; j < LB; ++j) {
        const uint32_t off = oob_unless(RPI * j < kl, vb + RPI * j * p.HW * 4u) | col_oob;
        if constexpr (BLD == B_IM1X1V) dma16(rsb, Bb + (wave * LB + j) * 256, off);
        else dma4(rsb, Bb + (wave * LB + j) * 64, off);
      }
    } else {
#pragma unroll
      for (int j = 0; j < LB; ++j) {
        // (ic, ky, kx) of the instruction's first row (wave-uniform, scalar), then this lane's row
        const uint32_t k1 = k0 + RPI * (wave * LB + j);
        uint32_t ic = fdiv(k1, p.kyx_m, p.kyx_s);
        const uint32_t rem = k1 - ic * p.KYX;
        uint32_t ky = fdiv(rem, p.kx_m, p.kx_s);
        uint32_t kx = rem - ky * p.KX;
        if constexpr (RPI > 1) {
          kx += lr;  // lr < RPI <= 2 and KX >= 1: at most one carry per level
          if (kx >= p.KX) { kx -= p.KX; ++ky; }
          if (ky * p.KX >= p.KYX) { ky = 0; ++ic; }  // ky == KY
        }
        const uint32_t k = k1 + lr;
        const int iy = iy0 + (int)ky, ix = ix0 + (int)kx;
        const bool ok = (k < kend) & ((uint32_t)iy < p.H) & ((uint32_t)ix < p.W);
        dma4(rsb, Bb + (wave * LB + j) * 64,
             oob_unless(ok, (uint32_t)(col_base + (int)(ic * p.HW + ky * p.W + kx)) * 4u) | col_oob);
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

  const int kh = lane >> 5, li = lane & 31;
  // wave w owns k rows KW*w .. KW*w+KW-1 of a stage; lane half h the KW/2 rows from
  // KW*w + h*KW/2 (the same k for A and B)
  auto compute = [&](int slot) {
    const float *const Ab = smem + slot * SLOT;
    const float *const Bb = Ab + A_LDS + TN * li;
#pragma unroll
    for (int kq = 0; kq < KW / 8; ++kq) {
      const int cc = (KW * wave + kh * (KW / 2)) / 4 + kq;  // 16-B k chunk of the A rows
      f32x4v am[AMM ? TM : 1];
      if constexpr (AMM) {
#pragma unroll
        for (int t = 0; t < TM; ++t) {
          const int m = TM * li + t;
          am[t] = *(const f32x4v *)&Ab[ALD == A_MVEC ? m * AST + 4 * (cc ^ (m & 15)) : m * AST + 4 * cc];
        }
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int krow = 4 * cc + q;
        float a[TM], b[TN];
        if constexpr (AMM) {
#pragma unroll
          for (int t = 0; t < TM; ++t) a[t] = am[t][q];
        } else {
          typename fvec<TM>::t av = *(const typename fvec<TM>::t *)&Ab[krow * BM + TM * li];
#pragma unroll
          for (int t = 0; t < TM; ++t) a[t] = vget<TM>(av, t);
        }
        typename fvec<TN>::t bv = *(const typename fvec<TN>::t *)&Bb[krow * BN];
#pragma unroll
        for (int j = 0; j < TN; ++j) b[j] = vget<TN>(bv, j);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i], b[j], acc[i][j], 0, 0, 0);
      }
    }
  };

  // ---- main loop: D-stage LDS-DMA ring, D-1 K tiles in flight
  const uint32_t nkt = (kend - kbeg + BK - 1) / BK;
  if constexpr (IM && SPL != 1) {
    // biases by one DMA of wave 0, issued before stage 0 so the first stage wait covers it
    const __amdgpu_buffer_rsrc_t rsbias = make_rsrc(p.bias, p.bias ? p.M * 4u : 0u);
    if (wave == 0) dma4(rsbias, Lbias, oob_unless((lane < BM) & (bm0 + lane < p.M), (bm0 + lane) * 4u));
  }
  // Stages past the split's end are issued too (their lanes read OOB zeros without
  // touching memory), so every wave always has exactly D-2 stages in flight behind
  // the one it waits for and the issue code has no branches (it interleaves with
  // the MFMAs); the ring is drained before the LDS is reused below.
#pragma unroll
  for (int s = 0; s < D - 1; ++s) issue_stage(s, kbeg + s * BK);
  int slot = 0;
  for (uint32_t kt = 0; kt < nkt; ++kt) {
    vm_wait<(D - 2) * LW>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // stage kt landed for all waves; all done reading kt-1
    asm volatile("" ::: "memory");
    if (kt == 0) KT(1);
    issue_stage(slot == 0 ? D - 1 : slot - 1, kbeg + (kt + D - 1) * BK);  // slot (kt-1) % D
    compute(slot);
    slot = slot == D - 1 ? 0 : slot + 1;
  }
  vm_wait<0>();
  KT(2);

  // ---- sum the four waves' partial tiles through LDS (row-major BM x BN per wave)
  __syncthreads();  // every wave is done reading the ring; no DMA is in flight
  {
    float *const Rw = smem + wave * (BM * BN);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = TM * ((r & 3) + 8 * (r >> 2) + 4 * kh) + i;
        typename fvec<TN>::t w;
        if constexpr (TN == 1) w = acc[i][0][r]; else {
#pragma unroll
          for (int j = 0; j < TN; ++j) w[j] = acc[i][j][r];
        }
        *(typename fvec<TN>::t *)&Rw[row * BN + TN * li] = w;
      }
  }
  __syncthreads();
  const bool has_chunk = NCH % NT == 0 || tid < NCH;
  f32x4v v[CH];
#pragma unroll
  for (int j = 0; j < CH; ++j) {
    const int c = has_chunk ? tid + j * NT : 0;
    v[j] = *(const f32x4v *)&smem[4 * c];
#pragma unroll
    for (int w = 1; w < NW; ++w) v[j] += *(const f32x4v *)&smem[w * BM * BN + 4 * c];
  }
  if constexpr (!SPLIT) {
    if (has_chunk) {
#pragma unroll
      for (int j = 0; j < CH; ++j)
        finish_store<IM ? 1 : 0>(p, tile_m, tile_n, tid + j * NT, v[j], IM ? Lbias : nullptr);
    }
#ifdef BH_KTRACE
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    KT(4);
#endif
    return;
  } else {
    const uint32_t tile = tile_m * p.tiles_n + tile_n;
    const size_t slab_off = ((size_t)split * p.tiles_m * p.tiles_n + tile) * (BM * BN);
    float *const wz = p.ws + slab_off;
    if constexpr (SPL == 1) {
      if (has_chunk) {
#pragma unroll
        for (int j = 0; j < CH; ++j) *(f32x4v *)&wz[4 * (tid + j * NT)] = v[j];
      }
      return;
    } else {
      const __amdgpu_buffer_rsrc_t rw = make_rsrc(wz, BM * BN * 4);
      if (has_chunk) {
#pragma unroll
        for (int j = 0; j < CH; ++j)
          __builtin_amdgcn_raw_buffer_store_b128(
              __builtin_bit_cast(__attribute__((ext_vector_type(4))) uint32_t, v[j]), rw, 16 * (tid + j * NT), 0,
              AUX_SC1);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) {
        const uint32_t old = __hip_atomic_fetch_add(&p.cnt[tile], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t last = old == gridDim.y - 1 ? 1u : 0u;
        if (last) __hip_atomic_store(&p.cnt[tile], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        *flag = last;
      }
      __syncthreads();
      KT(3);
      if (!*flag) return;
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // compiler-only: keep the loads below the ticket
      combine_tile<IM ? 1 : 0, NT, CH, CH, NCH>(p, tile, tile_m, tile_n, gridDim.y, IM ? Lbias : nullptr, tid);
#ifdef BH_KTRACE
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      KT(4);
#endif
    }
  }
}

// Split-K combine pass (SPL == 1): one thread per float4 chunk of every tile.
template <int IMODE>
__global__ __launch_bounds__(256) void splitk_reduce_kernel(GemmArgs p, uint32_t S) {
  const uint32_t per_tile = p.tbm * p.tbn / 4, ntiles = p.tiles_m * p.tiles_n;
  const uint64_t total = (uint64_t)per_tile * ntiles;
  for (uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t tile = (uint32_t)(e / per_tile), c = (uint32_t)(e - (uint64_t)tile * per_tile);
    const uint32_t tile_m = tile / p.tiles_n, tile_n = tile - tile_m * p.tiles_n;
    combine_store<IMODE>(p, tile, tile_m, tile_n, c, S, nullptr);
  }
}

// ---------------------------------------------------------------------------
// host side: tile-configuration table, split-K planning, tuning table, dispatch
// ---------------------------------------------------------------------------


template <int BM, int BN, int BK, int TM, int TN, int WM_, int WN_, int ALD, int BLD>
void reg_kernels(cfg_t &c) {
  c.k[ALD][BLD][0] = gemm_kernel<BM, BN, BK, TM, TN, WM_, WN_, ALD, BLD, 0>;
  c.k[ALD][BLD][1] = gemm_kernel<BM, BN, BK, TM, TN, WM_, WN_, ALD, BLD, 1>;
  c.k[ALD][BLD][2] = gemm_kernel<BM, BN, BK, TM, TN, WM_, WN_, ALD, BLD, 2>;
}
template <int BM, int BN, int NW, int D, int ALD, int BLD>
void reg_sk_kernels(cfg_t &c) {
  c.k[ALD][BLD][0] = gemm_sk_kernel<BM, BN, NW, D, ALD, BLD, 0>;
  c.k[ALD][BLD][1] = gemm_sk_kernel<BM, BN, NW, D, ALD, BLD, 1>;
  c.k[ALD][BLD][2] = gemm_sk_kernel<BM, BN, NW, D, ALD, BLD, 2>;
}
template <int BM, int BN, int NW, int D>
cfg_t conv_sk_cfg(const char *name) {
  cfg_t c{name, BM, BN, 64, NW * 64, {}};
  reg_sk_kernels<BM, BN, NW, D, A_MVEC, B_IM2COL>(c);
  reg_sk_kernels<BM, BN, NW, D, A_MSCALAR, B_IM2COL>(c);
  reg_sk_kernels<BM, BN, NW, D, A_MVEC, B_IM1X1>(c);
  reg_sk_kernels<BM, BN, NW, D, A_MSCALAR, B_IM1X1>(c);
  reg_sk_kernels<BM, BN, NW, D, A_MVEC, B_IM1X1V>(c);
  reg_sk_kernels<BM, BN, NW, D, A_MSCALAR, B_IM1X1V>(c);
  return c;
}
template <int BM, int BN, int NW, int D>
cfg_t sgemm_sk_cfg(const char *name) {
  cfg_t c{name, BM, BN, 64, NW * 64, {}};
  reg_sk_kernels<BM, BN, NW, D, A_KVEC, B_KVEC>(c);
  reg_sk_kernels<BM, BN, NW, D, A_KSCALAR, B_KSCALAR>(c);
  return c;
}
template <int BM, int BN, int BK, int TM, int TN, int WM_, int WN_>
cfg_t conv_cfg(const char *name) {
  cfg_t c{name, BM, BN, BK, WM_ * WN_ * 64, {}};
  reg_kernels<BM, BN, BK, TM, TN, WM_, WN_, A_MVEC, B_IM2COL>(c);
  reg_kernels<BM, BN, BK, TM, TN, WM_, WN_, A_MSCALAR, B_IM2COL>(c);
  reg_kernels<BM, BN, BK, TM, TN, WM_, WN_, A_MVEC, B_IM1X1>(c);
  reg_kernels<BM, BN, BK, TM, TN, WM_, WN_, A_MSCALAR, B_IM1X1>(c);
  return c;
}
template <int BM, int BN, int BK, int TM, int TN, int WM_, int WN_>
cfg_t sgemm_cfg(const char *name) {
  cfg_t c{name, BM, BN, BK, WM_ * WN_ * 64, {}};
  reg_kernels<BM, BN, BK, TM, TN, WM_, WN_, A_KVEC, B_KVEC>(c);
  reg_kernels<BM, BN, BK, TM, TN, WM_, WN_, A_KSCALAR, B_KSCALAR>(c);
  return c;
}

// Tile configurations (BM x BN x BK; 32x32 MFMA tiles per wave TM x TN; waves M x N).
std::vector<cfg_t> with_ring(int op, std::vector<cfg_t> v) {
  for (auto const &c : ring_cfgs(op)) v.push_back(c);
  for (auto const &c : ref64_cfgs()) v.push_back(c);
  if (op == 1) {
    for (auto const &c : gv_cfgs()) v.push_back(c);
    for (auto const &c : dc_cfgs()) v.push_back(c);
    for (auto const &c : dcm_cfgs()) v.push_back(c);
    for (auto const &c : k1s_cfgs()) v.push_back(c);
    for (auto const &c : wg_cfgs()) v.push_back(c);
    for (auto const &c : wgx_cfgs()) v.push_back(c);
  }
  return v;
}

const std::vector<cfg_t> &cfgs(int op) {
  static const std::vector<cfg_t> sg = with_ring(0, {
      sgemm_cfg<128, 128, 16, 2, 2, 2, 2>("128x128x16"),
      sgemm_cfg<128, 128, 32, 2, 2, 2, 2>("128x128x32"),
      sgemm_cfg<256, 128, 16, 4, 2, 2, 2>("256x128x16"),
      sgemm_cfg<128, 64, 16, 2, 1, 2, 2>("128x64x16"),
      sgemm_cfg<64, 64, 16, 1, 1, 2, 2>("64x64x16"),
      sgemm_sk_cfg<32, 32, 4, 4>("sk32x32x64"),
      sgemm_sk_cfg<64, 64, 4, 3>("sk64x64x64"),
      sgemm_sk_cfg<32, 32, 8, 4>("sk32x32x64w8"),
      sgemm_sk_cfg<64, 64, 8, 4>("sk64x64x64w8"),
  });
  static const std::vector<cfg_t> cv = with_ring(1, {
      conv_cfg<128, 128, 32, 2, 2, 2, 2>("128x128x32"),
      conv_cfg<128, 128, 16, 2, 2, 2, 2>("128x128x16"),
      conv_cfg<64, 128, 32, 1, 2, 2, 2>("64x128x32"),
      conv_cfg<32, 256, 32, 1, 2, 1, 4>("32x256x32"),
      conv_cfg<64, 64, 32, 1, 1, 2, 2>("64x64x32"),
      conv_cfg<128, 64, 32, 2, 1, 2, 2>("128x64x32"),
      conv_cfg<128, 32, 32, 1, 1, 4, 1>("128x32x32"),
      conv_cfg<256, 128, 16, 4, 2, 2, 2>("256x128x16"),
      conv_cfg<64, 32, 32, 1, 1, 2, 1>("64x32x32"),
      conv_sk_cfg<32, 32, 4, 4>("sk32x32x64"),
      conv_sk_cfg<32, 64, 4, 4>("sk32x64x64"),
      conv_sk_cfg<64, 32, 4, 4>("sk64x32x64"),
      conv_sk_cfg<64, 64, 4, 3>("sk64x64x64"),
      conv_sk_cfg<32, 32, 8, 4>("sk32x32x64w8"),
      conv_sk_cfg<32, 64, 8, 4>("sk32x64x64w8"),
      conv_sk_cfg<64, 64, 8, 4>("sk64x64x64w8"),
  });
  return op == 0 ? sg : cv;
}

int cfg_index(int op, std::string const &name) {
  auto const &v = cfgs(op);
  for (size_t i = 0; i < v.size(); ++i)
    if (name == v[i].name) return (int)i;
  return -1;
}

bool fits_buffer(uint64_t bytes) { return bytes < (uint64_t)OOB - 64; }

void set_fd(uint32_t d, uint32_t &m, uint32_t &s) {
  bh::fastdiv f = bh::make_fastdiv(d ? d : 1);
  m = f.m;
  s = f.s;
}

}  // namespace

namespace bhk {
int ensure_ws(bh_ctx *ctx, size_t bytes) {
  return bh::grow_buffer(ctx, ctx->ws, ctx->ws_bytes, bytes, false, "split-K workspace");
}

// split-K arrival tickets: zeroed at allocation, reset by each tile's last arriver
int ensure_cnt(bh_ctx *ctx, uint64_t n) {
  size_t have = ctx->cnt_n * 4;
  int rc = bh::grow_buffer(ctx, ctx->cnt, have, std::max<uint64_t>(n, 4096) * 4, true, "split-K tickets");
  ctx->cnt_n = have / 4;
  return rc;
}
}  // namespace bhk

namespace {

// Number of K splits: enough blocks to cover the CUs twice, at least MIN_KT K tiles per split.
uint32_t plan_splits(uint32_t tiles, uint32_t K, int BK, uint32_t ncu) {
  const uint32_t MIN_KT = 4;
  const uint32_t nkt = (K + BK - 1) / BK;
  if (tiles >= ncu || nkt < 2 * MIN_KT) return 1;
  uint32_t s = (2 * ncu + tiles - 1) / tiles;
  s = std::min(s, nkt / MIN_KT);
  s = std::min(s, 64u);
  return std::max(s, 1u);
}

// ---- tuning table ("wisdom" for this backend): exact-shape -> (config, splits)
struct choice_t {
  int cfg = -1;
  uint32_t splits = 0;  // 0 = plan
  int red = 0;          // split-K combine: 0 = plan, 1 = reduce kernel, 2 = in-kernel last arriver
  int wt = 0;           // output stores write through (GemmArgs::wt)
};
std::map<std::string, choice_t> g_tune;
std::once_flag g_tune_once;

std::string shape_key(int op, const uint32_t *d) {
  std::string k = op == 0 ? "sgemm" : "conv";
  int n = op == 0 ? 3 : 11;
  for (int i = 0; i < n; ++i) k += " " + std::to_string(d[i]);
  return k;
}

void load_tuning() {
  std::string path;
  if (const char *e = getenv("BH_TUNE_FILE")) path = e;
  else {
    Dl_info info;
    if (dladdr((void *)&load_tuning, &info) && info.dli_fname) {
      std::string so = info.dli_fname;
      size_t sl = so.rfind('/');
      path = (sl == std::string::npos ? std::string(".") : so.substr(0, sl)) + "/../tuning/gfx950.tune";
    }
  }
  FILE *f = path.empty() ? nullptr : fopen(path.c_str(), "r");
  if (!f) return;
  char line[512];
  while (fgets(line, sizeof(line), f)) {
    // "<op> d0 d1 ... cfg=<name> splits=<n>"
    std::string l(line);
    if (l.empty() || l[0] == '#') continue;
    size_t c = l.find(" cfg="), s = l.find(" splits=");
    if (c == std::string::npos || s == std::string::npos) continue;
    std::string key = l.substr(0, c);
    std::string name = l.substr(c + 5, s - c - 5);
    int op = key.rfind("sgemm", 0) == 0 ? 0 : 1;
    choice_t ch;
    ch.cfg = cfg_index(op, name);
    ch.splits = (uint32_t)strtoul(l.c_str() + s + 8, nullptr, 10);
    size_t r = l.find(" red=");
    if (r != std::string::npos) ch.red = l[r + 5] == 'k' ? 1 : 2;
    size_t w = l.find(" wt=");
    if (w != std::string::npos) ch.wt = l[w + 4] == '1' ? 1 : 0;
    if (ch.cfg >= 0) g_tune[key] = ch;
  }
  fclose(f);
}

// Kernel choice for shapes the tuning table lacks. ring = false: no ring (LDS-DMA, packed
// bank) config -- launch_conv's fallback when the bank or input is too large for it.
choice_t heuristic(int op, const uint32_t *d, bool ring = true, bool direct = true) {
  choice_t ch;
  if (op == 0) {
    // big SGEMMs: the LDS-DMA ring with 128 x 128 tiles, whole K per block (tuned on
    // sgemm-ops-full: 93-95 % of the fp32 peak from 4096^3 up); others: the tile kernel
    const uint64_t tiles = (uint64_t)((d[0] + 127) / 128) * ((d[1] + 127) / 128);
    ch.cfg = (ring && tiles >= 256 && d[2] >= 512) ? cfg_index(0, "r128x128x32d2") : 0;
    ch.splits = ch.cfg > 0 ? 1 : 0;
    return ch;
  }
  uint32_t B = d[0], H = d[2], W = d[3], OC = d[4], KY = d[5], KX = d[6], sy = d[7], sx = d[8], py = d[9], px = d[10];
  uint64_t N = (uint64_t)B * ((H + 2 * py - KY) / sy + 1) * ((W + 2 * px - KX) / sx + 1);
  uint32_t K = d[1] * KY * KX;
  // big grids: 128x128 tiles; grids that cannot fill the GPU: narrow tiles plus
  // split-K combined by the reduce kernel (the tuning table refines both)
  const char *n = "128x128x32";
  uint64_t tiles128 = ((OC + 127) / 128) * ((N + 127) / 128);
  if (N <= 64 && (uint64_t)OC * K >= (1u << 20) && K % 4 == 0) n = N <= 16 ? "gv64x16" : (N <= 32 ? "gv64x32" : "gv32x64");
  else if (N <= 32) n = "128x32x32";
  else if (OC <= 32) n = "32x256x32";
  // big convs: the ring kernels, as the tuner picks them for the nets' shapes (VGG-19 / ResNet-50
  // at b20, profiles/r01/nets/tune_nets_b20.log: 128x128 ring on big grids, 64-row rings below)
  else if (ring && K >= 256 && N >= 1024) n = tiles128 >= 256 ? "r128x128x32d2" : (OC <= 64 ? "r64x128x32d3" : "r64x64x32d3");
  else if (OC <= 64) n = "64x128x32";
  else if (tiles128 < 256 && K >= 256) n = "128x32x32";
  ch.cfg = cfg_index(1, n);
  ch.red = 1;
  return ch;
}

choice_t choose(bh_ctx *ctx, int op, const uint32_t *d) {
  choice_t ch;
  if (ctx && ctx->ovr_cfg[op] >= 0) {
    ch.cfg = ctx->ovr_cfg[op];
    ch.splits = ctx->ovr_splits[op];
    ch.red = ctx->ovr_red[op];
  } else {
    std::call_once(g_tune_once, load_tuning);
    auto it = g_tune.find(shape_key(op, d));
    ch = it != g_tune.end() ? it->second : heuristic(op, d);
  }
  if (ctx && ctx->ovr_wt[op] >= 0) ch.wt = ctx->ovr_wt[op];  // policy override (tuner)
  return ch;
}

uint32_t resolve_splits(cfg_t const &c, choice_t const &ch, uint32_t M, uint32_t N, uint32_t K, uint32_t ncu) {
  uint32_t tiles = ((M + c.BM - 1) / c.BM) * ((N + c.BN - 1) / c.BN);
  uint32_t nkt = (K + c.BK - 1) / c.BK;
  uint32_t S = ch.splits ? ch.splits : plan_splits(tiles, K, c.BK, ncu);
  S = std::max(1u, std::min(S, nkt));
  uint32_t ks = ((nkt + S - 1) / S) * c.BK;
  return (K + ks - 1) / ks;  // splits actually used (none empty)
}

int launch_gemm(bh_ctx *ctx, int op, choice_t const &ch, int ald, int bld, GemmArgs &p, const char *what,
                bool first = true) {
  cfg_t const &c = cfgs(op)[ch.cfg];
  p.tiles_m = (p.M + c.BM - 1) / c.BM;
  p.tiles_n = (p.N + c.BN - 1) / c.BN;
#ifdef BH_KTRACE
  p.trace = (unsigned long long *)ctx->stamps + 65536;
#endif
  const uint64_t nblk = (uint64_t)p.tiles_m * p.tiles_n;
  if (nblk > 0x7fffffffu) return bh::fail(BH_UNSUP, std::string(what) + ": grid too large");
  const uint32_t ncu = ctx->prop.multiProcessorCount > 0 ? ctx->prop.multiProcessorCount : 256;
  p.tbm = c.BM;
  p.tbn = c.BN;
  if (bld == B_IMTAB && !c.k[ald][bld][0]) bld = B_IM2COL;  // table / one-tap loaders: ring kernels only
  if (bld == B_IMTAP && !c.k[ald][bld][0]) bld = B_IMT2;
  if (bld == B_IM1X1S && !c.k[ald][bld][0]) bld = B_IM1X1;
  if (c.gv) {
    // filter-streaming kernel (bh_gv.hip): one block per (64-row tile, K chunk); the K chunks
    // of a tile are combined by its last arriver. ch.splits = K chunks (0: ~1024 blocks)
    kern_t k = c.k[ald][bld][0];
    if (!k) return bh::fail(BH_ERR, std::string(what) + ": gv loader not instantiated");
    const uint32_t gran = (uint32_t)c.BK;  // K chunks: multiples of 16 per wave
    const uint32_t ktg = (p.K + gran - 1) / gran;
    uint32_t S = ch.splits ? ch.splits : (uint32_t)std::max<uint64_t>(1, (1024 + nblk - 1) / nblk);
    S = std::max(1u, std::min(S, ktg));
    p.ks = ((ktg + S - 1) / S) * gran;
    S = (p.K + p.ks - 1) / p.ks;
    void *args[] = {&p};
    if (S > 1) {
      int rc = ensure_ws(ctx, (size_t)S * nblk * c.BM * c.BN * 4);
      if (rc == BH_OK) rc = ensure_cnt(ctx, nblk);
      if (rc != BH_OK) return rc;
      p.ws = (float *)ctx->ws;
      p.cnt = (uint32_t *)ctx->cnt;
    }
    return bh::launch(ctx, (const void *)k, dim3((uint32_t)nblk, S, 1), dim3(c.NT), args, first, true, what);
  }
  if (c.streamk) {
    // persistent stream-K grid (srk_kernel): ncu x blocks-per-CU blocks share the op's
    // (tile, K tile) iterations equally; ch.splits overrides blocks per CU
    kern_t k = c.k[ald][bld][0];
    if (!k) return bh::fail(BH_ERR, std::string(what) + ": loader combination not instantiated");
    const uint32_t ipt = (p.K + c.BK - 1) / c.BK;
    const uint64_t total = nblk * ipt;
    if (total >= (1ull << 31)) return bh::fail(BH_UNSUP, std::string(what) + ": too many K iterations");
    // splits 1..4: blocks per CU, iterations dealt equally (tiles cut between blocks);
    // 5..8: blocks per CU 1..4, whole tiles per block (a persistent data-parallel grid whose
    // DMA ring runs on across tiles: short-K ops, where cut tiles cost more than balance)
    const bool whole = ch.splits > 4;
    uint32_t bpc = ch.splits ? std::min<uint32_t>(whole ? ch.splits - 4 : ch.splits, 4)
                             : std::max(1, std::min(2, 163840 / c.lds_bytes));
    uint64_t G = (uint64_t)ncu * bpc;
    uint32_t ipb = (uint32_t)((total + G - 1) / G);
    if (whole) ipb = (uint32_t)((nblk + G - 1) / G) * ipt;
    G = (total + ipb - 1) / ipb;
    p.ipt = ipt;
    p.ipb = ipb;
    p.total_it = (uint32_t)total;
    set_fd(ipt, p.ipt_m, p.ipt_s);
    set_fd(p.tiles_m, p.tm_m, p.tm_s);
    int rc = ensure_ws(ctx, (size_t)2 * G * c.BM * c.BN * 4);
    if (rc == BH_OK) rc = ensure_cnt(ctx, nblk);
    if (rc != BH_OK) return rc;
    p.ws = (float *)ctx->ws;
    p.cnt = (uint32_t *)ctx->cnt;
    void *args[] = {&p};
    return bh::launch(ctx, (const void *)k, dim3((uint32_t)G, 1, 1), dim3(c.NT), args, first, true, what);
  }
  const uint32_t S = resolve_splits(c, ch, p.M, p.N, p.K, ncu);
  const uint32_t nkt = (p.K + c.BK - 1) / c.BK;
  p.ks = ((nkt + S - 1) / S) * c.BK;
  // in-kernel combine unless asked otherwise or the tile grid is large (then a separate,
  // fully parallel reduce pass is cheaper than serial combining by last arrivers)
  int red = S <= 1 ? 0 : (ch.red ? ch.red : (nblk >= 64 || S > 4 ? 1 : 2));
  if (red == 2 && (uint64_t)S * nblk * c.BM * c.BN * 4 >= 0x7fffff00ull) red = 1;  // sc1 offsets are 32-bit
  if (bld == B_IM1X1V && !c.k[ald][bld][red]) bld = B_IM1X1;  // tile kernels: no 4-pixel loader
  kern_t k = c.k[ald][bld][red];
  if (!k) return bh::fail(BH_ERR, std::string(what) + ": loader combination not instantiated");
  void *args[] = {&p};
  if (S > 1) {
    int rc = ensure_ws(ctx, (size_t)S * nblk * c.BM * c.BN * 4);
    if (rc != BH_OK) return rc;
    p.ws = (float *)ctx->ws;
    if (red == 2) {
      rc = ensure_cnt(ctx, nblk);
      if (rc != BH_OK) return rc;
      p.cnt = (uint32_t *)ctx->cnt;
      return bh::launch(ctx, (const void *)k, dim3((uint32_t)nblk, S, 1), dim3(c.NT), args, first, true, what);
    }
    rc = bh::launch(ctx, (const void *)k, dim3((uint32_t)nblk, S, 1), dim3(c.NT), args, first, false, what);
    if (rc != BH_OK) return rc;
    const uint64_t total = nblk * c.BM * c.BN / 4;
    const uint32_t grid = (uint32_t)std::min<uint64_t>((total + 255) / 256, 8192);
    const void *rk = (bld == B_IM2COL || bld == B_IMT2 || bld == B_IM1X1 || bld == B_IM1X1V || bld == B_IMTAB ||
                      bld == B_IMTAP || bld == B_IM1X1S)
                         ? (const void *)splitk_reduce_kernel<1>
                                                          : (const void *)splitk_reduce_kernel<0>;
    uint32_t Sv = S;
    void *rargs[] = {&p, &Sv};
    return bh::launch(ctx, rk, dim3(grid), dim3(256), rargs, false, true, "splitk_reduce");
  }
  return bh::launch(ctx, (const void *)k, dim3((uint32_t)nblk, 1, 1), dim3(c.NT), args, first, true, what);
}

void conv_dims(const uint32_t *d, uint32_t &M, uint32_t &N, uint32_t &K) {
  uint32_t B = d[0], IC = d[1], H = d[2], W = d[3], OC = d[4], KY = d[5], KX = d[6], sy = d[7], sx = d[8],
           py = d[9], px = d[10];
  M = OC;
  N = B * ((H + 2 * py - KY) / sy + 1) * ((W + 2 * px - KX) / sx + 1);
  K = IC * KY * KX;
}

std::string describe_cfg(int op, const uint32_t *d, choice_t const &ch);
std::string describe(int op, const uint32_t *d, choice_t const &ch) {
  return describe_cfg(op, d, ch) + (ch.wt ? "_wt" : "");
}
std::string describe_cfg(int op, const uint32_t *d, choice_t const &ch) {
  cfg_t const &c = cfgs(op)[ch.cfg];
  uint32_t M, N, K;
  std::string s;
  if (c.ref64) return std::string(op == 0 ? "ref64_sgemm" : "ref64_conv") + "_double";
  if (op == 0) {
    M = d[0]; N = d[1]; K = d[2];
    s = std::string("mfma32_sgemm_") + c.name + ((M % 4 == 0 && N % 4 == 0) ? "_vec" : "_scalar");
  } else {
    conv_dims(d, M, N, K);
    bool k1 = d[5] == 1 && d[6] == 1 && d[7] == 1 && d[8] == 1 && d[9] == 0 && d[10] == 0;
    s = std::string("mfma32_conv_") + (k1 ? "1x1_" : "im2col_") + c.name + ((K % 4 == 0) ? "_avec" : "_ascalar");
  }
  if (c.streamk) return s + "_streamk";
  if (c.dc == 2) return std::string("mfma32_conv_dm_") + c.name;
  if (c.dc == 3) return std::string("mfma32_conv_k1s_") + c.name;
  if (c.dc == 4 || c.dc == 5) return std::string("mfma32_conv_wino_") + c.name;
  if (c.dc) return std::string("mfma32_conv_direct_") + c.name;
  if (c.fcv) return std::string("conv_fcv_") + c.name;
  if (c.gv) return std::string("mfma16_conv_gv_") + c.name;
  uint32_t S = resolve_splits(c, ch, M, N, K, 256);
  if (S > 1) {
    uint64_t nblk = (uint64_t)((M + c.BM - 1) / c.BM) * ((N + c.BN - 1) / c.BN);
    int red = ch.red ? ch.red : (nblk >= 64 || S > 4 ? 1 : 2);
    if (red == 2 && (uint64_t)S * nblk * c.BM * c.BN * 4 >= 0x7fffff00ull) red = 1;
    s += red == 1 ? "_splitk_reduce" : "_splitk_inkernel";  // one name per kernel instantiation
  }
  return s;
}

}  // namespace

namespace bh {

std::string sgemm_variant(uint32_t M, uint32_t N, uint32_t K) {
  uint32_t d[3] = {M, N, K};
  return describe(0, d, choose(nullptr, 0, d));
}

std::string conv_variant(const uint32_t *d) { return describe(1, d, choose(nullptr, 1, d)); }

uint32_t conv_route_banks(bh_ctx *ctx, const uint32_t *d) {
  choice_t ch = choose(ctx, 1, d);
  return cfgs(1)[ch.cfg].packA ? bhk::route_bank(cfgs(1)[ch.cfg], d[5], d[6]) : 0u;
}

std::string sgemm_variant_ctx(bh_ctx *ctx, uint32_t M, uint32_t N, uint32_t K) {
  uint32_t d[3] = {M, N, K};
  return describe(0, d, choose(ctx, 0, d));
}

std::string conv_variant_ctx(bh_ctx *ctx, const uint32_t *d) { return describe(1, d, choose(ctx, 1, d)); }

int tune_set(bh_ctx *ctx, int op, int cfg, int splits) {
  if (op < 0 || op > 1) return fail(BH_ERR, "tune_set: op must be 0 (sgemm) or 1 (conv)");
  if (cfg >= (int)cfgs(op).size()) return fail(BH_UNSUP, "tune_set: no such config");
  ctx->ovr_cfg[op] = cfg < 0 ? -1 : cfg;
  // splits: 0 = planned; n > 0 = n splits, combined in-kernel; -n = n splits, reduce kernel
  ctx->ovr_splits[op] = splits > 0 ? (uint32_t)splits : (uint32_t)(-splits);
  ctx->ovr_red[op] = splits > 0 ? 2 : (splits < 0 ? 1 : 0);
  return BH_OK;
}

int tune_set_wt(bh_ctx *ctx, int op, int wt) {
  if (op < 0 || op > 1) return fail(BH_ERR, "tune_set_wt: op must be 0 (sgemm) or 1 (conv)");
  ctx->ovr_wt[op] = wt < 0 ? -1 : (wt ? 1 : 0);
  return BH_OK;
}

int tune_cfg_name(int op, int cfg, std::string &out) {
  if (op < 0 || op > 1) return fail(BH_ERR, "op must be 0 (sgemm) or 1 (conv)");
  if (cfg < 0 || cfg >= (int)cfgs(op).size()) return fail(BH_UNSUP, "no such config");
  out = cfgs(op)[cfg].name;
  return BH_OK;
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
  p.cvec = (N % 4 == 0) && ((uintptr_t)c % 16 == 0);
  uint32_t d[3] = {M, N, K};
  choice_t ch = choose(ctx, 0, d);
  p.wt = ch.wt && fits_buffer((uint64_t)M * N * 4);
  if (getenv("BH_EXP_RING_DWORD_B") && vec && cfgs(0)[ch.cfg].k[A_KSCALAR][B_KSCALAR][0])  // experiment
    return launch_gemm(ctx, 0, ch, A_KSCALAR, B_KSCALAR, p, "sgemm");
  if (cfgs(0)[ch.cfg].ref64) return launch_ref64_sgemm(ctx, p);
  if (!vec && (!cfgs(0)[ch.cfg].k[A_KSCALAR][B_KSCALAR][0] || cfgs(0)[ch.cfg].name[0] == 'r')) ch = heuristic(0, d, false);
  return launch_gemm(ctx, 0, ch, vec ? A_KVEC : A_KSCALAR, vec ? B_KVEC : B_KSCALAR, p, "sgemm");
}

int launch_conv(bh_ctx *ctx, const float *in, const float *filts, const float *packed, const float *biases, float *out, uint32_t B,
                uint32_t IC, uint32_t H, uint32_t W, uint32_t OC, uint32_t KY, uint32_t KX, uint32_t sy,
                uint32_t sx, uint32_t py, uint32_t px, int relu, uint32_t out_ctot, const float *res,
                bool no_dc, bool repacked, uint32_t pk_banks) {
  // repacked: a fallback call after this call's filter repack was already dispatched (that repack
  // recorded the call's start event; no kernel of the fallback may record it again)
  // out_ctot: channels of the tensor `out` points into (0: OC). Every conv epilogue addresses
  // image i of the output at i * OCOHW, so a conv can write its channel slab of a wider
  // tensor (a Concat's output) in place.
  if (!out_ctot) out_ctot = OC;
  const uint32_t OH = (H + 2 * py - KY) / sy + 1, OW = (W + 2 * px - KX) / sx + 1;
  const uint64_t K = (uint64_t)IC * KY * KX, P = (uint64_t)B * OH * OW;
  const uint64_t in_bytes = (uint64_t)B * IC * H * W * 4, w_bytes = (uint64_t)OC * K * 4;
  if (!fits_buffer(in_bytes) || !fits_buffer(w_bytes) || !fits_buffer((uint64_t)B * out_ctot * OH * OW * 4))
    return fail(BH_UNSUP, "conv: tensor larger than 2 GiB");
  if (K >= (1u << 31) || P >= (1u << 31)) return fail(BH_UNSUP, "conv: GEMM extent too large");
  GemmArgs p{};
  p.a = filts; p.b = in; p.c = out; p.bias = biases; p.res = res;
  p.M = OC; p.N = (uint32_t)P; p.K = (uint32_t)K;
  p.lda = (uint32_t)K; p.ldb = 0; p.ldc = 0;
  p.a_bytes = (uint32_t)w_bytes;
  p.b_bytes = (uint32_t)in_bytes;
  p.relu = relu;
  // output (and residual) rows take float4 accesses (dword-aligned tensors: any OH*OW; a quad
  // of columns running past its image is stored element by element)
  p.cvec = ((uintptr_t)out % 4 == 0) && ((uintptr_t)res % 4 == 0);
  p.H = H; p.W = W; p.KX = KX; p.KYX = KY * KX;
  p.sy = sy; p.sx = sx; p.py = py; p.px = px;
  p.OW = OW; p.OHW = OH * OW; p.HW = H * W; p.ICHW = IC * H * W; p.OCOHW = out_ctot * OH * OW;
  set_fd(p.KYX, p.kyx_m, p.kyx_s);
  set_fd(KX, p.kx_m, p.kx_s);
  set_fd(p.OHW, p.ohw_m, p.ohw_s);
  set_fd(OW, p.ow_m, p.ow_s);
  const bool k1 = KY == 1 && KX == 1 && sy == 1 && sx == 1 && py == 0 && px == 0;
  const bool k1v = k1 && (H * W) % 4 == 0 && ((uintptr_t)in % 16 == 0);
  const bool avec = (K % 4 == 0) && ((uintptr_t)filts % 16 == 0);
  uint32_t d[11] = {B, IC, H, W, OC, KY, KX, sy, sx, py, px};
  choice_t ch = choose(ctx, 1, d);
  p.wt = ch.wt;  // the output fits a 2 GiB buffer (checked above)
  if (no_dc && cfgs(1)[ch.cfg].dc) ch = heuristic(1, d, true, false);
  const bool first = !repacked;
  if (cfgs(1)[ch.cfg].ref64) {  // the double-accumulating known-good kernel (reference layouts)
    p.IC = IC;
    return launch_ref64_conv(ctx, p, B, KY, first);
  }
  if (cfgs(1)[ch.cfg].gv && !cfgs(1)[ch.cfg].packA) {
    // few output columns: stream the bank in its reference layout; the window covering the
    // whole unpadded input makes the im2col the input itself (B_FC, 16-B loads). Shape
    // mismatches are UNSUP; a shape the config serves with only a pointer misaligned for its
    // vector loads falls back to the plain gv kernel (input) or the tile kernel (bank)
    const bool fc_shape = OH == 1 && OW == 1 && KY == H && KX == W && py == 0 && px == 0;
    const bool in16 = (uintptr_t)in % 16 == 0, fc = fc_shape && in16;
    bool tile_fallback = !avec;
    if (cfgs(1)[ch.cfg].fcv) {
      // batch-streaming ipconv (bh_gv.hip fcv_kernel): a wave per BM / 4 bank rows
      const cfg_t &fc_c = cfgs(1)[ch.cfg];
      if (!fc_shape || K % 4 || B > (uint32_t)fc_c.BN)
        return fail(BH_UNSUP, "conv: fcv configs need an ipconv (window = the whole unpadded input) at batch <= " +
                                  std::to_string(fc_c.BN) + " with K % 4 == 0");
      if (fc && avec) {
        void *args[] = {&p};
        return bh::launch(ctx, (const void *)fc_c.k[A_MVEC][B_FC][0], dim3((OC + fc_c.BM - 1) / fc_c.BM), dim3(fc_c.NT),
                          args, first, true, "conv");
      }
      tile_fallback = true;  // 16-B loads of the bank or the input rows impossible
    } else if (cfgs(1)[ch.cfg].k[A_MVEC][B_IM1X1S][0]) {
      // gvo (bh_gv.hip): 1x1 over the reference-layout bank, 16-deep k groups; an ipconv takes
      // its input rows as the columns (B_FC, one 16-B load per column tile and k group)
      const int cx = cfgs(1)[ch.cfg].gv_cx;
      if (fc_shape && K % 16 == 0 && cfgs(1)[ch.cfg].k[A_MVEC][B_FC][0]) {
        if (fc && avec) return launch_gemm(ctx, 1, ch, A_MVEC, B_FC, p, "conv", first);
        tile_fallback = true;
      } else {
        if (!k1 || IC % 16) return fail(BH_UNSUP, "conv: gvo configs need a 1x1 conv with IC % 16 == 0");
        if ((OH * OW) % (uint32_t)cx) return fail(BH_UNSUP, "conv: interleaved-column configs need OH*OW % run == 0");
        if (avec && (uintptr_t)in % (4u * cx) == 0) return launch_gemm(ctx, 1, ch, A_MVEC, B_IM1X1S, p, "conv", first);
        tile_fallback = true;  // 16-B bank rows or CX-wide pixel runs of the input misaligned
      }
    } else if (avec) {
      return launch_gemm(ctx, 1, ch, A_MVEC, fc ? B_FC : (k1 ? B_IM1X1 : B_IM2COL), p, "conv", first);
    }
    if (tile_fallback) {
      ch = choice_t{};  // unaligned bank (K % 4 or pointer) or input: a tile kernel
      ch.cfg = cfg_index(1, "128x32x32");
      ch.red = 1;
    }
  }
  if (cfgs(1)[ch.cfg].packA) {
    // ring kernels read the filter bank k-major: repack it first (this call's first dispatch)
    // (K order (ky, kx, ic), rows padded to a multiple of 64; input offsets + 2^30 must miss).
    // A Winograd route reads its bank behind it: from the caller's pack when that holds the bank
    // (pk_banks), otherwise from a pack of just the k-major bank + that bank made here. The 2 GiB
    // check and the context's pack buffer are sized by what the route reads.
    const uint32_t need = route_bank(cfgs(1)[ch.cfg], KY, KX);
    pk_banks &= all_banks(KY, KX);
    const uint32_t oc4 = (OC + 3) & ~3u, kp = (uint32_t)(kmajor_floats(OC, IC, KY, KX) / oc4);
    const float *wp = packed;
    uint32_t banks = pk_banks;
    if (wp && need && !(pk_banks & need)) wp = nullptr;  // the caller's pack lacks the route's bank
    if (!wp) banks = need;
    if (banks_floats(OC, IC, KY, KX, need) * 4 >= 0x7fffffc0ull || in_bytes >= (1ull << 30)) {
      ch = heuristic(1, d, false);
    } else {
      bool rp = repacked;  // a repack of this call already dispatched (it recorded the start event)
      if (!wp) {
        int rc = ensure_wpack(ctx, banks_floats(OC, IC, KY, KX, banks) * 4);
        if (rc == BH_OK) rc = launch_pack_banks(ctx, filts, (float *)ctx->wpack, OC, IC, KY, KX, banks, first, false);
        if (rc != BH_OK) return rc;
        wp = (const float *)ctx->wpack;
        rp = true;
      }
      const bool kfirst = !rp;  // the main kernel is the call's first dispatch
      p.a = wp;
      p.lda = oc4;
      p.a_bytes = kp * oc4 * 4;
      p.IC = IC;
      set_fd(IC, p.ic_m, p.ic_s);
      if (cfgs(1)[ch.cfg].dc) {
        const cfg_t &dcc = cfgs(1)[ch.cfg];
        const int rc = dcc.dc == 2   ? launch_dcm(ctx, dcc, p, B, KY, KX, sy, sx, ch.splits, kfirst)
                       : dcc.dc == 3 ? launch_k1s(ctx, dcc, p, B, KY, KX, sy, sx, ch.splits, kfirst)
                       : dcc.dc == 4 ? (need
                                            ? launch_wg(ctx, dcc, wp + bank_offset(OC, IC, KY, KX, banks, need), in, biases, res,
                                                        out, out_ctot, B, IC, H, W, OC, KY, KX, sy, sx, py, px, relu, p.wt,
                                                        ch.splits, kfirst)
                                            : bh::fail(BH_UNSUP, std::string("conv: ") + dcc.name + " is for 3x3 convs"))
                       : dcc.dc == 5 ? (need
                                            ? launch_wgx(ctx, dcc, wp + bank_offset(OC, IC, KY, KX, banks, need), in, biases,
                                                         res, out, out_ctot, B, IC, H, W, OC, KY, KX, sy, sx, py, px, relu,
                                                         p.wt, ch.splits, kfirst)
                                            : bh::fail(BH_UNSUP, std::string("conv: ") + dcc.name + " is for other kernel sizes"))
                                     : launch_dc(ctx, dcc, p, B, KY, KX, sy, sx, kfirst);
        if (rc != BH_UNSUP || (ctx && ctx->ovr_cfg[1] >= 0)) return rc;
        return launch_conv(ctx, in, filts, wp, biases, out, B, IC, H, W, OC, KY, KX, sy, sx, py, px, relu, out_ctot,
                           res, true, rp, banks);
      }
      if (cfgs(1)[ch.cfg].gv) {
        // register streaming over the packed bank (bh_gv.hip gvp_kernel): 16-deep k groups
        // inside one filter tap
        if (IC % 16) return fail(BH_UNSUP, "conv: gvp configs need IC % 16 == 0");
        if (cfgs(1)[ch.cfg].gv_cx > 1 && (!k1 || (OH * OW) % (uint32_t)cfgs(1)[ch.cfg].gv_cx))
          return fail(BH_UNSUP, "conv: interleaved-column configs need a 1x1 conv with OH*OW % run == 0");
        return launch_gemm(ctx, 1, ch, A_KVEC, k1 ? B_IM1X1S : B_IMTAP, p, "conv", kfirst);
      }
      const uint32_t bk = (uint32_t)cfgs(1)[ch.cfg].BK;
      const bool tab = ((p.K + bk - 1) / bk) * bk <= (uint32_t)TAB_MAX;  // K rows a block tabulates
      const int bld = k1 ? (IC % bk == 0 ? B_IM1X1S : B_IM1X1)
                         : (IC >= bk ? (IC % bk == 0 ? B_IMTAP : B_IMT2) : (tab ? B_IMTAB : B_IM2COL));
      return launch_gemm(ctx, 1, ch, A_KVEC, bld, p, "conv", kfirst);
    }
  }
  return launch_gemm(ctx, 1, ch, avec ? A_MVEC : A_MSCALAR, k1v ? B_IM1X1V : (k1 ? B_IM1X1 : B_IM2COL), p, "conv",
                     first);
}

}  // namespace bh
