// bh_ring.hip -- LDS-DMA ring kernels for the MFMA-bound conv / SGEMM shapes, and the
// filter-bank repack they read.
//
// Why a second throughput kernel (bh_gemm.hip's gemm_kernel stays for the shapes the
// tuner prefers it on): on big convolutions the register-staged tile kernel spends
// ~450 SALU + ~250 VALU issue slots per 32-deep K tile and wave on the im2col gather
// (PMC, profiles/r01), its global loads land in VGPRs and must be waited for before the
// LDS write, and its m-major weight tile is read with bank conflicts. Here
//  * both operands go global -> LDS by LDS-DMA (`buffer_load ... lds`) into a ring of D
//    stages with D-1 K tiles in flight, one counted vmcnt + raw s_barrier per K tile
//    (cdna_hip_programming.md §5 "Pipelining across barriers"): no staging VGPRs, no
//    ds_write pass;
//  * the conv weights are read k-major ([K][OC4], repacked once per call by
//    xpose_filts_kernel -- the counterpart of Boda's xpose_filts, test/rtc/xpose_filts.cucl,
//    src/rtc_fwd.cc:306-326), so the A fragments come from the same conflict-free k-major
//    LDS image as SGEMM's `a` (K x M, test/rtc/sgemm.cucl:1-3);
//  * one B DMA instruction = one k row x 64 output columns; a wave's column set is fixed
//    for the whole kernel (columns are dealt to waves by wave % TN), so per instruction the
//    im2col address is a scalar (ic, ky, kx) offset plus two per-lane range compares;
//  * 4 waves as 2 x 2, each owning (32 TM) x (32 TN) of the block tile with TM x TN
//    independent v_mfma_f32_32x32x2_f32 accumulators (exact fp32, 64 FLOP/clk/SIMD).
// Same GemmArgs contract, split-K modes and slab layout as gemm_kernel (bh_gemm.hip).
#include "bh_gemm_dev.h"

namespace bhk {
namespace {

// WGM: waves along M (2: 4 waves as 2 x 2; 4: 8 waves as 4 x 2, two per SIMD sharing one
// stage: a 256-row SGEMM tile halves the B-panel DMA per MFMA of the 128-row tile)
template <int TM, int TN, int BK, int D, int BLD, int SPL, int WGM = 2>
__global__ __launch_bounds__(128 * WGM) void ring_kernel(GemmArgs p) {
  constexpr int NW = 2 * WGM, NT = 64 * NW;
  constexpr int BM = 32 * TM * WGM, BN = 64 * TN, WM = 32 * TM, WN = 32 * TN;
  constexpr bool IM = (BLD == B_IM2COL || BLD == B_IMT2 || BLD == B_IM1X1 || BLD == B_IMTAB || BLD == B_IMTAP ||
                       BLD == B_IM1X1S);
  constexpr bool SOFF = (BLD == B_IMTAP || BLD == B_IM1X1S);  // rows differ by a scalar soffset only
  // im2col row table (int2 per k row): up to TAB_MAX rows of K plus the D-1 dead stages past it
  constexpr int TABF = BLD == B_IMTAB ? 2 * (TAB_MAX + (D - 1) * BK) : 0;
  constexpr bool DW = IM || BLD == B_KSCALAR;  // B by dword DMA: one k row x 64 columns per instruction
  static_assert(BLD == B_KVEC || DW, "ring loaders: k-major 16-B or dword (SGEMM b), im2col / 1x1 dword");
  static_assert(NW % TN == 0, "a wave's B columns: one 64-column group");
  constexpr int A_LDS = BK * BM, B_LDS = BK * BN, SLOT = A_LDS + B_LDS;
  // LDS-DMA wave instructions per wave per stage: A [BK][BM] in 16-B pieces; B [BK][BN] in
  // 16-B pieces (SGEMM) or one k row x 64 columns of dwords (conv)
  constexpr int LA = BK * BM / (NW * 256);
  constexpr int LB = DW ? BK * TN / NW : BK * BN / (NW * 256);
  static_assert(BK * BM % (NW * 256) == 0 && (DW ? BK * TN % NW : BK * BN % (NW * 256)) == 0,
                "whole DMA instructions per wave");
  constexpr int LW = LA + LB;
  static_assert(LA >= 1 && LB >= 1 && D >= 2 && (D - 2) * LW <= 63, "vmcnt range");
  static_assert(BK % 2 == 0, "two k rows per MFMA");
  constexpr int NBI = IM && SPL != 1 ? BM / 64 : 0;  // bias DMA instructions (wave 0)

  // one __shared__ array only (a second object makes hipcc wait vmcnt(0) at ds_reads)
  __shared__ __attribute__((aligned(16))) float smem[D * SLOT + (IM ? BM : 0) + 4 + TABF];
  float *const Lbias = smem + D * SLOT;
  constexpr int TAB0 = D * SLOT + (IM ? BM : 0) + 4;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
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

  // ---- per-lane parts of the DMA source offsets (fixed for the whole kernel; an
  // out-of-range lane holds OOB, and OOB + any in-range row offset stays >= 2^31: a miss)
  // A [BK][BM] / SGEMM B [BK][BN] in 16-B pieces: piece `lane` of an instruction covers row
  // 4*lane / BM, columns (4*lane) % BM (BM, BN divide 256); rows past K / kend read
  // zeros or don't matter (see the k guards below)
  constexpr int RA = 256 / BM, RB = 256 / BN;  // k rows per 16-B instruction
  const uint32_t am = bm0 + (uint32_t)(4 * lane) % BM;
  const uint32_t a_lane = oob_unless(am < p.M, ((uint32_t)(4 * lane) / BM * p.lda + am) * 4u);
  uint32_t b_lane = 0;
  if constexpr (BLD == B_KVEC) {
    const uint32_t bn = bn0 + (uint32_t)(4 * lane) % BN;
    b_lane = oob_unless(bn < p.N, ((uint32_t)(4 * lane) / BN * p.ldb + bn) * 4u);
  } else if constexpr (BLD == B_KSCALAR) {
    const uint32_t bn = bn0 + (uint32_t)(wave % TN) * 64 + (uint32_t)lane;
    b_lane = oob_unless(bn < p.N, bn * 4u);
  }
  // conv: this lane's output column (group wave % TN of the tile; a wave's B rows step NW / TN)
  int col_base = 0, iy0 = 0, ix0 = 0;
  const uint32_t bgrp = (uint32_t)(wave % TN);
  const uint32_t rw0 = (uint32_t)(wave / TN);
  constexpr uint32_t RSTEP = NW / TN;
  if constexpr (IM) {
    const uint32_t col = bn0 + bgrp * 64 + (uint32_t)lane;
    const uint32_t img = fdiv(col, p.ohw_m, p.ohw_s);
    const uint32_t pix = col - img * p.OHW;
    if constexpr (BLD == B_IM1X1 || BLD == B_IM1X1S) {
      col_base = col < p.N ? (int)(img * p.ICHW + pix) * 4 : (int)OOB;
    } else {
      const uint32_t oy = fdiv(pix, p.ow_m, p.ow_s);
      const uint32_t ox = pix - oy * p.OW;
      iy0 = (int)(oy * p.sy) - (int)p.py;
      ix0 = (int)(ox * p.sx) - (int)p.px;
      col_base = (int)(img * p.ICHW) + iy0 * (int)p.W + ix0;
      if (col >= p.N) iy0 = -(1 << 29);  // every ky misses: the column is past N
    }
  }
  // im2col, K order (ky, kx, ic): byte offset of this lane's input pixel at filter tap kyx
  // (channel 0), or OOB when the tap falls in the padding
  auto tap_off = [&](uint32_t kyx) -> uint32_t {
    const uint32_t ky = fdiv(kyx, p.kx_m, p.kx_s), kx = kyx - ky * p.KX;
    const bool ok = (kyx < p.KYX) & ((uint32_t)(iy0 + (int)ky) < p.H) & ((uint32_t)(ix0 + (int)kx) < p.W);
    return oob_unless(ok, (uint32_t)(col_base + (int)(ky * p.W + kx)) * 4u);
  };

  // Per-lane source offsets of this wave's LW DMA instructions for the stage at k0 (A pieces
  // first, then B rows); computed up front so the DMA issues can be spread between MFMAs.
  auto plan_stage = [&](uint32_t k0, uint32_t(&vo)[LW], uint32_t(&so)[LW]) {
#pragma unroll
    for (int q = 0; q < LW; ++q) so[q] = 0;
#pragma unroll
    for (int j = 0; j < LA; ++j) vo[j] = a_lane + (k0 + RA * (wave * LA + j)) * p.lda * 4u;
    if constexpr (BLD == B_KVEC) {
#pragma unroll
      for (int j = 0; j < LB; ++j) vo[LA + j] = b_lane + (k0 + RB * (wave * LB + j)) * p.ldb * 4u;
    } else if constexpr (BLD == B_KSCALAR) {
#pragma unroll
      for (int j = 0; j < LB; ++j) vo[LA + j] = b_lane + (k0 + rw0 + RSTEP * j) * p.ldb * 4u;
    } else if constexpr (BLD == B_IM1X1) {
#pragma unroll
      for (int j = 0; j < LB; ++j) {
        const uint32_t k = k0 + rw0 + RSTEP * j;  // wave-uniform k row
        vo[LA + j] = (uint32_t)col_base + (k < kend ? k * p.HW * 4u : 0x40000000u);
      }
    } else if constexpr (BLD == B_IMT2) {
      // IC >= BK: this wave's rows of the tile lie on at most two taps; both tap offsets
      // up front, each row picks one by a uniform compare (no branches). Rows past K sit on
      // taps >= KY*KX, which tap_off turns into misses; rows past a split's end never occur
      // in a computed tile (splits are whole K tiles).
      const uint32_t kf = k0 + rw0;
      const uint32_t kyx = fdiv(kf, p.ic_m, p.ic_s);
      const uint32_t ic0 = kf - kyx * p.IC;
      const uint32_t t0 = tap_off(kyx), t1 = tap_off(kyx + 1);
      const uint32_t hw4 = p.HW * 4u, ichw4 = p.IC * hw4;
      uint32_t soff = ic0 * hw4;
#pragma unroll
      for (int j = 0; j < LB; ++j) {
        const bool nxt = ic0 + RSTEP * j >= p.IC;
        vo[LA + j] = (nxt ? t1 : t0) + (nxt ? soff - ichw4 : soff);
        soff += RSTEP * hw4;
      }
    } else if constexpr (BLD == B_IM1X1S) {
      // K % BK == 0 and splits are whole K tiles: a stage is live (all rows valid) or dead
      const uint32_t v = k0 < kend ? (uint32_t)col_base : OOB;
      const uint32_t hw4 = p.HW * 4u;
#pragma unroll
      for (int j = 0; j < LB; ++j) {
        vo[LA + j] = v;
        so[LA + j] = (k0 + rw0 + RSTEP * j) * hw4;
      }
    } else if constexpr (BLD == B_IMTAP) {
      // the stage's tap (scalar), its per-lane offset or a miss (one select for all rows),
      // each row's channel offset as the scalar soffset
      const uint32_t kyx = fdiv(k0, p.ic_m, p.ic_s);
      const uint32_t ic0 = k0 - kyx * p.IC;
      const uint32_t t0 = tap_off(kyx);
      const uint32_t hw4 = p.HW * 4u;
#pragma unroll
      for (int j = 0; j < LB; ++j) {
        vo[LA + j] = t0;
        so[LA + j] = (ic0 + rw0 + RSTEP * j) * hw4;
      }
    } else if constexpr (BLD == B_IMTAB) {
      // tabulated rows: {ic*HW + ky*W + kx, ky | kx << 16} (rows past the range: ky = 0x7fff)
#pragma unroll
      for (int j = 0; j < LB; ++j) {
        const uint32_t r = k0 - kbeg + rw0 + RSTEP * j;
        // float-typed reads (the ring's TBAA type: an int-typed read made hipcc wait vmcnt(0))
        const int ex = __builtin_bit_cast(int, smem[TAB0 + 2 * r]);
        const int ey = __builtin_bit_cast(int, smem[TAB0 + 2 * r + 1]);
        const int ky = ey & 0xffff, kx = ey >> 16;
        const bool ok = ((uint32_t)(iy0 + ky) < p.H) & ((uint32_t)(ix0 + kx) < p.W);
        vo[LA + j] = oob_unless(ok, (uint32_t)(col_base + ex) * 4u);
      }
    } else {
      // any IC: (tap, ic) of each row by division (scalar), the lane's tap offset per row
#pragma unroll
      for (int j = 0; j < LB; ++j) {
        const uint32_t k = k0 + rw0 + RSTEP * j;
        const uint32_t kyx = fdiv(k, p.ic_m, p.ic_s);
        const uint32_t ic = k - kyx * p.IC;
        vo[LA + j] = tap_off(kyx) + ic * p.HW * 4u;
      }
    }
  };
  // DMA instruction q of this wave into ring slot `slot`
  auto issue_one = [&](int q, int slot, uint32_t vo, uint32_t so) {
    float *const Ab = smem + slot * SLOT;
    float *const Bb = Ab + A_LDS;
    if (q < LA) {
      dma16(rsa, Ab + (wave * LA + q) * 256, vo);
    } else if constexpr (BLD == B_KVEC) {
      dma16(rsb, Bb + (wave * LB + q - LA) * 256, vo);
    } else {
      if constexpr (SOFF) dma4s(rsb, Bb + (rw0 + RSTEP * (q - LA)) * BN + bgrp * 64, vo, so);
      else dma4(rsb, Bb + (rw0 + RSTEP * (q - LA)) * BN + bgrp * 64, vo);
    }
  };
  auto issue_stage = [&](int slot, uint32_t k0) {
    uint32_t vo[LW], so[LW];
    plan_stage(k0, vo, so);
#pragma unroll
    for (int q = 0; q < LW; ++q) issue_one(q, slot, vo[q], so[q]);
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;

  const int kh = lane >> 5, li = lane & 31;
  // lane half h takes k rows h*BK/2 .. h*BK/2 + BK/2 - 1 of the tile (same k for A and B).
  // The next stage's DMAs (into slot islot) are issued between the MFMA steps, so their
  // issue cycles hide under MFMA execution instead of delaying the first MFMA.
  constexpr int S2 = BK / 2;
  constexpr int PF = TM * TN >= 4 ? 1 : 2;  // LDS fragment prefetch distance (k steps)
  auto compute = [&](int slot, int islot, uint32_t k0) {
    uint32_t vo[LW], so[LW];
    plan_stage(k0, vo, so);
    const float *const Ab = smem + slot * SLOT + kh * S2 * BM + wm * WM + TM * li;
    const float *const Bb = smem + slot * SLOT + A_LDS + kh * S2 * BN + wn * WN + TN * li;
    // fragments of step s+PF are read while step s's MFMAs run (a ds_read waited for right
    // before its MFMA leaves the SIMD idle for the LDS latency every step)
    typename fvec<TM>::t av[PF + 1];
    typename fvec<TN>::t bv[PF + 1];
#pragma unroll
    for (int s = 0; s < PF; ++s) {
      av[s] = *(const typename fvec<TM>::t *)&Ab[s * BM];
      bv[s] = *(const typename fvec<TN>::t *)&Bb[s * BN];
    }
#pragma unroll
    for (int s = 0; s < S2; ++s) {
      if (s + PF < S2) {
        av[(s + PF) % (PF + 1)] = *(const typename fvec<TM>::t *)&Ab[(s + PF) * BM];
        bv[(s + PF) % (PF + 1)] = *(const typename fvec<TN>::t *)&Bb[(s + PF) * BN];
      }
      __builtin_amdgcn_sched_barrier(0);  // keep the prefetch ahead of this step's MFMAs
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(vget<TM>(av[s % (PF + 1)], i), vget<TN>(bv[s % (PF + 1)], j),
                                                           acc[i][j], 0, 0, 0);
#pragma unroll
      for (int q = 0; q < LW; ++q)
        if (q * S2 / LW == s) issue_one(q, islot, vo[q], so[q]);
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  // ---- main loop: D-stage LDS-DMA ring, D-1 K tiles in flight
  const uint32_t nkt = (kend - kbeg + BK - 1) / BK;
  if constexpr (NBI > 0) {
    // biases by DMA of wave 0, issued before stage 0 so the first stage wait covers them
    const __amdgpu_buffer_rsrc_t rsbias = make_rsrc(p.bias, p.bias ? p.M * 4u : 0u);
    if (wave == 0) {
#pragma unroll
      for (int j = 0; j < NBI; ++j) {
        const uint32_t m = bm0 + 64 * j + lane;
        dma4(rsbias, Lbias + 64 * j, oob_unless(m < p.M, m * 4u));
      }
    }
  }
  if constexpr (BLD == B_IMTAB) {
    // this block's K rows kbeg .. kbeg + (nkt + D - 1) * BK (the host checks nkt * BK <= TAB_MAX)
    for (uint32_t r = tid; r < (nkt + D - 1) * BK; r += NT) {
      const uint32_t k = kbeg + r;
      const uint32_t kyx = k / p.IC, ic = k - kyx * p.IC;
      const uint32_t ky = kyx / p.KX, kx = kyx - ky * p.KX;
      const bool valid = k < kend;
      smem[TAB0 + 2 * r] = __builtin_bit_cast(float, valid ? (int)(ic * p.HW + ky * p.W + kx) : 0);
      smem[TAB0 + 2 * r + 1] = __builtin_bit_cast(float, valid ? (int)(ky | (kx << 16)) : 0x7fff);
    }
    __syncthreads();
  }
  // Stages past the split's end are issued too (their lanes read OOB zeros without
  // touching memory), so every wave always has exactly D-2 stages in flight behind the
  // one it waits for and the issue code has no branches.
#pragma unroll
  for (int s = 0; s < D - 1; ++s) issue_stage(s, kbeg + s * BK);
  int slot = 0;
  for (uint32_t kt = 0; kt < nkt; ++kt) {
    vm_wait<(D - 2) * LW>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // stage kt landed for all waves; all done reading kt-1
    asm volatile("" ::: "memory");
    if (kt == 0) KT(1);
    compute(slot, slot == 0 ? D - 1 : slot - 1, kbeg + (kt + D - 1) * BK);  // + stage kt+D-1 into slot (kt-1) % D
    slot = slot == D - 1 ? 0 : slot + 1;
  }
  vm_wait<0>();
  KT(2);

  // ---- epilogue (the mapping of gemm_kernel: acc[i][j][r] is row (r&3)+8(r>>2)+4kh of
  // MFMA tile (i, j), column li; block row wm*WM + TM*row + i, column wn*WN + TN*li + j)
  const uint32_t n_base = bn0 + wn * WN + TN * li;
  if constexpr (SPLIT) {
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
    // write-through slab hand-off (see gemm_kernel): drain, barrier, relaxed agent ticket
    uint32_t *const flag = (uint32_t *)smem;  // the ring is dead: every wave waited vmcnt(0)
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
    combine_tile<IM ? 1 : 0, NT, BM * BN / 4 / NT, 4>(p, tile, tile_m, tile_n, gridDim.y, IM ? Lbias : nullptr, tid);
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
#pragma unroll
        for (int j = 0; j < TN; ++j)
          if (cofs[j] >= 0) out_elem1(p, (size_t)m * p.OHW + cofs[j], v[j]);
      } else {
        const size_t crow = (size_t)m * p.ldc + n_base;
        if (p.cvec && n_base + TN <= p.N && TN == 4) {
          out_elem4(p, crow, f32x4v{v[0], v[TN > 1 ? 1 : 0], v[TN > 2 ? 2 : 0], v[TN > 3 ? 3 : 0]});
        } else if (p.cvec && n_base + TN <= p.N && !p.wt) {
          float *const cr = p.c + crow;
          typename fvec<TN>::t w;
          if constexpr (TN == 1) w = v[0]; else {
#pragma unroll
            for (int j = 0; j < TN; ++j) w[j] = v[j];
          }
          *(typename fvec<TN>::t *)cr = w;
        } else {
#pragma unroll
          for (int j = 0; j < TN; ++j)
            if (n_base + j < p.N) out_elem1(p, crow + j, v[j]);
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
// Stream-K ring kernel: the ring above as a persistent grid. A launch has G blocks (one or
// two per CU, whatever the LDS allows) and the op's work is the list of (output tile, K tile)
// iterations, tile-major; logical block l takes iterations [l*ipb, (l+1)*ipb). Every CU does
// the same number of MFMA steps whatever the tile count (no partial last wave of tiles),
// and the DMA ring runs on across tile boundaries, so only the very first stage of a block
// waits a full memory latency.
//  * a tile whose iterations all fall in one block is finished in place (bias, ReLU, store);
//  * a tile cut by block boundaries: each of its blocks writes its partial tile (write-through)
//    to its own slab (slot 0: the block's first tile, slot 1: its last), takes the tile's
//    ticket, and the last arriver sums the slabs in k order (block b0..b1) and stores -- the
//    same fixed-order rule as the split-K combine, so results are bitwise reproducible.
// Logical blocks are laid out XCD-contiguously (hardware deals blocks round-robin over the
// 8 XCDs), so each XCD's L2 sees a contiguous run of tiles.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t xcd_contig(uint32_t bid, uint32_t G) {
  const uint32_t xcd = bid & 7, q = G >> 3, r = G & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}
// tile index -> (tile_m, tile_n), m fastest: consecutive tiles of a block share the B
// (input) column panel, the big operand of a convolution
__device__ __forceinline__ void sk_tile_coords(const GemmArgs &p, uint32_t t, uint32_t &tm, uint32_t &tn) {
  tn = fdiv(t, p.tm_m, p.tm_s);
  tm = t - tn * p.tiles_m;
}

template <int TM, int TN, int BK, int D, int BLD>
__global__ __launch_bounds__(256) void srk_kernel(GemmArgs p) {
  constexpr int NW = 4, NT = 256;
  constexpr int BM = 64 * TM, BN = 64 * TN, WM = 32 * TM, WN = 32 * TN;
  constexpr bool IM = (BLD == B_IM2COL || BLD == B_IMT2 || BLD == B_IM1X1 || BLD == B_IMTAP || BLD == B_IM1X1S ||
                       BLD == B_IMTAB);
  constexpr int TABF = BLD == B_IMTAB ? 2 * TAB_MAX : 0;  // im2col row table of the op's K rows
  constexpr bool SOFF = (BLD == B_IMTAP || BLD == B_IM1X1S);
  constexpr bool DW = IM;
  static_assert(BLD == B_KVEC || DW, "stream-K loaders: SGEMM 16-B, conv im2col / 1x1 dword");
  static_assert(NW % TN == 0, "a wave's B columns: one 64-column group");
  constexpr int A_LDS = BK * BM, B_LDS = BK * BN, SLOT = A_LDS + B_LDS;
  constexpr int LA = BK * BM / (NW * 256);
  constexpr int LB = DW ? BK * TN / NW : BK * BN / (NW * 256);
  static_assert(BK * BM % (NW * 256) == 0 && (DW ? BK * TN % NW : BK * BN % (NW * 256)) == 0,
                "whole DMA instructions per wave");
  constexpr int LW = LA + LB;
  static_assert(LA >= 1 && LB >= 1 && D >= 2 && (D - 2) * LW <= 63, "vmcnt range");
  constexpr int NCH = BM * BN / 4, CH = NCH / NT;  // float4 chunks of a tile, per thread
  static_assert(NCH % NT == 0, "combine chunking");

  __shared__ __attribute__((aligned(16))) float smem[D * SLOT + 4 + TABF];
  uint32_t *const flag = (uint32_t *)(smem + D * SLOT);
  constexpr int TAB0 = D * SLOT + 4;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const uint32_t lb = xcd_contig(blockIdx.x, gridDim.x);
  const uint32_t it0 = lb * p.ipb, it1 = min(p.total_it, it0 + p.ipb);
  const __amdgpu_buffer_rsrc_t rsa = make_rsrc(p.a, p.a_bytes);
  const __amdgpu_buffer_rsrc_t rsb = make_rsrc(p.b, p.b_bytes);

  constexpr int RA = 256 / BM, RB = 256 / BN;
  const uint32_t bgrp = (uint32_t)(wave % TN);
  const uint32_t rw0 = (uint32_t)(wave / TN);
  constexpr uint32_t RSTEP = NW / TN;

  // ---- per-lane DMA source state of the tile being issued, recomputed for every stage
  // without branches (a branch around it made hipcc drain the DMA ring, vmcnt(0), at the
  // K loop head; the recomputation is ~20 VALU + a few SALU per 32-deep K tile)
  uint32_t a_lane = 0, b_lane = 0, ls_tile = 0xffffffffu;
  int col_base = 0, iy0 = 0, ix0 = 0;
  auto set_tile = [&](uint32_t t) {
    uint32_t tm, tn;
    sk_tile_coords(p, t, tm, tn);
    const uint32_t bm0 = tm * BM, bn0 = tn * BN;
    const uint32_t am = bm0 + (uint32_t)(4 * lane) % BM;
    a_lane = oob_unless(am < p.M, ((uint32_t)(4 * lane) / BM * p.lda + am) * 4u);
    if constexpr (BLD == B_KVEC) {
      const uint32_t bn = bn0 + (uint32_t)(4 * lane) % BN;
      b_lane = oob_unless(bn < p.N, ((uint32_t)(4 * lane) / BN * p.ldb + bn) * 4u);
    } else {
      const uint32_t col = bn0 + bgrp * 64 + (uint32_t)lane;
      const uint32_t img = fdiv(col, p.ohw_m, p.ohw_s);
      const uint32_t pix = col - img * p.OHW;
      if constexpr (BLD == B_IM1X1 || BLD == B_IM1X1S) {
        col_base = col < p.N ? (int)(img * p.ICHW + pix) * 4 : (int)OOB;
      } else {
        const uint32_t oy = fdiv(pix, p.ow_m, p.ow_s);
        const uint32_t ox = pix - oy * p.OW;
        iy0 = (int)(oy * p.sy) - (int)p.py;
        ix0 = (int)(ox * p.sx) - (int)p.px;
        col_base = (int)(img * p.ICHW) + iy0 * (int)p.W + ix0;
        if (col >= p.N) iy0 = -(1 << 29);
      }
    }
  };
  auto tap_off = [&](uint32_t kyx) -> uint32_t {
    const uint32_t ky = fdiv(kyx, p.kx_m, p.kx_s), kx = kyx - ky * p.KX;
    const bool ok = (kyx < p.KYX) & ((uint32_t)(iy0 + (int)ky) < p.H) & ((uint32_t)(ix0 + (int)kx) < p.W);
    return oob_unless(ok, (uint32_t)(col_base + (int)(ky * p.W + kx)) * 4u);
  };
  // source offsets of this wave's LW DMA instructions for iteration `it` (all OOB past it1)
  auto plan_stage = [&](uint32_t it, uint32_t(&vo)[LW], uint32_t(&so)[LW]) {
    const bool live = it < it1;
#pragma unroll
    for (int q = 0; q < LW; ++q) so[q] = 0;
    const uint32_t t = fdiv(it, p.ipt_m, p.ipt_s);
    if (t != ls_tile) {  // uniform: only at the issue side's tile changes
      set_tile(t);
      ls_tile = t;
    }
    const uint32_t k0 = (it - t * p.ipt) * BK;
#pragma unroll
    for (int j = 0; j < LA; ++j) vo[j] = a_lane + (k0 + RA * (wave * LA + j)) * p.lda * 4u;
    if constexpr (BLD == B_KVEC) {
#pragma unroll
      for (int j = 0; j < LB; ++j) vo[LA + j] = b_lane + (k0 + RB * (wave * LB + j)) * p.ldb * 4u;
    } else if constexpr (BLD == B_IM1X1) {
#pragma unroll
      for (int j = 0; j < LB; ++j) {
        const uint32_t k = k0 + rw0 + RSTEP * j;
        vo[LA + j] = (uint32_t)col_base + (k < p.K ? k * p.HW * 4u : 0x40000000u);
      }
    } else if constexpr (BLD == B_IM1X1S) {
      const uint32_t hw4 = p.HW * 4u;  // K % BK == 0: every row of a live stage is valid
#pragma unroll
      for (int j = 0; j < LB; ++j) {
        vo[LA + j] = (uint32_t)col_base;
        so[LA + j] = (k0 + rw0 + RSTEP * j) * hw4;
      }
    } else if constexpr (BLD == B_IMTAP) {
      const uint32_t kyx = fdiv(k0, p.ic_m, p.ic_s);  // IC % BK == 0: one tap per stage
      const uint32_t ic0 = k0 - kyx * p.IC;
      const uint32_t t0 = tap_off(kyx), hw4 = p.HW * 4u;
#pragma unroll
      for (int j = 0; j < LB; ++j) {
        vo[LA + j] = t0;
        so[LA + j] = (ic0 + rw0 + RSTEP * j) * hw4;
      }
    } else if constexpr (BLD == B_IMTAB) {
      // tabulated rows {ic*HW + ky*W + kx, ky | kx << 16} (float-typed reads, as in ring_kernel)
#pragma unroll
      for (int j = 0; j < LB; ++j) {
        const uint32_t r = k0 + rw0 + RSTEP * j;
        const int ex = __builtin_bit_cast(int, smem[TAB0 + 2 * r]);
        const int ey = __builtin_bit_cast(int, smem[TAB0 + 2 * r + 1]);
        const int ky = ey & 0xffff, kx = ey >> 16;
        const bool ok = ((uint32_t)(iy0 + ky) < p.H) & ((uint32_t)(ix0 + kx) < p.W);
        vo[LA + j] = oob_unless(ok, (uint32_t)(col_base + ex) * 4u);
      }
    } else if constexpr (BLD == B_IMT2) {
      const uint32_t kf = k0 + rw0;
      const uint32_t kyx = fdiv(kf, p.ic_m, p.ic_s);
      const uint32_t ic0 = kf - kyx * p.IC;
      const uint32_t t0 = tap_off(kyx), t1 = tap_off(kyx + 1);
      const uint32_t hw4 = p.HW * 4u, ichw4 = p.IC * hw4;
      uint32_t soff = ic0 * hw4;
#pragma unroll
      for (int j = 0; j < LB; ++j) {
        const bool nxt = ic0 + RSTEP * j >= p.IC;
        vo[LA + j] = (nxt ? t1 : t0) + (nxt ? soff - ichw4 : soff);
        soff += RSTEP * hw4;
      }
    } else {
#pragma unroll
      for (int j = 0; j < LB; ++j) {
        const uint32_t k = k0 + rw0 + RSTEP * j;
        const uint32_t kyx = fdiv(k, p.ic_m, p.ic_s);
        const uint32_t ic = k - kyx * p.IC;
        vo[LA + j] = tap_off(kyx) + ic * p.HW * 4u;
      }
    }
    // dead stages: set the top offset bit (a miss) -- a select, not a branch (a branch here
    // made hipcc wait vmcnt(0) at the join)
    const uint32_t dead = live ? 0u : OOB;
#pragma unroll
    for (int q = 0; q < LW; ++q) vo[q] |= dead;
  };
  auto issue_one = [&](int q, int slot, uint32_t vo, uint32_t so) {
    float *const Ab = smem + slot * SLOT;
    float *const Bb = Ab + A_LDS;
    if (q < LA) {
      dma16(rsa, Ab + (wave * LA + q) * 256, vo);
    } else if constexpr (BLD == B_KVEC) {
      dma16(rsb, Bb + (wave * LB + q - LA) * 256, vo);
    } else {
      if constexpr (SOFF) dma4s(rsb, Bb + (rw0 + RSTEP * (q - LA)) * BN + bgrp * 64, vo, so);
      else dma4(rsb, Bb + (rw0 + RSTEP * (q - LA)) * BN + bgrp * 64, vo);
    }
  };

  f32x16 acc[TM][TN];
  auto zero_acc = [&]() {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;
  };

  const int kh = lane >> 5, li = lane & 31;
  constexpr int S2 = BK / 2;
  constexpr int PF = TM * TN >= 4 ? 1 : 2;
  auto compute = [&](int slot, int islot, uint32_t it_issue) {
    uint32_t vo[LW], so[LW];
    plan_stage(it_issue, vo, so);
    const float *const Ab = smem + slot * SLOT + kh * S2 * BM + wm * WM + TM * li;
    const float *const Bb = smem + slot * SLOT + A_LDS + kh * S2 * BN + wn * WN + TN * li;
    typename fvec<TM>::t av[PF + 1];
    typename fvec<TN>::t bv[PF + 1];
#pragma unroll
    for (int s = 0; s < PF; ++s) {
      av[s] = *(const typename fvec<TM>::t *)&Ab[s * BM];
      bv[s] = *(const typename fvec<TN>::t *)&Bb[s * BN];
    }
#pragma unroll
    for (int s = 0; s < S2; ++s) {
      if (s + PF < S2) {
        av[(s + PF) % (PF + 1)] = *(const typename fvec<TM>::t *)&Ab[(s + PF) * BM];
        bv[(s + PF) % (PF + 1)] = *(const typename fvec<TN>::t *)&Bb[(s + PF) * BN];
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(vget<TM>(av[s % (PF + 1)], i), vget<TN>(bv[s % (PF + 1)], j),
                                                           acc[i][j], 0, 0, 0);
#pragma unroll
      for (int q = 0; q < LW; ++q)
        if (q * S2 / LW == s) issue_one(q, islot, vo[q], so[q]);
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  // finished tile t: this block's accumulators hold iterations [max(it0, t*ipt), min(it1, (t+1)*ipt))
  auto finish_tile = [&](uint32_t t) {
    uint32_t tm, tn;
    sk_tile_coords(p, t, tm, tn);
    const uint32_t bm0 = tm * BM, bn0 = tn * BN;
    const uint32_t tb = t * p.ipt;
    if (tb >= it0 && tb + p.ipt <= it1) {
      // whole tile here: bias, ReLU, store
      const uint32_t n_base = bn0 + wn * WN + TN * li;
      int cofs[TN];
      if constexpr (IM) {
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const uint32_t col = n_base + j;
          const uint32_t img = fdiv(col, p.ohw_m, p.ohw_s);
          cofs[j] = col < p.N ? (int)(img * p.OCOHW + (col - img * p.OHW)) : -1;
        }
      }
#pragma unroll
      for (int i = 0; i < TM; ++i) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const uint32_t m = bm0 + wm * WM + TM * ((r & 3) + 8 * (r >> 2) + 4 * kh) + i;
          if (m >= p.M) continue;
          const float bias = (IM && p.bias) ? p.bias[m] : 0.0f;
          float v[TN];
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            float x = acc[i][j][r] + bias;
            if constexpr (IM)
              if (p.res && cofs[j] >= 0) x += p.res[(size_t)m * p.OHW + cofs[j]];  // residual (Eltwise SUM)
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
      return;
    }
    // partial tile: slab (block, slot), ticket, the last arriver combines in k order
    const uint32_t slot = (t == fdiv(it0, p.ipt_m, p.ipt_s)) ? 0u : 1u;
    float *const wz = p.ws + ((size_t)lb * 2 + slot) * (BM * BN);
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
        if constexpr (TN == 1) {
          __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, w), rw, off * 4, 0, AUX_SC1);
        } else if constexpr (TN == 2) {
          __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(__attribute__((ext_vector_type(2))) uint32_t, w),
                                                rw, off * 4, 0, AUX_SC1);
        } else {
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) uint32_t, w),
                                                 rw, off * 4, 0, AUX_SC1);
        }
      }
    const uint32_t b0 = tb / p.ipb, b1 = (tb + p.ipt - 1) / p.ipb;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      const uint32_t old = __hip_atomic_fetch_add(&p.cnt[t], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const uint32_t last = old == b1 - b0 ? 1u : 0u;
      if (last) __hip_atomic_store(&p.cnt[t], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *flag = last;
    }
    __syncthreads();
    if (!*flag) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // compiler-only: keep the loads below the ticket
    const __amdgpu_buffer_rsrc_t rall = make_rsrc(p.ws, 0x7fffff00u);
    f32x4v sum[CH];
#pragma unroll
    for (int j = 0; j < CH; ++j) sum[j] = f32x4v{0.0f, 0.0f, 0.0f, 0.0f};
    for (uint32_t b = b0; b <= b1; ++b) {
      const uint32_t sl = (b == b0 && t != fdiv(b * p.ipb, p.ipt_m, p.ipt_s)) ? 1u : 0u;
      const uint32_t base = (b * 2 + sl) * (uint32_t)(BM * BN * 4);
      f32x4v x[CH];
#pragma unroll
      for (int j = 0; j < CH; ++j)
        x[j] = __builtin_bit_cast(f32x4v, __builtin_amdgcn_raw_buffer_load_b128(rall, base + 16 * (tid + j * NT), 0,
                                                                                 AUX_SC1));
#pragma unroll
      for (int j = 0; j < CH; ++j) sum[j] += x[j];
    }
#pragma unroll
    for (int j = 0; j < CH; ++j) finish_store<IM ? 1 : 0>(p, tm, tn, (uint32_t)(tid + j * NT), sum[j], nullptr);
  };

  if constexpr (BLD == B_IMTAB) {
    // the op's K rows 0 .. ipt * BK (the host checks <= TAB_MAX); rows past K: misses
    for (uint32_t r = tid; r < p.ipt * BK; r += NT) {
      const uint32_t kyx = r / p.IC, ic = r - kyx * p.IC;
      const uint32_t ky = kyx / p.KX, kx = kyx - ky * p.KX;
      const bool valid = r < p.K;
      smem[TAB0 + 2 * r] = __builtin_bit_cast(float, valid ? (int)(ic * p.HW + ky * p.W + kx) : 0);
      smem[TAB0 + 2 * r + 1] = __builtin_bit_cast(float, valid ? (int)(ky | (kx << 16)) : 0x7fff);
    }
    __syncthreads();
  }
  // ---- main loop over this block's iterations: D-stage ring running across tiles
#pragma unroll
  for (int s = 0; s < D - 1; ++s) {
    uint32_t vo[LW], so[LW];
    plan_stage(it0 + s, vo, so);
#pragma unroll
    for (int q = 0; q < LW; ++q) issue_one(q, s, vo[q], so[q]);
  }
  // outer loop over this block's tiles, inner loop over a tile's K iterations (a nested
  // loop keeps the accumulators in AGPRs: a flat loop with the tile epilogue inside made
  // hipcc copy them VGPR <-> AGPR around every K tile)
  int slot = 0;
  uint32_t it = it0;
  while (it < it1) {
    const uint32_t ct = fdiv(it, p.ipt_m, p.ipt_s);   // tile being accumulated
    const uint32_t ct_end = min(it1, (ct + 1) * p.ipt);
    zero_acc();
    for (; it < ct_end; ++it) {
      vm_wait<(D - 2) * LW>();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      compute(slot, slot == 0 ? D - 1 : slot - 1, it + D - 1);
      slot = slot == D - 1 ? 0 : slot + 1;
    }
    finish_tile(ct);
    // a real (compiler-visible) vmcnt(0) after the tile's stores: otherwise hipcc carries the
    // epilogue's pending stores into the K loop head and waits vmcnt(0) there every iteration
    __builtin_amdgcn_s_waitcnt(0x0F70);
  }
  vm_wait<0>();
}

// Filter-bank repack for the ring conv kernels: wp[(kyx * IC + ic)][m] = w[m][ic * KYX + kyx]
// for m < OC (K order (ky, kx, ic): one tap per run of IC rows), 0 for OC <= m < OC4 (rows
// padded to a multiple of 4 floats for 16-B DMA) and for rows K <= k < Kp (K padded to a
// multiple of the deepest ring K tile, so a K tile never reads past the bank). 64 x 64 tiles
// through LDS (row pad 1: conflict-free column reads); reads and writes are 256-B runs.
__global__ __launch_bounds__(256) void xpose_filts_kernel(const float *__restrict__ w, float *__restrict__ wp,
                                                          uint32_t OC, uint32_t K, uint32_t OC4, uint32_t IC,
                                                          uint32_t KYX, uint32_t Kp) {
  __shared__ float t[64][65];
  const uint32_t j0 = blockIdx.x * 64, m0 = blockIdx.y * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const uint32_t m = m0 + ty + 4 * i, j = j0 + tx;
    t[ty + 4 * i][tx] = (m < OC && j < K) ? w[(size_t)m * K + j] : 0.0f;
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const uint32_t j = j0 + ty + 4 * i, m = m0 + tx;
    if (j < Kp && m < OC4) {
      const uint32_t row = j < K ? (j % KYX) * IC + j / KYX : j;
      wp[(size_t)row * OC4 + m] = t[tx][ty + 4 * i];
    }
  }
}

template <int TM, int TN, int BK, int D, int BLD>
void reg_ring(cfg_t &c) {
  c.k[A_KVEC][BLD][0] = ring_kernel<TM, TN, BK, D, BLD, 0>;
  c.k[A_KVEC][BLD][1] = ring_kernel<TM, TN, BK, D, BLD, 1>;
  c.k[A_KVEC][BLD][2] = ring_kernel<TM, TN, BK, D, BLD, 2>;
}
template <int TM, int TN, int BK, int D>
cfg_t ring_conv_cfg(const char *name) {
  cfg_t c{name, 64 * TM, 64 * TN, BK, 256, {}, 1};
  reg_ring<TM, TN, BK, D, B_IM2COL>(c);
  reg_ring<TM, TN, BK, D, B_IMTAB>(c);
  reg_ring<TM, TN, BK, D, B_IMTAP>(c);
  reg_ring<TM, TN, BK, D, B_IM1X1S>(c);
  reg_ring<TM, TN, BK, D, B_IMT2>(c);
  reg_ring<TM, TN, BK, D, B_IM1X1>(c);
  return c;
}
template <int TM, int TN, int BK, int D>
cfg_t srk_conv_cfg(const char *name) {
  cfg_t c{name, 64 * TM, 64 * TN, BK, 256, {}, 1, 1, (D * BK * 64 * (TM + TN) + 4) * 4};
  c.k[A_KVEC][B_IM2COL][0] = srk_kernel<TM, TN, BK, D, B_IM2COL>;
  c.k[A_KVEC][B_IMT2][0] = srk_kernel<TM, TN, BK, D, B_IMT2>;
  c.k[A_KVEC][B_IM1X1][0] = srk_kernel<TM, TN, BK, D, B_IM1X1>;
  c.k[A_KVEC][B_IMTAP][0] = srk_kernel<TM, TN, BK, D, B_IMTAP>;
  c.k[A_KVEC][B_IM1X1S][0] = srk_kernel<TM, TN, BK, D, B_IM1X1S>;
  if constexpr (BK == 16 || TM * TN == 1) c.k[A_KVEC][B_IMTAB][0] = srk_kernel<TM, TN, BK, D, B_IMTAB>;
  return c;
}
template <int TM, int TN, int BK, int D>
cfg_t srk_sgemm_cfg(const char *name) {
  cfg_t c{name, 64 * TM, 64 * TN, BK, 256, {}, 0, 1, (D * BK * 64 * (TM + TN) + 4) * 4};
  c.k[A_KVEC][B_KVEC][0] = srk_kernel<TM, TN, BK, D, B_KVEC>;
  return c;
}
template <int TM, int TN, int BK, int D>
cfg_t ring_sgemm_cfg(const char *name) {
  cfg_t c{name, 64 * TM, 64 * TN, BK, 256, {}, 0};
  reg_ring<TM, TN, BK, D, B_KVEC>(c);
  c.k[A_KSCALAR][B_KSCALAR][0] = ring_kernel<TM, TN, BK, D, B_KSCALAR, 0>;  // (experiment: dword B, 16-B A)
  return c;
}
// 8 waves (4 x 2): 256-row tiles, two waves per SIMD on one stage
template <int TM, int TN, int BK, int D>
cfg_t ring_sgemm8_cfg(const char *name) {
  cfg_t c{name, 128 * TM, 64 * TN, BK, 512, {}, 0};
  c.k[A_KVEC][B_KVEC][0] = ring_kernel<TM, TN, BK, D, B_KVEC, 0, 4>;
  c.k[A_KVEC][B_KVEC][1] = ring_kernel<TM, TN, BK, D, B_KVEC, 1, 4>;
  c.k[A_KVEC][B_KVEC][2] = ring_kernel<TM, TN, BK, D, B_KVEC, 2, 4>;
  return c;
}

}  // namespace

std::vector<cfg_t> ring_cfgs(int op) {
  if (op == 0)
    return {
        ring_sgemm_cfg<2, 2, 32, 4>("r128x128x32d4"),
        ring_sgemm_cfg<2, 2, 64, 2>("r128x128x64d2"),
        ring_sgemm_cfg<2, 2, 32, 2>("r128x128x32d2"),
        ring_sgemm_cfg<2, 4, 32, 3>("r128x256x32d3"),
        ring_sgemm8_cfg<2, 2, 32, 2>("r256x128x32d2w8"),
        ring_sgemm8_cfg<2, 2, 16, 3>("r256x128x16d3w8"),
        ring_sgemm8_cfg<2, 2, 16, 4>("r256x128x16d4w8"),
        srk_sgemm_cfg<2, 2, 32, 2>("srk128x128x32d2"),
        srk_sgemm_cfg<2, 2, 16, 4>("srk128x128x16d4"),
        srk_sgemm_cfg<2, 2, 32, 4>("srk128x128x32d4"),
        srk_sgemm_cfg<2, 2, 32, 3>("srk128x128x32d3"),
    };
  return {
      ring_conv_cfg<2, 2, 32, 4>("r128x128x32d4"),
      ring_conv_cfg<2, 2, 32, 3>("r128x128x32d3"),
      ring_conv_cfg<1, 4, 32, 3>("r64x256x32d3"),
      ring_conv_cfg<2, 4, 32, 3>("r128x256x32d3"),
      ring_conv_cfg<1, 2, 32, 4>("r64x128x32d4"),
      ring_conv_cfg<2, 1, 32, 4>("r128x64x32d4"),
      ring_conv_cfg<1, 1, 32, 4>("r64x64x32d4"),
      // two blocks per CU (<= 80 KB LDS): one block's prologue / epilogue overlaps the other's loop
      ring_conv_cfg<2, 2, 32, 2>("r128x128x32d2"),
      ring_conv_cfg<2, 2, 16, 4>("r128x128x16d4"),
      ring_conv_cfg<2, 1, 32, 3>("r128x64x32d3"),
      ring_conv_cfg<1, 2, 32, 3>("r64x128x32d3"),
      ring_conv_cfg<1, 4, 32, 2>("r64x256x32d2"),
      // BK 16: IC % 16 == 0 shapes (144, 112, 48, 528 ...) take the one-tap loader
      ring_conv_cfg<1, 2, 16, 4>("r64x128x16d4"),
      ring_conv_cfg<2, 1, 16, 4>("r128x64x16d4"),
      ring_conv_cfg<1, 1, 16, 4>("r64x64x16d4"),
      // deeper rings: a short K (1x1, IC <= 80) fits the prologue, one memory round trip
      ring_conv_cfg<1, 1, 16, 5>("r64x64x16d5"),
      ring_conv_cfg<1, 1, 16, 7>("r64x64x16d7"),
      ring_conv_cfg<1, 2, 16, 5>("r64x128x16d5"),
      ring_conv_cfg<2, 1, 16, 5>("r128x64x16d5"),
      ring_conv_cfg<1, 1, 32, 3>("r64x64x32d3"),
      srk_conv_cfg<2, 2, 32, 2>("srk128x128x32d2"),
      srk_conv_cfg<2, 2, 16, 4>("srk128x128x16d4"),
      srk_conv_cfg<2, 2, 32, 4>("srk128x128x32d4"),
      srk_conv_cfg<2, 2, 32, 3>("srk128x128x32d3"),
      srk_conv_cfg<2, 1, 32, 4>("srk128x64x32d4"),
      srk_conv_cfg<2, 1, 32, 3>("srk128x64x32d3"),
      srk_conv_cfg<1, 2, 32, 4>("srk64x128x32d4"),
      srk_conv_cfg<1, 2, 32, 3>("srk64x128x32d3"),
      srk_conv_cfg<1, 1, 32, 4>("srk64x64x32d4"),
      srk_conv_cfg<1, 1, 16, 4>("srk64x64x16d4"),
      srk_conv_cfg<1, 2, 16, 4>("srk64x128x16d4"),
      srk_conv_cfg<1, 4, 32, 3>("srk64x256x32d3"),
  };
}

int launch_xpose_filts(bh_ctx *ctx, const float *w, float *wp, uint32_t OC, uint32_t IC, uint32_t KYX,
                       bool first, bool last) {
  const uint32_t OC4 = (OC + 3) & ~3u, K = IC * KYX, Kp = (K + 63) & ~63u;
  void *args[] = {(void *)&w, (void *)&wp, (void *)&OC, (void *)&K, (void *)&OC4, (void *)&IC, (void *)&KYX, (void *)&Kp};
  return bh::launch(ctx, (const void *)xpose_filts_kernel, dim3(Kp / 64, (OC4 + 63) / 64, 1), dim3(256), args, first,
                    last, "xpose_filts");
}

size_t kmajor_floats(uint32_t OC, uint32_t IC, uint32_t KY, uint32_t KX) {
  return (size_t)(((uint64_t)IC * KY * KX + 63) & ~63ull) * ((OC + 3) & ~3u);
}

uint32_t all_banks(uint32_t KY, uint32_t KX) {
  if (KY == 3 && KX == 3) return BANK_W23 | BANK_W43;
  if (KY == 5 && KX == 5) return BANK_W25;
  return 0;
}

static size_t bank_floats(uint32_t bank, uint32_t OC, uint32_t IC) {
  return bank == BANK_W23 ? wino_bank_floats(OC, IC) : wx_bank_floats(OC, IC);
}

size_t banks_floats(uint32_t OC, uint32_t IC, uint32_t KY, uint32_t KX, uint32_t banks) {
  banks &= all_banks(KY, KX);
  size_t n = kmajor_floats(OC, IC, KY, KX);
  for (uint32_t b = 1; b <= BANK_W25; b <<= 1)
    if (banks & b) n += bank_floats(b, OC, IC);
  return n;
}

size_t bank_offset(uint32_t OC, uint32_t IC, uint32_t KY, uint32_t KX, uint32_t banks, uint32_t bank) {
  return banks_floats(OC, IC, KY, KX, banks & (bank - 1));
}

uint32_t route_bank(const cfg_t &c, uint32_t KY, uint32_t KX) {
  if (c.dc == 4) return KY == 3 && KX == 3 ? BANK_W23 : 0;
  if (c.dc != 5 || (uint32_t)c.dc_ky != KY || KX != KY) return 0;
  if (KY == 5) return c.dc_s == 2 ? BANK_W25 : 0;
  if (KY == 3) return c.dc_s == 4 ? BANK_W43 : BANK_W23;
  return 0;
}

// the k-major bank, then the Winograd banks of the mask (cut to the kernel size's)
int launch_pack_banks(bh_ctx *ctx, const float *filts, float *packed, uint32_t OC, uint32_t IC, uint32_t KY, uint32_t KX,
                      uint32_t banks, bool first, bool last) {
  banks &= all_banks(KY, KX);
  int rc = launch_xpose_filts(ctx, filts, packed, OC, IC, KY * KX, first, last && !banks);
  for (uint32_t b = 1; rc == BH_OK && b <= BANK_W25; b <<= 1) {
    if (!(banks & b)) continue;
    float *u = packed + bank_offset(OC, IC, KY, KX, banks, b);
    const bool lb = last && !(banks & ~(2 * b - 1));  // the mask's last bank
    rc = b == BANK_W23 ? launch_wino_pack(ctx, filts, u, OC, IC, false, lb)
                       : launch_wx_pack(ctx, filts, u, OC, IC, b == BANK_W25 ? 5 : 3, false, lb);
  }
  return rc;
}

int ensure_wpack(bh_ctx *ctx, size_t bytes) {
  return bh::grow_buffer(ctx, ctx->wpack, ctx->wpack_bytes, bytes, false, "filter-bank pack buffer");
}

}  // namespace bhk

namespace bh {
// the k-major bank, then the Winograd banks of the mask (bhk::launch_pack_banks)
size_t conv_filts_packed_floats(uint32_t OC, uint32_t IC, uint32_t KY, uint32_t KX, uint32_t banks) {
  return bhk::banks_floats(OC, IC, KY, KX, banks);
}
int launch_conv_filts_pack(bh_ctx *ctx, const float *filts, float *packed, uint32_t OC, uint32_t IC, uint32_t KY,
                           uint32_t KX, uint32_t banks) {
  if (conv_filts_packed_floats(OC, IC, KY, KX, banks) * 4 >= 0x7fffffc0ull)
    return fail(BH_UNSUP, "conv_filts_pack: bank larger than 2 GiB");
  return bhk::launch_pack_banks(ctx, filts, packed, OC, IC, KY, KX, banks, true, true);  // a call of its own
}
}  // namespace bh
