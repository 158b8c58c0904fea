// bh_gemm_dev.h -- device-side building blocks shared by the GEMM / conv kernel sources
// (bh_gemm.hip: register-staged tile kernels + latency kernels; bh_ring.hip: LDS-DMA ring
// kernels). Internal to libboda_hip.so.
#pragma once
#include "bh_common.h"

namespace bhk {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4v __attribute__((ext_vector_type(4)));
typedef float f32x2v __attribute__((ext_vector_type(2)));

enum { A_KVEC = 0, A_KSCALAR = 1, A_MVEC = 2, A_MSCALAR = 3 };
enum { B_KVEC = 0, B_KSCALAR = 1, B_IM2COL = 2, B_IM1X1 = 3, B_IM1X1V = 4, B_IMT2 = 5, B_FC = 6, B_IMTAB = 7,
       B_IMTAP = 8, B_IM1X1S = 9, B_DIRECT = 10, NBLD = 11 };
// B_DIRECT: direct-conv kernels (bh_direct.hip): the input strip staged whole per block
// B_IM1X1S: ring kernels' 1x1 loader when K % BK == 0: the lane's pixel offset (VGPR, a miss
// for dead stages) + each row's channel offset as the scalar soffset
// B_IMTAP: ring kernels' im2col when IC % BK == 0: a K tile lies inside one filter tap, so a
// stage has ONE per-lane tap offset (VGPR) and each k row adds a scalar channel offset through
// the buffer instruction's soffset -- no per-row vector work
// B_IMTAB: ring kernels' im2col for IC < BK (stem convs): the per-k-row (ic, ky, kx) decomposition
// is tabulated in LDS once per block (TAB_MAX rows) instead of computed by scalar divisions
// for every row of every stage
constexpr int TAB_MAX = 512;
// B_FC: the im2col of a conv whose window covers the whole (unpadded) input -- Boda's ipconv /
// InnerProduct-as-conv -- is the input itself: column n = image n, X[k][n] = in[n * K + k]
// B_IMT2: ring kernels' im2col when IC >= BK: a wave's rows of one K tile touch at most two
// filter taps (ring kernels read K in (ky, kx, ic) order)
// B_IM1X1V: 1x1 conv whose OH*OW % 4 == 0 with a 16-B aligned input: four adjacent output
// columns are four adjacent input pixels of one image (latency kernel only; the tile
// kernel treats it as B_IM1X1)

constexpr uint32_t OOB = 0x80000000u;  // buffer offset that always misses (extents < 2^31)
constexpr int APAD = 4;                // m-major A tile row padding (floats)

struct GemmArgs {
  const float *a, *b;
  float *c;
  const float *bias;
  float *ws;       // split-K partial slabs, tile-major: [S][tile][BM*BN]
  uint32_t *cnt;   // split-K arrival tickets, one per tile (zero between calls)
  uint32_t M, N, K;
  uint32_t lda, ldb, ldc;
  uint32_t tbm, tbn;          // tile shape (for the split-K combine)
  uint32_t ks;                // K extent of one split (multiple of BK)
  uint32_t a_bytes, b_bytes;  // buffer extents in bytes (reads beyond come back 0)
  uint32_t c_bytes;           // output extent (direct conv: buffer stores; beyond = dropped)
  uint32_t tiles_m, tiles_n;
  int relu;
  int cvec;  // dense C rows can take TN-wide vector stores
  int wt;    // output stores write through (sc1): the output leaves L2 during the kernel instead of
             // at the next kernel boundary (set only when the output fits a 2 GiB buffer)
  const float *res;  // conv only, may be null: out = relu(conv + bias + res), res laid out like out
  // implicit im2col (B_IM2COL / B_IM1X1); N = B*OH*OW, K = IC*KY*KX
  uint32_t H, W, KX, KYX, sy, sx, py, px, OW, OHW, HW, ICHW, OCOHW;
  uint32_t kyx_m, kyx_s, kx_m, kx_s, ohw_m, ohw_s, ow_m, ow_s;  // fastdiv constants
  uint32_t IC, ic_m, ic_s;  // ring kernels: K order (ky, kx, ic) of the repacked filter bank
  // stream-K kernels (srk_kernel): K tiles per output tile, per block, in total; fastdiv of ipt
  uint32_t ipt, ipb, total_it, ipt_m, ipt_s, tm_m, tm_s;  // + fastdiv of tiles_m
#ifdef BH_KTRACE
  unsigned long long *trace;  // per-block device-clock marks (tools/ktrace.py)
#endif
};

#ifdef BH_KTRACE
#define KT(k)                                                                                     \
  do {                                                                                            \
    if (threadIdx.x == 0)                                                                         \
      p.trace[((size_t)blockIdx.y * gridDim.x + blockIdx.x) * 8 + (k)] = wall_clock64();          \
  } while (0)
#else
#define KT(k) \
  do {        \
  } while (0)
#endif

__device__ __forceinline__ uint32_t fdiv(uint32_t n, uint32_t m, uint32_t s) {
  return (__umulhi(n, m) + n) >> s;
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void *p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), (short)0, (int)bytes, 0x00020000);
}
// Offset, or the always-missing OOB offset when !ok. Callers combine conditions with
// bitwise & (no short-circuit): a && chain lets hipcc turn the select into a branch
// around each load, which also breaks its vmcnt bookkeeping for the ring.
__device__ __forceinline__ uint32_t oob_unless(bool ok, uint32_t off) { return ok ? off : OOB; }
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

template <int N>
__device__ __forceinline__ float vget(const typename fvec<N>::t &v, int i) {
  if constexpr (N == 1) return v;
  else return v[i];
}

constexpr int AUX_SC1 = 16;  // cache-policy bits: sc1 (write-through stores / L1-bypassing loads)
// Final output stores: write-through. Dirty L2 lines left at the end of a kernel are written back
// at the kernel boundary, before the next launch in the stream starts (MI355X_MICROARCH.md,
// boundary row: + bytes / ~6 TB/s); written through during the kernel they overlap the compute.
#ifndef BH_AUX_OUT
#define BH_AUX_OUT 0
#endif
constexpr int AUX_OUT = BH_AUX_OUT;

// Output stores under the call's policy (p.wt, wave-uniform): write-through (sc1) or AUX_OUT
__device__ __forceinline__ void out_store4(const GemmArgs &p, __amdgpu_buffer_rsrc_t r, uint32_t off, f32x4v v) {
  const auto u = __builtin_bit_cast(__attribute__((ext_vector_type(4))) uint32_t, v);
  if (p.wt) __builtin_amdgcn_raw_buffer_store_b128(u, r, off, 0, AUX_SC1);
  else __builtin_amdgcn_raw_buffer_store_b128(u, r, off, 0, AUX_OUT);
}
__device__ __forceinline__ void out_store1(const GemmArgs &p, __amdgpu_buffer_rsrc_t r, uint32_t off, float v) {
  if (p.wt) __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), r, off, 0, AUX_SC1);
  else __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), r, off, 0, AUX_OUT);
}
// element o of p.c (plain stores, or buffer stores through sc1 when p.wt)
__device__ __forceinline__ void out_elem4(const GemmArgs &p, size_t o, f32x4v v) {
  if (p.wt) __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) uint32_t, v),
                                                   make_rsrc(p.c, 0x7fffff00u), (uint32_t)(o * 4), 0, AUX_SC1);
  else *(f32x4v *)&p.c[o] = v;
}
__device__ __forceinline__ void out_elem1(const GemmArgs &p, size_t o, float v) {
  if (p.wt) __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), make_rsrc(p.c, 0x7fffff00u),
                                                  (uint32_t)(o * 4), 0, AUX_SC1);
  else p.c[o] = v;
}

// Split-K slabs are summed in fixed order s = 0..S-1 (bitwise reproducible whoever
// combines: the reduce kernel or a tile's last-arriving block).
// Bias, ReLU and store of one float4 chunk c (tile elements 4c..4c+3, row-major BM x BN)
// of tile (tile_m, tile_n): dense C rows, or NCHW scatter for conv (IMODE). p.cvec: rows
// take aligned float4 stores (dense: ldc % 4 == 0; conv: OH*OW % 4 == 0).
// finish_store_b: the same with the chunk's bias value already in hand (prefetched)
// (TBN > 0: the tile width p.tbn as a compile-time constant -- a run-time udiv is ~25 VALU on a
// small op's critical path)
template <int IMODE, int TBN = 0>
__device__ __forceinline__ void finish_store_b(const GemmArgs &p, uint32_t tile_m, uint32_t tile_n, uint32_t c,
                                               f32x4v sum, float b) {
  const uint32_t tbn = TBN > 0 ? (uint32_t)TBN : p.tbn;
  const uint32_t e0 = 4 * c, row = e0 / tbn, col0 = e0 - row * tbn;
  const uint32_t m = tile_m * p.tbm + row;
  if (m >= p.M) return;
  const uint32_t n0 = tile_n * tbn + col0;
#pragma unroll
  for (int t = 0; t < 4; ++t) sum[t] += b;
  // conv: four columns in one image are four adjacent floats of the output row, at any dword
  // alignment (OHW % 4 != 0 puts channel m's row at m * OHW; the hardware takes unaligned
  // dword-multiple accesses); element stores scatter a wave instruction over 4x the rows
  const uint32_t img0 = IMODE ? fdiv(n0, p.ohw_m, p.ohw_s) : 0u, pix0 = n0 - img0 * p.OHW;
  if (IMODE ? (p.cvec && n0 + 4 <= p.N && pix0 + 4 <= p.OHW) : (p.cvec && n0 + 4 <= p.N)) {
    size_t o;
    if constexpr (IMODE) {
      o = (size_t)img0 * p.OCOHW + (size_t)m * p.OHW + pix0;
      if (p.res) sum += *(const f32x4v *)&p.res[o];
    } else {
      o = (size_t)m * p.ldc + n0;
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) sum[t] = (p.relu && sum[t] < 0.0f) ? 0.0f : sum[t];
    out_elem4(p, o, sum);
    return;
  }
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const uint32_t n = n0 + t;
    if (n >= p.N) break;
    float x = sum[t];
    if constexpr (IMODE) {
      const uint32_t img = fdiv(n, p.ohw_m, p.ohw_s);
      const size_t o = (size_t)img * p.OCOHW + (size_t)m * p.OHW + (n - img * p.OHW);
      if (p.res) x += p.res[o];
      out_elem1(p, o, (p.relu && x < 0.0f) ? 0.0f : x);
    } else {
      out_elem1(p, (size_t)m * p.ldc + n, (p.relu && x < 0.0f) ? 0.0f : x);
    }
  }
}

template <int IMODE>
__device__ __forceinline__ void finish_store(const GemmArgs &p, uint32_t tile_m, uint32_t tile_n, uint32_t c,
                                             f32x4v sum, const float *bias_lds) {
  const uint32_t row = 4 * c / p.tbn, m = tile_m * p.tbm + row;
  if (m >= p.M) return;
  finish_store_b<IMODE>(p, tile_m, tile_n, c, sum, bias_lds ? bias_lds[row] : (p.bias ? p.bias[m] : 0.0f));
}



// Split-K combine of one float4 chunk c for the reduce kernel (after a kernel boundary,
// so plain loads): the S slabs summed in fixed order, four in flight.
template <int IMODE>
__device__ __forceinline__ void combine_store(const GemmArgs &p, uint32_t tile, uint32_t tile_m, uint32_t tile_n,
                                              uint32_t c, uint32_t S, const float *bias_lds) {
  const size_t tsz = (size_t)p.tbm * p.tbn, slab = tsz * p.tiles_m * p.tiles_n;
  f32x4v sum = {0.0f, 0.0f, 0.0f, 0.0f};
  uint32_t q = 0;
  const f32x4v *src = (const f32x4v *)(p.ws + (size_t)tile * tsz) + c;
  for (; q + 4 <= S; q += 4) {
    f32x4v a0 = src[(q + 0) * slab / 4], a1 = src[(q + 1) * slab / 4];
    f32x4v a2 = src[(q + 2) * slab / 4], a3 = src[(q + 3) * slab / 4];
    sum += a0; sum += a1; sum += a2; sum += a3;
  }
  for (; q < S; ++q) sum += src[q * slab / 4];
  finish_store<IMODE>(p, tile_m, tile_n, c, sum, bias_lds);
}

// In-kernel split-K combine of a whole tile by one block (the last arriver): each
// thread owns CH float4 chunks (c = tid + j*NT), processed G at a time with all of
// a group's loads for four slabs issued before any is consumed, so the slab reads
// overlap instead of costing one round trip per chunk and slab. Same fixed slab order as
// combine_store (bitwise identical results).
template <int IMODE, int NT, int CH, int G, int NCH = CH * NT>
__device__ __forceinline__ void combine_tile(const GemmArgs &p, uint32_t tile, uint32_t tile_m, uint32_t tile_n,
                                             uint32_t S, const float *bias_lds, int tid) {
  static_assert(CH % G == 0, "chunk grouping");
  if (NCH % NT != 0 && tid >= NCH) return;  // fewer chunks than threads (CH == 1)
  const uint32_t tsz = p.tbm * p.tbn, sstep = tsz * p.tiles_m * p.tiles_n * 4;
  const __amdgpu_buffer_rsrc_t rw = make_rsrc(p.ws, 0x7fffff00u);
#pragma unroll 1
  for (int g = 0; g < CH; g += G) {
    uint32_t off[G];
    f32x4v sum[G];
#pragma unroll
    for (int j = 0; j < G; ++j) {
      off[j] = (tile * tsz + 4 * (uint32_t)(tid + (g + j) * NT)) * 4;
      sum[j] = f32x4v{0.0f, 0.0f, 0.0f, 0.0f};
    }
    // four slabs per round trip (the last round's missing slabs read OOB zeros and are not
    // added: the sum is the same sequence of additions as combine_store's)
    for (uint32_t q = 0; q < S; q += 4) {
      f32x4v x[4][G];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < G; ++j)
          x[i][j] = __builtin_bit_cast(
              f32x4v, __builtin_amdgcn_raw_buffer_load_b128(rw, oob_unless(q + i < S, off[j] + (q + i) * sstep), 0,
                                                            AUX_SC1));
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < G; ++j)
          if (q + i < S) sum[j] += x[i][j];
    }
#pragma unroll
    for (int j = 0; j < G; ++j) finish_store<IMODE>(p, tile_m, tile_n, (uint32_t)(tid + (g + j) * NT), sum[j], bias_lds);
  }
}

// LDS-staged tile epilogue. Per-fragment stores from the MFMA accumulators move 128-256 B per
// store instruction, and a CU retires store instructions at a roughly fixed rate whatever their
// width (cdna_hip_programming.md T21: the store ISSUE bounds such an epilogue) -- a 64 KB tile
// took several microseconds. Here the waves' accumulators go to LDS row-major (the ring is
// dead: the caller has drained every DMA), and every thread then takes float4 chunks c of the
// BM x BN tile (row 4c / BN), handing each to f(c, value): one 16-B store per lane, 1 KB per
// wave instruction. Accumulator map of the tile kernels: acc[i][j][r] is row
// wm*WM + TM*((r&3) + 8*(r>>2) + 4*kh) + i, column wn*WN + TN*li + j.
// If the LDS cannot hold the whole tile (BM*BN > LDSF floats), it goes in two halves of BM/2
// rows (waves of one wave-row each). Ends with every thread past its last LDS read.
template <int BM, int BN, int TM, int TN, int WAVES_N, int NT, int LDSF, class F>
__device__ __forceinline__ void staged_epilogue(float *lds, f32x16 (&acc)[TM][TN], int wave, int lane, int tid,
                                                F &&f) {
  constexpr int WM = 32 * TM, WN = 32 * TN;
  constexpr int WAVES_M = NT / 64 / WAVES_N;
  constexpr int PASSES = BM * BN <= LDSF ? 1 : 2;
  static_assert(PASSES == 1 || (WAVES_M == 2 && (BM / 2) * BN <= LDSF), "staged epilogue: LDS too small");
  constexpr int PR = BM / PASSES;          // rows per pass
  constexpr int CPP = PR * BN / 4;         // float4 chunks per pass
  const int wm = wave / WAVES_N, wn = wave % WAVES_N, kh = lane >> 5, li = lane & 31;
#pragma unroll
  for (int h = 0; h < PASSES; ++h) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // every wave done with the LDS (ring reads / previous pass)
    asm volatile("" ::: "memory");
    if (PASSES == 1 || wm == h) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = (PASSES == 1 ? wm * WM : 0) + TM * ((r & 3) + 8 * (r >> 2) + 4 * kh) + i;
          typename fvec<TN>::t w;
          if constexpr (TN == 1) w = acc[i][0][r]; else {
#pragma unroll
            for (int j = 0; j < TN; ++j) w[j] = acc[i][j][r];
          }
          *(typename fvec<TN>::t *)&lds[row * BN + wn * WN + TN * li] = w;
        }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
#pragma unroll
    for (int k = 0; k < (CPP + NT - 1) / NT; ++k) {
      const int c = tid + k * NT;
      if (CPP % NT == 0 || c < CPP) f((uint32_t)(h * CPP + c), *(const f32x4v *)&lds[4 * c]);
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}

// max(x, floor) as one v_max_f32 (fmaxf adds a canonicalizing v_max per operand in IEEE mode);
// floor is 0 (ReLU) or a quiet NaN (none: v_max_f32 returns the other operand, so x passes as is, a NaN
// included), wave-uniform
__device__ __forceinline__ float relu_floor(float x, float floor) {
  float r;
  asm("v_max_f32 %0, %1, %2" : "=v"(r) : "s"(floor), "v"(x));
  return r;
}

template <int N>
__device__ __forceinline__ void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
typedef __attribute__((address_space(3))) void *lds_ptr_t;
__device__ __forceinline__ void dma4s(__amdgpu_buffer_rsrc_t r, const float *lds, uint32_t voff, uint32_t soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_ptr_t)lds, 4, voff, soff, 0, 0);
}
__device__ __forceinline__ void dma4(__amdgpu_buffer_rsrc_t r, const float *lds, uint32_t voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_ptr_t)lds, 4, voff, 0, 0, 0);
}
__device__ __forceinline__ void dma16s(__amdgpu_buffer_rsrc_t r, const float *lds, uint32_t voff, uint32_t soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_ptr_t)lds, 16, voff, soff, 0, 0);
}
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, const float *lds, uint32_t voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_ptr_t)lds, 16, voff, 0, 0, 0);
}


typedef void (*kern_t)(GemmArgs);

struct cfg_t {
  const char *name;
  int BM, BN, BK, NT;
  kern_t k[4][NBLD][3];  // [A loader][B loader][SPL]
  int packA;          // conv: A is the filter bank repacked k-major [K][OC4] (bh_ring.hip)
  int streamk = 0;    // persistent stream-K grid (srk_kernel): k[..][..][0] only
  int lds_bytes = 0;  // static LDS per block (stream-K grid sizing)
  int gv = 0;         // filter-streaming kernel (bh_gv.hip): grid (M / BM) x K chunks, BN >= N
  int dc_icmax = 0;   // dc == 1 resident-weight form: input channels it keeps resident (0: the ring form)
  int dc = 0;         // direct conv (bh_direct.hip; 2: bh_dcm.hip, 3: bh_k1s.hip): kernel dc_ky x dc_kx, stride dc_s, strip dc_rin x dc_wpm
  int dc_ky = 0, dc_kx = 0, dc_s = 0, dc_wpm = 0, dc_rin = 0;
  int dc_ci = 0;      // dc == 2 (bh_dcm.hip): input channels per stage
  int gv_cx = 1;      // gv: interleaved column tiles (1x1, a lane's gv_cx pixels per load)
  int fcv = 0;        // gv: batch-streaming ipconv kernel (bh_gv.hip fcv_kernel), batch <= BN
  int ref64 = 0;      // double-accumulating known-good kernel (bh_ref64.hip), never tuned in
  int k1n = 0;        // dc == 3: the pixels-on-N form (bh_k1s.hip k1n_kernel; gv_cx pixels per lane)
  int k1d = 0;        // dc == 3: the whole bank resident, input by 16-B LDS-DMA (bh_k1s.hip k1d_kernel)
  int k1w = 0;        // dc == 3: store waves of the k1w form (bh_k1s.hip k1w_kernel; NT counts them too)
  int k1w_sl = 0;     // k1w: LDS staging slots per compute wave
  int k1r = 0;        // dc == 3: the bank slice in VGPRs, K <= k1r (bh_k1s.hip k1r_kernel)
};

// bh_ring.hip: LDS-DMA ring configurations (conv ones read the repacked filter bank) and
// the repack itself (into the context's wpack buffer; first dispatch of a conv call)
std::vector<cfg_t> ring_cfgs(int op);
// bh_gv.hip: filter-streaming configurations for convs with few output columns
std::vector<cfg_t> gv_cfgs();
// bh_direct.hip: direct-conv configurations for the few-channel stem layers
std::vector<cfg_t> dc_cfgs();
// bh_ref64.hip: the double-accumulating known-good configuration "ref64" of conv and SGEMM
std::vector<cfg_t> ref64_cfgs();
int launch_ref64_conv(bh_ctx *ctx, GemmArgs &p, uint32_t B, uint32_t KY, bool first);
int launch_ref64_sgemm(bh_ctx *ctx, GemmArgs &p);
int launch_dc(bh_ctx *ctx, const cfg_t &c, GemmArgs &p, uint32_t B, uint32_t KY, uint32_t KX, uint32_t sy,
              uint32_t sx, bool first);
// bh_dcm.hip: multi-channel direct-conv configurations for stride-1 3x3 / 5x5 convs
std::vector<cfg_t> dcm_cfgs();
int launch_dcm(bh_ctx *ctx, const cfg_t &c, GemmArgs &p, uint32_t B, uint32_t KY, uint32_t KX, uint32_t sy,
               uint32_t sx, uint32_t splits, bool first);
// bh_k1s.hip: 1x1 convs with the bank slice resident in LDS, input streamed into registers
std::vector<cfg_t> k1s_cfgs();
int launch_k1s(bh_ctx *ctx, const cfg_t &c, GemmArgs &p, uint32_t B, uint32_t KY, uint32_t KX, uint32_t sy,
               uint32_t sx, uint32_t splits, bool first);
// bh_wino.hip: Winograd F(2x2, 3x3) configurations for stride-1 3x3 convs; u = the Winograd bank
// (the part of a 3x3 pack behind the k-major bank)
std::vector<cfg_t> wg_cfgs();
int launch_wg(bh_ctx *ctx, const cfg_t &c, const float *u, const float *in, const float *bias, const float *res,
              float *out, uint32_t out_ctot, uint32_t B, uint32_t IC, uint32_t H, uint32_t W, uint32_t OC, uint32_t KY,
              uint32_t KX, uint32_t sy, uint32_t sx, uint32_t py, uint32_t px, int relu, int wt, uint32_t splits,
              bool first);
size_t wino_bank_floats(uint32_t OC, uint32_t IC);
// bh_wgx.hip: position-split Winograd (F(4x4,3x3), F(2x2,5x5), F(2x2,3x3); two waves per SIMD); u = the
// bank of the configuration's form (wgx_bank_offset into a pack)
std::vector<cfg_t> wgx_cfgs();
int launch_wgx(bh_ctx *ctx, const cfg_t &c, const float *u, const float *in, const float *bias, const float *res,
               float *out, uint32_t out_ctot, uint32_t B, uint32_t IC, uint32_t H, uint32_t W, uint32_t OC, uint32_t KY,
               uint32_t KX, uint32_t sy, uint32_t sx, uint32_t py, uint32_t px, int relu, int wt, uint32_t splits,
               bool first);
size_t wx_bank_floats(uint32_t OC, uint32_t IC);
int launch_wx_pack(bh_ctx *ctx, const float *filts, float *u, uint32_t OC, uint32_t IC, uint32_t R, bool first,
                   bool last);
// A conv pack: the k-major bank, then the Winograd banks of its mask in bit order -- F(2x2,3x3)
// (BANK_W23, bh_wino.hip's [IC4][OC32][16]), F(4x4,3x3) (BANK_W43) and F(2x2,5x5) (BANK_W25, both
// wx_pack's [IC4][OC32][36]). A mask is cut to the banks of the kernel size (all_banks): the full
// pack of bh_conv_filts_pack is a 3x3's W23 + W43, a 5x5's W25.
constexpr uint32_t BANK_W23 = 1u, BANK_W43 = 2u, BANK_W25 = 4u, BANKS_ALL = 0xffffffffu;
uint32_t all_banks(uint32_t KY, uint32_t KX);
size_t banks_floats(uint32_t OC, uint32_t IC, uint32_t KY, uint32_t KX, uint32_t banks);
// offset in floats of bank (one BANK_*) in a pack holding banks (it must be one of them)
size_t bank_offset(uint32_t OC, uint32_t IC, uint32_t KY, uint32_t KX, uint32_t banks, uint32_t bank);
// the bank a configuration reads (0: the k-major bank only)
uint32_t route_bank(const cfg_t &c, uint32_t KY, uint32_t KX);
int launch_pack_banks(bh_ctx *ctx, const float *filts, float *packed, uint32_t OC, uint32_t IC, uint32_t KY,
                      uint32_t KX, uint32_t banks, bool first, bool last);
int launch_wino_pack(bh_ctx *ctx, const float *filts, float *u, uint32_t OC, uint32_t IC, bool first, bool last);
// floats of the k-major bank (the first part of every pack)
size_t kmajor_floats(uint32_t OC, uint32_t IC, uint32_t KY, uint32_t KX);
// split-K / stream-K workspace and arrival tickets of the context (bh_gemm.hip)
int ensure_ws(bh_ctx *ctx, size_t bytes);
int ensure_cnt(bh_ctx *ctx, uint64_t n);
int launch_xpose_filts(bh_ctx *ctx, const float *w, float *wp, uint32_t OC, uint32_t IC, uint32_t KYX, bool first,
                       bool last);
int ensure_wpack(bh_ctx *ctx, size_t bytes);

}  // namespace bhk
