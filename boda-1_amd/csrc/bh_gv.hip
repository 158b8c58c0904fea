// bh_gv.hip -- filter-streaming kernel for convolutions with few output columns.
//
// Boda's ipconv variant (src/cnn_op.cc:46-68, test/rtc/ipconv.cucl) and the fully connected
// layers run as convolutions whose output is a handful of columns: N = B*OH*OW is 1..64 while
// the filter bank is up to 151 MB (fc6: 4096 x 256*6*6). Such an op is a matrix-vector
// product bounded by streaming the filter bank from HBM once (53 of the 204
// conv ops are HBM-bound). The tile kernels read the bank through a 128-row LDS tile and an
// MFMA tile mostly wasted on padding columns; here
//  * the bank is read in its reference layout (OC x IC*KY*KX, row-major) straight into
//    registers with 16-B buffer loads -- each filter element is used by exactly one wave, so
//    there is nothing to share through LDS -- and a wave keeps its whole 64-deep K batch of
//    loads (R row tiles x 4 x 16 B per lane) in flight before the MFMAs consume them;
//  * v_mfma_f32_16x16x4_f32 (exact fp32; 16 output columns per tile, C tiles cover N): lane
//    (i = l & 15, g = l >> 4) holds rows/columns i and k = 4g + q of MFMA step q, so a lane's
//    16-B load of 4 consecutive k feeds four MFMA steps (a valid reduction order: A and B
//    use the same k map);
//  * the four waves of a block split the block's K chunk; their partial tiles are summed
//    through LDS in wave order, and the K chunks of a row tile (grid.y) are combined by the
//    tile's last-arriving block in chunk order (the split-K protocol of bh_gemm.hip) -- the
//    result is bitwise reproducible.
// Column operand loaders: B_FC (the input itself, 16-B loads along k), B_IM1X1 and B_IM2COL
// (scalar gathers by the implicit-im2col formulas of the tile kernels).
#include "bh_gemm_dev.h"

namespace bhk {
namespace {

typedef float f32x4t __attribute__((ext_vector_type(4)));


// Block geometry of the register-streaming kernels: R x C 16x16 MFMA tiles, NW waves.
template <int R, int C, int NW>
struct gv_geom {
  static constexpr int NT = NW * 64, BMr = 16 * R, NC = 16 * C;
  static constexpr int TSZ = BMr * NC;  // floats of a block's output tile
  static constexpr int NCH = TSZ / 4, CH = (NCH + NT - 1) / NT;
  static_assert(NCH % NT == 0 || NT % NCH == 0, "float4 chunks per thread");
};

// bias of the rows this thread stores in the epilogue, fetched at kernel entry (a dependent
// global load at the end of a small op costs a full memory round trip)
template <int R, int C, int NW>
__device__ __forceinline__ void gv_bias(const GemmArgs &p, uint32_t m0, int tid, float (&bias_r)[gv_geom<R, C, NW>::CH]) {
  using G = gv_geom<R, C, NW>;
  const bool has = G::NCH % G::NT == 0 || tid < G::NCH;
#pragma unroll
  for (int j = 0; j < G::CH; ++j) {
    const uint32_t m = m0 + 4 * (uint32_t)(tid + j * G::NT) / G::NC;
    bias_r[j] = (has && p.bias && m < p.M) ? p.bias[m] : 0.0f;
  }
}

// Epilogue of the register-streaming kernels: the NW waves' partial tiles -> LDS (row-major
// BMr x NC), summed in wave order; then either stored (one K chunk) or, with K chunks
// (grid.y > 1), written as this chunk's slab, and the tile's last-arriving block sums the
// slabs in chunk order (the split-K protocol of bh_gemm.hip: bitwise reproducible).
// RS: row interleave of the MFMA row tiles -- row rho of tile r is block row RS * rho + r
// (RS = 1: tile r owns rows 16 r .. 16 r + 15, written as 16 r + rho).
// CX > 1: column tiles interleaved -- column i of MFMA tile c is block column CX * i + c
template <int R, int C, int NW, int RS, int CX = 1>
__device__ __forceinline__ void gv_finish(const GemmArgs &p, f32x4t (&acc)[R][C], float *red, uint32_t tm, uint32_t tn,
                                          int tid, int wave, int lane,
                                          const float (&bias_r)[gv_geom<R, C, NW>::CH]) {
  using G = gv_geom<R, C, NW>;
  constexpr int NT = G::NT, NC = G::NC, TSZ = G::TSZ, NCH = G::NCH, CH = G::CH;
  uint32_t *const flag = (uint32_t *)(red + NW * TSZ);
  const int i = lane & 15, g = lane >> 4;
  const uint32_t tile = blockIdx.x, split = blockIdx.y;
  // 16x16x4 C/D map: register j of lane l is row 4 * (l >> 4) + j, column l & 15.
  {
    float *const Rw = red + wave * TSZ;
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int c = 0; c < C; ++c)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int row = RS == 1 ? 16 * r + 4 * g + j : RS * (4 * g + j) + r;
          Rw[row * NC + (CX > 1 ? CX * i + c : 16 * c + i)] = acc[r][c][j];
        }
  }
  __syncthreads();
  const bool has = NCH % NT == 0 || tid < NCH;
  f32x4v v[CH];
#pragma unroll
  for (int j = 0; j < CH; ++j) {
    const int ch = has ? tid + j * NT : 0;
    v[j] = *(const f32x4v *)&red[4 * ch];
#pragma unroll
    for (int w = 1; w < NW; ++w) v[j] += *(const f32x4v *)&red[w * TSZ + 4 * ch];
  }
  constexpr int IMODE = 1;
  if (gridDim.y == 1) {
    if (has) {
#pragma unroll
      for (int j = 0; j < CH; ++j) finish_store_b<IMODE, NC>(p, tm, tn, (uint32_t)(tid + j * NT), v[j], bias_r[j]);
    }
#ifdef BH_KTRACE
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    KT(4);
#endif
    return;
  }
  // ---- K chunks: slab [split][tile][TSZ] (write-through), ticket, last arriver combines
  const __amdgpu_buffer_rsrc_t rw = make_rsrc(p.ws + ((size_t)split * p.tiles_m * p.tiles_n + tile) * TSZ, TSZ * 4);
  if (has) {
#pragma unroll
    for (int j = 0; j < CH; ++j)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) uint32_t, v[j]),
                                             rw, 16 * (tid + j * NT), 0, AUX_SC1);
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
  if (!*flag) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // compiler-only: keep the loads below the ticket
  // the K chunks' slabs summed in chunk order (as combine_tile), all loads of a slab in flight
  if (!has) return;
  const uint32_t tstep = TSZ * p.tiles_m * p.tiles_n * 4;
  const __amdgpu_buffer_rsrc_t rall = make_rsrc(p.ws, 0x7fffff00u);
  f32x4v sum[CH];
#pragma unroll
  for (int j = 0; j < CH; ++j) sum[j] = f32x4v{0.0f, 0.0f, 0.0f, 0.0f};
  // four K chunks per round trip (missing ones read OOB zeros and are not added: same order)
  const uint32_t S = gridDim.y;
  for (uint32_t q = 0; q < S; q += 4) {
    f32x4v x[4][CH];
#pragma unroll
    for (int i2 = 0; i2 < 4; ++i2)
#pragma unroll
      for (int j = 0; j < CH; ++j)
        x[i2][j] = __builtin_bit_cast(
            f32x4v, __builtin_amdgcn_raw_buffer_load_b128(
                        rall, oob_unless(q + i2 < S, (q + i2) * tstep + (tile * TSZ + 4 * (uint32_t)(tid + j * NT)) * 4), 0,
                        AUX_SC1));
#pragma unroll
    for (int i2 = 0; i2 < 4; ++i2)
#pragma unroll
      for (int j = 0; j < CH; ++j)
        if (q + i2 < S) sum[j] += x[i2][j];
  }
#pragma unroll
  for (int j = 0; j < CH; ++j) finish_store_b<IMODE, NC>(p, tm, tn, (uint32_t)(tid + j * NT), sum[j], bias_r[j]);
}

// NW waves split the block's K chunk; NG 16-deep k groups per register batch; DB: the next
// batch's loads are issued before this batch's MFMAs (register double buffer)
template <int R, int C, int NW, int NG, int DB, int BLD>
__global__ __launch_bounds__(NW * 64) void gv_kernel(GemmArgs p) {
  using G = gv_geom<R, C, NW>;
  constexpr int BMr = G::BMr, NC = G::NC, KB = 16 * NG;
  __shared__ __attribute__((aligned(16))) float red[NW * G::TSZ + 4];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  KT(0);
  const uint32_t tm = blockIdx.x % p.tiles_m, tn = blockIdx.x / p.tiles_m, split = blockIdx.y;
  const uint32_t m0 = tm * BMr;
  // this wave's share of the block's K chunk (p.ks: a multiple of NW * 16)
  const uint32_t kq = p.ks / NW;
  const uint32_t kw0 = split * p.ks + wave * kq;
  const uint32_t kw1 = min(p.K, kw0 + kq);
  const int i = lane & 15, g = lane >> 4;

  const __amdgpu_buffer_rsrc_t rsa = make_rsrc(p.a, p.a_bytes);
  const __amdgpu_buffer_rsrc_t rsb = make_rsrc(p.b, p.b_bytes);
  // per-lane row offsets of the R row tiles (OOB past M)
  uint32_t arow[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const uint32_t m = m0 + 16 * r + i;
    arow[r] = oob_unless(m < p.M, m * p.lda * 4u);
  }
  // per-lane column state of the C column tiles
  uint32_t bcol[C];
  int iy0[C], ix0[C];
#pragma unroll
  for (int c = 0; c < C; ++c) {
    const uint32_t n = tn * NC + 16 * c + i;
    iy0[c] = 0;
    ix0[c] = 0;
    if constexpr (BLD == B_FC) {
      bcol[c] = oob_unless(n < p.N, n * p.K * 4u);
    } else {
      const uint32_t img = fdiv(n, p.ohw_m, p.ohw_s), pix = n - img * p.OHW;
      if constexpr (BLD == B_IM1X1) {
        bcol[c] = oob_unless(n < p.N, (img * p.ICHW + pix) * 4u);
      } else {
        const uint32_t oy = fdiv(pix, p.ow_m, p.ow_s), ox = pix - oy * p.OW;
        iy0[c] = (int)(oy * p.sy) - (int)p.py;
        ix0[c] = (int)(ox * p.sx) - (int)p.px;
        bcol[c] = (uint32_t)((int)(img * p.ICHW) + iy0[c] * (int)p.W + ix0[c]);
        if (n >= p.N) iy0[c] = -(1 << 29);  // every tap misses
      }
    }
  }
  // column operand of tile c, k = k4 .. k4+3 (k4 % 4 == 0)
  auto load_b = [&](int c, uint32_t k4) -> f32x4t {
    if constexpr (BLD == B_FC) {
      return ld4(rsb, oob_unless(k4 < kw1, bcol[c] + k4 * 4u));
    } else {
      f32x4t v;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint32_t k = k4 + q;
        if constexpr (BLD == B_IM1X1) {
          v[q] = ld1(rsb, oob_unless(k < kw1, bcol[c] + k * p.HW * 4u));
        } else {
          const uint32_t ic = fdiv(k, p.kyx_m, p.kyx_s), rem = k - ic * p.KYX;
          const uint32_t ky = fdiv(rem, p.kx_m, p.kx_s), kx = rem - ky * p.KX;
          const bool ok = (k < kw1) & ((uint32_t)(iy0[c] + (int)ky) < p.H) & ((uint32_t)(ix0[c] + (int)kx) < p.W);
          v[q] = ld1(rsb, oob_unless(ok, (bcol[c] + ic * p.HW + ky * p.W + kx) * 4u));
        }
      }
      return v;
    }
  };

  float bias_r[G::CH];
  gv_bias<R, C, NW>(p, m0, tid, bias_r);

  f32x4t acc[R][C];
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int c = 0; c < C; ++c) acc[r][c] = f32x4t{0.0f, 0.0f, 0.0f, 0.0f};

  // K batches of KB: all of a batch's loads are issued before its MFMAs
  f32x4t a0[NG][R], b0[NG][C], a1[DB ? NG : 1][R], b1[DB ? NG : 1][C];
  auto load_batch = [&](uint32_t kb, f32x4t(&a)[NG][R], f32x4t(&b)[NG][C]) {
#pragma unroll
    for (int gg = 0; gg < NG; ++gg) {
      const uint32_t k4 = kb + 16 * gg + 4 * g;
#pragma unroll
      for (int r = 0; r < R; ++r) a[gg][r] = ld4(rsa, oob_unless(k4 < kw1, arow[r] + k4 * 4u));
#pragma unroll
      for (int c = 0; c < C; ++c) b[gg][c] = load_b(c, k4);
    }
  };
  auto mma_batch = [&](const f32x4t(&a)[NG][R], const f32x4t(&b)[NG][C]) {
#pragma unroll
    for (int gg = 0; gg < NG; ++gg)
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
          for (int c = 0; c < C; ++c)
            acc[r][c] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[gg][r][q], b[gg][c][q], acc[r][c], 0, 0, 0);
  };
  uint32_t kb = kw0;
  if constexpr (DB) {
    if (kb < kw1) load_batch(kb, a0, b0);
    while (kb < kw1) {
      const uint32_t k1 = kb + KB;
      if (k1 < kw1) load_batch(k1, a1, b1);
      mma_batch(a0, b0);
      if (kb == kw0) KT(1);
      if (k1 >= kw1) break;
      const uint32_t k2 = k1 + KB;
      if (k2 < kw1) load_batch(k2, a0, b0);
      mma_batch(a1, b1);
      kb = k2;
    }
  } else {
    for (; kb < kw1; kb += KB) {
      load_batch(kb, a0, b0);
      mma_batch(a0, b0);
      if (kb == kw0) KT(1);
    }
  }

  KT(2);
  gv_finish<R, C, NW, 1>(p, acc, red, tm, tn, tid, wave, lane, bias_r);
}

// Loads of R consecutive floats (R = 1, 2, 4) at a per-lane offset + a scalar offset.
template <int R>
__device__ __forceinline__ typename fvec<R>::t ldv(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
  if constexpr (R == 4)
    return __builtin_bit_cast(f32x4v, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0));
  else if constexpr (R == 2)
    return __builtin_bit_cast(f32x2v, __builtin_amdgcn_raw_buffer_load_b64(r, voff, soff, 0));
  else
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, 0));
}

// gvp_kernel: the register-streaming structure of gv_kernel over the k-major packed bank
// ([Kp][OC4], K order (ky, kx, ic): bh_conv_filts_pack, the xpose_filts role) for convs with
// IC % 16 == 0, where every 16-deep k group lies inside one filter tap. gv_kernel's im2col
// gather spends ~20 VALU per element on (ic, ky, kx) divisions and range checks; on a small op
// that instruction stream IS the latency (a wave issues about one instruction per 4 clocks:
// tools/lat_bench.hip). Here nothing per element is vector work:
//  * A: MFMA step s of group gg takes packed row k = k16 + 4 s + g; one R-wide load per lane
//    holds that row's entries for output channels m0 + R i .. m0 + R i + R - 1, so row rho of
//    MFMA row tile r is block row R rho + r (gv_finish RS = R); the lane's channel offset is
//    its VGPR address, the row offset (k16 + 4 s) * OC4 the instruction's scalar soffset;
//  * B_IMTAP: the group's tap (ky, kx) and first channel ic0 are scalars; per column tile ONE
//    per-lane offset (its input pixel at that tap, or a miss in the padding / past N) serves the
//    group's four loads, whose channel offsets (ic0 + 4 s + g) * HW differ by scalar soffsets
//    (the g part is folded into the lane's base); B_IM1X1S: the lane's pixel + the same
//    scalar channel offsets;
//  * a group past the wave's K range reads misses on both operands (one select per group).
// The MFMA k map (step s, lane group g -> k16 + 4 s + g) is the same for A and B.
// PD > 0: instead of batches, a ring of PD + 1 single-group register buffers -- the loads of
// group g + PD are issued before group g's MFMAs, so PD groups of loads are always in flight
// (the batch form with DB = 0 exposes a whole memory round trip per batch; DB = 1 doubles its
// registers)
// CX = C (2 or 4, 1x1 only, OH*OW % CX == 0): the C column tiles are interleaved, so a lane's
// CX consecutive pixels are ONE CX-wide load per k (column i of tile c = pixel CX * i + c):
// a quarter / half of the B load instructions -- on small ops the loads a CU must issue
// through its address unit, not their bytes, set the time to the first MFMA
template <int R, int C, int NW, int NG, int DB, int BLD, int PD = 0, int CX = 1>
__global__ __launch_bounds__(NW * 64) void gvp_kernel(GemmArgs p) {
  // B_IM1X1 here: a 1x1 conv reading the bank in its reference layout (no packed bank): A rows
  // of 16-B loads along k (lane group g holds k = k16 + 4 g .. + 3, step s takes k16 + 4 g + s:
  // a quarter of the packed form's A loads at R = 1), B as B_IM1X1S with that k map
  // B_FC: an ipconv (window = whole input, OH = OW = 1, K % 16 == 0) over the reference-layout
  // bank: A as B_IM1X1, B = in[n * K + k] one 16-B load per column tile along the same k map
  static_assert(BLD == B_IMTAP || BLD == B_IM1X1S || BLD == B_IM1X1 || BLD == B_FC,
                "gvp loaders: one-tap im2col, 1x1 or ipconv");
  constexpr bool AO = BLD == B_IM1X1 || BLD == B_FC;
  static_assert(CX == 1 || (CX == C && (CX == 2 || CX == 4) && BLD != B_IMTAP), "column interleave: 1x1, CX == C");
  using G = gv_geom<R, C, NW>;
  constexpr int BMr = G::BMr, NC = G::NC, KB = 16 * NG;
  typedef typename fvec<R>::t av_t;
  __shared__ __attribute__((aligned(16))) float red[NW * G::TSZ + 4];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  KT(0);
  const uint32_t tm = blockIdx.x % p.tiles_m, tn = blockIdx.x / p.tiles_m, split = blockIdx.y;
  const uint32_t m0 = tm * BMr;
  // this wave's share of the block's K chunk (p.ks: a multiple of NW * 16)
  const uint32_t kq = p.ks / NW;
  const uint32_t kw0 = split * p.ks + wave * kq;
  const uint32_t kw1 = min(p.K, kw0 + kq);
  const int i = lane & 15, g = lane >> 4;
  const __amdgpu_buffer_rsrc_t rsa = make_rsrc(p.a, p.a_bytes);
  const __amdgpu_buffer_rsrc_t rsb = make_rsrc(p.b, p.b_bytes);
  const uint32_t lda4 = p.lda * 4u, hw4 = p.HW * 4u;
  // A: channels m0 + R i .. (one R-aligned group of the OC4-padded row, or all past it)
  const uint32_t arow = oob_unless(m0 + R * i < p.lda, (m0 + R * i) * 4u + g * lda4);
  uint32_t arow_o[AO ? R : 1];  // AO: row m0 + 16 r + i, k offset 4 g
#pragma unroll
  for (int r = 0; r < (AO ? R : 1); ++r) {
    const uint32_t m = m0 + 16 * r + i;
    arow_o[r] = oob_unless(m < p.M, (m * p.lda + 4 * g) * 4u);
  }
  // B: per column tile, the lane's input pixel for channel g at tap (0, 0)
  uint32_t bcol[C];
  int iy0[C], ix0[C];
#pragma unroll
  for (int c = 0; c < C; ++c) {
    const uint32_t n = CX > 1 ? tn * NC + CX * i : tn * NC + 16 * c + i;  // CX > 1: the lane's run
    const uint32_t img = fdiv(n, p.ohw_m, p.ohw_s), pix = n - img * p.OHW;
    iy0[c] = 0;
    ix0[c] = 0;
    if constexpr (BLD == B_FC) {
      bcol[c] = oob_unless(n < p.N, (n * p.ICHW + 4 * g) * 4u);
    } else if constexpr (BLD == B_IM1X1S || AO) {
      bcol[c] = oob_unless(n < p.N, (img * p.ICHW + pix + (AO ? 4 * g : g) * p.HW) * 4u);
    } else {
      const uint32_t oy = fdiv(pix, p.ow_m, p.ow_s), ox = pix - oy * p.OW;
      iy0[c] = (int)(oy * p.sy) - (int)p.py;
      ix0[c] = (int)(ox * p.sx) - (int)p.px;
      bcol[c] = (uint32_t)((int)(img * p.ICHW + g * p.HW) + iy0[c] * (int)p.W + ix0[c]);
      if (n >= p.N) iy0[c] = -(1 << 29);  // every tap misses
    }
  }

  float bias_r[G::CH];
  gv_bias<R, C, NW>(p, m0, tid, bias_r);

  f32x4t acc[R][C];
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int c = 0; c < C; ++c) acc[r][c] = f32x4t{0.0f, 0.0f, 0.0f, 0.0f};

  // loads of the 16-deep k group at k16 into one group buffer (misses past the wave's range)
  auto load_grp = [&](uint32_t k16, av_t(&a)[4], float(&b)[4][C]) {
    const bool live = k16 < kw1;  // wave-uniform
    const uint32_t av = live ? arow : OOB;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      if constexpr (!AO) a[s] = ldv<R>(rsa, av, (k16 + 4 * s) * lda4);
    }
    if constexpr (AO) {
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const f32x4v v = ld4(rsa, live ? arow_o[r] + k16 * 4u : OOB);
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          if constexpr (R == 1) a[s] = v[s];
          else a[s][r] = v[s];
        }
      }
    }
    uint32_t bv[C];
    uint32_t c0 = k16;
    if constexpr (BLD == B_IM1X1S || AO) {
#pragma unroll
      for (int c = 0; c < C; ++c) bv[c] = live ? bcol[c] : OOB;
    } else {
      const uint32_t kyx = fdiv(k16, p.ic_m, p.ic_s);
      const uint32_t ky = fdiv(kyx, p.kx_m, p.kx_s), kx = kyx - ky * p.KX;
      c0 = k16 - kyx * p.IC;
#pragma unroll
      for (int c = 0; c < C; ++c) {
        const bool ok = live & ((uint32_t)(iy0[c] + (int)ky) < p.H) & ((uint32_t)(ix0[c] + (int)kx) < p.W);
        bv[c] = oob_unless(ok, (uint32_t)((int)bcol[c] + (int)(ky * p.W + kx)) * 4u);
      }
    }
    if constexpr (BLD == B_FC) {
#pragma unroll
      for (int c = 0; c < C; ++c) {
        const f32x4v v = ld4(rsb, live ? bcol[c] + k16 * 4u : OOB);
#pragma unroll
        for (int s = 0; s < 4; ++s) b[s][c] = v[s];
      }
    } else if constexpr (CX > 1) {
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const typename fvec<CX>::t v = ldv<CX>(rsb, bv[0], (AO ? c0 + s : c0 + 4 * s) * hw4);
#pragma unroll
        for (int c = 0; c < C; ++c) b[s][c] = v[c];
      }
    } else {
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int c = 0; c < C; ++c)
        b[s][c] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rsb, bv[c], (AO ? c0 + s : c0 + 4 * s) * hw4, 0));
    }
  };
  auto mma_grp = [&](const av_t(&a)[4], const float(&b)[4][C]) {
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int r = 0; r < R; ++r)
#pragma unroll
        for (int c = 0; c < C; ++c)
          acc[r][c] = __builtin_amdgcn_mfma_f32_16x16x4f32(vget<R>(a[s], r), b[s][c], acc[r][c], 0, 0, 0);
  };
  if constexpr (PD > 0) {
    constexpr int RING = PD + 1;
    av_t ra[RING][4];
    float rb[RING][4][C];
#pragma unroll
    for (int r = 0; r < PD; ++r) load_grp(kw0 + 16u * r, ra[r], rb[r]);
    // whole trips of RING groups (no exits inside: the loop head sees the same PD groups in
    // flight from the prologue and from the back edge, so the waits stay counted), then a tail
    auto step = [&](int r, uint32_t kc) {
      // pinned order: the prefetch loads, then this group's MFMAs (else hipcc interleaves them
      // and waits on the prefetch)
      __builtin_amdgcn_sched_barrier(0);
      load_grp(kc + 16u * PD, ra[(r + PD) % RING], rb[(r + PD) % RING]);
      __builtin_amdgcn_sched_barrier(0);
      mma_grp(ra[r % RING], rb[r % RING]);
      __builtin_amdgcn_sched_barrier(0);
    };
    const uint32_t ngrp = kw1 > kw0 ? (kw1 - kw0 + 15) / 16 : 0;
    uint32_t k = kw0, g = 0;
    for (; g + RING <= ngrp; g += RING, k += 16u * RING) {
#pragma unroll
      for (int r = 0; r < RING; ++r) step(r, k + 16u * r);
      if (g == 0) KT(1);
    }
    // tail: < RING groups left, all already in flight -- MFMAs only (no dead prefetches)
#pragma unroll
    for (int r = 0; r < RING - 1; ++r)
      if (g + r < ngrp) {
        __builtin_amdgcn_sched_barrier(0);
        mma_grp(ra[r % RING], rb[r % RING]);
      }
  } else {
  av_t a0[NG][4], a1[DB ? NG : 1][4];
  float b0[NG][4][C], b1[DB ? NG : 1][4][C];
  auto load_batch = [&](uint32_t kb, av_t(&a)[NG][4], float(&b)[NG][4][C]) {
#pragma unroll
    for (int gg = 0; gg < NG; ++gg) load_grp(kb + 16 * gg, a[gg], b[gg]);
  };
  auto mma_batch = [&](const av_t(&a)[NG][4], const float(&b)[NG][4][C]) {
#pragma unroll
    for (int gg = 0; gg < NG; ++gg) mma_grp(a[gg], b[gg]);
  };
  uint32_t kb = kw0;
  if constexpr (DB) {
    if (kb < kw1) load_batch(kb, a0, b0);
    while (kb < kw1) {
      const uint32_t k1 = kb + KB;
      if (k1 < kw1) load_batch(k1, a1, b1);
      mma_batch(a0, b0);
      if (kb == kw0) KT(1);
      if (k1 >= kw1) break;
      const uint32_t k2 = k1 + KB;
      if (k2 < kw1) load_batch(k2, a0, b0);
      mma_batch(a1, b1);
      kb = k2;
    }
  } else {
    for (; kb < kw1; kb += KB) {
      load_batch(kb, a0, b0);
      mma_batch(a0, b0);
      if (kb == kw0) KT(1);
    }
  }

  }

  KT(2);
  gv_finish<R, C, NW, AO ? 1 : R, CX>(p, acc, red, tm, tn, tid, wave, lane, bias_r);
}

template <int R, int C, int NW, int NG, int DB>
cfg_t gv_cfg(const char *name) {
  cfg_t c{name, 16 * R, 16 * C, 16 * NW, NW * 64, {}, 0};  // BK: K granule of a block chunk
  c.gv = 1;
  c.k[A_MVEC][B_FC][0] = gv_kernel<R, C, NW, NG, DB, B_FC>;
  c.k[A_MVEC][B_IM1X1][0] = gv_kernel<R, C, NW, NG, DB, B_IM1X1>;
  c.k[A_MVEC][B_IM2COL][0] = gv_kernel<R, C, NW, NG, DB, B_IM2COL>;
  return c;
}

// fcv_kernel: ipconv / FC ops at batch N <= NB (a matrix-vector product per image): the op is
// one read of the bank, and the MFMA tiles waste 15/16 of their columns at N = 1 while their
// operand loads cover 16 rows x 64 B each. Here a wave owns R output channels (bank rows) and
// streams them along k, one 16-B piece per lane -- each load instruction is 1 KB of ONE row, as
// the contiguous stream that reaches HBM peak in tools/lat_bench.hip -- with U pieces per row
// in flight; the N input rows come in the same k pieces (L2-resident: K * N * 4 bytes), the
// products are summed per lane (fmaf chain over the lane's k, in k order), then across the wave
// by a butterfly, and R x N lanes store the results (bias, residual, ReLU as finish_store_b).
template <int R, int U, int NB>
__global__ __launch_bounds__(256) void fcv_kernel(GemmArgs p) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t m0 = (blockIdx.x * 4u + (uint32_t)wave) * R;
  const __amdgpu_buffer_rsrc_t rsa = make_rsrc(p.a, p.a_bytes);
  const __amdgpu_buffer_rsrc_t rsb = make_rsrc(p.b, p.b_bytes);
  const uint32_t K = p.K;
  uint32_t wrow[R], xrow[NB];
#pragma unroll
  for (int r = 0; r < R; ++r) wrow[r] = m0 + r < p.M ? (m0 + r) * K * 4u + 16u * lane : OOB;
#pragma unroll
  for (int b = 0; b < NB; ++b) xrow[b] = (uint32_t)b < p.N ? (uint32_t)b * p.ICHW * 4u + 16u * lane : OOB;
  float acc[R][NB];
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int b = 0; b < NB; ++b) acc[r][b] = 0.0f;
  for (uint32_t kc = 0; kc < K; kc += 256u * U) {
    f32x4v w[U][R], x[U][NB];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const bool live = kc + 256u * u + 4u * lane < K;  // (K % 4 == 0: a piece is whole or past the row)
      const uint32_t ko = (kc + 256u * u) * 4u;
#pragma unroll
      for (int r = 0; r < R; ++r) w[u][r] = ld4(rsa, live ? wrow[r] + ko : OOB);
#pragma unroll
      for (int b = 0; b < NB; ++b) x[u][b] = ld4(rsb, live ? xrow[b] + ko : OOB);
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int r = 0; r < R; ++r)
#pragma unroll
        for (int b = 0; b < NB; ++b)
#pragma unroll
          for (int e = 0; e < 4; ++e) acc[r][b] = __builtin_fmaf(w[u][r][e], x[u][b][e], acc[r][b]);
  }
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) acc[r][b] += __shfl_xor(acc[r][b], o, 64);
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const uint32_t m = m0 + r;
      if (lane == r * NB + b && m < p.M && (uint32_t)b < p.N) {
        const size_t o = (size_t)b * p.OCOHW + m;
        float v = acc[r][b] + (p.bias ? p.bias[m] : 0.0f);
        if (p.res) v += p.res[o];
        out_elem1(p, o, (p.relu && v < 0.0f) ? 0.0f : v);
      }
    }
}

template <int R, int U, int NB>
cfg_t fcv_cfg(const char *name) {
  cfg_t c{name, 4 * R, NB, 256 * U, 256, {}, 0};
  c.gv = 1;
  c.fcv = 1;
  c.k[A_MVEC][B_FC][0] = fcv_kernel<R, U, NB>;
  return c;
}

// gvo configurations: 1x1 convs over the bank in its reference layout (no pack), IC % 16 == 0
template <int R, int C, int NW, int PD, int CX = 1>
cfg_t gvo_cfg(const char *name) {
  cfg_t c{name, 16 * R, 16 * C, 16 * NW, NW * 64, {}, 0};
  c.gv = 1;
  c.gv_cx = CX;
  c.k[A_MVEC][B_IM1X1S][0] = gvp_kernel<R, C, NW, 1, 0, B_IM1X1, PD, CX>;
  if constexpr (CX == 1) c.k[A_MVEC][B_FC][0] = gvp_kernel<R, C, NW, 1, 0, B_FC, PD>;
  return c;
}
// gvs over the packed bank with interleaved column tiles (1x1 only)
template <int R, int C, int NW, int PD, int CX>
cfg_t gvx_cfg(const char *name) {
  cfg_t c{name, 16 * R, 16 * C, 16 * NW, NW * 64, {}, 1};
  c.gv = 1;
  c.gv_cx = CX;
  c.k[A_KVEC][B_IM1X1S][0] = gvp_kernel<R, C, NW, 1, 0, B_IM1X1S, PD, CX>;
  return c;
}

// gvp configurations: the packed bank (packA), IC % 16 == 0 (launch_conv refuses others)
template <int R, int C, int NW, int NG, int DB, int PD = 0>
cfg_t gvp_cfg(const char *name) {
  cfg_t c{name, 16 * R, 16 * C, 16 * NW, NW * 64, {}, 1};
  c.gv = 1;
  c.k[A_KVEC][B_IMTAP][0] = gvp_kernel<R, C, NW, NG, DB, B_IMTAP, PD>;
  c.k[A_KVEC][B_IM1X1S][0] = gvp_kernel<R, C, NW, NG, DB, B_IM1X1S, PD>;
  return c;
}

}  // namespace

std::vector<cfg_t> gv_cfgs() {
  return {
      // filter streaming (few columns, big banks)
      gv_cfg<4, 1, 4, 4, 1>("gv64x16"),
      gv_cfg<4, 2, 4, 4, 1>("gv64x32"),
      gv_cfg<2, 4, 4, 4, 1>("gv32x64"),
      gv_cfg<2, 2, 4, 4, 1>("gv32x32"),
      // latency configurations for small ops: 8 or 16 waves split K inside a block, so the
      // whole K of a small op is in flight in one or two memory round trips
      gv_cfg<2, 2, 8, 4, 1>("gv32x32w8"),
      gv_cfg<2, 2, 16, 2, 0>("gv32x32w16"),
      gv_cfg<4, 2, 8, 2, 1>("gv64x32w8"),
      gv_cfg<2, 4, 8, 2, 1>("gv32x64w8"),
      gv_cfg<4, 4, 8, 2, 0>("gv64x64w8"),
      gv_cfg<4, 4, 4, 2, 0>("gv64x64"),
      // small output tiles: more blocks (CUs) share a small op's loads
      gv_cfg<1, 1, 4, 4, 1>("gv16x16"),
      gv_cfg<1, 1, 8, 4, 1>("gv16x16w8"),
      gv_cfg<1, 2, 8, 4, 1>("gv16x32w8"),
      gv_cfg<2, 1, 8, 4, 1>("gv32x16w8"),
      // 16 waves: twice the loads in flight per CU for the smallest ops
      gv_cfg<1, 1, 16, 2, 1>("gv16x16w16"),
      gv_cfg<1, 2, 16, 2, 0>("gv16x32w16"),
      gv_cfg<2, 1, 16, 2, 0>("gv32x16w16"),
      // over the packed bank with scalar-offset loaders (IC % 16 == 0)
      gvp_cfg<1, 1, 4, 4, 1>("gvp16x16"),
      gvp_cfg<1, 1, 8, 4, 1>("gvp16x16w8"),
      gvp_cfg<1, 1, 16, 2, 1>("gvp16x16w16"),
      gvp_cfg<1, 2, 8, 4, 1>("gvp16x32w8"),
      gvp_cfg<1, 2, 16, 2, 0>("gvp16x32w16"),
      gvp_cfg<2, 1, 8, 4, 1>("gvp32x16w8"),
      gvp_cfg<2, 1, 16, 2, 0>("gvp32x16w16"),
      gvp_cfg<2, 2, 4, 4, 1>("gvp32x32"),
      gvp_cfg<2, 2, 8, 4, 1>("gvp32x32w8"),
      gvp_cfg<2, 2, 16, 2, 0>("gvp32x32w16"),
      gvp_cfg<4, 1, 4, 4, 1>("gvp64x16"),
      gvp_cfg<4, 2, 8, 2, 1>("gvp64x32w8"),
      gvp_cfg<2, 4, 8, 2, 1>("gvp32x64w8"),
      gvp_cfg<4, 4, 8, 2, 0>("gvp64x64w8"),
      // the same with a ring of single-group buffers, PD groups of loads in flight
      gvp_cfg<4, 4, 8, 1, 0, 2>("gvs64x64w8"),
      gvp_cfg<4, 4, 4, 1, 0, 3>("gvs64x64"),
      gvp_cfg<4, 2, 8, 1, 0, 2>("gvs64x32w8"),
      gvp_cfg<2, 4, 8, 1, 0, 2>("gvs32x64w8"),
      gvp_cfg<2, 2, 8, 1, 0, 3>("gvs32x32w8"),
      gvp_cfg<2, 2, 16, 1, 0, 2>("gvs32x32w16"),
      gvp_cfg<2, 1, 16, 1, 0, 2>("gvs32x16w16"),
      gvp_cfg<1, 1, 16, 1, 0, 2>("gvs16x16w16"),
      gvp_cfg<1, 1, 8, 1, 0, 3>("gvs16x16w8"),
      gvp_cfg<4, 2, 16, 1, 0, 2>("gvs64x32w16"),
      gvp_cfg<2, 4, 16, 1, 0, 2>("gvs32x64w16"),
      gvp_cfg<4, 2, 8, 1, 0, 3>("gvs64x32w8p3"),
      gvp_cfg<4, 4, 8, 1, 0, 1>("gvs64x64w8p1"),
      gvp_cfg<4, 1, 16, 1, 0, 2>("gvs64x16w16"),
      gvp_cfg<1, 2, 16, 1, 0, 2>("gvs16x32w16"),
      gvp_cfg<4, 2, 4, 1, 0, 3>("gvs64x32"),
      // 1x1 over the reference-layout bank (16-B A loads along k)
      gvo_cfg<1, 1, 8, 3>("gvo16x16w8"),
      gvo_cfg<1, 1, 16, 2>("gvo16x16w16"),
      gvo_cfg<1, 2, 16, 2>("gvo16x32w16"),
      gvo_cfg<2, 1, 16, 2>("gvo32x16w16"),
      gvo_cfg<2, 2, 8, 3>("gvo32x32w8"),
      gvo_cfg<2, 2, 16, 2>("gvo32x32w16"),
      gvo_cfg<4, 2, 8, 2>("gvo64x32w8"),
      gvo_cfg<4, 2, 16, 2>("gvo64x32w16"),
      gvo_cfg<2, 4, 8, 2>("gvo32x64w8"),
      // batch-streaming ipconv (batch <= 1 / 2 / 4; batch-5 variants measured slower than gv)
      fcv_cfg<2, 8, 1>("fcv2u8n1"),
      fcv_cfg<4, 4, 1>("fcv4u4n1"),
      fcv_cfg<1, 16, 1>("fcv1u16n1"),
      fcv_cfg<2, 4, 2>("fcv2u4n2"),
      fcv_cfg<4, 4, 4>("fcv4u4n4"),
      // interleaved column tiles: one 8-B / 16-B pixel-run load per k (1x1, OH*OW % CX == 0)
      gvo_cfg<1, 4, 8, 3, 4>("gvo16x64xw8"),
      gvo_cfg<1, 4, 16, 2, 4>("gvo16x64xw16"),
      gvo_cfg<1, 2, 16, 2, 2>("gvo16x32xw16"),
      gvo_cfg<2, 4, 8, 2, 4>("gvo32x64xw8"),
      gvo_cfg<2, 2, 16, 2, 2>("gvo32x32xw16"),
      gvx_cfg<4, 4, 8, 2, 4>("gvs64x64xw8"),
      gvx_cfg<2, 4, 16, 2, 4>("gvs32x64xw16"),
      gvx_cfg<4, 2, 16, 2, 2>("gvs64x32xw16"),
  };
}

}  // namespace bhk
