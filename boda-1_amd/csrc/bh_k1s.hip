// bh_k1s.hip -- 1x1 convolutions over many pixels with the filter bank resident in LDS and the
// input streamed straight into registers (Boda's k1conv role: test/rtc/k1conv.cucl, chosen at
// src/cnn_op.cc:51-58).
//
// A 1x1 conv is one GEMM per image, out[oc][p] = bias[oc] + sum_ic W[oc][ic] in[ic][p], with
// few channels (K = IC <= a few hundred) and many pixels: the op streams the input and output
// (HBM) and its MFMA work is of the same order, so nothing may stand between the two streams.
// The tile kernels re-fetch the bank per pixel tile, split K, stage the input through LDS and
// synchronise their waves at every stage (bh_dcm.hip's 1x1 mode: 0.32-0.36 of roofline on the
// conv set's batch-20 1x1 ops). Here:
//  * a block owns one OC tile of OCT = 32*TM output channels for its whole life: its slice of
//    the k-major packed bank (bh_conv_filts_pack, [K][OC4]), rows [IC][OCT], is DMA'd into LDS
//    once (16-B pieces, chunk by chunk along with the first unit's input, a barrier per chunk
//    in that unit only); lane li computes channels li + 32 t: one ds_read_b32 per tile and step;
//  * a wave owns a unit of 32 consecutive pixels of the flattened (image, pixel) space x the
//    block's OCT channels x the whole K: v_mfma_f32_32x32x2_f32 with A = the input (lane li's
//    pixel, channel 2s + lane/32: one dword load per lane per k step, 2 x 128 contiguous bytes
//    per wave instruction, straight into the operand register), B = the resident bank;
//  * the loads run Q-1 chunks of KC channels ahead through a register ring (vmcnt-counted, no
//    drains), across unit boundaries: a wave never waits for its next unit's first loads; the
//    waves of a block never synchronise after the prologue (no barrier, no split-K, no slabs);
//  * the epilogue stores float4 pixel quads (bias, residual, ReLU) straight from the
//    accumulators: lane (li, h) holds channel li + 32 t, pixels 8g + 4h .. + 3 of its unit.
// Blocks b, b + 8, ... share an XCD under round-robin placement; the blocks of one XCD cover all
// OC tiles of the same pixel units, so an input unit read by several OC tiles is re-read from
// that XCD's L2.
// Same GemmArgs contract as the other conv kernels: a = packed bank, lda = OC4, b = input,
// OCOHW = the output's image stride (channel-slab outputs work), tiles_m = OC tiles.
#include "bh_gemm_dev.h"

namespace bhk {
namespace {

// DBG (diagnostic builds in the instrumented library only; wrong results by design): bit 0 = no
// input loads after the prologue, bit 1 = no MFMA, bit 2 = no output stores (dropped instead)
template <int TM, int KC, int Q, int NW, int DBG = 0>
__global__ __launch_bounds__(NW * 64) void k1s_kernel(GemmArgs p) {
  constexpr int OCT = 32 * TM;           // output channels of the block (LDS floats per bank row)
  constexpr int SC = KC / 2;             // k steps (and input loads per lane) per chunk
  constexpr int S = 4 * TM;              // float4 stores per lane per unit
  constexpr int PF = 3;                  // LDS fragment prefetch (steps)
  constexpr int WPC = KC * OCT / 4;      // 16-B bank pieces per chunk
  constexpr int LWC = (WPC + NW * 64 - 1) / (NW * 64);  // bank DMA instructions per lane per chunk
  static_assert(TM >= 1 && TM <= 4 && KC % 2 == 0, "tile");
  static_assert(Q >= 2 && (Q - 1) * SC + S <= 63, "vmcnt range");
  static_assert(SC % (PF + 1) == 0, "fragment ring period divides a chunk");
  constexpr int SP = 36;                 // staging tile pitch (floats): 32 pixels + 4
  // the bank slice [IC][OCT] (packed-bank rows oc0 ..), then each wave's epilogue tile [32][SP]
  extern __shared__ __attribute__((aligned(16))) float wl[];

  const int tid = threadIdx.x, lane = tid & 63, li = lane & 31, kh = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  KT(0);
  // block -> (OC tile, index among the blocks of that tile); tiles_m = OC tiles, gridDim.x a
  // multiple of 8 * tiles_m
  const uint32_t l8 = blockIdx.x >> 3;
  const uint32_t oct = l8 % p.tiles_m;
  const uint32_t gi = (l8 / p.tiles_m) * 8 + (blockIdx.x & 7);
  const uint32_t wg = (gridDim.x / p.tiles_m) * NW;  // waves per OC tile
  const uint32_t oc0 = oct * OCT;
  const uint32_t npu = (p.N + 31) / 32, nch = p.K / KC;
  const uint32_t lds_w = p.K * OCT;  // floats of the bank slice
  const uint32_t hw4 = p.HW * 4u;

  const __amdgpu_buffer_rsrc_t rsw = make_rsrc(p.a, p.a_bytes);
  const __amdgpu_buffer_rsrc_t rsx = make_rsrc(p.b, p.b_bytes);
  const __amdgpu_buffer_rsrc_t rso = make_rsrc(p.c, p.c_bytes);
  const __amdgpu_buffer_rsrc_t rsbias = make_rsrc(p.bias, p.bias ? p.M * 4u : 0u);

  // lane (li, kh) computes output channels oc0 + li + 32 t (t < TM): B fragment of tile t at
  // step s is bank row 2s + kh, column li + 32 t -- one ds_read_b32 per tile and step
  float bias[TM];
#pragma unroll
  for (int t = 0; t < TM; ++t) {
    const uint32_t oc = oc0 + li + 32 * t;
    bias[t] = ld1(rsbias, oob_unless(oc < p.M, oc * 4u));
  }
  // the bank slice [IC][OCT] comes in with the first unit's chunks: 16-B pieces of packed-bank
  // row k, columns oc0 + 4 q .. (OC4-padded rows: columns past OC4 miss); piece e of a chunk
  // (lanes past the chunk's pieces write nothing: the next chunk's rows may already have landed.
  // No wait ever counts on these DMAs -- they only add younger operations -- so a wave that
  // issues fewer of them keeps every wait correct)
  uint32_t wsrc[LWC];
#pragma unroll
  for (int j = 0; j < LWC; ++j) {
    const uint32_t e = (uint32_t)((j * NW + wave) * 64 + lane), r = e / (OCT / 4), q = e % (OCT / 4);
    wsrc[j] = e < (uint32_t)WPC ? oob_unless(oc0 + 4 * q < p.lda, (r * p.lda + oc0 + 4 * q) * 4u) : 0xffffffffu;
  }
  auto issue_w = [&](uint32_t c) {  // chunk c's bank rows (the whole K of them stays resident)
#pragma unroll
    for (int j = 0; j < LWC; ++j)
      if (wsrc[j] != 0xffffffffu)
        dma16s(rsw, wl + (size_t)c * KC * OCT + (j * NW + wave) * 256, wsrc[j], c * KC * p.lda * 4u);
  };
  // per-lane input offset of unit pu (pixel pu*32 + li, channel kh); past the op: misses
  auto ubase = [&](uint32_t pu) -> uint32_t {
    const uint32_t n = pu * 32 + li;
    const uint32_t img = fdiv(n, p.ohw_m, p.ohw_s), pix = n - img * p.OHW;
    return oob_unless((pu < npu) & (n < p.N), (img * p.ICHW + pix + kh * p.HW) * 4u);
  };
  float xr[Q][SC];
  // chunk c of a unit: the chunk offset goes into the lane's VGPR offset (a miss stays a miss:
  // OOB + c * KC * HW * 4 < 2^32), step s's channel pair into the scalar soffset (SC values shared
  // by every chunk: few SGPRs)
  auto issue = [&](int q, uint32_t base, uint32_t c) {
    const uint32_t vb = (DBG & 1) ? OOB : base + c * KC * hw4;
#pragma unroll
    for (int s = 0; s < SC; ++s)
      xr[q][s] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rsx, vb, 2 * s * hw4, 0));
  };
  uint32_t pu = gi * NW + wave;
  uint32_t bcur = ubase(pu), bnext = ubase(pu + wg);
#pragma unroll
  for (int q = 0; q < Q - 1; ++q) {
    issue_w(q);
    issue(q, bcur, q);
  }
  // S dropped stores: the loop's waits count a unit's epilogue stores behind the first chunks
  // of the next unit, and the first unit has the same VMEM sequence (its bank DMAs only add
  // younger operations: those waits are stricter than needed)
#pragma unroll
  for (int s = 0; s < S; ++s) __builtin_amdgcn_raw_buffer_store_b32(0u, rso, OOB, 0, 0);

  f32x16 acc[TM];
  float wf[PF + 1][TM];
  const float *const wb = wl + kh * OCT + li;  // bank row kh, column li, this lane
  auto frag = [&](float (&w)[TM], uint32_t c, int s) {
#pragma unroll
    for (int t = 0; t < TM; ++t) w[t] = wb[(c * KC + 2 * s) * OCT + 32 * t];
  };

  // chunk c = cq + r (slot r % Q) of the current unit: wait for its loads (first unit: and for
  // every wave's bank DMA of the chunk), put chunk c + Q - 1 (of this unit or the next) in flight,
  // MFMAs with the fragments PF steps ahead (the first unit reads the next chunk's fragments only
  // after the next barrier)
  auto chunk = [&](int r, uint32_t cq, bool first, bool u0) {
    if (first && r < Q - 1) vm_wait<(Q - 2) * SC + S>();
    else vm_wait<(Q - 2) * SC>();
    if (u0) {
      __syncthreads();
#ifdef BH_KTRACE
      if (cq == 0 && r == 0) KT(1);
#endif
#pragma unroll
      for (int s = 0; s < PF; ++s) frag(wf[s], cq + r, s);
    }
    __builtin_amdgcn_sched_barrier(0);
    {
      const uint32_t c2 = cq + (uint32_t)(r + Q - 1);
      const bool nx = c2 >= nch;
      if (u0 && !nx) issue_w(c2);
      issue((r + Q - 1) % Q, nx ? bnext : bcur, nx ? c2 - nch : c2);
    }
    __builtin_amdgcn_sched_barrier(0);
    const uint32_t c = cq + (uint32_t)r, cn = c + 1 == nch ? 0u : c + 1;
#pragma unroll
    for (int s = 0; s < SC; ++s) {
      if (s + PF < SC) frag(wf[(s + PF) % (PF + 1)], c, s + PF);
      else if (!u0) frag(wf[(s + PF) % (PF + 1)], cn, s + PF - SC);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int t = 0; t < TM; ++t) {
        if constexpr ((DBG & 2) != 0) acc[t][s] += xr[r % Q][s] * wf[s % (PF + 1)][t];
        else acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(xr[r % Q][s], wf[s % (PF + 1)][t], acc[t], 0, 0, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  const bool vec_ok = !p.res;
  // unit loop; the first pass runs in every wave (a wave without a unit computes on misses and
  // stores nothing) so that all waves meet the first unit's per-chunk barriers
  for (bool u0 = true;; u0 = false) {
#pragma unroll
    for (int t = 0; t < TM; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[t][r] = 0.0f;
    if (u0) {
#pragma unroll
      for (int r = 0; r < Q; ++r) chunk(r, 0, true, true);
      for (uint32_t cq = Q; cq < nch; cq += Q) {
#pragma unroll
        for (int r = 0; r < Q; ++r) chunk(r, cq, false, true);
      }
      // the whole bank is resident from here on: fragments of the next unit's first steps
#pragma unroll
      for (int s = 0; s < PF; ++s) frag(wf[s], 0, s);
    } else {
#pragma unroll
      for (int r = 0; r < Q; ++r) chunk(r, 0, true, false);
      for (uint32_t cq = Q; cq < nch; cq += Q) {
#pragma unroll
        for (int r = 0; r < Q; ++r) chunk(r, cq, false, false);
      }
    }
#ifdef BH_KTRACE
    if (u0) KT(2);
#endif
    // epilogue, staged per OC tile through the wave's own LDS tile [32 oc][32 px] (no barrier):
    // lane (li, kh) holds channel oc0 + li + 32 t, pixels pu*32 + 8g + 4kh + e; read back, lane L
    // holds channel row 8j + L/8 of the tile, pixels 4 (L % 8) .. + 3, so a store instruction
    // writes 8 output rows x 128 contiguous bytes (not 32 rows x 32 B: 4x the line fragments)
    {
      const uint32_t q4 = 4u * (uint32_t)(lane & 7), rr = (uint32_t)(lane >> 3);
      const uint32_t n = pu * 32 + q4;  // this lane's first pixel after the transpose
      const uint32_t img = fdiv(n, p.ohw_m, p.ohw_s), pix = n - img * p.OHW;
      const bool quad = vec_ok & (pix + 4 <= p.OHW) & (n < p.N) & (pu < npu);
      const uint32_t obase = img * p.OCOHW + pix;
      float *const st = wl + lds_w + wave * (32 * SP);
#pragma unroll
      for (int t = 0; t < TM; ++t) {
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          f32x4v v;
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = acc[t][4 * g + e];
          *(f32x4v *)(st + li * SP + 8 * g + 4 * kh) = v;
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const uint32_t r = 8u * j + rr, oc = oc0 + 32u * t + r;
          f32x4v v = *(const f32x4v *)(st + r * SP + q4);
          const float bb = __shfl(bias[t], (int)r);  // bias of channel row r (held by lane r)
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] += bb;
          const uint32_t o = oob_unless((oc < p.M) & (pu < npu), (obase + oc * p.OHW) * 4u);
          f32x4v y = v;
#pragma unroll
          for (int e = 0; e < 4; ++e) y[e] = (p.relu && y[e] < 0.0f) ? 0.0f : y[e];
          // always issued (dropped where the quad goes element by element): every unit has at
          // least S vector stores, which the loop's waits count on
          out_store4(p, rso, quad && (DBG & 4) == 0 ? o : OOB, y);
          if (!quad && (oc < p.M) && (pu < npu)) {
            // a quad past its image or the op, or a residual epilogue: element by element (more
            // VMEM instructions than counted only make the waits stricter)
            const __amdgpu_buffer_rsrc_t rsr = make_rsrc(p.res, p.res ? p.c_bytes : 0u);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const uint32_t ne = n + e;
              const uint32_t ie = fdiv(ne, p.ohw_m, p.ohw_s);
              const uint32_t oe = oob_unless(ne < p.N, (ie * p.OCOHW + oc * p.OHW + ne - ie * p.OHW) * 4u);
              float z = v[e];
              if (p.res) z += ld1(rsr, oe);
              z = (p.relu && z < 0.0f) ? 0.0f : z;
              out_store1(p, rso, oe, z);
            }
          }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // reads done before the next tile's writes
      }
    }
#ifdef BH_KTRACE
    if (u0) KT(3);
#endif
    pu += wg;
    if (pu >= npu) break;
    bcur = bnext;
    bnext = ubase(pu + wg);
  }
  vm_wait<0>();
  KT(4);
}

// k1n: the same resident bank and register-streamed input with the MFMA's roles swapped (round 5).
// PMC of k1s on 20x96x54^2 -> 96 (profiles/r04/pmc_k1s.json): 5.1 VALU + 4.0 SALU per MFMA, most of
// it in the epilogue -- with pixels on the M side a lane's accumulators are 4 consecutive pixels of
// one channel, which k1s transposes through LDS (ds writes / reads, a bias shuffle, per-element
// fallbacks) to get 128-B store runs. Here the bank is the A operand (lane li: channel oc0 + 32 t +
// li of bank row 2 s + kh, the same ds_read_b32 as k1s's B) and the input the B operand, so C is
// [channel][pixel]: lane (li, kh) holds pixel column li of channels 32 t + 8 g + 4 kh + i, i.e. the
// output rows are already in memory order:
//  * a unit is 32 TN pixels; lane li owns TN adjacent pixels TN li .. + TN - 1 (column li of TN
//    interleaved N tiles): one TN-wide load per k step feeds TM x TN MFMAs, and one TN-wide store
//    per output row writes 32 x 4 TN contiguous bytes per half-wave (OH*OW % TN == 0, so a lane's
//    pixels never straddle two images);
//  * epilogue per tile and row: a bias (ds_read_b128 of 4 rows' biases), the add, the ReLU and one
//    store at the lane's VGPR pixel offset + the row's scalar offset -- no transposes, no shuffles;
//    rows past OC only in the last OC tile (a wave-uniform branch to the masked form).
// S = 16 TM stores per unit (TN-wide), so (Q - 1) SC + 16 TM <= 63 bounds the configurations.
template <int TN>
__device__ __forceinline__ typename fvec<TN>::t ldv(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
  if constexpr (TN == 1) return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, 0));
  else if constexpr (TN == 2)
    return __builtin_bit_cast(f32x2v, __builtin_amdgcn_raw_buffer_load_b64(r, voff, soff, 0));
  else return __builtin_bit_cast(f32x4v, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0));
}
template <int TN, int AUX>
__device__ __forceinline__ void stv(typename fvec<TN>::t v, __amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
  if constexpr (TN == 1) __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), r, voff, soff, AUX);
  else if constexpr (TN == 2)
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(__attribute__((ext_vector_type(2))) uint32_t, v), r, voff,
                                          soff, AUX);
  else
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) uint32_t, v), r, voff,
                                           soff, AUX);
}

// DBG (instrumented library only, wrong results by design): bit 0 = the epilogue's stores dropped (OOB)
template <int TM, int TN, int KC, int Q, int NW, int DBG = 0>
__global__ __launch_bounds__(NW * 64) void k1n_kernel(GemmArgs p) {
  constexpr int OCT = 32 * TM;           // output channels of the block
  constexpr int UPX = 32 * TN;           // pixels per unit
  constexpr int SC = KC / 2;             // k steps (and input loads per lane) per chunk
  constexpr int S = 16 * TM;             // TN-wide stores per lane per unit
  constexpr int PF = 3;                  // LDS fragment prefetch (steps)
  constexpr int WPC = KC * OCT / 4;      // 16-B bank pieces per chunk
  constexpr int LWC = (WPC + NW * 64 - 1) / (NW * 64);
  constexpr int BREG = ((OCT + 63) / 64) * 64;  // bias floats in LDS (whole 64-lane DMAs)
  static_assert(TM >= 1 && TM <= 3 && KC % 2 == 0 && (TN == 1 || TN == 2 || TN == 4), "tile");
  static_assert(Q >= 2 && (Q - 1) * SC + S <= 63, "vmcnt range");
  static_assert(SC % (PF + 1) == 0, "fragment ring period divides a chunk");
  static_assert(BREG <= NW * 64, "one bias DMA per wave at most");
  typedef typename fvec<TN>::t xv;
  // the bank slice [IC][OCT] (packed-bank rows, columns oc0 ..), then the tile's biases
  extern __shared__ __attribute__((aligned(16))) float wl[];

  const int tid = threadIdx.x, lane = tid & 63, li = lane & 31, kh = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint32_t l8 = blockIdx.x >> 3;
  const uint32_t oct = l8 % p.tiles_m;
  const uint32_t gi = (l8 / p.tiles_m) * 8 + (blockIdx.x & 7);
  const uint32_t wg = (gridDim.x / p.tiles_m) * NW;  // waves per OC tile
  const uint32_t oc0 = oct * OCT;
  const uint32_t npu = (p.N + UPX - 1) / UPX, nch = p.K / KC;
  const uint32_t lds_w = p.K * OCT;
  const uint32_t hw4 = p.HW * 4u, ohw4 = p.OHW * 4u;
  float *const bl = wl + lds_w;

  const __amdgpu_buffer_rsrc_t rsw = make_rsrc(p.a, p.a_bytes);
  const __amdgpu_buffer_rsrc_t rsx = make_rsrc(p.b, p.b_bytes);
  const __amdgpu_buffer_rsrc_t rso = make_rsrc(p.c, p.c_bytes);
  const __amdgpu_buffer_rsrc_t rsbias = make_rsrc(p.bias, p.bias ? p.M * 4u : 0u);

  // biases of the tile (zeros past OC or without biases): older than every wait's count
  if (64 * wave < BREG) {
    const uint32_t oc = oc0 + 64 * wave + lane;
    dma4(rsbias, bl + 64 * wave, oob_unless(oc < p.M, oc * 4u));
  }
  uint32_t wsrc[LWC];
#pragma unroll
  for (int j = 0; j < LWC; ++j) {
    const uint32_t e = (uint32_t)((j * NW + wave) * 64 + lane), r = e / (OCT / 4), q = e % (OCT / 4);
    wsrc[j] = e < (uint32_t)WPC ? oob_unless(oc0 + 4 * q < p.lda, (r * p.lda + oc0 + 4 * q) * 4u) : 0xffffffffu;
  }
  auto issue_w = [&](uint32_t c) {
#pragma unroll
    for (int j = 0; j < LWC; ++j)
      if (wsrc[j] != 0xffffffffu)
        dma16s(rsw, wl + (size_t)c * KC * OCT + (j * NW + wave) * 256, wsrc[j], c * KC * p.lda * 4u);
  };
  // lane li's first pixel of unit pu and its input offset (channel kh); past the op: misses
  auto ubase = [&](uint32_t pu) -> uint32_t {
    const uint32_t n = pu * UPX + TN * li;
    const uint32_t img = fdiv(n, p.ohw_m, p.ohw_s), pix = n - img * p.OHW;
    return oob_unless((pu < npu) & (n < p.N), (img * p.ICHW + pix + kh * p.HW) * 4u);
  };
  xv xr[Q][SC];
  auto issue = [&](int q, uint32_t base, uint32_t c) {
    const uint32_t vb = base + c * KC * hw4;
#pragma unroll
    for (int s = 0; s < SC; ++s) xr[q][s] = ldv<TN>(rsx, vb, 2 * s * hw4);
  };
  uint32_t pu = gi * NW + wave;
  uint32_t bcur = ubase(pu), bnext = ubase(pu + wg);
#pragma unroll
  for (int q = 0; q < Q - 1; ++q) {
    issue_w(q);
    issue(q, bcur, q);
  }
  // S dropped stores: the first unit has the VMEM sequence of every later one
#pragma unroll
  for (int s = 0; s < S; ++s) __builtin_amdgcn_raw_buffer_store_b32(0u, rso, OOB, 0, 0);

  f32x16 acc[TM][TN];
  float wf[PF + 1][TM];
  const float *const wb = wl + kh * OCT + li;
  auto frag = [&](float (&w)[TM], uint32_t c, int s) {
#pragma unroll
    for (int t = 0; t < TM; ++t) w[t] = wb[(c * KC + 2 * s) * OCT + 32 * t];
  };
  // the tile's biases as MFMA C operands: the first step of every unit accumulates onto them
  // (no zeroing, no bias add in the epilogue); row 8 (e / 4) + 4 kh + e % 4 of tile t
  f32x16 biasv[TM];
  auto chunk = [&](int r, uint32_t cq, bool first, bool u0) {
    if (first && r < Q - 1) vm_wait<(Q - 2) * SC + S>();
    else vm_wait<(Q - 2) * SC>();
    if (u0) {
      __syncthreads();
#pragma unroll
      for (int s = 0; s < PF; ++s) frag(wf[s], cq + r, s);
      if (first && r == 0) {
#pragma unroll
        for (int t = 0; t < TM; ++t)
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const f32x4v b4 = *(const f32x4v *)(bl + 32 * t + 8 * g + 4 * kh);
#pragma unroll
            for (int e = 0; e < 4; ++e) biasv[t][4 * g + e] = b4[e];
          }
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    {
      const uint32_t c2 = cq + (uint32_t)(r + Q - 1);
      const bool nx = c2 >= nch;
      if (u0 && !nx) issue_w(c2);
      issue((r + Q - 1) % Q, nx ? bnext : bcur, nx ? c2 - nch : c2);
    }
    __builtin_amdgcn_sched_barrier(0);
    const uint32_t c = cq + (uint32_t)r, cn = c + 1 == nch ? 0u : c + 1;
#pragma unroll
    for (int s = 0; s < SC; ++s) {
      if (s + PF < SC) frag(wf[(s + PF) % (PF + 1)], c, s + PF);
      else if (!u0) frag(wf[(s + PF) % (PF + 1)], cn, s + PF - SC);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int t = 0; t < TM; ++t)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[t][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(wf[s % (PF + 1)][t], vget<TN>(xr[r % Q][s], j),
                                                           first && r == 0 && s == 0 ? biasv[t] : acc[t][j], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  const bool full_m = oc0 + OCT <= p.M;
  const __amdgpu_buffer_rsrc_t rsr = make_rsrc(p.res, p.res ? p.c_bytes : 0u);
  // epilogue: row 8 g + 4 kh + i of tile t is channel oc0 + 32 t + 8 g + 4 kh + i; the lane's half
  // (4 kh rows) goes into its VGPR offset, the rest of the row into the scalar soffset
  // the epilogue's wave-uniform choices (mask, residual, store policy) are taken once per unit:
  // branches per row cost a basic block per store
  const float floor0 = p.relu ? 0.0f : __builtin_nanf("");  // relu_floor: NaN = no clamp
  auto epilogue = [&](auto masked, auto res, auto wt) {
    // the rows' scalar offsets are made here, per unit (laundered stride: hoisted out of the unit
    // loop, 16 TM of them spilled SGPRs into VGPR lanes)
    uint32_t h4 = ohw4;
    asm volatile("" : "+s"(h4));
    const uint32_t so0 = oc0 * h4;
    const uint32_t n = pu * UPX + TN * li;
    const uint32_t img = fdiv(n, p.ohw_m, p.ohw_s), pix = n - img * p.OHW;
    const uint32_t ob = (DBG & 1) ? OOB : oob_unless((pu < npu) & (n < p.N), (img * p.OCOHW + pix) * 4u + (uint32_t)(4 * kh) * h4);
#pragma unroll
    for (int t = 0; t < TM; ++t)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const uint32_t so = so0 + (uint32_t)(32 * t + 8 * g + i) * h4;
          uint32_t o = ob;
          if constexpr (decltype(masked)::value)
            o = oob_unless(oc0 + (uint32_t)(32 * t + 8 * g + 4 * kh + i) < p.M, ob);
          xv v;
          if constexpr (TN == 1) v = acc[t][0][4 * g + i];
          else {
#pragma unroll
            for (int j = 0; j < TN; ++j) v[j] = acc[t][j][4 * g + i];
          }
          if constexpr (decltype(res)::value) v += ldv<TN>(rsr, o, so);
          if constexpr (TN == 1) v = relu_floor(v, floor0);
          else {
#pragma unroll
            for (int j = 0; j < TN; ++j) v[j] = relu_floor(v[j], floor0);
          }
          if constexpr (decltype(wt)::value) stv<TN, AUX_SC1>(v, rso, o, so);
          else stv<TN, AUX_OUT>(v, rso, o, so);
        }
      }
  };
  auto epilogue_m = [&](auto masked) {
    if (p.res) {
      if (p.wt) epilogue(masked, std::true_type{}, std::true_type{});
      else epilogue(masked, std::true_type{}, std::false_type{});
    } else {
      if (p.wt) epilogue(masked, std::false_type{}, std::true_type{});
      else epilogue(masked, std::false_type{}, std::false_type{});
    }
  };

  for (bool u0 = true;; u0 = false) {
    if (u0) {
#pragma unroll
      for (int r = 0; r < Q; ++r) chunk(r, 0, true, true);
      for (uint32_t cq = Q; cq < nch; cq += Q) {
#pragma unroll
        for (int r = 0; r < Q; ++r) chunk(r, cq, false, true);
      }
#pragma unroll
      for (int s = 0; s < PF; ++s) frag(wf[s], 0, s);
    } else {
#pragma unroll
      for (int r = 0; r < Q; ++r) chunk(r, 0, true, false);
      for (uint32_t cq = Q; cq < nch; cq += Q) {
#pragma unroll
        for (int r = 0; r < Q; ++r) chunk(r, cq, false, false);
      }
    }
    // every unit issues exactly S stores (dropped where masked or past the op): the waits count them
    if (full_m) epilogue_m(std::false_type{});
    else epilogue_m(std::true_type{});
    pu += wg;
    if (pu >= npu) break;
    bcur = bnext;
    bnext = ubase(pu + wg);
  }
  vm_wait<0>();
}

// k1d_kernel (round 6, configs kd<OCT>c<KC>d<D>w<NW>): the pixels-on-N form with the input staged by
// 16-B LDS-DMA instead of dword loads into registers. Round-5 PMC of k1n on 20x96x54^2 -> 96
// (profiles/r05/pmc_k1n.json): 59.5 % of wave cycles in s_waitcnt on the input stream. Its in-flight
// input is capped by the vmcnt counter, which the loads share with the epilogue's 16 TM stores:
// (Q - 1) KC / 2 + 16 TM <= 63, so the 96-channel tile that reads each input pixel once could keep only
// ~3 KB per wave in flight (kn96*: slower than kn32, which re-reads the input per 32-channel tile). Here
// one 16-B DMA instruction moves 1 KB (eight channel rows of a unit's 32 pixels) where a dword load
// moved 256 B, so the same counter holds 4x the bytes, and the in-flight data needs no registers:
//  * the block holds the WHOLE bank [K][OCP] (OC rounded up to the unit's channels) and the biases in
//    LDS (IC * OC small enough), loaded once; a unit is 32 consecutive pixels of the flattened (image,
//    pixel) space x one sub-tile of OCT = 32 TM channels x all K; units are dealt to the grid's waves
//    round-robin (sub-tile fastest: a pixel group's sub-tiles run on neighbouring waves of one block,
//    so the re-read input comes from L1 / L2);
//  * each wave streams its units' input through its own ring of D slots [KC][32] (no barrier after the
//    prologue: a wave's DMA and its ds_reads of a slot are ordered by its own vmcnt wait), D - 1 chunks
//    ahead, across unit boundaries;
//  * step s of a chunk: A = bank row 2 s + kh (one ds_read_b32 per 32-channel tile), B = slot row
//    2 s + kh, column li (one ds_read_b32), TM MFMAs; biases as the first MFMA's C, epilogue as k1n
//    (TN = 1: one dword store per output row and lane, rows' offsets scalar).
// vmcnt: waiting for chunk g, the younger VMEM ops are the DMAs of chunks g+1 .. g+D-2 ((D-2) L) plus,
// when an epilogue ran after chunk g's DMA was issued (chunk index in its unit < D - 1), its S stores;
// S dropped stores after the prologue give the first unit the same sequence (as k1n). K / KC >= D - 1.
// DBG (instrumented library only, wrong results by design): bit 0 = the epilogue's stores dropped (OOB)
template <int TM, int KC, int D, int NW, int DBG = 0>
__global__ __launch_bounds__(NW * 64) void k1d_kernel(GemmArgs p) {
  constexpr int OCT = 32 * TM;
  constexpr int SC = KC / 2;   // k steps per chunk
  constexpr int L = KC / 8;    // 16-B DMA instructions per chunk and wave
  constexpr int S = 16 * TM;   // dword stores per lane per unit
  constexpr int PF = 3;        // LDS fragment prefetch (steps)
  constexpr int CH = KC * 32;  // floats per ring slot
  static_assert(TM >= 1 && TM <= 3 && KC % 8 == 0 && SC % (PF + 1) == 0, "tile");
  static_assert(D >= 3 && (D - 2) * L + S <= 63, "vmcnt range");
  // [K][OCP] bank, [OCP rounded up to 64] biases, then each wave's ring [D][KC][32]
  extern __shared__ __attribute__((aligned(16))) float wl[];
  const int tid = threadIdx.x, lane = tid & 63, li = lane & 31, kh = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  KT(0);
  const uint32_t OCP = p.tbm, ntm = p.tiles_m, nch = p.K / KC;
  const uint32_t U = p.total_it;  // units: pixel groups x OC sub-tiles
  const uint32_t W = gridDim.x * NW, w0 = blockIdx.x * NW + (uint32_t)wave;
  const uint32_t hw4 = p.HW * 4u, ohw4 = p.OHW * 4u;
  const uint32_t BREG = (OCP + 63) / 64 * 64;  // bias region: whole 64-lane DMAs
  float *const bl = wl + p.K * OCP;
  float *const ring = bl + BREG + wave * (D * CH);
  const __amdgpu_buffer_rsrc_t rsw = make_rsrc(p.a, p.a_bytes);
  const __amdgpu_buffer_rsrc_t rsx = make_rsrc(p.b, p.b_bytes);
  const __amdgpu_buffer_rsrc_t rso = make_rsrc(p.c, p.c_bytes);
  const __amdgpu_buffer_rsrc_t rsbias = make_rsrc(p.bias, p.bias ? p.M * 4u : 0u);

  // ---- resident bank and biases: piece e = (row k, columns 4q ..) of [K][OCP]; columns past OC4 miss
  {
    const uint32_t pr = OCP / 4, np = p.K * pr;
    // (np is a multiple of 64: a wave's DMA lies wholly inside the bank or is not issued -- a DMA past
    // the end would write over the biases and rings; no wait counts on these, they are older than all)
    for (uint32_t e0 = (uint32_t)wave * 64; e0 < np; e0 += NW * 64) {
      const uint32_t e = e0 + (uint32_t)lane, k = e / pr, q = e - k * pr;
      dma16(rsw, wl + 4 * e0, oob_unless(4 * q < p.lda, (k * p.lda + 4 * q) * 4u));
    }
    for (uint32_t c0 = (uint32_t)wave * 64; c0 < OCP; c0 += NW * 64) {
      const uint32_t c = c0 + (uint32_t)lane;
      dma4(rsbias, bl + c0, oob_unless(c < p.M, c * 4u));
    }
  }
  // ---- the wave's units u = w0 + i W; lane e of a chunk DMA: channel row e / 8 (+ 8 j), pixels 4 (e % 8)
  auto unit_of = [&](uint32_t u, uint32_t &pu, uint32_t &ocs) {
    pu = fdiv(u, p.tm_m, p.tm_s);
    ocs = u - pu * ntm;
  };
  auto dbase = [&](uint32_t u) -> uint32_t {  // this lane's DMA source offset of unit u (channel 0)
    uint32_t pu, ocs;
    unit_of(u, pu, ocs);
    const uint32_t n = pu * 32u + 4u * (uint32_t)(lane & 7);
    const uint32_t img = fdiv(n, p.ohw_m, p.ohw_s), pix = n - img * p.OHW;
    return oob_unless((u < U) & (n < p.N), (img * p.ICHW + pix + (uint32_t)(lane >> 3) * p.HW) * 4u);
  };
  uint32_t u = w0;
  uint32_t bcur = dbase(u), bnext = dbase(u + W);
  auto issue = [&](uint32_t slot, uint32_t base, uint32_t c) {
#pragma unroll
    for (int j = 0; j < L; ++j) dma16s(rsx, ring + slot * CH + j * 256, base, (c * KC + 8 * j) * hw4);
  };
  // prologue: chunks 0 .. D-2 of the first unit (K / KC >= D - 1), then S dropped stores
#pragma unroll
  for (int q = 0; q < D - 1; ++q) issue((uint32_t)q, bcur, (uint32_t)q);
#pragma unroll
  for (int s = 0; s < S; ++s) __builtin_amdgcn_raw_buffer_store_b32(0u, rso, OOB, 0, 0);
  vm_wait<(D - 2) * L + S>();  // the bank, the biases and chunk 0 landed (this wave's DMAs) ...
  __syncthreads();             // ... every wave's
  if (u >= U) return;

  f32x16 acc[TM];
  float wf[PF + 1][TM], xf[PF + 1];
  uint32_t pu, ocs;
  unit_of(u, pu, ocs);
  const float *wa = wl + kh * OCP + ocs * OCT + li;  // bank fragment base of the unit's sub-tile
  const float *const xa = ring + kh * 32 + li;       // slot fragment base (+ slot * CH)
  auto frag = [&](int b, uint32_t slot, uint32_t c, int s) {
#pragma unroll
    for (int t = 0; t < TM; ++t) wf[b][t] = wa[(c * KC + 2 * s) * OCP + 32 * t];
    xf[b] = xa[slot * CH + 2 * s * 32];
  };
  auto load_bias = [&]() {
#pragma unroll
    for (int t = 0; t < TM; ++t)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f32x4v b4 = *(const f32x4v *)(bl + ocs * OCT + 32 * t + 8 * g + 4 * kh);
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[t][4 * g + e] = b4[e];
      }
  };
  const float floor0 = p.relu ? 0.0f : __builtin_nanf("");  // relu_floor: NaN = no clamp
  const __amdgpu_buffer_rsrc_t rsr = make_rsrc(p.res, p.res ? p.c_bytes : 0u);
  auto epilogue = [&](auto masked, auto res, auto wt) {
    uint32_t h4 = ohw4;
    asm volatile("" : "+s"(h4));
    const uint32_t oc0 = ocs * OCT, so0 = oc0 * h4;
    const uint32_t n = pu * 32u + (uint32_t)li;
    const uint32_t img = fdiv(n, p.ohw_m, p.ohw_s), pix = n - img * p.OHW;
    const uint32_t ob = (DBG & 1) ? OOB : oob_unless(n < p.N, (img * p.OCOHW + pix) * 4u + (uint32_t)(4 * kh) * h4);
#pragma unroll
    for (int t = 0; t < TM; ++t)
#pragma unroll
      for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const uint32_t so = so0 + (uint32_t)(32 * t + 8 * g + i) * h4;
          uint32_t o = ob;
          if constexpr (decltype(masked)::value) o = oob_unless(oc0 + (uint32_t)(32 * t + 8 * g + 4 * kh + i) < p.M, ob);
          float v = acc[t][4 * g + i];
          if constexpr (decltype(res)::value) v += ldv<1>(rsr, o, so);
          v = relu_floor(v, floor0);
          if constexpr (decltype(wt)::value) stv<1, AUX_SC1>(v, rso, o, so);
          else stv<1, AUX_OUT>(v, rso, o, so);
        }
  };
  auto epilogue_m = [&](auto masked) {
    if (p.res) {
      if (p.wt) epilogue(masked, std::true_type{}, std::true_type{});
      else epilogue(masked, std::true_type{}, std::false_type{});
    } else {
      if (p.wt) epilogue(masked, std::false_type{}, std::true_type{});
      else epilogue(masked, std::false_type{}, std::false_type{});
    }
  };

  // the chunk stream: chunk c of the current unit sits in slot `slot`; the DMA issued with it is chunk
  // c + D - 1 (of this unit, or the next one's chunk c + D - 1 - nch) into the slot freed last chunk.
  // The first PF steps' fragments of the NEXT chunk are read in the last PF steps of this one, after
  // that chunk's wait: younger than its DMA are the DMAs of the D - 2 chunks after it, and, when its
  // index in its unit is 1 .. D - 2, the S stores of the epilogue that ran since it was issued
  uint32_t slot = 0, islot = D - 1;
  load_bias();
#pragma unroll
  for (int s = 0; s < PF; ++s) frag(s, 0, 0, s);  // chunk 0 landed (prologue wait)
  for (;;) {
    // the next unit's sub-tile: the last chunk prefetches its first fragments
    uint32_t pu_n, ocs_n;
    unit_of(u + W, pu_n, ocs_n);
    const float *const wa_n = wl + kh * OCP + ocs_n * OCT + li;
    for (uint32_t c = 0; c < nch; ++c) {
      {
        const uint32_t c2 = c + (uint32_t)(D - 1);
        const bool nx = c2 >= nch;
        issue(islot, nx ? bnext : bcur, nx ? c2 - nch : c2);
      }
      const uint32_t nslot = slot == D - 1 ? 0u : slot + 1;
      const bool last = c + 1 == nch;
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int s = 0; s < SC; ++s) {
        if (s + PF < SC) {
          frag((s + PF) % (PF + 1), slot, c, s + PF);
        } else {
          if (s + PF == SC) {  // the next chunk's DMA (uniform)
            if (!last && c + 1 <= (uint32_t)(D - 2)) vm_wait<(D - 2) * L + S>();
            else vm_wait<(D - 2) * L>();
          }
          if (last) {
            const float *const wsave = wa;
            wa = wa_n;
            frag((s + PF) % (PF + 1), nslot, 0, s + PF - SC);
            wa = wsave;
          } else {
            frag((s + PF) % (PF + 1), nslot, c + 1, s + PF - SC);
          }
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int t = 0; t < TM; ++t)
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(wf[s % (PF + 1)][t], xf[s % (PF + 1)], acc[t], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
      islot = slot;
      slot = nslot;
    }
    // every unit issues exactly S stores (dropped where masked or past the op): the waits count them
    if (ocs * OCT + OCT <= p.M) epilogue_m(std::false_type{});
    else epilogue_m(std::true_type{});
    u += W;
    if (u >= U) break;
    bcur = bnext;
    bnext = dbase(u + W);
    pu = pu_n;
    ocs = ocs_n;
    wa = wa_n;
    load_bias();
  }
  vm_wait<0>();
}

template <int TM, int KC, int D, int NW, int DBG = 0>
cfg_t k1d_cfg(const char *name) {
  cfg_t c{name, 32 * TM, 32 * NW, KC, 64 * NW, {}, 1};
  c.k[A_KVEC][B_DIRECT][0] = k1d_kernel<TM, KC, D, NW, DBG>;
  c.dc = 3;
  c.dc_ky = 1;
  c.dc_kx = 1;
  c.dc_ci = KC;
  c.dc_rin = D;
  c.k1d = 1;
  return c;
}

// k1w_kernel (round 6, configs kw<OCT>c<KC>q<Q>w<NW>s<NSW>l<NSL>): k1n (TN = 1) with the output stores moved to
// NSW store waves. vmcnt counts a wave's loads, LDS-DMAs and stores in issue order, so in k1n a wait for
// an input chunk issued after a unit's epilogue also waits for that epilogue's 16 TM stores to complete
// (round-3 diagnostics of k1s on 20x96x54^2 -> 96: 20.0 us with stores, 14.2 us with them dropped). Here a
// compute wave never stores: it writes its finished unit [OCT][32] (biases included) into one of its NSL
// LDS staging slots and bumps a counter; a store wave reads the slot back (ds_read_b128: 8 rows x 128 B per
// instruction), adds the residual, applies the ReLU and issues 16-B stores (OH*OW % 4 == 0), and frees
// the slot once its reads have returned -- it never waits for its stores. The compute waves' vmcnt then
// holds only input loads: every chunk waits (Q - 2) KC / 2 loads deep. The bank slice is DMA'd whole in
// the prologue (one barrier); after it no barrier runs, the hand-off is two LDS counters per compute wave
// (data writes drained by lgkmcnt before the counter write; the reader branches on the counter before it
// reads the data). Every spin is bounded (a hand-off that never comes ends the wave instead of hanging).
template <int TM, int KC, int Q, int NW, int NSW, int NSL>
__global__ __launch_bounds__((NW + NSW) * 64) void k1w_kernel(GemmArgs p) {
  constexpr int OCT = 32 * TM, SC = KC / 2, PF = 3, TILE = OCT * 32, NT = (NW + NSW) * 64;
  constexpr int BREG = ((OCT + 63) / 64) * 64;
  constexpr uint32_t SPIN = 1u << 20;
  static_assert(TM >= 1 && TM <= 3 && KC % 2 == 0 && SC % (PF + 1) == 0, "tile");
  static_assert(Q >= 2 && (Q - 1) * SC <= 63, "vmcnt range");
  static_assert(NW % NSW == 0 && NSW >= 1, "store waves serve whole groups of compute waves");
  static_assert(NSL == 1 || NSL == 2, "staging slots per compute wave");
  // [K][OCT] bank (padded to whole 64-lane 16-B DMAs), biases, staging [NW][NSL][OCT][32], counters full / done
  extern __shared__ __attribute__((aligned(16))) float wl[];
  const int tid = threadIdx.x, lane = tid & 63, li = lane & 31, kh = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint32_t l8 = blockIdx.x >> 3;
  const uint32_t oct = l8 % p.tiles_m;
  const uint32_t gi = (l8 / p.tiles_m) * 8 + (blockIdx.x & 7);
  const uint32_t wg = (gridDim.x / p.tiles_m) * NW;  // compute waves per OC tile
  const uint32_t oc0 = oct * OCT;
  const uint32_t npu = (p.N + 31) / 32, nch = p.K / KC;
  const uint32_t np = p.K * OCT / 4, lds_w = (np + 63) / 64 * 256;
  const uint32_t hw4 = p.HW * 4u, ohw4 = p.OHW * 4u;
  float *const bl = wl + lds_w;
  float *const stg = bl + BREG;
  volatile uint32_t *const full = (volatile uint32_t *)(stg + NW * NSL * TILE);
  volatile uint32_t *const done = full + NW;
  const __amdgpu_buffer_rsrc_t rsw = make_rsrc(p.a, p.a_bytes);
  const __amdgpu_buffer_rsrc_t rsx = make_rsrc(p.b, p.b_bytes);
  const __amdgpu_buffer_rsrc_t rsbias = make_rsrc(p.bias, p.bias ? p.M * 4u : 0u);

  if (tid < 2 * NW) full[tid] = 0u;  // full and done (before the prologue barrier)
  // the whole bank slice [K][OCT]: piece e = (row e / (OCT / 4), columns oc0 + 4 (e % (OCT / 4)))
  for (uint32_t e0 = (uint32_t)wave * 64; e0 < np; e0 += NT) {
    const uint32_t e = e0 + (uint32_t)lane, r = e / (OCT / 4), q = e % (OCT / 4);
    dma16(rsw, wl + 4 * e0, oob_unless((e < np) & (oc0 + 4 * q < p.lda), (r * p.lda + oc0 + 4 * q) * 4u));
  }
  if (64 * wave < BREG) dma4(rsbias, bl + 64 * wave, oob_unless(oc0 + 64 * wave + lane < p.M, (oc0 + 64 * wave + lane) * 4u));

  if (wave >= NW) {  // ---- store wave: serves compute waves w = sw, sw + NSW, ...
    vm_wait<0>();
    __syncthreads();
    const int sw = wave - NW;
    constexpr int NS = NW / NSW;
    uint32_t cnt[NS], dn[NS];
#pragma unroll
    for (int k = 0; k < NS; ++k) {
      const uint32_t pu0 = gi * NW + (uint32_t)(sw + k * NSW);
      cnt[k] = pu0 < npu ? (npu - pu0 + wg - 1) / wg : 0u;
      dn[k] = 0;
    }
    const __amdgpu_buffer_rsrc_t rso = make_rsrc(p.c, p.c_bytes);
    const __amdgpu_buffer_rsrc_t rsr = make_rsrc(p.res, p.res ? p.c_bytes : 0u);
    const float floor0 = p.relu ? 0.0f : __builtin_nanf("");  // relu_floor: NaN = no clamp
    const uint32_t rl = (uint32_t)lane >> 3, cq = 4u * ((uint32_t)lane & 7u);  // row in a group of 8, first pixel
    for (uint32_t spin = 0; spin < SPIN;) {
      bool all = true, prog = false;
#pragma unroll
      for (int k = 0; k < NS; ++k) {
        if (dn[k] >= cnt[k]) continue;
        all = false;
        const int w = sw + k * NSW;
        if (full[w] <= dn[k]) continue;
        prog = true;
        asm volatile("" ::: "memory");  // the slot's reads stay behind the counter's
        const uint32_t j = dn[k], pu = gi * NW + (uint32_t)w + j * wg;
        const float *const tile = stg + (w * NSL + (int)(j % NSL)) * TILE + (rl * 32 + cq);
        f32x4v v[OCT / 8];
#pragma unroll
        for (int g = 0; g < OCT / 8; ++g) v[g] = *(const f32x4v *)(tile + g * 8 * 32);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        done[w] = j + 1;  // the slot's data is in registers
        dn[k] = j + 1;
        const uint32_t n = pu * 32u + cq;
        const uint32_t img = fdiv(n, p.ohw_m, p.ohw_s), pix = n - img * p.OHW;
        const uint32_t ob = (img * p.OCOHW + pix) * 4u + rl * ohw4;
#pragma unroll
        for (int g = 0; g < OCT / 8; ++g) {
          const uint32_t oc = oc0 + (uint32_t)(8 * g) + rl, so = (oc0 + (uint32_t)(8 * g)) * ohw4;
          const uint32_t o = oob_unless((oc < p.M) & (n < p.N), ob);
          f32x4v x = v[g];
          if (p.res) x += ldv<4>(rsr, o, so);
#pragma unroll
          for (int e = 0; e < 4; ++e) x[e] = relu_floor(x[e], floor0);
          if (p.wt) stv<4, AUX_SC1>(x, rso, o, so);
          else stv<4, AUX_OUT>(x, rso, o, so);
        }
      }
      if (all) break;
      if (!prog) {
        __builtin_amdgcn_s_sleep(1);
        ++spin;
      }
    }
    return;
  }

  // ---- compute wave: k1n's stream (TN = 1), no stores
  auto ubase = [&](uint32_t pu) -> uint32_t {
    const uint32_t n = pu * 32u + (uint32_t)li;
    const uint32_t img = fdiv(n, p.ohw_m, p.ohw_s), pix = n - img * p.OHW;
    return oob_unless((pu < npu) & (n < p.N), (img * p.ICHW + pix + kh * p.HW) * 4u);
  };
  float xr[Q][SC];
  auto issue = [&](int q, uint32_t base, uint32_t c) {
    const uint32_t vb = base + c * KC * hw4;
#pragma unroll
    for (int s = 0; s < SC; ++s) xr[q][s] = ldv<1>(rsx, vb, 2 * s * hw4);
  };
  uint32_t pu = gi * NW + (uint32_t)wave;
  uint32_t bcur = ubase(pu), bnext = ubase(pu + wg);
#pragma unroll
  for (int q = 0; q < Q - 1; ++q) issue(q, bcur, (uint32_t)q);
  vm_wait<(Q - 2) * SC>();  // the bank, the biases and chunk 0 (this wave's)
  __syncthreads();          // every wave's bank DMAs
  if (pu >= npu) return;

  f32x16 acc[TM];
  float wf[PF + 1][TM];
  const float *const wb = wl + kh * OCT + li;
  auto frag = [&](float (&w)[TM], uint32_t c, int s) {
#pragma unroll
    for (int t = 0; t < TM; ++t) w[t] = wb[(c * KC + 2 * s) * OCT + 32 * t];
  };
  f32x16 biasv[TM];
#pragma unroll
  for (int t = 0; t < TM; ++t)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const f32x4v b4 = *(const f32x4v *)(bl + 32 * t + 8 * g + 4 * kh);
#pragma unroll
      for (int e = 0; e < 4; ++e) biasv[t][4 * g + e] = b4[e];
    }
  auto chunk = [&](int r, uint32_t cq, bool first) {
    vm_wait<(Q - 2) * SC>();  // (a no-op on the first unit's chunk 0)
    __builtin_amdgcn_sched_barrier(0);
    {
      const uint32_t c2 = cq + (uint32_t)(r + Q - 1);
      const bool nx = c2 >= nch;
      issue((r + Q - 1) % Q, nx ? bnext : bcur, nx ? c2 - nch : c2);
    }
    __builtin_amdgcn_sched_barrier(0);
    const uint32_t c = cq + (uint32_t)r, cn = c + 1 == nch ? 0u : c + 1;
#pragma unroll
    for (int s = 0; s < SC; ++s) {
      if (s + PF < SC) frag(wf[(s + PF) % (PF + 1)], c, s + PF);
      else frag(wf[(s + PF) % (PF + 1)], cn, s + PF - SC);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int t = 0; t < TM; ++t)
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(wf[s % (PF + 1)][t], xr[r % Q][s],
                                                       first && r == 0 && s == 0 ? biasv[t] : acc[t], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
  };
#pragma unroll
  for (int s = 0; s < PF; ++s) frag(wf[s], 0, s);
  for (uint32_t j = 0;; ++j) {
#pragma unroll
    for (int r = 0; r < Q; ++r) chunk(r, 0, true);
    for (uint32_t cq = Q; cq < nch; cq += Q) {
#pragma unroll
      for (int r = 0; r < Q; ++r) chunk(r, cq, false);
    }
    // hand the unit to the store wave: slot j % NSL once the store wave has read unit j - NSL out of it
    for (uint32_t spin = 0; j - done[wave] >= (uint32_t)NSL && spin < SPIN; ++spin) __builtin_amdgcn_s_sleep(1);
    asm volatile("" ::: "memory");
    float *const st = stg + (wave * NSL + (int)(j % NSL)) * TILE + (4 * kh) * 32 + li;
#pragma unroll
    for (int t = 0; t < TM; ++t)
#pragma unroll
      for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int i = 0; i < 4; ++i) st[(32 * t + 8 * g + i) * 32] = acc[t][4 * g + i];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    full[wave] = j + 1;
    pu += wg;
    if (pu >= npu) break;
    bcur = bnext;
    bnext = ubase(pu + wg);
  }
  vm_wait<0>();
}

template <int TM, int KC, int Q, int NW, int NSW, int NSL>
cfg_t k1w_cfg(const char *name) {
  cfg_t c{name, 32 * TM, 32 * NW, KC, 64 * (NW + NSW), {}, 1};
  c.k[A_KVEC][B_DIRECT][0] = k1w_kernel<TM, KC, Q, NW, NSW, NSL>;
  c.dc = 3;
  c.dc_ky = 1;
  c.dc_kx = 1;
  c.dc_ci = KC;
  c.dc_rin = Q;
  c.k1w = NSW;
  c.k1w_sl = NSL;
  return c;
}

// compile-time loop: f(integral_constant<int, I>) for I in [I0, N) (register-array indices must be constants)
template <int I, int N, class F>
__device__ __forceinline__ void k1_static_for(F &&f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    k1_static_for<I + 1, N>(f);
  }
}

// k1r_kernel (round 6, configs kr<OCT>k<KMAX>c<KC>q<Q>w<NW>): k1n (TN = 1) with the bank slice held in
// VGPRs instead of LDS, for K <= KMAX (TM * KMAX / 2 registers: lane (li, kh) keeps bank rows 2 s + kh of
// channels oc0 + 32 t + li). A wave loads its slice once (two 128-B row pieces per instruction) and
// then never touches LDS: no fragment reads per MFMA, no bank DMA, no barrier -- waves are independent
// from their first load. The chunk loop is unrolled over KMAX / KC chunks (register indices must be
// compile-time) and stops at the op's K / KC; the input ring, the unit stream and the epilogue are
// k1n's (the first unit's dropped stores keep every unit's VMEM sequence alike for the counted waits).
template <int TM, int KMAX, int KC, int Q, int NW>
__global__ __launch_bounds__(NW * 64) void k1r_kernel(GemmArgs p) {
  constexpr int OCT = 32 * TM, SC = KC / 2, S = 16 * TM, NCH = KMAX / KC;
  static_assert(TM >= 1 && TM <= 2 && KC % 2 == 0 && KMAX % (KC * Q) == 0, "tile");
  static_assert(Q >= 2 && (Q - 1) * SC + S <= 63, "vmcnt range");
  const int lane = threadIdx.x & 63, li = lane & 31, kh = lane >> 5;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t l8 = blockIdx.x >> 3;
  const uint32_t oct = l8 % p.tiles_m;
  const uint32_t gi = (l8 / p.tiles_m) * 8 + (blockIdx.x & 7);
  const uint32_t wg = (gridDim.x / p.tiles_m) * NW;
  const uint32_t oc0 = oct * OCT;
  const uint32_t npu = (p.N + 31) / 32, nch = p.K / KC;
  const uint32_t hw4 = p.HW * 4u, ohw4 = p.OHW * 4u;
  const __amdgpu_buffer_rsrc_t rsw = make_rsrc(p.a, p.a_bytes);
  const __amdgpu_buffer_rsrc_t rsx = make_rsrc(p.b, p.b_bytes);
  const __amdgpu_buffer_rsrc_t rso = make_rsrc(p.c, p.c_bytes);
  const __amdgpu_buffer_rsrc_t rsbias = make_rsrc(p.bias, p.bias ? p.M * 4u : 0u);
  uint32_t pu = gi * NW + (uint32_t)wave;
  if (pu >= npu) return;

  // the bank slice (rows past K and columns past the packed width: zeros) and the tile's biases as
  // each unit's first C operand (row 8 g + 4 kh + e of tile t)
  float wreg[TM][KMAX / 2];
#pragma unroll
  for (int t = 0; t < TM; ++t) {
    const uint32_t col = oc0 + 32u * t + (uint32_t)li;
    const uint32_t vo = oob_unless(col < p.lda, (kh * p.lda + col) * 4u);
#pragma unroll
    for (int s = 0; s < KMAX / 2; ++s)
      wreg[t][s] = ldv<1>(rsw, oob_unless(2u * s < p.K, vo), 2u * s * p.lda * 4u);
  }
  f32x16 biasv[TM];
#pragma unroll
  for (int t = 0; t < TM; ++t)
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const uint32_t oc = oc0 + 32u * t + 8u * g + 4u * kh + e;
        biasv[t][4 * g + e] = ldv<1>(rsbias, oob_unless(oc < p.M, oc * 4u), 0u);
      }
  auto ubase = [&](uint32_t u) -> uint32_t {
    const uint32_t n = u * 32u + (uint32_t)li;
    const uint32_t img = fdiv(n, p.ohw_m, p.ohw_s), pix = n - img * p.OHW;
    return oob_unless((u < npu) & (n < p.N), (img * p.ICHW + pix + kh * p.HW) * 4u);
  };
  float xr[Q][SC];
  auto issue = [&](int q, uint32_t base, uint32_t c) {
    const uint32_t vb = base + c * KC * hw4;
#pragma unroll
    for (int s = 0; s < SC; ++s) xr[q][s] = ldv<1>(rsx, vb, 2 * s * hw4);
  };
  uint32_t bcur = ubase(pu), bnext = ubase(pu + wg);
#pragma unroll
  for (int q = 0; q < Q - 1; ++q) issue(q, bcur, (uint32_t)q);
#pragma unroll
  for (int s = 0; s < S; ++s) __builtin_amdgcn_raw_buffer_store_b32(0u, rso, OOB, 0, 0);

  f32x16 acc[TM];
  const bool full_m = oc0 + OCT <= p.M;
  const __amdgpu_buffer_rsrc_t rsr = make_rsrc(p.res, p.res ? p.c_bytes : 0u);
  const float floor0 = p.relu ? 0.0f : __builtin_nanf("");  // relu_floor: NaN = no clamp
  auto epilogue = [&](auto masked, auto res, auto wt) {
    uint32_t h4 = ohw4;
    asm volatile("" : "+s"(h4));
    const uint32_t so0 = oc0 * h4;
    const uint32_t n = pu * 32u + (uint32_t)li;
    const uint32_t img = fdiv(n, p.ohw_m, p.ohw_s), pix = n - img * p.OHW;
    const uint32_t ob = oob_unless((pu < npu) & (n < p.N), (img * p.OCOHW + pix) * 4u + (uint32_t)(4 * kh) * h4);
#pragma unroll
    for (int t = 0; t < TM; ++t)
#pragma unroll
      for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const uint32_t so = so0 + (uint32_t)(32 * t + 8 * g + i) * h4;
          uint32_t o = ob;
          if constexpr (decltype(masked)::value) o = oob_unless(oc0 + (uint32_t)(32 * t + 8 * g + 4 * kh + i) < p.M, ob);
          float v = acc[t][4 * g + i];
          if constexpr (decltype(res)::value) v += ldv<1>(rsr, o, so);
          v = relu_floor(v, floor0);
          if constexpr (decltype(wt)::value) stv<1, AUX_SC1>(v, rso, o, so);
          else stv<1, AUX_OUT>(v, rso, o, so);
        }
  };
  auto epilogue_m = [&](auto masked) {
    if (p.res) {
      if (p.wt) epilogue(masked, std::true_type{}, std::true_type{});
      else epilogue(masked, std::true_type{}, std::false_type{});
    } else {
      if (p.wt) epilogue(masked, std::false_type{}, std::true_type{});
      else epilogue(masked, std::false_type{}, std::false_type{});
    }
  };
  for (;;) {
    k1_static_for<0, NCH>([&](auto cc) {
      constexpr int c = decltype(cc)::value;
      if ((uint32_t)c >= nch) return;
      // chunks 0 .. Q - 2 of a unit were issued before the previous unit's S stores
      if (c < Q - 1) vm_wait<(Q - 2) * SC + S>();
      else vm_wait<(Q - 2) * SC>();
      __builtin_amdgcn_sched_barrier(0);
      {
        const uint32_t c2 = (uint32_t)c + (uint32_t)(Q - 1);
        const bool nx = c2 >= nch;
        issue((c + Q - 1) % Q, nx ? bnext : bcur, nx ? c2 - nch : c2);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int s = 0; s < SC; ++s) {
#pragma unroll
        for (int t = 0; t < TM; ++t)
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(wreg[t][c * SC + s], xr[c % Q][s],
                                                         c == 0 && s == 0 ? biasv[t] : acc[t], 0, 0, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
    });
    if (full_m) epilogue_m(std::false_type{});
    else epilogue_m(std::true_type{});
    pu += wg;
    if (pu >= npu) break;
    bcur = bnext;
    bnext = ubase(pu + wg);
  }
  vm_wait<0>();
}

template <int TM, int KMAX, int KC, int Q, int NW>
cfg_t k1r_cfg(const char *name) {
  cfg_t c{name, 32 * TM, 32 * NW, KC, 64 * NW, {}, 1};
  c.k[A_KVEC][B_DIRECT][0] = k1r_kernel<TM, KMAX, KC, Q, NW>;
  c.dc = 3;
  c.dc_ky = 1;
  c.dc_kx = 1;
  c.dc_ci = KC;
  c.dc_rin = Q;
  c.k1r = KMAX;
  return c;
}

template <int TM, int TN, int KC, int Q, int NW, int DBG = 0>
cfg_t k1n_cfg(const char *name) {
  cfg_t c{name, 32 * TM, 32 * TN * NW, KC, 64 * NW, {}, 1};
  c.k[A_KVEC][B_DIRECT][0] = k1n_kernel<TM, TN, KC, Q, NW, DBG>;
  c.dc = 3;
  c.dc_ky = 1;
  c.dc_kx = 1;
  c.dc_ci = KC;
  c.dc_rin = Q;
  c.gv_cx = TN;
  c.k1n = 1;
  return c;
}

template <int TM, int KC, int Q, int NW, int DBG = 0>
cfg_t k1s_cfg(const char *name) {
  cfg_t c{name, 32 * TM, 32 * NW, KC, 64 * NW, {}, 1};
  c.k[A_KVEC][B_DIRECT][0] = k1s_kernel<TM, KC, Q, NW, DBG>;
  c.dc = 3;
  c.dc_ky = 1;
  c.dc_kx = 1;
  c.dc_ci = KC;
  c.dc_rin = Q;
  return c;
}

}  // namespace

std::vector<cfg_t> k1s_cfgs() {
  // <TM, KC, Q, NW>: OC tile 32*TM, KC-channel chunks, Q - 1 chunks in flight, NW waves
  return {
      k1s_cfg<1, 32, 3, 4>("ks32c32q3"),    k1s_cfg<2, 32, 3, 4>("ks64c32q3"),
      k1s_cfg<3, 32, 3, 4>("ks96c32q3"),    k1s_cfg<4, 32, 3, 4>("ks128c32q3"),
      k1s_cfg<1, 32, 4, 4>("ks32c32q4"),    k1s_cfg<2, 32, 4, 4>("ks64c32q4"),
      k1s_cfg<2, 32, 2, 4>("ks64c32q2"),    k1s_cfg<4, 32, 2, 4>("ks128c32q2"),
      k1s_cfg<2, 16, 4, 4>("ks64c16q4"),    k1s_cfg<3, 16, 4, 4>("ks96c16q4"),
      k1s_cfg<4, 16, 4, 4>("ks128c16q4"),   k1s_cfg<1, 16, 4, 4>("ks32c16q4"),
      k1s_cfg<2, 32, 3, 8>("ks64c32q3w8"),  k1s_cfg<3, 32, 3, 8>("ks96c32q3w8"),
      k1s_cfg<1, 32, 3, 8>("ks32c32q3w8"),  k1s_cfg<1, 16, 4, 8>("ks32c16q4w8"),
      // k1n <TM, TN, KC, Q, NW>: kn<OC tile>p<pixels per unit>c<KC>q<Q>w<NW>
      k1n_cfg<1, 1, 16, 4, 8>("kn32p32c16q4w8"),   k1n_cfg<1, 2, 16, 4, 8>("kn32p64c16q4w8"),
      k1n_cfg<1, 4, 16, 4, 4>("kn32p128c16q4w4"),  k1n_cfg<1, 2, 32, 3, 8>("kn32p64c32q3w8"),
      k1n_cfg<1, 1, 32, 3, 8>("kn32p32c32q3w8"),   k1n_cfg<2, 1, 16, 3, 8>("kn64p32c16q3w8"),
      k1n_cfg<2, 2, 16, 3, 8>("kn64p64c16q3w8"),   k1n_cfg<2, 2, 16, 4, 8>("kn64p64c16q4w8"),
      k1n_cfg<2, 2, 32, 2, 8>("kn64p64c32q2w8"),   k1n_cfg<2, 4, 16, 3, 4>("kn64p128c16q3w4"),
      k1n_cfg<2, 2, 16, 4, 4>("kn64p64c16q4w4"),   k1n_cfg<3, 1, 8, 4, 8>("kn96p32c8q4w8"),
      k1n_cfg<3, 2, 8, 4, 8>("kn96p64c8q4w8"),     k1n_cfg<3, 2, 16, 2, 8>("kn96p64c16q2w8"),
      k1n_cfg<3, 2, 8, 4, 4>("kn96p64c8q4w4"),
      // round 6: a unit's whole K (96) in flight, the ring waits never short of loads
      k1n_cfg<1, 1, 8, 12, 8>("kn32p32c8q12w8"),   k1n_cfg<1, 1, 16, 6, 8>("kn32p32c16q6w8"),
      k1n_cfg<1, 1, 16, 6, 4>("kn32p32c16q6w4"),
      // k1d <TM, KC, D, NW>: kd<OC sub-tile>c<KC>d<ring slots>w<NW>, the whole bank resident
      k1d_cfg<3, 16, 6, 4>("kd96c16d6w4"), k1d_cfg<3, 16, 8, 4>("kd96c16d8w4"), k1d_cfg<3, 16, 5, 8>("kd96c16d5w8"),
      k1d_cfg<2, 16, 6, 4>("kd64c16d6w4"), k1d_cfg<2, 16, 8, 4>("kd64c16d8w4"), k1d_cfg<2, 16, 5, 8>("kd64c16d5w8"),
      k1d_cfg<2, 32, 4, 4>("kd64c32d4w4"), k1d_cfg<1, 32, 5, 4>("kd32c32d5w4"), k1d_cfg<1, 16, 5, 8>("kd32c16d5w8"),
      k1d_cfg<3, 32, 3, 4>("kd96c32d3w4"),
      // D = K / KC + 1: a unit's whole input is in flight before the previous unit's stores go out, so no
      // ring wait orders behind a store (vmcnt counts loads, DMAs and stores in issue order)
      k1d_cfg<3, 32, 4, 4>("kd96c32d4w4"), k1d_cfg<3, 16, 7, 4>("kd96c16d7w4"), k1d_cfg<2, 32, 3, 4>("kd64c32d3w4"),
      k1d_cfg<2, 16, 5, 4>("kd64c16d5w4"), k1d_cfg<2, 32, 3, 8>("kd64c32d3w8"), k1d_cfg<1, 32, 4, 4>("kd32c32d4w4"),
      k1d_cfg<1, 32, 3, 8>("kd32c32d3w8"),
      // k1w <TM, KC, Q, NW, NSW, NSL>: kw<OC tile>c<KC>q<Q>w<compute waves>s<store waves>l<staging slots>
      k1w_cfg<1, 32, 3, 8, 2, 2>("kw32c32q3w8s2l2"), k1w_cfg<1, 16, 4, 8, 2, 2>("kw32c16q4w8s2l2"),
      k1w_cfg<1, 16, 3, 8, 2, 2>("kw32c16q3w8s2l2"), k1w_cfg<1, 16, 4, 4, 1, 2>("kw32c16q4w4s1l2"),
      k1w_cfg<2, 16, 4, 4, 1, 2>("kw64c16q4w4s1l2"), k1w_cfg<2, 16, 4, 8, 2, 1>("kw64c16q4w8s2l1"),
      k1w_cfg<2, 8, 4, 8, 2, 1>("kw64c8q4w8s2l1"),   k1w_cfg<3, 8, 4, 4, 1, 1>("kw96c8q4w4s1l1"),
      k1w_cfg<3, 16, 3, 4, 1, 1>("kw96c16q3w4s1l1"),
      k1w_cfg<3, 8, 12, 4, 1, 1>("kw96c8q12w4s1l1"), k1w_cfg<3, 16, 6, 4, 1, 1>("kw96c16q6w4s1l1"),
      k1w_cfg<1, 8, 12, 8, 2, 2>("kw32c8q12w8s2l2"),
      // k1r <TM, KMAX, KC, Q, NW>: kr<OC tile>k<largest K>c<KC>q<Q>w<NW>, the bank slice in VGPRs
      k1r_cfg<1, 64, 16, 4, 4>("kr32k64c16q4w4"),   k1r_cfg<1, 64, 16, 4, 8>("kr32k64c16q4w8"),
      k1r_cfg<1, 96, 16, 3, 4>("kr32k96c16q3w4"),   k1r_cfg<1, 96, 16, 3, 8>("kr32k96c16q3w8"),
      k1r_cfg<1, 96, 8, 4, 8>("kr32k96c8q4w8"),     k1r_cfg<1, 128, 16, 4, 4>("kr32k128c16q4w4"),
      k1r_cfg<1, 192, 16, 3, 4>("kr32k192c16q3w4"), k1r_cfg<2, 64, 16, 4, 4>("kr64k64c16q4w4"),
      k1r_cfg<2, 96, 16, 3, 4>("kr64k96c16q3w4"),
#ifdef BH_KTRACE
      k1d_cfg<3, 32, 4, 4, 1>("xkd96c32d4w4_nostore"), k1d_cfg<3, 16, 6, 4, 1>("xkd96c16d6w4_nostore"),
      k1n_cfg<1, 1, 32, 3, 8, 1>("xkn32p32c32q3w8_nostore"), k1n_cfg<1, 1, 16, 4, 8, 1>("xkn32p32c16q4w8_nostore"),
      k1n_cfg<3, 2, 8, 4, 4, 1>("xkn96p64c8q4w4_nostore"),
#endif
#ifdef BH_KTRACE
      k1s_cfg<3, 32, 3, 4, 1>("xks96c32q3_noload"), k1s_cfg<3, 32, 3, 4, 2>("xks96c32q3_nomfma"),
      k1s_cfg<3, 32, 3, 4, 4>("xks96c32q3_nostore"), k1s_cfg<3, 32, 3, 4, 7>("xks96c32q3_none"),
#endif
  };
}

// k1d: the whole bank [K][OCP] + biases + NW rings of D chunks [KC][32] in LDS; K a whole number of
// chunks, at least D - 1 of them; OH*OW % 4 == 0 and a 16-B aligned input (16-B DMA pieces of 4 pixels
// never straddle two images). splits: 0 = as many blocks per CU as fit (at most 4), 1..4 = blocks per
// CU, 8 = one unit per wave (the whole grid queued)
int launch_k1d(bh_ctx *ctx, const cfg_t &c, GemmArgs &p, uint32_t splits, bool first) {
  const uint32_t KC = (uint32_t)c.dc_ci, D = (uint32_t)c.dc_rin, NW = (uint32_t)c.NT / 64, BM = (uint32_t)c.BM;
  if (p.K % KC || p.K / KC < D - 1)
    return bh::fail(BH_UNSUP, std::string("conv: ") + c.name + " needs input channels a multiple of " +
                                  std::to_string(KC) + ", at least " + std::to_string((D - 1) * KC));
  if (p.OHW % 4 || (uintptr_t)p.b % 16)
    return bh::fail(BH_UNSUP, std::string("conv: ") + c.name + " needs OH*OW % 4 == 0 and a 16-B aligned input");
  const uint32_t ocp = (p.M + BM - 1) / BM * BM, ntm = ocp / BM;
  const uint64_t lds = ((uint64_t)p.K * ocp + (ocp + 63) / 64 * 64 + (uint64_t)NW * D * KC * 32) * 4;
  if (lds > 160 * 1024) return bh::fail(BH_UNSUP, std::string("conv: bank too large for ") + c.name);
  const uint64_t out_bytes = (uint64_t)p.OCOHW * (p.N / p.OHW) * 4;
  if (out_bytes >= 0x7fffff00ull) return bh::fail(BH_UNSUP, "conv: output too large for the k1d kernel");
  p.c_bytes = (uint32_t)out_bytes;
  const uint64_t units = (uint64_t)((p.N + 31) / 32) * ntm;
  if (units >= (1u << 31)) return bh::fail(BH_UNSUP, "conv: k1d grid too large");
  const void *k = (const void *)c.k[A_KVEC][B_DIRECT][0];
  if (hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
    return bh::fail(BH_ERR, "conv: k1d LDS attribute");
  int occ = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k, c.NT, (size_t)lds) != hipSuccess || occ < 1) occ = 1;
  const uint32_t ncu = ctx->prop.multiProcessorCount > 0 ? ctx->prop.multiProcessorCount : 256;
  const uint64_t need = (units + NW - 1) / NW;  // blocks for one unit per wave
  uint64_t G = need;
  if (splits < 8) G = std::min<uint64_t>(need, (uint64_t)ncu * std::min<uint32_t>(splits ? splits : 4, (uint32_t)std::min(occ, 4)));
  p.tbm = ocp;
  p.tiles_m = ntm;
  p.total_it = (uint32_t)units;
  bh::fastdiv f = bh::make_fastdiv(ntm);
  p.tm_m = f.m;
  p.tm_s = f.s;
#ifdef BH_KTRACE
  p.trace = (unsigned long long *)ctx->stamps + 65536;
#endif
  void *args[] = {&p};
  return bh::launch(ctx, k, dim3((uint32_t)G, 1, 1), dim3(c.NT), args, first, true, "conv_k1d", (uint32_t)lds);
}

// Launch a resident-bank 1x1 configuration (p filled by launch_conv with a = packed bank): UNSUP
// unless the shape is a stride-1 unpadded 1x1 conv whose K is a whole number of trips (Q chunks
// of KC channels) and whose bank slice fits the LDS. splits: 0 = two blocks per CU where they
// fit, 1..4 = blocks per CU (a persistent grid: a wave takes every wg-th unit), 8 = one unit per
// wave (the whole grid queued: no wave runs two units while another SIMD idles in the tail).
int launch_k1s(bh_ctx *ctx, const cfg_t &c, GemmArgs &p, uint32_t B, uint32_t KY, uint32_t KX, uint32_t sy,
               uint32_t sx, uint32_t splits, bool first) {
  (void)B;
  if (KY != 1 || KX != 1 || sy != 1 || sx != 1 || p.py || p.px)
    return bh::fail(BH_UNSUP, std::string("conv: ") + c.name + " is for unpadded stride-1 1x1 convs");
  const uint32_t KC = (uint32_t)c.dc_ci, Q = (uint32_t)c.dc_rin, NT = (uint32_t)c.NT;
  if (c.k1d) return launch_k1d(ctx, c, p, splits, first);
  if (p.K % KC || (p.K / KC) % Q)
    return bh::fail(BH_UNSUP, std::string("conv: input channels not a whole number of ") + c.name + " trips");
  if (c.k1r && p.K > (uint32_t)c.k1r)
    return bh::fail(BH_UNSUP, std::string("conv: ") + c.name + " holds at most " + std::to_string(c.k1r) +
                                  " input channels in registers");
  // k1w: a store-wave lane's 4 pixels lie in one image and its 16-B output / residual accesses are aligned
  if (c.k1w && (p.OHW % 4 || (uintptr_t)p.c % 16 || (uintptr_t)p.res % 16))
    return bh::fail(BH_UNSUP, std::string("conv: ") + c.name + " needs OH*OW % 4 == 0 and 16-B aligned output rows");
  // k1n: a lane's gv_cx pixels lie in one image (OH*OW % gv_cx == 0) and its vector loads / stores
  // are aligned
  const uint32_t tn = (uint32_t)c.gv_cx;
  if (c.k1n && tn > 1 &&
      (p.OHW % tn || (uintptr_t)p.b % (4u * tn) || (uintptr_t)p.c % (4u * tn) || (uintptr_t)p.res % (4u * tn)))
    return bh::fail(BH_UNSUP, std::string("conv: ") + c.name + " needs OH*OW % " + std::to_string(tn) +
                                  " == 0 and aligned input / output rows");
  // k1s: the bank slice [IC][OCT] and one [32][36] epilogue staging tile per wave; k1n: the bank
  // slice and the tile's biases (whole 64-float DMAs)
  // k1w: the bank slice padded to whole 64-lane 16-B DMAs, the biases, c.k1w_sl [BM][32] staging slots per
  // compute wave and two counters per compute wave
  const uint32_t nw = NT / 64 - (uint32_t)c.k1w;  // compute waves
  const uint64_t lds = c.k1r  ? 0
                       : c.k1w  ? (((uint64_t)p.K * c.BM / 4 + 63) / 64 * 256 + (uint64_t)((c.BM + 63) / 64) * 64 +
                                (uint64_t)nw * c.k1w_sl * c.BM * 32 + 2 * nw) * 4
                       : c.k1n ? ((uint64_t)p.K * c.BM + (uint64_t)((c.BM + 63) / 64) * 64) * 4
                               : ((uint64_t)p.K * c.BM + (uint64_t)(NT / 64) * 32 * 36) * 4;
  if (lds > 160 * 1024) return bh::fail(BH_UNSUP, std::string("conv: bank slice too large for ") + c.name);
  const uint64_t out_bytes = (uint64_t)p.OCOHW * (p.N / p.OHW) * 4;
  if (out_bytes >= 0x7fffff00ull) return bh::fail(BH_UNSUP, "conv: output too large for the k1s kernel");
  p.c_bytes = (uint32_t)out_bytes;
  const void *k = (const void *)c.k[A_KVEC][B_DIRECT][0];
  if (hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
    return bh::fail(BH_ERR, "conv: k1s LDS attribute");
  int occ = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k, c.NT, (size_t)lds) != hipSuccess || occ < 1) occ = 1;
  const uint32_t oct = (p.M + c.BM - 1) / c.BM;
  const uint32_t npu = (p.N + 32 * (c.k1n ? tn : 1u) - 1) / (32 * (c.k1n ? tn : 1u));
  const bool full = splits >= 8;
  uint32_t bpc = splits && !full ? splits : 2;
  bpc = std::max(1u, std::min<uint32_t>(bpc, (uint32_t)std::min(occ, 4)));
  const uint32_t ncu = ctx->prop.multiProcessorCount > 0 ? ctx->prop.multiProcessorCount : 256;
  // blocks per OC tile: enough waves for every pixel unit, at most the CUs' share; a multiple of 8
  // rounded DOWN where that still leaves a block per XCD: rounding up put G above the resident
  // blocks (264 blocks at one block per CU: the last 8 started when the first ones ended, +50 %)
  uint64_t per = std::max<uint64_t>(1, ((uint64_t)ncu * bpc) / oct);
  per = std::min<uint64_t>(per, (npu + nw - 1) / nw);
  per = per >= 8 ? per / 8 * 8 : 8;
  if (full) per = ((npu + nw - 1) / nw + 7) / 8 * 8;
  const uint64_t G = per * oct;
  if (G >= (1u << 31)) return bh::fail(BH_UNSUP, "conv: k1s grid too large");
  p.tiles_m = oct;
#ifdef BH_KTRACE
  p.trace = (unsigned long long *)ctx->stamps + 65536;
#endif
  void *args[] = {&p};
  return bh::launch(ctx, k, dim3((uint32_t)G, 1, 1), dim3(c.NT), args, first, true, "conv_k1s", (uint32_t)lds);
}

}  // namespace bhk
