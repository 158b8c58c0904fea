// bh_dcm.hip -- direct convolution for stride-1 convs with many input channels (3x3 p1, 5x5 p2:
// most of the conv set's MFMA-bound time).
//
// As an implicit GEMM (the ring kernels) every K row of every stage is a separate 64-column
// dword LDS-DMA gather of one input row segment: a 128-pixel x 32-deep B tile takes 64 DMA
// instructions, 0.31 DMA issues per MFMA, and those issues (not the data) hold the MFMA pipe
// at ~75 % of peak (PMC, profiles/r02). Here a stage is CI INPUT CHANNELS of one tile:
//  * the channels' weights [CI][KY*KX][OCT] (16-B LDS-DMA from the packed k-major bank of
//    bh_conv_filts_pack) and their input strip [CI][RIN][WPM] -- the input rows the tile's
//    pixels touch, at a pitch WPM >= W + px whose tail columns stay zero, rows above / below the
//    image zero (OOB misses), filled by LDS-DMA of row runs (16-B pieces when W % 4 == 0): every
//    input element of the strip is fetched once per tile, not once per filter tap (KY*KX times);
//  * the f32 MFMA runs on the vector datapath, so every other vector instruction of a step is
//    MFMA time lost (PMC + diagnostic builds, profiles/r02): a step is MFMAs plus one vector
//    LDS read per fragment at compile-time offsets -- no address arithmetic, no edge selects (a
//    tap left / right of the image reads a zero tail column or the zero guard);
//  * a tile is OCT = 32*TM output channels x NPX = 128*TN consecutive output pixels of the
//    flattened (image, oy, ox) space -- tiles run across image boundaries, so small images
//    (13x13, 7x7) waste no MFMA rows. The strip's rows are "virtual" padded input rows
//    img*(H+2py) + iy + py: one pixel's taps are one linear offset ky*WPM + kx from its base;
//  * v_mfma_f32_32x32x2_f32 (exact fp32) with A = the strip (MFMA rows: pixels), B = the
//    weights (columns: output channels); lane half h takes channels h*CI/2 .. of the stage, so
//    both halves read at the same compile-time offsets from a per-lane base: a fragment is one
//    ds_read_b32 with an immediate offset, no index arithmetic;
//  * a persistent grid shares the op's (tile, stage) iterations equally between blocks
//    (stream-K, as srk_kernel in bh_ring.hip): tiles cut between blocks are summed by their last
//    arriving block in block order (bitwise reproducible); the DMA ring runs on across tiles.
// Same GemmArgs contract as the other conv kernels (a = packed bank, lda = OC4; b = input;
// OCOHW = the output's image stride, so channel-slab outputs work).
#include "bh_gemm_dev.h"

namespace bhk {
namespace {

// logical block of hardware block bid: blocks b, b+8, ... share an XCD under round-robin
// placement, so give each XCD a contiguous run of iterations (its L2 sees neighbouring tiles)
__device__ __forceinline__ uint32_t dcm_lb(uint32_t bid, uint32_t G) {
  const uint32_t xcd = bid & 7, q = G >> 3, r = G & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

// Strip: [CI][RIN][WPM], WPM >= W + px; columns W .. WPM-1 of every row stay zero (misses), so a
// tap left of the image wraps into the previous row's zero tail (a zero guard precedes the strip
// for its first row) and a tap right of it reads this row's tail: no per-step select. V4: rows in
// 16-B pieces (W % 4 == 0), else dword elements.
// WO wave groups of 4 along the output channels (WO = 2: 8 waves, two per SIMD, sharing one
// stage); a wave owns 32*TN pixels (wave % 4) x 32*TM output channels (group wave / 4).
// DBG (diagnostic builds only, see dcm_cfgs): bit 0 = no DMA after the prologue, bit 1 = no MFMA,
// bit 3 = no LDS fragment reads
template <int KY, int KX, int WPM, int RIN, int V4, int CI, int TM, int TN, int WO, int D, int DBG = 0>
__global__ __launch_bounds__(256 * WO) void dcm_kernel(GemmArgs p) {
  constexpr int NW = 4 * WO, NT = 64 * NW;
  constexpr int NPX = 4 * 32 * TN, OCT = 32 * TM * WO;
  constexpr int KK = KY * KX, CH2 = CI / 2, STEPS = CH2 * KK;
  constexpr int WPC = CI * KK * OCT / 4;                 // 16-B weight pieces per stage
  constexpr int LWA = (WPC + NW * 64 - 1) / (NW * 64);   // weight DMA instructions per wave
  constexpr int WREG = LWA * NW * 256;                   // floats
  // P1 (1x1, no padding): a channel's strip is exactly the tile's NPX pixels, [CI][NPX]
  constexpr bool P1 = KY == 1 && KX == 1;
  constexpr int SLICE = P1 ? NPX : RIN * WPM;            // one channel's strip
  static_assert(WPM % 4 == 0, "16-B aligned rows");
  constexpr int PW = V4 ? 4 : 1;                         // floats per strip DMA lane
  constexpr int LWB = (CI * SLICE / PW + NW * 64 - 1) / (NW * 64);
  constexpr int SREG = LWB * NW * 64 * PW;
  constexpr int BREG = NW * 64;                          // the tile's biases, one DMA per wave
  constexpr int GZ = 4;                                  // zero guard before the strip
  constexpr int SLOT = WREG + GZ + SREG + BREG;
  constexpr int LW = LWA + LWB + 1;
  static_assert(CI % 2 == 0, "channel halves");
  static_assert(D >= 2 && (D - 2) * LW <= 63, "vmcnt range");
  static_assert(OCT % 4 == 0 && OCT <= BREG, "16-B weight pieces, biases of one tile");
  constexpr int PF = TM * TN >= 4 ? 2 : 3;  // LDS fragment prefetch (steps)
  static_assert(TM == 1 || TM == 2 || TM == 4, "weight fragments: one b32 / b64 / b128 read");
  constexpr int IS = STEPS > 3 ? STEPS / 2 : 1;                   // steps the next stage's DMAs spread over
  constexpr int NQ = TM * TN * 4;                                 // float4 pieces of a lane's accumulators

  // one __shared__ array only (a second object makes hipcc wait vmcnt(0) at ds_reads)
  __shared__ __attribute__((aligned(16))) float smem[D * SLOT + 4];
  uint32_t *const flag = (uint32_t *)(smem + D * SLOT);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int kh = lane >> 5, li = lane & 31;
  const int wp = wave & 3, wo = wave >> 2;  // pixel group, output-channel group
  KT(0);

  const uint32_t lb = dcm_lb(blockIdx.x, gridDim.x);
  const uint32_t it0 = lb * p.ipb, it1 = min(p.total_it, it0 + p.ipb);
  const uint32_t Hp = p.H + 2 * p.py;
  // the strip guards stay zero (no DMA targets them); the first stage's barrier orders these
  // writes before any read
  if (tid < D * GZ) smem[(tid / GZ) * SLOT + WREG + tid % GZ] = 0.0f;

  // tile t: OC tile fastest (consecutive tiles share the input strip through L2)
  auto tile_of = [&](uint32_t t, uint32_t &oc0, uint32_t &n0) {
    const uint32_t pt = fdiv(t, p.tm_m, p.tm_s);  // tiles_m = OC tiles
    oc0 = (t - pt * p.tiles_m) * OCT;
    n0 = pt * NPX;
  };
  // virtual padded input row of the first strip row of the tile starting at pixel n0
  auto vrow0 = [&](uint32_t n0) -> uint32_t {
    const uint32_t img = fdiv(n0, p.ohw_m, p.ohw_s), pix = n0 - img * p.OHW;
    return img * Hp + fdiv(pix, p.ow_m, p.ow_s);
  };

  // ---- tile-independent per-lane parts of the DMA source offsets
  const __amdgpu_buffer_rsrc_t rsw = make_rsrc(p.a, p.a_bytes);
  const __amdgpu_buffer_rsrc_t rsi = make_rsrc(p.b, p.b_bytes);
  const __amdgpu_buffer_rsrc_t rsbias = make_rsrc(p.bias, p.bias ? p.M * 4u : 0u);
  // weight piece e of the [CI][KK][OCT] image: packed-bank row tap*IC + (ic0 + c), column 4*c4
  uint32_t wrel[LWA], wc4[LWA];  // wc4 = 0xffff: a piece past the image (never loads)
#pragma unroll
  for (int j = 0; j < LWA; ++j) {
    const uint32_t e = (uint32_t)((wave * LWA + j) * 64 + lane);
    const uint32_t row = e / (OCT / 4), c4 = e % (OCT / 4);
    const uint32_t c = row / KK, tap = row % KK;
    wc4[j] = row < (uint32_t)(CI * KK) ? 4 * c4 : 0xffffu;
    wrel[j] = ((tap * p.IC + c) * p.lda + 4 * c4) * 4u;
  }
  // strip DMA lane e of the [CI][RIN][WPM] image: channel c, strip row r, input columns x ..
  // x + PW - 1 (columns at or past W: never loaded, zero)
  uint32_t sr[LWB], sx[LWB];  // sx = channel offset + input column, or 0xffffffff (never loads)
#pragma unroll
  for (int j = 0; j < LWB; ++j) {
    const uint32_t e = (uint32_t)((wave * LWB + j) * 64 + lane);
    const uint32_t c = e / (SLICE / PW), rem = e % (SLICE / PW);
    if constexpr (P1) {  // pixel slot rem*PW of the tile, channel c
      sr[j] = rem * PW;
      sx[j] = c < (uint32_t)CI ? c * p.HW : 0xffffffffu;
    } else {
      const uint32_t r = rem / (WPM / PW), x = (rem % (WPM / PW)) * PW;
      sr[j] = r;
      sx[j] = ((c < (uint32_t)CI) & (x < p.W)) ? c * p.HW + x : 0xffffffffu;
    }
  }
  // the per-lane DMA offsets of the tile being issued (channel 0 of the stage; OOB where the
  // element is padding, past the images or past the bank), recomputed only when the issue side
  // enters a new tile; a stage adds its channel group's offset as the scalar soffset, so issuing
  // a stage costs no vector work (every VALU op between f32 MFMAs is MFMA time lost)
  uint32_t wvo[LWA], srel[LWB], bvo = OOB;
  uint32_t ls_tile = 0xffffffffu;
  // a dead stage (past the block's iteration range) reads through zero-extent descriptors: all
  // misses (zeros, no memory traffic), so every wave always has the same number in flight
  const __amdgpu_buffer_rsrc_t rnull = make_rsrc(p.b, 0u);

  // scalar parts of iteration `it` (tile it / ipt, channel group it % ipt)
  auto plan = [&](uint32_t it, uint32_t &sw, uint32_t &ss) -> bool {
    const uint32_t t = fdiv(it, p.ipt_m, p.ipt_s), ic0 = (it - t * p.ipt) * CI;
    if (t != ls_tile) {  // uniform
      uint32_t oc0, n0;
      tile_of(t, oc0, n0);
      const uint32_t wlim = p.lda - min(oc0, p.lda);
#pragma unroll
      for (int j = 0; j < LWA; ++j) wvo[j] = oob_unless(wc4[j] < wlim, wrel[j] + oc0 * 4u);
      if constexpr (P1) {
#pragma unroll
        for (int j = 0; j < LWB; ++j) {
          // PW pixels from n0 + sr[j]: one image (OHW % PW == 0), past the op: misses
          const uint32_t n = n0 + sr[j];
          const uint32_t img = fdiv(n, p.ohw_m, p.ohw_s);
          srel[j] = oob_unless((sx[j] != 0xffffffffu) & (n < p.N), (img * p.ICHW + sx[j] + n - img * p.OHW) * 4u);
        }
      } else {
        const uint32_t v0 = vrow0(n0);
#pragma unroll
        for (int j = 0; j < LWB; ++j) {
          const uint32_t vr = v0 + sr[j];
          const uint32_t img = fdiv(vr, p.kyx_m, p.kyx_s);  // kyx fastdiv = H + 2py here
          const uint32_t iy = vr - img * Hp - p.py;         // wraps (misses) in the top padding
          const bool ok = (sx[j] != 0xffffffffu) & (iy < p.H) & (img < p.tiles_n);  // tiles_n = images
          srel[j] = oob_unless(ok, (img * p.ICHW + iy * p.W + sx[j]) * 4u);
        }
      }
      const uint32_t bo = (uint32_t)(64 * wave + lane);
      bvo = oob_unless((bo < (uint32_t)OCT) & (oc0 + bo < p.M), (oc0 + bo) * 4u);
      ls_tile = t;
    }
    sw = ic0 * p.lda * 4u;
    ss = ic0 * p.HW * 4u;
    return it >= it1;
  };
  auto issue_one = [&](int q, int slot, uint32_t sw, uint32_t ss, bool dead) {
    float *const base = smem + slot * SLOT;
    if (q < LWA) dma16s(dead ? rnull : rsw, base + (wave * LWA + q) * 256, wvo[q], sw);
    else if (q < LWA + LWB) {
      if constexpr (V4) dma16s(dead ? rnull : rsi, base + WREG + GZ + (wave * LWB + q - LWA) * 256, srel[q - LWA], ss);
      else dma4s(dead ? rnull : rsi, base + WREG + GZ + (wave * LWB + q - LWA) * 64, srel[q - LWA], ss);
    }
    else dma4(dead ? rnull : rsbias, base + WREG + GZ + SREG + 64 * wave, bvo);
  };

  f32x16 acc[TM][TN];
  uint32_t poff[TN];  // this lane's pixels' strip offsets in the current tile (bytes), half included

  // one stage = CI channels of one tile: STEPS steps of TM x TN MFMAs; iteration it_issue's DMAs
  // go out over the first IS steps; LDS fragments are read PF steps ahead
  auto compute = [&](int slot, int islot, uint32_t it_issue) {
    uint32_t sw, ss;
    const bool dead = plan(it_issue, sw, ss);
    // a lane's TM weight columns are adjacent (MFMA tile t, lane li: output channel TM*li + t of
    // the wave's group): one ds_read_b64 / b128 per step instead of TM ds_read_b32 (b32 reads
    // reach their rate only at ~4 waves per SIMD)
    const float *const Ab = smem + slot * SLOT + kh * (CH2 * KK * OCT) + wo * 32 * TM + TM * li;
    const char *const Sb = (const char *)(smem + slot * SLOT + WREG + GZ);
    auto frag = [&](int s, typename fvec<TM>::t &a, float (&b)[TN]) {
      const int cc = s / KK, tap = s % KK;
      if constexpr ((DBG & 8) != 0) {  // diagnostic build: no LDS fragment reads
        a = typename fvec<TM>::t{};
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) b[tn] = (float)(s + tn);
        return;
      }
      a = *(const typename fvec<TM>::t *)&Ab[(cc * KK + tap) * OCT];
#pragma unroll
      for (int tn = 0; tn < TN; ++tn)
        b[tn] = *(const float *)(Sb + poff[tn] + (cc * SLICE + (tap / KX) * WPM + tap % KX) * 4);
    };
    typename fvec<TM>::t a[PF + 1];
    float b[PF + 1][TN];
#pragma unroll
    for (int s = 0; s < PF; ++s) frag(s, a[s], b[s]);
#pragma unroll
    for (int s = 0; s < STEPS; ++s) {
      if (s + PF < STEPS) frag(s + PF, a[(s + PF) % (PF + 1)], b[(s + PF) % (PF + 1)]);
      __builtin_amdgcn_sched_barrier(0);  // keep the prefetch ahead of this step's MFMAs
      const float *const bm = b[s % (PF + 1)];
      if constexpr ((DBG & 2) != 0) {  // diagnostic build: no MFMA (the fragments are still consumed)
#pragma unroll
        for (int t = 0; t < TM; ++t)
#pragma unroll
          for (int tn = 0; tn < TN; ++tn) acc[t][tn][0] += bm[tn] * vget<TM>(a[s % (PF + 1)], t);
      } else {
#pragma unroll
        for (int t = 0; t < TM; ++t)
#pragma unroll
          for (int tn = 0; tn < TN; ++tn)
            acc[t][tn] = __builtin_amdgcn_mfma_f32_32x32x2f32(bm[tn], vget<TM>(a[s % (PF + 1)], t), acc[t][tn], 0, 0, 0);
      }
      if constexpr ((DBG & 1) == 0) {  // diagnostic build 1: no DMA after the prologue
#pragma unroll
        for (int q = (s * LW + IS - 1) / IS; q < ((s + 1) * LW + IS - 1) / IS && q < LW; ++q)
          issue_one(q, islot, sw, ss, dead);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  const __amdgpu_buffer_rsrc_t rso = make_rsrc(p.c, p.c_bytes);
  const __amdgpu_buffer_rsrc_t rsr = make_rsrc(p.res, p.res ? p.c_bytes : 0u);
  // float4 pixel quads, at any dword alignment (the output row of a channel starts at m * OHW);
  // a quad running past its image's last pixel (OHW % 4 != 0) goes element by element. Element
  // stores for every quad scatter each wave instruction over 32 rows: 4x the store instructions
  // and line writes of the quads (the 13x13 / 27x27 ops)
  const bool vec = !p.res;

  // bias, residual, ReLU and store of a tile's values: v[q], q = (t, tn, gq) holds output channel
  // oc0 + wo*32*TM + TM*li + t, pixels n0 + wp*32*TN + 32 tn + 8 gq + 4 kh + e (e = 0..3)
  auto store_tile = [&](uint32_t oc0, uint32_t n0, const float *Lb, f32x4v (&v)[NQ]) {
#pragma unroll
    for (int t = 0; t < TM; ++t) {
      const uint32_t m = oc0 + (uint32_t)(wo * 32 * TM + TM * li + t);
      const float bb = Lb[wo * 32 * TM + TM * li + t];
#pragma unroll
      for (int tn = 0; tn < TN; ++tn)
#pragma unroll
        for (int gq = 0; gq < 4; ++gq) {
          f32x4v x = v[(t * TN + tn) * 4 + gq];
          const uint32_t nq = n0 + (uint32_t)(wp * 32 * TN + 32 * tn + 8 * gq + 4 * kh);
          const uint32_t img = fdiv(nq, p.ohw_m, p.ohw_s), pix = nq - img * p.OHW;
          if (vec && pix + 4 <= p.OHW) {
            const uint32_t o = oob_unless((m < p.M) & (nq < p.N), (img * p.OCOHW + m * p.OHW + pix) * 4u);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              x[e] += bb;
              x[e] = (p.relu && x[e] < 0.0f) ? 0.0f : x[e];
            }
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) uint32_t, x),
                                                   rso, o, 0, AUX_OUT);
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const uint32_t n = nq + e;
              const uint32_t img = fdiv(n, p.ohw_m, p.ohw_s);
              const uint32_t o = oob_unless((m < p.M) & (n < p.N), (img * p.OCOHW + m * p.OHW + n - img * p.OHW) * 4u);
              float y = x[e] + bb;
              if (p.res) y += __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rsr, o, 0, 0));
              y = (p.relu && y < 0.0f) ? 0.0f : y;
              __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, y), rso, o, 0, AUX_OUT);
            }
          }
        }
    }
  };

  // tile t is done in this block (iterations [max(it0, t*ipt), min(it1, (t+1)*ipt)) are in acc):
  // store it, or hand the partial tile over through this block's slab and the tile's ticket
  auto finish_tile = [&](uint32_t t, int cslot) {
    uint32_t oc0, n0;
    tile_of(t, oc0, n0);
    const float *const Lb = smem + cslot * SLOT + WREG + GZ + SREG;
    f32x4v v[NQ];
#pragma unroll
    for (int t2 = 0; t2 < TM; ++t2)
#pragma unroll
      for (int tn = 0; tn < TN; ++tn)
#pragma unroll
        for (int gq = 0; gq < 4; ++gq)
#pragma unroll
          for (int e = 0; e < 4; ++e) v[(t2 * TN + tn) * 4 + gq][e] = acc[t2][tn][4 * gq + e];
    const uint32_t tb = t * p.ipt;
    if (tb >= it0 && tb + p.ipt <= it1) {
      store_tile(oc0, n0, Lb, v);
      return;
    }
    // partial tile: slab (block, slot 0 = the block's first tile, 1 = its last), write-through
    const uint32_t sl = (t == fdiv(it0, p.ipt_m, p.ipt_s)) ? 0u : 1u;
    const __amdgpu_buffer_rsrc_t rw = make_rsrc(p.ws + ((size_t)lb * 2 + sl) * (NQ * NT * 4), NQ * NT * 16);
#pragma unroll
    for (int q = 0; q < NQ; ++q)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) uint32_t, v[q]), rw,
                                             (uint32_t)((q * NT + tid) * 16), 0, AUX_SC1);
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
#pragma unroll
    for (int q = 0; q < NQ; ++q) v[q] = f32x4v{0.0f, 0.0f, 0.0f, 0.0f};
    for (uint32_t b = b0; b <= b1; ++b) {  // block order = k order: bitwise reproducible
      const uint32_t s2 = (b == b0 && t != fdiv(b * p.ipb, p.ipt_m, p.ipt_s)) ? 1u : 0u;
      const uint32_t base = (b * 2 + s2) * (uint32_t)(NQ * NT * 16);
      f32x4v x[NQ];
#pragma unroll
      for (int q = 0; q < NQ; ++q)
        x[q] = __builtin_bit_cast(f32x4v, __builtin_amdgcn_raw_buffer_load_b128(rall, base + (uint32_t)((q * NT + tid) * 16),
                                                                                 0, AUX_SC1));
#pragma unroll
      for (int q = 0; q < NQ; ++q) v[q] += x[q];
    }
    store_tile(oc0, n0, Lb, v);
  };

  // ---- prologue: iterations it0 .. it0+D-2 in flight
#pragma unroll
  for (int s = 0; s < D - 1; ++s) {
    uint32_t sw, ss;
    const bool dead = plan(it0 + (uint32_t)s, sw, ss);
#pragma unroll
    for (int q = 0; q < LW; ++q) issue_one(q, s, sw, ss, dead);
  }
  int slot = 0;
  uint32_t it = it0;
  // outer loop over the block's tiles, inner over the tile's channel groups in this block's
  // range (nested: the accumulators stay in AGPRs); the ring runs on across tiles
  while (it < it1) {
    const uint32_t t = fdiv(it, p.ipt_m, p.ipt_s);
    const uint32_t iend = min(it1, (t + 1) * p.ipt);
    uint32_t oc0, n0;
    tile_of(t, oc0, n0);
    const uint32_t v0 = P1 ? 0u : vrow0(n0);
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) {
      const uint32_t n = n0 + (uint32_t)(wp * 32 * TN + 32 * tn + li);
      if constexpr (P1) {  // the pixel's slot of the tile
        poff[tn] = (uint32_t)(wp * 32 * TN + 32 * tn + li) * 4u + (uint32_t)kh * CH2 * SLICE * 4u;
        continue;
      }
      const uint32_t img = fdiv(n, p.ohw_m, p.ohw_s), pix = n - img * p.OHW;
      const uint32_t oy = fdiv(pix, p.ow_m, p.ow_s), ox = pix - oy * p.OW;
      // pixels past the op read strip position 0 (their results are dropped)
      // (ox - px may be negative: the guard / the previous row's zero tail)
      poff[tn] = n < p.N ? ((img * Hp + oy - v0) * WPM + ox - p.px) * 4u : 0u;
      poff[tn] += (uint32_t)kh * CH2 * SLICE * 4u;
    }
#pragma unroll
    for (int t2 = 0; t2 < TM; ++t2)
#pragma unroll
      for (int tn = 0; tn < TN; ++tn)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[t2][tn][r] = 0.0f;
    int cslot = 0;
    for (; it < iend; ++it) {
      vm_wait<(DBG & 1) ? 0 : (D - 2) * LW>();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();  // stage it landed for all waves; all done reading it-1
      asm volatile("" ::: "memory");
      if (it == it0) KT(1);
      compute(slot, slot == 0 ? D - 1 : slot - 1, it + D - 1);  // + stage it+D-1 into slot (it-1) % D
      cslot = slot;
      slot = slot == D - 1 ? 0 : slot + 1;
    }
    if (t == fdiv(it0, p.ipt_m, p.ipt_s)) KT(2);
    finish_tile(t, cslot);
  }
  vm_wait<0>();
#ifdef BH_KTRACE
  KT(4);
#endif
}

template <int KY, int KX, int WPM, int RIN, int V4, int CI, int TM, int TN, int WO, int D, int DBG = 0>
cfg_t dcm_cfg(const char *name) {
  cfg_t c{name, 32 * TM * WO, 128 * TN, CI * KY * KX, 256 * WO, {}, 1};
  c.k[A_KVEC][B_DIRECT][0] = dcm_kernel<KY, KX, WPM, RIN, V4, CI, TM, TN, WO, D, DBG>;
  c.dc = 2;
  c.dc_ky = KY;
  c.dc_kx = KX;
  c.dc_s = V4;  // dcm: 16-B strip pieces (rows of W % 4 == 0)
  c.dc_wpm = WPM;
  c.dc_rin = RIN;
  c.dc_ci = CI;
  return c;
}

}  // namespace

std::vector<cfg_t> dcm_cfgs() {
  // <KY, KX, WPM, RIN, V4, CI, TM, TN, WO, D>: strip pitch / rows by input width class; x64 tiles
  // fit two blocks per CU, w8 (two wave groups) puts two waves per SIMD on one 128-channel stage
  return {
      // 3x3 p1: 13x13 / 14x14 (pitch 16, <= 16 rows), 6x6 / 7x7 (8, <= 44 rows over 4-5 images),
      // 28x28 (32, 16-B pieces), 56x56 (60, 16-B pieces)
      dcm_cfg<3, 3, 16, 16, 0, 8, 2, 1, 1, 2>("dm3w16x64c8"),
      dcm_cfg<3, 3, 16, 16, 0, 8, 2, 1, 2, 3>("dm3w16x128c8w8"),
      dcm_cfg<3, 3, 16, 16, 0, 4, 4, 1, 1, 3>("dm3w16x128c4"),
      dcm_cfg<3, 3, 8, 44, 0, 8, 2, 1, 1, 2>("dm3w8x64c8"),
      dcm_cfg<3, 3, 8, 44, 0, 8, 2, 1, 2, 2>("dm3w8x128c8w8"),
      dcm_cfg<3, 3, 32, 10, 1, 8, 2, 1, 1, 2>("dm3w32x64c8"),
      dcm_cfg<3, 3, 32, 10, 1, 8, 2, 1, 2, 2>("dm3w32x128c8w8"),
      dcm_cfg<3, 3, 60, 8, 1, 8, 2, 1, 1, 2>("dm3w60x64c8"),
      dcm_cfg<3, 3, 60, 8, 1, 8, 2, 1, 2, 2>("dm3w60x128c8w8"),
      dcm_cfg<3, 3, 60, 8, 1, 4, 2, 1, 1, 3>("dm3w60x64c4"),
      // 5x5 p2: 27x27 (pitch 32, dword), 28x28 (32, 16-B pieces), 14x14 (16, <= 20 rows)
      dcm_cfg<5, 5, 32, 14, 0, 4, 2, 1, 1, 2>("dm5w32x64c4"),
      dcm_cfg<5, 5, 32, 14, 0, 4, 2, 1, 2, 2>("dm5w32x128c4w8"),
      dcm_cfg<5, 5, 32, 14, 1, 4, 2, 1, 1, 2>("dm5w32vx64c4"),
      dcm_cfg<5, 5, 16, 20, 0, 4, 2, 1, 1, 2>("dm5w16x64c4"),
      // 256-pixel tiles (TN = 2): half the filter-bank DMA per MFMA (the bank is re-fetched for
      // every pixel tile: the largest cost left in the diagnostic builds)
      dcm_cfg<3, 3, 16, 28, 0, 8, 2, 2, 2, 2>("dm3w16x128n256c8w8"),
      dcm_cfg<3, 3, 16, 28, 0, 8, 2, 2, 1, 2>("dm3w16x64n256c8"),
      dcm_cfg<3, 3, 8, 72, 0, 8, 2, 2, 2, 2>("dm3w8x128n256c8w8"),
      dcm_cfg<3, 3, 32, 14, 1, 8, 2, 2, 1, 2>("dm3w32x64n256c8"),
      dcm_cfg<3, 3, 60, 10, 1, 8, 2, 2, 1, 2>("dm3w60x64n256c8"),
      dcm_cfg<5, 5, 32, 20, 0, 4, 2, 2, 1, 2>("dm5w32x64n256c4"),
      dcm_cfg<5, 5, 32, 20, 0, 4, 2, 2, 2, 2>("dm5w32x128n256c4w8"),
      // 1x1: CI channels of the tile's 128 pixels per stage (16-B pieces when OH*OW % 4 == 0)
      dcm_cfg<1, 1, 0, 0, 1, 32, 2, 1, 1, 3>("dm1vx64c32"),
      dcm_cfg<1, 1, 0, 0, 1, 32, 2, 1, 2, 3>("dm1vx128c32w8"),
      dcm_cfg<1, 1, 0, 0, 1, 16, 2, 1, 1, 4>("dm1vx64c16"),
      dcm_cfg<1, 1, 0, 0, 0, 32, 2, 1, 1, 3>("dm1x64c32"),
      dcm_cfg<1, 1, 0, 0, 0, 32, 2, 1, 2, 3>("dm1x128c32w8"),
      // short-K 1x1 (K = 64 / 96 / 128): the whole K, or half, in one stage -- one barrier per
      // tile, the ring runs across tiles
      dcm_cfg<1, 1, 0, 0, 1, 64, 2, 1, 1, 2>("dm1vx64c64"),
      dcm_cfg<1, 1, 0, 0, 1, 64, 2, 1, 1, 3>("dm1vx64c64d3"),
      dcm_cfg<1, 1, 0, 0, 1, 96, 2, 1, 1, 2>("dm1vx64c96"),
      dcm_cfg<1, 1, 0, 0, 1, 64, 2, 1, 2, 2>("dm1vx128c64w8"),
#ifdef BH_KTRACE
      // diagnostic builds (instrumented library only; wrong results by design)
      dcm_cfg<3, 3, 16, 16, 0, 8, 2, 1, 1, 2, 1>("xdm3w16x64c8_nodma"),
      dcm_cfg<3, 3, 16, 16, 0, 8, 2, 1, 1, 2, 2>("xdm3w16x64c8_nomfma"),
      dcm_cfg<3, 3, 16, 16, 0, 8, 2, 1, 1, 2, 3>("xdm3w16x64c8_none"),
      dcm_cfg<3, 3, 16, 16, 0, 8, 2, 1, 2, 3, 1>("xdm3w16x128c8w8_nodma"),
      dcm_cfg<3, 3, 16, 16, 0, 8, 2, 1, 2, 3, 2>("xdm3w16x128c8w8_nomfma"),
      dcm_cfg<3, 3, 16, 16, 0, 8, 2, 1, 1, 2, 9>("xdm3w16x64c8_nodma_noread"),
      dcm_cfg<3, 3, 16, 16, 0, 8, 2, 1, 1, 2, 8>("xdm3w16x64c8_noread"),
#endif
  };
}

// Launch a multi-channel direct-conv configuration (p filled by launch_conv with a = packed
// bank): UNSUP unless the shape is this instantiation's kernel at stride 1 with IC a multiple
// of its channel group and every tile's strip fitting. splits: 0 / 1..4 = blocks per CU with
// the (tile, channel group) iterations dealt equally; 5..8 = blocks per CU 1..4, whole tiles
// per block.
int launch_dcm(bh_ctx *ctx, const cfg_t &c, GemmArgs &p, uint32_t B, uint32_t KY, uint32_t KX, uint32_t sy,
               uint32_t sx, uint32_t splits, bool first) {
  if ((int)KY != c.dc_ky || (int)KX != c.dc_kx || sy != 1 || sx != 1 || p.py >= KY)
    return bh::fail(BH_UNSUP, std::string("conv: direct config ") + c.name + " is for another kernel / stride");
  if (p.IC % (uint32_t)c.dc_ci)
    return bh::fail(BH_UNSUP, std::string("conv: input channels not a multiple of ") + c.name + "'s group");
  const uint32_t npx = (uint32_t)c.BN, OW = p.OW, OHW = p.OHW, Hp = p.H + 2 * p.py;
  const bool p1 = KY == 1 && KX == 1;
  if (p1) {  // 1x1: strip = the tile's pixels; 16-B pieces need quads inside one image
    if (p.py || p.px || (c.dc_s && OHW % 4))
      return bh::fail(BH_UNSUP, std::string("conv: padded 1x1 / pixel quads across images for ") + c.name);
  } else if (p.W + p.px > (uint32_t)c.dc_wpm || p.px > 4 || (c.dc_s && p.W % 4)) {
    // strip pitch: the row plus a zero tail wide enough for the horizontal padding
    return bh::fail(BH_UNSUP, std::string("conv: input rows do not fit the strip of ") + c.name);
  }
  const uint32_t ptiles = (p.N + npx - 1) / npx;
  // strip rows the worst pixel tile touches (virtual padded rows img*Hp + oy .. + KY - 1)
  uint32_t rin = 0;
  for (uint32_t t = 0; t < ptiles; ++t) {
    const uint32_t a = t * npx, b = std::min(p.N, a + npx) - 1;
    const uint32_t va = (a / OHW) * Hp + (a % OHW) / OW, vb = (b / OHW) * Hp + (b % OHW) / OW;
    rin = std::max(rin, vb - va + KY);
  }
  if (!p1 && rin > (uint32_t)c.dc_rin)
    return bh::fail(BH_UNSUP, std::string("conv: pixel tile's input strip too large for ") + c.name);
  const uint64_t out_bytes = (uint64_t)B * p.OCOHW * 4;
  if (out_bytes >= 0x7fffff00ull) return bh::fail(BH_UNSUP, "conv: output too large for the direct kernel");
  p.c_bytes = (uint32_t)out_bytes;
  const uint32_t octiles = (p.M + c.BM - 1) / c.BM;
  const uint32_t ipt = p.IC / (uint32_t)c.dc_ci;
  const uint64_t ntile = (uint64_t)ptiles * octiles, total = ntile * ipt;
  if (total >= (1u << 31)) return bh::fail(BH_UNSUP, "conv: too many iterations");
  const void *k = (const void *)c.k[A_KVEC][B_DIRECT][0];
  int occ = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k, c.NT, 0) != hipSuccess || occ < 1) occ = 1;
  const bool whole = splits > 4;
  uint32_t bpc = splits ? (whole ? splits - 4 : splits) : 2;
  bpc = std::max(1u, std::min<uint32_t>(bpc, (uint32_t)std::min(occ, 4)));
  const uint32_t ncu = ctx->prop.multiProcessorCount > 0 ? ctx->prop.multiProcessorCount : 256;
  uint64_t G = (uint64_t)ncu * bpc;
  uint32_t ipb = (uint32_t)((total + G - 1) / G);
  if (whole) ipb = (uint32_t)((ntile + G - 1) / G) * ipt;
  G = (total + ipb - 1) / ipb;
  p.ipt = ipt;
  p.ipb = ipb;
  p.total_it = (uint32_t)total;
  p.tiles_m = octiles;
  p.tiles_n = B;  // images (strip rows past the last image miss)
  bh::fastdiv f = bh::make_fastdiv(ipt);
  p.ipt_m = f.m;
  p.ipt_s = f.s;
  f = bh::make_fastdiv(octiles);
  p.tm_m = f.m;
  p.tm_s = f.s;
  f = bh::make_fastdiv(Hp);
  p.kyx_m = f.m;
  p.kyx_s = f.s;
  int rc = ensure_ws(ctx, (size_t)2 * G * c.BM * c.BN * 4);  // two tile slabs per block
  if (rc == BH_OK) rc = ensure_cnt(ctx, (size_t)ntile);
  if (rc != BH_OK) return rc;
  p.ws = (float *)ctx->ws;
  p.cnt = (uint32_t *)ctx->cnt;
#ifdef BH_KTRACE
  p.trace = (unsigned long long *)ctx->stamps + 65536;
#endif
  void *args[] = {&p};
  return bh::launch(ctx, k, dim3((uint32_t)G, 1, 1), dim3(c.NT), args, first, true, "conv_direct_mc");
}

}  // namespace bhk
