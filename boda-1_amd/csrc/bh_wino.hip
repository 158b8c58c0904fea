// bh_wino.hip -- Winograd F(2x2, 3x3) convolution for stride-1 3x3 convs (pad 0 or 1).
//
// The conv set's 3x3 stride-1 layers (GoogLeNet 3x3 branches, AlexNet conv3-5, NiN, VGG, the
// ResNet bottleneck 3x3) are most of its MFMA-bound time (BASELINE.md §1.2 model: 2*M*N*K with
// K = IC*9). F(2x2, 3x3) computes each 2x2 output tile from a 4x4 input patch with 16
// elementwise products per (input, output) channel pair instead of 36: 2.25x fewer MFMA flops.
// Boda itself reaches this algorithm through its cudnn_conv comparator (src/rtc_prof.cc:314-319
// widens the compare tolerance for cuDNN's 3x3 Winograd); here it is a variant of the
// conv op like the reference's tconv / k1conv choices (src/cnn_op.cc:16-331), routed per shape
// by the tuning table only where it is faster, and checked against the direct-accumulation
// oracle at the same tolerances as every other route.
//
//   U = G g G^T (filters, 4x4 per (oc, ic)), V = B^T d B (input patch), M = sum_ic U . V,
//   Y = A^T M A (2x2 outputs), with
//   G = [1 0 0; .5 .5 .5; .5 -.5 .5; 0 0 1], B^T = [1 0 -1 0; 0 1 1 0; 0 -1 1 0; 0 1 0 -1],
//   A^T = [1 1 1 0; 0 1 -1 -1].
//
// MI355X structure (one fused kernel: nothing of U, V or M goes to HBM):
//  * the filter transform is part of the filter-bank pack (bh_conv_filts_pack, Boda's
//    xpose_filts role: once per net / op list, untimed as in the reference, src/rtc_prof.cc:93-99):
//    U [IC4][OC32][16], each (ic, oc) row's four 4-float chunks rotated by (oc >> 2) & 3;
//  * a block owns OCT = 32*NWO output channels x TT = 32*NWT Winograd tiles of the flattened
//    (image, tile row, tile column) space; a stage is WCI = 4 input channels. The stage's input
//    strip [4][RIN][WPM] -- the "virtual" padded rows the tiles' patches touch (img*VH + iy + py,
//    rows outside an image read as zero) at a pitch WPM > W whose zero tail also serves a patch's
//    left neighbour -- arrives by 16-B LDS-DMA in a D-slot ring;
//  * stage it+2's patches are transformed during stage it into a triple-buffered V [4][TT][16]
//    (each (tile, channel) once per block, shared by the NWO channel waves);
//  * a wave owns 32 channels x 32 tiles x all 16 Winograd positions: v_mfma_f32_32x32x2_f32
//    (exact fp32), A = U straight from L2 into registers, B = V fragments from LDS, both loaded
//    for stage it+1 in four groups right after stage it's MFMA group that freed their registers;
//    16 accumulator tiles (256 AGPRs, one wave per SIMD); every lane then holds all 16 positions
//    of its (channel, tile) pairs, so the output transform, bias, residual and ReLU run in
//    registers;
//  * a persistent stream-K grid deals the (tile, stage) iterations equally between blocks (as
//    bh_dcm.hip); a tile cut between blocks is summed after the output transform (linear) by
//    its last-arriving block in block order: bitwise reproducible.
#include <type_traits>

#include "bh_gemm_dev.h"

namespace bhk {

struct WgArgs {
  const float *u;    // Winograd bank [IC4][OC32][16] (rotated chunks)
  const float *in;   // B x IC x H x W
  float *out;        // image stride OCOHW (channel slabs)
  const float *bias; // OC or null
  const float *res;  // laid out like out, or null
  float *ws;         // stream-K slabs, two per block
  uint32_t *cnt;     // arrival tickets, one per tile
  uint32_t u_bytes, in_bytes, out_bytes;
  uint32_t OC, OC32, IC, B, H, W, py, px, OH, OW, OHW, HW, ICHW, OCOHW;
  uint32_t TW, TPI, VH, T;   // tiles per tile row / per image, virtual rows per image, tiles in all
  uint32_t WPM, RW;          // strip pitch, RIN * WPM
  uint32_t tw_m, tw_s, tpi_m, tpi_s, vh_m, vh_s, wpm_m, wpm_s, rw_m, rw_s;
  uint32_t tiles_m, tm_m, tm_s;  // output-channel tiles (+ fastdiv)
  uint32_t ngr, ngr_m, ngr_s;    // tile groups (+ fastdiv)
  int ocs;                       // tile order: 0 = output-channel tile fastest, 1 = slowest
  uint32_t ipt, ipt_m, ipt_s, ipb, total_it;
  int relu, wt;
  int ow2;                       // OW even: a tile row's two outputs go as one 8-B store
  int sepc;                      // cut tiles summed by wg_combine_kernel after the grid (no last arriver)
#ifdef BH_KTRACE
  unsigned long long *trace;
#endif
};

namespace {

#ifndef WG_QP
#define WG_QP 8
#endif
constexpr int WCI = 4;  // input channels per stage (two k-steps of 32x32x2 MFMAs)

// Filter transform: u[ic][oc][chunk rotated] = G g G^T for oc < OC32, ic < IC4 (zero past OC / IC)
__global__ __launch_bounds__(256) void wino_pack_kernel(const float *__restrict__ w, float *__restrict__ u,
                                                        uint32_t OC, uint32_t IC, uint32_t OC32, uint32_t IC4) {
  const uint32_t e = blockIdx.x * 256u + threadIdx.x;  // ic * OC32 + oc
  if (e >= IC4 * OC32) return;
  const uint32_t ic = e / OC32, oc = e - ic * OC32;
  float g[3][3];
  const bool ok = oc < OC && ic < IC;
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int c = 0; c < 3; ++c) g[r][c] = ok ? w[((size_t)oc * IC + ic) * 9 + r * 3 + c] : 0.0f;
  float t[4][3];
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    t[0][c] = g[0][c];
    t[1][c] = 0.5f * (g[0][c] + g[1][c] + g[2][c]);
    t[2][c] = 0.5f * (g[0][c] - g[1][c] + g[2][c]);
    t[3][c] = g[2][c];
  }
  float *const dst = u + (size_t)e * 16;
  const uint32_t rot = (oc >> 2) & 3u;
#pragma unroll
  for (int x = 0; x < 4; ++x) {
    const f32x4v v = {t[x][0], 0.5f * (t[x][0] + t[x][1] + t[x][2]), 0.5f * (t[x][0] - t[x][1] + t[x][2]), t[x][2]};
    *(f32x4v *)(dst + ((x + rot) & 3u) * 4) = v;
  }
}

// logical block of hardware block bid: blocks b, b+8, ... share an XCD under round-robin
// placement, so each XCD gets a contiguous run of iterations (neighbouring tiles in its L2)
__device__ __forceinline__ uint32_t wg_lb(uint32_t bid, uint32_t G) {
  const uint32_t xcd = bid & 7, q = G >> 3, r = G & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

// x where the lane's bit of m is set, else 0 (one v_cndmask against a wave mask held in SGPRs)
__device__ __forceinline__ float wg_lane_sel(uint64_t m, float x) {
  float r;
  asm("v_cndmask_b32_e64 %0, 0, %1, %2" : "=v"(r) : "v"(x), "s"(m));
  return r;
}

__device__ __forceinline__ void wg_store1(const WgArgs &p, __amdgpu_buffer_rsrc_t r, uint32_t off, float v) {
  if (p.wt) __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), r, off, 0, AUX_SC1);
  else __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), r, off, 0, AUX_OUT);
}

// wgp_kernel: a Winograd stage software-pipelined so that nothing but the barrier sits between one
// stage's MFMAs and the next (a first, unpipelined form spent per stage ~2000 MFMA cycles beside
// ~1000 of LDS-read latency after the barrier and ~700 of LDS-DMA issue, tools/wg_phases.py):
//  * U goes straight from L2 into registers (16-B loads of the lane's own [4 channels][16] rows;
//    group x of stage it+1 right after group x of stage it's MFMAs) -- no LDS slot, no DMA, no
//    ds_read for it;
//  * V is triple-buffered: stage it+2's patches are transformed during stage it, so stage it+1's V
//    is complete at the top of stage it and its fragments load under stage it's MFMAs;
//  * the strip ring (LDS-DMA) holds stages it+2 .. it+D+1: each strip has two stages to land.
template <int NWO, int NWT, int D, int V4, int SP, int IL, int DBG = 0>
__global__ __launch_bounds__(64 * NWO * NWT) void wgp_kernel(WgArgs p) {
  constexpr int NW = NWO * NWT, NT = 64 * NW, OCT = 32 * NWO, TT = 32 * NWT;
  constexpr int PW = 4;                       // floats per strip piece (16 B; rows of W % 4 != 0 run
                                              // into the next row: masked in the transform, !V4)
  constexpr int SCAP = SP * NT * PW;          // strip floats per slot
  constexpr int GZ = 4;                       // zero guard before the strip (a patch's left neighbour of row 0)
  constexpr int SLOT = GZ + SCAP;
  constexpr int VSZ = WCI * TT * 16;          // floats of one V buffer
  constexpr int NU = 8;                       // U loads per stage and lane
  constexpr int NQ = 16;                      // float4 results per lane: (a, b, j)
  constexpr int WTOP = (D - 2) * (SP + NU);  // younger than stage it+2's strip at the top
  static_assert(D >= 3 && WTOP <= 63, "vmcnt range");
  // the stage's WCI*TT patch transforms are spread over all NT threads: TS threads per patch, each
  // producing 4 / TS rows xi of V (every wave takes the same share of the VALU work)
  constexpr int TS = NT / (WCI * TT);
  static_assert(TS == 1 || TS == 2, "one or two threads per patch");
  static_assert(SLOT % 4 == 0, "16-B aligned slots");
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float *const vbase = smem + D * SLOT;
  uint32_t *const flag = (uint32_t *)(vbase + 3 * VSZ);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wo = wave % NWO, wtl = wave / NWO;
  const int li = lane & 31, kh = lane >> 5;
  const uint32_t lb = wg_lb(blockIdx.x, gridDim.x);
  const uint32_t it0 = lb * p.ipb, it1 = min(p.total_it, it0 + p.ipb);
  if (tid < D * GZ) smem[(tid / GZ) * SLOT + tid % GZ] = 0.0f;

  // tile t = (tile group, OC tile): OC tile fastest (consecutive tiles share the strip through L2),
  // or slowest (ocs: an XCD's run of tiles shares one OC tile's U slice -- U outgrows the L2 where
  // IC*OC is large)
  auto tile_of = [&](uint32_t t, uint32_t &oc0, uint32_t &g0) {
    if (p.ocs) {
      const uint32_t q = fdiv(t, p.ngr_m, p.ngr_s);
      oc0 = q * OCT;
      g0 = (t - q * p.ngr) * TT;
    } else {
      const uint32_t pt = fdiv(t, p.tm_m, p.tm_s);
      oc0 = (t - pt * p.tiles_m) * OCT;
      g0 = pt * TT;
    }
  };
  auto tpos = [&](uint32_t tg, uint32_t &v, int &x) {
    const uint32_t img = fdiv(tg, p.tpi_m, p.tpi_s), rem = tg - img * p.TPI;
    const uint32_t ty = fdiv(rem, p.tw_m, p.tw_s), tx = rem - ty * p.TW;
    v = img * p.VH + 2 * ty;
    x = 2 * (int)tx - (int)p.px;
  };

  const __amdgpu_buffer_rsrc_t rsu = make_rsrc(p.u, p.u_bytes);
  const __amdgpu_buffer_rsrc_t rsi = make_rsrc(p.in, p.in_bytes);
  const __amdgpu_buffer_rsrc_t rnull = make_rsrc(p.in, 0u);
  // v_mfma_f32_32x32x2_f32, lane (li, kh): A row = output channel oc0 + wo*32 + li, B column = tile
  // wtl*32 + li, k = channel ic0 + 2s + kh at k step s of the stage; chunk x of a row's 16
  // positions sits at ((x + rot) & 3) * 4 in U's and V's rows (a 16x16x4 form of this kernel ran
  // its 64 MFMAs per stage at ~51 cycles each instead of 32: tools/wg_phases.py, xwgp_onlymfma)
  const uint32_t rot = ((uint32_t)li >> 2) & 3u;
  uint32_t co[4];
#pragma unroll
  for (int x = 0; x < 4; ++x) co[x] = ((x + rot) & 3u) * 4u;

  // ---- strip DMA of stage it (channels ic0 .. ic0 + 3 of tile it / ipt)
  uint32_t svo[SP];
  uint32_t ls_tile = 0xffffffffu;
  auto plan_strip = [&](uint32_t it, uint32_t &ss) -> bool {
    const uint32_t t = fdiv(it, p.ipt_m, p.ipt_s), ic0 = (it - t * p.ipt) * WCI;
    if (t != ls_tile) {  // uniform
      uint32_t oc0, g0, v0;
      int x0;
      tile_of(t, oc0, g0);
      if constexpr ((DBG & 512) != 0) g0 = 0;  // diagnostic: every tile DMAs tile group 0's strip
      tpos(g0 < p.T ? g0 : 0u, v0, x0);
#pragma unroll
      for (int j = 0; j < SP; ++j) {  // piece: channel c, row s, column col of the [4][RIN][WPM] image
        const uint32_t f = (uint32_t)((j * NW + wave) * 64 + lane) * PW;
        const uint32_t c = fdiv(f, p.rw_m, p.rw_s), rr = f - c * p.RW;
        const uint32_t s = fdiv(rr, p.wpm_m, p.wpm_s), col = rr - s * p.WPM;
        const uint32_t v = v0 + s;
        const uint32_t img = fdiv(v, p.vh_m, p.vh_s);
        const uint32_t iy = v - img * p.VH - p.py;  // wraps (misses) in the top padding
        const bool ok = (c < (uint32_t)WCI) & (col < p.W) & (iy < p.H) & (img < p.B);
        svo[j] = oob_unless(ok, (img * p.ICHW + c * p.HW + iy * p.W + col) * 4u);
      }
      ls_tile = t;
    }
    ss = ic0 * p.HW * 4u;
    return it >= it1;
  };
  auto issue_strip = [&](int j, int sl, uint32_t ss, bool dead) {
    float *const base = smem + sl * SLOT + GZ;
    dma16s(dead ? rnull : rsi, base + (j * NW + wave) * 256, svo[j], ss);
  };

  // ---- U of stage it into registers: lane (li, kh) holds rows (channel ic0 + 2s + kh, output
  // channel oc0 + wo*32 + li), chunk x from position co[x]; one register buffer: group g of stage
  // it+1 (k step s = g >> 1, chunks 2 (g & 1) .. + 1) loads right after group g of stage it's MFMAs
  f32x4v ur[2][4];
  uint32_t uoff[2][4];
  uint32_t lu_tile = 0xffffffffu;
  auto plan_u = [&](uint32_t it) -> uint32_t {  // scalar offset of stage it's channels
    const uint32_t t = fdiv(it, p.ipt_m, p.ipt_s), ic0 = (it - t * p.ipt) * WCI;
    if (t != lu_tile) {  // uniform
      uint32_t oc0, g0;
      tile_of(t, oc0, g0);
      if constexpr ((DBG & 256) != 0) oc0 = 0;  // diagnostic: every tile reads OC tile 0's U (L2-resident)
      const uint32_t oc = oc0 + (uint32_t)(wo * 32 + li);
#pragma unroll
      for (int st = 0; st < 2; ++st)
#pragma unroll
        for (int x = 0; x < 4; ++x)
          uoff[st][x] = oob_unless(oc < p.OC32, ((uint32_t)(2 * st + kh) * p.OC32 + oc) * 64u + co[x] * 4u);
      lu_tile = t;
    }
    return it < it1 ? ic0 * p.OC32 * 64u : 0x7fffff00u;  // dead stages: misses
  };
  auto load_u = [&](int g, uint32_t su) {
    const int st = g >> 1;
#pragma unroll
    for (int x = 2 * (g & 1); x < 2 * (g & 1) + 2; ++x)
      ur[st][x] = __builtin_bit_cast(f32x4v, __builtin_amdgcn_raw_buffer_load_b128(rsu, uoff[st][x], su, 0));
  };

  // ---- input transform: thread (cl, tt) of the first 4*TT, the patch of tile g0 + tt, channel cl
  // (half h = tid / (4 TT): wave-uniform, so the two halves' different arithmetic does not diverge)
  const uint32_t xpr = (uint32_t)tid % (WCI * TT), xh = __builtin_amdgcn_readfirstlane((uint32_t)tid / (WCI * TT));
  const uint32_t xcl = xpr / TT, xtt = xpr % TT;
  // IL == 2 (configs wgl*): the TS == 2 transform with no per-half selects and fewer masks, per-lane
  // LDS bases made once per tile, the strip slot and V buffer of a stage one phase counter. Half h = 0 reads patch rows 0, 1, 2, half 1 rows 2, 3, 1 (into e0, e1, e2):
  // V rows 2h, 2h + 1 come from t0 = e0 - e2 (h0: r0 - r2, h1: r2 - r1) and t1 = e2 + sg e1 (sg = +1:
  // r1 + r2, sg = -1: r1 - r3) -- the same roundings as the per-half forms (bitwise equal V). Only patch
  // columns 2 and 3 ever reach past the row (x = 2 tx - px, pad <= 1) and column 0 before it (x = -1
  // reads the previous strip row's last column: a 16-B piece's spill from the next input row when
  // W % 4 != 0); column 1 never leaves it. Masking a column of t masks that column of the patch (each t
  // column combines one patch column): 6 selects instead of 12.
  constexpr bool LEAN = IL == 2;
  static_assert(!LEAN || (TS == 2 && D == 3), "lean transform: two threads per patch, three strip slots");
  const float *xp[3] = {smem, smem, smem};
  uint64_t cm0 = ~0ull, cm2 = ~0ull, cm3 = ~0ull;
  const float sg = xh ? -1.0f : 1.0f;
  uint32_t xb = GZ;
  uint32_t xm = 0xfu;  // !V4: patch columns inside the row (the rest of a 16-B piece is the next row's)
  uint32_t lx_tile = 0xffffffffu;
  auto xplan = [&](uint32_t it) {
    const uint32_t t = fdiv(it, p.ipt_m, p.ipt_s);
    if (t == lx_tile) return;
    lx_tile = t;
    uint32_t oc0, g0, v0;
    int x0;
    tile_of(t, oc0, g0);
    tpos(g0 < p.T ? g0 : 0u, v0, x0);
    const uint32_t tg = g0 + xtt;
    xb = GZ;
    if (tg < p.T) {
      uint32_t v;
      int x;
      tpos(tg, v, x);
      xb = (uint32_t)((int)(GZ + xcl * p.RW + (v - v0) * p.WPM) + x);
      xm = 0;
#pragma unroll
      for (int c = 0; c < 4; ++c) xm |= ((uint32_t)(x + c) < p.W ? 1u : 0u) << c;
    }
    if constexpr (LEAN) {  // the half's three patch rows (xh = 1 reads them permuted), column masks
#pragma unroll
      for (int r = 0; r < 3; ++r) xp[r] = smem + xb + (xh ? (r == 0 ? 2u : (r == 1 ? 3u : 1u)) : (uint32_t)r) * p.WPM;
      if constexpr (!V4) {
        cm0 = __builtin_amdgcn_ballot_w64((xm & 1u) != 0);
        cm2 = __builtin_amdgcn_ballot_w64(((xm >> 2) & 1u) != 0);
        cm3 = __builtin_amdgcn_ballot_w64(((xm >> 3) & 1u) != 0);
      }
    }
  };
  // TS == 1: patch rows 0..3, all four V rows; TS == 2: half h reads rows h .. h + 2 (d[0..2]) and
  // makes V rows 2h, 2h + 1 (B^T rows 0, 1 use d0 - d2, d1 + d2; rows 2, 3 use d2 - d1, d1 - d3)
  constexpr int NR = TS == 1 ? 4 : 3;
  float d[NR][4];
  auto tx_read = [&](int sl) {
    const float *const s = smem + sl * SLOT + xb + (TS == 2 ? xh * p.WPM : 0u);
    const uint32_t wpm = p.WPM;
#pragma unroll
    for (int r = 0; r < NR; ++r)
#pragma unroll
      for (int c = 0; c < 4; ++c) d[r][c] = s[r * wpm + c];
  };
  auto tx_write = [&](int vb) {
    // (the masks here, not in tx_read: hipcc would wait for the reads before the first MFMA group)
    if constexpr (!V4) {
#pragma unroll
      for (int r = 0; r < NR; ++r)
#pragma unroll
        for (int c = 0; c < 4; ++c) d[r][c] = (xm >> c) & 1u ? d[r][c] : 0.0f;
    }
    float *const vd = vbase + vb * VSZ + (xcl * TT + xtt) * 16;
    const uint32_t r2 = (xtt >> 2) & 3u;
    auto put = [&](uint32_t x, const float (&t)[4]) {
      const f32x4v v = {t[0] - t[2], t[1] + t[2], t[2] - t[1], t[1] - t[3]};
      *(f32x4v *)(vd + ((x + r2) & 3u) * 4) = v;
    };
    if constexpr (TS == 1) {
      float t[4][4];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        t[0][c] = d[0][c] - d[2][c];
        t[1][c] = d[1][c] + d[2][c];
        t[2][c] = d[2][c] - d[1][c];
        t[3][c] = d[1][c] - d[3][c];
      }
#pragma unroll
      for (int x = 0; x < 4; ++x) put((uint32_t)x, t[x]);
    } else {
      // h = 0: rows 0..2 in d -> t0 = d0 - d2, t1 = d1 + d2; h = 1: rows 1..3 -> t2 = d1 - d0, t3 = d0 - d2
      float ta[4], tb[4];
      if (xh) {
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          ta[c] = d[1][c] - d[0][c];
          tb[c] = d[0][c] - d[2][c];
        }
        put(2, ta);
        put(3, tb);
      } else {
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          ta[c] = d[0][c] - d[2][c];
          tb[c] = d[1][c] + d[2][c];
        }
        put(0, ta);
        put(1, tb);
      }
    }
  };

  // IL: the same transform in eight slices, one between each pair of MFMAs of the stage (a VALU /
  // LDS instruction issued while an MFMA runs costs no issue time; a run of them between MFMA groups
  // does)
  float tq[4][4];
  auto tx_part = [&](int vb, int part) {
    float *const vd = vbase + vb * VSZ + (xcl * TT + xtt) * 16;
    const uint32_t r2 = (xtt >> 2) & 3u;
    auto put = [&](uint32_t x, const float (&t)[4]) {
      const f32x4v v = {t[0] - t[2], t[1] + t[2], t[2] - t[1], t[1] - t[3]};
      *(f32x4v *)(vd + ((x + r2) & 3u) * 4) = v;
    };
    if constexpr (TS == 1) {
      if (part < 2) {
        if constexpr (!V4) {
#pragma unroll
          for (int r = 2 * part; r < 2 * part + 2; ++r)
#pragma unroll
            for (int c = 0; c < 4; ++c) d[r][c] = (xm >> c) & 1u ? d[r][c] : 0.0f;
        }
      } else if (part < 4) {
#pragma unroll
        for (int c = 2 * (part - 2); c < 2 * (part - 2) + 2; ++c) {
          tq[0][c] = d[0][c] - d[2][c];
          tq[1][c] = d[1][c] + d[2][c];
          tq[2][c] = d[2][c] - d[1][c];
          tq[3][c] = d[1][c] - d[3][c];
        }
      } else {
        put((uint32_t)(part - 4), tq[part - 4]);
      }
    } else {
      if (part < 3) {
        if constexpr (!V4) {
#pragma unroll
          for (int c = 0; c < 4; ++c) d[part][c] = (xm >> c) & 1u ? d[part][c] : 0.0f;
        }
      } else if (part == 3) {
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          tq[0][c] = xh ? d[1][c] - d[0][c] : d[0][c] - d[2][c];
          tq[1][c] = xh ? d[0][c] - d[2][c] : d[1][c] + d[2][c];
        }
      } else if (part == 4) {
        put(2 * xh, tq[0]);
      } else if (part == 5) {
        put(2 * xh + 1, tq[1]);
      }
    }
  };

  float *const vput0 = vbase + (xcl * TT + xtt) * 16 + ((2u * xh + ((xtt >> 2) & 3u)) & 3u) * 4;
  float *const vput1 = vbase + (xcl * TT + xtt) * 16 + ((2u * xh + 1u + ((xtt >> 2) & 3u)) & 3u) * 4;
  auto tx_read_l = [&](int sl) {
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int c = 0; c < 4; ++c) d[r][c] = xp[r][sl * SLOT + c];
  };
  auto tx_part_l = [&](int vb_, int part) {
    auto put = [&](float *vd, const float (&t)[4]) {
      *(f32x4v *)(vd + vb_ * VSZ) = f32x4v{t[0] - t[2], t[1] + t[2], t[2] - t[1], t[1] - t[3]};
    };
    if (part == 0) {
#pragma unroll
      for (int c = 0; c < 4; ++c) tq[0][c] = d[0][c] - d[2][c];
    } else if (part == 1) {
#pragma unroll
      for (int c = 0; c < 4; ++c) tq[1][c] = __builtin_fmaf(sg, d[1][c], d[2][c]);
    } else if (part == 2) {
      if constexpr (!V4) {
#pragma unroll
        for (int r = 0; r < 2; ++r) {
          tq[r][0] = wg_lane_sel(cm0, tq[r][0]);
          tq[r][2] = wg_lane_sel(cm2, tq[r][2]);
          tq[r][3] = wg_lane_sel(cm3, tq[r][3]);
        }
      }
    } else if (part == 3) {
      put(vput0, tq[0]);
    } else if (part == 4) {
      put(vput1, tq[1]);
    }
  };

  // ---- V fragments (buffer vb), group g: tile wtl*32 + li, channel 2s + kh; one register buffer
  // like U
  f32x4v vf[2][4];
  auto vfrag = [&](int vb, int g) {
    const int st = g >> 1;
    const float *const vp = vbase + vb * VSZ + ((2 * st + kh) * TT + wtl * 32 + li) * 16;
#pragma unroll
    for (int x = 2 * (g & 1); x < 2 * (g & 1) + 2; ++x) vf[st][x] = *(const f32x4v *)(vp + co[x]);
  };

  f32x16 acc[16];  // position p = 4 xi + nu
  auto mfma_x = [&](int g) {
    const int st = g >> 1;
#pragma unroll
    for (int x = 2 * (g & 1); x < 2 * (g & 1) + 2; ++x)
#pragma unroll
      for (int n = 0; n < 4; ++n)
        acc[4 * x + n] = __builtin_amdgcn_mfma_f32_32x32x2f32(ur[st][x][n], vf[st][x][n], acc[4 * x + n], 0, 0, 0);
  };

  const __amdgpu_buffer_rsrc_t rso = make_rsrc(p.out, p.out_bytes);
  const __amdgpu_buffer_rsrc_t rsr = make_rsrc(p.res, p.res ? p.out_bytes : 0u);
  const __amdgpu_buffer_rsrc_t rsb = make_rsrc(p.bias, p.bias ? p.OC * 4u : 0u);
  // output transform of accumulator element q (output channel oc0 + wo*32 + 8 (q >> 2) + 4 kh + (q & 3),
  // tile wtl*32 + li): {y00, y01, y10, y11}
  auto out_q = [&](int q) -> f32x4v {
    float s0[4], s1[4];
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      float m0, m1, m2, m3;
      asm volatile("v_accvgpr_read_b32 %0, %1" : "=v"(m0) : "a"(acc[n][q]));
      asm volatile("v_accvgpr_read_b32 %0, %1" : "=v"(m1) : "a"(acc[4 + n][q]));
      asm volatile("v_accvgpr_read_b32 %0, %1" : "=v"(m2) : "a"(acc[8 + n][q]));
      asm volatile("v_accvgpr_read_b32 %0, %1" : "=v"(m3) : "a"(acc[12 + n][q]));
      s0[n] = m0 + m1 + m2;
      s1[n] = m1 - m2 - m3;
    }
    return f32x4v{s0[0] + s0[1] + s0[2], s0[1] - s0[2] - s0[3], s1[0] + s1[1] + s1[2], s1[1] - s1[2] - s1[3]};
  };
  float bias[16];
  uint32_t sob;
  bool stv, sx1, sy1;
  auto store_pos = [&](uint32_t g0) {
    const uint32_t tg = g0 + (uint32_t)(wtl * 32 + li);
    stv = tg < p.T;
    const uint32_t tgc = stv ? tg : 0u;
    const uint32_t img = fdiv(tgc, p.tpi_m, p.tpi_s), rem = tgc - img * p.TPI;
    const uint32_t ty = fdiv(rem, p.tw_m, p.tw_s), tx = rem - ty * p.TW;
    sx1 = 2 * tx + 1 < p.OW;
    sy1 = 2 * ty + 1 < p.OH;
    sob = img * p.OCOHW + 2 * ty * p.OW + 2 * tx;
  };
  auto store_q = [&](uint32_t oc0, int q, f32x4v yy) {
    const uint32_t oc = oc0 + (uint32_t)(wo * 32 + 8 * (q >> 2) + 4 * kh + (q & 3));
    const bool ok = stv & (oc < p.OC);
    const uint32_t o = sob + oc * p.OHW;
    if (p.ow2) {  // uniform; o even, so both 8-B pieces are aligned (every tile has both columns)
      const uint32_t off[2] = {oob_unless(ok, o * 4u), oob_unless(ok & sy1, (o + p.OW) * 4u)};
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        float z0 = yy[2 * e] + bias[q], z1 = yy[2 * e + 1] + bias[q];
        if (p.res) {  // (two dword loads: hipcc lowered an 8-B raw_buffer_load here to a 4-B one)
          z0 += __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rsr, off[e], 0, 0));
          z1 += __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rsr, off[e], 4, 0));
        }
        if (p.relu) {
          z0 = z0 < 0.0f ? 0.0f : z0;
          z1 = z1 < 0.0f ? 0.0f : z1;
        }
        const __attribute__((ext_vector_type(2))) uint32_t v = {__builtin_bit_cast(uint32_t, z0),
                                                               __builtin_bit_cast(uint32_t, z1)};
        const uint32_t oo = (DBG & 8) ? OOB : off[e];
        if (p.wt) __builtin_amdgcn_raw_buffer_store_b64(v, rso, oo, 0, AUX_SC1);
        else __builtin_amdgcn_raw_buffer_store_b64(v, rso, oo, 0, AUX_OUT);
      }
      return;
    }
    const uint32_t off[4] = {oob_unless(ok, o * 4u), oob_unless(ok & sx1, (o + 1) * 4u),
                             oob_unless(ok & sy1, (o + p.OW) * 4u), oob_unless(ok & sx1 & sy1, (o + p.OW + 1) * 4u)};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float z = yy[e] + bias[q];
      if (p.res) z += __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rsr, off[e], 0, 0));
      z = (p.relu && z < 0.0f) ? 0.0f : z;
      wg_store1(p, rso, (DBG & 8) ? OOB : off[e], z);
    }
  };
  auto finish_tile = [&](uint32_t t) {
    uint32_t oc0, g0;
    tile_of(t, oc0, g0);
    const uint32_t tb = t * p.ipt;
    const bool whole = tb >= it0 && tb + p.ipt <= it1;  // uniform
    store_pos(g0);
    const uint32_t sl = (t == fdiv(it0, p.ipt_m, p.ipt_s)) ? 0u : 1u;
    const __amdgpu_buffer_rsrc_t rw = make_rsrc(p.ws + ((size_t)lb * 2 + sl) * (NQ * NT * 4), NQ * NT * 16);
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const f32x4v y = out_q(q);
      if (whole)
        store_q(oc0, q, y);
      else
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) uint32_t, y), rw,
                                               (uint32_t)((q * NT + tid) * 16), 0, AUX_SC1);
      __builtin_amdgcn_sched_barrier(0);
    }
    if (whole || p.sepc) return;  // (sepc: summed by wg_combine_kernel)
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
    // QP accumulator elements per pass: each slab's QP loads go out together, so a pass waits one
    // memory latency per slab (with 4 per pass the last arriver of a tile cut into ~11 pieces
    // spent about as long in this loop as the whole tile's stages, tools/wg_phases.py at batch 5)
    constexpr int QP = WG_QP;
#pragma unroll
    for (int q0 = 0; q0 < NQ; q0 += QP) {
      f32x4v y[QP];
#pragma unroll
      for (int i = 0; i < QP; ++i) y[i] = f32x4v{0.0f, 0.0f, 0.0f, 0.0f};
      for (uint32_t b = b0; b <= b1; ++b) {  // block order = k order: bitwise reproducible
        const uint32_t s2 = (b == b0 && t != fdiv(b * p.ipb, p.ipt_m, p.ipt_s)) ? 1u : 0u;
        const uint32_t base = (b * 2 + s2) * (uint32_t)(NQ * NT * 16);
        f32x4v x[QP];
#pragma unroll
        for (int i = 0; i < QP; ++i)
          x[i] = __builtin_bit_cast(f32x4v, __builtin_amdgcn_raw_buffer_load_b128(
                                                rall, base + (uint32_t)(((q0 + i) * NT + tid) * 16), 0, AUX_SC1));
#pragma unroll
        for (int i = 0; i < QP; ++i) y[i] += x[i];
      }
#pragma unroll
      for (int i = 0; i < QP; ++i) store_q(oc0, q0 + i, y[i]);
    }
  };

#ifdef BH_KTRACE
  uint64_t tk[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const uint64_t tk0 = __builtin_amdgcn_s_memtime();
  uint64_t tkp = tk0;
#endif

  // ---- prologue: strips of stages it0 .. it0+D-1 and U(it0) in flight; V(it0), V(it0+1)
  // transformed; stage it0+D's strip issued into stage it0's slot; V(it0)'s fragments read
#pragma unroll
  for (int s = 0; s < D; ++s) {
    uint32_t ss;
    const bool dead = plan_strip(it0 + (uint32_t)s, ss);
#pragma unroll
    for (int j = 0; j < SP; ++j) issue_strip(j, s, ss, dead);
  }
  {
    const uint32_t su = plan_u(it0);
#pragma unroll
    for (int x = 0; x < 4; ++x) load_u(x, su);
  }
  vm_wait<0>();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  if constexpr (LEAN) {
    xplan(it0);
    tx_read_l(0);
    for (int q = 0; q < 5; ++q) tx_part_l(0, q);
    xplan(it0 + 1);
    tx_read_l(1);
    for (int q = 0; q < 5; ++q) tx_part_l(1, q);
  } else {
    xplan(it0);
    tx_read(0);
    tx_write(0);
    xplan(it0 + 1);
    tx_read(1);
    tx_write(1);
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  {
    uint32_t ss;
    const bool dead = plan_strip(it0 + D, ss);
#pragma unroll
    for (int j = 0; j < SP; ++j) issue_strip(j, 0, ss, dead);
  }
#pragma unroll
  for (int x = 0; x < 4; ++x) vfrag(0, x);

  // stage it: strips of it+2 .. it+D+1 in slots (it - it0 + 2 .. ) % D; V(it) in buffer it % 3
  // (fragments in registers), V(it+1) complete, V(it+2) written this stage
  int sl2 = 2 % D;  // slot of stage it+2
  int vb = 0;       // V buffer of stage it (relative to it0)
  // per stage and lane, VMEM in issue order: after MFMA group x, U(it+1) group x (2 loads) then
  // strip share x of stage it+D+1 (QG DMAs); so U(it) group x has exactly 6 + SP younger loads when
  // group x needs it, and stage it+2's strip (D-2) whole stages of 8 + SP at the top of stage it
  auto stage = [&](uint32_t it) {
    vm_wait<WTOP>();  // stage it+2's strip landed (this wave's DMAs)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if constexpr ((DBG & 128) == 0) __builtin_amdgcn_s_barrier();  // every wave's; V(it+1) written; V(it+2)'s buffer and stage it+1's slot free
    asm volatile("" ::: "memory");
#ifdef BH_KTRACE
    { const uint64_t tn_ = __builtin_amdgcn_s_memtime(); tk[1] += tn_ - tkp; tkp = tn_; tk[6] += 1; }
#endif
    const int vb1 = vb == 2 ? 0 : vb + 1, vb2 = vb1 == 2 ? 0 : vb1 + 1;
    const int sl1 = sl2 == 0 ? D - 1 : sl2 - 1;  // slot of stage it+1 (its strip transformed last stage)
    if constexpr ((DBG & 1) == 0) {
      xplan(it + 2);
      tx_read(sl2);
    }
    uint32_t ss = 0;
    bool dead = true;
    if constexpr ((DBG & 4) == 0) dead = plan_strip(it + D + 1, ss);
    const uint32_t su = plan_u(it + 1);
    __builtin_amdgcn_sched_barrier(0);
    constexpr int QG = (SP + 3) / 4;
    if constexpr (IL) {
      auto mf = [&](int st, int x, int n) {
        acc[4 * x + n] = __builtin_amdgcn_mfma_f32_32x32x2f32(ur[st][x][n], vf[st][x][n], acc[4 * x + n], 0, 0, 0);
      };
      auto chunk = [&](int st, int x) {  // stage it+1's U and V fragments of chunk x, k step st
        ur[st][x] = __builtin_bit_cast(f32x4v, __builtin_amdgcn_raw_buffer_load_b128(rsu, uoff[st][x], su, 0));
        vf[st][x] = *(const f32x4v *)(vbase + vb1 * VSZ + ((2 * st + kh) * TT + wtl * 32 + li) * 16 + co[x]);
      };
#pragma unroll
      for (int x = 0; x < 4; ++x) {
        const int st = x >> 1, c0 = 2 * (x & 1), c1 = c0 + 1;
        vm_wait<6 + SP>();  // U(it) group x landed
        mf(st, c0, 0);
        mf(st, c0, 1);
        __builtin_amdgcn_sched_barrier(0);
        tx_part(vb2, 2 * x);
        __builtin_amdgcn_sched_barrier(0);
        mf(st, c0, 2);
        mf(st, c0, 3);
        __builtin_amdgcn_sched_barrier(0);
        chunk(st, c0);
        __builtin_amdgcn_sched_barrier(0);
        mf(st, c1, 0);
        mf(st, c1, 1);
        __builtin_amdgcn_sched_barrier(0);
        tx_part(vb2, 2 * x + 1);
        __builtin_amdgcn_sched_barrier(0);
        mf(st, c1, 2);
        mf(st, c1, 3);
        __builtin_amdgcn_sched_barrier(0);
        chunk(st, c1);
#pragma unroll
        for (int j = x * QG; j < (x + 1) * QG; ++j) {
          if (j < SP) issue_strip(j, sl1, ss, dead);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    } else {
#pragma unroll
    for (int x = 0; x < 4; ++x) {
      if constexpr ((DBG & 64) == 0) vm_wait<6 + SP>();  // U(it) group x landed
      if constexpr ((DBG & 2) == 0) mfma_x(x);
      else acc[x][0] += ur[0][x][0] + vf[0][x][0];
      __builtin_amdgcn_sched_barrier(0);
      if constexpr ((DBG & 16) == 0) load_u(x, su);
      if constexpr ((DBG & 32) == 0) vfrag(vb1, x);
      if constexpr ((DBG & 4) == 0) {
#pragma unroll
        for (int j = x * QG; j < (x + 1) * QG; ++j) {
          if (j < SP) issue_strip(j, sl1, ss, dead);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
      if (x == 0) {
        if constexpr ((DBG & 1) == 0) tx_write(vb2);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    }
#ifdef BH_KTRACE
    { const uint64_t tn_ = __builtin_amdgcn_s_memtime(); tk[4] += tn_ - tkp; tkp = tn_; }
#endif
    vb = vb1;
    sl2 = sl2 == D - 1 ? 0 : sl2 + 1;
  };

  // IL == 2: stage it at phase ph = (it - it0) % 3 -- V(it) in buffer ph, V(it+1) in ph + 1, stage it+2's
  // strip in slot ph + 2 (transformed into V buffer ph + 2), stage it+D+1's strip issued into slot ph + 1
  // (D == 3: the slot and buffer rotations coincide; a phase-unrolled form, every LDS address an
  // immediate, took 256 VGPRs and spilled)
  const float *vfq[4];
#pragma unroll
  for (int x = 0; x < 4; ++x) vfq[x] = vbase + ((uint32_t)kh * TT + (uint32_t)(wtl * 32 + li)) * 16 + co[x];
  auto stage_l = [&](uint32_t it, uint32_t ph) {
    const int vb1 = ph == 2 ? 0 : (int)ph + 1, vb2 = ph == 0 ? 2 : (int)ph - 1;
    vm_wait<WTOP>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    xplan(it + 2);
    tx_read_l(vb2);
    uint32_t ss = 0;
    const bool dead = plan_strip(it + D + 1, ss);
    const uint32_t su = plan_u(it + 1);
    __builtin_amdgcn_sched_barrier(0);
    constexpr int QG = (SP + 3) / 4;
    auto mf = [&](int st, int x, int n) {
      acc[4 * x + n] = __builtin_amdgcn_mfma_f32_32x32x2f32(ur[st][x][n], vf[st][x][n], acc[4 * x + n], 0, 0, 0);
    };
    auto chunk = [&](int st, int x) {  // stage it+1's U and V fragments of chunk x, k step st
      ur[st][x] = __builtin_bit_cast(f32x4v, __builtin_amdgcn_raw_buffer_load_b128(rsu, uoff[st][x], su, 0));
      vf[st][x] = *(const f32x4v *)(vfq[x] + vb1 * VSZ + 2 * st * TT * 16);
    };
#pragma unroll
    for (int x = 0; x < 4; ++x) {
      const int st = x >> 1, c0 = 2 * (x & 1), c1 = c0 + 1;
      vm_wait<6 + SP>();  // U(it) group x landed
      mf(st, c0, 0);
      mf(st, c0, 1);
      __builtin_amdgcn_sched_barrier(0);
      tx_part_l(vb2, 2 * x);
      __builtin_amdgcn_sched_barrier(0);
      mf(st, c0, 2);
      mf(st, c0, 3);
      __builtin_amdgcn_sched_barrier(0);
      chunk(st, c0);
      __builtin_amdgcn_sched_barrier(0);
      mf(st, c1, 0);
      mf(st, c1, 1);
      __builtin_amdgcn_sched_barrier(0);
      tx_part_l(vb2, 2 * x + 1);
      __builtin_amdgcn_sched_barrier(0);
      mf(st, c1, 2);
      mf(st, c1, 3);
      __builtin_amdgcn_sched_barrier(0);
      chunk(st, c1);
#pragma unroll
      for (int j = x * QG; j < (x + 1) * QG; ++j) {
        if (j < SP) issue_strip(j, vb1, ss, dead);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  uint32_t ph = 0;  // (it - it0) % 3, IL == 2

  uint32_t it = it0;
  while (it < it1) {
    const uint32_t t = fdiv(it, p.ipt_m, p.ipt_s);
    const uint32_t iend = min(it1, (t + 1) * p.ipt);
    {
      uint32_t oc0, g0;
      tile_of(t, oc0, g0);
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const uint32_t oc = oc0 + (uint32_t)(wo * 32 + 8 * (q >> 2) + 4 * kh + (q & 3));
        bias[q] = ld1(rsb, oob_unless(oc < p.OC, oc * 4u));
      }
    }
#pragma unroll
    for (int q = 0; q < 16; ++q)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[q][r] = 0.0f;
    if constexpr (LEAN) {
      for (; it < iend; ++it) {
        stage_l(it, ph);
        ph = ph == 2 ? 0u : ph + 1;
      }
    } else {
      for (; it < iend; ++it) stage(it);
    }
#ifdef BH_KTRACE
    tkp = __builtin_amdgcn_s_memtime();
#endif
    finish_tile(t);
#ifdef BH_KTRACE
    { const uint64_t tn_ = __builtin_amdgcn_s_memtime(); tk[5] += tn_ - tkp; tkp = tn_; }
#endif
  }
  vm_wait<0>();
#ifdef BH_KTRACE
  tk[7] = __builtin_amdgcn_s_memtime() - tk0;
  if (tid == 0) {
#pragma unroll
    for (int i = 0; i < 8; ++i) p.trace[(size_t)blockIdx.x * 8 + i] = tk[i];
  }
#endif
}

// wg_combine_kernel: the cut tiles of a stream-K wgp grid (p.sepc), summed after it. A last arriver
// inside the grid (the form without sepc) reads the tile's 3-5 slabs and stores its whole output --
// 64 dword stores per thread where OW is odd -- while its pieces' other CUs idle: ~31 k cycles against
// ~7 k for a piece's own epilogue, the grid's tail (tools/wg_phases.py --slowest). Here a block of the
// same thread layout takes one tile and QC of its 16 accumulator elements, sums the slabs in block
// order (the last arriver's order: bitwise the same output) and stores them with the grid's epilogue
// (bias, residual, ReLU, 8-B pairs where OW is even). Tiles inside one block's range are skipped.
template <int NWO, int NWT>
__global__ __launch_bounds__(64 * NWO * NWT) void wg_combine_kernel(WgArgs p) {
  constexpr int NW = NWO * NWT, NT = 64 * NW, OCT = 32 * NWO, TT = 32 * NWT, NQ = 16, QC = 4;
  const uint32_t t = blockIdx.x / (NQ / QC), q0 = (blockIdx.x % (NQ / QC)) * QC;
  const uint32_t tb = t * p.ipt, b0 = tb / p.ipb, b1 = (tb + p.ipt - 1) / p.ipb;
  if (b0 == b1) return;  // uniform: stored by the grid
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wo = wave % NWO, wtl = wave / NWO;
  const int li = lane & 31, kh = lane >> 5;
  uint32_t oc0, g0;
  if (p.ocs) {
    const uint32_t q = fdiv(t, p.ngr_m, p.ngr_s);
    oc0 = q * OCT;
    g0 = (t - q * p.ngr) * TT;
  } else {
    const uint32_t pt = fdiv(t, p.tm_m, p.tm_s);
    oc0 = (t - pt * p.tiles_m) * OCT;
    g0 = pt * TT;
  }
  const uint32_t tg = g0 + (uint32_t)(wtl * 32 + li);
  const bool stv = tg < p.T;
  const uint32_t tgc = stv ? tg : 0u;
  const uint32_t img = fdiv(tgc, p.tpi_m, p.tpi_s), rem = tgc - img * p.TPI;
  const uint32_t ty = fdiv(rem, p.tw_m, p.tw_s), tx = rem - ty * p.TW;
  const bool sx1 = 2 * tx + 1 < p.OW, sy1 = 2 * ty + 1 < p.OH;
  const uint32_t sob = img * p.OCOHW + 2 * ty * p.OW + 2 * tx;
  const __amdgpu_buffer_rsrc_t rso = make_rsrc(p.out, p.out_bytes);
  const __amdgpu_buffer_rsrc_t rsr = make_rsrc(p.res, p.res ? p.out_bytes : 0u);
  const __amdgpu_buffer_rsrc_t rsb = make_rsrc(p.bias, p.bias ? p.OC * 4u : 0u);
  const __amdgpu_buffer_rsrc_t rall = make_rsrc(p.ws, 0x7fffff00u);
  uint32_t oc[QC];
  float bias[QC];
#pragma unroll
  for (int i = 0; i < QC; ++i) {
    const uint32_t q = q0 + (uint32_t)i;
    oc[i] = oc0 + (uint32_t)(wo * 32) + 8u * (q >> 2) + 4u * (uint32_t)kh + (q & 3u);
    bias[i] = ld1(rsb, oob_unless(oc[i] < p.OC, oc[i] * 4u));
  }
  // slabs in groups of 4: all 16 loads in flight, one wait per group
  f32x4v y[QC];
#pragma unroll
  for (int i = 0; i < QC; ++i) y[i] = f32x4v{0.0f, 0.0f, 0.0f, 0.0f};
  for (uint32_t bg = b0; bg <= b1; bg += 4) {
    f32x4v x[4][QC];
#pragma unroll
    for (int sb = 0; sb < 4; ++sb) {
      const uint32_t b = bg + (uint32_t)sb;
      const uint32_t s2 = (b == b0 && t != fdiv(b * p.ipb, p.ipt_m, p.ipt_s)) ? 1u : 0u;
      const uint32_t base = (b * 2 + s2) * (uint32_t)(NQ * NT * 16);
#pragma unroll
      for (int i = 0; i < QC; ++i)
        x[sb][i] = __builtin_bit_cast(f32x4v, __builtin_amdgcn_raw_buffer_load_b128(
                                                  rall, oob_unless(b <= b1, base + (uint32_t)(((q0 + i) * NT + tid) * 16)),
                                                  0, AUX_SC1));
    }
#pragma unroll
    for (int sb = 0; sb < 4; ++sb)
#pragma unroll
      for (int i = 0; i < QC; ++i)
        if (bg + (uint32_t)sb <= b1) y[i] += x[sb][i];  // block order = k order
  }
#pragma unroll
  for (int i = 0; i < QC; ++i) {
    const bool ok = stv & (oc[i] < p.OC);
    const uint32_t o = sob + oc[i] * p.OHW;
    if (p.ow2) {  // uniform; o even: both 8-B pieces aligned
      const uint32_t off[2] = {oob_unless(ok, o * 4u), oob_unless(ok & sy1, (o + p.OW) * 4u)};
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        float z0 = y[i][2 * e] + bias[i], z1 = y[i][2 * e + 1] + bias[i];
        if (p.res) {
          z0 += __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rsr, off[e], 0, 0));
          z1 += __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rsr, off[e], 4, 0));
        }
        if (p.relu) {
          z0 = z0 < 0.0f ? 0.0f : z0;
          z1 = z1 < 0.0f ? 0.0f : z1;
        }
        const __attribute__((ext_vector_type(2))) uint32_t v = {__builtin_bit_cast(uint32_t, z0),
                                                               __builtin_bit_cast(uint32_t, z1)};
        if (p.wt) __builtin_amdgcn_raw_buffer_store_b64(v, rso, off[e], 0, AUX_SC1);
        else __builtin_amdgcn_raw_buffer_store_b64(v, rso, off[e], 0, AUX_OUT);
      }
    } else {
      const uint32_t off[4] = {oob_unless(ok, o * 4u), oob_unless(ok & sx1, (o + 1) * 4u),
                               oob_unless(ok & sy1, (o + p.OW) * 4u), oob_unless(ok & sx1 & sy1, (o + p.OW + 1) * 4u)};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float z = y[i][e] + bias[i];
        if (p.res) z += __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rsr, off[e], 0, 0));
        z = (p.relu && z < 0.0f) ? 0.0f : z;
        wg_store1(p, rso, off[e], z);
      }
    }
  }
}

template <int NWO, int NWT, int D, int V4, int SP, int IL, int DBG = 0>
cfg_t wgp_cfg(const char *name) {
  cfg_t c{name, 32 * NWO, 32 * NWT, WCI, 64 * NWO * NWT, {}, 1};
  c.k[A_KVEC][B_DIRECT][0] = (kern_t)(void *)wgp_kernel<NWO, NWT, D, V4, SP, IL, DBG>;
  c.k[A_KVEC][B_DIRECT][1] = (kern_t)(void *)wg_combine_kernel<NWO, NWT>;
  c.dc = 4;
  c.dc_ky = 3;
  c.dc_kx = 3;
  c.dc_s = V4;
  c.dc_rin = SP;
  c.dc_ci = D;
  return c;
}

}  // namespace

std::vector<cfg_t> wg_cfgs() {
  // <NWO, NWT, D, V4, SP>: OCT = 32 NWO channels x TT = 32 NWT tiles; D strip slots; V4: W % 4 == 0
  // (no row masks); SP strip DMA pieces per thread and stage
  return {
      wgp_cfg<2, 2, 3, 1, 4, 0>("wgp64x64v"), wgp_cfg<2, 2, 3, 0, 3, 0>("wgp64x64"),
      wgp_cfg<2, 2, 4, 1, 3, 0>("wgp64x64vd4"), wgp_cfg<2, 2, 4, 0, 3, 0>("wgp64x64d4"),
      wgp_cfg<4, 1, 3, 1, 2, 0>("wgp128x32v"), wgp_cfg<4, 1, 3, 0, 2, 0>("wgp128x32"),
      // IL: the stage's loads and transform interleaved with its MFMAs
      wgp_cfg<2, 2, 3, 1, 4, 1>("wgi64x64v"), wgp_cfg<2, 2, 3, 0, 3, 1>("wgi64x64"),
      wgp_cfg<2, 2, 4, 1, 3, 1>("wgi64x64vd4"), wgp_cfg<2, 2, 4, 0, 3, 1>("wgi64x64d4"),
      wgp_cfg<4, 1, 3, 1, 2, 1>("wgi128x32v"), wgp_cfg<4, 1, 3, 0, 2, 1>("wgi128x32"),
      // lean transform, stage loop unrolled over the buffers (round 6)
      wgp_cfg<4, 1, 3, 1, 2, 2>("wgl128x32v"), wgp_cfg<4, 1, 3, 0, 2, 2>("wgl128x32"),
#ifdef BH_WG_DIAG
      // diagnostic builds (wrong results by design): one part of the stage dropped each
      wgp_cfg<4, 1, 3, 0, 2, 0, 1>("xwgp_noxf"), wgp_cfg<4, 1, 3, 0, 2, 0, 2>("xwgp_nomfma"),
      wgp_cfg<4, 1, 3, 0, 2, 0, 4>("xwgp_nodma"), wgp_cfg<4, 1, 3, 0, 2, 0, 16>("xwgp_nou"),
      wgp_cfg<4, 1, 3, 0, 2, 0, 32>("xwgp_novf"), wgp_cfg<4, 1, 3, 0, 2, 0, 64>("xwgp_nouwait"),
      wgp_cfg<4, 1, 3, 0, 2, 0, 7>("xwgp_skel"), wgp_cfg<4, 1, 3, 0, 2, 0, 8>("xwgp_nostore"),
      wgp_cfg<4, 1, 3, 0, 2, 0, 256>("xwgp_ul2"), wgp_cfg<4, 1, 3, 0, 2, 0, 512>("xwgp_sl2"),
      wgp_cfg<4, 1, 3, 0, 2, 0, 768>("xwgp_usl2"),
      wgp_cfg<4, 1, 3, 0, 2, 0, 53>("xwgp_onlymfma"), wgp_cfg<4, 1, 3, 0, 2, 0, 181>("xwgp_onlymfma_nobar"),
#endif
  };
}

size_t wino_bank_floats(uint32_t OC, uint32_t IC) {
  return (size_t)((IC + 3) & ~3u) * ((OC + 31) & ~31u) * 16;
}

int launch_wino_pack(bh_ctx *ctx, const float *filts, float *u, uint32_t OC, uint32_t IC, bool first, bool last) {
  uint32_t OC32 = (OC + 31) & ~31u, IC4 = (IC + 3) & ~3u;
  const uint64_t n = (uint64_t)OC32 * IC4;
  void *args[] = {(void *)&filts, (void *)&u, (void *)&OC, (void *)&IC, (void *)&OC32, (void *)&IC4};
  return bh::launch(ctx, (const void *)wino_pack_kernel, dim3((uint32_t)((n + 255) / 256)), dim3(256), args, first, last,
                    "wino_pack");
}

// Launch a Winograd configuration: UNSUP unless a stride-1 3x3 conv with pad <= 1, IC % 4 == 0,
// whose strips fit the configuration's slot. splits: 0 / 1..4 blocks per CU, iterations dealt
// equally; 5..8: blocks per CU 1..4, whole tiles per block; + 10: OC tiles slowest; + 20: the
// stream-K modes' cut tiles summed by wg_combine_kernel (a second launch) instead of their last
// arrivers.
int launch_wg(bh_ctx *ctx, const cfg_t &c, const float *u, const float *in, const float *bias, const float *res,
              float *out, uint32_t out_ctot, uint32_t B, uint32_t IC, uint32_t H, uint32_t W, uint32_t OC, uint32_t KY,
              uint32_t KX, uint32_t sy, uint32_t sx, uint32_t py, uint32_t px, int relu, int wt, uint32_t splits,
              bool first) {
  if (KY != 3 || KX != 3 || sy != 1 || sx != 1 || py > 1 || px > 1)
    return bh::fail(BH_UNSUP, std::string("conv: ") + c.name + " is for stride-1 3x3 convs with pad <= 1");
  if (IC % WCI) return bh::fail(BH_UNSUP, std::string("conv: ") + c.name + " needs IC % 4 == 0");
  if (c.dc_s && W % 4) return bh::fail(BH_UNSUP, std::string("conv: ") + c.name + " is for W % 4 == 0 (no row masks)");
  WgArgs p{};
  const uint32_t OH = H + 2 * py - 2, OW = W + 2 * px - 2;
  const uint32_t TH = (OH + 1) / 2, TW = (OW + 1) / 2, TPI = TH * TW;
  const uint64_t T64 = (uint64_t)B * TPI;
  const uint32_t OCT = (uint32_t)c.BM, TT = (uint32_t)c.BN, NT = (uint32_t)c.NT, D = (uint32_t)c.dc_ci;
  const uint32_t VH = std::max(H + 2 * py, 2 * TH + 2);
  const uint32_t WPM = (std::max(W + 1, 2 * TW + 2 - px) + 3) & ~3u;
  if (T64 >= (1u << 30) || (uint64_t)B * VH >= (1u << 30)) return bh::fail(BH_UNSUP, "conv: too many Winograd tiles");
  const uint32_t T = (uint32_t)T64, ngroups = (T + TT - 1) / TT;
  auto vrow = [&](uint32_t tg) { return (tg / TPI) * VH + 2 * ((tg % TPI) / TW); };
  uint32_t rin = 0;
  for (uint32_t gi = 0; gi < ngroups; ++gi) {
    const uint32_t a = gi * TT, b = std::min(T, a + TT) - 1;
    rin = std::max(rin, vrow(b) + 4 - vrow(a));
  }
  const uint32_t PW = 4, SP = (uint32_t)c.dc_rin;  // 16-B strip pieces
  if ((uint64_t)WCI * rin * WPM > (uint64_t)SP * NT * PW)
    return bh::fail(BH_UNSUP, std::string("conv: input strip too large for ") + c.name);
  const uint64_t out_bytes = (uint64_t)B * out_ctot * OH * OW * 4;
  if (out_bytes >= 0x7fffff00ull) return bh::fail(BH_UNSUP, "conv: output too large for the Winograd kernel");
  const uint32_t OC32 = (OC + 31) & ~31u;
  p.u = u; p.in = in; p.out = out; p.bias = bias; p.res = res;
  p.u_bytes = (uint32_t)(wino_bank_floats(OC, IC) * 4);
  p.in_bytes = (uint32_t)((uint64_t)B * IC * H * W * 4);
  p.out_bytes = (uint32_t)out_bytes;
  p.OC = OC; p.OC32 = OC32; p.IC = IC; p.B = B; p.H = H; p.W = W; p.py = py; p.px = px;
  p.OH = OH; p.OW = OW; p.OHW = OH * OW; p.HW = H * W; p.ICHW = IC * H * W; p.OCOHW = out_ctot * OH * OW;
  p.TW = TW; p.TPI = TPI; p.VH = VH; p.T = T; p.WPM = WPM; p.RW = rin * WPM;
  bh::fastdiv f = bh::make_fastdiv(TW); p.tw_m = f.m; p.tw_s = f.s;
  f = bh::make_fastdiv(TPI); p.tpi_m = f.m; p.tpi_s = f.s;
  f = bh::make_fastdiv(VH); p.vh_m = f.m; p.vh_s = f.s;
  f = bh::make_fastdiv(WPM); p.wpm_m = f.m; p.wpm_s = f.s;
  f = bh::make_fastdiv(p.RW); p.rw_m = f.m; p.rw_s = f.s;
  const uint32_t octiles = (OC + OCT - 1) / OCT, ipt = IC / WCI;
  const uint64_t ntile = (uint64_t)ngroups * octiles, total = ntile * ipt;
  if (total >= (1u << 31)) return bh::fail(BH_UNSUP, "conv: too many iterations");
  p.tiles_m = octiles;
  f = bh::make_fastdiv(octiles); p.tm_m = f.m; p.tm_s = f.s;
  p.ipt = ipt;
  f = bh::make_fastdiv(ipt); p.ipt_m = f.m; p.ipt_s = f.s;
  p.relu = relu;
  p.wt = wt;
  // 8-B stores need an 8-B aligned output (and residual): callers may pass any float offset
  p.ow2 = (OW % 2 == 0 && ((uintptr_t)out & 7) == 0 && ((uintptr_t)res & 7) == 0) ? 1 : 0;
  // dynamic LDS: D strip slots (guard + strip), three V buffers, the ticket flag
  const uint32_t slot = 4 + SP * NT * PW;
  const uint32_t lds = (D * slot + 3 * WCI * TT * 16 + 4) * 4;
  if (lds > 160 * 1024) return bh::fail(BH_UNSUP, std::string("conv: LDS too small for ") + c.name);
  const void *k = (const void *)c.k[A_KVEC][B_DIRECT][0];
  if (hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
    return bh::fail(BH_ERR, "conv: Winograd LDS attribute");
  int occ = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k, (int)NT, (size_t)lds) != hipSuccess || occ < 1) occ = 1;
  // splits: + 20 = cut tiles summed by wg_combine_kernel after the grid (stream-K modes); + 10 = OC
  // tile slowest
  p.sepc = splits >= 20 ? 1 : 0;
  if (splits >= 20) splits -= 20;
  p.ocs = splits >= 10 ? 1 : 0;
  if (splits >= 10) splits -= 10;
  p.ngr = ngroups;
  f = bh::make_fastdiv(ngroups); p.ngr_m = f.m; p.ngr_s = f.s;
  const bool whole = splits > 4;
  uint32_t bpc = splits ? (whole ? splits - 4 : splits) : 1;
  bpc = std::max(1u, std::min<uint32_t>(bpc, (uint32_t)std::min(occ, 4)));
  const uint32_t ncu = ctx->prop.multiProcessorCount > 0 ? ctx->prop.multiProcessorCount : 256;
  uint64_t G = (uint64_t)ncu * bpc;
  uint32_t ipb = (uint32_t)((total + G - 1) / G);
  if (whole) ipb = (uint32_t)((ntile + G - 1) / G) * ipt;
  G = (total + ipb - 1) / ipb;
  p.ipb = ipb;
  p.total_it = (uint32_t)total;
  int rc = ensure_ws(ctx, (size_t)2 * G * NT * 16 * 16);  // two slabs of 16 float4 per thread per block
  if (rc == BH_OK) rc = ensure_cnt(ctx, (size_t)ntile);
  if (rc != BH_OK) return rc;
  p.ws = (float *)ctx->ws;
  p.cnt = (uint32_t *)ctx->cnt;
#ifdef BH_KTRACE
  p.trace = (unsigned long long *)ctx->stamps + 65536;
#endif
  void *args[] = {&p};
  if (whole) p.sepc = 0;  // no cut tiles
  if (!p.sepc) return bh::launch(ctx, k, dim3((uint32_t)G, 1, 1), dim3(NT), args, first, true, "conv_wino", lds);
  rc = bh::launch(ctx, k, dim3((uint32_t)G, 1, 1), dim3(NT), args, first, false, "conv_wino", lds);
  if (rc != BH_OK) return rc;
  return bh::launch(ctx, (const void *)c.k[A_KVEC][B_DIRECT][1], dim3((uint32_t)ntile * 4u, 1, 1), dim3(NT), args,
                    false, true, "conv_wino_combine");
}

}  // namespace bhk
