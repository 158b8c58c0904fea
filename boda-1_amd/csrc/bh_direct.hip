// bh_direct.hip -- direct convolution for the few-channel, large-kernel stem layers.
//
// The stems of the conv set -- 3 x 224^2 -> 64 7x7 s2 (GoogLeNet conv1) and 3 x 227^2 ->
// 96 11x11 s4 (AlexNet conv1), at batch 1 / 5 / 20 -- are the shapes Boda sends to its tconv
// variant (test/rtc/tconv.cucl:1-52, chosen at src/cnn_op.cc:60-63: kernel <= 11x11, output
// width >= 6): a "tiled" direct conv whose input is staged per block. As an implicit GEMM
// (the ring kernels) they are the wrong shape: K = 3*KY*KX = 147 / 363 is short and every k
// row of every stage is a separate 64-column gather of a strided input row, so each input
// pixel is fetched KY*KX/S^2 = 7.6-12 times. Here
//  * a block owns OCT = 32*TM output channels x NPX = 128*TN consecutive output pixels of one
//    image (a run that may straddle output rows) and a ring of D stages, one stage per INPUT
//    CHANNEL: the channel's weights [2*KK2 taps][OCT] (from the packed k-major bank of
//    bh_conv_filts_pack, 16-B LDS-DMA) and its input strip -- the RIN input rows the block's
//    pixels touch, whole rows at pitch WPM with the zero padding materialised -- filled once by
//    coalesced dword LDS-DMA (a row is contiguous in NCHW). Each input element is read from
//    L2 about once per block instead of once per filter tap;
//  * MFMA v_mfma_f32_32x32x2_f32 (exact fp32): A = weights (lane i: output channel 32t+i),
//    B = the strip (lane j: pixel 32*tn+j of the wave). Lane half h takes taps h*KK2+s at step
//    s; a tap's strip offset ky*WPM+kx is a compile-time constant, the pixel's offset
//    ((oy-oy_a)*S)*WPM + ox*S a per-lane register, so a B fragment is one ds_read_b32 with an
//    immediate offset plus one select per step -- no per-element index arithmetic;
//  * the epilogue adds the bias (staged in LDS by DMA), the optional residual, ReLU, and
//    stores NCHW rows: 32 consecutive pixels per lane group, 128-B segments.
// Same GemmArgs contract as the other conv kernels (a = packed bank, lda = OC4; b = input;
// OCOHW = the output's image stride, so slab outputs work).
#include "bh_gemm_dev.h"

namespace bhk {
namespace {

template <int KX, int WPM>
constexpr int dc_koff(int tap, int KK) {
  return tap < KK ? (tap / KX) * WPM + tap % KX : 0;  // padding taps (zero weights): any in-strip offset
}

// Phase-split strip (PSL): strip column c = S * i + f sits at f * (WPM / S) + i, so the 32 pixels of a
// fragment, S columns apart in the input, read 32 consecutive dwords (conflict-free) instead of
// falling on 32 / S banks. Tap (ky, kx) of a pixel is at its base + dc_koffp(tap).
template <int KX, int S, int WPM>
constexpr int dc_koffp(int tap, int KK) {
  return tap < KK ? (tap / KX) * WPM + ((tap % KX) % S) * (WPM / S) + (tap % KX) / S : 0;
}
// Lane half 1 reads tap KK2 + s where half 0 reads tap s; in the phase-split strip their offsets
// differ by one of a few constants (by the taps' column phases). dk[k]: the distinct differences,
// kind[s]: step s's.
template <int KY, int KX, int S, int WPM>
struct dc_pkinds {
  static constexpr int KK = KY * KX, KK2 = (KK + 1) / 2;
  struct tab_t {
    int nk;
    int dk[32];
    int kind[KK2];
  };
  static constexpr tab_t make() {
    tab_t t{};
    for (int s = 0; s < KK2; ++s) {
      const int d = dc_koffp<KX, S, WPM>(KK2 + s, KK) - dc_koffp<KX, S, WPM>(s, KK);
      int k = -1;
      for (int i = 0; i < t.nk; ++i)
        if (t.dk[i] == d) k = i;
      if (k < 0) {
        k = t.nk;
        t.dk[t.nk++] = d;
      }
      t.kind[s] = k;
    }
    return t;
  }
  static constexpr tab_t tab = make();
};

// compile-time loop: f(integral_constant<int, I>) for I in [I0, N) (hipcc leaves a long loop with many
// per-step constants rolled, and the constants then index register arrays dynamically: scratch)
template <int I, int N, class F>
__device__ __forceinline__ void dc_static_for(F &&f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    dc_static_for<I + 1, N>(f);
  }
}

// V4: input rows of W % 4 == 0 go into the strip as 16-B pieces (a quarter of the DMA
// instructions: the strip's dword DMAs were 0.34 issues per MFMA at 11x11 s4); column c of the
// strip then holds input x = c - PXA with PXA = 4 (0 without horizontal padding), so pieces start
// on 16-B input boundaries
// PFO > 0: the LDS fragment prefetch distance (steps) instead of the default for the tile (round 5: the
// stage loop waits on its fragment reads, one s_waitcnt per MFMA)
template <int KY, int KX, int S, int WPM, int RIN, int TM, int TN, int D, int V4 = 0, int PSL = 0, int PFO = 0>
__global__ __launch_bounds__(256) void dc_kernel(GemmArgs p) {
  constexpr int NW = 4;
  constexpr int NPX = NW * 32 * TN, OCT = 32 * TM;
  constexpr int KK = KY * KX, KK2 = (KK + 1) / 2;
  constexpr int WPC = 2 * KK2 * OCT / 4;                  // 16-B weight pieces per stage
  constexpr int LWA = (WPC + NW * 64 - 1) / (NW * 64);    // weight DMA instructions per wave
  constexpr int WREG = LWA * NW * 256;                    // floats
  constexpr int SF = RIN * WPM;
  constexpr int PW = V4 ? 4 : 1;                          // floats per strip DMA lane
  static_assert(WPM % PW == 0, "16-B strip rows");
  static_assert(!PSL || (!V4 && WPM % S == 0), "phase-split strip: dword DMA, whole phases per row");
  constexpr int WS = WPM / S;                             // PSL: strip floats per column phase
  constexpr int LWB = (SF / PW + NW * 64 - 1) / (NW * 64);  // strip DMA instructions per wave
  constexpr int SREG = LWB * NW * 64 * PW;
  constexpr int BREG = NW * 64;                           // the stage tile's biases, one DMA per wave
  constexpr int SLOT = WREG + SREG + BREG;
  constexpr int LW = LWA + LWB + 1;
  static_assert(D >= 2 && (D - 2) * LW <= 63, "vmcnt range");
  static_assert(OCT % 4 == 0 && OCT <= BREG, "16-B weight pieces, biases of one tile");
  constexpr int PF = PFO > 0 ? PFO : (TM * TN >= 4 ? 1 : (TM * TN >= 2 ? 2 : 3));  // LDS fragment prefetch distance (steps)
  constexpr int IS = (KK2 + 1) / 2 > 1 ? (KK2 + 1) / 2 : 1;     // steps the next stage's DMAs are spread over
  // epilogue: a lane's accumulators hold 4 consecutive pixels of one output channel per
  // register quad (the MFMA's rows are pixels), stored as NST float4 pieces per lane, deferred
  // into the first ISS steps of the next tile (one store per step or two): a CU retires store
  // instructions at a limited rate, so a burst of them at the end of a tile stalls the waves
  // while the MFMA pipe idles (cdna_hip_programming.md T21)
  constexpr int NST = TM * TN * 4;
  constexpr int ISS = KK2 > 2 * NST ? 2 * NST : KK2;
  // one __shared__ array only (a second object makes hipcc wait vmcnt(0) at ds_reads)
  __shared__ __attribute__((aligned(16))) float smem[D * SLOT];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int kh = lane >> 5, li = lane & 31;
  KT(0);

  // ---- this block's tiles: t = blockIdx.x + i * gridDim.x; tile t = (pixel run, image, OC tile)
  // with the OC tile fastest (consecutive tiles share the input strip through L2)
  const uint32_t G = gridDim.x, b0 = blockIdx.x;
  const uint32_t ntile = p.total_it;  // tiles of the op
  const uint32_t my_tiles = b0 < ntile ? (ntile - b0 + G - 1) / G : 0;
  auto decode = [&](uint32_t t, uint32_t &oc0, uint32_t &img, uint32_t &p0) {
    const uint32_t rest = fdiv(t, p.ipt_m, p.ipt_s);  // ipt = OC tiles
    oc0 = (t - rest * p.ipt) * OCT;
    img = fdiv(rest, p.tm_m, p.tm_s);                // tiles_n = pixel runs per image
    p0 = (rest - img * p.tiles_n) * NPX;
  };

  // ---- tile-independent per-lane parts of the DMA source offsets (a stage adds its tile's and
  // channel's): weight piece e of the [tap][OCT] image = packed-bank row tap*IC + ic (K order
  // (ky, kx, ic)), column 4*c4; strip element e = (row r, column c) of the [RIN][WPM] image
  const __amdgpu_buffer_rsrc_t rsw = make_rsrc(p.a, p.a_bytes);
  const __amdgpu_buffer_rsrc_t rsi = make_rsrc(p.b, p.b_bytes);
  const __amdgpu_buffer_rsrc_t rsbias = make_rsrc(p.bias, p.bias ? p.M * 4u : 0u);
  uint32_t wrel[LWA], wc4[LWA], srel[LWB], srow[LWB];  // wc4 / srow = 0xffff: a piece that never loads
#pragma unroll
  for (int j = 0; j < LWA; ++j) {
    const uint32_t e = (uint32_t)((wave * LWA + j) * 64 + lane);
    const uint32_t tap = e / (OCT / 4);
    wc4[j] = tap < (uint32_t)KK ? 4 * (e % (OCT / 4)) : 0xffffu;
    wrel[j] = (tap * p.IC * p.lda + 4 * (e % (OCT / 4))) * 4u;
  }
  const uint32_t pxa = V4 ? (p.px ? 4u : 0u) : p.px;  // strip column of input x = 0
#pragma unroll
  for (int j = 0; j < LWB; ++j) {
    const uint32_t e = (uint32_t)((wave * LWB + j) * 64 + lane) * PW;  // first strip element of the lane
    const uint32_t r = e / WPM, q = e - (e / WPM) * WPM;
    const uint32_t c = PSL ? (q % WS) * S + q / WS : q;  // PSL: LDS position q holds column c
    const int x = (int)c - (int)pxa;
    // V4: a piece is inside the row or outside it as a whole (W % 4 == 0, pxa % 4 == 0)
    srow[j] = ((r < (uint32_t)RIN) & ((uint32_t)x < p.W)) ? r : 0xffffu;
    srel[j] = (r * p.W + (uint32_t)x) * 4u;
  }

  // DMA sources of block stage g (tile g / IC, input channel g % IC): the per-lane part depends
  // on the tile only and is planned once per tile (tvo, VGPRs); the channel's part is a scalar
  // soffset (ic * HW for the strip, ic * OC4 for the bank rows), so issuing a stage costs no
  // vector work -- every VALU op between f32 MFMAs is MFMA time lost (one wave per SIMD).
  // Stages past the block's last tile belong to a dead tile: all misses (OOB zeros, no memory
  // traffic), so every wave always has the same number of DMAs in flight and nothing branches.
  uint32_t tvo[LW];
  auto plan_tile = [&](uint32_t i) {
    uint32_t oc0, img, p0;
    decode(b0 + i * G, oc0, img, p0);
    const uint32_t dead = i < my_tiles ? 0u : OOB;
    const uint32_t wlim = p.lda - min(oc0, p.lda), wb = oc0 * 4u;
#pragma unroll
    for (int j = 0; j < LWA; ++j) tvo[j] = oob_unless(wc4[j] < wlim, wrel[j] + wb) | dead;
    const int ya = (int)(fdiv(p0, p.ow_m, p.ow_s) * S) - (int)p.py;  // input row of strip row 0
    const uint32_t rlo = (uint32_t)max(0, -ya), rhi = (uint32_t)max(0, (int)p.H - ya);
    const uint32_t sb = img * p.ICHW * 4u + (uint32_t)(ya * (int)p.W) * 4u;
#pragma unroll
    for (int j = 0; j < LWB; ++j)
      tvo[LWA + j] = oob_unless((srow[j] >= rlo) & (srow[j] < rhi), srel[j] + sb) | dead;
    tvo[LW - 1] = oob_unless((uint32_t)(64 * wave + lane) < (uint32_t)OCT, (oc0 + 64 * wave + lane) * 4u) | dead;
  };
  auto issue_one = [&](int q, int slot, uint32_t ic) {
    float *const base = smem + slot * SLOT;
    if (q < LWA) dma16s(rsw, base + (wave * LWA + q) * 256, tvo[q], ic * p.lda * 4u);
    else if (q < LWA + LWB) {
      if constexpr (V4) dma16s(rsi, base + WREG + (wave * LWB + q - LWA) * 256, tvo[q], ic * p.HW * 4u);
      else dma4s(rsi, base + WREG + (wave * LWB + q - LWA) * 64, tvo[q], ic * p.HW * 4u);
    }
    else dma4(rsbias, base + WREG + SREG + 64 * wave, tvo[q]);
  };

  f32x16 acc[TM][TN];
  uint32_t poff[TN];  // this lane's pixels' strip offsets in the current tile (bytes)
  uint32_t hsel = kh ? 0xffffffffu : 0u;

  // deferred stores of the previous tile: float4 piece q = (t, tn, g) of this lane, at dstore[q]
  // (byte offset, or OOB where the piece is outside the output)
  f32x4v dval[NST];
  uint32_t dbase[TM], dpx = 0, dhw = 0;  // piece (t, tn, gq): byte offset dbase[t] + 4 (32 tn + 8 gq), pixel
                                         // dpx + 32 tn + 8 gq (dropped at >= dhw: past the image)
  const __amdgpu_buffer_rsrc_t rso = make_rsrc(p.c, p.c_bytes);
  // (any dword alignment: OHW % 4 != 0 puts a channel's row at m * OHW; a piece running past the
  // image's last pixel goes element by element)
  auto store_one = [&](int q) {
    const int t = q / (TN * 4), tn = (q / 4) % TN, gq = q % 4;
    const uint32_t px = dpx + (uint32_t)(32 * tn + 8 * gq);
    const uint32_t off = dbase[t] + (uint32_t)(32 * tn + 8 * gq) * 4u;
    if (px + 4 <= dhw) {
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) uint32_t, dval[q]),
                                             rso, off, 0, AUX_OUT);
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        // (a scalar first: __builtin_bit_cast of a vector component made hipcc store component 0
        // four times -- caught by the 224-wide, OH*OW % 4 == 2 test shapes)
        const float xe = dval[q][e];
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, xe), rso,
                                              oob_unless(px + (uint32_t)e < dhw, off + 4u * (uint32_t)e), 0, AUX_OUT);
      }
    }
  };

  // one stage = one input channel of one tile: KK2 steps of TM x TN MFMAs; stage g_issue's
  // DMAs are issued over the first IS steps, the previous tile's deferred stores (if any) over
  // the first ISS; LDS fragments are read PF steps ahead
  auto compute = [&](int slot, int islot, uint32_t g_issue, bool dstores) {
    const uint32_t i_issue = fdiv(g_issue, p.ic_m, p.ic_s), ic_issue = g_issue - i_issue * p.IC;
    if (ic_issue == 0) plan_tile(i_issue);  // wave-uniform
    const float *const Ab = smem + slot * SLOT + kh * KK2 * OCT + li;
    const char *const Sb = (const char *)(smem + slot * SLOT + WREG);
    if constexpr (PSL) {
      // phase-split strip: one per-lane base per distinct half-1 shift (a handful), the step loop
      // unrolled at compile time so that every fragment read is base[kind(s)] + immediate
      using PK = dc_pkinds<KY, KX, S, WPM>;
      constexpr int NK = PK::tab.nk;
      asm volatile("" : "+v"(hsel));
      const char *bs[NK][TN];
      dc_static_for<0, NK>([&](auto kc) {
        constexpr int dkv = PK::tab.dk[decltype(kc)::value];
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) bs[decltype(kc)::value][tn] = Sb + poff[tn] + (int)(hsel & (uint32_t)(dkv * 4));
      });
      auto fragp = [&](auto sc, float(&a)[TM], float(&b)[TN]) {
        constexpr int s = decltype(sc)::value;
        constexpr int k0 = dc_koffp<KX, S, WPM>(s, KK) * 4, kind = PK::tab.kind[s];
#pragma unroll
        for (int t = 0; t < TM; ++t) a[t] = Ab[s * OCT + 32 * t];
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) b[tn] = *(const float *)(bs[kind][tn] + k0);
      };
      float a[PF + 1][TM], b[PF + 1][TN];
      dc_static_for<0, PF>([&](auto sc) {
        constexpr int s = decltype(sc)::value;
        if constexpr (s < KK2) fragp(sc, a[s], b[s]);
      });
      dc_static_for<0, KK2>([&](auto sc) {
        constexpr int s = decltype(sc)::value;
        if constexpr (s + PF < KK2) fragp(std::integral_constant<int, s + PF>{}, a[(s + PF) % (PF + 1)], b[(s + PF) % (PF + 1)]);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int t = 0; t < TM; ++t)
#pragma unroll
          for (int tn = 0; tn < TN; ++tn)
            acc[t][tn] = __builtin_amdgcn_mfma_f32_32x32x2f32(b[s % (PF + 1)][tn], a[s % (PF + 1)][t], acc[t][tn], 0, 0, 0);
#pragma unroll
        for (int q = (s * LW + IS - 1) / IS; q < ((s + 1) * LW + IS - 1) / IS && q < LW; ++q) issue_one(q, islot, ic_issue);
        if (dstores) {
#pragma unroll
          for (int q = (s * NST + ISS - 1) / ISS; q < ((s + 1) * NST + ISS - 1) / ISS && q < NST; ++q) store_one(q);
        }
        __builtin_amdgcn_sched_barrier(0);
      });
      return;
    }
    // Lane half 1 reads tap KK2 + s where half 0 reads tap s: its strip offset is larger by
    // dk(s) = koff(KK2 + s) - koff(s), which takes only two values over the real taps (DLO while
    // the column shift KK2 % KX does not wrap, DHI when it does) and a third at the padding
    // tap (KK odd: the last step; zero weights, so any in-strip offset -- tap 0). Three per-lane
    // bases per stage, then every step's B fragment is one ds_read at base + a compile-time
    // immediate: no per-step select or add (each VALU op between f32 MFMAs is MFMA time lost).
    constexpr int CSH = KK2 % KX, RSH = KK2 / KX;
    constexpr int DLO = RSH * WPM + CSH, DHI = (RSH + 1) * WPM + CSH - KX;
    constexpr int DPAD = -dc_koff<KX, WPM>(KK2 - 1, KK);
    // opaque per stage: keeps the bases' lane-half selects from being rematerialized per step
    asm volatile("" : "+v"(hsel));
    const char *bs[3][TN];
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) {
      bs[0][tn] = Sb + poff[tn] + (hsel & (uint32_t)(DLO * 4));
      bs[1][tn] = Sb + poff[tn] + (hsel & (uint32_t)(DHI * 4));
      bs[2][tn] = Sb + poff[tn] + (int)(hsel & (uint32_t)(DPAD * 4));
    }
    auto frag = [&](int s, float (&a)[TM], float (&b)[TN]) {
#pragma unroll
      for (int t = 0; t < TM; ++t) a[t] = Ab[s * OCT + 32 * t];
      const int k0 = dc_koff<KX, WPM>(s, KK) * 4;
      const int kind = KK2 + s >= KK ? 2 : (s % KX < KX - CSH ? 0 : 1);
#pragma unroll
      for (int tn = 0; tn < TN; ++tn) b[tn] = *(const float *)(bs[kind][tn] + k0);
    };
    float a[PF + 1][TM], b[PF + 1][TN];
#pragma unroll
    for (int s = 0; s < PF; ++s) frag(s, a[s], b[s]);
#pragma unroll
    for (int s = 0; s < KK2; ++s) {
      if (s + PF < KK2) frag(s + PF, a[(s + PF) % (PF + 1)], b[(s + PF) % (PF + 1)]);
      __builtin_amdgcn_sched_barrier(0);  // keep the prefetch ahead of this step's MFMAs
      // A = the strip (MFMA rows: pixels), B = the weights (columns: output channels)
#pragma unroll
      for (int t = 0; t < TM; ++t)
#pragma unroll
        for (int tn = 0; tn < TN; ++tn)
          acc[t][tn] = __builtin_amdgcn_mfma_f32_32x32x2f32(b[s % (PF + 1)][tn], a[s % (PF + 1)][t], acc[t][tn], 0, 0, 0);
      // q in [QB(s), QB(s+1)), QB(s) = ceil(s * LW / IS): early, so that even the last DMA has
      // most of a stage to land before the wait that retires it (the very next stage at D = 2)
#pragma unroll
      for (int q = (s * LW + IS - 1) / IS; q < ((s + 1) * LW + IS - 1) / IS && q < LW; ++q)
        issue_one(q, islot, ic_issue);
      if (dstores) {
#pragma unroll
        for (int q = (s * NST + ISS - 1) / ISS; q < ((s + 1) * NST + ISS - 1) / ISS && q < NST; ++q) store_one(q);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  // ---- prologue: stages 0 .. D-2 in flight
#pragma unroll
  for (int s = 0; s < D - 1; ++s) {
    const uint32_t i_s = fdiv((uint32_t)s, p.ic_m, p.ic_s), ic_s = (uint32_t)s - i_s * p.IC;
    if (ic_s == 0) plan_tile(i_s);
#pragma unroll
    for (int q = 0; q < LW; ++q) issue_one(q, s, ic_s);
  }
  const bool vec = !p.res;  // float4 pieces, deferred (else stored at once)
  const __amdgpu_buffer_rsrc_t rsr = make_rsrc(p.res, p.res ? p.c_bytes : 0u);
  bool pending = false;  // deferred stores of the previous tile not yet issued
  int slot = 0;
  uint32_t g = 0;
  // outer loop over the block's tiles, inner over a tile's input channels (nested: the
  // accumulators stay in AGPRs); the ring runs on across tiles, so the next tile's first stage
  // lands while this tile's epilogue runs, and its stores go out during the next tile
  for (uint32_t i = 0; i < my_tiles; ++i) {
    uint32_t oc0, img, p0;
    decode(b0 + i * G, oc0, img, p0);
    const uint32_t oy_a = fdiv(p0, p.ow_m, p.ow_s);
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) {
      const uint32_t px = p0 + (uint32_t)(wave * 32 * TN + 32 * tn + li);
      const uint32_t oy = fdiv(px, p.ow_m, p.ow_s), ox = px - oy * p.OW;
      poff[tn] = px < p.OHW ? ((oy - oy_a) * S * WPM + (PSL ? ox : ox * S) + pxa - p.px) * 4u : 0u;
    }
#pragma unroll
    for (int t = 0; t < TM; ++t)
#pragma unroll
      for (int tn = 0; tn < TN; ++tn)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[t][tn][r] = 0.0f;
    int cslot = 0;
    for (uint32_t ic = 0; ic < p.IC; ++ic, ++g) {
      vm_wait<(D - 2) * LW>();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();  // stage g landed for all waves; all done reading g-1
      asm volatile("" ::: "memory");
      if (i == 0 && ic == 0) KT(1);
      if (i == 1 && ic == 0) KT(5);
      // + stage g+D-1 into slot (g-1) % D, and in a tile's first stage the previous tile's stores
      compute(slot, slot == 0 ? D - 1 : slot - 1, g + D - 1, pending);
      pending = false;
      cslot = slot;
      slot = slot == D - 1 ? 0 : slot + 1;
    }
    if (i == 0) KT(2);
    if (i == 1) KT(6);

    // ---- epilogue. acc[t][tn][4*gq + e] is output channel oc0 + 32 t + li, pixel
    // p0 + wave*32*TN + 32 tn + 8 gq + 4 kh + e (e = 0..3): bias (from the consumed slot: no DMA
    // targets it before the next stage's compute), ReLU, then 16-B pieces -- deferred into the
    // next tile's first stage, or stored now if this is the block's last tile. With a residual
    // or an output whose pixel runs are not 16-B pieces: element stores now.
    const float *const Lb = smem + cslot * SLOT + WREG + SREG;
    const uint32_t obase = img * p.OCOHW;
    if (vec) {
      dpx = p0 + (uint32_t)(wave * 32 * TN + 4 * kh);
      dhw = p.OHW;
#pragma unroll
      for (int t = 0; t < TM; ++t) {
        const uint32_t m = oc0 + 32 * t + li;
        const float bb = Lb[32 * t + li];
        dbase[t] = oob_unless(m < p.M, (obase + m * p.OHW + dpx) * 4u);
#pragma unroll
        for (int tn = 0; tn < TN; ++tn)
#pragma unroll
          for (int gq = 0; gq < 4; ++gq) {
            f32x4v v;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const float x = acc[t][tn][4 * gq + e] + bb;
              v[e] = (p.relu && x < 0.0f) ? 0.0f : x;
            }
            dval[(t * TN + tn) * 4 + gq] = v;
          }
      }
      if (i + 1 < my_tiles) {
        pending = true;
      } else {
#pragma unroll
        for (int q = 0; q < NST; ++q) store_one(q);
      }
    } else {
#pragma unroll
      for (int t = 0; t < TM; ++t) {
        const uint32_t m = oc0 + 32 * t + li;
        const float bb = Lb[32 * t + li];
#pragma unroll
        for (int tn = 0; tn < TN; ++tn)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const uint32_t px = p0 + (uint32_t)(wave * 32 * TN + 32 * tn + 8 * (r >> 2) + 4 * kh + (r & 3));
            const uint32_t o = oob_unless((m < p.M) & (px < p.OHW), (obase + m * p.OHW + px) * 4u);
            float x = acc[t][tn][r] + bb;
            if (p.res) x += __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rsr, o, 0, 0));
            x = (p.relu && x < 0.0f) ? 0.0f : x;
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, x), rso, o, 0, AUX_OUT);
          }
      }
    }
    if (i == 0) KT(3);
  }
  vm_wait<0>();
#ifdef BH_KTRACE
  KT(4);
#endif
}

// Resident-weight form (configs dc<k>s<s>r*, round 5). PMC of the b20 11x11 s4 stem on dc_kernel
// (profiles/r04/pmc_stems.json): the MFMA pipe 65 % busy, 64 % of wave cycles waiting on the stage
// ring, ~38 KB of LDS-DMA per 61-step stage (the weights [2 KK2][OCT] re-fetched for every tile and
// channel: 43 % of it) -- about 8.7 B/clk per CU at two blocks per CU, above what the LDS-DMA path
// sustains. Here a block of NW = 8 waves owns ONE OC tile for its whole life (a grid that is a
// multiple of the OC tiles, tiles dealt OC-fastest), so:
//  * every input channel's weights [2 KK2 taps][OCT] and the tile's biases are DMA'd into LDS once,
//    in the prologue (IC <= ICMAX), and stay resident;
//  * the ring carries only the input strips: one per (tile, input channel) stage, RIN rows of the
//    NPX = 32 NW pixels' input at pitch WPM -- 256 pixels' rows, which overlap, for what two
//    128-pixel blocks fetched twice;
//  * a step is as in dc_kernel: A = resident weights (one ds_read_b32 per tile), B = the strip at a
//    compile-time tap offset from one of three per-lane bases; the next stage's strip DMAs spread
//    over the first IS steps, the previous tile's output stores deferred into the first steps.
// DBG (diagnostic builds in the instrumented library only; wrong results by design): bit 0 = no strip DMA
// after the prologue, 1 = no MFMA, 2 = no output stores, 3 = no stage barrier, 4 = no B (strip) fragment
// reads, 5 = no A (weight) fragment reads
template <int KY, int KX, int S, int WPM, int RIN, int TM, int NW, int D, int V4, int ICMAX, int DBG = 0, int PFO = 0,
          int PSL = 0>
__global__ __launch_bounds__(NW * 64) void dcr_kernel(GemmArgs p) {
  constexpr int NT = NW * 64, NPX = NW * 32, OCT = 32 * TM;
  constexpr int KK = KY * KX, KK2 = (KK + 1) / 2;
  constexpr int WPC = 2 * KK2 * OCT / 4;                    // 16-B weight pieces per input channel
  constexpr int LWA = (WPC + NT - 1) / NT;                  // weight DMA instructions per wave and channel
  constexpr int WREGC = LWA * NT * 4;                       // floats per channel (whole DMA instructions)
  constexpr int BREG = ((OCT + 63) / 64) * 64;              // biases: one dword DMA per 64 channels
  constexpr int SF = RIN * WPM;
  constexpr int PW = V4 ? 4 : 1;
  static_assert(WPM % PW == 0, "16-B strip rows");
  static_assert(!PSL || (!V4 && WPM % S == 0), "phase-split strip: dword DMA, whole phases per row");
  constexpr int WS = WPM / S;                               // PSL: strip floats per column phase
  constexpr int LWB = (SF / PW + NT - 1) / NT;              // strip DMA instructions per wave and stage
  constexpr int SREG = LWB * NT * PW;                       // floats per strip slot
  static_assert(D >= 2 && (D - 2) * LWB <= 63, "vmcnt range");
  static_assert(OCT % 4 == 0 && BREG <= NT, "16-B weight pieces, one bias DMA per wave at most");
  constexpr int PF = PFO > 0 ? PFO : (TM >= 2 ? 2 : 3);    // LDS fragment prefetch distance (steps)
  constexpr int IS = (KK2 + 1) / 2 > 1 ? (KK2 + 1) / 2 : 1;   // steps the next stage's DMAs are spread over
  constexpr int NST = TM * 4;                               // deferred float4 stores per lane and tile
  constexpr int ISS = KK2 > 2 * NST ? 2 * NST : KK2;
  // one __shared__ array: [ICMAX channels' weights][biases][D strip slots]
  __shared__ __attribute__((aligned(16))) float smem[ICMAX * WREGC + BREG + D * SREG];
  float *const wres = smem, *const bres = smem + ICMAX * WREGC, *const ring = bres + BREG;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int kh = lane >> 5, li = lane & 31;
  KT(0);

  // ---- this block's OC tile (fixed: gridDim.x is a multiple of the OC tiles, p.ipt) and its tiles
  // t = blockIdx.x + i * gridDim.x = (pixel run, image, OC tile), OC tile fastest
  const uint32_t G = gridDim.x, b0 = blockIdx.x;
  const uint32_t ntile = p.total_it;
  const uint32_t my_tiles = b0 < ntile ? (ntile - b0 + G - 1) / G : 0;
  const uint32_t oc0 = (b0 - fdiv(b0, p.ipt_m, p.ipt_s) * p.ipt) * OCT;
  auto decode = [&](uint32_t t, uint32_t &img, uint32_t &p0) {
    const uint32_t rest = fdiv(t, p.ipt_m, p.ipt_s);
    img = fdiv(rest, p.tm_m, p.tm_s);
    p0 = (rest - img * p.tiles_n) * NPX;
  };
  const __amdgpu_buffer_rsrc_t rsw = make_rsrc(p.a, p.a_bytes);
  const __amdgpu_buffer_rsrc_t rsi = make_rsrc(p.b, p.b_bytes);
  const __amdgpu_buffer_rsrc_t rsbias = make_rsrc(p.bias, p.bias ? p.M * 4u : 0u);

  // ---- resident weights and biases: piece e of channel ic's [tap][OCT] image is packed-bank row
  // tap * IC + ic (K order (ky, kx, ic)), columns oc0 + 4 (e % (OCT / 4)); taps >= KK (the odd
  // kernel's padding tap) and columns past OC4 miss: zeros
#pragma unroll
  for (int j = 0; j < LWA; ++j) {
    const uint32_t e = (uint32_t)((j * NW + wave) * 64 + lane), tap = e / (OCT / 4), c4 = 4 * (e % (OCT / 4));
    const uint32_t off = oob_unless((tap < (uint32_t)KK) & (oc0 + c4 < p.lda), (tap * p.IC * p.lda + oc0 + c4) * 4u);
    for (uint32_t ic = 0; ic < p.IC; ++ic) dma16s(rsw, wres + ic * WREGC + (j * NW + wave) * 256, off, ic * p.lda * 4u);
  }
  if (64 * wave < BREG)
    dma4(rsbias, bres + 64 * wave, oob_unless(oc0 + 64 * wave + lane < p.M, (oc0 + 64 * wave + lane) * 4u));

  // ---- strip DMA sources: element e = (row r, column c) of the [RIN][WPM] image; per tile the lane
  // part (tvo, VGPRs), per channel the scalar soffset ic * HW; dead stages (past the block's last
  // tile) miss, so every wave always has the same DMAs in flight
  const uint32_t pxa = V4 ? (p.px ? 4u : 0u) : p.px;  // strip column of input x = 0
  uint32_t srel[LWB], srow[LWB], tvo[LWB];
#pragma unroll
  for (int j = 0; j < LWB; ++j) {
    const uint32_t e = (uint32_t)((wave * LWB + j) * 64 + lane) * PW;
    const uint32_t r = e / WPM, q = e - r * WPM;
    const uint32_t c = PSL ? (q % WS) * S + q / WS : q;  // PSL: LDS position q holds column c
    const int x = (int)c - (int)pxa;
    srow[j] = ((r < (uint32_t)RIN) & ((uint32_t)x < p.W)) ? r : 0xffffu;
    srel[j] = (r * p.W + (uint32_t)x) * 4u;
  }
  auto plan_tile = [&](uint32_t i) {
    uint32_t img, p0;
    decode(b0 + i * G, img, p0);
    const uint32_t dead = i < my_tiles ? 0u : OOB;
    const int ya = (int)(fdiv(p0, p.ow_m, p.ow_s) * S) - (int)p.py;  // input row of strip row 0
    const uint32_t rlo = (uint32_t)max(0, -ya), rhi = (uint32_t)max(0, (int)p.H - ya);
    const uint32_t sb = img * p.ICHW * 4u + (uint32_t)(ya * (int)p.W) * 4u;
#pragma unroll
    for (int j = 0; j < LWB; ++j) tvo[j] = oob_unless((srow[j] >= rlo) & (srow[j] < rhi), srel[j] + sb) | dead;
  };
  auto issue_one = [&](int q, int slot, uint32_t ic) {
    float *const base = ring + slot * SREG + (wave * LWB + q) * 64 * PW;
    if constexpr (V4) dma16s(rsi, base, tvo[q], ic * p.HW * 4u);
    else dma4s(rsi, base, tvo[q], ic * p.HW * 4u);
  };

  f32x16 acc[TM];
  uint32_t poff = 0;  // this lane's pixel's strip offset in the current tile (bytes)
  uint32_t hsel = kh ? 0xffffffffu : 0u;
  f32x4v dval[NST];
  uint32_t dbase[TM], dpx = 0, dhw = 0;
  const __amdgpu_buffer_rsrc_t rso = make_rsrc(p.c, p.c_bytes);
  auto store_one = [&](int q) {  // deferred float4 piece q = (t, gq) of the previous tile
    const int t = q / 4, gq = q % 4;
    const uint32_t px = dpx + (uint32_t)(8 * gq);
    const uint32_t off = (DBG & 4) ? OOB : dbase[t] + (uint32_t)(8 * gq) * 4u;
    if (px + 4 <= dhw) {
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) uint32_t, dval[q]),
                                             rso, off, 0, AUX_OUT);
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float xe = dval[q][e];
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, xe), rso,
                                              oob_unless(px + (uint32_t)e < dhw, off + 4u * (uint32_t)e), 0, AUX_OUT);
      }
    }
  };

  // one stage = one input channel of one tile (KK2 steps of TM MFMAs); stage g_issue's strip DMAs
  // go out over the first IS steps, the previous tile's deferred stores over the first ISS
  auto compute = [&](int slot, int islot, uint32_t ic, uint32_t g_issue, bool dstores) {
    const uint32_t i_issue = fdiv(g_issue, p.ic_m, p.ic_s), ic_issue = g_issue - i_issue * p.IC;
    if (ic_issue == 0) plan_tile(i_issue);  // wave-uniform
    const float *const Ab = wres + ic * WREGC + kh * KK2 * OCT + li;
    const char *const Sb = (const char *)(ring + slot * SREG);
    if constexpr (PSL) {
      // phase-split strip (dc_kernel): one per-lane base per distinct half-1 shift, every fragment read
      // base[kind(s)] + an immediate, the 32 pixels of a lane half on 32 consecutive dwords
      using PK = dc_pkinds<KY, KX, S, WPM>;
      constexpr int NK = PK::tab.nk;
      asm volatile("" : "+v"(hsel));
      const char *bs[NK];
      dc_static_for<0, NK>([&](auto kc) {
        constexpr int dkv = PK::tab.dk[decltype(kc)::value];
        bs[decltype(kc)::value] = Sb + poff + (int)(hsel & (uint32_t)(dkv * 4));
      });
      auto fragp = [&](auto sc, float(&a)[TM], float &b) {
        constexpr int s = decltype(sc)::value;
        constexpr int k0 = dc_koffp<KX, S, WPM>(s, KK) * 4, kind = PK::tab.kind[s];
#pragma unroll
        for (int t = 0; t < TM; ++t) a[t] = (DBG & 32) ? (float)(s + t) : Ab[s * OCT + 32 * t];
        b = (DBG & 16) ? (float)s : *(const float *)(bs[kind] + k0);
      };
      float a[PF + 1][TM], b[PF + 1];
      dc_static_for<0, PF>([&](auto sc) {
        constexpr int s = decltype(sc)::value;
        if constexpr (s < KK2) fragp(sc, a[s], b[s]);
      });
      dc_static_for<0, KK2>([&](auto sc) {
        constexpr int s = decltype(sc)::value;
        if constexpr (s + PF < KK2) fragp(std::integral_constant<int, s + PF>{}, a[(s + PF) % (PF + 1)], b[(s + PF) % (PF + 1)]);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int t = 0; t < TM; ++t) {
          if constexpr ((DBG & 2) != 0) acc[t][s % 16] += b[s % (PF + 1)] * a[s % (PF + 1)][t];
          else acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(b[s % (PF + 1)], a[s % (PF + 1)][t], acc[t], 0, 0, 0);
        }
        if constexpr ((DBG & 1) == 0) {
#pragma unroll
          for (int q = (s * LWB + IS - 1) / IS; q < ((s + 1) * LWB + IS - 1) / IS && q < LWB; ++q) issue_one(q, islot, ic_issue);
        }
        if (dstores) {
#pragma unroll
          for (int q = (s * NST + ISS - 1) / ISS; q < ((s + 1) * NST + ISS - 1) / ISS && q < NST; ++q) store_one(q);
        }
        __builtin_amdgcn_sched_barrier(0);
      });
      return;
    }
    // lane half 1 reads tap KK2 + s where half 0 reads tap s: three per-lane bases (dc_kernel)
    constexpr int CSH = KK2 % KX, RSH = KK2 / KX;
    constexpr int DLO = RSH * WPM + CSH, DHI = (RSH + 1) * WPM + CSH - KX;
    constexpr int DPAD = -dc_koff<KX, WPM>(KK2 - 1, KK);
    asm volatile("" : "+v"(hsel));
    const char *bs[3] = {Sb + poff + (hsel & (uint32_t)(DLO * 4)), Sb + poff + (hsel & (uint32_t)(DHI * 4)),
                         Sb + poff + (int)(hsel & (uint32_t)(DPAD * 4))};
    auto frag = [&](int s, float (&a)[TM], float &b) {
#pragma unroll
      for (int t = 0; t < TM; ++t) a[t] = (DBG & 32) ? (float)(s + t) : Ab[s * OCT + 32 * t];
      const int k0 = dc_koff<KX, WPM>(s, KK) * 4;
      const int kind = KK2 + s >= KK ? 2 : (s % KX < KX - CSH ? 0 : 1);
      b = (DBG & 16) ? (float)s : *(const float *)(bs[kind] + k0);
    };
    float a[PF + 1][TM], b[PF + 1];
#pragma unroll
    for (int s = 0; s < PF; ++s) frag(s, a[s], b[s]);
#pragma unroll
    for (int s = 0; s < KK2; ++s) {
      if (s + PF < KK2) frag(s + PF, a[(s + PF) % (PF + 1)], b[(s + PF) % (PF + 1)]);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int t = 0; t < TM; ++t) {
        if constexpr ((DBG & 2) != 0) acc[t][s % 16] += b[s % (PF + 1)] * a[s % (PF + 1)][t];
        else acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(b[s % (PF + 1)], a[s % (PF + 1)][t], acc[t], 0, 0, 0);
      }
      if constexpr ((DBG & 1) == 0) {
#pragma unroll
        for (int q = (s * LWB + IS - 1) / IS; q < ((s + 1) * LWB + IS - 1) / IS && q < LWB; ++q) issue_one(q, islot, ic_issue);
      }
      if (dstores) {
#pragma unroll
        for (int q = (s * NST + ISS - 1) / ISS; q < ((s + 1) * NST + ISS - 1) / ISS && q < NST; ++q) store_one(q);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  // ---- prologue: strips of stages 0 .. D-2 (behind the resident weights: the first stage's wait
  // covers them)
#pragma unroll
  for (int s = 0; s < D - 1; ++s) {
    const uint32_t i_s = fdiv((uint32_t)s, p.ic_m, p.ic_s), ic_s = (uint32_t)s - i_s * p.IC;
    if (ic_s == 0) plan_tile(i_s);
#pragma unroll
    for (int q = 0; q < LWB; ++q) issue_one(q, s, ic_s);
  }
  const bool vec = !p.res;
  const __amdgpu_buffer_rsrc_t rsr = make_rsrc(p.res, p.res ? p.c_bytes : 0u);
  // the tile's biases start every tile's accumulators (no bias add in the epilogue); the ReLU is one
  // v_max against a wave-uniform floor (0, or -inf without ReLU). Once per kernel: every DMA so far
  // (weights, biases, the prologue's strips) landed, every wave's
  vm_wait<0>();
  __syncthreads();
  float biasr[TM];
#pragma unroll
  for (int t = 0; t < TM; ++t) biasr[t] = bres[32 * t + li];
  const float floor0 = p.relu ? 0.0f : __builtin_nanf("");  // relu_floor: NaN = no clamp
  bool pending = false;
  int slot = 0;
  uint32_t g = 0;
  for (uint32_t i = 0; i < my_tiles; ++i) {
    uint32_t img, p0;
    decode(b0 + i * G, img, p0);
    const uint32_t oy_a = fdiv(p0, p.ow_m, p.ow_s);
    {
      const uint32_t px = p0 + (uint32_t)(wave * 32 + li);
      const uint32_t oy = fdiv(px, p.ow_m, p.ow_s), ox = px - oy * p.OW;
      poff = px < p.OHW ? ((oy - oy_a) * S * WPM + (PSL ? ox : ox * S) + pxa - p.px) * 4u : 0u;
    }
#pragma unroll
    for (int t = 0; t < TM; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[t][r] = biasr[t];
    for (uint32_t ic = 0; ic < p.IC; ++ic, ++g) {
      vm_wait<(D - 2) * LWB>();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (!(DBG & 8) || (i == 0 && ic == 0))
        __builtin_amdgcn_s_barrier();  // stage g (and, the first time, the weights) landed; all done with g-1
      asm volatile("" ::: "memory");
      if (i == 0 && ic == 0) KT(1);
      compute(slot, slot == 0 ? D - 1 : slot - 1, ic, g + D - 1, pending);
      pending = false;
      slot = slot == D - 1 ? 0 : slot + 1;
    }
    if (i == 0) KT(2);
    // ---- epilogue: acc[t][4 gq + e] is output channel oc0 + 32 t + li, pixel p0 + 32 wave + 8 gq +
    // 4 kh + e: bias, ReLU, 16-B pieces deferred into the next tile's first steps (stored now after
    // the block's last tile); with a residual, element stores now
    const uint32_t obase = img * p.OCOHW;
    if (vec) {
      dpx = p0 + (uint32_t)(wave * 32 + 4 * kh);
      dhw = p.OHW;
#pragma unroll
      for (int t = 0; t < TM; ++t) {
        const uint32_t m = oc0 + 32 * t + li;
        dbase[t] = oob_unless(m < p.M, (obase + m * p.OHW + dpx) * 4u);
#pragma unroll
        for (int gq = 0; gq < 4; ++gq) {
          f32x4v v;
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = relu_floor(acc[t][4 * gq + e], floor0);
          dval[t * 4 + gq] = v;
        }
      }
      if (i + 1 < my_tiles) {
        pending = true;
      } else {
#pragma unroll
        for (int q = 0; q < NST; ++q) store_one(q);
      }
    } else {
#pragma unroll
      for (int t = 0; t < TM; ++t) {
        const uint32_t m = oc0 + 32 * t + li;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const uint32_t px = p0 + (uint32_t)(wave * 32 + 8 * (r >> 2) + 4 * kh + (r & 3));
          const uint32_t o = oob_unless((m < p.M) & (px < p.OHW), (obase + m * p.OHW + px) * 4u);
          float x = acc[t][r];
          if (p.res) x += __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rsr, o, 0, 0));
          x = relu_floor(x, floor0);
          __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, x), rso, o, 0, AUX_OUT);
        }
      }
    }
    if (i == 0) KT(3);
  }
  vm_wait<0>();
#ifdef BH_KTRACE
  KT(4);
#endif
}

template <int KY, int KX, int S, int WPM, int RIN, int TM, int NW, int D, int V4, int ICMAX, int DBG = 0, int PFO = 0,
          int PSL = 0>
cfg_t dcr_cfg(const char *name) {
  cfg_t c{name, 32 * TM, 32 * NW, 2 * ((KY * KX + 1) / 2), 64 * NW, {}, 1};
  c.k[A_KVEC][B_DIRECT][0] = dcr_kernel<KY, KX, S, WPM, RIN, TM, NW, D, V4, ICMAX, DBG, PFO, PSL>;
  c.dc_ci = V4;
  c.dc = 1;
  c.dc_ky = KY;
  c.dc_kx = KX;
  c.dc_s = S;
  c.dc_wpm = WPM;
  c.dc_rin = RIN;
  c.dc_icmax = ICMAX;  // resident weights: input channels <= ICMAX, grid a multiple of the OC tiles
  return c;
}

template <int KY, int KX, int S, int WPM, int RIN, int TM, int TN, int D, int V4 = 0, int PSL = 0, int PFO = 0>
cfg_t dc_cfg(const char *name) {
  cfg_t c{name, 32 * TM, 128 * TN, 2 * ((KY * KX + 1) / 2), 256, {}, 1};
  c.k[A_KVEC][B_DIRECT][0] = dc_kernel<KY, KX, S, WPM, RIN, TM, TN, D, V4, PSL, PFO>;
  c.dc_ci = V4;  // dc == 1: 16-B strip pieces (input rows of W % 4 == 0)
  c.dc = 1;
  c.dc_ky = KY;
  c.dc_kx = KX;
  c.dc_s = S;
  c.dc_wpm = WPM;
  c.dc_rin = RIN;
  return c;
}

}  // namespace

std::vector<cfg_t> dc_cfgs() {
  return {
      // GoogLeNet conv1 (3 x 224^2 -> 64, 7x7 s2 p3); 96 channels: the op_sigs 7x7 s2 stem
      dc_cfg<7, 7, 2, 236, 13, 2, 2, 2>("dc7s2x64d2"),
      dc_cfg<7, 7, 2, 236, 13, 2, 2, 3>("dc7s2x64d3"),
      dc_cfg<7, 7, 2, 236, 13, 1, 2, 3>("dc7s2x32d3"),
      dc_cfg<7, 7, 2, 236, 13, 3, 2, 2>("dc7s2x96d2"),
      dc_cfg<7, 7, 2, 236, 11, 2, 1, 2>("dc7s2x64n128d2"),
      dc_cfg<7, 7, 2, 236, 11, 2, 1, 2, 1>("dc7s2x64n128d2v"),
      dc_cfg<7, 7, 2, 236, 13, 2, 2, 2, 1>("dc7s2x64d2v"),
      dc_cfg<7, 7, 2, 236, 11, 2, 1, 3, 1>("dc7s2x64n128d3v"),
      // AlexNet conv1 (3 x 227^2 / 224^2 -> 96, 11x11 s4)
      dc_cfg<11, 11, 4, 228, 23, 3, 1, 2>("dc11s4x96d2"),
      dc_cfg<11, 11, 4, 228, 23, 1, 1, 2>("dc11s4x32d2"),
      dc_cfg<11, 11, 4, 228, 23, 1, 1, 3>("dc11s4x32d3"),
      dc_cfg<11, 11, 4, 228, 23, 1, 1, 2, 1>("dc11s4x32d2v"),
      dc_cfg<11, 11, 4, 228, 23, 1, 1, 2, 0, 0, 6>("dc11s4x32d2f6"), dc_cfg<11, 11, 4, 228, 23, 1, 1, 2, 1, 0, 6>("dc11s4x32d2vf6"),
      dc_cfg<11, 11, 4, 228, 23, 1, 1, 2, 0, 0, 8>("dc11s4x32d2f8"),
      dc_cfg<7, 7, 2, 236, 11, 2, 1, 2, 1, 0, 4>("dc7s2x64n128d2vf4"),
      dc_cfg<11, 11, 4, 228, 23, 1, 1, 3, 1>("dc11s4x32d3v"),
      dc_cfg<11, 11, 4, 228, 23, 3, 1, 2, 1>("dc11s4x96d2v"),
      // phase-split strips (conflict-free fragment reads; dword strip DMA)
      dc_cfg<11, 11, 4, 228, 23, 1, 1, 2, 0, 1>("dc11s4x32d2p"),
      dc_cfg<11, 11, 4, 228, 23, 1, 1, 3, 0, 1>("dc11s4x32d3p"),
      dc_cfg<11, 11, 4, 228, 23, 3, 1, 2, 0, 1>("dc11s4x96d2p"),
      dc_cfg<7, 7, 2, 236, 11, 2, 1, 2, 0, 1>("dc7s2x64n128d2p"),
      dc_cfg<7, 7, 2, 236, 13, 2, 2, 2, 0, 1>("dc7s2x64d2p"),
      // op_sigs' wide stems: 3 x 516^2 -> 96 11x11 s4 and 6x6 s2, 3 x 224^2 -> 96 11x11 s2
      dc_cfg<11, 11, 4, 516, 19, 1, 1, 2, 1>("dc11s4x32w516d2v"),
      dc_cfg<6, 6, 2, 516, 10, 1, 1, 3, 1>("dc6s2x32w516d3v"),
      dc_cfg<6, 6, 2, 516, 10, 3, 1, 2, 1>("dc6s2x96w516d2v"),
      dc_cfg<6, 6, 2, 516, 10, 2, 2, 2, 1>("dc6s2x64n256w516d2v"),
      dc_cfg<11, 11, 2, 228, 15, 1, 1, 2, 1>("dc11s2x32d2v"),
      dc_cfg<11, 11, 2, 228, 15, 3, 1, 2, 1>("dc11s2x96d2v"),
      // resident weights, 8 waves x 32 pixels, one OC tile per block (round 5)
      dcr_cfg<11, 11, 4, 228, 31, 1, 8, 2, 0, 3>("dc11s4r32d2"),
      dcr_cfg<11, 11, 4, 228, 31, 1, 8, 3, 0, 3>("dc11s4r32d3"),
      dcr_cfg<11, 11, 4, 228, 31, 1, 8, 2, 1, 3>("dc11s4r32d2v"),
      dcr_cfg<11, 11, 4, 228, 31, 1, 8, 3, 1, 3>("dc11s4r32d3v"),
      dcr_cfg<7, 7, 2, 236, 13, 2, 8, 2, 0, 3>("dc7s2r64d2"),
      dcr_cfg<7, 7, 2, 236, 13, 2, 8, 3, 0, 3>("dc7s2r64d3"),
      dcr_cfg<7, 7, 2, 236, 13, 2, 8, 2, 1, 3>("dc7s2r64d2v"),
      dcr_cfg<7, 7, 2, 236, 13, 2, 8, 3, 1, 3>("dc7s2r64d3v"),
      dcr_cfg<7, 7, 2, 236, 13, 1, 8, 3, 1, 3>("dc7s2r32d3v"),
      // deeper fragment prefetch (f<PF>): the stage loops wait on their LDS reads
      dcr_cfg<7, 7, 2, 236, 13, 1, 8, 3, 1, 3, 0, 6>("dc7s2r32d3vf6"), dcr_cfg<7, 7, 2, 236, 13, 1, 8, 3, 1, 3, 0, 8>("dc7s2r32d3vf8"),
      dcr_cfg<11, 11, 4, 228, 31, 1, 8, 2, 0, 3, 0, 6>("dc11s4r32d2f6"), dcr_cfg<11, 11, 4, 228, 31, 1, 8, 2, 1, 3, 0, 6>("dc11s4r32d2vf6"),
      dcr_cfg<11, 11, 4, 228, 31, 1, 8, 2, 0, 3, 0, 8>("dc11s4r32d2f8"),
      // phase-split strip (round 6): the B fragment reads of a lane half on 32 consecutive dwords
      dcr_cfg<11, 11, 4, 228, 31, 1, 8, 2, 0, 3, 0, 0, 1>("dc11s4r32d2p"), dcr_cfg<11, 11, 4, 228, 31, 1, 8, 3, 0, 3, 0, 0, 1>("dc11s4r32d3p"),
      dcr_cfg<7, 7, 2, 236, 13, 1, 8, 3, 0, 3, 0, 0, 1>("dc7s2r32d3p"), dcr_cfg<7, 7, 2, 236, 13, 2, 8, 2, 0, 3, 0, 0, 1>("dc7s2r64d2p"),
      dcr_cfg<7, 7, 2, 236, 13, 2, 8, 3, 0, 3, 0, 0, 1>("dc7s2r64d3p"),
#ifdef BH_KTRACE
      // diagnostic forms of dc7s2r32d3v / dc11s4r32d2 (wrong results by design; tools/job_dcrdiag.sh)
      dcr_cfg<7, 7, 2, 236, 13, 1, 8, 3, 1, 3, 1>("xdc7r_nodma"), dcr_cfg<7, 7, 2, 236, 13, 1, 8, 3, 1, 3, 2>("xdc7r_nomfma"),
      dcr_cfg<7, 7, 2, 236, 13, 1, 8, 3, 1, 3, 4>("xdc7r_nostore"), dcr_cfg<7, 7, 2, 236, 13, 1, 8, 3, 1, 3, 8>("xdc7r_nobar"),
      dcr_cfg<7, 7, 2, 236, 13, 1, 8, 3, 1, 3, 16>("xdc7r_nob"), dcr_cfg<7, 7, 2, 236, 13, 1, 8, 3, 1, 3, 32>("xdc7r_noa"),
      dcr_cfg<7, 7, 2, 236, 13, 1, 8, 3, 1, 3, 48>("xdc7r_nolds"), dcr_cfg<7, 7, 2, 236, 13, 1, 8, 3, 1, 3, 61>("xdc7r_onlymfma"),
      dcr_cfg<7, 7, 2, 236, 13, 1, 8, 3, 1, 3, 63>("xdc7r_none"),
      dcr_cfg<11, 11, 4, 228, 31, 1, 8, 2, 0, 3, 1>("xdc11r_nodma"), dcr_cfg<11, 11, 4, 228, 31, 1, 8, 2, 0, 3, 2>("xdc11r_nomfma"),
      dcr_cfg<11, 11, 4, 228, 31, 1, 8, 2, 0, 3, 8>("xdc11r_nobar"), dcr_cfg<11, 11, 4, 228, 31, 1, 8, 2, 0, 3, 16>("xdc11r_nob"),
      dcr_cfg<11, 11, 4, 228, 31, 1, 8, 2, 0, 3, 48>("xdc11r_nolds"), dcr_cfg<11, 11, 4, 228, 31, 1, 8, 2, 0, 3, 61>("xdc11r_onlymfma"),
#endif
      // VGG conv1_1 (3 x 224^2 -> 64, 3x3 s1 p1)
      dc_cfg<3, 3, 1, 228, 5, 2, 2, 3>("dc3s1x64d3"),
      dc_cfg<3, 3, 1, 228, 5, 1, 2, 3>("dc3s1x32d3"),
  };
}

// Launch a direct-conv configuration (p filled by launch_conv with a = packed bank): UNSUP if
// the shape is not this instantiation's (kernel, stride) or its strip would not fit.
int launch_dc(bh_ctx *ctx, const cfg_t &c, GemmArgs &p, uint32_t B, uint32_t KY, uint32_t KX, uint32_t sy,
              uint32_t sx, bool first) {
  if ((int)KY != c.dc_ky || (int)KX != c.dc_kx || (int)sy != c.dc_s || (int)sx != c.dc_s)
    return bh::fail(BH_UNSUP, std::string("conv: direct config ") + c.name + " is for another kernel / stride");
  // strip columns: input x at column x + pxa; the rightmost tap column must exist (zero past W)
  const bool v4 = c.dc_ci != 0;
  if (v4 && (p.W % 4 || p.px > 4))
    return bh::fail(BH_UNSUP, std::string("conv: 16-B strip pieces need W % 4 == 0, pad <= 4 for ") + c.name);
  const uint32_t pxa = v4 ? (p.px ? 4u : 0u) : p.px;
  const uint64_t maxcol = (uint64_t)pxa + (uint64_t)(p.OW - 1) * sx + KX - 1 - p.px;
  if (pxa + p.W > (uint32_t)c.dc_wpm || maxcol >= (uint64_t)c.dc_wpm)
    return bh::fail(BH_UNSUP, std::string("conv: input row too wide for ") + c.name);
  const uint32_t npx = (uint32_t)c.BN, OW = p.OW, OHW = p.OHW;
  const uint32_t tiles = (OHW + npx - 1) / npx;
  // input rows the worst pixel tile touches
  for (uint32_t t = 0; t < tiles; ++t) {
    const uint32_t a = t * npx, b = std::min(OHW, a + npx) - 1;
    if ((b / OW - a / OW) * sy + KY > (uint32_t)c.dc_rin)
      return bh::fail(BH_UNSUP, std::string("conv: pixel tile spans too many input rows for ") + c.name);
  }
  const uint64_t out_bytes = (uint64_t)B * p.OCOHW * 4;
  if (out_bytes >= 0x7fffff00ull) return bh::fail(BH_UNSUP, "conv: output too large for the direct kernel");
  p.c_bytes = (uint32_t)out_bytes;
  const uint32_t octiles = (p.M + c.BM - 1) / c.BM;
  const uint64_t ntile = (uint64_t)B * tiles * octiles;
  if (ntile >= (1u << 31)) return bh::fail(BH_UNSUP, "conv: too many tiles");
  if (c.dc_icmax && p.IC > (uint32_t)c.dc_icmax)
    return bh::fail(BH_UNSUP, std::string("conv: ") + c.name + " keeps at most " + std::to_string(c.dc_icmax) +
                                  " input channels' weights resident");
  // persistent grid: as many blocks as fit on the device at once (each loops over tiles); the
  // resident-weight form: a multiple of the OC tiles, so that every block keeps one OC tile
  const void *k = (const void *)c.k[A_KVEC][B_DIRECT][0];
  int bpc = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&bpc, k, c.NT, 0) != hipSuccess || bpc < 1) bpc = 1;
  const uint32_t ncu = ctx->prop.multiProcessorCount > 0 ? ctx->prop.multiProcessorCount : 256;
  uint32_t G = (uint32_t)std::min<uint64_t>(ntile, (uint64_t)ncu * std::min(bpc, 4));
  if (c.dc_icmax) G = std::max(octiles, G / octiles * octiles);
  p.total_it = (uint32_t)ntile;
  p.tiles_n = tiles;
  p.ipt = octiles;
  bh::fastdiv f = bh::make_fastdiv(tiles);
  p.tm_m = f.m;
  p.tm_s = f.s;
  f = bh::make_fastdiv(octiles);
  p.ipt_m = f.m;
  p.ipt_s = f.s;
  f = bh::make_fastdiv(OW);
  p.ow_m = f.m;
  p.ow_s = f.s;
#ifdef BH_KTRACE
  p.trace = (unsigned long long *)ctx->stamps + 65536;
#endif
  void *args[] = {&p};
  return bh::launch(ctx, k, dim3(G, 1, 1), dim3(c.NT), args, first, true, "conv_direct");
}

}  // namespace bhk
