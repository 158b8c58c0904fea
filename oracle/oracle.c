/*
 * oracle.c -- CPU restatement of Boda's per-op Convolution / SGEMM semantics.
 *
 * *** TEST INFRASTRUCTURE ONLY. ***
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * this library, and only as the checker (or as the timed CPU baseline). The
 * product path (boda-1_amd/) never links, loads or calls anything in oracle/.
 *
 * Parity pinning: every function below is checked in tests/test_oracle_golden.py
 * against the known-good digests the reference itself ships in
 * /root/reference/test/good_tr/{sgemm-gen600,sgemm-gen5,conv-gen5,conv-debug,
 * conv-full-gen5,ops-prof-conv-3x3-cudnn-boda}/wisdom.wis, decoded into
 * the JSON fixtures in tests/golden/ by tests/golden/make_golden.py.
 *
 * Reference anchors (paths relative to the reference root):
 *   det_hash_rand ............ test/rtc/gen-util.h:1-9
 *   gen_data sgemm a / b ..... test/rtc/gen_data_sgemm_a.cucl:7-19, gen_data_sgemm_b.cucl:8-20
 *   gen_data conv in/filts/biases  test/rtc/gen_data_Convolution_{in,filts,biases}.cucl
 *   conv math ................ test/rtc/conv.cucl:25-44 (cross-correlation, zero pad),
 *                              src/cnn_codegen.cc:35-42 (bias + ReLU), src/cnn_op.cc:337 (ReLU always on)
 *   output size .............. src/conv_util.cc:167-173
 *   sgemm math ............... test/rtc/sgemm.cucl:1-3 (c[M][N] = sum_K a[K][M] b[K][N])
 *   digest ................... src/boda_base.cc:214-276 (strides, mt19937, uniform_int, strided sums)
 *   tolerance metric ......... src/boda_base.cc:140-153 (min_sig_mag_rel_diff), :284-310 (mrd_comp)
 *
 * Two compute flavours:
 *   orc_*_ref  : double accumulation (the correctness oracle),
 *   orc_*_fast : plain fp32, OpenMP, cache-blocked (the timed CPU baseline, "kind": "port").
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>
#include <omp.h>

#define ORC_API __attribute__((visibility("default")))

/* ------------------------------------------------------------------------- */
/* gen_data                                                                   */
/* ------------------------------------------------------------------------- */

/* murmur3 fmix32 -> [-5,5). gen-util.h:1-9. The reference JIT compiles with fmad
 * contraction on (nvrtc --use_fast_math), so the final a*b-c is one fused op. */
ORC_API float orc_det_hash_rand(uint32_t rv) {
  uint32_t h = rv;
  h ^= h >> 16;
  h *= 0x85ebca6bu;
  h ^= h >> 13;
  h *= 0xc2b2ae35u;
  h ^= h >> 16;
  return fmaf((float)h, 10.0f / 4294967296.0f, -5.0f);
}

enum { ORC_SEED_SGEMM = 12738732u, ORC_SEED_IN = 234234567u,
       ORC_SEED_FILTS = 8753985u, ORC_SEED_BIASES = 39475612u };

/* a is K x M (M innermost). gen_data_sgemm_a.cucl:7-19: modes >= 100 collapse to mode/100. */
ORC_API void orc_gen_sgemm_a(float *a, uint32_t K, uint32_t M, uint32_t mode, float vi) {
  uint32_t fin = mode >= 100 ? mode / 100 : mode;
  uint64_t n = (uint64_t)K * M;
#pragma omp parallel for schedule(static)
  for (uint64_t i = 0; i < n; ++i) {
    uint32_t m = (uint32_t)(i % M), k = (uint32_t)(i / M);
    float v = vi;
    if (fin == 2) v += (float)m;
    if (fin == 3) v += (float)k;
    else if (fin == 4) { if (m == M / 2 && k == K / 2) v += 1.0f; }
    else if (fin == 5) v += orc_det_hash_rand((uint32_t)i + ORC_SEED_SGEMM);
    else if (fin == 6) v += (float)(m * 1000u + k);
    a[i] = v;
  }
}

/* b is K x N (N innermost). gen_data_sgemm_b.cucl:8-20: mode >= 100 is the identity KAT. */
ORC_API void orc_gen_sgemm_b(float *b, uint32_t K, uint32_t N, uint32_t mode, float vi) {
  uint64_t n = (uint64_t)K * N;
#pragma omp parallel for schedule(static)
  for (uint64_t i = 0; i < n; ++i) {
    uint32_t nn = (uint32_t)(i % N), k = (uint32_t)(i / N);
    float v = vi;
    if (mode == 2) v += (float)nn;
    if (mode == 3) v += (float)k;
    else if (mode == 4) { if (nn == N / 2 && k == K / 2) v += 1.0f; }
    else if (mode == 5) v += orc_det_hash_rand((uint32_t)i + ORC_SEED_SGEMM);
    else if (mode >= 100) { if (nn == k) v += 1.0f; }
    b[i] = v;
  }
}

/* 4-D img:chan:y:x (in) or out_chan:in_chan:y:x (filts); modes from
 * gen_data_Convolution_{in,filts}.cucl. which: 0 = in, 1 = filts. */
ORC_API void orc_gen_conv4(float *p, uint32_t d0, uint32_t d1, uint32_t Y, uint32_t X,
                           int which, uint32_t mode, float vi) {
  uint64_t n = (uint64_t)d0 * d1 * Y * X;
  uint32_t seed = which ? ORC_SEED_FILTS : ORC_SEED_IN;
#pragma omp parallel for schedule(static)
  for (uint64_t i = 0; i < n; ++i) {
    uint32_t x = (uint32_t)(i % X), y = (uint32_t)((i / X) % Y);
    float v = vi;
    if (mode == 2) v += (float)x;
    if (mode == 3) v += (float)y;
    else if (mode == 4) { if (x == X / 2 && y == Y / 2) v += 1.0f; }
    else if (mode == 5) v += orc_det_hash_rand((uint32_t)i + seed);
    p[i] = v;
  }
}

ORC_API void orc_gen_conv_biases(float *p, uint32_t OC, uint32_t mode, float vi) {
  for (uint32_t i = 0; i < OC; ++i) {
    float v = vi;
    if (mode == 5) v += orc_det_hash_rand(i + ORC_SEED_BIASES);
    p[i] = v;
  }
}

/* ------------------------------------------------------------------------- */
/* shapes                                                                     */
/* ------------------------------------------------------------------------- */

/* conv_util.cc:167-173: floor((in + 2 pad - k) / stride) + 1, or 0 if the padded input is too small. */
ORC_API uint32_t orc_conv_out_sz(uint32_t in, uint32_t pad, uint32_t k, uint32_t stride) {
  uint32_t p = in + 2 * pad;
  if (p < k) return 0;
  return (p - k) / stride + 1;
}

/* ------------------------------------------------------------------------- */
/* correctness references (double accumulation)                              */
/* ------------------------------------------------------------------------- */

/* c[m][n] = sum_k a[k][m] * b[k][n]; a K x M, b K x N, c M x N. sgemm.cucl:1-3. */
ORC_API void orc_sgemm_ref(const float *a, const float *b, float *c, uint32_t M, uint32_t N, uint32_t K) {
#pragma omp parallel
  {
    double *acc = (double *)malloc(sizeof(double) * 4 * (size_t)N);
#pragma omp for schedule(dynamic, 1)
    for (uint32_t m0 = 0; m0 < M; m0 += 4) {
      uint32_t mr = M - m0 < 4 ? M - m0 : 4;
      memset(acc, 0, sizeof(double) * 4 * (size_t)N);
      for (uint32_t k = 0; k < K; ++k) {
        const float *bk = b + (size_t)k * N;
        for (uint32_t r = 0; r < mr; ++r) {
          double av = a[(size_t)k * M + m0 + r];
          double *ar = acc + (size_t)r * N;
          for (uint32_t n = 0; n < N; ++n) ar[n] += av * (double)bk[n];
        }
      }
      for (uint32_t r = 0; r < mr; ++r)
        for (uint32_t n = 0; n < N; ++n) c[(size_t)(m0 + r) * N + n] = (float)acc[(size_t)r * N + n];
    }
    free(acc);
  }
}

/* out[b][oc][oy][ox] = act(bias[oc] + sum_{ic,ky,kx} in[b][ic][oy*sy+ky-py][ox*sx+kx-px] * f[oc][ic][ky][kx]),
 * zero padding outside the input; act = ReLU when relu != 0. conv.cucl:25-44, cnn_codegen.cc:35-42. */
ORC_API void orc_conv_ref(const float *in, const float *filts, const float *biases, float *out,
                          uint32_t B, uint32_t IC, uint32_t H, uint32_t W, uint32_t OC,
                          uint32_t KY, uint32_t KX, uint32_t sy, uint32_t sx, uint32_t py, uint32_t px,
                          int relu) {
  uint32_t OH = orc_conv_out_sz(H, py, KY, sy), OW = orc_conv_out_sz(W, px, KX, sx);
  size_t plane = (size_t)OH * OW;
#pragma omp parallel
  {
    double *acc = (double *)malloc(sizeof(double) * (plane ? plane : 1));
#pragma omp for collapse(2) schedule(dynamic, 1)
    for (uint32_t b = 0; b < B; ++b)
      for (uint32_t oc = 0; oc < OC; ++oc) {
        double bias = biases ? (double)biases[oc] : 0.0;
        for (size_t i = 0; i < plane; ++i) acc[i] = bias;
        for (uint32_t ic = 0; ic < IC; ++ic) {
          const float *ip = in + ((size_t)b * IC + ic) * H * W;
          for (uint32_t ky = 0; ky < KY; ++ky)
            for (uint32_t kx = 0; kx < KX; ++kx) {
              double w = filts[(((size_t)oc * IC + ic) * KY + ky) * KX + kx];
              for (uint32_t oy = 0; oy < OH; ++oy) {
                int64_t iy = (int64_t)oy * sy + ky - py;
                if (iy < 0 || iy >= (int64_t)H) continue;
                const float *row = ip + (size_t)iy * W;
                double *ar = acc + (size_t)oy * OW;
                /* ox range where ix = ox*sx + kx - px is inside [0, W) */
                int64_t lo = (int64_t)px - (int64_t)kx;
                uint32_t ox0 = lo <= 0 ? 0 : (uint32_t)((lo + sx - 1) / sx);
                int64_t hi = (int64_t)W - 1 + px - kx; /* ox*sx <= hi */
                if (hi < 0) continue;
                uint32_t ox1 = (uint32_t)(hi / sx) + 1;
                if (ox1 > OW) ox1 = OW;
                for (uint32_t ox = ox0; ox < ox1; ++ox) ar[ox] += w * (double)row[(size_t)ox * sx + kx - px];
              }
            }
        }
        float *op = out + ((size_t)b * OC + oc) * plane;
        for (size_t i = 0; i < plane; ++i) {
          float v = (float)acc[i];
          op[i] = (relu && v < 0.0f) ? 0.0f : v;
        }
      }
    free(acc);
  }
}

/* The same sum for selected outputs only (flat NCHW output indices idx[0..n-1]), for shapes
 * too large for a full double-accumulated reference in a test's time budget. */
ORC_API void orc_conv_ref_at(const float *in, const float *filts, const float *biases, const uint64_t *idx,
                             uint64_t n, float *vals, uint32_t B, uint32_t IC, uint32_t H, uint32_t W,
                             uint32_t OC, uint32_t KY, uint32_t KX, uint32_t sy, uint32_t sx, uint32_t py,
                             uint32_t px, int relu) {
  uint32_t OH = orc_conv_out_sz(H, py, KY, sy), OW = orc_conv_out_sz(W, px, KX, sx);
#pragma omp parallel for schedule(dynamic, 64)
  for (uint64_t i = 0; i < n; ++i) {
    uint64_t e = idx[i];
    uint32_t ox = (uint32_t)(e % OW), oy = (uint32_t)((e / OW) % OH);
    uint32_t oc = (uint32_t)((e / ((uint64_t)OW * OH)) % OC), b = (uint32_t)(e / ((uint64_t)OW * OH * OC));
    double acc = biases ? (double)biases[oc] : 0.0;
    for (uint32_t ic = 0; ic < IC; ++ic)
      for (uint32_t ky = 0; ky < KY; ++ky) {
        int64_t iy = (int64_t)oy * sy + ky - py;
        if (iy < 0 || iy >= (int64_t)H) continue;
        for (uint32_t kx = 0; kx < KX; ++kx) {
          int64_t ix = (int64_t)ox * sx + kx - px;
          if (ix < 0 || ix >= (int64_t)W) continue;
          acc += (double)in[(((size_t)b * IC + ic) * H + iy) * W + ix] *
                 (double)filts[(((size_t)oc * IC + ic) * KY + ky) * KX + kx];
        }
      }
    float v = (float)acc;
    vals[i] = (relu && v < 0.0f) ? 0.0f : v;
  }
}

/* ------------------------------------------------------------------------- */
/* CPU baseline (fp32, OpenMP, blocked) -- timed by bench.py's cpu_baseline   */
/* ------------------------------------------------------------------------- */

ORC_API int orc_num_threads(void) { return omp_get_max_threads(); }
ORC_API void orc_set_num_threads(int n) { omp_set_num_threads(n); }

/* fp32 SGEMM: 64-row x 256-col output blocks held in L1/L2, k-blocked by 256. */
ORC_API void orc_sgemm_fast(const float *a, const float *b, float *c, uint32_t M, uint32_t N, uint32_t K) {
  const uint32_t MB = 32, NB = 512, KB = 256;
  uint32_t nmb = (M + MB - 1) / MB, nnb = (N + NB - 1) / NB;
#pragma omp parallel for collapse(2) schedule(dynamic, 1)
  for (uint32_t ib = 0; ib < nmb; ++ib)
    for (uint32_t jb = 0; jb < nnb; ++jb) {
      float acc[32 * 512] __attribute__((aligned(64)));
      uint32_t m0 = ib * MB, n0 = jb * NB;
      uint32_t mr = M - m0 < MB ? M - m0 : MB, nr = N - n0 < NB ? N - n0 : NB;
      memset(acc, 0, sizeof(acc));
      for (uint32_t k0 = 0; k0 < K; k0 += KB) {
        uint32_t k1 = k0 + KB < K ? k0 + KB : K;
        for (uint32_t r = 0; r < mr; ++r) {
          float *ar = acc + r * NB;
          for (uint32_t k = k0; k < k1; ++k) {
            float av = a[(size_t)k * M + m0 + r];
            const float *bk = b + (size_t)k * N + n0;
            for (uint32_t n = 0; n < nr; ++n) ar[n] += av * bk[n];
          }
        }
      }
      for (uint32_t r = 0; r < mr; ++r) memcpy(c + (size_t)(m0 + r) * N + n0, acc + r * NB, nr * sizeof(float));
    }
}

/* fp32 direct conv with 4 output channels per task sharing the input reads. */
ORC_API void orc_conv_fast(const float *in, const float *filts, const float *biases, float *out,
                           uint32_t B, uint32_t IC, uint32_t H, uint32_t W, uint32_t OC,
                           uint32_t KY, uint32_t KX, uint32_t sy, uint32_t sx, uint32_t py, uint32_t px,
                           int relu) {
  uint32_t OH = orc_conv_out_sz(H, py, KY, sy), OW = orc_conv_out_sz(W, px, KX, sx);
  size_t plane = (size_t)OH * OW;
  const uint32_t OCB = 4;
  uint32_t nocb = (OC + OCB - 1) / OCB;
#pragma omp parallel
  {
    float *acc = (float *)malloc(sizeof(float) * OCB * (plane ? plane : 1));
#pragma omp for collapse(2) schedule(dynamic, 1)
    for (uint32_t b = 0; b < B; ++b)
      for (uint32_t cb = 0; cb < nocb; ++cb) {
        uint32_t oc0 = cb * OCB, ocr = OC - oc0 < OCB ? OC - oc0 : OCB;
        for (uint32_t t = 0; t < ocr; ++t)
          for (size_t i = 0; i < plane; ++i) acc[t * plane + i] = biases ? biases[oc0 + t] : 0.0f;
        for (uint32_t ic = 0; ic < IC; ++ic) {
          const float *ip = in + ((size_t)b * IC + ic) * H * W;
          for (uint32_t ky = 0; ky < KY; ++ky)
            for (uint32_t kx = 0; kx < KX; ++kx) {
              float w[4] = {0, 0, 0, 0};
              for (uint32_t t = 0; t < ocr; ++t) w[t] = filts[((((size_t)oc0 + t) * IC + ic) * KY + ky) * KX + kx];
              int64_t lo = (int64_t)px - (int64_t)kx;
              uint32_t ox0 = lo <= 0 ? 0 : (uint32_t)((lo + sx - 1) / sx);
              int64_t hi = (int64_t)W - 1 + px - kx;
              if (hi < 0) continue;
              uint32_t ox1 = (uint32_t)(hi / sx) + 1;
              if (ox1 > OW) ox1 = OW;
              for (uint32_t oy = 0; oy < OH; ++oy) {
                int64_t iy = (int64_t)oy * sy + ky - py;
                if (iy < 0 || iy >= (int64_t)H) continue;
                const float *row = ip + (size_t)iy * W + kx - px;
                float *a0 = acc + (size_t)oy * OW, *a1 = a0 + plane, *a2 = a1 + plane, *a3 = a2 + plane;
                if (ocr == 4) {
                  for (uint32_t ox = ox0; ox < ox1; ++ox) {
                    float v = row[(size_t)ox * sx];
                    a0[ox] += w[0] * v; a1[ox] += w[1] * v; a2[ox] += w[2] * v; a3[ox] += w[3] * v;
                  }
                } else {
                  for (uint32_t t = 0; t < ocr; ++t) {
                    float *at = a0 + t * plane;
                    for (uint32_t ox = ox0; ox < ox1; ++ox) at[ox] += w[t] * row[(size_t)ox * sx];
                  }
                }
              }
            }
        }
        for (uint32_t t = 0; t < ocr; ++t) {
          float *op = out + ((size_t)b * OC + oc0 + t) * plane;
          for (size_t i = 0; i < plane; ++i) {
            float v = acc[t * plane + i];
            op[i] = (relu && v < 0.0f) ? 0.0f : v;
          }
        }
      }
    free(acc);
  }
}

/* ------------------------------------------------------------------------- */
/* nda digest (boda_base.cc:214-276)                                          */
/* ------------------------------------------------------------------------- */

typedef struct { uint32_t mt[624]; int idx; } orc_mt19937;

static void mt_seed(orc_mt19937 *g, uint32_t s) {
  g->mt[0] = s;
  for (int i = 1; i < 624; ++i) g->mt[i] = 1812433253u * (g->mt[i - 1] ^ (g->mt[i - 1] >> 30)) + (uint32_t)i;
  g->idx = 624;
}

static uint32_t mt_next(orc_mt19937 *g) {
  if (g->idx >= 624) {
    for (int i = 0; i < 624; ++i) {
      uint32_t y = (g->mt[i] & 0x80000000u) | (g->mt[(i + 1) % 624] & 0x7fffffffu);
      g->mt[i] = g->mt[(i + 397) % 624] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
    }
    g->idx = 0;
  }
  uint32_t y = g->mt[g->idx++];
  y ^= y >> 11;
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= y >> 18;
  return y;
}

/* boost::random::uniform_int_distribution<uint64_t>(0, range) over a 32-bit engine whose
 * range is 0xFFFFFFFF (the 'brange > range' bucket branch). range == 0 draws nothing. */
static uint64_t boost_uniform(orc_mt19937 *g, uint64_t range) {
  if (range == 0) return 0;
  uint32_t brange = 0xFFFFFFFFu, r = (uint32_t)range;
  uint32_t bucket = brange / (r + 1u);
  if (brange % (r + 1u) == r) ++bucket;
  for (;;) {
    uint32_t res = mt_next(g) / bucket;
    if (res <= r) return res;
  }
}

static int cmp_u64(const void *x, const void *y) {
  uint64_t a = *(const uint64_t *)x, b = *(const uint64_t *)y;
  return a < b ? -1 : a > b;
}

static uint32_t floor_log2_u64(uint64_t v) { uint32_t r = 0; while (v >>= 1) ++r; return r; }

/* Sample plan: (stride, offset, num_subsamps) triples, in the reference's order.
 * Returns the count; writes at most max_out triples into sis (3 u64 each). */
ORC_API int orc_digest_plan(uint64_t n, const uint64_t *dim_strides, int nd, uint64_t seed,
                            uint64_t *sis, int max_out) {
  static const uint64_t primes[11] = {1, 2, 3, 5, 7, 11, 13, 17, 19, 23, 29};
  uint64_t st[64];
  int ns = 0;
  for (int i = 0; i < 11; ++i) if (primes[i] <= n) st[ns++] = primes[i];
  for (int i = 0; i < nd && ns < 62; ++i) st[ns++] = dim_strides[i];
  st[ns++] = n;
  qsort(st, ns, sizeof(uint64_t), cmp_u64);
  orc_mt19937 g;
  mt_seed(&g, (uint32_t)seed);
  int cnt = 0;
  uint64_t prev = 0;
  for (int i = 0; i < ns; ++i) {
    if (i && st[i] == prev) continue; /* std::set semantics */
    prev = st[i];
    uint64_t stride = st[i];
    uint32_t no = floor_log2_u64(stride + 1);
    uint64_t seen[64];
    int nseen = 0;
    for (uint32_t j = 0; j < no; ++j) {
      uint64_t off = boost_uniform(&g, stride - 1);
      int dup = 0;
      for (int q = 0; q < nseen; ++q) if (seen[q] == off) { dup = 1; break; }
      if (dup) continue;
      seen[nseen++] = off;
      if (cnt < max_out) {
        sis[3 * cnt + 0] = stride;
        sis[3 * cnt + 1] = off;
        sis[3 * cnt + 2] = (n - off) / stride;
      }
      ++cnt;
    }
  }
  return cnt;
}

/* Full digest: min, max, and one sequential fp32 strided sum per planned sample. */
ORC_API int orc_digest(const float *v, uint64_t n, const uint64_t *dim_strides, int nd, uint64_t seed,
                       float *minv, float *maxv, float *samps, int max_out) {
  float mn = INFINITY, mx = -INFINITY;
  for (uint64_t i = 0; i < n; ++i) { if (v[i] < mn) mn = v[i]; if (v[i] > mx) mx = v[i]; }
  *minv = mn;
  *maxv = mx;
  uint64_t *sis = (uint64_t *)malloc(sizeof(uint64_t) * 3 * (size_t)max_out);
  int cnt = orc_digest_plan(n, dim_strides, nd, seed, sis, max_out);
  int m = cnt < max_out ? cnt : max_out;
#pragma omp parallel for schedule(dynamic, 1)
  for (int s = 0; s < m; ++s) {
    float sv = 0.0f;
    for (uint64_t i = sis[3 * s + 1]; i < n; i += sis[3 * s]) sv += v[i];
    samps[s] = sv;
  }
  free(sis);
  return cnt;
}

/* boda_base.cc:140-153 */
ORC_API double orc_min_sig_mag_rel_diff(double min_sig_mag, double v1, double v2) {
  double a1 = fabs(v1), a2 = fabs(v2);
  double amax = a1 > a2 ? a1 : a2;
  if (amax < min_sig_mag) amax = min_sig_mag;
  return fabs(v2 - v1) / amax;
}

/* boda_base.cc:284-310 (mrd_comp): returns the number of failing entries (min, max, samples);
 * worst[0] receives the largest rd / allowed-mrd ratio seen. */
ORC_API int orc_digest_compare(const float *kg_samps, float kg_min, float kg_max,
                               const float *samps, float mn, float mx,
                               const uint64_t *sis, int cnt, double mrd, double *worst) {
  int fails = 0;
  double w = 0.0, rd;
  rd = orc_min_sig_mag_rel_diff(1.0, kg_min, mn);
  if (rd > mrd) ++fails;
  if (rd / mrd > w) w = rd / mrd;
  rd = orc_min_sig_mag_rel_diff(1.0, kg_max, mx);
  if (rd > mrd) ++fails;
  if (rd / mrd > w) w = rd / mrd;
  for (int i = 0; i < cnt; ++i) {
    double adj = mrd;
    if (sis[3 * i + 2] > 1000) adj *= sqrt((double)sis[3 * i + 2] / 1000.0);
    rd = orc_min_sig_mag_rel_diff(1.0, kg_samps[i], samps[i]);
    if (rd > adj) ++fails;
    if (rd / adj > w) w = rd / adj;
  }
  if (worst) *worst = w;
  return fails;
}
