// bh_ref64.hip -- the "ref64" configuration of conv and SGEMM: every output summed in double from the
// fp32 operands and rounded once (bias added in double; a residual added to the rounded conv + bias,
// the order a separate Eltwise SUM computes; ReLU last).
//
// Boda's ops-prof compares every tune of an op element-wise against a known-good tune's full output
// (--kg-tune-tag, src/rtc_prof.cc:276-321). Two fp32 routes that sum K in different orders differ by
// about the error each has against the exact sum -- up to ~1.2e-3 of min_sig_mag_rel_diff at K ~ 2300
// on gen_data mode 5 (profiles/r05/route_acc_3x3.txt) -- so a kg tune that is itself an fp32 route
// spends half of a compare's tolerance on its own error. ref64 is the known-good tune for such sweeps
// (boda_hip_ops_prof --op-tunes='(kg=(cfg=ref64),...)'): one thread per output, double accumulation,
// the reference layouts read directly (no pack), plain loads. Not a fast path (the tuner never routes
// it); correctness only, and it is held to the double oracle in tests/test_gpu_ref64.py.
#include "bh_gemm_dev.h"

namespace bhk {
namespace {

__global__ __launch_bounds__(256) void ref64_conv_kernel(GemmArgs p, uint32_t B, uint32_t KY) {
  const uint64_t n = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  const uint64_t total = (uint64_t)B * p.M * p.OHW;
  if (n >= total) return;
  const uint32_t ox = (uint32_t)(n % p.OW), oy = (uint32_t)((n / p.OW) % (p.OHW / p.OW));
  const uint32_t oc = (uint32_t)((n / p.OHW) % p.M), img = (uint32_t)(n / ((uint64_t)p.OHW * p.M));
  const float *in = p.b + (uint64_t)img * p.ICHW;
  const float *w = p.a + (uint64_t)oc * p.K;
  double acc = 0.0;
  for (uint32_t ic = 0; ic < p.IC; ++ic)
    for (uint32_t ky = 0; ky < KY; ++ky) {
      const int iy = (int)(oy * p.sy + ky) - (int)p.py;
      if (iy < 0 || iy >= (int)p.H) continue;
      for (uint32_t kx = 0; kx < p.KX; ++kx) {
        const int ix = (int)(ox * p.sx + kx) - (int)p.px;
        if (ix < 0 || ix >= (int)p.W) continue;
        acc += (double)in[(uint64_t)ic * p.HW + (uint32_t)iy * p.W + (uint32_t)ix] *
               (double)w[(ic * KY + ky) * p.KX + kx];
      }
    }
  if (p.bias) acc += (double)p.bias[oc];
  const uint64_t o = (uint64_t)img * p.OCOHW + (uint64_t)oc * p.OHW + (uint64_t)oy * p.OW + ox;
  float y = (float)acc;
  if (p.res) y += p.res[o];
  p.c[o] = (p.relu && y < 0.0f) ? 0.0f : y;
}

__global__ __launch_bounds__(256) void ref64_sgemm_kernel(GemmArgs p) {
  const uint64_t n = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  if (n >= (uint64_t)p.M * p.N) return;
  const uint32_t m = (uint32_t)(n / p.N), c = (uint32_t)(n % p.N);
  double acc = 0.0;
  for (uint32_t k = 0; k < p.K; ++k) acc += (double)p.a[(uint64_t)k * p.lda + m] * (double)p.b[(uint64_t)k * p.ldb + c];
  p.c[n] = (float)acc;
}

}  // namespace

std::vector<cfg_t> ref64_cfgs() {
  cfg_t c{"ref64", 1, 1, 1, 256, {}, 0};
  c.ref64 = 1;
  return {c};
}

int launch_ref64_conv(bh_ctx *ctx, GemmArgs &p, uint32_t B, uint32_t KY, bool first) {
  const uint64_t total = (uint64_t)B * p.M * p.OHW;
  if ((total + 255) / 256 >= (1u << 31)) return bh::fail(BH_UNSUP, "conv: too many outputs for ref64");
  void *args[] = {&p, &B, &KY};
  return bh::launch(ctx, (const void *)ref64_conv_kernel, dim3((uint32_t)((total + 255) / 256)), dim3(256), args, first,
                    true, "conv_ref64");
}

int launch_ref64_sgemm(bh_ctx *ctx, GemmArgs &p) {
  const uint64_t total = (uint64_t)p.M * p.N;
  if ((total + 255) / 256 >= (1u << 31)) return bh::fail(BH_UNSUP, "sgemm: too many outputs for ref64");
  void *args[] = {&p};
  return bh::launch(ctx, (const void *)ref64_sgemm_kernel, dim3((uint32_t)((total + 255) / 256)), dim3(256), args, true,
                    true, "sgemm_ref64");
}

}  // namespace bhk
