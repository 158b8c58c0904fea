// kernarg_bench.hip -- what the kernel-argument fetch costs a small launch on gfx950 (diagnostic only,
// tools/). Per-launch time of a captured hipGraph of 200 back-to-back launches (the bench's per-op
// convention) of kernels doing one dependent load + store per block, their addresses taken from:
//   * a 256-B by-value struct (the GemmArgs shape: fetched by s_load from the kernarg segment);
//   * scalar arguments preloaded into SGPRs (-mllvm -amdgpu-kernarg-preload-count=16);
//   * an empty kernel for the floor.
//   hipcc --offload-arch=gfx950 -O3 -mllvm -amdgpu-kernarg-preload-count=16 -o tools/kernarg_bench \
//     tools/kernarg_bench.hip && tools/kernarg_bench
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e = (x);                                                          \
    if (e != hipSuccess) {                                                       \
      std::printf("%s: %s\n", #x, hipGetErrorString(e));                         \
      return 1;                                                                  \
    }                                                                            \
  } while (0)

struct Big {
  const float *a;
  float *c;
  uint32_t x[60];
};

__global__ void k_empty(float *) {}
__global__ void k_big(Big p) {
  const uint32_t i = blockIdx.x * 64 + (threadIdx.x & 63) + p.x[7];
  const float v = p.a[i];
  if (threadIdx.x < 64) p.c[i] = v * 2.0f + (float)p.x[33];
}
__global__ void k_pre(const float *a, float *c, uint32_t o7, uint32_t o33) {
  const uint32_t i = blockIdx.x * 64 + (threadIdx.x & 63) + o7;
  const float v = a[i];
  if (threadIdx.x < 64) c[i] = v * 2.0f + (float)o33;
}
// a two-step chain: the first load gives the second's offset (an indirection, e.g. a table)
__global__ void k_big2(Big p) {
  const uint32_t i = blockIdx.x * 64 + (threadIdx.x & 63) + p.x[7];
  const uint32_t j = (uint32_t)p.a[i] & 1023u;
  const float v = p.a[(1 << 20) + i + j];
  if (threadIdx.x < 64) p.c[i] = v * 2.0f + (float)p.x[33];
}
__global__ void k_pre2(const float *a, float *c, uint32_t o7, uint32_t o33) {
  const uint32_t i = blockIdx.x * 64 + (threadIdx.x & 63) + o7;
  const uint32_t j = (uint32_t)a[i] & 1023u;
  const float v = a[(1 << 20) + i + j];
  if (threadIdx.x < 64) c[i] = v * 2.0f + (float)o33;
}

template <typename F>
int run(const char *name, F launch, hipStream_t st) {
  const int reps = 200;
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
  for (int r = 0; r < reps; ++r) launch();
  CK(hipStreamEndCapture(st, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  float best = 1e9f;
  for (int t = 0; t < 6; ++t) {
    CK(hipEventRecord(a, st));
    CK(hipGraphLaunch(ge, st));
    CK(hipEventRecord(b, st));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    if (t && ms < best) best = ms;
  }
  std::printf("%-34s %.3f us per launch\n", name, best * 1e3f / reps);
  CK(hipGraphExecDestroy(ge));
  CK(hipGraphDestroy(g));
  return 0;
}

int main() {
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  float *p;
  CK(hipMalloc(&p, 64 << 20));
  CK(hipMemset(p, 0, 64 << 20));
  Big b{};
  b.a = p;
  b.c = p + (8 << 20);
  b.x[7] = 0;
  b.x[33] = 1;
  int rc = 0;
  for (int blocks : {64, 256, 1024}) {
    char n[64];
    std::snprintf(n, sizeof n, "empty (%d blocks)", blocks);
    rc |= run(n, [&] { k_empty<<<blocks, 256, 0, st>>>(p); }, st);
    std::snprintf(n, sizeof n, "struct arg, 1 load (%d)", blocks);
    rc |= run(n, [&] { k_big<<<blocks, 256, 0, st>>>(b); }, st);
    std::snprintf(n, sizeof n, "preloaded args, 1 load (%d)", blocks);
    rc |= run(n, [&] { k_pre<<<blocks, 256, 0, st>>>(p, p + (8 << 20), 0u, 1u); }, st);
    std::snprintf(n, sizeof n, "struct arg, 2 loads (%d)", blocks);
    rc |= run(n, [&] { k_big2<<<blocks, 256, 0, st>>>(b); }, st);
    std::snprintf(n, sizeof n, "preloaded args, 2 loads (%d)", blocks);
    rc |= run(n, [&] { k_pre2<<<blocks, 256, 0, st>>>(p, p + (8 << 20), 0u, 1u); }, st);
  }
  return rc;
}
