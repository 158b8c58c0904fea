// floor_bench.hip -- per-launch floor of a captured hipGraph of back-to-back kernels on one
// stream (the bench's per-op convention): empty kernel, one dependent load + store per block,
// and a 1-MB read + 64-KB write, at 256 / 1024 blocks. Diagnostic only (tools/).
//   hipcc --offload-arch=gfx950 -O3 -o tools/floor_bench tools/floor_bench.hip && tools/floor_bench
#include <hip/hip_runtime.h>
#include <cstdio>

#define CK(x)                                                                           \
  do {                                                                                  \
    hipError_t e = (x);                                                                 \
    if (e != hipSuccess) {                                                              \
      std::printf("%s: %s\n", #x, hipGetErrorString(e));                                \
      return 1;                                                                         \
    }                                                                                   \
  } while (0)

__global__ void k_empty(float *) {}
__global__ void k_ldst(float *p) {
  if (threadIdx.x == 0) p[4096 + blockIdx.x] = p[blockIdx.x] + 1.0f;
}
__global__ void k_stream(float *p) {  // each block reads 1 KB (float4 per thread), writes 64 B
  const float4 v = ((const float4 *)p)[blockIdx.x * 64 + (threadIdx.x & 63)];
  float s = v.x + v.y + v.z + v.w;
  for (int o = 32; o; o >>= 1) s += __shfl_xor(s, o);
  if ((threadIdx.x & 63) < 16) p[(1 << 22) + blockIdx.x * 16 + (threadIdx.x & 15)] = s;
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
  for (int t = 0; t < 5; ++t) {
    CK(hipEventRecord(a, st));
    CK(hipGraphLaunch(ge, st));
    CK(hipEventRecord(b, st));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    if (t && ms < best) best = ms;
  }
  std::printf("%-28s %.3f us per launch\n", name, best * 1e3f / reps);
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
  for (int blocks : {1, 256, 1024}) {
    char n[64];
    std::snprintf(n, sizeof n, "empty %d x 256", blocks);
    if (run(n, [&] { k_empty<<<blocks, 256, 0, st>>>(p); }, st)) return 1;
    std::snprintf(n, sizeof n, "load+store %d x 256", blocks);
    if (run(n, [&] { k_ldst<<<blocks, 256, 0, st>>>(p); }, st)) return 1;
    std::snprintf(n, sizeof n, "stream 1KB/blk %d x 256", blocks);
    if (run(n, [&] { k_stream<<<blocks, 256, 0, st>>>(p); }, st)) return 1;
  }
  return 0;
}
