// probe_launch.hip -- how much of a short op's measured time is the launch/timing
// machinery rather than the kernel. Standalone; run it under
// `rocprofv3 --kernel-trace --stats` to compare the profiler's view.
//   hipcc --offload-arch=gfx950 -O2 -o build/probe_launch tools/probe_launch.hip
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(2);                                                                      \
    }                                                                               \
  } while (0)

__global__ void k_empty() {}
__global__ void k_store(float *p) {
  if (threadIdx.x < 4) p[threadIdx.x] = 1.0f;
}
// busy-wait ~us microseconds on the 100 MHz constant clock (bounded: always exits)
__global__ void k_spin(unsigned us) {
  unsigned long long t0 = wall_clock64();
  while (wall_clock64() - t0 < (unsigned long long)us * 100ull) __builtin_amdgcn_s_sleep(8);
}

static float med(std::vector<float> v) {
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

int main(int argc, char **argv) {
  const int R = argc > 1 ? atoi(argv[1]) : 200;
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  float *d;
  CK(hipMalloc(&d, 1 << 20));
  hipEvent_t t0, t1;
  CK(hipEventCreate(&t0));
  CK(hipEventCreate(&t1));
  std::vector<hipEvent_t> eb(R), ee(R);
  for (int i = 0; i < R; ++i) {
    CK(hipEventCreate(&eb[i]));
    CK(hipEventCreate(&ee[i]));
  }
  void *noargs[] = {nullptr};
  void *stargs[] = {&d};
  float ms;
  // warm up
  for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(k_empty, 1, 64, 0, s);
  CK(hipStreamSynchronize(s));

  auto throughput = [&](const char *name, auto body) {
    unsigned spin = 3000;
    hipLaunchKernelGGL(k_spin, 1, 64, 0, s, spin);  // queue fills while this runs
    CK(hipEventRecord(t0, s));
    for (int i = 0; i < R; ++i) body(i);
    CK(hipEventRecord(t1, s));
    CK(hipStreamSynchronize(s));
    CK(hipEventElapsedTime(&ms, t0, t1));
    printf("%-52s %8.3f us per call (back-to-back, %d calls)\n", name, ms * 1e3f / R, R);
  };
  throughput("E1 empty kernel, hipLaunchKernel", [&](int) { CK(hipLaunchKernel((void *)k_empty, 1, 64, noargs, 0, s)); });
  throughput("E3 4-float store kernel, hipLaunchKernel", [&](int) { CK(hipLaunchKernel((void *)k_store, 1, 64, stargs, 0, s)); });
  throughput("E2 empty kernel, hipExtLaunchKernel + events", [&](int i) {
    CK(hipExtLaunchKernel((void *)k_empty, 1, 64, noargs, 0, s, eb[i], ee[i], 0));
  });
  {
    std::vector<float> v(R);
    for (int i = 0; i < R; ++i) CK(hipEventElapsedTime(&v[i], eb[i], ee[i]));
    printf("%-52s %8.3f us median per-call event duration\n", "   E2 per-call", med(v) * 1e3f);
  }
  throughput("E4 empty kernel between hipEventRecord pairs", [&](int i) {
    CK(hipEventRecord(eb[i], s));
    CK(hipLaunchKernel((void *)k_empty, 1, 64, noargs, 0, s));
    CK(hipEventRecord(ee[i], s));
  });
  {
    std::vector<float> v(R);
    for (int i = 0; i < R; ++i) CK(hipEventElapsedTime(&v[i], eb[i], ee[i]));
    printf("%-52s %8.3f us median per-call event duration\n", "   E4 per-call", med(v) * 1e3f);
  }
  // graph of R empty kernels
  {
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    for (int i = 0; i < R; ++i) CK(hipLaunchKernel((void *)k_empty, 1, 64, noargs, 0, s));
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CK(hipGraphLaunch(ge, s));
    CK(hipStreamSynchronize(s));
    hipLaunchKernelGGL(k_spin, 1, 64, 0, s, 2000u);
    CK(hipEventRecord(t0, s));
    CK(hipGraphLaunch(ge, s));
    CK(hipEventRecord(t1, s));
    CK(hipStreamSynchronize(s));
    CK(hipEventElapsedTime(&ms, t0, t1));
    printf("%-52s %8.3f us per call\n", "E6 graph of empty kernels", ms * 1e3f / R);
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
  }
  CK(hipStreamSynchronize(s));
  printf("done\n");
  return 0;
}
