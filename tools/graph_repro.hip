// graph_repro.hip -- minimal hipGraph replay, for the rocprofv3 kernel-trace crash inside
// hipGraphLaunch (tools/job_final.sh, step profgraph): one trivial kernel captured from a non-blocking
// stream and replayed, nothing of libboda_hip. Diagnostic only.
//   hipcc --offload-arch=gfx950 -O2 -o tools/graph_repro tools/graph_repro.hip
//   rocprofv3 --kernel-trace --stats -d out -o t -- tools/graph_repro [nodes] [big-args 0/1] [cycles] [replays]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                             \
  do {                                                                    \
    hipError_t e = (x);                                                   \
    if (e != hipSuccess) {                                                \
      std::printf("%s: %s\n", #x, hipGetErrorString(e));                  \
      return 1;                                                           \
    }                                                                     \
  } while (0)

__global__ void add_one(float *p, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] += 1.0f;
}
// a by-value argument block the size of libboda_hip's GemmArgs (~300 B)
struct big_args {
  float *p;
  int n;
  unsigned pad[72];
};
__global__ void add_one_big(big_args a) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < a.n) a.p[i] += 1.0f + (float)a.pad[71];
}

int main(int argc, char **argv) {
  const int nodes = argc > 1 ? std::atoi(argv[1]) : 1;
  const int big = argc > 2 ? std::atoi(argv[2]) : 0;  // 1: the ~300-B argument kernel
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  float *p;
  CK(hipMalloc(&p, 1 << 20));
  CK(hipMemset(p, 0, 1 << 20));
  const int cycles = argc > 3 ? std::atoi(argv[3]) : 1;  // capture / replay / destroy cycles
  const int replays = argc > 4 ? std::atoi(argv[4]) : (cycles > 1 ? 2 : 3);  // replays per cycle
  big_args ba{};
  ba.p = p;
  ba.n = 1 << 18;
  int launched = 0;
  for (int cyc = 0; cyc < cycles; ++cyc) {
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
    for (int i = 0; i < nodes; ++i) {
      if (big) add_one_big<<<256, 256, 0, st>>>(ba);
      else add_one<<<256, 256, 0, st>>>(p, 1 << 18);
    }
    CK(hipStreamEndCapture(st, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CK(hipGraphDestroy(g));
    for (int r = 0; r < replays; ++r) {
      CK(hipGraphLaunch(ge, st));
      launched += nodes;
      if (cycles == 1 && (r < 3 || r % 16 == 0)) {
        CK(hipStreamSynchronize(st));
        std::printf("replay %d ok\n", r);
        std::fflush(stdout);
      }
    }
    CK(hipStreamSynchronize(st));
    CK(hipGraphExecDestroy(ge));
    if (cycles > 1 && cyc % 16 == 0) {
      std::printf("cycle %d ok\n", cyc);
      std::fflush(stdout);
    }
  }
  float h = 0;
  CK(hipMemcpy(&h, p, 4, hipMemcpyDeviceToHost));
  std::printf("p[0] = %g (expect %d)\n", h, launched);
  return 0;
}
