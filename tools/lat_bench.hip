// lat_bench.hip -- latency composition of a small op inside a replayed hipGraph of back-to-back
// kernels (the bench's per-op convention), from device-clock marks (100 MHz wall clock):
//   gap    last block's store-ack of launch i -> first block's entry of launch i+1
//   load   entry -> first global load returned (data the previous launch read: warm)
//   load2  a second, dependent load (address from the first)
//   store  store issued -> acknowledged (s_waitcnt vmcnt(0))
// Diagnostic only (tools/).
//   hipcc --offload-arch=gfx950 -O3 -o tools/lat_bench tools/lat_bench.hip && tools/lat_bench
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

#define CK(x)                                                                           \
  do {                                                                                  \
    hipError_t e = (x);                                                                 \
    if (e != hipSuccess) {                                                              \
      std::printf("%s: %s\n", #x, hipGetErrorString(e));                                \
      return 1;                                                                         \
    }                                                                                   \
  } while (0)

constexpr int NL = 64;  // launches per graph

// each block: one float4 per lane from `in` (+ a dependent one), one float per lane to `out`
__global__ void lat_k(const float *in, float *out, unsigned long long *marks, int launch, int nbytes_per_blk) {
  const int lane = threadIdx.x;
  const unsigned long long t0 = wall_clock64();
  const float4 v = ((const float4 *)in)[(size_t)blockIdx.x * (nbytes_per_blk / 16) + lane];
  float s = v.x + v.y + v.z + v.w;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const unsigned long long t1 = wall_clock64();
  const int j = ((int)s & 15) + lane;  // dependent address (s is 0: data zeroed)
  const float w = in[(size_t)blockIdx.x * (nbytes_per_blk / 4) + j + 1024];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const unsigned long long t2 = wall_clock64();
  out[(size_t)blockIdx.x * 64 + lane] = s + w;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const unsigned long long t3 = wall_clock64();
  if (lane == 0) {
    unsigned long long *m = marks + ((size_t)launch * gridDim.x + blockIdx.x) * 4;
    m[0] = t0;
    m[1] = t1;
    m[2] = t2;
    m[3] = t3;
  }
}

// instruction fetch: 4096 straight-line s_nop (16 KB of code) vs the same count from a loop
__global__ void code_big(unsigned long long *marks, int launch) {
  const unsigned long long t0 = wall_clock64();
  asm volatile(".rept 4096\n s_nop 0\n .endr" ::: "memory");
  const unsigned long long t1 = wall_clock64();
  if (threadIdx.x == 0) {
    marks[((size_t)launch * gridDim.x + blockIdx.x) * 4] = t0;
    marks[((size_t)launch * gridDim.x + blockIdx.x) * 4 + 1] = t1;
  }
}
__global__ void code_loop(unsigned long long *marks, int launch, int n) {
  const unsigned long long t0 = wall_clock64();
  for (int i = 0; i < n; ++i) asm volatile(".rept 64\n s_nop 0\n .endr" ::: "memory");
  const unsigned long long t1 = wall_clock64();
  if (threadIdx.x == 0) {
    marks[((size_t)launch * gridDim.x + blockIdx.x) * 4] = t0;
    marks[((size_t)launch * gridDim.x + blockIdx.x) * 4 + 1] = t1;
  }
}

template <typename F>
int code_run(const char *name, F launch, unsigned long long *marks, hipStream_t st, int blocks) {
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
  for (int l = 0; l < NL; ++l) launch(l);
  CK(hipStreamEndCapture(st, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  for (int rep = 0; rep < 3; ++rep) {
    CK(hipGraphLaunch(ge, st));
    CK(hipStreamSynchronize(st));
    std::vector<unsigned long long> h((size_t)NL * blocks * 4);
    CK(hipMemcpy(h.data(), marks, h.size() * 8, hipMemcpyDeviceToHost));
    std::vector<double> d;
    for (int l = 0; l < NL; ++l)
      for (int b = 0; b < blocks; ++b) d.push_back((h[((size_t)l * blocks + b) * 4 + 1] - h[((size_t)l * blocks + b) * 4]) * 0.01);
    std::sort(d.begin(), d.end());
    if (rep) std::printf("%-34s blocks %4d: in-kernel %.2f us median, %.2f min, %.2f max\n", name, blocks, d[d.size() / 2], d[0], d.back());
  }
  CK(hipGraphExecDestroy(ge));
  CK(hipGraphDestroy(g));
  return 0;
}

// load-issue rate: each lane issues NL independent loads of W dwords (all in flight), 8 waves a
// block, one block per CU; in-kernel span from the first entry to the last completion
template <int NL, int W>
__global__ __launch_bounds__(512) void issue_k(const float *in, float *out, unsigned long long *marks, int launch) {
  const int tid = threadIdx.x;
  const unsigned long long t0 = wall_clock64();
  float s = 0.0f;
  const float *base = in + (size_t)blockIdx.x * (NL * 512 * W);
  if constexpr (W == 1) {
    float v[NL];
#pragma unroll
    for (int j = 0; j < NL; ++j) v[j] = base[j * 512 + tid];
#pragma unroll
    for (int j = 0; j < NL; ++j) s += v[j];
  } else {
    float4 v[NL];
#pragma unroll
    for (int j = 0; j < NL; ++j) v[j] = ((const float4 *)base)[j * 512 + tid];
#pragma unroll
    for (int j = 0; j < NL; ++j) s += v[j].x + v[j].y + v[j].z + v[j].w;
  }
  out[(size_t)blockIdx.x * 512 + tid] = s;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const unsigned long long t1 = wall_clock64();
  if (tid == 0) {
    marks[((size_t)launch * gridDim.x + blockIdx.x) * 4] = t0;
    marks[((size_t)launch * gridDim.x + blockIdx.x) * 4 + 1] = t1;
  }
}

int main() {
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  const int per_blk = 8192;  // bytes of `in` per block
  float *in, *out;
  unsigned long long *marks;
  CK(hipMalloc(&in, 1024 * per_blk));
  CK(hipMalloc(&out, 1024 * 64 * 4));
  CK(hipMalloc(&marks, (size_t)NL * 1024 * 4 * 8));
  CK(hipMemset(in, 0, 1024 * per_blk));
  for (int blocks : {32, 256, 1024}) {
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
    for (int l = 0; l < NL; ++l) lat_k<<<blocks, 64, 0, st>>>(in, out, marks, l, per_blk);
    CK(hipStreamEndCapture(st, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    for (int rep = 0; rep < 3; ++rep) {
      hipEvent_t a, b;
      CK(hipEventCreate(&a));
      CK(hipEventCreate(&b));
      CK(hipEventRecord(a, st));
      CK(hipGraphLaunch(ge, st));
      CK(hipEventRecord(b, st));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      std::vector<unsigned long long> h((size_t)NL * blocks * 4);
      CK(hipMemcpy(h.data(), marks, h.size() * 8, hipMemcpyDeviceToHost));
      std::vector<double> gap, ld, ld2, stl, span;
      for (int l = 0; l < NL; ++l) {
        unsigned long long mn0 = ~0ull, mx3 = 0;
        for (int b2 = 0; b2 < blocks; ++b2) {
          const unsigned long long *m = &h[((size_t)l * blocks + b2) * 4];
          mn0 = std::min(mn0, m[0]);
          mx3 = std::max(mx3, m[3]);
          ld.push_back((m[1] - m[0]) * 0.01);
          ld2.push_back((m[2] - m[1]) * 0.01);
          stl.push_back((m[3] - m[2]) * 0.01);
        }
        span.push_back((mx3 - mn0) * 0.01);
        if (l + 1 < NL) {
          unsigned long long nx = ~0ull;
          for (int b2 = 0; b2 < blocks; ++b2) nx = std::min(nx, h[((size_t)(l + 1) * blocks + b2) * 4]);
          gap.push_back(((double)nx - (double)mx3) * 0.01);
        }
      }
      auto med = [](std::vector<double> v) {
        std::sort(v.begin(), v.end());
        return v[v.size() / 2];
      };
      auto mx = [](const std::vector<double> &v) { return *std::max_element(v.begin(), v.end()); };
      if (rep)
        std::printf("blocks %4d: %.3f us/launch | gap %.2f (max %.2f) | span %.2f | load %.2f (max %.2f) | load2 %.2f "
                    "| store %.2f (max %.2f)\n",
                    blocks, ms * 1e3 / NL, med(gap), mx(gap), med(span), med(ld), mx(ld), med(ld2), med(stl), mx(stl));
      CK(hipEventDestroy(a));
      CK(hipEventDestroy(b));
    }
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
  }
  {
    float *big;
    CK(hipMalloc(&big, (size_t)256 * 64 * 512 * 16));
    CK(hipMemset(big, 0, (size_t)256 * 64 * 512 * 16));
    float *o2;
    CK(hipMalloc(&o2, 256 * 512 * 4));
    if (code_run("8 dword loads/lane, 8 waves", [&](int l) { issue_k<8, 1><<<256, 512, 0, st>>>(big, o2, marks, l); }, marks, st, 256)) return 1;
    if (code_run("32 dword loads/lane, 8 waves", [&](int l) { issue_k<32, 1><<<256, 512, 0, st>>>(big, o2, marks, l); }, marks, st, 256)) return 1;
    if (code_run("64 dword loads/lane, 8 waves", [&](int l) { issue_k<64, 1><<<256, 512, 0, st>>>(big, o2, marks, l); }, marks, st, 256)) return 1;
    if (code_run("8 dwordx4 loads/lane, 8 waves", [&](int l) { issue_k<8, 4><<<256, 512, 0, st>>>(big, o2, marks, l); }, marks, st, 256)) return 1;
    if (code_run("32 dwordx4 loads/lane, 8 waves", [&](int l) { issue_k<32, 4><<<256, 512, 0, st>>>(big, o2, marks, l); }, marks, st, 256)) return 1;
  }
  for (int blocks : {1, 256}) {
    if (code_run("4096 s_nop straight-line (16 KB)", [&](int l) { code_big<<<blocks, 64, 0, st>>>(marks, l); }, marks, st,
                 blocks))
      return 1;
    if (code_run("4096 s_nop as 64 x loop of 64", [&](int l) { code_loop<<<blocks, 64, 0, st>>>(marks, l, 64); }, marks,
                 st, blocks))
      return 1;
  }
  return 0;
}
