// mfma_fill.hip -- what issuing other instructions between v_mfma_f32_32x32x2_f32 costs on gfx950
// (diagnostic only, tools/). Every kernel runs one block per CU (256 blocks), NW waves per block,
// each wave a loop of groups of NACC independent MFMAs (one accumulator tile each, the Winograd /
// ring kernels' shape); between consecutive MFMAs F filler instructions of one kind, whose results
// never feed an MFMA. Reported: shader-clock cycles per MFMA per wave (s_memtime), median block.
//   hipcc --offload-arch=gfx950 -O3 -o tools/mfma_fill tools/mfma_fill.hip && tools/mfma_fill
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e = (x);                                                          \
    if (e != hipSuccess) {                                                       \
      std::printf("%s: %s\n", #x, hipGetErrorString(e));                         \
      return 1;                                                                  \
    }                                                                            \
  } while (0)

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int ITER = 64;

enum { K_NONE, K_VADD, K_VPK, K_DSR32, K_DSR128, K_VMEM, K_SALU, K_DSW128, K_VFMA_DEP, K_BAR };

template <int KIND>
__device__ __forceinline__ void filler(float &x0, float &x1, float &x2, float &x3, f32x4 &q, uint32_t lds, uint32_t voff,
                                       __amdgpu_buffer_rsrc_t r, int &s) {
  if constexpr (KIND == K_VADD) asm volatile("v_add_f32 %0, %0, %1" : "+v"(x0) : "v"(x1));
  if constexpr (KIND == K_VPK) {
    typedef float f2 __attribute__((ext_vector_type(2)));
    f2 a = {x0, x1}, b = {x2, x3};
    asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(a) : "v"(b));
    x0 = a[0];
  }
  if constexpr (KIND == K_DSR32) asm volatile("ds_read_b32 %0, %1" : "=v"(x2) : "v"(lds));
  if constexpr (KIND == K_DSR128) asm volatile("ds_read_b128 %0, %1" : "=v"(q) : "v"(lds));
  if constexpr (KIND == K_DSW128) asm volatile("ds_write_b128 %0, %1 offset:4096" : : "v"(lds), "v"(q));
  if constexpr (KIND == K_VMEM) x3 = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, voff, 0, 0));
  if constexpr (KIND == K_SALU) asm volatile("s_add_u32 %0, %0, 3" : "+s"(s));
  if constexpr (KIND == K_VFMA_DEP) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(x0) : "v"(x1), "v"(x2));
}

template <int NW, int NACC, int KIND, int F>
__global__ __launch_bounds__(NW * 64) void fill_k(const float *buf, float *out, unsigned long long *cyc) {
  __shared__ __attribute__((aligned(16))) float lds[2048];
  const int tid = threadIdx.x;
  lds[tid % 1024] = 0.0f;
  __syncthreads();
  f32x16 acc[NACC];
#pragma unroll
  for (int j = 0; j < NACC; ++j)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[j][e] = 0.0f;
  float a = buf[tid], b = buf[tid + 64];
  float x0 = a, x1 = b, x2 = 0.0f, x3 = 0.0f;
  f32x4 q = {a, b, a, b};
  const uint32_t ldsa = (uint32_t)(uintptr_t)lds + (uint32_t)(tid & 63) * 16u;
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void *)buf, 0, 65536 * 4, 0x00020000);
  const uint32_t voff = (uint32_t)((blockIdx.x * 256 + tid) % 16384) * 4u;
  int s = __builtin_amdgcn_readfirstlane((int)blockIdx.x);
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < ITER; ++it) {
#pragma unroll
    for (int j = 0; j < NACC; ++j) {
      asm volatile("v_mfma_f32_32x32x2_f32 %0, %1, %2, %0" : "+a"(acc[j]) : "v"(a), "v"(b));
#pragma unroll
      for (int f = 0; f < F; ++f) filler<KIND>(x0, x1, x2, x3, q, ldsa, voff, r, s);
    }
    if constexpr (KIND == K_DSR32 || KIND == K_DSR128 || KIND == K_DSW128) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if constexpr (KIND == K_VMEM) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if constexpr (KIND == K_BAR) __builtin_amdgcn_s_barrier();
  }
  asm volatile("s_nop 7\n s_nop 7\n s_nop 7" ::: "memory");
  float sum = x0 + x2 + x3 + q[0] + q[3] + (float)s;
#pragma unroll
  for (int j = 0; j < NACC; ++j) {
    f32x16 v;
    asm volatile("s_nop 7\n s_nop 7\n v_accvgpr_read_b32 %0, %1" : "=v"(v[0]) : "a"(acc[j][0]));
    sum += v[0];
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * NW * 64 + tid] = sum;
  if ((tid & 63) == 0) cyc[blockIdx.x * NW + (tid >> 6)] = t1 - t0;
}

// v_mfma_f32_16x16x4_f32 (half the flops of 32x32x2) with NACC independent accumulators, no fillers
template <int NW, int NACC>
__global__ __launch_bounds__(NW * 64) void m16_k(const float *buf, float *out, unsigned long long *cyc) {
  const int tid = threadIdx.x;
  f32x4 acc[NACC];
#pragma unroll
  for (int j = 0; j < NACC; ++j) acc[j] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
  float a = buf[tid], b = buf[tid + 64];
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < ITER; ++it) {
#pragma unroll
    for (int j = 0; j < NACC; ++j) asm volatile("v_mfma_f32_16x16x4_f32 %0, %1, %2, %0" : "+a"(acc[j]) : "v"(a), "v"(b));
  }
  asm volatile("s_nop 7\n s_nop 7\n s_nop 7" ::: "memory");
  float sum = 0.0f;
#pragma unroll
  for (int j = 0; j < NACC; ++j) {
    float v;
    asm volatile("s_nop 7\n s_nop 7\n v_accvgpr_read_b32 %0, %1" : "=v"(v) : "a"(acc[j][0]));
    sum += v;
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * NW * 64 + tid] = sum;
  if ((tid & 63) == 0) cyc[blockIdx.x * NW + (tid >> 6)] = t1 - t0;
}

template <int NW, int NACC>
int run16(const char *name, const float *buf, float *out, unsigned long long *cyc) {
  const int blocks = 256;
  for (int rep = 0; rep < 3; ++rep) m16_k<NW, NACC><<<blocks, NW * 64>>>(buf, out, cyc);
  CK(hipDeviceSynchronize());
  std::vector<unsigned long long> h((size_t)blocks * NW);
  CK(hipMemcpy(h.data(), cyc, h.size() * 8, hipMemcpyDeviceToHost));
  std::sort(h.begin(), h.end());
  std::printf("%-14s waves/SIMD %d  NACC %2d  16x16x4          : %6.1f cyc per MFMA\n", name, NW / 4, NACC,
              (double)h[h.size() / 2] / (ITER * NACC));
  return 0;
}

template <int NW, int NACC, int KIND, int F>
int run(const char *name, const float *buf, float *out, unsigned long long *cyc) {
  const int blocks = 256;
  for (int rep = 0; rep < 3; ++rep) fill_k<NW, NACC, KIND, F><<<blocks, NW * 64>>>(buf, out, cyc);
  CK(hipDeviceSynchronize());
  std::vector<unsigned long long> h((size_t)blocks * NW);
  CK(hipMemcpy(h.data(), cyc, h.size() * 8, hipMemcpyDeviceToHost));
  std::sort(h.begin(), h.end());
  const double per = (double)h[h.size() / 2] / (ITER * NACC);
  std::printf("%-14s waves/SIMD %d  NACC %2d  fillers/MFMA %2d : %6.1f cyc per MFMA (max wave %6.1f)\n", name, NW / 4,
              NACC, F, per, (double)h.back() / (ITER * NACC));
  return 0;
}

int main() {
  float *buf, *out;
  unsigned long long *cyc;
  CK(hipMalloc(&buf, 65536 * 4));
  CK(hipMemset(buf, 0, 65536 * 4));
  CK(hipMalloc(&out, 256 * 512 * 4));
  CK(hipMalloc(&cyc, 256 * 8 * 8));
  int rc = 0;
  rc |= run16<4, 1>("m16", buf, out, cyc);
  rc |= run16<4, 4>("m16", buf, out, cyc);
  rc |= run16<4, 8>("m16", buf, out, cyc);
  rc |= run16<4, 16>("m16", buf, out, cyc);
  rc |= run16<8, 8>("m16", buf, out, cyc);
  rc |= run<4, 16, K_NONE, 0>("none", buf, out, cyc);
  rc |= run<4, 1, K_NONE, 0>("none-dep", buf, out, cyc);
  rc |= run<4, 2, K_NONE, 0>("none-2acc", buf, out, cyc);
  rc |= run<4, 16, K_VADD, 2>("v_add", buf, out, cyc);
  rc |= run<4, 16, K_VADD, 4>("v_add", buf, out, cyc);
  rc |= run<4, 16, K_VADD, 8>("v_add", buf, out, cyc);
  rc |= run<4, 16, K_VADD, 12>("v_add", buf, out, cyc);
  rc |= run<4, 16, K_VADD, 16>("v_add", buf, out, cyc);
  rc |= run<4, 16, K_VFMA_DEP, 4>("v_fma dep", buf, out, cyc);
  rc |= run<4, 16, K_VFMA_DEP, 8>("v_fma dep", buf, out, cyc);
  rc |= run<4, 16, K_VPK, 2>("v_pk_add", buf, out, cyc);
  rc |= run<4, 16, K_VPK, 4>("v_pk_add", buf, out, cyc);
  rc |= run<4, 16, K_VPK, 8>("v_pk_add", buf, out, cyc);
  rc |= run<4, 16, K_SALU, 4>("s_add", buf, out, cyc);
  rc |= run<4, 16, K_SALU, 8>("s_add", buf, out, cyc);
  rc |= run<4, 16, K_SALU, 16>("s_add", buf, out, cyc);
  rc |= run<4, 16, K_DSR32, 1>("ds_read_b32", buf, out, cyc);
  rc |= run<4, 16, K_DSR32, 2>("ds_read_b32", buf, out, cyc);
  rc |= run<4, 16, K_DSR32, 4>("ds_read_b32", buf, out, cyc);
  rc |= run<4, 16, K_DSR128, 1>("ds_read_b128", buf, out, cyc);
  rc |= run<4, 16, K_DSR128, 2>("ds_read_b128", buf, out, cyc);
  rc |= run<4, 16, K_DSR128, 4>("ds_read_b128", buf, out, cyc);
  rc |= run<4, 16, K_DSW128, 1>("ds_write_b128", buf, out, cyc);
  rc |= run<4, 16, K_DSW128, 2>("ds_write_b128", buf, out, cyc);
  rc |= run<4, 16, K_VMEM, 1>("buffer_load", buf, out, cyc);
  rc |= run<4, 16, K_VMEM, 2>("buffer_load", buf, out, cyc);
  rc |= run<4, 16, K_VMEM, 4>("buffer_load", buf, out, cyc);
  rc |= run<4, 16, K_BAR, 0>("s_barrier/16", buf, out, cyc);
  rc |= run<4, 4, K_BAR, 0>("s_barrier/4", buf, out, cyc);
  rc |= run<8, 8, K_NONE, 0>("none", buf, out, cyc);
  rc |= run<8, 8, K_VADD, 8>("v_add", buf, out, cyc);
  rc |= run<8, 8, K_VADD, 16>("v_add", buf, out, cyc);
  rc |= run<8, 8, K_DSR128, 2>("ds_read_b128", buf, out, cyc);
  rc |= run<8, 8, K_VMEM, 2>("buffer_load", buf, out, cyc);
  return rc;
}
