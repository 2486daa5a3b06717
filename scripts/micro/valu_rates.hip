// Issue cost of the instructions the PF kernels lean on (v_mad_u64_u32 for Philox, v_fma_f32, v_fma_f64,
// v_cvt, DPP moves), measured as wall time of 8 independent chains per lane at full occupancy.
// Build: hipcc -O3 --offload-arch=gfx950 valu_rates.hip -o valu_rates
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int kIters = 4096;

__global__ void k_fma(float* out, float a) {
  float x[8];
  for (int i = 0; i < 8; ++i) x[i] = threadIdx.x + i;
  for (int it = 0; it < kIters; ++it)
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = __builtin_fmaf(x[i], a, 1.0f);
  float s = 0;
  for (int i = 0; i < 8; ++i) s += x[i];
  if (s == 12345.f) out[0] = s;
}
__global__ void k_mad64(uint32_t* out, uint32_t m) {
  uint32_t x[8];
  for (int i = 0; i < 8; ++i) x[i] = threadIdx.x + i;
  for (int it = 0; it < kIters; ++it)
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const uint64_t p = (uint64_t)x[i] * m;
      x[i] = (uint32_t)(p >> 32) ^ (uint32_t)p;
    }
  uint32_t s = 0;
  for (int i = 0; i < 8; ++i) s += x[i];
  if (s == 12345u) out[0] = s;
}
__global__ void k_mulhi(uint32_t* out, uint32_t m) {
  uint32_t x[8];
  for (int i = 0; i < 8; ++i) x[i] = threadIdx.x + i;
  for (int it = 0; it < kIters; ++it)
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = __umulhi(x[i], m) ^ x[i];
  uint32_t s = 0;
  for (int i = 0; i < 8; ++i) s += x[i];
  if (s == 12345u) out[0] = s;
}
__global__ void k_fma64(double* out, double a) {
  double x[8];
  for (int i = 0; i < 8; ++i) x[i] = threadIdx.x + i;
  for (int it = 0; it < kIters; ++it)
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = __builtin_fma(x[i], a, 1.0);
  double s = 0;
  for (int i = 0; i < 8; ++i) s += x[i];
  if (s == 12345.) out[0] = s;
}
__global__ void k_div64(double* out, double a) {
  double x[8];
  for (int i = 0; i < 8; ++i) x[i] = threadIdx.x + i + 1;
  for (int it = 0; it < kIters / 8; ++it)
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = a / x[i] + 1.0;
  double s = 0;
  for (int i = 0; i < 8; ++i) s += x[i];
  if (s == 12345.) out[0] = s;
}

template <typename F>
float time_it(F launch) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  launch();
  hipDeviceSynchronize();
  hipEventRecord(a);
  for (int r = 0; r < 5; ++r) launch();
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  return ms / 5;
}

int main() {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const int blocks = cus * 8, threads = 256;  // 8 waves per SIMD
  void* d = nullptr;
  hipMalloc(&d, 64);
  const double waves = (double)blocks * threads / 64;
  auto report = [&](const char* name, float ms, double ops_per_lane) {
    // cycles per wave-instruction per SIMD at 2.4 GHz: time * clk * SIMDs / (waves * ops)
    const double cyc = ms * 1e-3 * 2.4e9 * (cus * 4) / (waves * ops_per_lane);
    printf("%-28s %8.3f ms  %6.2f cycles per wave-instruction per SIMD (at 2.4 GHz)\n", name, ms, cyc);
  };
  report("v_fma_f32", time_it([&] { hipLaunchKernelGGL(k_fma, blocks, threads, 0, 0, (float*)d, 1.0001f); }),
         8.0 * kIters);
  report("v_mad_u64_u32 (+xor)", time_it([&] { hipLaunchKernelGGL(k_mad64, blocks, threads, 0, 0, (uint32_t*)d, 0xD2511F53u); }),
         8.0 * kIters);
  report("v_mul_hi_u32 (+xor)", time_it([&] { hipLaunchKernelGGL(k_mulhi, blocks, threads, 0, 0, (uint32_t*)d, 0xD2511F53u); }),
         8.0 * kIters);
  report("v_fma_f64", time_it([&] { hipLaunchKernelGGL(k_fma64, blocks, threads, 0, 0, (double*)d, 1.0001); }),
         8.0 * kIters);
  report("f64 division (+add)", time_it([&] { hipLaunchKernelGGL(k_div64, blocks, threads, 0, 0, (double*)d, 3.0); }),
         8.0 * kIters / 8);
  hipFree(d);
  return 0;
}
