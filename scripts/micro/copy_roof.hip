// Copy roofline of the resampling pass's HBM pattern at C4 (10M particles, fp16 state), standalone:
//   (a) 12 fp16 planes in / 12 out + two fp32 weight reads per particle (k_resample's 56 B), 2-byte accesses;
//   (b) the same bytes as 6 planes of 32-bit words (two fp16 planes interleaved);
//   (c) plain fp32 stream copy of the same byte count (56 B per particle as 14 dwords) for reference.
// Prints GB/s per variant (median of 20 launches).  Build: hipcc -O3 --offload-arch=gfx950 copy_roof.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>
#include <cstdint>
constexpr int N = 10000000;
__global__ void k_a(const float* __restrict__ w0, const float* __restrict__ w1, const uint16_t* __restrict__ src,
                    uint16_t* __restrict__ dst, size_t ld) {
  const int n = blockIdx.x * 256 + threadIdx.x;
  if (n >= N) return;
  const float s = w0[n] + w1[n];
  uint16_t v[12];
#pragma unroll
  for (int q = 0; q < 12; ++q) v[q] = src[q * ld + n];
  if (s == 12345.f) v[0] ^= 1;  // keep the weight loads
#pragma unroll
  for (int q = 0; q < 12; ++q) dst[q * ld + n] = v[q];
}
__global__ void k_b(const float* __restrict__ w0, const float* __restrict__ w1, const uint32_t* __restrict__ src,
                    uint32_t* __restrict__ dst, size_t ld) {
  const int n = blockIdx.x * 256 + threadIdx.x;
  if (n >= N) return;
  const float s = w0[n] + w1[n];
  uint32_t v[6];
#pragma unroll
  for (int q = 0; q < 6; ++q) v[q] = src[q * ld + n];
  if (s == 12345.f) v[0] ^= 1;
#pragma unroll
  for (int q = 0; q < 6; ++q) dst[q * ld + n] = v[q];
}
__global__ void k_c(const uint32_t* __restrict__ src, uint32_t* __restrict__ dst, size_t ld) {
  const int n = blockIdx.x * 256 + threadIdx.x;
  if (n >= N) return;
  uint32_t v[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) v[q] = src[q * ld + n];  // 32 B read
#pragma unroll
  for (int q = 0; q < 6; ++q) dst[q * ld + n] = v[q] ^ v[q + 2];  // 24 B written
}
int main() {
  const size_t ld = N;
  float *w0, *w1;
  void *src, *dst;
  hipMalloc(&w0, N * 4); hipMalloc(&w1, N * 4);
  hipMalloc(&src, 12 * ld * 4); hipMalloc(&dst, 12 * ld * 4);
  hipMemset(w0, 0, N * 4); hipMemset(w1, 0, N * 4); hipMemset(src, 0, 12 * ld * 4);
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  auto run = [&](const char* name, auto launch) {
    std::vector<float> t;
    for (int r = 0; r < 25; ++r) {
      hipEventRecord(a); launch(); hipEventRecord(b); hipEventSynchronize(b);
      float ms; hipEventElapsedTime(&ms, a, b); if (r >= 5) t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    const double us = t[t.size() / 2] * 1e3;
    printf("%-44s %8.1f us  %7.0f GB/s (56 B x 10M)\n", name, us, 56.0 * N / us / 1e3);
  };
  const int g = (N + 255) / 256;
  run("a: 12 fp16 planes, 2-B accesses", [&] { k_a<<<g, 256>>>(w0, w1, (uint16_t*)src, (uint16_t*)dst, ld); });
  run("b: 6 planes of fp16 pairs, 4-B accesses", [&] { k_b<<<g, 256>>>(w0, w1, (uint32_t*)src, (uint32_t*)dst, ld); });
  run("c: dword stream, 32 B in / 24 B out", [&] { k_c<<<g, 256>>>((uint32_t*)src, (uint32_t*)dst, ld); });
  return 0;
}
