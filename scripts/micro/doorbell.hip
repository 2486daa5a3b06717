// Host <-> persistent-kernel doorbell latency (round 5, the resident frame server's hand-off; measurement only).
// One wave polls a doorbell word, optionally reads a message of `msg` bytes, and answers in pinned host memory; the
// host rings, spins on the answer, repeats.  Round trip per iteration for:
//   A: doorbell + message in pinned host memory (system-scope loads over PCIe; the server's current form)
//   B: doorbell + message in fine-grained device memory written by the CPU through its pointer
//   C: the same in uncached device memory
// Every wait is bounded (s_memrealtime, ~1 s) on both sides.
//   hipcc --offload-arch=gfx950 -O2 -o doorbell doorbell.hip && ./doorbell
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>
#include <algorithm>

#define CHK(x)                                                                          \
  do {                                                                                  \
    hipError_t e_ = (x);                                                                \
    if (e_ != hipSuccess) {                                                             \
      printf("%s: %s\n", #x, hipGetErrorString(e_));                                    \
      return 1;                                                                         \
    }                                                                                   \
  } while (0)

__global__ void k_pong(const uint64_t* bell, const uint64_t* msg, int msg_words, uint64_t* pong, int iters,
                       uint64_t* sink) {
  const int lane = threadIdx.x;
  uint64_t acc = 0;
  for (int i = 1; i <= iters; ++i) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    bool ok = false;
    for (;;) {
      if (__hip_atomic_load(bell, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) >= (uint64_t)i) {
        ok = true;
        break;
      }
      if (__builtin_amdgcn_s_memrealtime() - t0 > 100000000ull) break;
      __builtin_amdgcn_s_sleep(1);
    }
    if (!ok) break;
    uint64_t w[4] = {0, 0, 0, 0};
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (lane + 64 * r < msg_words) w[r] = __hip_atomic_load(msg + lane + 64 * r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    acc += w[0] + w[1] + w[2] + w[3];
    if (lane == 0) __hip_atomic_store(pong, (uint64_t)i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  sink[lane] = acc;
}

static int run(const char* name, uint64_t* bell_host_view, uint64_t* bell_dev, uint64_t* msg_host_view, uint64_t* msg_dev,
               int msg_bytes, uint64_t* pong_host, uint64_t* pong_dev, uint64_t* sink, int iters) {
  *(volatile uint64_t*)bell_host_view = 0;
  *(volatile uint64_t*)pong_host = 0;
  __atomic_thread_fence(__ATOMIC_SEQ_CST);
  hipStream_t s;
  CHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  printf("%s msg %d: start\n", name, msg_bytes);
  hipLaunchKernelGGL(k_pong, dim3(1), dim3(64), 0, s, bell_dev, msg_dev, msg_bytes / 8, pong_dev, iters, sink);
  CHK(hipGetLastError());
  std::vector<double> rt;
  rt.reserve(iters);
  for (int i = 1; i <= iters; ++i) {
    const auto t0 = std::chrono::steady_clock::now();
    for (int k = 0; k < msg_bytes / 8; ++k) ((volatile uint64_t*)msg_host_view)[k] = (uint64_t)i * 1000 + k;
    __atomic_thread_fence(__ATOMIC_SEQ_CST);
    *(volatile uint64_t*)bell_host_view = (uint64_t)i;
    bool ok = false;
    for (;;) {
      if (*(volatile uint64_t*)pong_host >= (uint64_t)i) {
        ok = true;
        break;
      }
      if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) break;
    }
    if (!ok) {
      printf("%s: no answer at iteration %d\n", name, i);
      break;
    }
    rt.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
  }
  CHK(hipStreamSynchronize(s));
  CHK(hipStreamDestroy(s));
  std::vector<double> v(rt.begin() + rt.size() / 10, rt.end());
  std::sort(v.begin(), v.end());
  if (!v.empty())
    printf("%-34s msg %5d B: round trip median %6.2f us  p10 %6.2f  p90 %6.2f  (%zu)\n", name, msg_bytes, v[v.size() / 2],
           v[v.size() / 10], v[v.size() * 9 / 10], v.size());
  return 0;
}

int main() {
  setvbuf(stdout, nullptr, _IONBF, 0);
  const int iters = 3000;
  uint64_t *pong_h, *pong_d, *sink;
  CHK(hipHostMalloc((void**)&pong_h, 256, hipHostMallocMapped | hipHostMallocCoherent));
  CHK(hipHostGetDevicePointer((void**)&pong_d, pong_h, 0));
  CHK(hipMalloc((void**)&sink, 64 * 8));
  // A: pinned host memory
  uint64_t *hb, *hbd;
  CHK(hipHostMalloc((void**)&hb, 8192, hipHostMallocMapped | hipHostMallocCoherent));
  CHK(hipHostGetDevicePointer((void**)&hbd, hb, 0));
  for (int mb : {0, 1024})
    if (run("A pinned host doorbell+message", hb, hbd, hb + 64, hbd + 64, mb, pong_h, pong_d, sink, iters)) return 1;
  // B / C: device memory the CPU writes directly (large-BAR mapping), if the runtime gives a CPU-usable pointer
  for (unsigned flags : {(unsigned)hipDeviceMallocFinegrained, (unsigned)hipDeviceMallocUncached}) {
    uint64_t* db = nullptr;
    if (hipExtMallocWithFlags((void**)&db, 8192, flags) != hipSuccess) {
      printf("flags %u: allocation failed\n", flags);
      continue;
    }
    hipPointerAttribute_t at{};
    if (hipPointerGetAttributes(&at, db) == hipSuccess)
      printf("flags %u: device %p host %p type %d\n", flags, at.devicePointer, at.hostPointer, (int)at.type);
    uint64_t* hv = (uint64_t*)at.hostPointer;
    if (!hv) hv = db;  // unified address: try the device pointer from the CPU
    const char* nm = flags == hipDeviceMallocFinegrained ? "B fine-grained device doorbell+msg" : "C uncached device doorbell+msg";
    for (int mb : {0, 1024})
      if (run(nm, hv, db, hv + 64, db + 64, mb, pong_h, pong_d, sink, iters)) return 1;
  }
  printf("done\n");
  return 0;
}
