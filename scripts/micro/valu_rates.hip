// Issue cost of the VALU instructions the PF kernels lean on, measured on gfx950: each kernel runs 8
// independent chains of ONE instruction per lane (inline asm, so the instruction is exactly the one named)
// at 8 waves per SIMD; cost = wall time x clock x SIMDs / wave-instructions.  The clock is measured in the
// same kernels (s_memtime / s_memrealtime over one wave), so the figures are cycles, not ns.
// Build: hipcc -O3 --offload-arch=gfx950 valu_rates.hip -o valu_rates
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int kIters = 2048;

#define CHAIN8(ASM, CONS)                                                                           \
  for (int it = 0; it < kIters; ++it) {                                                             \
    asm volatile(ASM : "+v"(x0) : CONS : "vcc", "s0");                                                            \
    asm volatile(ASM : "+v"(x1) : CONS : "vcc", "s0");                                                            \
    asm volatile(ASM : "+v"(x2) : CONS : "vcc", "s0");                                                            \
    asm volatile(ASM : "+v"(x3) : CONS : "vcc", "s0");                                                            \
    asm volatile(ASM : "+v"(x4) : CONS : "vcc", "s0");                                                            \
    asm volatile(ASM : "+v"(x5) : CONS : "vcc", "s0");                                                            \
    asm volatile(ASM : "+v"(x6) : CONS : "vcc", "s0");                                                            \
    asm volatile(ASM : "+v"(x7) : CONS : "vcc", "s0");                                                            \
  }

#define KERNEL32(NAME, ASM, CONS_T, CONS)                                                            \
  __global__ void NAME(uint32_t* out, CONS_T c, uint64_t* clk) {                                    \
    uint32_t x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5,       \
             x6 = x0 + 6, x7 = x0 + 7;                                                              \
    const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();        \
    CHAIN8(ASM, CONS(c))                                                                            \
    const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();        \
    if (blockIdx.x == 0 && threadIdx.x == 0) {                                                      \
      clk[0] = t1 - t0;                                                                             \
      clk[1] = r1 - r0;                                                                             \
    }                                                                                               \
    const uint32_t s = x0 ^ x1 ^ x2 ^ x3 ^ x4 ^ x5 ^ x6 ^ x7;                                       \
    if (s == 0x12345u) out[0] = s;                                                                  \
  }

#define KERNEL64(NAME, ASM, CONS_T, CONS)                                                            \
  __global__ void NAME(uint32_t* out, CONS_T c, uint64_t* clk) {                                    \
    uint64_t x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5,       \
             x6 = x0 + 6, x7 = x0 + 7;                                                              \
    const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();        \
    CHAIN8(ASM, CONS(c))                                                                            \
    const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();        \
    if (blockIdx.x == 0 && threadIdx.x == 0) {                                                      \
      clk[0] = t1 - t0;                                                                             \
      clk[1] = r1 - r0;                                                                             \
    }                                                                                               \
    const uint64_t s = x0 ^ x1 ^ x2 ^ x3 ^ x4 ^ x5 ^ x6 ^ x7;                                       \
    if (s == 0x12345u) out[0] = (uint32_t)s;                                                        \
  }

#define S_(c) "s"(c)
#define V_(c) "v"(c)

KERNEL32(k_add_f32, "v_add_f32 %0, %1, %0", float, S_)
KERNEL32(k_fma_f32, "v_fma_f32 %0, %1, %0, %0", float, S_)
KERNEL32(k_mul_u32, "v_mul_lo_u32 %0, %1, %0", uint32_t, S_)
KERNEL32(k_mulhi_u32, "v_mul_hi_u32 %0, %1, %0", uint32_t, S_)
KERNEL32(k_add_u32, "v_add_u32 %0, %1, %0", uint32_t, S_)
KERNEL32(k_bitop3, "v_bitop3_b32 %0, %0, %0, %1 bitop3:0x96", uint32_t, S_)
KERNEL32(k_cndmask, "v_cndmask_b32 %0, %0, %1, vcc", uint32_t, V_)
KERNEL32(k_mov, "v_mov_b32 %0, %1", uint32_t, V_)
KERNEL32(k_cvt_f32_f16, "v_cvt_f32_f16 %0, %0", uint32_t, S_)
KERNEL32(k_cvt_f16_f32, "v_cvt_f16_f32 %0, %0", uint32_t, S_)
KERNEL32(k_cvt_i32_f32, "v_cvt_i32_f32 %0, %0", uint32_t, S_)
KERNEL32(k_rcp_f32, "v_rcp_f32 %0, %0", uint32_t, S_)
KERNEL32(k_sqrt_f32, "v_sqrt_f32 %0, %0", uint32_t, S_)
KERNEL32(k_sin_f32, "v_sin_f32 %0, %0", uint32_t, S_)
KERNEL32(k_med3_f32, "v_med3_f32 %0, %0, %1, %0", float, S_)
KERNEL32(k_mov_dpp, "v_mov_b32_dpp %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf", uint32_t, S_)
KERNEL32(k_readlane, "v_readlane_b32 s0, %0, 3\n v_add_u32 %0, s0, %0", uint32_t, S_)
KERNEL32(k_perm, "v_perm_b32 %0, %0, %0, %1", uint32_t, S_)
KERNEL32(k_lshl_add, "v_lshl_add_u32 %0, %0, 3, %1", uint32_t, S_)
KERNEL64(k_mad_u64, "v_mad_u64_u32 %0, vcc, %1, 7, %0", uint32_t, S_)
KERNEL64(k_pk_fma_f32, "v_pk_fma_f32 %0, %0, %0, %0", uint32_t, S_)
KERNEL64(k_pk_add_f32, "v_pk_add_f32 %0, %0, %0", uint32_t, S_)
KERNEL64(k_fma_f64, "v_fma_f64 %0, %0, %0, %0", uint32_t, S_)
KERNEL64(k_add_f64, "v_add_f64 %0, %0, %0", uint32_t, S_)
KERNEL64(k_mov_b64, "v_mov_b64 %0, %0", uint32_t, S_)
KERNEL64(k_cvt_f64_f32, "v_cvt_f64_f32 %0, %1", uint32_t, S_)

int main() {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const int blocks = cus * 8, threads = 256;  // 8 waves per SIMD
  uint32_t* d = nullptr;
  uint64_t* clk = nullptr;
  hipMalloc(&d, 64);
  hipMalloc(&clk, 16);
  const double waves = (double)blocks * threads / 64;
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  auto run = [&](const char* name, auto kern, auto c) {
    hipLaunchKernelGGL(kern, blocks, threads, 0, 0, d, c, clk);
    hipDeviceSynchronize();
    hipEventRecord(a);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(kern, blocks, threads, 0, 0, d, c, clk);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    ms /= 5;
    uint64_t h[2];
    hipMemcpy(h, clk, 16, hipMemcpyDeviceToHost);
    const double ghz = h[1] ? (double)h[0] / (double)h[1] * 0.1 : 2.4;  // s_memrealtime: 100 MHz
    const double cyc = ms * 1e-3 * ghz * 1e9 * (cus * 4) / (waves * 8.0 * kIters);
    printf("%-16s %7.3f ms  clock %.2f GHz  %6.2f cycles per wave-instruction per SIMD\n", name, ms, ghz, cyc);
  };
  run("v_add_f32", k_add_f32, 1.0f);
  run("v_fma_f32", k_fma_f32, 1.0f);
  run("v_pk_add_f32", k_pk_add_f32, 1u);
  run("v_pk_fma_f32", k_pk_fma_f32, 1u);
  run("v_add_u32", k_add_u32, 1u);
  run("v_lshl_add_u32", k_lshl_add, 1u);
  run("v_bitop3_b32", k_bitop3, 1u);
  run("v_perm_b32", k_perm, 0x05040100u);
  run("v_cndmask_b32", k_cndmask, 1u);
  run("v_mov_b32", k_mov, 1u);
  run("v_mov_b64", k_mov_b64, 1u);
  run("v_mov_b32_dpp", k_mov_dpp, 1u);
  run("v_readlane+add", k_readlane, 1u);
  run("v_med3_f32", k_med3_f32, 1.0f);
  run("v_cvt_f32_f16", k_cvt_f32_f16, 1u);
  run("v_cvt_f16_f32", k_cvt_f16_f32, 1u);
  run("v_cvt_i32_f32", k_cvt_i32_f32, 1u);
  run("v_cvt_f64_f32", k_cvt_f64_f32, 1u);
  run("v_rcp_f32", k_rcp_f32, 1u);
  run("v_sqrt_f32", k_sqrt_f32, 1u);
  run("v_sin_f32", k_sin_f32, 1u);
  run("v_mul_lo_u32", k_mul_u32, 3u);
  run("v_mul_hi_u32", k_mulhi_u32, 3u);
  run("v_mad_u64_u32", k_mad_u64, 0xD2511F53u);
  run("v_add_f64", k_add_f64, 1u);
  run("v_fma_f64", k_fma_f64, 1u);
  hipFree(d);
  hipFree(clk);
  return 0;
}
