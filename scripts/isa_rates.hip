// isa_rates.hip — issue cost of the vector instructions the weighing / resampling kernels are made of (gfx950).
// Diagnostic only (not part of the library).  Each kernel issues R rounds of 16 independent copies of one
// instruction (inline asm; outputs never read, inputs loop-invariant), W waves per SIMD on every CU, and reports
// s_memtime cycles per wave-instruction per SIMD = elapsed cycles / (instructions per wave * waves per SIMD).
//   hipcc --offload-arch=gfx950 -O2 scripts/isa_rates.hip -o /tmp/isa_rates && /tmp/isa_rates
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <algorithm>

constexpr int kRounds = 256;

#define REP16(X) X X X X X X X X X X X X X X X X

#define DEFK(NAME, BODY)                                                                           \
  __global__ __launch_bounds__(256) void NAME(uint64_t* cyc, uint32_t seed) {                     \
    uint32_t a = seed ^ threadIdx.x, b = seed * 3u + threadIdx.x, c = seed + 7u;                 \
    float fa = (float)a, fb = (float)b, fc = 1.5f;                                                 \
    double da = (double)a, db = (double)b;                                                         \
    uint64_t o64;                                                                                  \
    uint32_t o32;                                                                                  \
    float of;                                                                                      \
    double od;                                                                                     \
    const uint64_t m64 = __builtin_amdgcn_ballot_w64((threadIdx.x & 3) != 0);                     \
    __syncthreads();                                                                               \
    const uint64_t t0 = __builtin_amdgcn_s_memtime();                                              \
    for (int r = 0; r < kRounds; ++r) {                                                            \
      REP16(BODY)                                                                                  \
    }                                                                                              \
    const uint64_t t1 = __builtin_amdgcn_s_memtime();                                              \
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 4 + (threadIdx.x >> 6)] = t1 - t0;               \
    (void)o64; (void)o32; (void)of; (void)od; (void)fa; (void)fb; (void)fc; (void)da; (void)db;    \
    (void)a; (void)b; (void)c; (void)m64;                                                          \
  }

DEFK(k_mad_u64, asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %2, 0" : "=v"(o64) : "v"(a), "v"(b) : "s0", "s1");)
DEFK(k_mul_hi_u32, asm volatile("v_mul_hi_u32 %0, %1, %2" : "=v"(o32) : "v"(a), "v"(b));)
DEFK(k_mul_lo_u32, asm volatile("v_mul_lo_u32 %0, %1, %2" : "=v"(o32) : "v"(a), "v"(b));)
DEFK(k_mul_u24, asm volatile("v_mul_u32_u24 %0, %1, %2" : "=v"(o32) : "v"(a), "v"(b));)
DEFK(k_bitop3, asm volatile("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(o32) : "v"(a), "v"(b), "v"(c));)
DEFK(k_fma_f32, asm volatile("v_fma_f32 %0, %1, %2, %3" : "=v"(of) : "v"(fa), "v"(fb), "v"(fc));)
DEFK(k_pk_fma, asm volatile("v_pk_fma_f32 %0, %1, %2, %3" : "=v"(o64) : "v"(da), "v"(db), "v"(da));)
DEFK(k_pk_mul, asm volatile("v_pk_mul_f32 %0, %1, %2" : "=v"(o64) : "v"(da), "v"(db));)
DEFK(k_pk_add, asm volatile("v_pk_add_f32 %0, %1, %2" : "=v"(o64) : "v"(da), "v"(db));)
DEFK(k_fma_mix, asm volatile("v_fma_mix_f32 %0, %1, 1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "=v"(of) : "v"(a), "v"(fb));)
DEFK(k_sqrt_f32, asm volatile("v_sqrt_f32 %0, %1" : "=v"(of) : "v"(fa));)
DEFK(k_rcp_f32, asm volatile("v_rcp_f32 %0, %1" : "=v"(of) : "v"(fa));)
DEFK(k_cvt_i32_f32, asm volatile("v_cvt_i32_f32 %0, %1" : "=v"(o32) : "v"(fa));)
DEFK(k_med3_f32, asm volatile("v_med3_f32 %0, %1, %2, %3" : "=v"(of) : "v"(fa), "v"(fb), "v"(fc));)
DEFK(k_add_f64, asm volatile("v_add_f64 %0, %1, %2" : "=v"(od) : "v"(da), "v"(db));)
DEFK(k_fma_f64, asm volatile("v_fma_f64 %0, %1, %2, %1" : "=v"(od) : "v"(da), "v"(db));)
DEFK(k_rcp_f64, asm volatile("v_rcp_f64 %0, %1" : "=v"(od) : "v"(da));)
DEFK(k_cvt_f64_f32, asm volatile("v_cvt_f64_f32 %0, %1" : "=v"(od) : "v"(fa));)
DEFK(k_mov_dpp, asm volatile("v_mov_b32_dpp %0, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "=v"(o32) : "v"(a));)
DEFK(k_max_dpp, asm volatile("v_max_i32_dpp %0, %1, %2 row_shr:1 row_mask:0xf bank_mask:0xf" : "=v"(o32) : "v"(a), "v"(b));)
DEFK(k_readlane, asm volatile("v_readlane_b32 %0, %1, 5" : "=s"(o32) : "v"(a));)
DEFK(k_cvt_pk_f16, asm volatile("v_cvt_pk_f16_f32 %0, %1, %2" : "=v"(o32) : "v"(fa), "v"(fb));)
DEFK(k_cndmask, asm volatile("v_cndmask_b32 %0, %1, %2, vcc" : "=v"(o32) : "v"(a), "v"(b));)
DEFK(k_cmp_u32, asm volatile("v_cmp_eq_u32 vcc, %0, %1" :: "v"(a), "v"(b) : "vcc");)
DEFK(k_cmp_e64, asm volatile("v_cmp_eq_u32 %0, %1, %2" : "=s"(o64) : "v"(a), "v"(b));)

DEFK(k_add_f32, asm volatile("v_add_f32 %0, %1, %2" : "=v"(of) : "v"(fa), "v"(fb));)
DEFK(k_mul_f32, asm volatile("v_mul_f32 %0, %1, %2" : "=v"(of) : "v"(fa), "v"(fb));)
DEFK(k_fma_f32_s, asm volatile("v_fma_f32 %0, %1, %2, %3" : "=v"(of) : "v"(fa), "s"(fc), "v"(fb));)
DEFK(k_mov_b32, asm volatile("v_mov_b32 %0, %1" : "=v"(o32) : "v"(a));)
DEFK(k_cnd_e64, asm volatile("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(o32) : "v"(a), "v"(b), "s"(m64));)
DEFK(k_cmp_cnd, asm volatile("v_cmp_gt_u32 vcc, %1, %2\n\tv_cndmask_b32 %0, %1, %2, vcc" : "=v"(o32) : "v"(a), "v"(b) : "vcc");)
DEFK(k_cmp_cnd_s, asm volatile("v_cmp_gt_u32 %0, %2, %3\n\tv_cndmask_b32_e64 %1, %2, %3, %0" : "=&s"(o64), "=v"(o32) : "v"(a), "v"(b));)
DEFK(k_add_u32, asm volatile("v_add_u32 %0, %1, %2" : "=v"(o32) : "v"(a), "v"(b));)
DEFK(k_and_b32, asm volatile("v_and_b32 %0, %1, %2" : "=v"(o32) : "v"(a), "v"(b));)
DEFK(k_xor_b32, asm volatile("v_xor_b32 %0, %1, %2" : "=v"(o32) : "v"(a), "v"(b));)
DEFK(k_or3_b32, asm volatile("v_or3_b32 %0, %1, %2, %3" : "=v"(o32) : "v"(a), "v"(b), "v"(c));)
DEFK(k_lshl_add, asm volatile("v_lshl_add_u32 %0, %1, 2, %2" : "=v"(o32) : "v"(a), "v"(b));)
DEFK(k_alignbit, asm volatile("v_alignbit_b32 %0, %1, %2, 11" : "=v"(o32) : "v"(a), "v"(b));)
DEFK(k_max_i32, asm volatile("v_max_i32 %0, %1, %2" : "=v"(o32) : "v"(a), "v"(b));)
DEFK(k_add3_u32, asm volatile("v_add3_u32 %0, %1, %2, %3" : "=v"(o32) : "v"(a), "v"(b), "v"(c));)
DEFK(k_mad_u24, asm volatile("v_mad_u32_u24 %0, %1, %2, %3" : "=v"(o32) : "v"(a), "v"(b), "v"(c));)
DEFK(k_cvt_f32_u32, asm volatile("v_cvt_f32_u32 %0, %1" : "=v"(of) : "v"(a));)
DEFK(k_cvt_f32_f16, asm volatile("v_cvt_f32_f16 %0, %1" : "=v"(of) : "v"(a));)
DEFK(k_mul_f64, asm volatile("v_mul_f64 %0, %1, %2" : "=v"(od) : "v"(da), "v"(db));)
DEFK(k_floor_f64, asm volatile("v_floor_f64 %0, %1" : "=v"(od) : "v"(da));)
DEFK(k_exp_f32, asm volatile("v_exp_f32 %0, %1" : "=v"(of) : "v"(fa));)
DEFK(k_cmp_f32_s, asm volatile("v_cmp_gt_f32 %0, %1, %2" : "=s"(o64) : "v"(fa), "v"(fb));)
DEFK(k_rfl, asm volatile("v_readfirstlane_b32 %0, %1" : "=s"(o32) : "v"(a));)
DEFK(k_perm, asm volatile("v_perm_b32 %0, %1, %2, %3" : "=v"(o32) : "v"(a), "v"(b), "v"(c));)
DEFK(k_bfe, asm volatile("v_bfe_u32 %0, %1, 3, 10" : "=v"(o32) : "v"(a));)
DEFK(k_pk_fma_sel, asm volatile("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[1,0,1]" : "=v"(o64) : "v"(da), "v"(db), "v"(da));)
DEFK(k_fma_pair, asm volatile("v_fma_f32 %0, %1, %2, %3\n\tv_fma_f32 %0, %2, %3, %1" : "=&v"(of) : "v"(fa), "v"(fb), "v"(fc));)
DEFK(k_mad_mix2, asm volatile("v_mad_u64_u32 %0, s[0:1], %2, %3, 0\n\tv_fma_f32 %1, %4, %5, %4" : "=&v"(o64), "=&v"(of) : "v"(a), "v"(b), "v"(fa), "v"(fb) : "s0", "s1");)
DEFK(k_dpp_add, asm volatile("v_add_f32_dpp %0, %1, %2 row_shr:1 row_mask:0xf bank_mask:0xf" : "=v"(of) : "v"(fa), "v"(fb));)

typedef void (*Kfn)(uint64_t*, uint32_t);
struct Entry {
  const char* name;
  Kfn fn;
};

int main() {
  const Entry ks[] = {
      {"v_mad_u64_u32", k_mad_u64},   {"v_mul_hi_u32", k_mul_hi_u32}, {"v_mul_lo_u32", k_mul_lo_u32},
      {"v_mul_u32_u24", k_mul_u24},   {"v_bitop3_b32", k_bitop3},     {"v_fma_f32", k_fma_f32},
      {"v_pk_fma_f32", k_pk_fma},     {"v_pk_mul_f32", k_pk_mul},     {"v_pk_add_f32", k_pk_add},
      {"v_fma_mix_f32", k_fma_mix},   {"v_sqrt_f32", k_sqrt_f32},     {"v_rcp_f32", k_rcp_f32},
      {"v_cvt_i32_f32", k_cvt_i32_f32}, {"v_med3_f32", k_med3_f32},   {"v_add_f64", k_add_f64},
      {"v_fma_f64", k_fma_f64},       {"v_rcp_f64", k_rcp_f64},       {"v_cvt_f64_f32", k_cvt_f64_f32},
      {"v_mov_b32_dpp", k_mov_dpp},   {"v_max_i32_dpp", k_max_dpp},   {"v_readlane_b32", k_readlane},
      {"v_cvt_pk_f16_f32", k_cvt_pk_f16}, {"v_cndmask_b32", k_cndmask}, {"v_cmp_eq_u32 (vcc)", k_cmp_u32},
      {"v_cmp_eq_u32 (sgpr)", k_cmp_e64},
      {"v_add_f32", k_add_f32}, {"v_mul_f32", k_mul_f32}, {"v_fma_f32 (sgpr src)", k_fma_f32_s},
      {"v_mov_b32", k_mov_b32}, {"v_cndmask_b32_e64 (s mask)", k_cnd_e64}, {"cmp+cndmask vcc (2 ins)", k_cmp_cnd},
      {"cmp+cndmask sgpr (2 ins)", k_cmp_cnd_s}, {"v_add_u32", k_add_u32}, {"v_and_b32", k_and_b32},
      {"v_xor_b32", k_xor_b32}, {"v_or3_b32", k_or3_b32}, {"v_lshl_add_u32", k_lshl_add},
      {"v_alignbit_b32", k_alignbit}, {"v_max_i32", k_max_i32}, {"v_add3_u32", k_add3_u32},
      {"v_mad_u32_u24", k_mad_u24}, {"v_cvt_f32_u32", k_cvt_f32_u32}, {"v_cvt_f32_f16", k_cvt_f32_f16},
      {"v_mul_f64", k_mul_f64}, {"v_floor_f64", k_floor_f64}, {"v_exp_f32", k_exp_f32},
      {"v_cmp_gt_f32 (sgpr)", k_cmp_f32_s}, {"v_readfirstlane_b32", k_rfl}, {"v_perm_b32", k_perm},
      {"v_bfe_u32", k_bfe}, {"v_pk_fma_f32 op_sel_hi", k_pk_fma_sel}, {"2x v_fma_f32 dep (2 ins)", k_fma_pair},
      {"mad_u64 + fma_f32 (2 ins)", k_mad_mix2}, {"v_add_f32_dpp", k_dpp_add},
  };
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, 0) != hipSuccess) return 1;
  const int cus = prop.multiProcessorCount;
  uint64_t* d = nullptr;
  const int maxblk = cus * 4;  // 4 blocks of 4 waves per CU = 4 waves per SIMD
  if (hipMalloc(&d, sizeof(uint64_t) * maxblk * 4) != hipSuccess) return 1;
  std::vector<uint64_t> h(maxblk * 4);
  printf("CUs %d; cycles per wave-instruction per SIMD (s_memtime), 16 independent copies x %d rounds\n", cus, kRounds);
  printf("%-24s %10s %10s\n", "instruction", "1 wave/SIMD", "4 waves/SIMD");
  for (const Entry& e : ks) {
    double r[2];
    for (int v = 0; v < 2; ++v) {
      const int wps = v ? 4 : 1;
      const int blocks = cus * wps;  // one block of 4 waves per CU = one wave per SIMD
      e.fn<<<blocks, 256>>>(d, 12345u);  // warm
      e.fn<<<blocks, 256>>>(d, 777u);
      if (hipDeviceSynchronize() != hipSuccess) return 2;
      hipMemcpy(h.data(), d, sizeof(uint64_t) * blocks * 4, hipMemcpyDeviceToHost);
      std::vector<uint64_t> v2(h.begin(), h.begin() + blocks * 4);
      std::sort(v2.begin(), v2.end());
      const double med = (double)v2[v2.size() / 2];
      r[v] = med / (16.0 * kRounds) / wps;
    }
    printf("%-24s %10.2f %10.2f\n", e.name, r[0], r[1]);
  }
  hipFree(d);
  return 0;
}
