// pf_rng.hpp — random streams of the PF step, usable on host and device.
//
// Two streams (DESIGN.md "RNG"):
//  * reference: the reference seeds `std::default_random_engine generator(rd())` per frame (PE:476-477)
//    and draws uniform_real_distribution<double> values from it in a fixed order (PE:563-587, PE:671).
//    default_random_engine is minstd_rand0 (x <- 16807 x mod 2^31-1, libstdc++ bits/random.h:1555,1604);
//    every double draw consumes TWO engine outputs (generate_canonical with R = 2^31-2, k = 2,
//    bits/random.tcc:3348-3376) and maps u*(b-a)+a (bits/random.h:1870).  Because the engine is an LCG,
//    the j-th output is a^j * x0 mod m, so any particle's draws are reachable by O(log j) jump-ahead and
//    the device reproduces the reference stream bit-for-bit, in parallel.
//  * philox: counter-based Philox4x32-10 (Salmon et al., SC'11), counter = (particle, iter|tag<<24,
//    frame_lo, frame_hi), key = (seed_lo, seed_hi).  Stateless, so propagated particles are never
//    stored: they are regenerated from (prior[n], counter) wherever they are needed.
//
// This translation unit is compiled with -ffp-contract=off: double arithmetic here is plain IEEE
// mul/add, the same roundings as the reference's x86-64 build.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define PF_HD __host__ __device__ __forceinline__
#else
#define PF_HD inline
#endif

namespace pfmpe {

// ------------------------------------------------------------------------------------ minstd_rand0
constexpr uint32_t kLcgA = 16807u;
constexpr uint32_t kLcgM = 2147483647u;  // 2^31 - 1 (prime)

PF_HD uint32_t mulmod_m31(uint32_t a, uint32_t b) {
  const uint64_t p = (uint64_t)a * (uint64_t)b;  // < 2^62
  uint64_t r = (p & kLcgM) + (p >> 31);          // < 2^32
  r = (r & kLcgM) + (r >> 31);                   // <= 2^31
  return (uint32_t)(r >= kLcgM ? r - kLcgM : r);
}

// a^e mod m, e reduced mod (m-1) (Fermat: a^(m-1) = 1)
PF_HD uint32_t powmod_a(uint64_t e) {
  e %= (uint64_t)(kLcgM - 1u);
  uint32_t result = 1u, base = kLcgA;
  while (e) {
    if (e & 1u) result = mulmod_m31(result, base);
    base = mulmod_m31(base, base);
    e >>= 1;
  }
  return result;
}

// linear_congruential_engine::seed(s) (bits/random.tcc:117-124): x0 = s mod m, 0 -> 1
PF_HD uint32_t lcg_seed(uint32_t s) {
  const uint32_t x = s % kLcgM;
  return x == 0u ? 1u : x;
}

// engine output number j (1-based): a^j x0 mod m
PF_HD uint32_t lcg_output(uint32_t x0, uint64_t j) { return mulmod_m31(powmod_a(j), x0); }

PF_HD uint32_t lcg_next(uint32_t x) { return mulmod_m31(x, kLcgA); }

// generate_canonical<double,53>(g) from two consecutive outputs g1, g2 (bits/random.tcc:3348-3376):
//   sum = (g1-1)*1 + (g2-1)*R ; tmp = (double)(R*R as long double) ; ret = sum/tmp ; ret<1
// R = 2147483646; R*R = 2^62 - 2^33 + 4 rounds to the double 2^62 - 2^33 = 4611686009837453312.
PF_HD double ref_canonical(uint32_t g1, uint32_t g2) {
  double sum = (double)(g1 - 1u);
  const double t = (double)(g2 - 1u) * 2147483646.0;
  sum = sum + t;
  double ret = sum / 4611686009837453312.0;
  if (ret >= 1.0) ret = 0x1.fffffffffffffp-1;  // nextafter(1, 0)
  return ret;
}

// uniform_real_distribution<double>(a,b)(g) (bits/random.h:1870)
PF_HD double ref_uniform(double u, double a, double b) { return u * (b - a) + a; }

// ------------------------------------------------------------------------------------ Philox4x32-10
struct U32x4 {
  uint32_t x, y, z, w;
};

// a ^ b ^ k in ONE instruction on the device: gfx950's three-input bitwise op (truth table 0x96 = xor3), the
// round key k an SGPR operand
PF_HD uint32_t xor3_key(uint32_t a, uint32_t b, uint32_t k) {
#if defined(__HIP_DEVICE_COMPILE__)
  uint32_t r;
  asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(a), "v"(b), "s"(k));
  return r;
#else
  return a ^ b ^ k;
#endif
}

// The key must be wave-uniform (every call site passes the frame's seed).  On the device the round keys are
// derived from the key right here by scalar adds: the empty asm keeps the compiler from hoisting all twenty
// of them out of the streaming loops, where they held 20 SGPRs, spilled to VGPR lanes and cost a
// v_readlane + s_nop per use; the two per-round xors are one v_bitop3 (10 rounds: 20 v_mad_u64_u32 +
// 20 v_bitop3 per call, round keys on the scalar unit).
PF_HD U32x4 philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1) {
#if defined(__HIP_DEVICE_COMPILE__)
  asm volatile("" : "+s"(k0), "+s"(k1));
#endif
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    if (r) {
      k0 += 0x9E3779B9u;
      k1 += 0xBB67AE85u;
    }
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    const uint32_t n0 = xor3_key((uint32_t)(p1 >> 32), c1, k0);
    const uint32_t n1 = (uint32_t)p1;
    const uint32_t n2 = xor3_key((uint32_t)(p0 >> 32), c3, k1);
    const uint32_t n3 = (uint32_t)p0;
    c0 = n0; c1 = n1; c2 = n2; c3 = n3;
  }
  return U32x4{c0, c1, c2, c3};
}

// 24-bit uniform in [0,1): exactly representable in float and double
PF_HD float u24f(uint32_t x) { return (float)(x >> 8) * (1.0f / 16777216.0f); }
PF_HD double u24d(uint32_t x) { return (double)(x >> 8) * (1.0 / 16777216.0); }
// 53-bit uniform in [0,1)
PF_HD double u53(uint32_t x0, uint32_t x1) {
  return ((double)(x0 >> 5) * 67108864.0 + (double)(x1 >> 6)) * (1.0 / 9007199254740992.0);
}

enum : uint32_t { kTagMotion = 0u, kTagResample = 2u };

// Motion draws: ONE Philox4x32-10 call per (particle, iteration) yields the six 21-bit uniforms
// (angX, angY, angZ, tX, tY, tZ): the top 21 bits of each output word, then two more built from the
// low 11 bits.  k * 2^-21 is exact in float and double.
struct Draws6 {
  uint32_t v[6];
};
PF_HD Draws6 philox_motion6(uint32_t n, uint32_t iter, uint32_t flo, uint32_t fhi, uint32_t k0, uint32_t k1) {
  const U32x4 o = philox4x32_10(n, iter | (kTagMotion << 24), flo, fhi, k0, k1);
  Draws6 d;
  d.v[0] = o.x >> 11;
  d.v[1] = o.y >> 11;
  d.v[2] = o.z >> 11;
  d.v[3] = o.w >> 11;
  d.v[4] = ((o.x & 0x7FFu) << 10) | (o.y & 0x3FFu);
  d.v[5] = ((o.z & 0x7FFu) << 10) | (o.w & 0x3FFu);
  return d;
}
PF_HD float u21f(uint32_t v) { return (float)v * (1.0f / 2097152.0f); }
PF_HD double u21d(uint32_t v) { return (double)v * (1.0 / 2097152.0); }

}  // namespace pfmpe
