// pf_kernels.hpp — HIP kernels of the PF step for gfx950 (MI355X, CDNA4, wave64).
//
// One frame (reference PE:475-733) is two launches:
//
//   k_propagate_weigh  one particle per thread.  Per block: an x-bucketed blob table in LDS; per
//                      particle the motion model (PE:543-588) -> projection of M markers (PE:1017) ->
//                      likelihood (PE:2385) -> weight.  Per-block partials are handed (write-through,
//                      counter) to the last block of each 64-block GROUP, whose wave scans the group;
//                      group partials go to the last group, whose wave does the iteration bookkeeping
//                      and exit rule (PE:606-616) and, on the final iteration, the normaliser S, the
//                      group prefixes and the accept test (PE:627-633).  Re-launched only if the exit
//                      rule did not fire (rare in steady state).
//   k_resample         stratified resampling (PE:666-682) as a parallel scan + target count per
//                      particle + wave-cooperative scatter of the kept particles into the new prior.
//                      Count partials go up the same 2-level tree; the last group's wave picks the
//                      winner = argmax count (PE:685-688), computes its pose and pairs and writes the
//                      frame record straight into pinned host memory.
//
// The one-launch frames (k_frame, k_frame2) keep the propagated particle in registers, so their HBM
// traffic per particle-update is the compulsory 3*S + 8 bytes (S = 48 B for fp32 SoA state; DESIGN.md
// "Roofline").  The two-launch path, which is VALU-issue bound at large N, by default stores each
// iteration's propagated set next to its weights (PFMPE_OPT_KEEP_PROPAGATED; +2*S bytes) and k_resample
// gathers it, instead of regenerating it (motion model + RNG) from (prior[n], RNG counter).
//
// Normalised cumulative weight (DESIGN.md "Exact tiling of the stratified targets"): for particle i of
// block b in group g,   c_i = fl( fl( G_g + fl( E_b + incl_i ) ) / S )
// with incl_i the in-block prefix, E_b the in-group exclusive prefix and G_g the group prefix.  For a
// fixed (g, S) c_i is monotone in fl(E_b + incl_i), so every running maximum the resampler needs at a
// block boundary is composed EXACTLY (max has no rounding) from group-local max-scans: the slot ranges
// of all particles tile [0, N) with no gap and no overlap.
#pragma once
#include <hip/hip_runtime.h>
#include <float.h>
#include <math.h>
#include <stddef.h>
#include <stdint.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <type_traits>
#include <vector>

#include <hip/hip_fp16.h>

#include "pf_rng.hpp"
#include "pf_desc_tag.hpp"

namespace pfmpe {

constexpr int kBlock = 256;            // particles per block (4 waves)
constexpr int kWaves = kBlock / 64;
// Blocks per reduction group: ~sqrt(blocks), at most kGroup (one per lane of the group wave).  Arrival
// counters are agent-scope atomics that execute at the memory side and serialise per address (~25 ns
// each), so sqrt balances the group counters against the top counter (a single 391-way counter cost
// ~10 us at C2).  A grid of one group skips the top counter: its group wave is the top wave.
constexpr int kGroup = 64;
constexpr int kMaxMarkers = 16;
constexpr int kMaxBlobs = 1024;
constexpr int kMaxBuckets = 512;       // x-buckets of the blob table (see bucket_count)
constexpr int kMaxIter = 4096;         // PF iterations per frame (reference: 80); < 2^16 for k_frame's release tags
constexpr int kPlanes = 12;            // r00 r01 r02 t0 r10 r11 r12 t1 r20 r21 r22 t2

enum : int { kRngReference = 0, kRngPhilox = 1 };

// Marker-count buckets (pfmpe_ctx.hpp dispatch_m / multi_m): the per-particle loops are unrolled to MAXM slots.
// The 5-slot bucket serves exactly M == 5 (the README object: C1, C2, C4, C5), so its "slot j holds a marker"
// tests are compile-time true: no per-marker lane masks live across the streaming loops (they held SGPR pairs
// spilled to VGPR lanes, a v_readlane pair per use).  The other buckets test j < M.
constexpr int kExactM = 5;
template <int MAXM>
__host__ __device__ __forceinline__ bool marker_live(int j, int M) {
  return MAXM == kExactM ? j < kExactM : j < M;
}

// ----------------------------------------------------------------------------- kernel arguments
// Passed by value (kernarg segment -> scalar loads), pre-converted to the compute type T on the host.
// The frame's 2D blob grid as kernel arguments (scalar registers, reloadable from the kernarg segment /
// stream descriptor instead of held in VGPRs): build_blob_table_host's GridHdr plus the byte offsets of the
// grid's parts in the table; on = 0 when the table has no grid or one built for a narrower window.
// one 2D-grid list entry of a blob table (build_blob_table_host): position and original index, one ds_read_b128
struct alignas(16) GridEnt {
  float x, y;
  int32_t orig, pad;
};
struct GridArgs {
  float inv_c, ox, oy, pad0;       // cell of (u, v): (fma(u, inv_c, ox), fma(v, inv_c, oy)), clamped, truncated;
                                   // ox = -gx0 * inv_c (square cells)
  float fmaxx, fmaxy;              // ncx - 1, ncy - 1
  int32_t ncx4, on;               // 4 * ncx: the cell row pitch in bytes
  int32_t cell_off, ent_off;      // table offsets: uint32 cell[], GridEnt ent[]
  int32_t b0fin;                  // blob 0 of the table is finite (set whether or not the grid is on)
  int32_t pad2;
};

template <typename T>
struct FrameArgsT {
  T cur[12], pred[12], predm[12], cam[12];  // 3x4 row-major
  T markers[kMaxMarkers * 3];
  T K[9];
  T lo[6], hi[6];           // draw ranges angX angY angZ tX tY tZ (scaled by fac*), Philox stream
  T rgs[6];                 // (hi - lo) * 2^-21: hi - lo rounded once on the host, then scaled exactly (Philox draw
                            // lo + u21 * (hi - lo) with u21 = v * 2^-21, computed as v * rgs: the same product)
  double dlo[6], dhi[6];    // the same in double, reference stream (draws are computed in double)
  double growth;            // 0.025
  T tol, tol_pf, tolq;      // score normaliser / acceptance gate / pruning half-window
  double exit_thr, accept_thr;
  uint32_t key0, key1, flo, fhi;  // philox key / frame counter
  uint32_t lcg_x0;                // reference engine state after seeding
  uint32_t downgrade;             // bit j: marker j downgraded
  int32_t N, M, B, it;            // particles, markers, blobs, it_since_initialized_
  int32_t cam_identity, max_iter, force_iters, nblk;
  int32_t ngrp, gsz;              // reduction groups and blocks per group (~sqrt(nblk), <= kGroup)
  int32_t diag;                   // diagnostic switches (0 in production; pfmpe_ctx.hpp kDiag*)
  int32_t small_angles;           // every angle draw of the frame has |x| <= kSmallAngle (host bound, fp32)
  int32_t k_upper;                // K = [k0 k1 k2; 0 k4 k5; 0 0 1] (host check; fp32 skips the zero terms)
  uint32_t wait_ticks;            // bound of every in-launch wait, s_memrealtime ticks (100 MHz)
  uint32_t flat_base_w, flat_base_c;  // k_frame2: running totals of the flat counter sets at frame start
  int32_t tbytes;                 // this frame's blob table, bytes (base + grid: build_blob_table_host)
  uint32_t gtag;                  // k_frame2: this frame's granule tag base (frame << 12; the iteration in the low
                                  // 12 bits), never 0 (pfmpe_ctx.hpp next_gtag)
  GridArgs grid;                  // the table's 2D grid (fp32 pruned column minima)
  int64_t ld;                     // SoA plane stride in elements
  T anc_in[12], anc_out[12];      // fp16 state only: anchors of the prior / of the new prior
  // Deferred resampling: the prior may be stored as an earlier frame's kept propagated set plus
  // owner indices, prior particle n = stored particle owner[n] (null: stored in particle order).  owner_out
  // (two-launch frames with the kept set): k_resample writes the new prior's owner indices there instead of
  // gathering and scattering the particles (null: the new prior is materialised in the post buffer).
  const uint32_t* owner;
  uint32_t* owner_out;
};

// The frame-constant arrays, staged once per block into LDS and read from there (broadcast reads):
// kept in SGPRs they would spill into VGPR lanes and cap residency (MI355X_MICROARCH.md "Residency").
template <typename T>
struct LdsConst {
  T cur[12], pred[12], predm[12], cam[12];
  T markers[kMaxMarkers * 3];
  T K[9];
  T lo[6], hi[6];
  T rgs[6];
};

// Per-frame control record.  All-zero is the valid "start of frame" state (zeroed at create, set_prior
// and by the final wave of every frame).
struct Ctrl {
  double best_max;   // highestProb
  double S;          // probPartSum of the kept iteration
  double invS;       // fl(1 / S): k_resample's divisions by S as a product and two fma corrections (div_by_S)
  int32_t done, has_best, best_idx, best_iter, best_slot, cur_slot;
  int32_t iters, kept_slot, kept_iter, accepted, most_likely_idx, pad0;
  int64_t K_total;   // number of stratified targets that find a particle
};

// per block, per weight slot (written and read write-through)
struct alignas(16) BlockPart {
  double sum;             // block total (in-block scan order)
  double maxrel, minrel;  // extrema of the in-block inclusive prefix sums
  double maxw, minw;      // max / min weight
  int32_t argmax, argmin;
};
// per group, per weight slot (write-through)
struct alignas(16) GroupPart {
  double sum;          // group total
  double zmax, zmin;   // max / min over the group of fl(E_b + incl_i)
  double maxw, minw;
  int32_t argmax, argmin;
};
// per block, per weight slot: in-group exclusive prefix E_b and exclusive max/min of z (for k_resample)
struct alignas(16) BlockScan {
  double E, zin_max, zin_min, pad;
};
// per group, kept slot only: group prefix G_g and running max of c at the group start
struct alignas(16) GroupScan {
  double G, Gin;
};
struct alignas(8) CountPart {
  int32_t maxcount, idx;
};
// winner keys of the one-stream two-launch frame (k_resample -> k_resample_final): unsigned max of
// count << 32 | (2^31 - 1 - index) is the max count at its lowest index; 0 (count 0 at no index) is the identity
constexpr int kWinShards = 64;
constexpr int kWinStride = 16;  // keys one 128-B line apart: ~39k block atomics at C4 spread over 64 lines
// the key area: the key shards, then as many arrival shards of the fused finish (k_resample_owners), each counter at
// the start of its own 128-B line (one memory-side atomic unit serialises ~25 ns per arrival on one address: one
// counter for C4's 39k blocks took 400 us)
constexpr size_t kWinBytes = (size_t)(2 * kWinShards) * kWinStride * sizeof(unsigned long long);
__host__ __device__ __forceinline__ uint32_t* win_arrive(unsigned long long* winkey) {
  return (uint32_t*)(winkey + kWinShards * kWinStride);
}
constexpr int kArriveStride = 2 * kWinStride;  // uint32 words between arrival shards (128 B)
__host__ __device__ __forceinline__ unsigned long long win_key(int count, int idx) {
  return ((unsigned long long)(uint32_t)count << 32) | (uint32_t)(0x7fffffff - idx);
}

// frame record written by the final wave into pinned host memory: the pfmpe_frame_out layout, then the
// kept slot and the publication tag (2 * frame sequence + finished)
struct OutDev {
  int32_t iters, kept_iter, most_likely_idx, accepted, resampled, winner_idx, n_corr, flag_fail;
  double highest_prob, prob_sum;
  double winner_pose[12], most_likely_pose[12];
  uint32_t corr[2 * kMaxMarkers];
  int32_t kept_slot;
  int32_t tag;
};
// The record as the kernel publishes it: data-tagged granules (MI355X_MICROARCH.md "handoff-1to1"), 8-byte
// words {OutDev word k (low 32 bits), tag (high 32)}, each ONE relaxed system-scope store, so the host has
// the whole record once every granule carries the current tag, and the final wave needs no release (no
// wait for the PCIe write acknowledgements).  An unfinished iteration batch (two-launch path) writes
// granule 0 alone, with tag 2 * seq.
constexpr int kRecWords = (int)(offsetof(OutDev, tag) / 4);
constexpr int kRecGran = 128;
static_assert(offsetof(OutDev, tag) % 4 == 0 && kRecWords <= kRecGran && kRecWords > 64, "record granules");
struct RecOut {
  uint64_t g[kRecGran];
};

// ----------------------------------------------------------------------------- scalar helpers
__device__ __forceinline__ float fmadd(float a, float b, float c) { return __builtin_fmaf(a, b, c); }
// fp64: deliberately UNFUSED (TU built with -ffp-contract=off): a*b rounded, then +c rounded, the
// reference's x86-64 arithmetic.
__device__ __forceinline__ double fmadd(double a, double b, double c) { return a * b + c; }
// fp32: the motion noise angles are tiny (|x| <= 0.015 * 1.x rad with README parameters), so a short
// Taylor polynomial is accurate to float rounding there; larger angles take sincosf.
__device__ __forceinline__ void sincos_t(float x, float* s, float* c) {
  if (fabsf(x) <= 0.25f) {
    const float x2 = x * x;
    *s = x * fmadd(x2, fmadd(x2, fmadd(x2, fmadd(x2, 1.0f / 362880.0f, -1.0f / 5040.0f), 1.0f / 120.0f),
                             -1.0f / 6.0f), 1.0f);
    *c = fmadd(x2, fmadd(x2, fmadd(x2, fmadd(x2, 1.0f / 40320.0f, -1.0f / 720.0f), 1.0f / 24.0f), -0.5f), 1.0f);
  } else {
    sincosf(x, s, c);
  }
}
// |x| <= kSmallAngle (the host proves it for every angle draw of a frame: FrameArgsT::small_angles): the
// next Taylor terms are below half an fp32 ulp there (x^5/120 / x <= 6.8e-9, x^6/720 <= 1e-12)
constexpr float kSmallAngle = 0.03f;
__device__ __forceinline__ void sincos_small(float x, float* s, float* c) {
  const float x2 = x * x;
  *s = x * fmadd(x2, -1.0f / 6.0f, 1.0f);
  *c = fmadd(x2, fmadd(x2, 1.0f / 24.0f, -0.5f), 1.0f);
}
__device__ __forceinline__ void sincos_t(double x, double* s, double* c) {
  *s = sin(x);
  *c = cos(x);
}
__device__ __forceinline__ void sincos_small(double x, double* s, double* c) { sincos_t(x, s, c); }  // fp64: exact path
// fp32: the hardware square root (v_sqrt_f32, 1 ulp) instead of sqrtf's correctly rounded 14-instruction
// sequence (tolerance path, like div_t); fp64 stays IEEE
// max / min for the wave extrema (operands are never NaN: weights are finite, identities are +-inf)
__device__ __forceinline__ float fmax_t(float a, float b) { return __builtin_fmaxf(a, b); }
__device__ __forceinline__ double fmax_t(double a, double b) { return __builtin_fmax(a, b); }
__device__ __forceinline__ float fmin_t(float a, float b) { return __builtin_fminf(a, b); }
__device__ __forceinline__ double fmin_t(double a, double b) { return __builtin_fmin(a, b); }
__device__ __forceinline__ float sqrt_t(float x) { return __builtin_amdgcn_sqrtf(x); }
__device__ __forceinline__ double sqrt_t(double x) { return sqrt(x); }
// fp32 quotient a/b through the hardware reciprocal (v_rcp_f32, 1 ulp): one instruction instead of the
// ~10-instruction IEEE division sequence; the fp32 path is a tolerance path, fp64 divides
// exactly
__device__ __forceinline__ float rcp_t(float b) { return __builtin_amdgcn_rcpf(b); }
__device__ __forceinline__ float div_t(float a, float b) { return a * __builtin_amdgcn_rcpf(b); }
__device__ __forceinline__ double div_t(double a, double b) { return a / b; }
// perspective division: fp32 uses one hardware reciprocal, fp64 the exact IEEE quotient (PE:1032)
__device__ __forceinline__ void persp(float p0, float p1, float p2, float* u, float* v) {
  const float r = rcp_t(p2);
  *u = p0 * r;
  *v = p1 * r;
}
__device__ __forceinline__ void persp(double p0, double p1, double p2, double* u, double* v) {
  *u = p0 / p2;
  *v = p1 / p2;
}
template <typename T>
__device__ __forceinline__ T inf_t() {
  return (T)INFINITY;
}

// The frame-constant arrays lead FrameArgsT in exactly LdsConst's layout, and FrameArgsT is every
// kernel's first argument, so the block copies them from the kernarg segment with one vector load per
// lane (no SGPR round trip: kept in SGPRs they spill into VGPR lanes).  Callers barrier afterwards.
template <typename T>
__device__ __forceinline__ void stage_consts_from(const uint32_t* src, LdsConst<T>& sc) {
  static_assert(offsetof(FrameArgsT<T>, cur) == 0 && offsetof(FrameArgsT<T>, hi) == offsetof(LdsConst<T>, hi) &&
                    offsetof(FrameArgsT<T>, rgs) == offsetof(LdsConst<T>, rgs),
                "LdsConst must mirror the head of FrameArgsT");
  static_assert(sizeof(LdsConst<T>) % 4 == 0, "dword copy");
  uint32_t* dst = (uint32_t*)&sc;
  constexpr int kWordsC = (int)(sizeof(LdsConst<T>) / 4);
  for (int i = threadIdx.x; i < kWordsC; i += kBlock) dst[i] = src[i];
}
template <typename T>
__device__ __forceinline__ void stage_consts(const FrameArgsT<T>& fa, LdsConst<T>& sc) {
  (void)fa;
  stage_consts_from<T>((const uint32_t*)__builtin_amdgcn_kernarg_segment_ptr(), sc);
}

// ----------------------------------------------------------------------------- pose algebra
// 3x4 affine compose C = A*B with the reference's full-4x4 summation order (k = 0..3 sequential; the
// zero bottom-row terms add +0 and are skipped without changing any non-zero value).
template <typename T>
__device__ __forceinline__ void compose(const T* A, const T* B, T* C) {
#pragma unroll
  for (int i = 0; i < 3; ++i) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      T s = A[i * 4 + 0] * B[0 * 4 + j];
      s = fmadd(A[i * 4 + 1], B[1 * 4 + j], s);
      s = fmadd(A[i * 4 + 2], B[2 * 4 + j], s);
      if (j == 3) s = s + A[i * 4 + 3];
      C[i * 4 + j] = s;
    }
  }
}

typedef float f32x2 __attribute__((ext_vector_type(2)));  // packed fp32 pairs (v_pk_* forms)

// Particle state storage S for compute type T: S == T (fp32 / fp64 planes), or fp16 planes holding
// deltas to the set's anchor pose (PFMPE_STATE_F16, fp32 compute): 24 B per particle.
template <typename T, typename SP>
struct StateIO {
  static __device__ __forceinline__ T load(SP v, T) { return (T)v; }
  static __device__ __forceinline__ SP store(T v, T) { return (SP)v; }
};
template <>
struct StateIO<float, __half> {
  static __device__ __forceinline__ float load(__half v, float anchor) { return __half2float(v) + anchor; }
  static __device__ __forceinline__ __half store(float v, float anchor) { return __float2half(v - anchor); }
};

// SoA plane access through a buffer resource (cdna_hip_programming.md T8) for the fp32 / fp16 planes: every
// plane of particle n is at byte n*sizeof(SP) (one 32-bit VGPR offset shared by all 12 planes) plus the
// wave-uniform plane offset q*ld*sizeof(SP) in the SGPR soffset, so no plane costs a 64-bit VALU address
// (a flat access costs two v_mad_u64_u32 and moves per plane).  The resource covers the 12 planes
// (pfmpe_create caps 12*ld*sizeof(SP) below 4 GiB).  fp64 (the parity mode) keeps flat accesses.
template <typename SP>
struct BufPlanes : std::false_type {};
template <>
struct BufPlanes<float> : std::true_type {};
template <>
struct BufPlanes<__half> : std::true_type {};

template <typename SP>
__device__ __forceinline__ __amdgpu_buffer_rsrc_t plane_rsrc(const SP* base, int64_t ld) {
  const uint32_t bytes = (uint32_t)(12 * ld * (int64_t)sizeof(SP));
  return __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, (int)bytes, 0x00020000);
}
template <typename SP, int POL = 0>
__device__ __forceinline__ SP buf_ld(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
  if constexpr (std::is_same<SP, float>::value)
    return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, POL));
  else
    return __ushort_as_half(__builtin_amdgcn_raw_buffer_load_b16(r, voff, soff, POL));
}
// cache policy of a vector memory access: 16 = sc1 (a store writes through and drops the line from the XCD's L2)
constexpr int kPolSc1 = 16;
template <int POL = 0>
__device__ __forceinline__ void buf_st(float v, __amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), r, voff, soff, POL);
}
template <int POL = 0>
__device__ __forceinline__ void buf_st(__half v, __amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
  __builtin_amdgcn_raw_buffer_store_b16(__half_as_ushort(v), r, voff, soff, POL);
}

// fp16 state layout (PFMPE_F16_PAIRS, default 1): planes 2j and 2j + 1 interleaved as ONE plane of 32-bit pairs,
// element (q, n) at half index (q >> 1) * 2 ld + 2 n + (q & 1).  Every fp16 state access is then a 4-byte
// access per lane (6 instead of 12 VMEM instructions per particle, 256 B per wave instruction), and the pair is
// the register layout the kernels already use (RawState<__half>, store_state_words_f16).  0 keeps 12 planes of
// halves (A/B).  fp32 / fp64 planes are unchanged.
// fp32 state keeps 12 plain planes.  Round 3 also tried 6 planes of 64-bit pairs (PFMPE_F32_PAIRS): -2 us on C5's
// k_resample, +1..5 us on C3's weighing; round 4 removed it: deferred resampling (k_resample writes owner indices,
// no state planes) took away the only kernel it helped.
#ifndef PFMPE_F16_PAIRS
#define PFMPE_F16_PAIRS 1
#endif
template <typename SP>
__host__ __device__ __forceinline__ constexpr bool f16_pairs() {
  return std::is_same<SP, __half>::value && PFMPE_F16_PAIRS != 0;
}
template <typename SP>
__host__ __device__ __forceinline__ int64_t plane_index(int q, int64_t n, int64_t ld) {
  if constexpr (f16_pairs<SP>())
    return (int64_t)(q >> 1) * 2 * ld + 2 * n + (q & 1);
  else
    return (int64_t)q * ld + n;
}

// the 12 state values of particle n of a state buffer (raw SP values, no anchor / conversion).  POL kPolSc1: the
// loads bypass L1
template <typename SP, int POL = 0>
__device__ __forceinline__ void load_state_raw(const SP* __restrict__ base, int64_t ld, int n, SP* v) {
  if constexpr (f16_pairs<SP>()) {
    const __amdgpu_buffer_rsrc_t r = plane_rsrc(base, ld);
    const uint32_t pps = (uint32_t)(ld * 4);
#pragma unroll
    for (int p = 0; p < 6; ++p) {
      const uint32_t w = __builtin_amdgcn_raw_buffer_load_b32(r, (uint32_t)n * 4u, (uint32_t)p * pps, POL);
      v[2 * p] = __ushort_as_half((unsigned short)(w & 0xffffu));
      v[2 * p + 1] = __ushort_as_half((unsigned short)(w >> 16));
    }
  } else if constexpr (BufPlanes<SP>::value) {
    const __amdgpu_buffer_rsrc_t r = plane_rsrc(base, ld);
    const uint32_t ps = (uint32_t)(ld * (int64_t)sizeof(SP));
#pragma unroll
    for (int q = 0; q < 12; ++q) v[q] = buf_ld<SP, POL>(r, (uint32_t)n * (uint32_t)sizeof(SP), (uint32_t)q * ps);
  } else if constexpr (POL != 0) {
#pragma unroll
    for (int q = 0; q < 12; ++q)
      v[q] = __hip_atomic_load((const __attribute__((address_space(1))) SP*)(base + (int64_t)q * ld + n),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  } else {
#pragma unroll
    for (int q = 0; q < 12; ++q) v[q] = base[(int64_t)q * ld + n];
  }
}
// store 12 raw state values as particle k
template <typename SP>
__device__ __forceinline__ void store_state_raw(SP* __restrict__ base, int64_t ld, int k, const SP* v) {
  constexpr int pol = 0;
  if constexpr (f16_pairs<SP>()) {
    const __amdgpu_buffer_rsrc_t r = plane_rsrc((const SP*)base, ld);
    const uint32_t pps = (uint32_t)(ld * 4);
#pragma unroll
    for (int p = 0; p < 6; ++p) {
      const uint32_t w = (uint32_t)__half_as_ushort(v[2 * p]) | ((uint32_t)__half_as_ushort(v[2 * p + 1]) << 16);
      __builtin_amdgcn_raw_buffer_store_b32(w, r, (uint32_t)k * 4u, (uint32_t)p * pps, pol);
    }
  } else if constexpr (BufPlanes<SP>::value) {
    const __amdgpu_buffer_rsrc_t r = plane_rsrc((const SP*)base, ld);
    const uint32_t ps = (uint32_t)(ld * (int64_t)sizeof(SP));
#pragma unroll
    for (int q = 0; q < 12; ++q) buf_st<pol>(v[q], r, (uint32_t)k * (uint32_t)sizeof(SP), (uint32_t)q * ps);
  } else {
#pragma unroll
    for (int q = 0; q < 12; ++q) base[(int64_t)q * ld + k] = v[q];
  }
}

// fp16 planes, particle k from six words holding planes (2j, 2j + 1) in their (low, high) halves: the high half
// goes out through buffer_store_short_d16_hi, so no word is shifted first (the compiler does not select the
// _d16_hi form for a store of x >> 16).  A vector store; the "memory" clobber keeps it ordered with the
// compiler's own memory operations, and it carries its own VALU-SGPR-write -> VMEM wait states (below).
__device__ __forceinline__ void store_state_words_f16(__half* __restrict__ base, int64_t ld, int k, const uint32_t* w) {
  const __amdgpu_buffer_rsrc_t r = plane_rsrc((const __half*)base, ld);
  if constexpr (f16_pairs<__half>()) {  // the words are the layout: one dword store each
    const uint32_t pps = (uint32_t)(ld * 4);
#pragma unroll
    for (int j = 0; j < 6; ++j) __builtin_amdgcn_raw_buffer_store_b32(w[j], r, (uint32_t)k * 4u, (uint32_t)j * pps, 0);
    return;
  }
  const uint32_t ps = (uint32_t)(ld * (int64_t)sizeof(__half));
  const uint32_t voff = (uint32_t)k * 2u;
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    __builtin_amdgcn_raw_buffer_store_b16((uint16_t)w[j], r, voff, (uint32_t)(2 * j) * ps, 0);
    // s_nop 4 first: the compiler's hazard recognizer does not look inside inline asm, and the soffset /
    // resource SGPRs may have just been written by a VALU (v_readlane of a spilled SGPR), which a VMEM
    // instruction may read only 5 wait states later; without it the store used the stale offset
    asm volatile("s_nop 4\n\tbuffer_store_short_d16_hi %0, %1, %2, %3 offen" ::"v"(w[j]), "v"(voff), "s"(r),
                 "s"((uint32_t)(2 * j + 1) * ps)
                 : "memory");
  }
}

// Prefetch form (k_weigh_stream): the 12 raw plane words of particle n as 32-bit registers (fp16 values
// zero-extended), loaded by every lane without a branch.  The caller clamps the particle index into [0, N) for
// lanes past N (in_planes): the buffer resource's range check covers the VGPR offset only, not the plane offset
// in soffset, so an unclamped lane past ld read past the end of the allocation (up to a plane beyond it for the
// streaming pass's last prefetch); the loaded values of such lanes are never used.  Raw halves kept as halves were packed in pairs by the compiler right after the loads
// (v_perm), which waited for the prefetch at once; a branch around the loads made the next wait vmcnt(0).
// fp64 planes (flat accesses) keep the guarded load.
// fp16 planes: planes 2k and 2k + 1 share one register: one dword load from the pair plane (PFMPE_F16_PAIRS),
// or buffer_load_short_d16 / _d16_hi into its two halves (12 half planes), so the pair needs no packing.
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
template <typename SP>
struct RawState {
  SP v[12];
};
template <>
struct RawState<__half> {
  u16x2 p[6];
};
template <>
struct RawState<float> {
  uint32_t v[12];
};
// a particle index every plane access may use: n for n < N, else N - 1 (one v_min; see load_state_prefetch)
__device__ __forceinline__ int in_planes(int n, int N) { return (int)min((unsigned)n, (unsigned)(N - 1)); }
template <typename SP>
__device__ __forceinline__ void load_state_prefetch(const SP* __restrict__ base, int64_t ld, int n, bool want,
                                                    RawState<SP>& R) {
  if constexpr (BufPlanes<SP>::value) {
    const __amdgpu_buffer_rsrc_t r = plane_rsrc(base, ld);
    const uint32_t ps = (uint32_t)(ld * (int64_t)sizeof(SP));
    if constexpr (f16_pairs<SP>()) {  // one dword per pair plane
#pragma unroll
      for (int k = 0; k < 6; ++k)
        R.p[k] = __builtin_bit_cast(u16x2, __builtin_amdgcn_raw_buffer_load_b32(r, (uint32_t)n * 4u, (uint32_t)k * (uint32_t)(ld * 4), 0));
    } else if constexpr (sizeof(SP) == 2) {
#pragma unroll
      for (int k = 0; k < 6; ++k) {
        u16x2 x = R.p[k];
        x.x = __builtin_amdgcn_raw_buffer_load_b16(r, (uint32_t)n * 2u, (uint32_t)(2 * k) * ps, 0);
        x.y = __builtin_amdgcn_raw_buffer_load_b16(r, (uint32_t)n * 2u, (uint32_t)(2 * k + 1) * ps, 0);
        R.p[k] = x;
      }
    } else {
#pragma unroll
      for (int q = 0; q < 12; ++q) R.v[q] = __builtin_amdgcn_raw_buffer_load_b32(r, (uint32_t)n * 4u, (uint32_t)q * ps, 0);
    }
  } else {
    if (want) load_state_raw<SP>(base, ld, n, R.v);
  }
}
// StateIO::load of prefetched plane q
template <typename T, typename SP>
__device__ __forceinline__ T state_from_raw(const RawState<SP>& R, int q, T anchor) {
  if constexpr (std::is_same<SP, __half>::value)
    return StateIO<T, SP>::load(__ushort_as_half((q & 1) ? R.p[q >> 1].y : R.p[q >> 1].x), anchor);
  else if constexpr (std::is_same<SP, float>::value)
    return StateIO<T, SP>::load(__uint_as_float(R.v[q]), anchor);
  else
    return StateIO<T, SP>::load(R.v[q], anchor);
}

// prior particle n (SoA planes), loaded ahead of use so the loads overlap other work
// the stored row of prior particle n (deferred prior: its owner index)
template <typename T>
__device__ __forceinline__ int prior_row(const FrameArgsT<T>& fa, int n) {
  return fa.owner ? (int)fa.owner[n] : n;
}
template <typename T, typename SP, int POL = 0>
__device__ __forceinline__ void load_prior(const FrameArgsT<T>& fa, const SP* __restrict__ prior, int n, T* A) {
  SP v[12];
  load_state_raw<SP, POL>(prior, fa.ld, prior_row(fa, n), v);
#pragma unroll
  for (int q = 0; q < 12; ++q) A[q] = StateIO<T, SP>::load(v[q], fa.anc_in[q]);
}
// particle k of a state buffer from its pose P (quantised against the anchor `anc` for fp16 state)
template <typename T, typename SP>
__device__ __forceinline__ void store_pose(SP* __restrict__ dst, int64_t ld, int k, const T* P, const T* anc) {
  if constexpr (std::is_same<SP, __half>::value && std::is_same<T, float>::value) {
    // fp16 deltas two planes at a time: one v_pk_add_f32 (the same fp32 subtractions) and one v_cvt_pk_f16_f32
    // (round to nearest even, as __float2half) per pair, then the pair's halves as planes 2j / 2j + 1
    typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
    uint32_t w[6];
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      const f32x2 d = f32x2{P[2 * j], P[2 * j + 1]} - f32x2{anc[2 * j], anc[2 * j + 1]};
      w[j] = __builtin_bit_cast(uint32_t, __builtin_convertvector(d, f16x2));
    }
    store_state_words_f16(dst, ld, k, w);
    return;
  }
  SP v[12];
#pragma unroll
  for (int q = 0; q < 12; ++q) v[q] = StateIO<T, SP>::store(P[q], anc[q]);
  store_state_raw<SP>(dst, ld, k, v);
}

// The motion model (PE:543-588) for particle n in PF iteration `iter` from its prior pose A (loaded by
// load_prior; unused for n < 2); P receives the 3x4 pose.
template <typename T>
__device__ __forceinline__ T u21_t(uint32_t v);
template <>
__device__ __forceinline__ float u21_t<float>(uint32_t v) { return u21f(v); }
template <>
__device__ __forceinline__ double u21_t<double>(uint32_t v) { return u21d(v); }

template <typename T, int RNG>
__device__ __forceinline__ void propagate(const FrameArgsT<T>& fa, const LdsConst<T>& sc, const T* A_in, int n,
                                          int iter, T* P) {
  if (n == 0) {  // current_pose_ (PE:547)
#pragma unroll
    for (int q = 0; q < 12; ++q) P[q] = sc.cur[q];
    return;
  }
  if (n == 1) {  // predicted_pose_ (PE:551)
#pragma unroll
    for (int q = 0; q < 12; ++q) P[q] = sc.pred[q];
    return;
  }
  T A[12];
#pragma unroll
  for (int q = 0; q < 12; ++q) A[q] = A_in[q];
  if (fa.it > 1) {
    if (!fa.cam_identity) {  // camMoveInv * prior (PE:556-558)
      T X[12];
      compose(sc.cam, A, X);
#pragma unroll
      for (int q = 0; q < 12; ++q) A[q] = X[q];
    }
    if ((iter % 10) != 0) {  // ... * predictionMatrix (PE:556)
      T X[12];
      compose(A, sc.predm, X);
#pragma unroll
      for (int q = 0; q < 12; ++q) A[q] = X[q];
    }
  }
  // draws in reference order: angX, angY, angZ, tX, tY, tZ (PE:563-587)
  const double gd = 1.0 + fa.growth * (double)(iter / 10);
  T d[6];
  if (RNG == kRngReference) {
    const uint64_t before = 12u * ((uint64_t)(fa.N - 2) * (uint64_t)iter + (uint64_t)(n - 2));
    uint32_t g = lcg_output(fa.lcg_x0, before + 1u);
#pragma unroll
    for (int q = 0; q < 6; ++q) {
      const uint32_t g1 = g;
      const uint32_t g2 = lcg_next(g1);
      g = lcg_next(g2);
      d[q] = (T)(ref_uniform(ref_canonical(g1, g2), fa.dlo[q], fa.dhi[q]) * gd);
    }
  } else {
    const Draws6 r = philox_motion6((uint32_t)n, (uint32_t)iter, fa.flo, fa.fhi, fa.key0, fa.key1);
    // draw = u21 * (hi - lo) + lo, u21 = v * 2^-21 (exact): v * rgs is the same product rounded once, so the
    // conversion's scaling multiply is folded into the host constant
#pragma unroll
    for (int q = 0; q < 6; ++q) d[q] = (T)r.v[q] * sc.rgs[q] + sc.lo[q];
    if (iter >= 10) {  // wave-uniform: the growth factor 1 + growth * (iter / 10) is exactly 1 before iteration 10
      // (the empty asm keeps this a scalar branch: if-converted, every frame paid the six products and six
      // v_cndmask selects)
      asm volatile("");
      const T g = (T)gd;
#pragma unroll
      for (int q = 0; q < 6; ++q) d[q] = d[q] * g;
    }
  }
  T sa, ca, sb, cb, sz, cz;
  if (fa.small_angles) {  // wave-uniform (fp32 only: the host never sets it for fp64)
    sincos_small(d[0], &sa, &ca);
    sincos_small(d[1], &sb, &cb);
    sincos_small(d[2], &sz, &cz);
  } else {
    sincos_t(d[0], &sa, &ca);
    sincos_t(d[1], &sb, &cb);
    sincos_t(d[2], &sz, &cz);
  }
  // R = ((R_A * Rz(c)) * Ry(b)) * Rx(a)   (PE:582)
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const T a0 = A[i * 4 + 0], a1 = A[i * 4 + 1], a2 = A[i * 4 + 2];
    const T z0 = fmadd(a1, sz, a0 * cz);      // A*Rz col 0
    const T z1 = fmadd(a1, cz, a0 * (-sz));   // A*Rz col 1
    const T y0 = fmadd(a2, (-sb), z0 * cb);   // *Ry col 0
    const T y2 = fmadd(a2, cb, z0 * sb);      // *Ry col 2
    const T x1 = fmadd(y2, sa, z1 * ca);      // *Rx col 1
    const T x2 = fmadd(y2, ca, z1 * (-sa));   // *Rx col 2
    P[i * 4 + 0] = y0;
    P[i * 4 + 1] = x1;
    P[i * 4 + 2] = x2;
    P[i * 4 + 3] = A[i * 4 + 3] + d[3 + i];   // translation added unrotated (PE:585-587)
  }
}

template <typename T, int RNG, typename SP>
__device__ __forceinline__ void make_particle(const FrameArgsT<T>& fa, const LdsConst<T>& sc,
                                              const SP* __restrict__ prior, int n, int iter, T* P) {
  T A[12];
  if (n >= 2) load_prior(fa, prior, n, A);
  propagate<T, RNG>(fa, sc, A, n, iter, P);
}

// Q = K * P (3x4).  fp32 with an upper-triangular K whose last row is (0 0 1) (every pinhole CameraInfo,
// README.md:95-143; the host checks, FrameArgsT::k_upper): the zero terms are skipped, 16 instead of 36
// operations.  A skipped term is an exact +-0 added before the first rounding, so the sums are the same
// except for the sign of an exact zero.  fp64 (the parity mode) keeps the literal form.
// fp32 pairs for the packed VALU forms (v_pk_mul_f32 / v_pk_fma_f32 / v_pk_add_f32: two fp32 operations per
// instruction).  Each lane of a pair sees exactly the scalar operation sequence (mul, fma, add rounded the
// same way; the TUs are built with -ffp-contract=off, so nothing else fuses), so packed and scalar forms
// give the same bits.
// a * b + c for 0 <= a, b < 2^24: one full-rate v_mad_u32_u24 (v_mul_lo_u32 is quarter rate)
__device__ __forceinline__ int mad24(int a, int b, int c) {
  return (int)(((unsigned)a & 0xffffffu) * ((unsigned)b & 0xffffffu)) + c;
}
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2 pk_fma(f32x2 a, f32x2 b, f32x2 c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ f32x2 pk2(float a, float b) { return f32x2{a, b}; }

template <typename T>
__device__ __forceinline__ void k_times_pose(const LdsConst<T>& sc, const T* P, bool k_upper, T* Q) {
  if (std::is_same<T, float>::value && k_upper) {
#pragma unroll
    for (int j = 0; j < 4; j += 2) {  // columns j, j + 1 as one pair
      const f32x2 p0 = pk2(P[0 * 4 + j], P[0 * 4 + j + 1]);
      const f32x2 p1 = pk2(P[1 * 4 + j], P[1 * 4 + j + 1]);
      const f32x2 p2 = pk2(P[2 * 4 + j], P[2 * 4 + j + 1]);
      f32x2 s = p0 * sc.K[0];
      s = pk_fma(pk2(sc.K[1], sc.K[1]), p1, s);
      s = pk_fma(pk2(sc.K[2], sc.K[2]), p2, s);
      const f32x2 s1 = pk_fma(pk2(sc.K[5], sc.K[5]), p2, p1 * sc.K[4]);
      Q[0 * 4 + j] = s.x;
      Q[0 * 4 + j + 1] = s.y;
      Q[1 * 4 + j] = s1.x;
      Q[1 * 4 + j + 1] = s1.y;
      Q[2 * 4 + j] = P[2 * 4 + j];
      Q[2 * 4 + j + 1] = P[2 * 4 + j + 1];
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < 3; ++i) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      T s = sc.K[i * 3 + 0] * P[0 * 4 + j];
      s = fmadd(sc.K[i * 3 + 1], P[1 * 4 + j], s);
      s = fmadd(sc.K[i * 3 + 2], P[2 * 4 + j], s);
      Q[i * 4 + j] = s;
    }
  }
}

// project2d (PE:1017-1034): p = (K34*T) * [X;1], u = p/p.z — full K, no distortion, no z>0 test
template <typename T, int MAXM>
__device__ __forceinline__ void project_markers(const FrameArgsT<T>& fa, const LdsConst<T>& sc, const T* P, T* u,
                                                T* v) {
  T Q[12];
  k_times_pose<T>(sc, P, fa.k_upper != 0, Q);
  if constexpr (std::is_same<T, float>::value) {  // rows 0 and 1 as one packed pair, same operations
    // every slot up to MAXM is projected (markers past M are zeros, their u / v never read): no branch, so the
    // u / v arrays stay in registers (a conditional store per slot had put them in scratch)
    const f32x2 q0 = pk2(Q[0], Q[4]), q1 = pk2(Q[1], Q[5]), q2 = pk2(Q[2], Q[6]), q3 = pk2(Q[3], Q[7]);
#pragma unroll
    for (int j = 0; j < MAXM; ++j) {
      const float X = sc.markers[3 * j], Y = sc.markers[3 * j + 1], Z = sc.markers[3 * j + 2];
      f32x2 s = q0 * X;
      s = pk_fma(q1, pk2(Y, Y), s);
      s = pk_fma(q2, pk2(Z, Z), s);
      s = s + q3;
      float z = Q[8] * X;
      z = fmadd(Q[9], Y, z);
      z = fmadd(Q[10], Z, z);
      z = z + Q[11];
      const f32x2 uv = s * rcp_t(z);  // persp(): p0 * rcp(p2), p1 * rcp(p2)
      u[j] = uv.x;
      v[j] = uv.y;
    }
    return;
  }
#pragma unroll
  for (int j = 0; j < MAXM; ++j) {
    if (marker_live<MAXM>(j, fa.M)) {
      const T X = sc.markers[3 * j], Y = sc.markers[3 * j + 1], Z = sc.markers[3 * j + 2];
      T p[3];
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        T s = Q[i * 4 + 0] * X;
        s = fmadd(Q[i * 4 + 1], Y, s);
        s = fmadd(Q[i * 4 + 2], Z, s);
        p[i] = s + Q[i * 4 + 3];
      }
      persp(p[0], p[1], p[2], &u[j], &v[j]);
    } else {
      u[j] = v[j] = (T)0;
    }
  }
}

// project_markers' arithmetic for ONE marker j (wave-uniform index): the same operation order, so the
// same bits
template <typename T>
__device__ __forceinline__ void project_one(const LdsConst<T>& sc, const T* P, int j, bool k_upper, T& u, T& v) {
  T Q[12];
  k_times_pose<T>(sc, P, k_upper, Q);
  const T X = sc.markers[3 * j], Y = sc.markers[3 * j + 1], Z = sc.markers[3 * j + 2];
  T p[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    T s = Q[i * 4 + 0] * X;
    s = fmadd(Q[i * 4 + 1], Y, s);
    s = fmadd(Q[i * 4 + 2], Z, s);
    p[i] = s + Q[i * 4 + 3];
  }
  persp(p[0], p[1], p[2], &u, &v);
}

// x-buckets per frame: 2 per blob rounded up to a power of two, in [128, kMaxBuckets] — narrow enough
// that the +-tolq window stays close to its own width when B is large (C3: 200 blobs, 1.5 px buckets)
__host__ __device__ __forceinline__ constexpr int bucket_count(int B) {
  int nb = 128;
  while (nb < kMaxBuckets && nb < 2 * B) nb *= 2;
  return nb;
}
// x -> bucket index (monotone in x; identical formula for table build and queries)
template <typename T>
__host__ __device__ __forceinline__ int bucket_of(T x, T xmin, T inv_bw, int nb) {
  const T f = (x - xmin) * inv_bw;
  if (!(f >= (T)0)) return 0;
  if (f >= (T)(nb - 1)) return nb - 1;
  return (int)f;
}
template <typename T>
struct alignas(2 * sizeof(T)) BlobXY {
  T x, y;
};

// calculateEstimationProbability (PE:2385-2445) in its closed form.  Step 1: per marker the first-minimum
// blob over all blobs (column minimum of the B x M distance matrix; ties -> lowest blob index).
// Step 2 (score_minima): extraction in ascending (distance, marker) order — the order Eigen's minCoeff
// visitor finds them — with the same gate (tol_PF), score ((tol-d)/tol)^2 with tol NOT tol_PF,
// self-occlusion (3*s) and downgrade (2) penalties, capped at min(B, M) pairs.
//
// Exact pruning (DESIGN.md "Exact blob pruning"): only blobs in the x-buckets overlapping the window
// |bx-u| <= tolq (tolq >= tol_PF plus rounding slack) are visited.  Every blob within tol_PF lies in the
// window, and a marker whose true minimum lies outside it fails the gate anyway, so accepted pairs,
// penalties and the weight are unchanged; rejected markers only change their (unused) distance value.
// fp32 tables also carry a 2D cell grid (build_blob_table_host): a marker's candidates are then ONE cell's
// list (a 2D window instead of an x-strip), walked by column_minima's grid branch.
template <typename T>
struct LdsBlobs;

// bucket_of without branches (fp32 kernels): max(f, 0) maps NaN and negatives to 0 (v_max_f32 returns the
// non-NaN operand), min(., nb-1) clamps; the same bucket as bucket_of for every input
__device__ __forceinline__ int bucket_of_bf(float x, float xmin, float inv_bw, int nb) {
  const float f = (x - xmin) * inv_bw;
  return (int)__builtin_fminf(__builtin_fmaxf(f, 0.0f), (float)(nb - 1));
}

// PHASED (k_frame2, whose VGPR budget holds every marker's cell record): the grid branch in phases over the
// markers; the register-capped streaming kernels keep the per-marker form (the phases spill there)
template <typename T, int MAXM, bool PRUNE, bool PHASED = false>
__device__ __forceinline__ int column_minima(const FrameArgsT<T>& fa, const T* u, const T* v,
                                             const LdsBlobs<T>& tb, T* m, int* r) {
  const int B = fa.B, M = fa.M;
  int visited = 0;
  if constexpr (std::is_same<T, float>::value) {
    // fp32: branch-free visits on ONE 64-bit key per candidate, {distance bits : original index}.  Distances
    // are sums of squares (>= +0 or NaN), whose IEEE bits order like the values, and every NaN's bits lie
    // above +inf's, so "key < best key" is exactly "strictly closer, or equally close with a lower original
    // index" (the general form's tie rule) and a NaN distance is never taken.  A minimum that stays +inf keeps
    // r = 0 (the general form's bc < 0 case); it fails the gate anyway.  Candidates go two per step, the
    // second masked past the window end (its LDS reads stay inside the padded table, kTablePad).
    // The query buckets: f = (u - (xmin -+ tolq)) * inv_bw, clamped by one med3 (NaN -> bucket 0 or any
    // in-range bucket: a NaN projection never takes a candidate).  The two roundings of xmin -+ tolq and
    // u - base are each within half an ulp of a pixel coordinate, like bucket_of's own, far inside tolq's
    // slack (1e-3 px + 0.1 %): the window still holds every blob within tol_PF.
    // The 2D grid (when the table has one built for at least this frame's window): the candidates of marker j
    // are the one cell list its projection falls in (build_blob_table_host proves every blob within tol_PF is
    // listed there); ~1 candidate per marker instead of an x-strip's ~2, so the wave's candidate walk is
    // usually a single step.  Otherwise the x-buckets.
    const GridArgs& ga = fa.grid;
    if (PRUNE && ga.on) {  // wave-uniform (host: the table's grid covers this frame's window)
      // Grid walk: one cell list per marker (~1 candidate).  Its entries are in increasing original index, so
      // a strict "closer" test keeps the first (lowest-index) of equally close blobs, the key order above,
      // and a NaN distance is never taken.  The list's first entry (the +inf sentinel for an empty cell) is
      // taken without a test: bd = min(d, +inf) maps a NaN distance to +inf, and an empty cell leaves r = 0.
      // Further entries are walked only when some lane's cell lists more than one blob (wave-uniform branch;
      // the particles of a wave project each marker into one or two neighbouring cells, so it is rare).
      // A non-finite first distance leaves r at that entry's index instead of 0: r is read only for a finite
      // minimum within tol_PF (the gate), so no weight, pair or record changes.
      const unsigned char* cells = tb.base + ga.cell_off;
      const unsigned char* ents = tb.base + ga.ent_off;
      const f32x2 ic = pk2(ga.inv_c, ga.inv_c), oc = pk2(ga.ox, ga.oy);
      if constexpr (PHASED) {
        // In phases over the markers (every cell record, then every first entry, then the longer lists behind
        // one wave-uniform test): a per-marker branch kept each marker's two dependent LDS round trips from
        // overlapping the next marker's, and at C2 (1.5 waves per SIMD) nothing else hides them
        uint32_t rec[MAXM];
  #pragma unroll
        for (int j = 0; j < MAXM; ++j) {
          rec[j] = 0;
          if (marker_live<MAXM>(j, M)) {
            const f32x2 f = pk_fma(pk2(u[j], v[j]), ic, oc);  // both cell coordinates in one v_pk_fma_f32
            const int cx = (int)__builtin_amdgcn_fmed3f(f.x, 0.0f, ga.fmaxx);
            const int cy = (int)__builtin_amdgcn_fmed3f(f.y, 0.0f, ga.fmaxy);
            // byte offset cy * 4 ncx + 4 cx (the row pitch scaled on the host)
            rec[j] = *(const uint32_t*)(cells + mad24(cy, ga.ncx4, cx << 2));
          }
        }
        // The 12 / 16-marker buckets (C3: 200 blobs, clustered, most lists longer than one) read the first two
        // entries together; the exact 5-marker bucket (50 blobs) reads one and walks further entries only when
        // some lane of the wave needs them.
        constexpr int c1 = MAXM > kExactM ? 2 : 1;
        bool more = false;  // some live marker's list has more than c1 entries
  #pragma unroll
        for (int j = 0; j < MAXM; ++j) {
          float bd = INFINITY;
          int bo = 0;
          if (marker_live<MAXM>(j, M)) {
            const f32x2 uvj = pk2(u[j], v[j]);
            const GridEnt* e = (const GridEnt*)(ents + (rec[j] & 0xffffu));
            const int n = (int)(rec[j] >> 16);
            visited += n;
            more |= n > c1;
            const GridEnt e0 = e[0];
            const f32x2 dd = pk2(e0.x, e0.y) - uvj;  // (dx, dy) in one v_pk_add_f32
            bd = __builtin_fminf(fmadd(dd.x, dd.x, dd.y * dd.y), INFINITY);
            bo = e0.orig;
            if constexpr (c1 == 2) {
              const GridEnt e1 = e[1];
              const f32x2 d1 = pk2(e1.x, e1.y) - uvj;
              const float d = fmadd(d1.x, d1.x, d1.y * d1.y);
              const bool take = (n > 1) & (d < bd);
              bd = take ? d : bd;
              bo = take ? e1.orig : bo;
            }
          }
          m[j] = bd;
          r[j] = bo;
        }
        if (__builtin_amdgcn_ballot_w64(more)) {  // rare at 50 blobs
  #pragma unroll
          for (int j = 0; j < MAXM; ++j) {
            if (!marker_live<MAXM>(j, M)) continue;
            const int n = (int)(rec[j] >> 16);
            if (!__builtin_amdgcn_ballot_w64(n > c1)) continue;
            const f32x2 uvj = pk2(u[j], v[j]);
            const GridEnt* e = (const GridEnt*)(ents + (rec[j] & 0xffffu));
            float bd = m[j];
            int bo = r[j];
            auto visit = [&](const GridEnt& ec, bool in) {
              const f32x2 dd = pk2(ec.x, ec.y) - uvj;
              const float d = fmadd(dd.x, dd.x, dd.y * dd.y);
              const bool take = in & (d < bd);
              bd = take ? d : bd;
              bo = take ? ec.orig : bo;
            };
            // two entries per step, the second masked past the list end (its LDS read stays inside the table
            // or its 16-B tail granule, BlobTable::lds_bytes)
  #pragma unroll 2
            for (int c = c1; c < n; c += 2) {
              const GridEnt ea = e[c], eb = e[c + 1];
              visit(ea, true);
              visit(eb, c + 1 < n);
            }
            m[j] = bd;
            r[j] = bo;
          }
        }
      } else {
  #pragma unroll
        for (int j = 0; j < MAXM; ++j) {
          float bd = INFINITY;
          int bo = 0;
          if (marker_live<MAXM>(j, M)) {
            const f32x2 uvj = pk2(u[j], v[j]);
            const f32x2 f = pk_fma(uvj, ic, oc);  // both cell coordinates in one v_pk_fma_f32
            const int cx = (int)__builtin_amdgcn_fmed3f(f.x, 0.0f, ga.fmaxx);
            const int cy = (int)__builtin_amdgcn_fmed3f(f.y, 0.0f, ga.fmaxy);
            // byte offset cy * 4 ncx + 4 cx (the row pitch scaled on the host)
            const uint32_t rec = *(const uint32_t*)(cells + mad24(cy, ga.ncx4, cx << 2));
            const GridEnt* e = (const GridEnt*)(ents + (rec & 0xffffu));
            const int n = (int)(rec >> 16);
            visited += n;
            auto visit = [&](const GridEnt& ec, bool in) {
              const f32x2 dd = pk2(ec.x, ec.y) - uvj;
              const float d = fmadd(dd.x, dd.x, dd.y * dd.y);
              const bool take = in & (d < bd);
              bd = take ? d : bd;
              bo = take ? ec.orig : bo;
            };
            // The 12 / 16-marker buckets (C3: 200 blobs, clustered, most lists longer than one) read the first
            // two entries together; the exact 5-marker bucket (50 blobs) reads one and walks further entries only
            // when some lane of the wave needs them.
            constexpr int c1 = MAXM > kExactM ? 2 : 1;
            {
              const GridEnt e0 = e[0];
              const f32x2 dd = pk2(e0.x, e0.y) - uvj;  // (dx, dy) in one v_pk_add_f32
              bd = __builtin_fminf(fmadd(dd.x, dd.x, dd.y * dd.y), INFINITY);
              bo = e0.orig;
              if constexpr (c1 == 2) visit(e[1], n > 1);
            }
            if (__builtin_amdgcn_ballot_w64(n > c1)) {  // some lane's list has more entries (rare at 50 blobs)
              // two entries per step, the second masked past the list end (its LDS read stays inside the table
              // or its 16-B tail granule, BlobTable::lds_bytes)
  #pragma unroll 2
              for (int c = c1; c < n; c += 2) {
                const GridEnt ea = e[c], eb = e[c + 1];
                visit(ea, true);
                visit(eb, c + 1 < n);
              }
            }
          }
          m[j] = bd;
          r[j] = bo;
        }
      }
      return visited;
    }
    const float fmaxb = (float)(tb.nb - 1);
    const float base_lo = tb.xmin + fa.tolq, base_hi = tb.xmin - fa.tolq;
#pragma unroll
    for (int j = 0; j < MAXM; ++j) {
      uint64_t best = ((uint64_t)0x7f800000u << 32) | 0x7fffffffu;
      if (marker_live<MAXM>(j, M)) {
        int c0 = 0, c1 = B;
        if (PRUNE) {
          const float flo = (u[j] - base_lo) * tb.inv_bw;
          const float fhi = (u[j] - base_hi) * tb.inv_bw;
          c0 = tb.bstart[(int)__builtin_amdgcn_fmed3f(flo, 0.0f, fmaxb)];
          c1 = tb.bstart[(int)__builtin_amdgcn_fmed3f(fhi, 0.0f, fmaxb) + 1];
        }
        visited += c1 - c0;
        const float uj = u[j], vj = v[j];
        const f32x2 uvj = pk2(uj, vj);
        auto visit = [&](BlobXY<float> p, int o, bool in) {
          const f32x2 dd = pk2(p.x, p.y) - uvj;  // (dx, dy) in one v_pk_add_f32
          const float d = fmadd(dd.x, dd.x, dd.y * dd.y);
          const uint64_t key = ((uint64_t)__float_as_uint(d) << 32) | (uint32_t)o;
          best = (in & (key < best)) ? key : best;
        };
        for (int c = c0; c < c1; c += 2) {
          const BlobXY<float> pa = tb.bxy[c], pb = tb.bxy[c + 1];
          const int oa = tb.orig[c], ob = tb.orig[c + 1];
          visit(pa, oa, true);
          visit(pb, ob, c + 1 < c1);
        }
      }
      const float bm = __uint_as_float((uint32_t)(best >> 32));
      m[j] = bm;
      r[j] = bm < INFINITY ? (int)(uint32_t)best : 0;
    }
    return visited;
  }
#pragma unroll
  for (int j = 0; j < MAXM; ++j) {
    T best = inf_t<T>();
    int bc = -1;  // table position of the current minimum
    if (marker_live<MAXM>(j, M)) {
      int c0 = 0, c1 = B;
      if (PRUNE) {
        c0 = tb.bstart[bucket_of(u[j] - fa.tolq, tb.xmin, tb.inv_bw, tb.nb)];
        c1 = tb.bstart[bucket_of(u[j] + fa.tolq, tb.xmin, tb.inv_bw, tb.nb) + 1];
      }
      visited += c1 - c0;
      auto visit = [&](int c, BlobXY<T> p) {
        const T dx = p.x - u[j];
        const T dy = p.y - v[j];
        const T d = fmadd(dx, dx, dy * dy);
        if (d < best) {
          best = d;
          bc = c;
        } else if (d == best && bc >= 0 && tb.orig[c] < tb.orig[bc]) {
          bc = c;
        }
      };
      int c = c0;
      for (; c + 1 < c1; c += 2) {  // two candidates' LDS reads in flight per step
        const BlobXY<T> pa = tb.bxy[c], pb = tb.bxy[c + 1];
        visit(c, pa);
        visit(c + 1, pb);
      }
      if (c < c1) visit(c, tb.bxy[c]);
    }
    m[j] = best;
    r[j] = bc >= 0 ? tb.orig[bc] : 0;
  }
  return visited;
}

// Eigen's visitor starts from coeff(0,0): a NaN distance there poisons the first minCoeff -> break at k=0
template <typename T>
__device__ __forceinline__ bool nan_at_origin(T b0x, T b0y, T u0, T v0) {
  const T dx = b0x - u0, dy = b0y - v0;
  const T d = dx * dx + dy * dy;
  return d != d;
}
// The same test with the table's blob 0 finite (host flag, wave-uniform): (b0 - u0)^2 + (b0y - v0)^2 is NaN
// exactly when u0 or v0 is NaN (an infinite difference squares to +inf and inf + inf = inf), one v_cmp_u; the
// blob is read from the table header only when it is not finite.
template <typename T>
__device__ __forceinline__ bool nan_at_origin_tb(const FrameArgsT<T>& fa, const LdsBlobs<T>& tb, T u0, T v0) {
  if (fa.grid.b0fin) return __builtin_isunordered(u0, v0);
  const T* hdr = (const T*)tb.base;
  return nan_at_origin(hdr[2], hdr[3], u0, v0);
}

// Extraction order = ascending (m_j, j): column minima are never NaN (they start at +inf and a NaN
// distance never compares smaller), so a sorting network on the (m_j, j) keys yields exactly the pair
// sequence of the reference's repeated minCoeff.  Batcher's odd-even merge sort, fully unrolled
// (MAXM = 8: 19 compare-exchanges); markers j >= M sort last with key +inf and lie beyond L anyway.
template <typename T>
__device__ __forceinline__ void cas_key(T& ma, int& ja, int& ra, T& mb, int& jb, int& rb) {
  const bool sw = mb < ma || (mb == ma && jb < ja);
  const T m0 = sw ? mb : ma, m1 = sw ? ma : mb;
  const int j0 = sw ? jb : ja, j1 = sw ? ja : jb;
  const int r0 = sw ? rb : ra, r1 = sw ? ra : rb;
  ma = m0; mb = m1; ja = j0; jb = j1; ra = r0; rb = r1;
}
template <typename T, int MAXM>
__device__ __forceinline__ void sort_minima(T* km, int* kj, int* kr) {
#pragma unroll
  for (int p = 1; p < MAXM; p <<= 1)
#pragma unroll
    for (int k = p; k >= 1; k >>= 1)
#pragma unroll
      for (int j = k % p; j + k < MAXM; j += 2 * k)
#pragma unroll
        for (int i = 0; i < k; ++i)
          if (i + j + k < MAXM && (i + j) / (2 * p) == (i + j + k) / (2 * p))
            cas_key(km[i + j], kj[i + j], kr[i + j], km[i + j + k], kj[i + j + k], kr[i + j + k]);
}

template <typename T, int MAXM, bool PAIRS>
__device__ __forceinline__ T score_minima(const FrameArgsT<T>& fa, const T* m, const int* r, uint32_t* pairs,
                                          int* npairs) {
  const int B = fa.B, M = fa.M;
  const int L = B < M ? B : M;
  const T tol = fa.tol, tol_pf = fa.tol_pf, Mt = (T)M;
  T km[MAXM];
  int kj[MAXM], kr[MAXM];
#pragma unroll
  for (int j = 0; j < MAXM; ++j) {
    km[j] = marker_live<MAXM>(j, M) ? m[j] : inf_t<T>();
    kj[j] = j;
    kr[j] = r[j];
  }
  sort_minima<T, MAXM>(km, kj, kr);
  T Pr = (T)0;
  int s = 1;
  bool live = true;
  if (PAIRS) *npairs = 0;
#pragma unroll
  for (int k = 0; k < MAXM; ++k) {
    if (k < L && live) {
      const T d = sqrt_t(km[k]);
      if (!(d <= tol_pf)) {
        live = false;  // the reference's break
      } else {
        const T q = div_t(tol - d, tol);
        Pr = Pr + (Mt + q * q);
        bool dup = false;  // an earlier (accepted) pair holds the same blob
#pragma unroll
        for (int e = 0; e < k; ++e) dup |= kr[e] == kr[k];
        if (dup) {
          Pr = Pr - (T)(s * 3);
          ++s;
        }
        if ((fa.downgrade >> kj[k]) & 1u) Pr = Pr - (T)2;
        if (PAIRS) {
          pairs[2 * k] = (uint32_t)kj[k] + 1u;
          pairs[2 * k + 1] = (uint32_t)kr[k] + 1u;
          *npairs = k + 1;
        }
      }
    }
  }
  return Pr;
}

// The weight of score_minima<PAIRS = false> without the sort, for B >= M (fp32 tolerance path).  With
// L = min(B, M) = M the cap never binds, and since the extraction runs in ascending distance the reference's
// break leaves exactly the markers whose own minimum passes the gate: A = {j : sqrt(m_j) <= tol_PF}.  The
// penalties depend on A only: 3*(1 + ... + D) with D = |A| - #distinct blobs over A (each marker whose blob
// an earlier marker of A holds, in ANY fixed order, counts once: the same D as in extraction order), and 2
// per downgraded marker of A.  Only the order of the fp32 additions differs from the extraction order
// (a few ulp of a weight <= M(M+1)).
template <int MAXM>
__device__ __forceinline__ float score_unordered(const FrameArgsT<float>& fa, const float* m, const int* r) {
  const int M = fa.M;
  const float tol = fa.tol, tol_pf = fa.tol_pf, Mt = (float)M;
  const float rtol = rcp_t(tol);
  float Pr = 0.0f;
  int dups = 0;
  bool acc[MAXM];
#pragma unroll
  for (int j = 0; j < MAXM; ++j) {
    const float d = sqrt_t(m[j]);
    acc[j] = d <= tol_pf;  // markers past M have m = +inf (column_minima), never accepted
    const float q = (tol - d) * rtol;
    Pr = acc[j] ? Pr + (Mt + q * q) : Pr;
    bool dup = false;
#pragma unroll
    for (int e = 0; e < j; ++e) dup |= acc[e] & (r[e] == r[j]);
    dups += (acc[j] & dup) ? 1 : 0;
  }
  int ndg = 0;
  if (fa.downgrade) {  // wave-uniform: the downgrade penalties (2 per accepted downgraded marker)
#pragma unroll
    for (int j = 0; j < MAXM; ++j) ndg += (acc[j] && ((fa.downgrade >> j) & 1u)) ? 1 : 0;
  }
  return Pr - (float)(3 * dups * (dups + 1) / 2 + 2 * ndg);
}

// ----------------------------------------------------------------------------- wave/block helpers
__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }
// Lanes of ONE wave exchanging data through LDS without a workgroup barrier: the hardware keeps a
// wave's LDS operations in order, but the compiler must also be told that other lanes wrote (else it
// may forward a lane's own earlier store to its read).
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
__device__ __forceinline__ int wave_id() { return threadIdx.x >> 6; }
// the same, as an SGPR (block sizes are multiples of 64): a loop over the earlier waves then has a scalar trip
// count instead of a per-wave v_cndmask chain.  (Used where that pays: as the general wave_id it moved the
// weighing pass's register allocation for the worse.)
__device__ __forceinline__ int wave_id_u() { return __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)); }

// All wave-level scans and reductions run on DPP lane moves (no LDS, no ds_bpermute): row_shr 1/2/4/8
// builds the inclusive scan inside each 16-lane row, row_bcast:15 / row_bcast:31 carry row totals
// across rows (GFX9-family DPP, kept by gfx950), so lane 63 ends with the wave total.  The pattern is
// fixed, so a sum has ONE association everywhere it is evaluated (k_propagate_weigh and k_resample
// must agree bit-for-bit).  Every lane of the wave must execute these (no divergent calls).
enum : int {
  kDppRowShr1 = 0x111, kDppRowShr2 = 0x112, kDppRowShr4 = 0x114, kDppRowShr8 = 0x118,
  kDppWaveShr1 = 0x138, kDppBcast15 = 0x142, kDppBcast31 = 0x143
};
template <int CTRL, int RM = 0xf>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t src, uint32_t old) {
  return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)src, CTRL, RM, 0xf, false);
}
template <int CTRL, int RM = 0xf>
__device__ __forceinline__ int dpp(int src, int old) {
  return (int)dpp_u32<CTRL, RM>((uint32_t)src, (uint32_t)old);
}
template <int CTRL, int RM = 0xf>
__device__ __forceinline__ float dpp(float src, float old) {
  return __uint_as_float(dpp_u32<CTRL, RM>(__float_as_uint(src), __float_as_uint(old)));
}
template <int CTRL, int RM = 0xf>
__device__ __forceinline__ double dpp(double src, double old) {
  const uint64_t s = (uint64_t)__double_as_longlong(src), o = (uint64_t)__double_as_longlong(old);
  const uint32_t lo = dpp_u32<CTRL, RM>((uint32_t)s, (uint32_t)o);
  const uint32_t hi = dpp_u32<CTRL, RM>((uint32_t)(s >> 32), (uint32_t)(o >> 32));
  return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
// value of lane L in every lane (scalar result)
// A value the optimiser may not look through.  In a select chain over a register array (lane q picks word
// q) the loads would otherwise be folded into ONE load of a selected address, which pins the array in
// scratch memory (a VMEM round trip per use); with the values opaque the chain stays v_cndmask.
template <typename V>
__device__ __forceinline__ V opaque(V x) {
  asm volatile("" : "+v"(x));
  return x;
}
__device__ __forceinline__ int lane_value(int x, int L) { return __builtin_amdgcn_readlane(x, L); }
__device__ __forceinline__ float lane_value(float x, int L) {
  return __uint_as_float((uint32_t)__builtin_amdgcn_readlane((int)__float_as_uint(x), L));
}
__device__ __forceinline__ double lane_value(double x, int L) {
  const uint64_t v = (uint64_t)__double_as_longlong(x);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, L);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), L);
  return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
// lane i receives lane i-1's value, lane 0 receives `fill`
template <typename V>
__device__ __forceinline__ V wave_shr1(V x, V fill) {
  return dpp<kDppWaveShr1>(x, fill);
}

struct OpSum {
  __device__ double operator()(double a, double b) const { return a + b; }
};
struct OpMax {
  __device__ double operator()(double a, double b) const { return b > a ? b : a; }
};
struct OpMin {
  __device__ double operator()(double a, double b) const { return b < a ? b : a; }
};
struct OpMaxI {
  __device__ int operator()(int a, int b) const { return b > a ? b : a; }
};
// inclusive scan x_0 op ... op x_i; `id` is the identity of op
template <typename V, typename Op>
__device__ __forceinline__ V wave_scan(V x, V id, Op op) {
  x = op(x, dpp<kDppRowShr1>(x, id));
  x = op(x, dpp<kDppRowShr2>(x, id));
  x = op(x, dpp<kDppRowShr4>(x, id));
  x = op(x, dpp<kDppRowShr8>(x, id));
  x = op(x, dpp<kDppBcast15, 0xa>(x, id));
  x = op(x, dpp<kDppBcast31, 0xc>(x, id));
  return x;
}
// Sum scan of doubles: the four row_shr steps read 0 (bound_ctrl) from a lane outside the row, which is the
// sum's identity (+0.0 is all-zero bits), so they need no fill register; the two row_bcast steps write only
// some rows and keep the fill.  Bit-identical to wave_scan(v, 0.0, OpSum()).
template <int CTRL>
__device__ __forceinline__ double dpp_zf(double x) {
  const uint64_t v = (uint64_t)__double_as_longlong(x);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)v, CTRL, 0xf, 0xf, true);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)(v >> 32), CTRL, 0xf, 0xf, true);
  return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
__device__ __forceinline__ double wave_incl_sum(double x) {
  x = x + dpp_zf<kDppRowShr1>(x);
  x = x + dpp_zf<kDppRowShr2>(x);
  x = x + dpp_zf<kDppRowShr4>(x);
  x = x + dpp_zf<kDppRowShr8>(x);
  x = x + dpp<kDppBcast15, 0xa>(x, 0.0);
  x = x + dpp<kDppBcast31, 0xc>(x, 0.0);
  return x;
}
__device__ __forceinline__ double wave_incl_max(double v) { return wave_scan(v, -(double)INFINITY, OpMax()); }
__device__ __forceinline__ double wave_incl_min(double v) { return wave_scan(v, (double)INFINITY, OpMin()); }
__device__ __forceinline__ double wave_max(double v) { return lane_value(wave_incl_max(v), 63); }
__device__ __forceinline__ double wave_min(double v) { return lane_value(wave_incl_min(v), 63); }

// (value, index): larger value wins, lower index on ties
// (selects, not branches: the wave reductions stay one basic block)
template <typename V>
__device__ __forceinline__ void cmb_max(V& v, int& i, V v2, int i2) {
  const bool t = (v2 > v) | ((v2 == v) & (i2 < i));  // non-short-circuit: no exec-mask branches
  v = t ? v2 : v;
  i = t ? i2 : i;
}
template <typename V>
__device__ __forceinline__ void cmb_min(V& v, int& i, V v2, int i2) {
  const bool t = (v2 < v) | ((v2 == v) & (i2 < i));
  v = t ? v2 : v;
  i = t ? i2 : i;
}
// wave arg-reductions: the lexicographic (value, index) order is associative and commutative, so the
// scan pattern reduces it exactly; the result is broadcast to every lane
template <typename V, int CTRL, int RM = 0xf>
__device__ __forceinline__ void argmax_step(V& v, int& i, V idv) {
  const V v2 = dpp<CTRL, RM>(v, idv);
  const int i2 = dpp<CTRL, RM>(i, 0x7fffffff);
  cmb_max(v, i, v2, i2);
}
template <typename V, int CTRL, int RM = 0xf>
__device__ __forceinline__ void argmin_step(V& v, int& i, V idv) {
  const V v2 = dpp<CTRL, RM>(v, idv);
  const int i2 = dpp<CTRL, RM>(i, 0x7fffffff);
  cmb_min(v, i, v2, i2);
}
template <typename V>
__device__ __forceinline__ void wave_argmax(V& v, int& i) {
  const V id = -(V)INFINITY;
  argmax_step<V, kDppRowShr1>(v, i, id);
  argmax_step<V, kDppRowShr2>(v, i, id);
  argmax_step<V, kDppRowShr4>(v, i, id);
  argmax_step<V, kDppRowShr8>(v, i, id);
  argmax_step<V, kDppBcast15, 0xa>(v, i, id);
  argmax_step<V, kDppBcast31, 0xc>(v, i, id);
  v = lane_value(v, 63);
  i = lane_value(i, 63);
}
template <typename V>
__device__ __forceinline__ void wave_argmin(V& v, int& i) {
  const V id = (V)INFINITY;
  argmin_step<V, kDppRowShr1>(v, i, id);
  argmin_step<V, kDppRowShr2>(v, i, id);
  argmin_step<V, kDppRowShr4>(v, i, id);
  argmin_step<V, kDppRowShr8>(v, i, id);
  argmin_step<V, kDppBcast15, 0xa>(v, i, id);
  argmin_step<V, kDppBcast31, 0xc>(v, i, id);
  v = lane_value(v, 63);
  i = lane_value(i, 63);
}
// int counts: "-infinity" is INT_MIN
template <>
__device__ __forceinline__ void wave_argmax<int>(int& v, int& i) {
  const int id = (int)0x80000000;
  argmax_step<int, kDppRowShr1>(v, i, id);
  argmax_step<int, kDppRowShr2>(v, i, id);
  argmax_step<int, kDppRowShr4>(v, i, id);
  argmax_step<int, kDppRowShr8>(v, i, id);
  argmax_step<int, kDppBcast15, 0xa>(v, i, id);
  argmax_step<int, kDppBcast31, 0xc>(v, i, id);
  v = lane_value(v, 63);
  i = lane_value(i, 63);
}

// Deterministic block inclusive scan: pre_w = ((0 + t_0) + t_1) + ... over earlier waves' totals, then
// incl = pre_w + (wave inclusive).  k_propagate_weigh derives its partial extrema with exactly this
// association, so both launches see bit-identical prefixes.  sh: >= kWaves doubles.
// The wave scan of fp32 weights on the 2^-21 grid as integers.  Every weight of an M >= 4 frame is a multiple of
// 2^-21 (each score term Mt + q^2 is >= 4, so every partial score, the integer penalties subtracted, is too), so
// with 0 <= w < 32 in the wave, w * 2^21 is an integer below 2^26 and every 64-lane prefix lies below 2^32: the u32
// scan is the exact prefix sum, which wave_incl_sum's fp64 partial sums (at most 32 significant bits) also are.
// One v_add_u32_dpp per step instead of two v_mov_b32_dpp and a v_add_f64.
__device__ __forceinline__ double wave_incl_sum_fx(float w) {
  uint32_t x = (uint32_t)(w * 0x1p21f);
  x += (uint32_t)__builtin_amdgcn_mov_dpp((int)x, kDppRowShr1, 0xf, 0xf, true);
  x += (uint32_t)__builtin_amdgcn_mov_dpp((int)x, kDppRowShr2, 0xf, 0xf, true);
  x += (uint32_t)__builtin_amdgcn_mov_dpp((int)x, kDppRowShr4, 0xf, 0xf, true);
  x += (uint32_t)__builtin_amdgcn_mov_dpp((int)x, kDppRowShr8, 0xf, 0xf, true);
  x += dpp_u32<kDppBcast15, 0xa>(x, 0u);
  x += dpp_u32<kDppBcast31, 0xc>(x, 0u);
  return (double)x * 0x1p-21;
}
// block inclusive prefix from the wave's inclusive scan wi (the earlier waves' totals through LDS)
__device__ __forceinline__ void block_incl_from_wave(double wi, double& incl, double* sh) {
  if (lane_id() == 63) sh[wave_id()] = wi;
  __syncthreads();
  double pre = 0.0;
  const int wv = wave_id_u();
#pragma clang loop unroll(disable)
  for (int w = 0; w < wv; ++w) pre = pre + sh[w];  // a scalar trip count: no per-wave select chain
  incl = pre + wi;
}
__device__ __forceinline__ void block_incl_sum(double v, double& incl, double* sh) {
  const double wi = wave_incl_sum(v);
  if (lane_id() == 63) sh[wave_id()] = wi;
  __syncthreads();
  double pre = 0.0;
  const int wv = wave_id_u();
#pragma clang loop unroll(disable)
  for (int w = 0; w < wv; ++w) pre = pre + sh[w];  // a scalar trip count: no per-wave select chain
  incl = pre + wi;
}

// ---- interleaved wave scans: several independent chains advanced step by step in ONE basic block, so
// the DPP / f64 latencies of one chain hide behind the others.  Each chain's arithmetic is exactly that
// of wave_scan / wave_argmax / wave_argmin (same steps, same identities, same operand order).
template <int C, int R>
struct DppStep {
  static constexpr int ctrl = C, rm = R;
};
template <typename F>
__device__ __forceinline__ void scan_steps(F&& f) {
  f(DppStep<kDppRowShr1, 0xf>{});
  f(DppStep<kDppRowShr2, 0xf>{});
  f(DppStep<kDppRowShr4, 0xf>{});
  f(DppStep<kDppRowShr8, 0xf>{});
  f(DppStep<kDppBcast15, 0xa>{});
  f(DppStep<kDppBcast31, 0xc>{});
}
template <typename S>
__device__ __forceinline__ void st_sum(double& x) {
  x = x + dpp<S::ctrl, S::rm>(x, 0.0);
}
template <typename S>
__device__ __forceinline__ void st_max(double& x) {
  const double y = dpp<S::ctrl, S::rm>(x, -(double)INFINITY);
  x = y > x ? y : x;
}
template <typename S>
__device__ __forceinline__ void st_min(double& x) {
  const double y = dpp<S::ctrl, S::rm>(x, (double)INFINITY);
  x = y < x ? y : x;
}
template <typename S, typename V>
__device__ __forceinline__ void st_argmax(V& v, int& i) {
  const V v2 = dpp<S::ctrl, S::rm>(v, -(V)INFINITY);
  const int i2 = dpp<S::ctrl, S::rm>(i, 0x7fffffff);
  cmb_max(v, i, v2, i2);
}
template <typename S, typename V>
__device__ __forceinline__ void st_argmin(V& v, int& i) {
  const V v2 = dpp<S::ctrl, S::rm>(v, (V)INFINITY);
  const int i2 = dpp<S::ctrl, S::rm>(i, 0x7fffffff);
  cmb_min(v, i, v2, i2);
}
template <typename V>
__device__ __forceinline__ void bcast63(V& v, int& i) {
  v = lane_value(v, 63);
  i = lane_value(i, 63);
}

// fl(a / b) without the fp64 division: y = fl(1 / b) (Ctrl::invS, one division per frame), q0 = fl(a y), then two
// Newton corrections with fma residuals.  After the first, q1 is a faithful approximation of a / b, so its residual
// a - b q1 is exact, and fl(q1 + r1 y) = fl(a / b) (Markstein's theorem: y correctly rounded, no overflow or
// underflow; tests/test_div_by_s.py checks 10^7 cases against IEEE division).  Callers use it only where the
// quotient is in [0, ~1] and b is a normal positive double (fp32 weights, no negative weight in the wave), and
// keep the IEEE division otherwise.
__device__ __forceinline__ double div_by_S(double a, double b, double y) {
  const double q0 = a * y;
  const double r0 = __builtin_fma(-b, q0, a);
  const double q1 = __builtin_fma(r0, y, q0);
  const double r1 = __builtin_fma(-b, q1, a);
  return __builtin_fma(r1, y, q1);
}

// ----------------------------------------------------------------------------- stratified targets
// r_k = (k + U_k) / N  (PE:671); U_k is the k-th resample draw, taken after all motion draws.
// fl(k + U_k): the numerator of target r_k = fl(fl(k + U_k) / N)
template <typename T, int RNG>
__device__ __forceinline__ double target_num(const FrameArgsT<T>& fa, int iters, int64_t k) {
  double U;
  if (RNG == kRngReference) {
    const uint64_t motion = fa.N > 2 ? (uint64_t)12 * (uint64_t)(fa.N - 2) * (uint64_t)iters : 0u;
    const uint32_t g1 = lcg_output(fa.lcg_x0, motion + 2u * (uint64_t)k + 1u);
    const uint32_t g2 = lcg_next(g1);
    U = ref_uniform(ref_canonical(g1, g2), 0.0, 1.0);
  } else {
    const U32x4 o = philox4x32_10((uint32_t)k, kTagResample << 24, fa.flo, fa.fhi, fa.key0, fa.key1);
    U = u53(o.x, o.y);
  }
  return (double)(int32_t)k + U;  // 0 <= k <= N < 2^31: one v_cvt_f64_i32 (exact)
}

// r_k <= x, decided exactly without the fp64 division in all but a vanishing band.  With a = fl(k + U_k) and
// the exact real residual x*N - a, whose sign the single rounding of fma(x, N, -a) preserves:
//   x*N - a >= 0  ->  a/N <= x  ->  fl(a/N) <= x (rounding is monotone and x is a double);
//   a - x*N > N*ulp(x)  ->  a/N > x + ulp(x)  ->  fl(a/N) > x.
// thr = fl(x*N)*2^-50 + 2^-1000 bounds N*ulp(x) from above with a wide margin (ulp(x) <= x*2^-52 for normal x;
// the absolute term covers tiny x).  Between the two (a within ~2^-50 relative of x*N) the reference's own
// division decides.  xn = fl(x*N), thr = fma(xn, 2^-50, 2^-1000): per call site, computed once.
template <typename T, int RNG>
__device__ __forceinline__ bool target_le(const FrameArgsT<T>& fa, int iters, int64_t k, double x, double thr) {
  const double a = target_num<T, RNG>(fa, iters, k);
  const double Nd = (double)fa.N;
  const double e = __builtin_fma(x, Nd, -a);
  bool le = e >= 0.0;
  // the band: the reference's rounding decides (PE:674-679 compares the divided target).  Behind a wave-uniform
  // test: as a plain `return a / Nd <= x` the compiler evaluated the fp64 division for every lane with e < 0
  // (about half of them), i.e. in every wave of k_resample
  const bool band = !le && !(-e > thr);
  if (__builtin_amdgcn_ballot_w64(band)) {
    if (band) le = a / Nd <= x;
  }
  return le;
}

// F(x) = #{k : r_k <= x}.  r_k is non-decreasing in k, so target k finds the first particle i whose
// running-max cumulative weight R_i >= r_k (reference: first i with cumsum_i >= r_k, PE:674-679),
// and particle i receives F(R_i) - F(R_{i-1}) copies.
//
// One evaluation decides F(x) almost always.  With xn = fl(x N), k = floor(xn), f = xn - k (exact):
//   r_{k+1} >= fl((k+1)/N) >= (k+1)(1-2^-53)/N  and  x <= (k+f)/((1-2^-53)N), so r_{k+1} > x whenever
//   1 - f > (k+1) 2^-52;
//   r_{k-1} <= fl(k/N) <= k(1+2^-53)/N        and  x >= (k+f)/((1+2^-53)N), so r_{k-1} <= x whenever
//   f > k 2^-51.
// For N < 2^31 both bounds are below kEdge = 1e-6; inside that band (or for x N >= N) the neighbours
// are scanned explicitly.
template <typename T, int RNG>
__device__ __forceinline__ int64_t count_targets(const FrameArgsT<T>& fa, int iters, double x) {
  constexpr double kEdge = 1e-6;
  const int64_t N = fa.N;
  if (!(x >= 0.0)) return 0;  // r_k >= 0; also -inf / NaN
  const double xn = x * (double)N;
  const double fk = floor(xn);
  // the neighbour scans run almost never: kept as rolled loops (no unroll, no interleave), so their inlined
  // RNG copies add less scalar register pressure (static SGPR spills of k_resample 557 -> 293)
  const double thr = __builtin_fma(xn, 0x1p-50, 0x1p-1000);  // target_le's band (xn = +inf: never reached)
  if (!(fk < (double)N)) {  // x >= ~1: scan down from N
    int64_t k = N;
#pragma clang loop unroll(disable) interleave(disable) vectorize(disable)
    while (k > 0 && !target_le<T, RNG>(fa, iters, k - 1, x, thr)) --k;
    return k;
  }
  int64_t k = (int64_t)(int32_t)fk;  // 0 <= fk < N < 2^31: one v_cvt_i32_f64 (an int64 conversion is five)
  const double f = xn - fk;
  if (target_le<T, RNG>(fa, iters, k, x, thr)) {
    ++k;
    if (1.0 - f <= kEdge) {
#pragma clang loop unroll(disable) interleave(disable) vectorize(disable)
      while (k < N && target_le<T, RNG>(fa, iters, k, x, thr)) ++k;
    }
  } else if (f <= kEdge) {
#pragma clang loop unroll(disable) interleave(disable) vectorize(disable)
    while (k > 0 && !target_le<T, RNG>(fa, iters, k - 1, x, thr)) --k;
  }
  return k;
}

// count_targets for a whole wave, the common case straight-line: with x in [0, ~1), xn = x N away from an integer
// by more than kEdge on both sides, ONE target evaluation k = floor(xn) decides F(x) = k + [r_k <= x] (count_targets'
// argument), and outside the 2^-50 band its sign test needs no division.  Lanes that are not in that case (x < 0
// or NaN, x N >= N, near an integer, in the band) redo count_targets itself behind a wave-uniform test.  Without
// the exec-mask branches of count_targets' rare paths the common path is one basic block (k_resample: fewer SALU
// and VALU per wave).  Same result as count_targets for every active lane.
template <typename T, int RNG>
__device__ __forceinline__ int count_targets_wave(const FrameArgsT<T>& fa, int iters, double x, bool active) {
  constexpr double kEdge = 1e-6;  // count_targets' band around integers
  const double Nd = (double)fa.N;
  const double xn = x * Nd;
  const double fk = floor(xn);
  const double f = xn - fk;
  const bool simple = x >= 0.0 && fk < Nd && f > kEdge && 1.0 - f > kEdge;
  const int k = simple ? (int)fk : 0;
  const double a = target_num<T, RNG>(fa, iters, k);
  const double e = __builtin_fma(x, Nd, -a);
  const double thr = __builtin_fma(xn, 0x1p-50, 0x1p-1000);
  const bool le = e >= 0.0;
  const bool band = !le && !(-e > thr);
  int res = k + (le ? 1 : 0);
  const bool slow = active && (!simple || band);
  if (__builtin_amdgcn_ballot_w64(slow)) {
    if (slow) res = (int)count_targets<T, RNG>(fa, iters, x);
  }
  return res;
}

// ----------------------------------------------------------------------------- in-launch hand-off
// Per-block / per-group partials go to the last arriver (MI355X_MICROARCH.md "Valid forms", row 1):
// every partial word is stored write-through (sc1, agent scope) by the one lane that then drains
// (s_waitcnt vmcnt(0)) and adds to ONE unsharded counter; the arriver whose add returns count-1 is
// last and its wave reads the partials with sc1 loads.  No buffer_wbl2 / buffer_inv fences: those
// write back the XCD's whole dirty L2 (the weights / new prior this kernel streams) once per block.
typedef __attribute__((address_space(1))) uint64_t gu64_t;
typedef __attribute__((address_space(1))) uint32_t gu32_t;

// publication to the host: relaxed system-scope stores of tagged 8-byte granules (RecOut)
__device__ __forceinline__ void st_sys64(void* p, uint64_t v) {
  __hip_atomic_store((gu64_t*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ void st_wt(void* p, uint64_t v) {
  __hip_atomic_store((gu64_t*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_wt_d(double* p, double v) { st_wt(p, (uint64_t)__double_as_longlong(v)); }
__device__ __forceinline__ uint64_t ld_wt(const void* p) {
  return __hip_atomic_load((gu64_t*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_wt_d(const double* p) { return __longlong_as_double((long long)ld_wt(p)); }
// a whole BlockPart as three 16-B write-through-coherent (sc1) loads, issued without waiting.  The raw
// registers are asm outputs; wait_parts drains vmcnt with them as in/out operands, so no use of them can
// be scheduled before the wait.
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
struct PartRaw {
  u32x4_t a, b, c;
};
__device__ __forceinline__ void ld_part_issue(const BlockPart* p, PartRaw& r) {
  static_assert(sizeof(BlockPart) == 48, "BlockPart is three 16-B granules");
  asm volatile("global_load_dwordx4 %0, %1, off sc1" : "=v"(r.a) : "v"((const char*)p) : "memory");
  asm volatile("global_load_dwordx4 %0, %1, off offset:16 sc1" : "=v"(r.b) : "v"((const char*)p) : "memory");
  asm volatile("global_load_dwordx4 %0, %1, off offset:32 sc1" : "=v"(r.c) : "v"((const char*)p) : "memory");
}
__device__ __forceinline__ void wait_parts(PartRaw& r0, PartRaw& r1) {
  asm volatile("s_waitcnt vmcnt(0)" : "+v"(r0.a), "+v"(r0.b), "+v"(r0.c), "+v"(r1.a), "+v"(r1.b), "+v"(r1.c)::"memory");
}
__device__ __forceinline__ BlockPart unpack_part(const PartRaw& r) {
  BlockPart q;
  u32x4_t* d = (u32x4_t*)&q;
  d[0] = r.a;
  d[1] = r.b;
  d[2] = r.c;
  return q;
}
__device__ __forceinline__ uint64_t pack2(int a, int b) { return (uint64_t)(uint32_t)a | ((uint64_t)(uint32_t)b << 32); }
__device__ __forceinline__ int lo32(uint64_t v) { return (int)(uint32_t)v; }
__device__ __forceinline__ int hi32(uint64_t v) { return (int)(uint32_t)(v >> 32); }

// one lane, after its sc1 partial stores; returns true for the last of `count` arrivers
__device__ __forceinline__ bool arrive_last(uint32_t* counter, int count) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const uint32_t prev = __hip_atomic_fetch_add((gu32_t*)counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const bool last = prev == (uint32_t)(count - 1);
  if (last) __hip_atomic_store((gu32_t*)counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // next launch
  return last;
}
// wave-uniform "am I last" decided by lane 0
__device__ __forceinline__ bool wave_arrive_last(uint32_t* counter, int count) {
  int last = 0;
  if (lane_id() == 0) last = arrive_last(counter, count) ? 1 : 0;
  return lane_value(last, 0) != 0;
}

// Diagnostic stamps (fa.diag & 4 only): s_memrealtime (100 MHz).  0/4 first block start of K1/K2 (min),
// 1/5 last block partial (max), 2-3 / 6-7 top wave start/end, 8 table built, 9 weights done, 10 K2 scan
// done, 11 counts done, 12 scatter done, 13-18 finalize phases, 19 earliest table built (min).
constexpr int kStamps = 32;
// diagnostic switches (FrameArgsT::diag, pfmpe_set_option(ctx, 99, bits)); 0 in production
enum : int {
  kDiagStamps = 4,      // phase stamps (s_memrealtime) into d_stamps
  kDiagVisits = 8,      // pruned-candidate counts into d_stamps
  kDiagTreeCount = 16,  // k_frame: count barrier as a tree instead of flat
  kDiagSqrtGroups = 32, // groups of ~sqrt(nblk) blocks even when the frame fits k_frame2
  kDiagLagLoads = 64,   // k_frame2: the last block sleeps ~20 us before loading the block partials
  kDiagAbandon = 128,   // k_frame2: every block gives up its first weighing-barrier wait (recovery test)
  kDiagSortedScore = 256, // fp32: the sorted (extraction-order) score even when B >= M (A/B of score_unordered)
  kDiagNoStream = 512,     // two-launch path: never the streaming weighing pass (k_weigh_stream + k_group + k_top)
  kDiagForceStream = 1024, // two-launch path: always the streaming weighing pass (tests / A/B)
  kDiagSerialTop = 2048,   // streaming pass with > 64 groups: the one-wave k_top instead of k_top_wide (A/B)
  kDiagNoPk = 4096,        // two-launch path: never the two-particles-per-lane pass k_weigh_pk (A/B, tests)
  kDiagCorruptDesc = 8192, // pfmpe_step_multi: the first stream's descriptor is altered after its tag (test of the
                           // staging check; the altered word is a key word, never a pointer)
  kDiagNoDefer = 16384,    // two-launch frames materialise the new prior even with the kept set (A/B of deferral)
  kDiagMinSide = 65536,      // k_frame2: run the zmin scans (group_zmin2) even when no weight can be negative (tests)
  kDiagAbandonFinish = 131072,  // k_resample_owners(_multi): the finishing wave gives up before polling the arrivals
                                // (the two-launch recovery tests)
  kDiagBlockResample = 32768  // deferred two-launch frames resample with the block-per-256 k_resample instead of
                              // k_resample_owners' wave per 256 (A/B, identity tests)
};
__device__ __forceinline__ uint64_t rt_now() { return __builtin_amdgcn_s_memrealtime(); }
// per-block stamps go to the block's own row (plain stores, no contended atomics); the host reduces rows
// (min for 0/4/19, max otherwise).  Row 0 holds the single-writer stamps (top / final waves).
__device__ __forceinline__ void stamp_min(uint64_t* st, int idx, uint64_t t) {
  if (st) st[(size_t)(1 + blockIdx.x) * kStamps + idx] = t;
}
__device__ __forceinline__ void stamp_max(uint64_t* st, int idx, uint64_t t) {
  if (st) st[(size_t)(1 + blockIdx.x) * kStamps + idx] = t;
}

// ---- flat hand-off (k_frame2): sharded, monotonic arrival counters (no resets: the host tracks the running
// totals and passes this frame's bases, uint32 arithmetic that wraps consistently).  A counter set is
// kShards counters one 128-B line apart; an arrival goes to shard blk % kShards (one XCD's blocks under
// round-robin placement: speed only).  Set 0: weighing barrier (one arrival per block per iteration),
// set 1: count barrier (one per block per resampled frame).
constexpr int kShards = 8;
constexpr int kShardStride = 32;                         // uint32 words: 128 B
constexpr int kFlatCountSet = kShards * kShardStride;    // offset of set 1
constexpr int kFlatWords = 2 * kShards * kShardStride;
constexpr int kFlatMaxGroups = 8;                        // k_frame2: <= 512 blocks in groups of 64
__device__ __forceinline__ void flat_arrive(uint32_t* set, int blk) {  // one lane, after its sc1 stores
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __hip_atomic_fetch_add((gu32_t*)(set + (blk & (kShards - 1)) * kShardStride), 1u, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
}
// one wave: poll the set until its shards sum to `target` (true), or give up after ~2 s (false)
__device__ __forceinline__ bool flat_wait(const uint32_t* set, uint32_t target, uint32_t bound) {
  const int lane = lane_id();
  const uint64_t t0 = rt_now();
  for (;;) {
    uint32_t v = 0;
    if (lane < kShards)
      v = __hip_atomic_load((gu32_t*)(set + lane * kShardStride), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    uint32_t sum = 0;
#pragma unroll
    for (int k = 0; k < kShards; ++k) sum += (uint32_t)__builtin_amdgcn_readlane((int)v, k);
    if (sum == target) return true;
    if (rt_now() - t0 > bound) return false;  // PFMPE_OPT_WAIT_BOUND_US (default 2 s)
    __builtin_amdgcn_s_sleep(1);
  }
}


// ---- granule hand-offs (MI355X_MICROARCH.md / cdna_hip_programming.md Guideline 16 R2): the data IS the flag.  A
// 32-bit payload word travels in an 8-byte {payload, tag} granule written by ONE aligned write-through (sc1) store;
// the consumer re-reads granules (sc1 loads) until every tag equals the one it expects: no arrival counter, no
// drain before it, no separate load round.  Used for the flat count barrier (block 0 alone polls 2 granules per
// block).  Tags are unique per frame (FrameArgsT::gtag); the host zeroes the area at create and when its frame
// count wraps, so a stale word never carries a live tag.  (The weighing barrier keeps its counter: there every
// block reads every partial, and polling 391 blocks x 96 B of granules from every block hammered the fabric: the
// barrier took 20 us instead of 5 at C2, profiles/r05/granule_weighing_rejected.txt.)
// The flat path's area: the two parities of block partials (BlockPart, k_frame2's weighing barrier), then the count
// granules {count, index} of up to kFlatMaxGroups * kGroup blocks.
constexpr size_t kGranPartBytes = (size_t)kFlatMaxGroups * kGroup * sizeof(BlockPart);  // per parity
constexpr size_t kGranCountOff = 2 * kGranPartBytes;
constexpr size_t kGranBytes = kGranCountOff + (size_t)kFlatMaxGroups * kGroup * 16;
__device__ __forceinline__ void store_granule(uint64_t* g, uint32_t tag, uint32_t v) {
  __hip_atomic_store((gu64_t*)g, ((uint64_t)tag << 32) | v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// two granules as ONE 16-B write-through-coherent (sc1) load: {payload0, tag0, payload1, tag1}
__device__ __forceinline__ u32x4_t ld_gran2_issue(const uint64_t* p) {
  u32x4_t r;
  asm volatile("global_load_dwordx4 %0, %1, off sc1" : "=v"(r) : "v"((const char*)p) : "memory");
  return r;
}

// ============================================================================== kernels
// ---- blob table (DESIGN.md "Exact blob pruning"), built once per frame on the host (build_blob_table_host,
// O(B)) and copied whole into each block's LDS by the weighing kernels.  Layout, every part 16-byte aligned:
//   base  hdr {T xmin, inv_bw, b0x, b0y} | int32 bstart[nb+1] | BlobXY<T> xy[B] | int32 orig[B]
//         (the blobs grouped into nb = bucket_count(B) x-buckets, increasing original index within a bucket;
//         every blob once: the linear scans of pose_pairs / k_resample_final and the fp64 pruned minima)
//   grid  GridHdr | uint32 cell[ncell] (byte offset of the list in ent[] | count << 16) | GridEnt ent[nent + 1]
//         (fp32 tables: a 2D cell grid over the blobs' bounding box widened by the pruning half-window; cell c
//         lists every blob whose +-tolq box (plus 0.01 px) overlaps it, so a marker's candidates are ONE
//         cell's list.  ent[0] is a sentinel {+inf, +inf, 0}: an empty cell points at it, so every query reads
//         one entry without a test.  ncell = 0: no grid, the x-buckets serve; fp64 tables and large B never
//         build one)
__host__ __device__ constexpr size_t align16(size_t x) { return (x + 15) / 16 * 16; }
struct GridHdr {
  float inv_c, gx0, gy0, pad0;     // cell of (u, v): ((u - gx0) * inv_c, (v - gy0) * inv_c), clamped
  float fmaxx, fmaxy;              // ncx - 1, ncy - 1
  float gtolq;                     // half-window the lists were built for (>= the frame's tolq to be used)
  int32_t ncx, ncell, nent;        // columns, cells, list entries
  int32_t b0fin, pad;              // blob 0 finite (every table, grid or not)
};
static_assert(sizeof(GridHdr) == 48, "grid header");
// The cell budget of a table's grid: the coarse one (2,048 cells, 8 KB of records) for ordinary blob counts, the 4x
// finer one (8,192, 32 KB) from kGridFineMinBlobs blobs (C3's 200 with clutter), whose cell lists are otherwise long
// enough that most waves walk them: measured (profiles/r06/ab_grid_cells.txt) C3 weighing 56.5 -> 50.8 us with the
// fine grid, while at 50 blobs (C2 / C4 / C5) its larger table copy costs 1.5-1.8 us per frame.  A fine grid over the
// entry budget falls back to the coarse one, then to the x-buckets.
constexpr int kGridMaxCells = 8192;   // cell records: 32 KB
constexpr int kGridCoarseCells = 2048;
#ifndef PFMPE_GRID_FINE_MIN_BLOBS
#define PFMPE_GRID_FINE_MIN_BLOBS 128
#endif
constexpr int kGridFineMinBlobs = PFMPE_GRID_FINE_MIN_BLOBS;
constexpr int kGridMaxEntries = 1024; // list entries: 16 KB (B up to ~400 blobs at 2-3 cells each)
template <typename T>
struct BlobTable {
  static constexpr size_t off_bstart() { return align16(4 * sizeof(T)); }
  static constexpr size_t off_xy(int B) { return off_bstart() + align16((size_t)(bucket_count(B) + 1) * 4); }
  static constexpr size_t off_orig(int B) { return off_xy(B) + align16((size_t)B * sizeof(BlobXY<T>)); }
  // the base part (every blob once): all the linear scans need
  static constexpr size_t bytes(int B) { return off_orig(B) + align16((size_t)B * 4); }
  static constexpr size_t off_grid(int B) { return bytes(B); }
  static constexpr size_t grid_bytes(int ncell, int nent) {
    return sizeof(GridHdr) + align16((size_t)ncell * 4) + (size_t)(nent + 1) * sizeof(GridEnt);
  }
  // a table's total size: base + grid (the host builder returns it; FrameArgsT::tbytes carries it)
  static constexpr size_t total_bytes(int B, int ncell, int nent) { return bytes(B) + grid_bytes(ncell, nent); }
  static constexpr size_t max_bytes() { return total_bytes(kMaxBlobs, kGridMaxCells, kGridMaxEntries); }
  // LDS of the weighing kernels: the table plus one 16-B granule, so the masked second candidate of the
  // fp32 column_minima steps (x-buckets, grid lists) reads inside the allocation
  static constexpr size_t lds_bytes(size_t tbytes) { return tbytes + 16; }
};

template <typename T>
struct LdsBlobs {
  const unsigned char* base;  // the table (the grid's parts sit at FrameArgsT::grid offsets from it)
  const BlobXY<T>* bxy;
  const int32_t* orig;
  const int32_t* bstart;  // nb + 1
  T xmin, inv_bw;  // blob 0 (header words 2, 3): read where needed (nan_at_origin_tb)
  int nb;
};

template <typename T>
__host__ __device__ __forceinline__ LdsBlobs<T> view_table(const unsigned char* base, int B) {
  LdsBlobs<T> t;
  const T* hdr = (const T*)base;
  t.base = base;
  t.xmin = hdr[0];
  t.inv_bw = hdr[1];
  t.nb = bucket_count(B);
  t.bstart = (const int32_t*)(base + BlobTable<T>::off_bstart());
  t.bxy = (const BlobXY<T>*)(base + BlobTable<T>::off_xy(B));
  t.orig = (const int32_t*)(base + BlobTable<T>::off_orig(B));
  return t;
}

// The kernel arguments of a table's grid (host): on only when the table has a grid built for at least the
// frame's window (tolq: FrameArgsT::tolq of the frame).  gh: the table's GridHdr (at off_grid(B)).
template <typename T>
inline GridArgs grid_args(const GridHdr& gh, int B, float tolq) {
  GridArgs g{};
  g.b0fin = gh.b0fin;
  g.on = (gh.ncell > 0 && gh.gtolq >= tolq) ? 1 : 0;
  if (!g.on) return g;
  g.inv_c = gh.inv_c;
  g.ox = (float)(-(double)gh.gx0 * (double)gh.inv_c);  // build_blob_table_host's proof covers this rounding
  g.oy = (float)(-(double)gh.gy0 * (double)gh.inv_c);
  g.fmaxx = gh.fmaxx;
  g.fmaxy = gh.fmaxy;
  g.ncx4 = 4 * gh.ncx;
  g.cell_off = (int32_t)(BlobTable<T>::off_grid(B) + sizeof(GridHdr));
  g.ent_off = g.cell_off + (int32_t)align16((size_t)gh.ncell * 4);
  return g;
}

// Host builder; returns the table's size in bytes.  The bucket formula is bucket_of in T arithmetic (this TU:
// -ffp-contract=off), the same expression the kernels evaluate for their query windows.  tolq: the pruning
// half-window of the frames that will use the table (FrameArgsT::tolq, from tol_PF).
template <typename T>
inline size_t build_blob_table_host(const double* blobs, int B, double tolq, unsigned char* dst) {
  T xmin = (T)INFINITY, xmax = -(T)INFINITY;
  for (int i = 0; i < B; ++i) {
    const T x = (T)blobs[2 * i];
    xmin = x < xmin ? x : xmin;
    xmax = x > xmax ? x : xmax;
  }
  if (B == 0 || !(xmax - xmin < (T)INFINITY)) {
    xmin = (T)0;
    xmax = (T)1;
  }
  T span = xmax - xmin;
  if (!(span > (T)0)) span = (T)1;
  const int nb = bucket_count(B);
  const T inv_bw = (T)nb / span;
  T* hdr = (T*)dst;
  hdr[0] = xmin;
  hdr[1] = inv_bw;
  hdr[2] = B > 0 ? (T)blobs[0] : (T)0;
  hdr[3] = B > 0 ? (T)blobs[1] : (T)0;
  int32_t* bstart = (int32_t*)(dst + BlobTable<T>::off_bstart());
  BlobXY<T>* xy = (BlobXY<T>*)(dst + BlobTable<T>::off_xy(B));
  int32_t* orig = (int32_t*)(dst + BlobTable<T>::off_orig(B));
  int32_t cnt[kMaxBuckets + 1] = {0};
  for (int i = 0; i < B; ++i) ++cnt[bucket_of((T)blobs[2 * i], xmin, inv_bw, nb) + 1];
  for (int b = 0; b < nb; ++b) cnt[b + 1] += cnt[b];
  for (int b = 0; b <= nb; ++b) bstart[b] = cnt[b];
  for (int i = 0; i < B; ++i) {
    const int pos = cnt[bucket_of((T)blobs[2 * i], xmin, inv_bw, nb)]++;
    xy[pos].x = (T)blobs[2 * i];
    xy[pos].y = (T)blobs[2 * i + 1];
    orig[pos] = i;
  }
  // ---- the grid (fp32 tables).  Device query: cell coordinate f = fma(u, inv_c, ox), ox = fl(-gx0 * inv_c),
  // clamped by med3 to [0, ncx - 1], truncated.  Every blob within tol_PF of a query must be in the query's
  // cell list:
  //  * a blob is listed in every cell whose real-arithmetic interval [g(bx - m), g(bx + m)] it overlaps,
  //    g(x) = (x - gx0) * inv_c with the fp32 constants the device uses, m = tolq + 0.01 px;
  //  * the device's f differs from g(u) by the rounding of ox and of the fma (cell coordinates < 2^7: a few
  //    1e-6 cells, 1e-4 px), far below the m - tol_PF >= 0.01 px slack; a clamped query (outside the widened
  //    box) has no blob within tolq at all, so whatever its cell lists, its minimum fails the gate;
  //  * every blob's own interval is clamped to the grid the same way.
  // Each list holds its blobs in increasing original index (the fill below runs over i), so the device's
  // strict "closer" comparison keeps the lowest index among equally close blobs: the reference's tie rule.
  GridHdr* gh = (GridHdr*)(dst + BlobTable<T>::off_grid(B));
  std::memset(gh, 0, sizeof(GridHdr));
  gh->b0fin = (B > 0 && std::isfinite((double)hdr[2]) && std::isfinite((double)hdr[3])) ? 1 : 0;
  size_t total = BlobTable<T>::total_bytes(B, 0, 0);
  if (!std::is_same<T, float>::value || B == 0) return total;
  const double m = tolq + 0.01;
  double bx0 = INFINITY, bx1 = -INFINITY, by0 = INFINITY, by1 = -INFINITY;
  for (int i = 0; i < B; ++i) {
    const double x = (double)(float)blobs[2 * i], y = (double)(float)blobs[2 * i + 1];
    if (!(x - x == 0.0) || !(y - y == 0.0)) return total;  // a non-finite blob: no grid
    bx0 = std::min(bx0, x), bx1 = std::max(bx1, x), by0 = std::min(by0, y), by1 = std::max(by1, y);
  }
  const double gx0 = bx0 - m, gy0 = by0 - m, w = bx1 - bx0 + 2 * m, h = by1 - by0 + 2 * m;
  for (int budget = B >= kGridFineMinBlobs ? kGridMaxCells : kGridCoarseCells;; budget = kGridCoarseCells) {
  // square cells: at least the window (2m) and few enough for the cell budget
  double cs = std::max(2.0 * m, std::sqrt(w * h / (double)budget));
  int ncx = (int)std::ceil(w / cs), ncy = (int)std::ceil(h / cs);
  while ((int64_t)ncx * ncy > budget) {
    cs *= 1.0625;
    ncx = (int)std::ceil(w / cs);
    ncy = (int)std::ceil(h / cs);
  }
  ncx = std::max(1, ncx);
  ncy = std::max(1, ncy);
  const float inv_c = (float)(1.0 / cs), gx0f = (float)gx0, gy0f = (float)gy0;
  // The device's cell coordinate fma(u, inv_c, ox) rounds twice (ox = fl(-gx0 * inv_c), then the fma), each by at
  // most half an ulp of a value below |ox| + ncx cells, i.e. 2^-24 (|ox| + ncx) cells of cs px.  The lists hold
  // every blob within m = tolq + 0.01 px of a cell, so the proof needs that error well inside m - tolq = 0.01 px:
  // far-out blob coordinates (|gx0| ~ 1e5 px and beyond) make |ox| large, and then the x-buckets
  // serve instead of the grid.
  {
    const double ex = std::ldexp(std::abs((double)gx0f) * (double)inv_c + ncx + 1.0, -23) * cs;
    const double ey = std::ldexp(std::abs((double)gy0f) * (double)inv_c + ncy + 1.0, -23) * cs;
    if (!(std::max(ex, ey) <= 0.25 * (m - tolq))) return total;
  }
  auto crange = [&](double lo, double hi, float inv, float org, int n, int& c0, int& c1) {
    const double f0 = (lo - (double)org) * (double)inv, f1 = (hi - (double)org) * (double)inv;
    c0 = (int)std::max(0.0, std::min((double)(n - 1), std::floor(f0)));
    c1 = (int)std::max(0.0, std::min((double)(n - 1), std::floor(f1)));
  };
  const int ncell = ncx * ncy;
  std::vector<int32_t> count(ncell + 1, 0);
  int nent = 0;
  for (int pass = 0; pass < 2; ++pass) {
    std::vector<int32_t> fill;
    if (pass == 1) {
      for (int c = 0; c < ncell; ++c) count[c + 1] += count[c];
      fill.assign(count.begin(), count.end() - 1);
    }
    for (int i = 0; i < B; ++i) {
      const double x = (double)(float)blobs[2 * i], y = (double)(float)blobs[2 * i + 1];
      int cx0, cx1, cy0, cy1;
      crange(x - m, x + m, inv_c, gx0f, ncx, cx0, cx1);
      crange(y - m, y + m, inv_c, gy0f, ncy, cy0, cy1);
      for (int cy = cy0; cy <= cy1; ++cy)
        for (int cx = cx0; cx <= cx1; ++cx) {
          const int c = cy * ncx + cx;
          if (pass == 0) {
            ++count[c + 1];
            ++nent;
          } else {
            const int e = 1 + fill[c]++;  // ent[0]: the sentinel
            GridEnt* ent = (GridEnt*)((unsigned char*)gh + sizeof(GridHdr) + align16((size_t)ncell * 4));
            ent[e] = GridEnt{(float)blobs[2 * i], (float)blobs[2 * i + 1], i, 0};
          }
        }
    }
    if (pass == 0 && nent > kGridMaxEntries) break;  // too many entries: a coarser grid, then the x-buckets
  }
  if (nent > kGridMaxEntries) {
    if (budget == kGridCoarseCells) return total;
    continue;
  }
  uint32_t* cell = (uint32_t*)((unsigned char*)gh + sizeof(GridHdr));
  for (int c = 0; c < ncell; ++c) {  // an empty cell points at the sentinel (byte offset 0)
    const uint32_t n = (uint32_t)(count[c + 1] - count[c]);
    cell[c] = (n ? (uint32_t)(1 + count[c]) * (uint32_t)sizeof(GridEnt) : 0u) | (n << 16);
  }
  GridEnt* ent = (GridEnt*)((unsigned char*)cell + align16((size_t)ncell * 4));
  ent[0] = GridEnt{INFINITY, INFINITY, 0, 0};  // sentinel: distance +inf (NaN for a non-finite query), index 0

  gh->inv_c = inv_c;
  gh->gx0 = gx0f;
  gh->gy0 = gy0f;
  gh->fmaxx = (float)(ncx - 1);
  gh->fmaxy = (float)(ncy - 1);
  gh->gtolq = (float)tolq;
  gh->ncx = ncx;
  gh->ncell = ncell;
  gh->nent = nent;
  return BlobTable<T>::total_bytes(B, ncell, nent);
  }
}

// block-wide copy of the table into LDS (16-byte words); callers barrier before use
__device__ __forceinline__ void copy_table(const unsigned char* __restrict__ src, unsigned char* dst, size_t bytes) {
  // global loads (src may come from a batched launch's stream descriptor, which hides its address space)
  typedef __attribute__((address_space(1))) const u32x4_t gv4_t;
  gv4_t* s4 = (gv4_t*)src;
  u32x4_t* d4 = (u32x4_t*)dst;
  const int n4 = (int)(bytes / 16);
  for (int i = threadIdx.x; i < n4; i += kBlock) d4[i] = s4[i];
}

// copy_table + stage_consts_from with every load issued before the first LDS store: one memory round trip for the
// table (its first 8 KB: two 16-B loads per thread), the frame constants and whatever the caller issued before
// (k_frame2: the prior), instead of one per loop and per copy
template <typename T>
__device__ __forceinline__ void stage_table_consts(const unsigned char* __restrict__ src, unsigned char* dst, size_t bytes,
                                                   const uint32_t* cw_src, LdsConst<T>& sc) {
  typedef __attribute__((address_space(1))) const u32x4_t gv4_t;
  gv4_t* s4 = (gv4_t*)src;
  u32x4_t* d4 = (u32x4_t*)dst;
  const int n4 = (int)(bytes / 16);
  const int t = threadIdx.x;
  constexpr int kWordsC = (int)(sizeof(LdsConst<T>) / 4);
  static_assert(kWordsC <= kBlock, "one constant word per thread");
  u32x4_t r0 = {0u, 0u, 0u, 0u}, r1 = {0u, 0u, 0u, 0u};
  uint32_t cw = 0u;
  if (t < n4) r0 = s4[t];
  if (t + kBlock < n4) r1 = s4[t + kBlock];
  if (t < kWordsC) cw = cw_src[t];
  if (t < n4) d4[t] = r0;
  if (t + kBlock < n4) d4[t + kBlock] = r1;
  if (t < kWordsC) ((uint32_t*)&sc)[t] = cw;
  for (int i = t + 2 * kBlock; i < n4; i += kBlock) d4[i] = s4[i];  // tables past 8 KB (large B)
}

// Control record / scan records move between blocks of one launch (and, in k_frame, between the
// iterations of one launch) through write-through words only.
__device__ __forceinline__ Ctrl load_ctrl_wt(const Ctrl* __restrict__ ctrl) {
  static_assert(sizeof(Ctrl) % 8 == 0, "Ctrl words");
  Ctrl c;
  uint64_t* d = (uint64_t*)&c;
#pragma unroll
  for (int q = 0; q < (int)(sizeof(Ctrl) / 8); ++q) d[q] = ld_wt((const uint64_t*)ctrl + q);
  return c;
}
// The control record as written by the previous launch, in scalar registers, by scalar loads: the address is
// wave-uniform (a kernel argument, or read from a batched launch's stream descriptor, where the compiler would
// otherwise issue vector loads that wait behind the block's earlier vector loads in vmcnt order).  Scalar
// loads are safe here: the record was written by an earlier launch (the scalar cache starts each dispatch
// invalidated) and this launch writes it only after every read.  Decisions on it stay scalar branches and
// buffer resources built from it stay in SGPRs (no waterfall loops).
typedef uint32_t u32x16_t __attribute__((ext_vector_type(16)));
// one dword of the control record by a scalar load (same conditions as load_ctrl_uniform)
template <int OFF>
__device__ __forceinline__ int load_ctrl_word(const Ctrl* __restrict__ ctrl) {
  int v;
  asm volatile("s_load_dword %0, %1, %2\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(ctrl), "i"(OFF) : "memory");
  return v;
}
__device__ __forceinline__ Ctrl load_ctrl_uniform(const Ctrl* __restrict__ ctrl) {
  static_assert(sizeof(Ctrl) == 80, "Ctrl = 16 + 4 dwords");
  u32x16_t a;
  u32x4_t b;
  asm volatile("s_load_dwordx16 %0, %2, 0x0\n\ts_load_dwordx4 %1, %2, 0x40\n\ts_waitcnt lgkmcnt(0)"
               : "=s"(a), "=s"(b)
               : "s"(ctrl)
               : "memory");
  Ctrl c;
  uint32_t* d = (uint32_t*)&c;
#pragma unroll
  for (int q = 0; q < 16; ++q) d[q] = a[q];
#pragma unroll
  for (int q = 0; q < 4; ++q) d[16 + q] = b[q];
  return c;
}
__device__ __forceinline__ void store_ctrl_wt(Ctrl* __restrict__ ctrl, const Ctrl& c) {
  const uint64_t* s = (const uint64_t*)&c;
#pragma unroll
  for (int q = 0; q < (int)(sizeof(Ctrl) / 8); ++q) st_wt((uint64_t*)ctrl + q, s[q]);
}
__device__ __forceinline__ Ctrl zero_ctrl() {
  Ctrl z;
  z.best_max = 0.0;
  z.S = 0.0;
  z.invS = 0.0;
  z.done = z.has_best = z.best_idx = z.best_iter = z.best_slot = z.cur_slot = 0;
  z.iters = z.kept_slot = z.kept_iter = z.accepted = z.most_likely_idx = z.pad0 = 0;
  z.K_total = 0;
  return z;
}
__device__ __forceinline__ BlockScan load_bscan_wt(const BlockScan* p) {
  BlockScan s;
  s.E = ld_wt_d(&p->E);
  s.zin_max = ld_wt_d(&p->zin_max);
  s.zin_min = ld_wt_d(&p->zin_min);
  s.pad = 0.0;
  return s;
}
__device__ __forceinline__ GroupScan load_gscan_wt(const GroupScan* p) {
  GroupScan s;
  s.G = ld_wt_d(&p->G);
  s.Gin = ld_wt_d(&p->Gin);
  return s;
}

// ---- group wave of the weighing pass: the fa.gsz blocks of group g, 64 per tile (one per lane).
// Exclusive in-group prefixes E_b are carried across tiles, and so are the exclusive running extrema of
// z = fl(E_b + in-block prefix) (any fixed association works: k_resample evaluates every c_i and every
// block-start running max from these same stored E_b).  Returns the group partial.
// W4 (k_group after the streaming pass): `part` holds kWaves wave partials per block (BlockPart fields: wave
// total, max / min in-wave prefix, max / argmax, min / argmin), combined here into the block partial with
// publish_iteration's association (((0 + t0) + t1) + ..., the running extrema of pre + prefix, waves in order).
// W4: the partials are wave partials (four per block, the streaming passes)
template <bool W4 = false>
__device__ __forceinline__ GroupPart propagate_group(int nblk, int gsz, int g, const BlockPart* __restrict__ part,
                                                     BlockScan* __restrict__ bscan, GroupPart* __restrict__ gpart) {
  const int lane = lane_id();
  const int b0 = g * gsz;
  const int nb = min(gsz, nblk - b0);
  double cE = 0.0, cmax = -INFINITY, cmin = INFINITY;  // carries
  double maxw = -INFINITY, minw = INFINITY;
  int amax = 0x7fffffff, amin = 0x7fffffff;
  for (int t = 0; t < nb; t += 64) {  // one tile unless gsz > 64
    const int b = b0 + t + lane;
    const bool vb = t + lane < nb;
    double sum = 0.0, maxrel = -INFINITY, minrel = INFINITY;
    if (vb && W4) {  // written by the previous launch: plain loads
      const BlockPart* p = part + (size_t)b * kWaves;
      BlockPart w[kWaves];
#pragma unroll
      for (int ww = 0; ww < kWaves; ++ww) w[ww] = p[ww];
      double pre = 0.0, bmx = w[0].maxw, bmn = w[0].minw;
      int bix = w[0].argmax, bin = w[0].argmin;
#pragma unroll
      for (int ww = 0; ww < kWaves; ++ww) {
        const double a = pre + w[ww].maxrel, c = pre + w[ww].minrel;
        maxrel = a > maxrel ? a : maxrel;
        minrel = c < minrel ? c : minrel;
        if (ww) {
          cmb_max(bmx, bix, w[ww].maxw, w[ww].argmax);
          cmb_min(bmn, bin, w[ww].minw, w[ww].argmin);
        }
        pre = pre + w[ww].sum;
      }
      sum = pre;
      cmb_max(maxw, amax, bmx, bix);
      cmb_min(minw, amin, bmn, bin);
    } else if (vb) {
      const BlockPart* p = part + b;
      sum = ld_wt_d(&p->sum);
      maxrel = ld_wt_d(&p->maxrel);
      minrel = ld_wt_d(&p->minrel);
      const uint64_t ai = ld_wt(&p->argmax);
      cmb_max(maxw, amax, ld_wt_d(&p->maxw), lo32(ai));
      cmb_min(minw, amin, ld_wt_d(&p->minw), hi32(ai));
    }
    const double incl = wave_incl_sum(sum);
    const double E = cE + wave_shr1(incl, 0.0);  // exclusive prefix within the group
    const double zmax = vb ? E + maxrel : -INFINITY;
    const double zmin = vb ? E + minrel : INFINITY;
    const double zi_max = wave_incl_max(zmax), zi_min = wave_incl_min(zmin);
    double zp_max = wave_shr1(zi_max, -(double)INFINITY), zp_min = wave_shr1(zi_min, (double)INFINITY);
    zp_max = zp_max > cmax ? zp_max : cmax;
    zp_min = zp_min < cmin ? zp_min : cmin;
    if (vb) {
      BlockScan* s = bscan + b;
      st_wt_d(&s->E, E);
      st_wt_d(&s->zin_max, zp_max);
      st_wt_d(&s->zin_min, zp_min);
    }
    cE = cE + lane_value(incl, 63);
    const double tmax = lane_value(zi_max, 63), tmin = lane_value(zi_min, 63);
    cmax = tmax > cmax ? tmax : cmax;
    cmin = tmin < cmin ? tmin : cmin;
  }
  wave_argmax(maxw, amax);
  wave_argmin(minw, amin);
  GroupPart r;
  r.sum = cE;
  r.zmax = cmax;
  r.zmin = cmin;
  r.maxw = maxw;
  r.minw = minw;
  r.argmax = amax;
  r.argmin = amin;
  if (lane == 0) {
    GroupPart* gp = gpart + g;
    st_wt_d(&gp->sum, r.sum);
    st_wt_d(&gp->zmax, r.zmax);
    st_wt_d(&gp->zmin, r.zmin);
    st_wt_d(&gp->maxw, r.maxw);
    st_wt_d(&gp->minw, r.minw);
    st_wt(&gp->argmax, pack2(amax, amin));
  }
  return r;
}

// group partial g of a weight slot: from memory, or (single-group frames) this iteration's values still
// in registers
__device__ __forceinline__ GroupPart group_part(const GroupPart* __restrict__ gp, int g, const GroupPart& regs,
                                                bool use_regs) {
  if (use_regs) return regs;
  GroupPart r;
  r.sum = ld_wt_d(&gp[g].sum);
  r.zmax = ld_wt_d(&gp[g].zmax);
  r.zmin = ld_wt_d(&gp[g].zmin);
  r.maxw = ld_wt_d(&gp[g].maxw);
  r.minw = ld_wt_d(&gp[g].minw);
  const uint64_t ai = ld_wt(&gp[g].argmax);
  r.argmax = lo32(ai);
  r.argmin = hi32(ai);
  return r;
}

// ---- top wave of the weighing pass: iteration bookkeeping, exit rule, group prefixes, accept.  Reads
// and writes the control record through write-through words.  `gen` (k_frame only) is written last, after
// everything this wave wrote has drained: the value gen_base + iter + 1 releases the blocks waiting for
// this iteration's outcome (gen_base = frame sequence << 16, so no stale value can match).
// cur: this iteration's group partial when the frame has a single group (the group wave is the top).
template <typename T, int RNG>
__device__ __forceinline__ void propagate_top(const FrameArgsT<T>& fa, Ctrl* __restrict__ ctrl, int iter,
                                              const GroupPart* __restrict__ gp0, const GroupPart* __restrict__ gp1,
                                              GroupScan* __restrict__ gscan, uint32_t* __restrict__ gen,
                                              uint32_t gen_base, const GroupPart cur, bool have_cur, int slot,
                                              const GroupPart* lds_cur = nullptr) {
  const int lane = lane_id();
  const int ngrp = fa.ngrp;
  // <= 64 groups: each lane's group partial of this iteration is loaded ONCE, in the same round trip as
  // the control record, and serves every pass below
  const bool one_tile = ngrp <= 64;
  GroupPart q0;
  q0.sum = 0.0;
  q0.zmax = -INFINITY;
  q0.zmin = INFINITY;
  q0.maxw = -INFINITY;
  q0.minw = INFINITY;
  q0.argmax = q0.argmin = 0x7fffffff;
  if (one_tile && lane < ngrp) q0 = group_part(slot ? gp1 : gp0, lane, cur, have_cur);
  const Ctrl c0 = load_ctrl_wt(ctrl);
  // this iteration's max / first argmax
  double mv = -INFINITY;
  int mi = 0x7fffffff;
  if (one_tile) {
    mv = q0.maxw;
    mi = q0.argmax;
  } else {
    const GroupPart* P = slot ? gp1 : gp0;
    for (int g = lane; g < ngrp; g += 64) {
      const GroupPart q = lds_cur ? lds_cur[g] : group_part(P, g, cur, have_cur);
      cmb_max(mv, mi, q.maxw, q.argmax);
    }
  }
  wave_argmax(mv, mi);
  Ctrl c = c0;
  if (mv > c.best_max) {  // strict: PE:608
    c.best_max = mv;
    c.best_idx = mi;
    c.best_iter = iter;
    c.best_slot = slot;
    c.has_best = 1;
  }
  c.iters = iter + 1;
  const bool go_on = fa.force_iters > 0 ? (c.iters < fa.force_iters)
                                        : (c.iters < fa.max_iter && mv < fa.exit_thr);  // PE:616
  c.cur_slot = c.has_best ? 1 - c.best_slot : 1 - slot;
  if (!go_on) {
    c.done = 1;
    c.kept_slot = c.has_best ? c.best_slot : slot;
    c.kept_iter = c.has_best ? c.best_iter : iter;
    const GroupPart* KG = c.kept_slot ? gp1 : gp0;
    const bool kreg = have_cur && c.kept_slot == slot;
    // kept slot's partials of a one-tile frame: this iteration's (registers) or an earlier one's (load)
    GroupPart kq = q0;
    if (one_tile && c.kept_slot != slot && lane < ngrp) kq = group_part(KG, lane, cur, kreg);
    const bool kept_lds = lds_cur && c.kept_slot == slot;  // this iteration's parts, staged in LDS
    auto kept_part = [&](int g) -> GroupPart {
      return one_tile ? kq : (kept_lds ? lds_cur[g] : group_part(KG, g, cur, kreg));
    };

    // S = total over groups (tiles of 64 groups, carried)
    double carry = 0.0;
    for (int base = 0; base < ngrp; base += 64) {
      const int g = base + lane;
      const double s = g < ngrp ? kept_part(g).sum : 0.0;
      carry = carry + lane_value(wave_incl_sum(s), 63);
    }
    const double S = carry;
    // group prefixes G_g (same association as above, recomputed) and the running max of c at each group
    // start: Gin_g = max over earlier groups of fl(fl(G + z)/S)
    double run = -INFINITY;
    carry = 0.0;
    for (int base = 0; base < ngrp; base += 64) {
      const int g = base + lane;
      GroupPart q;
      q.sum = 0.0;
      q.zmax = -INFINITY;
      q.zmin = INFINITY;
      if (g < ngrp) q = kept_part(g);
      const double incl = wave_incl_sum(q.sum);
      const double prev = wave_shr1(incl, 0.0);
      const double G = lane == 0 ? carry : carry + prev;
      carry = carry + lane_value(incl, 63);
      double cm = -INFINITY;
      if (g < ngrp && S != 0.0) cm = (G + (S > 0.0 ? q.zmax : q.zmin)) / S;
      const double im = wave_incl_max(cm);
      double ex = wave_shr1(im, -(double)INFINITY);
      ex = ex > run ? ex : run;
      if (g < ngrp) {
        st_wt_d(&gscan[g].G, G);
        st_wt_d(&gscan[g].Gin, ex);
      }
      const double tm = lane_value(im, 63);
      run = tm > run ? tm : run;
    }
    if (S == 0.0) run = -INFINITY;
    // kept iteration's argmax / argmin (re-init branch, PE:714)
    double amv = -INFINITY, anv = INFINITY;
    int ami = 0x7fffffff, ani = 0x7fffffff;
    for (int g = lane; g < ngrp; g += 64) {
      const GroupPart q = kept_part(g);
      cmb_max(amv, ami, q.maxw, q.argmax);
      cmb_min(anv, ani, q.minw, q.argmin);
    }
    wave_argmax(amv, ami);
    wave_argmin(anv, ani);
    const double highest = c.has_best ? c.best_max : 0.0;
    c.S = S;
    c.invS = 1.0 / S;
    c.accepted = (S != 0.0 && highest > fa.accept_thr) ? 1 : 0;  // PE:633
    if (c.accepted) {
      c.most_likely_idx = c.best_idx;
      c.K_total = lane == 0 ? count_targets<T, RNG>(fa, c.iters, run) : 0;
    } else {
      // argmax of the normalised weights (PE:714): a negative sum flips the order
      c.most_likely_idx = (S < 0.0) ? ani : ami;
      c.K_total = 0;
    }
  }
  if (lane == 0) {
    store_ctrl_wt(ctrl, c);
    if (gen) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // ctrl / gscan words drained before the release
      __hip_atomic_store((gu32_t*)gen, gen_base + (uint32_t)iter + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// ---- one particle through the motion model, projection and likelihood (PE:543-604, PE:2385)
template <typename T, int RNG, int MAXM, bool PRUNE, bool PHASED = false>
__device__ __forceinline__ T weigh_particle(const FrameArgsT<T>& fa, const LdsConst<T>& sc, const LdsBlobs<T>& tb,
                                            const T* A, int n, int iter, T* P, int* nvisit = nullptr,
                                            uint64_t* st = nullptr) {
  T u[MAXM], v[MAXM];
  propagate<T, RNG>(fa, sc, A, n, iter, P);
  if (st && threadIdx.x == 0) stamp_max(st, 27, rt_now() + (P[11] == (T)12345 ? 1 : 0));
  project_markers<T, MAXM>(fa, sc, P, u, v);
  if (st && threadIdx.x == 0) stamp_max(st, 28, rt_now() + (u[0] == (T)12345 ? 1 : 0));
  T w = (T)0;
  if (fa.B > 0 && !nan_at_origin_tb(fa, tb, u[0], v[0])) {
    T m[MAXM];
    int r[MAXM];
    const int visited = column_minima<T, MAXM, PRUNE, PHASED>(fa, u, v, tb, m, r);
    if (nvisit) *nvisit = visited;
    if (st && threadIdx.x == 0) stamp_max(st, 29, rt_now() + (m[0] == (T)12345 ? 1 : 0));
    if constexpr (std::is_same<T, float>::value) {
      if (fa.B >= fa.M && !(fa.diag & kDiagSortedScore))  // wave-uniform
        w = score_unordered<MAXM>(fa, m, r);
      else
        w = score_minima<T, MAXM, false>(fa, m, r, nullptr, nullptr);
    } else {
      w = score_minima<T, MAXM, false>(fa, m, r, nullptr, nullptr);
    }
  }
  return w;
}

// A wave's weight partials (the wave-inclusive scan wi of the weights, the extrema of wi over valid lanes,
// max / argmax and min / argmin of the weights); the extrema and arg results are wave-uniform.
//  * max / min of the weights: value-only DPP reductions (max and min do not round, so any order is exact),
//    interleaved with the sum scan; argmax / argmin = the first valid lane holding that value (ballot),
//    i.e. the lowest particle index, exactly the lexicographic (value, index) order of cmb_max / cmb_min.
//  * min / argmin are only needed on the re-initialisation branch when the weight sum is negative (PE:714:
//    the most likely particle is the argmax of the normalised weights), and then the global minimum is
//    negative and lies in a wave holding a negative weight.  So a wave without negative weights reports
//    (+inf, none) and skips the min reduction (wave-uniform branch): the global argmin is unchanged.
//  * extrema of wi: when no valid weight is negative the DPP prefix is non-decreasing over the lanes (each
//    row_shr / row_bcast step adds a non-negative, lane-monotone addend, and rounding is monotone), so the
//    maximum is lane 63's total and the minimum lane 0's value (valid lanes are a prefix of the wave).
//    Only a wave holding a negative weight runs the two prefix max/min scans.
// Wave totals through a butterfly instead of a scan (fp32 weighing passes, where only lane 63's inclusive sum is
// needed).  quad_perm [1,0,3,2], quad_perm [2,3,0,1], row_half_mirror and row_mirror leave every lane of a quad /
// half-row / row holding the same pairwise-tree value that wave_scan's row_shr 1/2/4/8 steps leave in the last lane
// of each (lane 15 after shr8 = O1 + O0 = what lane 15 receives from lane 0 under row_mirror; fp addition is
// commutative bit for bit), and the two row_bcast steps are wave_scan's own.  So lane 63 holds exactly wave_scan's
// lane-63 value.  Every lane is a source in the first four steps (no fill value, no register init per step);
// the bcast steps leave the rows they do not write holding garbage, which no caller reads.
enum : int { kDppQuadXor1 = 0xB1, kDppQuadXor2 = 0x4E, kDppRowMirror = 0x140, kDppRowHalfMirror = 0x141 };
template <int CTRL, int RM = 0xf>
__device__ __forceinline__ double dpp_any(double x) {
  const uint64_t v = (uint64_t)__double_as_longlong(x);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)v, CTRL, RM, 0xf, false);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)(v >> 32), CTRL, RM, 0xf, false);
  return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
__device__ __forceinline__ double wave_total_lane63(double x) {
  x = x + dpp_any<kDppQuadXor1>(x);
  x = x + dpp_any<kDppQuadXor2>(x);
  x = x + dpp_any<kDppRowHalfMirror>(x);
  x = x + dpp_any<kDppRowMirror>(x);
  x = x + dpp_any<kDppBcast15, 0xa>(x);
  x = x + dpp_any<kDppBcast31, 0xc>(x);
  return x;
}
// max of a float over the wave as order-preserving integers (v_max_i32: no NaN canonicalisation per step; the
// weights are never NaN); the result is the maximum's exact bits.  Rows are combined by the two row broadcasts.
__device__ __forceinline__ int f32_sortable(float f) {
  const int b = (int)__float_as_uint(f);
  return b ^ ((b >> 31) & 0x7fffffff);
}
__device__ __forceinline__ float wave_max_f32(float x) {
  int k = f32_sortable(x);
  k = max(k, __builtin_amdgcn_mov_dpp(k, kDppQuadXor1, 0xf, 0xf, true));  // (folds into v_max_i32_dpp)
  k = max(k, __builtin_amdgcn_mov_dpp(k, kDppQuadXor2, 0xf, 0xf, true));
  k = max(k, __builtin_amdgcn_mov_dpp(k, kDppRowHalfMirror, 0xf, 0xf, true));
  k = max(k, __builtin_amdgcn_mov_dpp(k, kDppRowMirror, 0xf, 0xf, true));
  k = max(k, dpp<kDppBcast15, 0xa>(k, INT_MIN));
  k = max(k, dpp<kDppBcast31, 0xc>(k, INT_MIN));
  k = __builtin_amdgcn_readlane(k, 63);
  return __uint_as_float((uint32_t)(k ^ ((k >> 31) & 0x7fffffff)));  // the map is an involution
}

template <typename T>
__device__ __forceinline__ void wave_weight_partials(T w, bool valid, int n, double& wi, double& rmx, double& rmn,
                                                     T& mx, int& ix, T& mn, int& in_) {
  if constexpr (std::is_same<T, float>::value) {
    // fp32 weighing passes: the wave total (lane 63 of wave_scan, bit for bit) through the butterfly, the max as
    // integers; the inclusive prefix itself is formed only for a wave holding a negative weight (rare).
    const double x = valid ? (double)w : 0.0;
    const bool neg = __ballot(valid && w < 0.0f) != 0;  // wave-uniform
    const uint64_t vmask = __ballot(valid);
    mn = INFINITY;
    in_ = 0x7fffffff;
    if (!vmask) {  // no valid lane
      wi = 0.0;
      mx = -INFINITY;
      ix = 0x7fffffff;
      rmx = -INFINITY;
      rmn = INFINITY;
      return;
    }
    if (!neg) {
      wi = wave_total_lane63(x);
      mx = wave_max_f32(valid ? w : -INFINITY);
      rmx = lane_value(wi, 63);
      rmn = lane_value(x, 0);  // lane 0 is valid (valid lanes are a prefix of the wave)
    } else {
      wi = wave_incl_sum(x);
      float mxs = valid ? w : -INFINITY;
      mn = valid ? w : INFINITY;
      rmx = valid ? wi : -INFINITY;
      rmn = valid ? wi : INFINITY;
      scan_steps([&](auto st) {
        using S = decltype(st);
        mxs = fmax_t(mxs, dpp<S::ctrl, S::rm>(mxs, -INFINITY));
        mn = fmin_t(mn, dpp<S::ctrl, S::rm>(mn, INFINITY));
        st_max<S>(rmx);
        st_min<S>(rmn);
      });
      mx = lane_value(mxs, 63);
      mn = lane_value(mn, 63);
      const uint64_t bn = __ballot(valid && w == mn);
      in_ = bn ? __builtin_amdgcn_readlane(n, (int)__builtin_ctzll(bn)) : 0x7fffffff;
      rmx = lane_value(rmx, 63);
      rmn = lane_value(rmn, 63);
    }
    const uint64_t bx = __ballot(valid && w == mx);
    ix = bx ? __builtin_amdgcn_readlane(n, (int)__builtin_ctzll(bx)) : 0x7fffffff;
    return;
  }
  wi = valid ? (double)w : 0.0;
  mx = valid ? w : -inf_t<T>();
  const bool neg = __ballot(valid && w < (T)0) != 0;  // wave-uniform
  scan_steps([&](auto st) {
    using S = decltype(st);
    st_sum<S>(wi);
    mx = fmax_t(mx, dpp<S::ctrl, S::rm>(mx, -inf_t<T>()));
  });
  mx = lane_value(mx, 63);
  const uint64_t bx = __ballot(valid && w == mx);
  ix = bx ? __builtin_amdgcn_readlane(n, (int)__builtin_ctzll(bx)) : 0x7fffffff;
  mn = inf_t<T>();
  in_ = 0x7fffffff;
  if (!bx) {  // no valid lane
    rmx = -INFINITY;
    rmn = INFINITY;
  } else if (!neg) {
    rmx = lane_value(wi, 63);
    rmn = lane_value(wi, 0);
  } else {
    mn = valid ? w : inf_t<T>();
    rmx = valid ? wi : -INFINITY;
    rmn = valid ? wi : INFINITY;
    scan_steps([&](auto st) {
      using S = decltype(st);
      mn = fmin_t(mn, dpp<S::ctrl, S::rm>(mn, inf_t<T>()));
      st_max<S>(rmx);
      st_min<S>(rmn);
    });
    mn = lane_value(mn, 63);
    const uint64_t bn = __ballot(valid && w == mn);
    in_ = bn ? __builtin_amdgcn_readlane(n, (int)__builtin_ctzll(bn)) : 0x7fffffff;
    rmx = lane_value(rmx, 63);
    rmn = lane_value(rmn, 63);
  }
}

// LDS scratch of the per-iteration partials
struct WeighLds {
  double tot[kWaves], rmax[kWaves], rmin[kWaves], mx[kWaves], mn[kWaves];
  int ix[kWaves], in_[kWaves];
};

// ---- the iteration's partials: wave -> block (write-through + counter) -> group -> top.  Called by
// every thread (one barrier inside).  On return only wave 0 may have done hand-off work.
template <typename T, int RNG>
__device__ __forceinline__ void publish_iteration(const FrameArgsT<T>& fa, T w, bool valid, int n, int slot, int iter,
                                                  WeighLds& sh, BlockPart* __restrict__ part0,
                                                  BlockPart* __restrict__ part1, BlockScan* __restrict__ bscan0,
                                                  BlockScan* __restrict__ bscan1, GroupPart* __restrict__ gpart0,
                                                  GroupPart* __restrict__ gpart1, GroupScan* __restrict__ gscan,
                                                  Ctrl* __restrict__ ctrl, uint32_t* __restrict__ gcount,
                                                  uint32_t* __restrict__ tcount, uint32_t* __restrict__ gen,
                                                  uint32_t gen_base, uint64_t* __restrict__ stamps,
                                                  int blk) {
  // wave partials: scan total, extrema of the wave-inclusive prefix, max/argmax, min/argmin
  double wi, rmx, rmn;
  T mx, mn;
  int ix, in_;
  wave_weight_partials(w, valid, n, wi, rmx, rmn, mx, ix, mn, in_);
  const int lane = lane_id(), wv = wave_id();
  if (lane == 63) sh.tot[wv] = wi;
  if (lane == 0) {
    sh.rmax[wv] = rmx;
    sh.rmin[wv] = rmn;
    sh.mx[wv] = (double)mx;
    sh.mn[wv] = (double)mn;
    sh.ix[wv] = ix;
    sh.in_[wv] = in_;
  }
  __syncthreads();
  if (wv != 0) return;

  const int g = blk / fa.gsz;
  const int gsize = min(fa.gsz, fa.nblk - g * fa.gsz);
  int last = 0;
  if (lane == 0) {
    // block partial, same association as block_incl_sum: pre_w = ((0 + t0) + t1) + ...
    double pre = 0.0, maxrel = -INFINITY, minrel = INFINITY, bmx = sh.mx[0], bmn = sh.mn[0];
    int bix = sh.ix[0], bin = sh.in_[0];
#pragma unroll
    for (int ww = 0; ww < kWaves; ++ww) {
      const double a = pre + sh.rmax[ww], b = pre + sh.rmin[ww];
      maxrel = a > maxrel ? a : maxrel;
      minrel = b < minrel ? b : minrel;
      if (ww) {
        cmb_max(bmx, bix, sh.mx[ww], sh.ix[ww]);
        cmb_min(bmn, bin, sh.mn[ww], sh.in_[ww]);
      }
      pre = pre + sh.tot[ww];
    }
    BlockPart* bp = (slot ? part1 : part0) + blk;
    st_wt_d(&bp->sum, pre);
    st_wt_d(&bp->maxrel, maxrel);
    st_wt_d(&bp->minrel, minrel);
    st_wt_d(&bp->maxw, bmx);
    st_wt_d(&bp->minw, bmn);
    st_wt(&bp->argmax, pack2(bix, bin));
    if (stamps) stamp_max(stamps, 1, rt_now());
    last = arrive_last(gcount + g, gsize) ? 1 : 0;
  }
  if (!lane_value(last, 0)) return;
  const GroupPart gr =
      propagate_group(fa.nblk, fa.gsz, g, slot ? part1 : part0, slot ? bscan1 : bscan0, slot ? gpart1 : gpart0);
  const bool single = fa.ngrp == 1;
  if (!single && !wave_arrive_last(tcount, fa.ngrp)) return;
  if (stamps && lane == 0) stamps[2] = rt_now();
  propagate_top<T, RNG>(fa, ctrl, iter, gpart0, gpart1, gscan, gen, gen_base, gr, single, slot);
  if (stamps && lane == 0) stamps[3] = rt_now();
}

// ---- the streaming weighing pass (two-launch path, one stream): a grid of at most a few blocks per CU,
// each looping over the frame's 256-particle blocks vb = blockIdx.x, + gridDim.x, ...  The next block's
// prior loads are issued before this block's weights are stored and scanned, so the HBM latency of the
// state hides behind the arithmetic; the table and the frame constants are staged once per physical block;
// the block partials are plain stores read by k_group_top after the launch boundary (no arrival counters,
// no group / top tail in this launch).  Per 256-particle block the arithmetic and the partial are exactly
// k_propagate_weigh's, so the weights, partials and every later decision are bit-identical.
// Occupancy floor of k_weigh_stream (waves per SIMD; 1 = the compiler's choice): the fp16 and fp32 TUs set 6
// (85 -> 80 VGPRs: C4 weighing 241 -> 233 us, C5 30.6 -> 28.5 us); 7 was slower at C4 and C5.
#ifndef PFMPE_WEIGH_STREAM_MIN_WAVES
#define PFMPE_WEIGH_STREAM_MIN_WAVES 1
#endif
template <typename T, int RNG, int MAXM, bool PRUNE, typename SP>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(PFMPE_WEIGH_STREAM_MIN_WAVES))) void k_weigh_stream(const FrameArgsT<T> fa, const unsigned char* __restrict__ table,
                                                         const SP* __restrict__ prior, T* __restrict__ w0,
                                                         T* __restrict__ w1, BlockPart* __restrict__ part0,
                                                         BlockPart* __restrict__ part1, const Ctrl* __restrict__ ctrl,
                                                         SP* __restrict__ prop0, SP* __restrict__ prop1, int iter) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ LdsConst<T> sc;
  if (ctrl->done) return;  // the exit rule already fired (uniform)
  const int slot = ctrl->cur_slot;
  T* wout = slot ? w1 : w0;
  SP* pout = slot ? prop1 : prop0;
  BlockPart* parts = slot ? part1 : part0;
  const int lane = lane_id(), wv = wave_id();
  int vb = (int)blockIdx.x;
  copy_table(table, smem, (size_t)fa.tbytes);
  // raw state values of this block's particle (converted where they are used), so the loads of the next
  // block's particle can stay in flight across a whole block's arithmetic
  RawState<SP> R{};
  {
    const int n = vb * kBlock + (int)threadIdx.x;
    load_state_prefetch<SP>(prior, fa.ld, prior_row(fa, in_planes(n, fa.N)), n < fa.N && n >= 2, R);
  }
  stage_consts(fa, sc);
  __syncthreads();  // table + constants visible
  const LdsBlobs<T> tb = view_table<T>(smem, fa.B);
  const int step = (int)gridDim.x * kBlock;
  for (; vb < fa.nblk; vb += (int)gridDim.x) {
    const int n = vb * kBlock + (int)threadIdx.x;
    const bool valid = n < fa.N;
    T A[12];
#pragma unroll
    for (int q = 0; q < 12; ++q) A[q] = state_from_raw<T, SP>(R, q, fa.anc_in[q]);
    load_state_prefetch<SP>(prior, fa.ld, prior_row(fa, in_planes(n + step, fa.N)), n + step < fa.N && n + step >= 2,
                            R);  // next block
    T w = (T)0, P[12];
    if (valid) w = weigh_particle<T, RNG, MAXM, PRUNE>(fa, sc, tb, A, n, iter, P);
    if (valid) {
      wout[n] = w;
      if (prop0) store_pose<T, SP>(pout, fa.ld, n, P, fa.anc_out);
    }
    double wi, rmx, rmn;
    T mx, mn;
    int ix, in_;
    wave_weight_partials(w, valid, n, wi, rmx, rmn, mx, ix, mn, in_);
    // the wave's partial, as it is (k_group combines a block's kWaves wave partials with publish_iteration's
    // association): no LDS round trip, no block barrier and no serial combine in the loop
    const double tot = lane_value(wi, 63);
    if (lane == 0) {
      BlockPart q;
      q.sum = tot;
      q.maxrel = rmx;
      q.minrel = rmn;
      q.maxw = (double)mx;
      q.minw = (double)mn;
      q.argmax = ix;
      q.argmin = in_;
      parts[(size_t)vb * kWaves + wv] = q;
    }
  }
}

// ---- the iteration's group / top hand-off after a streaming weighing pass, as two small launches with no
// arrival counters (all groups finish at once here, and one counter taking ngrp arrivals back to back
// serialises them, ~25 ns each): k_group, block g (one wave) scans group g's block partials exactly as
// publish_iteration's last arriver does (propagate_group); k_top (one wave) runs propagate_top, with every
// group partial of the iteration staged in LDS in one round trip when there is more than one tile of groups.
// Same functions, same association as the other frame shapes.
template <typename T>
__global__ __launch_bounds__(64) void k_group(const FrameArgsT<T> fa, BlockPart* __restrict__ part0,
                                              BlockPart* __restrict__ part1, BlockScan* __restrict__ bscan0,
                                              BlockScan* __restrict__ bscan1, GroupPart* __restrict__ gpart0,
                                              GroupPart* __restrict__ gpart1, const Ctrl* __restrict__ ctrl) {
  if (ctrl->done) return;
  const int slot = ctrl->cur_slot;
  (void)propagate_group<true>(fa.nblk, fa.gsz, (int)blockIdx.x, slot ? part1 : part0, slot ? bscan1 : bscan0,
                              slot ? gpart1 : gpart0);
}
// k_group and k_top as ONE launch when the groups fit one tile (<= 64: C3, C5): every block scans its group, and
// the last to arrive on the top counter (write-through group partials, drained before the arrival, exactly the
// one-block pass's publish_iteration tail) runs propagate_top.  Saves the second launch and its gap; > 64 groups
// keep k_group + k_top_wide (a one-wave serial top over many tiles is slower than the wide one).
template <typename T, int RNG>
__global__ __launch_bounds__(64) void k_group_top(const FrameArgsT<T> fa, BlockPart* __restrict__ part0,
                                                  BlockPart* __restrict__ part1, BlockScan* __restrict__ bscan0,
                                                  BlockScan* __restrict__ bscan1, GroupPart* __restrict__ gpart0,
                                                  GroupPart* __restrict__ gpart1, GroupScan* __restrict__ gscan,
                                                  Ctrl* __restrict__ ctrl, uint32_t* __restrict__ tcount, int iter) {
  if (ctrl->done) return;  // every block reads ctrl before it arrives, so before the top can rewrite it
  const int slot = ctrl->cur_slot;
  const GroupPart gr = propagate_group<true>(fa.nblk, fa.gsz, (int)blockIdx.x, slot ? part1 : part0,
                                             slot ? bscan1 : bscan0, slot ? gpart1 : gpart0);
  const bool single = fa.ngrp == 1;
  if (!single && !wave_arrive_last(tcount, fa.ngrp)) return;
  propagate_top<T, RNG>(fa, ctrl, iter, gpart0, gpart1, gscan, nullptr, 0u, gr, single, slot);
}

template <typename T, int RNG>
__device__ __forceinline__ void top_body(const FrameArgsT<T>& fa, GroupPart* __restrict__ gpart0,
                                         GroupPart* __restrict__ gpart1, GroupScan* __restrict__ gscan,
                                         Ctrl* __restrict__ ctrl, int iter, int lds_groups, GroupPart* gsm) {
  if (ctrl->done) return;
  const int slot = ctrl->cur_slot;
  const GroupPart* src = slot ? gpart1 : gpart0;
  GroupPart none;
  none.sum = 0.0;
  none.zmax = -INFINITY;
  none.zmin = INFINITY;
  none.maxw = -INFINITY;
  none.minw = INFINITY;
  none.argmax = none.argmin = 0x7fffffff;
  const bool single = fa.ngrp == 1;
  const GroupPart g0 = single ? group_part(src, 0, none, false) : none;  // the one group's partial
  const GroupPart* staged = nullptr;
  if (fa.ngrp > 64 && lds_groups) {
    for (int base = 0; base < fa.ngrp; base += 64 * 8) {
      GroupPart q[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int gg = base + u * 64 + lane_id();
        if (gg < fa.ngrp) q[u] = group_part(src, gg, none, false);
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int gg = base + u * 64 + lane_id();
        if (gg < fa.ngrp) gsm[gg] = q[u];
      }
    }
    wave_lds_sync();
    staged = gsm;
  }
  propagate_top<T, RNG>(fa, ctrl, iter, gpart0, gpart1, gscan, nullptr, 0u, g0, single, slot, staged);
}
template <typename T, int RNG>
__global__ __launch_bounds__(64) void k_top(const FrameArgsT<T> fa, GroupPart* __restrict__ gpart0,
                                            GroupPart* __restrict__ gpart1, GroupScan* __restrict__ gscan,
                                            Ctrl* __restrict__ ctrl, int iter, int lds_groups) {
  extern __shared__ __attribute__((aligned(16))) GroupPart gsm[];  // lds_groups: ngrp entries
  top_body<T, RNG>(fa, gpart0, gpart1, gscan, ctrl, iter, lds_groups, gsm);
}

// ---- k_top for more than one tile of groups (ngrp > 64, partials staged in LDS): 16 waves instead of one.
// The per-tile work of propagate_top's final-iteration passes (the tile's inclusive sum, its G_g, the
// normalised group-start values and their in-tile max scan) runs one tile per wave in parallel; only the
// carried parts stay serial, in wave 0 and in the same order: S = ((0 + T_0) + T_1) + ... over the tile
// totals T_t (each the last lane of the tile's wave_incl_sum, as in propagate_top), the carry into tile t,
// and the running max over earlier tiles (a fold of `tm > run ? tm : run`, which ignores NaN and is the max
// of the rest: order-free).  So G_g, Gin_g, S, invS and the record are bit-identical to propagate_top's.
// Non-final iterations, and a final iteration whose kept partials are an earlier iteration's (not staged),
// run propagate_top itself in wave 0.
constexpr int kTopWaves = 16;
constexpr int kTopMaxTiles = 24;  // ngrp <= 1365 (staged) -> <= 22 tiles
struct TopWideLds {
  double tileT[kTopMaxTiles], tileM[kTopMaxTiles], carryT[kTopMaxTiles];
  double S_sh;
  int wide;
};
template <typename T, int RNG>
__device__ __forceinline__ void top_wide_body(const FrameArgsT<T>& fa, GroupPart* __restrict__ gpart0,
                                              GroupPart* __restrict__ gpart1, GroupScan* __restrict__ gscan,
                                              Ctrl* __restrict__ ctrl, int iter, GroupPart* gsm, TopWideLds& tw) {
  double* tileT = tw.tileT;
  double* tileM = tw.tileM;
  double* carryT = tw.carryT;
  double& S_sh = tw.S_sh;
  int& wide = tw.wide;
  if (ctrl->done) return;  // uniform
  const int slot = ctrl->cur_slot;
  const GroupPart* src = slot ? gpart1 : gpart0;
  const int lane = lane_id(), wv = (int)(threadIdx.x >> 6);
  const int ngrp = fa.ngrp, ntiles = (ngrp + 63) / 64;
  GroupPart none;
  none.sum = 0.0;
  none.zmax = -INFINITY;
  none.zmin = INFINITY;
  none.maxw = -INFINITY;
  none.minw = INFINITY;
  none.argmax = none.argmin = 0x7fffffff;
  // wave 0 requests the control record together with the group partials (the record was written by an earlier
  // launch; its load was a separate round trip after two barriers)
  Ctrl c;
  if (wv == 0) c = load_ctrl_wt(ctrl);
  for (int g = (int)threadIdx.x; g < ngrp; g += 64 * kTopWaves) gsm[g] = group_part(src, g, none, false);
  __syncthreads();
  // tile totals of this iteration's group sums (used if this iteration turns out to be the kept one); each wave
  // keeps its tiles' inclusive sums for the second pass
  constexpr int kTilesPerWave = (kTopMaxTiles + kTopWaves - 1) / kTopWaves;
  double inclT[kTilesPerWave];
#pragma unroll
  for (int i = 0; i < kTilesPerWave; ++i) {
    const int t = wv + i * kTopWaves;
    inclT[i] = 0.0;
    if (t < ntiles) {  // wave-uniform
      const int g = t * 64 + lane;
      inclT[i] = wave_incl_sum(g < ngrp ? gsm[g].sum : 0.0);
      if (lane == 63) tileT[t] = inclT[i];
    }
  }
  __syncthreads();
  if (wv == 0) {  // propagate_top's head: this iteration's max / first argmax, best, exit rule
    double mv = -INFINITY;
    int mi = 0x7fffffff;
    for (int g = lane; g < ngrp; g += 64) cmb_max(mv, mi, gsm[g].maxw, gsm[g].argmax);
    wave_argmax(mv, mi);
    if (mv > c.best_max) {  // strict: PE:608
      c.best_max = mv;
      c.best_idx = mi;
      c.best_iter = iter;
      c.best_slot = slot;
      c.has_best = 1;
    }
    c.iters = iter + 1;
    const bool go_on = fa.force_iters > 0 ? (c.iters < fa.force_iters)
                                          : (c.iters < fa.max_iter && mv < fa.exit_thr);  // PE:616
    const int kept_slot = c.has_best ? c.best_slot : slot;
    const int w = (!go_on && kept_slot == slot) ? 1 : 0;
    if (w) {
      c.cur_slot = c.has_best ? 1 - c.best_slot : 1 - slot;
      c.done = 1;
      c.kept_slot = kept_slot;
      c.kept_iter = c.has_best ? c.best_iter : iter;
      double carry = 0.0;
      for (int t = 0; t < ntiles; ++t) {
        if (lane == 0) carryT[t] = carry;
        carry = carry + tileT[t];
      }
      if (lane == 0) S_sh = carry;
    } else {
      propagate_top<T, RNG>(fa, ctrl, iter, gpart0, gpart1, gscan, nullptr, 0u, none, false, slot, gsm);
    }
    if (lane == 0) wide = w;
  }
  __syncthreads();
  if (!wide) return;
  const double S = S_sh;
  // per tile: G_g and the normalised group-start values' in-tile max scan (propagate_top's second pass)
  double exl[kTilesPerWave];
#pragma unroll
  for (int i = 0; i < kTilesPerWave; ++i) {
    const int t = wv + i * kTopWaves;
    exl[i] = -INFINITY;
    if (t < ntiles) {  // wave-uniform
      const int g = t * 64 + lane;
      GroupPart q;
      q.sum = 0.0;
      q.zmax = -INFINITY;
      q.zmin = INFINITY;
      if (g < ngrp) q = gsm[g];
      const double incl = inclT[i];  // the first pass's wave_incl_sum of the same values
      const double prev = wave_shr1(incl, 0.0);
      const double G = lane == 0 ? carryT[t] : carryT[t] + prev;
      double cm = -INFINITY;
      if (g < ngrp && S != 0.0) cm = (G + (S > 0.0 ? q.zmax : q.zmin)) / S;
      const double im = wave_incl_max(cm);
      exl[i] = wave_shr1(im, -(double)INFINITY);
      if (g < ngrp) st_wt_d(&gscan[g].G, G);
      if (lane == 63) tileM[t] = im;
    }
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < kTilesPerWave; ++i) {
    const int t = wv + i * kTopWaves;
    if (t < ntiles) {
      double run = -INFINITY;
      for (int u = 0; u < t; ++u) run = tileM[u] > run ? tileM[u] : run;
      const double ex = exl[i] > run ? exl[i] : run;
      const int g = t * 64 + lane;
      if (g < ngrp) st_wt_d(&gscan[g].Gin, ex);
    }
  }
  if (wv != 0) return;
  // propagate_top's tail: invS, the kept iteration's argmax / argmin, accept, the record
  double run = -INFINITY;
  for (int u = 0; u < ntiles; ++u) run = tileM[u] > run ? tileM[u] : run;
  if (S == 0.0) run = -INFINITY;
  double amv = -INFINITY, anv = INFINITY;
  int ami = 0x7fffffff, ani = 0x7fffffff;
  for (int g = lane; g < ngrp; g += 64) {
    cmb_max(amv, ami, gsm[g].maxw, gsm[g].argmax);
    cmb_min(anv, ani, gsm[g].minw, gsm[g].argmin);
  }
  wave_argmax(amv, ami);
  wave_argmin(anv, ani);
  const double highest = c.has_best ? c.best_max : 0.0;
  c.S = S;
  c.invS = 1.0 / S;
  c.accepted = (S != 0.0 && highest > fa.accept_thr) ? 1 : 0;  // PE:633
  if (c.accepted) {
    c.most_likely_idx = c.best_idx;
    c.K_total = lane == 0 ? count_targets<T, RNG>(fa, c.iters, run) : 0;
  } else {
    c.most_likely_idx = (S < 0.0) ? ani : ami;  // PE:714
    c.K_total = 0;
  }
  if (lane == 0) store_ctrl_wt(ctrl, c);
}
template <typename T, int RNG>
__global__ __launch_bounds__(64 * kTopWaves) void k_top_wide(const FrameArgsT<T> fa, GroupPart* __restrict__ gpart0,
                                                          GroupPart* __restrict__ gpart1,
                                                          GroupScan* __restrict__ gscan, Ctrl* __restrict__ ctrl,
                                                          int iter) {
  extern __shared__ __attribute__((aligned(16))) GroupPart gsm[];  // ngrp entries
  __shared__ TopWideLds tw;
  top_wide_body<T, RNG>(fa, gpart0, gpart1, gscan, ctrl, iter, gsm, tw);
}

// ---- launch 1 of the two-launch path: motion + projection + likelihood, one particle per thread.
// One block's work (block `blk` of its stream), shared by the one-stream kernel and the batched kernel
// (k_propagate_weigh_multi, many contexts in one launch).  fa_words: the frame constants' source, the
// kernarg segment (one-stream) or the stream's descriptor in HBM (batched).
template <typename T, int RNG, int MAXM, bool PRUNE, typename SP, bool MULTI>
__device__ __forceinline__ void propagate_weigh_block(
    const FrameArgsT<T>& fa, const uint32_t* fa_words, int blk, const unsigned char* __restrict__ table,
    const SP* __restrict__ prior, T* __restrict__ w0, T* __restrict__ w1, BlockPart* __restrict__ part0,
    BlockPart* __restrict__ part1, BlockScan* __restrict__ bscan0, BlockScan* __restrict__ bscan1,
    GroupPart* __restrict__ gpart0, GroupPart* __restrict__ gpart1, GroupScan* __restrict__ gscan,
    Ctrl* __restrict__ ctrl, uint32_t* __restrict__ gcount, uint32_t* __restrict__ tcount, SP* __restrict__ prop0,
    SP* __restrict__ prop1, int iter, uint64_t* __restrict__ stamps, unsigned char* smem, LdsConst<T>& sc,
    WeighLds& sh) {
  if (stamps && threadIdx.x == 0) stamp_min(stamps, 0, rt_now());
  const int n = blk * kBlock + threadIdx.x;
  const bool valid = n < fa.N;
  // table loads first: vmcnt retires in order, so the LDS copy then waits only for them while the
  // prior loads stay in flight across the barrier
  copy_table(table, smem, (size_t)fa.tbytes);
  T A[12];
  if (valid && n >= 2) load_prior(fa, prior, n, A);
  // written by the previous launch: the exit rule already fired (uniform), and this iteration's weight slot
  // (a kernel argument pointer: the compiler's own scalar loads; batched: explicit scalar loads)
  if (MULTI ? load_ctrl_word<(int)offsetof(Ctrl, done)>(ctrl) : ctrl->done) return;
  const int slot = MULTI ? load_ctrl_word<(int)offsetof(Ctrl, cur_slot)>(ctrl) : ctrl->cur_slot;
  stage_consts_from(fa_words, sc);
  __syncthreads();  // table + constants visible
  const LdsBlobs<T> tb = view_table<T>(smem, fa.B);
  if (stamps && threadIdx.x == 0) {
    const uint64_t t = rt_now();
    stamp_max(stamps, 8, t);
    stamp_min(stamps, 19, t);
  }
  T w = (T)0;
  if (valid) {
    T P[12];
    int nv = 0;
    w = weigh_particle<T, RNG, MAXM, PRUNE>(fa, sc, tb, A, n, iter, P, &nv);
    (slot ? w1 : w0)[n] = w;
    if (prop0)  // keep the propagated set next to its weights (same slot): k_resample gathers it
      store_pose<T, SP>(slot ? prop1 : prop0, fa.ld, n, P, fa.anc_out);
    if (stamps && (fa.diag & 8))  // diagnostic: pruned candidates visited (sum, max)
      atomicAdd((unsigned long long*)(stamps + 30), (unsigned long long)nv), atomicMax((unsigned long long*)(stamps + 31), (unsigned long long)nv);
  }
  if (stamps && threadIdx.x == 0) stamp_max(stamps, 9, rt_now());
  publish_iteration<T, RNG>(fa, w, valid, n, slot, iter, sh, part0, part1, bscan0, bscan1, gpart0, gpart1, gscan,
                            ctrl, gcount, tcount, nullptr, 0u, stamps, blk);
}

// Occupancy floor of k_propagate_weigh (waves per SIMD; 1 = the compiler's choice).  The fp32 / fp16 TUs set 6:
// the 5- and 8-marker instances fit 8 waves anyway (63-66 VGPRs); the 12-marker one drops 93 -> 80 VGPRs
// (5 -> 6 waves, a few values spilled): C3 weighing 96 -> 91 us.
#ifndef PFMPE_WEIGH_MIN_WAVES
#define PFMPE_WEIGH_MIN_WAVES 1
#endif
template <typename T, int RNG, int MAXM, bool PRUNE, typename SP>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(PFMPE_WEIGH_MIN_WAVES))) void k_propagate_weigh(
    const FrameArgsT<T> fa, const unsigned char* __restrict__ table, const SP* __restrict__ prior, T* __restrict__ w0,
    T* __restrict__ w1, BlockPart* __restrict__ part0, BlockPart* __restrict__ part1,
    BlockScan* __restrict__ bscan0, BlockScan* __restrict__ bscan1, GroupPart* __restrict__ gpart0,
    GroupPart* __restrict__ gpart1, GroupScan* __restrict__ gscan, Ctrl* __restrict__ ctrl,
    uint32_t* __restrict__ gcount, uint32_t* __restrict__ tcount, SP* __restrict__ prop0, SP* __restrict__ prop1,
    int iter, uint64_t* __restrict__ stamps) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ LdsConst<T> sc;
  __shared__ WeighLds sh;
  propagate_weigh_block<T, RNG, MAXM, PRUNE, SP, false>(fa, (const uint32_t*)__builtin_amdgcn_kernarg_segment_ptr(),
                                                 (int)blockIdx.x, table, prior, w0, w1, part0, part1, bscan0, bscan1,
                                                 gpart0, gpart1, gscan, ctrl, gcount, tcount, prop0, prop1, iter,
                                                 stamps, smem, sc, sh);
}

// ---- batched frames (pfmpe_step_multi): S independent contexts' frames in one launch.  Each context is one
// camera stream / tracked object (the reference's per-object loop, PE:89, state per object PE:113-114,
// 726-727); its blocks are contiguous in the grid.  A stream's descriptor holds its frame constants (the
// one-stream kernels' kernel arguments) and its device buffers; bmap[block] names the block's stream.
// Every stream keeps its own hand-off counters, control record and frame record, so the streams of a batch
// never wait on each other and each one computes exactly what its one-stream frame computes.
struct Cand;
template <typename T, typename SP>
struct alignas(16) StreamDesc {  // 16-B multiple: k_stage_multi copies 16-B words
  FrameArgsT<T> fa;  // first: stage_consts_from reads its head (LdsConst layout)
  const unsigned char* table;
  const SP* prior;
  SP* post;
  T* w0;
  T* w1;
  BlockPart* part0;
  BlockPart* part1;
  BlockScan* bscan0;
  BlockScan* bscan1;
  GroupPart* gpart0;
  GroupPart* gpart1;
  GroupScan* gscan;
  Ctrl* ctrl;
  uint32_t* gcount_w;
  uint32_t* tcount_w;
  uint32_t* gcount_r;
  uint32_t* tcount_r;
  SP* prop0;  // kept propagated sets (null: k_resample regenerates)
  SP* prop1;
  CountPart* cpart;
  CountPart* cgroup;
  uint32_t* counts;
  Cand* cand;
  double* mlpose;
  RecOut* out;
  unsigned long long* winkey;  // the stream's winner keys and arrival shards (k_resample_owners_multi's finish)
  int32_t seq;
  int32_t first_blk;  // the stream's first block in the grid
  int32_t wg;         // resident workgroups of the stream in a streaming batched weighing pass (k_weigh_pk_multi)
  int32_t pad_wg;
  uint64_t gen;       // the batch generation (staging launch counter; every kernel of the round gets it)
  uint64_t tag;       // desc_tag over every word before this one (pf_desc_tag.hpp)
};

// Batch staging (block s = stream s): the stream's descriptor and, for host-supplied blobs, its table, from
// the pinned host staging buffer (read over PCIe once) into HBM, and the block -> stream map of its blocks.
// A launch in the batch's own stream instead of a host-to-device copy: no copy-engine hand-off in front of
// the weighing launch.  dev / host: the device scratch and its pinned host image (same layout); a table
// pointer inside [dev, dev + tbytes) is a staged host table.
// The descriptor is checked before any of its words is used (pf_desc_tag.hpp): the tag recomputed over the words
// this block read must equal the tag word, and the generation word must equal `gen`.  status[s] = gen then; a
// failed check leaves status[s] != gen, writes no map entry and stages no table, and every later kernel of the
// round skips the stream (batch_block / k_resample_final_multi test status[s] == gen), so no pointer of a bad
// descriptor is ever followed.  The host finds the missing frame record and reports the descriptor the device
// saw (its HBM copy, written here word for word) against the one it wrote.
constexpr uint32_t kMapKept = 0xffffffffu;  // k_stage_multi's boff: the block map is unchanged
template <typename T, typename SP>
__global__ __launch_bounds__(kBlock) void k_stage_multi(const unsigned char* __restrict__ host,
                                                        unsigned char* __restrict__ dev, uint32_t doff, uint32_t tbytes,
                                                        uint32_t boff, uint32_t* __restrict__ status, uint32_t gen) {
  // The host rewrote the image with plain CPU stores that the runtime does not see, and the dispatch's own
  // acquire is agent scope, which leaves cached copies of host memory valid: a line an earlier batch or round
  // read from the image (same addresses, other contents: a later round stages a smaller layout) could be
  // served stale.  So every read of the image is a system-scope atomic load (a vector load with sc0 sc1,
  // coherent with the host; never a scalar load), which needs no cache invalidate in front of it.
  auto host_ld = [](const auto* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM); };
  using Desc = StreamDesc<T, SP>;
  const int s = blockIdx.x;
  const Desc* hd = (const Desc*)(host + doff) + s;
  static_assert(sizeof(Desc) % 16 == 0, "descriptor as 16-B words");
  constexpr int kWords = (int)(sizeof(Desc) / 8), kTagWords = (int)(offsetof(Desc, tag) / 8);
  static_assert(offsetof(Desc, tag) % 8 == 0 && offsetof(Desc, gen) + 8 == offsetof(Desc, tag), "tag layout");
  __shared__ unsigned long long h;
  __shared__ Desc ld;  // the words as this block read them (each word is read by one thread: no global re-read)
  if (threadIdx.x == 0) h = 0ull;
  __syncthreads();
  {
    const uint64_t* src = (const uint64_t*)hd;
    uint64_t* dst = (uint64_t*)((Desc*)(dev + doff) + s);
    uint64_t mine = 0;
    for (int i = threadIdx.x; i < kWords; i += kBlock) {
      const uint64_t v = host_ld(src + i);
      dst[i] = v;
      ((uint64_t*)&ld)[i] = v;
      if (i < kTagWords) mine ^= tag_mix(v, (uint32_t)i);
    }
    if (mine) atomicXor(&h, (unsigned long long)mine);
  }
  __syncthreads();  // the block's words and the tag terms in LDS
  const bool ok = __builtin_amdgcn_readfirstlane((int)(h == (unsigned long long)ld.tag && ld.gen == (uint64_t)gen));
  if (!ok) {
    if (threadIdx.x == 0) status[s] = ~gen;
    return;
  }
  const int first = __builtin_amdgcn_readfirstlane(ld.first_blk);
  const int nblk = __builtin_amdgcn_readfirstlane(ld.fa.nblk);
  const unsigned char* tab = ld.table;
  // the map entries [first, first + nblk): 16-B stores of eight entries where a whole aligned group of eight is the
  // stream's (a C4 stream's 39k entries were 153 two-byte stores per thread: 10 us of staging), single entries at
  // the two ends.  boff is 16-B aligned (batch_layout); kMapKept: the map in HBM is already this batch's (the host
  // keeps the layout of the last batch it staged: the same streams, sizes and offsets), nothing to write
  uint16_t* bm = (uint16_t*)(dev + (boff == kMapKept ? 0u : boff));
  if (boff != kMapKept) {
  const int g0 = (first + 7) >> 3, g1 = (first + nblk) >> 3;  // whole groups of eight: [g0, g1)
  if (g1 > g0) {
    const uint32_t v = (uint32_t)s | ((uint32_t)s << 16);
    uint4* bm16 = (uint4*)bm;
    for (int g = g0 + (int)threadIdx.x; g < g1; g += kBlock) bm16[g] = make_uint4(v, v, v, v);
    for (int b = first + (int)threadIdx.x; b < 8 * g0; b += kBlock) bm[b] = (uint16_t)s;
    for (int b = 8 * g1 + (int)threadIdx.x; b < first + nblk; b += kBlock) bm[b] = (uint16_t)s;
  } else {
    for (int b = threadIdx.x; b < nblk; b += kBlock) bm[first + b] = (uint16_t)s;
  }
  }
  const uintptr_t to = (uintptr_t)tab - (uintptr_t)dev;  // wraps above tbytes for bank tables
  if (to < tbytes) {
    const uint64_t* src = (const uint64_t*)(host + to);
    uint64_t* dst = (uint64_t*)(dev + to);
    const int n8 = __builtin_amdgcn_readfirstlane(ld.fa.tbytes) / 8;
    for (int i = threadIdx.x; i < n8; i += kBlock) dst[i] = host_ld(src + i);
  }
  if (threadIdx.x == 0) status[s] = gen;
}

// The block's stream and its stream-local block index, or -1 for a block the map does not place inside a
// stream of this batch whose descriptor passed the staging check (never on a consistent batch: the host audits
// the layout before every launch, pfmpe_ctx.hpp audit_batch, and tags every descriptor; the guard keeps a
// corrupt map or descriptor from turning into out-of-range accesses).  A stale map entry cannot misplace a
// block: the range test runs against a checked descriptor, and checked streams' ranges are disjoint.
template <typename T, typename SP>
__device__ __forceinline__ int batch_block(const StreamDesc<T, SP>* __restrict__ descs,
                                           const uint16_t* __restrict__ bmap, int S, const uint32_t* __restrict__ status,
                                           uint32_t gen, int* s_out) {
  const int s = __builtin_amdgcn_readfirstlane((int)bmap[blockIdx.x]);
  if (s >= S) return -1;
  if (__builtin_amdgcn_readfirstlane(status[s]) != gen) return -1;
  const int blk = (int)blockIdx.x - __builtin_amdgcn_readfirstlane(descs[s].first_blk);
  if (blk < 0 || blk >= __builtin_amdgcn_readfirstlane(descs[s].fa.nblk)) return -1;
  *s_out = s;
  return blk;
}

template <typename T, int RNG, int MAXM, bool PRUNE, typename SP>
__global__ __launch_bounds__(kBlock) void k_propagate_weigh_multi(const StreamDesc<T, SP>* __restrict__ descs,
                                                                  const uint16_t* __restrict__ bmap, int S,
                                                                  const uint32_t* __restrict__ status, uint32_t gen,
                                                                  int iter) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ LdsConst<T> sc;
  __shared__ WeighLds sh;
  int s = 0;
  const int blk = batch_block(descs, bmap, S, status, gen, &s);
  if (blk < 0) return;
  const StreamDesc<T, SP>& d = descs[s];
  propagate_weigh_block<T, RNG, MAXM, PRUNE, SP, true>(d.fa, (const uint32_t*)&d.fa, blk, d.table,
                                                 d.prior, d.w0, d.w1, d.part0, d.part1, d.bscan0, d.bscan1, d.gpart0,
                                                 d.gpart1, d.gscan, d.ctrl, d.gcount_w, d.tcount_w, d.prop0, d.prop1,
                                                 iter, nullptr, smem, sc, sh);
}

// Winner candidate of one block: the block's first max-count particle, its kept pose and its
// correspondences, published by the block's wave 1 (in parallel with wave 0's arrival) as data-tagged
// granules: 8-byte words {payload (low 32 bits), frame sequence (high 32)}, each written by ONE
// write-through store, so a reader that sees every tag current has every payload (MI355X_MICROARCH.md
// "handoff-1to1").  Granules 0-23: the 12 pose doubles as lo/hi halves; 24-55: the 32 corr words;
// 56: n_corr.  The global winner is one of these, so the final wave loads one block's granules.
constexpr int kCandGran = 57;
struct alignas(16) Cand {
  uint64_t g[64];
};

// correspondences (PE:2385-2445 with pairs) of ONE pose P (uniform across the wave): blobs spread over
// the lanes, (distance, original index) order as column_minima, then the sorting-network score.
// Pairs go to corr (LDS), written by lane 0.
// The pairs score_minima<PAIRS> lists (PE:2385-2445) from the per-marker minima m / blob indices r (uniform
// across the wave); u0, v0: marker 0's projection (the NaN-at-origin rule).  One whole wave; corr: the
// 2*kMaxMarkers LDS words of the (LED, blob) pairs, cleared first.  Returns the pair count.
template <typename T, int MAXM>
__device__ __forceinline__ int pairs_from_minima(const FrameArgsT<T>& fa, const LdsBlobs<T>& tb, const T* m,
                                                 const int* r, T u0, T v0, uint32_t* corr) {
  const int lane = lane_id();
  const int B = fa.B;
  if (lane < 2 * kMaxMarkers) corr[lane] = 0u;
  wave_lds_sync();  // the pairs are written over the cleared words
  // The pairs score_minima<PAIRS> lists (PE:2385-2445), lane-parallel: the keys (m_j, j) in ascending
  // order, cut at the first key whose distance fails the tol_PF gate and at min(B, M).  Lane j < MAXM
  // holds key j (+inf past M, as in score_minima) and computes its rank; keys are distinct, so the ranks
  // are exactly the sorted positions.
  int np = 0;
  if (B > 0 && !nan_at_origin_tb(fa, tb, u0, v0)) {
    const int M = fa.M;
    const int L = B < M ? B : M;
    T mj = inf_t<T>();
    int rj = 0;
#pragma unroll
    for (int j = 0; j < MAXM; ++j) {
      mj = (lane == j && marker_live<MAXM>(j, M)) ? opaque(m[j]) : mj;
      rj = lane == j ? opaque(r[j]) : rj;
    }
    int rank = 0;
#pragma unroll
    for (int i = 0; i < MAXM; ++i) {
      const T mi = i < M ? m[i] : inf_t<T>();
      rank += (mi < mj || (mi == mj && i < lane)) ? 1 : 0;
    }
    const bool key = lane < MAXM;
    const bool fail = !(sqrt_t(mj) <= fa.tol_pf);
    const int fr = (key && fail) ? rank : MAXM;
    const int F = -lane_value(wave_scan(-fr, -MAXM, OpMaxI()), 63);  // first failing rank
    np = F < L ? F : L;
    if (key && rank < np) {
      corr[2 * rank] = (uint32_t)lane + 1u;
      corr[2 * rank + 1] = (uint32_t)rj + 1u;
    }
  }
  wave_lds_sync();
  return np;
}
// pose_pairs' per-marker wave arg-minimum in fp32: wave_argmin's lexicographic (distance, original index) minimum,
// as two integer minimum reductions per marker.  Every lane's best is a number (it starts at +inf and a NaN distance
// never replaces it) and >= +0 (a sum of squares), so its bits order as integers and equal distances have equal bits:
// the minimum's bits first, then the lowest index among the lanes holding them.  One DPP-fed v_min_i32 per step (the
// quad / half-row / row / bcast pattern of wave_total_lane63: lane 63 ends with the whole wave; the bcast steps leave
// rows no one reads), all MAXM markers interleaved, instead of the (value, index) select chains.
template <int MAXM>
__device__ __forceinline__ void wave_argmin_dist(float (&best)[MAXM], int (&arg)[MAXM]) {
  auto wave_min_lane63 = [](int (&k)[MAXM]) {
#pragma unroll
    for (int j = 0; j < MAXM; ++j) k[j] = min(k[j], __builtin_amdgcn_mov_dpp(k[j], kDppQuadXor1, 0xf, 0xf, false));
#pragma unroll
    for (int j = 0; j < MAXM; ++j) k[j] = min(k[j], __builtin_amdgcn_mov_dpp(k[j], kDppQuadXor2, 0xf, 0xf, false));
#pragma unroll
    for (int j = 0; j < MAXM; ++j) k[j] = min(k[j], __builtin_amdgcn_mov_dpp(k[j], kDppRowHalfMirror, 0xf, 0xf, false));
#pragma unroll
    for (int j = 0; j < MAXM; ++j) k[j] = min(k[j], __builtin_amdgcn_mov_dpp(k[j], kDppRowMirror, 0xf, 0xf, false));
#pragma unroll
    for (int j = 0; j < MAXM; ++j) k[j] = min(k[j], __builtin_amdgcn_mov_dpp(k[j], kDppBcast15, 0xa, 0xf, false));
#pragma unroll
    for (int j = 0; j < MAXM; ++j) k[j] = min(k[j], __builtin_amdgcn_mov_dpp(k[j], kDppBcast31, 0xc, 0xf, false));
  };
  int k[MAXM], c[MAXM];
#pragma unroll
  for (int j = 0; j < MAXM; ++j) k[j] = (int)__float_as_uint(best[j]);
  wave_min_lane63(k);
#pragma unroll
  for (int j = 0; j < MAXM; ++j) {
    k[j] = __builtin_amdgcn_readlane(k[j], 63);
    c[j] = (int)__float_as_uint(best[j]) == k[j] ? arg[j] : 0x7fffffff;
  }
  wave_min_lane63(c);
#pragma unroll
  for (int j = 0; j < MAXM; ++j) {
    best[j] = __uint_as_float((uint32_t)k[j]);
    arg[j] = __builtin_amdgcn_readlane(c[j], 63);
  }
}

template <typename T, int MAXM>
__device__ __forceinline__ void pose_pairs(const FrameArgsT<T>& fa, const LdsConst<T>& sc, const LdsBlobs<T>& tb,
                                           const T* P, uint32_t* corr, int* np_out) {
  const int lane = lane_id();
  const int B = fa.B;
  T u[MAXM], v[MAXM], m[MAXM];
  int r[MAXM];
  project_markers<T, MAXM>(fa, sc, P, u, v);
  T best[MAXM];
  int arg[MAXM];
#pragma unroll
  for (int j = 0; j < MAXM; ++j) {
    best[j] = inf_t<T>();
    arg[j] = 0x7fffffff;
  }
  for (int i = lane; i < B; i += 64) {
    const BlobXY<T> p = tb.bxy[i];
    const T bx = p.x, by = p.y;
    const int o = tb.orig[i];
#pragma unroll
    for (int j = 0; j < MAXM; ++j) {
      const T dx = bx - u[j];
      const T dy = by - v[j];
      const T d = fmadd(dx, dx, dy * dy);
      if (d < best[j] || (d == best[j] && o < arg[j])) {
        best[j] = d;
        arg[j] = o;
      }
    }
  }
  // all MAXM reductions unconditionally (markers past M reduce +inf: harmless), so the DPP chains interleave
  if constexpr (std::is_same<T, float>::value) {
    wave_argmin_dist<MAXM>(best, arg);
  } else {
#pragma unroll
    for (int j = 0; j < MAXM; ++j) wave_argmin(best[j], arg[j]);
  }
#pragma unroll
  for (int j = 0; j < MAXM; ++j) {
    m[j] = best[j];
    r[j] = arg[j] == 0x7fffffff ? 0 : arg[j];
  }
  *np_out = pairs_from_minima<T, MAXM>(fa, tb, m, r, u[0], v[0], corr);
}

// ---- frame record (one wave) into pinned host memory: the scalars from the control record, the
// winner's pose and pairs from its block's candidate record, the most likely pose from `mlpose`; then
// the tag release and the reset of the control record for the next frame.  On the re-init branch
// (winner < 0) the most likely particle is regenerated here and there are no pairs.
template <typename T, int RNG, int MAXM, typename SP>
__device__ __forceinline__ void finalize_frame(const FrameArgsT<T>& fa, const LdsConst<T>& sc, const Ctrl& c,
                                               Ctrl* __restrict__ ctrl, const SP* __restrict__ prior, int winner,
                                               const Cand* __restrict__ cand, const double* __restrict__ mlpose,
                                               OutDev& rec, RecOut* __restrict__ out, int32_t tag,
                                               uint64_t* __restrict__ stamps, bool have_pl = false,
                                               uint32_t pl_reg = 0u, double ml_reg = 0.0) {
  const int lane = lane_id();
  if (c.accepted) {
    // the winner's candidate granules (one round trip; re-polled, bounded, while a tag is stale; or
    // handed over in registers, have_pl) and the most likely pose
    const Cand* wc = cand + winner / kBlock;
    double ml = ml_reg;
    if (lane < 12 && !have_pl) ml = ld_wt_d(mlpose + lane);
    uint64_t gv = pl_reg;
    const uint64_t t0 = rt_now();
    for (; !have_pl;) {
      if (lane < kCandGran) gv = ld_wt(&wc->g[lane]);
      const bool stale = lane < kCandGran && (uint32_t)(gv >> 32) != (uint32_t)(tag >> 1);
      if (!__builtin_amdgcn_ballot_w64(stale)) break;
      if (rt_now() - t0 > fa.wait_ticks) return;  // abandon (no record; the host reports it)
      __builtin_amdgcn_s_sleep(1);
    }
    const uint32_t pl = (uint32_t)gv;
    uint32_t* wp = (uint32_t*)rec.winner_pose;
    if (lane < 24) wp[lane] = pl;  // little-endian halves of the 12 doubles
    if (lane >= 24 && lane < 24 + 2 * kMaxMarkers) rec.corr[lane - 24] = pl;
    if (lane == 56) rec.n_corr = (int32_t)pl;
    if (lane < 12) rec.most_likely_pose[lane] = ml;
  } else {
    T Q[12];
    make_particle<T, RNG, SP>(fa, sc, prior, c.most_likely_idx, c.kept_iter, Q);
    if (lane < 12) {  // lane q writes pose word q (selects, no dynamic register indexing)
      T pm = Q[0];
#pragma unroll
      for (int q = 1; q < 12; ++q) pm = lane == q ? opaque(Q[q]) : pm;
      rec.most_likely_pose[lane] = (double)pm;
      rec.winner_pose[lane] = (double)pm;
    }
    if (lane < 2 * kMaxMarkers) rec.corr[lane] = 0u;
    if (lane == 0) rec.n_corr = 0;
  }
  if (stamps && lane == 0) stamps[13] = stamps[14] = stamps[15] = stamps[16] = rt_now();
  if (lane == 0) {
    rec.kept_slot = c.kept_slot;
    rec.iters = c.iters;
    rec.kept_iter = c.kept_iter;
    rec.most_likely_idx = c.most_likely_idx;
    rec.accepted = c.accepted;
    rec.resampled = c.accepted;
    rec.winner_idx = c.accepted ? winner : -1;
    rec.flag_fail = c.accepted ? 1 : 4;
    rec.highest_prob = c.has_best ? c.best_max : 0.0;
    rec.prob_sum = c.S;
    if (stamps) stamps[17] = rt_now();
  }
  wave_lds_sync();
  const uint32_t* rw = (const uint32_t*)&rec;
  const uint64_t th = (uint64_t)(uint32_t)tag << 32;
  st_sys64(&out->g[lane], th | rw[lane]);
  if (lane + 64 < kRecWords) st_sys64(&out->g[lane + 64], th | rw[lane + 64]);
  if (lane != 0) return;
  if (stamps) stamps[18] = rt_now();
  // the next frame starts from the all-zero control record
  store_ctrl_wt(ctrl, zero_ctrl());
}

// A candidate's record payload, one 32-bit word per lane: lanes 0-23 the 12 pose doubles (low, high
// halves), 24.. the (LED, blob) pairs, 56 the pair count.  One wave; ccorr: 2*kMaxMarkers LDS words.
template <typename T>
__device__ __forceinline__ uint32_t payload_word(const T* Pc, const uint32_t* ccorr, int np) {
  const int lane = lane_id();
  uint32_t pl = 0;
  if (lane < 24) {
    T pv = Pc[0];
#pragma unroll
    for (int q = 1; q < 12; ++q) pv = (lane >> 1) == q ? opaque(Pc[q]) : pv;
    const uint64_t bits = (uint64_t)__double_as_longlong((double)pv);
    pl = (lane & 1) ? (uint32_t)(bits >> 32) : (uint32_t)bits;
  } else if (lane < 24 + 2 * kMaxMarkers) {
    pl = ccorr[lane - 24];
  } else if (lane == 56) {
    pl = (uint32_t)np;
  }
  return pl;
}
template <typename T, int MAXM>
__device__ __forceinline__ uint32_t cand_payload(const FrameArgsT<T>& fa, const LdsConst<T>& sc, const LdsBlobs<T>& tb,
                                                 const T* Pc, uint32_t* ccorr) {
  int np = 0;
  pose_pairs<T, MAXM>(fa, sc, tb, Pc, ccorr, &np);
  return payload_word<T>(Pc, ccorr, np);
}

// LDS scratch of the resampling phase: scan partials, and per wave the staging of the scatter (the
// wave's 64 kept particles as rows, and the slot -> owner-lane map of the current 64-slot chunk)
template <typename T>
struct ResampleLds {
  double sum[kWaves], max[kWaves];
  int hi[kWaves], c[kWaves], ci[kWaves];
  uint32_t ccorr[2 * kMaxMarkers];  // wave 1's pair scratch for the block candidate
  struct alignas(16) Row {
    T q[12];
  } rows[kWaves][64];
  int map[kWaves][64];
};

// ---- stratified resampling of one block (PE:666-682) + count partials -> winner -> frame record.
// wd: the thread's kept raw weight (0 for invalid lanes); P: its kept propagated particle when have_P,
// else regenerated here from A (P_in unused).  Called by every thread; the caller checked c.done && c.accepted.
// MODE 1 (k_frame): the block also publishes its winner candidate and the last arriver of the count tree
// finishes the frame.  MODE 2 (k_frame2): the same candidate, then a flat arrival on the sharded count
// counters; block 0 waits for all of them and finishes.  MODE 0 (k_resample) the block only stores its
// count partial; k_resample_final finishes.
template <typename T, int RNG, int MAXM, typename SP, int MODE, bool RAW = false>
__device__ __forceinline__ void resample_phase(
    const FrameArgsT<T>& fa, const LdsConst<T>& sc, const Ctrl& c, Ctrl* __restrict__ ctrl,
    const unsigned char* __restrict__ table, const SP* __restrict__ prior, SP* __restrict__ post, double wd, const T* A,
    const T* P_in, bool have_P, const BlockScan& bs, const GroupScan& gs, ResampleLds<T>& sh, OutDev& rec,
    const LdsBlobs<T>& tb, Cand* __restrict__ cand, double* __restrict__ mlpose,
    CountPart* __restrict__ cpart, CountPart* __restrict__ cgroup, uint32_t* __restrict__ gcount,
    uint32_t* __restrict__ tcount, uint32_t* __restrict__ counts, RecOut* __restrict__ out, int32_t seq,
    uint64_t* __restrict__ stamps, uint32_t* __restrict__ flat, int blk, const RawState<SP>* raw_in = nullptr,
    unsigned long long* __restrict__ winkey = nullptr) {
  constexpr bool INLAUNCH = MODE != 0;
  // fp16 stored set (RAW): the wave stages its kept particles' stored values as they are (12 halves, 24 B a
  // row) and the scatter copies them out unchanged, no widening / narrowing (raw_in: the lane's values)
  constexpr bool RAWROW = RAW && !std::is_same<T, SP>::value;
  const int N = fa.N;
  const int lane = lane_id(), wv = wave_id();
  const int g = blk / fa.gsz;
  const int n = blk * kBlock + threadIdx.x;
  const bool valid = n < N;
  const int kiter = c.kept_iter, iters = c.iters;
  const double S = c.S;
  const int64_t Kt = c.K_total;

  // fp32 weights of an M >= 4 frame, all in [0, 32) in this wave: the in-wave prefix as a fixed-point integer scan
  // (wave_incl_sum_fx, exact and equal to the fp64 scan); otherwise the fp64 scan.  Wave-uniform choice.
  const bool fx = std::is_same<T, float>::value && fa.M >= 4 && __ballot(valid && !(wd >= 0.0 && wd < 32.0)) == 0;
  double wi;
  if (fx)
    wi = wave_incl_sum_fx((float)wd);
  else
    wi = wave_incl_sum(wd);
  double incl;
  block_incl_from_wave(wi, incl, sh.sum);
  if (stamps && threadIdx.x == 0) stamp_max(stamps, 10, rt_now());
  // fp32 weights, none negative in the wave, S a normal positive double: every quotient below lies in [0, ~1], so
  // div_by_S is exact (wave-uniform choice; the IEEE division otherwise)
  const bool nonneg = fx || __ballot(valid && wd < 0.0) == 0;
  const bool recip = std::is_same<T, float>::value && nonneg && S > 0x1p-1000 && S < 0x1p1000;
  const double num = gs.G + (bs.E + incl);
  double cn;
  if (recip)
    cn = div_by_S(num, S, c.invS);
  else
    cn = num / S;
  // running max of c seeded by the exact running max at the block start:
  // max(Gin_g, fl(fl(G_g + zin_b)/S)); zin_b = -inf (S > 0) / +inf (S < 0) for a group's first block
  const double zin = S > 0.0 ? bs.zin_max : bs.zin_min;
  const bool first_in_group = (blk % fa.gsz) == 0;
  double rin = gs.Gin;
  if (!first_in_group) {
    const double zn = gs.G + zin;
    const double cz = recip && zn >= 0.0 && zn <= 2.0 * S ? div_by_S(zn, S, c.invS) : zn / S;
    rin = cz > rin ? cz : rin;
  }
  // Running max of c over the wave.  With S > 0 and no negative weight in the wave, c is non-decreasing over
  // its valid lanes (the DPP prefix is lane-monotone, wave_weight_partials; fl(a + x) and x / S > 0 are
  // monotone in x), so the running max is c itself and the wave's maximum sits in its last valid lane.
  // Otherwise the fp64 max scan (wave-uniform branch).
  const uint64_t vmask = __ballot(valid);
  double rm;
  if (S > 0.0 && nonneg) {
    const double last = vmask ? lane_value(cn, 63 - __builtin_clzll(vmask)) : -INFINITY;
    rm = valid ? cn : last;
  } else {
    rm = wave_incl_max(valid ? cn : -INFINITY);
  }
  if (lane == 63) sh.max[wv] = rm;
  __syncthreads();
  double pm = rin;
  const int wvu = wave_id_u();
#pragma clang loop unroll(disable)
  for (int w = 0; w < wvu; ++w) pm = sh.max[w] > pm ? sh.max[w] : pm;
  const double R = rm > pm ? rm : pm;
  int hi = count_targets_wave<T, RNG>(fa, iters, R, valid);  // every lane (one basic block); invalid lanes:
  hi = valid ? hi : N;                                         // their R is the wave's last, the result unused
  if (lane == 63) sh.hi[wv] = hi;
  __syncthreads();
  int lo = wave_shr1(hi, 0);
  if (wv == 0) {  // F(rin), block-uniform: every lane of wave 0 takes the straight-line common case together (rin is
                  // the same in every lane), only lane 0 the rare paths
    const int lo0 = count_targets_wave<T, RNG>(fa, iters, rin, lane == 0);
    if (lane == 0) lo = lo0;
  } else if (lane == 0) {
    lo = sh.hi[wv - 1];
  }
  const int cntn = valid ? hi - lo : 0;
  if (stamps && threadIdx.x == 0) stamp_max(stamps, 11, rt_now());
  if (counts && valid) counts[n] = (uint32_t)cntn;

  // write range [a, e): targets past K_total find nothing and copy the last found particle (the
  // reference keeps the previous Particle_index, PE:681)
  int a, e;
  if (!valid) {
    a = e = N;
  } else if (Kt == 0) {
    a = 0;
    e = (n == N - 1) ? N : 0;
  } else if (lo >= Kt) {
    a = e = N;
  } else if (hi == Kt) {
    a = lo;
    e = N;
  } else {
    a = lo;
    e = hi;
  }

  {  // block max count, first index (winner candidates)
    int cv, ci;
    // wave-uniform: every count of the wave below 2^23 (always at N < 2^23; at larger N all but degenerate frames)
    if (N < (1 << 23) || __ballot(valid && cntn >= (1 << 23)) == 0) {
                          // (count, index) as ONE int key, count * 256 + (255 - thread), whose max
                          // is the max count at its lowest index; integer max needs no canonicalising, and the
                          // rows are combined through four lane reads
      // (bound_ctrl: every lane of these patterns has a source, so each move folds into a v_max_i32_dpp; the row
      // results are carried to lane 63 by the two row broadcasts and read once)
      int k = valid ? cntn * 256 + (255 - (int)threadIdx.x) : -1;
      k = max(k, __builtin_amdgcn_mov_dpp(k, kDppQuadXor1, 0xf, 0xf, true));
      k = max(k, __builtin_amdgcn_mov_dpp(k, kDppQuadXor2, 0xf, 0xf, true));
      k = max(k, __builtin_amdgcn_mov_dpp(k, kDppRowHalfMirror, 0xf, 0xf, true));
      k = max(k, __builtin_amdgcn_mov_dpp(k, kDppRowMirror, 0xf, 0xf, true));
      k = max(k, dpp<kDppBcast15, 0xa>(k, INT_MIN));
      k = max(k, dpp<kDppBcast31, 0xc>(k, INT_MIN));
      k = __builtin_amdgcn_readlane(k, 63);
      cv = k < 0 ? -1 : k >> 8;
      ci = k < 0 ? 0x7fffffff : blk * kBlock + 255 - (k & 255);
    } else {
      cv = valid ? cntn : -1;
      ci = valid ? n : 0x7fffffff;
      wave_argmax(cv, ci);
    }
    if (lane == 0) {
      sh.c[wv] = cv;
      sh.ci[wv] = ci;
    }
  }

  if (stamps && threadIdx.x == 0) stamp_max(stamps, 20, rt_now());
  // the kept-iteration particle (regenerated only by lanes that own slots)
  T P[12];
#pragma unroll
  for (int q = 0; q < 12; ++q) P[q] = have_P ? P_in[q] : (T)0;
  if (!have_P && e > a) propagate<T, RNG>(fa, sc, A, n, kiter, P);
  if (valid && n == c.most_likely_idx) {  // the most likely pose for the frame record (write-through)
    T Q[12];
#pragma unroll
    for (int q = 0; q < 12; ++q) Q[q] = P[q];
    if (RAW)  // P holds stored state values (fp16: deltas), not the pose: regenerate this one particle
      make_particle<T, RNG, SP>(fa, sc, prior, n, kiter, Q);
    else if (!have_P && !(e > a))
      propagate<T, RNG>(fa, sc, A, n, kiter, Q);
#pragma unroll
    for (int q = 0; q < 12; ++q) st_wt_d(mlpose + q, (double)Q[q]);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // drained before the block barrier / arrival
  }

  // Wave-cooperative scatter.  The wave's lanes own consecutive slot ranges [a, e) (empty lanes have
  // a = e = the next start), so slot k belongs to the highest non-empty lane whose start is <= k.  Per
  // 64-slot chunk: starts inside the chunk mark their lane in an LDS map, a DPP max-scan (carried
  // across chunks) fills every slot's owner, and the slot lane reads the owner's row from LDS.
  const int wa = lane_value(a, 0);
  const int we = lane_value(e, 63);
  auto& rows = sh.rows[wv];
  uint2* rraw = (uint2*)&rows[0];  // RAWROW: three 8-B words per row
  // Deferred resampling (two-launch frames with the kept set, MODE 0, fa.owner_out set): the new prior is the
  // kept set read through owner indices, so the scatter writes slot k's owner (a particle index, 4 B) instead of
  // the particle (S bytes), and nothing is staged: the next frame's weighing pass gathers kept[owner[k]].
  const bool owners = MODE == 0 && RAW && fa.owner_out != nullptr;  // wave-uniform
  if (owners) {
    // (no rows: k_resample_final regenerates the winner, as for every RAW frame)
  } else if constexpr (RAWROW) {
#pragma unroll
    for (int j = 0; j < 3; ++j)
      rraw[3 * lane + j] = make_uint2(__builtin_bit_cast(uint32_t, raw_in->p[2 * j]),
                                      __builtin_bit_cast(uint32_t, raw_in->p[2 * j + 1]));
  } else {
#pragma unroll
    for (int q = 0; q < 12; ++q) rows[lane].q[q] = P[q];  // also read by wave 0 for the block candidate
  }
  if (we > wa) {
    int* map = sh.map[wv];
    int carry = -1;
    if (stamps && threadIdx.x == 0) stamp_max(stamps, 21, rt_now());
    for (int base = wa; base < we; base += 64) {
      map[lane] = -1;
      wave_lds_sync();
      const int d = a - base;
      if (e > a && d >= 0 && d < 64) map[d] = lane;
      wave_lds_sync();
      int own = map[lane];
      own = wave_scan(own, INT_MIN, OpMaxI());  // INT_MIN fill: each step folds into one v_max_i32_dpp
      own = own > carry ? own : carry;
      carry = lane_value(own, 63);
      const int k = base + lane;
      wave_lds_sync();  // rows (before the loop) and this chunk's map reads are done before the next clear
      if (k < we && owners) {
        fa.owner_out[k] = (uint32_t)(blk * kBlock + wv * 64 + own);
      } else if (k < we) {
        if constexpr (RAWROW) {
          uint32_t w6[6];
#pragma unroll
          for (int j = 0; j < 3; ++j) {
            const uint2 x = rraw[3 * own + j];
            w6[2 * j] = x.x;
            w6[2 * j + 1] = x.y;
          }
          store_state_words_f16(post, fa.ld, k, w6);
        } else {
          SP v[12];
          const auto& row = rows[own];
#pragma unroll
          for (int q = 0; q < 12; ++q) v[q] = RAW ? SP(row.q[q]) : StateIO<T, SP>::store(row.q[q], fa.anc_out[q]);
          store_state_raw<SP>(post, fa.ld, k, v);
        }
      }
    }
  }

  if (stamps && threadIdx.x == 0) stamp_max(stamps, 12, rt_now());
  __syncthreads();
  if (!INLAUNCH) {  // block partial + the block argmax's kept pose (plain stores: the launch boundary
                    // publishes them); a block without copies has no propagated row, k_resample_final regenerates
    if (wv == 0) {
      int bv = sh.c[0], bi = sh.ci[0];
      for (int w = 1; w < kWaves; ++w) cmb_max(bv, bi, sh.c[w], sh.ci[w]);
      if (lane == 0) cpart[blk] = CountPart{bv, bi};
      // one-stream k_resample: the block's candidate also goes into the sharded winner keys (max count, then the
      // lowest index: count in the high word, 2^31 - 1 - index in the low one), so k_resample_final reads
      // kWinShards keys instead of every block's partial (C4: 39k partials, three round trips)
      if (winkey && lane == 0 && bv >= 0)
        __hip_atomic_fetch_max(winkey + (blk & (kWinShards - 1)) * kWinStride, win_key(bv, bi), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
      const int loc = bi - blk * kBlock;
      if (!RAW && lane < 12 && bv > 0) ((T*)(cand + blk))[lane] = sh.rows[loc >> 6][loc & 63].q[lane];
      if (stamps && lane == 0) stamp_max(stamps, 5, rt_now());
    }
    return;
  }
  if (wv == 1) {  // this block's winner candidate, in parallel with wave 0's arrival
    int cbv = sh.c[0], cbi = sh.ci[0];
    for (int w = 1; w < kWaves; ++w) cmb_max(cbv, cbi, sh.c[w], sh.ci[w]);
    // a candidate with copies was propagated by its lane (staged rows); with no copies anywhere in the
    // block (only possible when every count of the frame is 0: the winner is particle 0, PE:685) it is
    // regenerated here
    const int loc = cbi - blk * kBlock;
    T Pc[12];
    if (cbv > 0 && (!RAW || std::is_same<T, SP>::value)) {  // RAW rows are poses unless the state is fp16 deltas
#pragma unroll
      for (int q = 0; q < 12; ++q) Pc[q] = sh.rows[loc >> 6][loc & 63].q[q];
    } else {
      make_particle<T, RNG, SP>(fa, sc, prior, cbi, kiter, Pc);
    }
    const uint32_t pl = cand_payload<T, MAXM>(fa, sc, tb, Pc, sh.ccorr);
    if (lane < kCandGran) st_wt(&cand[blk].g[lane], ((uint64_t)(uint32_t)seq << 32) | pl);
    if (stamps && lane == 0) stamp_max(stamps, 22, rt_now());
    return;
  }
  if (wv != 0) return;

  if (MODE == 2) {  // flat: the count partial as two granules {count, index}; block 0 polls every block's and finishes
    {
      int bv = sh.c[0], bi = sh.ci[0];
      for (int w = 1; w < kWaves; ++w) cmb_max(bv, bi, sh.c[w], sh.ci[w]);
      if (lane < 2) store_granule((uint64_t*)cpart + 2 * blk + lane, fa.gtag, (uint32_t)(lane ? bi : bv));
      if (stamps && lane == 0) stamp_max(stamps, 5, rt_now());
    }
    if (blk != 0) return;
    // every count partial of the frame (nblk <= kFlatMaxGroups * kGroup = 8 per lane), one 16-B load each, all in
    // flight together, re-read until every tag is this frame's (bounded: abandoned); then combined, a lane past
    // nblk holding the identity (count -1)
    int bv = -1, bi = 0x7fffffff;
    {
      u32x4_t cp[kFlatMaxGroups] = {};
      const uint64_t t0 = rt_now();
      for (;;) {
#pragma unroll
        for (int j = 0; j < kFlatMaxGroups; ++j) {
          const int t = lane + 64 * j;
          cp[j] = ld_gran2_issue((const uint64_t*)cpart + 2 * (t < fa.nblk ? t : 0));
        }
        asm volatile("s_waitcnt vmcnt(0)" : "+v"(cp[0]), "+v"(cp[1]), "+v"(cp[2]), "+v"(cp[3]), "+v"(cp[4]), "+v"(cp[5]),
                     "+v"(cp[6]), "+v"(cp[7])::"memory");
        static_assert(kFlatMaxGroups == 8, "the wait's operand list");
        bool stale = false;
#pragma unroll
        for (int j = 0; j < kFlatMaxGroups; ++j)
          stale |= lane + 64 * j < fa.nblk && (cp[j].y != fa.gtag || cp[j].w != fa.gtag);
        if (!__builtin_amdgcn_ballot_w64(stale)) break;
        if (rt_now() - t0 > fa.wait_ticks) return;  // abandoned
        __builtin_amdgcn_s_sleep(1);
      }
#pragma unroll
      for (int j = 0; j < kFlatMaxGroups; ++j)
        if (lane + 64 * j < fa.nblk) cmb_max(bv, bi, (int)cp[j].x, (int)cp[j].z);
    }
    wave_argmax(bv, bi);
    if (stamps && lane == 0) stamps[6] = rt_now();
    finalize_frame<T, RNG, MAXM, SP>(fa, sc, c, ctrl, prior, bi, cand, mlpose, rec, out, 2 * seq + 1, stamps);
    if (stamps && lane == 0) stamps[7] = rt_now();
    return;
  }
  int last = 0;
  if (lane == 0) {
    int bv = sh.c[0], bi = sh.ci[0];
    for (int w = 1; w < kWaves; ++w) cmb_max(bv, bi, sh.c[w], sh.ci[w]);
    st_wt(cpart + blk, pack2(bv, bi));
    if (stamps) stamp_max(stamps, 5, rt_now());
    last = arrive_last(gcount + g, min(fa.gsz, fa.nblk - g * fa.gsz)) ? 1 : 0;
  }
  if (!lane_value(last, 0)) return;
  // group: max count over its blocks (first index on ties)
  int bv = -1, bi = 0x7fffffff;
  {
    const int b0 = g * fa.gsz, nb = min(fa.gsz, fa.nblk - b0);
    for (int t = lane; t < nb; t += 64) {
      const uint64_t cp = ld_wt(cpart + b0 + t);
      cmb_max(bv, bi, lo32(cp), hi32(cp));
    }
    wave_argmax(bv, bi);
  }
  if (fa.ngrp > 1) {
    if (lane == 0) st_wt(cgroup + g, pack2(bv, bi));
    if (!wave_arrive_last(tcount, fa.ngrp)) return;
    bv = -1;
    bi = 0x7fffffff;
    for (int gg = lane; gg < fa.ngrp; gg += 64) {
      const uint64_t cp = ld_wt(cgroup + gg);
      cmb_max(bv, bi, lo32(cp), hi32(cp));
    }
    wave_argmax(bv, bi);
  }
  if (stamps && lane == 0) stamps[6] = rt_now();
  // winner = argmax resample count, first index (PE:685-686)
  finalize_frame<T, RNG, MAXM, SP>(fa, sc, c, ctrl, prior, bi, cand, mlpose, rec, out, 2 * seq + 1, stamps);
  if (stamps && lane == 0) stamps[7] = rt_now();
}

// ---- launch 2 of the two-launch path: stratified resampling + winner + frame record.  One block's work
// (block `blk` of its stream), shared by k_resample and k_resample_multi.
// KEPT: every block of the launch has the kept propagated set (prop0 != null), so the regeneration path and its
// registers are compiled out (the generic form, KEPT = false, tests prop0 at run time).
template <typename T, int RNG, int MAXM, typename SP, bool MULTI, bool KEPT>
__device__ __forceinline__ void resample_block(
    const FrameArgsT<T>& fa, const uint32_t* fa_words, int blk, Ctrl* __restrict__ ctrl,
    const unsigned char* __restrict__ table, const SP* __restrict__ prior, SP* __restrict__ post,
    const T* __restrict__ w0, const T* __restrict__ w1, const BlockScan* __restrict__ bscan0,
    const BlockScan* __restrict__ bscan1, const GroupScan* __restrict__ gscan, CountPart* __restrict__ cpart,
    CountPart* __restrict__ cgroup, uint32_t* __restrict__ gcount, uint32_t* __restrict__ tcount,
    uint32_t* __restrict__ counts, Cand* __restrict__ cand, double* __restrict__ mlpose, RecOut* __restrict__ out,
    int32_t seq, uint64_t* __restrict__ stamps, const SP* __restrict__ prop0, const SP* __restrict__ prop1,
    LdsConst<T>& sc, OutDev& rec, ResampleLds<T>& sh, unsigned long long* __restrict__ winkey = nullptr) {
  if (stamps && threadIdx.x == 0) stamp_min(stamps, 4, rt_now());
  const int g = blk / fa.gsz;
  const int n = blk * kBlock + threadIdx.x;
  const bool valid = n < fa.N;
  // The frame constants go to LDS first (visible after block_incl_sum's barrier): their copy waits for its
  // own loads (vmcnt retires in order), so issued before the weight / state loads it does not wait for them.
  stage_consts_from(fa_words, sc);
  // Everything that does not depend on the control record is requested first (both weight slots: the
  // kept one is known only from ctrl), so the loads overlap the ctrl read.  Loading only the kept slot after
  // the ctrl read saves 4 B per particle of HBM reads but serialises the weight load behind it: C4 k_resample
  // 163 -> 174 us (profiles/r03/ab_grid2.log), so both slots stay.
  T wt0 = (T)0, wt1 = (T)0;
  if (valid) {
    wt0 = w0[n];
    wt1 = w1[n];
  }
  const BlockScan bsa = bscan0[blk], bsb = bscan1[blk];
  const GroupScan gs = gscan[g];
  const bool kept = KEPT || prop0 != nullptr;
  T A[12];
  if (!kept && valid && n >= 2) load_prior(fa, prior, n, A);
  const Ctrl c = MULTI ? load_ctrl_uniform(ctrl) : *ctrl;
  // speculative launch of an unfinished frame, or the re-init branch (PE:707-719): nothing to resample;
  // k_resample_final writes the record
  if (!c.done || !c.accepted) return;
  // the kept iteration's stored propagated set, gathered as raw state values (no regeneration).  fp16: planes
  // 2j and 2j + 1 are word j (one dword of the pair plane), which is the row layout resample_phase stages
  RawState<SP> KR{};
  // deferred resampling writes owner indices only: the kept set is not read here (fa.owner_out uniform)
  if (kept && !fa.owner_out) {
    const SP* src = c.kept_slot ? prop1 : prop0;
    // buffer-resource planes: every lane loads (a lane past N at the index clamped into [0, N), in_planes), so
    // no branch: behind one, the weights' wait before the block scan became vmcnt(0) and also waited for these
    // loads
    if constexpr (std::is_same<SP, __half>::value) {
      load_state_prefetch<SP>(src, fa.ld, in_planes(n, fa.N), true, KR);
    } else {
      SP V[12];
#pragma unroll
      for (int q = 0; q < 12; ++q) V[q] = SP(0.0f);
      if (BufPlanes<SP>::value || valid) load_state_raw<SP>(src, fa.ld, in_planes(n, fa.N), V);
#pragma unroll
      for (int q = 0; q < 12; ++q) A[q] = V[q];
    }
  }
  const int slot = c.kept_slot;
  const double wd = valid ? (double)(slot ? wt1 : wt0) : 0.0;
  const BlockScan bs = slot ? bsb : bsa;  // by value: a reference to either local would force both to memory
  const LdsBlobs<T> tb = view_table<T>(table, fa.B);  // global memory (L2) in this launch
  if (kept)
    resample_phase<T, RNG, MAXM, SP, 0, true>(fa, sc, c, ctrl, table, prior, post, wd, A, A, true, bs, gs, sh, rec, tb,
                                              cand, mlpose, cpart, cgroup, gcount, tcount, counts, out, seq, stamps,
                                              nullptr, blk, &KR, winkey);
  else
    resample_phase<T, RNG, MAXM, SP, 0>(fa, sc, c, ctrl, table, prior, post, wd, A, A, false, bs, gs, sh, rec, tb, cand,
                                        mlpose, cpart, cgroup, gcount, tcount, counts, out, seq, stamps, nullptr, blk,
                                        nullptr, winkey);
}

// Occupancy floor of k_resample / k_resample_multi (waves per SIMD; 1 = the compiler's choice).  Unconstrained
// the fp16-state k_resample takes 85 VGPRs (5 waves); the fp16 TUs set 7 (72 VGPRs, a few rarely-live values
// spilled): at C4 (10M particles) 196 -> 170 us, the kernel being latency bound.  The fp32 TUs
// set 6 (batched 16-32 x C2 / C5 +2-3 %).  8 waves spill 78 VGPRs.
#ifndef PFMPE_RESAMPLE_MIN_WAVES
#define PFMPE_RESAMPLE_MIN_WAVES 1
#endif
// The kept-set variants (KEPT: no regeneration path, 60-66 VGPRs) take their own floor.
#ifndef PFMPE_RESAMPLE_KEPT_MIN_WAVES
#define PFMPE_RESAMPLE_KEPT_MIN_WAVES 8
#endif
template <typename T, int RNG, int MAXM, typename SP, bool KEPT>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(KEPT ? PFMPE_RESAMPLE_KEPT_MIN_WAVES : PFMPE_RESAMPLE_MIN_WAVES))) void k_resample(
    const FrameArgsT<T> fa, Ctrl* __restrict__ ctrl, const unsigned char* __restrict__ table, const SP* __restrict__ prior,
    SP* __restrict__ post, const T* __restrict__ w0, const T* __restrict__ w1, const BlockScan* __restrict__ bscan0,
    const BlockScan* __restrict__ bscan1, const GroupScan* __restrict__ gscan, CountPart* __restrict__ cpart,
    CountPart* __restrict__ cgroup, uint32_t* __restrict__ gcount, uint32_t* __restrict__ tcount,
    uint32_t* __restrict__ counts, Cand* __restrict__ cand, double* __restrict__ mlpose, RecOut* __restrict__ out,
    int32_t seq, uint64_t* __restrict__ stamps, const SP* __restrict__ prop0, const SP* __restrict__ prop1,
    unsigned long long* __restrict__ winkey) {
  __shared__ LdsConst<T> sc;
  __shared__ OutDev rec;
  __shared__ ResampleLds<T> sh;
  resample_block<T, RNG, MAXM, SP, false, KEPT>(fa, (const uint32_t*)__builtin_amdgcn_kernarg_segment_ptr(), (int)blockIdx.x, ctrl,
                                   table, prior, post, w0, w1, bscan0, bscan1, gscan, cpart, cgroup, gcount, tcount,
                                   counts, cand, mlpose, out, seq, stamps, prop0, prop1, sc, rec, sh, winkey);
}

template <typename T, int RNG, int MAXM, typename SP, bool KEPT>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(KEPT ? PFMPE_RESAMPLE_KEPT_MIN_WAVES : PFMPE_RESAMPLE_MIN_WAVES))) void k_resample_multi(
    const StreamDesc<T, SP>* __restrict__ descs, const uint16_t* __restrict__ bmap, int S,
    const uint32_t* __restrict__ status, uint32_t gen) {
  __shared__ LdsConst<T> sc;
  __shared__ OutDev rec;
  __shared__ ResampleLds<T> sh;
  int s = 0;
  const int blk = batch_block(descs, bmap, S, status, gen, &s);
  if (blk < 0) return;
  const StreamDesc<T, SP>& d = descs[s];
  resample_block<T, RNG, MAXM, SP, true, KEPT>(d.fa, (const uint32_t*)&d.fa, blk, d.ctrl, d.table,
                                   d.prior, d.post, d.w0, d.w1, d.bscan0, d.bscan1, d.gscan, d.cpart, d.cgroup,
                                   d.gcount_r, d.tcount_r, d.counts, d.cand, d.mlpose, d.out, d.seq, nullptr, d.prop0,
                                   d.prop1, sc, rec, sh);
}

// ---- launch 2 of a deferred two-launch frame: stratified resampling by waves that each own
// whole 256-particle blocks.  The frame has the kept propagated set and defers the new prior (fa.owner_out), so a
// block's work is its scan, its target counts, its owner indices and its winner key: nothing that needs other waves.
// Lane l handles the block's particles l, 64 + l, 128 + l, 192 + l ("chunks" c = 0..3, exactly the four waves of
// resample_phase), so every scan keeps resample_phase's association: the chunk's DPP scan, then the earlier chunks'
// totals added in chunk order (block_incl_from_wave's `pre`), the running maximum carried from chunk to chunk in
// the order of its `pm` loop, and the lower target count of lane 0 taken from the previous chunk's lane 63 (the
// `sh.hi` hand-off) or, for chunk 0, F(rin).  The wave-uniform shortcuts (fixed-point scan, division by
// reciprocal, monotone running max, integer winner keys) are each decided once for the four chunks; every one of
// them yields the same bits as its general form wherever it is taken, so the decision granularity does not change
// any output.  Outputs are resample_phase's for MODE 0 with owner_out: owner_out, counts, the winner key and the
// most-likely pose (k_resample_final reads the keys, not the count partials, which are therefore not written).
// No workgroup barrier: the per-wave scalar work (control record, kernel arguments, loop control) is paid once per
// wave, and a wave never waits for another.
//
// (Tried: a wave owning 2-4 consecutive blocks, reusing the previous block's last target count as F(rin) when rin is
// bit-identical to its last R: 10 % fewer VALU and 17 % fewer SALU per particle at C4, but the carried state pushed
// the kernel past 100 SGPRs (54 spilled to VGPR lanes, scratch) and it measured 0-2 % slower at C4 and 7-22 %
// slower at C5 (profiles/r05/owners_bpw_ab.txt).)
template <typename T>
struct OwnersLds {
  LdsConst<T> sc;  // the frame constants, staged only by the wave holding the most-likely particle
};
// before_stores(key): called by the whole wave with the block's winner key (and the most-likely pose written
// through) before the owner stores are issued (the fused finish publishes the key and arrives there, so its drain
// does not wait for the owner stores).
template <typename T, int RNG, typename SP, typename BeforeStores>
__device__ __forceinline__ void resample_owners_block(const FrameArgsT<T>& fa, const uint32_t* fa_words, int blk,
                                                      const Ctrl& c, const SP* __restrict__ prior,
                                                      const T* __restrict__ wk, __amdgpu_buffer_rsrc_t orsrc,
                                                      const BlockScan* __restrict__ bsk,
                                                      const GroupScan* __restrict__ gscan, uint32_t* __restrict__ counts,
                                                      double* __restrict__ mlpose, OwnersLds<T>& sh, double& carry_R,
                                                      int& carry_hi, unsigned long long& key,
                                                      BeforeStores&& before_stores) {
  constexpr int kC = kBlock / 64;
  constexpr uint32_t kDrop = 0x80000000u;  // a buffer offset past num_records: the access is dropped / reads 0
  const int N = fa.N;
  const int lane = lane_id();
  const int base_n = blk * kBlock;
  const int iters = c.iters;
  const double S = c.S;
  const int64_t Kt = c.K_total;
  // the kept weight slot (wk) of the block's four chunks: one lane offset from the block's (uniform) base, the chunk
  // as an immediate; the weight buffers hold whole blocks (pfmpe_create), a lane past N is masked below
  const T* wb = wk + base_n;
  T w[kC];
#pragma unroll
  for (int q = 0; q < kC; ++q) w[q] = wb[lane + 64 * q];
  const BlockScan bs = bsk[blk];
  const GroupScan gs = gscan[blk / fa.gsz];
  bool valid[kC];
  bool out_fx = false, out_neg = false;
#pragma unroll
  for (int q = 0; q < kC; ++q) {
    valid[q] = base_n + q * 64 + lane < N;
    w[q] = valid[q] ? w[q] : (T)0;
    out_fx |= !(w[q] >= (T)0 && w[q] < (T)32);
    out_neg |= w[q] < (T)0;
  }
  // resample_phase's per-wave choices, taken for the four chunks at once (same bits either way, see above)
  const bool fx = std::is_same<T, float>::value && fa.M >= 4 && __ballot(out_fx) == 0;
  const bool nonneg = fx || __ballot(out_neg) == 0;
  const bool recip = std::is_same<T, float>::value && nonneg && S > 0x1p-1000 && S < 0x1p1000;
  // running max at the block start (resample_phase's rin)
  double rin = gs.Gin;
  if ((blk % fa.gsz) != 0) {
    const double zin = S > 0.0 ? bs.zin_max : bs.zin_min;
    const double zn = gs.G + zin;
    const double cz = recip && zn >= 0.0 && zn <= 2.0 * S ? div_by_S(zn, S, c.invS) : zn / S;
    rin = cz > rin ? cz : rin;
  }
  // F(rin): the previous block's last count when rin is its last R, else every lane takes the straight-line common
  // case together and lane 0 alone the rare paths
  int prev_hi = carry_hi;
  if (__double_as_longlong(rin) != __double_as_longlong(carry_R))
    prev_hi = lane_value(count_targets_wave<T, RNG>(fa, iters, rin, lane == 0), 0);
  double pre = 0.0;  // the earlier chunks' totals, summed in chunk order
  double pm = rin;   // the running max over rin and the earlier chunks
  int ra[kC], re[kC], rc[kC];
  int kmax = -1;  // max of count * 256 + (255 - particle in block): the max count at its lowest index
  int cmax = -1;  // the lane's largest count
#pragma unroll
  for (int q = 0; q < kC; ++q) {
    const double wi = fx ? wave_incl_sum_fx((float)w[q]) : wave_incl_sum((double)w[q]);
    const double incl = pre + wi;
    pre = pre + lane_value(wi, 63);
    const double num = gs.G + (bs.E + incl);
    const double cn = recip ? div_by_S(num, S, c.invS) : num / S;
    double rm;
    if (S > 0.0 && nonneg) {  // c is non-decreasing over the chunk's valid lanes: its running max is c itself
      const uint64_t vmask = __ballot(valid[q]);
      const double last = vmask ? lane_value(cn, 63 - __builtin_clzll(vmask)) : -INFINITY;
      rm = valid[q] ? cn : last;
    } else {
      rm = wave_incl_max(valid[q] ? cn : -INFINITY);
    }
    const double R = rm > pm ? rm : pm;
    const double mq = lane_value(rm, 63);
    pm = mq > pm ? mq : pm;
    int hi = count_targets_wave<T, RNG>(fa, iters, R, valid[q]);
    hi = valid[q] ? hi : N;
    int lo = wave_shr1(hi, 0);
    if (lane == 0) lo = prev_hi;
    prev_hi = lane_value(hi, 63);
    const int cntn = valid[q] ? hi - lo : 0;
    if (counts) counts[base_n + lane + 64 * q] = (uint32_t)cntn;  // (whole blocks allocated: pfmpe_create)
    // write range [a, e) (resample_phase: targets past K_total copy the last found particle, PE:681), as selects
    int a = lo, e = hi == Kt ? N : hi;
    a = lo >= Kt ? N : a;
    e = lo >= Kt ? N : e;
    if (Kt == 0) {  // (wave-uniform) no target found a particle: every slot copies the last one
      a = 0;
      e = base_n + q * 64 + lane == N - 1 ? N : 0;
    }
    ra[q] = valid[q] ? a : N;
    re[q] = valid[q] ? e : N;
    rc[q] = valid[q] ? cntn : -1;
    kmax = max(kmax, valid[q] ? cntn * 256 + (255 - (q * 64 + lane)) : -1);  // (unused if a count is >= 2^23)
    cmax = max(cmax, rc[q]);
  }
  carry_R = pm;        // the block's last R (its last particle's, when that one is valid)
  carry_hi = prev_hi;  // F of it
  // block max count, first index (the winner candidate): one integer key unless some count is >= 2^23 (always below
  // at N < 2^23; at larger N all but degenerate frames)
  int bv, bi;
  if (N < (1 << 23) || __ballot(cmax >= (1 << 23)) == 0) {
    int k = kmax;
    k = max(k, __builtin_amdgcn_mov_dpp(k, kDppQuadXor1, 0xf, 0xf, true));
    k = max(k, __builtin_amdgcn_mov_dpp(k, kDppQuadXor2, 0xf, 0xf, true));
    k = max(k, __builtin_amdgcn_mov_dpp(k, kDppRowHalfMirror, 0xf, 0xf, true));
    k = max(k, __builtin_amdgcn_mov_dpp(k, kDppRowMirror, 0xf, 0xf, true));
    k = max(k, dpp<kDppBcast15, 0xa>(k, INT_MIN));
    k = max(k, dpp<kDppBcast31, 0xc>(k, INT_MIN));
    k = __builtin_amdgcn_readlane(k, 63);
    bv = k < 0 ? -1 : k >> 8;
    bi = k < 0 ? 0x7fffffff : base_n + 255 - (k & 255);
  } else {
    bv = -1;
    bi = 0x7fffffff;
#pragma unroll
    for (int q = 0; q < kC; ++q) cmb_max(bv, bi, rc[q], rc[q] >= 0 ? base_n + q * 64 + lane : 0x7fffffff);
    wave_argmax(bv, bi);
  }
  if (bv >= 0) {  // the wave's key: max over its blocks (win_key orders as (count, lowest index))
    const unsigned long long kb = win_key(bv, bi);
    key = kb > key ? kb : key;
  }

  // the most likely pose for the frame record (write-through), regenerated by its lane (the kept set holds stored
  // state values, not poses); the frame constants are staged by this one wave (wave-uniform test)
  const int mli = c.most_likely_idx;
  if (mli >= base_n && mli < base_n + kBlock && mli < N) {
    uint32_t* dst = (uint32_t*)&sh.sc;
    constexpr int kWordsC = (int)(sizeof(LdsConst<T>) / 4);
    for (int i = lane; i < kWordsC; i += 64) dst[i] = fa_words[i];
    wave_lds_sync();
    if (lane == ((mli - base_n) & 63)) {
      T Q[12];
      make_particle<T, RNG, SP>(fa, sh.sc, prior, mli, c.kept_iter, Q);
#pragma unroll
      for (int q = 0; q < 12; ++q) st_wt_d(mlpose + q, (double)Q[q]);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }

  before_stores(key);
  // Owner indices: particle p of the block owns the slots [ra, re) of its lane and chunk (consecutive, non-empty
  // ranges in particle order).  Each lane writes its own particles' ranges: first 16-B stores of four slots while at
  // least four remain, then single slots; a store past its range goes to an offset the buffer's range check drops
  // (no exec-mask branches), the round's step in soffset.  In a typical frame every range is a few slots and the
  // lanes' ranges are adjacent, so a round's stores fall on a few consecutive lines; where the weight concentrates
  // (ranges of tens of slots over a whole region of the set) the 16-B stores quarter the write transactions.  A range
  // longer than kWide (one particle taking a large share of the targets) is written by the whole wave, 64
  // consecutive slots per store, one such particle after another.
  constexpr int kWide = 256;
  int nq[kC], nr[kC];
  int m4 = 0, m1 = 0;
  bool wide = false;
#pragma unroll
  for (int q = 0; q < kC; ++q) {
    const int len = re[q] - ra[q];
    nq[q] = len <= kWide ? len >> 2 : 0;
    nr[q] = len <= kWide ? len & 3 : 0;
    m4 = max(m4, nq[q]);
    m1 = max(m1, nr[q]);
    wide |= len > kWide;
  }
  m4 = max(m4, __builtin_amdgcn_mov_dpp(m4, kDppQuadXor1, 0xf, 0xf, true));
  m4 = max(m4, __builtin_amdgcn_mov_dpp(m4, kDppQuadXor2, 0xf, 0xf, true));
  m4 = max(m4, __builtin_amdgcn_mov_dpp(m4, kDppRowHalfMirror, 0xf, 0xf, true));
  m4 = max(m4, __builtin_amdgcn_mov_dpp(m4, kDppRowMirror, 0xf, 0xf, true));
  m4 = max(m4, dpp<kDppBcast15, 0xa>(m4, 0));
  m4 = max(m4, dpp<kDppBcast31, 0xc>(m4, 0));
  m4 = __builtin_amdgcn_readlane(m4, 63);
  // the largest remainder (<= 3) by ballots
  m1 = __builtin_amdgcn_ballot_w64(m1 >= 3) ? 3 : __builtin_amdgcn_ballot_w64(m1 >= 2) ? 2
                                                : __builtin_amdgcn_ballot_w64(m1 >= 1) ? 1 : 0;
  if (m4 > 0) {
    u32x4_t o4[kC];
#pragma unroll
    for (int q = 0; q < kC; ++q) {
      const uint32_t o = (uint32_t)(base_n + q * 64 + lane);
      o4[q] = u32x4_t{o, o, o, o};
    }
    for (int j = 0; j < m4; ++j) {
#pragma unroll
      for (int q = 0; q < kC; ++q)
        __builtin_amdgcn_raw_buffer_store_b128(o4[q], orsrc, j < nq[q] ? (uint32_t)ra[q] * 4u : kDrop,
                                               (uint32_t)(16 * j), 0);
    }
  }
  for (int j = 0; j < m1; ++j) {
#pragma unroll
    for (int q = 0; q < kC; ++q)
      __builtin_amdgcn_raw_buffer_store_b32((uint32_t)(base_n + q * 64 + lane), orsrc,
                                            j < nr[q] ? (uint32_t)(ra[q] + 4 * nq[q]) * 4u : kDrop, (uint32_t)(4 * j),
                                            0);
  }
  if (__builtin_amdgcn_ballot_w64(wide)) {
#pragma unroll
    for (int q = 0; q < kC; ++q) {
      uint64_t m = __builtin_amdgcn_ballot_w64(re[q] - ra[q] > kWide);
      while (m) {
        const int l = __builtin_ctzll(m);
        m &= m - 1;
        const int a = __builtin_amdgcn_readlane(ra[q], l);
        const int e = __builtin_amdgcn_readlane(re[q], l);
        const uint32_t own = (uint32_t)(base_n + q * 64 + l);
        for (int k = a; k < e; k += 64) {
          const int kk = k + lane;
          __builtin_amdgcn_raw_buffer_store_b32(own, orsrc, kk < e ? (uint32_t)kk * 4u : kDrop, 0u, 0);
        }
      }
    }
  }
}

// One wave per block, four per workgroup.
#ifndef PFMPE_RESAMPLE_OWNERS_MIN_WAVES
#define PFMPE_RESAMPLE_OWNERS_MIN_WAVES 6
#endif
// The frame's finish in the resampling launch (round 6, VERDICT r05 item 3: no k_resample_final launch after
// k_resample_owners).  Every wave's winner key goes to a key shard with a memory-side maximum; once it (and the wave's
// count / most-likely stores) has drained, the wave arrives on arrival shard blk % 64 (no return value: the wave
// ends).  The wave of the last block, dispatched last (workgroups dispatch in order), finishes the frame: after its
// own key it polls the 64 arrival shards (one per lane, bounded by the frame's wait bound) until each holds its
// blocks' count; then it takes the key shards (exchanged with the identity for the next frame, as k_resample_final
// did) and resets the arrival shards, regenerates the winner's kept pose (the kept set holds stored state values),
// pairs it (pose_pairs over the blob table in device memory) and writes the record (finalize_frame).  The outputs
// are k_resample_final's (same functions, same keys).  Per wave LDS: the frame constants, the record image and the
// pair scratch.
template <typename T>
struct OwnersFinalLds {
  OwnersLds<T> o;
  OutDev rec;
  uint32_t ccorr[2 * kMaxMarkers];
};
template <typename T, int RNG, int MAXM, typename SP>
__device__ __forceinline__ void owners_finish(const FrameArgsT<T>& fa, const uint32_t* fa_words, const Ctrl& c,
                                              Ctrl* __restrict__ ctrl, const SP* __restrict__ prior,
                                              const unsigned char* __restrict__ table, const double* __restrict__ mlpose,
                                              unsigned long long* __restrict__ winkey, RecOut* __restrict__ out,
                                              int32_t seq, uint64_t* __restrict__ stamps, OwnersFinalLds<T>& sh) {
  const int lane = lane_id();
  static_assert(kWinShards == 64, "one shard per lane");
  if (fa.diag & kDiagAbandonFinish) return;  // as if the wait bound expired: no record, keys and arrivals left set
  {  // every other block's arrival (the blocks b < nblk - 1 with b % 64 == lane)
    uint32_t* sh_arrive = win_arrive(winkey) + lane * kArriveStride;
    const uint32_t want = lane < fa.nblk - 1 ? (uint32_t)((fa.nblk - 2 - lane) / 64 + 1) : 0u;
    const uint64_t t0 = rt_now();
    for (;;) {
      const bool pend = __hip_atomic_load(sh_arrive, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < want;
      if (!__builtin_amdgcn_ballot_w64(pend)) break;
      if (rt_now() - t0 > fa.wait_ticks) return;  // (no record: the host reports the frame)
      __builtin_amdgcn_s_sleep(1);
    }
    __hip_atomic_store(sh_arrive, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // the next frame's
  }
  unsigned long long kmax = __hip_atomic_exchange(winkey + lane * kWinStride, 0ull, __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    const unsigned long long other = (unsigned long long)__shfl_xor((long long)kmax, o, 64);
    kmax = other > kmax ? other : kmax;
  }
  const int bi = kmax ? 0x7fffffff - (int)(uint32_t)kmax : 0x7fffffff;
  double ml = 0.0;
  if (lane < 12) ml = ld_wt_d(mlpose + lane);  // written through by the wave of the most likely particle
  uint32_t* dst = (uint32_t*)&sh.o.sc;
  constexpr int kWordsC = (int)(sizeof(LdsConst<T>) / 4);
  for (int i = lane; i < kWordsC; i += 64) dst[i] = fa_words[i];
  wave_lds_sync();
  if (stamps && lane == 0) stamps[24] = rt_now();
  T Pc[12];
  make_particle<T, RNG, SP>(fa, sh.o.sc, prior, bi, c.kept_iter, Pc);
  const LdsBlobs<T> tb = view_table<T>(table, fa.B);
  const uint32_t pl = cand_payload<T, MAXM>(fa, sh.o.sc, tb, Pc, sh.ccorr);
  if (stamps && lane == 0) stamps[26] = rt_now();
  finalize_frame<T, RNG, MAXM, SP>(fa, sh.o.sc, c, ctrl, prior, bi, nullptr, mlpose, sh.rec, out, 2 * seq + 1, stamps,
                                   true, pl, ml);
  if (stamps && lane == 0) stamps[7] = rt_now();
}
// The unfinished and re-init frames (no resampling): block 0's first wave writes the record.
template <typename T, int RNG, int MAXM, typename SP>
__device__ __forceinline__ void owners_no_resample(const FrameArgsT<T>& fa, const uint32_t* fa_words, const Ctrl& c,
                                                   Ctrl* __restrict__ ctrl, const SP* __restrict__ prior,
                                                   const double* __restrict__ mlpose, RecOut* __restrict__ out,
                                                   int32_t seq, uint64_t* __restrict__ stamps, OwnersFinalLds<T>& sh) {
  const int lane = lane_id();
  if (!c.done) {  // an iteration batch the exit rule has not ended: granule 0 alone, tag 2 * seq (the host goes on)
    if (lane == 0) st_sys64(&out->g[0], (uint64_t)(uint32_t)(2 * seq) << 32);
    return;
  }
  uint32_t* dst = (uint32_t*)&sh.o.sc;
  constexpr int kWordsC = (int)(sizeof(LdsConst<T>) / 4);
  for (int i = lane; i < kWordsC; i += 64) dst[i] = fa_words[i];
  wave_lds_sync();
  finalize_frame<T, RNG, MAXM, SP>(fa, sh.o.sc, c, ctrl, prior, -1, nullptr, mlpose, sh.rec, out, 2 * seq + 1, stamps);
}
template <typename T, int RNG, int MAXM, typename SP>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(PFMPE_RESAMPLE_OWNERS_MIN_WAVES))) void
k_resample_owners(const FrameArgsT<T> fa, Ctrl* __restrict__ ctrl, const SP* __restrict__ prior,
                  const T* __restrict__ w0, const T* __restrict__ w1, const BlockScan* __restrict__ bscan0,
                  const BlockScan* __restrict__ bscan1, const GroupScan* __restrict__ gscan,
                  uint32_t* __restrict__ counts, double* __restrict__ mlpose, unsigned long long* __restrict__ winkey,
                  uint32_t* __restrict__ arrive, const unsigned char* __restrict__ table, RecOut* __restrict__ out,
                  int32_t seq, uint64_t* __restrict__ stamps) {
  __shared__ OwnersFinalLds<T> shw[kWaves];  // per wave (a wave never waits for another)
  OwnersFinalLds<T>& sh = shw[wave_id_u()];
  const uint32_t* fa_words = (const uint32_t*)__builtin_amdgcn_kernarg_segment_ptr();
  const int blk = (int)blockIdx.x * kWaves + wave_id_u();
  if (blk >= fa.nblk) return;
  const Ctrl c = *ctrl;
  if (!c.done || !c.accepted) {  // unfinished batch or the re-init branch (PE:707-719)
    if (blk == 0) owners_no_resample<T, RNG, MAXM, SP>(fa, fa_words, c, ctrl, prior, mlpose, out, seq, stamps, sh);
    return;
  }
  const __amdgpu_buffer_rsrc_t ors =
      __builtin_amdgcn_make_buffer_rsrc((void*)fa.owner_out, (short)0, fa.N * 4, 0x00020000);
  double carry_R = __longlong_as_double(0x7ff8dead00000000ll);  // a NaN no R equals bitwise: evaluate F(rin)
  int carry_hi = 0;
  unsigned long long key = 0ull;
  const bool finisher = blk == fa.nblk - 1;
  // the block's candidate into the sharded winner keys (resample_phase, MODE 0) and, drained with the wave's count
  // and most-likely stores, the arrival: both before the owner stores, which the finish does not read
  resample_owners_block<T, RNG, SP>(fa, fa_words, blk, c, prior, c.kept_slot ? w1 : w0, ors,
                                    c.kept_slot ? bscan1 : bscan0, gscan, counts, mlpose, sh.o, carry_R, carry_hi,
                                    key, [&](unsigned long long k) {
                                      if (k && lane_id() == 0)
                                        __hip_atomic_fetch_max(winkey + (blk & (kWinShards - 1)) * kWinStride, k,
                                                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                                      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                                      if (!finisher && lane_id() == 0)
                                        (void)__hip_atomic_fetch_add(arrive + (blk & (kWinShards - 1)) * kArriveStride,
                                                                     1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                                    });
  if (!finisher) return;
  owners_finish<T, RNG, MAXM, SP>(fa, fa_words, c, ctrl, prior, table, mlpose, winkey, out, seq, stamps, sh);
}

// The batched form (pfmpe_step_multi, every stream deferred): wave i of the grid takes the batch's block i, its
// stream from the block map (batch_block's checks, per wave), and each stream is finished as one stream is
// (k_resample_owners' keys, arrival shards and finisher, on the stream's own key area): no k_resample_final_multi.
template <typename T, int RNG, int MAXM, typename SP>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(PFMPE_RESAMPLE_OWNERS_MIN_WAVES))) void
k_resample_owners_multi(const StreamDesc<T, SP>* __restrict__ descs, const uint16_t* __restrict__ bmap, int S,
                        const uint32_t* __restrict__ status, uint32_t gen, int total) {
  __shared__ OwnersFinalLds<T> shw[kWaves];  // per wave: the workgroup's waves may belong to different streams, each
                                              // staging its own stream's constants
  OwnersFinalLds<T>& sh = shw[wave_id_u()];
  const int gb = (int)blockIdx.x * kWaves + wave_id_u();
  if (gb >= total) return;
  const int s = __builtin_amdgcn_readfirstlane((int)bmap[gb]);
  if (s >= S || __builtin_amdgcn_readfirstlane(status[s]) != gen) return;
  const StreamDesc<T, SP>& d = descs[s];
  const int blk = gb - __builtin_amdgcn_readfirstlane(d.first_blk);
  if (blk < 0 || blk >= __builtin_amdgcn_readfirstlane(d.fa.nblk)) return;
  const Ctrl c = load_ctrl_uniform(d.ctrl);
  const uint32_t* fa_words = (const uint32_t*)&d.fa;
  if (!c.done || !c.accepted) {  // an unfinished stream (later rounds) or the re-init branch
    if (blk == 0) owners_no_resample<T, RNG, MAXM, SP>(d.fa, fa_words, c, d.ctrl, d.prior, d.mlpose, d.out, d.seq, nullptr, sh);
    return;
  }
  const __amdgpu_buffer_rsrc_t ors =
      __builtin_amdgcn_make_buffer_rsrc((void*)d.fa.owner_out, (short)0, d.fa.N * 4, 0x00020000);
  double carry_R = __longlong_as_double(0x7ff8dead00000000ll);
  int carry_hi = 0;
  unsigned long long key = 0ull;
  unsigned long long* winkey = d.winkey;
  const bool finisher = blk == __builtin_amdgcn_readfirstlane(d.fa.nblk) - 1;
  resample_owners_block<T, RNG, SP>(d.fa, fa_words, blk, c, d.prior, c.kept_slot ? d.w1 : d.w0, ors,
                                    c.kept_slot ? d.bscan1 : d.bscan0, d.gscan, d.counts, d.mlpose, sh.o, carry_R,
                                    carry_hi, key, [&](unsigned long long k) {
                                      if (k && lane_id() == 0)
                                        __hip_atomic_fetch_max(winkey + (blk & (kWinShards - 1)) * kWinStride, k,
                                                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                                      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                                      if (!finisher && lane_id() == 0)
                                        (void)__hip_atomic_fetch_add(
                                            win_arrive(winkey) + (blk & (kWinShards - 1)) * kArriveStride, 1u,
                                            __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                                    });
  if (!finisher) return;
  owners_finish<T, RNG, MAXM, SP>(d.fa, fa_words, c, d.ctrl, d.prior, d.table, d.mlpose, winkey, d.out, d.seq, nullptr,
                                  sh);
}

// ---- launch 3 of the two-launch path (one block): winner = argmax of the block count partials (first
// index, PE:685-686), its kept-iteration pose regenerated and paired once, then the frame record.  Also
// reports an unfinished frame (speculative launch) and the re-init branch (PE:707-719).
constexpr int kFinalBlock = 1024;
template <typename T, int RNG, int MAXM, typename SP, bool MULTI>
__device__ __forceinline__ void resample_final_block(
    const FrameArgsT<T>& fa, const uint32_t* fa_words, Ctrl* __restrict__ ctrl, const unsigned char* __restrict__ table,
    const SP* __restrict__ prior, const CountPart* __restrict__ cpart, Cand* __restrict__ cand,
    const double* __restrict__ mlpose, RecOut* __restrict__ out, int32_t seq, uint64_t* __restrict__ stamps,
    int regen, unsigned char* smem /* the blob table */, unsigned long long* __restrict__ winkey = nullptr) {
  __shared__ LdsConst<T> sc;
  __shared__ OutDev rec;
  __shared__ int sv[kFinalBlock / 64], si[kFinalBlock / 64];
  __shared__ uint32_t ccorr[2 * kMaxMarkers];
  __shared__ T mk[kMaxMarkers];
  __shared__ int rk[kMaxMarkers];
  static_assert(kMaxMarkers <= kFinalBlock / 64, "one wave per marker");
  const int lane = lane_id(), wv = (int)(threadIdx.x >> 6);
  if (stamps && threadIdx.x == 0) stamps[6] = rt_now();
  // nothing below depends on the control record until the reduction is done: the partial, table and
  // most-likely-pose loads go out together with it (on an unfinished frame they are simply unused)
  const Ctrl c = MULTI ? load_ctrl_uniform(ctrl) : *ctrl;
  double ml = 0.0;
  if (wv == 0 && lane < 12) ml = mlpose[lane];
  stage_consts_from(fa_words, sc);
  {
    const uint4* s4 = (const uint4*)table;
    uint4* d4 = (uint4*)smem;
    const int n4 = (int)(BlobTable<T>::bytes(fa.B) / 16);
    for (int q = (int)threadIdx.x; q < n4; q += kFinalBlock) d4[q] = s4[q];
  }
  int bv = -1, bi = 0x7fffffff;
  if (winkey) {
    // one-stream frame: the kWinShards winner keys k_resample's blocks maxed into (one round trip), each reset to
    // the identity by the thread that read it, for the next frame (the next k_resample is ordered after this
    // launch).  Key 0 decodes to count 0 at index 2^31 - 1, below every real candidate.
    static_assert(kWinShards <= kFinalBlock, "one key per thread");
    unsigned long long key = 0ull;
    if ((int)threadIdx.x < kWinShards) {
      key = winkey[threadIdx.x * kWinStride];
      winkey[threadIdx.x * kWinStride] = 0ull;
    }
    unsigned long long kmax = key;
    // max over the wave of the 64-bit keys (their halves through DPP would need two compares; lane reads are few)
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      const unsigned long long other = (unsigned long long)__shfl_xor((long long)kmax, o, 64);
      kmax = other > kmax ? other : kmax;
    }
    if (wv == 0 && kmax != 0ull) {
      bv = (int)(kmax >> 32);
      bi = 0x7fffffff - (int)(uint32_t)kmax;
    }
    if (lane == 0) {
      sv[wv] = bv;
      si[wv] = bi;
    }
  } else {
    // two partials per 16-B load, eight predicated loads in flight per thread (C4: 39k partials in about
    // three round trips); the buffer holds one spare partial for an odd count (pfmpe_create)
    const int nb = fa.nblk;
    const int n2 = (nb + 1) / 2;
    const u32x4_t* cp4 = (const u32x4_t*)cpart;
    for (int base = (int)threadIdx.x; base < n2; base += 8 * kFinalBlock) {
      u32x4_t p[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int i = base + u * kFinalBlock;
        const u32x4_t none = {0xffffffffu, 0x7fffffffu, 0xffffffffu, 0x7fffffffu};
        p[u] = i < n2 ? cp4[i] : none;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int i = base + u * kFinalBlock;
        cmb_max(bv, bi, (int)p[u].x, (int)p[u].y);
        if (2 * i + 1 < nb) cmb_max(bv, bi, (int)p[u].z, (int)p[u].w);
      }
    }
    wave_argmax(bv, bi);
    if (lane == 0) {
      sv[wv] = bv;
      si[wv] = bi;
    }
  }
  if (!c.done) {
    if (threadIdx.x == 0) st_sys64(&out->g[0], (uint64_t)(uint32_t)(2 * seq) << 32);
    return;
  }
  __syncthreads();  // partials, table and constants
  if (!c.accepted) {
    if (wv == 0)
      finalize_frame<T, RNG, MAXM, SP>(fa, sc, c, ctrl, prior, -1, cand, mlpose, rec, out, 2 * seq + 1, stamps);
    return;
  }
  // every wave: the winner (LDS broadcast) and its kept pose
  bv = sv[0];
  bi = si[0];
  for (int w = 1; w < kFinalBlock / 64; ++w) cmb_max(bv, bi, sv[w], si[w]);
  if (stamps && threadIdx.x == 0) stamps[24] = rt_now();
  const bool marker_wave = wv < fa.M || wv == 0;  // wave-uniform
  T Pc[12];
  T u0 = (T)0, v0 = (T)0;
  const LdsBlobs<T> tb = view_table<T>(smem, fa.B);
  if (marker_wave) {
  if (bv > 0 && !regen) {  // staged by the winner's k_resample block (regen: k_resample gathered stored
                           // state values, so the winner's pose is regenerated here)
    const T* row = (const T*)(cand + bi / kBlock);
#pragma unroll
    for (int q = 0; q < 12; ++q) Pc[q] = row[q];
  } else {  // regen, or every count is 0 (the winner is particle 0, PE:685, never propagated in k_resample)
    make_particle<T, RNG, SP>(fa, sc, prior, bi, c.kept_iter, Pc);
  }
  // wave j: marker j's nearest blob (pose_pairs' scan and tie rule, one marker per wave)
  project_one<T>(sc, Pc, wv, fa.k_upper != 0, u0, v0);
  T best = inf_t<T>();
  int arg = 0x7fffffff;
  for (int i = lane; i < fa.B; i += 64) {
    const BlobXY<T> p = tb.bxy[i];
    const int o = tb.orig[i];
    const T dx = p.x - u0;
    const T dy = p.y - v0;
    const T d = fmadd(dx, dx, dy * dy);
    if (d < best || (d == best && o < arg)) {
      best = d;
      arg = o;
    }
  }
  wave_argmin(best, arg);
  if (lane == 0) {
    mk[wv] = best;
    rk[wv] = arg == 0x7fffffff ? 0 : arg;
  }
  }
  if (stamps && threadIdx.x == 0) stamps[25] = rt_now();
  __syncthreads();  // the per-marker minima
  if (wv != 0) return;
  T m[MAXM];
  int r[MAXM];
#pragma unroll
  for (int j = 0; j < MAXM; ++j) {
    m[j] = marker_live<MAXM>(j, fa.M) ? mk[j] : inf_t<T>();
    r[j] = marker_live<MAXM>(j, fa.M) ? rk[j] : 0;
  }
  const int np = pairs_from_minima<T, MAXM>(fa, tb, m, r, u0, v0, ccorr);  // wave 0 projected marker 0
  const uint32_t pl = payload_word<T>(Pc, ccorr, np);
  if (stamps && lane == 0) stamps[26] = rt_now() + (uint64_t)(pl == 12345u ? 1 : 0);
  finalize_frame<T, RNG, MAXM, SP>(fa, sc, c, ctrl, prior, bi, cand, mlpose, rec, out, 2 * seq + 1, stamps, true, pl,
                                   ml);
  if (stamps && lane == 0) stamps[7] = rt_now();
}

template <typename T, int RNG, int MAXM, typename SP>
__global__ __launch_bounds__(kFinalBlock) void k_resample_final(
    const FrameArgsT<T> fa, Ctrl* __restrict__ ctrl, const unsigned char* __restrict__ table,
    const SP* __restrict__ prior, const CountPart* __restrict__ cpart, Cand* __restrict__ cand,
    const double* __restrict__ mlpose, RecOut* __restrict__ out, int32_t seq, uint64_t* __restrict__ stamps,
    int regen, unsigned long long* __restrict__ winkey) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  resample_final_block<T, RNG, MAXM, SP, false>(fa, (const uint32_t*)__builtin_amdgcn_kernarg_segment_ptr(), ctrl, table, prior,
                                         cpart, cand, mlpose, out, seq, stamps, regen, smem, winkey);
}
// batched: block s finishes stream s
template <typename T, int RNG, int MAXM, typename SP>
__global__ __launch_bounds__(kFinalBlock) void k_resample_final_multi(const StreamDesc<T, SP>* __restrict__ descs,
                                                                        const uint32_t* __restrict__ status,
                                                                        uint32_t gen) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  if (__builtin_amdgcn_readfirstlane(status[blockIdx.x]) != gen) return;  // descriptor failed the staging check
  const StreamDesc<T, SP>& d = descs[blockIdx.x];
  resample_final_block<T, RNG, MAXM, SP, true>(d.fa, (const uint32_t*)&d.fa, d.ctrl, d.table, d.prior, d.cpart, d.cand,
                                         d.mlpose, d.out, d.seq, nullptr, d.prop0 ? 1 : 0, smem);
}

// ---- the whole frame in ONE cooperative launch (every block co-resident, checked by the host): the
// PF iterations, the normalisation hand-off and the resampling.  Between the weighing pass and its
// outcome every block waits for the top wave's release of `gen`; the particle's prior, propagated pose
// and weight stay in registers across the wait, so nothing is re-read or regenerated (unless the kept
// iteration is an earlier one).  A wait longer than ~2 s abandons the frame (no record: host error).
struct FrameLds {
  Ctrl c;
  BlockScan bs[2];  // this block's scan words, both weight slots
  GroupScan gs;
  int abort;
};

template <typename T, int RNG, int MAXM, bool PRUNE, typename SP>
__global__ __launch_bounds__(kBlock) void k_frame(
    const FrameArgsT<T> fa, const unsigned char* __restrict__ table, const SP* __restrict__ prior,
    SP* __restrict__ post, T* __restrict__ w0, T* __restrict__ w1, BlockPart* __restrict__ part0,
    BlockPart* __restrict__ part1, BlockScan* __restrict__ bscan0, BlockScan* __restrict__ bscan1,
    GroupPart* __restrict__ gpart0, GroupPart* __restrict__ gpart1, GroupScan* __restrict__ gscan,
    Ctrl* __restrict__ ctrl, CountPart* __restrict__ cpart, CountPart* __restrict__ cgroup,
    uint32_t* __restrict__ gcount_w, uint32_t* __restrict__ tcount_w, uint32_t* __restrict__ gcount_r,
    uint32_t* __restrict__ tcount_r, uint32_t* __restrict__ gen, uint32_t* __restrict__ counts,
    Cand* __restrict__ cand, double* __restrict__ mlpose,
    RecOut* __restrict__ out, int32_t seq, uint64_t* __restrict__ stamps, uint32_t* __restrict__ flat) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ LdsConst<T> sc;
  __shared__ WeighLds wsh;
  __shared__ ResampleLds<T> rsh;
  __shared__ OutDev rec;
  __shared__ FrameLds fsh;

  if (stamps && threadIdx.x == 0) stamp_min(stamps, 0, rt_now());
  const int n = blockIdx.x * kBlock + threadIdx.x;
  const bool valid = n < fa.N;
  const int lane = lane_id(), wv = wave_id();
  const int blk = blockIdx.x, g = blk / fa.gsz;

  copy_table(table, smem, (size_t)fa.tbytes);
  T A[12];
  if (valid && n >= 2) load_prior(fa, prior, n, A);
  const uint32_t gen_base = ((uint32_t)seq & 0xffffu) << 16;  // iteration release values of this frame
  Ctrl c = load_ctrl_wt(ctrl);  // the all-zero start-of-frame record (previous launch)
  stage_consts(fa, sc);
  __syncthreads();
  const LdsBlobs<T> tb = view_table<T>(smem, fa.B);
  if (stamps && threadIdx.x == 0) {
    const uint64_t t = rt_now();
    stamp_max(stamps, 8, t);
    stamp_min(stamps, 19, t);
  }

  T P[12], w = (T)0;
  int iter = 0;
  for (;; ++iter) {
    const int slot = c.cur_slot;
    if (valid) {
      w = weigh_particle<T, RNG, MAXM, PRUNE>(fa, sc, tb, A, n, iter, P);
      (slot ? w1 : w0)[n] = w;
    }
    if (stamps && threadIdx.x == 0) stamp_max(stamps, 9, rt_now());
    publish_iteration<T, RNG>(fa, w, valid, n, slot, iter, wsh, part0, part1, bscan0, bscan1, gpart0, gpart1, gscan,
                              ctrl, gcount_w, tcount_w, gen, gen_base, stamps, blk);
    // wait for this iteration's outcome
    if (wv == 0) {
      int ab = 0;
      if (lane == 0) {
        const uint32_t want = gen_base + (uint32_t)iter + 1u;
        const uint64_t t0 = rt_now();
        while (__hip_atomic_load((gu32_t*)gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != want) {
          __builtin_amdgcn_s_sleep(2);
          if (rt_now() - t0 > fa.wait_ticks) {  // PFMPE_OPT_WAIT_BOUND_US (default 2 s)
            ab = 1;
            break;
          }
        }
      }
      ab = lane_value(ab, 0);
      if (!ab) {
        // one round trip: the control record's words, this block's scan words (both slots) and its
        // group's (the scan words are meaningful once the frame is done)
        constexpr int kCw = (int)(sizeof(Ctrl) / 8);
        static_assert(sizeof(Ctrl) % 8 == 0 && kCw + 8 <= 64, "Ctrl words");
        const uint64_t* src = nullptr;
        uint64_t* dst = nullptr;
        if (lane < kCw) {
          src = (const uint64_t*)ctrl + lane;
          dst = (uint64_t*)&fsh.c + lane;
        } else if (lane < kCw + 6) {
          const int sl = (lane - kCw) / 3, q = (lane - kCw) % 3;
          src = (const uint64_t*)((sl ? bscan1 : bscan0) + blk) + q;
          dst = (uint64_t*)&fsh.bs[sl] + q;
        } else if (lane < kCw + 8) {
          src = (const uint64_t*)(gscan + g) + (lane - kCw - 6);
          dst = (uint64_t*)&fsh.gs + (lane - kCw - 6);
        }
        if (src) *dst = ld_wt(src);
      }
      if (lane == 0) fsh.abort = ab;
    }
    __syncthreads();
    if (fsh.abort) return;
    c = fsh.c;
    if (c.done) break;
  }

  if (!c.accepted) {  // re-init branch (PE:707-719): no resampling, record only
    if (blk == 0 && wv == 0)
      finalize_frame<T, RNG, MAXM, SP>(fa, sc, c, ctrl, prior, -1, cand, mlpose, rec, out, 2 * seq + 1, stamps);
    return;
  }
  const int kslot = c.kept_slot;
  const bool have_P = c.kept_iter == iter;
  double wd = 0.0;
  if (valid) {
    if (have_P) {
      wd = (double)w;
    } else {  // the kept iteration is an earlier one: its weight is in the other slot (own write)
      wd = (double)(kslot ? w1 : w0)[n];  // this thread's own earlier store
    }
  }
  const BlockScan bs = fsh.bs[kslot];
  const GroupScan gs = fsh.gs;
  if (flat)  // the count barrier flat (block 0 waits for every arrival), the weighing barrier a tree
    resample_phase<T, RNG, MAXM, SP, 2>(fa, sc, c, ctrl, table, prior, post, wd, A, P, have_P, bs, gs, rsh, rec, tb, cand,
                                        mlpose, cpart, cgroup, gcount_r, tcount_r, counts, out, seq, stamps, flat, blk);
  else
    resample_phase<T, RNG, MAXM, SP, 1>(fa, sc, c, ctrl, table, prior, post, wd, A, P, have_P, bs, gs, rsh, rec, tb, cand,
                                        mlpose, cpart, cgroup, gcount_r, tcount_r, counts, out, seq, stamps, nullptr,
                                        blk);
}

// ---- the whole frame in ONE launch with FLAT hand-offs (k_frame2; <= 512 co-resident blocks, groups of 64).
// Weighing barrier: every block stores its partial write-through and makes one arrival on the sharded
// weighing counters; every block then waits for all arrivals, loads ALL block partials (one round trip)
// and reduces them itself with exactly the group / top arithmetic of the tree path (propagate_group with
// one tile, propagate_top's one-tile branch), so no top wave, release word or control-record round trip
// sits between the weighing pass and the resampling.  Count barrier: one arrival per block; block 0 waits
// and writes the frame record.  Every wait is bounded (~2 s): an abandoned frame has no record and the
// host redoes it with two launches.
struct WaveArg {
  double maxw, minw;
  int argmax, argmin;
};
struct Frame2Lds {
  GroupPart gp[2][kFlatMaxGroups];  // group partials per weight slot (sum, zmax, zmin; latest iteration)
  WaveArg wa[2][kWaves];            // per weight slot: each wave's max / argmax, min / argmin over its blocks
  BlockScan bs[2];                  // this block's in-group scan words per slot
  int dirty[kWaves];                // group_math2: a wave's blocks may hold a negative or NaN weight
  GroupScan gs;                     // this block's group prefix / running max (kept slot)
  Ctrl c;
  int abort;
};

// propagate_group's sum / running-extrema arithmetic for one-tile groups (gsz = 64), TWO groups per wave
// (the thread's blocks t and t + 256), their chains interleaved; the lane holding block `mine` also
// returns its scan words.  The max / argmax and min / argmin go straight over the wave's blocks (wa):
// the lexicographic (value, index) extremum is exact in any order, so the top combines the four waves'
// results into exactly the group-then-top answer (a block whose max is NaN drops out either way).
struct BlockIn {
  bool vb, mine;
  BlockPart p;
};
// The min side (min / argmin, and the zmin running-min scans) only matters when the kept iteration's S < 0, i.e.
// with a negative weight, and the NaN test below (S = NaN reaches the zin_min select of the resampling).  Two
// shortcuts, each exact:
//  - argmin chain: an fp32 wave with no negative weight leaves its min side as the pair (+inf, 0x7fffffff)
//    (wave_weight_partials), and so does every block built from such waves; when every block of this wave holds
//    that pair, the chain's result is that pair, so it is not run (wave-uniform test);
//  - zmin scans: left to group_zmin2, which frame2_body runs only when some block of the iteration (any wave: the
//    test is made block-wide after the next barrier) holds a negative minimum or a NaN sum.  Otherwise every weight
//    is >= 0 and none is NaN, so S >= 0, and no consumer reads zmin / zin_min (top_math_regs' cm takes zmax when
//    S > 0 and skips S == 0; a frame with S == 0 is not accepted, so it is not resampled).
// group_math2 returns whether this wave's blocks fail that test, and leaves the zmin scans' inputs in zmin_in.
__device__ __forceinline__ bool group_math2(const BlockIn (&in)[2], GroupPart (&out)[2], BlockScan* own, WaveArg& wa,
                                            double (&zmin_in)[2]) {
  double sum[2], maxrel[2], minrel[2];
  double maxw = -INFINITY, minw = INFINITY;
  int amax = 0x7fffffff, amin = 0x7fffffff;
  bool min_placeholder = true, dirty = false;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const bool vb = in[k].vb;
    if (vb) {
      cmb_max(maxw, amax, in[k].p.maxw, in[k].p.argmax);
      cmb_min(minw, amin, in[k].p.minw, in[k].p.argmin);
    }
    min_placeholder &= !vb || (in[k].p.minw == (double)INFINITY && in[k].p.argmin == 0x7fffffff);
    dirty |= vb && !(in[k].p.minw >= 0.0 && in[k].p.sum == in[k].p.sum);
    sum[k] = vb ? in[k].p.sum : 0.0;
    maxrel[k] = vb ? in[k].p.maxrel : -INFINITY;
    minrel[k] = vb ? in[k].p.minrel : INFINITY;
  }
  double incl[2] = {sum[0], sum[1]};
  if (__builtin_amdgcn_ballot_w64(!min_placeholder) == 0) {
    scan_steps([&](auto st) {
      using S = decltype(st);
      st_sum<S>(incl[0]);
      st_sum<S>(incl[1]);
      st_argmax<S>(maxw, amax);
    });
    minw = INFINITY;  // the argmin chain over inputs that are all this pair
    amin = 0x7fffffff;
  } else {
    scan_steps([&](auto st) {
      using S = decltype(st);
      st_sum<S>(incl[0]);
      st_sum<S>(incl[1]);
      st_argmax<S>(maxw, amax);
      st_argmin<S>(minw, amin);
    });
    bcast63(minw, amin);
  }
  double E[2], zi_max[2];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    E[k] = 0.0 + wave_shr1(incl[k], 0.0);
    zi_max[k] = in[k].vb ? E[k] + maxrel[k] : -INFINITY;
    zmin_in[k] = in[k].vb ? E[k] + minrel[k] : INFINITY;
  }
  scan_steps([&](auto st) {
    using S = decltype(st);
    st_max<S>(zi_max[0]);
    st_max<S>(zi_max[1]);
  });
  bcast63(maxw, amax);
  wa.maxw = maxw;
  wa.minw = minw;
  wa.argmax = amax;
  wa.argmin = amin;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    double zp_max = wave_shr1(zi_max[k], -(double)INFINITY);
    zp_max = zp_max > -INFINITY ? zp_max : -INFINITY;
    if (in[k].vb && in[k].mine) {
      own->E = E[k];
      own->zin_max = zp_max;
      own->zin_min = INFINITY;  // group_zmin2, when needed
      own->pad = 0.0;
    }
    const double tmax = lane_value(zi_max[k], 63);
    GroupPart& r = out[k];
    r.sum = 0.0 + lane_value(incl[k], 63);
    r.zmax = tmax > -INFINITY ? tmax : -INFINITY;
    r.zmin = INFINITY;   // group_zmin2, when needed
    r.maxw = -INFINITY;  // unused on this path (wa)
    r.minw = INFINITY;
    r.argmax = r.argmin = 0x7fffffff;
  }
  return __builtin_amdgcn_ballot_w64(dirty) != 0;
}
// the zmin running-min scans of group_math2's two groups (propagate_group's arithmetic): the block's own zin_min and
// the groups' zmin, into the LDS words group_math2 left as placeholders
__device__ __forceinline__ void group_zmin2(const BlockIn (&in)[2], double (&zi_min)[2], BlockScan* own, GroupPart* gp0,
                                            GroupPart* gp1) {
  scan_steps([&](auto st) {
    using S = decltype(st);
    st_min<S>(zi_min[0]);
    st_min<S>(zi_min[1]);
  });
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    double zp_min = wave_shr1(zi_min[k], (double)INFINITY);
    zp_min = zp_min < INFINITY ? zp_min : INFINITY;
    if (in[k].vb && in[k].mine) own->zin_min = zp_min;
    const double tmin = lane_value(zi_min[k], 63);
    GroupPart* g = k ? gp1 : gp0;
    if (g && lane_id() == 0) g->zmin = tmin < INFINITY ? tmin : INFINITY;
  }
}

// The 64-lane inclusive sum scan's value on lanes 0-7 when lanes 8-63 hold +0.0: the three in-row steps
// (the same association), then the one "+ 0.0" the identity steps leave (it only turns -0.0 into +0.0).
// wave_incl_sum's lane 63 is then 0.0 + this scan's lane 7.
__device__ __forceinline__ double lanes8_incl_sum(double x) {
  x = x + dpp<kDppRowShr1>(x, 0.0);
  x = x + dpp<kDppRowShr2>(x, 0.0);
  x = x + dpp<kDppRowShr4>(x, 0.0);
  return x + 0.0;
}

// propagate_top's one-tile arithmetic (<= 64 groups), partials in registers: q0 = this iteration's partial
// of the lane's group, qk(slot) = the partial of the lane's group in weight slot `slot` (for the kept
// slot).  Returns the new control record (wave-uniform) and the lane's group G / Gin when done.
template <typename T, int RNG, typename KeptF, typename ArgF>
__device__ __forceinline__ Ctrl top_math_regs(const FrameArgsT<T>& fa, Ctrl c, int iter, int slot, const GroupPart& q0,
                                              KeptF qk, ArgF garg, double* G_out, double* Gin_out) {
  const int lane = lane_id();
  const int ngrp = fa.ngrp;
  // the kept-slot sum chain, speculatively for kept slot == this slot (the kept iteration is an earlier
  // one only when that one holds the best weight); ngrp <= 8, so the 8-lane form of the scan
  double incl = lanes8_incl_sum(lane < ngrp ? q0.sum : 0.0);
  double mv, mn_;
  int mi, ni_;
  garg(slot, mv, mi, mn_, ni_);
  if (mv > c.best_max) {  // strict: PE:608
    c.best_max = mv;
    c.best_idx = mi;
    c.best_iter = iter;
    c.best_slot = slot;
    c.has_best = 1;
  }
  c.iters = iter + 1;
  const bool go_on = fa.force_iters > 0 ? (c.iters < fa.force_iters) : (c.iters < fa.max_iter && mv < fa.exit_thr);
  c.cur_slot = c.has_best ? 1 - c.best_slot : 1 - slot;
  if (!go_on) {
    c.done = 1;
    c.kept_slot = c.has_best ? c.best_slot : slot;
    c.kept_iter = c.has_best ? c.best_iter : iter;
    GroupPart kq = q0;
    double amv = mv, anv = mn_;
    int ami = mi, ani = ni_;
    if (c.kept_slot != slot) {  // the speculation missed: the kept slot's chain
      kq = qk(c.kept_slot);
      incl = lanes8_incl_sum(lane < ngrp ? kq.sum : 0.0);
      garg(c.kept_slot, amv, ami, anv, ani);
    }
    const double S = 0.0 + lane_value(incl, 7);
    double run = -INFINITY;
    {
      const double prev = wave_shr1(incl, 0.0);
      const double G = lane == 0 ? 0.0 : 0.0 + prev;
      double cm = -INFINITY;
      if (lane < ngrp && S != 0.0) cm = (G + (S > 0.0 ? kq.zmax : kq.zmin)) / S;
      const double im = wave_incl_max(cm);
      double ex = wave_shr1(im, -(double)INFINITY);
      ex = ex > run ? ex : run;
      *G_out = G;
      *Gin_out = ex;
      const double tm = lane_value(im, 63);
      run = tm > run ? tm : run;
    }
    if (S == 0.0) run = -INFINITY;
    const double highest = c.has_best ? c.best_max : 0.0;
    c.S = S;
    c.invS = 1.0 / S;
    c.accepted = (S != 0.0 && highest > fa.accept_thr) ? 1 : 0;  // PE:633
    if (c.accepted) {
      c.most_likely_idx = c.best_idx;
      int64_t kt = lane == 0 ? count_targets<T, RNG>(fa, c.iters, run) : 0;
      c.K_total = (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)kt, 0)) |
                            ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)kt >> 32), 0) << 32));
    } else {
      c.most_likely_idx = (S < 0.0) ? ani : ami;
      c.K_total = 0;
    }
  }
  return c;
}

// The flat frame is one launch only while 2 blocks fit per CU next to the occupancy margin (pfmpe_ctx.hpp
// frame_fused), i.e. 3 waves per SIMD (<= 168 VGPRs).  Without the cap fp64 took 214 VGPRs and fp32 187 once the
// granule polls kept 12 16-B loads per lane in flight (both would silently fall back to two launches above 256
// blocks); with it fp32 fits without scratch.
#ifndef PFMPE_FRAME2_MIN_WAVES
#define PFMPE_FRAME2_MIN_WAVES 3
#endif
// The LDS of a k_frame2 block
template <typename T>
struct Frame2Shared {
  LdsConst<T> sc;
  WeighLds wsh;
  ResampleLds<T> rsh;
  OutDev rec;
  Frame2Lds fl;
};
// One frame of k_frame2 for this block.  fa_words: the frame arguments as words (the kernarg segment) for the LDS
// constants.  Returns false when the block gave up at the weighing barrier's bound (an abandoned frame: no record).
template <typename T, int RNG, int MAXM, bool PRUNE, typename SP>
__device__ __forceinline__ bool frame2_body(
    const FrameArgsT<T>& fa, const uint32_t* fa_words, const unsigned char* __restrict__ table,
    const SP* __restrict__ prior, SP* __restrict__ post, T* __restrict__ w0, T* __restrict__ w1,
    BlockPart* __restrict__ part0, BlockPart* __restrict__ part1, Ctrl* __restrict__ ctrl,
    CountPart* __restrict__ cpart, uint32_t* __restrict__ flat, uint32_t* __restrict__ counts, Cand* __restrict__ cand,
    double* __restrict__ mlpose, RecOut* __restrict__ out, int32_t seq, uint64_t* __restrict__ stamps,
    unsigned char* smem, Frame2Shared<T>& S2) {
  LdsConst<T>& sc = S2.sc;
  WeighLds& wsh = S2.wsh;
  ResampleLds<T>& rsh = S2.rsh;
  OutDev& rec = S2.rec;
  Frame2Lds& fl = S2.fl;
  if (stamps && threadIdx.x == 0) stamp_min(stamps, 0, rt_now());
  const int n = blockIdx.x * kBlock + threadIdx.x;
  const bool valid = n < fa.N;
  const int lane = lane_id(), wv = wave_id();
  const int blk = blockIdx.x, g_own = blk / fa.gsz;

  // the prior's loads first: in flight together with the table's, one memory round trip before the weighing
  // instead of two (the table's wait would otherwise come before the prior loads were even issued)
  T A[12];
  if (valid && n >= 2) load_prior(fa, prior, n, A);
  stage_table_consts(table, smem, (size_t)fa.tbytes, fa_words, sc);
  if (threadIdx.x == 0) {
    fl.c = zero_ctrl();  // start of frame: every block keeps an identical copy of the control record
    fl.abort = 0;
  }
  __syncthreads();
  const LdsBlobs<T> tb = view_table<T>(smem, fa.B);
  if (stamps && threadIdx.x == 0) {
    const uint64_t t = rt_now();
    stamp_max(stamps, 8, t);
    stamp_min(stamps, 19, t);
  }

  T P[12], w = (T)0;
  Ctrl c = fl.c;
  int iter = 0;
  for (;; ++iter) {
    const int slot = c.cur_slot;
    if (valid) {
      w = weigh_particle<T, RNG, MAXM, PRUNE, true>(fa, sc, tb, A, n, iter, P, nullptr, stamps);
      (slot ? w1 : w0)[n] = w;
    }
    if (stamps && threadIdx.x == 0) stamp_max(stamps, 9, rt_now());
    // block partial (publish_iteration's block level), one arrival
    {
      double wi, rmx, rmn;
      T mx, mn;
      int ix, in_;
      wave_weight_partials(w, valid, n, wi, rmx, rmn, mx, ix, mn, in_);
      if (lane == 63) wsh.tot[wv] = wi;
      if (lane == 0) {
        wsh.rmax[wv] = rmx;
        wsh.rmin[wv] = rmn;
        wsh.mx[wv] = (double)mx;
        wsh.mn[wv] = (double)mn;
        wsh.ix[wv] = ix;
        wsh.in_[wv] = in_;
      }
      __syncthreads();
      if (wv == 0) {
        if (lane == 0) {
          double pre = 0.0, maxrel = -INFINITY, minrel = INFINITY, bmx = wsh.mx[0], bmn = wsh.mn[0];
          int bix = wsh.ix[0], bin = wsh.in_[0];
#pragma unroll
          for (int ww = 0; ww < kWaves; ++ww) {
            const double a = pre + wsh.rmax[ww], b = pre + wsh.rmin[ww];
            maxrel = a > maxrel ? a : maxrel;
            minrel = b < minrel ? b : minrel;
            if (ww) {
              cmb_max(bmx, bix, wsh.mx[ww], wsh.ix[ww]);
              cmb_min(bmn, bin, wsh.mn[ww], wsh.in_[ww]);
            }
            pre = pre + wsh.tot[ww];
          }
          // the partial buffer alternates by ITERATION parity, not by weight slot: an iteration that does
          // not improve the best weight reuses its slot, and a fast block would then overwrite its partial
          // while a lagging block still loads the previous iteration's.  Parity is safe: a block stores
          // iteration i+2's partial (same buffer as i) only after passing iteration i+1's barrier, i.e.
          // after every block has arrived at i+1, and each block arrives at i+1 only after its iteration-i
          // loads (wait_parts) have completed.  The per-slot results the frame keeps (group partials,
          // wave extrema, own scan words) live in LDS.
          BlockPart* bp = ((iter & 1) ? part1 : part0) + blk;
          st_wt_d(&bp->sum, pre);
          st_wt_d(&bp->maxrel, maxrel);
          st_wt_d(&bp->minrel, minrel);
          st_wt_d(&bp->maxw, bmx);
          st_wt_d(&bp->minw, bmn);
          st_wt(&bp->argmax, pack2(bix, bin));
          if (stamps) stamp_max(stamps, 1, rt_now());
          flat_arrive(flat, blk);
        }
        const uint32_t target = fa.flat_base_w + (uint32_t)(iter + 1) * (uint32_t)fa.nblk;
        // kDiagAbandon: behave as if the wait bound expired (the host's recovery path under test)
        const bool ok = !(fa.diag & kDiagAbandon) && flat_wait(flat, target, fa.wait_ticks);
        if (lane == 0 && !ok) fl.abort = 1;
      }
      __syncthreads();
      if (fl.abort) return false;
    }
    if (stamps && threadIdx.x == 0) stamp_max(stamps, 2, rt_now());
    // every block: the group partials from all block partials, then the top.  Groups are 64 blocks, so
    // thread t owns blocks t and t + 256 and wave w reduces groups w and w + 4; all six 16-B loads of the
    // thread are in flight together (one round trip)
    BlockIn in[2];
    double zmin_in[2];
    {
      const BlockPart* pp = (iter & 1) ? part1 : part0;  // iteration parity (see the store above)
      if ((fa.diag & kDiagLagLoads) && blk == fa.nblk - 1) {  // a lagging reader (the race test)
        const uint64_t t0 = rt_now();
        while (rt_now() - t0 < 2000u) __builtin_amdgcn_s_sleep(2);  // ~20 us
      }
      const int b0 = threadIdx.x, b1 = threadIdx.x + kBlock;
      const bool v0 = b0 < fa.nblk, v1 = b1 < fa.nblk;
      PartRaw r0, r1;
      ld_part_issue(pp + (v0 ? b0 : 0), r0);
      ld_part_issue(pp + (v1 ? b1 : 0), r1);
      wait_parts(r0, r1);
      if (stamps && threadIdx.x == 0) stamp_max(stamps, 24, rt_now());
      in[0].vb = v0;
      in[0].mine = b0 == blk;
      in[0].p = unpack_part(r0);
      in[1].vb = v1;
      in[1].mine = b1 == blk;
      in[1].p = unpack_part(r1);
      GroupPart gp[2];
      WaveArg wa;
      const bool dirty = group_math2(in, gp, &fl.bs[slot], wa, zmin_in);
      if (lane == 0) fl.wa[slot][wv] = wa;
      if (lane == 0 && wv < fa.ngrp) fl.gp[slot][wv] = gp[0];
      if (lane == 0 && wv + kWaves < fa.ngrp) fl.gp[slot][wv + kWaves] = gp[1];
      if (lane == 0) fl.dirty[wv] = dirty;
    }
    if (stamps && threadIdx.x == 0) stamp_max(stamps, 25, rt_now());
    __syncthreads();
    // the zmin scans only when some block of the iteration may hold a negative or NaN weight (group_math2's note);
    // every block reads the same partials, so every block takes the same branch
    int dirty = 0;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) dirty |= fl.dirty[w];
    if (dirty || (fa.diag & kDiagMinSide)) {
      group_zmin2(in, zmin_in, &fl.bs[slot], wv < fa.ngrp ? &fl.gp[slot][wv] : nullptr,
                  wv + kWaves < fa.ngrp ? &fl.gp[slot][wv + kWaves] : nullptr);
      __syncthreads();
    }
    if (wv == 0) {
      // field-wise LDS reads (an aggregate copy of the conditional struct went through scratch)
      auto qk = [&](int ks) {
        const bool v = lane < fa.ngrp;
        const GroupPart& src = fl.gp[ks][v ? lane : 0];
        GroupPart q;
        q.sum = v ? src.sum : 0.0;
        q.zmax = v ? src.zmax : -INFINITY;
        q.zmin = v ? src.zmin : INFINITY;
        q.maxw = v ? src.maxw : -INFINITY;
        q.minw = v ? src.minw : INFINITY;
        q.argmax = v ? src.argmax : 0x7fffffff;
        q.argmin = v ? src.argmin : 0x7fffffff;
        return q;
      };
      const GroupPart q0 = qk(slot);
      // the slot's max / argmax, min / argmin: the four waves' results combined (wave-uniform LDS reads)
      auto garg = [&](int ks, double& mxv, int& mxi, double& mnv, int& mni) {
        mxv = fl.wa[ks][0].maxw;
        mxi = fl.wa[ks][0].argmax;
        mnv = fl.wa[ks][0].minw;
        mni = fl.wa[ks][0].argmin;
#pragma unroll
        for (int w = 1; w < kWaves; ++w) {
          cmb_max(mxv, mxi, fl.wa[ks][w].maxw, fl.wa[ks][w].argmax);
          cmb_min(mnv, mni, fl.wa[ks][w].minw, fl.wa[ks][w].argmin);
        }
      };
      double G = 0.0, Gin = -INFINITY;
      const Ctrl cn = top_math_regs<T, RNG>(fa, c, iter, slot, q0, qk, garg, &G, &Gin);
      if (lane == g_own) {
        fl.gs.G = G;
        fl.gs.Gin = Gin;
      }
      if (lane == 0) fl.c = cn;
      if (stamps && lane == 0) stamp_max(stamps, 26, rt_now());
    }
    __syncthreads();
    c = fl.c;
    if (stamps && threadIdx.x == 0) stamp_max(stamps, 3, rt_now());
    if (c.done) break;
  }

  if (!c.accepted) {  // re-init branch (PE:707-719): no resampling, record only
    if (blk == 0 && wv == 0)
      finalize_frame<T, RNG, MAXM, SP>(fa, sc, c, ctrl, prior, -1, cand, mlpose, rec, out, 2 * seq + 1, stamps);
    return true;
  }
  const int kslot = c.kept_slot;
  const bool have_P = c.kept_iter == iter;
  double wd = 0.0;
  if (valid) wd = have_P ? (double)w : (double)(kslot ? w1 : w0)[n];
  const BlockScan bs = fl.bs[kslot];
  const GroupScan gs = fl.gs;
  resample_phase<T, RNG, MAXM, SP, 2>(fa, sc, c, ctrl, table, prior, post, wd, A, P, have_P, bs, gs, rsh, rec,
                                                 tb, cand, mlpose, cpart, nullptr, nullptr, nullptr, counts, out, seq,
                                                 stamps, flat, blk);
  return true;
}

template <typename T, int RNG, int MAXM, bool PRUNE, typename SP>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(PFMPE_FRAME2_MIN_WAVES))) void k_frame2(
    const FrameArgsT<T> fa, const unsigned char* __restrict__ table, const SP* __restrict__ prior,
    SP* __restrict__ post, T* __restrict__ w0, T* __restrict__ w1, BlockPart* __restrict__ part0,
    BlockPart* __restrict__ part1, Ctrl* __restrict__ ctrl, CountPart* __restrict__ cpart,
    uint32_t* __restrict__ flat, uint32_t* __restrict__ counts, Cand* __restrict__ cand,
    double* __restrict__ mlpose, RecOut* __restrict__ out, int32_t seq, uint64_t* __restrict__ stamps) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ Frame2Shared<T> S2;
  (void)frame2_body<T, RNG, MAXM, PRUNE, SP>(fa, (const uint32_t*)__builtin_amdgcn_kernarg_segment_ptr(), table, prior,
                                             post, w0, w1, part0, part1, ctrl, cpart, flat, counts, cand, mlpose, out,
                                             seq, stamps, smem, S2);
}

// ---- state import / export / regeneration (API helpers, not on the timed path).  anchor: the set's
// anchor pose (fp16 state), ignored for fp32 / fp64 planes.
template <typename T>
struct Pose12 {
  T v[12];
};
template <typename T, typename SP>
__global__ void k_import(const double* __restrict__ poses, SP* __restrict__ st, int N, int64_t ld,
                         const Pose12<T> anchor) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  for (int q = 0; q < 12; ++q)
    st[plane_index<SP>(q, n, ld)] = StateIO<T, SP>::store((T)poses[12 * (int64_t)n + q], anchor.v[q]);
}
template <typename T, typename SP>
__global__ void k_export(const SP* __restrict__ st, double* __restrict__ poses, int N, int64_t ld,
                         const Pose12<T> anchor, const uint32_t* __restrict__ owner) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  const int r = owner ? (int)owner[n] : n;  // a deferred prior: stored row owner[n]
  for (int q = 0; q < 12; ++q)
    poses[12 * (int64_t)n + q] = (double)StateIO<T, SP>::load(st[plane_index<SP>(q, r, ld)], anchor.v[q]);
}
template <typename T, int RNG, typename SP>
__global__ __launch_bounds__(kBlock) void k_regen(const FrameArgsT<T> fa, int kept_iter, const SP* __restrict__ prior,
                                                 double* __restrict__ poses) {
  __shared__ LdsConst<T> sc;
  stage_consts(fa, sc);
  __syncthreads();
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= fa.N) return;
  T P[12];
  make_particle<T, RNG, SP>(fa, sc, prior, n, kept_iter, P);
  for (int q = 0; q < 12; ++q) poses[12 * (int64_t)n + q] = (double)P[q];
}
// ---- ROI prediction (§8f next row 1): predictMarkerPositionsInImage (PE:1036-1053) projects every marker
// through camMoveInv * prior_j * predictionMatrix (Eigen left-to-right products) for all N particles of
// the current prior; LEDDetector::determineROI (led_detector.cpp:217-243) keeps x_min / y_min from +inf and
// x_max / y_max from 0 with strict comparisons (NaN positions never win).  fp64 throughout: the same
// arithmetic as the oracle, so the box is exact for every state type.  One partial per block, then one
// block reduces them.
struct RoiArgs {
  double cam[12], predm[12], K[9], markers[kMaxMarkers * 3], anchor[12];
  int32_t N, M;
  int64_t ld;
  const uint32_t* owner;  // a deferred prior's owner indices (FrameArgsT::owner), or null
};
template <typename T, typename SP>
__global__ __launch_bounds__(kBlock) void k_roi(const RoiArgs ra, const SP* __restrict__ prior,
                                               double* __restrict__ part) {
  __shared__ double sh[4][kWaves];
  const int n = blockIdx.x * kBlock + threadIdx.x;
  double xmin = INFINITY, xmax = 0.0, ymin = INFINITY, ymax = 0.0;
  if (n < ra.N) {
    double A[12], X[12], P[12];
    const int r = ra.owner ? (int)ra.owner[n] : n;
#pragma unroll
    for (int q = 0; q < 12; ++q)
      A[q] = (double)StateIO<T, SP>::load(prior[plane_index<SP>(q, r, ra.ld)], (T)ra.anchor[q]);
    compose(ra.cam, A, X);   // camMoveInv * newPoseEstimation[j]
    compose(X, ra.predm, P); // ... * predictionMatrix
    double Q[12];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        double s = ra.K[i * 3 + 0] * P[0 * 4 + j];
        s = s + ra.K[i * 3 + 1] * P[1 * 4 + j];
        s = s + ra.K[i * 3 + 2] * P[2 * 4 + j];
        Q[i * 4 + j] = s;
      }
    for (int m = 0; m < ra.M; ++m) {
      const double x = ra.markers[3 * m], y = ra.markers[3 * m + 1], z = ra.markers[3 * m + 2];
      double p[3];
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        double s = Q[i * 4 + 0] * x;
        s = s + Q[i * 4 + 1] * y;
        s = s + Q[i * 4 + 2] * z;
        p[i] = s + Q[i * 4 + 3];
      }
      const double u = p[0] / p[2], v = p[1] / p[2];
      if (u < xmin) xmin = u;
      if (u > xmax) xmax = u;
      if (v < ymin) ymin = v;
      if (v > ymax) ymax = v;
    }
  }
  xmin = wave_min(xmin);
  xmax = wave_max(xmax);
  ymin = wave_min(ymin);
  ymax = wave_max(ymax);
  const int lane = lane_id(), wv = wave_id();
  if (lane == 0) {
    sh[0][wv] = xmin;
    sh[1][wv] = xmax;
    sh[2][wv] = ymin;
    sh[3][wv] = ymax;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < kWaves; ++w) {
      xmin = sh[0][w] < xmin ? sh[0][w] : xmin;
      xmax = sh[1][w] > xmax ? sh[1][w] : xmax;
      ymin = sh[2][w] < ymin ? sh[2][w] : ymin;
      ymax = sh[3][w] > ymax ? sh[3][w] : ymax;
    }
    double* o = part + 4 * (size_t)blockIdx.x;
    o[0] = xmin;
    o[1] = xmax;
    o[2] = ymin;
    o[3] = ymax;
  }
}
template <typename T>  // (a template only for COMDAT linkage: the header is in several TUs)
__global__ __launch_bounds__(kBlock) void k_roi_final(const T* __restrict__ part, int nblk, T* __restrict__ out) {
  __shared__ double sh[4][kWaves];
  double xmin = INFINITY, xmax = 0.0, ymin = INFINITY, ymax = 0.0;
  for (int b = threadIdx.x; b < nblk; b += kBlock) {
    const double* o = part + 4 * (size_t)b;
    xmin = o[0] < xmin ? o[0] : xmin;
    xmax = o[1] > xmax ? o[1] : xmax;
    ymin = o[2] < ymin ? o[2] : ymin;
    ymax = o[3] > ymax ? o[3] : ymax;
  }
  xmin = wave_min(xmin);
  xmax = wave_max(xmax);
  ymin = wave_min(ymin);
  ymax = wave_max(ymax);
  if (lane_id() == 0) {
    sh[0][wave_id()] = xmin;
    sh[1][wave_id()] = xmax;
    sh[2][wave_id()] = ymin;
    sh[3][wave_id()] = ymax;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < kWaves; ++w) {
      xmin = sh[0][w] < xmin ? sh[0][w] : xmin;
      xmax = sh[1][w] > xmax ? sh[1][w] : xmax;
      ymin = sh[2][w] < ymin ? sh[2][w] : ymin;
      ymax = sh[3][w] > ymax ? sh[3][w] : ymax;
    }
    out[0] = xmin;
    out[1] = xmax;
    out[2] = ymin;
    out[3] = ymax;
  }
}

template <typename T>
__global__ void k_weights_export(const T* __restrict__ w, double* __restrict__ out, int N) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  out[n] = (double)w[n];
}

}  // namespace pfmpe

#include "pf_weigh_pk.hpp"
