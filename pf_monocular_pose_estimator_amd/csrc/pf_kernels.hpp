// pf_kernels.hpp — HIP kernels of the PF step for gfx950 (MI355X, CDNA4, wave64).
//
// One frame (reference PE:475-733) runs as:
//   k_prep            1 block : blob table (blobs sorted by x + x-bucket index) + control reset
//   k_propagate_weigh nblk    : per particle: motion model (PE:543-588) -> project M markers (PE:1017)
//                               -> likelihood (PE:2385) -> weight; per-block partials
//                               (sum / running-sum extrema / max / min of the weights)
//   k_iter_reduce     1 block : iteration max, best-iteration bookkeeping and exit rule (PE:606-616);
//                               on the last iteration: normaliser S, block prefixes, accept (PE:627-633)
//   (k_propagate_weigh, k_iter_reduce) repeat only if the exit rule is not met (rare in steady state)
//   k_resample        nblk    : stratified resampling (PE:666-682) as a parallel scan + target count
//                               + wave-cooperative scatter of regenerated particles into the new prior
//   k_final           1 block : winner = argmax resample count (PE:685-688), its pose + pairs
//
// Propagated particles are never written to HBM: they are regenerated from (prior[n], RNG counter)
// where needed (resample scatter, winner), so the HBM traffic per particle-update is the compulsory
// 3*S + 8 bytes (S = 48 B for fp32 SoA state; DESIGN.md "Roofline").
#pragma once
#include <hip/hip_runtime.h>
#include <float.h>
#include <math.h>
#include <stdint.h>

#include "pf_rng.hpp"

namespace pfmpe {

constexpr int kBlock = 256;            // particles per block (4 waves)
constexpr int kWaves = kBlock / 64;
constexpr int kMaxMarkers = 16;
constexpr int kMaxBlobs = 1024;
constexpr int kBuckets = 128;          // x-buckets of the blob table
constexpr int kReduceThreads = 1024;   // single-block reducer
constexpr int kPlanes = 12;            // r00 r01 r02 t0 r10 r11 r12 t1 r20 r21 r22 t2

enum : int { kRngReference = 0, kRngPhilox = 1 };

// ----------------------------------------------------------------------------- kernel arguments
// Passed by value (kernarg segment -> scalar loads).  Doubles are converted to T on use.
struct FrameArgs {
  double cur[12], pred[12], predm[12], cam[12];  // 3x4 row-major
  double markers[kMaxMarkers * 3];
  double K[9];
  double lo[6], hi[6];      // draw ranges: angX angY angZ tX tY tZ (already scaled by fac*)
  double growth;            // 0.025
  double tol, tol_pf;       // score normaliser / acceptance gate
  double exit_thr, accept_thr;
  uint32_t key0, key1, flo, fhi;  // philox key / frame counter
  uint32_t lcg_x0;                // reference engine state after seeding
  uint32_t downgrade;             // bit j: marker j downgraded
  int32_t N, M, B, it;            // particles, markers, blobs, it_since_initialized_
  int32_t cam_identity, max_iter, force_iters, nblk;
  int64_t ld;                     // SoA plane stride in elements
};

struct Ctrl {
  double best_max;   // highestProb
  double S;          // probPartSum of the kept iteration
  double Rmax;       // max running cumulative normalised weight
  int32_t done, has_best, best_idx, best_iter, best_slot, cur_slot;
  int32_t iters, kept_slot, kept_iter, accepted, most_likely_idx, pad0;
  int64_t K_total;   // number of stratified targets that find a particle
};

struct BlockPart {   // per propagate block, per weight slot
  double sum;        // sum of weights (fp64)
  double maxrel;     // max / min of the in-block inclusive prefix sums
  double minrel;
  double maxw, minw; // max / min weight
  int32_t argmax, argmin;
};

struct CountPart {
  int32_t maxcount, idx;
};

// device copy of the frame output (pfmpe_frame_out layout + done word)
struct OutDev {
  int32_t done, pad;
  int32_t iters, kept_iter, most_likely_idx, accepted, resampled, winner_idx, n_corr, flag_fail;
  double highest_prob, prob_sum;
  double winner_pose[12], most_likely_pose[12];
  uint32_t corr[2 * kMaxMarkers];
};

// blob table (written by k_prep, read into LDS by the propagate kernel)
template <typename T>
struct BlobTable {
  T bx[kMaxBlobs];       // sorted by (x, original index)
  T by[kMaxBlobs];
  int32_t orig[kMaxBlobs];
  int32_t bstart[kBuckets + 1];
  T xmin, inv_bw, b0x, b0y;  // bucket origin / inverse width, original blob 0
  T tolq;                    // conservative search half-width (>= tol_pf)
  int32_t B;
};

// ----------------------------------------------------------------------------- scalar helpers
__device__ __forceinline__ float fmadd(float a, float b, float c) { return __builtin_fmaf(a, b, c); }
// fp64: deliberately UNFUSED (TU built with -ffp-contract=off): a*b rounded, then +c rounded, the
// reference's x86-64 arithmetic.
__device__ __forceinline__ double fmadd(double a, double b, double c) { return a * b + c; }
__device__ __forceinline__ void sincos_t(float x, float* s, float* c) { sincosf(x, s, c); }
__device__ __forceinline__ void sincos_t(double x, double* s, double* c) {
  *s = sin(x);
  *c = cos(x);
}
__device__ __forceinline__ float sqrt_t(float x) { return sqrtf(x); }
__device__ __forceinline__ double sqrt_t(double x) { return sqrt(x); }
// perspective division: fp32 uses one reciprocal, fp64 the exact IEEE quotient (PE:1032)
__device__ __forceinline__ void persp(float p0, float p1, float p2, float* u, float* v) {
  const float r = 1.0f / p2;
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

template <typename T>
__device__ __forceinline__ void load12(const double* src, T* dst) {
#pragma unroll
  for (int q = 0; q < 12; ++q) dst[q] = (T)src[q];
}

// The motion model (PE:543-588) for particle n in PF iteration `iter`; P receives the 3x4 pose.
template <typename T, int RNG>
__device__ __forceinline__ void make_particle(const FrameArgs& fa, const T* __restrict__ prior, int n,
                                              int iter, T* P) {
  if (n == 0) {  // current_pose_ (PE:547)
    load12(fa.cur, P);
    return;
  }
  if (n == 1) {  // predicted_pose_ (PE:551)
    load12(fa.pred, P);
    return;
  }
  T A[12];
#pragma unroll
  for (int q = 0; q < 12; ++q) A[q] = prior[(int64_t)q * fa.ld + n];
  if (fa.it > 1) {
    if (!fa.cam_identity) {  // camMoveInv * prior (PE:556-558)
      T C[12], X[12];
      load12(fa.cam, C);
      compose(C, A, X);
#pragma unroll
      for (int q = 0; q < 12; ++q) A[q] = X[q];
    }
    if ((iter % 10) != 0) {  // ... * predictionMatrix (PE:556)
      T Pm[12], X[12];
      load12(fa.predm, Pm);
      compose(A, Pm, X);
#pragma unroll
      for (int q = 0; q < 12; ++q) A[q] = X[q];
    }
  }
  // draws in reference order: angX, angY, angZ, tX, tY, tZ (PE:563-587)
  const double gd = 1.0 + fa.growth * (double)(iter / 10);
  T d[6];
  if (RNG == kRngReference) {
    const uint64_t per_particle = 12u;
    const uint64_t before = per_particle * ((uint64_t)(fa.N - 2) * (uint64_t)iter + (uint64_t)(n - 2));
    uint32_t g = lcg_output(fa.lcg_x0, before + 1u);
#pragma unroll
    for (int q = 0; q < 6; ++q) {
      const uint32_t g1 = g;
      const uint32_t g2 = lcg_next(g1);
      g = lcg_next(g2);
      const double u = ref_canonical(g1, g2);
      d[q] = (T)(ref_uniform(u, fa.lo[q], fa.hi[q]) * gd);
    }
  } else {
    const U32x4 ra = philox4x32_10((uint32_t)n, (uint32_t)iter | (kTagMotionA << 24), fa.flo, fa.fhi,
                                   fa.key0, fa.key1);
    const U32x4 rb = philox4x32_10((uint32_t)n, (uint32_t)iter | (kTagMotionB << 24), fa.flo, fa.fhi,
                                   fa.key0, fa.key1);
    const uint32_t raw[6] = {ra.x, ra.y, ra.z, ra.w, rb.x, rb.y};
    const T g = (T)gd;
#pragma unroll
    for (int q = 0; q < 6; ++q) {
      const T lo = (T)fa.lo[q], hi = (T)fa.hi[q];
      const T u = (T)u24d(raw[q]);
      const T draw = u * (hi - lo) + lo;
      d[q] = draw * g;
    }
  }
  T sa, ca, sb, cb, sc, cc;
  sincos_t(d[0], &sa, &ca);
  sincos_t(d[1], &sb, &cb);
  sincos_t(d[2], &sc, &cc);
  // R = ((R_A * Rz(c)) * Ry(b)) * Rx(a)   (PE:582)
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const T a0 = A[i * 4 + 0], a1 = A[i * 4 + 1], a2 = A[i * 4 + 2];
    const T z0 = fmadd(a1, sc, a0 * cc);      // A*Rz col 0
    const T z1 = fmadd(a1, cc, a0 * (-sc));   // A*Rz col 1
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

// project2d (PE:1017-1034): p = (K34*T) * [X;1], u = p/p.z — full K, no distortion, no z>0 test
template <typename T, int MAXM>
__device__ __forceinline__ void project_markers(const FrameArgs& fa, const T* P, T* u, T* v) {
  T Q[12];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const T k0 = (T)fa.K[i * 3 + 0], k1 = (T)fa.K[i * 3 + 1], k2 = (T)fa.K[i * 3 + 2];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      T s = k0 * P[0 * 4 + j];
      s = fmadd(k1, P[1 * 4 + j], s);
      s = fmadd(k2, P[2 * 4 + j], s);
      Q[i * 4 + j] = s;
    }
  }
#pragma unroll
  for (int j = 0; j < MAXM; ++j) {
    if (j < fa.M) {
      const T X = (T)fa.markers[3 * j], Y = (T)fa.markers[3 * j + 1], Z = (T)fa.markers[3 * j + 2];
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

// x -> bucket index (monotone in x; identical formula for table build and queries)
template <typename T>
__device__ __forceinline__ int bucket_of(T x, T xmin, T inv_bw) {
  const T f = (x - xmin) * inv_bw;
  if (!(f >= (T)0)) return 0;
  if (f >= (T)(kBuckets - 1)) return kBuckets - 1;
  return (int)f;
}

// calculateEstimationProbability (PE:2385-2445) in its closed form: per marker the first-minimum blob
// (exact; candidates limited to the conservative x-window that contains every blob within tol_PF, so
// pruning never changes an accepted pair — DESIGN.md "Exact blob pruning"), then extraction in
// ascending (distance, marker) order = the order Eigen's minCoeff visits, with the same gate, score
// (tol, not tol_PF), self-occlusion and downgrade penalties.
template <typename T, int MAXM, bool PRUNE, bool PAIRS>
__device__ __forceinline__ T likelihood(const FrameArgs& fa, const T* u, const T* v, const T* bx,
                                        const T* by, const int32_t* orig, const int32_t* bstart,
                                        T xmin, T inv_bw, T b0x, T b0y, T tolq, uint32_t* pairs,
                                        int* npairs) {
  const int B = fa.B, M = fa.M;
  if (PAIRS) *npairs = 0;
  if (B == 0) return (T)0;
  {  // Eigen's visitor starts from coeff(0,0): a NaN there poisons the first minCoeff -> break
    const T dx = b0x - u[0], dy = b0y - v[0];
    const T d = dx * dx + dy * dy;
    if (d != d) return (T)0;
  }
  T m[MAXM];
  int r[MAXM];
#pragma unroll
  for (int j = 0; j < MAXM; ++j) {
    T best = inf_t<T>();
    int arg = 0x7fffffff;
    if (j < M) {
      int c0 = 0, c1 = B;
      if (PRUNE) {
        c0 = bstart[bucket_of(u[j] - tolq, xmin, inv_bw)];
        c1 = bstart[bucket_of(u[j] + tolq, xmin, inv_bw) + 1];
      }
      for (int c = c0; c < c1; ++c) {
        const T dx = bx[c] - u[j];
        const T dy = by[c] - v[j];
        const T d = fmadd(dx, dx, dy * dy);
        const int o = orig[c];
        if (d < best || (d == best && o < arg)) {
          best = d;
          arg = o;
        }
      }
    }
    m[j] = best;
    r[j] = (arg == 0x7fffffff) ? 0 : arg;
  }
  const int L = B < M ? B : M;
  const T tol = (T)fa.tol, tol_pf = (T)fa.tol_pf, Mt = (T)M;
  T Pr = (T)0;
  int s = 1;
  uint32_t taken = 0u;
  for (int k = 0; k < L; ++k) {
    T best = (T)0;
    int jb = -1, rb = 0;
#pragma unroll
    for (int j = 0; j < MAXM; ++j) {
      const bool avail = (j < M) && !((taken >> j) & 1u);
      if (avail && (jb < 0 || m[j] < best)) {
        best = m[j];
        jb = j;
        rb = r[j];
      }
    }
    const T d = sqrt_t(best);
    if (!(d <= tol_pf)) break;
    const T q = (tol - d) / tol;
    Pr = Pr + (Mt + q * q);
    bool dup = false;
#pragma unroll
    for (int j = 0; j < MAXM; ++j) dup |= ((taken >> j) & 1u) && (r[j] == rb);
    if (dup) {
      Pr = Pr - (T)(s * 3);
      ++s;
    }
    if ((fa.downgrade >> jb) & 1u) Pr = Pr - (T)2;
    taken |= 1u << jb;
    if (PAIRS) {
      pairs[2 * k] = (uint32_t)jb + 1u;
      pairs[2 * k + 1] = (uint32_t)rb + 1u;
      *npairs = k + 1;
    }
  }
  return Pr;
}

// ----------------------------------------------------------------------------- wave/block helpers
__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }
__device__ __forceinline__ int wave_id() { return threadIdx.x >> 6; }

__device__ __forceinline__ double wave_incl_sum(double v) {
  const int lane = lane_id();
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const double t = __shfl_up(v, off, 64);
    if (lane >= off) v = v + t;
  }
  return v;
}
__device__ __forceinline__ double wave_incl_max(double v) {
  const int lane = lane_id();
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const double t = __shfl_up(v, off, 64);
    if (lane >= off && t > v) v = t;
  }
  return v;
}
// (value, index): larger value wins, lower index on ties
__device__ __forceinline__ void cmb_max(double& v, int& i, double v2, int i2) {
  if (v2 > v || (v2 == v && i2 < i)) {
    v = v2;
    i = i2;
  }
}
__device__ __forceinline__ void cmb_min(double& v, int& i, double v2, int i2) {
  if (v2 < v || (v2 == v && i2 < i)) {
    v = v2;
    i = i2;
  }
}
__device__ __forceinline__ void wave_argmax(double& v, int& i) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) cmb_max(v, i, __shfl_xor(v, off, 64), __shfl_xor(i, off, 64));
}
__device__ __forceinline__ void wave_argmin(double& v, int& i) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) cmb_min(v, i, __shfl_xor(v, off, 64), __shfl_xor(i, off, 64));
}

// Deterministic block inclusive scan (same code in the propagate and resample kernels, so both see
// bit-identical prefix sums).  sh: >= kWaves doubles.
__device__ __forceinline__ void block_incl_sum(double v, double& incl, double& total, double* sh) {
  const double wi = wave_incl_sum(v);
  if (lane_id() == 63) sh[wave_id()] = wi;
  __syncthreads();
  double pre = 0.0, tot = 0.0;
#pragma unroll
  for (int w = 0; w < kWaves; ++w) {
    if (w < wave_id()) pre = pre + sh[w];
    tot = tot + sh[w];
  }
  incl = pre + wi;
  total = tot;
  __syncthreads();
}

// ----------------------------------------------------------------------------- stratified targets
// r_k = (k + U_k) / N  (PE:671); U_k is the k-th resample draw, taken after all motion draws.
template <int RNG>
__device__ __forceinline__ double target_r(const FrameArgs& fa, int iters, int64_t k) {
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
  return ((double)k + U) / (double)fa.N;
}

// F(x) = #{k : r_k <= x}.  r_k is non-decreasing in k, so target k finds the first particle i whose
// running-max cumulative weight R_i >= r_k (reference: first i with cumsum_i >= r_k, PE:674-679),
// and particle i receives F(R_i) - F(R_{i-1}) copies.
template <int RNG>
__device__ __forceinline__ int64_t count_targets(const FrameArgs& fa, int iters, double x) {
  const int64_t N = fa.N;
  if (!(x >= 0.0)) return 0;  // r_k >= 0; also -inf / NaN
  const double fk = floor(x * (double)N);
  int64_t k = fk < 0.0 ? 0 : (fk > (double)N ? N : (int64_t)fk);
  while (k < N && target_r<RNG>(fa, iters, k) <= x) ++k;
  while (k > 0 && target_r<RNG>(fa, iters, k - 1) > x) --k;
  return k;
}

// ============================================================================== kernels
// ---- per-frame preparation: blob table + control reset (1 block)
template <typename T>
__global__ __launch_bounds__(kBlock) void k_prep(const FrameArgs fa, const double* __restrict__ blobs,
                                                 BlobTable<T>* __restrict__ tab, Ctrl* __restrict__ ctrl) {
  __shared__ T sx[kMaxBlobs];
  __shared__ T sy[kMaxBlobs];
  __shared__ T sred[2 * kWaves];
  const int B = fa.B;
  T lmin = inf_t<T>(), lmax = -inf_t<T>();
  for (int i = threadIdx.x; i < B; i += kBlock) {
    const T x = (T)blobs[2 * i], y = (T)blobs[2 * i + 1];
    sx[i] = x;
    sy[i] = y;
    lmin = x < lmin ? x : lmin;
    lmax = x > lmax ? x : lmax;
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const T a = __shfl_xor(lmin, off, 64), b = __shfl_xor(lmax, off, 64);
    lmin = a < lmin ? a : lmin;
    lmax = b > lmax ? b : lmax;
  }
  if (lane_id() == 0) {
    sred[wave_id()] = lmin;
    sred[kWaves + wave_id()] = lmax;
  }
  __syncthreads();
  T xmin = sred[0], xmax = sred[kWaves];
#pragma unroll
  for (int w = 1; w < kWaves; ++w) {
    xmin = sred[w] < xmin ? sred[w] : xmin;
    xmax = sred[kWaves + w] > xmax ? sred[kWaves + w] : xmax;
  }
  if (B == 0 || !(xmax - xmin < inf_t<T>())) {
    xmin = (T)0;
    xmax = (T)1;
  }
  T span = xmax - xmin;
  if (!(span > (T)0)) span = (T)1;
  const T inv_bw = (T)kBuckets / span;
  // stable rank sort by (x, index)
  for (int i = threadIdx.x; i < B; i += kBlock) {
    const T x = sx[i];
    int rank = 0;
    for (int j = 0; j < B; ++j) {
      const T xj = sx[j];
      rank += (xj < x || (xj == x && j < i)) ? 1 : 0;
    }
    tab->bx[rank] = x;
    tab->by[rank] = sy[i];
    tab->orig[rank] = i;
  }
  // bstart[b] = #{i : bucket(x_i) < b}
  for (int b = threadIdx.x; b <= kBuckets; b += kBlock) {
    int c = 0;
    for (int i = 0; i < B; ++i) c += bucket_of(sx[i], xmin, inv_bw) < b ? 1 : 0;
    tab->bstart[b] = c;
  }
  if (threadIdx.x == 0) {
    tab->xmin = xmin;
    tab->inv_bw = inv_bw;
    tab->b0x = B > 0 ? sx[0] : (T)0;
    tab->b0y = B > 0 ? sy[0] : (T)0;
    // conservative window half-width: every blob with sqrt(d2) <= tol_pf in T arithmetic has
    // |dx| <= tolq (relative + absolute slack covers rounding of dx*dx+dy*dy and sqrt)
    tab->tolq = (T)(fa.tol_pf * (1.0 + 1e-3) + 1e-3);
    tab->B = B;
    Ctrl c;
    c.best_max = 0.0;
    c.S = 0.0;
    c.Rmax = -INFINITY;
    c.done = 0;
    c.has_best = 0;
    c.best_idx = 0;
    c.best_iter = 0;
    c.best_slot = 0;
    c.cur_slot = 0;
    c.iters = 0;
    c.kept_slot = 0;
    c.kept_iter = 0;
    c.accepted = 0;
    c.most_likely_idx = 0;
    c.pad0 = 0;
    c.K_total = 0;
    *ctrl = c;
  }
}

// ---- motion + projection + likelihood, one particle per thread
template <typename T, int RNG, int MAXM, bool PRUNE>
__global__ __launch_bounds__(kBlock) void k_propagate_weigh(
    const FrameArgs fa, const T* __restrict__ prior, T* __restrict__ w0, T* __restrict__ w1,
    BlockPart* __restrict__ p0, BlockPart* __restrict__ p1, const BlobTable<T>* __restrict__ tab,
    const Ctrl* __restrict__ ctrl, int iter) {
  __shared__ T s_bx[kMaxBlobs];
  __shared__ T s_by[kMaxBlobs];
  __shared__ int32_t s_orig[kMaxBlobs];
  __shared__ int32_t s_bstart[kBuckets + 1];
  __shared__ double s_sum[kWaves];
  __shared__ double s_ext[4 * kWaves];
  __shared__ int s_idx[2 * kWaves];

  if (ctrl->done) return;  // the exit rule already fired (uniform)
  const int slot = ctrl->cur_slot;
  const int B = fa.B;
  for (int i = threadIdx.x; i < B; i += kBlock) {
    s_bx[i] = tab->bx[i];
    s_by[i] = tab->by[i];
    s_orig[i] = tab->orig[i];
  }
  for (int b = threadIdx.x; b <= kBuckets; b += kBlock) s_bstart[b] = tab->bstart[b];
  const T xmin = tab->xmin, inv_bw = tab->inv_bw, b0x = tab->b0x, b0y = tab->b0y, tolq = tab->tolq;
  __syncthreads();

  const int n = blockIdx.x * kBlock + threadIdx.x;
  const bool valid = n < fa.N;
  T w = (T)0;
  if (valid) {
    T P[12], u[MAXM], v[MAXM];
    make_particle<T, RNG>(fa, prior, n, iter, P);
    project_markers<T, MAXM>(fa, P, u, v);
    w = likelihood<T, MAXM, PRUNE, false>(fa, u, v, s_bx, s_by, s_orig, s_bstart, xmin, inv_bw, b0x,
                                          b0y, tolq, nullptr, nullptr);
    (slot ? w1 : w0)[n] = w;
  }
  // per-block partials: sum, running-sum extrema, max/argmax, min/argmin
  const double wd = valid ? (double)w : 0.0;
  double incl, tot;
  block_incl_sum(wd, incl, tot, s_sum);
  double mx = valid ? wd : -INFINITY, mn = valid ? wd : INFINITY;
  int ix = valid ? n : 0x7fffffff, in_ = ix;
  double rmax = valid ? incl : -INFINITY, rmin = valid ? incl : INFINITY;
  wave_argmax(mx, ix);
  wave_argmin(mn, in_);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const double a = __shfl_xor(rmax, off, 64), b = __shfl_xor(rmin, off, 64);
    rmax = a > rmax ? a : rmax;
    rmin = b < rmin ? b : rmin;
  }
  if (lane_id() == 0) {
    s_ext[wave_id()] = mx;
    s_ext[kWaves + wave_id()] = mn;
    s_ext[2 * kWaves + wave_id()] = rmax;
    s_ext[3 * kWaves + wave_id()] = rmin;
    s_idx[wave_id()] = ix;
    s_idx[kWaves + wave_id()] = in_;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double bmx = s_ext[0], bmn = s_ext[kWaves], brx = s_ext[2 * kWaves], brn = s_ext[3 * kWaves];
    int bix = s_idx[0], bin = s_idx[kWaves];
#pragma unroll
    for (int ww = 1; ww < kWaves; ++ww) {
      cmb_max(bmx, bix, s_ext[ww], s_idx[ww]);
      cmb_min(bmn, bin, s_ext[kWaves + ww], s_idx[kWaves + ww]);
      brx = s_ext[2 * kWaves + ww] > brx ? s_ext[2 * kWaves + ww] : brx;
      brn = s_ext[3 * kWaves + ww] < brn ? s_ext[3 * kWaves + ww] : brn;
    }
    BlockPart bp;
    bp.sum = tot;
    bp.maxrel = brx;
    bp.minrel = brn;
    bp.maxw = bmx;
    bp.minw = bmn;
    bp.argmax = bix;
    bp.argmin = bin;
    (slot ? p1 : p0)[blockIdx.x] = bp;
  }
}

// ---- iteration bookkeeping + (on the last iteration) normaliser, prefixes, accept (1 block)
template <int RNG>
__global__ __launch_bounds__(kReduceThreads) void k_iter_reduce(const FrameArgs fa, Ctrl* __restrict__ ctrl,
                                                                const BlockPart* __restrict__ p0,
                                                                const BlockPart* __restrict__ p1,
                                                                double* __restrict__ Eb,
                                                                double* __restrict__ Rin, int iter) {
  constexpr int W = kReduceThreads / 64;
  __shared__ double sv[W], sv2[W];
  __shared__ int si[W], si2[W];
  __shared__ int s_flag[3];
  __shared__ double s_S;

  if (ctrl->done) return;
  const int nblk = fa.nblk;
  const int tid = threadIdx.x, lane = lane_id(), wv = wave_id();
  const int chunk = (nblk + kReduceThreads - 1) / kReduceThreads;
  const int b0 = tid * chunk, b1 = min(nblk, b0 + chunk);

  {  // this iteration's max / first argmax
    const int slot = ctrl->cur_slot;
    const BlockPart* P = slot ? p1 : p0;
    double mv = -INFINITY;
    int mi = 0x7fffffff;
    for (int b = b0; b < b1; ++b) cmb_max(mv, mi, P[b].maxw, P[b].argmax);
    wave_argmax(mv, mi);
    if (lane == 0) {
      sv[wv] = mv;
      si[wv] = mi;
    }
    __syncthreads();
    if (tid == 0) {
      for (int w = 1; w < W; ++w) cmb_max(mv, mi, sv[w], si[w]);
      Ctrl c = *ctrl;
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
      c.done = go_on ? 0 : 1;
      c.cur_slot = c.has_best ? 1 - c.best_slot : 1 - slot;
      if (c.done) {
        c.kept_slot = c.has_best ? c.best_slot : slot;
        c.kept_iter = c.has_best ? c.best_iter : iter;
      }
      *ctrl = c;
      s_flag[0] = c.done;
      s_flag[1] = c.kept_slot;
    }
    __syncthreads();
  }
  if (!s_flag[0]) return;
  const BlockPart* KP = s_flag[1] ? p1 : p0;

  // exclusive scan of block sums (deterministic chunked order); S = E_last + sum_last
  double ls = 0.0;
  for (int b = b0; b < b1; ++b) ls = ls + KP[b].sum;
  double wi = wave_incl_sum(ls);
  if (lane == 63) sv[wv] = wi;
  __syncthreads();
  double pre = 0.0;
  for (int w = 0; w < wv; ++w) pre = pre + sv[w];
  // exclusive prefix of this thread's chunk: previous waves + the previous lane's inclusive value
  const double prev_incl = __shfl_up(wi, 1, 64);
  double e = lane == 0 ? pre : pre + prev_incl;
  for (int b = b0; b < b1; ++b) {
    Eb[b] = e;
    e = e + KP[b].sum;
  }
  if (b1 == nblk && b0 < b1) s_S = e;
  if (nblk == 0 && tid == 0) s_S = 0.0;
  __syncthreads();
  const double S = s_S;

  // exclusive max-scan of per-block max normalised cumulative weight
  double lm = -INFINITY;
  if (S != 0.0)
    for (int b = b0; b < b1; ++b) {
      const double c = (Eb[b] + (S > 0.0 ? KP[b].maxrel : KP[b].minrel)) / S;
      lm = c > lm ? c : lm;
    }
  const double wm = wave_incl_max(lm);
  __syncthreads();
  if (lane == 63) sv2[wv] = wm;
  __syncthreads();
  double pm = -INFINITY;
  for (int w = 0; w < wv; ++w) pm = sv2[w] > pm ? sv2[w] : pm;
  {
    const double prev = __shfl_up(wm, 1, 64);
    if (lane > 0 && prev > pm) pm = prev;
  }
  double run = pm;
  for (int b = b0; b < b1; ++b) {
    Rin[b] = run;
    if (S != 0.0) {
      const double c = (Eb[b] + (S > 0.0 ? KP[b].maxrel : KP[b].minrel)) / S;
      run = c > run ? c : run;
    }
  }
  double gmax = -INFINITY;
  for (int w = 0; w < W; ++w) gmax = sv2[w] > gmax ? sv2[w] : gmax;

  // kept iteration's argmax / argmin (re-init branch, PE:714)
  double amv = -INFINITY, anv = INFINITY;
  int ami = 0x7fffffff, ani = 0x7fffffff;
  for (int b = b0; b < b1; ++b) {
    cmb_max(amv, ami, KP[b].maxw, KP[b].argmax);
    cmb_min(anv, ani, KP[b].minw, KP[b].argmin);
  }
  wave_argmax(amv, ami);
  wave_argmin(anv, ani);
  __syncthreads();
  if (lane == 0) {
    sv[wv] = amv;
    si[wv] = ami;
    sv2[wv] = anv;
    si2[wv] = ani;
  }
  __syncthreads();
  if (tid == 0) {
    for (int w = 1; w < W; ++w) {
      cmb_max(amv, ami, sv[w], si[w]);
      cmb_min(anv, ani, sv2[w], si2[w]);
    }
    Ctrl c = *ctrl;
    const double highest = c.has_best ? c.best_max : 0.0;
    c.S = S;
    c.Rmax = gmax;
    c.accepted = (S != 0.0 && highest > fa.accept_thr) ? 1 : 0;  // PE:633
    if (c.accepted) {
      c.most_likely_idx = c.best_idx;
      c.K_total = count_targets<RNG>(fa, c.iters, gmax);
    } else {
      // argmax of the normalised weights (PE:714): a negative sum flips the order
      c.most_likely_idx = (S < 0.0) ? ani : ami;
      c.K_total = 0;
    }
    *ctrl = c;
  }
}

// ---- stratified resampling: scan + target counts + wave-cooperative scatter of regenerated particles
template <typename T, int RNG>
__global__ __launch_bounds__(kBlock) void k_resample(
    const FrameArgs fa, const Ctrl* __restrict__ ctrl, const T* __restrict__ prior, T* __restrict__ post,
    const T* __restrict__ w0, const T* __restrict__ w1, const double* __restrict__ Eb,
    const double* __restrict__ Rin, CountPart* __restrict__ cparts, uint32_t* __restrict__ counts) {
  __shared__ double s_sum[kWaves];
  __shared__ double s_max[kWaves];
  __shared__ int s_hi[kWaves];
  __shared__ int s_c[kWaves], s_ci[kWaves];

  if (!ctrl->done || !ctrl->accepted) return;
  const int slot = ctrl->kept_slot, kiter = ctrl->kept_iter, iters = ctrl->iters;
  const double S = ctrl->S;
  const int64_t Kt = ctrl->K_total;
  const int N = fa.N;
  const int blk = blockIdx.x, lane = lane_id(), wv = wave_id();
  const int n = blk * kBlock + threadIdx.x;
  const bool valid = n < N;
  const T* W = slot ? w1 : w0;

  const double wd = valid ? (double)W[n] : 0.0;
  double incl, tot;
  block_incl_sum(wd, incl, tot, s_sum);
  const double c = (Eb[blk] + incl) / S;
  // inclusive running max over the block, seeded by the running max of all earlier blocks
  double rm = wave_incl_max(valid ? c : -INFINITY);
  if (lane == 63) s_max[wv] = rm;
  __syncthreads();
  double pm = Rin[blk];
  for (int w = 0; w < wv; ++w) pm = s_max[w] > pm ? s_max[w] : pm;
  const double R = rm > pm ? rm : pm;
  const int hi = valid ? (int)count_targets<RNG>(fa, iters, R) : N;
  if (lane == 63) s_hi[wv] = hi;
  __syncthreads();
  int lo = __shfl_up(hi, 1, 64);
  if (lane == 0) lo = (wv == 0) ? (int)count_targets<RNG>(fa, iters, Rin[blk]) : s_hi[wv - 1];
  const int cnt = valid ? hi - lo : 0;
  if (counts && valid) counts[n] = (uint32_t)cnt;

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

  // block max count, first index (winner candidates)
  {
    double cv = valid ? (double)cnt : -1.0;
    int ci = valid ? n : 0x7fffffff;
    wave_argmax(cv, ci);
    if (lane == 0) {
      s_c[wv] = (int)cv;
      s_ci[wv] = ci;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      double bv = s_c[0];
      int bi = s_ci[0];
      for (int w = 1; w < kWaves; ++w) cmb_max(bv, bi, (double)s_c[w], s_ci[w]);
      cparts[blk].maxcount = (int)bv;
      cparts[blk].idx = bi;
    }
  }

  // regenerate the kept-iteration particle (only lanes that own slots touch the prior)
  T P[12];
#pragma unroll
  for (int q = 0; q < 12; ++q) P[q] = (T)0;
  if (e > a) make_particle<T, RNG>(fa, prior, n, kiter, P);

  // wave-cooperative scatter: the wave's lanes own consecutive slot ranges [a, e)
  const int wa = __shfl(a, 0, 64);
  const int we = __shfl(e, 63, 64);
  for (int base = wa; base < we; base += 64) {
    const int k = base + lane;
    int l = 0;
#pragma unroll
    for (int step = 32; step > 0; step >>= 1) {
      const int ac = __shfl(a, l + step, 64);
      if (ac <= k) l += step;
    }
    T Q[12];
#pragma unroll
    for (int q = 0; q < 12; ++q) Q[q] = __shfl(P[q], l, 64);
    if (k < we) {
#pragma unroll
      for (int q = 0; q < 12; ++q) post[(int64_t)q * fa.ld + k] = Q[q];
    }
  }
}

// ---- winner selection + output record (1 block)
template <typename T, int RNG, int MAXM>
__global__ __launch_bounds__(kBlock) void k_final(const FrameArgs fa, const Ctrl* __restrict__ ctrl,
                                                  const T* __restrict__ prior,
                                                  const CountPart* __restrict__ cparts,
                                                  const BlobTable<T>* __restrict__ tab,
                                                  OutDev* __restrict__ out) {
  __shared__ double sv[kWaves];
  __shared__ int si[kWaves];
  const Ctrl c = *ctrl;
  if (!c.done) {
    if (threadIdx.x == 0) out->done = 0;
    return;
  }
  double bv = -1.0;
  int bi = 0x7fffffff;
  if (c.accepted)
    for (int b = threadIdx.x; b < fa.nblk; b += kBlock) cmb_max(bv, bi, (double)cparts[b].maxcount, cparts[b].idx);
  wave_argmax(bv, bi);
  if (lane_id() == 0) {
    sv[wave_id()] = bv;
    si[wave_id()] = bi;
  }
  __syncthreads();
  if (threadIdx.x != 0) return;
  for (int w = 1; w < kWaves; ++w) cmb_max(bv, bi, sv[w], si[w]);

  OutDev o;
  o.done = 1;
  o.pad = 0;
  o.iters = c.iters;
  o.kept_iter = c.kept_iter;
  o.most_likely_idx = c.most_likely_idx;
  o.accepted = c.accepted;
  o.resampled = c.accepted;
  o.winner_idx = c.accepted ? bi : -1;
  o.flag_fail = c.accepted ? 1 : 4;
  o.highest_prob = c.has_best ? c.best_max : 0.0;
  o.prob_sum = c.S;
  o.n_corr = 0;
  for (int q = 0; q < 2 * kMaxMarkers; ++q) o.corr[q] = 0u;

  T P[12];
  make_particle<T, RNG>(fa, prior, c.most_likely_idx, c.kept_iter, P);
  for (int q = 0; q < 12; ++q) o.most_likely_pose[q] = (double)P[q];
  if (c.accepted) {
    make_particle<T, RNG>(fa, prior, bi, c.kept_iter, P);
    T u[MAXM], v[MAXM];
    project_markers<T, MAXM>(fa, P, u, v);
    int np = 0;
    likelihood<T, MAXM, true, true>(fa, u, v, tab->bx, tab->by, tab->orig, tab->bstart, tab->xmin,
                                    tab->inv_bw, tab->b0x, tab->b0y, tab->tolq, o.corr, &np);
    o.n_corr = np;
  }
  for (int q = 0; q < 12; ++q) o.winner_pose[q] = (double)P[q];
  *out = o;
}

// ---- state import / export / regeneration (API helpers, not on the timed path)
template <typename T>
__global__ void k_import(const double* __restrict__ poses, T* __restrict__ st, int N, int64_t ld) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  for (int q = 0; q < 12; ++q) st[(int64_t)q * ld + n] = (T)poses[12 * (int64_t)n + q];
}
template <typename T>
__global__ void k_export(const T* __restrict__ st, double* __restrict__ poses, int N, int64_t ld) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  for (int q = 0; q < 12; ++q) poses[12 * (int64_t)n + q] = (double)st[(int64_t)q * ld + n];
}
template <typename T, int RNG>
__global__ void k_regen(const FrameArgs fa, const Ctrl* __restrict__ ctrl, const T* __restrict__ prior,
                        double* __restrict__ poses) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= fa.N) return;
  T P[12];
  make_particle<T, RNG>(fa, prior, n, ctrl->kept_iter, P);
  for (int q = 0; q < 12; ++q) poses[12 * (int64_t)n + q] = (double)P[q];
}
template <typename T>
__global__ void k_weights_export(const Ctrl* __restrict__ ctrl, const T* __restrict__ w0,
                                 const T* __restrict__ w1, double* __restrict__ out, int N) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  out[n] = (double)(ctrl->kept_slot ? w1 : w0)[n];
}

}  // namespace pfmpe
