// pfmpe_init.hip — brute-force P3P (re)initialisation on the device, and its
// C-ABI entry points pfmpe_p3p_histogram / pfmpe_initialise (include/pfmpe.h).
//
// Replaces PoseEstimator::initialise (pf_mpe_lib/src/pose_estimator.cpp:1503-1786, "PE") for the
// particle-filter configuration.  Work split:
//   device  k_init_prep   calculateImageVectors (PE:1072-1085), one thread per blob
//           k_p3p_filter  the 3-blob spread filter (PE:1554-1581), one thread per combination
//           k_p3p_hist    the histogram (PE:1543-1716): one thread per (combination, ordered marker
//                         triple), P3P + 4 back projections, exact x-window pruning of the
//                         nearest-projection search, LDS histogram flushed with integer atomics
//           k_p3p_check   checkCorrespondences' P3P stage (PE:1331-1475), one thread per
//                         (candidate correspondence vector, 3-subset)
//           k_init_seed   the particle seeding + fill loop (PE:1429-1437, 1755-1760) into the state
//   host    candidate vectors from the histogram (PE:1134-1288), the ordered bookkeeping of
//           checkCorrespondences (flags, particle slots, mean re-projections, PE:1425-1496) and
//           computeTransformation (PE:2139-2161)
// Integer histogram increments are commutative, so the device enumerates combinations in colex order
// and marker triples in any order; the reference's lexicographic order only matters for
// checkCorrespondences (particle slot order), which keeps it.
#include "pfmpe_ctx.hpp"
#include "pf_p3p.hpp"

using namespace pfmpe;
using namespace pfmpe_impl;

namespace pfmpe {

constexpr int kInitBlock = 256;
#ifndef PFMPE_P3P_MINB
#define PFMPE_P3P_MINB 2  // 2 waves per SIMD: 353 us vs 519 us at 1 (scratch 160 B vs 80 B), 476 us at 3 (spills)
#endif
constexpr double kThreshDist = 10000 * 100;  // threshDist / threshDist2 (PE:1557-1558), px^2

struct InitArgs {
  double K[9];
  double markers[kMaxMarkers * 3];
  double tol;      // back_projection_pixel_tolerance_
  double win;      // x half-window of the pruned nearest-projection search (> tol, exact superset)
  int M, B, nperm;
  int ncomb_m;     // C(M, 3) (check stage)
  int64_t ncomb;   // C(B, 3)
  int64_t items;   // ncomb * nperm (hist) or ncand * ncomb_m (check)
};

__device__ __forceinline__ int64_t c3(int64_t n) { return n * (n - 1) * (n - 2) / 6; }
__device__ __forceinline__ int64_t c2(int64_t n) { return n * (n - 1) / 2; }

// colex rank r -> a < b < c with r = C(c,3) + C(b,2) + a
__device__ __forceinline__ void unrank3(int64_t r, int& a, int& b, int& c) {
  int cc = (int)cbrt(6.0 * (double)r);
  cc = cc < 2 ? 2 : cc;
  while (c3(cc) > r) --cc;
  while (c3(cc + 1) <= r) ++cc;
  const int64_t r2 = r - c3(cc);
  int bb = (int)sqrt(2.0 * (double)r2);
  bb = bb < 1 ? 1 : bb;
  while (c2(bb) > r2) --bb;
  while (c2(bb + 1) <= r2) ++bb;
  a = (int)(r2 - c2(bb));
  b = bb;
  c = cc;
}

// p-th ordered triple of distinct markers (any fixed order: the histogram is a commutative sum)
__device__ __forceinline__ void perm3(int p, int M, int& i0, int& i1, int& i2) {
  const int m12 = (M - 1) * (M - 2);
  i0 = p / m12;
  const int rem = p - i0 * m12;
  const int j1 = rem / (M - 2);
  const int j2 = rem - j1 * (M - 2);
  i1 = j1 + (j1 >= i0 ? 1 : 0);
  const int lo = i0 < i1 ? i0 : i1, hi = i0 < i1 ? i1 : i0;
  i2 = j2;
  if (i2 >= lo) ++i2;
  if (i2 >= hi) ++i2;
}

// un[m] = the m-th index of {0, 1, ...} without x, y, z (ascending), in registers (no scratch)
template <int MAXU>
__device__ __forceinline__ void unused_markers(int x, int y, int z, int* un) {
  const int lo = min(x, min(y, z)), hi = max(x, max(y, z)), mid = x + y + z - lo - hi;
#pragma unroll
  for (int m = 0; m < MAXU; ++m) {
    int v = m;
    v += v >= lo ? 1 : 0;
    v += v >= mid ? 1 : 0;
    v += v >= hi ? 1 : 0;
    un[m] = v;
  }
}

__global__ void k_init_prep(const InitArgs ia, const double* __restrict__ blobs, double* __restrict__ iv) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= ia.B) return;
  double v[3];
  v[0] = (blobs[2 * i] - ia.K[2]) / ia.K[0];
  v[1] = (blobs[2 * i + 1] - ia.K[5]) / ia.K[4];
  v[2] = 1;
  const double n = p3p::norm3(v);
  for (int k = 0; k < 3; ++k) iv[3 * i + k] = v[k] / n;
}

__device__ __forceinline__ double sqd(double ax, double ay, double bx, double by) {
  const double dx = ax - bx, dy = ay - by;
  return dx * dx + dy * dy;
}

// PE:1554-1581: the three blobs pairwise within threshDist, and >= 5 blobs within threshDist2 of
// their centroid (the three themselves included)
__global__ void k_p3p_filter(const InitArgs ia, const double* __restrict__ blobs, uint8_t* __restrict__ pass) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= ia.ncomb) return;
  int a, b, c;
  unrank3(r, a, b, c);
  const double x1 = blobs[2 * a], y1 = blobs[2 * a + 1];
  const double x2 = blobs[2 * b], y2 = blobs[2 * b + 1];
  const double x3 = blobs[2 * c], y3 = blobs[2 * c + 1];
  bool ok = !(sqd(x1, y1, x2, y2) > kThreshDist) && !(sqd(x1, y1, x3, y3) > kThreshDist) &&
            !(sqd(x2, y2, x3, y3) > kThreshDist);
  if (ok) {
    const double mx = (x1 + x2 + x3) / 3, my = (y1 + y2 + y3) / 3;
    int cd = 0;
    for (int k = 0; k < ia.B; ++k) cd += sqd(mx, my, blobs[2 * k], blobs[2 * k + 1]) < kThreshDist ? 1 : 0;
    ok = cd >= 5;
  }
  pass[r] = ok ? 1 : 0;
}


// Stage 1: one thread per (colex combination, ordered marker triple), grid-stride.  HLDS: histogram in
// LDS (flushed once per block with integer atomics) or straight to global atomics for large B x M.
// Dynamic LDS: sorted blob x, y (doubles), original index (int), then the LDS histogram.
template <int MAXU, bool HLDS>
__global__ __launch_bounds__(kInitBlock, PFMPE_P3P_MINB) void k_p3p_hist(const InitArgs ia, const double* __restrict__ blobs,
                                                          const double* __restrict__ iv,
                                                          const double* __restrict__ sorted_xy,
                                                          const int* __restrict__ sorted_idx,
                                                          const uint8_t* __restrict__ pass,
                                                          uint32_t* __restrict__ hist) {
  extern __shared__ __align__(16) unsigned char lds[];
  __shared__ double s_mk[kMaxMarkers * 3];
  const int B = ia.B, M = ia.M;
  double* sx = (double*)lds;
  double* sy = sx + B;
  int* sidx = (int*)(sy + B);
  uint32_t* lh = (uint32_t*)(sidx + ((B + 3) & ~3));
  for (int i = threadIdx.x; i < B; i += blockDim.x) {
    sx[i] = sorted_xy[2 * i];
    sy[i] = sorted_xy[2 * i + 1];
    sidx[i] = sorted_idx[i];
  }
  for (int i = threadIdx.x; i < 3 * M; i += blockDim.x) s_mk[i] = ia.markers[i];
  if (HLDS)
    for (int i = threadIdx.x; i < B * M; i += blockDim.x) lh[i] = 0;
  __syncthreads();
  uint32_t* H = HLDS ? lh : hist;
  const double tol = ia.tol, win = ia.win;
  const int nuo = M - 3;

  for (int64_t item = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; item < ia.items;
       item += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = item / ia.nperm;
    const int p = (int)(item - r * ia.nperm);
    if (!pass[r]) continue;
    int sa[3];
    unrank3(r, sa[0], sa[1], sa[2]);
    int pm[3];
    perm3(p, M, pm[0], pm[1], pm[2]);
    double fv[3][3], wp[3][3];
    for (int k = 0; k < 3; ++k)
      for (int q = 0; q < 3; ++q) {
        fv[k][q] = iv[3 * sa[k] + q];
        wp[k][q] = s_mk[3 * pm[k] + q];
      }
    p3p::Setup st;
    double roots[4];
    if (!p3p::setup(fv, wp, st, roots)) continue;
    int un[MAXU > 0 ? MAXU : 1];
    unused_markers<MAXU>(pm[0], pm[1], pm[2], un);
    const double dmx = (blobs[2 * sa[0]] + blobs[2 * sa[1]] + blobs[2 * sa[2]]) / 3;
    const double dmy = (blobs[2 * sa[0] + 1] + blobs[2 * sa[1] + 1] + blobs[2 * sa[2] + 1]) / 3;
    double prev[12];
    for (int k = 0; k < 4; ++k) {
      double sol[12];
      p3p::solution(st, roots[k], sol);
      bool repeated = false;  // (solutions(k) - solutions(k-1)).all() == 0: some entry unchanged
      if (k > 0)
        for (int q = 0; q < 12; ++q) repeated = repeated || (sol[q] - prev[q] == 0);
      for (int q = 0; q < 12; ++q) prev[q] = sol[q];
      if (repeated || !p3p::finite12(sol)) continue;
      double inv[12];
      p3p::inverse34(sol, inv);
      double pu[MAXU > 0 ? MAXU : 1], pv[MAXU > 0 ? MAXU : 1];
#pragma unroll
      for (int m = 0; m < MAXU; ++m)
        if (m < nuo) p3p::project(ia.K, inv, &s_mk[3 * un[m]], pu[m], pv[m]);
      bool any = false;
#pragma unroll
      for (int m = 0; m < MAXU; ++m) {
        if (m >= nuo) break;
        const double u = pu[m];
        if (!(fabs(u) < 1e300) || !(fabs(pv[m]) < 1e300)) continue;  // NaN / inf never wins a strict '<'
        int lo = 0, hi = B;                                           // first sx >= u - win
        const double xl = u - win, xh = u + win;
        while (lo < hi) {
          const int mid = (lo + hi) >> 1;
          if (sx[mid] < xl) lo = mid + 1;
          else hi = mid;
        }
        for (int q = lo; q < B && sx[q] <= xh; ++q) {
          const int bi = sidx[q];
          if (bi == sa[0] || bi == sa[1] || bi == sa[2]) continue;
          const double bx = sx[q], by = sy[q];
          if (!(sqd(dmx, dmy, bx, by) < kThreshDist)) continue;
          // calculateMinDistancesAndPairs (PE:2093-2137): nearest projection, strict '<' from +inf
          double mind = INFINITY;
          int pr = -1;
#pragma unroll
          for (int m2 = 0; m2 < MAXU; ++m2)
            if (m2 < nuo) {
              const double d = sqd(bx, by, pu[m2], pv[m2]);
              if (d < mind) {
                mind = d;
                pr = m2;
              }
            }
          if (pr != m || !(sqrt(mind) < tol)) continue;
          if (!any) {
            any = true;
            for (int mm = 0; mm < 3; ++mm) atomicAdd(&H[sa[mm] * M + pm[mm]], 1u);
          }
          atomicAdd(&H[bi * M + un[m]], 1u);
        }
      }
    }
  }
  if (HLDS) {
    __syncthreads();
    for (int i = threadIdx.x; i < B * M; i += blockDim.x)
      if (lh[i]) atomicAdd(&hist[i], lh[i]);
  }
}

// Stage 3: checkCorrespondences' P3P part (PE:1331-1475) for candidate `ci`, lexicographic 3-subset q of
// its M correspondence rows.  cand: per candidate 2*M ints (LED, detection), 1-based.
// status: 0 = P3P failed (collinear), 1 = no solution within certainty_threshold, 2 = valid (inv = the
// inverse of the smallest-error valid solution, top 3 rows).
template <int MAXU>
__global__ __launch_bounds__(kInitBlock) void k_p3p_check(const InitArgs ia, double certainty_threshold,
                                                           const double* __restrict__ blobs,
                                                           const double* __restrict__ iv,
                                                           const int* __restrict__ cand,
                                                           const int* __restrict__ triples,
                                                           uint8_t* __restrict__ status, double* __restrict__ out_inv) {
  const int64_t item = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (item >= ia.items) return;
  const int ci = (int)(item / ia.ncomb_m);
  const int q = (int)(item - (int64_t)ci * ia.ncomb_m);
  const int M = ia.M;
  const int* cp = cand + (int64_t)ci * 2 * M;
  const int t = triples[q];
  const int s[3] = {t & 0xff, (t >> 8) & 0xff, (t >> 16) & 0xff};
  double fv[3][3], wp[3][3];
  for (int k = 0; k < 3; ++k)
    for (int d = 0; d < 3; ++d) {
      wp[k][d] = ia.markers[3 * (cp[2 * s[k]] - 1) + d];
      fv[k][d] = iv[3 * (cp[2 * s[k] + 1] - 1) + d];
    }
  int un[MAXU > 0 ? MAXU : 1];
  unused_markers<MAXU>(s[0], s[1], s[2], un);
  const int nu = M - 3;
  p3p::Setup st;
  double roots[4];
  if (!p3p::setup(fv, wp, st, roots)) {
    status[item] = 0;
    return;
  }
  const double tol2 = ia.tol * ia.tol;  // pow(tol, 2) folds to tol * tol
  double min_err = INFINITY;
  double best[12];
  bool any_valid = false;
  for (int j = 0; j < 4; ++j) {
    double sol[12];
    p3p::solution(st, roots[j], sol);
    if (!p3p::finite12(sol)) continue;
    double inv[12];
    p3p::inverse34(sol, inv);
    // calculateSquaredReprojectionErrorAndCertainty (PE:1087-1132): index-paired squared distances,
    // then up to min(size) extractions of Eigen's minCoeff (first minimum, from coeff(0)) while <= tol^2
    double dist[MAXU > 0 ? MAXU : 1];
#pragma unroll
    for (int a = 0; a < MAXU; ++a)
      if (a < nu) {
        double u, v;
        p3p::project(ia.K, inv, &ia.markers[3 * (cp[2 * un[a]] - 1)], u, v);
        const int bi = cp[2 * un[a] + 1] - 1;
        dist[a] = sqd(blobs[2 * bi], blobs[2 * bi + 1], u, v);
      }
    double sq_err = 0;
    int ncorr = 0;
    for (int it = 0; it < nu; ++it) {
      double mv = dist[0];
      int r = 0;
#pragma unroll
      for (int a = 1; a < MAXU; ++a)
        if (a < nu && dist[a] < mv) {
          mv = dist[a];
          r = a;
        }
      if (!(mv <= tol2)) break;
      sq_err += mv;
      ncorr++;
#pragma unroll
      for (int a = 0; a < MAXU; ++a)
        if (a == r) dist[a] = INFINITY;
    }
    const double certainty = (double)ncorr / (double)nu;
    if (certainty >= certainty_threshold) {
      any_valid = true;
      if (sq_err < min_err) {
        min_err = sq_err;
        for (int k = 0; k < 12; ++k) best[k] = inv[k];
      }
    }
  }
  status[item] = any_valid ? 2 : 1;
  if (any_valid)
    for (int k = 0; k < 12; ++k) out_inv[item * 12 + k] = best[k];
}

// Stage 4: PoseParticle after initialise (PE:1429-1437 stores, PE:1755-1760 fill): slot s >= 1 takes
// estimate ((N - s - 1) mod K) + 1 (1-based, estimate k sits at slot N - k); slot 0 only when K >= N.
__global__ void k_init_seed(const double* __restrict__ est, int K, int N, double* __restrict__ poses) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= N || (s == 0 && K < N)) return;
  const int e = (N - s - 1) % K;  // 0-based estimate
  for (int q = 0; q < 12; ++q) poses[12 * (int64_t)s + q] = est[12 * (int64_t)e + q];
}

}  // namespace pfmpe

// ===================================================================================== host side
namespace {

struct Arena {
  size_t off = 0;
  template <typename X>
  size_t take(size_t n) {
    const size_t o = off;
    off += (n * sizeof(X) + 255) & ~(size_t)255;
    return o;
  }
};

int ensure_init(pfmpe_ctx* c, size_t bytes) {
  if (bytes <= c->init_cap) return PFMPE_OK;
  if (c->d_init) {
    HIPCHK(c, hipStreamSynchronize(c->stream));
    HIPCHK(c, hipFree(c->d_init));
    c->d_init = nullptr;
    c->init_cap = 0;
  }
  HIPCHK(c, hipMalloc((void**)&c->d_init, bytes));
  c->init_cap = bytes;
  return PFMPE_OK;
}

int ensure_xfer(pfmpe_ctx* c) {
  if (!c->d_xfer) HIPCHK(c, hipMalloc((void**)&c->d_xfer, (size_t)c->max_particles * 12 * sizeof(double)));
  return PFMPE_OK;
}

template <typename T, typename SP>
void export1(pfmpe_ctx* c) {
  Pose12<T> a;
  for (int q = 0; q < 12; ++q) a.v[q] = (T)c->anchor[c->prior_idx][q];
  hipLaunchKernelGGL((k_export<T, SP>), dim3(1), dim3(64), 0, c->stream, (const SP*)c->d_state[c->prior_idx],
                     c->d_xfer, 1, c->ld, a, prior_owner_ptr(c));
}
// slot 0 of the resident set -> d_xfer[0..11]
int export_slot0(pfmpe_ctx* c) {
  if (c->state_dtype == PFMPE_STATE_F64)
    export1<double, double>(c);
  else if (c->state_dtype == PFMPE_STATE_F16)
    export1<float, __half>(c);
  else
    export1<float, float>(c);
  HIPCHK(c, hipGetLastError());
  return PFMPE_OK;
}

template <typename T, typename SP>
void import_n(pfmpe_ctx* c, int N, int slot) {
  Pose12<T> a;
  for (int q = 0; q < 12; ++q) a.v[q] = (T)c->anchor[slot][q];
  hipLaunchKernelGGL((k_import<T, SP>), dim3((N + 255) / 256), dim3(256), 0, c->stream, c->d_xfer,
                     (SP*)c->d_state[slot], N, c->ld, a);
}
// d_xfer (N x 12) -> the prior buffer, as pfmpe_set_prior does; anchor = the given pose
int import_xfer(pfmpe_ctx* c, int N, const double* anchor) {
  const int slot = c->prior_idx;
  std::memcpy(c->anchor[slot], anchor, 12 * sizeof(double));
  c->prior_owner = -1;  // stored in particle order
  if (c->state_dtype == PFMPE_STATE_F64)
    import_n<double, double>(c, N, slot);
  else if (c->state_dtype == PFMPE_STATE_F16)
    import_n<float, __half>(c, N, slot);
  else
    import_n<float, float>(c, N, slot);
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipMemsetAsync(c->d_ctrl, 0, sizeof(Ctrl), c->stream));
  HIPCHK(c, hipMemsetAsync(c->d_winkey, 0, kWinBytes, c->stream));
  HIPCHK(c, hipMemsetAsync(c->d_counters, 0, counters_bytes(c), c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  c->N = N;
  c->has_prior = true;
  c->has_last = false;
  return PFMPE_OK;
}

InitArgs make_args(const pfmpe_ctx* c, int B) {
  InitArgs ia{};
  std::memcpy(ia.K, c->K, sizeof(ia.K));
  std::memcpy(ia.markers, c->markers, sizeof(ia.markers));
  ia.tol = c->params.tol;
  ia.win = c->params.tol * (1.0 + 1e-6) + 1e-6;
  ia.M = c->M;
  ia.B = B;
  ia.nperm = c->M * (c->M - 1) * (c->M - 2);
  ia.ncomb_m = c->M * (c->M - 1) * (c->M - 2) / 6;
  ia.ncomb = (int64_t)B * (B - 1) * (B - 2) / 6;
  return ia;
}

template <int MAXU>
void launch_hist(pfmpe_ctx* c, const InitArgs& ia, bool hlds, size_t lds, int grid, const double* blobs,
                 const double* iv, const double* sxy, const int* sidx, const uint8_t* pass, uint32_t* hist) {
  if (hlds)
    hipLaunchKernelGGL((k_p3p_hist<MAXU, true>), dim3(grid), dim3(kInitBlock), lds, c->stream, ia, blobs, iv, sxy,
                       sidx, pass, hist);
  else
    hipLaunchKernelGGL((k_p3p_hist<MAXU, false>), dim3(grid), dim3(kInitBlock), lds, c->stream, ia, blobs, iv, sxy,
                       sidx, pass, hist);
}

// stage 1 on the device; hist (B x M) lands in host memory
int run_histogram(pfmpe_ctx* c, const double* blobs, int B, uint32_t* hist) {
  InitArgs ia = make_args(c, B);
  ia.items = ia.ncomb * ia.nperm;
  // host-built x-sorted blob list for the pruned search (a data-structure build, like the PF blob table)
  std::vector<int> order(B);
  for (int i = 0; i < B; ++i) order[i] = i;
  std::stable_sort(order.begin(), order.end(), [&](int x, int y) { return blobs[2 * x] < blobs[2 * y]; });
  std::vector<double> sxy(2 * (size_t)B);
  for (int i = 0; i < B; ++i) {
    sxy[2 * i] = blobs[2 * order[i]];
    sxy[2 * i + 1] = blobs[2 * order[i] + 1];
  }
  Arena ar;
  const size_t o_blobs = ar.take<double>(2 * (size_t)B), o_iv = ar.take<double>(3 * (size_t)B);
  const size_t o_sxy = ar.take<double>(2 * (size_t)B), o_sidx = ar.take<int>(B);
  const size_t o_pass = ar.take<uint8_t>((size_t)ia.ncomb), o_hist = ar.take<uint32_t>((size_t)B * c->M);
  RET(ensure_init(c, ar.off));
  unsigned char* d = c->d_init;
  double* d_blobs = (double*)(d + o_blobs);
  double* d_iv = (double*)(d + o_iv);
  double* d_sxy = (double*)(d + o_sxy);
  int* d_sidx = (int*)(d + o_sidx);
  uint8_t* d_pass = d + o_pass;
  uint32_t* d_hist = (uint32_t*)(d + o_hist);
  HIPCHK(c, hipMemcpyAsync(d_blobs, blobs, 2 * (size_t)B * sizeof(double), hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(d_sxy, sxy.data(), sxy.size() * sizeof(double), hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(d_sidx, order.data(), (size_t)B * sizeof(int), hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemsetAsync(d_hist, 0, (size_t)B * c->M * sizeof(uint32_t), c->stream));
  hipLaunchKernelGGL(k_init_prep, dim3((B + 255) / 256), dim3(256), 0, c->stream, ia, d_blobs, d_iv);
  HIPCHK(c, hipGetLastError());
  hipLaunchKernelGGL(k_p3p_filter, dim3((unsigned)((ia.ncomb + 255) / 256)), dim3(256), 0, c->stream, ia, d_blobs,
                     d_pass);
  HIPCHK(c, hipGetLastError());
  const size_t hist_bytes = (size_t)B * c->M * sizeof(uint32_t);
  const bool hlds = hist_bytes <= 32 * 1024;
  const size_t lds = (size_t)B * 16 + (size_t)((B + 3) & ~3) * 4 + (hlds ? hist_bytes : 0);
  const int64_t want = (ia.items + kInitBlock - 1) / kInitBlock;
  const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(want, (int64_t)std::max(c->num_cu, 1) * 8));
  RET(launch(c, PFMPE_K_P3P_HIST, [&] {
    const int nu = c->M - 3;
    if (nu <= 2)
      launch_hist<2>(c, ia, hlds, lds, grid, d_blobs, d_iv, d_sxy, d_sidx, d_pass, d_hist);
    else if (nu <= 9)
      launch_hist<9>(c, ia, hlds, lds, grid, d_blobs, d_iv, d_sxy, d_sidx, d_pass, d_hist);
    else
      launch_hist<kMaxMarkers - 3>(c, ia, hlds, lds, grid, d_blobs, d_iv, d_sxy, d_sidx, d_pass, d_hist);
  }));
  HIPCHK(c, hipMemcpyAsync(hist, d_hist, hist_bytes, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  if (c->timing_now) RET(harvest_timing(c));
  return PFMPE_OK;
}

// correspondencesFromHistogram (PE:1134-1288) with bInitialisation = true: candidate (LED, detection)
// vectors, most probable first; ambiguous ones (a detection used twice, zeros included) dropped.
int candidates(pfmpe_ctx* c, int B, int M, const uint32_t* hist, int max_cand,
               std::vector<std::vector<uint32_t>>& out) {
  out.clear();
  const double prob_threshold = (1.3 * 1.0) / (double)((unsigned)B * (unsigned)M);
  std::vector<double> hp((size_t)B * M);
  for (size_t i = 0; i < hp.size(); ++i) hp[i] = (double)hist[i];
  std::vector<uint32_t> rowSum(B, 0);
  for (int r = 0; r < B; ++r)
    for (int q = 0; q < M; ++q) rowSum[r] += hist[(size_t)r * M + q];
  for (int col = 0; col < M; ++col) {
    uint32_t colSum = 0;
    for (int r = 0; r < B; ++r) colSum += hist[(size_t)r * M + col];
    if (colSum == 0) continue;
    for (int r = 0; r < B; ++r) {
      const uint32_t den = colSum * rowSum[r];  // 32-bit unsigned product, as the reference's
      double& v = hp[(size_t)r * M + col];
      v = std::max(0.0, (v * v) / (double)den);
      if (v < prob_threshold) v = 0;
    }
  }
  std::vector<std::vector<double>> up(M);
  std::vector<std::vector<int>> un(M);
  for (int a = 0; a < M; ++a)
    for (int b = 0; b < B; ++b)
      if (hp[(size_t)b * M + a] != 0) {
        up[a].push_back(hp[(size_t)b * M + a]);
        un[a].push_back(b + 1);
      }
  int64_t Ntot = 1;
  for (int k = 0; k < M; ++k) {
    Ntot *= std::max<int64_t>(1, (int64_t)up[k].size());
    if (Ntot > max_cand) return fail(c, PFMPE_E_CAP, "initialise: correspondence vectors exceed max_candidates");
  }
  const int N = (int)Ntot;
  std::vector<double> vp(N);
  std::vector<int> comb((size_t)N * M);
  for (int i = 0; i < N; ++i) {
    double prob = 1;
    int n = 1;
    for (int led = M - 1; led > -1; --led) {
      const int nv = (int)un[led].size();
      if (nv > 0) {
        const int idx = (i / n) % nv;
        prob = prob * up[led][idx];
        comb[(size_t)i * M + led] = un[led][idx];
        n = n * nv;
      } else {
        comb[(size_t)i * M + led] = 0;
      }
    }
    vp[i] = prob;
  }
  double sum = 0;
  for (int i = 0; i < N; ++i) sum += vp[i];
  for (int i = 0; i < N; ++i) vp[i] = vp[i] / sum;
  // N rounds of std::max_element (first maximum) with the picked entry zeroed (PE:1256-1260).  Without
  // NaNs that is: the positive entries by (value desc, index asc), then index 0 (all zero by then) for
  // each entry that was not positive.  A NaN (sum 0 or inf) falls back to the literal O(N^2) rounds.
  std::vector<int> picks;
  picks.reserve(N);
  bool has_nan = false;
  for (int i = 0; i < N; ++i) has_nan = has_nan || !(vp[i] == vp[i]);
  if (!has_nan) {
    for (int i = 0; i < N; ++i)
      if (vp[i] > 0) picks.push_back(i);
    std::stable_sort(picks.begin(), picks.end(), [&](int x, int y) { return vp[x] > vp[y]; });
    while ((int)picks.size() < N) picks.push_back(0);
  } else {
    for (int bb = 0; bb < N; ++bb) {
      int row = 0;
      for (int i = 1; i < N; ++i)
        if (vp[row] < vp[i]) row = i;
      vp[row] = 0;
      picks.push_back(row);
    }
  }
  for (int bb = 0; bb < N; ++bb) {
    const int row = picks[bb];
    const int* det = &comb[(size_t)row * M];
    bool amb = false;  // checkAmbiguity (PE:2447-2458)
    for (int i = 0; i < M && !amb; ++i)
      for (int j = M - 1; j > i; --j)
        if (det[i] == det[j]) {
          amb = true;
          break;
        }
    if (amb) continue;
    std::vector<uint32_t> pr;
    for (int led = 0; led < M; ++led)
      if (det[led] != 0) {
        pr.push_back((uint32_t)(led + 1));
        pr.push_back((uint32_t)det[led]);
      }
    out.push_back(pr);
  }
  return PFMPE_OK;
}

// computeTransformation (PE:2139-2161): R = V U^T from the SVD of the 3x3 cross-covariance (one-sided
// Jacobi), t = mean(rep) - R mean(obj).
void compute_transformation(int M, const double* obj, const double* rep, double* T12) {
  double mo[3] = {0, 0, 0}, mr[3] = {0, 0, 0};
  for (int j = 0; j < M; ++j)
    for (int k = 0; k < 3; ++k) {
      mo[k] += obj[3 * j + k];
      mr[k] += rep[3 * j + k];
    }
  for (int k = 0; k < 3; ++k) {
    mo[k] /= M;
    mr[k] /= M;
  }
  double U[9], V[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
  for (int r = 0; r < 3; ++r)
    for (int col = 0; col < 3; ++col) {
      double s = 0;
      for (int j = 0; j < M; ++j) s += (obj[3 * j + r] - mo[r]) * (rep[3 * j + col] - mr[col]);
      U[3 * r + col] = s;
    }
  for (int sweep = 0; sweep < 60; ++sweep) {
    double off = 0;
    for (int p = 0; p < 2; ++p)
      for (int q = p + 1; q < 3; ++q) {
        double al = 0, be = 0, ga = 0;
        for (int i = 0; i < 3; ++i) {
          al += U[3 * i + p] * U[3 * i + p];
          be += U[3 * i + q] * U[3 * i + q];
          ga += U[3 * i + p] * U[3 * i + q];
        }
        if (ga == 0) continue;
        off = std::max(off, std::fabs(ga) / std::sqrt(al * be));
        const double zeta = (be - al) / (2 * ga);
        const double t = (zeta >= 0 ? 1.0 : -1.0) / (std::fabs(zeta) + std::sqrt(1 + zeta * zeta));
        const double cs = 1 / std::sqrt(1 + t * t), sn = cs * t;
        for (int i = 0; i < 3; ++i) {
          const double up = U[3 * i + p], uq = U[3 * i + q];
          U[3 * i + p] = cs * up - sn * uq;
          U[3 * i + q] = sn * up + cs * uq;
          const double vp = V[3 * i + p], vq = V[3 * i + q];
          V[3 * i + p] = cs * vp - sn * vq;
          V[3 * i + q] = sn * vp + cs * vq;
        }
      }
    if (off < 1e-15) break;
  }
  for (int k = 0; k < 3; ++k) {
    double n = 0;
    for (int i = 0; i < 3; ++i) n += U[3 * i + k] * U[3 * i + k];
    n = std::sqrt(n);
    for (int i = 0; i < 3; ++i) U[3 * i + k] = n > 0 ? U[3 * i + k] / n : 0.0;
  }
  for (int r = 0; r < 3; ++r) {
    double R[3];
    for (int col = 0; col < 3; ++col) {
      R[col] = V[3 * r + 0] * U[3 * col + 0] + V[3 * r + 1] * U[3 * col + 1] + V[3 * r + 2] * U[3 * col + 2];
      T12[4 * r + col] = R[col];
    }
    T12[4 * r + 3] = 0;  // filled below once every row of R is known
  }
  for (int r = 0; r < 3; ++r)
    T12[4 * r + 3] = mr[r] - (T12[4 * r + 0] * mo[0] + T12[4 * r + 1] * mo[1] + T12[4 * r + 2] * mo[2]);
}

}  // namespace

extern "C" {

void pfmpe_default_init_params(pfmpe_init_params* p) {
  if (!p) return;
  p->certainty_threshold = 1.0;   // README.md:245, launch file README.md:340
  p->valid_corr_threshold = 0.5;  // README.md:249
  p->n_particles = 0;
  p->max_candidates = 1 << 20;
}

int pfmpe_p3p_histogram(pfmpe_ctx* c, const double* blobs, int B, uint32_t* hist) {
  if (!c) return PFMPE_E_ARG;
  if (!blobs || !hist) return fail(c, PFMPE_E_ARG, "p3p_histogram: null blobs/hist");
  if (!c->has_model) return fail(c, PFMPE_E_STATE, "p3p_histogram: set_model first");
  if (c->M < 3) return fail(c, PFMPE_E_ARG, "p3p_histogram: needs M >= 3 markers");
  if (B < 3) return fail(c, PFMPE_E_ARG, "p3p_histogram: needs B >= 3 blobs");
  if (B > c->max_blobs) return fail(c, PFMPE_E_CAP, "p3p_histogram: B exceeds max_blobs");
  RET(set_device(c));
  c->timing_now = c->timing > 0;
  const size_t ev_mark = c->ev_used;  // pending brackets of earlier frames
  const int rc = run_histogram(c, blobs, B, hist);
  c->timing_now = false;
  if (rc != PFMPE_OK) c->ev_used = ev_mark;  // only this call's brackets are dropped (success harvested them all)
  return rc;
}

int pfmpe_initialise(pfmpe_ctx* c, const double* blobs, int B, const pfmpe_init_params* prm, pfmpe_init_out* out,
                     uint32_t* hist_out) {
  if (!c) return PFMPE_E_ARG;
  if (!out || (B > 0 && !blobs) || B < 0) return fail(c, PFMPE_E_ARG, "initialise: bad arguments");
  if (!c->has_model) return fail(c, PFMPE_E_STATE, "initialise: set_model first");
  if (c->M < 3) return fail(c, PFMPE_E_ARG, "initialise: needs M >= 3 markers");
  if (B > c->max_blobs) return fail(c, PFMPE_E_CAP, "initialise: B exceeds max_blobs");
  pfmpe_init_params p;
  pfmpe_default_init_params(&p);
  if (prm) p = *prm;
  if (p.max_candidates <= 0) p.max_candidates = 1 << 20;
  const int N = p.n_particles > 0 ? p.n_particles : (c->has_prior ? c->N : c->max_particles);
  if (N > c->max_particles) return fail(c, PFMPE_E_CAP, "initialise: n_particles exceeds max_particles");
  std::memset(out, 0, sizeof(*out));
  out->first_match = -1;
  const int M = c->M;
  if (B < M) {  // PE:1507-1512: the PF initialisation needs every marker detected
    out->flag_fail = 10;
    return PFMPE_OK;
  }
  RET(set_device(c));
  std::vector<uint32_t> hist((size_t)B * M);
  c->timing_now = c->timing > 0;
  int rc = run_histogram(c, blobs, B, hist.data());
  if (rc != PFMPE_OK) {
    c->timing_now = false;
    return rc;
  }
  if (hist_out) std::memcpy(hist_out, hist.data(), hist.size() * sizeof(uint32_t));
  uint64_t tot = 0;
  for (uint32_t h : hist) tot += h;
  out->hist_total = tot;
  if (tot == 0) {
    c->timing_now = false;
    out->flag_fail = 12;
    return PFMPE_OK;
  }
  std::vector<std::vector<uint32_t>> cands;
  rc = candidates(c, B, M, hist.data(), p.max_candidates, cands);
  if (rc != PFMPE_OK) {
    c->timing_now = false;
    return rc;
  }
  out->n_candidates = (int)cands.size();
  int flag = cands.empty() ? 11 : -1;

  // ---- stage 3 on the device: every candidate with M rows x every lexicographic 3-subset
  const int ncm = M * (M - 1) * (M - 2) / 6;
  std::vector<int> full;  // indices of candidates with M rows (the others fail with flag 6, no P3P)
  for (size_t i = 0; i < cands.size(); ++i)
    if ((int)cands[i].size() == 2 * M) full.push_back((int)i);
  std::vector<uint8_t> status((size_t)full.size() * ncm);
  std::vector<double> invs((size_t)full.size() * ncm * 12);
  if (!full.empty()) {
    InitArgs ia = make_args(c, B);
    ia.items = (int64_t)full.size() * ncm;
    std::vector<int> ctab((size_t)full.size() * 2 * M);
    for (size_t f = 0; f < full.size(); ++f)
      for (int k = 0; k < 2 * M; ++k) ctab[f * 2 * M + k] = (int)cands[full[f]][k];
    std::vector<int> trip;
    for (int a = 0; a < M; ++a)
      for (int b = a + 1; b < M; ++b)
        for (int d = b + 1; d < M; ++d) trip.push_back(a | (b << 8) | (d << 16));
    Arena ar;
    const size_t o_blobs = ar.take<double>(2 * (size_t)B), o_iv = ar.take<double>(3 * (size_t)B);
    const size_t o_c = ar.take<int>(ctab.size()), o_t = ar.take<int>(trip.size());
    const size_t o_s = ar.take<uint8_t>(status.size()), o_i = ar.take<double>(invs.size());
    rc = ensure_init(c, ar.off);
    if (rc != PFMPE_OK) {
      c->timing_now = false;
      return rc;
    }
    unsigned char* d = c->d_init;
    double* d_blobs = (double*)(d + o_blobs);
    double* d_iv = (double*)(d + o_iv);
    HIPCHK(c, hipMemcpyAsync(d_blobs, blobs, 2 * (size_t)B * sizeof(double), hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(d + o_c, ctab.data(), ctab.size() * sizeof(int), hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(d + o_t, trip.data(), trip.size() * sizeof(int), hipMemcpyHostToDevice, c->stream));
    hipLaunchKernelGGL(k_init_prep, dim3((B + 255) / 256), dim3(256), 0, c->stream, ia, d_blobs, d_iv);
    HIPCHK(c, hipGetLastError());
    const unsigned grid = (unsigned)((ia.items + kInitBlock - 1) / kInitBlock);
    const double ct = p.certainty_threshold;
    RET(launch(c, PFMPE_K_P3P_CHECK, [&] {
      const int nu = M - 3;
      if (nu <= 2)
        hipLaunchKernelGGL((k_p3p_check<2>), dim3(grid), dim3(kInitBlock), 0, c->stream, ia, ct, d_blobs, d_iv,
                           (const int*)(d + o_c), (const int*)(d + o_t), d + o_s, (double*)(d + o_i));
      else if (nu <= 9)
        hipLaunchKernelGGL((k_p3p_check<9>), dim3(grid), dim3(kInitBlock), 0, c->stream, ia, ct, d_blobs, d_iv,
                           (const int*)(d + o_c), (const int*)(d + o_t), d + o_s, (double*)(d + o_i));
      else
        hipLaunchKernelGGL((k_p3p_check<kMaxMarkers - 3>), dim3(grid), dim3(kInitBlock), 0, c->stream, ia, ct,
                           d_blobs, d_iv, (const int*)(d + o_c), (const int*)(d + o_t), d + o_s, (double*)(d + o_i));
    }));
    HIPCHK(c, hipMemcpyAsync(status.data(), d + o_s, status.size(), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(invs.data(), d + o_i, invs.size() * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
  }
  if (c->timing_now) RET(harvest_timing(c));
  c->timing_now = false;

  // ---- the ordered bookkeeping of initialise / checkCorrespondences (PE:1425-1496, 1733-1760)
  std::vector<double> est;  // stored P3P poses in store order (estimate k at slot N - k)
  int n_est = 1, found = 0;
  size_t fi = 0;
  for (size_t ci = 0; ci < cands.size(); ++ci) {
    int valid = 0;
    if ((int)cands[ci].size() < 2 * M) {
      flag = 6;
    } else {
      const size_t base = fi * ncm;
      ++fi;
      double mean_rep[kMaxMarkers][3] = {{0}};
      int num_valid = 0;
      for (int q = 0; q < ncm; ++q) {
        const uint8_t st = status[base + q];
        if (st == 0) {
          flag = 9;
          continue;
        }
        if (st != 2) continue;
        num_valid++;
        const double* inv = &invs[(base + q) * 12];
        if (N >= n_est) {
          est.insert(est.end(), inv, inv + 12);
          n_est++;
        }
        for (int jj = 0; jj < M; ++jj) {
          const double* X = c->markers + 3 * jj;
          for (int r = 0; r < 3; ++r) {
            const double v = inv[4 * r + 0] * X[0] + inv[4 * r + 1] * X[1] + inv[4 * r + 2] * X[2] + inv[4 * r + 3] * 1.0;
            mean_rep[jj][r] = mean_rep[jj][r] + v;
          }
        }
      }
      if ((double)num_valid / ncm >= p.valid_corr_threshold) {
        valid = 1;
        if (n_est < N && out->first_match < 0) {
          double rep[kMaxMarkers * 3];
          for (int jj = 0; jj < M; ++jj)
            for (int r = 0; r < 3; ++r) rep[3 * jj + r] = mean_rep[jj][r] / num_valid;
          compute_transformation(M, c->markers, rep, out->predicted_pose);
          out->first_match = (int)ci;
          out->n_corr = M;
          for (int k = 0; k < 2 * M; ++k) out->corr[k] = cands[ci][k];
        }
      } else {
        flag = num_valid > 0 ? 7 : 8;
      }
    }
    if (valid && n_est < N) found = 1;
  }
  out->found = found;
  out->n_estimates = n_est - 1;
  out->flag_fail = found ? 0 : flag;
  if (!found) return PFMPE_OK;

  // ---- seed the particle set: PoseParticle -> newPoseEstimation_Vec (PE:182-191)
  const int K = n_est - 1;
  RET(ensure_xfer(c));
  {
    Arena ar;
    const size_t o_e = ar.take<double>(est.size());
    RET(ensure_init(c, ar.off));
    HIPCHK(c, hipMemcpyAsync(c->d_init + o_e, est.data(), est.size() * sizeof(double), hipMemcpyHostToDevice,
                             c->stream));
    if (K < N) {  // slot 0 keeps the resident set's slot 0 (identity when there is none)
      if (c->has_prior) {
        RET(export_slot0(c));
      } else {
        static const double I12[12] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0};
        HIPCHK(c, hipMemcpyAsync(c->d_xfer, I12, sizeof(I12), hipMemcpyHostToDevice, c->stream));
      }
    }
    hipLaunchKernelGGL(k_init_seed, dim3((N + 255) / 256), dim3(256), 0, c->stream, (const double*)(c->d_init + o_e),
                       K, N, c->d_xfer);
    HIPCHK(c, hipGetLastError());
    RET(import_xfer(c, N, est.data()));  // anchor (fp16 state): the first stored estimate
  }
  return PFMPE_OK;
}

}  // extern "C"
