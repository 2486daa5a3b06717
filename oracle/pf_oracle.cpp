// =====================================================================================================
//  pf_oracle.cpp — CPU restatement of the reference particle-filter step.
//
//  TEST INFRASTRUCTURE ONLY.  This file is the *checker* for the MI355X engine, never the product:
//  only tests/, __graft_entry__.smoke() and bench.py's `cpu_baseline` leg may load it.  The product
//  library (pf_monocular_pose_estimator_amd/libpfmpe.so) has no link or runtime dependency on it.
//
//  What it restates (all paths relative to /root/reference, "PE" = pf_mpe_lib/src/pose_estimator.cpp):
//    * PF block of PoseEstimator::estimateBodyPose          PE:475-690 (+ reinit branch PE:707-719)
//    * project2d (full K, no distortion, no z>0 cull)        PE:1017-1034
//    * calculateEstimationProbability (literal, with the
//      B x M distance matrix and Eigen minCoeff visitor
//      semantics: column-major traversal, strict '<')       PE:2385-2445
//    * predictPose / exponentialMap / logarithmMap          PE:995-1010, PE:2194-2296
//    * optimisePose (Gauss-Newton, <=500 it, 1e-13 stop)     PE:1805-2009, computeJacobian PE:2163-2192
//    * optimiseAndUpdatePose / updatePose                   PE:2011-2035
//  and the libstdc++ (GCC 11) RNG the reference uses: std::default_random_engine == minstd_rand0
//  (bits/random.h:1555,1604), generate_canonical (bits/random.tcc:3348-3376, two engine outputs per
//  double) and uniform_real_distribution (bits/random.h:1870).  In "reference RNG" mode this oracle
//  instantiates those very library templates, so its draw stream is the reference's by construction.
//
//  It keeps the reference's complexity on purpose (per-particle heap allocations, B x M matrix with
//  min(B,M) full rescans, O(N^2) cumulative-search stratified resampling): bench.py times it as the
//  single-thread CPU baseline ("kind": "port").
//
//  Parity status: PARITY UNPINNED by the reference itself — it ships NO tests, fixtures or golden
//  vectors and cannot be compiled here (Eigen/OpenCV/ROS absent), so no reference
//  output exists to check against.  This restatement is instead pinned by known-answer tests derived
//  from the reference source (tests/test_oracle_kat.py: likelihood closed forms, libstdc++ RNG stream,
//  Philox4x32-10 published vectors) and frozen as golden fixtures (tests/golden/, make_golden.py).  Summation order of 4x4 products is sequential k=0..3 (Eigen's packet order is unverifiable
//  here); differences are at the ulp level.
//
//  Build: oracle/Makefile  (g++ -O2 -ffp-contract=off, no -march=native: no FMA contraction, so the
//  fp64 arithmetic is plain IEEE mul/add like the reference's x86-64 build).
// =====================================================================================================
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <random>
#include <vector>

namespace {

// ----------------------------------------------------------------------------- 4x4 row-major matrices
struct Mat4 {
  double a[16];
  double& operator()(int i, int j) { return a[i * 4 + j]; }
  double operator()(int i, int j) const { return a[i * 4 + j]; }
};

Mat4 identity4() {
  Mat4 m;
  std::memset(m.a, 0, sizeof(m.a));
  m(0, 0) = m(1, 1) = m(2, 2) = m(3, 3) = 1.0;
  return m;
}

// 3x4 row-major [R|t] (12 doubles) <-> homogeneous 4x4
Mat4 from12(const double* p) {
  Mat4 m = identity4();
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 4; ++j) m(i, j) = p[i * 4 + j];
  return m;
}
void to12(const Mat4& m, double* p) {
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 4; ++j) p[i * 4 + j] = m(i, j);
}

// Full 4x4 product, k summed sequentially 0..3 (the reference multiplies full 4x4 Eigen matrices).
Mat4 mul(const Mat4& A, const Mat4& B) {
  Mat4 C;
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j) {
      double s = A(i, 0) * B(0, j);
      s = s + A(i, 1) * B(1, j);
      s = s + A(i, 2) * B(2, j);
      s = s + A(i, 3) * B(3, j);
      C(i, j) = s;
    }
  return C;
}

Mat4 inverse_rigid(const Mat4& T) {  // T^-1 for [R|t] (previous_pose_.inverse(), PE:1000)
  Mat4 I = identity4();
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) I(i, j) = T(j, i);
  for (int i = 0; i < 3; ++i) I(i, 3) = -(I(i, 0) * T(0, 3) + I(i, 1) * T(1, 3) + I(i, 2) * T(2, 3));
  return I;
}

// ----------------------------------------------------------------------------- project2d  (PE:1017)
// temp = (K34 * T) * X ;  temp /= temp(2) ; return head<2>
void project2d(const double* K, const Mat4& T, const double X[3], double out[2]) {
  double K34[12];
  for (int i = 0; i < 3; ++i) {
    for (int j = 0; j < 3; ++j) K34[i * 4 + j] = K[i * 3 + j];
    K34[i * 4 + 3] = 0.0;
  }
  double Q[12];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 4; ++j) {
      double s = K34[i * 4 + 0] * T(0, j);
      s = s + K34[i * 4 + 1] * T(1, j);
      s = s + K34[i * 4 + 2] * T(2, j);
      s = s + K34[i * 4 + 3] * T(3, j);
      Q[i * 4 + j] = s;
    }
  double p[3];
  for (int i = 0; i < 3; ++i) {
    double s = Q[i * 4 + 0] * X[0];
    s = s + Q[i * 4 + 1] * X[1];
    s = s + Q[i * 4 + 2] * X[2];
    s = s + Q[i * 4 + 3] * 1.0;
    p[i] = s;
  }
  const double z = p[2];
  out[0] = p[0] / z;
  out[1] = p[1] / z;
}

// -------------------------------------------------- calculateEstimationProbability (PE:2385-2445)
// Literal form: B x M distance matrix (column-major, like Eigen's MatrixXYd), min(B,M) rescans with
// Eigen's minCoeff visitor (init at (0,0), then column-major, strict '<'), break at tol_PF, score uses
// `tol` (back_projection_pixel_tolerance_, NOT tol_PF), self-occlusion penalty 3*s, downgrade -2,
// and only the winning COLUMN is blanked (blobs may be reused).
double likelihood_literal(int M, int B, const double* proj /*M x 2*/, const double* blobs /*B x 2*/,
                          double tol, double tol_pf, const uint8_t* downgrade,
                          std::vector<unsigned>& pairs /* out: 2*n (LED, blob), 1-based */) {
  double Probability = 0;
  std::vector<double> distances((size_t)B * M);  // column-major: (i,j) at j*B + i
  for (int i = 0; i < B; ++i)
    for (int j = 0; j < M; ++j) {
      const double dx = blobs[2 * i] - proj[2 * j];
      const double dy = blobs[2 * i + 1] - proj[2 * j + 1];
      distances[(size_t)j * B + i] = dx * dx + dy * dy;
    }
  int numSelfocclusion = 1;
  std::vector<unsigned> usedDetections;
  pairs.clear();
  const int kmax = std::min(B, M);
  for (int k = 0; k < kmax; ++k) {
    // Eigen DenseBase::minCoeff(&row,&col): visitor.init(coeff(0,0)); then every other coeff in
    // storage (column-major) order with `value < res`.
    double minv = distances[0];
    int row = 0, col = 0;
    for (int j = 0; j < M; ++j)
      for (int i = (j == 0 ? 1 : 0); i < B; ++i) {
        const double v = distances[(size_t)j * B + i];
        if (v < minv) { minv = v; row = i; col = j; }
      }
    const double min_value = std::sqrt(minv);
    if (min_value <= tol_pf) {
      const double r = (tol - min_value) / tol;
      Probability += (double)M + std::pow(r, 2);
      pairs.push_back((unsigned)col + 1);
      pairs.push_back((unsigned)row + 1);
      if (std::any_of(usedDetections.begin(), usedDetections.end(),
                      [row](unsigned u) { return u == (unsigned)row; })) {
        Probability = Probability - numSelfocclusion * 3;
        numSelfocclusion++;
      }
      usedDetections.push_back((unsigned)row);
      if (downgrade && downgrade[col]) Probability = Probability - 2;
      for (int i = 0; i < B; ++i) distances[(size_t)col * B + i] = INFINITY;
    } else {
      break;
    }
  }
  return Probability;
}

// Closed form of the same function: columns are independent, so the extraction
// order is the ascending (column-min, column) order.  Used only to cross-check the literal form.
double likelihood_closed(int M, int B, const double* proj, const double* blobs, double tol,
                         double tol_pf, const uint8_t* downgrade, std::vector<unsigned>& pairs) {
  pairs.clear();
  if (B == 0 || M == 0) return 0.0;
  {
    const double dx = blobs[0] - proj[0], dy = blobs[1] - proj[1];
    if (std::isnan(dx * dx + dy * dy)) return 0.0;  // Eigen visitor seeded with a NaN (0,0)
  }
  std::vector<double> m(M);
  std::vector<int> r(M);
  for (int j = 0; j < M; ++j) {
    double best = INFINITY;
    int arg = 0;
    for (int i = 0; i < B; ++i) {
      const double dx = blobs[2 * i] - proj[2 * j], dy = blobs[2 * i + 1] - proj[2 * j + 1];
      const double d = dx * dx + dy * dy;
      if (d < best) { best = d; arg = i; }
    }
    m[j] = best;
    r[j] = arg;
  }
  std::vector<int> order(M);
  for (int j = 0; j < M; ++j) order[j] = j;
  std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return m[a] < m[b]; });
  double P = 0;
  int s = 1;
  std::vector<int> used;
  const int kmax = std::min(B, M);
  for (int k = 0; k < kmax; ++k) {
    const int j = order[k];
    const double d = std::sqrt(m[j]);
    if (!(d <= tol_pf)) break;
    const double q = (tol - d) / tol;
    P += (double)M + q * q;
    pairs.push_back((unsigned)j + 1);
    pairs.push_back((unsigned)r[j] + 1);
    if (std::find(used.begin(), used.end(), r[j]) != used.end()) { P = P - s * 3; s++; }
    used.push_back(r[j]);
    if (downgrade && downgrade[j]) P = P - 2;
  }
  return P;
}

// ------------------------------------------------------------------------------------- Philox4x32-10
// Salmon, Moraes, Dror, Shaw, "Parallel random numbers: as easy as 1, 2, 3" (SC'11); constants as in
// the published Random123 specification.
inline void philox4x32_10(const uint32_t ctr_in[4], const uint32_t key_in[2], uint32_t out[4]) {
  uint32_t c0 = ctr_in[0], c1 = ctr_in[1], c2 = ctr_in[2], c3 = ctr_in[3];
  uint32_t k0 = key_in[0], k1 = key_in[1];
  for (int r = 0; r < 10; ++r) {
    if (r) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    const uint32_t n0 = hi1 ^ c1 ^ k0, n1 = lo1, n2 = hi0 ^ c3 ^ k1, n3 = lo0;
    c0 = n0; c1 = n1; c2 = n2; c3 = n3;
  }
  out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

// Counter layout shared with the HIP engine (DESIGN.md "RNG"):
//   motion   ctr = {n, iter | 0<<24, frame_lo, frame_hi} -> six 21-bit uniforms (a,b,c,tx,ty,tz)
//   resample ctr = {k, 2<<24,        frame_lo, frame_hi} -> one 53-bit uniform
//   key      = {seed_lo, seed_hi}
inline double u21(uint32_t v) { return (double)v * (1.0 / 2097152.0); }
inline double u53(uint32_t x0, uint32_t x1) {
  return ((double)(x0 >> 5) * 67108864.0 + (double)(x1 >> 6)) * (1.0 / 9007199254740992.0);
}

enum { RNG_REFERENCE = 0, RNG_PHILOX = 1 };

}  // namespace

// ======================================================================================= C interface
extern "C" {

typedef struct {
  double tol;        // back_projection_pixel_tolerance_   (score normaliser, PE:2416)
  double tol_pf;     // back_projection_pixel_tolerance_PF (acceptance gate, PE:2414)
  double ang_min, ang_max;      // minAngularNoise / maxAngularNoise (rad)
  double trans_min, trans_max;  // minTransitionNoise / maxTransitionNoise (m)
  double growth;     // 0.025 noise growth per 10 iterations (PE:563)
  int max_iter;      // 80 (PE:616)
  int exit_cap;      // 5  (PE:616  M*min(5,numLED))
  int accept_cap;    // 3  (PE:633  M*min(3,numLED))
  int rng_mode;      // 0 reference (minstd_rand0 + generate_canonical), 1 Philox4x32-10
  int fast_search;   // test speed only: 1 = the cumulative search of PE:674-679 by binary search over the
                     // running max of the SAME sequential cumulative sums (first i with c_i >= r equals the
                     // first i with max(c_0..c_i) >= r), identical counts/indices; 0 = the reference's O(N^2)
                     // scan (the cpu_baseline timing keeps 0)
} orc_params;

typedef struct {
  double current_pose[12];    // current_pose_          (particle 0, PE:547)
  double predicted_pose[12];  // camMoveInv*predicted_pose_ (particle 1, PE:395/551)
  double prediction[12];      // predictionMatrix       (PE:234, 556)
  double cam_move_inv[12];    // camMoveInv             (PE:241-393)
  const double* blobs;        // B x 2 undistorted pixel coordinates (image_points_)
  int B;                      // numLED (PE:449)
  int it_since_init;          // it_since_initialized_
  double dt;                  // predicted_time_ - current_time_ (PE:499)
  uint64_t seed;              // replaces std::random_device (PE:476)
  uint64_t frame_idx;         // Philox counter word
  int force_iters;            // 0 = reference exit rule; >0 run exactly this many iterations
} orc_frame_in;

typedef struct {
  int iters;            // iterations executed (k)
  int kept_iter;        // iteration whose particle set was kept (PE:608-624)
  int most_likely_idx;  // mostLikelyParticleIdx (PE:610 / PE:714)
  int accepted;         // PE:633 condition
  int resampled;        // resampling executed (PE:666)
  int winner_idx;       // argmax resample count (PE:686)
  int n_corr;           // rows of correspondences_ of the winner
  int flag_fail;        // 1 accepted (PE:635), 4 re-init (PE:711)
  double highest_prob;  // highestProb
  double prob_sum;      // probPartSum before normalisation (PE:627)
  double winner_pose[12];       // PoseParticle[winner] (PE:687) ; on reinit PoseParticle[most likely]
  double most_likely_pose[12];  // PoseParticle[most_likely_idx]
  unsigned corr[64];            // (LED, blob) 1-based pairs of the winner, up to 32 rows
} orc_frame_out;

double orc_likelihood(int M, int B, const double* proj, const double* blobs, double tol, double tol_pf,
                      const uint8_t* downgrade, unsigned* pairs_out, int* npairs_out) {
  std::vector<unsigned> pairs;
  const double P = likelihood_literal(M, B, proj, blobs, tol, tol_pf, downgrade, pairs);
  if (pairs_out) std::copy(pairs.begin(), pairs.end(), pairs_out);
  if (npairs_out) *npairs_out = (int)pairs.size() / 2;
  return P;
}

double orc_likelihood_closed(int M, int B, const double* proj, const double* blobs, double tol,
                             double tol_pf, const uint8_t* downgrade, unsigned* pairs_out,
                             int* npairs_out) {
  std::vector<unsigned> pairs;
  const double P = likelihood_closed(M, B, proj, blobs, tol, tol_pf, downgrade, pairs);
  if (pairs_out) std::copy(pairs.begin(), pairs.end(), pairs_out);
  if (npairs_out) *npairs_out = (int)pairs.size() / 2;
  return P;
}

void orc_project(const double* K, const double* pose12, const double* X, double* uv) {
  project2d(K, from12(pose12), X, uv);
}

void orc_philox4x32_10(const uint32_t* ctr, const uint32_t* key, uint32_t* out) {
  philox4x32_10(ctr, key, out);
}

// n raw outputs of std::default_random_engine seeded with `seed` (reference RNG KAT).
void orc_minstd_outputs(uint32_t seed, int n, uint32_t* out) {
  std::default_random_engine g(seed);
  for (int i = 0; i < n; ++i) out[i] = (uint32_t)g();
}

// n successive uniform_real_distribution<double>(a,b) draws from one engine seeded with `seed`.
void orc_uniform_draws(uint32_t seed, double a, double b, int n, double* out) {
  std::default_random_engine g(seed);
  std::uniform_real_distribution<double> d(a, b);
  for (int i = 0; i < n; ++i) out[i] = d(g);
}

// ----------------------------------------------------------------------------- the PF step (PE:475)
int orc_pf_step(int N, int M, const double* markers /*M x 3*/, const double* K /*3x3 row-major*/,
                const uint8_t* downgrade /*M or NULL*/, const orc_params* prm,
                const orc_frame_in* in, const double* prior /*N x 12 = newPoseEstimation*/,
                orc_frame_out* out,
                double* propagated_out /*N x 12 kept PoseParticle, may be NULL*/,
                double* weights_out /*N raw kept probPart (before normalisation), may be NULL*/,
                double* resampled_out /*N x 12 new prior (only if resampled), may be NULL*/,
                int* resample_idx_out /*N, may be NULL*/, unsigned* counts_out /*N, may be NULL*/) {
  if (N < 1 || M < 1 || !prm || !in || !out || !prior || !markers || !K) return -1;
  const int B = in->B;
  const int numLED = B;
  std::memset(out, 0, sizeof(*out));

  const Mat4 current_pose = from12(in->current_pose);
  const Mat4 predicted_pose = from12(in->predicted_pose);
  const Mat4 predictionMatrix = from12(in->prediction);
  const Mat4 camMoveInv = from12(in->cam_move_inv);
  std::vector<Mat4> newPoseEstimation(N);
  for (int n = 0; n < N; ++n) newPoseEstimation[n] = from12(prior + 12 * (size_t)n);
  std::vector<Mat4> PoseParticle(N, current_pose);

  // ---- parameter initialisation (PE:475-531)
  std::default_random_engine generator((uint32_t)in->seed);
  double facTransX, facTransY, facTransZ, facRotX, facRotY, facRotZ;
  if (in->it_since_init == 1) {
    facTransX = facTransY = facTransZ = 1;
    facRotX = facRotY = facRotZ = 1;
  } else {
    const double timeDiffFrames = in->dt;
    // NB: all three translation factors use predictionMatrix(0,3) (PE:500-502)
    facTransX = std::min(std::max(0.2, std::abs(predictionMatrix(0, 3)) / timeDiffFrames), 1.0) / 4;
    facTransY = std::min(std::max(0.2, std::abs(predictionMatrix(0, 3)) / timeDiffFrames), 1.0) / 4;
    facTransZ = std::min(std::max(0.2, std::abs(predictionMatrix(0, 3)) / timeDiffFrames), 1.0) / 4;
    facRotX = facRotY = facRotZ = 0.2;
  }
  std::uniform_real_distribution<double> randTransX(prm->trans_min * facTransX, prm->trans_max * facTransX);
  std::uniform_real_distribution<double> randTransY(prm->trans_min * facTransY, prm->trans_max * facTransY);
  std::uniform_real_distribution<double> randTransZ(prm->trans_min * facTransZ, prm->trans_max * facTransZ);
  std::uniform_real_distribution<double> randAngleX(prm->ang_min * facRotX, prm->ang_max * facRotX);
  std::uniform_real_distribution<double> randAngleY(prm->ang_min * facRotY, prm->ang_max * facRotY);
  std::uniform_real_distribution<double> randAngleZ(prm->ang_min * facRotZ, prm->ang_max * facRotZ);
  // Philox mode uses the same affine map u*(b-a)+a (bits/random.h:1870) on counter-based uniforms
  const double lo[6] = {randAngleX.a(), randAngleY.a(), randAngleZ.a(), randTransX.a(), randTransY.a(), randTransZ.a()};
  const double hi[6] = {randAngleX.b(), randAngleY.b(), randAngleZ.b(), randTransX.b(), randTransY.b(), randTransZ.b()};
  const uint32_t key[2] = {(uint32_t)in->seed, (uint32_t)(in->seed >> 32)};
  const uint32_t flo = (uint32_t)in->frame_idx, fhi = (uint32_t)(in->frame_idx >> 32);

  int Particle_index = N - 1;  // reference leaves it uninitialised (UB) if the first draw finds nothing
  double probPartSum = 0;
  double highestProb = 0;
  std::vector<double> probPart(N, 0.0);
  const int N_Resamples = N;
  std::vector<unsigned> counterMeas(N, 0);
  std::vector<std::vector<unsigned>> correspondencesVec;
  int iter = 0;
  std::vector<Mat4> PoseParticle_likely;
  std::vector<std::vector<unsigned>> correspondencesVec_likely;
  std::vector<double> probPart_likely = probPart;
  int mostLikelyParticleIdx = 0;
  int kept_iter = -1;
  Mat4 PoseParticle_temp;
  const double exit_thr = (double)((size_t)M * (size_t)std::min(prm->exit_cap, numLED));
  const double accept_thr = (double)((size_t)M * (size_t)std::min(prm->accept_cap, numLED));
  std::vector<double> proj(2 * (size_t)M);

  // fast_search (test speed only) with the Philox stream also spreads the per-particle loop over OpenMP threads:
  // each particle's draws, pose and likelihood depend on nothing but its own index, every result lands in its own
  // slot, and the sums below stay sequential, so the outputs are bit-identical to the one-thread loop.  The
  // reference stream (one sequential engine) and the cpu_baseline timing (fast_search = 0) stay one thread.
  const bool threaded = prm->fast_search && prm->rng_mode != RNG_REFERENCE;
  do {
    correspondencesVec.assign((size_t)N, std::vector<unsigned>());
    const double g = 1 + prm->growth * std::floor(iter / 10);
#pragma omp parallel for schedule(static, 4096) if (threaded) firstprivate(PoseParticle_temp, proj)
    for (int n = 0; n < N; ++n) {
      if (n == 0) {
        PoseParticle[n] = current_pose;
      } else if (n == 1) {
        PoseParticle[n] = predicted_pose;
      } else {
        if (in->it_since_init > 1 && (iter % 10) != 0)
          PoseParticle_temp = mul(mul(camMoveInv, newPoseEstimation[n]), predictionMatrix);
        else if (in->it_since_init > 1)
          PoseParticle_temp = mul(camMoveInv, newPoseEstimation[n]);
        else
          PoseParticle_temp = newPoseEstimation[n];

        double dr[6];
        if (prm->rng_mode == RNG_REFERENCE) {
          dr[0] = randAngleX(generator);
          dr[1] = randAngleY(generator);
          dr[2] = randAngleZ(generator);
        } else {
          // one Philox call -> six 21-bit uniforms (top 21 bits of each word, then two from the low bits)
          uint32_t ca[4] = {(uint32_t)n, (uint32_t)iter | (0u << 24), flo, fhi}, o[4];
          philox4x32_10(ca, key, o);
          const uint32_t v[6] = {o[0] >> 11, o[1] >> 11, o[2] >> 11, o[3] >> 11,
                                 ((o[0] & 0x7FFu) << 10) | (o[1] & 0x3FFu), ((o[2] & 0x7FFu) << 10) | (o[3] & 0x3FFu)};
          for (int q = 0; q < 6; ++q) dr[q] = u21(v[q]) * (hi[q] - lo[q]) + lo[q];
        }
        const double a = dr[0] * g;
        const double b = dr[1] * g;
        const double c = dr[2] * g;
        Mat4 rotX = identity4(), rotY = identity4(), rotZ = identity4();
        rotX(1, 1) = std::cos(a); rotX(1, 2) = -std::sin(a); rotX(2, 1) = std::sin(a); rotX(2, 2) = std::cos(a);
        rotY(0, 0) = std::cos(b); rotY(0, 2) = std::sin(b); rotY(2, 0) = -std::sin(b); rotY(2, 2) = std::cos(b);
        rotZ(0, 0) = std::cos(c); rotZ(0, 1) = -std::sin(c); rotZ(1, 0) = std::sin(c); rotZ(1, 1) = std::cos(c);
        PoseParticle[n] = mul(mul(mul(PoseParticle_temp, rotZ), rotY), rotX);
        if (prm->rng_mode == RNG_REFERENCE) {
          dr[3] = randTransX(generator);
          dr[4] = randTransY(generator);
          dr[5] = randTransZ(generator);
        }
        PoseParticle[n](0, 3) = PoseParticle_temp(0, 3) + dr[3] * g;
        PoseParticle[n](1, 3) = PoseParticle_temp(1, 3) + dr[4] * g;
        PoseParticle[n](2, 3) = PoseParticle_temp(2, 3) + dr[5] * g;
      }
      for (int j = 0; j < M; ++j) project2d(K, PoseParticle[n], markers + 3 * j, &proj[2 * j]);
      std::vector<unsigned> pairs;
      probPart[n] = likelihood_literal(M, B, proj.data(), in->blobs, prm->tol, prm->tol_pf, downgrade, pairs);
      correspondencesVec[(size_t)n] = std::move(pairs);
    }
    iter++;
    // probPart.maxCoeff(&idx): first maximum
    int amax = 0;
    for (int n = 1; n < N; ++n)
      if (probPart[n] > probPart[amax]) amax = n;
    const double maxw = probPart[amax];
    if (maxw > highestProb) {
      highestProb = maxw;
      mostLikelyParticleIdx = amax;
      correspondencesVec_likely = correspondencesVec;
      PoseParticle_likely = PoseParticle;
      probPart_likely = probPart;
      kept_iter = iter - 1;
    }
    const bool go_on = in->force_iters > 0 ? (iter < in->force_iters)
                                           : (iter < prm->max_iter && maxw < exit_thr);
    if (!go_on) break;
  } while (true);

  if (PoseParticle_likely.size() != 0) {
    PoseParticle = PoseParticle_likely;
    correspondencesVec = correspondencesVec_likely;
    probPart = probPart_likely;
  } else {
    kept_iter = iter - 1;
  }
  out->iters = iter;
  out->kept_iter = kept_iter;
  if (weights_out) std::copy(probPart.begin(), probPart.end(), weights_out);
  if (propagated_out)
    for (int n = 0; n < N; ++n) to12(PoseParticle[n], propagated_out + 12 * (size_t)n);

  // ---- normalise (PE:627-629): sequential fp64 sum
  probPartSum = 0;
  for (int n = 0; n < N; ++n) probPartSum += probPart[n];
  out->prob_sum = probPartSum;
  if (probPartSum != 0)
    for (int n = 0; n < N; ++n) probPart[n] = probPart[n] / probPartSum;
  out->highest_prob = highestProb;

  int winner = -1;
  if (probPartSum != 0 && highestProb > accept_thr) {
    out->accepted = 1;
    out->flag_fail = 1;
    // PE:637 inner branch is unreachable (2/3*numLED == 0); uncertainty = 1; resample (PE:666)
    std::vector<double> runmax;  // fast_search: running max of the scan's own sequential sums
    if (prm->fast_search) {
      runmax.resize(N);
      double c = 0, r = -INFINITY;
      for (int i = 0; i < N; ++i) {
        c += probPart[i];
        r = c > r ? c : r;
        runmax[i] = r;
      }
    }
    for (int numResamples = 0; numResamples < N_Resamples; numResamples++) {
      double u;
      if (prm->rng_mode == RNG_REFERENCE) {
        std::uniform_real_distribution<double> randResample(0, 1);
        u = randResample(generator);
      } else {
        uint32_t cr[4] = {(uint32_t)numResamples, 2u << 24, flo, fhi}, o[4];
        philox4x32_10(cr, key, o);
        u = u53(o[0], o[1]);
      }
      const double randVar = (numResamples + u) / N_Resamples;
      if (prm->fast_search) {
        const auto it = std::lower_bound(runmax.begin(), runmax.end(), randVar);  // first runmax_i >= randVar
        if (it != runmax.end()) {
          Particle_index = (int)(it - runmax.begin());
          counterMeas[Particle_index]++;
        }
      } else {
        probPartSum = 0;
        for (int idxParticle = 0; idxParticle < N; idxParticle++) {
          probPartSum += probPart[idxParticle];
          if (probPartSum >= randVar) {
            Particle_index = idxParticle;
            counterMeas[idxParticle]++;
            break;
          }
        }
      }
      if (resample_idx_out) resample_idx_out[numResamples] = Particle_index;
      newPoseEstimation[numResamples] = PoseParticle[Particle_index];
    }
    out->resampled = 1;
    winner = 0;
    for (int n = 1; n < N; ++n)
      if (counterMeas[n] > counterMeas[winner]) winner = n;
    out->winner_idx = winner;
    out->most_likely_idx = mostLikelyParticleIdx;
    to12(PoseParticle[winner], out->winner_pose);
    const std::vector<unsigned>& c = correspondencesVec[winner];
    out->n_corr = (int)c.size() / 2;
    for (size_t q = 0; q < c.size() && q < 64; ++q) out->corr[q] = c[q];
    if (resampled_out)
      for (int n = 0; n < N; ++n) to12(newPoseEstimation[n], resampled_out + 12 * (size_t)n);
  } else {
    // re-init branch (PE:707-719): argmax of the (normalised) kept weights
    out->flag_fail = 4;
    int amax = 0;
    for (int n = 1; n < N; ++n)
      if (probPart[n] > probPart[amax]) amax = n;
    mostLikelyParticleIdx = amax;
    out->most_likely_idx = amax;
    out->winner_idx = -1;
    to12(PoseParticle[amax], out->winner_pose);
  }
  to12(PoseParticle[out->most_likely_idx], out->most_likely_pose);
  if (counts_out) std::copy(counterMeas.begin(), counterMeas.end(), counts_out);
  return 0;
}

// Stratified resampling alone (PE:627-682) on given raw weights: normalise (sequential fp64 sum), draw
// U_k from the stream position the PF block leaves it at (reference mode: after 12*(N-2)*iters engine
// outputs; Philox: resample counters), first-i cumulative search.  Used to check the GPU resampler on
// the GPU's own fp32 weights.  Returns 0 if resampled, 1 if the sum is zero.
// Particles idx[s] of PF iteration `iter` alone (Philox stream only), each from its prior pose prior[s] (12
// doubles): the propagated pose (PE:543-588, exactly orc_pf_step's motion model with the same draw ranges) and the
// literal likelihood (PE:2385-2445).  Philox draws depend only on (particle, iteration, frame, seed), so a sample of
// a large frame is checked without running the whole frame (tests/test_gpu_packed_oracle.py: the production
// two-launch packed pass at C4 / C5 sizes against this restatement).  Returns -1 for the reference stream (its
// draws are addressed through N), 0 otherwise.
int orc_pf_sample(int n_samples, const int* idx, int M, const double* markers, const double* K,
                  const uint8_t* downgrade, const orc_params* prm, const orc_frame_in* in, int iter,
                  const double* prior /*n_samples x 12*/, double* prop_out /*n_samples x 12*/,
                  double* w_out /*n_samples*/) {
  if (!prm || !in || prm->rng_mode != RNG_PHILOX || n_samples < 0 || M < 1) return -1;
  const Mat4 current_pose = from12(in->current_pose);
  const Mat4 predicted_pose = from12(in->predicted_pose);
  const Mat4 predictionMatrix = from12(in->prediction);
  const Mat4 camMoveInv = from12(in->cam_move_inv);
  double facTrans, facRot;  // PE:488-505 (all three translation factors from predictionMatrix(0,3))
  if (in->it_since_init == 1) {
    facTrans = facRot = 1;
  } else {
    facTrans = std::min(std::max(0.2, std::abs(predictionMatrix(0, 3)) / in->dt), 1.0) / 4;
    facRot = 0.2;
  }
  std::uniform_real_distribution<double> randTrans(prm->trans_min * facTrans, prm->trans_max * facTrans);
  std::uniform_real_distribution<double> randAngle(prm->ang_min * facRot, prm->ang_max * facRot);
  const double lo[6] = {randAngle.a(), randAngle.a(), randAngle.a(), randTrans.a(), randTrans.a(), randTrans.a()};
  const double hi[6] = {randAngle.b(), randAngle.b(), randAngle.b(), randTrans.b(), randTrans.b(), randTrans.b()};
  const uint32_t key[2] = {(uint32_t)in->seed, (uint32_t)(in->seed >> 32)};
  const uint32_t flo = (uint32_t)in->frame_idx, fhi = (uint32_t)(in->frame_idx >> 32);
  const double g = 1 + prm->growth * std::floor(iter / 10);
  std::vector<double> proj(2 * (size_t)M);
  for (int s = 0; s < n_samples; ++s) {
    const int n = idx[s];
    Mat4 P;
    if (n == 0) {
      P = current_pose;
    } else if (n == 1) {
      P = predicted_pose;
    } else {
      const Mat4 prior_n = from12(prior + 12 * (size_t)s);
      Mat4 temp;
      if (in->it_since_init > 1 && (iter % 10) != 0)
        temp = mul(mul(camMoveInv, prior_n), predictionMatrix);
      else if (in->it_since_init > 1)
        temp = mul(camMoveInv, prior_n);
      else
        temp = prior_n;
      uint32_t ca[4] = {(uint32_t)n, (uint32_t)iter | (0u << 24), flo, fhi}, o[4];
      philox4x32_10(ca, key, o);
      const uint32_t v[6] = {o[0] >> 11, o[1] >> 11, o[2] >> 11, o[3] >> 11,
                             ((o[0] & 0x7FFu) << 10) | (o[1] & 0x3FFu), ((o[2] & 0x7FFu) << 10) | (o[3] & 0x3FFu)};
      double dr[6];
      for (int q = 0; q < 6; ++q) dr[q] = u21(v[q]) * (hi[q] - lo[q]) + lo[q];
      const double a = dr[0] * g, b = dr[1] * g, c = dr[2] * g;
      Mat4 rotX = identity4(), rotY = identity4(), rotZ = identity4();
      rotX(1, 1) = std::cos(a); rotX(1, 2) = -std::sin(a); rotX(2, 1) = std::sin(a); rotX(2, 2) = std::cos(a);
      rotY(0, 0) = std::cos(b); rotY(0, 2) = std::sin(b); rotY(2, 0) = -std::sin(b); rotY(2, 2) = std::cos(b);
      rotZ(0, 0) = std::cos(c); rotZ(0, 1) = -std::sin(c); rotZ(1, 0) = std::sin(c); rotZ(1, 1) = std::cos(c);
      P = mul(mul(mul(temp, rotZ), rotY), rotX);
      P(0, 3) = temp(0, 3) + dr[3] * g;
      P(1, 3) = temp(1, 3) + dr[4] * g;
      P(2, 3) = temp(2, 3) + dr[5] * g;
    }
    to12(P, prop_out + 12 * (size_t)s);
    for (int j = 0; j < M; ++j) project2d(K, P, markers + 3 * j, &proj[2 * j]);
    std::vector<unsigned> pairs;
    w_out[s] = likelihood_literal(M, in->B, proj.data(), in->blobs, prm->tol, prm->tol_pf, downgrade, pairs);
  }
  return 0;
}

int orc_stratified_resample(int N, const double* raw_weights, int rng_mode, uint64_t seed, uint64_t frame_idx,
                            int iters, unsigned* counts_out, int* idx_out) {
  std::vector<double> w(raw_weights, raw_weights + N);
  double S = 0;
  for (int n = 0; n < N; ++n) S += w[n];
  std::fill(counts_out, counts_out + N, 0u);
  if (S == 0) return 1;
  for (int n = 0; n < N; ++n) w[n] = w[n] / S;
  std::default_random_engine generator((uint32_t)seed);
  if (rng_mode == RNG_REFERENCE && N > 2) generator.discard((unsigned long long)12 * (N - 2) * (unsigned long long)iters);
  const uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
  const uint32_t flo = (uint32_t)frame_idx, fhi = (uint32_t)(frame_idx >> 32);
  int Particle_index = N - 1;
  for (int k = 0; k < N; ++k) {
    double u;
    if (rng_mode == RNG_REFERENCE) {
      std::uniform_real_distribution<double> randResample(0, 1);
      u = randResample(generator);
    } else {
      uint32_t cr[4] = {(uint32_t)k, 2u << 24, flo, fhi}, o[4];
      philox4x32_10(cr, key, o);
      u = u53(o[0], o[1]);
    }
    const double randVar = (k + u) / N;
    double c = 0;
    for (int i = 0; i < N; ++i) {
      c += w[i];
      if (c >= randVar) { Particle_index = i; counts_out[i]++; break; }
    }
    if (idx_out) idx_out[k] = Particle_index;
  }
  return 0;
}

// --------------------------------------------------------------- SE(3) maps (PE:2194-2303)
static void skew(const double w[3], double O[9]) {
  O[0] = 0; O[1] = -w[2]; O[2] = w[1];
  O[3] = w[2]; O[4] = 0; O[5] = -w[0];
  O[6] = -w[1]; O[7] = w[0]; O[8] = 0;
}
static void mm3(const double* A, const double* B, double* C) {
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) C[i * 3 + j] = A[i * 3] * B[j] + A[i * 3 + 1] * B[3 + j] + A[i * 3 + 2] * B[6 + j];
}

void orc_exp_map(const double* twist /*6: upsilon, omega*/, double* pose12) {
  const double* ups = twist;
  const double* om = twist + 3;
  const double theta = std::sqrt(om[0] * om[0] + om[1] * om[1] + om[2] * om[2]);
  const double th2 = theta * theta;
  double O[9], O2[9], R[9], V[9];
  skew(om, O);
  mm3(O, O, O2);
  for (int i = 0; i < 9; ++i) { R[i] = (i % 4 == 0) ? 1.0 : 0.0; V[i] = R[i]; }
  if (theta != 0) {
    const double s = std::sin(theta), c = std::cos(theta);
    for (int i = 0; i < 9; ++i) {
      const double I = (i % 4 == 0) ? 1.0 : 0.0;
      R[i] = I + O[i] / theta * s + O2[i] / th2 * (1 - c);
      V[i] = I + (1 - c) / th2 * O[i] + (theta - s) / (th2 * theta) * O2[i];
    }
  }
  for (int i = 0; i < 3; ++i) {
    for (int j = 0; j < 3; ++j) pose12[i * 4 + j] = R[i * 3 + j];
    pose12[i * 4 + 3] = V[i * 3] * ups[0] + V[i * 3 + 1] * ups[1] + V[i * 3 + 2] * ups[2];
  }
}

void orc_log_map(const double* pose12, double* twist) {
  double R[9], t[3];
  for (int i = 0; i < 3; ++i) {
    for (int j = 0; j < 3; ++j) R[i * 3 + j] = pose12[i * 4 + j];
    t[i] = pose12[i * 4 + 3];
  }
  double w_hat[9] = {0};
  // R.isApprox(I, 1e-10): ||R - I||_F <= 1e-10 * min(||R||_F, ||I||_F)
  double dn = 0, rn = 0;
  for (int i = 0; i < 9; ++i) {
    const double I = (i % 4 == 0) ? 1.0 : 0.0;
    dn += (R[i] - I) * (R[i] - I);
    rn += R[i] * R[i];
  }
  const bool isI = std::sqrt(dn) <= 1e-10 * std::min(std::sqrt(rn), std::sqrt(3.0));
  if (!isI) {
    double temp = (R[0] + R[4] + R[8] - 1) / 2;
    if (temp > 1) temp = 1; else if (temp < -1) temp = -1;
    const double phi = std::acos(temp);
    if (phi != 0)
      for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) w_hat[i * 3 + j] = (R[i * 3 + j] - R[j * 3 + i]) / (2 * std::sin(phi)) * phi;
  }
  const double w[3] = {w_hat[7], w_hat[2], w_hat[3]};
  const double wn = std::sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
  double A[9];
  // t.isApproxToConstant(0, 1e-10): Eigen's scalar isApprox(x, 0, p) is |x| <= min(|x|, 0) * p,
  // i.e. true only for an exact zero vector
  const bool t0 = t[0] == 0 && t[1] == 0 && t[2] == 0;
  if (t0) {
    for (int i = 0; i < 9; ++i) A[i] = 0;
  } else if (wn == 0 || std::sin(wn) == 0) {
    for (int i = 0; i < 9; ++i) A[i] = (i % 4 == 0) ? 1.0 : 0.0;
  } else {
    double W2[9];
    mm3(w_hat, w_hat, W2);
    const double f = (2 * std::sin(wn) - wn * (1 + std::cos(wn))) / (2 * wn * wn * std::sin(wn));
    for (int i = 0; i < 9; ++i) A[i] = ((i % 4 == 0) ? 1.0 : 0.0) - w_hat[i] / 2 + f * W2[i];
  }
  for (int i = 0; i < 3; ++i) twist[i] = A[i * 3] * t[0] + A[i * 3 + 1] * t[1] + A[i * 3 + 2] * t[2];
  twist[3] = w[0]; twist[4] = w[1]; twist[5] = w[2];
}

// predictPose (PE:995-1010): returns predictionMatrix, writes predicted pose = current * prediction
void orc_predict_pose(const double* prev12, const double* cur12, double t_prev, double t_cur,
                      double t_pred, double* prediction12, double* predicted12) {
  const Mat4 prev = from12(prev12), cur = from12(cur12);
  double rel[12], delta[6], dh[6];
  to12(mul(inverse_rigid(prev), cur), rel);
  orc_log_map(rel, delta);
  for (int i = 0; i < 6; ++i) dh[i] = delta[i] / (t_cur - t_prev) * (t_pred - t_cur);
  orc_exp_map(dh, prediction12);
  to12(mul(cur, from12(prediction12)), predicted12);
}

// ------------------------------------------------------------- Gauss-Newton optimisePose (PE:1805)
static bool ldlt_solve6(const double A_in[36], const double b_in[6], double x[6]) {
  // LDL^T with symmetric diagonal pivoting (Eigen::LDLT strategy: largest remaining |diagonal|)
  double A[36];
  std::memcpy(A, A_in, sizeof(A));
  int perm[6] = {0, 1, 2, 3, 4, 5};
  for (int k = 0; k < 6; ++k) {
    int p = k;
    for (int i = k + 1; i < 6; ++i)
      if (std::abs(A[i * 6 + i]) > std::abs(A[p * 6 + p])) p = i;
    if (p != k) {
      std::swap(perm[k], perm[p]);
      for (int j = 0; j < 6; ++j) std::swap(A[k * 6 + j], A[p * 6 + j]);
      for (int i = 0; i < 6; ++i) std::swap(A[i * 6 + k], A[i * 6 + p]);
    }
    const double d = A[k * 6 + k];
    if (d == 0) return false;
    double l[6] = {0};
    for (int i = k + 1; i < 6; ++i) l[i] = A[i * 6 + k] / d;
    // Schur update with the ORIGINAL column k (multipliers are stored only afterwards)
    for (int i = k + 1; i < 6; ++i)
      for (int j = k + 1; j <= i; ++j) A[i * 6 + j] -= l[i] * A[j * 6 + k];
    for (int i = k + 1; i < 6; ++i) A[i * 6 + k] = l[i];
    for (int i = k + 1; i < 6; ++i)
      for (int j = i + 1; j < 6; ++j) A[i * 6 + j] = A[j * 6 + i];
  }
  double y[6];
  for (int i = 0; i < 6; ++i) y[i] = b_in[perm[i]];
  for (int i = 0; i < 6; ++i)
    for (int j = 0; j < i; ++j) y[i] -= A[i * 6 + j] * y[j];
  for (int i = 0; i < 6; ++i) y[i] /= A[i * 6 + i];
  for (int i = 5; i >= 0; --i)
    for (int j = i + 1; j < 6; ++j) y[i] -= A[j * 6 + i] * y[j];
  for (int i = 0; i < 6; ++i) x[perm[i]] = y[i];
  return true;
}

static bool inverse6(const double A[36], double Ai[36]) {
  for (int c = 0; c < 6; ++c) {
    double e[6] = {0}, x[6];
    e[c] = 1;
    if (!ldlt_solve6(A, e, x)) return false;
    for (int r = 0; r < 6; ++r) Ai[r * 6 + c] = x[r];
  }
  return true;
}

// corr: npairs (LED, blob) 1-based rows; returns GN iterations (PubData.numIter) or 500 if no conv.
int orc_optimise_pose(int M, const double* markers, const double* K, int B, const double* blobs,
                      const unsigned* corr, int npairs, const double* pose_in12, double* pose_out12,
                      double* cov36) {
  const double converged = 1e-13;
  const unsigned max_itr = 500;
  Mat4 pose = from12(pose_in12);
  const Mat4 pose_init = pose;
  const double fx = K[0], fy = K[4];
  double A[36], b[6], dT[6];
  double e_init = 0, e_end = 0;
  int iters = (int)max_itr;
  (void)M; (void)B;
  for (unsigned it = 0; it < max_itr; ++it) {
    std::memset(A, 0, sizeof(A));
    std::memset(b, 0, sizeof(b));
    for (int j = 0; j < npairs; ++j) {
      if (corr[2 * j + 1] == 0) continue;
      const double* X = markers + 3 * (corr[2 * j] - 1);
      double uv[2];
      project2d(K, pose, X, uv);
      const double* z = blobs + 2 * (corr[2 * j + 1] - 1);
      const double e[2] = {z[0] - uv[0], z[1] - uv[1]};
      if (it == 0) e_init = std::sqrt(e[0] * e[0] + e[1] * e[1]);
      else if (it + 1 == max_itr) e_end = std::sqrt(e[0] * e[0] + e[1] * e[1]);
      // computeJacobian (PE:2163) on the camera-frame point
      double pc[3];
      for (int r = 0; r < 3; ++r) pc[r] = pose(r, 0) * X[0] + pose(r, 1) * X[1] + pose(r, 2) * X[2] + pose(r, 3);
      const double x = pc[0], y = pc[1], zz = pc[2], z2 = zz * zz;
      double J[12];
      J[0] = 1 / zz * fx; J[1] = 0; J[2] = -x / z2 * fx; J[3] = -x * y / z2 * fx;
      J[4] = (1 + (x * x / z2)) * fx; J[5] = -y / zz * fx;
      J[6] = 0; J[7] = 1 / zz * fy; J[8] = -y / z2 * fy; J[9] = -(1 + y * y / z2) * fy;
      J[10] = x * y / z2 * fy; J[11] = x / zz * fy;
      for (int r = 0; r < 6; ++r) {
        for (int c = 0; c < 6; ++c) A[r * 6 + c] += J[r] * J[c] + J[6 + r] * J[6 + c];
        b[r] += J[r] * e[0] + J[6 + r] * e[1];
      }
    }
    if (!ldlt_solve6(A, b, dT)) std::memset(dT, 0, sizeof(dT));
    double dp[12];
    orc_exp_map(dT, dp);
    pose = mul(from12(dp), pose);
    double nm = -1;
    for (int r = 0; r < 6; ++r) nm = std::max(nm, std::abs(dT[r]));
    if (nm <= converged) { iters = (int)it; break; }
    if (it + 1 == max_itr && e_init < e_end) pose = pose_init;
  }
  to12(pose, pose_out12);
  if (cov36 && !inverse6(A, cov36)) std::memset(cov36, 0, 36 * sizeof(double));
  return iters;
}

// ------------------------------------------------------------------ ROI prediction (§8f row 1)
// predictMarkerPositionsInImage (PE:1036-1053) + LEDDetector::determineROI (led_detector.cpp:217-369) +
// distortPoints (led_detector.cpp:371-414), literally: the reference's loops and cv::Point2f roundings.
static void distort_point(const double* K, const double* D, float xin, float yin, float* xo, float* yo) {
  const double fx_K = K[0], fy_K = K[4], cx_K = K[2], cy_K = K[5];
  const double k1 = D[0], k2 = D[1], p1 = D[2], p2 = D[3], k3 = D[4];
  const double px = (double)xin, py = (double)yin;  // const cv::Point2d &p = src[i] (float -> double)
  const double x = (px - cx_K) / fx_K;
  const double y = (py - cy_K) / fy_K;
  const double r2 = x * x + y * y;
  double xC = x * (1. + k1 * r2 + k2 * r2 * r2 + k3 * r2 * r2 * r2);
  double yC = y * (1. + k1 * r2 + k2 * r2 * r2 + k3 * r2 * r2 * r2);
  xC = xC + (2. * p1 * x * y + p2 * (r2 + 2. * x * x));
  yC = yC + (p1 * (r2 + 2. * y * y) + 2. * p2 * x * y);
  xC = xC * fx_K + cx_K;
  yC = yC * fy_K + cy_K;
  *xo = (float)xC;  // dst.push_back(cv::Point2d(...)) into a std::vector<cv::Point2f>
  *yo = (float)yC;
}

int orc_predict_roi(int N, int M, const double* markers, const double* K, const double* D, const double* prior,
                    const double* cam12, const double* predm12, const double* predicted12, int W, int H,
                    int border, int* roi4, double* bbox4) {
  const Mat4 cam = from12(cam12), predm = from12(predm12), pred = from12(predicted12);
  std::vector<double> px, py;
  px.reserve((size_t)(N + 1) * M);
  py.reserve((size_t)(N + 1) * M);
  for (int i = 0; i < M; ++i)
    for (int j = 0; j < N; ++j) {
      const Mat4 T = mul(mul(cam, from12(prior + 12 * (size_t)j)), predm);
      double uv[2];
      project2d(K, T, markers + 3 * i, uv);
      px.push_back(uv[0]);
      py.push_back(uv[1]);
    }
  for (int k = 0; k < M; ++k) {
    double uv[2];
    project2d(K, pred, markers + 3 * k, uv);
    px.push_back(uv[0]);
    py.push_back(uv[1]);
  }
  double x_min = INFINITY, x_max = 0, y_min = INFINITY, y_max = 0;
  for (size_t i = 0; i < px.size(); ++i) {
    if (px[i] < x_min) x_min = px[i];
    if (px[i] > x_max) x_max = px[i];
    if (py[i] < y_min) y_min = py[i];
    if (py[i] > y_max) y_max = py[i];
  }
  bbox4[0] = x_min;
  bbox4[1] = x_max;
  bbox4[2] = y_min;
  bbox4[3] = y_max;
  float dx0, dy0, dx1, dy1;
  distort_point(K, D, (float)x_min, (float)y_min, &dx0, &dy0);  // cv::Point2f(x_min, y_min)
  distort_point(K, D, (float)x_max, (float)y_max, &dx1, &dy1);
  const double x0 = std::max(0.0, std::min((double)W, (double)dx0 - border));
  const double x1 = std::max(0.0, std::min((double)W, (double)dx1 + border));
  const double y0 = std::max(0.0, std::min((double)H, (double)dy0 - border));
  const double y1 = std::max(0.0, std::min((double)H, (double)dy1 + border));
  if (x1 - x0 < 1 || y1 - y0 < 1) {
    roi4[0] = 0;
    roi4[1] = 0;
    roi4[2] = W;
    roi4[3] = H;
  } else {  // cv::Rect int fields: x0 -> int, (x1 - x0) -> int (truncation)
    roi4[0] = (int)x0;
    roi4[1] = (int)y0;
    roi4[2] = (int)(x1 - x0);
    roi4[3] = (int)(y1 - y0);
  }
  return 0;
}

}  // extern "C"
