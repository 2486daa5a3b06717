// =====================================================================================================
//  init_oracle.cpp — CPU restatement of the reference's brute-force P3P (re)initialisation.
//
//  TEST INFRASTRUCTURE ONLY (same contract as pf_oracle.cpp): the checker for the engine's
//  pfmpe_p3p_histogram / pfmpe_initialise, and the CPU baseline bench_init times.  Never the product.
//
//  What it restates ("PE" = pf_mpe_lib/src/pose_estimator.cpp, "P3P" = pf_mpe_lib/src/p3p.cpp):
//    * calculateImageVectors                                   PE:1072-1085
//    * P3P::computePoses + solveQuartic (Kneip's parametrisation; the quartic is solved with
//      std::complex exactly as the reference does, so the libstdc++ pow/log/polar/csqrt and the
//      libgcc complex division are the reference's own arithmetic)          P3P:65-292
//    * initialise: correspondence histogram over every 3-blob combination x every ordered 3-marker
//      permutation x 4 P3P solutions, with the blob-spread filter (threshDist, cd >= 5), the
//      "repeated solution" skip, isFinite, back projection through H.inverse() and
//      calculateMinDistancesAndPairs                          PE:1526-1716, PE:2088-2137
//    * correspondencesFromHistogram (uint32 colSum*rowSum product, 1.3/(rows*cols) threshold,
//      enumeration with the last LED fastest, repeated max_element selection) + checkAmbiguity
//                                                              PE:1134-1288, PE:2447-2458
//    * checkCorrespondences + calculateSquaredReprojectionErrorAndCertainty
//                                                              PE:1312-1501, PE:1087-1132
//    * the particle seeding and fill loop of initialise        PE:1717-1766, PE:1429-1437
//    * computeTransformation (SVD of the 3x3 cross-covariance, R = V U^T, no reflection fix)
//                                                              PE:2139-2161
//    * Combinations::combinationsNoReplacement = lexicographic order (checked against the
//      reference's Matt-Fig index recurrence in tests/test_init_oracle.py)   combinations.cpp:64-133
//
//  Parity status: PARITY UNPINNED by the reference itself (no tests/fixtures, Eigen/OpenCV/ROS absent —
//  SURVEY.md §8c).  Unpinnable details, stated: Eigen's 4x4 inverse (here: cofactor expansion, also
//  used on the device), Eigen's reduction order for norms / 3x3 products (here: sequential), and
//  Eigen's JacobiSVD (here: one-sided Jacobi; R = V U^T is unique up to rounding when the singular
//  values are distinct).  checkAmbiguity reads one element past the end of its vector (PE:2451,
//  j = size()); that read is taken as "no match".
// =====================================================================================================
#include <algorithm>
#include <cmath>
#include <complex>
#include <cstdint>
#include <cstring>
#include <limits>
#include <vector>

namespace {

using cplx = std::complex<double>;

struct Pose34 {
  double a[12];  // row-major [R | C]
};

inline double sqnorm3(const double* v) { return v[0] * v[0] + v[1] * v[1] + v[2] * v[2]; }
inline double norm3(const double* v) { return std::sqrt(sqnorm3(v)); }
inline void cross3(const double* a, const double* b, double* c) {  // Eigen OrthoMethods order
  c[0] = a[1] * b[2] - a[2] * b[1];
  c[1] = a[2] * b[0] - a[0] * b[2];
  c[2] = a[0] * b[1] - a[1] * b[0];
}
inline double dot3(const double* a, const double* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
// y = A x, A row-major 3x3
inline void mv3(const double* A, const double* x, double* y) {
  for (int r = 0; r < 3; ++r) y[r] = A[3 * r + 0] * x[0] + A[3 * r + 1] * x[1] + A[3 * r + 2] * x[2];
}
// y = A^T x
inline void mtv3(const double* A, const double* x, double* y) {
  for (int r = 0; r < 3; ++r) y[r] = A[0 + r] * x[0] + A[3 + r] * x[1] + A[6 + r] * x[2];
}
inline void mm3(const double* A, const double* B, double* C) {
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) C[3 * i + j] = A[3 * i + 0] * B[0 + j] + A[3 * i + 1] * B[3 + j] + A[3 * i + 2] * B[6 + j];
}

// ------------------------------------------------------------------ P3P::solveQuartic (P3P:244-290)
void solve_quartic(const double f[5], double roots[4]) {
  const double A = f[0], B = f[1], C = f[2], D = f[3], E = f[4];
  const double A_pw2 = A * A, B_pw2 = B * B;
  const double A_pw3 = A_pw2 * A, B_pw3 = B_pw2 * B;
  const double A_pw4 = A_pw3 * A, B_pw4 = B_pw3 * B;
  const double alpha = -3 * B_pw2 / (8 * A_pw2) + C / A;
  const double beta = B_pw3 / (8 * A_pw3) - B * C / (2 * A_pw2) + D / A;
  const double gamma = -3 * B_pw4 / (256 * A_pw4) + B_pw2 * C / (16 * A_pw3) - B * D / (4 * A_pw2) + E / A;
  const double alpha_pw2 = alpha * alpha;
  const double alpha_pw3 = alpha_pw2 * alpha;
  const cplx P(-alpha_pw2 / 12 - gamma, 0);
  const cplx Q(-alpha_pw3 / 108 + alpha * gamma / 3 - std::pow(beta, 2) / 8, 0);
  const cplx R = -Q / 2.0 + std::sqrt(std::pow(Q, 2.0) / 4.0 + std::pow(P, 3.0) / 27.0);
  const cplx U = std::pow(R, (1.0 / 3.0));
  cplx y;
  if (U.real() == 0)
    y = -5.0 * alpha / 6.0 - std::pow(Q, (1.0 / 3.0));
  else
    y = -5.0 * alpha / 6.0 - P / (3.0 * U) + U;
  const cplx w = std::sqrt(alpha + 2.0 * y);
  cplx t;
  t = -B / (4.0 * A) + 0.5 * (w + std::sqrt(-(3.0 * alpha + 2.0 * y + 2.0 * beta / w)));
  roots[0] = t.real();
  t = -B / (4.0 * A) + 0.5 * (w - std::sqrt(-(3.0 * alpha + 2.0 * y + 2.0 * beta / w)));
  roots[1] = t.real();
  t = -B / (4.0 * A) + 0.5 * (-w + std::sqrt(-(3.0 * alpha + 2.0 * y - 2.0 * beta / w)));
  roots[2] = t.real();
  t = -B / (4.0 * A) + 0.5 * (-w - std::sqrt(-(3.0 * alpha + 2.0 * y - 2.0 * beta / w)));
  roots[3] = t.real();
}

// ------------------------------------------------------------------ P3P::computePoses (P3P:65-242)
// fv / wp: the three feature vectors / world points (fv[k], wp[k] = column k).  Returns -1 when the
// world points are collinear, else 0 with four [R|C] solutions (camera orientation and position in
// the world frame).
int p3p(const double fv[3][3], const double wp[3][3], Pose34 sol[4], double* roots_out = nullptr) {
  double P1[3], P2[3], P3[3];
  std::memcpy(P1, wp[0], sizeof(P1));
  std::memcpy(P2, wp[1], sizeof(P2));
  std::memcpy(P3, wp[2], sizeof(P3));
  double t1[3], t2[3], cr[3];
  for (int i = 0; i < 3; ++i) {
    t1[i] = P2[i] - P1[i];
    t2[i] = P3[i] - P1[i];
  }
  cross3(t1, t2, cr);
  if (norm3(cr) == 0) return -1;

  double f1[3], f2[3], f3[3];
  std::memcpy(f1, fv[0], sizeof(f1));
  std::memcpy(f2, fv[1], sizeof(f2));
  std::memcpy(f3, fv[2], sizeof(f3));
  double e1[3], e2[3], e3[3], T[9], f3t[3];
  auto frame = [&]() {
    std::memcpy(e1, f1, sizeof(e1));
    cross3(f1, f2, e3);
    const double n = norm3(e3);
    for (int i = 0; i < 3; ++i) e3[i] = e3[i] / n;
    cross3(e3, e1, e2);
    for (int i = 0; i < 3; ++i) {
      T[0 + i] = e1[i];
      T[3 + i] = e2[i];
      T[6 + i] = e3[i];
    }
    mv3(T, f3, f3t);
  };
  frame();
  if (f3t[2] > 0) {  // theta in [0, pi]: swap the first two correspondences
    std::memcpy(f1, fv[1], sizeof(f1));
    std::memcpy(f2, fv[0], sizeof(f2));
    std::memcpy(f3, fv[2], sizeof(f3));
    frame();
    std::memcpy(P1, wp[1], sizeof(P1));
    std::memcpy(P2, wp[0], sizeof(P2));
    std::memcpy(P3, wp[2], sizeof(P3));
  }
  std::memcpy(f3, f3t, sizeof(f3));

  double n1[3], n2[3], n3[3], d[3], N[9];
  for (int i = 0; i < 3; ++i) n1[i] = P2[i] - P1[i];
  {
    const double nn = norm3(n1);
    for (int i = 0; i < 3; ++i) n1[i] = n1[i] / nn;
  }
  for (int i = 0; i < 3; ++i) d[i] = P3[i] - P1[i];
  cross3(n1, d, n3);
  {
    const double nn = norm3(n3);
    for (int i = 0; i < 3; ++i) n3[i] = n3[i] / nn;
  }
  cross3(n3, n1, n2);
  for (int i = 0; i < 3; ++i) {
    N[0 + i] = n1[i];
    N[3 + i] = n2[i];
    N[6 + i] = n3[i];
  }
  double P3n[3];
  mv3(N, d, P3n);

  double dd[3];
  for (int i = 0; i < 3; ++i) dd[i] = P2[i] - P1[i];
  const double d_12 = norm3(dd);
  const double f_1 = f3[0] / f3[2];
  const double f_2 = f3[1] / f3[2];
  const double p_1 = P3n[0];
  const double p_2 = P3n[1];
  const double cos_beta = dot3(f1, f2);
  double b = 1 / (1 - std::pow(cos_beta, 2)) - 1;
  b = cos_beta < 0 ? -std::sqrt(b) : std::sqrt(b);

  const double f_1_pw2 = std::pow(f_1, 2);
  const double f_2_pw2 = std::pow(f_2, 2);
  const double p_1_pw2 = std::pow(p_1, 2);
  const double p_1_pw3 = p_1_pw2 * p_1;
  const double p_1_pw4 = p_1_pw3 * p_1;
  const double p_2_pw2 = std::pow(p_2, 2);
  const double p_2_pw3 = p_2_pw2 * p_2;
  const double p_2_pw4 = p_2_pw3 * p_2;
  const double d_12_pw2 = std::pow(d_12, 2);
  const double b_pw2 = std::pow(b, 2);

  // quartic in cos(theta): Kneip 2011, eq. (the reference's term order is kept: it fixes rounding)
  double fac[5];
  fac[0] = -f_2_pw2 * p_2_pw4 - p_2_pw4 * f_1_pw2 - p_2_pw4;
  fac[1] = 2 * p_2_pw3 * d_12 * b + 2 * f_2_pw2 * p_2_pw3 * d_12 * b - 2 * f_2 * p_2_pw3 * f_1 * d_12;
  fac[2] = -f_2_pw2 * p_2_pw2 * p_1_pw2 - f_2_pw2 * p_2_pw2 * d_12_pw2 * b_pw2 - f_2_pw2 * p_2_pw2 * d_12_pw2 +
           f_2_pw2 * p_2_pw4 + p_2_pw4 * f_1_pw2 + 2 * p_1 * p_2_pw2 * d_12 +
           2 * f_1 * f_2 * p_1 * p_2_pw2 * d_12 * b - p_2_pw2 * p_1_pw2 * f_1_pw2 +
           2 * p_1 * p_2_pw2 * f_2_pw2 * d_12 - p_2_pw2 * d_12_pw2 * b_pw2 - 2 * p_1_pw2 * p_2_pw2;
  fac[3] = 2 * p_1_pw2 * p_2 * d_12 * b + 2 * f_2 * p_2_pw3 * f_1 * d_12 - 2 * f_2_pw2 * p_2_pw3 * d_12 * b -
           2 * p_1 * p_2 * d_12_pw2 * b;
  fac[4] = -2 * f_2 * p_2_pw2 * f_1 * p_1 * d_12 * b + f_2_pw2 * p_2_pw2 * d_12_pw2 + 2 * p_1_pw3 * d_12 -
           p_1_pw2 * d_12_pw2 + f_2_pw2 * p_2_pw2 * p_1_pw2 - p_1_pw4 - 2 * f_2_pw2 * p_2_pw2 * p_1 * d_12 +
           p_2_pw2 * f_1_pw2 * p_1_pw2 + f_2_pw2 * p_2_pw2 * d_12_pw2 * b_pw2;
  double roots[4];
  solve_quartic(fac, roots);
  if (roots_out) std::memcpy(roots_out, roots, sizeof(roots));

  for (int i = 0; i < 4; ++i) {
    const double cot_alpha = (-f_1 * p_1 / f_2 - roots[i] * p_2 + d_12 * b) / (-f_1 * roots[i] * p_2 / f_2 + p_1 - d_12);
    const double cos_theta = roots[i];
    const double sin_theta = std::sqrt(1 - std::pow((double)roots[i], 2));
    const double sin_alpha = std::sqrt(1 / (std::pow(cot_alpha, 2) + 1));
    double cos_alpha = std::sqrt(1 - std::pow(sin_alpha, 2));
    if (cot_alpha < 0) cos_alpha = -cos_alpha;
    double Cl[3];
    Cl[0] = d_12 * cos_alpha * (sin_alpha * b + cos_alpha);
    Cl[1] = cos_theta * d_12 * sin_alpha * (sin_alpha * b + cos_alpha);
    Cl[2] = sin_theta * d_12 * sin_alpha * (sin_alpha * b + cos_alpha);
    double NtC[3];
    mtv3(N, Cl, NtC);
    double Cw[3];
    for (int k = 0; k < 3; ++k) Cw[k] = P1[k] + NtC[k];
    double Rl[9];
    Rl[0] = -cos_alpha;
    Rl[1] = -sin_alpha * cos_theta;
    Rl[2] = -sin_alpha * sin_theta;
    Rl[3] = sin_alpha;
    Rl[4] = -cos_alpha * cos_theta;
    Rl[5] = -cos_alpha * sin_theta;
    Rl[6] = 0;
    Rl[7] = -sin_theta;
    Rl[8] = cos_theta;
    // R = N^T * R^T * T, evaluated left to right
    double Nt[9], Rt[9], tmp[9], Rw[9];
    for (int r = 0; r < 3; ++r)
      for (int c = 0; c < 3; ++c) {
        Nt[3 * r + c] = N[3 * c + r];
        Rt[3 * r + c] = Rl[3 * c + r];
      }
    mm3(Nt, Rt, tmp);
    mm3(tmp, T, Rw);
    for (int r = 0; r < 3; ++r) {
      for (int c = 0; c < 3; ++c) sol[i].a[4 * r + c] = Rw[3 * r + c];
      sol[i].a[4 * r + 3] = Cw[r];
    }
  }
  return 0;
}

// ------------------------------------------------------------------ 4x4 helpers
bool is_finite34(const Pose34& s) {  // isFinite(H) (PE:2088): (x - x) == (x - x) for every entry
  for (int i = 0; i < 12; ++i) {
    const double z = s.a[i] - s.a[i];
    if (!(z == z)) return false;
  }
  return true;
}

// H.inverse() for H = [[R C];[0 0 0 1]] as a general 4x4 (cofactor expansion; see header).  The
// bottom row of the inverse is (0 0 0 1) up to rounding; only the top 3 rows feed project2d, and the
// 4th row is computed too because project2d multiplies the full 4x4.
void inverse44(const Pose34& s, double inv[16]) {
  double m[16];
  for (int i = 0; i < 12; ++i) m[i] = s.a[i];
  m[12] = 0;
  m[13] = 0;
  m[14] = 0;
  m[15] = 1;
  // 2x2 sub-determinants of rows 0-1 and rows 2-3
  const double s0 = m[0] * m[5] - m[4] * m[1];
  const double s1 = m[0] * m[6] - m[4] * m[2];
  const double s2 = m[0] * m[7] - m[4] * m[3];
  const double s3 = m[1] * m[6] - m[5] * m[2];
  const double s4 = m[1] * m[7] - m[5] * m[3];
  const double s5 = m[2] * m[7] - m[6] * m[3];
  const double c5 = m[10] * m[15] - m[14] * m[11];
  const double c4 = m[9] * m[15] - m[13] * m[11];
  const double c3 = m[9] * m[14] - m[13] * m[10];
  const double c2 = m[8] * m[15] - m[12] * m[11];
  const double c1 = m[8] * m[14] - m[12] * m[10];
  const double c0 = m[8] * m[13] - m[12] * m[9];
  const double det = s0 * c5 - s1 * c4 + s2 * c3 + s3 * c2 - s4 * c1 + s5 * c0;
  const double id = 1.0 / det;
  inv[0] = (m[5] * c5 - m[6] * c4 + m[7] * c3) * id;
  inv[1] = (-m[1] * c5 + m[2] * c4 - m[3] * c3) * id;
  inv[2] = (m[13] * s5 - m[14] * s4 + m[15] * s3) * id;
  inv[3] = (-m[9] * s5 + m[10] * s4 - m[11] * s3) * id;
  inv[4] = (-m[4] * c5 + m[6] * c2 - m[7] * c1) * id;
  inv[5] = (m[0] * c5 - m[2] * c2 + m[3] * c1) * id;
  inv[6] = (-m[12] * s5 + m[14] * s2 - m[15] * s1) * id;
  inv[7] = (m[8] * s5 - m[10] * s2 + m[11] * s1) * id;
  inv[8] = (m[4] * c4 - m[5] * c2 + m[7] * c0) * id;
  inv[9] = (-m[0] * c4 + m[1] * c2 - m[3] * c0) * id;
  inv[10] = (m[12] * s4 - m[13] * s2 + m[15] * s0) * id;
  inv[11] = (-m[8] * s4 + m[9] * s2 - m[11] * s0) * id;
  inv[12] = (-m[4] * c3 + m[5] * c1 - m[6] * c0) * id;
  inv[13] = (m[0] * c3 - m[1] * c1 + m[2] * c0) * id;
  inv[14] = (-m[12] * s3 + m[13] * s1 - m[14] * s0) * id;
  inv[15] = (m[8] * s3 - m[9] * s1 + m[10] * s0) * id;
}

// project2d (PE:1017-1034): ([K|0] * T) * [X;1], then / z — same order as pf_oracle.cpp's project2d
void project44(const double* K, const double T[16], const double* X, double uv[2]) {
  double Q[12];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 4; ++j) {
      double s = K[i * 3 + 0] * T[0 * 4 + j];
      s = s + K[i * 3 + 1] * T[1 * 4 + j];
      s = s + K[i * 3 + 2] * T[2 * 4 + j];
      s = s + 0.0 * T[3 * 4 + j];
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
  uv[0] = p[0] / p[2];
  uv[1] = p[1] / p[2];
}

inline double sqdist2(const double* a, const double* b) {
  const double dx = a[0] - b[0], dy = a[1] - b[1];
  return dx * dx + dy * dy;
}

// calculateImageVectors (PE:1072-1085)
void image_vectors(const double* K, int B, const double* blobs, std::vector<double>& iv) {
  iv.resize(3 * (size_t)B);
  for (int i = 0; i < B; ++i) {
    double v[3];
    v[0] = (blobs[2 * i] - K[2]) / K[0];
    v[1] = (blobs[2 * i + 1] - K[5]) / K[4];
    v[2] = 1;
    const double n = norm3(v);
    for (int k = 0; k < 3; ++k) iv[3 * i + k] = v[k] / n;
  }
}

// lexicographic k-subsets of {0..n-1} (Combinations::combinationsNoReplacement, 0-based here)
std::vector<int> combinations3(int n) {
  std::vector<int> out;
  for (int a = 0; a < n; ++a)
    for (int b = a + 1; b < n; ++b)
      for (int c = b + 1; c < n; ++c) {
        out.push_back(a);
        out.push_back(b);
        out.push_back(c);
      }
  return out;
}
// every ordered 3-permutation of {0..n-1}: the histogram is a commutative sum over them, so the
// enumeration order of Combinations::permutationsNoReplacement does not matter
std::vector<int> permutations3(int n) {
  std::vector<int> out;
  for (int a = 0; a < n; ++a)
    for (int b = 0; b < n; ++b)
      for (int c = 0; c < n; ++c)
        if (a != b && a != c && b != c) {
          out.push_back(a);
          out.push_back(b);
          out.push_back(c);
        }
  return out;
}

// ------------------------------------------------------------------ histogram (PE:1526-1716)
// hist: the reference's histogram.  lo / hi (optional): bounds that every implementation whose fp64
// arithmetic differs from this one only at the ulp level must fall between.  Three reference decisions
// hinge on exact floating-point equality or a threshold and are "fragile" when their margin is at the
// ulp level: the repeated-solution skip (two roots within 64 ulp: a complex-conjugate pair whose real
// parts come out equal or not depending on the last bits of the libm calls inside std::complex pow),
// a root at |cos theta| = 1 (isFinite), and a blob at the tol gate or tied between two projections.
// A fragile contribution goes to hi only; everything else to both.  *unbounded counts fragile
// isFinite cases (their contribution cannot be bounded from here).
void histogram(int M, const double* markers, const double* K, int B, const double* blobs, double tol,
               uint32_t* hist /* B x M, row-major */, uint32_t* lo = nullptr, uint32_t* hi = nullptr,
               int* unbounded = nullptr) {
  std::memset(hist, 0, sizeof(uint32_t) * (size_t)B * M);
  if (lo) std::memset(lo, 0, sizeof(uint32_t) * (size_t)B * M);
  if (hi) std::memset(hi, 0, sizeof(uint32_t) * (size_t)B * M);
  if (unbounded) *unbounded = 0;
  std::vector<double> iv;
  image_vectors(K, B, blobs, iv);
  const std::vector<int> cmb = combinations3(B);
  const std::vector<int> prm = permutations3(M);
  const double threshDist = 10000 * 100, threshDist2 = 10000 * 100;
  std::vector<double> un_im;
  std::vector<int> un_im_idx;
  std::vector<int> pair_obj(B), state(B);
  for (size_t ci = 0; ci < cmb.size() / 3; ++ci) {
    const int* s = &cmb[3 * ci];
    double fv[3][3];
    for (int k = 0; k < 3; ++k)
      for (int q = 0; q < 3; ++q) fv[k][q] = iv[3 * s[k] + q];
    const double* d1 = blobs + 2 * s[0];
    const double* d2 = blobs + 2 * s[1];
    const double* d3 = blobs + 2 * s[2];
    if (sqdist2(d1, d2) > threshDist) continue;
    if (sqdist2(d1, d3) > threshDist) continue;
    if (sqdist2(d2, d3) > threshDist) continue;
    const double dm[2] = {(d1[0] + d2[0] + d3[0]) / 3, (d1[1] + d2[1] + d3[1]) / 3};
    int cd = 0;
    for (int kk = 0; kk < B; ++kk)
      if (sqdist2(dm, blobs + 2 * kk) < threshDist2) cd++;
    if (cd < 5) continue;
    un_im.clear();
    un_im_idx.clear();
    for (int kk = 0; kk < B; ++kk) {
      if (kk == s[0] || kk == s[1] || kk == s[2]) continue;
      if (sqdist2(dm, blobs + 2 * kk) < threshDist2) {
        un_im.push_back(blobs[2 * kk]);
        un_im.push_back(blobs[2 * kk + 1]);
        un_im_idx.push_back(kk);
      }
      if ((int)un_im_idx.size() == B - 3) break;
    }
    const int nui = (int)un_im_idx.size();
    for (size_t pj = 0; pj < prm.size() / 3; ++pj) {
      const int* p = &prm[3 * pj];
      double wp[3][3];
      for (int k = 0; k < 3; ++k)
        for (int q = 0; q < 3; ++q) wp[k][q] = markers[3 * p[k] + q];
      Pose34 sol[4];
      double roots[4];
      if (p3p(fv, wp, sol, roots) != 0) continue;
      int un_obj[16];
      int nuo = 0;
      for (int ll = 0; ll < M; ++ll)
        if (ll != p[0] && ll != p[1] && ll != p[2]) un_obj[nuo++] = ll;
      for (int k = 0; k < 4; ++k) {
        bool repeated = false, frag_sol = false;
        if (k > 0) {  // (solutions(k) - solutions(k-1)).all() == 0  <=>  some entry difference is 0
          for (int q = 0; q < 12; ++q)
            if (sol[k].a[q] - sol[k - 1].a[q] == 0) repeated = true;
          const double a = roots[k], b = roots[k - 1];
          frag_sol = std::fabs(a - b) <= 64 * std::numeric_limits<double>::epsilon() * std::max(std::fabs(a), std::fabs(b));
        }
        if (repeated && !frag_sol) continue;
        if (!is_finite34(sol[k])) {
          if (unbounded && std::fabs(1.0 - std::fabs(roots[k])) < 1e-9) ++*unbounded;
          continue;
        }
        const bool counted_ref = !repeated;  // the reference's own decision
        double inv[16];
        inverse44(sol[k], inv);
        double proj[16][2];
        for (int m = 0; m < nuo; ++m) project44(K, inv, markers + 3 * un_obj[m], proj[m]);
        // calculateMinDistancesAndPairs(unused image points, back-projected unused markers)
        int n_in = 0, n_in_strict = 0;
        for (int a = 0; a < nui; ++a) {
          double mind = INFINITY, second = INFINITY;
          int pr = 0;
          for (int m = 0; m < nuo; ++m) {
            const double dsq = sqdist2(&un_im[2 * a], proj[m]);
            if (dsq < mind) {
              second = mind;
              mind = dsq;
              pr = m + 1;
            } else if (dsq < second) {
              second = dsq;
            }
          }
          const double d = std::sqrt(mind);
          const bool in = d < tol;
          const bool frag = std::fabs(d - tol) <= 1e-9 * tol || (second - mind <= 1e-9 * mind && d < tol * (1 + 1e-9));
          pair_obj[a] = pr;
          state[a] = in ? (frag ? 1 : 2) : (frag ? 1 : 0);  // 0 out, 1 fragile, 2 in
          if (in) n_in++;
          if (state[a] == 2) n_in_strict++;
        }
        if (counted_ref && n_in > 0) {
          for (int mm = 0; mm < 3; ++mm) hist[(size_t)s[mm] * M + p[mm]] += 1;
          for (int a = 0; a < nui; ++a)
            if (state[a] == 2 || (state[a] == 1 && std::sqrt(sqdist2(&un_im[2 * a], proj[pair_obj[a] - 1])) < tol))
              hist[(size_t)un_im_idx[a] * M + un_obj[pair_obj[a] - 1]] += 1;
        }
        if (!lo || !hi) continue;
        bool any_frag = false;
        for (int a = 0; a < nui; ++a) any_frag = any_frag || state[a] == 1;
        if (n_in_strict > 0 || any_frag) {  // the combination's 3 pairs: certain iff a certain blob counts
          const bool certain = !frag_sol && n_in_strict > 0;
          for (int mm = 0; mm < 3; ++mm) {
            hi[(size_t)s[mm] * M + p[mm]] += 1;
            if (certain) lo[(size_t)s[mm] * M + p[mm]] += 1;
          }
          for (int a = 0; a < nui; ++a) {
            if (state[a] == 0 || pair_obj[a] == 0) continue;
            const size_t e = (size_t)un_im_idx[a] * M + un_obj[pair_obj[a] - 1];
            hi[e] += 1;
            if (certain && state[a] == 2) lo[e] += 1;
          }
        }
      }
    }
  }
}

// ------------------------------------------------------------------ correspondencesFromHistogram
// (PE:1134-1288) with bInitialisation = true.  Each candidate is (LED+1, detection) rows.
struct Cand {
  std::vector<uint32_t> pairs;  // 2 * rows
};
bool check_ambiguity(const std::vector<int>& det) {  // PE:2447-2458 (the j = size() read: no match)
  const int n = (int)det.size();
  for (int i = 0; i < n; ++i)
    for (int j = n - 1; j > i; --j)
      if (det[i] == det[j]) return true;
  return false;
}
int candidates_from_histogram(int B, int M, const uint32_t* hist, int max_cand, std::vector<Cand>& out) {
  out.clear();
  const double prob_threshold = (1.3 * 1.0) / (B * M);
  std::vector<double> hp((size_t)B * M);
  for (size_t i = 0; i < hp.size(); ++i) hp[i] = (double)hist[i];
  for (int c = 0; c < M; ++c) {
    uint32_t colSum = 0;
    for (int r = 0; r < B; ++r) colSum += hist[(size_t)r * M + c];
    if (colSum == 0) continue;
    for (int r = 0; r < B; ++r) {
      uint32_t rowSum = 0;
      for (int q = 0; q < M; ++q) rowSum += hist[(size_t)r * M + q];
      const uint32_t den = colSum * rowSum;  // unsigned 32-bit product, as in the reference
      double& v = hp[(size_t)r * M + c];
      v = std::max(0.0, std::pow(v, 2) / den);
      if (v < prob_threshold) v = 0;
    }
  }
  std::vector<std::vector<double>> u_prob(M);
  std::vector<std::vector<int>> u_num(M);
  for (int a = 0; a < M; ++a)
    for (int b = 0; b < B; ++b)
      if (hp[(size_t)b * M + a] != 0) {
        u_prob[a].push_back(hp[(size_t)b * M + a]);
        u_num[a].push_back(b + 1);
      }
  int64_t Ntot = 1;
  for (int k = 0; k < M; ++k) {
    Ntot *= std::max<int64_t>(1, (int64_t)u_prob[k].size());
    if (Ntot > max_cand) return -1;
  }
  const int N = (int)Ntot;
  std::vector<double> v_prob(N);
  std::vector<std::vector<int>> v_comb(N);
  for (int i = 0; i < N; ++i) {
    double prob = 1;
    int n = 1;
    std::vector<int> comb;
    for (int led = M - 1; led > -1; --led) {
      const int nv = (int)u_num[led].size();
      if (nv > 0) {
        const int idx = (i / n) % nv;
        prob = prob * u_prob[led][idx];
        comb.push_back(u_num[led][idx]);
        n = n * std::max(1, nv);
      } else {
        comb.push_back(0);
      }
    }
    v_prob[i] = prob;
    std::reverse(comb.begin(), comb.end());
    v_comb[i] = comb;
  }
  double sum = 0;
  for (int i = 0; i < N; ++i) sum += v_prob[i];
  for (int i = 0; i < N; ++i) v_prob[i] = v_prob[i] / sum;
  for (int bb = 0; bb < N; ++bb) {
    const int row = (int)(std::max_element(v_prob.begin(), v_prob.end()) - v_prob.begin());
    v_prob[row] = 0;
    const std::vector<int>& det = v_comb[row];
    if (check_ambiguity(det)) continue;
    Cand cd;
    for (int led = 0; led < M; ++led)
      if (det[led] != 0) {
        cd.pairs.push_back((uint32_t)(led + 1));
        cd.pairs.push_back((uint32_t)det[led]);
      }
    out.push_back(cd);
  }
  return 0;
}

// ------------------------------------------------------------------ computeTransformation (PE:2139)
// one-sided Jacobi SVD of the 3x3 A = U S V^T; returns R = V U^T
void svd3_rotation(const double A_in[9], double R[9]) {
  double U[9], V[9];
  std::memcpy(U, A_in, sizeof(U));  // columns of U converge to A V (unnormalised)
  for (int i = 0; i < 9; ++i) V[i] = (i % 4 == 0) ? 1.0 : 0.0;
  for (int sweep = 0; sweep < 60; ++sweep) {
    double off = 0;
    for (int p = 0; p < 2; ++p)
      for (int q = p + 1; q < 3; ++q) {
        double alpha = 0, beta = 0, gamma = 0;
        for (int i = 0; i < 3; ++i) {
          alpha += U[3 * i + p] * U[3 * i + p];
          beta += U[3 * i + q] * U[3 * i + q];
          gamma += U[3 * i + p] * U[3 * i + q];
        }
        if (gamma == 0) continue;
        off = std::max(off, std::fabs(gamma) / std::sqrt(alpha * beta));
        const double zeta = (beta - alpha) / (2 * gamma);
        const double t = (zeta >= 0 ? 1.0 : -1.0) / (std::fabs(zeta) + std::sqrt(1 + zeta * zeta));
        const double c = 1 / std::sqrt(1 + t * t), s = c * t;
        for (int i = 0; i < 3; ++i) {
          const double up = U[3 * i + p], uq = U[3 * i + q];
          U[3 * i + p] = c * up - s * uq;
          U[3 * i + q] = s * up + c * uq;
          const double vp = V[3 * i + p], vq = V[3 * i + q];
          V[3 * i + p] = c * vp - s * vq;
          V[3 * i + q] = s * vp + c * vq;
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
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) R[3 * i + j] = V[3 * i + 0] * U[3 * j + 0] + V[3 * i + 1] * U[3 * j + 1] + V[3 * i + 2] * U[3 * j + 2];
}
void compute_transformation(int M, const double* obj /*M x 3*/, const double* rep /*M x 3*/, double* T12) {
  double mo[3] = {0, 0, 0}, mr[3] = {0, 0, 0};
  for (int j = 0; j < M; ++j)
    for (int k = 0; k < 3; ++k) {
      mo[k] += obj[3 * j + k];
      mr[k] += rep[3 * j + k];
    }
  for (int k = 0; k < 3; ++k) {
    mo[k] = mo[k] / M;
    mr[k] = mr[k] / M;
  }
  double A[9] = {0};  // obj_bar * rep_bar^T
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c) {
      double s = 0;
      for (int j = 0; j < M; ++j) s += (obj[3 * j + r] - mo[r]) * (rep[3 * j + c] - mr[c]);
      A[3 * r + c] = s;
    }
  double R[9];
  svd3_rotation(A, R);
  for (int r = 0; r < 3; ++r) {
    for (int c = 0; c < 3; ++c) T12[4 * r + c] = R[3 * r + c];
    T12[4 * r + 3] = mr[r] - (R[3 * r + 0] * mo[0] + R[3 * r + 1] * mo[1] + R[3 * r + 2] * mo[2]);
  }
}

}  // namespace

extern "C" {

typedef struct {
  double tol;                  // back_projection_pixel_tolerance_
  double certainty_threshold;  // certainty_threshold_
  double valid_corr_threshold; // valid_correspondence_threshold_
  int use_pf;                  // bUseParticleFilter
  int max_candidates;
} OrcInitParams;

typedef struct {
  int found, flag_fail, n_estimates, n_candidates, first_match, n_corr;
  uint32_t corr[32];
  double predicted_pose[12];
  uint64_t hist_total;
} OrcInitOut;

int orc_image_vectors(const double* K, int B, const double* blobs, double* out) {
  std::vector<double> iv;
  image_vectors(K, B, blobs, iv);
  std::memcpy(out, iv.data(), iv.size() * sizeof(double));
  return 0;
}

// P3P::computePoses on explicit inputs: fv / wp are 3 x 3 with ROWS = the three vectors / points.
int orc_p3p(const double* fv, const double* wp, double* sol48) {
  double f[3][3], w[3][3];
  for (int k = 0; k < 3; ++k)
    for (int q = 0; q < 3; ++q) {
      f[k][q] = fv[3 * k + q];
      w[k][q] = wp[3 * k + q];
    }
  Pose34 s[4];
  const int r = p3p(f, w, s);
  if (r == 0)
    for (int i = 0; i < 4; ++i) std::memcpy(sol48 + 12 * i, s[i].a, sizeof(s[i].a));
  return r;
}

void orc_inverse44(const double* sol12, double* inv16) {
  Pose34 s;
  std::memcpy(s.a, sol12, sizeof(s.a));
  inverse44(s, inv16);
}

int orc_init_histogram(int M, const double* markers, const double* K, int B, const double* blobs, double tol,
                       uint32_t* hist) {
  if (B < 3 || B > 1024 || M < 3 || M > 16) return -1;
  histogram(M, markers, K, B, blobs, tol, hist);
  return 0;
}

// initialise() (PE:1503-1786) for the particle-filter configuration.
//   particles: N x 12 in/out (PoseParticle: slots the reference writes are overwritten, the rest kept)
//   hist_in:   optional histogram to use instead of computing one (isolates the post-histogram stages)
// the histogram plus its fragility bounds lo <= any ulp-level reimplementation <= hi (see histogram())
int orc_init_histogram_bounds(int M, const double* markers, const double* K, int B, const double* blobs, double tol,
                              uint32_t* hist, uint32_t* lo, uint32_t* hi, int* unbounded) {
  if (B < 3 || B > 1024 || M < 3 || M > 16) return -1;
  histogram(M, markers, K, B, blobs, tol, hist, lo, hi, unbounded);
  return 0;
}

int orc_initialise(int M, const double* markers, const double* K, int B, const double* blobs,
                   const OrcInitParams* prm, int N_particle, const uint32_t* hist_in, uint32_t* hist_out,
                   double* particles, OrcInitOut* out) {
  std::memset(out, 0, sizeof(*out));
  out->first_match = -1;
  if (B > 1024 || M < 3 || M > 16 || N_particle < 1) return -1;
  const int minNumCorr = prm->use_pf ? M : 4;  // min_num_leds_detected_ = 4 (pose_estimator.h:104)
  if (B < (prm->use_pf ? M : 4)) {
    out->flag_fail = 10;
    return 0;
  }
  std::vector<uint32_t> hist((size_t)B * M);
  if (hist_in)
    std::memcpy(hist.data(), hist_in, hist.size() * sizeof(uint32_t));
  else
    histogram(M, markers, K, B, blobs, prm->tol, hist.data());
  if (hist_out) std::memcpy(hist_out, hist.data(), hist.size() * sizeof(uint32_t));
  uint64_t tot = 0;
  for (uint32_t h : hist) tot += h;
  out->hist_total = tot;
  if (tot == 0) {
    out->flag_fail = 12;
    return 0;
  }
  std::vector<Cand> cands;
  if (candidates_from_histogram(B, M, hist.data(), prm->max_candidates, cands) != 0) return -2;
  out->n_candidates = (int)cands.size();
  int flag = -1;  // -1: initialise wrote no Flag_Fail code
  if (cands.empty()) flag = 11;

  std::vector<double> iv;
  image_vectors(K, B, blobs, iv);
  int found = 0, n_est = 1, first = 0;
  const double tol2 = std::pow(prm->tol, 2);
  for (size_t ci = 0; ci < cands.size(); ++ci) {
    const std::vector<uint32_t>& cp = cands[ci].pairs;
    const int rows = (int)cp.size() / 2;
    int valid = 0;
    // ---- checkCorrespondences (PE:1312-1501)
    if (rows < minNumCorr) {
      flag = 6;
    } else {
      double mean_rep[16][3];
      std::memset(mean_rep, 0, sizeof(mean_rep));
      const std::vector<int> cmb = combinations3(rows);
      const int Nc = (int)cmb.size() / 3;
      int num_valid = 0;
      for (int q = 0; q < Nc; ++q) {
        const int* s = &cmb[3 * q];
        double fv[3][3], wp[3][3];
        for (int k = 0; k < 3; ++k)
          for (int d = 0; d < 3; ++d) {
            wp[k][d] = markers[3 * (cp[2 * s[k]] - 1) + d];
            fv[k][d] = iv[3 * (cp[2 * s[k] + 1] - 1) + d];
          }
        std::vector<int> un;  // unused correspondence rows, in row order
        for (int l = 0; l < rows; ++l)
          if (l != s[0] && l != s[1] && l != s[2]) un.push_back(l);
        Pose34 sol[4];
        if (p3p(fv, wp, sol) != 0) {
          flag = 9;
          continue;
        }
        double min_err = INFINITY;
        int best = -1;
        bool any_valid = false;
        for (int j = 0; j < 4; ++j) {
          if (!is_finite34(sol[j])) continue;
          double inv[16];
          inverse44(sol[j], inv);
          // calculateSquaredReprojectionErrorAndCertainty (PE:1087-1132): index-paired distances
          const int nu = (int)un.size();
          double dist[16];
          for (int a = 0; a < nu; ++a) {
            double uv[2];
            project44(K, inv, markers + 3 * (cp[2 * un[a]] - 1), uv);
            dist[a] = sqdist2(blobs + 2 * (cp[2 * un[a] + 1] - 1), uv);
          }
          double sq_err = 0;
          int ncorr = 0;
          for (int it = 1; it <= nu; ++it) {
            int r = 0;  // Eigen minCoeff: start at coeff(0), strict '<'
            double mv = dist[0];
            for (int a = 1; a < nu; ++a)
              if (dist[a] < mv) {
                mv = dist[a];
                r = a;
              }
            if (mv <= tol2) {
              sq_err += mv;
              ncorr++;
              dist[r] = INFINITY;
            } else {
              break;
            }
          }
          const double certainty = (double)ncorr / nu;
          if (certainty >= prm->certainty_threshold) {
            any_valid = true;
            if (sq_err < min_err) {
              min_err = sq_err;
              best = j;
            }
          }
        }
        if (any_valid) {
          num_valid++;
          double inv[16];
          inverse44(sol[best], inv);
          if (N_particle >= n_est && prm->use_pf) {
            for (int i = 0; i < 12; ++i) particles[12 * (size_t)(N_particle - n_est) + i] = inv[i];
            n_est++;
          }
          for (int jj = 0; jj < M; ++jj) {
            const double* X = markers + 3 * jj;
            for (int r = 0; r < 3; ++r) {
              const double v = inv[4 * r + 0] * X[0] + inv[4 * r + 1] * X[1] + inv[4 * r + 2] * X[2] + inv[4 * r + 3] * 1.0;
              mean_rep[jj][r] = mean_rep[jj][r] + v;
            }
          }
        }
      }
      if ((double)num_valid / Nc >= prm->valid_corr_threshold) {
        valid = 1;
        double rep[48];
        for (int jj = 0; jj < M; ++jj)
          for (int r = 0; r < 3; ++r) rep[3 * jj + r] = mean_rep[jj][r] / num_valid;
        double T12[12];
        compute_transformation(M, markers, rep, T12);
        if (valid && n_est < N_particle && first == 0) {
          first = 1;
          out->first_match = (int)ci;
          std::memcpy(out->predicted_pose, T12, sizeof(T12));
          out->n_corr = rows;
          for (int k = 0; k < 2 * rows; ++k) out->corr[k] = cp[k];
        }
      } else {
        flag = num_valid > 0 ? 7 : 8;
      }
    }
    if (valid && n_est < N_particle) found = 1;
  }
  const int n_reasonable = n_est - 1;
  while (n_est < N_particle && found && prm->use_pf) {
    for (int i = 0; i < 12; ++i)
      particles[12 * (size_t)(N_particle - n_est) + i] = particles[12 * (size_t)(N_particle - n_est + n_reasonable) + i];
    n_est++;
  }
  out->found = found;
  out->n_estimates = n_reasonable;
  out->flag_fail = found ? 0 : flag;
  return 0;
}

}  // extern "C"
