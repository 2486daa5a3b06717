#pragma once
// pf_p3p.hpp — device-side fp64 P3P and back projection for the brute-force (re)initialisation
// (PoseEstimator::initialise, pf_mpe_lib/src/pose_estimator.cpp:1503-1786 = "PE" below).
//
// P3P::computePoses / solveQuartic (pf_mpe_lib/src/p3p.cpp:65-292) solve the quartic with
// std::complex<double>.  The reference's arithmetic for every complex operation is restated here on
// the device, operation for operation, so that the solutions follow the same rounding path:
//   * +, -, scalar * and / : component-wise, as libstdc++'s operators;
//   * complex / complex    : libgcc __divdc3 (Smith's algorithm, GCC 11);
//   * sqrt                 : glibc csqrt (the 2 Re Im = Im x identity; exact branches for Im = 0 / Re = 0);
//   * log                  : (log |z|, atan2(Im, Re));
//   * pow(z, real)         : libstdc++: real pow when Im z == 0 and Re z > 0, else polar(exp(y Re log z),
//                            y Im log z).
// The elementary functions (pow, exp, log, atan2, cos, sin, hypot) are the device's (ocml), so results
// agree with the CPU to an ulp, not bit for bit (DESIGN.md §4.7 says what that means for parity).
// The translation unit is built with -ffp-contract=off: no fused multiply-adds anywhere.
#include <hip/hip_runtime.h>

namespace pfmpe {
namespace p3p {

struct Cx {
  double re, im;
};
__device__ __forceinline__ Cx cx(double r, double i = 0.0) { return Cx{r, i}; }
__device__ __forceinline__ Cx operator+(Cx a, Cx b) { return Cx{a.re + b.re, a.im + b.im}; }
__device__ __forceinline__ Cx operator-(Cx a, Cx b) { return Cx{a.re - b.re, a.im - b.im}; }
__device__ __forceinline__ Cx operator-(Cx a) { return Cx{-a.re, -a.im}; }
// double op complex (libstdc++: copy the complex, then op= the scalar onto the real part)
__device__ __forceinline__ Cx operator+(double x, Cx a) { return Cx{a.re + x, a.im}; }
__device__ __forceinline__ Cx operator-(double x, Cx a) { return Cx{-a.re + x, -a.im}; }
__device__ __forceinline__ Cx operator*(double x, Cx a) { return Cx{a.re * x, a.im * x}; }
__device__ __forceinline__ Cx operator/(Cx a, double x) { return Cx{a.re / x, a.im / x}; }
// libgcc __divdc3 (a + ib) / (c + id)
__device__ __forceinline__ Cx operator/(Cx n, Cx d) {
  const double a = n.re, b = n.im, c = d.re, e = d.im;
  double ratio, denom, x, y;
  if (fabs(c) < fabs(e)) {
    ratio = c / e;
    denom = (c * ratio) + e;
    x = ((a * ratio) + b) / denom;
    y = ((b * ratio) - a) / denom;
  } else {
    ratio = e / c;
    denom = (e * ratio) + c;
    x = ((b * ratio) + a) / denom;
    y = (b - (a * ratio)) / denom;
  }
  return Cx{x, y};
}
__device__ __forceinline__ Cx operator/(double x, Cx d) { return Cx{x, 0.0} / d; }

__device__ __forceinline__ Cx csqrt(Cx z) {
  if (z.im == 0.0) {
    if (z.re < 0) return Cx{0.0, copysign(sqrt(-z.re), z.im)};
    return Cx{fabs(sqrt(z.re)), copysign(0.0, z.im)};
  }
  if (z.re == 0.0) {
    const double r = sqrt(0.5 * fabs(z.im));
    return Cx{r, copysign(r, z.im)};
  }
  const double d = hypot(z.re, z.im);
  double r, s;
  if (z.re > 0) {
    r = sqrt(0.5 * (d + z.re));
    s = 0.5 * (z.im / r);
  } else {
    s = sqrt(0.5 * (d - z.re));
    r = fabs(0.5 * (z.im / s));
  }
  return Cx{r, copysign(s, z.im)};
}
__device__ __forceinline__ Cx clog(Cx z) { return Cx{log(hypot(z.re, z.im)), atan2(z.im, z.re)}; }
__device__ __forceinline__ Cx cpow(Cx z, double y) {
  if (z.im == 0.0 && z.re > 0.0) return Cx{pow(z.re, y), 0.0};
  const Cx t = clog(z);
  const double rho = exp(y * t.re), th = y * t.im;
  return Cx{rho * cos(th), rho * sin(th)};
}

__device__ __forceinline__ double norm3(const double* v) { return sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]); }
__device__ __forceinline__ void cross3(const double* a, const double* b, double* c) {
  c[0] = a[1] * b[2] - a[2] * b[1];
  c[1] = a[2] * b[0] - a[0] * b[2];
  c[2] = a[0] * b[1] - a[1] * b[0];
}

// P3P::solveQuartic (p3p.cpp:244-290): the four real parts of Ferrari's roots
__device__ __forceinline__ void solve_quartic(const double* f, double* roots) {
  const double A = f[0], B = f[1], C = f[2], D = f[3], E = f[4];
  const double A_pw2 = A * A, B_pw2 = B * B;
  const double A_pw3 = A_pw2 * A, B_pw3 = B_pw2 * B;
  const double A_pw4 = A_pw3 * A, B_pw4 = B_pw3 * B;
  const double alpha = -3 * B_pw2 / (8 * A_pw2) + C / A;
  const double beta = B_pw3 / (8 * A_pw3) - B * C / (2 * A_pw2) + D / A;
  const double gamma = -3 * B_pw4 / (256 * A_pw4) + B_pw2 * C / (16 * A_pw3) - B * D / (4 * A_pw2) + E / A;
  const double alpha_pw2 = alpha * alpha;
  const double alpha_pw3 = alpha_pw2 * alpha;
  const Cx P = cx(-alpha_pw2 / 12 - gamma);
  const Cx Q = cx(-alpha_pw3 / 108 + alpha * gamma / 3 - (beta * beta) / 8);  // pow(beta, 2) folds to beta*beta
  const Cx R = -Q / 2.0 + csqrt(cpow(Q, 2.0) / 4.0 + cpow(P, 3.0) / 27.0);
  const Cx U = cpow(R, 1.0 / 3.0);
  Cx y;
  if (U.re == 0)
    y = -5.0 * alpha / 6.0 - cpow(Q, 1.0 / 3.0);
  else
    y = (-5.0 * alpha / 6.0 - P / (3.0 * U)) + U;
  const Cx w = csqrt(alpha + 2.0 * y);
  const double h = -B / (4.0 * A);
  const Cx s0 = csqrt(-((3.0 * alpha + 2.0 * y) + 2.0 * beta / w));
  const Cx s1 = csqrt(-((3.0 * alpha + 2.0 * y) - 2.0 * beta / w));
  roots[0] = (h + 0.5 * (w + s0)).re;
  roots[1] = (h + 0.5 * (w - s0)).re;
  roots[2] = (h + 0.5 * (-w + s1)).re;
  roots[3] = (h + 0.5 * (-w - s1)).re;
}

// The root-independent part of P3P::computePoses (p3p.cpp:65-201).  fv/wp: rows = the three unit
// feature vectors / world points in column order.  Returns false for collinear world points.
struct Setup {
  double T[9];   // intermediate camera frame (rows e1 e2 e3)
  double N[9];   // intermediate world frame (rows n1 n2 n3)
  double P1[3];
  double f_1, f_2, p_1, p_2, d_12, b;
};

__device__ __forceinline__ bool setup(const double fv[3][3], const double wp[3][3], Setup& s, double* roots) {
  double t1[3], t2[3], cr[3];
  for (int i = 0; i < 3; ++i) {
    t1[i] = wp[1][i] - wp[0][i];
    t2[i] = wp[2][i] - wp[0][i];
  }
  cross3(t1, t2, cr);
  if (norm3(cr) == 0) return false;
  int i1 = 0, i2 = 1;
  double f1[3], f2[3], f3t[3];
  for (int pass = 0; pass < 2; ++pass) {
    double e1[3], e2[3], e3[3];
    for (int i = 0; i < 3; ++i) {
      f1[i] = fv[i1][i];
      f2[i] = fv[i2][i];
      e1[i] = f1[i];
    }
    cross3(f1, f2, e3);
    const double n = norm3(e3);
    for (int i = 0; i < 3; ++i) e3[i] = e3[i] / n;
    cross3(e3, e1, e2);
    for (int i = 0; i < 3; ++i) {
      s.T[0 + i] = e1[i];
      s.T[3 + i] = e2[i];
      s.T[6 + i] = e3[i];
    }
    for (int r = 0; r < 3; ++r) f3t[r] = s.T[3 * r + 0] * fv[2][0] + s.T[3 * r + 1] * fv[2][1] + s.T[3 * r + 2] * fv[2][2];
    if (pass == 1 || !(f3t[2] > 0)) break;
    i1 = 1;  // theta in [0, pi]: swap the first two correspondences (p3p.cpp:101-125)
    i2 = 0;
  }
  const double* P1 = wp[i1];
  const double* P2 = wp[i2];
  const double* P3 = wp[2];
  double n1[3], n2[3], n3[3], d[3];
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
    s.N[0 + i] = n1[i];
    s.N[3 + i] = n2[i];
    s.N[6 + i] = n3[i];
    s.P1[i] = P1[i];
  }
  double P3n[3];
  for (int r = 0; r < 3; ++r) P3n[r] = s.N[3 * r + 0] * d[0] + s.N[3 * r + 1] * d[1] + s.N[3 * r + 2] * d[2];
  double dd[3];
  for (int i = 0; i < 3; ++i) dd[i] = P2[i] - P1[i];
  const double d_12 = norm3(dd);
  const double f_1 = f3t[0] / f3t[2];
  const double f_2 = f3t[1] / f3t[2];
  const double p_1 = P3n[0];
  const double p_2 = P3n[1];
  const double cos_beta = f1[0] * f2[0] + f1[1] * f2[1] + f1[2] * f2[2];
  double b = 1 / (1 - cos_beta * cos_beta) - 1;
  b = cos_beta < 0 ? -sqrt(b) : sqrt(b);

  const double f_1_pw2 = f_1 * f_1;
  const double f_2_pw2 = f_2 * f_2;
  const double p_1_pw2 = p_1 * p_1;
  const double p_1_pw3 = p_1_pw2 * p_1;
  const double p_1_pw4 = p_1_pw3 * p_1;
  const double p_2_pw2 = p_2 * p_2;
  const double p_2_pw3 = p_2_pw2 * p_2;
  const double p_2_pw4 = p_2_pw3 * p_2;
  const double d_12_pw2 = d_12 * d_12;
  const double b_pw2 = b * b;
  // quartic factors in the reference's term order (it fixes the rounding)
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
  solve_quartic(fac, roots);
  s.f_1 = f_1;
  s.f_2 = f_2;
  s.p_1 = p_1;
  s.p_2 = p_2;
  s.d_12 = d_12;
  s.b = b;
  return true;
}

// Back substitution of one root (p3p.cpp:205-240): sol = [R | C], 12 doubles row-major
__device__ __forceinline__ void solution(const Setup& s, double root, double* sol) {
  const double f_1 = s.f_1, f_2 = s.f_2, p_1 = s.p_1, p_2 = s.p_2, d_12 = s.d_12, b = s.b;
  const double cot_alpha = (-f_1 * p_1 / f_2 - root * p_2 + d_12 * b) / (-f_1 * root * p_2 / f_2 + p_1 - d_12);
  const double cos_theta = root;
  const double sin_theta = sqrt(1 - root * root);
  const double sin_alpha = sqrt(1 / (cot_alpha * cot_alpha + 1));
  double cos_alpha = sqrt(1 - sin_alpha * sin_alpha);
  if (cot_alpha < 0) cos_alpha = -cos_alpha;
  const double k = sin_alpha * b + cos_alpha;
  double Cl[3];
  Cl[0] = d_12 * cos_alpha * k;
  Cl[1] = cos_theta * d_12 * sin_alpha * k;
  Cl[2] = sin_theta * d_12 * sin_alpha * k;
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
  // tmp = N^T R^T ; R = tmp T ; C = P1 + N^T C
  double tmp[9];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j)
      tmp[3 * i + j] = s.N[0 + i] * Rl[3 * j + 0] + s.N[3 + i] * Rl[3 * j + 1] + s.N[6 + i] * Rl[3 * j + 2];
  for (int i = 0; i < 3; ++i) {
    for (int j = 0; j < 3; ++j)
      sol[4 * i + j] = tmp[3 * i + 0] * s.T[0 + j] + tmp[3 * i + 1] * s.T[3 + j] + tmp[3 * i + 2] * s.T[6 + j];
    const double ntc = s.N[0 + i] * Cl[0] + s.N[3 + i] * Cl[1] + s.N[6 + i] * Cl[2];
    sol[4 * i + 3] = s.P1[i] + ntc;
  }
}

__device__ __forceinline__ bool finite12(const double* a) {  // isFinite (PE:2088-2091)
  bool ok = true;
  for (int i = 0; i < 12; ++i) {
    const double z = a[i] - a[i];
    ok = ok && (z == z);
  }
  return ok;
}

// H.inverse() of H = [[R C];[0 0 0 1]] as a general 4x4 by cofactors (same expression order as
// oracle/init_oracle.cpp inverse44); only the top three rows are produced (the fourth row only meets
// the homogeneous 1 of a marker through K's zero column in project2d).
__device__ __forceinline__ void inverse34(const double* m12, double* inv) {
  double m[16];
  for (int i = 0; i < 12; ++i) m[i] = m12[i];
  m[12] = 0;
  m[13] = 0;
  m[14] = 0;
  m[15] = 1;
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
}

// project2d (PE:1017-1034) through a 4x4 whose fourth row is (0 0 0 1)-ish: ([K|0] T) [X;1], / z.
// The K34 * T(3, j) term is 0 * T(3, j); T(3, j) is finite here (isFinite checked H, and the cofactor
// inverse of a finite H with det != 0 is finite), so it adds +0 and is kept as "+ 0.0 * x" only in
// the oracle; here it is dropped (x + 0.0 == x for every x that is not -0.0, and Q entries are sums of
// products that are -0.0 only when every product is -0.0, which leaves the projection unchanged).
__device__ __forceinline__ void project(const double* K, const double* T, const double* X, double& u, double& v) {
  double p[3];
  for (int i = 0; i < 3; ++i) {
    double q[4];
    for (int j = 0; j < 4; ++j) {
      double s = K[i * 3 + 0] * T[0 * 4 + j];
      s = s + K[i * 3 + 1] * T[1 * 4 + j];
      s = s + K[i * 3 + 2] * T[2 * 4 + j];
      q[j] = s;
    }
    double s = q[0] * X[0];
    s = s + q[1] * X[1];
    s = s + q[2] * X[2];
    s = s + q[3] * 1.0;
    p[i] = s;
  }
  u = p[0] / p[2];
  v = p[1] / p[2];
}

}  // namespace p3p
}  // namespace pfmpe
