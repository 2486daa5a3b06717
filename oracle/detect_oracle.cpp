// =====================================================================================================
//  detect_oracle.cpp — CPU restatement of the reference's LED detector (LEDDetector::findLeds).
//
//  TEST INFRASTRUCTURE ONLY (same contract as pf_oracle.cpp): the checker for pfmpe_find_leds and the
//  CPU baseline scripts/bench_detect.py times.  Never the product.
//
//  Reference: pf_mpe_lib/src/led_detector.cpp:46-215 ("LD").  The detector is OpenCV calls; OpenCV is not
//  installed here, so each call is restated from OpenCV 2.4's published algorithm (the version of the
//  reference's ROS Indigo / Ubuntu 14.04 target, README.md:15):
//    * cv::threshold THRESH_TOZERO (active markers) / THRESH_BINARY_INV                      LD:56-59
//    * cv::GaussianBlur, ksize (0,0) -> cvRound(sigma*3*2+1)|1 for 8U; getGaussianKernel(n, sigma,
//      CV_32F); 8U separable path: both kernels converted to int with 8 fraction bits, int row pass,
//      int column pass, (sum + 2^15) >> 16 saturated; BORDER_DEFAULT = BORDER_REFLECT_101 on the
//      ROI-sized thresholded image                                                             LD:62-67
//    * cv::findContours(RETR_EXTERNAL, CHAIN_APPROX_NONE): 2.4's cvStartFindContours first zeroes the
//      outermost 1-pixel frame of the image ("contours touching the image border will be clipped"),
//      then Suzuki-Abe outer border following from the
//      raster-first pixel of every 8-connected component, with icvFetchContour's direction table
//      (0 = +x, counter-clockwise in image coordinates) and stopping rule; contours are returned in
//      reverse discovery order (the C API prepends each new contour to the sequence)            LD:72
//    * cv::contourArea (|shoelace| / 2), cv::boundingRect, cv::moments(contour) (polygon moments,
//      Green's theorem, sign-normalised), the size / aspect / circularity filter with the reference's
//      integer `rect.width / 2`                                                                LD:86-108
//    * cv::undistortPoints(K, D, noArray(), P = K): 5 fixed iterations of the plumb_bob inverse, then
//      P (cvUndistortPoints)                                                                   LD:192-209
//  Parity status: PARITY UNPINNED (no OpenCV here, no reference fixtures).  Not restated: components
//  nested inside another component's hole (RETR_EXTERNAL drops them; this restatement keeps them),
//  the exposure-time control (LD:122-160, a camera side effect) and the simulated occlusions / false
//  detections (LD:170-183, test hooks off by default).
// =====================================================================================================
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

namespace {

int border_reflect101(int p, int len) {  // cv::borderInterpolate(BORDER_REFLECT_101)
  if (len == 1) return 0;
  while (p < 0 || p >= len) {
    if (p < 0) p = -p;
    else p = 2 * len - p - 2;
  }
  return p;
}

// getGaussianKernel(n, sigma, CV_32F) (imgproc/src/smooth.cpp, OpenCV 2.4) -> int kernel with 8
// fraction bits (Mat::convertTo(CV_32S, 256): cvRound)
std::vector<int> gaussian_kernel_q8(int n, double sigma) {
  std::vector<float> cf(n);
  const double sigmaX = sigma > 0 ? sigma : ((n - 1) * 0.5 - 1) * 0.3 + 0.8;
  const double scale2X = -0.5 / (sigmaX * sigmaX);
  double sum = 0;
  for (int i = 0; i < n; ++i) {
    const double x = i - (n - 1) * 0.5;
    cf[i] = (float)std::exp(scale2X * x * x);
    sum += cf[i];
  }
  sum = 1. / sum;
  std::vector<int> k(n);
  for (int i = 0; i < n; ++i) {
    cf[i] = (float)(cf[i] * sum);
    k[i] = (int)std::nearbyint((double)cf[i] * 256.0);
  }
  return k;
}

struct Contour {
  std::vector<int> x, y;  // points in ROI coordinates
};

// icvFetchContour (CHAIN_APPROX_NONE) on a mask with a zero frame: start = raster-first pixel.
// deltas: 0 +x, 1 (+x,-y), 2 -y, 3 (-x,-y), 4 -x, 5 (-x,+y), 6 +y, 7 (+x,+y)
Contour fetch_contour(const std::vector<uint8_t>& m, int W, int x0, int y0) {
  static const int dx[8] = {1, 1, 0, -1, -1, -1, 0, 1};
  static const int dy[8] = {0, -1, -1, -1, 0, 1, 1, 1};
  auto at = [&](int x, int y) { return m[(size_t)(y + 1) * (W + 2) + (x + 1)]; };
  Contour c;
  int s = 4;
  const int s_end0 = 4;
  int x1 = 0, y1 = 0;
  do {
    s = (s - 1) & 7;
    x1 = x0 + dx[s];
    y1 = y0 + dy[s];
  } while (at(x1, y1) == 0 && s != s_end0);
  if (s == s_end0) {  // single-pixel domain
    c.x.push_back(x0);
    c.y.push_back(y0);
    return c;
  }
  int x3 = x0, y3 = y0, px = x0, py = y0;
  for (;;) {
    int x4, y4;
    for (;;) {
      ++s;
      x4 = x3 + dx[s & 7];
      y4 = y3 + dy[s & 7];
      if (at(x4, y4) != 0) break;
    }
    s &= 7;
    c.x.push_back(px);
    c.y.push_back(py);
    px += dx[s];
    py += dy[s];
    if (x4 == x0 && y4 == y0 && x3 == x1 && y3 == y1) break;
    x3 = x4;
    y3 = y4;
    s = (s + 4) & 7;
  }
  return c;
}

}  // namespace

extern "C" {

typedef struct {
  int threshold_value;
  double gaussian_sigma;
  double min_blob_area, max_blob_area;
  double max_width_height_distortion, max_circular_distortion;
  int active_markers;
  int roi_x, roi_y, roi_w, roi_h;
} OrcDetectParams;

// Stage outputs for tests: mask (roi_h x roi_w: 1 = nonzero after the blur and the frame zeroing; may
// be NULL).
// Output: up to max_out detections in findContours order: distorted (float, full-image px) and
// undistorted (double(float)) centres; returns the count, or < 0 on bad arguments.
int orc_find_leds(const uint8_t* image, int width, int height, int pitch, const OrcDetectParams* p, const double* K,
                  const double* D, int max_out, float* distorted, double* undistorted, double* areas,
                  uint8_t* mask_out) {
  if (!image || !p || width < 1 || height < 1 || pitch < width) return -1;
  const int rx = p->roi_x, ry = p->roi_y, W = p->roi_w, H = p->roi_h;
  if (rx < 0 || ry < 0 || W < 1 || H < 1 || rx + W > width || ry + H > height) return -1;
  // threshold (LD:56-59)
  std::vector<int> bw((size_t)W * H);
  for (int y = 0; y < H; ++y)
    for (int x = 0; x < W; ++x) {
      const int v = image[(size_t)(ry + y) * pitch + rx + x];
      bw[(size_t)y * W + x] = p->active_markers ? (v > p->threshold_value ? v : 0) : (v > p->threshold_value ? 0 : 255);
    }
  // Gaussian blur (LD:62-67): row pass to int, column pass, fixed-point cast with 16 bits
  int n = (int)std::nearbyint(p->gaussian_sigma * 3 * 2 + 1) | 1;  // cvRound
  if (p->gaussian_sigma <= 0) n = 1;
  const std::vector<int> k = gaussian_kernel_q8(n, p->gaussian_sigma);
  const int r = n / 2;
  std::vector<int> rows((size_t)W * H);
  for (int y = 0; y < H; ++y)
    for (int x = 0; x < W; ++x) {
      int s = 0;
      for (int i = 0; i < n; ++i) s += k[i] * bw[(size_t)y * W + border_reflect101(x + i - r, W)];
      rows[(size_t)y * W + x] = s;
    }
  std::vector<uint8_t> m((size_t)(W + 2) * (H + 2), 0);  // 1-pixel zero frame (findContours' own border)
  for (int y = 0; y < H; ++y)
    for (int x = 0; x < W; ++x) {
      long long s = 0;
      for (int i = 0; i < n; ++i) s += (long long)k[i] * rows[(size_t)border_reflect101(y + i - r, H) * W + x];
      long long v = (s + (1 << 15)) >> 16;
      v = v < 0 ? 0 : (v > 255 ? 255 : v);
      const bool frame = x == 0 || y == 0 || x == W - 1 || y == H - 1;  // zeroed by cvStartFindContours
      const uint8_t b = (v != 0 && !frame) ? 1 : 0;
      m[(size_t)(y + 1) * (W + 2) + (x + 1)] = b;
      if (mask_out) mask_out[(size_t)y * W + x] = b;
    }
  // findContours(RETR_EXTERNAL, CHAIN_APPROX_NONE): one outer border per 8-connected component,
  // discovered in raster order at the component's first pixel
  std::vector<int> comp((size_t)W * H, -1);
  std::vector<Contour> found;
  std::vector<int> stack;
  for (int y = 0; y < H; ++y)
    for (int x = 0; x < W; ++x) {
      const size_t i = (size_t)y * W + x;
      if (!m[(size_t)(y + 1) * (W + 2) + (x + 1)] || comp[i] >= 0) continue;
      const int id = (int)found.size();
      comp[i] = id;
      stack.assign(1, (int)i);
      while (!stack.empty()) {  // flood fill the component (8-connectivity)
        const int q = stack.back();
        stack.pop_back();
        const int qx = q % W, qy = q / W;
        for (int ddy = -1; ddy <= 1; ++ddy)
          for (int ddx = -1; ddx <= 1; ++ddx) {
            const int nx = qx + ddx, ny = qy + ddy;
            if (nx < 0 || ny < 0 || nx >= W || ny >= H) continue;
            const size_t ni = (size_t)ny * W + nx;
            if (m[(size_t)(ny + 1) * (W + 2) + (nx + 1)] && comp[ni] < 0) {
              comp[ni] = id;
              stack.push_back((int)ni);
            }
          }
      }
      found.push_back(fetch_contour(m, W, x, y));
    }
  std::reverse(found.begin(), found.end());
  // per contour: area, bounding rect, moments, filter (LD:86-108); undistort (LD:192-209)
  const double fx = K[0], fy = K[4], cx = K[2], cy = K[5];
  const double ifx = 1. / fx, ify = 1. / fy;
  int out = 0;
  for (const Contour& c : found) {
    const int np = (int)c.x.size();
    double a00 = 0, a10 = 0, a01 = 0, area2 = 0;
    int minx = c.x[0], maxx = c.x[0], miny = c.y[0], maxy = c.y[0];
    double xi_1 = c.x[np - 1], yi_1 = c.y[np - 1];
    for (int i = 0; i < np; ++i) {
      const double xi = c.x[i], yi = c.y[i];
      const double dxy = xi_1 * yi - xi * yi_1;
      a00 += dxy;
      a10 += dxy * (xi_1 + xi);
      a01 += dxy * (yi_1 + yi);
      area2 += xi_1 * yi - yi_1 * xi;
      xi_1 = xi;
      yi_1 = yi;
      minx = std::min(minx, c.x[i]);
      maxx = std::max(maxx, c.x[i]);
      miny = std::min(miny, c.y[i]);
      maxy = std::max(maxy, c.y[i]);
    }
    double m00 = 0, m10 = 0, m01 = 0;
    if (std::fabs(a00) > 1.1920928955078125e-07) {  // FLT_EPSILON
      const double s2 = a00 > 0 ? 0.5 : -0.5, s6 = a00 > 0 ? 1.0 / 6 : -1.0 / 6;
      m00 = a00 * s2;
      m10 = a10 * s6;
      m01 = a01 * s6;
    }
    const double area = std::fabs(area2 * 0.5);
    const int rw = maxx - minx + 1, rh = maxy - miny + 1;
    const double pi = 3.1415926535897932384626433832795;
    const bool keep = area >= p->min_blob_area && area <= p->max_blob_area &&
                      std::fabs(1 - std::min((double)rw / (double)rh, (double)rh / (double)rw)) <= p->max_width_height_distortion &&
                      std::fabs(1 - (area / (pi * std::pow(rw / 2, 2)))) <= p->max_circular_distortion &&
                      std::fabs(1 - (area / (pi * std::pow(rh / 2, 2)))) <= p->max_circular_distortion;
    if (!keep) continue;
    const float mcx = (float)(m10 / m00) + (float)rx;
    const float mcy = (float)(m01 / m00) + (float)ry;
    if (out < max_out) {
      if (distorted) {
        distorted[2 * out] = mcx;
        distorted[2 * out + 1] = mcy;
      }
      if (areas) areas[out] = area;
      if (undistorted) {
        double x = ((double)mcx - cx) * ifx, y = ((double)mcy - cy) * ify;
        const double x0 = x, y0 = y;
        for (int j = 0; j < 5; ++j) {
          const double r2 = x * x + y * y;
          const double icdist = 1. / (1 + ((D[4] * r2 + D[1]) * r2 + D[0]) * r2);
          const double deltaX = 2 * D[2] * x * y + D[3] * (r2 + 2 * x * x);
          const double deltaY = D[2] * (r2 + 2 * y * y) + 2 * D[3] * x * y;
          x = (x0 - deltaX) * icdist;
          y = (y0 - deltaY) * icdist;
        }
        const double xx = K[0] * x + K[1] * y + K[2];
        const double yy = K[3] * x + K[4] * y + K[5];
        const double ww = 1. / (K[6] * x + K[7] * y + K[8]);
        undistorted[2 * out] = (double)(float)(xx * ww);
        undistorted[2 * out + 1] = (double)(float)(yy * ww);
      }
    }
    ++out;
  }
  return out;
}

}  // extern "C"
