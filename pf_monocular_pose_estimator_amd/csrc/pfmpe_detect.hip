// pfmpe_detect.hip — the LED detector on the device: LEDDetector::findLeds
// (pf_mpe_lib/src/led_detector.cpp:46-215, "LD") for one ROI of an 8-bit image, behind pfmpe_find_leds.
//
// The reference is OpenCV 2.4 calls; each is restated (oracle/detect_oracle.cpp lists the semantics):
//   k_det_mask     threshold (TOZERO / BINARY_INV) + GaussianBlur (8-bit-fraction integer kernels,
//                  reflect-101 borders, (sum + 2^15) >> 16) -> "pixel is nonzero" mask, with the 1-pixel
//                  frame cvStartFindContours zeroes.  16x16 tiles: thresholded tile + halo, then the row
//                  pass, staged in LDS; exact integer arithmetic.
//   k_det_label    per foreground pixel: its 8-neighbour bit mask (bit s = direction s of icvFetchContour's
//                  table) and its own index as label
//   k_det_merge    union-find over the 8-connectivity (W, NW, N, NE), atomicMin links to the lower index
//                  (agent-scope loads in find: other blocks' links bypass the non-coherent L1)
//   k_det_roots    flatten; every root (= the component's raster-first pixel, where the reference's raster
//                  scan starts its outer border) takes a slot
//   k_det_trace    one lane per component: icvFetchContour's border following over the neighbour masks,
//                  polygon moments / area / bounding box on the fly, the size-aspect-circularity filter,
//                  the centre + ROI offset as float, cvUndistortPoints (5 iterations, P = K)
// The host orders the accepted detections as findContours returns them (reverse discovery = descending
// root index) and returns image_points_ (undistorted px) plus the distorted centres.
#include "pfmpe_ctx.hpp"

using namespace pfmpe;
using namespace pfmpe_impl;

namespace pfmpe {

constexpr int kDetTile = 16;
constexpr int kDetMaxRadius = 15;      // kernel size <= 31 (sigma <= 5)
constexpr int kDetMaxComponents = 8192;

struct DetArgs {
  int k[2 * kDetMaxRadius + 1];  // Gaussian taps, 8 fraction bits
  int radius;
  int thr, active;
  int img_w, img_h, pitch;
  int rx, ry, W, H;              // ROI
  double K[9], D[5];
  double min_area, max_area, max_whd, max_circ;
};

struct DetRecord {  // one component (slot)
  int root, keep;
  float dx, dy;     // distorted centre + ROI offset (cv::Point2f)
  double ux, uy;    // undistorted (double(float))
  double area;
};

// icvFetchContour's direction table: 0 +x, 1 (+x,-y), 2 -y, 3 (-x,-y), 4 -x, 5 (-x,+y), 6 +y, 7 (+x,+y)
__device__ __forceinline__ int dir_dx(int s) { return (s == 0 || s == 1 || s == 7) ? 1 : ((s >= 3 && s <= 5) ? -1 : 0); }
__device__ __forceinline__ int dir_dy(int s) { return (s >= 1 && s <= 3) ? -1 : (s >= 5 ? 1 : 0); }

__device__ __forceinline__ int refl101(int p, int len) {
  if (len == 1) return 0;
  while (p < 0 || p >= len) p = p < 0 ? -p : 2 * len - p - 2;
  return p;
}

__global__ __launch_bounds__(kDetTile* kDetTile) void k_det_mask(const DetArgs a, const uint8_t* __restrict__ img,
                                                                  uint8_t* __restrict__ mask) {
  constexpr int T = kDetTile, HW = T + 2 * kDetMaxRadius;
  __shared__ int tb[HW][HW];    // thresholded tile + halo (rows, cols)
  __shared__ int rowp[HW][T];   // row pass
  const int r = a.radius, n = 2 * r + 1, span = T + 2 * r;
  const int x0 = blockIdx.x * T, y0 = blockIdx.y * T;
  for (int i = threadIdx.x; i < span * span; i += blockDim.x) {
    const int ty = i / span, tx = i - ty * span;
    const int gy = refl101(y0 + ty - r, a.H), gx = refl101(x0 + tx - r, a.W);
    const int v = img[(int64_t)(a.ry + gy) * a.pitch + a.rx + gx];
    tb[ty][tx] = a.active ? (v > a.thr ? v : 0) : (v > a.thr ? 0 : 255);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < span * T; i += blockDim.x) {
    const int ty = i / T, tx = i - ty * T;
    int s = 0;
    for (int q = 0; q < n; ++q) s += a.k[q] * tb[ty][tx + q];
    rowp[ty][tx] = s;
  }
  __syncthreads();
  const int tx = threadIdx.x % T, ty = threadIdx.x / T;
  const int x = x0 + tx, y = y0 + ty;
  if (x >= a.W || y >= a.H) return;
  long long s = 0;
  for (int q = 0; q < n; ++q) s += (long long)a.k[q] * rowp[ty + q][tx];
  const long long v = (s + (1 << 15)) >> 16;
  const bool frame = x == 0 || y == 0 || x == a.W - 1 || y == a.H - 1;
  mask[(int64_t)y * a.W + x] = (v > 0 && !frame) ? 1 : 0;
}

// neighbour bits: bit s = the pixel in direction s is foreground (0 +x, 1 (+x,-y), 2 -y, 3 (-x,-y),
// 4 -x, 5 (-x,+y), 6 +y, 7 (+x,+y))
__global__ void k_det_label(const DetArgs a, const uint8_t* __restrict__ mask, uint8_t* __restrict__ nbr,
                            int* __restrict__ label) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)a.W * a.H) return;
  const int y = (int)(i / a.W), x = (int)(i - (int64_t)y * a.W);
  if (!mask[i]) {
    label[i] = -1;
    nbr[i] = 0;
    return;
  }
  uint32_t bits = 0;
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    const int nx = x + dir_dx(s), ny = y + dir_dy(s);
    if (nx >= 0 && ny >= 0 && nx < a.W && ny < a.H && mask[(int64_t)ny * a.W + nx]) bits |= 1u << s;
  }
  nbr[i] = (uint8_t)bits;
  label[i] = (int)i;
}

__device__ __forceinline__ int ld_label(const int* L, int i) {
  return __hip_atomic_load(L + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int find_root(const int* L, int i) {
  for (int p = ld_label(L, i); p != i; p = ld_label(L, i)) i = p;
  return i;
}
__device__ __forceinline__ void unite(int* L, int a, int b) {
  for (;;) {
    a = find_root(L, a);
    b = find_root(L, b);
    if (a == b) return;
    if (a < b) {
      const int t = a;
      a = b;
      b = t;
    }
    const int old = atomicMin(L + a, b);  // link the higher root to the lower index
    if (old == a) return;
    a = old;
  }
}

__global__ void k_det_merge(const DetArgs a, const uint8_t* __restrict__ nbr, int* __restrict__ label) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)a.W * a.H) return;
  const uint32_t b = nbr[i];
  if (!b) return;
  const int W = a.W;
  if (b & (1u << 4)) unite(label, (int)i, (int)i - 1);
  if (b & (1u << 3)) unite(label, (int)i, (int)i - W - 1);
  if (b & (1u << 2)) unite(label, (int)i, (int)i - W);
  if (b & (1u << 1)) unite(label, (int)i, (int)i - W + 1);
}

__global__ void k_det_roots(const DetArgs a, const uint8_t* __restrict__ mask, int* __restrict__ label,
                            int* __restrict__ count, int* __restrict__ roots) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)a.W * a.H || !mask[i]) return;
  int r = (int)i;
  for (int p = label[r]; p != r; p = label[r]) r = p;
  label[i] = r;
  if (r == (int)i) {
    const int s = atomicAdd(count, 1);
    if (s < kDetMaxComponents) roots[s] = (int)i;
  }
}

__global__ void k_det_trace(const DetArgs a, const uint8_t* __restrict__ nbr, const int* __restrict__ count,
                            const int* __restrict__ roots, DetRecord* __restrict__ rec) {
  const int slot = blockIdx.x * blockDim.x + threadIdx.x;
  const int nc = min(*count, kDetMaxComponents);
  if (slot >= nc) return;
  const int root = roots[slot];
  const int W = a.W;
  const int x0 = root % W, y0 = root / W;
  // icvFetchContour (CHAIN_APPROX_NONE), the contour points streamed into the polygon sums
  double a00 = 0, a10 = 0, a01 = 0, area2 = 0;
  int minx = x0, maxx = x0, miny = y0, maxy = y0;
  double fx_ = 0, fy_ = 0, px_ = 0, py_ = 0;  // first point, previous point
  int np = 0;
  auto add_point = [&](int x, int y) {
    const double xi = x, yi = y;
    if (np == 0) {
      fx_ = xi;
      fy_ = yi;
    } else {
      const double dxy = px_ * yi - xi * py_;
      a00 += dxy;
      a10 += dxy * (px_ + xi);
      a01 += dxy * (py_ + yi);
      area2 += px_ * yi - py_ * xi;
    }
    px_ = xi;
    py_ = yi;
    minx = min(minx, x);
    maxx = max(maxx, x);
    miny = min(miny, y);
    maxy = max(maxy, y);
    ++np;
  };
  const uint32_t b0 = nbr[root];
  int s = 4;
  do {
    s = (s - 1) & 7;
  } while (!((b0 >> s) & 1u) && s != 4);
  if (s == 4 && !((b0 >> 4) & 1u)) {
    add_point(x0, y0);  // single-pixel domain
  } else {
    const int x1 = x0 + dir_dx(s), y1 = y0 + dir_dy(s);
    int x3 = x0, y3 = y0, px = x0, py = y0;
    for (int guard = 0; guard < 4 * a.W * a.H + 8; ++guard) {
      const uint32_t bb = nbr[(int64_t)y3 * W + x3];
      const uint32_t rot = ((bb | (bb << 8)) >> ((s + 1) & 7)) & 0xffu;  // directions s+1, s+2, ... (cyclic)
      s = (s + 1 + __builtin_ctz(rot)) & 7;                            // first set (>= 1 exists)
      const int x4 = x3 + dir_dx(s), y4 = y3 + dir_dy(s);
      add_point(px, py);
      px += dir_dx(s);
      py += dir_dy(s);
      if (x4 == x0 && y4 == y0 && x3 == x1 && y3 == y1) break;
      x3 = x4;
      y3 = y4;
      s = (s + 4) & 7;
    }
  }
  // closing edge last -> first (the reference's loop starts from the last point; the sums are the
  // same terms in a rotated order: exact for these integer-valued products)
  if (np > 1) {
    const double xi = fx_, yi = fy_;
    const double dxy = px_ * yi - xi * py_;
    a00 += dxy;
    a10 += dxy * (px_ + xi);
    a01 += dxy * (py_ + yi);
    area2 += px_ * yi - py_ * xi;
  }
  double m00 = 0, m10 = 0, m01 = 0;
  if (fabs(a00) > 1.1920928955078125e-07) {
    const double s2 = a00 > 0 ? 0.5 : -0.5, s6 = a00 > 0 ? 1.0 / 6 : -1.0 / 6;
    m00 = a00 * s2;
    m10 = a10 * s6;
    m01 = a01 * s6;
  }
  const double area = fabs(area2 * 0.5);
  const int rw = maxx - minx + 1, rh = maxy - miny + 1;
  const double pi = 3.1415926535897932384626433832795;
  const double hw = (double)(rw / 2), hh = (double)(rh / 2);  // the reference's integer rect.width / 2
  const bool keep = area >= a.min_area && area <= a.max_area &&
                    fabs(1 - fmin((double)rw / (double)rh, (double)rh / (double)rw)) <= a.max_whd &&
                    fabs(1 - (area / (pi * (hw * hw)))) <= a.max_circ && fabs(1 - (area / (pi * (hh * hh)))) <= a.max_circ;
  DetRecord o{};
  o.root = root;
  o.keep = keep ? 1 : 0;
  o.area = area;
  if (keep) {
    const float mcx = (float)(m10 / m00) + (float)a.rx;
    const float mcy = (float)(m01 / m00) + (float)a.ry;
    o.dx = mcx;
    o.dy = mcy;
    const double* K = a.K;
    const double* D = a.D;
    const double ifx = 1. / K[0], ify = 1. / K[4];
    double x = ((double)mcx - K[2]) * ifx, y = ((double)mcy - K[5]) * ify;
    const double xs = x, ys = y;
    for (int j = 0; j < 5; ++j) {
      const double r2 = x * x + y * y;
      const double icdist = 1. / (1 + ((D[4] * r2 + D[1]) * r2 + D[0]) * r2);
      const double deltaX = 2 * D[2] * x * y + D[3] * (r2 + 2 * x * x);
      const double deltaY = D[2] * (r2 + 2 * y * y) + 2 * D[3] * x * y;
      x = (xs - deltaX) * icdist;
      y = (ys - deltaY) * icdist;
    }
    const double xx = K[0] * x + K[1] * y + K[2];
    const double yy = K[3] * x + K[4] * y + K[5];
    const double ww = 1. / (K[6] * x + K[7] * y + K[8]);
    o.ux = (double)(float)(xx * ww);
    o.uy = (double)(float)(yy * ww);
  }
  rec[slot] = o;
}

}  // namespace pfmpe

namespace {

// getGaussianKernel(n, sigma, CV_32F) -> 8-bit-fraction ints (the 8U separable path of OpenCV 2.4)
std::vector<int> gaussian_q8(int n, double sigma) {
  std::vector<float> cf(n);
  const double sx = sigma > 0 ? sigma : ((n - 1) * 0.5 - 1) * 0.3 + 0.8;
  const double scale2X = -0.5 / (sx * sx);
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

struct DetBuffers {
  uint8_t* mask;
  uint8_t* nbr;
  int* label;
  int* count;
  int* roots;
  DetRecord* rec;
};

int det_buffers(pfmpe_ctx* c, int64_t npix, DetBuffers& b) {
  auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
  const size_t o_mask = 0, o_nbr = o_mask + al(npix), o_label = o_nbr + al(npix);
  const size_t o_count = o_label + al(npix * 4), o_roots = o_count + 256;
  const size_t o_rec = o_roots + al(kDetMaxComponents * 4), total = o_rec + al(kDetMaxComponents * sizeof(DetRecord));
  if (total > c->det_cap) {
    if (c->d_det) {
      HIPCHK(c, hipStreamSynchronize(c->stream));
      HIPCHK(c, hipFree(c->d_det));
      c->d_det = nullptr;
      c->det_cap = 0;
    }
    HIPCHK(c, hipMalloc((void**)&c->d_det, total));
    c->det_cap = total;
  }
  unsigned char* d = c->d_det;
  b = DetBuffers{d + o_mask, d + o_nbr, (int*)(d + o_label), (int*)(d + o_count), (int*)(d + o_roots),
                 (DetRecord*)(d + o_rec)};
  return PFMPE_OK;
}

}  // namespace

extern "C" {

void pfmpe_default_detect_params(pfmpe_detect_params* p) {
  if (!p) return;
  std::memset(p, 0, sizeof(*p));
  p->threshold_value = 240;  // README.md:331-337 launch values
  p->active_markers = 1;
  p->gaussian_sigma = 0.6;
  p->min_blob_area = 20;
  p->max_blob_area = 160;
  p->max_width_height_distortion = 0.7;
  p->max_circular_distortion = 0.7;
  p->roi_w = -1;  // whole image
  p->roi_h = -1;
}

int pfmpe_stage_image(pfmpe_ctx* c, const uint8_t* image, int width, int height, int pitch) {
  if (!c) return PFMPE_E_ARG;
  if (!image || width < 1 || height < 1 || pitch < width) return fail(c, PFMPE_E_ARG, "stage_image: bad image");
  RET(set_device(c));
  const size_t bytes = (size_t)pitch * height;
  if (bytes > c->img_cap) {
    if (c->d_img) {
      HIPCHK(c, hipStreamSynchronize(c->stream));
      HIPCHK(c, hipFree(c->d_img));
      c->d_img = nullptr;
      c->img_cap = 0;
    }
    HIPCHK(c, hipMalloc((void**)&c->d_img, bytes));
    c->img_cap = bytes;
  }
  HIPCHK(c, hipMemcpyAsync(c->d_img, image, bytes, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  c->img_w = width;
  c->img_h = height;
  c->img_pitch = pitch;
  return PFMPE_OK;
}

int pfmpe_find_leds(pfmpe_ctx* c, const uint8_t* image, int width, int height, int pitch,
                    const pfmpe_detect_params* prm, double* blobs, float* distorted, int max_out,
                    pfmpe_detect_out* out) {
  if (!c) return PFMPE_E_ARG;
  if (!prm || !out || max_out < 0 || (max_out > 0 && !blobs)) return fail(c, PFMPE_E_ARG, "find_leds: bad arguments");
  if (!c->has_model) return fail(c, PFMPE_E_STATE, "find_leds: set_model first (K)");
  if (image) {
    RET(pfmpe_stage_image(c, image, width, height, pitch));
  } else if (!c->d_img || c->img_w != width || c->img_h != height || c->img_pitch != pitch) {
    return fail(c, PFMPE_E_STATE, "find_leds: no staged image of this size (pfmpe_stage_image)");
  }
  const int rx = prm->roi_w < 0 ? 0 : prm->roi_x, ry = prm->roi_h < 0 ? 0 : prm->roi_y;
  const int W = prm->roi_w < 0 ? width : prm->roi_w, H = prm->roi_h < 0 ? height : prm->roi_h;
  if (rx < 0 || ry < 0 || W < 1 || H < 1 || rx + W > width || ry + H > height)
    return fail(c, PFMPE_E_ARG, "find_leds: ROI outside the image");
  if (!(prm->gaussian_sigma > 0) || prm->gaussian_sigma > 5.0)
    return fail(c, PFMPE_E_ARG, "find_leds: gaussian_sigma must be in (0, 5]");
  RET(set_device(c));
  DetArgs a{};
  const int n = (int)std::nearbyint(prm->gaussian_sigma * 3 * 2 + 1) | 1;  // ksize from sigma for 8U (cvRound)
  const std::vector<int> k = gaussian_q8(n, prm->gaussian_sigma);
  for (int i = 0; i < n; ++i) a.k[i] = k[i];
  a.radius = n / 2;
  a.thr = prm->threshold_value;
  a.active = prm->active_markers ? 1 : 0;
  a.img_w = width;
  a.img_h = height;
  a.pitch = pitch;
  a.rx = rx;
  a.ry = ry;
  a.W = W;
  a.H = H;
  std::memcpy(a.K, c->K, sizeof(a.K));
  std::memcpy(a.D, prm->D, sizeof(a.D));
  a.min_area = prm->min_blob_area;
  a.max_area = prm->max_blob_area;
  a.max_whd = prm->max_width_height_distortion;
  a.max_circ = prm->max_circular_distortion;
  const int64_t npix = (int64_t)W * H;
  DetBuffers b;
  RET(det_buffers(c, npix, b));
  HIPCHK(c, hipMemsetAsync(b.count, 0, sizeof(int), c->stream));
  const unsigned g1 = (unsigned)((npix + 255) / 256);
  c->timing_now = c->timing > 0;
  RET(launch(c, PFMPE_K_DETECT, [&] {
    hipLaunchKernelGGL(k_det_mask, dim3((W + kDetTile - 1) / kDetTile, (H + kDetTile - 1) / kDetTile),
                       dim3(kDetTile * kDetTile), 0, c->stream, a, c->d_img, b.mask);
    hipLaunchKernelGGL(k_det_label, dim3(g1), dim3(256), 0, c->stream, a, b.mask, b.nbr, b.label);
    hipLaunchKernelGGL(k_det_merge, dim3(g1), dim3(256), 0, c->stream, a, b.nbr, b.label);
    hipLaunchKernelGGL(k_det_roots, dim3(g1), dim3(256), 0, c->stream, a, b.mask, b.label, b.count, b.roots);
    hipLaunchKernelGGL(k_det_trace, dim3(kDetMaxComponents / 64), dim3(64), 0, c->stream, a, b.nbr, b.count, b.roots,
                       b.rec);
  }));
  int nc = 0;
  HIPCHK(c, hipMemcpyAsync(&nc, b.count, sizeof(int), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  const int ncs = std::min(nc, kDetMaxComponents);
  std::vector<DetRecord> rec(ncs);
  if (ncs > 0) {
    HIPCHK(c, hipMemcpyAsync(rec.data(), b.rec, ncs * sizeof(DetRecord), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
  }
  if (c->timing_now) RET(harvest_timing(c));
  c->timing_now = false;
  // findContours order: reverse discovery = descending raster index of the start pixel
  std::sort(rec.begin(), rec.end(), [](const DetRecord& x, const DetRecord& y) { return x.root > y.root; });
  int m = 0;
  for (const DetRecord& r : rec) {
    if (!r.keep) continue;
    if (m < max_out) {
      blobs[2 * m] = r.ux;
      blobs[2 * m + 1] = r.uy;
      if (distorted) {
        distorted[2 * m] = r.dx;
        distorted[2 * m + 1] = r.dy;
      }
    }
    ++m;
  }
  out->n = m;
  out->n_components = nc;
  out->overflow = nc > kDetMaxComponents ? 1 : 0;
  return PFMPE_OK;
}

}  // extern "C"
