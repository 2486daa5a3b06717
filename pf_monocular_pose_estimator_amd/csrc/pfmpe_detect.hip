// pfmpe_detect.hip — the LED detector on the device: LEDDetector::findLeds
// (pf_mpe_lib/src/led_detector.cpp:46-215, "LD") for one ROI of an 8-bit image, behind pfmpe_find_leds.
//
// The reference is OpenCV 2.4 calls; each is restated (oracle/detect_oracle.cpp lists the semantics):
//   k_det_mask     threshold (TOZERO / BINARY_INV) + GaussianBlur (8-bit-fraction integer kernels,
//                  reflect-101 borders, (sum + 2^15) >> 16) -> "pixel is nonzero" mask, with the 1-pixel
//                  frame cvStartFindContours zeroes.  16x16 tiles: thresholded tile + halo, then the row
//                  pass, staged in LDS; exact integer arithmetic.
//   k_det_label    per 32x32 tile in LDS: each pixel's 8-neighbour bit mask (bit s = direction s of
//                  icvFetchContour's table) and a tile-local union-find (W, NW, N, NE; atomicMin links to the
//                  lower index); the label is the local root's image index
//   k_det_merge    the global union-find over the links that cross tile borders only (agent-scope loads
//                  in find: other blocks' links bypass the non-coherent L1)
//   k_det_roots    flatten; every root (= the component's raster-first pixel, where the reference's raster
//                  scan starts its outer border) takes a slot
//   k_det_trace    one wave per component (grid-stride over the slots): a 64x64 window of neighbour masks
//                  staged in LDS, then lane 0 runs icvFetchContour's border following over it,
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

// Labelling, tile-local first: a 32 x 32 tile (+1 halo) of the mask in LDS gives each pixel its 8-neighbour
// bit mask (bit s = direction s of icvFetchContour's table: 0 +x, 1 (+x,-y), 2 -y, 3 (-x,-y), 4 -x,
// 5 (-x,+y), 6 +y, 7 (+x,+y)) and an LDS union-find over the tile's own W / NW / N / NE links (atomicMin
// to the lower index: the local root is the component's raster-first pixel in the tile).  The global
// label is that root's image index; k_det_merge then unites only links that cross a tile border.
constexpr int kLT = 32;
__device__ __forceinline__ int lfind(const int* L, int i) {
  for (int p = L[i]; p != i; p = L[i]) i = p;
  return i;
}
constexpr int kLabelBlock = 1024;
__global__ __launch_bounds__(kLabelBlock) void k_det_label(const DetArgs a, const uint8_t* __restrict__ mask,
                                                   uint8_t* __restrict__ nbr, int* __restrict__ label) {
  __shared__ uint8_t m[kLT + 2][kLT + 2];
  __shared__ int L[kLT * kLT];
  const int x0 = blockIdx.x * kLT, y0 = blockIdx.y * kLT;
  {  // branch-free: clamped in-bounds addresses, all loads in flight, then the selects
    constexpr int kN = ((kLT + 2) * (kLT + 2) + kLabelBlock - 1) / kLabelBlock;
    uint32_t v[kN];
    bool in[kN];
#pragma unroll
    for (int q = 0; q < kN; ++q) {
      const int i = threadIdx.x + kLabelBlock * q;
      const int ty = i / (kLT + 2), tx = i - ty * (kLT + 2);
      const int gx = x0 + tx - 1, gy = y0 + ty - 1;
      in[q] = i < (kLT + 2) * (kLT + 2) && gx >= 0 && gy >= 0 && gx < a.W && gy < a.H;
      v[q] = mask[(int64_t)min(max(gy, 0), a.H - 1) * a.W + min(max(gx, 0), a.W - 1)];
    }
#pragma unroll
    for (int q = 0; q < kN; ++q) {
      const int i = threadIdx.x + kLabelBlock * q;
      if (i < (kLT + 2) * (kLT + 2)) m[i / (kLT + 2)][i % (kLT + 2)] = in[q] ? (uint8_t)v[q] : (uint8_t)0;
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < kLT * kLT; i += blockDim.x) {
    const int ly = i / kLT, lx = i - ly * kLT;
    L[i] = m[ly + 1][lx + 1] ? i : -1;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < kLT * kLT; i += blockDim.x) {
    const int ly = i / kLT, lx = i - ly * kLT;
    if (!m[ly + 1][lx + 1]) continue;
    const int nb[4][2] = {{-1, 0}, {-1, -1}, {0, -1}, {1, -1}};  // W, NW, N, NE
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int nx = lx + nb[q][0], ny = ly + nb[q][1];
      if (nx < 0 || ny < 0 || nx >= kLT || !m[ny + 1][nx + 1]) continue;
      int u = i, v = ny * kLT + nx;
      for (;;) {  // LDS union-find: link the higher root to the lower index
        u = lfind(L, u);
        v = lfind(L, v);
        if (u == v) break;
        if (u < v) {
          const int t = u;
          u = v;
          v = t;
        }
        const int old = atomicMin(&L[u], v);
        if (old == u) break;
        u = old;
      }
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < kLT * kLT; i += blockDim.x) {
    const int ly = i / kLT, lx = i - ly * kLT;
    const int gx = x0 + lx, gy = y0 + ly;
    if (gx >= a.W || gy >= a.H) continue;
    const int64_t g = (int64_t)gy * a.W + gx;
    if (!m[ly + 1][lx + 1]) {
      label[g] = -1;
      nbr[g] = 0;
      continue;
    }
    uint32_t bits = 0;
#pragma unroll
    for (int s = 0; s < 8; ++s) bits |= m[ly + 1 + dir_dy(s)][lx + 1 + dir_dx(s)] ? 1u << s : 0u;
    nbr[g] = (uint8_t)bits;
    const int r = lfind(L, i);
    label[g] = (y0 + r / kLT) * a.W + (x0 + r % kLT);
  }
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

// the links that cross a tile border (the left column's W / NW, the top row's NW / N / NE)
__global__ void k_det_merge(const DetArgs a, const uint8_t* __restrict__ nbr, int* __restrict__ label) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)a.W * a.H) return;
  const int W = a.W;
  const int y = (int)(i / W), x = (int)(i - (int64_t)y * W);
  const bool left = (x % kLT) == 0, top = (y % kLT) == 0, right = (x % kLT) == kLT - 1;
  if (!left && !top && !right) return;
  const uint32_t b = nbr[i];
  if (!b) return;
  if (left && (b & (1u << 4))) unite(label, (int)i, (int)i - 1);
  if ((left || top) && (b & (1u << 3))) unite(label, (int)i, (int)i - W - 1);
  if (top && (b & (1u << 2))) unite(label, (int)i, (int)i - W);
  if ((top || right) && (b & (1u << 1))) unite(label, (int)i, (int)i - W + 1);
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

// One block (one wave) per component slot: the wave stages a 64 x 64 window of neighbour masks (rows
// y0 .. y0+63 from the root down, columns x0-31 .. x0+32) in LDS, then lane 0 follows the border there
// (a point outside the window falls back to the global masks).
constexpr int kWin = 64;
__global__ __launch_bounds__(64) void k_det_trace(const DetArgs a, const uint8_t* __restrict__ nbr,
                                                  const int* __restrict__ count, const int* __restrict__ roots,
                                                  DetRecord* __restrict__ rec) {
  __shared__ uint8_t win[kWin][kWin];
  const int nc = min(*count, kDetMaxComponents);
  for (int slot = blockIdx.x; slot < nc; slot += gridDim.x) {
  __syncthreads();  // the previous slot's window reads are done
  const int root = roots[slot];
  const int W = a.W;
  const int x0 = root % W, y0 = root / W;
  const int wx = x0 - kWin / 2 + 1, wy = y0;
  {  // branch-free: every lane loads from a clamped in-bounds address, 16 loads in flight per batch
    const int lane = threadIdx.x;
    const int gx = wx + lane;
    const bool xin = gx >= 0 && gx < W;
    const int cx = min(max(gx, 0), W - 1);
    for (int r0 = 0; r0 < kWin; r0 += 16) {
      uint32_t v[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) v[q] = nbr[(int64_t)min(wy + r0 + q, a.H - 1) * W + cx];
#pragma unroll
      for (int q = 0; q < 16; ++q) win[r0 + q][lane] = (xin && wy + r0 + q < a.H) ? (uint8_t)v[q] : (uint8_t)0;
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
  auto nb = [&](int x, int y) -> uint32_t {
    const int lx = x - wx, ly = y - wy;
    if ((unsigned)lx < (unsigned)kWin && (unsigned)ly < (unsigned)kWin) return win[ly][lx];
    return nbr[(int64_t)y * W + x];
  };
  // icvFetchContour (CHAIN_APPROX_NONE), the contour points streamed into the polygon sums
  // The reference sums these in double; every term is an integer far below 2^53, so int64 sums are the
  // same numbers (exact either way) with a shorter dependency chain.
  int64_t a00 = 0, a10 = 0, a01 = 0, area2 = 0;
  int minx = x0, maxx = x0, miny = y0, maxy = y0;
  int64_t fx_ = 0, fy_ = 0, px_ = 0, py_ = 0;  // first point, previous point
  int np = 0;
  auto add_point = [&](int x, int y) {
    const int64_t xi = x, yi = y;
    if (np == 0) {
      fx_ = xi;
      fy_ = yi;
    } else {
      const int64_t dxy = px_ * yi - xi * py_;
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
  const uint32_t b0 = nb(x0, y0);
  int s = 4;
  do {
    s = (s - 1) & 7;
  } while (!((b0 >> s) & 1u) && s != 4);
  if (s == 4) {
    add_point(x0, y0);  // single-pixel domain
  } else {
    const int x1 = x0 + dir_dx(s), y1 = y0 + dir_dy(s);
    int x3 = x0, y3 = y0, px = x0, py = y0;
    for (int64_t guard = 0; guard < 4 * (int64_t)a.W * a.H + 8; ++guard) {
      const uint32_t bb = nb(x3, y3);
      const uint32_t rot = ((bb | (bb << 8)) >> ((s + 1) & 7)) & 0xffu;  // directions s+1, s+2, ... (cyclic)
      s = (s + 1 + __builtin_ctz(rot)) & 7;                            // first set (one exists)
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
    const int64_t xi = fx_, yi = fy_;
    const int64_t dxy = px_ * yi - xi * py_;
    a00 += dxy;
    a10 += dxy * (px_ + xi);
    a01 += dxy * (py_ + yi);
    area2 += px_ * yi - py_ * xi;
  }
  double m00 = 0, m10 = 0, m01 = 0;
  if (a00 != 0) {  // |a00| > FLT_EPSILON for an integer
    const double s2 = a00 > 0 ? 0.5 : -0.5, s6 = a00 > 0 ? 1.0 / 6 : -1.0 / 6;
    m00 = (double)a00 * s2;
    m10 = (double)a10 * s6;
    m01 = (double)a01 * s6;
  }
  const double area = fabs((double)area2 * 0.5);
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
  }  // lane 0
  }  // slots
}

// Output in findContours order (reverse discovery = descending root index), written straight into pinned
// host memory: rank of a kept record = number of kept records with a larger root.  One block.
struct DetOutHost {
  int32_t n, n_components, overflow, pad;
  double und[2 * kMaxBlobs];
  float dist[2 * kMaxBlobs];
};
constexpr int kEmitBlock = 1024;
__global__ __launch_bounds__(kEmitBlock) void k_det_emit(const int* __restrict__ count, const DetRecord* __restrict__ rec,
                                                         DetOutHost* __restrict__ out) {
  __shared__ int kroot[kDetMaxComponents];
  __shared__ int nkept;
  const int nc = min(*count, kDetMaxComponents);
  if (threadIdx.x == 0) nkept = 0;
  __syncthreads();
  for (int i = threadIdx.x; i < nc; i += kEmitBlock)
    if (rec[i].keep) kroot[atomicAdd(&nkept, 1)] = i;  // slot ids, any order
  __syncthreads();
  const int nk = nkept;
  for (int t = threadIdx.x; t < nk; t += kEmitBlock) {
    const int i = kroot[t];
    const int r = rec[i].root;
    int rank = 0;
    for (int u = 0; u < nk; ++u) rank += rec[kroot[u]].root > r ? 1 : 0;
    if (rank < kMaxBlobs) {
      out->und[2 * rank] = rec[i].ux;
      out->und[2 * rank + 1] = rec[i].uy;
      out->dist[2 * rank] = rec[i].dx;
      out->dist[2 * rank + 1] = rec[i].dy;
    }
  }
  if (threadIdx.x == 0) {
    out->n = nk;
    out->n_components = *count;
    out->overflow = *count > kDetMaxComponents ? 1 : 0;
  }
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
  if (!c->h_det) {
    HIPCHK(c, hipHostMalloc((void**)&c->h_det, sizeof(DetOutHost), hipHostMallocMapped | hipHostMallocCoherent));
  }
  DetOutHost* hout = (DetOutHost*)c->h_det;
  DetOutHost* dout = nullptr;
  HIPCHK(c, hipHostGetDevicePointer((void**)&dout, hout, 0));
  RET(launch(c, PFMPE_K_DETECT, [&] {
    hipLaunchKernelGGL(k_det_mask, dim3((W + kDetTile - 1) / kDetTile, (H + kDetTile - 1) / kDetTile),
                       dim3(kDetTile * kDetTile), 0, c->stream, a, c->d_img, b.mask);
    hipLaunchKernelGGL(k_det_label, dim3((W + kLT - 1) / kLT, (H + kLT - 1) / kLT), dim3(kLabelBlock), 0, c->stream, a, b.mask,
                       b.nbr, b.label);
    hipLaunchKernelGGL(k_det_merge, dim3(g1), dim3(256), 0, c->stream, a, b.nbr, b.label);
    hipLaunchKernelGGL(k_det_roots, dim3(g1), dim3(256), 0, c->stream, a, b.mask, b.label, b.count, b.roots);
    hipLaunchKernelGGL(k_det_trace, dim3(512), dim3(64), 0, c->stream, a, b.nbr, b.count, b.roots, b.rec);
    hipLaunchKernelGGL(k_det_emit, dim3(1), dim3(kEmitBlock), 0, c->stream, b.count, b.rec, dout);
  }));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  if (c->timing_now) RET(harvest_timing(c));
  c->timing_now = false;
  const int m = hout->n;
  const int nc = hout->n_components;
  const int nw = std::min(std::min(m, max_out), kMaxBlobs);
  if (nw > 0) {
    std::memcpy(blobs, hout->und, 2 * (size_t)nw * sizeof(double));
    if (distorted) std::memcpy(distorted, hout->dist, 2 * (size_t)nw * sizeof(float));
  }
  out->n = m;
  out->n_components = nc;
  out->overflow = hout->overflow;
  return PFMPE_OK;
}

}  // extern "C"
