// pfmpe_engine.hip — host side of the MI355X PF engine: context, buffers, launch sequence, C-ABI.
//
// Replaces the PF block of PoseEstimator::estimateBodyPose (pf_mpe_lib/src/pose_estimator.cpp:475-733)
// behind include/pfmpe.h.  Device layout (DESIGN.md "HBM layout"): particle state as 12 SoA planes
// (r00 r01 r02 t0 r10 r11 r12 t1 r20 r21 r22 t2) of `ld` elements each, double-buffered (prior /
// posterior); two weight slots (current iteration / best iteration so far); per-block partials;
// one control record; one output record copied to pinned host memory at the end of the frame.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstddef>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/pfmpe.h"
#include "pf_kernels.hpp"

using namespace pfmpe;

static_assert(offsetof(OutDev, kept_slot) == sizeof(pfmpe_frame_out), "OutDev must start with pfmpe_frame_out");
static_assert(offsetof(OutDev, corr) == offsetof(pfmpe_frame_out, corr), "OutDev layout");
static_assert(offsetof(OutDev, prob_sum) == offsetof(pfmpe_frame_out, prob_sum), "OutDev layout");
static_assert(PFMPE_MAX_MARKERS == kMaxMarkers, "marker capacity mismatch");
static_assert(PFMPE_MAX_BLOBS == kMaxBlobs, "blob capacity mismatch");

struct EventPair {
  hipEvent_t a, b;
  int kid;
};

struct pfmpe_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  int max_particles = 0, max_markers = 0, max_blobs = 0, state_dtype = PFMPE_STATE_F32;
  size_t es = 4;       // bytes per state element
  int64_t ld = 0;      // plane stride (elements)
  int max_blk = 0;

  void* d_state[2] = {nullptr, nullptr};
  int prior_idx = 0;
  void* d_w[2] = {nullptr, nullptr};
  int max_grp = 0;
  BlockPart* d_part[2] = {nullptr, nullptr};
  BlockScan* d_bscan[2] = {nullptr, nullptr};
  GroupPart* d_gpart[2] = {nullptr, nullptr};
  GroupScan* d_gscan = nullptr;
  CountPart* d_cpart = nullptr;
  CountPart* d_cgroup = nullptr;
  uint32_t* d_counters = nullptr;  // [prop group x max_grp][prop top][res group x max_grp][res top]
  Ctrl* d_ctrl = nullptr;
  OutDev* h_out = nullptr;       // pinned host memory, written by the final wave
  OutDev* d_out = nullptr;       // its device address
  int32_t seq = 0;               // frame-record sequence number (publication tag = 2 * seq + finished)
  unsigned char* d_table = nullptr;  // this frame's blob table (BlobTable<T> layout)
  unsigned char* h_table = nullptr;  // pinned staging
  unsigned char* d_bank = nullptr;   // staged tables of a whole stream, back to back
  std::vector<size_t> bank_off;      // byte offset of frame f's table
  std::vector<int32_t> bank_B;
  double* d_xfer = nullptr;      // N x 12 doubles
  uint32_t* d_counts = nullptr;
  uint64_t* d_stamps = nullptr;  // diagnostic stamps (diag & 4)

  // model / params
  int M = 0;
  double markers[kMaxMarkers * 3] = {0};
  double K[9] = {0};
  uint32_t downgrade = 0;
  bool has_model = false;
  pfmpe_params params{};
  int N = 0;
  bool has_prior = false;

  // options
  bool record_counts = false;
  bool prune = true;
  int timing = 0;          // HIP-event sampling period in frames (0 = off)
  bool timing_now = false;  // this frame's launches are bracketed
  int64_t timing_frame = 0;
  int diag = 0;

  // last step (for get_particles / get_weights)
  FrameArgsT<float> last_fa_f{};
  FrameArgsT<double> last_fa_d{};
  bool has_last = false;
  int last_prior_idx = 0;
  bool last_accepted = false;
  int last_kept_slot = 0, last_kept_iter = 0;

  // timing
  std::vector<EventPair> ev_pool;
  size_t ev_used = 0;
  int64_t k_launches[PFMPE_K_COUNT] = {0};
  double k_ms[PFMPE_K_COUNT] = {0};

  std::string err;
};

namespace {

int fail(pfmpe_ctx* c, int code, const std::string& msg) {
  if (c) c->err = msg;
  return code;
}

#define HIPCHK(ctx, expr)                                                                       \
  do {                                                                                          \
    hipError_t e_ = (expr);                                                                     \
    if (e_ != hipSuccess)                                                                       \
      return fail((ctx), PFMPE_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));       \
  } while (0)

int set_device(pfmpe_ctx* c) {
  HIPCHK(c, hipSetDevice(c->device));
  return PFMPE_OK;
}

// ---------------------------------------------------------------------- timed launch wrapper
template <typename Launch>
int launch(pfmpe_ctx* c, int kid, Launch&& fn) {
  EventPair* ep = nullptr;
  if (c->timing_now) {
    if (c->ev_used == c->ev_pool.size()) {
      EventPair p{};
      p.kid = kid;
      HIPCHK(c, hipEventCreate(&p.a));
      HIPCHK(c, hipEventCreate(&p.b));
      c->ev_pool.push_back(p);
    }
    ep = &c->ev_pool[c->ev_used++];
    ep->kid = kid;
    HIPCHK(c, hipEventRecord(ep->a, c->stream));
  }
  fn();
  HIPCHK(c, hipGetLastError());
  if (ep) HIPCHK(c, hipEventRecord(ep->b, c->stream));
  return PFMPE_OK;
}

int harvest_timing(pfmpe_ctx* c) {
  for (size_t i = 0; i < c->ev_used; ++i) {
    float ms = 0.f;
    HIPCHK(c, hipEventElapsedTime(&ms, c->ev_pool[i].a, c->ev_pool[i].b));
    c->k_launches[c->ev_pool[i].kid] += 1;
    c->k_ms[c->ev_pool[i].kid] += ms;
  }
  c->ev_used = 0;
  return PFMPE_OK;
}

// Wait for the frame record: the final block writes it into pinned host memory (then a system-scope
// fence and the `done` word), so the host spins on that word instead of paying a stream synchronize.
// The spin is bounded by hipStreamQuery: an idle stream without a record is an error.
int wait_frame(pfmpe_ctx* c) {
  volatile int32_t* tag = &c->h_out->tag;
  const int32_t want = c->seq;
  for (uint64_t spin = 0;; ++spin) {
    const int32_t t = *tag;
    if ((t >> 1) == want) {
      __atomic_thread_fence(__ATOMIC_ACQUIRE);  // record loads may not move above the tag load
      return PFMPE_OK;
    }
    if ((spin & 1023u) == 1023u) {
      const hipError_t q = hipStreamQuery(c->stream);
      if (q == hipSuccess) {
        if ((*tag >> 1) == want) {
          __atomic_thread_fence(__ATOMIC_ACQUIRE);
          return PFMPE_OK;
        }
        return fail(c, PFMPE_E_HIP, "frame record was not written");
      }
      if (q != hipErrorNotReady) return fail(c, PFMPE_E_HIP, std::string("stream error: ") + hipGetErrorString(q));
    }
    __builtin_ia32_pause();
  }
}

bool frame_done(const pfmpe_ctx* c) { return (c->h_out->tag & 1) != 0; }

#define RET(expr)              \
  do {                         \
    int r_ = (expr);           \
    if (r_ != PFMPE_OK) return r_; \
  } while (0)

// ---------------------------------------------------------------------- typed launch sequence
template <typename T> FrameArgsT<T>& last_args(pfmpe_ctx* c);
template <> FrameArgsT<float>& last_args<float>(pfmpe_ctx* c) { return c->last_fa_f; }
template <> FrameArgsT<double>& last_args<double>(pfmpe_ctx* c) { return c->last_fa_d; }

template <typename T, int RNG, int MAXM>
struct Seq {
  static int iterate(pfmpe_ctx* c, const FrameArgsT<T>& fa, const unsigned char* table, int iter) {
    const T* prior = (const T*)c->d_state[c->prior_idx];
    const size_t lds = BlobTable<T>::bytes(fa.B);
    uint32_t* gcount = c->d_counters;
    uint32_t* tcount = c->d_counters + c->max_grp;
    return launch(c, PFMPE_K_PROPAGATE, [&] {
      if (c->prune)
        hipLaunchKernelGGL((k_propagate_weigh<T, RNG, MAXM, true>), dim3(fa.nblk), dim3(kBlock), lds, c->stream, fa,
                           table, prior, (T*)c->d_w[0], (T*)c->d_w[1], c->d_part[0], c->d_part[1], c->d_bscan[0],
                           c->d_bscan[1], c->d_gpart[0], c->d_gpart[1], c->d_gscan, c->d_ctrl, gcount, tcount, iter,
                           c->d_stamps);
      else
        hipLaunchKernelGGL((k_propagate_weigh<T, RNG, MAXM, false>), dim3(fa.nblk), dim3(kBlock), lds, c->stream, fa,
                           table, prior, (T*)c->d_w[0], (T*)c->d_w[1], c->d_part[0], c->d_part[1], c->d_bscan[0],
                           c->d_bscan[1], c->d_gpart[0], c->d_gpart[1], c->d_gscan, c->d_ctrl, gcount, tcount, iter,
                           c->d_stamps);
    });
  }
  static int finish(pfmpe_ctx* c, const FrameArgsT<T>& fa, const unsigned char* table) {
    const T* prior = (const T*)c->d_state[c->prior_idx];
    T* post = (T*)c->d_state[1 - c->prior_idx];
    uint32_t* gcount = c->d_counters + c->max_grp + 1;
    uint32_t* tcount = c->d_counters + 2 * c->max_grp + 1;
    c->seq = (c->seq + 1) & 0x3fffffff;
    const int32_t seq = c->seq;
    RET(launch(c, PFMPE_K_RESAMPLE, [&] {
      hipLaunchKernelGGL((k_resample<T, RNG, MAXM>), dim3(fa.nblk), dim3(kBlock), 0, c->stream, fa, c->d_ctrl, table,
                         prior, post, (const T*)c->d_w[0], (const T*)c->d_w[1], c->d_bscan[0], c->d_bscan[1],
                         c->d_gscan, c->d_cpart, c->d_cgroup, gcount, tcount,
                         c->record_counts ? c->d_counts : nullptr, c->d_out, seq, c->d_stamps);
    }));
    RET(wait_frame(c));
    if (c->timing_now) HIPCHK(c, hipStreamSynchronize(c->stream));  // end events must have completed
    return PFMPE_OK;
  }
  static int step(pfmpe_ctx* c, const FrameArgsT<T>& fa, const unsigned char* table) {
    const int iter_cap = fa.force_iters > 0 ? fa.force_iters : std::max(1, fa.max_iter);
    int iter = 0;
    RET(iterate(c, fa, table, iter++));
    RET(finish(c, fa, table));
    // Rare path: the exit rule did not fire on iteration 0.  Later iterations are queued in growing
    // batches; launches past the exit are no-ops (they read ctrl->done).
    int batch = 1;
    while (!frame_done(c)) {
      if (iter >= iter_cap) return fail(c, PFMPE_E_STATE, "PF iteration loop did not terminate");
      for (int b = 0; b < batch && iter < iter_cap; ++b) RET(iterate(c, fa, table, iter++));
      RET(finish(c, fa, table));
      batch = std::min(batch * 2, 16);
    }
    last_args<T>(c) = fa;
    return PFMPE_OK;
  }
  static int regen(pfmpe_ctx* c, int kept_iter, const void* prior, double* out) {
    const FrameArgsT<T>& fa = last_args<T>(c);
    return launch(c, PFMPE_K_AUX, [&] {
      hipLaunchKernelGGL((k_regen<T, RNG>), dim3((fa.N + 255) / 256), dim3(256), 0, c->stream, fa, kept_iter,
                         (const T*)prior, out);
    });
  }
};

template <typename T>
FrameArgsT<T> build_args(const pfmpe_ctx* c, const pfmpe_frame_in* in);

template <typename T, int RNG>
int dispatch_m(pfmpe_ctx* c, const pfmpe_frame_in* in, const unsigned char* table) {
  const FrameArgsT<T> fa = build_args<T>(c, in);
  // marker capacity buckets: the per-particle loops are unrolled to MAXM (5: the 5-LED configs C1/C2/C4)
  if (fa.M <= 5) return Seq<T, RNG, 5>::step(c, fa, table);
  if (fa.M <= 8) return Seq<T, RNG, 8>::step(c, fa, table);
  return Seq<T, RNG, 16>::step(c, fa, table);
}

int dispatch_step(pfmpe_ctx* c, const pfmpe_frame_in* in, const unsigned char* table) {
  const bool f64 = c->state_dtype == PFMPE_STATE_F64;
  const bool ref = c->params.rng_mode == PFMPE_RNG_REFERENCE;
  if (f64) return ref ? dispatch_m<double, kRngReference>(c, in, table) : dispatch_m<double, kRngPhilox>(c, in, table);
  return ref ? dispatch_m<float, kRngReference>(c, in, table) : dispatch_m<float, kRngPhilox>(c, in, table);
}

int dispatch_regen(pfmpe_ctx* c, int kept_iter, const void* prior, double* out) {
  const bool f64 = c->state_dtype == PFMPE_STATE_F64;
  const bool ref = c->params.rng_mode == PFMPE_RNG_REFERENCE;
  if (f64) return ref ? Seq<double, kRngReference, 8>::regen(c, kept_iter, prior, out)
                      : Seq<double, kRngPhilox, 8>::regen(c, kept_iter, prior, out);
  return ref ? Seq<float, kRngReference, 8>::regen(c, kept_iter, prior, out)
             : Seq<float, kRngPhilox, 8>::regen(c, kept_iter, prior, out);
}


bool is_identity12(const double* p) {
  static const double I[12] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0};
  for (int q = 0; q < 12; ++q)
    if (p[q] != I[q]) return false;
  return true;
}

// Kernel arguments from the host state + frame inputs (PE:488-531), pre-converted to T
template <typename T>
FrameArgsT<T> build_args(const pfmpe_ctx* c, const pfmpe_frame_in* in) {
  FrameArgsT<T> fa{};
  for (int q = 0; q < 12; ++q) {
    fa.cur[q] = (T)in->current_pose[q];
    fa.pred[q] = (T)in->predicted_pose[q];
    fa.predm[q] = (T)in->prediction[q];
    fa.cam[q] = (T)in->cam_move_inv[q];
  }
  for (int q = 0; q < kMaxMarkers * 3; ++q) fa.markers[q] = (T)c->markers[q];
  for (int q = 0; q < 9; ++q) fa.K[q] = (T)c->K[q];
  const pfmpe_params& p = c->params;
  double facT, facR;
  if (in->it_since_init == 1) {  // PE:488-496
    facT = 1;
    facR = 1;
  } else {                       // PE:499-505 (all three use predictionMatrix(0,3))
    facT = std::min(std::max(0.2, std::abs(in->prediction[3]) / in->dt), 1.0) / 4;
    facR = 0.2;
  }
  for (int q = 0; q < 3; ++q) {
    fa.dlo[q] = p.ang_min * facR;
    fa.dhi[q] = p.ang_max * facR;
    fa.dlo[3 + q] = p.trans_min * facT;
    fa.dhi[3 + q] = p.trans_max * facT;
  }
  for (int q = 0; q < 6; ++q) {
    fa.lo[q] = (T)fa.dlo[q];
    fa.hi[q] = (T)fa.dhi[q];
  }
  fa.growth = p.growth;
  fa.tol = (T)p.tol;
  fa.tol_pf = (T)p.tol_pf;
  // every blob with sqrt(d2) <= tol_pf (in T arithmetic) has |dx| <= tolq
  fa.tolq = (T)(p.tol_pf * (1.0 + 1e-3) + 1e-3);
  const int B = in->B;
  fa.exit_thr = (double)((size_t)c->M * (size_t)std::min(p.exit_cap, B));
  fa.accept_thr = (double)((size_t)c->M * (size_t)std::min(p.accept_cap, B));
  fa.key0 = (uint32_t)in->seed;
  fa.key1 = (uint32_t)(in->seed >> 32);
  fa.flo = (uint32_t)in->frame_idx;
  fa.fhi = (uint32_t)(in->frame_idx >> 32);
  fa.lcg_x0 = lcg_seed((uint32_t)in->seed);
  fa.downgrade = c->downgrade;
  fa.N = c->N;
  fa.M = c->M;
  fa.B = B;
  fa.it = in->it_since_init;
  fa.cam_identity = is_identity12(in->cam_move_inv) ? 1 : 0;
  fa.max_iter = p.max_iter;
  fa.force_iters = in->force_iters;
  fa.nblk = (c->N + kBlock - 1) / kBlock;
  fa.ngrp = (fa.nblk + kGroup - 1) / kGroup;
  fa.diag = c->diag;
  fa.ld = c->ld;
  return fa;
}

size_t table_bytes(const pfmpe_ctx* c, int B) {
  return c->state_dtype == PFMPE_STATE_F64 ? BlobTable<double>::bytes(B) : BlobTable<float>::bytes(B);
}
void build_table(const pfmpe_ctx* c, const double* blobs, int B, unsigned char* dst) {
  if (c->state_dtype == PFMPE_STATE_F64)
    build_blob_table_host<double>(blobs, B, dst);
  else
    build_blob_table_host<float>(blobs, B, dst);
}

size_t counters_bytes(const pfmpe_ctx* c) { return (size_t)(2 * c->max_grp + 2) * sizeof(uint32_t); }

void free_all(pfmpe_ctx* c) {
  void* dev[] = {c->d_state[0], c->d_state[1], c->d_w[0], c->d_w[1], c->d_part[0], c->d_part[1],
                 c->d_bscan[0], c->d_bscan[1], c->d_gpart[0], c->d_gpart[1], c->d_gscan, c->d_cpart,
                 c->d_cgroup, c->d_counters, c->d_ctrl, c->d_table, c->d_bank, c->d_xfer, c->d_counts,
                 c->d_stamps};
  for (void* p : dev)
    if (p) (void)hipFree(p);
  if (c->h_out) (void)hipHostFree(c->h_out);
  if (c->h_table) (void)hipHostFree(c->h_table);
  for (auto& e : c->ev_pool) {
    (void)hipEventDestroy(e.a);
    (void)hipEventDestroy(e.b);
  }
  if (c->stream) (void)hipStreamDestroy(c->stream);
}

}  // namespace

// ======================================================================================= C-ABI
extern "C" {

int pfmpe_abi_version(void) { return PFMPE_ABI_VERSION; }

void pfmpe_default_params(pfmpe_params* p) {
  if (!p) return;
  // README.md:338-361 launch defaults; constants of PE:563, 616, 633
  p->tol = 5.0;
  p->tol_pf = 4.0;
  p->ang_min = -0.015;
  p->ang_max = 0.015;
  p->trans_min = -0.035;
  p->trans_max = 0.035;
  p->growth = 0.025;
  p->max_iter = 80;
  p->exit_cap = 5;
  p->accept_cap = 3;
  p->rng_mode = PFMPE_RNG_PHILOX;
}

int pfmpe_create(pfmpe_ctx** out, int hip_device, int max_particles, int max_markers, int max_blobs,
                 int state_dtype) {
  if (!out) return PFMPE_E_ARG;
  *out = nullptr;
  if (max_particles < 1 || max_markers < 1 || max_markers > kMaxMarkers || max_blobs < 0 ||
      max_blobs > kMaxBlobs || (state_dtype != PFMPE_STATE_F32 && state_dtype != PFMPE_STATE_F64))
    return PFMPE_E_ARG;
  pfmpe_ctx* c = new pfmpe_ctx();
  c->device = hip_device;
  c->max_particles = max_particles;
  c->max_markers = max_markers;
  c->max_blobs = max_blobs;
  c->state_dtype = state_dtype;
  c->es = state_dtype == PFMPE_STATE_F64 ? 8 : 4;
  c->ld = ((int64_t)max_particles + 63) / 64 * 64;
  c->max_blk = (max_particles + kBlock - 1) / kBlock;
  pfmpe_default_params(&c->params);
  auto bad = [&](int code) {
    free_all(c);
    delete c;
    return code;
  };
  if (hipSetDevice(hip_device) != hipSuccess) return bad(PFMPE_E_HIP);
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) return bad(PFMPE_E_HIP);
  const size_t state_bytes = (size_t)kPlanes * c->ld * c->es;
  bool ok = true;
  c->max_grp = (c->max_blk + kGroup - 1) / kGroup;
  for (int i = 0; i < 2; ++i) {
    ok &= hipMalloc(&c->d_state[i], state_bytes) == hipSuccess;
    ok &= hipMalloc(&c->d_w[i], (size_t)c->ld * c->es) == hipSuccess;
    ok &= hipMalloc((void**)&c->d_part[i], (size_t)c->max_blk * sizeof(BlockPart)) == hipSuccess;
    ok &= hipMalloc((void**)&c->d_bscan[i], (size_t)c->max_blk * sizeof(BlockScan)) == hipSuccess;
    ok &= hipMalloc((void**)&c->d_gpart[i], (size_t)c->max_grp * sizeof(GroupPart)) == hipSuccess;
  }
  ok &= hipMalloc((void**)&c->d_gscan, (size_t)c->max_grp * sizeof(GroupScan)) == hipSuccess;
  ok &= hipMalloc((void**)&c->d_cpart, (size_t)c->max_blk * sizeof(CountPart)) == hipSuccess;
  ok &= hipMalloc((void**)&c->d_cgroup, (size_t)c->max_grp * sizeof(CountPart)) == hipSuccess;
  ok &= hipMalloc((void**)&c->d_counters, counters_bytes(c)) == hipSuccess;
  ok &= hipMalloc((void**)&c->d_ctrl, sizeof(Ctrl)) == hipSuccess;
  ok &= hipHostMalloc((void**)&c->h_out, sizeof(OutDev), hipHostMallocMapped | hipHostMallocCoherent) == hipSuccess;
  ok = ok && hipHostGetDevicePointer((void**)&c->d_out, c->h_out, 0) == hipSuccess;
  ok &= hipMalloc((void**)&c->d_table, table_bytes(c, kMaxBlobs)) == hipSuccess;
  ok &= hipHostMalloc((void**)&c->h_table, table_bytes(c, kMaxBlobs), hipHostMallocDefault) == hipSuccess;
  if (!ok) return bad(PFMPE_E_HIP);
  if (hipMemset(c->d_ctrl, 0, sizeof(Ctrl)) != hipSuccess) return bad(PFMPE_E_HIP);
  if (hipMemset(c->d_counters, 0, counters_bytes(c)) != hipSuccess) return bad(PFMPE_E_HIP);
  if (hipMemset(c->d_state[0], 0, state_bytes) != hipSuccess) return bad(PFMPE_E_HIP);
  if (hipMemset(c->d_state[1], 0, state_bytes) != hipSuccess) return bad(PFMPE_E_HIP);
  *out = c;
  return PFMPE_OK;
}

void pfmpe_destroy(pfmpe_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  free_all(c);
  delete c;
}

const char* pfmpe_last_error(const pfmpe_ctx* c) { return c ? c->err.c_str() : "null context"; }

int pfmpe_set_model(pfmpe_ctx* c, const double* markers_xyz, int M, const double* K, const uint8_t* downgrade) {
  if (!c) return PFMPE_E_ARG;
  if (!markers_xyz || !K || M < 1) return fail(c, PFMPE_E_ARG, "set_model: null markers/K or M < 1");
  if (M > c->max_markers) return fail(c, PFMPE_E_CAP, "set_model: M exceeds max_markers");
  c->M = M;
  std::memset(c->markers, 0, sizeof(c->markers));
  std::memcpy(c->markers, markers_xyz, sizeof(double) * 3 * M);
  std::memcpy(c->K, K, sizeof(c->K));
  c->downgrade = 0;
  if (downgrade)
    for (int j = 0; j < M; ++j)
      if (downgrade[j]) c->downgrade |= 1u << j;
  c->has_model = true;
  return PFMPE_OK;
}

int pfmpe_set_params(pfmpe_ctx* c, const pfmpe_params* p) {
  if (!c || !p) return PFMPE_E_ARG;
  if (!(p->tol > 0) || !(p->tol_pf >= 0) || p->max_iter < 1 || p->exit_cap < 0 || p->accept_cap < 0 ||
      (p->rng_mode != PFMPE_RNG_REFERENCE && p->rng_mode != PFMPE_RNG_PHILOX))
    return fail(c, PFMPE_E_ARG, "set_params: invalid parameter");
  c->params = *p;
  return PFMPE_OK;
}

int pfmpe_set_option(pfmpe_ctx* c, int option, int64_t value) {
  if (!c) return PFMPE_E_ARG;
  switch (option) {
    case PFMPE_OPT_RECORD_COUNTS:
      c->record_counts = value != 0;
      if (c->record_counts && !c->d_counts) {
        RET(set_device(c));
        HIPCHK(c, hipMalloc((void**)&c->d_counts, (size_t)c->ld * sizeof(uint32_t)));
      }
      return PFMPE_OK;
    case PFMPE_OPT_PRUNE:
      c->prune = value != 0;
      return PFMPE_OK;
    case PFMPE_OPT_TIMING:
      if (value < 0 || value > (1 << 20)) return fail(c, PFMPE_E_ARG, "set_option: timing period out of range");
      c->timing = (int)value;
      c->timing_frame = 0;
      return PFMPE_OK;
    case 99:  // undocumented: diagnostic kernel switches for timing experiments
      c->diag = (int)value;
      if ((c->diag & 4) && !c->d_stamps) {
        RET(set_device(c));
        HIPCHK(c, hipMalloc((void**)&c->d_stamps, kStamps * sizeof(uint64_t)));
      }
      return PFMPE_OK;
    default:
      return fail(c, PFMPE_E_ARG, "set_option: unknown option");
  }
}

static int ensure_xfer(pfmpe_ctx* c) {
  if (!c->d_xfer) HIPCHK(c, hipMalloc((void**)&c->d_xfer, (size_t)c->max_particles * 12 * sizeof(double)));
  return PFMPE_OK;
}

int pfmpe_set_prior(pfmpe_ctx* c, const double* poses, int N) {
  if (!c) return PFMPE_E_ARG;
  if (!poses || N < 1) return fail(c, PFMPE_E_ARG, "set_prior: null poses or N < 1");
  if (N > c->max_particles) return fail(c, PFMPE_E_CAP, "set_prior: N exceeds max_particles");
  RET(set_device(c));
  RET(ensure_xfer(c));
  HIPCHK(c, hipMemcpyAsync(c->d_xfer, poses, (size_t)N * 12 * sizeof(double), hipMemcpyHostToDevice, c->stream));
  if (c->state_dtype == PFMPE_STATE_F64)
    hipLaunchKernelGGL((k_import<double>), dim3((N + 255) / 256), dim3(256), 0, c->stream, c->d_xfer,
                       (double*)c->d_state[c->prior_idx], N, c->ld);
  else
    hipLaunchKernelGGL((k_import<float>), dim3((N + 255) / 256), dim3(256), 0, c->stream, c->d_xfer,
                       (float*)c->d_state[c->prior_idx], N, c->ld);
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipMemsetAsync(c->d_ctrl, 0, sizeof(Ctrl), c->stream));
  HIPCHK(c, hipMemsetAsync(c->d_counters, 0, counters_bytes(c), c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  c->N = N;
  c->has_prior = true;
  c->has_last = false;
  return PFMPE_OK;
}

int pfmpe_stage_blob_bank(pfmpe_ctx* c, const double* blobs, const int32_t* offsets, int nframes) {
  if (!c) return PFMPE_E_ARG;
  if (!blobs || !offsets || nframes < 1) return fail(c, PFMPE_E_ARG, "stage_blob_bank: bad arguments");
  for (int f = 0; f < nframes; ++f) {
    const int B = offsets[f + 1] - offsets[f];
    if (B < 0 || offsets[f] < 0) return fail(c, PFMPE_E_ARG, "stage_blob_bank: offsets not monotone");
    if (B > c->max_blobs) return fail(c, PFMPE_E_CAP, "stage_blob_bank: frame exceeds max_blobs");
  }
  RET(set_device(c));
  if (c->d_bank) {
    HIPCHK(c, hipStreamSynchronize(c->stream));
    HIPCHK(c, hipFree(c->d_bank));
    c->d_bank = nullptr;
  }
  c->bank_off.assign(nframes + 1, 0);
  c->bank_B.assign(nframes, 0);
  for (int f = 0; f < nframes; ++f) {
    c->bank_B[f] = offsets[f + 1] - offsets[f];
    c->bank_off[f + 1] = c->bank_off[f] + table_bytes(c, c->bank_B[f]);
  }
  std::vector<unsigned char> host(c->bank_off[nframes]);
  for (int f = 0; f < nframes; ++f)
    build_table(c, blobs + 2 * (size_t)offsets[f], c->bank_B[f], host.data() + c->bank_off[f]);
  HIPCHK(c, hipMalloc((void**)&c->d_bank, host.size()));
  HIPCHK(c, hipMemcpy(c->d_bank, host.data(), host.size(), hipMemcpyHostToDevice));
  return PFMPE_OK;
}

int pfmpe_step(pfmpe_ctx* c, const pfmpe_frame_in* in, pfmpe_frame_out* out) {
  if (!c) return PFMPE_E_ARG;
  if (!in || !out) return fail(c, PFMPE_E_ARG, "step: null in/out");
  if (!c->has_model || !c->has_prior) return fail(c, PFMPE_E_STATE, "step: set_model and set_prior first");
  if (in->B < 0) return fail(c, PFMPE_E_ARG, "step: B < 0");
  if (in->B > c->max_blobs) return fail(c, PFMPE_E_CAP, "step: B exceeds max_blobs");
  if (in->it_since_init >= 2 && !(in->dt != 0.0))
    return fail(c, PFMPE_E_ARG, "step: dt must be non-zero in steady state");
  RET(set_device(c));
  const unsigned char* table = c->d_table;
  const int B = in->B;
  if (in->bank_frame >= 0) {
    if (!c->d_bank || in->bank_frame >= (int)c->bank_B.size())
      return fail(c, PFMPE_E_ARG, "step: bank_frame out of range");
    if (c->bank_B[in->bank_frame] != B) return fail(c, PFMPE_E_ARG, "step: B does not match the staged bank frame");
    table = c->d_bank + c->bank_off[in->bank_frame];
  } else {
    if (B > 0 && !in->blobs) return fail(c, PFMPE_E_ARG, "step: null blobs");
    // the x-bucketed table is built here, O(B), and travels in the same copy the blobs would
    build_table(c, in->blobs, B, c->h_table);
    HIPCHK(c, hipMemcpyAsync(c->d_table, c->h_table, table_bytes(c, B), hipMemcpyHostToDevice, c->stream));
  }
  c->timing_now = c->timing > 0 && (c->timing_frame++ % c->timing) == 0;
  const int rs = dispatch_step(c, in, table);
  if (c->timing_now) {
    c->timing_now = false;
    if (rs == PFMPE_OK) RET(harvest_timing(c));
    c->ev_used = 0;
  }
  RET(rs);

  const OutDev& o = *(const OutDev*)c->h_out;
  out->iters = o.iters;
  out->kept_iter = o.kept_iter;
  out->most_likely_idx = o.most_likely_idx;
  out->accepted = o.accepted;
  out->resampled = o.resampled;
  out->winner_idx = o.winner_idx;
  out->n_corr = o.n_corr;
  out->flag_fail = o.flag_fail;
  out->highest_prob = o.highest_prob;
  out->prob_sum = o.prob_sum;
  std::memcpy(out->winner_pose, o.winner_pose, sizeof(out->winner_pose));
  std::memcpy(out->most_likely_pose, o.most_likely_pose, sizeof(out->most_likely_pose));
  std::memcpy(out->corr, o.corr, sizeof(out->corr));

  c->has_last = true;
  c->last_prior_idx = c->prior_idx;
  c->last_accepted = o.resampled != 0;
  c->last_kept_slot = o.kept_slot;
  c->last_kept_iter = o.kept_iter;
  if (o.resampled) c->prior_idx = 1 - c->prior_idx;  // newPoseEstimation = resampled set (PE:681, 727)
  return PFMPE_OK;
}

int pfmpe_step_batch(pfmpe_ctx* c, const pfmpe_frame_in* in, int n, pfmpe_frame_out* out, int* done) {
  if (!c) return PFMPE_E_ARG;
  if (done) *done = 0;
  if ((!in || !out) && n > 0) return fail(c, PFMPE_E_ARG, "step_batch: null in/out");
  for (int f = 0; f < n; ++f) {
    RET(pfmpe_step(c, in + f, out + f));
    if (done) *done = f + 1;
  }
  return PFMPE_OK;
}

int pfmpe_get_particles(pfmpe_ctx* c, int which, double* out) {
  if (!c) return PFMPE_E_ARG;
  if (!out || (which != 0 && which != 1)) return fail(c, PFMPE_E_ARG, "get_particles: bad arguments");
  if (!c->has_prior) return fail(c, PFMPE_E_STATE, "get_particles: no particle set");
  if (which == 0 && !c->has_last) return fail(c, PFMPE_E_STATE, "get_particles(0): no step yet");
  RET(set_device(c));
  RET(ensure_xfer(c));
  const int N = c->N;
  if (which == 0) {
    RET(dispatch_regen(c, c->last_kept_iter, c->d_state[c->last_prior_idx], c->d_xfer));
  } else if (c->state_dtype == PFMPE_STATE_F64) {
    hipLaunchKernelGGL((k_export<double>), dim3((N + 255) / 256), dim3(256), 0, c->stream,
                       (const double*)c->d_state[c->prior_idx], c->d_xfer, N, c->ld);
  } else {
    hipLaunchKernelGGL((k_export<float>), dim3((N + 255) / 256), dim3(256), 0, c->stream,
                       (const float*)c->d_state[c->prior_idx], c->d_xfer, N, c->ld);
  }
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipMemcpyAsync(out, c->d_xfer, (size_t)N * 12 * sizeof(double), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  c->ev_used = 0;
  return PFMPE_OK;
}

int pfmpe_get_weights(pfmpe_ctx* c, double* out) {
  if (!c) return PFMPE_E_ARG;
  if (!out) return fail(c, PFMPE_E_ARG, "get_weights: null out");
  if (!c->has_last) return fail(c, PFMPE_E_STATE, "get_weights: no step yet");
  RET(set_device(c));
  RET(ensure_xfer(c));
  const int N = c->N;
  if (c->state_dtype == PFMPE_STATE_F64)
    hipLaunchKernelGGL((k_weights_export<double>), dim3((N + 255) / 256), dim3(256), 0, c->stream,
                       (const double*)c->d_w[c->last_kept_slot], c->d_xfer, N);
  else
    hipLaunchKernelGGL((k_weights_export<float>), dim3((N + 255) / 256), dim3(256), 0, c->stream,
                       (const float*)c->d_w[c->last_kept_slot], c->d_xfer, N);
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipMemcpyAsync(out, c->d_xfer, (size_t)N * sizeof(double), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return PFMPE_OK;
}

int pfmpe_get_counts(pfmpe_ctx* c, uint32_t* out) {
  if (!c) return PFMPE_E_ARG;
  if (!out) return fail(c, PFMPE_E_ARG, "get_counts: null out");
  if (!c->record_counts || !c->d_counts) return fail(c, PFMPE_E_STATE, "get_counts: PFMPE_OPT_RECORD_COUNTS off");
  if (!c->has_last || !c->last_accepted) return fail(c, PFMPE_E_STATE, "get_counts: last step did not resample");
  RET(set_device(c));
  HIPCHK(c, hipMemcpy(out, c->d_counts, (size_t)c->N * sizeof(uint32_t), hipMemcpyDeviceToHost));
  return PFMPE_OK;
}

// Undocumented diagnostic: reset (out == NULL) or read the kStamps stamps of the last frame (diag & 4).
int pfmpe_debug_stamps(pfmpe_ctx* c, uint64_t* out) {
  if (!c || !c->d_stamps) return PFMPE_E_STATE;
  RET(set_device(c));
  if (!out) {
    uint64_t init[kStamps] = {0};
    init[0] = init[4] = init[19] = ~0ull;  // min-stamps
    HIPCHK(c, hipMemcpy(c->d_stamps, init, sizeof(init), hipMemcpyHostToDevice));
    return PFMPE_OK;
  }
  HIPCHK(c, hipStreamSynchronize(c->stream));
  HIPCHK(c, hipMemcpy(out, c->d_stamps, kStamps * sizeof(uint64_t), hipMemcpyDeviceToHost));
  return PFMPE_OK;
}

int pfmpe_get_kernel_stats(pfmpe_ctx* c, int kernel, int64_t* launches, double* total_ms) {
  if (!c || kernel < 0 || kernel >= PFMPE_K_COUNT) return PFMPE_E_ARG;
  if (launches) *launches = c->k_launches[kernel];
  if (total_ms) *total_ms = c->k_ms[kernel];
  return PFMPE_OK;
}

int pfmpe_reset_kernel_stats(pfmpe_ctx* c) {
  if (!c) return PFMPE_E_ARG;
  for (int k = 0; k < PFMPE_K_COUNT; ++k) {
    c->k_launches[k] = 0;
    c->k_ms[k] = 0;
  }
  return PFMPE_OK;
}

const char* pfmpe_kernel_name(int kernel) {
  static const char* names[PFMPE_K_COUNT] = {"k_propagate_weigh", "k_resample", "aux"};
  return (kernel >= 0 && kernel < PFMPE_K_COUNT) ? names[kernel] : "?";
}

// ---- host-side evaluation of the device RNG code (CPU tests pin it against the oracle)
double pfmpe_host_ref_uniform(uint32_t seed, uint64_t j, double a, double b) {
  const uint32_t x0 = lcg_seed(seed);
  const uint32_t g1 = lcg_output(x0, 2 * j + 1);
  const uint32_t g2 = lcg_next(g1);
  return ref_uniform(ref_canonical(g1, g2), a, b);
}

void pfmpe_host_philox(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
  const U32x4 o = philox4x32_10(ctr[0], ctr[1], ctr[2], ctr[3], key[0], key[1]);
  out[0] = o.x;
  out[1] = o.y;
  out[2] = o.z;
  out[3] = o.w;
}

}  // extern "C"
