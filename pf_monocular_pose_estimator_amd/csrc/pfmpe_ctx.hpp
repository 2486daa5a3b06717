#pragma once
// pfmpe_ctx.hpp — engine internals shared by the C-ABI TU (pfmpe_engine.hip) and the four kernel TUs
// (pfmpe_k_<state>_<rng>.hip, one (T, RNG) instantiation each, compiled in parallel).
//
// Replaces the PF block of PoseEstimator::estimateBodyPose (pf_mpe_lib/src/pose_estimator.cpp:475-733)
// behind include/pfmpe.h.  Device layout (DESIGN.md "HBM layout"): particle state as 12 SoA planes
// (r00 r01 r02 t0 r10 r11 r12 t1 r20 r21 r22 t2) of `ld` elements each, double-buffered (prior /
// posterior); two weight slots (current iteration / best iteration so far); per-block partials;
// one control record; one output record copied to pinned host memory at the end of the frame.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <time.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstddef>
#include <cstring>
#include <string>
#include <map>
#include <memory>
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

// A batch leader's fence (pfmpe_step_multi), shared by the batch's other contexts until their next work is ordered
// after the batch; destroyed with the last reference.  The event is recorded on the leader's stream lazily: when a
// member needs the order (order_after, destroy), or when the leader puts other work on its stream while members
// still hold the fence (seal_lead_fence, ADVICE r05: a member's read-back then does not wait for the leader's later
// frames).  A steady multi-stream loop, whose members never use their own streams, records nothing (one record per
// batch cost 3-5 us of host time per batch).  stream: the leader's stream; null once the leader was destroyed (its
// destroy drained the stream first, so nothing of the batch is pending then).  recorded: the event holds the end of
// the fence's latest batch.
struct BatchFence {
  hipEvent_t ev = nullptr;
  hipStream_t stream = nullptr;
  bool recorded = false;
  ~BatchFence() {
    if (ev) (void)hipEventDestroy(ev);
  }
};

struct pfmpe_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  int max_particles = 0, max_markers = 0, max_blobs = 0, state_dtype = PFMPE_STATE_F32;
  size_t es = 4;       // bytes per state element (4 fp32, 8 fp64, 2 fp16 deltas)
  size_t ws = 4;       // bytes per weight (compute type)
  double anchor[2][12] = {{0}};  // fp16 state: anchor pose of each state buffer
  int64_t ld = 0;      // plane stride (elements)
  int max_blk = 0;

  void* d_state[2] = {nullptr, nullptr};
  int prior_idx = 0;
  void* d_w[2] = {nullptr, nullptr};
  void* d_prop[2] = {nullptr, nullptr};  // two-launch path: propagated set per weight slot (keep_prop)
  // Deferred resampling (PFMPE_OPT_DEFER_RESAMPLE): a two-launch frame with the kept set writes the
  // new prior's owner indices (d_owner[frame_owner_out]) instead of the particles; the frame's kept buffer then
  // becomes the prior's storage (swapped with the unused post buffer at take_step) and prior particle n is stored
  // row d_owner[prior_owner][n].  prior_owner = -1: the prior is stored in particle order.
  uint32_t* d_owner[2] = {nullptr, nullptr};
  int prior_owner = -1;
  int frame_owner_out = -1;  // this frame's owner buffer (-1: materialised resample)
  bool defer = true;
  int max_grp = 0;
  BlockPart* d_part[2] = {nullptr, nullptr};
  BlockScan* d_bscan[2] = {nullptr, nullptr};
  GroupPart* d_gpart[2] = {nullptr, nullptr};
  GroupScan* d_gscan = nullptr;
  CountPart* d_cpart = nullptr;
  unsigned long long* d_winkey = nullptr;  // kWinShards winner keys + the owners finish's arrival shards (kWinBytes), zero between frames
  CountPart* d_cgroup = nullptr;
  uint32_t* d_counters = nullptr;  // [prop group x max_grp][prop top][res group x max_grp][res top]
  uint32_t* d_gen = nullptr;       // k_frame iteration release word (monotonic)
  Cand* d_cand = nullptr;          // per-block winner candidates
  double* d_mlpose = nullptr;      // most likely pose (12)
  double* d_roi = nullptr;         // ROI box [4] + per-block partials
  unsigned char* d_init = nullptr; // initialisation scratch (pfmpe_init.hip), grown on demand
  size_t init_cap = 0;
  unsigned char* d_det = nullptr;  // detector scratch (pfmpe_detect.hip), grown on demand
  size_t det_cap = 0;
  uint8_t* d_img = nullptr;        // staged camera image (pfmpe_stage_image)
  size_t img_cap = 0;
  int img_w = 0, img_h = 0, img_pitch = 0;
  void* h_det = nullptr;           // detector output record (pinned, host-mapped)
  int num_cu = 0;
  bool coop = false;               // device supports cooperative launches
  int fused = 2;                   // PFMPE_OPT_FUSED: 2 flat one-launch (k_frame2), 1 tree (k_frame), 0 two launches
  uint32_t* d_flat = nullptr;      // k_frame2 sharded arrival counters (kFlatWords)
  unsigned char* d_gran = nullptr; // k_frame2 granule hand-offs (kGranBytes: block partials x 2 parities, counts)
  uint32_t gframe = 0;             // granule tag frame count (1 .. kGranFrames; the area is zeroed on wrap)
  uint32_t flat_base_w = 0, flat_base_c = 0;  // their running totals (host mirror)
  int64_t fused_fallbacks = 0;     // fused frames redone with two launches
  int fused_user = 2;              // the PFMPE_OPT_FUSED value asked for (fused drops to 0 after a fallback)
  int64_t fused_rearm = 0;         // PFMPE_OPT_FUSED_REARM: clean two-launch frames before fusing again (0: never)
  int64_t clean_since_fallback = 0;
  int64_t wait_bound_us = 2000000; // PFMPE_OPT_WAIT_BOUND_US: bound of every in-launch wait
  int64_t multi_max_blocks = 160000; // PFMPE_OPT_MULTI_MAX_BLOCKS: largest batch this context leads (blocks)
  int last_shape = -1;             // PFMPE_SHAPE_* of the last frame
  int last_weigh_pass = -1;        // PFMPE_WEIGH_* of the last two-launch weighing launch
  int last_resample = -1;          // PFMPE_RESAMPLE_* of the last two-launch resampling launch
  int64_t guard_skips = 0;         // one-launch frames run as two launches because another was in flight
  std::map<std::pair<const void*, size_t>, int> occ;  // (kernel, LDS bytes) -> blocks per CU
  // host-side timing of batches this context leads (undocumented info keys 110-114): entry -> first launch,
  // the launches, last launch -> records, records -> return, batches counted
  int64_t mt_enter = 0, mt_ns[4] = {0, 0, 0, 0}, mt_batches = 0;
  Ctrl* d_ctrl = nullptr;
  RecOut* h_rec = nullptr;       // pinned host memory: the record granules, written by the final wave
  RecOut* d_out = nullptr;       // its device address
  OutDev* h_out = nullptr;       // the last record, unpacked on the host by wait_frame
  int32_t seq = 0;               // frame-record sequence number (publication tag = 2 * seq + finished)
  unsigned char* d_table = nullptr;  // this frame's blob table (BlobTable<T> layout)
  unsigned char* h_table = nullptr;  // pinned staging
  unsigned char* d_bank = nullptr;   // staged tables of a whole stream, back to back
  std::vector<size_t> bank_off;      // byte offset of frame f's table
  std::vector<int32_t> bank_B;
  std::vector<GridHdr> bank_grid;    // frame f's table grid header (host copy, for the kernel arguments)
  std::vector<double> bank_blobs;    // the staged blobs and per-frame offsets, kept to rebuild the tables when
  std::vector<int32_t> bank_offsets; // set_params changes tol_PF (the grid's window depends on it)
  double bank_tol_pf = 0.0;          // the tol_PF the bank's tables were built for
  int last_grid = -1;                // PFMPE_INFO_LAST_GRID
  double* d_xfer = nullptr;      // N x 12 doubles
  uint32_t* d_counts = nullptr;
  uint64_t* d_stamps = nullptr;  // diagnostic stamps (diag & 4)
  // batch scratch (pfmpe_step_multi, owned by the batch's first context): stream descriptors, the
  // block -> stream map and host-supplied blob tables; the host writes the descriptors and tables into the
  // pinned image, a staging launch (k_stage_multi) moves them to HBM and builds the map
  unsigned char* d_multi = nullptr;
  hipEvent_t br_a = nullptr, br_b = nullptr;  // the open timing bracket (launch / klaunch)
  unsigned char* h_multi = nullptr;
  unsigned char* hd_multi = nullptr;  // device address of h_multi
  size_t multi_cap = 0;
  uint32_t multi_gen = 0;  // batch generation: one per staging launch this context leads (StreamDesc::gen)
  std::vector<int64_t> map_sig;  // the block map now in d_multi: {boff, total, then (first, nblk) per stream}
  // Cross-stream ordering.  A context's work runs on its own stream (pfmpe_step, read-backs, ...) or, inside a
  // batch, on the batch leader's stream.  last_stream is where its latest work went (nullptr: none since
  // create); when the next work goes to a different stream it is ordered after that work: through the
  // leader's fence when the latest work was a batch, else through own_ev recorded then on the own stream.
  hipStream_t last_stream = nullptr;
  std::shared_ptr<BatchFence> last_fence;
  hipEvent_t own_ev = nullptr;
  std::shared_ptr<BatchFence> lead_fence;  // this context as a batch leader

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
  bool keep_prop = true;           // PFMPE_OPT_KEEP_PROPAGATED (batched fp32 / fp64 frames regenerate: step_multi)
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

namespace pfmpe_impl {

// One spin-waiting (one-launch) frame per device at a time within this process: two such kernels that each
// hold part of the CUs could wait on each other until the wait bound abandons a frame.  A context that finds
// its device busy runs the frame as two launches (they never wait on other blocks, so they always drain).
constexpr int kMaxDevices = 64;
inline std::atomic<int>& fused_inflight(int dev) {
  static std::atomic<int> flags[kMaxDevices];
  return flags[(dev >= 0 && dev < kMaxDevices) ? dev : 0];
}

inline int fail(pfmpe_ctx* c, int code, const std::string& msg) {
  if (c) c->err = msg;
  return code;
}

#define HIPCHK(ctx, expr)                                                                       \
  do {                                                                                          \
    hipError_t e_ = (expr);                                                                     \
    if (e_ != hipSuccess)                                                                       \
      return fail((ctx), PFMPE_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));       \
  } while (0)

// Order work about to be enqueued for context c on stream `to` after c's latest work, when that went to
// another stream (a batch runs on the leader's stream, unordered with each member's own stream).
// Free when consecutive work stays on one stream, which is every steady-state loop (pfmpe_step only, or
// batches of the same contexts only).  err: the context that reports a failure.
inline int order_after(pfmpe_ctx* c, hipStream_t to, pfmpe_ctx* err) {
  if (!c->last_stream || c->last_stream == to) return PFMPE_OK;
  if (c->last_fence) {
    if (c->last_fence->stream) {
      if (!c->last_fence->recorded) {
        HIPCHK(err, hipEventRecord(c->last_fence->ev, c->last_fence->stream));
        c->last_fence->recorded = true;
      }
      HIPCHK(err, hipStreamWaitEvent(to, c->last_fence->ev, 0));
    }
  } else {
    if (!c->own_ev) HIPCHK(err, hipEventCreateWithFlags(&c->own_ev, hipEventDisableTiming));
    HIPCHK(err, hipEventRecord(c->own_ev, c->last_stream));
    HIPCHK(err, hipStreamWaitEvent(to, c->own_ev, 0));
  }
  c->last_stream = nullptr;
  c->last_fence.reset();
  return PFMPE_OK;
}

// A batch leader about to put other work on its stream while members of its latest batch still hold the fence:
// record the fence first, so their order_after waits for the batch and not for this later work.
inline int seal_lead_fence(pfmpe_ctx* c) {
  BatchFence* f = c->lead_fence.get();
  if (!f || f->recorded || c->lead_fence.use_count() < 2) return PFMPE_OK;
  HIPCHK(c, hipEventRecord(f->ev, c->stream));
  f->recorded = true;
  return PFMPE_OK;
}

// Every C-ABI entry that enqueues work on the context's own stream starts here: the device, the leader's fence, then
// the order after the context's latest batch (if any).
inline int set_device(pfmpe_ctx* c) {
  HIPCHK(c, hipSetDevice(c->device));
  if (const int r_ = seal_lead_fence(c)) return r_;
  if (const int r_ = order_after(c, c->stream, c)) return r_;
  c->last_stream = c->stream;
  return PFMPE_OK;
}

// ---------------------------------------------------------------------- timed launch wrapper
// A bracketed launch passes its events to the dispatch itself (hipExtLaunchKernel: the start event takes the
// first kernel's start, the stop event each kernel's end, so the last one's), so the bracket is the kernels'
// own execution time as the profiler's kernel trace reports it.  Plain hipEventRecord brackets on an idle
// stream (every one-launch frame: the host waited for the previous record) also held the dispatch of the
// kernel, +8 us at C2 (37.5 against rocprofv3's 29.4).  Every kernel of a launch_ext bracket goes through
// klaunch.
inline int open_bracket(pfmpe_ctx* c, int kid, EventPair** out) {
  *out = nullptr;
  if (!c->timing_now) return PFMPE_OK;
  if (c->ev_used == c->ev_pool.size()) {
    EventPair p{};
    p.kid = kid;
    HIPCHK(c, hipEventCreate(&p.a));
    HIPCHK(c, hipEventCreate(&p.b));
    c->ev_pool.push_back(p);
  }
  *out = &c->ev_pool[c->ev_used++];
  (*out)->kid = kid;
  return PFMPE_OK;
}
// the PF frame's kernels (launched through klaunch)
template <typename Launch>
int launch_ext(pfmpe_ctx* c, int kid, Launch&& fn) {
  EventPair* ep = nullptr;
  if (const int r_ = open_bracket(c, kid, &ep)) return r_;
  if (ep) {
    c->br_a = ep->a;
    c->br_b = ep->b;
  }
  fn();
  c->br_a = c->br_b = nullptr;
  HIPCHK(c, hipGetLastError());
  return PFMPE_OK;
}
// the initialisation, ROI and detector launches: hipEventRecord brackets around the stream's work
template <typename Launch>
int launch(pfmpe_ctx* c, int kid, Launch&& fn) {
  EventPair* ep = nullptr;
  if (const int r_ = open_bracket(c, kid, &ep)) return r_;
  if (ep) HIPCHK(c, hipEventRecord(ep->a, c->stream));
  fn();
  HIPCHK(c, hipGetLastError());
  if (ep) HIPCHK(c, hipEventRecord(ep->b, c->stream));
  return PFMPE_OK;
}
template <typename... KArgs, typename... Args>
inline void klaunch(pfmpe_ctx* c, void (*kernel)(KArgs...), dim3 grid, dim3 block, size_t lds, Args... args) {
  if (c->br_b) {
    hipExtLaunchKernelGGL(kernel, grid, block, (uint32_t)lds, c->stream, c->br_a, c->br_b, 0u, args...);
    c->br_a = nullptr;  // the bracket starts at its first kernel
  } else {
    hipLaunchKernelGGL(kernel, grid, block, lds, c->stream, args...);
  }
}

// Brackets are harvested lazily: a timed PF frame leaves its event pairs pending (no stream synchronize on the
// frame path, which had added a host round trip to every sampled frame: at --steps 20 one frame in two), and
// they are read here, when the pool holds kHarvestPairs of them, at pfmpe_get_kernel_stats, or after the
// host-synchronous entries (ROI, read-backs, initialisation, detector).  Every bracket is recorded on c->stream,
// so waiting for the last one's end event completes them all.
constexpr size_t kHarvestPairs = 256;
constexpr size_t kEventPrealloc = 64;  // event pairs created when timing is switched on (PFMPE_OPT_TIMING)
inline int harvest_timing(pfmpe_ctx* c) {
  if (c->ev_used == 0) return PFMPE_OK;
  HIPCHK(c, hipEventSynchronize(c->ev_pool[c->ev_used - 1].b));
  for (size_t i = 0; i < c->ev_used; ++i) {
    float ms = 0.f;
    HIPCHK(c, hipEventElapsedTime(&ms, c->ev_pool[i].a, c->ev_pool[i].b));
    c->k_launches[c->ev_pool[i].kid] += 1;
    c->k_ms[c->ev_pool[i].kid] += ms;
  }
  c->ev_used = 0;
  return PFMPE_OK;
}

// Wait for the frame record: the final wave writes it into pinned host memory as tagged granules (RecOut),
// so the host spins on those words instead of paying a stream synchronize, and unpacks them into h_out once
// every granule carries the tag.  Granule 0 alone with an even tag is an unfinished iteration batch.  The
// spin is bounded by hipStreamQuery: an idle stream without a record is an error.
inline bool take_record(pfmpe_ctx* c, int32_t want) {
  volatile const uint64_t* g = c->h_rec->g;
  const uint32_t t = (uint32_t)(g[0] >> 32);
  if ((int32_t)(t >> 1) != want) return false;
  if (t & 1u) {
    for (int k = kRecWords - 1; k > 0; --k)
      if ((uint32_t)(g[k] >> 32) != t) return false;
    __atomic_thread_fence(__ATOMIC_ACQUIRE);
    uint32_t* w = (uint32_t*)c->h_out;
    for (int k = 0; k < kRecWords; ++k) w[k] = (uint32_t)g[k];
  }
  c->h_out->tag = (int32_t)t;
  return true;
}
// The stream is queried only after the record has been awaited for kQueryAfterNs, then at that interval: a query
// costs microseconds of host time (3.4 us under the HIP API trace), and one issued while the record lands delays
// the frame by that much (at C2 the old every-1,024-spins query fell inside nearly every frame).
constexpr int64_t kQueryAfterNs = 200000;
inline int64_t now_ns() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (int64_t)ts.tv_sec * 1000000000ll + ts.tv_nsec;
}
inline int wait_frame(pfmpe_ctx* c, hipStream_t on = nullptr) {  // on: the frame's stream
  const int32_t want = c->seq;
  int64_t next_query = 0;
  for (uint64_t spin = 0;; ++spin) {
    if (take_record(c, want)) return PFMPE_OK;
    if ((spin & 63u) != 63u) {
      __builtin_ia32_pause();
      continue;
    }
    const int64_t t = now_ns();
    if (next_query == 0) next_query = t + kQueryAfterNs;
    if (t >= next_query) {
      next_query = t + kQueryAfterNs;
      const hipError_t q = hipStreamQuery(on ? on : c->stream);
      if (q == hipSuccess) {
        if (take_record(c, want)) return PFMPE_OK;
        return fail(c, PFMPE_E_HIP, "frame record was not written");
      }
      if (q != hipErrorNotReady) return fail(c, PFMPE_E_HIP, std::string("stream error: ") + hipGetErrorString(q));
    }
    __builtin_ia32_pause();
  }
}

inline size_t counters_bytes(const pfmpe_ctx* c) { return (size_t)(2 * c->max_grp + 2) * sizeof(uint32_t); }

inline bool frame_done(const pfmpe_ctx* c) { return (c->h_out->tag & 1) != 0; }

#define RET(expr)              \
  do {                         \
    int r_ = (expr);           \
    if (r_ != PFMPE_OK) return r_; \
  } while (0)

// ---------------------------------------------------------------------- typed launch sequence
template <typename T> FrameArgsT<T>& last_args(pfmpe_ctx* c);
template <> inline FrameArgsT<float>& last_args<float>(pfmpe_ctx* c) { return c->last_fa_f; }
template <> inline FrameArgsT<double>& last_args<double>(pfmpe_ctx* c) { return c->last_fa_d; }

// the two-launch path's propagated-set buffers (PFMPE_OPT_KEEP_PROPAGATED), allocated on first use: the
// one-launch frames keep the propagated particle in registers and never need them
inline int ensure_prop(pfmpe_ctx* c) {
  if (!c->keep_prop) return PFMPE_OK;
  if (!c->d_prop[0]) {
    const size_t bytes = (size_t)kPlanes * c->ld * c->es;
    for (int i = 0; i < 2; ++i) HIPCHK(c, hipMalloc(&c->d_prop[i], bytes));
  }
  if (c->defer && !c->d_owner[0]) {  // both or neither: deferral is gated on both pointers
    const size_t bytes = (size_t)c->ld * sizeof(uint32_t);
    hipError_t e = hipMalloc((void**)&c->d_owner[0], bytes);
    if (e == hipSuccess) e = hipMalloc((void**)&c->d_owner[1], bytes);
    if (e != hipSuccess) {
      if (c->d_owner[0]) (void)hipFree(c->d_owner[0]);
      c->d_owner[0] = c->d_owner[1] = nullptr;
      return fail(c, PFMPE_E_HIP, std::string("owner buffers: ") + hipGetErrorString(e));
    }
  }
  return PFMPE_OK;
}
// the owner indices of the current prior (null: stored in particle order)
inline const uint32_t* prior_owner_ptr(const pfmpe_ctx* c) {
  return c->prior_owner >= 0 ? c->d_owner[c->prior_owner] : nullptr;
}

// Batch scratch layout (pfmpe_step_multi), the same in the pinned host image and in HBM: host-supplied blob
// tables [0, tbytes), then `na` stream descriptors from doff, then the uint16 block -> stream map of `total`
// blocks from boff; `need` bytes in all.
struct BatchLayout {
  size_t doff, boff, soff, need;
};
template <typename Desc>
inline BatchLayout batch_layout(int na, int64_t total, size_t tbytes) {
  BatchLayout L;
  L.doff = tbytes;
  L.boff = L.doff + ((size_t)na * sizeof(Desc) + 255) / 256 * 256;
  L.soff = L.boff + ((size_t)total * sizeof(uint16_t) + 255) / 256 * 256;  // uint32 status[na] (k_stage_multi)
  L.need = L.soff + (size_t)na * sizeof(uint32_t) + 256;
  return L;
}
// Blocks per batch accepted by pfmpe_step_multi (PFMPE_E_CAP above): the size the GPU tests cover
// (tests/test_gpu_multi.py: 4 x 10M fp16 particles in one batch = 156,252 blocks; 32 x 1M in the bench).
constexpr int64_t kMultiMaxBlocks = 160000;

// The frames k_weigh_pk covers (pf_weigh_pk.hpp): fp32 compute, the Philox stream, exactly five markers (the
// instance), fp32 or fp16 pair-plane state, and per frame: the blob grid on (which implies pruning and fp32), the
// short sincos polynomials, an identity camMoveInv, an upper-triangular K, B >= M (the order-free score),
// blob 0 finite (the NaN-at-origin test by one comparison).  Everything else: k_weigh_stream.
template <typename T, int RNG, int MAXM, typename SP>
constexpr bool kPkInstance = std::is_same<T, float>::value && RNG == kRngPhilox && MAXM == kExactM &&
                             (std::is_same<SP, float>::value || std::is_same<SP, __half>::value);
inline bool pk_eligible(const FrameArgsT<float>& fa) {
  return fa.grid.on && fa.grid.b0fin && fa.small_angles && fa.cam_identity && fa.k_upper && fa.M == kExactM &&
         fa.B >= fa.M && !(fa.diag & (kDiagNoPk | kDiagSortedScore));
}
// the 12-marker packed pass (k_weigh_pk12, pf_weigh_pk.hpp; C3): the same frames with exactly 12 markers
template <typename T, int RNG, int MAXM, typename SP>
constexpr bool kPk12Instance = std::is_same<T, float>::value && RNG == kRngPhilox && MAXM == kPk12M &&
                               (std::is_same<SP, float>::value || std::is_same<SP, __half>::value);
inline bool pk12_eligible(const FrameArgsT<float>& fa) {
  return fa.grid.on && fa.grid.b0fin && fa.small_angles && fa.cam_identity && fa.k_upper && fa.M == kPk12M &&
         fa.B >= fa.M && !(fa.diag & (kDiagNoPk | kDiagSortedScore));
}
template <typename T, int RNG, int MAXM, typename SP>
inline const void* pk_kernel() {
  if constexpr (kPkInstance<T, RNG, MAXM, SP>)
    return (const void*)k_weigh_pk<SP>;
  else if constexpr (kPk12Instance<T, RNG, MAXM, SP>)
    return (const void*)k_weigh_pk12<SP>;
  else
    return nullptr;
}

// A two-launch frame or batch that left no record (a bounded wait expired, or a HIP error): the control record, the
// winner keys, the fused finish's arrival shards and the hand-off counters may hold the failed frame's partial state,
// which the next frame would take as its own (the control record's iteration state; a finisher that stops polling
// early).  Zero them once `on` has drained, as abandoned() does for a one-launch frame; the prior is untouched.
inline int reset_handoffs(pfmpe_ctx* c, hipStream_t on) {
  HIPCHK(c, hipStreamSynchronize(on));
  HIPCHK(c, hipMemsetAsync(c->d_ctrl, 0, sizeof(Ctrl), c->stream));
  HIPCHK(c, hipMemsetAsync(c->d_counters, 0, counters_bytes(c), c->stream));
  HIPCHK(c, hipMemsetAsync(c->d_winkey, 0, kWinBytes, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return PFMPE_OK;
}

// A one-launch frame abandoned by a bounded wait (blocks not co-resident: other work on the device): clear the
// hand-off state, stop fusing on this context; the caller redoes the frame with two launches.
inline int abandoned(pfmpe_ctx* c) {
  HIPCHK(c, hipStreamSynchronize(c->stream));
  HIPCHK(c, hipMemsetAsync(c->d_counters, 0, counters_bytes(c), c->stream));
  HIPCHK(c, hipMemsetAsync(c->d_ctrl, 0, sizeof(Ctrl), c->stream));
  HIPCHK(c, hipMemsetAsync(c->d_winkey, 0, kWinBytes, c->stream));
  if (c->d_flat) HIPCHK(c, hipMemsetAsync(c->d_flat, 0, kFlatWords * sizeof(uint32_t), c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  c->flat_base_w = c->flat_base_c = 0;
  c->fused_fallbacks += 1;
  c->fused = 0;
  c->clean_since_fallback = 0;
  // not an error (the frame is redone and returns OK); the text and pfmpe_get_info report it
  c->err = "one-launch frame abandoned at the wait bound (blocks not co-resident: other work on the device?); "
           "redone with two launches, one-launch frames off" +
           std::string(c->fused_rearm > 0 ? " until PFMPE_OPT_FUSED_REARM clean frames" : "");
  return PFMPE_OK;
}
// This flat frame's granule tag base (FrameArgsT::gtag): frame count << 12, never 0.  On wrap the granule area is
// zeroed first, so no stored word carries a tag a later frame uses (the stream must be free: no server running).
constexpr uint32_t kGranFrames = 0xFFFFF;
inline int next_gtag(pfmpe_ctx* c, uint32_t* gtag) {
  if (c->gframe >= kGranFrames) {
    HIPCHK(c, hipMemsetAsync(c->d_gran, 0, kGranBytes, c->stream));
    c->gframe = 0;
  }
  c->gframe += 1;
  *gtag = c->gframe << 12;
  return PFMPE_OK;
}
inline BlockPart* gran_part(const pfmpe_ctx* c, int parity) {
  return (BlockPart*)(c->d_gran + (size_t)parity * kGranPartBytes);
}
inline CountPart* gran_count(const pfmpe_ctx* c) { return (CountPart*)(c->d_gran + kGranCountOff); }

template <typename T, int RNG, int MAXM, typename SP>
struct Seq {
  static int iterate(pfmpe_ctx* c, const FrameArgsT<T>& fa, const unsigned char* table, int iter) {
    const SP* prior = (const SP*)c->d_state[c->prior_idx];
    const size_t lds = BlobTable<T>::lds_bytes(fa.tbytes);
    uint32_t* gcount = c->d_counters;
    uint32_t* tcount = c->d_counters + c->max_grp;
    RET(ensure_prop(c));
    SP* prop0 = c->keep_prop ? (SP*)c->d_prop[0] : nullptr;
    SP* prop1 = c->keep_prop ? (SP*)c->d_prop[1] : nullptr;
    // The streaming weighing pass (k_weigh_stream: resident blocks looping over the 256-particle blocks, the
    // next particle's state prefetched) with the group / top hand-off as two small launches.  It wins for
    // every marker bucket: C5 52 -> 31 us weighing (round 2), C4 265 -> 233 us; at 12 markers (C3) it lost while
    // the pass staged block partials through LDS behind two barriers per block, and wins since it stores wave
    // partials (round 3: C3 116-117 -> 111-113 us per frame, profiles/r03/ab_c3_stream.log).
    // kDiagNoStream / kDiagForceStream pick either pass for tests and A/B.
    const bool stream = !(c->diag & kDiagNoStream);
    // k_weigh_pk: the streaming pass with two particles per lane in packed fp32 (pf_weigh_pk.hpp), for the
    // frames it covers (pk_eligible); same outputs, same bits
    bool pk = false;
    if constexpr (kPkInstance<T, RNG, MAXM, SP>) pk = stream && c->prune && pk_eligible(fa);
    if constexpr (kPk12Instance<T, RNG, MAXM, SP>) pk = stream && c->prune && pk12_eligible(fa);
    c->last_weigh_pass = pk ? PFMPE_WEIGH_PK : (stream ? PFMPE_WEIGH_STREAM : PFMPE_WEIGH_BLOCKS);
    if (stream) {
      const void* fn = pk ? pk_kernel<T, RNG, MAXM, SP>()
                          : (c->prune ? (const void*)k_weigh_stream<T, RNG, MAXM, true, SP>
                                      : (const void*)k_weigh_stream<T, RNG, MAXM, false, SP>);
      auto key = std::make_pair(fn, lds);
      auto it = c->occ.find(key);
      if (it == c->occ.end()) {
        int per_cu = 0;
        HIPCHK(c, hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, kBlock, lds));
        it = c->occ.emplace(key, std::max(1, per_cu)).first;
      }
      // k_weigh_pk: a wave per 128-particle task, 2 * nblk tasks
      const int grid = std::min(pk ? (fa.nblk + 1) / 2 : fa.nblk, it->second * std::max(1, c->num_cu));
      RET(launch_ext(c, PFMPE_K_PROPAGATE, [&] {
        if constexpr (kPkInstance<T, RNG, MAXM, SP>) {
          if (pk) {
            klaunch(c, k_weigh_pk<SP>, dim3(grid), dim3(kBlock), lds, fa, table, prior, (float*)c->d_w[0],
                    (float*)c->d_w[1], c->d_part[0], c->d_part[1], (const Ctrl*)c->d_ctrl, prop0, prop1, iter);
            return;
          }
        }
        if constexpr (kPk12Instance<T, RNG, MAXM, SP>) {
          if (pk) {
            klaunch(c, k_weigh_pk12<SP>, dim3(grid), dim3(kBlock), lds, fa, table, prior, (float*)c->d_w[0],
                    (float*)c->d_w[1], c->d_part[0], c->d_part[1], (const Ctrl*)c->d_ctrl, prop0, prop1, iter);
            return;
          }
        }
        if (c->prune)
          klaunch(c, k_weigh_stream<T, RNG, MAXM, true, SP>, dim3(grid), dim3(kBlock), lds, fa,
                             table, prior, (T*)c->d_w[0], (T*)c->d_w[1], c->d_part[0], c->d_part[1], c->d_ctrl, prop0,
                             prop1, iter);
        else
          klaunch(c, k_weigh_stream<T, RNG, MAXM, false, SP>, dim3(grid), dim3(kBlock), lds, fa,
                             table, prior, (T*)c->d_w[0], (T*)c->d_w[1], c->d_part[0], c->d_part[1], c->d_ctrl, prop0,
                             prop1, iter);
      }));
      // the top's group partials fit LDS up to 1,365 groups (22M particles); beyond, it reads them from L2
      const size_t glds = fa.ngrp > 64 ? (size_t)fa.ngrp * sizeof(GroupPart) : 0;
      const bool staged = glds > 0 && glds <= 64 * 1024;
      if (fa.ngrp <= 64 && !(c->diag & kDiagSerialTop))  // one tile: group scans + top in one launch
        return launch_ext(c, PFMPE_K_AUX, [&] {
          klaunch(c, k_group_top<T, RNG>, dim3(fa.ngrp), dim3(64), 0, fa, c->d_part[0], c->d_part[1], c->d_bscan[0],
                  c->d_bscan[1], c->d_gpart[0], c->d_gpart[1], c->d_gscan, c->d_ctrl, tcount, iter);
        });
      return launch_ext(c, PFMPE_K_AUX, [&] {
        klaunch(c, k_group<T>, dim3(fa.ngrp), dim3(64), 0, fa, c->d_part[0], c->d_part[1],
                           c->d_bscan[0], c->d_bscan[1], c->d_gpart[0], c->d_gpart[1], (const Ctrl*)c->d_ctrl);
        if (staged && fa.ngrp <= 64 * kTopMaxTiles && !(c->diag & kDiagSerialTop))  // > 1 tile: k_top_wide
          klaunch(c, k_top_wide<T, RNG>, dim3(1), dim3(64 * kTopWaves), glds, fa, c->d_gpart[0], c->d_gpart[1],
                  c->d_gscan, c->d_ctrl, iter);
        else
          klaunch(c, k_top<T, RNG>, dim3(1), dim3(64), staged ? glds : 0, fa, c->d_gpart[0],
                             c->d_gpart[1], c->d_gscan, c->d_ctrl, iter, staged ? 1 : 0);
      });
    }
    return launch_ext(c, PFMPE_K_PROPAGATE, [&] {
      if (c->prune)
        klaunch(c, k_propagate_weigh<T, RNG, MAXM, true, SP>, dim3(fa.nblk), dim3(kBlock), lds, fa,
                           table, prior, (T*)c->d_w[0], (T*)c->d_w[1], c->d_part[0], c->d_part[1], c->d_bscan[0],
                           c->d_bscan[1], c->d_gpart[0], c->d_gpart[1], c->d_gscan, c->d_ctrl, gcount, tcount, prop0,
                           prop1, iter, c->d_stamps);
      else
        klaunch(c, k_propagate_weigh<T, RNG, MAXM, false, SP>, dim3(fa.nblk), dim3(kBlock), lds, fa,
                           table, prior, (T*)c->d_w[0], (T*)c->d_w[1], c->d_part[0], c->d_part[1], c->d_bscan[0],
                           c->d_bscan[1], c->d_gpart[0], c->d_gpart[1], c->d_gscan, c->d_ctrl, gcount, tcount, prop0,
                           prop1, iter, c->d_stamps);
    });
  }
  static int finish(pfmpe_ctx* c, const FrameArgsT<T>& fa, const unsigned char* table) {
    const SP* prior = (const SP*)c->d_state[c->prior_idx];
    SP* post = (SP*)c->d_state[1 - c->prior_idx];
    uint32_t* gcount = c->d_counters + c->max_grp + 1;
    uint32_t* tcount = c->d_counters + 2 * c->max_grp + 1;
    c->seq = (c->seq + 1) & 0x3fffffff;
    const int32_t seq = c->seq;
    const bool kept = c->keep_prop && c->d_prop[0];  // iterate() allocated them
    // deferred resampling: the new prior's owner indices go to the owner buffer the current prior does not use
    FrameArgsT<T> far = fa;
    c->frame_owner_out = -1;
    if (kept && c->defer && c->d_owner[0] && c->d_owner[1] && !(c->diag & kDiagNoDefer)) {
      c->frame_owner_out = c->prior_owner == 0 ? 1 : 0;
      far.owner_out = c->d_owner[c->frame_owner_out];
    }
    bool owners = false;
    RET(launch_ext(c, PFMPE_K_RESAMPLE, [&] {
      // a deferred frame: one wave per 256-particle block (k_resample_owners), same outputs; its
      // last wave finishes the frame (no k_resample_final)
      if (far.owner_out && !(c->diag & kDiagBlockResample)) {
        owners = true;
        klaunch(c, k_resample_owners<T, RNG, MAXM, SP>, dim3((unsigned)((fa.nblk + kWaves - 1) / kWaves)),
                dim3(kBlock), 0, far, c->d_ctrl, prior, (const T*)c->d_w[0], (const T*)c->d_w[1], c->d_bscan[0],
                c->d_bscan[1], c->d_gscan, c->record_counts ? c->d_counts : nullptr, c->d_mlpose, c->d_winkey,
                win_arrive(c->d_winkey), table, c->d_out, seq, c->d_stamps);
        return;
      }
      // the kept-set variant compiles the regeneration path out (its registers spilled in the generic form)
      auto k = kept ? k_resample<T, RNG, MAXM, SP, true> : k_resample<T, RNG, MAXM, SP, false>;
      klaunch(c, k, dim3(fa.nblk), dim3(kBlock), 0, far, c->d_ctrl, table,
                         prior, post, (const T*)c->d_w[0], (const T*)c->d_w[1], c->d_bscan[0], c->d_bscan[1],
                         c->d_gscan, c->d_cpart, c->d_cgroup, gcount, tcount,
                         c->record_counts ? c->d_counts : nullptr, c->d_cand, c->d_mlpose, c->d_out, seq,
                         c->d_stamps, kept ? (const SP*)c->d_prop[0] : nullptr,
                         kept ? (const SP*)c->d_prop[1] : nullptr, c->d_winkey);
    }));
    c->last_resample = owners ? PFMPE_RESAMPLE_OWNERS : PFMPE_RESAMPLE_BLOCKS;
    if (!owners)
      RET(launch_ext(c, PFMPE_K_FINAL, [&] {
        klaunch(c, k_resample_final<T, RNG, MAXM, SP>, dim3(1), dim3(kFinalBlock), BlobTable<T>::bytes(fa.B), fa,
                c->d_ctrl, table, prior, c->d_cpart, c->d_cand, c->d_mlpose, c->d_out, seq, c->d_stamps, kept ? 1 : 0,
                c->d_winkey);
      }));
    if (const int rc = wait_frame(c); rc != PFMPE_OK) {
      const std::string err = c->err;
      (void)reset_handoffs(c, c->stream);
      return fail(c, rc, err);
    }
    return PFMPE_OK;
  }
  // the whole frame as one launch, if every block can be resident at once: k_frame2 (flat hand-offs,
  // c->fused == 2, <= 512 blocks) or k_frame (tree hand-offs)
  template <bool PRUNE>
  static int frame_fused(pfmpe_ctx* c, const FrameArgsT<T>& fa_in, const unsigned char* table, bool* launched) {
    *launched = false;
    const bool flat = c->fused == 2 && fa_in.nblk <= kFlatMaxGroups * kGroup && fa_in.gsz == kGroup && c->d_flat;
    const void* fn = flat ? (const void*)k_frame2<T, RNG, MAXM, PRUNE, SP> : (const void*)k_frame<T, RNG, MAXM, PRUNE, SP>;
    const size_t lds = BlobTable<T>::lds_bytes(fa_in.tbytes);
    auto key = std::make_pair(fn, lds);
    auto it = c->occ.find(key);
    if (it == c->occ.end()) {
      int per_cu = 0;
      HIPCHK(c, hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, kBlock, lds));
      it = c->occ.emplace(key, per_cu).first;
    }
    // Residency by grid size alone (cdna_hip_programming.md §1): at most 2 blocks per CU and one below the
    // occupancy answer (which over-reports by one for SGPR-heavy kernels).  A plain launch: the
    // cooperative launch would only add this check at +15-19 us per frame (MI355X_MICROARCH.md
    // "coop-launch"); every in-kernel wait is bounded anyway.
    const int per_cu = std::min(2, it->second - 1);
    if (per_cu < 1 || (int64_t)per_cu * c->num_cu < fa_in.nblk) return PFMPE_OK;  // two-launch path
    std::atomic<int>& busy = fused_inflight(c->device);
    int expect = 0;
    if (!busy.compare_exchange_strong(expect, 1)) {  // another context's one-launch frame is on the device
      c->guard_skips += 1;
      return PFMPE_OK;
    }
    struct Release {
      std::atomic<int>& b;
      ~Release() { b.store(0); }
    } release{busy};
    FrameArgsT<T> a = fa_in;
    a.flat_base_w = c->flat_base_w;
    a.flat_base_c = c->flat_base_c;
    // granule tags: k_frame2's hand-offs, and k_frame's count barrier unless it runs as a tree (kDiagTreeCount)
    // (the flat count barrier's poll covers <= kFlatMaxGroups * kGroup blocks: at most 2 per CU on 256 CUs)
    const bool tree_count = !flat && ((c->diag & kDiagTreeCount) || a.nblk > kFlatMaxGroups * kGroup);
    if (!tree_count) RET(next_gtag(c, &a.gtag));
    const SP* prior = (const SP*)c->d_state[c->prior_idx];
    SP* post = (SP*)c->d_state[1 - c->prior_idx];
    T* w0 = (T*)c->d_w[0];
    T* w1 = (T*)c->d_w[1];
    uint32_t* gcount_w = c->d_counters;
    uint32_t* tcount_w = c->d_counters + c->max_grp;
    uint32_t* gcount_r = c->d_counters + c->max_grp + 1;
    uint32_t* tcount_r = c->d_counters + 2 * c->max_grp + 1;
    uint32_t* counts = c->record_counts ? c->d_counts : nullptr;
    c->seq = (c->seq + 1) & 0x3fffffff;
    int32_t seq = c->seq;
    RET(launch_ext(c, PFMPE_K_FRAME, [&] {
      if (flat)
        klaunch(c, k_frame2<T, RNG, MAXM, PRUNE, SP>, dim3(a.nblk), dim3(kBlock), lds, a, table,
                           prior, post, w0, w1, gran_part(c, 0), gran_part(c, 1), c->d_ctrl, gran_count(c), c->d_flat,
                           counts, c->d_cand, c->d_mlpose, c->d_out, seq, c->d_stamps);
      else
        klaunch(c, k_frame<T, RNG, MAXM, PRUNE, SP>, dim3(a.nblk), dim3(kBlock), lds, a, table,
                           prior, post, w0, w1, c->d_part[0], c->d_part[1], c->d_bscan[0], c->d_bscan[1],
                           c->d_gpart[0], c->d_gpart[1], c->d_gscan, c->d_ctrl,
                           tree_count ? c->d_cpart : gran_count(c), c->d_cgroup, gcount_w,
                           tcount_w, gcount_r, tcount_r, c->d_gen, counts, c->d_cand, c->d_mlpose, c->d_out, seq,
                           c->d_stamps, tree_count ? nullptr : c->d_flat);
    }));
    *launched = true;
    if (wait_frame(c) != PFMPE_OK) {
      RET(abandoned(c));
      *launched = false;
      return PFMPE_OK;
    }
    if (flat || !(c->diag & kDiagTreeCount)) {  // the flat counters' new running totals (k_frame: the count set only)
      const OutDev& o = *(const OutDev*)c->h_out;
      if (flat) c->flat_base_w += (uint32_t)o.iters * (uint32_t)a.nblk;
      if (o.resampled) c->flat_base_c += (uint32_t)a.nblk;
    }
    return PFMPE_OK;
  }

  static int step(pfmpe_ctx* c, const FrameArgsT<T>& fa, const unsigned char* table) {
    if (!c->fused && c->fused_user && c->fused_rearm > 0 && c->clean_since_fallback >= c->fused_rearm)
      c->fused = c->fused_user;  // re-armed after enough clean two-launch frames
    const int64_t fallbacks0 = c->fused_fallbacks;
    if (c->fused) {
      bool launched = false;
      RET(c->prune ? frame_fused<true>(c, fa, table, &launched) : frame_fused<false>(c, fa, table, &launched));
      if (launched) {
        if (!frame_done(c)) return fail(c, PFMPE_E_STATE, "fused frame did not finish");
        c->last_shape = (c->fused == 2 && fa.nblk <= kFlatMaxGroups * kGroup && fa.gsz == kGroup) ? PFMPE_SHAPE_FRAME2
                                                                                                   : PFMPE_SHAPE_FRAME;
        last_args<T>(c) = fa;
        return PFMPE_OK;
      }
    }
    c->last_shape = PFMPE_SHAPE_TWO_LAUNCH;
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
    if (!c->fused && c->fused_fallbacks == fallbacks0) c->clean_since_fallback += 1;  // not the redone frame
    last_args<T>(c) = fa;
    return PFMPE_OK;
  }
  // A stream of a batch left no frame record.  If some descriptor failed the staging check (status != gen),
  // report it as PFMPE_E_STATE with the words the device read that differ from the ones the host wrote (the
  // HBM copy k_stage_multi made); otherwise it is the wait's own error.  No kernel followed a pointer of a
  // failed descriptor, and a failed batch changes no context's prior (take_step is not reached).
  static int batch_failure(pfmpe_ctx* c0, pfmpe_ctx* const* cs, const std::vector<int>& act,
                           const std::vector<StreamDesc<T, SP>>& want, const unsigned char* ddesc, const uint32_t* dstat,
                           uint32_t gen, const std::string& wait_err) {
    using Desc = StreamDesc<T, SP>;
    const int na = (int)act.size();
    std::vector<uint32_t> st(na, 0);
    std::vector<Desc> seen(na);
    if (hipStreamSynchronize(c0->stream) != hipSuccess ||
        hipMemcpy(st.data(), dstat, (size_t)na * sizeof(uint32_t), hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy((void*)seen.data(), ddesc, (size_t)na * sizeof(Desc), hipMemcpyDeviceToHost) != hipSuccess)
      return fail(c0, PFMPE_E_HIP, "step_multi: " + wait_err);
    static const std::pair<size_t, const char*> kFields[] = {
        {offsetof(Desc, table), "table"},   {offsetof(Desc, prior), "prior"},   {offsetof(Desc, post), "post"},
        {offsetof(Desc, w0), "w0"},         {offsetof(Desc, w1), "w1"},         {offsetof(Desc, part0), "part0"},
        {offsetof(Desc, part1), "part1"},   {offsetof(Desc, bscan0), "bscan0"}, {offsetof(Desc, bscan1), "bscan1"},
        {offsetof(Desc, gpart0), "gpart0"}, {offsetof(Desc, gpart1), "gpart1"}, {offsetof(Desc, gscan), "gscan"},
        {offsetof(Desc, ctrl), "ctrl"},     {offsetof(Desc, gcount_w), "gcount_w"}, {offsetof(Desc, tcount_w), "tcount_w"},
        {offsetof(Desc, gcount_r), "gcount_r"}, {offsetof(Desc, tcount_r), "tcount_r"}, {offsetof(Desc, prop0), "prop0"},
        {offsetof(Desc, prop1), "prop1"},   {offsetof(Desc, cpart), "cpart"},   {offsetof(Desc, cgroup), "cgroup"},
        {offsetof(Desc, counts), "counts"}, {offsetof(Desc, cand), "cand"},     {offsetof(Desc, mlpose), "mlpose"},
        {offsetof(Desc, out), "out"},       {offsetof(Desc, winkey), "winkey"},
        {offsetof(Desc, seq), "seq|first_blk"}, {offsetof(Desc, gen), "gen"},
        {offsetof(Desc, tag), "tag"},       {offsetof(FrameArgsT<T>, key0), "fa.key0|key1"},
        {offsetof(FrameArgsT<T>, flo), "fa.flo|fhi"}};
    auto name = [&](size_t off) -> std::string {
      for (const auto& f : kFields)
        if (f.first == off) return f.second;
      return off < sizeof(FrameArgsT<T>) ? "fa+" + std::to_string(off) : "+" + std::to_string(off);
    };
    for (int i = 0; i < na; ++i) {
      if (st[i] == gen) continue;
      std::string msg = "step_multi: stream " + std::to_string(act[i]) + ": descriptor failed the staging check (gen " +
                        std::to_string(gen) + ", status " + std::to_string(st[i]) + "); words read != written:";
      const uint64_t* a = (const uint64_t*)&want[i];
      const uint64_t* b = (const uint64_t*)&seen[i];
      int shown = 0;
      for (size_t k = 0; k < sizeof(Desc) / 8 && shown < 8; ++k)
        if (a[k] != b[k]) {
          char buf[96];
          std::snprintf(buf, sizeof buf, " %s host 0x%llx device 0x%llx;", name(8 * k).c_str(), (unsigned long long)a[k],
                        (unsigned long long)b[k]);
          msg += buf;
          ++shown;
        }
      if (!shown) msg += " none (the tag or generation check failed on words equal to the host's)";
      cs[act[i]]->err = msg;
      return fail(c0, PFMPE_E_STATE, msg);
    }
    return fail(c0, PFMPE_E_HIP, "step_multi: " + wait_err);
  }
  // S contexts' frames as ONE batch on cs[0]'s HIP stream (pfmpe_step_multi): one weighing launch over every
  // stream's blocks, one resampling launch, one finishing launch with a block per stream.  Streams whose exit
  // rule did not fire on the first iteration get further iteration batches (the others are not relaunched),
  // exactly as step()'s two-launch path does for one stream.  h / d: the batch scratch, whose first
  // `tbytes` bytes already hold the host-supplied blob tables; tables[s] are device addresses.  The caller
  // (multi_m) audited the layout of the whole batch (audit_batch); every later round is a subset of it.
  static int step_multi(pfmpe_ctx* const* cs, int S, const FrameArgsT<T>* fas, const unsigned char* const* tables,
                        unsigned char* h, const unsigned char* hdev, unsigned char* d, size_t tbytes) {
    using Desc = StreamDesc<T, SP>;
    pfmpe_ctx* c0 = cs[0];
    std::vector<int> act(S);
    for (int s = 0; s < S; ++s) act[s] = s;
    int iter = 0, nb = 1;
    for (int round = 0;; ++round) {
      const int na = (int)act.size();
      const BatchLayout L = batch_layout<Desc>(na, 0, tbytes);
      Desc* hd = (Desc*)(h + L.doff);
      int64_t total = 0;
      size_t lds_w = 0, lds_f = 0;
      bool all_kept = true;  // every stream has its kept propagated set: k_resample_multi<KEPT = true>
      bool all_owners = true;  // ... and defers its new prior: k_resample_owners_multi
      if (++c0->multi_gen == 0u || c0->multi_gen == ~0u) c0->multi_gen = 1u;  // never 0 / ~0 (status words)
      const uint32_t gen = c0->multi_gen;
      std::vector<Desc> want(na);  // the descriptors as written (the staging check's reference for a report)
      for (int i = 0; i < na; ++i) {
        pfmpe_ctx* c = cs[act[i]];
        const FrameArgsT<T>& fa = fas[act[i]];
        Desc& x = want[i];
        std::memset((void*)&x, 0, sizeof(Desc));
        x.fa = fa;
        x.table = tables[act[i]];
        x.prior = (const SP*)c->d_state[c->prior_idx];
        x.post = (SP*)c->d_state[1 - c->prior_idx];
        x.w0 = (T*)c->d_w[0];
        x.w1 = (T*)c->d_w[1];
        x.part0 = c->d_part[0];
        x.part1 = c->d_part[1];
        x.bscan0 = c->d_bscan[0];
        x.bscan1 = c->d_bscan[1];
        x.gpart0 = c->d_gpart[0];
        x.gpart1 = c->d_gpart[1];
        x.gscan = c->d_gscan;
        x.ctrl = c->d_ctrl;
        x.gcount_w = c->d_counters;
        x.tcount_w = c->d_counters + c->max_grp;
        x.gcount_r = c->d_counters + c->max_grp + 1;
        x.tcount_r = c->d_counters + 2 * c->max_grp + 1;
        // The stored set with deferred resampling (k_resample_multi writes owner indices; the kept buffer becomes the
        // stream's prior at take_step, as in finish()) for every state type; without deferral it pays in batches only
        // for fp16 state (round-3 A/B, DESIGN.md §4.2: 8 x C5 batches 5-8 % faster regenerating).  No choice here
        // changes a result.
        const bool defer = c->defer && c->d_owner[0] && c->d_owner[1] && !(c->diag & kDiagNoDefer);
        const bool kept = c->keep_prop && c->d_prop[0] && (defer || std::is_same<SP, __half>::value);
        x.prop0 = kept ? (SP*)c->d_prop[0] : nullptr;
        x.prop1 = kept ? (SP*)c->d_prop[1] : nullptr;
        all_kept = all_kept && kept;
        c->frame_owner_out = -1;
        if (kept && defer) {
          c->frame_owner_out = c->prior_owner == 0 ? 1 : 0;
          x.fa.owner_out = c->d_owner[c->frame_owner_out];
        } else {
          all_owners = false;
        }
        x.cpart = c->d_cpart;
        x.cgroup = c->d_cgroup;
        x.counts = c->record_counts ? c->d_counts : nullptr;
        x.cand = c->d_cand;
        x.mlpose = c->d_mlpose;
        x.out = c->d_out;
        x.winkey = c->d_winkey;
        c->seq = (c->seq + 1) & 0x3fffffff;
        x.seq = c->seq;
        x.first_blk = (int32_t)total;
        x.gen = gen;
        x.tag = desc_tag((const uint64_t*)&x, (int)(offsetof(Desc, tag) / 8));
        std::memcpy((void*)&hd[i], (const void*)&x, sizeof(Desc));
        if (i == 0 && (c0->diag & kDiagCorruptDesc)) hd[0].fa.key0 ^= 1u;  // test: altered after the tag
        total += fa.nblk;
        lds_w = std::max(lds_w, BlobTable<T>::lds_bytes(fa.tbytes));
        lds_f = std::max(lds_f, BlobTable<T>::bytes(fa.B));
      }
      // The streaming packed pass for the whole batch (k_weigh_pk_multi + the batched group / top hand-off) when
      // every stream's frame is one k_weigh_pk covers; otherwise the one-block pass with its in-launch hand-off
      // (k_propagate_weigh_multi).  Each stream gets a share of the resident workgroups in proportion to its
      // particles (at least one, at most one per four tasks), written into its descriptor before the tag.
      bool pk = false;
      int pk_grid_x = 0, max_ngrp = 0;
      if constexpr (kPkInstance<T, RNG, MAXM, SP>) {
        pk = c0->prune && !(c0->diag & (kDiagNoStream | kDiagNoPk));
        for (int i = 0; i < na && pk; ++i) pk = pk_eligible(fas[act[i]]);
        if (pk) {
          const void* fn = (const void*)k_weigh_pk_multi<SP>;
          auto key = std::make_pair(fn, lds_w);
          auto it = c0->occ.find(key);
          if (it == c0->occ.end()) {
            int per_cu = 0;
            HIPCHK(c0, hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, kBlock, lds_w));
            it = c0->occ.emplace(key, std::max(1, per_cu)).first;
          }
          const int64_t cap = (int64_t)it->second * std::max(1, c0->num_cu);
          for (int i = 0; i < na; ++i) {
            const FrameArgsT<T>& fa = fas[act[i]];
            const int64_t tasks = 2 * (int64_t)fa.nblk;
            const int64_t share = std::max<int64_t>(1, cap * fa.nblk / std::max<int64_t>(1, total));
            const int wg = (int)std::max<int64_t>(1, std::min<int64_t>(share, (tasks + kWaves - 1) / kWaves));
            Desc& x = want[i];
            x.wg = wg;
            x.tag = desc_tag((const uint64_t*)&x, (int)(offsetof(Desc, tag) / 8));
            std::memcpy((void*)&hd[i], (const void*)&x, sizeof(Desc));
            if (i == 0 && (c0->diag & kDiagCorruptDesc)) hd[0].fa.key0 ^= 1u;
            pk_grid_x = std::max(pk_grid_x, wg);
            max_ngrp = std::max(max_ngrp, fa.ngrp);
          }
        }
      }
      const BatchLayout Lt = batch_layout<Desc>(na, total, tbytes);
      uint32_t* dstat = (uint32_t*)(d + Lt.soff);
      // iterations of this round: no launch past the largest remaining cap of the active streams (a launch past
      // a stream's own cap would be a no-op on its ctrl->done, but it also runs with an iteration number the
      // host's small-angle bound did not cover)
      int room = 0;
      for (int i = 0; i < na; ++i) {
        const FrameArgsT<T>& fa = fas[act[i]];
        room = std::max(room, (fa.force_iters > 0 ? fa.force_iters : std::max(1, fa.max_iter)) - iter);
      }
      const int nit = std::max(1, std::min(nb, room));
      // descriptors, host tables (first round) and the block map go to HBM by a staging launch in the same
      // stream (k_stage_multi reads the pinned image once), not by a copy-engine transfer
      const Desc* dd = (const Desc*)(d + Lt.doff);
      const uint16_t* db = (const uint16_t*)(d + Lt.boff);
      // the block map is rewritten only when this batch's layout differs from the one staged last (a steady
      // multi-stream loop stages it once: 2 x C4's 78k entries were most of k_stage_multi's 8 us)
      std::vector<int64_t> sig;
      sig.reserve(2 + 2 * (size_t)na);
      sig.push_back((int64_t)Lt.boff);
      sig.push_back(total);
      for (int i = 0; i < na; ++i) {
        sig.push_back(want[i].first_blk);
        sig.push_back(want[i].fa.nblk);
      }
      const bool map_kept = sig == c0->map_sig;
      c0->map_sig.swap(sig);
      const int64_t t_l0 = now_ns();
      if (round == 0) c0->mt_ns[0] += t_l0 - c0->mt_enter;
      RET(launch_ext(c0, PFMPE_K_AUX, [&] {
        klaunch(c0, k_stage_multi<T, SP>, dim3((unsigned)na), dim3(kBlock), 0, hdev, d, (uint32_t)Lt.doff,
                (uint32_t)(round == 0 ? tbytes : 0), map_kept ? kMapKept : (uint32_t)Lt.boff, dstat, gen);
      }));
      for (int k = 0; k < nit; ++k, ++iter) {
        if constexpr (kPkInstance<T, RNG, MAXM, SP>) {
          if (pk) {
            const uint32_t* cst = dstat;
            RET(launch_ext(c0, PFMPE_K_PROPAGATE, [&] {
              klaunch(c0, k_weigh_pk_multi<SP>, dim3((unsigned)pk_grid_x, (unsigned)na), dim3(kBlock), lds_w, dd, na,
                      cst, gen, iter);
            }));
            // the group / top hand-off: one launch when every stream's groups fit one tile, else group scans +
            // the wide top (group partials staged in LDS) or, beyond its LDS, the one-wave top
            const size_t glds = (size_t)max_ngrp * sizeof(GroupPart);
            const bool wide = glds <= 64 * 1024 && max_ngrp <= 64 * kTopMaxTiles && !(c0->diag & kDiagSerialTop);
            RET(launch_ext(c0, PFMPE_K_AUX, [&] {
              if (max_ngrp <= 64 && !(c0->diag & kDiagSerialTop)) {
                klaunch(c0, k_group_top_multi<T, RNG, SP>, dim3((unsigned)max_ngrp, (unsigned)na), dim3(64), 0, dd, na,
                        cst, gen, iter);
              } else {
                klaunch(c0, k_group_multi<T, SP>, dim3((unsigned)max_ngrp, (unsigned)na), dim3(64), 0, dd, na, cst, gen);
                if (wide)
                  klaunch(c0, k_top_wide_multi<T, RNG, SP>, dim3((unsigned)na), dim3(64 * kTopWaves), glds, dd, na, cst,
                          gen, iter);
                else
                  klaunch(c0, k_top_multi<T, RNG, SP>, dim3((unsigned)na), dim3(64), 0, dd, na, cst, gen, iter);
              }
            }));
            continue;
          }
        }
        RET(launch_ext(c0, PFMPE_K_PROPAGATE, [&] {
          if (c0->prune)
            klaunch(c0, k_propagate_weigh_multi<T, RNG, MAXM, true, SP>, dim3((unsigned)total), dim3(kBlock), lds_w, dd,
                    db, na, (const uint32_t*)dstat, gen, iter);
          else
            klaunch(c0, k_propagate_weigh_multi<T, RNG, MAXM, false, SP>, dim3((unsigned)total), dim3(kBlock), lds_w,
                    dd, db, na, (const uint32_t*)dstat, gen, iter);
        }));
      }
      for (int i = 0; i < na; ++i) {
        cs[act[i]]->last_weigh_pass = pk ? PFMPE_WEIGH_PK : PFMPE_WEIGH_BLOCKS;
        cs[act[i]]->last_resample =
            all_owners && !(c0->diag & kDiagBlockResample) ? PFMPE_RESAMPLE_OWNERS : PFMPE_RESAMPLE_BLOCKS;
      }
      const bool owners = all_owners && !(c0->diag & kDiagBlockResample);
      RET(launch_ext(c0, PFMPE_K_RESAMPLE, [&] {
        if (owners)  // a wave per block (§4.2d), each stream finished by its last block's wave
          klaunch(c0, k_resample_owners_multi<T, RNG, MAXM, SP>, dim3((unsigned)((total + kWaves - 1) / kWaves)),
                  dim3(kBlock), 0, dd, db, na, (const uint32_t*)dstat, gen, (int)total);
        else if (all_kept)
          klaunch(c0, k_resample_multi<T, RNG, MAXM, SP, true>, dim3((unsigned)total), dim3(kBlock), 0, dd, db, na,
                  (const uint32_t*)dstat, gen);
        else
          klaunch(c0, k_resample_multi<T, RNG, MAXM, SP, false>, dim3((unsigned)total), dim3(kBlock), 0, dd, db, na,
                  (const uint32_t*)dstat, gen);
      }));
      if (!owners)
        RET(launch_ext(c0, PFMPE_K_FINAL, [&] {
          klaunch(c0, k_resample_final_multi<T, RNG, MAXM, SP>, dim3((unsigned)na), dim3(kFinalBlock), lds_f, dd,
                  (const uint32_t*)dstat, gen);
        }));
      const int64_t t_l1 = now_ns();
      c0->mt_ns[1] += t_l1 - t_l0;
      std::vector<int> next;
      for (int i = 0; i < na; ++i) {
        pfmpe_ctx* c = cs[act[i]];
        if (wait_frame(c, c0->stream) != PFMPE_OK) {
          const std::string err = c->err;
          for (int k = 0; k < na; ++k) (void)reset_handoffs(cs[act[k]], c0->stream);
          return batch_failure(c0, cs, act, want, d + Lt.doff, dstat, gen, err);
        }
        if (!frame_done(c)) next.push_back(act[i]);
      }
      c0->mt_ns[2] += now_ns() - t_l1;
      if (next.empty()) break;
      for (int s : next) {
        const FrameArgsT<T>& fa = fas[s];
        const int cap = fa.force_iters > 0 ? fa.force_iters : std::max(1, fa.max_iter);
        if (iter >= cap) return fail(c0, PFMPE_E_STATE, "step_multi: PF iteration loop did not terminate");
      }
      act.swap(next);
      nb = round == 0 ? 1 : std::min(nb * 2, 16);
    }
    for (int s = 0; s < S; ++s) {
      cs[s]->last_shape = PFMPE_SHAPE_TWO_LAUNCH;
      last_args<T>(cs[s]) = fas[s];
    }
    return PFMPE_OK;
  }
  static int regen(pfmpe_ctx* c, int kept_iter, const void* prior, double* out) {
    const FrameArgsT<T>& fa = last_args<T>(c);
    return launch_ext(c, PFMPE_K_AUX, [&] {
      klaunch(c, k_regen<T, RNG, SP>, dim3((fa.N + 255) / 256), dim3(256), 0, fa, kept_iter,
                         (const SP*)prior, out);
    });
  }
};

template <typename T>
FrameArgsT<T> build_args(const pfmpe_ctx* c, const pfmpe_frame_in* in);

template <typename T, int RNG, typename SP>
int dispatch_m(pfmpe_ctx* c, const pfmpe_frame_in* in, const unsigned char* table, size_t tbytes, const GridHdr& gh) {
  c->frame_owner_out = -1;  // one-launch frames materialise the new prior (finish() may set it)
  FrameArgsT<T> fa = build_args<T>(c, in);
  fa.tbytes = (int32_t)tbytes;
  fa.grid = grid_args<T>(gh, fa.B, (float)fa.tolq);
  c->last_grid = fa.grid.on;
  for (int q = 0; q < 12; ++q) {  // fp16 state: anchors of the prior and of the new prior (current pose)
    fa.anc_in[q] = (T)c->anchor[c->prior_idx][q];
    fa.anc_out[q] = (T)in->current_pose[q];
  }
  // marker capacity buckets: the per-particle loops are unrolled to MAXM (5: the 5-LED configs C1/C2/C4,
  // 12: C3)
  if (fa.M == kExactM) return Seq<T, RNG, kExactM, SP>::step(c, fa, table);  // the 5-slot bucket is exact (marker_live)
  if (fa.M <= 8) return Seq<T, RNG, 8, SP>::step(c, fa, table);
  if (fa.M <= 12) return Seq<T, RNG, 12, SP>::step(c, fa, table);
  return Seq<T, RNG, 16, SP>::step(c, fa, table);
}

// Host-side bounds audit of a batch (the batched fault at 8 x 10M fp16 streams).  Everything a
// batched kernel indexes is derived here from the descriptors it will read, and checked against what each
// context allocated at create (pfmpe_create: max_blk blocks, max_grp = max_blk groups, ld-element planes,
// a blob bank of bank_off.back() bytes) and against the batch scratch: a stream's blocks, groups, planes,
// table, count partials and candidates all stay inside its own buffers, the block map covers [0, total)
// exactly once, and the scratch holds tables + descriptors + map.  A failing check returns PFMPE_E_STATE
// (a bug, never an input error: check_step validated the inputs) instead of launching.
template <typename T, typename SP>
int audit_batch(pfmpe_ctx* const* cs, int S, const FrameArgsT<T>* fas, const pfmpe_frame_in* in,
                const std::vector<size_t>& toff, size_t tbytes, int64_t total, size_t cap) {
  pfmpe_ctx* c0 = cs[0];
  auto bad = [&](int s, const char* what) {
    return fail(c0, PFMPE_E_STATE, "step_multi: batch audit failed for stream " + std::to_string(s) + ": " + what);
  };
  int64_t first = 0;
  for (int s = 0; s < S; ++s) {
    const pfmpe_ctx* c = cs[s];
    const FrameArgsT<T>& fa = fas[s];
    if (fa.N != c->N || fa.N < 1 || fa.N > c->max_particles || (int64_t)fa.N > c->ld) return bad(s, "particle count");
    if (fa.nblk != (fa.N + kBlock - 1) / kBlock || fa.nblk > c->max_blk) return bad(s, "block count");
    if (fa.gsz < 1 || fa.gsz > kGroup || fa.ngrp != (fa.nblk + fa.gsz - 1) / fa.gsz || fa.ngrp > c->max_grp)
      return bad(s, "group count");
    if (fa.ld != c->ld) return bad(s, "plane stride");
    if (c->state_dtype != PFMPE_STATE_F64 && (int64_t)kPlanes * c->ld * (int64_t)c->es >= ((int64_t)1 << 32))
      return bad(s, "plane buffer resource range");
    if (fa.M != c->M || fa.M < 1 || fa.M > c->max_markers || fa.B < 0 || fa.B > c->max_blobs) return bad(s, "M / B");
    if (c->keep_prop && (!c->d_prop[0] || !c->d_prop[1])) return bad(s, "kept propagated set not allocated");
    if (c->record_counts && !c->d_counts) return bad(s, "count buffer not allocated");
    if (in[s].bank_frame >= 0) {
      const size_t f = (size_t)in[s].bank_frame;
      if (!c->d_bank || f >= c->bank_B.size() || c->bank_B[f] != fa.B ||
          c->bank_off[f] + (size_t)fa.tbytes != c->bank_off[f + 1] || fa.tbytes < (int)BlobTable<T>::bytes(fa.B))
        return bad(s, "bank table");
    } else if (toff[s] + (size_t)fa.tbytes > tbytes || fa.tbytes < (int)BlobTable<T>::bytes(fa.B)) {
      return bad(s, "host table");
    }
    first += fa.nblk;
  }
  if (first != total || total < 1 || total > kMultiMaxBlocks) return bad(0, "block total");
  if (batch_layout<StreamDesc<T, SP>>(S, total, tbytes).need > cap) return bad(0, "batch scratch");
  return PFMPE_OK;
}

// pfmpe_step_multi for S validated contexts of one (state type, RNG): frame arguments and blob tables
// (host-supplied tables staged into the batch scratch of cs[0]), the bounds audit, the order after each
// member's latest work on other streams, then Seq::step_multi on the marker bucket of the largest M, then the
// fence every member's next work on its own stream is ordered after.
template <typename T, int RNG, typename SP>
int multi_m(pfmpe_ctx* const* cs, int S, const pfmpe_frame_in* in) {
  using Desc = StreamDesc<T, SP>;
  pfmpe_ctx* c0 = cs[0];
  std::vector<FrameArgsT<T>> fas(S);
  std::vector<size_t> toff(S, 0);
  std::vector<std::vector<unsigned char>> hosttab(S);
  size_t tbytes = 0;
  int64_t total = 0;
  int maxM = 1;
  bool all5 = true;  // every stream has exactly kExactM markers: the exact 5-slot bucket serves the batch
  for (int s = 0; s < S; ++s) {
    pfmpe_ctx* c = cs[s];
    c->frame_owner_out = -1;  // step_multi sets it for the streams it defers
    all5 = all5 && c->M == kExactM;
    fas[s] = build_args<T>(c, &in[s]);
    for (int q = 0; q < 12; ++q) {
      fas[s].anc_in[q] = (T)c->anchor[c->prior_idx][q];
      fas[s].anc_out[q] = (T)in[s].current_pose[q];
    }
    if (in[s].bank_frame < 0) {  // host blobs: the table is built now (its size depends on the blobs)
      hosttab[s].resize(BlobTable<T>::max_bytes());
      fas[s].tbytes = (int32_t)build_blob_table_host<T>(in[s].blobs, in[s].B, (double)fas[s].tolq, hosttab[s].data());
      fas[s].grid = grid_args<T>(*(const GridHdr*)(hosttab[s].data() + BlobTable<T>::off_grid(in[s].B)), in[s].B,
                                 (float)fas[s].tolq);
      toff[s] = tbytes;
      tbytes += ((size_t)fas[s].tbytes + 255) / 256 * 256;
    } else {
      const size_t f = (size_t)in[s].bank_frame;
      fas[s].tbytes = (int32_t)(c->bank_off[f + 1] - c->bank_off[f]);
      fas[s].grid = grid_args<T>(c->bank_grid[f], in[s].B, (float)fas[s].tolq);
    }
    c->last_grid = fas[s].grid.on;
    total += fas[s].nblk;
    maxM = std::max(maxM, c->M);
  }
  const int64_t max_blocks = std::min(kMultiMaxBlocks, c0->multi_max_blocks);
  if (total > max_blocks)
    return fail(c0, PFMPE_E_CAP, "step_multi: " + std::to_string(total) + " blocks in one batch (at most " +
                                     std::to_string(max_blocks) + " = " + std::to_string(max_blocks * kBlock) +
                                     " particles, PFMPE_OPT_MULTI_MAX_BLOCKS)");
  const size_t need = batch_layout<Desc>(S, total, tbytes).need;
  if (need > c0->multi_cap) {
    HIPCHK(c0, hipStreamSynchronize(c0->stream));
    if (c0->d_multi) HIPCHK(c0, hipFree(c0->d_multi));
    if (c0->h_multi) HIPCHK(c0, hipHostFree(c0->h_multi));
    c0->d_multi = nullptr;
    c0->h_multi = nullptr;
    c0->hd_multi = nullptr;
    c0->multi_cap = 0;
    c0->map_sig.clear();  // a new scratch holds no map
    const size_t cap = std::max(need * 2, (size_t)1 << 16);
    HIPCHK(c0, hipMalloc((void**)&c0->d_multi, cap));
    // read by k_stage_multi over PCIe: mapped, coherent (the host rewrites it between batches)
    HIPCHK(c0, hipHostMalloc((void**)&c0->h_multi, cap, hipHostMallocMapped | hipHostMallocCoherent));
    HIPCHK(c0, hipHostGetDevicePointer((void**)&c0->hd_multi, c0->h_multi, 0));
    c0->multi_cap = cap;
  }
  for (int s = 0; s < S; ++s) RET(ensure_prop(cs[s]));
  RET((audit_batch<T, SP>(cs, S, fas.data(), in, toff, tbytes, total, c0->multi_cap)));
  if (!c0->lead_fence) {  // created before any member's ordering state changes (no early return after)
    auto f = std::make_shared<BatchFence>();
    HIPCHK(c0, hipEventCreateWithFlags(&f->ev, hipEventDisableTiming));
    f->stream = c0->stream;
    c0->lead_fence = f;
  } else {
    // a context of the leader's previous batch that is not in this one: its fence ends before this batch (members of
    // both batches need no fence: their work stays on this stream; a steady loop of batches records nothing)
    long held = 0;
    for (int s = 0; s < S; ++s) held += cs[s]->last_fence.get() == c0->lead_fence.get();
    if (c0->lead_fence.use_count() - 1 > held) RET(seal_lead_fence(c0));
  }
  // every member's work so far is ordered before the batch (its own stream, or an earlier batch led elsewhere).
  // order_after clears a member's ordering state; if a later member's ordering fails, the earlier ones get their
  // state back (their pending work is still unordered with their own streams)
  {
    std::vector<std::pair<hipStream_t, std::shared_ptr<BatchFence>>> saved(S);
    for (int s = 0; s < S; ++s) saved[s] = {cs[s]->last_stream, cs[s]->last_fence};
    for (int s = 0; s < S; ++s)
      if (const int r = order_after(cs[s], c0->stream, c0)) {
        for (int e = 0; e < S; ++e) {
          cs[e]->last_stream = saved[e].first;
          cs[e]->last_fence = saved[e].second;
        }
        return r;
      }
  }
  std::vector<const unsigned char*> tables(S);
  for (int s = 0; s < S; ++s) {
    pfmpe_ctx* c = cs[s];
    if (in[s].bank_frame >= 0) {
      tables[s] = c->d_bank + c->bank_off[in[s].bank_frame];
    } else {
      std::memcpy(c0->h_multi + toff[s], hosttab[s].data(), (size_t)fas[s].tbytes);
      tables[s] = c0->d_multi + toff[s];
    }
  }
  int rc;
  if (all5)
    rc = Seq<T, RNG, kExactM, SP>::step_multi(cs, S, fas.data(), tables.data(), c0->h_multi, c0->hd_multi, c0->d_multi, tbytes);
  else if (maxM <= 8)
    rc = Seq<T, RNG, 8, SP>::step_multi(cs, S, fas.data(), tables.data(), c0->h_multi, c0->hd_multi, c0->d_multi, tbytes);
  else if (maxM <= 12)
    rc = Seq<T, RNG, 12, SP>::step_multi(cs, S, fas.data(), tables.data(), c0->h_multi, c0->hd_multi, c0->d_multi, tbytes);
  else
    rc = Seq<T, RNG, 16, SP>::step_multi(cs, S, fas.data(), tables.data(), c0->h_multi, c0->hd_multi, c0->d_multi, tbytes);
  // the batch's kernels may still be retiring when the records are in (or when a step failed part-way): each
  // member's next work on its own stream is ordered after the leader's stream through the fence, recorded when
  // that work comes (the leader's own stream is the batch stream).  Set whatever step_multi returned.
  for (int s = 0; s < S; ++s) {
    cs[s]->last_stream = c0->stream;
    cs[s]->last_fence = s == 0 ? nullptr : c0->lead_fence;
  }
  c0->lead_fence->recorded = false;  // this batch is not in the event yet
  return rc;
}

template <typename T, int RNG, typename SP>
int regen_m(pfmpe_ctx* c, int kept_iter, const void* prior, double* out) {
  return Seq<T, RNG, 8, SP>::regen(c, kept_iter, prior, out);
}

inline bool is_identity12(const double* p) {
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
    // hi - lo in T (the value the device formed before: bit-identical draws), times 2^-21 (exact)
    fa.rgs[q] = (T)(fa.hi[q] - fa.lo[q]) * (T)0x1p-21;
  }
  fa.growth = p.growth;
  {  // fp32: every angle draw of the frame within kSmallAngle -> the short sincos polynomials (wave-uniform)
    const int cap = in->force_iters > 0 ? in->force_iters : std::max(1, p.max_iter);
    const double gmax = 1.0 + p.growth * (double)((cap - 1) / 10);
    double amax = 0.0;
    for (int q = 0; q < 3; ++q) amax = std::max(amax, std::max(std::abs(fa.dlo[q]), std::abs(fa.dhi[q])));
    fa.small_angles = (sizeof(T) == 4 && amax * std::abs(gmax) <= 0.999 * (double)kSmallAngle) ? 1 : 0;
  }
  fa.k_upper = (fa.K[3] == (T)0 && fa.K[6] == (T)0 && fa.K[7] == (T)0 && fa.K[8] == (T)1) ? 1 : 0;
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
  // groups of 64 whenever the frame can run as one flat launch (k_frame2 reduces one group per wave), so
  // the one-launch and two-launch shapes keep the same summation association; ~sqrt(nblk) beyond
  fa.gsz = (fa.nblk <= kFlatMaxGroups * kGroup && !(c->diag & kDiagSqrtGroups))
               ? kGroup
               : std::min(kGroup, std::max(1, (int)std::ceil(std::sqrt((double)std::max(1, fa.nblk)))));
  fa.ngrp = (fa.nblk + fa.gsz - 1) / fa.gsz;
  // (c->max_grp = max_blk >= ngrp for every N <= max_particles)
  fa.diag = c->diag;
  fa.wait_ticks = (uint32_t)std::min<int64_t>(c->wait_bound_us * 100, 0xffffffffll);  // s_memrealtime: 100 MHz
  fa.ld = c->ld;
  fa.owner = prior_owner_ptr(c);
  fa.owner_out = nullptr;
  return fa;
}


#define PFMPE_DECLARE_INSTANCE(T, RNG, SP, EXT)                                                           \
  EXT template int dispatch_m<T, RNG, SP>(pfmpe_ctx*, const pfmpe_frame_in*, const unsigned char*, size_t, const GridHdr&);        \
  EXT template int regen_m<T, RNG, SP>(pfmpe_ctx*, int, const void*, double*);                            \
  EXT template int multi_m<T, RNG, SP>(pfmpe_ctx* const*, int, const pfmpe_frame_in*);

}  // namespace pfmpe_impl
