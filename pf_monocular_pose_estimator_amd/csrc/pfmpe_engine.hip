// pfmpe_engine.hip — host side of the MI355X PF engine: context, buffers, C-ABI (include/pfmpe.h).
//
// Replaces the PF block of PoseEstimator::estimateBodyPose (pf_mpe_lib/src/pose_estimator.cpp:475-733).
// The launch sequences live in pfmpe_ctx.hpp (Seq) and are instantiated per (state type, RNG) in the
// pfmpe_k_*.hip translation units.
#include "pfmpe_ctx.hpp"

using namespace pfmpe;
using namespace pfmpe_impl;

namespace pfmpe_impl {
PFMPE_DECLARE_INSTANCE(float, kRngReference, float, extern)
PFMPE_DECLARE_INSTANCE(float, kRngPhilox, float, extern)
PFMPE_DECLARE_INSTANCE(double, kRngReference, double, extern)
PFMPE_DECLARE_INSTANCE(double, kRngPhilox, double, extern)
PFMPE_DECLARE_INSTANCE(float, kRngReference, __half, extern)
PFMPE_DECLARE_INSTANCE(float, kRngPhilox, __half, extern)
}  // namespace pfmpe_impl

namespace {
using namespace pfmpe_impl;

int dispatch_step(pfmpe_ctx* c, const pfmpe_frame_in* in, const unsigned char* table, size_t tbytes,
                  const GridHdr& gh) {
  const bool ref = c->params.rng_mode == PFMPE_RNG_REFERENCE;
  switch (c->state_dtype) {
    case PFMPE_STATE_F64:
      return ref ? dispatch_m<double, kRngReference, double>(c, in, table, tbytes, gh)
                 : dispatch_m<double, kRngPhilox, double>(c, in, table, tbytes, gh);
    case PFMPE_STATE_F16:
      return ref ? dispatch_m<float, kRngReference, __half>(c, in, table, tbytes, gh)
                 : dispatch_m<float, kRngPhilox, __half>(c, in, table, tbytes, gh);
    default:
      return ref ? dispatch_m<float, kRngReference, float>(c, in, table, tbytes, gh)
                 : dispatch_m<float, kRngPhilox, float>(c, in, table, tbytes, gh);
  }
}

int dispatch_regen(pfmpe_ctx* c, int kept_iter, const void* prior, double* out) {
  const bool ref = c->params.rng_mode == PFMPE_RNG_REFERENCE;
  switch (c->state_dtype) {
    case PFMPE_STATE_F64:
      return ref ? regen_m<double, kRngReference, double>(c, kept_iter, prior, out)
                 : regen_m<double, kRngPhilox, double>(c, kept_iter, prior, out);
    case PFMPE_STATE_F16:
      return ref ? regen_m<float, kRngReference, __half>(c, kept_iter, prior, out)
                 : regen_m<float, kRngPhilox, __half>(c, kept_iter, prior, out);
    default:
      return ref ? regen_m<float, kRngReference, float>(c, kept_iter, prior, out)
                 : regen_m<float, kRngPhilox, float>(c, kept_iter, prior, out);
  }
}

// state import / export for the three storage types (anchor: fp16 state only)
template <typename T, typename SP>
void launch_import(pfmpe_ctx* c, int N, const double* anchor) {
  Pose12<T> a;
  for (int q = 0; q < 12; ++q) a.v[q] = (T)anchor[q];
  hipLaunchKernelGGL((k_import<T, SP>), dim3((N + 255) / 256), dim3(256), 0, c->stream, c->d_xfer,
                     (SP*)c->d_state[c->prior_idx], N, c->ld, a);
}
template <typename T, typename SP>
void launch_export(pfmpe_ctx* c, int N, const double* anchor) {
  Pose12<T> a;
  for (int q = 0; q < 12; ++q) a.v[q] = (T)anchor[q];
  hipLaunchKernelGGL((k_export<T, SP>), dim3((N + 255) / 256), dim3(256), 0, c->stream,
                     (const SP*)c->d_state[c->prior_idx], c->d_xfer, N, c->ld, a, prior_owner_ptr(c));
}


// byte offset of a table's GridHdr
size_t grid_off(const pfmpe_ctx* c, int B) {
  return c->state_dtype == PFMPE_STATE_F64 ? BlobTable<double>::off_grid(B) : BlobTable<float>::off_grid(B);
}
// largest blob table of this context's type (base part at kMaxBlobs + the largest grid)
size_t table_max_bytes(const pfmpe_ctx* c) {
  return c->state_dtype == PFMPE_STATE_F64 ? BlobTable<double>::max_bytes() : BlobTable<float>::max_bytes();
}
// the frame's blob table for the context's current parameters (pruning half-window as build_args computes
// it); returns its size
size_t build_table(const pfmpe_ctx* c, const double* blobs, int B, unsigned char* dst) {
  const double tolq = c->state_dtype == PFMPE_STATE_F64 ? (c->params.tol_pf * (1.0 + 1e-3) + 1e-3)
                                                        : (double)(float)(c->params.tol_pf * (1.0 + 1e-3) + 1e-3);
  if (c->state_dtype == PFMPE_STATE_F64) return build_blob_table_host<double>(blobs, B, tolq, dst);
  return build_blob_table_host<float>(blobs, B, tolq, dst);
}


void free_all(pfmpe_ctx* c) {
  void* dev[] = {c->d_state[0], c->d_state[1], c->d_w[0], c->d_w[1], c->d_prop[0], c->d_prop[1], c->d_part[0], c->d_part[1],
                 c->d_bscan[0], c->d_bscan[1], c->d_gpart[0], c->d_gpart[1], c->d_gscan, c->d_cpart, c->d_winkey,
                 c->d_cgroup, c->d_counters, c->d_ctrl, c->d_gen, c->d_cand, c->d_mlpose, c->d_flat, c->d_roi, c->d_gran, c->d_init, c->d_det, c->d_img, c->d_table, c->d_bank, c->d_xfer, c->d_counts,
                 c->d_stamps, c->d_owner[0], c->d_owner[1]};
  for (void* p : dev)
    if (p) (void)hipFree(p);
  if (c->h_rec) (void)hipHostFree(c->h_rec);
  delete c->h_out;
  c->h_out = nullptr;
  if (c->h_table) (void)hipHostFree(c->h_table);
  if (c->h_det) (void)hipHostFree(c->h_det);
  for (auto& e : c->ev_pool) {
    (void)hipEventDestroy(e.a);
    (void)hipEventDestroy(e.b);
  }
  if (c->d_multi) (void)hipFree(c->d_multi);
  if (c->h_multi) (void)hipHostFree(c->h_multi);
  if (c->stream) (void)hipStreamDestroy(c->stream);
}

// pfmpe_step's argument and state checks (also per stream of pfmpe_step_multi)
int check_step(pfmpe_ctx* c, const pfmpe_frame_in* in, const pfmpe_frame_out* out) {
  if (!c) return PFMPE_E_ARG;
  if (!in || !out) return fail(c, PFMPE_E_ARG, "step: null in/out");
  if (!c->has_model || !c->has_prior) return fail(c, PFMPE_E_STATE, "step: set_model and set_prior first");
  if (in->B < 0) return fail(c, PFMPE_E_ARG, "step: B < 0");
  if (in->force_iters < 0 || in->force_iters > kMaxIter) return fail(c, PFMPE_E_ARG, "step: force_iters out of range");
  if (in->B > c->max_blobs) return fail(c, PFMPE_E_CAP, "step: B exceeds max_blobs");
  if (in->it_since_init >= 2 && !(in->dt != 0.0))
    return fail(c, PFMPE_E_ARG, "step: dt must be non-zero in steady state");
  if (in->bank_frame >= 0) {
    if (!c->d_bank || in->bank_frame >= (int)c->bank_B.size())
      return fail(c, PFMPE_E_ARG, "step: bank_frame out of range");
    if (c->bank_B[in->bank_frame] != in->B) return fail(c, PFMPE_E_ARG, "step: B does not match the staged bank frame");
  } else if (in->B > 0 && !in->blobs) {
    return fail(c, PFMPE_E_ARG, "step: null blobs");
  }
  return PFMPE_OK;
}

// the frame record into pfmpe_frame_out, and the context's state after the frame (PE:681, 727)
void take_step(pfmpe_ctx* c, const pfmpe_frame_in* in, pfmpe_frame_out* out) {
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
  if (o.resampled) {  // newPoseEstimation = resampled set (PE:681, 727), anchored at this frame's current pose
    if (c->frame_owner_out >= 0 && c->d_owner[c->frame_owner_out] && o.kept_slot >= 0 && o.kept_slot < 2 &&
        c->d_prop[o.kept_slot]) {
      // deferred resampling: the kept buffer is the new prior's storage (read through the owner indices k_resample
      // wrote); the unused post buffer becomes that weight slot's kept buffer for the next frame
      std::swap(c->d_prop[o.kept_slot], c->d_state[1 - c->prior_idx]);
      c->prior_owner = c->frame_owner_out;
    } else {
      c->prior_owner = -1;
    }
    c->frame_owner_out = -1;
    c->prior_idx = 1 - c->prior_idx;
    std::memcpy(c->anchor[c->prior_idx], in->current_pose, 12 * sizeof(double));
  }
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
      max_blobs > kMaxBlobs ||
      (state_dtype != PFMPE_STATE_F32 && state_dtype != PFMPE_STATE_F64 && state_dtype != PFMPE_STATE_F16))
    return PFMPE_E_ARG;
  pfmpe_ctx* c = new pfmpe_ctx();
  c->device = hip_device;
  c->max_particles = max_particles;
  c->max_markers = max_markers;
  c->max_blobs = max_blobs;
  c->state_dtype = state_dtype;
  c->es = state_dtype == PFMPE_STATE_F64 ? 8 : (state_dtype == PFMPE_STATE_F16 ? 2 : 4);
  c->ws = state_dtype == PFMPE_STATE_F64 ? 8 : 4;
  c->ld = ((int64_t)max_particles + 63) / 64 * 64;

  c->max_blk = (max_particles + kBlock - 1) / kBlock;
  // fp32 / fp16 planes are addressed through one 32-bit buffer resource per state buffer
  // (pf_kernels.hpp BufPlanes): 12 planes must stay below 4 GiB (89M fp32 / 178M fp16 particles)
  if (state_dtype != PFMPE_STATE_F64 && (int64_t)kPlanes * c->ld * (int64_t)c->es >= ((int64_t)1 << 32)) {
    delete c;
    return PFMPE_E_CAP;
  }
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
  c->max_grp = c->max_blk;  // groups hold ~sqrt(blocks) blocks (build_args): size group buffers per block
  for (int i = 0; i < 2; ++i) {
    ok &= hipMalloc(&c->d_state[i], state_bytes) == hipSuccess;
    ok &= hipMalloc(&c->d_w[i], (size_t)c->max_blk * kBlock * c->ws) == hipSuccess;  // whole blocks: k_resample_owners
    // kWaves entries per block: the streaming weighing pass stores wave partials (k_group combines them)
    ok &= hipMalloc((void**)&c->d_part[i], (size_t)c->max_blk * kWaves * sizeof(BlockPart)) == hipSuccess;
    ok &= hipMalloc((void**)&c->d_bscan[i], (size_t)c->max_blk * sizeof(BlockScan)) == hipSuccess;
    ok &= hipMalloc((void**)&c->d_gpart[i], (size_t)c->max_grp * sizeof(GroupPart)) == hipSuccess;
  }
  ok &= hipMalloc((void**)&c->d_gscan, (size_t)c->max_grp * sizeof(GroupScan)) == hipSuccess;
  ok &= hipMalloc((void**)&c->d_cpart, (size_t)(c->max_blk + 1) * sizeof(CountPart)) == hipSuccess;  // +1: 16-B reads
  ok &= hipMalloc((void**)&c->d_cgroup, (size_t)c->max_grp * sizeof(CountPart)) == hipSuccess;
  ok &= hipMalloc((void**)&c->d_winkey, kWinBytes) == hipSuccess;
  ok &= hipMalloc((void**)&c->d_counters, counters_bytes(c)) == hipSuccess;
  ok &= hipMalloc((void**)&c->d_ctrl, sizeof(Ctrl)) == hipSuccess;
  ok &= hipMalloc((void**)&c->d_gen, sizeof(uint32_t)) == hipSuccess;
  ok &= hipMalloc((void**)&c->d_cand, (size_t)c->max_blk * sizeof(Cand)) == hipSuccess;
  ok &= hipMalloc((void**)&c->d_mlpose, 12 * sizeof(double)) == hipSuccess;
  ok &= hipMalloc((void**)&c->d_flat, kFlatWords * sizeof(uint32_t)) == hipSuccess;
  ok &= hipMalloc((void**)&c->d_gran, kGranBytes) == hipSuccess;
  {
    int coop = 0;
    ok = ok && hipDeviceGetAttribute(&c->num_cu, hipDeviceAttributeMultiprocessorCount, c->device) == hipSuccess;
    ok = ok && hipDeviceGetAttribute(&coop, hipDeviceAttributeCooperativeLaunch, c->device) == hipSuccess;
    c->coop = coop != 0;
  }
  ok &= hipHostMalloc((void**)&c->h_rec, sizeof(RecOut), hipHostMallocMapped | hipHostMallocCoherent) == hipSuccess;
  ok = ok && hipHostGetDevicePointer((void**)&c->d_out, c->h_rec, 0) == hipSuccess;
  if (ok) {
    memset(c->h_rec, 0, sizeof(RecOut));
    c->h_out = new OutDev();
  }
  ok &= hipMalloc((void**)&c->d_table, table_max_bytes(c)) == hipSuccess;
  ok &= hipHostMalloc((void**)&c->h_table, table_max_bytes(c), hipHostMallocDefault) == hipSuccess;
  if (!ok) return bad(PFMPE_E_HIP);
  // Zeroed in the context's own stream and waited for: the stream is non-blocking, so a null-stream
  // hipMemset could still be in flight when the first frame's kernels read these words (freed memory of an
  // earlier context: a stale control record, counters or candidate tags).
  ok = ok && hipMemsetAsync(c->d_gen, 0, sizeof(uint32_t), c->stream) == hipSuccess;
  ok = ok && hipMemsetAsync(c->d_ctrl, 0, sizeof(Ctrl), c->stream) == hipSuccess;
  ok = ok && hipMemsetAsync(c->d_cand, 0, (size_t)c->max_blk * sizeof(Cand), c->stream) == hipSuccess;
  ok = ok && hipMemsetAsync(c->d_counters, 0, counters_bytes(c), c->stream) == hipSuccess;
  ok = ok && hipMemsetAsync(c->d_flat, 0, kFlatWords * sizeof(uint32_t), c->stream) == hipSuccess;
  ok = ok && hipMemsetAsync(c->d_gran, 0, kGranBytes, c->stream) == hipSuccess;  // no stale word holds a live tag
  ok = ok && hipMemsetAsync(c->d_winkey, 0, kWinBytes, c->stream) == hipSuccess;
  ok = ok && hipMemsetAsync(c->d_state[0], 0, state_bytes, c->stream) == hipSuccess;
  ok = ok && hipMemsetAsync(c->d_state[1], 0, state_bytes, c->stream) == hipSuccess;
  ok = ok && hipStreamSynchronize(c->stream) == hipSuccess;
  if (!ok) return bad(PFMPE_E_HIP);
  *out = c;
  return PFMPE_OK;
}

void pfmpe_destroy(pfmpe_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  if (c->last_fence && c->last_fence->stream) {  // a batch led by another context: its stream up to its end
    if (c->last_fence->recorded || hipEventRecord(c->last_fence->ev, c->last_fence->stream) == hipSuccess)
      (void)hipEventSynchronize(c->last_fence->ev);
    else
      (void)hipStreamSynchronize(c->last_fence->stream);
  }
  c->last_fence.reset();
  if (c->lead_fence) c->lead_fence->stream = nullptr;  // drained above; members find nothing pending
  c->lead_fence.reset();
  if (c->own_ev) (void)hipEventDestroy(c->own_ev);
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

static int build_bank(pfmpe_ctx* c);

int pfmpe_set_params(pfmpe_ctx* c, const pfmpe_params* p) {
  if (!c || !p) return PFMPE_E_ARG;
  if (!(p->tol > 0) || !(p->tol_pf >= 0) || p->max_iter < 1 || p->max_iter > kMaxIter || p->exit_cap < 0 ||
      p->accept_cap < 0 ||
      (p->rng_mode != PFMPE_RNG_REFERENCE && p->rng_mode != PFMPE_RNG_PHILOX))
    return fail(c, PFMPE_E_ARG, "set_params: invalid parameter");
  const bool retable = c->d_bank && p->tol_pf != c->bank_tol_pf;
  const pfmpe_params prev = c->params;
  c->params = *p;
  if (retable) {  // the staged bank's grids were built for another tol_PF
    int r = set_device(c);
    if (r == PFMPE_OK) r = build_bank(c);  // builds the new bank aside; the old one stays until it succeeds
    if (r != PFMPE_OK) c->params = prev;   // all or nothing: the previous parameters and bank stay in force
    return r;
  }
  return PFMPE_OK;
}

int pfmpe_set_option(pfmpe_ctx* c, int option, int64_t value) {
  if (!c) return PFMPE_E_ARG;
  switch (option) {
    case PFMPE_OPT_RECORD_COUNTS:
      c->record_counts = value != 0;
      if (c->record_counts && !c->d_counts) {
        RET(set_device(c));
        HIPCHK(c, hipMalloc((void**)&c->d_counts, (size_t)c->max_blk * kBlock * sizeof(uint32_t)));  // whole blocks
      }
      return PFMPE_OK;
    case PFMPE_OPT_FUSED:
      if (value < 0 || value > 2) return fail(c, PFMPE_E_ARG, "set_option: FUSED is 0, 1 or 2");
      c->fused = c->fused_user = (int)value;
      c->clean_since_fallback = 0;
      return PFMPE_OK;
    case PFMPE_OPT_WAIT_BOUND_US:
      if (value < 1 || value > 40000000) return fail(c, PFMPE_E_ARG, "set_option: WAIT_BOUND_US is 1 .. 4e7");
      c->wait_bound_us = value;
      return PFMPE_OK;
    case PFMPE_OPT_FUSED_REARM:
      if (value < 0) return fail(c, PFMPE_E_ARG, "set_option: FUSED_REARM >= 0");
      c->fused_rearm = value;
      return PFMPE_OK;
    case PFMPE_OPT_PRUNE:
      c->prune = value != 0;
      return PFMPE_OK;
    case PFMPE_OPT_KEEP_PROPAGATED:
      c->keep_prop = value != 0;
      return PFMPE_OK;
    case PFMPE_OPT_DEFER_RESAMPLE:
      c->defer = value != 0;
      return PFMPE_OK;
    case PFMPE_OPT_MULTI_MAX_BLOCKS:
      if (value < 1 || value > kMultiMaxBlocks) return fail(c, PFMPE_E_ARG, "set_option: MULTI_MAX_BLOCKS is 1 .. 160000");
      c->multi_max_blocks = value;
      return PFMPE_OK;
    case PFMPE_OPT_TIMING:
      if (value < 0 || value > (1 << 20)) return fail(c, PFMPE_E_ARG, "set_option: timing period out of range");
      c->timing = (int)value;
      c->timing_frame = 0;
      // the brackets' events are created now, not by the first timed frames: hipEventCreate inside a timed frame
      // had added its cost to every bracket of a short run (the pool starts empty)
      if (value > 0 && c->ev_pool.size() < kEventPrealloc) {
        RET(set_device(c));
        while (c->ev_pool.size() < kEventPrealloc) {
          EventPair p{};
          HIPCHK(c, hipEventCreate(&p.a));
          HIPCHK(c, hipEventCreate(&p.b));
          c->ev_pool.push_back(p);
        }
      }
      return PFMPE_OK;
    case 99:  // undocumented: diagnostic kernel switches for timing experiments
      c->diag = (int)value;
      if ((c->diag & kDiagStamps) && !c->d_stamps) {
        RET(set_device(c));
        HIPCHK(c, hipMalloc((void**)&c->d_stamps, (1 + (size_t)c->max_blk) * kStamps * sizeof(uint64_t)));
        HIPCHK(c, hipMemsetAsync(c->d_stamps, 0, (1 + (size_t)c->max_blk) * kStamps * sizeof(uint64_t), c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
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
  // fp16 state: the set's anchor is its first particle (deltas of a concentrated set stay small)
  std::memcpy(c->anchor[c->prior_idx], poses, 12 * sizeof(double));
  c->prior_owner = -1;  // stored in particle order
  if (c->state_dtype == PFMPE_STATE_F64)
    launch_import<double, double>(c, N, c->anchor[c->prior_idx]);
  else if (c->state_dtype == PFMPE_STATE_F16)
    launch_import<float, __half>(c, N, c->anchor[c->prior_idx]);
  else
    launch_import<float, float>(c, N, c->anchor[c->prior_idx]);
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

// (Re)builds the device bank from c->bank_blobs / bank_offsets with the parameters current now.  The table of a
// frame carries a grid whose window is tol_PF's: set_params rebuilds the bank when tol_PF changes, so a bank
// staged before set_params (or a later change) never leaves the frames on the slower x-bucket path
// (ADVICE r03).
// The new bank is built beside the old one and swapped in only once it is on the device, so a failure (an
// allocation or copy error) leaves the previous bank, its tables and its tol_PF in force.
static int build_bank(pfmpe_ctx* c) {
  const int nframes = (int)c->bank_offsets.size() - 1;
  std::vector<size_t> off(nframes + 1, 0);
  std::vector<int32_t> nb(nframes, 0);
  std::vector<GridHdr> grid(nframes, GridHdr{});
  std::vector<unsigned char> host, one(table_max_bytes(c));
  for (int f = 0; f < nframes; ++f) {
    nb[f] = c->bank_offsets[f + 1] - c->bank_offsets[f];
    const size_t n = build_table(c, c->bank_blobs.data() + 2 * (size_t)c->bank_offsets[f], nb[f], one.data());
    host.insert(host.end(), one.begin(), one.begin() + n);
    off[f + 1] = off[f] + n;
    grid[f] = *(const GridHdr*)(one.data() + grid_off(c, nb[f]));
  }
  unsigned char* d = nullptr;
  HIPCHK(c, hipMalloc((void**)&d, host.size()));
  hipError_t e = hipMemcpyAsync(d, host.data(), host.size(), hipMemcpyHostToDevice, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);  // `host` goes out of scope; frames read in this stream
  if (e != hipSuccess) {
    (void)hipFree(d);
    return fail(c, PFMPE_E_HIP, std::string("build_bank: ") + hipGetErrorString(e));
  }
  if (c->d_bank) (void)hipFree(c->d_bank);  // the stream is idle (synchronised above)
  c->d_bank = d;
  c->bank_off.swap(off);
  c->bank_B.swap(nb);
  c->bank_grid.swap(grid);
  c->bank_tol_pf = c->params.tol_pf;
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
  c->bank_offsets.assign(offsets, offsets + nframes + 1);
  c->bank_blobs.assign(blobs + 2 * (size_t)offsets[0], blobs + 2 * (size_t)offsets[nframes]);
  for (auto& o : c->bank_offsets) o -= offsets[0];
  return build_bank(c);
}

int pfmpe_step(pfmpe_ctx* c, const pfmpe_frame_in* in, pfmpe_frame_out* out) {
  RET(check_step(c, in, out));
  RET(set_device(c));
  const unsigned char* table = c->d_table;
  const int B = in->B;
  size_t tbytes = 0;
  GridHdr gh{};
  if (in->bank_frame >= 0) {
    table = c->d_bank + c->bank_off[in->bank_frame];
    tbytes = c->bank_off[in->bank_frame + 1] - c->bank_off[in->bank_frame];
    gh = c->bank_grid[in->bank_frame];
  } else {
    // the x-bucketed table is built here, O(B), and travels in the same copy the blobs would
    tbytes = build_table(c, in->blobs, B, c->h_table);
    gh = *(const GridHdr*)(c->h_table + grid_off(c, B));
    HIPCHK(c, hipMemcpyAsync(c->d_table, c->h_table, tbytes, hipMemcpyHostToDevice, c->stream));
  }
  c->timing_now = c->timing > 0 && (c->timing_frame++ % c->timing) == 0;
  const size_t ev_mark = c->ev_used;  // brackets of earlier frames still pending (harvested lazily)
  const int rs = dispatch_step(c, in, table, tbytes, gh);
  c->timing_now = false;
  if (rs != PFMPE_OK) c->ev_used = ev_mark;  // only the failed frame's own brackets are dropped
  else if (c->ev_used >= kHarvestPairs) RET(harvest_timing(c));  // pending brackets: harvest_timing
  RET(rs);
  take_step(c, in, out);
  return PFMPE_OK;
}

int pfmpe_step_multi(pfmpe_ctx* const* ctxs, int S, const pfmpe_frame_in* in, pfmpe_frame_out* out) {
  if (!ctxs || S < 1 || !ctxs[0]) return PFMPE_E_ARG;
  pfmpe_ctx* c0 = ctxs[0];
  if (!in || !out) return fail(c0, PFMPE_E_ARG, "step_multi: null in/out");
  if (S > 65535) return fail(c0, PFMPE_E_CAP, "step_multi: at most 65535 streams per batch");
  for (int s = 0; s < S; ++s) {
    pfmpe_ctx* c = ctxs[s];
    const std::string who = "step_multi: stream " + std::to_string(s) + ": ";
    if (!c) return fail(c0, PFMPE_E_ARG, who + "null context");
    if (c->device != c0->device || c->state_dtype != c0->state_dtype ||
        c->params.rng_mode != c0->params.rng_mode || c->prune != c0->prune)
      return fail(c0, PFMPE_E_ARG, who + "device, state type, RNG mode and pruning must match ctxs[0]");
    for (int e = 0; e < s; ++e)
      if (ctxs[e] == c) return fail(c0, PFMPE_E_ARG, who + "context appears twice");
    const int rc = check_step(c, &in[s], &out[s]);
    if (rc != PFMPE_OK) return fail(c0, rc, who + c->err);  // the per-stream code (E_ARG / E_CAP / E_STATE)
  }
  c0->mt_enter = now_ns();
  RET(set_device(c0));
  c0->timing_now = c0->timing > 0 && (c0->timing_frame++ % c0->timing) == 0;  // batches timed on the leader
  const bool ref = c0->params.rng_mode == PFMPE_RNG_REFERENCE;
  const size_t ev_mark = c0->ev_used;
  int rs;
  switch (c0->state_dtype) {
    case PFMPE_STATE_F64:
      rs = ref ? multi_m<double, kRngReference, double>(ctxs, S, in) : multi_m<double, kRngPhilox, double>(ctxs, S, in);
      break;
    case PFMPE_STATE_F16:
      rs = ref ? multi_m<float, kRngReference, __half>(ctxs, S, in) : multi_m<float, kRngPhilox, __half>(ctxs, S, in);
      break;
    default:
      rs = ref ? multi_m<float, kRngReference, float>(ctxs, S, in) : multi_m<float, kRngPhilox, float>(ctxs, S, in);
  }
  c0->timing_now = false;
  if (rs != PFMPE_OK) c0->ev_used = ev_mark;  // only the failed batch's own brackets are dropped
  else if (c0->ev_used >= kHarvestPairs) RET(harvest_timing(c0));
  RET(rs);
  const int64_t t_r = now_ns();
  for (int s = 0; s < S; ++s) {
    take_step(ctxs[s], &in[s], &out[s]);
    if (!ctxs[s]->fused) ctxs[s]->clean_since_fallback += 1;  // a clean two-launch frame (PFMPE_OPT_FUSED_REARM)
  }
  c0->mt_ns[3] += now_ns() - t_r;
  c0->mt_batches += 1;
  return PFMPE_OK;
}

int pfmpe_step_multi_batch(pfmpe_ctx* const* ctxs, int S, const pfmpe_frame_in* in, int n, pfmpe_frame_out* out,
                           int* done) {
  if (done) *done = 0;
  if (!ctxs || S < 1 || !ctxs[0]) return PFMPE_E_ARG;
  if ((!in || !out) && n > 0) return fail(ctxs[0], PFMPE_E_ARG, "step_multi_batch: null in/out");
  for (int f = 0; f < n; ++f) {
    RET(pfmpe_step_multi(ctxs, S, in + (size_t)f * S, out + (size_t)f * S));
    if (done) *done = f + 1;
  }
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

namespace {
// project2d (PE:1017-1034) in double on the host: (K34 * T) * [X;1], then / z
void host_project(const double* K, const double* T12, const double* X, double* uv) {
  double Q[12];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 4; ++j) {
      double s = K[i * 3 + 0] * T12[0 * 4 + j];
      s = s + K[i * 3 + 1] * T12[1 * 4 + j];
      s = s + K[i * 3 + 2] * T12[2 * 4 + j];
      Q[i * 4 + j] = s;
    }
  double p[3];
  for (int i = 0; i < 3; ++i) {
    double s = Q[i * 4 + 0] * X[0];
    s = s + Q[i * 4 + 1] * X[1];
    s = s + Q[i * 4 + 2] * X[2];
    p[i] = s + Q[i * 4 + 3];
  }
  uv[0] = p[0] / p[2];
  uv[1] = p[1] / p[2];
}
// LEDDetector::distortPoints (led_detector.cpp:371-414) on cv::Point2f inputs, result back to float
void host_distort(const double* K, const double* D, float xin, float yin, float* xo, float* yo) {
  const double fx = K[0], fy = K[4], cx = K[2], cy = K[5];
  const double k1 = D[0], k2 = D[1], p1 = D[2], p2 = D[3], k3 = D[4];
  const double x = ((double)xin - cx) / fx;
  const double y = ((double)yin - cy) / fy;
  const double r2 = x * x + y * y;
  double xc = x * (1. + k1 * r2 + k2 * r2 * r2 + k3 * r2 * r2 * r2);
  double yc = y * (1. + k1 * r2 + k2 * r2 * r2 + k3 * r2 * r2 * r2);
  xc = xc + (2. * p1 * x * y + p2 * (r2 + 2. * x * x));
  yc = yc + (p1 * (r2 + 2. * y * y) + 2. * p2 * x * y);
  *xo = (float)(xc * fx + cx);
  *yo = (float)(yc * fy + cy);
}
}  // namespace

int pfmpe_predict_roi(pfmpe_ctx* c, const pfmpe_roi_in* in, pfmpe_roi_out* out) {
  if (!c) return PFMPE_E_ARG;
  if (!in || !out) return fail(c, PFMPE_E_ARG, "predict_roi: null in/out");
  if (!c->has_model || !c->has_prior) return fail(c, PFMPE_E_STATE, "predict_roi: set_model and set_prior first");
  if (in->image_w < 1 || in->image_h < 1) return fail(c, PFMPE_E_ARG, "predict_roi: bad image size");
  RET(set_device(c));
  const int N = c->N;
  const int nblk = (N + kBlock - 1) / kBlock;
  if (!c->d_roi) HIPCHK(c, hipMalloc((void**)&c->d_roi, ((size_t)c->max_blk + 1) * 4 * sizeof(double)));
  RoiArgs ra{};
  std::memcpy(ra.cam, in->cam_move_inv, sizeof(ra.cam));
  std::memcpy(ra.predm, in->prediction, sizeof(ra.predm));
  std::memcpy(ra.K, c->K, sizeof(ra.K));
  std::memcpy(ra.markers, c->markers, sizeof(ra.markers));
  std::memcpy(ra.anchor, c->anchor[c->prior_idx], sizeof(ra.anchor));
  ra.N = N;
  ra.M = c->M;
  ra.ld = c->ld;
  ra.owner = prior_owner_ptr(c);
  double* part = c->d_roi + 4;
  RET(launch(c, PFMPE_K_ROI, [&] {
    const void* st = c->d_state[c->prior_idx];
    if (c->state_dtype == PFMPE_STATE_F64)
      hipLaunchKernelGGL((k_roi<double, double>), dim3(nblk), dim3(kBlock), 0, c->stream, ra, (const double*)st, part);
    else if (c->state_dtype == PFMPE_STATE_F16)
      hipLaunchKernelGGL((k_roi<float, __half>), dim3(nblk), dim3(kBlock), 0, c->stream, ra, (const __half*)st, part);
    else
      hipLaunchKernelGGL((k_roi<float, float>), dim3(nblk), dim3(kBlock), 0, c->stream, ra, (const float*)st, part);
    hipLaunchKernelGGL((k_roi_final<double>), dim3(1), dim3(kBlock), 0, c->stream, part, nblk, c->d_roi);
  }));
  double bb[4];
  HIPCHK(c, hipMemcpyAsync(bb, c->d_roi, sizeof(bb), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  RET(harvest_timing(c));
  // + the markers at predicted_pose_ (PE:1049-1052)
  for (int m = 0; m < c->M; ++m) {
    double uv[2];
    host_project(c->K, in->predicted_pose, c->markers + 3 * m, uv);
    if (uv[0] < bb[0]) bb[0] = uv[0];
    if (uv[0] > bb[1]) bb[1] = uv[0];
    if (uv[1] < bb[2]) bb[2] = uv[1];
    if (uv[1] > bb[3]) bb[3] = uv[1];
  }
  std::memcpy(out->bbox, bb, sizeof(bb));
  // determineROI (led_detector.cpp:317-368): corners as cv::Point2f, distorted, border, clamp, cv::Rect
  float x0f, y0f, x1f, y1f;
  host_distort(c->K, in->D, (float)bb[0], (float)bb[2], &x0f, &y0f);
  host_distort(c->K, in->D, (float)bb[1], (float)bb[3], &x1f, &y1f);
  const double W = in->image_w, H = in->image_h, b = in->border;
  const double x0 = std::max(0.0, std::min(W, (double)x0f - b));
  const double x1 = std::max(0.0, std::min(W, (double)x1f + b));
  const double y0 = std::max(0.0, std::min(H, (double)y0f - b));
  const double y1 = std::max(0.0, std::min(H, (double)y1f + b));
  if (x1 - x0 < 1 || y1 - y0 < 1) {
    out->x = 0;
    out->y = 0;
    out->width = in->image_w;
    out->height = in->image_h;
  } else {
    out->x = (int32_t)x0;
    out->y = (int32_t)y0;
    out->width = (int32_t)(x1 - x0);
    out->height = (int32_t)(y1 - y0);
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
    launch_export<double, double>(c, N, c->anchor[c->prior_idx]);
  } else if (c->state_dtype == PFMPE_STATE_F16) {
    launch_export<float, __half>(c, N, c->anchor[c->prior_idx]);
  } else {
    launch_export<float, float>(c, N, c->anchor[c->prior_idx]);
  }
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipMemcpyAsync(out, c->d_xfer, (size_t)N * 12 * sizeof(double), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  RET(harvest_timing(c));
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
  // in the context's stream: the frame's kernel may still be retiring after its record reached the host
  HIPCHK(c, hipMemcpyAsync(out, c->d_counts, (size_t)c->N * sizeof(uint32_t), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return PFMPE_OK;
}

// Undocumented diagnostic: reset (out == NULL) or read the kStamps stamps of the last frame (diag & 4).
int pfmpe_debug_stamps(pfmpe_ctx* c, uint64_t* out) {
  if (!c || !c->d_stamps) return PFMPE_E_STATE;
  RET(set_device(c));
  hipStream_t st = c->stream;
  const size_t rows = 1 + (size_t)c->max_blk;
  if (!out) {
    HIPCHK(c, hipMemsetAsync(c->d_stamps, 0, rows * kStamps * sizeof(uint64_t), st));
    HIPCHK(c, hipStreamSynchronize(st));
    return PFMPE_OK;
  }
  std::vector<uint64_t> h(rows * kStamps);
  HIPCHK(c, hipMemcpyAsync(h.data(), c->d_stamps, h.size() * sizeof(uint64_t), hipMemcpyDeviceToHost, st));
  HIPCHK(c, hipStreamSynchronize(st));
  for (int i = 0; i < kStamps; ++i) {
    const bool is_min = i == 0 || i == 4 || i == 19;
    uint64_t v = h[i];
    for (size_t r = 1; r < rows; ++r) {
      const uint64_t x = h[r * kStamps + i];
      if (!x) continue;
      if (!v || (is_min ? x < v : x > v)) v = x;
    }
    out[i] = v;
  }
  return PFMPE_OK;
}

int pfmpe_get_kernel_stats(pfmpe_ctx* c, int kernel, int64_t* launches, double* total_ms) {
  if (!c || kernel < 0 || kernel >= PFMPE_K_COUNT) return PFMPE_E_ARG;
  if (c->ev_used) {  // pending brackets of timed frames
    HIPCHK(c, hipSetDevice(c->device));
    RET(harvest_timing(c));
  }
  if (launches) *launches = c->k_launches[kernel];
  if (total_ms) *total_ms = c->k_ms[kernel];
  return PFMPE_OK;
}

int pfmpe_get_info(const pfmpe_ctx* c, int key, int64_t* value) {
  if (!c || !value) return PFMPE_E_ARG;
  switch (key) {
    case PFMPE_INFO_FUSED: *value = c->fused; return PFMPE_OK;
    case PFMPE_INFO_FUSED_FALLBACKS: *value = c->fused_fallbacks; return PFMPE_OK;
    case PFMPE_INFO_LAST_SHAPE: *value = c->last_shape; return PFMPE_OK;
    case PFMPE_INFO_LAST_WEIGH_PASS: *value = c->last_weigh_pass; return PFMPE_OK;
    case PFMPE_INFO_LAST_RESAMPLE: *value = c->last_resample; return PFMPE_OK;
    case PFMPE_INFO_LAST_GRID: *value = c->last_grid; return PFMPE_OK;
    case PFMPE_INFO_GUARD_SKIPS: *value = c->guard_skips; return PFMPE_OK;
    case PFMPE_INFO_N: *value = c->N; return PFMPE_OK;
    case 110: case 111: case 112: case 113: *value = c->mt_ns[key - 110]; return PFMPE_OK;  // batch host timing
    case 114: *value = c->mt_batches; return PFMPE_OK;
    default: return PFMPE_E_ARG;
  }
}

int pfmpe_reset_kernel_stats(pfmpe_ctx* c) {
  if (!c) return PFMPE_E_ARG;
  if (c->ev_used) {  // pending brackets belong to the statistics being reset
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipEventSynchronize(c->ev_pool[c->ev_used - 1].b));  // before their events are recorded again
    c->ev_used = 0;
  }
  for (int k = 0; k < PFMPE_K_COUNT; ++k) {
    c->k_launches[k] = 0;
    c->k_ms[k] = 0;
  }
  return PFMPE_OK;
}

const char* pfmpe_kernel_name(int kernel) {
  static const char* names[PFMPE_K_COUNT] = {"k_propagate_weigh", "k_resample", "aux", "k_frame", "k_roi",
                                                 "k_resample_final", "k_p3p_hist", "k_p3p_check",
                                                 "k_det (detector pipeline)"};
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
