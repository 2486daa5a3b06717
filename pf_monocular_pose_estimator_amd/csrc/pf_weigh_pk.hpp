// pf_weigh_pk.hpp — the streaming weighing pass with TWO particles per lane, packed fp32 (gfx950).
//
// Same job, same outputs and the same bits as k_weigh_stream (pf_kernels.hpp; PE:543-604: motion model,
// project2d, calculateEstimationProbability), for the frames the throughput configurations run: fp32 compute,
// the Philox stream, exactly 5 markers, the 2D blob grid, small motion angles, an identity camMoveInv, an
// upper-triangular K and at least as many blobs as markers (the host checks: pk_eligible in pfmpe_ctx.hpp;
// every other frame takes k_weigh_stream).
//
// Why: k_weigh_stream is VALU-issue bound (C4: 486 VALU per particle at ~4.3 cycles per wave instruction,
// DESIGN.md §4.1).  Here lane l of a wave carries particles n and n + 64 of a 128-particle task, and every fp32
// quantity is a pair {particle n, particle n + 64} in one 64-bit register pair, so each v_pk_fma_f32 /
// v_pk_mul_f32 / v_pk_add_f32 does the same operation for both particles: the rotation composition, the K*P
// product, the five projections, the grid-cell coordinates and the score arithmetic run at two operations per
// instruction.  Each lane of a packed instruction performs exactly the scalar operation (fp32 fma, mul or add,
// rounded to nearest; the TUs are built with -ffp-contract=off), so every weight, propagated particle and
// partial equals k_weigh_stream's bit for bit (tests/test_gpu_weigh_pk.py).
//
// Other cuts against k_weigh_stream, all exact:
//  * Philox rounds 1-3 with the wave-uniform counter words (iteration, frame) and key on the scalar unit;
//  * fp16 state decoded by v_fma_mix_f32 (half -> float plus the anchor, one rounding: the same value as the
//    conversion followed by the fp32 add), one instruction per plane;
//  * the kept propagated set is stored right after the motion model, so the pose does not stay live across
//    the likelihood;
//  * the first grid entry's distance is not clamped to +inf (a NaN distance only arises from a NaN / infinite
//    projection, whose gate fails either way: acc = sqrt(m) <= tol_PF is false for NaN and +inf alike, and the
//    later entries' strict `<` cannot take a finite distance then; the weight depends on m only through acc
//    and q of accepted markers);
//  * the self-occlusion / downgrade penalty is evaluated only in a wave where some lane has one (Pr - 0 = Pr:
//    the running sum starts at +0 and never becomes -0).
//
// The wave partials are k_weigh_stream's: one per 64 consecutive particles (wave_weight_partials on the A and
// on the B particles of the task), stored at part[2 * task] and part[2 * task + 1], i.e. part[4 * block + wave]
// of the 256-particle block numbering, so k_group / k_group_top / k_top read them unchanged.
#pragma once
#include "pf_kernels.hpp"

namespace pfmpe {

__device__ __forceinline__ f32x2 pk_splat(float a) { return f32x2{a, a}; }

// v_fma_mix_f32: half h (the low or high half of a dword) as float, plus the fp32 anchor, rounded once.
// (float)h is exact, so this is (float)h + a with one rounding: __half2float(h) + a, bit for bit.
template <int HI>
__device__ __forceinline__ float f16_plus(uint32_t w, float a) {
  float r;
  if (HI)
    asm("v_fma_mix_f32 %0, %1, 1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "=v"(r) : "v"(w), "v"(a));
  else
    asm("v_fma_mix_f32 %0, %1, 1.0, %2 op_sel:[0,0,0] op_sel_hi:[1,0,0]" : "=v"(r) : "v"(w), "v"(a));
  return r;
}

// Philox4x32-10 (pf_rng.hpp philox4x32_10) for the motion counters of particles nA and nB:
// counter {n, c1, c2, c3} with c1 = iter | tag << 24, c2 = frame_lo, c3 = frame_hi wave-uniform, key uniform.
// The uniform parts of rounds 1-3 are scalar: round 1's c2 product and its output words 0 / 1, round 2's
// c0 product and its output word 3; the two particles' rounds are interleaved.
struct Phx2 {
  U32x4 a, b;
};
__device__ __forceinline__ uint32_t mulhi_u(uint32_t a, uint32_t b) { return (uint32_t)(((uint64_t)a * b) >> 32); }
__device__ __forceinline__ Phx2 philox_motion_pair(uint32_t nA, uint32_t nB, uint32_t c1, uint32_t c2, uint32_t c3,
                                                   uint32_t k0, uint32_t k1) {
  constexpr uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u, W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
  // c1, c2, c3, k0, k1: kernel arguments (SGPRs), so the uniform products and xors below are scalar.  They are
  // loop-invariant in the task loop; pinned per call, the ~12 scalar ops run per task instead of their results
  // being hoisted into SGPRs that spilled to VGPR lanes (a v_readlane, a VALU slot, per use)
  asm volatile("" : "+s"(c1), "+s"(c2), "+s"(c3), "+s"(k0), "+s"(k1));
  // round 1: p1 = M1 * c2 (uniform): n0 = hi(p1) ^ c1 ^ k0, n1 = lo(p1) uniform; p0 = M0 * n (per lane)
  const uint32_t r1n0 = mulhi_u(M1, c2) ^ c1 ^ k0;
  const uint32_t r1n1 = M1 * c2;
  const uint32_t s13 = c3 ^ k1;
  uint64_t pA = (uint64_t)M0 * nA, pB = (uint64_t)M0 * nB;
  uint32_t a2 = (uint32_t)(pA >> 32) ^ s13, a3 = (uint32_t)pA;
  uint32_t b2 = (uint32_t)(pB >> 32) ^ s13, b3 = (uint32_t)pB;
  // round 2 (keys +W): c0 = r1n0, c1 = r1n1 uniform; p0 = M0 * r1n0 uniform
  uint32_t rk0 = k0 + W0, rk1 = k1 + W1;
  const uint32_t r2p0h = mulhi_u(M0, r1n0), r2n3 = M0 * r1n0;
  const uint32_t s20 = r1n1 ^ rk0, s22 = r2p0h ^ rk1;
  pA = (uint64_t)M1 * a2;
  pB = (uint64_t)M1 * b2;
  uint32_t a0 = (uint32_t)(pA >> 32) ^ s20, a1 = (uint32_t)pA;
  uint32_t b0 = (uint32_t)(pB >> 32) ^ s20, b1 = (uint32_t)pB;
  a2 = a3 ^ s22;
  b2 = b3 ^ s22;
  // round 3: c3 = r2n3 uniform
  rk0 += W0;
  rk1 += W1;
  const uint32_t s33 = r2n3 ^ rk1;
  {
    const uint64_t qA0 = (uint64_t)M0 * a0, qA1 = (uint64_t)M1 * a2;
    const uint64_t qB0 = (uint64_t)M0 * b0, qB1 = (uint64_t)M1 * b2;
    const uint32_t na0 = xor3_key((uint32_t)(qA1 >> 32), a1, rk0), na2 = (uint32_t)(qA0 >> 32) ^ s33;
    const uint32_t nb0 = xor3_key((uint32_t)(qB1 >> 32), b1, rk0), nb2 = (uint32_t)(qB0 >> 32) ^ s33;
    a1 = (uint32_t)qA1;
    a3 = (uint32_t)qA0;
    b1 = (uint32_t)qB1;
    b3 = (uint32_t)qB0;
    a0 = na0;
    a2 = na2;
    b0 = nb0;
    b2 = nb2;
  }
  // rounds 4-10: every word per lane (the round keys on the scalar unit, kept there by the empty asm)
  asm volatile("" : "+s"(rk0), "+s"(rk1));
#pragma unroll
  for (int r = 3; r < 10; ++r) {
    rk0 += W0;
    rk1 += W1;
    const uint64_t qA0 = (uint64_t)M0 * a0, qA1 = (uint64_t)M1 * a2;
    const uint64_t qB0 = (uint64_t)M0 * b0, qB1 = (uint64_t)M1 * b2;
    const uint32_t na0 = xor3_key((uint32_t)(qA1 >> 32), a1, rk0), na2 = xor3_key((uint32_t)(qA0 >> 32), a3, rk1);
    const uint32_t nb0 = xor3_key((uint32_t)(qB1 >> 32), b1, rk0), nb2 = xor3_key((uint32_t)(qB0 >> 32), b3, rk1);
    a1 = (uint32_t)qA1;
    a3 = (uint32_t)qA0;
    b1 = (uint32_t)qB1;
    b3 = (uint32_t)qB0;
    a0 = na0;
    a2 = na2;
    b0 = nb0;
    b2 = nb2;
  }
  return Phx2{U32x4{a0, a1, a2, a3}, U32x4{b0, b1, b2, b3}};
}

// The six motion draws' integers (philox_motion6) as exact floats: v < 2^21, so bits 0x4b000000 | v are the float
// 2^23 + v and subtracting 2^23 is exact; v_alignbit places o >> 11 under the exponent in one instruction.
__device__ __forceinline__ float u21_bits(uint32_t bits) { return __uint_as_float(bits); }
__device__ __forceinline__ void draw_words(const U32x4& o, float* f) {
  f[0] = u21_bits(__builtin_amdgcn_alignbit(0x258u, o.x, 11));
  f[1] = u21_bits(__builtin_amdgcn_alignbit(0x258u, o.y, 11));
  f[2] = u21_bits(__builtin_amdgcn_alignbit(0x258u, o.z, 11));
  f[3] = u21_bits(__builtin_amdgcn_alignbit(0x258u, o.w, 11));
  // ((x & 0x7FF) << 10) | (y & 0x3FF), with the exponent bits: one and-or and one bitfield insert
  f[4] = u21_bits(((o.x << 10) & 0x1FFC00u) | ((o.y & 0x3FFu) | 0x4B000000u));
  f[5] = u21_bits(((o.z << 10) & 0x1FFC00u) | ((o.w & 0x3FFu) | 0x4B000000u));
}

// 12 state values of both particles of the task as pairs {A, B} (fp16: plus the anchor), from the raw words
// prefetched for each (fp16: the six pair-plane dwords; fp32: twelve).  Two separate RawState objects: held as
// one aggregate {a, b}, the fp32 instance kept a's words in scratch across the loop (stored right after the
// prefetch loads, which made the wave wait for them, and reloaded at the next task).
template <typename SP>
__device__ __forceinline__ void decode2(const RawState<SP>& Ra, const RawState<SP>& Rb, const float* anc, f32x2* A) {
  if constexpr (std::is_same<SP, __half>::value) {
#pragma unroll
    for (int k = 0; k < 6; ++k) {
      const uint32_t wa = __builtin_bit_cast(uint32_t, Ra.p[k]), wb = __builtin_bit_cast(uint32_t, Rb.p[k]);
      A[2 * k] = f32x2{f16_plus<0>(wa, anc[2 * k]), f16_plus<0>(wb, anc[2 * k])};
      A[2 * k + 1] = f32x2{f16_plus<1>(wa, anc[2 * k + 1]), f16_plus<1>(wb, anc[2 * k + 1])};
    }
  } else {
#pragma unroll
    for (int q = 0; q < 12; ++q) A[q] = f32x2{__uint_as_float(Ra.v[q]), __uint_as_float(Rb.v[q])};
  }
}

// the kept propagated set (PFMPE_OPT_KEEP_PROPAGATED) for one particle of the pair (HI: the B particle):
// store_pose's values (fp16: the fp32 difference to the anchor, converted to nearest even, pair planes)
template <typename SP, int HI>
__device__ __forceinline__ void store_kept(SP* __restrict__ dst, int64_t ld, int n, const f32x2* P, const f32x2* D) {
  const __amdgpu_buffer_rsrc_t r = plane_rsrc((const SP*)dst, ld);
  if constexpr (std::is_same<SP, __half>::value) {
    static_assert(PFMPE_F16_PAIRS != 0, "k_weigh_pk stores fp16 pair planes");
    typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
    const uint32_t pps = (uint32_t)(ld * 4);
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      const f32x2 d = HI ? f32x2{D[2 * j].y, D[2 * j + 1].y} : f32x2{D[2 * j].x, D[2 * j + 1].x};
      const uint32_t w = __builtin_bit_cast(uint32_t, __builtin_convertvector(d, f16x2));
      __builtin_amdgcn_raw_buffer_store_b32(w, r, (uint32_t)n * 4u, (uint32_t)j * pps, 0);
    }
  } else {
    (void)D;
    const uint32_t ps = (uint32_t)(ld * 4);
#pragma unroll
    for (int q = 0; q < 12; ++q)
      __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(HI ? P[q].y : P[q].x), r, (uint32_t)n * 4u,
                                            (uint32_t)q * ps, 0);
  }
}

// one grid lookup of marker (u, v) for one particle: column_minima's grid branch (first entry untested)
struct GridHit {
  float bd;
  int bo;
  uint32_t rec;
};
__device__ __forceinline__ uint32_t grid_rec(const unsigned char* cells, int ncx4, float fmaxx, float fmaxy, float fx,
                                             float fy) {
  const int cx = (int)__builtin_amdgcn_fmed3f(fx, 0.0f, fmaxx);
  const int cy = (int)__builtin_amdgcn_fmed3f(fy, 0.0f, fmaxy);
  return *(const uint32_t*)(cells + 4 * mad24(cy, ncx4 >> 2, cx));  // v_mad_u32_u24 + v_lshl_add_u32
}
// further entries of a cell list (rare: some lane of the wave has a longer list), two per step as in
// column_minima: strict `<`, so the lowest original index among equally close blobs stays
__device__ __forceinline__ void grid_walk(const unsigned char* ents, uint32_t rec, float u, float v, float& bd,
                                          int& bo) {
  const GridEnt* e = (const GridEnt*)(ents + (rec & 0xffffu));
  const int n = (int)(rec >> 16);
  const f32x2 uvj = pk2(u, v);
  auto visit = [&](const GridEnt& ec, bool in) {
    const f32x2 dd = pk2(ec.x, ec.y) - uvj;
    const float d = fmadd(dd.x, dd.x, dd.y * dd.y);
    const bool take = in & (d < bd);
    bd = take ? d : bd;
    bo = take ? ec.orig : bo;
  };
#pragma unroll 2
  for (int c = 1; c < n; c += 2) {
    const GridEnt ea = e[c], eb = e[c + 1];
    visit(ea, true);
    visit(eb, c + 1 < n);
  }
}

// One 64-particle wave partial (BlockPart: wave_weight_partials' values, k_weigh_stream's record) of fp32 weights
// w of particles nbase + lane.  The steady state (every lane valid, no negative weight) is computed directly:
//  * the total: the scan's lane-63 value, bit for bit (as integers on the 2^-21 grid when every weight is below
//    32, else wave_total_lane63); it is also the maximum in-wave prefix (non-negative addends: the prefix is
//    lane-monotone), and lane 0's weight the minimum;
//  * the maximum weight as the integer maximum of the weights' bits (no weight is NaN or -0: the score adds
//    positive terms to +0 and subtracts penalties, and fl(x - x) = +0, so the bits of non-negative weights
//    order like their values), DPP max steps across quads and rows, then the two row broadcasts to lane 63;
//  * the first lane holding it by ballot: argmax = nbase + that lane;
//  * lane 63 stores {sum, maxrel} from its own registers, lane 0 {minrel, maxw, minw = +inf, argmax,
//    argmin = none}.
// Anything else (a partial wave past N, a negative weight) takes wave_weight_partials as k_weigh_stream does.
// full: every particle of the task is below N (wave-uniform, decided on the scalar unit: no validity ballots).
__device__ __forceinline__ void pk_wave_partial(float w, bool valid, bool full, int nbase, BlockPart* __restrict__ dst) {
  const int lane = lane_id();
  if (full && __builtin_amdgcn_ballot_w64(w < 0.0f) == 0) {
    const double x = (double)w;
    int k = __float_as_int(w);
    k = max(k, __builtin_amdgcn_mov_dpp(k, kDppQuadXor1, 0xf, 0xf, true));
    k = max(k, __builtin_amdgcn_mov_dpp(k, kDppQuadXor2, 0xf, 0xf, true));
    k = max(k, __builtin_amdgcn_mov_dpp(k, kDppRowHalfMirror, 0xf, 0xf, true));
    k = max(k, __builtin_amdgcn_mov_dpp(k, kDppRowMirror, 0xf, 0xf, true));
    // (bound_ctrl: every lane of these patterns has a source, and with it the moves fold into v_max_i32_dpp)
    k = max(k, dpp<kDppBcast15, 0xa>(k, INT_MIN));  // row totals carried into rows 1 / 3, then 2 / 3: lane 63
    k = max(k, dpp<kDppBcast31, 0xc>(k, INT_MIN));
    const int mxb = __builtin_amdgcn_readlane(k, 63);
    const uint64_t bx = __builtin_amdgcn_ballot_w64(__float_as_int(w) == mxb);
    const int ix = nbase + (int)__builtin_ctzll(bx);
    // the total: with every weight below 32 (the usual case: at most 5 * 6), as integers on the 2^-21 grid every
    // weight of this pass lies on (wave_incl_sum_fx, pf_kernels.hpp): the exact sum, which is what the fp64
    // butterfly yields too (its partial sums need at most 32 significant bits)
    double wi;
    if (mxb < 0x42000000) {  // 32.0f; a scalar branch
      uint32_t t = (uint32_t)(w * 0x1p21f);
      t += (uint32_t)__builtin_amdgcn_mov_dpp((int)t, kDppQuadXor1, 0xf, 0xf, true);
      t += (uint32_t)__builtin_amdgcn_mov_dpp((int)t, kDppQuadXor2, 0xf, 0xf, true);
      t += (uint32_t)__builtin_amdgcn_mov_dpp((int)t, kDppRowHalfMirror, 0xf, 0xf, true);
      t += (uint32_t)__builtin_amdgcn_mov_dpp((int)t, kDppRowMirror, 0xf, 0xf, true);
      t += dpp_u32<kDppBcast15, 0xa>(t, 0u);
      t += dpp_u32<kDppBcast31, 0xc>(t, 0u);
      wi = (double)(uint32_t)__builtin_amdgcn_readlane((int)t, 63) * 0x1p-21;
    } else {
      wi = wave_total_lane63(x);
    }
    if (lane == 63) {
      dst->sum = wi;
      dst->maxrel = wi;
    }
    if (lane == 0) {
      dst->minrel = x;
      dst->maxw = (double)__int_as_float(mxb);
      dst->minw = (double)INFINITY;
      dst->argmax = ix;
      dst->argmin = 0x7fffffff;
    }
    return;
  }
  double wi, rmx, rmn;
  float mx, mn;
  int ix, in_;
  wave_weight_partials(w, valid, nbase + lane, wi, rmx, rmn, mx, ix, mn, in_);
  const double tot = lane_value(wi, 63);
  if (lane == 0) {
    BlockPart q;
    q.sum = tot;
    q.maxrel = rmx;
    q.minrel = rmn;
    q.maxw = (double)mx;
    q.minw = (double)mn;
    q.argmax = ix;
    q.argmin = in_;
    *dst = q;
  }
}

// Per-block LDS copies of the frame constants the loop reads besides LdsConst (the anchors and the grid's float
// parameters): held in SGPRs they are loop-invariant kernel arguments the compiler hoists, and with the buffer
// resources and plane offsets they exceed the SGPR file (spilled to VGPR lanes: a v_readlane per use).  From
// LDS they arrive in VGPRs, which is also what the packed and mixed-precision operations take.
struct PkLds {
  float anc_in[12], anc_out[12];
  float inv_c, ox, oy, fmaxx, fmaxy, pad[3];
};
// a wave-uniform value the compiler may not hoist out of the loop (recomputed per iteration on the scalar unit)
__device__ __forceinline__ uint32_t sopaque(uint32_t x) {
  asm volatile("" : "+s"(x));
  return x;
}

// 1: k_weigh_pk's self-occlusion test as one packed 16-bit minimum over the marker pairs' key xors (A/B)
#ifndef PFMPE_PK_DUP_MIN
#define PFMPE_PK_DUP_MIN 1
#endif
// Occupancy floor (waves per SIMD; 1 = the compiler's choice), set by the fp16 / fp32 TUs
#ifndef PFMPE_WEIGH_PK_MIN_WAVES
#define PFMPE_WEIGH_PK_MIN_WAVES 1
#endif


// The pass for one stream: workgroup wg of nwg resident workgroups (the one-stream kernel: blockIdx / gridDim; the
// batched kernel: the stream's share of the grid).  fa_words: the frame arguments as words (kernarg segment or the
// stream's descriptor) for the LDS constants.
template <typename SP, bool MULTI>
__device__ __forceinline__ void weigh_pk_body(const FrameArgsT<float>& fa, const uint32_t* fa_words, int wg, int nwg,
                                              const unsigned char* __restrict__ table, const SP* __restrict__ prior,
                                              float* __restrict__ w0, float* __restrict__ w1,
                                              BlockPart* __restrict__ part0, BlockPart* __restrict__ part1,
                                              const Ctrl* __restrict__ ctrl, SP* __restrict__ prop0,
                                              SP* __restrict__ prop1, int iter, unsigned char* smem,
                                              LdsConst<float>& sc, PkLds& pl) {
  constexpr int MAXM = kExactM;
  // the exit rule already fired (uniform); this iteration's weight slot (batched: explicit scalar loads of a
  // record written by an earlier launch, pf_kernels.hpp load_ctrl_word)
  if (MULTI ? load_ctrl_word<(int)offsetof(Ctrl, done)>(ctrl) : ctrl->done) return;
  const int slot = MULTI ? load_ctrl_word<(int)offsetof(Ctrl, cur_slot)>(ctrl) : ctrl->cur_slot;
  float* wout = slot ? w1 : w0;
  SP* pout = slot ? prop1 : prop0;
  BlockPart* parts = slot ? part1 : part0;
  const int lane = lane_id();
  const int ntask = 2 * fa.nblk;  // 128-particle tasks: every wave partial slot 4 * nblk gets written
  const int nwaves = nwg * kWaves;
  int tk = wg * kWaves + wave_id_u();
  copy_table(table, smem, (size_t)fa.tbytes);
  // stored rows of a task's two particles: n itself, or owner[n] for a deferred prior (FrameArgsT::owner).  The
  // owner indices are loaded one task ahead of the state they address (software pipelining: the state loads of
  // task t + 1, issued while task t computes, use owner values that arrived during task t - 1)
  const uint32_t* own = fa.owner;
  auto rows_of = [&](int t, int& ra, int& rb) {
    const int n = in_planes(t * 128 + lane, fa.N), m = in_planes(t * 128 + 64 + lane, fa.N);
    ra = own ? (int)own[n] : n;
    rb = own ? (int)own[m] : m;
  };
  RawState<SP> Ra{}, Rb{};
  int rA, rB;
  rows_of(tk, rA, rB);
  load_state_prefetch<SP>(prior, fa.ld, rA, true, Ra);
  load_state_prefetch<SP>(prior, fa.ld, rB, true, Rb);
  rows_of(tk + nwaves, rA, rB);
  stage_consts_from(fa_words, sc);
  if (threadIdx.x < 12) {
    pl.anc_in[threadIdx.x] = fa.anc_in[threadIdx.x];
    pl.anc_out[threadIdx.x] = fa.anc_out[threadIdx.x];
  } else if (threadIdx.x == 12) {
    pl.inv_c = fa.grid.inv_c;
    pl.ox = fa.grid.ox;
    pl.oy = fa.grid.oy;
    pl.fmaxx = fa.grid.fmaxx;
    pl.fmaxy = fa.grid.fmaxy;
  }
  __syncthreads();  // table + constants visible; no barrier after this point (each wave loops on its own)
  const LdsBlobs<float> tb = view_table<float>(smem, fa.B);
  const GridArgs& ga = fa.grid;
  const unsigned char* cells = tb.base + ga.cell_off;
  const unsigned char* ents = tb.base + ga.ent_off;
  const bool predict = fa.it > 1 && (iter % 10) != 0;  // ... * predictionMatrix (PE:556); cam_identity (host)
  const float gsc = (float)(1.0 + fa.growth * (double)(iter / 10));
  const float tol = fa.tol, tol_pf = fa.tol_pf, Mt = (float)kExactM, rtol = rcp_t(fa.tol);
  for (; tk < ntask; tk += nwaves) {
    const int nA = tk * 128 + lane, nB = nA + 64;
    const bool vA = nA < fa.N, vB = nB < fa.N;
    // ---- motion model (propagate, PE:543-588), both particles per instruction.  The draws come first: they need
    // no memory, so the wait for this task's prefetched state (and, the loop's waits being conservative, for the
    // previous task's stores) sits after ~130 instructions of the generator instead of at the top of the loop
    const Phx2 ph = philox_motion_pair((uint32_t)nA, (uint32_t)nB, (uint32_t)iter | (kTagMotion << 24), fa.flo, fa.fhi,
                                       fa.key0, fa.key1);
    __builtin_amdgcn_sched_barrier(0);  // the scheduler would otherwise pull the decode (and its wait) back up
    f32x2 A[12];
    decode2<SP>(Ra, Rb, pl.anc_in, A);
    // the plane stride, re-derived each task on the scalar unit (hoisted, its plane offsets held SGPRs across the
    // loop and spilled)
    const int64_t ldl = (int64_t)sopaque((uint32_t)fa.ld);
    // the next task's state, in flight across this task's arithmetic; then the rows of the task after it
    load_state_prefetch<SP>(prior, ldl, rA, true, Ra);
    load_state_prefetch<SP>(prior, ldl, rB, true, Rb);
    rows_of(tk + 2 * nwaves, rA, rB);
    f32x2 d[6];
    {
      float fa6[6], fb6[6];
      draw_words(ph.a, fa6);
      draw_words(ph.b, fb6);
#pragma unroll
      for (int q = 0; q < 6; ++q) {
        const f32x2 v = f32x2{fa6[q], fb6[q]} - pk_splat(8388608.0f);  // the 21-bit integer, exact
        d[q] = v * sc.rgs[q] + sc.lo[q];
      }
    }
    if (iter >= 10) {  // wave-uniform; exactly 1 before iteration 10
      asm volatile("");
#pragma unroll
      for (int q = 0; q < 6; ++q) d[q] = d[q] * gsc;
    }
    if (predict) {  // A = A * predictionMatrix (compose: k = 0..3 sequential, the translation column + A[i][3])
      f32x2 X[12];
#pragma unroll
      for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          f32x2 s = A[i * 4 + 0] * sc.predm[0 * 4 + j];
          s = pk_fma(A[i * 4 + 1], pk_splat(sc.predm[1 * 4 + j]), s);
          s = pk_fma(A[i * 4 + 2], pk_splat(sc.predm[2 * 4 + j]), s);
          if (j == 3) s = s + A[i * 4 + 3];
          X[i * 4 + j] = s;
        }
#pragma unroll
      for (int q = 0; q < 12; ++q) A[q] = X[q];
    }
    f32x2 sa, ca, sb, cb, sz, cz;
    {  // sincos_small (the host proved |angle| <= kSmallAngle for every draw of the frame)
      auto scs = [&](f32x2 x, f32x2& s, f32x2& c) {
        const f32x2 x2 = x * x;
        s = x * pk_fma(x2, pk_splat(-1.0f / 6.0f), pk_splat(1.0f));
        c = pk_fma(x2, pk_fma(x2, pk_splat(1.0f / 24.0f), pk_splat(-0.5f)), pk_splat(1.0f));
      };
      scs(d[0], sa, ca);
      scs(d[1], sb, cb);
      scs(d[2], sz, cz);
    }
    f32x2 P[12];
#pragma unroll
    for (int i = 0; i < 3; ++i) {  // R = ((R_A * Rz(c)) * Ry(b)) * Rx(a), t = t_A + (tX, tY, tZ) (PE:582-587)
      const f32x2 a0 = A[i * 4 + 0], a1 = A[i * 4 + 1], a2 = A[i * 4 + 2];
      const f32x2 z0 = pk_fma(a1, sz, a0 * cz);
      const f32x2 z1 = pk_fma(a1, cz, a0 * (-sz));
      const f32x2 y0 = pk_fma(a2, -sb, z0 * cb);
      const f32x2 y2 = pk_fma(a2, cb, z0 * sb);
      const f32x2 x1 = pk_fma(y2, sa, z1 * ca);
      const f32x2 x2 = pk_fma(y2, ca, z1 * (-sa));
      P[i * 4 + 0] = y0;
      P[i * 4 + 1] = x1;
      P[i * 4 + 2] = x2;
      P[i * 4 + 3] = A[i * 4 + 3] + d[3 + i];
    }
    if (tk == 0) {  // particles 0 / 1: current_pose_ / predicted_pose_ (PE:547, 551); wave-uniform branch
#pragma unroll
      for (int q = 0; q < 12; ++q) P[q].x = lane == 0 ? sc.cur[q] : (lane == 1 ? sc.pred[q] : P[q].x);
    }
    if (prop0) {  // the kept propagated set, stored now (its registers are free for the likelihood)
      f32x2 D[12];
      if constexpr (std::is_same<SP, __half>::value) {
#pragma unroll
        for (int q = 0; q < 12; ++q) D[q] = P[q] - pk_splat(pl.anc_out[q]);
      }
      if (vA) store_kept<SP, 0>(pout, ldl, nA, P, D);
      if (vB) store_kept<SP, 1>(pout, ldl, nB, P, D);
    }
    // ---- project2d (PE:1017-1034): Q = K * P (upper-triangular K, k_times_pose's operations), then u = p / p.z
    f32x2 Q[12];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      Q[j] = pk_fma(pk_splat(sc.K[2]), P[8 + j], pk_fma(pk_splat(sc.K[1]), P[4 + j], P[j] * sc.K[0]));
      Q[4 + j] = pk_fma(pk_splat(sc.K[5]), P[8 + j], P[4 + j] * sc.K[4]);
      Q[8 + j] = P[8 + j];
    }
    f32x2 u[MAXM], v[MAXM];
#pragma unroll
    for (int j = 0; j < MAXM; ++j) {
      const float X = sc.markers[3 * j], Y = sc.markers[3 * j + 1], Z = sc.markers[3 * j + 2];
      f32x2 su = Q[0] * X, sv = Q[4] * X, sz2 = Q[8] * X;
      su = pk_fma(Q[1], pk_splat(Y), su);
      sv = pk_fma(Q[5], pk_splat(Y), sv);
      sz2 = pk_fma(Q[9], pk_splat(Y), sz2);
      su = pk_fma(Q[2], pk_splat(Z), su);
      sv = pk_fma(Q[6], pk_splat(Z), sv);
      sz2 = pk_fma(Q[10], pk_splat(Z), sz2);
      su = su + Q[3];
      sv = sv + Q[7];
      sz2 = sz2 + Q[11];
      const f32x2 rz = f32x2{rcp_t(sz2.x), rcp_t(sz2.y)};
      u[j] = su * rz;
      v[j] = sv * rz;
    }
    // ---- column minima over the 2D grid (column_minima's grid branch), both particles.  In phases over the
    // markers (every cell record, then every first entry, then the rare longer lists behind one test): a
    // per-marker branch kept each marker's two dependent LDS round trips from overlapping the next marker's
    float mA[MAXM], mB[MAXM];
    int rA[MAXM], rB[MAXM];
    uint32_t recA[MAXM], recB[MAXM];
#pragma unroll
    for (int j = 0; j < MAXM; ++j) {
      const f32x2 fx = pk_fma(u[j], pk_splat(pl.inv_c), pk_splat(pl.ox));
      const f32x2 fy = pk_fma(v[j], pk_splat(pl.inv_c), pk_splat(pl.oy));
      recA[j] = grid_rec(cells, ga.ncx4, pl.fmaxx, pl.fmaxy, fx.x, fy.x);
      recB[j] = grid_rec(cells, ga.ncx4, pl.fmaxx, pl.fmaxy, fx.y, fy.y);
    }
    uint32_t lists = 0;  // a record above 0x1ffff: a list longer than one
#pragma unroll
    for (int j = 0; j < MAXM; ++j) {
      const GridEnt eA = *(const GridEnt*)(ents + (recA[j] & 0xffffu));
      const GridEnt eB = *(const GridEnt*)(ents + (recB[j] & 0xffffu));
      const f32x2 dx = f32x2{eA.x, eB.x} - u[j];
      const f32x2 dy = f32x2{eA.y, eB.y} - v[j];
      const f32x2 dd = pk_fma(dx, dx, dy * dy);
      mA[j] = dd.x;
      mB[j] = dd.y;
      rA[j] = eA.orig;
      rB[j] = eB.orig;
      lists |= recA[j] | recB[j];
    }
    if (__builtin_amdgcn_ballot_w64(lists > 0x1ffffu)) {  // rare (wave-uniform)
#pragma unroll
      for (int j = 0; j < MAXM; ++j)
        if (__builtin_amdgcn_ballot_w64((recA[j] > 0x1ffffu) | (recB[j] > 0x1ffffu))) {
          grid_walk(ents, recA[j], u[j].x, v[j].x, mA[j], rA[j]);
          grid_walk(ents, recB[j], u[j].y, v[j].y, mB[j], rB[j]);
        }
    }
    // ---- score (score_unordered: B >= M, the host checks), both particles
    f32x2 Pr = pk_splat(0.0f);
    bool accA[MAXM], accB[MAXM];
    // dup keys: the blob of an accepted marker, a value no blob index takes (0x8000 + j: blob indices are below
    // kMaxBlobs = 1024) otherwise; two equal keys are exactly two accepted markers on one blob (score_unordered's
    // dups > 0)
    int kA[MAXM], kB[MAXM];
#pragma unroll
    for (int j = 0; j < MAXM; ++j) {
      const f32x2 dj = f32x2{sqrt_t(mA[j]), sqrt_t(mB[j])};
      accA[j] = dj.x <= tol_pf;
      accB[j] = dj.y <= tol_pf;
      kA[j] = accA[j] ? rA[j] : 0x8000 + j;
      kB[j] = accB[j] ? rB[j] : 0x8000 + j;
      const f32x2 q = (pk_splat(tol) - dj) * rtol;
      const f32x2 t = pk_splat(Mt) + q * q;
      Pr = Pr + f32x2{accA[j] ? t.x : 0.0f, accB[j] ? t.y : 0.0f};  // Pr + 0 = Pr (Pr is never -0)
    }
    // any self-occlusion in the wave
#if PFMPE_PK_DUP_MIN
    // the keys' pairwise xors as 16-bit halves (A low, B high) folded into one packed 16-bit minimum (k_weigh_pk12's
    // form): no lane masks live on the scalar unit
    typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
    u16x2 dmin = {0xffff, 0xffff};
#pragma unroll
    for (int j = 1; j < MAXM; ++j)
#pragma unroll
      for (int e = 0; e < j; ++e)
        dmin = __builtin_elementwise_min(
            dmin, __builtin_bit_cast(u16x2, ((uint32_t)(kA[e] ^ kA[j]) & 0xffffu) | ((uint32_t)(kB[e] ^ kB[j]) << 16)));
    const uint64_t anydup = __builtin_amdgcn_ballot_w64((dmin.x == 0) | (dmin.y == 0));
#else
    // the pairwise key comparisons' lane masks ORed on the scalar unit
    uint64_t anydup = 0;
#pragma unroll
    for (int j = 1; j < MAXM; ++j)
#pragma unroll
      for (int e = 0; e < j; ++e)
        anydup |= __builtin_amdgcn_ballot_w64(kA[e] == kA[j]) | __builtin_amdgcn_ballot_w64(kB[e] == kB[j]);
#endif
    float wA = Pr.x, wB = Pr.y;
    if (anydup || fa.downgrade) {  // rare (wave-uniform): the penalties, as score_unordered counts them
      asm volatile("");  // a scalar branch (if-converted, every task paid the counting)
      auto pen = [&](const bool* acc, const int* r) {
        int dups = 0, ndg = 0;
#pragma unroll
        for (int j = 0; j < MAXM; ++j) {
          bool dup = false;
#pragma unroll
          for (int e = 0; e < j; ++e) dup |= acc[e] & (r[e] == r[j]);
          dups += (acc[j] & dup) ? 1 : 0;
          ndg += (acc[j] && ((fa.downgrade >> j) & 1u)) ? 1 : 0;
        }
        return (float)(3 * dups * (dups + 1) / 2 + 2 * ndg);
      };
      wA = wA - pen(accA, rA);
      wB = wB - pen(accB, rB);
    }
    // Eigen's visitor starts at coeff(0, 0): a NaN distance there gives weight 0 (blob 0 finite: host check)
    if (__builtin_isunordered(u[0].x, v[0].x)) wA = 0.0f;
    if (__builtin_isunordered(u[0].y, v[0].y)) wB = 0.0f;
    // ---- the weights and the two wave partials (k_weigh_stream's, one per 64 particles).  full (scalar): every
    // particle of the task is below N, so no per-lane validity selects, predicated stores or validity ballots
    const bool full = (tk + 1) * 128 <= fa.N;
    if (full) {
      wout[nA] = wA;
      wout[nB] = wB;
    } else {
      if (!vA) wA = 0.0f;
      if (!vB) wB = 0.0f;
      if (vA) wout[nA] = wA;
      if (vB) wout[nB] = wB;
    }
    pk_wave_partial(wA, vA, full, tk * 128, parts + (size_t)tk * 2);
    pk_wave_partial(wB, vB, full, tk * 128 + 64, parts + (size_t)tk * 2 + 1);
  }
}

template <typename SP>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(PFMPE_WEIGH_PK_MIN_WAVES))) void k_weigh_pk(
    const FrameArgsT<float> fa, const unsigned char* __restrict__ table, const SP* __restrict__ prior,
    float* __restrict__ w0, float* __restrict__ w1, BlockPart* __restrict__ part0, BlockPart* __restrict__ part1,
    const Ctrl* __restrict__ ctrl, SP* __restrict__ prop0, SP* __restrict__ prop1, int iter) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ LdsConst<float> sc;
  __shared__ PkLds pl;
  weigh_pk_body<SP, false>(fa, (const uint32_t*)__builtin_amdgcn_kernarg_segment_ptr(), (int)blockIdx.x,
                           (int)gridDim.x, table, prior, w0, w1, part0, part1, ctrl, prop0, prop1, iter, smem, sc, pl);
}

// ---- the packed pass for 12 markers (C3: BASELINE.json configs[2]; round 6).  The task loop,
// the motion model, the kept-set store and the wave partials are weigh_pk_body's; the likelihood runs over the
// markers in phases of PH (project2d, the grid's first entries, the rare longer lists, the score terms), so only one
// phase's projections, cell records and minima are live at a time: five markers' worth fit the 128-VGPR floor, twelve
// would not.  Every per-marker operation is the 5-marker pass's, hence k_weigh_stream's (column_minima's grid branch,
// score_unordered's terms, summed in marker order), so the weights, kept set and partials are k_weigh_stream's bit for
// bit (tests/test_gpu_weigh_pk.py).  Self-occlusion: each marker's key (its blob when accepted, 0x8000 + j otherwise;
// blob indices < kMaxBlobs = 1024) goes into a 16-bit half of one register per marker, A low, B high; a new marker's
// key is xored with each earlier one's and the result folded into a packed 16-bit minimum (v_pk_min_u16: both
// particles per instruction, no lane masks held on the scalar unit, where 66 pairs of ballots spilled), so a zero half
// at the end means two accepted markers on one blob, and the exact penalty count (score_unordered's) runs only in a
// wave where some lane has one.
#ifndef PFMPE_WEIGH_PK12_PHASE
#define PFMPE_WEIGH_PK12_PHASE 4
#endif
#ifndef PFMPE_WEIGH_PK12_FENCE
#define PFMPE_WEIGH_PK12_FENCE 1
#endif
constexpr int kPk12M = 12;
template <typename SP>
__device__ __forceinline__ void weigh_pk12_body(const FrameArgsT<float>& fa, const uint32_t* fa_words, int wg, int nwg,
                                                const unsigned char* __restrict__ table, const SP* __restrict__ prior,
                                                float* __restrict__ w0, float* __restrict__ w1,
                                                BlockPart* __restrict__ part0, BlockPart* __restrict__ part1,
                                                const Ctrl* __restrict__ ctrl, SP* __restrict__ prop0,
                                                SP* __restrict__ prop1, int iter, unsigned char* smem,
                                                LdsConst<float>& sc, PkLds& pl) {
  constexpr int MAXM = kPk12M, PH = PFMPE_WEIGH_PK12_PHASE;
  static_assert(MAXM % PH == 0, "whole phases");
  static_assert(kMaxBlobs <= 0x8000, "blob keys in 16 bits");
  if (ctrl->done) return;
  const int slot = ctrl->cur_slot;
  float* wout = slot ? w1 : w0;
  SP* pout = slot ? prop1 : prop0;
  BlockPart* parts = slot ? part1 : part0;
  const int lane = lane_id();
  const int ntask = 2 * fa.nblk;
  const int nwaves = nwg * kWaves;
  int tk = wg * kWaves + wave_id_u();
  copy_table(table, smem, (size_t)fa.tbytes);
  const uint32_t* own = fa.owner;
  auto rows_of = [&](int t, int& ra, int& rb) {
    const int n = in_planes(t * 128 + lane, fa.N), m = in_planes(t * 128 + 64 + lane, fa.N);
    ra = own ? (int)own[n] : n;
    rb = own ? (int)own[m] : m;
  };
  RawState<SP> Ra{}, Rb{};
  int rA, rB;
  rows_of(tk, rA, rB);
  load_state_prefetch<SP>(prior, fa.ld, rA, true, Ra);
  load_state_prefetch<SP>(prior, fa.ld, rB, true, Rb);
  rows_of(tk + nwaves, rA, rB);
  stage_consts_from(fa_words, sc);
  if (threadIdx.x < 12) {
    pl.anc_in[threadIdx.x] = fa.anc_in[threadIdx.x];
    pl.anc_out[threadIdx.x] = fa.anc_out[threadIdx.x];
  } else if (threadIdx.x == 12) {
    pl.inv_c = fa.grid.inv_c;
    pl.ox = fa.grid.ox;
    pl.oy = fa.grid.oy;
    pl.fmaxx = fa.grid.fmaxx;
    pl.fmaxy = fa.grid.fmaxy;
  }
  __syncthreads();
  const LdsBlobs<float> tb = view_table<float>(smem, fa.B);
  const GridArgs& ga = fa.grid;
  const unsigned char* cells = tb.base + ga.cell_off;
  const unsigned char* ents = tb.base + ga.ent_off;
  const bool predict = fa.it > 1 && (iter % 10) != 0;
  const float gsc = (float)(1.0 + fa.growth * (double)(iter / 10));
  const float tol = fa.tol, tol_pf = fa.tol_pf, Mt = (float)MAXM, rtol = rcp_t(fa.tol);
  for (; tk < ntask; tk += nwaves) {
    const int nA = tk * 128 + lane, nB = nA + 64;
    const bool vA = nA < fa.N, vB = nB < fa.N;
    // ---- motion model (weigh_pk_body's)
    const Phx2 ph = philox_motion_pair((uint32_t)nA, (uint32_t)nB, (uint32_t)iter | (kTagMotion << 24), fa.flo, fa.fhi,
                                       fa.key0, fa.key1);
    __builtin_amdgcn_sched_barrier(0);
    f32x2 A[12];
    decode2<SP>(Ra, Rb, pl.anc_in, A);
    const int64_t ldl = (int64_t)sopaque((uint32_t)fa.ld);
    load_state_prefetch<SP>(prior, ldl, rA, true, Ra);
    load_state_prefetch<SP>(prior, ldl, rB, true, Rb);
    rows_of(tk + 2 * nwaves, rA, rB);
    f32x2 d[6];
    {
      float fa6[6], fb6[6];
      draw_words(ph.a, fa6);
      draw_words(ph.b, fb6);
#pragma unroll
      for (int q = 0; q < 6; ++q) {
        const f32x2 v = f32x2{fa6[q], fb6[q]} - pk_splat(8388608.0f);
        d[q] = v * sc.rgs[q] + sc.lo[q];
      }
    }
    if (iter >= 10) {
      asm volatile("");
#pragma unroll
      for (int q = 0; q < 6; ++q) d[q] = d[q] * gsc;
    }
    if (predict) {
      f32x2 X[12];
#pragma unroll
      for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          f32x2 s = A[i * 4 + 0] * sc.predm[0 * 4 + j];
          s = pk_fma(A[i * 4 + 1], pk_splat(sc.predm[1 * 4 + j]), s);
          s = pk_fma(A[i * 4 + 2], pk_splat(sc.predm[2 * 4 + j]), s);
          if (j == 3) s = s + A[i * 4 + 3];
          X[i * 4 + j] = s;
        }
#pragma unroll
      for (int q = 0; q < 12; ++q) A[q] = X[q];
    }
    f32x2 sa, ca, sb, cb, sz, cz;
    {
      auto scs = [&](f32x2 x, f32x2& s, f32x2& c) {
        const f32x2 x2 = x * x;
        s = x * pk_fma(x2, pk_splat(-1.0f / 6.0f), pk_splat(1.0f));
        c = pk_fma(x2, pk_fma(x2, pk_splat(1.0f / 24.0f), pk_splat(-0.5f)), pk_splat(1.0f));
      };
      scs(d[0], sa, ca);
      scs(d[1], sb, cb);
      scs(d[2], sz, cz);
    }
    f32x2 P[12];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const f32x2 a0 = A[i * 4 + 0], a1 = A[i * 4 + 1], a2 = A[i * 4 + 2];
      const f32x2 z0 = pk_fma(a1, sz, a0 * cz);
      const f32x2 z1 = pk_fma(a1, cz, a0 * (-sz));
      const f32x2 y0 = pk_fma(a2, -sb, z0 * cb);
      const f32x2 y2 = pk_fma(a2, cb, z0 * sb);
      const f32x2 x1 = pk_fma(y2, sa, z1 * ca);
      const f32x2 x2 = pk_fma(y2, ca, z1 * (-sa));
      P[i * 4 + 0] = y0;
      P[i * 4 + 1] = x1;
      P[i * 4 + 2] = x2;
      P[i * 4 + 3] = A[i * 4 + 3] + d[3 + i];
    }
    if (tk == 0) {
#pragma unroll
      for (int q = 0; q < 12; ++q) P[q].x = lane == 0 ? sc.cur[q] : (lane == 1 ? sc.pred[q] : P[q].x);
    }
    if (prop0) {
      f32x2 D[12];
      if constexpr (std::is_same<SP, __half>::value) {
#pragma unroll
        for (int q = 0; q < 12; ++q) D[q] = P[q] - pk_splat(pl.anc_out[q]);
      }
      if (vA) store_kept<SP, 0>(pout, ldl, nA, P, D);
      if (vB) store_kept<SP, 1>(pout, ldl, nB, P, D);
    }
    // ---- project2d's Q = K * P (upper-triangular K), then the markers in phases
    f32x2 Q[12];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      Q[j] = pk_fma(pk_splat(sc.K[2]), P[8 + j], pk_fma(pk_splat(sc.K[1]), P[4 + j], P[j] * sc.K[0]));
      Q[4 + j] = pk_fma(pk_splat(sc.K[5]), P[8 + j], P[4 + j] * sc.K[4]);
      Q[8 + j] = P[8 + j];
    }
    f32x2 Pr = pk_splat(0.0f);
    typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
    uint32_t key[MAXM];     // marker j's dup keys, A in the low half, B in the high half
    u16x2 dmin = {0xffff, 0xffff};  // min over marker pairs of key[e] ^ key[j], per half
    bool nanA = false, nanB = false;  // marker 0's projection is NaN (Eigen's visitor at coeff(0, 0))
#pragma unroll
    for (int p0 = 0; p0 < MAXM; p0 += PH) {
      f32x2 u[PH], v[PH];
#pragma unroll
      for (int i = 0; i < PH; ++i) {
        const int j = p0 + i;
        const float X = sc.markers[3 * j], Y = sc.markers[3 * j + 1], Z = sc.markers[3 * j + 2];
        f32x2 su = Q[0] * X, sv = Q[4] * X, sz2 = Q[8] * X;
        su = pk_fma(Q[1], pk_splat(Y), su);
        sv = pk_fma(Q[5], pk_splat(Y), sv);
        sz2 = pk_fma(Q[9], pk_splat(Y), sz2);
        su = pk_fma(Q[2], pk_splat(Z), su);
        sv = pk_fma(Q[6], pk_splat(Z), sv);
        sz2 = pk_fma(Q[10], pk_splat(Z), sz2);
        su = su + Q[3];
        sv = sv + Q[7];
        sz2 = sz2 + Q[11];
        const f32x2 rz = f32x2{rcp_t(sz2.x), rcp_t(sz2.y)};
        u[i] = su * rz;
        v[i] = sv * rz;
      }
      if (p0 == 0) {
        nanA = __builtin_isunordered(u[0].x, v[0].x);
        nanB = __builtin_isunordered(u[0].y, v[0].y);
      }
      float mA[PH], mB[PH];
      int rA_[PH], rB_[PH];
      uint32_t recA[PH], recB[PH];
#pragma unroll
      for (int i = 0; i < PH; ++i) {
        const f32x2 fx = pk_fma(u[i], pk_splat(pl.inv_c), pk_splat(pl.ox));
        const f32x2 fy = pk_fma(v[i], pk_splat(pl.inv_c), pk_splat(pl.oy));
        recA[i] = grid_rec(cells, ga.ncx4, pl.fmaxx, pl.fmaxy, fx.x, fy.x);
        recB[i] = grid_rec(cells, ga.ncx4, pl.fmaxx, pl.fmaxy, fx.y, fy.y);
      }
      uint32_t lists = 0;
#pragma unroll
      for (int i = 0; i < PH; ++i) {
        const GridEnt eA = *(const GridEnt*)(ents + (recA[i] & 0xffffu));
        const GridEnt eB = *(const GridEnt*)(ents + (recB[i] & 0xffffu));
        const f32x2 dx = f32x2{eA.x, eB.x} - u[i];
        const f32x2 dy = f32x2{eA.y, eB.y} - v[i];
        const f32x2 dd = pk_fma(dx, dx, dy * dy);
        mA[i] = dd.x;
        mB[i] = dd.y;
        rA_[i] = eA.orig;
        rB_[i] = eB.orig;
        lists |= recA[i] | recB[i];
      }
      if (__builtin_amdgcn_ballot_w64(lists > 0x1ffffu)) {  // some lane has a longer list (wave-uniform)
#pragma unroll
        for (int i = 0; i < PH; ++i)
          if (__builtin_amdgcn_ballot_w64((recA[i] > 0x1ffffu) | (recB[i] > 0x1ffffu))) {
            // (one loop over both particles' entries measured slower: C3 weighing 56.5 -> 59.6 us)
            grid_walk(ents, recA[i], u[i].x, v[i].x, mA[i], rA_[i]);
            grid_walk(ents, recB[i], u[i].y, v[i].y, mB[i], rB_[i]);
          }
      }
      // the phase's score terms (score_unordered's, in marker order) and dup keys
#pragma unroll
      for (int i = 0; i < PH; ++i) {
        const int j = p0 + i;
        const f32x2 dj = f32x2{sqrt_t(mA[i]), sqrt_t(mB[i])};
        const bool accA = dj.x <= tol_pf, accB = dj.y <= tol_pf;
        const uint32_t kA = accA ? (uint32_t)rA_[i] : 0x8000u + (uint32_t)j;
        const uint32_t kB = accB ? (uint32_t)rB_[i] : 0x8000u + (uint32_t)j;
        key[j] = kA | (kB << 16);
        const f32x2 q = (pk_splat(tol) - dj) * rtol;
        const f32x2 t = pk_splat(Mt) + q * q;
        Pr = Pr + f32x2{accA ? t.x : 0.0f, accB ? t.y : 0.0f};
#pragma unroll
        for (int e = 0; e < j; ++e)
          dmin = __builtin_elementwise_min(dmin, __builtin_bit_cast(u16x2, key[e] ^ key[j]));
      }
#if PFMPE_WEIGH_PK12_FENCE
      __builtin_amdgcn_sched_barrier(0);  // one phase's registers at a time (the scheduler would interleave them)
#endif
    }
    const uint64_t anydup = __builtin_amdgcn_ballot_w64((dmin.x == 0) | (dmin.y == 0));
    float wA = Pr.x, wB = Pr.y;
    if (anydup || fa.downgrade) {  // rare (wave-uniform): score_unordered's penalty count
      asm volatile("");
      auto pen = [&](int sh) {
        int dups = 0, ndg = 0;
#pragma unroll
        for (int j = 0; j < MAXM; ++j) {
          const uint32_t kj = (key[j] >> sh) & 0xffffu;
          const bool acc = kj < 0x8000u;
          bool dup = false;
#pragma unroll
          for (int e = 0; e < j; ++e) dup |= (((key[e] >> sh) & 0xffffu) == kj);  // equal keys: both accepted
          dups += (acc & dup) ? 1 : 0;
          ndg += (acc && ((fa.downgrade >> j) & 1u)) ? 1 : 0;
        }
        return (float)(3 * dups * (dups + 1) / 2 + 2 * ndg);
      };
      wA = wA - pen(0);
      wB = wB - pen(16);
    }
    if (nanA) wA = 0.0f;
    if (nanB) wB = 0.0f;
    const bool full = (tk + 1) * 128 <= fa.N;
    if (full) {
      wout[nA] = wA;
      wout[nB] = wB;
    } else {
      if (!vA) wA = 0.0f;
      if (!vB) wB = 0.0f;
      if (vA) wout[nA] = wA;
      if (vB) wout[nB] = wB;
    }
    pk_wave_partial(wA, vA, full, tk * 128, parts + (size_t)tk * 2);
    pk_wave_partial(wB, vB, full, tk * 128 + 64, parts + (size_t)tk * 2 + 1);
  }
}

#ifndef PFMPE_WEIGH_PK12_MIN_WAVES
#define PFMPE_WEIGH_PK12_MIN_WAVES 3
#endif
template <typename SP>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(PFMPE_WEIGH_PK12_MIN_WAVES))) void k_weigh_pk12(
    const FrameArgsT<float> fa, const unsigned char* __restrict__ table, const SP* __restrict__ prior,
    float* __restrict__ w0, float* __restrict__ w1, BlockPart* __restrict__ part0, BlockPart* __restrict__ part1,
    const Ctrl* __restrict__ ctrl, SP* __restrict__ prop0, SP* __restrict__ prop1, int iter) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ LdsConst<float> sc;
  __shared__ PkLds pl;
  weigh_pk12_body<SP>(fa, (const uint32_t*)__builtin_amdgcn_kernarg_segment_ptr(), (int)blockIdx.x, (int)gridDim.x,
                      table, prior, w0, w1, part0, part1, ctrl, prop0, prop1, iter, smem, sc, pl);
}

// ---- batched streams (pfmpe_step_multi): the streaming packed pass for every stream of a batch in ONE launch.
// Grid (max wg, streams): workgroup (x, s) is workgroup x of the desc.wg resident workgroups the host gave stream
// s (its share of the device's resident capacity, in proportion to its particles), so a workgroup stages one
// stream's table and constants once and loops over that stream's tasks only: each stream computes exactly its
// one-stream k_weigh_pk.  A stream whose descriptor failed the staging check (status != gen) is skipped.
template <typename SP>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(PFMPE_WEIGH_PK_MIN_WAVES))) void k_weigh_pk_multi(
    const StreamDesc<float, SP>* __restrict__ descs, int S, const uint32_t* __restrict__ status, uint32_t gen,
    int iter) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ LdsConst<float> sc;
  __shared__ PkLds pl;
  const int s = (int)blockIdx.y;
  if (s >= S || __builtin_amdgcn_readfirstlane(status[s]) != gen) return;
  const StreamDesc<float, SP>& d = descs[s];
  const int nwg = __builtin_amdgcn_readfirstlane(d.wg);
  if ((int)blockIdx.x >= nwg) return;
  weigh_pk_body<SP, true>(d.fa, (const uint32_t*)&d.fa, (int)blockIdx.x, nwg, d.table, d.prior, d.w0, d.w1, d.part0,
                          d.part1, d.ctrl, d.prop0, d.prop1, iter, smem, sc, pl);
}

// ---- the batched streaming pass's group / top hand-off (k_group_top / k_group + k_top_wide / k_top of every
// stream of the batch, one launch each): grid (max groups, streams) for the group scans, (streams) for the tops.
// The bodies are the one-stream kernels' (same functions, same association), with the stream's frame arguments,
// buffers and counters from its descriptor; blocks past a stream's groups, and streams that failed the staging
// check, return at once.
template <typename T, int RNG, typename SP>
__global__ __launch_bounds__(64) void k_group_top_multi(const StreamDesc<T, SP>* __restrict__ descs, int S,
                                                        const uint32_t* __restrict__ status, uint32_t gen, int iter) {
  const int s = (int)blockIdx.y;
  if (s >= S || __builtin_amdgcn_readfirstlane(status[s]) != gen) return;
  const StreamDesc<T, SP>& d = descs[s];
  const int g = (int)blockIdx.x;
  const int ngrp = __builtin_amdgcn_readfirstlane(d.fa.ngrp);
  if (g >= ngrp) return;
  Ctrl* ctrl = d.ctrl;
  if (load_ctrl_word<(int)offsetof(Ctrl, done)>(ctrl)) return;  // every block reads ctrl before it arrives
  const int slot = load_ctrl_word<(int)offsetof(Ctrl, cur_slot)>(ctrl);
  const GroupPart gr = propagate_group<true>(__builtin_amdgcn_readfirstlane(d.fa.nblk), __builtin_amdgcn_readfirstlane(d.fa.gsz),
                                             g, slot ? d.part1 : d.part0, slot ? d.bscan1 : d.bscan0,
                                             slot ? d.gpart1 : d.gpart0);
  const bool single = ngrp == 1;
  if (!single && !wave_arrive_last(d.tcount_w, ngrp)) return;
  propagate_top<T, RNG>(d.fa, ctrl, iter, d.gpart0, d.gpart1, d.gscan, nullptr, 0u, gr, single, slot);
}
template <typename T, typename SP>
__global__ __launch_bounds__(64) void k_group_multi(const StreamDesc<T, SP>* __restrict__ descs, int S,
                                                    const uint32_t* __restrict__ status, uint32_t gen) {
  const int s = (int)blockIdx.y;
  if (s >= S || __builtin_amdgcn_readfirstlane(status[s]) != gen) return;
  const StreamDesc<T, SP>& d = descs[s];
  const int g = (int)blockIdx.x;
  if (g >= __builtin_amdgcn_readfirstlane(d.fa.ngrp)) return;
  if (load_ctrl_word<(int)offsetof(Ctrl, done)>(d.ctrl)) return;
  const int slot = load_ctrl_word<(int)offsetof(Ctrl, cur_slot)>(d.ctrl);
  (void)propagate_group<true>(__builtin_amdgcn_readfirstlane(d.fa.nblk), __builtin_amdgcn_readfirstlane(d.fa.gsz), g,
                              slot ? d.part1 : d.part0, slot ? d.bscan1 : d.bscan0, slot ? d.gpart1 : d.gpart0);
}
template <typename T, int RNG, typename SP>
__global__ __launch_bounds__(64 * kTopWaves) void k_top_wide_multi(const StreamDesc<T, SP>* __restrict__ descs, int S,
                                                                const uint32_t* __restrict__ status, uint32_t gen,
                                                                int iter) {
  extern __shared__ __attribute__((aligned(16))) GroupPart gsm[];  // the largest stream's ngrp entries
  __shared__ TopWideLds tw;
  const int s = (int)blockIdx.x;
  if (s >= S || __builtin_amdgcn_readfirstlane(status[s]) != gen) return;
  const StreamDesc<T, SP>& d = descs[s];
  top_wide_body<T, RNG>(d.fa, d.gpart0, d.gpart1, d.gscan, d.ctrl, iter, gsm, tw);
}
template <typename T, int RNG, typename SP>
__global__ __launch_bounds__(64) void k_top_multi(const StreamDesc<T, SP>* __restrict__ descs, int S,
                                                  const uint32_t* __restrict__ status, uint32_t gen, int iter) {
  const int s = (int)blockIdx.x;
  if (s >= S || __builtin_amdgcn_readfirstlane(status[s]) != gen) return;
  const StreamDesc<T, SP>& d = descs[s];
  top_body<T, RNG>(d.fa, d.gpart0, d.gpart1, d.gscan, d.ctrl, iter, 0, nullptr);
}

}  // namespace pfmpe
