// capi_caller.cpp — a C++11 host that makes exactly the calls of INTEGRATION.md §3-5 (the reference-side
// binding that replaces pose_estimator.cpp:475-733) through include/pfmpe.h, with no HIP or torch headers.
// Built by __graft_entry__.build(); run by tests/test_gpu_capi_caller.py, which writes the inputs, runs this
// program on the GPU and compares its outputs with the oracle.
//
// usage: capi_caller <inputs.bin> <outputs.bin> <state: 0 f32 | 1 f64 | 2 f16> <rng: 0 reference | 1 philox>
// inputs (float64 little-endian): M N F, markers M x 3, K 9, prior N x 12, then per frame:
//   B dt seed it_since_init, current_pose 12, predicted_pose 12, prediction 12, blobs B x 2
// outputs (float64): per frame 8 scalars {iters kept_iter most_likely_idx accepted winner_idx n_corr flag_fail
//   resampled}, highest_prob, prob_sum, winner_pose 12, most_likely_pose 12, corr 32; then the propagated set
//   of the last frame (N x 12, getPoseParticles) and the resampled set (N x 12, getResampledParticles).
#include <pfmpe.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

static bool rd(FILE* f, double* p, size_t n) { return fread(p, sizeof(double), n, f) == n; }

int main(int argc, char** argv) {
  if (argc != 5) {
    fprintf(stderr, "usage: %s in.bin out.bin state rng\n", argv[0]);
    return 2;
  }
  FILE* fi = fopen(argv[1], "rb");
  FILE* fo = fopen(argv[2], "wb");
  if (!fi || !fo) return 2;
  const int state = atoi(argv[3]), rng = atoi(argv[4]);
  double hdr[3];
  if (!rd(fi, hdr, 3)) return 3;
  const int M = (int)hdr[0], N = (int)hdr[1], F = (int)hdr[2];
  std::vector<double> xyz(3 * M), prior(12 * (size_t)N);
  double K[9];
  if (!rd(fi, xyz.data(), xyz.size()) || !rd(fi, K, 9) || !rd(fi, prior.data(), prior.size())) return 3;

  // §3: model and parameters
  pfmpe_ctx* ctx = nullptr;
  if (pfmpe_create(&ctx, /*hip_device*/ 0, N, M, /*max_blobs*/ 1024, state) != PFMPE_OK) {
    fprintf(stderr, "pfmpe_create failed\n");
    return 4;
  }
  uint8_t dg[16] = {0};
  if (pfmpe_set_model(ctx, xyz.data(), M, K, dg) != PFMPE_OK) return 5;
  pfmpe_params p;
  pfmpe_default_params(&p);
  p.rng_mode = rng;
  if (pfmpe_set_params(ctx, &p) != PFMPE_OK) return 5;
  // §4: seeding the particle set
  if (pfmpe_set_prior(ctx, prior.data(), N) != PFMPE_OK) return 5;

  // §5: the replaced block, once per frame
  for (int f = 0; f < F; ++f) {
    double fh[4];
    if (!rd(fi, fh, 4)) return 3;
    const int B = (int)fh[0];
    pfmpe_frame_in in;
    if (!rd(fi, in.current_pose, 12) || !rd(fi, in.predicted_pose, 12) || !rd(fi, in.prediction, 12)) return 3;
    std::vector<double> blobs(2 * (size_t)B + 2);
    if (!rd(fi, blobs.data(), 2 * (size_t)B)) return 3;
    for (int q = 0; q < 12; ++q) in.cam_move_inv[q] = (q == 0 || q == 5 || q == 10) ? 1.0 : 0.0;
    in.blobs = blobs.data();
    in.B = B;
    in.bank_frame = -1;
    in.it_since_init = (int)fh[3];
    in.force_iters = 0;
    in.dt = fh[1];
    in.seed = (uint64_t)fh[2];
    in.frame_idx = (uint64_t)f;
    pfmpe_frame_out out;
    if (pfmpe_step(ctx, &in, &out) != PFMPE_OK) {
      fprintf(stderr, "pfmpe_step: %s\n", pfmpe_last_error(ctx));
      return 6;
    }
    const double s[8] = {(double)out.iters, (double)out.kept_iter, (double)out.most_likely_idx, (double)out.accepted,
                         (double)out.winner_idx, (double)out.n_corr, (double)out.flag_fail, (double)out.resampled};
    double corr[2 * PFMPE_MAX_MARKERS];
    for (int k = 0; k < 2 * PFMPE_MAX_MARKERS; ++k) corr[k] = out.corr[k];
    fwrite(s, sizeof(double), 8, fo);
    fwrite(&out.highest_prob, sizeof(double), 1, fo);
    fwrite(&out.prob_sum, sizeof(double), 1, fo);
    fwrite(out.winner_pose, sizeof(double), 12, fo);
    fwrite(out.most_likely_pose, sizeof(double), 12, fo);
    fwrite(corr, sizeof(double), 2 * PFMPE_MAX_MARKERS, fo);
  }
  // getPoseParticles / getResampledParticles (PE:917-927)
  std::vector<double> buf(12 * (size_t)N);
  for (int which = 0; which < 2; ++which) {
    if (pfmpe_get_particles(ctx, which, buf.data()) != PFMPE_OK) return 7;
    fwrite(buf.data(), sizeof(double), buf.size(), fo);
  }
  pfmpe_destroy(ctx);
  fclose(fo);
  fclose(fi);
  return 0;
}
