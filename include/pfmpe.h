/*
 * pfmpe.h — C-ABI of the MI355X particle-filter pose engine (the drop-in boundary).
 *
 * The reference has no function/plugin boundary around its PF step: the step is ~200 inline lines in
 * PoseEstimator::estimateBodyPose (pf_mpe_lib/src/pose_estimator.cpp:475-733, "PE" below) sharing ~15
 * member fields (pf_mpe_lib/include/pf_mpe_lib/pose_estimator.h:65-169).  This header cuts it at the
 * PE:535 seam: the host keeps detection, prediction (predictPose PE:995), initialisation and Gauss-Newton
 * (PE:1805) and replaces PE:475-733 with one pfmpe_step() call.  Each entry point below cites the
 * reference state or code it replaces.  Plain C types only — no HIP/torch types cross the boundary.
 *
 * Conventions
 *   - Poses are 12 doubles: the top 3 rows of the homogeneous 4x4, row-major:
 *       [r00 r01 r02 t0  r10 r11 r12 t1  r20 r21 r22 t2]   (the Eigen::Matrix4d of the reference).
 *   - Blob coordinates are undistorted pixels (image_points_, PE:469 / led_detector.cpp:198-209), B x 2.
 *   - Return codes: 0 = OK, < 0 = error (PFMPE_E_*); pfmpe_last_error() gives text.  Algorithmic
 *     outcomes (accept / re-initialise) are NOT errors: see pfmpe_frame_out.flag_fail (reference codes).
 *   - A context is bound to one HIP device and one HIP stream and is not thread-safe; distinct contexts
 *     share nothing and may run concurrently (one per camera stream / tracked object / GPU).
 *   - pfmpe_step() is blocking: it returns after the frame's scalars and winner pose are on the host.
 *     The resampled particle set stays resident in HBM across frames (newPoseEstimation, PE:681).
 */
#ifndef PFMPE_H_
#define PFMPE_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PFMPE_ABI_VERSION 1
#define PFMPE_MAX_MARKERS 16   /* reference bMarkerDowngrade has 5 entries; we take per-marker flags */
#define PFMPE_MAX_BLOBS 1024

enum {
  PFMPE_OK = 0,
  PFMPE_E_ARG = -1,   /* bad argument / size                      */
  PFMPE_E_HIP = -2,   /* HIP runtime failure (device, alloc, launch) */
  PFMPE_E_CAP = -3,   /* exceeds the capacity given at create time  */
  PFMPE_E_STATE = -4  /* call order (e.g. step before set_model)    */
};

/* particle state storage in HBM (SoA planes).  F16: fp16 deltas to an anchor pose per particle set
 * (the frame's current pose for a resampled set, the first particle for pfmpe_set_prior), fp32 compute
 * and fp32 weights: 24 B per particle (BASELINE.json configs[3]), stored as 6 planes of fp16 pairs.  The
 * layout is internal: every entry point exchanges poses as 12 doubles per particle. */
enum { PFMPE_STATE_F32 = 0, PFMPE_STATE_F64 = 1, PFMPE_STATE_F16 = 2 };

/* motion / resample random streams */
enum {
  PFMPE_RNG_REFERENCE = 0, /* std::default_random_engine (minstd_rand0) stream of PE:476-477, 510-523,
                              reproduced on device by LCG jump-ahead: bit-identical draws */
  PFMPE_RNG_PHILOX = 1     /* counter-based Philox4x32-10 keyed by (seed, frame, iter, particle) */
};

/* flag_fail codes (pf_mpe/include/pf_mpe/monocular_pose_estimator.h:121-137, PE:635, PE:711) */
enum { PFMPE_FLAG_ACCEPTED = 1, PFMPE_FLAG_REINIT = 4 };

typedef struct pfmpe_ctx pfmpe_ctx;

/* PF parameters — the public fields of PoseEstimator (pose_estimator.h:121-155) that the PF block reads,
 * plus the constants the reference hard-codes (made explicit, defaults = reference values). */
typedef struct {
  double tol;        /* back_projection_pixel_tolerance_   score normaliser (PE:2416)           */
  double tol_pf;     /* back_projection_pixel_tolerance_PF acceptance gate (PE:2414)            */
  double ang_min;    /* minAngularNoise   (rad)                                                 */
  double ang_max;    /* maxAngularNoise   (rad)                                                 */
  double trans_min;  /* minTransitionNoise (m)                                                  */
  double trans_max;  /* maxTransitionNoise (m)                                                  */
  double growth;     /* 0.025: noise growth per 10 iterations (PE:563)                          */
  int32_t max_iter;  /* 80  (PE:616)                                                            */
  int32_t exit_cap;  /* 5   exit when max w >= M*min(exit_cap, B)   (PE:616)                    */
  int32_t accept_cap;/* 3   accept when best > M*min(accept_cap, B) (PE:633)                    */
  int32_t rng_mode;  /* PFMPE_RNG_*                                                             */
} pfmpe_params;

/* Per-frame host inputs */
typedef struct {
  double current_pose[12];   /* current_pose_   -> particle 0 (PE:547)                          */
  double predicted_pose[12]; /* camMoveInv * predicted_pose_ (PE:395) -> particle 1 (PE:551)    */
  double prediction[12];     /* predictionMatrix = predictPose() (PE:234, PE:995-1010)          */
  double cam_move_inv[12];   /* camMoveInv (identity unless bUseCamPos, PE:241-393)             */
  const double* blobs;       /* B x 2 undistorted px; host pointer (ignored if bank_frame >= 0)  */
  int32_t B;                 /* numLED (PE:449)                                                 */
  int32_t bank_frame;        /* -1: use `blobs`; >= 0: frame index in the device blob bank       */
  int32_t it_since_init;     /* it_since_initialized_ (1 right after init, 2 steady state)      */
  int32_t force_iters;       /* 0: reference exit rule; > 0: run exactly this many iterations   */
  double dt;                 /* predicted_time_ - current_time_ (PE:499)                        */
  uint64_t seed;             /* replaces std::random_device (PE:476); reference mode uses low 32 */
  uint64_t frame_idx;        /* Philox counter word                                             */
} pfmpe_frame_in;

/* Per-frame outputs: the scalars the host needs after PE:733 */
typedef struct {
  int32_t iters;            /* PF iterations executed (k)                                        */
  int32_t kept_iter;        /* iteration whose particle set was kept (PE:608-624)                */
  int32_t most_likely_idx;  /* mostLikelyParticleIdx (PE:610; PE:714 on the re-init branch)      */
  int32_t accepted;         /* probPartSum != 0 && highestProb > M*min(3,B)  (PE:633)            */
  int32_t resampled;        /* stratified resampling ran (PE:666-682); new prior is resident     */
  int32_t winner_idx;       /* argmax resample count (PE:685-686), -1 if not resampled           */
  int32_t n_corr;           /* rows of correspondences_ for the winner (PE:688)                  */
  int32_t flag_fail;        /* PFMPE_FLAG_ACCEPTED / PFMPE_FLAG_REINIT                           */
  double highest_prob;      /* highestProb                                                        */
  double prob_sum;          /* probPartSum = sum of kept raw weights (PE:627)                     */
  double winner_pose[12];   /* PoseParticle[winner] -> predicted_pose_ before GN (PE:687);
                               on re-init: PoseParticle[most_likely_idx] (PE:716)                */
  double most_likely_pose[12]; /* PoseParticle[most_likely_idx]                                  */
  uint32_t corr[2 * PFMPE_MAX_MARKERS]; /* (LED, blob) 1-based pairs, extraction order (PE:2417) */
} pfmpe_frame_out;

/* ---------------------------------------------------------------------------------- lifetime */
/* Replaces the PoseEstimator member state of pose_estimator.h:65-70 (PoseParticle, newPoseEstimation,
 * probPart) with device-resident SoA buffers sized for max_particles. */
int pfmpe_create(pfmpe_ctx** out, int hip_device, int max_particles, int max_markers, int max_blobs,
                 int state_dtype);
void pfmpe_destroy(pfmpe_ctx* ctx);
const char* pfmpe_last_error(const pfmpe_ctx* ctx);
int pfmpe_abi_version(void);

/* ----------------------------------------------------------------------------------- model/params */
/* object_points_ (PoseEstimator::setMarkerPositions PE:56), camera_matrix_K_ (3x3 row-major,
 * monocular_pose_estimator.cpp:215-238) and bMarkerDowngrade (monocular_pose_estimator.cpp:510-517,
 * here one flag per marker; NULL = none). */
int pfmpe_set_model(pfmpe_ctx* ctx, const double* markers_xyz, int M, const double* K,
                    const uint8_t* downgrade);
/* Fills the PF parameter fields (dynamicParametersCallback, monocular_pose_estimator.cpp:480-527). */
int pfmpe_set_params(pfmpe_ctx* ctx, const pfmpe_params* params);
void pfmpe_default_params(pfmpe_params* params);

/* Sets N = N_Particle and the prior newPoseEstimation (N x 12).  Called after (re)initialisation,
 * which seeds the particle set (PE:1429-1437, 1756-1760). */
int pfmpe_set_prior(pfmpe_ctx* ctx, const double* poses, int N);

/* ------------------------------------------------------------------------------------- the step */
/* One PF step = PE:475-690 (+ PE:707-719): propagate, project, weigh (iterating per PE:535-616),
 * normalise, accept, stratified-resample, pick the winner.  Blocking. */
int pfmpe_step(pfmpe_ctx* ctx, const pfmpe_frame_in* in, pfmpe_frame_out* out);

/* n consecutive frames of one stream, in order, each exactly as pfmpe_step (blocking on its own frame
 * record before the next frame is launched) — the loop a C/C++ tracker runs, without per-call FFI
 * overhead.  Stops at the first error; *done receives the number of frames completed. */
int pfmpe_step_batch(pfmpe_ctx* ctx, const pfmpe_frame_in* in, int n, pfmpe_frame_out* out, int* done);

/* One frame of each of S independent contexts (camera streams / tracked objects: the reference's
 * per-object loop, PE:89, with per-object state PE:113-114, 726-727) as ONE batch on the device: the S
 * weighing passes run as one launch, the S resampling passes as a second, the S frame records as a third
 * (plus iteration batches for streams whose exit rule does not fire at once).  in[s] / out[s] belong to
 * ctxs[s]; each context's outputs and state equal what pfmpe_step(ctxs[s], &in[s], &out[s]) gives.
 * All contexts must be distinct, on one device, of one state type, RNG mode and pruning option; the batch
 * runs on ctxs[0]'s HIP stream and uses ctxs[0]'s batch scratch.  Work a member context has pending on
 * its own stream (an earlier pfmpe_step, ...) is ordered before the batch, and the member's next work on
 * its own stream after it (events, only when the streams differ).  Blocking.  At most
 * PFMPE_OPT_MULTI_MAX_BLOCKS (of ctxs[0]) 256-particle blocks per batch, in all: 160000 (~41M particles).
 * Errors (nothing launched): PFMPE_E_ARG for a mismatch, the failing stream's own pfmpe_step code
 * (E_ARG / E_CAP / E_STATE) for a bad frame, PFMPE_E_CAP above the block limit; the text, prefixed with
 * the stream index, in pfmpe_last_error(ctxs[0]).  With PFMPE_OPT_TIMING set on ctxs[0] the batch's
 * launches are timed into ctxs[0]'s kernel statistics (weighing, resampling, finishing, staging = aux). */
int pfmpe_step_multi(pfmpe_ctx* const* ctxs, int S, const pfmpe_frame_in* in, pfmpe_frame_out* out);

/* n consecutive batches of pfmpe_step_multi (in / out: n x S, batch-major), each blocking on its records
 * before the next is launched — the loop a multi-object C/C++ tracker runs, without per-call FFI overhead.
 * Stops at the first error; *done receives the number of batches completed. */
int pfmpe_step_multi_batch(pfmpe_ctx* const* ctxs, int S, const pfmpe_frame_in* in, int n, pfmpe_frame_out* out,
                           int* done);

/* ---------------------------------------------------------------------- ROI prediction (§8f row 1) */
/* predictMarkerPositionsInImage (PE:1036-1053) + LEDDetector::determineROI (led_detector.cpp:217-369),
 * as called at PE:396-412: every marker projected through camMoveInv * prior_j * predictionMatrix for all
 * N particles of the current prior, plus the markers at predicted_pose_; the bounding box (x_min/y_min
 * from +inf, x_max/y_max from 0); its corners as cv::Point2f through distortPoints (plumb_bob D, in
 * double); border, clamp to the image, integer cv::Rect (the whole image when narrower than 1 px).
 * Call it before pfmpe_step of the same frame (the prior is the resampled set of the previous one). */
typedef struct {
  double cam_move_inv[12];   /* camMoveInv (PE:241-393)                                          */
  double prediction[12];     /* predictionMatrix (PE:234)                                        */
  double predicted_pose[12]; /* predicted_pose_ (PE:1051)                                        */
  double D[5];               /* camera_distortion_coeffs_ k1 k2 p1 p2 k3 (led_detector.cpp:380)  */
  int32_t image_w, image_h;  /* image.size()                                                     */
  int32_t border;            /* roi_border_thickness_                                            */
  int32_t pad;
} pfmpe_roi_in;
typedef struct {
  int32_t x, y, width, height; /* region_of_interest_ (cv::Rect)                                 */
  double bbox[4];              /* undistorted x_min, x_max, y_min, y_max of the projections       */
} pfmpe_roi_out;
int pfmpe_predict_roi(pfmpe_ctx* ctx, const pfmpe_roi_in* in, pfmpe_roi_out* out);

/* ------------------------------------------------- brute-force P3P (re)initialisation (§8f row 2) */
/* PoseEstimator::initialise (PE:1503-1786) for the particle-filter configuration, run when the track is
 * lost (it_since_initialized_ < 1, PE:128-205).  Blobs are image_points_ (undistorted px).  Stages:
 *   1. histogram (PE:1526-1716, device): for every 3-blob combination passing the spread filter
 *      (threshDist, >= 5 blobs near the centroid) x every ordered 3-marker permutation, P3P
 *      (p3p.cpp:65-292) gives 4 poses; each finite, non-repeated pose back-projects the unused markers
 *      through H.inverse() and, when at least one unused blob lies within tol of its nearest projection,
 *      the 3 P3P pairs and every such (blob, nearest marker) pair are counted;
 *   2. candidate correspondence vectors (correspondencesFromHistogram PE:1134-1288, host);
 *   3. checkCorrespondences of every candidate (PE:1312-1501; P3P over each 3-subset, device), the
 *      particle seeding and the fill loop (PE:1429-1437, 1755-1760), predicted_pose_ by
 *      computeTransformation (PE:2139-2161, host) for the first match.
 * tol = the context's params.tol (back_projection_pixel_tolerance_, shared with the PF score). */
typedef struct {
  double certainty_threshold;  /* certainty_threshold_ (PE:1411), README default 1                    */
  double valid_corr_threshold; /* valid_correspondence_threshold_ (PE:1477), README default 0.5        */
  int32_t n_particles;         /* N_Particle; 0 = the context's current N (max_particles if none)      */
  int32_t max_candidates;      /* cap on correspondence vectors (PFMPE_E_CAP beyond it); default 2^20  */
} pfmpe_init_params;
typedef struct {
  int32_t found;            /* initialise() == 1; the particle set is then seeded (see below)       */
  int32_t flag_fail;        /* 0 when found, else the last PubData.Flag_Fail code initialise wrote:
                               10 too few blobs, 12 empty histogram, 11 no candidate, 6 too few
                               correspondences, 9 P3P failed, 7 / 8 validity ratio; -1 none          */
  int32_t n_estimates;      /* P3P poses stored into PoseParticle (NumberOfP3PEstimation - 1)        */
  int32_t n_candidates;     /* correspondence vectors from the histogram                            */
  int32_t first_match;      /* candidate giving correspondences_ / predicted_pose_ (-1: none)      */
  int32_t n_corr;           /* rows of correspondences_                                             */
  uint32_t corr[2 * PFMPE_MAX_MARKERS]; /* (LED, blob) 1-based pairs                                 */
  double predicted_pose[12];/* predicted_pose_ (computeTransformation of the mean re-projections)   */
  uint64_t hist_total;      /* sum of the histogram                                                 */
} pfmpe_init_out;
void pfmpe_default_init_params(pfmpe_init_params* p);
/* Stage 1 alone: hist (B x M uint32, row-major: hist[blob * M + marker]).  3 <= B <= max_blobs. */
int pfmpe_p3p_histogram(pfmpe_ctx* ctx, const double* blobs, int B, uint32_t* hist);
/* The whole initialise().  On success (out->found) the context's particle set becomes PoseParticle
 * (newPoseEstimation_Vec = PoseParticle, PE:191): slot N-k holds the k-th stored P3P pose (k = 1..K),
 * slots below repeat them with period K (the fill loop), and slot 0 keeps the resident set's slot 0
 * (identity if there is none) unless K >= N.  hist (optional, B x M) receives stage 1's histogram. */
int pfmpe_initialise(pfmpe_ctx* ctx, const double* blobs, int B, const pfmpe_init_params* params,
                     pfmpe_init_out* out, uint32_t* hist);

/* ---------------------------------------------------------------- LED detector (§8f row 4) */
/* LEDDetector::findLeds (pf_mpe_lib/src/led_detector.cpp:46-215) on the device for one ROI of an 8-bit
 * grey image: threshold (THRESH_TOZERO for active markers, else THRESH_BINARY_INV), GaussianBlur (ksize
 * from sigma, OpenCV 2.4's 8-bit integer separable path, reflect-101), findContours(RETR_EXTERNAL,
 * CHAIN_APPROX_NONE) with 2.4's zeroed 1-pixel frame, contourArea / boundingRect / moments, the blob
 * size-aspect-circularity filter, the centre + ROI offset (cv::Point2f) and undistortPoints(K, D, P = K).
 * K is the context's model K.  Output: image_points_ (undistorted px, findContours order) and the
 * distorted centres (distorted_detection_centers_).  image = NULL uses the staged image. */
typedef struct {
  int32_t threshold_value;          /* detection_threshold_value_ (threshold_value, README default 240) */
  int32_t active_markers;           /* 1: THRESH_TOZERO, 0: THRESH_BINARY_INV (LD:56-59)               */
  double gaussian_sigma;            /* gaussian_sigma_ (0.6), in (0, 5]                               */
  double min_blob_area;             /* min_blob_area_ (the tracker's adapted value, PE:432-435)       */
  double max_blob_area;             /* max_blob_area_                                                 */
  double max_width_height_distortion; /* 0.7                                                          */
  double max_circular_distortion;   /* 0.7                                                            */
  double D[5];                      /* camera_distortion_coeffs_ k1 k2 p1 p2 k3                       */
  int32_t roi_x, roi_y, roi_w, roi_h; /* region_of_interest_; roi_w / roi_h < 0 = the whole image   */
} pfmpe_detect_params;
typedef struct {
  int32_t n;                        /* detections (all of them; min(n, max_out) written)              */
  int32_t n_components;             /* 8-connected components (contours) examined                     */
  int32_t overflow;                 /* more than 8192 components: the rest were not examined          */
  int32_t pad;
} pfmpe_detect_out;
void pfmpe_default_detect_params(pfmpe_detect_params* p);
int pfmpe_stage_image(pfmpe_ctx* ctx, const uint8_t* image, int width, int height, int pitch);
int pfmpe_find_leds(pfmpe_ctx* ctx, const uint8_t* image, int width, int height, int pitch,
                    const pfmpe_detect_params* params, double* blobs, float* distorted, int max_out,
                    pfmpe_detect_out* out);

/* ---------------------------------------- configuration files and recorded streams (§8f row 3) */
/* Host-only (no GPU): pfmpe_io.cpp.  The reference reads these through ROS (rosparam / getParam /
 * dynamic_reconfigure, pf_mpe/src/monocular_pose_estimator.cpp:81-126, 479-527) and the CameraInfo topic.
 * Marker YAML (README.md:95-117): `marker_positions:` followed by a list of {x, y, z} maps (block or flow
 * style).  Writes min(count, max_markers) rows of xyz; returns the number of markers, or < 0. */
int pfmpe_parse_marker_yaml(const char* text, double* xyz, int max_markers);
/* The PF / initialisation / marker-split parameters of a ROS launch file (<param name=.. value=../>,
 * pf_mpe/launch/<name>.launch): the names dynamicParametersCallback copies into PoseEstimator.  Absent names
 * keep the defaults of pfmpe_default_launch_config (the engine's defaults).  Returns how many names
 * were recognised. */
typedef struct {
  pfmpe_params pf;                       /* back_projection_pixel_tolerance(_PF), min/maxAngularNoise,
                                            min/maxTransitionNoise                                       */
  pfmpe_init_params init;                /* certainty_threshold, valid_correspondence_threshold, N_Particle */
  int32_t num_objects;                   /* numUAV                                                       */
  int32_t markers_per_object[4];         /* numberOfMarkersUAV1..4: split of the marker list per object  */
  int32_t use_particle_filter;           /* bUseParticleFilter                                           */
  uint8_t downgrade[PFMPE_MAX_MARKERS];  /* bMarkerNr1..5 -> bMarkerDowngrade                           */
} pfmpe_launch_config;
void pfmpe_default_launch_config(pfmpe_launch_config* cfg);
int pfmpe_parse_launch(const char* text, pfmpe_launch_config* cfg);
/* sensor_msgs/CameraInfo as echoed in README.md:127-143: K (9, row-major), D (plumb_bob k1 k2 p1 p2 k3),
 * width, height (any pointer may be NULL).  Returns a bit mask of what was found (1 K, 2 D, 4 width,
 * 8 height) or < 0 on a malformed K / D list. */
int pfmpe_parse_camera_info(const char* text, double* K, double* D, int32_t* width, int32_t* height);
/* Recorded detection streams (image_points_ per frame, undistorted px), little-endian binary:
 *   header "PFMB" | u32 version = 1 | u32 n_frames | u32 reserved
 *   frame  f64 timestamp | u32 B | u32 flags = 0 | B x {f64 x, f64 y}
 * offsets: n_frames + 1 prefix offsets into blobs (rows), as pfmpe_stage_blob_bank.  read: call with
 * NULL buffers to get n_frames / n_blobs; PFMPE_E_CAP if the buffers are too small. */
int pfmpe_write_blob_stream(const char* path, const double* timestamps, const double* blobs, const int32_t* offsets,
                            int n_frames);
int pfmpe_read_blob_stream(const char* path, double* timestamps, double* blobs, int32_t* offsets, int max_frames,
                           int64_t max_blobs, int* n_frames, int64_t* n_blobs);
/* Reads a stream file and stages every frame in the context's device blob bank (bank_frame = index). */
int pfmpe_stage_blob_stream(pfmpe_ctx* ctx, const char* path, int* n_frames);

/* getPoseParticles (PE:917, which = 0: kept propagated set of the last step) and getResampledParticles
 * (PE:923, which = 1: current prior).  N x 12 doubles. */
int pfmpe_get_particles(pfmpe_ctx* ctx, int which, double* out);
/* probPart of the last step: the kept iteration's raw (un-normalised) weights, N doubles. */
int pfmpe_get_weights(pfmpe_ctx* ctx, double* out);
/* counterMeas of the last step (PE:524, 678): N uint32; requires PFMPE_OPT_RECORD_COUNTS. */
int pfmpe_get_counts(pfmpe_ctx* ctx, uint32_t* out);

/* Engine options (value semantics in brackets; defaults first):
 *   PFMPE_OPT_RECORD_COUNTS [0|1]  keep counterMeas on device for pfmpe_get_counts
 *   PFMPE_OPT_PRUNE         [1|0]  exact x-window blob pruning in the likelihood (0 = scan all B blobs)
 *   PFMPE_OPT_TIMING        [0|P]  bracket the kernel launches of every P-th frame with HIP events
 *                                  (pfmpe_get_kernel_stats); P = 1 times every frame, 0 is off
 *   PFMPE_OPT_FUSED         [2|1|0] run a frame as ONE launch whenever all its blocks fit on the device
 *                                  at once: 2 (default) k_frame2 with flat hand-offs (every block reduces
 *                                  all block partials itself; <= 512 blocks), 1 k_frame with tree
 *                                  hand-offs; 0 forces the two-launch path (k_propagate_weigh + k_resample)
 *   PFMPE_OPT_KEEP_PROPAGATED [1|0] two-launch path: k_propagate_weigh stores each iteration's propagated
 *                                  set (two extra state buffers, allocated on first use) and k_resample
 *                                  gathers from it; 0 regenerates the kept set in k_resample instead.
 *                                  Results are bit-identical either way.  Default 1; batched frames
 *                                  (pfmpe_step_multi) use the stored set for fp16 state only (measured)
 *   PFMPE_OPT_WAIT_BOUND_US [2000000|>=1] bound of every in-launch wait of a one-launch frame.  A frame whose
 *                                  blocks are not all resident (other work holding CUs) is abandoned at the
 *                                  bound, redone with two launches (same result) and one-launch frames are
 *                                  switched off on this context (PFMPE_INFO_FUSED_FALLBACKS counts it;
 *                                  pfmpe_last_error describes it, the step still returns PFMPE_OK)
 *   PFMPE_OPT_FUSED_REARM   [0|n]  after such a fallback, switch one-launch frames back on after n clean
 *                                  two-launch frames (0: stay off)
 *   PFMPE_OPT_MULTI_MAX_BLOCKS [160000|1..160000] largest pfmpe_step_multi batch this context leads, in
 *                                  256-particle blocks (PFMPE_E_CAP above); the default is the tested limit
 *   PFMPE_OPT_DEFER_RESAMPLE [1|0] two-launch frames with the kept propagated set: resampling writes each
 *                                  slot's owner index (4 B) instead of gathering and scattering the particle,
 *                                  and the next frame reads the prior through those indices.
 *                                  Results are bit-identical either way (pfmpe_get_particles gathers)
 * Within one process at most one one-launch frame runs per device at a time: a context that finds another
 * context's one-launch frame in flight on its device runs that frame as two launches (PFMPE_INFO_GUARD_SKIPS). */
enum { PFMPE_OPT_RECORD_COUNTS = 1, PFMPE_OPT_PRUNE = 2, PFMPE_OPT_TIMING = 3, PFMPE_OPT_FUSED = 4,
       PFMPE_OPT_KEEP_PROPAGATED = 5, PFMPE_OPT_WAIT_BOUND_US = 6, PFMPE_OPT_FUSED_REARM = 7,
       PFMPE_OPT_MULTI_MAX_BLOCKS = 8, PFMPE_OPT_DEFER_RESAMPLE = 9 };
int pfmpe_set_option(pfmpe_ctx* ctx, int option, int64_t value);

/* Context state for monitoring and tests (no reference counterpart: engine introspection). */
enum { PFMPE_SHAPE_TWO_LAUNCH = 0, /* weighing pass (+ re-launches) + hand-off + resampling (+ final)   */
       PFMPE_SHAPE_FRAME = 1,      /* k_frame: one launch, tree hand-offs                                */
       PFMPE_SHAPE_FRAME2 = 2 };   /* k_frame2: one launch, flat hand-offs                               */
enum { PFMPE_INFO_FUSED = 1,            /* current one-launch mode (0/1/2; 0 after a fallback)       */
       PFMPE_INFO_FUSED_FALLBACKS = 2,  /* one-launch frames abandoned at the wait bound and redone  */
       PFMPE_INFO_LAST_SHAPE = 3,       /* PFMPE_SHAPE_* of the last step (-1 before the first)      */
       PFMPE_INFO_GUARD_SKIPS = 4,      /* frames run as two launches because another was in flight  */
       PFMPE_INFO_N = 5,                /* current particle count                                    */
       PFMPE_INFO_LAST_WEIGH_PASS = 6,  /* PFMPE_WEIGH_* of the last two-launch weighing (-1: none)  */
       PFMPE_INFO_LAST_GRID = 7,        /* 1: the last frame's blob table searched its cell grid; 0: the
                                         * x-buckets (no grid for this table or its window; fp64)    */
       PFMPE_INFO_LAST_RESAMPLE = 8 };  /* PFMPE_RESAMPLE_* of the last two-launch resampling (-1: none) */
/* The two-launch shape's weighing pass: one block per 256 particles (k_propagate_weigh), or
 * resident blocks streaming over them with the next block's state prefetched (k_weigh_stream + k_group +
 * k_top), or the streaming pass with two particles per lane in packed fp32 (k_weigh_pk: 5 markers, fp32 / fp16
 * state; k_weigh_pk12: 12 markers, fp32 state; the Philox stream, the blob grid).  All give bit-identical
 * results. */
enum { PFMPE_WEIGH_BLOCKS = 0, PFMPE_WEIGH_STREAM = 1, PFMPE_WEIGH_PK = 2 };
/* The two-launch shape's resampling launch: one block per 256 particles with the new prior materialised
 * (k_resample, then k_resample_final), or, for a deferred frame, one wave per 256-particle block writing owner
 * indices whose last wave finishes the frame (k_resample_owners).  Same outputs. */
enum { PFMPE_RESAMPLE_BLOCKS = 0, PFMPE_RESAMPLE_OWNERS = 1 };
int pfmpe_get_info(const pfmpe_ctx* ctx, int key, int64_t* value);

/* ----------------------------------------------------------------------- device-resident inputs */
/* Stages a bank of frames' blob lists in HBM (frame f = blobs[offsets[f] .. offsets[f+1]) rows), so a
 * caller replaying recorded detections (or the benchmark) passes bank_frame instead of host pointers. */
int pfmpe_stage_blob_bank(pfmpe_ctx* ctx, const double* blobs, const int32_t* offsets, int nframes);

/* ------------------------------------------------------------------------------ instrumentation */
/* Per-kernel statistics collected while PFMPE_OPT_TIMING is on: launches and summed device time (ms)
 * measured with HIP events on the ctx stream. */
enum { PFMPE_K_PROPAGATE = 0, /* k_propagate_weigh (+ last-block iteration reduce)  */
       PFMPE_K_RESAMPLE = 1,  /* k_resample / k_resample_owners: resampling           */
       PFMPE_K_AUX = 2,       /* hand-off kernels (k_group*, k_top*), regeneration   */
       PFMPE_K_FRAME = 3,     /* k_frame: the whole frame in one launch              */
       PFMPE_K_ROI = 4,       /* k_roi + k_roi_final (pfmpe_predict_roi)             */
       PFMPE_K_FINAL = 5,     /* k_resample_final (non-deferred frames): the record   */
       PFMPE_K_P3P_HIST = 6,  /* k_p3p_hist: initialisation histogram                */
       PFMPE_K_P3P_CHECK = 7, /* k_p3p_check: checkCorrespondences of all candidates */
       PFMPE_K_DETECT = 8,    /* k_det_*: the LED detector pipeline (pfmpe_find_leds) */
       PFMPE_K_COUNT = 9 };
int pfmpe_get_kernel_stats(pfmpe_ctx* ctx, int kernel, int64_t* launches, double* total_ms);
int pfmpe_reset_kernel_stats(pfmpe_ctx* ctx);
const char* pfmpe_kernel_name(int kernel);

/* ------------------------------------------------------------------------------ host-side checks */
/* Pure host functions (no GPU needed): they evaluate the same __host__ __device__ code the kernels use,
 * so CPU tests can pin RNG/geometry semantics against the oracle without a GPU. */
/* j-th (0-based) uniform_real_distribution<double>(a,b) draw of a default_random_engine(seed) */
double pfmpe_host_ref_uniform(uint32_t seed, uint64_t j, double a, double b);
void pfmpe_host_philox(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);

#ifdef __cplusplus
}
#endif
#endif /* PFMPE_H_ */
