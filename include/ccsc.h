/*
 * ccsc.h -- C-ABI of libccsc, the MI355X (gfx950) consensus-ADMM convolutional
 * sparse coding engine.  Drop-in boundary for the four learners of the CCSC
 * reference (paths relative to the reference repository):
 *
 *   admm_learn_conv2D_large_dParallel   2D/admm_learn_conv2D_large_dParallel.m:1-4
 *   admm_learn_conv2D_large_dzParallel  2D/admm_learn_conv2D_large_dzParallel.m:1-4
 *   admm_learn_conv3D_large             3D/admm_learn_conv3D_large.m:1-4
 *   admm_learn_conv4D_lightfield        4D/admm_learn_conv4D_lightfield.m:1-4
 *   admm_learn (2-3D hyperspectral)     2-3D/DictionaryLearning/admm_learn.m:1-4
 *
 * Each MATLAB function above becomes a thin .m wrapper over a MEX gateway that
 * calls ccsc_learn(); the Python mirror in
 * ccsc_code_iccv2017_amd/learners.py binds the same entry points via ctypes.
 *
 * Conventions
 *  - Plain pointers and sizes only.  Every host array is MATLAB column-major
 *    (first index fastest), float64, caller-owned; the library never retains a
 *    host pointer past return.  Output pointers are nullable: a NULL output is
 *    not computed/copied (z_res at the 10^4-patch config is ~97 GB).
 *  - Every function returns 0 on success or a negative CCSC_E* code; when
 *    `err` is non-NULL a NUL-terminated message (<= errlen bytes) says why.
 *    No C++ exception crosses the ABI.
 *  - Calls on one context come from one thread (MATLAB's / Python's).  The
 *    progress callback runs on that calling thread only.
 *  - Multi-GPU, one process per GPU (bench, MPI/torch jobs): rank 0 calls ccsc_get_unique_id(); the
 *    caller ships the 128 bytes to every rank (torch.distributed / MPI / file)
 *    and each rank calls ccsc_create(device, rank, nranks, uid).  Blocks of
 *    `ni` patches are sharded contiguously over ranks (ccsc_shard); the
 *    consensus mean of the reference (dP:114-121) becomes one RCCL all-reduce
 *    per d-iteration, the z-step's use of block 1's filters (dP:143) one RCCL
 *    broadcast per outer iteration.
 *  - Multi-GPU, one process (the MATLAB drop-in): ccsc_create_multi(devices, ndev)
 *    and one ccsc_learn call over the whole problem; same sharding and exchanges.
 */
#ifndef CCSC_H_
#define CCSC_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CCSC_ABI_VERSION 7

/* status codes */
#define CCSC_OK 0
#define CCSC_E_INVALID (-1)    /* bad argument / shape (e.g. n % ni != 0, Q13) */
#define CCSC_E_HIP (-2)        /* HIP runtime error                            */
#define CCSC_E_RCCL (-3)       /* RCCL error                                   */
#define CCSC_E_NOMEM (-4)      /* device memory plan exceeds the GPU           */
#define CCSC_E_UNSUPPORTED (-5)/* valid reference input not supported yet      */
#define CCSC_E_STATE (-6)      /* call out of order                            */

/* learner variants */
#define CCSC_DPAR 0  /* 2D dParallel   dP:1-199  */
#define CCSC_DZPAR 1 /* 2D dzParallel  dZ:1-206  */
#define CCSC_L3D 2   /* 3D             L3:1-230  */
#define CCSC_L4D 3   /* 4D light field L4:1-212  */
#define CCSC_HS23 4  /* 2-3D hyperspectral admm_learn L23:1-237 (ccsc_learn_hs23)  */

/* verbose: which objectives the reference evaluates (dP:50-60,126,161) */
#define CCSC_VERBOSE_NONE 0
#define CCSC_VERBOSE_BRIEF 1
#define CCSC_VERBOSE_ALL 2

/* arithmetic and storage precision: double only, as the reference computes (MATLAB
 * double; the 4D driver's single-precision b, learn_kernels_4D_extract_patches.m:46,
 * is widened on input).  A reduced-precision storage mode was declared in earlier
 * rounds and never built.  ABI 7 keeps its value as a deprecated name so callers built
 * against ABI <= 6 still compile; requesting it returns CCSC_E_UNSUPPORTED. */
#define CCSC_FP64 0
#define CCSC_FP32 1 /* deprecated (ABI <= 6): always CCSC_E_UNSUPPORTED */

/* form of the per-frequency D-step factor (precompute_H_hat_D, dP:221-237).
 * AUTO: Woodbury when blocks hold few patches (ni <= 8 and 4 ni <= K), else the
 * K x K Cholesky of A^H A + rho I.  The Woodbury solve (I - A^H M^-1 A) / rho,
 * M = rho I + A A^H, is the reference's own pinv form; it loses digits when
 * ||A||^2 >> rho, so CHOLESKY forces the better-conditioned K x K factor.
 * WOODBURY forces the ni x ni form (ni <= 8, ni K + ni^2 <= K (K + 1) / 2). */
#define CCSC_DFACTOR_AUTO 0
#define CCSC_DFACTOR_CHOLESKY 1
#define CCSC_DFACTOR_WOODBURY 2

typedef struct ccsc_problem {
  int32_t variant;          /* CCSC_DPAR .. CCSC_HS23                               */
  int32_t ndim;             /* spatial dims of b: 2 (2D, 4D) or 3 (3D)              */
  int64_t sb[3];            /* spatial size of b: x, y (, t for 3D)                 */
  int32_t views[2];         /* 4D: U, V (angular views; kernel_size(3:4));
                               2-3D: W, 1 (wavelengths, kernel_size(3)); else 1,1      */
  int64_t n;                /* number of patches (size(b, end))                     */
  int32_t K;                /* number of filters (kernel_size(end)); K <= 400 (2-3D:
                               K <= 192), larger K returns CCSC_E_UNSUPPORTED         */
  int32_t psf;              /* psf_s = kernel_size(1), odd                          */
  double lambda_residual;   /* objective weight only (dP:21, Q-note)                */
  double lambda_prior;      /* lambda: soft threshold = lambda / theta_div          */
  int32_t max_it;           /* outer iterations                                     */
  double tol;               /* relative-change tolerance; <= 0 disables the tests   */
  int32_t verbose;          /* CCSC_VERBOSE_*                                       */
  /* internal constants of the learners; 0 / <= 0 selects the variant default   */
  int32_t ni;               /* patches per block (dP:11 = 100, L3:11 = sqrt(n))     */
  int32_t max_it_d;         /* dP:75                                                */
  int32_t max_it_z;         /* dP:76                                                */
  double rho_d;             /* dP:98,111                                            */
  double rho_z;             /* dP:153                                               */
  double theta_div;         /* soft threshold = lambda_prior / theta_div (dP:150)   */
  int32_t precision;        /* CCSC_FP64 (the only value; others: CCSC_E_INVALID)   */
  int32_t trace_objective;  /* 1: evaluate the objective after every inner iter     */
  uint64_t seed;            /* device RNG seed for d0/z0 when not supplied          */
  int32_t dfactor;          /* CCSC_DFACTOR_* (0 = AUTO)                            */
} ccsc_problem;

typedef struct ccsc_outputs {
  double* d_res; /* [psf,psf,(psf | U,V),K] cropped filters of block 1 (dP:195-196) */
  double* z_res; /* this rank's codes: [X,Y,(T),K,n_local]; 4D: real part of the complex
                    [X,Y,1,1,K,n_local] (L4:164; its imaginary part is round-off, Q8)  */
  double* DZ;    /* this rank's reconstruction (dP:193 uncropped; L4:205-206 cropped) */
  double* obj_val; /* scalar final objective (L3:229, L4:211)                           */
} ccsc_outputs;

typedef struct ccsc_iterlog {
  int32_t capacity;      /* entries available per array below (>= max_it + 1)         */
  int32_t count;         /* entries written (outer iterations run + 1)                */
  double* obj_vals_d;    /* iterations.obj_vals_d (dP:63,174), nullable                 */
  double* obj_vals_z;    /* iterations.obj_vals_z (dP:64,175), nullable                 */
  double* tim_vals;      /* iterations.tim_vals, seconds, objective excluded (dP:176)   */
  /* extended trace (nullable; sized capacity * max_it_d / max_it_z)                   */
  double* trace_obj_d;   /* objective after each d-iteration (trace_objective=1)        */
  double* trace_obj_z;   /* objective after each z-iteration                            */
  double* trace_d_diff;  /* ||D1 - D1_old|| / ||D1|| per d-iteration (tol > 0)          */
  double* trace_z_diff;  /* ||z - z_old|| / ||z|| per z-iteration (tol > 0)             */
  int32_t* n_d;          /* d-iterations run per outer iteration                        */
  int32_t* n_z;          /* z-iterations run per outer iteration                        */
  int32_t* flags;        /* per outer iteration, bit 0: the 2-3D learner rolled back to
                            the previous iterate and stopped (L23:204-213); nullable      */
} ccsc_iterlog;

/* Progress callback, on the calling thread after each outer iteration. */
typedef void (*ccsc_cb)(void* user, int32_t outer_it, double obj_d, double obj_z,
                        double seconds);

typedef struct ccsc_ctx ccsc_ctx;
typedef struct ccsc_session ccsc_session;

/* ---- host-only helpers (no GPU needed) ---------------------------------- */
int32_t ccsc_abi_version(void);
/* Fill variant defaults (Appendix A) in place and validate shapes. */
int32_t ccsc_resolve(ccsc_problem* p, char* err, size_t errlen);
/* CCSC_OK if this build runs the (valid) problem on the GPU engine, else
 * CCSC_E_UNSUPPORTED with the reason (grid radices, LDS budget, K, variant). */
int32_t ccsc_supported(const ccsc_problem* p, char* err, size_t errlen);
/* Blocks [*block_begin, *block_begin + *block_count) of ni patches go to `rank`.  The 2-3D
 * learner (one block of all n images, L23) shards single images: its "blocks" are images; on
 * several ranks each passes its images' b / smooth_init / z0 with the global n in the problem,
 * and every rank holds the same filters (the Gram Z'Z and Z'xi1 are summed over the ranks). */
int32_t ccsc_shard(const ccsc_problem* p, int32_t rank, int32_t nranks,
                   int64_t* block_begin, int64_t* block_count, char* err, size_t errlen);
/* Device bytes one rank needs for this problem. */
int32_t ccsc_plan_bytes(const ccsc_problem* p, int32_t rank, int32_t nranks,
                        uint64_t* bytes, char* err, size_t errlen);

/* ---- device / communicator ---------------------------------------------- */
int32_t ccsc_device_count(int32_t* count, char* err, size_t errlen);
/* RCCL unique id (128 bytes) for a multi-rank context; call on rank 0. */
int32_t ccsc_get_unique_id(uint8_t* uid128, char* err, size_t errlen);
/* nranks == 1: uid may be NULL and no communicator is created. */
ccsc_ctx* ccsc_create(int32_t device, int32_t rank, int32_t nranks, const uint8_t* uid128,
                      char* err, size_t errlen);
/* Host-transport communicator (testing / hosts without RCCL): the engine stages
 * each exchange through host memory and calls fn on the calling thread.
 * op 0 = in-place sum all-reduce, op 1 = in-place broadcast from rank 0.
 * fn returns 0 on success. */
#define CCSC_COMM_ALLREDUCE_SUM 0
#define CCSC_COMM_BCAST0 1
typedef int32_t (*ccsc_comm_fn)(void* user, int32_t op, double* buf, int64_t count);
ccsc_ctx* ccsc_create_hostcomm(int32_t device, int32_t rank, int32_t nranks, ccsc_comm_fn fn,
                               void* user, char* err, size_t errlen);
/* Single-process multi-device context: the drop-in path of one MATLAB call over a
 * node's GPUs (learn_kernels_2D_large.m:28 calls the learner once).
 * devices[0..ndev-1] become ranks 0..ndev-1 (one stream each, ncclCommInitAll over
 * xGMI; a list that repeats a device, e.g. {0, 0} on a one-GPU host, exchanges
 * through host memory instead).  ccsc_learn on this context takes the caller's
 * WHOLE problem (b and z0 over all n patches, outputs for all n), shards the blocks
 * with ccsc_shard, runs rank i in a host thread on devices[i] and calls back on the
 * calling thread only.  Sessions and the 2-3D learner need a one-device context
 * (CCSC_E_UNSUPPORTED here).  ndev == 1 is ccsc_create(devices[0], 0, 1, NULL). */
ccsc_ctx* ccsc_create_multi(const int32_t* devices, int32_t ndev, char* err, size_t errlen);
void ccsc_destroy(ccsc_ctx* ctx);
/* Ranks the context's communicator spans and its transport: RCCL reports
 * ncclCommCount (of rank 0's communicator for a multi-device context), the host
 * transport its nranks; a one-rank context reports 1 and NONE.  Evidence that a
 * multi-GPU run exchanged over RCCL across the ranks it claims (bench.py). */
#define CCSC_TRANSPORT_NONE 0
#define CCSC_TRANSPORT_RCCL 1
#define CCSC_TRANSPORT_HOST 2
int32_t ccsc_comm_ranks(ccsc_ctx* ctx, int32_t* ranks, int32_t* transport, char* err,
                        size_t errlen);

/* ---- one-shot learner: the literal drop-in for the .m functions --------- */
/* b: this rank's patches, [sb..., (U,V), n_local] column-major float64.
 * d0: [psf,psf,(psf|U,V),K] (init.d) or NULL (device RNG from p->seed).
 * z0: init.z -- dP/L3/L4: size_z of this rank's patches; dZ: size_z_crop
 *     ([X,Y,K,ni], replicated into every block, dZ:44-47); NULL = device RNG. */
int32_t ccsc_learn(ccsc_ctx* ctx, const ccsc_problem* p, const double* b, const double* d0,
                   const double* z0, ccsc_outputs* out, ccsc_iterlog* log, ccsc_cb cb,
                   void* user, char* err, size_t errlen);

/* 2-3D hyperspectral learner, the drop-in for admm_learn(b, kernel_size, lambda_residual,
 * lambda, max_it, tol, verbose, init, smooth_init) (2-3D/DictionaryLearning/admm_learn.m:1-4,
 * called by learn_hyperspectral.m:30).  p->variant = CCSC_HS23, p->views[0] = W.
 * b, smooth_init: [x, y, W, n] (smooth_init = the caller's low-pass of b,
 * learn_hyperspectral.m:16-17).  d0: [psf, psf, K], replicated over the W wavelengths
 * (L23:54-56), or NULL; z0: [X, Y, K, n] or NULL (device RNG from p->seed).
 * Outputs: d_res [psf,psf,W,K]; z_res [X,Y,K,n]; DZ [X,Y,W,n] = Dz incl. smoothinit,
 * uncropped (L23:234-235); obj_val = the last objective evaluated (L23:195 / :211).
 * One rank only (its d-solve couples every image per frequency). */
int32_t ccsc_learn_hs23(ccsc_ctx* ctx, const ccsc_problem* p, const double* b,
                        const double* smooth_init, const double* d0, const double* z0,
                        ccsc_outputs* out, ccsc_iterlog* log, ccsc_cb cb, void* user, char* err,
                        size_t errlen);

/* ---- stateful session (bench / warm restart) ---------------------------- */
ccsc_session* ccsc_session_create(ccsc_ctx* ctx, const ccsc_problem* p, const double* b,
                                  const double* d0, const double* z0, char* err, size_t errlen);
/* The 2-3D learner's session (arguments as ccsc_learn_hs23). */
ccsc_session* ccsc_session_create_hs23(ccsc_ctx* ctx, const ccsc_problem* p, const double* b,
                                       const double* smooth_init, const double* d0,
                                       const double* z0, char* err, size_t errlen);
/* Run `n_outer` outer iterations (tol tests honoured); returns when the device is
 * idle.  *done = 1 when the tol test ended the learning early. */
int32_t ccsc_session_step(ccsc_session* s, int32_t n_outer, int32_t* done, char* err,
                          size_t errlen);
/* Objective of the current iterate: lambda_res/2||crop(Dz) - b||^2 + lambda|z|_1. */
int32_t ccsc_session_objective(ccsc_session* s, double* obj, char* err, size_t errlen);
int32_t ccsc_session_results(ccsc_session* s, ccsc_outputs* out, char* err, size_t errlen);
int32_t ccsc_session_iterlog(ccsc_session* s, ccsc_iterlog* log, char* err, size_t errlen);
/* Per-kernel timing with HIP events on the engine stream.  kernel ids: 0 = fused
 * z-step, 1 = gram+cholesky, 2 = d-solve, 3 = dual+R2C, 4 = C2R+support.  Returns
 * launches, total milliseconds and the algorithmic bytes of ONE launch. */
int32_t ccsc_session_set_profiling(ccsc_session* s, int32_t on);
int32_t ccsc_session_kernel_stats(ccsc_session* s, int32_t kernel_id, int64_t* launches,
                                  double* total_ms, double* alg_bytes_per_launch, char* err,
                                  size_t errlen);
void ccsc_session_destroy(ccsc_session* s);

/* ---- reconstruction solvers ------------------------
 * Sparse-coding reconstruction of images from learned filters; each variant is the
 * drop-in for one reference function (paths relative to the reference root):
 *   CCSC_SOLVE_INPAINT2D  [z, res] = admm_solve_conv2D_weighted_sampling(b, kernels, mask,
 *                         lambda_residual, lambda_prior, smooth_init, max_it, tol, x_orig,
 *                         verbose)          2D/Inpainting/admm_solve_conv2D_weighted_sampling.m:1-4
 *   CCSC_SOLVE_POISSON2D  [z, res] = admm_solve_conv_poisson(b, kmat, mask, lambda_residual,
 *                         lambda_prior, max_it, tol, x_orig, verbose)
 *                                           2D/Poisson_deconv/admm_solve_conv_poisson.m:1-2
 *   CCSC_SOLVE_MULTICH    [z, res] = admm_solve_conv23D_weighted_sampling(b, kmat, mask,
 *                         lambda_residual, lambda_prior, max_it, tol, ~, verbose, smooth_init)
 *                                           2-3D/Demosaicing/admm_solve_conv23D_weighted_sampling.m:1-2
 *                         and admm_solve_conv_weighted_sampling_lf (the same text)
 *                                           4D/ViewSynthesis/admm_solve_conv_weighted_sampling_lf.m:1-2
 *   CCSC_SOLVE_VIDEO3D    [z, res] = admm_solve_video_weighted_sampling(b, kmat, mask,
 *                         lambda_residual, lambda_prior, max_it, tol, verbose, psf, smooth_init)
 *                                           3D/Deblurring/admm_solve_video_weighted_sampling.m:1-2
 * One call solves n independent images of one shape (the reference's callers loop over
 * images, e.g. reconstruct_poisson_noise.m:24); each image keeps its own gamma
 * heuristic (c * lambda_prior / max(b(:))) and its own tol test.  Arrays are
 * column-major float64 with the image index last. */
#define CCSC_SOLVE_INPAINT2D 0
#define CCSC_SOLVE_POISSON2D 1
#define CCSC_SOLVE_MULTICH 2
#define CCSC_SOLVE_VIDEO3D 3

typedef struct ccsc_solve_problem {
  int32_t variant;          /* CCSC_SOLVE_*                                                */
  int64_t sb[3];            /* image extent x, y (, t for VIDEO3D)                         */
  int32_t nch;              /* MULTICH: channels W = size(b, 3) (wavelengths / views); else 1 */
  int64_t n;                /* images solved by this call                                  */
  int32_t K;                /* learned filters (kernel_size(end)), without the dirac that
                               POISSON2D appends and VIDEO3D prepends                      */
  int32_t ksize[3];         /* filter extent x, y (, t); odd                                 */
  int32_t psf_size[3];      /* VIDEO3D: extent of the blur psf                             */
  double lambda_residual;
  double lambda_prior;
  int32_t max_it;
  double tol;               /* relative change ||z - z_old|| / ||z||; <= 0: never stops early */
  int32_t verbose;          /* CCSC_VERBOSE_*: BRIEF/ALL fill the objective / PSNR trace   */
} ccsc_solve_problem;

typedef struct ccsc_solve_inputs {
  const double* b;           /* [sx, sy, (st | W), n]                                       */
  const double* kernels;     /* INPAINT2D/POISSON2D [k,k,K]; MULTICH [k,k,W,K]; VIDEO3D [k,k,k,K] */
  const double* mask;        /* same shape as b                                              */
  const double* smooth_init; /* same shape as b; NULL for POISSON2D (it has none)            */
  const double* psf;         /* VIDEO3D: blur kernel [psf_size]; else NULL                   */
  const double* x_orig;      /* INPAINT2D/POISSON2D: [sx, sy, n] for the PSNR trace; nullable */
} ccsc_solve_inputs;

typedef struct ccsc_solve_outputs {
  double* z;    /* [X, Y, (T), K', n] codes on the padded grid (K' includes the dirac:
                   POISSON2D last, VIDEO3D first; MULTICH: X, Y = sx, sy); nullable       */
  double* res;  /* INPAINT2D/POISSON2D [sx, sy, n]; MULTICH [sx, sy, W, n];
                   VIDEO3D [sx, sy, st, n]; nullable                                       */
} ccsc_solve_outputs;

typedef struct ccsc_solvelog {
  int32_t capacity;   /* entries per image in the arrays below (>= max_it + 1)            */
  int32_t* iters;     /* [n] ADMM iterations run per image (tol may stop an image early)  */
  double* obj;        /* [n][capacity] objective of iterate 0..iters (verbose BRIEF/ALL)  */
  double* psnr;       /* [n][capacity] PSNR vs x_orig (INPAINT2D/POISSON2D)               */
  double* diff;       /* [n][capacity] ||z - z_old|| / ||z|| (0 for iterate 0)            */
  double* seconds;    /* [1] device time of the ADMM iterations (setup and output excluded) */
} ccsc_solvelog;

/* CCSC_OK if this build runs the (valid) problem, else CCSC_E_INVALID /
 * CCSC_E_UNSUPPORTED with the reason (e.g. a grid length with no FFT plan). */
int32_t ccsc_solve_supported(const ccsc_solve_problem* p, char* err, size_t errlen);
int32_t ccsc_solve(ccsc_ctx* ctx, const ccsc_solve_problem* p, const ccsc_solve_inputs* in,
                   ccsc_solve_outputs* out, ccsc_solvelog* log, char* err, size_t errlen);

/* ---- input preprocessing ----------------------------
 * Local contrast normalisation of the learners' input images: the 'local_cn' and
 * ZERO_MEAN branches of image_helpers/CreateImages.m:299-369, :652-657 (13x13 Gaussian,
 * sigma 3*1.591, reflection padding of image_helpers/rconv2.m:22-58, std floored at
 * its median, single-precision result), one GPU workgroup per image.
 * in/out: n column-major [H, W] float64 images (out = double(single(...)), may alias in).
 * ccsc_local_cn takes host arrays; ccsc_local_cn_dev device arrays on the context's
 * device (e.g. torch tensors), ordered on the context's stream, synchronised on return. */
int32_t ccsc_local_cn(ccsc_ctx* ctx, const double* in, double* out, int64_t n, int32_t H,
                      int32_t W, char* err, size_t errlen);
int32_t ccsc_local_cn_dev(ccsc_ctx* ctx, const double* in, double* out, int64_t n, int32_t H,
                          int32_t W, char* err, size_t errlen);

/* ---- kernel-level entry points (parity tests of single stages) ---------- */
/* 2D R2C of `count` real slices [X,Y] -> half spectra [Y][X/2+1] (re,im). */
int32_t ccsc_test_fft2d(ccsc_ctx* ctx, int32_t X, int32_t Y, int32_t count, const double* in,
                        double* out_halfspec, double* roundtrip, char* err, size_t errlen);

#ifdef __cplusplus
}
#endif
#endif /* CCSC_H_ */
