/*
 * viabel_amd.h — C ABI of the MI355X (gfx950) Monte Carlo VI hot path.
 *
 * This is the drop-in boundary behind which the viabel.vb / viabel.bounds /
 * psis Python API (mirrored by the `viabel_amd` package) runs on HIP kernels.
 * Plain C types only: pointers + sizes, no torch / numpy types.  Every pointer
 * argument may be host memory or device memory (hipMalloc / torch.cuda); the
 * library detects which with hipPointerGetAttributes and stages host buffers
 * through the context's device scratch.  The library never retains a caller
 * pointer after a call returns.
 *
 * Error convention: every entry point returns VB_OK (0) or a negative code;
 * vb_last_error() returns a thread-local message for the last failure.
 * No C++ exception crosses this boundary.
 *
 * Reference interfaces replaced (paths relative to the reference repo):
 *   vb_family_*            viabel/vb.py:42-82 (mean_field_gaussian_variational_family),
 *                          viabel/vb.py:140-182 (mean_field_t_variational_family),
 *                          viabel/vb.py:192-233 (t_variational_family, full rank) with
 *                          viabel/_distributions.py:8-38 (multivariate_t_logpdf)
 *   vb_family_moments      viabel/vb.py:215-229 (full-rank mean_and_cov / pth_moment
 *                          eigvalsh / entropy det)
 *   vb_objective_value_grad viabel/vb.py:236-245 (black_box_klvi),
 *                          viabel/vb.py:248-266 (black_box_chivi)
 *   vb_run_*               viabel/vb.py:324-389 (learning_rate_schedule, adagrad_optimize),
 *                          viabel/vb.py:392-712 (the RMSProp-IA / Adam-IA updates)
 *   vb_rhat                viabel/functions.py:8-65 (compute_R_hat and its windowed /
 *                          halfway drivers)
 *   vb_rhat_stats / vb_rhat_combine  viabel/functions.py:8-31 split at the chain axis,
 *                          for the chains of viabel/vb.py:417-421 sharded over ranks
 *   vb_iterate_average     viabel/functions.py:68-77 (stochastic_iterate_averaging)
 *   vb_adagrad_update      viabel/vb.py:364-374 (one adagrad step for a foreign objective)
 *   vb_adagrad_update_scaled  viabel/vb.py:364-374 with has_log_norm (grad_scale, :371-373)
 *   vb_ia_update           viabel/vb.py:436-453, 606-617 (one RMSProp-IA / Adam-IA step for a
 *                          foreign objective, or with avg_grad_norm)
 *   vb_log_weights         notebooks/experiments.py:60-63 (get_samples_and_log_weights)
 *   vb_log_weights_rows    notebooks/experiments.py:60-63 for every restart of
 *                          vb.py:417-421's restart loop in one launch
 *   vb_divergence_bound    viabel/bounds.py:142-192 (divergence_bound, mean_and_check_mc_error)
 *   vb_divergence_bound_rows viabel/bounds.py:142-192 (divergence_bound over many log-weight rows)
 *   vb_centered_moments    viabel/bounds.py:127-135 (wasserstein_bounds sample moments)
 *   vb_covariance          viabel/bounds.py:55-56 (np.cov(samples.T), ddof = 1)
 *   vb_weighted_covariance notebooks/experiments.py:83-85 (PSIS-weighted mean / np.cov)
 *   vb_weighted_covariance_logw notebooks/experiments.py:80-85 (weights from log weights)
 *   vb_psislw              notebooks/psis.py:112-208 (psislw)
 *   vb_psislw_colmajor     notebooks/psis.py:112-208 (psislw, Fortran-ordered input)
 *   vb_gpdfit              notebooks/psis.py:211-331 (gpdfitnew)
 *   vb_gpinv               notebooks/psis.py:334-376 (gpinv)
 *   vb_sumlogs             notebooks/psis.py:379-395 (sumlogs)
 *   vb_sumlogs_rows        notebooks/psis.py:379-395 (sumlogs with an axis)
 */
#ifndef VIABEL_AMD_H
#define VIABEL_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VB_ABI_VERSION 1

/* ---- status codes ---------------------------------------------------- */
enum {
  VB_OK = 0,
  VB_EINVAL = -1,       /* bad argument: Python raises ValueError */
  VB_EDEVICE = -2,      /* HIP runtime failure: RuntimeError */
  VB_ENOMEM = -3,       /* allocation failure: MemoryError */
  VB_EUNSUPPORTED = -4  /* valid but not implemented on device: NotImplementedError */
};

/* ---- descriptors ----------------------------------------------------- */
enum vb_family_kind {
  VB_FAMILY_MF_GAUSSIAN = 0, /* lambda = [mean(D), log_std(D)]       vb.py:48-82   */
  VB_FAMILY_MF_T = 1,        /* lambda = [mean(D), log_scale(D)], df  vb.py:140-182 */
  VB_FAMILY_FR_T = 2         /* lambda = [mu(D), tril(M) row-major (D(D+1)/2)], df;
                                L = M with exp'd diagonal, Sigma = L L^T  vb.py:192-233 */
};

enum vb_target_kind {
  VB_TARGET_ISOGAUSS = 0,       /* N(0, I_D)                                  (separable) */
  VB_TARGET_MIXTURE = 1,        /* prod_d 0.5 N(-2,1) + 0.5 N(2,1)            (separable) */
  VB_TARGET_FUNNEL = 2,         /* Neal's funnel, x[1] = log sigma ~ N(0,1.35^2)           */
  VB_TARGET_EIGHT_SCHOOLS_NCP = 3, /* eight_schools_ncp.stan log_prob, D = 10              */
  VB_TARGET_CORR_GAUSS = 4,   /* N(0, Sigma*): params = [inv(Sigma*) (D x D row-major),
                                 log normaliser]; full-rank family only (SURVEY §8d cfg 4) */
  VB_TARGET_CALLBACK = 5      /* user model through vb_target.callback (make_stan_log_density,
                                 vb.py:314-321): evaluated on the host once per step on the
                                 batch of samples; everything else stays on the device */
};

/* User target: log p and d log p / dx of the n rows of x [n][d] (HOST memory,
 * C order) into logp [n] and grad [n][d]; return 0, or non-zero to abort the
 * call with VB_EDEVICE. */
typedef int (*vb_target_callback)(void* user, const double* x, int64_t n, int64_t d,
                                  double* logp, double* grad);

enum vb_objective_kind {
  VB_OBJ_KLVI = 0,     /* value = -(entropy + mean log p)              vb.py:236-245 */
  VB_OBJ_CHIVI = 1,    /* value = CUBO_alpha, grad = alpha/N sum w dlw vb.py:248-266 */
  VB_OBJ_KLVI_PD = 2   /* value = -(mean log p - mean log q(x)), gradient = KLVI's
                          (black_box_klvi_pd / _pd2, vb.py:268-295) */
};

enum vb_noise_kind {
  VB_NOISE_HOST = 0,   /* standardized draws supplied by the caller (numpy legacy RNG parity) */
  VB_NOISE_PHILOX = 1  /* in-kernel Philox4x32-10, counter = (pair, sample, step, stream) */
};

typedef struct vb_family {
  int32_t kind;   /* vb_family_kind */
  int32_t reserved;
  int64_t dim;    /* D */
  double df;      /* degrees of freedom (t family), ignored otherwise */
} vb_family;

typedef struct vb_target {
  int32_t kind;   /* vb_target_kind */
  int32_t reserved;
  int64_t dim;    /* D (must equal the family's) */
  const double* params; /* target parameters (host or device), NULL if none */
  int64_t n_params;
  vb_target_callback callback; /* VB_TARGET_CALLBACK only */
  void* user;
} vb_target;

typedef struct vb_objective {
  int32_t kind;      /* vb_objective_kind */
  int32_t reserved;
  double alpha;      /* CHIVI order (> 1); ignored for KLVI */
  int64_t n_samples; /* N Monte Carlo draws per call */
} vb_objective;

/* Noise source.  HOST: `eps` holds standardized draws laid out
 * [problem][step][sample][dim] (C order): N(0,1) for the Gaussian family,
 * standard_t(df) for the t family.  PHILOX: `seed` keys the generator;
 * problem q of a call draws from stream `stream + q * stream_stride`
 * (24 bits; stride 0 means 1); `step` is the global step index of the first
 * step of the call.  Full-rank t family (VB_FAMILY_FR_T): each step's block of
 * `eps` is [s (N), z (N x D)] with s = sqrt(chisquare(df)/df) and z ~ N(0, I),
 * drawn in that order (vb.py:204-206). */
typedef struct vb_noise {
  int32_t kind;      /* vb_noise_kind */
  uint32_t stream;
  uint64_t seed;
  uint64_t step;
  const double* eps; /* HOST only */
  uint32_t stream_stride;
  uint32_t reserved;
} vb_noise;

enum vb_optimizer_kind {
  VB_OPT_ADAGRAD = 0,      /* adagrad_optimize, vb.py:345-389 (window of W gradients) */
  VB_OPT_RMSPROP_IA = 1,   /* rmsprop_IA_optimize_with_rhat's update, vb.py:436-453 */
  VB_OPT_ADAM_IA = 2,      /* adam_IA_optimize_with_rhat's update, vb.py:606-617 */
  VB_OPT_RMSPROP_IA_NORM = 3 /* rmsprop_IA with avg_grad_norm=True (vb_ia_update only) */
};

/* Optimiser settings, vb.py:345-347 defaults: window 10, lr .01, eps .1.
 * ADAGRAD: window = gradient window (<= 64); history = parameters AFTER the
 * update for the last n_iters - 3 n_iters / 4 iterations (vb.py:375-376).
 * RMSPROP_IA / ADAM_IA: history = parameters BEFORE each update for the last
 * min(n_iters, 100 window) iterations (vb.py:455-457, 622-624). */
typedef struct vb_adagrad_config {
  int64_t n_iters;
  int32_t window;
  int32_t optimizer; /* vb_optimizer_kind */
  double learning_rate;
  double learning_rate_end; /* NaN = None (constant schedule) */
  double epsilon;
} vb_adagrad_config;

typedef struct vb_ctx vb_ctx;
typedef struct vb_run vb_run;

/* ---- context --------------------------------------------------------- */
int vb_abi_version(void);
const char* vb_last_error(void);
/* sha256 (first 16 hex digits) of the library's sources, in the fixed order of
 * viabel_amd/csrc/Makefile's HASH_SRCS, fixed at build time: which sources the
 * loaded binary was built from (measurement provenance; not part of the path). */
const char* vb_build_id(void);
/* Matrix-core flops of the products the calling thread has launched since the
 * last reset (each launch: tiles computed x tile area x depth x 2; launches the
 * device skips past convergence count too); reset != 0 zeroes the tally.  Measurement
 * aid for the full-rank step's executed-flop figure; not part of the reference API. */
double vb_flop_tally(int reset);
/* `hip_stream` may be NULL (the context creates its own stream) or an
 * existing hipStream_t (e.g. torch.cuda.current_stream().cuda_stream). */
int vb_ctx_create(int device, void* hip_stream, vb_ctx** out);
int vb_ctx_destroy(vb_ctx* ctx);
int vb_ctx_synchronize(vb_ctx* ctx);
void* vb_ctx_stream(vb_ctx* ctx);

/* ---- variational family (vb.py:54-65, 148-162) ------------------------ */
/* x_out[n, d] = sample of q(lambda); n = 0..n-1.  Noise as above (one problem). */
int vb_family_sample(vb_ctx* ctx, const vb_family* fam, const double* lam,
                     int64_t n, const vb_noise* noise, double* x_out);
/* out[n] = log q(x[n, :]; lambda) with all normalising constants. */
int vb_family_logdensity(vb_ctx* ctx, const vb_family* fam, const double* lam,
                         const double* x, int64_t n, double* out);
/* Full-rank family only: sigma_out [D][D] = Sigma = L L^T and eig_out [D] =
 * its eigenvalues in ascending order (both nullable).  mean_and_cov is
 * (mu, df/(df-2) Sigma), entropy .5 sum log eig, pth_moment from eig. */
int vb_family_moments(vb_ctx* ctx, const vb_family* fam, const double* lam,
                      double* sigma_out, double* eig_out);
/* out[n] = log p(x[n, :]); grad_out (nullable) = d log p / dx, [n, D]. */
int vb_target_logdensity(vb_ctx* ctx, const vb_target* tgt, const double* x,
                         int64_t n, double* out, double* grad_out);

/* ---- estimators (vb.py:236-266) -------------------------------------- */
/* One stochastic objective value and gradient at lambda (P = 2D values for
 * the mean-field families, D + D(D+1)/2 for the full-rank t family). */
int vb_objective_value_grad(vb_ctx* ctx, const vb_family* fam, const vb_target* tgt,
                            const vb_objective* obj, const double* lam,
                            const vb_noise* noise, double* value, double* grad);

/* ---- device-resident adagrad (vb.py:324-389) -------------------------- */
/* n_problems independent restarts share (fam, tgt, obj, cfg); init is
 * [n_problems][P].  Philox streams are noise.stream + problem. */
int vb_run_create(vb_ctx* ctx, const vb_family* fam, const vb_target* tgt,
                  const vb_objective* obj, const vb_adagrad_config* cfg,
                  int64_t n_problems, const double* init, vb_run** out);
/* Advance every problem by n_steps adagrad iterations (lr schedule and
 * history bookkeeping as vb.py:356-376).  HOST noise: eps covers
 * [n_problems][n_steps][N][D]. */
int vb_run_advance(vb_run* run, int64_t n_steps, const vb_noise* noise);
int vb_run_steps_done(vb_run* run, int64_t* out);
/* Full-rank runs (measurement / test support, no reference counterpart): how many
 * advances ran again because a warm Newton-Schulz root launched too few
 * iterations (the rerun restores lambda, the adagrad window and the warm state). */
int vb_run_fr_retries(vb_run* run, int64_t* out);
/* Peak-rate microbenchmarks (measurement support, no reference counterpart;
 * BASELINE.md §2 asks for the roofline peaks to be confirmed on the box): kind 0
 * HBM copy and 1 HBM read over n bytes (GB/s of bytes moved), 2 fp64 MFMA
 * (TFLOP/s), 3 fp64 FMA and 4 u64 multiply VALU issue (G wave-instructions/s)
 * over n iterations; best of reps timed launches on the context's stream. */
int vb_peak_probe(vb_ctx* ctx, int32_t kind, int64_t n, int32_t reps, double* out);
/* Launch timing (measurement support, no reference counterpart): with enable
 * != 0 every later vb_run_advance brackets its device work with HIP events on
 * the context's stream, one pair per kernel chunk (column-pair path) or per
 * call (other paths).  vb_run_launch_times waits for that work, returns up to
 * max (steps, milliseconds) records in launch order, n_out = their count, and
 * forgets them. */
int vb_run_set_timing(vb_run* run, int enable);
int vb_run_launch_times(vb_run* run, int64_t max, int64_t* steps_out, float* ms_out,
                        int64_t* n_out);
/* Latency floor of the block-per-problem step (measurement support, no reference
 * counterpart): runs n_steps of the block kernel's step skeleton -- the same
 * block shape for (D <= 16, N, objective; host_layout != 0: the device-noise /
 * pre-drawn layout of row waves only), barriers, reductions and adagrad update,
 * but no draws and no target -- on n_problems blocks, and returns the device
 * microseconds per step (HIP events on the context's stream). */
int vb_block_floor(vb_ctx* ctx, int32_t D, int32_t N, int32_t chivi, int32_t host_layout,
                   int64_t n_steps, int64_t n_problems, double* us_per_step);
/* Results (all nullable): lam_out [n_problems][P]; hist_out
 * [n_problems][n_hist][P] (n_hist per vb_adagrad_config); values_out [n_problems][n_iters];
 * smoothed_out [n_problems][P] = mean of the history rows (vb.py:386-387). */
int vb_run_result(vb_run* run, double* lam_out, double* hist_out,
                  double* values_out, double* smoothed_out);
/* Progress snapshot of problem 0's objective values (the reference's progress bar,
 * vb.py:378-381, without stalling the device): vb_run_values_async queues a copy of
 * values[0 .. count) into a pinned buffer of the run behind the work already queued
 * and returns at once; the caller may queue further advances; vb_run_values_wait
 * waits for that copy only, writes the count values to out and count_out.  One
 * snapshot per context is pending at a time (the context's pinned buffer). */
int vb_run_values_async(vb_run* run, int64_t count);
int vb_run_values_wait(vb_run* run, double* out, int64_t* count_out);
int vb_run_destroy(vb_run* run);

/* One adagrad step (vb.py:364-374) for a caller-supplied gradient (foreign
 * objectives).  lam [P] and ring [window][P] are DEVICE pointers holding the
 * optimiser state; step is the 0-based iteration index (ring slot step % window). */
int vb_adagrad_update(vb_ctx* ctx, int64_t P, double* lam, const double* grad,
                      double* ring, int32_t window, int64_t step, double lr,
                      double epsilon);
/* vb_adagrad_update for objectives with log norms (has_log_norm=True,
 * vb.py:371-373): window_scale [min(step + 1, window)] holds, oldest first, the
 * reference's grad_scale = exp(min(log_norms) - log_norm_j) over the window;
 * accum = sum_j (window_scale_j g_j)^2. */
int vb_adagrad_update_scaled(vb_ctx* ctx, int64_t P, double* lam, const double* grad,
                             double* ring, int32_t window, int64_t step, double lr,
                             double epsilon, const double* window_scale);
/* One RMSProp-IA (vb.py:436-453) or Adam-IA (vb.py:606-617) step for a
 * caller-supplied gradient.  lam [P] and state [2][P] are DEVICE pointers
 * (state row 0: second moment, row 1: first moment; zeros before step 0);
 * old_out (nullable) receives the pre-update lam, which the reference's
 * history keeps.  VB_OPT_RMSPROP_IA_NORM is avg_grad_norm=True: every
 * coordinate is divided by sqrt(epsilon + norm2), with norm2 the reference's
 * scalar sum_grad_squared (vb.py:443-451); norm2 is ignored otherwise. */
int vb_ia_update(vb_ctx* ctx, int32_t optimizer, int64_t P, double* lam, const double* grad,
                 double* state, int64_t step, double lr, double epsilon, double norm2,
                 double* old_out);

/* ---- convergence diagnostics (functions.py:8-77) ------------------------ */
/* Split-chain R-hat (compute_R_hat) of chains [n_chains][n_iters][P] on n_jobs
 * iteration segments [job_start[j], job_start[j] + job_len[j]) (job_len even):
 * var_hat_out (nullable) and rhat_out are [n_jobs][P]. */
int vb_rhat(vb_ctx* ctx, const double* chains, int64_t n_chains, int64_t n_iters, int64_t P,
            int64_t n_jobs, const int64_t* job_start, const int64_t* job_len,
            double* var_hat_out, double* rhat_out);
/* The two stages of vb_rhat, for chains held by different processes
 * (viabel/vb.py:417-421's chain loop sharded over ranks, then
 * viabel/functions.py:8-52 on the union).  vb_rhat_stats: per segment j,
 * half-chain i (= 2 chain + half) and parameter p, the half-chain mean and
 * centred sum of squares, mean_out / ss_out [n_jobs][2 n_chains][P].
 * vb_rhat_combine: R-hat of n_halves half-chains from those statistics
 * (n_halves = 2 x the chains of all ranks, in chain order; job_len the segment
 * lengths); the same bits as vb_rhat on the gathered chains. */
int vb_rhat_stats(vb_ctx* ctx, const double* chains, int64_t n_chains, int64_t n_iters, int64_t P,
                  int64_t n_jobs, const int64_t* job_start, const int64_t* job_len,
                  double* mean_out, double* ss_out);
int vb_rhat_combine(vb_ctx* ctx, const double* mean, const double* ss, int64_t n_halves, int64_t P,
                    int64_t n_jobs, const int64_t* job_len, double* var_hat_out, double* rhat_out);
/* stochastic_iterate_averaging: out [n - start][cols] = cumulative means of
 * x[start:, 0:cols] (row stride ld). */
int vb_iterate_average(vb_ctx* ctx, const double* x, int64_t n, int64_t ld, int64_t cols,
                       int64_t start, double* out);

/* ---- log weights for bounds / PSIS (experiments.py:60-63) ------------ */
/* Philox noise: the mean-field t family's draws here are Bailey's trigonometric
 * t variates (one Philox block per column pair, no rejection; oracle/vbrng.c
 * family 2), not the estimators' normal / gamma construction -- the same t(df)
 * distribution (the Philox mode is a statistical contract).
 * Host noise (the reference's numpy streams) is used as given. */
int vb_log_weights(vb_ctx* ctx, const vb_family* fam, const vb_target* tgt,
                   const double* lam, int64_t m, const vb_noise* noise,
                   double* lw_out, double* samples_out /* nullable, [m, D] */);
/* vb_log_weights for `rows` parameter vectors of a mean-field family at once
 * (lam [rows][2D]; Philox noise only, row r drawing from stream
 * noise->stream + r * noise->stream_stride), lw_out [rows][m], one launch.
 * Targets / dimensions of the block kernel's range (D <= 16, or separable).
 * rows <= 65535. */
int vb_log_weights_rows(vb_ctx* ctx, const vb_family* fam, const vb_target* tgt,
                        const double* lam, int64_t rows, int64_t m, const vb_noise* noise,
                        double* lw_out);

/* ---- bounds (bounds.py:142-192, 127-135) ------------------------------ */
/* out[0] = d_alpha, out[1] = log_norm_bound (ELBO), out[2] = CUBO mean of
 * rescaled weights, out[3] = its MC standard error, out[4] = ELBO mean,
 * out[5] = ELBO MC standard error (NaN when elbo supplied), out[6] = log max. */
int vb_divergence_bound(vb_ctx* ctx, const double* lw, int64_t n, double alpha,
                        int32_t has_elbo, double elbo, double* out7);
/* vb_divergence_bound for `rows` independent log-weight vectors of length n,
 * row r at lw + r * ld (ld >= n), in one launch chain: out7 [rows][7] as above
 * (row r's d_alpha, elbo, ...).  rows <= 65535. */
int vb_divergence_bound_rows(vb_ctx* ctx, const double* lw, int64_t rows, int64_t n, int64_t ld,
                             double alpha, int32_t has_elbo, double elbo, double* out7);
/* c2 = mean_n sum_d (x - xbar)^2, c4 = mean_n sum_d (x - xbar)^4. */
int vb_centered_moments(vb_ctx* ctx, const double* x, int64_t n, int64_t d,
                        double* c2, double* c4);
/* column means [d] and covariance [d, d] (ddof = 1, np.cov(x.T)) of x [n, d]
 * (d <= 64: fixed-order pairwise reduction; larger d: fp64 MFMA product). */
int vb_covariance(vb_ctx* ctx, const double* x, int64_t n, int64_t d,
                  double* mean_out, double* cov_out);
/* np.cov(x.T, aweights=w, ddof=ddof) and the weighted mean (np.average with
 * weights) of x [n, d]; w [n] nullable (unweighted).  improve_with_psis
 * (notebooks/experiments.py:73-89) with the PSIS-smoothed weights. */
int vb_weighted_covariance(vb_ctx* ctx, const double* x, int64_t n, int64_t d,
                           const double* w, int32_t ddof, double* mean_out, double* cov_out);
/* vb_weighted_covariance with w = exp(log_w - max log_w), normalised on the
 * device: improve_with_psis's weights from the smoothed log weights
 * (notebooks/experiments.py:80-85). */
int vb_weighted_covariance_logw(vb_ctx* ctx, const double* x, int64_t n, int64_t d,
                                const double* log_w, int32_t ddof, double* mean_out,
                                double* cov_out);

/* ---- PSIS (psis.py:112-395) ------------------------------------------ */
/* lw [n, m] C order (m columns of n log weights).  lw_out same layout, or null
 * for k (and the tails) only: the smoothing and renormalisation, which feed only
 * lw_out, are skipped.  k_out [m].  tail_idx_out (nullable) [m, tail_cap]: the tail indices in
 * ascending order of the tail values (tailinds[x2si]); n_tail_out (nullable) [m]. */
int vb_psislw(vb_ctx* ctx, const double* lw, int64_t n, int64_t m, double reff,
              double* lw_out, double* k_out, int64_t* tail_idx_out,
              int64_t tail_cap, int64_t* n_tail_out);
/* vb_psislw for column-major input: lw holds m columns of n contiguous log
 * weights (a Fortran-ordered [n, m] array, the layout psis.py:146 copies the
 * input into); lw_out likewise.  All m columns run through the pipeline
 * together (column-batched launches). */
int vb_psislw_colmajor(vb_ctx* ctx, const double* lw, int64_t n, int64_t m, double reff,
                       double* lw_out, double* k_out, int64_t* tail_idx_out,
                       int64_t tail_cap, int64_t* n_tail_out);
/* Zhang-Stephens GPD fit of x[n] (any order).  ks_out / w_out nullable,
 * length 30 + floor(sqrt(n)); *n_w_out = number of weights kept. */
int vb_gpdfit(vb_ctx* ctx, const double* x, int64_t n, double* k, double* sigma,
              double* ks_out, double* w_out, int64_t* n_w_out);
int vb_gpinv(vb_ctx* ctx, const double* p, int64_t n, double k, double sigma,
             double* out);
int vb_sumlogs(vb_ctx* ctx, const double* x, int64_t n, double* out);
/* out[r] = sumlogs of row r of x [rows][n] (sumlogs with an axis, psis.py:379-395),
 * all rows in one launch chain. */
int vb_sumlogs_rows(vb_ctx* ctx, const double* x, int64_t rows, int64_t n, double* out);

#ifdef __cplusplus
}
#endif
#endif /* VIABEL_AMD_H */
