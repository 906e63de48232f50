// vb_internal.hpp — host-side launch interface between the C ABI layer
// (vb_capi.hip) and the kernel translation units.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "vb_gemm.hpp"

namespace vbk {

constexpr int kBlockDMax = 16;  // largest D handled by the block-per-problem kernel

// learning_rate_schedule (vb.py:324-342) evaluated on the device for local step i.
// a, b, start, end are computed on the host with the reference's own float
// expression order; device fp64 division is IEEE, so lr(i) matches bit for bit.
struct LrSched {
  double lr, lr_end, a, b;
  long long start, end;
  int has_end;
  __host__ __device__ double at(long long i) const {
    if (!has_end || i < start) return lr;
    if (i < end) return a / (((b + (double)i) - (double)start) + 1.0);
    return lr_end;
  }
};

// Arguments of the column-pair persistent KLVI kernel (separable targets).
struct SepArgs {
  int D, N, W, n_pairs, n_steps, emit_grad;
  int pd;  // value with the sampled log q (black_box_klvi_pd): 0 off, 1 Gaussian, 2 t family
  long long step0, hist_start;  // local step index of the first step; 3*n_iters//4
  long long rng_step0;          // Philox step counter of the first step
  int n_waves;
  double t_scale, shape;  // t family: sqrt(df/2), df/2
  double eps;             // adagrad epsilon
  LrSched lr;
  double* lam;            // [P]
  double* ring;           // [W][P]
  double* hist;           // [n_hist][P]
  double* vpart;          // [n_steps][n_waves]
  double* grad;           // [P] (emit_grad)
  const double* noise;    // host noise [n_steps][N][D] or null
  uint32_t k0, k1, stream;
  int pairs2, blocks2, blocks1;  // filled by the launcher (2-pair / 1-pair split)
};

// Arguments of the block-per-problem kernel (any target, D <= kBlockDMax).
struct BlockArgs {
  int D, N, W, P, n_steps, emit_grad, chivi;
  int pd;   // KLVI value -(mean log p - mean log q(x)) (black_box_klvi_pd)
  int opt;  // 0 adagrad window (history: post-update, tail quarter); 1 RMSProp-IA, 2 Adam-IA
            // (state in ring rows 0/1, history: pre-update, last n_hist iterations)
  long long step0, hist_start, n_iters, n_hist, rng_step0;
  double alpha;
  double t_scale, shape, t_const, df;  // t family constants
  double eps;
  LrSched lr;
  double* lam;          // [n_problems][P]
  double* ring;         // [n_problems][W][P]
  double* hist;         // [n_problems][n_hist][P]
  double* values;       // [n_problems][n_iters] (indexed by global step)
  double* grad;         // [n_problems][P] (emit_grad)
  const double* noise;  // host noise [n_problems][n_steps][N][D] or null
  // with noise: per-sample log q partials [n_problems][n_steps][N] (sum over the
  // column pairs, without -sum log sigma) from launch_block_predraw, or null
  const double* noise_lq;
  uint32_t k0, k1, stream, stream_stride;
  int pf;   // device-noise rows staged into LDS by a copy wave (VIABEL_AMD_BLOCK_PF, default on);
            // 2: also split rows (two lanes per sample) where block_layout allows them
};

// family kind 0 = mf gaussian, 1 = mf t; target kind per vb_target_kind.
hipError_t launch_sep(int fam, int tgt, bool host_noise, const SepArgs& a, hipStream_t s);
// block step skeleton without draws / target (vb_block_floor)
hipError_t launch_block_floor(int D, int N, bool host_layout, bool chivi, int n_steps, int nprob,
                              double* out, hipStream_t s, int pf = 0);
hipError_t launch_block(int fam, int tgt, bool host_noise, const BlockArgs& a, int n_problems,
                        hipStream_t s);
// whether device-noise blocks of this shape get the copy wave (its LDS ring fits)
bool block_pf_layout(int N, int D, bool need_lq, int pf_mode);
bool target_separable(int tgt);
// Pre-drawn block-kernel noise: the standardized draws of n_steps steps of
// n_problems problems, [q][s][N][D], bit-identical to the block kernel's own
// Philox draws (same counters: pair, sample, rng_step0 + s, stream + q * stride),
// and, when lq is non-null, each sample's log q partial sum [q][s][N].
hipError_t launch_block_predraw(int fam, int D, int N, int n_steps, int n_problems, uint32_t k0,
                                uint32_t k1, uint32_t stream, uint32_t stride,
                                long long rng_step0, double t_scale, double shape, double df,
                                double t_const, double* noise, double* lq, hipStream_t s);

// values[i] = -(c0 + sum_w vpart[s][w]) for i = step0 + s
hipError_t launch_sep_values(const double* vpart, int n_steps, int n_waves, double c0,
                             double* values_at_step0, hipStream_t s);
// out[p] = mean over rows of hist [rows][P]   (per problem block of rows)
hipError_t launch_row_mean(const double* hist, long long rows, long long P, long long n_problems,
                           double* out, hipStream_t s);

// elementwise family helpers
// Bailey t samples of a mean-field t family (the log-weight draws, vbrng.c family 2)
hipError_t launch_sample_bailey(int D, long long m, const double* lam, double df, uint32_t k0,
                                uint32_t k1, uint32_t stream, uint32_t step, double* x,
                                hipStream_t s);
hipError_t launch_sample(int fam, int D, long long n, const double* lam, double t_scale,
                         double shape, const double* noise, uint32_t k0, uint32_t k1,
                         uint32_t stream, uint32_t step, double* x, hipStream_t s);
hipError_t launch_family_logdensity(int fam, int D, long long n, const double* lam, double df,
                                    double t_const, const double* x, double* out, hipStream_t s);
hipError_t launch_target_logdensity(int tgt, int D, long long n, const double* x, double* out,
                                    double* grad, hipStream_t s);
// fused materialised step rows (draw, x, target log p + gradient, optional log q)
// for separable device targets with wide rows; see mfw_rows_kernel.  logp / logq
// receive mfw_rows_parts(D) chunk partials per row, laid out [part][n].
bool mfw_rows_fusable(int tgt, int D, long long n);
int mfw_rows_parts(int D);
hipError_t launch_mfw_rows(int fam, int tgt, int D, long long n, const double* lam, double t_scale,
                           double shape, double df, double t_const, bool with_lq,
                           const double* noise, uint32_t k0, uint32_t k1, uint32_t stream,
                           uint32_t step, double* x, double* grad, double* logp, double* logq,
                           hipStream_t s);
hipError_t launch_log_weights(int fam, int tgt, int D, long long m, const double* lam,
                              double t_scale, double shape, double df, double t_const,
                              const double* noise, uint32_t k0, uint32_t k1, uint32_t stream,
                              uint32_t step, double* lw, double* xs, hipStream_t s, int rows = 1,
                              uint32_t stride = 0);
// scale (nullable): [min(step + 1, W)] window scales, oldest first
hipError_t launch_adagrad_update(long long P, double* lam, const double* g, double* ring, int W,
                                 long long step, double lr, double eps, const double* scale,
                                 hipStream_t s,
                                 double* hrow = nullptr);
// RMSProp-IA / Adam-IA step (opt 1 / 2) on device state [2][P], or (opt 3)
// RMSProp-IA with avg_grad_norm: every coordinate divided by sqrt(eps + norm2);
// old_out (nullable) receives the pre-update parameters.
hipError_t launch_ia_update(int opt, long long P, double* lam, const double* g, double* state,
                            long long step, double lr, double eps, double norm2,
                            double* old_out, hipStream_t s);
// R-hat (functions.py:8-31) of chains [nc][n][P] (row stride P) over n_jobs
// iteration segments [start, start + len) (len even): out [n_jobs][P] (var_hat
// in var_out when non-null).
hipError_t launch_rhat_stats(const double* chains, long long nc, long long n, long long P,
                             long long n_jobs, const long long* start, const long long* len,
                             double* mean_out, double* ss_out, hipStream_t s);
hipError_t launch_rhat_combine(const double* mean, const double* ss, long long nc2, long long P,
                               long long n_jobs, const long long* len, double* var_out,
                               double* rhat_out, hipStream_t s);
// cumulative means (functions.py:68-77) of x[start:, cols] with row stride ld
hipError_t launch_iterate_average(const double* x, long long n, long long ld, long long cols,
                                  long long start, double* out, hipStream_t s);

// bounds
hipError_t bounds_divergence(const double* lw, long long n, double alpha, int has_elbo,
                             double elbo, double* dev_scratch, double* out7_dev, hipStream_t s);
hipError_t bounds_divergence_rows(const double* lw, long long rows, long long n, long long ld,
                                  double alpha, int has_elbo, double elbo, double* scratch,
                                  double* out7, hipStream_t s);
size_t bounds_divergence_scratch_doubles(long long rows);
hipError_t bounds_centered_moments(const double* x, long long n, long long d,
                                   double* dev_scratch, double* out2_dev, hipStream_t s);
hipError_t bounds_covariance(const double* x, long long n, long long d, double* dev_scratch,
                             double* mean_dev, double* cov_dev, hipStream_t s);
size_t bounds_scratch_doubles(long long n, long long d);
size_t bounds_wcov_scratch_doubles(long long n, long long d);
hipError_t bounds_weighted_covariance(const double* x, long long n, long long d, const double* w,
                                      bool logw, int ddof, double* scratch, double* sc_out,
                                      double* mean, double* cov, hipStream_t s);
constexpr int kCovDMax = 64;

// PSIS (vb_psis.hip)
size_t psis_scratch_bytes(long long tail_cap);  // scratch for tails / gpdfit inputs <= tail_cap
long long psis_tail_max();
size_t psis_col_stride(long long tail_cap);      // scratch bytes per column of psis_columns
hipError_t psis_columns(const double* lw, double* out, long long n, int m, long long rs,
                        long long cs, long long Mt, void* scratch, double* k_dev,
                        long long* tail_idx_dev, long long tail_cap, long long* n_tail_dev,
                        hipStream_t s, unsigned* flag_dev = nullptr,
                        unsigned* flag_host = nullptr);
hipError_t psis_gpdfit(const double* x, long long n, void* scratch, double* out4,
                       double* ks_out, double* w_out, hipStream_t s);
hipError_t psis_gpinv(const double* p, long long n, double k, double sigma, double* out,
                      hipStream_t s);
size_t psis_sumlogs_rows_scratch_bytes(long long rows, long long n);
hipError_t psis_sumlogs_rows(const double* x, long long rows, long long n, void* scratch,
                             double* out, hipStream_t s);
hipError_t psis_sumlogs(const double* x, long long n, void* scratch, double* out, hipStream_t s);

}  // namespace vbk

// ---- full-rank Student-t family (vb_fr.hip) ----------------------------------
namespace vbk {

int vb_set_error(int code, const char* fmt, ...);  // defined in vb_capi.hip

constexpr int kFamilyFrT = 2;
constexpr int kTargetCorrGauss = 4;
constexpr int kTargetCallback = 5;
// host model callback (vb_target_callback) + its user pointer
struct HostTarget {
  int (*fn)(void* user, const double* x, int64_t n, int64_t d, double* logp, double* grad);
  void* user;
};
struct FrWork;
// Evaluate a host target on device x [n][D] into device logp [n] / grad [n][D]
// (grad nullable): staged through pinned buffers of the workspace; synchronises.
int host_target_eval(FrWork* W, const HostTarget& t, int D, long long n, const double* x,
                     double* logp, double* grad, hipStream_t st);


struct FrWork;  // per-context workspace + rocBLAS handle
FrWork* fr_work_create();
void fr_work_destroy(FrWork* w);

struct FrSpec {
  int D, N, tgt, chivi, pd;
  double df, t_const, alpha;
  const double* tparams;  // device; corr_gauss: P*[D][D]
  double tconst;          // corr_gauss log normaliser
  HostTarget host;        // tgt == kTargetCallback
};

// All return 0 or a VB_E* code (message via vb_set_error).
int fr_prepare(FrWork* W, int D, const double* lam, hipStream_t st);  // eigh of Sigma
// Newton-Schulz sqrtm; warm: Sigma is close to the previous call's (optimisation run)
int fr_sqrt(FrWork* W, int D, const double* lam, hipStream_t st, bool warm = false,
            const void* owner = nullptr, bool ready = false);
constexpr int kFrNSMax = 40;  // Newton-Schulz iterations launched at most per root
constexpr int kFrPcgMax = 192; // PCG iterations launched at most per gradient
int fr_draw(FrWork* W, int D, long long n, double df, const double* host_eps, uint32_t k0,
            uint32_t k1, uint32_t stream, uint32_t step, const double** s_out,
            const double** z_out, hipStream_t st);
int fr_transform(FrWork* W, int D, long long n, const double* mu, const double* s,
                 const double* z, double* x, hipStream_t st);
int fr_target(FrWork* W, int tgt, int D, long long n, const double* tparams, double tconst,
              const double* x, double* logp, double* G, hipStream_t st);
struct MfUpdate;
// The next step of a fused run: its draws (rng step `step`) and L are prepared by
// this step's last kernel when `prep`.
struct FrNext {
  bool prep;
  uint32_t step;
};
// up (non-null, Philox draws): the windowed adagrad step is fused into the last
// kernel (lam updated in place, ring / history row written; grad keeps only the
// mean part), and with next->prep the step after it is prepared (FrWork).
int fr_value_grad(FrWork* W, const FrSpec& f, const double* lam, const double* host_eps,
                  uint32_t k0, uint32_t k1, uint32_t stream, uint32_t step, double* value,
                  double* grad, hipStream_t st, bool warm = false,
                  const void* owner = nullptr, const MfUpdate* up = nullptr,
                  const FrNext* next = nullptr);
int fr_logdensity(FrWork* W, int D, double df, double t_const, const double* lam, const double* x,
                  long long n, double* out, hipStream_t st);
int fr_log_weights(FrWork* W, const FrSpec& f, const double* lam, long long m,
                   const double* host_eps, uint32_t k0, uint32_t k1, uint32_t stream,
                   uint32_t step, double* lw, double* xs, hipStream_t st);
int fr_moments(FrWork* W, int D, const double* lam, double* sigma, double* eig, hipStream_t st);

// Mean-field families on the materialised path (any D, any objective / target).
struct MfSpec {
  int fam, D, N, tgt, chivi, pd;
  double alpha, t_scale, shape, df, t_const;
  HostTarget host;  // tgt == kTargetCallback
};
// Optional windowed-adagrad step fused into the gradient pass (lam updated in
// place, the step's gradient pushed into ring [W][P], new parameters copied to
// hrow when non-null); same arithmetic as launch_adagrad_update without scales.
struct MfUpdate {
  double* ring;
  int W;
  long long step;
  double lr, eps;
  double* hrow;
};
int mf_wide_value_grad(FrWork* W, const MfSpec& f, const double* lam, const double* host_eps,
                       uint32_t k0, uint32_t k1, uint32_t stream, uint32_t step, double* value,
                       double* grad, hipStream_t st, const MfUpdate* up = nullptr);
int mf_wide_log_weights(FrWork* W, const MfSpec& f, const double* lam, long long m,
                        const double* host_eps, uint32_t k0, uint32_t k1, uint32_t stream,
                        uint32_t step, double* lw, double* xs, hipStream_t st);
// 0, or a VB_E* code with the message set (eigendecomposition / Newton-Schulz /
// PCG failure since the last call); synchronises the stream.
// retry (non-null): a warm Newton-Schulz root that did not converge sets *retry,
// raises the learnt count and returns 0 (the caller runs the steps again).
int fr_info(FrWork* W, hipStream_t st, bool* retry = nullptr);
// Warm state of the next full-rank step (previous root, power vectors, schedule
// block): saved before a run's advance, restored when the advance runs again.
// Peak-rate microbenchmarks (vb_probe.hip): kind 0 HBM copy / 1 HBM read (GB/s,
// n bytes), 2 fp64 MFMA (TFLOP/s), 3 fp64 FMA / 4 u64 multiply VALU issue (G
// wave-instructions/s; n iterations).
int probe_rate(int kind, long long n, int reps, hipStream_t st, double* out);
int fr_warm_save(FrWork* W, hipStream_t st);
int fr_warm_restore(FrWork* W, hipStream_t st);
// Clears the Newton-Schulz floor a rerun set (the rerun's own warm steps have
// taught fr_info the count they need).
void fr_retry_done(FrWork* W);
hipError_t launch_fr_lw(int D, long long m, double df, double t_const, const double* logp,
                        const double* zz, const double* s, const double* scal, double* lw,
                        hipStream_t st);

}  // namespace vbk
