/*
 * bo_amd.h — C ABI of the MI355X-native GP-predict + acquisition hot path.
 *
 * Drop-in boundary for alebal123bal/BayesOpt_smart's inner loop
 * (bayesopt/bayesian_optimization.py:129-207, the functions it imports by name at
 * :24-42).  Every entry point names the reference function it replaces.
 *
 * Conventions (all entry points):
 *   - plain pointers and sizes; no torch / HIP types in the signatures;
 *   - "device" pointers are HIP device memory owned by the caller (the library never
 *     allocates or frees caller memory); "host" pointers are read during the call;
 *   - `stream` is a hipStream_t passed as void* (NULL = the null stream); every call is
 *     asynchronous on that stream unless stated otherwise;
 *   - the return value is a bo_status; no C++ exception crosses the ABI.
 *   - all floating point is IEEE binary64 (the reference's NUMBA_FLOAT_TYPE,
 *     bayesopt/config.py:54); the reference's float32 branch (config.py:57-61: jitters 1e-3 /
 *     1e-4, variance floor 1e-6) is reachable through the *_jitter entry points and
 *     BO_PREDICT_F32_FLOOR.
 */
#ifndef BO_AMD_H
#define BO_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BO_ABI_VERSION 5
#define BO_MAX_OBJ 8      /* objectives per call                              */
#define BO_MAX_DIM 8      /* input dimensions                                 */
#define BO_MAX_TOPQ 48    /* batch size of the fused top-q selection          */

typedef enum bo_status {
  BO_OK = 0,
  BO_ERR_ARG = 1,          /* invalid argument / shape                          */
  BO_ERR_UNSUPPORTED = 2,  /* valid but outside what this build implements       */
  BO_ERR_WORKSPACE = 3,    /* workspace missing or too small                     */
  BO_ERR_HIP = 4,          /* a HIP runtime call failed                          */
  BO_ERR_NOT_PD = 5,       /* matrix not positive definite (np.linalg.LinAlgError) */
  BO_ERR_SINGULAR = 6      /* singular matrix (np.linalg.LinAlgError)            */
} bo_status;

typedef enum bo_cand_kind {
  BO_CAND_I64 = 0,   /* explicit candidates, int64 [n_cand][dim] (the reference's input_space) */
  BO_CAND_F64 = 1,   /* explicit candidates, f64 [n_cand][dim] (e.g. a Sobol set)            */
  BO_CAND_GRID = 2,  /* implicit 'ij' integer grid: bayesian_optimization.py:338-340           */
  BO_CAND_SOBOL = 3  /* implicit unscrambled Sobol sequence, generated on the device from the
                        global index: point i of scipy.stats.qmc.Sobol(dim, scramble=False,
                        bits) mapped to lo + u * scale (bit-identical; `cand` is a HOST
                        bo_sobol_desc*, read during the call).  A candidate-shard generates its
                        own index range: no candidate array exists in HBM or crosses PCIe.   */
} bo_cand_kind;

/* Parameters of kind BO_CAND_SOBOL: coordinate k of point i is lo[k] + u_k(i) * scale[k]
 * (multiply, then add: numpy's `lo + sample * (hi - lo)`), u_k(i) = x_k(i) / 2^bits with
 * x_k(i) = XOR of the direction numbers v_kj over the set bits j of gray(i) = i ^ (i >> 1)
 * (Joe-Kuo direction numbers, the table scipy ships).  bits in [1, 32]; i < 2^bits. */
typedef struct bo_sobol_desc {
  int32_t bits;
  int32_t reserved;
  double lo[BO_MAX_DIM];
  double scale[BO_MAX_DIM];
} bo_sobol_desc;

/* HOST (no device, synchronous): coordinates out[t][k] (t < n, k < dim) of the Sobol points with
 * global indices idx[t], bit-identical to the device generator; the direction numbers
 * v[dim][bits] (uint32, row-major). */
int bo_sobol_points(const bo_sobol_desc* s, int32_t dim, const int64_t* idx, int64_t n, double* out);
int bo_sobol_direction_numbers(int32_t dim, int32_t bits, uint32_t* out);

int bo_abi_version(void);
const char* bo_status_string(int status);
/* number of HIP devices visible; <0 on HIP error (no compute launched) */
int bo_device_count(void);

/* ------------------------------------------------------------------------------------
 * Fused GP predict + acquisition + top-q:   replaces, for one candidate shard,
 *   update_k_star     bayesopt/numba_kernels.py:406-442
 *   update_mean       bayesopt/numba_kernels.py:450-488
 *   update_variance   bayesopt/numba_kernels.py:491-535
 *   standardize_objectives                 :538-570
 *   update_ucb        bayesopt/acquisition.py:55-81
 *   update_hypervolume_improvement         bayesopt/acquisition.py:89-108
 *   select_next_batch bayesopt/acquisition.py:116-144 (local top-q with exclusion)
 * No N x M k_star array is materialised: candidate tiles are generated, contracted
 * against K^-1 on the f64 matrix cores and reduced to outputs in one pass.
 * ---------------------------------------------------------------------------------- */
/* Variance formulation.  DENSE: q = k^T (K^-1 k) exactly as update_variance (2N^2 flops per
 * candidate and objective).  AUTO (default): q = 2 k^T (U k) with U the upper triangle of
 * sym(K^-1) = (K^-1 + K^-T)/2 and its diagonal halved -- the same quadratic form (k^T A k =
 * k^T sym(A) k), half the matrix-core work, no factorisation and no positive-definiteness
 * requirement. */
/* mode is a bit set: BO_PREDICT_DENSE forces the dense formulation; BO_PREDICT_NO_SEPARABLE
 * disables the integer-grid fast K* generation (K* = pv * R(f) * T[x_last - c_last], an exp
 * table over the last grid axis; used only when the candidates are a grid whose last axis is
 * a multiple of 16 and every training point's last coordinate is an integer on that axis,
 * checked on the device).  BO_PREDICT_FP32 (BASELINE config C5, "fp32 with fp64 reference
 * check"): K* and the upper-form contraction in f32 on v_mfma_f32_16x16x4_f32, the mean and
 * quadratic form accumulated in f32, everything after them in f64; every candidate evaluates
 * exp (no grid table); DENSE / NO_SEPARABLE are ignored with it. */
/* BO_PREDICT_F32_FLOOR: the posterior variance floor of the reference's float32 branch,
 * MIN_VARIANCE = 1e-6 (config.py:57-61), instead of the fp64 branch's 1e-10 (:63-66). */
typedef enum bo_predict_mode {
  BO_PREDICT_AUTO = 0,
  BO_PREDICT_DENSE = 1,
  BO_PREDICT_NO_SEPARABLE = 2,
  BO_PREDICT_FP32 = 4,
  BO_PREDICT_F32_FLOOR = 8
} bo_predict_mode;

typedef struct bo_predict_desc {
  int32_t n_obj;              /* objectives (<= BO_MAX_OBJ)                                 */
  int32_t dim;                /* input dimensions (<= BO_MAX_DIM)                            */
  int64_t n_train;            /* N = current_eval                                            */
  const double* x_train;      /* device [n_train][dim] (x_vector[:N])                        */
  const double* y_train;      /* device, y_vector rows with row stride ld_y (>= n_obj)        */
  int64_t ld_y;
  const double* kinv;         /* device [n_obj][ld_k][ld_k]; leading N x N block = invert_k() */
  int64_t ld_k;
  int32_t cand_kind;          /* bo_cand_kind                                                 */
  int32_t mode;               /* bo_predict_mode                                              */
  const void* cand;           /* device [n_cand][dim] (kinds I64/F64); host bo_sobol_desc* (SOBOL) */
  int64_t n_cand;             /* candidates scored by this call                               */
  int64_t cand_offset;        /* global index of this call's first candidate                  */
  int64_t grid_lo[BO_MAX_DIM];     /* kind GRID: lower bound of each axis                    */
  int64_t grid_shape[BO_MAX_DIM];  /* kind GRID: points per axis (axis dim-1 fastest)        */
  const double* excl_points;  /* device [n_excl][dim] evaluated points; NULL = x_train        */
  int64_t n_excl;
  double prior_mean[BO_MAX_OBJ];
  double prior_var[BO_MAX_OBJ];
  double length_scale[BO_MAX_OBJ];
  double beta[BO_MAX_OBJ];
  /* optional device outputs (NULL = not written); per-objective arrays are
   * [n_obj][ld_out] and this call writes columns [0, n_cand) of each row. */
  double* mu;                 /* mu_objectives             */
  double* var;                /* variance_objectives       */
  double* std_mu;             /* std_mu_objectives         */
  double* std_var;            /* std_variance_objectives   */
  double* ucb;                /* ucb                       */
  double* acq;                /* acquisition_values [n_cand] */
  int64_t ld_out;
  /* top-q selection of this call's candidates (0 = none), ordered NaN first, then
   * descending acquisition value, ties by ascending global index; candidates equal to
   * an evaluated point are skipped.  Device outputs. */
  int32_t topq;
  int32_t reserved1;
  double* top_val;            /* [topq]                                          */
  int64_t* top_idx;           /* [topq] global candidate index, -1 = no candidate */
} bo_predict_desc;

/* bytes of device workspace bo_predict_acquire needs for `desc` (0 on bad args) */
size_t bo_predict_workspace_size(const bo_predict_desc* desc);
int bo_predict_acquire(const bo_predict_desc* desc, void* workspace, size_t workspace_bytes,
                       void* stream);

/* ------------------------------------------------------------------------------------
 * Unfused drop-ins with the reference's in-place semantics (device arrays).
 * ---------------------------------------------------------------------------------- */

/* update_k  bayesopt/numba_kernels.py:329-367: kernel_matrix[o][i][j] for
 * last_eval <= i < current_eval, i <= j < current_eval, then mirror.
 * kernel_matrix: device [n_obj][ld][ld]; x: device [*][dim]. prior_variance/length_scales host. */
int bo_update_k(double* kernel_matrix, int64_t ld, int32_t n_obj, const double* x, int32_t dim,
                int64_t last_eval, int64_t current_eval, const double* prior_variance,
                const double* length_scales, void* stream);

/* update_k_star  bayesopt/numba_kernels.py:406-442: k_star device [n_obj][ld_rows][n_cand];
 * candidates: explicit int64/f64 device array (kind I64/F64). Rows [last_eval, current_eval). */
int bo_update_k_star(double* k_star, int64_t ld_rows, int32_t n_obj, const double* x, int32_t dim,
                     int32_t cand_kind, const void* cand, int64_t n_cand, int64_t last_eval,
                     int64_t current_eval, const double* prior_variance,
                     const double* length_scales, void* stream);

/* update_mean + update_variance (numba_kernels.py:450-535) from a materialised k_star
 * (device [n_obj][ld_rows][n_cand]).  mu/var: device [n_obj][n_cand] (either may be NULL). */
int bo_update_mean_variance(double* mu, double* var, const double* k_star, int64_t ld_rows,
                            int32_t n_obj, int64_t n_cand, const double* kinv, int64_t ld_k,
                            const double* y, int64_t ld_y, int64_t current_eval,
                            const double* prior_mean, const double* prior_variance,
                            void* workspace, size_t workspace_bytes, void* stream);
size_t bo_update_mean_variance_workspace_size(int32_t n_obj, int64_t current_eval);

/* standardize_objectives + update_ucb + update_hypervolume_improvement
 * (numba_kernels.py:538-570, acquisition.py:55-108): elementwise over [n_obj][n_cand].
 * Any output may be NULL. */
int bo_standardize_ucb_hvi(double* std_mu, double* std_var, double* ucb, double* acq,
                           const double* mu, const double* var, int32_t n_obj, int64_t n_cand,
                           const double* prior_mean, const double* prior_variance,
                           const double* betas, void* stream);

/* update_ucb  bayesopt/acquisition.py:55-81: ucb[o][i] = mu[o][i] + betas[o] sqrt(|var[o][i]|)
 * (arrays [n_obj][n]; betas host). */
int bo_update_ucb(double* ucb, const double* mu, const double* var, int32_t n_obj, int64_t n,
                  const double* betas, void* stream);

/* update_hypervolume_improvement  bayesopt/acquisition.py:89-108: acq[i] = sum_o ucb[o][i]. */
int bo_update_hypervolume_improvement(double* acq, const double* ucb, int32_t n_obj, int64_t n,
                                      void* stream);

/* select_next_batch  bayesopt/acquisition.py:116-144 over an acquisition array:
 * top-q (q <= BO_MAX_TOPQ) skipping candidates equal to any evaluated point. */
int bo_select_topq(const double* acq, int64_t n_cand, int32_t cand_kind, const void* cand,
                   const int64_t* grid_lo, const int64_t* grid_shape, int32_t dim,
                   int64_t cand_offset, const double* excl_points, int64_t n_excl, int32_t topq,
                   double* top_val, int64_t* top_idx, void* workspace, size_t workspace_bytes,
                   void* stream);
size_t bo_select_topq_workspace_size(int64_t n_cand, int32_t topq);

/* The exclusion of acquisition.py:137-139 ("candidate equal in every coordinate to an evaluated
 * point") as a candidate bit mask, kept across iterations (ABI 5).  The evaluated set grows by
 * q points per iteration, so the mask is built once and then extended by the new rows only.
 *
 * bo_excl_mask_update: sets bit j (word j / 32, bit j % 32) of `mask` (device, bo_excl_mask_bytes
 * (n_cand)) for every local candidate j (global index cand_offset + j) equal to one of the rows
 * excl_points[first_excl .. n_excl) (device [n_excl][dim]); clear != 0 zeroes the mask first.
 * Candidates as bo_select_topq's.  Grid candidates: one thread per point, the grid index found
 * arithmetically.  Other kinds: a hash set of the new rows in `workspace`
 * (bo_excl_mask_workspace_size(n_excl - first_excl) bytes; unused for a grid) and one pass over
 * the candidates.
 * bo_select_topq_masked / bo_hvi_select_topq_masked: bo_select_topq / bo_hvi_select_topq with
 * the mask in place of the points: an excluded element is dropped as it is loaded (no hash build,
 * no probes).  Same results as the unmasked calls given the same evaluated points. */
size_t bo_excl_mask_bytes(int64_t n_cand);
size_t bo_excl_mask_workspace_size(int64_t n_excl);
int bo_excl_mask_update(uint32_t* mask, int64_t n_cand, int32_t cand_kind, const void* cand,
                        const int64_t* grid_lo, const int64_t* grid_shape, int32_t dim,
                        int64_t cand_offset, const double* excl_points, int64_t first_excl,
                        int64_t n_excl, int32_t clear, void* workspace, size_t workspace_bytes,
                        void* stream);
int bo_select_topq_masked(const double* acq, int64_t n_cand, int64_t cand_offset,
                          const uint32_t* mask, int32_t topq, double* top_val, int64_t* top_idx,
                          void* workspace, size_t workspace_bytes, void* stream);

/* is_pareto_efficient  bayesopt/pareto.py:12-45: mask[i] = 1 iff no row j dominates row i
 * (maximisation, weak dominance; NaN rows never dominate nor are dominated).
 * y: device [n][n_obj] row-major; mask: device uint8 [n]. Bit-exact. */
int bo_pareto_mask(const double* y, int64_t n, int32_t n_obj, uint8_t* mask, void* stream);

/* Exact hypervolume improvement (opt-in acquisition; the reference's
 * update_hypervolume_improvement, acquisition.py:89-108, is the sum of UCBs above and stays the
 * default).  The reference point it would use is bayesian_optimization.py:65 / :425 (unused
 * there).  Maximisation.
 *
 * bo_hvi_boxes (HOST, synchronous, no device memory): decomposes the region above ref_point not
 * dominated by `front` (host [n][n_obj] row-major; rows with NaN / not strictly above ref_point
 * are ignored, dominated rows are harmless) into disjoint boxes, host [*][2 n_obj]
 * (lower[n_obj], upper[n_obj]; upper may be +inf).  Writes the count to *n_boxes; returns
 * BO_ERR_WORKSPACE (count still written) when it exceeds `capacity`.  n_obj <= 4.
 *
 * bo_hypervolume_improvement_exact: acq[i] = sum_b prod_k max(0, min(p_k, upper_bk) - lower_bk)
 * = HV(front u {p}) - HV(front), p_k = shift[k] + scale[k] * ucb[k][i] (ucb device
 * [n_obj][ld], the standardised UCB; shift = prior mean, scale = sqrt(prior variance) give
 * mu + beta sigma in objective units).  boxes: device copy of bo_hvi_boxes' output.  NaN in p
 * gives NaN (selected first, as NaN is by the reference's argsort).  shift/scale host. */
/* bo_hvi_select_topq: the exact HVI of bo_hypervolume_improvement_exact written into acq AND
 * the top-q selection of bo_select_topq over it, in one pass over the UCB arrays, any
 * q <= BO_MAX_TOPQ, n_obj <= 4.  Arguments as those two functions'; workspace
 * bo_select_topq_workspace_size(n_cand, topq). */
int bo_hvi_select_topq(double* acq, const double* ucb, int64_t ld, int64_t n_cand, int32_t n_obj,
                       const double* shift, const double* scale, const double* boxes,
                       int64_t n_boxes, int32_t cand_kind, const void* cand, const int64_t* grid_lo,
                       const int64_t* grid_shape, int32_t dim, int64_t cand_offset,
                       const double* excl_points, int64_t n_excl, int32_t topq, double* top_val,
                       int64_t* top_idx, void* workspace, size_t workspace_bytes, void* stream);
int bo_hvi_select_topq_masked(double* acq, const double* ucb, int64_t ld, int64_t n_cand,
                              int32_t n_obj, const double* shift, const double* scale,
                              const double* boxes, int64_t n_boxes, int64_t cand_offset,
                              const uint32_t* mask, int32_t topq, double* top_val,
                              int64_t* top_idx, void* workspace, size_t workspace_bytes,
                              void* stream);
/* bo_box_volume_sum: out[0] (device) = sum_b prod_k max(0, min(upper_bk, upper[k]) - lower_bk)
 * over `boxes` (device, bo_hvi_boxes layout): the volume of the boxes clipped above at `upper`
 * (host [n_obj]).  With the boxes of the region a front does NOT dominate and upper = the
 * front's per-objective maximum, HV(front) = prod_k (upper_k - ref_k) - that volume; a rank's
 * share of the boxes gives its partial sum for the all-reduce "hypervolume accumulator"
 * (bayesopt_smart_amd/distributed.py).  Deterministic (one workgroup, fixed-order tree). */
int bo_box_volume_sum(const double* boxes, int64_t n_boxes, int32_t n_obj, const double* upper,
                      double* out, void* stream);
int bo_hvi_boxes(const double* front, int64_t n, int32_t n_obj, const double* ref_point,
                 double* boxes, int64_t capacity, int64_t* n_boxes);
int bo_hypervolume_improvement_exact(double* acq, const double* ucb, int64_t ld, int64_t n,
                                     int32_t n_obj, const double* shift, const double* scale,
                                     const double* boxes, int64_t n_boxes, void* stream);

/* ------------------------------------------------------------------------------------
 * GP fit on device.
 * ---------------------------------------------------------------------------------- */

/* invert_k  bayesopt/numba_kernels.py:370-403: out[o] = inv(K[o][:N,:N] + 1e-6 I) (the
 * reference's LAPACK gesv with the identity): a blocked Cholesky when K is symmetric, followed
 * by one Newton step X + X (I - (K + 1e-6 I) X) on the matrix cores (the residual of gesv's
 * backward-stable solves), or the blocked LU with partial pivoting (getrf's row choice) + getrs
 * when the Cholesky fails or K is not symmetric.  kernel_matrix device [n_obj][ld][ld];
 * out device [n_obj][n][n]. Returns BO_ERR_SINGULAR on an exactly singular pivot.
 * Synchronous (the status depends on the factorisation). */
int bo_invert_k(double* out, const double* kernel_matrix, int64_t ld, int32_t n_obj, int64_t n,
                void* workspace, size_t workspace_bytes, void* stream);
/* bo_invert_k_jitter with per-objective path control and report (ABI 4).  lu_hint (host
 * [n_obj], may be NULL): when EVERY objective's entry is non-zero the Cholesky attempt is skipped
 * and all of them go straight to the blocked LU -- the caller's knowledge that the previous
 * iteration's Cholesky failed for them (a drop-in loop at Powell-fitted length scales, where
 * cond(K + 1e-6 I) > 1e16).  The result is the LU path's either way.  path_out
 * (host [n_obj], may be NULL): 0 Cholesky (+ Newton step), 1 blocked LU, 2 Gauss-Jordan. */
int bo_invert_k_ex(double* out, const double* kernel_matrix, int64_t ld, int32_t n_obj, int64_t n,
                   double jitter, const int32_t* lu_hint, int32_t* path_out, void* workspace,
                   size_t workspace_bytes, void* stream);
/* Per-objective counts of the paths bo_invert_k took since the library was loaded (process-wide,
 * host counters): counts[0] Cholesky, [1] blocked LU (Cholesky failed or K not symmetric;
 * N <= 2048), [2] Gauss-Jordan (the same above N = 2048).  Diagnostics for the fallback's
 * frequency. */
int bo_invert_k_path_counts(int64_t* counts);
/* bo_invert_k with the diagonal jitter given: KERNEL_JITTER of config.py:57-66 (1e-6 in the fp64
 * branch, which bo_invert_k uses; 1e-3 in the float32 branch). */
int bo_invert_k_jitter(double* out, const double* kernel_matrix, int64_t ld, int32_t n_obj, int64_t n,
                       double jitter, void* workspace, size_t workspace_bytes, void* stream);
size_t bo_invert_k_workspace_size(int32_t n_obj, int64_t n);
/* Process-wide counts of the factorisation schedules bo_invert_k / bo_compute_mll* ran:
 * counts[0] the persistent launch (one task-queue kernel: panels and trailing-update tiles hand
 * off through flags), [1] one launch per 32-column step (N > 1536 by default -- more than 48
 * column blocks of 32; the environment variable BO_FIT_PERSIST_MAX_NBT sets that block count --
 * or BO_FIT_PATH=launches), [2] persistent launches that gave up a wait (bounded spin) and were
 * rerun step by step. */
int bo_fit_path_counts(int64_t* counts);

/* compute_mll  bayesopt/numba_kernels.py:152-235 (Gram rebuilt into kernel_matrix first, as
 * the reference does).  Writes the summed MLL to *mll_out (host).  Returns BO_ERR_NOT_PD when
 * a Cholesky pivot is not positive.  Synchronous. */
int bo_compute_mll(double* mll_out, const double* x, int32_t dim, const double* y, int64_t ld_y,
                   double* kernel_matrix, int64_t ld, int32_t n_obj, const double* prior_mean,
                   const double* prior_variance, const double* length_scales,
                   int64_t current_eval, void* workspace, size_t workspace_bytes, void* stream);
/* The per-objective terms of compute_mll: mll_obj[o] (host, [n_obj]); compute_mll is their sum in
 * objective order.  Each term depends on (x, y[:, o], pm[o], ls[o]) only -- the correlation
 * matrix K / pv does not depend on pv -- so a caller may memoise terms across calls (the Powell
 * driver of bayesopt_smart_amd.kernels does).  Same arguments and errors as bo_compute_mll. */
int bo_compute_mll_each(double* mll_obj, const double* x, int32_t dim, const double* y, int64_t ld_y,
                        double* kernel_matrix, int64_t ld, int32_t n_obj, const double* prior_mean,
                        const double* prior_var, const double* length_scale, int64_t n,
                        void* workspace, size_t workspace_bytes, void* stream);
/* bo_compute_mll_each with the correlation matrix's jitter given: CHOLESKY_JITTER of
 * config.py:57-66 (1e-8 in the fp64 branch, which bo_compute_mll_each uses; 1e-4 in float32). */
int bo_compute_mll_each_jitter(double* mll_obj, const double* x, int32_t dim, const double* y, int64_t ld_y,
                               double* kernel_matrix, int64_t ld, int32_t n_obj, const double* prior_mean,
                               const double* prior_var, const double* length_scale, int64_t n, double jitter,
                               void* workspace, size_t workspace_bytes, void* stream);
size_t bo_compute_mll_workspace_size(int32_t n_obj, int64_t n);

/* ------------------------------------------------------------------------------------
 * The fit's driver, native (HOST code calling the device MLL): scipy.optimize.minimize(
 * method="Powell", bounds=...) as optimize_hyperparams_mll calls it (numba_kernels.py:238-321,
 * :305-315), restated from scipy 1.15's _minimize_powell / _linesearch_powell / _line_for_search /
 * _minimize_scalar_bounded operation for operation (tan/atan from the C library).
 * ---------------------------------------------------------------------------------- */
/* objective: *f = f(x[0..n)); a non-zero return aborts the minimisation with that status */
typedef int (*bo_objective_fn)(const double* x, int32_t n, double* f, void* user);
/* tan (which = 0) / atan (which = 1) of the one-sided line searches' transform; NULL = the C
 * library's.  A caller wanting scipy's evaluation points bit for bit passes numpy's (its SIMD
 * tan differs from the C library's in the last bit for ~0.5 % of arguments). */
typedef double (*bo_trig_fn)(double x, int32_t which);
typedef struct bo_powell_result {
  double fun;             /* final objective value                                          */
  int64_t nfev;           /* objective evaluations                                          */
  int64_t nit;            /* Powell iterations                                              */
  int64_t device_calls;   /* bo_optimize_hyperparams_mll: device MLL calls (memo misses)     */
  int32_t warnflag;       /* scipy's status: 0 success, 1 maxfev, 2 maxiter, 3 nan, 4 bounds  */
  int32_t reserved;
} bo_powell_result;
/* Minimise fn from x (in: x0, out: the result) within lb <= x <= ub (host [n]; +-inf allowed);
 * maxiter / maxfev < 0 = None (scipy's defaults).  direc (optional, host [n][n]) receives the
 * final direction set.  BO_ERR_UNSUPPORTED when a line search is unbounded in both directions
 * (scipy's bracketing Brent; the fit's bounds never need it). */
int bo_powell_minimize(bo_objective_fn fn, void* user, double* x, int32_t n, const double* lb,
                       const double* ub, double xtol, double ftol, int64_t maxiter, int64_t maxfev,
                       bo_trig_fn trig, double* direc, bo_powell_result* res);
/* optimize_hyperparams_mll (numba_kernels.py:238-321) as ONE call: Powell over [ls..., pv...] from
 * the given values (host, updated in place on success), bounds [min_bound, inf), maximising the
 * device MLL (bo_compute_mll_each_jitter; each per-objective term memoised per distinct ls_o, a
 * device call only for the objectives whose ls changed).  kernel_matrix ends as the Gram of the
 * last evaluated hyper-parameters (the reference's side effect).  Workspace:
 * bo_compute_mll_workspace_size(n_obj, n).  Synchronous. */
int bo_optimize_hyperparams_mll(const double* x, int32_t dim, const double* y, int64_t ld_y,
                                double* kernel_matrix, int64_t ld, int32_t n_obj, const double* prior_mean,
                                double* prior_variance, double* length_scales, int64_t n, double jitter,
                                double xtol, double ftol, int64_t maxiter, double min_bound, bo_trig_fn trig,
                                void* workspace, size_t workspace_bytes, void* stream, bo_powell_result* res,
                                double* direc);

/* ------------------------------------------------------------------------------------
 * Measurement hooks (bench.py): while enabled, each fused predict kernel launch (the
 * dominant kernel of bo_predict_acquire) is bracketed by HIP events on its stream;
 * bo_profile_stop synchronises them and returns the summed kernel time.
 * ---------------------------------------------------------------------------------- */
int bo_profile_start(int max_launches);
int bo_profile_stop(double* total_ms, int* launches);

/* ------------------------------------------------------------------------------------
 * Self test: D[16][16] = A[16][4] * B[4][16] on one f64 MFMA (layout check). Device ptrs.
 * ---------------------------------------------------------------------------------- */
int bo_selftest_mfma_f64(const double* a16x4, const double* b4x16, double* d16x16, void* stream);
/* the same on one v_mfma_f32_16x16x4_f32 (the BO_PREDICT_FP32 kernel's layout). Device ptrs. */
int bo_selftest_mfma_f32(const float* a16x4, const float* b4x16, float* d16x16, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* BO_AMD_H */
