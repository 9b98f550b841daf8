/*
 * cpu_ref.c -- C/OpenMP restatement of the reference's GP-predict + acquisition chain, used as
 * the timed CPU baseline of bench.py (kind "port").  TEST / MEASUREMENT INFRASTRUCTURE ONLY:
 * nothing in bayesopt_smart_amd links or calls it.
 *
 * It keeps the reference's algorithm and data flow (alebal123bal/BayesOpt_smart,
 * bayesopt/bayesian_optimization.py:145-207), parallel over candidates the way the Numba path
 * is (prange, numba_kernels.py:432), in candidate blocks so the k_star block stays in cache:
 *   update_k_star        numba_kernels.py:406-442   K*[o][e][i] = pv exp(-0.5 |x_e - c_i|^2 / ls^2)
 *   update_mean          numba_kernels.py:450-488   mu = pm + K*^T (K^-1 (y - pm))
 *   update_variance      numba_kernels.py:491-535   Z = K^-1 K* (the reference's DGEMM, :521),
 *                                                   q_i = sum_e K*[e][i] Z[e][i] (:525-529),
 *                                                   var = max(pv - q, 1e-10)
 *   standardize_objectives numba_kernels.py:538-570
 *   update_ucb / update_hypervolume_improvement   acquisition.py:55-108
 *   select_next_batch    acquisition.py:116-144     full descending sort, skip evaluated points
 * Pinned against the numpy oracle (oracle_np.py, itself pinned to the reference's outputs) by
 * tests/test_oracle_golden.py::test_cpu_ref_matches_oracle.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <omp.h>

#define CB 128 /* candidates per block */

typedef double v4d __attribute__((vector_size(32)));

/* System DGEMM (cblas_dgemm with 64-bit integers: numpy's bundled OpenBLAS, the BLAS the
 * reference's np.dot / Numba would call), installed by oracle/cpu_ref.py; NULL -> the built-in
 * AVX2 register-tiled loop below. */
typedef void (*dgemm_fn)(int order, int ta, int tb, long m, long n, long k, double alpha,
                         const double* a, long lda, const double* b, long ldb, double beta,
                         double* c, long ldc);
static dgemm_fn g_dgemm = 0;
void bo_cpu_set_dgemm(void* fn) { g_dgemm = (dgemm_fn)fn; }
int bo_cpu_has_dgemm(void) { return g_dgemm != 0; }

static void block(int n, int d, int n_obj, const double* x, const double* cand, long i0, int cb,
                  const double* kinv, const double* alpha, const double* pm, const double* pv,
                  const double* ls, const double* beta, double* ks, double* z, double* mu,
                  double* var, double* ucb, double* acq, long m_stride) {
  double acc_b[CB];
  for (int i = 0; i < cb; ++i) acc_b[i] = 0.0;
  for (int o = 0; o < n_obj; ++o) {
    const double nh = 0.5 / (ls[o] * ls[o]);
    /* k_star block [n][cb] */
    for (int e = 0; e < n; ++e) {
      const double* xe = x + (long)e * d;
      double* kr = ks + (long)e * CB;
      for (int i = 0; i < cb; ++i) {
        const double* ci = cand + (i0 + i) * d;
        double sq = 0.0;
        for (int k = 0; k < d; ++k) {
          const double df = xe[k] - ci[k];
          sq += df * df;
        }
        kr[i] = pv[o] * exp(-sq * nh);
      }
    }
    /* Z = K^-1 K* (the reference's DGEMM): 8-candidate strips (a 32 KiB K* strip stays in
     * L1) x 6-row register tiles of K^-1 (12 AVX2 accumulators) */
    const double* w = kinv + (long)o * n * n;
    if (g_dgemm) /* row-major Z[n][CB] = K^-1[n][n] . K*[n][CB] */
      g_dgemm(101, 111, 111, n, cb, n, 1.0, w, n, ks, CB, 0.0, z, CB);
    else
    for (int i0 = 0; i0 < CB; i0 += 8) {
      int e = 0;
      for (; e + 6 <= n; e += 6) {
        const double* w0 = w + (long)e * n;
        v4d acc[6][2];
        for (int r = 0; r < 6; ++r) acc[r][0] = acc[r][1] = (v4d){0.0, 0.0, 0.0, 0.0};
        for (int f = 0; f < n; ++f) {
          v4d k0, k1;
          memcpy(&k0, ks + (long)f * CB + i0, sizeof(k0));
          memcpy(&k1, ks + (long)f * CB + i0 + 4, sizeof(k1));
          for (int r = 0; r < 6; ++r) {
            const double b = w0[(long)r * n + f];
            const v4d bb = {b, b, b, b};
            acc[r][0] += bb * k0;
            acc[r][1] += bb * k1;
          }
        }
        for (int r = 0; r < 6; ++r) memcpy(z + (long)(e + r) * CB + i0, acc[r], sizeof(acc[r]));
      }
      for (; e < n; ++e) {
        double* zr = z + (long)e * CB + i0;
        for (int i = 0; i < 8; ++i) zr[i] = 0.0;
        const double* wr = w + (long)e * n;
        for (int f = 0; f < n; ++f)
          for (int i = 0; i < 8; ++i) zr[i] += wr[f] * ks[(long)f * CB + i0 + i];
      }
    }
    /* mu, q (e ascending per candidate, like the reference's serial loop), epilogue */
    const double* al = alpha + (long)o * n;
    const double rpv = sqrt(pv[o]);
    for (int i = 0; i < cb; ++i) {
      double mp = 0.0, q = 0.0;
      for (int e = 0; e < n; ++e) {
        mp += ks[(long)e * CB + i] * al[e];
        q += ks[(long)e * CB + i] * z[(long)e * CB + i];
      }
      const double muv = pm[o] + mp;
      double v = pv[o] - q;
      if (v < 1e-10) v = 1e-10;
      if (mu) mu[(long)o * m_stride + i0 + i] = muv;
      if (var) var[(long)o * m_stride + i0 + i] = v;
      const double smu = (muv - pm[o]) / rpv, svar = v / pv[o];
      const double u = smu + beta[o] * sqrt(fabs(svar));
      if (ucb) ucb[(long)o * m_stride + i0 + i] = u;
      acc_b[i] = (o == 0) ? u : acc_b[i] + u;
    }
  }
  for (int i = 0; i < cb; ++i) acq[i0 + i] = acc_b[i];
}

/* Scores candidates [0, m) (f64 [m][d]); mu/var/ucb [n_obj][m] optional, acq [m] required.
 * kinv [n_obj][n][n]; y [n][n_obj].  Returns 0. */
int bo_cpu_predict_acquire(int n, int d, int n_obj, const double* x, const double* y,
                           const double* cand, long m, const double* kinv, const double* pm,
                           const double* pv, const double* ls, const double* beta, double* mu,
                           double* var, double* ucb, double* acq, int threads) {
  double* alpha = (double*)malloc(sizeof(double) * n_obj * n);
  for (int o = 0; o < n_obj; ++o)
    for (int e = 0; e < n; ++e) {
      double s = 0.0;
      for (int f = 0; f < n; ++f) s += kinv[((long)o * n + e) * n + f] * (y[(long)f * n_obj + o] - pm[o]);
      alpha[(long)o * n + e] = s;
    }
  const long nblk = (m + CB - 1) / CB;
#pragma omp parallel num_threads(threads)
  {
    double* ks = (double*)malloc(sizeof(double) * n * CB);
    double* z = (double*)malloc(sizeof(double) * n * CB);
#pragma omp for schedule(dynamic, 4)
    for (long b = 0; b < nblk; ++b) {
      const long i0 = b * CB;
      const int cb = (int)(m - i0 < CB ? m - i0 : CB);
      block(n, d, n_obj, x, cand, i0, cb, kinv, alpha, pm, pv, ls, beta, ks, z, mu, var, ucb, acq, m);
    }
    free(ks);
    free(z);
  }
  free(alpha);
  return 0;
}

/* select_next_batch (acquisition.py:116-144): indices of the first q candidates of the
 * descending order that equal no evaluated point.  NaN first, ties by ascending index. */
static const double* g_acq;
static int cmp_desc(const void* a, const void* b) {
  const long i = *(const long*)a, j = *(const long*)b;
  const double x = g_acq[i], y = g_acq[j];
  const int nx = x != x, ny = y != y;
  if (nx != ny) return nx ? -1 : 1;
  if (!nx && x != y) return x > y ? -1 : 1;
  return (i > j) - (i < j);
}

int bo_cpu_select(const double* acq, const double* cand, long m, int d, const double* excl,
                  long n_excl, int q, long* out) {
  long* idx = (long*)malloc(sizeof(long) * m);
  for (long i = 0; i < m; ++i) idx[i] = i;
  g_acq = acq;
  qsort(idx, m, sizeof(long), cmp_desc);
  int got = 0;
  for (long t = 0; t < m && got < q; ++t) {
    const double* c = cand + idx[t] * d;
    int hit = 0;
    for (long e = 0; e < n_excl && !hit; ++e) {
      int eq = 1;
      for (int k = 0; k < d; ++k) eq = eq && (excl[e * d + k] == c[k]);
      hit = eq;
    }
    if (!hit) out[got++] = idx[t];
  }
  for (int t = got; t < q; ++t) out[t] = -1;
  free(idx);
  return got;
}
