// GP fit on device.
//
//   bo_invert_k     numba_kernels.py:370-403  inv(K + 1e-6 I) -- Gauss-Jordan elimination
//                   with partial pivoting (row interchanges chosen like LAPACK's idamax:
//                   first row of largest |a_ik|), one launch per pivot step, each a pure
//                   function of the previous matrix (ping-pong buffers), columns
//                   unscrambled at the end.  Exactly-zero pivot -> BO_ERR_SINGULAR.
//   bo_compute_mll  numba_kernels.py:152-235  Gram rebuilt with the trial hyper-parameters
//                   (update_k), K/pv + 1e-8 I factored by a right-looking blocked Cholesky
//                   (32x32 blocks: diagonal factor, panel solve and trailing update, one
//                   launch each), then the two triangular solves, log-determinant
//                   and the three MLL terms; a non-positive pivot -> BO_ERR_NOT_PD.
// Both are latency-bound small dense problems (N <= a few thousand); the launches are
// grid-wide per step so the N x N update spreads over every CU.

#include "bo_common.h"

#include <math.h>
#include <string.h>

#include <vector>

namespace {

constexpr int GJ_TILE = 64;   // Gauss-Jordan output tile (64 x 64 per 256-thread block)
constexpr int NB = 32;        // Cholesky block size

// ------------------------------------------------------------------------- inverse
// copy K[o][:n,:n] (leading dim ld) + jitter on the diagonal into a dense n x n buffer
__global__ void jitter_copy_kernel(double* __restrict__ dst, const double* __restrict__ src,
                                   long long ld, int n, int n_obj, double jitter) {
  const long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  const long long per = (long long)n * n;
  if (t >= per * n_obj) return;
  const int o = (int)(t / per);
  const long long r = t - o * per;
  const int i = (int)(r / n), j = (int)(r - (long long)i * n);
  double v = src[(long long)o * ld * ld + (long long)i * ld + j];
  if (i == j) v += jitter;
  dst[t] = v;
}

// One Gauss-Jordan step k on every objective: B = step_k(A).
// pivot p = first argmax_{i>=k} |A[i][k]|; row k of B = row p of A / pivot (entry k = 1/pivot);
// other rows i (source row s = p if i == k... swapped): B[i][j] = a_s[j] - A[s][k] * rowk[j]
// with a_s[k] := 0 -- the in-place elimination written out-of-place.
__global__ __launch_bounds__(256) void gj_step_kernel(double* __restrict__ B,
                                                      const double* __restrict__ A, int n, int k,
                                                      int* __restrict__ piv,
                                                      int* __restrict__ status) {
  __shared__ double col[2048 + 64];
  __shared__ double red_v[256];
  __shared__ int red_i[256];
  __shared__ double rowk[GJ_TILE];
  const int o = blockIdx.z;
  const double* a = A + (long long)o * n * n;
  double* b = B + (long long)o * n * n;
  const int tid = threadIdx.x;
  // column k (full) into LDS and the pivot search over rows >= k
  double best = -1.0;
  int bi = n;
  for (int i = tid; i < n; i += 256) {
    const double v = a[(long long)i * n + k];
    col[i] = v;
    if (i >= k) {
      const double av = fabs(v);
      if (av > best) { best = av; bi = i; }   // strided scan: first max per thread
    }
  }
  red_v[tid] = best;
  red_i[tid] = bi;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (tid < s) {
      const double v2 = red_v[tid + s];
      const int i2 = red_i[tid + s];
      if (v2 > red_v[tid] || (v2 == red_v[tid] && i2 < red_i[tid])) { red_v[tid] = v2; red_i[tid] = i2; }
    }
    __syncthreads();
  }
  const int p = red_i[0] < n ? red_i[0] : k;
  const double pivot = col[p];
  if (blockIdx.x == 0 && blockIdx.y == 0 && tid == 0) {
    piv[o * n + k] = p;
    if (pivot == 0.0) atomicOr(status, 1);
  }
  const int c0 = blockIdx.x * GJ_TILE, r0 = blockIdx.y * GJ_TILE;
  // normalised (swapped) pivot row for this tile's columns
  if (tid < GJ_TILE) {
    const int j = c0 + tid;
    if (j < n) rowk[tid] = (j == k) ? 1.0 / pivot : a[(long long)p * n + j] / pivot;
  }
  __syncthreads();
  const int jl = tid & 63;
  const int j = c0 + jl;
  if (j >= n) return;
  for (int ii = tid >> 6; ii < GJ_TILE; ii += 4) {
    const int i = r0 + ii;
    if (i >= n) break;
    double v;
    if (i == k) {
      v = rowk[jl];
    } else {
      const int s = (i == p) ? k : i;
      const double f = col[s];
      const double as = (j == k) ? 0.0 : a[(long long)s * n + j];
      v = __builtin_fma(-f, rowk[jl], as);
    }
    b[(long long)i * n + j] = v;
  }
}

// out[o][i][j] = B[o][i][perm[o][j]]  (column unscramble)
__global__ void gather_cols_kernel(double* __restrict__ out, const double* __restrict__ B,
                                   const int* __restrict__ perm, int n, int n_obj) {
  const long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  const long long per = (long long)n * n;
  if (t >= per * n_obj) return;
  const int o = (int)(t / per);
  const long long r = t - o * per;
  const int i = (int)(r / n), j = (int)(r - (long long)i * n);
  out[t] = B[o * per + (long long)i * n + perm[o * n + j]];
}

// --------------------------------------------------------------------------- MLL
struct MllParams {
  double pv[BO_MAX_OBJ], pm[BO_MAX_OBJ], nhl[BO_MAX_OBJ];
};

// C[o] = K[o][:n,:n] / pv[o] + 1e-8 I   (numba_kernels.py:195-214), dense n x n
__global__ void corr_kernel(double* __restrict__ dst, const double* __restrict__ km, long long ld,
                            int n, int n_obj, MllParams p) {
  const long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  const long long per = (long long)n * n;
  if (t >= per * n_obj) return;
  const int o = (int)(t / per);
  const long long r = t - o * per;
  const int i = (int)(r / n), j = (int)(r - (long long)i * n);
  double v = km[(long long)o * ld * ld + (long long)i * ld + j] / p.pv[o];
  if (i == j) v += BO_CHOLESKY_JITTER;
  dst[t] = v;
}

// Factor diagonal block kb in place (one workgroup per objective; unblocked right-looking
// Cholesky in LDS, LAPACK potf2 order of terms).  Its own launch: the panel solves below read
// the finished factor, so no workgroup ever sees the block half-written.
__global__ __launch_bounds__(256) void potrf_diag_kernel(double* __restrict__ C, int n, int kb,
                                                         int* __restrict__ status) {
  __shared__ double Lk[NB][NB + 1];
  const int o = blockIdx.x;
  double* c = C + (long long)o * n * n;
  const int k0 = kb * NB;
  const int kn = min(NB, n - k0);
  const int tid = threadIdx.x;
  for (int t = tid; t < NB * NB; t += 256) {
    const int r = t / NB, q = t % NB;
    Lk[r][q] = (r < kn && q < kn && q <= r) ? c[(long long)(k0 + r) * n + k0 + q] : (r == q ? 1.0 : 0.0);
  }
  __syncthreads();
  bool bad = false;
  for (int j = 0; j < kn; ++j) {
    const double d = Lk[j][j];
    if (!(d > 0.0)) bad = true;
    const double sd = sqrt(d);
    __syncthreads();
    if (tid == 0) Lk[j][j] = sd;
    for (int r = j + 1 + tid; r < kn; r += 256) Lk[r][j] = Lk[r][j] / sd;
    __syncthreads();
    for (int t = tid; t < kn * kn; t += 256) {
      const int r = t / kn, q = t % kn;
      if (q > j && r >= q) Lk[r][q] = __builtin_fma(-Lk[r][j], Lk[q][j], Lk[r][q]);
    }
    __syncthreads();
  }
  if (bad && tid == 0) atomicOr(status, 1);
  for (int t = tid; t < kn * kn; t += 256) {
    const int r = t / kn, q = t % kn;
    if (q <= r) c[(long long)(k0 + r) * n + k0 + q] = Lk[r][q];
  }
}

// Panel solve of row block ib = kb + 1 + blockIdx.x: L_ib = A_ib L_kk^-T, reading the factored
// diagonal block.  Goes through W = L_kk^-1 (one column per lane, register-resident forward
// substitution) so the 32 x 32 product X = A_ib W^T runs fully parallel.
__global__ __launch_bounds__(256) void trsm_panel_kernel(double* __restrict__ C, int n, int kb) {
  __shared__ double Lk[NB][NB + 1];
  __shared__ double Wi[NB][NB + 1];
  __shared__ double Ab[NB][NB + 1];
  const int o = blockIdx.y;
  double* c = C + (long long)o * n * n;
  const int k0 = kb * NB;
  const int kn = min(NB, n - k0);
  const int ib = kb + 1 + blockIdx.x;
  const int i0 = ib * NB;
  const int in = min(NB, n - i0);
  const int tid = threadIdx.x;
  for (int t = tid; t < NB * NB; t += 256) {
    const int r = t / NB, q = t % NB;
    Lk[r][q] = (r < kn && q < kn && q <= r) ? c[(long long)(k0 + r) * n + k0 + q] : (r == q ? 1.0 : 0.0);
    Ab[r][q] = (r < in && q < kn) ? c[(long long)(i0 + r) * n + k0 + q] : 0.0;
  }
  __syncthreads();
  // W = L_kk^-1: lane `col` forward-substitutes the unit vector e_col (rows >= kn are
  // identity-padded, so W stays well defined for a partial last block)
  if (tid < NB) {
    const int col = tid;
    double x[NB];
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      double v = (j == col) ? 1.0 : 0.0;
#pragma unroll
      for (int t = 0; t < j; ++t) v = __builtin_fma(-Lk[j][t], x[t], v);
      x[j] = (j < col) ? 0.0 : v / Lk[j][j];
    }
#pragma unroll
    for (int j = 0; j < NB; ++j) Wi[j][col] = x[j];
  }
  __syncthreads();
  // X[r][j] = sum_{t <= j} A[r][t] W[j][t]
  {
    const int r = tid >> 3, jg = (tid & 7) * 4;
    double acc[4] = {0.0, 0.0, 0.0, 0.0};
    for (int t = 0; t < NB; ++t) {
      const double av = Ab[r][t];
#pragma unroll
      for (int u = 0; u < 4; ++u) acc[u] = __builtin_fma(av, Wi[jg + u][t], acc[u]);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (r < in && jg + u < kn) c[(long long)(i0 + r) * n + k0 + jg + u] = acc[u];
  }
}

// trailing update of block column kb: A_ij -= L_ik L_jk^T for kb < jb <= ib
__global__ __launch_bounds__(256) void syrk_kernel(double* __restrict__ C, int n, int kb, int nb) {
  __shared__ double Li[NB][NB + 1];
  __shared__ double Lj[NB][NB + 1];
  const int o = blockIdx.y;
  double* c = C + (long long)o * n * n;
  // decode the lower-triangular tile index blockIdx.x -> (ib, jb), kb < jb <= ib < nb
  const int m = nb - kb - 1;
  int t = blockIdx.x, ib = 0, jb = 0;
  for (int r = 0; r < m; ++r) {
    if (t <= r) { ib = kb + 1 + r; jb = kb + 1 + t; break; }
    t -= r + 1;
  }
  const int k0 = kb * NB, kn = min(NB, n - k0);
  const int i0 = ib * NB, in = min(NB, n - i0);
  const int j0 = jb * NB, jn = min(NB, n - j0);
  const int tid = threadIdx.x;
  for (int u = tid; u < NB * NB; u += 256) {
    const int r = u / NB, q = u % NB;
    Li[r][q] = (r < in && q < kn) ? c[(long long)(i0 + r) * n + k0 + q] : 0.0;
    Lj[r][q] = (r < jn && q < kn) ? c[(long long)(j0 + r) * n + k0 + q] : 0.0;
  }
  __syncthreads();
  for (int u = tid; u < in * jn; u += 256) {
    const int r = u / jn, q = u % jn;
    if (ib == jb && q > r) continue;
    double s = c[(long long)(i0 + r) * n + j0 + q];
    for (int tt = 0; tt < kn; ++tt) s = __builtin_fma(-Li[r][tt], Lj[q][tt], s);
    c[(long long)(i0 + r) * n + j0 + q] = s;
  }
}

// Per objective (one 1024-thread block): yc = (y - pm) / std(y - pm) (population std, skipped
// when 0), z = L^-1 yc, alpha = L^-T z, mll = -0.5 yc.alpha - sum log L_ii - 0.5 n log(2 pi).
__global__ __launch_bounds__(1024) void mll_solve_kernel(const double* __restrict__ C,
                                                         const double* __restrict__ y,
                                                         long long ld_y, int n, MllParams p,
                                                         double* __restrict__ work,
                                                         double* __restrict__ mll_out) {
  __shared__ double red[1024];
  const int o = blockIdx.x, tid = threadIdx.x, nt = blockDim.x;
  const double* L = C + (long long)o * n * n;
  double* yc = work + (long long)o * 3 * n;
  double* z = yc + n;
  double* al = z + n;
  // centre and standardise (numba_kernels.py:201-208): mean then population std
  double s = 0.0;
  for (int i = tid; i < n; i += nt) {
    const double v = y[(long long)i * ld_y + o] - p.pm[o];
    yc[i] = v;
    s += v;
  }
  red[tid] = s;
  __syncthreads();
  for (int w = nt / 2; w > 0; w >>= 1) { if (tid < w) red[tid] += red[tid + w]; __syncthreads(); }
  const double mean = red[0] / n;
  __syncthreads();
  s = 0.0;
  for (int i = tid; i < n; i += nt) { const double d = yc[i] - mean; s += d * d; }
  red[tid] = s;
  __syncthreads();
  for (int w = nt / 2; w > 0; w >>= 1) { if (tid < w) red[tid] += red[tid + w]; __syncthreads(); }
  const double sd = sqrt(red[0] / n);
  __syncthreads();
  if (sd > 0.0)
    for (int i = tid; i < n; i += nt) yc[i] = yc[i] / sd;
  for (int i = tid; i < n; i += nt) z[i] = yc[i];
  __syncthreads();
  // forward substitution L z = yc, blocked by NB rows: diagonal block serially by one wave,
  // then the rows below updated in parallel
  for (int k0 = 0; k0 < n; k0 += NB) {
    const int kn = min(NB, n - k0);
    if (tid == 0) {
      for (int j = k0; j < k0 + kn; ++j) {
        double x = z[j];
        for (int t = k0; t < j; ++t) x = __builtin_fma(-L[(long long)j * n + t], z[t], x);
        z[j] = x / L[(long long)j * n + j];
      }
    }
    __syncthreads();
    for (int i = k0 + kn + tid; i < n; i += nt) {
      double x = z[i];
      for (int t = k0; t < k0 + kn; ++t) x = __builtin_fma(-L[(long long)i * n + t], z[t], x);
      z[i] = x;
    }
    __syncthreads();
  }
  for (int i = tid; i < n; i += nt) al[i] = z[i];
  __syncthreads();
  // back substitution L^T alpha = z
  for (int k1 = n; k1 > 0; k1 -= NB) {
    const int k0 = k1 - NB > 0 ? k1 - NB : 0;
    if (tid == 0) {
      for (int j = k1 - 1; j >= k0; --j) {
        double x = al[j];
        for (int t = j + 1; t < k1; ++t) x = __builtin_fma(-L[(long long)t * n + j], al[t], x);
        al[j] = x / L[(long long)j * n + j];
      }
    }
    __syncthreads();
    for (int i = tid; i < k0; i += nt) {
      double x = al[i];
      for (int t = k0; t < k1; ++t) x = __builtin_fma(-L[(long long)t * n + i], al[t], x);
      al[i] = x;
    }
    __syncthreads();
  }
  // terms (numba_kernels.py:222-232)
  double fit = 0.0, ld = 0.0;
  for (int i = tid; i < n; i += nt) {
    fit = __builtin_fma(yc[i], al[i], fit);
    ld += log(L[(long long)i * n + i]);
  }
  red[tid] = fit;
  __syncthreads();
  for (int w = nt / 2; w > 0; w >>= 1) { if (tid < w) red[tid] += red[tid + w]; __syncthreads(); }
  const double dfit = red[0];
  __syncthreads();
  red[tid] = ld;
  __syncthreads();
  for (int w = nt / 2; w > 0; w >>= 1) { if (tid < w) red[tid] += red[tid + w]; __syncthreads(); }
  if (tid == 0) {
    const double logdet = 2.0 * red[0];
    mll_out[o] = -0.5 * dfit + (-0.5 * logdet) + (-0.5 * n * log(2.0 * 3.141592653589793));
  }
}

inline size_t a256(size_t x) { return (x + 255) & ~(size_t)255; }

}  // namespace

// Blocked lower Cholesky, in place, of n_obj dense n x n matrices (lower triangle read and
// written); any non-positive pivot sets *d_status = 1.  Asynchronous (no host sync).
__attribute__((visibility("hidden"))) int bo_internal_potrf(double* C, int n, int n_obj,
                                                            int* d_status, hipStream_t s) {
  const int nb = (n + NB - 1) / NB;
  for (int kb = 0; kb < nb; ++kb) {
    hipLaunchKernelGGL(potrf_diag_kernel, dim3(n_obj), dim3(256), 0, s, C, n, kb, d_status);
    const int m = nb - kb - 1;
    if (m > 0)
      hipLaunchKernelGGL(trsm_panel_kernel, dim3(m, n_obj), dim3(256), 0, s, C, n, kb);
    if (m > 0)
      hipLaunchKernelGGL(syrk_kernel, dim3(m * (m + 1) / 2, n_obj), dim3(256), 0, s, C, n, kb, nb);
  }
  return hipGetLastError() == hipSuccess ? BO_OK : BO_ERR_HIP;
}

extern "C" {

size_t bo_invert_k_workspace_size(int32_t n_obj, int64_t n) {
  if (n_obj < 1 || n < 1) return 0;
  return 2 * a256((size_t)n_obj * n * n * sizeof(double)) + a256((size_t)n_obj * n * sizeof(int)) * 2 + 512;
}

int bo_invert_k(double* out, const double* km, int64_t ld, int32_t n_obj, int64_t n, void* ws,
                size_t ws_bytes, void* stream) {
  if (!out || !km || n_obj < 1 || n_obj > BO_MAX_OBJ || n < 1 || ld < n) return BO_ERR_ARG;
  if (n > 2048) return BO_ERR_UNSUPPORTED;
  if (!ws || ws_bytes < bo_invert_k_workspace_size(n_obj, n)) return BO_ERR_WORKSPACE;
  hipStream_t s = (hipStream_t)stream;
  char* w = (char*)ws;
  const size_t mat = a256((size_t)n_obj * n * n * sizeof(double));
  double* bufA = (double*)w;
  double* bufB = (double*)(w + mat);
  int* piv = (int*)(w + 2 * mat);
  int* perm = (int*)(w + 2 * mat + a256((size_t)n_obj * n * sizeof(int)));
  int* status = (int*)(w + 2 * mat + 2 * a256((size_t)n_obj * n * sizeof(int)));
  BO_CHECK_HIP(hipMemsetAsync(status, 0, sizeof(int), s));
  const long long total = (long long)n_obj * n * n;
  hipLaunchKernelGGL(jitter_copy_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s,
                     bufA, km, (long long)ld, (int)n, n_obj, BO_KERNEL_JITTER);
  BO_CHECK_HIP(hipGetLastError());
  const int tiles = (int)((n + GJ_TILE - 1) / GJ_TILE);
  double* src = bufA;
  double* dst = bufB;
  for (int k = 0; k < n; ++k) {
    hipLaunchKernelGGL(gj_step_kernel, dim3(tiles, tiles, n_obj), dim3(256), 0, s, dst, src,
                       (int)n, k, piv, status);
    double* t = src; src = dst; dst = t;
  }
  BO_CHECK_HIP(hipGetLastError());
  std::vector<int> hpiv((size_t)n_obj * n);
  int hstatus = 0;
  BO_CHECK_HIP(hipMemcpyAsync(hpiv.data(), piv, sizeof(int) * hpiv.size(), hipMemcpyDeviceToHost, s));
  BO_CHECK_HIP(hipMemcpyAsync(&hstatus, status, sizeof(int), hipMemcpyDeviceToHost, s));
  BO_CHECK_HIP(hipStreamSynchronize(s));
  if (hstatus) return BO_ERR_SINGULAR;
  // column permutation: apply swaps (k, piv[k]) for k = n-1 .. 0 to the identity ordering
  std::vector<int> hperm((size_t)n_obj * n);
  for (int o = 0; o < n_obj; ++o) {
    int* pr = hperm.data() + (size_t)o * n;
    for (int j = 0; j < n; ++j) pr[j] = j;
    for (long long k = n - 1; k >= 0; --k) {
      const int p = hpiv[(size_t)o * n + k];
      const int t = pr[k]; pr[k] = pr[p]; pr[p] = t;
    }
  }
  BO_CHECK_HIP(hipMemcpyAsync(perm, hperm.data(), sizeof(int) * hperm.size(), hipMemcpyHostToDevice, s));
  hipLaunchKernelGGL(gather_cols_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s,
                     out, src, perm, (int)n, n_obj);
  BO_CHECK_HIP(hipGetLastError());
  BO_CHECK_HIP(hipStreamSynchronize(s));
  return BO_OK;
}

size_t bo_compute_mll_workspace_size(int32_t n_obj, int64_t n) {
  if (n_obj < 1 || n < 1) return 0;
  return a256((size_t)n_obj * n * n * sizeof(double)) + a256((size_t)n_obj * 3 * n * sizeof(double)) +
         a256((size_t)BO_MAX_OBJ * sizeof(double)) + 512;
}

int bo_update_k(double* km, int64_t ld, int32_t n_obj, const double* x, int32_t dim,
                int64_t last_eval, int64_t cur, const double* pv, const double* ls, void* stream);

int bo_compute_mll(double* mll_out, const double* x, int32_t dim, const double* y, int64_t ld_y,
                   double* km, int64_t ld, int32_t n_obj, const double* pm, const double* pv,
                   const double* ls, int64_t n, void* ws, size_t ws_bytes, void* stream) {
  if (!mll_out || !x || !y || !km || !pm || !pv || !ls || n_obj < 1 || n_obj > BO_MAX_OBJ ||
      n < 1 || ld < n || ld_y < n_obj)
    return BO_ERR_ARG;
  if (!ws || ws_bytes < bo_compute_mll_workspace_size(n_obj, n)) return BO_ERR_WORKSPACE;
  hipStream_t s = (hipStream_t)stream;
  // the Gram is rebuilt into the caller's kernel_matrix, as the reference does (:178-185)
  int st = bo_update_k(km, ld, n_obj, x, dim, 0, n, pv, ls, stream);
  if (st != BO_OK) return st;
  char* w = (char*)ws;
  double* C = (double*)w;
  double* work = (double*)(w + a256((size_t)n_obj * n * n * sizeof(double)));
  double* dmll = (double*)((char*)work + a256((size_t)n_obj * 3 * n * sizeof(double)));
  int* status = (int*)((char*)dmll + a256((size_t)BO_MAX_OBJ * sizeof(double)));
  MllParams p;
  memset(&p, 0, sizeof(p));
  for (int o = 0; o < n_obj; ++o) { p.pv[o] = pv[o]; p.pm[o] = pm[o]; }
  BO_CHECK_HIP(hipMemsetAsync(status, 0, sizeof(int), s));
  const long long total = (long long)n_obj * n * n;
  hipLaunchKernelGGL(corr_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, C, km,
                     (long long)ld, (int)n, n_obj, p);
  BO_CHECK_HIP(hipGetLastError());
  st = bo_internal_potrf(C, (int)n, n_obj, status, s);
  if (st != BO_OK) return st;
  hipLaunchKernelGGL(mll_solve_kernel, dim3(n_obj), dim3(1024), 0, s, C, y, (long long)ld_y, (int)n,
                     p, work, dmll);
  BO_CHECK_HIP(hipGetLastError());
  double h[BO_MAX_OBJ];
  int hstatus = 0;
  BO_CHECK_HIP(hipMemcpyAsync(h, dmll, sizeof(double) * n_obj, hipMemcpyDeviceToHost, s));
  BO_CHECK_HIP(hipMemcpyAsync(&hstatus, status, sizeof(int), hipMemcpyDeviceToHost, s));
  BO_CHECK_HIP(hipStreamSynchronize(s));
  if (hstatus) return BO_ERR_NOT_PD;
  // np.sum over objectives (numba_kernels.py:235): pairwise for >= 8, sequential below
  double tot = 0.0;
  for (int o = 0; o < n_obj; ++o) tot += h[o];
  *mll_out = tot;
  return BO_OK;
}

}  // extern "C"
