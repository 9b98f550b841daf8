// GP fit on device: compute_mll and invert_k on one blocked, MFMA-backed Cholesky.
//
//   bo_compute_mll  numba_kernels.py:152-235   sum over objectives of the GP marginal log
//                   likelihood of K/pv + 1e-8 I with y centred on the prior mean and scaled by
//                   its population std.
//   bo_invert_k     numba_kernels.py:370-403   inv(K + 1e-6 I) per objective (the reference's
//                   LAPACK gesv); Cholesky first, Gauss-Jordan with partial pivoting (LAPACK's
//                   idamax row choice) for any objective whose Cholesky fails.
//
// One factorisation serves both: the right-looking blocked Cholesky (64 x 64 tiles) of an
// AUGMENTED lower-triangular matrix
//
//        [ K    .  ]      factoring only the first n_p columns leaves     [ L          .          ]
//    A = [ B    C  ]      (n_p = N padded to 64 with an identity block)   [ B L^-T     C - B K^-1 B^T ]
//
//   * compute_mll: B = yc^T (one row), C = 0:  the bottom row holds z = L^-1 yc and the corner
//     holds -yc^T K^-1 yc, the data-fit term (numba_kernels.py:216-222: solve(L, yc),
//     solve(L^T, .), yc . alpha); log det = 2 sum log L_ii (:225-229);
//   * invert_k:    B = I, C = 0:  the bottom-right block holds -K^-1 (lower triangle); the zero
//     blocks of L^-T (upper triangular) are skipped, so the whole inverse costs about 3/2 of a
//     Cholesky of the 2N system's first half.
//
// A is stored COLUMN-major (element (i, j) of the lower triangle at j * Na + i), so that the
// row-per-lane accesses of the panel kernel and the row-contiguous tile loads of the update are
// coalesced.  Per 64-column step k: chol_panel_kernel factors the diagonal tile (one wave, one
// row per lane) and solves the tiles below it (row substitution, one row per lane; 4 row blocks
// per workgroup); chol_update_kernel applies A_pq -= L_pk L_qk^T to every live tile of the
// trailing matrix with v_mfma_f64_16x16x4_f64 (64 x 64 x 64 per workgroup).  A non-positive or NaN pivot
// sets the objective's status (compute_mll: BO_ERR_NOT_PD = LinAlgError, as cholesky raises at
// :214; invert_k: the LU fallback).  Sizes are not capped: the workspace is n_obj (N + 64)^2
// doubles (MLL) or n_obj (2 N_p)^2 (inverse).

#include "bo_common.h"

#include <math.h>
#include <string.h>

#include <vector>

namespace {

constexpr int NB = 64;      // tile size
constexpr int LS = 66;      // LDS row stride (doubles) of staged tiles

struct FitParams {
  double pv[BO_MAX_OBJ], pm[BO_MAX_OBJ], ls2[BO_MAX_OBJ], jitter, scale_by_pv;
};

// Geometry of the augmented system: top part n_p = nbt * 64 rows (N padded), bottom part
// rb * 64 rows; leading dimension Na = n_p + 64 rb.  ident: B = I (structurally upper-triangular
// bottom-left tiles, inverse); otherwise every bottom tile is live (MLL).
struct Aug {
  int n, nbt, rb, ident;
  long long Na;
};

// --------------------------------------------------------------------------- init
// Lower triangle of the augmented matrix, per objective (blockIdx.y), column j = blockIdx.x,
// rows i >= j over the threads (coalesced column-major writes):
//   i, j < N:           MLL: v / pv + 1e-8 d_ij with v = pv exp(-0.5 |x_i - x_j|^2 / ls^2) exactly
//                       as update_k (numba_kernels.py:352-361), also written to the caller's
//                       kernel_matrix (both triangles, the reference rebuilds it in compute_mll);
//                       inverse: K[i][j] + 1e-6 d_ij from the caller's kernel_matrix;
//   padding of K:       identity;
//   bottom rows:        MLL: row n_p = yc (ycv), the rest 0; inverse: B = I; C = 0.
__global__ __launch_bounds__(256) void aug_init_kernel(double* __restrict__ A, Aug g,
                                                      double* __restrict__ km, long long ld,
                                                      const double* __restrict__ x, int dim,
                                                      const double* __restrict__ ycv, FitParams p,
                                                      int gram) {
  const int o = blockIdx.y;
  const long long j = blockIdx.x;
  const long long np_ = (long long)g.nbt * NB;
  double* Ao = A + (long long)o * g.Na * g.Na;
  double* ko = km + (long long)o * ld * ld;
  for (long long i = j + threadIdx.x; i < g.Na; i += blockDim.x) {
    double v = 0.0;
    if (i < np_) {
      if (i < g.n && j < g.n) {
        double kv;
        if (gram) {
          double sq = 0.0;
          for (int k = 0; k < dim; ++k) {
            const double d = x[i * dim + k] - x[j * dim + k];
            sq = __builtin_fma(d, d, sq);
          }
          kv = p.pv[o] * exp(-0.5 * sq / p.ls2[o]);
          ko[i * ld + j] = kv;
          ko[j * ld + i] = kv;
        } else {
          kv = ko[i * ld + j];
        }
        v = (p.scale_by_pv != 0.0 ? kv / p.pv[o] : kv) + (i == j ? p.jitter : 0.0);
      } else {
        v = (i == j) ? 1.0 : 0.0;
      }
    } else if (j < np_) {
      const long long r = i - np_;
      if (g.ident) v = (r == j && j < g.n) ? 1.0 : 0.0;
      else v = (r == 0 && j < g.n) ? ycv[(long long)o * g.n + j] : 0.0;
    }
    Ao[j * g.Na + i] = v;
  }
}

// yc = (y - pm) / std(y - pm) per objective (population std; unscaled when 0),
// numba_kernels.py:201-208.  One workgroup per objective.
__global__ __launch_bounds__(1024) void ystd_kernel(double* __restrict__ ycv, const double* __restrict__ y,
                                                    long long ld_y, int n, FitParams p) {
  __shared__ double red[1024];
  const int o = blockIdx.x, tid = threadIdx.x, nt = blockDim.x;
  double* yc = ycv + (long long)o * n;
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
  if (sd > 0.0)
    for (int i = tid; i < n; i += nt) yc[i] = yc[i] / sd;
}

// ------------------------------------------------------------------------ panel
// lane l's value of a wave-uniform broadcast (v_readlane on both halves)
__device__ __forceinline__ double rdlane(double v, int l) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffll), l);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// Row blocks of step k: [k, k+1, ..., nbt-1, nbt, ..., nbt+ra-1] (ra live bottom blocks).
__device__ __forceinline__ int panel_row(int idx, int k, int nbt) {
  return idx < nbt - k ? k + idx : nbt + (idx - (nbt - k));
}

// Step k, per objective (blockIdx.y), 4 row blocks per workgroup (one per wave):
//   wave 0 factors the diagonal tile A_kk in LDS (lane r = row r, right-looking, column j of L
//   broadcast through LDS; single wave, so no barrier between the columns);
//   then wave w takes row block R[4 blockIdx.x + w]: the diagonal block writes L_kk, the others
//   solve X L_kk^T = A_ik by row substitution (lane r = row r of the block).
__global__ __launch_bounds__(256) void chol_panel_kernel(double* __restrict__ A, Aug g, int k, int n_rows,
                                                        int* __restrict__ status) {
  __shared__ double L[NB][NB + 1];
  __shared__ double col[NB];
  __shared__ double rdiag[NB];
  const int o = blockIdx.y;
  double* Ao = A + (long long)o * g.Na * g.Na;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const long long k0 = (long long)k * NB;
  if (wave == 0) {
    double a[NB];
    const double* src = Ao + k0 * g.Na + k0 + lane;       // (k0 + lane, k0 + t) at src[t Na]
#pragma unroll
    for (int t = 0; t < NB; ++t) a[t] = t <= lane ? src[t * g.Na] : 0.0;
    // a[t > lane] is scratch: it only ever receives updates, never feeds a real entry
    bool bad = false;
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const double piv = rdlane(a[j], j);
      bad = bad || !(piv > 0.0);             // potrf: ajj <= 0 or NaN -> not positive definite
      const double d = sqrt(piv);
      const double rd = 1.0 / d;               // wave-uniform: one reciprocal per column
      const double lj = lane == j ? d : (lane > j ? a[j] * rd : 0.0);
      a[j] = lj;
      col[lane] = lj;
      if (lane == 0) rdiag[j] = rd;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
      for (int t = j + 1; t < NB; ++t) a[t] = __builtin_fma(-lj, col[t], a[t]);
      __builtin_amdgcn_wave_barrier();
    }
#pragma unroll
    for (int t = 0; t < NB; ++t) L[lane][t] = a[t];
    // identity padding and the never-factored bottom rows cannot fail: any bad pivot is real
    if (bad && blockIdx.x == 0 && lane == 0) atomicOr(status + o, 1);
  }
  __syncthreads();
  const int idx = 4 * blockIdx.x + wave;
  if (idx >= n_rows) return;
  const long long i0 = (long long)panel_row(idx, k, g.nbt) * NB;
  double* dst = Ao + k0 * g.Na + i0 + lane;              // (i0 + lane, k0 + t) at dst[t Na]
  if (idx == 0) {
#pragma unroll
    for (int t = 0; t < NB; ++t)
      if (t <= lane) dst[t * g.Na] = L[lane][t];
    return;
  }
  // x L_kk^T = a:  x_j = (a_j - sum_{t<j} x_t L_jt) / L_jj   (two partial sums for ILP; the
  // division as a product with the reciprocal the factorisation computed)
  double x[NB];
#pragma unroll
  for (int t = 0; t < NB; ++t) x[t] = dst[t * g.Na];
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    double s0 = x[j], s1 = 0.0;
#pragma unroll
    for (int t = 0; t < j; ++t) {
      if (t & 1) s1 = __builtin_fma(-x[t], L[j][t], s1);
      else s0 = __builtin_fma(-x[t], L[j][t], s0);
    }
    x[j] = (s0 + s1) * rdiag[j];
  }
#pragma unroll
  for (int t = 0; t < NB; ++t) dst[t * g.Na] = x[t];
}

// ----------------------------------------------------------------------- update
__device__ __forceinline__ d4 mfma64(double a, double b, d4 c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

// triangular index t -> (i, j), j <= i, t = i (i + 1) / 2 + j
__device__ __forceinline__ void tri_decode(long long t, int& i, int& j) {
  int r = (int)((sqrt(8.0 * (double)t + 1.0) - 1.0) * 0.5);
  while ((long long)(r + 1) * (r + 2) / 2 <= t) ++r;
  while ((long long)r * (r + 1) / 2 > t) --r;
  i = r;
  j = (int)(t - (long long)r * (r + 1) / 2);
}

// Trailing update of step k: A_pq -= L_pk L_qk^T for every live tile, k < q <= p:
//   T1 top x top (m (m + 1) / 2), T2 bottom x top (ra m), T3 bottom x bottom (ra (ra + 1) / 2),
//   m = nbt - k - 1.  L_pk and L_qk are staged in LDS transposed (PT[c][r], stride 66, from
//   coalesced column-major loads); the MFMAs compute C^T = L_qk L_pk^T so that a lane's output
//   rows are consecutive rows of the column-major A: wave w takes q-rows 16 w .. 16 w + 15 of
//   the tile against 4 blocks of 16 p-rows, over 16 k-steps.
__global__ __launch_bounds__(256) void chol_update_kernel(double* __restrict__ A, Aug g, int k, int ra) {
  extern __shared__ double lds[];
  double* P = lds;
  double* Q = lds + NB * LS;
  const int o = blockIdx.y;
  double* Ao = A + (long long)o * g.Na * g.Na;
  const int m = g.nbt - k - 1;
  const long long T1 = (long long)m * (m + 1) / 2, T2 = (long long)ra * m;
  long long t = blockIdx.x;
  int p, q;
  if (t < T1) {
    int i, j;
    tri_decode(t, i, j);
    p = k + 1 + i;
    q = k + 1 + j;
  } else if (t < T1 + T2) {
    t -= T1;
    p = g.nbt + (int)(t / m);
    q = k + 1 + (int)(t % m);
  } else {
    int i, j;
    tri_decode(t - T1 - T2, i, j);
    p = g.nbt + i;
    q = g.nbt + j;
  }
  const long long k0 = (long long)k * NB, p0 = (long long)p * NB, q0 = (long long)q * NB;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int e = tid; e < NB * NB; e += 256) {
    const int r = e & 63, c = e >> 6;                     // (row r, column c) of the tiles
    P[c * LS + r] = Ao[(k0 + c) * g.Na + p0 + r];
    Q[c * LS + r] = Ao[(k0 + c) * g.Na + q0 + r];
  }
  __syncthreads();
  d4 acc[4];
#pragma unroll
  for (int b = 0; b < 4; ++b) acc[b] = (d4){0.0, 0.0, 0.0, 0.0};
  const int arow = 16 * wave + (lane & 15), ca = lane >> 4;
#pragma unroll
  for (int s = 0; s < NB / 4; ++s) {
    const double av = Q[(4 * s + ca) * LS + arow];        // A = L_qk rows 16 w ..
#pragma unroll
    for (int b = 0; b < 4; ++b)                           // B = L_pk^T, p-rows 16 b ..
      acc[b] = mfma64(av, P[(4 * s + ca) * LS + 16 * b + (lane & 15)], acc[b]);
  }
  // D[(l >> 4) + 4 r][l & 15] of block (wave, b): q-row 16 wave + (l >> 4) + 4 r, p-row
  // 16 b + (l & 15), i.e. element (p0 + p-row, q0 + q-row) of A, column-major
#pragma unroll
  for (int b = 0; b < 4; ++b)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      double* c = Ao + (q0 + 16 * wave + (lane >> 4) + 4 * r) * g.Na + p0 + 16 * b + (lane & 15);
      *c -= acc[b][r];
    }
}

// ------------------------------------------------------------------------ finish
// mll[o] = -0.5 yc . alpha - 0.5 log det - 0.5 N log(2 pi)   (numba_kernels.py:222-232):
// yc . alpha = |z|^2 = -(corner), log det = 2 sum_{i<N} log L_ii.
__global__ __launch_bounds__(1024) void mll_finish_kernel(const double* __restrict__ A, Aug g,
                                                          double* __restrict__ mll) {
  __shared__ double red[1024];
  const int o = blockIdx.x, tid = threadIdx.x;
  const double* Ao = A + (long long)o * g.Na * g.Na;
  double s = 0.0;
  for (int i = tid; i < g.n; i += blockDim.x) s += log(Ao[(long long)i * g.Na + i]);
  red[tid] = s;
  __syncthreads();
  for (int w = blockDim.x / 2; w > 0; w >>= 1) { if (tid < w) red[tid] += red[tid + w]; __syncthreads(); }
  if (tid == 0) {
    const long long c = (long long)g.nbt * NB;
    const double fit = -Ao[c * g.Na + c];
    const double logdet = 2.0 * red[0];
    mll[o] = -0.5 * fit + (-0.5 * logdet) + (-0.5 * g.n * log(2.0 * 3.141592653589793));
  }
}

// out[o][i][j] = -A[n_p + i][n_p + j] (lower), mirrored: the symmetric K^-1.
__global__ void inv_finish_kernel(double* __restrict__ out, const double* __restrict__ A, Aug g,
                                  const int* __restrict__ status) {
  const int o = blockIdx.y;
  if (status[o]) return;                       // this objective goes through the LU fallback
  const long long np_ = (long long)g.nbt * NB;
  const double* Ao = A + (long long)o * g.Na * g.Na;
  const long long n = g.n;
  for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < n * n;
       t += (long long)gridDim.x * blockDim.x) {
    const long long i = t / n, j = t - i * n;
    const long long r = i >= j ? i : j, c = i >= j ? j : i;
    out[(long long)o * n * n + t] = -Ao[(np_ + c) * g.Na + np_ + r];
  }
}

// ------------------------------------------------------------- LU fallback (invert_k)
constexpr int GJ_TILE = 64;   // Gauss-Jordan output tile (64 x 64 per 256-thread block)

// copy K[o][:n,:n] (leading dim ld) + jitter on the diagonal into a dense n x n buffer
__global__ void jitter_copy_kernel(double* __restrict__ dst, const double* __restrict__ src,
                                   long long ld, int n, int o, double jitter) {
  const long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  const long long per = (long long)n * n;
  if (t >= per) return;
  const int i = (int)(t / n), j = (int)(t - (long long)i * n);
  double v = src[(long long)o * ld * ld + (long long)i * ld + j];
  if (i == j) v += jitter;
  dst[t] = v;
}

// One Gauss-Jordan step k of one matrix: B = step_k(A).  pivot p = first argmax_{i>=k}
// |A[i][k]| (LAPACK idamax); row k of B = row p of A / pivot (entry k = 1/pivot); other rows
// i (source row s = k if i == p): B[i][j] = a_s[j] - A[s][k] * rowk[j] with a_s[k] := 0 -- the
// in-place elimination written out-of-place.  Column k in dynamic LDS (any n).
__global__ __launch_bounds__(256) void gj_step_kernel(double* __restrict__ B,
                                                      const double* __restrict__ A, int n, int k,
                                                      int* __restrict__ piv,
                                                      int* __restrict__ status) {
  extern __shared__ double col[];
  __shared__ double red_v[256];
  __shared__ int red_i[256];
  __shared__ double rowk[GJ_TILE];
  const int tid = threadIdx.x;
  double best = -1.0;
  int bi = n;
  for (int i = tid; i < n; i += 256) {
    const double v = A[(long long)i * n + k];
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
    piv[k] = p;
    if (pivot == 0.0) atomicOr(status, 1);
  }
  const int c0 = blockIdx.x * GJ_TILE, r0 = blockIdx.y * GJ_TILE;
  if (tid < GJ_TILE) {
    const int j = c0 + tid;
    if (j < n) rowk[tid] = (j == k) ? 1.0 / pivot : A[(long long)p * n + j] / pivot;
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
      const double as = (j == k) ? 0.0 : A[(long long)s * n + j];
      v = __builtin_fma(-f, rowk[jl], as);
    }
    B[(long long)i * n + j] = v;
  }
}

// out[i][j] = B[i][perm[j]]  (column unscramble)
__global__ void gather_cols_kernel(double* __restrict__ out, const double* __restrict__ B,
                                   const int* __restrict__ perm, int n) {
  const long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  const long long per = (long long)n * n;
  if (t >= per) return;
  const int i = (int)(t / n), j = (int)(t - (long long)i * n);
  out[t] = B[(long long)i * n + perm[j]];
}

inline size_t a256(size_t x) { return (x + 255) & ~(size_t)255; }

Aug make_aug(int n, bool ident) {
  Aug g;
  g.n = n;
  g.nbt = (n + NB - 1) / NB;
  g.rb = ident ? g.nbt : 1;
  g.ident = ident ? 1 : 0;
  g.Na = (long long)(g.nbt + g.rb) * NB;
  return g;
}

// Blocked Cholesky of the first nbt tile columns of every objective's augmented matrix.
int aug_factor(double* A, const Aug& g, int n_obj, int* status, hipStream_t s) {
  static bool attr = false;
  const size_t lds = 2 * NB * LS * sizeof(double);
  if (!attr) {
    BO_CHECK_HIP(hipFuncSetAttribute((const void*)chol_update_kernel,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    attr = true;
  }
  for (int k = 0; k < g.nbt; ++k) {
    const int ra = g.ident ? (k + 1 < g.rb ? k + 1 : g.rb) : g.rb;
    const int m = g.nbt - k - 1;
    const int rows = 1 + m + ra;
    hipLaunchKernelGGL(chol_panel_kernel, dim3((rows + 3) / 4, n_obj), dim3(256), 0, s, A, g, k, rows,
                       status);
    const long long tiles = (long long)m * (m + 1) / 2 + (long long)ra * m + (long long)ra * (ra + 1) / 2;
    if (tiles > 0)
      hipLaunchKernelGGL(chol_update_kernel, dim3((unsigned)tiles, n_obj), dim3(256), lds, s, A, g, k, ra);
  }
  return hipGetLastError() == hipSuccess ? BO_OK : BO_ERR_HIP;
}

size_t aug_bytes(int n_obj, const Aug& g) { return a256((size_t)n_obj * g.Na * g.Na * sizeof(double)); }

}  // namespace

extern "C" {

size_t bo_invert_k_workspace_size(int32_t n_obj, int64_t n) {
  if (n_obj < 1 || n < 1) return 0;
  const Aug g = make_aug((int)n, true);
  const size_t lu = 2 * a256((size_t)n * n * sizeof(double)) + 2 * a256((size_t)n * sizeof(int));
  return aug_bytes(n_obj, g) + lu + 512;
}

int bo_invert_k(double* out, const double* km, int64_t ld, int32_t n_obj, int64_t n, void* ws,
                size_t ws_bytes, void* stream) {
  if (!out || !km || n_obj < 1 || n_obj > BO_MAX_OBJ || n < 1 || ld < n) return BO_ERR_ARG;
  if (n > (1 << 15)) return BO_ERR_UNSUPPORTED;
  if (!ws || ws_bytes < bo_invert_k_workspace_size(n_obj, n)) return BO_ERR_WORKSPACE;
  hipStream_t s = (hipStream_t)stream;
  const Aug g = make_aug((int)n, true);
  char* w = (char*)ws;
  double* A = (double*)w;
  char* lu = w + aug_bytes(n_obj, g);
  double* bufA = (double*)lu;
  double* bufB = (double*)(lu + a256((size_t)n * n * sizeof(double)));
  int* piv = (int*)(lu + 2 * a256((size_t)n * n * sizeof(double)));
  int* perm = piv + a256((size_t)n * sizeof(int)) / sizeof(int);
  int* status = (int*)(lu + 2 * a256((size_t)n * n * sizeof(double)) + 2 * a256((size_t)n * sizeof(int)));
  BO_CHECK_HIP(hipMemsetAsync(status, 0, 256, s));
  FitParams p;
  memset(&p, 0, sizeof(p));
  p.jitter = BO_KERNEL_JITTER;                 // numba_kernels.py:397-398
  hipLaunchKernelGGL(aug_init_kernel, dim3((unsigned)g.Na, n_obj), dim3(256), 0, s, A, g,
                     (double*)km, (long long)ld, (const double*)nullptr, 0, (const double*)nullptr, p, 0);
  BO_CHECK_HIP(hipGetLastError());
  int st = aug_factor(A, g, n_obj, status, s);
  if (st != BO_OK) return st;
  hipLaunchKernelGGL(inv_finish_kernel, dim3(1024, n_obj), dim3(256), 0, s, out, A, g, status);
  BO_CHECK_HIP(hipGetLastError());
  int hstat[BO_MAX_OBJ + 1];
  BO_CHECK_HIP(hipMemcpyAsync(hstat, status, sizeof(int) * n_obj, hipMemcpyDeviceToHost, s));
  BO_CHECK_HIP(hipStreamSynchronize(s));
  // LU fallback (Gauss-Jordan, partial pivoting) for the objectives whose Cholesky failed
  for (int o = 0; o < n_obj; ++o) {
    if (!hstat[o]) continue;
    int* gstat = status + BO_MAX_OBJ + 1;
    BO_CHECK_HIP(hipMemsetAsync(gstat, 0, sizeof(int), s));
    const long long total = (long long)n * n;
    hipLaunchKernelGGL(jitter_copy_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s,
                       bufA, km, (long long)ld, (int)n, o, BO_KERNEL_JITTER);
    BO_CHECK_HIP(hipGetLastError());
    const int tiles = (int)((n + GJ_TILE - 1) / GJ_TILE);
    const size_t col_lds = (size_t)n * sizeof(double);
    if (col_lds > 64 * 1024)
      BO_CHECK_HIP(hipFuncSetAttribute((const void*)gj_step_kernel,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)col_lds));
    double* src = bufA;
    double* dst = bufB;
    for (int k = 0; k < n; ++k) {
      hipLaunchKernelGGL(gj_step_kernel, dim3(tiles, tiles), dim3(256), col_lds, s, dst, src, (int)n,
                         k, piv, gstat);
      double* t = src; src = dst; dst = t;
    }
    BO_CHECK_HIP(hipGetLastError());
    std::vector<int> hpiv((size_t)n);
    int gs = 0;
    BO_CHECK_HIP(hipMemcpyAsync(hpiv.data(), piv, sizeof(int) * n, hipMemcpyDeviceToHost, s));
    BO_CHECK_HIP(hipMemcpyAsync(&gs, gstat, sizeof(int), hipMemcpyDeviceToHost, s));
    BO_CHECK_HIP(hipStreamSynchronize(s));
    if (gs) return BO_ERR_SINGULAR;
    // column permutation: apply swaps (k, piv[k]) for k = n-1 .. 0 to the identity ordering
    std::vector<int> hperm((size_t)n);
    for (int j = 0; j < n; ++j) hperm[j] = j;
    for (long long k = n - 1; k >= 0; --k) {
      const int pk = hpiv[k];
      const int t = hperm[k]; hperm[k] = hperm[pk]; hperm[pk] = t;
    }
    BO_CHECK_HIP(hipMemcpyAsync(perm, hperm.data(), sizeof(int) * n, hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(gather_cols_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s,
                       out + (long long)o * n * n, src, perm, (int)n);
    BO_CHECK_HIP(hipGetLastError());
    BO_CHECK_HIP(hipStreamSynchronize(s));
  }
  return BO_OK;
}

size_t bo_compute_mll_workspace_size(int32_t n_obj, int64_t n) {
  if (n_obj < 1 || n < 1) return 0;
  const Aug g = make_aug((int)n, false);
  return aug_bytes(n_obj, g) + a256((size_t)n_obj * n * sizeof(double)) +
         a256((size_t)BO_MAX_OBJ * sizeof(double)) + 512;
}

int bo_compute_mll(double* mll_out, const double* x, int32_t dim, const double* y, int64_t ld_y,
                   double* km, int64_t ld, int32_t n_obj, const double* pm, const double* pv,
                   const double* ls, int64_t n, void* ws, size_t ws_bytes, void* stream) {
  if (!mll_out || !x || !y || !km || !pm || !pv || !ls || n_obj < 1 || n_obj > BO_MAX_OBJ ||
      n < 1 || ld < n || ld_y < n_obj || dim < 1)
    return BO_ERR_ARG;
  if (n > (1 << 16)) return BO_ERR_UNSUPPORTED;
  if (!ws || ws_bytes < bo_compute_mll_workspace_size(n_obj, n)) return BO_ERR_WORKSPACE;
  hipStream_t s = (hipStream_t)stream;
  const Aug g = make_aug((int)n, false);
  char* w = (char*)ws;
  double* A = (double*)w;
  double* ycv = (double*)(w + aug_bytes(n_obj, g));
  double* dmll = (double*)((char*)ycv + a256((size_t)n_obj * n * sizeof(double)));
  int* status = (int*)((char*)dmll + a256((size_t)BO_MAX_OBJ * sizeof(double)));
  FitParams p;
  memset(&p, 0, sizeof(p));
  for (int o = 0; o < n_obj; ++o) {
    p.pv[o] = pv[o];
    p.pm[o] = pm[o];
    p.ls2[o] = ls[o] * ls[o];
  }
  p.jitter = BO_CHOLESKY_JITTER;               // numba_kernels.py:211-214
  p.scale_by_pv = 1.0;                         // correlation matrix K / pv (:195-198)
  BO_CHECK_HIP(hipMemsetAsync(status, 0, 256, s));
  hipLaunchKernelGGL(ystd_kernel, dim3(n_obj), dim3(1024), 0, s, ycv, y, (long long)ld_y, (int)n, p);
  hipLaunchKernelGGL(aug_init_kernel, dim3((unsigned)g.Na, n_obj), dim3(256), 0, s, A, g, km,
                     (long long)ld, x, dim, ycv, p, 1);
  BO_CHECK_HIP(hipGetLastError());
  int st = aug_factor(A, g, n_obj, status, s);
  if (st != BO_OK) return st;
  hipLaunchKernelGGL(mll_finish_kernel, dim3(n_obj), dim3(1024), 0, s, A, g, dmll);
  BO_CHECK_HIP(hipGetLastError());
  double h[BO_MAX_OBJ];
  int hstat[BO_MAX_OBJ];
  BO_CHECK_HIP(hipMemcpyAsync(h, dmll, sizeof(double) * n_obj, hipMemcpyDeviceToHost, s));
  BO_CHECK_HIP(hipMemcpyAsync(hstat, status, sizeof(int) * n_obj, hipMemcpyDeviceToHost, s));
  BO_CHECK_HIP(hipStreamSynchronize(s));
  for (int o = 0; o < n_obj; ++o)
    if (hstat[o]) return BO_ERR_NOT_PD;
  // np.sum over objectives (numba_kernels.py:235): sequential for fewer than 8 terms
  double tot = 0.0;
  for (int o = 0; o < n_obj; ++o) tot += h[o];
  *mll_out = tot;
  return BO_OK;
}

}  // extern "C"
