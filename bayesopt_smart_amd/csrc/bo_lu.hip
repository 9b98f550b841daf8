// invert_k's LU path (numba_kernels.py:370-403: np.linalg.inv = LAPACK gesv(A, I)): blocked
// right-looking LU with partial pivoting (getrf's pivot: the first row of largest |a_ij| in
// the column, rows >= j), then inv(A) = U^-1 L^-1 P one 16-column strip of the identity at a
// time (getrs).  Taken by bo_invert_k for the objectives whose Cholesky fails (cond(K + 1e-6 I)
// of 1e14..1e18 with Powell-fitted hyper-parameters) or whose K is not symmetric.
//
// A (N padded to 16 with identity) is column-major in the workspace.  A 16-column STRIP's rows
// are held up to four per thread of a 512-thread workgroup (16 doubles per row in registers).
// Launch k (one per 16-column step):
//   * panel (strip k): applies the pending step k-1 to its strip -- the step's 16 row swaps (as
//     one permutation of <= 32 rows through LDS), U12 = L11^-1 A12 (unit lower 16 x 16) and the
//     rank-16 update of the rows below -- then factors the strip: per column a workgroup argmax
//     (wave shuffles + 16 wave results in LDS), the row swap through LDS, the scaled column and
//     the rank-1 update of the strip's remaining columns;
//   * update (strips > k): step k-1 applied to each strip by its own workgroup (lookahead: the
//     panel of step k needs only its own strip).
// The L columns keep the row order of their own step (later swaps are not applied to them:
// LAPACK's laswp on the left columns), so the solve interleaves the swaps with the forward
// substitution exactly as the elimination applied them.  Solve (one launch, one workgroup per
// strip of the identity, no inter-workgroup dependency): W = e_strip; per step s: the 16 swaps,
// W_s = L11^-1 W_s, W_below -= L21 W_s; then per step from the last: W_s = U_ss^-1 W_s,
// W_above -= U_above,s W_s.  W's rows are out[:, strip].
//
// Round 2 ran one Gauss-Jordan launch per pivot (N launches, ~105 ms at N = 2048).

#include "bo_common.h"

#include <math.h>
#include <string.h>

#include <vector>

namespace {

constexpr int LB = 16;          // strip width
constexpr int LT = 512;         // threads per strip workgroup (256 VGPRs: the rows stay in registers)
constexpr int LR = 4;           // rows per thread: N_p <= LT * LR = 2048

struct LuGeo {
  int n, n_p, nbs;              // N, N padded to 16, strips
  long long Na;                 // leading dimension (= n_p)
};

// ------------------------------------------------------------------------------ init
// A(i, j) = K[i][j] + 1e-6 d_ij (i, j < N), identity padding: 32 x 32 tiles, coalesced both ways
__global__ __launch_bounds__(256) void lu_init_kernel(double* __restrict__ A, LuGeo g,
                                                      const double* __restrict__ km, long long ld, double jitter) {
  __shared__ double tile[32][33];
  const int ti = blockIdx.y, tj = blockIdx.x, tid = threadIdx.x;
  for (int e = tid; e < 32 * 32; e += 256) {
    const int rr = e >> 5, cc = e & 31;               // K row-major: consecutive threads -> columns
    const long long i = (long long)ti * 32 + rr, j = (long long)tj * 32 + cc;
    tile[rr][cc] = (i < g.n && j < g.n) ? km[i * ld + j] : 0.0;
  }
  __syncthreads();
  for (int e = tid; e < 32 * 32; e += 256) {
    const int cc = e >> 5, rr = e & 31;               // A column-major: consecutive threads -> rows
    const long long i = (long long)ti * 32 + rr, j = (long long)tj * 32 + cc;
    if (i >= g.n_p || j >= g.n_p) continue;
    double v = (i < g.n && j < g.n) ? tile[rr][cc] + (i == j ? jitter : 0.0) : (i == j ? 1.0 : 0.0);
    A[j * g.Na + i] = v;
  }
}

// --------------------------------------------------------------------- strip helpers
struct StripLds {
  double buf[32][LB];           // swapped rows in flight
  int pos[32], src[32];         // the step's row permutation: pos <- src
  int trow[32], tsrc[32];       // thread 0's scratch while building it
  int m;                        // its length
  double T[LB][LB + 1];         // the 16 x 16 block being solved
  double L11[LB][LB + 1];       // the step's diagonal block (L unit lower / U upper)
  double redv[LT / 64];
  int redi[LT / 64];
  double prow[LB], grow[LB];    // pivot row / displaced row
  int pivot;
  double pivv;
};

// row `base + t + LT r` of the strip is w[r][*] of thread t
__device__ __forceinline__ long long own_row(int base, int r) { return (long long)base + threadIdx.x + (long long)LT * r; }

// The row permutation of step s's 16 swaps (rows 16 s + j <-> ipiv[16 s + j], in order), as
// pos <- src pairs over the <= 32 rows it moves; built by thread 0.
__device__ void step_perm(StripLds& L, const int* __restrict__ ipiv, int s) {
  if (threadIdx.x == 0) {
    int* rows = L.trow;
    int* src = L.tsrc;
    int m = 0;
    for (int j = 0; j < LB; ++j) {
      const int a = LB * s + j, b = ipiv[LB * s + j];
      int ia = -1, ib = -1;
      for (int u = 0; u < m; ++u) { if (rows[u] == a) ia = u; if (rows[u] == b) ib = u; }
      if (ia < 0) { rows[m] = a; src[m] = a; ia = m++; }
      if (ib < 0) { rows[m] = b; src[m] = b; ib = m++; }
      const int t = src[ia]; src[ia] = src[ib]; src[ib] = t;
    }
    int k = 0;
    for (int u = 0; u < m; ++u)
      if (src[u] != rows[u]) { L.pos[k] = rows[u]; L.src[k] = src[u]; ++k; }
    L.m = k;
  }
  __syncthreads();
}

// apply the permutation to the rows held in registers (rows >= base)
__device__ __forceinline__ void apply_perm(StripLds& L, double (&w)[LR][LB], int base) {
  const int m = L.m;
#pragma unroll
  for (int r = 0; r < LR; ++r) {
    const long long row = own_row(base, r);
    for (int u = 0; u < m; ++u)
      if (L.src[u] == row) {
#pragma unroll
        for (int c = 0; c < LB; ++c) L.buf[u][c] = w[r][c];
      }
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < LR; ++r) {
    const long long row = own_row(base, r);
    for (int u = 0; u < m; ++u)
      if (L.pos[u] == row) {
#pragma unroll
        for (int c = 0; c < LB; ++c) w[r][c] = L.buf[u][c];
      }
  }
  __syncthreads();
}

// Step s applied to a strip whose rows [16 s, n_p) are in registers (base = 16 s): swaps,
// U12 = L11^-1 A12 (rows 16 s .. 16 s + 15), A22 -= L21 U12.
__device__ void strip_apply(const double* __restrict__ A, const LuGeo& g, const int* __restrict__ ipiv, int s,
                            StripLds& L, double (&w)[LR][LB]) {
  const int base = LB * s, tid = threadIdx.x;
  step_perm(L, ipiv, s);
  apply_perm(L, w, base);
  // L11 (unit lower) and the 16 top rows into LDS
  if (tid < LB * LB) {
    const int i = tid & 15, j = tid >> 4;
    L.L11[i][j] = A[(long long)(base + j) * g.Na + base + i];
  }
  if (tid < LB) {
#pragma unroll
    for (int c = 0; c < LB; ++c) L.T[tid][c] = w[0][c];
  }
  __syncthreads();
  if (tid < LB) {                                    // column tid: forward substitution
    for (int i = 1; i < LB; ++i) {
      double x = L.T[i][tid];
      for (int m2 = 0; m2 < i; ++m2) x = __builtin_fma(-L.L11[i][m2], L.T[m2][tid], x);
      L.T[i][tid] = x;
    }
  }
  __syncthreads();
  if (tid < LB) {
#pragma unroll
    for (int c = 0; c < LB; ++c) w[0][c] = L.T[tid][c];
  }
#pragma unroll
  for (int r = 0; r < LR; ++r) {
    const long long row = own_row(base, r);
    if (row < base + LB || row >= g.n_p) continue;
#pragma unroll
    for (int m2 = 0; m2 < LB; ++m2) {                 // one L value live at a time (<= 128 VGPRs)
      const double l = A[(long long)(base + m2) * g.Na + row];
#pragma unroll
      for (int c = 0; c < LB; ++c) w[r][c] = __builtin_fma(-l, L.T[m2][c], w[r][c]);
    }
  }
  __syncthreads();                                   // L.T is rewritten by the next phase
}

// Launch k: block 0 = panel (strip k), blocks 1.. = strips k + 1 .. (update of step k-1).
__global__ __launch_bounds__(LT) void lu_step_kernel(double* __restrict__ A, LuGeo g, int k,
                                                     int* __restrict__ ipiv, int* __restrict__ status) {
  __shared__ StripLds L;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int strip = k + (int)blockIdx.x;
  const int base = k > 0 ? LB * (k - 1) : 0;
  const long long c0 = (long long)LB * strip;
  double w[LR][LB];
#pragma unroll
  for (int r = 0; r < LR; ++r) {
    const long long row = own_row(base, r);
#pragma unroll
    for (int c = 0; c < LB; ++c) w[r][c] = row < g.n_p ? A[(c0 + c) * g.Na + row] : 0.0;
  }
  if (k > 0) strip_apply(A, g, ipiv, k - 1, L, w);
  if (blockIdx.x == 0) {
    // factor strip k: columns j, pivot rows g0 = 16 k + j (unrolled: w is indexed by j)
#pragma unroll
    for (int j = 0; j < LB; ++j) {
      const long long g0 = (long long)LB * k + j;
      double bv = -1.0;
      long long bi = g.n_p;
#pragma unroll
      for (int r = 0; r < LR; ++r) {
        const long long row = own_row(base, r);
        const double av = fabs(w[r][j]);
        if (row >= g0 && row < g.n_p && av > bv) { bv = av; bi = row; }   // first max per thread
      }
#pragma unroll
      for (int m2 = 32; m2 > 0; m2 >>= 1) {
        const double ov = __shfl_xor(bv, m2, 64);
        const long long oi = __shfl_xor(bi, m2, 64);
        if (ov > bv || (ov == bv && oi < bi)) { bv = ov; bi = oi; }
      }
      if (lane == 0) { L.redv[wave] = bv; L.redi[wave] = (int)bi; }
      __syncthreads();
      double pv = L.redv[0];
      long long p = L.redi[0];
      for (int u = 1; u < LT / 64; ++u)
        if (L.redv[u] > pv || (L.redv[u] == pv && L.redi[u] < p)) { pv = L.redv[u]; p = L.redi[u]; }
      // swap rows g0 <-> p inside the strip; prow = the pivot row
#pragma unroll
      for (int r = 0; r < LR; ++r) {
        const long long row = own_row(base, r);
        if (row == p) {
#pragma unroll
          for (int c = 0; c < LB; ++c) L.prow[c] = w[r][c];
        }
        if (row == g0) {
#pragma unroll
          for (int c = 0; c < LB; ++c) L.grow[c] = w[r][c];
        }
      }
      if (tid == 0) {
        ipiv[g0] = (int)p;
        if (!(pv > 0.0)) atomicOr(status, 1);        // an exactly zero (or NaN) pivot: singular
      }
      __syncthreads();
      const double rp = 1.0 / L.prow[j];
#pragma unroll
      for (int r = 0; r < LR; ++r) {
        const long long row = own_row(base, r);
        if (row == g0) {
#pragma unroll
          for (int c = 0; c < LB; ++c) w[r][c] = L.prow[c];
        } else if (row == p) {
#pragma unroll
          for (int c = 0; c < LB; ++c) w[r][c] = L.grow[c];
        }
        if (row > g0 && row < g.n_p) {
          const double l = w[r][j] * rp;
          w[r][j] = l;
#pragma unroll
          for (int c = 0; c < LB; ++c)
            if (c > j) w[r][c] = __builtin_fma(-l, L.prow[c], w[r][c]);
        }
      }
    }
  }
#pragma unroll
  for (int r = 0; r < LR; ++r) {
    const long long row = own_row(base, r);
    if (row >= g.n_p) continue;
#pragma unroll
    for (int c = 0; c < LB; ++c) A[(c0 + c) * g.Na + row] = w[r][c];
  }
}

// ------------------------------------------------------------------------------ solve
// out[:, 16 strip .. 16 strip + 15] = inv(A) e_col: forward with the interleaved swaps and L,
// backward with U.  One workgroup per strip of the identity.
__global__ __launch_bounds__(LT) void lu_solve_kernel(double* __restrict__ out, const double* __restrict__ A,
                                                      LuGeo g, const int* __restrict__ ipiv) {
  __shared__ StripLds L;
  const int tid = threadIdx.x;
  const int strip = blockIdx.x;
  double w[LR][LB];
#pragma unroll
  for (int r = 0; r < LR; ++r) {
    const long long row = own_row(0, r);
#pragma unroll
    for (int c = 0; c < LB; ++c) w[r][c] = row == (long long)LB * strip + c ? 1.0 : 0.0;
  }
  // forward: per step the swaps, W_s = L11^-1 W_s, W_below -= L21 W_s
  for (int s = 0; s < g.nbs; ++s) {
    const int b = LB * s;
    step_perm(L, ipiv, s);
    apply_perm(L, w, 0);
    if (tid < LB * LB) {
      const int i = tid & 15, j = tid >> 4;
      L.L11[i][j] = A[(long long)(b + j) * g.Na + b + i];
    }
#pragma unroll
    for (int r = 0; r < LR; ++r) {
      const long long row = own_row(0, r);
      if (row >= b && row < b + LB) {
#pragma unroll
        for (int c = 0; c < LB; ++c) L.T[row - b][c] = w[r][c];
      }
    }
    __syncthreads();
    if (tid < LB) {
      for (int i = 1; i < LB; ++i) {
        double x = L.T[i][tid];
        for (int m2 = 0; m2 < i; ++m2) x = __builtin_fma(-L.L11[i][m2], L.T[m2][tid], x);
        L.T[i][tid] = x;
      }
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < LR; ++r) {
      const long long row = own_row(0, r);
      if (row >= b && row < b + LB) {
#pragma unroll
        for (int c = 0; c < LB; ++c) w[r][c] = L.T[row - b][c];
      } else if (row >= b + LB && row < g.n_p) {
#pragma unroll
        for (int m2 = 0; m2 < LB; ++m2) {
          const double l = A[(long long)(b + m2) * g.Na + row];
#pragma unroll
          for (int c = 0; c < LB; ++c) w[r][c] = __builtin_fma(-l, L.T[m2][c], w[r][c]);
        }
      }
    }
    __syncthreads();
  }
  // backward: per step from the last, W_s = U_ss^-1 W_s, W_above -= U_above,s W_s
  for (int s = g.nbs - 1; s >= 0; --s) {
    const int b = LB * s;
    if (tid < LB * LB) {
      const int i = tid & 15, j = tid >> 4;
      L.L11[i][j] = A[(long long)(b + j) * g.Na + b + i];     // U block (upper incl. diagonal)
    }
#pragma unroll
    for (int r = 0; r < LR; ++r) {
      const long long row = own_row(0, r);
      if (row >= b && row < b + LB) {
#pragma unroll
        for (int c = 0; c < LB; ++c) L.T[row - b][c] = w[r][c];
      }
    }
    __syncthreads();
    if (tid < LB) {
      for (int i = LB - 1; i >= 0; --i) {
        double x = L.T[i][tid];
        for (int m2 = i + 1; m2 < LB; ++m2) x = __builtin_fma(-L.L11[i][m2], L.T[m2][tid], x);
        L.T[i][tid] = x / L.L11[i][i];
      }
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < LR; ++r) {
      const long long row = own_row(0, r);
      if (row >= b && row < b + LB) {
#pragma unroll
        for (int c = 0; c < LB; ++c) w[r][c] = L.T[row - b][c];
      } else if (row < b) {
#pragma unroll
        for (int m2 = 0; m2 < LB; ++m2) {
          const double uu = A[(long long)(b + m2) * g.Na + row];
#pragma unroll
          for (int c = 0; c < LB; ++c) w[r][c] = __builtin_fma(-uu, L.T[m2][c], w[r][c]);
        }
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int r = 0; r < LR; ++r) {
    const long long row = own_row(0, r);
    if (row >= g.n) continue;
#pragma unroll
    for (int c = 0; c < LB; ++c) {
      const long long col = (long long)LB * strip + c;
      if (col < g.n) out[row * g.n + col] = w[r][c];
    }
  }
}

inline size_t a256(size_t x) { return (x + 255) & ~(size_t)255; }

LuGeo make_lu_geo(int n) {
  LuGeo g;
  g.n = n;
  g.n_p = (n + LB - 1) / LB * LB;
  g.nbs = g.n_p / LB;
  g.Na = g.n_p;
  return g;
}

}  // namespace

// Internal (bo_fit.hip): workspace bytes and the LU inverse of one objective (BO_OK,
// BO_ERR_SINGULAR on an exactly zero pivot, BO_ERR_UNSUPPORTED above the register capacity).
size_t bo_lu_workspace_size(int64_t n) {
  const LuGeo g = make_lu_geo((int)n);
  return a256((size_t)g.Na * g.n_p * sizeof(double)) + a256((size_t)g.n_p * sizeof(int)) + 256;
}

int bo_lu_max_n() { return LT * LR; }

int bo_lu_inverse(double* out, const double* km, int64_t ld, int64_t n, double jitter, void* ws,
                  size_t ws_bytes, hipStream_t s) {
  if (n < 1 || n > LT * LR) return BO_ERR_UNSUPPORTED;
  if (ws_bytes < bo_lu_workspace_size(n)) return BO_ERR_WORKSPACE;
  const LuGeo g = make_lu_geo((int)n);
  double* A = (double*)ws;
  int* ipiv = (int*)((char*)ws + a256((size_t)g.Na * g.n_p * sizeof(double)));
  int* status = (int*)((char*)ipiv + a256((size_t)g.n_p * sizeof(int)));
  BO_CHECK_HIP(hipMemsetAsync(status, 0, sizeof(int), s));
  const unsigned tiles = (unsigned)((g.n_p + 31) / 32);
  hipLaunchKernelGGL(lu_init_kernel, dim3(tiles, tiles), dim3(256), 0, s, A, g, km, (long long)ld,
                     jitter);
  for (int k = 0; k < g.nbs; ++k) {
    const int blocks = k > 0 ? g.nbs - k : 1;      // the panel + the strips right of it
    hipLaunchKernelGGL(lu_step_kernel, dim3(blocks), dim3(LT), 0, s, A, g, k, ipiv, status);
  }
  hipLaunchKernelGGL(lu_solve_kernel, dim3(g.nbs), dim3(LT), 0, s, out, (const double*)A, g, (const int*)ipiv);
  BO_CHECK_HIP(hipGetLastError());
  int hs = 0;
  BO_CHECK_HIP(hipMemcpyAsync(&hs, status, sizeof(int), hipMemcpyDeviceToHost, s));
  BO_CHECK_HIP(hipStreamSynchronize(s));
  return hs ? BO_ERR_SINGULAR : BO_OK;
}
