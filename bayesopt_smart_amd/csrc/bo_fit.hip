// GP fit on device: compute_mll and invert_k on one blocked right-looking Cholesky, one kernel
// launch per 32-column step.
//
//   bo_compute_mll  numba_kernels.py:152-235   sum over objectives of the GP marginal log
//                   likelihood of K/pv + 1e-8 I with y centred on the prior mean and scaled by
//                   its population std.
//   bo_invert_k     numba_kernels.py:370-403   inv(K + 1e-6 I) per objective (the reference's
//                   LAPACK gesv); Cholesky first, blocked LU with partial pivoting (LAPACK's
//                   getrf row choice) for any objective whose Cholesky fails or whose K is not
//                   symmetric.
//
// One factorisation serves both: the Cholesky of an AUGMENTED lower-triangular matrix
//
//        [ K    .  ]      factoring only the first n_p columns leaves     [ L          .          ]
//    A = [ B    C  ]      (n_p = N padded to 32 with an identity block)   [ B L^-T     C - B K^-1 B^T ]
//
//   * compute_mll: B = (y - pm)^T (one row), no C:  the bottom row becomes z = L^-1 (y - pm), so
//     |z|^2 / var(y) is the data-fit term yc . alpha of :216-222 (yc = (y - pm) / std), and
//     log det = 2 sum log L_ii (:225-229);
//   * invert_k:    B = I, C = 0:  the bottom-right block becomes -K^-1 (lower triangle).  B L^-T
//     is upper triangular: bottom row block b is structurally zero in column blocks < b, and C's
//     tile (b, c) receives its first contribution at step b (no zero fill).
//
// A is COLUMN-major (element (i, j) at j * Na + i) and lives in the workspace.  Launch k (32-column
// step k, one launch per step; the kernel boundary is the only synchronisation) runs two roles:
//   * panel (column block k): every panel workgroup applies step k-1's update to the diagonal
//     tile and to ITS 32-row slab (MFMA, 4 waves), then wave 0 factors the diagonal tile and
//     solves its slab rows in the same register sweep -- lanes 0..31 hold the diagonal rows,
//     lanes 32..63 the slab rows, one row per lane: column j's pivot is a v_readlane, its
//     entries below the diagonal are both L_jj^-1 a_j for the tile and the triangular solve of
//     the slab (X L_kk^T = A_pk), and the next column is updated first so that the chain per
//     column is readlane -> rsqrt -> mul -> readlane -> fma.  Every panel workgroup factors the
//     diagonal tile redundantly (no inter-workgroup hand-off inside the launch);
//   * update (column blocks > k, and C for the inverse): A_pc -= L_p,k-1 L_c,k-1^T for every live
//     32 x 32 tile, one tile per wave (32 v_mfma_f64_16x16x4_f64), applying step k-1 one launch
//     late (lookahead: the panel of step k needs only its own column block).
// The critical path per step is one panel: ~0.4 us of MFMA, a 32-column register factorisation
// and the kernel boundary.  Round 2 used two launches per 64-column step with a 64-long serial
// substitution chain on one wave (45 us per panel at N = 2048).

#include "bo_common.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

#include <vector>
#include <chrono>

namespace {

constexpr int NB = 32;      // column block (panel width) and update tile

// waves per SIMD the step kernel is compiled for (register budget 512 / BO_FIT_WAVES per lane)
// launch-per-step path: write-through (sc1) stores of the panel columns and updated tiles, so
// that no step ends with dirty L2 lines to write back at its kernel boundary
// (r04h, N = 2048: MLL 0.966 -> 0.865 ms, inverse 1.535 -> 1.44 ms)
#ifndef BO_FIT_WB
constexpr int kStepStoreAux = 16;
#else
constexpr int kStepStoreAux = 0;
#endif

#if defined(BO_FIT_U8) && !defined(BO_FIT_NODEFER)
#error "BO_FIT_U8 (8-byte tile accesses, A/B only) has no rank-64 form: build it with BO_FIT_NODEFER"
#endif
#ifdef BO_FIT_NODEFER
constexpr bool kFitNoDefer = true;
#else
constexpr bool kFitNoDefer = false;
#endif

#ifndef BO_FIT_WAVES
#define BO_FIT_WAVES 2
#endif

// Diagnostic build (BO_BUILD_VARIANT=DEF_FIT_TIMING): workgroup 0 of every role stamps the
// 100 MHz real-time clock at its phase boundaries; bo_debug_fit_timing reads them back.
#ifdef BO_FIT_TIMING
__device__ long long bo_fit_tstamp[8192];
__device__ int bo_fit_tcount;
#define FIT_STAMP(tag)                                                              \
  do {                                                                              \
    if ((threadIdx.x & 63) == 0) {                                                  \
      const int _i = atomicAdd(&bo_fit_tcount, 1);                                  \
      if (_i < 4096) {                                                              \
        bo_fit_tstamp[2 * _i] = ((long long)k << 16) | ((long long)blockIdx.x << 4) | (tag); \
        bo_fit_tstamp[2 * _i + 1] = (long long)wall_clock64();                      \
      }                                                                             \
    }                                                                               \
  } while (0)
#else
#define FIT_STAMP(tag) ((void)0)
#endif
constexpr int CS = 33;      // LDS row stride (doubles) of the panel tile
constexpr int FG = 8;       // columns per LDS broadcast group of the panel factorisation

struct FitParams {
  double pv[BO_MAX_OBJ], pm[BO_MAX_OBJ], ls2[BO_MAX_OBJ], jitter;
};

// Geometry of the augmented system (per objective): K part n_p = 32 nbt rows/columns; bottom
// rows 32 (MLL: row n_p = y - pm) or n_p (inverse: B = I); columns n_p (MLL) or 2 n_p (inverse:
// the C block).  ostride = Na * ncols doubles per objective.
struct Geo {
  int n, nbt, ident, n_obj;
  long long Na, ncols, ostride;
};

// per-objective partials of the MLL: [2 nbt + 1] doubles (log det partial per step, |z|^2
// partial per step, var(y - pm)); statuses after all objectives' partials
__host__ __device__ inline int part_len(const Geo& g) { return 2 * g.nbt + 1; }

typedef unsigned int u2v __attribute__((ext_vector_type(2)));
typedef unsigned int u4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ d4 mfma64(double a, double b, d4 c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

// 1 / sqrt(x) and sqrt(x) from v_rsq_f64 (about 2^-29 relative) by two Goldschmidt steps: g ->
// sqrt(x), h -> 1 / (2 sqrt(x)); five dependent operations after the rsq.  NaN for x <= 0 or NaN
// (the caller flags the pivot).
__device__ __forceinline__ void rsqrt_sqrt(double x, double& rs, double& sq) {
  const double y = __builtin_amdgcn_rsq(x);
  double g = x * y, h = 0.5 * y;
  double r = __builtin_fma(-g, h, 0.5);
  g = __builtin_fma(g, r, g);
  h = __builtin_fma(h, r, h);
  r = __builtin_fma(-g, h, 0.5);
  sq = __builtin_fma(g, r, g);
  rs = 2.0 * __builtin_fma(h, r, h);
}

__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// triangular index t -> row u, t = u (u + 1) / 2 + rest
__device__ __forceinline__ int tri_row(long long t) {
  int u = (int)((sqrt(8.0 * (double)t + 1.0) - 1.0) * 0.5);
  while ((long long)(u + 1) * (u + 2) / 2 <= t) ++u;
  while ((long long)u * (u + 1) / 2 > t) --u;
  return u;
}

// ------------------------------------------------------------------------------- init
// Lower 32 x 32 tiles of the augmented matrix (one workgroup per tile, linear tile index over the
// lower triangle of the K part, then the bottom tiles that are live in their column block).
//   K part (i, j < N):  MLL: e + 1e-8 d_ij with e = exp(-0.5 |x_i - x_j|^2 / ls^2), the
//                       correlation matrix K / pv of :195-198 (the reference's (pv e) / pv, within
//                       an ulp: the value depends on ls only, so per-objective MLLs memoise
//                       across Powell's pv moves), and pv e -- update_k's value
//                       (numba_kernels.py:352-361) -- stored to the caller's kernel_matrix in
//                       both triangles (compute_mll rebuilds it, :178-185);
//                       inverse: K[i][j] + 1e-6 d_ij from the caller's kernel_matrix, with
//                       K[i][j] == K[j][i] checked (an asymmetric K takes the LU path);
//   K padding:          identity;
//   bottom:             MLL: row n_p = y_j - pm (j < N), the rest 0; inverse: B = I on the live
//                       tiles (bottom block b in column block j >= b).
// Extra workgroups (MLL, one per objective) compute var(y - pm), population (np.std squared).
__global__ __launch_bounds__(256) void fit_init_kernel(double* __restrict__ A, Geo g,
                                                       double* __restrict__ km, long long ld,
                                                       const double* __restrict__ x, int dim,
                                                       const double* __restrict__ y, long long ld_y,
                                                       FitParams p, double* __restrict__ part,
                                                       int* __restrict__ status, int tiles_per_obj,
                                                       int* __restrict__ flags, long long n_flags) {
  __shared__ double tile[NB][NB + 1];
  __shared__ double red[256];
  const int tid = threadIdx.x;
  const long long np_ = (long long)g.nbt * NB;
  const int work_blocks = g.n_obj * tiles_per_obj + (g.ident ? 0 : g.n_obj);
  if ((int)blockIdx.x >= work_blocks) {
    // the persistent factorisation's flag words (dequeue counter, panel flags, tile versions):
    // zeroed here, one launch before the kernel that polls them
    for (long long i = (long long)(blockIdx.x - work_blocks) * 256 + tid; i < n_flags;
         i += (long long)(gridDim.x - work_blocks) * 256)
      flags[i] = 0;
    return;
  }
  if ((int)blockIdx.x >= g.n_obj * tiles_per_obj) {
    // var(y - pm) of one objective (two passes, as np.std)
    const int o = blockIdx.x - g.n_obj * tiles_per_obj;
    double s = 0.0;
    for (int i = tid; i < g.n; i += 256) s += y[(long long)i * ld_y + o] - p.pm[o];
    red[tid] = s;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) { if (tid < w) red[tid] += red[tid + w]; __syncthreads(); }
    const double mean = red[0] / g.n;
    __syncthreads();
    s = 0.0;
    for (int i = tid; i < g.n; i += 256) {
      const double d = (y[(long long)i * ld_y + o] - p.pm[o]) - mean;
      s += d * d;
    }
    red[tid] = s;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) { if (tid < w) red[tid] += red[tid + w]; __syncthreads(); }
    if (tid == 0) part[(long long)o * part_len(g) + 2 * g.nbt] = red[0] / g.n;
    return;
  }
  const int o = blockIdx.x / tiles_per_obj;
  long long t = blockIdx.x % tiles_per_obj;
  const long long tri = (long long)g.nbt * (g.nbt + 1) / 2;
  int ti, tj;                                  // tile row / column block
  if (t < tri) {
    ti = tri_row(t);
    tj = (int)(t - (long long)ti * (ti + 1) / 2);
  } else {                                      // bottom tiles
    t -= tri;
    if (g.ident) {                              // (nbt + b, j) for b <= j: column-wise triangle
      const int u = tri_row(t);
      tj = u;
      ti = g.nbt + (int)(t - (long long)u * (u + 1) / 2);
    } else {
      ti = g.nbt;
      tj = (int)t;
    }
  }
  double* Ao = A + (long long)o * g.ostride;
  const long long r0 = (long long)ti * NB, c0 = (long long)tj * NB;
  const int c = tid >> 5, r = tid & 31;         // column-major writes: lane r = row, c + 8 pass
  if (ti < g.nbt) {
    // K part: values into the LDS tile [row][col]
    if (!g.ident) {
      double* ko = km + (long long)o * ld * ld;
      for (int e = tid; e < NB * NB; e += 256) {
        const int rr = e >> 5, cc = e & 31;     // row rr, column cc (consecutive threads: columns)
        const long long i = r0 + rr, j = c0 + cc;
        double v = 0.0;
        if (i < g.n && j < g.n) {
          double sq = 0.0;
          for (int k = 0; k < dim; ++k) {
            const double d = x[i * dim + k] - x[j * dim + k];
            sq = __builtin_fma(d, d, sq);
          }
          v = exp(-0.5 * sq / p.ls2[o]);        // K / pv, the correlation matrix of :195-198
          ko[i * ld + j] = p.pv[o] * v;         // row i of the caller's matrix (update_k's value)
        }
        tile[rr][cc] = v;
      }
      __syncthreads();
      if (ti != tj) {                           // the mirrored tile (rows j, columns i) from LDS
        double* ko2 = km + (long long)o * ld * ld;
        for (int e = tid; e < NB * NB; e += 256) {
          const int rr = e >> 5, cc = e & 31;   // row c0 + rr, column r0 + cc
          const long long i = c0 + rr, j = r0 + cc;
          if (i < g.n && j < g.n) ko2[i * ld + j] = p.pv[o] * tile[cc][rr];
        }
      }
    } else {
      const double* ko = km + (long long)o * ld * ld;
      bool asym = false;
      for (int e = tid; e < NB * NB; e += 256) {
        const int rr = e >> 5, cc = e & 31;
        const long long i = r0 + rr, j = c0 + cc;
        tile[rr][cc] = (i < g.n && j < g.n) ? ko[i * ld + j] : 0.0;
      }
      __syncthreads();
      if (ti != tj) {                           // K[j][i] (the upper tile) against K[i][j]
        for (int e = tid; e < NB * NB; e += 256) {
          const int rr = e >> 5, cc = e & 31;   // K[c0 + rr][r0 + cc] vs tile[cc][rr]
          const long long i = c0 + rr, j = r0 + cc;
          if (i < g.n && j < g.n) {
            const double u = ko[i * ld + j], l = tile[cc][rr];
            asym = asym || !(u == l || (u != u && l != l));
          }
        }
      } else {
        for (int e = tid; e < NB * NB; e += 256) {
          const int rr = e >> 5, cc = e & 31;
          const long long i = r0 + rr, j = c0 + cc;
          if (i < g.n && j < g.n && rr > cc) {
            const double u = tile[cc][rr], l = tile[rr][cc];
            asym = asym || !(u == l || (u != u && l != l));
          }
        }
      }
      if (asym) atomicOr(status + o, 2);
    }
    __syncthreads();
#pragma unroll
    for (int pass = 0; pass < NB / 8; ++pass) {
      const int cc = c + 8 * pass;
      const long long i = r0 + r, j = c0 + cc;
      if (i < j) continue;
      double v;
      if (i < g.n && j < g.n) {
        v = tile[r][cc] + (i == j ? p.jitter : 0.0);
      } else {
        v = i == j ? 1.0 : 0.0;
      }
      Ao[j * g.Na + i] = v;
    }
    return;
  }
  // bottom tiles
#pragma unroll
  for (int pass = 0; pass < NB / 8; ++pass) {
    const int cc = c + 8 * pass;
    const long long i = r0 + r, j = c0 + cc;
    double v;
    if (g.ident) v = (i - np_ == j && j < g.n) ? 1.0 : 0.0;
    else v = (i == np_ && j < g.n) ? y[j * ld_y + o] - p.pm[o] : 0.0;
    Ao[j * g.Na + i] = v;
  }
}

// ------------------------------------------------------------------------------- step
// Panel role of launch k, one workgroup per (objective, slab block sb > k); wave 0 factors.
__device__ __forceinline__ void panel_role(double* __restrict__ Ao, const Geo& g, int o, int k, int w_slab, int n_panel,
                                           double* __restrict__ part, int* __restrict__ status,
                                           double* Cs, double* colb) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 15, lg = lane >> 4;
  const long long Na = g.Na;
  const long long cK = (long long)k * NB;
  const int sb = k + 1 + w_slab;
  const int lr0 = 16 * wave;                                      // local rows: 0..31 diagonal, 32..63 slab
  const long long grow0 = wave < 2 ? cK + lr0 : (long long)sb * NB + (lr0 - 32);
  const int ntb = wave == 0 ? 1 : 2;                              // rows 0..15: t 16..31 are upper
  const bool stamp = w_slab == 0 && wave == 0 && o == 0;
  const bool stamp_last = w_slab == n_panel - 1 && wave == 0 && o == g.n_obj - 1;
  if (stamp) FIT_STAMP(1);
  if (stamp_last) FIT_STAMP(5);
  // this wave's A values at its D positions (t = 16 tb + lg + 4 i, row grow0 + li), issued first
  // with the operand loads: one memory round trip before the MFMAs
  double av_a[2][4];
#pragma unroll
  for (int tb = 0; tb < 2; ++tb)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int t = 16 * tb + lg + 4 * i;
      av_a[tb][i] = (tb < ntb && !(wave < 2 && lr0 + li < t)) ? Ao[(cK + t) * Na + grow0 + li] : 0.0;
    }
  d4 acc[2];
  acc[0] = (d4){0.0, 0.0, 0.0, 0.0};
  acc[1] = acc[0];
  if (k > 0) {
    // step k-1's update of this wave's 16 rows: D[t][r] = sum_s L(diag t, s) L(row r, s)
    const double* Lp = Ao + (cK - NB) * Na;
    double av[2][8], bv[8];
    // bottom block k of the inverse is structurally zero in column block k-1 (never written)
    const bool zero_rows = g.ident && wave >= 2 && sb == g.nbt + k;
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) bv[ks] = zero_rows ? 0.0 : Lp[(4 * ks + lg) * Na + grow0 + li];
#pragma unroll
    for (int tb = 0; tb < 2; ++tb)
#pragma unroll
      for (int ks = 0; ks < 8; ++ks)
        av[tb][ks] = tb < ntb ? Lp[(4 * ks + lg) * Na + cK + 16 * tb + li] : 0.0;
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      acc[0] = mfma64(av[0][ks], bv[ks], acc[0]);
      if (ntb > 1) acc[1] = mfma64(av[1][ks], bv[ks], acc[1]);
    }
  }
  // C = A - D into LDS, row-major [local row][t]; diagonal rows' upper entries zeroed
#pragma unroll
  for (int tb = 0; tb < 2; ++tb)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int t = 16 * tb + lg + 4 * i;
      const int rl = lr0 + li;
      Cs[rl * CS + t] = av_a[tb][i] - acc[tb][i];               // masked entries: 0 - 0
    }
  if (stamp) FIT_STAMP(2);
  __syncthreads();
  if (stamp_last) FIT_STAMP(6);
  if (wave != 0) return;
  double a[NB];
#pragma unroll
  for (int t = 0; t < NB; ++t) a[t] = Cs[lane * CS + t];
  const long long row_l = lane < NB ? cK + lane : (long long)sb * NB + lane - NB;   // this lane's row
  // column block k as a buffer resource: element (row, cK + j) at row * 8 + j * col_bytes
  const int col_bytes = (int)(Na * 8);
  const __amdgpu_buffer_rsrc_t colr =
      __builtin_amdgcn_make_buffer_rsrc((void*)(Ao + cK * Na), (short)0, NB * col_bytes, 0x00020000);
  const int row_off = (int)(row_l * 8);
  double dj = 1.0;
  bool bad = false;
  // Groups of FG columns: inside a group each new column reaches the group's later columns by
  // v_readlane (the pivot chain: readlane -> rsqrt -> mul -> readlane -> fma); at the end of the
  // group its FG columns reach the remaining columns through ONE LDS round trip (lanes 0..31 store
  // their FG values, every lane reads row t's FG values as a broadcast) -- 4 LDS round trips on
  // the chain instead of 32 (one per column: 4.5 us per factorisation measured).
#pragma unroll
  for (int j0 = 0; j0 < NB; j0 += FG) {
#pragma unroll
    for (int j = j0; j < j0 + FG; ++j) {
      const double piv = bo_readlane_d(a[j], j);
      bad = bad || !(piv > 0.0);                                 // potrf: a_jj <= 0 or NaN
      double rs, d;
      rsqrt_sqrt(piv, rs, d);
      a[j] = lane == j ? d : a[j] * rs;                         // lanes > j: L_ij; lanes < j: unused
      dj = lane == j ? d : dj;
      // column j is final: store it now (the slab rows; the diagonal tile's L is read by no later
      // step and the step's other panel workgroups read that tile's input), so that the stores
      // drain under the rest of the factorisation
      // (a buffer store: the lane's row offset in one VGPR, the column offset in an SGPR -- plain
      // stores kept 32 64-bit addresses live and spilled)
      // branch-free: the lanes that must not store get an offset past the resource (dropped)
      __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2v, a[j]), colr,
                                            lane >= NB ? row_off : 0x40000000, j * col_bytes, kStepStoreAux);
#pragma unroll
      for (int t = j + 1; t < j0 + FG; ++t) a[t] = __builtin_fma(-a[j], bo_readlane_d(a[j], t), a[t]);
    }
    if (j0 + FG < NB) {
      if (lane < NB) {
#pragma unroll
        for (int c = 0; c < FG; ++c) colb[lane * FG + c] = a[j0 + c];
      }
      wave_lds_sync();
#pragma unroll
      for (int t = j0 + FG; t < NB; ++t) {
        double s0 = a[t];
#pragma unroll
        for (int c = 0; c < FG; ++c) s0 = __builtin_fma(-a[j0 + c], colb[t * FG + c], s0);
        a[t] = s0;
      }
      wave_lds_sync();                                           // colb is rewritten by the next group
    }
  }
  if (stamp) FIT_STAMP(3);
#ifdef BO_FIT_TIMING
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (stamp) FIT_STAMP(4);
  if (stamp_last) FIT_STAMP(7);
#endif
  if (g.ident) {
    if (w_slab == 0 && bad && lane == 0) atomicOr(status + o, 1);
    return;
  }
  if (w_slab == 0) {
    double v = (lane < NB && cK + lane < g.n) ? log(dj) : 0.0;
#pragma unroll
    for (int m = 32; m > 0; m >>= 1) v += __shfl_xor(v, m, 64);
    if (lane == 0) {
      part[(long long)o * part_len(g) + k] = v;
      if (bad) status[o] = 1;                  // MLL: one flag, plain store (pinned host memory)
    }
  }
  if (sb == g.nbt && lane == NB) {                               // the bottom row z = L^-1 (y - pm)
    double s = 0.0;
#pragma unroll
    for (int t = 0; t < NB; ++t) s = __builtin_fma(a[t], a[t], s);
    part[(long long)o * part_len(g) + g.nbt + k] = s;
  }
}

// L part (MLL and inverse): the column blocks c = k+1 .. nbt-1, each with its row blocks
// [c, RB); numbered from the last column, whose count is `base`:  S(u) = u base + u (u - 1) / 2.
__device__ __forceinline__ long long lpart_S(long long u, long long base) { return u * base + u * (u - 1) / 2; }

// Update role of launch k: one 32 x 32 tile per wave.
//   UPD 0: step k-1 on every column block >= k+1 (and the inverse's C part)
//   UPD 1: step k-1 on column block k+1 only (the MLL's odd launches: what the next panel needs)
//   UPD 2: steps k-2 and k-1 together (rank 64) on every column block >= k+1 (the MLL's even
//          launches: each trailing tile is read and written once per two steps)
template <int UPD>
__device__ __forceinline__ void update_role(double* __restrict__ A, const Geo& g, int k, long long TL,
                                            long long TC, long long wt) {
  const int lane = threadIdx.x & 63, li = lane & 15, lg = lane >> 4;
  const long long per = TL + TC;
  if (wt >= per * g.n_obj) return;
  const int o = (int)(wt / per);
  long long t = wt % per;
  const long long np_ = (long long)g.nbt * NB;
  long long row0, col0;
  bool first = false;
  if (UPD == 1) {
    col0 = (long long)(k + 1) * NB;
    row0 = (k + 1 + t) * NB;
  } else if (t < TL) {
    const long long base = g.ident ? k + 1 : 2;
    const double bb = 2.0 * (double)base - 1.0;
    long long u = (long long)((-bb + sqrt(bb * bb + 8.0 * (double)t)) * 0.5);
    if (u < 0) u = 0;
    while (lpart_S(u + 1, base) <= t) ++u;
    while (lpart_S(u, base) > t) --u;
    const long long c = g.nbt - 1 - u;
    row0 = (c + (t - lpart_S(u, base))) * NB;
    col0 = c * NB;
  } else {
    t -= TL;
    const int u = tri_row(t);
    const long long cp = k - 1 - u;
    const long long b = cp + (t - (long long)u * (u + 1) / 2);
    row0 = np_ + b * NB;
    col0 = np_ + cp * NB;
    first = b == k - 1;                          // C tile (b, cp): first contribution at step b
  }
  double* Ao = A + (long long)o * g.ostride;
  const long long Na = g.Na;
  constexpr int R = UPD == 2 ? 2 : 1;                             // steps applied
  const double* Lp = Ao + (long long)(k - R) * NB * Na;           // L columns (k - R) * NB ..
  const bool stamp = wt == 0;
  const bool stamp_last = wt == per * g.n_obj - 1;
  if (stamp) FIT_STAMP(8);
  if (stamp_last) FIT_STAMP(10);
#ifndef BO_FIT_U8
  // 16-byte accesses: the MFMA rows are interleaved (A-side m -> tile column 2 m + tb, B-side n ->
  // tile row 2 n + rb), so that each lane's two 16 x 16 blocks sit in adjacent doubles: every load
  // and store moves a double2 (the 8-byte forms run at 0.54-0.70x the 16-byte rate)
  typedef double dv2 __attribute__((ext_vector_type(2)));
  dv2 cv[2][4];
#pragma unroll
  for (int tb = 0; tb < 2; ++tb)
#pragma unroll
    for (int i = 0; i < 4; ++i)
      cv[tb][i] = first ? (dv2){0.0, 0.0}
                        : *(const dv2*)(Ao + (col0 + 2 * (lg + 4 * i) + tb) * Na + row0 + 2 * li);
  dv2 av[8 * R], bv[8 * R];
#pragma unroll
  for (int ks = 0; ks < 8 * R; ++ks) {
    av[ks] = *(const dv2*)(Lp + (4 * ks + lg) * Na + col0 + 2 * li);
    bv[ks] = *(const dv2*)(Lp + (4 * ks + lg) * Na + row0 + 2 * li);
  }
  d4 acc[2][2];
#pragma unroll
  for (int tb = 0; tb < 2; ++tb)
#pragma unroll
    for (int rb = 0; rb < 2; ++rb) acc[tb][rb] = (d4){0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int ks = 0; ks < 8 * R; ++ks)
#pragma unroll
    for (int tb = 0; tb < 2; ++tb)
#pragma unroll
      for (int rb = 0; rb < 2; ++rb) acc[tb][rb] = mfma64(av[ks][tb], bv[ks][rb], acc[tb][rb]);
  // D[m][n] (m = lg + 4 i, n = li) of block (tb, rb) is tile element (column 2 m + tb, row 2 n + rb)
  const int col_bytes = (int)(Na * 8);
  const __amdgpu_buffer_rsrc_t tr =
      __builtin_amdgcn_make_buffer_rsrc((void*)(Ao + col0 * Na), (short)0, NB * col_bytes, 0x00020000);
  const int voff = (int)(((long long)(2 * lg) * Na + row0 + 2 * li) * 8);
#pragma unroll
  for (int tb = 0; tb < 2; ++tb)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const dv2 v = {cv[tb][i].x - acc[tb][0][i], cv[tb][i].y - acc[tb][1][i]};
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4v, v), tr, voff, (8 * i + tb) * col_bytes,
                                             kStepStoreAux);
    }
#else
  // the tile's current values first (one memory round trip with the operands)
  double cv[2][2][4];
#pragma unroll
  for (int tb = 0; tb < 2; ++tb)
#pragma unroll
    for (int rb = 0; rb < 2; ++rb)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        cv[tb][rb][i] = first ? 0.0 : Ao[(col0 + 16 * tb + lg + 4 * i) * Na + row0 + 16 * rb + li];
  double av[2][8], bv[2][8];
#pragma unroll
  for (int ks = 0; ks < 8; ++ks)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      av[h][ks] = Lp[(4 * ks + lg) * Na + col0 + 16 * h + li];
      bv[h][ks] = Lp[(4 * ks + lg) * Na + row0 + 16 * h + li];
    }
  d4 acc[2][2];
#pragma unroll
  for (int tb = 0; tb < 2; ++tb)
#pragma unroll
    for (int rb = 0; rb < 2; ++rb) acc[tb][rb] = (d4){0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int ks = 0; ks < 8; ++ks)
#pragma unroll
    for (int tb = 0; tb < 2; ++tb)
#pragma unroll
      for (int rb = 0; rb < 2; ++rb) acc[tb][rb] = mfma64(av[tb][ks], bv[rb][ks], acc[tb][rb]);
  // D[t][r]: t = 16 tb + lg + 4 i (tile column), r = 16 rb + li (tile row)
#pragma unroll
  for (int tb = 0; tb < 2; ++tb)
#pragma unroll
    for (int rb = 0; rb < 2; ++rb)
#pragma unroll
      for (int i = 0; i < 4; ++i)
      {
        double* dst = Ao + (col0 + 16 * tb + lg + 4 * i) * Na + row0 + 16 * rb + li;
        if constexpr (kStepStoreAux != 0) __hip_atomic_store(dst, cv[tb][rb][i] - acc[tb][rb][i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else *dst = cv[tb][rb][i] - acc[tb][rb][i];
      }
#endif
#ifdef BO_FIT_TIMING
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (stamp) FIT_STAMP(9);
  if (stamp_last) FIT_STAMP(11);
#endif
}

// ---------------------------------------------------------------------------- finish
// out[o][i][j] = -C[max(i, j)][min(i, j)] (C = the bottom-right block, lower triangle): the
// symmetric K^-1.  32 x 32 output tiles: lower tiles read C column-major (coalesced), upper tiles
// the mirrored lower tile through LDS; writes are row-major.
__global__ __launch_bounds__(256) void inv_extract_kernel(double* __restrict__ out, long long out_stride,
                                                          const double* __restrict__ A,
                                                          Geo g, const int* __restrict__ status) {
  __shared__ double tile[NB][NB + 1];
  const int o = blockIdx.z;
  if (status[o]) return;                        // this objective goes through the LU path
  const int bi = blockIdx.y, bj = blockIdx.x;   // output tile (rows 32 bi, columns 32 bj)
  const long long np_ = (long long)g.nbt * NB;
  const double* Ao = A + (long long)o * g.ostride;
  out += (long long)o * out_stride;
  const long long n = g.n;
  const int lo = bi >= bj ? bi : bj, hi = bi >= bj ? bj : bi;   // source lower tile (lo, hi)
  const int tid = threadIdx.x, c = tid >> 5, r = tid & 31;
  // tile[cc][rr] = C(32 lo + rr, 32 hi + cc): column-major reads (rr consecutive)
#pragma unroll
  for (int pass = 0; pass < NB / 8; ++pass) {
    const int cc = c + 8 * pass;
    tile[cc][r] = Ao[(np_ + (long long)hi * NB + cc) * g.Na + np_ + (long long)lo * NB + r];
  }
  __syncthreads();
#pragma unroll
  for (int pass = 0; pass < NB / 8; ++pass) {
    const int rr = c + 8 * pass;                 // output row 32 bi + rr, column 32 bj + r
    const long long i = (long long)bi * NB + rr, j = (long long)bj * NB + r;
    if (i >= n || j >= n) continue;
    // element (i, j): lower (i >= j) -> C(i, j) = tile[j - 32 hi][i - 32 lo] with lo = bi
    const long long gr = i >= j ? i : j, gc = i >= j ? j : i;
    const double v = tile[gc - (long long)hi * NB][gr - (long long)lo * NB];
    out[i * n + j] = -v;
  }
}

// the f64 MFMA's read wait states (BO_NOPS_F64_MFMA, bo_common.h) between the last MFMA writing
// the accumulators and their first VALU read (the round-1 gfx950 hazard)
__device__ __forceinline__ void mfma_fence_acc(d4 (&acc)[2][2]) {
  asm volatile(BO_NOPS_F64_MFMA
               : "+v"(acc[0][0]), "+v"(acc[0][1]), "+v"(acc[1][0]), "+v"(acc[1][1]));
}

// --------------------------------------------------------------- inverse refinement
// One Newton step on the Cholesky-path inverse, X' = X + X (I - A X) with A = K + jitter I: the
// residual I - A X' is (I - A X)^2 up to the rounding of the two products, so X' carries the
// residual of a backward-stable solve (LAPACK gesv's, the reference's np.linalg.inv,
// numba_kernels.py:401) where the product form L^-T L^-1 of the factorisation alone was 12x (N =
// 512) to 144x (N = 2048) above it (round-4 GPU log).  Two MFMA GEMMs per objective:
//   MODE 0:  R = I - (K + jitter I) X          (A operand: the caller's K, leading dimension ld)
//   MODE 1:  out = X + X R                     (A operand: X)
// Both A operands are symmetric (the Cholesky path runs only for a symmetric K; X is the
// mirrored lower triangle), so A[i][k] is read as A[k][i]: every operand load is 16 consecutive
// doubles of a row.  32 x 32 per wave (2 x 2 v_mfma_f64_16x16x4_f64 blocks), k in blocks of 32
// with the next block's loads in flight.
//   SPLITK (n <= 1024): a 32 x 32 tile per workgroup, k split over its 4 waves (a quarter of n
//     each), the partial tiles summed through LDS in a fixed order (deterministic): 4x the waves
//     of the other form at N = 512, where it was latency-bound (update_k + invert_k 0.272 ->
//     0.241 ms at C3);
//   otherwise a 64 x 64 tile per workgroup, each wave its own 32 x 32 tile over the whole k (at
//     N = 2048 the split form measured 4.29 vs 4.14 ms).
template <int MODE, bool SPLITK>
__global__ __launch_bounds__(256) void inv_refine_kernel(const double* __restrict__ Am, long long lda, long long a_os,
                                                         double jitter, const double* __restrict__ Bm,
                                                         long long b_os, const double* __restrict__ Xm,
                                                         long long x_os, double* __restrict__ D, long long d_os,
                                                         int n, const int* __restrict__ status) {
  __shared__ double part[SPLITK ? 3 : 1][32][33];
  const int o = blockIdx.z;
  if (status[o]) return;                        // LU objective: refined by nothing (gesv itself)
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int li = lane & 15, lg = lane >> 4;
  const int i0 = SPLITK ? blockIdx.y * 32 : blockIdx.y * 64 + (wave >> 1) * 32;
  const int j0 = SPLITK ? blockIdx.x * 32 : blockIdx.x * 64 + (wave & 1) * 32;
  if (!SPLITK && (i0 >= n || j0 >= n)) return;   // wave-uniform; no barriers below
  const double* Ao = Am + (long long)o * a_os;
  const double* Bo = Bm + (long long)o * b_os;
  const long long ldb = n;
  // this wave's k range: a quarter of n, rounded to whole k-steps of 4 (SPLITK), else all of it
  const int kq = ((n + 15) / 16) * 4;
  const int k_lo = SPLITK ? wave * kq : 0, k_hi = SPLITK ? min(n, (wave + 1) * kq) : n;
  bool ca[2], cb[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    ca[t] = i0 + 16 * t + li < n;
    cb[t] = j0 + 16 * t + li < n;
  }
  constexpr int KS = 8;                         // k-steps (of 4) per block
  double av[2][KS][2], bv[2][KS][2];
  auto load = [&](int buf, int kb) {
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const int k = kb + 4 * s + lg;
      const bool kok = k < k_hi;
      const double* ra = Ao + (long long)k * lda;
      const double* rb = Bo + (long long)k * ldb;
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int ci = i0 + 16 * t + li, cj = j0 + 16 * t + li;
        double a = (kok && ca[t]) ? ra[ci] : 0.0;
        if (MODE == 0 && k == ci) a += jitter;   // numba_kernels.py:397-398
        av[buf][s][t] = a;
        bv[buf][s][t] = (kok && cb[t]) ? rb[cj] : 0.0;
      }
    }
  };
  d4 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = (d4){0.0, 0.0, 0.0, 0.0};
  auto compute = [&](int buf) {
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) acc[a][b] = mfma64(av[buf][s][a], bv[buf][s][b], acc[a][b]);
  };
  // ping-pong with static buffer indices (a variable index puts the arrays in scratch)
  if (k_lo < k_hi) {                            // wave-uniform
    load(0, k_lo);
    for (int kb = k_lo; kb < k_hi; kb += 8 * KS) {
      if (kb + 4 * KS < k_hi) load(1, kb + 4 * KS);
      compute(0);
      if (kb + 4 * KS >= k_hi) break;
      if (kb + 8 * KS < k_hi) load(0, kb + 8 * KS);
      compute(1);
    }
  }
  mfma_fence_acc(acc);
  // waves 1..3 hand their partial tiles to wave 0 (D layout: row 16 a + lg + 4 r, column 16 b + li)
  if (SPLITK && wave > 0) {
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int r = 0; r < 4; ++r) part[wave - 1][16 * a + lg + 4 * r][16 * b + li] = acc[a][b][r];
  }
  if constexpr (SPLITK) {
    __syncthreads();
    if (wave != 0) return;
  }
  const double* Xo = Xm + (long long)o * x_os;
  double* Do = D + (long long)o * d_os;
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int ti = 16 * a + lg + 4 * r, tj = 16 * b + li;
        const int i = i0 + ti, j = j0 + tj;
        if (i >= n || j >= n) continue;
        const double v = SPLITK ? ((acc[a][b][r] + part[0][ti][tj]) + part[1][ti][tj]) + part[SPLITK ? 2 : 0][ti][tj]
                                : acc[a][b][r];
        const long long e = (long long)i * n + j;
        Do[e] = MODE == 0 ? ((i == j ? 1.0 : 0.0) - v) : Xo[e] + v;
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

// ------------------------------------------------------------- persistent factorisation
// The same factorisation as one launch (after fit_init_kernel): the launch-per-step schedule's
// work units become TASKS of one queue that every workgroup of a persistent grid dequeues in
// order (one returning atomic add per task), each task waiting only on tasks before it in the
// queue (a dependency flag per panel and a version counter per tile): the kernel boundary per
// 32-column step (~3.7 us at N = 512, profiles/r03_fit_stamps_a.txt) becomes a flag hand-off,
// and the panel of step k+1 starts while the bulk of step k's trailing update still runs.
//
// Tasks of block k (the old launch k), in queue order:
//   A_{k-1}[k+1]   step k-1 applied to column block k+1's tiles (what the panel of step k+1 needs;
//                  4 tiles per task, one per wave)
//   P(k, w)        the panel of step k for slab k+1+w (applies step k-1 to its rows of column
//                  block k, factors the diagonal tile redundantly and solves the slab)
//   A_{k-1}[rest]  step k-1 applied to column blocks >= k+2 (and to the inverse's C block)
// Every dependency points backwards (P(k) needs P(k-1) and A_{k-2}[k]; A_s needs P(s) and the
// tile's previous version), so any number of resident workgroups makes progress: the queue order
// is a topological order and a workgroup takes its next task only after finishing the current.
//
// Hand-off (MI355X guide, Guideline 16, R1 with sc1 loads): every store of A is an sc1 store, every
// load of A an sc1 load (L1 bypassed: no acquire needed); each storing wave drains vmcnt(0), the
// workgroup meets at a barrier, then one lane stores the flag (relaxed, agent scope).  Waits are
// bounded: a wave that spins past the bound (or sees another's abort) sets the abort word and
// the task is skipped; the host then reruns the call on the launch-per-step path.
constexpr int PMAX_STEPS = 128;

struct PPlan {
  int steps, total;
  int force_abort;                           // test-only (BO_FIT_TEST_ABORT=1): abort at once
  int blk[PMAX_STEPS + 1];                   // first task of block k
};

// flag words (fit_init_kernel zeroes them): [0] dequeue counter, [1] abort; per objective from
// word 16: pflag [nbt][nbt] (P(k) of slab k+1+w done), tver [RB][nbt] (L-part tile versions:
// steps applied), tverC [nbt][nbt] (the inverse's C tiles)
__host__ __device__ inline int p_rb(const Geo& g) { return g.ident ? 2 * g.nbt : g.nbt + 1; }
__host__ __device__ inline long long p_per_obj(const Geo& g) {
  return 2ll * g.nbt * g.nbt + (long long)p_rb(g) * g.nbt;
}
__host__ __device__ inline long long p_flag_words(const Geo& g) { return 16 + g.n_obj * p_per_obj(g); }
__device__ __forceinline__ int* pf_panel(int* f, const Geo& g, int o, int k, int w) {
  return f + 16 + o * p_per_obj(g) + (long long)k * g.nbt + w;
}
__device__ __forceinline__ int* pf_tver(int* f, const Geo& g, int o, int rb, int cb) {
  return f + 16 + o * p_per_obj(g) + (long long)g.nbt * g.nbt + (long long)rb * g.nbt + cb;
}
__device__ __forceinline__ int* pf_tverc(int* f, const Geo& g, int o, int b, int cp) {
  return f + 16 + o * p_per_obj(g) + (long long)g.nbt * g.nbt + (long long)p_rb(g) * g.nbt + (long long)b * g.nbt + cp;
}

__device__ __forceinline__ int ld_flag(const int* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_flag(int* p, int v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_sc1(const double* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1(double* p, double v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The calling wave waits until *fp >= want on every active lane (one flag per lane, all loads in
// flight at once).  false on abort: the spin bound (~1 s) passed here or another wave gave up.
__device__ bool wave_wait(const int* fp, int want, bool active, int* abort_w) {
  for (unsigned spins = 0;; ++spins) {
    const bool ok = !active || ld_flag(fp) >= want;
    if (__ballot(!ok) == 0ull) return true;
    if ((spins & 63u) == 63u) {
      if (ld_flag(abort_w) != 0) return false;
      if (spins > (1u << 20)) {
        if ((threadIdx.x & 63) == 0) st_flag(abort_w, 1);
        return false;
      }
    }
    __builtin_amdgcn_s_sleep(2);
  }
}

// rows of L-part row block rb start receiving updates at step s0 (the inverse's bottom block b
// is structurally zero in column blocks < b)
__device__ __forceinline__ int p_s0(const Geo& g, int rb) { return (g.ident && rb >= g.nbt) ? rb - g.nbt : 0; }

__device__ __forceinline__ int p_n1(const Geo& g, int k) {      // tiles per objective of A_{k-1}[k+1]
  if (k < 1 || k + 1 >= g.nbt) return 0;
  return g.ident ? g.nbt - 1 : g.nbt - k;
}
__device__ __forceinline__ int p_npanel(const Geo& g, int k) { return k < g.nbt ? (g.ident ? g.nbt : g.nbt - k) : 0; }
__device__ __forceinline__ void p_n2(const Geo& g, int k, long long& TL2, long long& TC) {
  TL2 = 0;
  TC = 0;
  if (k < 1) return;
  const long long m2 = g.nbt - k - 2, base = g.ident ? k + 1 : 2;
  TL2 = m2 > 0 ? m2 * base + m2 * (m2 - 1) / 2 : 0;
  TC = g.ident ? (long long)k * (k + 1) / 2 : 0;
}

struct PTile {
  int o, rb, cb;            // L part: row / column block; C part: b / cp
  bool cpart, first;
};

// One 32 x 32 tile of step s's trailing update on one wave (the update role's body with sc1
// loads and stores).  Returns after the wave's stores are issued.
__device__ __forceinline__ void p_tile_update(double* __restrict__ A, const Geo& g, int s, const PTile& t) {
  const int lane = threadIdx.x & 63, li = lane & 15, lg = lane >> 4;
  const long long np_ = (long long)g.nbt * NB;
  long long row0, col0;
  if (t.cpart) {
    row0 = np_ + (long long)t.rb * NB;
    col0 = np_ + (long long)t.cb * NB;
  } else {
    row0 = (long long)t.rb * NB;
    col0 = (long long)t.cb * NB;
  }
  double* Ao = A + (long long)t.o * g.ostride;
  const long long Na = g.Na;
  const double* Lp = Ao + (long long)s * NB * Na;
#ifndef BO_FIT_U8
  // 16-byte sc1 buffer loads and stores, rows interleaved as in update_role
  typedef double dv2 __attribute__((ext_vector_type(2)));
  const int col_bytes = (int)(Na * 8);
  const __amdgpu_buffer_rsrc_t lr = __builtin_amdgcn_make_buffer_rsrc((void*)Lp, (short)0, NB * col_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t tr =
      __builtin_amdgcn_make_buffer_rsrc((void*)(Ao + col0 * Na), (short)0, NB * col_bytes, 0x00020000);
  const int voff_t = (int)(((long long)(2 * lg) * Na + row0 + 2 * li) * 8);
  dv2 cv[2][4];
#pragma unroll
  for (int tb = 0; tb < 2; ++tb)
#pragma unroll
    for (int i = 0; i < 4; ++i)
      cv[tb][i] = t.first ? (dv2){0.0, 0.0}
                          : __builtin_bit_cast(dv2, __builtin_amdgcn_raw_buffer_load_b128(tr, voff_t, (8 * i + tb) * col_bytes, 16));
  const int voff_a = (int)(((long long)lg * Na + col0 + 2 * li) * 8), voff_b = (int)(((long long)lg * Na + row0 + 2 * li) * 8);
  dv2 av[8], bv[8];
#pragma unroll
  for (int ks = 0; ks < 8; ++ks) {
    av[ks] = __builtin_bit_cast(dv2, __builtin_amdgcn_raw_buffer_load_b128(lr, voff_a, 4 * ks * col_bytes, 16));
    bv[ks] = __builtin_bit_cast(dv2, __builtin_amdgcn_raw_buffer_load_b128(lr, voff_b, 4 * ks * col_bytes, 16));
  }
  d4 acc[2][2];
#pragma unroll
  for (int tb = 0; tb < 2; ++tb)
#pragma unroll
    for (int rb = 0; rb < 2; ++rb) acc[tb][rb] = (d4){0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int ks = 0; ks < 8; ++ks)
#pragma unroll
    for (int tb = 0; tb < 2; ++tb)
#pragma unroll
      for (int rb = 0; rb < 2; ++rb) acc[tb][rb] = mfma64(av[ks][tb], bv[ks][rb], acc[tb][rb]);
#pragma unroll
  for (int tb = 0; tb < 2; ++tb)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const dv2 v = {cv[tb][i].x - acc[tb][0][i], cv[tb][i].y - acc[tb][1][i]};
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4v, v), tr, voff_t, (8 * i + tb) * col_bytes, 16);
    }
#else
  double cv[2][2][4];
#pragma unroll
  for (int tb = 0; tb < 2; ++tb)
#pragma unroll
    for (int rb = 0; rb < 2; ++rb)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        cv[tb][rb][i] = t.first ? 0.0 : ld_sc1(Ao + (col0 + 16 * tb + lg + 4 * i) * Na + row0 + 16 * rb + li);
  double av[2][8], bv[2][8];
#pragma unroll
  for (int ks = 0; ks < 8; ++ks)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      av[h][ks] = ld_sc1(Lp + (4 * ks + lg) * Na + col0 + 16 * h + li);
      bv[h][ks] = ld_sc1(Lp + (4 * ks + lg) * Na + row0 + 16 * h + li);
    }
  d4 acc[2][2];
#pragma unroll
  for (int tb = 0; tb < 2; ++tb)
#pragma unroll
    for (int rb = 0; rb < 2; ++rb) acc[tb][rb] = (d4){0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int ks = 0; ks < 8; ++ks)
#pragma unroll
    for (int tb = 0; tb < 2; ++tb)
#pragma unroll
      for (int rb = 0; rb < 2; ++rb) acc[tb][rb] = mfma64(av[tb][ks], bv[rb][ks], acc[tb][rb]);
#pragma unroll
  for (int tb = 0; tb < 2; ++tb)
#pragma unroll
    for (int rb = 0; rb < 2; ++rb)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        st_sc1(Ao + (col0 + 16 * tb + lg + 4 * i) * Na + row0 + 16 * rb + li, cv[tb][rb][i] - acc[tb][rb][i]);
#endif
}

// The panel of step k for slab sb = k + 1 + w of objective o, on the whole workgroup: step k-1's
// update of the diagonal tile and the slab (MFMA, 4 waves x 16 rows), then the 32-column
// factorisation with the columns split over the waves: wave g owns columns 8g..8g+7 for all 64
// rows (lane = row: 0..31 the diagonal tile, 32..63 the slab).  Wave g factors its 8 columns
// (in-wave pivot chain: readlane -> rsqrt -> scale -> readlane -> fma), publishes them in LDS,
// and every later wave applies their rank-8 update to its own columns: the critical path holds 4
// groups of 8 pivots plus 3 rank-8 updates, where one wave used to do all 32 columns' updates.
// SC: the persistent kernel's hand-off (sc1 loads and write-through stores, the completion flag);
// false for the launch-per-step path, whose kernel boundaries order the steps.
template <bool SC>
__device__ __forceinline__ double ld_a(const double* p) {
  if constexpr (SC) return ld_sc1(p);
  else return *p;
}

template <bool SC>
__device__ __forceinline__ void p_panel(double* __restrict__ Ao, const Geo& g, int o, int k, int w,
                                        double* Cs, double* colb, double* red, int* pflag) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 15, lg = lane >> 4;
  const long long Na = g.Na;
  const long long cK = (long long)k * NB;
  const int sb = k + 1 + w;
  const int lr0 = 16 * wave;
  const long long grow0 = wave < 2 ? cK + lr0 : (long long)sb * NB + (lr0 - 32);
  const int ntb = wave == 0 ? 1 : 2;
  const bool stamp = w == 0 && wave == 0 && o == 0;
  (void)stamp;
  double av_a[2][4];
#pragma unroll
  for (int tb = 0; tb < 2; ++tb)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int t = 16 * tb + lg + 4 * i;
      av_a[tb][i] = (tb < ntb && !(wave < 2 && lr0 + li < t)) ? ld_a<SC>(Ao + (cK + t) * Na + grow0 + li) : 0.0;
    }
  d4 acc[2];
  acc[0] = (d4){0.0, 0.0, 0.0, 0.0};
  acc[1] = acc[0];
  if (k > 0) {
    const double* Lp = Ao + (cK - NB) * Na;
    double av[2][8], bv[8];
    const bool zero_rows = g.ident && wave >= 2 && sb == g.nbt + k;
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) bv[ks] = zero_rows ? 0.0 : ld_a<SC>(Lp + (4 * ks + lg) * Na + grow0 + li);
#pragma unroll
    for (int tb = 0; tb < 2; ++tb)
#pragma unroll
      for (int ks = 0; ks < 8; ++ks)
        av[tb][ks] = tb < ntb ? ld_a<SC>(Lp + (4 * ks + lg) * Na + cK + 16 * tb + li) : 0.0;
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      acc[0] = mfma64(av[0][ks], bv[ks], acc[0]);
      if (ntb > 1) acc[1] = mfma64(av[1][ks], bv[ks], acc[1]);
    }
  }
#pragma unroll
  for (int tb = 0; tb < 2; ++tb)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int t = 16 * tb + lg + 4 * i;
      Cs[(lr0 + li) * CS + t] = av_a[tb][i] - acc[tb][i];
    }
  __syncthreads();
  if (stamp) FIT_STAMP(3);
  // wave g: columns 8g .. 8g + 7 of every row
  const int c0 = 8 * wave;
  double a[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) a[c] = Cs[lane * CS + c0 + c];
  const int col_bytes = (int)(Na * 8);
  const __amdgpu_buffer_rsrc_t colr =
      __builtin_amdgcn_make_buffer_rsrc((void*)(Ao + cK * Na), (short)0, NB * col_bytes, 0x00020000);
  const long long row_l = lane < NB ? cK + lane : (long long)sb * NB + lane - NB;
  const int row_off = (int)(row_l * 8);
  double dj = 1.0;
  bool bad = false;
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    if (wave == p) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int J = 8 * p + j;                                 // == c0 + j (wave == p)
        const double piv = bo_readlane_d(a[j], J);
        bad = bad || !(piv > 0.0);                               // potrf: a_jj <= 0 or NaN
        double rs, d;
        rsqrt_sqrt(piv, rs, d);
        a[j] = lane == J ? d : a[j] * rs;
        dj = lane == J ? d : dj;
        // column J is final: the slab rows store it at once, write-through (sc1: the hand-off
        // to other CUs).  The diagonal tile's L is read by no later task (the panels of step k+1
        // and the trailing updates read only rows below it), and the other panels of this step
        // still read that tile's input values: it is not stored.
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2v, a[j]), colr,
                                              lane >= NB ? row_off : 0x40000000, J * col_bytes, SC ? 16 : kStepStoreAux);
#pragma unroll
        for (int t = j + 1; t < 8; ++t) a[t] = __builtin_fma(-a[j], bo_readlane_d(a[j], 8 * p + t), a[t]);
      }
      if (p < 3) {
#pragma unroll
        for (int c = 0; c < 8; ++c) colb[(p * 64 + lane) * 8 + c] = a[c];
      }
    }
    if (p < 3) {
      __syncthreads();
      if (wave > p) {                                            // rank-8 update from group p
        const double* L = colb + p * 64 * 8;
        double lr[8];
#pragma unroll
        for (int c = 0; c < 8; ++c) lr[c] = L[lane * 8 + c];
#pragma unroll
        for (int t = 0; t < 8; ++t) {
          double s0 = a[t];
#pragma unroll
          for (int c = 0; c < 8; ++c) s0 = __builtin_fma(-lr[c], L[(c0 + t) * 8 + c], s0);
          a[t] = s0;
        }
      }
    }
  }
  if (stamp) FIT_STAMP(4);
  // the panel is complete once every wave's column stores have drained: publish it now; the
  // partials below (a log per lane, two wave reductions) only feed the host
  if constexpr (SC) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) st_flag(pflag, 1);
  }
  // per-wave partials (own columns), combined through LDS
  double ldp = (lane >= c0 && lane < c0 + 8 && cK + lane < g.n) ? log(dj) : 0.0;
  double zp = 0.0;
#pragma unroll
  for (int c = 0; c < 8; ++c) zp = __builtin_fma(a[c], a[c], zp);
#pragma unroll
  for (int m = 32; m > 0; m >>= 1) ldp += __shfl_xor(ldp, m, 64);
  const double z_lane = __shfl(zp, NB, 64);                     // slab row 0 = the bottom row (MLL)
  if (lane == 0) {
    red[wave] = ldp;
    red[4 + wave] = z_lane;
    red[8 + wave] = bad ? 1.0 : 0.0;
  }
  __syncthreads();
}

// The panel's partials and status (thread 0), stored AFTER its completion flag: for the MLL they
// go to pinned host memory, and a drain behind such a store (~3 us, phase stamps) would sit on
// the critical path of the next panel.
__device__ __forceinline__ void p_panel_partials(const Geo& g, int o, int k, int w, double* __restrict__ part,
                                                 int* __restrict__ status, const double* red) {
  const int sb = k + 1 + w;
  const bool any_bad = red[8] + red[9] + red[10] + red[11] != 0.0;
  if (g.ident) {
    if (w == 0 && any_bad) atomicOr(status + o, 1);
  } else {
    if (w == 0) {
      part[(long long)o * part_len(g) + k] = ((red[0] + red[1]) + red[2]) + red[3];
      if (any_bad) status[o] = 1;
    }
    if (sb == g.nbt) part[(long long)o * part_len(g) + g.nbt + k] = ((red[4] + red[5]) + red[6]) + red[7];
  }
}

// Launch k: blocks [0, n_obj * n_panel) panel role, the rest update role (4 tiles per block).
// SPLIT: the persistent kernel's panel (4 waves share the 32-column sweep; the MLL), else the
// one-wave sweep (the inverse, whose nbt panels per step would crowd the trailing update's CUs:
// r04h, N = 2048, inverse 1.60 ms split vs 1.44 one-wave; MLL 0.865 vs 0.882)
template <bool SPLIT, int UPD>
__global__ __launch_bounds__(256, BO_FIT_WAVES) void fit_step_kernel(double* __restrict__ A, Geo g, int k, int n_panel,
                                                       long long TL, long long TC,
                                                       double* __restrict__ part, int* __restrict__ status) {
  __shared__ double Cs[2 * NB * CS];
  __shared__ double colb[SPLIT ? 3 * 64 * 8 : NB * NB];
  __shared__ double red[16];
  const int np = g.n_obj * n_panel;
  if ((int)blockIdx.x < np) {
    const int o = blockIdx.x / n_panel, w = blockIdx.x % n_panel;
    if constexpr (SPLIT) {
      p_panel<false>(A + (long long)o * g.ostride, g, o, k, w, Cs, colb, red, nullptr);
      if (threadIdx.x == 0) p_panel_partials(g, o, k, w, part, status, red);
    } else {
      panel_role(A + (long long)o * g.ostride, g, o, k, w, n_panel, part, status, Cs, colb);
    }
  } else {
    update_role<UPD>(A, g, k, TL, TC, ((long long)blockIdx.x - np) * 4 + (threadIdx.x >> 6));
  }
}

__global__ __launch_bounds__(256, 2) void fit_persist_kernel(double* __restrict__ A, Geo g, PPlan pl,
                                                             int* __restrict__ flags, double* __restrict__ part,
                                                             int* __restrict__ status, int* __restrict__ habort,
                                                             int* __restrict__ hdone) {
  __shared__ double Cs[2 * NB * CS];
  __shared__ double colb[3 * 64 * 8];
  __shared__ double red[16];
  __shared__ int s_task;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  int* abort_w = flags + 1;
  if (pl.force_abort && blockIdx.x == 0 && tid == 0) {
    // the recovery path under test: every wait that has to spin gives up, the host reruns
    st_flag(abort_w, 1);
    *habort = 1;
  }
  while (true) {
    if (tid == 0) s_task = atomicAdd(flags, 1);                  // dequeue (returning atomic)
    __syncthreads();
    const int t = s_task;
    __syncthreads();                                             // s_task is rewritten next round
    if (t >= pl.total) {
      if (hdone) {
        // completion word in pinned host memory, stored by the last workgroup to leave after every
        // workgroup's host-memory stores (partials, statuses, abort) drained: the host polls it
        // instead of waiting for the kernel's completion signal
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) {
          __threadfence_system();
          if (atomicAdd(flags + 2, 1) == (int)gridDim.x - 1) {
            __threadfence_system();
            __hip_atomic_store(hdone, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
          }
        }
      }
      return;
    }
    // block k: blk[k] <= t < blk[k + 1]
    int lo = 0, hi = pl.steps - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (pl.blk[mid] <= t) lo = mid;
      else hi = mid - 1;
    }
    const int k = lo;
    int r = t - pl.blk[k];
    const int n1 = p_n1(g, k);
    const int T1 = (g.n_obj * n1 + 3) / 4;
    const int nP = g.n_obj * p_npanel(g, k);
    if (r >= T1 && r < T1 + nP) {
      // ---- panel P(k, w)
      const int np = p_npanel(g, k);
      const int o = (r - T1) / np, w = (r - T1) % np;
      const int sb = k + 1 + w;
      const bool stamp = w == 0 && o == 0 && wave == 0;
      (void)stamp;
      if (stamp) FIT_STAMP(1);
      if (wave == 0) {
        // lanes 0..3: slab k's and slab sb's L column k-1, tiles (k, k) and (sb, k) at version k-1
        bool act = false;
        const int* fp = flags;
        int want = 0;
        if (k > 0) {
          const bool zero_rows = g.ident && sb == g.nbt + k;
          if (lane == 0) { fp = pf_panel(flags, g, o, k - 1, 0); want = 1; act = true; }
          if (lane == 1 && !zero_rows) { fp = pf_panel(flags, g, o, k - 1, sb - k); want = 1; act = true; }
          if (lane == 2) { fp = pf_tver(flags, g, o, k, k); want = k - 1; act = true; }
          if (lane == 3) { fp = pf_tver(flags, g, o, sb, k); want = max(k - 1 - p_s0(g, sb), 0); act = true; }
        }
        const bool ok = wave_wait(fp, want, act, abort_w);
        if (lane == 0) red[15] = ok ? 1.0 : 0.0;
        if (!ok && lane == 0) *habort = 1;                       // the host reruns the call
      }
      __syncthreads();
      if (stamp) FIT_STAMP(2);
      if (red[15] != 0.0) {
        // publishes its completion flag itself (after its stores drain), then the partials
        p_panel<true>(A + (long long)o * g.ostride, g, o, k, w, Cs, colb, red, pf_panel(flags, g, o, k, w));
        if (stamp) FIT_STAMP(5);
        if (tid == 0) p_panel_partials(g, o, k, w, part, status, red);
      }
      __syncthreads();
      continue;
    }
    // ---- 4 tiles of step s = k - 1 (one per wave)
    const int s = k - 1;
    PTile tl;
    bool have = false;
    if (r < T1) {
      const long long u = 4ll * r + wave;
      if (u < (long long)g.n_obj * n1) {
        have = true;
        tl.o = (int)(u / n1);
        const int i = (int)(u % n1);
        tl.cb = k + 1;
        tl.cpart = false;
        tl.first = false;
        if (!g.ident) tl.rb = k + 1 + i;
        else tl.rb = i < g.nbt - k - 1 ? k + 1 + i : g.nbt + (i - (g.nbt - k - 1));
      }
    } else {
      long long TL2, TC;
      p_n2(g, k, TL2, TC);
      const long long per = TL2 + TC;
      const long long u = 4ll * (r - T1 - nP) + wave;
      if (per > 0 && u < (long long)g.n_obj * per) {
        have = true;
        tl.o = (int)(u / per);
        long long tt = u % per;
        if (tt < TL2) {
          const long long base = g.ident ? k + 1 : 2;
          const double bb = 2.0 * (double)base - 1.0;
          long long uu = (long long)((-bb + sqrt(bb * bb + 8.0 * (double)tt)) * 0.5);
          if (uu < 0) uu = 0;
          while (lpart_S(uu + 1, base) <= tt) ++uu;
          while (lpart_S(uu, base) > tt) --uu;
          const long long c = g.nbt - 1 - uu;
          tl.cb = (int)c;
          tl.rb = (int)(c + (tt - lpart_S(uu, base)));
          tl.cpart = false;
          tl.first = false;
        } else {
          tt -= TL2;
          const int uu = tri_row(tt);
          const int cp = k - 1 - uu;
          const int b = cp + (int)(tt - (long long)uu * (uu + 1) / 2);
          tl.rb = b;
          tl.cb = cp;
          tl.cpart = true;
          tl.first = b == s;
        }
      }
    }
    const bool tstamp = r == 0 && T1 > 0 && wave == 0;
    (void)tstamp;
    if (tstamp) FIT_STAMP(8);
    // this wave's dependencies: L column s of both row blocks, the tile's previous version
    bool ok = true;
    if (have) {
      const int* fp = flags;
      int want = 0;
      bool act = false;
      const int sr = tl.cpart ? g.nbt + tl.rb : tl.rb, sc = tl.cpart ? g.nbt + tl.cb : tl.cb;
      if (lane == 0) { fp = pf_panel(flags, g, tl.o, s, sr - s - 1); want = 1; act = true; }
      if (lane == 1) { fp = pf_panel(flags, g, tl.o, s, sc - s - 1); want = 1; act = true; }
      if (lane == 2 && !tl.first) {
        fp = tl.cpart ? pf_tverc(flags, g, tl.o, tl.rb, tl.cb) : pf_tver(flags, g, tl.o, tl.rb, tl.cb);
        want = tl.cpart ? s - tl.rb : s - p_s0(g, tl.rb);
        act = true;
      }
      ok = wave_wait(fp, want, act, abort_w);
      if (tstamp) FIT_STAMP(9);
      if (ok) p_tile_update(A, g, s, tl);
    }
    if (!ok && lane == 0) *habort = 1;                            // the host reruns the call
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");            // every storing wave drains
    __syncthreads();
    if (tstamp) FIT_STAMP(10);
    if (have && ok && lane == 0) {
      // the tile's new version (steps applied), stored after the barrier that follows every
      // wave's drain
      int* vp = tl.cpart ? pf_tverc(flags, g, tl.o, tl.rb, tl.cb) : pf_tver(flags, g, tl.o, tl.rb, tl.cb);
      st_flag(vp, tl.cpart ? s - tl.rb + 1 : s - p_s0(g, tl.rb) + 1);
    }
    __syncthreads();
  }
}

inline size_t a256(size_t x) { return (x + 255) & ~(size_t)255; }

Geo make_geo(int n, int n_obj, bool ident) {
  Geo g;
  g.n = n;
  g.nbt = (n + NB - 1) / NB;
  g.ident = ident ? 1 : 0;
  g.n_obj = n_obj;
  const long long np_ = (long long)g.nbt * NB;
  g.Na = ident ? 2 * np_ : np_ + NB;
  g.ncols = ident ? 2 * np_ : np_;
  g.ostride = g.Na * g.ncols;
  return g;
}

size_t geo_bytes(const Geo& g) { return a256((size_t)g.n_obj * g.ostride * sizeof(double)); }

// init launch + one launch per step (inverse: one more, the last step's update of C)
int fit_factor(double* A, const Geo& g, const double* km, long long ld, const double* x, int dim,
               const double* y, long long ld_y, const FitParams& p, double* part, int* status,
               hipStream_t s) {
  const long long tri = (long long)g.nbt * (g.nbt + 1) / 2;
  const long long tiles = g.ident ? 2 * tri : tri + g.nbt;
  const long long blocks = g.n_obj * tiles + (g.ident ? 0 : g.n_obj);
  hipLaunchKernelGGL(fit_init_kernel, dim3((unsigned)blocks), dim3(256), 0, s, A, g, (double*)km, ld,
                     x, dim, y, ld_y, p, part, status, (int)tiles, (int*)nullptr, 0ll);
  BO_CHECK_HIP(hipGetLastError());
  const int steps = g.ident ? g.nbt + 1 : g.nbt;
  for (int k = 0; k < steps; ++k) {
    const int n_panel = k < g.nbt ? (g.ident ? g.nbt : g.nbt - k) : 0;
    // the MLL defers every odd step's trailing update to the next launch (UPD 1 / 2 above)
    const int upd_kind = g.ident || kFitNoDefer ? 0 : (k & 1) ? 1 : 2;
    long long TL = 0, TC = 0;
    if (k >= 1) {
      const long long m = g.nbt - 1 - k;
      const long long base = g.ident ? k + 1 : 2;
      TL = m > 0 ? m * base + m * (m - 1) / 2 : 0;
      TC = g.ident ? (long long)k * (k + 1) / 2 : 0;
      if (upd_kind == 1) TL = k + 1 < g.nbt ? g.nbt - k : 0;      // tiles (k+1 .. nbt, k+1)
    }
    const long long upd = ((TL + TC) * g.n_obj + 3) / 4;
    const long long grid = (long long)g.n_obj * n_panel + upd;
    if (grid == 0) continue;
    if (g.ident)
      hipLaunchKernelGGL((fit_step_kernel<false, 0>), dim3((unsigned)grid), dim3(256), 0, s, A, g, k, n_panel, TL, TC,
                         part, status);
    else if (upd_kind == 0)
      hipLaunchKernelGGL((fit_step_kernel<true, 0>), dim3((unsigned)grid), dim3(256), 0, s, A, g, k, n_panel, TL, TC,
                         part, status);
    else if (upd_kind == 1)
      hipLaunchKernelGGL((fit_step_kernel<true, 1>), dim3((unsigned)grid), dim3(256), 0, s, A, g, k, n_panel, TL, TC,
                         part, status);
    else
      hipLaunchKernelGGL((fit_step_kernel<true, 2>), dim3((unsigned)grid), dim3(256), 0, s, A, g, k, n_panel, TL, TC,
                         part, status);
  }
  return hipGetLastError() == hipSuccess ? BO_OK : BO_ERR_HIP;
}

// BO_FIT_TEST_ABORT=1 (tests only): every persistent launch raises its abort word at once, so
// that the host's rerun on the launch-per-step path runs (tests/test_gpu_fit_abort.py)
bool test_abort_enabled() {
  static const int on = [] {
    const char* e = getenv("BO_FIT_TEST_ABORT");
    return (e && strcmp(e, "1") == 0) ? 1 : 0;
  }();
  return on != 0;
}

// The persistent path: init launch (which also zeroes the flag words) + ONE fit_persist_kernel
// launch.  BO_ERR_UNSUPPORTED when the task list exceeds PMAX_STEPS blocks (the caller uses
// fit_factor).  *habort (host-visible) is set when a wait gave up: the caller reruns fit_factor.
// the largest column-block count the persistent schedule takes (BO_FIT_PERSIST_MAX_NBT overrides):
// at N = 2048 (64 blocks) the launch-per-step schedule measured faster (r04c: MLL 0.99 vs 1.06 ms,
// inverse 1.76 vs 2.38 ms) -- there the trailing update's throughput, not the panel chain, sets
// the time, and the one-atomic task queue serialises ~13k dequeues
int persist_max_nbt() {
  static const int v = [] {
    const char* e = getenv("BO_FIT_PERSIST_MAX_NBT");
    return e ? atoi(e) : 48;
  }();
  return v;
}

int fit_factor_persist(double* A, const Geo& g, const double* km, long long ld, const double* x, int dim,
                       const double* y, long long ld_y, const FitParams& p, double* part, int* status,
                       int* flags, int* habort, hipStream_t s, int* hdone = nullptr) {
  const int steps = g.ident ? g.nbt + 1 : g.nbt;
  if (steps > PMAX_STEPS || g.nbt > persist_max_nbt()) return BO_ERR_UNSUPPORTED;
  PPlan pl;
  memset(&pl, 0, sizeof(pl));
  pl.steps = steps;
  pl.force_abort = test_abort_enabled() ? 1 : 0;
  long long tot = 0;
  for (int k = 0; k < steps; ++k) {
    pl.blk[k] = (int)tot;
    const long long n1 = (k >= 1 && k + 1 < g.nbt) ? (g.ident ? g.nbt - 1 : g.nbt - k) : 0;
    const long long np = k < g.nbt ? (g.ident ? g.nbt : g.nbt - k) : 0;
    long long TL2 = 0, TC = 0;
    if (k >= 1) {
      const long long m2 = g.nbt - k - 2, base = g.ident ? k + 1 : 2;
      TL2 = m2 > 0 ? m2 * base + m2 * (m2 - 1) / 2 : 0;
      TC = g.ident ? (long long)k * (k + 1) / 2 : 0;
    }
    tot += (g.n_obj * n1 + 3) / 4 + g.n_obj * np + (g.n_obj * (TL2 + TC) + 3) / 4;
  }
  if (tot >= (1ll << 30)) return BO_ERR_UNSUPPORTED;
  pl.blk[steps] = (int)tot;
  pl.total = (int)tot;
  const long long tri = (long long)g.nbt * (g.nbt + 1) / 2;
  const long long tiles = g.ident ? 2 * tri : tri + g.nbt;
  const long long work = g.n_obj * tiles + (g.ident ? 0 : g.n_obj);
  const long long nf = p_flag_words(g);
  const long long zb = (nf + 4095) / 4096;
  hipLaunchKernelGGL(fit_init_kernel, dim3((unsigned)(work + zb)), dim3(256), 0, s, A, g, (double*)km, ld, x, dim,
                     y, ld_y, p, part, status, (int)tiles, flags, nf);
  BO_CHECK_HIP(hipGetLastError());
  const unsigned grid = (unsigned)(tot < 256 ? tot : 256);
  hipLaunchKernelGGL(fit_persist_kernel, dim3(grid), dim3(256), 0, s, A, g, pl, flags, part, status, habort, hdone);
  return hipGetLastError() == hipSuccess ? BO_OK : BO_ERR_HIP;
}

size_t flag_bytes(const Geo& g) { return a256((size_t)p_flag_words(g) * sizeof(int)); }

// BO_FIT_PATH=launches forces the launch-per-step path (A/B measurements); read once
bool persist_enabled() {
  static const int on = [] {
    const char* e = getenv("BO_FIT_PATH");
    return (e && strcmp(e, "launches") == 0) ? 0 : 1;
  }();
  return on != 0;
}
long long g_fit_paths[3];     // persistent, launch-per-step, persistent aborted -> rerun

// The MLL's wait for the persistent kernel: poll the completion word it stores in pinned memory
// (BO_FIT_HOSTWAIT=sync: the stream synchronisation instead).  false when the word did not come
// within ~0.5 s (the caller then synchronises the stream, which reports any fault).
bool host_poll_enabled() {
  static const int on = [] {
    const char* e = getenv("BO_FIT_HOSTWAIT");
    return (e && strcmp(e, "sync") == 0) ? 0 : 1;
  }();
  return on != 0;
}
bool host_poll(const int* hdone) {
  const auto t0 = std::chrono::steady_clock::now();
  for (unsigned i = 0;; ++i) {
    if (__atomic_load_n(hdone, __ATOMIC_ACQUIRE) != 0) return true;
    if ((i & 1023u) == 1023u && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(500)) return false;
    __builtin_ia32_pause();
  }
}

// how often each inverse path ran (per objective; bo_invert_k_path_counts)
long long g_inv_paths[3];     // Cholesky, blocked LU, Gauss-Jordan

// BO_INV_REFINE=0 leaves the Cholesky-path inverse unrefined (A/B measurements only)
bool refine_enabled() {
  static const int on = [] {
    const char* e = getenv("BO_INV_REFINE");
    return (e && strcmp(e, "0") == 0) ? 0 : 1;
  }();
  return on != 0;
}

// The Cholesky path's result: -C mirrored into X (the dead first columns of each objective's
// augmented matrix), then one Newton step X + X (I - (K + jitter I) X) into `out`
// (inv_refine_kernel).  Objectives whose factorisation failed are skipped on the device.
int inv_finish(double* out, double* A, const Geo& g, const double* km, long long ld, double jitter,
               const int* status, hipStream_t s) {
  const unsigned nt = (unsigned)g.nbt;
  const long long n = g.n;
  if (!refine_enabled()) {
    hipLaunchKernelGGL(inv_extract_kernel, dim3(nt, nt, g.n_obj), dim3(256), 0, s, out, n * n, A, g, status);
    return hipGetLastError() == hipSuccess ? BO_OK : BO_ERR_HIP;
  }
  double* X = A;                               // objective o: X at A_o, R at A_o + n^2 (< 2 n_p^2)
  double* R = A + n * n;
  hipLaunchKernelGGL(inv_extract_kernel, dim3(nt, nt, g.n_obj), dim3(256), 0, s, X, g.ostride, A, g, status);
  const bool split = n <= 1024;
  const unsigned tt = (unsigned)(split ? (n + 31) / 32 : (n + 63) / 64);
  auto k0 = split ? inv_refine_kernel<0, true> : inv_refine_kernel<0, false>;
  auto k1 = split ? inv_refine_kernel<1, true> : inv_refine_kernel<1, false>;
  hipLaunchKernelGGL(k0, dim3(tt, tt, g.n_obj), dim3(256), 0, s, km, ld, ld * ld, jitter, (const double*)X, g.ostride,
                     (const double*)nullptr, 0ll, R, g.ostride, (int)n, status);
  hipLaunchKernelGGL(k1, dim3(tt, tt, g.n_obj), dim3(256), 0, s, (const double*)X, n, g.ostride, 0.0,
                     (const double*)R, g.ostride, (const double*)X, g.ostride, out, n * n, (int)n, status);
  return hipGetLastError() == hipSuccess ? BO_OK : BO_ERR_HIP;
}

// pinned staging for the per-call read-back (one per host thread)
void* pinned(size_t bytes) {
  thread_local void* buf = nullptr;
  thread_local size_t cap = 0;
  if (cap < bytes) {
    if (buf) (void)hipHostFree(buf);
    buf = nullptr;
    cap = 0;
    if (hipHostMalloc(&buf, bytes, hipHostMallocDefault) != hipSuccess) return nullptr;
    cap = bytes;
  }
  return buf;
}

}  // namespace

extern "C" {

size_t bo_invert_k_workspace_size(int32_t n_obj, int64_t n) {
  if (n_obj < 1 || n < 1) return 0;
  const Geo g = make_geo((int)n, n_obj, true);
  // Gauss-Jordan scratch only above the blocked LU's capacity (the LU reuses the augmented region)
  const size_t lu = n > bo_lu_max_n() ? 2 * a256((size_t)n * n * sizeof(double)) : 0;
  return geo_bytes(g) + lu + 2 * a256((size_t)n * sizeof(int)) + 512 + flag_bytes(g);
}

int bo_invert_k(double* out, const double* km, int64_t ld, int32_t n_obj, int64_t n, void* ws,
                size_t ws_bytes, void* stream) {
  return bo_invert_k_jitter(out, km, ld, n_obj, n, BO_KERNEL_JITTER, ws, ws_bytes, stream);   // numba_kernels.py:397-398
}

int bo_invert_k_jitter(double* out, const double* km, int64_t ld, int32_t n_obj, int64_t n, double jitter,
                       void* ws, size_t ws_bytes, void* stream) {
  return bo_invert_k_ex(out, km, ld, n_obj, n, jitter, nullptr, nullptr, ws, ws_bytes, stream);
}

int bo_invert_k_ex(double* out, const double* km, int64_t ld, int32_t n_obj, int64_t n, double jitter,
                   const int32_t* lu_hint, int32_t* path_out, void* ws, size_t ws_bytes, void* stream) {
  if (!out || !km || n_obj < 1 || n_obj > BO_MAX_OBJ || n < 1 || ld < n) return BO_ERR_ARG;
  if (n > (1 << 15)) return BO_ERR_UNSUPPORTED;
  if (!ws || ws_bytes < bo_invert_k_workspace_size(n_obj, n)) return BO_ERR_WORKSPACE;
  hipStream_t s = (hipStream_t)stream;
  const Geo g = make_geo((int)n, n_obj, true);
  char* w = (char*)ws;
  double* A = (double*)w;
  char* lu = w + geo_bytes(g);
  const size_t gj = n > bo_lu_max_n() ? a256((size_t)n * n * sizeof(double)) : 0;
  double* bufA = (double*)lu;
  double* bufB = (double*)(lu + gj);
  int* piv = (int*)(lu + 2 * gj);
  int* perm = piv + a256((size_t)n * sizeof(int)) / sizeof(int);
  int* status = (int*)(lu + 2 * gj + 2 * a256((size_t)n * sizeof(int)));
  int* flags = (int*)(lu + 2 * gj + 2 * a256((size_t)n * sizeof(int)) + 512);
  int* dabort = status + BO_MAX_OBJ + 2;          // set by the persistent kernel when a wait gave up
  FitParams p;
  memset(&p, 0, sizeof(p));
  p.jitter = jitter;
  int fail[BO_MAX_OBJ], path[BO_MAX_OBJ];
  bool all_lu = lu_hint != nullptr;
  for (int o = 0; o < n_obj; ++o) {
    path[o] = 0;
    if (all_lu && lu_hint[o] == 0) all_lu = false;
  }
  if (all_lu) {
    // every objective's Cholesky failed last time (the caller's hint): no doomed attempt
    for (int o = 0; o < n_obj; ++o) fail[o] = 1;
  } else {
  int* hstat = (int*)pinned(sizeof(int) * (BO_MAX_OBJ + 4));
  if (!hstat) return BO_ERR_HIP;
  bool done = false;
  if (persist_enabled()) {
    BO_CHECK_HIP(hipMemsetAsync(status, 0, 256, s));
    const int st = fit_factor_persist(A, g, km, ld, nullptr, 0, nullptr, 0, p, nullptr, status, flags, dabort, s);
    if (st == BO_OK) {
      // after an abort the statuses are incomplete: the rerun below redoes the whole call
      const int st_f = inv_finish(out, A, g, km, ld, jitter, status, s);
      if (st_f != BO_OK) return st_f;
      BO_CHECK_HIP(hipMemcpyAsync(hstat, status, sizeof(int) * (BO_MAX_OBJ + 4), hipMemcpyDeviceToHost, s));
      BO_CHECK_HIP(hipStreamSynchronize(s));
      done = hstat[BO_MAX_OBJ + 2] == 0;
      __atomic_fetch_add(&g_fit_paths[done ? 0 : 2], 1, __ATOMIC_RELAXED);
    } else if (st != BO_ERR_UNSUPPORTED) {
      return st;
    }
  }
  if (!done) {
    __atomic_fetch_add(&g_fit_paths[1], 1, __ATOMIC_RELAXED);
    BO_CHECK_HIP(hipMemsetAsync(status, 0, 256, s));
    int st = fit_factor(A, g, km, ld, nullptr, 0, nullptr, 0, p, nullptr, status, s);
    if (st != BO_OK) return st;
    const int st_f = inv_finish(out, A, g, km, ld, jitter, status, s);
    if (st_f != BO_OK) return st_f;
    BO_CHECK_HIP(hipMemcpyAsync(hstat, status, sizeof(int) * n_obj, hipMemcpyDeviceToHost, s));
    BO_CHECK_HIP(hipStreamSynchronize(s));
  }
  for (int o = 0; o < n_obj; ++o) {
    fail[o] = hstat[o];
    if (!fail[o]) __atomic_fetch_add(&g_inv_paths[0], 1, __ATOMIC_RELAXED);
  }
  }   // Cholesky attempt
  for (int o = 0; o < n_obj; ++o) path[o] = fail[o] ? 1 : 0;
  // LU path for the objectives whose Cholesky failed or whose K is not symmetric: the blocked
  // LU with partial pivoting of bo_lu.hip, all of them in one launch sequence, in the (now free)
  // augmented-matrix region; Gauss-Jordan with partial pivoting above its register capacity
  // (N > 2048)
  {
    double* lu_out[BO_MAX_OBJ];
    const double* lu_km[BO_MAX_OBJ];
    int n_lu = 0;
    for (int o = 0; o < n_obj; ++o)
      if (fail[o]) { lu_out[n_lu] = out + (long long)o * n * n; lu_km[n_lu] = km + (long long)o * ld * ld; ++n_lu; }
    if (n_lu > 0 && n <= bo_lu_max_n() && geo_bytes(g) >= bo_lu_workspace_size(n, n_lu)) {
      const int st2 = bo_lu_inverse(lu_out, lu_km, n_lu, ld, n, jitter, A, geo_bytes(g), s);
      __atomic_fetch_add(&g_inv_paths[1], n_lu, __ATOMIC_RELAXED);
      if (st2 != BO_OK) return st2;
      for (int o = 0; o < n_obj; ++o) fail[o] = 0;
    }
  }
  for (int o = 0; o < n_obj; ++o) path[o] = fail[o] ? 2 : path[o];
  if (path_out)
    for (int o = 0; o < n_obj; ++o) path_out[o] = path[o];
  for (int o = 0; o < n_obj; ++o) {
    if (!fail[o]) continue;
    __atomic_fetch_add(&g_inv_paths[2], 1, __ATOMIC_RELAXED);
    int* gstat = status + BO_MAX_OBJ + 1;
    BO_CHECK_HIP(hipMemsetAsync(gstat, 0, sizeof(int), s));
    const long long total = (long long)n * n;
    hipLaunchKernelGGL(jitter_copy_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s,
                       bufA, km, (long long)ld, (int)n, o, jitter);
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

int bo_invert_k_path_counts(int64_t* counts) {
  if (!counts) return BO_ERR_ARG;
  for (int i = 0; i < 3; ++i) counts[i] = __atomic_load_n(&g_inv_paths[i], __ATOMIC_RELAXED);
  return BO_OK;
}

#ifdef BO_FIT_TIMING
// diagnostic build only: copy the phase stamps of the calls since the last read (pairs of
// [tag word, 100 MHz clock]) to `out` (host, 2 cap words) and reset the count; returns the count
__attribute__((visibility("default"))) int bo_debug_fit_timing(long long* out, int cap) {
  int cnt = 0;
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  if (hipMemcpyFromSymbol(&cnt, HIP_SYMBOL(bo_fit_tcount), sizeof(int)) != hipSuccess) return -1;
  if (cnt > cap) cnt = cap;
  if (cnt > 4096) cnt = 4096;
  if (cnt > 0 && hipMemcpyFromSymbol(out, HIP_SYMBOL(bo_fit_tstamp), sizeof(long long) * 2 * cnt) != hipSuccess)
    return -1;
  const int zero = 0;
  if (hipMemcpyToSymbol(HIP_SYMBOL(bo_fit_tcount), &zero, sizeof(int)) != hipSuccess) return -1;
  return cnt;
}
#endif

int bo_fit_path_counts(int64_t* counts) {
  if (!counts) return BO_ERR_ARG;
  for (int i = 0; i < 3; ++i) counts[i] = __atomic_load_n(&g_fit_paths[i], __ATOMIC_RELAXED);
  return BO_OK;
}

size_t bo_compute_mll_workspace_size(int32_t n_obj, int64_t n) {
  if (n_obj < 1 || n < 1) return 0;
  const Geo g = make_geo((int)n, n_obj, false);
  return geo_bytes(g) + a256((size_t)n_obj * part_len(g) * sizeof(double) + BO_MAX_OBJ * sizeof(int)) + 512 +
         flag_bytes(g);
}

int bo_compute_mll_each(double* mll_obj, const double* x, int32_t dim, const double* y, int64_t ld_y,
                        double* km, int64_t ld, int32_t n_obj, const double* pm, const double* pv,
                        const double* ls, int64_t n, void* ws, size_t ws_bytes, void* stream) {
  return bo_compute_mll_each_jitter(mll_obj, x, dim, y, ld_y, km, ld, n_obj, pm, pv, ls, n, BO_CHOLESKY_JITTER,
                                    ws, ws_bytes, stream);   // numba_kernels.py:211-214
}

int bo_compute_mll_each_jitter(double* mll_obj, const double* x, int32_t dim, const double* y, int64_t ld_y,
                               double* km, int64_t ld, int32_t n_obj, const double* pm, const double* pv,
                               const double* ls, int64_t n, double jitter, void* ws, size_t ws_bytes,
                               void* stream) {
  if (!mll_obj || !x || !y || !km || !pm || !pv || !ls || n_obj < 1 || n_obj > BO_MAX_OBJ ||
      n < 1 || ld < n || ld_y < n_obj || dim < 1)
    return BO_ERR_ARG;
  if (n > (1 << 16)) return BO_ERR_UNSUPPORTED;
  if (!ws || ws_bytes < bo_compute_mll_workspace_size(n_obj, n)) return BO_ERR_WORKSPACE;
  hipStream_t s = (hipStream_t)stream;
  const Geo g = make_geo((int)n, n_obj, false);
  double* A = (double*)ws;
  // the per-step partials and the status flags go straight to pinned host memory (plain device
  // stores; visible after the stream synchronisation): no status memset and no read-back copy
  // per call -- two launches and their boundaries less per Powell evaluation
  const size_t bytes = (size_t)n_obj * part_len(g) * sizeof(double) + sizeof(int) * (n_obj + 2);
  double* h = (double*)pinned(bytes);
  if (!h) return BO_ERR_HIP;
  double* part = h;
  int* status = (int*)(part + (size_t)n_obj * part_len(g));
  int* habort = status + n_obj;
  int* hdone = habort + 1;
  int* flags = (int*)((char*)ws + geo_bytes(g) +
                      a256((size_t)n_obj * part_len(g) * sizeof(double) + BO_MAX_OBJ * sizeof(int)) + 512);
  FitParams p;
  memset(&p, 0, sizeof(p));
  for (int o = 0; o < n_obj; ++o) {
    p.pv[o] = pv[o];
    p.pm[o] = pm[o];
    p.ls2[o] = ls[o] * ls[o];
  }
  p.jitter = jitter;
  bool done = false;
  if (persist_enabled()) {
    for (int o = 0; o <= n_obj + 1; ++o) status[o] = 0;          // statuses, abort, done
    const bool poll = host_poll_enabled();
    const int st = fit_factor_persist(A, g, km, ld, x, dim, y, ld_y, p, part, status, flags, habort, s,
                                      poll ? hdone : nullptr);
    if (st == BO_OK) {
      if (!poll || !host_poll(hdone)) BO_CHECK_HIP(hipStreamSynchronize(s));
      done = __atomic_load_n(habort, __ATOMIC_RELAXED) == 0;
      __atomic_fetch_add(&g_fit_paths[done ? 0 : 2], 1, __ATOMIC_RELAXED);
    } else if (st != BO_ERR_UNSUPPORTED) {
      return st;
    }
  }
  if (!done) {
    __atomic_fetch_add(&g_fit_paths[1], 1, __ATOMIC_RELAXED);
    for (int o = 0; o < n_obj; ++o) status[o] = 0;
    const int st = fit_factor(A, g, km, ld, x, dim, y, ld_y, p, part, status, s);
    if (st != BO_OK) return st;
    BO_CHECK_HIP(hipStreamSynchronize(s));
  }
  const int* hstat = (const int*)(h + (size_t)n_obj * part_len(g));
  for (int o = 0; o < n_obj; ++o)
    if (hstat[o]) return BO_ERR_NOT_PD;
  // mll_o = -0.5 yc.alpha - 0.5 log det - 0.5 N log(2 pi) (numba_kernels.py:222-232); yc.alpha =
  // |z|^2 / var(y - pm) (unscaled when the std is 0, :206-207)
  for (int o = 0; o < n_obj; ++o) {
    const double* q = h + (size_t)o * part_len(g);
    double ld_sum = 0.0, fit = 0.0;
    for (int k = 0; k < g.nbt; ++k) {
      ld_sum += q[k];
      fit += q[g.nbt + k];
    }
    const double var = q[2 * g.nbt];
    if (sqrt(var) > 0.0) fit /= var;
    mll_obj[o] = -0.5 * fit + (-0.5 * (2.0 * ld_sum)) + (-0.5 * (double)n * log(2.0 * 3.141592653589793));
  }
  return BO_OK;
}

int bo_compute_mll(double* mll_out, const double* x, int32_t dim, const double* y, int64_t ld_y,
                   double* km, int64_t ld, int32_t n_obj, const double* pm, const double* pv,
                   const double* ls, int64_t n, void* ws, size_t ws_bytes, void* stream) {
  double v[BO_MAX_OBJ];
  if (!mll_out) return BO_ERR_ARG;
  const int st = bo_compute_mll_each(v, x, dim, y, ld_y, km, ld, n_obj, pm, pv, ls, n, ws, ws_bytes, stream);
  if (st != BO_OK) return st;
  double tot = 0.0;                            // np.sum over objectives (:235): sequential, < 8 terms
  for (int o = 0; o < n_obj; ++o) tot += v[o];
  *mll_out = tot;
  return BO_OK;
}

}  // extern "C"
