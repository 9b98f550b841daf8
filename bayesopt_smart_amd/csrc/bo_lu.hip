// invert_k's LU path (numba_kernels.py:370-403: np.linalg.inv = LAPACK gesv(A, I)): blocked
// right-looking LU with partial pivoting (getrf's pivot: the first row of largest |a_ij| in
// the column, rows >= j), then inv(A) = U^-1 L^-1 P one 16-column strip of the identity at a
// time (getrs).  Taken by bo_invert_k for the objectives whose Cholesky fails (cond(K + 1e-6 I)
// of 1e14..1e18 with Powell-fitted hyper-parameters) or whose K is not symmetric;
// every such objective of one call is factored in the same launches (grid y = the objective).
//
// A (N padded to 16 with identity) is column-major in the workspace.  A 16-column STRIP's rows
// are held 1, 2 or 4 per thread of a 512-thread workgroup (16 doubles per row in registers; each
// step launch takes the fewest that hold its rows).  Launch k (one per 16-column step):
//   * panel (strip k): applies the pending step k-1 to its strip -- the step's row permutation
//     (<= 32 rows through LDS), U12 = inv(L11) A12 (four MFMAs; inv(L11) left by step k-1's panel)
//     and the rank-16 update of the rows below (MFMAs through an LDS transpose at 1-2 rows per
//     thread) -- then factors the strip (panel_columns, on 8 waves or on 4 after an LDS hand-off).
//     Per column ONE barrier: every wave publishes its pivot candidate (the u32 DPP maximum of
//     the |a| keys, the lowest row holding it by ballots, the row's 16 entries), the owner of row
//     j that row; after the barrier every wave picks the pivot among the wave candidates, swaps and
//     applies the rank-1 update to its rows, the next column's search issued ahead of the other
//     columns' FMAs.  Wave 0 then composes the step's 16 swaps into one permutation record (pos <-
//     src pairs) that every later consumer reads, while wave 1 inverts the new L11;
//   * update (strips > k): step k-1 applied to each strip by its own workgroup (lookahead: the
//     panel of step k needs only its own strip).
// The L columns keep the row order of their own step during the factorisation.  After the last
// step, lu_finalize_kernel applies the later interchanges to them (LAPACK's laswp on the left
// columns: P A = L U), composes the permutation (P e_c = e at row sinv[c]) and inverts each step's
// 16 x 16 diagonal blocks L11 and U11.  Solve (lu_solve_mfma_kernel, N <= 1024: one launch, one
// workgroup per 16-column strip of the identity and objective, no inter-workgroup dependency):
// W = P e_strip in MFMA accumulator layout; per step s its owner wave applies the inverted
// diagonal block (4 MFMAs) and publishes T = W_s, then every wave updates its live blocks,
// W_b -= A[b, s] T (4 MFMAs per block), forward with L then backward with U.  Above N = 1024
// (lu_solve_kernel): the round-4 solve on the unpermuted factors -- W = e_strip; per step s: the
// step's permutation record, W_s = L11^-1 W_s by substitution, W_below -= L21 W_s; then per step
// from the last: W_s = U_ss^-1 W_s, W_above -= U_above,s W_s.  W's rows are out[:, strip].
//
// Round 2 ran one Gauss-Jordan launch per pivot (N launches, ~105 ms at N = 2048); round 3's
// version of this file (one objective per launch sequence, the permutation rebuilt serially by
// one thread in every consumer, two barriers per pivot column) took 3.2 ms per objective at
// N = 512.

#include "bo_common.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

namespace {

constexpr int LB = 16;          // strip width
constexpr int LT = 512;         // threads per strip workgroup (256 VGPRs: the rows stay in registers)
constexpr int LRMAX = 4;        // rows per thread (kernels templated on LR = 1, 2, 4 by N_p): N_p <= 2048
constexpr int LW = LT / 64;     // waves per workgroup
constexpr int PREC = 72;        // ints per step's permutation record: [0] m, [8, 40) pos, [40, 72) src

// Diagnostic build (BO_BUILD_VARIANT=DEF_FIT_TIMING): the panel workgroup of each step launch
// and workgroup 0 of the solve stamp the 100 MHz real-time clock at their phase boundaries
// (word: step << 16 | slot << 4 | tag); bo_debug_lu_timing reads them back.
#define LB_DIAG 16
#ifdef BO_FIT_TIMING
__device__ long long bo_lu_tstamp[8192];
__device__ int bo_lu_tcount;
#define LU_STAMP(step, tag)                                                          \
  do {                                                                               \
    if (threadIdx.x == 0) {                                                          \
      const int _i = atomicAdd(&bo_lu_tcount, 1);                                    \
      if (_i < 4096) {                                                               \
        bo_lu_tstamp[2 * _i] = ((long long)(step) << 16) | ((long long)blockIdx.y << 4) | (tag); \
        bo_lu_tstamp[2 * _i + 1] = (long long)wall_clock64();                        \
      }                                                                              \
    }                                                                                \
  } while (0)
// per pivot column of the panel (slot 0, steps < 64; BO_LU_COLSTAMP builds only -- the stores
// are waited for at every barrier, which inflates the phases they time): plain stores of the
// clock, no atomics, and the shader clock beside it (their ratio is the core clock)
__device__ long long bo_lu_cstamp[64 * LB_DIAG * 4];
__device__ long long bo_lu_cclk[64 * LB_DIAG * 4];
#ifdef BO_LU_COLSTAMP
#define LU_CSTAMP(step, j, t)                                                        \
  do {                                                                               \
    if (threadIdx.x == 0 && blockIdx.y == 0 && (step) < 64) {                        \
      bo_lu_cstamp[((step) * LB_DIAG + (j)) * 4 + (t)] = (long long)wall_clock64();  \
      bo_lu_cclk[((step) * LB_DIAG + (j)) * 4 + (t)] = (long long)clock64();         \
    }                                                                                \
  } while (0)
#else
#define LU_CSTAMP(step, j, t) ((void)0)
#endif
#else
#define LU_STAMP(step, tag) ((void)0)
#define LU_CSTAMP(step, j, t) ((void)0)
#endif

struct LuGeo {
  int n, n_p, nbs;              // N, N padded to 16, strips
  long long Na;                 // leading dimension (= n_p)
  int small_panel;              // 0 never, 1 above N_p = 512, 2 always: the 4-wave panel (panel_small)
};

constexpr int SPW = 4;                  // waves of the small panel (one per SIMD)

struct LuBatch {                // one factorisation per slot (the objectives whose Cholesky failed)
  double* A[BO_MAX_OBJ];
  int* prec[BO_MAX_OBJ];        // nbs permutation records
  int* sinv[BO_MAX_OBJ];        // [n_p] P's column c is e at row sinv[c] (lu_finalize_kernel)
  double* tinv[BO_MAX_OBJ];     // [nbs][2][16][16] inverses of each step's L11 and U11, row-major
  const double* km[BO_MAX_OBJ];
  double* out[BO_MAX_OBJ];
  int* status;                  // [slot]: 1 = an exactly zero (or NaN) pivot
};

// ------------------------------------------------------------------------------ init
// A(i, j) = K[i][j] + jitter d_ij (i, j < N), identity padding: 32 x 32 tiles, coalesced both ways
__global__ __launch_bounds__(256) void lu_init_kernel(LuBatch bt, LuGeo g, long long ld, double jitter) {
  __shared__ double tile[32][33];
  const int ti = blockIdx.y, tj = blockIdx.x, tid = threadIdx.x;
  const double* __restrict__ km = bt.km[blockIdx.z];
  double* __restrict__ A = bt.A[blockIdx.z];
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
  double buf[32][LB];           // permuted rows in flight
  int pos[32], src[32];         // the step's row permutation: pos <- src
  int m;                        // its length
  double T[LB][LB + 1];         // the 16 x 16 block being solved
  double L11[LB][LB + 1];       // the step's diagonal block (L unit lower / U upper)
  alignas(16) double cand[2][LW][LB];   // panel: each wave's best row, by column parity
  unsigned long long ck[2][LW]; //        its pivot key (piv_key; 0: no candidate row)
  int cr[2][LW];                //        its row index
  double crp[2][LW];            //        1 / its entry in the column (the pivot's reciprocal)
  alignas(16) double grow[2][LB];       //        row j of the column
  int piv[LB];                  //        the step's pivot rows
  short smap[LT * LRMAX];          // row -> its slot as a source of the permutation (-1: none)
  short pmap[LT * LRMAX];          // row -> its slot as a destination
};

__device__ __forceinline__ void init_maps(StripLds& L) {
  for (int i = threadIdx.x; i < LT * LRMAX; i += LT) { L.smap[i] = -1; L.pmap[i] = -1; }
}

// row `base + t + LT r` of the strip is w[r][*] of thread t
__device__ __forceinline__ long long own_row(int base, int r) { return (long long)base + threadIdx.x + (long long)LT * r; }

// the permutation record's pairs into LDS (threads 0..31 hold them in registers, loaded earlier),
// and the row -> slot maps
__device__ __forceinline__ void put_perm(StripLds& L, int m, int pos, int src) {
  if (threadIdx.x < 32) { L.pos[threadIdx.x] = pos; L.src[threadIdx.x] = src; }
  if ((int)threadIdx.x < m) { L.smap[src] = (short)threadIdx.x; L.pmap[pos] = (short)threadIdx.x; }
  if (threadIdx.x == 0) L.m = m;
}

__device__ __forceinline__ void get_perm(const int* __restrict__ rec, int& m, int& pos, int& src) {
  const int t = threadIdx.x & 31;
  m = rec[0];
  pos = rec[8 + t];
  src = rec[40 + t];
}

// apply the permutation in LDS to the rows held in registers (rows >= base); the caller has
// synchronised after put_perm.  One map lookup per row (a scan over the <= 32 slots per row, with
// its dependent LDS reads, cost ~5 us per call).
template <int LR>
__device__ __forceinline__ void apply_perm(StripLds& L, double (&w)[LR][LB], int base, int n_p) {
  const int m = L.m;
  if (m == 0) return;                                 // uniform
#pragma unroll
  for (int r = 0; r < LR; ++r) {
    const long long row = own_row(base, r);
    const int u = row < n_p ? L.smap[row] : -1;
    if (u >= 0) {
#pragma unroll
      for (int c = 0; c < LB; ++c) L.buf[u][c] = w[r][c];
    }
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < LR; ++r) {
    const long long row = own_row(base, r);
    const int u = row < n_p ? L.pmap[row] : -1;
    if (u >= 0) {
#pragma unroll
      for (int c = 0; c < LB; ++c) w[r][c] = L.buf[u][c];
    }
  }
  __syncthreads();
  if ((int)threadIdx.x < m) { L.smap[L.src[threadIdx.x]] = -1; L.pmap[L.pos[threadIdx.x]] = -1; }
}

// Wave 0: the 16 swaps (rows 16 s + j <-> piv[j], in order) composed into pos <- src pairs over
// the <= 32 rows they move.  Data-parallel: lane j < 16 takes row 16 s + j, lane 16 + j row piv[j]
// (a row named twice keeps its first lane); each lane follows its row's DATA through the 16 swaps
// (compare-and-select, no ballots), so its data ends at position `v`: the pair is (pos = v,
// src = its row).  The moved rows' pairs are compacted by a ballot prefix.  (Round 4 simulated
// the swaps on slots with two ballots and readlanes per swap: ~2.7 us per step at N = 512.)
__device__ void build_perm(const StripLds& L, int s, int* __restrict__ rec) {
  const int lane = threadIdx.x & 63;
  const int pivl = L.piv[lane & (LB - 1)];             // lane j (and 16 + j) holds pivot j
  const int r0 = lane < LB ? LB * s + lane : (lane < 2 * LB ? pivl : -1);
  bool dup = false;
#pragma unroll
  for (int m = 0; m < 2 * LB; ++m) {
    const int rm = __builtin_amdgcn_readlane(r0, m);
    dup = dup || (m < lane && rm == r0);
  }
  int v = r0;
#pragma unroll
  for (int j = 0; j < LB; ++j) {
    const int a = LB * s + j, b = __builtin_amdgcn_readlane(pivl, j);
    v = v == a ? b : (v == b ? a : v);
  }
  const bool moved = lane < 2 * LB && !dup && v != r0;
  const unsigned long long mk = __ballot(moved);
  const int k = __popcll(mk & ((1ull << lane) - 1ull));
  if (moved) { rec[8 + k] = v; rec[40 + k] = r0; }
  if (lane == 0) rec[0] = __popcll(mk);
}

// L.T = L11^-1 L.T (unit lower), one column per lane 0..15, the chain in registers
__device__ __forceinline__ void trsm_lower(StripLds& L) {
  const int t = threadIdx.x;
  if (t < LB) {
    double x[LB];
#pragma unroll
    for (int i = 0; i < LB; ++i) x[i] = L.T[i][t];
#pragma unroll
    for (int i = 1; i < LB; ++i)
#pragma unroll
      for (int m2 = 0; m2 < i; ++m2) x[i] = __builtin_fma(-L.L11[i][m2], x[m2], x[i]);
#pragma unroll
    for (int i = 0; i < LB; ++i) L.T[i][t] = x[i];
  }
}

// L.T = U^-1 L.T (upper with its diagonal)
__device__ __forceinline__ void trsm_upper(StripLds& L) {
  const int t = threadIdx.x;
  if (t < LB) {
    double x[LB];
#pragma unroll
    for (int i = 0; i < LB; ++i) x[i] = L.T[i][t];
#pragma unroll
    for (int i = LB - 1; i >= 0; --i) {
#pragma unroll
      for (int m2 = i + 1; m2 < LB; ++m2) x[i] = __builtin_fma(-L.L11[i][m2], x[m2], x[i]);
      x[i] = x[i] / L.L11[i][i];
    }
#pragma unroll
    for (int i = 0; i < LB; ++i) L.T[i][t] = x[i];
  }
}

// w[r] -= sum_m2 A(b + m2 column, row_r) T[m2][*] on the rows with act[r]: a rolled loop over
// groups of 4 columns with the next group's column values in flight (the fully unrolled form,
// 1024 FMAs with their loads, was ~10 KB of code per copy run once per launch).  r16_start issues
// the first group's loads, early (before the barriers that precede the update).
template <int LR>
struct R16 {
  long long ra[LR];             // the row each lane loads (inactive rows: row b, never used)
  double lq[4][LR];
};

template <int LR>
__device__ __forceinline__ void r16_start(const double* __restrict__ A, long long Na, int b, int base,
                                          const bool (&act)[LR], R16<LR>& st) {
#pragma unroll
  for (int r = 0; r < LR; ++r) st.ra[r] = act[r] ? own_row(base, r) : b;
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int r = 0; r < LR; ++r) st.lq[q][r] = A[(long long)(b + q) * Na + st.ra[r]];
}

template <int LR>
__device__ __forceinline__ void r16_finish(const double* __restrict__ A, long long Na, int b, const StripLds& L,
                                           double (&w)[LR][LB], const bool (&act)[LR], R16<LR>& st) {
#pragma unroll 1
  for (int m0 = 0; m0 < LB; m0 += 4) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      double lc[LR];
#pragma unroll
      for (int r = 0; r < LR; ++r) lc[r] = st.lq[q][r];
      if (m0 + 4 < LB) {
#pragma unroll
        for (int r = 0; r < LR; ++r) st.lq[q][r] = A[(long long)(b + m0 + 4 + q) * Na + st.ra[r]];
      }
      double t[LB];
#pragma unroll
      for (int c = 0; c < LB; ++c) t[c] = L.T[m0 + q][c];
#pragma unroll
      for (int r = 0; r < LR; ++r)
        if (act[r]) {
#pragma unroll
          for (int c = 0; c < LB; ++c) w[r][c] = __builtin_fma(-lc[r], t[c], w[r][c]);
        }
    }
  }
}

// an f64 MFMA's result is read by plain VALU / LDS instructions only after its latency: wait states
__device__ __forceinline__ void acc_fence(d4& x) {
  asm volatile(BO_NOPS_F64_MFMA : "+v"(x));         // bo_common.h
}

// Step s applied to a strip whose rows [16 s, n_p) are in registers (base = 16 s): the
// permutation, U12 = L11^-1 A12 (rows 16 s .. 16 s + 15), A22 -= L21 U12.
// The rank-16 update's transpose: per wave 64 rows of 16 columns, rows padded to 17 doubles
constexpr int TPS = LB + 1;
template <int LR>
__device__ void strip_apply(const double* __restrict__ A, const LuGeo& g, const int* __restrict__ rec, int s,
                            const double* __restrict__ tinv_s, StripLds& L, double* __restrict__ tp,
                            double (&w)[LR][LB]) {
  const int base = LB * s, tid = threadIdx.x, lane = tid & 63, li = lane & 15, lg = lane >> 4;
  // every global load of the step issued first: the permutation record, inv(L11) (wave 0: the
  // MFMA A operand, row li and columns 4 ks + lg; written by the panel of step s), the first
  // columns of L21
  int pm = 0, pp = 0, ps = 0;
  if (tid < 32) get_perm(rec, pm, pp, ps);
  double tl[4] = {0.0, 0.0, 0.0, 0.0};
  if (tid < 64) {
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) tl[ks] = tinv_s[li * LB + 4 * ks + lg];
  }
  bool act[LR];
#pragma unroll
  for (int r = 0; r < LR; ++r) act[r] = own_row(base, r) >= base + LB && own_row(base, r) < g.n_p;
  // the rank-16 update's A operand (L21: rows of this wave's 16-row tiles, columns 4 ks + lg of the
  // step), row block r = 0 issued now; rows past n_p read row `base` (their result is dropped)
  const int wave = tid >> 6;
  auto l21_load = [&](int r, double (&am)[4][4]) {
#pragma unroll
    for (int rt = 0; rt < 4; ++rt) {
      const long long row = (long long)base + LT * r + 64 * wave + 16 * rt + li;
      const long long rr = row < g.n_p ? row : base;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) am[rt][ks] = A[(long long)(base + 4 * ks + lg) * g.Na + rr];
    }
  };
  // the matrix-core form at 1 and 2 rows per thread; 4 keep the 256-FMA form (two waves per SIMD
  // share the matrix pipe there: N = 2048 8.47 vs 8.60 ms, same box).  BO_BUILD_VARIANT=
  // DEF_LU_R16_MFMA4 builds the matrix-core form at 4 too (A/B only).
#ifdef BO_LU_R16_MFMA4
  constexpr bool mf = true;
#else
  constexpr bool mf = LR < 4;
#endif
  double am[4][4];
  R16<LR> st;
  if constexpr (mf) l21_load(0, am);
  else r16_start(A, g.Na, base, base, act, st);
  put_perm(L, pm, pp, ps);
  __syncthreads();
  if (blockIdx.x == 0) LU_STAMP(s + 1, 5);          // (diagnostic builds: the panel workgroup's phases)
  // the permutation (apply_perm without its map reset: every launch starts from init_maps), with
  // L11 (unit lower) and the 16 permuted top rows into LDS in the same phase: four barriers per
  // strip instead of six
  const int m = L.m;
  if (m != 0) {                                      // uniform
#pragma unroll
    for (int r = 0; r < LR; ++r) {
      const long long row = own_row(base, r);
      const int u = row < g.n_p ? L.smap[row] : -1;
      if (u >= 0) {
#pragma unroll
        for (int c = 0; c < LB; ++c) L.buf[u][c] = w[r][c];
      }
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < LR; ++r) {
      const long long row = own_row(base, r);
      const int u = row < g.n_p ? L.pmap[row] : -1;
      if (u >= 0) {
#pragma unroll
        for (int c = 0; c < LB; ++c) w[r][c] = L.buf[u][c];
      }
    }
  }
  if (tid < LB) {
#pragma unroll
    for (int c = 0; c < LB; ++c) L.T[tid][c] = w[0][c];
  }
  __syncthreads();
  if (blockIdx.x == 0) LU_STAMP(s + 1, 6);
  // U12 = inv(L11) A12: four MFMAs on wave 0 (B operand T[4 ks + lg][li]; the accumulator holds
  // U12[lg + 4 i][li]), in place of the 16-lane substitution chain (~1.7 us per step)
  if (tid < 64) {
    double tb[4];
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) tb[ks] = L.T[4 * ks + lg][li];
    d4 u = (d4){0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) u = __builtin_amdgcn_mfma_f64_16x16x4f64(tl[ks], tb[ks], u, 0, 0, 0);
    acc_fence(u);
#pragma unroll
    for (int i = 0; i < 4; ++i) L.T[lg + 4 * i][li] = u[i];
  }
  __syncthreads();
  if (blockIdx.x == 0) LU_STAMP(s + 1, 7);
  if (tid < LB) {
#pragma unroll
    for (int c = 0; c < LB; ++c) w[0][c] = L.T[tid][c];
  }
  // A22 -= L21 U12 on the matrix cores: per wave and row block, four 16-row tiles x four k-steps
  // (B operand U12[4 ks + lg][li], shared by the tiles), the product transposed to rows through
  // the wave's LDS block; the round-4 form was 256 FMAs per row against 256 LDS broadcasts
  if constexpr (!mf) {
    r16_finish(A, g.Na, base, L, w, act, st);
    return;
  }
  double tb[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) tb[ks] = L.T[4 * ks + lg][li];
  double* __restrict__ pw = tp + (size_t)wave * 64 * TPS;
#pragma unroll
  for (int r = 0; r < LR; ++r) {
    d4 acc[4];
#pragma unroll
    for (int rt = 0; rt < 4; ++rt) {
      acc[rt] = (d4){0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) acc[rt] = __builtin_amdgcn_mfma_f64_16x16x4f64(am[rt][ks], tb[ks], acc[rt], 0, 0, 0);
    }
    if (r + 1 < LR) l21_load(r + 1, am);
#pragma unroll
    for (int rt = 0; rt < 4; ++rt) acc_fence(acc[rt]);
#pragma unroll
    for (int rt = 0; rt < 4; ++rt)
#pragma unroll
      for (int i = 0; i < 4; ++i) pw[(16 * rt + lg + 4 * i) * TPS + li] = acc[rt][i];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (act[r]) {
#pragma unroll
      for (int c = 0; c < LB; ++c) w[r][c] -= pw[lane * TPS + c];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");       // the block is rewritten next
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  // (no barrier: nothing later in the launch writes L.T, L.L11 or L.buf -- the panel uses its own
  // fields, the small panel's hand-off its own array)
}

// ------------------------------------------------------------- the pivot columns of a panel
// Pivot search key of an entry: 0 for a row outside the column (or NaN: idamax skips it), else
// the bits of |a| + 1 (monotone in |a| for non-negative doubles; 1 for an exact zero).  Ties go to
// the lower row.
__device__ __forceinline__ unsigned long long piv_key(double a, bool in) {
  const double f = fabs(a);
  return (in && f == f) ? (unsigned long long)__double_as_longlong(f) + 1ull : 0ull;
}
template <int CTRL, int RM = 0xF>
__device__ __forceinline__ unsigned int dpp_max_u32(unsigned int x) {
  // lanes off the row mask read 0, max's identity: the move folds into v_max_u32_dpp
  return max(x, (unsigned int)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, RM, 0xF, false));
}
// the wave's largest u32, uniform: each 16-lane row by quad_perm, half-mirror and mirror, then
// row_bcast:15 (rows 1, 3) and row_bcast:31 (rows 2, 3) carry the row maxima to lane 63
__device__ __forceinline__ unsigned int wave_max_u32(unsigned int x) {
  x = dpp_max_u32<0xB1>(x);
  x = dpp_max_u32<0x4E>(x);
  x = dpp_max_u32<0x141>(x);
  x = dpp_max_u32<0x140>(x);
  x = dpp_max_u32<0x142, 0xA>(x);
  x = dpp_max_u32<0x143, 0xC>(x);
  return (unsigned int)__builtin_amdgcn_readlane((int)x, 63);
}
// the wave's largest 64-bit key: the high words, then the low words of the lanes holding that high
// word (u32 DPP maxima: a 64-bit compare-and-select per step chained VCC through every step)
__device__ __forceinline__ unsigned long long wave_max_key(unsigned long long k) {
  const unsigned int h = wave_max_u32((unsigned int)(k >> 32));
  const unsigned int l = wave_max_u32((unsigned int)(k >> 32) == h ? (unsigned int)k : 0u);
  return ((unsigned long long)h << 32) | l;
}
// the same over each aligned group of NW = 1, 2, 4 or 8 lanes, held by every lane of the group
template <int NW>
__device__ __forceinline__ unsigned int group_max_u32(unsigned int x) {
  if (NW >= 2) x = dpp_max_u32<0xB1>(x);
  if (NW >= 4) x = dpp_max_u32<0x4E>(x);
  if (NW >= 8) x = dpp_max_u32<0x141>(x);
  return x;
}
template <int NW>
__device__ __forceinline__ unsigned long long group_max_key(unsigned long long k) {
  const unsigned int h = group_max_u32<NW>((unsigned int)(k >> 32));
  const unsigned int l = group_max_u32<NW>((unsigned int)(k >> 32) == h ? (unsigned int)k : 0u);
  return ((unsigned long long)h << 32) | l;
}
template <int NW>
__device__ __forceinline__ int group_min_i(int x) {
  if (NW >= 2) x = min(x, __builtin_amdgcn_update_dpp(x, x, 0xB1, 0xF, 0xF, false));
  if (NW >= 4) x = min(x, __builtin_amdgcn_update_dpp(x, x, 0x4E, 0xF, 0xF, false));
  if (NW >= 8) x = min(x, __builtin_amdgcn_update_dpp(x, x, 0x141, 0xF, 0xF, false));
  return x;
}

// getf2 on the 16 columns of strip k, rows top .. n_p - 1, held by NW waves in registers: v[r][*]
// of lane l of wave w is row row0 + rstride r + l (row0 per wave).  The loop is rolled and the rows
// rotate (an unrolled loop's code is fetched cold on every launch: instruction fetch, not
// arithmetic, set the time): at column j, v[r][0] is column j, v[r][c] column j + c for c < 16 - j,
// and v[r][16 - j + i] the finished column i; sixteen rotations restore the natural order.
// Per column:
//   * each wave's pivot candidate: the key of |a| (piv_key: 0 for rows above g0 = top + j, past n_p,
//     or NaN, which idamax skips), the wave maximum by u32 DPP maxima, and the wave's lowest row
//     holding it by one ballot per register (the rows of a register rise with the lane, registers
//     with r);
//   * the wave publishes (key, row, the row's 16 entries, 1 / its entry) into a buffer
//     alternating by column parity, the owner of row g0 its row; ONE barrier;
//   * the NW candidates reduced by an NW-lane butterfly (maximum, then the lowest row among the
//     waves holding it: getrf's first largest |a|), the pivot row read, the swap, the scaling by the
//     reciprocal and the rank-1 update -- branch-free, the finished columns masked out of the pivot
//     row (they hold L, not live entries).
// Pivot choice, reciprocal and FMAs are those of LAPACK's getf2 (and of the round-4 loop: bit-
// identical factors, up to the sign of an exact zero in a finished column).  Returns true if a
// column had no nonzero candidate (no swap and no scaling there; the slot reports it singular).
// ABL (scripts/ubench/lu_panel_ubench.hip only; 0 in the library): parts of the column step left
// out, to time the rest -- 1 the barrier, 2 the wave reduction, 4 the cross-wave reduction, 8 the
// update, 16 the swap, 32 the reciprocal, 64 the finished columns' mask; 128: the update without
// the row branch (the multiplier zeroed on inactive rows).
// A wave's pivot candidate for the column held in v[r][CI] (rows >= gmin and < n_p): the maximum
// key, the first register and lane holding it, and the reciprocal of the lane's first largest
// entry (computed before the reduction so that its latency overlaps it).
struct ColSearch {
  unsigned long long gk;
  int wr, wl;
  double brp;
};
template <int RPL, int CI, int ABL>
__device__ __forceinline__ void col_search(const double (&v)[RPL][LB], const long long (&row)[RPL], long long gmin,
                                           int n_p, ColSearch& s) {
  unsigned long long key[RPL], mk = 0ull;
  double bv = 1.0;
#pragma unroll
  for (int r = 0; r < RPL; ++r) {
    key[r] = piv_key(v[r][CI], row[r] >= gmin && row[r] < n_p);
    if (key[r] > mk) { mk = key[r]; bv = v[r][CI]; }              // the lane's first largest
  }
  double brp = (ABL & 32) ? bv : 1.0 / bv;                        // in flight under the reduction
  asm volatile("" : "+v"(brp));                                   // (not sunk into the publish)
  s.brp = brp;
  s.gk = (ABL & 2) ? bo_readlane_u(mk, 0) : wave_max_key(mk);
  unsigned long long wm = 0ull;
  int wr = 0;
#pragma unroll
  for (int r = RPL - 1; r >= 0; --r) {
    const unsigned long long m = __ballot(key[r] == s.gk);
    if (m) { wm = m; wr = r; }
  }
  s.wr = wr;
  s.wl = (int)__builtin_ctzll(wm | (1ull << 63));
}

// PIPE (the default for <= 2 rows per lane; ABL 256 forces it, 512 turns it off): the next
// column's search issued right after that column's update, ahead of the other columns' FMAs
// (branch-free update: the multiplier is 0 on inactive rows), so that its DPP chain overlaps them
// -- per column 3,207 -> 2,912 clocks at 4 waves x 2 rows, 3,073 -> 2,964 at 8 x 1; at 4 rows per
// lane the branch-free form spills (18,208 clocks) and the row branch stays.
template <int NW, int RPL, int ABL = 0>
__device__ bool panel_columns(StripLds& L, double (&v)[RPL][LB], long long row0, int rstride, int top, int n_p,
                              int k) {
  constexpr bool PIPE = (ABL & 256) != 0 || (RPL <= 2 && (ABL & 512) == 0);
  const int lane = threadIdx.x & 63, wv = (threadIdx.x >> 6) & (NW - 1);
  long long row[RPL];
#pragma unroll
  for (int r = 0; r < RPL; ++r) row[r] = row0 + (long long)rstride * r + lane;
  bool singular = false;
  (void)k;
  ColSearch cs;
  if constexpr (PIPE) col_search<RPL, 0, ABL>(v, row, top, n_p, cs);
#pragma unroll 1
  for (int j = 0; j < LB; ++j) {
    const int bf = j & 1;
    const long long g0 = (long long)top + j;
    LU_CSTAMP(k, j, 0);
    if constexpr (!PIPE) col_search<RPL, 0, ABL>(v, row, g0, n_p, cs);
    const unsigned long long gk = cs.gk;
    const int wr = cs.wr, wl = cs.wl;
    const double brp = cs.brp;
    const bool has = gk != 0ull;
    LU_CSTAMP(k, j, 1);
#pragma unroll
    for (int r = 0; r < RPL; ++r)
      if (has && r == wr && lane == wl) {
#pragma unroll
        for (int c = 0; c < LB; c += 2) *(d2*)&L.cand[bf][wv][c] = (d2){v[r][c], v[r][c + 1]};
        L.crp[bf][wv] = brp;
      }
    if (lane == 0) {
      L.ck[bf][wv] = gk;
      L.cr[bf][wv] = has ? (int)(row0 + (long long)rstride * wr + wl) : 0x7fffffff;
    }
#pragma unroll
    for (int r = 0; r < RPL; ++r)
      if (row[r] == g0) {
#pragma unroll
        for (int c = 0; c < LB; c += 2) *(d2*)&L.grow[bf][c] = (d2){v[r][c], v[r][c + 1]};
      }
    if (!(ABL & 1)) __syncthreads();
    LU_CSTAMP(k, j, 2);
    const int u = lane & (NW - 1);
    const unsigned long long cku = L.ck[bf][u];
    const int cru = L.cr[bf][u];
    const unsigned long long G = (ABL & 4) ? cku : group_max_key<NW>(cku);
    const int pmin = (ABL & 4) ? cru : group_min_i<NW>(cku == G ? cru : 0x7fffffff);
    const unsigned long long pwm = __ballot(lane < NW && cru == pmin);
    const unsigned long long Gu = bo_readlane_u(G, 0);
    const bool zero = Gu <= 1ull;                                // all zero, or no candidate
    const int p = zero ? (int)g0 : __builtin_amdgcn_readlane(pmin, 0);
    const int pw = zero ? -1 : (int)__builtin_ctzll(pwm | (1ull << 63));
    singular = singular || zero;
    if (threadIdx.x == 0) L.piv[j] = p;
    const double* prow = pw >= 0 ? L.cand[bf][pw] : L.grow[bf];
    double pr[LB];
#pragma unroll
    for (int c = 0; c < LB; c += 2) {
      const d2 x = *(const d2*)(prow + c);
      pr[c] = x.x;
      pr[c + 1] = x.y;
    }
    const double rp = pw >= 0 ? L.crp[bf][pw] : 0.0;
#pragma unroll
    for (int r = 0; r < RPL; ++r) {
      if (ABL & 16) {
      } else if (row[r] == g0) {
#pragma unroll
        for (int c = 0; c < LB; ++c) v[r][c] = pr[c];
      } else if (row[r] == p) {
#pragma unroll
        for (int c = 0; c < LB; c += 2) {
          const d2 x = *(const d2*)&L.grow[bf][c];
          v[r][c] = x.x;
          v[r][c + 1] = x.y;
        }
      }
    }
    const int live = LB - j;                                     // rotated columns 1 .. live - 1
#pragma unroll
    for (int c = 1; c < LB; ++c) {                               // (after the swap: in place)
      // a bitwise AND with a uniform mask (~0 iff c < live): per-column selects on VCC serialised
      // their SALU -> VALU hand-offs (~700 clocks per column)
      const unsigned int m = (ABL & 64) ? ~0u : (unsigned int)((c - live) >> 31);
      const unsigned long long b = (unsigned long long)__double_as_longlong(pr[c]);
      pr[c] = __longlong_as_double((long long)(b & (((unsigned long long)m << 32) | m)));
    }
    if constexpr (PIPE) {
      double l[RPL];
#pragma unroll
      for (int r = 0; r < RPL; ++r) {
        const bool act = row[r] > g0 && row[r] < n_p;
        l[r] = act ? v[r][0] * rp : 0.0;
        v[r][0] = act ? l[r] : v[r][0];
        v[r][1] = __builtin_fma(-l[r], pr[1], v[r][1]);
      }
      col_search<RPL, 1, ABL>(v, row, g0 + 1, n_p, cs);           // (at j = 15: unused)
#pragma unroll
      for (int r = 0; r < RPL; ++r)
#pragma unroll
        for (int c = 2; c < LB; ++c) v[r][c] = __builtin_fma(-l[r], pr[c], v[r][c]);
    } else if constexpr ((ABL & 128) != 0) {
#pragma unroll
      for (int r = 0; r < RPL; ++r) {
        const bool act = row[r] > g0 && row[r] < n_p;
        const double l = act ? v[r][0] * rp : 0.0;
        v[r][0] = act ? l : v[r][0];
#pragma unroll
        for (int c = 1; c < LB; ++c) v[r][c] = __builtin_fma(-l, pr[c], v[r][c]);
      }
    } else {
#pragma unroll
      for (int r = 0; r < RPL; ++r)
        if (!(ABL & 8) && row[r] > g0 && row[r] < n_p) {
          const double l = v[r][0] * rp;
          v[r][0] = l;
#pragma unroll
          for (int c = 1; c < LB; ++c) v[r][c] = __builtin_fma(-l, pr[c], v[r][c]);
        }
    }
#pragma unroll
    for (int r = 0; r < RPL; ++r) {
      const double t = v[r][0];                                  // rotate: column j goes last
#pragma unroll
      for (int c = 0; c + 1 < LB; ++c) v[r][c] = v[r][c + 1];
      v[r][LB - 1] = t;
    }
    LU_CSTAMP(k, j, 3);
  }
  return singular;
}

// inv(L11) of the step just factored, for the next launch's strip apply (U12 = inv(L11) A12 on the
// matrix cores instead of a 16-lane substitution): the panel's diagonal rows were staged in L.L11;
// wave 1 (lanes 0..15, one column each) substitutes on the identity -- the operations of
// diag_block_inverses, so the finalize kernel later writes the same values -- while wave 0 builds
// the permutation record.
__device__ __forceinline__ void l11_inverse_to(const StripLds& L, double* __restrict__ tinv_k) {
  const int lane = threadIdx.x & 63;
  if ((threadIdx.x >> 6) != 1 || lane >= LB) return;
  const int t = lane;
  double x[LB];
#pragma unroll
  for (int i = 0; i < LB; ++i) x[i] = i == t ? 1.0 : 0.0;
#pragma unroll
  for (int i = 1; i < LB; ++i)
#pragma unroll
    for (int m = 0; m < i; ++m) x[i] = __builtin_fma(-L.L11[i][m], x[m], x[i]);
#pragma unroll
  for (int i = 0; i < LB; ++i) tinv_k[i * LB + t] = x[i];
}

// The panel of strip k when its rows to factor (16 k .. n_p) number at most 256 RPL: they move
// through LDS (P, column-major, PR rows) from the workgroup's 8 waves to SPW = 4 waves, one per SIMD,
// RPL rows per lane in registers (row offset o = 64 RPL wave + 64 r + lane); the other waves end.
// The column loop is issue-bound (each wave runs the whole pivot selection; measured ~4200 clocks
// per column with two waves per SIMD), so one wave per SIMD with more rows each is the faster
// shape.  The rows of step k-1's U block (base .. 16 k) are stored by their threads before the
// hand-off.
template <int NW, int RPL, int PR>
__device__ void panel_small(LuBatch& bt, const LuGeo& g, int k, StripLds& L, const double* __restrict__ P,
                            long long c0, double* __restrict__ A, int* __restrict__ prec, int slot) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int top = LB * k, R = g.n_p - top;
  double v[RPL][LB];
  int off[RPL];
#pragma unroll
  for (int r = 0; r < RPL; ++r) {
    off[r] = wave * 64 * RPL + 64 * r + lane;
#pragma unroll
    for (int c = 0; c < LB; ++c) v[r][c] = off[r] < R ? P[c * PR + off[r]] : 0.0;
  }
  const bool singular = panel_columns<NW, RPL>(L, v, (long long)top + wave * 64 * RPL, 64, top, g.n_p, k);
  if (tid == 0 && singular) bt.status[slot] = 1;
  LU_STAMP(k, 3);
  // the factored rows first (the stores drain while wave 0 builds the permutation record and wave
  // 1 inverts L11); the diagonal rows (offsets 0..15: wave 0, r = 0) staged for wave 1
#pragma unroll
  for (int r = 0; r < RPL; ++r)
    if (off[r] < R) {
#pragma unroll
      for (int c = 0; c < LB; ++c) A[(c0 + c) * g.Na + top + off[r]] = v[r][c];
    }
  if (wave == 0 && lane < LB) {
#pragma unroll
    for (int c = 0; c < LB; ++c) L.L11[lane][c] = v[0][c];
  }
  __syncthreads();                                   // L.piv and the staged rows
  if (wave == 0) build_perm(L, k, prec + (long long)k * PREC);
  l11_inverse_to(L, bt.tinv[slot] + (long long)k * 512);
  LU_STAMP(k, 4);
}

// Launch k: block 0 = panel (strip k), blocks 1.. = strips k + 1 .. (update of step k-1);
// grid y = the batch slot.
template <int LR>
__global__ __launch_bounds__(LT) void lu_step_kernel(LuBatch bt, LuGeo g, int k) {
  __shared__ StripLds L;
  const int tid = threadIdx.x, wave = tid >> 6;
  const int slot = blockIdx.y;
  double* __restrict__ A = bt.A[slot];
  int* __restrict__ prec = bt.prec[slot];
  const int strip = k + (int)blockIdx.x;
  const int base = k > 0 ? LB * (k - 1) : 0;
  const long long c0 = (long long)LB * strip;
  const bool stamp = blockIdx.x == 0;
  (void)stamp;
  if (stamp) LU_STAMP(k, 1);
  init_maps(L);
  __syncthreads();
  double w[LR][LB];
#pragma unroll
  for (int r = 0; r < LR; ++r) {
    const long long row = own_row(base, r);
    const long long rc = row < g.n_p ? row : g.n_p - 1;          // clamped: every load unconditional
#pragma unroll
    for (int c = 0; c < LB; ++c) w[r][c] = A[(c0 + c) * g.Na + rc];
#pragma unroll
    for (int c = 0; c < LB; ++c) w[r][c] = row < g.n_p ? w[r][c] : 0.0;
  }
  __shared__ double TP[LW * 64 * TPS];          // the strip apply's transpose (68 KB)
  if (k > 0)
    strip_apply(A, g, prec + (long long)(k - 1) * PREC, k - 1, bt.tinv[slot] + (long long)(k - 1) * 512, L, TP, w);
  if (stamp) LU_STAMP(k, 2);
  // the panel on 4 waves (1 or 2 rows per lane) once its rows fit 512 (LR <= 2) or 256: the
  // workgroup's rows >= 16 k go through LDS (P, column-major, PR rows), the rows of step k-1's U
  // block (base .. 16 k) are stored by their threads, waves 4..7 end; the earlier steps of N > 512
  // run the panel on all 8 waves, LR rows per lane
  {
    constexpr int PR = 512;                    // the hand-off's rows (64 KB)
    __shared__ double P[LB * PR];
    const int top = LB * k, R = g.n_p - top;
    // (at N_p <= 512, LR = 1, the hand-off costs more than it saves: 1.18 vs 1.14 ms per inverse,
    // same box; at N = 1024 / 2048 the small panel wins, 2.75 vs 2.86 / 9.39 vs 9.66 ms)
    const bool small = LR <= 2 && (g.small_panel == 2 || (g.small_panel == 1 && LR == 2) ||
                                   (g.small_panel == 3 && R <= 256));
    if (blockIdx.x == 0 && small && R <= 512) {   // workgroup-uniform
#pragma unroll
      for (int r = 0; r < LR; ++r) {
        const long long row = own_row(base, r);
        if (row >= top && row < g.n_p) {
#pragma unroll
          for (int c = 0; c < LB; ++c) P[c * PR + (row - top)] = w[r][c];
        } else if (row < top) {
#pragma unroll
          for (int c = 0; c < LB; ++c) A[(c0 + c) * g.Na + row] = w[r][c];
        }
      }
      __syncthreads();
      if (wave >= SPW) return;                 // s_barrier then counts the SPW waves left
      // (4 rows per lane, for 1024 rows, would spill: the rows, the pivot row and the swap's
      // loads need ~100 + 45 RPL VGPRs)
      if (R <= 256) panel_small<SPW, 1, PR>(bt, g, k, L, P, c0, A, prec, slot);
      else if constexpr (LR <= 2) panel_small<SPW, 2, PR>(bt, g, k, L, P, c0, A, prec, slot);
      return;
    }
  }
  if (blockIdx.x == 0) {
    // factor strip k on the workgroup's 8 waves (row own_row(base, r) = base + 64 wave + lane + LT r)
    const bool singular = panel_columns<LW, LR>(L, w, (long long)base + 64 * wave, LT, LB * k, g.n_p, k);
    if (tid == 0 && singular) bt.status[slot] = 1;
    LU_STAMP(k, 3);
#pragma unroll
    for (int r = 0; r < LR; ++r) {                    // the factored rows first (they drain while
      const long long row = own_row(base, r);         // wave 0 builds the permutation record)
      if (row >= g.n_p) continue;
#pragma unroll
      for (int c = 0; c < LB; ++c) A[(c0 + c) * g.Na + row] = w[r][c];
    }
    {                                                 // the diagonal rows (row 16 k + i: thread
      const int t0 = LB * k - base;                   // t0 + i, r = 0) staged for wave 1
      if (tid >= t0 && tid < t0 + LB) {
#pragma unroll
        for (int c = 0; c < LB; ++c) L.L11[tid - t0][c] = w[0][c];
      }
    }
    __syncthreads();                                  // L.piv and the staged rows
    if (wave == 0) build_perm(L, k, prec + (long long)k * PREC);
    l11_inverse_to(L, bt.tinv[slot] + (long long)k * 512);
    LU_STAMP(k, 4);
    return;
  }
#pragma unroll
  for (int r = 0; r < LR; ++r) {
    const long long row = own_row(base, r);
    if (row >= g.n_p) continue;
#pragma unroll
    for (int c = 0; c < LB; ++c) A[(c0 + c) * g.Na + row] = w[r][c];
  }
}

// ----------------------------------------------------------------------- finalize (laswp)
// After the last step: getrf's form P A = L U.  Workgroup s < nbs applies the row interchanges of
// the steps after s to strip s's L columns (LAPACK's laswp on the left columns): wave 0 composes
// the records s+1 .. nbs-1 into the gather map g (position i <- stored row g(i)) in LDS, then the
// strip's rows below its diagonal block are gathered in place (every load of the workgroup before
// any store; the workgroups own disjoint columns).  Workgroup nbs composes every record into
// sigma (position i <- original row sigma(i)) and stores sinv = sigma^-1 (column c of P is e at
// row sinv(c)) and the reciprocals of U's diagonal for the solve.
__device__ void compose_records(int* __restrict__ gmap, const int* __restrict__ prec, int t0, int t1, int n_p) {
  const int lane = threadIdx.x & 63;
  for (int i = lane; i < n_p; i += 64) gmap[i] = i;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  int m = 0, pos = 0, src = 0;
  if (t0 < t1 && lane < 32) get_perm(prec + (long long)t0 * PREC, m, pos, src);
  for (int t = t0; t < t1; ++t) {
    const int cm = m, cp = pos, cs = src;
    if (t + 1 < t1 && lane < 32) get_perm(prec + (long long)(t + 1) * PREC, m, pos, src);   // next, in flight
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int v = lane < cm ? gmap[cs] : 0;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    if (lane < cm) gmap[cp] = v;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Inverses of strip s's diagonal blocks (final after step s; later interchanges never reach rows
// < 16 (s + 1)) by substitution on the identity, one column per lane: wave 1 the unit lower L11,
// wave 2 the upper U11.  The solve then applies each step's triangle as four MFMAs.  (Inverted
// diagonal blocks are rocBLAS trsm's method; against substitution they moved the residual
// |A X - I| by 1.0-1.8x in a numpy model at cond 1e4..2e19, scripts/lu_invdiag_model.py.)
__device__ void diag_block_inverses(const double* __restrict__ A, long long Na, int s, double* __restrict__ tinv) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if ((wave != 1 && wave != 2) || lane >= LB) return;
  const long long cs = (long long)LB * s;
  const int t = lane;
  double x[LB];
  if (wave == 1) {                                     // L11^-1 (unit lower)
#pragma unroll
    for (int i = 0; i < LB; ++i) x[i] = i == t ? 1.0 : 0.0;
#pragma unroll
    for (int i = 1; i < LB; ++i)
#pragma unroll
      for (int m = 0; m < i; ++m) x[i] = __builtin_fma(-A[(cs + m) * Na + cs + i], x[m], x[i]);
#pragma unroll
    for (int i = 0; i < LB; ++i) tinv[(long long)s * 512 + i * LB + t] = x[i];
  } else {                                             // U11^-1 (upper, with its diagonal)
#pragma unroll
    for (int i = 0; i < LB; ++i) x[i] = i == t ? 1.0 : 0.0;
#pragma unroll
    for (int i = LB - 1; i >= 0; --i) {
#pragma unroll
      for (int m = i + 1; m < LB; ++m) x[i] = __builtin_fma(-A[(cs + m) * Na + cs + i], x[m], x[i]);
      x[i] = x[i] / A[(cs + i) * Na + cs + i];
    }
#pragma unroll
    for (int i = 0; i < LB; ++i) tinv[(long long)s * 512 + 256 + i * LB + t] = x[i];
  }
}

template <int LR>
__global__ __launch_bounds__(LT) void lu_finalize_kernel(LuBatch bt, LuGeo g) {
  __shared__ int gmap[LT * LRMAX];
  const int s = blockIdx.x, slot = blockIdx.y, tid = threadIdx.x;
  double* __restrict__ A = bt.A[slot];
  const int* __restrict__ prec = bt.prec[slot];
  if (s == g.nbs) {
    if (tid < 64) compose_records(gmap, prec, 0, g.nbs, g.n_p);
    __syncthreads();
    for (int i = tid; i < g.n_p; i += LT) bt.sinv[slot][gmap[i]] = i;
    return;
  }
  diag_block_inverses(A, g.Na, s, bt.tinv[slot]);
  if (s + 1 >= g.nbs) return;                          // the last strip: no later interchanges
  if (tid < 64) compose_records(gmap, prec, s + 1, g.nbs, g.n_p);
  __syncthreads();
  const long long c0 = (long long)LB * s;
  const int base = LB * (s + 1);
  double w[LR][LB];
#pragma unroll
  for (int r = 0; r < LR; ++r) {
    const long long row = own_row(base, r);
    const long long src = row < g.n_p ? gmap[row] : base;
#pragma unroll
    for (int c = 0; c < LB; ++c) w[r][c] = A[(c0 + c) * g.Na + src];
  }
  __syncthreads();                                     // every gather load before any store
#pragma unroll
  for (int r = 0; r < LR; ++r) {
    const long long row = own_row(base, r);
    if (row >= g.n_p || gmap[row] == row) continue;
#pragma unroll
    for (int c = 0; c < LB; ++c) A[(c0 + c) * g.Na + row] = w[r][c];
  }
}

// ------------------------------------------------------------------------------ solve
// getrs with the identity on the matrix cores: out[:, 16 strip + c] = U^-1 L^-1 P e_{16 strip + c}
// (P e_col = e at row sinv(col)).  One 512-thread workgroup per strip of the identity (grid x) and
// slot (grid y), no inter-workgroup dependency.  W (n_p x 16) lives in v_mfma_f64_16x16x4_f64
// accumulator layout: 16-row block b is wave b % 8's accumulator b / 8, lane (li, lg) holding
// W[16 b + lg + 4 i][li].  Per step s the block's owner wave solves the 16 x 16 triangle (16 lanes,
// one column each, the chain in registers; L11 / U_ss staged in LDS), publishes T = W_s in LDS, and
// after one barrier every wave applies the rank-16 update to its live blocks: W_b -= A[b rows, s
// columns] T, four MFMAs per block with the A operand read straight from the column-major factors
// (16 consecutive rows per column: coalesced).  Forward from the first block holding a non-zero of
// P e (the blocks above it stay zero), backward over every block.  The previous version held one
// row per thread and read T as LDS broadcasts (256 per row per step: ~1.7 us of LDS per step at
// N = 512) with the step's permutation applied through LDS (three barriers per step).

// One direction of the solve.  Step s: its owner wave (s & 7) applies the step's triangle to its
// block, T = tinv_s W_s (four MFMAs: the f64 accumulator layout -- lane (li, lg) holds rows
// lg + 4 i of column li -- is exactly the B-operand layout of the four k-steps), and publishes T
// in LDS; after one barrier every wave subtracts A[rows of its live blocks, columns of s] T.  The
// triangle's A operand (row li, columns 4 ks + lg of the inverse) is prefetched one owned step
// ahead, the update's before the barrier.
template <bool FWD, int NBW>
__device__ __forceinline__ void solve_phase(double (&Ts)[2][LB][LB + 1], d4 (&acc)[NBW], const double* __restrict__ A,
                                            const double* __restrict__ tinv, long long Na, int nbs, int first,
                                            int& par) {
  constexpr int PF = NBW <= 4 ? NBW : 2;     // blocks whose A operand is prefetched a step ahead
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, li = lane & 15, lg = lane >> 4;
  // the update's A operand for step st (rows of this wave's live blocks, columns of st): issued one
  // step ahead, so that its L2 latency overlaps the previous step
  auto av_load = [&](int st, double (&v)[PF][4]) {
    const long long cst = (long long)LB * st;
#pragma unroll
    for (int q = 0; q < PF; ++q) {
      const int b = 8 * q + wave;
      const bool live = b < nbs && (FWD ? b > st : b < st);
#pragma unroll
      for (int ks = 0; ks < 4; ++ks)
        v[q][ks] = live ? -A[(cst + 4 * ks + lg) * Na + (long long)LB * b + li] : 0.0;
    }
  };
  auto tri_load = [&](int st, double (&v)[4]) {
    const double* ti = tinv + (long long)st * 512 + (FWD ? 0 : 256) + li * LB + lg;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) v[ks] = ti[4 * ks];
  };
  const int s_beg = FWD ? first : nbs - 1;
  int my = FWD ? s_beg + ((wave - s_beg) & 7) : s_beg - ((s_beg - wave) & 7);
  double tri[4] = {0.0, 0.0, 0.0, 0.0};
  if (FWD ? my < nbs : my >= 0) tri_load(my, tri);
  double avn[PF][4];
  av_load(s_beg, avn);
  // steps in groups of 8: step s = 8 gq + w8 is wave w8's block gq, so the owner's accumulator
  // index is static (a runtime index put acc in scratch)
#pragma unroll
  for (int gi = 0; gi < NBW; ++gi) {
    const int gq = FWD ? gi : NBW - 1 - gi;
#pragma unroll 1
    for (int u = 0; u < 8; ++u) {
      const int w8 = FWD ? u : 7 - u;
      const int s = 8 * gq + w8;
      if (s >= nbs || (FWD && s < first)) continue;            // uniform
      const long long cs = (long long)LB * s;
      double av[PF][4];
#pragma unroll
      for (int q = 0; q < PF; ++q)
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) av[q][ks] = avn[q][ks];
      const int sn = FWD ? s + 1 : s - 1;
      if (FWD ? sn < nbs : sn >= 0) av_load(sn, avn);
      if (wave == w8) {
        acc_fence(acc[gq]);
        d4 tq = (d4){0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) tq = __builtin_amdgcn_mfma_f64_16x16x4f64(tri[ks], acc[gq][ks], tq, 0, 0, 0);
        acc_fence(tq);
        acc[gq] = tq;
#pragma unroll
        for (int i = 0; i < 4; ++i) Ts[par][lg + 4 * i][li] = tq[i];
        my = FWD ? s + 8 : s - 8;
        if (FWD ? my < nbs : my >= 0) tri_load(my, tri);
      }
      __syncthreads();
      double tb[4];
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) tb[ks] = Ts[par][4 * ks + lg][li];
#pragma unroll
      for (int q = 0; q < NBW; ++q) {
        const int b = 8 * q + wave;
        if (b >= nbs || (FWD ? b <= s : b >= s)) continue;      // wave-uniform
        double a2[4];
#pragma unroll
        for (int ks = 0; ks < 4; ++ks)
          a2[ks] = q < PF ? av[q < PF ? q : 0][ks] : -A[(cs + 4 * ks + lg) * Na + (long long)LB * b + li];
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) acc[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(a2[ks], tb[ks], acc[q], 0, 0, 0);
      }
      par ^= 1;
    }
  }
}

template <int NBW>
__global__ __launch_bounds__(LT) void lu_solve_mfma_kernel(LuBatch bt, LuGeo g) {
  __shared__ double Ts[2][LB][LB + 1];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 15, lg = lane >> 4;
  const int strip = blockIdx.x, slot = blockIdx.y;
  const double* __restrict__ A = bt.A[slot];
  const double* __restrict__ tinv = bt.tinv[slot];
  double* __restrict__ out = bt.out[slot];
  // W = P e_strip
  const int srow = bt.sinv[slot][LB * strip + li];
  d4 acc[NBW];
#pragma unroll
  for (int q = 0; q < NBW; ++q)
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[q][i] = (LB * (8 * q + wave) + lg + 4 * i == srow) ? 1.0 : 0.0;
  // the first block with a non-zero of P e_strip: the forward steps before it change nothing
  int first = srow / LB;
#pragma unroll
  for (int m = 1; m < 16; m <<= 1) first = min(first, __shfl_xor(first, m, 64));
  first = __builtin_amdgcn_readfirstlane(first);
  int par = 0;
  solve_phase<true, NBW>(Ts, acc, A, tinv, g.Na, g.nbs, first, par);
  solve_phase<false, NBW>(Ts, acc, A, tinv, g.Na, g.nbs, 0, par);
#pragma unroll
  for (int q = 0; q < NBW; ++q) {
    const int b = 8 * q + wave;
    if (b >= g.nbs) continue;
    acc_fence(acc[q]);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const long long row = (long long)LB * b + lg + 4 * i, col = (long long)LB * strip + li;
      if (row < g.n && col < g.n) out[row * g.n + col] = acc[q][i];
    }
  }
}

// (round 4) out[:, 16 strip .. 16 strip + 15] = inv(A) e_col: forward with the interleaved
// permutations and L, backward with U.  One workgroup per strip of the identity (grid x) and slot
// (grid y).  Kept for A/B measurements (BO_LU_SOLVE=rows).
template <int LR>
__global__ __launch_bounds__(LT) void lu_solve_kernel(LuBatch bt, LuGeo g) {
  __shared__ StripLds L;
  const int tid = threadIdx.x;
  const int strip = blockIdx.x, slot = blockIdx.y;
  const double* __restrict__ A = bt.A[slot];
  const int* __restrict__ prec = bt.prec[slot];
  double* __restrict__ out = bt.out[slot];
  double w[LR][LB];
#pragma unroll
  for (int r = 0; r < LR; ++r) {
    const long long row = own_row(0, r);
#pragma unroll
    for (int c = 0; c < LB; ++c) w[r][c] = row == (long long)LB * strip + c ? 1.0 : 0.0;
  }
  // forward: per step the permutation, W_s = L11^-1 W_s, W_below -= L21 W_s
  init_maps(L);
  __syncthreads();
  int pm = 0, pp = 0, ps = 0;
  if (tid < 32) get_perm(prec, pm, pp, ps);
  const bool stamp = strip == 0;
  (void)stamp;
  for (int s = 0; s < g.nbs; ++s) {
    const int b = LB * s;
    if (stamp) LU_STAMP(s, 8);
    // the step's loads first: L11, the first columns of L21 (the permutation record was
    // prefetched one step ahead)
    const double l11 = tid < LB * LB ? A[(long long)(b + (tid >> 4)) * g.Na + b + (tid & 15)] : 0.0;
    bool act[LR];
#pragma unroll
    for (int r = 0; r < LR; ++r) act[r] = own_row(0, r) >= b + LB && own_row(0, r) < g.n_p;
    R16<LR> st;
    r16_start(A, g.Na, b, 0, act, st);
    put_perm(L, pm, pp, ps);
    if (tid < 32 && s + 1 < g.nbs) get_perm(prec + (long long)(s + 1) * PREC, pm, pp, ps);   // next step's, in flight
    __syncthreads();
    apply_perm(L, w, 0, g.n_p);
    if (stamp) LU_STAMP(s, 9);
    // W_s == 0 (the identity strip's rows lie below, and no pivot pulled one up): the step adds
    // nothing -- dtrsm skips zero entries of B too (its `IF (B(K,J).NE.ZERO)`)
    int nz = 0;
#pragma unroll
    for (int r = 0; r < LR; ++r) {
      const long long row = own_row(0, r);
      if (row >= b && row < b + LB) {
#pragma unroll
        for (int c = 0; c < LB; ++c) nz |= w[r][c] != 0.0;
      }
    }
    if (!__syncthreads_or(nz)) continue;
    if (tid < LB * LB) L.L11[tid & 15][tid >> 4] = l11;
#pragma unroll
    for (int r = 0; r < LR; ++r) {
      const long long row = own_row(0, r);
      if (row >= b && row < b + LB) {
#pragma unroll
        for (int c = 0; c < LB; ++c) L.T[row - b][c] = w[r][c];
      }
    }
    __syncthreads();
    trsm_lower(L);
    __syncthreads();
#pragma unroll
    for (int r = 0; r < LR; ++r) {
      const long long row = own_row(0, r);
      if (row >= b && row < b + LB) {
#pragma unroll
        for (int c = 0; c < LB; ++c) w[r][c] = L.T[row - b][c];
      }
    }
    r16_finish(A, g.Na, b, L, w, act, st);
    __syncthreads();
  }
  // backward: per step from the last, W_s = U_ss^-1 W_s, W_above -= U_above,s W_s
  for (int s = g.nbs - 1; s >= 0; --s) {
    const int b = LB * s;
    if (stamp) LU_STAMP(s, 12);
    bool act[LR];
#pragma unroll
    for (int r = 0; r < LR; ++r) act[r] = own_row(0, r) < b;
    R16<LR> st;
    r16_start(A, g.Na, b, 0, act, st);                         // U_above,s's first columns, early
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
    trsm_upper(L);
    __syncthreads();
#pragma unroll
    for (int r = 0; r < LR; ++r) {
      const long long row = own_row(0, r);
      if (row >= b && row < b + LB) {
#pragma unroll
        for (int c = 0; c < LB; ++c) w[r][c] = L.T[row - b][c];
      }
    }
    r16_finish(A, g.Na, b, L, w, act, st);
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
  // BO_LU_PANEL=wide: every panel on the 8-wave loop; =small: the 4-wave panel at N <= 512 too
  // (A/B only)
  static const int small = [] {
    const char* e = getenv("BO_LU_PANEL");
    return (e && strcmp(e, "wide") == 0) ? 0 : (e && strcmp(e, "small") == 0) ? 2 :
           (e && strcmp(e, "small256") == 0) ? 3 : 1;
  }();
  g.small_panel = small;
  return g;
}

size_t slot_bytes(const LuGeo& g) {
  return a256((size_t)g.Na * g.n_p * sizeof(double)) + a256((size_t)g.nbs * PREC * sizeof(int)) +
         a256((size_t)g.n_p * sizeof(int)) + a256((size_t)g.nbs * 512 * sizeof(double));
}

// BO_LU_SOLVE=rows: the round-4 solve (interleaved permutations, one row per thread) for A/B
bool lu_solve_rows() {
  static const int v = [] {
    const char* e = getenv("BO_LU_SOLVE");
    return (e && strcmp(e, "rows") == 0) ? 1 : 0;
  }();
  return v != 0;
}

}  // namespace

// Internal (bo_fit.hip): workspace bytes for `n_lu` factorisations and the LU inverses of those
// objectives in one launch sequence (BO_OK, BO_ERR_SINGULAR on an exactly zero pivot of any of
// them, BO_ERR_UNSUPPORTED above the register capacity).
size_t bo_lu_workspace_size(int64_t n, int n_lu) {
  const LuGeo g = make_lu_geo((int)n);
  return (size_t)n_lu * slot_bytes(g) + 256;
}

int bo_lu_max_n() { return LT * LRMAX; }

int bo_lu_inverse(double* const* out, const double* const* km, int n_lu, int64_t ld, int64_t n, double jitter,
                  void* ws, size_t ws_bytes, hipStream_t s) {
  if (n < 1 || n > LT * LRMAX || n_lu < 1 || n_lu > BO_MAX_OBJ) return BO_ERR_UNSUPPORTED;
  if (ws_bytes < bo_lu_workspace_size(n, n_lu)) return BO_ERR_WORKSPACE;
  const LuGeo g = make_lu_geo((int)n);
  LuBatch bt;
  memset(&bt, 0, sizeof(bt));
  char* w = (char*)ws;
  for (int b = 0; b < n_lu; ++b) {
    bt.A[b] = (double*)w;
    bt.prec[b] = (int*)(w + a256((size_t)g.Na * g.n_p * sizeof(double)));
    bt.sinv[b] = (int*)((char*)bt.prec[b] + a256((size_t)g.nbs * PREC * sizeof(int)));
    bt.tinv[b] = (double*)((char*)bt.sinv[b] + a256((size_t)g.n_p * sizeof(int)));
    bt.km[b] = km[b];
    bt.out[b] = out[b];
    w += slot_bytes(g);
  }
  bt.status = (int*)w;
  BO_CHECK_HIP(hipMemsetAsync(bt.status, 0, sizeof(int) * BO_MAX_OBJ, s));
  const unsigned tiles = (unsigned)((g.n_p + 31) / 32);
  hipLaunchKernelGGL(lu_init_kernel, dim3(tiles, tiles, n_lu), dim3(256), 0, s, bt, g, (long long)ld, jitter);
  // rows per thread: the fewest that hold N_p (at N = 512 one row, so no predicated-off rows);
  // each step launch holds only the rows from its base (16 (k - 1)) down, so it takes the fewest
  // that hold those (N = 2048: 4 rows per thread for the first 97 steps, then 2, then 1)
  const int lr = (g.n_p + LT - 1) / LT;
  for (int k = 0; k < g.nbs; ++k) {
    const int blocks = k > 0 ? g.nbs - k : 1;      // the panel + the strips right of it
    const int rows = g.n_p - (k > 0 ? LB * (k - 1) : 0);
    auto step = rows <= LT ? lu_step_kernel<1> : rows <= 2 * LT ? lu_step_kernel<2> : lu_step_kernel<4>;
    hipLaunchKernelGGL(step, dim3(blocks, n_lu), dim3(LT), 0, s, bt, g, k);
  }
  const int nbw = (g.nbs + 7) / 8;
  if (lu_solve_rows() || nbw > 8) {
    // N > 1024 (the 16-accumulator solve spills) or BO_LU_SOLVE=rows: the row-per-thread solve
    auto solve = lr == 1 ? lu_solve_kernel<1> : lr == 2 ? lu_solve_kernel<2> : lu_solve_kernel<4>;
    hipLaunchKernelGGL(solve, dim3(g.nbs, n_lu), dim3(LT), 0, s, bt, g);
  } else {
    // laswp of the L columns, the permutation and the diagonal blocks' inverses, then the
    // matrix-core solve
    auto fin = lr == 1 ? lu_finalize_kernel<1> : lr == 2 ? lu_finalize_kernel<2> : lu_finalize_kernel<4>;
    hipLaunchKernelGGL(fin, dim3(g.nbs + 1, n_lu), dim3(LT), 0, s, bt, g);
    auto solve = nbw <= 1 ? lu_solve_mfma_kernel<1> : nbw <= 2 ? lu_solve_mfma_kernel<2> :
                 nbw <= 4 ? lu_solve_mfma_kernel<4> : lu_solve_mfma_kernel<8>;
    hipLaunchKernelGGL(solve, dim3(g.nbs, n_lu), dim3(LT), 0, s, bt, g);
  }
  BO_CHECK_HIP(hipGetLastError());
  int hs[BO_MAX_OBJ];
  BO_CHECK_HIP(hipMemcpyAsync(hs, bt.status, sizeof(int) * BO_MAX_OBJ, hipMemcpyDeviceToHost, s));
  BO_CHECK_HIP(hipStreamSynchronize(s));
  for (int b = 0; b < n_lu; ++b)
    if (hs[b]) return BO_ERR_SINGULAR;
  return BO_OK;
}

#ifdef BO_FIT_TIMING
// diagnostic build only: the LU stamps since the last read ([tag word, 100 MHz clock] pairs into
// `out`, 2 cap words); resets the count and returns it
extern "C" __attribute__((visibility("default"))) int bo_debug_lu_timing(long long* out, int cap) {
  int cnt = 0;
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  if (hipMemcpyFromSymbol(&cnt, HIP_SYMBOL(bo_lu_tcount), sizeof(int)) != hipSuccess) return -1;
  if (cnt > cap) cnt = cap;
  if (cnt > 4096) cnt = 4096;
  if (cnt > 0 && hipMemcpyFromSymbol(out, HIP_SYMBOL(bo_lu_tstamp), sizeof(long long) * 2 * cnt) != hipSuccess)
    return -1;
  const int zero = 0;
  if (hipMemcpyToSymbol(HIP_SYMBOL(bo_lu_tcount), &zero, sizeof(int)) != hipSuccess) return -1;
  return cnt;
}

// the per-column panel stamps: [step][column][4] (0 start, 1 wave max found, 2 after the
// barrier, 3 updated and rotated)
extern "C" __attribute__((visibility("default"))) int bo_debug_lu_cols(long long* out, int n) {
  if (n > 64 * LB_DIAG * 4) n = 64 * LB_DIAG * 4;
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(bo_lu_cstamp), sizeof(long long) * n) != hipSuccess) return -1;
  return n;
}

// the shader-clock stamps taken with them (same layout)
extern "C" __attribute__((visibility("default"))) int bo_debug_lu_cclk(long long* out, int n) {
  if (n > 64 * LB_DIAG * 4) n = 64 * LB_DIAG * 4;
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(bo_lu_cclk), sizeof(long long) * n) != hipSuccess) return -1;
  return n;
}
#endif
