// Fused GP posterior + UCB / "hypervolume improvement" + top-q over a candidate shard.
//
// Replaces the reference chain bayesopt/bayesian_optimization.py:145-207:
//   update_k_star (numba_kernels.py:406-442) -> update_mean (:450-488) ->
//   update_variance (:491-535) -> standardize_objectives (:538-570) ->
//   update_ucb / update_hypervolume_improvement (acquisition.py:55-108) ->
//   select_next_batch (acquisition.py:116-144, local top-q part).
//
// MI355X design:
//   * One wave owns 16 candidates.  For objective o it generates the K* column block
//     K*[f][j] = pv_o * exp(-0.5 |x_f - c_j|^2 / ls_o^2) straight into the B-operand
//     registers of v_mfma_f64_16x16x4_f64 (lane l: f = 4s + (l>>4), j = l & 15), so
//     K* never touches LDS or HBM.
//   * Z = K^-1 K* runs on the f64 matrix cores: the A operand (K^-1) is pre-packed in
//     fragment order (one coalesced 16-B load per lane covers two k-steps) and streamed
//     from L2 with a 4-deep register prefetch ring.
//   * The quadratic form sum_e K*[e][j] Z[e][j] needs K* in the accumulator layout; for
//     v_mfma_f64_16x16x4 the C rows (l>>4)+4r coincide with the B-fragment rows of k-step
//     4E+r, so the epilogue selects them from registers (single-panel) or recomputes the
//     4 exps (multi-panel, N > 512).
//   * mu, var, standardisation, UCB and Sigma-UCB are computed in registers; the local
//     top-q runs as a 64-lane bitonic network over shuffles with a ballot threshold.
//   * Persistent grid (one 256-thread workgroup per CU, 1 wave per SIMD), tiles of 64
//     candidates grid-strided; per-wave top-q lists merged by a second tiny kernel.

#include "bo_common.h"

#include <string.h>
#include <math.h>

#include <type_traits>
#include <vector>

#ifdef BO_ABL_STAMPS
// Diagnostic build only: per-wave phase cycle sums (s_memtime), never in a product build.
__device__ unsigned long long g_stamps[4096][8];
#define STAMP(var)                                                                    \
  do {                                                                                \
    __builtin_amdgcn_sched_barrier(0);                                                \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(var)::"memory");      \
    __builtin_amdgcn_sched_barrier(0);                                                \
  } while (0)
#else
#define STAMP(var) do { } while (0)
#endif
#ifdef BO_ABL_DBGQ
// Diagnostic build only: triangular-mode accumulators of tile 0 / wave 0 / objective 0.
__device__ double g_dbgq[64][2][4][64];
__device__ long long g_dbg_tile;
#endif

namespace {

constexpr int kWaves = 4;               // waves per workgroup
constexpr int kTile = 16 * kWaves;      // candidates per workgroup tile
constexpr int kPanelSteps = 128;        // k-steps of 4 training rows per register panel (512 rows)
#ifdef BO_ABL_PF8
constexpr int kPF = 8;                  // ablation: 8 pairs in flight (dense mode only)
#else
constexpr int kPF = 4;                  // prefetch depth (pairs of k-steps)
#endif

struct FusedArgs {
  int n_obj, dim, n_train, n_pad;       // n_pad = padded training rows (multiple of 32)
  int n_panels;                          // register panels of 512 rows (multi-panel only)
  int n_excl;
  int cand_kind, topq;
  long long n_cand, cand_offset, ld_out, n_tiles;
  long long grid_lo[BO_MAX_DIM], grid_shape[BO_MAX_DIM];
  const void* cand;
  const double* xpad;                    // [n_pad][DIM] training rows, padded rows = 1e200
  const double* excl;                    // [n_excl][DIM] evaluated points
  const d2* wpack;                       // packed K^-1 (pack_kinv_kernel layout)
  unsigned int wpack_bytes;
  const double* alpha;                   // [n_obj][n_pad] = K^-1 (y - pm)
  double pm[BO_MAX_OBJ], pv[BO_MAX_OBJ], nhl[BO_MAX_OBJ], beta[BO_MAX_OBJ], rsq_pv[BO_MAX_OBJ];
  double *mu, *var, *std_mu, *std_var, *ucb, *acq;
  TopEntry* partial;                     // [gridDim.x * kWaves][topq]
  const double* kstar;                   // KMEM: materialised k_star [n_obj][ks_rows][n_cand]
  long long ks_rows;
  int upper;                             // cm kernel: W = upper triangle of sym(K^-1), diagonal halved
  // separable K* on an integer grid (see sep_generate): device flag (0 => usable), last-axis
  // extent S and lower bound, LDS offsets (doubles) of the exp tables and per-wave R scratch
  const int* sep_flag;
  int sep_S;
  long long sep_lo;
  int off_tbl, off_rw;
  int rw_cache;                          // SEP row factors kept for every objective (LDS permitting)
  int off_sq;                            // > 0: explicit-candidate exponent in dot form (KRows DOTX)
};

template <int DIM>
__device__ __forceinline__ void load_candidate(const FusedArgs& a, long long j, bool valid,
                                               double (&c)[DIM]) {
#pragma unroll
  for (int k = 0; k < DIM; ++k) c[k] = 0.0;
  if (!valid) return;
  if (a.cand_kind == BO_CAND_GRID) {
    long long gi = a.cand_offset + j;
#pragma unroll
    for (int k = DIM - 1; k >= 0; --k) {
      if (k < a.dim) {
        const long long n = a.grid_shape[k];
        const long long q = gi / n;
        c[k] = (double)(a.grid_lo[k] + (gi - q * n));
        gi = q;
      }
    }
  } else if (a.cand_kind == BO_CAND_I64) {
    const long long* p = (const long long*)a.cand + j * a.dim;
#pragma unroll
    for (int k = 0; k < DIM; ++k)
      if (k < a.dim) c[k] = (double)p[k];
  } else {
    const double* p = (const double*)a.cand + j * a.dim;
#pragma unroll
    for (int k = 0; k < DIM; ++k)
      if (k < a.dim) c[k] = p[k];
  }
}

// squared distance between LDS row `row` ([*][DIM], 16-B aligned) and the candidate;
// numba_kernels.py:436-437 (diff = x_e - c_i, then diff . diff)
template <int DIM>
__device__ __forceinline__ double sqdist(const double* xs, int row, const double (&c)[DIM]) {
  const d2* r = (const d2*)(xs + row * DIM);
  double sq = 0.0;
#pragma unroll
  for (int k = 0; k < DIM / 2; ++k) {
    const d2 x = r[k];
    const double d0 = x.x - c[2 * k], d1 = x.y - c[2 * k + 1];
    sq = __builtin_fma(d0, d0, sq);
    sq = __builtin_fma(d1, d1, sq);
  }
  return sq;
}

__device__ __forceinline__ double kstar_at(const FusedArgs& a, int o, int f, long long j, bool valid) {
  return (valid && f < a.n_train) ? a.kstar[((long long)o * a.ks_rows + f) * a.n_cand + j] : 0.0;
}

__device__ __forceinline__ d4 mfma64(double a, double b, d4 c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

// Fence between the last MFMA of a contraction and the first read of its accumulators.
// hipcc's gfx950 hazard recognizer under-counts the wait states a VALU / v_accvgpr_read needs
// after v_mfma_f64_16x16x4_f64 when the reading block is reached through a branch that skips
// another block (observed: stale rows of the last MFMA, deterministic data-dependent errors
// up to 0.15 pv in the triangular variance).  The asm consumes and "redefines" both
// accumulators in place, so it cannot be scheduled before the MFMAs that produce them and no
// read of them can be hoisted above it; its 64 wait states cover the MFMA's full latency.
// AGPR: accumulators allocated in AGPRs (the register-resident kernel) or VGPRs (grid kernel).
template <bool AGPR, int NOPS = 64>
__device__ __forceinline__ void mfma_fence(d4& x, d4& y) {
#define BO_NOPS8 "s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7"
  if (NOPS == 0) {
    if (AGPR) asm volatile("" : "+a"(x), "+a"(y));
    else asm volatile("" : "+v"(x), "+v"(y));
  } else {
    if (AGPR) asm volatile(BO_NOPS8 : "+a"(x), "+a"(y));
    else asm volatile(BO_NOPS8 : "+v"(x), "+v"(y));
  }
#undef BO_NOPS8
}

// vmcnt(n) with expcnt / lgkmcnt left at their maxima (gfx9 s_waitcnt encoding)
#define BO_WAIT_VMCNT(n) __builtin_amdgcn_s_waitcnt(((n) & 0xF) | (((n) >> 4) << 14) | 0x70 | 0xF00)

__device__ __forceinline__ d2 wload(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
  return __builtin_bit_cast(d2, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0));
}

// One E-pair (E = 2ep, 2ep+1: 32 training rows) of one panel: acc0/acc1 += W[E, panel] . B.
// The k-steps are walked in chunks of 8 (4 pairs, 32 rows); a chunk's 4 pairs use ring
// slots 0..3, so every E-pair starts at slot 0 and the ring index stays static.
// The packed stream is consumed strictly in order: `pos` counts pairs (2 KiB each: the A
// fragments of E and E+1) and the load for pair pos+4 refills the slot just consumed.
// Past the end of the stream the buffer range check returns zeros (no fault, no branch).
//   dense (tri = false): every chunk; K*[e][j] for the epilogue is selected from B by
//     masked FMAs (chunk c == ep holds rows 32ep .. 32ep+31).
//   triangular (tri = true): W = R^T is upper triangular, so E-pair ep needs chunks c >= ep
//     only (about half the MFMAs); the epilogue is |v|^2 and needs no selection.
// Multi-panel (N > 512, RECOMP): the epilogue rows of E-pair ep+1 are recomputed (8 exps per
// lane), one per chunk during E-pair ep's MFMAs, so that VALU work issues in the matrix-core
// shadow instead of serialising after the contraction.
template <int NS, int DIM, bool SELECT, bool RECOMP>
__device__ __forceinline__ void contract_epair(__amdgpu_buffer_rsrc_t wr, int voff, int base,
                                               int& pos, int ep, bool tri, const double (&B)[NS],
                                               d2 (&wa)[kPF], d2 (&wb)[kPF], d4& acc0, d4& acc1,
                                               d4& acc2, d4& acc3,
                                               double (&sel0)[4], double (&sel1)[4],
                                               const double* xs, const double (&cc)[DIM],
                                               double pv, double nhl, int g, double (&nxt)[8]) {
  constexpr int NCH = NS / 8;
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
#ifdef BO_ABL_SYNCCHUNK
    if (!tri || c >= ep) __builtin_amdgcn_s_barrier();
#endif
    if (RECOMP && c < 8) {
      // row of E-pair ep+1 for slot c: e = 32(ep+1) + 16(c>>2) + g + 4(c&3)
      const int e = 32 * (ep + 1) + 16 * (c >> 2) + g + 4 * (c & 3);
      nxt[c] = pv * exp(sqdist<DIM>(xs, e, cc) * nhl);
    }
    if (!tri || c >= ep) {
#pragma unroll
      for (int pp = 0; pp < 4; ++pp) {
        const int p = 4 * c + pp;
        const int sl = (kPF == 8) ? 4 * (c & 1) + pp : pp;   // PF8: valid for dense streams only
        const d2 ca = wa[sl];
        const d2 cb = wb[sl];
        const int so = base + ((pos + kPF) << 11);
#ifndef BO_ABL_NOLOAD
        wa[sl] = wload(wr, voff, so);
        wb[sl] = wload(wr, voff, so + 1024);
#else   // ablation build only: keep the stream's address arithmetic, drop the loads
        wa[pp] = ca * 0.999 + (double)so;
        wb[pp] = cb * 0.999;
#endif
        ++pos;
        acc0 = mfma64(ca.x, B[2 * p], acc0);
        acc1 = mfma64(cb.x, B[2 * p], acc1);
#ifdef BO_ABL_ACC4
        acc2 = mfma64(ca.y, B[2 * p + 1], acc2);
        acc3 = mfma64(cb.y, B[2 * p + 1], acc3);
#else
        acc0 = mfma64(ca.y, B[2 * p + 1], acc0);
        acc1 = mfma64(cb.y, B[2 * p + 1], acc1);
#endif
      }
      if (SELECT && !tri) {
        const double m = (c == ep) ? 1.0 : 0.0;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          sel0[r] = __builtin_fma(m, B[8 * c + r], sel0[r]);
          sel1[r] = __builtin_fma(m, B[8 * c + 4 + r], sel1[r]);
        }
      }
    }
  }
}

__device__ __forceinline__ void prime_ring(__amdgpu_buffer_rsrc_t wr, int voff, int base,
                                           d2 (&wa)[kPF], d2 (&wb)[kPF]) {
#pragma unroll
  for (int p = 0; p < kPF; ++p) {
    wa[p] = wload(wr, voff, base + (p << 11));
    wb[p] = wload(wr, voff, base + (p << 11) + 1024);
  }
}

// NS = k-steps held in registers per panel (NS*4 training rows); DIM = padded input
// dimension (2, 4 or 8; padded coordinates are 0 on both sides); MULTI = several panels.
template <int NS, int DIM, bool MULTI, bool KMEM>
__global__ __launch_bounds__(256, 1) void fused_predict_kernel(const FusedArgs a) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  double* xs = smem;                                   // [n_pad][DIM] training rows
  double* alpha = xs + (size_t)a.n_pad * DIM;          // [n_obj][n_pad]
  double* exs_buf = alpha + (size_t)a.n_obj * a.n_pad; // [n_excl][DIM] (separate set only)

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, jl = lane & 15;

  for (int t = tid; t < a.n_pad * DIM; t += blockDim.x) xs[t] = a.xpad[t];
  for (int t = tid; t < a.n_obj * a.n_pad; t += blockDim.x) alpha[t] = a.alpha[t];
  const double* exs = a.excl ? exs_buf : xs;   // NULL: the evaluated points are x_train
  const int n_excl = a.excl ? a.n_excl : a.n_train;
  if (a.excl)
    for (int t = tid; t < a.n_excl * DIM; t += blockDim.x) exs_buf[t] = a.excl[t];
  __syncthreads();

  const __amdgpu_buffer_rsrc_t wr =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.wpack, (short)0, (int)a.wpack_bytes, 0x00020000);
  const int voff = lane * 16;
  // triangular variance formulation (set on the device by the K^-1 Cholesky, see
  // predict_impl); uniform across the grid
  const bool tri = false;   // (the triangular variance form lives in cm_predict_kernel only)

  double top_v = -__builtin_inf();
  long long top_i = -1;
  const int n_ep = a.n_pad / 32;                           // E-block pairs over all rows
  const int w_obj = a.n_pad * a.n_pad * 8;                 // bytes per objective
  const int w_panel = a.n_pad * (NS * 4) * 8;              // bytes per panel

#ifdef BO_ABL_STAMPS
  unsigned long long st_sum[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long t_a = 0, t_b = 0;
#endif
  for (long long tile = blockIdx.x; tile < a.n_tiles; tile += gridDim.x) {
#ifdef BO_ABL_STAMPS
    STAMP(t_b);
    if (tile != blockIdx.x) st_sum[4] += t_b - t_a;   // top-q insert + loop overhead
    t_a = t_b;
#endif
    const long long j = tile * kTile + wave * 16 + jl;
    const bool valid = j < a.n_cand;
    double c[DIM];
    if (!KMEM) load_candidate<DIM>(a, j, valid, c);
    else {
#pragma unroll
      for (int k = 0; k < DIM; ++k) c[k] = 0.0;
    }

    // exclusion (acquisition.py:137-139): candidate equal, coordinate by coordinate, to an
    // evaluated point.  Lane group g checks points g, g+4, ...
    // With the default set (the training points, a.excl == nullptr) the test is folded into
    // objective 0's K* generation below: all coordinates equal <=> squared distance == 0
    // (finite coordinates).
    bool hit = false;
    // (multi-panel kernels keep the explicit loop: their register budget is tighter)
    for (int e = g; e < ((KMEM || (!MULTI && !a.excl)) ? 0 : n_excl); e += 4) {
      const d2* r = (const d2*)(exs + e * DIM);
      bool eq = true;
#pragma unroll
      for (int k = 0; k < DIM / 2; ++k) {
        const d2 x = r[k];
        eq = eq && (x.x == c[2 * k]) && (x.y == c[2 * k + 1]);
      }
      hit = hit || eq;
    }
    double acq = 0.0;
#ifdef BO_ABL_STAMPS
    STAMP(t_b); st_sum[0] += t_b - t_a; t_a = t_b;   // candidate load + exclusion
#endif
    for (int o = 0; o < a.n_obj; ++o) {
      const double pv = a.pv[o], nhl = a.nhl[o];
      const double* al = alpha + o * a.n_pad;
      double qpart = 0.0, mpart = 0.0;
      for (int panel = 0; panel < (MULTI ? a.n_panels : 1); ++panel) {
        const int f0 = panel * NS * 4;
        // K* block for this lane: B[s] = K*[f0 + 4s + g][j]  (numba_kernels.py:440-442);
        // padded rows sit at 1e200 so their exp underflows to exactly 0.
        double B[NS];
#pragma unroll
        for (int s = 0; s < NS; ++s) {
          const int f = f0 + 4 * s + g;
          if (KMEM) {
            B[s] = kstar_at(a, o, f, j, valid);
          } else {
            const double sq = sqdist<DIM>(xs, f, c);
            if (!MULTI && !a.excl && o == 0) hit = hit || (sq == 0.0);
#ifndef BO_ABL_NOEXP
            B[s] = pv * exp(sq * nhl);
#else   // ablation build only: K* without the exp
            B[s] = pv * (sq * nhl);
#endif
          }
          if ((s & 3) == 3) __builtin_amdgcn_sched_barrier(0);
        }
        const int base = o * w_obj + panel * w_panel;
        d2 wa[kPF], wb[kPF];
#ifdef BO_ABL_STAMPS
        STAMP(t_b); st_sum[1] += t_b - t_a; t_a = t_b;   // K* generation (exp)
#endif
        prime_ring(wr, voff, base, wa, wb);
        int pos = 0;
        // multi-panel epilogue rows: K*[e][j], e = 32ep + 16h + g + 4r -> nxt[4h + r]
        double nxt[8];
        if (MULTI) {
#pragma unroll
          for (int t = 0; t < 8; ++t) {
            const int e = 16 * (t >> 2) + g + 4 * (t & 3);
            nxt[t] = KMEM ? kstar_at(a, o, e, j, valid) : pv * exp(sqdist<DIM>(xs, e, c) * nhl);
          }
        }
        for (int ep = 0; ep < n_ep; ++ep) {
#ifdef BO_ABL_SYNCEP
          __builtin_amdgcn_s_barrier();
#endif
          d4 acc0 = {0.0, 0.0, 0.0, 0.0}, acc1 = {0.0, 0.0, 0.0, 0.0};
          d4 acc2 = {0.0, 0.0, 0.0, 0.0}, acc3 = {0.0, 0.0, 0.0, 0.0};
          double sel0[4] = {0.0, 0.0, 0.0, 0.0}, sel1[4] = {0.0, 0.0, 0.0, 0.0};
          if (MULTI) {
#pragma unroll
            for (int r = 0; r < 4; ++r) { sel0[r] = nxt[r]; sel1[r] = nxt[4 + r]; }
            if (KMEM) {
#pragma unroll
              for (int t = 0; t < 8; ++t) {
                const int e = 32 * (ep + 1) + 16 * (t >> 2) + g + 4 * (t & 3);
                nxt[t] = kstar_at(a, o, e, j, valid);
              }
            }
          }
          contract_epair<NS, DIM, !MULTI, MULTI && !KMEM>(wr, voff, base, pos, ep, tri, B, wa, wb,
                                                          acc0, acc1, acc2, acc3, sel0, sel1, xs, c, pv, nhl,
                                                          g, nxt);
          mfma_fence<true>(acc0, acc1);
#ifdef BO_ABL_ACC4
          acc0 += acc2;
          acc1 += acc3;
#endif
          if (tri) {
#ifdef BO_ABL_DBGQ
            if (tile == g_dbg_tile && wave == 0 && o == 0 && ep < 64)
              for (int r = 0; r < 4; ++r) { g_dbgq[ep][0][r][lane] = acc0[r]; g_dbgq[ep][1][r][lane] = acc1[r]; }
#endif
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              qpart = __builtin_fma(acc0[r], acc0[r], qpart);
              qpart = __builtin_fma(acc1[r], acc1[r], qpart);
            }
            continue;
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            qpart = __builtin_fma(sel0[r], acc0[r], qpart);
            qpart = __builtin_fma(sel1[r], acc1[r], qpart);
          }
        }
#pragma unroll
        for (int s = 0; s < NS; ++s) mpart = __builtin_fma(al[f0 + 4 * s + g], B[s], mpart);
      }
      // reduce over the 4 lane groups holding the same candidate
#ifdef BO_ABL_STAMPS
      STAMP(t_b); st_sum[2] += t_b - t_a; t_a = t_b;   // contraction (MFMA loop + mu dot)
#endif
      qpart += __shfl_xor(qpart, 16, 64);
      qpart += __shfl_xor(qpart, 32, 64);
      mpart += __shfl_xor(mpart, 16, 64);
      mpart += __shfl_xor(mpart, 32, 64);

      const double pm = a.pm[o];
      const double mu = pm + mpart;                                   // :486-488
      const double var = fmax(pv - qpart, BO_MIN_VARIANCE);           // :532-535
      const double smu = (mu - pm) / a.rsq_pv[o];                      // :563-565
      const double svar = var / pv;                                    // :568-570
      const double u = smu + a.beta[o] * sqrt(fabs(svar));             // acquisition.py:52
      acq = (o == 0) ? u : acq + u;                                    // acquisition.py:108
      if (valid && g == 0) {
        const long long off = (long long)o * a.ld_out + j;
        if (a.mu) a.mu[off] = mu;
        if (a.var) a.var[off] = var;
        if (a.std_mu) a.std_mu[off] = smu;
        if (a.std_var) a.std_var[off] = svar;
        if (a.ucb) a.ucb[off] = u;
      }
    }
#ifdef BO_ABL_STAMPS
    STAMP(t_b); st_sum[3] += t_b - t_a; t_a = t_b;   // per-objective epilogues + stores
#endif
    if (valid && g == 0 && a.acq) a.acq[j] = acq;
    if (a.topq > 0) {
      const unsigned long long hb = __ballot(hit);
      const bool excluded =
          ((hb >> jl) | (hb >> (jl + 16)) | (hb >> (jl + 32)) | (hb >> (jl + 48))) & 1ull;
      const long long gi = (valid && !excluded) ? a.cand_offset + j : -1;
      bo_wave_topq_insert(top_v, top_i, acq, gi, a.topq);
    }
  }
#ifdef BO_ABL_STAMPS
  if (lane == 0) {
    const int w = blockIdx.x * kWaves + wave;
    for (int k = 0; k < 5; ++k) g_stamps[w][k] = st_sum[k];
    g_stamps[w][4] = 1;
  }
#endif
  if (a.topq > 0 && lane < a.topq) {
    TopEntry* dst = a.partial + ((size_t)blockIdx.x * kWaves + wave) * a.topq;
    dst[lane].v = top_v;
    dst[lane].i = top_i;
  }
}

// ---------------------------------------------------------------------------------------
// Chunk-major fused kernel (N <= 512, every candidate kind): the production path.
//
// f64 MFMAs and f64 VALU instructions share the SIMD's DP pipe (measured on MI355X: they
// serialise even across waves), so the time of this kernel is  sum(MFMA) + sum(f64 VALU).
// The loop order is therefore chosen to generate every K* value exactly ONCE:
//   for each 32-row chunk c of K* (rows 32c .. 32c+31, 8 values per lane):
//       generate K*[chunk c][16 candidates]  (B operand, registers)
//       for each E-pair ep (32 rows of W) that touches chunk c  -- all 16, or ep <= c when
//       W = R^T is upper triangular:   acc[ep] += W[ep-rows, chunk c] . K*[chunk c]
// with the accumulators of all (up to 16) E-pairs resident (256 AGPRs, one wave per SIMD).
// The W stream is packed in exactly this (c, ep, k-step pair) order and streamed from L2
// through a 4-deep register ring; the next chunk's K* is generated while the current chunk's
// MFMAs run.  Per 16-MFMA E-pair block there is no VALU work at all.
//
// Variance forms (the reference: q = k . (K^-1 k), update_variance numba_kernels.py:521-529):
//   upper (default): q = 2 k . (U k) with U = upper triangle of sym(K^-1) = (K^-1 + K^-T)/2,
//     diagonal halved -- exactly k^T K^-1 k in exact arithmetic (k^T A k = k^T sym(A) k), half
//     the MFMAs, no factorisation;
//   dense: z = K^-1 k verbatim; q = k . z after the last chunk (chunk ep regenerated).
//
// K* generation:
//   * integer 'ij' grid (bayesian_optimization.py:338-340) whose 16-candidate wave tiles lie
//     in one grid row (SEP): K*[f][j] = (pv R(f)) * T[x_f,last - c_j,last], R(f) =
//     exp(nhl sum_{k != last} (x_fk - c_k)^2) computed once per row and wave tile, T the
//     exp(nhl m^2) table over last-axis differences (LDS); one multiply per value;
//   * otherwise pv exp(nhl |x_f - c_j|^2) per value (numba_kernels.py:436-442).
// ---------------------------------------------------------------------------------------
constexpr int kCMaxEp = 16;              // E-pairs (32 rows each): N <= 512

// Nested guards over the unrolled E-pair bodies: body E runs iff E < n, and is entered only
// from body E - 1 (see chunk_step in cm_tiles).
template <int E, int N>
struct EpChain {
  template <class F>
  static __device__ __forceinline__ void run(F& f, int n) {
    if (E < n) {
      f(std::integral_constant<int, E>{});
      EpChain<E + 1, N>::run(f, n);
    }
  }
};
template <int N>
struct EpChain<N, N> {
  template <class F>
  static __device__ __forceinline__ void run(F&, int) {}
};

// 2^t for the non-positive exponents of K* (t = -inf or very negative -> exactly 0): range
// reduction to r in [-1/2, 1/2], Taylor degree 13 in r ln 2 (|term 14| < 2e-16 relative), no
// overflow branches (the argument is never positive).
__device__ __forceinline__ double exp2_nonpos(double t) {
  const double x = fmax(t, -1100.0);
  const double n = __builtin_rint(x);
  const double r = x - n;
  double p = 1.36914888539041241e-12;
  p = __builtin_fma(p, r, 2.56784359934881958e-11);
  p = __builtin_fma(p, r, 4.44553827187081007e-10);
  p = __builtin_fma(p, r, 7.05491162080112088e-09);
  p = __builtin_fma(p, r, 1.01780860092396960e-07);
  p = __builtin_fma(p, r, 1.32154867901443053e-06);
  p = __builtin_fma(p, r, 1.52527338040598377e-05);
  p = __builtin_fma(p, r, 1.54035303933816061e-04);
  p = __builtin_fma(p, r, 1.33335581464284411e-03);
  p = __builtin_fma(p, r, 9.61812910762847688e-03);
  p = __builtin_fma(p, r, 5.55041086648215762e-02);
  p = __builtin_fma(p, r, 2.40226506959100694e-01);
  p = __builtin_fma(p, r, 6.93147180559945286e-01);
  p = __builtin_fma(p, r, 1.0);
  return __builtin_ldexp(p, (int)n);
}

// DOTX (explicit candidates, LDS permitting): the exponent of pv exp(nhl |x_f - c|^2) in base 2
// as nl2 |x_f|^2 + (nl2 |c|^2 + log2 pv) + sum_k x_fk (-2 nl2 c_k), nl2 = nhl log2 e, with
// |x_f|^2 from LDS and the candidate terms per lane: DIM + 1 FMAs instead of 2 DIM + 2 f64
// instructions, pv folded into the exponent, and exp2_nonpos instead of exp.
template <int DIM, bool SEP, bool DOTX = false>
struct KRows {
  const double* sq;   // DOTX: [n_pad] |x_f|^2 (inf for padded rows)
  double cj, nl2, dk[DIM];
  const double* rv;   // SEP: [n_pad] pv * R(f) (0 for padded rows)
  const int* rb;      // SEP: [n_pad] table index base (x_f,last - lo_last) + S - 1; jl = col0 + lane
  const double* tb;   // SEP: objective's table T
  const double* xs;   // !SEP: training rows [n_pad][DIM] (padded rows at 1e200)
  double c[DIM];      // !SEP: this lane's candidate
  double pv, nhl;
  int jl;
  __device__ __forceinline__ double at(int f) const {
#ifdef BO_ABL_NOGEN   // ablation build only: K* values without the generation work
    return pv * (double)(f + jl);
#endif
    if (SEP) return rv[f] * tb[rb[f] - jl];
    if (DOTX) {
      const d2* r = (const d2*)(xs + f * DIM);
      double t = __builtin_fma(nl2, sq[f], cj);
#pragma unroll
      for (int k = 0; k < DIM / 2; ++k) {
        const d2 x = r[k];
        t = __builtin_fma(x.x, dk[2 * k], t);
        t = __builtin_fma(x.y, dk[2 * k + 1], t);
      }
      return exp2_nonpos(t);
    }
    return pv * exp(sqdist<DIM>(xs, f, c) * nhl);
  }
  // the 8 values of 32-row chunk `ch` this lane feeds to the MFMAs: rows 32 ch + 4 s + g
  __device__ __forceinline__ void chunk(int ch, int g, double (&B)[8]) const {
#pragma unroll
    for (int s = 0; s < 8; ++s) B[s] = at(32 * ch + 4 * s + g);
  }
};

// Next-chunk generation split into three stages that chunk_step places between the MFMA
// pairs of the chunk's first E-pair (sched barriers pin them), so that every LDS round trip
// of the generation (SEP: row factor + table index, then the table value; the alpha values
// of the mean) completes under MFMAs instead of stalling the wave before the chunk:
//   s0: rv[f], rb[f], alpha[f] loads     s1: table loads T[rb - jl]     s2: the products.
// The exp path (!SEP) is VALU work that serialises with f64 MFMAs anyway: all of it in s2.
template <int DIM, bool SEP, bool DOTX = false>
struct KGen {
  using KR = KRows<DIM, SEP, DOTX>;
  double rv[8], tv[8];
  int rb[8];
  __device__ __forceinline__ void s0(const KR& K, const double* al, bool mu_on, int ch,
                                     int g, double (&A)[8]) {
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const int f = 32 * ch + 4 * s + g;
      const double a = al[f];
      A[s] = mu_on ? a : 0.0;
      if (SEP) { rv[s] = K.rv[f]; rb[s] = K.rb[f]; }
    }
  }
  // s0 without the alpha values (the variance epilogue's regeneration)
  __device__ __forceinline__ void s0k(const KR& K, int ch, int g) {
    if (SEP) {
#pragma unroll
      for (int s = 0; s < 8; ++s) {
        const int f = 32 * ch + 4 * s + g;
        rv[s] = K.rv[f];
        rb[s] = K.rb[f];
      }
    }
  }
  __device__ __forceinline__ void s1(const KR& K) {
    if (SEP) {
#pragma unroll
      for (int s = 0; s < 8; ++s) tv[s] = K.tb[rb[s] - K.jl];
    }
  }
  __device__ __forceinline__ void s2(const KR& K, int ch, int g, double (&B)[8]) {
#ifdef BO_ABL_NOGEN
    K.chunk(ch, g, B);
    return;
#endif
    if (SEP) {
#pragma unroll
      for (int s = 0; s < 8; ++s) B[s] = rv[s] * tv[s];
    } else {
      K.chunk(ch, g, B);
    }
  }
};

template <int DIM, bool SEP, bool UPPER, bool DOTX = false>
__device__ __forceinline__ void cm_tiles(const FusedArgs& a, double* smem) {
  constexpr bool upper = UPPER;
  const double* xs = smem;                                  // [n_pad][DIM]
  const double* alpha = xs + (size_t)a.n_pad * DIM;         // [n_obj][n_pad]
  const double* exs = alpha + (size_t)a.n_obj * a.n_pad;    // [n_excl][DIM] (explicit set)
  const double* tbl = smem + a.off_tbl;                     // [n_obj][2S - 1]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, jl = lane & 15;
  // SEP row factors, per wave: rv[nslot][n_pad] = pv_o R(f) (one slot per objective when they
  // are cached across the tiles of a grid row, else one slot rebuilt per objective and tile),
  // then rb[n_pad] = table index base (x_f,last - lo_last) + S - 1 and on[n_pad] = "training
  // point f lies on this grid row" (all other coordinates equal)
  const int nslot = a.rw_cache ? a.n_obj : 1;
  double* rv = smem + a.off_rw + (size_t)wave * a.n_pad * (nslot + 1);
  int* rb = (int*)(rv + (size_t)nslot * a.n_pad);
  int* on = rb + a.n_pad;
  long long cur_row = -1;
  const int TS = 2 * a.sep_S - 1;
  const int nch = a.n_pad / 32;
  const int last = a.dim - 1;
  const int w_obj = a.n_pad * a.n_pad * 8;
  const __amdgpu_buffer_rsrc_t wr =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.wpack, (short)0, (int)a.wpack_bytes, 0x00020000);
  const int voff = lane * 16;

  double top_v = -__builtin_inf();
  long long top_i = -1;
#ifdef BO_ABL_STAMPS
  unsigned long long st_sum[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long t_a = 0, t_b = 0;
  STAMP(t_a);
#endif
  // SEP: contiguous tile ranges per workgroup, so that a wave walks along grid rows and its
  // row factors are rebuilt once per row (every S / 64 tiles) instead of once per tile;
  // otherwise grid-strided tiles
  const long long tpw = (a.n_tiles + gridDim.x - 1) / gridDim.x;
  const long long t_first = SEP ? blockIdx.x * tpw : blockIdx.x;
  const long long t_end = SEP ? (t_first + tpw < a.n_tiles ? t_first + tpw : a.n_tiles) : a.n_tiles;
  const long long t_step = SEP ? 1 : gridDim.x;
  // row pass (numba_kernels.py:436-442 split along the grid): per training row f, the squared
  // distance over the non-last coordinates is shared by the wave's 16 candidates
  auto row_pass = [&](const double (&c)[DIM], int o_lo, int o_hi) {
    __builtin_amdgcn_wave_barrier();
    for (int f = lane; f < a.n_pad; f += 64) {
      int b = a.sep_S - 1, onrow = 0;                      // padded rows: any in-range index, v = 0
      double sqs = 0.0;
      if (f < a.n_train) {
        const double* r = xs + f * DIM;
        double xl = 0.0;
#pragma unroll
        for (int k = 0; k < DIM; ++k) {
          if (k == last) xl = r[k];
          else { const double d = r[k] - c[k]; sqs = __builtin_fma(d, d, sqs); }
        }
        b = (int)(xl - (double)a.sep_lo) + a.sep_S - 1;
        onrow = sqs == 0.0;
      }
      for (int o = o_lo; o < o_hi; ++o)
        rv[(size_t)(o - o_lo) * a.n_pad + f] = f < a.n_train ? a.pv[o] * exp(sqs * a.nhl[o]) : 0.0;
      rb[f] = b;
      on[f] = onrow;
    }
    __builtin_amdgcn_wave_barrier();
  };
  for (long long tile = t_first; tile < t_end; tile += t_step) {
    const long long j = tile * kTile + wave * 16 + jl;
    const bool valid = j < a.n_cand;
    double c[DIM];
    int col0 = 0;                 // SEP: the wave's first candidate's offset on the last axis
    if (SEP) {
      // the wave's 16 candidates: one grid row, consecutive along the last axis
      const long long j0 = tile * kTile + wave * 16;
      const long long jj = j0 < a.n_cand ? j0 : 0;
      load_candidate<DIM>(a, jj, true, c);
#pragma unroll
      for (int k = 0; k < DIM; ++k)
        if (k == last) { col0 = (int)(c[k] - (double)a.sep_lo); c[k] += (double)jl; }
      if (a.rw_cache) {
        const long long row = (a.cand_offset + jj) / a.sep_S;
        if (row != cur_row) { row_pass(c, 0, a.n_obj); cur_row = row; }
      }
    } else {
      load_candidate<DIM>(a, j, valid, c);
    }
    // exclusion (acquisition.py:137-139): an explicit set (or no grid structure) -> compare
    // coordinates, lane group g checking points g, g+4, ...; the default set on the grid ->
    // from the row pass below
    bool hit = false;
    if (a.excl || !SEP) {
      const double* es = a.excl ? exs : xs;
      const int ne = a.excl ? a.n_excl : a.n_train;
      for (int e = g; e < ne; e += 4) {
        const double* r = es + e * DIM;
        bool eq = true;
#pragma unroll
        for (int k = 0; k < DIM; ++k) eq = eq && (r[k] == c[k]);
        hit = hit || eq;
      }
    }
    unsigned int xmask = 0;
    double acq = 0.0;
    for (int o = 0; o < a.n_obj; ++o) {
      if (SEP && !a.rw_cache) row_pass(c, o, o + 1);
      KRows<DIM, SEP, DOTX> K;
      K.rv = rv + (a.rw_cache ? (size_t)o * a.n_pad : 0); K.rb = rb; K.tb = tbl + (size_t)o * TS;
      K.xs = xs; K.pv = a.pv[o]; K.nhl = a.nhl[o];
      K.jl = SEP ? col0 + jl : jl;   // T index = rb[f] - (col0 + jl) = x_f,last - c_last + S - 1
#pragma unroll
      for (int k = 0; k < DIM; ++k) K.c[k] = c[k];
      if (DOTX) {
        K.sq = smem + a.off_sq;
        K.nl2 = a.nhl[o] * 1.4426950408889634;
        double cc = 0.0;
#pragma unroll
        for (int k = 0; k < DIM; ++k) { cc = __builtin_fma(c[k], c[k], cc); K.dk[k] = -2.0 * K.nl2 * c[k]; }
        K.cj = __builtin_fma(K.nl2, cc, log2(a.pv[o]));
      }
#ifdef BO_ABL_STAMPS
      STAMP(t_b); st_sum[0] += t_b - t_a; t_a = t_b;   // tile setup + row pass
#endif
      const double* al = alpha + (size_t)o * a.n_pad;
      const int base = o * w_obj;
      d2 wa[kPF], wb[kPF];
      prime_ring(wr, voff, base, wa, wb);
      int pos = 0;
      double mpart = 0.0, qpart = 0.0;
      d4 acc[kCMaxEp][2];
      // E-pairs in groups of kCMaxEp (the accumulators one wave holds: 512 rows); a group
      // streams the chunks that touch it (c >= its first E-pair when upper, all otherwise) and
      // regenerates their K*.  One group when N <= 512.
      for (int e0 = 0; e0 < nch; e0 += kCMaxEp) {
        const int eN = nch - e0 < kCMaxEp ? nch - e0 : kCMaxEp;
#pragma unroll
        for (int e = 0; e < kCMaxEp; ++e) {
          acc[e][0] = (d4){0.0, 0.0, 0.0, 0.0};
          acc[e][1] = (d4){0.0, 0.0, 0.0, 0.0};
        }
        // one chunk: MFMAs from register set B while the next chunk's K* (and its alpha
        // values, An) is generated into Bn in three stages inside E-pair 0's MFMA stream (the
        // sets alternate: no register copies between the chunks).  Branch-free: the last chunk
        // regenerates itself (chn clamped) and groups after the first add 0 x alpha to mu.
        const bool mu_on = e0 == 0;
        KGen<DIM, SEP, DOTX> gen;
        auto chunk_step = [&](int ch, const double (&B)[8], double (&Bn)[8], const double (&A)[8],
                              double (&An)[8]) {
          // next chunk: ascending (dense) / descending (upper); the last one regenerates itself
          const int chn = upper ? (ch > e0 ? ch - 1 : ch) : (ch + 1 < nch ? ch + 1 : ch);
          // the group's E-pairs touching chunk ch, ascending: the first n_here of them (e0 + e
          // <= ch when upper).  EpChain nests the guards (body e+1 is reached only from body e),
          // so every body has one predecessor and hipcc's vmcnt waits inside the chunk stay
          // exact; independent guards made every body a join and cost a vmcnt(0) drain of the
          // W ring per E-pair.
          const int n_here = upper ? (ch - e0 + 1 < eN ? ch - e0 + 1 : eN) : eN;
          auto ep_body = [&](auto e_c) {
            constexpr int e = decltype(e_c)::value;
            (void)B;
#ifdef BO_ABL_SYNC64
            __builtin_amdgcn_s_barrier();
#endif
            if constexpr (e == 0) {
              gen.s0(K, al, mu_on, chn, g, An);
              __builtin_amdgcn_sched_barrier(0);
            }
#pragma unroll
            for (int pp = 0; pp < 4; ++pp) {
              // MFMAs first, then the refill of the same ring slot (no operand copies)
              acc[e][0] = mfma64(wa[pp].x, B[2 * pp], acc[e][0]);
              acc[e][1] = mfma64(wb[pp].x, B[2 * pp], acc[e][1]);
              acc[e][0] = mfma64(wa[pp].y, B[2 * pp + 1], acc[e][0]);
              acc[e][1] = mfma64(wb[pp].y, B[2 * pp + 1], acc[e][1]);
              const int so = base + ((pos + kPF) << 11);
#ifndef BO_ABL_NOLOAD
              wa[pp] = wload(wr, voff, so);
              wb[pp] = wload(wr, voff, so + 1024);
#else   // ablation build only: no W stream (operands stay in the ring)
              asm volatile("" : "+v"(wa[pp]), "+v"(wb[pp]) : "s"(so));
#endif
              ++pos;
              if constexpr (e == 0) {
                if (pp == 0) {
                  __builtin_amdgcn_sched_barrier(0);
                  gen.s1(K);
                  __builtin_amdgcn_sched_barrier(0);
                } else if (pp == 1) {
                  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                  for (int s = 0; s < 8; ++s) mpart = __builtin_fma(A[s], B[s], mpart);
                  __builtin_amdgcn_sched_barrier(0);
                } else if (pp == 2) {
                  __builtin_amdgcn_sched_barrier(0);
                  gen.s2(K, chn, g, Bn);
                  __builtin_amdgcn_sched_barrier(0);
                }
              }
            }
            // upper: E-pair e0 + e is complete after its own chunk (chunks descend), the last
            // body of that chunk: q += K*[chunk rows] . acc with the rows still in B (rows
            // 32 ep + g + 4r (+16) = B slots r (4 + r)); no regeneration
            if constexpr (UPPER) {
              if (ch - e0 == e) {
                mfma_fence<true, 64>(acc[e][0], acc[e][1]);
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                  qpart = __builtin_fma(B[r], acc[e][0][r], qpart);
                  qpart = __builtin_fma(B[4 + r], acc[e][1][r], qpart);
                }
              }
            }
          };
          EpChain<0, kCMaxEp>::run(ep_body, n_here);
        };
        const int c0 = upper ? nch - 1 : 0;
        double BX[8], BY[8], AX[8], AY[8];
        K.chunk(c0, g, BX);
#pragma unroll
        for (int s = 0; s < 8; ++s) AX[s] = mu_on ? al[32 * c0 + 4 * s + g] : 0.0;
        int ch = c0;
        if (upper) {
          for (; ch - 1 >= e0; ch -= 2) {
            chunk_step(ch, BX, BY, AX, AY);
            chunk_step(ch - 1, BY, BX, AY, AX);
          }
          if (ch >= e0) chunk_step(ch, BX, BY, AX, AY);
        } else {
          for (; ch + 1 < nch; ch += 2) {
            chunk_step(ch, BX, BY, AX, AY);
            chunk_step(ch + 1, BY, BX, AY, AX);
          }
          if (ch < nch) chunk_step(ch, BX, BY, AX, AY);
        }
        // q = k . z (dense): the rows 32 ep + g + 4r (+16) of K* = chunk ep's slots r (4 + r),
        // regenerated here (the upper form's q was accumulated inside the chunk loop).  A full
        // fence per accumulator: the scheduler may sink any E-pair's last MFMAs down to it.
#ifdef BO_ABL_STAMPS
        STAMP(t_b); st_sum[1] += t_b - t_a; t_a = t_b;   // chunk loop (MFMAs)
#endif
        // dense: q = k . z after the last chunk, chunk ep's K* regenerated.  Software-pipelined:
        // E-pair e+1's rows are loaded (KGen s0/s1) before E-pair e's fence and multiplied after
        // its FMAs, so the fences' wait states cover the LDS round trips.
        if (!upper) {
          KGen<DIM, SEP, DOTX> gq[2];
          double S[2][8];
          gq[0].s0k(K, e0, g);
          gq[0].s1(K);
          gq[0].s2(K, e0, g, S[0]);
#pragma unroll
          for (int e = 0; e < kCMaxEp; ++e) {
            if (e < eN) {
              const int cur = e & 1, nxt = cur ^ 1;
              const bool more = e + 1 < eN;
              if (more) gq[nxt].s0k(K, e0 + e + 1, g);
              mfma_fence<true, 64>(acc[e][0], acc[e][1]);
              if (more) gq[nxt].s1(K);
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                qpart = __builtin_fma(S[cur][r], acc[e][0][r], qpart);
                qpart = __builtin_fma(S[cur][4 + r], acc[e][1][r], qpart);
              }
              if (more) gq[nxt].s2(K, e0 + e + 1, g, S[nxt]);
            }
          }
        }
      }
      if (upper) qpart *= 2.0;
#ifdef BO_ABL_STAMPS
      STAMP(t_b); st_sum[2] += t_b - t_a; t_a = t_b;   // variance epilogue
#endif
      qpart += __shfl_xor(qpart, 16, 64);
      qpart += __shfl_xor(qpart, 32, 64);
      mpart += __shfl_xor(mpart, 16, 64);
      mpart += __shfl_xor(mpart, 32, 64);
      const double pv = a.pv[o], pm = a.pm[o];
      const double mu = pm + mpart;                                   // :486-488
      const double var = fmax(pv - qpart, BO_MIN_VARIANCE);           // :532-535
      const double smu = (mu - pm) / a.rsq_pv[o];                      // :563-565
      const double svar = var / pv;                                    // :568-570
      const double u = smu + a.beta[o] * sqrt(fabs(svar));             // acquisition.py:52
      acq = (o == 0) ? u : acq + u;                                    // acquisition.py:108
      if (valid && g == 0) {
        const long long off = (long long)o * a.ld_out + j;
        if (a.mu) a.mu[off] = mu;
        if (a.var) a.var[off] = var;
        if (a.std_mu) a.std_mu[off] = smu;
        if (a.std_var) a.std_var[off] = svar;
        if (a.ucb) a.ucb[off] = u;
      }
    }
    if (valid && g == 0 && a.acq) a.acq[j] = acq;
    if (a.topq > 0) {
      if (SEP && !a.excl) {
        // training points on this grid row whose last coordinate falls in the wave's 16
        // columns (all coordinates equal: acquisition.py:137-139); OR over the wave, bit jl
        // is this lane's candidate
        for (int f = lane; f < a.n_train; f += 64) {
          const int dx = rb[f] - (a.sep_S - 1) - col0;
          if (on[f] && dx >= 0 && dx < 16) xmask |= 1u << dx;
        }
        unsigned int m = xmask;
#pragma unroll
        for (int sh = 32; sh > 0; sh >>= 1) m |= (unsigned int)__shfl_xor((int)m, sh, 64);
        hit = (m >> jl) & 1u;
      }
      const unsigned long long hb = __ballot(hit);
      const bool excluded =
          ((hb >> jl) | (hb >> (jl + 16)) | (hb >> (jl + 32)) | (hb >> (jl + 48))) & 1ull;
      const long long gi = (valid && !excluded) ? a.cand_offset + j : -1;
      bo_wave_topq_insert(top_v, top_i, acq, gi, a.topq);
    }
  }
  BO_WAIT_VMCNT(0);                                          // no W load in flight at exit
#ifdef BO_ABL_STAMPS
  STAMP(t_b); st_sum[3] += t_b - t_a;
  if (lane == 0) {
    const int w = blockIdx.x * kWaves + wave;
    for (int k = 0; k < 4; ++k) g_stamps[w][k] = st_sum[k];
    g_stamps[w][4] = 1;
  }
#endif
  if (a.topq > 0 && lane < a.topq) {
    TopEntry* dst = a.partial + ((size_t)blockIdx.x * kWaves + wave) * a.topq;
    dst[lane].v = top_v;
    dst[lane].i = top_i;
  }
}

// GRID: the host found the grid structure usable (rows of 16); the device flag then says
// whether every training point lies on the grid's last axis (sep_check_kernel).
template <int DIM, bool GRID, bool UPPER>
__global__ __launch_bounds__(256, 1) void cm_predict_kernel(const FusedArgs a) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int tid = threadIdx.x;
  double* xs = smem;
  double* alpha = xs + (size_t)a.n_pad * DIM;
  double* exs = alpha + (size_t)a.n_obj * a.n_pad;
  for (int t = tid; t < a.n_pad * DIM; t += blockDim.x) xs[t] = a.xpad[t];
  for (int t = tid; t < a.n_obj * a.n_pad; t += blockDim.x) alpha[t] = a.alpha[t];
  if (a.excl)
    for (int t = tid; t < a.n_excl * DIM; t += blockDim.x) exs[t] = a.excl[t];
  const bool sep = GRID && __builtin_amdgcn_readfirstlane(*a.sep_flag) == 0;
  if (sep) {
    double* tbl = smem + a.off_tbl;
    const int TS = 2 * a.sep_S - 1;
    for (int t = tid; t < a.n_obj * TS; t += blockDim.x) {
      const int o = t / TS;
      const double m = (double)(t - o * TS - (a.sep_S - 1));
      tbl[t] = exp(a.nhl[o] * (m * m));
    }
  }
  if (!GRID && UPPER && a.off_sq > 0)
    for (int f = tid; f < a.n_pad; f += blockDim.x) {
      double q = 0.0;
      for (int k = 0; k < DIM; ++k) q = __builtin_fma(xs[f * DIM + k], xs[f * DIM + k], q);
      smem[a.off_sq + f] = q;                                   // padded rows: inf
    }
  __syncthreads();
  if (GRID && sep) cm_tiles<DIM, true, UPPER>(a, smem);
  else if (!GRID && UPPER && a.off_sq > 0) cm_tiles<DIM, false, UPPER, !GRID && UPPER>(a, smem);
  else cm_tiles<DIM, false, UPPER>(a, smem);
}

// Pack W into the chunk-major MFMA stream of cm_predict_kernel: per objective, for each group of
// kCMaxEp E-pairs, for chunk c ascending (from the group's first E-pair when upper), for the
// group's E-pairs ep ascending (ep <= c when upper),
// for k-step pair pp = 0..3 (k-steps s = 8c + 2pp, +1): the A fragments of E = 2ep and
// E = 2ep + 1, 64 lanes x 16 B each: {W[16E + (l&15)][4s + (l>>4)], same at s+1}.
//   dense: W = K^-1 (leading dim ld);
//   upper: W[e][f] = (K^-1[e][f] + K^-1[f][e]) / 2 for f > e, K^-1[e][e] / 2 for f == e, else 0.
__device__ __forceinline__ long long cm_group_blocks(int nch, int e0, int upper) {
  const int eN = nch - e0 < kCMaxEp ? nch - e0 : kCMaxEp;
  if (!upper) return (long long)nch * eN;
  // chunks e0 .. e0+eN-2 hold 1 .. eN-1 blocks, the nch - e0 - eN + 1 later ones eN each
  return (long long)(eN - 1) * eN / 2 + (long long)(nch - e0 - eN + 1) * eN;
}

__global__ void pack_cm_kernel(d2* __restrict__ out, const double* __restrict__ kinv, long long ld,
                               int upper, int n, int n_pad, int n_obj) {
  const int nch = n_pad / 32;
  long long blocks = 0;
  for (int e0 = 0; e0 < nch; e0 += kCMaxEp) blocks += cm_group_blocks(nch, e0, upper);
  const long long per_obj = blocks * 512;                     // d2 entries (4 pairs x 2 x 64)
  const long long stride_obj = (long long)n_pad * n_pad / 2;  // d2 entries reserved per objective
  for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < per_obj * n_obj;
       t += (long long)gridDim.x * blockDim.x) {
    const int o = (int)(t / per_obj);
    long long r = t - (long long)o * per_obj;
    const int lane = (int)(r & 63); r >>= 6;
    const int which = (int)(r & 1); r >>= 1;
    const int pp = (int)(r & 3); r >>= 2;
    // r = block index: groups of kCMaxEp E-pairs in order; within a group chunks c
    // ascending (dense) or descending (upper), within a chunk the group's E-pairs ascending
    // (ep <= c when upper)
    int e0 = 0;
    for (;; e0 += kCMaxEp) {
      const long long nb = cm_group_blocks(nch, e0, upper);
      if (r < nb) break;
      r -= nb;
    }
    const int eN = nch - e0 < kCMaxEp ? nch - e0 : kCMaxEp;
    int c, el;
    if (!upper) {
      c = (int)(r / eN);
      el = (int)(r % eN);
    } else {
      // upper: chunks DESCENDING (E-pair ep is complete after chunk ep, whose K* is then still
      // in the kernel's registers): full chunks c = nch-1 .. e0+eN-1 (eN blocks each), then
      // partial chunks c = e0+eN-2 .. e0 (eN-1, ..., 1 blocks)
      const long long full = (long long)(nch - (e0 + eN - 1)) * eN;
      if (r < full) {
        c = nch - 1 - (int)(r / eN);
        el = (int)(r % eN);
      } else {
        r -= full;
        int sz = eN - 1;
        while (r >= sz) { r -= sz; --sz; }
        c = e0 + sz - 1;
        el = (int)r;
      }
    }
    const int ep = e0 + el;
    const int row = 16 * (2 * ep + which) + (lane & 15);
    const int s = 8 * c + 2 * pp;
    const int col0 = 4 * s + (lane >> 4), col1 = col0 + 4;
    const double* wo = kinv + (long long)o * ld * ld;
    auto w = [&](int e, int f) -> double {
      if (e >= n || f >= n) return 0.0;
      if (!upper) return wo[(long long)e * ld + f];
      if (f < e) return 0.0;
      if (f == e) return 0.5 * wo[(long long)e * ld + e];
      return 0.5 * (wo[(long long)e * ld + f] + wo[(long long)f * ld + e]);
    };
    d2 v;
    v.x = w(row, col0);
    v.y = w(row, col1);
    out[(long long)o * stride_obj + (t - (long long)o * per_obj)] = v;
  }
}

// Separable-K* precondition on the training rows: last coordinate integral and inside the
// grid's last axis [lo, lo + S - 1] (else *flag = 1 and the kernel keeps the exp path).
__global__ void sep_check_kernel(const double* __restrict__ x, int n, int dim, long long lo, int S,
                                 int* __restrict__ flag) {
  const int f = blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= n) return;
  const double v = x[(long long)f * dim + dim - 1];
  const bool ok = v == __builtin_rint(v) && v >= (double)lo && v <= (double)(lo + S - 1);
  if (!ok) atomicOr(flag, 1);
}

// Training rows / evaluated points padded to [rows_pad][DIM]: coordinates beyond `dim`
// are 0; rows beyond `rows` are `fill` (1e200 puts padded training rows at infinite
// distance so exp() underflows to exactly 0).
__global__ void pad_points_kernel(double* __restrict__ out, const double* __restrict__ in,
                                  int rows, int rows_pad, int dim, int DIM, double fill) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= rows_pad * DIM) return;
  const int r = t / DIM, k = t - r * DIM;
  out[t] = r < rows ? (k < dim ? in[r * dim + k] : 0.0) : fill;
}

// Pack K^-1 into the MFMA fragment order of fused_predict_kernel (N > 512 panels and the
// materialised-K* path), zero padded.  Element (panel, ep, pair, which, lane) holds
// W[16E + (l&15)][4s + (l>>4)] and the same at s+1 (E = 2ep + which, s = panel*ns_panel + 2*pair).
__global__ void pack_kernel(d2* __restrict__ out, const double* __restrict__ kinv, long long ld,
                            int n, int n_pad, int ns_panel, int n_obj) {
  const long long per_obj = (long long)n_pad * n_pad / 2;
  const long long total = per_obj * n_obj;
  const int n_ep = n_pad / 32;
  const int npair = ns_panel / 2;
  for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < total;
       t += (long long)gridDim.x * blockDim.x) {
    const int o = (int)(t / per_obj);
    long long r = t - (long long)o * per_obj;
    const int lane = (int)(r & 63); r >>= 6;
    const int which = (int)(r & 1); r >>= 1;
    const int pair = (int)(r % npair); r /= npair;
    const int ep = (int)(r % n_ep); r /= n_ep;
    const int panel = (int)r;
    const int row = 16 * (2 * ep + which) + (lane & 15);
    const int s = panel * ns_panel + 2 * pair;
    const int col0 = 4 * s + (lane >> 4), col1 = col0 + 4;
    const double* wo = kinv + (long long)o * ld * ld;
    d2 v;
    v.x = (row < n && col0 < n) ? wo[(long long)row * ld + col0] : 0.0;
    v.y = (row < n && col1 < n) ? wo[(long long)row * ld + col1] : 0.0;
    out[t] = v;
  }
}

// alpha[o][f] = sum_e Kinv[o][f][e] * (y[e][o] - pm[o])   (numba_kernels.py:477-483),
// e ascending, zero for padded rows.  One wave per row: lane-strided partial sums then
// a shuffle tree (order differs from BLAS dgemv only in the last bits).
__global__ void alpha_kernel(double* __restrict__ alpha, const double* __restrict__ kinv,
                             long long ld, const double* __restrict__ y, long long ld_y, int n,
                             int n_pad, int n_obj, FusedArgs a) {
  const int lane = threadIdx.x & 63;
  const long long row_id = blockIdx.x * (long long)(blockDim.x / 64) + (threadIdx.x >> 6);
  if (row_id >= (long long)n_obj * n_pad) return;
  const int o = (int)(row_id / n_pad), f = (int)(row_id % n_pad);
  double s = 0.0;
  if (f < n) {
    const double* wr = kinv + (long long)o * ld * ld + (long long)f * ld;
    const double pm = a.pm[o];
    for (int e = lane; e < n; e += 64) s = __builtin_fma(wr[e], y[(long long)e * ld_y + o] - pm, s);
  }
#pragma unroll
  for (int m = 32; m > 0; m >>= 1) s += __shfl_xor(s, m, 64);
  if (lane == 0) alpha[row_id] = s;
}

// Merge the per-wave lists [n_lists][q] into the final top-q (one workgroup, 16 waves).
__global__ __launch_bounds__(1024) void topq_merge_kernel(const TopEntry* __restrict__ lists,
                                                          int n_lists, int q,
                                                          double* __restrict__ out_v,
                                                          long long* __restrict__ out_i) {
  __shared__ TopEntry stage[16 * BO_MAX_TOPQ];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  double lv = -__builtin_inf();
  long long li = -1;
  const long long total = (long long)n_lists * q;
  for (long long base = (long long)wave * 16; base < total; base += (long long)nw * 16) {
    double nv = -__builtin_inf();
    long long ni = -1;
    if (lane < 16 && base + lane < total) { nv = lists[base + lane].v; ni = lists[base + lane].i; }
    bo_wave_topq_insert(lv, li, nv, ni, q);
  }
  if (lane < q) { stage[wave * q + lane].v = lv; stage[wave * q + lane].i = li; }
  __syncthreads();
  if (wave == 0) {
    double fv = -__builtin_inf();
    long long fi = -1;
    for (int base = 0; base < nw * q; base += 16) {
      double nv = -__builtin_inf();
      long long ni = -1;
      if (lane < 16 && base + lane < nw * q) { nv = stage[base + lane].v; ni = stage[base + lane].i; }
      bo_wave_topq_insert(fv, fi, nv, ni, q);
    }
    if (lane < q) { out_v[lane] = fv; out_i[lane] = fi; }
  }
}

// Small q (<= 16): q rounds of a workgroup-wide arg-best over all list entries held in
// registers (<= 8 per thread), instead of bitonic inserts: a few shuffle reductions per round.
__global__ __launch_bounds__(1024) void topq_argbest_kernel(const TopEntry* __restrict__ lists,
                                                            int n_lists, int q,
                                                            double* __restrict__ out_v,
                                                            long long* __restrict__ out_i) {
  __shared__ TopEntry wbest[16];
  __shared__ TopEntry win;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nw = blockDim.x >> 6;
  const long long total = (long long)n_lists * q;
  double v[8];
  long long ix[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const long long at = tid + (long long)k * blockDim.x;
    v[k] = -__builtin_inf();
    ix[k] = -1;
    if (at < total) { v[k] = lists[at].v; ix[k] = lists[at].i; }
  }
  for (int r = 0; r < q; ++r) {
    double bv = -__builtin_inf();
    long long bi = -1;
#pragma unroll
    for (int k = 0; k < 8; ++k)
      if (bo_better(v[k], ix[k], bv, bi)) { bv = v[k]; bi = ix[k]; }
#pragma unroll
    for (int m = 32; m > 0; m >>= 1) {
      const double ov = __shfl_xor(bv, m, 64);
      const long long oi = __shfl_xor(bi, m, 64);
      if (bo_better(ov, oi, bv, bi)) { bv = ov; bi = oi; }
    }
    if (lane == 0) { wbest[wave].v = bv; wbest[wave].i = bi; }
    __syncthreads();
    if (wave == 0) {
      bv = lane < nw ? wbest[lane].v : -__builtin_inf();
      bi = lane < nw ? wbest[lane].i : -1;
#pragma unroll
      for (int m = 32; m > 0; m >>= 1) {
        const double ov = __shfl_xor(bv, m, 64);
        const long long oi = __shfl_xor(bi, m, 64);
        if (bo_better(ov, oi, bv, bi)) { bv = ov; bi = oi; }
      }
      if (lane == 0) {
        win.v = bv;
        win.i = bi;
        out_v[r] = bv;
        out_i[r] = bi;
      }
    }
    __syncthreads();
    // retire the winner (global candidate indices are unique across the lists)
    const long long wi = win.i;
#pragma unroll
    for (int k = 0; k < 8; ++k)
      if (wi >= 0 && ix[k] == wi) { v[k] = -__builtin_inf(); ix[k] = -1; }
    __syncthreads();
  }
}

__global__ void selftest_mfma_kernel(const double* a, const double* b, double* d) {
  const int l = threadIdx.x;
  const double av = a[(l & 15) * 4 + (l >> 4)];  // A[i=l&15][k=l>>4]
  const double bv = b[(l >> 4) * 16 + (l & 15)]; // B[k=l>>4][j=l&15]
  d4 acc = {0.0, 0.0, 0.0, 0.0};
  acc = mfma64(av, bv, acc);
#pragma unroll
  for (int r = 0; r < 4; ++r) d[((l >> 4) + 4 * r) * 16 + (l & 15)] = acc[r];
}

// ---------------------------------------------------------------------------------------
// fp32 variant (BO_PREDICT_FP32; BASELINE config C5 "fp32 with fp64 reference check"):
// the upper form q = 2 k.(U k) on v_mfma_f32_16x16x4_f32 (32 cycles per MFMA per SIMD, twice
// the f64 rate), K* = 2^(nhl log2e |x_f - c_j|^2 + log2 pv) on v_exp_f32, mu / q accumulated
// in f32 and everything after them (variance floor, standardisation, UCB, sum, top-q) in f64.
//
// Body = E-quad: 64 rows of U (4 MFMA row blocks b), chunk = 64 rows of K* (16 k-steps).
// f32 D layout (lane l holds D[4 (l >> 4) + r][l & 15]) differs from f64's, so the K* row fed
// at k-step s by lane group g is permuted: f(s, g) = 64 c + 16 (s >> 2) + 4 g + (s & 3).  Then
// the rows a completing E-quad's accumulator block b holds in its lane (64 ep + 16 b + 4 g + r)
// are exactly B slots s = 4 b + r of chunk ep: the in-register epilogue of the f64 kernel.
// Chunks descend (E-quad ep is complete at chunk ep); W streams per (group, chunk, E-quad,
// k-quad kq, block b) as one 16-B float4 per lane (k-steps 4 kq .. 4 kq + 3), through a
// 16-entry register ring that holds exactly one E-quad block (static slot indices).
// Exclusion of evaluated points is tested (exactly, in f64 from HBM) only for candidates that
// would enter the wave's top-q.
// ---------------------------------------------------------------------------------------
typedef float f4 __attribute__((ext_vector_type(4)));
constexpr int kC32MaxEp = 16;   // E-quads per group (1024 rows)

__device__ __forceinline__ f4 mfma32(float a, float b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f4 wload32(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
  return __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0));
}
__device__ __forceinline__ void mfma_fence32(f4& a, f4& b, f4& c, f4& d) {
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7"
               : "+a"(a), "+a"(b), "+a"(c), "+a"(d));
}

// (chunk, E-quad) blocks of group e0, upper form
__host__ __device__ inline long long c32_group_blocks(int nch, int e0) {
  const int eN = nch - e0 < kC32MaxEp ? nch - e0 : kC32MaxEp;
  return (long long)(eN - 1) * eN / 2 + (long long)(nch - e0 - eN + 1) * eN;
}
__host__ __device__ inline long long c32_blocks(int nch) {
  long long b = 0;
  for (int e0 = 0; e0 < nch; e0 += kC32MaxEp) b += c32_group_blocks(nch, e0);
  return b;
}

// float4 entry (o, block, kq, b, lane) = {W[row][col0 + t], t = 0..3}, row = 64 ep + 16 b +
// (lane & 15), col0 = 64 c + 16 kq + 4 (lane >> 4); W = triu(sym(K^-1)) with halved diagonal.
__global__ void pack32_kernel(f4* __restrict__ out, const double* __restrict__ kinv, long long ld,
                              int n, int n_pad, int n_obj) {
  const int nch = n_pad / 64;
  const long long per_obj = c32_blocks(nch) * 1024;
  for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < per_obj * n_obj;
       t += (long long)gridDim.x * blockDim.x) {
    const int o = (int)(t / per_obj);
    long long r = t - (long long)o * per_obj;
    const int lane = (int)(r & 63); r >>= 6;
    const int b = (int)(r & 3); r >>= 2;
    const int kq = (int)(r & 3); r >>= 2;
    int e0 = 0;
    for (;; e0 += kC32MaxEp) {
      const long long nb = c32_group_blocks(nch, e0);
      if (r < nb) break;
      r -= nb;
    }
    const int eN = nch - e0 < kC32MaxEp ? nch - e0 : kC32MaxEp;
    int c, el;
    const long long full = (long long)(nch - (e0 + eN - 1)) * eN;
    if (r < full) {
      c = nch - 1 - (int)(r / eN);
      el = (int)(r % eN);
    } else {
      r -= full;
      int sz = eN - 1;
      while (r >= sz) { r -= sz; --sz; }
      c = e0 + sz - 1;
      el = (int)r;
    }
    const int row = 64 * (e0 + el) + 16 * b + (lane & 15);
    const int col0 = 64 * c + 16 * kq + 4 * (lane >> 4);
    const double* wo = kinv + (long long)o * ld * ld;
    f4 v;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int f = col0 + q;
      double w = 0.0;
      if (row < n && f < n && f >= row)
        w = f == row ? 0.5 * wo[(long long)row * ld + row]
                     : 0.5 * (wo[(long long)row * ld + f] + wo[(long long)f * ld + row]);
      v[q] = (float)w;
    }
    out[(size_t)o * per_obj + (t - (long long)o * per_obj)] = v;
  }
}

template <int DIM>
__global__ __launch_bounds__(256, 1) void cm32_predict_kernel(const FusedArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem32[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, jl = lane & 15;
  float* xs = smem32;                                        // [n_pad][DIM]
  float* al = xs + (size_t)a.n_pad * DIM;                    // [n_obj][n_pad]
  for (int t = tid; t < a.n_pad * DIM; t += blockDim.x) xs[t] = (float)a.xpad[t];   // 1e200 -> inf
  for (int t = tid; t < a.n_obj * a.n_pad; t += blockDim.x) al[t] = (float)a.alpha[t];
  __syncthreads();
  const int nch = a.n_pad / 64;
  const long long w_obj = c32_blocks(nch) * 1024 * 16;       // bytes per objective
  const __amdgpu_buffer_rsrc_t wr =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.wpack, (short)0, (int)a.wpack_bytes, 0x00020000);
  const int voff = lane * 16;
  const double* es = a.excl ? a.excl : a.xpad;               // f64 [*][DIM] (exact equality)
  const int ne = a.excl ? a.n_excl : a.n_train;
  double top_v = -__builtin_inf();
  long long top_i = -1;
  for (long long tile = blockIdx.x; tile < a.n_tiles; tile += gridDim.x) {
    const long long j = tile * kTile + wave * 16 + jl;
    const bool valid = j < a.n_cand;
    double c[DIM];
    load_candidate<DIM>(a, j, valid, c);
    float c32[DIM];
#pragma unroll
    for (int k = 0; k < DIM; ++k) c32[k] = (float)c[k];
    double acq = 0.0;
    for (int o = 0; o < a.n_obj; ++o) {
      const float nl2 = (float)(a.nhl[o] * 1.4426950408889634);
      const float lpv = (float)log2(a.pv[o]);
      auto kval = [&](int f) -> float {
        const float* r = xs + f * DIM;
        float d2 = 0.0f;
#pragma unroll
        for (int k = 0; k < DIM; ++k) { const float d = r[k] - c32[k]; d2 = __builtin_fmaf(d, d, d2); }
        return __builtin_amdgcn_exp2f(__builtin_fmaf(d2, nl2, lpv));
      };
      auto chunk = [&](int ch, float (&B)[16]) {
#pragma unroll
        for (int s = 0; s < 16; ++s) B[s] = kval(64 * ch + 16 * (s >> 2) + 4 * g + (s & 3));
      };
      const float* alo = al + (size_t)o * a.n_pad;
      const int base = (int)(o * w_obj);
      f4 w[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) w[q] = wload32(wr, voff, base + q * 1024);
      int pos = 0;
      float mpart = 0.0f, qpart = 0.0f;
      f4 acc[kC32MaxEp][4];
      for (int e0 = 0; e0 < nch; e0 += kC32MaxEp) {
        const int eN = nch - e0 < kC32MaxEp ? nch - e0 : kC32MaxEp;
#pragma unroll
        for (int e = 0; e < kC32MaxEp; ++e)
#pragma unroll
          for (int b = 0; b < 4; ++b) acc[e][b] = (f4){0.0f, 0.0f, 0.0f, 0.0f};
        const bool mu_on = e0 == 0;
        auto chunk_step = [&](int ch, const float (&B)[16], float (&Bn)[16]) {
          const int chn = ch > e0 ? ch - 1 : ch;
          const int n_here = ch - e0 + 1 < eN ? ch - e0 + 1 : eN;
          auto ep_body = [&](auto e_c) {
            constexpr int e = decltype(e_c)::value;
            // keep the workgroup's 4 waves on the same E-quad block: they stream identical W
            // data, so the lockstep turns 3 of 4 L2 reads into L1 hits (C5: W = 8.6 MB per
            // objective does not fit an XCD's L2; measured 141 -> 108 ms per 2^20 candidates)
            __builtin_amdgcn_s_barrier();
            if constexpr (e == 0) {
              // branch-free (a join here would drain the W ring with vmcnt(0))
#pragma unroll
              for (int s = 0; s < 16; ++s) {
                const float av = alo[64 * ch + 16 * (s >> 2) + 4 * g + (s & 3)];
                mpart = __builtin_fmaf(mu_on ? av : 0.0f, B[s], mpart);
              }
              chunk(chn, Bn);
            }
#pragma unroll
            for (int kq = 0; kq < 4; ++kq) {
#pragma unroll
              for (int t = 0; t < 4; ++t)
#pragma unroll
                for (int b = 0; b < 4; ++b) acc[e][b] = mfma32(w[4 * kq + b][t], B[4 * kq + t], acc[e][b]);
              const int so = base + (pos + 1) * 16384 + kq * 4096;
#pragma unroll
              for (int b = 0; b < 4; ++b) w[4 * kq + b] = wload32(wr, voff, so + b * 1024);
            }
            ++pos;
            if (ch - e0 == e) {
              mfma_fence32(acc[e][0], acc[e][1], acc[e][2], acc[e][3]);
#pragma unroll
              for (int b = 0; b < 4; ++b)
#pragma unroll
                for (int r = 0; r < 4; ++r) qpart = __builtin_fmaf(B[4 * b + r], acc[e][b][r], qpart);
            }
          };
          EpChain<0, kC32MaxEp>::run(ep_body, n_here);
        };
        float BX[16], BY[16];
        chunk(nch - 1, BX);
        int ch = nch - 1;
        for (; ch - 1 >= e0; ch -= 2) {
          chunk_step(ch, BX, BY);
          chunk_step(ch - 1, BY, BX);
        }
        if (ch >= e0) chunk_step(ch, BX, BY);
      }
      qpart += __shfl_xor(qpart, 16, 64);
      qpart += __shfl_xor(qpart, 32, 64);
      mpart += __shfl_xor(mpart, 16, 64);
      mpart += __shfl_xor(mpart, 32, 64);
      const double pv = a.pv[o], pm = a.pm[o];
      const double mu = pm + (double)mpart;                               // :486-488
      const double var = fmax(pv - 2.0 * (double)qpart, BO_MIN_VARIANCE);  // :532-535
      const double smu = (mu - pm) / a.rsq_pv[o];                         // :563-565
      const double svar = var / pv;                                       // :568-570
      const double u = smu + a.beta[o] * sqrt(fabs(svar));                // acquisition.py:52
      acq = (o == 0) ? u : acq + u;                                       // acquisition.py:108
      if (valid && g == 0) {
        const long long off = (long long)o * a.ld_out + j;
        if (a.mu) a.mu[off] = mu;
        if (a.var) a.var[off] = var;
        if (a.std_mu) a.std_mu[off] = smu;
        if (a.std_var) a.std_var[off] = svar;
        if (a.ucb) a.ucb[off] = u;
      }
    }
    if (valid && g == 0 && a.acq) a.acq[j] = acq;
    if (a.topq > 0) {
      long long gi = valid ? a.cand_offset + j : -1;
      const double tv = __shfl(top_v, a.topq - 1, 64);
      const long long ti = __shfl(top_i, a.topq - 1, 64);
      const bool need = gi >= 0 && bo_better(acq, gi, tv, ti);
      if (__ballot(need) != 0ull) {
        // acquisition.py:137-139, exact f64 coordinates; lane group g checks points g, g+4, ...
        bool hit = false;
        for (int e = g; e < ne; e += 4) {
          const double* r = es + (size_t)e * DIM;
          bool eq = true;
#pragma unroll
          for (int k = 0; k < DIM; ++k) eq = eq && (r[k] == c[k]);
          hit = hit || eq;
        }
        const unsigned long long hb = __ballot(hit);
        if (((hb >> jl) | (hb >> (jl + 16)) | (hb >> (jl + 32)) | (hb >> (jl + 48))) & 1ull) gi = -1;
      }
      bo_wave_topq_insert(top_v, top_i, acq, gi, a.topq);
    }
  }
  BO_WAIT_VMCNT(0);                                          // no W load in flight at exit
  if (a.topq > 0 && lane < a.topq) {
    TopEntry* dst = a.partial + ((size_t)blockIdx.x * kWaves + wave) * a.topq;
    dst[lane].v = top_v;
    dst[lane].i = top_i;
  }
}

__global__ void selftest_mfma32_kernel(const float* a, const float* b, float* d) {
  const int l = threadIdx.x;
  const float av = a[(l & 15) * 4 + (l >> 4)];   // A[i=l&15][k=l>>4]
  const float bv = b[(l >> 4) * 16 + (l & 15)];  // B[k=l>>4][j=l&15]
  f4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
  acc = mfma32(av, bv, acc);
#pragma unroll
  for (int r = 0; r < 4; ++r) d[(4 * (l >> 4) + r) * 16 + (l & 15)] = acc[r];
}

inline int pad_rows(long long n) { return (int)((n + 31) / 32 * 32); }
inline int pad_dim(int d) { return d <= 2 ? 2 : (d <= 4 ? 4 : (d <= 6 ? 6 : 8)); }
inline size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

struct Plan {
  int n_pad, ns, n_panels, dim_pad, n_excl;
  bool multi;
  size_t off_alpha, off_xpad, off_excl, off_partial, off_chol, off_status, total;
  bool cm;               // chunk-major kernel (cm_predict_kernel)
  bool sep;              // ... with the integer-grid K* generation
  int off_tbl, off_rw;   // LDS offsets in doubles
  bool rw_cache;          // SEP row factors cached per objective
  bool fp32;              // cm32_predict_kernel (BO_PREDICT_FP32)
  int off_sq;             // LDS offset (doubles) of |x_f|^2 for the dot-form exponent, 0 = off
  int grid, waves;       // persistent grid, waves per workgroup
  long long n_tiles;
  size_t lds;
};

int num_cus() {
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 256;
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, dev) != hipSuccess) return 256;
    cus = p.multiProcessorCount;
  }
  return cus;
}

int make_plan(const bo_predict_desc* d, Plan* pl, bool query_device, bool kmem = false) {
  if (!d || d->n_obj < 1 || d->n_obj > BO_MAX_OBJ || d->dim < 1 || d->dim > BO_MAX_DIM)
    return BO_ERR_ARG;
  if (d->n_train < 1 || d->n_cand < 0 || d->topq < 0 || d->topq > BO_MAX_TOPQ) return BO_ERR_ARG;
  if (d->cand_kind < 0 || d->cand_kind > 2) return BO_ERR_ARG;
  if (d->mode & ~(BO_PREDICT_DENSE | BO_PREDICT_NO_SEPARABLE | BO_PREDICT_FP32)) return BO_ERR_ARG;
  if (d->excl_points && d->n_excl < 0) return BO_ERR_ARG;
  const long long n = d->n_train;
  if (n > (1 << 14)) return BO_ERR_UNSUPPORTED;
  pl->dim_pad = pad_dim(d->dim);
  pl->n_excl = (int)(d->excl_points ? d->n_excl : n);
  const size_t excl_lds = d->excl_points ? (size_t)pl->n_excl * pl->dim_pad : 0;
  // chunk-major kernel (cm_predict_kernel) for N <= 512; on the reference's 'ij' grid with
  // 16-aligned rows it generates K* from per-row factors and an exp table (pl->sep)
  pl->sep = false;
  pl->fp32 = false;
  pl->off_sq = 0;
  pl->rw_cache = false;
  pl->cm = false;
  pl->off_tbl = pl->off_rw = 0;
  pl->fp32 = (d->mode & BO_PREDICT_FP32) && !kmem;
  if (pl->fp32) {
    const int n_pad = (int)((n + 63) / 64 * 64);
    pl->n_pad = n_pad;
    pl->ns = 16;
    pl->multi = false;
    pl->n_panels = 1;
    pl->lds = ((size_t)n_pad * pl->dim_pad + (size_t)d->n_obj * n_pad) * sizeof(float);
    if (pl->lds > 160 * 1024) return BO_ERR_UNSUPPORTED;
  } else if (!kmem) {
    const int n_pad = pad_rows(n);
    const size_t base = (size_t)n_pad * pl->dim_pad + (size_t)d->n_obj * n_pad + excl_lds;
    pl->cm = true;
    pl->n_pad = n_pad;
    pl->ns = n_pad / 4;
    pl->multi = false;
    pl->n_panels = 1;
    pl->lds = base * sizeof(double);
    if (pl->lds > 160 * 1024) return BO_ERR_UNSUPPORTED;
    if (d->cand_kind == BO_CAND_GRID && !(d->mode & BO_PREDICT_NO_SEPARABLE)) {
      const long long S = d->grid_shape[d->dim - 1];
      const size_t tbl = (size_t)d->n_obj * (2 * S - 1);
      // per wave: n_obj (cached) or 1 slot of row factors + the int index / on-row arrays
      const size_t lds_c = base + tbl + (size_t)kWaves * n_pad * (d->n_obj + 1);
      const size_t lds_1 = base + tbl + (size_t)kWaves * n_pad * 2;
      if (S % 16 == 0 && S <= 32768 && d->cand_offset % 16 == 0 && lds_1 * sizeof(double) <= 160 * 1024) {
        pl->sep = true;
        pl->rw_cache = lds_c * sizeof(double) <= 160 * 1024;
        pl->off_tbl = (int)base;
        pl->off_rw = (int)(base + tbl);
        pl->lds = (pl->rw_cache ? lds_c : lds_1) * sizeof(double);
      }
    }
    // explicit candidates, upper form: |x_f|^2 per training row for the dot-form exponent
    if (d->cand_kind != BO_CAND_GRID && !(d->mode & BO_PREDICT_DENSE) &&
        (base + n_pad) * sizeof(double) <= 160 * 1024) {
      pl->off_sq = (int)base;
      pl->lds = (base + n_pad) * sizeof(double);
    }
  }
  if (!pl->cm && !pl->fp32) {
    int n_pad = pad_rows(n);
    int ns;
    bool multi = false;
    if (n_pad <= 32) ns = 8;
    else if (n_pad <= 64) ns = 16;
    else if (n_pad <= 128) ns = 32;
    else if (n_pad <= 256) ns = 64;
    else if (n_pad <= 384 && !kmem) ns = 96;
    else if (n_pad <= 512 && !kmem) ns = 128;
    else { ns = kPanelSteps; multi = true; }   // (materialised-K* path: panels above 256 rows)
    n_pad = multi ? (int)((n + 511) / 512 * 512) : ns * 4;
    pl->n_pad = n_pad;
    pl->ns = ns;
    pl->multi = multi;
    pl->n_panels = multi ? n_pad / 512 : 1;
    pl->lds = ((size_t)n_pad * pl->dim_pad + (size_t)d->n_obj * n_pad + excl_lds) * sizeof(double);
    if (pl->lds > 160 * 1024) return BO_ERR_UNSUPPORTED;
  }
  const int n_pad = pl->n_pad;
  const bool multi = pl->multi;
  const size_t w_bytes = (size_t)d->n_obj * n_pad * n_pad * sizeof(double);
  if (w_bytes >= (1ull << 31)) return BO_ERR_UNSUPPORTED;
  pl->waves = kWaves;
  const long long n_tiles = (d->n_cand + kTile - 1) / kTile;
  pl->n_tiles = n_tiles;
  const int cus = query_device ? num_cus() : 256;
  pl->grid = (int)(n_tiles < cus ? (n_tiles > 0 ? n_tiles : 1) : cus);
  pl->off_alpha = align256(w_bytes);
  pl->off_xpad = pl->off_alpha + align256((size_t)d->n_obj * n_pad * sizeof(double));
  pl->off_excl = pl->off_xpad + align256((size_t)n_pad * pl->dim_pad * sizeof(double));
  pl->off_partial = pl->off_excl + align256((size_t)(pl->n_excl + 1) * pl->dim_pad * sizeof(double));
  // partial lists sized for the largest persistent grid any device could use
  pl->off_chol = pl->off_partial +
                 align256((size_t)1024 * kWaves * (d->topq > 0 ? d->topq : 1) * sizeof(TopEntry));
  pl->off_status = pl->off_chol;
  pl->total = pl->off_status + 256 + 256;   // +0: tri status, +16: separable-K* status
  return BO_OK;
}

template <int NS, int DIM, bool MULTI, bool KMEM = false>
hipError_t launch_fused(const FusedArgs& fa, int grid, size_t lds, hipStream_t st) {
  auto k = fused_predict_kernel<NS, DIM, MULTI, KMEM>;
  if (lds > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)lds);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(k, dim3(grid), dim3(256), lds, st, fa);
  return hipGetLastError();
}

// Optional timing of the fused kernel itself (bench.py's roofline): when enabled, every
// fused launch is bracketed by a pair of HIP events on its stream.
struct KernelTimer {
  bool on = false;
  int used = 0;
  std::vector<hipEvent_t> ev;
} g_timer;

void timer_mark(hipStream_t s) {
  if (!g_timer.on || g_timer.used >= (int)g_timer.ev.size()) return;
  (void)hipEventRecord(g_timer.ev[g_timer.used++], s);
}

template <int DIM, bool GRID, bool UPPER>
hipError_t launch_cm_k(const FusedArgs& fa, int grid, size_t lds, hipStream_t st) {
  auto k = cm_predict_kernel<DIM, GRID, UPPER>;
  if (lds > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)lds);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(k, dim3(grid), dim3(256), lds, st, fa);
  return hipGetLastError();
}

template <int DIM>
hipError_t launch_cm(const Plan& pl, const FusedArgs& fa, hipStream_t st) {
  if (fa.upper)
    return pl.sep ? launch_cm_k<DIM, true, true>(fa, pl.grid, pl.lds, st)
                  : launch_cm_k<DIM, false, true>(fa, pl.grid, pl.lds, st);
  return pl.sep ? launch_cm_k<DIM, true, false>(fa, pl.grid, pl.lds, st)
                : launch_cm_k<DIM, false, false>(fa, pl.grid, pl.lds, st);
}

template <int DIM>
hipError_t launch_c32(const Plan& pl, const FusedArgs& fa, hipStream_t st) {
  auto k = cm32_predict_kernel<DIM>;
  if (pl.lds > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)pl.lds);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(k, dim3(pl.grid), dim3(256), pl.lds, st, fa);
  return hipGetLastError();
}

hipError_t launch_kmem(const Plan& pl, const FusedArgs& fa, hipStream_t s) {
  if (pl.multi) return launch_fused<kPanelSteps, 2, true, true>(fa, pl.grid, pl.lds, s);
  switch (pl.ns) {
    case 8: return launch_fused<8, 2, false, true>(fa, pl.grid, pl.lds, s);
    case 16: return launch_fused<16, 2, false, true>(fa, pl.grid, pl.lds, s);
    case 32: return launch_fused<32, 2, false, true>(fa, pl.grid, pl.lds, s);
    default: return launch_fused<64, 2, false, true>(fa, pl.grid, pl.lds, s);
  }
}

}  // namespace

extern "C" {

size_t bo_predict_workspace_size(const bo_predict_desc* d) {
  Plan pl;
  if (make_plan(d, &pl, false) != BO_OK) return 0;
  return pl.total;
}

static int predict_impl(const bo_predict_desc* d, const double* kstar, long long ks_rows,
                        void* workspace, size_t ws_bytes, void* stream) {
  const bool kmem = kstar != nullptr;
  Plan pl;
  int st = make_plan(d, &pl, true, kmem);
  if (st != BO_OK) return st;
  if (!workspace || ws_bytes < pl.total) return BO_ERR_WORKSPACE;
  if ((!kmem && !d->x_train) || !d->y_train || !d->kinv || d->ld_k < d->n_train ||
      d->ld_y < d->n_obj)
    return BO_ERR_ARG;
  if (d->cand_kind != BO_CAND_GRID && d->n_cand > 0 && !d->cand) return BO_ERR_ARG;
  if (d->topq > 0 && (!d->top_val || !d->top_idx)) return BO_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;

  char* ws = (char*)(((uintptr_t)workspace + 255) & ~(uintptr_t)255);
  d2* wpack = (d2*)ws;
  double* alpha = (double*)(ws + pl.off_alpha);
  double* xpad = (double*)(ws + pl.off_xpad);
  double* excl = (double*)(ws + pl.off_excl);
  TopEntry* partial = (TopEntry*)(ws + pl.off_partial);

  FusedArgs fa;
  memset(&fa, 0, sizeof(fa));
  fa.n_obj = d->n_obj;
  fa.dim = d->dim;
  fa.n_train = (int)d->n_train;
  fa.n_pad = pl.n_pad;
  fa.n_panels = pl.n_panels;
  fa.n_excl = pl.n_excl;
  fa.cand_kind = d->cand_kind;
  fa.topq = d->topq;
  fa.n_cand = d->n_cand;
  fa.cand_offset = d->cand_offset;
  fa.ld_out = d->ld_out > 0 ? d->ld_out : d->n_cand;
  fa.n_tiles = pl.n_tiles;
  for (int k = 0; k < BO_MAX_DIM; ++k) {
    fa.grid_lo[k] = d->grid_lo[k];
    fa.grid_shape[k] = d->grid_shape[k] > 0 ? d->grid_shape[k] : 1;
  }
  if (d->cand_kind == BO_CAND_GRID) {
    long long total = 1;
    for (int k = 0; k < d->dim; ++k) {
      if (d->grid_shape[k] <= 0) return BO_ERR_ARG;
      total *= d->grid_shape[k];
    }
    if (d->cand_offset < 0 || d->cand_offset + d->n_cand > total) return BO_ERR_ARG;
  }
  fa.cand = d->cand;
  fa.xpad = xpad;
  fa.excl = d->excl_points ? excl : nullptr;
  fa.wpack = wpack;
  fa.wpack_bytes = (unsigned int)((size_t)d->n_obj * pl.n_pad * pl.n_pad * sizeof(double));
  fa.alpha = alpha;
  for (int o = 0; o < d->n_obj; ++o) {
    fa.pm[o] = d->prior_mean[o];
    fa.pv[o] = d->prior_var[o];
    const double ls = d->length_scale[o];
    fa.nhl[o] = -0.5 / (ls * ls);
    fa.beta[o] = d->beta[o];
    fa.rsq_pv[o] = sqrt(d->prior_var[o]);
  }
  fa.mu = d->mu;
  fa.var = d->var;
  fa.std_mu = d->std_mu;
  fa.std_var = d->std_var;
  fa.ucb = d->ucb;
  fa.acq = d->acq;
  fa.partial = partial;
  fa.kstar = kstar;
  fa.ks_rows = ks_rows;

  fa.upper = (pl.cm && !(d->mode & BO_PREDICT_DENSE)) ? 1 : 0;
  int* sep_flag = (int*)(ws + pl.off_status + 16);
  fa.sep_flag = pl.sep ? sep_flag : nullptr;
  fa.sep_S = pl.sep ? (int)d->grid_shape[d->dim - 1] : 1;
  fa.sep_lo = pl.sep ? d->grid_lo[d->dim - 1] : 0;
  fa.off_tbl = pl.off_tbl;
  fa.off_rw = pl.off_rw;
  fa.rw_cache = pl.rw_cache ? 1 : 0;
  fa.off_sq = pl.off_sq;
  if (pl.sep) {
    BO_CHECK_HIP(hipMemsetAsync(sep_flag, 0, sizeof(int), s));
    hipLaunchKernelGGL(sep_check_kernel, dim3((unsigned)((d->n_train + 255) / 256)), dim3(256), 0, s,
                       d->x_train, (int)d->n_train, d->dim, (long long)fa.sep_lo, fa.sep_S, sep_flag);
    BO_CHECK_HIP(hipGetLastError());
  }
  {
    const long long total = (long long)d->n_obj * pl.n_pad * pl.n_pad / 2;
    const int blocks = (int)((total + 255) / 256 < 4096 ? (total + 255) / 256 : 4096);
    if (pl.fp32)
      hipLaunchKernelGGL(pack32_kernel, dim3(blocks), dim3(256), 0, s, (f4*)wpack, d->kinv, d->ld_k,
                         (int)d->n_train, pl.n_pad, d->n_obj);
    else if (pl.cm)
      hipLaunchKernelGGL(pack_cm_kernel, dim3(blocks), dim3(256), 0, s, wpack, d->kinv, d->ld_k, fa.upper,
                         (int)d->n_train, pl.n_pad, d->n_obj);
    else
      hipLaunchKernelGGL(pack_kernel, dim3(blocks), dim3(256), 0, s, wpack, d->kinv, d->ld_k,
                         (int)d->n_train, pl.n_pad, pl.ns, d->n_obj);
    BO_CHECK_HIP(hipGetLastError());
    const long long rows = (long long)d->n_obj * pl.n_pad;
    hipLaunchKernelGGL(alpha_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, s, alpha,
                       d->kinv, d->ld_k, d->y_train, d->ld_y, (int)d->n_train, pl.n_pad,
                       d->n_obj, fa);
    BO_CHECK_HIP(hipGetLastError());
    int cnt = kmem ? 0 : pl.n_pad * pl.dim_pad;
    if (cnt > 0) hipLaunchKernelGGL(pad_points_kernel, dim3((cnt + 255) / 256), dim3(256), 0, s, xpad,
                       d->x_train, (int)d->n_train, pl.n_pad, d->dim, pl.dim_pad, 1e200);
    BO_CHECK_HIP(hipGetLastError());
    cnt = (kmem || !d->excl_points) ? 0 : pl.n_excl * pl.dim_pad;
    if (cnt > 0) {
      hipLaunchKernelGGL(pad_points_kernel, dim3((cnt + 255) / 256), dim3(256), 0, s, excl,
                         d->excl_points ? d->excl_points : d->x_train, pl.n_excl, pl.n_excl,
                         d->dim, pl.dim_pad, 0.0);
      BO_CHECK_HIP(hipGetLastError());
    }
  }
  if (d->n_cand == 0) {
    if (d->topq > 0) {
      BO_CHECK_HIP(hipMemsetAsync(d->top_idx, 0xff, sizeof(int64_t) * d->topq, s));
    }
    return BO_OK;
  }
  hipError_t e;
  const bool timed = g_timer.on && g_timer.used + 2 <= (int)g_timer.ev.size();
  if (timed) timer_mark(s);
  if (kmem) e = launch_kmem(pl, fa, s);
  else if (pl.fp32) switch (pl.dim_pad) {
    case 2: e = launch_c32<2>(pl, fa, s); break;
    case 4: e = launch_c32<4>(pl, fa, s); break;
    case 6: e = launch_c32<6>(pl, fa, s); break;
    default: e = launch_c32<8>(pl, fa, s); break;
  }
  else if (pl.cm) switch (pl.dim_pad) {
    case 2: e = launch_cm<2>(pl, fa, s); break;
    case 4: e = launch_cm<4>(pl, fa, s); break;
    case 6: e = launch_cm<6>(pl, fa, s); break;
    default: e = launch_cm<8>(pl, fa, s); break;
  }
  else return BO_ERR_UNSUPPORTED;
  if (e != hipSuccess) return BO_ERR_HIP;
  if (timed) timer_mark(s);
  if (d->topq > 0) {
    const int n_lists = pl.grid * pl.waves;
    if (d->topq <= 16 && (long long)n_lists * d->topq <= 8 * 1024)
      hipLaunchKernelGGL(topq_argbest_kernel, dim3(1), dim3(1024), 0, s, partial, n_lists,
                         d->topq, d->top_val, (long long*)d->top_idx);
    else
      hipLaunchKernelGGL(topq_merge_kernel, dim3(1), dim3(1024), 0, s, partial, n_lists,
                         d->topq, d->top_val, (long long*)d->top_idx);
    BO_CHECK_HIP(hipGetLastError());
  }
  return BO_OK;
}

int bo_predict_acquire(const bo_predict_desc* d, void* workspace, size_t ws_bytes, void* stream) {
  return predict_impl(d, nullptr, 0, workspace, ws_bytes, stream);
}

static void fill_mv_desc(bo_predict_desc* d, int32_t n_obj, int64_t n_cand, int64_t n) {
  memset(d, 0, sizeof(*d));
  d->n_obj = n_obj;
  d->dim = 1;
  d->n_train = n;
  d->cand_kind = BO_CAND_GRID;
  d->n_cand = n_cand;
  d->grid_shape[0] = n_cand > 0 ? n_cand : 1;
  d->n_excl = 0;
  d->mode = BO_PREDICT_DENSE;
}

size_t bo_update_mean_variance_workspace_size(int32_t n_obj, int64_t current_eval) {
  bo_predict_desc d;
  fill_mv_desc(&d, n_obj, 0, current_eval);
  d.excl_points = (const double*)1;  // no exclusion set
  Plan pl;
  if (make_plan(&d, &pl, false, true) != BO_OK) return 0;
  return pl.total;
}

int bo_update_mean_variance(double* mu, double* var, const double* k_star, int64_t ld_rows,
                            int32_t n_obj, int64_t n_cand, const double* kinv, int64_t ld_k,
                            const double* y, int64_t ld_y, int64_t current_eval,
                            const double* prior_mean, const double* prior_variance,
                            void* workspace, size_t workspace_bytes, void* stream) {
  if (!k_star || ld_rows < current_eval || !prior_mean || !prior_variance) return BO_ERR_ARG;
  if (n_obj < 1 || n_obj > BO_MAX_OBJ) return BO_ERR_ARG;
  bo_predict_desc d;
  fill_mv_desc(&d, n_obj, n_cand, current_eval);
  d.excl_points = (const double*)1;
  d.y_train = y;
  d.ld_y = ld_y;
  d.kinv = kinv;
  d.ld_k = ld_k;
  for (int o = 0; o < n_obj; ++o) {
    d.prior_mean[o] = prior_mean[o];
    d.prior_var[o] = prior_variance[o];
    d.length_scale[o] = 1.0;
    d.beta[o] = 0.0;
  }
  d.mu = mu;
  d.var = var;
  d.ld_out = n_cand;
  return predict_impl(&d, k_star, ld_rows, workspace, workspace_bytes, stream);
}

int bo_profile_start(int max_launches) {
  if (max_launches < 1) return BO_ERR_ARG;
  for (auto& e : g_timer.ev) (void)hipEventDestroy(e);
  g_timer.ev.assign(2 * (size_t)max_launches, nullptr);
  for (auto& e : g_timer.ev) BO_CHECK_HIP(hipEventCreate(&e));
  g_timer.used = 0;
  g_timer.on = true;
  return BO_OK;
}

int bo_profile_stop(double* total_ms, int* launches) {
  g_timer.on = false;
  double tot = 0.0;
  const int n = g_timer.used / 2;
  for (int i = 0; i < n; ++i) {
    BO_CHECK_HIP(hipEventSynchronize(g_timer.ev[2 * i + 1]));
    float ms = 0.f;
    BO_CHECK_HIP(hipEventElapsedTime(&ms, g_timer.ev[2 * i], g_timer.ev[2 * i + 1]));
    tot += ms;
  }
  if (total_ms) *total_ms = tot;
  if (launches) *launches = n;
  g_timer.used = 0;
  return BO_OK;
}

#ifdef BO_ABL_STAMPS
int bo_debug_stamps(unsigned long long* host, int n_waves) {
  BO_CHECK_HIP(hipDeviceSynchronize());
  BO_CHECK_HIP(hipMemcpyFromSymbol(host, HIP_SYMBOL(g_stamps), sizeof(unsigned long long) * 8 * n_waves));
  return BO_OK;
}
#endif

#ifdef BO_ABL_DBGQ
int bo_debug_set_tile(long long t) {
  BO_CHECK_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_dbg_tile), &t, sizeof(t)));
  return BO_OK;
}
int bo_debug_dbgq(double* host) {
  BO_CHECK_HIP(hipDeviceSynchronize());
  BO_CHECK_HIP(hipMemcpyFromSymbol(host, HIP_SYMBOL(g_dbgq), sizeof(double) * 64 * 2 * 4 * 64));
  return BO_OK;
}
#endif

int bo_selftest_mfma_f32(const float* a, const float* b, float* dd, void* stream) {
  if (!a || !b || !dd) return BO_ERR_ARG;
  hipLaunchKernelGGL(selftest_mfma32_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, a, b, dd);
  BO_CHECK_HIP(hipGetLastError());
  return BO_OK;
}

int bo_selftest_mfma_f64(const double* a, const double* b, double* dd, void* stream) {
  if (!a || !b || !dd) return BO_ERR_ARG;
  hipLaunchKernelGGL(selftest_mfma_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, a, b, dd);
  BO_CHECK_HIP(hipGetLastError());
  return BO_OK;
}

}  // extern "C"
