// Internal header of the fused GP-posterior + acquisition + top-q kernels (bo_predict*.hip).
//
// Replaces the reference chain bayesopt/bayesian_optimization.py:145-207:
//   update_k_star (numba_kernels.py:406-442) -> update_mean (:450-488) ->
//   update_variance (:491-535) -> standardize_objectives (:538-570) ->
//   update_ucb / update_hypervolume_improvement (acquisition.py:55-108) ->
//   select_next_batch (acquisition.py:116-144, local top-q part).
//
// The chunk-major kernels are instantiated per padded input dimension in bo_predict_d{2,4,6,8}.hip
// (parallel compilation); bo_predict.hip holds the preparation kernels, the merge kernels, the
// planner and the C ABI.  DESIGN.md §3 describes the kernels.
#pragma once

#include "bo_common.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

#include <type_traits>

namespace bo {

constexpr int kWaves = 4;               // waves per workgroup
constexpr int kTile = 16 * kWaves;      // candidates per workgroup tile
constexpr int kPanelSteps = 128;        // k-steps of 4 training rows per register panel (KMEM path)
constexpr int kPF = 4;                  // W prefetch ring depth (pairs of k-steps)
constexpr int kCMaxEp = 16;             // E-pairs (32 rows each) whose accumulators one wave holds
constexpr int kC32MaxEp = 16;           // E-quads (64 rows each) per group of the f32 kernel
constexpr int kExpTab = 256;            // 2^(j/256) table of exp2_tab

struct FusedArgs {
  int n_obj, dim, n_train, n_pad;       // n_pad = padded training rows (multiple of 32 / 64)
  int n_panels;                          // register panels of 512 rows (KMEM path only)
  int n_excl;
  int cand_kind, topq;
  long long n_cand, cand_offset, ld_out, n_tiles;
  long long grid_lo[BO_MAX_DIM], grid_shape[BO_MAX_DIM];
  const void* cand;
  const double* xpad;                    // [n_pad][DIM] training rows, padded rows = 1e200 (global)
  const double* xc;                      // [n_pad][DIM] rows minus row 0 (the centre z) (global)
  const double* excl;                    // [n_excl][DIM] evaluated points (global), NULL = x_train
  const d2* wpack;                       // packed W (pack_cm_range / pack_range / pack32_range layout)
  unsigned int wpack_bytes;
  int w_pairs;                           // cm: 2-KiB pairs of all objectives' contiguous streams
  const double* alpha;                   // [n_obj][n_pad] = K^-1 (y - pm) (global)
  double pm[BO_MAX_OBJ], pv[BO_MAX_OBJ], nhl[BO_MAX_OBJ], beta[BO_MAX_OBJ];
  double inv_rsq_pv[BO_MAX_OBJ], inv_pv[BO_MAX_OBJ];   // 1 / sqrt(pv), 1 / pv (epilogue multiplies)
  double min_var;                        // MIN_VARIANCE (config.py:57-66): 1e-10, or 1e-6 (F32_FLOOR)
  int idx32;                             // grid: every linear index and extent below 2^31
  double *mu, *var, *std_mu, *std_var, *ucb, *acq;
  TopEntry* partial;                     // [gridDim.x * kWaves][topq]
  const double* kstar;                   // KMEM: materialised k_star [n_obj][ks_rows][n_cand]
  long long ks_rows;
  int upper;                             // W = upper triangle of sym(K^-1), diagonal halved
  // separable K* on an integer grid: device flag (0 => usable), last-axis extent S and lower
  // bound, LDS offsets (doubles) of the exp tables and per-wave row-factor scratch
  const int* sep_flag;
  int sep_S;
  long long sep_lo;
  int off_tbl, off_rw;
  int rw_cache;                          // SEP row factors kept for every objective (LDS permitting)
  int rw_stride;                         // doubles of one wave's row-factor region
  int off_exp;                           // LDS offset (doubles) of the 2^(j/256) table
  SobolArgs sob;                         // kind BO_CAND_SOBOL: direction numbers, lo, scale
  const unsigned long long* hkeys;       // hash set of the exclusion rows (excl or xpad), built
  const int* hidx;                       // by the prep launch (bo_point_key over DIM coordinates)
  unsigned int hmask;
};

// Host-side plan of one bo_predict_acquire call (bo_predict.hip: make_plan).
struct Plan {
  int n_pad, ns, n_panels, dim_pad, n_excl;
  bool multi;
  size_t off_alpha, off_xpad, off_xc, off_excl, off_hash, off_partial, off_status, total;
  unsigned int hash_slots;
  bool cm;               // chunk-major kernel (cm_predict_kernel)
  bool sep;              // ... with the integer-grid K* generation
  bool grows;            // ... training rows / alpha read from global memory (N beyond LDS)
  int off_tbl, off_rw;   // LDS offsets in doubles
  bool rw_cache;         // SEP row factors cached per objective
  int rw_stride;         // doubles per wave of the row-factor region
  bool fp32;             // cm32_predict_kernel (BO_PREDICT_FP32)
  bool small;            // N <= 128: 4 E-pair accumulators, two workgroups per CU
  int off_exp;
  int grid, waves;       // persistent grid, waves per workgroup
  long long n_tiles;
  size_t lds;
};

// launch wrappers (one translation unit per padded dimension)
hipError_t launch_cm_d2(const Plan& pl, const FusedArgs& fa, hipStream_t st);
hipError_t launch_cm_d4(const Plan& pl, const FusedArgs& fa, hipStream_t st);
hipError_t launch_cm_d6(const Plan& pl, const FusedArgs& fa, hipStream_t st);
hipError_t launch_cm_d8(const Plan& pl, const FusedArgs& fa, hipStream_t st);
hipError_t launch_c32_d2(const Plan& pl, const FusedArgs& fa, hipStream_t st);
hipError_t launch_c32_d4(const Plan& pl, const FusedArgs& fa, hipStream_t st);
hipError_t launch_c32_d6(const Plan& pl, const FusedArgs& fa, hipStream_t st);
hipError_t launch_c32_d8(const Plan& pl, const FusedArgs& fa, hipStream_t st);
// the small-N kernels (MAXEP = 4, two workgroups per CU): bo_predict_s<D>.hip, compiled with the
// MFMA accumulators in arch VGPRs (-amdgpu-mfma-vgpr-form): in the default split of the 256
// registers of a 2-waves-per-SIMD kernel (128 VGPR + 128 AGPR) they spilled 40-100 VGPRs to
// scratch while using 32 of their AGPRs
hipError_t launch_cms_d2(const Plan& pl, const FusedArgs& fa, hipStream_t st);
hipError_t launch_cms_d4(const Plan& pl, const FusedArgs& fa, hipStream_t st);
hipError_t launch_cms_d6(const Plan& pl, const FusedArgs& fa, hipStream_t st);
hipError_t launch_cms_d8(const Plan& pl, const FusedArgs& fa, hipStream_t st);

}  // namespace bo

namespace {

using bo::FusedArgs;
using bo::Plan;
using bo::kWaves;
using bo::kTile;
using bo::kPF;
using bo::kCMaxEp;
using bo::kC32MaxEp;
using bo::kExpTab;

template <int DIM>
__device__ __forceinline__ void load_candidate(const FusedArgs& a, long long j, bool valid,
                                               double (&c)[DIM]) {
#pragma unroll
  for (int k = 0; k < DIM; ++k) c[k] = 0.0;
  if (!valid) return;
  if (a.cand_kind == BO_CAND_GRID) {
    if (a.idx32) {                       // 32-bit divisions (the 64-bit ones are ~10x longer)
      unsigned int gi = (unsigned int)(a.cand_offset + j);
#pragma unroll
      for (int k = DIM - 1; k >= 0; --k) {
        if (k < a.dim) {
          const unsigned int n = (unsigned int)a.grid_shape[k];
          const unsigned int q = gi / n;
          c[k] = (double)(a.grid_lo[k] + (long long)(gi - q * n));
          gi = q;
        }
      }
      return;
    }
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
  } else if (a.cand_kind == BO_CAND_SOBOL) {
    // generated from the global index (scipy.stats.qmc.Sobol(scramble=False), bit-identical)
    const unsigned long long gi = (unsigned long long)(a.cand_offset + j);
#pragma unroll
    for (int k = 0; k < DIM; ++k)
      if (k < a.dim) c[k] = bo_sobol_coord(a.sob, k, gi);
  } else {
    const double* p = (const double*)a.cand + j * a.dim;
#pragma unroll
    for (int k = 0; k < DIM; ++k)
      if (k < a.dim) c[k] = p[k];
  }
}

// squared distance between row `row` of xs ([*][DIM], 16-B aligned) and the candidate;
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

__device__ __forceinline__ d4 mfma64(double a, double b, d4 c) {
#ifdef BO_ABL_NOMFMA
  c.x += a * b;
  return c;
#else
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
#endif
}

// Fence between the last MFMA of a contraction and the first read of its accumulators.
// hipcc's gfx950 hazard recognizer under-counts the wait states a VALU / v_accvgpr_read needs
// after v_mfma_f64_16x16x4_f64 when the reading block is reached through a branch that skips
// another block (observed: stale rows of the last MFMA, deterministic data-dependent errors
// up to 0.15 pv).  The asm consumes and "redefines" both accumulators in place, so it cannot be
// scheduled before the MFMAs that produce them and no read of them can be hoisted above it;
// its wait states (BO_NOPS_F64_MFMA, bo_common.h) cover the MFMA's latency.
// (bo_predict_s<D>.hip keeps the accumulators in arch VGPRs: the fence's operand constraint follows)
#ifdef BO_PREDICT_SMALL_DIM
#define BO_ACC_AGPR false
#else
#define BO_ACC_AGPR true
#endif
// NOPS: 0 = ordering only (ablation builds), else the f64 MFMA's read wait states (bo_common.h)
template <bool AGPR, int NOPS = 1>
__device__ __forceinline__ void mfma_fence(d4& x, d4& y) {
  if (NOPS == 0) {
    if (AGPR) asm volatile("" : "+a"(x), "+a"(y));
    else asm volatile("" : "+v"(x), "+v"(y));
  } else {
    if (AGPR) asm volatile(BO_NOPS_F64_MFMA : "+a"(x), "+a"(y));
    else asm volatile(BO_NOPS_F64_MFMA : "+v"(x), "+v"(y));
  }
}

// vmcnt(n) with expcnt / lgkmcnt left at their maxima (gfx9 s_waitcnt encoding)
#define BO_WAIT_VMCNT(n) __builtin_amdgcn_s_waitcnt(((n) & 0xF) | (((n) >> 4) << 14) | 0x70 | 0xF00)

__device__ __forceinline__ d2 wload(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
  return __builtin_bit_cast(d2, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0));
}

template <int PF>
__device__ __forceinline__ void prime_ring(__amdgpu_buffer_rsrc_t wr, int voff, int base,
                                           d2 (&wa)[PF], d2 (&wb)[PF]) {
#pragma unroll
  for (int p = 0; p < PF; ++p) {
    wa[p] = wload(wr, voff, base + (p << 11));
    wb[p] = wload(wr, voff, base + (p << 11) + 1024);
  }
}

// 2^t for the K* exponents (t <= a few tens; -inf / very negative -> exactly 0), with the
// 2^(j/256) table `tb` in LDS: t = n + j/256 + r, |r| <= 1/512; 2^r by its degree-4 Taylor
// polynomial in r ln 2 (|term 5| < 4e-17 relative).  The round-to-nearest k = 256 t comes from
// the 1.5 * 2^52 shifter, whose low 32 bits hold k in two's complement (j = k & 255, n = k >> 8).
// 10 f64 operations (the libm-style exp costs ~20).
__device__ __forceinline__ double exp2_tab(double t, const double* tb) {
  const double x = fmax(t, -1075.0);
  const double s = __builtin_fma(x, 256.0, 6755399441055744.0);
  const int ki = (int)__double_as_longlong(s);
  const double kd = s - 6755399441055744.0;
  const double r = __builtin_fma(kd, -0.00390625, x);
  double p = __builtin_fma(9.6181291076284772e-03, r, 5.5504108664821580e-02);
  p = __builtin_fma(p, r, 2.4022650695910071e-01);
  p = __builtin_fma(p, r, 6.9314718055994531e-01);
  p = __builtin_fma(p, r, 1.0);
  return __builtin_ldexp(p * tb[ki & (kExpTab - 1)], ki >> 8);
}


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

// K* values K*[f][j] = pv exp(-0.5 |x_f - c_j|^2 / ls^2) (numba_kernels.py:436-442) of lane j.
//   SEP (integer 'ij' grid): rv[f] * T[rb[f] - jl] (row factor times the last-axis table; rb
//   and jl are kept as byte offsets and tbj = T - jl, so the address is ONE add per value);
//   otherwise the exponent in base 2 with pv folded in, t = nl2 |x_f - c|^2 + log2 pv
//   (nl2 = nhl log2 e), then exp2_tab.  Coordinates are CENTRED on z = training row 0 (xs holds
//   x_f - z, c is c - z): distances are translation invariant, and f64 differences of centred
//   coordinates keep full precision for point sets far from the origin.  (Round 1's dot form
//   nl2 (|x|^2 + |c|^2 - 2 x.c) saved DIM operations per value but cancels catastrophically
//   when |x| >> ls; with the table exp2 the direct form measures as fast, so it is gone.)
template <int DIM, bool SEP>
struct KRows {
  double nl2, lpv;
  const double* rv;   // SEP: [n_pad] pv * R(f) (0 for padded rows)
  const int* rb;      // SEP: [n_pad] table index base ((x_f,last - lo_last) + S - 1) x 8 bytes
  const double* tb;   // SEP: objective's table T; otherwise the 2^(j/256) table
  const char* tbj;    // SEP: T - jl (bytes), jl = col0 + lane: T[index] = *(tbj + rb[f])
  const double* xs;   // !SEP: training rows [n_pad][DIM] (padded rows at 1e200)
  double c[DIM];      // !SEP: this lane's candidate
  int jl;
  __device__ __forceinline__ double at(int f) const {
    if (SEP) return rv[f] * *(const double*)(tbj + rb[f]);
    return exp2_tab(__builtin_fma(sqdist<DIM>(xs, f, c), nl2, lpv), tb);
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
//   s0: rv[f], rb[f] (next chunk), alpha[f] (this chunk) loads   s1: table loads T[rb - jl] into
//   Bn   s2: Bn *= rv.
// The exp path (!SEP) is VALU work that serialises with f64 MFMAs anyway: all of it in s2.
// The mean takes the chunk being consumed (mu += A . B, every chunk once per group; the groups
// after the first add to a copy that is dropped): no per-value select for the regenerated last
// chunk or the later groups (every VALU instruction of this loop costs MFMA time).
template <int DIM, bool SEP>
struct KGen {
  using KR = KRows<DIM, SEP>;
  double rv[8];
  int rb[8];
  __device__ __forceinline__ void s0(const KR& K, const double* al, int cha, int ch, int g,
                                     double (&A)[8]) {
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      A[s] = al[32 * cha + 4 * s + g];
      const int f = 32 * ch + 4 * s + g;
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
  __device__ __forceinline__ void s1(const KR& K, double (&B)[8]) {
    if (SEP) {
#pragma unroll
      for (int s = 0; s < 8; ++s) B[s] = *(const double*)(K.tbj + rb[s]);
    }
  }
  __device__ __forceinline__ void s2(const KR& K, int ch, int g, double (&B)[8]) {
    if (SEP) {
#pragma unroll
      for (int s = 0; s < 8; ++s) B[s] *= rv[s];
    } else {
      K.chunk(ch, g, B);
    }
  }
};

// ---------------------------------------------------------------------------------------
// Chunk-major fused kernel: the production path.
//
// f64 MFMAs and f64 VALU instructions share the SIMD's DP pipe (measured on MI355X: they
// serialise even across waves), so the time of this kernel is  sum(MFMA) + sum(f64 VALU).
// The loop order is therefore chosen to generate every K* value exactly ONCE per group:
//   for each 32-row chunk c of K* (rows 32c .. 32c+31, 8 values per lane):
//       generate K*[chunk c][16 candidates]  (B operand, registers)
//       for each E-pair ep (32 rows of W) that touches chunk c  -- all 16, or ep <= c when
//       W is upper triangular:   acc[ep] += W[ep-rows, chunk c] . K*[chunk c]
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
// GROWS: the training rows, |x_f|^2 and alpha are read from global memory (L2-resident)
// instead of LDS, for N whose rows do not fit the 160 KiB LDS (the reference has no N cap).
// ---------------------------------------------------------------------------------------
#ifndef BO_SMALL_PF
#define BO_SMALL_PF 2
#endif
// the upper form's completion fence: 1 = BO_NOPS_F64_MFMA (bo_common.h); 0 (ordering only, no
// wait states) only in diagnostic builds, BO_BUILD_VARIANT=DEF_FENCE_NOPS=0
#ifndef BO_FENCE_NOPS
#define BO_FENCE_NOPS 1
#endif
// Diagnostic build (BO_BUILD_VARIANT=DEF_PREDICT_CLK, 2-D kernels): every wave of cm_tiles
// records its shader-clock and 100 MHz real-time-clock spans; bo_debug_predict_clk reads them
// back, so the core clock the kernel ran at is sum(clock) / sum(realtime) x 100 MHz.
#if defined(BO_PREDICT_CLK) && defined(BO_PREDICT_DIM) && BO_PREDICT_DIM == 2
#define BO_CLK_ON 1
__device__ long long bo_predict_clk[2 * 4096];
#else
#define BO_CLK_ON 0
#endif
// PART (UPPER, N not a multiple of 32): the first chunk each group streams -- the last rows,
// partly padding -- is peeled and its all-padding k-step pairs skip their MFMAs (their K* rows
// are exactly 0, so the outputs are bit-identical) and, with the 4-deep ring, their W refills
// (one instantiation per count of live pairs: the refills issued anyway cost N = 518 2 %).  A separate instantiation: the multiples
// of 32 keep the loop's code layout (peeling it into the one kernel cost C3 1.5 %, C4 3 %).
// the sched barriers that place the next chunk's generation stages between E-pair 0's MFMA
// pairs (BO_BUILD_VARIANT=DEF_NO_SCHED_PIN drops them: A/B only)
#ifdef BO_NO_SCHED_PIN
#define BO_GEN_SB ((void)0)
#else
#define BO_GEN_SB __builtin_amdgcn_sched_barrier(0)
#endif
// LANEQ (1 <= q <= 4, the integer-grid SEP path): every lane keeps its own top-4 of the candidates
// it scores (lane group 0; order keys), inserted only when a candidate beats the lane's q-th entry
// and is not an evaluated point; the wave's list is formed once, at the end (one 64-entry sort).
// The general path shares one wave list and tests every tile against its q-th entry by readlanes
// (SGPR spills to VGPR lanes: 199 -> 86 in the C2 kernel without it); with the top-q compiled out
// C2 ran 5 % faster (0.2195 -> 0.2073 ms, C3 -0.3 %, C4 -0.6 %).  Same box, outputs bit-identical
// (profiles/r06_topq_ab.jsonl): C2 0.2205 -> 0.2136 ms, C3 unchanged; on the Sobol path (C4) the
// lanes' lower thresholds send more candidates through the exclusion's hash probe in global
// memory: 108.1 -> 111.2 ms, so the explicit / Sobol kernels keep the wave list.
constexpr int kLaneQ = 4;
template <int DIM, bool SEP, bool UPPER, bool GROWS, int MAXEP, bool PART = false, bool LANEQ = false>
__device__ __forceinline__ void cm_tiles(const FusedArgs& a, double* smem) {
  constexpr bool upper = UPPER;
  // W ring depth in pairs of k-steps: kPF, or BO_SMALL_PF = 2 for the small-N kernels (their W
  // is L2-resident; 16 VGPRs fewer: C2 spills 39 -> 4 VGPRs, kernel -1.3 %)
  constexpr int PF = MAXEP <= 4 ? BO_SMALL_PF : kPF;
  static_assert(4 % PF == 0, "the ring depth divides the 4 pairs of an E-pair body");
  // training rows (SEP: original grid coordinates; otherwise centred on z = row 0), alpha
  const double* xs = GROWS ? a.xc : smem;
  const double* alpha = GROWS ? a.alpha : smem + (size_t)a.n_pad * DIM;
  const double* etab = smem + a.off_exp;                    // 2^(j/256) (!SEP)
  const double* tbl = smem + a.off_tbl;                     // [n_obj][2S - 1] (SEP)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, jl = lane & 15;
  // SEP row factors, per wave: rv[nslot][n_pad] = pv_o R(f) (one slot per objective when they
  // are cached across the tiles of a grid row, else one slot rebuilt per objective and tile),
  // then rb[n_pad] = table index base (x_f,last - lo_last) + S - 1 and on[n_pad] = "training
  // point f lies on this grid row" (all other coordinates equal); with the cache, bm = the
  // row's evaluated columns as a bitmap of S bits (the exclusion is one LDS read per tile)
  const int nslot = a.rw_cache ? a.n_obj : 1;
  double* rv = smem + a.off_rw + (size_t)wave * a.rw_stride;
  int* rb = (int*)(rv + (size_t)nslot * a.n_pad);
  int* on = rb + a.n_pad;
  unsigned int* bm = (unsigned int*)(on + a.n_pad);
  const int bm_words = (a.sep_S + 31) >> 5;
  long long cur_row = -1;
  const int TS = 2 * a.sep_S - 1;
  const int nch = a.n_pad / 32;
  const int last = a.dim - 1;
  const __amdgpu_buffer_rsrc_t wr =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.wpack, (short)0, (int)a.wpack_bytes, 0x00020000);
  const int voff = lane * 16;
  const int w_obj = a.w_pairs / a.n_obj * 2048;             // bytes of one objective's stream

  // the centre z (training row 0) of the non-SEP generation
  double z[DIM];
#pragma unroll
  for (int k = 0; k < DIM; ++k) z[k] = SEP ? 0.0 : a.xpad[k];

#if BO_CLK_ON
  const long long clk0 = clock64(), rt0 = wall_clock64();
#endif
  double top_v = -__builtin_inf();
  long long top_i = -1;
  unsigned long long lk[kLaneQ];        // LANEQ: the lane's list (order keys, selection order)
  long long lx[kLaneQ];
#pragma unroll
  for (int t = 0; t < kLaneQ; ++t) { lk[t] = 0ull; lx[t] = -1; }
  double held_v = -__builtin_inf();     // a tile's candidates waiting for the paired insert
  long long held_i = -1;
  bool held = false;
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
    if (a.rw_cache)
      for (int w = lane; w < bm_words; w += 64) bm[w] = 0u;
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
      rb[f] = b * 8;
      on[f] = onrow;
      const int col = b - (a.sep_S - 1);
      if (a.rw_cache && onrow && col >= 0 && col < a.sep_S) atomicOr(bm + (col >> 5), 1u << (col & 31));
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
        const long long row = a.idx32 ? (long long)((unsigned int)(a.cand_offset + jj) / (unsigned int)a.sep_S)
                                      : (a.cand_offset + jj) / a.sep_S;
        if (row != cur_row) { row_pass(c, 0, a.n_obj); cur_row = row; }
      }
    } else {
      load_candidate<DIM>(a, j, valid, c);
#pragma unroll
      for (int k = 0; k < DIM; ++k) c[k] -= z[k];
    }
    double acq = 0.0;
#ifndef BO_RING_RESET
    // W ring: primed once per tile and running on across the objectives: the objectives' streams
    // lie back to back, so the last refills of objective o load objective o + 1's first pairs
    // (past the last objective they read beyond the stream: zeros or the next pairs, never used)
    d2 wa[PF], wb[PF];
    prime_ring(wr, voff, 0, wa, wb);
    int pos = 0;
#endif
    for (int o = 0; o < a.n_obj; ++o) {
      if (SEP && !a.rw_cache) row_pass(c, o, o + 1);
      KRows<DIM, SEP> K;
      K.rv = rv + (a.rw_cache ? (size_t)o * a.n_pad : 0); K.rb = rb;
      K.tb = SEP ? tbl + (size_t)o * TS : etab;
      K.xs = xs;
      K.nl2 = a.nhl[o] * 1.4426950408889634;
      K.lpv = log2(a.pv[o]);
      K.jl = SEP ? col0 + jl : jl;   // T index = rb[f] - (col0 + jl) = x_f,last - c_last + S - 1
      K.tbj = (const char*)K.tb - (size_t)K.jl * 8;
#pragma unroll
      for (int k = 0; k < DIM; ++k) K.c[k] = c[k];
      const double* al = alpha + (size_t)o * a.n_pad;
#ifdef BO_RING_RESET
      // (A/B build: the ring primed per objective.  A ring running on across the TILES too,
      // wrapping at the end of the packed streams, measured 1.7 % slower at C4 and 3 % faster at
      // C2 in round 2: its modular refill offsets defeat the immediate-offset addressing)
      const int base = o * w_obj;
      d2 wa[PF], wb[PF];
      prime_ring(wr, voff, base, wa, wb);
      int pos = 0;
#else
      constexpr int base = 0;
      (void)w_obj;
#endif
      double mpart = 0.0, qpart = 0.0, msave = 0.0;
      d4 acc[MAXEP][2];
      // E-pairs in groups of kCMaxEp (the accumulators one wave holds: 512 rows); a group
      // streams the chunks that touch it (c >= its first E-pair when upper, all otherwise) and
      // regenerates their K*.  One group when N <= 512.
      for (int e0 = 0; e0 < nch; e0 += MAXEP) {
        const int eN = nch - e0 < MAXEP ? nch - e0 : MAXEP;
        // all kCMaxEp accumulator pairs zeroed unconditionally (zeroing only the group's eN
        // pairs behind nested guards measured 1-2 % slower at C2/C3/C4; starting them instead
        // with the inline constant 0 as C in a peeled first chunk: C2/C3 unchanged, C4 +1.2 %)
#ifndef BO_ABL_NOZERO
#pragma unroll
        for (int e = 0; e < MAXEP; ++e) {
          acc[e][0] = (d4){0.0, 0.0, 0.0, 0.0};
          acc[e][1] = (d4){0.0, 0.0, 0.0, 0.0};
        }
#else
        // ablation: the accumulators are not zeroed (wrong results; timing only)
        if (tile == t_first && o == 0 && e0 == 0) {
#pragma unroll
          for (int e = 0; e < MAXEP; ++e) {
            acc[e][0] = (d4){0.0, 0.0, 0.0, 0.0};
            acc[e][1] = (d4){0.0, 0.0, 0.0, 0.0};
          }
        }
#endif
        // one chunk: MFMAs from register set B while the next chunk's K* is generated into Bn
        // in three stages inside E-pair 0's MFMA stream (the sets alternate: no register
        // copies between the chunks), and mu += alpha . B.  Branch-free: the last chunk
        // regenerates itself (chn clamped) and the groups after the first accumulate a mean
        // that is dropped (msave).
        KGen<DIM, SEP> gen;
        using K4 = std::integral_constant<int, 4>;
        // kp: the chunk's k-step pairs (8 rows each) that hold a training row (4 unless PART's
        // peeled last chunk)
        auto chunk_step = [&](auto kp_c, int ch, const double (&B)[8], double (&Bn)[8]) {
          constexpr int kp = decltype(kp_c)::value;
          double An[8];
          // next chunk: ascending (dense) / descending (upper); the last one regenerates itself
          const int chn = upper ? (ch > e0 ? ch - 1 : ch) : (ch + 1 < nch ? ch + 1 : ch);
          // the group's E-pairs touching chunk ch, ascending: the first n_here of them (e0 + e
          // <= ch when upper).  EpChain nests the guards (body e+1 is reached only from body e),
          // so every body has one predecessor and hipcc's vmcnt waits inside the chunk stay
          // exact; independent guards made every body a join and cost a vmcnt(0) drain of the
          // W ring per E-pair.
          const int n_here = upper ? (ch - e0 + 1 < eN ? ch - e0 + 1 : eN) : eN;
          // PART's peeled chunk: its bodies neither multiply nor refill the pairs >= kp (all
          // padding); those ring slots are loaded once, here, with the next chunk's first body
          // (pairs pos + 4 n_here + s: the chunk's stream keeps 4 pairs per body)
          if constexpr (PART && PF == 4 && kp < 4) {
#pragma unroll
            for (int s = kp; s < 4; ++s) {
              wa[s] = wload(wr, voff, base + ((pos + 4 * n_here + s) << 11));
              wb[s] = wload(wr, voff, base + ((pos + 4 * n_here + s) << 11) + 1024);
            }
          }
          auto ep_body = [&](auto e_c) {
            constexpr int e = decltype(e_c)::value;
            // explicit / Sobol candidates: keep the workgroup's 4 waves on the same E-pair block
            // (they stream identical W data, so 3 of 4 L2 requests become L1 hits).  W beyond
            // the L2s (C5: 50 MB) otherwise comes from MALL once per wave: C5-f64 1124 -> 869 ms
            // (round 2, same box).  The SEP path is left unsynchronised (lockstep measured 4 %
            // slower at C3, 7 % at C2: its W fits L2).
            // (a barrier every 2nd or 4th body measured the same at C4 / C5-f64)
            // Round 3: without it C4 ran 1.7 % faster (108.3 vs 110.1 ms) but fetched 84 GB
            // per launch from beyond the L2 instead of 22 GB, and C5-f64 (W 50 MB) ran 982 vs
            // 822 ms at 4.7 TB of fetches; a runtime switch around the barrier cost 1 % in both
            // settings.  Kept for every explicit / Sobol kernel.
            if constexpr (!SEP) __builtin_amdgcn_s_barrier();
#ifdef BO_ABL_NOGEN
            // ablation: no next-chunk generation and no mean (every chunk reuses the first
            // chunk's K*; wrong results, timing only)
            if constexpr (false) {
#else
            if constexpr (e == 0) {
#endif
              gen.s0(K, al, ch, chn, g, An);
              BO_GEN_SB;
            }
#pragma unroll
            for (int pp = 0; pp < 4; ++pp) {
              // MFMAs first, then the refill of the same ring slot (no operand copies)
              const int sl = pp % PF;         // ring slot (PF divides the 4 pairs of a body)
              if (!PART || pp < kp) {         // (the W ring advances either way)
                acc[e][0] = mfma64(wa[sl].x, B[2 * pp], acc[e][0]);
                acc[e][1] = mfma64(wb[sl].x, B[2 * pp], acc[e][1]);
                acc[e][0] = mfma64(wa[sl].y, B[2 * pp + 1], acc[e][0]);
                acc[e][1] = mfma64(wb[sl].y, B[2 * pp + 1], acc[e][1]);
              }
              const int so = base + ((pos + PF) << 11);
#ifndef BO_ABL_NOREFILL
              if (!(PART && PF == 4) || pp < kp) {
                wa[sl] = wload(wr, voff, so);
                wb[sl] = wload(wr, voff, so + 1024);
              }
#else
              (void)so;   // ablation: the primed W values are reused (no W traffic; timing only)
#endif
              ++pos;
#ifdef BO_ABL_NOGEN
              if constexpr (false) {
#else
              if constexpr (e == 0) {
#endif
                if (pp == 0) {
                  BO_GEN_SB;
                  gen.s1(K, Bn);
                  BO_GEN_SB;
                } else if (pp == 2) {
                  BO_GEN_SB;
                  gen.s2(K, chn, g, Bn);
#ifdef BO_GEN_PIN
                  // A/B only (BO_BUILD_VARIANT=DEF_GEN_PIN): LLVM sinks s2 and the mean out of this
                  // body into the chunk's exit block, past the sched barriers (their values are
                  // next read after the chunk).  Pinning them here with an IR-level use measured
                  // slower everywhere, outputs bit-identical (round 6, same box: C3 8.32 -> 8.37,
                  // C4 108.4 -> 116.2, C5-fp32 394 -> 406, C5-f64 813 -> 867 ms;
                  // profiles/r06_gen_pin_ab.jsonl): the sunk placement stays
                  asm volatile("" : "+v"(Bn[0]), "+v"(Bn[1]), "+v"(Bn[2]), "+v"(Bn[3]), "+v"(Bn[4]),
                               "+v"(Bn[5]), "+v"(Bn[6]), "+v"(Bn[7]));
#endif
                  BO_GEN_SB;
                } else if (pp == 3) {
                  BO_GEN_SB;
#pragma unroll
                  for (int s = 0; s < 8; ++s) mpart = __builtin_fma(An[s], B[s], mpart);
#ifdef BO_GEN_PIN
                  asm volatile("" : "+v"(mpart));
#endif
                  BO_GEN_SB;
                }
              }
            }
            // upper: E-pair e0 + e is complete after its own chunk (chunks descend), the last
            // body of that chunk: q += K*[chunk rows] . acc with the rows still in B (rows
            // 32 ep + g + 4r (+16) = B slots r (4 + r)); no regeneration
#ifdef BO_ABL_NOQ
            if constexpr (false) {
#else
            if constexpr (UPPER) {
#endif
              if (ch - e0 == e) {
                mfma_fence<BO_ACC_AGPR, BO_FENCE_NOPS>(acc[e][0], acc[e][1]);
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                  qpart = __builtin_fma(B[r], acc[e][0][r], qpart);
                  qpart = __builtin_fma(B[4 + r], acc[e][1][r], qpart);
                }
              }
            }
          };
          EpChain<0, MAXEP>::run(ep_body, n_here);
        };
        const int c0 = upper ? nch - 1 : 0;
        double BX[8], BY[8];
        K.chunk(c0, g, BX);
#ifdef BO_ABL_NOGEN
#pragma unroll
        for (int s = 0; s < 8; ++s) BY[s] = BX[s];
#endif
        int ch = c0;
        if constexpr (PART && UPPER) {
          const int r_last = a.n_train - 32 * (nch - 1);
          const int kpv = (r_last + 7) >> 3;
          if (kpv == 1) chunk_step(std::integral_constant<int, 1>{}, ch, BX, BY);
          else if (kpv == 2) chunk_step(std::integral_constant<int, 2>{}, ch, BX, BY);
          else if (kpv == 3) chunk_step(std::integral_constant<int, 3>{}, ch, BX, BY);
          else chunk_step(K4{}, ch, BX, BY);
          --ch;
          for (; ch - 1 >= e0; ch -= 2) {
            chunk_step(K4{}, ch, BY, BX);
            chunk_step(K4{}, ch - 1, BX, BY);
          }
          if (ch >= e0) chunk_step(K4{}, ch, BY, BX);
        } else if (upper) {
          for (; ch - 1 >= e0; ch -= 2) {
            chunk_step(K4{}, ch, BX, BY);
            chunk_step(K4{}, ch - 1, BY, BX);
          }
          if (ch >= e0) chunk_step(K4{}, ch, BX, BY);
        } else {
          for (; ch + 1 < nch; ch += 2) {
            chunk_step(K4{}, ch, BX, BY);
            chunk_step(K4{}, ch + 1, BY, BX);
          }
          if (ch < nch) chunk_step(K4{}, ch, BX, BY);
        }
        // dense: q = k . z after the last chunk, chunk ep's K* regenerated.  Software-pipelined:
        // E-pair e+1's rows are loaded (KGen s0/s1) before E-pair e's fence and multiplied after
        // its FMAs, so the fences' wait states cover the LDS round trips.
        if (!upper) {
          KGen<DIM, SEP> gq[2];
          double S[2][8];
          gq[0].s0k(K, e0, g);
          gq[0].s1(K, S[0]);
          gq[0].s2(K, e0, g, S[0]);
#pragma unroll
          for (int e = 0; e < MAXEP; ++e) {
            if (e < eN) {
              const int cur = e & 1, nxt = cur ^ 1;
              const bool more = e + 1 < eN;
              if (more) gq[nxt].s0k(K, e0 + e + 1, g);
              mfma_fence<BO_ACC_AGPR>(acc[e][0], acc[e][1]);
              if (more) gq[nxt].s1(K, S[nxt]);
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                qpart = __builtin_fma(S[cur][r], acc[e][0][r], qpart);
                qpart = __builtin_fma(S[cur][4 + r], acc[e][1][r], qpart);
              }
              if (more) gq[nxt].s2(K, e0 + e + 1, g, S[nxt]);
            }
          }
        }
        if (e0 == 0) msave = mpart;             // the mean is group 0's (every chunk once)
      }
      mpart = msave;
      if (upper) qpart *= 2.0;
      qpart += __shfl_xor(qpart, 16, 64);
      qpart += __shfl_xor(qpart, 32, 64);
      mpart += __shfl_xor(mpart, 16, 64);
      mpart += __shfl_xor(mpart, 32, 64);
      const double pv = a.pv[o], pm = a.pm[o];
      const double mu = pm + mpart;                                   // :486-488
      const double var = fmax(pv - qpart, a.min_var);                 // :532-535
#ifdef BO_ABL_NOEPI
      const double smu = mu - pm, svar = var, u = smu + a.beta[o] * svar;
#else
      const double smu = (mu - pm) * a.inv_rsq_pv[o];                  // :563-565 (x 1/sqrt(pv))
      const double svar = var * a.inv_pv[o];                           // :568-570 (x 1/pv)
      const double u = smu + a.beta[o] * sqrt(fabs(svar));             // acquisition.py:52
#endif
      acq = (o == 0) ? u : acq + u;                                    // acquisition.py:108
      if (valid && g == 0) {
        const long long off = (long long)o * a.ld_out + j;
        if (a.mu) bo_out_store(a.mu + off, mu);
        if (a.var) bo_out_store(a.var + off, var);
        if (a.std_mu) bo_out_store(a.std_mu + off, smu);
        if (a.std_var) bo_out_store(a.std_var + off, svar);
        if (a.ucb) bo_out_store(a.ucb + off, u);
      }
    }
    if (valid && g == 0 && a.acq) bo_out_store(a.acq + j, acq);
#ifdef BO_ABL_NOTOPQ
    if (false) {
#else
    if (a.topq > 0) {
#endif
      // exclusion of evaluated points (acquisition.py:137-139: all coordinates equal), tested
      // only when a candidate would enter the wave's list (LANEQ: the lane's list)
      const long long gi0 = valid ? a.cand_offset + j : -1;
      bool need;
      unsigned long long kc = 0ull;
      if constexpr (LANEQ) {
        kc = bo_order_key(acq, gi0);
        const int q = a.topq;
        const unsigned long long kq = q == 1 ? lk[0] : q == 2 ? lk[1] : q == 3 ? lk[2] : lk[3];
        const long long xq = q == 1 ? lx[0] : q == 2 ? lx[1] : q == 3 ? lx[2] : lx[3];
        need = g == 0 && gi0 >= 0 && bo_key_before(kc, gi0, kq, xq);
      } else {
        double tv;
        long long ti;
        bo_wave_topq_threshold(top_v, top_i, a.topq, tv, ti);
        need = gi0 >= 0 && bo_better(acq, gi0, tv, ti);
      }
      bool hit = false;
      if (__ballot(need) != 0ull) {
        if (SEP && !a.excl && a.rw_cache) {
          // the row's bitmap of evaluated columns
          const int col = col0 + jl;
          hit = valid && ((bm[col >> 5] >> (col & 31)) & 1u);
        } else if (SEP && !a.excl) {
          // training points on this grid row whose last coordinate falls in the wave's 16
          // columns; OR over the wave, bit jl is this lane's candidate
          unsigned int xmask = 0;
          for (int f = lane; f < a.n_train; f += 64) {
            const int dx = (rb[f] >> 3) - (a.sep_S - 1) - col0;
            if (on[f] && dx >= 0 && dx < 16) xmask |= 1u << dx;
          }
          unsigned int m = xmask;
#pragma unroll
          for (int sh = 32; sh > 0; sh >>= 1) m |= (unsigned int)__shfl_xor((int)m, sh, 64);
          hit = (m >> jl) & 1u;
        } else {
          // compared exactly, in the original coordinates, with the evaluated points of the
          // same hash (the prep launch's table; global memory)
          double co[DIM];
          load_candidate<DIM>(a, j, valid, co);
          hit = valid && bo_hash_contains(a.hkeys, a.hidx, a.hmask, a.excl ? a.excl : a.xpad, DIM, co, DIM);
        }
      }
      if constexpr (LANEQ) {
        // (group 0's lane holds this candidate's own exclusion result)
        if (need && !hit) {
          // sorted insertion: entries the new one beats move down one slot
#pragma unroll
          for (int t = kLaneQ - 1; t >= 0; --t) {
            const bool before_t = bo_key_before(kc, gi0, lk[t], lx[t]);
            const bool after_prev = t == 0 || !bo_key_before(kc, gi0, lk[t > 0 ? t - 1 : 0], lx[t > 0 ? t - 1 : 0]);
            if (before_t) {
              lk[t] = after_prev ? kc : lk[t > 0 ? t - 1 : 0];
              lx[t] = after_prev ? gi0 : lx[t > 0 ? t - 1 : 0];
            }
          }
        }
        continue;
      }
      const unsigned long long hb = __ballot(hit);
      const bool excluded =
          ((hb >> jl) | (hb >> (jl + 16)) | (hb >> (jl + 32)) | (hb >> (jl + 48))) & 1ull;
      const long long gi = excluded ? -1 : gi0;
      // q <= 16: the tiles are inserted in pairs (the first held in registers; the exclusion
      // above tested it against the then-current threshold, a lower bound of the later ones)
      if (a.topq <= 16) {
        if (held) bo_wave_topq_insert16x2(top_v, top_i, acq, gi, held_v, held_i, a.topq);
        else { held_v = acq; held_i = gi; }
        held = !held;
      } else {
        bo_wave_topq_insert(top_v, top_i, acq, gi, a.topq);
      }
    }
  }
  if (held) bo_wave_topq_insert16(top_v, top_i, held_v, held_i, a.topq);
  if constexpr (LANEQ) {
    // the wave's list from the 16 lanes' lists: entry t of group-0 lane jl goes to lane jl + 16 t,
    // then one 64-entry sort in selection order (lanes 0 .. q-1 are written below)
    const int src = lane & 15, t = lane >> 4;
    unsigned long long kk = 0ull;
    long long xx = -1;
#pragma unroll
    for (int u = 0; u < kLaneQ; ++u) {
      const unsigned long long ku = __shfl(lk[u], src, 64);
      const long long xu = __shfl(lx[u], src, 64);
      kk = t == u ? ku : kk;
      xx = t == u ? xu : xx;
    }
    top_v = bo_key_value(kk);
    top_i = kk == 0ull ? -1 : xx;
    bo_wave_sort64(top_v, top_i);
  }
  BO_WAIT_VMCNT(0);                                          // no W load in flight at exit
#if BO_CLK_ON
  {
    const long long clk1 = clock64(), rt1 = wall_clock64();
    const int wid = blockIdx.x * kWaves + wave;
    if (lane == 0 && wid < 4096) {
      bo_predict_clk[2 * wid] = clk1 - clk0;
      bo_predict_clk[2 * wid + 1] = rt1 - rt0;
    }
  }
#endif
  if (a.topq > 0) {
    if (lane < a.topq) {
      TopEntry* dst = a.partial + ((size_t)blockIdx.x * kWaves + wave) * a.topq;
      dst[lane].v = top_v;
      dst[lane].i = top_i;
    }
  }
}

// GRID: the host found the grid structure usable (rows of 16); the device flag then says
// whether every training point lies on the grid's last axis (sep_check in the prep kernel).
// GROWS: training rows / alpha stay in global memory (N beyond the LDS budget).
// MAXEP: E-pair accumulators per wave.  16 (256 AGPRs, one wave per SIMD) in general; 4 for
// N <= 128 (one group), with two workgroups per CU: at such N the per-tile serial sections
// (W ring priming, first-chunk generation, accumulator fences, the epilogue's divisions and
// square roots, the top-q shuffles) are long against the tile's 160 MFMAs, and the second
// wave on each SIMD issues its MFMAs while the first waits in them.
template <int DIM, bool GRID, bool UPPER, bool GROWS, int MAXEP, bool PART = false, bool LANEQ = false>
__global__ __launch_bounds__(256, MAXEP <= 4 ? 2 : 1) void cm_predict_kernel(const FusedArgs a) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int tid = threadIdx.x;
  const bool sep = !GROWS && GRID && __builtin_amdgcn_readfirstlane(*a.sep_flag) == 0;
  if (!GROWS) {
    // rows: original grid coordinates for the row pass (SEP), centred otherwise
    const double* src = sep ? a.xpad : a.xc;
    for (int t = tid; t < a.n_pad * DIM; t += blockDim.x) smem[t] = src[t];
    double* alpha = smem + (size_t)a.n_pad * DIM;
    for (int t = tid; t < a.n_obj * a.n_pad; t += blockDim.x) alpha[t] = a.alpha[t];
  }
  if (sep) {
    double* tbl = smem + a.off_tbl;
    const int TS = 2 * a.sep_S - 1;
    for (int t = tid; t < a.n_obj * TS; t += blockDim.x) {
      const int o = t / TS;
      const double m = (double)(t - o * TS - (a.sep_S - 1));
      tbl[t] = exp(a.nhl[o] * (m * m));
    }
  } else {
    for (int t = tid; t < kExpTab; t += blockDim.x) smem[a.off_exp + t] = exp2((double)t / kExpTab);
  }
  __syncthreads();
  if constexpr (GRID && !GROWS) {
    if (sep) { cm_tiles<DIM, true, UPPER, false, MAXEP, PART, LANEQ>(a, smem); return; }
  }
  cm_tiles<DIM, false, UPPER, GROWS, MAXEP, PART>(a, smem);   // (the lane lists: SEP only)
}

template <int DIM, bool GRID, bool UPPER, bool GROWS, int MAXEP, bool PART = false, bool LANEQ = false>
hipError_t launch_cm_k(const FusedArgs& fa, int grid, size_t lds, hipStream_t st) {
  auto k = cm_predict_kernel<DIM, GRID, UPPER, GROWS, MAXEP, PART, LANEQ>;
  if (lds > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)lds);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(k, dim3(grid), dim3(256), lds, st, fa);
  return hipGetLastError();
}

// the lane-local top-q (cm_tiles LANEQ) for 1 <= q <= 4; BO_TOPQ_WAVE=1 keeps the wave list (A/B)
inline bool lane_topq(const FusedArgs& fa) {
  static const bool off = getenv("BO_TOPQ_WAVE") != nullptr;
  return !off && fa.topq >= 1 && fa.topq <= kLaneQ;
}

template <int DIM, bool UPPER, bool GROWS>
hipError_t launch_cm_u(const Plan& pl, const FusedArgs& fa, hipStream_t st) {
  if constexpr (GROWS) return launch_cm_k<DIM, false, UPPER, true, bo::kCMaxEp>(fa, pl.grid, pl.lds, st);
  if (pl.small) {
    if constexpr (DIM == 2) return bo::launch_cms_d2(pl, fa, st);
    else if constexpr (DIM == 4) return bo::launch_cms_d4(pl, fa, st);
    else if constexpr (DIM == 6) return bo::launch_cms_d6(pl, fa, st);
    else return bo::launch_cms_d8(pl, fa, st);
  }
  if constexpr (UPPER) {
    const bool laneq = lane_topq(fa);
    // a partly padded last chunk (the drop-in loop's N) with at least one all-padding k-step
    // pair; with 25..31 rows (nothing to skip) the peeled layout measured +1.4 %
    if (fa.n_train % 32 != 0 && fa.n_train % 32 <= 24) {
      if (laneq && pl.sep) return launch_cm_k<DIM, true, true, false, bo::kCMaxEp, true, true>(fa, pl.grid, pl.lds, st);
      return pl.sep ? launch_cm_k<DIM, true, true, false, bo::kCMaxEp, true>(fa, pl.grid, pl.lds, st)
                    : launch_cm_k<DIM, false, true, false, bo::kCMaxEp, true>(fa, pl.grid, pl.lds, st);
    }
    if (laneq && pl.sep) return launch_cm_k<DIM, true, true, false, bo::kCMaxEp, false, true>(fa, pl.grid, pl.lds, st);
  }
  return pl.sep ? launch_cm_k<DIM, true, UPPER, false, bo::kCMaxEp>(fa, pl.grid, pl.lds, st)
                : launch_cm_k<DIM, false, UPPER, false, bo::kCMaxEp>(fa, pl.grid, pl.lds, st);
}

template <int DIM>
hipError_t launch_cm(const Plan& pl, const FusedArgs& fa, hipStream_t st) {
  if (fa.upper)
    return pl.grows ? launch_cm_u<DIM, true, true>(pl, fa, st) : launch_cm_u<DIM, true, false>(pl, fa, st);
  return pl.grows ? launch_cm_u<DIM, false, true>(pl, fa, st) : launch_cm_u<DIM, false, false>(pl, fa, st);
}

// ---------------------------------------------------------------------------------------
// fp32 variant (BO_PREDICT_FP32; BASELINE config C5 "fp32 with fp64 reference check"):
// the upper form q = 2 k.(U k) on v_mfma_f32_16x16x4_f32 (32 cycles per MFMA per SIMD, twice
// the f64 rate), K* = 2^(nhl log2e |x_f - c_j|^2 + log2 pv) on v_exp_f32 over coordinates
// centred on training row 0 (f32 keeps only ~7 digits of absolute coordinates), mu / q
// accumulated in f32 and everything after them (variance floor, standardisation, UCB, sum,
// top-q) in f64.
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

__device__ __forceinline__ f4 mfma32(float a, float b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f4 wload32(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
  return __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0));
}
__device__ __forceinline__ void mfma_fence32(f4& a, f4& b, f4& c, f4& d) {
  asm volatile(BO_NOPS_F32_MFMA
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

// PART (N not a multiple of 64, at most 48 rows in the last chunk): as in the f64 kernel, the
// first chunk each group streams -- the last 64 rows, partly padding -- is peeled.  Its k-quads
// (16 rows each) that hold only padding rows skip their MFMAs, their W refills, the mean's FMAs
// and the first-chunk generation: those K* rows are exactly 0 (padded rows at inf, exp2f(-inf)),
// so the outputs are bit-identical.  One KERNEL per count of live k-quads KQV (1..3; 4 = no
// peel): a runtime switch between the peeled variants inside one kernel spilled 460 B per lane
// (the joins of 256 accumulators), against 52 B for the unpeeled kernel.  The
// ring slots the skipped refills would have filled are loaded once, at the chunk's start, with
// the body after the chunk.  Every loop N of C5 (2064 ... 2240) is such an N: before the peel
// N = 2049 cost what N = 2112 does (+6.6 % over N = 2048, profiles/r05_c5_fp32_npad_probe.txt).
template <int DIM, int KQV = 4>
__global__ __launch_bounds__(256, 1) void cm32_predict_kernel(const FusedArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem32[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, jl = lane & 15;
  float* xs = smem32;                                        // [n_pad][DIM] centred rows
  float* al = xs + (size_t)a.n_pad * DIM;                    // [n_obj][n_pad]
  for (int t = tid; t < a.n_pad * DIM; t += blockDim.x) xs[t] = (float)a.xc[t];   // 1e200 -> inf
  for (int t = tid; t < a.n_obj * a.n_pad; t += blockDim.x) al[t] = (float)a.alpha[t];
  __syncthreads();
  double z[DIM];
#pragma unroll
  for (int k = 0; k < DIM; ++k) z[k] = a.xpad[k];
  const int nch = a.n_pad / 64;
  const long long w_obj = c32_blocks(nch) * 1024 * 16;       // bytes per objective
  const __amdgpu_buffer_rsrc_t wr =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.wpack, (short)0, (int)a.wpack_bytes, 0x00020000);
  const int voff = lane * 16;
  const double* es = a.excl ? a.excl : a.xpad;               // f64 [*][DIM] (exact equality)
  double top_v = -__builtin_inf();
  long long top_i = -1;
  for (long long tile = blockIdx.x; tile < a.n_tiles; tile += gridDim.x) {
    const long long j = tile * kTile + wave * 16 + jl;
    const bool valid = j < a.n_cand;
    double c[DIM];
    load_candidate<DIM>(a, j, valid, c);
    float c32[DIM];
#pragma unroll
    for (int k = 0; k < DIM; ++k) c32[k] = (float)(c[k] - z[k]);
    double acq = 0.0;
#ifndef BO_RING_RESET
    // the W ring runs on across the objectives (their streams lie back to back), as in cm_tiles
    f4 w[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) w[q] = wload32(wr, voff, q * 1024);
    int pos = 0;
#endif
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
      // the chunk's K* in the permuted k-step order; k-quads >= KQ (all padding) are 0
      auto chunk_kq = [&](auto kq_c, int ch, float (&B)[16]) {
        constexpr int KQ = decltype(kq_c)::value;
#pragma unroll
        for (int s = 0; s < 16; ++s)
          B[s] = (s >> 2) < KQ ? kval(64 * ch + 16 * (s >> 2) + 4 * g + (s & 3)) : 0.0f;
      };
      using Q4 = std::integral_constant<int, 4>;
      auto chunk = [&](int ch, float (&B)[16]) { chunk_kq(Q4{}, ch, B); };
      const float* alo = al + (size_t)o * a.n_pad;
#ifdef BO_RING_RESET
      const int base = (int)(o * w_obj);
      f4 w[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) w[q] = wload32(wr, voff, base + q * 1024);
      int pos = 0;
#else
      constexpr int base = 0;
      (void)w_obj;
#endif
      float mpart = 0.0f, qpart = 0.0f, msave = 0.0f;
      f4 acc[kC32MaxEp][4];
      for (int e0 = 0; e0 < nch; e0 += kC32MaxEp) {
        const int eN = nch - e0 < kC32MaxEp ? nch - e0 : kC32MaxEp;
#pragma unroll
        for (int e = 0; e < kC32MaxEp; ++e)
#pragma unroll
          for (int b = 0; b < 4; ++b) acc[e][b] = (f4){0.0f, 0.0f, 0.0f, 0.0f};
        // kqv: the chunk's k-quads that hold a training row (4 unless PART's peeled last chunk)
        auto chunk_step = [&](auto kq_c, int ch, const float (&B)[16], float (&Bn)[16]) {
          constexpr int kqv = decltype(kq_c)::value;
          const int chn = ch > e0 ? ch - 1 : ch;
          const int n_here = ch - e0 + 1 < eN ? ch - e0 + 1 : eN;
          if constexpr (kqv < 4) {
            // the ring slots of the skipped k-quads: the body after this chunk's n_here bodies
#pragma unroll
            for (int kq = kqv; kq < 4; ++kq)
#pragma unroll
              for (int b = 0; b < 4; ++b)
                w[4 * kq + b] = wload32(wr, voff, base + (pos + n_here) * 16384 + kq * 4096 + b * 1024);
          }
          auto ep_body = [&](auto e_c) {
            constexpr int e = decltype(e_c)::value;
            // keep the workgroup's 4 waves on the same E-quad block: they stream identical W
            // data, so the lockstep turns 3 of 4 L2 reads into L1 hits (C5: W = 8.6 MB per
            // objective does not fit an XCD's L2; measured 141 -> 108 ms per 2^20 candidates)
            __builtin_amdgcn_s_barrier();
            if constexpr (e == 0) {
              // branch-free (a join here would drain the W ring with vmcnt(0))
#pragma unroll
              for (int s = 0; s < 4 * kqv; ++s) {
                const float av = alo[64 * ch + 16 * (s >> 2) + 4 * g + (s & 3)];
                mpart = __builtin_fmaf(av, B[s], mpart);   // group 0's is kept (msave)
              }
              chunk(chn, Bn);
#ifdef BO_GEN_PIN
              // (A/B only, as in cm_tiles: pinning the generation here measured slower)
              asm volatile("" : "+v"(Bn[0]), "+v"(Bn[1]), "+v"(Bn[2]), "+v"(Bn[3]), "+v"(Bn[4]), "+v"(Bn[5]),
                           "+v"(Bn[6]), "+v"(Bn[7]), "+v"(Bn[8]), "+v"(Bn[9]), "+v"(Bn[10]), "+v"(Bn[11]),
                           "+v"(Bn[12]), "+v"(Bn[13]), "+v"(Bn[14]), "+v"(Bn[15]), "+v"(mpart));
#endif
            }
#pragma unroll
            for (int kq = 0; kq < kqv; ++kq) {
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
              for (int b = 0; b < kqv; ++b)       // blocks b >= kqv: B rows of padding (0)
#pragma unroll
                for (int r = 0; r < 4; ++r) qpart = __builtin_fmaf(B[4 * b + r], acc[e][b][r], qpart);
            }
          };
          EpChain<0, kC32MaxEp>::run(ep_body, n_here);
        };
        float BX[16], BY[16];
        int ch = nch - 1;
        if constexpr (KQV < 4) {
          using QP = std::integral_constant<int, KQV>;
          chunk_kq(QP{}, ch, BX);
          chunk_step(QP{}, ch, BX, BY);
          --ch;
          for (; ch - 1 >= e0; ch -= 2) {
            chunk_step(Q4{}, ch, BY, BX);
            chunk_step(Q4{}, ch - 1, BX, BY);
          }
          if (ch >= e0) chunk_step(Q4{}, ch, BY, BX);
        } else {
          chunk(ch, BX);
          for (; ch - 1 >= e0; ch -= 2) {
            chunk_step(Q4{}, ch, BX, BY);
            chunk_step(Q4{}, ch - 1, BY, BX);
          }
          if (ch >= e0) chunk_step(Q4{}, ch, BX, BY);
        }
        if (e0 == 0) msave = mpart;
      }
      mpart = msave;
      qpart += __shfl_xor(qpart, 16, 64);
      qpart += __shfl_xor(qpart, 32, 64);
      mpart += __shfl_xor(mpart, 16, 64);
      mpart += __shfl_xor(mpart, 32, 64);
      const double pv = a.pv[o], pm = a.pm[o];
      const double mu = pm + (double)mpart;                               // :486-488
      const double var = fmax(pv - 2.0 * (double)qpart, a.min_var);  // :532-535
      const double smu = (mu - pm) * a.inv_rsq_pv[o];                     // :563-565 (x 1/sqrt(pv))
      const double svar = var * a.inv_pv[o];                              // :568-570 (x 1/pv)
      const double u = smu + a.beta[o] * sqrt(fabs(svar));                // acquisition.py:52
      acq = (o == 0) ? u : acq + u;                                       // acquisition.py:108
      if (valid && g == 0) {
        const long long off = (long long)o * a.ld_out + j;
        if (a.mu) bo_out_store(a.mu + off, mu);
        if (a.var) bo_out_store(a.var + off, var);
        if (a.std_mu) bo_out_store(a.std_mu + off, smu);
        if (a.std_var) bo_out_store(a.std_var + off, svar);
        if (a.ucb) bo_out_store(a.ucb + off, u);
      }
    }
    if (valid && g == 0 && a.acq) bo_out_store(a.acq + j, acq);
    if (a.topq > 0) {
      long long gi = valid ? a.cand_offset + j : -1;
      double tv;
      long long ti;
      bo_wave_topq_threshold(top_v, top_i, a.topq, tv, ti);
      const bool need = gi >= 0 && bo_better(acq, gi, tv, ti);
      if (__ballot(need) != 0ull) {
        // acquisition.py:137-139, exact f64 coordinates (hash probe + exact comparison)
        const bool hit = valid && bo_hash_contains(a.hkeys, a.hidx, a.hmask, es, DIM, c, DIM);
        const unsigned long long hb = __ballot(hit);
        if (((hb >> jl) | (hb >> (jl + 16)) | (hb >> (jl + 32)) | (hb >> (jl + 48))) & 1ull) gi = -1;
      }
      if (a.topq <= 16) bo_wave_topq_insert16(top_v, top_i, acq, gi, a.topq);
      else bo_wave_topq_insert(top_v, top_i, acq, gi, a.topq);
    }
  }
  BO_WAIT_VMCNT(0);                                          // no W load in flight at exit
  if (a.topq > 0) {
    if (lane < a.topq) {
      TopEntry* dst = a.partial + ((size_t)blockIdx.x * kWaves + wave) * a.topq;
      dst[lane].v = top_v;
      dst[lane].i = top_i;
    }
  }
}

template <int DIM>
hipError_t launch_c32(const Plan& pl, const FusedArgs& fa, hipStream_t st) {
  // peeled when the last 64-row chunk has at least one all-padding k-quad (<= 48 live rows)
  const int r_last = fa.n_train % 64;
  int kqv = (r_last == 0 || getenv("BO_C32_NOPART") != nullptr) ? 4 : (r_last + 15) >> 4;
  if (const char* f = getenv("BO_C32_KQV")) {   // A/B only: a larger count is still exact
    const int v = atoi(f);
    if (v > kqv && v <= 4) kqv = v;
  }
  // two live k-quads run the 3-quad kernel: the KQV = 2 instantiation measured slower than it
  // (C5 at N = 2064 / 2080, the same problem forced onto each: KQV 1 407.5, 2 427.4, 3 423.3,
  // 4 431.6 ms, profiles/r06_c5_fp32_kqv_probe.txt) -- its code, not its MFMA count, which is
  // lower; every peeled kernel is exact for any larger count of live k-quads
  auto k = kqv == 1 ? cm32_predict_kernel<DIM, 1>
         : kqv <= 3 ? cm32_predict_kernel<DIM, 3> : cm32_predict_kernel<DIM, 4>;
  if (pl.lds > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)pl.lds);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(k, dim3(pl.grid), dim3(256), pl.lds, st, fa);
  return hipGetLastError();
}

}  // namespace

// one translation unit per padded dimension: bo_predict_d<D>.hip defines BO_PREDICT_DIM;
// bo_predict_s<D>.hip defines BO_PREDICT_SMALL_DIM (the MAXEP = 4 kernels only)
#define BO_CAT_(a, b) a##b
#define BO_CAT(a, b) BO_CAT_(a, b)
#ifdef BO_PREDICT_SMALL_DIM
namespace bo {
hipError_t BO_CAT(launch_cms_d, BO_PREDICT_SMALL_DIM)(const Plan& pl, const FusedArgs& fa, hipStream_t st) {
  constexpr int D = BO_PREDICT_SMALL_DIM;
  if (fa.upper && pl.sep && lane_topq(fa)) return launch_cm_k<D, true, true, false, 4, false, true>(fa, pl.grid, pl.lds, st);
  if (fa.upper)
    return pl.sep ? launch_cm_k<D, true, true, false, 4>(fa, pl.grid, pl.lds, st)
                  : launch_cm_k<D, false, true, false, 4>(fa, pl.grid, pl.lds, st);
  return pl.sep ? launch_cm_k<D, true, false, false, 4>(fa, pl.grid, pl.lds, st)
                : launch_cm_k<D, false, false, false, 4>(fa, pl.grid, pl.lds, st);
}
}  // namespace bo
#endif
#if BO_CLK_ON
// diagnostic build only: the per-wave (shader clock, 100 MHz clock) spans of the last 2-D
// launch (2 words per wave, `n` waves at most); returns the waves copied
extern "C" __attribute__((visibility("default"))) int bo_debug_predict_clk(long long* out, int n) {
  if (n > 4096) n = 4096;
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(bo_predict_clk), sizeof(long long) * 2 * n) != hipSuccess) return -1;
  return n;
}
#endif
#ifdef BO_PREDICT_DIM
namespace bo {
hipError_t BO_CAT(launch_cm_d, BO_PREDICT_DIM)(const Plan& pl, const FusedArgs& fa, hipStream_t st) {
  return launch_cm<BO_PREDICT_DIM>(pl, fa, st);
}
hipError_t BO_CAT(launch_c32_d, BO_PREDICT_DIM)(const Plan& pl, const FusedArgs& fa, hipStream_t st) {
  return launch_c32<BO_PREDICT_DIM>(pl, fa, st);
}
}  // namespace bo
#endif
