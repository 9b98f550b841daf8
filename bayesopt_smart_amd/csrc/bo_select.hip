// Elementwise / selection / Pareto kernels of the drop-in ABI:
//   bo_update_k            numba_kernels.py:329-367  (RBF Gram)
//   bo_update_k_star       numba_kernels.py:406-442  (materialised K*, unfused API)
//   bo_standardize_ucb_hvi numba_kernels.py:538-570 + acquisition.py:55-108
//   bo_select_topq         acquisition.py:116-144
//   bo_pareto_mask         pareto.py:12-45
// These are HBM-bound integer/compare/elementwise kernels: coalesced, one pass.

#include "bo_common.h"

#include <math.h>
#include <string.h>

namespace {

struct HostParams {
  double a[BO_MAX_OBJ], b[BO_MAX_OBJ], c[BO_MAX_OBJ];
};

// ----------------------------------------------------------------------------- Gram
// One thread per (i, j>=i) pair of rows [last, cur): K[o][i][j] = K[o][j][i].
__global__ void gram_kernel(double* __restrict__ km, long long ld, int n_obj,
                            const double* __restrict__ x, int dim, int last, int cur,
                            HostParams p) {
  const int i = last + blockIdx.y;
  const int j = i + blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= cur || j >= cur) return;
  double sq = 0.0;
  for (int k = 0; k < dim; ++k) {
    const double d = x[(long long)i * dim + k] - x[(long long)j * dim + k];
    sq = __builtin_fma(d, d, sq);
  }
  for (int o = 0; o < n_obj; ++o) {
    // pv * exp(-0.5 * sq / ls^2)  (numba_kernels.py:358-360); p.b = ls^2
    const double v = p.a[o] * exp(-0.5 * sq / p.b[o]);
    double* ko = km + (long long)o * ld * ld;
    ko[(long long)i * ld + j] = v;
    ko[(long long)j * ld + i] = v;
  }
}

// ------------------------------------------------------------------------------ K*
__global__ void kstar_kernel(double* __restrict__ ks, long long ld_rows, int n_obj,
                             const double* __restrict__ x, int dim, int kind,
                             const void* __restrict__ cand, long long n_cand, int last, int cur,
                             HostParams p) {
  const long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  const int e = last + blockIdx.y;
  if (i >= n_cand || e >= cur) return;
  double sq = 0.0;
  for (int k = 0; k < dim; ++k) {
    const double c = kind == BO_CAND_I64 ? (double)((const long long*)cand)[i * dim + k]
                                         : ((const double*)cand)[i * dim + k];
    const double d = x[(long long)e * dim + k] - c;
    sq = __builtin_fma(d, d, sq);
  }
  for (int o = 0; o < n_obj; ++o)
    ks[((long long)o * ld_rows + e) * n_cand + i] = p.a[o] * exp(-0.5 * sq / p.b[o]);
}

// --------------------------------------------------------------- standardise/UCB/HVI
__global__ void std_ucb_hvi_kernel(double* __restrict__ smu, double* __restrict__ svar,
                                   double* __restrict__ ucb, double* __restrict__ acq,
                                   const double* __restrict__ mu, const double* __restrict__ var,
                                   int n_obj, long long n, HostParams p, HostParams q) {
  const long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (i >= n) return;
  double a = 0.0;
  for (int o = 0; o < n_obj; ++o) {
    const long long off = (long long)o * n + i;
    const double m = (mu[off] - p.a[o]) / q.a[o];      // (mu - pm) / sqrt(pv)
    const double v = var[off] / p.b[o];                 // var / pv
    const double u = m + p.c[o] * sqrt(fabs(v));        // mu + beta * sqrt(|var|)
    if (smu) smu[off] = m;
    if (svar) svar[off] = v;
    if (ucb) ucb[off] = u;
    a = (o == 0) ? u : a + u;
  }
  if (acq) acq[i] = a;
}

__global__ void ucb_kernel(double* __restrict__ ucb, const double* __restrict__ mu,
                           const double* __restrict__ var, int n_obj, long long n, HostParams p) {
  const long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (i >= n) return;
  for (int o = 0; o < n_obj; ++o) {
    const long long off = (long long)o * n + i;
    ucb[off] = mu[off] + p.a[o] * sqrt(fabs(var[off]));
  }
}

__global__ void hvi_kernel(double* __restrict__ acq, const double* __restrict__ ucb, int n_obj,
                           long long n) {
  const long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (i >= n) return;
  double a = ucb[i];
  for (int o = 1; o < n_obj; ++o) a += ucb[(long long)o * n + i];
  acq[i] = a;
}

// ------------------------------------------------------------------------ selection
struct SelArgs {
  const double* acq;
  long long n_cand, cand_offset;
  int kind, dim, n_excl, topq;
  const void* cand;
  long long grid_lo[BO_MAX_DIM], grid_shape[BO_MAX_DIM];
  const double* excl;
  // open-addressing hash set of the evaluated points (keys: bo_point_key, 0 = empty; idx: the
  // point's row): built per workgroup in LDS (lds_slots > 0), else in the
  // workspace (hkeys), else NULL (the exclusion scans the points)
  int lds_slots;
  const unsigned long long* hkeys;
  const int* hidx;
  unsigned int hmask;
  TopEntry* partial;
  long long partial_cap;    // entries of `partial` (the debug build checks every write)
  int idx32;                // grid: every global index below 2^31 (32-bit decode)
  SobolArgs sob;            // kind BO_CAND_SOBOL
  // candidate exclusion mask (bo_excl_mask_update): bit j of word j / 32 set = local candidate j
  // equals an evaluated point.  When given, an excluded element is dropped as it is loaded (key
  // 0, as an out-of-range one) and n_excl is 0: no hash, no probes.
  const unsigned int* xbits;
};

__device__ __forceinline__ bool xbit(const unsigned int* xb, long long j) {
  return xb && ((xb[j >> 5] >> (j & 31)) & 1u);
}

__global__ void excl_hash_kernel(unsigned long long* __restrict__ keys, int* __restrict__ idx,
                                 unsigned int mask, const double* __restrict__ excl, int first,
                                 int n_excl, int dim) {
  const int e = first + blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n_excl) return;
  const unsigned long long key = bo_point_key(excl + (long long)e * dim, dim);
  if (key != 0ull) bo_hash_insert(keys, idx, mask, key, e);
}

__device__ __forceinline__ double cand_coord(const SelArgs& a, long long j, int k);

// candidate j equal (every coordinate) to an evaluated point?  Hash probe when a table is
// given, else the O(n_excl) scan.
__device__ __forceinline__ bool cand_excluded(const SelArgs& a, long long j,
                                              const unsigned long long* hk, const int* hi,
                                              unsigned int hm) {
  double c[BO_MAX_DIM];
  if (a.kind == BO_CAND_GRID && a.idx32) {   // 32-bit divisions (the 64-bit ones are ~10x longer)
    unsigned int gi = (unsigned int)(a.cand_offset + j);
#pragma unroll
    for (int k = BO_MAX_DIM - 1; k >= 0; --k) {
      c[k] = 0.0;
      if (k < a.dim) {
        const unsigned int n = (unsigned int)a.grid_shape[k];
        const unsigned int q = gi / n;
        c[k] = (double)(a.grid_lo[k] + (long long)(gi - q * n));
        gi = q;
      }
    }
  } else if (a.kind == BO_CAND_GRID) {   // all coordinates from one chain of divisions
    long long gi = a.cand_offset + j;
#pragma unroll
    for (int k = BO_MAX_DIM - 1; k >= 0; --k) {
      c[k] = 0.0;
      if (k < a.dim) {
        c[k] = (double)(a.grid_lo[k] + gi % a.grid_shape[k]);
        gi /= a.grid_shape[k];
      }
    }
  } else {
#pragma unroll
    for (int k = 0; k < BO_MAX_DIM; ++k) c[k] = k < a.dim ? cand_coord(a, j, k) : 0.0;
  }
  if (hk) return bo_hash_contains(hk, hi, hm, a.excl, a.dim, c, a.dim, a.n_excl);
  for (int e = 0; e < a.n_excl; ++e) {
    bool eq = true;
#pragma unroll
    for (int k = 0; k < BO_MAX_DIM; ++k) eq = eq && (k >= a.dim || a.excl[(long long)e * a.dim + k] == c[k]);
    if (eq) return true;
  }
  return false;
}

__device__ __forceinline__ double cand_coord(const SelArgs& a, long long j, int k) {
  if (a.kind == BO_CAND_I64) return (double)((const long long*)a.cand)[j * a.dim + k];
  if (a.kind == BO_CAND_F64) return ((const double*)a.cand)[j * a.dim + k];
  if (a.kind == BO_CAND_SOBOL) return bo_sobol_coord(a.sob, k, (unsigned long long)(a.cand_offset + j));
  long long gi = a.cand_offset + j;
  for (int t = a.dim - 1; t > k; --t) gi /= a.grid_shape[t];
  return (double)(a.grid_lo[k] + gi % a.grid_shape[k]);
}

// ---------------------------------------------------------------------------------------
// The candidate exclusion mask (bo_excl_mask_update): the set acquisition.py:137-139 tests
// per candidate -- "equal in every coordinate to an evaluated point" -- as one bit per local
// candidate index, built once per iteration (or extended by the q new points), so that the
// selection drops an excluded element as it loads it.
// Grid candidates (every coordinate below 2^53): point e maps to at most one grid index, found
// arithmetically -- each coordinate must be an integer lo_k + t_k, 0 <= t_k < shape_k.
__global__ void excl_mask_grid_kernel(unsigned int* __restrict__ bits, SelArgs a, int first) {
  const int e = first + blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= a.n_excl) return;
  const double* p = a.excl + (long long)e * a.dim;
  long long gi = 0;
  for (int k = 0; k < a.dim; ++k) {
    const double x = p[k];
    const double lo = (double)a.grid_lo[k];
    // NaN or outside [lo, lo + shape) or not an integer: no candidate equals it
    if (!(x >= lo && x < lo + (double)a.grid_shape[k]) || x != __builtin_floor(x)) return;
    gi = gi * a.grid_shape[k] + ((long long)x - a.grid_lo[k]);
  }
  const long long j = gi - a.cand_offset;
  if (j < 0 || j >= a.n_cand) return;
  atomicOr(bits + (j >> 5), 1u << (j & 31));
}

// Any other candidate kind: every candidate probes the hash set of the points (global memory);
// a wave's 64 consecutive candidates set their bits with at most two atomics.
__global__ void excl_mask_scan_kernel(unsigned int* __restrict__ bits, SelArgs a,
                                      const unsigned long long* __restrict__ hk,
                                      const int* __restrict__ hi, unsigned int hm) {
  const long long j = (long long)blockIdx.x * blockDim.x + threadIdx.x;   // blockDim 256
  const bool hit = j < a.n_cand && cand_excluded(a, j, hk, hi, hm);
  const unsigned long long b = __ballot(hit);
  if ((threadIdx.x & 63) == 0 && b) {
    const long long w = j >> 5;                  // j is a multiple of 64 in lane 0
    if ((unsigned int)b) atomicOr(bits + w, (unsigned int)b);
    if ((unsigned int)(b >> 32)) atomicOr(bits + w + 1, (unsigned int)(b >> 32));
  }
}

// ---------------------------------------------------------------------------------------
// select_next_batch (acquisition.py:116-144) over a stored acquisition array -- or, M >= 1,
// over the exact hypervolume improvement computed from the UCB arrays in the same pass (the
// HVI of bo_hvi.hip, written to acq as it is computed).  One HBM pass at stream rate, any
// q <= BO_MAX_TOPQ.  Each wave keeps its running top-q sorted in lanes 0..q-1 and the list's
// q-th entry T wave-uniform; the sweep loads U elements per lane and looks again only at the
// elements not below T (one compare per element; NaN passes).  When some element beats T (an
// "event": every batch of a wave's first step, rarely later):
//  * more than 64 such elements: the q-th best of the lanes' best ones (bitonic over 64 lanes)
//    bounds them -- q elements are not worse than it -- and only the elements not worse than
//    the bound are taken (normally q .. 2q); the rest stay pending and are taken in a second
//    round only if they still beat the updated T (when the bound's q elements included
//    evaluated points);
//  * the taken elements are compacted into LDS, 64 at a time one per lane, tested against the
//    evaluated points (hash set, built in LDS by every workgroup, else in the workspace) and
//    inserted by ranks (wave_rank_insert; the first insert of a wave sorts instead).
// Every wave writes its list to `partial` ([blocks * 4][q]); bo_topq_merge_kernel merges them.
// The first round-2 version kept a sorted top-Q per thread (Q = 8/16/24 >= q + 4, exclusion
// deferred to the list entries): 100-300 KB of unrolled code per instantiation and up to 400
// VGPRs (scratch at Q = 24) -- 38 us at C3 and 1.9 ms at C5 (q = 16) for 8 / 32 MB.
// ---------------------------------------------------------------------------------------
struct HviIn {
  const double* ucb;          // [M][ld]
  long long ld;
  const double* boxes;        // [n_boxes][2 M]
  long long n_boxes;
  double shift[BO_MAX_OBJ], scale[BO_MAX_OBJ];
  double* acq_out;
};

// LDS written by some lanes of a wave and read back by others: keep the compiler's order (the
// LDS executes one wave's operations in issue order).
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Insert the entries (nv, ni) of the lanes with `pass` into the wave's list (sorted in lanes
// 0..q-1, q <= 64; empty entries have i = -1).  Every list entry and every new entry counts the
// entries before it in selection order -- its rank in the union: list entries know their own
// position and compare with the new ones, new entries compare with both (v_readlane broadcasts,
// |new| + q rounds) -- and ranks < q are written to LDS slot `rank` of this wave's `buf`.
__device__ __forceinline__ void wave_rank_insert(double& lv, long long& li, double nv, long long ni,
                                                 bool pass, int q, TopEntry* buf) {
  const int lane = threadIdx.x & 63;
  const unsigned long long nb = __ballot(pass);
  if (nb == 0ull) return;
  const unsigned long long kn = bo_order_key(nv, ni), kl = bo_order_key(lv, li);
  int rl = lane, rn = 0;
  for (unsigned long long m = nb; m; m &= m - 1) {
    const int s = __builtin_ctzll(m);
    const unsigned long long sk = bo_readlane_u(kn, s);
    const long long si = bo_readlane_i(ni, s);
    rn += bo_key_before(sk, si, kn, ni) ? 1 : 0;
    rl += bo_key_before(sk, si, kl, li) ? 1 : 0;
  }
  for (int l = 0; l < q; ++l)
    rn += bo_key_before(bo_readlane_u(kl, l), bo_readlane_i(li, l), kn, ni) ? 1 : 0;
  wave_lds_sync();
  if (lane < q && rl < q && BO_IN(rl, 64, "rank insert buf[rl]")) { buf[rl].v = lv; buf[rl].i = li; }
  if (pass && rn < q && BO_IN(rn, 64, "rank insert buf[rn]")) { buf[rn].v = nv; buf[rn].i = ni; }
  wave_lds_sync();
  if (lane < q) { lv = buf[lane].v; li = buf[lane].i; }
}

// ---------------------------------------------------------------------------------------
// Small-q selection (q <= 16), the default for those q.  One workgroup of 16 waves per CU (the
// evaluated points' LDS hash set is built once per CU), U elements per lane, every load in
// flight at once.  Per span of 16 x 64 U elements:
//   * each lane sorts its U elements (order keys, best first) -- its "head" is then its best;
//   * round 1: every wave's best non-excluded element (wave arg-best of the lane heads: DPP
//     inside the 16-lane rows, v_readlane of the 4 row bests; the winner is probed against the
//     evaluated points and, if it is one, its lane moves to its next element);
//   * the q-th best of the 16 wave bests is a bound B for the workgroup: q non-excluded
//     elements are not worse than it, so the workgroup's top-q is not worse than it; a wave
//     whose best is worse than B is done;
//   * the other waves extract up to q - 1 more heads strictly better than B (and than their
//     running list's q-th), probe them in parallel and rank-insert them (wave_rank_insert);
//     an excluded one leaves the batch short and the extraction goes on;
//   * the 16 wave lists are ranked in LDS, 4 lists per wave and level (block_lists_merge).
// select_merge_kernel runs the same machinery over the [blocks][q] lists (each lane one list).
// Round-3 A/B history: a 64-lane bitonic sort of the lane bests at one wave per SIMD took 39 us
// at C3 (q = 3) and 176 us at C5 (q = 16); q arg-best rounds in every wave of 1024 four-wave
// workgroups, 34 / 254 us -- VALU-bound on the 64-bit key compares (an extraction round of
// every wave cost ~2.5 us); the event kernel below: 33 / 79 us.
// ---------------------------------------------------------------------------------------
struct NoExcl {
  __device__ bool operator()(long long) const { return false; }
};
struct SelExcl {
  const SelArgs* a;
  const unsigned long long* hk;
  const int* hi;
  unsigned int hm;
  __device__ bool operator()(long long gi) const {
    return a->n_excl > 0 && cand_excluded(*a, gi - a->cand_offset, hk, hi, hm);
  }
};

// order of (key, index) pairs; valid keys are never 0 (bo_order_key), empty entries have key 0
__device__ __forceinline__ bool kbefore(unsigned long long ka, long long ia, unsigned long long kb, long long ib) {
  return ka > kb || (ka == kb && ia < ib);
}

template <int CTRL>
__device__ __forceinline__ unsigned long long dpp_u64(unsigned long long x) {
  const int lo = __builtin_amdgcn_update_dpp(0, (int)x, CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(x >> 32), CTRL, 0xF, 0xF, false);
  return ((unsigned long long)(unsigned int)hi << 32) | (unsigned int)lo;
}
template <int CTRL>
__device__ __forceinline__ void dpp_best_step(unsigned long long& k, long long& i) {
  const unsigned long long ok = dpp_u64<CTRL>(k);
  const long long oi = (long long)dpp_u64<CTRL>((unsigned long long)i);
  const bool t = kbefore(ok, oi, k, i);
  k = t ? ok : k;
  i = t ? oi : i;
}
// The wave's best (order key, index) over the lanes' (k, i), wave-uniform: quad_perm xor 1 and
// xor 2, row_half_mirror, row_mirror (every lane of a 16-lane row then holds the row's best),
// then the 4 row bests by v_readlane.
__device__ __forceinline__ void wave_argbest(unsigned long long k, long long i, unsigned long long& wk,
                                             long long& wi) {
  dpp_best_step<0xB1>(k, i);
  dpp_best_step<0x4E>(k, i);
  dpp_best_step<0x141>(k, i);
  dpp_best_step<0x140>(k, i);
  wk = bo_readlane_u(k, 0);
  wi = bo_readlane_i(i, 0);
#pragma unroll
  for (int r = 16; r < 64; r += 16) {
    const unsigned long long rk = bo_readlane_u(k, r);
    const long long ri = bo_readlane_i(i, r);
    const bool t = kbefore(rk, ri, wk, wi);
    wk = t ? rk : wk;
    wi = t ? ri : wi;
  }
}

// A lane's U entries, sorted best first, and the position of its head (the best not taken).
template <int U>
struct LaneRun {
  unsigned long long k[U];
  long long i[U];
  int h;
  __device__ __forceinline__ void sort() {
    auto cx = [&](int x, int y) {
      const bool sw = kbefore(k[y], i[y], k[x], i[x]);
      const unsigned long long tk = k[x];
      const long long ti = i[x];
      k[x] = sw ? k[y] : k[x];
      i[x] = sw ? i[y] : i[x];
      k[y] = sw ? tk : k[y];
      i[y] = sw ? ti : i[y];
    };
    if constexpr (U == 2) cx(0, 1);
    if constexpr (U == 4) { cx(0, 1); cx(2, 3); cx(0, 2); cx(1, 3); cx(1, 2); }
    static_assert(U == 1 || U == 2 || U == 4, "sorting network for U in {1, 2, 4}");
  }
  __device__ __forceinline__ void head(unsigned long long& hk, long long& hi) const {
    hk = 0ull;
    hi = -1;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      hk = h == u ? k[u] : hk;
      hi = h == u ? i[u] : hi;
    }
  }
};

// Extract this wave's entries strictly better than (bk, bi) -- and than the running list's q-th
// -- up to q of them, excluded ones skipped, into the list (lv, li: lanes 0..q-1 sorted).  `first`
// (wave-uniform, optional) is an entry already taken from the lanes, inserted with the batch.
template <int U, class EX>
__device__ __forceinline__ void wave_extract(LaneRun<U>& r, unsigned long long bk, long long bi, double& lv,
                                             long long& li, int q, TopEntry* rbuf, const EX& excluded,
                                             unsigned long long fk, long long fi) {
  const int lane = threadIdx.x & 63;
  for (;;) {
    // the tighter of the bound and the list's q-th entry
    const double lq = bo_readlane_d(lv, q - 1);
    const long long lqi = bo_readlane_i(li, q - 1);
    const unsigned long long lk = bo_order_key(lq, lqi);
    if (kbefore(lk, lqi, bk, bi)) { bk = lk; bi = lqi; }
    double nv = -__builtin_inf();
    long long ni = -1;
    int nb = 0;
    if (fk) {                                   // the pre-taken entry (already probed)
      if (lane == 0) { nv = bo_key_value(fk); ni = fi; }
      nb = 1;
      fk = 0ull;
    }
    const int first_new = nb;
    for (; nb < q; ++nb) {
      unsigned long long hk;
      long long hi;
      r.head(hk, hi);
      unsigned long long wk;
      long long wi;
      wave_argbest(hk, hi, wk, wi);
      if (wk == 0ull || !kbefore(wk, wi, bk, bi)) break;
      if (hi == wi) ++r.h;                       // the owner lane moves to its next entry
      if (lane == nb) { nv = bo_key_value(wk); ni = wi; }
    }
    if (nb == 0) return;
    const bool probe = lane >= first_new && lane < nb;
    const bool ex = probe && excluded(ni);
    const bool ok = lane < nb && !ex;
    wave_rank_insert(lv, li, nv, ni, ok, q, rbuf);
    if (nb < q || __ballot(ex) == 0ull) return;  // the batch ended at the bound, or nothing was excluded
  }
}

// The nw wave lists in wl[w q .. w q + q) (LDS, flat, sorted) merged into dst[0..q) (empty slots
// -inf / -1): groups of 4 lists (4 q <= 64 contiguous entries, one per lane) ranked by one wave
// each, level by level (the next level's lists again flat at wl[g q]).  Every thread of the
// workgroup calls it.
__device__ __forceinline__ void block_lists_merge(TopEntry* wl, int nw, int q, TopEntry* dst) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (nw == 1) {
    __syncthreads();
    if (threadIdx.x < q) dst[threadIdx.x] = wl[threadIdx.x];
    return;
  }
  for (; nw > 1; nw = (nw + 3) / 4) {
    __syncthreads();
    const int groups = (nw + 3) / 4;
    TopEntry e = {-__builtin_inf(), -1};
    int rank = 64;
    bool mine = false;
    if (wave < groups) {
      const int l0 = 4 * wave, nl = nw - l0 < 4 ? nw - l0 : 4, n = nl * q;
      const TopEntry* g = wl + l0 * q;
      mine = lane < n;
      if (mine) e = g[lane];
      const unsigned long long ke = bo_order_key(e.v, e.i);
      rank = 0;
      for (int t = 0; t < n; ++t) {
        const TopEntry o = g[t];
        rank += kbefore(bo_order_key(o.v, o.i), o.i, ke, e.i) ? 1 : 0;
      }
    }
    __syncthreads();
    if (wave < groups) {
      // valid entries have distinct indices (distinct ranks); empty slots fill the rest
      const int nvalid = __popcll(__ballot(mine && e.i >= 0));
      TopEntry* out = nw <= 4 ? dst : wl + wave * q;
      if (mine && e.i >= 0 && rank < q) out[rank] = e;
      if (lane >= nvalid && lane < q) out[lane] = TopEntry{-__builtin_inf(), -1};
    }
  }
}

// One span of the workgroup (16 waves): round 1, the bound, the rest (see above).  Every thread
// of the workgroup calls it.
// NW waves per workgroup (<= 16); SORTED: the lanes' entries arrive sorted (the merge's lists).
template <int U, int NW, bool SORTED, class EX>
__device__ __forceinline__ void block_span_select(LaneRun<U>& r, double& lv, long long& li, int q,
                                                  TopEntry* rbuf, TopEntry* wmax, const EX& excluded) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if constexpr (!SORTED) r.sort();
  r.h = 0;
  // round 1: the wave's best non-excluded element (probed by lane 0)
  unsigned long long wk;
  long long wi;
  for (;;) {
    unsigned long long hk;
    long long hi;
    r.head(hk, hi);
    wave_argbest(hk, hi, wk, wi);
    if (wk == 0ull) break;
    if (hi == wi) ++r.h;
    const bool ex = __ballot(lane == 0 && excluded(wi)) != 0ull;
    if (!ex) break;
  }
  if (lane == 0) { wmax[wave].v = bo_key_value(wk); wmax[wave].i = wk ? wi : -1; }
  __syncthreads();
  // B: the q-th best of the NW wave bests (lanes 0..NW-1 rank them); empty when fewer than q
  unsigned long long bk = 0ull;
  long long bi = -1;
  {
    const TopEntry me = lane < NW ? wmax[lane] : TopEntry{-__builtin_inf(), -1};
    const unsigned long long mk = bo_order_key(me.v, me.i);
    int rank = 0;
#pragma unroll
    for (int t = 0; t < NW; ++t) {
      const TopEntry o = wmax[t];
      rank += kbefore(bo_order_key(o.v, o.i), o.i, mk, me.i) ? 1 : 0;
    }
    const unsigned long long m = __ballot(lane < NW && me.i >= 0 && rank == q - 1);
    if (m) {
      const int s = __builtin_ctzll(m);
      bk = bo_readlane_u(mk, s);
      bi = bo_readlane_i(me.i, s);
    }
  }
  __syncthreads();                               // wmax is rewritten by the next span
  if (wk == 0ull || kbefore(bk, bi, wk, wi)) return;     // this wave's best is worse than B
  // the wave's best is in; then up to q - 1 more strictly better than B
  wave_extract<U>(r, bk, bi, lv, li, q, rbuf, excluded, wk, wi);
}

// ---------------------------------------------------------------------------------------
// The lean form, when no element needs an exclusion probe (an exclusion mask dropped the
// evaluated points at load, or there are none): the top-q of a wave is q rounds of the wave
// arg-best over the lanes' sorted runs (the owner lane of each winner moves to its next entry),
// produced in selection order -- no bound, no rank insertion -- and the workgroup's top-q is
// q more rounds in wave 0 over the NW x q wave results, one per lane.
// ---------------------------------------------------------------------------------------
// acc := the best U entries (sorted) of acc and nx (both sorted): a bitonic merge
template <int U>
__device__ __forceinline__ void lane_keep_best(LaneRun<U>& acc, const LaneRun<U>& nx) {
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const bool t = kbefore(nx.k[U - 1 - u], nx.i[U - 1 - u], acc.k[u], acc.i[u]);
    acc.k[u] = t ? nx.k[U - 1 - u] : acc.k[u];
    acc.i[u] = t ? nx.i[U - 1 - u] : acc.i[u];
  }
  auto cx = [&](int x, int y) {
    const bool sw = kbefore(acc.k[y], acc.i[y], acc.k[x], acc.i[x]);
    const unsigned long long tk = acc.k[x];
    const long long ti = acc.i[x];
    acc.k[x] = sw ? acc.k[y] : acc.k[x];
    acc.i[x] = sw ? acc.i[y] : acc.i[x];
    acc.k[y] = sw ? tk : acc.k[y];
    acc.i[y] = sw ? ti : acc.i[y];
  };
  if constexpr (U == 2) cx(0, 1);
  if constexpr (U == 4) { cx(0, 2); cx(1, 3); cx(0, 1); cx(2, 3); }
}

// q rounds of the wave arg-best over the lanes' runs (r.h = 0 on entry): round t's winner is
// the wave's t-th best.  Lane t of the wave receives it in (tk, ti) (key 0 / -1: none left).
template <int U>
__device__ __forceinline__ void wave_topq_rounds(LaneRun<U>& r, int q, unsigned long long& tk, long long& ti) {
  const int lane = threadIdx.x & 63;
  tk = 0ull;
  ti = -1;
  for (int t = 0; t < q; ++t) {
    unsigned long long hk;
    long long hi;
    r.head(hk, hi);
    unsigned long long wk;
    long long wi;
    wave_argbest(hk, hi, wk, wi);
    if (wk == 0ull) break;                       // wave-uniform: nothing left
    if (hi == wi) ++r.h;                         // the owner moves on (valid indices are distinct)
    if (lane == t) { tk = wk; ti = wi; }
  }
}

// The workgroup's top-q (q <= 16) of its NW waves' runs: the waves' rounds, their lists through
// LDS (wl: NW * q entries), q rounds in wave 0.  Lane t < q of wave 0 returns entry t in (ov, oi)
// (-inf / -1 when fewer exist); the other waves return at once.  Every thread calls it.
template <int U>
__device__ __forceinline__ bool block_topq_rounds(LaneRun<U>& r, int q, int nw, TopEntry* wl, double& ov,
                                                  long long& oi) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  unsigned long long tk;
  long long ti;
  r.h = 0;
  wave_topq_rounds<U>(r, q, tk, ti);
  if (lane < q) { wl[wave * q + lane].v = tk ? bo_key_value(tk) : -__builtin_inf(); wl[wave * q + lane].i = ti; }
  __syncthreads();
  if (wave != 0) return false;
  LaneRun<1> m;
  const bool mine = lane < nw * q;
  const TopEntry e = mine ? wl[lane] : TopEntry{-__builtin_inf(), -1};
  m.k[0] = e.i >= 0 ? bo_order_key(e.v, 0) : 0ull;
  m.i[0] = e.i;
  m.h = 0;
  wave_topq_rounds<1>(m, q, tk, ti);
  ov = tk ? bo_key_value(tk) : -__builtin_inf();
  oi = ti;
  return true;
}

// Diagnostic build (BO_BUILD_VARIANT=DEF_SEL_TIMING): phase stamps of workgroups 0 and the last
// (wave 0, real-time clock, 10 ns ticks) printed at the end of select_small_kernel.
#ifdef BO_SEL_TIMING
#include <stdio.h>
#define SEL_STAMP(n) _t[n] = wall_clock64()
#else
#define SEL_STAMP(n) ((void)0)
#endif

template <int M, int U>
__global__ __launch_bounds__(1024) void select_small_kernel(SelArgs a, HviIn h) {
  extern __shared__ __attribute__((aligned(16))) unsigned long long lkeys[];   // [lds_slots], then idx
  __shared__ TopEntry rbuf[16][64];
  __shared__ TopEntry wl[16 * 16];
  __shared__ TopEntry wmax[16];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, q = a.topq;
  const unsigned long long* hk = a.hkeys;
  const int* hi = a.hidx;
  unsigned int hm = a.hmask;
  // workgroup spans of 16 x 64 U consecutive elements; load u of lane l of wave w reads
  // element span + 64 (U w + u) + l
  const long long wspan = 64LL * U;
  const long long b_first = (long long)blockIdx.x * 16 * wspan;
  const long long b_stride = (long long)gridDim.x * 16 * wspan;
#ifdef BO_SEL_TIMING
  long long _t[5];
#endif
  SEL_STAMP(0);
  LaneRun<U> run;
  auto load_span = [&](long long s0, LaneRun<U>& dst) {
    if constexpr (M == 0) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const long long j = s0 + wave * wspan + 64 * u + lane;
        const bool in = j < a.n_cand;
        const double v = in ? __builtin_nontemporal_load(a.acq + j) : 0.0;
        const bool ok = in && !xbit(a.xbits, j);
        dst.i[u] = ok ? a.cand_offset + j : -1;
        dst.k[u] = ok ? bo_order_key(v, 0) : 0ull;
      }
    } else {
      // the U elements' UCB loads first, then the boxes outer: one (wave-uniform) load of a box
      // serves the lane's U elements; per element the sum over boxes and the product over
      // objectives run in the standalone scan's order (bit-identical acq)
      double p[U][M], hv[U];
      bool nan[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const long long j = s0 + wave * wspan + 64 * u + lane;
        const bool in = j < a.n_cand;
        nan[u] = false;
        hv[u] = 0.0;
#pragma unroll
        for (int k = 0; k < M; ++k) {
          p[u][k] = __builtin_fma(h.scale[k], in ? __builtin_nontemporal_load(h.ucb + (long long)k * h.ld + j) : 0.0,
                                  h.shift[k]);
          nan[u] = nan[u] || (p[u][k] != p[u][k]);
        }
      }
      const double* b = h.boxes;
      for (long long t = 0; t < h.n_boxes; ++t, b += 2 * M) {
        double lo[M], up[M];
#pragma unroll
        for (int k = 0; k < M; ++k) { lo[k] = b[k]; up[k] = b[M + k]; }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          double w = 1.0;
#pragma unroll
          for (int k = 0; k < M; ++k) {
            const double hi2 = p[u][k] < up[k] ? p[u][k] : up[k];
            w *= fmax(hi2 - lo[k], 0.0);
          }
          hv[u] += w;
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const long long j = s0 + wave * wspan + 64 * u + lane;
        const bool in = j < a.n_cand;
        const double v = nan[u] ? __builtin_nan("") : hv[u];
        if (in) __builtin_nontemporal_store(v, h.acq_out + j);      // streamed: read by nothing here
        const bool ok = in && !xbit(a.xbits, j);
        dst.i[u] = ok ? a.cand_offset + j : -1;
        dst.k[u] = ok ? bo_order_key(v, 0) : 0ull;
      }
    }
  };
  // the first span's loads go out before the hash build (they need no table)
  if (b_first < a.n_cand) load_span(b_first, run);
  if (a.n_excl == 0) {
    // lean form: nothing to probe (the exclusion mask dropped the evaluated points at load, or
    // there are none); a lane keeps the best U of all its spans, then the rounds
    if (b_first >= a.n_cand) {
#pragma unroll
      for (int u = 0; u < U; ++u) { run.k[u] = 0ull; run.i[u] = -1; }
    }
    run.sort();
    for (long long s0 = b_first + b_stride; s0 < a.n_cand; s0 += b_stride) {   // workgroup-uniform
      LaneRun<U> nx;
      load_span(s0, nx);
      nx.sort();
      lane_keep_best<U>(run, nx);
    }
#ifdef BO_SEL_TIMING
    __builtin_amdgcn_s_waitcnt(0);
#endif
    SEL_STAMP(1);
    double ov;
    long long oi;
    const bool w0 = block_topq_rounds<U>(run, q, 16, wl, ov, oi);
    if (w0 && lane < q) a.partial[(size_t)blockIdx.x * q + lane] = TopEntry{ov, oi};
#ifdef BO_SEL_TIMING
    SEL_STAMP(2);
    if ((blockIdx.x == 0 || blockIdx.x == gridDim.x - 1) && threadIdx.x == 0)
      printf("lean sel block %d: loads %lld rounds %lld ticks (x10 ns)\n", (int)blockIdx.x, _t[1] - _t[0],
             _t[2] - _t[1]);
#endif
    return;
  }
  if (a.lds_slots > 0) {
    int* lidx = (int*)(lkeys + a.lds_slots);
    for (int t = tid; t < a.lds_slots; t += blockDim.x) lkeys[t] = 0ull;
    __syncthreads();
    for (int e = tid; e < a.n_excl; e += blockDim.x) {
      const unsigned long long key = bo_point_key(a.excl + (long long)e * a.dim, a.dim);
      if (key != 0ull) bo_hash_insert(lkeys, lidx, (unsigned int)a.lds_slots - 1, key, e);
    }
    if (!BO_IN(a.n_excl, a.lds_slots / 2 + 1, "LDS hash load")) return;
    __syncthreads();
    hk = lkeys;
    hi = lidx;
    hm = (unsigned int)a.lds_slots - 1;
  }
  SEL_STAMP(1);
  const SelExcl ex{&a, hk, hi, hm};
  double lv = -__builtin_inf();
  long long li = -1;
  for (long long s0 = b_first; s0 < a.n_cand; s0 += b_stride) {     // workgroup-uniform
    if (s0 != b_first) load_span(s0, run);
#ifdef BO_SEL_TIMING
    __builtin_amdgcn_s_waitcnt(0);
#endif
    SEL_STAMP(2);
    block_span_select<U, 16, false>(run, lv, li, q, rbuf[wave], wmax, ex);
  }
  SEL_STAMP(3);
  if (lane < q) { wl[wave * q + lane].v = lv; wl[wave * q + lane].i = li; }
  block_lists_merge(wl, 16, q, a.partial + (size_t)blockIdx.x * q);
#ifdef BO_SEL_TIMING
  SEL_STAMP(4);
  if ((blockIdx.x == 0 || blockIdx.x == gridDim.x - 1) && (threadIdx.x == 0 || threadIdx.x == 64 * 15))
    printf("sel block %d wave %d: hash %lld loads %lld span %lld merge %lld ticks (x10 ns)\n", (int)blockIdx.x,
           (int)(threadIdx.x >> 6), _t[1] - _t[0], _t[2] - _t[1], _t[3] - _t[2], _t[4] - _t[3]);
#endif
}

// Final merge of n_lists sorted top-q lists ([n_lists][q], q <= 4): one workgroup of up to 1024
// threads, a lane per list (further lists folded in by the keep-best merge), the lean rounds
// (block_topq_rounds) -- the lists hold no evaluated point.
__global__ __launch_bounds__(1024) void select_rounds_merge_kernel(const TopEntry* __restrict__ L, int n_lists,
                                                                   int q, double* __restrict__ out_v,
                                                                   long long* __restrict__ out_i) {
  __shared__ TopEntry wl[16 * 4];
  const int lane = threadIdx.x & 63;
  LaneRun<4> run;
  // a lane per list; more lists than threads fold in by the keep-best merge
  for (int l = threadIdx.x; l < n_lists || l == (int)threadIdx.x; l += blockDim.x) {
    LaneRun<4> nx;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const TopEntry e = (l < n_lists && u < q) ? L[(size_t)l * q + u] : TopEntry{-__builtin_inf(), -1};
      nx.i[u] = e.i;
      nx.k[u] = e.i >= 0 ? bo_order_key(e.v, 0) : 0ull;
    }
    if (l == (int)threadIdx.x) run = nx;
    else lane_keep_best<4>(run, nx);
  }
  double ov;
  long long oi;
  if (block_topq_rounds<4>(run, q, (int)(blockDim.x >> 6), wl, ov, oi) && lane < q) {
    out_v[lane] = ov;
    out_i[lane] = oi;
  }
}

// Final merge of n_lists sorted top-q lists ([n_lists][q], q <= U <= 16): one workgroup of 4
// waves; a lane holds one list (sorted already), spans of 256 lists.
template <int U>
__global__ __launch_bounds__(256) void select_merge_kernel(const TopEntry* __restrict__ L, long long n_lists,
                                                           int q, double* __restrict__ out_v,
                                                           long long* __restrict__ out_i) {
  __shared__ TopEntry rbuf[4][64];
  __shared__ TopEntry wl[4 * 16];
  __shared__ TopEntry wmax[4];
  __shared__ TopEntry res[16];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  double lv = -__builtin_inf();
  long long li = -1;
  const NoExcl ex;
  LaneRun<U> run;
  for (long long l0 = 0; l0 < n_lists; l0 += 256) {               // workgroup-uniform
    const long long l = l0 + threadIdx.x;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const TopEntry e = (l < n_lists && u < q) ? L[l * q + u] : TopEntry{-__builtin_inf(), -1};
      run.i[u] = e.i;
      run.k[u] = e.i >= 0 ? bo_order_key(e.v, 0) : 0ull;
    }
    block_span_select<U, 4, true>(run, lv, li, q, rbuf[wave], wmax, ex);
  }
  if (lane < q) { wl[wave * q + lane].v = lv; wl[wave * q + lane].i = li; }
  block_lists_merge(wl, 4, q, res);
  __syncthreads();
  if (threadIdx.x < q) {
    const TopEntry e = res[threadIdx.x];
    out_v[threadIdx.x] = e.i >= 0 ? e.v : -__builtin_inf();
    out_i[threadIdx.x] = e.i;
  }
}

template <int M, int U>
__global__ __launch_bounds__(256) void select_stream_kernel(SelArgs a, HviIn h) {
  extern __shared__ __attribute__((aligned(16))) unsigned long long lkeys[];   // [lds_slots], then idx
  __shared__ TopEntry wbuf[4][64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, q = a.topq;
  TopEntry* buf = wbuf[wave];
  // the evaluated points' hash set, in LDS when small (built by every workgroup: no extra
  // launches), else the workspace table, else none (scan)
  const unsigned long long* hk = a.hkeys;
  const int* hi = a.hidx;
  unsigned int hm = a.hmask;
  const long long stride = (long long)gridDim.x * blockDim.x;
  const long long b_first = (long long)blockIdx.x * blockDim.x + wave * 64;
  // M == 0: the first step's loads are issued before the hash build (they need no table)
  double pre[U];
  if constexpr (M == 0) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long j = b_first + u * stride + lane;
      pre[u] = j < a.n_cand ? __builtin_nontemporal_load(a.acq + j) : 0.0;
    }
  }
  if (a.lds_slots > 0) {
    int* lidx = (int*)(lkeys + a.lds_slots);
    for (int t = tid; t < a.lds_slots; t += blockDim.x) lkeys[t] = 0ull;
    __syncthreads();
    for (int e = tid; e < a.n_excl; e += blockDim.x) {
      const unsigned long long key = bo_point_key(a.excl + (long long)e * a.dim, a.dim);
      if (key != 0ull) bo_hash_insert(lkeys, lidx, (unsigned int)a.lds_slots - 1, key, e);
    }
    if (!BO_IN(a.n_excl, a.lds_slots / 2 + 1, "LDS hash load")) return;
    __syncthreads();
    hk = lkeys;
    hi = lidx;
    hm = (unsigned int)a.lds_slots - 1;
  }
  double lv = -__builtin_inf(), tv = -__builtin_inf();   // list entry; the list's q-th (uniform)
  long long li = -1, ti = -1;
  const unsigned long long below = (1ull << lane) - 1ull;
  // wave-uniform trip count: every lane stays in the loop for the ballots and broadcasts
  for (long long b0 = b_first; b0 < a.n_cand; b0 += U * stride) {
    double val[U];
    bool live[U];                     // in range and not masked out (xbits)
    bool any = false;
#pragma unroll
    for (int u = 0; u < U; ++u) {     // all U loads in flight before any element is looked at
      const long long j = b0 + u * stride + lane;
      const bool in = j < a.n_cand;
      live[u] = in && !xbit(a.xbits, j);
      if constexpr (M == 0) {
        val[u] = b0 == b_first ? pre[u] : (in ? __builtin_nontemporal_load(a.acq + j) : 0.0);
      } else {
        double p[M];
        bool nan = false;
#pragma unroll
        for (int k = 0; k < M; ++k) {
          p[k] = __builtin_fma(h.scale[k], in ? __builtin_nontemporal_load(h.ucb + (long long)k * h.ld + j) : 0.0, h.shift[k]);
          nan = nan || (p[k] != p[k]);
        }
        double hv = 0.0;
        const double* b = h.boxes;
        for (long long t = 0; t < h.n_boxes; ++t, b += 2 * M) {
          double w = 1.0;
#pragma unroll
          for (int k = 0; k < M; ++k) {
            const double hi2 = p[k] < b[M + k] ? p[k] : b[M + k];
            w *= fmax(hi2 - b[k], 0.0);
          }
          hv += w;
        }
        val[u] = nan ? __builtin_nan("") : hv;
        if (in) __builtin_nontemporal_store(val[u], h.acq_out + j);
      }
      any = any || (live[u] && !(val[u] < tv));
    }
    if (__ballot(any) == 0ull) continue;
    // ---- event: the elements beating T (exact order) are pending
    bool pend[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long j = b0 + u * stride + lane;
      pend[u] = live[u] && bo_better(val[u], a.cand_offset + j, tv, ti);
    }
    for (;;) {
      int cnt = 0;
#pragma unroll
      for (int u = 0; u < U; ++u) cnt += __popcll(__ballot(pend[u]));
      if (cnt == 0) break;
      double bv = -__builtin_inf();   // the bound (empty: take every pending element)
      long long bix = -1;
      if (cnt > 64) {
        unsigned long long mk = 0ull;
        long long mi = -1;
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const long long gi = a.cand_offset + b0 + u * stride + lane;
          const unsigned long long k = pend[u] ? bo_order_key(val[u], gi) : 0ull;
          const bool b = bo_key_before(k, gi, mk, mi);
          mk = b ? k : mk;
          mi = b ? gi : mi;
        }
        double mv = bo_key_value(mk);
        bo_wave_sort64(mv, mi);
        bv = bo_readlane_d(mv, q - 1);
        bix = bo_readlane_i(mi, q - 1);
      }
      bool take[U];
      int off[U], total = 0;
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const long long gi = a.cand_offset + b0 + u * stride + lane;
        take[u] = pend[u] && !bo_better(bv, bix, val[u], gi);
        const unsigned long long bb = __ballot(take[u]);
        off[u] = total + __popcll(bb & below);
        total += __popcll(bb);
      }
#pragma unroll 1
      for (int c0 = 0; c0 < total; c0 += 64) {
        wave_lds_sync();
#pragma unroll
        for (int u = 0; u < U; ++u)
          if (take[u] && off[u] >= c0 && off[u] < c0 + 64 && BO_IN(off[u] - c0, 64, "chunk buf[off - c0]")) {
            buf[off[u] - c0].v = val[u];
            buf[off[u] - c0].i = a.cand_offset + b0 + u * stride + lane;
          }
        wave_lds_sync();
        bool p = lane < total - c0;
        const double nv = p ? buf[lane].v : -__builtin_inf();
        const long long ni = p ? buf[lane].i : -1;
        p = p && bo_better(nv, ni, tv, ti);
        if (a.n_excl > 0 && p && BO_IN(ni - a.cand_offset, a.n_cand, "chunk candidate"))
          p = !cand_excluded(a, ni - a.cand_offset, hk, hi, hm);
        if (__ballot(p) == 0ull) continue;
        if (bo_readlane_i(li, 0) < 0 && __popcll(__ballot(p)) > 24) {
          // empty list and a large chunk: the sorted chunk's head is the list (rank insertion
          // costs |chunk| + q broadcast rounds)
          double sv = p ? nv : -__builtin_inf();
          long long si = p ? ni : -1;
          bo_wave_sort64(sv, si);
          lv = lane < q ? sv : -__builtin_inf();
          li = lane < q ? si : -1;
        } else {
          wave_rank_insert(lv, li, nv, ni, p, q, buf);
        }
        tv = bo_readlane_d(lv, q - 1);
        ti = bo_readlane_i(li, q - 1);
      }
      // what the bound held back stays pending only while it still beats T
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const long long gi = a.cand_offset + b0 + u * stride + lane;
        pend[u] = pend[u] && !take[u] && bo_better(val[u], gi, tv, ti);
      }
    }
  }
  if (lane < q && BO_IN(((long long)blockIdx.x * 4 + wave) * q + lane, a.partial_cap, "partial list entry")) {
    TopEntry* dst = a.partial + ((size_t)blockIdx.x * 4 + wave) * q;
    dst[lane].v = lv;
    dst[lane].i = li;
  }
}

template <int M>
int launch_select_stream(const SelArgs& a, const HviIn& h, int blocks, hipStream_t s) {
  const size_t lds = (size_t)a.lds_slots * 12;
  hipLaunchKernelGGL((select_stream_kernel<M, M == 0 ? 8 : 4>), dim3(blocks), dim3(256), lds, s, a, h);
  BO_CHECK_HIP(hipGetLastError());
  return BO_OK;
}

// elements per lane and span of select_small_kernel
constexpr int kSmallU0 = 4;       // stored acquisition array: 4 loads of 8 B per lane, 16 waves per CU
constexpr int kSmallUM = 4;       // exact HVI from the UCB arrays
#ifdef BO_ABL_OLDSELECT
constexpr int kSmallQ = 0;        // A/B: every q through select_stream_kernel + bo_topq_merge_kernel
#else
constexpr int kSmallQ = 4;        // q up to this: select_small_kernel + select_merge_kernel (faster at
                                  // q <= 4; at q = 16 the event kernel: C3 44 vs 80 us, C5 79 vs 151 us)
#endif

template <int M>
int launch_select_small(const SelArgs& a, const HviIn& h, int blocks, hipStream_t s) {
  const size_t lds = (size_t)a.lds_slots * 12;
  hipLaunchKernelGGL((select_small_kernel<M, M == 0 ? kSmallU0 : kSmallUM>), dim3(blocks), dim3(1024), lds, s, a, h);
  BO_CHECK_HIP(hipGetLastError());
  return BO_OK;
}

// --------------------------------------------------------------------------- Pareto
// mask[i] = 0 iff some row j (j != i) weakly dominates row i under maximisation:
// y_j >= y_i in every objective and y_j > y_i in at least one (pareto.py:35-41 with
// y negated).  Comparisons only: bit-exact, NaN never dominates nor is dominated.
// The reference's scan order (break on the first dominator, marks only rows it
// reaches) yields exactly this set; see oracle/oracle_np.py:is_pareto_efficient.
__global__ __launch_bounds__(256) void pareto_kernel(const double* __restrict__ y, long long n,
                                                     int n_obj, uint8_t* __restrict__ mask) {
  __shared__ double tile[256 * BO_MAX_OBJ];
  const long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  double yi[BO_MAX_OBJ];
  for (int o = 0; o < BO_MAX_OBJ; ++o) yi[o] = (i < n && o < n_obj) ? y[i * n_obj + o] : 0.0;
  bool dominated = false;
  for (long long t0 = 0; t0 < n; t0 += 256) {
    __syncthreads();
    const long long tj = t0 + threadIdx.x;
    for (int o = 0; o < n_obj; ++o) tile[threadIdx.x * n_obj + o] = tj < n ? y[tj * n_obj + o] : 0.0;
    __syncthreads();
    const int cnt = (int)(n - t0 < 256 ? n - t0 : 256);
    if (i < n && !dominated) {
      for (int t = 0; t < cnt; ++t) {
        bool ge = true, gt = false;
        for (int o = 0; o < n_obj; ++o) {
          const double yj = tile[t * n_obj + o];
          ge = ge && (yj >= yi[o]);
          gt = gt || (yj > yi[o]);
        }
        if (ge && gt) { dominated = true; break; }
      }
    }
  }
  if (i < n) mask[i] = dominated ? 0 : 1;
}

// partial lists: <= 1024 workgroups x 4 waves x q entries
size_t sel_lists_bytes(int topq) {
  const size_t e = (size_t)1024 * 4 * (topq > 0 ? topq : 1);
  return (e > 8192 ? e : 8192) * sizeof(TopEntry);
}

int cus_count() {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    hipDeviceProp_t p;
    if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&p, dev) != hipSuccess) return 256;
    cus = p.multiProcessorCount;
  }
  return cus;
}

}  // namespace

// Internal (bo_predict.hip): the final merge of the fused kernel's per-wave lists by the lean
// rounds when q <= 4 (returns false otherwise: the caller's general merge)
bool bo_launch_rounds_merge(const TopEntry* lists, long long n_lists, int q, double* out_v, int64_t* out_i,
                            hipStream_t s) {
  if (q < 1 || q > 4 || n_lists < 1 || n_lists > (1LL << 30)) return false;
  const long long t = n_lists < 1024 ? n_lists : 1024;
  const unsigned threads = (unsigned)((t + 63) / 64 * 64);
  hipLaunchKernelGGL(select_rounds_merge_kernel, dim3(1), dim3(threads), 0, s, lists, (int)n_lists, q, out_v,
                     (long long*)out_i);
  return hipGetLastError() == hipSuccess;
}

extern "C" {

int bo_update_k(double* km, int64_t ld, int32_t n_obj, const double* x, int32_t dim,
                int64_t last_eval, int64_t cur, const double* pv, const double* ls, void* stream) {
  if (!km || !x || !pv || !ls || n_obj < 1 || n_obj > BO_MAX_OBJ || dim < 1 || ld < cur ||
      last_eval < 0 || cur > (1 << 20))
    return BO_ERR_ARG;
  if (cur <= last_eval) return BO_OK;
  HostParams p;
  memset(&p, 0, sizeof(p));
  for (int o = 0; o < n_obj; ++o) { p.a[o] = pv[o]; p.b[o] = ls[o] * ls[o]; }
  const int rows = (int)(cur - last_eval);
  dim3 grid((unsigned)((cur + 127) / 128), (unsigned)rows);
  hipLaunchKernelGGL(gram_kernel, grid, dim3(128), 0, (hipStream_t)stream, km, (long long)ld,
                     n_obj, x, dim, (int)last_eval, (int)cur, p);
  BO_CHECK_HIP(hipGetLastError());
  return BO_OK;
}

int bo_update_k_star(double* ks, int64_t ld_rows, int32_t n_obj, const double* x, int32_t dim,
                     int32_t kind, const void* cand, int64_t n_cand, int64_t last_eval,
                     int64_t cur, const double* pv, const double* ls, void* stream) {
  if (!ks || !x || !cand || !pv || !ls || n_obj < 1 || n_obj > BO_MAX_OBJ || dim < 1 ||
      ld_rows < cur || (kind != BO_CAND_I64 && kind != BO_CAND_F64) || last_eval < 0)
    return BO_ERR_ARG;
  if (cur <= last_eval || n_cand == 0) return BO_OK;
  HostParams p;
  memset(&p, 0, sizeof(p));
  for (int o = 0; o < n_obj; ++o) { p.a[o] = pv[o]; p.b[o] = ls[o] * ls[o]; }
  dim3 grid((unsigned)((n_cand + 255) / 256), (unsigned)(cur - last_eval));
  hipLaunchKernelGGL(kstar_kernel, grid, dim3(256), 0, (hipStream_t)stream, ks,
                     (long long)ld_rows, n_obj, x, dim, kind, cand, (long long)n_cand,
                     (int)last_eval, (int)cur, p);
  BO_CHECK_HIP(hipGetLastError());
  return BO_OK;
}

int bo_standardize_ucb_hvi(double* smu, double* svar, double* ucb, double* acq, const double* mu,
                           const double* var, int32_t n_obj, int64_t n, const double* pm,
                           const double* pv, const double* betas, void* stream) {
  if (!mu || !var || !pm || !pv || !betas || n_obj < 1 || n_obj > BO_MAX_OBJ || n < 0)
    return BO_ERR_ARG;
  if (n == 0) return BO_OK;
  HostParams p, q;
  memset(&p, 0, sizeof(p));
  memset(&q, 0, sizeof(q));
  for (int o = 0; o < n_obj; ++o) {
    p.a[o] = pm[o];
    p.b[o] = pv[o];
    p.c[o] = betas[o];
    q.a[o] = sqrt(pv[o]);
  }
  hipLaunchKernelGGL(std_ucb_hvi_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, smu, svar, ucb, acq, mu, var, n_obj, (long long)n, p, q);
  BO_CHECK_HIP(hipGetLastError());
  return BO_OK;
}

int bo_update_ucb(double* ucb, const double* mu, const double* var, int32_t n_obj, int64_t n,
                  const double* betas, void* stream) {
  if (!ucb || !mu || !var || !betas || n_obj < 1 || n_obj > BO_MAX_OBJ || n < 0) return BO_ERR_ARG;
  if (n == 0) return BO_OK;
  HostParams p;
  memset(&p, 0, sizeof(p));
  for (int o = 0; o < n_obj; ++o) p.a[o] = betas[o];
  hipLaunchKernelGGL(ucb_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, ucb, mu, var, n_obj, (long long)n, p);
  BO_CHECK_HIP(hipGetLastError());
  return BO_OK;
}

int bo_update_hypervolume_improvement(double* acq, const double* ucb, int32_t n_obj, int64_t n,
                                      void* stream) {
  if (!acq || !ucb || n_obj < 1 || n < 0) return BO_ERR_ARG;
  if (n == 0) return BO_OK;
  hipLaunchKernelGGL(hvi_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, acq, ucb, n_obj, (long long)n);
  BO_CHECK_HIP(hipGetLastError());
  return BO_OK;
}

size_t bo_select_topq_workspace_size(int64_t n_cand, int32_t topq) {
  const size_t lists = sel_lists_bytes(topq);
  const size_t bits = ((size_t)(n_cand > 0 ? n_cand : 0) + 31) / 32 * 4;
  return lists + (bits + 255) / 256 * 256;
}

}  // extern "C"

namespace {

// select_next_batch over an acquisition array (m == 0) or over the exact HVI computed from the
// UCB arrays in the same pass (m >= 1, `h`), written into h->acq_out first.
int select_impl(const double* acq, int64_t n_cand, int32_t kind, const void* cand,
                const int64_t* grid_lo, const int64_t* grid_shape, int32_t dim,
                int64_t cand_offset, const double* excl, int64_t n_excl, int32_t topq,
                double* top_val, int64_t* top_idx, void* ws, size_t ws_bytes, hipStream_t s,
                const HviIn* h, int m, const unsigned int* xbits = nullptr) {
  static const int64_t kOne[BO_MAX_DIM] = {1, 1, 1, 1, 1, 1, 1, 1};
  static const int64_t kZero[BO_MAX_DIM] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (xbits) {                            // the mask replaces the points: no candidate decode
    kind = BO_CAND_GRID;
    cand = nullptr;
    grid_lo = kZero;
    grid_shape = kOne;
    dim = 1;
    excl = nullptr;
    n_excl = 0;
  }
  if ((!acq && m == 0) || topq < 1 || topq > BO_MAX_TOPQ || dim < 1 || dim > BO_MAX_DIM ||
      n_cand < 0 || !top_val || !top_idx || (n_excl > 0 && !excl) || kind < 0 || kind > BO_CAND_SOBOL)
    return BO_ERR_ARG;
  if (kind != BO_CAND_GRID && !cand) return BO_ERR_ARG;
  if (kind == BO_CAND_GRID && (!grid_lo || !grid_shape)) return BO_ERR_ARG;
  if (!ws || ws_bytes < bo_select_topq_workspace_size(n_cand, topq)) return BO_ERR_WORKSPACE;
  SelArgs a;
  memset(&a, 0, sizeof(a));
  a.xbits = xbits;
  a.acq = acq;
  a.n_cand = n_cand;
  a.cand_offset = cand_offset;
  a.kind = kind;
  a.dim = dim;
  a.n_excl = (int)n_excl;
  a.topq = topq;
  a.cand = cand;
  if (kind == BO_CAND_SOBOL) {            // `cand` is a host bo_sobol_desc*
    const int st = bo_sobol_fill(&a.sob, dim, (const bo_sobol_desc*)cand);
    if (st != BO_OK) return st;
    a.cand = nullptr;
  }
  for (int k = 0; k < BO_MAX_DIM; ++k) a.grid_shape[k] = 1;
  if (kind == BO_CAND_GRID) {
    for (int k = 0; k < dim; ++k) {
      if (grid_shape[k] <= 0) return BO_ERR_ARG;
      a.grid_lo[k] = grid_lo[k];
      a.grid_shape[k] = grid_shape[k];
    }
    a.idx32 = cand_offset >= 0 && cand_offset + n_cand < (1LL << 31) ? 1 : 0;
    for (int k = 0; k < dim; ++k)
      if (grid_shape[k] >= (1LL << 31)) a.idx32 = 0;
  }
  a.excl = excl;
  a.partial = (TopEntry*)ws;
  a.partial_cap = (long long)(sel_lists_bytes(topq) / sizeof(TopEntry));
  if (n_excl > 0 && n_cand > 0) {
    // the evaluated points' hash set: per workgroup in LDS (<= 1024 points),
    // else in the workspace region after the lists when it fits (2 n_excl .. 4 n_excl slots of
    // 12 B), else none (the exclusion scans the points)
    const unsigned int slots = bo_hash_slots(n_excl);
    const size_t region = ((size_t)n_cand + 31) / 32 * 4;
    if (n_excl <= 1024) {
      a.lds_slots = (int)slots;
    } else if ((size_t)slots * 12 <= region) {
      unsigned long long* keys = (unsigned long long*)((char*)ws + sel_lists_bytes(topq));
      int* idx = (int*)(keys + slots);
      BO_CHECK_HIP(hipMemsetAsync(keys, 0, (size_t)slots * 8, s));
      hipLaunchKernelGGL(excl_hash_kernel, dim3((unsigned)((n_excl + 255) / 256)), dim3(256), 0, s,
                         keys, idx, slots - 1, excl, 0, (int)n_excl, dim);
      BO_CHECK_HIP(hipGetLastError());
      a.hkeys = keys;
      a.hidx = idx;
      a.hmask = slots - 1;
    }
  }
  HviIn hz;
  memset(&hz, 0, sizeof(hz));
  const HviIn& hv = h ? *h : hz;
  int st;
  if (topq <= kSmallQ) {
    // one span (16 waves x 64 U elements) per workgroup, one workgroup per CU; [blocks][q] lists
    const long long per_block = 16LL * 64 * (m == 0 ? kSmallU0 : kSmallUM);
    long long blocks = (n_cand + per_block - 1) / per_block;
    const int max_blocks = cus_count() < 1024 ? cus_count() : 1024;
    if (blocks > max_blocks) blocks = max_blocks;
    if (blocks < 1) blocks = 1;
    switch (m) {
      case 0: st = launch_select_small<0>(a, hv, (int)blocks, s); break;
      case 1: st = launch_select_small<1>(a, hv, (int)blocks, s); break;
      case 2: st = launch_select_small<2>(a, hv, (int)blocks, s); break;
      case 3: st = launch_select_small<3>(a, hv, (int)blocks, s); break;
      case 4: st = launch_select_small<4>(a, hv, (int)blocks, s); break;
      default: return BO_ERR_UNSUPPORTED;
    }
    if (st != BO_OK) return st;
    static_assert(kSmallQ <= 4, "the merge kernels hold q <= 4 entries per list");
    if (blocks <= 1024) {          // a lane per list (blocks <= 1024 always: max_blocks above)
      const unsigned threads = (unsigned)((blocks + 63) / 64 * 64);
      hipLaunchKernelGGL(select_rounds_merge_kernel, dim3(1), dim3(threads), 0, s, (const TopEntry*)ws,
                         (int)blocks, topq, top_val, (long long*)top_idx);
    } else {
      hipLaunchKernelGGL(select_merge_kernel<4>, dim3(1), dim3(256), 0, s, (const TopEntry*)ws, blocks,
                         topq, top_val, (long long*)top_idx);
    }
    BO_CHECK_HIP(hipGetLastError());
    return BO_OK;
  }
  // U = 8 elements per thread and step (M == 0): one workgroup per 2048 elements, at most 4 per
  // CU (16 waves; the whole C3 array in flight at once); [blocks * 4][q] lists for the merge
  const long long per_block = 256LL * (m == 0 ? 8 : 4);
  long long blocks = (n_cand + per_block - 1) / per_block;
  const int max_blocks = 4 * cus_count() < 1024 ? 4 * cus_count() : 1024;
  if (blocks > max_blocks) blocks = max_blocks;
  if (blocks < 1) blocks = 1;
  switch (m) {
    case 0: st = launch_select_stream<0>(a, hv, (int)blocks, s); break;
    case 1: st = launch_select_stream<1>(a, hv, (int)blocks, s); break;
    case 2: st = launch_select_stream<2>(a, hv, (int)blocks, s); break;
    case 3: st = launch_select_stream<3>(a, hv, (int)blocks, s); break;
    case 4: st = launch_select_stream<4>(a, hv, (int)blocks, s); break;
    default: return BO_ERR_UNSUPPORTED;
  }
  if (st != BO_OK) return st;
  hipLaunchKernelGGL(bo_topq_merge_kernel, dim3(1), dim3(256), 0, s, (const TopEntry*)ws,
                     blocks * 4, topq, top_val, (long long*)top_idx);
  BO_CHECK_HIP(hipGetLastError());
  return BO_OK;
}

}  // namespace

extern "C" {

int bo_select_topq(const double* acq, int64_t n_cand, int32_t kind, const void* cand,
                   const int64_t* grid_lo, const int64_t* grid_shape, int32_t dim,
                   int64_t cand_offset, const double* excl, int64_t n_excl, int32_t topq,
                   double* top_val, int64_t* top_idx, void* ws, size_t ws_bytes, void* stream) {
  return select_impl(acq, n_cand, kind, cand, grid_lo, grid_shape, dim, cand_offset, excl, n_excl,
                     topq, top_val, top_idx, ws, ws_bytes, (hipStream_t)stream, nullptr, 0);
}

int bo_hvi_select_topq(double* acq, const double* ucb, int64_t ld, int64_t n_cand, int32_t n_obj,
                       const double* shift, const double* scale, const double* boxes,
                       int64_t n_boxes, int32_t kind, const void* cand, const int64_t* grid_lo,
                       const int64_t* grid_shape, int32_t dim, int64_t cand_offset,
                       const double* excl, int64_t n_excl, int32_t topq, double* top_val,
                       int64_t* top_idx, void* ws, size_t ws_bytes, void* stream) {
  if (!acq || !ucb || !shift || !scale || n_obj < 1 || n_obj > 4 || ld < n_cand || n_boxes < 0 ||
      (n_boxes > 0 && !boxes))
    return BO_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  HviIn h;
  memset(&h, 0, sizeof(h));
  h.ucb = ucb;
  h.ld = ld;
  h.boxes = boxes;
  h.n_boxes = n_boxes;
  for (int k = 0; k < n_obj; ++k) { h.shift[k] = shift[k]; h.scale[k] = scale[k]; }
  h.acq_out = acq;
  return select_impl(acq, n_cand, kind, cand, grid_lo, grid_shape, dim, cand_offset, excl, n_excl,
                     topq, top_val, top_idx, ws, ws_bytes, s, &h, n_obj);
}

size_t bo_excl_mask_bytes(int64_t n_cand) {
  const size_t words = ((size_t)(n_cand > 0 ? n_cand : 0) + 31) / 32 + 2;
  return (words * 4 + 255) / 256 * 256;
}

size_t bo_excl_mask_workspace_size(int64_t n_excl) {
  return (size_t)bo_hash_slots(n_excl > 0 ? n_excl : 0) * 12 + 256;
}

int bo_excl_mask_update(uint32_t* mask, int64_t n_cand, int32_t kind, const void* cand,
                        const int64_t* grid_lo, const int64_t* grid_shape, int32_t dim,
                        int64_t cand_offset, const double* excl, int64_t first_excl, int64_t n_excl,
                        int32_t clear, void* ws, size_t ws_bytes, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (!mask || n_cand < 0 || dim < 1 || dim > BO_MAX_DIM || first_excl < 0 || n_excl < first_excl ||
      n_excl > (1LL << 30) || (n_excl > first_excl && !excl) || kind < 0 || kind > BO_CAND_SOBOL)
    return BO_ERR_ARG;
  if (kind != BO_CAND_GRID && !cand) return BO_ERR_ARG;
  if (kind == BO_CAND_GRID && (!grid_lo || !grid_shape)) return BO_ERR_ARG;
  if (clear) BO_CHECK_HIP(hipMemsetAsync(mask, 0, bo_excl_mask_bytes(n_cand), s));
  if (n_excl == first_excl || n_cand == 0) return BO_OK;
  SelArgs a;
  memset(&a, 0, sizeof(a));
  a.n_cand = n_cand;
  a.cand_offset = cand_offset;
  a.kind = kind;
  a.dim = dim;
  a.n_excl = (int)n_excl;
  a.cand = cand;
  a.excl = excl;
  for (int k = 0; k < BO_MAX_DIM; ++k) a.grid_shape[k] = 1;
  bool arith = kind == BO_CAND_GRID;
  if (kind == BO_CAND_SOBOL) {
    const int st = bo_sobol_fill(&a.sob, dim, (const bo_sobol_desc*)cand);
    if (st != BO_OK) return st;
    a.cand = nullptr;
  }
  if (kind == BO_CAND_GRID) {
    unsigned long long total = 1;
    for (int k = 0; k < dim; ++k) {
      if (grid_shape[k] <= 0) return BO_ERR_ARG;
      a.grid_lo[k] = grid_lo[k];
      a.grid_shape[k] = grid_shape[k];
      const long long lim = 1LL << 53;          // every grid coordinate exact in f64
      if (grid_lo[k] <= -lim || grid_lo[k] >= lim || grid_shape[k] >= lim - grid_lo[k]) arith = false;
      total = total * (unsigned long long)grid_shape[k];
      if (total >= (1ull << 62)) arith = false;
    }
    a.idx32 = cand_offset >= 0 && cand_offset + n_cand < (1LL << 31) ? 1 : 0;
    for (int k = 0; k < dim; ++k)
      if (grid_shape[k] >= (1LL << 31)) a.idx32 = 0;
  }
  const int first = (int)first_excl, cnt = (int)(n_excl - first_excl);
  if (arith) {
    hipLaunchKernelGGL(excl_mask_grid_kernel, dim3((unsigned)((cnt + 255) / 256)), dim3(256), 0, s,
                       (unsigned int*)mask, a, first);
    BO_CHECK_HIP(hipGetLastError());
    return BO_OK;
  }
  // hash set of the new points (rows first .. n_excl) in the workspace, then the candidate scan
  const unsigned int slots = bo_hash_slots(cnt);
  if (!ws || ws_bytes < bo_excl_mask_workspace_size(cnt)) return BO_ERR_WORKSPACE;
  unsigned long long* keys = (unsigned long long*)ws;
  int* idx = (int*)(keys + slots);
  BO_CHECK_HIP(hipMemsetAsync(keys, 0, (size_t)slots * 8, s));
  hipLaunchKernelGGL(excl_hash_kernel, dim3((unsigned)((cnt + 255) / 256)), dim3(256), 0, s, keys, idx,
                     slots - 1, excl, first, (int)n_excl, dim);
  BO_CHECK_HIP(hipGetLastError());
  hipLaunchKernelGGL(excl_mask_scan_kernel, dim3((unsigned)((n_cand + 255) / 256)), dim3(256), 0, s,
                     (unsigned int*)mask, a, (const unsigned long long*)keys, (const int*)idx, slots - 1);
  BO_CHECK_HIP(hipGetLastError());
  return BO_OK;
}

int bo_select_topq_masked(const double* acq, int64_t n_cand, int64_t cand_offset, const uint32_t* mask,
                          int32_t topq, double* top_val, int64_t* top_idx, void* ws, size_t ws_bytes,
                          void* stream) {
  if (!mask) return BO_ERR_ARG;
  return select_impl(acq, n_cand, BO_CAND_GRID, nullptr, nullptr, nullptr, 1, cand_offset, nullptr, 0,
                     topq, top_val, top_idx, ws, ws_bytes, (hipStream_t)stream, nullptr, 0,
                     (const unsigned int*)mask);
}

int bo_hvi_select_topq_masked(double* acq, const double* ucb, int64_t ld, int64_t n_cand, int32_t n_obj,
                              const double* shift, const double* scale, const double* boxes,
                              int64_t n_boxes, int64_t cand_offset, const uint32_t* mask, int32_t topq,
                              double* top_val, int64_t* top_idx, void* ws, size_t ws_bytes,
                              void* stream) {
  if (!acq || !ucb || !shift || !scale || !mask || n_obj < 1 || n_obj > 4 || ld < n_cand ||
      n_boxes < 0 || (n_boxes > 0 && !boxes))
    return BO_ERR_ARG;
  HviIn h;
  memset(&h, 0, sizeof(h));
  h.ucb = ucb;
  h.ld = ld;
  h.boxes = boxes;
  h.n_boxes = n_boxes;
  for (int k = 0; k < n_obj; ++k) { h.shift[k] = shift[k]; h.scale[k] = scale[k]; }
  h.acq_out = acq;
  return select_impl(acq, n_cand, BO_CAND_GRID, nullptr, nullptr, nullptr, 1, cand_offset, nullptr, 0,
                     topq, top_val, top_idx, ws, ws_bytes, (hipStream_t)stream, &h, n_obj,
                     (const unsigned int*)mask);
}

int bo_pareto_mask(const double* y, int64_t n, int32_t n_obj, uint8_t* mask, void* stream) {
  if (!y || !mask || n < 0 || n_obj < 1 || n_obj > BO_MAX_OBJ) return BO_ERR_ARG;
  if (n == 0) return BO_OK;
  hipLaunchKernelGGL(pareto_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, y, (long long)n, n_obj, mask);
  BO_CHECK_HIP(hipGetLastError());
  return BO_OK;
}

}  // extern "C"
