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
  SobolArgs sob;            // kind BO_CAND_SOBOL
};

__global__ void excl_hash_kernel(unsigned long long* __restrict__ keys, int* __restrict__ idx,
                                 unsigned int mask, const double* __restrict__ excl, int n_excl, int dim) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
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
  if (a.kind == BO_CAND_GRID) {          // all coordinates from one chain of divisions
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
      pre[u] = j < a.n_cand ? a.acq[j] : 0.0;
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
    bool any = false;
#pragma unroll
    for (int u = 0; u < U; ++u) {     // all U loads in flight before any element is looked at
      const long long j = b0 + u * stride + lane;
      const bool in = j < a.n_cand;
      if constexpr (M == 0) {
        val[u] = b0 == b_first ? pre[u] : (in ? a.acq[j] : 0.0);
      } else {
        double p[M];
        bool nan = false;
#pragma unroll
        for (int k = 0; k < M; ++k) {
          p[k] = __builtin_fma(h.scale[k], in ? h.ucb[(long long)k * h.ld + j] : 0.0, h.shift[k]);
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
        if (in) h.acq_out[j] = val[u];
      }
      any = any || (in && !(val[u] < tv));
    }
    if (__ballot(any) == 0ull) continue;
    // ---- event: the elements beating T (exact order) are pending
    bool pend[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long j = b0 + u * stride + lane;
      pend[u] = j < a.n_cand && bo_better(val[u], a.cand_offset + j, tv, ti);
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

// --------------------------------------------------------------------------- Pareto
// mask[i] = 0 iff some row j (j != i) weakly dominates row i under maximisation:
// y_j >= y_i in every objective and y_j > y_i in at least one (pareto.py:279-287 with
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
                const HviIn* h, int m) {
  if ((!acq && m == 0) || topq < 1 || topq > BO_MAX_TOPQ || dim < 1 || dim > BO_MAX_DIM ||
      n_cand < 0 || !top_val || !top_idx || (n_excl > 0 && !excl) || kind < 0 || kind > BO_CAND_SOBOL)
    return BO_ERR_ARG;
  if (kind != BO_CAND_GRID && !cand) return BO_ERR_ARG;
  if (kind == BO_CAND_GRID && (!grid_lo || !grid_shape)) return BO_ERR_ARG;
  if (!ws || ws_bytes < bo_select_topq_workspace_size(n_cand, topq)) return BO_ERR_WORKSPACE;
  SelArgs a;
  memset(&a, 0, sizeof(a));
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
  if (kind == BO_CAND_GRID)
    for (int k = 0; k < dim; ++k) {
      if (grid_shape[k] <= 0) return BO_ERR_ARG;
      a.grid_lo[k] = grid_lo[k];
      a.grid_shape[k] = grid_shape[k];
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
                         keys, idx, slots - 1, excl, (int)n_excl, dim);
      BO_CHECK_HIP(hipGetLastError());
      a.hkeys = keys;
      a.hidx = idx;
      a.hmask = slots - 1;
    }
  }
  // U = 8 elements per thread and step (M == 0): one workgroup per 2048 elements, at most 4 per
  // CU (16 waves; the whole C3 array in flight at once); [blocks * 4][q] lists for the merge
  const long long per_block = 256LL * (m == 0 ? 8 : 4);
  long long blocks = (n_cand + per_block - 1) / per_block;
  const int max_blocks = 4 * cus_count() < 1024 ? 4 * cus_count() : 1024;
  if (blocks > max_blocks) blocks = max_blocks;
  if (blocks < 1) blocks = 1;
  HviIn hz;
  memset(&hz, 0, sizeof(hz));
  const HviIn& hv = h ? *h : hz;
  int st;
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

int bo_pareto_mask(const double* y, int64_t n, int32_t n_obj, uint8_t* mask, void* stream) {
  if (!y || !mask || n < 0 || n_obj < 1 || n_obj > BO_MAX_OBJ) return BO_ERR_ARG;
  if (n == 0) return BO_OK;
  hipLaunchKernelGGL(pareto_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, y, (long long)n, n_obj, mask);
  BO_CHECK_HIP(hipGetLastError());
  return BO_OK;
}

}  // extern "C"
