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
  // point's row): built per workgroup in LDS (lds_slots > 0, select_lane_kernel), else in the
  // workspace (hkeys), else NULL (the exclusion scans the points)
  int lds_slots;
  const unsigned long long* hkeys;
  const int* hidx;
  unsigned int hmask;
  TopEntry* partial;
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
  for (int k = 0; k < a.dim; ++k) c[k] = cand_coord(a, j, k);
  if (hk) return bo_hash_contains(hk, hi, hm, a.excl, a.dim, c, a.dim);
  for (int e = 0; e < a.n_excl; ++e) {
    bool eq = true;
    for (int k = 0; k < a.dim; ++k) eq = eq && (a.excl[(long long)e * a.dim + k] == c[k]);
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

// grid-stride over candidates; each wave folds 64 candidates per step into its running
// top-q (4 inserts of 16), then writes its list to `partial`.
__global__ __launch_bounds__(256) void select_kernel(SelArgs a) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  double lv = -__builtin_inf();
  long long li = -1;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long base = (long long)blockIdx.x * blockDim.x + wave * 64; base < a.n_cand;
       base += stride) {
    const long long j = base + lane;
    double v = -__builtin_inf();
    long long gi = -1;
    if (j < a.n_cand) {
      v = a.acq[j];
      gi = a.cand_offset + j;
    }
    // the O(n_excl) exclusion test only for candidates that beat the wave's current q-th entry
    // (the others cannot enter the list whether excluded or not); after the first steps of the
    // grid-stride almost no wave-step needs it
    const double tv = __shfl(lv, a.topq - 1, 64);
    const long long ti = __shfl(li, a.topq - 1, 64);
    const bool need = a.n_excl > 0 && gi >= 0 && bo_better(v, gi, tv, ti);
    if (__ballot(need) != 0ull && need) {
      if (cand_excluded(a, j, a.hkeys, a.hidx, a.hmask)) gi = -1;
    }
#pragma unroll
    for (int grp = 0; grp < 4; ++grp) {
      const double nv = __shfl(v, (lane & 15) + 16 * grp, 64);
      const long long ni = __shfl(gi, (lane & 15) + 16 * grp, 64);
      bo_wave_topq_insert(lv, li, nv, ni, a.topq);
    }
  }
  if (lane < a.topq) {
    TopEntry* dst = a.partial + ((size_t)blockIdx.x * 4 + wave) * a.topq;
    dst[lane].v = lv;
    dst[lane].i = li;
  }
}

// ---------------------------------------------------------------------------------------
// Selection for q <= 16 (every batch the reference's demos use), ONE pass at HBM rate:
// every thread keeps its own sorted top-Q (Q = 8 / 16 / 24, at least q + 4) in registers over
// a coalesced grid-stride sweep -- almost every element is rejected by one comparison with the
// thread's Q-th entry.  The exclusion of evaluated points is deferred to the Q list entries of
// each thread (hash set of the points, built in LDS by every workgroup), so the sweep reads
// nothing but the acquisition values.  Then the wave (wave_lists_topq: threshold set + ranks)
// and the workgroup (ranks of the 4 wave lists) reduce the lists to the workgroup's top-q, and
// bo_topq_merge_kernel merges those.
// M > 0 fuses the exact hypervolume improvement of bo_hvi.hip into the sweep: the acquisition
// of candidate i is computed from its M UCB values and the boxes (wave-uniform, scalar loads),
// written to acq, and selected in the same pass (one HBM read of the UCB arrays in total).
// ---------------------------------------------------------------------------------------
struct HviIn {
  const double* ucb;          // [M][ld]
  long long ld;
  const double* boxes;        // [n_boxes][2 M]
  long long n_boxes;
  double shift[BO_MAX_OBJ], scale[BO_MAX_OBJ];
  double* acq_out;
};

template <int Q>
__device__ __forceinline__ void lane_insert(double (&v)[Q], long long (&ix)[Q], double nv, long long ni) {
  // sorted best-first; nv beats v[Q - 1] (checked by the caller)
#pragma unroll
  for (int k = Q - 1; k >= 0; --k) {
    const bool beats_k = bo_better(nv, ni, v[k], ix[k]);
    const bool beats_prev = k > 0 && bo_better(nv, ni, v[k > 0 ? k - 1 : 0], ix[k > 0 ? k - 1 : 0]);
    if (beats_k) {
      v[k] = beats_prev ? v[k - (k > 0)] : nv;
      ix[k] = beats_prev ? ix[k - (k > 0)] : ni;
    }
  }
}

// The top-q (q <= Q) of a wave's per-lane sorted lists, into out[0..q-1] (LDS):
//   T = the best of the lanes' q-th entries; S = the entries not worse than T -- a prefix of
//   every lane's list, normally about q .. 2q entries -- compacted into buf (64 entries, LDS)
//   by one ballot per list slot, each ranked by a scan of S.  |S| > 64 (fewer than q valid
//   entries per lane, or mass ties): q rounds of a wave arg-best, the owner popping its head.
// (Round 1 ran Q arg-best rounds at the wave and again at the workgroup level: 6 shuffle
// stages of (value, index) pairs per round.)  Called by all waves of the workgroup together.
constexpr int BO_SEL_Q = 16;
// `excluded(idx)` tests a list entry (global index) against the evaluated points; `purge()`
// drops every excluded entry of the calling lane's list (and rebuilds the list if too few
// remain).  The exclusion is only tested on S: when no entry of S is excluded, S also holds the
// top-q of the non-excluded elements; otherwise (rare) every lane purges and T, S are redone.
template <int Q, class Excl, class Purge>
__device__ __forceinline__ void wave_lists_topq(double (&v)[Q], long long (&ix)[Q], int q,
                                                TopEntry* buf, TopEntry* out, bool check,
                                                Excl excluded, Purge purge) {
  const int lane = threadIdx.x & 63;
  double bv;
  long long bi;
  int c;
  for (;;) {
    bv = -__builtin_inf();
    bi = -1;
#pragma unroll
    for (int k = 0; k < Q; ++k)
      if (k == q - 1) { bv = v[k]; bi = ix[k]; }
#pragma unroll
    for (int m = 32; m > 0; m >>= 1) {
      const double ov = __shfl_xor(bv, m, 64);
      const long long oi = __shfl_xor(bi, m, 64);
      if (bo_better(ov, oi, bv, bi)) { bv = ov; bi = oi; }
    }
    c = 0;                                            // length of this lane's prefix in S
#pragma unroll
    for (int k = 0; k < Q; ++k)
      if (k < q && ix[k] >= 0 && !bo_better(bv, bi, v[k], ix[k])) c = k + 1;
    if (!check) break;
    bool bad = false;
#pragma unroll
    for (int k = 0; k < Q; ++k)
      if (k < c) bad = bad || excluded(ix[k]);
    if (__ballot(bad) == 0ull) break;
    purge();
    check = false;
  }
  int total = 0;
  const unsigned long long lt = (1ull << lane) - 1ull;
#pragma unroll
  for (int k = 0; k < Q; ++k) {
    if (k >= q) break;
    const unsigned long long b = __ballot(c > k);
    const int off = total + __popcll(b & lt);
    if (c > k && off < 64) { buf[off].v = v[k]; buf[off].i = ix[k]; }
    total += __popcll(b);
  }
  __syncthreads();
  if (total <= 64) {
    if (lane < total) {
      const TopEntry me = buf[lane];
      int rank = 0;
      for (int m = 0; m < total; ++m) rank += bo_better(buf[m].v, buf[m].i, me.v, me.i) ? 1 : 0;
      if (rank < q) out[rank] = me;
    } else if (lane < q) {
      out[lane].v = -__builtin_inf();
      out[lane].i = -1;
    }
    return;
  }
#pragma unroll 1
  for (int r = 0; r < q; ++r) {
    double hv = v[0];
    long long hi = ix[0];
#pragma unroll
    for (int m = 32; m > 0; m >>= 1) {
      const double ov = __shfl_xor(hv, m, 64);
      const long long oi = __shfl_xor(hi, m, 64);
      if (bo_better(ov, oi, hv, hi)) { hv = ov; hi = oi; }
    }
    if (lane == 0) { out[r].v = hv; out[r].i = hi; }
    if (hi >= 0 && ix[0] == hi) {
#pragma unroll
      for (int k = 0; k + 1 < Q; ++k) { v[k] = v[k + 1]; ix[k] = ix[k + 1]; }
      v[Q - 1] = -__builtin_inf();
      ix[Q - 1] = -1;
    }
  }
}

template <int Q, int M>
__global__ __launch_bounds__(256) void select_lane_kernel(SelArgs a, HviIn h) {
  extern __shared__ __attribute__((aligned(16))) unsigned long long lkeys[];   // [lds_slots], then idx
  __shared__ TopEntry wl[4 * BO_SEL_Q];
  __shared__ TopEntry wbuf[4 * 64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // the evaluated points' hash set, in LDS when small (built by every workgroup: no extra
  // launches), else the workspace table, else none (scan)
  const unsigned long long* hk = a.hkeys;
  const int* hi = a.hidx;
  unsigned int hm = a.hmask;
  if (a.lds_slots > 0) {
    int* lidx = (int*)(lkeys + a.lds_slots);
    for (int t = tid; t < a.lds_slots; t += blockDim.x) lkeys[t] = 0ull;
    __syncthreads();
    for (int e = tid; e < a.n_excl; e += blockDim.x) {
      const unsigned long long key = bo_point_key(a.excl + (long long)e * a.dim, a.dim);
      if (key != 0ull) bo_hash_insert(lkeys, lidx, (unsigned int)a.lds_slots - 1, key, e);
    }
    __syncthreads();
    hk = lkeys;
    hi = lidx;
    hm = (unsigned int)a.lds_slots - 1;
  }
  double v[Q];
  long long ix[Q];
  const long long stride = (long long)gridDim.x * blockDim.x;
  // U elements per thread and sweep step, all loaded before any is processed (the loads of a
  // step are in flight together; the loop body alone would expose one latency per element).
  // The sweep itself ignores the exclusion (check = false): see below.
  constexpr int U = 4;
  auto sweep = [&](bool check) {
#pragma unroll
    for (int k = 0; k < Q; ++k) { v[k] = -__builtin_inf(); ix[k] = -1; }
    for (long long j0 = (long long)blockIdx.x * blockDim.x + tid; j0 < a.n_cand; j0 += U * stride) {
      double val[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const long long j = j0 + u * stride;
        const bool in = j < a.n_cand;
        if constexpr (M == 0) {
          val[u] = in ? a.acq[j] : 0.0;
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
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const long long j = j0 + u * stride;
        if (j >= a.n_cand) break;
        const long long gi = a.cand_offset + j;
        if (!bo_better(val[u], gi, v[Q - 1], ix[Q - 1])) continue;
        if (check && cand_excluded(a, j, hk, hi, hm)) continue;
        lane_insert<Q>(v, ix, val[u], gi);
      }
    }
  };
  sweep(false);
  // Deferred exclusion (acquisition.py:137-139): tested on the wave's threshold set S only
  // (wave_lists_topq); purge() runs when an entry of S is an evaluated point.  Without its
  // excluded entries a list still holds its thread's best non-excluded elements; it needs q of
  // them unless it held every element of the thread (Q - q >= 4), else the thread rescans with
  // per-element tests.
  auto excluded = [&](long long gi) { return gi >= 0 && cand_excluded(a, gi - a.cand_offset, hk, hi, hm); };
  auto purge = [&]() {
    const bool full = ix[Q - 1] >= 0;
    bool ex[Q];
    int removed = 0;
#pragma unroll
    for (int k = 0; k < Q; ++k) {
      ex[k] = excluded(ix[k]);
      removed += ex[k] ? 1 : 0;
    }
    if (removed == 0) return;
    if (full && Q - removed < a.topq) {
      sweep(true);
      return;
    }
#pragma unroll
    for (int k = Q - 1; k >= 0; --k) {
      if (ex[k]) {
#pragma unroll
        for (int t = k; t + 1 < Q; ++t) { v[t] = v[t + 1]; ix[t] = ix[t + 1]; }
        v[Q - 1] = -__builtin_inf();
        ix[Q - 1] = -1;
      }
    }
  };
  // wave, then workgroup: the top-q of the lanes' lists (wave_lists_topq), then of the 4 wave
  // lists (rank by LDS scan); the workgroup's list goes to `partial` ([blocks][q])
  wave_lists_topq<Q>(v, ix, a.topq, wbuf + wave * 64, wl + wave * BO_SEL_Q, a.n_excl > 0,
                     excluded, purge);
  __syncthreads();
  if (wave == 0) {
    const int n = 4 * a.topq;
    TopEntry* dst = a.partial + (size_t)blockIdx.x * a.topq;
    if (lane < a.topq) { dst[lane].v = -__builtin_inf(); dst[lane].i = -1; }
    if (lane < n) {
      const TopEntry me = wl[(lane / a.topq) * BO_SEL_Q + lane % a.topq];
      if (me.i >= 0) {
        int rank = 0;
        for (int m = 0; m < n; ++m) {
          const TopEntry o = wl[(m / a.topq) * BO_SEL_Q + m % a.topq];
          rank += bo_better(o.v, o.i, me.v, me.i) ? 1 : 0;
        }
        if (rank < a.topq) dst[rank] = me;
      }
    }
  }
}

template <int M>
int launch_select_lane(const SelArgs& a, const HviIn& h, int q, int blocks, hipStream_t s) {
  const size_t lds = (size_t)a.lds_slots * 12;
  if (q <= 4) hipLaunchKernelGGL((select_lane_kernel<8, M>), dim3(blocks), dim3(256), lds, s, a, h);
  else if (q <= 12) hipLaunchKernelGGL((select_lane_kernel<16, M>), dim3(blocks), dim3(256), lds, s, a, h);
  else hipLaunchKernelGGL((select_lane_kernel<24, M>), dim3(blocks), dim3(256), lds, s, a, h);
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

// partial lists: bitonic path <= 1024 workgroups x 4 waves x q; lane path <= 8192 entries
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
  if (n_excl > 0 && n_cand > 0) {
    // the evaluated points' hash set: per workgroup in LDS (<= 1024 points, one-pass kernel),
    // else in the workspace region after the lists when it fits (2 n_excl .. 4 n_excl slots of
    // 12 B), else none (the exclusion scans the points)
    const unsigned int slots = bo_hash_slots(n_excl);
    const size_t region = ((size_t)n_cand + 31) / 32 * 4;
    if (topq <= 16 && n_excl <= 1024) {
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
  long long blocks = (n_cand + 255) / 256;
  if (topq <= 16) {
    // two workgroups per CU (8 per CU measured slower: the per-workgroup list merges and the
    // longer final merge outweigh the extra loads in flight); blocks x Q <= 8192 list entries
    const int max_blocks = 2 * cus_count() < 512 ? 2 * cus_count() : 512;
    if (blocks > max_blocks) blocks = max_blocks;
    if (blocks < 1) blocks = 1;
    HviIn hz;
    memset(&hz, 0, sizeof(hz));
    const HviIn& hv = h ? *h : hz;
    int st;
    switch (m) {
      case 0: st = launch_select_lane<0>(a, hv, topq, (int)blocks, s); break;
      case 1: st = launch_select_lane<1>(a, hv, topq, (int)blocks, s); break;
      case 2: st = launch_select_lane<2>(a, hv, topq, (int)blocks, s); break;
      case 3: st = launch_select_lane<3>(a, hv, topq, (int)blocks, s); break;
      case 4: st = launch_select_lane<4>(a, hv, topq, (int)blocks, s); break;
      default: return BO_ERR_UNSUPPORTED;
    }
    if (st != BO_OK) return st;
    hipLaunchKernelGGL(bo_topq_merge_kernel, dim3(1), dim3(1024), 0, s, (const TopEntry*)ws,
                       blocks, topq, top_val, (long long*)top_idx);
    BO_CHECK_HIP(hipGetLastError());
    return BO_OK;
  }
  if (m != 0) return BO_ERR_UNSUPPORTED;   // (the caller runs the HVI scan first for q > 16)
  // q > 16: per-wave bitonic lists, one workgroup per CU
  const int max_blocks = cus_count() < 1024 ? cus_count() : 1024;
  if (blocks > max_blocks) blocks = max_blocks;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(select_kernel, dim3((unsigned)blocks), dim3(256), 0, s, a);
  BO_CHECK_HIP(hipGetLastError());
  hipLaunchKernelGGL(bo_topq_merge_kernel, dim3(1), dim3(1024), 0, s, (const TopEntry*)ws,
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
  if (topq > 16) {   // large batches: the standalone HVI scan, then the bitonic selection
    const int st = bo_hypervolume_improvement_exact(acq, ucb, ld, n_cand, n_obj, shift, scale, boxes,
                                                    n_boxes, stream);
    if (st != BO_OK) return st;
    return select_impl(acq, n_cand, kind, cand, grid_lo, grid_shape, dim, cand_offset, excl, n_excl,
                       topq, top_val, top_idx, ws, ws_bytes, s, nullptr, 0);
  }
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
