// Shared device helpers for the bo_amd kernels (gfx950 / CDNA4 only).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include "../../include/bo_amd.h"

typedef double d2 __attribute__((ext_vector_type(2)));
typedef double d4 __attribute__((ext_vector_type(4)));

#define BO_CHECK_HIP(expr)                         \
  do {                                             \
    hipError_t _e = (expr);                        \
    if (_e != hipSuccess) return BO_ERR_HIP;       \
  } while (0)

// Bounds checks of the diagnostic build (BO_BUILD_VARIANT=DEF_DEBUG_BOUNDS -> -DBO_DEBUG_BOUNDS):
// every checked index is printed when out of range and the access is skipped, so that a bad
// index names itself instead of faulting the device.  The release build compiles them away.
#ifdef BO_DEBUG_BOUNDS
#include <stdio.h>
__device__ __forceinline__ bool bo_bound(bool ok, const char* what, long long v, long long cap, int line) {
  if (!ok)
    printf("BO_DEBUG_BOUNDS line %d: %s = %lld outside [0, %lld) (block %d, thread %d)\n", line, what, v, cap,
           (int)blockIdx.x, (int)threadIdx.x);
  return ok;
}
#define BO_IN(v, cap, what) bo_bound((long long)(v) >= 0 && (long long)(v) < (long long)(cap), what, \
                                     (long long)(v), (long long)(cap), __LINE__)
#else
#define BO_IN(v, cap, what) true
#endif

// MIN_VARIANCE / KERNEL_JITTER / CHOLESKY_JITTER: bayesopt/config.py:57-66 (fp64 branch).
// Wait states between an MFMA writing its accumulators and their first VALU / v_accvgpr_read,
// supplied INSIDE the fences' asm statements (hipcc pads after an asm statement only by its own
// estimate, which under-counted gfx950's f64 MFMA in round 1).  One wait state is
// one s_nop issue slot, 4 clocks (MI355X guide: `s_nop 0` costs 4 cycles).  gfx950 runs
// v_mfma_f64_16x16x4_f64 in 16 passes (64 clocks, measured): the dependent read needs passes + 4
// = 20 states, given 24 here; v_mfma_f32_16x16x4_f32 is 8 passes (12 states), given 16.  Rounds
// 1-5 used 64 states (256 clocks), the MFMA's latency counted in clocks: that padding cost 2.6 %
// of the C3 kernel (32 fences per 64-candidate tile; profiles/r06_c3_ablation.jsonl).
#define BO_NOPS_F64_MFMA "s_nop 7\n\ts_nop 7\n\ts_nop 7"
#define BO_NOPS_F32_MFMA "s_nop 7\n\ts_nop 7"

#define BO_MIN_VARIANCE 1e-10
#define BO_MIN_VARIANCE_F32 1e-6    // the float32 branch's floor (config.py:57-61), BO_PREDICT_F32_FLOOR
#define BO_KERNEL_JITTER 1e-6
#define BO_CHOLESKY_JITTER 1e-8

// ---------------------------------------------------------------------------------------
// Selection order of select_next_batch (bayesopt/acquisition.py:134): the reference walks
// np.argsort(acq)[::-1], so NaN comes first, then descending value.  Ties (unspecified
// order in the reference) break by ascending global index.  Excluded / empty entries have
// rank 0 and are never selected.
// ---------------------------------------------------------------------------------------
struct TopEntry {
  double v;
  long long i;  // global candidate index, -1 = empty/excluded
};

// Branch-free order key: empty 0 < valid values (monotone in the value; -0.0 == 0.0) < NaN.
__device__ __forceinline__ unsigned long long bo_order_key(double v, long long i) {
  const unsigned long long b = (unsigned long long)__double_as_longlong(v + 0.0);   // -0.0 -> +0.0
  const unsigned long long m = (b >> 63) ? ~b : (b | 0x8000000000000000ull);
  return i < 0 ? 0ull : (v != v ? ~0ull : m);
}

// strict "a comes before b" in the selection order (selects only: the branchy three-way form
// cost every comparison site a chain of exec-mask branches)
__device__ __forceinline__ bool bo_better(double av, long long ai, double bv, long long bi) {
  const unsigned long long ka = bo_order_key(av, ai), kb = bo_order_key(bv, bi);
  return ka > kb || (ka == kb && ka != 0ull && ai < bi);
}

// "a comes before b" on precomputed order keys (bo_order_key) and indices
__device__ __forceinline__ bool bo_key_before(unsigned long long ka, long long ia, unsigned long long kb,
                                              long long ib) {
  return ka > kb || (ka == kb && ka != 0ull && ia < ib);
}

// the value of an order key (empty -> -inf; NaN -> the canonical NaN; -0.0 comes back as +0.0)
__device__ __forceinline__ double bo_key_value(unsigned long long k) {
  const unsigned long long b = (k >> 63) ? (k & 0x7FFFFFFFFFFFFFFFull) : ~k;
  return k == 0ull ? -__builtin_inf() : (k == ~0ull ? __builtin_nan("") : __longlong_as_double((long long)b));
}

// Sort the 64 (v, i) pairs held one per lane into selection order (lane 0 best): bitonic
// network over __shfl_xor (64-wide wavefront) on the order keys -- one key per element instead
// of the three-way comparison per stage and direction (4x fewer instructions per stage).
__device__ __forceinline__ void bo_wave_sort64(double& v, long long& i) {
  const int lane = threadIdx.x & 63;
  unsigned long long k = bo_order_key(v, i);
  long long x = i;
#pragma unroll
  for (int k2 = 2; k2 <= 64; k2 <<= 1) {
#pragma unroll
    for (int j = k2 >> 1; j > 0; j >>= 1) {
      const unsigned long long pk = __shfl_xor(k, j, 64);
      const long long px = __shfl_xor(x, j, 64);
      const bool lower = (lane & j) == 0;
      const bool desc = (lane & k2) == 0;
      const bool take = (lower == desc) ? bo_key_before(pk, px, k, x) : bo_key_before(k, x, pk, px);
      k = take ? pk : k;
      x = take ? px : x;
    }
  }
  v = bo_key_value(k);
  i = x;
}

// Merge up to 16 new entries (held by lanes 0..15 as nv/ni) into the wave's running
// top-q list (lanes 0..q-1 hold it sorted; lanes >= q are empty).  q <= 48.
__device__ __forceinline__ void bo_wave_topq_insert(double& lv, long long& li, double nv,
                                                    long long ni, int q) {
  const int lane = threadIdx.x & 63;
  // threshold: does any new entry beat the current q-th entry?
  const double tv = __shfl(lv, q - 1, 64);
  const long long ti = __shfl(li, q - 1, 64);
  const bool cand = lane < 16 && bo_better(nv, ni, tv, ti);
  if (__ballot(cand) == 0ull) return;
  const double sv = __shfl(nv, lane - 48, 64);
  const long long si = __shfl(ni, lane - 48, 64);
  if (lane >= 48) { lv = sv; li = si; }
  bo_wave_sort64(lv, li);
  if (lane >= q) { lv = -__builtin_inf(); li = -1; }
}

__device__ __forceinline__ double bo_readlane_d(double v, int l) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)b, l);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
__device__ __forceinline__ unsigned long long bo_readlane_u(unsigned long long v, int l) {
  const int lo = __builtin_amdgcn_readlane((int)v, l);
  const int hi = __builtin_amdgcn_readlane((int)(v >> 32), l);
  return ((unsigned long long)(unsigned int)hi << 32) | (unsigned int)lo;
}
__device__ __forceinline__ long long bo_readlane_i(long long v, int l) {
  const int lo = __builtin_amdgcn_readlane((int)v, l);
  const int hi = __builtin_amdgcn_readlane((int)(v >> 32), l);
  return ((long long)hi << 32) | (unsigned int)lo;
}

// The wave's running list: its q-th entry (the admission threshold), wave-uniform.
__device__ __forceinline__ void bo_wave_topq_threshold(double lv, long long li, int q,
                                                       double& tv, long long& ti) {
  tv = bo_readlane_d(lv, q - 1);
  ti = bo_readlane_i(li, q - 1);
}

// Merge the 16 candidates of a fused-kernel tile into the wave's running top-q list, q <= 16.
// The list is in lanes 0..q-1 (sorted; lanes >= q empty); the candidates are (nv, ni) of lane
// group 1 (lanes 16..31; every lane group holds the same 16).  Only the candidates beating the
// list's q-th entry (N') take part: each element of list + N' counts the elements before it in
// selection order (its final rank: list entries know their own position; the N' entries and the
// list entries are broadcast by v_readlane, |N'| + q rounds), and the ranks < q are scattered
// to their lanes by ds_permute.  Round 1 re-sorted all 64 lanes with a bitonic network (21
// shuffle stages) whenever a candidate entered -- on spatially coherent acquisition surfaces
// (a wave walking up a grid row) nearly every tile, ~6 us per tile at C2.
// core: the new entries are (nv, ni) of the lanes 16..47 with `in_new`
__device__ __forceinline__ void bo_wave_topq_insert_lanes(double& lv, long long& li, double nv,
                                                          long long ni, bool in_new, int q) {
  const int lane = threadIdx.x & 63;
  double tv;
  long long ti;
  bo_wave_topq_threshold(lv, li, q, tv, ti);
  const bool beat = in_new && bo_better(nv, ni, tv, ti);
  const unsigned long long nb = __ballot(beat);
  if (nb == 0ull) return;
  const bool isL = lane < q;
  const double mv = isL ? lv : nv;
  const long long mi = isL ? li : ni;
  // order keys computed once; the rounds broadcast keys and indices
  const unsigned long long kn = bo_order_key(nv, ni), kl = bo_order_key(lv, li), km = isL ? kl : kn;
  int rank = isL ? lane : 0;
  for (unsigned long long m = nb; m; m &= m - 1) {
    const int s = __builtin_ctzll(m);
    rank += bo_key_before(bo_readlane_u(kn, s), bo_readlane_i(ni, s), km, mi) ? 1 : 0;
  }
  for (int l = 0; l < q; ++l) {
    const bool b = bo_key_before(bo_readlane_u(kl, l), bo_readlane_i(li, l), km, mi);
    rank += (beat && b) ? 1 : 0;
  }
  const bool keep = (isL || beat) && rank < q;
  // targets: kept elements -> lane rank (< q <= 16); the others -> a lane >= 16 (the list
  // lanes' own slot + 48, or their own lane), never one of 0..q-1
  const int dst = keep ? rank : (lane < 16 ? lane + 48 : lane);
  const long long vb = __double_as_longlong(mv);
  const int v0 = __builtin_amdgcn_ds_permute(dst << 2, (int)vb);
  const int v1 = __builtin_amdgcn_ds_permute(dst << 2, (int)(vb >> 32));
  const int i0 = __builtin_amdgcn_ds_permute(dst << 2, (int)mi);
  const int i1 = __builtin_amdgcn_ds_permute(dst << 2, (int)(mi >> 32));
  if (lane < q) {
    lv = __longlong_as_double(((long long)v1 << 32) | (unsigned int)v0);
    li = ((long long)i1 << 32) | (unsigned int)i0;
  } else {
    lv = -__builtin_inf();
    li = -1;
  }
}

__device__ __forceinline__ void bo_wave_topq_insert16(double& lv, long long& li, double nv,
                                                      long long ni, int q) {
  bo_wave_topq_insert_lanes(lv, li, nv, ni, ((threadIdx.x & 63) >> 4) == 1, q);
}

// Two tiles' 16 candidates at once (lane group 1: (nv1, ni1), lane group 2: (nv2, ni2)): one
// threshold test, ballot and q broadcast rounds per two tiles.
__device__ __forceinline__ void bo_wave_topq_insert16x2(double& lv, long long& li, double nv1,
                                                        long long ni1, double nv2, long long ni2,
                                                        int q) {
  const int grp = (threadIdx.x & 63) >> 4;
  bo_wave_topq_insert_lanes(lv, li, grp == 2 ? nv2 : nv1, grp == 2 ? ni2 : ni1,
                            grp == 1 || grp == 2, q);
}

// Hash key of a point for the exclusion of evaluated points (acquisition.py:137-139, exact
// equality of every coordinate): -0.0 == 0.0, so the sign of zero is dropped; a point with a NaN
// coordinate equals nothing (key 0 = "no key", never stored).  Keys are odd (0 marks empty
// slots of the open-addressing tables).
__host__ __device__ inline unsigned long long bo_point_key(const double* c, int dim) {
  unsigned long long h = 0x9E3779B97F4A7C15ull;
  // constant trip count (fully unrolled): a caller's coordinate array stays in registers
#pragma unroll
  for (int k = 0; k < BO_MAX_DIM; ++k) {
    if (k >= dim) break;
    if (c[k] != c[k]) return 0ull;
    const double z = c[k] == 0.0 ? 0.0 : c[k];
    unsigned long long b;
    memcpy(&b, &z, 8);
    b ^= h + 0x9E3779B97F4A7C15ull + (h << 6) + (h >> 2);
    b ^= b >> 31; b *= 0x7FB5D329728EA185ull; b ^= b >> 27; b *= 0x81DADEF4BC2DD44Dull; b ^= b >> 33;
    h = b;
  }
  return h | 1ull;
}

// Insert point `e` (key != 0) into an open-addressing table of mask + 1 slots.
__device__ __forceinline__ void bo_hash_insert(unsigned long long* keys, int* idx, unsigned int mask,
                                               unsigned long long key, int e) {
  for (unsigned int t = (unsigned int)key & mask;; t = (t + 1) & mask)
    if (atomicCAS(keys + t, 0ull, key) == 0ull) { idx[t] = e; return; }
}

// Is point c (dim coordinates) one of the rows of pts ([*][ld]) stored in the table?
__device__ __forceinline__ bool bo_hash_contains(const unsigned long long* keys, const int* idx,
                                                 unsigned int mask, const double* pts, int ld,
                                                 const double* c, int dim, long long n_pts = 1ll << 40) {
  const unsigned long long key = bo_point_key(c, dim);
  if (key == 0ull) return false;
  for (unsigned int t = (unsigned int)key & mask;; t = (t + 1) & mask) {
    const unsigned long long kt = keys[t];
    if (kt == 0ull) return false;
    if (kt == key && BO_IN(idx[t], n_pts, "hash idx[t]")) {
      const double* r = pts + (long long)idx[t] * ld;
      bool eq = true;
#pragma unroll
      for (int k = 0; k < BO_MAX_DIM; ++k) eq = eq && (k >= dim || r[k] == c[k]);
      if (eq) return true;
    }
  }
}

// table slots for n points: a power of two >= 2 n (load <= 1/2), at least 64
inline unsigned int bo_hash_slots(long long n) {
  unsigned int s = 64;
  while (s < 2ull * (unsigned long long)(n > 0 ? n : 0)) s <<= 1;
  return s;
}

// Per-candidate outputs (mu, var, UCB, acq, ...): written once, read by the next launch or the
// host -- streaming stores, so that they do not evict the L2-resident W stream.
__device__ __forceinline__ void bo_out_store(double* p, double v) { __builtin_nontemporal_store(v, p); }

// Workgroup-wide best entry (selection order) of one entry per thread; every thread gets it.
// `red` is a __shared__ scratch of blockDim.x / 64 entries.
__device__ __forceinline__ TopEntry bo_block_best(double v, long long i, TopEntry* red) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
#pragma unroll
  for (int m = 32; m > 0; m >>= 1) {
    const double ov = __shfl_xor(v, m, 64);
    const long long oi = __shfl_xor(i, m, 64);
    if (bo_better(ov, oi, v, i)) { v = ov; i = oi; }
  }
  if (lane == 0) { red[wave].v = v; red[wave].i = i; }
  __syncthreads();
  TopEntry b = red[0];
  for (int w = 1; w < nw; ++w)
    if (bo_better(red[w].v, red[w].i, b.v, b.i)) b = red[w];
  __syncthreads();
  return b;
}

// Final merge of n_lists sorted top-q lists ([n_lists][q], any q <= BO_MAX_TOPQ) into out_v /
// out_i in selection order; one workgroup of 256 threads (1024 measured slower: every wave sorts).
//   T: every thread takes the best head of its lists, every wave sorts its 64 maxima (bitonic)
//   and takes the q-th, T is the best of those -- q list heads (valid entries) are not worse
//   than T, so the global top-q lies in S = {entries not worse than T}.  Only lists whose head is
//   not worse than T contribute (normally about q of them); their entries not worse than T are
//   compacted into LDS and each one's rank in S (the number of S entries before it) is counted;
//   rank r < q goes to slot r.  Fallback when S exceeds the LDS (mass ties, or T empty because
//   fewer than q entries exist and S is large): q rounds of a workgroup arg-best over every entry.
// (The previous T -- the best of the lists' q-th entries -- left thousands of entries in S once
// the lists came from blocks of thousands of candidates: 19 us at q = 3, 150 us at q = 16 and
// 900 us at q = 48 for 512 lists, nearly all in the fallback.)
#define BO_MERGE_CAP 1024
static __global__ __launch_bounds__(256) void bo_topq_merge_kernel(const TopEntry* __restrict__ L,
                                                                    long long n_lists, int q,
                                                                    double* __restrict__ out_v,
                                                                    long long* __restrict__ out_i) {
  __shared__ TopEntry s_red[16];
  __shared__ TopEntry s_buf[BO_MERGE_CAP];
  __shared__ int s_lists[BO_MERGE_CAP], s_lists2[BO_MERGE_CAP];
  __shared__ int s_cnt, s_nl, s_nl2;
  const int tid = threadIdx.x, nt = blockDim.x, lane = tid & 63, wave = tid >> 6;
  if (tid == 0) { s_cnt = 0; s_nl = 0; }
  // the heads of lists tid + u nt, u < 16, stay in registers for the second pass (all of them
  // up to 16 x 256 = 4096 lists); more lists are re-read
  constexpr int HC = 16;
  TopEntry hd[HC];
  double bv = -__builtin_inf();
  long long bi = -1;
#pragma unroll
  for (int u = 0; u < HC; ++u) {
    const long long l = tid + (long long)u * nt;
    hd[u] = l < n_lists ? L[l * q] : TopEntry{-__builtin_inf(), -1};
  }
#pragma unroll
  for (int u = 0; u < HC; ++u)
    if (bo_better(hd[u].v, hd[u].i, bv, bi)) { bv = hd[u].v; bi = hd[u].i; }
  for (long long l = tid + (long long)HC * nt; l < n_lists; l += nt) {
    const TopEntry e = L[l * q];
    if (bo_better(e.v, e.i, bv, bi)) { bv = e.v; bi = e.i; }
  }
  bo_wave_sort64(bv, bi);
  {
    const double wv = bo_readlane_d(bv, q - 1);
    const long long wi = bo_readlane_i(bi, q - 1);
    if (lane == 0) { s_red[wave].v = wv; s_red[wave].i = wi; }
  }
  __syncthreads();
  TopEntry T = s_red[0];
  for (int w = 1; w < (nt >> 6); ++w)
    if (bo_better(s_red[w].v, s_red[w].i, T.v, T.i)) T = s_red[w];
#pragma unroll
  for (int u = 0; u < HC; ++u) {
    const long long l = tid + (long long)u * nt;
    if (l < n_lists && hd[u].i >= 0 && !bo_better(T.v, T.i, hd[u].v, hd[u].i)) {
      const int p = atomicAdd(&s_nl, 1);
      if (p < BO_MERGE_CAP) s_lists[p] = (int)l;
    }
  }
  for (long long l = tid + (long long)HC * nt; l < n_lists; l += nt) {
    const TopEntry e = L[l * q];
    if (e.i >= 0 && !bo_better(T.v, T.i, e.v, e.i)) {
      const int p = atomicAdd(&s_nl, 1);
      if (p < BO_MERGE_CAP) s_lists[p] = (int)l;
    }
  }
  __syncthreads();
  int nl = s_nl;
  const int* lists = s_lists;
  if (nl <= BO_MERGE_CAP && nl > 2 * q && nl * q > 2048) {
    // T is loose (large q, many lists: the entry scan below would read more than 2048 entries
    // and usually overflow S): tighten it to the q-th best head of the qualifying lists (bitonic
    // sort of their heads in LDS) and keep only the lists whose head is not worse.  q = 48 over
    // 4096 lists: 124 -> 76 us per selection
    int P = 1;
    while (P < nl) P <<= 1;
    for (int k = tid; k < P; k += nt)
      if (BO_IN(k, BO_MERGE_CAP, "merge s_buf[k] (heads)"))
        s_buf[k] = k < nl ? L[(long long)s_lists[k] * q] : TopEntry{-__builtin_inf(), -1};
    __syncthreads();
    for (int k2 = 2; k2 <= P; k2 <<= 1)
      for (int j = k2 >> 1; j > 0; j >>= 1) {
        for (int k = tid; k < P; k += nt) {
          const int pk = k ^ j;
          if (pk > k) {
            const TopEntry x = s_buf[k], y = s_buf[pk];
            const bool best_first = (k & k2) == 0;
            if (best_first ? bo_better(y.v, y.i, x.v, x.i) : bo_better(x.v, x.i, y.v, y.i)) {
              s_buf[k] = y;
              s_buf[pk] = x;
            }
          }
        }
        __syncthreads();
      }
    const TopEntry T2 = s_buf[q - 1];
    if (T2.i >= 0) T = T2;
    if (tid == 0) s_nl2 = 0;
    __syncthreads();
    for (int k = tid; k < nl; k += nt) {
      const int l = s_lists[k];
      const TopEntry h = L[(long long)l * q];
      if (h.i >= 0 && !bo_better(T.v, T.i, h.v, h.i)) {
        const int p2 = atomicAdd(&s_nl2, 1);
        if (BO_IN(p2, BO_MERGE_CAP, "merge s_lists2")) s_lists2[p2] = l;
      }
    }
    __syncthreads();
    nl = s_nl2;
    lists = s_lists2;
  }
  if (nl <= BO_MERGE_CAP) {
    for (int k = tid; k < nl * q; k += nt) {
      if (!BO_IN(lists[k / q], n_lists, "merge lists[k / q]")) continue;
      const TopEntry e = L[(long long)lists[k / q] * q + k % q];
      if (e.i >= 0 && !bo_better(T.v, T.i, e.v, e.i)) {
        const int p = atomicAdd(&s_cnt, 1);
        if (p < BO_MERGE_CAP) s_buf[p] = e;
      }
    }
    __syncthreads();
    const int cnt = s_cnt;
    if (cnt <= BO_MERGE_CAP) {
      for (int k = tid; k < cnt; k += nt) {
        const TopEntry me = s_buf[k];
        int rank = 0;
        for (int m = 0; m < cnt; ++m) rank += bo_better(s_buf[m].v, s_buf[m].i, me.v, me.i) ? 1 : 0;
        if (rank < q && BO_IN(rank, q, "merge rank")) { out_v[rank] = me.v; out_i[rank] = me.i; }
      }
      for (int t = cnt + tid; t < q; t += nt) { out_v[t] = -__builtin_inf(); out_i[t] = -1; }
      return;
    }
  }
  const long long total = n_lists * q;
  double pv = 0.0;
  long long pi = -1;                                 // previous winner (none yet)
  for (int r = 0; r < q; ++r) {
    double cv = -__builtin_inf();
    long long ci = -1;
    for (long long k = tid; k < total; k += nt) {
      const TopEntry e = L[k];
      if (e.i < 0 || bo_better(T.v, T.i, e.v, e.i)) continue;
      if (pi >= 0 && !bo_better(pv, pi, e.v, e.i)) continue;   // already selected
      if (bo_better(e.v, e.i, cv, ci)) { cv = e.v; ci = e.i; }
    }
    const TopEntry w = bo_block_best(cv, ci, s_red);
    if (tid == 0) { out_v[r] = w.i >= 0 ? w.v : -__builtin_inf(); out_i[r] = w.i; }
    pv = w.v;
    pi = w.i;
    if (w.i < 0) {
      for (int t = r + 1 + tid; t < q; t += nt) { out_v[t] = -__builtin_inf(); out_i[t] = -1; }
      break;
    }
  }
}

// invert_k's blocked LU path (bo_lu.hip), called by bo_invert_k (bo_fit.hip) once for all the
// objectives whose Cholesky failed (out[b] / km[b], b < n_lu)
size_t bo_lu_workspace_size(int64_t n, int n_lu);
int bo_lu_max_n();
int bo_lu_inverse(double* const* out, const double* const* km, int n_lu, int64_t ld, int64_t n, double jitter,
                  void* ws, size_t ws_bytes, hipStream_t s);

// the lean final merge of sorted top-q lists (bo_select.hip; q <= 4, n_lists <= 1024), used after
// the fused kernel; false when it does not apply
bool bo_launch_rounds_merge(const TopEntry* lists, long long n_lists, int q, double* out_v, int64_t* out_i,
                            hipStream_t s);

// ---------------------------------------------------------------------------------------
// Sobol candidates (BO_CAND_SOBOL): direction numbers (host) and one coordinate (device).
// ---------------------------------------------------------------------------------------
struct SobolArgs {
  unsigned int v[BO_MAX_DIM][32];   // direction numbers scaled to `bits`
  double lo[BO_MAX_DIM], scale[BO_MAX_DIM];
  int bits;
};

// Direction numbers of scipy.stats.qmc.Sobol (Joe & Kuo's table, first BO_MAX_DIM dimensions:
// primitive polynomials and initial m_j), built as Bratley & Fox's recurrence; bo_misc.hip.
int bo_sobol_fill(SobolArgs* s, int dim, const bo_sobol_desc* d);

// coordinate k of Sobol point i: lo + (x / 2^bits) * scale, x = XOR_{bits j of gray(i)} v[k][j]
__host__ __device__ inline double bo_sobol_coord(const SobolArgs& s, int k, unsigned long long i) {
  const unsigned long long g = i ^ (i >> 1);
  unsigned int x = 0;
  for (int b = 0; b < s.bits; ++b)
    if ((g >> b) & 1ull) x ^= s.v[k][b];
  const double u = ldexp((double)x, -s.bits);          // exact
#ifdef __HIP_DEVICE_COMPILE__
  return __dadd_rn(s.lo[k], __dmul_rn(u, s.scale[k]));  // numpy: lo + sample * scale, unfused
#else
  volatile double t = u * s.scale[k];
  return s.lo[k] + t;
#endif
}
