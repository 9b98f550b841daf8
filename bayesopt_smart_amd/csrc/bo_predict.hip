// Fused GP posterior + UCB / "hypervolume improvement" + top-q over a candidate shard: the
// preparation kernels, the top-q merges, the planner and the C ABI (bo_predict_acquire and the
// materialised-k_star drop-in bo_update_mean_variance).  The chunk-major kernels themselves are
// in bo_predict_impl.h, instantiated per padded dimension by bo_predict_d{2,4,6,8}.hip.
//
// Replaces the reference chain bayesopt/bayesian_optimization.py:145-207:
//   update_k_star (numba_kernels.py:406-442) -> update_mean (:450-488) ->
//   update_variance (:491-535) -> standardize_objectives (:538-570) ->
//   update_ucb / update_hypervolume_improvement (acquisition.py:55-108) ->
//   select_next_batch (acquisition.py:116-144, local top-q part).

#include "bo_predict_impl.h"

#include <vector>

namespace {

// ---------------------------------------------------------------------------------------
// Materialised-k_star path (bo_update_mean_variance, the unfused drop-in of update_mean +
// update_variance, numba_kernels.py:450-535): K* is read from HBM, Z = K^-1 K* runs on the f64
// matrix cores (dense form, the reference's DGEMM), q = sum_e K* Z and mu = pm + K*^T alpha.
// One wave owns 16 candidates; the K* block of a panel (NS k-steps of 4 rows) is held in
// registers as the B operand (lane l: row 4s + (l >> 4), candidate l & 15); K^-1 streams in
// fragment order through the W ring.  The D rows (l >> 4) + 4r of E-block E coincide with the
// B rows of k-steps 4E + r: the single-panel epilogue selects them from B; the multi-panel one
// (N > 512) reloads them.
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ double kstar_at(const FusedArgs& a, int o, int f, long long j, bool valid) {
  return (valid && f < a.n_train) ? a.kstar[((long long)o * a.ks_rows + f) * a.n_cand + j] : 0.0;
}

// one E-pair (E = 2ep, 2ep + 1: 32 training rows) of one panel: acc0/acc1 += W[E, panel] . B;
// the ring's 4 pairs are consumed strictly in order (pos counts 2-KiB pairs; past the end the
// buffer range check returns zeros).  SELECT: the epilogue rows of E-pair ep (chunk c == ep)
// picked from B by masked FMAs.
template <int NS, bool SELECT>
__device__ __forceinline__ void contract_epair(__amdgpu_buffer_rsrc_t wr, int voff, int base,
                                               int& pos, int ep, const double (&B)[NS],
                                               d2 (&wa)[kPF], d2 (&wb)[kPF], d4& acc0, d4& acc1,
                                               double (&sel0)[4], double (&sel1)[4]) {
  constexpr int NCH = NS / 8;
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
#pragma unroll
    for (int pp = 0; pp < 4; ++pp) {
      const int p = 4 * c + pp;
      const d2 ca = wa[pp];
      const d2 cb = wb[pp];
      const int so = base + ((pos + kPF) << 11);
      wa[pp] = wload(wr, voff, so);
      wb[pp] = wload(wr, voff, so + 1024);
      ++pos;
      acc0 = mfma64(ca.x, B[2 * p], acc0);
      acc1 = mfma64(cb.x, B[2 * p], acc1);
      acc0 = mfma64(ca.y, B[2 * p + 1], acc0);
      acc1 = mfma64(cb.y, B[2 * p + 1], acc1);
    }
    if (SELECT) {
      const double m = (c == ep) ? 1.0 : 0.0;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        sel0[r] = __builtin_fma(m, B[8 * c + r], sel0[r]);
        sel1[r] = __builtin_fma(m, B[8 * c + 4 + r], sel1[r]);
      }
    }
  }
}

template <int NS, bool MULTI>
__global__ __launch_bounds__(256, 1) void kmem_predict_kernel(const FusedArgs a) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  double* alpha = smem;                                // [n_obj][n_pad]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, jl = lane & 15;
  for (int t = tid; t < a.n_obj * a.n_pad; t += blockDim.x) alpha[t] = a.alpha[t];
  __syncthreads();
  const __amdgpu_buffer_rsrc_t wr =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.wpack, (short)0, (int)a.wpack_bytes, 0x00020000);
  const int voff = lane * 16;
  const int n_ep = a.n_pad / 32;                           // E-block pairs over all rows
  const int w_obj = a.n_pad * a.n_pad * 8;                 // bytes per objective
  const int w_panel = a.n_pad * (NS * 4) * 8;              // bytes per panel
  for (long long tile = blockIdx.x; tile < a.n_tiles; tile += gridDim.x) {
    const long long j = tile * kTile + wave * 16 + jl;
    const bool valid = j < a.n_cand;
    for (int o = 0; o < a.n_obj; ++o) {
      const double pv = a.pv[o];
      const double* al = alpha + o * a.n_pad;
      double qpart = 0.0, mpart = 0.0;
      for (int panel = 0; panel < (MULTI ? a.n_panels : 1); ++panel) {
        const int f0 = panel * NS * 4;
        double B[NS];                                      // B[s] = K*[f0 + 4s + g][j]
#pragma unroll
        for (int s = 0; s < NS; ++s) B[s] = kstar_at(a, o, f0 + 4 * s + g, j, valid);
        const int base = o * w_obj + panel * w_panel;
        d2 wa[kPF], wb[kPF];
        prime_ring(wr, voff, base, wa, wb);
        int pos = 0;
        // multi-panel epilogue rows: K*[e][j], e = 32 ep + 16 h + g + 4 r -> nxt[4 h + r]
        double nxt[8];
        if (MULTI) {
#pragma unroll
          for (int t = 0; t < 8; ++t) nxt[t] = kstar_at(a, o, 16 * (t >> 2) + g + 4 * (t & 3), j, valid);
        }
        for (int ep = 0; ep < n_ep; ++ep) {
          d4 acc0 = {0.0, 0.0, 0.0, 0.0}, acc1 = {0.0, 0.0, 0.0, 0.0};
          double sel0[4] = {0.0, 0.0, 0.0, 0.0}, sel1[4] = {0.0, 0.0, 0.0, 0.0};
          if (MULTI) {
#pragma unroll
            for (int r = 0; r < 4; ++r) { sel0[r] = nxt[r]; sel1[r] = nxt[4 + r]; }
#pragma unroll
            for (int t = 0; t < 8; ++t)
              nxt[t] = kstar_at(a, o, 32 * (ep + 1) + 16 * (t >> 2) + g + 4 * (t & 3), j, valid);
          }
          contract_epair<NS, !MULTI>(wr, voff, base, pos, ep, B, wa, wb, acc0, acc1, sel0, sel1);
          mfma_fence<true>(acc0, acc1);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            qpart = __builtin_fma(sel0[r], acc0[r], qpart);
            qpart = __builtin_fma(sel1[r], acc1[r], qpart);
          }
        }
#pragma unroll
        for (int s = 0; s < NS; ++s) mpart = __builtin_fma(al[f0 + 4 * s + g], B[s], mpart);
      }
      qpart += __shfl_xor(qpart, 16, 64);
      qpart += __shfl_xor(qpart, 32, 64);
      mpart += __shfl_xor(mpart, 16, 64);
      mpart += __shfl_xor(mpart, 32, 64);
      if (valid && g == 0) {
        const long long off = (long long)o * a.ld_out + j;
        if (a.mu) a.mu[off] = a.pm[o] + mpart;                      // :486-488
        if (a.var) a.var[off] = fmax(pv - qpart, a.min_var);  // :532-535
      }
    }
  }
  BO_WAIT_VMCNT(0);
}

// Pack W into the chunk-major MFMA stream of cm_predict_kernel: per objective, for each group of
// kCMaxEp E-pairs, for chunk c ascending (from the group's first E-pair when upper), for the
// group's E-pairs ep ascending (ep <= c when upper),
// for k-step pair pp = 0..3 (k-steps s = 8c + 2pp, +1): the A fragments of E = 2ep and
// E = 2ep + 1, 64 lanes x 16 B each: {W[16E + (l&15)][4s + (l>>4)], same at s+1}.
//   dense: W = K^-1 (leading dim ld);
//   upper: W[e][f] = (K^-1[e][f] + K^-1[f][e]) / 2 for f > e, K^-1[e][e] / 2 for f == e, else 0.
__host__ __device__ inline long long cm_group_blocks(int nch, int e0, int upper) {
  const int eN = nch - e0 < kCMaxEp ? nch - e0 : kCMaxEp;
  if (!upper) return (long long)nch * eN;
  // chunks e0 .. e0+eN-2 hold 1 .. eN-1 blocks, the nch - e0 - eN + 1 later ones eN each
  return (long long)(eN - 1) * eN / 2 + (long long)(nch - e0 - eN + 1) * eN;
}

__host__ __device__ inline long long cm_blocks(int nch, int upper) {
  long long blocks = 0;
  for (int e0 = 0; e0 < nch; e0 += kCMaxEp) blocks += cm_group_blocks(nch, e0, upper);
  return blocks;
}

// The objectives' streams are contiguous (objective o starts at pair 4 o blocks), so that the
// kernel's W ring runs on from one objective into the next without a restart.
__device__ void pack_cm_range(long long t0, long long stride, d2* __restrict__ out,
                              const double* __restrict__ kinv, long long ld, int upper, int n,
                              int n_pad, int n_obj) {
  const int nch = n_pad / 32;
  const long long per_obj = cm_blocks(nch, upper) * 512;      // d2 entries (4 pairs x 2 x 64)
  for (long long t = t0; t < per_obj * n_obj; t += stride) {
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
    out[t] = v;
  }
}


// Pack K^-1 into the MFMA fragment order of kmem_predict_kernel (the materialised-K* path),
// zero padded.  Element (panel, ep, pair, which, lane) holds W[16E + (l&15)][4s + (l>>4)] and
// the same at s+1 (E = 2ep + which, s = panel*ns_panel + 2*pair).
__device__ void pack_range(long long t0, long long stride, d2* __restrict__ out,
                           const double* __restrict__ kinv, long long ld, int n, int n_pad,
                           int ns_panel, int n_obj) {
  const long long per_obj = (long long)n_pad * n_pad / 2;
  const long long total = per_obj * n_obj;
  const int n_ep = n_pad / 32;
  const int npair = ns_panel / 2;
  for (long long t = t0; t < total; t += stride) {
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

__global__ void selftest_mfma_kernel(const double* a, const double* b, double* d) {
  const int l = threadIdx.x;
  const double av = a[(l & 15) * 4 + (l >> 4)];  // A[i=l&15][k=l>>4]
  const double bv = b[(l >> 4) * 16 + (l & 15)]; // B[k=l>>4][j=l&15]
  d4 acc = {0.0, 0.0, 0.0, 0.0};
  acc = mfma64(av, bv, acc);
#pragma unroll
  for (int r = 0; r < 4; ++r) d[((l >> 4) + 4 * r) * 16 + (l & 15)] = acc[r];
}


// float4 entry (o, block, kq, b, lane) = {W[row][col0 + t], t = 0..3}, row = 64 ep + 16 b +
// (lane & 15), col0 = 64 c + 16 kq + 4 (lane >> 4); W = triu(sym(K^-1)) with halved diagonal.
__device__ void pack32_range(long long t0, long long stride, f4* __restrict__ out,
                             const double* __restrict__ kinv, long long ld, int n, int n_pad,
                             int n_obj) {
  const int nch = n_pad / 64;
  const long long per_obj = c32_blocks(nch) * 1024;
  for (long long t = t0; t < per_obj * n_obj; t += stride) {
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


// ---------------------------------------------------------------------------------------
// Per-call preparation, ONE launch (blocks by role; the two single-block roles, serial chains of
// dependent memory round trips, come first so that they are dispatched before the bulk):
//   block 0                        training rows: xpad (original; padded rows 1e200 so their
//                                  K* is exactly 0) and xc = x - x_0 (centred); the
//                                  separable-grid precondition flag (every training point's last
//                                  coordinate an integer on the grid's last axis); the
//                                  evaluated points padded to [n_excl][DIM];
//   block 1                        the hash set of the exclusion rows (zeroed, then filled);
//   [2, 2 + alpha_blocks)          alpha[o][f] = sum_e K^-1[o][f][e] (y[e][o] - pm[o])
//                                  (numba_kernels.py:477-483), one wave per row, e ascending
//                                  per lane then a shuffle tree;
//   [.., + pack_blocks)            W packed into the kernel's MFMA stream (pack_cm_range /
//                                  pack_range / pack32_range).
// ---------------------------------------------------------------------------------------
struct PrepArgs {
  int pack_mode;                         // 0 chunk-major (cm), 1 panels (kmem), 2 f32 (cm32)
  void* wpack;
  const double* kinv;
  long long ld_k;
  int upper, n, n_pad, ns, n_obj;
  int pack_blocks, alpha_blocks;
  double* alpha;
  const double* y;
  long long ld_y;
  double pm[BO_MAX_OBJ];
  int rows;                              // training-row preparation (not on the kmem path)
  double *xpad, *xc;
  const double* x;
  int dim, DIM;
  int* sep_flag;                         // NULL: no separable grid check
  long long sep_lo;
  int sep_S;
  double* excl;
  const double* excl_in;
  int n_excl;
  // hash set of the exclusion rows (the evaluated points, or the training rows when none are
  // given): zeroed, then filled, by the rows block
  unsigned long long* hkeys;
  int* hidx;
  unsigned int hslots;
  int n_hash;                            // rows to insert (0: no table)
  int hash_lds;                          // 1: built in the launch's dynamic LDS, then stored
};

__global__ __launch_bounds__(256) void predict_prep_kernel(const PrepArgs p) {
  const int tid = threadIdx.x;
  int b = blockIdx.x;
  if (b == 0) {
    if (!p.rows) return;
    int sep_bad = 0;
    for (int f = tid; f < p.n_pad; f += 256) {
      for (int k = 0; k < p.DIM; ++k) {
        const bool real = f < p.n && k < p.dim;
        const double v = f < p.n ? (real ? p.x[(long long)f * p.dim + k] : 0.0) : 1e200;
        p.xpad[(long long)f * p.DIM + k] = v;
        p.xc[(long long)f * p.DIM + k] = f < p.n ? v - (k < p.dim ? p.x[k] : 0.0) : 1e200;
      }
      if (f < p.n && p.sep_flag) {
        const double v = p.x[(long long)f * p.dim + p.dim - 1];
        const bool ok = v == __builtin_rint(v) && v >= (double)p.sep_lo && v <= (double)(p.sep_lo + p.sep_S - 1);
        sep_bad |= !ok;
      }
    }
    const int any_bad = __syncthreads_or(sep_bad);
    if (tid == 0 && p.sep_flag) *p.sep_flag = any_bad ? 1 : 0;
    for (int t = tid; t < p.n_excl * p.DIM; t += 256) {
      const int r = t / p.DIM, k = t - r * p.DIM;
      p.excl[t] = k < p.dim ? p.excl_in[(long long)r * p.dim + k] : 0.0;
    }
    return;
  }
  if (b == 1) {
    if (p.n_hash <= 0) return;
    // keys over the DIM-padded coordinates (zeros past dim), read from the inputs; the first
    // 4 x 256 rows' keys are computed before the table is zeroed, so that their loads overlap it
    const double* src = p.excl_in ? p.excl_in : p.x;
    constexpr int KP = 4;
    unsigned long long kp[KP];
#pragma unroll
    for (int u = 0; u < KP; ++u) {
      const int e = tid + 256 * u;
      kp[u] = 0ull;
      if (e < p.n_hash) {
        double c[BO_MAX_DIM];
        for (int k = 0; k < p.DIM; ++k) c[k] = k < p.dim ? src[(long long)e * p.dim + k] : 0.0;
        kp[u] = bo_point_key(c, p.DIM);
      }
    }
    // small tables (hash_lds) are built in LDS -- LDS compare-and-swaps instead of a chain of
    // global atomic round trips -- and then stored with plain coalesced stores
    extern __shared__ unsigned long long hls[];
    unsigned long long* keys = p.hash_lds ? hls : p.hkeys;
    int* idx = p.hash_lds ? (int*)(hls + p.hslots) : p.hidx;
    for (unsigned int t = tid; t < p.hslots; t += 256) keys[t] = 0ull;
    __syncthreads();
#pragma unroll
    for (int u = 0; u < KP; ++u)
      if (kp[u] != 0ull) bo_hash_insert(keys, idx, p.hslots - 1, kp[u], tid + 256 * u);
    for (int e = tid + 256 * KP; e < p.n_hash; e += 256) {
      double c[BO_MAX_DIM];
      for (int k = 0; k < p.DIM; ++k) c[k] = k < p.dim ? src[(long long)e * p.dim + k] : 0.0;
      const unsigned long long key = bo_point_key(c, p.DIM);
      if (key != 0ull) bo_hash_insert(keys, idx, p.hslots - 1, key, e);
    }
    if (p.hash_lds) {
      __syncthreads();
      for (unsigned int t = tid; t < p.hslots; t += 256) {
        p.hkeys[t] = keys[t];
        p.hidx[t] = idx[t];
      }
    }
    return;
  }
  b -= 2;
  const int lane = tid & 63, wave = tid >> 6;
  if (b < p.alpha_blocks) {
    const long long row_id = (long long)b * 4 + wave;
    if (row_id >= (long long)p.n_obj * p.n_pad) return;
    const int o = (int)(row_id / p.n_pad), f = (int)(row_id % p.n_pad);
    double s = 0.0;
    if (f < p.n) {
      const double* wr = p.kinv + (long long)o * p.ld_k * p.ld_k + (long long)f * p.ld_k;
      const double pm = p.pm[o];
      for (int e = lane; e < p.n; e += 64) s = __builtin_fma(wr[e], p.y[(long long)e * p.ld_y + o] - pm, s);
    }
#pragma unroll
    for (int m = 32; m > 0; m >>= 1) s += __shfl_xor(s, m, 64);
    if (lane == 0) p.alpha[row_id] = s;
    return;
  }
  b -= p.alpha_blocks;
  const long long t0 = (long long)b * 256 + tid, stride = (long long)p.pack_blocks * 256;
  if (p.pack_mode == 0) pack_cm_range(t0, stride, (d2*)p.wpack, p.kinv, p.ld_k, p.upper, p.n, p.n_pad, p.n_obj);
  else if (p.pack_mode == 1) pack_range(t0, stride, (d2*)p.wpack, p.kinv, p.ld_k, p.n, p.n_pad, p.ns, p.n_obj);
  else pack32_range(t0, stride, (f4*)p.wpack, p.kinv, p.ld_k, p.n, p.n_pad, p.n_obj);
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
constexpr size_t kLdsBytes = 160 * 1024;
constexpr size_t kLdsDoubles = kLdsBytes / sizeof(double);

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

// Kernel choice and workspace layout of one call.
//   fp32: cm32_predict_kernel (rows + alpha in LDS as f32; falls back to the f64 kernel when
//         they do not fit);
//   cm:   cm_predict_kernel; LDS: rows [n_pad][DIM] + alpha [n_obj][n_pad], then either the SEP
//         tables (integer grid) or |x_f|^2 (explicit, upper form) + the 2^(j/256) table; when
//         that exceeds 160 KiB the rows / alpha stay in global memory (grows) and only the
//         table is in LDS -- no cap on N beyond the packed W's 2 GiB;
//   kmem: kmem_predict_kernel (materialised k_star).
int make_plan(const bo_predict_desc* d, Plan* pl, bool query_device, bool kmem = false) {
  if (!d || d->n_obj < 1 || d->n_obj > BO_MAX_OBJ || d->dim < 1 || d->dim > BO_MAX_DIM)
    return BO_ERR_ARG;
  if (d->n_train < 1 || d->n_cand < 0 || d->topq < 0 || d->topq > BO_MAX_TOPQ) return BO_ERR_ARG;
  if (d->cand_kind < 0 || d->cand_kind > BO_CAND_SOBOL) return BO_ERR_ARG;
  if (d->mode & ~(BO_PREDICT_DENSE | BO_PREDICT_NO_SEPARABLE | BO_PREDICT_FP32 | BO_PREDICT_F32_FLOOR)) return BO_ERR_ARG;
  if (d->excl_points && d->n_excl < 0) return BO_ERR_ARG;
  const long long n = d->n_train;
  if (n > (1 << 14)) return BO_ERR_UNSUPPORTED;
  memset(pl, 0, sizeof(*pl));
  pl->dim_pad = pad_dim(d->dim);
  pl->n_excl = (int)(d->excl_points ? d->n_excl : n);
  pl->n_panels = 1;
  if ((d->mode & BO_PREDICT_FP32) && !kmem) {
    const int n_pad = (int)((n + 63) / 64 * 64);
    const size_t lds = ((size_t)n_pad * pl->dim_pad + (size_t)d->n_obj * n_pad) * sizeof(float);
    if (lds <= kLdsBytes) {
      pl->fp32 = true;
      pl->n_pad = n_pad;
      pl->ns = 16;
      pl->lds = lds;
    }
  }
  if (!pl->fp32 && !kmem) {
    const int n_pad = pad_rows(n);
    const size_t base = (size_t)n_pad * pl->dim_pad + (size_t)d->n_obj * n_pad;
    pl->cm = true;
    pl->n_pad = n_pad;
    pl->ns = n_pad / 4;
    // non-SEP layout: rows + alpha, exp table
    const size_t plain = base + bo::kExpTab;
    size_t lds = plain;
    if (d->cand_kind == BO_CAND_GRID && !(d->mode & BO_PREDICT_NO_SEPARABLE)) {
      const long long S = d->grid_shape[d->dim - 1];
      const size_t tbl = (size_t)d->n_obj * (2 * S - 1);
      // per wave: n_obj (cached; + the row's S-bit bitmap of evaluated columns) or 1 slot of row
      // factors + the int index / on-row arrays
      const size_t rw_c = (size_t)n_pad * (d->n_obj + 1) + (size_t)(S + 63) / 64;
      const size_t lds_c = base + tbl + (size_t)kWaves * rw_c;
      const size_t lds_1 = base + tbl + (size_t)kWaves * n_pad * 2;
      if (S % 16 == 0 && S <= 32768 && d->cand_offset % 16 == 0 && lds_1 <= kLdsDoubles) {
        pl->sep = true;
        pl->rw_cache = lds_c <= kLdsDoubles;
        pl->rw_stride = (int)(pl->rw_cache ? rw_c : (size_t)n_pad * 2);
        pl->off_tbl = (int)base;
        pl->off_rw = (int)(base + tbl);
        lds = pl->rw_cache ? lds_c : lds_1;
        if (lds < plain) lds = plain;          // the non-SEP fallback shares the kernel's LDS
      }
    }
    pl->off_exp = (int)base;
    if (lds > kLdsDoubles) {
      // rows / |x_f|^2 / alpha from global memory; the exp table alone in LDS
      pl->sep = false;
      pl->grows = true;
      pl->off_exp = 0;
      lds = bo::kExpTab;
    }
    pl->lds = lds * sizeof(double);
    // N <= 128: the 4-accumulator kernel, two workgroups per CU (LDS permitting)
#ifndef BO_ABL_NOSMALL
    pl->small = !pl->grows && n_pad <= 4 * 32 && pl->lds <= kLdsBytes / 2 - 1024;
#endif
  }
  if (kmem) {
    int n_pad = pad_rows(n);
    int ns;
    bool multi = false;
    if (n_pad <= 32) ns = 8;
    else if (n_pad <= 64) ns = 16;
    else if (n_pad <= 128) ns = 32;
    else if (n_pad <= 256) ns = 64;
    else { ns = bo::kPanelSteps; multi = true; }   // panels of 512 rows above 256 rows
    n_pad = multi ? (int)((n + 511) / 512 * 512) : ns * 4;
    pl->n_pad = n_pad;
    pl->ns = ns;
    pl->multi = multi;
    pl->n_panels = multi ? n_pad / 512 : 1;
    pl->lds = (size_t)d->n_obj * n_pad * sizeof(double);
    if (pl->lds > 160 * 1024) return BO_ERR_UNSUPPORTED;
  }
  const int n_pad = pl->n_pad;
  const size_t w_bytes = (size_t)d->n_obj * n_pad * n_pad * sizeof(double);
  if (w_bytes >= (1ull << 31)) return BO_ERR_UNSUPPORTED;
  pl->waves = kWaves;
  const long long n_tiles = (d->n_cand + kTile - 1) / kTile;
  pl->n_tiles = n_tiles;
  const int cus = query_device ? num_cus() : 256;
#ifdef BO_SMALL_ONE_SLOT
  // diagnostic build (BO_BUILD_VARIANT=DEF_SMALL_ONE_SLOT): the small kernel on one workgroup per
  // CU, i.e. one wave per SIMD -- what a two-tile wave would run at
  const int slots = cus;
#else
  const int slots = pl->small ? 2 * cus : cus;
#endif
  pl->grid = (int)(n_tiles < slots ? (n_tiles > 0 ? n_tiles : 1) : slots);
  pl->off_alpha = align256(w_bytes);
  pl->off_xpad = pl->off_alpha + align256((size_t)d->n_obj * n_pad * sizeof(double));
  pl->off_xc = pl->off_xpad + align256((size_t)n_pad * pl->dim_pad * sizeof(double));
  pl->off_excl = pl->off_xc + align256((size_t)n_pad * pl->dim_pad * sizeof(double));
  pl->off_hash = pl->off_excl + align256((size_t)(pl->n_excl + 1) * pl->dim_pad * sizeof(double));
  pl->hash_slots = bo_hash_slots(pl->n_excl);
  pl->off_partial = pl->off_hash + align256((size_t)pl->hash_slots * 12);
  // partial lists sized for the largest persistent grid any device could use
  pl->off_status = pl->off_partial +
                   align256((size_t)1024 * kWaves * (d->topq > 0 ? d->topq : 1) * sizeof(TopEntry));
  pl->total = pl->off_status + 256 + 256;   // +16: separable-K* flag
  return BO_OK;
}

template <int NS, bool MULTI>
hipError_t launch_kmem_k(const FusedArgs& fa, int grid, size_t lds, hipStream_t st) {
  auto k = kmem_predict_kernel<NS, MULTI>;
  if (lds > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)lds);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(k, dim3(grid), dim3(256), lds, st, fa);
  return hipGetLastError();
}

hipError_t launch_kmem(const Plan& pl, const FusedArgs& fa, hipStream_t s) {
  if (pl.multi) return launch_kmem_k<bo::kPanelSteps, true>(fa, pl.grid, pl.lds, s);
  switch (pl.ns) {
    case 8: return launch_kmem_k<8, false>(fa, pl.grid, pl.lds, s);
    case 16: return launch_kmem_k<16, false>(fa, pl.grid, pl.lds, s);
    case 32: return launch_kmem_k<32, false>(fa, pl.grid, pl.lds, s);
    default: return launch_kmem_k<64, false>(fa, pl.grid, pl.lds, s);
  }
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
  double* xc = (double*)(ws + pl.off_xc);
  double* excl = (double*)(ws + pl.off_excl);
  TopEntry* partial = (TopEntry*)(ws + pl.off_partial);
  int* sep_flag = (int*)(ws + pl.off_status + 16);

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
    fa.idx32 = d->cand_offset + d->n_cand < (1LL << 31) ? 1 : 0;
    for (int k = 0; k < d->dim; ++k) fa.idx32 = fa.idx32 && d->grid_shape[k] < (1LL << 31);
  }
  fa.cand = d->cand;
  if (d->cand_kind == BO_CAND_SOBOL) {
    if (!d->cand) return BO_ERR_ARG;
    st = bo_sobol_fill(&fa.sob, d->dim, (const bo_sobol_desc*)d->cand);
    if (st != BO_OK) return st;
    if (d->cand_offset < 0 || (unsigned long long)(d->cand_offset + d->n_cand) > (1ull << fa.sob.bits))
      return BO_ERR_ARG;
  }
  fa.xpad = xpad;
  fa.xc = xc;
  fa.excl = d->excl_points ? excl : nullptr;
  fa.hkeys = (const unsigned long long*)(ws + pl.off_hash);
  fa.hidx = (const int*)(ws + pl.off_hash + (size_t)pl.hash_slots * 8);
  fa.hmask = pl.hash_slots - 1;
  fa.wpack = wpack;
  fa.upper = (pl.cm && !(d->mode & BO_PREDICT_DENSE)) ? 1 : 0;
  fa.wpack_bytes = (unsigned int)((size_t)d->n_obj * pl.n_pad * pl.n_pad * sizeof(double));
  if (pl.cm) {
    // contiguous objective streams of 2-KiB pairs (pack_cm_range); the ring wraps at the end
    fa.w_pairs = (int)(cm_blocks(pl.n_pad / 32, fa.upper) * 4 * d->n_obj);
    fa.wpack_bytes = (unsigned int)((size_t)fa.w_pairs * 2048);
  }
  fa.alpha = alpha;
  for (int o = 0; o < d->n_obj; ++o) {
    fa.pm[o] = d->prior_mean[o];
    fa.pv[o] = d->prior_var[o];
    const double ls = d->length_scale[o];
    fa.nhl[o] = -0.5 / (ls * ls);
    fa.beta[o] = d->beta[o];
    fa.inv_rsq_pv[o] = 1.0 / sqrt(d->prior_var[o]);
    fa.inv_pv[o] = 1.0 / d->prior_var[o];
  }
  fa.min_var = (d->mode & BO_PREDICT_F32_FLOOR) ? BO_MIN_VARIANCE_F32 : BO_MIN_VARIANCE;
  fa.mu = d->mu;
  fa.var = d->var;
  fa.std_mu = d->std_mu;
  fa.std_var = d->std_var;
  fa.ucb = d->ucb;
  fa.acq = d->acq;
  fa.partial = partial;
  fa.kstar = kstar;
  fa.ks_rows = ks_rows;

  fa.sep_flag = pl.sep ? sep_flag : nullptr;
  fa.sep_S = pl.sep ? (int)d->grid_shape[d->dim - 1] : 1;
  fa.sep_lo = pl.sep ? d->grid_lo[d->dim - 1] : 0;
  fa.off_tbl = pl.off_tbl;
  fa.off_rw = pl.off_rw;
  fa.rw_cache = pl.rw_cache ? 1 : 0;
  fa.rw_stride = pl.rw_stride;
  fa.off_exp = pl.off_exp;
  {
    PrepArgs pa;
    memset(&pa, 0, sizeof(pa));
    pa.pack_mode = pl.fp32 ? 2 : (pl.cm ? 0 : 1);
    pa.wpack = wpack;
    pa.kinv = d->kinv;
    pa.ld_k = d->ld_k;
    pa.upper = fa.upper;
    pa.n = (int)d->n_train;
    pa.n_pad = pl.n_pad;
    pa.ns = pl.ns;
    pa.n_obj = d->n_obj;
    const long long total = pl.fp32 ? c32_blocks(pl.n_pad / 64) * 1024 * d->n_obj
                          : pl.cm ? cm_blocks(pl.n_pad / 32, fa.upper) * 512 * d->n_obj
                                  : (long long)d->n_obj * pl.n_pad * pl.n_pad / 2;
    pa.pack_blocks = (int)((total + 255) / 256 < 2048 ? (total + 255) / 256 : 2048);
    pa.alpha_blocks = (int)(((long long)d->n_obj * pl.n_pad + 3) / 4);
    pa.alpha = alpha;
    pa.y = d->y_train;
    pa.ld_y = d->ld_y;
    for (int o = 0; o < d->n_obj; ++o) pa.pm[o] = d->prior_mean[o];
    pa.rows = kmem ? 0 : 1;
    pa.xpad = xpad;
    pa.xc = xc;
    pa.x = d->x_train;
    pa.dim = d->dim;
    pa.DIM = pl.dim_pad;
    pa.sep_flag = pl.sep ? sep_flag : nullptr;
    pa.sep_lo = fa.sep_lo;
    pa.sep_S = fa.sep_S;
    pa.excl = excl;
    pa.excl_in = d->excl_points;
    pa.n_excl = (kmem || !d->excl_points) ? 0 : pl.n_excl;
    pa.hkeys = (unsigned long long*)fa.hkeys;
    pa.hidx = (int*)fa.hidx;
    pa.hslots = pl.hash_slots;
    pa.n_hash = (kmem || d->topq == 0) ? 0 : pl.n_excl;
    pa.hash_lds = pa.n_hash > 0 && pl.hash_slots <= 2048 ? 1 : 0;     // <= 24 KiB of LDS
    const size_t prep_lds = pa.hash_lds ? (size_t)pl.hash_slots * 12 : 0;
    hipLaunchKernelGGL(predict_prep_kernel, dim3((unsigned)(2 + pa.alpha_blocks + pa.pack_blocks)), dim3(256),
                       prep_lds, s, pa);
    BO_CHECK_HIP(hipGetLastError());
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
    case 2: e = bo::launch_c32_d2(pl, fa, s); break;
    case 4: e = bo::launch_c32_d4(pl, fa, s); break;
    case 6: e = bo::launch_c32_d6(pl, fa, s); break;
    default: e = bo::launch_c32_d8(pl, fa, s); break;
  }
  else switch (pl.dim_pad) {
    case 2: e = bo::launch_cm_d2(pl, fa, s); break;
    case 4: e = bo::launch_cm_d4(pl, fa, s); break;
    case 6: e = bo::launch_cm_d6(pl, fa, s); break;
    default: e = bo::launch_cm_d8(pl, fa, s); break;
  }
  if (e != hipSuccess) return BO_ERR_HIP;
  if (timed) timer_mark(s);
  if (d->topq > 0) {
    // q <= 4: the lean rounds merge (a lane per wave list, bo_select.hip); else the general one
    const long long nl = (long long)pl.grid * pl.waves;
    if (!bo_launch_rounds_merge(partial, nl, d->topq, d->top_val, d->top_idx, s)) {
      hipLaunchKernelGGL(bo_topq_merge_kernel, dim3(1), dim3(256), 0, s, partial, nl, d->topq, d->top_val,
                         (long long*)d->top_idx);
      BO_CHECK_HIP(hipGetLastError());
    }
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
