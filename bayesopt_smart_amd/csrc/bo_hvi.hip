// Exact hypervolume improvement of each candidate's optimistic objective vector over the
// Pareto front of the evaluated points (maximisation, reference point r).
//
// The reference names this acquisition (bayesian_optimization.py:65 `reference_point`,
// :195-199 "Update hypervolume improvement acquisition function", acquisition.py:89-108) but
// computes the sum of per-objective UCBs; its reference point is unused.  bo_predict_acquire
// keeps that sum bit-for-bit as the default.  This file is the true HVI the reference's name
// promises, an opt-in acquisition:
//
//   HVI(p) = HV(F u {p}) - HV(F) = vol([r, p] n N),   N = {x >= r : no f in F with f >= x}
//
// N (the region not dominated by the front) is decomposed once per iteration on the host into
// disjoint axis-aligned boxes [l_b, u_b) (bo_hvi_boxes: grid columns over the front's
// coordinates on the first m-1 axes, each column open upwards from the highest front value
// dominating it; equal neighbouring columns merged), so that per candidate
//
//   HVI(p) = sum_b prod_k max(0, min(p_k, u_bk) - l_bk)
//
// which is one HBM pass over the stored UCB arrays (8 m bytes in, 8 bytes out per candidate)
// plus m-wide min/sub/max/mul per box on the VALU, with the boxes read at wave-uniform
// addresses (scalar loads, no LDS).
//
// p is the candidate's UCB in the objectives' own units: p_k = shift_k + scale_k * ucb_k, with
// ucb the reference's standardised UCB array (acquisition.py:52 over numba_kernels.py:538-570:
// shift = prior mean, scale = sqrt(prior variance) maps it back to mu + beta sigma).

#include "bo_common.h"

#include <math.h>
#include <string.h>

#include <algorithm>
#include <cmath>
#include <vector>

namespace {

struct HviArgs {
  double* acq;
  const double* ucb;
  long long ld, n;
  const double* boxes;     // [n_boxes][2 m]: lower[m], upper[m] (+inf allowed)
  long long n_boxes;
  double shift[BO_MAX_OBJ], scale[BO_MAX_OBJ];
};

// One thread per candidate (grid-stride).  Boxes are walked in order at a wave-uniform index,
// so their loads are scalar and shared by the wave; the product is accumulated per box.
template <int M>
__global__ __launch_bounds__(256) void hvi_exact_kernel(const HviArgs a) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i0 = (long long)blockIdx.x * blockDim.x; i0 < a.n; i0 += stride) {
    const long long i = i0 + threadIdx.x;
    const bool valid = i < a.n;
    double p[M];
    bool nan = false;
#pragma unroll
    for (int k = 0; k < M; ++k) {
      const double u = valid ? a.ucb[(long long)k * a.ld + i] : 0.0;
      p[k] = __builtin_fma(a.scale[k], u, a.shift[k]);
      nan = nan || (p[k] != p[k]);
    }
    double h = 0.0;
    const double* b = a.boxes;
    for (long long t = 0; t < a.n_boxes; ++t, b += 2 * M) {
      double v = 1.0;
#pragma unroll
      for (int k = 0; k < M; ++k) {
        const double hi = p[k] < b[M + k] ? p[k] : b[M + k];
        v *= fmax(hi - b[k], 0.0);
      }
      h += v;
    }
    if (valid) a.acq[i] = nan ? __builtin_nan("") : h;
  }
}

// out[0] = sum over boxes [b0, b1) of prod_k max(0, min(upper_bk, ub_k) - lower_bk): the volume
// of the boxes clipped to [., ub].  One workgroup, boxes strided over its threads, fixed-order
// tree reduction (deterministic).
__global__ __launch_bounds__(1024) void box_volume_kernel(const double* __restrict__ boxes, long long n_boxes,
                                                          int m, HviArgs ub, double* __restrict__ out) {
  __shared__ double red[1024];
  double s = 0.0;
  for (long long b = threadIdx.x; b < n_boxes; b += blockDim.x) {
    double v = 1.0;
    for (int k = 0; k < m; ++k) {
      const double hi = boxes[b * 2 * m + m + k] < ub.shift[k] ? boxes[b * 2 * m + m + k] : ub.shift[k];
      v *= fmax(hi - boxes[b * 2 * m + k], 0.0);
    }
    s += v;
  }
  red[threadIdx.x] = s;
  __syncthreads();
  for (int w = blockDim.x / 2; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[0] = red[0];
}

int launch_hvi(const HviArgs& a, int m, hipStream_t s) {
  long long blocks = (a.n + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  if (blocks < 1) blocks = 1;
  switch (m) {
    case 1: hipLaunchKernelGGL(hvi_exact_kernel<1>, dim3((unsigned)blocks), dim3(256), 0, s, a); break;
    case 2: hipLaunchKernelGGL(hvi_exact_kernel<2>, dim3((unsigned)blocks), dim3(256), 0, s, a); break;
    case 3: hipLaunchKernelGGL(hvi_exact_kernel<3>, dim3((unsigned)blocks), dim3(256), 0, s, a); break;
    case 4: hipLaunchKernelGGL(hvi_exact_kernel<4>, dim3((unsigned)blocks), dim3(256), 0, s, a); break;
    default: return BO_ERR_UNSUPPORTED;
  }
  BO_CHECK_HIP(hipGetLastError());
  return BO_OK;
}

}  // namespace

extern "C" {

// Host-side decomposition of the non-dominated region (see the file comment).
int bo_hvi_boxes(const double* front, int64_t n, int32_t n_obj, const double* ref_point,
                 double* boxes, int64_t capacity, int64_t* n_boxes) {
  if (!ref_point || !n_boxes || n < 0 || (n > 0 && !front) || n_obj < 1 || n_obj > 4 ||
      capacity < 0 || (capacity > 0 && !boxes))
    return BO_ERR_ARG;
  const int m = n_obj, ax = m - 1;            // grid axes 0..m-2, open axis m-1
  for (int k = 0; k < m; ++k)
    if (!(ref_point[k] == ref_point[k]) || std::isinf(ref_point[k])) return BO_ERR_ARG;
  // front points that bound any volume above r: finite and strictly above r on every axis
  // (others, and NaN rows, add nothing to HV(F))
  std::vector<double> f;
  for (int64_t i = 0; i < n; ++i) {
    bool ok = true;
    for (int k = 0; k < m; ++k) {
      const double v = front[i * m + k];
      ok = ok && std::isfinite(v) && v > ref_point[k];
    }
    if (ok) f.insert(f.end(), front + i * m, front + (i + 1) * m);
  }
  const int64_t P = (int64_t)f.size() / m;
  // per grid axis: sorted unique {r_k} u {f_ik}; cell t spans [c[t], c[t+1]) (last: +inf)
  std::vector<std::vector<double>> c(ax > 0 ? ax : 0);
  int64_t cols = 1;
  for (int k = 0; k < ax; ++k) {
    c[k].push_back(ref_point[k]);
    for (int64_t i = 0; i < P; ++i) c[k].push_back(f[i * m + k]);
    std::sort(c[k].begin(), c[k].end());
    c[k].erase(std::unique(c[k].begin(), c[k].end()), c[k].end());
    cols *= (int64_t)c[k].size();
    if (cols > ((int64_t)1 << 26)) return BO_ERR_UNSUPPORTED;
  }
  const double inf = __builtin_inf();
  std::vector<int64_t> idx(ax > 0 ? ax : 1, 0);
  int64_t count = 0;
  // columns in row-major order over the grid axes; the last grid axis varies fastest, so
  // neighbouring columns with equal open-axis floor are merged into one box along it
  double prev_h = 0.0;
  bool open = false;                     // a pending box that may still be extended
  std::vector<double> lo(m), hi(m);
  auto flush = [&]() {
    if (!open) return;
    if (count < capacity)
      for (int k = 0; k < m; ++k) { boxes[count * 2 * m + k] = lo[k]; boxes[count * 2 * m + m + k] = hi[k]; }
    ++count;
    open = false;
  };
  for (int64_t col = 0; col < cols; ++col) {
    // decode the column index (last grid axis fastest)
    int64_t r = col;
    for (int k = ax - 1; k >= 0; --k) { idx[k] = r % (int64_t)c[k].size(); r /= (int64_t)c[k].size(); }
    // floor of the column's non-dominated part: max f_open over front points whose first m-1
    // coordinates reach the column's upper corner
    double h = ref_point[ax];
    for (int64_t i = 0; i < P; ++i) {
      bool dom = true;
      for (int k = 0; k < ax && dom; ++k) {
        const int64_t t = idx[k] + 1;
        dom = t < (int64_t)c[k].size() && f[i * m + k] >= c[k][t];
      }
      if (dom && f[i * m + ax] > h) h = f[i * m + ax];
    }
    const bool first_in_run = ax == 0 || idx[ax - 1] == 0;
    if (open && !first_in_run && h == prev_h) {
      const int64_t t = idx[ax - 1] + 1;       // extend along the last grid axis
      hi[ax - 1] = t < (int64_t)c[ax - 1].size() ? c[ax - 1][t] : inf;
      continue;
    }
    flush();
    for (int k = 0; k < ax; ++k) {
      lo[k] = c[k][idx[k]];
      const int64_t t = idx[k] + 1;
      hi[k] = t < (int64_t)c[k].size() ? c[k][t] : inf;
    }
    lo[ax] = h;
    hi[ax] = inf;
    prev_h = h;
    open = true;
  }
  flush();
  *n_boxes = count;
  return count > capacity ? BO_ERR_WORKSPACE : BO_OK;
}

int bo_hypervolume_improvement_exact(double* acq, const double* ucb, int64_t ld, int64_t n,
                                     int32_t n_obj, const double* shift, const double* scale,
                                     const double* boxes, int64_t n_boxes, void* stream) {
  if (!acq || !ucb || !shift || !scale || n < 0 || ld < n || n_obj < 1 || n_obj > 4 ||
      n_boxes < 0 || (n_boxes > 0 && !boxes))
    return BO_ERR_ARG;
  if (n == 0) return BO_OK;
  HviArgs a;
  memset(&a, 0, sizeof(a));
  a.acq = acq;
  a.ucb = ucb;
  a.ld = ld;
  a.n = n;
  a.boxes = boxes;
  a.n_boxes = n_boxes;
  for (int k = 0; k < n_obj; ++k) { a.shift[k] = shift[k]; a.scale[k] = scale[k]; }
  return launch_hvi(a, n_obj, (hipStream_t)stream);
}

int bo_box_volume_sum(const double* boxes, int64_t n_boxes, int32_t n_obj, const double* upper,
                      double* out, void* stream) {
  if (!out || !upper || n_obj < 1 || n_obj > 4 || n_boxes < 0 || (n_boxes > 0 && !boxes)) return BO_ERR_ARG;
  HviArgs ub;
  memset(&ub, 0, sizeof(ub));
  for (int k = 0; k < n_obj; ++k) ub.shift[k] = upper[k];
  hipLaunchKernelGGL(box_volume_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, boxes,
                     (long long)n_boxes, n_obj, ub, out);
  BO_CHECK_HIP(hipGetLastError());
  return BO_OK;
}

}  // extern "C"
