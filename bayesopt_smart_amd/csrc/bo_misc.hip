// ABI housekeeping (status strings, device count) and the host side of the Sobol candidates.
#include "bo_common.h"

#include <string.h>

// Joe & Kuo direction-number table (new-joe-kuo-6.21201, the table scipy.stats.qmc.Sobol ships
// in _sobol_direction_numbers.npz): primitive polynomial and initial m_j of dimensions 1..8.
static const unsigned int kSobolPoly[BO_MAX_DIM] = {1, 3, 7, 11, 13, 19, 25, 37};
static const unsigned int kSobolInit[BO_MAX_DIM][8] = {
    {1, 0, 0, 0, 0, 0, 0, 0}, {1, 0, 0, 0, 0, 0, 0, 0}, {1, 3, 0, 0, 0, 0, 0, 0},
    {1, 3, 1, 0, 0, 0, 0, 0}, {1, 1, 1, 0, 0, 0, 0, 0}, {1, 1, 3, 3, 0, 0, 0, 0},
    {1, 3, 5, 13, 0, 0, 0, 0}, {1, 1, 5, 5, 17, 0, 0, 0}};

// Bratley & Fox (1988) recurrence: v_j = v_{j-m} ^ (v_{j-m} << m) ^ XOR_k a_k 2^k v_{j-k} over
// the polynomial's coefficients; dimension 1 is van der Corput (all m_j = 1); then v_j is
// scaled by 2^(bits - 1 - j).
int bo_sobol_fill(SobolArgs* s, int dim, const bo_sobol_desc* d) {
  if (!s || !d || dim < 1 || dim > BO_MAX_DIM || d->bits < 1 || d->bits > 32) return BO_ERR_ARG;
  memset(s, 0, sizeof(*s));
  const int bits = d->bits;
  s->bits = bits;
  for (int k = 0; k < dim; ++k) {
    unsigned long long v[32];
    if (k == 0) {
      for (int j = 0; j < bits; ++j) v[j] = 1;
    } else {
      const unsigned int p = kSobolPoly[k];
      int m = 0;
      while ((p >> (m + 1)) != 0) ++m;                 // degree = bit length - 1
      for (int j = 0; j < m && j < bits; ++j) v[j] = kSobolInit[k][j];
      for (int j = m; j < bits; ++j) {
        unsigned long long nv = v[j - m];
        unsigned long long pow2 = 1;
        for (int t = 0; t < m; ++t) {
          pow2 <<= 1;
          if ((p >> (m - 1 - t)) & 1u) nv ^= pow2 * v[j - t - 1];
        }
        v[j] = nv;
      }
    }
    for (int j = 0; j < bits; ++j) s->v[k][j] = (unsigned int)(v[j] << (bits - 1 - j));
    s->lo[k] = d->lo[k];
    s->scale[k] = d->scale[k];
  }
  return BO_OK;
}

extern "C" {

int bo_abi_version(void) { return BO_ABI_VERSION; }

const char* bo_status_string(int s) {
  switch (s) {
    case BO_OK: return "ok";
    case BO_ERR_ARG: return "invalid argument";
    case BO_ERR_UNSUPPORTED: return "unsupported configuration";
    case BO_ERR_WORKSPACE: return "workspace missing or too small";
    case BO_ERR_HIP: return "HIP runtime error";
    case BO_ERR_NOT_PD: return "Matrix is not positive definite";
    case BO_ERR_SINGULAR: return "Singular matrix";
    default: return "unknown status";
  }
}

int bo_sobol_direction_numbers(int32_t dim, int32_t bits, uint32_t* out) {
  if (!out) return BO_ERR_ARG;
  bo_sobol_desc d;
  memset(&d, 0, sizeof(d));
  d.bits = bits;
  SobolArgs s;
  const int st = bo_sobol_fill(&s, dim, &d);
  if (st != BO_OK) return st;
  for (int k = 0; k < dim; ++k)
    for (int j = 0; j < bits; ++j) out[k * bits + j] = s.v[k][j];
  return BO_OK;
}

int bo_sobol_points(const bo_sobol_desc* d, int32_t dim, const int64_t* idx, int64_t n, double* out) {
  if (!d || !idx || !out || n < 0) return BO_ERR_ARG;
  SobolArgs s;
  const int st = bo_sobol_fill(&s, dim, d);
  if (st != BO_OK) return st;
  const unsigned long long lim = s.bits == 32 ? (1ull << 32) : (1ull << s.bits);
  for (int64_t t = 0; t < n; ++t) {
    if (idx[t] < 0 || (unsigned long long)idx[t] >= lim) return BO_ERR_ARG;
    for (int k = 0; k < dim; ++k) out[t * dim + k] = bo_sobol_coord(s, k, (unsigned long long)idx[t]);
  }
  return BO_OK;
}

int bo_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return -1;
  return n;
}

}  // extern "C"
