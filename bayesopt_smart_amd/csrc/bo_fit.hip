// GP fit on device: invert_k (numba_kernels.py:370-403) and compute_mll (:152-235).
#include "bo_common.h"

extern "C" {

size_t bo_invert_k_workspace_size(int32_t n_obj, int64_t n) {
  return (size_t)n_obj * n * n * sizeof(double) + 4096;
}

int bo_invert_k(double* out, const double* km, int64_t ld, int32_t n_obj, int64_t n, void* ws,
                size_t ws_bytes, void* stream) {
  (void)out; (void)km; (void)ld; (void)n_obj; (void)n; (void)ws; (void)ws_bytes; (void)stream;
  return BO_ERR_UNSUPPORTED;
}

size_t bo_compute_mll_workspace_size(int32_t n_obj, int64_t n) {
  return (size_t)n_obj * n * n * sizeof(double) + 4096;
}

int bo_compute_mll(double* mll_out, const double* x, int32_t dim, const double* y, int64_t ld_y,
                   double* km, int64_t ld, int32_t n_obj, const double* pm, const double* pv,
                   const double* ls, int64_t cur, void* ws, size_t ws_bytes, void* stream) {
  (void)mll_out; (void)x; (void)dim; (void)y; (void)ld_y; (void)km; (void)ld; (void)n_obj;
  (void)pm; (void)pv; (void)ls; (void)cur; (void)ws; (void)ws_bytes; (void)stream;
  return BO_ERR_UNSUPPORTED;
}

}  // extern "C"
