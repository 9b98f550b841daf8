// Small-N (MAXEP = 4) chunk-major predict kernels for padded input dimension 6, compiled with
// the MFMA accumulators in arch VGPRs (build.py: -amdgpu-mfma-vgpr-form); see bo_predict_impl.h.
#define BO_PREDICT_SMALL_DIM 6
#include "bo_predict_impl.h"
