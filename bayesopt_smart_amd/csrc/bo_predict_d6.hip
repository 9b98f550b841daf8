// Chunk-major predict kernels for padded input dimension 6 (see bo_predict_impl.h).
#define BO_PREDICT_DIM 6
#include "bo_predict_impl.h"
