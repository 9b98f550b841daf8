// Chunk-major predict kernels for padded input dimension 8 (see bo_predict_impl.h).
#define BO_PREDICT_DIM 8
#include "bo_predict_impl.h"
