// Chunk-major predict kernels for padded input dimension 2 (see bo_predict_impl.h).
#define BO_PREDICT_DIM 2
#include "bo_predict_impl.h"
