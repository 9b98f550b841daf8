// Chunk-major predict kernels for padded input dimension 4 (see bo_predict_impl.h).
#define BO_PREDICT_DIM 4
#include "bo_predict_impl.h"
