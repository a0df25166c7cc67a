// Explicit instantiation table for gemm_f32_kernel<AM_ROW, BM_NN, ...> with the
// BatchNorm-backward statistics epilogue (data gradients feeding a BN backward).
#include "gemm_dispatch.h"
GEMM_DEFINE_TABLE_E(g_gemm_row_nn_bnb, AM_ROW, BM_NN, PRO_NONE, PRO_NONE, 1)
