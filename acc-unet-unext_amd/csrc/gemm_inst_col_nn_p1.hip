// Explicit instantiation table for gemm_f32_kernel<AM_COL, BM_NN, PRO_NONE, PRO_AFFINE, ...>.
#include "gemm_dispatch.h"
GEMM_DEFINE_TABLE(g_gemm_col_nn_p1, AM_COL, BM_NN, PRO_NONE, PRO_AFFINE)
