// Explicit instantiation table for gemm_f32_kernel<AM_COL, BM_NN, PRO_NONE, PRO_AFFINE_LRELU, ...>.
#include "gemm_dispatch.h"
GEMM_DEFINE_TABLE(g_gemm_col_nn_p2, AM_COL, BM_NN, PRO_NONE, PRO_AFFINE_LRELU)
