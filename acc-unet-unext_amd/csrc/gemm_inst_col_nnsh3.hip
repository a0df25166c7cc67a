// Explicit instantiation table for gemm_f32_kernel<AM_COL, BM_NN_SHIFT3, PRO_NONE, PRO_NONE, ...>.
#include "gemm_dispatch.h"
GEMM_DEFINE_TABLE(g_gemm_col_nnsh3, AM_COL, BM_NN_SHIFT3, PRO_NONE, PRO_NONE)
