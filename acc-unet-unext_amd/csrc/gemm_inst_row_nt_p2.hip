// Explicit instantiation table for gemm_f32_kernel<AM_ROW, BM_NT, PRO_AFFINE_LRELU, PRO_NONE, ...>.
#include "gemm_dispatch.h"
GEMM_DEFINE_TABLE_S(g_gemm_row_nt_p2, AM_ROW, BM_NT, PRO_AFFINE_LRELU, PRO_NONE)
