// Explicit instantiation table for gemm_f32_kernel<AM_ROW, BM_NT, PRO_AFFINE, PRO_NONE, ...>.
#include "gemm_dispatch.h"
GEMM_DEFINE_TABLE_S(g_gemm_row_nt_p1, AM_ROW, BM_NT, PRO_AFFINE, PRO_NONE)
