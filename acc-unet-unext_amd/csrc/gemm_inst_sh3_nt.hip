// Explicit instantiation table for gemm_f32_kernel<AM_SHIFT3, BM_NT, PRO_NONE, PRO_NONE, ...>.
#include "gemm_dispatch.h"
GEMM_DEFINE_TABLE_S(g_gemm_sh3_nt, AM_SHIFT3, BM_NT, PRO_NONE, PRO_NONE)
