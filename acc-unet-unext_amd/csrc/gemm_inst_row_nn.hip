// Explicit instantiation table for gemm_f32_kernel<AM_ROW, BM_NN, PRO_NONE, PRO_NONE, ...>.
#include "gemm_dispatch.h"
GEMM_DEFINE_TABLE(g_gemm_row_nn, AM_ROW, BM_NN, PRO_NONE, PRO_NONE)
