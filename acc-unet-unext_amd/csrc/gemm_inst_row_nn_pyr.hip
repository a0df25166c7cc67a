// gemm_f32_kernel<AM_ROW, BM_NN, ...> with the fused HANCLayer pyramid backward epilogue.
#include "gemm_dispatch.h"
GEMM_DEFINE_TABLE_E(g_gemm_row_nn_pyr, AM_ROW, BM_NN, PRO_NONE, PRO_NONE, EPI_PYR)
