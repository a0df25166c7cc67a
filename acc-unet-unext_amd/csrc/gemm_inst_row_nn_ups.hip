// gemm_f32_kernel<AM_ROW, BM_NN, PRO_NONE, PRO_NONE, ...> with epilogue addends: data
// gradients accumulated in place into a shared gradient buffer (addend = C itself).
#include "gemm_dispatch.h"
GEMM_DEFINE_TABLE_E(g_gemm_row_nn_ups, AM_ROW, BM_NN, PRO_NONE, PRO_NONE, EPI_UPS)
