// gemm_f32g_kernel<AM_ROW, BM_NN, PRO_NONE, PRO_NONE, ...> with epilogue addends (data
// gradients accumulated in place): LDS-DMA fp32 engine table.
#include "gemm_dispatch.h"
GEMM_DEFINE_GTABLE(g_ggemm_row_nn_ups, AM_ROW, BM_NN, PRO_NONE, PRO_NONE, EPI_UPS)
