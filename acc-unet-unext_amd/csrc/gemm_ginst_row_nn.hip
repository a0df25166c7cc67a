// gemm_f32g_kernel<AM_ROW, BM_NN, PRO_NONE, PRO_NONE, ...>: LDS-DMA fp32 engine table.
#include "gemm_dispatch.h"
GEMM_DEFINE_GTABLE(g_ggemm_row_nn, AM_ROW, BM_NN, PRO_NONE, PRO_NONE, 0)
