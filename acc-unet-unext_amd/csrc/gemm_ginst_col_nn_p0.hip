// gemm_f32g_kernel<AM_COL, BM_NN, PRO_NONE, PRO_NONE, ...>: LDS-DMA fp32 engine table.
#include "gemm_dispatch.h"
GEMM_DEFINE_GTABLE(g_ggemm_col_nn_p0, AM_COL, BM_NN, PRO_NONE, PRO_NONE, 0)
