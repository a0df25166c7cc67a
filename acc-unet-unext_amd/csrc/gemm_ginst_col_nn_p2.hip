// gemm_f32g_kernel<AM_COL, BM_NN, PRO_NONE, PRO_AFFINE_LRELU, ...>: LDS-DMA fp32 engine table.
#include "gemm_dispatch.h"
GEMM_DEFINE_GTABLE(g_ggemm_col_nn_p2, AM_COL, BM_NN, PRO_NONE, PRO_AFFINE_LRELU, 0)
