// gemm_f32g_kernel<AM_ROW, BM_NT, PRO_AFFINE_LRELU, PRO_NONE, ...>: LDS-DMA fp32 engine table.
#include "gemm_dispatch.h"
GEMM_DEFINE_GTABLE(g_ggemm_row_nt_p2, AM_ROW, BM_NT, PRO_AFFINE_LRELU, PRO_NONE, EPI_STATS)
