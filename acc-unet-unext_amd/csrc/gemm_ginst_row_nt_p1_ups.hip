// gemm_f32g_kernel<AM_ROW, BM_NT, PRO_AFFINE, PRO_NONE, ...>: LDS-DMA fp32 engine table.
#include "gemm_dispatch.h"
GEMM_DEFINE_GTABLE(g_ggemm_row_nt_p1_ups, AM_ROW, BM_NT, PRO_AFFINE, PRO_NONE, EPI_UPS | EPI_STATS)
