// gemm_f32g_kernel<AM_SHIFT3, BM_NT, PRO_NONE, PRO_NONE, ...> with epilogue addends (3x3
// data gradient accumulated in place): LDS-DMA fp32 engine table.
#include "gemm_dispatch.h"
GEMM_DEFINE_GTABLE(g_ggemm_sh3_nt_ups, AM_SHIFT3, BM_NT, PRO_NONE, PRO_NONE, EPI_UPS)
