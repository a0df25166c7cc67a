// gemm_f32_kernel<AM_ROW, BM_NT, PRO_NONE, ...> with nearest-upsampled addends in the
// epilogue (HANCLayer coarse branches, MLFC coarse sources).
#include "gemm_dispatch.h"
GEMM_DEFINE_TABLE_E(g_gemm_row_nt_p0_ups, AM_ROW, BM_NT, PRO_NONE, PRO_NONE, EPI_UPS | EPI_STATS)
