// gemm_f32_kernel<AM_SHIFT3, BM_NT, PRO_NONE, PRO_NONE, ...> with epilogue addends: the 3x3
// data gradient accumulated in place into a shared gradient buffer (addend = C itself).
#include "gemm_dispatch.h"
GEMM_DEFINE_TABLE_E(g_gemm_sh3_nt_ups, AM_SHIFT3, BM_NT, PRO_NONE, PRO_NONE, EPI_UPS)
