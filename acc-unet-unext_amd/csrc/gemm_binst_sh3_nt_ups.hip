// bf16-engine table gemm_bf16_kernel<AM_SHIFT3, BM_NT, PRO_NONE, PRO_NONE, ...> with epilogue
// addends (3x3 data gradient accumulated in place; bf16 x fp32 weights -> bf16).
#include "gemm_dispatch.h"
GEMM_DEFINE_BTABLE_FWD(g_bgemm_sh3_nt_ups, AM_SHIFT3, BM_NT, PRO_NONE, PRO_NONE, EPI_UPS)
