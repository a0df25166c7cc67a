// bf16-engine table gemm_bf16_kernel<AM_ROW, BM_NT, PRO_AFFINE_LRELU, PRO_NONE, ...> (bf16 activations x fp32 weights -> bf16).
#include "gemm_dispatch.h"
GEMM_DEFINE_BTABLE_FWD(g_bgemm_row_nt_p2, AM_ROW, BM_NT, PRO_AFFINE_LRELU, PRO_NONE, EPI_STATS)
