// bf16-engine table gemm_bf16_kernel<AM_COL, BM_NN_SHIFT3, PRO_NONE, PRO_NONE, ...> (bf16 x bf16 activations -> fp32 weight gradient).
#include "gemm_dispatch.h"
GEMM_DEFINE_BTABLE_WGRAD(g_bgemm_col_nnsh3, AM_COL, BM_NN_SHIFT3, PRO_NONE, PRO_NONE)
