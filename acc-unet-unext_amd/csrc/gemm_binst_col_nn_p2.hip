// bf16-engine table gemm_bf16_kernel<AM_COL, BM_NN, PRO_NONE, PRO_AFFINE_LRELU, ...> (bf16 x bf16 activations -> fp32 weight gradient).
#include "gemm_dispatch.h"
GEMM_DEFINE_BTABLE_WGRAD(g_bgemm_col_nn_p2, AM_COL, BM_NN, PRO_NONE, PRO_AFFINE_LRELU)
