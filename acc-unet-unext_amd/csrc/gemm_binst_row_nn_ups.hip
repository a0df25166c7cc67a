// bf16-engine table gemm_bf16_kernel<AM_ROW, BM_NN, PRO_NONE, PRO_NONE, ...> with epilogue
// addends (data gradients accumulated in place; bf16 activations x fp32 weights -> bf16).
#include "gemm_dispatch.h"
GEMM_DEFINE_BTABLE_FWD(g_bgemm_row_nn_ups, AM_ROW, BM_NN, PRO_NONE, PRO_NONE, EPI_UPS)
