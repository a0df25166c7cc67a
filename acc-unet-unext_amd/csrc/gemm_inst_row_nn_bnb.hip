// Explicit instantiation tables for gemm_f32_kernel<AM_ROW, BM_NN, ...> data
// gradients with the BatchNorm-backward statistics and/or HANCLayer pyramid epilogues.
#include "gemm_dispatch.h"
GEMM_DEFINE_TABLE_E(g_gemm_row_nn_bnb, AM_ROW, BM_NN, PRO_NONE, PRO_NONE, EPI_BNB)
