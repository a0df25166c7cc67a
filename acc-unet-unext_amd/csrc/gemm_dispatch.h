// Tile selection + template dispatch for gemm_f32_kernel / gemm_bf16_kernel.
#pragma once
#include "gemm_f32.h"
#include "gemm_f32g.h"
#include "gemm_bf16.h"

// Tile configurations (WM, TM, TN) -> (BM, BN):
//   T_A 128x128 (2,2,2)  T_B 128x64 (2,2,1)  T_C 128x32 (4,1,1)
//   T_D 32x128  (1,1,1)  T_E 64x64  (2,1,1)
enum { TILE_A = 0, TILE_B, TILE_C, TILE_D, TILE_E, TILE_COUNT };

static inline int tile_bm(int t) {
  switch (t) { case TILE_A: case TILE_B: case TILE_C: return 128; case TILE_D: return 32; default: return 64; }
}
static inline int tile_bn(int t) {
  switch (t) { case TILE_A: case TILE_D: return 128; case TILE_B: case TILE_E: return 64; default: return 32; }
}

typedef void (*gemm_kfn)(const GemmParams);

// One translation unit per (AMODE,BMODE,PRO_A,PRO_B) defines this table.
#define GEMM_DECLARE_TABLE(NAME) extern gemm_kfn NAME[2][TILE_COUNT];

#define GEMM_DEFINE_TABLE_E(NAME, AM, BMo, PA, PB, EPI)                                   \
  gemm_kfn NAME[2][TILE_COUNT] = {                                                        \
      {gemm_f32_kernel<AM, BMo, PA, PB, false, false, 2, 2, 2, EPI>,                      \
       gemm_f32_kernel<AM, BMo, PA, PB, false, false, 2, 2, 1, EPI>,                      \
       gemm_f32_kernel<AM, BMo, PA, PB, false, false, 4, 1, 1, EPI>,                      \
       gemm_f32_kernel<AM, BMo, PA, PB, false, false, 1, 1, 1, EPI>,                      \
       gemm_f32_kernel<AM, BMo, PA, PB, false, false, 2, 1, 1, EPI>},                     \
      {gemm_f32_kernel<AM, BMo, PA, PB, true, true, 2, 2, 2, EPI>,                        \
       gemm_f32_kernel<AM, BMo, PA, PB, true, true, 2, 2, 1, EPI>,                        \
       gemm_f32_kernel<AM, BMo, PA, PB, true, true, 4, 1, 1, EPI>,                        \
       gemm_f32_kernel<AM, BMo, PA, PB, true, true, 1, 1, 1, EPI>,                        \
       gemm_f32_kernel<AM, BMo, PA, PB, true, true, 2, 1, 1, EPI>}};
#define GEMM_DEFINE_TABLE(NAME, AM, BMo, PA, PB) GEMM_DEFINE_TABLE_E(NAME, AM, BMo, PA, PB, 0)
// forward GEMMs: optional (sum, sumsq) statistics of C for the consumer BatchNorm
#define GEMM_DEFINE_TABLE_S(NAME, AM, BMo, PA, PB) GEMM_DEFINE_TABLE_E(NAME, AM, BMo, PA, PB, EPI_STATS)

// bf16 engine tables (same tile order). Storage per table: forward / data-gradient
// GEMMs read bf16 activations and fp32 weights and write bf16; weight gradients
// read two bf16 activation operands and write fp32.
#define GEMM_DEFINE_BTABLE_E(NAME, AM, BMo, PA, PB, EPI, TA, TB, TC)                        \
  gemm_kfn NAME[2][TILE_COUNT] = {                                                        \
      {gemm_bf16_kernel<AM, BMo, PA, PB, false, false, 2, 2, 2, EPI, TA, TB, TC>,         \
       gemm_bf16_kernel<AM, BMo, PA, PB, false, false, 2, 2, 1, EPI, TA, TB, TC>,         \
       gemm_bf16_kernel<AM, BMo, PA, PB, false, false, 4, 1, 1, EPI, TA, TB, TC>,         \
       gemm_bf16_kernel<AM, BMo, PA, PB, false, false, 1, 1, 1, EPI, TA, TB, TC>,         \
       gemm_bf16_kernel<AM, BMo, PA, PB, false, false, 2, 1, 1, EPI, TA, TB, TC>},        \
      {gemm_bf16_kernel<AM, BMo, PA, PB, true, true, 2, 2, 2, EPI, TA, TB, TC>,           \
       gemm_bf16_kernel<AM, BMo, PA, PB, true, true, 2, 2, 1, EPI, TA, TB, TC>,           \
       gemm_bf16_kernel<AM, BMo, PA, PB, true, true, 4, 1, 1, EPI, TA, TB, TC>,           \
       gemm_bf16_kernel<AM, BMo, PA, PB, true, true, 1, 1, 1, EPI, TA, TB, TC>,           \
       gemm_bf16_kernel<AM, BMo, PA, PB, true, true, 2, 1, 1, EPI, TA, TB, TC>}};
// forward / data gradient: bf16 x fp32-weight -> bf16; weight gradient: bf16 x bf16 -> fp32
#define GEMM_DEFINE_BTABLE_FWD(NAME, AM, BMo, PA, PB, EPI) \
  GEMM_DEFINE_BTABLE_E(NAME, AM, BMo, PA, PB, EPI, bf16_t, float, bf16_t)
#define GEMM_DEFINE_BTABLE_WGRAD(NAME, AM, BMo, PA, PB) \
  GEMM_DEFINE_BTABLE_E(NAME, AM, BMo, PA, PB, 0, bf16_t, bf16_t, float)

// LDS-DMA fp32 engine (gemm_f32g.h): vector-aligned operands only, so both rows of
// the [2][TILE_COUNT] table hold the same kernels (GEMM_TABLE_SELECT shape)
#define GEMM_DEFINE_GTABLE(NAME, AM, BMo, PA, PB, EPI)                                      \
  gemm_kfn NAME[2][TILE_COUNT] = {                                                         \
      {gemm_f32g_kernel<AM, BMo, PA, PB, 2, 2, 2, EPI>, gemm_f32g_kernel<AM, BMo, PA, PB, 2, 2, 1, EPI>, \
       gemm_f32g_kernel<AM, BMo, PA, PB, 4, 1, 1, EPI>, gemm_f32g_kernel<AM, BMo, PA, PB, 1, 1, 1, EPI>, \
       gemm_f32g_kernel<AM, BMo, PA, PB, 2, 1, 1, EPI>},                                   \
      {gemm_f32g_kernel<AM, BMo, PA, PB, 2, 2, 2, EPI>, gemm_f32g_kernel<AM, BMo, PA, PB, 2, 2, 1, EPI>, \
       gemm_f32g_kernel<AM, BMo, PA, PB, 4, 1, 1, EPI>, gemm_f32g_kernel<AM, BMo, PA, PB, 1, 1, 1, EPI>, \
       gemm_f32g_kernel<AM, BMo, PA, PB, 2, 1, 1, EPI>}};

GEMM_DECLARE_TABLE(g_ggemm_col_nn_p0)
GEMM_DECLARE_TABLE(g_ggemm_col_nn_p1)
GEMM_DECLARE_TABLE(g_ggemm_col_nn_p2)
GEMM_DECLARE_TABLE(g_ggemm_col_nnsh3)
GEMM_DECLARE_TABLE(g_ggemm_row_nn)
GEMM_DECLARE_TABLE(g_ggemm_row_nn_ups)
GEMM_DECLARE_TABLE(g_ggemm_row_nn_bnb)
GEMM_DECLARE_TABLE(g_ggemm_row_nn_bnb_pyr)
GEMM_DECLARE_TABLE(g_ggemm_row_nn_pyr)
GEMM_DECLARE_TABLE(g_ggemm_row_nt_p0)
GEMM_DECLARE_TABLE(g_ggemm_row_nt_p0_ups)
GEMM_DECLARE_TABLE(g_ggemm_row_nt_p1)
GEMM_DECLARE_TABLE(g_ggemm_row_nt_p1_ups)
GEMM_DECLARE_TABLE(g_ggemm_row_nt_p2)
GEMM_DECLARE_TABLE(g_ggemm_row_nt_p2_ups)
GEMM_DECLARE_TABLE(g_ggemm_sh3_nt)
GEMM_DECLARE_TABLE(g_ggemm_sh3_nt_ups)
GEMM_DECLARE_TABLE(g_gemm_row_nt_p0)
GEMM_DECLARE_TABLE(g_gemm_row_nt_p1)
GEMM_DECLARE_TABLE(g_gemm_row_nt_p2)
GEMM_DECLARE_TABLE(g_gemm_row_nt_p0_ups)
GEMM_DECLARE_TABLE(g_gemm_row_nt_p1_ups)
GEMM_DECLARE_TABLE(g_gemm_row_nt_p2_ups)
GEMM_DECLARE_TABLE(g_gemm_sh3_nt)
GEMM_DECLARE_TABLE(g_gemm_sh3_nt_ups)
GEMM_DECLARE_TABLE(g_gemm_row_nn)
GEMM_DECLARE_TABLE(g_gemm_row_nn_ups)
GEMM_DECLARE_TABLE(g_gemm_row_nn_bnb)
GEMM_DECLARE_TABLE(g_gemm_row_nn_pyr)
GEMM_DECLARE_TABLE(g_gemm_row_nn_bnb_pyr)
GEMM_DECLARE_TABLE(g_gemm_col_nn_p0)
GEMM_DECLARE_TABLE(g_gemm_col_nn_p1)
GEMM_DECLARE_TABLE(g_gemm_col_nn_p2)
GEMM_DECLARE_TABLE(g_gemm_col_nnsh3)
GEMM_DECLARE_TABLE(g_bgemm_row_nt_p0)
GEMM_DECLARE_TABLE(g_bgemm_row_nt_p1)
GEMM_DECLARE_TABLE(g_bgemm_row_nt_p2)
GEMM_DECLARE_TABLE(g_bgemm_row_nt_p0_ups)
GEMM_DECLARE_TABLE(g_bgemm_row_nt_p1_ups)
GEMM_DECLARE_TABLE(g_bgemm_row_nt_p2_ups)
GEMM_DECLARE_TABLE(g_bgemm_sh3_nt)
GEMM_DECLARE_TABLE(g_bgemm_sh3_nt_ups)
GEMM_DECLARE_TABLE(g_bgemm_row_nn)
GEMM_DECLARE_TABLE(g_bgemm_row_nn_ups)
GEMM_DECLARE_TABLE(g_bgemm_row_nn_bnb)
GEMM_DECLARE_TABLE(g_bgemm_row_nn_pyr)
GEMM_DECLARE_TABLE(g_bgemm_row_nn_bnb_pyr)
GEMM_DECLARE_TABLE(g_bgemm_col_nn_p0)
GEMM_DECLARE_TABLE(g_bgemm_col_nn_p1)
GEMM_DECLARE_TABLE(g_bgemm_col_nn_p2)
GEMM_DECLARE_TABLE(g_bgemm_col_nnsh3)

// Host-side driver: picks a tile, split-K factor and launches. ws (workspace,
// may be null) is used for split-K partial slabs; if the split would not fit it
// falls back to no split. Returns ACC_OK or an error code.
// adt / bdt / cdt: storage of A, B and C (+ activation-shaped epilogue operands):
// all ACC_F32 -> fp32 engine; adt = ACC_BF16 -> bf16 engine (bdt fp32 weights or bf16
// activations, cdt bf16 or fp32 as the tables above).
int gemm_run(GemmParams p, int amode, int bmode, int pro_a, int pro_b, bool allow_split,
             float* ws, size_t ws_elems, int adt, int bdt, int cdt, hipStream_t stream);

// ResPath 3x3 over 32 channels as a halo-tile direct convolution (csrc/conv3x3.hip):
// ACC_OK / an error when it ran the launch, -1 when the GEMM engine should
int conv3x3_c32_try(const GemmParams& p, int amode, int bmode, int pro_a, int pro_b, int epi,
                    int dmode, int tile, hipStream_t stream);

// its weight gradient: the number of [M][N] slabs written into ws (0: not this shape)
int conv3x3_c32_wgrad_try(const GemmParams& p, int amode, int bmode, int pro_a, int pro_b,
                          bool fp32, float* ws, size_t ws_elems, hipStream_t stream);

// Skinny weight-gradient path (csrc/gemm_skinny.hip): returns the number of
// [M][N] partial slabs written into ws (to be summed by the split-K reduction),
// or 0 when the shape does not qualify.
int gemm_skinny_try(const GemmParams& p, int amode, int bmode, int pro_a, int pro_b, float* ws,
                    size_t ws_elems, int dt, hipStream_t stream);
