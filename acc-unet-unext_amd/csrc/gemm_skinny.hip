// Skinny weight-gradient GEMM: C[M][N] = sum_k A(m,k) B(k,n) with A column-mode
// ([K][lda] rows of M values, AMODE_COL) and B row-major ([K][ldb], BMODE_NN), small
// M and N (multiples of 32, at most 3 output tiles of 32x32) and a huge K (the
// pixels of a batch): the weight gradients of the 1x1 convolutions (dW = X^T dZ)
// and of narrow layers. The tiled GEMM gives such a shape one output tile and
// splits K 1024 ways, each split streaming 2 KB operand panels through LDS per
// 16-row step: latency-bound at 2-3x the HBM time.
//
// Here every wave streams its own K range straight from global memory into the
// v_mfma_f32_32x32x2_f32 operands: lane l loads A[k0 + l/32][32 i + l%32] and
// B[k0 + l/32][32 j + l%32] (256 contiguous bytes per wave-instruction, two K rows),
// which is exactly the MFMA operand layout, so there is no LDS staging in the main
// loop and 4 K-pairs of loads are issued ahead of their MFMAs. The 4 waves of a
// block reduce their partial tiles in LDS in a fixed order, each block writes one
// slab, and the existing split-K reduction (gemm_run.hip) sums the slabs in a
// fixed order: deterministic, no float atomics.
#include "gemm_dispatch.h"

#define SK_U 4  // K-pairs of loads in flight per wave

struct SkinnyParams {
  int M, N, K;
  const float* A;
  int lda;
  const float* B;
  int ldb;
  const float* b_scale;
  const float* b_shift;
  int rows_per_block;  // multiple of 8
  float* slabs;        // [gridDim.x][M][N]
};

template <int TI, int TJ, int PROB>
__global__ void __launch_bounds__(256) gemm_skinny_kernel(const SkinnyParams p) {
  __shared__ float red[4][32 * 32];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int l31 = lane & 31, lh = lane >> 5;
  const long kb = (long)blockIdx.x * p.rows_per_block;
  const long kend = min((long)p.K, kb + p.rows_per_block);
  const int q = p.rows_per_block / 4;  // rows per wave (even)
  const long k0 = kb + (long)wave * q, k1 = min(kend, k0 + q);
  float bs[TJ], bh[TJ];
#pragma unroll
  for (int j = 0; j < TJ; ++j) {
    bs[j] = PROB != PRO_NONE ? p.b_scale[j * 32 + l31] : 1.f;
    bh[j] = PROB != PRO_NONE ? p.b_shift[j * 32 + l31] : 0.f;
  }
  floatx16 acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  for (long k = k0; k < k1; k += 2 * SK_U) {
    float a[SK_U][TI], b[SK_U][TJ];
#pragma unroll
    for (int u = 0; u < SK_U; ++u) {
      const long kk = k + 2 * u + lh;
      const bool ok = kk < k1;
      const float* ar = p.A + kk * p.lda + l31;
      const float* br = p.B + kk * p.ldb + l31;
#pragma unroll
      for (int i = 0; i < TI; ++i) a[u][i] = ok ? ar[i * 32] : 0.f;
#pragma unroll
      for (int j = 0; j < TJ; ++j) {
        float v = ok ? br[j * 32] : 0.f;
        if (PROB != PRO_NONE && ok) v = pro_apply<PROB>(v, bs[j], bh[j]);
        b[u][j] = v;
      }
    }
#pragma unroll
    for (int u = 0; u < SK_U; ++u)
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[u][i], b[u][j], acc[i][j], 0, 0, 0);
  }
  // block reduction per output tile: wave partials summed in wave order
  float* slab = p.slabs + (size_t)blockIdx.x * p.M * p.N;
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j) {
#pragma unroll
      for (int r = 0; r < 16; ++r)
        red[wave][((r & 3) + 8 * (r >> 2) + 4 * lh) * 32 + l31] = acc[i][j][r];
      __syncthreads();
      for (int e = tid; e < 1024; e += 256) {
        const float s = ((red[0][e] + red[1][e]) + red[2][e]) + red[3][e];
        slab[(size_t)(i * 32 + (e >> 5)) * p.N + j * 32 + (e & 31)] = s;
      }
      __syncthreads();
    }
}

typedef void (*skinny_kfn)(const SkinnyParams);

template <int PROB>
static skinny_kfn skinny_pick(int TI, int TJ) {
#define SK_CASE(I, J) \
  if (TI == I && TJ == J) return gemm_skinny_kernel<I, J, PROB>;
  SK_CASE(1, 1) SK_CASE(1, 2) SK_CASE(2, 1) SK_CASE(1, 3) SK_CASE(3, 1)
#undef SK_CASE
  return nullptr;
}

// Launches the skinny path if the shape qualifies; returns the number of slabs it
// wrote into ws (the caller reduces them), or 0 if the tiled GEMM should run.
int gemm_skinny_try(const GemmParams& p, int amode, int bmode, int pro_a, int pro_b, float* ws,
                    size_t ws_elems, hipStream_t stream) {
  static int off = -1;
  if (off < 0) {
    const char* e = getenv("ACCUNET_NO_SKINNY");  // A/B knob
    off = (e && atoi(e)) ? 1 : 0;
  }
  if (off || amode != AM_COL || bmode != BM_NN || pro_a != PRO_NONE || p.nsrc != 1) return 0;
  if (p.bias || p.nup || p.stats || p.pd2 || p.bz || !ws) return 0;
  if ((p.M & 31) || (p.N & 31) || p.K < 16384) return 0;
  const int TI = p.M / 32, TJ = p.N / 32;
  // measured (tools/gemm_census.py): a clear win while the stream dominates (up to 3
  // output tiles: 32x32 2.1x, 32x96 / 96x32 faster); from 4 tiles the MFMA work per
  // K pair makes the tiled kernel equal or better (64x64 at K 262144: 40 vs 36 us)
  if (TI * TJ > 3) return 0;
  skinny_kfn fn = pro_b == PRO_NONE ? skinny_pick<PRO_NONE>(TI, TJ)
                  : pro_b == PRO_AFFINE ? skinny_pick<PRO_AFFINE>(TI, TJ)
                                        : skinny_pick<PRO_AFFINE_LRELU>(TI, TJ);
  if (!fn) return 0;
  // blocks: ~4 per CU for the stream, fewer if the slabs would not fit ws
  long nb = 1024;
  const long per_slab = (long)p.M * p.N;
  while (nb > 64 && (size_t)(nb * per_slab) > ws_elems) nb >>= 1;
  if ((size_t)(nb * per_slab) > ws_elems) return 0;
  long rows = (p.K + nb - 1) / nb;
  rows = (rows + 7) / 8 * 8;
  nb = (p.K + rows - 1) / rows;
  SkinnyParams s;
  s.M = p.M; s.N = p.N; s.K = p.K;
  s.A = p.A[0]; s.lda = p.lda[0];
  s.B = p.B; s.ldb = p.ldb;
  s.b_scale = p.b_scale; s.b_shift = p.b_shift;
  s.rows_per_block = (int)rows;
  s.slabs = ws;
  hipLaunchKernelGGL(fn, dim3((unsigned)nb), dim3(256), 0, stream, s);
  return (int)nb;
}
