// Skinny weight-gradient GEMM: C[M][N] = sum_k A(m,k) B(k,n) with A column-mode
// ([K][lda] rows of M values, AMODE_COL) and B row-major ([K][ldb], BMODE_NN) or the
// 3x3 tap gather (BMODE_NN_SHIFT3), small M and N (at most 3 output tiles of 32x32,
// edge tiles masked) and a huge K (the
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
  const void* A;  // fp32 or bf16 (kernel type T)
  int lda;
  const void* B;
  int ldb;
  const float* b_scale;
  const float* b_shift;
  int rows_per_block;  // multiple of 8
  float* slabs;        // [gridDim.x][M][N]
  // BMODE_NN_SHIFT3 (3x3 weight gradient): B(k = pixel, n = tap*cin + ci) =
  // X[shift_tap(k)*ldb + ci], zero outside the H x W image
  int H, W, cin;
  FastDiv fW, fH;
};

template <int TI, int TJ, int PROB, bool SH3, typename T>
__global__ void __launch_bounds__(256) gemm_skinny_kernel(const SkinnyParams p) {
  __shared__ float red[4][32 * 32];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int l31 = lane & 31, lh = lane >> 5;
  const long kb = (long)blockIdx.x * p.rows_per_block;
  const long kend = min((long)p.K, kb + p.rows_per_block);
  const int q = p.rows_per_block / 4;  // rows per wave (even)
  const long k0 = kb + (long)wave * q, k1 = min(kend, k0 + q);
  float bs[TJ], bh[TJ];
  bool nok[TJ];
  int boff[TJ], bdh[TJ], bdw[TJ];  // SH3: per-lane tap offset (constant over k)
#pragma unroll
  for (int j = 0; j < TJ; ++j) {
    const int n = j * 32 + l31;
    nok[j] = n < p.N;
    bs[j] = (PROB != PRO_NONE && nok[j]) ? p.b_scale[n] : 1.f;
    bh[j] = (PROB != PRO_NONE && nok[j]) ? p.b_shift[n] : 0.f;
    boff[j] = n;
    bdh[j] = bdw[j] = 0;
    if (SH3) {
      const int tap = nok[j] ? n / p.cin : 0, ci = nok[j] ? n - tap * p.cin : 0;
      bdh[j] = tap / 3 - 1;
      bdw[j] = tap - (tap / 3) * 3 - 1;
      boff[j] = (bdh[j] * p.W + bdw[j]) * p.ldb + ci;
    }
  }
  bool mok[TI];
#pragma unroll
  for (int i = 0; i < TI; ++i) mok[i] = i * 32 + l31 < p.M;
  floatx16 acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  // Loads are unconditional (masked elements read a valid dummy address, zeroed after
  // the load) and kept raw until every load of the step is issued: a conditional or
  // immediately widened bf16 load makes hipcc wait for it on the spot (vmcnt(0) per
  // element), which serialised the bf16 kernel.
  const T* A0 = (const T*)p.A;
  const T* B0 = (const T*)p.B;
  for (long k = k0; k < k1; k += 2 * SK_U) {
    T ar[SK_U][TI], br[SK_U][TJ];
    bool aok[SK_U][TI], bok[SK_U][TJ];
#pragma unroll
    for (int u = 0; u < SK_U; ++u) {
      const long kk = k + 2 * u + lh;
      const bool ok = kk < k1;
      const T* arow = A0 + kk * p.lda + l31;
#pragma unroll
      for (int i = 0; i < TI; ++i) {
        aok[u][i] = ok && mok[i];
        ar[u][i] = *(aok[u][i] ? arow + i * 32 : A0);
      }
      int hh = 0, ww = 0;
      if (SH3) {
        const uint32_t q = fdiv((uint32_t)kk, p.fW);
        ww = (int)kk - (int)q * p.W;
        hh = (int)(q - fdiv(q, p.fH) * p.H);
      }
      const T* brow = B0 + kk * p.ldb;
#pragma unroll
      for (int j = 0; j < TJ; ++j) {
        bool in = ok && nok[j];
        if (SH3)
          in = in && hh + bdh[j] >= 0 && hh + bdh[j] < p.H && ww + bdw[j] >= 0 &&
               ww + bdw[j] < p.W;
        bok[u][j] = in;
        br[u][j] = *(in ? brow + boff[j] : B0);
      }
    }
    // keep every load of the step ahead of the first MFMA (the scheduler would
    // otherwise interleave the 2-byte bf16 loads with the MFMAs and drain them early)
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < SK_U; ++u) {
      float a[TI], b[TJ];
#pragma unroll
      for (int i = 0; i < TI; ++i) a[i] = aok[u][i] ? ld1(&ar[u][i]) : 0.f;
#pragma unroll
      for (int j = 0; j < TJ; ++j) {
        float v = ld1(&br[u][j]);
        if (PROB != PRO_NONE) v = pro_apply<PROB>(v, bs[j], bh[j]);
        b[j] = bok[u][j] ? v : 0.f;
      }
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i], b[j], acc[i][j], 0, 0, 0);
    }
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
        const int m = i * 32 + (e >> 5), n = j * 32 + (e & 31);
        const float s = ((red[0][e] + red[1][e]) + red[2][e]) + red[3][e];
        if (m < p.M && n < p.N) slab[(size_t)m * p.N + n] = s;
      }
      __syncthreads();
    }
}

typedef void (*skinny_kfn)(const SkinnyParams);

template <int PROB, bool SH3, typename T>
static skinny_kfn skinny_pick(int TI, int TJ) {
#define SK_CASE(I, J) \
  if (TI == I && TJ == J) return gemm_skinny_kernel<I, J, PROB, SH3, T>;
  SK_CASE(1, 1) SK_CASE(1, 2) SK_CASE(2, 1) SK_CASE(1, 3) SK_CASE(3, 1)
#undef SK_CASE
  return nullptr;
}

// Launches the skinny path if the shape qualifies; returns the number of slabs it
// wrote into ws (the caller reduces them), or 0 if the tiled GEMM should run.
template <typename T>
static skinny_kfn skinny_fn(bool sh3, int pro_b, int TI, int TJ) {
  return sh3 ? skinny_pick<PRO_NONE, true, T>(TI, TJ)
         : pro_b == PRO_NONE ? skinny_pick<PRO_NONE, false, T>(TI, TJ)
         : pro_b == PRO_AFFINE ? skinny_pick<PRO_AFFINE, false, T>(TI, TJ)
                               : skinny_pick<PRO_AFFINE_LRELU, false, T>(TI, TJ);
}

// dt: storage of both operands (A = dY, B = X); the slabs are fp32
int gemm_skinny_try(const GemmParams& p, int amode, int bmode, int pro_a, int pro_b, float* ws,
                    size_t ws_elems, int dt, hipStream_t stream) {
  static int off = -1;
  if (off < 0) {
    const char* e = getenv("ACCUNET_NO_SKINNY");  // A/B knob
    off = (e && atoi(e)) ? 1 : 0;
  }
  const bool sh3 = bmode == BM_NN_SHIFT3;
  if (off || amode != AM_COL || (bmode != BM_NN && !sh3) || pro_a != PRO_NONE || p.nsrc != 1)
    return 0;
  if (sh3 && pro_b != PRO_NONE) return 0;
  if (p.bias || p.nup || p.stats || p.pd2 || p.bz || !ws) return 0;
  if (p.K < 16384) return 0;
  const int TI = (p.M + 31) / 32, TJ = (p.N + 31) / 32;  // edge tiles masked
  // measured (tools/gemm_census.py): a clear win while the stream dominates (up to 3
  // output tiles: 32x32 2.1x, 32x96 / 96x32 faster); from 4 tiles the MFMA work per
  // K pair makes the tiled kernel equal or better (64x64 at K 262144: 40 vs 36 us;
  // the 32 x 288 3x3 weight gradient as 1 x 9 tiles: 539 vs 361 us)
  if (TI * TJ > 3) return 0;
  skinny_kfn fn = dt == ACC_BF16 ? skinny_fn<bf16_t>(sh3, pro_b, TI, TJ)
                                 : skinny_fn<float>(sh3, pro_b, TI, TJ);
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
  s.H = p.H; s.W = p.W; s.cin = p.cin;
  s.fW = p.fW; s.fH = p.fH;
  hipLaunchKernelGGL(fn, dim3((unsigned)nb), dim3(256), 0, stream, s);
  return (int)nb;
}
