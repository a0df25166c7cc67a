// ResPath 3x3 convolution over 32 channels as a halo-tile direct convolution: the
// first-level ResPath (ACC_UNet/ACC_UNet.py:316-318, 32 -> 32 channels at the full
// image size) forward, and its data gradient (the same convolution of dY with the
// flipped, transposed weights, csrc/pool.hip relayout "c3f"). Both are
//   C[m][n] = sum_{tap, ci} X[shift_tap(m)][ci] * Wt[n][tap*32 + ci]  (+ epilogue)
// which the GEMM engine runs as an implicit GEMM (AM_SHIFT3 x BM_NT): there every
// 128-pixel tile stages its A operand tap by tap, i.e. each input pixel goes L2 -> LDS
// nine times, and the 128x32 tile does 8 MFMAs per 16-k stage (0.40 of fp32 MFMA at
// 1048576x32x288, profiles/r04_*).
//
// Here a workgroup owns 128 consecutive output pixels of one image row (W % 128 == 0)
// and all 32 output channels of its column block:
//   * the halo (3 input rows x 130 pixels x 32 channels) is staged once per tile: each
//     input pixel goes to LDS ~3.05 times instead of 9; out-of-image slots are zeroed at
//     staging, so the main loop has no masks;
//   * the 36 KB weight block is read into registers per tile (9 taps x 8 channel
//     quads: 36 float4 per lane, L2-resident), alongside the halo, which goes global ->
//     LDS by LDS-DMA (no staging registers); workgroups are persistent over a
//     contiguous run of tiles (neighbouring halos share input rows in L2) and the second
//     resident workgroup of the CU computes while one stages;
//   * v_mfma_f32_32x32x2_f32, 4 waves x 32 pixels: a lane reads 4 consecutive channels
//     of its pixel (one ds_read_b128, padded 36-float slots) and feeds 4 MFMAs, pairing
//     channel 8g + t with 8g + 4 + t, the same pairing for the weights (the engine's k
//     order: within the parity tolerances of the implicit GEMM);
//   * the accumulator tile is the engine's 128x32 (WM 4, TM 1, TN 1) layout, so the
//     shared epilogue (bias, fp64 statistics rows per 128-pixel tile, in-place addend)
//     runs unchanged: statistics rows and results are indexed exactly as the engine's.
#include "gemm_dispatch.h"

#define C3_CIN 32
#define C3_BM 128
#define C3_SLOTS (C3_BM + 2)
#define C3_CS 36                                   // floats per halo slot (32 + 4 pad)
#define C3_HALO_F (3 * C3_SLOTS * C3_CS)
#define C3_ROW_PIECES (C3_SLOTS * (C3_CS / 4))    // 16-B pieces of one halo row, padding included (1170)
#define C3_DMA_ROW 5                               // DMA instructions per wave and row
#define C3_DMA_LANES ((C3_ROW_PIECES + 4 * C3_DMA_ROW - 1) / (4 * C3_DMA_ROW))  // 59 pieces each
static_assert(C3_DMA_LANES <= 64 && (4 * C3_DMA_ROW - 1) * C3_DMA_LANES < C3_ROW_PIECES,
              "every DMA instruction has live lanes");

static __device__ __attribute__((aligned(16))) float g_c3_zero4[4];

template <int EPI>
__global__ void __launch_bounds__(256, 2) conv3x3_c32_kernel(const GemmParams p, int ntiles) {
  __shared__ __attribute__((aligned(16))) float hal[C3_HALO_F];
  __shared__ __attribute__((aligned(16))) float epi[gemm_epi_floats<4, 1, 1>()];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l31 = lane & 31, lh = lane >> 5;
  const int n0 = blockIdx.y * 32;
  const int H = p.H, W = p.W;
  const float* X = (const float*)p.A[0];
  const long ldx = p.lda[0];

  // this workgroup's contiguous run of 128-pixel tiles
  const int per = (ntiles + gridDim.x - 1) / gridDim.x;
  const int t0 = blockIdx.x * per;
  const int t1 = min(ntiles, t0 + per);
  if (t0 >= t1) return;

  // halo of tile mt -> LDS by LDS-DMA (global_load_lds_dwordx4, lane-linear 16-B
  // pieces): piece e = (slot, k), slot = dh*130 + j holds input pixel
  // (h + dh - 1, w0 - 1 + j) of the tile's image row, k < 8 its channel quads, k = 8 the
  // slot's padding; the zero page outside the image and for the padding
  auto dma = [&](int mt) {
    const int m0 = mt * C3_BM;
    const uint32_t q = fdiv((uint32_t)m0, p.fW);  // image row index b*H + h
    const int w0 = m0 - (int)q * W;
    const int h = (int)(q - fdiv(q, p.fH) * H);
#pragma unroll
    for (int dh = 0; dh < 3; ++dh) {  // input row by input row (waited for in that order)
      const int hh = h + dh - 1;
      const bool rok = hh >= 0 && hh < H;
      const float* xrow = X + (long)((int)q + dh - 1) * W * ldx;
#pragma unroll 1
      for (int u = 0; u < C3_DMA_ROW; ++u) {
        // C3_DMA_LANES pieces per instruction so that every wave issues exactly
        // C3_DMA_ROW instructions per row (the counted waits below assume it)
        const int base = (u * 4 + wave) * C3_DMA_LANES;
        const int e = base + lane;
        const int j = e / 9, k = e - j * 9;
        const int ww = w0 - 1 + j;
        const bool ok = rok && k < 8 && ww >= 0 && ww < W;
        const float* src = ok ? xrow + (long)ww * ldx + 4 * k : g_c3_zero4;
        if (lane < C3_DMA_LANES && e < C3_ROW_PIECES)
          gg_dma16(src, hal + (dh * C3_ROW_PIECES + base) * 4);
      }
    }
  };

  // weights of output channel n0 + l31: wr[tap][g] = Wt[n][tap*32 + 8g + 4lh .. +3],
  // read once (the workgroup is persistent)
  float4 wr[9][4];
  {
    const float* wrow = (const float*)p.B + (long)(n0 + l31) * p.ldb + 4 * lh;
#pragma unroll
    for (int tap = 0; tap < 9; ++tap)
#pragma unroll
      for (int g = 0; g < 4; ++g)
        wr[tap][g] = *reinterpret_cast<const float4*>(wrow + tap * C3_CIN + 8 * g);
  }
  const int px = wave * 32 + l31;  // this lane's output pixel in the tile (A row)
  for (int mt = t0; mt < t1; ++mt) {
    __syncthreads();  // every read of the previous halo is done
    dma(mt);
    floatx16 acc[1][1];
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[0][0][r] = 0.f;
#pragma unroll
    for (int dh = 0; dh < 3; ++dh) {
      // input row dh of this wave has landed (the later rows' 5 instructions each may
      // still be in flight), and every wave's once all pass the barrier: the taps of row
      // dh run while rows dh+1.. stream in
      if (dh == 0) gg_wait_vm<2 * C3_DMA_ROW>();
      else if (dh == 1) gg_wait_vm<C3_DMA_ROW>();
      else gg_wait_vm<0>();
      __builtin_amdgcn_s_barrier();
#pragma unroll
      for (int dw = 0; dw < 3; ++dw) {
        const int tap = dh * 3 + dw;
        const float* a = hal + (dh * C3_SLOTS + px + dw) * C3_CS + 4 * lh;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const float4 f = *reinterpret_cast<const float4*>(a + 8 * g);
          const float4 b = wr[tap][g];
          acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(f.x, b.x, acc[0][0], 0, 0, 0);
          acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(f.y, b.y, acc[0][0], 0, 0, 0);
          acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(f.z, b.z, acc[0][0], 0, 0, 0);
          acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(f.w, b.w, acc[0][0], 0, 0, 0);
        }
      }
    }
    gemm_epilogue<float, EPI, 4, 1, 1>(p, acc, epi, mt * C3_BM, n0);
  }
}

static int conv3x3_c32_on() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("ACCUNET_CONV3_HALO");  // A/B knob: 0 = the implicit GEMM
    v = e ? atoi(e) : 1;
  }
  return v;
}

// Runs the halo kernel when the launch is one it covers (fp32, 32 input channels, 3x3
// with the weights [N][9*32], image rows of whole 128-pixel tiles, no split, an epilogue
// of bias / statistics / in-place addend) and returns ACC_OK, else -1 (caller runs the
// GEMM engine). p.evec must already be set (gemm_run).
int conv3x3_c32_try(const GemmParams& p, int amode, int bmode, int pro_a, int pro_b, int epi,
                    bool fp32, int tile, hipStream_t stream) {
  // (tile: the engine's choice; the statistics rows are per 128x32 tile, so only where
  // the engine would run 128x32 tiles too)
  if (!conv3x3_c32_on() || !fp32 || tile != TILE_C || amode != AM_SHIFT3 || bmode != BM_NT || pro_a != PRO_NONE ||
      pro_b != PRO_NONE || (epi != 0 && epi != EPI_STATS && epi != EPI_UPS))
    return -1;
  if (p.cin != C3_CIN || p.K != 9 * C3_CIN || p.nsrc != 1 || p.N % 32 || p.W % C3_BM ||
      p.M % C3_BM || (long)p.M != (long)(p.M / ((long)p.H * p.W)) * p.H * p.W)
    return -1;
  if ((p.lda[0] & 3) || ((uintptr_t)p.A[0] & 15) || (p.ldb & 3) || ((uintptr_t)p.B & 15))
    return -1;
  const int ntiles = p.M / C3_BM;
  // two resident workgroups per CU (74.6 KB of LDS each), persistent over their tiles
  int nwg = 512 / (p.N / 32);
  if (nwg < 8) nwg = 8;
  if (nwg > ntiles) nwg = ntiles;
  dim3 grid(nwg, p.N / 32);
  if (epi & EPI_UPS)
    hipLaunchKernelGGL(conv3x3_c32_kernel<EPI_UPS>, grid, dim3(256), 0, stream, p, ntiles);
  else
    hipLaunchKernelGGL(conv3x3_c32_kernel<EPI_STATS>, grid, dim3(256), 0, stream, p, ntiles);
  return hipGetLastError() == hipSuccess ? ACC_OK : ACC_ELAUNCH;
}
