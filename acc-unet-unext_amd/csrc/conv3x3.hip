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
// Here a workgroup owns a column strip of 128 pixels (W % 128 == 0) of one image and a
// run of its output rows, walked top to bottom, for 32 output channels:
//   * a ring of 3 input rows (130 pixels x 32 channels each, padded slots) sits in LDS;
//     each output row needs one new input row, which streams in (LDS-DMA) into the
//     slot of the row just finished while the last row's taps and the epilogue run, so
//     an input pixel goes to LDS ~1.02 times instead of the implicit GEMM's 9;
//     out-of-image pixels are zero-filled at staging, so the main loop has no masks;
//   * the 36 KB weight block stays in registers for the workgroup's life (9 taps x 8
//     channel quads: 36 float4 per lane); two workgroups are resident per CU;
//   * v_mfma_f32_32x32x2_f32, 4 waves x 32 pixels: a lane reads 4 consecutive channels
//     of its pixel (one ds_read_b128, padded 36-float slots) and feeds 4 MFMAs, pairing
//     channel 8g + t with 8g + 4 + t, the same pairing for the weights (the engine's k
//     order: within the parity tolerances of the implicit GEMM);
//   * the accumulator tile is the engine's 128x32 (WM 4, TM 1, TN 1) layout, so the
//     shared epilogue (bias, fp64 statistics rows per 128-pixel tile, in-place addend)
//     runs unchanged: statistics rows and results are indexed exactly as the engine's.
#include "gemm_dispatch.h"

#include <atomic>

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
__global__ void __launch_bounds__(256, 2) conv3x3_c32_kernel(const GemmParams p, int rows_per) {
  __shared__ __attribute__((aligned(16))) float hal[C3_HALO_F];
  __shared__ __attribute__((aligned(16))) float epi[gemm_epi_floats<4, 1, 1>()];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l31 = lane & 31, lh = lane >> 5;
  const int n0 = blockIdx.y * 32;
  const int H = p.H, W = p.W;
  const float* X = (const float*)p.A[0];
  const long ldx = p.lda[0];

  // this workgroup's strip: 128 columns [w0, w0 + 128) of image b, output rows
  // [hb, he), walked top to bottom
  const int cps = (H + rows_per - 1) / rows_per;  // row chunks per column strip
  const int strip = blockIdx.x / cps, chunk = blockIdx.x - strip * cps;
  const int nstrip_w = W / C3_BM;
  const int b = strip / nstrip_w;
  const int w0 = (strip - b * nstrip_w) * C3_BM;
  const int hb = chunk * rows_per, he = min(H, hb + rows_per);
  if (hb >= he) return;

  // input row r (-1 .. H) of the strip -> ring slot r mod 3 by LDS-DMA
  // (global_load_lds_dwordx4, lane-linear 16-B pieces): piece e = (j, k), slot pixel j
  // holds input pixel (r, w0 - 1 + j), k < 8 its channel quads, k = 8 the padding; the
  // zero page outside the image and for the padding. Every wave issues exactly
  // C3_DMA_ROW instructions per row (the counted waits below rely on it).
  auto dma_row = [&](int r) {
    const bool rok = r >= 0 && r < H;
    const float* xrow = X + ((long)b * H + r) * W * ldx;
    float* dst = hal + ((r + 3) % 3) * C3_ROW_PIECES * 4;
#pragma unroll 1
    for (int u = 0; u < C3_DMA_ROW; ++u) {
      const int base = (u * 4 + wave) * C3_DMA_LANES;
      const int e = base + lane;
      const int j = e / 9, k = e - j * 9;
      const int ww = w0 - 1 + j;
      const bool ok = rok && k < 8 && ww >= 0 && ww < W;
      const float* src = ok ? xrow + (long)ww * ldx + 4 * k : g_c3_zero4;
      if (lane < C3_DMA_LANES && e < C3_ROW_PIECES) gg_dma16(src, dst + base * 4);
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

  auto taps = [&](floatx16& acc, int dh, int r) {  // the 3 taps of input row r
    const float* a = hal + ((r + 3) % 3) * C3_ROW_PIECES * 4 + px * C3_CS + 4 * lh;
#pragma unroll
    for (int dw = 0; dw < 3; ++dw) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const float4 f = *reinterpret_cast<const float4*>(a + dw * C3_CS + 8 * g);
        const float4 w = wr[dh * 3 + dw][g];
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(f.x, w.x, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(f.y, w.y, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(f.z, w.z, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(f.w, w.w, acc, 0, 0, 0);
      }
    }
  };

  dma_row(hb - 1);
  dma_row(hb);
  dma_row(hb + 1);
  for (int h = hb; h < he; ++h) {
    // Rows h-1 .. h+1 are needed. Past the first row, rows h-1 and h are in place and
    // row h+1 (issued during the previous row's taps) is waited for explicitly after
    // taps(0, h-1) below; at the first row: rows hb-1 and hb have landed (hb+1 may
    // still be in flight) in every wave.
    if (h == hb) {
      gg_wait_vm<C3_DMA_ROW>();
      __builtin_amdgcn_s_barrier();
    }
    floatx16 acc[1][1];
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[0][0][r] = 0.f;
    taps(acc[0][0], 0, h - 1);
    // past the first row, row h+1 (issued during the previous row) must have landed in
    // every wave before taps(2, h+1): an explicit wait here, not the epilogue's drain
    if (h > hb) gg_wait_vm<0>();
    // every wave is done with row h-1's slot: row h+2 streams into it during the taps
    // of rows h, h+1 and the epilogue
    __builtin_amdgcn_s_barrier();
    const bool more = h + 1 < he;
    if (more) dma_row(h + 2);
    taps(acc[0][0], 1, h);
    if (h == hb) {  // row hb+1 (the prologue's third row) visible
      if (more) gg_wait_vm<C3_DMA_ROW>();
      else gg_wait_vm<0>();
      __builtin_amdgcn_s_barrier();
    }
    taps(acc[0][0], 2, h + 1);
    gemm_epilogue<float, EPI, 4, 1, 1>(p, acc, epi, (int)(((long)b * H + h) * W + w0), n0);
  }
}

// ---------------------------------------------------------------------------
// bf16 activation mode (BASELINE configs[2]): the same strips and ring on
// v_mfma_f32_32x32x16_bf16. Slots hold 32 bf16 channels padded to 40 (80 B, as the
// bf16 engine's LDS rows); a lane's A operand is one ds_read_b128 of 8 channels
// (k = 16 g + 8 lh + j), its B operand 8 weights rounded to bf16 once (fp32 master
// weights, round-to-nearest-even as the engine rounds them on load). Per tap the two
// k-steps run in channel order and the taps in order 0..8: the bf16 engine's k order
// (its 32-k stage is one tap), so the sums, and with the shared epilogue the stored
// bf16 values, are the engine's.
// ---------------------------------------------------------------------------
#define C3B_CS 40                                   // bf16 per slot (32 + 8 pad)
#define C3B_ROW_PIECES (C3_SLOTS * (C3B_CS / 8))    // 16-B pieces per ring row (650)
#define C3B_DMA_ROW 3                               // DMA instructions per wave and row
#define C3B_DMA_LANES ((C3B_ROW_PIECES + 4 * C3B_DMA_ROW - 1) / (4 * C3B_DMA_ROW))  // 55
static_assert(C3B_DMA_LANES <= 64 && (4 * C3B_DMA_ROW - 1) * C3B_DMA_LANES < C3B_ROW_PIECES,
              "every DMA instruction has live lanes");

template <int EPI>
__global__ void __launch_bounds__(256, 2) conv3x3_c32_bf16_kernel(const GemmParams p, int rows_per) {
  __shared__ __attribute__((aligned(16))) bf16_t hal[3 * C3_SLOTS * C3B_CS];
  __shared__ __attribute__((aligned(16))) float epi[gemm_epi_floats<4, 1, 1>()];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l31 = lane & 31, lh = lane >> 5;
  const int n0 = blockIdx.y * 32;
  const int H = p.H, W = p.W;
  const bf16_t* X = (const bf16_t*)p.A[0];
  const long ldx = p.lda[0];

  const int cps = (H + rows_per - 1) / rows_per;
  const int strip = blockIdx.x / cps, chunk = blockIdx.x - strip * cps;
  const int nstrip_w = W / C3_BM;
  const int b = strip / nstrip_w;
  const int w0 = (strip - b * nstrip_w) * C3_BM;
  const int hb = chunk * rows_per, he = min(H, hb + rows_per);
  if (hb >= he) return;

  auto dma_row = [&](int r) {  // input row r -> ring slot r mod 3 (pieces: 4 data + 1 pad)
    const bool rok = r >= 0 && r < H;
    const bf16_t* xrow = X + ((long)b * H + r) * W * ldx;
    float* dst = reinterpret_cast<float*>(hal + ((r + 3) % 3) * C3_SLOTS * C3B_CS);
#pragma unroll 1
    for (int u = 0; u < C3B_DMA_ROW; ++u) {
      const int base = (u * 4 + wave) * C3B_DMA_LANES;
      const int e = base + lane;
      const int j = e / 5, k = e - j * 5;
      const int ww = w0 - 1 + j;
      const bool ok = rok && k < 4 && ww >= 0 && ww < W;
      const float* src = ok ? reinterpret_cast<const float*>(xrow + (long)ww * ldx + 8 * k) : g_c3_zero4;
      if (lane < C3B_DMA_LANES && e < C3B_ROW_PIECES) gg_dma16(src, dst + base * 4);
    }
  };

  // weights of output channel n0 + l31 rounded to bf16: wb[tap][g] = k 16g + 8lh .. +7
  bf16x8_v wb[9][2];
  {
    const float* wrow = (const float*)p.B + (long)(n0 + l31) * p.ldb + 8 * lh;
#pragma unroll
    for (int tap = 0; tap < 9; ++tap)
#pragma unroll
      for (int g = 0; g < 2; ++g) {
        const uint4 u = ld8_bf(wrow + tap * C3_CIN + 16 * g);
        wb[tap][g] = __builtin_bit_cast(bf16x8_v, u);
      }
  }
  const int px = wave * 32 + l31;

  auto taps = [&](floatx16& acc, int dh, int r) {
    const bf16_t* a = hal + ((r + 3) % 3) * C3_SLOTS * C3B_CS + px * C3B_CS + 8 * lh;
#pragma unroll
    for (int dw = 0; dw < 3; ++dw)
#pragma unroll
      for (int g = 0; g < 2; ++g) {
        const bf16x8_v f = *reinterpret_cast<const bf16x8_v*>(a + dw * C3B_CS + 16 * g);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f, wb[dh * 3 + dw][g], acc, 0, 0, 0);
      }
  };

  dma_row(hb - 1);
  dma_row(hb);
  dma_row(hb + 1);
  for (int h = hb; h < he; ++h) {  // the same schedule as the fp32 kernel
    if (h == hb) {
      gg_wait_vm<C3B_DMA_ROW>();
      __builtin_amdgcn_s_barrier();
    }
    floatx16 acc[1][1];
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[0][0][r] = 0.f;
    taps(acc[0][0], 0, h - 1);
    if (h > hb) gg_wait_vm<0>();  // row h+1 landed in every wave (as the fp32 kernel)
    __builtin_amdgcn_s_barrier();
    const bool more = h + 1 < he;
    if (more) dma_row(h + 2);
    taps(acc[0][0], 1, h);
    if (h == hb) {
      if (more) gg_wait_vm<C3B_DMA_ROW>();
      else gg_wait_vm<0>();
      __builtin_amdgcn_s_barrier();
    }
    taps(acc[0][0], 2, h + 1);
    gemm_epilogue<bf16_t, EPI, 4, 1, 1>(p, acc, epi, (int)(((long)b * H + h) * W + w0), n0);
  }
}

// host-side launch counts (accunet_conv3x3_halo_launches): [0] forward / data gradient,
// [1] weight gradient
static std::atomic<long long> g_c3_launches[2];

extern "C" long long accunet_conv3x3_halo_launches(int wgrad) {
  return g_c3_launches[wgrad ? 1 : 0].load();
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
                    int dmode, int tile, hipStream_t stream) {
  // (tile: the engine's choice; the statistics rows are per 128x32 tile, so only where
  // the engine would run 128x32 tiles too. dmode: 1 fp32, 2 bf16 activations with fp32
  // weights, 0 neither)
  if (!conv3x3_c32_on() || !dmode || tile != TILE_C || amode != AM_SHIFT3 || bmode != BM_NT || pro_a != PRO_NONE ||
      pro_b != PRO_NONE || (epi != 0 && epi != EPI_STATS && epi != EPI_UPS))
    return -1;
  if (p.cin != C3_CIN || p.K != 9 * C3_CIN || p.nsrc != 1 || p.N % 32 || p.W % C3_BM ||
      p.M % C3_BM || (long)p.M != (long)(p.M / ((long)p.H * p.W)) * p.H * p.W)
    return -1;
  if ((p.lda[0] & (dmode == 2 ? 7 : 3)) || ((uintptr_t)p.A[0] & 15) || (p.ldb & 3) ||
      ((uintptr_t)p.B & 15))
    return -1;
  // persistent workgroups, two resident per CU (74.6 KB of LDS each): column strips of
  // 128 pixels cut into row chunks so that there are ~512 per column block
  const long B = p.M / ((long)p.H * p.W);
  const long strips = B * (p.W / C3_BM);
  const int nb = p.N / 32;
  const long want = 512 / nb > 8 ? 512 / nb : 8;
  int rows_per = (int)((strips * p.H + want - 1) / want);
  if (rows_per < 1) rows_per = 1;
  const long cps = (p.H + rows_per - 1) / rows_per;
  dim3 grid((unsigned)(strips * cps), nb);
  if (dmode == 2) {
    if (epi & EPI_UPS)
      hipLaunchKernelGGL(conv3x3_c32_bf16_kernel<EPI_UPS>, grid, dim3(256), 0, stream, p, rows_per);
    else
      hipLaunchKernelGGL(conv3x3_c32_bf16_kernel<EPI_STATS>, grid, dim3(256), 0, stream, p, rows_per);
  } else if (epi & EPI_UPS) {
    hipLaunchKernelGGL(conv3x3_c32_kernel<EPI_UPS>, grid, dim3(256), 0, stream, p, rows_per);
  } else {
    hipLaunchKernelGGL(conv3x3_c32_kernel<EPI_STATS>, grid, dim3(256), 0, stream, p, rows_per);
  }
  g_c3_launches[0]++;
  return hipGetLastError() == hipSuccess ? ACC_OK : ACC_ELAUNCH;
}

// ---------------------------------------------------------------------------
// The weight gradient of the same convolution,
//   dW[co][tap*32 + ci] = sum_p dY[p][co] * X[shift_tap(p)][ci]      (M 32, N 288, K pixels)
// (AM_COL x BM_NN_SHIFT3 in the engine: 0.31 of fp32 MFMA, its 32x128 tiles waste a
// quarter of the 384 columns and re-gather X per tap). Same strips and 3-row X ring as
// above; per output row a wave takes 32 pixels in pairs (the MFMA k): its dY values
// (one per lane, lane (co, k)) are loaded once into 16 registers and serve all 9 taps,
// whose X operand is one ds_read_b32 from the ring (lane (k, ci)). The 9 accumulator
// tiles (144 registers) sum the workgroup's pixels; at the end the 4 waves are added in
// wave order through LDS and the workgroup writes one [32][288] slab, which the split-K
// reduction (gemm_run.hip) sums in slab order: deterministic.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256, 2)
conv3x3_c32_wgrad_kernel(const GemmParams p, int rows_per, float* __restrict__ slabs) {
  // channel block of this workgroup (blockIdx.y): output channels [co0, co0 + 32) of
  // M = C_out, input channels [ci0, ci0 + 32) of cin (32-channel slices of wider layers,
  // each block its own [32][9][32] part of the [M][9*cin] slab)
  const int nci = p.cin / C3_CIN;
  const int co0 = (blockIdx.y / nci) * 32, ci0 = (blockIdx.y % nci) * C3_CIN;
  __shared__ __attribute__((aligned(16))) float hal[C3_HALO_F];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l31 = lane & 31, lh = lane >> 5;
  const int H = p.H, W = p.W;
  const float* X = (const float*)p.B;
  const long ldx = p.ldb;
  const float* dY = (const float*)p.A[0];
  const long ldy = p.lda[0];

  const int cps = (H + rows_per - 1) / rows_per;
  const int strip = blockIdx.x / cps, chunk = blockIdx.x - strip * cps;
  const int nstrip_w = W / C3_BM;
  const int b = strip / nstrip_w;
  const int w0 = (strip - b * nstrip_w) * C3_BM;
  const int hb = chunk * rows_per, he = min(H, hb + rows_per);

  auto dma_row = [&](int r) {  // as in the forward kernel
    const bool rok = r >= 0 && r < H;
    const float* xrow = X + ((long)b * H + r) * W * ldx;
    float* dst = hal + ((r + 3) % 3) * C3_ROW_PIECES * 4;
#pragma unroll 1
    for (int u = 0; u < C3_DMA_ROW; ++u) {
      const int base = (u * 4 + wave) * C3_DMA_LANES;
      const int e = base + lane;
      const int j = e / 9, k = e - j * 9;
      const int ww = w0 - 1 + j;
      const bool ok = rok && k < 8 && ww >= 0 && ww < W;
      const float* src = ok ? xrow + (long)ww * ldx + ci0 + 4 * k : g_c3_zero4;
      if (lane < C3_DMA_LANES && e < C3_ROW_PIECES) gg_dma16(src, dst + base * 4);
    }
  };
  // dY of output row h for this wave's pixel pairs: a[i] = dY[pixel w0 + 32 wave + 2i + lh][l31]
  auto load_dy = [&](int h, float (&a)[16]) {
    const float* row = dY + (((long)b * H + h) * W + w0 + wave * 32 + lh) * ldy + co0 + l31;
#pragma unroll
    for (int i = 0; i < 16; ++i) a[i] = row[(long)(2 * i) * ldy];
  };

  floatx16 acc[9];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;

  // this lane's X operand: ring slot pixel 32 wave + 2i + lh + dw, channel l31
  auto taps_row = [&](const float (&a)[16], int dh, int r) {
    const float* xr = hal + ((r + 3) % 3) * C3_ROW_PIECES * 4 + (wave * 32 + lh) * C3_CS + l31;
#pragma unroll
    for (int i = 0; i < 16; ++i)
#pragma unroll
      for (int dw = 0; dw < 3; ++dw)
        acc[dh * 3 + dw] = __builtin_amdgcn_mfma_f32_32x32x2f32(
            a[i], xr[(2 * i + dw) * C3_CS], acc[dh * 3 + dw], 0, 0, 0);
  };

  if (hb < he) {
    float a[16], an[16];
    dma_row(hb - 1);
    dma_row(hb);
    dma_row(hb + 1);
    load_dy(hb, a);
    gg_wait_vm<0>();  // the first three rows and the first dY row have landed ...
    __builtin_amdgcn_s_barrier();  // ... in every wave
    for (int h = hb; h < he; ++h) {
      taps_row(a, 0, h - 1);
      // row h+1 (issued during the previous row) has landed in this wave, and after the
      // barrier in every wave, which is also done with row h-1's slot
      gg_wait_vm<0>();
      __builtin_amdgcn_s_barrier();
      const bool more = h + 1 < he;
      if (more) {
        dma_row(h + 2);  // streams in during the taps of rows h, h+1 and the next h-1
        load_dy(h + 1, an);
      }
      taps_row(a, 1, h);
      taps_row(a, 2, h + 1);
      if (more) {
#pragma unroll
        for (int i = 0; i < 16; ++i) a[i] = an[i];
      }
    }
  }
  // the 4 waves' partial tiles summed in wave order, 3 taps per round through the ring
  __syncthreads();
  const int N = 9 * p.cin;
  float* slab = slabs + (size_t)blockIdx.x * p.M * N + (size_t)co0 * N + ci0;
#pragma unroll
  for (int t0 = 0; t0 < 9; t0 += 3) {
#pragma unroll
    for (int t = 0; t < 3; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r)
        hal[((wave * 3 + t) * 32 + ((r & 3) + 8 * (r >> 2) + 4 * lh)) * 32 + l31] = acc[t0 + t][r];
    __syncthreads();
    for (int e = tid; e < 3 * 1024; e += 256) {
      const int t = e >> 10, co = (e >> 5) & 31, ci = e & 31;
      const float s = ((hal[((0 * 3 + t) * 32 + co) * 32 + ci] + hal[((1 * 3 + t) * 32 + co) * 32 + ci]) +
                       hal[((2 * 3 + t) * 32 + co) * 32 + ci]) + hal[((3 * 3 + t) * 32 + co) * 32 + ci];
      slab[(size_t)co * N + (t0 + t) * p.cin + ci] = s;
    }
    __syncthreads();
  }
}

// The weight-gradient launch (AM_COL dY x BM_NN_SHIFT3 X, M = C_out and cin multiples
// of 32, N = 9 cin, image rows of whole 128-pixel strips, no epilogue features): slabs in ws, then the split-K reduction; returns the slab count, or 0 when
// the shape is not this kernel's (the caller runs the GEMM engine).
int conv3x3_c32_wgrad_try(const GemmParams& p, int amode, int bmode, int pro_a, int pro_b,
                          bool fp32, float* ws, size_t ws_elems, hipStream_t stream) {
  if (!conv3x3_c32_on() || !fp32 || amode != AM_COL || bmode != BM_NN_SHIFT3 ||
      pro_a != PRO_NONE || pro_b != PRO_NONE || !ws)
    return 0;
  if (p.cin % C3_CIN || p.M % 32 || p.N != 9 * p.cin || p.nsrc != 1 || p.W % C3_BM ||
      (p.lda[0] & 3) || (p.ldb & 3) ||
      p.bias || p.nup || p.stats || p.pd2 || p.bz ||
      (long)p.K != (long)(p.K / ((long)p.H * p.W)) * p.H * p.W)
    return 0;
  const long B = p.K / ((long)p.H * p.W);
  const long strips = B * (p.W / C3_BM);
  const int nblk = (p.M / 32) * (p.cin / C3_CIN);  // 32x32 channel blocks
  const long want = 512 / nblk > 8 ? 512 / nblk : 8;  // workgroups per block
  int rows_per = (int)((strips * p.H + want - 1) / want);
  if (rows_per < 1) rows_per = 1;
  const long cps = (p.H + rows_per - 1) / rows_per;
  const long nb = strips * cps;  // slabs
  if ((size_t)nb * p.M * p.N > ws_elems) return 0;
  hipLaunchKernelGGL(conv3x3_c32_wgrad_kernel, dim3((unsigned)nb, nblk), dim3(256), 0, stream, p,
                     rows_per, ws);
  g_c3_launches[1]++;
  return (int)nb;
}
