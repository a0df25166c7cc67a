// Host driver for the MFMA GEMM engines (fp32: gemm_f32.h, bf16: gemm_bf16.h): engine
// and tile choice, split-K, deterministic split-K reduction (fixed slab order, no
// float atomics).
#include "gemm_dispatch.h"
#include <string.h>
#include <stdlib.h>

// One block = 64 consecutive outputs x 16 slab groups (1024 threads): thread (c, g)
// sums slabs g, g+16, ... in order, then the 16 group sums are added in fixed order ->
// deterministic, and S-way parallel enough that a 32x32 weight gradient split 1024
// ways does not serialise on one thread per output. (16 outputs x 64 groups for deep
// splits measured 1.7x slower: 64-B row segments instead of 256-B ones.)
#define SPLITK_COLS 64
#define SPLITK_GROUPS 16
__global__ void __launch_bounds__(1024)
splitk_reduce_kernel(const float* __restrict__ ws, float* __restrict__ C, int M, int N, int ldc,
                     int S, size_t zstride) {
  __shared__ float part[SPLITK_GROUPS][SPLITK_COLS];
  const int c = threadIdx.x & (SPLITK_COLS - 1), g = threadIdx.x / SPLITK_COLS;
  const long total = (long)M * N;
  const long i = (long)blockIdx.x * SPLITK_COLS + c;
  float acc = 0.f;
  if (i < total) {
    const float* src = ws + i;
    int z = g;
    for (; z + 3 * SPLITK_GROUPS < S; z += 4 * SPLITK_GROUPS) {
      float a0 = src[(size_t)z * zstride];
      float a1 = src[(size_t)(z + SPLITK_GROUPS) * zstride];
      float a2 = src[(size_t)(z + 2 * SPLITK_GROUPS) * zstride];
      float a3 = src[(size_t)(z + 3 * SPLITK_GROUPS) * zstride];
      acc += a0;
      acc += a1;
      acc += a2;
      acc += a3;
    }
    for (; z < S; z += SPLITK_GROUPS) acc += src[(size_t)z * zstride];
  }
  part[g][c] = acc;
  __syncthreads();
  if (g == 0 && i < total) {
    float s = part[0][c];
#pragma unroll
    for (int k = 1; k < SPLITK_GROUPS; ++k) s += part[k][c];
    int m = (int)(i / N), n = (int)(i - (long)m * N);
    C[(size_t)m * ldc + n] = s;
  }
}

// Quad form (N % 4 == 0): a 256-thread block = (256 / G) output quads x G slab groups;
// thread (quad, g) sums slabs g, g + G, ... as float4 (8 loads in flight), then the G
// group sums are added in group order (deterministic). G grows with S so that deep
// splits of small outputs still spread over many lanes.
template <int G>
__global__ void __launch_bounds__(256)
splitk_reduce4_kernel(const float* __restrict__ ws, float* __restrict__ C, int M, int N, int ldc,
                      int S, size_t zstride) {
  constexpr int QC = 256 / G;
  __shared__ float4 part[G][QC];
  const int qc = threadIdx.x % QC, g = threadIdx.x / QC;
  const long nq = (long)M * N / 4;
  const long i = (long)blockIdx.x * QC + qc;  // output quad
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  if (i < nq) {
    const float4* src = reinterpret_cast<const float4*>(ws) + i;
    const size_t zs = zstride / 4;
    int z = g;
    for (; z + 7 * G < S; z += 8 * G) {
      float4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = src[(size_t)(z + u * G) * zs];
#pragma unroll
      for (int u = 0; u < 8; ++u) { acc.x += v[u].x; acc.y += v[u].y; acc.z += v[u].z; acc.w += v[u].w; }
    }
    for (; z < S; z += G) {
      const float4 v = src[(size_t)z * zs];
      acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
  }
  if (G > 1) {
    part[g][qc] = acc;
    __syncthreads();
    if (g != 0) return;
    acc = part[0][qc];
#pragma unroll
    for (int k = 1; k < G; ++k) {
      const float4 v = part[k][qc];
      acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
  }
  if (i >= nq) return;
  const long e = 4 * i;
  const int m = (int)(e / N), n = (int)(e - (long)m * N);
  float* dst = C + (size_t)m * ldc + n;
  if ((ldc & 3) == 0 && ((uintptr_t)C & 15) == 0) {
    *reinterpret_cast<float4*>(dst) = acc;
  } else {
    dst[0] = acc.x; dst[1] = acc.y; dst[2] = acc.z; dst[3] = acc.w;
  }
}

static int splitk_v4_on() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("ACCUNET_SPLITK_V4");  // A/B knob: 0 = the scalar reduce only
    v = e ? atoi(e) : 1;
  }
  return v;
}

static void splitk_reduce(const float* ws, float* C, int M, int N, int ldc, int S, size_t zstride,
                          hipStream_t stream) {
  const long total = (long)M * N;
  if (splitk_v4_on() && (N & 3) == 0 && (zstride & 3) == 0 && ((uintptr_t)ws & 15) == 0) {
    const long nq = total / 4;
    auto go = [&](auto kfn, int G) {
      const int QC = 256 / G;
      hipLaunchKernelGGL(kfn, dim3((unsigned)((nq + QC - 1) / QC)), dim3(256), 0, stream, ws, C, M,
                         N, ldc, S, zstride);
    };
    // slab groups: enough lanes for the deep splits of small outputs
    if (S >= 64 && nq < 65536) go(splitk_reduce4_kernel<16>, 16);
    else if (S >= 16) go(splitk_reduce4_kernel<4>, 4);
    else go(splitk_reduce4_kernel<1>, 1);
    return;
  }
  hipLaunchKernelGGL(splitk_reduce_kernel, dim3((unsigned)((total + SPLITK_COLS - 1) / SPLITK_COLS)),
                     dim3(SPLITK_COLS * SPLITK_GROUPS), 0, stream, ws, C, M, N, ldc, S, zstride);
}

// epi: the EPI_* features this launch needs
#define GEMM_TABLE_SELECT(P)                                                                    \
  if (epi & (EPI_BNB | EPI_PYR)) { /* data-gradient epilogues */                               \
    if (amode != AM_ROW || bmode != BM_NN || pro_a != PRO_NONE || pro_b != PRO_NONE ||          \
        (epi & (EPI_UPS | EPI_STATS)))                                                          \
      return nullptr;                                                                           \
    if (epi == EPI_BNB) return P##row_nn_bnb[0];                                                \
    if (epi == EPI_PYR) return P##row_nn_pyr[0];                                                \
    return P##row_nn_bnb_pyr[0];                                                                \
  }                                                                                             \
  if (amode == AM_ROW && bmode == BM_NT && pro_b == PRO_NONE) {                                 \
    const bool u = (epi & EPI_UPS) != 0;                                                        \
    if (pro_a == PRO_NONE) return u ? P##row_nt_p0_ups[0] : P##row_nt_p0[0];                    \
    if (pro_a == PRO_AFFINE) return u ? P##row_nt_p1_ups[0] : P##row_nt_p1[0];                  \
    if (pro_a == PRO_AFFINE_LRELU) return u ? P##row_nt_p2_ups[0] : P##row_nt_p2[0];            \
  }                                                                                             \
  if (epi == EPI_UPS && amode == AM_ROW && bmode == BM_NN && pro_a == PRO_NONE &&               \
      pro_b == PRO_NONE)                                                                        \
    return P##row_nn_ups[0]; /* data gradient accumulated in place (addend = C) */              \
  if (epi == EPI_UPS && amode == AM_SHIFT3 && bmode == BM_NT && pro_a == PRO_NONE &&            \
      pro_b == PRO_NONE)                                                                        \
    return P##sh3_nt_ups[0]; /* 3x3 data gradient accumulated in place */                      \
  if (epi & EPI_UPS) return nullptr;                                                            \
  if (amode == AM_SHIFT3 && bmode == BM_NT && pro_a == PRO_NONE && pro_b == PRO_NONE)           \
    return P##sh3_nt[0];                                                                        \
  if (epi & EPI_STATS) return nullptr; /* C statistics: forward tables only */                  \
  if (amode == AM_ROW && bmode == BM_NN && pro_a == PRO_NONE && pro_b == PRO_NONE)              \
    return P##row_nn[0];                                                                        \
  if (amode == AM_COL && bmode == BM_NN && pro_a == PRO_NONE) {                                 \
    if (pro_b == PRO_NONE) return P##col_nn_p0[0];                                              \
    if (pro_b == PRO_AFFINE) return P##col_nn_p1[0];                                            \
    if (pro_b == PRO_AFFINE_LRELU) return P##col_nn_p2[0];                                      \
  }                                                                                             \
  if (amode == AM_COL && bmode == BM_NN_SHIFT3 && pro_a == PRO_NONE && pro_b == PRO_NONE)       \
    return P##col_nnsh3[0];                                                                     \
  return nullptr;

// bf16 engine: forward / data-gradient tables take (bf16, fp32 weights) -> bf16, the
// weight-gradient (AM_COL) tables (bf16, bf16) -> fp32
static gemm_kfn* table_for_bf16(int amode, int bmode, int pro_a, int pro_b, int epi, int bdt,
                                int cdt) {
  const bool wgrad = amode == AM_COL;
  if (wgrad ? (bdt != ACC_BF16 || cdt != ACC_F32) : (bdt != ACC_F32 || cdt != ACC_BF16))
    return nullptr;
  GEMM_TABLE_SELECT(g_bgemm_)
}

static gemm_kfn* table_for(int amode, int bmode, int pro_a, int pro_b, int epi) {
  GEMM_TABLE_SELECT(g_gemm_)
}

static gemm_kfn* table_v(int amode, int bmode, int pro_a, int pro_b, int epi, int v, int adt,
                         int bdt, int cdt) {
  // the tables are [2][TILE_COUNT]; table_for returns row 0
  gemm_kfn* t0 = nullptr;
  if (adt == ACC_F32 && bdt == ACC_F32 && cdt == ACC_F32)
    t0 = table_for(amode, bmode, pro_a, pro_b, epi);
  else if (adt == ACC_BF16)
    t0 = table_for_bf16(amode, bmode, pro_a, pro_b, epi, bdt, cdt);
  return t0 ? t0 + v * TILE_COUNT : nullptr;
}

// LDS-DMA fp32 engine (gemm_f32g.h) for vector-aligned fp32 GEMMs (ACCUNET_GEMM_G=0: off)
static gemm_kfn* gtable_for(int amode, int bmode, int pro_a, int pro_b, int epi) {
  GEMM_TABLE_SELECT(g_ggemm_)
}
static gemm_kfn ggemm_for(int amode, int bmode, int pro_a, int pro_b, int epi, int tile) {
  static int on = -1;
  if (on < 0) {
    const char* e = getenv("ACCUNET_GEMM_G");
    on = e ? atoi(e) : 1;
  }
  if (!on) return nullptr;
  gemm_kfn* t = gtable_for(amode, bmode, pro_a, pro_b, epi);
  return t ? t[tile] : nullptr;
}

static long split_min_tiles() {
  static long v = -1;
  if (v < 0) {
    const char* e = getenv("ACCUNET_SPLIT_MIN_TILES");  // tuning knob
    v = e ? atol(e) : 256;
  }
  return v;
}

// workgroups a split-K GEMM aims for (ACCUNET_SPLIT_TARGET, tuning knob): more slabs fill
// the chip for longer K but write and re-read S*M*N fp32 partials
static long split_target() {
  static long v = -1;
  if (v < 0) {
    const char* e = getenv("ACCUNET_SPLIT_TARGET");
    // 768 with the float4 reduce (fp32 step +0.6 % over 1024, bf16 equal:
    // profiles/r03_split_target_ab.txt)
    v = e ? atol(e) : 768;
  }
  return v;
}

// raster groups for wide-B GEMMs (gemm_tile): B bytes per group in KB
// (ACCUNET_GEMM_NGRP_KB, tuning knob; 0 = plain N-fastest order). 1 MB groups cut the
// pyramid data gradient's fetch (65536x4352x128) from 3.23 to 2.46 GB per launch at
// the same time; the whole step is neutral (profiles/r03_gemm_lab.txt)
static long ngrp_kb() {
  static long v = -1;
  if (v < 0) {
    const char* e = getenv("ACCUNET_GEMM_NGRP_KB");
    v = e ? atol(e) : 1024;
  }
  return v;
}

static int smallk_tile() {
  static int v = -2;
  if (v == -2) {
    const char* e = getenv("ACCUNET_SMALLK_TILE");  // tuning knob: -1 = off, else tile id
    v = e ? atoi(e) : TILE_E;
  }
  return v;
}

static int pick_tile(int M, int N, int K, int bmode, int cin, bool can_split) {
  static int force = -2;
  if (force == -2) {
    const char* e = getenv("ACCUNET_GEMM_TILE");  // tuning knob (tools/gbench): force a tile
    force = e ? atoi(e) : -1;
  }
  if (force >= 0 && force < TILE_COUNT) return force;
  int t;
  // short-K GEMMs over many pixels (1x1 data gradients, K = the forward's N <= 64):
  // epilogue-dominated, so smaller tiles (more resident waves to hide its gathers)
  const int sk = smallk_tile();
  // (128x32 tiles for 64 < N <= 96: 1Mx96x32 pyramid dgrad 368 vs 447 us; N = 64 is
  // slower with them: 262144x64x64 +10 us. 128x64 tiles for N > 96: at K = 64, N = 192
  // the forward is 11-14 % faster, the pyramid data gradient 3-8 %, the plain data
  // gradient 5 % than with 64x64, profiles/r04_k64_tile_ab.txt)
  static int wide = -1;
  if (wide < 0) {
    const char* e = getenv("ACCUNET_K64_TILE_B");  // A/B knob: 0 = 64x64 for N > 96 too
    wide = e ? atoi(e) : 1;
  }
  if (sk >= 0 && K <= 64 && M >= 65536 && N > 32)
    return (N > 64 && N <= 96) ? TILE_C : (wide && N > 96) ? TILE_B : sk;
  if (M <= 32) t = TILE_D;
  else if (M <= 64) t = TILE_E;
  else if (N <= 32) t = TILE_C;
  else if (N <= 64) t = TILE_B;
  else t = TILE_A;
  // too few output tiles to occupy the 256 CUs (small-M layers: UNeXt's 14x14 / 28x28
  // token stages, ACC-UNet's 16x16 and 32x32 levels): 64x64 tiles give 2-4x the workgroups.
  // Not for split-K GEMMs (weight gradients): their K split already fills the chip
  // and the larger tile needs fewer operand loads per MFMA.
  // (below 256 tiles: 128 left the 16x16-level GEMMs -- 4096x512x1536, 16384x128x256 --
  // on 128x128 tiles over half the CUs; 256: -0.25 ms of GEMM time per step, step +0.35 %,
  // profiles/r04_few_tiles_ab.txt)
  static long few = -1;
  if (few < 0) {
    const char* e = getenv("ACCUNET_FEW_TILES");  // tuning knob: the tile-count threshold
    few = e ? atol(e) : 256;
  }
  if (!can_split && t != TILE_D && t != TILE_E && M > 64) {
    const long tiles = (long)ceil_div(M, tile_bm(t)) * ceil_div(N, tile_bn(t));
    if (tiles < few) t = TILE_E;
  }
  (void)bmode;
  (void)cin;
  return t;
}

int gemm_run(GemmParams p, int amode, int bmode, int pro_a, int pro_b, bool allow_split,
             float* ws, size_t ws_elems, int adt, int bdt, int cdt, hipStream_t stream) {
  if (p.M <= 0 || p.N <= 0) return ACC_OK;
  if ((amode == AM_SHIFT3 || bmode == BM_NN_SHIFT3) && p.cin <= 0) return ACC_EBADSHAPE;
  const bool bf = adt == ACC_BF16;
  // vectorised operand loads need every contiguous extent to be a whole number of
  // chunks: fp32 engine float4 (4 elements, 16 B), bf16 engine 8 elements (16 B bf16 /
  // 32 B fp32 weights), with chunk-aligned base pointers
  const int q = bf ? 7 : 3;
  const uintptr_t aal = 15, bal = 15;
  bool vec = true;
  if (amode == AM_ROW) {
    for (int s = 0; s < p.nsrc; ++s) {
      int w = p.kbeg[s + 1] - p.kbeg[s];
      if ((w & q) || (p.lda[s] & q) || ((uintptr_t)p.A[s] & aal)) vec = false;
    }
    if (p.K & q) vec = false;
  } else if (amode == AM_SHIFT3) {
    if ((p.cin & q) || (p.lda[0] & q) || ((uintptr_t)p.A[0] & aal)) vec = false;
  } else {  // AM_COL
    if ((p.M & q) || (p.lda[0] & q) || ((uintptr_t)p.A[0] & aal)) vec = false;
  }
  if (bmode == BM_NT) {
    if ((p.K & q) || (p.ldb & q) || ((uintptr_t)p.B & bal)) vec = false;
  } else {
    if ((p.N & q) || (p.ldb & q) || ((uintptr_t)p.B & bal)) vec = false;
    if (bmode == BM_NN_SHIFT3 && (p.cin & q)) vec = false;
  }
  if (amode == AM_ROW && p.nsrc == 1) { p.kbeg[0] = 0; p.kbeg[1] = p.K; }
  if (allow_split && vec && adt == ACC_F32 && bdt == ACC_F32 && cdt == ACC_F32) {
    const int S = conv3x3_c32_wgrad_try(p, amode, bmode, pro_a, pro_b, true, ws, ws_elems, stream);
    if (S > 0) {
      splitk_reduce(ws, (float*)p.C, p.M, p.N, p.ldc, S, (size_t)p.M * p.N, stream);
      return hipGetLastError() == hipSuccess ? ACC_OK : ACC_ELAUNCH;
    }
  }
  if (allow_split && cdt == ACC_F32 && adt == bdt) {
    const int S = gemm_skinny_try(p, amode, bmode, pro_a, pro_b, ws, ws_elems, adt, stream);
    if (S > 0) {
      splitk_reduce(ws, (float*)p.C, p.M, p.N, p.ldc, S, (size_t)p.M * p.N, stream);
      return hipGetLastError() == hipSuccess ? ACC_OK : ACC_ELAUNCH;
    }
  }
  const int epi = (p.bz ? EPI_BNB : 0) | (p.pd2 ? EPI_PYR : 0) | (p.nup > 0 ? EPI_UPS : 0) |
                  ((p.stats && !p.bz) ? EPI_STATS : 0);
  gemm_kfn* tab = table_v(amode, bmode, pro_a, pro_b, epi, vec ? 1 : 0, adt, bdt, cdt);
  if (!tab) return ACC_EBADARG;
  // split-K slabs are fp32: only GEMMs whose C is fp32 (weight gradients) split
  const bool can_split = allow_split && ws != nullptr && p.bias == nullptr && p.nup == 0 &&
                         p.stats == nullptr && p.pd2 == nullptr && cdt == ACC_F32;
  const int BK = bf ? GB_BK : GEMM_BK;
  int t = pick_tile(p.M, p.N, p.K, bmode, p.cin, can_split);
  int BM = tile_bm(t), BN = tile_bn(t);
  int gx = ceil_div(p.M, BM), gy = ceil_div(p.N, BN);

  int S = 1;
  p.kchunk = p.K;
  p.zstride = 0;
  float* Cfinal = (float*)p.C;  // split-K runs only with cdt == ACC_F32
  int ldc_final = p.ldc;
  if (can_split) {
    long tiles = (long)gx * gy;
    long target = tiles >= split_min_tiles() ? 1 : split_target();  // enough tiles: no split
    long maxS = p.K / (BK * 4);
    long want = (target + tiles - 1) / tiles;
    S = (int)(want < maxS ? want : maxS);
    if (S < 1) S = 1;
    while (S > 1 && (size_t)S * p.M * p.N > ws_elems) --S;
    if (S > 1) {
      int kt = ceil_div(p.K, S);
      kt = ceil_div(kt, BK) * BK;
      S = ceil_div(p.K, kt);
      p.kchunk = kt;
      p.zstride = (size_t)p.M * p.N;
      p.C = ws;
      p.ldc = p.N;
    }
  }
  {
    // quad (4-element) epilogue accesses: C rows, up-add rows and pyramid rows all
    // 4-element aligned (16 B fp32 / 8 B bf16)
    const uintptr_t cal = (cdt == ACC_BF16 && S == 1) ? 7 : 15;
    bool ev = (p.N % 4 == 0) && (p.ldc % 4 == 0) && (((uintptr_t)p.C & cal) == 0);
    for (int u = 0; u < p.nup; ++u)
      if ((p.upld[u] % 4) || ((uintptr_t)p.up[u] & cal)) ev = false;
    p.evec = ev ? 1 : 0;
  }
  if (S == 1) {
    const int dmode = !vec ? 0
                      : (adt == ACC_F32 && bdt == ACC_F32 && cdt == ACC_F32) ? 1
                      : (adt == ACC_BF16 && bdt == ACC_F32 && cdt == ACC_BF16) ? 2 : 0;
    const int r = conv3x3_c32_try(p, amode, bmode, pro_a, pro_b, epi, dmode, t, stream);
    if (r >= 0) return r;
  }
  p.ngrp = 0;
  if (S == 1 && gy > 1 && ngrp_kb() > 0) {
    const long per_tile = (long)p.K * BN * (bdt == ACC_BF16 ? 2 : 4);  // B bytes per N tile
    long g = ngrp_kb() * 1024 / per_tile;
    if (g < 1) g = 1;
    if (g < gy) p.ngrp = (int)g;
  }
  dim3 grid(gx, gy, S);
  gemm_kfn kfn = tab[t];
  // (weight gradients, AM_COL: both operands k-major, 4 ds_read_b32 per fragment and
  // k-chunk; the register-staged kernel is as fast or faster there, tools/gg_ab.sh)
  static int gwg = -1;
  if (gwg < 0) {
    const char* e = getenv("ACCUNET_GEMM_G_WGRAD");  // tuning knob: weight gradients on the DMA engine
    gwg = e ? atoi(e) : 0;
  }
  if (vec && adt == ACC_F32 && (amode != AM_COL || gwg)) {
    gemm_kfn g = ggemm_for(amode, bmode, pro_a, pro_b, epi, t);
    if (g) kfn = g;
  }
  hipLaunchKernelGGL(kfn, grid, dim3(GEMM_THREADS), 0, stream, p);
  if (S > 1) splitk_reduce(ws, Cfinal, p.M, p.N, ldc_final, S, p.zstride, stream);
  return hipGetLastError() == hipSuccess ? ACC_OK : ACC_ELAUNCH;
}

// ----------------------------------------------------------------------------
// C ABI (include/accunet.h: AccGemmDesc / accunet_gemm)
// ----------------------------------------------------------------------------
#include "../../include/accunet.h"

extern "C" int accunet_gemm(const AccGemmDesc* d, float* ws, size_t ws_elems, void* stream) {
  if (!d) return ACC_EBADARG;
  GemmParams p;
  memset(&p, 0, sizeof(p));
  p.M = d->M;
  p.N = d->N;
  p.K = d->K;
  p.nsrc = d->nsrc < 1 ? 1 : d->nsrc;
  if (p.nsrc > 4) return ACC_EBADARG;
  for (int s = 0; s < 4; ++s) {
    p.A[s] = d->a[s];
    p.lda[s] = d->lda[s];
  }
  for (int s = 0; s < 5; ++s) p.kbeg[s] = d->kbeg[s];
  p.a_scale = d->a_scale;
  p.a_shift = d->a_shift;
  p.B = d->b;
  p.ldb = d->ldb;
  p.b_scale = d->b_scale;
  p.b_shift = d->b_shift;
  p.H = d->H > 0 ? d->H : 1;
  p.W = d->W > 0 ? d->W : 1;
  p.fW = make_fastdiv((uint32_t)p.W);
  p.fH = make_fastdiv((uint32_t)p.H);
  p.cin = d->cin;
  p.fC = make_fastdiv((uint32_t)(p.cin > 0 ? p.cin : 1));
  p.C = d->c;
  p.ldc = d->ldc;
  p.bias = d->bias;
  p.nup = d->nup;
  if (p.nup < 0 || p.nup > 3) return ACC_EBADARG;
  for (int u = 0; u < 3; ++u) {
    p.up[u] = d->up[u];
    p.upld[u] = d->upld[u];
    p.uplog[u] = d->uplog[u];
  }
  p.stats = d->stats;
  p.pd2 = d->pd2;
  p.pd4 = d->pd4;
  p.mk2 = d->mk2;
  p.mk4 = d->mk4;
  p.bz = d->bz;
  p.bst = d->bst;
  p.bact = d->bact;
  if (p.bz && (!p.bst || !p.stats)) return ACC_EBADARG;
  if (d->adt < ACC_F32 || d->adt > ACC_BF16 || d->bdt < ACC_F32 || d->bdt > ACC_BF16 ||
      d->cdt < ACC_F32 || d->cdt > ACC_BF16)
    return ACC_EBADARG;
  if (p.pd2 && (!p.mk2 || (p.pd4 && !p.mk4) || (p.H & 1) || (p.W & 1) ||
                (p.pd4 && ((p.H & 3) || (p.W & 3))) || p.ldc != p.N))
    return ACC_EBADARG;
  return gemm_run(p, d->amode, d->bmode, d->pro_a, d->pro_b, d->allow_split != 0, ws, ws_elems,
                  d->adt, d->bdt, d->cdt, (hipStream_t)stream);
}

extern "C" int accunet_gemm_stats_rows(int M, int N, int K, int amode, int bmode, int cin) {
  int t = pick_tile(M, N, K, bmode, cin, false);  // statistics GEMMs never split
  return ceil_div(M, tile_bm(t));
}
