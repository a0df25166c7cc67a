// K1 candidate lab, round 5: full-arithmetic K1 structures (prologue BN+LeakyReLU, 3x3
// depthwise + bias, fp64 norm2 statistics) at the north-star shape 16x256x256x96 fp32,
// timed beside the product K1 (libaccunet_hip.so, accunet_dw3x3_fwd) and a
// non-temporal float4 copy of the same bytes, with z compared bit for bit against the
// product and the statistics totals against the product's.
//   make -C tools k1lab2 && tools/k1lab2 [iters]
//
// colx<CR, DB, ARITH>: "column-register strip". A block owns 32 pixels x 8 channel quads
// (one channel group) of a 32-row strip, like the product. Each thread loads ITS OWN
// pixel-quad column row by row (16 lanes of wave 0 also load the two halo pixels), so
// the centre values never go through LDS: per input row a thread writes its activated
// quad to an exchange row in LDS and reads back only the left and right neighbours,
// and keeps three rolling output-row accumulators (12 registers). Input rows arrive in chunks of
// CR rows, the next chunk's loads in flight during the current chunk's arithmetic; DB
// double-buffers the exchange rows (one barrier per chunk instead of two).
// Same FMA order as the product (bias, then taps row-major), so z is bit-identical.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <math.h>
#include <vector>
#include <algorithm>

#include "../include/accunet.h"
#include "../acc-unet-unext_amd/csrc/common.h"
#include "../acc-unet-unext_amd/csrc/chan.h"

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

constexpr int B = 16, H = 256, W = 256, C = 96, TCQ = 8, TP = 32, SR = 32;
constexpr int NCG = C / 4 / TCQ;                  // channel groups (3)
constexpr int NT = B * (H / SR) * (W / TP);       // tiles (1024)
constexpr unsigned IMG = H * W * C * 4;

typedef float v4f __attribute__((ext_vector_type(4)));
__global__ void copy_x4_nt(const v4f* __restrict__ a, v4f* __restrict__ b) {
  long base = (long)blockIdx.x * 1024 + threadIdx.x;
  v4f v[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) v[k] = __builtin_nontemporal_load(&a[base + 256 * k]);
#pragma unroll
  for (int k = 0; k < 4; ++k) __builtin_nontemporal_store(v[k], &b[base + 256 * k]);
}

ACC_DEV float4 act4(float4 a, float4 s, float4 t) {
  a.x = lrelu(a.x * s.x + t.x);
  a.y = lrelu(a.y * s.y + t.y);
  a.z = lrelu(a.z * s.z + t.z);
  a.w = lrelu(a.w * s.w + t.w);
  return a;
}

template <int CR, bool DB, bool ARITH>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(CR >= 8 ? 2 : 3)))
colx(const float* __restrict__ x, const float* __restrict__ wt, const float* __restrict__ bias,
     const float* __restrict__ sc, const float* __restrict__ sh, float* __restrict__ z,
     double* __restrict__ stats) {
  constexpr int IP = TP + 2;                   // exchange row: 34 pixels x 8 quads
  constexpr int NB = DB ? 2 : 1;
  constexpr int NIN = SR + 2;                  // input rows of the strip (with halo)
  constexpr int NCH = (NIN + CR - 1) / CR;
  __shared__ float4 xb[NB][CR][IP][TCQ];
  const int tid = threadIdx.x;
  const int q = tid % TCQ, p = tid / TCQ;
  int bid = blockIdx.x;
  {  // XCD-contiguous runs, channel groups of a tile adjacent (the product's order)
    const int per = gridDim.x >> 3;
    bid = (bid & 7) * per + (bid >> 3);
  }
  const int cg = bid % NCG;
  int t = bid / NCG;
  const int srow = t;
  const int tw = t % (W / TP);
  t /= (W / TP);
  const int th = t % (H / SR);
  const int b = t / (H / SR);
  const int c0 = cg * TCQ * 4, c = c0 + 4 * q;
  const int w0 = tw * TP, w = w0 + p, hbeg = th * SR;
  const long img = (long)b * H * W * C;
  const auto rx = acc_rsrc(x + img, IMG), rz = acc_rsrc(z + img, IMG);
  // halo: 2 pixels (w0 - 1, w0 + 32) x 8 quads x CR rows per chunk = 16 CR quads, one per
  // thread t < 16 CR: row t / 16, side (t / 8) & 1, quad t & 7
  const bool hl = tid < 16 * CR;
  const int hr = tid >> 4, hs = (tid >> 3) & 1, hq = tid & 7;
  const int hw = hs ? w0 + TP : w0 - 1;
  const bool hin = hl && hw >= 0 && hw < W;
  // weights, bias, prologue first (in flight with the first chunk's rows)
  float k[9][4], bi[4];
  float4 ps, pb, hps, hpb;
  {
    float wv[36];
#pragma unroll
    for (int e = 0; e < 9; ++e) {
      const float4 w4 = ld4(wt + c * 9 + 4 * e);
      wv[4 * e] = w4.x; wv[4 * e + 1] = w4.y; wv[4 * e + 2] = w4.z; wv[4 * e + 3] = w4.w;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int tp = 0; tp < 9; ++tp) k[tp][j] = wv[j * 9 + tp];
    const float4 b4 = ld4(bias + c);
    bi[0] = b4.x; bi[1] = b4.y; bi[2] = b4.z; bi[3] = b4.w;
    ps = ld4(sc + c); pb = ld4(sh + c);
    hps = ld4(sc + c0 + 4 * hq); hpb = ld4(sh + c0 + 4 * hq);
  }
  auto fetch = [&](float4 (&v)[CR], float4& vh, int i0) {
#pragma unroll
    for (int r = 0; r < CR; ++r) {
      const int i = i0 + r;
      const bool rin = i >= 0 && i < H && i < hbeg + SR + 1;
      v[r] = bufq_ld<2>(rx, rin ? (unsigned)(((i * W + w) * C + c) * 4) : ACC_OOB, (const float*)nullptr);
    }
    const int i = i0 + hr;
    const bool rin = hin && i >= 0 && i < H && i < hbeg + SR + 1;
    vh = bufq_ld<2>(rx, rin ? (unsigned)(((i * W + hw) * C + c0 + 4 * hq) * 4) : ACC_OOB,
                    (const float*)nullptr);
  };
  float4 cur[CR], nxt[CR], curh, nxth;
  fetch(cur, curh, hbeg - 1);
  // rolling accumulators: an arriving input row i completes output row i - 1 (a0 holds
  // its bias + dy 0 + dy 1 taps; + dy 2), continues row i (a1: bias + dy 0; + dy 1) and
  // starts row i + 1 (bias + dy 0). Rows arrive in order, so every output sums bias,
  // then dy = 0, 1, 2 (dx = 0, 1, 2 within): the product's FMA order.
  float a0[4], a1[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) a0[j] = a1[j] = 0.f;
  double s1[4] = {0.0, 0.0, 0.0, 0.0}, s2[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll 1
  for (int n = 0; n < NCH; ++n) {
    const int i0 = hbeg - 1 + n * CR;
    if (n + 1 < NCH) fetch(nxt, nxth, i0 + CR);
    const int bsel = DB ? (n & 1) : 0;
    // activate (in-image rows only) and publish this chunk's rows
#pragma unroll
    for (int r = 0; r < CR; ++r) {
      const int i = i0 + r;
      const bool rin = i >= 0 && i < H;
      float4 a = cur[r];
      if (ARITH) a = rin ? act4(a, ps, pb) : make_float4(0.f, 0.f, 0.f, 0.f);
      cur[r] = a;
      xb[bsel][r][p + 1][q] = a;
    }
    if (hl) {
      const int i = i0 + hr;
      float4 ah = curh;
      if (ARITH) ah = (hin && i >= 0 && i < H) ? act4(ah, hps, hpb) : make_float4(0.f, 0.f, 0.f, 0.f);
      xb[bsel][hr][hs ? IP - 1 : 0][hq] = ah;
    }
    __syncthreads();
    float c1[4] = {0.f, 0.f, 0.f, 0.f}, c2[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int r = 0; r < CR; ++r) {
      const int i = i0 + r;  // input row arriving; completes output row i - 1
      const float4 L = xb[bsel][r][p][q], R = xb[bsel][r][p + 2][q];
      const float vL[4] = {L.x, L.y, L.z, L.w};
      const float vC[4] = {cur[r].x, cur[r].y, cur[r].z, cur[r].w};
      const float vR[4] = {R.x, R.y, R.z, R.w};
      const int h = i - 1;
      const bool on = h >= hbeg && h < hbeg + SR;  // rows outside the strip: not kept
      float o[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (ARITH) {
          float t0 = a0[j], t1 = a1[j], t2 = bi[j];
          t0 = fmaf(k[6][j], vL[j], t0); t0 = fmaf(k[7][j], vC[j], t0); t0 = fmaf(k[8][j], vR[j], t0);
          t1 = fmaf(k[3][j], vL[j], t1); t1 = fmaf(k[4][j], vC[j], t1); t1 = fmaf(k[5][j], vR[j], t1);
          t2 = fmaf(k[0][j], vL[j], t2); t2 = fmaf(k[1][j], vC[j], t2); t2 = fmaf(k[2][j], vR[j], t2);
          o[j] = t0;
          a0[j] = t1;
          a1[j] = t2;
          const float am = on ? t0 : 0.f;
          c1[j] += am;
          c2[j] = fmaf(am, am, c2[j]);
        } else {
          o[j] = vC[j];
        }
      }
      bufq_st<2>(rz, on ? (unsigned)(((h * W + w) * C + c) * 4) : ACC_OOB,
                 make_float4(o[0], o[1], o[2], o[3]), (float*)nullptr);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      s1[j] += (double)c1[j];
      s2[j] += (double)c2[j];
    }
    if (!DB) __syncthreads();  // every thread has read this chunk's exchange rows
#pragma unroll
    for (int r = 0; r < CR; ++r) cur[r] = nxt[r];
    curh = nxth;
  }
  if (ARITH) {
    __syncthreads();
    double v[8] = {s1[0], s1[1], s1[2], s1[3], s2[0], s2[1], s2[2], s2[3]};
    if (block_slot_reduce<TCQ, 8, double>(v, reinterpret_cast<double*>(&xb[0][0][0][0]))) {
      const long row = (long)srow * 2 * C;
      const int cc = c0 + 4 * threadIdx.x;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        stats[row + cc + j] = v[j];
        stats[row + C + cc + j] = v[4 + j];
      }
    }
  }
}

// os<R, DMA>: one-shot tiles. A block owns R output rows x 32 pixels x 8 quads and
// is gone after one tile (no walk), so the resident blocks of a CU cover neighbouring
// tiles and every block's loads are issued at once (the lab's fastest shapes).
// DMA = false: each thread loads its own pixel-quad column (R + 2 rows) into registers
// and lanes < 16 (R + 2) load the two halo pixels; the activated values go to an LDS
// exchange tile, of which a thread reads back only its left / right neighbours.
// DMA = true: the whole (R + 2) x 34 x 8 input tile goes HBM -> LDS by
// global_load_lds_dwordx4 (zero page outside the image), every thread applies the
// prologue to the three quads of each row it reads (in-image only).
// Weights / bias / prologue vectors are issued before the tile loads.
__device__ __attribute__((aligned(16))) float g_zero4[4] = {0.f, 0.f, 0.f, 0.f};
ACC_DEV void dma16(const float* src, float4* lds_dst) {
  const unsigned dst = __builtin_amdgcn_readfirstlane(
      (unsigned)(size_t)(__attribute__((address_space(3))) float4*)lds_dst);
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(src), "s"(dst)
               : "memory");
}

// STM (statistics): 0 none, 1 fp32 per thread + fp64 block reduce through the exchange
// tile (the product), 2 fp32 in-wave shuffles + fp64 across the 4 waves in a separate LDS
// slab (no barrier before it), 3 per-thread sums only (lanes p == 0 write theirs: the
// accumulation without the reduction), 4 fp64 in-wave shuffles, one partial row per wave
template <int R, bool DMA, int WPE, int PH = 1, bool FULL = false, int AUXL = 2, int AUXS = 2,
          int STM = 1>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE)))
os(const float* __restrict__ x, const float* __restrict__ wt, const float* __restrict__ bias,
   const float* __restrict__ sc, const float* __restrict__ sh, float* __restrict__ z,
   double* __restrict__ stats, int remap) {
  constexpr int IP = TP + 2, IR = R + 2;
  static_assert(IR % PH == 0 && (!DMA || PH == 1), "phases split the input rows");
  constexpr int XR = IR / PH;  // exchange rows per phase (PH = 2: half the LDS)
  // FULL: an exchange row per input row (no reuse across phases: one barrier per phase,
  // and phase 0 waits only for its own rows, issued first)
  constexpr int LR = FULL ? IR : XR;
  __shared__ float4 xb[LR][IP][TCQ];
  const int tid = threadIdx.x;
  const int q = tid % TCQ, p = tid / TCQ;
  int bid = blockIdx.x;
  if (remap) {
    const int per = gridDim.x >> 3;
    bid = (bid & 7) * per + (bid >> 3);
  }
  const int cg = bid % NCG;
  int t = bid / NCG;
  const int srow = t;
  const int tw = t % (W / TP);
  t /= (W / TP);
  constexpr int NTH = (H + R - 1) / R;
  const int th = t % NTH;
  const int b = t / NTH;
  const int c0 = cg * TCQ * 4, c = c0 + 4 * q;
  const int w0 = tw * TP, w = w0 + p, h0 = th * R;
  const long img = (long)b * H * W * C;
  const auto rx = acc_rsrc(x + img, IMG), rz = acc_rsrc(z + img, IMG);
  float k[9][4], bi[4];
  float4 ps, pb;
  {
    float wv[36];
#pragma unroll
    for (int e = 0; e < 9; ++e) {
      const float4 w4 = ld4(wt + c * 9 + 4 * e);
      wv[4 * e] = w4.x; wv[4 * e + 1] = w4.y; wv[4 * e + 2] = w4.z; wv[4 * e + 3] = w4.w;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int tp = 0; tp < 9; ++tp) k[tp][j] = wv[j * 9 + tp];
    const float4 b4 = ld4(bias + c);
    bi[0] = b4.x; bi[1] = b4.y; bi[2] = b4.z; bi[3] = b4.w;
    ps = ld4(sc + c); pb = ld4(sh + c);
  }
  float4 own[IR], hv[PH];
  // halo lanes: per phase 2 pixels x 8 quads x XR rows, lane tid < 16 XR: row tid / 16
  const bool hl = tid < 16 * XR;
  const int hr = tid >> 4, hs = (tid >> 3) & 1;
  const int hw = hs ? w0 + TP : w0 - 1;
  if (DMA) {
    constexpr int NE = IR * IP * TCQ, NI = (NE + 63) / 64;
    const int lane = tid & 63, wave = tid >> 6;
    for (int u = wave; u < NI; u += 4) {
      const int e = u * 64 + lane;
      const int r = e / (IP * TCQ), pp = (e / TCQ) % IP, qq = e % TCQ;
      const int hh = h0 - 1 + r, ww = w0 - 1 + pp;
      const bool ok = e < NE && hh >= 0 && hh < H && ww >= 0 && ww < W;
      const float* src = ok ? x + img + ((long)(hh * W + ww) * C + c0 + 4 * qq) : g_zero4;
      if (e < NE) dma16(src, &xb[0][0][0] + u * 64);
    }
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
  } else {
#pragma unroll
    for (int ph = 0; ph < PH; ++ph) {
#pragma unroll
      for (int rr = 0; rr < XR; ++rr) {
        const int r = ph * XR + rr, i = h0 - 1 + r;
        const bool rin = i >= 0 && i < H;
        own[r] = bufq_ld<AUXL>(rx, rin ? (unsigned)(((i * W + w) * C + c) * 4) : ACC_OOB, (const float*)nullptr);
      }
      const int hrow = h0 - 1 + ph * XR + hr;
      const bool hin = hl && hw >= 0 && hw < W && hrow >= 0 && hrow < H;
      hv[ph] = bufq_ld<AUXL>(rx, hin ? (unsigned)(((hrow * W + hw) * C + c) * 4) : ACC_OOB,
                             (const float*)nullptr);
    }
  }
  float a0[4] = {0.f, 0.f, 0.f, 0.f}, a1[4] = {0.f, 0.f, 0.f, 0.f};
  float c1[4] = {0.f, 0.f, 0.f, 0.f}, c2[4] = {0.f, 0.f, 0.f, 0.f};
  const bool lin = w - 1 >= 0, rinw = w + 1 < W;
#pragma unroll
  for (int ph = 0; ph < PH; ++ph) {
    if (!DMA) {
      if (ph > 0 && !FULL) __syncthreads();  // every thread is done with the previous phase's rows
#pragma unroll
      for (int rr = 0; rr < XR; ++rr) {
        const int r = ph * XR + rr, i = h0 - 1 + r;
        own[r] = (i >= 0 && i < H) ? act4(own[r], ps, pb) : make_float4(0.f, 0.f, 0.f, 0.f);
        xb[FULL ? r : rr][p + 1][q] = own[r];
      }
      if (hl) {
        const int hrow = h0 - 1 + ph * XR + hr;
        const bool hin = hw >= 0 && hw < W && hrow >= 0 && hrow < H;
        xb[FULL ? ph * XR + hr : hr][hs ? IP - 1 : 0][q] = hin ? act4(hv[ph], ps, pb) : make_float4(0.f, 0.f, 0.f, 0.f);
      }
      __syncthreads();
    }
#pragma unroll
    for (int rr = 0; rr < XR; ++rr) {
      const int r = ph * XR + rr, i = h0 - 1 + r;
      const int xr = FULL ? r : rr;
      float4 L = xb[xr][p][q], Cc, Rr = xb[xr][p + 2][q];
      if (DMA) {
        const bool rin = i >= 0 && i < H;
        Cc = xb[xr][p + 1][q];
        Cc = rin ? act4(Cc, ps, pb) : make_float4(0.f, 0.f, 0.f, 0.f);
        L = (rin && lin) ? act4(L, ps, pb) : make_float4(0.f, 0.f, 0.f, 0.f);
        Rr = (rin && rinw) ? act4(Rr, ps, pb) : make_float4(0.f, 0.f, 0.f, 0.f);
      } else {
        Cc = own[r];
      }
      const float vL[4] = {L.x, L.y, L.z, L.w};
      const float vC[4] = {Cc.x, Cc.y, Cc.z, Cc.w};
      const float vR[4] = {Rr.x, Rr.y, Rr.z, Rr.w};
      float o[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float t0 = a0[j], t1 = a1[j], t2 = bi[j];
        t0 = fmaf(k[6][j], vL[j], t0); t0 = fmaf(k[7][j], vC[j], t0); t0 = fmaf(k[8][j], vR[j], t0);
        t1 = fmaf(k[3][j], vL[j], t1); t1 = fmaf(k[4][j], vC[j], t1); t1 = fmaf(k[5][j], vR[j], t1);
        t2 = fmaf(k[0][j], vL[j], t2); t2 = fmaf(k[1][j], vC[j], t2); t2 = fmaf(k[2][j], vR[j], t2);
        o[j] = t0;
        a0[j] = t1;
        a1[j] = t2;
        if (STM && r >= 2 && i - 1 < H) {
          c1[j] += t0;
          c2[j] = fmaf(t0, t0, c2[j]);
        }
      }
      if (r >= 2 && i - 1 < H)
        bufq_st<AUXS>(rz, (unsigned)((((i - 1) * W + w) * C + c) * 4), make_float4(o[0], o[1], o[2], o[3]),
                   (float*)nullptr);
    }
  }
  if (STM == 0) return;
  if (STM == 3) {
    if (p == 0) {
      const long row = (long)srow * 2 * C;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        stats[row + c + j] = c1[j];
        stats[row + C + c + j] = c2[j];
      }
    }
    return;
  }
  if (STM == 2) {
    __shared__ double sw[4][TCQ][8];
    float f[8] = {c1[0], c1[1], c1[2], c1[3], c2[0], c2[1], c2[2], c2[3]};
#pragma unroll
    for (int off = TCQ; off < 64; off <<= 1)
#pragma unroll
      for (int e = 0; e < 8; ++e) f[e] += __shfl_xor(f[e], off);
    const int lane = tid & 63, wave = tid >> 6;
    if (lane < TCQ)
#pragma unroll
      for (int e = 0; e < 8; ++e) sw[wave][lane][e] = (double)f[e];
    __syncthreads();
    if (tid < TCQ) {
      const long row = (long)srow * 2 * C;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const double v = ((sw[0][tid][e] + sw[1][tid][e]) + sw[2][tid][e]) + sw[3][tid][e];
        stats[row + (e >> 2) * C + c0 + 4 * tid + (e & 3)] = v;
      }
    }
    return;
  }
  if (STM == 4) {
    double v[8] = {c1[0], c1[1], c1[2], c1[3], c2[0], c2[1], c2[2], c2[3]};
#pragma unroll
    for (int off = TCQ; off < 64; off <<= 1)
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] += __shfl_xor(v[e], off);
    const int lane = tid & 63, wave = tid >> 6;
    if (lane < TCQ) {
      const long row = ((long)srow * 4 + wave) * 2 * C;
#pragma unroll
      for (int e = 0; e < 8; ++e) stats[row + (e >> 2) * C + c0 + 4 * lane + (e & 3)] = v[e];
    }
    return;
  }
  __syncthreads();
  double v[8] = {c1[0], c1[1], c1[2], c1[3], c2[0], c2[1], c2[2], c2[3]};
  if (block_slot_reduce<TCQ, 8, double>(v, reinterpret_cast<double*>(&xb[0][0][0]))) {
    const long row = (long)srow * 2 * C;
    const int cc = c0 + 4 * threadIdx.x;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      stats[row + cc + j] = v[j];
      stats[row + C + cc + j] = v[4 + j];
    }
  }
}

__global__ void fill(float* p, long n, unsigned salt, float lo, float span) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    p[i] = lo + span * (float)(((i + salt) * 2654435761u) % 10007) / 10007.f;
}

template <class F>
static double timeit(F f, int iters) {
  f();
  std::vector<hipEvent_t> ev(2 * iters);
  for (auto& e : ev) CK(hipEventCreate(&e));
  for (int i = 0; i < iters; ++i) {
    CK(hipEventRecord(ev[2 * i], 0));
    f();
    CK(hipEventRecord(ev[2 * i + 1], 0));
  }
  CK(hipEventSynchronize(ev.back()));
  std::vector<float> t(iters);
  for (int i = 0; i < iters; ++i) CK(hipEventElapsedTime(&t[i], ev[2 * i], ev[2 * i + 1]));
  for (auto& e : ev) CK(hipEventDestroy(e));
  std::sort(t.begin(), t.end());
  return 1000.0 * t[iters / 2];
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 20;
  const size_t n = (size_t)B * H * W * C;
  const double bytes = 2.0 * 4 * n;
  float *x, *z, *zr, *wt, *bi, *sc, *sh;
  CK(hipMalloc(&x, n * 4));
  CK(hipMalloc(&z, n * 4));
  CK(hipMalloc(&zr, n * 4));
  CK(hipMalloc(&wt, 9 * C * 4));
  CK(hipMalloc(&bi, C * 4));
  CK(hipMalloc(&sc, C * 4));
  CK(hipMalloc(&sh, C * 4));
  hipLaunchKernelGGL(fill, dim3(8192), dim3(256), 0, 0, x, (long)n, 1u, -1.f, 2.f);
  hipLaunchKernelGGL(fill, dim3(8), dim3(256), 0, 0, wt, (long)9 * C, 7u, -0.3f, 0.6f);
  hipLaunchKernelGGL(fill, dim3(1), dim3(256), 0, 0, bi, (long)C, 3u, -0.1f, 0.2f);
  hipLaunchKernelGGL(fill, dim3(1), dim3(256), 0, 0, sc, (long)C, 5u, 0.5f, 1.f);
  hipLaunchKernelGGL(fill, dim3(1), dim3(256), 0, 0, sh, (long)C, 9u, -0.2f, 0.4f);
  const int rows = accunet_dw3x3_rows(B, H, W, C, ACC_F32, 0);
  double *st, *str;
  const int st_cap = std::max(rows, 16 * NT);  // rows of the largest grid (R = 8, a row per wave)
  CK(hipMalloc(&st, (size_t)st_cap * 2 * C * 8));
  CK(hipMalloc(&str, (size_t)rows * 2 * C * 8));
  CK(hipDeviceSynchronize());
  auto totals = [&](const double* d, int R) {
    std::vector<double> h((size_t)R * 2 * C), s(2 * C, 0.0);
    CK(hipMemcpy(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost));
    for (int r = 0; r < R; ++r)
      for (int e = 0; e < 2 * C; ++e) s[e] += h[(size_t)r * 2 * C + e];
    return s;
  };
  auto report = [&](const char* name, double us) {
    printf("%-44s %8.2f us %7.1f GB/s %5.1f%%\n", name, us, bytes / us / 1e3,
           100.0 * bytes / us / 1e3 / 8000.0);
    fflush(stdout);
  };
  const long n4 = (long)(n / 4);
  report("copy x4 nt (same bytes)", timeit([&] {
    hipLaunchKernelGGL(copy_x4_nt, dim3(n4 / 1024), dim3(256), 0, 0, (const v4f*)x, (v4f*)z); }, iters));
  auto prod = [&] {
    if (accunet_dw3x3_fwd(x, wt, bi, sc, sh, 1, 0, zr, str, B, H, W, C, nullptr, nullptr, 0, ACC_F32, 0))
      exit(2);
  };
  report("K1 product (dw3x3_tile_fwd_kernel)", timeit(prod, iters));
  prod();
  CK(hipDeviceSynchronize());
  const std::vector<double> sref = totals(str, rows);
  std::vector<unsigned> hz(n), hr(n);
  CK(hipMemcpy(hr.data(), zr, n * 4, hipMemcpyDeviceToHost));
  int stat_rows = NT;
  auto check = [&](const char* name, bool arith) {
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(hz.data(), z, n * 4, hipMemcpyDeviceToHost));
    long bad = 0;
    if (arith)
      for (size_t i = 0; i < n; ++i) bad += hz[i] != hr[i];
    double es = 0.0;
    if (arith) {
      const std::vector<double> s = totals(st, stat_rows);
      for (int e = 0; e < 2 * C; ++e) es = std::max(es, fabs(s[e] - sref[e]) / (fabs(sref[e]) + 1e-30));
    }
    printf("  %-42s z %s (%ld differ), stats max rel %.2e\n", name,
           arith ? (bad ? "MISMATCH" : "bit-identical") : "(no arithmetic)", bad, es);
    fflush(stdout);
  };
  const int grid = NT * NCG;
#define RUN(CR, DB, AR, NAME)                                                                 \
  {                                                                                           \
    auto f = [&] { hipLaunchKernelGGL((colx<CR, DB, AR>), dim3(grid), dim3(256), 0, 0, x, wt, bi, \
                                      sc, sh, z, st); };                                      \
    CK(hipMemset(z, 0, n * 4));                                                               \
    report(NAME, timeit(f, iters));                                                           \
    CK(hipGetLastError());                                                                    \
    check(NAME, AR);                                                                          \
  }
#define RUNOS(R, DMA, WPE, REMAP, NAME) RUNOSP(R, DMA, WPE, REMAP, 1, NAME)
#define RUNOSX(R, WPE, PH, FULL, AL, AS, NAME)                                                 \
  {                                                                                            \
    stat_rows = B * ((H + R - 1) / R) * (W / TP);                                              \
    if (stat_rows > st_cap) { fprintf(stderr, "stats rows %d > %d\n", stat_rows, st_cap); exit(3); } \
    auto f = [&] { hipLaunchKernelGGL((os<R, false, WPE, PH, FULL, AL, AS>), dim3(stat_rows * NCG), dim3(256), 0, 0, \
                                      x, wt, bi, sc, sh, z, st, 0); };                          \
    CK(hipMemset(z, 0, n * 4));                                                                \
    report(NAME, timeit(f, iters));                                                            \
    CK(hipGetLastError());                                                                     \
    check(NAME, true);                                                                         \
    stat_rows = NT;                                                                            \
  }
#define RUNOSP(R, DMA, WPE, REMAP, PH, NAME)                                                   \
  {                                                                                            \
    stat_rows = B * (H / R) * (W / TP);                                                        \
    if (stat_rows > st_cap) { fprintf(stderr, "stats rows %d > %d\n", stat_rows, st_cap); exit(3); } \
    auto f = [&] { hipLaunchKernelGGL((os<R, DMA, WPE, PH>), dim3(stat_rows * NCG), dim3(256), 0, 0, x, wt, \
                                      bi, sc, sh, z, st, REMAP); };                            \
    CK(hipMemset(z, 0, n * 4));                                                                \
    report(NAME, timeit(f, iters));                                                            \
    CK(hipGetLastError());                                                                     \
    check(NAME, true);                                                                         \
    stat_rows = NT;                                                                            \
  }
#define RUNOSS(STM, NAME)                                                                       \
  {                                                                                            \
    stat_rows = B * (H / 8) * (W / TP);                                                        \
    const int srows = STM == 4 ? 4 * stat_rows : stat_rows;                                    \
    if (srows > st_cap) { fprintf(stderr, "stats rows %d > %d\n", srows, st_cap); exit(3); }   \
    auto f = [&] { hipLaunchKernelGGL((os<8, false, 3, 1, false, 2, 2, STM>), dim3(stat_rows * NCG), dim3(256), 0, 0, \
                                      x, wt, bi, sc, sh, z, st, 0); };                          \
    CK(hipMemset(z, 0, n * 4));                                                                \
    report(NAME, timeit(f, iters));                                                            \
    CK(hipGetLastError());                                                                     \
    stat_rows = srows;                                                                         \
    check(NAME, STM == 1 || STM == 2 || STM == 4);                                             \
    stat_rows = NT;                                                                            \
  }
  RUNOS(8, false, 3, 0, "os R8 regs");
  RUNOSS(0, "os R8 stats: none");
  RUNOSS(3, "os R8 stats: per-thread sums only");
  RUNOSS(2, "os R8 stats: fp32 wave shuffles + fp64 slab");
  RUNOSS(4, "os R8 stats: fp64 shuffles, row per wave");
  RUNOSS(1, "os R8 stats: product form");
  RUNOS(8, false, 3, 0, "os R8 regs (again)");
  report("K1 product (again)", timeit(prod, iters));
  report("copy x4 nt (again)", timeit([&] {
    hipLaunchKernelGGL(copy_x4_nt, dim3(n4 / 1024), dim3(256), 0, 0, (const v4f*)x, (v4f*)z); }, iters));
  return 0;
}
