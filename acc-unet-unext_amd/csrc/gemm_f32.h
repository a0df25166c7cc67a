// fp32 MFMA GEMM engine (the precision the reference trains in): every convolution
// on the ACC-UNet path in fp32 activation mode. Operand modes, the prologue and the
// epilogue: gemm_common.h.
//
// Matrix core: v_mfma_f32_32x32x2_f32 (exact fp32 fma chain, 64 cyc/SIMD), 4 waves
// (64-wide) per 256-thread workgroup laid out WM x WN, each wave owning TM x TN
// 32x32 accumulator tiles (16 regs each). K is staged 16 at a time through a
// double-buffered, padded, k-major LDS image so every MFMA operand read is a
// conflict-free ds_read_b32 (lanes 0-31 and 32-63 sit in different bank groups).
#pragma once
#include "gemm_common.h"

#define GEMM_BK 16
// k-tiles of register-staged prefetch in flight. 2 gives each tile two iterations of
// MFMA work to land, but measured slower on every weight-gradient family (AM_COL 128x128
// 73 -> 86 us per call, profiles/r03_step_ab.txt), so the default stays 1.
#ifndef GEMM_PF
#define GEMM_PF 1
#endif

template <int AMODE, int BMODE, int PRO_A, int PRO_B, bool VA, bool VB, int WM, int TM, int TN,
          int EPI = 0>
__global__ void __launch_bounds__(GEMM_THREADS)
gemm_f32_kernel(const GemmParams p) {
  constexpr int WN = 4 / WM;
  constexpr int BM = WM * TM * 32;
  constexpr int BN = WN * TN * 32;
  constexpr int BK = GEMM_BK;
  constexpr int SA = BM + GEMM_PAD;
  constexpr int SB = BN + GEMM_PAD;
  constexpr int QPR = BK / 4;  // float4 quads per BK-slice of one row
  constexpr int NA4 = BM * QPR, NB4 = BN * QPR;  // float4 elements per stage
  constexpr int NPA = (NA4 + GEMM_THREADS - 1) / GEMM_THREADS;
  constexpr int NPB = (NB4 + GEMM_THREADS - 1) / GEMM_THREADS;

  __shared__ __attribute__((aligned(16))) float smem[2 * BK * SA + 2 * BK * SB];
  float* As = smem;
  float* Bs = smem + 2 * BK * SA;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave % WM;
  const int wn = wave / WM;
  const int l31 = lane & 31;
  const int lh = lane >> 5;

  int mt, nt;
  gemm_tile(mt, nt, p.ngrp);
  const int m0 = mt * BM;
  const int n0 = nt * BN;
  const int M = p.M, N = p.N, K = p.K;

  int kstart = 0, kend = K;
  if (gridDim.z > 1) {
    kstart = blockIdx.z * p.kchunk;
    kend = min(K, kstart + p.kchunk);
  }
  const int nkt = kend > kstart ? (kend - kstart + BK - 1) / BK : 0;

  // ---- per-thread A row geometry for the implicit 3x3 conv -----------------
  int a_h[NPA], a_w[NPA];
  if (AMODE == AM_SHIFT3) {
#pragma unroll
    for (int i = 0; i < NPA; ++i) {
      int idx = tid + i * GEMM_THREADS;
      int r = idx / QPR;
      uint32_t g = (uint32_t)(m0 + r);
      uint32_t q = fdiv(g, p.fW);
      a_w[i] = (int)(g - q * p.W);
      a_h[i] = (int)(q - fdiv(q, p.fH) * p.H);
    }
  }

  // register staging: PF k-tiles in flight (tile kt+PF is loaded while kt is computed;
  // tile kt+1 is written to the other LDS buffer at the end of iteration kt)
  constexpr int PF = GEMM_PF;
  static_assert(PF == 1 || PF == 2, "register prefetch depth 1 or 2");
  float4 ra[PF][NPA], rb[PF][NPB];
  // BM_NN prologue coefficients: thread i-slot always loads the same column quad
  float4 bsc[NPB], bsh[NPB];
  if (BMODE == BM_NN && PRO_B != PRO_NONE) {
#pragma unroll
    for (int i = 0; i < NPB; ++i) {
      const int n = n0 + 4 * ((tid + i * GEMM_THREADS) % (BN / 4));
      float e[8];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        e[j] = (n + j < N) ? p.b_scale[n + j] : 1.f;
        e[4 + j] = (n + j < N) ? p.b_shift[n + j] : 0.f;
      }
      bsc[i] = make_float4(e[0], e[1], e[2], e[3]);
      bsh[i] = make_float4(e[4], e[5], e[6], e[7]);
    }
  }

  const float* Bp = (const float*)p.B;
  auto load_tiles = [&](int k0, int sl) {
    // ------------------------------ A ---------------------------------------
    if (AMODE == AM_ROW) {
      // up to 4 channel-concatenated sources; source seams may fall anywhere (a
      // float4 never straddles one in the vectorised path: widths are % 4 == 0)
#pragma unroll
      for (int i = 0; i < NPA; ++i) {
        int idx = tid + i * GEMM_THREADS;
        int r = idx / QPR, q = idx % QPR;
        int g = m0 + r;
        int k = k0 + 4 * q;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if ((idx < NA4) && (g < M)) {
          if (VA) {
            if (k < K) {
              // source of this quad (a float4 never straddles a seam): explicit selects
              // over the kernel arguments keep base / ld / kbeg in SGPRs -> v_cndmask,
              // instead of a lane-indexed p.A[s] that hipcc turns into dependent
              // global loads of the argument block inside the k-loop
              const float* base = (const float*)p.A[0];
              int ld = p.lda[0], kb = 0;
              if (p.nsrc > 1) {
                if (k >= p.kbeg[1]) { base = (const float*)p.A[1]; ld = p.lda[1]; kb = p.kbeg[1]; }
                if (p.nsrc > 2 && k >= p.kbeg[2]) { base = (const float*)p.A[2]; ld = p.lda[2]; kb = p.kbeg[2]; }
                if (p.nsrc > 3 && k >= p.kbeg[3]) { base = (const float*)p.A[3]; ld = p.lda[3]; kb = p.kbeg[3]; }
              }
              v = ld4(base + (long)g * ld + (k - kb));
              if (PRO_A != PRO_NONE && kb == 0) {  // the pending BatchNorm sits on source 0
                const float4 sc = ld4(p.a_scale + k), sh = ld4(p.a_shift + k);
                v.x = pro_apply<PRO_A>(v.x, sc.x, sh.x);
                v.y = pro_apply<PRO_A>(v.y, sc.y, sh.y);
                v.z = pro_apply<PRO_A>(v.z, sc.z, sh.z);
                v.w = pro_apply<PRO_A>(v.w, sc.w, sh.w);
              }
            }
          } else {
            float e[4];
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) {
              int kk = k + jj;
              e[jj] = 0.f;
              if (kk < K) {
                int s = 0;
#pragma unroll
                for (int j = 1; j < 4; ++j)
                  if (j < p.nsrc && kk >= p.kbeg[j]) s = j;
                float x = ((const float*)p.A[s])[(long)g * p.lda[s] + (kk - p.kbeg[s])];
                if (PRO_A != PRO_NONE && s == 0) x = pro_apply<PRO_A>(x, p.a_scale[kk], p.a_shift[kk]);
                e[jj] = x;
              }
            }
            v = make_float4(e[0], e[1], e[2], e[3]);
          }
        }
        ra[sl][i] = v;
      }
    } else if (AMODE == AM_SHIFT3) {
      // implicit 3x3: k = tap*cin + ci; zero padding outside the image
      const float* Ab = (const float*)p.A[0];
      const int lda = p.lda[0];
#pragma unroll
      for (int i = 0; i < NPA; ++i) {
        int idx = tid + i * GEMM_THREADS;
        int r = idx / QPR, q = idx % QPR;
        int g = m0 + r;
        int k = k0 + 4 * q;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if ((idx < NA4) && (g < M)) {
          if (VA) {  // cin % 4 == 0: the quad shares one tap
            if (k < K) {
              int tap = (int)fdiv((uint32_t)k, p.fC);
              int ci = k - tap * p.cin;
              int dh = tap / 3 - 1, dw = tap - (tap / 3) * 3 - 1;
              int hh = a_h[i] + dh, ww = a_w[i] + dw;
              if (hh >= 0 && hh < p.H && ww >= 0 && ww < p.W)
                v = ld4(Ab + ((long)g + dh * p.W + dw) * lda + ci);
            }
          } else {
            float e[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              e[j] = 0.f;
              int kk = k + j;
              if (kk < K) {
                int tap = (int)fdiv((uint32_t)kk, p.fC);
                int ci = kk - tap * p.cin;
                int dh = tap / 3 - 1, dw = tap - (tap / 3) * 3 - 1;
                int hh = a_h[i] + dh, ww = a_w[i] + dw;
                if (hh >= 0 && hh < p.H && ww >= 0 && ww < p.W)
                  e[j] = Ab[((long)g + dh * p.W + dw) * lda + ci];
              }
            }
            v = make_float4(e[0], e[1], e[2], e[3]);
          }
        }
        ra[sl][i] = v;
      }
    } else {  // AM_COL: A(m,k) = A[k*lda + m]
      const float* Ab = (const float*)p.A[0];
      const int lda = p.lda[0];
#pragma unroll
      for (int i = 0; i < NPA; ++i) {
        int idx = tid + i * GEMM_THREADS;
        int kr = idx / (BM / 4), q = idx % (BM / 4);
        int k = k0 + kr;
        int m = m0 + 4 * q;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (idx < NA4 && k < kend) {
          const float* ptr = Ab + (long)k * lda + m;
          if (VA) {
            if (m < M) v = ld4(ptr);
          } else {
            if (m + 0 < M) v.x = ptr[0];
            if (m + 1 < M) v.y = ptr[1];
            if (m + 2 < M) v.z = ptr[2];
            if (m + 3 < M) v.w = ptr[3];
          }
        }
        ra[sl][i] = v;
      }
    }
    // ------------------------------ B ---------------------------------------
    if (BMODE == BM_NT) {
#pragma unroll
      for (int i = 0; i < NPB; ++i) {
        int idx = tid + i * GEMM_THREADS;
        int r = idx / QPR, q = idx % QPR;
        int n = n0 + r;
        int k = k0 + 4 * q;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (idx < NB4 && n < N) {
          const float* ptr = Bp + (long)n * p.ldb + k;
          if (VB) {
            if (k < kend) v = ld4(ptr);
          } else {
            if (k + 0 < kend) v.x = ptr[0];
            if (k + 1 < kend) v.y = ptr[1];
            if (k + 2 < kend) v.z = ptr[2];
            if (k + 3 < kend) v.w = ptr[3];
          }
        }
        rb[sl][i] = v;
      }
    } else if (BMODE == BM_NN) {  // B(k,n) = B[k*ldb + n]
#pragma unroll
      for (int i = 0; i < NPB; ++i) {
        int idx = tid + i * GEMM_THREADS;
        int kr = idx / (BN / 4), q = idx % (BN / 4);
        int k = k0 + kr;
        int n = n0 + 4 * q;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (idx < NB4 && k < kend) {
          const float* ptr = Bp + (long)k * p.ldb + n;
          if (VB) {
            if (n < N) v = ld4(ptr);
          } else {
            if (n + 0 < N) v.x = ptr[0];
            if (n + 1 < N) v.y = ptr[1];
            if (n + 2 < N) v.z = ptr[2];
            if (n + 3 < N) v.w = ptr[3];
          }
          if (PRO_B != PRO_NONE) {  // per-column coefficients, loaded once (bsc/bsh)
            if (n + 0 < N) v.x = pro_apply<PRO_B>(v.x, bsc[i].x, bsh[i].x);
            if (n + 1 < N) v.y = pro_apply<PRO_B>(v.y, bsc[i].y, bsh[i].y);
            if (n + 2 < N) v.z = pro_apply<PRO_B>(v.z, bsc[i].z, bsh[i].z);
            if (n + 3 < N) v.w = pro_apply<PRO_B>(v.w, bsc[i].w, bsh[i].w);
          }
        }
        rb[sl][i] = v;
      }
    } else {  // BM_NN_SHIFT3: B(k = pixel p, n = tap*cin + ci) = X[shift_tap(p)*ldb + ci]
#pragma unroll
      for (int i = 0; i < NPB; ++i) {
        int idx = tid + i * GEMM_THREADS;
        int kr = idx / (BN / 4), q = idx % (BN / 4);
        int k = k0 + kr;
        int n = n0 + 4 * q;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (idx < NB4 && k < kend) {
          uint32_t qq = fdiv((uint32_t)k, p.fW);
          int ww0 = k - (int)qq * p.W;
          int hh0 = (int)(qq - fdiv(qq, p.fH) * p.H);
          if (VB) {  // cin % 4 == 0: the quad shares one tap
            if (n < N) {
              int tap = (int)fdiv((uint32_t)n, p.fC);
              int ci = n - tap * p.cin;
              int dh = tap / 3 - 1, dw = tap - (tap / 3) * 3 - 1;
              if (hh0 + dh >= 0 && hh0 + dh < p.H && ww0 + dw >= 0 && ww0 + dw < p.W)
                v = ld4(Bp + ((long)k + dh * p.W + dw) * p.ldb + ci);
            }
          } else {
            float e[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              e[j] = 0.f;
              int nn = n + j;
              if (nn < N) {
                int tap = (int)fdiv((uint32_t)nn, p.fC);
                int ci = nn - tap * p.cin;
                int dh = tap / 3 - 1, dw = tap - (tap / 3) * 3 - 1;
                if (hh0 + dh >= 0 && hh0 + dh < p.H && ww0 + dw >= 0 && ww0 + dw < p.W)
                  e[j] = Bp[((long)k + dh * p.W + dw) * p.ldb + ci];
              }
            }
            v = make_float4(e[0], e[1], e[2], e[3]);
          }
        }
        rb[sl][i] = v;
      }
    }
  };

  auto store_tiles = [&](int buf, int sl) {
    float* as = As + buf * BK * SA;
    float* bs = Bs + buf * BK * SB;
    if (AMODE == AM_COL) {
#pragma unroll
      for (int i = 0; i < NPA; ++i) {
        int idx = tid + i * GEMM_THREADS;
        if (idx < NA4) {
          int kr = idx / (BM / 4), q = idx % (BM / 4);
          st4(as + kr * SA + 4 * q, ra[sl][i]);
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < NPA; ++i) {
        int idx = tid + i * GEMM_THREADS;
        if (idx < NA4) {
          int r = idx / QPR, q = idx % QPR;
          as[(4 * q + 0) * SA + r] = ra[sl][i].x;
          as[(4 * q + 1) * SA + r] = ra[sl][i].y;
          as[(4 * q + 2) * SA + r] = ra[sl][i].z;
          as[(4 * q + 3) * SA + r] = ra[sl][i].w;
        }
      }
    }
    if (BMODE == BM_NT) {
#pragma unroll
      for (int i = 0; i < NPB; ++i) {
        int idx = tid + i * GEMM_THREADS;
        if (idx < NB4) {
          int r = idx / QPR, q = idx % QPR;
          bs[(4 * q + 0) * SB + r] = rb[sl][i].x;
          bs[(4 * q + 1) * SB + r] = rb[sl][i].y;
          bs[(4 * q + 2) * SB + r] = rb[sl][i].z;
          bs[(4 * q + 3) * SB + r] = rb[sl][i].w;
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < NPB; ++i) {
        int idx = tid + i * GEMM_THREADS;
        if (idx < NB4) {
          int kr = idx / (BN / 4), q = idx % (BN / 4);
          st4(bs + kr * SB + 4 * q, rb[sl][i]);
        }
      }
    }
  };

  floatx16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int am_off = wm * TM * 32 + l31;
  const int bn_off = wn * TN * 32 + l31;

  if (nkt > 0) {
#pragma unroll
    for (int sl = 0; sl < PF; ++sl) load_tiles(kstart + sl * BK, sl);
    store_tiles(0, 0);
    __syncthreads();
    for (int kt = 0; kt < nkt; ++kt) {
      const int buf = kt & 1;
      // unconditional (tiles past kend load zeros under the lane masks), so the
      // compiler's vmcnt counting stays exact across iterations
      // (tile t lives in register slot t % PF; the slot of tile kt is free: kt is in LDS)
      if (PF == 2) {
        if ((kt & 1) == 0) load_tiles(kstart + (kt + 2) * BK, 0);
        else load_tiles(kstart + (kt + 2) * BK, 1);
      } else if (kt + 1 < nkt) {
        load_tiles(kstart + (kt + 1) * BK, 0);
      }
      const float* as = As + buf * BK * SA;
      const float* bs = Bs + buf * BK * SB;
      // fragments for step kk+1 are read from LDS before the MFMAs of step kk issue
      float a[2][TM], b[2][TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) a[0][i] = as[lh * SA + am_off + i * 32];
#pragma unroll
      for (int j = 0; j < TN; ++j) b[0][j] = bs[lh * SB + bn_off + j * 32];
#pragma unroll
      for (int kk = 0; kk < BK / 2; ++kk) {
        const int cur = kk & 1;
        if (kk + 1 < BK / 2) {
#pragma unroll
          for (int i = 0; i < TM; ++i) a[cur ^ 1][i] = as[(2 * kk + 2 + lh) * SA + am_off + i * 32];
#pragma unroll
          for (int j = 0; j < TN; ++j) b[cur ^ 1][j] = bs[(2 * kk + 2 + lh) * SB + bn_off + j * 32];
        }
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[cur][i], b[cur][j], acc[i][j], 0, 0, 0);
      }
      if (kt + 1 < nkt) {  // tile kt+1 (slot (kt+1) % PF) -> the other LDS buffer
        if (PF == 2 && (kt & 1) == 0) store_tiles(buf ^ 1, 1);
        else store_tiles(buf ^ 1, 0);
      }
      __syncthreads();
    }
  }

  static_assert(gemm_epi_floats<WM, TM, TN>() <= 2 * BK * SA + 2 * BK * SB,
                "epilogue staging exceeds the LDS tile");
  gemm_epilogue<float, EPI, WM, TM, TN>(p, acc, smem, m0, n0);
}
