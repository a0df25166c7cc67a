// bf16 MFMA GEMM engine: every convolution on the ACC-UNet path in bf16 activation
// mode (BASELINE configs[2]: bf16 activations, fp32 master weights and statistics).
// Same operand modes, prologue and epilogue as the fp32 engine (gemm_common.h):
// A / B operands are staged to LDS as bf16 (activations are bf16 in HBM, fp32
// weights are rounded on the way), accumulation is fp32, C is bf16 (activations,
// data gradients) or fp32 (weight gradients, split-K slabs).
//
// Matrix core: v_mfma_f32_32x32x16_bf16. Lane l holds A[row l&31][k = 8(l>>5)+j] and
// B[k = 8(l>>5)+j][col l&31], j < 8: a 16-byte ds_read_b128 of a k-contiguous LDS row.
// So both operands live in LDS as [row][k] images (row = m for A, n for B), BK = 32 k
// per stage (2 MFMA k-steps), rows padded to 40 elements (80 B: the 16 rows a
// ds_read_b128 pass serves land on 16 distinct 4-bank groups), double-buffered.
// Operands whose k axis is contiguous in HBM (AM_ROW / AM_SHIFT3 activations, BM_NT
// weights) move as 16-byte chunks of 8 k; operands whose k axis is the slow one
// (AM_COL dY^T, BM_NN weights / activations, BM_NN_SHIFT3) are read as 16-byte chunks
// of 8 consecutive m / n at one k and transposed on the LDS write (8 ds_write_b16;
// consecutive lanes take consecutive k so a wave's writes spread over the banks).
#pragma once
#include "gemm_common.h"

#define GB_BK 32
#define GB_SK (GB_BK + 8)
// k-tiles of register-staged operands in flight: 1 (tile kt+1 loads while kt computes)
// or 2 (tiles kt+1 and kt+2; the main loop unrolled by two so every staging slot index
// is a compile-time constant). Depth 2 applies to the fp32-output vector instances
// without an A prologue (split-K slabs, weight gradients), whose blocks walk long k
// ranges: the bf16 GEMM census has those 6 % faster with it (16384 x 128 x 8704
// split-K: 218 -> 139 us), but they run on the side stream beside the data gradients,
// and the bf16 step did not move (profiles/r06_gb_pf_ab.txt); the bf16-output GEMMs
// (short K, heavy epilogues) and the A-prologue instances ran slower with depth 2 (more
// VGPRs: a wave per SIMD less). Default 1.
#ifndef GB_PF
#define GB_PF 1
#endif

// ---- 8-element chunks -----------------------------------------------------
ACC_DEV void unpack8(uint4 u, float (&f)[8]) {
  f[0] = bflo(u.x); f[1] = bfhi(u.x); f[2] = bflo(u.y); f[3] = bfhi(u.y);
  f[4] = bflo(u.z); f[5] = bfhi(u.z); f[6] = bflo(u.w); f[7] = bfhi(u.w);
}
ACC_DEV uint4 pack8(const float (&f)[8]) {
  return make_uint4(pack_bf2(f[0], f[1]), pack_bf2(f[2], f[3]), pack_bf2(f[4], f[5]),
                    pack_bf2(f[6], f[7]));
}
ACC_DEV uint4 ld8_bf(const bf16_t* p) { return *reinterpret_cast<const uint4*>(p); }
ACC_DEV uint4 ld8_bf(const float* p) {
  const float4 a = ld4(p), b = ld4(p + 4);
  return make_uint4(pack_bf2(a.x, a.y), pack_bf2(a.z, a.w), pack_bf2(b.x, b.y), pack_bf2(b.z, b.w));
}
ACC_DEV void ld8f(const bf16_t* p, float (&f)[8]) { unpack8(ld8_bf(p), f); }
ACC_DEV void ld8f(const float* p, float (&f)[8]) {
  const float4 a = ld4(p), b = ld4(p + 4);
  f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w; f[4] = b.x; f[5] = b.y; f[6] = b.z; f[7] = b.w;
}
ACC_DEV bf16_t u4get(const uint4& u, int j) {
  const unsigned w = j < 2 ? u.x : j < 4 ? u.y : j < 6 ? u.z : u.w;
  return (bf16_t)((j & 1) ? (w >> 16) : (w & 0xffffu));
}

template <int AMODE, int BMODE, int PRO_A, int PRO_B, bool VA, bool VB, int WM, int TM, int TN,
          int EPI, typename TA, typename TB, typename TC>
__global__ void __launch_bounds__(GEMM_THREADS)
gemm_bf16_kernel(const GemmParams p) {
  constexpr int WN = 4 / WM;
  constexpr int BM = WM * TM * 32;
  constexpr int BN = WN * TN * 32;
  constexpr int BK = GB_BK, SK = GB_SK;
  constexpr int NCA = BM * BK / 8, NCB = BN * BK / 8;  // 8-element chunks per stage
  constexpr int NPA = (NCA + GEMM_THREADS - 1) / GEMM_THREADS;
  constexpr int NPB = (NCB + GEMM_THREADS - 1) / GEMM_THREADS;
  constexpr bool TRA = AMODE == AM_COL;     // A staged through a transpose
  constexpr bool TRB = BMODE != BM_NT;      // B staged through a transpose
  constexpr int MAIN_BYTES = 2 * (BM + BN) * SK * 2;
  constexpr int EPI_BYTES = gemm_epi_floats<WM, TM, TN>() * 4;
  constexpr int SMEM_BYTES = MAIN_BYTES > EPI_BYTES ? MAIN_BYTES : EPI_BYTES;
  __shared__ __attribute__((aligned(16))) unsigned char smem_raw[SMEM_BYTES];
  bf16_t* As = reinterpret_cast<bf16_t*>(smem_raw);
  bf16_t* Bs = As + 2 * BM * SK;

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

  // ---- per-slot constant geometry -------------------------------------------
  // row-type operand slot i: chunk c = tid + 256 i -> row c / (BK/8), chunk-in-row c % (BK/8)
  // transposed slot i: k-row c % BK, 8-column group c / BK
  int a_h[NPA], a_w[NPA];  // AM_SHIFT3 pixel of the slot's row
  if (AMODE == AM_SHIFT3) {
#pragma unroll
    for (int i = 0; i < NPA; ++i) {
      const int r = (tid + i * GEMM_THREADS) / (BK / 8);
      const uint32_t g = (uint32_t)(m0 + r);
      const uint32_t q = fdiv(g, p.fW);
      a_w[i] = (int)(g - q * p.W);
      a_h[i] = (int)(q - fdiv(q, p.fH) * p.H);
    }
  }
  float bsc[BMODE == BM_NN && PRO_B != PRO_NONE ? NPB : 1][8];
  float bsh[BMODE == BM_NN && PRO_B != PRO_NONE ? NPB : 1][8];
  if (BMODE == BM_NN && PRO_B != PRO_NONE) {
#pragma unroll
    for (int i = 0; i < NPB; ++i) {
      const int n = n0 + 8 * ((tid + i * GEMM_THREADS) / BK);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        bsc[i][j] = (n + j < N) ? p.b_scale[n + j] : 1.f;
        bsh[i][j] = (n + j < N) ? p.b_shift[n + j] : 0.f;
      }
    }
  }

  const TA* A0 = (const TA*)p.A[0];
  const TB* Bp = (const TB*)p.B;
  // Staged operands stay raw until store_tiles: the vector paths (VA / VB) load
  // unconditionally (masked chunks read a valid address and are zeroed at the store)
  // and convert / apply the prologue only when parking in LDS, so the compiler waits
  // for the loads there, after this k-tile's MFMAs, not right after issuing them.
  // The scalar fallback paths (!VA / !VB) finish their chunk at load time.
  constexpr bool BF = sizeof(TB) == 4;  // fp32 B operand (weights): rounded at the store
  static_assert(GB_PF == 1 || GB_PF == 2, "register prefetch depth 1 or 2");
  constexpr bool PF2OK = GB_PF == 2 && VA && VB && PRO_A == PRO_NONE && EPI == 0 &&
                        sizeof(TC) == 4;
  constexpr int PF = PF2OK ? 2 : 1;
  uint4 ra[PF][NPA], rb[PF][NPB];
  float4 rbl[PF][BF ? NPB : 1], rbh[PF][BF ? NPB : 1];
  float4 asl[PF][PRO_A != PRO_NONE ? NPA : 1], ash[PF][PRO_A != PRO_NONE ? NPA : 1];
  float4 asl2[PF][PRO_A != PRO_NONE ? NPA : 1], ash2[PF][PRO_A != PRO_NONE ? NPA : 1];
  bool aok[PF][NPA], apro[PF][NPA], bok[PF][NPB];

  // sl: staging slot (compile-time after unrolling)
  auto load_tiles = [&](int k0, int sl) {
    // ------------------------------ A ---------------------------------------
#pragma unroll
    for (int i = 0; i < NPA; ++i) {
      const int c = tid + i * GEMM_THREADS;
      aok[sl][i] = false;
      apro[sl][i] = false;
      if (AMODE == AM_ROW) {
        const int r = c / (BK / 8), q = c % (BK / 8);
        const int g = m0 + r, k = k0 + 8 * q;
        if (VA) {
          const bool ok = c < NCA && g < M && k < K;
          // source of this chunk (widths % 8 == 0: a chunk never straddles a seam);
          // explicit selects keep base / ld / kbeg scalar (see gemm_f32.h)
          const TA* base = A0;
          int ld = p.lda[0], kb = 0;
          if (p.nsrc > 1) {
            if (k >= p.kbeg[1]) { base = (const TA*)p.A[1]; ld = p.lda[1]; kb = p.kbeg[1]; }
            if (p.nsrc > 2 && k >= p.kbeg[2]) { base = (const TA*)p.A[2]; ld = p.lda[2]; kb = p.kbeg[2]; }
            if (p.nsrc > 3 && k >= p.kbeg[3]) { base = (const TA*)p.A[3]; ld = p.lda[3]; kb = p.kbeg[3]; }
          }
          const TA* src = ok ? base + (long)g * ld + (k - kb) : A0;
          ra[sl][i] = ld8_bf(src);
          aok[sl][i] = ok;
          if (PRO_A != PRO_NONE) {  // the pending BatchNorm sits on source 0
            apro[sl][i] = kb == 0;
            // coefficients exist for source 0's columns only: other sources' chunks read
            // element 0 (unused: apro false) instead of past the end of a_scale / a_shift
            const int kk = (ok && kb == 0) ? k : 0;
            asl[sl][i] = ld4(p.a_scale + kk);
            asl2[sl][i] = ld4(p.a_scale + kk + 4);
            ash[sl][i] = ld4(p.a_shift + kk);
            ash2[sl][i] = ld4(p.a_shift + kk + 4);
          }
        } else {
          uint4 v = make_uint4(0u, 0u, 0u, 0u);
          if (c < NCA && g < M) {
            float f[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              const int kk = k + j;
              f[j] = 0.f;
              if (kk < K) {
                int s = 0;
#pragma unroll
                for (int t = 1; t < 4; ++t)
                  if (t < p.nsrc && kk >= p.kbeg[t]) s = t;
                float x = ld1((const TA*)p.A[s] + (long)g * p.lda[s] + (kk - p.kbeg[s]));
                if (PRO_A != PRO_NONE && s == 0) x = pro_apply<PRO_A>(x, p.a_scale[kk], p.a_shift[kk]);
                f[j] = x;
              }
            }
            v = pack8(f);
          }
          ra[sl][i] = v;
        }
      } else if (AMODE == AM_SHIFT3) {
        const int r = c / (BK / 8), q = c % (BK / 8);
        const int g = m0 + r, k = k0 + 8 * q;
        const int lda = p.lda[0];
        if (VA) {  // cin % 8 == 0: the chunk shares one tap
          const int tap = (int)fdiv((uint32_t)k, p.fC);
          const int ci = k - tap * p.cin;
          const int dh = tap / 3 - 1, dw = tap - (tap / 3) * 3 - 1;
          const int hh = a_h[i] + dh, ww = a_w[i] + dw;
          const bool ok = c < NCA && g < M && k < K && hh >= 0 && hh < p.H && ww >= 0 && ww < p.W;
          ra[sl][i] = ld8_bf(ok ? A0 + ((long)g + dh * p.W + dw) * lda + ci : A0);
          aok[sl][i] = ok;
        } else {
          uint4 v = make_uint4(0u, 0u, 0u, 0u);
          if (c < NCA && g < M) {
            float f[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              f[j] = 0.f;
              const int kk = k + j;
              if (kk < K) {
                const int tap = (int)fdiv((uint32_t)kk, p.fC);
                const int ci = kk - tap * p.cin;
                const int dh = tap / 3 - 1, dw = tap - (tap / 3) * 3 - 1;
                const int hh = a_h[i] + dh, ww = a_w[i] + dw;
                if (hh >= 0 && hh < p.H && ww >= 0 && ww < p.W)
                  f[j] = ld1(A0 + ((long)g + dh * p.W + dw) * lda + ci);
              }
            }
            v = pack8(f);
          }
          ra[sl][i] = v;
        }
      } else {  // AM_COL (transposed): A(m,k) = A[k*lda + m], 8 consecutive m at one k
        const int kr = c % BK, cq = c / BK;
        const int k = k0 + kr, m = m0 + 8 * cq;
        const TA* src = A0 + (long)k * p.lda[0] + m;
        if (VA) {
          const bool ok = c < NCA && k < kend && m < M;
          ra[sl][i] = ld8_bf(ok ? src : A0);
          aok[sl][i] = ok;
        } else {
          uint4 v = make_uint4(0u, 0u, 0u, 0u);
          if (c < NCA && k < kend) {
            float f[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) f[j] = (m + j < M) ? ld1(src + j) : 0.f;
            v = pack8(f);
          }
          ra[sl][i] = v;
        }
      }
    }
    // ------------------------------ B ---------------------------------------
#pragma unroll
    for (int i = 0; i < NPB; ++i) {
      const int c = tid + i * GEMM_THREADS;
      bok[sl][i] = false;
      const TB* src = Bp;
      bool vec = false;  // this chunk goes through the raw (store-time) path
      uint4 v = make_uint4(0u, 0u, 0u, 0u);
      if (BMODE == BM_NT) {  // B(k,n) = B[n*ldb + k]: 8 consecutive k of row n
        const int r = c / (BK / 8), q = c % (BK / 8);
        const int n = n0 + r, k = k0 + 8 * q;
        if (VB) {
          bok[sl][i] = c < NCB && n < N && k < kend;
          src = bok[sl][i] ? Bp + (long)n * p.ldb + k : Bp;
          vec = true;
        } else if (c < NCB && n < N) {
          const TB* s0 = Bp + (long)n * p.ldb + k;
          float f[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) f[j] = (k + j < kend) ? ld1(s0 + j) : 0.f;
          v = pack8(f);
        }
      } else if (BMODE == BM_NN) {  // B(k,n) = B[k*ldb + n]: 8 consecutive n at one k
        const int kr = c % BK, cq = c / BK;
        const int k = k0 + kr, n = n0 + 8 * cq;
        if (VB) {
          bok[sl][i] = c < NCB && k < kend && n < N;
          src = bok[sl][i] ? Bp + (long)k * p.ldb + n : Bp;
          vec = true;
        } else if (c < NCB && k < kend) {
          const TB* s0 = Bp + (long)k * p.ldb + n;
          float f[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            f[j] = 0.f;
            if (n + j < N) {
              f[j] = ld1(s0 + j);
              if (PRO_B != PRO_NONE) f[j] = pro_apply<PRO_B>(f[j], bsc[i][j], bsh[i][j]);
            }
          }
          v = pack8(f);
        }
      } else {  // BM_NN_SHIFT3: B(k = pixel, n = tap*cin + ci) = X[shift_tap(k)*ldb + ci]
        const int kr = c % BK, cq = c / BK;
        const int k = k0 + kr, n = n0 + 8 * cq;
        const uint32_t qq = fdiv((uint32_t)k, p.fW);
        const int ww0 = k - (int)qq * p.W;
        const int hh0 = (int)(qq - fdiv(qq, p.fH) * p.H);
        if (VB) {  // cin % 8 == 0: the chunk shares one tap
          const int tap = (int)fdiv((uint32_t)n, p.fC);
          const int ci = n - tap * p.cin;
          const int dh = tap / 3 - 1, dw = tap - (tap / 3) * 3 - 1;
          bok[sl][i] = c < NCB && k < kend && n < N && hh0 + dh >= 0 && hh0 + dh < p.H &&
                   ww0 + dw >= 0 && ww0 + dw < p.W;
          src = bok[sl][i] ? Bp + ((long)k + dh * p.W + dw) * p.ldb + ci : Bp;
          vec = true;
        } else if (c < NCB && k < kend) {
          float f[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            f[j] = 0.f;
            const int nn = n + j;
            if (nn < N) {
              const int tap = (int)fdiv((uint32_t)nn, p.fC);
              const int ci = nn - tap * p.cin;
              const int dh = tap / 3 - 1, dw = tap - (tap / 3) * 3 - 1;
              if (hh0 + dh >= 0 && hh0 + dh < p.H && ww0 + dw >= 0 && ww0 + dw < p.W)
                f[j] = ld1(Bp + ((long)k + dh * p.W + dw) * p.ldb + ci);
            }
          }
          v = pack8(f);
        }
      }
      if (vec) {
        if constexpr (BF) {
          rbl[sl][i] = ld4((const float*)src);
          rbh[sl][i] = ld4((const float*)src + 4);
        } else {
          rb[sl][i] = *reinterpret_cast<const uint4*>(src);
        }
      } else {
        rb[sl][i] = v;
      }
    }
  };

  // the LDS image of A / B chunk i, finished from its raw staging registers
  auto a_chunk = [&](int i, int sl) -> uint4 {
    if (!VA) return ra[sl][i];
    const uint4 z = make_uint4(0u, 0u, 0u, 0u);
    if (PRO_A != PRO_NONE && AMODE == AM_ROW) {
      float f[8];
      unpack8(ra[sl][i], f);
      const float sc[8] = {asl[sl][i].x, asl[sl][i].y, asl[sl][i].z, asl[sl][i].w, asl2[sl][i].x, asl2[sl][i].y, asl2[sl][i].z, asl2[sl][i].w};
      const float sh[8] = {ash[sl][i].x, ash[sl][i].y, ash[sl][i].z, ash[sl][i].w, ash2[sl][i].x, ash2[sl][i].y, ash2[sl][i].z, ash2[sl][i].w};
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] = apro[sl][i] ? pro_apply<PRO_A>(f[j], sc[j], sh[j]) : f[j];
      return aok[sl][i] ? pack8(f) : z;
    }
    return aok[sl][i] ? ra[sl][i] : z;
  };
  auto b_chunk = [&](int i, int sl) -> uint4 {
    if (!VB) return rb[sl][i];
    const uint4 z = make_uint4(0u, 0u, 0u, 0u);
    if constexpr (BF) {
      float f[8] = {rbl[sl][i].x, rbl[sl][i].y, rbl[sl][i].z, rbl[sl][i].w, rbh[sl][i].x, rbh[sl][i].y, rbh[sl][i].z, rbh[sl][i].w};
      if (BMODE == BM_NN && PRO_B != PRO_NONE) {
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] = pro_apply<PRO_B>(f[j], bsc[i][j], bsh[i][j]);
      }
      return bok[sl][i] ? pack8(f) : z;
    } else {
      if (BMODE == BM_NN && PRO_B != PRO_NONE) {
        float f[8];
        unpack8(rb[sl][i], f);
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] = pro_apply<PRO_B>(f[j], bsc[i][j], bsh[i][j]);
        return bok[sl][i] ? pack8(f) : z;
      }
      return bok[sl][i] ? rb[sl][i] : z;
    }
  };

  auto store_tiles = [&](int buf, int sl) {
    bf16_t* as = As + buf * BM * SK;
    bf16_t* bs = Bs + buf * BN * SK;
#pragma unroll
    for (int i = 0; i < NPA; ++i) {
      const int c = tid + i * GEMM_THREADS;
      if (c < NCA) {
        const uint4 v = a_chunk(i, sl);
        if (!TRA) {
          *reinterpret_cast<uint4*>(as + (c / (BK / 8)) * SK + 8 * (c % (BK / 8))) = v;
        } else {
          const int kr = c % BK, cq = c / BK;
#pragma unroll
          for (int j = 0; j < 8; ++j) as[(8 * cq + j) * SK + kr] = u4get(v, j);
        }
      }
    }
#pragma unroll
    for (int i = 0; i < NPB; ++i) {
      const int c = tid + i * GEMM_THREADS;
      if (c < NCB) {
        const uint4 v = b_chunk(i, sl);
        if (!TRB) {
          *reinterpret_cast<uint4*>(bs + (c / (BK / 8)) * SK + 8 * (c % (BK / 8))) = v;
        } else {
          const int kr = c % BK, cq = c / BK;
#pragma unroll
          for (int j = 0; j < 8; ++j) bs[(8 * cq + j) * SK + kr] = u4get(v, j);
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

  const int am_off = (wm * TM * 32 + l31) * SK + 8 * lh;
  const int bn_off = (wn * TN * 32 + l31) * SK + 8 * lh;

  // the MFMAs of one k-tile from LDS buffer buf
  auto compute = [&](int buf) {
    const bf16_t* as = As + buf * BM * SK;
    const bf16_t* bs = Bs + buf * BN * SK;
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
      bf16x8_v a[TM], b[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i)
        a[i] = *reinterpret_cast<const bf16x8_v*>(as + am_off + i * 32 * SK + 16 * ks);
#pragma unroll
      for (int j = 0; j < TN; ++j)
        b[j] = *reinterpret_cast<const bf16x8_v*>(bs + bn_off + j * 32 * SK + 16 * ks);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
  };

  if constexpr (!PF2OK) {
    if (nkt > 0) {
      load_tiles(kstart, 0);
      store_tiles(0, 0);
      __syncthreads();
      for (int kt = 0; kt < nkt; ++kt) {
        const int buf = kt & 1;
        // unconditional (the last iteration reloads its own tile, unused): no branch
        // around the loads, so their waits are counted at the store below
        load_tiles(kstart + min(kt + 1, nkt - 1) * BK, 0);
        // keep the loads ahead of this tile's MFMAs (the scheduler would otherwise sink
        // them next to their LDS stores and expose their latency)
        __builtin_amdgcn_sched_barrier(0);
        compute(buf);
        __builtin_amdgcn_sched_barrier(0);
        if (kt + 1 < nkt) store_tiles(buf ^ 1, 0);
        __syncthreads();
      }
    }
  } else if (nkt > 0) {
    // tile t sits in staging slot t & 1 and LDS buffer t & 1; two tiles in flight
    load_tiles(kstart, 0);
    load_tiles(kstart + min(1, nkt - 1) * BK, 1);
    store_tiles(0, 0);
    __syncthreads();
    int kt = 0;
    for (; kt + 1 < nkt; kt += 2) {  // tiles kt (buffer 0) and kt + 1 (buffer 1)
      load_tiles(kstart + min(kt + 2, nkt - 1) * BK, 0);
      __builtin_amdgcn_sched_barrier(0);
      compute(0);
      __builtin_amdgcn_sched_barrier(0);
      store_tiles(1, 1);
      __syncthreads();
      load_tiles(kstart + min(kt + 3, nkt - 1) * BK, 1);
      __builtin_amdgcn_sched_barrier(0);
      compute(1);
      __builtin_amdgcn_sched_barrier(0);
      if (kt + 2 < nkt) store_tiles(0, 0);
      __syncthreads();
    }
    if (kt < nkt) compute(0);  // odd count: the last tile is already in buffer 0
  }
  gemm_epilogue<TC, EPI, WM, TM, TN>(p, acc, reinterpret_cast<float*>(smem_raw), m0, n0);
}
