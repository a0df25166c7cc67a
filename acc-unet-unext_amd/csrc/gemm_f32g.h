// fp32 MFMA GEMM engine with LDS-DMA staging: the forward 1x1 convolutions
// (AM_ROW x BM_NT, both operands k-contiguous, vector-aligned), which gemm_f32.h's
// register-staged kernel runs at about half MFMA occupancy.
//
//   * operand tiles go global -> LDS by global_load_lds_dwordx4 (no VGPR staging,
//     no transposing ds_writes), into a GG_STAGES-deep ring: tiles kt+1 .. kt+3 are in
//     flight while tile kt is computed; each wave waits for its own DMA of tile kt with a counted
//     s_waitcnt vmcnt(N) and one raw s_barrier per k-tile publishes it (no
//     __syncthreads in the loop: its implied vmcnt(0) would drain the ring);
//   * LDS image = the global tile, lane-linear per DMA instruction, [row][16 k] with
//     the 16-B chunk index XOR-swizzled by (row >> 2) & 3 through the per-lane SOURCE
//     address, so the fragment reads (ds_read_b128, 32 rows x one chunk per half-wave)
//     are bank-conflict free;
//   * v_mfma_f32_32x32x2_f32 consumes k in pairs (lanes 0-31 / 32-63); a lane reads 4
//     consecutive k of its row (chunk 2j + half) and feeds them to 4 successive MFMAs,
//     so MFMA step (j, t) pairs k = 8j + t with k = 8j + 4 + t. A and B use the same
//     pairing, so the sum over k is the same set of products (fp32 fma chain in a
//     different k order than gemm_f32.h: within the parity tolerances);
//   * the pending-BatchNorm prologue of A (PRO_A) is applied to the fragments after
//     the LDS read, from per-stage coefficient chunks staged by the same DMA.
// Out-of-range rows / k chunks load a zero page. Epilogue: gemm_common.h.
#pragma once
#include "gemm_common.h"

#define GG_BK 16
// ring depth: GG_STAGES - 1 k-tiles (16 k each) in flight ahead of the one computed.
// 3 stages of 16.5 KB (128x128 tiles) keep 3 workgroups per CU in LDS; 4 stages keep 2,
// the same k-tiles in flight per CU, and measured 1-3 % slower per GEMM family
// (profiles/r03_step_ab.txt), so 3 is the default.
#ifndef GG_STAGES
#define GG_STAGES 3
#endif
// narrow tiles (128x32: 8 MFMAs per wave and k-tile, 10 KB per stage) run a deeper ring,
// so the k-tiles in flight per CU cover the load latency (A/B knob)
#ifndef GG_STAGES_NARROW
#define GG_STAGES_NARROW 3
#endif

static __device__ __attribute__((aligned(16))) float g_gemm_zero16[4];

// One LDS-DMA instruction: lane i copies 16 B from its `src` to lds_dst + 16 i
// (lds_dst wave-uniform). Issued from inline asm, so hipcc neither counts it nor
// guards later ds_reads of the same array with vmcnt(0) (it cannot tell the ring
// buffers apart and would drain the pipeline every k-tile): the kernel waits for its
// DMA itself (gg_wait_vm) before the barrier that publishes a stage.
ACC_DEV void gg_dma16(const float* src, float* lds_dst) {
  const unsigned dst = __builtin_amdgcn_readfirstlane(
      (unsigned)(size_t)(__attribute__((address_space(3))) float*)lds_dst);
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(src), "s"(dst)
               : "memory");
}

// s_waitcnt vmcnt(N) with every other counter left alone (gfx9 encoding)
template <int N>
ACC_DEV void gg_wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

// s_waitcnt vmcnt(ahead * GPW) for a run-time ahead in [0, MAXA]
template <int GPW, int MAXA>
ACC_DEV void gg_wait_ahead(int ahead) {
  if constexpr (MAXA > 0) {
    if (ahead >= MAXA) { gg_wait_vm<MAXA * GPW>(); return; }
    gg_wait_ahead<GPW, MAXA - 1>(ahead);
  } else {
    gg_wait_vm<0>();
  }
}

// LDS image of one operand tile (R = BM or BN):
//   k-contiguous (AM_ROW, AM_SHIFT3, BM_NT): [R][16] floats, row r's 16-B chunk c at
//     position c ^ ((r >> 2) & 3)
//   k-major (AM_COL, BM_NN, BM_NN_SHIFT3): [16][R] floats, row k's element x at
//     x ^ kmaj_swz(k): rows k and k+4 (the two half-waves of one MFMA step) then sit in
//     opposite bank halves (R >= 64; a 32-wide row keeps a 2-way conflict)
template <int R>
ACC_DEV int kmaj_swz(int k) { return R >= 64 ? ((k >> 2) & 1) << 5 : 0; }

#ifndef GG_PYR_WAVES
#define GG_PYR_WAVES 3
#endif
template <int AMODE, int BMODE, int PRO_A, int PRO_B, int WM, int TM, int TN, int EPI>
__global__ void __launch_bounds__(GEMM_THREADS)
__attribute__((amdgpu_waves_per_eu(((EPI & EPI_PYR) && (EPI & EPI_BNB)) ? GG_PYR_WAVES : 1)))
gemm_f32g_kernel(const GemmParams p) {
  constexpr int WN = 4 / WM;
  constexpr int BM = WM * TM * 32;
  constexpr int BN = WN * TN * 32;
  constexpr int BK = GG_BK;
  constexpr bool AKC = AMODE != AM_COL;  // A k-contiguous
  constexpr bool BKC = BMODE == BM_NT;   // B k-contiguous
  constexpr int AF = BM * BK, BF = BN * BK;              // floats per stage and operand
  constexpr int CF = (AMODE == AM_ROW && PRO_A != PRO_NONE) ? 2 * BK : 0;  // A prologue
  constexpr int SF = AF + BF + CF;
  constexpr int STG = BN == 32 ? GG_STAGES_NARROW : GG_STAGES;
  constexpr int RING = STG * SF;
  constexpr int EPF = gemm_epi_floats<WM, TM, TN>();
  constexpr int LDS_F = RING > EPF ? RING : EPF;
  // 16-B pieces per wave and stage (BK = 16): A: BM, B: BN
  constexpr int PWA = AF / 16, PWB = BF / 16;
  constexpr int IA = (PWA + 63) / 64, IB = (PWB + 63) / 64, IC = CF ? 1 : 0;
  constexpr int GPW = IA + IB + IC;  // DMA instructions per wave and stage
  static_assert(BK == 16, "the chunk swizzle assumes 4 chunks per row");
  static_assert(STG >= 2 && STG <= 8, "the vmcnt ladder covers up to 7 tiles ahead");
  static_assert((STG - 2) * GPW < 64, "vmcnt range");
  static_assert(PWA % 64 == 0 || PWA < 64, "A pieces per wave");
  static_assert(PWB % 64 == 0 || PWB < 64, "B pieces per wave");
  static_assert(PRO_A == PRO_NONE || AMODE == AM_ROW, "A prologue: row-major A only");
  static_assert(PRO_B == PRO_NONE || BMODE == BM_NN, "B prologue: BM_NN only");

  __shared__ __attribute__((aligned(16))) float smem[LDS_F];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
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
  const int kb1 = p.nsrc > 1 ? p.kbeg[1] : K;  // end of source 0 (the prologue's channels)
  const float* Bp = (const float*)p.B;
  const float* zp = g_gemm_zero16;

  // ---- source address of one 16-B piece (zero page when out of range) ---------
  // A, k-contiguous: tile row r (= m0 + r), k chunk at k
  auto a_src_kc = [&](int r, int k) -> const float* {
    const int g = m0 + r;
    if (AMODE == AM_SHIFT3) {  // implicit 3x3: k = tap*cin + ci (cin % 4 == 0)
      const uint32_t q = fdiv((uint32_t)g, p.fW);
      const int w = g - (int)q * p.W;
      const int h = (int)(q - fdiv(q, p.fH) * p.H);
      const int tap = (int)fdiv((uint32_t)k, p.fC);
      const int ci = k - tap * p.cin;
      const int dh = tap / 3 - 1, dw = tap - (tap / 3) * 3 - 1;
      const bool ok = g < M && k < kend && h + dh >= 0 && h + dh < p.H && w + dw >= 0 &&
                      w + dw < p.W;
      return ok ? (const float*)p.A[0] + ((long)g + dh * p.W + dw) * p.lda[0] + ci : zp;
    }
    const float* base = (const float*)p.A[0];
    int ld = p.lda[0], kb = 0;
    if (p.nsrc > 1) {
      if (k >= p.kbeg[1]) { base = (const float*)p.A[1]; ld = p.lda[1]; kb = p.kbeg[1]; }
      if (p.nsrc > 2 && k >= p.kbeg[2]) { base = (const float*)p.A[2]; ld = p.lda[2]; kb = p.kbeg[2]; }
      if (p.nsrc > 3 && k >= p.kbeg[3]) { base = (const float*)p.A[3]; ld = p.lda[3]; kb = p.kbeg[3]; }
    }
    const bool ok = g < M && k < kend;
    return ok ? base + (long)g * ld + (k - kb) : zp;
  };
  // A, k-major (AM_COL): row k, columns m0 + x .. +3
  auto a_src_km = [&](int k, int x) -> const float* {
    const int m = m0 + x;
    const bool ok = k < kend && m < M;
    return ok ? (const float*)p.A[0] + (long)k * p.lda[0] + m : zp;
  };
  // B, k-contiguous (BM_NT): tile row n0 + r, k chunk at k
  auto b_src_kc = [&](int r, int k) -> const float* {
    const int n = n0 + r;
    const bool ok = n < N && k < kend;
    return ok ? Bp + (long)n * p.ldb + k : zp;
  };
  // B, k-major: row k, columns n0 + x .. +3
  auto b_src_km = [&](int k, int x) -> const float* {
    const int n = n0 + x;
    if (BMODE == BM_NN_SHIFT3) {  // B(k = pixel, n = tap*cin + ci) = X[shift_tap(k)][ci]
      const uint32_t q = fdiv((uint32_t)k, p.fW);
      const int w = k - (int)q * p.W;
      const int h = (int)(q - fdiv(q, p.fH) * p.H);
      const int tap = (int)fdiv((uint32_t)n, p.fC);
      const int ci = n - tap * p.cin;
      const int dh = tap / 3 - 1, dw = tap - (tap / 3) * 3 - 1;
      const bool ok = k < kend && n < N && h + dh >= 0 && h + dh < p.H && w + dw >= 0 &&
                      w + dw < p.W;
      return ok ? Bp + ((long)k + dh * p.W + dw) * p.ldb + ci : zp;
    }
    const bool ok = k < kend && n < N;
    return ok ? Bp + (long)k * p.ldb + n : zp;
  };

  // ---- one stage of DMA: this wave's pieces of A, B (and the coefficients) ----
  auto stage = [&](int kt, int buf) {
    const int k0 = kstart + kt * BK;
    float* sA = smem + buf * SF;
    float* sB = sA + AF;
#pragma unroll
    for (int ii = 0; ii < IA; ++ii) {
      const int q = wave * PWA + ii * 64 + lane;
      const float* src;
      if (AKC) {  // piece q: row q/4, LDS chunk position q%4
        const int r = q >> 2;
        src = a_src_kc(r, k0 + 4 * ((q & 3) ^ ((r >> 2) & 3)));
      } else {    // piece q: row q/(BM/4), LDS column quad q%(BM/4)
        const int kr = q / (BM / 4);
        src = a_src_km(k0 + kr, ((q % (BM / 4)) * 4) ^ kmaj_swz<BM>(kr));
      }
      if (PWA >= 64 || lane < PWA) gg_dma16(src, sA + (wave * PWA + ii * 64) * 4);
    }
#pragma unroll
    for (int ii = 0; ii < IB; ++ii) {
      const int q = wave * PWB + ii * 64 + lane;
      const float* src;
      if (BKC) {
        const int r = q >> 2;
        src = b_src_kc(r, k0 + 4 * ((q & 3) ^ ((r >> 2) & 3)));
      } else {
        const int kr = q / (BN / 4);
        src = b_src_km(k0 + kr, ((q % (BN / 4)) * 4) ^ kmaj_swz<BN>(kr));
      }
      if (PWB >= 64 || lane < PWB) gg_dma16(src, sB + (wave * PWB + ii * 64) * 4);
    }
    if (CF) {  // wave w stages coefficient chunks 2w, 2w+1: scale[0..15] | shift[0..15]
      const int e = 2 * wave + (lane & 1);
      const int k = k0 + 4 * (e & 3);
      const bool ok = k < kend && k < kb1;
      const float* src = ok ? ((e < 4) ? p.a_scale : p.a_shift) + k : zp;
      if (lane < 2) gg_dma16(src, sB + BF + 2 * wave * 4);
    }
  };

  floatx16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // fragment rows / columns of this lane (tile-local)
  int ar[TM], br[TN];
#pragma unroll
  for (int i = 0; i < TM; ++i) ar[i] = wm * TM * 32 + i * 32 + l31;
#pragma unroll
  for (int j = 0; j < TN; ++j) br[j] = wn * TN * 32 + j * 32 + l31;
  // BM_NN prologue: per-column coefficients of this lane's TN columns
  float bsc[TN], bsh[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    bsc[j] = 1.f;
    bsh[j] = 0.f;
    if (PRO_B != PRO_NONE) {
      const int n = min(n0 + br[j], N - 1);
      bsc[j] = p.b_scale[n];
      bsh[j] = p.b_shift[n];
    }
  }

  auto compute = [&](int kt, int buf) {
    const float* sA = smem + buf * SF;
    const float* sB = sA + AF;
    const int k0 = kstart + kt * BK;
#pragma unroll
    for (int j = 0; j < BK / 8; ++j) {
      const int c = 2 * j + lh;  // this half-wave's k chunk: k = 4c + t at MFMA step t
      float av[TM][4], bv[TN][4];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        if (AKC) {
          const float4 f = *reinterpret_cast<const float4*>(sA + ar[i] * BK + ((c ^ ((ar[i] >> 2) & 3)) << 2));
          av[i][0] = f.x; av[i][1] = f.y; av[i][2] = f.z; av[i][3] = f.w;
        } else {
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            const int kr = 4 * c + t;
            av[i][t] = sA[kr * BM + (ar[i] ^ kmaj_swz<BM>(kr))];
          }
        }
      }
#pragma unroll
      for (int jn = 0; jn < TN; ++jn) {
        if (BKC) {
          const float4 f = *reinterpret_cast<const float4*>(sB + br[jn] * BK + ((c ^ ((br[jn] >> 2) & 3)) << 2));
          bv[jn][0] = f.x; bv[jn][1] = f.y; bv[jn][2] = f.z; bv[jn][3] = f.w;
        } else {
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            const int kr = 4 * c + t;
            float v = sB[kr * BN + (br[jn] ^ kmaj_swz<BN>(kr))];
            // (rows past kend are zero in A, so the prologue of a zero B row is harmless)
            if (PRO_B != PRO_NONE) v = pro_apply<PRO_B>(v, bsc[jn], bsh[jn]);
            bv[jn][t] = v;
          }
        }
      }
      if (CF) {
        const float4 sc = *reinterpret_cast<const float4*>(sB + BF + 4 * c);
        const float4 sh = *reinterpret_cast<const float4*>(sB + BF + 16 + 4 * c);
        if (k0 + 4 * c < kb1) {
#pragma unroll
          for (int i = 0; i < TM; ++i) {
            av[i][0] = pro_apply<PRO_A>(av[i][0], sc.x, sh.x);
            av[i][1] = pro_apply<PRO_A>(av[i][1], sc.y, sh.y);
            av[i][2] = pro_apply<PRO_A>(av[i][2], sc.z, sh.z);
            av[i][3] = pro_apply<PRO_A>(av[i][3], sc.w, sh.w);
          }
        }
      }
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int jn = 0; jn < TN; ++jn)
            acc[i][jn] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[i][t], bv[jn][t], acc[i][jn], 0,
                                                             0, 0);
    }
  };

  constexpr int D = STG - 1;  // k-tiles in flight ahead of the computed one
  if (nkt > 0) {
#pragma unroll
    for (int s = 0; s < D; ++s)
      if (s < nkt) stage(s, s);
    for (int kt = 0; kt < nkt; ++kt) {
      // this wave's DMA of tile kt has landed (the up to D-1 later tiles may still be
      // in flight: their GPW instructions each are the newest in the counter) ...
      const int ahead = min(D - 1, nkt - 1 - kt);
      gg_wait_ahead<GPW, D - 1>(ahead);
      // ... and so has every wave's once all pass the barrier; the barrier also
      // retires every read of the buffer that tile kt+D overwrites (computed at kt-1)
      __builtin_amdgcn_s_barrier();
      if (kt + D < nkt) stage(kt + D, (kt + D) % STG);
      compute(kt, kt % STG);
    }
  }
  gemm_epilogue<float, EPI, WM, TM, TN>(p, acc, smem, m0, n0);
}
