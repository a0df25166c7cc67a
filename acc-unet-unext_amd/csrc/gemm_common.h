// Shared pieces of the MFMA GEMM engines (gemm_f32.h: fp32 operands on
// v_mfma_f32_32x32x2_f32; gemm_bf16.h: bf16 operands on v_mfma_f32_32x32x16_bf16):
// the parameter block, the operand prologue and the epilogue.
//
//   C[M,N] = sum_k A(m,k) * B(k,n)  (+ bias[n]) (+ nearest-upsampled adds) ,
//   with optional per-column BatchNorm partial statistics in the epilogue.
//
// Operand "modes" (reference ACC_UNet/ACC_UNet.py: 1x1 convolutions of HANCBlock /
// HANCLayer / MLFC / Conv2d_batchnorm :229-286, :77-142, :146-186, :338-527, dense
// 3x3 ResPath convolutions :290-328, their data / weight gradients):
//   A: AM_ROW    A(m,k) = A[m*lda + k]          (pixels x channels, NHWC; up to 4
//                                                 channel-concatenated sources)
//      AM_COL    A(m,k) = A[k*lda + m]          (dY^T for weight gradients)
//      AM_SHIFT3 A(m,k) = X[shift_tap(m)*lda+ci] (implicit 3x3 conv, k = tap*cin+ci,
//                                                 zero padding 1)
//   B: BM_NT     B(k,n) = B[n*ldb + k]          (weights [N][K])
//      BM_NN     B(k,n) = B[k*ldb + n]          (weights [K][N] / activations for dW)
//      BM_NN_SHIFT3 B(k=p, n=tap*cin+ci) = X[shift_tap(p)*ldb + ci]  (3x3 dW)
// Optional operand prologue y = act(x*scale[ch] + shift[ch]) applies a pending
// BatchNorm(+LeakyReLU) to A's channel axis (AM_ROW) or B's channel axis (BM_NN)
// so the normalised activation never has to be written to HBM.
// Operand / output storage: A and B are typed by the kernel (TA, TB: fp32 or bf16),
// C and every activation-shaped epilogue operand (up[], pd2/pd4, bz) by TC.
#pragma once
#include "common.h"
#include "chan.h"

enum { AM_ROW = 0, AM_COL = 1, AM_SHIFT3 = 2 };
enum { BM_NT = 0, BM_NN = 1, BM_NN_SHIFT3 = 2 };

#define GEMM_PAD 4
// cache policy (buffer aux bits: 2 = nt, 16 = sc1) of the vector epilogue's streams:
// the BatchNorm-backward input bz (read once) and the C stores
#ifndef GEMM_EPI_ZB_AUX
#define GEMM_EPI_ZB_AUX 0
#endif
#ifndef GEMM_EPI_ST_AUX
#define GEMM_EPI_ST_AUX 2
#endif
#define GEMM_THREADS 256

struct GemmParams {
  int M, N, K;
  const void* A[4];
  int lda[4];
  int kbeg[5];  // A source s covers k in [kbeg[s], kbeg[s+1])
  int nsrc;
  const float* a_scale;
  const float* a_shift;
  const void* B;
  int ldb;
  const float* b_scale;
  const float* b_shift;
  int H, W;  // pixel grid of the "pixel" operand (SHIFT3 modes, up-adds)
  FastDiv fW, fH, fC;
  int cin;  // channels per tap for the SHIFT3 modes
  void* C;
  int ldc;
  const float* bias;
  int nup;
  const void* up[3];
  int upld[3];
  int uplog[3];  // log2 of the nearest-upsample factor of each added source
  double* stats;  // [gridDim.x][2][N] fp64 partial column (sum, sumsq) of final C, or null
  // fused HANCLayer pyramid backward (see AccGemmDesc in include/accunet.h)
  const void* pd2;
  const void* pd4;
  const unsigned char* mk2;
  const unsigned char* mk4;
  // BatchNorm-backward statistics in the epilogue (see AccGemmDesc.bz)
  const void* bz;
  const float* bst;
  int bact;
  int kchunk;    // K range per blockIdx.z (split-K); >= K means no split
  size_t zstride;  // element stride between split-K partial slabs
  int evec;      // epilogue may use quad (4-element) accesses (host-checked alignment)
  int ngrp;      // N tiles per raster group (0: plain N-fastest order; see gemm_tile)
};

template <int PRO>
ACC_DEV float pro_apply(float v, float sc, float sh) {
  if (PRO == PRO_NONE) return v;
  float y = v * sc + sh;
  if (PRO == PRO_AFFINE_LRELU) y = lrelu(y);
  return y;
}

// EPI: compile-time epilogue features (bit set) so that GEMMs without them do not pay
// their registers: EPI_BNB BatchNorm-backward statistics (GemmParams.bz; data
// gradients), EPI_PYR fused HANCLayer pyramid backward (pd2/pd4), EPI_UPS
// nearest-upsampled addends (up[]). A launch whose arguments need a feature must
// use a table that has it (gemm_run checks).
enum { EPI_BNB = 1, EPI_PYR = 2, EPI_UPS = 4, EPI_STATS = 8 };  // EPI_STATS: (sum, sumsq) of C

// LDS floats the epilogue stages through (one WM*32-row pass of the BN-wide tile)
template <int WM, int TM, int TN>
constexpr int gemm_epi_floats() {
  return WM * 32 * ((4 / WM) * TN * 32 + 4);
}

// Output tile (mt, nt) of this workgroup. Split-K grids and single-column grids keep
// (blockIdx.x, blockIdx.y). Otherwise tiles run N-fastest: the N tiles of one M row
// panel are consecutive, so they share that panel of A (the pixel-sized operand; B is
// a weight panel) while it is hot. Workgroups are dealt round-robin to the 8 XCDs, so
// when the tile count is a multiple of 8 each XCD takes a contiguous run of tiles and
// an A panel is fetched into one XCD's L2 once, not once per N tile.
// ngrp > 0 (wide B: many N tiles x long K): the N tiles are cut into groups of ngrp
// and the order is group-major (M panels within a group, N-fastest inside): the B
// panels of one group stay in the XCD's L2 while every M panel passes, instead of the
// whole B being evicted by the epilogue streams and re-fetched for every M panel.
ACC_DEV void gemm_tile(int& mt, int& nt, int ngrp) {
  const int gy = gridDim.y;
  if (gridDim.z > 1 || gy == 1) {
    mt = blockIdx.x;
    nt = blockIdx.y;
    return;
  }
  const int T = gridDim.x * gy;
  int bid = blockIdx.x + gridDim.x * blockIdx.y;  // dispatch order
  if ((T & 7) == 0) bid = (bid & 7) * (T >> 3) + (bid >> 3);
  if (ngrp > 0 && ngrp < gy) {
    const int per = gridDim.x * ngrp;  // tiles of one full group
    const int g = bid / per;
    const int gn0 = g * ngrp;
    const int gw = min(ngrp, gy - gn0);
    const int r = bid - g * per;
    mt = r / gw;
    nt = gn0 + (r - mt * gw);
    return;
  }
  nt = bid % gy;
  mt = bid / gy;
}

// The epilogue shared by both engines. acc[i][j] holds this wave's 32x32 tile (i, j)
// in the MFMA C/D layout (row = (r&3) + 8*(r>>2) + 4*(lane>>5), col = lane&31; the
// same for v_mfma_f32_32x32x2_f32 and v_mfma_f32_32x32x16_bf16). smem: >=
// gemm_epi_floats<WM,TM,TN>() floats, free when called.
template <typename TC, int EPI, int WM, int TM, int TN>
ACC_DEV void gemm_epilogue_generic(const GemmParams& p, floatx16 (&acc)[TM][TN], float* smem,
                                   int m0, int n0) {
  constexpr int WN = 4 / WM;
  constexpr int BN = WN * TN * 32;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave % WM;
  const int wn = wave / WM;
  const int l31 = lane & 31;
  const int lh = lane >> 5;
  const int M = p.M, N = p.N;
  // The accumulators are staged through LDS one 32-row subtile per wave at a time
  // (pass i of TM) and re-read by a row-major thread layout: thread (rr, cq) owns
  // column quad cq of tile rows rr, rr + RPP, ... so bias / up-adds / pyramid
  // terms / stores are 16-byte, row-contiguous accesses (a tile row is BN*4 bytes
  // of one C row) and the per-column fp64 statistics stay per thread until one
  // deterministic block reduction at the end.
  constexpr int CQN = BN / 4;               // column quads per tile row
  constexpr int RPP = GEMM_THREADS / CQN;   // tile rows per sweep
  constexpr int PR = WM * 32;               // tile rows staged per pass
  constexpr int SC = BN + 4;                // LDS row stride (floats)
  constexpr int NR = PR / RPP;              // rows per thread per pass
  // rows per load chunk (more for the gather-heavy data-gradient epilogues)
  // (2-row chunks pay for the pyramid gathers of the 128-row tiles; the 64x64 small-K
  // tiles keep 1 for occupancy: tools/gemm_census.py)
  // (the BN-backward + pyramid form keeps 1: with 2 its 128x128 instance spills)
  constexpr int ECMAX = ((EPI & EPI_PYR) && !(EPI & EPI_BNB) && TM == 2) ? 2
                        : (EPI & (EPI_PYR | EPI_BNB)) ? 1 : 2;
  constexpr int EC = NR < ECMAX ? NR : ECMAX;
  static_assert(PR % RPP == 0, "pass rows must split evenly over the sweeps");
  static_assert(GEMM_THREADS % CQN == 0, "BN/4 must divide the block");
  const bool split = gridDim.z > 1;  // (split-K slabs are fp32: the host splits only TC = float)
  TC* Cout = (TC*)p.C + (split ? (size_t)blockIdx.z * p.zstride : 0);
  const int cq = tid % CQN, rr0 = tid / CQN;
  const int nq = n0 + 4 * cq;
  const bool evec = p.evec && (nq + 3 < N);
  float bq[4] = {0.f, 0.f, 0.f, 0.f};
  if (!split && p.bias) {
#pragma unroll
    for (int e = 0; e < 4; ++e) bq[e] = (nq + e < N) ? p.bias[nq + e] : 0.f;
  }
  double s1[4] = {0.0, 0.0, 0.0, 0.0}, s2[4] = {0.0, 0.0, 0.0, 0.0};
  // BatchNorm-backward statistics mode: this thread's column-quad state
  const bool bnb = (EPI & EPI_BNB) && !split && p.stats && p.bz;
  float bmu[4] = {0.f, 0.f, 0.f, 0.f}, bsc4[4] = {0.f, 0.f, 0.f, 0.f}, bsh4[4] = {0.f, 0.f, 0.f, 0.f};
  if (bnb) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int n = nq + e < N ? nq + e : N - 1;
      bmu[e] = p.bst[BN_MEAN * N + n];
      bsc4[e] = p.bst[BN_SCALE * N + n];
      bsh4[e] = p.bst[BN_SHIFT * N + n];
    }
  }
  const bool need_pix = !split && (((EPI & EPI_UPS) && p.nup > 0) || ((EPI & EPI_PYR) && p.pd2));
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    __syncthreads();  // LDS free (main loop / previous pass)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r)
        smem[(wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh) * SC + wn * TN * 32 + j * 32 + l31] =
            acc[i][j][r];
    __syncthreads();
    // rows of this pass are handled EC at a time: first every global load of the
    // chunk (nearest-up addends / pyramid terms) is issued, then the rows are combined
    // and stored, so a chunk costs one L2 round trip instead of one per row (the
    // compiler cannot hoist those loads above the previous row's C stores itself)
#pragma unroll
    for (int r0 = 0; r0 < NR; r0 += EC) {
      int mrow[EC];
      bool ok[EC];
      float v[EC][4];
      float4 zb[EC];
#pragma unroll
      for (int c = 0; c < EC; ++c) {
        const int rr = rr0 + (r0 + c) * RPP;
        mrow[c] = m0 + (rr >> 5) * TM * 32 + i * 32 + (rr & 31);
        ok[c] = (r0 + c < NR) && mrow[c] < M && nq < N;
        zb[c] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (bnb && ok[c]) {  // pre-BN input of the BatchNorm whose backward this feeds
          const TC* zr = (const TC*)p.bz + (size_t)mrow[c] * p.ldc + nq;
          if (evec) {
            zb[c] = ldq(zr);
          } else {
            float t[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) t[e] = (nq + e < N) ? ld1(zr + e) : 0.f;
            zb[c] = make_float4(t[0], t[1], t[2], t[3]);
          }
        }
        const float4 a4 = *reinterpret_cast<const float4*>(smem + (ok[c] ? rr : 0) * SC + 4 * cq);
        v[c][0] = a4.x; v[c][1] = a4.y; v[c][2] = a4.z; v[c][3] = a4.w;
        if (!split) {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[c][e] += bq[e];
        }
      }
      if ((EPI & EPI_PYR) && need_pix && p.pd2) {
        const TC* pd2 = (const TC*)p.pd2;
        const TC* pd4 = (const TC*)p.pd4;
        // fused HANCLayer pyramid backward: same accumulation order as the standalone
        // pyramid backward, g = (avg2/4 [+ max2]) + avg4/16 [+ max4]; C += g
        float4 av2[EC], mx2[EC], av4[EC], mx4[EC];
        unsigned k2[EC], k4[EC];
        int pos2[EC], pos4[EC];
#pragma unroll
        for (int c = 0; c < EC; ++c) {
          av2[c] = mx2[c] = av4[c] = mx4[c] = make_float4(0.f, 0.f, 0.f, 0.f);
          k2[c] = 0u;
          k4[c] = 0xffffffffu;
          pos2[c] = pos4[c] = 0;
          if (ok[c]) {
            const int m = mrow[c];
            const uint32_t q = fdiv((uint32_t)m, p.fW);
            const int w = m - (int)q * p.W;
            const uint32_t b = fdiv(q, p.fH);
            const int h = (int)(q - b * p.H);
            const long q2 = ((long)b * (p.H >> 1) + (h >> 1)) * (p.W >> 1) + (w >> 1);
            const long q4 = ((long)b * (p.H >> 2) + (h >> 2)) * (p.W >> 2) + (w >> 2);
            pos2[c] = (h & 1) * 2 + (w & 1);
            pos4[c] = (h & 3) * 4 + (w & 3);
            if (evec) {  // vector rows of dP, 4-byte rows of codes
              av2[c] = ldq(pd2 + q2 * 2 * N + nq);
              mx2[c] = ldq(pd2 + q2 * 2 * N + N + nq);
              k2[c] = *reinterpret_cast<const unsigned*>(p.mk2 + q2 * N + nq);
              if (p.pd4) {
                av4[c] = ldq(pd4 + q4 * 2 * N + nq);
                mx4[c] = ldq(pd4 + q4 * 2 * N + N + nq);
                k4[c] = *reinterpret_cast<const unsigned*>(p.mk4 + q4 * N + nq);
              }
            } else {
              float t[4][4];
              unsigned u2 = 0u, u4 = 0u;
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                const int n = nq + e < N ? nq + e : N - 1;
                t[0][e] = ld1(pd2 + q2 * 2 * N + n);
                t[1][e] = ld1(pd2 + q2 * 2 * N + N + n);
                u2 |= (unsigned)p.mk2[q2 * N + n] << (8 * e);
                t[2][e] = t[3][e] = 0.f;
                if (p.pd4) {
                  t[2][e] = ld1(pd4 + q4 * 2 * N + n);
                  t[3][e] = ld1(pd4 + q4 * 2 * N + N + n);
                  u4 |= (unsigned)p.mk4[q4 * N + n] << (8 * e);
                }
              }
              av2[c] = make_float4(t[0][0], t[0][1], t[0][2], t[0][3]);
              mx2[c] = make_float4(t[1][0], t[1][1], t[1][2], t[1][3]);
              av4[c] = make_float4(t[2][0], t[2][1], t[2][2], t[2][3]);
              mx4[c] = make_float4(t[3][0], t[3][1], t[3][2], t[3][3]);
              k2[c] = u2;
              k4[c] = p.pd4 ? u4 : 0xffffffffu;
            }
          }
        }
#pragma unroll
        for (int c = 0; c < EC; ++c) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            float g = f4get(av2[c], e) * 0.25f;
            if (((k2[c] >> (8 * e)) & 255u) == (unsigned)pos2[c]) g += f4get(mx2[c], e);
            if (p.pd4) {
              g += f4get(av4[c], e) * (1.f / 16.f);
              if (((k4[c] >> (8 * e)) & 255u) == (unsigned)pos4[c]) g += f4get(mx4[c], e);
            }
            v[c][e] += g;
          }
        }
      } else if ((EPI & EPI_UPS) && need_pix) {
        // nearest-upsampled addends (HANCLayer coarse branches, MLFC coarse sources),
        // added in source order
        float4 up4[EC][3];
#pragma unroll
        for (int c = 0; c < EC; ++c) {
          const int m = mrow[c];
          const uint32_t q = fdiv((uint32_t)m, p.fW);
          const int w = m - (int)q * p.W;
          const uint32_t b = fdiv(q, p.fH);
          const int h = (int)(q - b * p.H);
#pragma unroll
          for (int u = 0; u < 3; ++u) {
            up4[c][u] = make_float4(0.f, 0.f, 0.f, 0.f);
            if (u < p.nup && ok[c]) {
              const int lg = p.uplog[u];
              const long uo = (((long)b * (p.H >> lg) + (h >> lg)) * (p.W >> lg) + (w >> lg)) *
                                  p.upld[u] + nq;
              const TC* ub = (const TC*)p.up[u];
              if (evec) {
                up4[c][u] = ldq(ub + uo);
              } else {
                float t[4];
#pragma unroll
                for (int e = 0; e < 4; ++e) t[e] = (nq + e < N) ? ld1(ub + uo + e) : 0.f;
                up4[c][u] = make_float4(t[0], t[1], t[2], t[3]);
              }
            }
          }
        }
#pragma unroll
        for (int c = 0; c < EC; ++c)
#pragma unroll
          for (int u = 0; u < 3; ++u)
            if (u < p.nup) {
#pragma unroll
              for (int e = 0; e < 4; ++e) v[c][e] += f4get(up4[c][u], e);
            }
      }
#pragma unroll
      for (int c = 0; c < EC; ++c) {
        if (!ok[c]) continue;
        if (!split) {  // statistics describe the stored tensor (bf16: the rounded values)
#pragma unroll
          for (int e = 0; e < 4; ++e) v[c][e] = rnd<TC>(v[c][e]);
        }
        if (bnb) {
          // g = dC * act'(z*scale + shift); (sum g, sum g*(z - mean)) as bn_bwd_reduce_kernel
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (nq + e < N) {
              const float z = f4get(zb[c], e);
              float g = v[c][e];
              if (p.bact == ACT_LRELU) g *= lrelu_d(z * bsc4[e] + bsh4[e]);
              s1[e] += g;
              s2[e] += (double)g * ((double)z - bmu[e]);
            }
        } else if ((EPI & EPI_STATS) && !split && p.stats) {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (nq + e < N) {
              s1[e] += v[c][e];
              s2[e] += (double)v[c][e] * v[c][e];
            }
        }
        TC* dst = Cout + (size_t)mrow[c] * (split ? N : p.ldc) + nq;
        if (evec) {
          stq_nt(dst, make_float4(v[c][0], v[c][1], v[c][2], v[c][3]));  // streaming: C is not re-read by this kernel
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (nq + e < N) st1(dst + e, v[c][e]);
        }
      }
    }
  }

  if ((EPI & (EPI_STATS | EPI_BNB)) && !split && p.stats) {
    __syncthreads();  // LDS reused as the reduction buffer
    double vv[8] = {s1[0], s1[1], s1[2], s1[3], s2[0], s2[1], s2[2], s2[3]};
    if (block_slot_reduce<CQN, 8, double>(vv, reinterpret_cast<double*>(smem))) {
      // thread tid (< CQN) holds column quad tid
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int n = n0 + 4 * tid + e;
        if (n < N) {
          p.stats[((size_t)(m0 / (WM * TM * 32)) * 2 + 0) * N + n] = vv[e];
          p.stats[((size_t)(m0 / (WM * TM * 32)) * 2 + 1) * N + n] = vv[4 + e];
        }
      }
    }
  }
}

// pixel (b, h, w) of GEMM row m on the p.H x p.W grid
ACC_DEV void gemm_pix(const GemmParams& p, int m, int& b, int& h, int& w) {
  const uint32_t q = fdiv((uint32_t)m, p.fW);
  w = m - (int)q * p.W;
  const uint32_t bb = fdiv(q, p.fH);
  h = (int)(q - bb * p.H);
  b = (int)bb;
}
// index of the pixel that covers (b, h, w) on the grid downsampled by 2^lg
ACC_DEV long gemm_pix_lg(const GemmParams& p, int b, int h, int w, int lg) {
  return ((long)b * (p.H >> lg) + (h >> lg)) * (p.W >> lg) + (w >> lg);
}

// The epilogue operands of one C row quad, raw as loaded (unused members are dead)
template <typename TC>
struct EpiRow {
  typedef typename QuadRaw<TC>::type R;
  R zb;                  // EPI_BNB: pre-BN input
  R av2, mx2, av4, mx4;  // EPI_PYR: pyramid gradients
  unsigned k2, k4;       // EPI_PYR: argmax codes
  R up[3];               // EPI_UPS: nearest-upsampled addends
};

// Vector epilogue (p.evec, no split-K): the same arithmetic as gemm_epilogue_generic,
// with every global access a branch-free buffer load / store (lanes and rows that
// are masked off use out-of-range offsets; absent operands get zero-size
// descriptors). The exact instruction count lets the compiler wait for one chunk's
// operand loads alone, and the loads of chunk t+1 are issued before chunk t is
// stored, so neither the C stores nor the next chunk's gathers are ever drained
// by a vmcnt(0) (the generic path pays about one L2/HBM round trip per chunk).
// Descriptors cover one block's rows (wave-uniform bases from m0), so tensors of
// any size stay within 32-bit offsets.
#ifndef GEMM_PYR_EC
#define GEMM_PYR_EC 1
#endif
template <typename TC, int EPI, int WM, int TM, int TN>
ACC_DEV void gemm_epilogue_vec(const GemmParams& p, floatx16 (&acc)[TM][TN], float* smem, int m0,
                               int n0) {
  constexpr int WN = 4 / WM;
  constexpr int BN = WN * TN * 32;
  constexpr int BM = WM * TM * 32;
  constexpr int CQN = BN / 4;
  constexpr int RPP = GEMM_THREADS / CQN;
  constexpr int PR = WM * 32;
  constexpr int SC = BN + 4;
  constexpr int NR = PR / RPP;
  constexpr bool LOADS = (EPI & (EPI_BNB | EPI_PYR | EPI_UPS)) != 0;
  // rows per chunk; two chunks of operands in flight (the BN-backward + pyramid epilogue
  // gathers 6 operands per row: one row per chunk keeps it within 3 waves per SIMD)
  // pyramid data gradient (EPI_PYR): a thread's rows come in horizontal pixel pairs
  // (w even, w + 1: tile rows 2k, 2k + 1, since m0 and W are even), which share their
  // 2x2 and 4x4 windows, so each pair issues ONE set of pyramid gathers (6 loads)
  // beside its two BN-backward rows
  constexpr bool PAIR = (EPI & EPI_PYR) != 0;
  constexpr int EC = PAIR ? 2 : ((EPI & EPI_PYR) && (EPI & EPI_BNB)) ? GEMM_PYR_EC : LOADS ? 2 : NR;
  constexpr int NCH = NR / EC;
  constexpr int NT = TM * NCH;        // chunks of the whole tile
  constexpr int SZ = (int)sizeof(TC);
  static_assert(NR % EC == 0, "chunks must split the pass rows");
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave % WM;
  const int wn = wave / WM;
  const int l31 = lane & 31;
  const int lh = lane >> 5;
  const int M = p.M, N = p.N, ldc = p.ldc;
  const int cq = tid % CQN, rr0 = tid / CQN;
  const int nq = n0 + 4 * cq;
  const int mlast = min(M, m0 + BM) - 1;
  const unsigned rows = (unsigned)(mlast - m0 + 1);
  const __amdgpu_buffer_rsrc_t rC = acc_rsrc((const TC*)p.C + (size_t)m0 * ldc, rows * ldc * SZ);
  float bq[4] = {0.f, 0.f, 0.f, 0.f};
  if (p.bias) {
#pragma unroll
    for (int e = 0; e < 4; ++e) bq[e] = (nq + e < N) ? p.bias[nq + e] : 0.f;
  }
  // ---- operand descriptors (block-local bases) -----------------------------
  const bool bnb = (EPI & EPI_BNB) && p.stats && p.bz;
  __amdgpu_buffer_rsrc_t rZ = rC, rP2 = rC, rK2 = rC, rP4 = rC, rK4 = rC, rU[3] = {rC, rC, rC};
  long q2a = 0, q4a = 0, ua[3] = {0, 0, 0};
  if (EPI & EPI_BNB)
    rZ = acc_rsrc(bnb ? (const TC*)p.bz + (size_t)m0 * ldc : (const TC*)p.C,
                  bnb ? rows * ldc * SZ : 0u);
  if (EPI & (EPI_PYR | EPI_UPS)) {
    int ba, ha, wa, bb, hb, wb;
    gemm_pix(p, m0, ba, ha, wa);
    gemm_pix(p, mlast, bb, hb, wb);
    if (EPI & EPI_PYR) {
      const bool on2 = p.pd2 != nullptr, on4 = on2 && p.pd4 != nullptr;
      q2a = gemm_pix_lg(p, ba, ha, wa, 1);
      q4a = gemm_pix_lg(p, ba, ha, wa, 2);
      const unsigned n2 = (unsigned)(gemm_pix_lg(p, bb, hb, wb, 1) - q2a + 1);
      const unsigned n4 = (unsigned)(gemm_pix_lg(p, bb, hb, wb, 2) - q4a + 1);
      rP2 = acc_rsrc(on2 ? (const TC*)p.pd2 + q2a * 2 * N : (const TC*)p.C, on2 ? n2 * 2 * N * SZ : 0u);
      rK2 = acc_rsrc(on2 ? p.mk2 + q2a * N : p.mk2, on2 ? n2 * N : 0u);
      rP4 = acc_rsrc(on4 ? (const TC*)p.pd4 + q4a * 2 * N : (const TC*)p.C, on4 ? n4 * 2 * N * SZ : 0u);
      rK4 = acc_rsrc(on4 ? p.mk4 + q4a * N : p.mk2, on4 ? n4 * N : 0u);
    }
    if (EPI & EPI_UPS) {
#pragma unroll
      for (int u = 0; u < 3; ++u) {
        const bool on = u < p.nup;
        const int lg = on ? p.uplog[u] : 0;
        ua[u] = gemm_pix_lg(p, ba, ha, wa, lg);
        const unsigned nu = (unsigned)(gemm_pix_lg(p, bb, hb, wb, lg) - ua[u] + 1);
        rU[u] = acc_rsrc(on ? (const TC*)p.up[u] + ua[u] * p.upld[u] : (const TC*)p.C,
                         on ? nu * p.upld[u] * SZ : 0u);
      }
    }
  }
  float bmu[4] = {0.f, 0.f, 0.f, 0.f}, bsc4[4] = {0.f, 0.f, 0.f, 0.f}, bsh4[4] = {0.f, 0.f, 0.f, 0.f};
  if (bnb) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int n = nq + e < N ? nq + e : N - 1;
      bmu[e] = p.bst[BN_MEAN * N + n];
      bsc4[e] = p.bst[BN_SCALE * N + n];
      bsh4[e] = p.bst[BN_SHIFT * N + n];
    }
  }
  // tile row (of the pass's PR rows) of chunk t's row c
  auto tile_row = [&](int t, int c) {
    return PAIR ? 2 * (rr0 + (t % NCH) * RPP) + c : rr0 + ((t % NCH) * EC + c) * RPP;
  };
  // rows of chunk t (pass t / NCH): C row and in-range flag of its row c
  auto row_of = [&](int t, int c, int& m) {
    const int i = t / NCH;
    const int rr = tile_row(t, c);
    m = m0 + (rr >> 5) * TM * 32 + i * 32 + (rr & 31);
    return m < M && nq < N;
  };
  auto issue = [&](EpiRow<TC> (&L)[EC], int t) {
#pragma unroll
    for (int c = 0; c < EC; ++c) {
      int m;
      const bool ok = row_of(t, c, m);
      if (EPI & EPI_BNB)
        L[c].zb = bufq_ld<GEMM_EPI_ZB_AUX>(rZ, ok ? (unsigned)(((m - m0) * ldc + nq) * SZ) : ACC_OOB, (const TC*)nullptr);
      if (EPI & (EPI_PYR | EPI_UPS)) {
        int b, h, w;
        gemm_pix(p, ok ? m : m0, b, h, w);
        if ((EPI & EPI_PYR) && c == 0) {  // (PAIR: row c = 1 shares row 0's windows)
          const unsigned i2 = (unsigned)(gemm_pix_lg(p, b, h, w, 1) - q2a);
          const unsigned i4 = (unsigned)(gemm_pix_lg(p, b, h, w, 2) - q4a);
          const unsigned o2 = ok ? (i2 * 2 * N + nq) * SZ : ACC_OOB;
          const unsigned o4 = ok ? (i4 * 2 * N + nq) * SZ : ACC_OOB;
          L[c].av2 = bufq_ld<0>(rP2, o2, (const TC*)nullptr);
          L[c].mx2 = bufq_ld<0>(rP2, o2 + N * SZ, (const TC*)nullptr);
          L[c].k2 = __builtin_amdgcn_raw_buffer_load_b32(rK2, ok ? i2 * N + nq : ACC_OOB, 0, 0);
          L[c].av4 = bufq_ld<0>(rP4, o4, (const TC*)nullptr);
          L[c].mx4 = bufq_ld<0>(rP4, o4 + N * SZ, (const TC*)nullptr);
          L[c].k4 = __builtin_amdgcn_raw_buffer_load_b32(rK4, ok ? i4 * N + nq : ACC_OOB, 0, 0);
        }
        if (EPI & EPI_UPS) {
#pragma unroll
          for (int u = 0; u < 3; ++u) {
            const int lg = u < p.nup ? p.uplog[u] : 0;
            const unsigned iu = (unsigned)(gemm_pix_lg(p, b, h, w, lg) - ua[u]);
            L[c].up[u] = bufq_ld<0>(rU[u], ok ? (iu * p.upld[u] + nq) * SZ : ACC_OOB,
                                    (const TC*)nullptr);
          }
        }
      }
    }
  };
  double s1[4] = {0.0, 0.0, 0.0, 0.0}, s2[4] = {0.0, 0.0, 0.0, 0.0};
  EpiRow<TC> L[2][EC];
  if (LOADS) issue(L[0], 0);
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int i = t / NCH;
    if (t % NCH == 0) {
      __syncthreads();  // LDS free (main loop / previous pass)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          smem[(wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh) * SC + wn * TN * 32 + j * 32 + l31] =
              acc[i][j][r];
      __syncthreads();
    }
    if (LOADS && t + 1 < NT) issue(L[(t + 1) & 1], t + 1);
    EpiRow<TC>(&R)[EC] = L[t & 1];
#pragma unroll
    for (int c = 0; c < EC; ++c) {
      int m;
      const bool ok = row_of(t, c, m);
      const int rr = tile_row(t, c);
      const float4 a4 = *reinterpret_cast<const float4*>(smem + rr * SC + 4 * cq);
      float v[4] = {a4.x + bq[0], a4.y + bq[1], a4.z + bq[2], a4.w + bq[3]};
      if ((EPI & EPI_PYR) && p.pd2) {
        {
          int b, h, w;
          gemm_pix(p, ok ? m : m0, b, h, w);
          const unsigned pos2 = (h & 1) * 2 + (w & 1), pos4 = (h & 3) * 4 + (w & 3);
          const EpiRow<TC>& G = R[0];  // the pair's windows
          const float4 av2 = q2f(G.av2), mx2 = q2f(G.mx2);
          const float4 av4 = q2f(G.av4), mx4 = q2f(G.mx4);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            float g = f4get(av2, e) * 0.25f;
            if (((G.k2 >> (8 * e)) & 255u) == pos2) g += f4get(mx2, e);
            if (p.pd4) {
              g += f4get(av4, e) * (1.f / 16.f);
              if (((G.k4 >> (8 * e)) & 255u) == pos4) g += f4get(mx4, e);
            }
            v[e] += g;
          }
        }
      } else if (EPI & EPI_UPS) {
#pragma unroll
        for (int u = 0; u < 3; ++u)
          if (u < p.nup) {
            const float4 a = q2f(R[c].up[u]);
            v[0] += a.x; v[1] += a.y; v[2] += a.z; v[3] += a.w;
          }
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = rnd<TC>(v[e]);  // statistics of the stored values
      if (ok) {
        if (bnb) {
          const float4 z4 = q2f(R[c].zb);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float z = f4get(z4, e);
            float g = v[e];
            if (p.bact == ACT_LRELU) g *= lrelu_d(z * bsc4[e] + bsh4[e]);
            s1[e] += g;
            s2[e] += (double)g * ((double)z - bmu[e]);
          }
        } else if ((EPI & EPI_STATS) && p.stats) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            s1[e] += v[e];
            s2[e] += (double)v[e] * v[e];
          }
        }
      }
      bufq_st<GEMM_EPI_ST_AUX>(rC, ok ? (unsigned)(((m - m0) * ldc + nq) * SZ) : ACC_OOB,
                 make_float4(v[0], v[1], v[2], v[3]), (TC*)nullptr);
    }
  }
  if ((EPI & (EPI_STATS | EPI_BNB)) && p.stats) {
    __syncthreads();  // LDS reused as the reduction buffer
    double vv[8] = {s1[0], s1[1], s1[2], s1[3], s2[0], s2[1], s2[2], s2[3]};
    if (block_slot_reduce<CQN, 8, double>(vv, reinterpret_cast<double*>(smem))) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int n = n0 + 4 * tid + e;
        if (n < N) {
          p.stats[((size_t)(m0 / (WM * TM * 32)) * 2 + 0) * N + n] = vv[e];
          p.stats[((size_t)(m0 / (WM * TM * 32)) * 2 + 1) * N + n] = vv[4 + e];
        }
      }
    }
  }
}

template <typename TC, int EPI, int WM, int TM, int TN>
ACC_DEV void gemm_epilogue(const GemmParams& p, floatx16 (&acc)[TM][TN], float* smem, int m0,
                           int n0) {
  if (p.evec && gridDim.z == 1)
    gemm_epilogue_vec<TC, EPI, WM, TM, TN>(p, acc, smem, m0, n0);
  else
    gemm_epilogue_generic<TC, EPI, WM, TM, TN>(p, acc, smem, m0, n0);
}
