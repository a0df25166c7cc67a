// fp32 MFMA GEMM engine for every convolution on the ACC-UNet path.
//
//   C[M,N] = sum_k A(m,k) * B(k,n)  (+ bias[n]) (+ nearest-upsampled adds) ,
//   with optional per-column BatchNorm partial statistics in the epilogue.
//
// The 1x1 convolutions of HANCBlock / HANCLayer / MLFC / Conv2d_batchnorm
// (reference ACC_UNet/ACC_UNet.py:229-286, :77-142, :146-186, :338-527), the
// dense 3x3 ResPath convolutions (:290-328) and their data / weight gradients
// all map onto this one kernel through operand "modes":
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
//
// Matrix core: v_mfma_f32_32x32x2_f32 (exact fp32 fma chain, 64 cyc/SIMD), 4 waves
// (64-wide) per 256-thread workgroup laid out WM x WN, each wave owning TM x TN
// 32x32 accumulator tiles (16 regs each). K is staged 16 at a time through a
// double-buffered, padded, k-major LDS image so every MFMA operand read is a
// conflict-free ds_read_b32 (lanes 0-31 and 32-63 sit in different bank groups).
#pragma once
#include "common.h"
#include "chan.h"

enum { AM_ROW = 0, AM_COL = 1, AM_SHIFT3 = 2 };
enum { BM_NT = 0, BM_NN = 1, BM_NN_SHIFT3 = 2 };

#define GEMM_BK 16
#define GEMM_PAD 4
#define GEMM_THREADS 256

struct GemmParams {
  int M, N, K;
  const float* A[4];
  int lda[4];
  int kbeg[5];  // A source s covers k in [kbeg[s], kbeg[s+1])
  int nsrc;
  const float* a_scale;
  const float* a_shift;
  const float* B;
  int ldb;
  const float* b_scale;
  const float* b_shift;
  int H, W;  // pixel grid of the "pixel" operand (SHIFT3 modes, up-adds)
  FastDiv fW, fH, fC;
  int cin;  // channels per tap for the SHIFT3 modes
  float* C;
  int ldc;
  const float* bias;
  int nup;
  const float* up[3];
  int upld[3];
  int uplog[3];  // log2 of the nearest-upsample factor of each added source
  double* stats;  // [gridDim.x][2][N] fp64 partial column (sum, sumsq) of final C, or null
  // fused HANCLayer pyramid backward (see AccGemmDesc in include/accunet.h)
  const float* pd2;
  const float* pd4;
  const unsigned char* mk2;
  const unsigned char* mk4;
  // BatchNorm-backward statistics in the epilogue (see AccGemmDesc.bz)
  const float* bz;
  const float* bst;
  int bact;
  int kchunk;    // K range per blockIdx.z (split-K); >= K means no split
  size_t zstride;  // element stride between split-K partial slabs
  int evec;      // epilogue may use 16-byte accesses (host-checked alignment)
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

  const int m0 = blockIdx.x * BM;
  const int n0 = blockIdx.y * BN;
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

  float4 ra[NPA], rb[NPB];
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

  auto load_tiles = [&](int k0) {
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
              const float* base = p.A[0];
              int ld = p.lda[0], kb = 0;
              if (p.nsrc > 1) {
                if (k >= p.kbeg[1]) { base = p.A[1]; ld = p.lda[1]; kb = p.kbeg[1]; }
                if (p.nsrc > 2 && k >= p.kbeg[2]) { base = p.A[2]; ld = p.lda[2]; kb = p.kbeg[2]; }
                if (p.nsrc > 3 && k >= p.kbeg[3]) { base = p.A[3]; ld = p.lda[3]; kb = p.kbeg[3]; }
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
                float x = p.A[s][(long)g * p.lda[s] + (kk - p.kbeg[s])];
                if (PRO_A != PRO_NONE && s == 0) x = pro_apply<PRO_A>(x, p.a_scale[kk], p.a_shift[kk]);
                e[jj] = x;
              }
            }
            v = make_float4(e[0], e[1], e[2], e[3]);
          }
        }
        ra[i] = v;
      }
    } else if (AMODE == AM_SHIFT3) {
      // implicit 3x3: k = tap*cin + ci; zero padding outside the image
      const float* Ab = p.A[0];
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
        ra[i] = v;
      }
    } else {  // AM_COL: A(m,k) = A[k*lda + m]
      const float* Ab = p.A[0];
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
        ra[i] = v;
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
          const float* ptr = p.B + (long)n * p.ldb + k;
          if (VB) {
            if (k < kend) v = ld4(ptr);
          } else {
            if (k + 0 < kend) v.x = ptr[0];
            if (k + 1 < kend) v.y = ptr[1];
            if (k + 2 < kend) v.z = ptr[2];
            if (k + 3 < kend) v.w = ptr[3];
          }
        }
        rb[i] = v;
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
          const float* ptr = p.B + (long)k * p.ldb + n;
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
        rb[i] = v;
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
                v = ld4(p.B + ((long)k + dh * p.W + dw) * p.ldb + ci);
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
                  e[j] = p.B[((long)k + dh * p.W + dw) * p.ldb + ci];
              }
            }
            v = make_float4(e[0], e[1], e[2], e[3]);
          }
        }
        rb[i] = v;
      }
    }
  };

  auto store_tiles = [&](int buf) {
    float* as = As + buf * BK * SA;
    float* bs = Bs + buf * BK * SB;
    if (AMODE == AM_COL) {
#pragma unroll
      for (int i = 0; i < NPA; ++i) {
        int idx = tid + i * GEMM_THREADS;
        if (idx < NA4) {
          int kr = idx / (BM / 4), q = idx % (BM / 4);
          st4(as + kr * SA + 4 * q, ra[i]);
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < NPA; ++i) {
        int idx = tid + i * GEMM_THREADS;
        if (idx < NA4) {
          int r = idx / QPR, q = idx % QPR;
          as[(4 * q + 0) * SA + r] = ra[i].x;
          as[(4 * q + 1) * SA + r] = ra[i].y;
          as[(4 * q + 2) * SA + r] = ra[i].z;
          as[(4 * q + 3) * SA + r] = ra[i].w;
        }
      }
    }
    if (BMODE == BM_NT) {
#pragma unroll
      for (int i = 0; i < NPB; ++i) {
        int idx = tid + i * GEMM_THREADS;
        if (idx < NB4) {
          int r = idx / QPR, q = idx % QPR;
          bs[(4 * q + 0) * SB + r] = rb[i].x;
          bs[(4 * q + 1) * SB + r] = rb[i].y;
          bs[(4 * q + 2) * SB + r] = rb[i].z;
          bs[(4 * q + 3) * SB + r] = rb[i].w;
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < NPB; ++i) {
        int idx = tid + i * GEMM_THREADS;
        if (idx < NB4) {
          int kr = idx / (BN / 4), q = idx % (BN / 4);
          st4(bs + kr * SB + 4 * q, rb[i]);
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
    load_tiles(kstart);
    store_tiles(0);
    __syncthreads();
    for (int kt = 0; kt < nkt; ++kt) {
      const int buf = kt & 1;
      if (kt + 1 < nkt) load_tiles(kstart + (kt + 1) * BK);
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
      if (kt + 1 < nkt) store_tiles(buf ^ 1);
      __syncthreads();
    }
  }

  // ------------------------------- epilogue ---------------------------------
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
  constexpr int ECMAX = ((EPI & EPI_PYR) && TM == 2) ? 2 : (EPI & (EPI_PYR | EPI_BNB)) ? 1 : 2;
  constexpr int EC = NR < ECMAX ? NR : ECMAX;
  static_assert(PR % RPP == 0, "pass rows must split evenly over the sweeps");
  static_assert(PR * SC <= 2 * BK * SA + 2 * BK * SB, "epilogue staging exceeds the LDS tile");
  static_assert(GEMM_THREADS % CQN == 0, "BN/4 must divide the block");
  const bool split = gridDim.z > 1;
  float* Cout = split ? p.C + (size_t)blockIdx.z * p.zstride : p.C;
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
          const float* zr = p.bz + (size_t)mrow[c] * p.ldc + nq;
          if (evec) {
            zb[c] = ld4(zr);
          } else {
            float t[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) t[e] = (nq + e < N) ? zr[e] : 0.f;
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
            if (evec) {  // 16-byte rows of dP, 4-byte rows of codes
              av2[c] = ld4(p.pd2 + q2 * 2 * N + nq);
              mx2[c] = ld4(p.pd2 + q2 * 2 * N + N + nq);
              k2[c] = *reinterpret_cast<const unsigned*>(p.mk2 + q2 * N + nq);
              if (p.pd4) {
                av4[c] = ld4(p.pd4 + q4 * 2 * N + nq);
                mx4[c] = ld4(p.pd4 + q4 * 2 * N + N + nq);
                k4[c] = *reinterpret_cast<const unsigned*>(p.mk4 + q4 * N + nq);
              }
            } else {
              float t[4][4];
              unsigned u2 = 0u, u4 = 0u;
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                const int n = nq + e < N ? nq + e : N - 1;
                t[0][e] = p.pd2[q2 * 2 * N + n];
                t[1][e] = p.pd2[q2 * 2 * N + N + n];
                u2 |= (unsigned)p.mk2[q2 * N + n] << (8 * e);
                t[2][e] = t[3][e] = 0.f;
                if (p.pd4) {
                  t[2][e] = p.pd4[q4 * 2 * N + n];
                  t[3][e] = p.pd4[q4 * 2 * N + N + n];
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
              if (evec) {
                up4[c][u] = ld4(p.up[u] + uo);
              } else {
                float t[4];
#pragma unroll
                for (int e = 0; e < 4; ++e) t[e] = (nq + e < N) ? p.up[u][uo + e] : 0.f;
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
        float* dst = Cout + (size_t)mrow[c] * (split ? N : p.ldc) + nq;
        if (evec) {
          st4_nt(dst, make_float4(v[c][0], v[c][1], v[c][2], v[c][3]));  // streaming: C is not re-read by this kernel
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (nq + e < N) dst[e] = v[c][e];
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
          p.stats[((size_t)blockIdx.x * 2 + 0) * N + n] = vv[e];
          p.stats[((size_t)blockIdx.x * 2 + 1) * N + n] = vv[4 + e];
        }
      }
    }
  }
}
