// Large-kernel depthwise convolution (stride 1, groups = C, any kh x kw up to 31),
// NCHW fp32: the reference's native extension kernels/dwconv2d
// (dwconv2d.cpp:14-28 bindings, depthwise_fwd/launch.cu:12-80 launchers,
// depthwise_fwd/kernel.cuh:77-120 tile fill), re-designed for gfx950, plus the
// backward the reference leaves unbound (dwconv2d.cpp:30-52 are commented out, so
// its DepthwiseFunction.backward, Dwconv/dwconv_layer.py:20-31, cannot run).
//
// Padding: `replicate` selects the reference's own kernel semantics (the tile fill
// clamps the source row / column into the image, kernel.cuh:104-115, with the
// window bounded by pad_h in both directions); replicate = 0 is zero padding, which
// the reference launchers use for 3 x 3 kernels (launch.cu:28-35 without bias and
// padding 1, :61-66 with bias: cudnn_convolution / at::conv2d). The host layer
// (accunet/dwconv2d.py) applies that dispatch rule.
//   out[n,c,oh,ow] = bias[c] + sum_{i,j} w[c,i,j] * x[n,c, src(oh - ph + i), src(ow - pw + j)]
//   with oH = H - kh + 1 + 2 ph, oW = W - kw + 1 + 2 pw (launch.cu:22-23).
//
// Forward: a 256-thread block owns TH output rows of one (n, c) plane and stages
// the padded input window ((TH + kh - 1) x (oW + kw - 1)) and the kernel in LDS;
// each thread computes 4 consecutive outputs of a row from a register window slid
// along the row. Data gradient: the same kernel correlates dy with the flipped
// kernel (the gradient of the padded input), then a fold kernel sums the padded
// border back onto the image pixels it was clamped from. Weight / bias gradients:
// per-(n, c, row-tile) partials over the staged windows, one thread per (tap, row
// group), reduced in a fixed order by a second kernel (deterministic, no float
// atomics).
#include "common.h"

#define DWK_MAXK 31
#define DWK_LDS_FLOATS 14336  // 56 KB of staged window per block (at most)
// square kernels up to 7 x 7 stage row tiles of at most 24 KB, so several blocks share
// a CU (the 64 x 64 planes of the reference benchmark: 32-row tiles, 17 KB for k = 3)
#define DWK_LDS_SMALL 6144

struct DwkGeom {
  int N, C, H, W, kh, kw, ph, pw, oH, oW;
  int replicate;  // 1: clamp source indices, 0: zero outside the image
  int TH;         // output rows per block
  int tilesH;
  int lds;        // floats of dynamic LDS: window (TH + kh - 1) x ldw + the wgrad dy rows
  int ldw;        // window row stride: ncol = oW + kw - 1 rounded up to 1 mod 4, so the 4
                  // rows of 16 quads a wave reads sit in different bank residues
};

ACC_DEV float dwk_src(const float* __restrict__ plane, const DwkGeom& g, int r, int c) {
  if (g.replicate) {
    // the reference bounds the replicate window by pad_h in BOTH directions
    // (copy_src(param.pad_h), kernel.cuh:104,186): beyond it the tile holds 0
    if (r < -g.ph || r >= g.H + g.ph || c < -g.ph || c >= g.W + g.ph) return 0.f;
    r = min(max(r, 0), g.H - 1);
    c = min(max(c, 0), g.W - 1);
    return plane[(long)r * g.W + c];
  }
  if (r < 0 || r >= g.H || c < 0 || c >= g.W) return 0.f;
  return plane[(long)r * g.W + c];
}

// stage rows [r0 - ph, r0 - ph + nr) x cols [-pw, -pw + ncol) of the padded input (row
// stride g.ldw): one
// wave per window row (row source and validity computed once per row, no per-element
// division), 4 rows in flight per block
ACC_DEV void dwk_stage(float* __restrict__ s, const float* __restrict__ plane, const DwkGeom& g,
                       int r0, int nr, int ncol) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int lim = g.replicate ? g.ph : 0;  // replicate window bound (rows and columns)
  // source row of window row rr (clamped / zero outside), as an offset and a flag
  auto src_row = [&](int rr, bool& rok) -> long {
    int r = r0 - g.ph + rr;
    if (g.replicate) {
      rok = rr < nr && r >= -lim && r < g.H + lim;
      r = min(max(r, 0), g.H - 1);
    } else {
      rok = rr < nr && r >= 0 && r < g.H;
    }
    return (long)(rok ? r : 0) * g.W;
  };
  auto src_col = [&](int cc, bool& ok) -> int {
    int c = cc - g.pw;
    if (g.replicate) {
      ok = ok && cc < ncol && c >= -lim && c < g.W + lim;
      c = min(max(c, 0), g.W - 1);
    } else {
      ok = ok && cc < ncol && c >= 0 && c < g.W;
    }
    return ok ? c : 0;
  };
  if (ncol <= 128) {
    // every load of RB rows x 2 column slots issued before the LDS stores (the staging is
    // latency-bound: one round trip per RB rows instead of one per row)
    constexpr int RB = 4;
    for (int rb = wv; rb < nr; rb += 4 * RB) {
      float v[RB][2];
      bool ok[RB][2];
#pragma unroll
      for (int b = 0; b < RB; ++b) {
        bool rok;
        const long ro = src_row(rb + 4 * b, rok);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          ok[b][h] = rok;
          const int c = src_col(lane + 64 * h, ok[b][h]);
          v[b][h] = plane[ro + c];
        }
      }
#pragma unroll
      for (int b = 0; b < RB; ++b)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int rr = rb + 4 * b, cc = lane + 64 * h;
          if (rr < nr && cc < ncol) s[rr * g.ldw + cc] = ok[b][h] ? v[b][h] : 0.f;
        }
    }
    return;
  }
  for (int rr = wv; rr < nr; rr += 4) {
    bool rok;
    const long ro = src_row(rr, rok);
    float* dst = s + rr * g.ldw;
    for (int cc = lane; cc < ncol; cc += 64) {
      bool ok = rok;
      const int c = src_col(cc, ok);
      dst[cc] = ok ? plane[ro + c] : 0.f;
    }
  }
}

// KT > 0: square KT x KT kernel known at compile time (unrolled window, the reference's
// benchmark sizes 3 / 7 / 13 / 31); KT = 0: any kh x kw. Same arithmetic order in both:
// acc = bias, then fma over kernel rows i, columns j.
template <int KT>
__global__ void __launch_bounds__(256)
dwk_fwd_kernel(const float* __restrict__ x, const float* __restrict__ w,
               const float* __restrict__ bias, float* __restrict__ out, DwkGeom g, int flip) {
  extern __shared__ float win[];  // g.lds floats (dynamic)
  __shared__ float wk[DWK_MAXK * DWK_MAXK];
  const int kh = KT ? KT : g.kh, kw = KT ? KT : g.kw;
  const int plane_id = blockIdx.y;  // n * C + c
  const int c = plane_id % g.C;
  const int r0 = blockIdx.x * g.TH;
  const int nrow = min(g.TH, g.oH - r0);
  const int ncol = g.oW + kw - 1;
  const float* xp = x + (long)plane_id * g.H * g.W;
  dwk_stage(win, xp, g, r0, nrow + kh - 1, ncol);
  const int nt = kh * kw;
  for (int e = threadIdx.x; e < nt; e += blockDim.x) wk[e] = w[(long)c * nt + (flip ? nt - 1 - e : e)];
  __syncthreads();
  const float b = bias ? bias[c] : 0.f;
  const int qpr = (g.oW + 3) / 4;  // 4-output groups per row
  float* op = out + (long)plane_id * g.oH * g.oW;
  for (int t = threadIdx.x; t < nrow * qpr; t += blockDim.x) {
    const int r = t / qpr, c4 = (t - r * qpr) * 4;
    float acc[4] = {b, b, b, b};
    if (KT) {
      // the window row holds ncol >= c4 + KT + 3 floats past c4 except in the last group
      // of a row (oW % 4 != 0): those reads stay inside the LDS buffer and only feed
      // outputs that are not stored
      // kernel rows unrolled only for small kernels (KT >= 7 would hold every row's
      // window in registers at once and spill)
#pragma unroll KT <= 5 ? KT : 1
      for (int i = 0; i < KT; ++i) {
        const float* row = win + (r + i) * g.ldw + c4;
        float v[KT + 3];
#pragma unroll
        for (int j = 0; j < KT + 3; ++j) v[j] = row[j];
#pragma unroll
        for (int j = 0; j < KT; ++j) {
          const float kk = wk[i * KT + j];
          acc[0] = fmaf(kk, v[j], acc[0]);
          acc[1] = fmaf(kk, v[j + 1], acc[1]);
          acc[2] = fmaf(kk, v[j + 2], acc[2]);
          acc[3] = fmaf(kk, v[j + 3], acc[3]);
        }
      }
    } else {
      for (int i = 0; i < kh; ++i) {
        const float* row = win + (r + i) * g.ldw + c4;
        float v0 = row[0], v1 = (c4 + 1 < ncol) ? row[1] : 0.f, v2 = (c4 + 2 < ncol) ? row[2] : 0.f;
        for (int j = 0; j < kw; ++j) {
          const float v3 = (c4 + j + 3 < ncol) ? row[j + 3] : 0.f;
          const float kk = wk[i * kw + j];
          acc[0] = fmaf(kk, v0, acc[0]);
          acc[1] = fmaf(kk, v1, acc[1]);
          acc[2] = fmaf(kk, v2, acc[2]);
          acc[3] = fmaf(kk, v3, acc[3]);
          v0 = v1; v1 = v2; v2 = v3;
        }
      }
    }
    float* o = op + (long)(r0 + r) * g.oW + c4;
    if (c4 + 3 < g.oW && ((((long)(r0 + r) * g.oW + c4) & 3) == 0) && ((uintptr_t)op & 15) == 0) {
      *reinterpret_cast<float4*>(o) = make_float4(acc[0], acc[1], acc[2], acc[3]);
    } else {
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (c4 + u < g.oW) o[u] = acc[u];
    }
  }
}

// square odd kernels 3..31 (the reference benchmark's sizes, test.py) run compile-time
// unrolled kernels; ACCUNET_DWK_GENERIC=1 forces the generic loops (A/B knob)
static bool dwk_square_on() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("ACCUNET_DWK_GENERIC");
    v = (e && atoi(e)) ? 0 : 1;
  }
  return v != 0;
}

// LDS floats of dwk_wgrad_part_tpl<K>'s pixel-group partials
static int dwk_red_floats(int K) {
  const int KI = K <= 5 ? 1 : K;
  return (256 / KI) * (K * K + 1);
}

// launch the forward / flipped correlation for geometry g (kernel size from g)
static void dwk_fwd_launch(const float* x, const float* w, const float* bias, float* out,
                           const DwkGeom& g, int flip, hipStream_t s) {
  const dim3 grid(g.tilesH, g.N * g.C);
  auto go = [&](auto kfn) {
    hipLaunchKernelGGL(kfn, grid, dim3(256), (size_t)g.lds * 4, s, x, w, bias, out, g, flip);
  };
  if (g.kh != g.kw || !dwk_square_on()) go(dwk_fwd_kernel<0>);
#define DWK_F(K) else if (g.kh == K) go(dwk_fwd_kernel<K>);
  DWK_F(3) DWK_F(5) DWK_F(7) DWK_F(9) DWK_F(11) DWK_F(13) DWK_F(15) DWK_F(17) DWK_F(19)
  DWK_F(21) DWK_F(23) DWK_F(25) DWK_F(27) DWK_F(29) DWK_F(31)
#undef DWK_F
  else go(dwk_fwd_kernel<0>);
}

// Data gradient = the adjoint of "pad (replicate or zero), then correlate":
//   1. the full correlation of dy with the flipped kernel gives the gradient of the
//      padded input, gp[L] for L in [-ph, H-1+ph] x [-pw, W-1+pw] (dwk_fwd_kernel on
//      dy with flip = 1 and zero padding kh-1 / kw-1);
//   2. replicate: fold gp back onto the image, dx[h][w] = sum of gp[L] over the L
//      that clamp onto (h, w) — [-lim, 0] onto 0, [n-1, n-1+lim] onto n-1 with
//      lim = pad_h (the reference's window bound, also for columns) — zero padding
//      needs no fold (step 1 then writes dx directly with padding kh-1-ph, kw-1-pw).
ACC_DEV void dwk_fold_range(int s, int n, int lim, int* lo, int* hi) {
  *lo = s;
  *hi = s;
  if (s == 0) *lo = -lim;
  if (s == n - 1) *hi = n - 1 + lim;
}

__global__ void __launch_bounds__(256)
dwk_fold_kernel(const float* __restrict__ gp, float* __restrict__ dx, DwkGeom g) {
  const long total = (long)g.N * g.C * g.H * g.W;
  const long e = blockIdx.x * 256L + threadIdx.x;
  if (e >= total) return;
  const long pl = e / ((long)g.H * g.W);
  const int h = (int)((e / g.W) % g.H), w = (int)(e % g.W);
  const int PH = g.H + 2 * g.ph, PW = g.W + 2 * g.pw;
  const float* gpp = gp + pl * PH * PW;
  int h0, h1, w0, w1;
  dwk_fold_range(h, g.H, g.replicate ? g.ph : 0, &h0, &h1);
  dwk_fold_range(w, g.W, g.replicate ? g.ph : 0, &w0, &w1);
  h0 = max(h0, -g.ph); h1 = min(h1, g.H - 1 + g.ph);
  w0 = max(max(w0, -g.pw), -g.ph); w1 = min(min(w1, g.W - 1 + g.pw), g.W - 1 + g.ph);
  float acc = 0.f;
  for (int a = h0; a <= h1; ++a)
    for (int b = w0; b <= w1; ++b) acc += gpp[(long)(a + g.ph) * PW + (b + g.pw)];
  dx[e] = acc;
}

// partials[(n * tilesH + tile) * C + c][kh*kw + 1]: sum over the tile's outputs of
// dy * x_shifted per tap, and sum dy (bias)
__global__ void __launch_bounds__(256)
dwk_wgrad_part_kernel(const float* __restrict__ x, const float* __restrict__ dy,
                      float* __restrict__ part, DwkGeom g) {
  extern __shared__ float win[];  // g.lds floats (dynamic)
  const int plane_id = blockIdx.y;
  const int n = plane_id / g.C, c = plane_id % g.C;
  const int r0 = blockIdx.x * g.TH;
  const int nrow = min(g.TH, g.oH - r0);
  const int ncol = g.oW + g.kw - 1;
  const float* xp = x + (long)plane_id * g.H * g.W;
  const float* dp = dy + (long)plane_id * g.oH * g.oW + (long)r0 * g.oW;
  dwk_stage(win, xp, g, r0, nrow + g.kh - 1, ncol);
  float* dys = win + (nrow + g.kh - 1) * g.ldw;  // the tile's dy rows after the window
  for (int e = threadIdx.x; e < nrow * g.oW; e += blockDim.x) dys[e] = dp[e];
  __syncthreads();
  const int ntap = g.kh * g.kw;
  float* pr = part + ((long)(n * g.tilesH + blockIdx.x) * g.C + c) * (ntap + 1);
  // thread = (tap, row group): RG row groups share a tap when there are few taps
  const int T1 = ntap + 1;
  const int RG = T1 >= 256 ? 1 : 256 / T1;
  __shared__ float red[256];
  for (int tb = 0; tb < T1; tb += 256 / RG) {
    const int tl = threadIdx.x % (256 / RG), rg = threadIdx.x / (256 / RG);
    const int tap = tb + tl;
    float s = 0.f;
    if (tap < T1 && rg < RG) {
      if (tap == ntap) {
        for (int r = rg; r < nrow; r += RG)
          for (int q = 0; q < g.oW; ++q) s += dys[r * g.oW + q];
      } else {
        const int i = tap / g.kw, j = tap - i * g.kw;
        for (int r = rg; r < nrow; r += RG) {
          const float* xr = win + (r + i) * g.ldw + j;
          const float* dr = dys + r * g.oW;
          for (int q = 0; q < g.oW; ++q) s = fmaf(dr[q], xr[q], s);
        }
      }
    }
    red[threadIdx.x] = s;
    __syncthreads();
    if (rg == 0 && tap < T1) {
      float t = 0.f;
      for (int k = 0; k < RG; ++k) t += red[k * (256 / RG) + tl];  // fixed order
      pr[tap] = t;
    }
    __syncthreads();
  }
}

// Square KT x KT kernels: the same partials, pixel-parallel. Thread (i-group, pg) owns
// output quads pg, pg + PG, ... of the tile and accumulates, for kernel rows i of its
// group (all KT rows when KT <= 5, else row i = its group), the KT taps of each row as
// sum over its quads of dy[q..q+3] . x[q+j..q+j+3] (+ sum dy for the bias); the PG
// pixel-group partials are then summed per tap in pixel-group order (deterministic).
template <int KT>
__global__ void __launch_bounds__(256)
dwk_wgrad_part_tpl(const float* __restrict__ x, const float* __restrict__ dy,
                   float* __restrict__ part, DwkGeom g) {
  constexpr int KI = KT <= 5 ? 1 : KT;  // kernel-row groups
  constexpr int PG = 256 / KI;          // pixel groups
  constexpr int RPT = KT <= 5 ? KT : 1; // kernel rows per thread
  constexpr int NT1 = KT * KT + 1;
  static_assert(PG * NT1 <= DWK_LDS_FLOATS, "partials fit the staging buffer");
  extern __shared__ float win[];  // max(g.lds, PG * NT1) floats (dynamic, dwk_red_floats)
  const int plane_id = blockIdx.y;
  const int n = plane_id / g.C, c = plane_id % g.C;
  const int r0 = blockIdx.x * g.TH;
  const int nrow = min(g.TH, g.oH - r0);
  const int ncol = g.oW + KT - 1;
  const float* xp = x + (long)plane_id * g.H * g.W;
  const float* dp = dy + (long)plane_id * g.oH * g.oW + (long)r0 * g.oW;
  dwk_stage(win, xp, g, r0, nrow + KT - 1, ncol);
  float* dys = win + (nrow + KT - 1) * g.ldw;  // the tile's dy rows after the window
  for (int e = threadIdx.x; e < nrow * g.oW; e += blockDim.x) dys[e] = dp[e];
  __syncthreads();
  const int grp = threadIdx.x / PG, pg = threadIdx.x - grp * PG;
  const bool act = grp < KI;
  const int i0 = KI == 1 ? 0 : grp;
  float acc[RPT][KT];
#pragma unroll
  for (int a = 0; a < RPT; ++a)
#pragma unroll
    for (int j = 0; j < KT; ++j) acc[a][j] = 0.f;
  float bsum = 0.f;
  const int qpr = (g.oW + 3) / 4;
  if (act) {
    for (int t = pg; t < nrow * qpr; t += PG) {
      const int r = t / qpr, c4 = (t - r * qpr) * 4;
      float d[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) d[u] = (c4 + u < g.oW) ? dys[r * g.oW + c4 + u] : 0.f;
      bsum += ((d[0] + d[1]) + d[2]) + d[3];
#pragma unroll
      for (int a = 0; a < RPT; ++a) {
        const float* row = win + (r + i0 + a) * g.ldw + c4;
        float v[KT + 3];
#pragma unroll
        for (int j = 0; j < KT + 3; ++j) v[j] = (c4 + j < ncol) ? row[j] : 0.f;
#pragma unroll
        for (int j = 0; j < KT; ++j) {
          float s = acc[a][j];
          s = fmaf(d[0], v[j], s);
          s = fmaf(d[1], v[j + 1], s);
          s = fmaf(d[2], v[j + 2], s);
          s = fmaf(d[3], v[j + 3], s);
          acc[a][j] = s;
        }
      }
    }
  }
  __syncthreads();  // the window is dead: reuse it for the pixel-group partials
  float* red = win;
  if (act) {
#pragma unroll
    for (int a = 0; a < RPT; ++a)
#pragma unroll
      for (int j = 0; j < KT; ++j) red[pg * NT1 + (i0 + a) * KT + j] = acc[a][j];
    if (grp == 0) red[pg * NT1 + KT * KT] = bsum;
  }
  __syncthreads();
  float* pr = part + ((long)(n * g.tilesH + blockIdx.x) * g.C + c) * NT1;
  for (int tap = threadIdx.x; tap < NT1; tap += 256) {
    float t = 0.f;
    for (int k = 0; k < PG; ++k) t += red[k * NT1 + tap];  // fixed order
    pr[tap] = t;
  }
}

// dw[c][tap] = sum over (n, tile) in order; db[c] likewise
__global__ void __launch_bounds__(256)
dwk_wgrad_sum_kernel(const float* __restrict__ part, float* __restrict__ dw,
                     float* __restrict__ db, DwkGeom g) {
  const int ntap = g.kh * g.kw;
  const long e = blockIdx.x * 256L + threadIdx.x;
  if (e >= (long)g.C * (ntap + 1)) return;
  const int c = (int)(e / (ntap + 1)), tap = (int)(e % (ntap + 1));
  double s = 0.0;
  for (int k = 0; k < g.N * g.tilesH; ++k) s += part[((long)k * g.C + c) * (ntap + 1) + tap];
  if (tap < ntap) dw[(long)c * ntap + tap] = (float)s;
  else if (db) db[c] = (float)s;
}

static int dwk_geom(int N, int C, int H, int W, int kh, int kw, int ph, int pw, int replicate,
                    DwkGeom* g) {
  if (N <= 0 || C <= 0 || H <= 0 || W <= 0 || kh <= 0 || kw <= 0 || kh > DWK_MAXK ||
      kw > DWK_MAXK || ph < 0 || pw < 0)
    return ACC_EBADSHAPE;
  g->N = N; g->C = C; g->H = H; g->W = W; g->kh = kh; g->kw = kw; g->ph = ph; g->pw = pw;
  g->oH = H - kh + 1 + 2 * ph;
  g->oW = W - kw + 1 + 2 * pw;
  if (g->oH <= 0 || g->oW <= 0) return ACC_EBADSHAPE;
  g->replicate = replicate ? 1 : 0;
  const int ncol = g->oW + kw - 1;
  const int ld = ncol + ((1 - ncol) & 3);  // ncol <= ld, ld % 4 == 1
  g->ldw = ld;
  // window rows (TH + kh - 1) * ld + the wgrad dy rows TH * oW must fit the LDS buffer
  const int cap = (kh == kw && kh <= 7 && dwk_square_on()) ? DWK_LDS_SMALL : DWK_LDS_FLOATS;
  int th = (cap - (kh - 1) * ld) / (ld + g->oW);
  if (th < 1) th = (DWK_LDS_FLOATS - (kh - 1) * ld) / (ld + g->oW);  // wide rows
  if (th < 1) return ACC_EBADSHAPE;  // a row wider than the staging buffer
  g->TH = th < g->oH ? th : g->oH;
  g->tilesH = ceil_div(g->oH, g->TH);
  g->TH = ceil_div(g->oH, g->tilesH);  // balanced tiles (64 rows at <= 45 per tile: 2 x 32)
  g->lds = (g->TH + kh - 1) * ld + g->TH * g->oW;
  return ACC_OK;
}

extern "C" int accunet_dwconvk_out_hw(int H, int W, int kh, int kw, int ph, int pw, int* oH,
                                      int* oW) {
  DwkGeom g;
  int rc = dwk_geom(1, 1, H, W, kh, kw, ph, pw, 1, &g);
  if (rc) return rc;
  *oH = g.oH;
  *oW = g.oW;
  return ACC_OK;
}

extern "C" int accunet_dwconvk_fwd(const float* x, const float* w, const float* bias, float* out,
                                   int N, int C, int H, int W, int kh, int kw, int ph, int pw,
                                   int replicate, void* stream) {
  DwkGeom g;
  int rc = dwk_geom(N, C, H, W, kh, kw, ph, pw, replicate, &g);
  if (rc) return rc;
  dwk_fwd_launch(x, w, bias, out, g, 0, (hipStream_t)stream);
  return hipGetLastError() == hipSuccess ? ACC_OK : ACC_ELAUNCH;
}

extern "C" size_t accunet_dwconvk_dgrad_ws(int N, int C, int H, int W, int kh, int kw, int ph,
                                           int pw, int replicate) {
  if (!replicate && ph <= kh - 1 && pw <= kw - 1) return 0;  // direct path, no fold
  return (size_t)N * C * (H + 2 * ph) * (W + 2 * pw);
}

extern "C" int accunet_dwconvk_dgrad(const float* dy, const float* w, float* dx, int N, int C,
                                     int H, int W, int kh, int kw, int ph, int pw, int replicate,
                                     float* ws, size_t ws_elems, void* stream) {
  DwkGeom g;
  int rc = dwk_geom(N, C, H, W, kh, kw, ph, pw, replicate, &g);
  if (rc) return rc;
  hipStream_t s = (hipStream_t)stream;
  // correlate dy (oH x oW) with the flipped kernel, zero padding
  DwkGeom t;
  if (!replicate && ph <= kh - 1 && pw <= kw - 1) {
    // zero padding: straight into dx, output H x W with padding kh-1-ph, kw-1-pw
    rc = dwk_geom(N, C, g.oH, g.oW, kh, kw, kh - 1 - ph, kw - 1 - pw, 0, &t);
    if (rc) return rc;
    dwk_fwd_launch(dy, w, nullptr, dx, t, 1, s);
    return hipGetLastError() == hipSuccess ? ACC_OK : ACC_ELAUNCH;
  }
  if (ws_elems < accunet_dwconvk_dgrad_ws(N, C, H, W, kh, kw, ph, pw, replicate)) return ACC_EBADARG;
  rc = dwk_geom(N, C, g.oH, g.oW, kh, kw, kh - 1, kw - 1, 0, &t);  // -> (H+2ph) x (W+2pw)
  if (rc) return rc;
  dwk_fwd_launch(dy, w, nullptr, ws, t, 1, s);
  const long total = (long)N * C * H * W;
  hipLaunchKernelGGL(dwk_fold_kernel, dim3((unsigned)ceil_div(total, 256)), dim3(256), 0, s, ws, dx,
                     g);
  return hipGetLastError() == hipSuccess ? ACC_OK : ACC_ELAUNCH;
}

extern "C" size_t accunet_dwconvk_wgrad_ws(int N, int C, int H, int W, int kh, int kw, int ph,
                                           int pw) {
  DwkGeom g;
  if (dwk_geom(N, C, H, W, kh, kw, ph, pw, 1, &g)) return 0;
  return (size_t)N * g.tilesH * C * (kh * kw + 1);
}

extern "C" int accunet_dwconvk_wgrad(const float* x, const float* dy, float* dw, float* db, int N,
                                     int C, int H, int W, int kh, int kw, int ph, int pw,
                                     int replicate, float* ws, size_t ws_elems, void* stream) {
  DwkGeom g;
  int rc = dwk_geom(N, C, H, W, kh, kw, ph, pw, replicate, &g);
  if (rc) return rc;
  if (ws_elems < (size_t)N * g.tilesH * C * (kh * kw + 1)) return ACC_EBADARG;
  hipStream_t s = (hipStream_t)stream;
  const dim3 grid(g.tilesH, N * C);
  auto part = [&](auto kfn, int red) {
    const int f = g.lds > red ? g.lds : red;
    hipLaunchKernelGGL(kfn, grid, dim3(256), (size_t)f * 4, s, x, dy, ws, g);
  };
  if (kh != kw || !dwk_square_on()) part(dwk_wgrad_part_kernel, 0);
#define DWK_W(K) else if (kh == K) part(dwk_wgrad_part_tpl<K>, dwk_red_floats(K));
  DWK_W(3) DWK_W(5) DWK_W(7) DWK_W(9) DWK_W(11) DWK_W(13) DWK_W(15) DWK_W(17) DWK_W(19)
  DWK_W(21) DWK_W(23) DWK_W(25) DWK_W(27) DWK_W(29) DWK_W(31)
#undef DWK_W
  else part(dwk_wgrad_part_kernel, 0);
  hipLaunchKernelGGL(dwk_wgrad_sum_kernel, dim3((unsigned)ceil_div((long)C * (kh * kw + 1), 256)),
                     dim3(256), 0, s, ws, dw, db, g);
  return hipGetLastError() == hipSuccess ? ACC_OK : ACC_ELAUNCH;
}
