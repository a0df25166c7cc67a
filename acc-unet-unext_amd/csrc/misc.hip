// Head, loss and optimizer kernels on the training step.
//
//  - head: 1x1 conv n_filts -> 1 (+bias) with optional Sigmoid
//    (ACC_UNet.out / last_activation, ACC_UNet/ACC_UNet.py:594-599,653-659).
//  - WeightedDiceBCE(dice 0.5, BCE 0.5) forward/backward
//    (Experiments/utils.py:21-74 WeightedBCE, :109-138 WeightedDiceLoss,
//    :140-171 WeightedDiceBCE) on the logits [B, N].
//  - Adam (torch.optim.Adam, lr 1e-3, betas (0.9, 0.999), eps 1e-8, no weight decay;
//    Experiments/train_model.py:647) as one multi-tensor launch over every parameter.
#include "common.h"
#include "chan.h"
#include "kernels.h"
#include <stdlib.h>

// ---------------------------------------------------------------------------
// head
// ---------------------------------------------------------------------------
// Forward: TQ = C/4 lanes per pixel (a power of two <= 64) each load one 16-byte
// channel quad (coalesced rows), dot with w, xor-shuffle sum over the TQ lanes.
template <typename T>
__global__ void __launch_bounds__(256)
head_fwd_kernel(const T* __restrict__ x, const float* __restrict__ w, const float* __restrict__ b,
                int sigm, float* __restrict__ y, long P, int C, int TQ) {
  const int q = threadIdx.x % TQ;
  const int ppb = 256 / TQ;  // pixels per block sweep
  const float4 wq = ld4(w + 4 * q);
  const float bias = b[0];
  for (long p = (long)blockIdx.x * ppb + threadIdx.x / TQ; p < P; p += (long)gridDim.x * ppb) {
    const float4 xv = ldq(x + p * C + 4 * q);
    float acc = xv.x * wq.x;
    acc = fmaf(xv.y, wq.y, acc);
    acc = fmaf(xv.z, wq.z, acc);
    acc = fmaf(xv.w, wq.w, acc);
    for (int off = 1; off < TQ; off <<= 1) acc += __shfl_xor(acc, off);
    if (q == 0) {
      acc += bias;
      y[p] = sigm ? 1.f / (1.f + expf(-acc)) : acc;
    }
  }
}

// generic fallback (C % 4 != 0 or C/4 not a power of two): one thread per pixel
template <typename T>
__global__ void __launch_bounds__(256)
head_fwd_scalar_kernel(const T* __restrict__ x, const float* __restrict__ w,
                       const float* __restrict__ b, int sigm, float* __restrict__ y, long P, int C) {
  for (long p = blockIdx.x * (long)blockDim.x + threadIdx.x; p < P; p += (long)gridDim.x * blockDim.x) {
    const T* xr = x + p * C;
    float acc = 0.f;
    for (int c = 0; c < C; ++c) acc = fmaf(ld1(xr + c), w[c], acc);
    acc += b[0];
    y[p] = sigm ? 1.f / (1.f + expf(-acc)) : acc;
  }
}

// Backward (C % 4 == 0, C/4 a power of two <= 64): dx[p,c] = g[p]*w[c],
// g = dy (* y(1-y) for the Sigmoid); per-block partials part[blk][2][C] of
// (sum g*x[c], sum g) through the channel-tiled deterministic block reduction.
template <typename T>
__global__ void __launch_bounds__(256)
head_bwd_kernel(const T* __restrict__ x, const float* __restrict__ w, const float* __restrict__ y,
                const float* __restrict__ dy, int sigm, T* __restrict__ dx, long P, int C,
                float* __restrict__ part) {
  ChanTile t = chan_tile<4>(C);
  float a[4] = {0.f, 0.f, 0.f, 0.f}, gs[4] = {0.f, 0.f, 0.f, 0.f};
  long per = (P + gridDim.x - 1) / gridDim.x;
  long p0 = blockIdx.x * per, p1 = min(P, p0 + per);
  if (t.active) {
    const float4 wq = ld4(w + t.c0);
    for (long p = p0 + t.rg; p < p1; p += t.RG) {
      float g = dy[p];
      if (sigm) {
        const float yy = y[p];
        g *= yy * (1.f - yy);
      }
      const float4 xv = ldq(x + p * C + t.c0);
      stq(dx + p * C + t.c0, make_float4(g * wq.x, g * wq.y, g * wq.z, g * wq.w));
      a[0] = fmaf(g, xv.x, a[0]);
      a[1] = fmaf(g, xv.y, a[1]);
      a[2] = fmaf(g, xv.z, a[2]);
      a[3] = fmaf(g, xv.w, a[3]);
      gs[0] += g;
    }
  }
  block_chan_reduce2<4>(t, a, gs, part, blockIdx.x, C);
}

template <typename T>
__global__ void __launch_bounds__(256)
head_bwd_scalar_kernel(const T* __restrict__ x, const float* __restrict__ w,
                       const float* __restrict__ y, const float* __restrict__ dy, int sigm,
                       T* __restrict__ dx, long P, int C, float* __restrict__ part) {
  __shared__ float red[256][33];
  float acc[33];
  for (int c = 0; c <= C && c < 33; ++c) acc[c] = 0.f;
  long per = (P + gridDim.x - 1) / gridDim.x;
  long p0 = blockIdx.x * per, p1 = min(P, p0 + per);
  for (long p = p0 + threadIdx.x; p < p1; p += blockDim.x) {
    float g = dy[p];
    if (sigm) {
      float yy = y[p];
      g *= yy * (1.f - yy);
    }
    const T* xr = x + p * C;
    T* dr = dx + p * C;
    for (int c = 0; c < C; ++c) {
      st1(dr + c, g * w[c]);
      acc[c] = fmaf(g, ld1(xr + c), acc[c]);
    }
    acc[C] += g;
  }
  for (int c = 0; c <= C; ++c) red[threadIdx.x][c] = acc[c];
  __syncthreads();
  // same [blk][2][C] layout as head_bwd_kernel: row 0 = sum g*x[c], row 1 col 0 = sum g
  for (int c = threadIdx.x; c <= C; c += blockDim.x) {
    float s = 0.f;
    for (int t = 0; t < 256; ++t) s += red[t][c];
    part[(long)blockIdx.x * 2 * C + c] = s;  // c == C lands on row 1, column 0
  }
}

// [R][2][C] partial rows -> dw[c] = sum row0, db = sum row1[0]
__global__ void head_bwd_finish_kernel(const float* __restrict__ sums, int C, float* __restrict__ dw,
                                       float* __restrict__ db) {
  const int c = threadIdx.x;
  if (c < C) dw[c] = sums[c];
  if (c == 0) db[0] = sums[C];
}

static int head_tq(int C) {
  if (C % 4) return 0;
  const int q = C / 4;
  return (q & (q - 1)) == 0 && q <= 64 ? q : 0;
}

extern "C" int accunet_head_fwd(const void* x, const float* w, const float* b, int sigm, float* y,
                                long P, int C, int dt, void* stream) {
  const int tq = head_tq(C);
  if (with_dt(dt, [&](auto tag) {
        using T = decltype(tag);
        if (tq) {
          long blocks = (P * tq + 255) / 256;
          if (blocks > 8192) blocks = 8192;
          hipLaunchKernelGGL((head_fwd_kernel<T>), dim3(blocks), dim3(256), 0, (hipStream_t)stream,
                             (const T*)x, w, b, sigm, y, P, C, tq);
        } else {
          long blocks = (P + 255) / 256;
          if (blocks > 4096) blocks = 4096;
          hipLaunchKernelGGL((head_fwd_scalar_kernel<T>), dim3(blocks), dim3(256), 0,
                             (hipStream_t)stream, (const T*)x, w, b, sigm, y, P, C);
        }
      }))
    return ACC_EBADARG;
  return hipGetLastError() == hipSuccess ? ACC_OK : ACC_ELAUNCH;
}

#define HEAD_NB 1024
extern "C" size_t accunet_head_ws_elems(long P, int C) {
  return (size_t)HEAD_NB * 2 * C + accunet_partials_ws_elems(HEAD_NB, 2 * C) + 2 * (size_t)C + 64;
}

extern "C" int accunet_head_bwd(const void* x, const float* w, const float* y, const float* dy,
                                int sigm, void* dx, float* dw, float* db, long P, int C, float* ws,
                                size_t ws_elems, int dt, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const int tq = head_tq(C);
  if (!tq && C > 32) return ACC_EBADSHAPE;
  if (ws_elems < accunet_head_ws_elems(P, C)) return ACC_EBADARG;
  long nb = (P + 255) / 256;
  if (nb > HEAD_NB) nb = HEAD_NB;
  float* part = ws;
  float* scratch = ws + (size_t)HEAD_NB * 2 * C;
  float* sums = scratch + accunet_partials_ws_elems(HEAD_NB, 2 * C);
  if (with_dt(dt, [&](auto tag) {
        using T = decltype(tag);
        if (tq)
          hipLaunchKernelGGL((head_bwd_kernel<T>), dim3((unsigned)nb, ceil_div(C / 4, 64)), dim3(256),
                             0, s, (const T*)x, w, y, dy, sigm, (T*)dx, P, C, part);
        else
          hipLaunchKernelGGL((head_bwd_scalar_kernel<T>), dim3((unsigned)nb), dim3(256), 0, s,
                             (const T*)x, w, y, dy, sigm, (T*)dx, P, C, part);
      }))
    return ACC_EBADARG;
  (void)sums;
  FinishArgs fa{};
  fa.kind = FIN_HEAD;
  fa.ncols = C + 1;  // dw columns, then the bias column
  fa.C = C;
  fa.out_f = dw;
  fa.out2 = db;
  return reduce_finish(part, false, (int)nb, 2 * C, reinterpret_cast<double*>(scratch), fa, s);
}

// ---------------------------------------------------------------------------
// WeightedDiceBCE
//   partial row per block (block covers a chunk of one sample b):
//   [0] sum p*t'  [1] sum p^2  [2] sum tw^2  [3] n_pos  [4] sum pos*l  [5] sum neg*l
//   (p = w*sigmoid(x), tw = w*t, w = t*(w1-w0)+w0 ; BCE on t_b = normalised truth)
// ---------------------------------------------------------------------------
#define LOSS_NCH 64

__global__ void __launch_bounds__(256)
max_kernel(const float* __restrict__ t, long n, float* __restrict__ out) {
  __shared__ float red[256];
  float m = -INFINITY;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    m = fmaxf(m, t[i]);
  red[threadIdx.x] = m;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < s) red[threadIdx.x] = fmaxf(red[threadIdx.x], red[threadIdx.x + s]);
    __syncthreads();
  }
  if (threadIdx.x == 0) out[blockIdx.x] = red[0];
}

ACC_DEV float bce_logits(float x, float t) {
  // max(x,0) - x*t + log(1 + exp(-|x|))  (torch binary_cross_entropy_with_logits)
  return fmaxf(x, 0.f) - x * t + log1pf(expf(-fabsf(x)));
}

__global__ void __launch_bounds__(256)
loss_reduce_kernel(const float* __restrict__ x, const float* __restrict__ t, int B, long N,
                   const float* __restrict__ tmax_part, int nmax, float dw0, float dw1,
                   float* __restrict__ part) {
  __shared__ float red[6][256];
  const int b = blockIdx.x / LOSS_NCH, ch = blockIdx.x % LOSS_NCH;
  float tmax = -INFINITY;
  for (int i = 0; i < nmax; ++i) tmax = fmaxf(tmax, tmax_part[i]);
  const bool binarize = tmax > 1.f;
  long per = (N + LOSS_NCH - 1) / LOSS_NCH;
  long i0 = ch * per, i1 = min(N, i0 + per);
  float a[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (long i = i0 + threadIdx.x; i < i1; i += 256) {
    float xv = x[(long)b * N + i], tv = t[(long)b * N + i];
    float w = tv * (dw1 - dw0) + dw0;
    float p = w * (1.f / (1.f + expf(-xv)));
    float tw = w * tv;
    a[0] += p * tw;
    a[1] += p * p;
    a[2] += tw * tw;
    float tb = binarize ? (tv > 0.f ? 1.f : 0.f) : tv;
    float l = bce_logits(xv, tb);
    float pos = tb > 0.5f ? 1.f : 0.f;
    a[3] += pos;
    a[4] += pos * l;
    a[5] += (1.f - pos) * l;
  }
  for (int k = 0; k < 6; ++k) red[k][threadIdx.x] = a[k];
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < s)
      for (int k = 0; k < 6; ++k) red[k][threadIdx.x] += red[k][threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x < 6) part[(long)blockIdx.x * 6 + threadIdx.x] = red[threadIdx.x][0];
}

// res layout: [0] loss [1] dice [2] bce [3] pw [4] nw [5] binarize flag, then per b: I, U
// One block: thread b (< B) sums sample b's LOSS_NCH chunk rows; the per-sample Dice
// terms and the BCE counts are then added over b in fixed order by thread 0.
__global__ void __launch_bounds__(256)
loss_finalize_kernel(const float* __restrict__ part, int B, long N,
                     const float* __restrict__ tmax_part, int nmax, float bw0, float bw1,
                     float dice_w, float bce_w, float smooth, float* __restrict__ res) {
  __shared__ double red[4][256];
  __shared__ float tm[256];
  const int t = threadIdx.x;
  tm[t] = t < nmax ? tmax_part[t] : -INFINITY;
  for (int b = t; b < B; b += 256) {
    double I = 0, P2 = 0, T2 = 0, np = 0, sp = 0, sn = 0;
    for (int ch = 0; ch < LOSS_NCH; ++ch) {
      const float* pr = part + ((long)b * LOSS_NCH + ch) * 6;
      I += pr[0];
      P2 += pr[1];
      T2 += pr[2];
      np += pr[3];
      sp += pr[4];
      sn += pr[5];
    }
    const double U = P2 + T2;
    res[8 + 2 * b] = (float)I;
    res[8 + 2 * b + 1] = (float)U;
    red[0][b] = 1.0 - (2.0 * I + smooth) / (U + smooth);
    red[1][b] = np;
    red[2][b] = sp;
    red[3][b] = sn;
  }
  __syncthreads();
  if (t != 0) return;
  double dice = 0.0, npos = 0.0, spos = 0.0, sneg = 0.0;
  for (int b = 0; b < B && b < 256; ++b) {
    dice += red[0][b];
    npos += red[1][b];
    spos += red[2][b];
    sneg += red[3][b];
  }
  dice /= B;
  double nneg = (double)B * N - npos;
  double pw = npos < 1.0 ? 1.0 : npos;
  double nw = nneg < 1.0 ? 1.0 : nneg;
  double bce = bw0 * spos / pw + bw1 * sneg / nw;
  float tmax = -INFINITY;
  for (int i = 0; i < nmax && i < 256; ++i) tmax = fmaxf(tmax, tm[i]);
  res[0] = (float)(dice_w * dice + bce_w * bce);
  res[1] = (float)dice;
  res[2] = (float)bce;
  res[3] = (float)pw;
  res[4] = (float)nw;
  res[5] = tmax > 1.f ? 1.f : 0.f;
}

__global__ void __launch_bounds__(256)
loss_bwd_kernel(const float* __restrict__ x, const float* __restrict__ t, int B, long N,
                const float* __restrict__ res, const float* __restrict__ gout, float dw0, float dw1,
                float bw0, float bw1, float dice_w, float bce_w, float smooth,
                float* __restrict__ dx) {
  const float g0 = gout ? gout[0] : 1.f;
  const float pw = res[3], nw = res[4];
  const bool binarize = res[5] > 0.5f;
  long total = (long)B * N;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    int b = (int)(i / N);
    float I = res[8 + 2 * b], U = res[8 + 2 * b + 1];
    float xv = x[i], tv = t[i];
    float sg = 1.f / (1.f + expf(-xv));
    float w = tv * (dw1 - dw0) + dw0;
    float p = w * sg, tw = w * tv;
    float den = U + smooth;
    float dD_dp = -(2.f * tw * den - (2.f * I + smooth) * 2.f * p) / (den * den);
    float gd = dD_dp * w * sg * (1.f - sg) * (dice_w / B);
    float tb = binarize ? (tv > 0.f ? 1.f : 0.f) : tv;
    float pos = tb > 0.5f ? 1.f : 0.f;
    float gb = (sg - tb) * (pos * bw0 / pw + (1.f - pos) * bw1 / nw) * bce_w;
    dx[i] = g0 * (gd + gb);
  }
}

extern "C" size_t accunet_loss_ws_elems(int B) { return (size_t)B * LOSS_NCH * 6 + 256 + 8 + 2 * (size_t)B; }

// res (device, >= 8 + 2B floats) receives [loss, dice, bce, pw, nw, binarize, -, -, (I,U) per b]
extern "C" int accunet_loss_fwd(const float* x, const float* t, int B, long N, float dice_w,
                                float bce_w, float* res, float* ws, size_t ws_elems, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (ws_elems < accunet_loss_ws_elems(B)) return ACC_EBADARG;
  if (B < 1 || B > 256) return ACC_EBADSHAPE;  // loss_finalize_kernel: one thread per sample
  float* part = ws;
  float* tmax = ws + (size_t)B * LOSS_NCH * 6;
  const int nmax = 256;
  hipLaunchKernelGGL(max_kernel, dim3(nmax), dim3(256), 0, s, t, (long)B * N, tmax);
  hipLaunchKernelGGL(loss_reduce_kernel, dim3(B * LOSS_NCH), dim3(256), 0, s, x, t, B, N, tmax,
                     nmax, 0.5f, 0.5f, part);
  hipLaunchKernelGGL(loss_finalize_kernel, dim3(1), dim3(256), 0, s, part, B, N, tmax, nmax, 0.5f,
                     0.5f, dice_w, bce_w, 1e-5f, res);
  return hipGetLastError() == hipSuccess ? ACC_OK : ACC_ELAUNCH;
}

extern "C" int accunet_loss_bwd(const float* x, const float* t, int B, long N, float dice_w,
                                float bce_w, const float* res, const float* gout, float* dx,
                                void* stream) {
  long total = (long)B * N;
  long blocks = (total + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(loss_bwd_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, x, t, B, N,
                     res, gout, 0.5f, 0.5f, 0.5f, 0.5f, dice_w, bce_w, 1e-5f, dx);
  return hipGetLastError() == hipSuccess ? ACC_OK : ACC_ELAUNCH;
}

// ---------------------------------------------------------------------------
// Multi-tensor Adam: one launch over every parameter tensor.
// table: per tensor {p, g, m, v} device pointers + numel; chunks map blocks to
// (tensor, start). Same arithmetic order as torch.optim.Adam (foreach path):
//   m = m + (1-b1)*(g-m);  v = v*b2 + (1-b2)*g*g;
//   p = p - step_size * m / (sqrt(v)/bc2_sqrt + eps)
// ---------------------------------------------------------------------------
struct AdamTensor {
  float* p;
  const float* g;
  float* m;
  float* v;
  long long n;
};

#define ADAM_CHUNK 16384

__global__ void __launch_bounds__(256)
adam_kernel(const AdamTensor* __restrict__ tab, const int* __restrict__ chunk_t,
            const long long* __restrict__ chunk_s, float b1, float b2, float eps, float step_size,
            float bc2_sqrt, float wd) {
  const int c = blockIdx.x;
  const AdamTensor T = tab[chunk_t[c]];
  long long s0 = chunk_s[c];
  long long s1 = min(T.n, s0 + (long long)ADAM_CHUNK);
  for (long long i = s0 + threadIdx.x; i < s1; i += blockDim.x) {
    float g = T.g[i];
    float p = T.p[i];
    if (wd != 0.f) g = g + wd * p;
    float m = T.m[i];
    m = m + (1.f - b1) * (g - m);
    float v = T.v[i] * b2 + (1.f - b2) * g * g;
    float denom = sqrtf(v) / bc2_sqrt + eps;
    T.m[i] = m;
    T.v[i] = v;
    T.p[i] = p - step_size * (m / denom);
  }
}

extern "C" int accunet_adam_chunk_elems() { return ADAM_CHUNK; }

extern "C" int accunet_adam_step(const void* table, const int* chunk_t, const long long* chunk_s,
                                 int nchunks, float lr, float b1, float b2, float eps, float wd,
                                 int step, void* stream) {
  if (nchunks <= 0) return ACC_OK;
  double bc1 = 1.0 - pow((double)b1, step);
  double bc2 = 1.0 - pow((double)b2, step);
  float step_size = (float)(lr / bc1);
  float bc2_sqrt = (float)sqrt(bc2);
  hipLaunchKernelGGL(adam_kernel, dim3(nchunks), dim3(256), 0, (hipStream_t)stream,
                     (const AdamTensor*)table, chunk_t, chunk_s, b1, b2, eps, step_size, bc2_sqrt,
                     wd);
  return hipGetLastError() == hipSuccess ? ACC_OK : ACC_ELAUNCH;
}

// ---------------------------------------------------------------------------
// out[0] = sum_i g[i] * (a[i] - b[i])  (gradient of ACC_UNet_W's scalar merge weight,
// ACC_UNet/ACC_UNet_w.py:497-522: y = m*W + x*(1-W)); deterministic two-level sum.
// ---------------------------------------------------------------------------
template <typename T>
__global__ void __launch_bounds__(256)
dotdiff_kernel(const T* __restrict__ g, const T* __restrict__ a, const T* __restrict__ b,
               long n, float* __restrict__ part) {
  __shared__ float red[256];
  float s = 0.f;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    s += ld1(g + i) * (ld1(a + i) - ld1(b + i));
  red[threadIdx.x] = s;
  __syncthreads();
  for (int k = 128; k > 0; k >>= 1) {
    if (threadIdx.x < k) red[threadIdx.x] += red[threadIdx.x + k];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[blockIdx.x] = red[0];
}

__global__ void finish_sum_kernel(const float* __restrict__ part, int n, float* __restrict__ out,
                                  int accumulate) {
  if (threadIdx.x != 0) return;
  double s = 0.0;
  for (int i = 0; i < n; ++i) s += part[i];
  out[0] = accumulate ? out[0] + (float)s : (float)s;
}

extern "C" int accunet_dotdiff(const void* g, const void* a, const void* b, long n, float* out,
                               int accumulate, float* ws, int dt, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (with_dt(dt, [&](auto tag) {
        using T = decltype(tag);
        hipLaunchKernelGGL((dotdiff_kernel<T>), dim3(1024), dim3(256), 0, s, (const T*)g,
                           (const T*)a, (const T*)b, n, ws);
      }))
    return ACC_EBADARG;
  hipLaunchKernelGGL(finish_sum_kernel, dim3(1), dim3(64), 0, s, ws, 1024, out, accumulate);
  return hipGetLastError() == hipSuccess ? ACC_OK : ACC_ELAUNCH;
}

// y = a*w + b*(1-w) (w device scalar), with optional partial channel stats of y
template <int V, typename T>
__global__ void __launch_bounds__(256)
wmerge_kernel(const T* __restrict__ a, const T* __restrict__ b, const float* __restrict__ w,
              T* __restrict__ y, long P, int C, double* __restrict__ stats) {
  ChanTile t = chan_tile<V>(C);
  long rows_per = (P + gridDim.x - 1) / gridDim.x;
  long r0 = blockIdx.x * rows_per, r1 = min(P, r0 + rows_per);
  double s1[V], s2[V];
#pragma unroll
  for (int j = 0; j < V; ++j) { s1[j] = 0.0; s2[j] = 0.0; }
  const float wv = w[0];
  if (t.active) {
    for (long r = r0 + t.rg; r < r1; r += t.RG) {
      float va[V], vb[V];
      ldv<V>(a + r * C + t.c0, va);
      ldv<V>(b + r * C + t.c0, vb);
#pragma unroll
      for (int j = 0; j < V; ++j) {
        va[j] = rnd<T>(va[j] * wv + vb[j] * (1.f - wv));  // statistics of the stored value
        s1[j] += va[j];
        s2[j] += (double)va[j] * va[j];
      }
      stv<V>(y + r * C + t.c0, va);
    }
  }
  if (stats) block_chan_reduce2<V>(t, s1, s2, stats, blockIdx.x, C);
}

extern "C" int accunet_wmerge_fwd(const void* a, const void* b, const float* w, void* y, long P,
                                  int C, double* stats, int dt, void* stream) {
  int V = (C % 4 == 0) ? 4 : 1;
  int nb = stream_rowblocks(P, C);
  dim3 grid(nb, ceil_div(C / V, 64));
  if (with_dt(dt, [&](auto tag) {
        using T = decltype(tag);
        if (V == 4)
          hipLaunchKernelGGL((wmerge_kernel<4, T>), grid, dim3(256), 0, (hipStream_t)stream,
                             (const T*)a, (const T*)b, w, (T*)y, P, C, stats);
        else
          hipLaunchKernelGGL((wmerge_kernel<1, T>), grid, dim3(256), 0, (hipStream_t)stream,
                             (const T*)a, (const T*)b, w, (T*)y, P, C, stats);
      }))
    return ACC_EBADARG;
  return hipGetLastError() == hipSuccess ? ACC_OK : ACC_ELAUNCH;
}

// dA = w*g, dB = (1-w)*g (B gradient optionally accumulated)
template <typename T>
__global__ void __launch_bounds__(256)
wmerge_bwd_kernel(const T* __restrict__ g, const float* __restrict__ w, T* __restrict__ da,
                  T* __restrict__ db, long n) {
  const float wv = w[0];
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    float gv = ld1(g + i);
    st1(da + i, wv * gv);
    st1(db + i, (1.f - wv) * gv);
  }
}

extern "C" int accunet_wmerge_bwd(const void* g, const float* w, void* da, void* db, long n, int dt,
                                  void* stream) {
  long blocks = (n + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  if (with_dt(dt, [&](auto tag) {
        using T = decltype(tag);
        hipLaunchKernelGGL((wmerge_bwd_kernel<T>), dim3(blocks), dim3(256), 0, (hipStream_t)stream,
                           (const T*)g, w, (T*)da, (T*)db, n);
      }))
    return ACC_EBADARG;
  return hipGetLastError() == hipSuccess ? ACC_OK : ACC_ELAUNCH;
}

// ---------------------------------------------------------------------------
// HIP events for the graph-mode gradient all-reduce (accunet/train.py). While the
// backward is captured, accunet_graph_marker(id) leaves a 1-thread marker kernel in
// the stream at the point where gradient bucket `id` is complete. After capture (the
// graph kept un-instantiated, torch CUDAGraph(keep_graph=True)),
// accunet_graph_events_after_markers adds an event-record node behind every marker
// (hipGraphAddEventRecordNode; recording events *during* capture needs external event
// records, which the HIP runtime torch ships rejects). Each graph launch re-records
// the events, so a side stream that waits on them (accunet_stream_wait_event) after
// the launch starts that bucket's RCCL all-reduce while the graph still runs the rest
// of backward.
// ---------------------------------------------------------------------------
#define ACC_MAX_MARKERS 32
template <int ID>
__global__ void graph_marker_kernel() {}

template <int... I>
struct MarkerTable {
  static void* get(int i) {
    static void* const t[] = {reinterpret_cast<void*>(&graph_marker_kernel<I>)...};
    return t[i];
  }
};
template <int N, int... I>
struct MakeMarkers : MakeMarkers<N - 1, N - 1, I...> {};
template <int... I>
struct MakeMarkers<0, I...> {
  typedef MarkerTable<I...> type;
};
typedef MakeMarkers<ACC_MAX_MARKERS>::type Markers;

// The probes' streaming ceiling (include/accunet.h accunet_copy_nt): one 16-KB chunk per
// 256-thread block, 4 float4 per thread, non-temporal both ways.
typedef float acc_v4f __attribute__((ext_vector_type(4)));
__global__ void __launch_bounds__(256) copy_nt_kernel(const acc_v4f* __restrict__ a,
                                                      acc_v4f* __restrict__ b, long n) {
  const long base = (long)blockIdx.x * 1024 + threadIdx.x;
  acc_v4f v[4];
#pragma unroll
  for (int k = 0; k < 4; ++k)
    if (base + 256 * k < n) v[k] = __builtin_nontemporal_load(&a[base + 256 * k]);
#pragma unroll
  for (int k = 0; k < 4; ++k)
    if (base + 256 * k < n) __builtin_nontemporal_store(v[k], &b[base + 256 * k]);
}

extern "C" int accunet_copy_nt(const void* src, void* dst, long long n_bytes, void* stream) {
  if (!src || !dst || n_bytes < 0 || (n_bytes & 15) || (((uintptr_t)src | (uintptr_t)dst) & 15))
    return ACC_EBADARG;
  const long n = (long)(n_bytes / 16);
  if (n == 0) return ACC_OK;
  hipLaunchKernelGGL(copy_nt_kernel, dim3((unsigned)((n + 1023) / 1024)), dim3(256), 0,
                     (hipStream_t)stream, (const acc_v4f*)src, (acc_v4f*)dst, n);
  return hipGetLastError() == hipSuccess ? ACC_OK : ACC_ELAUNCH;
}

extern "C" int accunet_graph_marker(int id, void* stream) {
  if (id < 0 || id >= ACC_MAX_MARKERS) return ACC_EBADARG;
  if (hipLaunchKernel(Markers::get(id), dim3(1), dim3(1), nullptr, 0, (hipStream_t)stream) !=
      hipSuccess)
    return ACC_ELAUNCH;
  return hipGetLastError() == hipSuccess ? ACC_OK : ACC_ELAUNCH;
}

// returns the number of event-record nodes added (one per marker found), or < 0
extern "C" int accunet_graph_events_after_markers(void* graph, void* const* events, int n) {
  if (!graph || !events || n < 0 || n > ACC_MAX_MARKERS) return ACC_EBADARG;
  hipGraph_t g = (hipGraph_t)graph;
  size_t nn = 0;
  if (hipGraphGetNodes(g, nullptr, &nn) != hipSuccess) return ACC_ELAUNCH;
  hipGraphNode_t* nodes = (hipGraphNode_t*)malloc(sizeof(hipGraphNode_t) * (nn ? nn : 1));
  if (!nodes) return ACC_EBADARG;
  int found = 0, status = ACC_OK;
  if (hipGraphGetNodes(g, nodes, &nn) != hipSuccess) status = ACC_ELAUNCH;
  for (size_t k = 0; k < nn && status == ACC_OK; ++k) {
    hipGraphNodeType t;
    if (hipGraphNodeGetType(nodes[k], &t) != hipSuccess || t != hipGraphNodeTypeKernel) continue;
    hipKernelNodeParams kp;
    if (hipGraphKernelNodeGetParams(nodes[k], &kp) != hipSuccess) continue;
    for (int id = 0; id < n; ++id) {
      if (kp.func != Markers::get(id)) continue;
      hipGraphNode_t ev;
      if (hipGraphAddEventRecordNode(&ev, g, &nodes[k], 1, (hipEvent_t)events[id]) != hipSuccess)
        status = ACC_ELAUNCH;
      ++found;
    }
  }
  free(nodes);
  return status == ACC_OK ? found : status;
}

extern "C" int accunet_event_create(void** ev) {
  if (!ev) return ACC_EBADARG;
  hipEvent_t e;
  if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return ACC_ELAUNCH;
  *ev = (void*)e;
  return ACC_OK;
}

extern "C" int accunet_event_create_timed(void** ev) {
  if (!ev) return ACC_EBADARG;
  hipEvent_t e;
  if (hipEventCreate(&e) != hipSuccess) return ACC_ELAUNCH;
  *ev = (void*)e;
  return ACC_OK;
}

// the one kernel node of graph g that launches marker id (nullptr: none or several)
static hipGraphNode_t find_marker(hipGraph_t g, int id) {
  size_t nn = 0;
  if (hipGraphGetNodes(g, nullptr, &nn) != hipSuccess || nn == 0) return nullptr;
  hipGraphNode_t* nodes = (hipGraphNode_t*)malloc(sizeof(hipGraphNode_t) * nn);
  if (!nodes) return nullptr;
  hipGraphNode_t hit = nullptr;
  int count = 0;
  if (hipGraphGetNodes(g, nodes, &nn) == hipSuccess) {
    for (size_t k = 0; k < nn; ++k) {
      hipGraphNodeType t;
      if (hipGraphNodeGetType(nodes[k], &t) != hipSuccess || t != hipGraphNodeTypeKernel) continue;
      hipKernelNodeParams kp;
      if (hipGraphKernelNodeGetParams(nodes[k], &kp) != hipSuccess) continue;
      if (kp.func == Markers::get(id)) {
        hit = nodes[k];
        ++count;
      }
    }
  }
  free(nodes);
  return count == 1 ? hit : nullptr;
}

// event-record node in place of marker node m: same dependencies, same dependents;
// the marker is removed only once the new node is wired (a failure leaves a valid graph)
static int replace_marker(hipGraph_t g, hipGraphNode_t m, hipEvent_t ev, hipGraphNode_t* out) {
  size_t np = 0, ns = 0;
  if (hipGraphNodeGetDependencies(m, nullptr, &np) != hipSuccess ||
      hipGraphNodeGetDependentNodes(m, nullptr, &ns) != hipSuccess)
    return ACC_ELAUNCH;
  hipGraphNode_t* pr = (hipGraphNode_t*)malloc(sizeof(hipGraphNode_t) * (np + ns + 1));
  if (!pr) return ACC_EBADARG;
  hipGraphNode_t* su = pr + np;
  int rc = ACC_OK;
  if ((np && hipGraphNodeGetDependencies(m, pr, &np) != hipSuccess) ||
      (ns && hipGraphNodeGetDependentNodes(m, su, &ns) != hipSuccess))
    rc = ACC_ELAUNCH;
  hipGraphNode_t e = nullptr;
  if (rc == ACC_OK && hipGraphAddEventRecordNode(&e, g, np ? pr : nullptr, np, ev) != hipSuccess)
    rc = ACC_ELAUNCH;
  for (size_t k = 0; rc == ACC_OK && k < ns; ++k)
    if (hipGraphAddDependencies(g, &e, &su[k], 1) != hipSuccess) rc = ACC_ELAUNCH;
  if (rc == ACC_OK && hipGraphDestroyNode(m) != hipSuccess) rc = ACC_ELAUNCH;
  free(pr);
  if (rc == ACC_OK) *out = e;
  return rc;
}

extern "C" int accunet_graph_time_markers(void* graph, int id_start, int id_end, void* ev_start,
                                          void* ev_end, void** nodes) {
  if (!graph || !ev_start || !ev_end || !nodes || id_start == id_end || id_start < 0 ||
      id_end < 0 || id_start >= ACC_MAX_MARKERS || id_end >= ACC_MAX_MARKERS)
    return ACC_EBADARG;
  hipGraph_t g = (hipGraph_t)graph;
  hipGraphNode_t ms = find_marker(g, id_start), me = find_marker(g, id_end);
  if (!ms || !me) return ACC_EBADSHAPE;
  hipGraphNode_t es = nullptr, ee = nullptr;
  int rc = replace_marker(g, ms, (hipEvent_t)ev_start, &es);
  if (rc != ACC_OK) return rc;
  rc = replace_marker(g, me, (hipEvent_t)ev_end, &ee);
  if (rc != ACC_OK) return rc;
  nodes[0] = (void*)es;
  nodes[1] = (void*)ee;
  return ACC_OK;
}

extern "C" int accunet_graph_exec_event_set(void* exec, void* node, void* ev) {
  if (!exec || !node || !ev) return ACC_EBADARG;
  return hipGraphExecEventRecordNodeSetEvent((hipGraphExec_t)exec, (hipGraphNode_t)node,
                                             (hipEvent_t)ev) == hipSuccess
             ? ACC_OK
             : ACC_ELAUNCH;
}

extern "C" int accunet_event_elapsed_ms(void* start, void* end, float* ms) {
  if (!start || !end || !ms) return ACC_EBADARG;
  return hipEventElapsedTime(ms, (hipEvent_t)start, (hipEvent_t)end) == hipSuccess ? ACC_OK
                                                                                   : ACC_ELAUNCH;
}

extern "C" int accunet_event_destroy(void* ev) {
  return hipEventDestroy((hipEvent_t)ev) == hipSuccess ? ACC_OK : ACC_ELAUNCH;
}

extern "C" int accunet_stream_wait_event(void* stream, void* ev) {
  return hipStreamWaitEvent((hipStream_t)stream, (hipEvent_t)ev, 0) == hipSuccess ? ACC_OK
                                                                                  : ACC_ELAUNCH;
}

extern "C" int accunet_event_synchronize(void* ev) {
  return hipEventSynchronize((hipEvent_t)ev) == hipSuccess ? ACC_OK : ACC_ELAUNCH;
}
