// Kernels of the UNeXt tokenized-MLP model (reference Experiments/nets/UNext.py),
// NHWC fp32 (a token sequence [B, N = H*W, C] is the same memory as NHWC).
//
//   layernorm   nn.LayerNorm(C) over the channels of every token (norm2 :181,
//               OverlapPatchEmbed.norm :221, norm3/norm4/dnorm3/dnorm4 :244-248):
//               fp32 in/out, per-token mean / rstd saved for the backward; the
//               gamma / beta gradients are per-block partials summed in a fixed order.
//   gelu        nn.GELU() (exact erf form, shiftmlp.act :49).
//   token shift the shifted-MLP shift (shiftmlp.forward :86-93 and :104-111): pad 2,
//               chunk the channels into 5 groups of ceil(C/5), roll group g by g-2
//               along H (or W), crop -> y[h][w][c] = x[h - s(c)][w][c] (zero outside),
//               s(c) = c / ceil(C/5) - 2; its backward is the opposite shift.
//   up2         F.interpolate(scale_factor=2, mode='bilinear') (align_corners=False,
//               :313,318,325,329,333) fused with the ReLU after it and the skip add
//               (torch.add(out, t_k)); the ReLU mask is kept as bytes for the backward.
//   relu        F.relu after the encoder max-pools (:257-265).
//   subsample2  the stride 2 of OverlapPatchEmbed.proj (3x3, pad 1, :219): the model
//               evaluates the stride-1 convolution and keeps even pixels.
#include "common.h"

// ------------------------------------------------------------------ LayerNorm
// One wave per token, lane = channel quad (C % 4 == 0, C <= 256).
#define LN_TOK_PER_BLOCK 64  // 4 waves x 16 tokens (fewer gamma/beta partial rows)

ACC_DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

__global__ void __launch_bounds__(256)
layernorm_fwd_kernel(const float* __restrict__ x, const float* __restrict__ g,
                     const float* __restrict__ b, float* __restrict__ y, float* __restrict__ mr,
                     long P, int C, float eps) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int CQ = C >> 2;
  const bool act = lane < CQ;
  float4 gg = make_float4(0.f, 0.f, 0.f, 0.f), bb = gg;
  if (act) {
    gg = ld4(g + 4 * lane);
    bb = ld4(b + 4 * lane);
  }
  for (int t = 0; t < LN_TOK_PER_BLOCK / 4; ++t) {
    const long p = (long)blockIdx.x * LN_TOK_PER_BLOCK + wave * (LN_TOK_PER_BLOCK / 4) + t;
    if (p >= P) break;
    float4 v = act ? ld4(x + p * C + 4 * lane) : make_float4(0.f, 0.f, 0.f, 0.f);
    const float mean = wave_sum(v.x + v.y + v.z + v.w) / (float)C;
    float4 d = make_float4(v.x - mean, v.y - mean, v.z - mean, v.w - mean);
    if (!act) d = make_float4(0.f, 0.f, 0.f, 0.f);
    const float var = wave_sum(d.x * d.x + d.y * d.y + d.z * d.z + d.w * d.w) / (float)C;
    const float rs = 1.f / sqrtf(var + eps);
    if (act)
      st4(y + p * C + 4 * lane, make_float4(d.x * rs * gg.x + bb.x, d.y * rs * gg.y + bb.y,
                                            d.z * rs * gg.z + bb.z, d.w * rs * gg.w + bb.w));
    if (lane == 0) {
      mr[2 * p] = mean;
      mr[2 * p + 1] = rs;
    }
  }
}

// dx = rstd * (dyg - mean(dyg) - xhat * mean(dyg * xhat)), dyg = dy * gamma;
// part[block][2][C] = (sum dy * xhat, sum dy) over the block's tokens
__global__ void __launch_bounds__(256)
layernorm_bwd_kernel(const float* __restrict__ x, const float* __restrict__ g,
                     const float* __restrict__ mr, const float* __restrict__ dy,
                     float* __restrict__ dx, float* __restrict__ part, long P, int C) {
  __shared__ float4 red[4][2][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int CQ = C >> 2;
  const bool act = lane < CQ;
  const float4 gg = act ? ld4(g + 4 * lane) : make_float4(0.f, 0.f, 0.f, 0.f);
  float4 sg = make_float4(0.f, 0.f, 0.f, 0.f), sb = sg;
  for (int t = 0; t < LN_TOK_PER_BLOCK / 4; ++t) {
    const long p = (long)blockIdx.x * LN_TOK_PER_BLOCK + wave * (LN_TOK_PER_BLOCK / 4) + t;
    if (p >= P) break;
    const float mean = mr[2 * p], rs = mr[2 * p + 1];
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f), d = v;
    if (act) {
      v = ld4(x + p * C + 4 * lane);
      d = ld4(dy + p * C + 4 * lane);
    }
    const float4 xh = make_float4((v.x - mean) * rs, (v.y - mean) * rs, (v.z - mean) * rs,
                                  (v.w - mean) * rs);
    const float4 dg = make_float4(d.x * gg.x, d.y * gg.y, d.z * gg.z, d.w * gg.w);
    const float m1 = wave_sum(dg.x + dg.y + dg.z + dg.w) / (float)C;
    const float m2 = wave_sum(dg.x * xh.x + dg.y * xh.y + dg.z * xh.z + dg.w * xh.w) / (float)C;
    if (act) {
      st4(dx + p * C + 4 * lane,
          make_float4(rs * (dg.x - m1 - xh.x * m2), rs * (dg.y - m1 - xh.y * m2),
                      rs * (dg.z - m1 - xh.z * m2), rs * (dg.w - m1 - xh.w * m2)));
      sg.x += d.x * xh.x; sg.y += d.y * xh.y; sg.z += d.z * xh.z; sg.w += d.w * xh.w;
      sb.x += d.x; sb.y += d.y; sb.z += d.z; sb.w += d.w;
    }
  }
  red[wave][0][lane] = sg;
  red[wave][1][lane] = sb;
  __syncthreads();
  if (wave == 0 && act) {
    float4 a = red[0][0][lane], c = red[0][1][lane];
#pragma unroll
    for (int w = 1; w < 4; ++w) {
      const float4 a2 = red[w][0][lane], c2 = red[w][1][lane];
      a.x += a2.x; a.y += a2.y; a.z += a2.z; a.w += a2.w;
      c.x += c2.x; c.y += c2.y; c.z += c2.z; c.w += c2.w;
    }
    st4(part + (long)blockIdx.x * 2 * C + 4 * lane, a);
    st4(part + (long)blockIdx.x * 2 * C + C + 4 * lane, c);
  }
}

// out[c] (c < W) = sum over R partial rows, fixed order: 16 row groups x 64 columns
// per 1024-thread block, each group with 4 independent accumulators (rows r, r+16,
// r+32, r+48 of its stride-64 sweep) so the loads are not one dependent chain.
__global__ void __launch_bounds__(1024)
colsum_rows_kernel(const float* __restrict__ part, int R, int W, float* __restrict__ out) {
  __shared__ double red[16][64];
  const int cl = threadIdx.x & 63, gq = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
  if (c < W) {
    int r = gq;
    for (; r + 48 < R; r += 64) {
      s0 += part[(long)r * W + c];
      s1 += part[(long)(r + 16) * W + c];
      s2 += part[(long)(r + 32) * W + c];
      s3 += part[(long)(r + 48) * W + c];
    }
    for (; r < R; r += 16) s0 += part[(long)r * W + c];
  }
  red[gq][cl] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  if (gq == 0 && c < W) {
    double t = 0.0;
#pragma unroll
    for (int k = 0; k < 16; ++k) t += red[k][cl];
    out[c] = (float)t;
  }
}

// ------------------------------------------------------------------ GELU (exact)
__global__ void __launch_bounds__(256)
gelu_fwd_kernel(const float* __restrict__ x, float* __restrict__ y, long n4) {
  const long i = blockIdx.x * 256L + threadIdx.x;
  if (i >= n4) return;
  float4 v = ld4(x + 4 * i);
  auto f = [](float a) { return 0.5f * a * (1.f + erff(a * 0.70710678118654752f)); };
  st4(y + 4 * i, make_float4(f(v.x), f(v.y), f(v.z), f(v.w)));
}

__global__ void __launch_bounds__(256)
gelu_bwd_kernel(const float* __restrict__ x, const float* __restrict__ dy, float* __restrict__ dx,
                long n4) {
  const long i = blockIdx.x * 256L + threadIdx.x;
  if (i >= n4) return;
  float4 v = ld4(x + 4 * i), d = ld4(dy + 4 * i);
  auto df = [](float a) {
    const float cdf = 0.5f * (1.f + erff(a * 0.70710678118654752f));
    const float pdf = expf(-0.5f * a * a) * 0.39894228040143268f;
    return cdf + a * pdf;
  };
  st4(dx + 4 * i, make_float4(d.x * df(v.x), d.y * df(v.y), d.z * df(v.z), d.w * df(v.w)));
}

// ------------------------------------------------------------------ token shift
// axis 0: along H, 1: along W; dir +1 forward (y[h] = x[h - s]), -1 backward
__global__ void __launch_bounds__(256)
token_shift_kernel(const float* __restrict__ x, float* __restrict__ y, int B, int H, int W, int C,
                   int axis, int dir, int chunk, int pad) {
  const long total = (long)B * H * W * C;
  const long e = blockIdx.x * 256L + threadIdx.x;
  if (e >= total) return;
  const int c = (int)(e % C);
  long t = e / C;
  const int w = (int)(t % W);
  t /= W;
  const int h = (int)(t % H);
  const int b = (int)(t / H);
  const int s = dir * (c / chunk - pad);
  int hh = h, ww = w;
  if (axis == 0) hh = h - s; else ww = w - s;
  float v = 0.f;
  if (hh >= 0 && hh < H && ww >= 0 && ww < W) v = x[(((long)b * H + hh) * W + ww) * C + c];
  y[e] = v;
}

// ------------------------------------------------------------------ bilinear x2
// torch upsample_bilinear2d, align_corners=False, scale 2: source s = (d + 0.5)/2 - 0.5
// clamped at 0; i0 = floor(s), i1 = i0 + (i0 < n - 1), l1 = s - i0
ACC_DEV void up2_src(int d, int n, int* i0, int* i1, float* l0, float* l1) {
  float s = ((float)d + 0.5f) * 0.5f - 0.5f;
  if (s < 0.f) s = 0.f;
  int a = (int)s;
  *i0 = a;
  *i1 = a + (a < n - 1 ? 1 : 0);
  *l1 = s - (float)a;
  *l0 = 1.f - *l1;
}

// out = relu(up2(x)) (+ skip); mask = (up2(x) > 0)
__global__ void __launch_bounds__(256)
up2_relu_add_fwd_kernel(const float* __restrict__ x, const float* __restrict__ skip,
                        float* __restrict__ out, unsigned char* __restrict__ mask, int B, int H,
                        int W, int C) {
  const int OH = 2 * H, OW = 2 * W;
  const long total = (long)B * OH * OW * C;
  const long e = blockIdx.x * 256L + threadIdx.x;
  if (e >= total) return;
  const int c = (int)(e % C);
  long t = e / C;
  const int ox = (int)(t % OW);
  t /= OW;
  const int oy = (int)(t % OH);
  const int b = (int)(t / OH);
  int y0, y1, x0, x1;
  float ly0, ly1, lx0, lx1;
  up2_src(oy, H, &y0, &y1, &ly0, &ly1);
  up2_src(ox, W, &x0, &x1, &lx0, &lx1);
  const float* xb = x + (long)b * H * W * C + c;
  const float v00 = xb[((long)y0 * W + x0) * C], v01 = xb[((long)y0 * W + x1) * C];
  const float v10 = xb[((long)y1 * W + x0) * C], v11 = xb[((long)y1 * W + x1) * C];
  const float u = ly0 * (lx0 * v00 + lx1 * v01) + ly1 * (lx0 * v10 + lx1 * v11);
  const bool pos = u > 0.f;
  mask[e] = pos ? 1 : 0;
  out[e] = (pos ? u : 0.f) + (skip ? skip[e] : 0.f);
}

// dx[i][j] = sum over the output rows / cols reading (i, j) of weight * dout * mask
ACC_DEV int up2_readers(int i, int n, int* d, float* wt) {
  // candidates 2i-1, 2i, 2i+1, 2i+2; weight of source i in each
  int k = 0;
  for (int o = 2 * i - 1; o <= 2 * i + 2; ++o) {
    if (o < 0 || o >= 2 * n) continue;
    int a0, a1;
    float l0, l1;
    up2_src(o, n, &a0, &a1, &l0, &l1);
    float w = 0.f;
    if (a0 == i) w += l0;
    if (a1 == i) w += l1;
    if (w != 0.f) {
      d[k] = o;
      wt[k] = w;
      ++k;
    }
  }
  return k;
}

__global__ void __launch_bounds__(256)
up2_relu_bwd_kernel(const float* __restrict__ dout, const unsigned char* __restrict__ mask,
                    float* __restrict__ dx, int B, int H, int W, int C) {
  const long total = (long)B * H * W * C;
  const long e = blockIdx.x * 256L + threadIdx.x;
  if (e >= total) return;
  const int c = (int)(e % C);
  long t = e / C;
  const int j = (int)(t % W);
  t /= W;
  const int i = (int)(t % H);
  const int b = (int)(t / H);
  const int OH = 2 * H, OW = 2 * W;
  int ry[4], rx[4];
  float wy[4], wx[4];
  const int ny = up2_readers(i, H, ry, wy), nx = up2_readers(j, W, rx, wx);
  const long ob = (long)b * OH * OW * C + c;
  float acc = 0.f;
  for (int a = 0; a < ny; ++a) {
    float row = 0.f;
    for (int q = 0; q < nx; ++q) {
      const long o = ob + ((long)ry[a] * OW + rx[q]) * C;
      row += wx[q] * (mask[o] ? dout[o] : 0.f);
    }
    acc += wy[a] * row;
  }
  dx[e] = acc;
}

// ------------------------------------------------------------------ relu, subsample
__global__ void __launch_bounds__(256)
relu_kernel(const float* __restrict__ x, const float* __restrict__ dy, float* __restrict__ y,
            long n) {
  const long i = blockIdx.x * 256L + threadIdx.x;
  if (i >= n) return;
  // forward (dy null): y = max(x, 0); backward: y = dy * (x > 0) with x the forward output
  y[i] = dy ? (x[i] > 0.f ? dy[i] : 0.f) : fmaxf(x[i], 0.f);
}

// fwd: y[b,h,w,:] = x[b,2h,2w,:] (x is B x 2H x 2W); bwd: x-grad zero except even pixels
__global__ void __launch_bounds__(256)
subsample2_kernel(const float* __restrict__ src, float* __restrict__ dst, int B, int H, int W,
                  int C, int bwd) {
  // H, W: the full (stride-1) resolution
  const long total = (long)B * H * W * C;
  const long e = blockIdx.x * 256L + threadIdx.x;
  if (e >= total) return;
  const int c = (int)(e % C);
  long t = e / C;
  const int w = (int)(t % W);
  t /= W;
  const int h = (int)(t % H);
  const int b = (int)(t / H);
  const int Ho = (H + 1) / 2, Wo = (W + 1) / 2;
  const long s = (((long)b * Ho + (h >> 1)) * Wo + (w >> 1)) * C + c;
  const bool even = !(h & 1) && !(w & 1);
  if (bwd) {
    dst[e] = even ? src[s] : 0.f;  // dst = full-res gradient, src = strided gradient
  } else if (even) {
    dst[s] = src[e];               // dst = strided output, src = full-res conv output
  }
}

// ------------------------------------------------------------------ C ABI
static inline unsigned nblk(long n) { return (unsigned)((n + 255) / 256); }
#define LAUNCH_OK (hipGetLastError() == hipSuccess ? ACC_OK : ACC_ELAUNCH)

extern "C" int accunet_layernorm_rows(long P) { return ceil_div(P, LN_TOK_PER_BLOCK); }

extern "C" int accunet_layernorm_fwd(const float* x, const float* g, const float* b, float* y,
                                     float* mr, long P, int C, float eps, void* stream) {
  if (C % 4 || C > 256 || P <= 0) return ACC_EBADSHAPE;
  hipLaunchKernelGGL(layernorm_fwd_kernel, dim3(ceil_div(P, LN_TOK_PER_BLOCK)), dim3(256), 0,
                     (hipStream_t)stream, x, g, b, y, mr, P, C, eps);
  return LAUNCH_OK;
}

// part: [accunet_layernorm_rows(P)][2][C] scratch; dg, db: [C]
extern "C" int accunet_layernorm_bwd(const float* x, const float* g, const float* mr,
                                     const float* dy, float* dx, float* dg, float* db,
                                     float* part, long P, int C, void* stream) {
  if (C % 4 || C > 256 || P <= 0) return ACC_EBADSHAPE;
  hipStream_t s = (hipStream_t)stream;
  const int R = ceil_div(P, LN_TOK_PER_BLOCK);
  hipLaunchKernelGGL(layernorm_bwd_kernel, dim3(R), dim3(256), 0, s, x, g, mr, dy, dx, part, P, C);
  // columns [0, C) -> dgamma, [C, 2C) -> dbeta (contiguous when dg, db are the halves of
  // one buffer; otherwise two launches)
  if (db == dg + C) {
    hipLaunchKernelGGL(colsum_rows_kernel, dim3(ceil_div(2 * C, 64)), dim3(1024), 0, s, part, R,
                       2 * C, dg);
  } else {
    return ACC_EBADARG;
  }
  return LAUNCH_OK;
}

extern "C" int accunet_gelu_fwd(const float* x, float* y, long n, void* stream) {
  if (n % 4) return ACC_EBADSHAPE;
  hipLaunchKernelGGL(gelu_fwd_kernel, dim3(nblk(n / 4)), dim3(256), 0, (hipStream_t)stream, x, y,
                     n / 4);
  return LAUNCH_OK;
}

extern "C" int accunet_gelu_bwd(const float* x, const float* dy, float* dx, long n, void* stream) {
  if (n % 4) return ACC_EBADSHAPE;
  hipLaunchKernelGGL(gelu_bwd_kernel, dim3(nblk(n / 4)), dim3(256), 0, (hipStream_t)stream, x, dy,
                     dx, n / 4);
  return LAUNCH_OK;
}

extern "C" int accunet_token_shift(const float* x, float* y, int B, int H, int W, int C, int axis,
                                   int dir, int shift_size, void* stream) {
  if (shift_size <= 0 || (axis != 0 && axis != 1) || (dir != 1 && dir != -1)) return ACC_EBADARG;
  const int chunk = (C + shift_size - 1) / shift_size;  // torch.chunk sizes
  hipLaunchKernelGGL(token_shift_kernel, dim3(nblk((long)B * H * W * C)), dim3(256), 0,
                     (hipStream_t)stream, x, y, B, H, W, C, axis, dir, chunk, shift_size / 2);
  return LAUNCH_OK;
}

extern "C" int accunet_up2_relu_add_fwd(const float* x, const float* skip, float* out,
                                        unsigned char* mask, int B, int H, int W, int C,
                                        void* stream) {
  hipLaunchKernelGGL(up2_relu_add_fwd_kernel, dim3(nblk((long)B * 4 * H * W * C)), dim3(256), 0,
                     (hipStream_t)stream, x, skip, out, mask, B, H, W, C);
  return LAUNCH_OK;
}

extern "C" int accunet_up2_relu_bwd(const float* dout, const unsigned char* mask, float* dx, int B,
                                    int H, int W, int C, void* stream) {
  hipLaunchKernelGGL(up2_relu_bwd_kernel, dim3(nblk((long)B * H * W * C)), dim3(256), 0,
                     (hipStream_t)stream, dout, mask, dx, B, H, W, C);
  return LAUNCH_OK;
}

extern "C" int accunet_relu(const float* x, const float* dy, float* y, long n, void* stream) {
  hipLaunchKernelGGL(relu_kernel, dim3(nblk(n)), dim3(256), 0, (hipStream_t)stream, x, dy, y, n);
  return LAUNCH_OK;
}

extern "C" int accunet_subsample2(const float* src, float* dst, int B, int H, int W, int C,
                                  int bwd, void* stream) {
  hipLaunchKernelGGL(subsample2_kernel, dim3(nblk((long)B * H * W * C)), dim3(256), 0,
                     (hipStream_t)stream, src, dst, B, H, W, C, bwd);
  return LAUNCH_OK;
}
