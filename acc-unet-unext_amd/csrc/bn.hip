// Training-mode BatchNorm2d (+LeakyReLU) on NHWC fp32 / bf16 activations, split into streaming
// passes whose per-channel statistics are reduced deterministically
// (per-block partials -> fixed-order reduction, fp64 final accumulation).
//
// Reference semantics (torch.nn.BatchNorm2d as used throughout
// ACC_UNet/ACC_UNet.py, e.g. :235-262): normalise with the biased batch
// variance, update running_mean / running_var with momentum 0.1 using the
// UNBIASED variance, eps = 1e-5; eval mode uses the running statistics.
#include "common.h"
#include "kernels.h"

#include "chan.h"

__global__ void inc_i64_kernel(long long* p) { *p += 1; }

// out[c] = sum_r part[r*stride + c], fp64 accumulation, c < ncols
__global__ void __launch_bounds__(256)
sum_rows_kernel(const float* __restrict__ part, int R, int stride, int ncols,
                float* __restrict__ out) {
  __shared__ double red[4][64];
  int cl = threadIdx.x & 63, g = threadIdx.x >> 6;
  int c = blockIdx.x * 64 + cl;
  double s1[1] = {0.0};
  if (c < ncols)
    ordered_strided_sum<8>(s1, g, R, 4, [&](int r, double (&v)[1]) {
      v[0] = (double)part[(long)r * stride + c];
    });
  red[g][cl] = s1[0];
  __syncthreads();
  if (g == 0 && c < ncols) out[c] = (float)(red[0][cl] + red[1][cl] + red[2][cl] + red[3][cl]);
}

template <typename TOUT>
__global__ void __launch_bounds__(256)
sum_rows_d_kernel(const double* __restrict__ part, int R, int stride, int ncols,
                  TOUT* __restrict__ out) {
  __shared__ double red[4][64];
  int cl = threadIdx.x & 63, g = threadIdx.x >> 6;
  int c = blockIdx.x * 64 + cl;
  double s1[1] = {0.0};
  if (c < ncols)
    ordered_strided_sum<8>(s1, g, R, 4, [&](int r, double (&v)[1]) {
      v[0] = part[(long)r * stride + c];
    });
  red[g][cl] = s1[0];
  __syncthreads();
  if (g == 0 && c < ncols) out[c] = (TOUT)(red[0][cl] + red[1][cl] + red[2][cl] + red[3][cl]);
}

// ---------------------------------------------------------------------------
// colreduce: out[r/RB][w] = sum of in[r][w] over RB consecutive rows (stage 1 of
// the partial-statistics reduction when there are many partial rows).
// ---------------------------------------------------------------------------
template <typename T>
__global__ void __launch_bounds__(256)
colreduce_kernel(const T* __restrict__ in, T* __restrict__ out, int R, int Wd, int RB) {
  __shared__ T red[4][64];
  int c = blockIdx.y * 64 + (threadIdx.x & 63);
  int g = threadIdx.x >> 6;
  int r0 = blockIdx.x * RB;
  int r1 = min(R, r0 + RB);
  T s[1] = {0};
  if (c < Wd)
    ordered_strided_sum<8>(s, r0 + g, r1, 4, [&](int r, T (&v)[1]) { v[0] = in[(long)r * Wd + c]; });
  red[g][threadIdx.x & 63] = s[0];
  __syncthreads();
  if (g == 0 && c < Wd) out[(long)blockIdx.x * Wd + c] = red[0][threadIdx.x] + red[1][threadIdx.x] +
                                                     red[2][threadIdx.x] + red[3][threadIdx.x];
}

// Reduce [R][Wd] partial rows into at most 64 rows using ws; returns pointer+rows.
template <typename T>
const T* reduce_partials_t(const T* part, int R, int Wd, T* ws, int* Rout, hipStream_t s) {
  const T* cur = part;
  int rows = R;
  T* bufs[2] = {ws, ws + (size_t)ceil_div(R, 32) * Wd};
  int which = 0;
  while (rows > 64) {
    const int RB = 32;  // many small blocks: the reduction is latency-, not bandwidth-bound
    int nb = ceil_div(rows, RB);
    hipLaunchKernelGGL(colreduce_kernel<T>, dim3(nb, ceil_div(Wd, 64)), dim3(256), 0, s, cur,
                       bufs[which], rows, Wd, RB);
    cur = bufs[which];
    which ^= 1;
    rows = nb;
  }
  *Rout = rows;
  return cur;
}

const float* reduce_partials(const float* part, int R, int Wd, float* ws, int* Rout,
                             hipStream_t s) {
  return reduce_partials_t<float>(part, R, Wd, ws, Rout, s);
}

const double* reduce_partials_d(const double* part, int R, int Wd, double* ws, int* Rout,
                                hipStream_t s) {
  return reduce_partials_t<double>(part, R, Wd, ws, Rout, s);
}

void sum_rows_d_to_f(const double* pr, int rows, int stride, int ncols, float* out,
                     hipStream_t s) {
  hipLaunchKernelGGL(sum_rows_d_kernel<float>, dim3(ceil_div(ncols, 64)), dim3(256), 0, s, pr,
                     rows, stride, ncols, out);
}

size_t accunet_partials_ws_elems(int R, int Wd) {
  int r1 = ceil_div(R, 32);
  return (size_t)(r1 + ceil_div(r1, 32) + 2) * Wd;
}

// ---------------------------------------------------------------------------
// bn_finalize: partial (sum, sumsq) rows -> mean, rstd, scale, shift; running
// statistics update (training) or running-stat normalisation (eval).
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256)
bn_finalize_kernel(const double* __restrict__ part, int R, int C, double count,
                   const float* __restrict__ gamma, const float* __restrict__ beta,
                   float* __restrict__ rmean, float* __restrict__ rvar, float momentum, float eps,
                   int training, float* __restrict__ st, long long* __restrict__ nbt) {
  __shared__ double red[2][4][64];
  int cl = threadIdx.x & 63, g = threadIdx.x >> 6;
  int c = blockIdx.x * 64 + cl;
  if (nbt && blockIdx.x == 0 && threadIdx.x == 0) *nbt += 1;  // num_batches_tracked
  double s[2] = {0.0, 0.0};
  if (training && c < C)
    ordered_strided_sum<8>(s, g, R, 4, [&](int r, double (&v)[2]) {
      v[0] = part[(long)r * 2 * C + c];
      v[1] = part[(long)r * 2 * C + C + c];
    });
  double s1 = s[0], s2 = s[1];
  red[0][g][cl] = s1;
  red[1][g][cl] = s2;
  __syncthreads();
  if (g != 0 || c >= C) return;
  float mean, var;
  if (training) {
    s1 = red[0][0][cl] + red[0][1][cl] + red[0][2][cl] + red[0][3][cl];
    s2 = red[1][0][cl] + red[1][1][cl] + red[1][2][cl] + red[1][3][cl];
    double m = s1 / count;
    double v = s2 / count - m * m;
    if (v < 0.0) v = 0.0;
    mean = (float)m;
    var = (float)v;
    if (rmean) rmean[c] = (1.f - momentum) * rmean[c] + momentum * mean;
    if (rvar) {
      double unb = count > 1.0 ? v * count / (count - 1.0) : v;
      rvar[c] = (1.f - momentum) * rvar[c] + momentum * (float)unb;
    }
  } else {
    mean = rmean[c];
    var = rvar[c];
  }
  float rstd = 1.0f / sqrtf(var + eps);
  float ga = gamma ? gamma[c] : 1.f;
  float be = beta ? beta[c] : 0.f;
  float sc = ga * rstd;
  st[BN_MEAN * C + c] = mean;
  st[BN_RSTD * C + c] = rstd;
  st[BN_SCALE * C + c] = sc;
  st[BN_SHIFT * C + c] = be - mean * sc;
}

extern "C" int accunet_bn_finalize(const double* part, int R, int C, double count,
                                   const float* gamma, const float* beta, float* rmean,
                                   float* rvar, long long* nbt, float momentum, float eps,
                                   int training, float* st, double* ws, void* stream_) {
  hipStream_t s = (hipStream_t)stream_;
  if (C <= 0) return ACC_EBADSHAPE;
  int rows = R;
  const double* p = part;
  if (training) p = reduce_partials_t<double>(part, R, 2 * C, ws, &rows, s);
  hipLaunchKernelGGL(bn_finalize_kernel, dim3(ceil_div(C, 64)), dim3(256), 0, s, p, rows, C,
                     count, gamma, beta, rmean, rvar, momentum, eps, training, st,
                     training ? nbt : nullptr);
  return hipGetLastError() == hipSuccess ? ACC_OK : ACC_ELAUNCH;
}


// ---------------------------------------------------------------------------
// affine_act: y = act(x*scale[c] + shift[c]) (+ res), optional partial stats of y
// ---------------------------------------------------------------------------
template <int V, typename T>
__global__ void __launch_bounds__(256)
affine_act_kernel(const T* __restrict__ x, const float* __restrict__ sc,
                  const float* __restrict__ sh, int act, const T* __restrict__ res,
                  T* __restrict__ y, long P, int C, double* __restrict__ stats) {
  ChanTile t = chan_tile<V>(C);
  long rows_per = (P + gridDim.x - 1) / gridDim.x;
  long r0 = blockIdx.x * rows_per, r1 = min(P, r0 + rows_per);
  double a[V], b[V];
#pragma unroll
  for (int j = 0; j < V; ++j) { a[j] = 0.0; b[j] = 0.0; }
  if (t.active) {
    float s[V], h[V];
#pragma unroll
    for (int j = 0; j < V; ++j) {
      s[j] = sc ? sc[t.c0 + j] : 1.f;
      h[j] = sh ? sh[t.c0 + j] : 0.f;
    }
    // rows are processed U at a time with all their loads issued first, so each
    // thread keeps 2U-4U 16-byte loads in flight (latency hiding at 4 blocks/CU)
    constexpr int U = 4;
    for (long rb = r0 + t.rg; rb < r1; rb += U * t.RG) {
      float v[U][V], q[U][V];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        long r = rb + (long)u * t.RG;
        if (r < r1) {
          ldv<V>(x + r * C + t.c0, v[u]);
          if (res) ldv<V>(res + r * C + t.c0, q[u]);
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        long r = rb + (long)u * t.RG;
        if (r < r1) {
#pragma unroll
          for (int j = 0; j < V; ++j) {
            v[u][j] = apply_act(v[u][j] * s[j] + h[j], act);
            if (res) v[u][j] += q[u][j];
          }
          if (y) stv_r<V>(y + r * C + t.c0, v[u]);  // y == nullptr: statistics only (accunet_colsum)
#pragma unroll
          for (int j = 0; j < V; ++j) { a[j] += v[u][j]; b[j] += (double)v[u][j] * v[u][j]; }
        }
      }
    }
  }
  if (stats) block_chan_reduce2<V>(t, a, b, stats, blockIdx.x, C);
}

int stream_rowblocks(long P, int C) {
  long elems = P * (long)C;
  long want = elems / (256 * 16);  // ~16 elements per thread
  if (want < 1) want = 1;
  if (want > 1024) want = 1024;
  if (want > P) want = P;
  return (int)want;
}

extern "C" int accunet_affine_act_fwd(const void* x, const float* sc, const float* sh, int act,
                                      const void* res, void* y, long P, int C, double* stats,
                                      int* stats_rows, int dt, void* stream_) {
  hipStream_t s = (hipStream_t)stream_;
  int V = (C % 4 == 0) ? 4 : 1;
  int CQ = C / V;
  int nb = stream_rowblocks(P, C);
  if (stats_rows) *stats_rows = nb;
  dim3 grid(nb, ceil_div(CQ, 64));
  if (with_dt(dt, [&](auto tag) {
        using T = decltype(tag);
        if (V == 4)
          hipLaunchKernelGGL((affine_act_kernel<4, T>), grid, dim3(256), 0, s, (const T*)x, sc, sh,
                             act, (const T*)res, (T*)y, P, C, stats);
        else
          hipLaunchKernelGGL((affine_act_kernel<1, T>), grid, dim3(256), 0, s, (const T*)x, sc, sh,
                             act, (const T*)res, (T*)y, P, C, stats);
      }))
    return ACC_EBADARG;
  return hipGetLastError() == hipSuccess ? ACC_OK : ACC_ELAUNCH;
}

extern "C" int accunet_stream_rows(long P, int C) { return stream_rowblocks(P, C); }

// ---------------------------------------------------------------------------
// BatchNorm(+act) backward.
//   pre = x*scale + shift, g = dy * act'(pre), xhat = (x-mean)*rstd
//   reduce:   partial (sum g, sum g*xhat) per channel
//   finalize: dgamma, dbeta, dx = k1*g + k2*x + k3
//   apply:    dx (optionally accumulated), optional partial column sums of dx
// ---------------------------------------------------------------------------
template <int V, typename T>
__global__ void __launch_bounds__(256)
bn_bwd_reduce_kernel(const T* __restrict__ x, const T* __restrict__ dy,
                     const float* __restrict__ st, int act, long P, int C,
                     double* __restrict__ part) {
  // fp64 accumulation, as ATen's CPU batch_norm backward (acc_type<float> = double)
  ChanTile t = chan_tile<V>(C);
  long rows_per = (P + gridDim.x - 1) / gridDim.x;
  long r0 = blockIdx.x * rows_per, r1 = min(P, r0 + rows_per);
  double a[V], b[V];
#pragma unroll
  for (int j = 0; j < V; ++j) { a[j] = 0.0; b[j] = 0.0; }
  if (t.active) {
    float mu[V], rs[V], s[V], h[V];
#pragma unroll
    for (int j = 0; j < V; ++j) {
      mu[j] = st[BN_MEAN * C + t.c0 + j];
      rs[j] = st[BN_RSTD * C + t.c0 + j];
      s[j] = st[BN_SCALE * C + t.c0 + j];
      h[j] = st[BN_SHIFT * C + t.c0 + j];
    }
    constexpr int U = 4;  // see affine_act_kernel
    for (long rb = r0 + t.rg; rb < r1; rb += U * t.RG) {
      float xv[U][V], dv[U][V];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        long r = rb + (long)u * t.RG;
        if (r < r1) {
          ldv<V>(x + r * C + t.c0, xv[u]);
          ldv<V>(dy + r * C + t.c0, dv[u]);
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (rb + (long)u * t.RG < r1) {
#pragma unroll
          for (int j = 0; j < V; ++j) {
            float g = dv[u][j];
            if (act == ACT_LRELU) g *= lrelu_d(xv[u][j] * s[j] + h[j]);
            a[j] += g;
            b[j] += (double)g * ((double)xv[u][j] - mu[j]) * rs[j];
          }
        }
      }
    }
  }
  block_chan_reduce2<V>(t, a, b, part, blockIdx.x, C);
}

__global__ void __launch_bounds__(256)
bn_bwd_finalize_kernel(const double* __restrict__ part, int R, int C, double count,
                       const float* __restrict__ st, const float* __restrict__ gamma,
                       int training, float* __restrict__ dgamma, float* __restrict__ dbeta,
                       float* __restrict__ coef, int xc_form) {
  __shared__ double red[2][4][64];
  int cl = threadIdx.x & 63, g = threadIdx.x >> 6;
  int c = blockIdx.x * 64 + cl;
  double s[2] = {0.0, 0.0};
  if (c < C)
    ordered_strided_sum<8>(s, g, R, 4, [&](int r, double (&v)[2]) {
      v[0] = part[(long)r * 2 * C + c];
      v[1] = part[(long)r * 2 * C + C + c];
    });
  double s1 = s[0], s2 = s[1];
  red[0][g][cl] = s1;
  red[1][g][cl] = s2;
  __syncthreads();
  if (g != 0 || c >= C) return;
  s1 = red[0][0][cl] + red[0][1][cl] + red[0][2][cl] + red[0][3][cl];
  s2 = red[1][0][cl] + red[1][1][cl] + red[1][2][cl] + red[1][3][cl];
  // producer-side partials carry sum g*(x - mean): scale to sum g*xhat
  if (xc_form) s2 *= (double)st[BN_RSTD * C + c];
  if (dgamma) dgamma[c] = (float)s2;
  if (dbeta) dbeta[c] = (float)s1;
  float ga = gamma ? gamma[c] : 1.f;
  float rstd = st[BN_RSTD * C + c];
  float mean = st[BN_MEAN * C + c];
  float k1 = ga * rstd;
  float k2 = 0.f, k3 = 0.f;
  (void)mean;
  if (training) {
    // dx = k1*(g - mean(g) - xhat*mean(g*xhat)) = k1*g + k2*(x - mean) + k3
    float mg = (float)(s1 / count), mgx = (float)(s2 / count);
    k2 = -k1 * rstd * mgx;
    k3 = -k1 * mg;
  }
  coef[c] = k1;
  coef[C + c] = k2;
  coef[2 * C + c] = k3;
}

template <int V, typename T>
__global__ void __launch_bounds__(256)
bn_bwd_apply_kernel(const T* __restrict__ x, const T* __restrict__ dy,
                    const float* __restrict__ st, const float* __restrict__ coef, int act,
                    long P, int C, T* __restrict__ dx, int accumulate,
                    double* __restrict__ colsum) {
  ChanTile t = chan_tile<V>(C);
  long rows_per = (P + gridDim.x - 1) / gridDim.x;
  long r0 = blockIdx.x * rows_per, r1 = min(P, r0 + rows_per);
  // optional fp64 column sums of the written d: sum_p dx = the bias gradient of the
  // convolution that produced x (its output feeds only this BatchNorm)
  double a[V], b[V];
#pragma unroll
  for (int j = 0; j < V; ++j) { a[j] = 0.0; b[j] = 0.0; }
  if (t.active) {
    float s[V], h[V], k1[V], k2[V], k3[V], mu[V];
#pragma unroll
    for (int j = 0; j < V; ++j) {
      mu[j] = st[BN_MEAN * C + t.c0 + j];
      s[j] = st[BN_SCALE * C + t.c0 + j];
      h[j] = st[BN_SHIFT * C + t.c0 + j];
      k1[j] = coef[t.c0 + j];
      k2[j] = coef[C + t.c0 + j];
      k3[j] = coef[2 * C + t.c0 + j];
    }
    constexpr int U = 4;  // see affine_act_kernel
    for (long rb = r0 + t.rg; rb < r1; rb += U * t.RG) {
      float xv[U][V], dv[U][V], o[U][V];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        long r = rb + (long)u * t.RG;
        if (r < r1) {
          ldv<V>(x + r * C + t.c0, xv[u]);
          ldv<V>(dy + r * C + t.c0, dv[u]);
          if (accumulate) ldv<V>(dx + r * C + t.c0, o[u]);
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        long r = rb + (long)u * t.RG;
        if (r < r1) {
#pragma unroll
          for (int j = 0; j < V; ++j) {
            float g = dv[u][j];
            if (act == ACT_LRELU) g *= lrelu_d(xv[u][j] * s[j] + h[j]);
            float d = k1[j] * g + k2[j] * (xv[u][j] - mu[j]) + k3[j];
            // statistics describe the stored tensor (bf16: the rounded value)
            const float dd = rnd<T>(d);
            if (colsum) a[j] += accumulate ? d : dd;
            o[u][j] = accumulate ? rnd<T>(o[u][j] + d) : dd;
          }
          stv<V>(dx + r * C + t.c0, o[u]);
        }
      }
    }
  }
  if (colsum) block_chan_reduce2<V>(t, a, b, colsum, blockIdx.x, C);
}

extern "C" size_t accunet_bn_bwd_ws_elems(long P, int C) {
  int nb = stream_rowblocks(P, C);
  return (size_t)nb * 2 * C * 2 + accunet_partials_ws_elems(nb, 2 * C) * 2 + 3 * (size_t)C;
}

// dsum (optional, [C]): sum over pixels of dx (fp64 partials in the apply pass, reduced
// after it into the stats workspace, which the finalize no longer needs by then)
static void bn_dsum_finish(double* part, int nb, int C, double* scratch, float* dsum,
                           hipStream_t s) {
  int rows;
  const double* pr = reduce_partials_t<double>(part, nb, 2 * C, scratch, &rows, s);
  hipLaunchKernelGGL(sum_rows_d_kernel<float>, dim3(ceil_div(C, 64)), dim3(256), 0, s, pr, rows,
                     2 * C, C, dsum);
}

extern "C" int accunet_bn_bwd(const void* x, const void* dy, const float* st,
                              const float* gamma, int act, int training, long P, int C,
                              void* dx, int accumulate, float* dgamma, float* dbeta,
                              float* dsum, float* ws, size_t ws_elems, int dt, void* stream_) {
  hipStream_t s = (hipStream_t)stream_;
  int V = (C % 4 == 0) ? 4 : 1;
  int nb = stream_rowblocks(P, C);
  dim3 grid(nb, ceil_div(C / V, 64));
  // ws layout (floats): fp64 partials [nb][2][C] | fp64 reduce scratch | coef [3][C]
  size_t part_f = (size_t)nb * 2 * C * 2;
  size_t scr_f = accunet_partials_ws_elems(nb, 2 * C) * 2;
  if (part_f + scr_f + 3 * (size_t)C > ws_elems) return ACC_EBADARG;
  if ((uintptr_t)ws & 7) return ACC_EBADARG;
  double* part = reinterpret_cast<double*>(ws);
  double* scratch = reinterpret_cast<double*>(ws + part_f);
  float* coef = ws + part_f + scr_f;
  if (dt != ACC_F32 && dt != ACC_BF16) return ACC_EBADARG;
  with_dt(dt, [&](auto tag) {
    using T = decltype(tag);
    if (V == 4)
      hipLaunchKernelGGL((bn_bwd_reduce_kernel<4, T>), grid, dim3(256), 0, s, (const T*)x,
                         (const T*)dy, st, act, P, C, part);
    else
      hipLaunchKernelGGL((bn_bwd_reduce_kernel<1, T>), grid, dim3(256), 0, s, (const T*)x,
                         (const T*)dy, st, act, P, C, part);
  });
  int rows;
  const double* pr = reduce_partials_t<double>(part, nb, 2 * C, scratch, &rows, s);
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3(ceil_div(C, 64)), dim3(256), 0, s, pr, rows, C,
                     (double)P, st, gamma, training, dgamma, dbeta, coef, 0);
  double* cpart = dsum ? part : nullptr;  // the reduce partials are consumed by now
  with_dt(dt, [&](auto tag) {
    using T = decltype(tag);
    if (V == 4)
      hipLaunchKernelGGL((bn_bwd_apply_kernel<4, T>), grid, dim3(256), 0, s, (const T*)x,
                         (const T*)dy, st, coef, act, P, C, (T*)dx, accumulate, cpart);
    else
      hipLaunchKernelGGL((bn_bwd_apply_kernel<1, T>), grid, dim3(256), 0, s, (const T*)x,
                         (const T*)dy, st, coef, act, P, C, (T*)dx, accumulate, cpart);
  });
  if (dsum) bn_dsum_finish(part, nb, C, scratch, dsum, s);
  return hipGetLastError() == hipSuccess ? ACC_OK : ACC_ELAUNCH;
}

// BatchNorm backward whose reduce pass ran in the producer of dy (GEMM / depthwise
// data-gradient epilogues): part = [R][2][C] (sum g, sum g*(x - mean)).
// coef [3][C] floats, padded to an even count so what follows stays 8-byte aligned
static size_t bn_coef_floats(int C) { return ((3 * (size_t)C + 1) / 2) * 2; }

// ws (floats): fp64 reduce scratch (R rows) | coef [3][C] (even pad) | fp64 dsum partials
// [nb][2][C] | fp64 dsum reduce scratch; nb = stream_rowblocks(P, C)
static size_t bn_bwd_part_ws(long P, int R, int C) {
  const int nb = stream_rowblocks(P, C);
  return accunet_partials_ws_elems(R, 2 * C) * 2 + bn_coef_floats(C) + (size_t)nb * 2 * C * 2 +
         accunet_partials_ws_elems(nb, 2 * C) * 2;
}
extern "C" size_t accunet_bn_bwd_part_ws_elems(long P, int R, int C) {
  return bn_bwd_part_ws(P, R, C);
}

extern "C" int accunet_bn_bwd_part(const void* x, const void* dy, const float* st,
                                   const float* gamma, int act, int training, long P, int C,
                                   const double* part, int R, void* dx, float* dgamma,
                                   float* dbeta, float* dsum, float* ws, size_t ws_elems, int dt,
                                   void* stream_) {
  hipStream_t s = (hipStream_t)stream_;
  if (C <= 0 || R <= 0) return ACC_EBADSHAPE;
  if (dt != ACC_F32 && dt != ACC_BF16) return ACC_EBADARG;
  if (ws_elems < bn_bwd_part_ws(P, R, C) || ((uintptr_t)ws & 7)) return ACC_EBADARG;
  const int V = (C % 4 == 0) ? 4 : 1;
  const int nb = stream_rowblocks(P, C);
  dim3 grid(nb, ceil_div(C / V, 64));
  const size_t scr_f = accunet_partials_ws_elems(R, 2 * C) * 2;
  double* scratch = reinterpret_cast<double*>(ws);
  float* coef = ws + scr_f;
  double* cpart = reinterpret_cast<double*>(ws + scr_f + bn_coef_floats(C));
  double* cscr = cpart + (size_t)nb * 2 * C;
  int rows;
  const double* pr = reduce_partials_t<double>(part, R, 2 * C, scratch, &rows, s);
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3(ceil_div(C, 64)), dim3(256), 0, s, pr, rows, C,
                     (double)P, st, gamma, training, dgamma, dbeta, coef, 1);
  with_dt(dt, [&](auto tag) {
    using T = decltype(tag);
    if (V == 4)
      hipLaunchKernelGGL((bn_bwd_apply_kernel<4, T>), grid, dim3(256), 0, s, (const T*)x,
                         (const T*)dy, st, coef, act, P, C, (T*)dx, 0, dsum ? cpart : nullptr);
    else
      hipLaunchKernelGGL((bn_bwd_apply_kernel<1, T>), grid, dim3(256), 0, s, (const T*)x,
                         (const T*)dy, st, coef, act, P, C, (T*)dx, 0, dsum ? cpart : nullptr);
  });
  if (dsum) bn_dsum_finish(cpart, nb, C, cscr, dsum, s);
  return hipGetLastError() == hipSuccess ? ACC_OK : ACC_ELAUNCH;
}

// ---------------------------------------------------------------------------
// Column sums (conv bias gradients when no BN-backward pass precedes them).
// ---------------------------------------------------------------------------
extern "C" int accunet_colsum(const void* x, long P, int C, float* out, double* ws,
                              size_t ws_elems, int dt, void* stream_) {
  hipStream_t s = (hipStream_t)stream_;
  int V = (C % 4 == 0) ? 4 : 1;
  int nb = stream_rowblocks(P, C);
  dim3 grid(nb, ceil_div(C / V, 64));
  double* part = ws;
  double* scratch = ws + (size_t)nb * 2 * C;
  if ((size_t)nb * 2 * C + accunet_partials_ws_elems(nb, 2 * C) > ws_elems) return ACC_EBADARG;
  if (with_dt(dt, [&](auto tag) {
        using T = decltype(tag);
        if (V == 4)
          hipLaunchKernelGGL((affine_act_kernel<4, T>), grid, dim3(256), 0, s, (const T*)x, nullptr,
                             nullptr, ACT_NONE, nullptr, nullptr, P, C, part);
        else
          hipLaunchKernelGGL((affine_act_kernel<1, T>), grid, dim3(256), 0, s, (const T*)x, nullptr,
                             nullptr, ACT_NONE, nullptr, nullptr, P, C, part);
      }))
    return ACC_EBADARG;
  int rows;
  const double* pr = reduce_partials_t<double>(part, nb, 2 * C, scratch, &rows, s);
  hipLaunchKernelGGL(sum_rows_d_kernel<float>, dim3(ceil_div(C, 64)), dim3(256), 0, s, pr, rows,
                     2 * C, C, out);
  return hipGetLastError() == hipSuccess ? ACC_OK : ACC_ELAUNCH;
}

// Reduce a partial-stats block [R][2][C] to totals [2][C] (fp64).
extern "C" int accunet_reduce_stats(const double* part, int R, int C, double* out2C, double* ws,
                                    void* stream_) {
  hipStream_t s = (hipStream_t)stream_;
  int rows;
  const double* pr = reduce_partials_t<double>(part, R, 2 * C, ws, &rows, s);
  hipLaunchKernelGGL(sum_rows_d_kernel<double>, dim3(ceil_div(2 * C, 64)), dim3(256), 0, s, pr,
                     rows, 2 * C, 2 * C, out2C);
  return hipGetLastError() == hipSuccess ? ACC_OK : ACC_ELAUNCH;
}
