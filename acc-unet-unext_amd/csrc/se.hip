// Squeeze-and-excitation gate fused with the BatchNorm(+LeakyReLU) that precedes it
// and the BatchNorm + LeakyReLU inside it: ChannelSELayer.forward,
// reference ACC_UNet/ACC_UNet.py:37-49 (r = 8, LeakyReLU after fc1, BN + LeakyReLU
// after the gating), always fed by lrelu(bn(conv(...))) in HANCBlock (:281-284),
// ResPath (:326), Conv2d_batchnorm (:183-186) and MLFC (:522-525).
//
// Forward (K3 "SE gate"), z = pending input, a = act(z*sc1+sh1) (or a = z):
//   pass 1 (se_reduce): per-(b,c) S = sum_hw a, Q = sum_hw a^2      [reads z once]
//   mid   (se_mid_sample, one block per sample): S, Q from the chunk partials,
//                      m = S/HW, s = sigmoid(fc2(lrelu(fc1(m))))
//   mid   (se_mid_bn, one thread per channel): BN stats of y = a*s derived exactly
//                      from (S, Q, s): mean = sum_b s*S / n,  E[y^2] = sum_b s^2*Q / n
//                      -> per-(b,c) alpha = gamma*rstd*s, per-c beta' = beta - gamma*rstd*mean
//   pass 2 (se_apply): out = lrelu(alpha*a + beta')                [reads z, writes out]
// so neither a nor y = a*s is ever materialised.
//
// Backward:
//   pass 1: per-(b,c) T1 = sum g2, T2 = sum g2*a   (g2 = dout * lrelu'(alpha*a+beta'))
//   mid:    BN backward reduced to per-(b,c) terms, SE fc backward, and coefficients of
//           da = A*g2 + Bc*a + Cc
//   pass 2: da (then the caller runs the preceding BatchNorm's backward on it)
#include "common.h"
#include "chan.h"
#include "kernels.h"

struct SeGeom {
  int B, HW, C, NCH;
  long rows_per;  // rows per chunk
};

// Forward state saved for the backward (one float buffer, doubles first):
//   S[B*C], Q[B*C] (fp64: per-(b,c) sum a, sum a^2), then fp32 hpre[B*Cr], s[B*C],
//   mean[C], rstd[C], alpha[B*C], betap[C]
struct SeSave {
  double* S;
  double* Q;
  float *hpre, *sg, *mean, *rstd, *alpha, *betap;
};

ACC_DEV SeSave se_save_view(float* base, int B, int C, int Cr) {
  SeSave v;
  v.S = reinterpret_cast<double*>(base);
  v.Q = v.S + (size_t)B * C;
  float* f = reinterpret_cast<float*>(v.Q + (size_t)B * C);
  v.hpre = f;
  v.sg = v.hpre + (size_t)B * Cr;
  v.mean = v.sg + (size_t)B * C;
  v.rstd = v.mean + C;
  v.alpha = v.rstd + C;
  v.betap = v.alpha + (size_t)B * C;
  return v;
}

static size_t se_save_floats(int B, int C, int Cr) {
  return (size_t)B * C * 4 + (size_t)B * Cr + (size_t)B * C * 2 + 3 * (size_t)C;
}
static size_t se_alpha_offset(int B, int C, int Cr) {  // floats
  return (size_t)B * C * 4 + (size_t)B * Cr + (size_t)B * C + 2 * (size_t)C;
}

static SeGeom se_geom(int B, int HW, int C) {
  SeGeom g;
  g.B = B;
  g.HW = HW;
  g.C = C;
  int want = 1024 / (B > 0 ? B : 1);
  int maxch = HW / 32;
  if (maxch < 1) maxch = 1;
  g.NCH = want < maxch ? want : maxch;
  if (g.NCH < 1) g.NCH = 1;
  g.rows_per = (HW + g.NCH - 1) / g.NCH;
  return g;
}

// pass 1 forward: partials part[(b*NCH + chunk)][2][C] of (sum a, sum a^2)
template <int V, typename T>
__global__ void __launch_bounds__(256)
se_reduce_kernel(const T* __restrict__ z, const float* __restrict__ sc,
                 const float* __restrict__ sh, int act, SeGeom g, double* __restrict__ part) {
  ChanTile t = chan_tile<V>(g.C);
  const int b = blockIdx.x / g.NCH, ch = blockIdx.x % g.NCH;
  long r0 = (long)b * g.HW + ch * g.rows_per;
  long r1 = min((long)b * g.HW + g.HW, r0 + g.rows_per);
  double a[V], q[V];
#pragma unroll
  for (int j = 0; j < V; ++j) { a[j] = 0.0; q[j] = 0.0; }
  if (t.active) {
    float s[V], h[V];
#pragma unroll
    for (int j = 0; j < V; ++j) {
      s[j] = sc ? sc[t.c0 + j] : 1.f;
      h[j] = sh ? sh[t.c0 + j] : 0.f;
    }
    const bool pro = sc != nullptr;
    for (long r = r0 + t.rg; r < r1; r += t.RG) {
      float v[V];
      ldv<V>(z + r * g.C + t.c0, v);
#pragma unroll
      for (int j = 0; j < V; ++j) {
        double x = pro ? apply_act(v[j] * s[j] + h[j], act) : v[j];
        a[j] += x;
        q[j] += x * x;
      }
    }
  }
  block_chan_reduce2<V>(t, a, q, part, blockIdx.x, g.C);
}

// chunk partials [B*NCH][N][C] -> per-(b,c) sums out[i][B*C] (i < N): block = 64
// channels x 4 chunk groups of one sample; each group sums its chunks in order, the 4
// group sums are added in order.
template <int N>
__global__ void __launch_bounds__(256)
se_part_sum_kernel(const double* __restrict__ part, SeGeom g, double* __restrict__ out) {
  __shared__ double r[N][4][64];
  const int C = g.C, b = blockIdx.y, t = threadIdx.x;
  const int c = blockIdx.x * 64 + (t & 63), grp = t >> 6;
  double s[N];
#pragma unroll
  for (int i = 0; i < N; ++i) s[i] = 0.0;
  if (c < C)
    ordered_strided_sum<4>(s, grp, g.NCH, 4, [&](int k, double (&v)[N]) {
      const double* pr = part + ((long)(b * g.NCH + k) * N) * C;
#pragma unroll
      for (int i = 0; i < N; ++i) v[i] = pr[(long)i * C + c];
    });
#pragma unroll
  for (int i = 0; i < N; ++i) r[i][grp][t & 63] = s[i];
  __syncthreads();
  if (grp == 0 && c < C) {
    const long BC = (long)g.B * C;
#pragma unroll
    for (int i = 0; i < N; ++i)
      out[i * BC + b * C + c] = ((r[i][0][t] + r[i][1][t]) + r[i][2][t]) + r[i][3][t];
  }
}

// mid forward, fused per sample (one block per sample b): the chunk partials of b
// -> S[b,c], Q[b,c] (same fixed summation order as se_part_sum_kernel: 4 chunk
// groups k = grp mod 4, each in chunk order, then ((g0 + g1) + g2) + g3), then the
// channel means, fc1 (+LeakyReLU) and fc2 (+sigmoid) of that sample (as
// the reference gate, :41-45). One launch for the whole per-sample middle step.
__global__ void __launch_bounds__(256)
se_mid_sample_kernel(const double* __restrict__ part, SeGeom g, int Cr,
                     const float* __restrict__ w1, const float* __restrict__ b1,
                     const float* __restrict__ w2, const float* __restrict__ b2,
                     float* __restrict__ save) {
  extern __shared__ __attribute__((aligned(16))) float sm[];  // m[C] | h'[Cr]
  __shared__ double r[2][4][64];
  const int B = g.B, C = g.C, b = blockIdx.x, tid = threadIdx.x;
  SeSave sv = se_save_view(save, B, C, Cr);
  float* m = sm;
  float* hp = sm + C;
  const int cl = tid & 63, grp = tid >> 6;
  for (int cb = 0; cb < C; cb += 64) {
    const int c = cb + cl;
    double s2[2] = {0.0, 0.0};
    if (c < C)
      ordered_strided_sum<8>(s2, grp, g.NCH, 4, [&](int k, double (&v)[2]) {
        const double* pr = part + ((long)(b * g.NCH + k) * 2) * C;
        v[0] = pr[c];
        v[1] = pr[(long)C + c];
      });
    r[0][grp][cl] = s2[0];
    r[1][grp][cl] = s2[1];
    __syncthreads();
    if (grp == 0 && c < C) {
      const double S = ((r[0][0][cl] + r[0][1][cl]) + r[0][2][cl]) + r[0][3][cl];
      const double Q = ((r[1][0][cl] + r[1][1][cl]) + r[1][2][cl]) + r[1][3][cl];
      sv.S[b * C + c] = S;
      sv.Q[b * C + c] = Q;
      m[c] = (float)(S / g.HW);
    }
    __syncthreads();
  }
  // fc1: 4 threads per output, interleaved over the input channels
  for (int o = tid; o < Cr * 4; o += 256) {
    int j = o >> 2, part_i = o & 3;
    float acc = 0.f;
    const float* wr = w1 + (long)j * C;
    #pragma unroll 8
    for (int c = part_i; c < C; c += 4) acc = fmaf(wr[c], m[c], acc);
    acc += __shfl_xor(acc, 1);
    acc += __shfl_xor(acc, 2);
    if (part_i == 0) {
      acc += b1[j];
      sv.hpre[b * Cr + j] = acc;
      hp[j] = lrelu(acc);
    }
  }
  __syncthreads();
  for (int c = tid; c < C; c += 256) {
    float acc = b2[c];
    const float* wr = w2 + (long)c * Cr;
    #pragma unroll 8
    for (int j = 0; j < Cr; ++j) acc = fmaf(wr[j], hp[j], acc);
    sv.sg[b * C + c] = 1.f / (1.f + expf(-acc));
  }
}

// mid forward, part 2: one thread per channel — BatchNorm statistics of y = a*s
// derived from (S, Q, s), running-stat update, per-(b,c) coefficients.
__global__ void __launch_bounds__(256)
se_mid_bn_kernel(SeGeom g, int Cr, const float* __restrict__ gamma,
                 const float* __restrict__ beta, float* __restrict__ rmean,
                 float* __restrict__ rvar, float momentum, float eps, int training,
                 float* __restrict__ save, long long* __restrict__ nbt) {
  const int B = g.B, C = g.C;
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (nbt && c == 0) *nbt += 1;  // num_batches_tracked (training only; null otherwise)
  if (c >= C) return;
  SeSave sv = se_save_view(save, B, C, Cr);
  const double n = (double)B * g.HW;
  float mu, var;
  if (training) {
    double m1 = 0.0, m2 = 0.0;
    #pragma unroll 8
    for (int b = 0; b < B; ++b) {
      double s = sv.sg[b * C + c];
      m1 += s * sv.S[b * C + c];
      m2 += s * s * sv.Q[b * C + c];
    }
    m1 /= n;
    m2 = m2 / n - m1 * m1;
    if (m2 < 0.0) m2 = 0.0;
    mu = (float)m1;
    var = (float)m2;
    if (rmean) rmean[c] = (1.f - momentum) * rmean[c] + momentum * mu;
    if (rvar) rvar[c] = (1.f - momentum) * rvar[c] + momentum * (float)(m2 * n / (n - 1.0));
  } else {
    mu = rmean[c];
    var = rvar[c];
  }
  float rs = 1.f / sqrtf(var + eps);
  float k = gamma[c] * rs;
  sv.mean[c] = mu;
  sv.rstd[c] = rs;
  sv.betap[c] = beta[c] - k * mu;
  #pragma unroll 8
  for (int b = 0; b < B; ++b) sv.alpha[b * C + c] = k * sv.sg[b * C + c];
}

// pass 2 forward: out = lrelu(alpha[b,c]*a + betap[c])
template <int V, typename T>
__global__ void __launch_bounds__(256)
se_apply_kernel(const T* __restrict__ z, const float* __restrict__ sc,
                const float* __restrict__ sh, int act, SeGeom g, const float* __restrict__ alpha,
                const float* __restrict__ betap, T* __restrict__ out,
                double* __restrict__ ostats) {
  ChanTile t = chan_tile<V>(g.C);
  const int b = blockIdx.x / g.NCH, ch = blockIdx.x % g.NCH;
  long r0 = (long)b * g.HW + ch * g.rows_per;
  long r1 = min((long)b * g.HW + g.HW, r0 + g.rows_per);
  double o1[V], o2[V];
#pragma unroll
  for (int j = 0; j < V; ++j) { o1[j] = 0.0; o2[j] = 0.0; }
  if (t.active) {
    float s[V], h[V], al[V], be[V];
#pragma unroll
    for (int j = 0; j < V; ++j) {
      s[j] = sc ? sc[t.c0 + j] : 1.f;
      h[j] = sh ? sh[t.c0 + j] : 0.f;
      al[j] = alpha[b * g.C + t.c0 + j];
      be[j] = betap[t.c0 + j];
    }
    const bool pro = sc != nullptr;
    for (long r = r0 + t.rg; r < r1; r += t.RG) {
      float v[V];
      ldv<V>(z + r * g.C + t.c0, v);
#pragma unroll
      for (int j = 0; j < V; ++j) {
        float x = pro ? apply_act(v[j] * s[j] + h[j], act) : v[j];
        v[j] = rnd<T>(lrelu(al[j] * x + be[j]));  // statistics of the stored value
        o1[j] += v[j];
        o2[j] += (double)v[j] * v[j];
      }
      stv<V>(out + r * g.C + t.c0, v);
    }
  }
  // optional statistics of the SE output (MLFC feeds it straight into bns_l, :427-487)
  if (ostats) block_chan_reduce2<V>(t, o1, o2, ostats, blockIdx.x, g.C);
}

// backward pass 1: partials of (T1 = sum g2, T2 = sum g2*a) per (b,c)
template <int V, typename T>
__global__ void __launch_bounds__(256)
se_bwd_reduce_kernel(const T* __restrict__ z, const T* __restrict__ dout,
                     const float* __restrict__ sc, const float* __restrict__ sh, int act,
                     SeGeom g, const float* __restrict__ alpha, const float* __restrict__ betap,
                     double* __restrict__ part) {
  ChanTile t = chan_tile<V>(g.C);
  const int b = blockIdx.x / g.NCH, ch = blockIdx.x % g.NCH;
  long r0 = (long)b * g.HW + ch * g.rows_per;
  long r1 = min((long)b * g.HW + g.HW, r0 + g.rows_per);
  double t1[V], t2[V];
#pragma unroll
  for (int j = 0; j < V; ++j) { t1[j] = 0.0; t2[j] = 0.0; }
  if (t.active) {
    float s[V], h[V], al[V], be[V];
#pragma unroll
    for (int j = 0; j < V; ++j) {
      s[j] = sc ? sc[t.c0 + j] : 1.f;
      h[j] = sh ? sh[t.c0 + j] : 0.f;
      al[j] = alpha[b * g.C + t.c0 + j];
      be[j] = betap[t.c0 + j];
    }
    const bool pro = sc != nullptr;
    for (long r = r0 + t.rg; r < r1; r += t.RG) {
      float v[V], d[V];
      ldv<V>(z + r * g.C + t.c0, v);
      ldv<V>(dout + r * g.C + t.c0, d);
#pragma unroll
      for (int j = 0; j < V; ++j) {
        float x = pro ? apply_act(v[j] * s[j] + h[j], act) : v[j];
        float g2 = d[j] * lrelu_d(al[j] * x + be[j]);
        t1[j] += g2;
        t2[j] += (double)g2 * x;
      }
    }
  }
  block_chan_reduce2<V>(t, t1, t2, part, blockIdx.x, g.C);
}

// backward mid (three small launches). coef (fp32): A[B*C] Bc[B*C] Cc[B*C] with
//   da = A*g2 + Bc*(a*s - mean) + Cc
// scratch (fp64): G[C] GY[C] du[B*C] dh[B*Cr] T1[B*C] T2[B*C]
// part 1: one thread per channel — BN backward sums and du = ds * s * (1 - s)
// SE_LANES lanes per channel: lane l handles samples b = l, l + SE_LANES, ...; the
// per-channel sums are reduced with an xor butterfly inside the lane group and lane 0's
// value is broadcast, so every lane uses identical totals (deterministic).
#define SE_LANES 16
ACC_DEV double se_lane_sum(double v) {
#pragma unroll
  for (int off = 1; off < SE_LANES; off <<= 1) v += __shfl_xor(v, off);
  return __shfl(v, (threadIdx.x & 63) & ~(SE_LANES - 1));
}

__global__ void __launch_bounds__(256)
se_bwd_chan_kernel(SeGeom g, int Cr,
                   const float* __restrict__ gamma, int training, float* __restrict__ save,
                   float* __restrict__ dgamma, float* __restrict__ dbeta,
                   double* __restrict__ scratch) {
  const int B = g.B, C = g.C;
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  const int c = gid / SE_LANES, lane = gid % SE_LANES;
  const bool live = c < C;  // dead lanes still join the shuffles
  const int cc = live ? c : 0;
  SeSave sv = se_save_view(save, B, C, Cr);
  double* G = scratch;
  double* GY = G + C;
  double* du = GY + C;
  const double* T1 = du + (size_t)B * C + (size_t)B * Cr;
  const double* T2 = T1 + (size_t)B * C;
  const double n = (double)B * g.HW;
  const double mean = sv.mean[cc], rstd = sv.rstd[cc];
  double gs = 0.0, gy = 0.0;
  // per-(b,c) T1 = sum g2, T2 = sum g2*a (se_part_sum_kernel)
  if (live)
    for (int b = lane; b < B; b += SE_LANES) {
      double t1 = T1[b * C + c];
      gs += t1;
      gy += (double)sv.sg[b * C + c] * T2[b * C + c] - mean * t1;
    }
  gs = se_lane_sum(gs);
  gy = se_lane_sum(gy) * rstd;
  if (!live) return;
  if (lane == 0) {
    G[c] = gs;
    GY[c] = gy;
    if (dgamma) dgamma[c] = (float)gy;
    if (dbeta) dbeta[c] = (float)gs;
  }
  const double k = (double)gamma[c] * rstd;
  for (int b = lane; b < B; b += SE_LANES) {
    double s = sv.sg[b * C + c];
    double t2 = T2[b * C + c];
    double ds;
    if (training) {
      double yha = rstd * (s * sv.Q[b * C + c] - mean * sv.S[b * C + c]);
      ds = k * (t2 - (gs / n) * sv.S[b * C + c] - (gy / n) * yha);
    } else {
      ds = k * t2;
    }
    du[b * C + c] = ds * s * (1.0 - s);
  }
}

// part 2: one block per sample — dh = lrelu'(hpre) * W2^T du, dm = W1^T dh, coefficients
__global__ void __launch_bounds__(256)
se_bwd_sample_kernel(SeGeom g, int Cr, const float* __restrict__ w1,
                     const float* __restrict__ w2, const float* __restrict__ gamma, int training,
                     float* __restrict__ save, double* __restrict__ scratch,
                     float* __restrict__ coef) {
  extern __shared__ __attribute__((aligned(16))) double smd[];  // dh[Cr]
  const int B = g.B, C = g.C, b = blockIdx.x, tid = threadIdx.x;
  SeSave sv = se_save_view(save, B, C, Cr);
  double* G = scratch;
  double* GY = G + C;
  double* du = GY + C;
  double* dh = du + (size_t)B * C;
  for (int o = tid; o < Cr * 4; o += 256) {
    int j = o >> 2, part_i = o & 3;
    double acc = 0.0;
    #pragma unroll 8
    for (int c = part_i; c < C; c += 4) acc += (double)w2[(long)c * Cr + j] * du[b * C + c];
    acc += __shfl_xor(acc, 1);
    acc += __shfl_xor(acc, 2);
    if (part_i == 0) {
      double v = acc * lrelu_d(sv.hpre[b * Cr + j]);
      smd[j] = v;
      dh[b * Cr + j] = v;
    }
  }
  __syncthreads();
  const double n = (double)B * g.HW;
  float* A = coef;
  float* Bc = A + (size_t)B * C;
  float* Cc = Bc + (size_t)B * C;
  for (int c = tid; c < C; c += 256) {
    double dm = 0.0;
    #pragma unroll 8
    for (int j = 0; j < Cr; ++j) dm += (double)w1[(long)j * C + c] * smd[j];
    double k = (double)gamma[c] * sv.rstd[c];
    double s = sv.sg[b * C + c];
    int i = b * C + c;
    A[i] = (float)(s * k);
    if (training) {
      Bc[i] = (float)(-s * k * sv.rstd[c] * (GY[c] / n));
      Cc[i] = (float)(-s * k * (G[c] / n) + dm / g.HW);
    } else {
      Bc[i] = 0.f;
      Cc[i] = (float)(dm / g.HW);
    }
  }
}

// part 3: parameter gradients of fc1 / fc2 (sums over the batch)
__global__ void __launch_bounds__(256)
se_bwd_param_kernel(SeGeom g, int Cr, float* __restrict__ save, const double* __restrict__ scratch,
                    float* __restrict__ dw1, float* __restrict__ db1, float* __restrict__ dw2,
                    float* __restrict__ db2) {
  const int B = g.B, C = g.C;
  SeSave sv = se_save_view(save, B, C, Cr);
  const double* du = scratch + 2 * (size_t)C;
  const double* dh = du + (size_t)B * C;
  const long nW = (long)C * Cr;
  const long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (i < nW) {  // dw2[c][j] = sum_b du[b,c] * lrelu(hpre[b,j])
    int c = (int)(i / Cr), j = (int)(i % Cr);
    double acc = 0.0;
    #pragma unroll 8
    for (int b = 0; b < B; ++b) acc += du[b * C + c] * lrelu(sv.hpre[b * Cr + j]);
    dw2[i] = (float)acc;
  } else if (i < 2 * nW) {  // dw1[j][c] = sum_b dh[b,j] * m[b,c]
    long t = i - nW;
    int j = (int)(t / C), c = (int)(t % C);
    double acc = 0.0;
    #pragma unroll 8
    for (int b = 0; b < B; ++b) acc += dh[b * Cr + j] * (sv.S[b * C + c] / g.HW);
    dw1[t] = (float)acc;
  } else if (i < 2 * nW + C) {
    int c = (int)(i - 2 * nW);
    double acc = 0.0;
    #pragma unroll 8
    for (int b = 0; b < B; ++b) acc += du[b * C + c];
    db2[c] = (float)acc;
  } else if (i < 2 * nW + C + Cr) {
    int j = (int)(i - 2 * nW - C);
    double acc = 0.0;
    #pragma unroll 8
    for (int b = 0; b < B; ++b) acc += dh[b * Cr + j];
    db1[j] = (float)acc;
  }
}

template <int V, typename T>
__global__ void __launch_bounds__(256)
se_bwd_apply_kernel(const T* __restrict__ z, const T* __restrict__ dout,
                    const float* __restrict__ sc, const float* __restrict__ sh, int act, SeGeom g,
                    const float* __restrict__ alpha, const float* __restrict__ betap,
                    const float* __restrict__ sgate, const float* __restrict__ mean,
                    const float* __restrict__ coef, T* __restrict__ da) {
  ChanTile t = chan_tile<V>(g.C);
  if (!t.active) return;
  const int b = blockIdx.x / g.NCH, ch = blockIdx.x % g.NCH;
  long r0 = (long)b * g.HW + ch * g.rows_per;
  long r1 = min((long)b * g.HW + g.HW, r0 + g.rows_per);
  const int BC = g.B * g.C;
  float s[V], h[V], al[V], be[V], A[V], Bc[V], Cc[V], sgv[V], mu[V];
#pragma unroll
  for (int j = 0; j < V; ++j) {
    int i = b * g.C + t.c0 + j;
    sgv[j] = sgate[i];
    mu[j] = mean[t.c0 + j];
    s[j] = sc ? sc[t.c0 + j] : 1.f;
    h[j] = sh ? sh[t.c0 + j] : 0.f;
    al[j] = alpha[i];
    be[j] = betap[t.c0 + j];
    A[j] = coef[i];
    Bc[j] = coef[BC + i];
    Cc[j] = coef[2 * BC + i];
  }
  const bool pro = sc != nullptr;
  for (long r = r0 + t.rg; r < r1; r += t.RG) {
    float v[V], d[V];
    ldv<V>(z + r * g.C + t.c0, v);
    ldv<V>(dout + r * g.C + t.c0, d);
#pragma unroll
    for (int j = 0; j < V; ++j) {
      float x = pro ? apply_act(v[j] * s[j] + h[j], act) : v[j];
      float g2 = d[j] * lrelu_d(al[j] * x + be[j]);
      d[j] = A[j] * g2 + Bc[j] * (x * sgv[j] - mu[j]) + Cc[j];
    }
    stv<V>(da + r * g.C + t.c0, d);
  }
}

// ---------------------------------------------------------------------------
// SE backward fused with the backward of the BatchNorm(+act) prologue that feeds it
// (the preceding layer's BN: HANCBlock.norm3 :281-283, ResPath.bns[i] :326,
// Conv2d_batchnorm.batchnorm :183-185, MLFC.bns_mrg :520).
//
// With pre = z*sc1 + sh1, a = act(pre), l' = act'(pre), xc = z - mean1, the SE
// backward gives da = A*g2 + Bc*(a*s - mean) + Cc (per-(b,c) A, Bc, Cc); the
// prologue BN backward needs g = da*l' reduced per channel:
//   sum_p g      = A*U1 + Bc*s*U2 + (Cc - Bc*mean)*U3
//   sum_p g*xc   = A*W1 + Bc*s*W2 + (Cc - Bc*mean)*W3
// with U1 = sum l'g2, U2 = sum l'a, U3 = sum l', W1 = sum l'g2*xc, W2 = sum l'a*xc,
// W3 = sum l'*xc: per-(b,c) sums the SE's own first backward pass can collect. So
// the pair costs 2 read passes of (z, dout) + 1 write of dz, instead of 4 read
// passes + 2 writes (da is never materialised).
// ---------------------------------------------------------------------------
#define SE_PRO_NQ 8  // T1, T2, U1, U2, U3, W1, W2, W3

template <int V, typename T>
__global__ void __launch_bounds__(256)
se_bwd_reduce_pro_kernel(const T* __restrict__ z, const T* __restrict__ dout,
                         const float* __restrict__ pst, int act, SeGeom g,
                         const float* __restrict__ alpha, const float* __restrict__ betap,
                         double* __restrict__ part) {
  ChanTile t = chan_tile<V>(g.C);
  const int C = g.C;
  const int b = blockIdx.x / g.NCH, ch = blockIdx.x % g.NCH;
  long r0 = (long)b * g.HW + ch * g.rows_per;
  long r1 = min((long)b * g.HW + g.HW, r0 + g.rows_per);
  double acc[SE_PRO_NQ][V];
#pragma unroll
  for (int i = 0; i < SE_PRO_NQ; ++i)
#pragma unroll
    for (int j = 0; j < V; ++j) acc[i][j] = 0.0;
  if (t.active) {
    float s[V], h[V], mu[V], al[V], be[V];
#pragma unroll
    for (int j = 0; j < V; ++j) {
      mu[j] = pst[BN_MEAN * C + t.c0 + j];
      s[j] = pst[BN_SCALE * C + t.c0 + j];
      h[j] = pst[BN_SHIFT * C + t.c0 + j];
      al[j] = alpha[b * C + t.c0 + j];
      be[j] = betap[t.c0 + j];
    }
    for (long r = r0 + t.rg; r < r1; r += t.RG) {
      float v[V], d[V];
      ldv<V>(z + r * C + t.c0, v);
      ldv<V>(dout + r * C + t.c0, d);
#pragma unroll
      for (int j = 0; j < V; ++j) {
        const float pre = v[j] * s[j] + h[j];
        const float x = apply_act(pre, act);
        const float lp = act == ACT_LRELU ? lrelu_d(pre) : 1.f;
        const float g2 = d[j] * lrelu_d(al[j] * x + be[j]);
        const double xc = (double)v[j] - mu[j];
        const double lg = (double)lp * g2, la = (double)lp * x;
        acc[0][j] += g2;
        acc[1][j] += (double)g2 * x;
        acc[2][j] += lg;
        acc[3][j] += la;
        acc[4][j] += lp;
        acc[5][j] += lg * xc;
        acc[6][j] += la * xc;
        acc[7][j] += lp * xc;
      }
    }
  }
  block_chan_reduceN<V, SE_PRO_NQ>(t, acc, part, blockIdx.x, C);
}

// one thread per channel: the prologue BN's backward coefficients
//   dz = k1*g + k2*(z - mean1) + k3, dgamma1 = sum g*xhat, dbeta1 = sum g
// from the per-(b,c) sums (UW[i][B*C], i = 0..5 -> U1 U2 U3 W1 W2 W3) and the SE
// coefficients A, Bc, Cc.
__global__ void __launch_bounds__(256)
se_pro_coef_kernel(SeGeom g, int Cr, const float* __restrict__ save,
                   const double* __restrict__ UW, const float* __restrict__ coef,
                   const float* __restrict__ pst, const float* __restrict__ pgamma,
                   int ptraining, float* __restrict__ dpg, float* __restrict__ dpb,
                   float* __restrict__ pcoef) {
  const int B = g.B, C = g.C;
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  const int c = gid / SE_LANES, lane = gid % SE_LANES;  // SE_LANES lanes per channel
  const bool live = c < C;
  SeSave sv = se_save_view(const_cast<float*>(save), B, C, Cr);
  const long BC = (long)B * C;
  const float* A = coef;
  const float* Bc = A + BC;
  const float* Cc = Bc + BC;
  double sg = 0.0, sgx = 0.0;
  if (live) {
    const double mean = sv.mean[c];
    for (int b = lane; b < B; b += SE_LANES) {
      const long i = (long)b * C + c;
      const double a = A[i], bb = Bc[i], s = sv.sg[i];
      const double cst = (double)Cc[i] - bb * mean;
      sg += a * UW[0 * BC + i] + bb * s * UW[1 * BC + i] + cst * UW[2 * BC + i];
      sgx += a * UW[3 * BC + i] + bb * s * UW[4 * BC + i] + cst * UW[5 * BC + i];
    }
  }
  sg = se_lane_sum(sg);
  sgx = se_lane_sum(sgx);
  if (!live || lane != 0) return;
  const float rstd1 = pst[BN_RSTD * C + c];
  sgx *= rstd1;  // sum g*xhat
  if (dpg) dpg[c] = (float)sgx;
  if (dpb) dpb[c] = (float)sg;
  const double n = (double)B * g.HW;
  const float ga = pgamma ? pgamma[c] : 1.f;
  const float k1 = ga * rstd1;
  float k2 = 0.f, k3 = 0.f;
  if (ptraining) {  // same coefficients as bn_bwd_finalize_kernel (csrc/bn.hip)
    const float mg = (float)(sg / n), mgx = (float)(sgx / n);
    k2 = -k1 * rstd1 * mgx;
    k3 = -k1 * mg;
  }
  pcoef[c] = k1;
  pcoef[C + c] = k2;
  pcoef[2 * C + c] = k3;
}

template <int V, typename T>
__global__ void __launch_bounds__(256)
se_bwd_apply_pro_kernel(const T* __restrict__ z, const T* __restrict__ dout,
                        const float* __restrict__ pst, int act, SeGeom g,
                        const float* __restrict__ alpha, const float* __restrict__ betap,
                        const float* __restrict__ sgate, const float* __restrict__ mean,
                        const float* __restrict__ coef, const float* __restrict__ pcoef,
                        T* __restrict__ dz, double* __restrict__ colsum) {
  ChanTile t = chan_tile<V>(g.C);
  // optional fp64 column sums of dz (the bias gradient of z's producer convolution)
  double cs[V], cz[V];
#pragma unroll
  for (int j = 0; j < V; ++j) { cs[j] = 0.0; cz[j] = 0.0; }
  if (!t.active) {
    if (colsum) block_chan_reduce2<V>(t, cs, cz, colsum, blockIdx.x, g.C);
    return;
  }
  const int C = g.C;
  const int b = blockIdx.x / g.NCH, ch = blockIdx.x % g.NCH;
  long r0 = (long)b * g.HW + ch * g.rows_per;
  long r1 = min((long)b * g.HW + g.HW, r0 + g.rows_per);
  const int BC = g.B * C;
  float s[V], h[V], mu1[V], al[V], be[V], A[V], Bc[V], Cc[V], sgv[V], mu[V], k1[V], k2[V],
      k3[V];
#pragma unroll
  for (int j = 0; j < V; ++j) {
    const int c = t.c0 + j, i = b * C + c;
    sgv[j] = sgate[i];
    mu[j] = mean[c];
    mu1[j] = pst[BN_MEAN * C + c];
    s[j] = pst[BN_SCALE * C + c];
    h[j] = pst[BN_SHIFT * C + c];
    al[j] = alpha[i];
    be[j] = betap[c];
    A[j] = coef[i];
    Bc[j] = coef[BC + i];
    Cc[j] = coef[2 * BC + i];
    k1[j] = pcoef[c];
    k2[j] = pcoef[C + c];
    k3[j] = pcoef[2 * C + c];
  }
  constexpr int U = 2;  // rows per iteration with all loads issued first
  for (long rb = r0 + t.rg; rb < r1; rb += U * t.RG) {
    float v[U][V], d[U][V];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long r = rb + (long)u * t.RG;
      if (r < r1) {
        ldv<V>(z + r * C + t.c0, v[u]);
        ldv<V>(dout + r * C + t.c0, d[u]);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long r = rb + (long)u * t.RG;
      if (r < r1) {
#pragma unroll
        for (int j = 0; j < V; ++j) {
          const float pre = v[u][j] * s[j] + h[j];
          const float x = apply_act(pre, act);
          const float g2 = d[u][j] * lrelu_d(al[j] * x + be[j]);
          float da = A[j] * g2 + Bc[j] * (x * sgv[j] - mu[j]) + Cc[j];
          if (act == ACT_LRELU) da *= lrelu_d(pre);
          d[u][j] = rnd<T>(k1[j] * da + k2[j] * (v[u][j] - mu1[j]) + k3[j]);
          if (colsum) cs[j] += d[u][j];
        }
        stv<V>(dz + r * C + t.c0, d[u]);
      }
    }
  }
  if (colsum) block_chan_reduce2<V>(t, cs, cz, colsum, blockIdx.x, g.C);
}

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------
extern "C" size_t accunet_se_save_elems(int B, int C, int Cr) { return se_save_floats(B, C, Cr); }

// rows of the optional SE-output statistics block written by accunet_se_fwd
extern "C" int accunet_se_stats_rows(int B, int HW, int C) {
  SeGeom g = se_geom(B, HW, C);
  return B * g.NCH;
}

// workspace (floats): fp64 partials [B*NCH][SE_PRO_NQ][C] | fp64 scratch | fp32 coef [3][B*C]
// | fp32 prologue coefficients [3][C]
static size_t se_part_floats(const SeGeom& g) {
  return (size_t)g.B * g.NCH * SE_PRO_NQ * g.C * 2;
}
// fp64 scratch: G[C] GY[C] du[B*C] dh[B*Cr] T1 T2 U1 U2 U3 W1 W2 W3 [B*C each]
static size_t se_scratch_floats(int B, int C, int Cr) {
  return ((size_t)B * C * (1 + SE_PRO_NQ) + 2 * (size_t)C + (size_t)B * Cr) * 2;
}

// + fp64 reduce scratch for the optional dz column sums (accunet_se_bwd_pro dsum)
static size_t se_dsum_scr_floats(const SeGeom& g) {
  return accunet_partials_ws_elems(g.B * g.NCH, 2 * g.C) * 2;
}

extern "C" size_t accunet_se_ws_elems(int B, int HW, int C, int Cr) {
  SeGeom g = se_geom(B, HW, C);
  return se_part_floats(g) + se_scratch_floats(B, C, Cr) + (size_t)B * C * 3 + 3 * (size_t)C + 4 +
         se_dsum_scr_floats(g);
}

extern "C" int accunet_se_fwd(const void* z, const float* sc, const float* sh, int act, int B,
                              int HW, int C, int Cr, const float* w1, const float* b1,
                              const float* w2, const float* b2, const float* gamma,
                              const float* beta, float* rmean, float* rvar, long long* nbt,
                              float momentum, float eps, int training, void* out, float* save,
                              double* ostats, float* ws, size_t ws_elems, int dt, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (dt != ACC_F32 && dt != ACC_BF16) return ACC_EBADARG;
  if (ws_elems < accunet_se_ws_elems(B, HW, C, Cr)) return ACC_EBADARG;
  if (((uintptr_t)ws & 7) || ((uintptr_t)save & 7)) return ACC_EBADARG;
  SeGeom g = se_geom(B, HW, C);
  int V = (C % 4 == 0) ? 4 : 1;
  dim3 grid(B * g.NCH, ceil_div(C / V, 64));
  double* part = reinterpret_cast<double*>(ws);
  with_dt(dt, [&](auto tag) {
    using T = decltype(tag);
    if (V == 4)
      hipLaunchKernelGGL((se_reduce_kernel<4, T>), grid, dim3(256), 0, s, (const T*)z, sc, sh, act,
                         g, part);
    else
      hipLaunchKernelGGL((se_reduce_kernel<1, T>), grid, dim3(256), 0, s, (const T*)z, sc, sh, act,
                         g, part);
  });
  // S, Q and the gate per sample, then the BN-of-gated statistics per channel
  hipLaunchKernelGGL(se_mid_sample_kernel, dim3(B), dim3(256), (C + Cr) * sizeof(float), s, part,
                     g, Cr, w1, b1, w2, b2, save);
  hipLaunchKernelGGL(se_mid_bn_kernel, dim3(ceil_div(C, 256)), dim3(256), 0, s, g, Cr, gamma, beta,
                     rmean, rvar, momentum, eps, training, save, training ? nbt : nullptr);
  const float* alpha = save + se_alpha_offset(B, C, Cr);
  const float* betap = alpha + (size_t)B * C;
  with_dt(dt, [&](auto tag) {
    using T = decltype(tag);
    if (V == 4)
      hipLaunchKernelGGL((se_apply_kernel<4, T>), grid, dim3(256), 0, s, (const T*)z, sc, sh, act, g,
                         alpha, betap, (T*)out, ostats);
    else
      hipLaunchKernelGGL((se_apply_kernel<1, T>), grid, dim3(256), 0, s, (const T*)z, sc, sh, act, g,
                         alpha, betap, (T*)out, ostats);
  });
  return hipGetLastError() == hipSuccess ? ACC_OK : ACC_ELAUNCH;
}

// shared by accunet_se_bwd / accunet_se_bwd_pro: the per-(b,c) sums in scratch (from
// part) -> BN / gate / fc backward, coef (A, Bc, Cc), fc parameter gradients
static void se_bwd_mid(const SeGeom& g, int Cr, const double* part, int nq, const float* w1,
                       const float* w2, const float* gamma, int training, float* sv,
                       double* scratch, float* coef, float* dw1, float* db1, float* dw2,
                       float* db2, float* dgamma, float* dbeta, hipStream_t s) {
  const int B = g.B, C = g.C;
  double* T1 = scratch + 2 * (size_t)C + (size_t)B * C + (size_t)B * Cr;
  if (nq == 2)
    hipLaunchKernelGGL(se_part_sum_kernel<2>, dim3(ceil_div(C, 64), B), dim3(256), 0, s, part, g,
                       T1);
  else
    hipLaunchKernelGGL(se_part_sum_kernel<SE_PRO_NQ>, dim3(ceil_div(C, 64), B), dim3(256), 0, s,
                       part, g, T1);
  hipLaunchKernelGGL(se_bwd_chan_kernel, dim3(ceil_div((long)C * SE_LANES, 256)), dim3(256), 0, s,
                     g, Cr, gamma,
                     training, sv, dgamma, dbeta, scratch);
  hipLaunchKernelGGL(se_bwd_sample_kernel, dim3(B), dim3(256), (Cr > 0 ? Cr : 1) * sizeof(double),
                     s, g, Cr, w1, w2, gamma, training, sv, scratch, coef);
  long nparam = 2L * C * Cr + C + Cr;
  hipLaunchKernelGGL(se_bwd_param_kernel, dim3(ceil_div(nparam, 256)), dim3(256), 0, s, g, Cr, sv,
                     scratch, dw1, db1, dw2, db2);
}

extern "C" int accunet_se_bwd(const void* z, const void* dout, const float* sc, const float* sh,
                              int act, int B, int HW, int C, int Cr, const float* w1,
                              const float* w2, const float* gamma, int training,
                              const float* save, void* da, float* dw1, float* db1, float* dw2,
                              float* db2, float* dgamma, float* dbeta, float* ws, size_t ws_elems,
                              int dt, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (dt != ACC_F32 && dt != ACC_BF16) return ACC_EBADARG;
  if (ws_elems < accunet_se_ws_elems(B, HW, C, Cr)) return ACC_EBADARG;
  if (((uintptr_t)ws & 7) || ((uintptr_t)save & 7)) return ACC_EBADARG;
  SeGeom g = se_geom(B, HW, C);
  int V = (C % 4 == 0) ? 4 : 1;
  dim3 grid(B * g.NCH, ceil_div(C / V, 64));
  double* part = reinterpret_cast<double*>(ws);
  double* scratch = reinterpret_cast<double*>(ws + se_part_floats(g));
  float* coef = ws + se_part_floats(g) + se_scratch_floats(B, C, Cr);
  const float* alpha = save + se_alpha_offset(B, C, Cr);
  const float* betap = alpha + (size_t)B * C;
  const float* sgate = save + (size_t)B * C * 4 + (size_t)B * Cr;
  const float* mean = sgate + (size_t)B * C;
  with_dt(dt, [&](auto tag) {
    using T = decltype(tag);
    if (V == 4)
      hipLaunchKernelGGL((se_bwd_reduce_kernel<4, T>), grid, dim3(256), 0, s, (const T*)z,
                         (const T*)dout, sc, sh, act, g, alpha, betap, part);
    else
      hipLaunchKernelGGL((se_bwd_reduce_kernel<1, T>), grid, dim3(256), 0, s, (const T*)z,
                         (const T*)dout, sc, sh, act, g, alpha, betap, part);
  });
  float* sv = const_cast<float*>(save);
  se_bwd_mid(g, Cr, part, 2, w1, w2, gamma, training, sv, scratch, coef, dw1, db1, dw2, db2,
             dgamma, dbeta, s);
  with_dt(dt, [&](auto tag) {
    using T = decltype(tag);
    if (V == 4)
      hipLaunchKernelGGL((se_bwd_apply_kernel<4, T>), grid, dim3(256), 0, s, (const T*)z,
                         (const T*)dout, sc, sh, act, g, alpha, betap, sgate, mean, coef, (T*)da);
    else
      hipLaunchKernelGGL((se_bwd_apply_kernel<1, T>), grid, dim3(256), 0, s, (const T*)z,
                         (const T*)dout, sc, sh, act, g, alpha, betap, sgate, mean, coef, (T*)da);
  });
  return hipGetLastError() == hipSuccess ? ACC_OK : ACC_ELAUNCH;
}

extern "C" int accunet_se_bwd_pro(const void* z, const void* dout, const float* pst, int act,
                                  const float* pgamma, int ptraining, int B, int HW, int C,
                                  int Cr, const float* w1, const float* w2, const float* gamma,
                                  int training, const float* save, void* dz, float* dpgamma,
                                  float* dpbeta, float* dsum, float* dw1, float* db1, float* dw2,
                                  float* db2,
                                  float* dgamma, float* dbeta, float* ws, size_t ws_elems, int dt,
                                  void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (dt != ACC_F32 && dt != ACC_BF16) return ACC_EBADARG;
  if (ws_elems < accunet_se_ws_elems(B, HW, C, Cr)) return ACC_EBADARG;
  if (((uintptr_t)ws & 7) || ((uintptr_t)save & 7)) return ACC_EBADARG;
  if (!pst || !dz) return ACC_EBADARG;
  SeGeom g = se_geom(B, HW, C);
  int V = (C % 4 == 0) ? 4 : 1;
  dim3 grid(B * g.NCH, ceil_div(C / V, 64));
  double* part = reinterpret_cast<double*>(ws);
  double* scratch = reinterpret_cast<double*>(ws + se_part_floats(g));
  float* coef = ws + se_part_floats(g) + se_scratch_floats(B, C, Cr);
  float* pcoef = coef + (size_t)B * C * 3;
  // dsum scratch after pcoef (3C floats + 4 pad), 8-byte aligned
  double* dscr = reinterpret_cast<double*>(pcoef + ((3 * (size_t)C + 4 + 1) / 2) * 2);
  const float* alpha = save + se_alpha_offset(B, C, Cr);
  const float* betap = alpha + (size_t)B * C;
  const float* sgate = save + (size_t)B * C * 4 + (size_t)B * Cr;
  const float* mean = sgate + (size_t)B * C;
  with_dt(dt, [&](auto tag) {
    using T = decltype(tag);
    if (V == 4)
      hipLaunchKernelGGL((se_bwd_reduce_pro_kernel<4, T>), grid, dim3(256), 0, s, (const T*)z,
                         (const T*)dout, pst, act, g, alpha, betap, part);
    else
      hipLaunchKernelGGL((se_bwd_reduce_pro_kernel<1, T>), grid, dim3(256), 0, s, (const T*)z,
                         (const T*)dout, pst, act, g, alpha, betap, part);
  });
  float* sv = const_cast<float*>(save);
  se_bwd_mid(g, Cr, part, SE_PRO_NQ, w1, w2, gamma, training, sv, scratch, coef, dw1, db1, dw2,
             db2, dgamma, dbeta, s);
  const double* UW = scratch + 2 * (size_t)C + (size_t)B * C + (size_t)B * Cr + 2 * (size_t)B * C;
  hipLaunchKernelGGL(se_pro_coef_kernel, dim3(ceil_div((long)C * SE_LANES, 256)), dim3(256), 0, s,
                     g, Cr, save, UW,
                     coef, pst, pgamma, ptraining, dpgamma, dpbeta, pcoef);
  // the reduce-pass partials are consumed by the mid kernels: reuse them for dz's column sums
  double* cpart = dsum ? part : nullptr;
  with_dt(dt, [&](auto tag) {
    using T = decltype(tag);
    if (V == 4)
      hipLaunchKernelGGL((se_bwd_apply_pro_kernel<4, T>), grid, dim3(256), 0, s, (const T*)z,
                         (const T*)dout, pst, act, g, alpha, betap, sgate, mean, coef, pcoef, (T*)dz,
                         cpart);
    else
      hipLaunchKernelGGL((se_bwd_apply_pro_kernel<1, T>), grid, dim3(256), 0, s, (const T*)z,
                         (const T*)dout, pst, act, g, alpha, betap, sgate, mean, coef, pcoef, (T*)dz,
                         cpart);
  });
  if (dsum) {
    FinishArgs fa{};
    fa.kind = FIN_SUM_F;
    fa.ncols = C;
    fa.out_f = dsum;
    return reduce_finish(cpart, true, B * g.NCH, 2 * C, dscr, fa, s);
  }
  return hipGetLastError() == hipSuccess ? ACC_OK : ACC_ELAUNCH;
}
