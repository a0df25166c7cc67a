// Squeeze-and-excitation gate fused with the BatchNorm(+LeakyReLU) that precedes it
// and the BatchNorm + LeakyReLU inside it: ChannelSELayer.forward,
// reference ACC_UNet/ACC_UNet.py:37-49 (r = 8, LeakyReLU after fc1, BN + LeakyReLU
// after the gating), always fed by lrelu(bn(conv(...))) in HANCBlock (:281-284),
// ResPath (:326), Conv2d_batchnorm (:183-186) and MLFC (:522-525).
//
// Forward (K3 "SE gate"), z = pending input, a = act(z*sc1+sh1) (or a = z):
//   pass 1 (se_reduce): per-(b,c) S = sum_hw a, Q = sum_hw a^2      [reads z once]
//   mid   (se_mid):    m = S/HW, s = sigmoid(fc2(lrelu(fc1(m)))),
//                      BN stats of y = a*s derived exactly from (S, Q, s):
//                        mean = sum_b s*S / n,  E[y^2] = sum_b s^2*Q / n
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
template <int V>
__global__ void __launch_bounds__(256)
se_reduce_kernel(const float* __restrict__ z, const float* __restrict__ sc,
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

// chunk partials -> per-(b,c) sums: block = 64 channels x 4 chunk groups of one
// sample; each group sums its chunks in order, the 4 group sums are added in order.
__global__ void __launch_bounds__(256)
se_part_sum_kernel(const double* __restrict__ part, SeGeom g, double* __restrict__ o1,
                   double* __restrict__ o2) {
  __shared__ double r1[4][64], r2[4][64];
  const int C = g.C, b = blockIdx.y, t = threadIdx.x;
  const int c = blockIdx.x * 64 + (t & 63), grp = t >> 6;
  double s1 = 0.0, s2 = 0.0;
  if (c < C) {
    for (int k = grp; k < g.NCH; k += 4) {
      const double* pr = part + ((long)(b * g.NCH + k) * 2) * C;
      s1 += pr[c];
      s2 += pr[C + c];
    }
  }
  r1[grp][t & 63] = s1;
  r2[grp][t & 63] = s2;
  __syncthreads();
  if (grp == 0 && c < C) {
    o1[b * C + c] = ((r1[0][t] + r1[1][t]) + r1[2][t]) + r1[3][t];
    o2[b * C + c] = ((r2[0][t] + r2[1][t]) + r2[2][t]) + r2[3][t];
  }
}

// mid forward, part 1: one block per sample b — the channel means (from the
// per-(b,c) sums S), fc1 (+LeakyReLU) and fc2 (+sigmoid) of that sample.
__global__ void __launch_bounds__(256)
se_mid_gate_kernel(SeGeom g, int Cr,
                   const float* __restrict__ w1, const float* __restrict__ b1,
                   const float* __restrict__ w2, const float* __restrict__ b2,
                   float* __restrict__ save) {
  extern __shared__ __attribute__((aligned(16))) float sm[];  // m[C] | h'[Cr]
  const int B = g.B, C = g.C, b = blockIdx.x, tid = threadIdx.x;
  SeSave sv = se_save_view(save, B, C, Cr);
  float* m = sm;
  float* hp = sm + C;
  for (int c = tid; c < C; c += 256) m[c] = (float)(sv.S[b * C + c] / g.HW);
  __syncthreads();
  // fc1: 4 threads per output, interleaved over the input channels
  for (int o = tid; o < Cr * 4; o += 256) {
    int j = o >> 2, part_i = o & 3;
    float acc = 0.f;
    const float* wr = w1 + (long)j * C;
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
                 float* __restrict__ save) {
  const int B = g.B, C = g.C;
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  SeSave sv = se_save_view(save, B, C, Cr);
  const double n = (double)B * g.HW;
  float mu, var;
  if (training) {
    double m1 = 0.0, m2 = 0.0;
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
  for (int b = 0; b < B; ++b) sv.alpha[b * C + c] = k * sv.sg[b * C + c];
}

// pass 2 forward: out = lrelu(alpha[b,c]*a + betap[c])
template <int V>
__global__ void __launch_bounds__(256)
se_apply_kernel(const float* __restrict__ z, const float* __restrict__ sc,
                const float* __restrict__ sh, int act, SeGeom g, const float* __restrict__ alpha,
                const float* __restrict__ betap, float* __restrict__ out,
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
        v[j] = lrelu(al[j] * x + be[j]);
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
template <int V>
__global__ void __launch_bounds__(256)
se_bwd_reduce_kernel(const float* __restrict__ z, const float* __restrict__ dout,
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
__global__ void __launch_bounds__(256)
se_bwd_chan_kernel(SeGeom g, int Cr,
                   const float* __restrict__ gamma, int training, float* __restrict__ save,
                   float* __restrict__ dgamma, float* __restrict__ dbeta,
                   double* __restrict__ scratch) {
  const int B = g.B, C = g.C;
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  SeSave sv = se_save_view(save, B, C, Cr);
  double* G = scratch;
  double* GY = G + C;
  double* du = GY + C;
  const double* T1 = du + (size_t)B * C + (size_t)B * Cr;
  const double* T2 = T1 + (size_t)B * C;
  const double n = (double)B * g.HW;
  const double mean = sv.mean[c], rstd = sv.rstd[c];
  double gs = 0.0, gy = 0.0;
  // per-(b,c) T1 = sum g2, T2 = sum g2*a (se_part_sum_kernel)
  for (int b = 0; b < B; ++b) {
    double t1 = T1[b * C + c];
    gs += t1;
    gy += (double)sv.sg[b * C + c] * T2[b * C + c] - mean * t1;
  }
  gy *= rstd;
  G[c] = gs;
  GY[c] = gy;
  if (dgamma) dgamma[c] = (float)gy;
  if (dbeta) dbeta[c] = (float)gs;
  const double k = (double)gamma[c] * rstd;
  for (int b = 0; b < B; ++b) {
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
    for (int b = 0; b < B; ++b) acc += du[b * C + c] * lrelu(sv.hpre[b * Cr + j]);
    dw2[i] = (float)acc;
  } else if (i < 2 * nW) {  // dw1[j][c] = sum_b dh[b,j] * m[b,c]
    long t = i - nW;
    int j = (int)(t / C), c = (int)(t % C);
    double acc = 0.0;
    for (int b = 0; b < B; ++b) acc += dh[b * Cr + j] * (sv.S[b * C + c] / g.HW);
    dw1[t] = (float)acc;
  } else if (i < 2 * nW + C) {
    int c = (int)(i - 2 * nW);
    double acc = 0.0;
    for (int b = 0; b < B; ++b) acc += du[b * C + c];
    db2[c] = (float)acc;
  } else if (i < 2 * nW + C + Cr) {
    int j = (int)(i - 2 * nW - C);
    double acc = 0.0;
    for (int b = 0; b < B; ++b) acc += dh[b * Cr + j];
    db1[j] = (float)acc;
  }
}

template <int V>
__global__ void __launch_bounds__(256)
se_bwd_apply_kernel(const float* __restrict__ z, const float* __restrict__ dout,
                    const float* __restrict__ sc, const float* __restrict__ sh, int act, SeGeom g,
                    const float* __restrict__ alpha, const float* __restrict__ betap,
                    const float* __restrict__ sgate, const float* __restrict__ mean,
                    const float* __restrict__ coef, float* __restrict__ da) {
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
// C ABI
// ---------------------------------------------------------------------------
extern "C" size_t accunet_se_save_elems(int B, int C, int Cr) { return se_save_floats(B, C, Cr); }

// rows of the optional SE-output statistics block written by accunet_se_fwd
extern "C" int accunet_se_stats_rows(int B, int HW, int C) {
  SeGeom g = se_geom(B, HW, C);
  return B * g.NCH;
}

// workspace (floats): fp64 partials [B*NCH][2][C] | fp64 scratch | fp32 coef [3][B*C]
static size_t se_part_floats(const SeGeom& g) { return (size_t)g.B * g.NCH * 2 * g.C * 2; }
static size_t se_scratch_floats(int B, int C, int Cr) {
  return ((size_t)B * C * 3 + 2 * (size_t)C + (size_t)B * Cr) * 2;
}

extern "C" size_t accunet_se_ws_elems(int B, int HW, int C, int Cr) {
  SeGeom g = se_geom(B, HW, C);
  return se_part_floats(g) + se_scratch_floats(B, C, Cr) + (size_t)B * C * 3 + 4;
}

extern "C" int accunet_se_fwd(const float* z, const float* sc, const float* sh, int act, int B,
                              int HW, int C, int Cr, const float* w1, const float* b1,
                              const float* w2, const float* b2, const float* gamma,
                              const float* beta, float* rmean, float* rvar, long long* nbt,
                              float momentum, float eps, int training, float* out, float* save,
                              double* ostats, float* ws, size_t ws_elems, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (ws_elems < accunet_se_ws_elems(B, HW, C, Cr)) return ACC_EBADARG;
  if (((uintptr_t)ws & 7) || ((uintptr_t)save & 7)) return ACC_EBADARG;
  SeGeom g = se_geom(B, HW, C);
  int V = (C % 4 == 0) ? 4 : 1;
  dim3 grid(B * g.NCH, ceil_div(C / V, 64));
  double* part = reinterpret_cast<double*>(ws);
  if (V == 4)
    hipLaunchKernelGGL(se_reduce_kernel<4>, grid, dim3(256), 0, s, z, sc, sh, act, g, part);
  else
    hipLaunchKernelGGL(se_reduce_kernel<1>, grid, dim3(256), 0, s, z, sc, sh, act, g, part);
  {
    double* S = reinterpret_cast<double*>(save);  // SeSave: S[B*C] then Q[B*C]
    hipLaunchKernelGGL(se_part_sum_kernel, dim3(ceil_div(C, 64), B), dim3(256), 0, s, part, g, S,
                       S + (size_t)B * C);
  }
  hipLaunchKernelGGL(se_mid_gate_kernel, dim3(B), dim3(256), (C + Cr) * sizeof(float), s, g, Cr, w1,
                     b1, w2, b2, save);
  hipLaunchKernelGGL(se_mid_bn_kernel, dim3(ceil_div(C, 256)), dim3(256), 0, s, g, Cr, gamma, beta,
                     rmean, rvar, momentum, eps, training, save);
  if (training && nbt) hipLaunchKernelGGL(inc_i64_kernel, dim3(1), dim3(1), 0, s, nbt);
  const float* alpha = save + se_alpha_offset(B, C, Cr);
  const float* betap = alpha + (size_t)B * C;
  if (V == 4)
    hipLaunchKernelGGL(se_apply_kernel<4>, grid, dim3(256), 0, s, z, sc, sh, act, g, alpha, betap,
                       out, ostats);
  else
    hipLaunchKernelGGL(se_apply_kernel<1>, grid, dim3(256), 0, s, z, sc, sh, act, g, alpha, betap,
                       out, ostats);
  return hipGetLastError() == hipSuccess ? ACC_OK : ACC_ELAUNCH;
}

extern "C" int accunet_se_bwd(const float* z, const float* dout, const float* sc, const float* sh,
                              int act, int B, int HW, int C, int Cr, const float* w1,
                              const float* w2, const float* gamma, int training,
                              const float* save, float* da, float* dw1, float* db1, float* dw2,
                              float* db2, float* dgamma, float* dbeta, float* ws, size_t ws_elems,
                              void* stream) {
  hipStream_t s = (hipStream_t)stream;
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
  if (V == 4)
    hipLaunchKernelGGL(se_bwd_reduce_kernel<4>, grid, dim3(256), 0, s, z, dout, sc, sh, act, g,
                       alpha, betap, part);
  else
    hipLaunchKernelGGL(se_bwd_reduce_kernel<1>, grid, dim3(256), 0, s, z, dout, sc, sh, act, g,
                       alpha, betap, part);
  float* sv = const_cast<float*>(save);
  {
    double* T1 = scratch + 2 * (size_t)C + (size_t)B * C + (size_t)B * Cr;
    hipLaunchKernelGGL(se_part_sum_kernel, dim3(ceil_div(C, 64), B), dim3(256), 0, s, part, g, T1,
                       T1 + (size_t)B * C);
  }
  hipLaunchKernelGGL(se_bwd_chan_kernel, dim3(ceil_div(C, 256)), dim3(256), 0, s, g, Cr, gamma,
                     training, sv, dgamma, dbeta, scratch);
  hipLaunchKernelGGL(se_bwd_sample_kernel, dim3(B), dim3(256), (Cr > 0 ? Cr : 1) * sizeof(double),
                     s, g, Cr, w1, w2, gamma, training, sv, scratch, coef);
  long nparam = 2L * C * Cr + C + Cr;
  hipLaunchKernelGGL(se_bwd_param_kernel, dim3(ceil_div(nparam, 256)), dim3(256), 0, s, g, Cr, sv,
                     scratch, dw1, db1, dw2, db2);
  if (V == 4)
    hipLaunchKernelGGL(se_bwd_apply_kernel<4>, grid, dim3(256), 0, s, z, dout, sc, sh, act, g,
                       alpha, betap, sgate, mean, coef, da);
  else
    hipLaunchKernelGGL(se_bwd_apply_kernel<1>, grid, dim3(256), 0, s, z, dout, sc, sh, act, g,
                       alpha, betap, sgate, mean, coef, da);
  return hipGetLastError() == hipSuccess ? ACC_OK : ACC_ELAUNCH;
}
