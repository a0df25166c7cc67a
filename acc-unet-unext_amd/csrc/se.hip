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
                 const float* __restrict__ sh, int act, SeGeom g, float* __restrict__ part) {
  ChanTile t = chan_tile<V>(g.C);
  const int b = blockIdx.x / g.NCH, ch = blockIdx.x % g.NCH;
  long r0 = (long)b * g.HW + ch * g.rows_per;
  long r1 = min((long)b * g.HW + g.HW, r0 + g.rows_per);
  float a[V], q[V];
#pragma unroll
  for (int j = 0; j < V; ++j) { a[j] = 0.f; q[j] = 0.f; }
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
        float x = pro ? apply_act(v[j] * s[j] + h[j], act) : v[j];
        a[j] += x;
        q[j] += x * x;
      }
    }
  }
  block_chan_reduce2<V>(t, a, q, part, blockIdx.x, g.C);
}

// mid forward. One block of 256 threads. save layout (floats):
//   S[B*C] Q[B*C] hpre[B*Cr] s[B*C] mean[C] rstd[C] alpha[B*C] betap[C]
__global__ void __launch_bounds__(256)
se_mid_kernel(const float* __restrict__ part, SeGeom g, int Cr, const float* __restrict__ w1,
              const float* __restrict__ b1, const float* __restrict__ w2,
              const float* __restrict__ b2, const float* __restrict__ gamma,
              const float* __restrict__ beta, float* __restrict__ rmean, float* __restrict__ rvar,
              float momentum, float eps, int training, float* __restrict__ save) {
  const int B = g.B, C = g.C;
  float* S = save;
  float* Q = S + B * C;
  float* hpre = Q + B * C;
  float* sg = hpre + B * Cr;
  float* mean = sg + B * C;
  float* rstd = mean + C;
  float* alpha = rstd + C;
  float* betap = alpha + B * C;
  const int tid = threadIdx.x;
  const float inv_hw = 1.f / (float)g.HW;
  // 1) S, Q
  for (int i = tid; i < B * C; i += 256) {
    int b = i / C, c = i % C;
    double s1 = 0.0, s2 = 0.0;
    for (int k = 0; k < g.NCH; ++k) {
      const float* pr = part + ((long)(b * g.NCH + k) * 2) * C;
      s1 += pr[c];
      s2 += pr[C + c];
    }
    S[i] = (float)s1;
    Q[i] = (float)s2;
  }
  __syncthreads();
  // 2) fc1 + lrelu (pre-activation saved)
  for (int i = tid; i < B * Cr; i += 256) {
    int b = i / Cr, j = i % Cr;
    float acc = b1[j];
    const float* wr = w1 + (long)j * C;
    const float* Sb = S + b * C;
    for (int c = 0; c < C; ++c) acc = fmaf(wr[c], Sb[c] / (float)g.HW, acc);
    hpre[i] = acc;
  }
  __syncthreads();
  // 3) fc2 + sigmoid
  for (int i = tid; i < B * C; i += 256) {
    int b = i / C, c = i % C;
    float acc = b2[c];
    const float* wr = w2 + (long)c * Cr;
    const float* hb = hpre + b * Cr;
    for (int j = 0; j < Cr; ++j) acc = fmaf(wr[j], lrelu(hb[j]), acc);
    sg[i] = 1.f / (1.f + expf(-acc));
  }
  __syncthreads();
  // 4) BN statistics of y = a*s, running update, coefficients
  const double n = (double)B * g.HW;
  for (int c = tid; c < C; c += 256) {
    float mu, var;
    if (training) {
      double m1 = 0.0, m2 = 0.0;
      for (int b = 0; b < B; ++b) {
        double s = sg[b * C + c];
        m1 += s * S[b * C + c];
        m2 += s * s * Q[b * C + c];
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
    mean[c] = mu;
    rstd[c] = rs;
    betap[c] = beta[c] - k * mu;
    for (int b = 0; b < B; ++b) alpha[b * C + c] = k * sg[b * C + c];
  }
}

// pass 2 forward: out = lrelu(alpha[b,c]*a + betap[c])
template <int V>
__global__ void __launch_bounds__(256)
se_apply_kernel(const float* __restrict__ z, const float* __restrict__ sc,
                const float* __restrict__ sh, int act, SeGeom g, const float* __restrict__ alpha,
                const float* __restrict__ betap, float* __restrict__ out,
                float* __restrict__ ostats) {
  ChanTile t = chan_tile<V>(g.C);
  const int b = blockIdx.x / g.NCH, ch = blockIdx.x % g.NCH;
  long r0 = (long)b * g.HW + ch * g.rows_per;
  long r1 = min((long)b * g.HW + g.HW, r0 + g.rows_per);
  float o1[V], o2[V];
#pragma unroll
  for (int j = 0; j < V; ++j) { o1[j] = 0.f; o2[j] = 0.f; }
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
        o2[j] += v[j] * v[j];
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
                     float* __restrict__ part) {
  ChanTile t = chan_tile<V>(g.C);
  const int b = blockIdx.x / g.NCH, ch = blockIdx.x % g.NCH;
  long r0 = (long)b * g.HW + ch * g.rows_per;
  long r1 = min((long)b * g.HW + g.HW, r0 + g.rows_per);
  float t1[V], t2[V];
#pragma unroll
  for (int j = 0; j < V; ++j) { t1[j] = 0.f; t2[j] = 0.f; }
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
        t2[j] += g2 * x;
      }
    }
  }
  block_chan_reduce2<V>(t, t1, t2, part, blockIdx.x, g.C);
}

// backward mid. One block. coef layout: A[B*C] Bc[B*C] Cc[B*C]
__global__ void __launch_bounds__(256)
se_bwd_mid_kernel(const float* __restrict__ part, SeGeom g, int Cr, const float* __restrict__ w1,
                  const float* __restrict__ w2, const float* __restrict__ gamma, int training,
                  const float* __restrict__ save, float* __restrict__ dw1, float* __restrict__ db1,
                  float* __restrict__ dw2, float* __restrict__ db2, float* __restrict__ dgamma,
                  float* __restrict__ dbeta, float* __restrict__ scratch, float* __restrict__ coef) {
  const int B = g.B, C = g.C;
  const float* S = save;
  const float* Q = S + B * C;
  const float* hpre = Q + B * C;
  const float* sg = hpre + B * Cr;
  const float* mean = sg + B * C;
  const float* rstd = mean + C;
  float* T1 = scratch;
  float* T2 = T1 + B * C;
  float* G = T2 + B * C;   // [C]
  float* GY = G + C;       // [C]
  float* du = GY + C;      // [B*C]
  float* dh = du + B * C;  // [B*Cr]
  float* A = coef;
  float* Bc = A + B * C;
  float* Cc = Bc + B * C;
  const int tid = threadIdx.x;
  const float inv_hw = 1.f / (float)g.HW;
  const double n = (double)B * g.HW;
  for (int i = tid; i < B * C; i += 256) {
    int b = i / C, c = i % C;
    double s1 = 0.0, s2 = 0.0;
    for (int k = 0; k < g.NCH; ++k) {
      const float* pr = part + ((long)(b * g.NCH + k) * 2) * C;
      s1 += pr[c];
      s2 += pr[C + c];
    }
    T1[i] = (float)s1;
    T2[i] = (float)s2;
  }
  __syncthreads();
  for (int c = tid; c < C; c += 256) {
    double gs = 0.0, gy = 0.0;
    for (int b = 0; b < B; ++b) {
      gs += T1[b * C + c];
      gy += (double)sg[b * C + c] * T2[b * C + c] - (double)mean[c] * T1[b * C + c];
    }
    gy *= rstd[c];
    G[c] = (float)gs;
    GY[c] = (float)gy;
    if (dgamma) dgamma[c] = (float)gy;
    if (dbeta) dbeta[c] = (float)gs;
  }
  __syncthreads();
  // ds -> du = ds * s * (1 - s)
  for (int i = tid; i < B * C; i += 256) {
    int c = i % C;
    float k = gamma[c] * rstd[c];
    float s = sg[i];
    float ds;
    if (training) {
      float yhx = rstd[c] * (s * Q[i] - mean[c] * S[i]);  // sum_hw yhat * a
      ds = k * (T2[i] - (float)(G[c] / n) * S[i] - (float)(GY[c] / n) * yhx);
    } else {
      ds = k * T2[i];
    }
    du[i] = ds * s * (1.f - s);
  }
  __syncthreads();
  // fc2 backward: dw2[c][j] = sum_b du[b,c] * lrelu(hpre[b,j]); db2[c] = sum_b du[b,c]
  for (int i = tid; i < C * Cr; i += 256) {
    int c = i / Cr, j = i % Cr;
    float acc = 0.f;
    for (int b = 0; b < B; ++b) acc += du[b * C + c] * lrelu(hpre[b * Cr + j]);
    dw2[i] = acc;
  }
  for (int c = tid; c < C; c += 256) {
    float acc = 0.f;
    for (int b = 0; b < B; ++b) acc += du[b * C + c];
    db2[c] = acc;
  }
  // dh[b,j] = lrelu'(hpre) * sum_c w2[c][j] du[b,c]
  for (int i = tid; i < B * Cr; i += 256) {
    int b = i / Cr, j = i % Cr;
    float acc = 0.f;
    for (int c = 0; c < C; ++c) acc = fmaf(w2[(long)c * Cr + j], du[b * C + c], acc);
    dh[i] = acc * lrelu_d(hpre[i]);
  }
  __syncthreads();
  // fc1 backward: dw1[j][c] = sum_b dh[b,j] * m[b,c]; db1[j] = sum_b dh[b,j]
  for (int i = tid; i < Cr * C; i += 256) {
    int j = i / C, c = i % C;
    float acc = 0.f;
    for (int b = 0; b < B; ++b) acc += dh[b * Cr + j] * (S[b * C + c] * inv_hw);
    dw1[i] = acc;
  }
  for (int j = tid; j < Cr; j += 256) {
    float acc = 0.f;
    for (int b = 0; b < B; ++b) acc += dh[b * Cr + j];
    db1[j] = acc;
  }
  // coefficients: da = A*g2 + Bc*a + Cc
  for (int i = tid; i < B * C; i += 256) {
    int b = i / C, c = i % C;
    float dm = 0.f;
    for (int j = 0; j < Cr; ++j) dm = fmaf(w1[(long)j * C + c], dh[b * Cr + j], dm);
    float k = gamma[c] * rstd[c];
    float s = sg[i];
    if (training) {
      float gn = (float)(G[c] / n), gyn = (float)(GY[c] / n);
      A[i] = s * k;
      Bc[i] = -s * s * k * rstd[c] * gyn;
      Cc[i] = -s * k * gn + s * k * rstd[c] * mean[c] * gyn + dm * inv_hw;
    } else {
      A[i] = s * k;
      Bc[i] = 0.f;
      Cc[i] = dm * inv_hw;
    }
  }
}

template <int V>
__global__ void __launch_bounds__(256)
se_bwd_apply_kernel(const float* __restrict__ z, const float* __restrict__ dout,
                    const float* __restrict__ sc, const float* __restrict__ sh, int act, SeGeom g,
                    const float* __restrict__ alpha, const float* __restrict__ betap,
                    const float* __restrict__ coef, float* __restrict__ da) {
  ChanTile t = chan_tile<V>(g.C);
  if (!t.active) return;
  const int b = blockIdx.x / g.NCH, ch = blockIdx.x % g.NCH;
  long r0 = (long)b * g.HW + ch * g.rows_per;
  long r1 = min((long)b * g.HW + g.HW, r0 + g.rows_per);
  const int BC = g.B * g.C;
  float s[V], h[V], al[V], be[V], A[V], Bc[V], Cc[V];
#pragma unroll
  for (int j = 0; j < V; ++j) {
    int i = b * g.C + t.c0 + j;
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
      d[j] = A[j] * g2 + Bc[j] * x + Cc[j];
    }
    stv<V>(da + r * g.C + t.c0, d);
  }
}

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------
extern "C" size_t accunet_se_save_elems(int B, int C, int Cr) {
  return (size_t)B * C * 4 + (size_t)B * Cr + 3 * (size_t)C;
}

// rows of the optional SE-output statistics block written by accunet_se_fwd
extern "C" int accunet_se_stats_rows(int B, int HW, int C) {
  SeGeom g = se_geom(B, HW, C);
  return B * g.NCH;
}

extern "C" size_t accunet_se_ws_elems(int B, int HW, int C, int Cr) {
  SeGeom g = se_geom(B, HW, C);
  size_t part = (size_t)B * g.NCH * 2 * C;
  size_t scratch = (size_t)B * C * 3 + 2 * (size_t)C + (size_t)B * Cr;
  size_t coef = (size_t)B * C * 3;
  return part + scratch + coef;
}

extern "C" int accunet_se_fwd(const float* z, const float* sc, const float* sh, int act, int B,
                              int HW, int C, int Cr, const float* w1, const float* b1,
                              const float* w2, const float* b2, const float* gamma,
                              const float* beta, float* rmean, float* rvar, long long* nbt,
                              float momentum, float eps, int training, float* out, float* save,
                              float* ostats, float* ws, size_t ws_elems, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (ws_elems < accunet_se_ws_elems(B, HW, C, Cr)) return ACC_EBADARG;
  SeGeom g = se_geom(B, HW, C);
  int V = (C % 4 == 0) ? 4 : 1;
  dim3 grid(B * g.NCH, ceil_div(C / V, 64));
  float* part = ws;
  if (V == 4)
    hipLaunchKernelGGL(se_reduce_kernel<4>, grid, dim3(256), 0, s, z, sc, sh, act, g, part);
  else
    hipLaunchKernelGGL(se_reduce_kernel<1>, grid, dim3(256), 0, s, z, sc, sh, act, g, part);
  hipLaunchKernelGGL(se_mid_kernel, dim3(1), dim3(256), 0, s, part, g, Cr, w1, b1, w2, b2, gamma,
                     beta, rmean, rvar, momentum, eps, training, save);
  if (training && nbt) hipLaunchKernelGGL(inc_i64_kernel, dim3(1), dim3(1), 0, s, nbt);
  const float* alpha = save + (size_t)B * C * 3 + (size_t)B * Cr + 2 * (size_t)C;
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
  SeGeom g = se_geom(B, HW, C);
  int V = (C % 4 == 0) ? 4 : 1;
  dim3 grid(B * g.NCH, ceil_div(C / V, 64));
  float* part = ws;
  float* scratch = part + (size_t)B * g.NCH * 2 * C;
  float* coef = scratch + (size_t)B * C * 3 + 2 * (size_t)C + (size_t)B * Cr;
  const float* alpha = save + (size_t)B * C * 3 + (size_t)B * Cr + 2 * (size_t)C;
  const float* betap = alpha + (size_t)B * C;
  if (V == 4)
    hipLaunchKernelGGL(se_bwd_reduce_kernel<4>, grid, dim3(256), 0, s, z, dout, sc, sh, act, g,
                       alpha, betap, part);
  else
    hipLaunchKernelGGL(se_bwd_reduce_kernel<1>, grid, dim3(256), 0, s, z, dout, sc, sh, act, g,
                       alpha, betap, part);
  hipLaunchKernelGGL(se_bwd_mid_kernel, dim3(1), dim3(256), 0, s, part, g, Cr, w1, w2, gamma,
                     training, save, dw1, db1, dw2, db2, dgamma, dbeta, scratch, coef);
  if (V == 4)
    hipLaunchKernelGGL(se_bwd_apply_kernel<4>, grid, dim3(256), 0, s, z, dout, sc, sh, act, g,
                       alpha, betap, coef, da);
  else
    hipLaunchKernelGGL(se_bwd_apply_kernel<1>, grid, dim3(256), 0, s, z, dout, sc, sh, act, g,
                       alpha, betap, coef, da);
  return hipGetLastError() == hipSuccess ? ACC_OK : ACC_ELAUNCH;
}
