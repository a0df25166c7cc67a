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
//   pass 2 (se_apply): prologue = BN stats of y = a*s derived exactly from (S, Q, s)
//                      for the block's channels: mean = sum_b s*S / n, E[y^2] = sum_b
//                      s^2*Q / n -> per-(b,c) alpha = gamma*rstd*s, per-c beta' = beta -
//                      gamma*rstd*mean (se_chan_bn); then out = lrelu(alpha*a + beta')
//                                                                  [reads z, writes out]
// so neither a nor y = a*s is ever materialised.
//
// Backward:
//   pass 1: per-(b,c) T1 = sum g2, T2 = sum g2*a   (g2 = dout * lrelu'(alpha*a+beta'))
//   mid:    BN backward reduced to per-(b,c) terms, SE fc backward, and coefficients of
//           da = A*g2 + Bc*a + Cc
//   pass 2: da (then the caller runs the preceding BatchNorm's backward on it)
#include <stdlib.h>
#include "common.h"
#include "chan.h"
#include "kernels.h"
#include <cstdlib>
#include <type_traits>

#define SE_F32_ROWS 64  // rows a thread sums in fp32 before the fp64 block reduction

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
  // a thread walks rows_per / RG rows of its chunk (RG = 256 / min(C/V, 64) row groups,
  // chan_tile); the backward's first pass sums them in fp32 (se_bwd_reduce_pro_kernel),
  // so chunks are cut short enough that no thread sums more than SE_F32_ROWS rows
  // (ACC-UNet's shapes at 256^2 / 512^2 walk at most 32 -- only larger images get
  // more chunks)
  const int cq = (C % 4 == 0) ? C / 4 : C;
  const int rg = 256 / (cq < 64 ? (cq > 0 ? cq : 1) : 64);
  const long cap = (long)SE_F32_ROWS * rg;
  const long need = (HW + cap - 1) / cap;
  if (need > g.NCH) g.NCH = (int)need;
  g.rows_per = (HW + g.NCH - 1) / g.NCH;
  return g;
}

// Forward middle-step arguments (the gate MLP and the BatchNorm of the gated tensor)
struct SeMid {
  int Cr;
  const float *w1, *b1, *w2, *b2, *gamma, *beta;
  float *rmean, *rvar;
  long long* nbt;
  float momentum, eps;
  int training;
  float* save;
};

// Per-thread fp64 sums of a = act(z*sc + sh) and a^2 over the thread's rows of the
// block's row chunk [r0, r1) (row order, so bit-identical to the plain loop).
template <int V, typename T, bool PRO>
ACC_DEV void se_fwd_sums(const T* __restrict__ z, const float* __restrict__ sc,
                         const float* __restrict__ sh, int act, const SeGeom& g,
                         const ChanTile& t, long r0, long r1, double (&a)[V], double (&q)[V]) {
  if (!t.active) return;
  float s[V], h[V];
#pragma unroll
  for (int j = 0; j < V; ++j) {
    s[j] = PRO ? sc[t.c0 + j] : 1.f;
    h[j] = PRO ? sh[t.c0 + j] : 0.f;
  }
  if constexpr (V == 4) {
    quad_rows1<8>(z + r0 * g.C, r1 > r0 ? r1 - r0 : 0, t.rg, t.RG, g.C, t.c0,
                  [&](bool ok, float4 x4, unsigned) {
                    const float v[4] = {x4.x, x4.y, x4.z, x4.w};
#pragma unroll
                    for (int j = 0; j < V; ++j) {
                      double x = PRO ? apply_act(v[j] * s[j] + h[j], act) : v[j];
                      x = ok ? x : 0.0;
                      a[j] += x;
                      q[j] += x * x;
                    }
                  });
    return;
  }
  for (long r = r0 + t.rg; r < r1; r += t.RG) {
    float v[V];
    ldv<V>(z + r * g.C + t.c0, v);
#pragma unroll
    for (int j = 0; j < V; ++j) {
      double x = PRO ? apply_act(v[j] * s[j] + h[j], act) : v[j];
      a[j] += x;
      q[j] += x * x;
    }
  }
}

// middle step of one sample b: the chunk partials of b -> S[b,c], Q[b,c] (fixed
// summation order: 4 chunk groups k = grp mod 4, each in chunk order, then
// ((g0 + g1) + g2) + g3), the channel means, fc1 (+LeakyReLU) and fc2 (+sigmoid) of
// that sample (the reference gate, :41-45). sm: LDS m[C] | h'[Cr].
ACC_DEV void se_mid_sample_body(const double* __restrict__ part, const SeGeom& g, const SeMid& m,
                                int b, float* sm) {
  __shared__ double r[2][4][64];
  const int B = g.B, C = g.C, Cr = m.Cr, tid = threadIdx.x;
  SeSave sv = se_save_view(m.save, B, C, Cr);
  float* mm = sm;
  float* hp = sm + C;
  const int cl = tid & 63, grp = tid >> 6;
  for (int cb = 0; cb < C; cb += 64) {
    const int c = cb + cl;
    double s2[2] = {0.0, 0.0};
    if (c < C)
      ordered_strided_sum<8>(s2, grp, g.NCH, 4, [&](int k, double (&v)[2]) {
        const double* pr = part + ((long)(b * g.NCH + k) * 2) * C;
        v[0] = *(pr + c);
        v[1] = *(pr + C + c);
      });
    r[0][grp][cl] = s2[0];
    r[1][grp][cl] = s2[1];
    __syncthreads();
    if (grp == 0 && c < C) {
      const double S = ((r[0][0][cl] + r[0][1][cl]) + r[0][2][cl]) + r[0][3][cl];
      const double Q = ((r[1][0][cl] + r[1][1][cl]) + r[1][2][cl]) + r[1][3][cl];
      sv.S[b * C + c] = S;
      sv.Q[b * C + c] = Q;
      mm[c] = (float)(S / g.HW);
    }
    __syncthreads();
  }
  // fc1: 4 threads per output, interleaved over the input channels
  for (int o = tid; o < Cr * 4; o += 256) {
    int j = o >> 2, part_i = o & 3;
    float acc = 0.f;
    const float* wr = m.w1 + (long)j * C;
#pragma unroll 8
    for (int c = part_i; c < C; c += 4) acc = fmaf(wr[c], mm[c], acc);
    acc += __shfl_xor(acc, 1);
    acc += __shfl_xor(acc, 2);
    if (part_i == 0) {
      acc += m.b1[j];
      sv.hpre[b * Cr + j] = acc;
      hp[j] = lrelu(acc);
    }
  }
  __syncthreads();
  for (int c = tid; c < C; c += 256) {
    float acc = m.b2[c];
    const float* wr = m.w2 + (long)c * Cr;
#pragma unroll 8
    for (int j = 0; j < Cr; ++j) acc = fmaf(wr[j], hp[j], acc);
    sv.sg[b * C + c] = 1.f / (1.f + expf(-acc));
  }
}

// middle step, part 2, channel c: BatchNorm statistics of y = a*s derived from
// (S, Q, s) -> k = gamma*rstd and beta' = beta - k*mean. Every apply block computes this
// for its own channels in its prologue (same loop, same order: identical values in every
// block, and no launch of its own); the block `writer` also updates the running
// statistics and stores mean, rstd and beta' for the backward.
struct SeChanBN {
  float k, betap;
};
ACC_DEV SeChanBN se_chan_bn(const SeGeom& g, const SeMid& m, int c, bool writer) {
  const int B = g.B, C = g.C;
  SeSave sv = se_save_view(m.save, B, C, m.Cr);
  const double n = (double)B * g.HW;
  float mu, var;
  if (m.training) {
    double m1 = 0.0, m2 = 0.0;
#pragma unroll 8
    for (int b = 0; b < B; ++b) {
      double s = *(sv.sg + b * C + c);
      m1 += s * *(sv.S + b * C + c);
      m2 += s * s * *(sv.Q + b * C + c);
    }
    m1 /= n;
    m2 = m2 / n - m1 * m1;
    if (m2 < 0.0) m2 = 0.0;
    mu = (float)m1;
    var = (float)m2;
    if (writer && m.rmean) m.rmean[c] = (1.f - m.momentum) * m.rmean[c] + m.momentum * mu;
    if (writer && m.rvar)
      m.rvar[c] = (1.f - m.momentum) * m.rvar[c] + m.momentum * (float)(m2 * n / (n - 1.0));
  } else {
    mu = m.rmean[c];
    var = m.rvar[c];
  }
  float rs = 1.f / sqrtf(var + m.eps);
  float k = m.gamma[c] * rs;
  SeChanBN r{k, m.beta[c] - k * mu};
  if (writer) {
    sv.mean[c] = mu;
    sv.rstd[c] = rs;
    sv.betap[c] = r.betap;
  }
  return r;
}

// pass 1 forward: partials part[(b*NCH + chunk)][2][C] of (sum a, sum a^2).
// (The middle step stays two launches: folding it into this launch's last blocks with
// ticketed hand-offs measured slower, as its cost is the chain of dependent memory
// round trips, not the launches.)
template <int V, typename T, bool PRO>
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
  se_fwd_sums<V, T, PRO>(z, sc, sh, act, g, t, r0, r1, a, q);
  block_chan_reduce2<V>(t, a, q, part, blockIdx.x, g.C);
}

// middle step: per sample, then per channel
__global__ void __launch_bounds__(256)
se_mid_sample_kernel(const double* __restrict__ part, SeGeom g, SeMid m) {
  extern __shared__ __attribute__((aligned(16))) float se_dyn[];
  se_mid_sample_body(part, g, m, blockIdx.x, se_dyn);
}

// pass 2 forward: out = lrelu(alpha[b,c]*a + betap[c]) (+ res: the residual add that
// follows the SE in ResPath, ACC_UNet.py:326, and in the MLFC merge, :489-520, fused
// so the SE output itself is never written: the sum is, as rnd(rnd(y) + res), the
// value the separate add would have stored)
template <int V, typename T, bool PRO, bool RES>
__global__ void __launch_bounds__(256)
se_apply_kernel(const T* __restrict__ z, const float* __restrict__ sc,
                const float* __restrict__ sh, int act, SeGeom g, SeMid m,
                const T* __restrict__ res, T* __restrict__ out,
                double* __restrict__ ostats, int rev) {
  __shared__ float s_k[256], s_bp[256];
  ChanTile t = chan_tile<V>(g.C);
  // rev: the blocks walk the chunks in the reverse of the reduce's order, so the first
  // re-reads are of the lines the reduce fetched last (Infinity Cache residency)
  const int lin = rev ? (int)(gridDim.x - 1 - blockIdx.x) : (int)blockIdx.x;
  const int b = lin / g.NCH, ch = lin % g.NCH;
  // prologue: the BatchNorm-of-gated step of the block's channels (se_chan_bn); the
  // blocks of chunk 0 store alpha = k*s of their sample, block (0, y) the per-channel
  // state and the running statistics
  const SeSave sv = se_save_view(m.save, g.B, g.C, m.Cr);
  {
    const int cbase = blockIdx.y * 64 * V, ncb = min(64 * V, g.C - cbase);
    const bool writer = lin == 0;
    for (int i = threadIdx.x; i < ncb; i += 256) {
      const int c = cbase + i;
      const SeChanBN r = se_chan_bn(g, m, c, writer);
      s_k[i] = r.k;
      s_bp[i] = r.betap;
      if (ch == 0) sv.alpha[b * g.C + c] = r.k * *(sv.sg + b * g.C + c);
    }
    // num_batches_tracked (training only; null otherwise)
    if (writer && blockIdx.y == 0 && threadIdx.x == 0 && m.nbt) *m.nbt += 1;
    __syncthreads();
  }
  long r0 = (long)b * g.HW + ch * g.rows_per;
  long r1 = min((long)b * g.HW + g.HW, r0 + g.rows_per);
  double o1[V], o2[V];
#pragma unroll
  for (int j = 0; j < V; ++j) { o1[j] = 0.0; o2[j] = 0.0; }
  if (t.active) {
    float s[V], h[V], al[V], be[V];
#pragma unroll
    for (int j = 0; j < V; ++j) {
      s[j] = PRO ? sc[t.c0 + j] : 1.f;
      h[j] = PRO ? sh[t.c0 + j] : 0.f;
      const int cl = t.c0 + j - (int)blockIdx.y * 64 * V;  // block-local channel
      al[j] = s_k[cl] * sv.sg[b * g.C + t.c0 + j];
      be[j] = s_bp[cl];
    }
    const bool st = ostats != nullptr;
    auto elem = [&](bool ok, const float (&x)[V], const float (&rv)[V], float (&v)[V]) {
#pragma unroll
      for (int j = 0; j < V; ++j) {
        const float a = PRO ? apply_act(x[j] * s[j] + h[j], act) : x[j];
        v[j] = rnd<T>(lrelu(al[j] * a + be[j]));  // statistics of the stored value
        if (RES) v[j] = rnd<T>(v[j] + rv[j]);
        const double y = (st && ok) ? (double)v[j] : 0.0;
        o1[j] += y;
        o2[j] += y * y;
      }
    };
    if constexpr (V == 4) {
      const long nr = r1 > r0 ? r1 - r0 : 0;
      const __amdgpu_buffer_rsrc_t ro = acc_rsrc(out + r0 * g.C, (unsigned)(nr * g.C * sizeof(T)));
      auto body = [&](bool ok, float4 x4, float4 r4, unsigned off) {
        const float x[4] = {x4.x, x4.y, x4.z, x4.w}, rv[4] = {r4.x, r4.y, r4.z, r4.w};
        float v[4];
        elem(ok, x, rv, v);
        bufq_st<ACC_STREAM_STORE_AUX>(ro, off, make_float4(v[0], v[1], v[2], v[3]), (T*)nullptr);
      };
      if (RES)
        quad_rows2<8>(z + r0 * g.C, res + r0 * g.C, nr, t.rg, t.RG, g.C, t.c0, body);
      else
        quad_rows1<8>(z + r0 * g.C, nr, t.rg, t.RG, g.C, t.c0, [&](bool ok, float4 x4, unsigned off) {
          body(ok, x4, make_float4(0.f, 0.f, 0.f, 0.f), off);
        });
    } else {
      for (long r = r0 + t.rg; r < r1; r += t.RG) {
        float x[V], rv[V], v[V];
        ldv<V>(z + r * g.C + t.c0, x);
        if (RES) ldv<V>(res + r * g.C + t.c0, rv);
        else {
#pragma unroll
          for (int j = 0; j < V; ++j) rv[j] = 0.f;
        }
        elem(true, x, rv, v);
        stv<V>(out + r * g.C + t.c0, v);
      }
    }
  }
  // optional statistics of the SE output (MLFC feeds it straight into bns_l, :427-487)
  if (ostats) block_chan_reduce2<V>(t, o1, o2, ostats, lin, g.C);
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
  block_chan_reduce2<V, double, true>(t, t1, t2, part, blockIdx.x, g.C, (long)g.B * g.NCH);
}

// backward middle step. coef (fp32): A[B*C] Bc[B*C] Cc[B*C] with
//   da = A*g2 + Bc*(a*s - mean) + Cc
// scratch (fp64): G[C] GY[C] du[B*C] dh[B*Cr] T1[B*C] T2[B*C] (+ U1..W3 with a prologue)
// Three launches: part sums + channel step (se_bwd_chan_sum_kernel), sample step,
// parameter + prologue-coefficient step (se_bwd_tail_kernel).
struct SeBwdMid {
  int Cr;
  const float *w1, *w2, *gamma;
  int training;
  float* save;
  double* scratch;
  float* coef;
  float *dw1, *db1, *dw2, *db2, *dgamma, *dbeta;
  // prologue BatchNorm (accunet_se_bwd_pro)
  const float *pst, *pgamma;
  int ptraining;
  float *dpg, *dpb, *pcoef;
  float* dsum;  // sum_p dz: the bias gradient of z's producer (bn_dsum), or null
};

ACC_DEV double* se_T1(const SeGeom& g, const SeBwdMid& m) {
  return m.scratch + 2 * (size_t)g.C + (size_t)g.B * g.C + (size_t)g.B * m.Cr;
}

// SE_LANES lanes per channel: lane l handles samples b = l, l + SE_LANES, ...; the
// per-channel sums are reduced with an xor butterfly inside the lane group and lane 0's
// value is broadcast, so every lane uses identical totals (deterministic). All lanes of
// the wave take part (dead channels too).
#define SE_LANES 16
ACC_DEV double se_lane_sum(double v) {
#pragma unroll
  for (int off = 1; off < SE_LANES; off <<= 1) v += __shfl_xor(v, off);
  return __shfl(v, (threadIdx.x & 63) & ~(SE_LANES - 1));
}

// channel step, channel c (lane `lane` of its group): BN backward sums and
// du = ds * s * (1 - s).
ACC_DEV void se_bwd_chan_body(const SeGeom& g, const SeBwdMid& m, int c, int lane) {
  const int B = g.B, C = g.C;
  const bool live = c < C;
  const int cc = live ? c : 0;
  SeSave sv = se_save_view(m.save, B, C, m.Cr);
  double* G = m.scratch;
  double* GY = G + C;
  double* du = GY + C;
  const double* T1 = se_T1(g, m);
  const double* T2 = T1 + (size_t)B * C;
  const double n = (double)B * g.HW;
  const double mean = sv.mean[cc], rstd = sv.rstd[cc];
  double gs = 0.0, gy = 0.0;
  if (live)
    for (int b = lane; b < B; b += SE_LANES) {
      double t1 = *(T1 + b * C + c);
      gs += t1;
      gy += (double)sv.sg[b * C + c] * *(T2 + b * C + c) - mean * t1;
    }
  gs = se_lane_sum(gs);
  gy = se_lane_sum(gy) * rstd;
  if (!live) return;
  if (lane == 0) {
    G[c] = gs;
    GY[c] = gy;
    if (m.dgamma) m.dgamma[c] = (float)gy;
    if (m.dbeta) m.dbeta[c] = (float)gs;
  }
  const double k = (double)m.gamma[c] * rstd;
  for (int b = lane; b < B; b += SE_LANES) {
    double s = sv.sg[b * C + c];
    double t2 = *(T2 + b * C + c);
    double ds;
    if (m.training) {
      double yha = rstd * (s * sv.Q[b * C + c] - mean * sv.S[b * C + c]);
      ds = k * (t2 - (gs / n) * sv.S[b * C + c] - (gy / n) * yha);
    } else {
      ds = k * t2;
    }
    du[b * C + c] = ds * s * (1.0 - s);
  }
}


// Part sums + channel step in one launch, one block per channel c: 16 lanes per
// sample b sum the chunk partials k = lane, lane + 16, ... (every quantity's loads in
// flight together), an xor butterfly inside the 16-lane group adds the lane sums in a
// fixed order, lane 0 stores T[q][b, c] (fp64 scratch, read by the prologue step
// too); then the first wave runs the channel step of c (se_bwd_chan_body). One
// launch and two memory round trips instead of two launches.
template <int NQ>
__global__ void __launch_bounds__(256)
se_bwd_chan_sum_kernel(const double* __restrict__ part, SeGeom g, SeBwdMid m) {
  const int C = g.C, c = blockIdx.x, tid = threadIdx.x;
  const int lane = tid % 16;
  const long RB = (long)g.B * g.NCH;  // partial rows
  double* T = se_T1(g, m);
  const long BC = (long)g.B * C;
  for (int b0 = 0; b0 < g.B; b0 += 16) {
    const int b = b0 + tid / 16;
    double s[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) s[q] = 0.0;
    if (b < g.B)
      ordered_strided_sum<4>(s, lane, g.NCH, 16, [&](int k, double (&v)[NQ]) {
        // channel-major partials [q][c][b*NCH + k]: the 16 lanes of a sample read 16
        // consecutive chunks, the block's samples consecutive runs of them
        const double* pr = part + (long)c * RB + (long)b * g.NCH + k;
#pragma unroll
        for (int q = 0; q < NQ; ++q) v[q] = pr[(long)q * C * RB];
      });
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
#pragma unroll
      for (int off = 1; off < 16; off <<= 1) s[q] += __shfl_xor(s[q], off);
    }
    if (b < g.B && lane == 0) {
#pragma unroll
      for (int q = 0; q < NQ; ++q) T[q * BC + (long)b * C + c] = s[q];
    }
  }
  __syncthreads();  // T of channel c complete (same-block global stores)
  if (tid < 64) se_bwd_chan_body(g, m, tid < SE_LANES ? c : C, tid % SE_LANES);
}

// sample step, sample b: dh = lrelu'(hpre) * W2^T du, dm = W1^T dh, coefficients.
// smd: LDS dh[Cr]. Ends with a barrier (smd reusable).
ACC_DEV void se_bwd_sample_body(const SeGeom& g, const SeBwdMid& m, int b, double* smd) {
  const int B = g.B, C = g.C, Cr = m.Cr, tid = threadIdx.x;
  SeSave sv = se_save_view(m.save, B, C, Cr);
  const double* G = m.scratch;
  const double* GY = G + C;
  const double* du = GY + C;
  double* dh = const_cast<double*>(du) + (size_t)B * C;
  for (int o = tid; o < Cr * 4; o += 256) {
    int j = o >> 2, part_i = o & 3;
    double acc = 0.0;
#pragma unroll 8
    for (int c = part_i; c < C; c += 4) acc += (double)m.w2[(long)c * Cr + j] * du[b * C + c];
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
  float* A = m.coef;
  float* Bc = A + (size_t)B * C;
  float* Cc = Bc + (size_t)B * C;
  for (int c = tid; c < C; c += 256) {
    double dm = 0.0;
#pragma unroll 8
    for (int j = 0; j < Cr; ++j) dm += (double)m.w1[(long)j * C + c] * smd[j];
    double k = (double)m.gamma[c] * sv.rstd[c];
    double s = sv.sg[b * C + c];
    int i = b * C + c;
    A[i] = (float)(s * k);
    if (m.training) {
      Bc[i] = (float)(-s * k * sv.rstd[c] * (GY[c] / n));
      Cc[i] = (float)(-s * k * (G[c] / n) + dm / g.HW);
    } else {
      Bc[i] = 0.f;
      Cc[i] = (float)(dm / g.HW);
    }
  }
  __syncthreads();
}

__global__ void __launch_bounds__(256) se_bwd_sample_kernel(SeGeom g, SeBwdMid m) {
  extern __shared__ __attribute__((aligned(16))) double smd[];  // dh[Cr]
  se_bwd_sample_body(g, m, blockIdx.x, smd);
}

// parameter step, output i of [dw2 | dw1 | db2 | db1] (sums over the batch)
ACC_DEV void se_bwd_param_body(const SeGeom& g, const SeBwdMid& m, long i) {
  const int B = g.B, C = g.C, Cr = m.Cr;
  SeSave sv = se_save_view(m.save, B, C, Cr);
  const double* du = m.scratch + 2 * (size_t)C;
  const double* dh = du + (size_t)B * C;
  const long nW = (long)C * Cr;
  if (i < nW) {  // dw2[c][j] = sum_b du[b,c] * lrelu(hpre[b,j])
    int c = (int)(i / Cr), j = (int)(i % Cr);
    double acc = 0.0;
#pragma unroll 8
    for (int b = 0; b < B; ++b) acc += du[b * C + c] * lrelu(sv.hpre[b * Cr + j]);
    m.dw2[i] = (float)acc;
  } else if (i < 2 * nW) {  // dw1[j][c] = sum_b dh[b,j] * m[b,c]
    long t = i - nW;
    int j = (int)(t / C), c = (int)(t % C);
    double acc = 0.0;
#pragma unroll 8
    for (int b = 0; b < B; ++b) acc += dh[b * Cr + j] * (sv.S[b * C + c] / g.HW);
    m.dw1[t] = (float)acc;
  } else if (i < 2 * nW + C) {
    int c = (int)(i - 2 * nW);
    double acc = 0.0;
#pragma unroll 8
    for (int b = 0; b < B; ++b) acc += du[b * C + c];
    m.db2[c] = (float)acc;
  } else if (i < 2 * nW + C + Cr) {
    int j = (int)(i - 2 * nW - C);
    double acc = 0.0;
#pragma unroll 8
    for (int b = 0; b < B; ++b) acc += dh[b * Cr + j];
    m.db1[j] = (float)acc;
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

#define SE_PRO_NQ 8  // T1, T2, U1, U2, U3, W1, W2, W3

// prologue coefficient step, channel c (lane `lane` of its group): the prologue BN's
// backward coefficients dz = k1*g + k2*(z - mean1) + k3, dgamma1 = sum g*xhat,
// dbeta1 = sum g, from the per-(b,c) sums UW[i][B*C] (i = 0..5 -> U1 U2 U3 W1 W2 W3)
// and the SE coefficients A, Bc, Cc.
ACC_DEV void se_pro_coef_body(const SeGeom& g, const SeBwdMid& m, int c, int lane) {
  const int B = g.B, C = g.C;
  const bool live = c < C;
  SeSave sv = se_save_view(m.save, B, C, m.Cr);
  const long BC = (long)B * C;
  const double* UW = se_T1(g, m) + 2 * BC;
  const float* A = m.coef;
  const float* Bc = A + BC;
  const float* Cc = Bc + BC;
  double sg = 0.0, sgx = 0.0;
  if (live) {
    const double mean = sv.mean[c];
    for (int b = lane; b < B; b += SE_LANES) {
      const long i = (long)b * C + c;
      const double a = A[i], bb = Bc[i], s = sv.sg[i];
      const double cst = (double)Cc[i] - bb * mean;
      sg += a * *(UW + 0 * BC + i) + bb * s * *(UW + 1 * BC + i) +
            cst * *(UW + 2 * BC + i);
      sgx += a * *(UW + 3 * BC + i) + bb * s * *(UW + 4 * BC + i) +
             cst * *(UW + 5 * BC + i);
    }
  }
  sg = se_lane_sum(sg);
  sgx = se_lane_sum(sgx);
  if (!live || lane != 0) return;
  const float rstd1 = m.pst[BN_RSTD * C + c];
  sgx *= rstd1;  // sum g*xhat
  if (m.dpg) m.dpg[c] = (float)sgx;
  if (m.dpb) m.dpb[c] = (float)sg;
  const double n = (double)B * g.HW;
  const float ga = m.pgamma ? m.pgamma[c] : 1.f;
  const float k1 = ga * rstd1;
  float k2 = 0.f, k3 = 0.f;
  if (m.ptraining) {  // same coefficients as bn_bwd_finalize_kernel (csrc/bn.hip)
    const float mg = (float)(sg / n), mgx = (float)(sgx / n);
    k2 = -k1 * rstd1 * mgx;
    k3 = -k1 * mg;
  }
  m.pcoef[c] = k1;
  m.pcoef[C + c] = k2;
  m.pcoef[2 * C + c] = k3;
  // sum_p dz = k1 sum g + n k3 (+ k2 sum (z - mean1) = 0 up to the mean's rounding), as
  // bn_dsum in csrc/bn.hip: no column-sum pass over dz
  if (m.dsum) m.dsum[c] = (float)((double)k1 * sg + n * (double)k3);
}


// parameter step and (prologue) coefficient step in one launch: they depend on the
// sample step only, not on each other. Blocks [0, npb) run the parameter step.
__global__ void __launch_bounds__(256) se_bwd_tail_kernel(SeGeom g, SeBwdMid m, int npb) {
  if ((int)blockIdx.x < npb) {
    se_bwd_param_body(g, m, blockIdx.x * (long)blockDim.x + threadIdx.x);
  } else {
    const int gid = (blockIdx.x - npb) * blockDim.x + threadIdx.x;
    se_pro_coef_body(g, m, gid / SE_LANES, gid % SE_LANES);
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
  // fp32 sums over the thread's rows (at most SE_F32_ROWS: se_geom cuts the chunks so),
  // fp64 from the block reduction on: half the VALU work of per-element fp64 accumulation
  float accf[SE_PRO_NQ][V];
#pragma unroll
  for (int i = 0; i < SE_PRO_NQ; ++i)
#pragma unroll
    for (int j = 0; j < V; ++j) accf[i][j] = 0.f;
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
    auto row = [&](const float (&v)[V], const float (&d)[V]) {
#pragma unroll
      for (int j = 0; j < V; ++j) {
        const float pre = v[j] * s[j] + h[j];
        const float x = apply_act(pre, act);
        const float lp = act == ACT_LRELU ? lrelu_d(pre) : 1.f;
        const float g2 = d[j] * lrelu_d(al[j] * x + be[j]);
        const float xc = v[j] - mu[j];
        const float lg = lp * g2, la = lp * x;
        accf[0][j] += g2;
        accf[1][j] = fmaf(g2, x, accf[1][j]);
        accf[2][j] += lg;
        accf[3][j] += la;
        accf[4][j] += lp;
        accf[5][j] = fmaf(lg, xc, accf[5][j]);
        accf[6][j] = fmaf(la, xc, accf[6][j]);
        accf[7][j] = fmaf(lp, xc, accf[7][j]);
      }
    };
    for (long r = r0 + t.rg; r < r1; r += t.RG) {
      float v[V], d[V];
      ldv<V>(z + r * C + t.c0, v);
      ldv<V>(dout + r * C + t.c0, d);
      row(v, d);
    }
  }
  double acc[SE_PRO_NQ][V];
#pragma unroll
  for (int i = 0; i < SE_PRO_NQ; ++i)
#pragma unroll
    for (int j = 0; j < V; ++j) acc[i][j] = (double)accf[i][j];
  block_chan_reduceN<V, SE_PRO_NQ, double, true>(t, acc, part, blockIdx.x, C, (long)g.B * g.NCH);
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
  const bool want_cs = colsum != nullptr;
  auto row = [&](bool ok, float (&v)[V], float (&d)[V]) {
#pragma unroll
    for (int j = 0; j < V; ++j) {
      const float pre = v[j] * s[j] + h[j];
      const float x = apply_act(pre, act);
      const float g2 = d[j] * lrelu_d(al[j] * x + be[j]);
      float da = A[j] * g2 + Bc[j] * (x * sgv[j] - mu[j]) + Cc[j];
      if (act == ACT_LRELU) da *= lrelu_d(pre);
      d[j] = rnd<T>(k1[j] * da + k2[j] * (v[j] - mu1[j]) + k3[j]);
      cs[j] += (want_cs && ok) ? (double)d[j] : 0.0;
    }
  };
  if constexpr (V == 4) {
    const long nr = r1 > r0 ? r1 - r0 : 0;
    const __amdgpu_buffer_rsrc_t ro = acc_rsrc(dz + r0 * C, (unsigned)(nr * C * sizeof(T)));
    quad_rows2<4>(z + r0 * C, dout + r0 * C, nr, t.rg, t.RG, C, t.c0,
                  [&](bool ok, float4 z4, float4 d4, unsigned off) {
                    float v[V] = {z4.x, z4.y, z4.z, z4.w};  // V == 4 here
                    float d[V] = {d4.x, d4.y, d4.z, d4.w};
                    row(ok, v, d);
                    bufq_st<ACC_STREAM_STORE_AUX>(ro, off, make_float4(d[0], d[1 % V], d[2 % V], d[3 % V]), (T*)nullptr);
                  });
  } else {
    for (long r = r0 + t.rg; r < r1; r += t.RG) {
      float v[V], d[V];
      ldv<V>(z + r * C + t.c0, v);
      ldv<V>(dout + r * C + t.c0, d);
      row(true, v, d);
      stv<V>(dz + r * C + t.c0, d);
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

// the streaming loops address a row chunk through one buffer descriptor (< 2^31 bytes)
static bool se_chunk_ok(const SeGeom& g, int dt) {
  return g.rows_per * (long)g.C * (dt == ACC_BF16 ? 2 : 4) < (1L << 31);
}

// ACCUNET_SE_REV=1: the apply pass walks the chunks in reverse (A/B knob, default off)
static int se_rev() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("ACCUNET_SE_REV");
    v = e ? atoi(e) : 0;
  }
  return v;
}

extern "C" int accunet_se_fwd(const void* z, const float* sc, const float* sh, int act, int B,
                              int HW, int C, int Cr, const float* w1, const float* b1,
                              const float* w2, const float* b2, const float* gamma,
                              const float* beta, float* rmean, float* rvar, long long* nbt,
                              float momentum, float eps, int training, void* out,
                              const void* res, float* save, double* ostats, float* ws,
                              size_t ws_elems, int dt, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (dt != ACC_F32 && dt != ACC_BF16) return ACC_EBADARG;
  if (ws_elems < accunet_se_ws_elems(B, HW, C, Cr)) return ACC_EBADARG;
  if (((uintptr_t)ws & 7) || ((uintptr_t)save & 7)) return ACC_EBADARG;
  SeGeom g = se_geom(B, HW, C);
  if (!se_chunk_ok(g, dt)) return ACC_EBADSHAPE;
  int V = (C % 4 == 0) ? 4 : 1;
  dim3 grid(B * g.NCH, ceil_div(C / V, 64));
  double* part = reinterpret_cast<double*>(ws);
  SeMid m{Cr, w1, b1, w2, b2, gamma, beta, rmean, rvar, training ? nbt : nullptr,
          momentum, eps, training, save};
  const bool pro = sc != nullptr;
  with_dt(dt, [&](auto tag) {
    using T = decltype(tag);
    auto go = [&](auto kv, auto kp) {
      constexpr int KV = decltype(kv)::value;
      constexpr bool KP = decltype(kp)::value;
      hipLaunchKernelGGL((se_reduce_kernel<KV, T, KP>), grid, dim3(256), 0, s, (const T*)z, sc, sh,
                         act, g, part);
    };
    using I4 = std::integral_constant<int, 4>;
    using I1 = std::integral_constant<int, 1>;
    if (V == 4) pro ? go(I4{}, std::true_type{}) : go(I4{}, std::false_type{});
    else pro ? go(I1{}, std::true_type{}) : go(I1{}, std::false_type{});
  });
  // S, Q and the gate per sample, then the BN-of-gated statistics per channel
  hipLaunchKernelGGL(se_mid_sample_kernel, dim3(B), dim3(256), (C + Cr) * sizeof(float), s, part,
                     g, m);
  // (the BatchNorm-of-gated step runs in the apply's prologue, se_chan_bn)
  with_dt(dt, [&](auto tag) {
    using T = decltype(tag);
    auto go = [&](auto kv, auto kp, auto kr) {
      hipLaunchKernelGGL((se_apply_kernel<decltype(kv)::value, T, decltype(kp)::value,
                                          decltype(kr)::value>),
                         grid, dim3(256), 0, s, (const T*)z, sc, sh, act, g, m,
                         (const T*)res, (T*)out, ostats, se_rev());
    };
    using I4 = std::integral_constant<int, 4>;
    using I1 = std::integral_constant<int, 1>;
    using BT = std::true_type;
    using BF = std::false_type;
    auto by_res = [&](auto kv, auto kp) { res ? go(kv, kp, BT{}) : go(kv, kp, BF{}); };
    if (V == 4) pro ? by_res(I4{}, BT{}) : by_res(I4{}, BF{});
    else pro ? by_res(I1{}, BT{}) : by_res(I1{}, BF{});
  });
  return hipGetLastError() == hipSuccess ? ACC_OK : ACC_ELAUNCH;
}

// the unfused backward middle step: per-(b,c) sums in scratch (from part) -> BN /
// gate / fc backward, coef (A, Bc, Cc), fc parameter gradients (+ the prologue
// coefficient step when m.pcoef is set)
static void se_bwd_mid(const SeGeom& g, const SeBwdMid& m, const double* part, int nq,
                       hipStream_t s) {
  const int B = g.B, C = g.C, Cr = m.Cr;
  if (nq == 2)
    hipLaunchKernelGGL(se_bwd_chan_sum_kernel<2>, dim3(C), dim3(256), 0, s, part, g, m);
  else
    hipLaunchKernelGGL(se_bwd_chan_sum_kernel<SE_PRO_NQ>, dim3(C), dim3(256), 0, s, part, g, m);
  hipLaunchKernelGGL(se_bwd_sample_kernel, dim3(B), dim3(256), (Cr > 0 ? Cr : 1) * sizeof(double),
                     s, g, m);
  const long nparam = 2L * C * Cr + C + Cr;
  const int npb = ceil_div(nparam, 256);
  const int ncb = m.pcoef ? ceil_div((long)C * SE_LANES, 256) : 0;
  hipLaunchKernelGGL(se_bwd_tail_kernel, dim3(npb + ncb), dim3(256), 0, s, g, m, npb);
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
  SeBwdMid m{Cr, w1, w2, gamma, training, const_cast<float*>(save), scratch, coef,
             dw1, db1, dw2, db2, dgamma, dbeta, nullptr, nullptr, 0, nullptr, nullptr, nullptr,
             nullptr};
  se_bwd_mid(g, m, part, 2, s);
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
  if (!se_chunk_ok(g, dt)) return ACC_EBADSHAPE;
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
  SeBwdMid m{Cr, w1, w2, gamma, training, const_cast<float*>(save), scratch, coef,
             dw1, db1, dw2, db2, dgamma, dbeta, pst, pgamma, ptraining, dpgamma, dpbeta, pcoef,
             dsum};
  with_dt(dt, [&](auto tag) {
    using T = decltype(tag);
    if (V == 4)
      hipLaunchKernelGGL((se_bwd_reduce_pro_kernel<4, T>), grid, dim3(256), 0, s, (const T*)z,
                         (const T*)dout, pst, act, g, alpha, betap, part);
    else
      hipLaunchKernelGGL((se_bwd_reduce_pro_kernel<1, T>), grid, dim3(256), 0, s, (const T*)z,
                         (const T*)dout, pst, act, g, alpha, betap, part);
  });
  se_bwd_mid(g, m, part, SE_PRO_NQ, s);
  double* cpart = nullptr;  // (dz's column sums: computed analytically, se_pro_coef_body)
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
  (void)dscr;
  return hipGetLastError() == hipSuccess ? ACC_OK : ACC_ELAUNCH;
}
