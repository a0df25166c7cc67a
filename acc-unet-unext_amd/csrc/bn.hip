// Training-mode BatchNorm2d (+LeakyReLU) on NHWC fp32 / bf16 activations, split into streaming
// passes whose per-channel statistics are reduced deterministically
// (per-block partials -> fixed-order reduction, fp64 final accumulation).
//
// Reference semantics (torch.nn.BatchNorm2d as used throughout
// ACC_UNet/ACC_UNet.py, e.g. :235-262): normalise with the biased batch
// variance, update running_mean / running_var with momentum 0.1 using the
// UNBIASED variance, eps = 1e-5; eval mode uses the running statistics.
#include <mutex>
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
// reduce_finish: the whole partial-row reduction and its finish in ONE launch
// (it replaces the colreduce stages + finish kernel: 2-4 launches of a few us each
// per BatchNorm). Grid (nchunk, column blocks of 64). Block (k, y) sums rows
// [k*rpc, (k+1)*rpc) of its 64 columns in a fixed order (fp64) into chunk row k;
// the last block of column block y to arrive (ticket counter; the chunk totals are
// handed over with write-through stores and sc1 loads, no fences -- see handoff_last
// in common.h) adds the nchunk chunk rows in index order and runs the finish. The chunking depends on R only, so the result is
// bitwise reproducible. Paired kinds (BatchNorm) map thread column cl < 32 to the
// first moment of channel 32y+cl and cl >= 32 to its second moment (column C+ch).
// The tickets live in a zero-initialised device array; every last arriver resets
// its word, so consecutive launches on a stream (and graph replays) reuse it.
// ---------------------------------------------------------------------------
#define FIN_MAX_CB 16384  // column blocks (ncols <= 262144: dw wgrad of cnv72 has 10 x 4352)
// One ticket array per bank: launches that may run concurrently must not share
// tickets. The bank is a property of the STREAM a reduction is enqueued on: the host
// registers its side streams (accunet_stream_ticket_bank, e.g. the backward's
// weight-gradient stream -> bank 1) and every other stream uses bank 0. Keying by
// stream (not by a "current bank" switch) keeps the choice correct whatever thread
// enqueues the launch; the ticket array itself is per device (a __device__ symbol).
#define FIN_BANKS 2
__device__ unsigned g_fin_tickets[FIN_BANKS * FIN_MAX_CB];
#define FIN_MAX_STREAMS 64
static std::mutex g_bank_mu;
static hipStream_t g_bank_stream[FIN_MAX_STREAMS];
static int g_bank_of[FIN_MAX_STREAMS];
static int g_bank_n = 0;

extern "C" int accunet_stream_ticket_bank(void* stream, int bank) {
  if (bank < 0 || bank >= FIN_BANKS || !stream) return ACC_EBADARG;
  std::lock_guard<std::mutex> lk(g_bank_mu);
  for (int i = 0; i < g_bank_n; ++i)
    if (g_bank_stream[i] == (hipStream_t)stream) {
      g_bank_of[i] = bank;
      return ACC_OK;
    }
  if (g_bank_n == FIN_MAX_STREAMS) return ACC_EBADARG;
  g_bank_stream[g_bank_n] = (hipStream_t)stream;
  g_bank_of[g_bank_n++] = bank;
  return ACC_OK;
}

extern "C" int accunet_stream_ticket_unregister(void* stream) {
  if (!stream) return ACC_EBADARG;
  std::lock_guard<std::mutex> lk(g_bank_mu);
  for (int i = 0; i < g_bank_n; ++i)
    if (g_bank_stream[i] == (hipStream_t)stream) {
      g_bank_stream[i] = g_bank_stream[g_bank_n - 1];
      g_bank_of[i] = g_bank_of[g_bank_n - 1];
      --g_bank_n;
      return ACC_OK;
    }
  return ACC_EBADARG;
}

static int stream_bank(hipStream_t s) {
  if (!s) return 0;
  std::lock_guard<std::mutex> lk(g_bank_mu);
  for (int i = 0; i < g_bank_n; ++i)
    if (g_bank_stream[i] == s) return g_bank_of[i];
  return 0;
}
int acc_stream_bank(hipStream_t s) { return stream_bank(s); }

ACC_DEV void fin_column(const FinishArgs& fa, int col, double tot) {
  switch (fa.kind) {
    case FIN_SUM_F: fa.out_f[col] = (float)tot; break;
    case FIN_SUM_D: fa.out_d[col] = tot; break;
    case FIN_DW:  // [10][C] sums -> dW[c][tap] (torch layout [C][1][3][3]) and db[c]
      if (col < 9 * fa.C) fa.out_f[(col % fa.C) * 9 + col / fa.C] = (float)tot;
      else if (fa.out2) fa.out2[col - 9 * fa.C] = (float)tot;
      break;
    case FIN_HEAD:
      if (col < fa.C) fa.out_f[col] = (float)tot;
      else if (col == fa.C) fa.out2[0] = (float)tot;
      break;
    default: break;
  }
}

// BatchNorm forward finish (training): see bn_finalize_kernel for the eval form
ACC_DEV void fin_bn_fwd(const FinishArgs& fa, int c, double s1, double s2) {
  const int C = fa.ncols;
  const double m = s1 / fa.count;
  double v = s2 / fa.count - m * m;
  if (v < 0.0) v = 0.0;
  const float mean = (float)m, var = (float)v;
  if (fa.rmean) fa.rmean[c] = (1.f - fa.momentum) * fa.rmean[c] + fa.momentum * mean;
  if (fa.rvar) {
    const double unb = fa.count > 1.0 ? v * fa.count / (fa.count - 1.0) : v;
    fa.rvar[c] = (1.f - fa.momentum) * fa.rvar[c] + fa.momentum * (float)unb;
  }
  const float rstd = 1.0f / sqrtf(var + fa.eps);
  const float ga = fa.gamma ? fa.gamma[c] : 1.f;
  const float be = fa.beta ? fa.beta[c] : 0.f;
  const float sc = ga * rstd;
  float* st = fa.out_f;
  st[BN_MEAN * C + c] = mean;
  st[BN_RSTD * C + c] = rstd;
  st[BN_SCALE * C + c] = sc;
  st[BN_SHIFT * C + c] = be - mean * sc;
}

// Bias gradient of the convolution whose output x feeds only a BatchNorm (training or
// eval): sum_p dx with dx = k1*g + k2*(x - mean) + k3 is k1*sum g + count*k3 exactly,
// save the k2 * sum (x - mean) term, which vanishes but for the rounding of the fp32
// mean (the batch mean in training; eval has k2 = k3 = 0). ATen gets the same value,
// zero up to rounding in training, as an fp32 column sum of dx; the column-sum pass and
// its reduction are gone (ACC_UNet.py conv biases before every BatchNorm).
ACC_DEV float bn_dsum(float k1, float k3, double s1, double count) {
  return (float)((double)k1 * s1 + count * (double)k3);
}

// BatchNorm backward finish: (sum g, sum g*xhat | g*(x-mean)) -> dgamma, dbeta, coef
ACC_DEV void fin_bn_bwd(const FinishArgs& fa, int c, double s1, double s2) {
  const int C = fa.ncols;
  const float* st = fa.st;
  if (fa.xc_form) s2 *= (double)st[BN_RSTD * C + c];
  if (fa.out2) fa.out2[c] = (float)s2;
  if (fa.out3) fa.out3[c] = (float)s1;
  const float ga = fa.gamma ? fa.gamma[c] : 1.f;
  const float rstd = st[BN_RSTD * C + c];
  const float k1 = ga * rstd;
  float k2 = 0.f, k3 = 0.f;
  if (fa.training) {
    // dx = k1*(g - mean(g) - xhat*mean(g*xhat)) = k1*g + k2*(x - mean) + k3
    const float mg = (float)(s1 / fa.count), mgx = (float)(s2 / fa.count);
    k2 = -k1 * rstd * mgx;
    k3 = -k1 * mg;
  }
  fa.out_f[c] = k1;
  fa.out_f[C + c] = k2;
  fa.out_f[2 * C + c] = k3;
  // sum_p dx = k1 sum g + k2 sum (x - mean) + count k3, and sum (x - mean) = 0 up to the
  // rounding of the stored mean: the bias gradient of the convolution feeding this
  // BatchNorm (bn_dsum) without a column-sum pass over dx
  if (fa.out4) fa.out4[c] = bn_dsum(k1, k3, s1, fa.count);
}

// 256 threads = FIN_COLS columns x FIN_GROUPS row groups: with 8 loads in flight per
// thread a block covers FIN_GROUPS*8 = 128 rows per memory round trip, which is
// exactly one chunk, and the last arriver's pass over the chunk rows is one more.
#define FIN_COLS 16
#define FIN_GROUPS 16
template <typename TP>
__global__ void __launch_bounds__(256)
reduce_finish_kernel(const TP* __restrict__ part, int R, int stride, int rpc, double* chunks,
                     FinishArgs fa) {
  __shared__ double red[FIN_GROUPS][FIN_COLS];
  const int cl = threadIdx.x % FIN_COLS, g = threadIdx.x / FIN_COLS;
  const bool paired = fa.kind == FIN_BN_FWD || fa.kind == FIN_BN_BWD;
  constexpr int HC = FIN_COLS / 2;
  int col;
  bool valid;
  if (paired) {
    const int ch = blockIdx.y * HC + (cl % HC);
    valid = ch < fa.ncols;
    col = cl < HC ? ch : fa.ncols + ch;
  } else {
    col = blockIdx.y * FIN_COLS + cl;
    valid = col < fa.ncols;
  }
  auto combine = [&](double v) {  // fixed-order sum over the row groups
    red[g][cl] = v;
    __syncthreads();
    double t = 0.0;
#pragma unroll
    for (int k = 0; k < FIN_GROUPS; ++k) t += red[k][cl];
    __syncthreads();
    return t;
  };
  const int nchunk = gridDim.x;
  const int r0 = blockIdx.x * rpc, r1 = min(R, r0 + rpc);
  double s[1] = {0.0};
  if (valid)
    ordered_strided_sum<8>(s, r0 + g, r1, FIN_GROUPS, [&](int r, double (&v)[1]) {
      v[0] = (double)part[(long)r * stride + col];
    });
  double tot = combine(s[0]);
  if (nchunk > 1) {
    // hand-off without fences: the chunk totals are stored write-through (agent-scope
    // atomic store = sc1) and drained before the ticket, and the last arriver reads
    // them with sc1 loads (L1 bypass), so neither an L2 write-back (release) nor an L1
    // invalidate (acquire) is needed (MI355X guide section 6, Guideline 16, R1/R2)
    if (g == 0 && valid) st_wt(chunks + (long)blockIdx.x * stride + col, tot);
    if (!handoff_last(g_fin_tickets + fa.bank * FIN_MAX_CB + blockIdx.y, nchunk)) return;
    double c1[1] = {0.0};
    if (valid)
      ordered_strided_sum<8>(c1, g, nchunk, FIN_GROUPS, [&](int k, double (&v)[1]) {
        v[0] = ld_wt(chunks + (long)k * stride + col);
      });
    tot = combine(c1[0]);
  }
  if (paired) {
    if (g == 0) red[0][cl] = tot;
    __syncthreads();
    if (g == 0 && cl < HC && valid) {
      const int ch = blockIdx.y * HC + cl;
      if (fa.kind == FIN_BN_FWD) {
        fin_bn_fwd(fa, ch, red[0][cl], red[0][cl + HC]);
        if (fa.nbt && ch == 0) *fa.nbt += 1;  // num_batches_tracked
      } else {
        fin_bn_bwd(fa, ch, red[0][cl], red[0][cl + HC]);
      }
    }
  } else if (g == 0 && valid) {
    fin_column(fa, col, tot);
  }
}

static int fin_rows_per_chunk(int) { return FIN_GROUPS * 8; }

size_t reduce_finish_ws(int R, int stride) {
  const int nchunk = ceil_div(R, fin_rows_per_chunk(R));
  return nchunk > 1 ? (size_t)nchunk * stride : 0;
}

int reduce_finish(const void* part, bool part_f64, int R, int stride, double* chunks,
                  const FinishArgs& fa_in, hipStream_t s) {
  FinishArgs fa = fa_in;
  fa.bank = stream_bank(s);
  const bool paired = fa.kind == FIN_BN_FWD || fa.kind == FIN_BN_BWD;
  const int rpc = fin_rows_per_chunk(R);
  const int nchunk = max(1, ceil_div(R, rpc));
  const int ncb = paired ? ceil_div(fa.ncols, FIN_COLS / 2) : ceil_div(fa.ncols, FIN_COLS);
  // (float workspaces may hand over a 4-byte aligned scratch: the partials workspace
  // sizes keep two spare rows, so rounding up to 8 bytes stays inside it)
  chunks = reinterpret_cast<double*>(((uintptr_t)chunks + 7) & ~(uintptr_t)7);
  if (ncb > FIN_MAX_CB || (nchunk > 1 && !chunks)) return ACC_EBADARG;
  const int wd = paired ? 2 * fa.ncols : fa.ncols;
  if (wd > stride) return ACC_EBADARG;
  if (part_f64)
    hipLaunchKernelGGL(reduce_finish_kernel<double>, dim3(nchunk, ncb), dim3(256), 0, s,
                       (const double*)part, R, stride, rpc, chunks, fa);
  else
    hipLaunchKernelGGL(reduce_finish_kernel<float>, dim3(nchunk, ncb), dim3(256), 0, s,
                       (const float*)part, R, stride, rpc, chunks, fa);
  return hipGetLastError() == hipSuccess ? ACC_OK : ACC_ELAUNCH;
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
  if (training) {
    FinishArgs fa{};
    fa.kind = FIN_BN_FWD;
    fa.ncols = C;
    fa.count = count;
    fa.gamma = gamma;
    fa.beta = beta;
    fa.rmean = rmean;
    fa.rvar = rvar;
    fa.nbt = nbt;
    fa.momentum = momentum;
    fa.eps = eps;
    fa.out_f = st;
    return reduce_finish(part, true, R, 2 * C, ws, fa, s);
  }
  hipLaunchKernelGGL(bn_finalize_kernel, dim3(ceil_div(C, 64)), dim3(256), 0, s, part, 0, C,
                     count, gamma, beta, rmean, rvar, momentum, eps, 0, st, nullptr);
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
    auto row = [&](bool ok, float (&v)[V], const float (&q)[V]) {
#pragma unroll
      for (int j = 0; j < V; ++j) {
        v[j] = apply_act(v[j] * s[j] + h[j], act);
        if (res) v[j] += q[j];
        if (y) v[j] = rnd<T>(v[j]);  // statistics of the stored value
        const double e = ok ? (double)v[j] : 0.0;
        a[j] += e;
        b[j] += e * e;
      }
    };
    if constexpr (V == 4) {
      // branch-free streaming (chan.h quad_rows*): rows past the chunk are masked
      const long nr = r1 > r0 ? r1 - r0 : 0;
      const __amdgpu_buffer_rsrc_t ry =
          acc_rsrc(y ? y + r0 * C : x, y ? (unsigned)(nr * C * sizeof(T)) : 0u);
      auto put = [&](const float (&v)[V], unsigned off) {
        bufq_st<ACC_STREAM_STORE_AUX>(ry, off, make_float4(v[0], v[1 % V], v[2 % V], v[3 % V]), (T*)nullptr);
      };
      if (res) {
        quad_rows2<4>(x + r0 * C, res + r0 * C, nr, t.rg, t.RG, C, t.c0,
                      [&](bool ok, float4 x4, float4 q4, unsigned off) {
                        float v[V] = {x4.x, x4.y, x4.z, x4.w};
                        const float q[V] = {q4.x, q4.y, q4.z, q4.w};
                        row(ok, v, q);
                        put(v, off);
                      });
      } else {
        quad_rows1<8>(x + r0 * C, nr, t.rg, t.RG, C, t.c0, [&](bool ok, float4 x4, unsigned off) {
          float v[V] = {x4.x, x4.y, x4.z, x4.w};
          const float q[V] = {0.f, 0.f, 0.f, 0.f};
          row(ok, v, q);
          put(v, off);
        });
      }
    } else {
      for (long r = r0 + t.rg; r < r1; r += t.RG) {
        float v[V], q[V];
        ldv<V>(x + r * C + t.c0, v);
        if (res) ldv<V>(res + r * C + t.c0, q);
        row(true, v, q);
        if (y) stv<V>(y + r * C + t.c0, v);  // y == nullptr: statistics only (accunet_colsum)
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
    auto row = [&](bool ok, const float (&xv)[V], const float (&dv)[V]) {
#pragma unroll
      for (int j = 0; j < V; ++j) {
        float g = ok ? dv[j] : 0.f;
        if (act == ACT_LRELU) g *= lrelu_d(xv[j] * s[j] + h[j]);
        a[j] += g;
        b[j] += (double)g * ((double)xv[j] - mu[j]) * rs[j];
      }
    };
    if constexpr (V == 4) {
      quad_rows2<4>(x + r0 * C, dy + r0 * C, r1 > r0 ? r1 - r0 : 0, t.rg, t.RG, C, t.c0,
                    [&](bool ok, float4 x4, float4 d4, unsigned) {
                      const float xv[V] = {x4.x, x4.y, x4.z, x4.w};
                      const float dv[V] = {d4.x, d4.y, d4.z, d4.w};
                      row(ok, xv, dv);
                    });
    } else {
      for (long r = r0 + t.rg; r < r1; r += t.RG) {
        float xv[V], dv[V];
        ldv<V>(x + r * C + t.c0, xv);
        ldv<V>(dy + r * C + t.c0, dv);
        row(true, xv, dv);
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

template <int V, int U, typename T>
__global__ void __launch_bounds__(256)
bn_bwd_apply_kernel(const T* __restrict__ x, const T* __restrict__ dy,
                    const float* __restrict__ st, const float* __restrict__ coef, int act,
                    long P, int C, T* __restrict__ dx, int accumulate) {
  ChanTile t = chan_tile<V>(C);
  long rows_per = (P + gridDim.x - 1) / gridDim.x;
  long r0 = blockIdx.x * rows_per, r1 = min(P, r0 + rows_per);
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
    // d = k1*g + k2*(x - mean) + k3; o (accumulate) = the value already in dx
    auto row = [&](bool ok, const float (&xv)[V], const float (&dv)[V], float (&o)[V]) {
#pragma unroll
      for (int j = 0; j < V; ++j) {
        float g = dv[j];
        if (act == ACT_LRELU) g *= lrelu_d(xv[j] * s[j] + h[j]);
        float d = k1[j] * g + k2[j] * (xv[j] - mu[j]) + k3[j];
        o[j] = accumulate ? rnd<T>(o[j] + d) : rnd<T>(d);
      }
    };
    auto plain = [&]() {
      for (long r = r0 + t.rg; r < r1; r += t.RG) {
        float xv[V], dv[V], o[V];
        ldv<V>(x + r * C + t.c0, xv);
        ldv<V>(dy + r * C + t.c0, dv);
        if (accumulate) ldv<V>(dx + r * C + t.c0, o);
        row(true, xv, dv, o);
        stv<V>(dx + r * C + t.c0, o);
      }
    };
    if constexpr (V == 4) {
      if (!accumulate) {
        const long nr = r1 > r0 ? r1 - r0 : 0;
        const __amdgpu_buffer_rsrc_t rd = acc_rsrc(dx + r0 * C, (unsigned)(nr * C * sizeof(T)));
        quad_rows2<U>(x + r0 * C, dy + r0 * C, nr, t.rg, t.RG, C, t.c0,
                      [&](bool ok, float4 x4, float4 d4, unsigned off) {
                        const float xv[V] = {x4.x, x4.y, x4.z, x4.w};
                        const float dv[V] = {d4.x, d4.y, d4.z, d4.w};
                        float o[V];
                        row(ok, xv, dv, o);
                        bufq_st<ACC_STREAM_STORE_AUX>(rd, off, make_float4(o[0], o[1], o[2], o[3]), (T*)nullptr);
                      });
      } else {
        plain();
      }
    } else {
      plain();
    }
  }
}

// rows of loads a thread of the BatchNorm-backward apply keeps in flight (per input):
// ACCUNET_BN_APPLY_U=8 (A/B knob; default 4)
static int bn_apply_u() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("ACCUNET_BN_APPLY_U");
    v = (e && atoi(e) == 8) ? 8 : 4;
  }
  return v;
}

extern "C" size_t accunet_bn_bwd_ws_elems(long P, int C) {
  int nb = stream_rowblocks(P, C);
  return (size_t)nb * 2 * C * 2 + accunet_partials_ws_elems(nb, 2 * C) * 2 + 3 * (size_t)C;
}

// BatchNorm backward finish arguments (see fin_bn_bwd)
static FinishArgs bn_bwd_fin(int C, long P, const float* st, const float* gamma, int training,
                             float* dgamma, float* dbeta, float* coef, int xc_form, float* dsum) {
  FinishArgs fa{};
  fa.out4 = dsum;
  fa.kind = FIN_BN_BWD;
  fa.ncols = C;
  fa.count = (double)P;
  fa.st = st;
  fa.gamma = gamma;
  fa.training = training;
  fa.xc_form = xc_form;
  fa.out_f = coef;
  fa.out2 = dgamma;
  fa.out3 = dbeta;
  return fa;
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
  int rc = reduce_finish(part, true, nb, 2 * C, scratch,
                         bn_bwd_fin(C, P, st, gamma, training, dgamma, dbeta, coef, 0, dsum), s);
  if (rc != ACC_OK) return rc;
  const dim3 agrid = grid;
  with_dt(dt, [&](auto tag) {
    using T = decltype(tag);
    if (V == 4 && bn_apply_u() == 8)
      hipLaunchKernelGGL((bn_bwd_apply_kernel<4, 8, T>), agrid, dim3(256), 0, s, (const T*)x,
                         (const T*)dy, st, coef, act, P, C, (T*)dx, accumulate);
    else if (V == 4)
      hipLaunchKernelGGL((bn_bwd_apply_kernel<4, 4, T>), agrid, dim3(256), 0, s, (const T*)x,
                         (const T*)dy, st, coef, act, P, C, (T*)dx, accumulate);
    else
      hipLaunchKernelGGL((bn_bwd_apply_kernel<1, 4, T>), agrid, dim3(256), 0, s, (const T*)x,
                         (const T*)dy, st, coef, act, P, C, (T*)dx, accumulate);
  });
  return hipGetLastError() == hipSuccess ? ACC_OK : ACC_ELAUNCH;
}

// BatchNorm backward whose reduce pass ran in the producer of dy (GEMM / depthwise
// data-gradient epilogues): part = [R][2][C] (sum g, sum g*(x - mean)).
// coef [3][C] floats, padded to an even count so what follows stays 8-byte aligned
static size_t bn_coef_floats(int C) { return ((3 * (size_t)C + 1) / 2) * 2; }

// ws (floats): fp64 reduce scratch (R rows) | coef [3][C] (even pad)
static size_t bn_bwd_part_ws(long P, int R, int C) {
  (void)P;
  return accunet_partials_ws_elems(R, 2 * C) * 2 + bn_coef_floats(C);
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
  int rc = reduce_finish(part, true, R, 2 * C, scratch,
                         bn_bwd_fin(C, P, st, gamma, training, dgamma, dbeta, coef, 1, dsum), s);
  if (rc != ACC_OK) return rc;
  const dim3 agrid = grid;
  with_dt(dt, [&](auto tag) {
    using T = decltype(tag);
    if (V == 4 && bn_apply_u() == 8)
      hipLaunchKernelGGL((bn_bwd_apply_kernel<4, 8, T>), agrid, dim3(256), 0, s, (const T*)x,
                         (const T*)dy, st, coef, act, P, C, (T*)dx, 0);
    else if (V == 4)
      hipLaunchKernelGGL((bn_bwd_apply_kernel<4, 4, T>), agrid, dim3(256), 0, s, (const T*)x,
                         (const T*)dy, st, coef, act, P, C, (T*)dx, 0);
    else
      hipLaunchKernelGGL((bn_bwd_apply_kernel<1, 4, T>), agrid, dim3(256), 0, s, (const T*)x,
                         (const T*)dy, st, coef, act, P, C, (T*)dx, 0);
  });
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
  FinishArgs fa{};
  fa.kind = FIN_SUM_F;
  fa.ncols = C;
  fa.out_f = out;
  return reduce_finish(part, true, nb, 2 * C, scratch, fa, s);
}

// Reduce a partial-stats block [R][2][C] to totals [2][C] (fp64).
extern "C" int accunet_reduce_stats(const double* part, int R, int C, double* out2C, double* ws,
                                    void* stream_) {
  hipStream_t s = (hipStream_t)stream_;
  FinishArgs fa{};
  fa.kind = FIN_SUM_D;
  fa.ncols = 2 * C;
  fa.out_d = out2C;
  return reduce_finish(part, true, R, 2 * C, ws, fa, s);
}
