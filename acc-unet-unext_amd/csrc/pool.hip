// Pooling / resampling / layout kernels on NHWC fp32 / bf16 activations.
//
//  - HANC neighbourhood pyramid (HANCLayer, ACC_UNet/ACC_UNet.py:86-106): from the
//    pending-BN input a = act(x*scale+shift) produce at 1/2 resolution
//    P2 = [avg2(a) | max2(a)] and at 1/4 resolution P4 = [avg4(a) | max4(a)]
//    (2C channels each) in ONE read of x. Backward routes avg gradients uniformly and
//    max gradients to the first maximal element of the window (row-major scan,
//    torch CPU max_pool2d tie rule), recomputing the argmax from x.
//  - MaxPool2d(2) between encoder levels (ACC_UNet.py:552,608-623), AvgPool2d(2)
//    chain of MLFC (:361), nearest-upsample backward (block sums), channel concat /
//    slice copies (decoder torch.cat, :639-648), ConvTranspose2d(2,2) pixel
//    shuffle (:578-590), and generic 4-D permutes for weight / boundary layouts.
#include "common.h"
#include "kernels.h"
#include "chan.h"
#include <type_traits>

// ---------------------------------------------------------------------------
// pyramid forward: one thread per (low-res 4x4 or 2x2 cell, V consecutive channels);
// V = 4 moves channel quads (16-byte loads/stores, 4-byte mask stores). The
// per-element arithmetic is the same for every V.
// ---------------------------------------------------------------------------
template <int V, typename T, int CS, bool PRO>
__global__ void __launch_bounds__(256)
hanc_pyramid_fwd_kernel(const T* __restrict__ x, const float* __restrict__ sc,
                        const float* __restrict__ sh, int act, int B, int H, int W, int C,
                        T* __restrict__ p2, T* __restrict__ p4,
                        unsigned char* __restrict__ mk2, unsigned char* __restrict__ mk4) {
  // CS = 4 (k == 3): cell = 4x4 (one P4 pixel, four P2 pixels); CS = 2 (k == 2): one P2
  // pixel. The CS*CS quads of a cell are loaded raw and unconditionally before any is
  // used (compile-time cell size, prologue flag as a template argument), so they are
  // in flight together instead of one dependent round trip each.
  typedef typename QuadRaw<T>::type RawQ;
  const int Hc = H / CS, Wc = W / CS, CV = C / V;
  const long total = (long)B * Hc * Wc * CV;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % CV) * V;
    const long cell = i / CV;
    const int wc = (int)(cell % Wc);
    const long t = cell / Wc;
    const int hc = (int)(t % Hc);
    const int b = (int)(t / Hc);
    float v[CS][CS][V];
    const T* src = x + (((long)b * H + hc * CS) * W + wc * CS) * C + c;
    if (V == 4) {
      RawQ r[CS][CS];
#pragma unroll
      for (int dy = 0; dy < CS; ++dy)
#pragma unroll
        for (int dx = 0; dx < CS; ++dx) r[dy][dx] = ldq_raw(src + ((long)dy * W + dx) * C, false);
      float4 s4 = make_float4(1.f, 1.f, 1.f, 1.f), h4 = make_float4(0.f, 0.f, 0.f, 0.f);
      if (PRO) {
        s4 = ld4(sc + c);
        h4 = ld4(sh + c);
      }
      const float s[4] = {s4.x, s4.y, s4.z, s4.w}, h[4] = {h4.x, h4.y, h4.z, h4.w};
#pragma unroll
      for (int dy = 0; dy < CS; ++dy)
#pragma unroll
        for (int dx = 0; dx < CS; ++dx) {
          const float4 q4 = q2f(r[dy][dx]);
          const float q[4] = {q4.x, q4.y, q4.z, q4.w};
#pragma unroll
          for (int j = 0; j < V; ++j)
            v[dy][dx][j] = PRO ? apply_act(q[j] * s[j % 4] + h[j % 4], act) : q[j % 4];
        }
    } else {
#pragma unroll
      for (int dy = 0; dy < CS; ++dy)
#pragma unroll
        for (int dx = 0; dx < CS; ++dx) {
          float q[V];
          ldv<V>(src + ((long)dy * W + dx) * C, q);
#pragma unroll
          for (int j = 0; j < V; ++j)
            v[dy][dx][j] = PRO ? apply_act(q[j] * sc[c + j] + sh[c + j], act) : q[j];
        }
    }
    const int H2 = H / 2, W2 = W / 2;
    constexpr int n2 = CS / 2;
#pragma unroll
    for (int qy = 0; qy < n2; ++qy)
#pragma unroll
      for (int qx = 0; qx < n2; ++qx) {
        float sum[V], mx[V];
        unsigned char code[V];
#pragma unroll
        for (int j = 0; j < V; ++j) {
          float a0 = v[2 * qy][2 * qx][j], a1 = v[2 * qy][2 * qx + 1][j];
          float a2 = v[2 * qy + 1][2 * qx][j], a3 = v[2 * qy + 1][2 * qx + 1][j];
          sum[j] = (((a0 + a1) + a2) + a3) * 0.25f;  // torch CPU avg_pool2d summation order
          mx[j] = fmaxf(fmaxf(a0, a1), fmaxf(a2, a3));
          // first maximum in window order (0,0) (0,1) (1,0) (1,1)
          code[j] = a0 == mx[j] ? 0 : a1 == mx[j] ? 1 : a2 == mx[j] ? 2 : a3 == mx[j] ? 3 : 255;
        }
        const long q2 = ((long)b * H2 + hc * n2 + qy) * W2 + wc * n2 + qx;
        const long o = q2 * (2 * C);
        stv<V>(p2 + o + c, sum);
        stv<V>(p2 + o + C + c, mx);
        if (mk2) {
          if (V == 4) {
            uchar4 cv = make_uchar4(code[0], code[V > 1 ? 1 : 0], code[V > 2 ? 2 : 0],
                                    code[V > 3 ? 3 : 0]);
            *reinterpret_cast<uchar4*>(mk2 + q2 * C + c) = cv;
          } else {
#pragma unroll
            for (int j = 0; j < V; ++j) mk2[q2 * C + c + j] = code[j];
          }
        }
      }
    if (CS == 4) {
      float s4[V], m4[V];
      unsigned char code[V];
#pragma unroll
      for (int j = 0; j < V; ++j) {
        float a = 0.f, m = -INFINITY;
#pragma unroll
        for (int dy = 0; dy < CS; ++dy)
#pragma unroll
          for (int dx = 0; dx < CS; ++dx) {
            a += v[dy][dx][j];
            m = fmaxf(m, v[dy][dx][j]);
          }
        s4[j] = a * (1.f / 16.f);
        m4[j] = m;
        unsigned char cd = 255;
#pragma unroll
        for (int e = CS * CS - 1; e >= 0; --e)
          if (v[e / CS][e % CS][j] == m) cd = (unsigned char)e;
        code[j] = cd;
      }
      const long q4 = ((long)b * Hc + hc) * Wc + wc;
      const long o = q4 * (2 * C);
      stv<V>(p4 + o + c, s4);
      stv<V>(p4 + o + C + c, m4);
      if (mk4) {
        if (V == 4) {
          uchar4 cv = make_uchar4(code[0], code[V > 1 ? 1 : 0], code[V > 2 ? 2 : 0],
                                  code[V > 3 ? 3 : 0]);
          *reinterpret_cast<uchar4*>(mk4 + q4 * C + c) = cv;
        } else {
#pragma unroll
          for (int j = 0; j < V; ++j) mk4[q4 * C + c + j] = code[j];
        }
      }
    }
  }
}

// pyramid backward: da (+)= spread(dP2) + spread(dP4); accumulate into da
template <typename T>
__global__ void __launch_bounds__(256)
hanc_pyramid_bwd_kernel(const T* __restrict__ x, const float* __restrict__ sc,
                        const float* __restrict__ sh, int act, int B, int H, int W, int C, int k,
                        const T* __restrict__ p2, const T* __restrict__ p4,
                        const T* __restrict__ dp2, const T* __restrict__ dp4,
                        T* __restrict__ da) {
  const int cs = (k == 3) ? 4 : 2;
  const int Hc = H / cs, Wc = W / cs;
  long total = (long)B * Hc * Wc * C;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    int c = (int)(i % C);
    long cell = i / C;
    int wc = (int)(cell % Wc);
    long t = cell / Wc;
    int hc = (int)(t % Hc);
    int b = (int)(t / Hc);
    float s = sc ? sc[c] : 1.f, h = sh ? sh[c] : 0.f;
    const bool pro = sc != nullptr;
    float v[4][4], g[4][4];
#pragma unroll
    for (int dy = 0; dy < 4; ++dy)
#pragma unroll
      for (int dx = 0; dx < 4; ++dx) {
        g[dy][dx] = 0.f;
        if (dy < cs && dx < cs) {
          float q = ld1(x + (((long)b * H + hc * cs + dy) * W + wc * cs + dx) * C + c);
          v[dy][dx] = pro ? apply_act(q * s + h, act) : q;
        }
      }
    const int H2 = H / 2, W2 = W / 2;
    const int n2 = cs / 2;
    for (int qy = 0; qy < n2; ++qy)
      for (int qx = 0; qx < n2; ++qx) {
        long o = (((long)b * H2 + hc * n2 + qy) * W2 + wc * n2 + qx) * (2 * C);
        float gav = ld1(dp2 + o + c) * 0.25f;
        float gmx = ld1(dp2 + o + C + c);
        float mx = ld1(p2 + o + C + c);
        bool done = false;
        for (int dy = 0; dy < 2; ++dy)
          for (int dx = 0; dx < 2; ++dx) {
            int yy = 2 * qy + dy, xx = 2 * qx + dx;
            g[yy][xx] += gav;
            if (!done && v[yy][xx] == mx) {
              g[yy][xx] += gmx;
              done = true;
            }
          }
      }
    if (k == 3) {
      long o = (((long)b * Hc + hc) * Wc + wc) * (2 * C);
      float gav = ld1(dp4 + o + c) * (1.f / 16.f);
      float gmx = ld1(dp4 + o + C + c);
      float mx = ld1(p4 + o + C + c);
      bool done = false;
#pragma unroll
      for (int dy = 0; dy < 4; ++dy)
#pragma unroll
        for (int dx = 0; dx < 4; ++dx) {
          g[dy][dx] += gav;
          if (!done && v[dy][dx] == mx) {
            g[dy][dx] += gmx;
            done = true;
          }
        }
    }
#pragma unroll
    for (int dy = 0; dy < 4; ++dy)
#pragma unroll
      for (int dx = 0; dx < 4; ++dx)
        if (dy < cs && dx < cs) {
          T* d = da + (((long)b * H + hc * cs + dy) * W + wc * cs + dx) * C + c;
          st1(d, ld1(d) + g[dy][dx]);
        }
  }
}

static int grid_for(long total) {
  long b = (total + 255) / 256;
  if (b > 8192) b = 8192;
  if (b < 1) b = 1;
  return (int)b;
}

extern "C" int accunet_hanc_pyramid_fwd(const void* x, const float* sc, const float* sh, int act,
                                        int B, int H, int W, int C, int k, void* p2, void* p4,
                                        unsigned char* mk2, unsigned char* mk4, int dt,
                                        void* stream) {
  if (k < 2 || k > 3) return ACC_EBADARG;
  int cs = (k == 3) ? 4 : 2;
  if (H % cs || W % cs) return ACC_EBADSHAPE;
  long total = (long)B * (H / cs) * (W / cs) * C;
  // quads need aligned rows (16 B fp32 / 8 B bf16): C % 4 == 0 and aligned base pointers
  const uintptr_t al = dt == ACC_BF16 ? 7 : 15;
  const bool q4 = C % 4 == 0 && !((uintptr_t)x & al) && !((uintptr_t)p2 & al) &&
                  (k != 3 || !((uintptr_t)p4 & al)) && !((uintptr_t)mk2 & 3) &&
                  (k != 3 || !((uintptr_t)mk4 & 3));
  if (with_dt(dt, [&](auto tag) {
        using T = decltype(tag);
        auto go = [&](auto vc, auto csc, auto proc) {
          constexpr int KV = decltype(vc)::value, KCS = decltype(csc)::value;
          constexpr bool KP = decltype(proc)::value;
          hipLaunchKernelGGL((hanc_pyramid_fwd_kernel<KV, T, KCS, KP>),
                             dim3(grid_for(total / KV)), dim3(256), 0, (hipStream_t)stream,
                             (const T*)x, sc, sh, act, B, H, W, C, (T*)p2, (T*)p4, mk2,
                             k == 3 ? mk4 : nullptr);
        };
        auto by_pro = [&](auto vc, auto csc) {
          if (sc) go(vc, csc, std::true_type{});
          else go(vc, csc, std::false_type{});
        };
        using I4 = std::integral_constant<int, 4>;
        using I2 = std::integral_constant<int, 2>;
        using I1 = std::integral_constant<int, 1>;
        if (q4) k == 3 ? by_pro(I4{}, I4{}) : by_pro(I4{}, I2{});
        else k == 3 ? by_pro(I1{}, I4{}) : by_pro(I1{}, I2{});
      }))
    return ACC_EBADARG;
  return hipGetLastError() == hipSuccess ? ACC_OK : ACC_ELAUNCH;
}

extern "C" int accunet_hanc_pyramid_bwd(const void* x, const float* sc, const float* sh, int act,
                                        int B, int H, int W, int C, int k, const void* p2,
                                        const void* p4, const void* dp2, const void* dp4,
                                        void* da, int dt, void* stream) {
  if (k < 2 || k > 3) return ACC_EBADARG;
  int cs = (k == 3) ? 4 : 2;
  long total = (long)B * (H / cs) * (W / cs) * C;
  if (with_dt(dt, [&](auto tag) {
        using T = decltype(tag);
        hipLaunchKernelGGL((hanc_pyramid_bwd_kernel<T>), dim3(grid_for(total)), dim3(256), 0,
                           (hipStream_t)stream, (const T*)x, sc, sh, act, B, H, W, C, k,
                           (const T*)p2, (const T*)p4, (const T*)dp2, (const T*)dp4, (T*)da);
      }))
    return ACC_EBADARG;
  return hipGetLastError() == hipSuccess ? ACC_OK : ACC_ELAUNCH;
}

// ---------------------------------------------------------------------------
// 2x2 pooling (stride 2): mode 0 = max, 1 = avg. Backward recomputes argmax.
// ---------------------------------------------------------------------------
template <typename T>
__global__ void __launch_bounds__(256)
pool2_fwd_kernel(const T* __restrict__ x, T* __restrict__ y, int B, int H, int W, int C,
                 int mode) {
  const int Ho = H / 2, Wo = W / 2;
  long total = (long)B * Ho * Wo * C;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    int c = (int)(i % C);
    long pix = i / C;
    int wo = (int)(pix % Wo);
    long t = pix / Wo;
    int ho = (int)(t % Ho);
    int b = (int)(t / Ho);
    const T* p = x + (((long)b * H + 2 * ho) * W + 2 * wo) * C + c;
    float a0 = ld1(p), a1 = ld1(p + C), a2 = ld1(p + (long)W * C), a3 = ld1(p + (long)W * C + C);
    st1(y + i, mode == 0 ? fmaxf(fmaxf(a0, a1), fmaxf(a2, a3)) : (((a0 + a1) + a2) + a3) * 0.25f);
  }
}

template <typename T>
__global__ void __launch_bounds__(256)
pool2_bwd_kernel(const T* __restrict__ x, const T* __restrict__ y,
                 const T* __restrict__ dy, T* __restrict__ dx, int B, int H, int W, int C,
                 int mode, int accumulate) {
  const int Ho = H / 2, Wo = W / 2;
  long total = (long)B * Ho * Wo * C;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    int c = (int)(i % C);
    long pix = i / C;
    int wo = (int)(pix % Wo);
    long t = pix / Wo;
    int ho = (int)(t % Ho);
    int b = (int)(t / Ho);
    long base = (((long)b * H + 2 * ho) * W + 2 * wo) * C + c;
    long off[4] = {base, base + C, base + (long)W * C, base + (long)W * C + C};
    float g = ld1(dy + i);
    float gv[4];
    if (mode == 0) {
      float m = ld1(y + i);
      bool done = false;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        gv[j] = 0.f;
        if (!done && ld1(x + off[j]) == m) {
          gv[j] = g;
          done = true;
        }
      }
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) gv[j] = 0.25f * g;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) st1(dx + off[j], accumulate ? ld1(dx + off[j]) + gv[j] : gv[j]);
  }
}

extern "C" int accunet_pool2_fwd(const void* x, void* y, int B, int H, int W, int C, int mode,
                                 int dt, void* stream) {
  if (H % 2 || W % 2) return ACC_EBADSHAPE;
  long total = (long)B * (H / 2) * (W / 2) * C;
  if (with_dt(dt, [&](auto tag) {
        using T = decltype(tag);
        hipLaunchKernelGGL((pool2_fwd_kernel<T>), dim3(grid_for(total)), dim3(256), 0,
                           (hipStream_t)stream, (const T*)x, (T*)y, B, H, W, C, mode);
      }))
    return ACC_EBADARG;
  return hipGetLastError() == hipSuccess ? ACC_OK : ACC_ELAUNCH;
}

extern "C" int accunet_pool2_bwd(const void* x, const void* y, const void* dy, void* dx, int B,
                                 int H, int W, int C, int mode, int accumulate, int dt,
                                 void* stream) {
  long total = (long)B * (H / 2) * (W / 2) * C;
  if (with_dt(dt, [&](auto tag) {
        using T = decltype(tag);
        hipLaunchKernelGGL((pool2_bwd_kernel<T>), dim3(grid_for(total)), dim3(256), 0,
                           (hipStream_t)stream, (const T*)x, (const T*)y, (const T*)dy, (T*)dx, B, H,
                           W, C, mode, accumulate);
      }))
    return ACC_EBADARG;
  return hipGetLastError() == hipSuccess ? ACC_OK : ACC_ELAUNCH;
}

// ---------------------------------------------------------------------------
// Nearest-upsample backward: out[b,hs,ws,c] (+)= sum over the f x f block of
// in[b, hs*f+dy, ws*f+dx, in_off + c] (in has ld_in channels per pixel).
// ---------------------------------------------------------------------------
template <int F, typename T>  // F > 0: compile-time factor (the f*f loads unrolled); 0: runtime f
__global__ void __launch_bounds__(256)
blocksum_kernel(const T* __restrict__ in, int ld_in, int in_off, T* __restrict__ out,
                int ld_out, int B, int H, int W, int C, int f_rt, int accumulate) {
  const int f = F > 0 ? F : f_rt;
  const int Hs = H / f, Ws = W / f;
  long total = (long)B * Hs * Ws * C;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    int c = (int)(i % C);
    long pix = i / C;
    int ws = (int)(pix % Ws);
    long t = pix / Ws;
    int hs = (int)(t % Hs);
    int b = (int)(t / Hs);
    const T* src = in + (((long)b * H + hs * f) * W + ws * f) * ld_in + in_off + c;
    float s = 0.f;
    if (F > 0) {
      float v[F > 0 ? F * F : 1];
#pragma unroll
      for (int dy = 0; dy < F; ++dy)
#pragma unroll
        for (int dx = 0; dx < F; ++dx) v[dy * F + dx] = ld1(src + ((long)dy * W + dx) * ld_in);
#pragma unroll
      for (int k = 0; k < F * F; ++k) s += v[k];  // same (dy, dx) order as below
    } else {
      for (int dy = 0; dy < f; ++dy)
        for (int dx = 0; dx < f; ++dx) s += ld1(src + ((long)dy * W + dx) * ld_in);
    }
    T* o = out + pix * ld_out + c;
    st1(o, accumulate ? ld1(o) + s : s);
  }
}

extern "C" int accunet_upsample_bwd(const void* in, int ld_in, int in_off, void* out, int ld_out,
                                    int B, int H, int W, int C, int f, int accumulate, int dt,
                                    void* stream) {
  if (H % f || W % f) return ACC_EBADSHAPE;
  long total = (long)B * (H / f) * (W / f) * C;
  hipStream_t s = (hipStream_t)stream;
  dim3 grid(grid_for(total));
  if (with_dt(dt, [&](auto tag) {
        using T = decltype(tag);
        const T* i = (const T*)in;
        T* o = (T*)out;
        if (f == 2)
          hipLaunchKernelGGL((blocksum_kernel<2, T>), grid, dim3(256), 0, s, i, ld_in, in_off, o,
                             ld_out, B, H, W, C, f, accumulate);
        else if (f == 4)
          hipLaunchKernelGGL((blocksum_kernel<4, T>), grid, dim3(256), 0, s, i, ld_in, in_off, o,
                             ld_out, B, H, W, C, f, accumulate);
        else if (f == 8)
          hipLaunchKernelGGL((blocksum_kernel<8, T>), grid, dim3(256), 0, s, i, ld_in, in_off, o,
                             ld_out, B, H, W, C, f, accumulate);
        else
          hipLaunchKernelGGL((blocksum_kernel<0, T>), grid, dim3(256), 0, s, i, ld_in, in_off, o,
                             ld_out, B, H, W, C, f, accumulate);
      }))
    return ACC_EBADARG;
  return hipGetLastError() == hipSuccess ? ACC_OK : ACC_ELAUNCH;
}

// The k = 3 HANCLayer pyramid's two backward sums from one read of in: a thread owns one
// 4x4 pixel block of one channel, adds each 2x2 quarter in (dy, dx) order (= blocksum
// <2>) and the 16 values in row-major order (= blocksum<4>), so both outputs carry the
// bits of the two separate launches.
template <typename T>
__global__ void __launch_bounds__(256)
blocksum24_kernel(const T* __restrict__ in, int ld_in, T* __restrict__ out2, int ld_out2,
                  T* __restrict__ out4, int ld_out4, int B, int H, int W, int C) {
  const int H4 = H / 4, W4 = W / 4;
  const long total = (long)B * H4 * W4 * C;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    const long pix = i / C;
    const int w4 = (int)(pix % W4);
    const long t = pix / W4;
    const int h4 = (int)(t % H4);
    const int b = (int)(t / H4);
    const T* src = in + (((long)b * H + h4 * 4) * W + w4 * 4) * ld_in + c;
    float v[16];
#pragma unroll
    for (int dy = 0; dy < 4; ++dy)
#pragma unroll
      for (int dx = 0; dx < 4; ++dx) v[dy * 4 + dx] = ld1(src + ((long)dy * W + dx) * ld_in);
    float s4 = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) s4 += v[k];
    st1(out4 + pix * ld_out4 + c, s4);
    const int H2 = H / 2, W2 = W / 2;
#pragma unroll
    for (int qy = 0; qy < 2; ++qy)
#pragma unroll
      for (int qx = 0; qx < 2; ++qx) {
        float s2 = 0.f;
        s2 += v[(2 * qy) * 4 + 2 * qx];
        s2 += v[(2 * qy) * 4 + 2 * qx + 1];
        s2 += v[(2 * qy + 1) * 4 + 2 * qx];
        s2 += v[(2 * qy + 1) * 4 + 2 * qx + 1];
        const long p2 = ((long)b * H2 + h4 * 2 + qy) * W2 + w4 * 2 + qx;
        st1(out2 + p2 * ld_out2 + c, s2);
      }
  }
}

extern "C" int accunet_upsample_bwd24(const void* in, int ld_in, void* out2, int ld_out2,
                                      void* out4, int ld_out4, int B, int H, int W, int C, int dt,
                                      void* stream) {
  if (H % 4 || W % 4) return ACC_EBADSHAPE;
  if (!in || !out2 || !out4) return ACC_EBADARG;
  const long total = (long)B * (H / 4) * (W / 4) * C;
  if (with_dt(dt, [&](auto tag) {
        using T = decltype(tag);
        hipLaunchKernelGGL(blocksum24_kernel<T>, dim3(grid_for(total)), dim3(256), 0,
                           (hipStream_t)stream, (const T*)in, ld_in, (T*)out2, ld_out2, (T*)out4,
                           ld_out4, B, H, W, C);
      }))
    return ACC_EBADARG;
  return hipGetLastError() == hipSuccess ? ACC_OK : ACC_ELAUNCH;
}

// ---------------------------------------------------------------------------
// Strided channel-slice copy: dst[p, dst_off + c] (+)= src[p, src_off + c], c < C
// ---------------------------------------------------------------------------
template <typename T>
__global__ void __launch_bounds__(256)
slice_copy_kernel(const T* __restrict__ src, int ld_src, int src_off, T* __restrict__ dst,
                  int ld_dst, int dst_off, long P, int C, int accumulate) {
  long total = P * C;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    long p = i / C;
    int c = (int)(i - p * C);
    T* d = dst + p * ld_dst + dst_off + c;
    if (accumulate) st1(d, ld1(d) + ld1(src + p * ld_src + src_off + c));
    else *d = src[p * ld_src + src_off + c];  // exact copy in the storage type
  }
}

extern "C" int accunet_slice_copy(const void* src, int ld_src, int src_off, void* dst,
                                  int ld_dst, int dst_off, long P, int C, int accumulate, int dt,
                                  void* stream) {
  if (with_dt(dt, [&](auto tag) {
        using T = decltype(tag);
        hipLaunchKernelGGL((slice_copy_kernel<T>), dim3(grid_for(P * C)), dim3(256), 0,
                           (hipStream_t)stream, (const T*)src, ld_src, src_off, (T*)dst, ld_dst,
                           dst_off, P, C, accumulate);
      }))
    return ACC_EBADARG;
  return hipGetLastError() == hipSuccess ? ACC_OK : ACC_ELAUNCH;
}

// ---------------------------------------------------------------------------
// ConvTranspose2d(k=2,s=2) pixel shuffle. GEMM output T[b,i,j,(d*Cout+co)],
// d = di*2+dj  ->  Y[b,2i+di,2j+dj,co] (+bias). Inverse for the backward.
// ---------------------------------------------------------------------------
template <typename T>
__global__ void __launch_bounds__(256)
pixel_shuffle2_kernel(const T* __restrict__ t, const float* __restrict__ bias,
                      T* __restrict__ y, int B, int Hi, int Wi, int Cout, int inverse) {
  const int Ho = 2 * Hi, Wo = 2 * Wi;
  long total = (long)B * Ho * Wo * Cout;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    int co = (int)(i % Cout);
    long pix = i / Cout;
    int wo = (int)(pix % Wo);
    long q = pix / Wo;
    int ho = (int)(q % Ho);
    int b = (int)(q / Ho);
    int d = (ho & 1) * 2 + (wo & 1);
    long ti = (((long)b * Hi + (ho >> 1)) * Wi + (wo >> 1)) * (4 * Cout) + d * Cout + co;
    if (!inverse) {
      st1(y + i, ld1(t + ti) + (bias ? bias[co] : 0.f));
    } else {
      // here y is the gradient dY (input), t is dT (output)
      const_cast<T*>(t)[ti] = y[i];
    }
  }
}

extern "C" int accunet_pixel_shuffle2(const void* t, const float* bias, void* y, int B, int Hi,
                                      int Wi, int Cout, int inverse, int dt, void* stream) {
  long total = (long)B * 4 * Hi * Wi * Cout;
  if (with_dt(dt, [&](auto tag) {
        using T = decltype(tag);
        hipLaunchKernelGGL((pixel_shuffle2_kernel<T>), dim3(grid_for(total)), dim3(256), 0,
                           (hipStream_t)stream, (const T*)t, bias, (T*)y, B, Hi, Wi, Cout, inverse);
      }))
    return ACC_EBADARG;
  return hipGetLastError() == hipSuccess ? ACC_OK : ACC_ELAUNCH;
}

// ---------------------------------------------------------------------------
// Decoder up-sampling + channel concat in one pass (ACC_UNet.py:637-648:
// torch.cat([ConvTranspose2d(x), skip], dim=1)): the ConvT GEMM output T [b,i,j,
// (d*Co+co)] is pixel-shuffled (+bias) into channels [0, Co) of Y [b,ho,wo,Co+Cs] and
// the skip tensor copied into channels [Co, Co+Cs); a block walks one output row in
// channel quads. inverse: dY -> dT (shuffled back) and dskip (null: not wanted). The
// shuffled values and the bias add are the pixel_shuffle2 kernel's, element for
// element; the up-sampled tensor itself is never written (no slice copies).
// ---------------------------------------------------------------------------
template <typename T>
__global__ void __launch_bounds__(256)
convt_cat_kernel(T* __restrict__ t, const float* __restrict__ bias, T* __restrict__ skip,
                 T* __restrict__ y, int Hi, int Wi, int Co, int Cs, int inverse) {
  const int Ho = 2 * Hi, Wo = 2 * Wi, Ct = Co + Cs;
  const int CQt = Ct / 4, CQo = Co / 4;
  const int row = blockIdx.x;  // b * Ho + ho
  const int ho = row % Ho, b = row / Ho;
  const int di = ho & 1, hi = ho >> 1;
  const long yrow = (long)row * Wo * Ct;
  const long trow = ((long)b * Hi + hi) * Wi * (4 * Co);
  const long srow = (long)row * Wo * Cs;
  const int n = Wo * CQt;
  for (int e = threadIdx.x; e < n; e += blockDim.x) {
    const int wo = e / CQt, cq = e - wo * CQt;
    T* yp = y + yrow + (long)wo * Ct + 4 * cq;
    if (cq < CQo) {
      const int d = di * 2 + (wo & 1), c = 4 * cq;
      T* tp = t + trow + (long)(wo >> 1) * (4 * Co) + d * Co + c;
      if (!inverse) {
        float4 v = ldq(tp);
        if (bias) {
          const float4 bb = ld4(bias + c);
          v.x += bb.x; v.y += bb.y; v.z += bb.z; v.w += bb.w;
        }
        stq(yp, v);
      } else {
        stq(tp, ldq(yp));
      }
    } else {
      T* sp = skip ? skip + srow + (long)wo * Cs + 4 * (cq - CQo) : nullptr;
      if (!inverse) stq(yp, ldq(sp));
      else if (sp) stq(sp, ldq(yp));
    }
  }
}

extern "C" int accunet_convt_cat(void* t, const float* bias, void* skip, void* y, int B, int Hi,
                                 int Wi, int Co, int Cs, int inverse, int dt, void* stream) {
  if (B <= 0 || Hi <= 0 || Wi <= 0 || Co <= 0 || Cs < 0 || (Co % 4) || (Cs % 4))
    return ACC_EBADSHAPE;
  if (!t || !y || (!inverse && Cs > 0 && !skip)) return ACC_EBADARG;
  if (with_dt(dt, [&](auto tag) {
        using T = decltype(tag);
        hipLaunchKernelGGL((convt_cat_kernel<T>), dim3(B * 2 * Hi), dim3(256), 0,
                           (hipStream_t)stream, (T*)t, bias, (T*)skip, (T*)y, Hi, Wi, Co, Cs,
                           inverse);
      }))
    return ACC_EBADARG;
  return hipGetLastError() == hipSuccess ? ACC_OK : ACC_ELAUNCH;
}

// ---------------------------------------------------------------------------
// Generic 4-D permute: out[i0,i1,i2,i3] (out dims d) = in[...] with in strides
// given per OUTPUT axis (so any permutation / flip is expressed by strides and
// per-axis flip flags). accumulate adds into out.
// ---------------------------------------------------------------------------
struct Perm4 {
  int d[4];
  long s[4];
  int flip[4];
};

template <typename TI, typename TO>
__global__ void __launch_bounds__(256)
permute4_kernel(const TI* __restrict__ in, TO* __restrict__ out, Perm4 p, int accumulate) {
  long total = (long)p.d[0] * p.d[1] * p.d[2] * p.d[3];
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    long r = i;
    long off = 0;
    for (int a = 3; a >= 0; --a) {
      int ia = (int)(r % p.d[a]);
      r /= p.d[a];
      if (p.flip[a]) ia = p.d[a] - 1 - ia;
      off += ia * p.s[a];
    }
    st1(out + i, accumulate ? ld1(out + i) + ld1(in + off) : ld1(in + off));
  }
}

extern "C" int accunet_permute4(const void* in, void* out, const int* dims, const long long* strides,
                                const int* flips, int accumulate, int in_dt, int out_dt,
                                void* stream) {
  Perm4 p;
  for (int a = 0; a < 4; ++a) {
    p.d[a] = dims[a];
    p.s[a] = strides[a];
    p.flip[a] = flips ? flips[a] : 0;
  }
  long total = (long)p.d[0] * p.d[1] * p.d[2] * p.d[3];
  if (with_dt(in_dt, [&](auto ti) {
        using TI = decltype(ti);
        if (with_dt(out_dt, [&](auto to) {
              using TO = decltype(to);
              hipLaunchKernelGGL((permute4_kernel<TI, TO>), dim3(grid_for(total)), dim3(256), 0,
                                 (hipStream_t)stream, (const TI*)in, (TO*)out, p, accumulate);
            }))
          in_dt = -1;
      }) || in_dt < 0)
    return ACC_EBADARG;
  return hipGetLastError() == hipSuccess ? ACC_OK : ACC_ELAUNCH;
}

// ---------------------------------------------------------------------------
// Grouped-column weight relayout for the channel-interleaved concats:
//   HANCLayer: input channel c*J + j of hnc.cnv is branch j of channel c
//   (ACC_UNet/ACC_UNet.py:96-106,138); MLFC merge: 2c = x_c, 2c+1 = x (:492)
// out[n][jj][c] = W[n][c*J + order[jj]]   (inverse: scatter back, accumulate opt.)
// ---------------------------------------------------------------------------
struct JOrder {
  int o[8];
};

__global__ void __launch_bounds__(256)
group_relayout_kernel(const float* __restrict__ in, float* __restrict__ out, int N, int C, int J,
                      JOrder ord, int inverse) {
  long total = (long)N * J * C;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    int c = (int)(i % C);
    long t = i / C;
    int jj = (int)(t % J);
    int n = (int)(t / J);
    long src = (long)n * C * J + (long)c * J + ord.o[jj];
    if (!inverse) out[i] = in[src];
    else out[src] = in[i];
  }
}

extern "C" int accunet_group_relayout(const float* in, float* out, int N, int C, int J,
                                      const int* order, int inverse, void* stream) {
  if (J < 1 || J > 8) return ACC_EBADARG;
  JOrder o;
  for (int j = 0; j < 8; ++j) o.o[j] = (order && j < J) ? order[j] : j;
  long total = (long)N * J * C;
  hipLaunchKernelGGL(group_relayout_kernel, dim3(grid_for(total)), dim3(256), 0,
                     (hipStream_t)stream, in, out, N, C, J, o, inverse);
  return hipGetLastError() == hipSuccess ? ACC_OK : ACC_ELAUNCH;
}

// ---------------------------------------------------------------------------
// Batched weight relayouts: every forward-layout weight copy of a training step in one
// launch (accunet/ops.py: WeightPrep, used by the graph-mode TrainStep before each
// replay) instead of one small launch per layer. Item i (AccRelayout, device memory)
// owns blocks [blk0_i, blk0_{i+1}); kind 0 = accunet_permute4's gather, kind 1 =
// accunet_group_relayout's forward, kind 2 its inverse (the backward's weight
// gradients, ops.DeferredRelayouts); the same index arithmetic, so the copies are the
// ones the per-layer launches make. kind 3 / 4 = flat copies into a gradient bucket
// (fp32 / rounded to bf16 like torch's .to(bfloat16), times `scale` = 1/world: the
// graph-mode data-parallel step packs each sealed bucket in one launch and all-reduces
// it with SUM, accunet/train.py _GraphBuckets).
// ---------------------------------------------------------------------------
#define RL_EPT 4
__global__ void __launch_bounds__(256)
relayout_batch_kernel(const AccRelayout* __restrict__ items, int n) {
  // the item of this block: the last one whose blk0 <= blockIdx.x (blk0 ascending),
  // searched in LDS (the blk0 column fetched in one parallel round trip instead of a
  // chain of ~log2(n) dependent loads per block: the bucket packs run thousands of blocks)
  constexpr int RL_LDS = 1024;
  __shared__ int sblk[RL_LDS];
  const bool in_lds = n <= RL_LDS;  // (uniform)
  if (in_lds) {
    for (int i = threadIdx.x; i < n; i += blockDim.x) sblk[i] = items[i].blk0;
    __syncthreads();
  }
  int lo = 0, hi = n - 1;
  const int bid = (int)blockIdx.x;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if ((in_lds ? sblk[mid] : items[mid].blk0) <= bid) lo = mid; else hi = mid - 1;
  }
  const AccRelayout& it = items[lo];
  const long base = ((long)(bid - it.blk0) * 256 + threadIdx.x) * RL_EPT;
  static_assert(RL_EPT == 4, "the flat copies move one float4 per thread");
  if (it.kind >= 3 && base + 3 < it.total) {
    // flat copy, whole quad: one 16-byte load, one 16-byte (fp32) / 8-byte (bf16) store
    // where both ends are aligned (the bucket views start at 4-element offsets)
    const float* src = it.in + base;
    const bool k3 = it.kind == 3;
    const uintptr_t dst = k3 ? (uintptr_t)(it.out + base) : (uintptr_t)(reinterpret_cast<bf16_t*>(it.out) + base);
    if ((((uintptr_t)src) & 15) == 0 && (dst & (k3 ? 15 : 7)) == 0) {
      float4 v = *reinterpret_cast<const float4*>(src);
      v.x *= it.scale; v.y *= it.scale; v.z *= it.scale; v.w *= it.scale;
      if (k3) {
        *reinterpret_cast<float4*>(dst) = v;
      } else {
        uint2 u;
        u.x = (unsigned)f2bf(v.x) | ((unsigned)f2bf(v.y) << 16);
        u.y = (unsigned)f2bf(v.z) | ((unsigned)f2bf(v.w) << 16);
        *reinterpret_cast<uint2*>(dst) = u;
      }
      return;
    }
  }
#pragma unroll
  for (int e = 0; e < RL_EPT; ++e) {
    const long i = base + e;
    if (i >= it.total) break;
    if (it.kind >= 3) {  // flat copy (data-parallel bucket packing): fp32, or rounded to bf16
      if (it.kind == 3) it.out[i] = it.in[i] * it.scale;
      else reinterpret_cast<bf16_t*>(it.out)[i] = f2bf(it.in[i] * it.scale);
      continue;
    }
    long src;
    if (it.kind == 0) {
      long r = i;
      src = 0;
      for (int a = 3; a >= 0; --a) {
        int ia = (int)(r % it.d[a]);
        r /= it.d[a];
        if (it.flip[a]) ia = it.d[a] - 1 - ia;
        src += ia * it.s[a];
      }
    } else {
      const int c = (int)(i % it.C);
      const long t = i / it.C;
      const int jj = (int)(t % it.J);
      const int nn = (int)(t / it.J);
      src = (long)nn * it.C * it.J + (long)c * it.J + it.order[jj];
    }
    if (it.kind == 2) it.out[src] = it.in[i];  // the group relayout's inverse (scatter)
    else it.out[i] = it.in[src];
  }
}

extern "C" int accunet_relayout_blocks(long long total) {
  return (int)((total + 256L * RL_EPT - 1) / (256L * RL_EPT));
}

extern "C" int accunet_relayout_batch(const void* items_dev, int n, int nblocks, void* stream) {
  if (!items_dev || n <= 0 || nblocks <= 0) return ACC_EBADARG;
  hipLaunchKernelGGL(relayout_batch_kernel, dim3(nblocks), dim3(256), 0, (hipStream_t)stream,
                     (const AccRelayout*)items_dev, n);
  return hipGetLastError() == hipSuccess ? ACC_OK : ACC_ELAUNCH;
}
