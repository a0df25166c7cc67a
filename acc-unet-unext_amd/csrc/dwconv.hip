// Depthwise 3x3 convolution (stride 1, zero padding 1, +bias) on NHWC fp32 / bf16:
// HANCBlock.conv2 + norm2 statistics, reference ACC_UNet/ACC_UNet.py:240-247,273-275.
//
// K1 (forward): z[b,h,w,c] = bias[c] + sum_tap W[c][tap] * a[b,h+dh,w+dw,c] where the
// input a = act(x*scale[c] + shift[c]) is the pending BatchNorm(norm1)+LeakyReLU of the
// conv1 output x, applied in registers (a is never written to HBM). The epilogue
// writes per-block per-channel (sum z, sum z^2) partials for norm2.
//
// Mapping: a 256-thread block owns TCQ channel vectors (4 channels each) x (256/TCQ)
// consecutive pixels of one image row-strip of TR rows. Each thread slides a 3x3
// register window down its pixel column: per output row it issues 3 new 16-byte
// loads (its own column + the two neighbours, which are L1/L2 hits shared with the
// adjacent threads) and one 16-byte store, so HBM sees ~1 read + 1 write per element.
#include <type_traits>
#include "common.h"
#include "kernels.h"
#include "chan.h"
#include <stdlib.h>

#define DW_TR 8  // output rows per thread strip

// The tile prologue a = act(x*scale + shift) of one channel quad on packed pairs
// (v_pk_fma_f32 / v_pk_mul_f32), LeakyReLU as max(v, slope*v). Without a prologue it
// is the identity bit for bit: scale 1, shift -0 (x + -0 = x for every x), slope 1.
typedef float dwf2 __attribute__((ext_vector_type(2)));
struct DwPro {
  dwf2 s01, s23, t01, t23;
  float sl;
};
ACC_DEV DwPro dw_pro(float4 ps, float4 pb, bool pro, int act) {
  DwPro P;
  if (!pro) {
    ps = make_float4(1.f, 1.f, 1.f, 1.f);
    pb = make_float4(-0.f, -0.f, -0.f, -0.f);
  }
  P.s01 = dwf2{ps.x, ps.y};
  P.s23 = dwf2{ps.z, ps.w};
  P.t01 = dwf2{pb.x, pb.y};
  P.t23 = dwf2{pb.z, pb.w};
  P.sl = pro ? act_slope(act) : 1.f;
  return P;
}
ACC_DEV float4 dw_act(const DwPro& P, float4 a) {
  dwf2 lo = {a.x, a.y}, hi = {a.z, a.w};
  lo = lo * P.s01 + P.t01;
  hi = hi * P.s23 + P.t23;
  const dwf2 ml = lo * P.sl, mh = hi * P.sl;
  return make_float4(__builtin_fmaxf(lo.x, ml.x), __builtin_fmaxf(lo.y, ml.y),
                     __builtin_fmaxf(hi.x, mh.x), __builtin_fmaxf(hi.y, mh.y));
}
// component-wise keep-or-zero (a float4 ?: can be lowered through a scratch slot)
ACC_DEV float4 dw_keep(bool in, float4 v) {
  return make_float4(in ? v.x : 0.f, in ? v.y : 0.f, in ? v.z : 0.f, in ? v.w : 0.f);
}

template <int V>
struct VecT;
template <>
struct VecT<4> {
  typedef float4 T;
};
template <>
struct VecT<1> {
  typedef float T;
};

template <int V, typename T>
ACC_DEV void vload(const T* p, float (&v)[V]) {
  ldv<V>(p, v);
}
template <int V, typename T>
ACC_DEV void vstore(T* p, const float (&v)[V]) {
  stv<V>(p, v);
}

struct DwGeom {
  int B, H, W, C;
  int TCQ;      // channel vectors per block
  int TW;       // pixels per block row
  int tilesW, tilesH;
};

// flip != 0: use W[c][8-tap] (data gradient = correlation with the flipped kernel)
template <int V, typename T>
__global__ void __launch_bounds__(256)
dw3x3_fwd_kernel(const T* __restrict__ x, const float* __restrict__ wt,
                 const float* __restrict__ bias, const float* __restrict__ sc,
                 const float* __restrict__ sh, int act, int flip, T* __restrict__ z,
                 double* __restrict__ stats, DwGeom g, const T* __restrict__ bz,
                 const float* __restrict__ bst, int bact) {
  const bool bnb = stats != nullptr && bz != nullptr;  // see dw3x3_tile_fwd_kernel
  const int tid = threadIdx.x;
  const int cql = tid % g.TCQ;
  const int px = tid / g.TCQ;
  const int cq = blockIdx.y * g.TCQ + cql;
  const int c0 = cq * V;
  int t = blockIdx.x;
  const int tw = t % g.tilesW;
  t /= g.tilesW;
  const int th = t % g.tilesH;
  const int b = t / g.tilesH;
  const int w = tw * g.TW + px;
  const int h0 = th * DW_TR;
  const bool active = (px < g.TW) && (w < g.W) && (c0 < g.C);
  const int C = g.C;

  double s1[V], s2[V];
#pragma unroll
  for (int j = 0; j < V; ++j) { s1[j] = 0.0; s2[j] = 0.0; }

  if (active) {
    float k[9][V], bi[V], psc[V], psh[V];
#pragma unroll
    for (int j = 0; j < V; ++j) {
#pragma unroll
      for (int tp = 0; tp < 9; ++tp) k[tp][j] = wt[(c0 + j) * 9 + (flip ? 8 - tp : tp)];
      bi[j] = bias ? bias[c0 + j] : 0.f;
      psc[j] = sc ? sc[c0 + j] : 1.f;
      psh[j] = sh ? sh[c0 + j] : 0.f;
    }
    const bool pro = sc != nullptr;
    // window rows r0 (h-1), r1 (h), r2 (h+1); columns w-1, w, w+1
    float win[3][3][V];
    auto load_row = [&](int hh, float (&row)[3][V]) {
#pragma unroll
      for (int dx = 0; dx < 3; ++dx) {
        int ww = w + dx - 1;
        if (hh >= 0 && hh < g.H && ww >= 0 && ww < g.W) {
          vload<V>(x + (((long)b * g.H + hh) * g.W + ww) * C + c0, row[dx]);
          if (pro) {
#pragma unroll
            for (int j = 0; j < V; ++j) row[dx][j] = apply_act(row[dx][j] * psc[j] + psh[j], act);
          }
        } else {
#pragma unroll
          for (int j = 0; j < V; ++j) row[dx][j] = 0.f;
        }
      }
    };
    load_row(h0 - 1, win[0]);
    load_row(h0, win[1]);
    const int h1 = min(g.H, h0 + DW_TR);
    for (int h = h0; h < h1; ++h) {
      load_row(h + 1, win[2]);
      float o[V];
#pragma unroll
      for (int j = 0; j < V; ++j) {
        float acc = bi[j];
#pragma unroll
        for (int dy = 0; dy < 3; ++dy)
#pragma unroll
          for (int dx = 0; dx < 3; ++dx) acc = fmaf(k[dy * 3 + dx][j], win[dy][dx][j], acc);
        acc = rnd<T>(acc);  // statistics of the stored value
        o[j] = acc;
        if (bnb) {
          const float zz = ld1(bz + (((long)b * g.H + h) * g.W + w) * C + c0 + j);
          float gg = acc;
          if (bact == ACT_LRELU)
            gg *= lrelu_d(zz * bst[BN_SCALE * C + c0 + j] + bst[BN_SHIFT * C + c0 + j]);
          s1[j] += gg;
          s2[j] += (double)gg * ((double)zz - bst[BN_MEAN * C + c0 + j]);
        } else {
          s1[j] += acc;
          s2[j] += (double)acc * acc;
        }
      }
      vstore<V>(z + (((long)b * g.H + h) * g.W + w) * C + c0, o);
#pragma unroll
      for (int dx = 0; dx < 3; ++dx)
#pragma unroll
        for (int j = 0; j < V; ++j) {
          win[0][dx][j] = win[1][dx][j];
          win[1][dx][j] = win[2][dx][j];
        }
    }
  }

  if (stats) {
    __shared__ double red[2][256 * 4];
#pragma unroll
    for (int j = 0; j < V; ++j) {
      red[0][tid * V + j] = s1[j];
      red[1][tid * V + j] = s2[j];
    }
    __syncthreads();
    if (px == 0 && c0 < C) {
      int npx = 256 / g.TCQ;
#pragma unroll
      for (int j = 0; j < V; ++j) {
        double a = 0.0, q = 0.0;
        for (int i = 0; i < npx; ++i) {
          a += red[0][(i * g.TCQ + cql) * V + j];
          q += red[1][(i * g.TCQ + cql) * V + j];
        }
        stats[(long)blockIdx.x * 2 * C + c0 + j] = a;
        stats[(long)blockIdx.x * 2 * C + C + c0 + j] = q;
      }
    }
  }
}

// Weight + bias gradient: dW[c][tap] = sum_p dz[p,c] * a[shift_tap(p), c],
// db[c] = sum_p dz[p,c]; a = act(x*scale+shift) recomputed. Output partials
// [block][10][C] (taps 0..8, then bias).
template <int V, typename T>
__global__ void __launch_bounds__(256)
dw3x3_wgrad_kernel(const T* __restrict__ x, const T* __restrict__ dz,
                   const float* __restrict__ sc, const float* __restrict__ sh, int act,
                   float* __restrict__ part, DwGeom g) {
  const int tid = threadIdx.x;
  const int cql = tid % g.TCQ;
  const int px = tid / g.TCQ;
  const int cq = blockIdx.y * g.TCQ + cql;
  const int c0 = cq * V;
  int t = blockIdx.x;
  const int tw = t % g.tilesW;
  t /= g.tilesW;
  const int th = t % g.tilesH;
  const int b = t / g.tilesH;
  const int w = tw * g.TW + px;
  const int h0 = th * DW_TR;
  const bool active = (px < g.TW) && (w < g.W) && (c0 < g.C);
  const int C = g.C;

  float acc[10][V];
#pragma unroll
  for (int i = 0; i < 10; ++i)
#pragma unroll
    for (int j = 0; j < V; ++j) acc[i][j] = 0.f;

  if (active) {
    float psc[V], psh[V];
#pragma unroll
    for (int j = 0; j < V; ++j) {
      psc[j] = sc ? sc[c0 + j] : 1.f;
      psh[j] = sh ? sh[c0 + j] : 0.f;
    }
    const bool pro = sc != nullptr;
    float win[3][3][V];
    auto load_row = [&](int hh, float (&row)[3][V]) {
#pragma unroll
      for (int dx = 0; dx < 3; ++dx) {
        int ww = w + dx - 1;
        if (hh >= 0 && hh < g.H && ww >= 0 && ww < g.W) {
          vload<V>(x + (((long)b * g.H + hh) * g.W + ww) * C + c0, row[dx]);
          if (pro) {
#pragma unroll
            for (int j = 0; j < V; ++j) row[dx][j] = apply_act(row[dx][j] * psc[j] + psh[j], act);
          }
        } else {
#pragma unroll
          for (int j = 0; j < V; ++j) row[dx][j] = 0.f;
        }
      }
    };
    load_row(h0 - 1, win[0]);
    load_row(h0, win[1]);
    const int h1 = min(g.H, h0 + DW_TR);
    for (int h = h0; h < h1; ++h) {
      load_row(h + 1, win[2]);
      float d[V];
      vload<V>(dz + (((long)b * g.H + h) * g.W + w) * C + c0, d);
#pragma unroll
      for (int j = 0; j < V; ++j) {
#pragma unroll
        for (int dy = 0; dy < 3; ++dy)
#pragma unroll
          for (int dx = 0; dx < 3; ++dx) acc[dy * 3 + dx][j] = fmaf(d[j], win[dy][dx][j], acc[dy * 3 + dx][j]);
        acc[9][j] += d[j];
      }
#pragma unroll
      for (int dx = 0; dx < 3; ++dx)
#pragma unroll
        for (int j = 0; j < V; ++j) {
          win[0][dx][j] = win[1][dx][j];
          win[1][dx][j] = win[2][dx][j];
        }
    }
  }

  __shared__ float red[256 * 4];
  const int npx = 256 / g.TCQ;
  for (int i = 0; i < 10; ++i) {
#pragma unroll
    for (int j = 0; j < V; ++j) red[tid * V + j] = acc[i][j];
    __syncthreads();
    if (px == 0 && c0 < C) {
#pragma unroll
      for (int j = 0; j < V; ++j) {
        float a = 0.f;
        for (int k = 0; k < npx; ++k) a += red[(k * g.TCQ + cql) * V + j];
        part[((long)blockIdx.x * 10 + i) * C + c0 + j] = a;
      }
    }
    __syncthreads();
  }
}

// [10][C] sums -> dW[c][tap] (torch layout [C][1][3][3]) and db[c]
__global__ void dw_wgrad_finish_kernel(const float* __restrict__ sums, int C, float* __restrict__ dw,
                                       float* __restrict__ db) {
  int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
#pragma unroll
  for (int tp = 0; tp < 9; ++tp) dw[c * 9 + tp] = sums[tp * C + c];
  if (db) db[c] = sums[9 * C + c];
}

// ----------------------------------------------------------------------------
// LDS-tiled kernels (C % 32 == 0: every ACC-UNet HANC width except cnv11's 9).
// A block owns TR=8 output rows x TP pixels x TCQ channel quads; it first pulls the
// whole (TR+2) x (TP+2) x TCQ input halo tile into LDS with ~11 independent 16-byte
// loads per thread (prologue BN+act applied on the way, zero padding after the
// activation), so each CU keeps >100 KB of HBM reads in flight instead of the
// ~3 dependent loads per row of the register-window kernel above; then every
// thread slides its 3x3 window down LDS. Tiles are handed out XCD-contiguously
// (consecutive workgroup ids land on different XCDs; the remap gives each XCD a
// contiguous run of tiles so halo rows/columns shared by neighbours hit its L2).
// ----------------------------------------------------------------------------
// forward statistics accumulated in fp32 over each 4-row chunk, then in fp64 (one fp64
// add per chunk instead of per element: bf16 K1 100 -> 95 us, fp32 unchanged; tools/kbench)
#ifndef K1_CHUNK_STATS
#define K1_CHUNK_STATS 1
#endif
struct DwTGeom {
  int B, H, W, C;
  int tilesW, tilesH;
  int rch;    // 8-row chunks per block (forward kernel: a vertical strip of 8*rch rows)
  int ntl;    // non-temporal input loads (tuning knob ACCUNET_DW_NTL)
  int remap;  // ntiles % 8 == 0: XCD-contiguous tile order
  int cgf;    // forward: > 0 = 1-D grid, channel group fastest (cgf groups per tile)
};

ACC_DEV int dw_tile_id(const DwTGeom& g) {
  int bid = blockIdx.x;
  if (g.remap) {
    int per = gridDim.x >> 3;
    bid = (bid & 7) * per + (bid >> 3);
  }
  return bid;
}

template <int TCQ>
struct DwT {
  static constexpr int TP = 256 / TCQ;  // output pixels per tile row
  static constexpr int IP = TP + 2;
  static constexpr int IR = DW_TR + 2;
  static constexpr int N4 = IR * IP * TCQ;  // float4 elements of the input tile
  static constexpr int NK = (N4 + 255) / 256;
  static constexpr int CR = 4;                 // strip pipeline: rows per chunk
  static constexpr int N8 = CR * IP * TCQ;     // float4 elements of CR new input rows
  static constexpr int NK8 = (N8 + 255) / 256;
};

// 16-byte raw loads of the staging paths: QL quads per load (fp32: 1 float4; bf16: 2
// quads = 8 channels, so a bf16 tile moves in half the load instructions of fp32)
template <typename T> struct Raw16 { typedef float4 type; static constexpr int QL = 1; };
template <> struct Raw16<bf16_t> { typedef uint4 type; static constexpr int QL = 2; };
template <int AUX>
ACC_DEV float4 buf16_ld(__amdgpu_buffer_rsrc_t r, unsigned off, const float*) {
  return bufq_ld<AUX>(r, off, (const float*)nullptr);
}
template <int AUX>
ACC_DEV uint4 buf16_ld(__amdgpu_buffer_rsrc_t r, unsigned off, const bf16_t*) {
  const acc_u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, AUX);
  return make_uint4(v[0], v[1], v[2], v[3]);
}
ACC_DEV float4 r16q(float4 v, int) { return v; }
ACC_DEV float4 r16q(uint4 u, int j) {
  return j == 0 ? make_float4(bflo(u.x), bfhi(u.x), bflo(u.y), bfhi(u.y))
                : make_float4(bflo(u.z), bfhi(u.z), bflo(u.w), bfhi(u.w));
}
ACC_DEV uint4 ld16_raw(const bf16_t* p) { return *reinterpret_cast<const uint4*>(p); }
ACC_DEV float4 ld16_raw(const float* p) { return ld4(p); }

// prologue (BN scale/shift) of the QL quads a thread always stages: quads q0 .. q0+QL-1,
// q0 = (tid * QL) % TCQ (256 * QL % TCQ == 0, so the same quads for every load)
template <int TCQ, int QL>
ACC_DEV void dw_stage_pro(const float* sc, const float* sh, int c0, float4 (&ps)[QL],
                          float4 (&pb)[QL]) {
  const int q0 = (threadIdx.x * QL) % TCQ;
#pragma unroll
  for (int j = 0; j < QL; ++j) {
    ps[j] = sc ? ld4(sc + c0 + 4 * (q0 + j)) : make_float4(1.f, 1.f, 1.f, 1.f);
    pb[j] = sc ? ld4(sh + c0 + 4 * (q0 + j)) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
}

// Strip pipeline helpers: input rows live in a 10-slot LDS ring, row h of the
// block's strip (which starts at output row hbeg) in slot (h - hbeg + 1) % 10.
// Fetch `n` quads of consecutive input rows starting at row hA into registers, raw
// (zero outside the image / past n: ACC_OOB offsets, no branches), QL quads per
// 16-byte load. rx covers one image.
template <int TCQ, int NKK, int AUX, typename TX>
ACC_DEV void dw_fetch_rows(typename Raw16<TX>::type (&v)[NKK], __amdgpu_buffer_rsrc_t rx,
                           const DwTGeom& g, int hA, int n, int w0, int c0) {
  typedef DwT<TCQ> G;
  constexpr int QL = Raw16<TX>::QL;
  const int tid = threadIdx.x;
#pragma unroll
  for (int k = 0; k < NKK; ++k) {
    const int i = (tid + 256 * k) * QL;  // first quad of this load
    const int rp = i / TCQ, q = i % TCQ;
    const int p = rp % G::IP, r = rp / G::IP;
    const int hh = hA + r, ww = w0 - 1 + p;
    const bool in = i < n && hh >= 0 && hh < g.H && ww >= 0 && ww < g.W;
    const unsigned off = in ? (unsigned)(((hh * g.W + ww) * g.C + c0 + 4 * q) * (int)sizeof(TX))
                            : ACC_OOB;
    v[k] = buf16_ld<AUX>(rx, off, (const TX*)nullptr);
  }
}

// Activate (prologue BN+act, in-image elements only) and park fetched rows in the ring.
template <int TCQ, int NKK, int QL, typename R>
ACC_DEV void dw_park_rows(float4* __restrict__ ring, const R (&v)[NKK], const DwTGeom& g,
                          int hA, int n, int w0, int hbeg, const DwPro (&P)[QL]) {
  typedef DwT<TCQ> G;
  const int tid = threadIdx.x;
#pragma unroll
  for (int k = 0; k < NKK; ++k) {
    const int i = (tid + 256 * k) * QL;
    if (i < n) {
      const int rp = i / TCQ, q = i % TCQ;
      const int p = rp % G::IP, r = rp / G::IP;
      const int hh = hA + r, ww = w0 - 1 + p;
      const bool in = hh >= 0 && hh < g.H && ww >= 0 && ww < g.W;
      const int slot = (hh - hbeg + 1) % G::IR;
#pragma unroll
      for (int j = 0; j < QL; ++j)  // out-of-image quads loaded as zeros stay zero
        ring[(slot * G::IP + p) * TCQ + q + j] = dw_keep(in, dw_act(P[j], r16q(v[k], j)));
    }
  }
}

// load the activated input tile a = act(x*sc+sh) (zero outside the image) into LDS
template <int TCQ, typename TX>
ACC_DEV void dw_fill_tile(float4* __restrict__ tile, const TX* __restrict__ x,
                          const float* __restrict__ sc, const float* __restrict__ sh, int act,
                          const DwTGeom& g, int b, int h0, int w0, int c0) {
  typedef DwT<TCQ> G;
  constexpr int QL = Raw16<TX>::QL;
  constexpr int NL = (G::N4 / QL + 255) / 256;  // 16-byte loads per thread
  const int tid = threadIdx.x;
  float4 ps[QL], pb[QL];
  dw_stage_pro<TCQ, QL>(sc, sh, c0, ps, pb);
  DwPro P[QL];
#pragma unroll
  for (int j = 0; j < QL; ++j) P[j] = dw_pro(ps[j], pb[j], sc != nullptr, act);
  // raw, unconditional loads (out-of-image quads read the image origin and are zeroed
  // at the LDS write): all NL in flight together, bf16 widened only when parked
  typedef typename Raw16<TX>::type RawL;
  RawL v[NL];
  bool in[NL];
#pragma unroll
  for (int k = 0; k < NL; ++k) {
    const int i = (tid + 256 * k) * QL;
    const int rp = i / TCQ, q = i % TCQ;
    const int p = rp % G::IP, r = rp / G::IP;
    const int hh = h0 - 1 + r, ww = w0 - 1 + p;
    in[k] = (i < G::N4) && hh >= 0 && hh < g.H && ww >= 0 && ww < g.W;
    v[k] = ld16_raw(in[k] ? x + (((long)b * g.H + hh) * g.W + ww) * g.C + c0 + 4 * q : x);
  }
#pragma unroll
  for (int k = 0; k < NL; ++k) {
    const int i = (tid + 256 * k) * QL;
    if (i < G::N4) {
#pragma unroll
      for (int j = 0; j < QL; ++j) tile[i + j] = dw_keep(in[k], dw_act(P[j], r16q(v[k], j)));
    }
  }
}

// Forward: a block owns a vertical strip of 8*rch output rows x TP pixels x TCQ
// channel quads and walks it in CR=4-row chunks over a 10-slot LDS ring that holds
// input rows r0-1 .. r0+8 at the start of the chunk at row r0. The CR rows the
// NEXT chunk adds (r0+9 .. r0+12) are fetched into registers before this chunk is
// computed and parked afterwards in the slots of rows r0-1 .. r0+2 (dead by then),
// so HBM reads stay in flight through the compute (software pipeline).
// The strip loop is branch-free in its memory operations (buffer loads / stores
// with out-of-range offsets for the lanes and rows that are masked off), so the
// park waits for the prefetched rows only (vmcnt(N)), not for the chunk's stores.
template <int TCQ, bool BNB, int AUX, typename T>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(BNB ? 2 : 3)))
dw3x3_tile_fwd_kernel(const T* __restrict__ x, const float* __restrict__ wt,
                      const float* __restrict__ bias, const float* __restrict__ sc,
                      const float* __restrict__ sh, int act, int flip, T* __restrict__ z,
                      double* __restrict__ stats, DwTGeom g, const T* __restrict__ bz,
                      const float* __restrict__ bst, int bact) {
  typedef DwT<TCQ> G;
  typedef typename QuadRaw<T>::type RawQ;
  typedef typename Raw16<T>::type RawL;
  constexpr int CR = G::CR;
  constexpr int QL = Raw16<T>::QL;
  constexpr int NL = (G::N4 / QL + 255) / 256;   // 16-byte loads: whole tile
  constexpr int NL8 = (G::N8 / QL + 255) / 256;  // 16-byte loads: CR new rows
  __shared__ float4 tile[G::N4 > 1024 ? G::N4 : 1024];
  // BNB (data gradient, flip = 1): stats receive the BatchNorm-backward partials
  // (sum g, sum g*(bz - mean)) of g = out * act'(bz*scale + shift) instead of (sum, sumsq)
  const int tid = threadIdx.x;
  const int q = tid % TCQ, p = tid / TCQ;
  int t = dw_tile_id(g);
  int cg = blockIdx.y;
  if (g.cgf) {  // the channel groups of one tile are neighbours in dispatch order
    cg = t % g.cgf;
    t /= g.cgf;
  }
  const int srow = g.cgf ? t : (int)blockIdx.x;  // statistics partial row of this tile
  const int c0 = cg * TCQ * 4;
  const int c = c0 + 4 * q;
  const int tw = t % g.tilesW;
  t /= g.tilesW;
  const int th = t % g.tilesH;
  const int b = t / g.tilesH;
  const int hbeg = th * DW_TR * g.rch, w0 = tw * G::TP;
  const int hend = min(g.H, hbeg + DW_TR * g.rch);
  const int nch = (hend - hbeg + CR - 1) / CR;
  // one image per descriptor (the host keeps H*W*C*4 < 2^31)
  const long img = (long)b * g.H * g.W * g.C;
  const unsigned ibytes = (unsigned)(g.H * g.W * g.C * (int)sizeof(T));
  const __amdgpu_buffer_rsrc_t rx = acc_rsrc(x + img, ibytes);
  const __amdgpu_buffer_rsrc_t rz = acc_rsrc(z + img, ibytes);
  const __amdgpu_buffer_rsrc_t rb = acc_rsrc(BNB ? bz + img : x + img, BNB ? ibytes : 0u);
  DwPro P[QL];
  {
    float4 ps[QL], pb[QL];
    dw_stage_pro<TCQ, QL>(sc, sh, c0, ps, pb);
#pragma unroll
    for (int j = 0; j < QL; ++j) P[j] = dw_pro(ps[j], pb[j], sc != nullptr, act);
  }
  {
    RawL v[NL];
    dw_fetch_rows<TCQ, NL, AUX, T>(v, rx, g, hbeg - 1, G::N4, w0, c0);
    dw_park_rows<TCQ, NL, QL>(tile, v, g, hbeg - 1, G::N4, w0, hbeg, P);
  }
  // the quad's 4 channels x 9 taps are 36 contiguous floats of wt ([C][9], 16-B aligned
  // since c % 4 == 0): 9 float4 loads instead of 36 scalar ones
  float k[9][4], bi[4];
  {
    float wv[36];
#pragma unroll
    for (int e = 0; e < 9; ++e) {
      const float4 w4 = ld4(wt + c * 9 + 4 * e);
      wv[4 * e] = w4.x; wv[4 * e + 1] = w4.y; wv[4 * e + 2] = w4.z; wv[4 * e + 3] = w4.w;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int tp = 0; tp < 9; ++tp) k[tp][j] = wv[j * 9 + (flip ? 8 - tp : tp)];
    const float4 b4 = bias ? ld4(bias + c) : make_float4(0.f, 0.f, 0.f, 0.f);
    bi[0] = b4.x; bi[1] = b4.y; bi[2] = b4.z; bi[3] = b4.w;
  }
  float bmu[4] = {0.f, 0.f, 0.f, 0.f}, bsc[4] = {0.f, 0.f, 0.f, 0.f}, bsh[4] = {0.f, 0.f, 0.f, 0.f};
  if (BNB) {
    const float4 m4 = ld4(bst + BN_MEAN * g.C + c), s4 = ld4(bst + BN_SCALE * g.C + c),
                 h4 = ld4(bst + BN_SHIFT * g.C + c);
    bmu[0] = m4.x; bmu[1] = m4.y; bmu[2] = m4.z; bmu[3] = m4.w;
    bsc[0] = s4.x; bsc[1] = s4.y; bsc[2] = s4.z; bsc[3] = s4.w;
    bsh[0] = h4.x; bsh[1] = h4.y; bsh[2] = h4.z; bsh[3] = h4.w;
  }
  // Retire every load issued so far (weights, bias, BN vectors) before the strip loop.
  // Left pending, the waitcnt pass merges them into the loop's state and guards each
  // row's first weight use with vmcnt(0), which then also drains the prefetched rows
  // and the previous row's store -- one full HBM round trip per output row.
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  double s1[4] = {0.0, 0.0, 0.0, 0.0}, s2[4] = {0.0, 0.0, 0.0, 0.0};
  const int w = w0 + p;
  const bool wv = w < g.W;
  // BNB: the bz rows of a chunk are fetched one chunk ahead (registers), like the input rows
  RawQ zcur[CR], znext[CR];
  auto fetch_z = [&](RawQ (&zz)[CR], int rbase, bool on) {
#pragma unroll
    for (int r = 0; r < CR; ++r) {
      const bool in = on && wv && rbase + r < hend;
      const unsigned off = in ? (unsigned)((((rbase + r) * g.W + w) * g.C + c) * (int)sizeof(T))
                              : ACC_OOB;
      zz[r] = bufq_ld<0>(rb, off, (const T*)nullptr);
    }
  };
  if (BNB) fetch_z(zcur, hbeg, true);
  for (int kc = 0; kc < nch; ++kc) {
    const int r0 = hbeg + CR * kc;
    // rows r0+9 .. are needed only if the strip's last input row (hend) lies there
    const bool more = kc + 1 < nch && r0 + 9 <= hend;
    RawL nx[NL8];
    dw_fetch_rows<TCQ, NL8, AUX, T>(nx, rx, g, r0 + 9, more ? G::N8 : 0, w0, c0);
    if (BNB) fetch_z(znext, r0 + CR, kc + 1 < nch);
    const int base = (CR * kc) % G::IR;  // slot of input row r0 - 1
    float win[3][3][4];
    auto rd = [&](int j, float (&row)[3][4]) {
      int sl = base + j;
      sl = sl >= G::IR ? sl - G::IR : sl;
#pragma unroll
      for (int dx = 0; dx < 3; ++dx) {
        float4 a = tile[(sl * G::IP + p + dx) * TCQ + q];
        row[dx][0] = a.x; row[dx][1] = a.y; row[dx][2] = a.z; row[dx][3] = a.w;
      }
    };
    rd(0, win[0]);
    rd(1, win[1]);
    const int nr = min(CR, hend - r0);
    // forward statistics of this chunk's CR rows in fp32, folded into the fp64 sums once
    // per chunk (K1_CHUNK_STATS; 0 = every element straight into fp64). The fp32 sums are
    // of d = z - pv, pv = the thread's first output of the chunk (a per-thread pivot):
    // sum d^2 stays at the scale of the spread, so a channel whose mean is large against
    // its spread does not lose its variance to cancellation (the fold adds n pv^2 +
    // 2 pv sum d in fp64)
    float c1[4] = {0.f, 0.f, 0.f, 0.f}, c2[4] = {0.f, 0.f, 0.f, 0.f}, pv[4];
#pragma unroll
    for (int r = 0; r < CR; ++r) {
      // rows past the strip end (r >= nr) read stale ring slots: computed, not kept
      const bool on = wv && r < nr;
      rd(r + 2, win[2]);
      float o[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float acc = bi[j];
#pragma unroll
        for (int dy = 0; dy < 3; ++dy)
#pragma unroll
          for (int dx = 0; dx < 3; ++dx) acc = fmaf(k[dy * 3 + dx][j], win[dy][dx][j], acc);
        acc = rnd<T>(acc);  // statistics of the stored value
        o[j] = acc;
        if (r == 0) pv[j] = acc;  // (computed from finite values even when not kept)
        const float am = on ? acc : 0.f;
        if (BNB) {
          const float zz = f4get(q2f(zcur[r]), j);
          float gg = am;
          if (bact == ACT_LRELU) gg *= lrelu_d(zz * bsc[j] + bsh[j]);
          s1[j] += gg;
          s2[j] += (double)gg * ((double)zz - bmu[j]);
        } else if (K1_CHUNK_STATS) {
          const float d = on ? acc - pv[j] : 0.f;
          c1[j] += d;
          c2[j] = fmaf(d, d, c2[j]);
        } else {
          s1[j] += am;
          s2[j] += (double)am * am;
        }
      }
      const unsigned off =
          on ? (unsigned)((((r0 + r) * g.W + w) * g.C + c) * (int)sizeof(T)) : ACC_OOB;
      bufq_st<2>(rz, off, make_float4(o[0], o[1], o[2], o[3]), (T*)nullptr);
#pragma unroll
      for (int dx = 0; dx < 3; ++dx)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          win[0][dx][j] = win[1][dx][j];
          win[1][dx][j] = win[2][dx][j];
        }
    }
    if (!BNB && K1_CHUNK_STATS) {
      const double n = wv ? (double)nr : 0.0;  // elements kept in this chunk
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const double k0 = pv[j], d1 = c1[j];
        s1[j] += n * k0 + d1;
        s2[j] += (n * k0 * k0 + 2.0 * k0 * d1) + (double)c2[j];
      }
    }
    if (more) {
      __syncthreads();  // every thread is done with rows r0-1 .. r0+CR-2
      dw_park_rows<TCQ, NL8, QL>(tile, nx, g, r0 + 9, G::N8, w0, hbeg, P);
      __syncthreads();
    }
    if (BNB) {
#pragma unroll
      for (int r = 0; r < CR; ++r) zcur[r] = znext[r];
    }
  }
  if (stats) {
    __syncthreads();  // the tile is reused as the reduction buffer
    double v[8] = {s1[0], s1[1], s1[2], s1[3], s2[0], s2[1], s2[2], s2[3]};
    if (block_slot_reduce<TCQ, 8, double>(v, reinterpret_cast<double*>(tile))) {
      const long row = (long)srow * 2 * g.C;
      const int cc = c0 + 4 * threadIdx.x;  // slot = quad index q
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        stats[row + cc + j] = v[j];
        stats[row + g.C + cc + j] = v[4 + j];
      }
    }
  }
}

// ----------------------------------------------------------------------------
// K1 one-shot tiles (forward, data gradient, BN-backward data gradient). A block owns
// R output rows x TP = 256/TCQ pixels x TCQ channel quads of one image and exits after
// it: every load of the tile is issued at once, and the blocks resident on a CU at any
// moment cover neighbouring tiles (the strip kernel above walks long column strips, so
// its resident blocks are spread over the whole tensor; tools/k1lab2: one-shot tiles
// 3-4 % faster with identical z). Each thread loads ITS OWN pixel-quad column (R + 2
// rows) into registers; lanes t < 2 TCQ (R + 2) also load the two halo pixels. The
// prologue (pending BN + LeakyReLU) is applied once per element, the activated quads go
// to an LDS exchange tile, and a thread reads back only its left and right neighbours.
// Three rolling accumulators carry the output rows (an arriving input row completes
// the row above it, continues its own and starts the one below): per output the sum is
// bias, then the taps row-major, the strip kernel's FMA order, so z is bit-identical.
// Statistics: fp32 per thread over its R rows, fp64 across the block (one partial row
// per tile); BNB (data gradient, flip = 1): the BatchNorm-backward partials
// (sum g, sum g*(bz - mean)), g = out * act'(bz*scale + shift), in fp64 per element.
// Blocks are dispatched channel group fastest, then tiles in row-major image order.
// ----------------------------------------------------------------------------
// The statistics pivot of the one-shot tiles: output (row h0, pixel w0) of quad q --
// bias, then the 9 taps row-major over exchange-tile rows 0..2, pixels 0..2 (the tap
// loops' order: the value that pixel's own lane stores), rounded as stored. xb is the
// [IR][IP][TCQ] float4 tile; every lane of the quad reads the same 9 elements.
template <int TCQ, typename T>
ACC_DEV void dw_os_pivot(const float4* xb, int IP, int q, const float (&k)[9][4],
                         const float (&bi)[4], dwf2 (&pv)[2]) {
  float t[4] = {bi[0], bi[1], bi[2], bi[3]};
#pragma unroll
  for (int dy = 0; dy < 3; ++dy)
#pragma unroll
    for (int dx = 0; dx < 3; ++dx) {
      const float4 v = xb[(dy * IP + dx) * TCQ + q];
      const float vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) t[j] = fmaf(k[dy * 3 + dx][j], vv[j], t[j]);
    }
  pv[0] = dwf2{rnd<T>(t[0]), rnd<T>(t[1])};
  pv[1] = dwf2{rnd<T>(t[2]), rnd<T>(t[3])};
}

struct DwOGeom {
  int B, H, W, C;
  int tilesW, tilesH, ncg;
  int ntl;  // non-temporal input loads
  int xcd;  // channel groups of a tile on one XCD (tiles % 8 == 0): blocks 8 apart
};

template <int TCQ, int R, bool BNB, int AUX, typename T>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3)))
dw3x3_os_fwd_kernel(const T* __restrict__ x, const float* __restrict__ wt,
                    const float* __restrict__ bias, const float* __restrict__ sc,
                    const float* __restrict__ sh, int act, int flip, T* __restrict__ z,
                    double* __restrict__ stats, DwOGeom g, const T* __restrict__ bz,
                    const float* __restrict__ bst, int bact) {
  constexpr int TP = 256 / TCQ, IP = TP + 2, IR = R + 2;
  constexpr int NH = (2 * TCQ * IR + 255) / 256;  // halo loads per lane
  typedef typename QuadRaw<T>::type RawQ;
  __shared__ float4 xb[IR][IP][TCQ];
  const int tid = threadIdx.x;
  const int q = tid % TCQ, p = tid / TCQ;
  int t = (int)blockIdx.x, cg;
  if (g.xcd) {
    // workgroups are dealt round-robin over the 8 XCDs (b and b + 8 share one): the ncg
    // channel groups of a tile run 8 apart, on one XCD, so 64-B (bf16) pixel segments
    // that share a 128-B line are fetched into one L2; tiles stay in dispatch order
    const int xs = t & 7, j = t >> 3;
    cg = j % g.ncg;
    t = (j / g.ncg) * 8 + xs;
  } else {
    cg = t % g.ncg;
    t /= g.ncg;
  }
  const int srow = t;  // statistics partial row of this tile
  const int tw = t % g.tilesW;
  t /= g.tilesW;
  const int th = t % g.tilesH;
  const int b = t / g.tilesH;
  const int c0 = cg * TCQ * 4, c = c0 + 4 * q;
  const int w0 = tw * TP, w = w0 + p, h0 = th * R;
  const long img = (long)b * g.H * g.W * g.C;
  const unsigned ibytes = (unsigned)(g.H * g.W * g.C * (int)sizeof(T));
  const __amdgpu_buffer_rsrc_t rx = acc_rsrc(x + img, ibytes);
  const __amdgpu_buffer_rsrc_t rz = acc_rsrc(z + img, ibytes);
  const __amdgpu_buffer_rsrc_t rb = acc_rsrc(BNB ? bz + img : x + img, BNB ? ibytes : 0u);
  const bool pro = sc != nullptr;
  const bool win = w < g.W;
  // weights, bias, prologue and BatchNorm vectors first: in flight with the tile
  float k[9][4], bi[4];
  float4 ps = make_float4(1.f, 1.f, 1.f, 1.f), pb = make_float4(0.f, 0.f, 0.f, 0.f);
  float bmu[4] = {0.f, 0.f, 0.f, 0.f}, bsc[4] = {0.f, 0.f, 0.f, 0.f}, bsh[4] = {0.f, 0.f, 0.f, 0.f};
  {
    float wv[36];
#pragma unroll
    for (int e = 0; e < 9; ++e) {
      const float4 w4 = ld4(wt + c * 9 + 4 * e);
      wv[4 * e] = w4.x; wv[4 * e + 1] = w4.y; wv[4 * e + 2] = w4.z; wv[4 * e + 3] = w4.w;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int tp = 0; tp < 9; ++tp) k[tp][j] = wv[j * 9 + (flip ? 8 - tp : tp)];
    const float4 b4 = bias ? ld4(bias + c) : make_float4(0.f, 0.f, 0.f, 0.f);
    bi[0] = b4.x; bi[1] = b4.y; bi[2] = b4.z; bi[3] = b4.w;
    if (pro) {
      ps = ld4(sc + c);
      pb = ld4(sh + c);
    }
    if (BNB) {
      const float4 m4 = ld4(bst + BN_MEAN * g.C + c), s4 = ld4(bst + BN_SCALE * g.C + c),
                   h4 = ld4(bst + BN_SHIFT * g.C + c);
      bmu[0] = m4.x; bmu[1] = m4.y; bmu[2] = m4.z; bmu[3] = m4.w;
      bsc[0] = s4.x; bsc[1] = s4.y; bsc[2] = s4.z; bsc[3] = s4.w;
      bsh[0] = h4.x; bsh[1] = h4.y; bsh[2] = h4.z; bsh[3] = h4.w;
    }
  }
  // the whole tile: own column (R + 2 rows) and the halo pixels
  RawQ own[IR], hv[NH], zb[BNB ? R : 1];
#pragma unroll
  for (int r = 0; r < IR; ++r) {
    const int i = h0 - 1 + r;
    const bool in = win && i >= 0 && i < g.H;
    own[r] = bufq_ld<AUX>(rx, in ? (unsigned)(((i * g.W + w) * g.C + c) * (int)sizeof(T)) : ACC_OOB,
                          (const T*)nullptr);
  }
  auto halo = [&](int m, int& hr, int& hs, int& hq, int& hw, int& hi) {
    const int e = tid + 256 * m;  // halo element: (row, side, quad)
    hr = e / (2 * TCQ);
    hs = (e / TCQ) & 1;
    hq = e % TCQ;
    hw = hs ? w0 + TP : w0 - 1;
    hi = h0 - 1 + hr;
    return e < 2 * TCQ * IR && hw >= 0 && hw < g.W && hi >= 0 && hi < g.H;
  };
#pragma unroll
  for (int m = 0; m < NH; ++m) {
    int hr, hs, hq, hw, hi;
    const bool in = halo(m, hr, hs, hq, hw, hi);
    hv[m] = bufq_ld<AUX>(rx, in ? (unsigned)(((hi * g.W + hw) * g.C + c0 + 4 * hq) * (int)sizeof(T))
                                : ACC_OOB, (const T*)nullptr);
  }
  typedef dwf2 f2v;
  const DwPro P = dw_pro(ps, pb, pro, act);
  auto activate = [&](float4 a) { return dw_act(P, a); };
  auto keep = dw_keep;
  // interior tile (block-uniform): every input row and pixel of the tile is inside the
  // image and every output row is stored, so no per-element masking
  const bool interior = h0 >= 1 && h0 + R + 1 <= g.H && w0 + TP <= g.W;
  float a0[4] = {0.f, 0.f, 0.f, 0.f}, a1[4] = {0.f, 0.f, 0.f, 0.f};
  // forward statistics: fp32 sums of d = z - pv per thread, pv = the lane's own first
  // output: the squares stay at the scale of the spread (no cancellation for a channel
  // whose mean is large against its spread). At the tail the sums are re-centred on the
  // pivot of the wave's pixel-0 lane of the quad (one shuffle, after the stores; a
  // shuffle inside the tap loop, or recomputing that pivot from the tile, cost K1 ~5 %),
  // added over the wave's pixels in fp32, and the fp64 fold restores sum z, sum z^2
  f2v c1[2] = {{0.f, 0.f}, {0.f, 0.f}}, c2[2] = {{0.f, 0.f}, {0.f, 0.f}}, pv[2] = {{0.f, 0.f}, {0.f, 0.f}};
  float cnt = 0.f;
  double s1[4] = {0.0, 0.0, 0.0, 0.0}, s2[4] = {0.0, 0.0, 0.0, 0.0};
  float4 cen[IR];
  if (interior) {
#pragma unroll
    for (int r = 0; r < IR; ++r) {
      cen[r] = activate(q2f(own[r]));
      xb[r][p + 1][q] = cen[r];
    }
  } else {
#pragma unroll
    for (int r = 0; r < IR; ++r) {
      const int i = h0 - 1 + r;
      const bool in = win && i >= 0 && i < g.H;
      cen[r] = keep(in, activate(q2f(own[r])));
      xb[r][p + 1][q] = cen[r];
    }
  }
#pragma unroll
  for (int m = 0; m < NH; ++m) {
    int hr, hs, hq, hw, hi;
    const bool in = halo(m, hr, hs, hq, hw, hi);
    // (256 % TCQ == 0: a halo lane's quad hq is its own quad q, so its prologue too)
    if (tid + 256 * m < 2 * TCQ * IR) {
      xb[hr][hs ? IP - 1 : 0][hq] = keep(in, activate(q2f(hv[m])));
    }
  }
  __syncthreads();
  if (BNB) {  // the pre-BN rows, issued once the raw tile has been consumed (registers)
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int h = h0 + r;
      const bool in = win && h < g.H;
      zb[r] = bufq_ld<0>(rb, in ? (unsigned)(((h * g.W + w) * g.C + c) * (int)sizeof(T)) : ACC_OOB,
                         (const T*)nullptr);
    }
  }
  auto taps = [&](auto interior_c) {
    constexpr bool IN = decltype(interior_c)::value;
#pragma unroll
    for (int r = 0; r < IR; ++r) {
      const float4 L = xb[r][p][q], Rr = xb[r][p + 2][q];
      const float vL[4] = {L.x, L.y, L.z, L.w};
      const float vC[4] = {cen[r].x, cen[r].y, cen[r].z, cen[r].w};
      const float vR[4] = {Rr.x, Rr.y, Rr.z, Rr.w};
      const int h = h0 + r - 2;  // output row completed by input row h0 - 1 + r
      const bool on = r >= 2 && (IN || (win && h < g.H));
      float o[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float t0 = a0[j], t1 = a1[j], t2 = bi[j];
        t0 = fmaf(k[6][j], vL[j], t0); t0 = fmaf(k[7][j], vC[j], t0); t0 = fmaf(k[8][j], vR[j], t0);
        t1 = fmaf(k[3][j], vL[j], t1); t1 = fmaf(k[4][j], vC[j], t1); t1 = fmaf(k[5][j], vR[j], t1);
        t2 = fmaf(k[0][j], vL[j], t2); t2 = fmaf(k[1][j], vC[j], t2); t2 = fmaf(k[2][j], vR[j], t2);
        a0[j] = t1;
        a1[j] = t2;
        o[j] = rnd<T>(t0);  // statistics of the stored value
      }
      if (r < 2) continue;
      if (!BNB && r == 2) {  // the lane's statistics pivot: its first output (registers)
        pv[0] = f2v{o[0], o[1]};
        pv[1] = f2v{o[2], o[3]};
      }
      if (BNB) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float am = on ? o[j] : 0.f;
          const float zz = f4get(q2f(zb[r - 2]), j);
          float gg = am;
          if (bact == ACT_LRELU) gg *= lrelu_d(zz * bsc[j] + bsh[j]);
          s1[j] += gg;
          s2[j] += (double)gg * ((double)zz - bmu[j]);
        }
      } else {
        // fp32 per-thread sums on packed pairs (same adds and fmas as the scalar form)
        f2v m01 = f2v{o[0], o[1]} - pv[0], m23 = f2v{o[2], o[3]} - pv[1];
        if (!IN) {
          m01 = on ? m01 : f2v{0.f, 0.f};
          m23 = on ? m23 : f2v{0.f, 0.f};
          cnt += on ? 1.f : 0.f;
        }
        c1[0] += m01;
        c1[1] += m23;
        c2[0] = m01 * m01 + c2[0];
        c2[1] = m23 * m23 + c2[1];
      }
      bufq_st<2>(rz, on ? (unsigned)(((h * g.W + w) * g.C + c) * (int)sizeof(T)) : ACC_OOB,
                 make_float4(o[0], o[1], o[2], o[3]), (T*)nullptr);
    }
  };
  if (!BNB && interior)  // (the BN-backward form keeps one copy: registers are tight)
    taps(std::true_type{});
  else
    taps(std::false_type{});
  if (stats && !BNB) {
    // forward statistics: the fp32 per-thread sums (R rows) are added over the wave's
    // pixels in fp32 (shuffles), then over the 4 waves in fp64 through a small slab of
    // its own -- no barrier before it, the exchange tile stays untouched (tools/k1lab2:
    // 2-3 us of K1's 150 against the block reduction through the tile)
    constexpr int WL = TCQ < 64 ? TCQ : 64;
    __shared__ double sw[4][WL][8];
    // re-centre on the quad's common pivot kc (lane q): sum (z - kc) = sum d + n dl,
    // sum (z - kc)^2 = sum d^2 + dl (2 sum d + n dl), dl = pv - kc (fp32, small)
    const float nl = interior ? (float)R : cnt;
    f2v kc[2];
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      kc[e].x = __shfl(pv[e].x, q, 64);
      kc[e].y = __shfl(pv[e].y, q, 64);
      const f2v dl = pv[e] - kc[e];
      c2[e] = dl * (c1[e] * 2.f + dl * nl) + c2[e];
      c1[e] = dl * nl + c1[e];
    }
    float f[9] = {c1[0].x, c1[0].y, c1[1].x, c1[1].y, c2[0].x, c2[0].y, c2[1].x, c2[1].y, cnt};
#pragma unroll
    for (int off = TCQ; off < 64; off <<= 1)
#pragma unroll
      for (int e = 0; e < 8; ++e) f[e] += __shfl_xor(f[e], off);
    if (!interior) {  // (block-uniform) the kept-element count of the wave's lanes
#pragma unroll
      for (int off = TCQ; off < 64; off <<= 1) f[8] += __shfl_xor(f[8], off);
    }
    const int lane = tid & 63, wave = tid >> 6;
    if (lane < WL) {
      const double n = interior ? (double)(R * (64 / WL)) : (double)f[8];
      const float k0[4] = {kc[0].x, kc[0].y, kc[1].x, kc[1].y};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const double kk = k0[j], d1 = f[j];
        sw[wave][lane][j] = n * kk + d1;
        sw[wave][lane][4 + j] = (n * kk * kk + 2.0 * kk * d1) + (double)f[4 + j];
      }
    }
    __syncthreads();
    if (tid < TCQ) {  // (TCQ <= 64: every wave holds every quad)
      const long row = (long)srow * 2 * g.C;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const double v = ((sw[0][tid][e] + sw[1][tid][e]) + sw[2][tid][e]) + sw[3][tid][e];
        stats[row + (e >> 2) * g.C + c0 + 4 * tid + (e & 3)] = v;
      }
    }
    return;
  }
  if (stats) {
    __syncthreads();  // the exchange tile is reused as the reduction buffer
    double v[8] = {s1[0], s1[1], s1[2], s1[3], s2[0], s2[1], s2[2], s2[3]};
    if (block_slot_reduce<TCQ, 8, double>(v, reinterpret_cast<double*>(&xb[0][0][0]))) {
      const long row = (long)srow * 2 * g.C;
      const int cc = c0 + 4 * threadIdx.x;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        stats[row + cc + j] = v[j];
        stats[row + g.C + cc + j] = v[4 + j];
      }
    }
  }
}

// ----------------------------------------------------------------------------
// K1 one-shot tiles of 16 rows (fp32 forward / plain data gradient; no BN-backward
// form). A 512-thread block owns 16 output rows x TP pixels x TCQ quads as two halves of
// 256 threads with 8 output rows each: every input row of the tile (18 with the halo) is
// fetched once -- each half loads its own 9 rows, the rows the halves share cross through
// the LDS exchange tile -- so a tile re-fetches 2 of 18 input rows from its neighbours'
// fetches instead of 2 of 10, and the statistics tail (shuffles, the cross-wave slab, one
// partial row) is paid once per 16 rows. The centre column comes from LDS too (no
// register copy), so a thread stays within 128 VGPRs: 2 blocks = 4 waves per SIMD in
// 2 x 78 KB of LDS. Per output the sum is bias, then the taps row-major: z bit-identical
// to the 8-row tiles and the strip kernel.
// ----------------------------------------------------------------------------
template <int TCQ, typename T>
__global__ void __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4)))
dw3x3_os16_fwd_kernel(const T* __restrict__ x, const float* __restrict__ wt,
                      const float* __restrict__ bias, const float* __restrict__ sc,
                      const float* __restrict__ sh, int act, int flip, T* __restrict__ z,
                      double* __restrict__ stats, DwOGeom g) {
  constexpr int R = 8, HR = R + 1;  // output rows / own input rows per half
  constexpr int TP = 256 / TCQ, IP = TP + 2, IR = 2 * R + 2;
  constexpr int NH = (2 * TCQ * IR + 511) / 512;  // halo loads per lane
  typedef typename QuadRaw<T>::type RawQ;
  __shared__ float4 xb[IR][IP][TCQ];
  const int tid = threadIdx.x, half = tid >> 8, ht = tid & 255;
  const int q = ht % TCQ, p = ht / TCQ;
  int t = (int)blockIdx.x;
  const int cg = t % g.ncg;
  t /= g.ncg;
  const int srow = t;  // statistics partial row of this tile
  const int tw = t % g.tilesW;
  t /= g.tilesW;
  const int th = t % g.tilesH;
  const int b = t / g.tilesH;
  const int c0 = cg * TCQ * 4, c = c0 + 4 * q;
  const int w0 = tw * TP, w = w0 + p, h0 = th * 2 * R;
  const long img = (long)b * g.H * g.W * g.C;
  const unsigned ibytes = (unsigned)(g.H * g.W * g.C * (int)sizeof(T));
  const __amdgpu_buffer_rsrc_t rx = acc_rsrc(x + img, ibytes);
  const __amdgpu_buffer_rsrc_t rz = acc_rsrc(z + img, ibytes);
  const bool pro = sc != nullptr;
  const bool win = w < g.W;
  // this half's own column: input rows h0 - 1 + half*HR + r (LDS rows half*HR + r)
  RawQ own[HR], hv[NH];
#pragma unroll
  for (int r = 0; r < HR; ++r) {
    const int i = h0 - 1 + half * HR + r;
    const bool in = win && i >= 0 && i < g.H;
    own[r] = bufq_ld<0>(rx, in ? (unsigned)(((i * g.W + w) * g.C + c) * (int)sizeof(T)) : ACC_OOB,
                        (const T*)nullptr);
  }
  auto halo = [&](int m, int& hr, int& hs, int& hq, int& hw, int& hi) {
    const int e = tid + 512 * m;  // halo element: (row, side, quad)
    hr = e / (2 * TCQ);
    hs = (e / TCQ) & 1;
    hq = e % TCQ;
    hw = hs ? w0 + TP : w0 - 1;
    hi = h0 - 1 + hr;
    return e < 2 * TCQ * IR && hw >= 0 && hw < g.W && hi >= 0 && hi < g.H;
  };
#pragma unroll
  for (int m = 0; m < NH; ++m) {
    int hr, hs, hq, hw, hi;
    const bool in = halo(m, hr, hs, hq, hw, hi);
    hv[m] = bufq_ld<0>(rx, in ? (unsigned)(((hi * g.W + hw) * g.C + c0 + 4 * hq) * (int)sizeof(T))
                              : ACC_OOB, (const T*)nullptr);
  }
  float4 ps = make_float4(1.f, 1.f, 1.f, 1.f), pb = make_float4(0.f, 0.f, 0.f, 0.f);
  if (pro) {
    ps = ld4(sc + c);
    pb = ld4(sh + c);
  }
  const DwPro P = dw_pro(ps, pb, pro, act);
  const bool interior = h0 >= 1 && h0 + 2 * R + 1 <= g.H && w0 + TP <= g.W;
  if (interior) {
#pragma unroll
    for (int r = 0; r < HR; ++r) xb[half * HR + r][p + 1][q] = dw_act(P, q2f(own[r]));
  } else {
#pragma unroll
    for (int r = 0; r < HR; ++r) {
      const int i = h0 - 1 + half * HR + r;
      xb[half * HR + r][p + 1][q] = dw_keep(win && i >= 0 && i < g.H, dw_act(P, q2f(own[r])));
    }
  }
#pragma unroll
  for (int m = 0; m < NH; ++m) {
    int hr, hs, hq, hw, hi;
    const bool in = halo(m, hr, hs, hq, hw, hi);
    // (512 % TCQ == 0: a halo lane's quad hq is its own quad q, so its prologue too)
    if (tid + 512 * m < 2 * TCQ * IR) xb[hr][hs ? IP - 1 : 0][hq] = dw_keep(in, dw_act(P, q2f(hv[m])));
  }
  // weights and bias (needed from the taps on; loaded behind the tile's stores)
  float k[9][4], bi[4];
  {
    float wv[36];
#pragma unroll
    for (int e = 0; e < 9; ++e) {
      const float4 w4 = ld4(wt + c * 9 + 4 * e);
      wv[4 * e] = w4.x; wv[4 * e + 1] = w4.y; wv[4 * e + 2] = w4.z; wv[4 * e + 3] = w4.w;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int tp = 0; tp < 9; ++tp) k[tp][j] = wv[j * 9 + (flip ? 8 - tp : tp)];
    const float4 b4 = bias ? ld4(bias + c) : make_float4(0.f, 0.f, 0.f, 0.f);
    bi[0] = b4.x; bi[1] = b4.y; bi[2] = b4.z; bi[3] = b4.w;
  }
  __syncthreads();
  typedef dwf2 f2v;
  float a0[4] = {0.f, 0.f, 0.f, 0.f}, a1[4] = {0.f, 0.f, 0.f, 0.f};
  // statistics as in dw3x3_os_fwd_kernel: fp32 sums of z - pv (pv block-uniform per quad)
  f2v c1[2] = {{0.f, 0.f}, {0.f, 0.f}}, c2[2] = {{0.f, 0.f}, {0.f, 0.f}}, pv[2];
  dw_os_pivot<TCQ, T>(&xb[0][0][0], IP, q, k, bi, pv);
  float cnt = 0.f;
  auto taps = [&](auto interior_c) {
    constexpr bool IN = decltype(interior_c)::value;
    auto row = [&](int j, float (&o)[4]) {
      const int lr = half * R + j;  // LDS row of input row h0 - 1 + lr
      const float4 L = xb[lr][p][q], Cm = xb[lr][p + 1][q], Rr = xb[lr][p + 2][q];
      const float vL[4] = {L.x, L.y, L.z, L.w};
      const float vC[4] = {Cm.x, Cm.y, Cm.z, Cm.w};
      const float vR[4] = {Rr.x, Rr.y, Rr.z, Rr.w};
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        float t0 = a0[jj], t1 = a1[jj], t2 = bi[jj];
        t0 = fmaf(k[6][jj], vL[jj], t0); t0 = fmaf(k[7][jj], vC[jj], t0); t0 = fmaf(k[8][jj], vR[jj], t0);
        t1 = fmaf(k[3][jj], vL[jj], t1); t1 = fmaf(k[4][jj], vC[jj], t1); t1 = fmaf(k[5][jj], vR[jj], t1);
        t2 = fmaf(k[0][jj], vL[jj], t2); t2 = fmaf(k[1][jj], vC[jj], t2); t2 = fmaf(k[2][jj], vR[jj], t2);
        a0[jj] = t1;
        a1[jj] = t2;
        o[jj] = rnd<T>(t0);  // statistics of the stored value
      }
    };
    float o[4];
    row(0, o);  // the first two input rows only start outputs
    row(1, o);
    // (rolled: an unrolled loop hoists the LDS reads of every row and spills at 128 VGPRs)
#pragma unroll 2
    for (int j = 2; j < R + 2; ++j) {
      row(j, o);
      const int h = h0 + half * R + j - 2;  // output row completed by this input row
      const bool on = IN || (win && h < g.H);
      f2v m01 = f2v{o[0], o[1]} - pv[0], m23 = f2v{o[2], o[3]} - pv[1];
      if (!IN) {
        m01 = on ? m01 : f2v{0.f, 0.f};
        m23 = on ? m23 : f2v{0.f, 0.f};
        cnt += on ? 1.f : 0.f;
      }
      c1[0] += m01;
      c1[1] += m23;
      c2[0] = m01 * m01 + c2[0];
      c2[1] = m23 * m23 + c2[1];
      bufq_st<2>(rz, on ? (unsigned)(((h * g.W + w) * g.C + c) * (int)sizeof(T)) : ACC_OOB,
                 make_float4(o[0], o[1], o[2], o[3]), (T*)nullptr);
    }
  };
  if (interior)
    taps(std::true_type{});
  else
    taps(std::false_type{});
  if (!stats) return;
  constexpr int WL = TCQ < 64 ? TCQ : 64;
  if (interior) cnt = (float)R;
  float f[9] = {c1[0].x, c1[0].y, c1[1].x, c1[1].y, c2[0].x, c2[0].y, c2[1].x, c2[1].y, cnt};
#pragma unroll
  for (int off = TCQ; off < 64; off <<= 1)
#pragma unroll
    for (int e = 0; e < 9; ++e) f[e] += __shfl_xor(f[e], off);
  __syncthreads();  // the exchange tile is reused as the 8-wave slab
  double* sw = reinterpret_cast<double*>(&xb[0][0][0]);  // [8 waves][WL][8]
  const int lane = tid & 63, wave = tid >> 6;
  if (lane < WL) {
    const double n = f[8];
    const float k0[4] = {pv[0].x, pv[0].y, pv[1].x, pv[1].y};
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      const double kk = k0[jj], d1 = f[jj];
      sw[(wave * WL + lane) * 8 + jj] = n * kk + d1;
      sw[(wave * WL + lane) * 8 + 4 + jj] = (n * kk * kk + 2.0 * kk * d1) + (double)f[4 + jj];
    }
  }
  __syncthreads();
  if (tid < TCQ) {  // (TCQ <= 64: every wave holds every quad)
    const long row = (long)srow * 2 * g.C;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      double v = 0.0;
#pragma unroll
      for (int wv = 0; wv < 8; ++wv) v += sw[(wv * WL + tid) * 8 + e];
      stats[row + (e >> 2) * g.C + c0 + 4 * tid + (e & 3)] = v;
    }
  }
}

template <int TCQ, typename T>
__global__ void __launch_bounds__(256)
dw3x3_tile_wgrad_kernel(const T* __restrict__ x, const T* __restrict__ dz,
                        const float* __restrict__ sc, const float* __restrict__ sh, int act,
                        float* __restrict__ part, DwTGeom g) {
  typedef DwT<TCQ> G;
  __shared__ float4 tile[G::N4 > 1024 ? G::N4 : 1024];
  const int tid = threadIdx.x;
  const int q = tid % TCQ, p = tid / TCQ;
  const int c0 = blockIdx.y * TCQ * 4;
  const int c = c0 + 4 * q;
  int t = dw_tile_id(g);
  const int tw = t % g.tilesW;
  t /= g.tilesW;
  const int th = t % g.tilesH;
  const int b = t / g.tilesH;
  const int h0 = th * DW_TR, w0 = tw * G::TP;
  const int w = w0 + p;
  const int nr = min(DW_TR, g.H - h0);
  // this thread's dz column (independent raw loads issued before the tile fill; rows
  // outside the image read dz's origin and are zeroed when widened)
  typename QuadRaw<T>::type dr[DW_TR];
#pragma unroll
  for (int r = 0; r < DW_TR; ++r) {
    const bool ok = w < g.W && r < nr;
    dr[r] = ldq_raw(ok ? dz + (((long)b * g.H + h0 + r) * g.W + w) * g.C + c : dz, false);
  }
  dw_fill_tile<TCQ>(tile, x, sc, sh, act, g, b, h0, w0, c0);
  __syncthreads();
  float4 d[DW_TR];
#pragma unroll
  for (int r = 0; r < DW_TR; ++r)
    d[r] = (w < g.W && r < nr) ? q2f(dr[r]) : make_float4(0.f, 0.f, 0.f, 0.f);
  float acc[10][4];
#pragma unroll
  for (int i = 0; i < 10; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = 0.f;
  if (w < g.W) {
    float win[3][3][4];
    auto rd = [&](int r, float (&row)[3][4]) {
#pragma unroll
      for (int dx = 0; dx < 3; ++dx) {
        float4 a = tile[(r * G::IP + p + dx) * TCQ + q];
        row[dx][0] = a.x; row[dx][1] = a.y; row[dx][2] = a.z; row[dx][3] = a.w;
      }
    };
    rd(0, win[0]);
    rd(1, win[1]);
#pragma unroll
    for (int r = 0; r < DW_TR; ++r) {
      if (r < nr) {
        rd(r + 2, win[2]);
        const float dv[4] = {d[r].x, d[r].y, d[r].z, d[r].w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
#pragma unroll
          for (int dy = 0; dy < 3; ++dy)
#pragma unroll
            for (int dx = 0; dx < 3; ++dx)
              acc[dy * 3 + dx][j] = fmaf(dv[j], win[dy][dx][j], acc[dy * 3 + dx][j]);
          acc[9][j] += dv[j];
        }
#pragma unroll
        for (int dx = 0; dx < 3; ++dx)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            win[0][dx][j] = win[1][dx][j];
            win[1][dx][j] = win[2][dx][j];
          }
      }
    }
  }
  __syncthreads();  // the tile is reused as the reduction buffer
  float v[40];
#pragma unroll
  for (int i = 0; i < 10; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) v[i * 4 + j] = acc[i][j];
  if (block_slot_reduce<TCQ, 40, float>(v, reinterpret_cast<float*>(tile))) {
    const int cc = c0 + 4 * threadIdx.x;
#pragma unroll
    for (int i = 0; i < 10; ++i)
      st4(part + ((long)blockIdx.x * 10 + i) * g.C + cc,
          make_float4(v[i * 4], v[i * 4 + 1], v[i * 4 + 2], v[i * 4 + 3]));
  }
}

// ----------------------------------------------------------------------------
// Span kernel (CQ = C/4 quads per pixel, CQ even and <= 64: every HANC width up to
// 256 channels). A block owns R output rows x PX = NT/CQ whole pixels of one image, so
// each row of its input tile -- pixels w0-1 .. w0+PX, every channel -- is ONE
// contiguous (PX+2)*C-element segment of the NHWC row. Non-persistent: the whole
// (R+2)-row halo tile is fetched with every load in flight (branch-free buffer loads,
// out-of-image quads masked by the descriptor range), activated (prologue BN+act) into
// LDS, and each of the PX*CQ compute lanes slides its 3x3 window down its pixel-quad
// column. tools/k1lab (16x256x256x96 fp32, copies of K1's bytes without arithmetic):
// whole-pixel spans stream at 78 % of HBM peak, the 32-pixel x 32-channel tiles of
// the kernel above at 73 % (70 % through an LDS halo tile) and its persistent strip
// pipeline at 66 %.
// ----------------------------------------------------------------------------
struct DwSGeom {
  int B, H, W, C;
  int CQ, PX;      // quads per pixel, output pixels per span (NT / CQ)
  int NS, tilesH;  // spans per image row, row bands (of nrt R-row tiles) per image
  int nrt;         // R-row tiles per block, walked in order
  int remap;       // XCD-contiguous block order (tuning knob ACCUNET_DW_SPAN_REMAP)
};

#define DWS_R 8  // output rows per span block

// workgroup barrier for LDS reuse only: drains this wave's LDS operations
// (lgkmcnt(0)), leaves its global loads / stores in flight (no fence)
ACC_DEV void lds_barrier() {
  __builtin_amdgcn_s_waitcnt(0xc07f);  // gfx9: vmcnt 63, expcnt 7, lgkmcnt 0
  __builtin_amdgcn_s_barrier();
}

template <int NT>
struct DwS {
  static constexpr int R = DWS_R;
  static constexpr int RWMAX = NT + 2 * (NT == 256 ? 32 : 64);  // (PX+2)*CQ, CQ <= NT/8
  static constexpr int TILE = (R + 2) * RWMAX;                   // float4 slots
  // 16-byte fill loads per lane: (R+2)*(PX+2)*CQ quads over PX*CQ lanes, PX >= 8
  static constexpr int NLMAX = ((R + 2) * 10 + 7) / 8;
};

// Span-tile fill, split in two so independent work can sit between the loads and
// their use: dws_issue fetches the (R+2)-row halo tile of rows h0-1 .. h0+R, pixels
// w0-1 .. w0+PX (units of QL quads, fill lane f < NA/QL taking units f, f + NA/QL, ...:
// a stride that is a multiple of CQ/QL, so a lane always stages the same QL quads),
// out-of-image units masked by the descriptor range; dws_park activates them
// (prologue BN+act, in-image only) into the LDS tile [R+2][RW] and zero-fills the rest.
template <int NT, int AUX, typename T>
struct DwsFill {
  static constexpr int QL = Raw16<T>::QL;
  typedef typename Raw16<T>::type RawL;
  RawL v[DwS<NT>::NLMAX];
  unsigned inb;
  float4 ps[QL], pb[QL];
  ACC_DEV void issue(__amdgpu_buffer_rsrc_t rx, const DwSGeom& g, int h0, int s0,
                     const float* sc, const float* sh) {
    constexpr int R = DwS<NT>::R;
    // (tid laundered through an empty asm: inside a caller's loop the per-unit index
    // math is then recomputed per call instead of hoisted and kept live in registers)
    int tid = threadIdx.x;
    asm volatile("" : "+v"(tid));
    const int CQ = g.CQ, RW = (g.PX + 2) * CQ, NF = g.PX * CQ / QL;
    const int nunits = (R + 2) * RW / QL, L = g.W * CQ;
    const int qf = (tid * QL) % CQ;
#pragma unroll
    for (int j = 0; j < QL; ++j) {
      ps[j] = sc ? ld4(sc + 4 * (qf + j)) : make_float4(1.f, 1.f, 1.f, 1.f);
      pb[j] = sc ? ld4(sh + 4 * (qf + j)) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    inb = 0;
    // unit k sits at tile quad i = (tid + NF k) QL = row r, column jq; NF QL = PX CQ < RW, so
    // each step advances jq by PX CQ and wraps into the next row at most once
    int r = (tid * QL) / RW, jq = tid * QL - r * RW;
#pragma unroll
    for (int k = 0; k < DwS<NT>::NLMAX; ++k) {
      const int u = tid + NF * k;
      const int hh = h0 - 1 + r, pos = s0 - CQ + jq;
      const bool in = tid < NF && u < nunits && hh >= 0 && hh < g.H && pos >= 0 && pos < L;
      inb |= (in ? 1u : 0u) << k;
      v[k] = buf16_ld<AUX>(rx, in ? (unsigned)((hh * L + pos) * 4 * (int)sizeof(T)) : ACC_OOB,
                           (const T*)nullptr);
      jq += NF * QL;
      const bool wrap = jq >= RW;
      jq -= wrap ? RW : 0;
      r += wrap ? 1 : 0;
    }
  }
  ACC_DEV void park(float4* __restrict__ tile, const DwSGeom& g, bool pro, int act) const {
    constexpr int R = DwS<NT>::R;
    int tid = threadIdx.x;
    asm volatile("" : "+v"(tid));
    const int RW = (g.PX + 2) * g.CQ, NF = g.PX * g.CQ / QL;
    const int nunits = (R + 2) * RW / QL;
    DwPro P[QL];
#pragma unroll
    for (int j = 0; j < QL; ++j) P[j] = dw_pro(ps[j], pb[j], pro, act);
#pragma unroll
    for (int k = 0; k < DwS<NT>::NLMAX; ++k) {
      const int u = tid + NF * k;
      if (tid < NF && u < nunits) {
        const bool in = (inb >> k) & 1u;
#pragma unroll
        for (int j = 0; j < QL; ++j) tile[u * QL + j] = dw_keep(in, dw_act(P[j], r16q(v[k], j)));
      }
    }
  }
};

template <int NT, bool BNB, int AUX, typename T>
__global__ void __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(BNB || NT == 512 ? 2 : 3)))
dw3x3_span_fwd_kernel(const T* __restrict__ x, const float* __restrict__ wt,
                      const float* __restrict__ bias, const float* __restrict__ sc,
                      const float* __restrict__ sh, int act, int flip, T* __restrict__ z,
                      double* __restrict__ stats, DwSGeom g, const T* __restrict__ bz,
                      const float* __restrict__ bst, int bact) {
  typedef DwS<NT> G;
  constexpr int R = G::R;
  typedef typename QuadRaw<T>::type RawQ;
  __shared__ float4 tile[G::TILE];
  const int tid = threadIdx.x;
  const int CQ = g.CQ, PX = g.PX;
  const int RW = (PX + 2) * CQ, NA = PX * CQ;
  int bid = blockIdx.x;
  if (g.remap) {
    const int per = gridDim.x >> 3;
    bid = (bid & 7) * per + (bid >> 3);
  }
  const int sp = bid % g.NS;
  int t = bid / g.NS;
  const int tb = t % g.tilesH;  // row band: tiles tb*nrt .. tb*nrt + nrt - 1 of R rows
  const int b = t / g.tilesH;
  const int w0 = sp * PX;
  const int L = g.W * CQ;  // quads per image row
  const int s0 = w0 * CQ;  // first output quad of the span in its row
  const long img = (long)b * g.H * g.W * g.C;
  const unsigned ibytes = (unsigned)(g.H * g.W * g.C * (int)sizeof(T));
  const __amdgpu_buffer_rsrc_t rx = acc_rsrc(x + img, ibytes);
  const __amdgpu_buffer_rsrc_t rz = acc_rsrc(z + img, ibytes);
  const __amdgpu_buffer_rsrc_t rb = acc_rsrc(BNB ? bz + img : x + img, BNB ? ibytes : 0u);
  constexpr unsigned QB = 4 * sizeof(T);  // bytes per quad

  // compute lane: pixel p of the span, quad q
  const int p = tid / CQ, q = tid - (tid / CQ) * CQ;
  const bool lane_on = tid < NA && w0 + p < g.W;
  const int c = 4 * q;

  const bool pro = sc != nullptr;
  // the lane's 4 channels x 9 taps are 36 contiguous floats of wt ([C][9], 16-B aligned
  // since c % 4 == 0): 9 float4 loads instead of 36 scalar ones
  float k9[9][4], bi[4];
  float bmu[4] = {0.f, 0.f, 0.f, 0.f}, bsc[4] = {0.f, 0.f, 0.f, 0.f}, bsh[4] = {0.f, 0.f, 0.f, 0.f};
  const int cc = tid < NA ? c : 0;
  {
    float wv[36];
#pragma unroll
    for (int e = 0; e < 9; ++e) {
      const float4 w4 = ld4(wt + cc * 9 + 4 * e);
      wv[4 * e] = w4.x; wv[4 * e + 1] = w4.y; wv[4 * e + 2] = w4.z; wv[4 * e + 3] = w4.w;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int tp = 0; tp < 9; ++tp) k9[tp][j] = wv[j * 9 + (flip ? 8 - tp : tp)];
    const float4 b4 = bias ? ld4(bias + cc) : make_float4(0.f, 0.f, 0.f, 0.f);
    bi[0] = b4.x; bi[1] = b4.y; bi[2] = b4.z; bi[3] = b4.w;
    if (BNB) {
      const float4 m4 = ld4(bst + BN_MEAN * g.C + cc), s4 = ld4(bst + BN_SCALE * g.C + cc),
                   h4 = ld4(bst + BN_SHIFT * g.C + cc);
      bmu[0] = m4.x; bmu[1] = m4.y; bmu[2] = m4.z; bmu[3] = m4.w;
      bsc[0] = s4.x; bsc[1] = s4.y; bsc[2] = s4.z; bsc[3] = s4.w;
      bsh[0] = h4.x; bsh[1] = h4.y; bsh[2] = h4.z; bsh[3] = h4.w;
    }
  }
  double s1[4] = {0.0, 0.0, 0.0, 0.0}, s2[4] = {0.0, 0.0, 0.0, 0.0};
  for (int it = 0; it < g.nrt; ++it) {
    const int h0 = (tb * g.nrt + it) * R;
    if (h0 >= g.H) break;  // block-uniform
    // BNB: this lane's R rows of bz, in flight with the tile fill
    RawQ zr[R];
    if (BNB) {
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const bool in = lane_on && h0 + r < g.H;
        zr[r] = bufq_ld<0>(rb, in ? (unsigned)(((h0 + r) * L + s0 + tid) * QB) : ACC_OOB,
                           (const T*)nullptr);
      }
    }
    {
      DwsFill<NT, AUX, T> fill;
      fill.issue(rx, g, h0, s0, sc, sh);
      if (it > 0) lds_barrier();  // every lane is done with the previous tile
      fill.park(tile, g, pro, act);
    }
    lds_barrier();
    if (tid < NA) {
      // (the lane's tile base laundered per tile: the 30 window addresses are then
      // recomputed per tile instead of hoisted out of the tile loop into registers)
      int base = p * CQ + q;
      asm volatile("" : "+v"(base));
      float win[3][3][4];
      auto rd = [&](int r, float (&row)[3][4]) {
#pragma unroll
        for (int dx = 0; dx < 3; ++dx) {
          const float4 a = tile[r * RW + base + dx * CQ];
          row[dx][0] = a.x; row[dx][1] = a.y; row[dx][2] = a.z; row[dx][3] = a.w;
        }
      };
      rd(0, win[0]);
      rd(1, win[1]);
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const bool on = lane_on && h0 + r < g.H;
        rd(r + 2, win[2]);
        float o[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          float acc = bi[j];
#pragma unroll
          for (int dy = 0; dy < 3; ++dy)
#pragma unroll
            for (int dx = 0; dx < 3; ++dx) acc = fmaf(k9[dy * 3 + dx][j], win[dy][dx][j], acc);
          acc = rnd<T>(acc);  // statistics of the stored value
          o[j] = acc;
          const float am = on ? acc : 0.f;
          if (BNB) {
            const float zz = f4get(q2f(zr[r]), j);
            float gg = am;
            if (bact == ACT_LRELU) gg *= lrelu_d(zz * bsc[j] + bsh[j]);
            s1[j] += gg;
            s2[j] += (double)gg * ((double)zz - bmu[j]);
          } else {
            s1[j] += am;
            s2[j] += (double)am * am;
          }
        }
        bufq_st<2>(rz, on ? (unsigned)(((h0 + r) * L + s0 + tid) * QB) : ACC_OOB,
                   make_float4(o[0], o[1], o[2], o[3]), (T*)nullptr);
#pragma unroll
        for (int dx = 0; dx < 3; ++dx)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            win[0][dx][j] = win[1][dx][j];
            win[1][dx][j] = win[2][dx][j];
          }
      }
    }
  }
  if (stats) {
    // per-channel sums over the span's PX pixels, in pixel order (deterministic). LDS-only
    // barriers: __syncthreads' release fence would make every wave wait for its z stores
    // to complete (vmcnt(0)) before the reduction, once per 8-row block
    lds_barrier();  // the tile is reused as the reduction buffer
    double* red = reinterpret_cast<double*>(tile);  // [8][NA]: lane-contiguous, no conflicts
    if (tid < NA) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        red[j * NA + tid] = s1[j];
        red[(4 + j) * NA + tid] = s2[j];
      }
    }
    lds_barrier();
    if (tid < CQ) {
      double a[8] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
      for (int pp = 0; pp < PX; ++pp)
#pragma unroll
        for (int e = 0; e < 8; ++e) a[e] += red[e * NA + pp * CQ + tid];
      const long row = (long)bid * 2 * g.C;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        stats[row + 4 * tid + j] = a[j];
        stats[row + g.C + 4 * tid + j] = a[4 + j];
      }
    }
  }
}

// ACCUNET_DW_SPAN (tuning knob): which depthwise passes run the span kernels.
// bit 0: weight gradient (default on: 16x256x256x96 fp32 169-171 us against the tile
// kernel's 180 us), bit 1: forward / data gradient (default off: with the statistics
// epilogue 178-198 us against 161 us; its halo tile re-reads neighbours' pixels from
// other XCDs, tools/k1lab span_lds 65-68 % vs tile_lds 70 %)
static int dw_span_on() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("ACCUNET_DW_SPAN");
    v = e ? atoi(e) : 1;
  }
  return v;
}

// span-kernel threads per block for C, or 0 when the span kernel does not apply to
// pass `bit` (1 = weight gradient, 2 = forward)
static int dw_span_nt(int H, int W, int C, int bit = 2) {
  if (!(dw_span_on() & bit) || C % 8) return 0;  // CQ even (bf16 fill units are quad pairs)
  if ((long)H * W * C * 4 >= (1L << 31)) return 0;
  const int CQ = C / 4;
  // the weight gradient runs 256-thread spans (CQ <= 32) only; 512-thread blocks (CQ
  // 33..64) hold 102 KB of LDS, one block per CU, and run only for the forward knob
  if (bit == 1) return CQ <= 32 ? 256 : 0;
  return CQ <= 32 ? 256 : (CQ <= 64 ? 512 : 0);
}

static DwSGeom dw_sgeom(int B, int H, int W, int C, int nt, dim3* grid) {
  DwSGeom g;
  g.B = B; g.H = H; g.W = W; g.C = C;
  g.CQ = C / 4;
  g.PX = nt / g.CQ;
  g.NS = ceil_div(W, g.PX);
  static const char* nr = getenv("ACCUNET_DW_SPAN_NRT");  // tuning knob: tiles per block
  g.nrt = nr && atoi(nr) > 0 ? atoi(nr) : 1;
  g.tilesH = ceil_div(ceil_div(H, DWS_R), g.nrt);
  static const char* rm = getenv("ACCUNET_DW_SPAN_REMAP");  // tuning knob
  const long nb = (long)B * g.tilesH * g.NS;
  g.remap = (rm && atoi(rm) && nb % 8 == 0) ? 1 : 0;
  *grid = dim3((unsigned)nb);
  return g;
}


// Weight + bias gradient in span geometry: dW[c][tap] = sum_p dz[p,c] * a[shift_tap(p), c],
// db[c] = sum_p dz[p,c]. A block walks `nrt` consecutive R-row tiles of one span (fill,
// then the R dz rows of its lanes, window sums in registers), then reduces its lanes'
// 10 x 4 sums over the span's pixels (pixel order, deterministic) into partial row bid
// of part[rows][10][C].
template <int NT, int AUX, typename T>
__global__ void __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(NT == 256 ? 3 : 2)))
dw3x3_span_wgrad_kernel(const T* __restrict__ x, const T* __restrict__ dz,
                        const float* __restrict__ sc, const float* __restrict__ sh, int act,
                        float* __restrict__ part, DwSGeom g) {
  const int nrt = g.nrt;
  typedef DwS<NT> G;
  constexpr int R = G::R;
  typedef typename QuadRaw<T>::type RawQ;
  __shared__ float4 tile[G::TILE];
  const int tid = threadIdx.x;
  const int CQ = g.CQ, PX = g.PX;
  const int RW = (PX + 2) * CQ, NA = PX * CQ;
  const int bid = blockIdx.x;
  const int sp = bid % g.NS;
  int t = bid / g.NS;
  const int tb = t % g.tilesH;  // tile band: row tiles tb*nrt .. tb*nrt + nrt - 1
  const int b = t / g.tilesH;
  const int w0 = sp * PX;
  const int L = g.W * CQ;
  const int s0 = w0 * CQ;
  const long img = (long)b * g.H * g.W * g.C;
  const unsigned ibytes = (unsigned)(g.H * g.W * g.C * (int)sizeof(T));
  const __amdgpu_buffer_rsrc_t rx = acc_rsrc(x + img, ibytes);
  const __amdgpu_buffer_rsrc_t rd_ = acc_rsrc(dz + img, ibytes);
  constexpr unsigned QB = 4 * sizeof(T);
  const int p = tid / CQ, q = tid - (tid / CQ) * CQ;
  const bool lane_on = tid < NA && w0 + p < g.W;
  const bool pro = sc != nullptr;
  float acc[10][4];
#pragma unroll
  for (int i = 0; i < 10; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = 0.f;
  for (int it = 0; it < nrt; ++it) {
    const int h0 = (tb * nrt + it) * R;
    if (h0 >= g.H) break;  // block-uniform
    RawQ dr[R];
    auto issue_dz = [&]() {
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const bool in = lane_on && h0 + r < g.H;
        dr[r] = bufq_ld<0>(rd_, in ? (unsigned)(((h0 + r) * L + s0 + tid) * QB) : ACC_OOB,
                           (const T*)nullptr);
      }
    };
    {
      DwsFill<NT, AUX, T> fill;
      fill.issue(rx, g, h0, s0, sc, sh);
      // bf16: the dz rows (8 B per lane and row) fit beside the fill registers, so they
      // are issued with the tile and one memory round trip covers both
      if constexpr (sizeof(T) == 2) issue_dz();
      if (it > 0) __syncthreads();  // every lane is done with the previous tile
      fill.park(tile, g, pro, act);
    }
    __builtin_amdgcn_sched_barrier(0);  // keep the fp32 dz loads behind the park (registers)
    // fp32: this lane's dz rows, issued once the fill registers are free (in flight
    // across the barrier)
    if constexpr (sizeof(T) != 2) issue_dz();
    __syncthreads();
    if (tid < NA) {
      float win[3][3][4];
      auto rd = [&](int r, float (&row)[3][4]) {
#pragma unroll
        for (int dx = 0; dx < 3; ++dx) {
          const float4 a = tile[r * RW + (p + dx) * CQ + q];
          row[dx][0] = a.x; row[dx][1] = a.y; row[dx][2] = a.z; row[dx][3] = a.w;
        }
      };
      rd(0, win[0]);
      rd(1, win[1]);
#pragma unroll
      for (int r = 0; r < R; ++r) {
        rd(r + 2, win[2]);
        const float4 d4 = q2f(dr[r]);  // zero outside the image (descriptor range)
        const float dv[4] = {d4.x, d4.y, d4.z, d4.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
#pragma unroll
          for (int dy = 0; dy < 3; ++dy)
#pragma unroll
            for (int dx = 0; dx < 3; ++dx)
              acc[dy * 3 + dx][j] = fmaf(dv[j], win[dy][dx][j], acc[dy * 3 + dx][j]);
          acc[9][j] += dv[j];
        }
#pragma unroll
        for (int dx = 0; dx < 3; ++dx)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            win[0][dx][j] = win[1][dx][j];
            win[1][dx][j] = win[2][dx][j];
          }
      }
    }
  }
  // lanes' sums -> per-channel partials: one thread per (tap i, quad qq) adds the span's
  // pixels in order
  __syncthreads();
  float4* red = reinterpret_cast<float4*>(tile);  // [10][NA] float4: lane-contiguous
  if (tid < NA) {
#pragma unroll
    for (int i = 0; i < 10; ++i) red[i * NA + tid] = make_float4(acc[i][0], acc[i][1], acc[i][2], acc[i][3]);
  }
  __syncthreads();
  for (int e = tid; e < 10 * CQ; e += NT) {
    const int i = e / CQ, qq = e - (e / CQ) * CQ;
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int pp = 0; pp < PX; ++pp) {
      const float4 v = red[i * NA + pp * CQ + qq];
      a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
    }
    st4(part + ((long)bid * 10 + i) * g.C + 4 * qq, a);
  }
}

// span wgrad geometry: row-tile bands of nrt tiles (fewer partial rows)
#define DWS_WG_NRT 4
static DwSGeom dw_sgeom_wgrad(int B, int H, int W, int C, int nt, dim3* grid) {
  DwSGeom g = dw_sgeom(B, H, W, C, nt, grid);
  g.remap = 0;
  g.nrt = DWS_WG_NRT;
  g.tilesH = ceil_div(ceil_div(H, DWS_R), DWS_WG_NRT);  // bands
  *grid = dim3((unsigned)((long)B * g.tilesH * g.NS));
  return g;
}

// tile-kernel selection: 0 = none (register-window kernel), else TCQ. 64-channel tiles
// (TCQ 16) for narrow images, and in bf16 wherever C % 64 == 0: a bf16 pixel segment is
// then one whole 128-B line (16 x 256 x 256 x 192 bf16: 253 -> 227 us, bf16 step +0.8 %;
// fp32 keeps 32-channel tiles: step -0.2 %, profiles/r03_tcq16_ab.txt).
// ACCUNET_DW_TCQ16 (tuning knob): 0 = narrow images only, 1 = wherever C % 64 == 0.
static int dw_tile_tcq(int H, int W, int C, int dt) {
  if (C % 32) return 0;
  if ((long)H * W * C * 4 >= (1L << 31)) return 0;  // one image per 32-bit buffer descriptor
  int CQ = C / 4;
  static int t16 = -2;
  if (t16 == -2) {
    const char* e = getenv("ACCUNET_DW_TCQ16");
    t16 = e ? atoi(e) : -1;
  }
  const bool wide = t16 == 1 || (t16 < 0 && dt == ACC_BF16);
  if ((W <= 16 || wide) && CQ % 16 == 0) return 16;
  return 8;
}

// Non-temporal input loads: by default only for inputs larger than the 256 MB
// Infinity Cache (streamed once, nothing to keep); ACCUNET_DW_NTL=0/1 forces it.
static int dw_ntl(long bytes) {
  static int v = -2;
  if (v == -2) {
    const char* e = getenv("ACCUNET_DW_NTL");
    v = e ? atoi(e) : -1;
  }
  return v >= 0 ? v : (bytes > (256L << 20) ? 1 : 0);
}

static int dw_cgfast() {
  static int v = -1;
  if (v < 0) {
    // default on: the channel groups of one tile run together, so each pixel's
    // 384-byte row is fetched as a unit (tools/k1_sweep2.sh: 161 -> 157.5 us on K1)
    const char* e = getenv("ACCUNET_DW_CGFAST");  // tuning knob (tools/kbench)
    v = e ? atoi(e) : 1;
  }
  return v;
}

// Which forward-type tile kernel a launch takes (ACCUNET_DW_OS): 1 (default) = one-shot
// 8-row tiles (dw3x3_os_fwd_kernel) for the fp32 forward and plain data gradient of
// inputs above the 256 MB Infinity Cache (the K1 shapes, 16 x 256^2 x 96 / 192), the
// strip kernel for everything else; 2 = one-shot tiles for every tile shape, dtype and
// launch kind; 0 = the strip kernel everywhere. Single-stream traces of the step
// (profiles/r05_dw_os_ab.txt): one-shot tiles are faster only on the streamed (> 256 MB)
// shapes; the BN-backward data gradient (a second pre-BN operand per output) and the
// cached 64^2..128^2 shapes run faster as strips. Per shape (tools/kbench KB_DWSWEEP,
// profiles/r05_dw_sweep.txt): one-shot 4-7 % faster at C = 96 / 192 / 384, 10 % slower
// at cnv72's 64^2 x 4352 (a tile's 136 channel groups, vertical neighbours 272 blocks
// apart), so C > 1024 keeps the strips. The statistics rows follow the kernel
// (accunet_dw3x3_rows takes the launch kind). tests/test_kernels_gpu.py runs the three
// settings bit for bit against each other.
static int dw_os() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("ACCUNET_DW_OS");
    v = e ? atoi(e) : 1;
  }
  return v;
}
static bool dw_os_on(int B, int H, int W, int C, int dt, bool bnb) {
  if (dw_os() == 2) return true;
  if (dw_os() != 1 || dt != ACC_F32 || bnb) return false;
  return (long)B * H * W * C * 4 > (256L << 20) && C <= 1024;
}
#define DW_OS_R 8
// ACCUNET_DW_OS16=1: the one-shot launches without a BN-backward operand run the
// 16-row, 512-thread tiles (dw3x3_os16_fwd_kernel). Off by default: at the K1 shape they
// measured 160.4 us against 146.4 us for the 8-row tiles on one box (bench probe,
// profiles/r06_os16_ab.txt) -- 4 waves per SIMD in 2 x 78 KB of LDS with the centre
// column read from LDS lose more than the halved halo re-fetch and statistics tails gain.
static bool dw_os16(bool bnb) {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("ACCUNET_DW_OS16");
    v = e ? atoi(e) : 0;
  }
  return v != 0 && !bnb;
}

static DwOGeom dw_ogeom(int B, int H, int W, int C, int tcq, dim3* grid, int rows = DW_OS_R) {
  DwOGeom g;
  g.B = B; g.H = H; g.W = W; g.C = C;
  g.tilesW = ceil_div(W, 256 / tcq);
  g.tilesH = ceil_div(H, rows);
  g.ncg = C / 4 / tcq;
  g.ntl = 0;
  g.xcd = 0;
  *grid = dim3((unsigned)((long)B * g.tilesH * g.tilesW * g.ncg));
  return g;
}

static int dw_rch_max() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("ACCUNET_DW_RCH");  // tuning knob (tools/kbench); default 32
    v = e ? atoi(e) : 32;
    if (v < 1) v = 1;
  }
  return v;
}

// rch_max > 1 (forward only): strips of up to 8*rch_max rows, as long as the grid
// keeps >= 768 workgroups (3 per CU); the weight-gradient kernel uses 1.
static DwTGeom dw_tgeom(int B, int H, int W, int C, int tcq, dim3* grid, int rch_max = 1) {
  DwTGeom g;
  g.B = B; g.H = H; g.W = W; g.C = C;
  g.tilesW = ceil_div(W, 256 / tcq);
  long cols = (long)B * g.tilesW * (C / 4 / tcq);
  int rch = 1;
  static const char* force = getenv("ACCUNET_DW_RCH_FORCE");  // tuning knob (tools/kbench)
  if (force && rch_max > 1) {
    rch = atoi(force) > 0 ? atoi(force) : 1;
  } else {
      // the longest strips (powers of two) that still give >= 4 rounds of 3 resident
      // blocks per CU (3072 blocks): 16x256x256x96 fp32 rch 1/2/4/8/16 = 180/159/154/155/
      // 160 us, 32-row strips (3072 blocks) best (profiles/r03_k1lab.txt)
      for (int r = 1; r <= rch_max; r *= 2) {
        rch = r;
        if (DW_TR * r >= H) break;
        if (cols * ceil_div(H, DW_TR * 2 * r) < 3072) break;
      }
  }
  g.rch = rch;
  g.ntl = dw_ntl((long)B * H * W * C * 4);
  g.tilesH = ceil_div(H, DW_TR * rch);
  long nt = (long)B * g.tilesH * g.tilesW;
  static const char* noremap = getenv("ACCUNET_DW_NOREMAP");  // tuning knob (tools/kbench)
  g.remap = (nt % 8 == 0 && !noremap) ? 1 : 0;
  g.cgf = 0;
  *grid = dim3((unsigned)nt, C / 4 / tcq);
  return g;
}

static DwGeom dw_geom(int B, int H, int W, int C, int V, dim3* grid) {
  DwGeom g;
  g.B = B; g.H = H; g.W = W; g.C = C;
  int CQ = C / V;
  if (CQ % 8 == 0) g.TCQ = 8;
  else if (CQ <= 64) g.TCQ = CQ;
  else g.TCQ = 8;  // (not hit on the ACC-UNet shapes)
  g.TW = 256 / g.TCQ;
  g.tilesW = ceil_div(W, g.TW);
  g.tilesH = ceil_div(H, DW_TR);
  *grid = dim3(B * g.tilesH * g.tilesW, ceil_div(CQ, g.TCQ));
  return g;
}

// which forward kernel accunet_dw3x3_fwd runs for this shape and storage dtype without
// a BN-backward epilogue: 2 = span, 1 = tile (strip), 0 = register window (profiling
// names / the bench probe); it follows the same two choices the launch below makes
extern "C" int accunet_dw3x3_variant(int B, int H, int W, int C, int dt) {
  if (dw_span_nt(H, W, C)) return 2;
  const int tcq = dw_tile_tcq(H, W, C, dt);
  if (tcq && dw_os_on(B, H, W, C, dt, false)) return dw_os16(false) ? 4 : 3;
  return tcq ? 1 : 0;
}

extern "C" int accunet_dw3x3_rows(int B, int H, int W, int C, int dt, int bnb) {
  dim3 grid;
  if (const int nt = dw_span_nt(H, W, C)) {
    dw_sgeom(B, H, W, C, nt, &grid);
    return (int)grid.x;
  }
  int tcq = dw_tile_tcq(H, W, C, dt);
  if (tcq && dw_os_on(B, H, W, C, dt, bnb != 0)) {
    const DwOGeom og = dw_ogeom(B, H, W, C, tcq, &grid, dw_os16(bnb != 0) ? 2 * DW_OS_R : DW_OS_R);
    return B * og.tilesH * og.tilesW;
  }
  if (tcq) dw_tgeom(B, H, W, C, tcq, &grid, dw_rch_max());
  else dw_geom(B, H, W, C, (C % 4 == 0) ? 4 : 1, &grid);
  return (int)grid.x;
}

// Every depthwise kernel addresses one image through a buffer descriptor whose byte
// count and offsets are 32-bit (the masked offset ACC_OOB = 2^31 must stay out of
// range): images of 2 GiB or more are refused (ACC_EBADSHAPE) instead of wrapping.
// ACC_UNet.forward raises before it gets here (accunet/model.py).
static bool dw_image_ok(int H, int W, int C, int dt) {
  const long bytes = (long)H * W * C * (dt == ACC_BF16 ? 2 : 4);
  return H > 0 && W > 0 && C > 0 && bytes < (1L << 31);
}

extern "C" int accunet_dw3x3_fwd(const void* x, const float* wt, const float* bias,
                                 const float* sc, const float* sh, int act, int flip, void* z,
                                 double* stats, int B, int H, int W, int C, const void* bz,
                                 const float* bst, int bact, int dt, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (!dw_image_ok(H, W, C, dt)) return ACC_EBADSHAPE;
  if (bz && (!bst || !stats)) return ACC_EBADARG;
  dim3 grid;
  if (const int nt = dw_span_nt(H, W, C)) {
    const DwSGeom sg = dw_sgeom(B, H, W, C, nt, &grid);
    // non-temporal input loads above the Infinity Cache (bytes as stored)
    const bool ntl = dw_ntl((long)B * H * W * C * (dt == ACC_BF16 ? 2 : 4)) != 0;
    auto launch = [&](auto tag, auto ntc, auto bnbc, auto auxc) {
      using T = decltype(tag);
      hipLaunchKernelGGL((dw3x3_span_fwd_kernel<decltype(ntc)::value, decltype(bnbc)::value,
                                                decltype(auxc)::value, T>),
                         grid, dim3(decltype(ntc)::value), 0, s, (const T*)x, wt, bias, sc, sh, act,
                         flip, (T*)z, stats, sg, (const T*)bz, bst, bact);
    };
    using N256 = std::integral_constant<int, 256>;
    using N512 = std::integral_constant<int, 512>;
    using BT = std::integral_constant<bool, true>;
    using BF = std::integral_constant<bool, false>;
    using A2 = std::integral_constant<int, 2>;
    using A0 = std::integral_constant<int, 0>;
    if (with_dt(dt, [&](auto tag) {
          auto by_aux = [&](auto n, auto bn) {
            if (ntl) launch(tag, n, bn, A2{});
            else launch(tag, n, bn, A0{});
          };
          auto by_bnb = [&](auto n) {
            if (bz) by_aux(n, BT{});
            else by_aux(n, BF{});
          };
          if (nt == 256) by_bnb(N256{});
          else by_bnb(N512{});
        }))
      return ACC_EBADARG;
    return hipGetLastError() == hipSuccess ? ACC_OK : ACC_ELAUNCH;
  }
  int tcq = dw_tile_tcq(H, W, C, dt);
  if (tcq && dw_os_on(B, H, W, C, dt, bz != nullptr) && dw_os16(bz != nullptr)) {
    DwOGeom og = dw_ogeom(B, H, W, C, tcq, &grid, 2 * DW_OS_R);
    auto launch = [&](auto tag, auto tcqc) {
      using T = decltype(tag);
      hipLaunchKernelGGL((dw3x3_os16_fwd_kernel<decltype(tcqc)::value, T>), grid, dim3(512), 0, s,
                         (const T*)x, wt, bias, sc, sh, act, flip, (T*)z, stats, og);
    };
    if (with_dt(dt, [&](auto tag) {
          if (tcq == 16) launch(tag, std::integral_constant<int, 16>{});
          else launch(tag, std::integral_constant<int, 8>{});
        }))
      return ACC_EBADARG;
    return hipGetLastError() == hipSuccess ? ACC_OK : ACC_ELAUNCH;
  }
  if (tcq && dw_os_on(B, H, W, C, dt, bz != nullptr)) {
    DwOGeom og = dw_ogeom(B, H, W, C, tcq, &grid);
    // default-policy input loads: a tile re-reads 2 of its 10 input rows and 2 of its 34
    // pixels from its neighbours' fetches, and non-temporal loads evict those lines
    // before the neighbour runs (kbench, same box: K1 149.0 -> 143.2 us, the flipped data
    // gradient 143.2 -> 135.4 us without them; the strips keep nt loads above 256 MB)
    const int seg = tcq * 4 * (dt == ACC_BF16 ? 2 : 4);
    og.ntl = 0;
    // half-line pixel segments (bf16, 32 channels): the channel groups sharing a line on
    // one XCD
    og.xcd = seg % 128 != 0 && og.ncg > 1 && (long)B * og.tilesH * og.tilesW % 8 == 0;
    auto launch = [&](auto tag, auto tcqc, auto bnbc, auto auxc) {
      using T = decltype(tag);
      hipLaunchKernelGGL((dw3x3_os_fwd_kernel<decltype(tcqc)::value, DW_OS_R,
                                              decltype(bnbc)::value, decltype(auxc)::value, T>),
                         grid, dim3(256), 0, s, (const T*)x, wt, bias, sc, sh, act, flip, (T*)z,
                         stats, og, (const T*)bz, bst, bact);
    };
    using I16 = std::integral_constant<int, 16>;
    using I8 = std::integral_constant<int, 8>;
    using BT = std::integral_constant<bool, true>;
    using BF = std::integral_constant<bool, false>;
    using A0 = std::integral_constant<int, 0>;  // (default-policy loads, see above)
    if (with_dt(dt, [&](auto tag) {
          auto by_bnb = [&](auto tc) {
            if (bz) launch(tag, tc, BT{}, A0{});
            else launch(tag, tc, BF{}, A0{});
          };
          if (tcq == 16) by_bnb(I16{});
          else by_bnb(I8{});
        }))
      return ACC_EBADARG;
    return hipGetLastError() == hipSuccess ? ACC_OK : ACC_ELAUNCH;
  }
  if (tcq) {
    DwTGeom tg = dw_tgeom(B, H, W, C, tcq, &grid, dw_rch_max());
    // non-temporal loads only for inputs above the Infinity Cache (bytes as stored)
    // and only when a block's pixel segment is whole 128-B lines: bf16 TCQ-8 blocks read
    // 64 B of each line, and a streamed line is fetched again for the neighbouring
    // channel group (16x256x256x192 bf16 forward 304 us in-model with them)
    const int seg = tcq * 4 * (dt == ACC_BF16 ? 2 : 4);
    tg.ntl = seg % 128 == 0 ? dw_ntl((long)B * H * W * C * (dt == ACC_BF16 ? 2 : 4)) : 0;
    if (dw_cgfast() && grid.y > 1) {
      tg.cgf = (int)grid.y;
      grid = dim3(grid.x * grid.y, 1);
    }
    // both fixed-function choices (channel-group width, nt loads) are template arguments
    auto launch = [&](auto tag, auto tcqc, auto bnbc, auto auxc) {
      using T = decltype(tag);
      hipLaunchKernelGGL((dw3x3_tile_fwd_kernel<decltype(tcqc)::value, decltype(bnbc)::value,
                                                decltype(auxc)::value, T>),
                         grid, dim3(256), 0, s, (const T*)x, wt, bias, sc, sh, act, flip, (T*)z,
                         stats, tg, (const T*)bz, bst, bact);
    };
    using I16 = std::integral_constant<int, 16>;
    using I8 = std::integral_constant<int, 8>;
    using BT = std::integral_constant<bool, true>;
    using BF = std::integral_constant<bool, false>;
    using A2 = std::integral_constant<int, 2>;
    using A0 = std::integral_constant<int, 0>;
    if (with_dt(dt, [&](auto tag) {
          auto by_aux = [&](auto tc, auto bn) {
            if (tg.ntl) launch(tag, tc, bn, A2{});
            else launch(tag, tc, bn, A0{});
          };
          auto by_bnb = [&](auto tc) {
            if (bz) by_aux(tc, BT{});
            else by_aux(tc, BF{});
          };
          if (tcq == 16) by_bnb(I16{});
          else by_bnb(I8{});
        }))
      return ACC_EBADARG;
    return hipGetLastError() == hipSuccess ? ACC_OK : ACC_ELAUNCH;
  }
  int V = (C % 4 == 0) ? 4 : 1;
  DwGeom g = dw_geom(B, H, W, C, V, &grid);
  if (with_dt(dt, [&](auto tag) {
        using T = decltype(tag);
        if (V == 4)
          hipLaunchKernelGGL((dw3x3_fwd_kernel<4, T>), grid, dim3(256), 0, s, (const T*)x, wt, bias,
                             sc, sh, act, flip, (T*)z, stats, g, (const T*)bz, bst, bact);
        else
          hipLaunchKernelGGL((dw3x3_fwd_kernel<1, T>), grid, dim3(256), 0, s, (const T*)x, wt, bias,
                             sc, sh, act, flip, (T*)z, stats, g, (const T*)bz, bst, bact);
      }))
    return ACC_EBADARG;
  return hipGetLastError() == hipSuccess ? ACC_OK : ACC_ELAUNCH;
}

static int dw_wgrad_rows(int B, int H, int W, int C, int dt) {
  dim3 grid;
  if (const int nt = dw_span_nt(H, W, C, 1)) {
    dw_sgeom_wgrad(B, H, W, C, nt, &grid);
    return (int)grid.x;
  }
  int tcq = dw_tile_tcq(H, W, C, dt);
  if (tcq) dw_tgeom(B, H, W, C, tcq, &grid);
  else dw_geom(B, H, W, C, (C % 4 == 0) ? 4 : 1, &grid);
  return (int)grid.x;
}

size_t dw_wgrad_ws(int B, int H, int W, int C, int dt) {
  int R = dw_wgrad_rows(B, H, W, C, dt);
  return (size_t)R * 10 * C + accunet_partials_ws_elems(R, 10 * C) + 10 * (size_t)C;
}

extern "C" size_t accunet_dw3x3_wgrad_ws(int B, int H, int W, int C, int dt) {
  return dw_wgrad_ws(B, H, W, C, dt);
}

extern "C" int accunet_dw3x3_wgrad(const void* x, const void* dz, const float* sc,
                                   const float* sh, int act, float* dw, float* db, int B, int H,
                                   int W, int C, float* ws, size_t ws_elems, int dt, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (!dw_image_ok(H, W, C, dt)) return ACC_EBADSHAPE;
  int V = (C % 4 == 0) ? 4 : 1;
  dim3 grid;
  int tcq = dw_tile_tcq(H, W, C, dt);
  DwTGeom tg;
  DwGeom g;
  if (tcq) tg = dw_tgeom(B, H, W, C, tcq, &grid);
  else g = dw_geom(B, H, W, C, V, &grid);
  int R = (int)grid.x;
  if (ws_elems < dw_wgrad_ws(B, H, W, C, dt)) return ACC_EBADARG;
  float* part = ws;
  float* scratch = ws + (size_t)R * 10 * C;
  float* sums = scratch + accunet_partials_ws_elems(R, 10 * C);
  if (const int nt = dw_span_nt(H, W, C, 1)) {
    dim3 sgrid;
    const DwSGeom sg = dw_sgeom_wgrad(B, H, W, C, nt, &sgrid);
    R = (int)sgrid.x;
    if (ws_elems < dw_wgrad_ws(B, H, W, C, dt)) return ACC_EBADARG;
    part = ws;
    scratch = ws + (size_t)R * 10 * C;
    // dw_span_nt(.., 1) is 256 or 0: the weight gradient runs 256-thread spans only
    if (nt != 256) return ACC_EBADARG;
    if (with_dt(dt, [&](auto tag) {
          using T = decltype(tag);
          hipLaunchKernelGGL((dw3x3_span_wgrad_kernel<256, 0, T>), sgrid, dim3(256), 0, s,
                             (const T*)x, (const T*)dz, sc, sh, act, part, sg);
        }))
      return ACC_EBADARG;
  } else if (with_dt(dt, [&](auto tag) {
        using T = decltype(tag);
        const T* xx = (const T*)x;
        const T* dd = (const T*)dz;
        if (tcq == 16)
          hipLaunchKernelGGL((dw3x3_tile_wgrad_kernel<16, T>), grid, dim3(256), 0, s, xx, dd, sc, sh,
                             act, part, tg);
        else if (tcq == 8)
          hipLaunchKernelGGL((dw3x3_tile_wgrad_kernel<8, T>), grid, dim3(256), 0, s, xx, dd, sc, sh,
                             act, part, tg);
        else if (V == 4)
          hipLaunchKernelGGL((dw3x3_wgrad_kernel<4, T>), grid, dim3(256), 0, s, xx, dd, sc, sh, act,
                             part, g);
        else
          hipLaunchKernelGGL((dw3x3_wgrad_kernel<1, T>), grid, dim3(256), 0, s, xx, dd, sc, sh, act,
                             part, g);
      }))
    return ACC_EBADARG;
  (void)sums;
  FinishArgs fa{};
  fa.kind = FIN_DW;
  fa.ncols = 10 * C;
  fa.C = C;
  fa.out_f = dw;
  fa.out2 = db;
  return reduce_finish(part, false, R, 10 * C, reinterpret_cast<double*>(scratch), fa, s);
}
