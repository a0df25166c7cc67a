// K1 access-shape lab: streaming kernels with the geometry of the HANC depthwise
// forward (16x256x256x96 fp32 NHWC, 402 MB in + 402 MB out), no arithmetic, to find
// which part of K1's structure costs bandwidth against a flat copy.
//   hipcc -O3 --offload-arch=gfx950 tools/k1lab.hip -o tools/k1lab && tools/k1lab
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include <algorithm>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

typedef unsigned u32x4 __attribute__((__vector_size__(16)));
#define OOB 0x80000000u
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* b, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(b), 0, (int)bytes, 0x00020000);
}
template <int AUX>
__device__ __forceinline__ u32x4 ld(__amdgpu_buffer_rsrc_t r, unsigned off) {
  return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, AUX);
}
template <int AUX>
__device__ __forceinline__ void st(__amdgpu_buffer_rsrc_t r, unsigned off, u32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, AUX);
}

constexpr int B = 16, H = 256, W = 256, C = 96, CQ = C / 4;
constexpr unsigned IMG = H * W * C * 4;  // bytes per image

typedef float v4f __attribute__((ext_vector_type(4)));
__global__ void copy_flat(const v4f* __restrict__ a, v4f* __restrict__ b, long n) {
  long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (i < n) __builtin_nontemporal_store(__builtin_nontemporal_load(&a[i]), &b[i]);
}
__global__ void copy_x4(const v4f* __restrict__ a, v4f* __restrict__ b, long n) {
  long base = (long)blockIdx.x * 1024 + threadIdx.x;
  v4f v[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) v[k] = __builtin_nontemporal_load(&a[base + 256 * k]);
#pragma unroll
  for (int k = 0; k < 4; ++k) __builtin_nontemporal_store(v[k], &b[base + 256 * k]);
}

// tile geometry: R rows x 32 px x 8 quads (one channel group), channel group fastest
// in dispatch order; XCD-contiguous remap (consecutive ids go round-robin to XCDs)
template <int R, int AUX, bool REMAP>
__global__ void __launch_bounds__(256) tile_reg(const float* x, float* z) {
  int bid = blockIdx.x;
  if (REMAP) {
    const int per = gridDim.x >> 3;
    bid = (bid & 7) * per + (bid >> 3);
  }
  const int cg = bid % 3;
  int t = bid / 3;
  const int tw = t % 8;
  t /= 8;
  const int th = t % (H / R);
  const int b = t / (H / R);
  const int q = threadIdx.x % 8, p = threadIdx.x / 8;
  const int w = tw * 32 + p, c = cg * 32 + 4 * q;
  const auto rx = rsrc(x + (long)b * H * W * C, IMG), rz = rsrc(z + (long)b * H * W * C, IMG);
  u32x4 v[R];
#pragma unroll
  for (int r = 0; r < R; ++r) v[r] = ld<AUX>(rx, (((th * R + r) * W + w) * C + c) * 4);
#pragma unroll
  for (int r = 0; r < R; ++r) st<AUX>(rz, (((th * R + r) * W + w) * C + c) * 4, v[r]);
}

// rch=1 K1 without arithmetic: the (R+2) x 34 x 8 halo tile into LDS (all loads in
// flight), barrier, each thread stores its R interior rows read back from LDS
template <int R, int AUX>
__global__ void __launch_bounds__(256) tile_lds(const float* x, float* z) {
  constexpr int IP = 34, IR = R + 2, N4 = IR * IP * 8, NL = (N4 + 255) / 256;
  __shared__ u32x4 tile[N4];
  int bid = blockIdx.x;
  const int per = gridDim.x >> 3;
  bid = (bid & 7) * per + (bid >> 3);
  const int cg = bid % 3;
  int t = bid / 3;
  const int tw = t % 8;
  t /= 8;
  const int th = t % (H / R);
  const int b = t / (H / R);
  const int c0 = cg * 32;
  const auto rx = rsrc(x + (long)b * H * W * C, IMG), rz = rsrc(z + (long)b * H * W * C, IMG);
  u32x4 v[NL];
#pragma unroll
  for (int k = 0; k < NL; ++k) {
    const int i = threadIdx.x + 256 * k;
    const int q = i % 8, rp = i / 8, pp = rp % IP, r = rp / IP;
    const int hh = th * R - 1 + r, ww = tw * 32 - 1 + pp;
    const bool in = i < N4 && hh >= 0 && hh < H && ww >= 0 && ww < W;
    v[k] = ld<AUX>(rx, in ? (unsigned)(((hh * W + ww) * C + c0 + 4 * q) * 4) : OOB);
  }
#pragma unroll
  for (int k = 0; k < NL; ++k) {
    const int i = threadIdx.x + 256 * k;
    if (i < N4) tile[i] = v[k];
  }
  __syncthreads();
  const int q = threadIdx.x % 8, p = threadIdx.x / 8;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    u32x4 a = tile[((r + 1) * IP + p + 1) * 8 + q];
    st<AUX>(rz, (((th * R + r) * W + tw * 32 + p) * C + c0 + 4 * q) * 4, a);
  }
}

// span geometry: a block = 10 whole pixels (240 active lanes) x R rows; contiguous
// 3840-B row segments; registers only
template <int R, int AUX>
__global__ void __launch_bounds__(256) span_reg(const float* x, float* z) {
  constexpr int PX = 10, NA = PX * CQ;
  const int nsp = (W + PX - 1) / PX;  // 26 spans per row (last partial)
  int bid = blockIdx.x;
  const int sp = bid % nsp;
  int t = bid / nsp;
  const int th = t % (H / R);
  const int b = t / (H / R);
  const int i = threadIdx.x;
  const int pos = sp * NA + i;  // flattened quad index within the row
  const bool on = i < NA && pos < W * CQ;
  const auto rx = rsrc(x + (long)b * H * W * C, IMG), rz = rsrc(z + (long)b * H * W * C, IMG);
  u32x4 v[R];
#pragma unroll
  for (int r = 0; r < R; ++r)
    v[r] = ld<AUX>(rx, on ? (unsigned)(((th * R + r) * W * CQ + pos) * 16) : OOB);
#pragma unroll
  for (int r = 0; r < R; ++r)
    st<AUX>(rz, on ? (unsigned)(((th * R + r) * W * CQ + pos) * 16) : OOB, v[r]);
}

// row geometry: a block = one full image row (6144 quads) as 256 threads x 24 quads,
// contiguous 1 KB per wave-instruction; R rows per block
template <int R, int AUX>
__global__ void __launch_bounds__(256) row_reg(const float* x, float* z) {
  const long row0 = (long)blockIdx.x * R;  // global row index (b*H + h)
  const char* xb = (const char*)x;
  char* zb = (char*)z;
  for (int r = 0; r < R; ++r) {
    const long base = (row0 + r) * (long)W * C * 4;
    const auto rx = rsrc(xb + base, W * C * 4), rz = rsrc(zb + base, W * C * 4);
    u32x4 v[CQ];
#pragma unroll
    for (int k = 0; k < CQ; ++k) v[k] = ld<AUX>(rx, (threadIdx.x + 256 * k) * 16);
#pragma unroll
    for (int k = 0; k < CQ; ++k) st<AUX>(rz, (threadIdx.x + 256 * k) * 16, v[k]);
  }
}


// span geometry with the LDS halo tile (the span K1 without arithmetic): R+2 rows of
// 12 whole pixels into LDS (240 fill lanes, stride 240), each of 240 lanes stores its
// R interior quads read back from LDS
template <int R, int AUX, bool REMAP = false>
__global__ void __launch_bounds__(256) span_lds(const float* x, float* z) {
  constexpr int PX = 10, NA = PX * CQ, RW = (PX + 2) * CQ, NU = (R + 2) * RW;
  constexpr int NL = (NU + NA - 1) / NA;
  __shared__ u32x4 tile[NU];
  const int nsp = (W + PX - 1) / PX;
  int bid = blockIdx.x;
  if (REMAP) {  // XCD-contiguous: the spans of one row (and the next rows) share an L2
    const int per = gridDim.x >> 3;
    bid = (bid & 7) * per + (bid >> 3);
  }
  const int sp = bid % nsp;
  int t = bid / nsp;
  const int th = t % (H / R);
  const int b = t / (H / R);
  const int L = W * CQ, s0 = sp * PX * CQ, h0 = th * R;
  const auto rx = rsrc(x + (long)b * H * W * C, IMG), rz = rsrc(z + (long)b * H * W * C, IMG);
  const int tid = threadIdx.x;
  u32x4 v[NL];
#pragma unroll
  for (int k = 0; k < NL; ++k) {
    const int u = tid + NA * k;
    const int r = u / RW, jq = u % RW;
    const int hh = h0 - 1 + r, pos = s0 - CQ + jq;
    const bool in = tid < NA && u < NU && hh >= 0 && hh < H && pos >= 0 && pos < L;
    v[k] = ld<AUX>(rx, in ? (unsigned)((hh * L + pos) * 16) : OOB);
  }
#pragma unroll
  for (int k = 0; k < NL; ++k) {
    const int u = tid + NA * k;
    if (tid < NA && u < NU) tile[u] = v[k];
  }
  __syncthreads();
  const int p = tid / CQ, q = tid % CQ;
  const bool on = tid < NA && sp * PX + p < W;
#pragma unroll
  for (int r = 0; r < R; ++r)
    st<AUX>(rz, on ? (unsigned)(((h0 + r) * L + s0 + tid) * 16) : OOB, tile[(r + 1) * RW + (p + 1) * CQ + q]);
}

// current K1's persistent strip structure without arithmetic: 768 blocks, each a
// 32 px x 8 quad column strip of 128 rows walked in 4-row chunks over a 10-slot LDS
// ring; the next chunk's 4 rows are fetched into registers before this chunk's rows
// are stored and parked after it (the software pipeline of dw3x3_tile_fwd_kernel)
template <int AUX>
__global__ void __launch_bounds__(256) strip_lds(const float* x, float* z) {
  constexpr int IP = 34, IR = 10, CR = 4, SR = 128;
  constexpr int N4 = IR * IP * 8, NL = (N4 + 255) / 256;
  constexpr int N8 = CR * IP * 8, NL8 = (N8 + 255) / 256;
  __shared__ u32x4 ring[N4];
  int bid = blockIdx.x;
  const int per = gridDim.x >> 3;
  bid = (bid & 7) * per + (bid >> 3);
  const int cg = bid % 3;
  int t = bid / 3;
  const int tw = t % 8;
  t /= 8;
  const int th = t % (H / SR);
  const int b = t / (H / SR);
  const int c0 = cg * 32, hbeg = th * SR;
  const auto rx = rsrc(x + (long)b * H * W * C, IMG), rz = rsrc(z + (long)b * H * W * C, IMG);
  auto fetch = [&](u32x4* v, int nl, int hA, int n) {
    for (int k = 0; k < nl; ++k) {
      const int i = threadIdx.x + 256 * k;
      const int q = i % 8, rp = i / 8, pp = rp % IP, r = rp / IP;
      const int hh = hA + r, ww = tw * 32 - 1 + pp;
      const bool in = i < n && hh >= 0 && hh < H && ww >= 0 && ww < W;
      v[k] = ld<AUX>(rx, in ? (unsigned)(((hh * W + ww) * C + c0 + 4 * q) * 4) : OOB);
    }
  };
  auto park = [&](const u32x4* v, int nl, int hA, int n) {
    for (int k = 0; k < nl; ++k) {
      const int i = threadIdx.x + 256 * k;
      if (i < n) {
        const int q = i % 8, rp = i / 8, pp = rp % IP, r = rp / IP;
        const int slot = (hA + r - hbeg + 1) % IR;
        ring[(slot * IP + pp) * 8 + q] = v[k];
      }
    }
  };
  {
    u32x4 v[NL];
    fetch(v, NL, hbeg - 1, N4);
    park(v, NL, hbeg - 1, N4);
  }
  __syncthreads();
  const int q = threadIdx.x % 8, p = threadIdx.x / 8;
  for (int kc = 0; kc < SR / CR; ++kc) {
    const int r0 = hbeg + CR * kc;
    const bool more = kc + 1 < SR / CR;
    u32x4 nx[NL8];
    fetch(nx, NL8, r0 + 9, more ? N8 : 0);
#pragma unroll
    for (int r = 0; r < CR; ++r) {
      const int slot = (r0 + r - hbeg + 1) % IR;
      st<AUX>(rz, (((r0 + r) * W + tw * 32 + p) * C + c0 + 4 * q) * 4, ring[(slot * IP + p + 1) * 8 + q]);
    }
    if (more) {
      __syncthreads();
      park(nx, NL8, r0 + 9, N8);
      __syncthreads();
    }
  }
}


// the strip structure with D chunks of register prefetch in flight (D = 1 is
// strip_lds): rows for chunk kc + 1 + D are issued at chunk kc, parked at the end of
// chunk kc + D - 1; the 10-slot ring is unchanged, so LDS per block stays 43.5 KB.
// SR = strip rows (32: 3072 blocks, the K1 default; 128: 768 blocks)
template <int SR, int D, int AUX>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3)))
strip_lds_d(const float* x, float* z) {
  constexpr int IP = 34, IR = 10, CR = 4, NCH = SR / CR;
  constexpr int N4 = IR * IP * 8, NL = (N4 + 255) / 256;
  constexpr int N8 = CR * IP * 8, NL8 = (N8 + 255) / 256;
  static_assert(NCH % D == 0, "chunks per strip divisible by D");
  __shared__ u32x4 ring[N4];
  int bid = blockIdx.x;
  const int per = gridDim.x >> 3;
  bid = (bid & 7) * per + (bid >> 3);
  const int cg = bid % 3;
  int t = bid / 3;
  const int tw = t % 8;
  t /= 8;
  const int th = t % (H / SR);
  const int b = t / (H / SR);
  const int c0 = cg * 32, hbeg = th * SR;
  const auto rx = rsrc(x + (long)b * H * W * C, IMG), rz = rsrc(z + (long)b * H * W * C, IMG);
  auto fetch = [&](u32x4* v, int nl, int hA, int n) {
#pragma unroll
    for (int k = 0; k < nl; ++k) {
      const int i = threadIdx.x + 256 * k;
      const int q = i % 8, rp = i / 8, pp = rp % IP, r = rp / IP;
      const int hh = hA + r, ww = tw * 32 - 1 + pp;
      const bool in = i < n && hh >= 0 && hh < H && ww >= 0 && ww < W;
      v[k] = ld<AUX>(rx, in ? (unsigned)(((hh * W + ww) * C + c0 + 4 * q) * 4) : OOB);
    }
  };
  auto park = [&](const u32x4* v, int nl, int hA, int n) {
#pragma unroll
    for (int k = 0; k < nl; ++k) {
      const int i = threadIdx.x + 256 * k;
      if (i < n) {
        const int q = i % 8, rp = i / 8, pp = rp % IP, r = rp / IP;
        const int slot = (hA + r - hbeg + 1) % IR;
        ring[(slot * IP + pp) * 8 + q] = v[k];
      }
    }
  };
  {
    u32x4 v[NL];
    fetch(v, NL, hbeg - 1, N4);
    park(v, NL, hbeg - 1, N4);
  }
  u32x4 nx[D][NL8];
  // chunks 1 .. D-1 ahead are issued before the loop (rows r0+9+4j for chunk j)
#pragma unroll
  for (int j = 0; j + 1 < D; ++j) fetch(nx[j], NL8, hbeg + 9 + CR * j, (j + 2 < NCH + 1) ? N8 : 0);
  __syncthreads();
  const int q = threadIdx.x % 8, p = threadIdx.x / 8;
  for (int kb = 0; kb < NCH; kb += D) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const int kc = kb + d;
      const int r0 = hbeg + CR * kc;
      // issue the rows of chunk kc + D + 1 (r0 + 9 + 4 (D-1) ..) into buffer (d + D - 1) % D
      const int ahead = kc + D - 1;
      fetch(nx[(d + D - 1) % D], NL8, hbeg + 9 + CR * ahead, ahead + 1 < NCH ? N8 : 0);
#pragma unroll
      for (int r = 0; r < CR; ++r) {
        const int slot = (r0 + r - hbeg + 1) % IR;
        st<AUX>(rz, (((r0 + r) * W + tw * 32 + p) * C + c0 + 4 * q) * 4, ring[(slot * IP + p + 1) * 8 + q]);
      }
      if (kc + 1 < NCH) {
        __syncthreads();
        park(nx[d], NL8, r0 + 9, N8);
        __syncthreads();
      }
    }
  }
}


// cross-lane strip through wave-private LDS (no block barrier): a wave owns 8 pixels x
// 8 quads (one 128-B channel segment per pixel, 8 lines per load instruction) and walks
// SR rows down; per row it loads its 64 quads plus the two halo pixels (lanes 0..15),
// writes them to its own 10-pixel LDS row and reads back the left / right neighbours
// (in-order LDS within a wave: lgkmcnt, no barrier). PF rows of loads in flight.
// Block = 4 waves = 32 pixels of one channel group (the K1 tile footprint).
template <int SR, int PF, int AUX>
__global__ void __launch_bounds__(256) xl_lds(const float* x, float* z) {
  __shared__ u32x4 sm[4][2][80];
  int bid = blockIdx.x;
  const int per = gridDim.x >> 3;
  bid = (bid & 7) * per + (bid >> 3);
  const int cg = bid % 3;
  int t = bid / 3;
  const int tw = t % 8;
  t /= 8;
  const int th = t % (H / SR);
  const int b = t / (H / SR);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int p = lane >> 3, q = lane & 7;
  const int wbase = tw * 32 + wv * 8;
  const int c0 = cg * 32;
  const int hbeg = th * SR;
  const auto rx = rsrc(x + (long)b * H * W * C, IMG), rz = rsrc(z + (long)b * H * W * C, IMG);
  const int hw = lane < 8 ? wbase - 1 : wbase + 8;
  const bool hon = lane < 16 && hw >= 0 && hw < W;
  auto ldrow = [&](int h, u32x4& m, u32x4& hv) {
    const bool rin = h >= 0 && h < H;
    m = ld<AUX>(rx, rin ? (unsigned)(((h * W + wbase + p) * C + c0 + 4 * q) * 4) : OOB);
    hv = ld<AUX>(rx, (rin && hon) ? (unsigned)(((h * W + hw) * C + c0 + 4 * q) * 4) : OOB);
  };
  u32x4 mm[PF], hh[PF];
#pragma unroll
  for (int i = 0; i < PF; ++i) ldrow(hbeg - 1 + i, mm[i], hh[i]);
  u32x4 acc = {0u, 0u, 0u, 0u};
  for (int r0 = -1; r0 < SR + 1; r0 += PF) {
#pragma unroll
    for (int i = 0; i < PF; ++i) {
      const int h = hbeg + r0 + i;
      const u32x4 m = mm[i], hv = hh[i];
      ldrow(h + PF, mm[i], hh[i]);  // the row PF ahead into the freed slot
      u32x4* row = sm[wv][i & 1];
      row[(p + 1) * 8 + q] = m;
      if (lane < 16) row[lane < 8 ? q : 72 + q] = hv;
      const u32x4 lf = row[p * 8 + q], rt = row[(p + 2) * 8 + q];
      acc ^= lf ^ rt;
      if (h >= hbeg && h < hbeg + SR)
        st<AUX>(rz, (((h * W + wbase + p) * C + c0 + 4 * q) * 4), m);
    }
  }
  if (acc[0] == 0x12345678u && acc[1] == 0x9abcdef0u) z[0] = 1.f;  // (never)
}

// cross-lane geometry (a K1 without an LDS halo): a wave = 64 consecutive pixels of one
// row x NQ channel quads (lane = pixel), walking R rows down the image: each row's NQ
// quads are loaded once per lane (vertical window in registers), the left / right
// neighbours come from lanes -1 / +1 (ds_bpermute here; DPP wave shifts in a kernel), and
// the two halo pixels of the wave are loaded by the edge lanes. Stores its own quads.
template <int NQ, int R, int AUX>
__global__ void __launch_bounds__(256) pix_xlane(const float* x, float* z) {
  constexpr int NG = CQ / NQ;  // channel groups
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  int bid = blockIdx.x;
  const int per = gridDim.x >> 3;
  bid = (bid & 7) * per + (bid >> 3);
  // block = 4 waves: 4 channel groups (or fewer) of the same 64-pixel segment
  const int segs = W / 64;
  const int g0 = (bid % ((NG + 3) / 4)) * 4 + wv;
  int t = bid / ((NG + 3) / 4);
  const int sg = t % segs;
  t /= segs;
  const int th = t % (H / R);
  const int b = t / (H / R);
  const bool on = g0 < NG;
  const int w = sg * 64 + lane, c0 = g0 * NQ * 4;
  const auto rx = rsrc(x + (long)b * H * W * C, IMG), rz = rsrc(z + (long)b * H * W * C, IMG);
  u32x4 acc = {0u, 0u, 0u, 0u};
  for (int r = 0; r < R; ++r) {
    const int h = th * R + r;
    u32x4 v[NQ];
#pragma unroll
    for (int k = 0; k < NQ; ++k)
      v[k] = ld<AUX>(rx, on ? (unsigned)(((h * W + w) * C + c0 + 4 * k) * 4) : OOB);
    // halo pixels of the wave (lane 0: w - 1, lane 63: w + 1)
    const int hw = lane == 0 ? w - 1 : w + 1;
    const bool hon = on && (lane == 0 || lane == 63) && hw >= 0 && hw < W;
    u32x4 hv = ld<AUX>(rx, hon ? (unsigned)(((h * W + hw) * C + c0) * 4) : OOB);
#pragma unroll
    for (int k = 0; k < NQ; ++k) {
      // neighbours' quads (left, right) through the cross-lane network
      u32x4 lft, rgt;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        lft[e] = __builtin_amdgcn_ds_bpermute(((lane + 63) & 63) * 4, (int)v[k][e]);
        rgt[e] = __builtin_amdgcn_ds_bpermute(((lane + 1) & 63) * 4, (int)v[k][e]);
      }
      acc ^= lft ^ rgt ^ hv;  // consumed, so the exchange is not optimised away
      st<AUX>(rz, on ? (unsigned)(((h * W + w) * C + c0 + 4 * k) * 4) : OOB, v[k]);
    }
  }
  if (acc[0] == 0x12345678u && acc[1] == 0x9abcdef0u) z[0] = 1.f;  // (never)
}

__global__ void fill(float* p, long n) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    p[i] = (float)((i * 2654435761u) % 1000) / 1000.f;
}

template <class F>
static double timeit(F f, int iters) {
  f();
  std::vector<hipEvent_t> ev(2 * iters);
  for (auto& e : ev) CK(hipEventCreate(&e));
  for (int i = 0; i < iters; ++i) {
    CK(hipEventRecord(ev[2 * i], 0));
    f();
    CK(hipEventRecord(ev[2 * i + 1], 0));
  }
  CK(hipEventSynchronize(ev.back()));
  std::vector<float> t(iters);
  for (int i = 0; i < iters; ++i) CK(hipEventElapsedTime(&t[i], ev[2 * i], ev[2 * i + 1]));
  for (auto& e : ev) CK(hipEventDestroy(e));
  std::sort(t.begin(), t.end());
  return 1000.0 * t[iters / 2];
}

static unsigned long long sum(const float* d, size_t n) {
  std::vector<unsigned> h(n);
  CK(hipMemcpy(h.data(), d, n * 4, hipMemcpyDeviceToHost));
  unsigned long long s = 0;
  for (unsigned v : h) s += v;
  return s;
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 20;
  const size_t n = (size_t)B * H * W * C;
  const double bytes = 2.0 * 4 * n;
  float *x, *z;
  CK(hipMalloc(&x, n * 4));
  CK(hipMalloc(&z, n * 4));
  hipLaunchKernelGGL(fill, dim3(8192), dim3(256), 0, 0, x, (long)n);
  CK(hipDeviceSynchronize());
  const unsigned long long want = sum(x, n);
  auto rep = [&](const char* name, auto launch) {
    CK(hipMemset(z, 0, n * 4));
    const double us = timeit(launch, iters);
    CK(hipGetLastError());
    const bool ok = sum(z, n) == want;
    printf("%-40s %8.2f us %7.1f GB/s %5.1f%%  %s\n", name, us, bytes / us / 1e3,
           100.0 * bytes / us / 1e3 / 8000.0, ok ? "ok" : "MISMATCH");
    fflush(stdout);
  };
  const long n4 = (long)(n / 4);
  rep("copy flat nt", [&] { hipLaunchKernelGGL(copy_flat, dim3((n4 + 255) / 256), dim3(256), 0, 0, (const v4f*)x, (v4f*)z, n4); });
  rep("copy x4 nt", [&] { hipLaunchKernelGGL(copy_x4, dim3(n4 / 1024), dim3(256), 0, 0, (const v4f*)x, (v4f*)z, n4); });
  rep("tile_reg R8 nt remap", [&] { hipLaunchKernelGGL((tile_reg<8, 2, true>), dim3(B * 32 * 8 * 3), dim3(256), 0, 0, x, z); });
  rep("tile_reg R8 nt", [&] { hipLaunchKernelGGL((tile_reg<8, 2, false>), dim3(B * 32 * 8 * 3), dim3(256), 0, 0, x, z); });
  rep("tile_reg R8 default", [&] { hipLaunchKernelGGL((tile_reg<8, 0, true>), dim3(B * 32 * 8 * 3), dim3(256), 0, 0, x, z); });
  rep("tile_reg R4 nt remap", [&] { hipLaunchKernelGGL((tile_reg<4, 2, true>), dim3(B * 64 * 8 * 3), dim3(256), 0, 0, x, z); });
  rep("tile_reg R16 nt remap", [&] { hipLaunchKernelGGL((tile_reg<16, 2, true>), dim3(B * 16 * 8 * 3), dim3(256), 0, 0, x, z); });
  rep("tile_lds R8 nt (rch=1 K1 shape)", [&] { hipLaunchKernelGGL((tile_lds<8, 2>), dim3(B * 32 * 8 * 3), dim3(256), 0, 0, x, z); });
  rep("tile_lds R16 nt", [&] { hipLaunchKernelGGL((tile_lds<16, 2>), dim3(B * 16 * 8 * 3), dim3(256), 0, 0, x, z); });
  rep("strip_lds nt (current K1 structure)", [&] { hipLaunchKernelGGL((strip_lds<2>), dim3(B * 2 * 8 * 3), dim3(256), 0, 0, x, z); });
  rep("strip_lds default policy", [&] { hipLaunchKernelGGL((strip_lds<0>), dim3(B * 2 * 8 * 3), dim3(256), 0, 0, x, z); });
  rep("strip_lds_d SR32 D1 nt", [&] { hipLaunchKernelGGL((strip_lds_d<32, 1, 2>), dim3(B * 8 * 8 * 3), dim3(256), 0, 0, x, z); });
  rep("strip_lds_d SR32 D2 nt", [&] { hipLaunchKernelGGL((strip_lds_d<32, 2, 2>), dim3(B * 8 * 8 * 3), dim3(256), 0, 0, x, z); });
  rep("strip_lds_d SR32 D4 nt", [&] { hipLaunchKernelGGL((strip_lds_d<32, 4, 2>), dim3(B * 8 * 8 * 3), dim3(256), 0, 0, x, z); });
  rep("strip_lds_d SR64 D2 nt", [&] { hipLaunchKernelGGL((strip_lds_d<64, 2, 2>), dim3(B * 4 * 8 * 3), dim3(256), 0, 0, x, z); });
  rep("strip_lds_d SR128 D2 nt", [&] { hipLaunchKernelGGL((strip_lds_d<128, 2, 2>), dim3(B * 2 * 8 * 3), dim3(256), 0, 0, x, z); });
  rep("strip_lds_d SR128 D4 nt", [&] { hipLaunchKernelGGL((strip_lds_d<128, 4, 2>), dim3(B * 2 * 8 * 3), dim3(256), 0, 0, x, z); });
  rep("xl_lds SR32 PF2 nt", [&] { hipLaunchKernelGGL((xl_lds<32, 2, 2>), dim3(B * 8 * 8 * 3), dim3(256), 0, 0, x, z); });
  rep("xl_lds SR32 PF4 nt", [&] { hipLaunchKernelGGL((xl_lds<32, 4, 2>), dim3(B * 8 * 8 * 3), dim3(256), 0, 0, x, z); });
  rep("xl_lds SR32 PF8 nt", [&] { hipLaunchKernelGGL((xl_lds<32, 8, 2>), dim3(B * 8 * 8 * 3), dim3(256), 0, 0, x, z); });
  rep("xl_lds SR64 PF4 nt", [&] { hipLaunchKernelGGL((xl_lds<64, 4, 2>), dim3(B * 4 * 8 * 3), dim3(256), 0, 0, x, z); });
  rep("xl_lds SR16 PF4 nt", [&] { hipLaunchKernelGGL((xl_lds<16, 4, 2>), dim3(B * 16 * 8 * 3), dim3(256), 0, 0, x, z); });
  rep("xl_lds SR128 PF4 nt", [&] { hipLaunchKernelGGL((xl_lds<128, 4, 2>), dim3(B * 2 * 8 * 3), dim3(256), 0, 0, x, z); });
  rep("span_reg R8 nt", [&] { hipLaunchKernelGGL((span_reg<8, 2>), dim3(B * 32 * 26), dim3(256), 0, 0, x, z); });
  rep("span_lds R8 nt (span K1 shape)", [&] { hipLaunchKernelGGL((span_lds<8, 2>), dim3(B * 32 * 26), dim3(256), 0, 0, x, z); });
  rep("span_lds R8 nt remap", [&] { hipLaunchKernelGGL((span_lds<8, 2, true>), dim3(B * 32 * 26), dim3(256), 0, 0, x, z); });
  rep("span_lds R16 nt", [&] { hipLaunchKernelGGL((span_lds<16, 2>), dim3(B * 16 * 26), dim3(256), 0, 0, x, z); });
  rep("span_reg R4 nt", [&] { hipLaunchKernelGGL((span_reg<4, 2>), dim3(B * 64 * 26), dim3(256), 0, 0, x, z); });
  rep("row_reg R1 nt", [&] { hipLaunchKernelGGL((row_reg<1, 2>), dim3(B * H), dim3(256), 0, 0, x, z); });
  rep("row_reg R2 nt", [&] { hipLaunchKernelGGL((row_reg<2, 2>), dim3(B * H / 2), dim3(256), 0, 0, x, z); });
  // 64-pixel segments x channel groups of NQ quads, 4 groups per block
  rep("pix_xlane NQ4 R8 nt", [&] { hipLaunchKernelGGL((pix_xlane<4, 8, 2>), dim3(B * (H / 8) * (W / 64) * ((CQ / 4 + 3) / 4)), dim3(256), 0, 0, x, z); });
  rep("pix_xlane NQ8 R8 nt", [&] { hipLaunchKernelGGL((pix_xlane<8, 8, 2>), dim3(B * (H / 8) * (W / 64) * ((CQ / 8 + 3) / 4)), dim3(256), 0, 0, x, z); });
  rep("pix_xlane NQ4 R32 nt", [&] { hipLaunchKernelGGL((pix_xlane<4, 32, 2>), dim3(B * (H / 32) * (W / 64) * ((CQ / 4 + 3) / 4)), dim3(256), 0, 0, x, z); });
  rep("pix_xlane NQ8 R32 default", [&] { hipLaunchKernelGGL((pix_xlane<8, 32, 0>), dim3(B * (H / 32) * (W / 64) * ((CQ / 8 + 3) / 4)), dim3(256), 0, 0, x, z); });
  CK(hipFree(x));
  CK(hipFree(z));
  return 0;
}
