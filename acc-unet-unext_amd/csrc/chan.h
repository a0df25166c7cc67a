// Channel-tiled streaming helpers shared by the NHWC elementwise / reduction kernels.
#pragma once
#include "common.h"

// --------------------------------------------------------------------------
// Channel-tiled streaming geometry: thread t of a 256-thread block owns channel
// vector cq = t % TCQ (V = 4 or 1 channels) of channel group blockIdx.y and walks
// rows rg, rg + RG, ... of the block's row range.
// --------------------------------------------------------------------------
struct ChanTile {
  int CQ, TCQ, RG, cq, rg, c0;
  bool active;
};

template <int V>
ACC_DEV ChanTile chan_tile(int C) {
  ChanTile t;
  t.CQ = C / V;
  t.TCQ = t.CQ < 64 ? t.CQ : 64;
  t.RG = 256 / t.TCQ;
  int tid = threadIdx.x;
  t.cq = blockIdx.y * 64 + tid % t.TCQ;
  t.rg = tid / t.TCQ;
  t.c0 = t.cq * V;
  t.active = (t.rg < t.RG) && (t.cq < t.CQ) && (tid % t.TCQ) < t.TCQ;
  return t;
}

template <int V, typename T>
ACC_DEV void ldv(const T* p, float (&v)[V]) {
  if (V == 4) {
    float4 q = ldq(p);
    v[0] = q.x; v[1 % V] = q.y; v[2 % V] = q.z; v[3 % V] = q.w;
  } else {
    v[0] = ld1(p);
  }
}
template <int V, typename T>
ACC_DEV void stv(T* p, const float (&v)[V]) {
  if (V == 4) {
    stq(p, make_float4(v[0], v[1 % V], v[2 % V], v[3 % V]));
  } else {
    st1(p, v[0]);
  }
}
// stv that also rounds v to what was stored (so statistics describe the tensor)
template <int V, typename T>
ACC_DEV void stv_r(T* p, float (&v)[V]) {
#pragma unroll
  for (int j = 0; j < V; ++j) v[j] = rnd<T>(v[j]);
  stv<V>(p, v);
}

// Streaming visit of one thread's rows of a row chunk: local rows lr = rg, rg + RG, ...
// < nrows of a chunk whose base pointers are block-uniform, channel quad c0 of C.
// U rows (per input) are loaded raw before any is used, branch-free: rows past the
// chunk read as 0 through the buffer range check (ACC_OOB), so the compiler waits for
// each load alone instead of draining every outstanding access per row. f(ok, x...,
// off) runs in row order (sums stay bit-identical to the plain row loop); off is the
// row's byte offset or ACC_OOB, usable for a masked bufq_st of an output chunk.
// Chunks must stay below 2^31 bytes (callers check).
template <int U, typename T, typename F>
ACC_DEV void quad_rows1(const T* base, long nrows, int rg, int RG, int C, int c0, F f) {
  typedef typename QuadRaw<T>::type QR;
  const __amdgpu_buffer_rsrc_t rs = acc_rsrc(base, (unsigned)(nrows * C * sizeof(T)));
  const long nit = (nrows + RG - 1) / RG;
  __builtin_amdgcn_s_waitcnt(0);  // no pre-loop load left pending across the loop
  for (long i0 = 0; i0 < nit; i0 += U) {
    QR raw[U];
    unsigned off[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long lr = rg + (i0 + u) * RG;
      off[u] = lr < nrows ? (unsigned)((lr * C + c0) * sizeof(T)) : ACC_OOB;
      raw[u] = bufq_ld<0>(rs, off[u], (const T*)nullptr);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) f(off[u] != ACC_OOB, q2f(raw[u]), off[u]);
  }
}
template <int U, typename T, typename F>
ACC_DEV void quad_rows2(const T* base1, const T* base2, long nrows, int rg, int RG, int C, int c0,
                        F f) {
  typedef typename QuadRaw<T>::type QR;
  const unsigned bytes = (unsigned)(nrows * C * sizeof(T));
  const __amdgpu_buffer_rsrc_t r1 = acc_rsrc(base1, bytes), r2 = acc_rsrc(base2, bytes);
  const long nit = (nrows + RG - 1) / RG;
  __builtin_amdgcn_s_waitcnt(0);
  for (long i0 = 0; i0 < nit; i0 += U) {
    QR x1[U], x2[U];
    unsigned off[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long lr = rg + (i0 + u) * RG;
      off[u] = lr < nrows ? (unsigned)((lr * C + c0) * sizeof(T)) : ACC_OOB;
      x1[u] = bufq_ld<0>(r1, off[u], (const T*)nullptr);
      x2[u] = bufq_ld<0>(r2, off[u], (const T*)nullptr);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) f(off[u] != ACC_OOB, q2f(x1[u]), q2f(x2[u]), off[u]);
  }
}

// Reduce per-thread (a[V], b[V]) across the RG row-groups of the block and write
// the block's partial row out[(row)*2*C + {0,C} + c].
// CM (channel-major): quantity q of channel c goes to out[(q*C + c)*R + row] instead,
// so a reader of one channel's R rows (se_bwd_chan_sum_kernel) reads contiguous memory.
template <int V, typename T, bool CM = false>
ACC_DEV void block_chan_reduce2(const ChanTile& t, T (&a)[V], T (&b)[V], T* out, long row,
                                int C, long R = 0) {
  auto at = [&](int q, int c) -> T& {
    return CM ? out[((long)q * C + c) * R + row] : out[row * 2 * C + (long)q * C + c];
  };
  __shared__ T red[2][256 * 4];
  int tid = threadIdx.x;
  if ((t.TCQ & (t.TCQ - 1)) == 0) {
    // power-of-two slot count: lanes sharing a channel vector are xor partners;
    // reduce within the wave, then the 4 wave sums in order (deterministic)
    for (int off = t.TCQ; off < 64; off <<= 1) {
#pragma unroll
      for (int j = 0; j < V; ++j) {
        a[j] += __shfl_xor(a[j], off);
        b[j] += __shfl_xor(b[j], off);
      }
    }
    const int lane = tid & 63, wave = tid >> 6;
    if (lane < t.TCQ) {
#pragma unroll
      for (int j = 0; j < V; ++j) {
        red[0][(wave * 64 + lane) * V + j] = a[j];
        red[1][(wave * 64 + lane) * V + j] = b[j];
      }
    }
    __syncthreads();
    if (tid < t.TCQ && t.cq < t.CQ) {
#pragma unroll
      for (int j = 0; j < V; ++j) {
        T sa = 0, sb = 0;
        for (int w = 0; w < 4; ++w) {
          sa += red[0][(w * 64 + tid) * V + j];
          sb += red[1][(w * 64 + tid) * V + j];
        }
        at(0, t.c0 + j) = sa;
        at(1, t.c0 + j) = sb;
      }
    }
    return;
  }
#pragma unroll
  for (int j = 0; j < V; ++j) {
    red[0][tid * V + j] = a[j];
    red[1][tid * V + j] = b[j];
  }
  __syncthreads();
  if (t.rg == 0 && t.cq < t.CQ) {
    int lt = tid % t.TCQ;
#pragma unroll
    for (int j = 0; j < V; ++j) {
      T sa = 0, sb = 0;
      for (int g = 0; g < t.RG; ++g) {
        sa += red[0][(g * t.TCQ + lt) * V + j];
        sb += red[1][(g * t.TCQ + lt) * V + j];
      }
      at(0, t.c0 + j) = sa;
      at(1, t.c0 + j) = sb;
    }
  }
}

// N-quantity version of block_chan_reduce2: per-thread v[i][V] (i < N) reduced over
// the block's row groups into out[(row*N + i)*C + c], one quantity at a time through
// one LDS buffer (same deterministic order as block_chan_reduce2).
template <int V, int N, typename T, bool CM = false>
ACC_DEV void block_chan_reduceN(const ChanTile& t, T (&v)[N][V], T* out, long row, int C,
                                long R = 0) {
  auto at = [&](int q, int c) -> T& {
    return CM ? out[((long)q * C + c) * R + row] : out[(row * N + q) * C + c];
  };
  __shared__ T red[256 * 4];
  const int tid = threadIdx.x;
  const bool p2 = (t.TCQ & (t.TCQ - 1)) == 0;
  const int lane = tid & 63, wave = tid >> 6;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    if (p2) {
      for (int off = t.TCQ; off < 64; off <<= 1) {
#pragma unroll
        for (int j = 0; j < V; ++j) v[i][j] += __shfl_xor(v[i][j], off);
      }
      if (lane < t.TCQ) {
#pragma unroll
        for (int j = 0; j < V; ++j) red[(wave * 64 + lane) * V + j] = v[i][j];
      }
      __syncthreads();
      if (tid < t.TCQ && t.cq < t.CQ) {
#pragma unroll
        for (int j = 0; j < V; ++j) {
          T s = 0;
          for (int w = 0; w < 4; ++w) s += red[(w * 64 + tid) * V + j];
          at(i, t.c0 + j) = s;
        }
      }
    } else {
#pragma unroll
      for (int j = 0; j < V; ++j) red[tid * V + j] = v[i][j];
      __syncthreads();
      if (t.rg == 0 && t.cq < t.CQ) {
        const int lt = tid % t.TCQ;
#pragma unroll
        for (int j = 0; j < V; ++j) {
          T s = 0;
          for (int g = 0; g < t.RG; ++g) s += red[(g * t.TCQ + lt) * V + j];
          at(i, t.c0 + j) = s;
        }
      }
    }
    __syncthreads();
  }
}

// Deterministic block reduction for power-of-two slot counts: thread t contributes
// v[0..N) to slot t % TCQ (TCQ | 256). Lanes of one wave sharing a slot are summed
// with xor shuffles (offsets TCQ, 2*TCQ, ..., 32), the per-wave sums go through LDS
// ([waves][slot][N]) and threads t < TCQ add them in wave order. Returns true in
// the threads that hold a slot's total (t < TCQ), whose v[] then holds the sums.
// `lds` must hold 4 * min(TCQ, 64) * N elements; the caller syncs before reusing it.
template <int TCQ, int N, typename T>
ACC_DEV bool block_slot_reduce(T (&v)[N], T* lds) {
  static_assert(TCQ > 0 && (TCQ & (TCQ - 1)) == 0 && TCQ <= 256, "TCQ: power of two <= 256");
  constexpr int WL = TCQ < 64 ? TCQ : 64;  // slots per wave
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int off = TCQ; off < 64; off <<= 1)
#pragma unroll
    for (int i = 0; i < N; ++i) v[i] += __shfl_xor(v[i], off);
  if (lane < WL) {
#pragma unroll
    for (int i = 0; i < N; ++i) lds[(wave * WL + lane) * N + i] = v[i];
  }
  __syncthreads();
  const int t = threadIdx.x;
  if (t >= TCQ) return false;
  constexpr int WPS = 4 * WL / TCQ;  // waves holding each slot
#pragma unroll
  for (int i = 0; i < N; ++i) {
    T s = 0;
#pragma unroll
    for (int k = 0; k < WPS; ++k) {
      const int w = (t / 64) + k * (TCQ / WL);  // TCQ <= 64: w = k; TCQ = 128: t/64, +2
      s += lds[(w * WL + (t % WL)) * N + i];
    }
    v[i] = s;
  }
  return true;
}
