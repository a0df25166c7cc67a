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

template <int V>
ACC_DEV void ldv(const float* p, float (&v)[V]) {
  if (V == 4) {
    float4 q = ld4(p);
    v[0] = q.x; v[1] = q.y; v[2 % V] = q.z; v[3 % V] = q.w;
  } else {
    v[0] = p[0];
  }
}
template <int V>
ACC_DEV void stv(float* p, const float (&v)[V]) {
  if (V == 4) {
    st4(p, make_float4(v[0], v[1 % V], v[2 % V], v[3 % V]));
  } else {
    p[0] = v[0];
  }
}

// Reduce per-thread (a[V], b[V]) across the RG row-groups of the block and write
// the block's partial row out[(row)*2*C + {0,C} + c].
template <int V, typename T>
ACC_DEV void block_chan_reduce2(const ChanTile& t, T (&a)[V], T (&b)[V], T* out, long row,
                                int C) {
  __shared__ T red[2][256 * 4];
  int tid = threadIdx.x;
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
      out[row * 2 * C + t.c0 + j] = sa;
      out[row * 2 * C + C + t.c0 + j] = sb;
    }
  }
}
