// Shared device helpers for the ACC-UNet gfx950 kernels.
//
// Layout convention for every activation tensor handed to this library:
// NHWC (channels-last), contiguous, viewed as a row-major matrix
// [P = B*H*W pixels][C channels]. A "pixel row" is therefore C contiguous
// elements, which makes 1x1 convolutions plain row-major GEMMs and keeps the
// per-channel BatchNorm / SE statistics coalesced along the fast axis.
// Activations (and activation gradients) are stored as fp32 or bf16 (`dt` =
// ACC_F32 / ACC_BF16 on the C ABI); arithmetic is always fp32 in registers,
// statistics fp64, parameters and their gradients fp32.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../include/accunet.h"

#define ACC_DEV __device__ __forceinline__

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float floatx4v __attribute__((ext_vector_type(4)));

// LeakyReLU slope used everywhere in the reference (torch default 0.01).
#define LRELU_SLOPE 0.01f

// status codes returned through the C ABI
#define ACC_OK 0
#define ACC_EBADSHAPE -1
#define ACC_EBADARG -2
#define ACC_ELAUNCH -3

// Fast unsigned division by a runtime-constant divisor (n < 2^31).
struct FastDiv {
  uint32_t d, m, s;
};

static inline FastDiv make_fastdiv(uint32_t d) {
  FastDiv f;
  f.d = d;
  uint32_t s = 0;
  while ((1ull << s) < d) ++s;
  f.s = s;
  uint64_t m = ((1ull << 32) * ((1ull << s) - d)) / d + 1;
  f.m = (uint32_t)m;
  return f;
}

ACC_DEV uint32_t fdiv(uint32_t n, const FastDiv& f) {
  uint32_t t = __umulhi(n, f.m);
  return (t + n) >> f.s;
}

// s[i] += v_r[i] for r = r, r+st, ... < r1 in that order (so the result is bit-identical
// to the plain loop), with the loads of U consecutive terms issued before any add:
// the small partial-row reductions are load-latency chains, not bandwidth bound.
template <int U, int N, typename T, class L>
ACC_DEV void ordered_strided_sum(T (&s)[N], int r, int r1, int st, L load) {
  for (; r + (U - 1) * st < r1; r += U * st) {
    T v[U][N];
#pragma unroll
    for (int u = 0; u < U; ++u) load(r + u * st, v[u]);
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int i = 0; i < N; ++i) s[i] += v[u][i];
  }
  for (; r < r1; r += st) {
    T v[N];
    load(r, v);
#pragma unroll
    for (int i = 0; i < N; ++i) s[i] += v[i];
  }
}

// LeakyReLU as max(x, slope*x): bit-identical to x > 0 ? x : slope*x for 0 < slope < 1
// (signed zeros and infinities included), 2 VALU ops (v_mul + v_max) instead of 3
ACC_DEV float lrelu(float x) { return __builtin_fmaxf(x, x * LRELU_SLOPE); }
// torch LeakyReLU backward: grad * (input > 0 ? 1 : slope)
ACC_DEV float lrelu_d(float pre) { return pre > 0.f ? 1.f : LRELU_SLOPE; }

ACC_DEV float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
ACC_DEV void st4(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }
// Streaming (non-temporal) 16-byte accesses for data touched once per kernel: on
// gfx950 a float4 stream with several accesses in flight per thread runs at ~6.2
// TB/s with nt hints vs ~3.8 TB/s without (tools/kbench copy variants).
typedef float accv4 __attribute__((ext_vector_type(4)));
ACC_DEV float4 ld4_nt(const float* p) {
  accv4 v = __builtin_nontemporal_load(reinterpret_cast<const accv4*>(p));
  return make_float4(v.x, v.y, v.z, v.w);
}
ACC_DEV void st4_nt(float* p, float4 v) {
  accv4 w = {v.x, v.y, v.z, v.w};
  __builtin_nontemporal_store(w, reinterpret_cast<accv4*>(p));
}

// ---------------------------------------------------------------------------
// bf16 activation storage (round-to-nearest-even via v_cvt_pk_bf16_f32)
// ---------------------------------------------------------------------------
typedef unsigned short bf16_t;
typedef __bf16 bf16x2_v __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x8_v __attribute__((ext_vector_type(8)));

ACC_DEV float bf2f(bf16_t v) { return __uint_as_float((unsigned)v << 16); }
ACC_DEV bf16_t f2bf(float f) { return __builtin_bit_cast(bf16_t, (__bf16)f); }
ACC_DEV unsigned pack_bf2(float a, float b) {
  bf16x2_v v = {(__bf16)a, (__bf16)b};
  return __builtin_bit_cast(unsigned, v);
}
ACC_DEV float bflo(unsigned u) { return __uint_as_float(u << 16); }
ACC_DEV float bfhi(unsigned u) { return __uint_as_float(u & 0xffff0000u); }

// Typed activation access: fp32 in registers whatever the storage type.
ACC_DEV float ld1(const float* p) { return *p; }
ACC_DEV float ld1(const bf16_t* p) { return bf2f(*p); }
ACC_DEV void st1(float* p, float v) { *p = v; }
ACC_DEV void st1(bf16_t* p, float v) { *p = f2bf(v); }
// channel quads: 16 bytes (fp32) / 8 bytes (bf16)
ACC_DEV float4 ldq(const float* p) { return ld4(p); }
ACC_DEV float4 ldq(const bf16_t* p) {
  const uint2 u = *reinterpret_cast<const uint2*>(p);
  return make_float4(bflo(u.x), bfhi(u.x), bflo(u.y), bfhi(u.y));
}
ACC_DEV void stq(float* p, float4 v) { st4(p, v); }
ACC_DEV void stq(bf16_t* p, float4 v) {
  uint2 u;
  u.x = pack_bf2(v.x, v.y);
  u.y = pack_bf2(v.z, v.w);
  *reinterpret_cast<uint2*>(p) = u;
}
typedef unsigned accu2 __attribute__((ext_vector_type(2)));
ACC_DEV float4 ldq_nt(const float* p) { return ld4_nt(p); }
ACC_DEV float4 ldq_nt(const bf16_t* p) {
  const accu2 u = __builtin_nontemporal_load(reinterpret_cast<const accu2*>(p));
  return make_float4(bflo(u.x), bfhi(u.x), bflo(u.y), bfhi(u.y));
}
ACC_DEV void stq_nt(float* p, float4 v) { st4_nt(p, v); }
ACC_DEV void stq_nt(bf16_t* p, float4 v) {
  accu2 u = {pack_bf2(v.x, v.y), pack_bf2(v.z, v.w)};
  __builtin_nontemporal_store(u, reinterpret_cast<accu2*>(p));
}
// A channel quad as loaded, before widening (float4 / 4 packed bf16). Prefetch
// buffers hold this raw form: widening right after the load would make the
// compiler wait for the load there, not where the data is consumed.
template <typename T> struct QuadRaw;
template <> struct QuadRaw<float> { typedef float4 type; };
template <> struct QuadRaw<bf16_t> { typedef uint2 type; };
ACC_DEV float4 ldq_raw(const float* p, bool nt) { return nt ? ld4_nt(p) : ld4(p); }
ACC_DEV uint2 ldq_raw(const bf16_t* p, bool nt) {
  if (nt) {
    const accu2 u = __builtin_nontemporal_load(reinterpret_cast<const accu2*>(p));
    return make_uint2(u.x, u.y);
  }
  return *reinterpret_cast<const uint2*>(p);
}
ACC_DEV float4 q2f(float4 v) { return v; }
ACC_DEV float4 q2f(uint2 u) { return make_float4(bflo(u.x), bfhi(u.x), bflo(u.y), bfhi(u.y)); }
ACC_DEV void qzero(float4& v) { v = make_float4(0.f, 0.f, 0.f, 0.f); }
ACC_DEV void qzero(uint2& v) { v = make_uint2(0u, 0u); }

// Raw buffer access through a 128-bit resource descriptor whose num_records range
// check loads 0 / drops the store for any offset at or past it (ACC_OOB). Masking
// a lane this way instead of branching around the access keeps the instruction
// stream branch-free, so the compiler knows how many memory operations follow a
// load and can wait for that load alone (s_waitcnt vmcnt(N)), not for vmcnt(0).
// AUX: 0 = default cache policy, 2 = non-temporal. Descriptor bases and sizes
// must be wave-uniform (kernel arguments / blockIdx-derived).
#define ACC_OOB 0x80000000u
// cache policy of the streaming kernels' output stores (BatchNorm apply / backward
// apply, SE apply, SE backward apply): 0 = default, 2 = non-temporal
#ifndef ACC_STREAM_STORE_AUX
#define ACC_STREAM_STORE_AUX 0
#endif
typedef unsigned acc_u32x4 __attribute__((__vector_size__(16)));
typedef unsigned acc_u32x2 __attribute__((__vector_size__(8)));
ACC_DEV __amdgpu_buffer_rsrc_t acc_rsrc(const void* base, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)bytes, 0x00020000);
}
template <int AUX>
ACC_DEV float4 bufq_ld(__amdgpu_buffer_rsrc_t r, unsigned off, const float*) {
  const acc_u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, AUX);
  return make_float4(__uint_as_float(v[0]), __uint_as_float(v[1]), __uint_as_float(v[2]),
                     __uint_as_float(v[3]));
}
template <int AUX>
ACC_DEV uint2 bufq_ld(__amdgpu_buffer_rsrc_t r, unsigned off, const bf16_t*) {
  const acc_u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, AUX);
  return make_uint2(v[0], v[1]);
}
template <int AUX>
ACC_DEV void bufq_st(__amdgpu_buffer_rsrc_t r, unsigned off, float4 v, float*) {
  acc_u32x4 u = {__float_as_uint(v.x), __float_as_uint(v.y), __float_as_uint(v.z),
                 __float_as_uint(v.w)};
  __builtin_amdgcn_raw_buffer_store_b128(u, r, off, 0, AUX);
}
template <int AUX>
ACC_DEV void bufq_st(__amdgpu_buffer_rsrc_t r, unsigned off, float4 v, bf16_t*) {
  acc_u32x2 u = {pack_bf2(v.x, v.y), pack_bf2(v.z, v.w)};
  __builtin_amdgcn_raw_buffer_store_b64(u, r, off, 0, AUX);
}

// the value v takes once stored as T (statistics are taken of what is stored)
ACC_DEV float rnd_as(float v, const float*) { return v; }
ACC_DEV float rnd_as(float v, const bf16_t*) { return bf2f(f2bf(v)); }
template <typename T>
ACC_DEV float rnd(float v) { return rnd_as(v, (const T*)nullptr); }

// Host: run f(T{}) with T = the storage type named by dt (ACC_F32 / ACC_BF16).
template <typename F>
static inline int with_dt(int dt, F f) {
  if (dt == ACC_BF16) { f(bf16_t{}); return ACC_OK; }
  if (dt == ACC_F32) { f(float{}); return ACC_OK; }
  return ACC_EBADARG;
}

// ---- inter-workgroup hand-off: the last block of a group to arrive continues ----
// Published values are stored write-through (agent-scope relaxed atomic store = sc1)
// and every storing wave drains them before the group ticket is taken; the last
// arriver reads them back with agent-scope loads (sc1: L1 bypass). No L2 write-back
// or L1 invalidate fence is needed (MI355X guide section 6, Guideline 16, R1/R2).
// Tickets live in zero-initialised __device__ arrays; the last arriver resets its
// word, so consecutive launches on one stream (and graph replays) reuse them.
typedef __attribute__((address_space(1))) unsigned long long acc_gu64;
typedef __attribute__((address_space(1))) unsigned acc_gu32;
ACC_DEV void st_wt(double* p, double v) {
  __hip_atomic_store((acc_gu64*)p, (unsigned long long)__double_as_longlong(v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
ACC_DEV double ld_wt(const double* p) {
  return __longlong_as_double(
      (long long)__hip_atomic_load((acc_gu64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
ACC_DEV void st_wt(float* p, float v) {
  __hip_atomic_store((acc_gu32*)p, __float_as_uint(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
ACC_DEV float ld_wt(const float* p) {
  return __uint_as_float(__hip_atomic_load((acc_gu32*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
// Every thread of the block calls this after its write-through stores; true (block-
// uniform) in the block whose arrival is the count-th on *ticket.
ACC_DEV bool handoff_last(unsigned* ticket, unsigned count) {
  __shared__ int last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned k = __hip_atomic_fetch_add((acc_gu32*)ticket, 1u, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
    const int me = k == count - 1;
    if (me) __hip_atomic_store((acc_gu32*)ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = me;
  }
  __syncthreads();
  return last;
}

ACC_DEV float f4get(const float4& v, int i) {
  return i == 0 ? v.x : (i == 1 ? v.y : (i == 2 ? v.z : v.w));
}


// the activation as a slope (ACT_NONE: max(v, 1*v) = v), so a runtime act costs no select
ACC_DEV float act_slope(int act) { return act == ACT_LRELU ? LRELU_SLOPE : 1.f; }
ACC_DEV float apply_act(float v, int act) { return __builtin_fmaxf(v, v * act_slope(act)); }

// Per-channel BatchNorm state block produced by bn_finalize:
//   st[0*C + c] = mean, st[1*C + c] = rstd, st[2*C + c] = scale (= gamma*rstd),
//   st[3*C + c] = shift (= beta - mean*scale)
// so that bn(x) = x*scale + shift.
#define BN_MEAN 0
#define BN_RSTD 1
#define BN_SCALE 2
#define BN_SHIFT 3

static inline int ceil_div(long a, long b) { return (int)((a + b - 1) / b); }
