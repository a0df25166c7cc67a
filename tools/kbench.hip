// Standalone kernel microbenchmark for the streaming hot kernels, linked against
// libaccunet_hip.so through the public C ABI (include/accunet.h). No torch, so a
// GPU box runs it in seconds:
//   make -C tools kbench && tools/kbench [iters]
// Reports per-launch average (hipEvent over `iters` back-to-back launches) and
// algorithmic GB/s next to a float4 copy of the same byte count (the practical
// HBM ceiling for this footprint).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include <algorithm>

#include "../include/accunet.h"

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)
#define CA(x)                                                 \
  do {                                                        \
    int r_ = (x);                                             \
    if (r_ != 0) {                                            \
      fprintf(stderr, "%s:%d accunet rc %d\n", __FILE__, __LINE__, r_); \
      exit(1);                                                \
    }                                                         \
  } while (0)

__global__ void copy4(const float4* __restrict__ a, float4* __restrict__ b, long n) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    b[i] = a[i];
}

typedef float v4f __attribute__((ext_vector_type(4)));
__global__ void copy4_nt(const float4* __restrict__ a0, float4* __restrict__ b0, long n) {
  const v4f* a = (const v4f*)a0;
  v4f* b = (v4f*)b0;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    __builtin_nontemporal_store(a[i], &b[i]);
}
__global__ void copy4_flat(const float4* __restrict__ a, float4* __restrict__ b, long n) {
  long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (i < n) b[i] = a[i];
}
// 4 independent float4 per thread per iteration (block-contiguous)
__global__ void copy4_x4(const float4* __restrict__ a, float4* __restrict__ b, long n) {
  long base = (long)blockIdx.x * 1024 + threadIdx.x;
  float4 v[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) if (base + 256 * k < n) v[k] = a[base + 256 * k];
#pragma unroll
  for (int k = 0; k < 4; ++k) if (base + 256 * k < n) b[base + 256 * k] = v[k];
}
__global__ void copy4_x4_nt(const float4* __restrict__ a0, float4* __restrict__ b0, long n) {
  const v4f* a = (const v4f*)a0;
  v4f* b = (v4f*)b0;
  long base = (long)blockIdx.x * 1024 + threadIdx.x;
  v4f v[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) if (base + 256 * k < n) v[k] = __builtin_nontemporal_load(&a[base + 256 * k]);
#pragma unroll
  for (int k = 0; k < 4; ++k) if (base + 256 * k < n) __builtin_nontemporal_store(v[k], &b[base + 256 * k]);
}
// c = a + b, 4 independent float4 per thread (the byte pattern of a 2-read 1-write pass)
__global__ void add4_x4_nt(const float4* __restrict__ a0, const float4* __restrict__ b0,
                           float4* __restrict__ c0, long n) {
  const v4f* a = (const v4f*)a0;
  const v4f* b = (const v4f*)b0;
  v4f* c = (v4f*)c0;
  long base = (long)blockIdx.x * 1024 + threadIdx.x;
  v4f u[4], v[4];
#pragma unroll
  for (int k = 0; k < 4; ++k)
    if (base + 256 * k < n) {
      u[k] = __builtin_nontemporal_load(&a[base + 256 * k]);
      v[k] = __builtin_nontemporal_load(&b[base + 256 * k]);
    }
#pragma unroll
  for (int k = 0; k < 4; ++k) if (base + 256 * k < n) __builtin_nontemporal_store(u[k] + v[k], &c[base + 256 * k]);
}

__global__ void fill(float* p, long n, float s) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    p[i] = s * (float)((i * 2654435761u) % 1000) / 1000.f - 0.5f * s;
}

static float* dalloc(size_t n, float s = 1.f) {
  float* p;
  CK(hipMalloc(&p, n * sizeof(float)));
  hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, p, (long)n, s);
  return p;
}

// median per-launch time (an event pair around every launch): robust to the clock
// ramp / power give-back that makes back-to-back means drift (MI355X DVFS)
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

static void report(const char* name, double us, double bytes) {
  printf("%-44s %9.2f us  %8.1f GB/s  (%.1f%% of 8 TB/s)\n", name, us, bytes / us / 1e3,
         100.0 * bytes / us / 1e3 / 8000.0);
}

// KB_DWSWEEP=1: the step's large depthwise shapes only (forward with prologue + statistics,
// and the flipped data gradient), with whatever kernel the library picks (ACCUNET_DW_OS
// decides between one-shot tiles and strips: run twice to compare)
static void dw_sweep(int iters) {
  struct S { int B, H, W, C; const char* what; };
  const S shapes[] = {{16, 256, 256, 96, "cnv12/92 (K1)"}, {16, 256, 256, 192, "cnv91 (C 192)"},
                      {16, 128, 128, 192, "cnv22/82"}, {16, 128, 128, 384, "cnv81"},
                      {16, 64, 64, 4352, "cnv72 (inv_fctr 34)"}, {16, 64, 64, 384, "cnv32/71"}};
  size_t nmax = 0;
  for (const S& s : shapes) nmax = std::max(nmax, (size_t)s.B * s.H * s.W * s.C);
  float *x = dalloc(nmax), *z = dalloc(nmax), *wt = dalloc(9 * 4352, 0.3f), *bi = dalloc(4352, 0.1f);
  float *sc = dalloc(4352, 1.f), *sh = dalloc(4352, 0.1f);
  for (const S& s : shapes) {
    const int rows = accunet_dw3x3_rows(s.B, s.H, s.W, s.C, ACC_F32, 0);
    double* st;
    CK(hipMalloc(&st, (size_t)rows * 2 * s.C * sizeof(double)));
    const double bytes = 2.0 * 4 * s.B * s.H * s.W * s.C;
    char name[96];
    snprintf(name, sizeof name, "dw fwd %dx%dx%dx%d %s v%d", s.B, s.H, s.W, s.C, s.what,
             accunet_dw3x3_variant(s.B, s.H, s.W, s.C, ACC_F32));
    report(name, timeit([&] { CA(accunet_dw3x3_fwd(x, wt, bi, sc, sh, 1, 0, z, st, s.B, s.H, s.W, s.C, nullptr, nullptr, 0, ACC_F32, 0)); }, iters), bytes);
    snprintf(name, sizeof name, "dw dgrad %dx%dx%dx%d %s", s.B, s.H, s.W, s.C, s.what);
    report(name, timeit([&] { CA(accunet_dw3x3_fwd(x, wt, nullptr, nullptr, nullptr, 0, 1, z, nullptr, s.B, s.H, s.W, s.C, nullptr, nullptr, 0, ACC_F32, 0)); }, iters), bytes);
    CK(hipFree(st));
  }
  CK(hipFree(x)); CK(hipFree(z)); CK(hipFree(wt)); CK(hipFree(bi)); CK(hipFree(sc)); CK(hipFree(sh));
}

int main(int argc, char** argv) {
  int iters = argc > 1 ? atoi(argv[1]) : 30;
  if (getenv("KB_DWSWEEP") && atoi(getenv("KB_DWSWEEP"))) {
    dw_sweep(iters);
    return 0;
  }
  const int B = 16, H = 256, W = 256;
  // ---- K1: cnv12 depthwise, C = 96 ----
  {
    const int C = 96;
    size_t n = (size_t)B * H * W * C;
    float *x = dalloc(n), *z = dalloc(n), *wt = dalloc(9 * C, 0.3f), *bi = dalloc(C, 0.1f);
    float *sc = dalloc(C, 1.f), *sh = dalloc(C, 0.1f);
    // (forward and BN-backward partials, fp32 and bf16: the largest)
    int rows = std::max(std::max(accunet_dw3x3_rows(B, H, W, C, ACC_F32, 0), accunet_dw3x3_rows(B, H, W, C, ACC_F32, 1)),
                        std::max(accunet_dw3x3_rows(B, H, W, C, ACC_BF16, 0), accunet_dw3x3_rows(B, H, W, C, ACC_BF16, 1)));
    double* st;
    CK(hipMalloc(&st, (size_t)rows * 2 * C * sizeof(double)));
    double bytes = 2.0 * 4 * n;
    report("copy float4 (same bytes as K1)",
           timeit([&] { hipLaunchKernelGGL(copy4, dim3(8192), dim3(256), 0, 0, (const float4*)x,
                                           (float4*)z, (long)(n / 4)); }, iters), bytes);
    long n4 = (long)(n / 4);
    report("copy float4 nt-store grid-stride",
           timeit([&] { hipLaunchKernelGGL(copy4_nt, dim3(8192), dim3(256), 0, 0, (const float4*)x,
                                           (float4*)z, n4); }, iters), bytes);
    report("copy float4 flat (1/thread)",
           timeit([&] { hipLaunchKernelGGL(copy4_flat, dim3((n4 + 255) / 256), dim3(256), 0, 0,
                                           (const float4*)x, (float4*)z, n4); }, iters), bytes);
    report("copy float4 x4/thread",
           timeit([&] { hipLaunchKernelGGL(copy4_x4, dim3((n4 + 1023) / 1024), dim3(256), 0, 0,
                                           (const float4*)x, (float4*)z, n4); }, iters), bytes);
    report("copy float4 x4/thread nt",
           timeit([&] { hipLaunchKernelGGL(copy4_x4_nt, dim3((n4 + 1023) / 1024), dim3(256), 0, 0,
                                           (const float4*)x, (float4*)z, n4); }, iters), bytes);
    report("K1 dw3x3_fwd 16x256x256x96 pro+stats",
           timeit([&] { CA(accunet_dw3x3_fwd(x, wt, bi, sc, sh, 1, 0, z, st, B, H, W, C, nullptr, nullptr, 0, ACC_F32, 0)); }, iters),
           bytes);
    {  // bit pattern checksum of z and the stats partials (compare kernel variants)
      std::vector<unsigned> hz(n);
      std::vector<unsigned long long> hs((size_t)rows * 2 * C);
      CK(hipMemcpy(hz.data(), z, n * 4, hipMemcpyDeviceToHost));
      CK(hipMemcpy(hs.data(), st, hs.size() * 8, hipMemcpyDeviceToHost));
      unsigned long long hh = 1469598103934665603ull;
      for (unsigned v : hz) hh = (hh ^ v) * 1099511628211ull;
      for (unsigned long long v : hs) hh = (hh ^ v) * 1099511628211ull;
      printf("K1 checksum %016llx\n", hh);
    }
    report("K1 bf16 dw3x3_fwd 16x256x256x96 pro+stats",
           timeit([&] { CA(accunet_dw3x3_fwd(x, wt, bi, sc, sh, 1, 0, z, st, B, H, W, C, nullptr, nullptr, 0, ACC_BF16, 0)); }, iters),
           bytes / 2);
    {  // cnv91 forward in the bf16 mode: 16x256x256x192 bf16 = the same buffers' bytes
      const int C2 = 2 * C;
      int rows2 = accunet_dw3x3_rows(B, H, W, C2, ACC_BF16, 0);
      double* st2;
      CK(hipMalloc(&st2, (size_t)rows2 * 2 * C2 * sizeof(double)));
      float *wt2 = dalloc(9 * C2, 0.3f), *bi2 = dalloc(C2, 0.1f), *sc2 = dalloc(C2, 1.f),
            *sh2 = dalloc(C2, 0.1f);
      report("K1 bf16 dw3x3_fwd 16x256x256x192 pro+stats",
             timeit([&] { CA(accunet_dw3x3_fwd(x, wt2, bi2, sc2, sh2, 1, 0, z, st2, B, H, W, C2, nullptr, nullptr, 0, ACC_BF16, 0)); }, iters),
             bytes);
      CK(hipFree(st2)); CK(hipFree(wt2)); CK(hipFree(bi2)); CK(hipFree(sc2)); CK(hipFree(sh2));
    }
    report("copy float4 (same bytes as bf16 K1)",
           timeit([&] { hipLaunchKernelGGL(copy4, dim3(8192), dim3(256), 0, 0, (const float4*)x,
                                           (float4*)z, (long)(n / 8)); }, iters), bytes / 2);
    report("K1 dw3x3_fwd flip (dgrad) no pro/stats",
           timeit([&] { CA(accunet_dw3x3_fwd(x, wt, nullptr, nullptr, nullptr, 0, 1, z, nullptr, B, H, W, C, nullptr, nullptr, 0, ACC_F32, 0)); }, iters),
           bytes);
    // what K1's prologue and statistics cost, one at a time (same tile kernel)
    report("K1 dw3x3_fwd pro, no stats",
           timeit([&] { CA(accunet_dw3x3_fwd(x, wt, bi, sc, sh, 1, 0, z, nullptr, B, H, W, C, nullptr, nullptr, 0, ACC_F32, 0)); }, iters),
           bytes);
    report("K1 dw3x3_fwd stats, no pro",
           timeit([&] { CA(accunet_dw3x3_fwd(x, wt, bi, nullptr, nullptr, 0, 0, z, st, B, H, W, C, nullptr, nullptr, 0, ACC_F32, 0)); }, iters),
           bytes);
    {  // the BatchNorm-backward data gradient (flip, bz / bst, BN-backward partials):
       // reads dz and bz, writes dA -- 3 x B*H*W*C*4 bytes
      float *bz = dalloc(n), *bst = dalloc(4 * C, 1.f);
      report("K1 dw3x3_fwd BN-backward dgrad (flip, bz, partials)",
             timeit([&] { CA(accunet_dw3x3_fwd(x, wt, nullptr, nullptr, nullptr, 0, 1, z, st, B, H, W, C, bz, bst, 1, ACC_F32, 0)); }, iters),
             1.5 * bytes);
      report("K1 bf16 BN-backward dgrad (flip, bz, partials)",
             timeit([&] { CA(accunet_dw3x3_fwd(x, wt, nullptr, nullptr, nullptr, 0, 1, z, st, B, H, W, C, bz, bst, 1, ACC_BF16, 0)); }, iters),
             0.75 * bytes);
      CK(hipFree(bz)); CK(hipFree(bst));
    }
    size_t wse = std::max(accunet_dw3x3_wgrad_ws(B, H, W, C, ACC_F32), accunet_dw3x3_wgrad_ws(B, H, W, C, ACC_BF16));
    float* ws = dalloc(wse);
    float *dw = dalloc(9 * C), *db = dalloc(C);
    report("K1' dw3x3_wgrad 16x256x256x96 pro",
           timeit([&] { CA(accunet_dw3x3_wgrad(x, z, sc, sh, 1, dw, db, B, H, W, C, ws, wse, ACC_F32, 0)); }, iters),
           bytes);
    report("K1' bf16 dw3x3_wgrad 16x256x256x96 pro",
           timeit([&] { CA(accunet_dw3x3_wgrad(x, z, sc, sh, 1, dw, db, B, H, W, C, ws, wse, ACC_BF16, 0)); }, iters),
           bytes / 2);
    CK(hipFree(x)); CK(hipFree(z)); CK(hipFree(ws)); CK(hipFree(st));
  }
  // ---- K1 channel-width sweep (1..6 channel groups of 32) ----
  if (getenv("KB_SWEEP")) {
    for (int C : {32, 64, 96, 128, 192}) {
      size_t n = (size_t)B * H * W * C;
      float *x = dalloc(n), *z = dalloc(n), *wt = dalloc(9 * C, 0.3f), *bi = dalloc(C, 0.1f);
      float *sc = dalloc(C, 1.f), *sh = dalloc(C, 0.1f);
      int rows = accunet_dw3x3_rows(B, H, W, C, ACC_F32, 0);
      double* st;
      CK(hipMalloc(&st, (size_t)rows * 2 * C * sizeof(double)));
      char name[96];
      snprintf(name, sizeof name, "K1 sweep 16x256x256x%d", C);
      report(name, timeit([&] { CA(accunet_dw3x3_fwd(x, wt, bi, sc, sh, 1, 0, z, st, B, H, W, C, nullptr, nullptr, 0, ACC_F32, 0)); }, iters),
             2.0 * 4 * n);
      CK(hipFree(x)); CK(hipFree(z)); CK(hipFree(st)); CK(hipFree(wt)); CK(hipFree(bi));
      CK(hipFree(sc)); CK(hipFree(sh));
    }
  }
  // ---- K3: cnv12 SE, C = 32 ----
  {
    const int C = 32, Cr = 4, HW = H * W;
    size_t n = (size_t)B * HW * C;
    float *z = dalloc(n), *out = dalloc(n), *dout = dalloc(n), *da = dalloc(n);
    float *sc = dalloc(C, 1.f), *sh = dalloc(C, 0.1f);
    float *w1 = dalloc(Cr * C, 0.3f), *b1 = dalloc(Cr, 0.1f), *w2 = dalloc(C * Cr, 0.3f),
          *b2 = dalloc(C, 0.1f), *g = dalloc(C, 1.f), *be = dalloc(C, 0.1f), *rm = dalloc(C),
          *rv = dalloc(C);
    float *dw1 = dalloc(Cr * C), *db1 = dalloc(Cr), *dw2 = dalloc(C * Cr), *db2 = dalloc(C),
          *dg = dalloc(C), *dbe = dalloc(C);
    float* save = dalloc(accunet_se_save_elems(B, C, Cr));
    size_t wse = accunet_se_ws_elems(B, HW, C, Cr);
    float* ws = dalloc(wse);
    double bytes = 2.0 * 4 * n;
    report("copy float4 (same bytes as K3)",
           timeit([&] { hipLaunchKernelGGL(copy4, dim3(8192), dim3(256), 0, 0, (const float4*)z,
                                           (float4*)out, (long)(n / 4)); }, iters), bytes);
    {
      int rows = accunet_stream_rows((long)B * HW, C);
      double* st2;
      CK(hipMalloc(&st2, (size_t)rows * 2 * C * sizeof(double)));
      report("affine_act+stats 16x65536x32 (1 rd + 1 wr)",
             timeit([&] { CA(accunet_affine_act_fwd(z, sc, sh, 1, nullptr, out, (long)B * HW, C, st2,
                                                    nullptr, ACC_F32, 0)); }, iters), bytes);
      float* stb = dalloc(4 * C, 1.f);
      size_t bws = accunet_bn_bwd_ws_elems((long)B * HW, C);
      float* bw = dalloc(bws);
      report("bn_bwd 16x65536x32 (rd 2 + rd 2 + wr 1)",
             timeit([&] { CA(accunet_bn_bwd(z, dout, stb, g, 1, 1, (long)B * HW, C, da, 0, dg, dbe,
                                            nullptr, bw, bws, ACC_F32, 0)); }, iters),
             5.0 * 4 * n);
      // the BatchNorm backward whose reduce ran in the producer's epilogue (finish + apply)
      const int R = 64;
      double* bpart;
      CK(hipMalloc(&bpart, (size_t)R * 2 * C * sizeof(double)));
      CK(hipMemset(bpart, 0, (size_t)R * 2 * C * sizeof(double)));
      size_t pws = accunet_bn_bwd_part_ws_elems((long)B * HW, R, C);
      float* pw = dalloc(pws);
      report("add float4 x4/thread nt (2 rd + 1 wr)",
             timeit([&] { hipLaunchKernelGGL(add4_x4_nt, dim3((unsigned)((n / 4 + 1023) / 1024)), dim3(256), 0, 0,
                                             (const float4*)z, (const float4*)dout, (float4*)da, (long)(n / 4)); }, iters),
             3.0 * 4 * n);
      report("bn_bwd apply 16x65536x32 (2 rd + 1 wr)",
             timeit([&] { CA(accunet_bn_bwd_part(z, dout, stb, g, 1, 1, (long)B * HW, C, bpart, R, da, dg, dbe,
                                                 nullptr, pw, pws, ACC_F32, 0)); }, iters),
             3.0 * 4 * n);
      report("bn_bwd apply bf16 16x65536x32",
             timeit([&] { CA(accunet_bn_bwd_part(z, dout, stb, g, 1, 1, (long)B * HW, C, bpart, R, da, dg, dbe,
                                                 nullptr, pw, pws, ACC_BF16, 0)); }, iters),
             3.0 * 2 * n);
      CK(hipFree(bpart));
    }
    report("K3 se_fwd 16x65536x32 pro",
           timeit([&] { CA(accunet_se_fwd(z, sc, sh, 1, B, HW, C, Cr, w1, b1, w2, b2, g, be, rm, rv,
                                          nullptr, 0.1f, 1e-5f, 1, out, nullptr, save, nullptr, ws, wse, ACC_F32, 0)); }, iters),
           bytes);
    report("K3' se_bwd 16x65536x32 pro (2 rd + 1 rd/wr)",
           timeit([&] { CA(accunet_se_bwd(z, dout, sc, sh, 1, B, HW, C, Cr, w1, w2, g, 1, save, da,
                                          dw1, db1, dw2, db2, dg, dbe, ws, wse, ACC_F32, 0)); }, iters),
           4.0 * 4 * n);
    // the fused SE + prologue-BN backward the model runs (HANC / ResPath / MLFC)
    float *pst = dalloc(4 * C, 1.f), *pg = dalloc(C, 1.f), *dpg = dalloc(C), *dpb = dalloc(C);
    report("K3' se_bwd_pro 16x65536x32 (2 rd + 2 rd + 1 wr)",
           timeit([&] { CA(accunet_se_bwd_pro(z, dout, pst, 1, pg, 1, B, HW, C, Cr, w1, w2, g, 1, save,
                                              da, dpg, dpb, nullptr, dw1, db1, dw2, db2, dg, dbe, ws,
                                              wse, ACC_F32, 0)); }, iters),
           5.0 * 4 * n);
    report("K3' bf16 se_bwd_pro 16x65536x32",
           timeit([&] { CA(accunet_se_bwd_pro(z, dout, pst, 1, pg, 1, B, HW, C, Cr, w1, w2, g, 1, save,
                                              da, dpg, dpb, nullptr, dw1, db1, dw2, db2, dg, dbe, ws,
                                              wse, ACC_BF16, 0)); }, iters),
           5.0 * 2 * n);
  }
  {  // cnv72's BatchNorm backward apply (16 x 64 x 64 pixels x 4352 channels)
    const long P = 16L * 64 * 64;
    const int C = 4352, R = 64;
    const size_t n = (size_t)P * C;
    float *x = dalloc(n), *dy = dalloc(n), *dx = dalloc(n);
    float *st = dalloc(4 * C, 1.f), *ga = dalloc(C, 1.f), *dg = dalloc(C), *dbe = dalloc(C);
    double* bpart;
    CK(hipMalloc(&bpart, (size_t)R * 2 * C * sizeof(double)));
    CK(hipMemset(bpart, 0, (size_t)R * 2 * C * sizeof(double)));
    size_t pws = accunet_bn_bwd_part_ws_elems(P, R, C);
    float* pw = dalloc(pws);
    report("add float4 x4/thread nt 65536x4352",
           timeit([&] { hipLaunchKernelGGL(add4_x4_nt, dim3((unsigned)((n / 4 + 1023) / 1024)), dim3(256), 0, 0,
                                           (const float4*)x, (const float4*)dy, (float4*)dx, (long)(n / 4)); }, iters),
           3.0 * 4 * n);
    report("bn_bwd apply 65536x4352 (2 rd + 1 wr)",
           timeit([&] { CA(accunet_bn_bwd_part(x, dy, st, ga, 1, 1, P, C, bpart, R, dx, dg, dbe, nullptr, pw,
                                               pws, ACC_F32, 0)); }, iters),
           3.0 * 4 * n);
    report("bn_bwd apply bf16 65536x4352",
           timeit([&] { CA(accunet_bn_bwd_part(x, dy, st, ga, 1, 1, P, C, bpart, R, dx, dg, dbe, nullptr, pw,
                                               pws, ACC_BF16, 0)); }, iters),
           3.0 * 2 * n);
    CK(hipFree(x)); CK(hipFree(dy)); CK(hipFree(dx)); CK(hipFree(bpart)); CK(hipFree(pw));
  }
  CK(hipDeviceSynchronize());
  return 0;
}
