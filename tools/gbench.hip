// Standalone fp32 GEMM microbenchmark through the C ABI (accunet_gemm): representative
// ACC-UNet training-step shapes, median of per-launch HIP-event times, TFLOP/s against
// the 157.3 TF fp32 MFMA peak. Links the in-tree libaccunet_hip.so:
//   make -C tools gbench && tools/gbench [iters]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
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

struct Shape {
  const char* name;
  int M, N, K, amode, bmode, pro_a, stats, split, H, W, cin;
  int pyr = 0;  // HANCLayer pyramid backward + BatchNorm-backward statistics epilogue
};

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 20;
  const Shape shapes[] = {
      {"cnv72 x-branch fwd  65536x128x4352 NT proA stats", 65536, 128, 4352, AMODE_ROW, BMODE_NT, PRO_AFFINE_LRELU, 1, 0, 0, 0, 0},
      {"cnv72 conv1 fwd     65536x4352x128 NT stats", 65536, 4352, 128, AMODE_ROW, BMODE_NT, PRO_NONE, 1, 0, 0, 0, 0},
      {"cnv12 conv1 fwd   1048576x96x32 NT stats", 1048576, 96, 32, AMODE_ROW, BMODE_NT, PRO_NONE, 1, 0, 0, 0, 0},
      {"cnv32 hnc fwd      262144x128x384 NT proA stats", 262144, 128, 384, AMODE_ROW, BMODE_NT, PRO_AFFINE_LRELU, 1, 0, 0, 0, 0},
      {"cnv72 x dgrad       65536x4352x128 NN", 65536, 4352, 128, AMODE_ROW, BMODE_NN, PRO_NONE, 0, 0, 0, 0, 0},
      {"cnv72 pyr dgrad     65536x4352x128 NN bnb+pyr", 65536, 4352, 128, AMODE_ROW, BMODE_NN, PRO_NONE, 1, 0, 64, 64, 0, 1},
      {"k64 cnv91 pyr dgrad   1048576x192x64 NN bnb+pyr", 1048576, 192, 64, AMODE_ROW, BMODE_NN, PRO_NONE, 1, 0, 256, 256, 0, 1},
      {"k64 cnv81 pyr dgrad    262144x192x64 NN bnb+pyr", 262144, 192, 64, AMODE_ROW, BMODE_NN, PRO_NONE, 1, 0, 128, 128, 0, 1},
      {"cnv92 pyr dgrad   1048576x96x32 NN bnb+pyr", 1048576, 96, 32, AMODE_ROW, BMODE_NN, PRO_NONE, 1, 0, 256, 256, 0, 1},
      {"cnv32 pyr dgrad    262144x384x128 NN bnb+pyr", 262144, 384, 128, AMODE_ROW, BMODE_NN, PRO_NONE, 1, 0, 128, 128, 0, 1},
      {"cnv72 x wgrad       4352x128x65536 COL NN split", 4352, 128, 65536, AMODE_COL, BMODE_NN, PRO_NONE, 0, 1, 0, 0, 0},
      {"rspth1 3x3 fwd   1048576x32x288 SHIFT3 stats", 1048576, 32, 288, AMODE_SHIFT3, BMODE_NT, PRO_NONE, 1, 0, 256, 256, 32},
      {"rspth1 3x3 wgrad    32x288x1048576 COL SHIFT3 split", 32, 288, 1048576, AMODE_COL, BMODE_NN_SHIFT3, PRO_NONE, 0, 1, 256, 256, 32},
      {"rspth2 3x3 fwd    262144x64x576 SHIFT3 stats", 262144, 64, 576, AMODE_SHIFT3, BMODE_NT, PRO_NONE, 1, 0, 128, 128, 64},
      {"rspth2 3x3 wgrad    64x576x262144 COL SHIFT3 split", 64, 576, 262144, AMODE_COL, BMODE_NN_SHIFT3, PRO_NONE, 0, 1, 128, 128, 64},
      {"rspth3 3x3 fwd     65536x128x1152 SHIFT3 stats", 65536, 128, 1152, AMODE_SHIFT3, BMODE_NT, PRO_NONE, 1, 0, 64, 64, 128},
      {"rspth3 3x3 wgrad   128x1152x65536 COL SHIFT3 split", 128, 1152, 65536, AMODE_COL, BMODE_NN_SHIFT3, PRO_NONE, 0, 1, 64, 64, 128},
      {"rspth2w 3x3 wgrad   64x576x262144 COL SHIFT3 split", 64, 576, 262144, AMODE_COL, BMODE_NN_SHIFT3, PRO_NONE, 0, 1, 128, 128, 64},
      {"k64 cnv91 conv1-like fwd 1048576x192x64 NT stats", 1048576, 192, 64, AMODE_ROW, BMODE_NT, PRO_NONE, 1, 0, 0, 0, 0},
      {"k64 cnv81 conv1-like fwd  262144x192x64 NT stats", 262144, 192, 64, AMODE_ROW, BMODE_NT, PRO_NONE, 1, 0, 0, 0, 0},
      {"k64 dgrad 1048576x192x64 NN", 1048576, 192, 64, AMODE_ROW, BMODE_NN, PRO_NONE, 0, 0, 0, 0, 0},
      {"narrow conv 1x1 fwd 1048576x32x96 NT stats", 1048576, 32, 96, AMODE_ROW, BMODE_NT, PRO_NONE, 1, 0, 0, 0, 0},
  };
  // operand buffers sized for the largest shape (65536 x 4352 activations, 1M x 32 for B
  // of the 3x3 weight gradient)
  const size_t nA = (size_t)300 << 20, nB = (size_t)40 << 20, nC = (size_t)300 << 20;
  float *A = dalloc(nA), *B = dalloc(nB, 0.1f), *C = dalloc(nC);
  float *sc = dalloc(8192, 1.f), *sh = dalloc(8192, 0.1f);
  const size_t wse = (size_t)1 << 26;
  float* ws = dalloc(wse);
  // statistics partials: [ceil(M / BM)][2][N] doubles; BM >= 32 for every tile, so
  // 65536/32 x 2 x 4352 x 8 B (142 MB) bounds any tile choice (ACCUNET_GEMM_TILE)
  double* st;
  CK(hipMalloc(&st, (size_t)160 << 20));
  // pyramid-backward operands of the 65536x4352 data gradient (16 x 64 x 64 pixels):
  // bz [M][N], dP2 [M/4][2N], dP4 [M/16][2N], codes [M/4][N], [M/16][N]
  const size_t PM = 65536, PN = 4352;
  float* bz = dalloc(PM * PN);
  float* bst = dalloc(4 * PN, 0.5f);
  float* pd2 = dalloc(PM / 4 * 2 * PN, 0.1f);
  float* pd4 = dalloc(PM / 16 * 2 * PN, 0.1f);
  unsigned char *mk2, *mk4;
  CK(hipMalloc(&mk2, PM / 4 * PN));
  CK(hipMalloc(&mk4, PM / 16 * PN));
  CK(hipMemset(mk2, 1, PM / 4 * PN));
  CK(hipMemset(mk4, 5, PM / 16 * PN));
  const char* only = getenv("GB_ONLY");  // run only the shapes whose name contains this
  for (const Shape& s : shapes) {
    if (only && !strstr(s.name, only)) continue;
    AccGemmDesc d;
    memset(&d, 0, sizeof(d));
    d.M = s.M; d.N = s.N; d.K = s.K;
    d.amode = s.amode; d.bmode = s.bmode; d.pro_a = s.pro_a; d.pro_b = PRO_NONE;
    d.nsrc = 1;
    d.a[0] = A;
    d.lda[0] = s.amode == AMODE_COL ? s.M : (s.amode == AMODE_SHIFT3 ? s.cin : s.K);
    d.kbeg[0] = 0; d.kbeg[1] = s.K;
    d.a_scale = s.pro_a ? sc : nullptr;
    d.a_shift = s.pro_a ? sh : nullptr;
    d.b = B;
    d.ldb = s.bmode == BMODE_NT ? s.K : (s.bmode == BMODE_NN_SHIFT3 ? s.cin : s.N);
    d.H = s.H; d.W = s.W; d.cin = s.cin;
    d.c = C; d.ldc = s.N;
    d.stats = s.stats ? st : nullptr;
    d.allow_split = s.split;
    d.adt = d.bdt = d.cdt = ACC_F32;
    if (s.pyr) {
      d.bz = bz; d.bst = bst; d.bact = 1;
      d.pd2 = pd2; d.pd4 = pd4; d.mk2 = mk2; d.mk4 = mk4;
    }
    const double us = timeit([&] {
      int r = accunet_gemm(&d, ws, wse, 0);
      if (r) { fprintf(stderr, "accunet_gemm rc %d (%s)\n", r, s.name); exit(1); }
    }, iters);
    const double tf = 2.0 * s.M * s.N * (double)s.K / us / 1e6;
    printf("%-54s %9.2f us %7.1f TF/s (%.3f of 157.3)\n", s.name, us, tf, tf / 157.3);
    fflush(stdout);
  }
  CK(hipDeviceSynchronize());
  return 0;
}
