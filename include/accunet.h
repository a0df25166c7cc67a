/*
 * accunet.h — C ABI of libaccunet_hip.so, the MI355X (gfx950) kernels behind the
 * ACC-UNet drop-in (acc-unet-unext_amd/accunet/model.py: ACC_UNet).
 *
 * Conventions
 *   - every tensor is fp32, NHWC (channels-last), contiguous unless an explicit
 *     leading dimension is given; a [B,H,W,C] activation is a row-major matrix
 *     [P = B*H*W][C].
 *   - pointers are device pointers; `stream` is a hipStream_t passed as void*
 *     (kernels are enqueued on it, nothing synchronises the host).
 *   - every entry point returns 0 (ACC_OK) or a negative code:
 *       -1 bad shape, -2 bad argument / workspace too small, -3 launch failure.
 *   - no entry point allocates memory: scratch ("ws") is caller provided
 *     (the Python host takes it from the PyTorch caching allocator).
 *
 * The reference implements this path as PyTorch modules whose arithmetic runs in
 * ATen/cuDNN (ACC_UNet/ACC_UNet.py). Each group below names the reference module
 * (file:line) whose computation it replaces.
 */
#ifndef ACCUNET_H
#define ACCUNET_H
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------------------------- *
 * GEMM engine (fp32 MFMA 32x32x2).  Replaces every nn.Conv2d 1x1 / 3x3 forward
 * and their autograd data/weight gradients:
 *   HANCBlock.conv1/conv3  ACC_UNet/ACC_UNet.py:233,259
 *   HANCLayer.cnv          ACC_UNet/ACC_UNet.py:72,140 (restructured)
 *   Conv2d_batchnorm.conv1 ACC_UNet/ACC_UNet.py:171,183 (MLFC)
 *   ResPath.convs          ACC_UNet/ACC_UNet.py:317-318 (3x3, amode=AMODE_SHIFT3)
 *   ConvTranspose2d up6..9 ACC_UNet/ACC_UNet.py:578-590 (pixel-shuffled GEMM)
 * C[m,n] = sum_k A(m,k) B(k,n) (+bias[n]) (+ sum_u up_u[pixel(m)>>uplog_u][n])
 * ------------------------------------------------------------------------- */
enum { AMODE_ROW = 0, AMODE_COL = 1, AMODE_SHIFT3 = 2 };
enum { BMODE_NT = 0, BMODE_NN = 1, BMODE_NN_SHIFT3 = 2 };
enum { PRO_NONE = 0, PRO_AFFINE = 1, PRO_AFFINE_LRELU = 2 };
enum { ACT_NONE = 0, ACT_LRELU = 1 };

typedef struct AccGemmDesc {
  int M, N, K;
  int amode, bmode, pro_a, pro_b;
  int nsrc;                 /* AMODE_ROW: up to 4 channel-concatenated A sources */
  const float* a[4];
  int lda[4];
  int kbeg[5];              /* source s covers k in [kbeg[s], kbeg[s+1]) */
  const float* a_scale;     /* prologue act(x*scale[k]+shift[k]) on A (AMODE_ROW) */
  const float* a_shift;
  const float* b;
  int ldb;
  const float* b_scale;     /* prologue on B's n axis (BMODE_NN) */
  const float* b_shift;
  int H, W, cin;            /* pixel grid (SHIFT3 modes, up-adds); channels per tap */
  float* c;
  int ldc;
  const float* bias;        /* [N] or NULL */
  int nup;                  /* 0..3 nearest-upsampled addends */
  const float* up[3];
  int upld[3];
  int uplog[3];
  float* stats;             /* [rows][2][N] partial (sum,sumsq) of C, or NULL */
  int allow_split;          /* split-K through ws (weight gradients) */
} AccGemmDesc;

int accunet_gemm(const AccGemmDesc* d, float* ws, size_t ws_elems, void* stream);
/* number of partial-statistics rows accunet_gemm writes for this shape */
int accunet_gemm_stats_rows(int M, int N, int amode, int bmode, int cin);

/* ------------------------------------------------------------------------- *
 * BatchNorm2d (training: batch statistics, running-stat update with momentum
 * and unbiased variance; eval: running statistics) + LeakyReLU(0.01).
 * Replaces torch.nn.BatchNorm2d / LeakyReLU used at ACC_UNet/ACC_UNet.py
 * :235-262 (HANCBlock norms), :73-74 (HANCLayer), :172-184 (Conv2d_batchnorm),
 * :309-325 (ResPath), :393-414 (MLFC).
 * st = [4][C]: mean, rstd, scale(=gamma*rstd), shift(=beta-mean*scale)
 * ------------------------------------------------------------------------- */
int accunet_stream_rows(long P, int C);
int accunet_bn_finalize(const float* part, int R, int C, double count, const float* gamma,
                        const float* beta, float* rmean, float* rvar, long long* nbt,
                        float momentum, float eps, int training, float* st, float* ws,
                        void* stream);
int accunet_affine_act_fwd(const float* x, const float* sc, const float* sh, int act,
                           const float* res, float* y, long P, int C, float* stats,
                           int* stats_rows, void* stream);
int accunet_bn_bwd(const float* x, const float* dy, const float* st, const float* gamma, int act,
                   int training, long P, int C, float* dx, int accumulate, float* dgamma,
                   float* dbeta, float* colsum, int* colsum_rows, float* ws, size_t ws_elems,
                   void* stream);
int accunet_colsum(const float* x, long P, int C, float* out, float* ws, size_t ws_elems,
                   void* stream);
int accunet_reduce_stats(const float* part, int R, int C, float* out2C, float* ws, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* ACCUNET_H */
