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
 * GEMM engines (fp32 MFMA 32x32x2 / bf16 MFMA 32x32x16).  Replaces every nn.Conv2d 1x1 / 3x3 forward
 * and their autograd data/weight gradients:
 *   HANCBlock.conv1/conv3  ACC_UNet/ACC_UNet.py:233,259
 *   HANCLayer.cnv          ACC_UNet/ACC_UNet.py:72,140 (restructured)
 *   Conv2d_batchnorm.conv1 ACC_UNet/ACC_UNet.py:171,183 (MLFC)
 *   ResPath.convs          ACC_UNet/ACC_UNet.py:317-318 (3x3, amode=AMODE_SHIFT3)
 *   ConvTranspose2d up6..9 ACC_UNet/ACC_UNet.py:578-590 (pixel-shuffled GEMM)
 * C[m,n] = sum_k A(m,k) B(k,n) (+bias[n]) (+ sum_u up_u[pixel(m)>>uplog_u][n])
 * ------------------------------------------------------------------------- */
/* Activation storage types (`dt` arguments, AccGemmDesc.adt/bdt/cdt): the
 * activation-shaped tensors of a call (inputs, outputs, activation gradients,
 * pyramid / upsample operands) are fp32 or bf16; parameters, parameter gradients,
 * BatchNorm / SE state are always fp32 and partial statistics fp64. */
enum { ACC_F32 = 0, ACC_BF16 = 1 };

enum { AMODE_ROW = 0, AMODE_COL = 1, AMODE_SHIFT3 = 2 };
enum { BMODE_NT = 0, BMODE_NN = 1, BMODE_NN_SHIFT3 = 2 };
enum { PRO_NONE = 0, PRO_AFFINE = 1, PRO_AFFINE_LRELU = 2 };
enum { ACT_NONE = 0, ACT_LRELU = 1 };

typedef struct AccGemmDesc {
  int M, N, K;
  int amode, bmode, pro_a, pro_b;
  int nsrc;                 /* AMODE_ROW: up to 4 channel-concatenated A sources */
  const void* a[4];         /* storage adt */
  int lda[4];
  int kbeg[5];              /* source s covers k in [kbeg[s], kbeg[s+1]) */
  const float* a_scale;     /* prologue act(x*scale[k]+shift[k]) on A (AMODE_ROW) */
  const float* a_shift;
  const void* b;            /* storage bdt */
  int ldb;
  const float* b_scale;     /* prologue on B's n axis (BMODE_NN) */
  const float* b_shift;
  int H, W, cin;            /* pixel grid (SHIFT3 modes, up-adds); channels per tap */
  void* c;                  /* storage cdt (also up[], pd2/pd4, bz) */
  int ldc;
  const float* bias;        /* [N] or NULL */
  int nup;                  /* 0..3 nearest-upsampled addends */
  const void* up[3];
  int upld[3];
  int uplog[3];
  double* stats;            /* [rows][2][N] fp64 partial (sum,sumsq) of C, or NULL */
  int allow_split;          /* split-K through ws (weight gradients) */
  /* HANCLayer pyramid backward fused into the x-branch data-gradient epilogue
   * (ACC_UNet/ACC_UNet.py:86-106 pooling + nearest upsample, differentiated):
   * C[m,n] += dP2avg/4 + [argmax2 == pos] dP2max + dP4avg/16 + [argmax4 == pos] dP4max
   * with dP2 = pd2 [P/4][2N] ([avg | max] columns), dP4 = pd4 [P/16][2N] (or NULL),
   * mk2 [P/4][N], mk4 [P/16][N] the first-max codes written by
   * accunet_hanc_pyramid_fwd. pd2 == NULL disables it. */
  const void* pd2;
  const void* pd4;
  const unsigned char* mk2;
  const unsigned char* mk4;
  /* BatchNorm backward statistics in the epilogue (data gradients whose input went
   * through a pending BatchNorm(+LeakyReLU) prologue in the forward): with bz the
   * pre-BN input z [M][ldc] and bst its [4][N] state block, `stats` receives per-row-
   * block (sum g, sum g*(z - mean)) of g = C * act'(z*scale + shift) instead of
   * (sum C, sum C^2); accunet_bn_bwd_part finishes the BatchNorm backward. */
  const void* bz;
  const float* bst;
  int bact;
  /* storage of A, B and C (ACC_F32 / ACC_BF16). All fp32: fp32 engine (fp32 MFMA).
   * adt = ACC_BF16: bf16 engine (v_mfma_f32_32x32x16_bf16) with either bdt = ACC_F32
   * (weights, rounded to bf16 on load) and cdt = ACC_BF16 (forward / data gradients),
   * or bdt = ACC_BF16 and cdt = ACC_F32 (amode = AMODE_COL weight gradients). */
  int adt, bdt, cdt;
} AccGemmDesc;

int accunet_gemm(const AccGemmDesc* d, float* ws, size_t ws_elems, void* stream);
/* number of partial-statistics rows accunet_gemm writes for this shape */
int accunet_gemm_stats_rows(int M, int N, int K, int amode, int bmode, int cin);

/* ------------------------------------------------------------------------- *
 * BatchNorm2d (training: batch statistics, running-stat update with momentum
 * and unbiased variance; eval: running statistics) + LeakyReLU(0.01).
 * Replaces torch.nn.BatchNorm2d / LeakyReLU used at ACC_UNet/ACC_UNet.py
 * :235-262 (HANCBlock norms), :73-74 (HANCLayer), :172-184 (Conv2d_batchnorm),
 * :309-325 (ResPath), :393-414 (MLFC).
 * st = [4][C]: mean, rstd, scale(=gamma*rstd), shift(=beta-mean*scale)
 * Statistics partial blocks ("stats"/"part": [rows][2][C] sum, sum of squares) are
 * fp64 everywhere (ATen's CPU BatchNorm also accumulates in double).
 * ------------------------------------------------------------------------- */
int accunet_stream_rows(long P, int C);
/* Ticket bank (0 or 1) of the one-launch statistics reductions enqueued on `stream`
 * (their last-arriver hand-off counts arrivals in a per-device ticket array): streams
 * that may run reductions concurrently must use different banks. Unregistered streams
 * (and the null stream) use bank 0; the registration is keyed by the stream, so it
 * holds whatever host thread enqueues the launch. Returns 0, or -2 for a bank outside
 * 0..1, a null stream or a full table (64 streams). No reference counterpart (the
 * reference's reductions are ATen's). */
int accunet_stream_ticket_bank(void* stream, int bank);
/* Drop a stream's registration (call before destroying a registered stream, so a
 * later stream that reuses the handle does not inherit its bank). Returns 0, or -2
 * for a null or unregistered stream. */
int accunet_stream_ticket_unregister(void* stream);
/* ABI identity: the first 15 hex digits of this header's sha256, fixed when the
 * library was built. The Python binding refuses a library whose hash differs from
 * the header it binds against. */
long long accunet_abi_hash(void);
/* Diagnostic: how many launches of the ResPath halo-tile 3x3 kernels (forward / data
 * gradient, and weight gradient) accunet_gemm has made in this process since it was
 * loaded (host-side counts; a launch captured into a graph counts once). Lets a test
 * prove which implementation ran. No reference counterpart. */
long long accunet_conv3x3_halo_launches(int wgrad);
int accunet_bn_finalize(const double* part, int R, int C, double count, const float* gamma,
                        const float* beta, float* rmean, float* rvar, long long* nbt,
                        float momentum, float eps, int training, float* st, double* ws,
                        void* stream);
int accunet_affine_act_fwd(const void* x, const float* sc, const float* sh, int act,
                           const void* res, void* y, long P, int C, double* stats,
                           int* stats_rows, int dt, void* stream);
size_t accunet_bn_bwd_ws_elems(long P, int C);
/* dsum (optional, [C]) receives sum_p dx: the bias gradient of the convolution whose
 * output x feeds only this BatchNorm, without a separate pass over dx. */
int accunet_bn_bwd(const void* x, const void* dy, const float* st, const float* gamma, int act,
                   int training, long P, int C, void* dx, int accumulate, float* dgamma,
                   float* dbeta, float* dsum, float* ws, size_t ws_elems, int dt, void* stream);
/* BatchNorm backward from producer-side partials: part = [R][2][C] (sum g,
 * sum g*(x - mean)) written by a data-gradient epilogue (AccGemmDesc.bz,
 * accunet_dw3x3_fwd bz) -> dgamma, dbeta, dx = k1*g + k2*(x - mean) + k3 in one
 * streaming pass (the reduce pass of accunet_bn_bwd is skipped). */
size_t accunet_bn_bwd_part_ws_elems(long P, int R, int C);
int accunet_bn_bwd_part(const void* x, const void* dy, const float* st, const float* gamma,
                        int act, int training, long P, int C, const double* part, int R,
                        void* dx, float* dgamma, float* dbeta, float* dsum, float* ws,
                        size_t ws_elems, int dt, void* stream);
int accunet_colsum(const void* x, long P, int C, float* out, double* ws, size_t ws_elems,
                   int dt, void* stream);
int accunet_reduce_stats(const double* part, int R, int C, double* out2C, double* ws,
                         void* stream);

/* ------------------------------------------------------------------------- *
 * HANCBlock.conv2 — depthwise 3x3 (+bias), pad 1, groups = C
 * (ACC_UNet/ACC_UNet.py:240-247, forward :273). Input may carry a pending
 * BatchNorm+LeakyReLU (sc/sh/act, norm1 :236) applied on load; `stats` receives
 * per-block (sum, sumsq) of z for norm2. flip=1 runs the kernel with W[c][8-tap]
 * (the data gradient); with bz/bst/bact (the pre-BN input of norm1 and its state)
 * `stats` then receives the BatchNorm-backward partials (sum g, sum g*(bz - mean)),
 * g = out * act'(bz*scale + shift), for accunet_bn_bwd_part. wgrad writes dW [C][1][3][3] and db [C].
 * Both return -1 (bad shape) when one image, H*W*C elements as stored, reaches 2 GiB:
 * the kernels address an image through a 32-bit buffer descriptor.
 * ------------------------------------------------------------------------- */
/* rows of `stats` ([rows][2][C] fp64) accunet_dw3x3_fwd writes for this shape and
 * storage dtype dt (bf16 runs 64-channel tiles where C % 64 == 0): the forward's norm2
 * partials (bnb = 0) or the BN-backward data gradient's (bnb = 1, bz given); the two
 * launch kinds may run different tile kernels. */
int accunet_dw3x3_rows(int B, int H, int W, int C, int dt, int bnb);
/* Which forward kernel runs for the shape and storage dtype dt (without bz): 3 = one-shot
 * 8-row tiles (fp32, C % 32 == 0, inputs above 256 MB), 1 = the LDS strip kernel (the
 * other C % 32 == 0 shapes), 0 = register-window kernel; 2 = whole-pixel span kernel,
 * only with the tuning knob ACCUNET_DW_SPAN bit 2 set (off by default) and then for
 * C % 8 == 0, C/4 <= 64. */
int accunet_dw3x3_variant(int B, int H, int W, int C, int dt);
int accunet_dw3x3_fwd(const void* x, const float* wt, const float* bias, const float* sc,
                      const float* sh, int act, int flip, void* z, double* stats, int B, int H,
                      int W, int C, const void* bz, const float* bst, int bact, int dt,
                      void* stream);
size_t accunet_dw3x3_wgrad_ws(int B, int H, int W, int C, int dt);
int accunet_dw3x3_wgrad(const void* x, const void* dz, const float* sc, const float* sh,
                        int act, float* dw, float* db, int B, int H, int W, int C, float* ws,
                        size_t ws_elems, int dt, void* stream);

/* ------------------------------------------------------------------------- *
 * Batched forward-layout weight copies (the graph-mode training step makes them all
 * in one launch before each replay, accunet/ops.py WeightPrep): `items_dev` is a
 * device array of n AccRelayout, blk0 ascending from 0, item i owning blocks
 * [blk0_i, blk0_{i+1}) with accunet_relayout_blocks(total_i) blocks; nblocks = their
 * sum. kind 0 = the gather of accunet_permute4 (d, s, flip), kind 1 = the forward of
 * accunet_group_relayout (N, C, J, order), kind 2 = its inverse (the backward's weight
 * gradients back into the reference layout, ops.DeferredRelayouts; total = N*J*C),
 * kind 3 = flat copy in -> out (fp32), kind 4 = flat copy with `out` a bf16 array
 * (round to nearest even): the data-parallel gradient-bucket packing, each value
 * multiplied by `scale` first (1/world: the packed gradients are pre-divided, so the
 * RCCL all-reduce is a plain SUM, the PreMulSum form of AVG). `in` is fp32.
 * ------------------------------------------------------------------------- */
typedef struct AccRelayout {
  const float* in;
  float* out;
  long long total;
  int kind;
  int blk0;
  int d[4];
  long long s[4];
  int flip[4];
  int N, C, J;
  int order[8];
  float scale; /* kinds 3 / 4 */
} AccRelayout;
int accunet_relayout_blocks(long long total);
int accunet_relayout_batch(const void* items_dev, int n, int nblocks, void* stream);

/* ------------------------------------------------------------------------- *
 * HANCLayer neighbourhood pyramid (ACC_UNet/ACC_UNet.py:86-106): from
 * a = act(x*sc+sh): P2 = [avg2 a | max2 a] at H/2, P4 = [avg4 a | max4 a] at H/4
 * (k = 3) in one read. mk2 / mk4 (optional, uint8 [P/4][C] / [P/16][C]) receive the
 * index of the first maximum in each window (row-major, 255 if none), which the
 * x-branch data-gradient GEMM uses to route the max-pool gradient (AccGemmDesc.pd2).
 * Backward (standalone form) accumulates into da (max: first max in window).
 * ------------------------------------------------------------------------- */
int accunet_hanc_pyramid_fwd(const void* x, const float* sc, const float* sh, int act, int B,
                             int H, int W, int C, int k, void* p2, void* p4,
                             unsigned char* mk2, unsigned char* mk4, int dt, void* stream);
int accunet_hanc_pyramid_bwd(const void* x, const float* sc, const float* sh, int act, int B,
                             int H, int W, int C, int k, const void* p2, const void* p4,
                             const void* dp2, const void* dp4, void* da, int dt, void* stream);
/* HANCLayer / MLFC-merge channel interleave (ACC_UNet.py:138, :492):
 * out[n][jj][c] = W[n][c*J + order[jj]]  (inverse scatters back) */
int accunet_group_relayout(const float* in, float* out, int N, int C, int J, const int* order,
                           int inverse, void* stream);

/* ------------------------------------------------------------------------- *
 * Resampling / layout: MaxPool2d(2) (ACC_UNet.py:552), AvgPool2d(2) (MLFC :361),
 * nearest Upsample backward (block sums, :360), channel concat slices
 * (torch.cat dim=1, :639-648), ConvTranspose2d(2,2,s2) pixel shuffle (:578-590),
 * generic 4-D permute (weights, NCHW<->NHWC at the module boundary).
 * mode: 0 = max, 1 = avg.
 * ------------------------------------------------------------------------- */
int accunet_pool2_fwd(const void* x, void* y, int B, int H, int W, int C, int mode, int dt,
                      void* stream);
int accunet_pool2_bwd(const void* x, const void* y, const void* dy, void* dx, int B, int H,
                      int W, int C, int mode, int accumulate, int dt, void* stream);
int accunet_upsample_bwd(const void* in, int ld_in, int in_off, void* out, int ld_out, int B,
                         int H, int W, int C, int f, int accumulate, int dt, void* stream);
/* Both backward sums of a k = 3 HANCLayer's pyramid (ACC_UNet.py:96-106: the 2x and 4x
 * nearest upsamples of the pooled branches) in one pass over in: out2 = 2x2 block sums,
 * out4 = 4x4 block sums, each added in the order accunet_upsample_bwd adds them (the
 * same bits as its f = 2 and f = 4 launches). H, W multiples of 4. */
int accunet_upsample_bwd24(const void* in, int ld_in, void* out2, int ld_out2, void* out4,
                           int ld_out4, int B, int H, int W, int C, int dt, void* stream);
int accunet_slice_copy(const void* src, int ld_src, int src_off, void* dst, int ld_dst,
                       int dst_off, long P, int C, int accumulate, int dt, void* stream);
int accunet_pixel_shuffle2(const void* t, const float* bias, void* y, int B, int Hi, int Wi,
                           int Cout, int inverse, int dt, void* stream);
/* Decoder up-sampling and concat in one pass (ACC_UNet.py:637-648, torch.cat([up(x),
 * skip], dim=1)): t = the ConvT GEMM output [B][Hi][Wi][4*Co] is pixel-shuffled (+bias)
 * into channels [0, Co) of y [B][2Hi][2Wi][Co+Cs], skip [B][2Hi][2Wi][Cs] into
 * [Co, Co+Cs). inverse = 1: y is the incoming gradient; t receives dT and skip (if not
 * NULL) the skip's gradient. Co, Cs multiples of 4. */
int accunet_convt_cat(void* t, const float* bias, void* skip, void* y, int B, int Hi, int Wi,
                      int Co, int Cs, int inverse, int dt, void* stream);
/* in_dt / out_dt: storage of in / out (e.g. NCHW fp32 input -> NHWC bf16 activations) */
int accunet_permute4(const void* in, void* out, const int* dims, const long long* strides,
                     const int* flips, int accumulate, int in_dt, int out_dt, void* stream);

/* ------------------------------------------------------------------------- *
 * ChannelSELayer (ACC_UNet/ACC_UNet.py:9-49) fused with the BatchNorm(+LReLU)
 * that precedes it (sc/sh/act) and its own BN + LeakyReLU; the BN statistics of
 * a*s are derived from per-(b,c) sums, so the input is read twice and the output
 * written once. `save` (accunet_se_save_elems) holds the forward state for
 * accunet_se_bwd, which returns da (gradient w.r.t. the SE input a) and the fc /
 * BN parameter gradients. ostats (optional) = statistics of the output.
 * ------------------------------------------------------------------------- */
size_t accunet_se_save_elems(int B, int C, int Cr);
size_t accunet_se_ws_elems(int B, int HW, int C, int Cr);
int accunet_se_stats_rows(int B, int HW, int C);
int accunet_se_fwd(const void* z, const float* sc, const float* sh, int act, int B, int HW,
                   int C, int Cr, const float* w1, const float* b1, const float* w2,
                   const float* b2, const float* gamma, const float* beta, float* rmean,
                   float* rvar, long long* nbt, float momentum, float eps, int training,
                   void* out, const void* res, float* save, double* ostats, float* ws,
                   size_t ws_elems, int dt, void* stream);
/* res (optional, same shape and storage as z): out = SE(z) + res, the residual add
 * that follows the SE in ResPath (ACC_UNet/ACC_UNet.py:326) and in the MLFC merge
 * (:489-520), fused into the apply pass so the SE output itself is never written;
 * ostats then describe out. */
int accunet_se_bwd(const void* z, const void* dout, const float* sc, const float* sh, int act,
                   int B, int HW, int C, int Cr, const float* w1, const float* w2,
                   const float* gamma, int training, const float* save, void* da, float* dw1,
                   float* db1, float* dw2, float* db2, float* dgamma, float* dbeta, float* ws,
                   size_t ws_elems, int dt, void* stream);
/* accunet_se_bwd fused with the backward of the BatchNorm(+act) prologue that feeds
 * the SE (HANCBlock.norm3 :281-283, ResPath.bns :326, Conv2d_batchnorm.batchnorm
 * :183-185, MLFC.bns_mrg :520): pst = that BatchNorm's [4][C] (mean, rstd, scale,
 * shift) block, pgamma its weight, ptraining its mode. Returns dz (gradient w.r.t.
 * the pre-BN input z) and the prologue's dgamma/dbeta directly: 2 read passes over
 * (z, dout) and one write, da is never materialised. dsum (optional) = sum_p dz, the
 * bias gradient of z's producer convolution. */
int accunet_se_bwd_pro(const void* z, const void* dout, const float* pst, int act,
                       const float* pgamma, int ptraining, int B, int HW, int C, int Cr,
                       const float* w1, const float* w2, const float* gamma, int training,
                       const float* save, void* dz, float* dpgamma, float* dpbeta, float* dsum,
                       float* dw1,
                       float* db1, float* dw2, float* db2, float* dgamma, float* dbeta, float* ws,
                       size_t ws_elems, int dt, void* stream);

/* ------------------------------------------------------------------------- *
 * Head: out 1x1 conv n_filts -> 1 (+ Sigmoid when sigm) (ACC_UNet.py:594-599,653-659);
 * x / dx are activations (dt), y / dy (the model output, fed to the loss) fp32
 * ------------------------------------------------------------------------- */
int accunet_head_fwd(const void* x, const float* w, const float* b, int sigm, float* y, long P,
                     int C, int dt, void* stream);
size_t accunet_head_ws_elems(long P, int C);
int accunet_head_bwd(const void* x, const float* w, const float* y, const float* dy, int sigm,
                     void* dx, float* dw, float* db, long P, int C, float* ws, size_t ws_elems,
                     int dt, void* stream);

/* ------------------------------------------------------------------------- *
 * WeightedDiceBCE (Experiments/utils.py:140-171; WeightedBCE :21-74 with the
 * truth.max() > 1 binarisation, WeightedDiceLoss :109-138), weights [0.5, 0.5].
 * res (device, 8 + 2B floats): [loss, dice, bce, pos_w, neg_w, binarised, -, -, (I,U)/b]
 * ------------------------------------------------------------------------- */
size_t accunet_loss_ws_elems(int B);
int accunet_loss_fwd(const float* x, const float* t, int B, long N, float dice_w, float bce_w,
                     float* res, float* ws, size_t ws_elems, void* stream);
int accunet_loss_bwd(const float* x, const float* t, int B, long N, float dice_w, float bce_w,
                     const float* res, const float* gout, float* dx, void* stream);

/* ------------------------------------------------------------------------- *
 * Adam (torch.optim.Adam as used at Experiments/train_model.py:647) over every
 * parameter in one launch. table: device array of {float* p; const float* g;
 * float* m; float* v; long long n;}; chunk_t / chunk_s map each block to
 * (tensor, first element), accunet_adam_chunk_elems() elements per chunk.
 * ------------------------------------------------------------------------- */
int accunet_adam_chunk_elems(void);
int accunet_adam_step(const void* table, const int* chunk_t, const long long* chunk_s,
                      int nchunks, float lr, float b1, float b2, float eps, float wd, int step,
                      void* stream);

/* ------------------------------------------------------------------------- *
 * ACC_UNet_W learnable merge y = a*w + b*(1-w) (ACC_UNet/ACC_UNet_w.py:497-522)
 * ------------------------------------------------------------------------- */
int accunet_wmerge_fwd(const void* a, const void* b, const float* w, void* y, long P, int C,
                       double* stats, int dt, void* stream);
int accunet_wmerge_bwd(const void* g, const float* w, void* da, void* db, long n, int dt,
                       void* stream);
int accunet_dotdiff(const void* g, const void* a, const void* b, long n, float* out,
                    int accumulate, float* ws, int dt, void* stream);

/* ------------------------------------------------------------------------- *
 * HIP graph / event plumbing for the graph-mode data-parallel step
 * (accunet/train.py; the reference has no data parallelism,
 * Experiments/train_model.py:696-698). graph_marker(id) launches an empty marker
 * kernel; after capture, graph_events_after_markers(graph, events, n) adds an
 * event-record node behind each marker id < n of the (un-instantiated) hipGraph_t
 * and returns how many it added. Every launch of the graph re-records the events; a
 * side stream waiting on one (stream_wait_event) starts the RCCL all-reduce of the
 * gradient bucket that marker closed while the graph runs the rest of backward.
 * ------------------------------------------------------------------------- */
int accunet_graph_marker(int id, void* stream);
int accunet_graph_events_after_markers(void* graph, void* const* events, int n);
int accunet_event_create(void** ev);
int accunet_event_destroy(void* ev);
int accunet_stream_wait_event(void* stream, void* ev);
int accunet_event_synchronize(void* ev);

/* In-graph kernel timing (bench.py's roofline over the timed region; no reference
 * counterpart). event_create_timed makes an event that records timestamps.
 * graph_time_markers(graph, id_start, id_end, ev_start, ev_end, nodes[2]) replaces the
 * marker kernels id_start / id_end of the un-instantiated hipGraph_t by event-record
 * nodes with the markers' dependencies and dependents (no marker launch is left in
 * the graph) and returns the two node handles; exec_event_set(exec, node, ev) points
 * such a node of the instantiated graph at another event for the next launches
 * (one event pair per replay); event_elapsed_ms(a, b, &ms) reads the time between
 * two completed records. */
int accunet_event_create_timed(void** ev);
int accunet_graph_time_markers(void* graph, int id_start, int id_end, void* ev_start,
                               void* ev_end, void** nodes);
int accunet_graph_exec_event_set(void* exec, void* node, void* ev);
int accunet_event_elapsed_ms(void* start, void* end, float* ms);

/* ------------------------------------------------------------------------- *
 * Streaming ceiling for the roofline probes (accunet/probe.py): copies n_bytes
 * (a multiple of 16, 16-B aligned buffers) from src to dst with non-temporal float4
 * loads and stores, four per thread per 16-KB block -- the fastest copy form measured
 * on MI355X (tools/kbench "x4/thread nt"). Not on the model path.
 * ------------------------------------------------------------------------- */
int accunet_copy_nt(const void* src, void* dst, long long n_bytes, void* stream);

/* ------------------------------------------------------------------------- *
 * Input preparation (csrc/data.hip). Replaces the per-image host work of
 * ImageToImage2D.__getitem__, Experiments/Load_Dataset.py:453-487, for a whole
 * batch: image_prep takes N raw channel planes [N][Hin][Win] (fp32) and writes
 * [N][1][S][S] = z-score((INTER_LINEAR resize to S x S if needed)) with
 * torch's unbiased std and +1e-8 (:470-472); mask_prep takes N raw masks
 * (dtype 0 = uint8/bool, 1 = float32, 2 = int64) and writes fp32 {0,1}
 * (INTER_NEAREST resize, mask > 0, :478-481).
 * ------------------------------------------------------------------------- */
int accunet_image_prep(const float* raw, int N, int Hin, int Win, int S, float* out, void* stream);
int accunet_mask_prep(const void* raw, int dtype, int N, int Hin, int Win, int S, float* out,
                      void* stream);

/* ------------------------------------------------------------------------- *
 * Training augmentation (csrc/augment.hip): RandomGenerator's geometric
 * transforms, Experiments/Load_Dataset.py:19-32 (random_rot_flip: np.rot90 k
 * times + np.flip(axis); random_rotate: scipy.ndimage.rotate(order=0,
 * reshape=False)), one parameter block per sample, applied to a batch
 * [B][S][S][C] of uint8 or fp32 elements (out != in). The host draws the
 * parameters in the reference's random-call order and computes r / o as scipy
 * does (accunet/augment.py).
 * ------------------------------------------------------------------------- */
enum { ACC_AUG_F32 = 0, ACC_AUG_U8 = 1 };
typedef struct AccAugParam {
  double r00, r01, r10, r11; /* mode 2: source = r @ (row, col) + o */
  double o0, o1;
  int mode;                  /* 0 copy, 1 rot90 + flip, 2 rotate */
  int k;                     /* mode 1: quarter turns (counter-clockwise) */
  int axis;                  /* mode 1: np.flip axis (0 rows, 1 columns) */
  int pad;
} AccAugParam;
int accunet_aug_geom(const void* in, void* out, int dtype, int B, int S, int C,
                     const AccAugParam* params, void* stream);

/* ------------------------------------------------------------------------- *
 * Large-kernel depthwise convolution, NCHW fp32 (csrc/dwconvk.hip). Replaces the
 * reference's native extension kernels/dwconv2d: dwconv2d_fp32 /
 * dwconv2dbias_fp32 (dwconv2d.cpp:14-28 -> depthwise_fwd/launch.cu:12-80), and
 * adds the data / weight / bias gradients whose bindings the reference leaves
 * commented out (dwconv2d.cpp:30-52; Dwconv/dwconv_layer.py:20-31 calls them).
 * replicate = 1: the reference kernel's clamped tile fill (kernel.cuh:104-115,
 * window bounded by pad_h in both directions); 0: zero padding (its 3x3 routes).
 * Output size oH = H - kh + 1 + 2 ph, oW = W - kw + 1 + 2 pw; kh, kw <= 31.
 * ------------------------------------------------------------------------- */
int accunet_dwconvk_out_hw(int H, int W, int kh, int kw, int ph, int pw, int* oH, int* oW);
int accunet_dwconvk_fwd(const float* x, const float* w, const float* bias, float* out, int N,
                        int C, int H, int W, int kh, int kw, int ph, int pw, int replicate,
                        void* stream);
size_t accunet_dwconvk_dgrad_ws(int N, int C, int H, int W, int kh, int kw, int ph, int pw,
                                int replicate);
int accunet_dwconvk_dgrad(const float* dy, const float* w, float* dx, int N, int C, int H, int W,
                          int kh, int kw, int ph, int pw, int replicate, float* ws, size_t ws_elems,
                          void* stream);
size_t accunet_dwconvk_wgrad_ws(int N, int C, int H, int W, int kh, int kw, int ph, int pw);
int accunet_dwconvk_wgrad(const float* x, const float* dy, float* dw, float* db, int N, int C,
                          int H, int W, int kh, int kw, int ph, int pw, int replicate, float* ws,
                          size_t ws_elems, void* stream);

/* ------------------------------------------------------------------------- *
 * UNeXt tokenized-MLP model (Experiments/nets/UNext.py), NHWC fp32 = token rows
 * [B*H*W][C] (csrc/unext.hip). Together with the GEMM (Linear fc1/fc2, 3x3 convs),
 * the depthwise 3x3 (DWConv :150-161), BatchNorm, max-pool and head entry points
 * above, these replace every ATen op of UNext.forward (:251-358):
 *   layernorm   nn.LayerNorm (:181,221,244-248); mr = [P][2] mean, rstd saved;
 *               backward writes dx and dgamma | dbeta (db must be dg + C);
 *               part = [accunet_layernorm_rows(P)][2][C] scratch
 *   gelu        nn.GELU() exact (:49)
 *   token_shift shiftmlp's pad / chunk / roll / narrow (:86-111), axis 0 = H, 1 = W,
 *               dir +1 forward, -1 its backward
 *   up2_relu_*  relu(F.interpolate(x2, bilinear)) (+ skip add) (:313-333); mask = relu
 *               mask bytes [B][2H][2W][C] for the backward
 *   relu        F.relu (:257-265): dy == NULL -> y = relu(x); else y = dy * (x > 0)
 *   subsample2  stride-2 pick of even pixels (OverlapPatchEmbed.proj stride 2, :219);
 *               H, W = full resolution; bwd = 1 scatters the strided gradient back
 * ------------------------------------------------------------------------- */
int accunet_layernorm_rows(long P);
int accunet_layernorm_fwd(const float* x, const float* g, const float* b, float* y, float* mr,
                          long P, int C, float eps, void* stream);
int accunet_layernorm_bwd(const float* x, const float* g, const float* mr, const float* dy,
                          float* dx, float* dg, float* db, float* part, long P, int C,
                          void* stream);
int accunet_gelu_fwd(const float* x, float* y, long n, void* stream);
int accunet_gelu_bwd(const float* x, const float* dy, float* dx, long n, void* stream);
int accunet_token_shift(const float* x, float* y, int B, int H, int W, int C, int axis, int dir,
                        int shift_size, void* stream);
int accunet_up2_relu_add_fwd(const float* x, const float* skip, float* out, unsigned char* mask,
                             int B, int H, int W, int C, void* stream);
int accunet_up2_relu_bwd(const float* dout, const unsigned char* mask, float* dx, int B, int H,
                         int W, int C, void* stream);
int accunet_relu(const float* x, const float* dy, float* y, long n, void* stream);
int accunet_subsample2(const float* src, float* dst, int B, int H, int W, int C, int bwd,
                       void* stream);

#ifdef __cplusplus
}
#endif
#endif /* ACCUNET_H */
