// Cross-file host helpers of the ACC-UNet HIP library.
#pragma once
#include "common.h"

// number of row-blocks a channel-tiled streaming kernel over [P][C] launches
// (= rows of the partial-statistics block it produces)
int stream_rowblocks(long P, int C);

// reduce a partial-statistics block [R][Wd] to <= 64 rows (ws scratch);
// returns the pointer to the reduced rows and their count in *Rout
const float* reduce_partials(const float* part, int R, int Wd, float* ws, int* Rout,
                             hipStream_t s);
size_t accunet_partials_ws_elems(int R, int Wd);
// fp64 versions: reduce [R][Wd] double partials to <= 64 rows; then sum those rows of
// the first ncols columns (row stride `stride`) into out[ncols] (fp32)
const double* reduce_partials_d(const double* part, int R, int Wd, double* ws, int* Rout,
                                hipStream_t s);
void sum_rows_d_to_f(const double* rows_ptr, int rows, int stride, int ncols, float* out,
                     hipStream_t s);

__global__ void sum_rows_kernel(const float* __restrict__ part, int R, int stride, int ncols,
                                float* __restrict__ out);

__global__ void inc_i64_kernel(long long* p);

// One-launch reduction of a partial block [R][stride] (fp32 or fp64 rows, fp64
// accumulation) followed by a per-column finish (bn.hip: reduce_finish_kernel).
enum { FIN_SUM_F = 0, FIN_SUM_D, FIN_DW, FIN_HEAD, FIN_BN_FWD, FIN_BN_BWD };
struct FinishArgs {
  int kind;
  int ncols;         // columns reduced (paired BN kinds: channels C; columns C..2C-1 are the second moments)
  int C;             // FIN_DW / FIN_HEAD: channels
  double count;      // BN kinds: pixels per channel
  const float* gamma;
  const float* beta;
  float* rmean;
  float* rvar;
  long long* nbt;
  float momentum, eps;
  const float* st;   // FIN_BN_BWD: the forward BatchNorm state block
  int training, xc_form;
  float* out_f;      // FIN_SUM_F totals / FIN_BN_FWD state block / FIN_BN_BWD coef / FIN_DW+HEAD dw
  double* out_d;     // FIN_SUM_D totals
  float* out2;       // FIN_DW / FIN_HEAD: db ; FIN_BN_BWD: dgamma
  float* out3;       // FIN_BN_BWD: dbeta
  float* out4;       // FIN_BN_BWD: sum_p dx (the producer convolution's bias gradient), or null
  int bank;          // ticket bank (set by reduce_finish from the launch stream)
};
// chunks: fp64 scratch of reduce_finish_ws(R, stride) doubles, 8-byte aligned
size_t reduce_finish_ws(int R, int stride);
// ticket bank (0 / 1) of launches enqueued on stream s (accunet_stream_ticket_bank)
int acc_stream_bank(hipStream_t s);
int reduce_finish(const void* part, bool part_f64, int R, int stride, double* chunks,
                  const FinishArgs& fa, hipStream_t s);
