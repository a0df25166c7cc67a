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
