// Input preparation of a training batch on the device: the per-sample work of the
// reference loader ImageToImage2D.__getitem__ (Experiments/Load_Dataset.py:453-487)
// done for a whole batch in two launches after one host->device copy of the raw
// planes, instead of per image on the host.
//
//   image: channel plane of the raw .npy (already selected by the host), resized to
//          S x S if needed with cv2.resize's default INTER_LINEAR rule
//          (Load_Dataset.py:465-466: half-pixel centres, source coordinate clamped
//          at 0, right/bottom neighbour clamped to the last pixel), then per-image
//          z-score (img - mean) / (std + 1e-8) with the unbiased std of
//          torch.Tensor.std (:470-472). mean and the centred sum of squares are
//          accumulated in fp64 (fixed-order block tree), then rounded to fp32 as
//          torch's float32 results are, and the normalisation runs in fp32.
//   mask:  resized with INTER_NEAREST if needed (:478-479: source index
//          floor(dst * in / out)), binarised (mask > 0) (:481) and written as fp32
//          {0, 1}, the dtype the loss consumes (Train_one_epoch.py:117 casts the
//          int64 label to float).
//
// One 1024-thread block per image: a 256 x 256 plane is 256 KB, so the three passes
// (resize+sum, centred sum of squares, normalise) stay in L2 and the whole batch is
// a few microseconds; the batch is tiny next to one training step.
#include "common.h"

#define PREP_THREADS 1024

ACC_DEV float bilinear_cv(const float* __restrict__ src, int Hin, int Win, int S, int y, int x) {
  // cv2 INTER_LINEAR (float): fx = (x + 0.5) * Win / S - 0.5, clamped at 0
  const float sy = (float)Hin / (float)S, sx = (float)Win / (float)S;
  float fy = ((float)y + 0.5f) * sy - 0.5f;
  float fx = ((float)x + 0.5f) * sx - 0.5f;
  int y0 = (int)floorf(fy), x0 = (int)floorf(fx);
  float ay = fy - (float)y0, ax = fx - (float)x0;
  if (y0 < 0) { y0 = 0; ay = 0.f; }
  if (x0 < 0) { x0 = 0; ax = 0.f; }
  if (y0 >= Hin - 1) { y0 = Hin - 1; ay = 0.f; }
  if (x0 >= Win - 1) { x0 = Win - 1; ax = 0.f; }
  const int y1 = min(y0 + 1, Hin - 1), x1 = min(x0 + 1, Win - 1);
  const float v00 = src[(long)y0 * Win + x0], v01 = src[(long)y0 * Win + x1];
  const float v10 = src[(long)y1 * Win + x0], v11 = src[(long)y1 * Win + x1];
  return (v00 * (1.f - ax) + v01 * ax) * (1.f - ay) + (v10 * (1.f - ax) + v11 * ax) * ay;
}

ACC_DEV double block_sum_d(double v, double* red) {
  const int tid = threadIdx.x;
  red[tid] = v;
  __syncthreads();
  for (int s = PREP_THREADS / 2; s > 0; s >>= 1) {
    if (tid < s) red[tid] += red[tid + s];
    __syncthreads();
  }
  const double r = red[0];
  __syncthreads();
  return r;
}

__global__ void __launch_bounds__(PREP_THREADS)
image_prep_kernel(const float* __restrict__ raw, int Hin, int Win, int S, float* __restrict__ out) {
  __shared__ double red[PREP_THREADS];
  const int b = blockIdx.x, tid = threadIdx.x;
  const float* src = raw + (long)b * Hin * Win;
  float* dst = out + (long)b * S * S;
  const long n = (long)S * S;
  const bool resize = (Hin != S || Win != S);
  double s1 = 0.0;
  for (long i = tid; i < n; i += PREP_THREADS) {
    const float v = resize ? bilinear_cv(src, Hin, Win, S, (int)(i / S), (int)(i % S)) : src[i];
    dst[i] = v;
    s1 += v;
  }
  const double mean = block_sum_d(s1, red) / (double)n;
  const float meanf = (float)mean;
  double s2 = 0.0;
  for (long i = tid; i < n; i += PREP_THREADS) {
    const double d = (double)dst[i] - mean;
    s2 += d * d;
  }
  const double var = block_sum_d(s2, red) / (double)(n > 1 ? n - 1 : 1);
  const float den = (float)sqrt(var) + 1e-8f;
  for (long i = tid; i < n; i += PREP_THREADS) dst[i] = (dst[i] - meanf) / den;
}

// mask dtype: 0 = uint8 / bool, 1 = float32, 2 = int64
__global__ void __launch_bounds__(256)
mask_prep_kernel(const void* __restrict__ raw, int dtype, int Hin, int Win, int S,
                 float* __restrict__ out, long total) {
  const long i = blockIdx.x * 256L + threadIdx.x;
  if (i >= total) return;
  const long n = (long)S * S;
  const long b = i / n;
  const int y = (int)((i % n) / S), x = (int)(i % S);
  // cv2 INTER_NEAREST: floor(dst * in / out), clamped
  const int sy = min((int)floorf((float)y * ((float)Hin / (float)S)), Hin - 1);
  const int sx = min((int)floorf((float)x * ((float)Win / (float)S)), Win - 1);
  const long j = b * Hin * Win + (long)sy * Win + sx;
  bool pos;
  if (dtype == 0) pos = static_cast<const unsigned char*>(raw)[j] > 0;
  else if (dtype == 1) pos = static_cast<const float*>(raw)[j] > 0.f;
  else pos = static_cast<const long long*>(raw)[j] > 0;
  out[i] = pos ? 1.f : 0.f;
}

extern "C" int accunet_image_prep(const float* raw, int N, int Hin, int Win, int S, float* out,
                                  void* stream) {
  if (N <= 0 || Hin <= 0 || Win <= 0 || S <= 0) return ACC_EBADSHAPE;
  hipLaunchKernelGGL(image_prep_kernel, dim3(N), dim3(PREP_THREADS), 0, (hipStream_t)stream, raw,
                     Hin, Win, S, out);
  return hipGetLastError() == hipSuccess ? ACC_OK : ACC_ELAUNCH;
}

extern "C" int accunet_mask_prep(const void* raw, int dtype, int N, int Hin, int Win, int S,
                                 float* out, void* stream) {
  if (N <= 0 || Hin <= 0 || Win <= 0 || S <= 0) return ACC_EBADSHAPE;
  if (dtype < 0 || dtype > 2) return ACC_EBADARG;
  const long total = (long)N * S * S;
  hipLaunchKernelGGL(mask_prep_kernel, dim3((unsigned)ceil_div(total, 256)), dim3(256), 0,
                     (hipStream_t)stream, raw, dtype, Hin, Win, S, out, total);
  return hipGetLastError() == hipSuccess ? ACC_OK : ACC_ELAUNCH;
}
