// Training augmentation of Experiments/Load_Dataset.py:19-117 (RandomGenerator's
// random_rot_flip / random_rotate) on device-resident batches: one launch applies
// each sample's own geometric transform to its image and its label.
//
//   mode 1 (random_rot_flip, :19-26): out = flip(rot90(x, k), axis) -- np.rot90
//          (counter-clockwise in the (row, col) plane) then np.flip; square planes
//   mode 2 (random_rotate, :28-32): scipy.ndimage.rotate(x, angle, order=0,
//          reshape=False), constant 0 outside. For output (r, c) the source point is
//          (R00 r + R01 c + o0, R10 r + R11 c + o1) in fp64 with the rotation matrix
//          and offset computed on the host exactly as scipy does; the sample is
//          taken iff both coordinates lie in [0, n-1], at floor(coord + 0.5).
//          The products and sums are evaluated unfused, in scipy's order
//          (tests/test_augment.py pins this bit-for-bit against scipy).
//   mode 0: copy.
// Layout: [B][S][S][C] (C = 1: NCHW == NHWC), uint8 or fp32 elements.
#include "common.h"
#include "../../include/accunet.h"

template <typename T>
__global__ void __launch_bounds__(256)
aug_geom_kernel(const T* __restrict__ in, T* __restrict__ out, int S, int C,
                const AccAugParam* __restrict__ prm) {
  const int b = blockIdx.y;
  const long plane = (long)S * S;
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= plane) return;
  const AccAugParam q = prm[b];
  const int r = (int)(i / S), c = (int)(i - (long)r * S);
  int sr = r, sc = c;
  bool ok = true;
  if (q.mode == 1) {
    // undo the flip, then the k counter-clockwise quarter turns:
    // rot90 once maps out[i][j] = in[j][S-1-i]
    int rr = q.axis == 0 ? S - 1 - r : r, cc = q.axis == 0 ? c : S - 1 - c;
    for (int t = 0; t < (q.k & 3); ++t) {
      const int nr = cc, nc = S - 1 - rr;
      rr = nr;
      cc = nc;
    }
    sr = rr;
    sc = cc;
  } else if (q.mode == 2) {
    const double fr = (double)r, fc = (double)c;
    const double y = __dadd_rn(__dadd_rn(__dmul_rn(q.r00, fr), __dmul_rn(q.r01, fc)), q.o0);
    const double x = __dadd_rn(__dadd_rn(__dmul_rn(q.r10, fr), __dmul_rn(q.r11, fc)), q.o1);
    const double hi = (double)(S - 1);
    ok = y >= 0.0 && y <= hi && x >= 0.0 && x <= hi;
    sr = ok ? (int)floor(y + 0.5) : 0;
    sc = ok ? (int)floor(x + 0.5) : 0;
  }
  const T* src = in + (long)b * plane * C + ((long)sr * S + sc) * C;
  T* dst = out + (long)b * plane * C + i * C;
  for (int ch = 0; ch < C; ++ch) dst[ch] = ok ? src[ch] : (T)0;
}

extern "C" int accunet_aug_geom(const void* in, void* out, int dtype, int B, int S, int C,
                                const AccAugParam* params, void* stream) {
  if (B <= 0 || S <= 0 || C <= 0) return ACC_EBADSHAPE;
  if (!in || !out || !params || in == out) return ACC_EBADARG;
  const long plane = (long)S * S;
  dim3 grid((unsigned)((plane + 255) / 256), (unsigned)B);
  hipStream_t s = (hipStream_t)stream;
  if (dtype == ACC_AUG_U8)
    hipLaunchKernelGGL(aug_geom_kernel<unsigned char>, grid, dim3(256), 0, s,
                       (const unsigned char*)in, (unsigned char*)out, S, C, params);
  else if (dtype == ACC_AUG_F32)
    hipLaunchKernelGGL(aug_geom_kernel<float>, grid, dim3(256), 0, s, (const float*)in,
                       (float*)out, S, C, params);
  else
    return ACC_EBADARG;
  return hipGetLastError() == hipSuccess ? ACC_OK : ACC_ELAUNCH;
}
