// Probe: does hipEventRecordWithFlags(..., hipEventRecordExternal) work inside stream
// capture on this ROCm, and does a stream wait after hipGraphLaunch gate on it?
#include <hip/hip_runtime.h>
#include <stdio.h>
__global__ void spin(float* x, int n, int iters) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) { float v = x[i]; for (int k = 0; k < iters; ++k) v = v * 0.999999f + 1e-6f; x[i] = v; }
}
__global__ void add1(float* x) { x[0] += 1.f; }
__global__ void copy1(const float* x, float* y) { y[0] = x[0]; }
#define CK(e) do { hipError_t r = (e); if (r != hipSuccess) { printf("%s -> %d %s\n", #e, (int)r, hipGetErrorString(r)); } } while (0)
int main() {
  float *x, *y, *big;
  CK(hipMalloc(&x, 4)); CK(hipMalloc(&y, 4)); CK(hipMalloc(&big, 4 << 20));
  CK(hipMemset(x, 0, 4)); CK(hipMemset(big, 0, 4 << 20));
  hipStream_t s, side; CK(hipStreamCreate(&s)); CK(hipStreamCreate(&side));
  for (unsigned flags : {(unsigned)hipEventDisableTiming, 0u}) {
    for (int mode = 0; mode < 3; ++mode) {
      hipEvent_t ev; CK(hipEventCreateWithFlags(&ev, flags));
      hipGraph_t g; hipGraphExec_t ge;
      CK(hipStreamBeginCapture(s, (hipStreamCaptureMode)mode));
      hipLaunchKernelGGL(spin, dim3(4096), dim3(256), 0, s, big, 1 << 20, 20000);
      hipLaunchKernelGGL(add1, dim3(1), dim3(1), 0, s, x);
      hipError_t r = hipEventRecordWithFlags(ev, s, hipEventRecordExternal);
      printf("flags %u mode %d: record external -> %d %s\n", flags, mode, (int)r, hipGetErrorString(r));
      hipLaunchKernelGGL(spin, dim3(4096), dim3(256), 0, s, big, 1 << 20, 20000);
      CK(hipStreamEndCapture(s, &g));
      if (r != hipSuccess) { (void)hipGetLastError(); continue; }
      CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
      for (int it = 0; it < 3; ++it) {
        CK(hipGraphLaunch(ge, s));
        CK(hipStreamWaitEvent(side, ev, 0));
        hipLaunchKernelGGL(copy1, dim3(1), dim3(1), 0, side, x, y);
        CK(hipDeviceSynchronize());
        float hx, hy; CK(hipMemcpy(&hx, x, 4, hipMemcpyDeviceToHost)); CK(hipMemcpy(&hy, y, 4, hipMemcpyDeviceToHost));
        printf("  replay %d: x %.0f y(after wait) %.0f %s\n", it, hx, hy, hx == hy ? "gated OK" : "NOT gated");
      }
    }
  }
  return 0;
}
