// HIP-graph capture of origin -> A -> B -> A -> origin (stream A forks stream B and joins it
// back before A joins the origin), plain HIP: the pattern of the ZeRO-1 update on a second
// stream (dqn_agent._fc_branch, zero_update_stream) without torch, RCCL or this package.
//   hipcc --offload-arch=gfx950 -O2 tools/micro/capture_fork.hip -o tools/micro/capture_fork.bin
//   ./tools/micro/capture_fork.bin <steps>
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e = (x);                                                          \
    if (e != hipSuccess) {                                                       \
      printf("%s -> %s\n", #x, hipGetErrorString(e));                            \
      return 1;                                                                  \
    }                                                                            \
  } while (0)

__global__ void k_add(float* x, float v, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) x[i] += v;
}
__global__ void k_mul(float* x, float v, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) x[i] *= v;
}
__global__ void k_acc(float* y, const float* x, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) y[i] += x[i];
}

int main(int argc, char** argv) {
  const int steps = argc > 1 ? atoi(argv[1]) : 1;
  const int n = 1 << 20;
  float *x, *y;
  CK(hipMalloc(&x, n * 4));
  CK(hipMalloc(&y, n * 4));
  CK(hipMemset(x, 0, n * 4));
  CK(hipMemset(y, 0, n * 4));
  hipStream_t s0, a, b;
  CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
  const dim3 g(n / 256), t(256);
  CK(hipStreamBeginCapture(s0, hipStreamCaptureModeThreadLocal));
  hipEvent_t pending = nullptr;
  for (int s = 0; s < steps; ++s) {
    if (pending) CK(hipStreamWaitEvent(s0, pending, 0));
    hipLaunchKernelGGL(k_add, g, t, 0, s0, x, 1.0f, n);
    hipEvent_t ev, e1, e2;
    CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&e1, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&e2, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&pending, hipEventDisableTiming));
    CK(hipEventRecord(ev, s0));
    CK(hipStreamWaitEvent(a, ev, 0));
    hipLaunchKernelGGL(k_mul, g, t, 0, a, x, 2.0f, n);
    CK(hipEventRecord(e1, a));
    CK(hipStreamWaitEvent(b, e1, 0));
    hipLaunchKernelGGL(k_acc, g, t, 0, b, y, x, n);
    CK(hipEventRecord(e2, b));
    CK(hipStreamWaitEvent(a, e2, 0));
    hipLaunchKernelGGL(k_acc, g, t, 0, a, x, y, n);
    CK(hipEventRecord(pending, a));
  }
  CK(hipStreamWaitEvent(s0, pending, 0));
  hipGraph_t graph;
  CK(hipStreamEndCapture(s0, &graph));
  printf("captured %d steps\n", steps);
  fflush(stdout);
  hipGraphExec_t ge;
  CK(hipGraphInstantiate(&ge, graph, nullptr, nullptr, 0));
  CK(hipGraphLaunch(ge, s0));
  CK(hipStreamSynchronize(s0));
  float hx, hy;
  CK(hipMemcpy(&hx, x, 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(&hy, y, 4, hipMemcpyDeviceToHost));
  double xr = 0, yr = 0;
  for (int s = 0; s < steps; ++s) {
    xr = (xr + 1) * 2;
    yr += xr;
    xr += yr;
  }
  printf("%s: x %g (want %g), y %g (want %g)\n", (hx == xr && hy == yr) ? "ok" : "MISMATCH", hx, xr,
         hy, yr);
  return 0;
}
