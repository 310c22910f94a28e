// Per-launch floor on MI355X: empty kernels of the grouped GEMM launches' shapes
// (blocks x threads, static LDS), back to back in a HIP graph.
//   hipcc --offload-arch=gfx950 -O3 tools/micro/launch_floor.hip -o tools/micro/launch_floor.bin
#include <hip/hip_runtime.h>
#include <cstdio>

template <int T, int LDS>
__global__ __launch_bounds__(T) void k_empty(float* out, int flag) {
  __shared__ float s[LDS / 4 > 0 ? LDS / 4 : 1];
  if (flag == 12345) {            // never true: keeps the LDS allocation
    s[threadIdx.x % (LDS / 4 > 0 ? LDS / 4 : 1)] = 1.0f;
    __syncthreads();
    out[blockIdx.x] = s[0];
  }
}

// one barrier + LDS round trip + one store per thread
template <int T, int LDS>
__global__ __launch_bounds__(T) void k_touch(float* out, int flag) {
  __shared__ float s[LDS / 4 > 0 ? LDS / 4 : 1];
  s[threadIdx.x] = (float)threadIdx.x;
  __syncthreads();
  out[(size_t)blockIdx.x * T + threadIdx.x] = s[(threadIdx.x + 1) % T] + flag;
}

template <int T, int LDS, bool TOUCH>
void run(const char* name, int blocks, float* out) {
  hipStream_t st;
  hipStreamCreate(&st);
  hipGraph_t g;
  hipGraphExec_t ge;
  const int iters = 200;
  hipStreamBeginCapture(st, hipStreamCaptureModeGlobal);
  for (int i = 0; i < iters; ++i) {
    if (TOUCH)
      hipLaunchKernelGGL((k_touch<T, LDS>), dim3(blocks), dim3(T), 0, st, out, 0);
    else
      hipLaunchKernelGGL((k_empty<T, LDS>), dim3(blocks), dim3(T), 0, st, out, 0);
  }
  hipStreamEndCapture(st, &g);
  hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
  hipGraphLaunch(ge, st);
  hipStreamSynchronize(st);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  float best = 1e9;
  for (int r = 0; r < 5; ++r) {
    hipEventRecord(e0, st);
    hipGraphLaunch(ge, st);
    hipEventRecord(e1, st);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    best = ms < best ? ms : best;
  }
  printf("%-8s blocks %5d x %4d thr, LDS %6d B: %6.2f us/launch\n", name, blocks, T, LDS,
         best * 1e3 / iters);
}

// a graph of n empty kernels replayed back to back: the per-replay cost beyond n launches
void graph_gap(int n, int reps) {
  hipStream_t st;
  hipStreamCreate(&st);
  float* out;
  hipMalloc(&out, 4096);
  hipGraph_t g;
  hipGraphExec_t ge;
  hipStreamBeginCapture(st, hipStreamCaptureModeGlobal);
  for (int i = 0; i < n; ++i) hipLaunchKernelGGL((k_empty<1024, 0>), dim3(256), dim3(1024), 0, st, out, 0);
  hipStreamEndCapture(st, &g);
  hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
  for (int i = 0; i < 10; ++i) hipGraphLaunch(ge, st);
  hipStreamSynchronize(st);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0, st);
  for (int i = 0; i < reps; ++i) hipGraphLaunch(ge, st);
  hipEventRecord(e1, st);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  printf("graph of %3d empty kernels: %7.2f us per replay (%5.2f us per kernel)\n", n,
         ms * 1e3 / reps, ms * 1e3 / reps / n);
}

int main() {
  graph_gap(1, 500);
  graph_gap(14, 500);
  graph_gap(28, 500);
  graph_gap(200, 50);
  float* out;
  hipMalloc(&out, 64 << 20);
  run<64, 0, false>("empty", 1, out);
  run<1024, 0, false>("empty", 1, out);
  run<1024, 0, false>("empty", 32, out);
  run<1024, 0, false>("empty", 256, out);
  run<1024, 0, false>("empty", 512, out);
  run<1024, 0, false>("empty", 1024, out);
  run<1024, 65536, false>("empty", 256, out);
  run<1024, 65536, false>("empty", 512, out);
  run<1024, 131072, false>("empty", 512, out);
  run<512, 32768, false>("empty", 242, out);
  run<256, 0, false>("empty", 1650, out);
  run<1024, 4096, true>("touch", 256, out);
  run<1024, 4096, true>("touch", 512, out);
  run<1024, 65536, true>("touch", 512, out);
  return 0;
}
