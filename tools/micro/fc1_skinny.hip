// fc1's forward at B = 32 (the step's launch F4: h_part[z] = a3[:, slab z] . W1[:, slab z]^T
// for the online and the target net, 2 x 15.9 MB of weights) as tile variants of the
// package's igemm_block, timed back to back in a HIP graph: weights MALL-hot (one set) or
// streamed from HBM (16 rotating sets, 507 MB).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I dopamine_amd/csrc \
//     tools/micro/fc1_skinny.hip -o tools/micro/fc1_skinny.bin
#include <cstdio>
#include <vector>

#include "cnn_tile.h"

namespace dq {
void set_error(const std::string&) {}
}  // namespace dq

using namespace dq::cnn;

constexpr int B = 32, K = 7744, N = 1024;   // both nets' 512 outputs stacked

template <int WM, int WN, int WK, bool kLate>
__global__ __launch_bounds__(64 * WM * WN * WK) void k_var(RowK a, RowK w, EpiPartial e, int kchunk) {
  constexpr int kTile = Tile<WM, WN, WK>::template lds<RowK, RowK>();
  __shared__ __attribute__((aligned(16))) float smem[kTile];
  igemm_block<WM, WN, WK, RowK, RowK, EpiPartial, kLate>(a, w, e, B, N, K, kchunk, blockIdx.x,
                                                         blockIdx.y, blockIdx.z, smem);
}

template <int WM, int WN, int WK, bool kLate>
void run(const char* name, int kchunk, const float* a, const std::vector<float*>& ws, float* part) {
  const int gx = (B + 32 * WM - 1) / (32 * WM), gy = N / (32 * WN), gz = (K + kchunk - 1) / kchunk;
  hipStream_t st;
  hipStreamCreate(&st);
  for (int sets : {1, (int)ws.size()}) {
    hipGraph_t g;
    hipGraphExec_t ge;
    const int iters = 160;
    hipStreamBeginCapture(st, hipStreamCaptureModeGlobal);
    for (int i = 0; i < iters; ++i)
      hipLaunchKernelGGL((k_var<WM, WN, WK, kLate>), dim3(gx, gy, gz), dim3(64 * WM * WN * WK), 0, st,
                         RowK{a, K}, RowK{ws[i % sets], K}, EpiPartial{part, B, N}, kchunk);
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
    const double us = best * 1e3 / iters;
    printf("%-22s %4d blocks x %4d thr, slabs %2d, %s: %6.2f us  (weights %.2f TB/s)\n", name,
           gx * gy * gz, 64 * WM * WN * WK, gz, sets == 1 ? "hot " : "HBM ", us,
           (double)N * K * 4 / (us * 1e-6) / 1e12);
    hipGraphExecDestroy(ge);
    hipGraphDestroy(g);
  }
  hipStreamDestroy(st);
}

int main() {
  float *a, *part;
  hipMalloc(&a, (size_t)B * K * 4);
  hipMalloc(&part, (size_t)64 * B * N * 4);
  std::vector<float*> ws(16);
  for (auto& w : ws) {
    hipMalloc(&w, (size_t)N * K * 4);
    hipMemset(w, 0, (size_t)N * K * 4);
  }
  hipMemset(a, 0, (size_t)B * K * 4);
  run<1, 1, 16, true>("1x1x16 late (now)", 512, a, ws, part);
  run<1, 1, 16, false>("1x1x16 early", 512, a, ws, part);
  run<1, 1, 8, true>("1x1x8 late", 256, a, ws, part);
  run<1, 1, 8, false>("1x1x8 early", 256, a, ws, part);
  run<1, 2, 8, true>("1x2x8 (shared)", 512, a, ws, part);
  run<1, 4, 4, true>("1x4x4 (shared)", 512, a, ws, part);
  run<1, 4, 4, true>("1x4x4 (shared) k256", 256, a, ws, part);
  run<1, 2, 8, true>("1x2x8 (shared) k256", 256, a, ws, part);
  return 0;
}
