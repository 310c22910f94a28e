// Microbenchmark: TF1 Adam over a 1.7M-float flat parameter vector (Rainbow's
// Nature CNN) -- launch shapes and a same-traffic copy ceiling.
//   hipcc --offload-arch=gfx950 -O3 -I dopamine_amd/csrc tools/micro/adam_shapes.hip -o /tmp/adam_shapes
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include "common.h"
using namespace dq;

template <int U>
__global__ __launch_bounds__(256) void k_adam_u(float* __restrict__ var, const float* __restrict__ grad,
                                                float* __restrict__ m, float* __restrict__ v,
                                                const float* state, int64_t n4, float lr) {
  const float alpha = adam_alpha_of(state, 0, lr);
  const float omb1 = 0.1f, omb2 = 0.001f, eps = 1.5e-4f;
  const int64_t base = (int64_t)blockIdx.x * 256 * U + threadIdx.x;
  float4 p[U], g[U], mm[U], vv[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = base + 256 * u;
    if (i < n4) {
      p[u] = ((float4*)var)[i]; g[u] = ((const float4*)grad)[i];
      mm[u] = ((float4*)m)[i]; vv[u] = ((float4*)v)[i];
    }
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = base + 256 * u;
    if (i < n4) {
      adam1(p[u].x, g[u].x, mm[u].x, vv[u].x, alpha, omb1, omb2, eps);
      adam1(p[u].y, g[u].y, mm[u].y, vv[u].y, alpha, omb1, omb2, eps);
      adam1(p[u].z, g[u].z, mm[u].z, vv[u].z, alpha, omb1, omb2, eps);
      adam1(p[u].w, g[u].w, mm[u].w, vv[u].w, alpha, omb1, omb2, eps);
      ((float4*)var)[i] = p[u]; ((float4*)m)[i] = mm[u]; ((float4*)v)[i] = vv[u];
    }
  }
}

typedef float f4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void nt_store(float4 x, float4* p) {
  f4v v = {x.x, x.y, x.z, x.w};
  __builtin_nontemporal_store(v, (f4v*)p);
}

// nontemporal stores for the moments (streamed: next read one step later) and/or the weights
template <bool NT_MV, bool NT_VAR>
__global__ __launch_bounds__(256) void k_adam_nt(float* __restrict__ var, const float* __restrict__ grad,
                                                 float* __restrict__ m, float* __restrict__ v,
                                                 const float* state, int64_t n4, float lr) {
  const float alpha = adam_alpha_of(state, 0, lr);
  const float omb1 = 0.1f, omb2 = 0.001f, eps = 1.5e-4f;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n4) return;
  float4 p = ((float4*)var)[i], g = ((const float4*)grad)[i];
  float4 mm = ((float4*)m)[i], vv = ((float4*)v)[i];
  adam1(p.x, g.x, mm.x, vv.x, alpha, omb1, omb2, eps);
  adam1(p.y, g.y, mm.y, vv.y, alpha, omb1, omb2, eps);
  adam1(p.z, g.z, mm.z, vv.z, alpha, omb1, omb2, eps);
  adam1(p.w, g.w, mm.w, vv.w, alpha, omb1, omb2, eps);
  if (NT_VAR) {
    nt_store(p, (float4*)var + i);
  } else {
    ((float4*)var)[i] = p;
  }
  if (NT_MV) {
    nt_store(mm, (float4*)m + i);
    nt_store(vv, (float4*)v + i);
  } else {
    ((float4*)m)[i] = mm; ((float4*)v)[i] = vv;
  }
}

// same traffic, no math
__global__ __launch_bounds__(256) void k_copy7(float* __restrict__ var, const float* __restrict__ grad,
                                               float* __restrict__ m, float* __restrict__ v, int64_t n4) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n4) return;
  float4 p = ((float4*)var)[i], g = ((const float4*)grad)[i], a = ((float4*)m)[i], b = ((float4*)v)[i];
  p.x += g.x; a.y += g.y; b.z += g.z;
  ((float4*)var)[i] = p; ((float4*)m)[i] = a; ((float4*)v)[i] = b;
}

// math with fast reciprocal sqrt instead of IEEE div/sqrt -- NOT bit-exact, shows the math cost
__global__ __launch_bounds__(256) void k_adam_fast(float* __restrict__ var, const float* __restrict__ grad,
                                                   float* __restrict__ m, float* __restrict__ v,
                                                   const float* state, int64_t n4, float lr) {
  const float alpha = adam_alpha_of(state, 0, lr);
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n4) return;
  float4 p = ((float4*)var)[i], g = ((const float4*)grad)[i], a = ((float4*)m)[i], b = ((float4*)v)[i];
#define ONE(c) a.c += (g.c - a.c) * 0.1f; b.c += (g.c * g.c - b.c) * 0.001f; \
  p.c -= a.c * alpha / (sqrtf(b.c) + 1.5e-4f);
  ONE(x) ONE(y) ONE(z) ONE(w)
  ((float4*)var)[i] = p; ((float4*)m)[i] = a; ((float4*)v)[i] = b;
}

int main() {
  const int64_t n = 1689831 + 3;  // Rainbow Nature CNN (9 actions x 51 atoms), rounded to 4
  const int64_t n4 = n / 4;
  float *var, *grad, *m, *v, *state, *flush;
  hipMalloc(&var, n * 4); hipMalloc(&grad, n * 4); hipMalloc(&m, n * 4); hipMalloc(&v, n * 4);
  hipMalloc(&state, 64); hipMalloc(&flush, 512 << 20);
  std::vector<float> h(n);
  for (int64_t i = 0; i < n; ++i) h[i] = 1e-3f * (float)((i * 7919) % 1000 - 500);
  hipMemcpy(var, h.data(), n * 4, hipMemcpyHostToDevice);
  hipMemcpy(grad, h.data(), n * 4, hipMemcpyHostToDevice);
  hipMemset(m, 0, n * 4); hipMemset(v, 0, n * 4);
  float st[4] = {0.9f, 0.999f, 0.9f, 0.999f};
  hipMemcpy(state, st, 16, hipMemcpyHostToDevice);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  const double bytes = 7.0 * n * 4;
  auto run = [&](const char* name, auto launch, size_t flush_mb) {
    float tot = 0; int it = 100;
    for (int r = 0; r < 10; ++r) launch();
    for (int r = 0; r < it; ++r) {
      if (flush_mb) hipMemsetAsync(flush, r & 0xff, flush_mb << 20, 0);
      hipEventRecord(e0, 0); launch(); hipEventRecord(e1, 0);
      hipEventSynchronize(e1); float ms; hipEventElapsedTime(&ms, e0, e1); tot += ms;
    }
    const double us = 1e3 * tot / it;
    printf("%-28s flush %4zu MB %8.2f us  %7.1f GB/s\n", name, flush_mb, us, bytes / us * 1e-3);
  };
  const unsigned g1 = (unsigned)((n4 + 255) / 256);
  for (size_t mb : {0, 16, 32, 64, 128, 256, 512}) {
    run("adam U1", [&] { hipLaunchKernelGGL(k_adam_u<1>, dim3(g1), dim3(256), 0, 0, var, grad, m, v, state, n4, 1e-4f); }, mb);
    run("adam nt m,v", [&] { hipLaunchKernelGGL((k_adam_nt<true, false>), dim3(g1), dim3(256), 0, 0, var, grad, m, v, state, n4, 1e-4f); }, mb);
    run("adam nt m,v,var", [&] { hipLaunchKernelGGL((k_adam_nt<true, true>), dim3(g1), dim3(256), 0, 0, var, grad, m, v, state, n4, 1e-4f); }, mb);
  }
  return 0;
}
