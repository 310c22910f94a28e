// Calibrates rocprofv3's FETCH_SIZE / WRITE_SIZE on gfx950 for the access widths the Nature-CNN
// launches use (MI355X_MICROARCH.md: only 16-B streaming reads and writes
// are calibrated).  Each kernel moves a known byte count; run it once per counter:
//   hipcc --offload-arch=gfx950 -O3 tools/micro/pmc_calib.hip -o /tmp/pmc_calib
//   rocprofv3 --pmc FETCH_SIZE -d F -o run --output-format csv -- /tmp/pmc_calib
//   rocprofv3 --pmc WRITE_SIZE -d W -o run --output-format csv -- /tmp/pmc_calib
//   python tools/pmc_calib.py F W
// The stream kernels cover 512 MiB (twice the Infinity Cache), so re-reads cannot hide in it.
// k_bcast16: every workgroup reads the same 1 MiB: how many of the 8 XCDs' L2s fetch it.
// k_write4_half: lanes store 4 B to every other dword (each 64-B line half written).
// k_read4_stride2: 4-B loads of every other dword (each line half used).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int kT = 256;

__global__ __launch_bounds__(kT) void k_read4(const float* __restrict__ x, int64_t n, float* out) {
  float s = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * kT + threadIdx.x; i < n; i += (int64_t)gridDim.x * kT)
    s += x[i];
  if (s == 1234.5f) out[blockIdx.x] = s;       // never true for the zero input: no store traffic
}

__global__ __launch_bounds__(kT) void k_read16(const float4* __restrict__ x, int64_t n4, float* out) {
  float s = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * kT + threadIdx.x; i < n4; i += (int64_t)gridDim.x * kT) {
    const float4 v = x[i];
    s += v.x + v.y + v.z + v.w;
  }
  if (s == 1234.5f) out[blockIdx.x] = s;
}

__global__ __launch_bounds__(kT) void k_read4_stride2(const float* __restrict__ x, int64_t n, float* out) {
  float s = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * kT + threadIdx.x; 2 * i < n; i += (int64_t)gridDim.x * kT)
    s += x[2 * i];
  if (s == 1234.5f) out[blockIdx.x] = s;
}

__global__ __launch_bounds__(kT) void k_write4(float* __restrict__ y, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * kT + threadIdx.x; i < n; i += (int64_t)gridDim.x * kT)
    y[i] = (float)(i & 7);
}

__global__ __launch_bounds__(kT) void k_write16(float4* __restrict__ y, int64_t n4) {
  for (int64_t i = (int64_t)blockIdx.x * kT + threadIdx.x; i < n4; i += (int64_t)gridDim.x * kT)
    y[i] = make_float4(1.f, 2.f, 3.f, (float)(i & 7));
}

__global__ __launch_bounds__(kT) void k_write4_half(float* __restrict__ y, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * kT + threadIdx.x; 2 * i < n; i += (int64_t)gridDim.x * kT)
    y[2 * i] = (float)(i & 7);
}

__global__ __launch_bounds__(kT) void k_bcast16(const float4* __restrict__ x, int64_t n4, float* out) {
  float s = 0.f;
  for (int64_t i = threadIdx.x; i < n4; i += kT) {
    const float4 v = x[i];
    s += v.x + v.y + v.z + v.w;
  }
  if (s == 1234.5f) out[blockIdx.x] = s;
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  printf("%s failed: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

int main() {
  const int64_t n = (int64_t)512 << 20 >> 2;            // 512 MiB of floats
  const int64_t nb = (int64_t)1 << 20 >> 2;             // 1 MiB of floats
  float *x, *y, *out, *b;
  CK(hipMalloc(&x, n * 4));
  CK(hipMalloc(&y, n * 4));
  CK(hipMalloc(&b, nb * 4));
  CK(hipMalloc(&out, 65536 * 4));
  CK(hipMemset(x, 0, n * 4));
  CK(hipMemset(y, 0, n * 4));
  CK(hipMemset(b, 0, nb * 4));
  const int grid = 4096;
  for (int rep = 0; rep < 3; ++rep) {
    k_read4<<<grid, kT>>>(x, n, out);
    k_read16<<<grid, kT>>>((const float4*)x, n / 4, out);
    k_read4_stride2<<<grid, kT>>>(x, n, out);
    k_write4<<<grid, kT>>>(y, n);
    k_write16<<<grid, kT>>>((float4*)y, n / 4);
    k_write4_half<<<grid, kT>>>(y, n);
    k_bcast16<<<2048, kT>>>((const float4*)b, nb / 4, out);
    CK(hipDeviceSynchronize());
  }
  CK(hipGetLastError());
  printf("bytes: stream %lld, half-used stream %lld, broadcast buffer %lld (x 2048 workgroups)\n",
         (long long)(n * 4), (long long)(n * 2), (long long)(nb * 4));
  CK(hipFree(x));
  CK(hipFree(y));
  CK(hipFree(b));
  CK(hipFree(out));
  return 0;
}
