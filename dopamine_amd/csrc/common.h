// Shared helpers for the dopamine_amd HIP kernels (gfx950 / CDNA4, wave64).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <string>

#include "../../include/dopamine_amd.h"

namespace dq {

void set_error(const std::string& msg);

#define DQ_CHECK_ARG(cond, msg)        \
  do {                                 \
    if (!(cond)) {                     \
      ::dq::set_error(msg);            \
      return DQ_E_ARG;                 \
    }                                  \
  } while (0)

#define DQ_CHECK_LAUNCH(what)                                                   \
  do {                                                                          \
    hipError_t e_ = hipGetLastError();                                          \
    if (e_ != hipSuccess) {                                                     \
      ::dq::set_error(std::string(what) + ": " + hipGetErrorString(e_));        \
      return DQ_E_HIP;                                                          \
    }                                                                           \
  } while (0)

#define DQ_CHECK_HIP(expr)                                                      \
  do {                                                                          \
    hipError_t e_ = (expr);                                                     \
    if (e_ != hipSuccess) {                                                     \
      ::dq::set_error(std::string(#expr) + ": " + hipGetErrorString(e_));       \
      return DQ_E_HIP;                                                          \
    }                                                                           \
  } while (0)

constexpr int kWave = 64;

// Python / numpy floor modulo for a positive modulus.
__device__ __forceinline__ int64_t pymod(int64_t a, int64_t m) {
  int64_t r = a % m;
  return r < 0 ? r + m : r;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  return v;
}

}  // namespace dq
