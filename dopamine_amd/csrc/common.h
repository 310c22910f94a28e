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

// Warm the scalar cache with a kernel's argument block: one s_load per 64-byte line, all in
// flight together and waited for once.  The compiler loads argument fields lazily, each
// behind the branch that needs it (an op of a grouped launch, a compile-time-absent
// pointer), so without this a launch pays one dependent scalar miss round per branch
// level before its first global load.  kBytes: the explicit arguments' size (reading a
// line past them stays inside the argument block, whose hidden arguments follow).
template <int kBytes>
__device__ __forceinline__ void warm_kernargs() {
  typedef const uint32_t __attribute__((address_space(4)))* KPtr;
  const KPtr p = (KPtr)__builtin_amdgcn_kernarg_segment_ptr();
  constexpr int n = (kBytes + 63) / 64;
  static_assert(n <= 32, "argument block larger than the warm-up covers");
  uint32_t v[32];
#pragma unroll
  for (int i = 0; i < 32; ++i) v[i] = p[(i < n ? i : n - 1) * 16];   // all issued, then
#pragma unroll
  for (int i = 0; i < 32; i += 8)                                   // one wait for all
    if (i < n)
      asm volatile("" ::"s"(v[i]), "s"(v[i + 1]), "s"(v[i + 2]), "s"(v[i + 3]), "s"(v[i + 4]),
                   "s"(v[i + 5]), "s"(v[i + 6]), "s"(v[i + 7]));
}

// IEEE square root, correctly rounded, as TF1's CPU kernels (std::sqrt) and numpy compute
// it.  hipcc's __fsqrt_rn is __ocml_native_sqrt_f32 -- v_sqrt_f32 with denormal scaling,
// not correctly rounded -- unless OCML_BASIC_ROUNDED_OPERATIONS is defined; the builtin
// lowers to the exact expansion (v_sqrt_f32, then the +-1 ulp residual test).
__device__ __forceinline__ float sqrt_rn(float x) { return __builtin_sqrtf(x); }

// Python / numpy floor modulo for a positive modulus.  The replay's operands are almost
// always within one period of [0, m) (a sampled index, index + k for a short trajectory or
// frame stack): those take a compare and an add; only the rest run the 64-bit division,
// whose ~130-instruction software sequence sat in the gather's index -> frame-address
// chain four times per wave.
__device__ __forceinline__ int64_t pymod(int64_t a, int64_t m) {
  if (a >= -m && a < 2 * m) return a < 0 ? a + m : (a >= m ? a - m : a);
  const int64_t r = a % m;
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

__device__ __forceinline__ float wave_min(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fminf(v, __shfl_xor(v, o));
  return v;
}

// ---- TF1 ApplyAdam, shared by the optimizer kernels and the fused CNN epilogues.
// state = {beta1^t, beta2^t} x 2 slots: step t reads slot t % 2 and writes the
// next powers into the other slot (one thread per step does that).
__device__ __forceinline__ float adam_alpha_of(const float* state, int slot, float lr) {
  const float b1p = state[2 * slot], b2p = state[2 * slot + 1];
  // alpha = lr * sqrt(1 - beta2^t) / (1 - beta1^t)
  return __fdiv_rn(__fmul_rn(lr, sqrt_rn(__fsub_rn(1.0f, b2p))), __fsub_rn(1.0f, b1p));
}

__device__ __forceinline__ void adam_bump(float* state, int slot, float b1, float b2) {
  float* nxt = state + 2 * (slot ^ 1);
  nxt[0] = __fmul_rn(state[2 * slot], b1);
  nxt[1] = __fmul_rn(state[2 * slot + 1], b2);
}

__device__ __forceinline__ void adam1(float& var, float g, float& m, float& v, float alpha,
                                      float omb1, float omb2, float eps) {
  m = __fadd_rn(m, __fmul_rn(__fsub_rn(g, m), omb1));
  v = __fadd_rn(v, __fmul_rn(__fsub_rn(__fmul_rn(g, g), v), omb2));
  var = __fsub_rn(var, __fdiv_rn(__fmul_rn(m, alpha), __fadd_rn(sqrt_rn(v), eps)));
}

// ---- TF1 ApplyRMSProp / ApplyCenteredRMSProp (omr = 1 - rho), shared by k_rmsprop and
// the fused CNN optimizer ops: ms += (g^2 - ms)(1 - rho); centered: mg += (g - mg)(1 - rho),
// denom = ms - mg^2 + eps (else ms + eps); mom = mu mom + lr g / sqrt(denom); var -= mom.
__device__ __forceinline__ void rms1(float& var, float g, float& ms, float& mg, float& mom,
                                     float lr, float omr, float mu, float eps, bool centered) {
  ms = __fadd_rn(ms, __fmul_rn(__fsub_rn(__fmul_rn(g, g), ms), omr));
  float denom;
  if (centered) {
    mg = __fadd_rn(mg, __fmul_rn(__fsub_rn(g, mg), omr));
    denom = __fadd_rn(__fsub_rn(ms, __fmul_rn(mg, mg)), eps);
  } else {
    denom = __fadd_rn(ms, eps);
  }
  mom = __fadd_rn(__fmul_rn(mom, mu), __fdiv_rn(__fmul_rn(g, lr), sqrt_rn(denom)));
  var = __fsub_rn(var, mom);
}

}  // namespace dq
