// C51 device pieces shared by learner.hip (the loss kernels) and nature_cnn.hip (the
// target half riding in the fused forward): logit sources, DPP wave reductions, and the
// target half of rainbow_agent.py:200-251 + 340-494 (target softmax / Q / greedy action /
// Eq.-7 projection) as a per-sample block body.
#pragma once
#include "common.h"

namespace dq {

// Logit sources: stored logits, or (the fused Rainbow path) fc2's 16 k-band
// partial products summed in band order plus the bias -- exactly the reduction
// order of the CNN's fc2 tile, so the logits are bitwise dq_cnn_forward's.
// load() issues an element's loads, sum() forms it from them (get = sum(load)): a kernel
// can put independent work between the two while the loads are in flight.
struct LogitsDirect {
  const float* p;
  int NO;
  struct Pend {
    float v;
  };
  __device__ __forceinline__ Pend load(int64_t i) const { return Pend{p[i]}; }
  __device__ __forceinline__ Pend load_bc(int b, int col) const {
    return Pend{p[(int64_t)b * NO + col]};
  }
  __device__ __forceinline__ float sum(const Pend& q) const { return q.v; }
  __device__ __forceinline__ float get(int64_t i) const { return p[i]; }
};
struct LogitsParts {
  const float* part;   // [np][B * NO]
  const float* bias;   // [NO]
  int64_t stride;      // B * NO
  int np, NO;          // np <= 16: straight-line loads, all in flight before the first add
  struct Pend {
    float v[16];
    float bias;
  };
  // element (b, col) of the (B, NO) logits: one buffer load per slab -- the slab's byte
  // offset in a scalar register, the element's in a 32-bit vector one (the slabs span
  // < 2 GB) -- so the loss kernel's prologue has no 64-bit address or index arithmetic
  __device__ __forceinline__ Pend load_bc(int b, int col) const {
    Pend q;
    const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(part), 0, 0x7fffffff,
                                                        0x00020000);
    const int off = (b * NO + col) * 4;
#pragma unroll
    for (int z = 0; z < 16; ++z)
      q.v[z] = __builtin_bit_cast(
          float, __builtin_amdgcn_raw_buffer_load_b32(rsrc, off, (int)(min(z, np - 1) * stride * 4), 0));
    q.bias = bias[col];
    return q;
  }
  __device__ __forceinline__ Pend load(int64_t i) const {
    return load_bc((int)(i / NO), (int)(i % NO));
  }
  __device__ __forceinline__ float sum(const Pend& q) const {   // get()'s order
    float x = q.v[0];
#pragma unroll
    for (int z = 1; z < 16; ++z)
      if (z < np) x = __fadd_rn(x, q.v[z]);
    return __fadd_rn(x, q.bias);
  }
  __device__ __forceinline__ float get(int64_t i) const {
    float v[16];
#pragma unroll
    for (int z = 0; z < 16; ++z) v[z] = part[(int64_t)min(z, np - 1) * stride + i];
    float x = v[0];
#pragma unroll
    for (int z = 1; z < 16; ++z)
      if (z < np) x = __fadd_rn(x, v[z]);
    return __fadd_rn(x, bias[i % NO]);
  }
};

// Wave-wide reductions on DPP row rotations (no LDS round trips, unlike __shfl_xor's
// ds_bpermute chain): each 16-lane row reduces by row_ror 8, 4, 2, 1, then lanes 0, 16,
// 32, 48 combine as (r0 op r1) op (r2 op r3) -- one value, the same in every lane.
template <int kCtrl>
__device__ __forceinline__ float dpp_ror(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), kCtrl, 0xf, 0xf, false));
}
__device__ __forceinline__ float rl(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
__device__ __forceinline__ float fast_sum(float v) {
  v = __fadd_rn(v, dpp_ror<0x128>(v));
  v = __fadd_rn(v, dpp_ror<0x124>(v));
  v = __fadd_rn(v, dpp_ror<0x122>(v));
  v = __fadd_rn(v, dpp_ror<0x121>(v));
  return __fadd_rn(__fadd_rn(rl(v, 0), rl(v, 16)), __fadd_rn(rl(v, 32), rl(v, 48)));
}
__device__ __forceinline__ float fast_max(float v) {
  v = fmaxf(v, dpp_ror<0x128>(v));
  v = fmaxf(v, dpp_ror<0x124>(v));
  v = fmaxf(v, dpp_ror<0x122>(v));
  v = fmaxf(v, dpp_ror<0x121>(v));
  return fmaxf(fmaxf(rl(v, 0), rl(v, 16)), fmaxf(rl(v, 32), rl(v, 48)));
}
__device__ __forceinline__ float fast_min(float v) {
  v = fminf(v, dpp_ror<0x128>(v));
  v = fminf(v, dpp_ror<0x124>(v));
  v = fminf(v, dpp_ror<0x122>(v));
  v = fminf(v, dpp_ror<0x121>(v));
  return fminf(fminf(rl(v, 0), rl(v, 16)), fminf(rl(v, 32), rl(v, 48)));
}

// The fused d h's dot product for column `col` of LDS-resident W2 rows (row stride `ld`):
// sum_i g_i W2[i][col] as four interleaved partial sums (i mod 4, each in i order) added
// pairwise -- a 13-deep dependent add chain instead of N = 51, the loss kernels' tail.
// k_c51 and k_c51_online share it, so their d h stay bitwise equal.
__device__ __forceinline__ float dh_dot(const float* s_g, const float* s_w, int ld, int col, int N) {
  float acc[4] = {0.0f, 0.0f, 0.0f, 0.0f};
  int i = 0;
  for (; i + 8 <= N; i += 8) {
    float t[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) t[u] = __fmul_rn(s_g[i + u], s_w[(i + u) * ld + col]);
#pragma unroll
    for (int u = 0; u < 8; ++u) acc[u & 3] = __fadd_rn(acc[u & 3], t[u]);
  }
  for (; i < N; ++i) acc[i & 3] = __fadd_rn(acc[i & 3], __fmul_rn(s_g[i], s_w[i * ld + col]));
  return __fadd_rn(__fadd_rn(acc[0], acc[1]), __fadd_rn(acc[2], acc[3]));
}

// The target half of the C51 loss for sample b, split off k_c51 so it can ride in the
// fused forward's last launch (TgtC51Op, nature_cnn.hip) while the loss kernel keeps only
// the online half (k_c51_online): the same operations in the same order as k_c51's, so
// the projected target distribution m is bitwise what k_c51 forms in registers.
//   rb:200-251  Tz = clip(r + gamma^n (1 - term) z), a* = first argmax_a Q_tgt(s', a)
//   rb:340-494  m_i = sum_j clip(1 - |Tz_j - z_i| / dz, 0, 1) p_tgt(s', a*)_j, j in order
// kT threads (nw = kT / 64 waves; wave w takes actions w, w + nw, .., at most 4 each).
struct C51Target {
  LogitsParts tl;          // the target net's fc2 partials
  const float* rew;
  const uint8_t* term;
  const float* support;
  int B, A, N;
  float cg;
  float* m;                // (B, N) out
  float* tl_out;           // (B, A * N) target logits out, may be NULL
};

constexpr int kC51TgtMaxWaveRows = 4;
constexpr int c51_target_lds(int A, int N) { return A * N + A + N * 64; }   // floats

template <int kT>
__device__ __forceinline__ void c51_target_block(const C51Target& t, int b, float* smem) {
  constexpr int nw = kT / 64;
  const int N = t.N, A = t.A;
  float* s_p = smem;                 // [A][N] target probabilities
  float* s_q = s_p + A * N;          // [A]    target Q
  float* s_c = s_q + A;              // [N][64] projection terms c(i, j)
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const bool on = lane < N;
  const float ninf = -__builtin_inff();
  const float z = on ? t.support[lane] : 0.0f;
  const float rew_b = t.rew[b], term_b = (float)t.term[b];
  const float vmin = t.support[0], vmax = t.support[N - 1], z1 = t.support[1];
  const int lc = min(lane, N - 1);
  float xv[kC51TgtMaxWaveRows];
#pragma unroll
  for (int r = 0; r < kC51TgtMaxWaveRows; ++r) {
    const int act = wave + r * nw;
    const float x = t.tl.get(((int64_t)b * A + min(act, A - 1)) * N + lc);   // clamped: branch-free
    xv[r] = (act < A && on) ? x : ninf;
  }
  {
    const float dz = __fsub_rn(z1, vmin);
    const float gt = __fmul_rn(t.cg, __fsub_rn(1.0f, term_b));
    for (int j = __builtin_amdgcn_readfirstlane(wave); j < N; j += nw) {
      const float zj = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(z), j));
      const float tzj = fminf(fmaxf(__fadd_rn(rew_b, __fmul_rn(gt, zj)), vmin), vmax);
      if (on) {
        float c = __fsub_rn(1.0f, __fdiv_rn(fabsf(__fsub_rn(tzj, z)), dz));
        s_c[j * 64 + lane] = fminf(fmaxf(c, 0.0f), 1.0f);
      }
    }
  }
#pragma unroll
  for (int r = 0; r < kC51TgtMaxWaveRows; ++r) {
    const int act = wave + r * nw;
    if (act >= A) break;
    const float v = xv[r];
    if (t.tl_out && on) t.tl_out[((int64_t)b * A + act) * N + lane] = v;
    const float mx = fast_max(v);
    const float e = on ? expf(__fsub_rn(v, mx)) : 0.0f;
    const float p = __fdiv_rn(e, fast_sum(e));
    const float q = fast_sum(on ? __fmul_rn(z, p) : 0.0f);
    if (on) s_p[act * N + lane] = p;
    if (lane == 0) s_q[act] = q;
  }
  __syncthreads();
  if (wave != 0) return;
  int astar = 0;                     // greedy target action, first max
  const float qv = lane < A ? s_q[lane] : 0.0f;
  float best = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(qv), 0));
  for (int act = 1; act < A; ++act) {
    const float qa = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(qv), act));
    if (qa > best) {
      best = qa;
      astar = act;
    }
  }
  const float* pst = s_p + astar * N;
  if (on) {
    float proj = 0.0f;               // sum_j c(i, j) p_j in j order
    int j = 0;
    for (; j + 8 <= N; j += 8) {
      float tt[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) tt[u] = __fmul_rn(s_c[(j + u) * 64 + lane], pst[j + u]);
#pragma unroll
      for (int u = 0; u < 8; ++u) proj = __fadd_rn(proj, tt[u]);
    }
    for (; j < N; ++j) proj = __fadd_rn(proj, __fmul_rn(s_c[j * 64 + lane], pst[j]));
    t.m[(int64_t)b * N + lane] = proj;
  }
}

}  // namespace dq
