// The implicit-quantile head of ImplicitQuantileNetwork (atari_lib.py:147-199) and its
// backward, on the matrix cores through the tile engine of cnn_tile.h (the big GEMMs on
// its split-bf16 form, fp32 to rounding; the rest on v_mfma_f32_32x32x2_f32).  The Nature-CNN torso runs on nature_cnn.hip
// (dq_cnn_forward_torso / dq_cnn_backward_torso); this file owns everything after
// the 7744-wide state vector.
//
// Rows: R = nq * B quantile rows, row r = q * B + b (tf.tile of the state, atari_lib.py:174),
// so the state row of r is r % B.  E = quantile_embedding_dim, F = 7744, H = 512.
//
//   forward                                                   (FLOP at R = 4096, E = 64)
//     cos[r][i] = cos((i+1) * pi * tau[r])                     atari_lib.py:176-178
//     emb = relu(cos We^T + be); x = state[r % B] * emb         :179-185     4.1 G  (1 launch)
//     h   = relu(x W1^T + b1)                                   :186-188    32.5 G  (split-K 4 + sum)
//     q   = h W2^T + b2                                         :189-191    small
//   backward (TF autodiff of the same graph)
//     dh   = (dq W2) * (h > 0);   dW2 | db2 = dq^T [h | 1]
//     dx   = dh W1  ->  d tiled = dx * emb,  d pre = (emb > 0) ? dx * state : 0     32.5 G
//     dW1 | db1 = dh^T [x | 1]                                                     32.5 G
//     dWe | dbe = dpre^T [cos | 1]                                                   4.1 G
//       (dbe summed in the dX epilogue when nq | 128: dWe then a 128 x 64 tile, not 128 x 128)
//     d state[b] = (state[b] > 0) * sum_q d tiled[q B + b]   (the torso's ReLU, then its backward)
// The 7744-wide intermediates (emb, x, d tiled, d pre: 127 MB each at R = 4096) are
// kept in HBM: each is written once and read by the next GEMM as a streamed operand.
#include "cnn_tile.h"

namespace dq {
namespace iqn {

using namespace dq::cnn;

constexpr int F = 11 * 11 * 64;   // 7744, the torso's state vector
constexpr int H = 512;
// h = relu(x W1^T + b1): K = 7744, 4 slabs (R/128 x 4 tiles x 4) -- two 16-wave blocks per
// CU; 4 fills the 512 slots once at R = 4096 and 1.5 times at R = 6144, measured best
// (config 5: 4 -> 614-616, 6 -> 609-610, 8 -> 607-608 steps/s, profiles/r2_s5_iqn_fc1_split_ab.log)
constexpr int kSplitFc1 = 4;
constexpr int kSplitW1 = 2;       // dW1: K = R (1 / 4 measured equal, profiles/r2_s5_iqn_dw1_split_ab.log)
constexpr int kSplitWe = 8;       // dWe: K = R, 61 row tiles
constexpr int kSplitW2 = 32;      // dW2: M = A, K = R

// The 7744-wide GEMMs on the split-bf16 matrix-core form (cnn_tile.h X6Img / X6ImgT:
// fp32 operands as exact hi + mid + lo bf16 sums, the six pairs above fp32 rounding,
// v_mfma_f32_32x32x16_bf16): the embedding, both FC1 forwards, dW1 and dWe.  dX stays
// on the exact-f32 form: its d state feeds the torso's weight gradients, sums over every
// pixel that cancel to ~1/100 of their terms, and the single-accumulator split form
// moved them from 5e-7 to 1.3e-5 of scale against float64 at B = 64, N = 64 (a bias
// from the small correction products rounding into the large accumulator; with the
// corrections in their own accumulator they fall to 5e-7 but the 16 extra
// registers cost the second 16-wave block per CU, config 5 727 vs 751 steps/s), and x6
// bought dX no time in the two-stream step (734 with vs 751 without).
// Measured (config 5, same box): exact f32 616, this 751 steps/s (profiles/r3_s3_x6/).
constexpr bool kIqnX6 = true;
constexpr bool kDxX6 = false;
template <int WM, int WN, int WK, class AL, class BL, class EP>
void gemm_iqn(Ctx& c, AL a, BL b, EP e, int M, int N, int K, int splits = 1) {
  gemm_form<WM, WN, WK, kIqnX6>(c, a, b, e, M, N, K, splits);
}

__device__ __forceinline__ float uniform_of(uint64_t seed, int64_t call, int64_t i) {
  // a splitmix64 hash of (seed, call, i), 24 random bits -> k * 2^-24
  uint64_t z = seed + (uint64_t)call * 0x9E3779B97F4A7C15ull + (uint64_t)(i + 1) * 0xD1B54A32D192ED03ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (float)(z >> 40) * (1.0f / 16777216.0f);
}

__device__ __forceinline__ float cos_feature(int k, float tau) {
  const float pi = 3.14159265358979323846f;           // tf.constant(math.pi), float32
  // tf.cast(tf.range(1, E + 1), float32) * pi * quantile_net, left to right, then tf.cos
  return cosf(__fmul_rn(__fmul_rn((float)(k + 1), pi), tau));
}

__global__ __launch_bounds__(256) void k_cos_embedding(const float* __restrict__ tau, int64_t n,
                                                        int E, float* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t r = i / E;
  out[i] = cos_feature((int)(i - r * E), tau[r]);
}

// tau (k_uniform_draw's draws of call counter[0]) and their cosine embedding in one launch
// (the counter is bumped by the next launch, k_bump_counter: a last-block ticket on one
// counter costs ~12 ns per arriving block, more than the launch it would save)
__global__ __launch_bounds__(256) void k_tau_cos(const int64_t* __restrict__ counter, uint64_t seed,
                                                 int64_t R, int E, float* __restrict__ tau_out,
                                                 float* __restrict__ cos_out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= R * E) return;
  const int64_t r = i / E;
  const int k = (int)(i - r * E);
  const float tau = uniform_of(seed, counter[0], r);
  if (k == 0) tau_out[r] = tau;
  cos_out[i] = cos_feature(k, tau);
}

__device__ __forceinline__ float4 mul4(float4 a, float4 b) {
  return make_float4(__fmul_rn(a.x, b.x), __fmul_rn(a.y, b.y), __fmul_rn(a.z, b.z), __fmul_rn(a.w, b.w));
}

// x = tiled state * emb (atari_lib.py:185) formed by the operand loaders from the kept emb
// and the (B, 7744) state instead of read from a stored x: the online network's forward
// then writes emb only (one 127 MB stream instead of two) and its FC1 forward / dW1 read
// emb + state (L2-resident, 2 MB) in place of x -- the same products, bitwise.
// FC1 forward's A operand: x[r][k..k+3]
struct RowKHad {
  static constexpr bool kFast = true;
  const float* emb;
  const float* state;
  int B;
  __device__ __forceinline__ float4 get(int r, int k, int rlim, int klim) const {
    const bool ok = r < rlim && k < klim;
    return mul4(bload4(state, (r % B) * F + k, ok), bload4(emb, r * F + k, ok));
  }
};
// dW1's B operand (ColKOnes over x): B(n, k = quantile row) = x[k][n], ones column at n == F
struct ColKOnesHad {
  static constexpr bool kFast = false;
  const float* emb;
  const float* state;
  int B;
  __device__ __forceinline__ float4 get(int n, int k, int, int klim) const {
    const bool ok = n < F && k < klim;
    const float4 v = mul4(bload4(state, (k % B) * F + n, ok), bload4(emb, k * F + n, ok));
    return (n == F && k < klim) ? make_float4(1.0f, 0.0f, 0.0f, 0.0f) : v;
  }
};

// emb = relu(acc + be[n]) (kept for the backward if emb != null); x = state[r % B][n] * emb
// (not stored if x == null: the loaders above form it)
struct EpiEmb {
  float* emb;
  float* x;
  const float* bias;
  const float* state;
  int B;
  static constexpr bool kVec = true;      // 4 columns per call: 16-B loads and stores
  __device__ __forceinline__ void operator()(int m, int n, float v, int) const {
    const float e = fmaxf(__fadd_rn(v, bias[n]), 0.0f);
    const int64_t i = (int64_t)m * F + n;
    if (emb) emb[i] = e;
    if (x) x[i] = __fmul_rn(state[(int64_t)(m % B) * F + n], e);
  }
  __device__ __forceinline__ void vec4(int m, int n, float4 v) const {
    const float4 b = ld4(bias + n);
    float4 e;
    e.x = fmaxf(__fadd_rn(v.x, b.x), 0.0f);
    e.y = fmaxf(__fadd_rn(v.y, b.y), 0.0f);
    e.z = fmaxf(__fadd_rn(v.z, b.z), 0.0f);
    e.w = fmaxf(__fadd_rn(v.w, b.w), 0.0f);
    const int64_t i = (int64_t)m * F + n;
    if (emb) *reinterpret_cast<float4*>(emb + i) = e;
    if (x) *reinterpret_cast<float4*>(x + i) = mul4(ld4(state + (int64_t)(m % B) * F + n), e);
  }
};

// dx -> d tiled = dx * emb, d pre = (emb > 0) ? dx * state[r % B] : 0  (Mul + ReluGrad)
struct EpiDx {
  float* dtl;
  float* dpre;
  const float* emb;
  const float* state;
  int B;
  static constexpr bool kVec = true;
  __device__ __forceinline__ void operator()(int m, int n, float v, int) const {
    const int64_t i = (int64_t)m * F + n;
    const float e = emb[i];
    dtl[i] = __fmul_rn(v, e);
    dpre[i] = e > 0.0f ? __fmul_rn(v, state[(int64_t)(m % B) * F + n]) : 0.0f;
  }
  __device__ __forceinline__ void vec4(int m, int n, float4 v) const {
    const int64_t i = (int64_t)m * F + n;
    const float4 e = ld4(emb + i), s = ld4(state + (int64_t)(m % B) * F + n);
    *reinterpret_cast<float4*>(dtl + i) =
        make_float4(__fmul_rn(v.x, e.x), __fmul_rn(v.y, e.y), __fmul_rn(v.z, e.z), __fmul_rn(v.w, e.w));
    *reinterpret_cast<float4*>(dpre + i) =
        make_float4(e.x > 0.0f ? __fmul_rn(v.x, s.x) : 0.0f, e.y > 0.0f ? __fmul_rn(v.y, s.y) : 0.0f,
                    e.z > 0.0f ? __fmul_rn(v.z, s.z) : 0.0f, e.w > 0.0f ? __fmul_rn(v.w, s.w) : 0.0f);
  }
};

// dX with the rows taken b-major (RowKQ, nq | 128): the block holds whole samples, so
// tf.tile's gradient -- d state[b] = sum over q in order of dx * emb, then the torso's
// last ReLU -- is summed in LDS and d tiled never goes to HBM (k_tile_grad's order and
// arithmetic, without its 127 MB write + read and launch); d pre as EpiDx.
//
// With dbe_part set it also sums the tile's d pre rows per column (the embedding's bias
// gradient, dbe = sum over the R rows of d pre): each thread over its 4 rows, the wave's two
// row groups by one lane exchange, the 16 waves' partials in LDS in wave order -> one row of
// dbe_part (R/128, F) per block, summed over the row tiles in order by k_colsum.  dWe then
// needs only the E cosine columns (a 128 x 64 tile instead of 128 x 128 for E + 1 = 65).
struct EpiDxQ {
  static constexpr bool kBlock = true;
  static constexpr int kBlockExtra = 16 * 128;   // per-wave column partials of d pre
  float* dpre;
  float* dstate;
  float* dbe_part;
  const float* emb;
  const float* state;
  int B, nq;
  // the per-element form is never reached (kBlock takes the block path); it only has to compile
  __device__ __forceinline__ void operator()(int, int, float, int) const {}
  __device__ __forceinline__ void block(float* T, int ldt, int m0, int n0, int M, int N) const {
    constexpr int BM = 128, BN = 128;
    float cs0 = 0.0f, cs1 = 0.0f, cs2 = 0.0f, cs3 = 0.0f;   // blockDim 1024: c is fixed per thread
    for (int idx = threadIdx.x; idx < BM * BN / 4; idx += blockDim.x) {
      const int t = idx / (BN / 4), c = 4 * (idx % (BN / 4));
      const int m = m0 + t, n = n0 + c;
      if (m >= M || n >= N) continue;
      const int b = m / nq, r = (m - b * nq) * B + b;
      const int64_t i = (int64_t)r * F + n;
      const float4 e = ld4(emb + i), s = ld4(state + (int64_t)b * F + n);
      float* v = T + t * ldt + c;
      const float4 dp =
          make_float4(e.x > 0.0f ? __fmul_rn(v[0], s.x) : 0.0f, e.y > 0.0f ? __fmul_rn(v[1], s.y) : 0.0f,
                      e.z > 0.0f ? __fmul_rn(v[2], s.z) : 0.0f, e.w > 0.0f ? __fmul_rn(v[3], s.w) : 0.0f);
      *reinterpret_cast<float4*>(dpre + i) = dp;
      cs0 = __fadd_rn(cs0, dp.x);
      cs1 = __fadd_rn(cs1, dp.y);
      cs2 = __fadd_rn(cs2, dp.z);
      cs3 = __fadd_rn(cs3, dp.w);
      v[0] = __fmul_rn(v[0], e.x);        // d tiled, kept in LDS
      v[1] = __fmul_rn(v[1], e.y);
      v[2] = __fmul_rn(v[2], e.z);
      v[3] = __fmul_rn(v[3], e.w);
    }
    float* P = T + BM * ldt;              // [16 waves][BN]
    if (dbe_part) {
      const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
      cs0 = __fadd_rn(cs0, __shfl_down(cs0, 32));
      cs1 = __fadd_rn(cs1, __shfl_down(cs1, 32));
      cs2 = __fadd_rn(cs2, __shfl_down(cs2, 32));
      cs3 = __fadd_rn(cs3, __shfl_down(cs3, 32));
      if (lane < 32)
        *reinterpret_cast<float4*>(P + w * BN + 4 * lane) = make_float4(cs0, cs1, cs2, cs3);
    }
    __syncthreads();
    if (dbe_part && (int)threadIdx.x >= (int)blockDim.x - BN) {   // waves the q sums below leave idle
      const int c = threadIdx.x - (blockDim.x - BN), n = n0 + c;
      if (n < N) {
        float acc = P[c];
        for (int w = 1; w < 16; ++w) acc = __fadd_rn(acc, P[w * BN + c]);
        dbe_part[(int64_t)(m0 / BM) * F + n] = acc;
      }
    }
    const int nb = BM / nq;
    for (int j = threadIdx.x; j < nb * BN; j += blockDim.x) {
      const int bl = j / BN, c = j - bl * BN;
      const int b = m0 / nq + bl, n = n0 + c;
      if (b * nq >= M || n >= N) continue;
      float acc = 0.0f;
      for (int q = 0; q < nq; ++q) acc = __fadd_rn(acc, T[(bl * nq + q) * ldt + c]);
      const int64_t i = (int64_t)b * F + n;
      dstate[i] = state[i] > 0.0f ? acc : 0.0f;
    }
  }
};

// tf.tile's gradient (the sum over the nq copies, q in order) and the torso's last ReLU
__global__ __launch_bounds__(256) void k_tile_grad(const float* __restrict__ dtl,
                                                    const float* __restrict__ state, int B, int nq,
                                                    float* __restrict__ dstate) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)B * F) return;
  float s = 0.0f;
  for (int q = 0; q < nq; ++q) s = __fadd_rn(s, dtl[(int64_t)q * B * F + i]);
  dstate[i] = state[i] > 0.0f ? s : 0.0f;
}

// dbe[n] = sum over the row tiles t, in order, of part[t][n]
__global__ __launch_bounds__(256) void k_colsum(const float* __restrict__ part, int tiles, int n,
                                                 float* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float s = part[i];
  for (int t0 = 1; t0 < tiles; t0 += 8) {     // 8 loads in flight, then the sums in order
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = part[(int64_t)min(t0 + u, tiles - 1) * n + i];
#pragma unroll
    for (int u = 0; u < 8; ++u) s = t0 + u < tiles ? __fadd_rn(s, v[u]) : s;
  }
  out[i] = s;
}

void forward(Ctx& c, const dq_iqn_head* hp, int B, int nq, const float* state, const float* tau,
             const dq_iqn_acts* a) {
  const int R = nq * B, E = hp->embed_dim, A = hp->num_actions;
  if (!c.dry && tau) {               // tau NULL: a->cos came with the draws (k_tau_cos)
    const int64_t n = (int64_t)R * E;
    hipLaunchKernelGGL(k_cos_embedding, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, c.s, tau,
                       n, E, a->cos);
  }
  gemm_iqn<4, 4, 1>(c, RowK{a->cos, E}, RowK{hp->emb_w, E}, EpiEmb{a->emb, a->x, hp->emb_b, state, B},
                R, F, E);
  if (a->x)
    gemm_iqn<4, 4, 1>(c, RowK{a->x, F}, RowK{hp->fc1_w, F}, EpiBiasAct{a->h, hp->fc1_b, H, true}, R, H,
                  F, kSplitFc1);
  else                               // x formed from emb and state by the loader
    gemm_iqn<4, 4, 1>(c, RowKHad{a->emb, state, B}, RowK{hp->fc1_w, F},
                  EpiBiasAct{a->h, hp->fc1_b, H, true}, R, H, F, kSplitFc1);
  gemm<1, 1, 16>(c, RowK{a->h, H}, RowK{hp->fc2_w, H}, EpiBiasAct{a->q, hp->fc2_b, A, false}, R,
                 A, H);
}

void backward(Ctx& c, const dq_iqn_head* hp, const dq_iqn_head* hg, int B, int nq,
              const float* state, const dq_iqn_acts* a, const float* dq, dq_iqn_grads* d,
              float* dstate) {
  const int R = nq * B, E = hp->embed_dim, A = hp->num_actions;
  gemm<1, 1, 16>(c, RowKScalar{dq, A}, ColK{hp->fc2_w, H}, EpiMask{d->dh, a->h, H}, R, H, A);
  gemm<1, 4, 4>(c, ColKScalar{dq, A}, ColKOnes{a->h, H}, EpiGrad{hg->fc2_w, hg->fc2_b, H}, A,
                H + 1, R, kSplitW2);
  const bool fuse_tile = 128 % nq == 0;   // whole samples per 128-row tile
  // the bias gradient of the embedding from the dX epilogue (d tiled's buffer, unused when
  // fuse_tile, holds the (R/128, F) column partials)
  const bool we_narrow = fuse_tile;
  auto dw1 = [&]() {
    if (a->x)
      gemm_iqn<4, 4, 1>(c, ColK{d->dh, H}, ColKOnes{a->x, F}, EpiGrad{hg->fc1_w, hg->fc1_b, F}, H,
                        F + 1, R, kSplitW1);
    else
      gemm_iqn<4, 4, 1>(c, ColK{d->dh, H}, ColKOnesHad{a->emb, state, B},
                        EpiGrad{hg->fc1_w, hg->fc1_b, F}, H, F + 1, R, kSplitW1);
  };
  // dX before dW1 (dW1 first, so the store-bound target embedding would run beside dW1's
  // matrix work on the two-stream step, measured 1% slower)
  if (fuse_tile) {
    if (!c.dry)
      hipLaunchKernelGGL((k_igemm<4, 4, 1, RowKQ, ColK, EpiDxQ, kDxX6>), dim3((R + 127) / 128, (F + 127) / 128),
                         dim3(1024), 0, c.s, RowKQ{d->dh, H, B, nq}, ColK{hp->fc1_w, F},
                         EpiDxQ{d->dpre, dstate, we_narrow ? d->dtl : nullptr, a->emb, state, B, nq},
                         R, F, H, H);
  } else {
    gemm_form<4, 4, 1, kDxX6>(c, RowK{d->dh, H}, ColK{hp->fc1_w, F},
                              EpiDx{d->dtl, d->dpre, a->emb, state, B}, R, F, H, 1);
  }
  dw1();
  if (we_narrow) {           // dWe over the E cosine columns, dbe from the row-tile partials
    gemm_iqn<4, 2, 2>(c, ColK{d->dpre, F}, ColK{a->cos, E}, EpiGrad{hg->emb_w, hg->emb_b, E}, F, E, R,
                  kSplitWe);
    if (!c.dry)
      hipLaunchKernelGGL(k_colsum, dim3((F + 255) / 256), dim3(256), 0, c.s, d->dtl, (R + 127) / 128, F,
                         hg->emb_b);
  } else                     // 128 x 128 tiles over [cos | 1]
    gemm_iqn<4, 4, 1>(c, ColK{d->dpre, F}, ColKOnes{a->cos, E}, EpiGrad{hg->emb_w, hg->emb_b, E}, F,
                  E + 1, R, kSplitWe);
  if (!c.dry && !fuse_tile) {
    const int64_t n = (int64_t)B * F;
    hipLaunchKernelGGL(k_tile_grad, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, c.s, d->dtl,
                       state, B, nq, dstate);
  }
}

// U[0, 1) float32 draws of call `counter[0]` of a generator: a splitmix64 hash of (seed,
// call, i), 24 random bits -> k * 2^-24.  The call counter lives on the device and is
// bumped by a second one-thread launch, so replaying a captured graph draws new values
// exactly as the same sequence of eager calls does.
__global__ __launch_bounds__(256) void k_uniform_draw(const int64_t* __restrict__ counter,
                                                       uint64_t seed, int64_t n,
                                                       float* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  out[i] = uniform_of(seed, counter[0], i);
}

__global__ void k_bump_counter(int64_t* counter) { counter[0] += 1; }

}  // namespace iqn
}  // namespace dq

using namespace dq;

static bool head_ok(const dq_iqn_head* h) {
  return h && h->embed_dim >= 4 && h->embed_dim % 4 == 0 && h->num_actions >= 1 && h->emb_w &&
         h->emb_b && h->fc1_w && h->fc1_b && h->fc2_w && h->fc2_b;
}

extern "C" {

int dq_iqn_head_forward(const dq_iqn_head* hp, int32_t batch, int32_t nq, const float* state,
                        const float* taus, dq_iqn_acts* a, float* ws, void* stream) {
  DQ_CHECK_ARG(head_ok(hp) && state && a && ws && batch >= 1 && nq >= 1, "bad arguments");
  DQ_CHECK_ARG(a->cos && (a->x || a->emb) && a->h && a->q, "null activation buffer");
  DQ_CHECK_ARG((int64_t)batch * nq * iqn::F < ((int64_t)1 << 31), "R * 7744 must fit int32");
  cnn::Ctx c{(hipStream_t)stream, ws, false, 0};
  iqn::forward(c, hp, batch, nq, state, taus, a);
  DQ_CHECK_LAUNCH("dq_iqn_head_forward");
  return DQ_OK;
}

int dq_iqn_head_backward(const dq_iqn_head* hp, const dq_iqn_head* hg, int32_t batch, int32_t nq,
                         const float* state, const dq_iqn_acts* a, const float* dq,
                         dq_iqn_grads* d, float* dstate, float* ws, void* stream) {
  DQ_CHECK_ARG(head_ok(hp) && head_ok(hg) && state && a && dq && d && dstate && ws && batch >= 1 &&
               nq >= 1, "bad arguments");
  DQ_CHECK_ARG(hg->embed_dim == hp->embed_dim && hg->num_actions == hp->num_actions,
               "gradient head shape differs");
  DQ_CHECK_ARG(a->cos && a->emb && a->h && d->dh && d->dtl && d->dpre,
               "the backward needs the forward's emb (kept) and gradient buffers");
  cnn::Ctx c{(hipStream_t)stream, ws, false, 0};
  iqn::backward(c, hp, hg, batch, nq, state, a, dq, d, dstate);
  DQ_CHECK_LAUNCH("dq_iqn_head_backward");
  return DQ_OK;
}

int dq_uniform_draw(int64_t* counter, uint64_t seed, int64_t n, float* out, void* stream) {
  DQ_CHECK_ARG(counter && out && n >= 0, "bad arguments");
  if (n > 0)
    hipLaunchKernelGGL(iqn::k_uniform_draw, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, counter, seed, n, out);
  hipLaunchKernelGGL(iqn::k_bump_counter, dim3(1), dim3(1), 0, (hipStream_t)stream, counter);
  DQ_CHECK_LAUNCH("dq_uniform_draw");
  return DQ_OK;
}

int dq_iqn_tau_cos(int64_t* counter, uint64_t seed, int32_t rows, int32_t embed_dim, float* taus,
                   float* cos_out, void* stream) {
  DQ_CHECK_ARG(counter && taus && cos_out && rows >= 1 && embed_dim >= 1, "bad arguments");
  const int64_t n = (int64_t)rows * embed_dim;
  hipLaunchKernelGGL(iqn::k_tau_cos, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, counter, seed, (int64_t)rows, (int)embed_dim, taus, cos_out);
  hipLaunchKernelGGL(iqn::k_bump_counter, dim3(1), dim3(1), 0, (hipStream_t)stream, counter);
  DQ_CHECK_LAUNCH("dq_iqn_tau_cos");
  return DQ_OK;
}

size_t dq_iqn_workspace_floats(int32_t batch, int32_t nq, int32_t num_actions, int32_t embed_dim) {
  dq_iqn_head h = {};
  h.embed_dim = embed_dim;
  h.num_actions = num_actions;
  dq_iqn_acts a = {};
  dq_iqn_grads d = {};
  cnn::Ctx f{nullptr, nullptr, true, 0};
  iqn::forward(f, &h, batch, nq, nullptr, nullptr, &a);
  cnn::Ctx b{nullptr, nullptr, true, 0};
  iqn::backward(b, &h, &h, batch, nq, nullptr, &a, nullptr, &d, nullptr);
  return f.need > b.need ? f.need : b.need;
}

}  // extern "C"
