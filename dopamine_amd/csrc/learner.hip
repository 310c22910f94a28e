// Learner-side kernels: C51 target + projection + cross-entropy (+ PER weights
// and new priorities), DQN Huber target, IQN quantile-Huber loss, and the TF1
// Adam / RMSProp updates over one flat fp32 parameter buffer.
// Restates the TF1 graph code of rainbow_agent.py:200-305 + 340-494,
// dqn_agent.py:283-322, implicit_quantile_agent.py:190-321 and the TF1
// ApplyAdam / ApplyCenteredRMSProp op semantics.
#include <algorithm>

#include "c51_dev.h"

namespace dq {

// ---------------------------------------------------------------------------
// C51.  One 1024-thread block; wave w handles samples w, w+16, ...; lane = atom.
// ---------------------------------------------------------------------------
struct C51Args {
  const float* ol;
  const float* tl;
  const int32_t* act;
  const float* rew;
  const uint8_t* term;
  const float* probs;
  const float* support;
  int B, A, N;
  float cg;
  float* grad;
  float* loss_out;
  float* prio_out;
  float* mean_out;
};

// The fused path's extras: logits written out (the CNN never stores them), and the
// fc2 input gradient d h = (dlogits . W2) * (h > 0) -- only the chosen action's
// N logits of a sample have a nonzero gradient, so row b of d h is an N-term sum.
struct C51Extra {
  float* ol_out;       // (B, A*N) online logits, may be NULL
  float* tl_out;       // (B, A*N) target logits, may be NULL
  const float* w2;     // (A*N, H) online fc2 weights; NULL: no d h
  const float* h;      // (B, H) online fc1 activation (ReLU mask)
  float* dh;           // (B, H)
  int H;
};

// One block per sample b.  Wave a (strided) computes the target softmax / Q of
// action a; every wave then takes the greedy action (first max) and builds Tz,
// the waves split the Eq.-7 projection's source atoms j between them (lane =
// target atom i, term c(i, j) * p_j into LDS), and wave 0 sums the terms in j
// order -- the reference's arithmetic and order, in N / waves serial steps
// instead of N -- before the softmax cross-entropy of the chosen online logits.
// The fused path (x.w2) also forms d h from the chosen action's N logit
// gradients; its W2 rows are fetched into LDS at the start, under the chain.

#ifdef DQ_C51_PROF
__device__ long long g_c51_t[256][8];
__device__ long long g_c51_w[256][16];
__device__ long long g_c51_w2[256][16];
__device__ long long g_c51_w0[256][16];
#define C51_W0() if ((threadIdx.x & 63) == 0) g_c51_w0[blockIdx.x][threadIdx.x >> 6] = wall_clock64()
#define C51_T(k) if (threadIdx.x == 0) g_c51_t[blockIdx.x][k] = wall_clock64()
#define C51_W2() if ((threadIdx.x & 63) == 0) g_c51_w2[blockIdx.x][threadIdx.x >> 6] = wall_clock64()
#define C51_W() if ((threadIdx.x & 63) == 0) g_c51_w[blockIdx.x][threadIdx.x >> 6] = wall_clock64()
#else
#define C51_T(k)
#define C51_W()
#define C51_W2()
#define C51_W0()
#endif
// Compile-time switches of k_c51 (the runtime pointers they stand for are non-NULL exactly
// when the bit is set): no kernel-argument test is left in the chain, so the compiler loads
// the arguments in one batch instead of one dependent scalar round per branch.
constexpr int kC51Probs = 1, kC51W2 = 2, kC51LogitsOut = 4;
// the fused path's d h: 4 blocks per sample (8 or 2 measured a tie)
constexpr int kC51Split = 4;

// LDS floats of k_c51's head (before the fused path's W2 rows), 4-float aligned
__host__ __device__ constexpr int c51_head_floats(int A, int N, int nw) {
  return (A * N + A + N + N * kWave + 2 * nw * kWave + 3) / 4 * 4;
}

template <class LS, int kF>
__global__ __launch_bounds__(1024) void k_c51(C51Args a, LS ol, LS tl, C51Extra x) {
  constexpr bool kProbs = kF & kC51Probs, kW2 = kF & kC51W2, kOut = kF & kC51LogitsOut;
  warm_kernargs<sizeof(C51Args) + 2 * sizeof(LS) + sizeof(C51Extra)>();
  extern __shared__ __attribute__((aligned(16))) float smem[];
  // S blocks per sample (gridDim.x = B * S): each runs the whole loss chain (latency-bound,
  // so the copies cost nothing) and forms d h for its 1/S of the H columns -- the W2 rows'
  // LDS traffic, what bounds that product, split over S CUs.  Part 0 writes the outputs.
  const int N = a.N, A = a.A, T = blockDim.x, S = gridDim.x / a.B;
  const int b = blockIdx.x / S, part = blockIdx.x - b * S, HS = kW2 ? x.H / S : 0;
  const bool writer = part == 0;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = T >> 6;
  float* s_p = smem;                 // [A][N] target probabilities
  float* s_q = s_p + A * N;          // [A]    target Q
  float* s_g = s_q + A;              // [N]    the chosen action's logit gradient
  float* s_c = s_g + N;              // [N][64] projection terms c(i, j)
  int* s_lo = reinterpret_cast<int*>(s_c + N * kWave);   // [nw][64] first / last source atom
  int* s_hi = s_lo + nw * kWave;                          // with c(i, j) > 0, per wave
  float* s_w = smem + c51_head_floats(A, N, nw);          // [N][HS] fc2 row slices, 16-B aligned
  const bool on = lane < N;
  const float ninf = -__builtin_inff();
  C51_T(0);
  // every ordinary global load of the chain is issued here, before any LDS-DMA
  // (hipcc drains vmcnt to 0 at the first use of a plain load issued behind one)
  const float z = on ? a.support[lane] : 0.0f;
  const int ab = a.act[b];
  const float rew_b = a.rew[b], term_b = (float)a.term[b];
  const float vmin = a.support[0], vmax = a.support[N - 1], z1 = a.support[1];
  // PER: every wave loads all B probabilities (B <= 64: one per lane) and takes their min
  // itself, so the importance weight needs no cross-wave step
  const float pr_t = kProbs ? a.probs[min(lane, a.B - 1)] : 0.0f;
  const float pr_b = kProbs ? a.probs[b] : 0.0f;
  const float hv = kW2 ? x.h[(int64_t)b * x.H + part * HS + min((int)threadIdx.x, HS - 1)] : 0.0f;
  // the chosen online logit row (wave 0 uses it last) and the first target row of each
  // wave (nw <= A): loaded by every lane at clamped indices, so both rows' loads sit in one
  // basic block and are all in flight before the first wait
  // (their sums are formed after the c(i, j) loop below, which runs under the loads)
  const int lc = min(lane, N - 1);
  const typename LS::Pend x0 = tl.load_bc(b, min(wave, A - 1) * N + lc);   // (not behind act[b])
  typename LS::Pend y0;
  if (wave == 0)              // (the vector-memory issue of 16-band rows is what costs)
    y0 = ol.load_bc(b, ab * N + lc);
  // The Eq.-7 clipped quotients c(i, j) = clip(1 - |clip(Tz_j) - z_i| / dz, 0, 1) need only
  // the reward, the terminal flag and the support: formed now, while the logits load
  // (wave w takes source atoms j = w, w + nw, ...; lane = target atom i).  clip(Tz_j) is
  // non-decreasing in j, so the j with c(i, j) > 0 are one run [lo_i, hi_i]: each wave
  // records its own first and last such j per lane.
  {
    const float dz = __fsub_rn(z1, vmin);
    const float gt = __fmul_rn(a.cg, __fsub_rn(1.0f, term_b));
    C51_W0();
    int lo = kWave, hi = -1;
    for (int j = __builtin_amdgcn_readfirstlane(wave); j < N; j += nw) {
      const float zj = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(z), j));
      const float tzj = fminf(fmaxf(__fadd_rn(rew_b, __fmul_rn(gt, zj)), vmin), vmax);
      if (on) {
        float c = __fsub_rn(1.0f, __fdiv_rn(fabsf(__fsub_rn(tzj, z)), dz));
        c = fminf(fmaxf(c, 0.0f), 1.0f);
        s_c[j * kWave + lane] = c;
        if (c > 0.0f) {
          lo = min(lo, j);
          hi = j;
        }
      }
    }
    s_lo[wave * kWave + lane] = lo;
    s_hi[wave * kWave + lane] = hi;
  }
  C51_W2();
  float y = ninf;
  if (wave == 0) y = on ? ol.sum(y0) : ninf;
  float xv[4];
  xv[0] = (wave < A && on) ? tl.sum(x0) : ninf;
#pragma unroll
  for (int r = 1; r < 4; ++r) {
    const int act = wave + r * nw;
    xv[r] = (act < A && on) ? tl.sum(tl.load_bc(b, act * N + lane)) : ninf;
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int act = wave + r * nw;
    if (act >= A) break;
    const float v = xv[r];
    if (kOut && x.tl_out && on && writer) x.tl_out[((int64_t)b * A + act) * N + lane] = v;
    const float mx = fast_max(v);
    const float e = on ? expf(__fsub_rn(v, mx)) : 0.0f;
    const float p = __fdiv_rn(e, fast_sum(e));
    const float q = fast_sum(on ? __fmul_rn(z, p) : 0.0f);
    if (on) s_p[act * N + lane] = p;
    if (lane == 0) s_q[act] = q;
  }
  C51_T(1);
  C51_W();
  // the chosen online row's softmax terms and the PER importance weight (wave 0), before
  // the barrier.  rb:277-280: w_b = r(p_b) / max_i r(p_i), r(p) = 1 / sqrt(p + eps); r
  // rounds monotonically (non-increasing), so max_i r(p_i) = r(min_i p_i) exactly.
  float sh = 0.0f, ey = 0.0f, lse = 0.0f, py = 0.0f, w = 1.0f;
  if (wave == 0) {
    if (kProbs) {
      float pm = pr_t;
      for (int i = lane + kWave; i < a.B; i += kWave) pm = fminf(pm, a.probs[i]);
      pm = fast_min(pm);
      const float m = __fdiv_rn(1.0f, sqrt_rn(__fadd_rn(pm, 1e-10f)));
      w = __fdiv_rn(__fdiv_rn(1.0f, sqrt_rn(__fadd_rn(pr_b, 1e-10f))), m);
    }
    const float my = fast_max(y);
    sh = on ? __fsub_rn(y, my) : 0.0f;
    ey = on ? expf(sh) : 0.0f;
    const float sy = fast_sum(ey);
    lse = logf(sy);
    py = __fdiv_rn(ey, sy);
  }
  if (kOut && x.ol_out && writer)
    for (int act = wave; act < A; act += nw) {
      const int64_t i = ((int64_t)b * A + act) * N + lane;
      if (on) x.ol_out[i] = act == ab && wave == 0 ? y : ol.get(i);
    }
  // s_p, s_q, s_c, s_lo/hi complete.  A bare barrier: __syncthreads' release fence would
  // also wait for vmcnt(0), i.e. for the whole LDS-DMA issued next
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  C51_T(2);
  // fused d h: this block's column slice of the chosen action's N W2 rows (N x HS floats)
  // streams into LDS by LDS-DMA (global_load_lds: 16 B per lane from its own address, 1 KB
  // contiguous in LDS per wave instruction, no registers), landing under the rest of the
  // loss chain.  Issued by waves 1.. (wave 0 runs the chain) after the
  // barrier, so neither the chain nor the barrier waits behind the issue.  (Measured: the
  // rows as plain loads into registers, issued with the logits or after the softmax,
  // queue the logits' loads behind them: 7,585 / 7,610 vs 7,700 steps/s.)
  if (kW2 && (wave > 0 || nw == 1)) {
    const int rc = HS >> 2, chunks = N * rc, nq = (chunks + 63) >> 6;   // 16-B chunks
    const int w0 = nw > 1 ? wave - 1 : 0, nwd = nw > 1 ? nw - 1 : 1;
    const float* src = x.w2 + (int64_t)ab * N * x.H + part * HS;
    for (int q = w0; q < nq; q += nwd) {
      const int c = min(q * 64 + lane, chunks - 1);   // the tail re-reads in-bounds chunks
      const int row = c / rc;
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(src + (int64_t)row * x.H +
                                                                     4 * (c - row * rc)),
                                       (__attribute__((address_space(3))) void*)(
                                           reinterpret_cast<char*>(s_w) + q * 1024),
                                       16, 0, 0);
    }
  }
  C51_T(3);
  const float gscale = __fmul_rn(w, __fdiv_rn(1.0f, (float)a.B));
  for (int act = wave; act < A && writer; act += nw) {
    if (act == ab) continue;
    if (on) a.grad[((int64_t)b * A + act) * N + lane] = 0.0f;
  }
  if (wave == 0) {
    // greedy target action (first max)
    int astar = 0;
    const float qv = lane < A ? s_q[lane] : 0.0f;   // one LDS read, then lane reads (A <= 64)
    float best = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(qv), 0));
    for (int act = 1; act < A; ++act) {
      const float qa = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(qv), act));
      if (qa > best) {
        best = qa;
        astar = act;
      }
    }
    const float* pst = s_p + astar * N;
    // sum_j c(i, j) p_j in j order (rb:340-494) over the run [lo, hi] only: every other
    // term is c = 0 times a finite p >= 0, i.e. +0, and adding +0 to the non-negative
    // partial sum changes no bit -- the same sum as all N terms, in 8-term batches
    int lo = kWave, hi = -1;
    for (int v = 0; v < nw; ++v) {
      lo = min(lo, s_lo[v * kWave + lane]);
      hi = max(hi, s_hi[v * kWave + lane]);
    }
    float proj = 0.0f;       // (lanes >= N: lo > hi, no term)
    if (term_b != 0.0f || a.cg == 0.0f) {
      // gamma_t = 0: every source atom lands on clip(r), c(i, j) = c(i, 0) for all j and the
      // run is all N atoms -- the same j-ordered sum with c in a register and p_j read
      // across lanes (no per-term LDS round trip)
      const float ci = on ? s_c[lane] : 0.0f;
      const float pl = pst[lc];
      int j = 0;
      for (; j + 8 <= N; j += 8) {   // the lane reads of a batch ahead of its add chain
        float t[8];
#pragma unroll
        for (int u = 0; u < 8; ++u)
          t[u] = __fmul_rn(ci, __int_as_float(__builtin_amdgcn_readlane(__float_as_int(pl), j + u)));
#pragma unroll
        for (int u = 0; u < 8; ++u) proj = __fadd_rn(proj, t[u]);
      }
      for (; j < N; ++j)
        proj = __fadd_rn(proj, __fmul_rn(ci, __int_as_float(__builtin_amdgcn_readlane(__float_as_int(pl), j))));
      lo = 0;
      hi = -1;
    }
    for (int j = lo; j <= hi; j += 8) {   // 8 terms' LDS reads in flight, then summed in order
      float t[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {       // unconditional (clamped) reads, then a select:
        const int jj = min(j + u, N - 1); // a guarded read became a branch per term
        const float tt = __fmul_rn(s_c[jj * kWave + lane], pst[jj]);
        t[u] = j + u <= hi ? tt : 0.0f;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) proj = __fadd_rn(proj, t[u]);
    }
    const float loss = fast_sum(on ? __fmul_rn(proj, __fsub_rn(lse, sh)) : 0.0f);
    const float gr = on ? __fmul_rn(gscale, __fsub_rn(py, proj)) : 0.0f;
    if (on) {
      if (writer) a.grad[((int64_t)b * A + ab) * N + lane] = gr;
      s_g[lane] = gr;
    }
    if (lane == 0 && writer) {
      if (a.loss_out) a.loss_out[b] = loss;
      if (a.prio_out) a.prio_out[b] = sqrt_rn(__fadd_rn(loss, 1e-10f));
    }
  }
  C51_T(4);
  if (!kW2) return;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's LDS-DMA has landed
  __syncthreads();
  C51_T(5);
  // d h[b][j] = (h[b][j] > 0) * sum_i g_i W2[ab*N + i][j] (dh_dot's order), j in this block's slice
  for (int jl = threadIdx.x; jl < HS; jl += T) {
    const float m = jl == (int)threadIdx.x ? hv : x.h[(int64_t)b * x.H + part * HS + jl];
    const float acc = dh_dot(s_g, s_w, HS, jl, N);
    x.dh[(int64_t)b * x.H + part * HS + jl] = m > 0.0f ? acc : 0.0f;
  }
  C51_T(6);
}
#ifdef DQ_C51_PROF
extern "C" int dq_debug_c51_times(long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_c51_t), sizeof(g_c51_t)) == hipSuccess ? 0 : -1;
}
extern "C" int dq_debug_c51_wave_times(long long* out) {
  if (hipMemcpyFromSymbol(out + 256 * 16, HIP_SYMBOL(g_c51_w2), sizeof(g_c51_w2)) != hipSuccess)
    return -1;
  if (hipMemcpyFromSymbol(out + 2 * 256 * 16, HIP_SYMBOL(g_c51_w0), sizeof(g_c51_w0)) != hipSuccess)
    return -1;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_c51_w), sizeof(g_c51_w)) == hipSuccess ? 0 : -1;
}
#endif

// The online half of k_c51 (the fused Rainbow path with the target half riding in the
// forward, TgtC51Op): m = the projected target distribution (B, N) is read instead of
// formed.  Everything else is k_c51's online arithmetic in k_c51's order -- the chosen
// online row's log-softmax, the cross-entropy, PER weights, priorities, dlogits and
// d h = (dlogits . W2) * (h > 0) -- so loss, gradient and priorities are bitwise k_c51's.
// One block per sample, T = 64 * waves threads.
template <class LS>
__global__ __launch_bounds__(1024) void k_c51_online(C51Args a, LS ol, const float* __restrict__ m,
                                                     C51Extra x) {
  warm_kernargs<sizeof(C51Args) + sizeof(LS) + 8 + sizeof(C51Extra)>();
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int N = a.N, A = a.A, b = blockIdx.x, T = blockDim.x;
  float* s_g = smem;                                   // [N] the chosen row's logit gradient
  float* s_w = smem + (N + 3) / 4 * 4;                 // [N][H] fc2 rows, 16-B aligned
  __shared__ float s_red[16];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = T >> 6;
  const bool on = lane < N;
  const float ninf = -__builtin_inff();
  const int ab = a.act[b];
  const float pr_t = a.probs ? a.probs[min((int)threadIdx.x, a.B - 1)] : 0.0f;
  const float pr_b = a.probs ? a.probs[b] : 0.0f;
  const float hv = x.w2 ? x.h[(int64_t)b * x.H + min((int)threadIdx.x, x.H - 1)] : 0.0f;
  const int lc = min(lane, N - 1);
  float y = ninf, proj = 0.0f;
  if (wave == 0) {
    const float y0 = ol.get(((int64_t)b * A + ab) * N + lc);
    const float m0 = m[(int64_t)b * N + lc];
    y = on ? y0 : ninf;
    proj = on ? m0 : 0.0f;
  }
  if (a.probs) {
    float pm = pr_t;
    for (int i = threadIdx.x + T; i < a.B; i += T) pm = fminf(pm, a.probs[i]);
    pm = fast_min(pm);
    if (lane == 0) s_red[wave] = pm;
  }
  float sh = 0.0f, ey = 0.0f, lse = 0.0f, py = 0.0f;
  if (wave == 0) {
    const float my = fast_max(y);
    sh = on ? __fsub_rn(y, my) : 0.0f;
    ey = on ? expf(sh) : 0.0f;
    const float sy = fast_sum(ey);
    lse = logf(sy);
    py = __fdiv_rn(ey, sy);
  }
  if (x.ol_out)
    for (int act = wave; act < A; act += nw) {
      const int64_t i = ((int64_t)b * A + act) * N + lane;
      if (on) x.ol_out[i] = act == ab && wave == 0 ? y : ol.get(i);
    }
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");   // s_red complete (bare: see k_c51)
  if (x.w2 && (wave > 0 || nw == 1)) {
    const int bytes = N * x.H * 4, nq = (bytes + 1023) >> 10;
    const int w0 = nw > 1 ? wave - 1 : 0, nwd = nw > 1 ? nw - 1 : 1;
    const char* src = reinterpret_cast<const char*>(x.w2 + (int64_t)ab * N * x.H);
    for (int q = w0; q < nq; q += nwd) {
      const int off = min(q * 1024 + lane * 16, bytes - 16);
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(src + off),
                                       (__attribute__((address_space(3))) void*)(
                                           reinterpret_cast<char*>(s_w) + q * 1024),
                                       16, 0, 0);
    }
  }
  float w = 1.0f;
  if (a.probs) {
    float pm = s_red[0];
    for (int i = 1; i < nw; ++i) pm = fminf(pm, s_red[i]);
    const float mm = __fdiv_rn(1.0f, sqrt_rn(__fadd_rn(pm, 1e-10f)));
    w = __fdiv_rn(__fdiv_rn(1.0f, sqrt_rn(__fadd_rn(pr_b, 1e-10f))), mm);
  }
  const float gscale = __fmul_rn(w, __fdiv_rn(1.0f, (float)a.B));
  for (int act = wave; act < A; act += nw) {
    if (act == ab) continue;
    if (on) a.grad[((int64_t)b * A + act) * N + lane] = 0.0f;
  }
  if (wave == 0) {
    const float loss = fast_sum(on ? __fmul_rn(proj, __fsub_rn(lse, sh)) : 0.0f);
    const float gr = on ? __fmul_rn(gscale, __fsub_rn(py, proj)) : 0.0f;
    if (on) {
      a.grad[((int64_t)b * A + ab) * N + lane] = gr;
      s_g[lane] = gr;
    }
    if (lane == 0) {
      if (a.loss_out) a.loss_out[b] = loss;
      if (a.prio_out) a.prio_out[b] = sqrt_rn(__fadd_rn(loss, 1e-10f));
    }
  }
  if (!x.w2) return;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int j = threadIdx.x; j < x.H; j += T) {
    const float mk = j == (int)threadIdx.x ? hv : x.h[(int64_t)b * x.H + j];
    const float acc = dh_dot(s_g, s_w, x.H, j, N);
    x.dh[(int64_t)b * x.H + j] = mk > 0.0f ? acc : 0.0f;
  }
}

// bytes the LDS-DMA of N rows x H floats writes: every wave instruction lands a whole 1 KB
// (64 lanes x 16 B, the tail lanes re-reading in-bounds chunks), so the region is rounded up
// to 1 KB -- the destination is not clamped, only the source
static size_t c51_w2_lds_bytes(int N, int H) {
  return ((size_t)N * H * sizeof(float) + 1023) / 1024 * 1024;
}

// dynamic LDS of k_c51 (bytes): the head, plus the W2 rows in the LDS-DMA form
static size_t c51_lds(int A, int N, int H, int nw) {
  return (size_t)c51_head_floats(A, N, nw) * sizeof(float) + (H ? c51_w2_lds_bytes(N, H) : 0);
}

// mean(w * loss) for summaries (rb:298-301); launched only when requested.
__global__ __launch_bounds__(64) void k_wmean(const float* loss, const float* probs, int B,
                                              float* out) {
  float wmax = 1.0f;
  if (probs) {
    float m = 0.0f;
    for (int i = threadIdx.x; i < B; i += 64)
      m = fmaxf(m, __fdiv_rn(1.0f, sqrt_rn(__fadd_rn(probs[i], 1e-10f))));
    wmax = wave_max(m);
  }
  float acc = 0.0f;
  for (int b = threadIdx.x; b < B; b += 64) {
    const float w = probs ? __fdiv_rn(__fdiv_rn(1.0f, sqrt_rn(__fadd_rn(probs[b], 1e-10f))), wmax) : 1.0f;
    acc = __fadd_rn(acc, __fmul_rn(w, loss[b]));
  }
  acc = wave_sum(acc);
  if (threadIdx.x == 0) out[0] = __fdiv_rn(acc, (float)B);
}

// ---------------------------------------------------------------------------
// DQN: Bellman max target + Huber(1).  One thread per sample.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_dqn(const float* oq, const float* tq, const int32_t* act,
                                             const float* rew, const uint8_t* term, int B, int A,
                                             float cg, float* grad, float* loss_out,
                                             float* mean_out) {
  __shared__ float s_red[4];
  float part = 0.0f;
  const float invB = __fdiv_rn(1.0f, (float)B);
  for (int b = threadIdx.x; b < B; b += blockDim.x) {
    float mx = tq[(int64_t)b * A];
    for (int j = 1; j < A; ++j) mx = fmaxf(mx, tq[(int64_t)b * A + j]);
    // r + cumulative_gamma * max_a Q' * (1 - terminal)   (dqn:298-299)
    const float target =
        __fadd_rn(rew[b], __fmul_rn(__fmul_rn(cg, mx), __fsub_rn(1.0f, (float)term[b])));
    const int ab = act[b];
    const float err = __fsub_rn(oq[(int64_t)b * A + ab], target);  // predictions - labels
    const float ae = fabsf(err);
    const float quad = fminf(ae, 1.0f);
    const float lin = __fsub_rn(ae, quad);
    const float loss = __fadd_rn(__fmul_rn(__fmul_rn(0.5f, quad), quad), lin);
    if (loss_out) loss_out[b] = loss;
    part = __fadd_rn(part, loss);
    const float g = __fmul_rn(fminf(fmaxf(err, -1.0f), 1.0f), invB);
    for (int j = 0; j < A; ++j) grad[(int64_t)b * A + j] = (j == ab) ? g : 0.0f;
  }
  part = wave_sum(part);
  if ((threadIdx.x & 63) == 0) s_red[threadIdx.x >> 6] = part;
  __syncthreads();
  if (threadIdx.x == 0 && mean_out) {
    float t = 0.0f;
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) t = __fadd_rn(t, s_red[i]);
    mean_out[0] = __fdiv_rn(t, (float)B);
  }
}

// The fused DQN head (the DQN counterpart of k_c51<LogitsParts>): one 128-thread block
// per sample b.  Q(s, .) and Q'(s', .) are fc2's 16 k-band partials summed in band
// order plus the bias (bitwise dq_cnn_forward's outputs), the Bellman max target and
// Huber(1) follow k_dqn operation for operation (the max in action order), and since
// only the chosen action's output has a gradient, fc2's input gradient is one product
// per element: d h[b][k] = (h[b][k] > 0) ? g * W2[a_b][k] : 0 -- exactly what the
// backward's K = A GEMM forms (every other product is a zero).
struct DqnFusedArgs {
  LogitsParts ol, tl;
  const int32_t* act;
  const float* rew;
  const uint8_t* term;
  int B, A, H;
  float cg;
  float* grad;        // (B, A)
  float* loss_out;    // (B,)
  const float* w2;    // (A, H) online fc2 weights
  const float* h;     // (B, H) online fc1 activation (ReLU mask)
  float* dh;          // (B, H)
  float* oq_out;      // (B, A) or NULL
  float* tq_out;      // (B, A) or NULL
};

__global__ __launch_bounds__(128) void k_dqn_fused(DqnFusedArgs a) {
  warm_kernargs<sizeof(DqnFusedArgs)>();
  const int b = blockIdx.x, t = threadIdx.x, A = a.A, H = a.H;
  const int ab = a.act[b];
  // the d h operands first: they depend on the action only, not on the loss chain
  const int k4 = 4 * t;
  float4 w = make_float4(0.f, 0.f, 0.f, 0.f), hv = w;
  if (k4 < H) {
    w = *reinterpret_cast<const float4*>(a.w2 + (int64_t)ab * H + k4);
    hv = *reinterpret_cast<const float4*>(a.h + (int64_t)b * H + k4);
  }
  const int j = t & 63;
  const int64_t i = (int64_t)b * A + min(j, A - 1);
  const float oq = a.ol.get(i), tq = a.tl.get(i);
  const float r = a.rew[b], tm = (float)a.term[b];
  float mx = rl(tq, 0);
  for (int c = 1; c < A; ++c) mx = fmaxf(mx, rl(tq, c));
  // r + cumulative_gamma * max_a Q' * (1 - terminal)   (dqn:298-299)
  const float target = __fadd_rn(r, __fmul_rn(__fmul_rn(a.cg, mx), __fsub_rn(1.0f, tm)));
  const float err = __fsub_rn(rl(oq, ab), target);       // predictions - labels
  const float ae = fabsf(err);
  const float quad = fminf(ae, 1.0f);
  const float lin = __fsub_rn(ae, quad);
  const float g = __fmul_rn(fminf(fmaxf(err, -1.0f), 1.0f), __fdiv_rn(1.0f, (float)a.B));
  if (t < A) {
    a.grad[(int64_t)b * A + t] = (t == ab) ? g : 0.0f;
    if (a.oq_out) a.oq_out[(int64_t)b * A + t] = oq;
    if (a.tq_out) a.tq_out[(int64_t)b * A + t] = tq;
  }
  if (t == 0 && a.loss_out) a.loss_out[b] = __fadd_rn(__fmul_rn(__fmul_rn(0.5f, quad), quad), lin);
  if (k4 < H)
    *reinterpret_cast<float4*>(a.dh + (int64_t)b * H + k4) =
        make_float4(hv.x > 0.0f ? __fmul_rn(g, w.x) : 0.0f, hv.y > 0.0f ? __fmul_rn(g, w.y) : 0.0f,
                    hv.z > 0.0f ? __fmul_rn(g, w.z) : 0.0f, hv.w > 0.0f ? __fmul_rn(g, w.w) : 0.0f);
}

// ---------------------------------------------------------------------------
// IQN quantile-Huber.  One 64-thread block per sample b; lane = online quantile.
// ---------------------------------------------------------------------------
struct IqnArgs {
  const float* oq;
  const float* tq;
  const float* ta;
  const float* tau;
  const int32_t* act;
  const float* rew;
  const uint8_t* term;
  int B, A, N, Np, K;
  float cg, kappa;
  float* grad;
  float* loss_out;
};

__global__ __launch_bounds__(64) void k_iqn(IqnArgs a) {
  extern __shared__ __attribute__((aligned(16))) float s_T[];  // [Np]
  const int b = blockIdx.x, lane = threadIdx.x;
  const int B = a.B, A = a.A;
  // greedy next action from the mean over K target quantiles (iqn:170-188)
  float best = 0.0f;
  int astar = 0;
  for (int act = 0; act < A; ++act) {
    float s = 0.0f;
    for (int k = lane; k < a.K; k += 64) s = __fadd_rn(s, a.ta[((int64_t)k * B + b) * A + act]);
    const float m = __fdiv_rn(wave_sum(s), (float)a.K);
    if (act == 0 || m > best) {
      best = m;
      astar = act;
    }
  }
  const float gt = __fmul_rn(a.cg, __fsub_rn(1.0f, (float)a.term[b]));
  for (int j = lane; j < a.Np; j += 64)
    s_T[j] = __fadd_rn(a.rew[b], __fmul_rn(gt, a.tq[((int64_t)j * B + b) * A + astar]));
  __syncthreads();
  const int ab = a.act[b];
  const float kappa = a.kappa, hk = __fmul_rn(0.5f, kappa);
  const float gscale = __fdiv_rn(-1.0f, __fmul_rn(__fmul_rn((float)a.Np, (float)B), kappa));
  float rho_acc = 0.0f;
  for (int i = lane; i < a.N; i += 64) {
    const int64_t row = (int64_t)i * B + b;
    const float theta = a.oq[row * A + ab];
    const float tau = a.tau[row];
    float rho = 0.0f, g = 0.0f;
    for (int j = 0; j < a.Np; ++j) {
      const float u = __fsub_rn(s_T[j], theta);
      const float au = fabsf(u);
      const bool inner = au <= kappa;
      const float h = inner ? __fmul_rn(__fmul_rn(0.5f, u), u) : __fmul_rn(kappa, __fsub_rn(au, hk));
      const float w = fabsf(__fsub_rn(tau, u < 0.0f ? 1.0f : 0.0f));
      rho = __fadd_rn(rho, __fdiv_rn(__fmul_rn(w, h), kappa));
      const float dh = inner ? u : (u > 0.0f ? kappa : (u < 0.0f ? -kappa : 0.0f));
      g = __fadd_rn(g, __fmul_rn(w, dh));
    }
    rho_acc = __fadd_rn(rho_acc, rho);
    const float gv = __fmul_rn(g, gscale);
    for (int c = 0; c < A; ++c) a.grad[row * A + c] = (c == ab) ? gv : 0.0f;
  }
  const float tot = wave_sum(rho_acc);
  if (lane == 0 && a.loss_out) a.loss_out[b] = __fdiv_rn(tot, (float)a.Np);
}

__global__ __launch_bounds__(64) void k_mean(const float* x, int n, float* out) {
  float s = 0.0f;
  for (int i = threadIdx.x; i < n; i += 64) s = __fadd_rn(s, x[i]);
  s = wave_sum(s);
  if (threadIdx.x == 0) out[0] = __fdiv_rn(s, (float)n);
}

// ---------------------------------------------------------------------------
// TF1 Adam (ApplyAdam): alpha = lr sqrt(1 - b2^t) / (1 - b1^t) from the float32
// beta powers, then m/v/var updates (float4 vectorised).
// ---------------------------------------------------------------------------
// The float32 beta powers are double-buffered: state = {b1p, b2p}[2]; a launch
// reads slot `slot` (this step's beta^t) and block 0 writes slot^1 = beta^(t+1)
// (TF's beta_power *= beta after the apply, adam.py _finish), so no separate
// "prepare" launch and no intra-launch race.
__device__ __forceinline__ float adam_alpha(const float* state, int slot, float lr, float b1,
                                            float b2) {
  if (blockIdx.x == 0 && threadIdx.x == 0) adam_bump(const_cast<float*>(state), slot, b1, b2);
  return adam_alpha_of(state, slot, lr);
}

__device__ __forceinline__ void adam_range(float* __restrict__ var, const float* __restrict__ grad,
                                           float* __restrict__ m, float* __restrict__ v,
                                           int64_t n, int64_t first4, int64_t stride4,
                                           float alpha, float omb1, float omb2, float eps) {
  const int64_t n4 = n >> 2;
  for (int64_t i = first4; i < n4; i += stride4) {
    float4 p = ((float4*)var)[i], g = ((const float4*)grad)[i];
    float4 mm = ((float4*)m)[i], vv = ((float4*)v)[i];
    adam1(p.x, g.x, mm.x, vv.x, alpha, omb1, omb2, eps);
    adam1(p.y, g.y, mm.y, vv.y, alpha, omb1, omb2, eps);
    adam1(p.z, g.z, mm.z, vv.z, alpha, omb1, omb2, eps);
    adam1(p.w, g.w, mm.w, vv.w, alpha, omb1, omb2, eps);
    ((float4*)var)[i] = p;
    ((float4*)m)[i] = mm;
    ((float4*)v)[i] = vv;
  }
  for (int64_t i = (n4 << 2) + first4; i < n; i += stride4)
    adam1(var[i], grad[i], m[i], v[i], alpha, omb1, omb2, eps);
}

// one part of a step split over several launches: only the part with bump != 0
// advances the beta powers (every part reads this step's slot)
__global__ __launch_bounds__(256) void k_adam_part(float* __restrict__ var,
                                                   const float* __restrict__ grad,
                                                   float* __restrict__ m, float* __restrict__ v,
                                                   float* state, int slot, int64_t n, float lr,
                                                   float b1, float b2, float eps, int bump) {
  if (bump && blockIdx.x == 0 && threadIdx.x == 0) adam_bump(state, slot, b1, b2);
  const float alpha = adam_alpha_of(state, slot, lr);
  const float omb1 = __fsub_rn(1.0f, b1), omb2 = __fsub_rn(1.0f, b2);
  adam_range(var, grad, m, v, n, (int64_t)blockIdx.x * blockDim.x + threadIdx.x,
             (int64_t)gridDim.x * blockDim.x, alpha, omb1, omb2, eps);
}

__global__ __launch_bounds__(256) void k_adam(float* __restrict__ var, const float* __restrict__ grad,
                                              float* __restrict__ m, float* __restrict__ v,
                                              float* state, int slot, int64_t n, float lr,
                                              float b1, float b2, float eps) {
  const float alpha = adam_alpha(state, slot, lr, b1, b2);
  const float omb1 = __fsub_rn(1.0f, b1), omb2 = __fsub_rn(1.0f, b2);
  adam_range(var, grad, m, v, n, (int64_t)blockIdx.x * blockDim.x + threadIdx.x,
             (int64_t)gridDim.x * blockDim.x, alpha, omb1, omb2, eps);
}

// Multi-tensor form: one launch over up to 16 separately allocated gradients
// (autograd's own grad tensors, no flat-gradient zeroing / accumulation).
struct AdamMulti {
  float* var[DQ_MAX_TENSORS];
  const float* grad[DQ_MAX_TENSORS];
  float* m[DQ_MAX_TENSORS];
  float* v[DQ_MAX_TENSORS];
  int64_t n[DQ_MAX_TENSORS];
  int32_t block_start[DQ_MAX_TENSORS + 1];
  int32_t count;
};

__global__ __launch_bounds__(256) void k_adam_multi(AdamMulti a, float* state, int slot, float lr,
                                                    float b1, float b2, float eps) {
  const float alpha = adam_alpha(state, slot, lr, b1, b2);
  const float omb1 = __fsub_rn(1.0f, b1), omb2 = __fsub_rn(1.0f, b2);
  int t = 0;
  while (t + 1 < a.count && (int)blockIdx.x >= a.block_start[t + 1]) ++t;
  const int64_t lb = blockIdx.x - a.block_start[t];
  const int64_t nb = a.block_start[t + 1] - a.block_start[t];
  adam_range(a.var[t], a.grad[t], a.m[t], a.v[t], a.n[t], lb * blockDim.x + threadIdx.x,
             nb * blockDim.x, alpha, omb1, omb2, eps);
}

__global__ __launch_bounds__(256) void k_rmsprop(float* var, const float* grad, float* ms, float* mg,
                                                 float* mom, int64_t n, float lr, float rho,
                                                 float mu, float eps, int centered) {
  const float omr = __fsub_rn(1.0f, rho);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    float p = var[i], s = ms[i], a = centered ? mg[i] : 0.0f, mo = mom[i];
    rms1(p, grad[i], s, a, mo, lr, omr, mu, eps, centered != 0);
    ms[i] = s;
    if (centered) mg[i] = a;
    mom[i] = mo;
    var[i] = p;
  }
}

static int elementwise_grid(int64_t n) {
  int64_t blocks = (n + 1023) / 1024;
  if (blocks < 1) blocks = 1;
  if (blocks > 2048) blocks = 2048;
  return (int)blocks;
}

}  // namespace dq

using namespace dq;

extern "C" {

int dq_c51_loss(const float* online_logits, const float* target_logits, const int32_t* actions,
                const float* rewards, const uint8_t* terminals, const float* probs,
                const float* support, int32_t batch, int32_t num_actions, int32_t num_atoms,
                float cumulative_gamma, float* grad_logits, float* loss_out,
                float* priorities_out, float* mean_loss_out, void* stream) {
  DQ_CHECK_ARG(online_logits && target_logits && actions && rewards && terminals && support &&
                   grad_logits,
               "null argument");
  DQ_CHECK_ARG(num_atoms >= 2 && num_atoms <= 64, "num_atoms must be in [2, 64]");
  DQ_CHECK_ARG(batch >= 1 && num_actions >= 1 && num_actions <= 256, "bad batch / num_actions");
  C51Args a{online_logits, target_logits, actions, rewards, terminals, probs, support,
            batch, num_actions, num_atoms, cumulative_gamma, grad_logits, loss_out,
            priorities_out, mean_loss_out};
  DQ_CHECK_ARG(!mean_loss_out || loss_out, "mean_loss_out needs loss_out");
  DQ_CHECK_ARG(num_actions <= 64, "num_actions must be <= 64");
  const int waves = num_actions < 16 ? num_actions : 16;
  const size_t shm = c51_lds(num_actions, num_atoms, 0, waves);
  auto kern = probs ? k_c51<LogitsDirect, kC51Probs> : k_c51<LogitsDirect, 0>;
  hipLaunchKernelGGL(kern, dim3(batch), dim3(64 * waves), shm, (hipStream_t)stream,
                     a, LogitsDirect{online_logits, num_actions * num_atoms},
                     LogitsDirect{target_logits, num_actions * num_atoms}, C51Extra{});
  DQ_CHECK_LAUNCH("k_c51");
  if (mean_loss_out) {
    hipLaunchKernelGGL(k_wmean, dim3(1), dim3(64), 0, (hipStream_t)stream, loss_out, probs, batch,
                       mean_loss_out);
    DQ_CHECK_LAUNCH("k_wmean");
  }
  return DQ_OK;
}

int dq_c51_loss_fused(const float* online_parts, const float* online_bias,
                      const float* target_parts, const float* target_bias, int32_t n_parts,
                      const int32_t* actions, const float* rewards, const uint8_t* terminals,
                      const float* probs, const float* support, int32_t batch,
                      int32_t num_actions, int32_t num_atoms, float cumulative_gamma,
                      float* grad_logits, float* loss_out, float* priorities_out,
                      const float* fc2_w, const float* h, float* dh, int32_t hidden,
                      float* online_logits_out, float* target_logits_out, void* stream) {
  DQ_CHECK_ARG(online_parts && online_bias && target_parts && target_bias && actions && rewards &&
                   terminals && support && grad_logits,
               "null argument");
  DQ_CHECK_ARG(n_parts >= 1 && n_parts <= 16, "n_parts must be in [1, 16]");
  DQ_CHECK_ARG(num_atoms >= 2 && num_atoms <= 64, "num_atoms must be in [2, 64]");
  DQ_CHECK_ARG(batch >= 1 && num_actions >= 1 && num_actions <= 256, "bad batch / num_actions");
  DQ_CHECK_ARG(!fc2_w || (h && dh && hidden >= 1), "d h needs h, dh and hidden");
  C51Args a{nullptr, nullptr, actions, rewards, terminals, probs, support, batch, num_actions,
            num_atoms, cumulative_gamma, grad_logits, loss_out, priorities_out, nullptr};
  const int NO = num_actions * num_atoms;
  const int64_t stride = (int64_t)batch * NO;
  DQ_CHECK_ARG(num_actions <= 64, "num_actions must be <= 64");
  const int waves = num_actions < 16 ? num_actions : 16;
  // d h split over S blocks per sample when the column slices stay whole 16-B chunks
  const int S = fc2_w && hidden % (4 * kC51Split) == 0 ? kC51Split : 1;
  const size_t shm = c51_lds(num_actions, num_atoms, fc2_w ? hidden / S : 0, waves);
  DQ_CHECK_ARG(shm <= 160 * 1024, "num_atoms * hidden exceeds the LDS");
  static void (*const kerns[8])(C51Args, LogitsParts, LogitsParts, C51Extra) = {
      k_c51<LogitsParts, 0>, k_c51<LogitsParts, 1>, k_c51<LogitsParts, 2>, k_c51<LogitsParts, 3>,
      k_c51<LogitsParts, 4>, k_c51<LogitsParts, 5>, k_c51<LogitsParts, 6>, k_c51<LogitsParts, 7>};
  const int f = (probs ? kC51Probs : 0) | (fc2_w ? kC51W2 : 0) |
                (online_logits_out || target_logits_out ? kC51LogitsOut : 0);
  hipLaunchKernelGGL(kerns[f], dim3(batch * S), dim3(64 * waves), shm, (hipStream_t)stream,
                     a, LogitsParts{online_parts, online_bias, stride, n_parts, NO},
                     LogitsParts{target_parts, target_bias, stride, n_parts, NO},
                     C51Extra{online_logits_out, target_logits_out, fc2_w, h, dh, hidden});
  DQ_CHECK_LAUNCH("k_c51 fused");
  return DQ_OK;
}

int dq_c51_loss_online(const float* online_parts, const float* online_bias, int32_t n_parts,
                       const float* target_m, const int32_t* actions, const float* probs,
                       int32_t batch, int32_t num_actions, int32_t num_atoms, float* grad_logits,
                       float* loss_out, float* priorities_out, const float* fc2_w, const float* h,
                       float* dh, int32_t hidden, float* online_logits_out, void* stream) {
  DQ_CHECK_ARG(online_parts && online_bias && target_m && actions && grad_logits, "null argument");
  DQ_CHECK_ARG(n_parts >= 1 && n_parts <= 16, "n_parts must be in [1, 16]");
  DQ_CHECK_ARG(num_atoms >= 2 && num_atoms <= 64, "num_atoms must be in [2, 64]");
  DQ_CHECK_ARG(batch >= 1 && num_actions >= 1 && num_actions <= 64, "bad batch / num_actions");
  DQ_CHECK_ARG(!fc2_w || (h && dh && hidden >= 1), "d h needs h, dh and hidden");
  C51Args a{nullptr, nullptr, actions, nullptr, nullptr, probs, nullptr, batch, num_actions,
            num_atoms, 0.0f, grad_logits, loss_out, priorities_out, nullptr};
  const int NO = num_actions * num_atoms;
  const size_t shm = (size_t)(num_atoms + 3) / 4 * 4 * sizeof(float) +
                     (fc2_w ? c51_w2_lds_bytes(num_atoms, hidden) : 0);
  DQ_CHECK_ARG(shm <= 160 * 1024, "num_atoms * hidden exceeds the LDS");
  hipLaunchKernelGGL(k_c51_online<LogitsParts>, dim3(batch), dim3(512), shm, (hipStream_t)stream, a,
                     LogitsParts{online_parts, online_bias, (int64_t)batch * NO, n_parts, NO},
                     target_m, C51Extra{online_logits_out, nullptr, fc2_w, h, dh, hidden});
  DQ_CHECK_LAUNCH("k_c51_online");
  return DQ_OK;
}

int dq_dqn_huber_loss(const float* online_q, const float* target_q, const int32_t* actions,
                      const float* rewards, const uint8_t* terminals, int32_t batch,
                      int32_t num_actions, float cumulative_gamma, float* grad_q,
                      float* loss_out, float* mean_loss_out, void* stream) {
  DQ_CHECK_ARG(online_q && target_q && actions && rewards && terminals && grad_q, "null argument");
  DQ_CHECK_ARG(batch >= 1 && num_actions >= 1, "bad sizes");
  hipLaunchKernelGGL(k_dqn, dim3(1), dim3(256), 0, (hipStream_t)stream, online_q, target_q,
                     actions, rewards, terminals, batch, num_actions, cumulative_gamma, grad_q,
                     loss_out, mean_loss_out);
  DQ_CHECK_LAUNCH("k_dqn");
  return DQ_OK;
}

int dq_dqn_huber_loss_fused(const float* online_parts, const float* online_bias,
                            const float* target_parts, const float* target_bias, int32_t n_parts,
                            const int32_t* actions, const float* rewards,
                            const uint8_t* terminals, int32_t batch, int32_t num_actions,
                            float cumulative_gamma, float* grad_q, float* loss_out,
                            const float* fc2_w, const float* h, float* dh, int32_t hidden,
                            float* online_q_out, float* target_q_out, void* stream) {
  DQ_CHECK_ARG(online_parts && online_bias && target_parts && target_bias && actions && rewards &&
                   terminals && grad_q && fc2_w && h && dh,
               "null argument");
  DQ_CHECK_ARG(n_parts >= 1 && n_parts <= 16, "n_parts must be in [1, 16]");
  DQ_CHECK_ARG(batch >= 1 && num_actions >= 1 && num_actions <= 64, "bad batch / num_actions");
  DQ_CHECK_ARG(hidden >= 4 && hidden <= 512 && hidden % 4 == 0, "hidden must be a multiple of 4 <= 512");
  const int64_t stride = (int64_t)batch * num_actions;
  DqnFusedArgs a{LogitsParts{online_parts, online_bias, stride, n_parts, num_actions},
                 LogitsParts{target_parts, target_bias, stride, n_parts, num_actions},
                 actions, rewards, terminals, batch, num_actions, hidden, cumulative_gamma,
                 grad_q, loss_out, fc2_w, h, dh, online_q_out, target_q_out};
  hipLaunchKernelGGL(k_dqn_fused, dim3(batch), dim3(128), 0, (hipStream_t)stream, a);
  DQ_CHECK_LAUNCH("k_dqn_fused");
  return DQ_OK;
}

int dq_iqn_loss(const float* online_qv, const float* target_qv, const float* target_qv_action,
                const float* taus, const int32_t* actions, const float* rewards,
                const uint8_t* terminals, int32_t batch, int32_t num_actions,
                int32_t num_tau, int32_t num_tau_prime, int32_t num_quantile,
                float cumulative_gamma, float kappa, float* grad_qv, float* loss_out,
                float* mean_loss_out, void* stream) {
  DQ_CHECK_ARG(online_qv && target_qv && target_qv_action && taus && actions && rewards &&
                   terminals && grad_qv && loss_out,
               "null argument (loss_out is required)");
  DQ_CHECK_ARG(batch >= 1 && num_actions >= 1 && num_tau >= 1 && num_tau_prime >= 1 &&
                   num_quantile >= 1 && kappa > 0.0f,
               "bad sizes");
  IqnArgs a{online_qv, target_qv, target_qv_action, taus, actions, rewards, terminals,
            batch, num_actions, num_tau, num_tau_prime, num_quantile, cumulative_gamma, kappa,
            grad_qv, loss_out};
  hipLaunchKernelGGL(k_iqn, dim3(batch), dim3(64), sizeof(float) * num_tau_prime,
                     (hipStream_t)stream, a);
  DQ_CHECK_LAUNCH("k_iqn");
  if (mean_loss_out) {
    hipLaunchKernelGGL(k_mean, dim3(1), dim3(64), 0, (hipStream_t)stream, loss_out, batch,
                       mean_loss_out);
    DQ_CHECK_LAUNCH("k_mean");
  }
  return DQ_OK;
}

int dq_adam_tf1(float* var, const float* grad, float* m, float* v, float* state, int32_t slot,
                int64_t n, float lr, float beta1, float beta2, float eps, void* stream) {
  DQ_CHECK_ARG(var && grad && m && v && state && n >= 0 && (slot == 0 || slot == 1), "bad arguments");
  DQ_CHECK_ARG(((uintptr_t)var | (uintptr_t)grad | (uintptr_t)m | (uintptr_t)v) % 16 == 0,
               "adam buffers must be 16-byte aligned");
  hipLaunchKernelGGL(k_adam, dim3(elementwise_grid(n)), dim3(256), 0, (hipStream_t)stream, var,
                     grad, m, v, state, slot, n, lr, beta1, beta2, eps);
  DQ_CHECK_LAUNCH("k_adam");
  return DQ_OK;
}

int dq_adam_tf1_part(float* var, const float* grad, float* m, float* v, float* state,
                     int32_t slot, int64_t n, float lr, float beta1, float beta2, float eps,
                     int32_t bump, void* stream) {
  DQ_CHECK_ARG(var && grad && m && v && state && n >= 0 && (slot == 0 || slot == 1), "bad arguments");
  DQ_CHECK_ARG(((uintptr_t)var | (uintptr_t)grad | (uintptr_t)m | (uintptr_t)v) % 16 == 0,
               "adam buffers must be 16-byte aligned");
  constexpr int kMaxBlocks = 256;   // N > 1's fc update beside the main queue: a cap leaves it CUs
  hipLaunchKernelGGL(k_adam_part, dim3(std::min(elementwise_grid(n), kMaxBlocks)), dim3(256), 0,
                     (hipStream_t)stream,
                     var, grad, m, v, state, slot, n, lr, beta1, beta2, eps, bump);
  DQ_CHECK_LAUNCH("k_adam_part");
  return DQ_OK;
}

int dq_adam_tf1_multi(const dq_tensor_list* t, float* state, int32_t slot, float lr, float beta1,
                      float beta2, float eps, void* stream) {
  DQ_CHECK_ARG(t && state && (slot == 0 || slot == 1), "bad arguments");
  DQ_CHECK_ARG(t->count >= 1 && t->count <= DQ_MAX_TENSORS, "1..16 tensors");
  AdamMulti a;
  a.count = t->count;
  int32_t blocks = 0;
  for (int i = 0; i < t->count; ++i) {
    DQ_CHECK_ARG(t->var[i] && t->grad[i] && t->m[i] && t->v[i] && t->n[i] > 0, "null tensor");
    DQ_CHECK_ARG(((uintptr_t)t->var[i] | (uintptr_t)t->grad[i] | (uintptr_t)t->m[i] |
                  (uintptr_t)t->v[i]) % 16 == 0, "adam tensors must be 16-byte aligned");
    a.var[i] = t->var[i];
    a.grad[i] = t->grad[i];
    a.m[i] = t->m[i];
    a.v[i] = t->v[i];
    a.n[i] = t->n[i];
    a.block_start[i] = blocks;
    int64_t nb = (t->n[i] + 4095) / 4096;   // 16 floats per thread per block pass
    if (nb > 512) nb = 512;
    blocks += (int32_t)nb;
  }
  a.block_start[t->count] = blocks;
  hipLaunchKernelGGL(k_adam_multi, dim3(blocks), dim3(256), 0, (hipStream_t)stream, a, state,
                     slot, lr, beta1, beta2, eps);
  DQ_CHECK_LAUNCH("k_adam_multi");
  return DQ_OK;
}

int dq_rmsprop_tf1(float* var, const float* grad, float* ms, float* mg, float* mom, int64_t n,
                   float lr, float decay, float momentum, float eps, int32_t centered,
                   void* stream) {
  DQ_CHECK_ARG(var && grad && ms && mom && (mg || !centered) && n >= 0, "bad arguments");
  if (n == 0) return DQ_OK;
  hipLaunchKernelGGL(k_rmsprop, dim3(elementwise_grid(n)), dim3(256), 0, (hipStream_t)stream, var,
                     grad, ms, mg, mom, n, lr, decay, momentum, eps, centered);
  DQ_CHECK_LAUNCH("k_rmsprop");
  return DQ_OK;
}

}  // extern "C"
