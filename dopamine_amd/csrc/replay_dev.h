// Device bodies of the replay kernels, shared by replay.hip (their own launches)
// and nature_cnn.hip (the same code riding as extra blocks in the backward's
// grouped launches, see RiderOp).  Restates the reference's numpy code:
// circular_replay_buffer.py:381-555, prioritized_replay_buffer.py:152-170,
// sum_tree.py:128-139 and :178-205.
//
// Numerics: every float64 step of the sampler (stratum edges, uniform(), the
// q * total scaling, the descent's compare/subtract) and the float32 n-step
// reward are written with explicit _rn intrinsics and compiled with
// -ffp-contract=off, so results are bit-identical to the reference.
#pragma once
#include "common.h"

namespace dq {

struct ReplayView {
  int64_t C;
  int64_t obs_bytes;
  int32_t S;
  int32_t n;
  int32_t depth;
  int32_t max_attempts;
  const uint8_t* frames;
  const int32_t* actions;
  const float* rewards;
  const uint8_t* terminals;
  double* tree;
  dq_replay_meta* meta;
  const uint32_t* tape;
  const float* discount;
};

__device__ __forceinline__ void latch(dq_replay_meta* m, int code, int arg, double val) {
  if (atomicCAS(&m->status, 0, code) == 0) {
    m->status_arg = arg;
    m->status_value = val;
  }
}

// Python's random.random(): genrand_res53 from two consecutive 32-bit words.
__device__ __forceinline__ double res53(uint32_t w0, uint32_t w1) {
  const double a = (double)(w0 >> 5), b = (double)(w1 >> 6);
  return __dmul_rn(__dadd_rn(__dmul_rn(a, 67108864.0), b), 1.0 / 9007199254740992.0);
}

// SumTree.sample descent (sum_tree.py:128-139) on the flat heap; q already
// scaled by the root total.
__device__ __forceinline__ int64_t descend(const double* tree, int depth, double q) {
  int64_t node = 0;
  for (int d = 1; d <= depth; ++d) {
    const double left = tree[((int64_t)1 << d) - 1 + 2 * node];
    if (q < left) {
      node = 2 * node;
    } else {
      node = 2 * node + 1;
      q = __dsub_rn(q, left);
    }
  }
  return node;
}

// OutOfGraphReplayBuffer.is_valid_transition (circular_replay_buffer.py:381-414).
__device__ inline bool is_valid(const ReplayView& v, int64_t idx, int64_t add_count) {
  if (idx < 0 || idx >= v.C) return false;
  const int64_t cursor = add_count % v.C;
  if (add_count < v.C) {
    if (idx >= cursor - v.n) return false;
    if (idx < v.S - 1) return false;
  }
  // invalid_range(cursor) = {(cursor - n + k) mod C : 0 <= k < n + S}
  if (pymod(idx - (cursor - v.n), v.C) < (int64_t)(v.n + v.S)) return false;
  // a terminal in any but the last frame of the stack
  for (int k = 0; k < v.S - 1; ++k)
    if (v.terminals[pymod(idx - v.S + 1 + k, v.C)]) return false;
  return true;
}

// trajectory length L (circular_replay_buffer.py:517-526).
__device__ __forceinline__ int traj_len(const ReplayView& v, int64_t idx, bool* term) {
  for (int j = 0; j < v.n; ++j) {
    if (v.terminals[pymod(idx + j, v.C)]) {
      *term = true;
      return j + 1;
    }
  }
  *term = false;
  return v.n;
}

constexpr int kMaxBatch = 1024;

// ---------------------------------------------------------------------------
// Prioritized index sampling: stratified descent (one lane per stratum), then
// the reference's sequential retry loop (prioritized_replay_buffer.py:152-170).
// One wave (threads 0..63 of the block; any others have returned).
// ---------------------------------------------------------------------------
constexpr int kPerSampleLds = kMaxBatch * 8 + kMaxBatch;   // bytes

__device__ inline void per_sample_body(const ReplayView& v, int B, int32_t* out, void* lds) {
  int64_t* s_idx = (int64_t*)lds;
  uint8_t* s_ok = (uint8_t*)(s_idx + kMaxBatch);
  const int lane = threadIdx.x;
  dq_replay_meta* meta = v.meta;
  const int64_t add_count = meta->add_count;
  int64_t pos = meta->tape_pos;
  const int64_t pos0 = pos;
  const int64_t len = meta->tape_len;
  const double total = v.tree[0];
  bool fail = meta->status != 0;
  if (!fail && total == 0.0) {
    if (lane == 0) latch(meta, DQ_ST_EMPTY_TREE, 0, 0.0);
    fail = true;
  }
  if (!fail && pos + 2 * (int64_t)B > len) {
    if (lane == 0) latch(meta, DQ_ST_TAPE_EXHAUSTED, 0, 0.0);
    fail = true;
  }
  if (fail) {
    if (lane == 0) meta->reserved[0] = pos0;
    for (int i = lane; i < B; i += kWave) out[i] = 0;
    return;
  }
  // np.linspace(0, 1, B + 1): edge_i = i * (1/B), last edge exactly 1.0
  const double step = 1.0 / (double)B;
  for (int i = lane; i < B; i += kWave) {
    const double u = res53(v.tape[pos + 2 * i], v.tape[pos + 2 * i + 1]);
    const double lo = __dmul_rn((double)i, step);
    const double hi = (i + 1 == B) ? 1.0 : __dmul_rn((double)(i + 1), step);
    const double q = __dadd_rn(lo, __dmul_rn(__dsub_rn(hi, lo), u));  // random.uniform
    const int64_t node = descend(v.tree, v.depth, __dmul_rn(q, total));
    s_idx[i] = node;
    s_ok[i] = is_valid(v, node, add_count);
  }
  pos += 2 * (int64_t)B;
  __syncthreads();
  if (lane == 0) {
    int budget = v.max_attempts;
    for (int i = 0; i < B; ++i) {
      if (s_ok[i]) continue;
      if (budget == 0) {
        latch(meta, DQ_ST_MAX_ATTEMPTS, i, 0.0);
        break;
      }
      int64_t cand = s_idx[i];
      bool tape_dry = false;
      while (budget > 0) {
        if (pos + 2 > len) {
          tape_dry = true;
          break;
        }
        const double u = res53(v.tape[pos], v.tape[pos + 1]);
        pos += 2;
        cand = descend(v.tree, v.depth, __dmul_rn(u, total));
        --budget;
        if (is_valid(v, cand, add_count)) break;
      }
      s_idx[i] = cand;
      if (tape_dry) {
        latch(meta, DQ_ST_TAPE_EXHAUSTED, i, 0.0);
        break;
      }
    }
    meta->reserved[0] = pos0;   // entry cursor, for dq_replay_rewind_last_sample
    meta->tape_pos = pos;
  }
  __syncthreads();
  for (int i = lane; i < B; i += kWave) out[i] = (int32_t)s_idx[i];
}

// ---------------------------------------------------------------------------
// Uniform index sampling (circular_replay_buffer.py:449-477).  numpy legacy
// randint(min_id, max_id) = min_id + masked-rejection draw of 32-bit words.
// The draw/validate chain is evaluated 64 words at a time speculatively; a
// ballot/prefix-count finds where the reference's loop would have stopped.
// ---------------------------------------------------------------------------
__device__ inline void uniform_sample_body(const ReplayView& v, int B, int32_t* out) {
  const int lane = threadIdx.x;
  dq_replay_meta* meta = v.meta;
  int64_t pos = meta->tape_pos;
  const int64_t pos0 = pos;
  if (meta->status != 0) {
    if (lane == 0) meta->reserved[0] = pos0;
    for (int i = lane; i < B; i += kWave) out[i] = 0;
    return;
  }
  const int64_t add_count = meta->add_count;
  const int64_t cursor = add_count % v.C;
  int64_t min_id, max_id;
  if (add_count >= v.C) {
    min_id = cursor - v.C + v.S - 1;
    max_id = cursor - v.n;
  } else {
    min_id = v.S - 1;
    max_id = cursor - v.n;
    if (max_id <= min_id) {
      if (lane == 0) {
        latch(meta, DQ_ST_TOO_FEW, 0, 0.0);
        meta->reserved[0] = pos0;
      }
      for (int i = lane; i < B; i += kWave) out[i] = 0;
      return;
    }
  }
  const uint64_t rng = (uint64_t)(max_id - min_id - 1);
  uint64_t mask = rng;
  mask |= mask >> 1; mask |= mask >> 2; mask |= mask >> 4;
  mask |= mask >> 8; mask |= mask >> 16; mask |= mask >> 32;
  const int64_t len = meta->tape_len;
  int count = 0, fails = 0;
  bool tape_dry = false;
  if (rng == 0) {  // randint consumes no word when high - low == 1
    const int64_t idx = pymod(min_id, v.C);
    const bool ok = is_valid(v, idx, add_count);
    if (ok) {
      for (int i = lane; i < B; i += kWave) out[i] = (int32_t)idx;
      count = B;
    } else {
      fails = v.max_attempts;
    }
  } else {
    const uint64_t below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    while (count < B && fails < v.max_attempts) {
      const int64_t avail = len - pos;
      if (avail <= 0) { tape_dry = true; break; }
      const bool live = lane < avail;
      const uint64_t w = live ? (uint64_t)v.tape[pos + lane] : 0ull;
      const uint64_t val = w & mask;
      const bool drawn = live && val <= rng;
      const int64_t idx = pymod(min_id + (int64_t)val, v.C);
      const bool ok = drawn && is_valid(v, idx, add_count);
      const bool bad = drawn && !ok;
      const uint64_t okm = __ballot(ok), badm = __ballot(bad);
      const int cok = count + __popcll(okm & below) + (ok ? 1 : 0);
      const int cbad = fails + __popcll(badm & below) + (bad ? 1 : 0);
      const bool stop = (ok && cok == B) || (bad && cbad == v.max_attempts);
      const uint64_t stopm = __ballot(stop);
      if (stopm) {
        const int s = __ffsll((unsigned long long)stopm) - 1;
        if (ok && lane <= s) out[cok - 1] = (int32_t)idx;
        count = __shfl(cok, s);
        fails = __shfl(cbad, s);
        pos += s + 1;
        break;
      }
      if (ok) out[cok - 1] = (int32_t)idx;
      count += __popcll(okm);
      fails += __popcll(badm);
      const int64_t used = avail < kWave ? avail : kWave;
      pos += used;
      if (used < kWave) { tape_dry = true; break; }
    }
  }
  if (lane == 0) {
    if (tape_dry) latch(meta, DQ_ST_TAPE_EXHAUSTED, count, 0.0);
    else if (count != B) latch(meta, DQ_ST_MAX_ATTEMPTS, count, 0.0);
    meta->reserved[0] = pos0;   // entry cursor, for dq_replay_rewind_last_sample
    meta->tape_pos = pos;
  }
}

// G > 1 consecutive batches of B (the draws of G sample_index_batch(B) calls in a row, each with
// its own max-attempts budget and its own error) into out[g * B + i]: the learner-only loop
// draws a whole chunk's uniform batches at once (they do not depend on priorities).  The
// rewind cursor (meta->reserved[0]) is the entry of the LAST batch, so
// dq_replay_rewind_last_sample gives back exactly the one batch a prefetch holds.  Riders run
// inside the CNN's grouped launches, whose GEMM tiles are held to 64 VGPRs: only the launches
// that carry a grouped sample instantiate this loop (run_rider<T, true>).
__device__ inline void uniform_sample_groups(const ReplayView& v, int B, int32_t* out, int G) {
  const int lane = threadIdx.x;
  dq_replay_meta* meta = v.meta;
  int64_t pos = meta->tape_pos;
  int64_t entry = pos;
  if (meta->status != 0) {
    if (lane == 0) meta->reserved[0] = entry;
    for (int i = lane; i < G * B; i += kWave) out[i] = 0;
    return;
  }
  const int64_t add_count = meta->add_count;
  const int64_t cursor = add_count % v.C;
  int64_t min_id, max_id;
  if (add_count >= v.C) {
    min_id = cursor - v.C + v.S - 1;
    max_id = cursor - v.n;
  } else {
    min_id = v.S - 1;
    max_id = cursor - v.n;
    if (max_id <= min_id) {
      if (lane == 0) {
        latch(meta, DQ_ST_TOO_FEW, 0, 0.0);
        meta->reserved[0] = entry;
      }
      for (int i = lane; i < G * B; i += kWave) out[i] = 0;
      return;
    }
  }
  const uint64_t rng = (uint64_t)(max_id - min_id - 1);
  uint64_t mask = rng;
  mask |= mask >> 1; mask |= mask >> 2; mask |= mask >> 4;
  mask |= mask >> 8; mask |= mask >> 16; mask |= mask >> 32;
  const int64_t len = meta->tape_len;
  const uint64_t below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  for (int g = 0; g < G; ++g) {
    int32_t* o = out + (int64_t)g * B;
    entry = pos;
    int count = 0, fails = 0;
    bool tape_dry = false;
    if (rng == 0) {  // randint consumes no word when high - low == 1
      const int64_t idx = pymod(min_id, v.C);
      const bool ok = is_valid(v, idx, add_count);
      if (ok) {
        for (int i = lane; i < B; i += kWave) o[i] = (int32_t)idx;
        count = B;
      } else {
        fails = v.max_attempts;
      }
    } else {
      while (count < B && fails < v.max_attempts) {
        const int64_t avail = len - pos;
        if (avail <= 0) { tape_dry = true; break; }
        const bool live = lane < avail;
        const uint64_t w = live ? (uint64_t)v.tape[pos + lane] : 0ull;
        const uint64_t val = w & mask;
        const bool drawn = live && val <= rng;
        const int64_t idx = pymod(min_id + (int64_t)val, v.C);
        const bool ok = drawn && is_valid(v, idx, add_count);
        const bool bad = drawn && !ok;
        const uint64_t okm = __ballot(ok), badm = __ballot(bad);
        const int cok = count + __popcll(okm & below) + (ok ? 1 : 0);
        const int cbad = fails + __popcll(badm & below) + (bad ? 1 : 0);
        const bool stop = (ok && cok == B) || (bad && cbad == v.max_attempts);
        const uint64_t stopm = __ballot(stop);
        if (stopm) {
          const int s = __ffsll((unsigned long long)stopm) - 1;
          if (ok && lane <= s) o[cok - 1] = (int32_t)idx;
          count = __shfl(cok, s);
          fails = __shfl(cbad, s);
          pos += s + 1;
          break;
        }
        if (ok) o[cok - 1] = (int32_t)idx;
        count += __popcll(okm);
        fails += __popcll(badm);
        const int64_t used = avail < kWave ? avail : kWave;
        pos += used;
        if (used < kWave) { tape_dry = true; break; }
      }
    }
    if (tape_dry || count != B) {      // this batch's error, as its own call would raise it
      if (lane == 0) latch(meta, tape_dry ? DQ_ST_TAPE_EXHAUSTED : DQ_ST_MAX_ATTEMPTS, count, 0.0);
      for (int i = lane + (g + 1) * B; i < G * B; i += kWave) out[i] = 0;
      break;
    }
  }
  if (lane == 0) {
    meta->reserved[0] = entry;   // the last batch's entry cursor, for dq_replay_rewind_last_sample
    meta->tape_pos = pos;
  }
}

// ---------------------------------------------------------------------------
// Frame-stack gather.  grid.y = (sample b, state|next_state, stack slot k);
// each block copies one 84x84 frame (contiguous obs_bytes) of the stack.  Frames
// are independent contiguous blocks, so the store is fully coalesced and the
// stacking axis becomes the channel axis (NCHW) for free.
// ---------------------------------------------------------------------------
struct GatherOut {
  const int32_t* indices;
  void* state;
  void* next_state;
  int32_t* action;
  float* reward;
  int32_t* next_action;
  float* next_reward;
  uint8_t* terminal;
  int32_t* indices_out;
  float* probs;
};

// n-step trajectory length with every terminal byte of the trajectory loaded up
// front (independent loads, no serial early exit).  Same result as traj_len.
__device__ __forceinline__ int traj_len_par(const ReplayView& v, int64_t idx, bool* term) {
  for (int j0 = 0; j0 < v.n; j0 += 8) {
    uint8_t t[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) t[q] = (j0 + q < v.n) ? v.terminals[pymod(idx + j0 + q, v.C)] : 0;
    int first = -1;
#pragma unroll
    for (int q = 7; q >= 0; --q)
      if (t[q]) first = q;
    if (first >= 0) {
      *term = true;
      return j0 + first + 1;
    }
  }
  *term = false;
  return v.n;
}

__device__ __forceinline__ int64_t stack_base(const ReplayView& v, const GatherOut& g, int b,
                                              int which) {
  int64_t base = pymod((int64_t)g.indices[b], v.C);
  if (which) {
    bool term;
    base = pymod(base + traj_len_par(v, base, &term), v.C);
  }
  return base;
}

// Per-sample scalars (crb:517-555), one wave: lanes load the trajectory's
// terminal/reward bytes in parallel, the ballot finds L, lane 0 sums the
// float32 products left to right exactly as numpy's n < 8 reduction does.
// Loads that need L (next_action/next_reward at idx + L) are issued for the
// usual L = n together with the trajectory and re-read only when a terminal
// cuts it short, so the wave waits on two dependent loads (index, then
// everything else), not three.
__device__ inline void write_scalars_wave(const ReplayView& v, const GatherOut& g, int b,
                                          int64_t idx) {
  const int lane = threadIdx.x & 63;
  float p = 0.0f;
  bool t = false;
  // independent of L: issued with the trajectory
  const int64_t nspec = pymod(idx + v.n, v.C);
  int32_t a0 = 0, na = 0;
  float nr = 0.0f, pr = 0.0f;
  if (lane == 0) {
    a0 = v.actions[idx];
    na = v.actions[nspec];
    nr = v.rewards[nspec];
    if (g.probs) pr = (float)v.tree[((int64_t)1 << v.depth) - 1 + idx];
  }
  if (lane < v.n) {
    const int64_t j = pymod(idx + lane, v.C);
    t = v.terminals[j] != 0;
    p = __fmul_rn(v.discount[lane], v.rewards[j]);
  }
  // trajectories longer than a wave are finished by lane 0 below (n > 64 is unheard of)
  const uint64_t tm = __ballot(t);
  int L = v.n;
  bool term = false;
  if (tm) {
    L = __ffsll((unsigned long long)tm);
    term = true;
  }
  float acc = 0.0f;
  for (int k = 0; k < L && k < kWave; ++k) acc = __fadd_rn(acc, __shfl(p, k));
  if (lane == 0) {
    if (v.n > kWave) {  // generic tail, serial
      bool tt;
      L = traj_len(v, idx, &tt);
      term = tt;
      acc = 0.0f;
      for (int k = 0; k < L; ++k)
        acc = __fadd_rn(acc, __fmul_rn(v.discount[k], v.rewards[pymod(idx + k, v.C)]));
    }
    if (L != v.n) {     // a terminal ended the trajectory early: the loads at idx + L
      const int64_t nxt = pymod(idx + L, v.C);
      na = v.actions[nxt];
      nr = v.rewards[nxt];
    }
    if (g.action) g.action[b] = a0;
    if (g.reward) g.reward[b] = acc;
    if (g.next_action) g.next_action[b] = na;
    if (g.next_reward) g.next_reward[b] = nr;
    if (g.terminal) g.terminal[b] = term ? 1 : 0;
    if (g.indices_out) g.indices_out[b] = (int32_t)idx;
    if (g.probs) g.probs[b] = pr;
  }
}

// tf.div(tf.cast(x, f32), 255.) for a byte x, correctly rounded: q = x * fl(1/255)
// is off by one ulp for 126 of the 256 bytes; one Newton residual step
// r = fma(-q, 255, x), q + r * fl(1/255) (fused) restores the correctly rounded
// quotient for every byte (checked exhaustively against x / 255.f, and against
// the oracle by the gather parity tests) -- 3 VALU ops instead of the IEEE
// division sequence (div_scale/rcp/fma chain/div_fixup).
__device__ __forceinline__ float u8_unit(uint32_t x) {
  constexpr float kInv = 1.0f / 255.0f;
  const float xf = (float)x;
  const float q = __fmul_rn(xf, kInv);
  return __builtin_fmaf(__builtin_fmaf(-q, 255.0f, xf), kInv, q);
}

typedef uint32_t gather_u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float4 u8x4_to_f32_255(uint32_t w) {
  float4 o;
  o.x = u8_unit(w & 0xffu);
  o.y = u8_unit((w >> 8) & 0xffu);
  o.z = u8_unit((w >> 16) & 0xffu);
  o.w = u8_unit(w >> 24);
  return o;
}

// NHWC float32 (the reference's state layout (B, H, W, stack), stack == 4): one
// block column per (b, which) stack; each wave takes R chunks of 64 dwords (256
// pixels) of each of the 4 frames -- all 4R loads in flight together -- and
// writes 4 pixels x 4 channels = 64 contiguous bytes per lane per store.
// (bx, slot) = the block's coordinates in the (column blocks, 2B) grid; tid in [0, 256).
// kScalars: where the per-sample scalars are written --
//   kScalEarly: by the first wave of the sample's state column, before its frame loads
//               (the riders: the late form's live frame registers raise the grouped
//               launch's VGPR count, -1% per learner step, measured);
//   kScalLate:  by that wave after issuing its frame loads;
//   kScalNone:  not here (the standalone kernel gives them a block column of their own,
//               so no frame wave waits on the scalar chain: 5.58 -> 5.20 us at B = 32
//               with kNt, tools/micro/gather_nhwc.hip).
// kNt: non-temporal float4 stores (the line stays in L2; 5.58 -> 5.42 us alone).
enum { kScalEarly = 0, kScalLate = 1, kScalNone = 2 };

#ifdef DQ_GATHER_PROF
// Stamp build of the standalone gather (tools/gather_stamps.py; never the product: the
// waits below serialise what the product overlaps only where a stamp is taken).  Each wave
// takes s_memrealtime (100 MHz) at its start, once its index is in, once its frames are in,
// and once its stores are acknowledged, and writes the four to its own slot of a ring of
// kGpRing launches (the slot from a counter only that wave position reads and advances: no
// atomics, no shared words).  Stamp words only ever go to these buffers.
constexpr int kGpRing = 64, kGpWaves = 2048;
__device__ unsigned long long g_gp_wave[kGpRing][kGpWaves][4];
__device__ unsigned int g_gp_seq[kGpWaves];
#define GP_STAMP(gp, k)                                      \
  do {                                                       \
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");         \
    (gp)[k] = __builtin_amdgcn_s_memrealtime();              \
  } while (0)
#else
#define GP_STAMP(gp, k) do { } while (0)
#endif

template <int R, int kScalars = kScalEarly, bool kNt = false>
__device__ __forceinline__ void gather_nhwc4_body(const ReplayView& v, const GatherOut& g, int bx,
                                                  int slot, int tid,
                                                  unsigned long long* gp = nullptr) {
  constexpr bool kLateScalars = kScalars == kScalLate;
  const int b = slot >> 1, which = slot & 1;
  const bool scal = kScalars != kScalNone && bx == 0 && which == 0 && tid < 64;
  if (!kLateScalars && scal) write_scalars_wave(v, g, b, pymod((int64_t)g.indices[b], v.C));
  float* dst_base = (float*)(which ? g.next_state : g.state);
  const int64_t nd = v.obs_bytes >> 2;
  const int lane = tid & 63;
  // this wave's R x 64 dwords of each of the 4 frames
  const int64_t w0 = ((int64_t)bx * 256 + (tid & ~63)) * R;
  if (!dst_base || w0 >= nd) {
    if (kLateScalars && scal) write_scalars_wave(v, g, b, pymod((int64_t)g.indices[b], v.C));
    return;
  }
  // next_state's stack ends at idx + L (L = n-step length, crb:517-531).  Its
  // frames are loaded for the usual L = n together with the trajectory's
  // terminal bytes and re-loaded only when a terminal makes L < n (wave-uniform
  // branch), so frames wait on the index alone: two dependent cold loads, not three.
  const int64_t idx = pymod((int64_t)g.indices[b], v.C);
  if (gp) GP_STAMP(gp, 1);
  uint32_t w[R][4];
  auto load = [&](int64_t base) {
    const uint32_t* fr[4];
#pragma unroll
    for (int k = 0; k < 4; ++k)
      fr[k] = (const uint32_t*)(v.frames + pymod(base - 3 + k, v.C) * v.obs_bytes);
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int64_t d = w0 + 64 * r + lane;
#pragma unroll
      for (int k = 0; k < 4; ++k) w[r][k] = d < nd ? fr[k][d] : 0u;
    }
  };
  if (which) {
    const int64_t spec = pymod(idx + v.n, v.C);
    load(spec);
    bool term;
    const int64_t base = pymod(idx + traj_len_par(v, idx, &term), v.C);
    if (base != spec) load(base);
  } else {
    load(idx);
    if (kLateScalars && scal) write_scalars_wave(v, g, b, idx);
  }
  if (gp) GP_STAMP(gp, 2);
  // store j of chunk r: lane l writes pixel 64j + l of the chunk (its 4 channels =
  // 16 B), so every store instruction covers 1 KiB contiguous; the bytes come from
  // lane 16j + l/4.
  const int sh = 8 * (lane & 3);
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int64_t d0 = w0 + 64 * r;
    float4* dst = (float4*)(dst_base + (int64_t)b * 4 * v.obs_bytes) + 4 * d0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int src = 16 * j + (lane >> 2);
      float4 o;
      o.x = u8_unit((__shfl(w[r][0], src) >> sh) & 0xffu);
      o.y = u8_unit((__shfl(w[r][1], src) >> sh) & 0xffu);
      o.z = u8_unit((__shfl(w[r][2], src) >> sh) & 0xffu);
      o.w = u8_unit((__shfl(w[r][3], src) >> sh) & 0xffu);
      if (4 * d0 + 64 * j + lane < 4 * nd) {
        if constexpr (kNt)   // buffer store, cache policy nt (aux = 2); dst is wave-uniform
          __builtin_amdgcn_raw_buffer_store_b128(
              *(const gather_u32x4*)&o, __builtin_amdgcn_make_buffer_rsrc(dst, 0, 0x7fffffff, 0x00020000),
              (64 * j + lane) * 16, 0, 2);
        else
          dst[64 * j + lane] = o;
      }
    }
  }
}

// R = 1: measured fastest at B = 32 (R = 2 / 4: 5.3 / 6.7 us vs 5.1 us per launch)
constexpr int kNhwcR = 1;

// ---------------------------------------------------------------------------
// Sum-tree ordered batch update (sum_tree.py:178-205 called in order by
// prioritized_replay_buffer.py:213-214 or :139).  One wave; lane L owns tree
// level L.  For each update i (in order) the leaf lane computes
// delta_i = value_i - leaf, every level adds delta_i to its node, and the new
// value is forwarded (through LDS) to the next update hitting the same node, so
// each node receives exactly the reference's ordered chain of float64 adds.
// Threads 0..63 of the block (any others have returned).
// Index source: explicit array, or (add path) consecutive cursor slots.
// ---------------------------------------------------------------------------
struct SetArgs {
  const int32_t* indices;  // NULL => (add_count + i) mod C
  const float* values;     // float32 priorities (set_priority, _add) ...
  int64_t n;
  const double* values64;  // ... or, if non-null, float64 values (a standalone SumTree.set)
};

// ---------------------------------------------------------------------------
// Block-parallel forms of the two single-wave chains above (same float64
// operations in the same order, so bitwise the same trees and indices), for a
// block of T threads: the riders get a whole 1024-thread block anyway.
// ---------------------------------------------------------------------------
__device__ __forceinline__ int readlane_i(int x, int l) { return __builtin_amdgcn_readlane(x, l); }
__device__ __forceinline__ double readlane_d(double x, int l) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(x), l);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(x), l);
  return __hiloint2double(hi, lo);
}

// Ordered chain of float64 adds per tree node: update i (lane i) hits node n_i,
// prev_i = the latest earlier update on n_i (-1: none).  before_i = the node's value
// before update i (the tree value, or after_prev), after_i = before_i + delta_i --
// resolved in rounds along the prev links, each round one shuffle.
__device__ __forceinline__ double node_chain(bool act, int prev, double tree_val, double& delta,
                                             bool leaf, double val) {
  bool done = act && prev < 0;
  double before = tree_val, after = 0.0;
  if (done) {
    if (leaf) delta = __dsub_rn(val, before);
    after = __dadd_rn(before, delta);
  }
  while (__ballot(act && !done)) {
    const int src = prev < 0 ? 0 : prev;
    const double ap = __shfl(after, src);
    const int dp = __shfl((int)done, src);
    if (act && !done && dp) {
      before = ap;
      if (leaf) delta = __dsub_rn(val, before);
      after = __dadd_rn(before, delta);
      done = true;
    }
  }
  return after;
}

constexpr int kSumtreeParLds = kWave * 8;   // bytes: the chunk's deltas

// sum_tree.py:178-205 called in order for each (index, value) of the batch
// (prioritized_replay_buffer.py:213-214): wave w owns tree levels w, w + T/64, ...,
// lane i = update i of a <= 64-update chunk.  Phase 1: the leaf level's chain gives
// every update's delta (value - the leaf as left by the earlier updates); phase 2:
// each level's nodes take their updates' deltas in update order, and the last
// update on a node stores it.
template <int T>
__device__ inline void sumtree_set_par(const ReplayView& v, const SetArgs& a, void* lds) {
  constexpr int NW = T / 64;
  double* s_delta = (double*)lds;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  dq_replay_meta* meta = v.meta;
  // the first chunk's (index, value) pairs load with the control block (clamped, no
  // branch), so the tree loads wait on one memory round, not two
  const int64_t l0 = a.n > 0 ? (lane < a.n ? lane : a.n - 1) : 0;
  const int32_t pre_i = (a.indices && a.n > 0) ? a.indices[l0] : 0;
  const double pre_v = a.n > 0 ? (a.values64 ? a.values64[l0] : (double)a.values[l0]) : 0.0;
  if (meta->status != 0) return;
  const int depth = v.depth;
  const int64_t base = meta->add_count;
  double maxrec = meta->max_recorded_priority;
  bool stop = false;
  for (int64_t c0 = 0; c0 < a.n && !stop; c0 += kWave) {
    const int m = (int)((a.n - c0) < kWave ? (a.n - c0) : kWave);
    int64_t idx = 0;
    double val = 0.0;
    if (lane < m) {
      if (c0 == 0) {
        idx = a.indices ? (int64_t)pre_i : pymod(base + lane, v.C);
        val = pre_v;
      } else {
        idx = a.indices ? (int64_t)a.indices[c0 + lane] : pymod(base + c0 + lane, v.C);
        val = a.values64 ? a.values64[c0 + lane] : (double)a.values[c0 + lane];
      }
    }
    // the reference raises at the first negative value, after applying the earlier ones
    const bool badi = lane < m && (idx < 0 || idx >= ((int64_t)1 << depth));
    const uint64_t negm = __ballot(lane < m && (val < 0.0 || badi));
    int me = m;
    if (negm) {
      me = __ffsll((unsigned long long)negm) - 1;
      stop = true;
    }
    const bool act = lane < me;
    if (wave == 0)
      for (int i = 0; i < me; ++i) {   // max(value, max_rec) with Python's argument order
        const double x = readlane_d(val, i);
        maxrec = (maxrec > x) ? maxrec : x;
      }
    const int node_leaf = act ? (int)idx : 0;
    // same-node links at level L (node = leaf >> (depth - L))
    auto links = [&](int L, int& prev, bool& last) {
      const int node = node_leaf >> (depth - L);
      prev = -1;
      last = true;
      for (int j = 0; j < me; ++j) {
        const int nj = readlane_i(node_leaf, j) >> (depth - L);
        if (nj == node) {
          if (j < lane) prev = j;
          if (j > lane) last = false;
        }
      }
    };
    // this wave's levels: issue every node load first
    constexpr int KL = (64 + NW - 1) / NW;   // levels per wave, depth < 63
    double tv[KL];
#pragma unroll
    for (int k = 0; k < KL; ++k) {
      const int L = wave + NW * k;
      tv[k] = (act && L <= depth) ? v.tree[((int64_t)1 << L) - 1 + (node_leaf >> (depth - L))] : 0.0;
    }
    if (wave == depth % NW) {          // the leaf level's owner: deltas
      int prev;
      bool last;
      links(depth, prev, last);
      double delta = 0.0;
      node_chain(act, prev, tv[depth / NW], delta, true, val);
      if (act) s_delta[lane] = delta;
    }
    __syncthreads();
    double delta = act ? s_delta[lane] : 0.0;
#pragma unroll
    for (int k = 0; k < KL; ++k) {
      const int L = wave + NW * k;
      if (L > depth) break;
      int prev;
      bool last;
      links(L, prev, last);
      const double after = node_chain(act, prev, tv[k], delta, false, val);
      if (act && last) v.tree[((int64_t)1 << L) - 1 + (node_leaf >> (depth - L))] = after;
    }
    if (stop) {                        // the first bad update: a bad index, else its value
      const int64_t bi = (int64_t)readlane_i((int)idx, me);   // indices are int32
      const double bv = readlane_d(val, me);
      const bool oob = bi < 0 || bi >= ((int64_t)1 << depth);
      if (threadIdx.x == 0)
        latch(meta, oob ? DQ_ST_BAD_INDEX : DQ_ST_NEG_PRIORITY, (int)(c0 + me),
              oob ? (double)bi : bv);
    }
    __threadfence_block();
    __syncthreads();                   // the next chunk reads what this one stored
  }
  if (threadIdx.x == 0) meta->max_recorded_priority = maxrec;
}

// Prioritized stratified sampling (prioritized_replay_buffer.py:152-170 /
// sum_tree.py:99-139) with T threads.  The tree's top kTopLevels levels (2047 nodes,
// 16 KB) are read by the whole block in the same memory round as the control block,
// and every stratum walks its first 10 levels in LDS; below them 32 lanes per
// stratum descend 5 levels per round -- lane j of the group loads the left-child
// sum of subtree node j (breadth-first), then the group walks the 5 levels through
// shuffles: for a 2^20-leaf tree 2 dependent rounds instead of 4 (or 20).  The
// retry loop for invalid draws is the reference's sequential one (thread 0).
constexpr int kTopLevels = 11;
constexpr int kPerSampleParLds = kPerSampleLds + ((1 << kTopLevels) - 1) * 8;

template <int T>
__device__ inline void per_sample_par(const ReplayView& v, int B, int32_t* out, void* lds) {
  static_assert(T % 32 == 0, "32-lane groups");
  static_assert(kPerSampleLds % 8 == 0, "s_top alignment");
  int64_t* s_idx = (int64_t*)lds;
  uint8_t* s_ok = (uint8_t*)(s_idx + kMaxBatch);
  double* s_top = (double*)((uint8_t*)lds + kPerSampleLds);
  const int t = threadIdx.x, g = t >> 5, j = t & 31;
  dq_replay_meta* meta = v.meta;
  // the top levels first: their loads do not wait for the control block's
  const int ktop = v.depth + 1 < kTopLevels ? v.depth + 1 : kTopLevels;
  const int ntop = (1 << ktop) - 1;
  constexpr int kTopR = ((1 << kTopLevels) - 1 + T - 1) / T;
  double top[kTopR];
#pragma unroll
  for (int r = 0; r < kTopR; ++r) top[r] = v.tree[min(t + r * T, ntop - 1)];
  const int64_t add_count = meta->add_count;
  const int64_t pos0 = meta->tape_pos;
  const int64_t len = meta->tape_len;
  const double total = v.tree[0];
  bool fail = meta->status != 0;
  if (!fail && total == 0.0) {
    if (t == 0) latch(meta, DQ_ST_EMPTY_TREE, 0, 0.0);
    fail = true;
  }
  if (!fail && pos0 + 2 * (int64_t)B > len) {
    if (t == 0) latch(meta, DQ_ST_TAPE_EXHAUSTED, 0, 0.0);
    fail = true;
  }
  if (fail) {
    if (t == 0) meta->reserved[0] = pos0;
    for (int i = t; i < B; i += T) out[i] = 0;
    return;
  }
#pragma unroll
  for (int r = 0; r < kTopR; ++r)
    if (t + r * T < ntop) s_top[t + r * T] = top[r];
  __syncthreads();
  // subtree node j of the group: level offset l (0..4), position p within it
  const int l = 31 - __clz(j + 1), p = j + 1 - (1 << l);
  const double step = 1.0 / (double)B;        // np.linspace(0, 1, B + 1)
  for (int i0 = 0; i0 < B; i0 += T / 32) {
    const int i = i0 + g;
    const bool mine = i < B;
    double q = 0.0;
    if (mine) {
      const double u = res53(v.tape[pos0 + 2 * i], v.tape[pos0 + 2 * i + 1]);
      const double lo = __dmul_rn((double)i, step);
      const double hi = (i + 1 == B) ? 1.0 : __dmul_rn((double)(i + 1), step);
      q = __dmul_rn(__dadd_rn(lo, __dmul_rn(__dsub_rn(hi, lo), u)), total);   // uniform * total
    }
    int64_t node = 0;                          // index at level d
    for (int d = 0; d < ktop - 1; ++d) {       // children within the staged levels
      const double lf = s_top[(2 << d) - 1 + 2 * node];
      if (q < lf) {
        node = 2 * node;
      } else {
        node = 2 * node + 1;
        q = __dsub_rn(q, lf);
      }
    }
    for (int d = ktop - 1; d < v.depth; d += 5) {
      const int lv = d + l + 1;                // level of the left child this lane fetches
      double left = 0.0;
      if (mine && j < 31 && lv <= v.depth)
        left = v.tree[((int64_t)1 << lv) - 1 + 2 * ((node << l) + p)];
      int64_t pc = 0;                          // path position within the subtree level
#pragma unroll
      for (int s = 0; s < 5; ++s) {
        if (d + s >= v.depth) break;
        const double lf = __shfl(left, (int)((1 << s) - 1 + pc), 32);
        if (q < lf) {
          pc = 2 * pc;
        } else {
          pc = 2 * pc + 1;
          q = __dsub_rn(q, lf);
        }
      }
      const int levels = v.depth - d < 5 ? v.depth - d : 5;
      node = (node << levels) + pc;
    }
    if (mine && j == 0) {
      s_idx[i] = node;
      s_ok[i] = is_valid(v, node, add_count);
    }
  }
  __syncthreads();
  if (t == 0) {
    int64_t pos = pos0 + 2 * (int64_t)B;
    int budget = v.max_attempts;
    for (int i = 0; i < B; ++i) {
      if (s_ok[i]) continue;
      if (budget == 0) {
        latch(meta, DQ_ST_MAX_ATTEMPTS, i, 0.0);
        break;
      }
      int64_t cand = s_idx[i];
      bool tape_dry = false;
      while (budget > 0) {
        if (pos + 2 > len) {
          tape_dry = true;
          break;
        }
        const double u = res53(v.tape[pos], v.tape[pos + 1]);
        pos += 2;
        cand = descend(v.tree, v.depth, __dmul_rn(u, total));
        --budget;
        if (is_valid(v, cand, add_count)) break;
      }
      s_idx[i] = cand;
      if (tape_dry) {
        latch(meta, DQ_ST_TAPE_EXHAUSTED, i, 0.0);
        break;
      }
    }
    meta->reserved[0] = pos0;   // entry cursor, for dq_replay_rewind_last_sample
    meta->tape_pos = pos;
  }
  __syncthreads();
  for (int i = t; i < B; i += T) out[i] = (int32_t)s_idx[i];
}

// A replay operation recorded for a grouped launch instead of launched (the
// opaque dq_rider of the C ABI): the sum-tree update, an index sample or the
// NHWC gather, run by RiderOp (nature_cnn.hip) as extra blocks of a launch.
enum RiderKind : int32_t { kRiderNone = 0, kRiderSet = 1, kRiderPerSample = 2,
                           kRiderUniformSample = 3, kRiderGatherNhwc = 4, kRiderSetSample = 5 };

struct RiderDesc {
  int32_t kind;
  int32_t batch;
  int32_t gx;        // gather: column blocks of 256 threads per (b, which) stack
  int32_t groups;    // uniform sample: consecutive batches of `batch` (0 or 1: one)
  ReplayView v;
  GatherOut g;
  SetArgs s;
  int32_t* out;      // sample: indices
};
static_assert(sizeof(RiderDesc) <= sizeof(dq_rider), "dq_rider too small");

constexpr int kRiderLds = kSumtreeParLds > kPerSampleParLds ? kSumtreeParLds : kPerSampleParLds;

// Runs rider r as block blk of a launch with T >= 256 threads per block.  kGroups: the
// launch carries a grouped uniform sample (the DQN learner loop's chunk gather).
template <int T, bool kGroups = false>
__device__ __forceinline__ void run_rider(const RiderDesc& r, int blk, void* lds) {
  static_assert(T % 256 == 0, "rider blocks are whole 256-thread gather sub-blocks");
  const int t = threadIdx.x;
  switch (r.kind) {
    case kRiderSet:
      sumtree_set_par<T>(r.v, r.s, lds);
      return;
    case kRiderPerSample:
      per_sample_par<T>(r.v, r.batch, r.out, lds);
      return;
    case kRiderSetSample:      // the write-back, then the next draw, in one block (dq_rider_chain)
      sumtree_set_par<T>(r.v, r.s, lds);
      __threadfence_block();
      __syncthreads();         // the draw reads the nodes (and status) the write-back stored
      per_sample_par<T>(r.v, r.batch, r.out, lds);
      return;
    case kRiderUniformSample:
      if (t < kWave) {
        if constexpr (kGroups)
          uniform_sample_groups(r.v, r.batch, r.out, r.groups > 1 ? r.groups : 1);
        else
          uniform_sample_body(r.v, r.batch, r.out);
      }
      return;
    case kRiderGatherNhwc: {
      const int sub = blk * (T / 256) + t / 256;
      const int slot = sub / r.gx;
      if (slot < 2 * r.batch) gather_nhwc4_body<kNhwcR>(r.v, r.g, sub - slot * r.gx, slot, t & 255);
      return;
    }
    default:
      return;
  }
}

template <int T>
inline int rider_blocks(const RiderDesc& r) {
  if (r.kind == kRiderGatherNhwc) return (r.gx * 2 * r.batch + T / 256 - 1) / (T / 256);
  return r.kind == kRiderNone ? 0 : 1;
}

}  // namespace dq
