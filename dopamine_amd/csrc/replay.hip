// Replay memory on the device: prioritized sum tree, uniform / stratified index
// sampling driven by a device-resident MT19937 word tape, validity rules and the
// frame-stack gather with n-step reward.  Restates (not translates) the
// reference's numpy code: circular_replay_buffer.py:53-558,
// prioritized_replay_buffer.py:117-235, sum_tree.py:65-205.
//
// Numerics: every float64 step of the sampler (stratum edges, uniform(), the
// q * total scaling, the descent's compare/subtract) and the float32 n-step
// reward are written with explicit _rn intrinsics and compiled with
// -ffp-contract=off, so results are bit-identical to the reference.
#include "common.h"

#include <algorithm>
#include <new>

namespace dq {

static thread_local std::string g_err;
void set_error(const std::string& msg) { g_err = msg; }

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

}  // namespace dq

struct dq_replay {
  dq_replay_config cfg;
  dq_replay_storage st;
  int depth;
  dq::ReplayView view() const {
    dq::ReplayView v;
    v.C = cfg.capacity;
    v.obs_bytes = cfg.obs_bytes;
    v.S = cfg.stack_size;
    v.n = cfg.update_horizon;
    v.depth = depth;
    v.max_attempts = cfg.max_sample_attempts;
    v.frames = st.frames;
    v.actions = st.actions;
    v.rewards = st.rewards;
    v.terminals = st.terminals;
    v.tree = st.tree;
    v.meta = st.meta;
    v.tape = st.tape;
    v.discount = st.discount;
    return v;
  }
};

namespace dq {

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
__device__ bool is_valid(const ReplayView& v, int64_t idx, int64_t add_count) {
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
// One wave.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(64) void k_per_sample(ReplayView v, int B, int32_t* out) {
  __shared__ int64_t s_idx[kMaxBatch];
  __shared__ uint8_t s_ok[kMaxBatch];
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
__global__ __launch_bounds__(64) void k_uniform_sample(ReplayView v, int B, int32_t* out) {
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

// Undo the tape consumption of the most recent sample (its indices are discarded):
// lets a speculatively prefetched batch be re-drawn after adds / host RNG use.
__global__ void k_rewind(dq_replay_meta* m) { m->tape_pos = m->reserved[0]; }

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
__device__ void write_scalars_wave(const ReplayView& v, const GatherOut& g, int b) {
  const int lane = threadIdx.x & 63;
  const int64_t idx = pymod((int64_t)g.indices[b], v.C);
  float p = 0.0f;
  bool t = false;
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
    const int64_t nxt = pymod(idx + L, v.C);
    if (g.action) g.action[b] = v.actions[idx];
    if (g.reward) g.reward[b] = acc;
    if (g.next_action) g.next_action[b] = v.actions[nxt];
    if (g.next_reward) g.next_reward[b] = v.rewards[nxt];
    if (g.terminal) g.terminal[b] = term ? 1 : 0;
    if (g.indices_out) g.indices_out[b] = (int32_t)idx;
    if (g.probs) g.probs[b] = (float)v.tree[((int64_t)1 << v.depth) - 1 + idx];
  }
}

__device__ __forceinline__ float4 u8x4_to_f32_255(uint32_t w) {
  float4 o;  // tf.div(tf.cast(x, f32), 255.) -- correctly rounded division
  o.x = __fdiv_rn((float)(w & 0xffu), 255.0f);
  o.y = __fdiv_rn((float)((w >> 8) & 0xffu), 255.0f);
  o.z = __fdiv_rn((float)((w >> 16) & 0xffu), 255.0f);
  o.w = __fdiv_rn((float)(w >> 24), 255.0f);
  return o;
}

// NCHW float32: grid.y = (b, which, k) frame; each thread converts kGatherR dwords
// strided by the block (kGatherR independent loads in flight before the stores;
// 2 blocks per 84x84 frame -> 512 blocks at B = 32, measured best in
// tools/bench_gather.hip).
constexpr int kGatherR = 4;

__global__ __launch_bounds__(256) void k_gather_f32(ReplayView v, GatherOut g) {
  const int S = v.S;
  const int slot = blockIdx.y;
  const int b = slot / (2 * S);
  const int r = slot - b * 2 * S;
  const int which = r / S;
  const int k = r - which * S;
  if (blockIdx.x == 0 && which == 0 && k == 0 && threadIdx.x < 64) write_scalars_wave(v, g, b);
  float* dst_base = (float*)(which ? g.next_state : g.state);
  if (!dst_base) return;
  const int64_t f = pymod(stack_base(v, g, b, which) - S + 1 + k, v.C);
  const int64_t nd = v.obs_bytes >> 2;  // obs_bytes % 4 == 0 checked on host
  const uint32_t* src = (const uint32_t*)(v.frames + f * v.obs_bytes);
  float4* dst = (float4*)(dst_base + ((int64_t)b * S + k) * v.obs_bytes);
  const int64_t t0 = (int64_t)blockIdx.x * blockDim.x * kGatherR + threadIdx.x;
  uint32_t w[kGatherR];
#pragma unroll
  for (int q = 0; q < kGatherR; ++q) {
    const int64_t t = t0 + (int64_t)q * blockDim.x;
    w[q] = t < nd ? src[t] : 0u;
  }
#pragma unroll
  for (int q = 0; q < kGatherR; ++q) {
    const int64_t t = t0 + (int64_t)q * blockDim.x;
    if (t < nd) dst[t] = u8x4_to_f32_255(w[q]);
  }
}

// NHWC float32 (the reference's state layout (B, H, W, stack), stack == 4): one
// block column per (b, which) stack; each thread loads the same dword of the 4
// frames (4 loads in flight) and writes 4 pixels x 4 channels = 64 contiguous bytes.
__global__ __launch_bounds__(256) void k_gather_nhwc4(ReplayView v, GatherOut g) {
  const int slot = blockIdx.y;
  const int b = slot >> 1, which = slot & 1;
  if (blockIdx.x == 0 && which == 0 && threadIdx.x < 64) write_scalars_wave(v, g, b);
  float* dst_base = (float*)(which ? g.next_state : g.state);
  if (!dst_base) return;
  const int64_t base = stack_base(v, g, b, which);
  const int64_t nd = v.obs_bytes >> 2;
  const int lane = threadIdx.x & 63;
  // this wave's 64 dwords (256 pixels) of each of the 4 frames
  const int64_t d0 = ((int64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63));
  if (d0 >= nd) return;
  const int64_t d = d0 + lane;
  uint32_t w[4];
#pragma unroll
  for (int k = 0; k < 4; ++k)
    w[k] = d < nd ? ((const uint32_t*)(v.frames + pymod(base - 3 + k, v.C) * v.obs_bytes))[d] : 0u;
  // store j: lane l writes pixel 64j + l (its 4 channels = 16 B), so every store
  // instruction covers 1 KiB contiguous; the bytes come from lane 16j + l/4.
  float4* dst = (float4*)(dst_base + (int64_t)b * 4 * v.obs_bytes) + 4 * d0;
  const int sh = 8 * (lane & 3);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int src = 16 * j + (lane >> 2);
    float4 o;
    o.x = __fdiv_rn((float)((__shfl(w[0], src) >> sh) & 0xffu), 255.0f);
    o.y = __fdiv_rn((float)((__shfl(w[1], src) >> sh) & 0xffu), 255.0f);
    o.z = __fdiv_rn((float)((__shfl(w[2], src) >> sh) & 0xffu), 255.0f);
    o.w = __fdiv_rn((float)((__shfl(w[3], src) >> sh) & 0xffu), 255.0f);
    if (4 * d0 + 64 * j + lane < 4 * nd) dst[64 * j + lane] = o;
  }
}

__device__ __forceinline__ int64_t frame_of(const ReplayView& v, const GatherOut& g, int slot,
                                            int* b_out, int* which_out, int* k_out) {
  const int S = v.S;
  const int b = slot / (2 * S);
  const int r = slot - b * 2 * S;
  const int which = r / S;
  const int k = r - which * S;
  *b_out = b;
  *which_out = which;
  *k_out = k;
  return pymod(stack_base(v, g, b, which) - S + 1 + k, v.C);
}

// raw byte copy of each stacked frame (reference dtype preserved).
__global__ __launch_bounds__(256) void k_gather_raw(ReplayView v, GatherOut g) {
  int b, which, k;
  const int slot = blockIdx.y;
  const int64_t f = frame_of(v, g, slot, &b, &which, &k);
  if (blockIdx.x == 0 && threadIdx.x < 64 && which == 0 && k == 0) write_scalars_wave(v, g, b);
  uint8_t* dst_base = (uint8_t*)(which ? g.next_state : g.state);
  if (!dst_base) return;
  const uint8_t* src = v.frames + f * v.obs_bytes;
  uint8_t* dst = dst_base + ((int64_t)b * v.S + k) * v.obs_bytes;
  const int64_t t0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  if ((v.obs_bytes & 15) == 0) {
    for (int64_t t = t0; t < (v.obs_bytes >> 4); t += stride)
      ((uint4*)dst)[t] = ((const uint4*)src)[t];
  } else {
    for (int64_t t = t0; t < v.obs_bytes; t += stride) dst[t] = src[t];
  }
}

// ---------------------------------------------------------------------------
// Sum-tree ordered batch update (sum_tree.py:178-205 called in order by
// prioritized_replay_buffer.py:213-214 or :139).  One wave; lane L owns tree
// level L.  For each update i (in order) the leaf lane computes
// delta_i = value_i - leaf, every level adds delta_i to its node, and the new
// value is forwarded (through LDS) to the next update hitting the same node, so
// each node receives exactly the reference's ordered chain of float64 adds.
// Index source: explicit array, or (add path) consecutive cursor slots.
// ---------------------------------------------------------------------------
struct SetArgs {
  const int32_t* indices;  // NULL => (add_count + i) mod C
  const float* values;
  int64_t n;
};

__global__ __launch_bounds__(64) void k_sumtree_set(ReplayView v, SetArgs a) {
  __shared__ int64_t s_idx[kWave];
  __shared__ float s_val[kWave];
  __shared__ double s_cur[kWave][kWave + 1];
  __shared__ int8_t s_next[kWave][kWave];  // [level][i] -> next update sharing the node
  const int lane = threadIdx.x;
  dq_replay_meta* meta = v.meta;
  if (meta->status != 0) return;
  const int depth = v.depth;
  const int64_t base = meta->add_count;
  double maxrec = meta->max_recorded_priority;
  bool stop = false;
  for (int64_t c0 = 0; c0 < a.n && !stop; c0 += kWave) {
    const int m = (int)((a.n - c0) < kWave ? (a.n - c0) : kWave);
    if (lane < m) {
      s_idx[lane] = a.indices ? (int64_t)a.indices[c0 + lane] : pymod(base + c0 + lane, v.C);
      s_val[lane] = a.values[c0 + lane];
    }
    __syncthreads();
    // the reference raises at the first negative value, after applying the earlier ones
    const bool badi = lane < m && (s_idx[lane] < 0 || s_idx[lane] >= ((int64_t)1 << depth));
    const uint64_t negm = __ballot(lane < m && (s_val[lane] < 0.0f || badi));
    int me = m;
    if (negm) {
      me = __ffsll((unsigned long long)negm) - 1;
      stop = true;
    }
    for (int i = 0; i < me; ++i) {  // max(value, max_rec) with Python's argument order
      const double x = (double)s_val[i];
      maxrec = (maxrec > x) ? maxrec : x;
    }
    // next-same table: levels 0..D(i,j) share a node between updates i < j
    for (int d = 0; d <= depth; ++d)
      if (lane < me) s_next[d][lane] = -1;
    __syncthreads();
    if (lane < me) {
      int covered = -1;
      for (int j = lane + 1; j < me && covered < depth; ++j) {
        const uint64_t x = (uint64_t)(s_idx[lane] ^ s_idx[j]);
        const int D = x ? depth - (64 - __clzll(x)) : depth;
        for (int d = covered + 1; d <= D; ++d) s_next[d][lane] = (int8_t)j;
        if (D > covered) covered = D;
      }
    }
    __syncthreads();
    const bool mine = lane <= depth;
    const int shift = depth - lane;
    const int64_t loff = ((int64_t)1 << (mine ? lane : 0)) - 1;
    if (mine)
      for (int i = 0; i < me; ++i) s_cur[lane][i] = v.tree[loff + (s_idx[i] >> shift)];
    __syncthreads();
    for (int i = 0; i < me; ++i) {
      const double cur = mine ? s_cur[lane][i] : 0.0;
      const double dl = __dsub_rn((double)s_val[i], cur);  // meaningful on the leaf lane
      const double delta = __shfl(dl, depth);
      if (mine) {
        const double x = __dadd_rn(cur, delta);
        const int j = s_next[lane][i];
        if (j >= 0)
          s_cur[lane][j] = x;
        else
          v.tree[loff + (s_idx[i] >> shift)] = x;
      }
    }
    __syncthreads();
    if (stop && lane == 0) {
      const bool oob = s_idx[me] < 0 || s_idx[me] >= ((int64_t)1 << depth);
      latch(meta, oob ? DQ_ST_BAD_INDEX : DQ_ST_NEG_PRIORITY, (int)(c0 + me),
            oob ? (double)s_idx[me] : (double)s_val[me]);
    }
  }
  if (lane == 0) meta->max_recorded_priority = maxrec;
}

__global__ void k_sumtree_get(ReplayView v, const int32_t* idx, int64_t n, float* out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    const int64_t leaf = idx[i];
    const bool ok = leaf >= 0 && leaf < ((int64_t)1 << v.depth);
    out[i] = ok ? (float)v.tree[((int64_t)1 << v.depth) - 1 + leaf] : 0.0f;
  }
}

__global__ void k_sumtree_level(double* tree, int d) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t n = (int64_t)1 << d;
  if (i < n) {
    const double* ch = tree + ((int64_t)1 << (d + 1)) - 1;
    tree[n - 1 + i] = __dadd_rn(ch[2 * i], ch[2 * i + 1]);
  }
}

// add(): write n transitions at consecutive cursor slots, then advance add_count.
__global__ __launch_bounds__(256) void k_add(ReplayView v, int64_t n, const uint8_t* frames,
                                             const int32_t* actions, const float* rewards,
                                             const uint8_t* terminals, uint8_t* fr_dst,
                                             int32_t* act_dst, float* rew_dst,
                                             uint8_t* term_dst) {
  const int64_t base = v.meta->add_count;
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t total = n * v.obs_bytes;
  for (int64_t t = tid; t < total; t += stride) {
    const int64_t r = t / v.obs_bytes, o = t - r * v.obs_bytes;
    fr_dst[pymod(base + r, v.C) * v.obs_bytes + o] = frames[t];
  }
  for (int64_t r = tid; r < n; r += stride) {
    const int64_t c = pymod(base + r, v.C);
    act_dst[c] = actions[r];
    rew_dst[c] = rewards[r];
    term_dst[c] = terminals[r];
  }
}

__global__ void k_bump(dq_replay_meta* m, int64_t n) { m->add_count += n; }

__global__ void k_set_meta(dq_replay_meta* m, int64_t add_count, double max_rec) {
  m->add_count = add_count;
  m->max_recorded_priority = max_rec;
  m->status = 0;
  m->status_arg = 0;
  m->status_value = 0.0;
}

__global__ void k_set_tape(dq_replay_meta* m, int64_t len) {
  m->tape_pos = 0;
  m->tape_len = len;
}

}  // namespace dq

using namespace dq;

extern "C" {

int dq_abi_version(void) { return DQ_ABI_VERSION; }
const char* dq_last_error(void) { return g_err.c_str(); }

int dq_sumtree_depth(int64_t capacity) {
  int d = 0;
  while (((int64_t)1 << d) < capacity) ++d;  // == ceil(log2(capacity)) for capacity >= 1
  return d;
}

int dq_replay_create(const dq_replay_config* cfg, const dq_replay_storage* st, dq_replay** out) {
  DQ_CHECK_ARG(cfg && st && out, "null argument");
  DQ_CHECK_ARG(cfg->capacity > 0, "capacity must be positive");
  DQ_CHECK_ARG(cfg->capacity >= (int64_t)cfg->update_horizon + cfg->stack_size,
               "There is not enough capacity to cover update_horizon and stack_size.");
  DQ_CHECK_ARG(cfg->stack_size >= 1 && cfg->update_horizon >= 1, "stack_size/update_horizon must be >= 1");
  DQ_CHECK_ARG(cfg->obs_bytes > 0, "obs_bytes must be positive");
  DQ_CHECK_ARG(st->frames && st->actions && st->rewards && st->terminals && st->meta && st->discount,
               "storage pointers must be non-null");
  DQ_CHECK_ARG(!cfg->prioritized || st->tree, "prioritized buffer needs a tree");
  DQ_CHECK_ARG(cfg->capacity < ((int64_t)1 << 31), "capacity must fit int32 indices");
  dq_replay* h = new (std::nothrow) dq_replay;
  DQ_CHECK_ARG(h, "out of host memory");
  h->cfg = *cfg;
  h->st = *st;
  h->depth = dq_sumtree_depth(cfg->capacity);
  *out = h;
  return DQ_OK;
}

int dq_replay_destroy(dq_replay* h) {
  delete h;
  return DQ_OK;
}

int dq_replay_add(dq_replay* h, int64_t n, const uint8_t* frames, const int32_t* actions,
                  const float* rewards, const uint8_t* terminals, const float* priorities,
                  void* stream) {
  DQ_CHECK_ARG(h && n >= 0, "bad handle/count");
  if (n == 0) return DQ_OK;
  DQ_CHECK_ARG(frames && actions && rewards && terminals, "null transition array");
  DQ_CHECK_ARG(!h->cfg.prioritized || priorities, "prioritized add needs priorities");
  hipStream_t s = (hipStream_t)stream;
  ReplayView v = h->view();
  if (h->cfg.prioritized) {  // _add: sum_tree.set(cursor, p) before the write (prb:139)
    SetArgs a{nullptr, priorities, n};
    hipLaunchKernelGGL(k_sumtree_set, dim3(1), dim3(64), 0, s, v, a);
    DQ_CHECK_LAUNCH("k_sumtree_set");
  }
  const int64_t work = std::max<int64_t>(n * h->cfg.obs_bytes, n);
  const int blocks = (int)std::min<int64_t>((work + 255) / 256, 4096);
  hipLaunchKernelGGL(k_add, dim3(blocks), dim3(256), 0, s, v, n, frames, actions, rewards,
                     terminals, h->st.frames, h->st.actions, h->st.rewards, h->st.terminals);
  DQ_CHECK_LAUNCH("k_add");
  hipLaunchKernelGGL(k_bump, dim3(1), dim3(1), 0, s, h->st.meta, n);
  DQ_CHECK_LAUNCH("k_bump");
  return DQ_OK;
}

int dq_replay_sample_indices(dq_replay* h, int32_t batch, int32_t* indices_out, void* stream) {
  DQ_CHECK_ARG(h && indices_out, "null argument");
  DQ_CHECK_ARG(batch >= 1 && batch <= kMaxBatch, "batch must be in [1, 1024]");
  DQ_CHECK_ARG(h->st.tape, "RNG tape not attached");
  hipStream_t s = (hipStream_t)stream;
  if (h->cfg.prioritized)
    hipLaunchKernelGGL(k_per_sample, dim3(1), dim3(64), 0, s, h->view(), batch, indices_out);
  else
    hipLaunchKernelGGL(k_uniform_sample, dim3(1), dim3(64), 0, s, h->view(), batch, indices_out);
  DQ_CHECK_LAUNCH("sample_indices");
  return DQ_OK;
}

int dq_replay_gather(dq_replay* h, const int32_t* indices, int32_t batch, int32_t layout,
                     void* state_out, void* next_state_out, int32_t* action_out,
                     float* reward_out, int32_t* next_action_out, float* next_reward_out,
                     uint8_t* terminal_out, int32_t* indices_out, float* probs_out,
                     void* stream) {
  DQ_CHECK_ARG(h && indices && batch >= 1, "bad arguments");
  DQ_CHECK_ARG(!probs_out || h->cfg.prioritized, "probs requested from a uniform buffer");
  GatherOut g{indices, state_out, next_state_out, action_out, reward_out, next_action_out,
              next_reward_out, terminal_out, indices_out, probs_out};
  hipStream_t s = (hipStream_t)stream;
  const int64_t slots = (int64_t)batch * 2 * h->cfg.stack_size;
  DQ_CHECK_ARG(slots < 65536, "batch * 2 * stack too large");
  if (layout == DQ_LAYOUT_F32_NORM) {
    DQ_CHECK_ARG(h->cfg.obs_is_u8, "F32_NORM layout needs uint8 observations");
    DQ_CHECK_ARG((h->cfg.obs_bytes & 3) == 0, "F32_NORM layout needs obs_bytes % 4 == 0");
    const int64_t nd = h->cfg.obs_bytes >> 2;
    dim3 grid((unsigned)((nd + 256 * kGatherR - 1) / (256 * kGatherR)), (unsigned)slots);
    hipLaunchKernelGGL(k_gather_f32, grid, dim3(256), 0, s, h->view(), g);
  } else if (layout == DQ_LAYOUT_F32_NHWC) {
    DQ_CHECK_ARG(h->cfg.obs_is_u8, "F32_NHWC layout needs uint8 observations");
    DQ_CHECK_ARG(h->cfg.stack_size == 4, "F32_NHWC layout needs stack_size == 4");
    DQ_CHECK_ARG((h->cfg.obs_bytes & 3) == 0, "F32_NHWC layout needs obs_bytes % 4 == 0");
    const int64_t nd = h->cfg.obs_bytes >> 2;
    dim3 grid((unsigned)((nd + 255) / 256), (unsigned)(2 * batch));
    hipLaunchKernelGGL(k_gather_nhwc4, grid, dim3(256), 0, s, h->view(), g);
  } else if (layout == DQ_LAYOUT_RAW) {
    const int64_t units = (h->cfg.obs_bytes & 15) == 0 ? h->cfg.obs_bytes >> 4 : h->cfg.obs_bytes;
    const int64_t bx = std::min<int64_t>((units + 255) / 256, 64);
    hipLaunchKernelGGL(k_gather_raw, dim3((unsigned)bx, (unsigned)slots), dim3(256), 0, s,
                       h->view(), g);
  } else {
    DQ_CHECK_ARG(false, "unknown layout");
  }
  DQ_CHECK_LAUNCH("gather");
  return DQ_OK;
}

int dq_sumtree_set(dq_replay* h, const int32_t* indices, const float* priorities, int64_t n,
                   void* stream) {
  DQ_CHECK_ARG(h && h->cfg.prioritized, "sum tree needs a prioritized buffer");
  DQ_CHECK_ARG(indices && priorities && n >= 0, "bad arguments");
  DQ_CHECK_ARG(h->depth < 63, "tree too deep");
  if (n == 0) return DQ_OK;
  SetArgs a{indices, priorities, n};
  hipLaunchKernelGGL(k_sumtree_set, dim3(1), dim3(64), 0, (hipStream_t)stream, h->view(), a);
  DQ_CHECK_LAUNCH("k_sumtree_set");
  return DQ_OK;
}

int dq_sumtree_get(dq_replay* h, const int32_t* indices, int64_t n, float* out, void* stream) {
  DQ_CHECK_ARG(h && h->cfg.prioritized && indices && out && n >= 0, "bad arguments");
  if (n == 0) return DQ_OK;
  hipLaunchKernelGGL(k_sumtree_get, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, h->view(), indices, n, out);
  DQ_CHECK_LAUNCH("k_sumtree_get");
  return DQ_OK;
}

int dq_sumtree_rebuild(dq_replay* h, void* stream) {
  DQ_CHECK_ARG(h && h->cfg.prioritized, "sum tree needs a prioritized buffer");
  for (int d = h->depth - 1; d >= 0; --d) {
    const int64_t n = (int64_t)1 << d;
    hipLaunchKernelGGL(k_sumtree_level, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, h->st.tree, d);
    DQ_CHECK_LAUNCH("k_sumtree_level");
  }
  return DQ_OK;
}

int dq_replay_set_meta(dq_replay* h, int64_t add_count, double max_rec, void* stream) {
  DQ_CHECK_ARG(h && add_count >= 0, "bad arguments");
  hipLaunchKernelGGL(k_set_meta, dim3(1), dim3(1), 0, (hipStream_t)stream, h->st.meta,
                     add_count, max_rec);
  DQ_CHECK_LAUNCH("k_set_meta");
  return DQ_OK;
}

int dq_replay_set_tape(dq_replay* h, int64_t len, void* stream) {
  DQ_CHECK_ARG(h && len >= 0 && len <= h->st.tape_capacity, "tape length out of range");
  hipLaunchKernelGGL(k_set_tape, dim3(1), dim3(1), 0, (hipStream_t)stream, h->st.meta, len);
  DQ_CHECK_LAUNCH("k_set_tape");
  return DQ_OK;
}

int dq_replay_rewind_last_sample(dq_replay* h, void* stream) {
  DQ_CHECK_ARG(h, "null handle");
  hipLaunchKernelGGL(k_rewind, dim3(1), dim3(1), 0, (hipStream_t)stream, h->st.meta);
  DQ_CHECK_LAUNCH("k_rewind");
  return DQ_OK;
}

int dq_replay_read_meta(dq_replay* h, dq_replay_meta* out, void* stream) {
  DQ_CHECK_ARG(h && out, "null argument");
  DQ_CHECK_HIP(hipMemcpyAsync(out, h->st.meta, sizeof(dq_replay_meta), hipMemcpyDeviceToHost,
                              (hipStream_t)stream));
  DQ_CHECK_HIP(hipStreamSynchronize((hipStream_t)stream));
  return DQ_OK;
}

int dq_sync_copy(void* dst, const void* src, int64_t bytes, void* stream) {
  DQ_CHECK_ARG(dst && src && bytes >= 0, "bad arguments");
  if (bytes == 0) return DQ_OK;
  DQ_CHECK_HIP(hipMemcpyAsync(dst, src, (size_t)bytes, hipMemcpyDeviceToDevice, (hipStream_t)stream));
  return DQ_OK;
}

}  // extern "C"
