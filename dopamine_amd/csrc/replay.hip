// Replay memory on the device: prioritized sum tree, uniform / stratified index
// sampling driven by a device-resident MT19937 word tape, validity rules and the
// frame-stack gather with n-step reward.  Restates (not translates) the
// reference's numpy code: circular_replay_buffer.py:53-558,
// prioritized_replay_buffer.py:117-235, sum_tree.py:65-205.  The device bodies
// live in replay_dev.h (shared with the grouped launches of nature_cnn.hip).
#include "replay_dev.h"

#include <hip/hip_fp16.h>

#include <algorithm>
#include <cstring>
#include <new>

namespace dq {

static thread_local std::string g_err;
void set_error(const std::string& msg) { g_err = msg; }

}  // namespace dq

struct dq_replay {
  dq_replay_config cfg;
  dq_replay_storage st;
  int depth;
  bool tree_only;   // dq_sumtree_create: a standalone SumTree (no transition store)
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

constexpr int kTreeT = 1024;   // block of the block-parallel sum-tree kernels

__global__ __launch_bounds__(kTreeT) void k_per_sample(ReplayView v, int B, int32_t* out) {
  warm_kernargs<sizeof(ReplayView) + 16>();
  __shared__ __attribute__((aligned(16))) uint8_t lds[kPerSampleParLds];
  per_sample_par<kTreeT>(v, B, out, lds);
}

__global__ __launch_bounds__(64) void k_uniform_sample(ReplayView v, int B, int32_t* out, int G) {
  warm_kernargs<sizeof(ReplayView) + 24>();
  if (G > 1)
    uniform_sample_groups(v, B, out, G);
  else
    uniform_sample_body(v, B, out);
}

// SumTree.sample / stratified_sample (sum_tree.py:99-166) on the flat heap, one
// lane per query: DQ_SUMTREE_QUERY uses the caller's query values, DQ_SUMTREE_RANDOM
// one random.random() per query (two tape words each, in order), DQ_SUMTREE_STRATIFIED
// random.uniform(i/n, (i+1)/n) per stratum -- the same float64 steps as the PER
// sampler's first phase (per_sample_body), without the validity rule.
__global__ __launch_bounds__(256) void k_sumtree_sample(ReplayView v, int mode, int n,
                                                        const double* query, int64_t* out) {
  dq_replay_meta* meta = v.meta;
  const int64_t pos = meta->tape_pos;
  const bool random = mode != DQ_SUMTREE_QUERY;
  const double total = v.tree[0];
  bool fail = meta->status != 0;
  if (!fail && total == 0.0) {
    if (threadIdx.x == 0) latch(meta, DQ_ST_EMPTY_TREE, 0, 0.0);
    fail = true;
  }
  if (!fail && random && pos + 2 * (int64_t)n > meta->tape_len) {
    if (threadIdx.x == 0) latch(meta, DQ_ST_TAPE_EXHAUSTED, 0, 0.0);
    fail = true;
  }
  const double step = 1.0 / (double)n;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    int64_t node = 0;
    if (!fail) {
      double q;
      if (!random) {
        q = query[i];
      } else {
        const double u = res53(v.tape[pos + 2 * i], v.tape[pos + 2 * i + 1]);
        if (mode == DQ_SUMTREE_RANDOM) {
          q = u;
        } else {
          const double lo = __dmul_rn((double)i, step);
          const double hi = (i + 1 == n) ? 1.0 : __dmul_rn((double)(i + 1), step);
          q = __dadd_rn(lo, __dmul_rn(__dsub_rn(hi, lo), u));
        }
      }
      node = descend(v.tree, v.depth, __dmul_rn(q, total));
    }
    out[i] = node;
  }
  __syncthreads();
  if (threadIdx.x == 0 && !fail && random) {
    meta->reserved[0] = pos;
    meta->tape_pos = pos + 2 * (int64_t)n;
  }
}

// Undo the tape consumption of the most recent sample (its indices are discarded):
// lets a speculatively prefetched batch be re-drawn after adds / host RNG use.
__global__ void k_rewind(dq_replay_meta* m) { m->tape_pos = m->reserved[0]; }

// _select_action (dqn_agent.py:394-416) for a replay that samples from Python's `random`
// (PER), on the tape: u = random.random() (genrand_res53, 2 words); u <= epsilon:
// random.randint(0, A - 1) = Python's _randbelow(A): getrandbits(k = A.bit_length()) =
// word >> (32 - k), redrawn while >= A; else the first argmax of q (dqn:416).  The tape
// advances by exactly the words the reference consumes, so the host's `random` needs no
// synchronisation per action.  A run past the tape consumes nothing and returns -1.
__global__ void k_egreedy(dq_replay_meta* meta, const uint32_t* tape, const float* q, int A,
                          double epsilon, int32_t* action) {
  int64_t pos = meta->tape_pos;
  const int64_t len = meta->tape_len;
  int32_t a = -1;
  if (meta->status == 0 && pos + 2 <= len) {
    const double u = res53(tape[pos], tape[pos + 1]);
    pos += 2;
    if (u <= epsilon) {
      const int k = 32 - __clz(A);
      while (pos < len) {
        const uint32_t r = tape[pos++] >> (32 - k);
        if (r < (uint32_t)A) {
          a = (int32_t)r;
          break;
        }
      }
    } else {
      int best = 0;
      float bq = q[0];
      for (int j = 1; j < A; ++j)
        if (q[j] > bq) {
          bq = q[j];
          best = j;
        }
      a = best;
    }
  }
  if (a >= 0) meta->tape_pos = pos;
  action[0] = a;
}


// NCHW float32: grid.y = (b, which, k) frame; each thread converts kGatherR dwords
// strided by the block (kGatherR independent loads in flight before the stores;
// 2 blocks per 84x84 frame -> 512 blocks at B = 32, measured best in
// tools/bench_gather.hip).
constexpr int kGatherR = 4;

__global__ __launch_bounds__(256) void k_gather_f32(ReplayView v, GatherOut g) {
  warm_kernargs<sizeof(ReplayView) + sizeof(GatherOut)>();
  const int S = v.S;
  const int slot = blockIdx.y;
  const int b = slot / (2 * S);
  const int r = slot - b * 2 * S;
  const int which = r / S;
  const int k = r - which * S;
  if (blockIdx.x == 0 && which == 0 && k == 0 && threadIdx.x < 64)
    write_scalars_wave(v, g, b, pymod((int64_t)g.indices[b], v.C));
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

// Standalone NHWC gather: block columns 0 .. gx-1 copy the frames, the last column's
// first wave writes the sample's scalars (state slots only), so no frame wave waits on
// the scalar chain.
template <int R>
__global__ __launch_bounds__(256) void k_gather_nhwc4(ReplayView v, GatherOut g) {
#ifdef DQ_GATHER_PROF
  unsigned long long gp[4] = {__builtin_amdgcn_s_memrealtime(), 0, 0, 0};
  unsigned long long* gpp = gp;
  const unsigned gp_wid = (blockIdx.y * gridDim.x + blockIdx.x) * (blockDim.x / 64) + (threadIdx.x >> 6);
  const unsigned gp_seq = gp_wid < (unsigned)kGpWaves ? g_gp_seq[gp_wid] : 0u;   // issued first
#else
  unsigned long long* gpp = nullptr;
#endif
  warm_kernargs<sizeof(ReplayView) + sizeof(GatherOut)>();
  const int slot = blockIdx.y;
  if (blockIdx.x == gridDim.x - 1) {
    if ((slot & 1) == 0 && threadIdx.x < kWave)
      write_scalars_wave(v, g, slot >> 1, pymod((int64_t)g.indices[slot >> 1], v.C));
  } else {
    gather_nhwc4_body<R, kScalNone, true>(v, g, blockIdx.x, slot, threadIdx.x, gpp);
  }
#ifdef DQ_GATHER_PROF
  GP_STAMP(gp, 3);
  if ((threadIdx.x & 63) == 0 && gp_wid < (unsigned)kGpWaves) {
    unsigned long long* d = g_gp_wave[gp_seq % kGpRing][gp_wid];
    d[0] = gp[0];
    d[1] = gp[1];
    d[2] = gp[2];
    d[3] = gp[3];
    g_gp_seq[gp_wid] = gp_seq + 1;
  }
#endif
}

#ifdef DQ_GATHER_PROF
// tools/gather_stamps.py: zero the ring and the per-wave counters; read them back
extern "C" int dq_debug_gather_reset(int32_t) {
  static unsigned long long zw[kGpRing][kGpWaves][4];
  static unsigned zs[kGpWaves];
  if (hipMemcpyToSymbol(HIP_SYMBOL(g_gp_wave), zw, sizeof(zw)) != hipSuccess) return -1;
  return hipMemcpyToSymbol(HIP_SYMBOL(g_gp_seq), zs, sizeof(zs)) == hipSuccess ? 0 : -1;
}
extern "C" int dq_debug_gather_read(unsigned long long* ring, unsigned* seq, unsigned* dims) {
  dims[0] = kGpRing;
  dims[1] = kGpWaves;
  if (hipMemcpyFromSymbol(ring, HIP_SYMBOL(g_gp_wave), sizeof(g_gp_wave)) != hipSuccess) return -1;
  return hipMemcpyFromSymbol(seq, HIP_SYMBOL(g_gp_seq), sizeof(g_gp_seq)) == hipSuccess ? 0 : -1;
}
#endif

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

// ---------------------------------------------------------------------------
// Action / reward elements of buffers whose action or reward is not a scalar int32 /
// float32 (circular_replay_buffer.py:96-183, sampled at :530-548).  One block per
// sample: L from the terminal store, the action rows copied as bytes, the n-step reward
// as numpy's np.sum(discount[:L] * trajectory_rewards, axis=0) -- the (L,) float32
// discount broadcast against the LAST axis of (L,) + reward_shape, products and the
// left-to-right sum (numpy's axis-0 order) in the promoted type -- then cast to the
// reward dtype as the assignment into the batch array does.
// ---------------------------------------------------------------------------
struct ElemArgs {
  const int32_t* indices;
  const uint8_t* act;        // (C, act_bytes)
  int act_bytes;
  const void* rew;           // (C, rew_elems) of dtype rew_dt
  int rew_elems, rew_last, rew_dt, acc64;
  uint8_t* act_out;
  uint8_t* nact_out;
  void* rew_out;
  void* nrew_out;
};

__device__ __forceinline__ int dt_size(int dt) {
  return dt == DQ_DT_F64 || dt == DQ_DT_I64 ? 8 : dt == DQ_DT_F32 || dt == DQ_DT_I32 ? 4
         : dt == DQ_DT_F16 || dt == DQ_DT_I16 ? 2 : 1;
}

// the element as a double: exact for every type here (int64 beyond 2^53 rounds as
// numpy's int64 -> float64 promotion does)
__device__ __forceinline__ double dt_load(const void* p, int64_t i, int dt) {
  switch (dt) {
    case DQ_DT_F32: return (double)((const float*)p)[i];
    case DQ_DT_F64: return ((const double*)p)[i];
    case DQ_DT_F16: return (double)__half2float(((const __half*)p)[i]);
    case DQ_DT_I8: return (double)((const int8_t*)p)[i];
    case DQ_DT_U8: return (double)((const uint8_t*)p)[i];
    case DQ_DT_I16: return (double)((const int16_t*)p)[i];
    case DQ_DT_I32: return (double)((const int32_t*)p)[i];
    default: return (double)((const int64_t*)p)[i];
  }
}

// store a float32-mode (f) or float64-mode (d) result with numpy's cast to the dtype
__device__ __forceinline__ void dt_store(void* p, int64_t i, int dt, bool acc64, float f, double d) {
  switch (dt) {
    case DQ_DT_F32: ((float*)p)[i] = acc64 ? __double2float_rn(d) : f; return;
    case DQ_DT_F64: ((double*)p)[i] = acc64 ? d : (double)f; return;
    case DQ_DT_F16: ((__half*)p)[i] = __float2half_rn(acc64 ? __double2float_rn(d) : f); return;
    case DQ_DT_I8: ((int8_t*)p)[i] = (int8_t)(acc64 ? (int64_t)d : (int64_t)f); return;
    case DQ_DT_U8: ((uint8_t*)p)[i] = (uint8_t)(acc64 ? (int64_t)d : (int64_t)f); return;
    case DQ_DT_I16: ((int16_t*)p)[i] = (int16_t)(acc64 ? (int64_t)d : (int64_t)f); return;
    case DQ_DT_I32: ((int32_t*)p)[i] = (int32_t)(acc64 ? (int64_t)d : (int64_t)f); return;
    default: ((int64_t*)p)[i] = acc64 ? (int64_t)d : (int64_t)f; return;
  }
}

__global__ __launch_bounds__(256) void k_gather_elems(ReplayView v, ElemArgs e) {
  const int b = blockIdx.x;
  const int64_t idx = pymod((int64_t)e.indices[b], v.C);
  bool term;
  const int L = traj_len(v, idx, &term);
  const int64_t nxt = pymod(idx + L, v.C);
  for (int i = threadIdx.x; i < e.act_bytes; i += blockDim.x) {
    if (e.act_out) e.act_out[(int64_t)b * e.act_bytes + i] = e.act[idx * e.act_bytes + i];
    if (e.nact_out) e.nact_out[(int64_t)b * e.act_bytes + i] = e.act[nxt * e.act_bytes + i];
  }
  const int es = dt_size(e.rew_dt);
  if (e.nrew_out)
    for (int i = threadIdx.x; i < e.rew_elems * es; i += blockDim.x)
      ((uint8_t*)e.nrew_out)[(int64_t)b * e.rew_elems * es + i] =
          ((const uint8_t*)e.rew)[nxt * e.rew_elems * es + i];
  if (!e.rew_out) return;
  // (L,) against (L,) + reward_shape: scalar reward -> elementwise; else the last axis m
  // must equal L (discount indexed by the element's last coordinate) or be broadcast
  // from 1 on either side; m == 1 < L broadcasts but its (.., L) sum cannot be assigned
  const int m = e.rew_last;
  if (m > 0 && L != m && L != 1) {
    if (threadIdx.x == 0) latch(v.meta, DQ_ST_BROADCAST, L, m == 1 ? 1.0 : 0.0);
    return;
  }
  for (int j = threadIdx.x; j < e.rew_elems; j += blockDim.x) {
    const int di = m > 0 && L == m ? j % m : -1;     // -1: discount index = trajectory step
    float f = 0.0f;
    double d = 0.0;
    for (int k = 0; k < L; ++k) {
      const float disc = v.discount[di < 0 ? k : di];
      const double r = dt_load(e.rew, pymod(idx + k, v.C) * e.rew_elems + j, e.rew_dt);
      if (e.acc64)
        d = __dadd_rn(d, __dmul_rn((double)disc, r));
      else
        f = __fadd_rn(f, __fmul_rn(disc, (float)r));
    }
    dt_store(e.rew_out, (int64_t)b * e.rew_elems + j, e.rew_dt, e.acc64 != 0, f, d);
  }
}

// raw byte copy of each stacked frame (reference dtype preserved).
__global__ __launch_bounds__(256) void k_gather_raw(ReplayView v, GatherOut g) {
  int b, which, k;
  const int slot = blockIdx.y;
  const int64_t f = frame_of(v, g, slot, &b, &which, &k);
  if (blockIdx.x == 0 && threadIdx.x < 64 && which == 0 && k == 0)
    write_scalars_wave(v, g, b, pymod((int64_t)g.indices[b], v.C));
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

__global__ __launch_bounds__(kTreeT) void k_sumtree_set(ReplayView v, SetArgs a) {
  warm_kernargs<sizeof(ReplayView) + sizeof(SetArgs)>();
  __shared__ __attribute__((aligned(16))) uint8_t lds[kSumtreeParLds];
  sumtree_set_par<kTreeT>(v, a, lds);
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

// the extra -D flags every translation unit was compiled with (dopamine_amd/_build.py
// passes them as DQ_BUILD_FLAGS): "" for the product library
#ifdef DQ_BUILD_FLAGS
const char* dq_build_flags(void) { return DQ_BUILD_FLAGS; }
#else
const char* dq_build_flags(void) { return "(unrecorded: not built by dopamine_amd/_build.py)"; }
#endif
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
  h->tree_only = false;
  *out = h;
  return DQ_OK;
}

int dq_sumtree_create(int64_t capacity, double* tree, dq_replay_meta* meta, uint32_t* tape,
                      int64_t tape_capacity, dq_replay** out) {
  DQ_CHECK_ARG(out && tree && meta, "null argument");
  DQ_CHECK_ARG(capacity > 0, "Sum tree capacity should be positive.");
  DQ_CHECK_ARG(capacity < ((int64_t)1 << 31), "capacity must fit int32 indices");
  dq_replay* h = new (std::nothrow) dq_replay;
  DQ_CHECK_ARG(h, "out of host memory");
  memset(&h->cfg, 0, sizeof(h->cfg));
  memset(&h->st, 0, sizeof(h->st));
  h->cfg.capacity = capacity;
  h->cfg.stack_size = 1;
  h->cfg.update_horizon = 1;
  h->cfg.prioritized = 1;
  h->st.tree = tree;
  h->st.meta = meta;
  h->st.tape = tape;
  h->st.tape_capacity = tape ? tape_capacity : 0;
  h->depth = dq_sumtree_depth(capacity);
  h->tree_only = true;
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
  DQ_CHECK_ARG(!h->tree_only, "a standalone sum tree has no transition store");
  if (n == 0) return DQ_OK;
  DQ_CHECK_ARG(frames && actions && rewards && terminals, "null transition array");
  DQ_CHECK_ARG(!h->cfg.prioritized || priorities || n == 1,
               "prioritized add needs priorities (NULL: one transition at the max recorded one)");
  hipStream_t s = (hipStream_t)stream;
  ReplayView v = h->view();
  if (h->cfg.prioritized) {  // _add: sum_tree.set(cursor, p) before the write (prb:139)
    // priorities NULL: p = SumTree.max_recorded_priority as the set kernel finds it in the
    // control block (float64, as rainbow_agent.py:331 reads it), no host round trip
    SetArgs a{nullptr, priorities, n, priorities ? nullptr : &h->st.meta->max_recorded_priority};
    hipLaunchKernelGGL(k_sumtree_set, dim3(1), dim3(kTreeT), 0, s, v, a);
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
  DQ_CHECK_ARG(!h->tree_only, "a standalone sum tree has no transition store");
  DQ_CHECK_ARG(batch >= 1 && batch <= kMaxBatch, "batch must be in [1, 1024]");
  DQ_CHECK_ARG(h->st.tape, "RNG tape not attached");
  hipStream_t s = (hipStream_t)stream;
  if (h->cfg.prioritized)
    hipLaunchKernelGGL(k_per_sample, dim3(1), dim3(kTreeT), 0, s, h->view(), batch, indices_out);
  else
    hipLaunchKernelGGL(k_uniform_sample, dim3(1), dim3(64), 0, s, h->view(), batch, indices_out, 1);
  DQ_CHECK_LAUNCH("sample_indices");
  return DQ_OK;
}

int dq_replay_sample_indices_groups(dq_replay* h, int32_t batch, int32_t groups,
                                    int32_t* indices_out, void* stream) {
  DQ_CHECK_ARG(h && indices_out, "null argument");
  DQ_CHECK_ARG(!h->tree_only, "a standalone sum tree has no transition store");
  DQ_CHECK_ARG(!h->cfg.prioritized, "grouped sampling needs a uniform buffer (a prioritized "
               "draw depends on the previous batch's priorities)");
  DQ_CHECK_ARG(batch >= 1 && groups >= 1 && (int64_t)batch * groups <= kMaxBatch,
               "batch * groups must be in [1, 1024]");
  DQ_CHECK_ARG(h->st.tape, "RNG tape not attached");
  hipLaunchKernelGGL(k_uniform_sample, dim3(1), dim3(64), 0, (hipStream_t)stream, h->view(), batch,
                     indices_out, groups);
  DQ_CHECK_LAUNCH("sample_indices_groups");
  return DQ_OK;
}

int dq_replay_gather(dq_replay* h, const int32_t* indices, int32_t batch, int32_t layout,
                     void* state_out, void* next_state_out, int32_t* action_out,
                     float* reward_out, int32_t* next_action_out, float* next_reward_out,
                     uint8_t* terminal_out, int32_t* indices_out, float* probs_out,
                     void* stream) {
  DQ_CHECK_ARG(h && indices && batch >= 1, "bad arguments");
  DQ_CHECK_ARG(!h->tree_only, "a standalone sum tree has no transition store");
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
    dim3 grid((unsigned)((nd + 256 * kNhwcR - 1) / (256 * kNhwcR) + 1), (unsigned)(2 * batch));
    hipLaunchKernelGGL(k_gather_nhwc4<kNhwcR>, grid, dim3(256), 0, s, h->view(), g);
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

int dq_replay_gather_elems(dq_replay* h, const int32_t* indices, int32_t batch,
                           const void* action_rows, int32_t action_bytes, const void* rewards,
                           int32_t reward_elems, int32_t reward_last, int32_t reward_dtype,
                           int32_t acc_f64, void* action_out, void* next_action_out,
                           void* reward_out, void* next_reward_out, void* stream) {
  DQ_CHECK_ARG(h && indices && batch >= 1, "bad arguments");
  DQ_CHECK_ARG(!h->tree_only, "a standalone sum tree has no transition store");
  DQ_CHECK_ARG(action_bytes >= 0 && (action_rows || action_bytes == 0 ||
                                     (!action_out && !next_action_out)), "bad action rows");
  DQ_CHECK_ARG(reward_elems >= 1 && reward_last >= 0 && reward_dtype >= DQ_DT_F32 &&
               reward_dtype <= DQ_DT_I64 && (rewards || (!reward_out && !next_reward_out)),
               "bad reward store");
  DQ_CHECK_ARG(reward_last == 0 || reward_elems % reward_last == 0,
               "reward_last must divide reward_elems");
  ElemArgs e{indices, (const uint8_t*)action_rows, action_bytes, rewards, reward_elems,
             reward_last, reward_dtype, acc_f64 ? 1 : 0, (uint8_t*)action_out,
             (uint8_t*)next_action_out, reward_out, next_reward_out};
  hipLaunchKernelGGL(k_gather_elems, dim3((unsigned)batch), dim3(256), 0, (hipStream_t)stream,
                     h->view(), e);
  DQ_CHECK_LAUNCH("k_gather_elems");
  return DQ_OK;
}

int dq_sumtree_set(dq_replay* h, const int32_t* indices, const float* priorities, int64_t n,
                   void* stream) {
  DQ_CHECK_ARG(h && h->cfg.prioritized, "sum tree needs a prioritized buffer");
  DQ_CHECK_ARG(indices && priorities && n >= 0, "bad arguments");
  DQ_CHECK_ARG(h->depth < 63, "tree too deep");
  if (n == 0) return DQ_OK;
  SetArgs a{indices, priorities, n};
  hipLaunchKernelGGL(k_sumtree_set, dim3(1), dim3(kTreeT), 0, (hipStream_t)stream, h->view(), a);
  DQ_CHECK_LAUNCH("k_sumtree_set");
  return DQ_OK;
}

int dq_sumtree_set_f64(dq_replay* h, const int32_t* indices, const double* values, int64_t n,
                       void* stream) {
  DQ_CHECK_ARG(h && h->cfg.prioritized, "sum tree needs a prioritized buffer");
  DQ_CHECK_ARG(indices && values && n >= 0, "bad arguments");
  DQ_CHECK_ARG(h->depth < 63, "tree too deep");
  if (n == 0) return DQ_OK;
  SetArgs a{indices, nullptr, n, values};
  hipLaunchKernelGGL(k_sumtree_set, dim3(1), dim3(kTreeT), 0, (hipStream_t)stream, h->view(), a);
  DQ_CHECK_LAUNCH("k_sumtree_set");
  return DQ_OK;
}

int dq_sumtree_sample(dq_replay* h, int32_t mode, int32_t n, const double* query_values,
                      int64_t* out, void* stream) {
  DQ_CHECK_ARG(h && h->cfg.prioritized && out, "bad arguments");
  DQ_CHECK_ARG(n >= 1 && n <= (1 << 20), "query count must be in [1, 2^20]");
  DQ_CHECK_ARG(mode == DQ_SUMTREE_QUERY || mode == DQ_SUMTREE_RANDOM ||
               mode == DQ_SUMTREE_STRATIFIED, "unknown sum-tree sample mode");
  DQ_CHECK_ARG(mode != DQ_SUMTREE_QUERY || query_values, "query mode needs query values");
  DQ_CHECK_ARG(mode == DQ_SUMTREE_QUERY || h->st.tape, "RNG tape not attached");
  DQ_CHECK_ARG(h->depth < 63, "tree too deep");
  hipLaunchKernelGGL(k_sumtree_sample, dim3(1), dim3(256), 0, (hipStream_t)stream, h->view(),
                     (int)mode, (int)n, query_values, out);
  DQ_CHECK_LAUNCH("k_sumtree_sample");
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

int dq_replay_egreedy(dq_replay* h, const float* q, int32_t num_actions, double epsilon,
                      int32_t* action_out, void* stream) {
  DQ_CHECK_ARG(h && q && action_out && num_actions >= 1, "bad arguments");
  DQ_CHECK_ARG(h->st.tape, "RNG tape not attached");
  hipLaunchKernelGGL(k_egreedy, dim3(1), dim3(1), 0, (hipStream_t)stream, h->st.meta,
                     (const uint32_t*)h->st.tape, q, num_actions, epsilon, action_out);
  DQ_CHECK_LAUNCH("k_egreedy");
  return DQ_OK;
}

int dq_replay_read_meta(dq_replay* h, dq_replay_meta* out, void* stream) {
  DQ_CHECK_ARG(h && out, "null argument");
  DQ_CHECK_HIP(hipMemcpyAsync(out, h->st.meta, sizeof(dq_replay_meta), hipMemcpyDeviceToHost,
                              (hipStream_t)stream));
  DQ_CHECK_HIP(hipStreamSynchronize((hipStream_t)stream));
  return DQ_OK;
}

int dq_replay_read_meta_async(dq_replay* h, dq_replay_meta* out, void* stream) {
  DQ_CHECK_ARG(h && out, "null argument");
  DQ_CHECK_HIP(hipMemcpyAsync(out, h->st.meta, sizeof(dq_replay_meta), hipMemcpyDeviceToHost,
                              (hipStream_t)stream));
  return DQ_OK;
}

static int record(dq_replay* h, RiderDesc& r, dq_rider* out) {
  DQ_CHECK_ARG(out, "null rider");
  r.v = h->view();
  memset(out, 0, sizeof(*out));
  memcpy(out, &r, sizeof(r));
  return DQ_OK;
}

int dq_replay_record_sumtree_set(dq_replay* h, const int32_t* indices, const float* priorities,
                                 int64_t n, dq_rider* out) {
  DQ_CHECK_ARG(h && h->cfg.prioritized, "sum tree needs a prioritized buffer");
  DQ_CHECK_ARG(indices && priorities && n >= 0, "bad arguments");
  DQ_CHECK_ARG(h->depth < 63, "tree too deep");
  RiderDesc r{};
  r.kind = n == 0 ? kRiderNone : kRiderSet;
  r.s = SetArgs{indices, priorities, n};
  return record(h, r, out);
}

int dq_replay_record_sample(dq_replay* h, int32_t batch, int32_t* indices_out, dq_rider* out) {
  DQ_CHECK_ARG(h && indices_out, "null argument");
  DQ_CHECK_ARG(!h->tree_only, "a standalone sum tree has no transition store");
  DQ_CHECK_ARG(batch >= 1 && batch <= kMaxBatch, "batch must be in [1, 1024]");
  DQ_CHECK_ARG(h->st.tape, "RNG tape not attached");
  RiderDesc r{};
  r.kind = h->cfg.prioritized ? kRiderPerSample : kRiderUniformSample;
  r.batch = batch;
  r.out = indices_out;
  return record(h, r, out);
}

int dq_replay_record_sample_groups(dq_replay* h, int32_t batch, int32_t groups,
                                   int32_t* indices_out, dq_rider* out) {
  DQ_CHECK_ARG(h && indices_out, "null argument");
  DQ_CHECK_ARG(!h->tree_only, "a standalone sum tree has no transition store");
  DQ_CHECK_ARG(!h->cfg.prioritized, "grouped sampling needs a uniform buffer");
  DQ_CHECK_ARG(batch >= 1 && groups >= 1 && (int64_t)batch * groups <= kMaxBatch,
               "batch * groups must be in [1, 1024]");
  DQ_CHECK_ARG(h->st.tape, "RNG tape not attached");
  RiderDesc r{};
  r.kind = kRiderUniformSample;
  r.batch = batch;
  r.groups = groups;
  r.out = indices_out;
  return record(h, r, out);
}

int dq_replay_record_gather_nhwc(dq_replay* h, const int32_t* indices, int32_t batch,
                                 float* state_out, float* next_state_out, int32_t* action_out,
                                 float* reward_out, int32_t* next_action_out,
                                 float* next_reward_out, uint8_t* terminal_out,
                                 int32_t* indices_out, float* probs_out, dq_rider* out) {
  DQ_CHECK_ARG(h && indices && batch >= 1 && batch <= kMaxBatch, "bad arguments");
  DQ_CHECK_ARG(!h->tree_only, "a standalone sum tree has no transition store");
  DQ_CHECK_ARG(!probs_out || h->cfg.prioritized, "probs requested from a uniform buffer");
  DQ_CHECK_ARG(h->cfg.obs_is_u8, "F32_NHWC layout needs uint8 observations");
  DQ_CHECK_ARG(h->cfg.stack_size == 4, "F32_NHWC layout needs stack_size == 4");
  DQ_CHECK_ARG((h->cfg.obs_bytes & 3) == 0, "F32_NHWC layout needs obs_bytes % 4 == 0");
  RiderDesc r{};
  r.kind = kRiderGatherNhwc;
  r.batch = batch;
  const int64_t nd = h->cfg.obs_bytes >> 2;
  r.gx = (int32_t)((nd + 256 * kNhwcR - 1) / (256 * kNhwcR));
  r.g = GatherOut{indices, state_out, next_state_out, action_out, reward_out, next_action_out,
                  next_reward_out, terminal_out, indices_out, probs_out};
  return record(h, r, out);
}

int dq_rider_chain(const dq_rider* first, const dq_rider* second, dq_rider* out) {
  DQ_CHECK_ARG(first && second && out, "null rider");
  RiderDesc a, b;
  memcpy(&a, first, sizeof(a));
  memcpy(&b, second, sizeof(b));
  DQ_CHECK_ARG(a.kind == kRiderSet && b.kind == kRiderPerSample,
               "dq_rider_chain chains a sum-tree write-back and a prioritized sample");
  DQ_CHECK_ARG(a.v.tree == b.v.tree && a.v.meta == b.v.meta, "riders of different buffers");
  RiderDesc r = b;
  r.kind = kRiderSetSample;
  r.s = a.s;
  memset(out, 0, sizeof(*out));
  memcpy(out, &r, sizeof(r));
  return DQ_OK;
}

int dq_sync_copy(void* dst, const void* src, int64_t bytes, void* stream) {
  DQ_CHECK_ARG(dst && src && bytes >= 0, "bad arguments");
  if (bytes == 0) return DQ_OK;
  DQ_CHECK_HIP(hipMemcpyAsync(dst, src, (size_t)bytes, hipMemcpyDeviceToDevice, (hipStream_t)stream));
  return DQ_OK;
}

}  // extern "C"
