/* dopamine_amd -- C ABI of the MI355X replay-sampling + Q-learning update path.
 *
 * The reference (K-Kielak/dopamine, TF1 + numpy) has no native ABI: its hot path
 * sits behind the out-of-graph Python replay API and the TF graph of the agents.
 * Each entry point below replaces one such Python/TF call; the reference
 * interface it stands in for is cited as path:line (relative to the reference
 * root).  Everything is plain C: opaque handles, raw pointers, sizes and an
 * `hipStream_t` passed as `void*`.  All device buffers are owned by the caller
 * (the Python host hands in torch allocations); the library never frees them.
 * Every call is asynchronous on the given stream and graph-capturable except
 * where noted "synchronous".
 *
 * Return values: 0 on success, negative DQ_E_* on a host-side argument/launch
 * error (text via dq_last_error()).  Errors the reference raises *during*
 * sampling (empty tree, max attempts, negative priority) are detected on the
 * device and latched into dq_replay_meta.status; the host raises them with the
 * reference's exception type and message at its next synchronisation point.
 */
#ifndef DOPAMINE_AMD_H
#define DOPAMINE_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DQ_ABI_VERSION 9

/* host-side return codes */
#define DQ_OK 0
#define DQ_E_ARG -1
#define DQ_E_HIP -2

/* device-latched status codes (dq_replay_meta.status) */
#define DQ_ST_OK 0
#define DQ_ST_EMPTY_TREE 1        /* sum_tree.py:116-117, 159-160 */
#define DQ_ST_MAX_ATTEMPTS 2      /* circular_replay_buffer.py:471-475, prioritized_replay_buffer.py:159-163 */
#define DQ_ST_TAPE_EXHAUSTED 3    /* RNG tape ran dry: host must refill before sampling */
#define DQ_ST_NEG_PRIORITY 4      /* sum_tree.py:191-193 */
#define DQ_ST_TOO_FEW 5           /* circular_replay_buffer.py:457-460 */
#define DQ_ST_BAD_INDEX 6         /* leaf index outside the tree (numpy IndexError in sum_tree.py:196) */
#define DQ_ST_BROADCAST 7         /* n-step reward: the (L,) discount vector does not broadcast
                                     against (L,) + reward_shape (numpy ValueError at
                                     circular_replay_buffer.py:540-541); status_arg = L,
                                     status_value = 1 if the sum's shape could not be assigned */

/* dq_sumtree_sample modes */
#define DQ_SUMTREE_QUERY 0        /* SumTree.sample(query_value) for given values (sum_tree.py:99-141) */
#define DQ_SUMTREE_RANDOM 1       /* SumTree.sample() with random.random() (sum_tree.py:123) */
#define DQ_SUMTREE_STRATIFIED 2   /* SumTree.stratified_sample(n) (sum_tree.py:143-166) */

/* gather output layouts */
#define DQ_LAYOUT_RAW 0           /* (B, stack, obs_bytes) bytes, stack-major (moveaxis on host = reference NHWC) */
#define DQ_LAYOUT_F32_NORM 1      /* (B, stack, H*W) float32 = uint8 / 255 (atari_lib.py:96-97), NCHW */
#define DQ_LAYOUT_F32_NHWC 2      /* (B, H*W, stack) float32 = uint8 / 255, the reference NHWC state (stack == 4) */

/* Device control block (caller allocates >= sizeof, 64-byte aligned). */
typedef struct dq_replay_meta {
  int64_t add_count;              /* circular_replay_buffer.py:177 */
  int64_t tape_pos;               /* RNG words consumed from the tape */
  int64_t tape_len;               /* RNG words valid on the tape */
  double max_recorded_priority;   /* sum_tree.py:89, 196 */
  int32_t status;                 /* DQ_ST_* (first error latched) */
  int32_t status_arg;             /* e.g. #valid indices sampled before failing */
  double status_value;            /* e.g. the negative priority */
  int64_t reserved[2];
} dq_replay_meta;

typedef struct dq_replay_config {
  int64_t capacity;               /* replay_capacity */
  int64_t obs_bytes;              /* bytes of one observation (84*84 for Atari) */
  int32_t stack_size;
  int32_t update_horizon;
  int32_t max_sample_attempts;
  int32_t prioritized;            /* 1: OutOfGraphPrioritizedReplayBuffer, 0: uniform */
  int32_t obs_is_u8;              /* enables DQ_LAYOUT_F32_NORM */
  int32_t pad_;
  double gamma;
} dq_replay_config;

typedef struct dq_replay_storage {   /* all device pointers, caller-owned */
  uint8_t* frames;                /* [capacity][obs_bytes]   _store['observation'] */
  int32_t* actions;               /* [capacity]              _store['action'] */
  float* rewards;                 /* [capacity]              _store['reward'] */
  uint8_t* terminals;             /* [capacity]              _store['terminal'] */
  double* tree;                   /* [2^(depth+1)-1] heap of SumTree.nodes, or NULL (uniform) */
  dq_replay_meta* meta;           /* control block */
  uint32_t* tape;                 /* [tape_capacity] raw MT19937 words continuing the host stream */
  int64_t tape_capacity;
  float* discount;                /* [update_horizon] float32(gamma^k) (circular_replay_buffer.py:181-183) */
} dq_replay_storage;

typedef struct dq_replay dq_replay;

int dq_abi_version(void);
/* the extra -D flags the library was compiled with: "" for the product build, the bf16
   throughput build's flags for libdopamine_amd_bf16.so (dopamine_amd/_lib.py refuses any
   other build unless DQ_DIAGNOSTIC_BUILD=1 is set, e.g. by a tools/ stamp run) */
const char* dq_build_flags(void);
const char* dq_last_error(void);
/* depth of the sum tree for a capacity: ceil(log2(capacity)) (sum_tree.py:80) */
int dq_sumtree_depth(int64_t capacity);

/* OutOfGraphReplayBuffer.__init__ (circular_replay_buffer.py:98-183) /
 * OutOfGraphPrioritizedReplayBuffer.__init__ (prioritized_replay_buffer.py:43-97). */
int dq_replay_create(const dq_replay_config* cfg, const dq_replay_storage* st, dq_replay** out);
int dq_replay_destroy(dq_replay* h);
/* SumTree.__init__ (sum_tree.py:65-89) as a standalone object: a handle over a caller-owned
 * float64 heap of 2^(depth+1)-1 nodes, depth = ceil(log2 capacity) (0 for capacity 1),
 * a control block and an optional RNG tape.  Valid with dq_sumtree_set[_f64]/get/sample/
 * rebuild, dq_replay_set_meta/set_tape/read_meta and dq_replay_destroy; the transition
 * calls (add, sample_indices, gather, riders) reject it. */
int dq_sumtree_create(int64_t capacity, double* tree, dq_replay_meta* meta, uint32_t* tape,
                      int64_t tape_capacity, dq_replay** out);

/* add() / _add() for n consecutive transitions at the cursor
 * (circular_replay_buffer.py:234-287, prioritized_replay_buffer.py:117-140).
 * Inputs are device arrays; priorities NULL for the uniform buffer, or, for the
 * prioritized one with n == 1, "the maximum priority recorded so far" read on the device
 * (rainbow_agent.py:326-335: SumTree.max_recorded_priority as float64).  Padding
 * (zero transitions) is decided by the host, which passes them explicitly. */
int dq_replay_add(dq_replay* h, int64_t n, const uint8_t* frames, const int32_t* actions,
                  const float* rewards, const uint8_t* terminals, const float* priorities,
                  void* stream);

/* sample_index_batch (uniform: circular_replay_buffer.py:436-477 with
 * np.random.randint; prioritized: prioritized_replay_buffer.py:142-171 with
 * SumTree.stratified_sample / sample, sum_tree.py:99-166).  Random numbers come
 * from the device RNG tape; exact draw-for-draw equivalent of the reference. */
int dq_replay_sample_indices(dq_replay* h, int32_t batch, int32_t* indices_out, void* stream);
/* `groups` consecutive uniform sample_index_batch(batch) calls (crb:436-477) in one launch,
 * indices_out[g * batch + i]: the same draws, RNG words and per-call max-attempts budgets and
 * errors as the calls in a row (the first failing batch latches its error).  The rewind
 * cursor is the last batch's, so dq_replay_rewind_last_sample gives back that batch only.
 * Uniform buffers only (a prioritized draw depends on the previous batch's write-back). */
int dq_replay_sample_indices_groups(dq_replay* h, int32_t batch, int32_t groups,
                                    int32_t* indices_out, void* stream);

/* sample_transition_batch given indices (circular_replay_buffer.py:479-558 +
 * prioritized_replay_buffer.py:173-201).  Any output pointer may be NULL. */
int dq_replay_gather(dq_replay* h, const int32_t* indices, int32_t batch, int32_t layout,
                     void* state_out, void* next_state_out, int32_t* action_out,
                     float* reward_out, int32_t* next_action_out, float* next_reward_out,
                     uint8_t* terminal_out, int32_t* indices_out, float* probs_out,
                     void* stream);

/* The action / reward elements of a transition batch for buffers whose action or reward
 * is not a scalar int32 / float32 (action_shape, action_dtype, reward_shape, reward_dtype of
 * circular_replay_buffer.py:96-183; the sampling at :530-548).  Per sample b with
 * idx = indices[b] and L its n-step length (the terminal store, crb:517-526):
 *   action_out[b] = action_rows[idx], next_action_out[b] = action_rows[(idx + L) % C]
 *     (action_bytes-byte rows, copied as they are);
 *   reward_out[b] = sum over i < L of disc * rewards[(idx + i) % C], numpy's
 *     np.sum(discount[:L] * trajectory_rewards, axis=0): the (L,) float32 discount vector
 *     broadcasts against the LAST axis of (L,) + reward_shape (reward_last = its size, 0 for
 *     a scalar reward), products and the left-to-right sum in float64 when acc_f64 (numpy's
 *     float32 x reward_dtype promotion) else float32, then cast to reward_dtype;
 *   next_reward_out[b] = rewards[(idx + L) % C].
 * reward_dtype: DQ_DT_*; reward_elems = prod(reward_shape).  A sample whose L does not
 * broadcast latches DQ_ST_BROADCAST.  Any output pointer may be NULL. */
#define DQ_DT_F32 0
#define DQ_DT_F64 1
#define DQ_DT_F16 2
#define DQ_DT_I8 3
#define DQ_DT_U8 4
#define DQ_DT_I16 5
#define DQ_DT_I32 6
#define DQ_DT_I64 7
int dq_replay_gather_elems(dq_replay* h, const int32_t* indices, int32_t batch,
                           const void* action_rows, int32_t action_bytes, const void* rewards,
                           int32_t reward_elems, int32_t reward_last, int32_t reward_dtype,
                           int32_t acc_f64, void* action_out, void* next_action_out,
                           void* reward_out, void* next_reward_out, void* stream);

/* set_priority (prioritized_replay_buffer.py:203-214 -> sum_tree.py:178-205):
 * ordered, delta-propagating float64 updates, duplicates honoured. */
int dq_sumtree_set(dq_replay* h, const int32_t* indices, const float* priorities, int64_t n,
                   void* stream);
/* SumTree.set with float64 values (sum_tree.py:178-205; a standalone tree is
 * set with Python floats, not the buffer's float32 priorities). */
int dq_sumtree_set_f64(dq_replay* h, const int32_t* indices, const double* values, int64_t n,
                       void* stream);
/* SumTree.sample(query_value) / sample() / stratified_sample(n) (sum_tree.py:99-166):
 * n leaf indices into out (int64).  RANDOM / STRATIFIED consume 2n tape words (the
 * Python `random` stream: random.random() per sample, random.uniform per stratum).
 * An empty tree latches DQ_ST_EMPTY_TREE (sum_tree.py:116-117, 159-160); the
 * query_value range check (sum_tree.py:119-120) is the host's. */
int dq_sumtree_sample(dq_replay* h, int32_t mode, int32_t n, const double* query_values,
                      int64_t* out, void* stream);
/* get_priority (prioritized_replay_buffer.py:216-235). */
int dq_sumtree_get(dq_replay* h, const int32_t* indices, int64_t n, float* out, void* stream);
/* Bulk (re)build of internal nodes from the leaves (parents = sum of children).
 * Used for synthetic fills and checkpoint restore of the leaves only. */
int dq_sumtree_rebuild(dq_replay* h, void* stream);

/* Host <-> control block.  `set_meta` writes add_count / max_rec, clears status. */
int dq_replay_set_meta(dq_replay* h, int64_t add_count, double max_recorded_priority, void* stream);
/* Declare `len` fresh words on the tape (caller has copied them in); pos := 0. */
int dq_replay_set_tape(dq_replay* h, int64_t len, void* stream);
/* Undo the RNG-tape consumption of the most recent dq_replay_sample_indices call
 * (its indices must then be discarded).  Lets a speculatively prefetched batch be
 * redrawn when transitions were added or the host stream was used in between, so
 * the draw order stays the reference's. */
int dq_replay_rewind_last_sample(dq_replay* h, void* stream);
/* _select_action (dqn_agent.py:394-416) on the device for a buffer whose sampler draws from
   Python's `random` (the prioritized one): the epsilon test random.random() <= epsilon and
   the explore draw random.randint(0, num_actions - 1) consume the tape's next words exactly
   as CPython would (genrand_res53; _randbelow by getrandbits(bit_length) rejection), else
   the first argmax of q (num_actions floats, device); *action_out (device) = the action, or
   -1 if the tape ran out (nothing consumed: sync and draw on the host). */
int dq_replay_egreedy(dq_replay* h, const float* q, int32_t num_actions, double epsilon,
                      int32_t* action_out, void* stream);
/* synchronous: copies the control block to host memory. */
int dq_replay_read_meta(dq_replay* h, dq_replay_meta* out, void* stream);
/* the same copy, stream-ordered and NOT waited for: `out` must be pinned host memory and is
   valid once the stream reaches this point (e.g. an event recorded after the call). */
int dq_replay_read_meta_async(dq_replay* h, dq_replay_meta* out, void* stream);

/* Recorded replay operations ("riders").  Instead of launching, these fill an
 * opaque descriptor with exactly the work the matching call above would launch
 * (same device code, same arguments); dq_cnn_backward_riders then runs rider i
 * as extra blocks of its i-th grouped launch, so the next batch's priority
 * write-back -> sample -> gather chain rides inside the backward on ONE stream
 * (kernel boundaries keep the chain ordered).  Same semantics as
 * dq_sumtree_set / dq_replay_sample_indices / dq_replay_gather(DQ_LAYOUT_F32_NHWC). */
typedef struct dq_rider {
  int64_t words[40];              /* opaque */
} dq_rider;
int dq_replay_record_sumtree_set(dq_replay* h, const int32_t* indices, const float* priorities,
                                 int64_t n, dq_rider* out);
int dq_replay_record_sample(dq_replay* h, int32_t batch, int32_t* indices_out, dq_rider* out);
int dq_replay_record_sample_groups(dq_replay* h, int32_t batch, int32_t groups,
                                   int32_t* indices_out, dq_rider* out);
int dq_replay_record_gather_nhwc(dq_replay* h, const int32_t* indices, int32_t batch,
                                 float* state_out, float* next_state_out, int32_t* action_out,
                                 float* reward_out, int32_t* next_action_out,
                                 float* next_reward_out, uint8_t* terminal_out,
                                 int32_t* indices_out, float* probs_out, dq_rider* out);
/* One rider running `first` (a dq_replay_record_sumtree_set) and then `second` (a
 * prioritized dq_replay_record_sample of the same buffer) in ONE block: the write-back
 * (prioritized_replay_buffer.py:203-214) and the next stratified draw (:142-171) in their
 * reference order, one launch instead of two. */
int dq_rider_chain(const dq_rider* first, const dq_rider* second, dq_rider* out);

/* ---------------- learner-side kernels (stateless) ---------------- */

/* Rainbow/C51 target distribution + projection + softmax cross-entropy + PER
 * weights + new priorities (rainbow_agent.py:200-305, project_distribution
 * rainbow_agent.py:340-494).  Logits (B, A, N) float32.  grad_logits (B,A,N) is
 * fully written: d mean(w * loss) / d online_logits (TF CE backprop
 * softmax - labels).  probs NULL => replay_scheme 'uniform' (weights 1).
 * loss_out/priorities_out (B,), mean_loss_out (1,): may be NULL. */
int dq_c51_loss(const float* online_logits, const float* target_logits, const int32_t* actions,
                const float* rewards, const uint8_t* terminals, const float* probs,
                const float* support, int32_t batch, int32_t num_actions, int32_t num_atoms,
                float cumulative_gamma, float* grad_logits, float* loss_out,
                float* priorities_out, float* mean_loss_out, void* stream);

/* The online half of dq_c51_loss_fused (rainbow_agent.py:253-305: softmax cross-entropy of
   the chosen online logits against the projected target distribution, PER weights, new
   priorities, dlogits and d h) given target_m (B, num_atoms) from dq_cnn_forward_fused_c51;
   loss, gradient, priorities and d h are bitwise dq_c51_loss_fused's. */
int dq_c51_loss_online(const float* online_parts, const float* online_bias, int32_t n_parts,
                       const float* target_m, const int32_t* actions, const float* probs,
                       int32_t batch, int32_t num_actions, int32_t num_atoms, float* grad_logits,
                       float* loss_out, float* priorities_out, const float* fc2_w, const float* h,
                       float* dh, int32_t hidden, float* online_logits_out, void* stream);

/* dq_c51_loss on the CNN's fc2 k-band partials (dq_cnn_forward_fused): logits = the n_parts
   partial slabs [n_parts][B][A*N] summed in order + bias (bitwise dq_cnn_forward's logits,
   written to *_logits_out when non-NULL); with fc2_w set it also writes the fc2 input
   gradient dh = (grad_logits . fc2_w) * (h > 0), (B, hidden), so the CNN backward can start
   at its launch 1.  The mean-loss summary is not produced here. */
int dq_c51_loss_fused(const float* online_parts, const float* online_bias,
                      const float* target_parts, const float* target_bias, int32_t n_parts,
                      const int32_t* actions, const float* rewards, const uint8_t* terminals,
                      const float* probs, const float* support, int32_t batch,
                      int32_t num_actions, int32_t num_atoms, float cumulative_gamma,
                      float* grad_logits, float* loss_out, float* priorities_out,
                      const float* fc2_w, const float* h, float* dh, int32_t hidden,
                      float* online_logits_out, float* target_logits_out, void* stream);
/* DQN Bellman max target + Huber(delta=1) (dqn_agent.py:283-322). */
int dq_dqn_huber_loss(const float* online_q, const float* target_q, const int32_t* actions,
                      const float* rewards, const uint8_t* terminals, int32_t batch,
                      int32_t num_actions, float cumulative_gamma, float* grad_q,
                      float* loss_out, float* mean_loss_out, void* stream);
/* dq_dqn_huber_loss on the CNN's fc2 k-band partials (dq_cnn_forward_fused), the DQN fast
   path (dqn_agent.py:283-322): Q / Q' = the n_parts partial slabs [n_parts][B][A] summed in
   order + bias (bitwise dq_cnn_forward's outputs, written to *_q_out when non-NULL); target,
   loss and gradient bitwise dq_dqn_huber_loss's; also writes the fc2 input gradient
   dh = (grad_q . fc2_w) * (h > 0), (B, hidden), bitwise the backward's launch 0, so the CNN
   backward starts at its launch 1.  num_actions <= 64, hidden <= 512 and a multiple of 4.
   The mean-loss summary is not produced here. */
int dq_dqn_huber_loss_fused(const float* online_parts, const float* online_bias,
                            const float* target_parts, const float* target_bias, int32_t n_parts,
                            const int32_t* actions, const float* rewards,
                            const uint8_t* terminals, int32_t batch, int32_t num_actions,
                            float cumulative_gamma, float* grad_q, float* loss_out,
                            const float* fc2_w, const float* h, float* dh, int32_t hidden,
                            float* online_q_out, float* target_q_out, void* stream);

/* IQN quantile-Huber loss (implicit_quantile_agent.py:190-321).  Row order of
 * the tiled tensors is q*B + b (atari_lib.py:174).  grad (N*B, A) fully written. */
int dq_iqn_loss(const float* online_qv, const float* target_qv, const float* target_qv_action,
                const float* taus, const int32_t* actions, const float* rewards,
                const uint8_t* terminals, int32_t batch, int32_t num_actions,
                int32_t num_tau, int32_t num_tau_prime, int32_t num_quantile,
                float cumulative_gamma, float kappa, float* grad_qv, float* loss_out,
                float* mean_loss_out, void* stream);

/* tf.train.AdamOptimizer.apply_gradients over ONE flat fp32 parameter buffer.
 * state = {beta1_power, beta2_power}[2] (float32, device; slot 0 initialised to
 * {beta1, beta2}); step t reads slot t%2 and writes beta^(t+1) into the other. */
int dq_adam_tf1(float* var, const float* grad, float* m, float* v, float* state, int32_t slot,
                int64_t n, float lr, float beta1, float beta2, float eps, void* stream);

/* The same update over up to DQ_MAX_TENSORS separately allocated tensors in ONE
 * launch (e.g. autograd's per-parameter gradients; no flat-gradient copy). */
#define DQ_MAX_TENSORS 16
/* dq_adam_tf1 over one part [var, var + n) of the parameters: a step may be split into
   parts (e.g. each all-reduce bucket as soon as it lands); every part reads the beta powers
   of slot `slot`, and exactly one part per step passes bump = 1 to advance them. */
int dq_adam_tf1_part(float* var, const float* grad, float* m, float* v, float* state,
                     int32_t slot, int64_t n, float lr, float beta1, float beta2, float eps,
                     int32_t bump, void* stream);
typedef struct dq_tensor_list {
  int32_t count;
  int32_t pad_;
  float* var[DQ_MAX_TENSORS];
  const float* grad[DQ_MAX_TENSORS];
  float* m[DQ_MAX_TENSORS];
  float* v[DQ_MAX_TENSORS];
  int64_t n[DQ_MAX_TENSORS];
} dq_tensor_list;
int dq_adam_tf1_multi(const dq_tensor_list* tensors, float* state, int32_t slot, float lr,
                      float beta1, float beta2, float eps, void* stream);

/* tf.train.RMSPropOptimizer(centered=True) (dqn_agent.py:100-105; rms init 1). */
int dq_rmsprop_tf1(float* var, const float* grad, float* ms, float* mg, float* mom, int64_t n,
                   float lr, float decay, float momentum, float eps, int32_t centered,
                   void* stream);

/* ---------------- Nature-CNN (atari_lib.py:85-144) on fp32 MFMA ----------------
 * Input x: (B, 84, 84, 4) NHWC float32 (the gather's DQ_LAYOUT_F32_NHWC).  Weights
 * are views into the flat parameter buffer: conv (out, kh, kw, in), FC (out, in).
 * Activations NHWC; the 7744 flatten is TF's (h, w, c) order. */
typedef struct dq_cnn_params {
  int32_t in_channels;            /* stack size, 4 */
  int32_t n_out;                  /* num_actions (DQN) or num_actions * num_atoms (C51) */
  float* conv1_w; float* conv1_b; /* (32, 8, 8, 4), (32) */
  float* conv2_w; float* conv2_b; /* (64, 4, 4, 32), (64) */
  float* conv3_w; float* conv3_b; /* (64, 3, 3, 64), (64) */
  float* fc1_w; float* fc1_b;     /* (512, 7744), (512) */
  float* fc2_w; float* fc2_b;     /* (n_out, 512), (n_out) */
} dq_cnn_params;
typedef struct dq_cnn_acts {      /* per-call activations (or their gradients) */
  float* a1;                      /* (B, 21, 21, 32) */
  float* a2;                      /* (B, 11, 11, 64) */
  float* a3;                      /* (B, 7744) */
  float* h;                       /* (B, 512) */
  float* out;                     /* (B, n_out) */
} dq_cnn_acts;
/* forward: relu(conv1..3), relu(fc1), fc2 -> a->out.  ws: dq_cnn_workspace_floats() floats
   (split-K slabs); one ws per stream that runs the network concurrently. */
int dq_cnn_forward(const dq_cnn_params* p, int32_t batch, const float* x, dq_cnn_acts* a,
                   float* ws, void* stream);
/* backward from d out (B, n_out): writes EVERY weight/bias gradient into g (plain stores,
 * no accumulation); d holds the intermediate activation gradients. */
/* two forwards in one pass (the online net on s and the target net on s', say): the same
   results as two dq_cnn_forward calls, bit for bit, in half the launches. */
int dq_cnn_forward_pair(const dq_cnn_params* p0, const float* x0, dq_cnn_acts* a0, float* ws0,
                        const dq_cnn_params* p1, const float* x1, dq_cnn_acts* a1, float* ws1,
                        int32_t batch, void* stream);
int dq_cnn_backward(const dq_cnn_params* p, const dq_cnn_params* g, int32_t batch, const float* x,
                    const dq_cnn_acts* a, const float* dout, dq_cnn_acts* d, float* ws,
                    void* stream);
/* The optimizer applied inside the backward's grouped launches: TF1 Adam (as dq_adam_tf1,
   kind DQ_OPT_ADAM -- a zero-initialised tail) or TF1 RMSProp (as dq_rmsprop_tf1, kind
   DQ_OPT_RMSPROP: the gin-bound optimizer of dqn.gin:19-25). */
#define DQ_OPT_ADAM 0
#define DQ_OPT_RMSPROP 1
typedef struct dq_adam_args {
  float* var;        /* flat parameter buffer the dq_cnn_params pointers point into */
  float* m;          /* Adam: moments, same layout as var; RMSProp: m = ms (the rms slot), */
  float* v;          /*   v = mom (the momentum slot) */
  float* state;      /* Adam: {beta1^t, beta2^t} x 2 slots, as dq_adam_tf1 */
  int32_t slot;      /* Adam: step parity: reads state slot, writes the other */
  float lr, beta1, beta2, epsilon;
  int32_t kind;      /* DQ_OPT_ADAM / DQ_OPT_RMSPROP */
  int32_t centered;  /* RMSProp: ApplyCenteredRMSProp (reads / writes mg) */
  float* mg;         /* RMSProp, centered: the mean-gradient slot, same layout as var */
  float decay, momentum;   /* RMSProp: rho, mu */
  int32_t no_grad_store;   /* 1: where the update is fused into a gradient epilogue, the
                              gradient is consumed in registers and not written to g (the
                              parameters and moments come out bitwise the same); 0: write it */
} dq_adam_args;
/* backward + optimizer step in one pass (single-replica training: no gradient
   all-reduce between them).  Gradients are written to g unless opt->no_grad_store = 1, in
   which case the updates fused into gradient epilogues consume them in registers and those
   ranges of g are left unwritten (parameters and moments bitwise the same either way). */
int dq_cnn_backward_adam(const dq_cnn_params* p, const dq_cnn_params* g, int32_t batch,
                         const float* x, const dq_cnn_acts* a, const float* dout, dq_cnn_acts* d,
                         float* ws, const dq_adam_args* opt, void* stream);
/* launches [first, last) of dq_cnn_backward's 7 grouped launches (the full call is [0, 7)):
   after launch 3 the fc1 / fc2 weight gradients are final, so a data-parallel learner can
   start their all-reduce while launches 3..6 run.  Bitwise the same results. */
int dq_cnn_backward_groups(const dq_cnn_params* p, const dq_cnn_params* g, int32_t batch,
                           const float* x, const dq_cnn_acts* a, const float* dout,
                           dq_cnn_acts* d, float* ws, int32_t first, int32_t last, void* stream);
/* A network's forward split in two, so the head can run where it is cheapest:
   head = conv1..conv3 and fc1's split-K partial sums (into ws), tail = their sum
   (+ bias, ReLU) and fc2.  head followed by tail == dq_cnn_forward, bit for bit. */
typedef struct dq_cnn_net {
  const dq_cnn_params* p;
  const float* x;
  dq_cnn_acts* a;
  float* ws;
} dq_cnn_net;
int dq_cnn_forward_head(const dq_cnn_params* p, int32_t batch, const float* x, dq_cnn_acts* a,
                        float* ws, void* stream);
/* net 0's whole forward, with net 1's tail (its head already run into a1 / ws1) in net 0's
   last two launches. */
int dq_cnn_forward_with_tail(const dq_cnn_params* p0, const float* x0, dq_cnn_acts* a0, float* ws0,
                             const dq_cnn_params* p1, dq_cnn_acts* a1, float* ws1, int32_t batch,
                             void* stream);
/* dq_cnn_backward (opt NULL) or dq_cnn_backward_adam (opt set) with riders[i] (recorded by
   dq_replay_record_*) as extra blocks of grouped launch i, i < n_riders <= 7: a chain of
   riders runs in order, each after the launches before its own.  Riders must not touch
   x, a, dout, d, g or ws.  head (may be NULL): another network's forward head (e.g. the
   target network on the next batch, which riders gathered) runs in launches 4..7
   (head_from = 3: conv1..conv3 + fc1 slabs) or 5..7 (head_from = 4: conv1..conv3, the fc1
   slabs then run in dq_cnn_forward_fused).  head_from = 5 selects the five-launch backward
   (launches 0..5; conv2's input gradient by sub-pixel class, the split-K sums of conv2 and
   conv1 both in launch 5) with the head's conv1 / conv2 in launches 4 / 5 and its conv3
   and fc1 slabs left to dq_cnn_forward_fused (fc1_1 = 3); head_from = 6: the head's conv1 in
   launch 5 only, its conv2 too left to dq_cnn_forward_fused (fc1_1 = 19, the Rainbow agent's
   default); 7: no head here at all (fc1_1 = 51 with x1 = the head's input).  Rider i rides in launch first + i.  Only
   launches [first, last) are issued (as dq_cnn_backward_groups; riders and head ops of
   other launches are skipped; opt needs [0, 7)).  CNN results are bitwise those of the
   separate calls. */
int dq_cnn_backward_riders(const dq_cnn_params* p, const dq_cnn_params* g, int32_t batch,
                           const float* x, const dq_cnn_acts* a, const float* dout,
                           dq_cnn_acts* d, float* ws, const dq_rider* riders, int32_t n_riders,
                           const dq_adam_args* opt, const dq_cnn_net* head, int32_t head_from,
                           int32_t first, int32_t last, void* stream);
/* The Rainbow fast path (rainbow_agent.py:200-305 on the Nature CNN, one launch less in
   the forward and one in the backward than dq_cnn_forward_with_tail + dq_c51_loss +
   dq_cnn_backward_riders(first 0)):
   dq_cnn_forward_fused: net 0 (online) conv1..fc1 and net 1's (target's) fc1 slabs (if fc1_1
   bit 0; its conv1..conv3 ran earlier, e.g. as head_from = 4 riders of the previous backward;
   with bit 1 its conv3 runs here too, in net 0's conv3 launch: head_from = 5; bit 4 (16): its
   conv2 in net 0's conv2 launch (head_from = 6); bit 5 (32): its conv1 on x1 in net 0's conv1
   launch (head_from = 7; x1 may be NULL otherwise); bit 2: only the
   three conv launches, bit 3: only the fc launches -- a data-parallel learner waits for the
   previous step's fc update in between), then
   ONE launch that sums both nets' fc1 slabs (+ bias, ReLU -> a->h) and stores fc2's 16 k-band
   partial products at ws + dq_cnn_fc2_parts_offset(batch) ([16][B][n_out]).  The logits are
   never stored by the CNN: dq_c51_loss_fused sums the partials in band order and adds the
   bias -- bit for bit the logits of dq_cnn_forward.  The backward then starts at launch 1
   (dq_cnn_backward_riders with first = 1, riders numbered from it): dq_c51_loss_fused also
   writes d h. */
int dq_cnn_forward_fused(const dq_cnn_params* p0, const float* x0, dq_cnn_acts* a0, float* ws0,
                         const dq_cnn_params* p1, const float* x1, dq_cnn_acts* a1, float* ws1,
                         int32_t batch, int32_t fc1_1, void* stream);
size_t dq_cnn_fc2_parts_offset(int32_t batch);
/* The target network's half of the C51 loss (rainbow_agent.py:200-251 target softmax, Q,
   greedy action, and project_distribution rainbow_agent.py:340-494) for the fused path. */
typedef struct dq_c51_target {
  const float* rewards;            /* (B,) n-step rewards of the batch */
  const uint8_t* terminals;        /* (B,) */
  const float* support;            /* (num_atoms,) linspace(-vmax, vmax) */
  int32_t num_atoms;
  float cumulative_gamma;          /* gamma^n as float32 (dqn_agent.py:175) */
  float* m_out;                    /* (B, num_atoms) projected target distribution */
  float* target_logits_out;        /* (B, n_out) or NULL */
} dq_c51_target;
/* dq_cnn_forward_fused with the target network one launch earlier (head_from = 8: its
   conv1 rode in launch 5 of the previous backward, as for head_from = 6): net 1's conv2 in
   net 0's conv1 launch, its conv3 in net 0's conv2 launch, its fc1 slabs in net 0's conv3
   launch, its fused head in net 0's fc1 launch, and the target half of the C51 loss (one
   block per sample) in net 0's fused-head launch -- the loss launch then runs only the
   online half (dq_c51_loss_online), off the critical path's target chain.  flags: bit 2
   only the conv launches, bit 3 only the fc launches (as dq_cnn_forward_fused).
   num_actions = p1->n_out / num_atoms <= 16.  m_out is bitwise what dq_c51_loss_fused
   forms internally. */
int dq_cnn_forward_fused_c51(const dq_cnn_params* p0, const float* x0, dq_cnn_acts* a0, float* ws0,
                             const dq_cnn_params* p1, dq_cnn_acts* a1, float* ws1, int32_t batch,
                             const dq_c51_target* c51, int32_t flags, void* stream);
/* one layer of the backward: layer 0..4 = fc2, fc1, conv3, conv2, conv1; part 1 = weight and
   bias gradient, part 0 = input gradient (not for conv1).  dW(L) depends only on dX(L-1),
   so the weight gradients may run on a second stream, each with its own ws. */
int dq_cnn_backward_layer(const dq_cnn_params* p, const dq_cnn_params* g, int32_t batch,
                          const float* x, const dq_cnn_acts* a, const float* dout, dq_cnn_acts* d,
                          float* ws, int32_t layer, int32_t part, void* stream);
size_t dq_cnn_workspace_floats(int32_t batch, int32_t n_out);
/* The Nature-CNN torso alone (conv1..conv3 + ReLU -> a->a3, the (B, 7744) state vector of
   atari_lib.py:98-101), the trunk of ImplicitQuantileNetwork; and its backward from
   d->a3 = d loss / d (conv3 pre-activation) (already masked by a3 > 0) into the conv
   weight / bias gradients of g.  Same tiles as the full forward / backward. */
int dq_cnn_forward_torso(const dq_cnn_params* p, int32_t batch, const float* x, dq_cnn_acts* a,
                         float* ws, void* stream);
int dq_cnn_backward_torso(const dq_cnn_params* p, const dq_cnn_params* g, int32_t batch,
                          const float* x, const dq_cnn_acts* a, dq_cnn_acts* d, float* ws,
                          void* stream);
/* dq_cnn_backward_torso + the whole network's optimizer step (ABI 6; IQN's single-replica
   learner: the head's gradients are already final in g): TF1 Adam / RMSProp (opt->kind) on
   [head_begin, head_end) -- the parameters after the torso in opt->var, e.g. IQN's quantile
   head -- and on conv3 as float4 riders of the torso's launches, conv2 and conv1 in their
   split-K sums' epilogues (conv1's advances Adam's beta powers).  Parameters, moments and
   gradients bitwise those of dq_cnn_backward_torso followed by dq_adam_tf1 / dq_rmsprop_tf1
   over the whole buffer (replaces the separate optimizer launch of dqn:322 / iqn:321). */
int dq_cnn_backward_torso_opt(const dq_cnn_params* p, const dq_cnn_params* g, int32_t batch,
                              const float* x, const dq_cnn_acts* a, dq_cnn_acts* d, float* ws,
                              const dq_adam_args* opt, float* head_begin, float* head_end,
                              void* stream);

/* ImplicitQuantileNetwork's quantile head (atari_lib.py:147-199) on the fp32 matrix cores.
   R = nq * batch rows ordered q * batch + b (tf.tile, atari_lib.py:174). */
typedef struct dq_iqn_head {
  int32_t embed_dim;              /* quantile_embedding_dim (multiple of 4; 64) */
  int32_t num_actions;
  float* emb_w; float* emb_b;     /* (7744, E), (7744) */
  float* fc1_w; float* fc1_b;     /* (512, 7744), (512) */
  float* fc2_w; float* fc2_b;     /* (A, 512), (A) */
} dq_iqn_head;
typedef struct dq_iqn_acts {
  float* cos;                     /* (R, E)    cos(pi * i * tau), i = 1..E   (atari_lib.py:176-178) */
  float* emb;                     /* (R, 7744) relu(cos We^T + be), kept for the backward; may be NULL */
  float* x;                       /* (R, 7744) tiled state * emb             (atari_lib.py:185);
                                     NULL with emb given: formed from emb and state by the FC1
                                     forward / dW1 operand loaders (never stored) */
  float* h;                       /* (R, 512)  relu(x W1^T + b1) */
  float* q;                       /* (R, A)    quantile values              (atari_lib.py:189-191) */
} dq_iqn_acts;
typedef struct dq_iqn_grads {
  float* dh;                      /* (R, 512) */
  float* dpre;                    /* (R, 7744) d loss / d (cos We^T + be) */
  float* dtl;                     /* (R, 7744) d loss / d tiled state */
} dq_iqn_grads;
/* forward: state = the torso's (B, 7744) output, taus (R). ws: dq_iqn_workspace_floats.
   taus NULL: a->cos already holds the cosine embedding (dq_iqn_tau_cos). */
int dq_iqn_head_forward(const dq_iqn_head* hp, int32_t batch, int32_t nq, const float* state,
                        const float* taus, dq_iqn_acts* a, float* ws, void* stream);
/* backward from dq = d loss / d q (R, A) (dq_iqn_loss): head weight / bias gradients into hg,
   dstate (B, 7744) = the torso's d->a3 for dq_cnn_backward_torso (tile sum, ReLU mask). */
int dq_iqn_head_backward(const dq_iqn_head* hp, const dq_iqn_head* hg, int32_t batch, int32_t nq,
                         const float* state, const dq_iqn_acts* a, const float* dq,
                         dq_iqn_grads* d, float* dstate, float* ws, void* stream);
size_t dq_iqn_workspace_floats(int32_t batch, int32_t nq, int32_t num_actions, int32_t embed_dim);
/* tf.random_uniform([n], 0, 1) for the quantile samples (atari_lib.py:171-172; TF's stream
   itself is not reproducible without TF): n float32 draws of call counter[0] of the
   generator `seed` (a splitmix64 hash of seed, call, index; 24 random bits), then
   counter[0] += 1 on the device -- graph replays continue the eager sequence. */
int dq_uniform_draw(int64_t* counter, uint64_t seed, int64_t n, float* out, void* stream);
/* dq_uniform_draw of `rows` taus (bitwise the same draws, then counter[0] += 1) fused with
   their cosine embedding cos[r][i] = cos((i + 1) * pi * tau[r]) (atari_lib.py:176-178), for
   dq_iqn_head_forward with taus NULL: two launches instead of three. */
int dq_iqn_tau_cos(int64_t* counter, uint64_t seed, int32_t rows, int32_t embed_dim, float* taus,
                   float* cos_out, void* stream);

/* _build_sync_op (dqn_agent.py:324-339): online -> target copy of the flat buffer. */
int dq_sync_copy(void* dst, const void* src, int64_t bytes, void* stream);

/* ---------------- data-parallel gradient exchange (BASELINE config 4) ----------------
 * The reference trains one replica (dqn_agent.py:432, _train_op); config 4 runs one learner
 * and one 1M buffer per GPU and averages their gradients each step.  A dq_comm is one RCCL
 * communicator over the learners; every call is issued on the given stream (graph-capturable),
 * in place, float32, ReduceOp AVG, so the learner chooses the queue each bucket runs on.
 * RCCL (librccl.so.1) is opened on first use.  Bootstrap: rank 0's dq_comm_unique_id is
 * handed to every rank (torch.distributed broadcast), then every rank calls dq_comm_create
 * (synchronous, collective). */
#define DQ_COMM_ID_BYTES 128
typedef struct dq_comm dq_comm;
int dq_comm_unique_id(uint8_t* id_out /* DQ_COMM_ID_BYTES */);
int dq_comm_create(const uint8_t* id, int32_t nranks, int32_t rank, int32_t device, dq_comm** out);
int dq_comm_destroy(dq_comm* c);
/* buf[0, n) := mean over the ranks of buf[0, n) */
int dq_comm_allreduce_mean(dq_comm* c, float* buf, int64_t n, void* stream);
/* slice r = buf[r n, (r + 1) n) := its mean over the ranks, on rank r (ZeRO-1) */
int dq_comm_reduce_scatter_mean(dq_comm* c, float* buf, int64_t n_per_rank, void* stream);
/* every slice r of buf := rank r's slice r */
int dq_comm_all_gather(dq_comm* c, float* buf, int64_t n_per_rank, void* stream);
/* RCCL's version code, or -1 if it cannot be opened */
int dq_comm_version(void);

/* ---------------- the same exchange over peer memory, on ONE queue --------------------
 * ("one-queue exchange").  Learners on one node map each other's flat
 * gradient, parameter and flag buffers (IPC handles, exchanged by the host) and the exchange
 * runs as extra blocks ("riders") of the backward's grouped launches plus one short launch:
 *   launch 3: publish "my fc-bucket gradient of step e is final" (flags[1] = e + 1); the
 *             reduce-scatter + TF1 Adam of this rank's slice of [lo, n): wait until every
 *             rank's flags[1] > e, sum the slice over the ranks IN RANK ORDER, times 1 / N
 *             (the gloo reference's order, parallel.allreduce_mean_), ApplyAdam on the slice;
 *   launch 4: the second half of that slice;
 *   launch 5: publish "my slice's parameters of step e are updated" (flags[2] = e + 1);
 *             all-gather: every other rank's slice of the parameters once its flags[2] > e;
 *   launch 6: publish the conv bucket [0, lo) (flags[3]), wait for every rank's, its rank-
 *             ordered mean and ApplyAdam (replicated; this one advances the beta powers);
 *             the step counter flags[0] += 1 by the launch's last block.
 * No collective library, no second queue, no graph fork or join.  Remote loads are
 * system-coherent (sc0 sc1) behind an acquire; a flag is stored by the last of 16 blocks
 * that each wrote back their XCD's L2 behind a system release (counted per XCD in flags[6],
 * read from HW_REG_XCC_ID; a publication whose blocks ran on fewer than `xcds` XCDs latches an
 * error instead of publishing); every wait is bounded (max_polls), polls every rank's error
 * word too, and a timeout or another rank's error latches flags[4], after which the rank
 * publishes nothing (DQ_PEER_FLAG_WORDS words per rank, zero-initialised; flags[0] = the
 * step counter, equal on every rank; flags[8..10] / [11..13]: 100 MHz ticks waited / waits
 * counted at the grad / param / conv points; flags[14]: XCDs seen by the last publication). */
#define DQ_PEER_MAX 8
#define DQ_PEER_FLAG_WORDS 16
typedef struct dq_ipc_handle {
  uint8_t handle[64];             /* hipIpcMemHandle_t of the allocation holding the pointer */
  int64_t offset;                 /* the pointer's byte offset in that allocation */
} dq_ipc_handle;
int dq_peer_ipc_get(const void* ptr, dq_ipc_handle* out);
/* maps another process's allocation: *ptr_out = its base + offset; close with the base */
int dq_peer_ipc_open(const dq_ipc_handle* h, void** ptr_out, void** base_out);
int dq_peer_ipc_close(void* base);
/* hipDeviceCanAccessPeer: 1 if `device` can map `peer`'s memory (always 1 for itself) */
int dq_peer_can_access(int32_t device, int32_t peer);
typedef struct dq_peer {
  int32_t world, rank;
  int64_t lo, n;                  /* the sharded range [lo, n) of the flat buffers (floats);
                                     (n - lo) % (4 world) == 0, lo % 4 == 0 */
  float* grad[DQ_PEER_MAX];       /* rank q's flat gradient, mapped here ([rank]: own) */
  float* param[DQ_PEER_MAX];      /* rank q's flat parameters */
  uint64_t* flags[DQ_PEER_MAX];   /* rank q's DQ_PEER_FLAG_WORDS flag words */
  int64_t max_polls;              /* per wait; then flags[4] := 1 + which flag timed out */
  int32_t xcds;                   /* XCDs a publication's blocks must cover (0: unchecked) */
  int32_t reserved;
} dq_peer;
/* dq_cnn_backward_riders of the fused Rainbow schedule (head_from 6, first 1, last 7, TF1
   Adam) with the exchange above in place of the fused optimizer's fc / conv updates: the
   gradients are stored (keep them in g), launches 1-5 as there plus the exchange riders,
   then launch 6.  world = 1 runs the same protocol with itself. */
int dq_cnn_backward_peer(const dq_cnn_params* p, const dq_cnn_params* g, int32_t batch,
                         const float* x, const dq_cnn_acts* a, const float* dout,
                         dq_cnn_acts* d, float* ws, const dq_rider* riders, int32_t n_riders,
                         const dq_adam_args* opt, const dq_cnn_net* head, const dq_peer* peer,
                         int32_t defer_ag, void* stream);
/* defer_ag != 0: launch 5 publishes this rank's slice and gathers the first quarter of the
   others'; the next step's dq_cnn_forward_fused_peer gathers the rest in its three conv
   launches (which read no fc parameter), or dq_peer_all_gather in a launch of its own (the
   learner loop's last step: every parameter is current when the loop returns).  var: this
   rank's flat parameters. */
int dq_cnn_forward_fused_peer(const dq_cnn_params* p0, const float* x0, dq_cnn_acts* a0, float* ws0,
                              const dq_cnn_params* p1, const float* x1, dq_cnn_acts* a1, float* ws1,
                              int32_t batch, int32_t fc1_1, const dq_peer* peer, float* var,
                              void* stream);
int dq_peer_all_gather(const dq_peer* peer, float* var, void* stream);
/* The construction-time check of the exchange's memory path (no reference counterpart: it
   guards config 4's data-parallel learners).  Three launches on `stream`: every
   workgroup of a full grid stores a (rank, tag)-keyed pattern over this rank's whole flat
   gradient buffer grad[rank][0, n) with plain stores (dirty lines in every XCD's L2, as the
   backward's epilogues leave them); the product publication (peer_publish_xcd) raises flags[7];
   every rank waits for every rank's flags[7] and reads every rank's buffer through the
   exchange's system-coherent loads, adding the words that differ from that rank's pattern to
   *mismatches_out (a device int32, zeroed by the caller).  A timeout latches flags[4].  The
   pattern is left in the gradient buffers: the caller zeroes its own once every rank is done. */
int dq_peer_selftest(const dq_peer* peer, uint32_t tag, int32_t* mismatches_out, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* DOPAMINE_AMD_H */
