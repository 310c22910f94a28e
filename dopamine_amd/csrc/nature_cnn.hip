// The Nature-CNN (atari_lib.py:85-144: conv 32@8x8/4, 64@4x4/2, 64@3x3/1 with TF
// "SAME" padding, ReLU, flatten 7744 in NHWC order, FC 512 + ReLU, FC n_out)
// forward and backward as implicit-GEMM kernels on the exact-fp32 matrix cores
// (v_mfma_f32_32x32x2_f32).
//
// One templated tile kernel serves every product.  A block is always 4 waves;
// they tile the output WM x WN (32x32 per wave) and split each K slice WK ways
// (WM*WN*WK = 4), the WK partial accumulators being summed in wave order through
// LDS at the end.  Operands come from loaders that produce 16-byte groups along
// their contiguous dimension (implicit im2col with compile-time geometry, the
// stride-1 transposed-conv gather, plain row/column-major), with a scalar path
// only for ragged edges and unaligned leading dimensions.  Results go to
// epilogues (bias + ReLU, ReLU-mask, plain store, weight/bias gradient -- the
// bias gradient is the GEMM's extra "ones" column -- written straight into the
// flat gradient buffer).  Split-K partial slabs are summed in slab order by a
// reduce kernel (deterministic).  An in-launch last-arriver reduction (agent
// release/acquire tickets) was measured no faster here: its fences cost what the
// launch boundary does.
//
// The stride-2 conv2 input gradient is NOT an implicit GEMM over the 4x4 taps
// (3/4 of those MACs would hit stride holes): it is four dense GEMMs, one per
// sub-pixel class (py, px) of the input, each over that class's 2x2 taps
// (K = 4 * 64), with the ReLU mask in the epilogue (SubPix below).
//
// Activations are NHWC fp32; weights live in the flat parameter buffer as
// conv (out, kh, kw, in) and FC (out, in) -- the GEMM's natural [M][K] layouts.
#include <algorithm>


#include "cnn_tile.h"
#include "c51_dev.h"

#include <cstring>

namespace dq {
namespace cnn {

// ------------------------------------------------------------ grouped launches
// Independent operations of the backward (layer L's weight gradient beside layer
// L+1's input gradient, a split-K reduce beside the next GEMMs) share ONE launch:
// each op owns a contiguous range of blockIdx.x.  All ops of a group run with
// the same block size kGroupT, and the block's LDS is the largest op's.
constexpr int kGroupT = 1024;

template <int WM, int WN, int WK, class AL, class BL, class EP, bool kLate = true>
struct GemmOp {
  static constexpr int kT = 64 * WM * WN * WK;
  static constexpr bool kLateFetch = kLate;
  static constexpr int kLds = Tile<WM, WN, WK>::template lds<AL, BL>();
  AL a;
  BL b;
  EP e;
  int M, N, K, kchunk, gx, gy, gz;
  __device__ __forceinline__ void run(int blk, float* smem, int tid_base = 0) const {
    const int bx = blk % gx, by = (blk / gx) % gy, bz = blk / (gx * gy);
    igemm_block<WM, WN, WK, AL, BL, EP, kLate, cnn_x6<WM, WN, WK, AL>()>(a, b, e, M, N, K, kchunk,
                                                                      bx, by, bz, smem, tid_base);
  }
  __host__ __device__ int blocks() const { return gx * gy * gz; }
};

// Two tiles of a GemmOp per block (threads [0, kT) and [kT, 2 kT), LDS halves): an 8-wave
// op in a launch of 16-wave blocks then fills its slots instead of leaving half of each
// block's waves idle.  With an odd tile count the last block's second half recomputes the
// last tile (pure-store epilogues only: the same bits stored twice).
template <class Op>
struct PairOp {
  static constexpr int kT = 2 * Op::kT;
  static constexpr int kLds = 2 * Op::kLds;
  static constexpr bool kLateFetch = Op::kLateFetch;
  Op op;
  __device__ __forceinline__ void run(int blk, float* smem) const {
    const int half = (int)threadIdx.x >= Op::kT ? 1 : 0;
    op.run(min(2 * blk + half, op.blocks() - 1), smem + half * Op::kLds, half * Op::kT);
  }
  int blocks() const { return (op.blocks() + 1) / 2; }
};

template <class EP, int T = kGroupT>
struct ReduceOp {                 // ordered split-K sum of nz slabs + epilogue
  static constexpr int kT = T;
  static constexpr int kLds = 0;
  const float* ws;
  int nz, M, N;
  EP e;
  __device__ __forceinline__ void run(int blk, float*) const {
    splitk_sum(ws, nz, M, N, e, (int64_t)blk * T + threadIdx.x);
  }
  int blocks() const { return (int)(((int64_t)M * N + T - 1) / T); }
};

// fc1's split-K sum (+ bias, ReLU) fused with fc2's k-band products: block
// (m tile, k band j of the 16 32-wide bands of fc2's K = 512, group of 4 fc2
// n-tiles) sums the fc1 slabs of its 32 x 32 slice of h in slab order (as
// splitk_sum), applies bias + ReLU (as EpiBiasAct), writes that slice of h (first
// n-group only) and keeps it in LDS; each wave then runs the 16-MFMA chain of one
// fc2 n-tile over band j in exactly the operand order of the tile kernel's wave j
// and stores the 32 x 32 partial to part[j].  Summing part[0..15] in order and
// adding the bias (dq_c51_loss_fused) reproduces the separate fc1-sum + fc2
// launches bit for bit, with one launch fewer on the forward's critical path.
struct FcHeadOp {
  static constexpr int kT = 256;
  static constexpr int kBands = kHidden / 32;      // 16
  static constexpr int kLds = 32 * 33;             // the h slice, rows padded to 33
  const float* ws;      // fc1 split-K slabs [nz][B][512]
  int nz;
  const float* b1;
  const float* w2;      // [NO][512]
  float* h;             // [B][512]
  float* part;          // [16][B][NO]
  int B, NO, mt, ng;
  int blocks() const { return mt * kBands * ng; }
  static int groups(int NO) { return ((NO + 31) / 32 + 3) / 4; }
  __device__ __forceinline__ void run(int blk, float* smem) const {
    const int g = blk % ng, j = (blk / ng) % kBands, m0 = 32 * (blk / (ng * kBands));
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int nt = 4 * g + wave;
    const int r = lane & 31, hh = lane >> 5, n = 32 * nt + r;
    // B operand: lane r's 8 k of each half, straight from W2's row n (k contiguous), loaded
    // after the slab sums (issuing it before them measured slower)
    float bv[2][8];
    auto load_w2 = [&]() {
#pragma unroll
      for (int hf = 0; hf < 2; ++hf) {
        const float* src = w2 + (int64_t)min(n, NO - 1) * kHidden + 32 * j + 16 * hf + 8 * hh;
        const float4 x0 = *reinterpret_cast<const float4*>(src);
        const float4 x1 = *reinterpret_cast<const float4*>(src + 4);
        const bool ok = n < NO;
        bv[hf][0] = ok ? x0.x : 0.0f; bv[hf][1] = ok ? x0.y : 0.0f;
        bv[hf][2] = ok ? x0.z : 0.0f; bv[hf][3] = ok ? x0.w : 0.0f;
        bv[hf][4] = ok ? x1.x : 0.0f; bv[hf][5] = ok ? x1.y : 0.0f;
        bv[hf][6] = ok ? x1.z : 0.0f; bv[hf][7] = ok ? x1.w : 0.0f;
      }
    };
    {
      const int r = tid >> 3, c = 4 * (tid & 7);
      const int m = min(m0 + r, B - 1);
      const int64_t i = (int64_t)m * kHidden + 32 * j + c, MN = (int64_t)B * kHidden;
      const float4 bb = *reinterpret_cast<const float4*>(b1 + 32 * j + c);
      float4 s = *reinterpret_cast<const float4*>(ws + i);
      for (int z0 = 1; z0 < nz; z0 += 8) {   // 8 slab loads in flight, summed in slab order
        float4 v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u)
          v[u] = *reinterpret_cast<const float4*>(ws + (int64_t)min(z0 + u, nz - 1) * MN + i);
#pragma unroll
        for (int u = 0; u < 8; ++u)
          if (z0 + u < nz) {
            s.x = __fadd_rn(s.x, v[u].x);
            s.y = __fadd_rn(s.y, v[u].y);
            s.z = __fadd_rn(s.z, v[u].z);
            s.w = __fadd_rn(s.w, v[u].w);
          }
      }
      s.x = fmaxf(__fadd_rn(s.x, bb.x), 0.0f);
      s.y = fmaxf(__fadd_rn(s.y, bb.y), 0.0f);
      s.z = fmaxf(__fadd_rn(s.z, bb.z), 0.0f);
      s.w = fmaxf(__fadd_rn(s.w, bb.w), 0.0f);
      if (g == 0 && m0 + r < B) *reinterpret_cast<float4*>(h + i) = s;
      float* q = smem + r * 33 + c;
      q[0] = s.x;
      q[1] = s.y;
      q[2] = s.z;
      q[3] = s.w;
    }
    __syncthreads();
    if (32 * nt >= NO) return;
    load_w2();
    f32x16 acc;
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[e] = 0.0f;
#pragma unroll
    for (int hf = 0; hf < 2; ++hf)
#pragma unroll
      for (int s8 = 0; s8 < 8; ++s8)
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(smem[r * 33 + 16 * hf + 8 * hh + s8],
                                                    bv[hf][s8], acc, 0, 0, 0);
    float* dst = part + (int64_t)j * B * NO;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int m = m0 + (e & 3) + 8 * (e >> 2) + 4 * hh;
      if (m < B && n < NO) dst[(int64_t)m * NO + n] = acc[e];
    }
  }
};

// TF1 Adam (the arithmetic of dq_adam_tf1) over a contiguous range of the flat
// parameter buffer, float4 grid-stride: the optimizer rides in the backward's last
// launch for every parameter whose gradient is final by then.
struct AdamOp {
  static constexpr int kT = kGroupT;
  static constexpr int kLds = 0;
  float* var;
  const float* grad;
  float* m;
  float* v;
  int64_t n;
  AdamDev o;
  int nb;
  // kU float4 per array per thread, all 4 kU loads issued before the first update
  // (kU = 2 / 4 measured no faster: the rider's cost is its CU slots and bytes)
  static constexpr int kU = 1;
  __device__ __forceinline__ void run(int blk, float*) const {
    const float alpha = adam_alpha_of(o.state, o.slot, o.lr);
    const float omb1 = __fsub_rn(1.0f, o.b1), omb2 = __fsub_rn(1.0f, o.b2);
    const int64_t n4 = n >> 2, stride = (int64_t)nb * kT * kU;
    for (int64_t i0 = (int64_t)blk * kT * kU + threadIdx.x; i0 < n4; i0 += stride) {
      float4 p[kU], g[kU], mm[kU], vv[kU];
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const int64_t i = min(i0 + (int64_t)u * kT, n4 - 1);   // clamped: loads never branch
        p[u] = reinterpret_cast<float4*>(var)[i];
        g[u] = reinterpret_cast<const float4*>(grad)[i];
        mm[u] = reinterpret_cast<float4*>(m)[i];
        vv[u] = reinterpret_cast<float4*>(v)[i];
      }
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const int64_t i = i0 + (int64_t)u * kT;
        if (i >= n4) break;
        adam1(p[u].x, g[u].x, mm[u].x, vv[u].x, alpha, omb1, omb2, o.eps);
        adam1(p[u].y, g[u].y, mm[u].y, vv[u].y, alpha, omb1, omb2, o.eps);
        adam1(p[u].z, g[u].z, mm[u].z, vv[u].z, alpha, omb1, omb2, o.eps);
        adam1(p[u].w, g[u].w, mm[u].w, vv[u].w, alpha, omb1, omb2, o.eps);
        reinterpret_cast<float4*>(var)[i] = p[u];
        reinterpret_cast<float4*>(m)[i] = mm[u];
        reinterpret_cast<float4*>(v)[i] = vv[u];
      }
    }
    if (blk == 0 && threadIdx.x < (n & 3)) {
      const int64_t i = (n4 << 2) + threadIdx.x;
      adam1(var[i], grad[i], m[i], v[i], alpha, omb1, omb2, o.eps);
    }
  }
  int blocks() const { return nb; }
};

// ------------------------------------------------- data-parallel exchange over peer memory
// (dq_peer, include/dopamine_amd.h).  Every rank's flat gradient, parameter and
// flag buffers are mapped into every learner; the exchange runs as ops of the backward's
// grouped launches.  Flag words per rank: [0] step counter e (local; the exchange launch's
// last block advances it), [1] fc-bucket gradient of step e final (= e + 1), [2] this rank's
// slice of the parameters updated, [3] conv bucket gradient final, [4] error latch (below),
// [5] the exchange launch's block ticket, [6] the publishing blocks' per-XCD arrival counts,
// [7] the self-test's flag (dq_peer_selftest), [8..10] 100 MHz ticks waited at the grad /
// param / conv exchange points (block 0 of each waiting op), [11..13] how many such waits,
// [14] how many XCDs the last publication saw.
// Error latch: 1 + which (this rank's wait for flag `which` timed out), kErrPeer + q (rank q
// had latched an error: every waiter gives up with it), kErrXcd + k (a publication's blocks
// ran on k XCDs, fewer than P.xcds: a write-back may be missing, nothing is published).
// Once it is set the rank publishes no flag again.
// Loads of another rank's (and, uniformly, one's own) exchanged words are system-coherent
// (sc0 sc1: no stale line of a previous step in this GPU's caches); a flag is a system-scope
// store behind a system release (s_waitcnt after it: the guide's compiler-hazard rule).
enum { kPeerStep = 0, kPeerGrad = 1, kPeerParam = 2, kPeerConv = 3, kPeerErr = 4, kPeerTicket = 5,
       kPeerPubCount = 6, kPeerTest = 7, kPeerWaitTicks = 8, kPeerWaitCount = 11,
       kPeerPubXcds = 14 };
enum { kErrPeer = 16, kErrXcd = 32 };
static_assert(kPeerPubXcds < DQ_PEER_FLAG_WORDS, "flag words");

// the XCD this wave runs on (HW_REG_XCC_ID bits 3:0; s_getreg_b32 simm16 = size-1 << 11 | id 20)
__device__ __forceinline__ unsigned xcc_id() {
  return (unsigned)__builtin_amdgcn_s_getreg((3 << 11) | 20) & 15u;
}

__device__ __forceinline__ uint64_t peer_load(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void peer_store(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// 16 bytes at base[4 i4 ..] with the system-coherent cache policy (cpol sc0 | sc1 = 1 | 16);
// the resource is the (wave-uniform) base, the lane's offset a VGPR (buffers < 2 GB)
__device__ __forceinline__ float4 peer_load4(const float* base, int64_t i4) {
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), 0, 0x7fffffff, 0x00020000),
      (int)(i4 * 16), 0, 17);
  return make_float4(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z),
                     __uint_as_float(v.w));
}
// the step counter, read once per block (a previous launch wrote it)
__device__ __forceinline__ uint64_t peer_step(const dq_peer& P) {
  return __hip_atomic_load(&P.flags[P.rank][kPeerStep], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// publish flag `which` of step e: everything this rank stored before this launch is final.
// The stores were made by earlier launches on every XCD, and each XCD's L2 holds its own
// dirty lines: a release fence writes back only the L2 of the XCD it runs on, and a peer's
// loads (over xGMI, or through another process's mapping of this memory) do not see lines
// still dirty in this device's L2s.  So kPubBlocks blocks -- consecutive workgroups, dealt
// round-robin over the XCDs -- each write back their XCD's L2, wait for it, and count
// themselves on a per-rank word of eight 8-bit per-XCD counts (HW_REG_XCC_ID); the last to
// arrive stores the flag, and only if the blocks ran on at least P.xcds distinct XCDs -- the
// round-robin dealing is observed, not promised (the guide's dispatch contract), so a
// placement that missed an XCD latches kErrXcd + k instead of publishing over a dirty L2.
// (Publishing from one block left stale slices at world 8: tools/peer_world_diag.py)
// Diagnostic builds only (tools/build_variant.py, never the product): -DDQ_PEER_DROP_XCD_FENCE=k
// skips the write-back on XCD k; -DDQ_PEER_HIDE_XCD=k counts XCD k's blocks as the next XCD's.
constexpr int kPubBlocks = 16;
__device__ __forceinline__ void peer_publish_xcd(const dq_peer& P, int which) {
  if (threadIdx.x != 0) return;
  const uint64_t e = peer_step(P);
  unsigned x = xcc_id() & 7u;
#ifdef DQ_PEER_DROP_XCD_FENCE
  if (x != DQ_PEER_DROP_XCD_FENCE)
#endif
  {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");      // this XCD's L2 written back
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
#ifdef DQ_PEER_HIDE_XCD
  if (x == DQ_PEER_HIDE_XCD) x = (x + 1) & 7u;
#endif
  uint64_t* cnt = &P.flags[P.rank][kPeerPubCount];
  const uint64_t add = 1ull << (8 * x);
  const uint64_t now =
      __hip_atomic_fetch_add(cnt, add, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + add;
  int total = 0, seen = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int f = (int)((now >> (8 * k)) & 0xffu);
    total += f;
    seen += f != 0 ? 1 : 0;
  }
  if (total == kPubBlocks) {                           // every block's write-back is done
    // (the next publication is a later launch: the counts restart from zero)
    __hip_atomic_store(cnt, (uint64_t)0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&P.flags[P.rank][kPeerPubXcds], (uint64_t)seen, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
    uint64_t* err = &P.flags[P.rank][kPeerErr];
    if (seen < P.xcds) {
      if (peer_load(err) == 0) peer_store(err, (uint64_t)(kErrXcd + seen));
      return;
    }
    if (peer_load(err) != 0) return;                   // a latched error: publish nothing more
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    peer_store(&P.flags[P.rank][which], e + 1);
  }
}
// the whole block waits until every rank's flag `which` passed step e (lane q of wave 0
// polls rank q; bounded: a timeout latches the error word).  Every 64 polls the lanes also
// read every rank's error word: one latched anywhere (a rank that timed out, or stopped
// publishing) ends this wait too, latching kErrPeer + q here, so every live learner gives up
// instead of reading a failed rank's stale buffers.  account: add the wait's duration (100 MHz
// ticks) to this rank's counters for `which` (block 0 of each waiting op).
// Returns false on a timeout or a latched error.
__device__ __forceinline__ bool peer_wait(const dq_peer& P, int which, uint64_t e, float* smem,
                                          bool account = false) {
  int* ok = reinterpret_cast<int*>(smem);
  if (threadIdx.x < 64) {
    const int q = threadIdx.x;
    uint64_t* err = &P.flags[P.rank][kPeerErr];
    const uint64_t t0 = account ? __builtin_amdgcn_s_memrealtime() : 0;
    bool done = q >= P.world;
    int bad = 0;
    int64_t polls = 0;
    while (true) {                      // every exit condition is wave-uniform
      if (!done) done = peer_load(&P.flags[q][which]) > e;
      if (__all(done ? 1 : 0)) break;
      if (++polls > P.max_polls) {
        if (q == 0 && peer_load(err) == 0) peer_store(err, (uint64_t)(1 + which));
        bad = 1;
        break;
      }
      if ((polls & 63) == 0) {          // an error latched on any rank: give up as well
        const bool eq = q < P.world && peer_load(&P.flags[q][kPeerErr]) != 0;
        const uint64_t any = __ballot(eq ? 1 : 0);
        if (any != 0) {
          if (q == 0 && peer_load(err) == 0)
            peer_store(err, (uint64_t)(kErrPeer + __builtin_ctzll(any)));
          bad = 1;
          break;
        }
      }
      __builtin_amdgcn_s_sleep(2);
    }
    if (q == 0) {
      *ok = bad ? 0 : 1;
      if (account && which >= kPeerGrad && which <= kPeerConv) {
        const uint64_t dt = __builtin_amdgcn_s_memrealtime() - t0;
        __hip_atomic_fetch_add(&P.flags[P.rank][kPeerWaitTicks + which - kPeerGrad], dt,
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_fetch_add(&P.flags[P.rank][kPeerWaitCount + which - kPeerGrad], (uint64_t)1,
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    // acquire: this CU's L1 and this XCD's L2 drop lines of the peers' memory read before
    // the flags moved
    if (!bad) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  }
  __syncthreads();
  const bool r = *ok != 0;
  __syncthreads();
  return r;
}
// the exchange launch's last block (ticket) advances the step counter: every block of the
// launch has read it by then
__device__ __forceinline__ void peer_ticket(const dq_peer& P, int total_blocks, uint64_t e) {
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t* t = &P.flags[P.rank][kPeerTicket];
    if (atomicAdd((unsigned long long*)t, 1ull) == (unsigned long long)(total_blocks - 1)) {
      __hip_atomic_store(t, (uint64_t)0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&P.flags[P.rank][kPeerStep], e + 1, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// publish flag `which` (kPeerGrad / kPeerParam; kPeerConv is PeerExchOp's first blocks'):
// kPubBlocks one-wave blocks, peer_publish_xcd
struct PeerPubOp {
  static constexpr int kT = 64;
  static constexpr int kLds = 0;
  dq_peer P;
  int which;
  __device__ __forceinline__ void run(int, float*) const { peer_publish_xcd(P, which); }
  int blocks() const { return kPubBlocks; }
};

// float4 i of the rank-ordered mean over the ranks' gradients, ApplyAdam'd into var / m / v
// (the loads of kU elements issued before the first update)
template <int kU>
__device__ __forceinline__ void peer_mean_adam(const dq_peer& P, float* var, float* m, float* v,
                                               const int64_t (&idx)[kU], int64_t end4, float alpha,
                                               float omb1, float omb2, float eps, float inv) {
  float4 g[kU], p[kU], mm[kU], vv[kU];
#pragma unroll
  for (int u = 0; u < kU; ++u) {
    const int64_t i = min(idx[u], end4 - 1);          // clamped: the loads never branch
    g[u] = peer_load4(P.grad[0], i);
#pragma unroll
    for (int q = 1; q < DQ_PEER_MAX; ++q)
      if (q < P.world) {
        const float4 x = peer_load4(P.grad[q], i);
        g[u].x = __fadd_rn(g[u].x, x.x);
        g[u].y = __fadd_rn(g[u].y, x.y);
        g[u].z = __fadd_rn(g[u].z, x.z);
        g[u].w = __fadd_rn(g[u].w, x.w);
      }
    p[u] = reinterpret_cast<float4*>(var)[i];
    mm[u] = reinterpret_cast<float4*>(m)[i];
    vv[u] = reinterpret_cast<float4*>(v)[i];
  }
#pragma unroll
  for (int u = 0; u < kU; ++u) {
    if (idx[u] >= end4) break;
    const int64_t i = idx[u];
    const float4 gm = make_float4(__fmul_rn(g[u].x, inv), __fmul_rn(g[u].y, inv),
                                  __fmul_rn(g[u].z, inv), __fmul_rn(g[u].w, inv));
    adam1(p[u].x, gm.x, mm[u].x, vv[u].x, alpha, omb1, omb2, eps);
    adam1(p[u].y, gm.y, mm[u].y, vv[u].y, alpha, omb1, omb2, eps);
    adam1(p[u].z, gm.z, mm[u].z, vv[u].z, alpha, omb1, omb2, eps);
    adam1(p[u].w, gm.w, mm[u].w, vv[u].w, alpha, omb1, omb2, eps);
    reinterpret_cast<float4*>(var)[i] = p[u];
    reinterpret_cast<float4*>(m)[i] = mm[u];
    reinterpret_cast<float4*>(v)[i] = vv[u];
  }
}

// The ops below hold at most kPeerMaxBlocks blocks each (grid-stride): blocks that wait for
// other learners hold CU slots, and learners sharing a GPU (the one-GPU tests) must leave
// the others room to reach the flags being waited for.
constexpr int kPeerMaxBlocks = 128;

// reduce-scatter + TF1 Adam of floats [b0, b1) of this rank's slice: wait for every rank's
// fc gradient, their sum in rank order times 1 / world, ApplyAdam (this rank keeps the
// slice's moments).  grid-stride over float4 pairs, nb blocks.
struct PeerRsAdamOp {
  static constexpr int kT = kGroupT;
  static constexpr int kLds = 1;
  dq_peer P;
  AdamDev o;
  float* var;          // own flat parameters (= P.param[P.rank])
  float* m;
  float* v;
  int64_t b0, b1;      // float offsets in the flat buffers, multiples of 4
  int nb;
  __device__ __forceinline__ void run(int blk, float* smem) const {
    const uint64_t e = peer_step(P);
    if (!peer_wait(P, kPeerGrad, e, smem, blk == 0)) return;
    const float alpha = adam_alpha_of(o.state, o.slot, o.lr);
    const float omb1 = __fsub_rn(1.0f, o.b1), omb2 = __fsub_rn(1.0f, o.b2);
    const float inv = __fdiv_rn(1.0f, (float)P.world);
    const int64_t e4 = b1 >> 2, st = (int64_t)nb * kT;
    for (int64_t i = (b0 >> 2) + (int64_t)blk * kT + threadIdx.x; i < e4; i += 2 * st) {
      const int64_t idx[2] = {i, i + st};
      peer_mean_adam<2>(P, var, m, v, idx, e4, alpha, omb1, omb2, o.eps, inv);
    }
  }
  int blocks() const { return nb; }
};

// all-gather: every other rank's updated slice of [lo, n) once its kPeerParam flag shows the
// step, float4s [f0, f1) of the (world - 1) slices in rank order.  lag 0: in the step that
// updated them (launch 5, publishing this rank's; the step counter is still e); lag 1: after
// that step's exchange launch advanced the counter -- the next step's conv forward launches
// (the learner loop's deferred gather) or a launch of its own (dq_peer_all_gather).
struct PeerAgOp {
  static constexpr int kT = kGroupT;
  static constexpr int kLds = 1;
  dq_peer P;
  float* var;
  int nb, lag;
  int64_t f0, f1;
  __device__ __forceinline__ void run(int blk, float* smem) const {
    const uint64_t e = peer_step(P);
    if (e < (uint64_t)lag) return;                 // before the first step: nothing updated
    if (!peer_wait(P, kPeerParam, e - lag, smem, blk == 0)) return;
    const int64_t S4 = ((P.n - P.lo) / P.world) >> 2;       // float4 per slice
    const int64_t tot = min(f1, S4 * (P.world - 1)), st = (int64_t)nb * kT;
    for (int64_t j0 = f0 + (int64_t)blk * kT + threadIdx.x; j0 < tot; j0 += 4 * st) {
      float4 x[4];
      int64_t at[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {                // loads of 4 elements in flight
        const int64_t j = min(j0 + u * st, tot - 1);
        int q = (int)(j / S4);
        q += q >= P.rank ? 1 : 0;                    // every rank but this one
        at[u] = (P.lo >> 2) + (int64_t)q * S4 + (j - (int64_t)(j / S4) * S4);
        x[u] = peer_load4(P.param[q], at[u]);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (j0 + u * st < tot) reinterpret_cast<float4*>(var)[at[u]] = x[u];
    }
  }
  int blocks() const { return nb; }
};

#ifdef DQ_GROUP_PROF
// stamp build only (tools/group_stamps.py GS_PEER=1): thread 0 of each of the exchange
// launch's first 16 blocks stamps entry / published / waited / updated / ticket into a ring
// of its own (one writer per ring, like the grouped launches' records)
constexpr int kPeerPhRing = 128;
__device__ unsigned long long g_peer_ph[16][kPeerPhRing][5];
__device__ unsigned g_peer_ph_seq[16];
#define DQ_PEER_PH(k) if (threadIdx.x == 0 && blk < 16) ph[k] = __builtin_amdgcn_s_memrealtime()
#else
#define DQ_PEER_PH(k)
#endif
// the exchange launch (6): blocks 0..kPubBlocks-1 publish the conv bucket; every block waits for every
// rank's, takes the rank-ordered mean of [0, lo) and applies TF1 Adam (replicated; block 0
// also advances the beta powers).  Every block takes a ticket; the last advances the step
// counter.
struct PeerExchOp {
  static constexpr int kT = kGroupT;
  static constexpr int kLds = 1;
  dq_peer P;
  AdamDev o;
  float* var;
  float* m;
  float* v;
  int nc;
  __device__ __forceinline__ void run(int blk, float* smem) const {
#ifdef DQ_GROUP_PROF
    unsigned long long ph[5] = {0, 0, 0, 0, 0};
#endif
    DQ_PEER_PH(0);
    const uint64_t e = peer_step(P);
    if (blk < kPubBlocks) peer_publish_xcd(P, kPeerConv);
    DQ_PEER_PH(1);
    const bool ok = peer_wait(P, kPeerConv, e, smem, blk == 0);
    DQ_PEER_PH(2);
    if (ok) {
      const float alpha = adam_alpha_of(o.state, o.slot, o.lr);
      const float omb1 = __fsub_rn(1.0f, o.b1), omb2 = __fsub_rn(1.0f, o.b2);
#ifdef DQ_PEER_FAULT_REPLICA
      // fault injection (tools/build_variant.py only): this rank's replicated conv-bucket
      // mean is off by 2^-20, so its replica drifts from the others' (bench.py must report
      // the schedule as failed)
      const float inv = __fdiv_rn(P.rank == DQ_PEER_FAULT_REPLICA ? 1.00000095f : 1.0f,
                                  (float)P.world);
#else
      const float inv = __fdiv_rn(1.0f, (float)P.world);
#endif
      const int64_t e4 = P.lo >> 2, st = (int64_t)nc * kT;
      for (int64_t i = (int64_t)blk * kT + threadIdx.x; i < e4; i += 2 * st) {
        const int64_t idx[2] = {i, i + st};
        peer_mean_adam<2>(P, var, m, v, idx, e4, alpha, omb1, omb2, o.eps, inv);
      }
      if (blk == 0 && threadIdx.x == 0) adam_bump(o.state, o.slot, o.b1, o.b2);
    }
    DQ_PEER_PH(3);
    peer_ticket(P, nc, e);
    DQ_PEER_PH(4);
#ifdef DQ_GROUP_PROF
    if (threadIdx.x == 0 && blk < 16) {
      const unsigned sq = g_peer_ph_seq[blk];
      g_peer_ph_seq[blk] = sq + 1;
      for (int k = 0; k < 5; ++k) g_peer_ph[blk][sq % kPeerPhRing][k] = ph[k];
    }
#endif
  }
  int blocks() const { return nc; }
};

// dq_peer_selftest: word i of rank q's pattern for this tag (a 32-bit mix, so a stale or
// misplaced line almost never matches by chance)
__device__ __forceinline__ unsigned selftest_word(unsigned q, unsigned tag, unsigned i) {
  unsigned h = i * 0x9E3779B1u ^ (q + 1u) * 0x85EBCA77u ^ tag;
  h ^= h >> 16;
  h *= 0x7feb352du;
  h ^= h >> 15;
  h *= 0x846ca68bu;
  h ^= h >> 16;
  return h;
}
// every block of a full grid stores its share of this rank's pattern over grad[rank][0, n)
// with plain 16-byte stores, as the backward's epilogues store gradients
struct SelfTestFillOp {
  static constexpr int kT = 256;
  static constexpr int kLds = 0;
  dq_peer P;
  unsigned tag;
  int nb;
  __device__ __forceinline__ void run(int blk, float*) const {
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
    u32x4* g = reinterpret_cast<u32x4*>(P.grad[P.rank]);
    for (int64_t i = (int64_t)blk * kT + threadIdx.x; i < P.n / 4; i += (int64_t)nb * kT) {
      const unsigned w = (unsigned)(4 * i);
      g[i] = u32x4{selftest_word(P.rank, tag, w), selftest_word(P.rank, tag, w + 1),
                   selftest_word(P.rank, tag, w + 2), selftest_word(P.rank, tag, w + 3)};
    }
  }
  int blocks() const { return nb; }
};
// wait for every rank's self-test flag, then read every rank's buffer with the exchange's
// loads and count the words that are not its pattern
struct SelfTestCheckOp {
  static constexpr int kT = 256;
  static constexpr int kLds = 1;
  dq_peer P;
  unsigned tag;
  int* out;
  int nb;
  __device__ __forceinline__ void run(int blk, float* smem) const {
    const uint64_t e = peer_step(P);
    if (!peer_wait(P, kPeerTest, e, smem)) return;
    int bad = 0;
    for (int q = 0; q < P.world; ++q)
      for (int64_t i = (int64_t)blk * kT + threadIdx.x; i < P.n / 4; i += (int64_t)nb * kT) {
        const float4 v = peer_load4(P.grad[q], i);
        const unsigned w = (unsigned)(4 * i);
        bad += (__float_as_uint(v.x) != selftest_word(q, tag, w)) +
               (__float_as_uint(v.y) != selftest_word(q, tag, w + 1)) +
               (__float_as_uint(v.z) != selftest_word(q, tag, w + 2)) +
               (__float_as_uint(v.w) != selftest_word(q, tag, w + 3));
      }
    if (bad) atomicAdd(out, bad);
  }
  int blocks() const { return nb; }
};

// TF1 RMSProp (the arithmetic of dq_rmsprop_tf1) over a contiguous range, as AdamOp
struct RmsOp {
  static constexpr int kT = kGroupT;
  static constexpr int kLds = 0;
  float* var;
  const float* grad;
  float* ms;
  float* mom;
  float* mg;            // centered only (else any valid pointer)
  int64_t n;
  RmsDev o;
  int nb;
  static constexpr int kU = 1;
  __device__ __forceinline__ void run(int blk, float*) const {
    const bool c = o.centered != 0;
    const int64_t n4 = n >> 2, stride = (int64_t)nb * kT * kU;
    for (int64_t i0 = (int64_t)blk * kT * kU + threadIdx.x; i0 < n4; i0 += stride) {
      float4 p[kU], g[kU], s[kU], mo[kU], a[kU];
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const int64_t i = min(i0 + (int64_t)u * kT, n4 - 1);   // clamped: loads never branch
        p[u] = reinterpret_cast<float4*>(var)[i];
        g[u] = reinterpret_cast<const float4*>(grad)[i];
        s[u] = reinterpret_cast<float4*>(ms)[i];
        mo[u] = reinterpret_cast<float4*>(mom)[i];
        a[u] = c ? reinterpret_cast<float4*>(mg)[i] : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const int64_t i = i0 + (int64_t)u * kT;
        if (i >= n4) break;
        rms1(p[u].x, g[u].x, s[u].x, a[u].x, mo[u].x, o.lr, o.omr, o.mu, o.eps, c);
        rms1(p[u].y, g[u].y, s[u].y, a[u].y, mo[u].y, o.lr, o.omr, o.mu, o.eps, c);
        rms1(p[u].z, g[u].z, s[u].z, a[u].z, mo[u].z, o.lr, o.omr, o.mu, o.eps, c);
        rms1(p[u].w, g[u].w, s[u].w, a[u].w, mo[u].w, o.lr, o.omr, o.mu, o.eps, c);
        reinterpret_cast<float4*>(var)[i] = p[u];
        reinterpret_cast<float4*>(ms)[i] = s[u];
        reinterpret_cast<float4*>(mom)[i] = mo[u];
        if (c) reinterpret_cast<float4*>(mg)[i] = a[u];
      }
    }
    if (blk == 0 && threadIdx.x < (n & 3)) {
      const int64_t i = (n4 << 2) + threadIdx.x;
      float q = c ? mg[i] : 0.0f;
      rms1(var[i], grad[i], ms[i], q, mom[i], o.lr, o.omr, o.mu, o.eps, c);
      if (c) mg[i] = q;
    }
  }
  int blocks() const { return nb; }
};

// the fused optimizer's range op (kOpt 1: AdamOp, 2: RmsOp) over [w0, w1) of the flat buffer
template <int kOpt>
struct OptPart;
template <>
struct OptPart<1> {
  static AdamOp make(const dq_cnn_params* p, const dq_cnn_params* g, const dq_adam_args* o,
                     float* w0, float* w1) {
    const ptrdiff_t off = w0 - o->var;
    const int64_t n = (int64_t)(w1 - w0);
    const int64_t per = (int64_t)kGroupT * AdamOp::kU;
    const int nb = (int)std::max<int64_t>(1, ((n >> 2) + per - 1) / per);
    const AdamDev od{o->state, o->slot, o->lr, o->beta1, o->beta2, o->epsilon, 1};   // reads g
    return AdamOp{w0, g->conv1_w + (w0 - p->conv1_w), o->m + off, o->v + off, n, od, nb};
  }
};
template <>
struct OptPart<2> {
  static RmsOp make(const dq_cnn_params* p, const dq_cnn_params* g, const dq_adam_args* o,
                    float* w0, float* w1) {
    const ptrdiff_t off = w0 - o->var;
    const int64_t n = (int64_t)(w1 - w0);
    const int64_t per = (int64_t)kGroupT * RmsOp::kU;
    const int nb = (int)std::max<int64_t>(1, ((n >> 2) + per - 1) / per);
    float* mg = o->centered ? o->mg : o->m;
    return RmsOp{w0, g->conv1_w + (w0 - p->conv1_w), o->m + off, o->v + off, mg + off, n,
                 rms_dev(o), nb};
  }
};

// fc1's weight gradient + its optimizer in the vector epilogue: TF1 Adam
// or centered RMSProp over fc1_w and fc1_b, the riders' arithmetic.  RMSProp's four state
// arrays made the epilogue the longer path at first (config 2: 8,060 vs 8,143 steps/s with
// riders); with the next row group's loads issued before this group's stores (kVecPre) it
// is the shorter one: 8,295-8,348 vs 8,235-8,250 (profiles/r3_s3_rmsepi_ab.log)
template <int kOpt>
struct Fc1EpiOpt;
template <>
struct Fc1EpiOpt<1> {
  static EpiGradAdamVec make(const dq_cnn_params* p, const dq_cnn_params* g, const dq_adam_args* o) {
    const ptrdiff_t ow = p->fc1_w - o->var, ob = p->fc1_b - o->var;
    return EpiGradAdamVec{g->fc1_w, g->fc1_b, kFlat, p->fc1_w, o->m + ow, o->v + ow, p->fc1_b,
                          o->m + ob, o->v + ob,
                          AdamDev{o->state, o->slot, o->lr, o->beta1, o->beta2, o->epsilon,
                                  o->no_grad_store == 0}};
  }
};

template <>
struct Fc1EpiOpt<2> {       // centered RMSProp (DQN, config 2)
  static EpiGradRmsVec make(const dq_cnn_params* p, const dq_cnn_params* g, const dq_adam_args* o) {
    return EpiGradRmsVec{GradEpi<2>::make(g->fc1_w, g->fc1_b, kFlat, p->fc1_w, p->fc1_b,
                                          AdamHost{o}, 0)};
  }
};

// the same for fc2: fc2's weight gradient + optimizer in one vector epilogue
template <int kOpt>
struct Fc2EpiOpt;
template <>
struct Fc2EpiOpt<1> {
  static EpiGradAdamVec make(const dq_cnn_params* p, const dq_cnn_params* g, const dq_adam_args* o) {
    const ptrdiff_t ow = p->fc2_w - o->var, ob = p->fc2_b - o->var;
    return EpiGradAdamVec{g->fc2_w, g->fc2_b, kHidden, p->fc2_w, o->m + ow, o->v + ow, p->fc2_b,
                          o->m + ob, o->v + ob,
                          AdamDev{o->state, o->slot, o->lr, o->beta1, o->beta2, o->epsilon,
                                  o->no_grad_store == 0}};
  }
};
template <>
struct Fc2EpiOpt<2> {
  static EpiGradRmsVec make(const dq_cnn_params* p, const dq_cnn_params* g, const dq_adam_args* o) {
    return EpiGradRmsVec{GradEpi<2>::make(g->fc2_w, g->fc2_b, kHidden, p->fc2_w, p->fc2_b,
                                          AdamHost{o}, 0)};
  }
};

// A recorded replay operation (replay_dev.h) riding in a grouped launch: its
// blocks come first in the launch so the single-wave sum-tree update / sampler
// chains start before the GEMM blocks fill the machine.
template <bool kGroups = false>
struct RiderOpT {
  static constexpr int kT = kGroupT;
  static constexpr int kLds = (kRiderLds + 3) / 4;
  RiderDesc r;
  __device__ __forceinline__ void run(int blk, float* smem) const {
    run_rider<kT, kGroups>(r, blk, smem);
  }
  int blocks() const { return rider_blocks<kT>(r); }
};
using RiderOp = RiderOpT<false>;

template <class... Ops>
constexpr int max_lds() {
  int m = 1;
  ((m = Ops::kLds > m ? Ops::kLds : m), ...);
  return m;
}

// An op with fewer threads than the launch's block leaves its spare waves idle:
// they exit at once, and the op's barriers then wait for its own waves only
// (s_barrier counts the waves of the workgroup that have not ended).
template <class Op>
__device__ __forceinline__ bool dispatch(const Op& op, int nb, int& blk, float* smem) {
  if (blk < nb) {
    if (Op::kT >= (int)blockDim.x || (int)threadIdx.x < Op::kT) op.run(blk, smem);
    return true;
  }
  blk -= nb;
  return false;
}

template <class... Ops>
constexpr int max_threads() {
  int m = 64;
  ((m = Ops::kT > m ? Ops::kT : m), ...);
  return m;
}

template <class... Ops>
struct GroupArgs {
  int nblocks[sizeof...(Ops)];
};

constexpr bool kB1Late = false;   // backward launch 1 is one round of blocks: early fetch (+1.5%)
constexpr bool kF4Late = true;
constexpr bool kB6Late = true;
// 8 waves per SIMD (<= 64 VGPRs: two 16-wave blocks per CU) unless a tile op of the
// group fetches early (single-round launches, where the registers buy more)
template <class Op, class = void>
struct LateOk {
  static constexpr bool value = true;
};
template <class Op>
struct LateOk<Op, decltype((void)Op::kLateFetch)> {
  static constexpr bool value = Op::kLateFetch;
};
template <class... Ops>
constexpr int group_wpe() {
  return (LateOk<Ops>::value && ...) ? 8 : 1;
}
#ifdef DQ_GROUP_PROF
// Stamp build of the grouped launches (tools/group_stamps.py; never the product): every wave
// that runs an op writes one record -- s_memrealtime (100 MHz) at the kernel's entry and after
// its op returned, the launch's block count, the op's index in the group, the op-local block,
// the wave and its XCD -- into its own slot of a per-wave-position ring (position = block x
// 16 + wave; the slot from a counter only that position reads and advances: no atomics, no
// shared words, one launch at a time on the stream).  Only these buffers receive stamp words.
struct GrpRec {
  unsigned long long t0, t1;
  unsigned total, op_blk;      // op_blk: op index << 24 | op-local block << 8 | wave << 4 | XCD
};
constexpr unsigned kGrpPos = 1024 * 16, kGrpRing = 128;
__device__ GrpRec g_grp_rec[kGrpPos][kGrpRing];
__device__ unsigned g_grp_seq[kGrpPos];
template <class Op>
__device__ __forceinline__ bool dispatch_prof(const Op& op, int nb, int& blk, float* smem, int k,
                                              unsigned long long t0) {
  if (blk < nb) {
    if (Op::kT >= (int)blockDim.x || (int)threadIdx.x < Op::kT) {
      op.run(blk, smem);
      const unsigned p = blockIdx.x * 16 + (threadIdx.x >> 6);
      if ((threadIdx.x & 63) == 0 && p < kGrpPos) {
        const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
        const unsigned sq = g_grp_seq[p];
        g_grp_seq[p] = sq + 1;
        g_grp_rec[p][sq % kGrpRing] = GrpRec{t0, t1, gridDim.x,
                                             ((unsigned)k << 24) | ((unsigned)blk << 8) |
                                                 ((threadIdx.x >> 6) << 4) | xcc_id()};
      }
    }
    return true;
  }
  blk -= nb;
  return false;
}
#endif

template <int T, class... Ops>
__global__ __launch_bounds__(T) __attribute__((amdgpu_waves_per_eu(group_wpe<Ops...>())))
void k_grouped(GroupArgs<Ops...> g, Ops... ops) {
  warm_kernargs<sizeof(GroupArgs<Ops...>) + (sizeof(Ops) + ...) + 8 * sizeof...(Ops)>();
  __shared__ __attribute__((aligned(16))) float smem[max_lds<Ops...>()];
  int blk = blockIdx.x, i = 0;
#ifdef DQ_GROUP_PROF
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  ((dispatch_prof(ops, g.nblocks[i], blk, smem, i, t0) || (++i, false)) || ...);
#else
  ((dispatch(ops, g.nblocks[i++], blk, smem)) || ...);
#endif
}

// Launch context: a dry run only sizes the workspace, so the two can never disagree.
// a grouped GEMM op; split-K ops write slabs into ws + off (EpiPartial)
template <int WM, int WN, int WK, bool kLate = true, class AL, class BL, class EP>
GemmOp<WM, WN, WK, AL, BL, EP, kLate> gemm_op(AL a, BL b, EP e, int M, int N, int K, int kchunk) {
  GemmOp<WM, WN, WK, AL, BL, EP, kLate> op{a, b, e, M, N, K, kchunk, 0, 0, 0};
  op.gx = (M + 32 * WM - 1) / (32 * WM);
  op.gy = (N + 32 * WN - 1) / (32 * WN);
  op.gz = (K + kchunk - 1) / kchunk;
  return op;
}

template <class Op0, class... Ops>
void group(Ctx& c, Op0 op0, Ops... ops) {
  constexpr int T = max_threads<Op0, Ops...>();   // block = the largest op's
  if (c.dry) return;
  GroupArgs<Op0, Ops...> g;
  int i = 0, total = 0;
  g.nblocks[i++] = op0.blocks();
  total += op0.blocks();
  ((g.nblocks[i++] = ops.blocks(), total += ops.blocks()), ...);
  hipLaunchKernelGGL((k_grouped<T, Op0, Ops...>), dim3(total), dim3(T), 0, c.s, g, op0, ops...);
}

// group() with rider r (if any) in front
template <class... Ops>
void group_r(Ctx& c, const RiderDesc* r, Ops... ops) {
  if (r && r->kind != kRiderNone)
    if (r->kind == kRiderUniformSample && r->groups > 1)   // a chunk's grouped draw
      group(c, RiderOpT<true>{*r}, ops...);
    else
      group(c, RiderOp{*r}, ops...);
  else
    group(c, ops...);
}

// Tile shapes: WM = WN = 1 with WK k-bands sized so K takes one or two slices
// (BKT = 32 * WK); split-K only where the grid would otherwise leave most of the
// 256 CUs idle (weight streaming of fc1, the pixel-deep weight gradients).
// conv2 / conv3 weight gradients: 8 split-K slabs over B * 121; conv1's 28 over B * 441
// (4 / 14 measured slower)
constexpr int kSplitFc1 = 16, kSplitConvW = 8, kSplitConv1W = 28;

void forward(Ctx& c, const dq_cnn_params* p, int B, const float* x, dq_cnn_acts* a) {
  // conv1 / conv2 / conv3 + bias + ReLU  (implicit GEMM: M = pixels, N = out channels)
  gemm<1, 1, 8>(c, Im2col<Conv1>{x}, RowK{p->conv1_w, Conv1::K},
                EpiBiasAct{a->a1, p->conv1_b, 32, true}, B * 441, 32, Conv1::K);
  gemm<1, 1, 16>(c, Im2col<Conv2>{a->a1}, RowK{p->conv2_w, Conv2::K},
                 EpiBiasAct{a->a2, p->conv2_b, 64, true}, B * 121, 64, Conv2::K);
  gemm<1, 1, 9>(c, Im2col<Conv3>{a->a2}, RowK{p->conv3_w, Conv3::K},
                EpiBiasAct{a->a3, p->conv3_b, 64, true}, B * 121, 64, Conv3::K);
  // fc1 (7744 -> 512) + ReLU: weight streaming, split-K over the 7744 inputs
  gemm<1, 1, 16>(c, RowK{a->a3, kFlat}, RowK{p->fc1_w, kFlat},
                 EpiBiasAct{a->h, p->fc1_b, kHidden, true}, B, kHidden, kFlat, kSplitFc1);
  // fc2 (512 -> n_out), no activation
  gemm<1, 1, 16>(c, RowK{a->h, kHidden}, RowK{p->fc2_w, kHidden},
                 EpiBiasAct{a->out, p->fc2_b, p->n_out, false}, B, p->n_out, kHidden);
}

// The forward's grouped ops for one network (the same tiles and split order as
// forward(): bitwise identical outputs).  head = conv1, conv2, conv3, fc1 split-K
// slabs (into ws); tail = the slab sum (+ bias, ReLU) and fc2.
struct FwdOps {
  const dq_cnn_params* p;
  const float* x;
  dq_cnn_acts* a;
  float* ws;
  int B;
  static int fc1_chunk() { return split_chunk(kFlat, kSplitFc1, 32 * 16); }
  static int fc1_slabs() { return (kFlat + fc1_chunk() - 1) / fc1_chunk(); }
  static size_t ws_floats(int B) { return (size_t)fc1_slabs() * B * kHidden; }
  template <bool kLate = true>
  auto conv1() const {
    return gemm_op<1, 1, 8, kLate>(Im2col<Conv1>{x}, RowK{p->conv1_w, Conv1::K},
                            EpiBiasAct{a->a1, p->conv1_b, 32, true}, B * 441, 32, Conv1::K, Conv1::K);
  }
  template <bool kLate = true>
  auto conv2() const {
    return gemm_op<1, 1, 16, kLate>(Im2col<Conv2>{a->a1}, RowK{p->conv2_w, Conv2::K},
                             EpiBiasAct{a->a2, p->conv2_b, 64, true}, B * 121, 64, Conv2::K, Conv2::K);
  }
  template <bool kLate = true>
  auto conv3() const {
    return gemm_op<1, 1, 9, kLate>(Im2col<Conv3>{a->a2}, RowK{p->conv3_w, Conv3::K},
                            EpiBiasAct{a->a3, p->conv3_b, 64, true}, B * 121, 64, Conv3::K, Conv3::K);
  }
  template <bool kLate = true>
  auto fc1() const {
    return gemm_op<1, 1, 16, kLate>(RowK{a->a3, kFlat}, RowK{p->fc1_w, kFlat}, EpiPartial{ws, B, kHidden},
                             B, kHidden, kFlat, fc1_chunk());
  }
  auto fc1_sum() const {
    return ReduceOp<EpiBiasAct, 256>{ws, fc1_slabs(), B, kHidden,
                                     EpiBiasAct{a->h, p->fc1_b, kHidden, true}};
  }
  auto fc2() const {
    return gemm_op<1, 1, 16>(RowK{a->h, kHidden}, RowK{p->fc2_w, kHidden},
                             EpiBiasAct{a->out, p->fc2_b, p->n_out, false}, B, p->n_out, kHidden,
                             kHidden);
  }
  // fc2's 16 k-band partials live in ws right after fc1's slabs
  static size_t part_offset(int B) { return ws_floats(B); }
  static size_t fused_ws_floats(int B, int NO) {
    return ws_floats(B) + (size_t)FcHeadOp::kBands * B * NO;
  }
  FcHeadOp fchead() const {
    return FcHeadOp{ws, fc1_slabs(), p->fc1_b, p->fc2_w, a->h, ws + part_offset(B), B, p->n_out,
                    (B + 31) / 32, FcHeadOp::groups(p->n_out)};
  }
};

// The Rainbow fast path's forward: net 0 (online) whole up to fc2's k-band
// partials, net 1 (target, head run earlier: conv1..conv3 into a1) finishing with
// its fc1 slabs (if fc1_1) in net 0's fc1 launch and its fused head beside net 0's:
// 5 launches.  The logits are summed by dq_c51_loss_fused.
// The peer exchange's deferred all-gather: the first kAgLaunch5 / 16 of the (world - 1)
// slices' float4s in the step's own launch 5 (lag 0, beside the publish), the rest in thirds
// in the next forward's three conv launches (lag 1: they read no fc parameter; fc1's launch
// follows) -- launch 5 (~8 us) and the conv launches (~27 us) share the pull about in
// proportion to their length (tools/peer_n8_model.py).  The learner loop's last step leaves
// the rest to dq_peer_all_gather.
constexpr int kAgLaunch5 = 4;
struct AgParts {
  const dq_peer* P;
  float* var;
  int64_t total() const { return ((P->n - P->lo) / P->world / 4) * (P->world - 1); }
  int64_t split() const { return total() * kAgLaunch5 / 16; }
  PeerAgOp op(int64_t a, int64_t b, int lag) const {
    const int nb = (int)std::min<int64_t>(kPeerMaxBlocks,
                                          std::max<int64_t>(1, (b - a + 4 * kGroupT - 1) / (4 * kGroupT)));
    return PeerAgOp{*P, var, nb, lag, a, b};
  }
  PeerAgOp head() const { return op(0, split(), 0); }
  PeerAgOp part(int i) const {
    const int64_t s = split(), t = total();
    return op(s + (t - s) * i / 3, s + (t - s) * (i + 1) / 3, 1);
  }
};

void forward_fused(Ctx& c0, Ctx& c1, const FwdOps& f0, const FwdOps& f1, bool fc1_1,
                   bool conv3_1 = false, bool convs = true, bool fcs = true,
                   bool conv2_1 = false, bool conv1_1 = false, const AgParts* ag = nullptr) {
  const size_t n0 = FwdOps::fused_ws_floats(f0.B, f0.p->n_out);
  const size_t n1 = FwdOps::fused_ws_floats(f1.B, f1.p->n_out);
  c0.need = n0 > c0.need ? n0 : c0.need;
  c1.need = n1 > c1.need ? n1 : c1.need;
  if (c0.dry) return;
  if (convs && ag) {           // head_from 6 (the Rainbow fast path) with the deferred gather
    group(c0, f0.conv1<false>(), ag->part(0));
    if (conv2_1)
      group(c0, f0.conv2<true>(), f1.conv2(), ag->part(1));
    else
      group(c0, f0.conv2<false>(), ag->part(1));
    if (conv3_1)
      group(c0, f0.conv3<false>(), f1.conv3(), ag->part(2));
    else
      group(c0, f0.conv3<false>(), ag->part(2));
  } else if (convs) {
    // single-round launches fetch early; the conv2 launch with the target's conv2 late
    // (+0.9%); net 1's conv3 (head_from = 5) rides in net 0's conv3 launch (+1.1% over the
    // conv1 launch, +2.2% over the conv2 launch)
    if (conv1_1)                     // net 1's conv1 (head_from = 7) beside net 0's conv1
      group(c0, f0.conv1<false>(), f1.conv1());
    else
      group(c0, f0.conv1<false>());
    if (conv2_1)                     // net 1's conv2 (head_from = 6) beside net 0's conv2
      group(c0, f0.conv2<true>(), f1.conv2());
    else
      group(c0, f0.conv2<false>());
    if (conv3_1)
      group(c0, f0.conv3<false>(), f1.conv3());
    else
      group(c0, f0.conv3<false>());
  }
  if (!fcs) return;
  if (fc1_1)
    group(c0, f0.fc1<kF4Late>(), f1.fc1<kF4Late>());
  else
    group(c0, f0.fc1());
  group(c0, f0.fchead(), f1.fchead());
}

// The target half of the C51 loss (c51_dev.h) as a grouped-launch op: one 256-thread
// block per sample, riding in the online fused-head launch (head_from = 8).
struct TgtC51Op {
  static constexpr int kT = 256;
  static constexpr int kLds = c51_target_lds(4 * kC51TgtMaxWaveRows, 64);
  C51Target t;
  int blocks() const { return t.B; }
  __device__ __forceinline__ void run(int blk, float* smem) const {
    c51_target_block<kT>(t, blk, smem);
  }
};

// head_from = 8: the target network one launch earlier than head_from = 6 (its conv1 rode
// in the previous backward's last launch), so its fused head is final one launch before
// the online one's and the C51 target half rides beside the online head.
void forward_fused_c51(Ctx& c0, Ctx& c1, const FwdOps& f0, const FwdOps& f1, const C51Target& t,
                       bool convs, bool fcs) {
  const size_t n0 = FwdOps::fused_ws_floats(f0.B, f0.p->n_out);
  const size_t n1 = FwdOps::fused_ws_floats(f1.B, f1.p->n_out);
  c0.need = n0 > c0.need ? n0 : c0.need;
  c1.need = n1 > c1.need ? n1 : c1.need;
  if (c0.dry) return;
  if (convs) {
    group(c0, f0.conv1<false>(), f1.conv2());
    group(c0, f0.conv2<true>(), f1.conv3());
    group(c0, f0.conv3<false>(), f1.fc1());
  }
  if (!fcs) return;
  group(c0, f0.fc1<kF4Late>(), f1.fchead());
  group(c0, f0.fchead(), TgtC51Op{t});
}

// The online and target networks' forwards together: one grouped launch per layer
// holding both nets' ops -- 6 launches instead of 12.
void forward_pair(Ctx& c0, Ctx& c1, const dq_cnn_params* p0, const float* x0, dq_cnn_acts* a0,
                  const dq_cnn_params* p1, const float* x1, dq_cnn_acts* a1, int B) {
  const size_t need = FwdOps::ws_floats(B);
  c0.need = need > c0.need ? need : c0.need;
  c1.need = need > c1.need ? need : c1.need;
  if (c0.dry) return;
  const FwdOps f0{p0, x0, a0, c0.ws, B}, f1{p1, x1, a1, c1.ws, B};
  group(c0, f0.conv1(), f1.conv1());
  group(c0, f0.conv2(), f1.conv2());
  group(c0, f0.conv3(), f1.conv3());
  group(c0, f0.fc1(), f1.fc1());
  group(c0, f0.fc1_sum(), f1.fc1_sum());
  group(c0, f0.fc2(), f1.fc2());
}

// Net 0's whole forward with net 1's tail (whose head ran earlier, e.g. as riders of
// the previous backward) in net 0's last two launches.
void forward_with_tail(Ctx& c0, Ctx& c1, const FwdOps& f0, const FwdOps& f1) {
  const size_t need = FwdOps::ws_floats(f0.B);
  c0.need = need > c0.need ? need : c0.need;
  c1.need = need > c1.need ? need : c1.need;
  if (c0.dry) return;
  group(c0, f0.conv1());
  group(c0, f0.conv2());
  group(c0, f0.conv3());
  group(c0, f0.fc1());
  group(c0, f0.fc1_sum(), f1.fc1_sum());
  group(c0, f0.fc2(), f1.fc2());
}

void forward_head(Ctx& c, const FwdOps& f) {
  const size_t need = FwdOps::ws_floats(f.B);
  c.need = need > c.need ? need : c.need;
  if (c.dry) return;
  group(c, f.conv1());
  group(c, f.conv2());
  group(c, f.conv3());
  group(c, f.fc1());
}

// conv2's input gradient as its 4 sub-pixel classes (SubPix): da1 straight from da2,
// masked by a1 > 0, in one grouped launch of 8-wave tiles (K = 2 x 2 taps x 64 = 256)
template <int PY, int PX>
auto subpix_op(const dq_cnn_params* p, const dq_cnn_acts* a, dq_cnn_acts* d, int B) {
  using SP = SubPix<Conv2, PY, PX>;
  return gemm_op<1, 1, 8, true>(SubPixDy<Conv2, PY, PX>{d->a2}, SubPixW<Conv2, PY, PX>{p->conv2_w},
                          EpiMaskPix<SP, Conv2::CI>{d->a1, a->a1}, B * SP::NY * SP::NX, Conv2::CI,
                          SP::K, SP::K);
}

// Backward of one layer: part 1 = weight/bias gradient, part 0 = input gradient.
// Layers 0..4 = fc2, fc1, conv3, conv2, conv1 (conv1 has no input gradient).
// Same tiles and split factors as the grouped schedule below: bitwise identical.
bool backward_layer(Ctx& c, const dq_cnn_params* p, const dq_cnn_params* g, int B, const float* x,
                    const dq_cnn_acts* a, const float* dout, dq_cnn_acts* d, int layer, int part) {
  const int NO = p->n_out;
  switch (layer * 2 + part) {
    case 0 * 2 + 1:   // fc2: dW2|db2 = dout^T [h | 1]
      gemm<4, 4, 1>(c, ColKScalar{dout, NO}, ColKOnes{a->h, kHidden},
                    EpiGrad{g->fc2_w, g->fc2_b, kHidden}, NO, kHidden + 1, B);
      return true;
    case 0 * 2 + 0:   // dh = (dout W2) * (h > 0)
      gemm<1, 1, 16>(c, RowKScalar{dout, NO}, ColK{p->fc2_w, kHidden}, EpiMask{d->h, a->h, kHidden},
                     B, kHidden, NO);
      return true;
    case 1 * 2 + 1:   // fc1: dW1|db1 = dh^T [a3 | 1]
      gemm<4, 4, 1>(c, ColK{d->h, kHidden}, ColKOnes{a->a3, kFlat},
                    EpiGrad{g->fc1_w, g->fc1_b, kFlat}, kHidden, kFlat + 1, B);
      return true;
    case 1 * 2 + 0:   // da3 = (dh W1) * (a3 > 0)
      gemm<1, 1, 16>(c, RowK{d->h, kHidden}, ColK{p->fc1_w, kFlat}, EpiMask{d->a3, a->a3, kFlat},
                     B, kFlat, kHidden);
      return true;
    case 2 * 2 + 1:   // conv3: dW3|db3 = da3^T [im2col(a2) | 1]
      gemm<1, 1, 16>(c, DyT<64>{d->a3}, Im2colT<Conv3>{a->a2},
                     EpiGrad{g->conv3_w, g->conv3_b, Conv3::K}, 64, Conv3::K + 1, B * 121, kSplitConvW);
      return true;
    case 2 * 2 + 0:   // da2 = col2im(da3, W3) * (a2 > 0)
      gemm<1, 1, 16>(c, Col2im<Conv3>{d->a3}, WeightT<Conv3>{p->conv3_w}, EpiMask{d->a2, a->a2, 64},
                     B * 121, 64, Conv3::K);
      return true;
    case 3 * 2 + 1:   // conv2: dW2|db2 = da2^T [im2col(a1) | 1]
      gemm<1, 1, 16>(c, DyT<64>{d->a2}, Im2colT<Conv2>{a->a1},
                     EpiGrad{g->conv2_w, g->conv2_b, Conv2::K}, 64, Conv2::K + 1, B * 121, kSplitConvW);
      return true;
    case 3 * 2 + 0:   // da1 = conv2^T(da2) * (a1 > 0), by sub-pixel class
      group(c, subpix_op<0, 0>(p, a, d, B), subpix_op<0, 1>(p, a, d, B),
            subpix_op<1, 0>(p, a, d, B), subpix_op<1, 1>(p, a, d, B));
      return true;
    case 4 * 2 + 1:   // conv1: dW1|db1 = da1^T [im2col(x) | 1]   (no input gradient needed)
      gemm<1, 1, 16>(c, DyT<32>{d->a1}, Im2colT<Conv1>{x}, EpiGrad{g->conv1_w, g->conv1_b, Conv1::K},
                     32, Conv1::K + 1, B * 441, kSplitConv1W);
      return true;
    default:
      return false;
  }
}

// The torso's backward (conv3 .. conv1 from d a3, e.g. IQN's d state) in four grouped
// launches of the full backward's tiles -- [dX conv3 | dW conv3 slabs] · [conv2's input
// gradient by sub-pixel class | dW conv2 slabs | sum conv3] · [dW conv1 slabs | sum conv2] ·
// [sum conv1] -- instead of nine per-layer GEMM and split-K-sum launches: bitwise the same
// gradients (same tiles, same slab order).
// kOpt (1 Adam, 2 RMSProp): the same four launches with the whole network's optimizer step
// spread over them -- [head_begin, head_end) (gradients final before the torso's backward) as
// float4 riders of launches 1-2, conv3 (final after launch 2) in launch 3, conv2 and conv1 in
// their split-K sums' epilogues (launches 3, 4; conv1's advances the beta powers).
template <int kOpt = 0>
void backward_torso_grouped(Ctx& c, const dq_cnn_params* p, const dq_cnn_params* g, int B,
                            const float* x, const dq_cnn_acts* a, dq_cnn_acts* d,
                            const AdamHost& opt = AdamHost{nullptr}, float* head_begin = nullptr,
                            float* head_end = nullptr) {
  using W16 = Tile<1, 1, 16>;
  const int K3 = B * 121, K1 = B * 441;
  const int ch3 = split_chunk(K3, kSplitConvW, W16::BKT), nz3 = (K3 + ch3 - 1) / ch3;
  const int ch1 = split_chunk(K1, kSplitConv1W, W16::BKT), nz1 = (K1 + ch1 - 1) / ch1;
  const size_t o3 = c.take((size_t)nz3 * 64 * (Conv3::K + 1));
  const size_t o2 = c.take((size_t)nz3 * 64 * (Conv2::K + 1));
  const size_t o1 = c.take((size_t)nz1 * 32 * (Conv1::K + 1));
  float* ws = c.ws;
  if (c.dry) return;
  auto dX_c3 = gemm_op<1, 1, 16>(Col2im<Conv3>{d->a3}, WeightT<Conv3>{p->conv3_w},
                                 EpiMask{d->a2, a->a2, 64}, K3, 64, Conv3::K, Conv3::K);
  auto dW_c3 = gemm_op<1, 1, 16>(DyT<64>{d->a3}, Im2colT<Conv3>{a->a2},
                                 EpiPartial{ws + o3, 64, Conv3::K + 1}, 64, Conv3::K + 1, K3, ch3);
  auto sum_c3 = ReduceOp<EpiGrad>{ws + o3, nz3, 64, Conv3::K + 1,
                                  EpiGrad{g->conv3_w, g->conv3_b, Conv3::K}};
  auto dW_c2 = gemm_op<1, 1, 16>(DyT<64>{d->a2}, Im2colT<Conv2>{a->a1},
                                 EpiPartial{ws + o2, 64, Conv2::K + 1}, 64, Conv2::K + 1, K3, ch3);
  auto sum_c2 = ReduceOp<EpiGrad>{ws + o2, nz3, 64, Conv2::K + 1,
                                  EpiGrad{g->conv2_w, g->conv2_b, Conv2::K}};
  auto dW_c1 = gemm_op<1, 1, 16>(DyT<32>{d->a1}, Im2colT<Conv1>{x},
                                 EpiPartial{ws + o1, 32, Conv1::K + 1}, 32, Conv1::K + 1, K1, ch1);
  auto sum_c1 = ReduceOp<EpiGrad>{ws + o1, nz1, 32, Conv1::K + 1,
                                  EpiGrad{g->conv1_w, g->conv1_b, Conv1::K}};
  // (the sub-pixel tiles unpaired here: two per block measured a tie for IQN)
  if constexpr (kOpt == 0) {
    group(c, dW_c3, dX_c3);
    group(c, dW_c2, subpix_op<0, 0>(p, a, d, B), subpix_op<0, 1>(p, a, d, B),
          subpix_op<1, 0>(p, a, d, B), subpix_op<1, 1>(p, a, d, B), sum_c3);
    group(c, dW_c1, sum_c2);
    group(c, sum_c1);
  } else {
    using GE = GradEpi<kOpt>;
    auto part = [&](float* w0, float* w1) { return OptPart<kOpt>::make(p, g, opt.a, w0, w1); };
    float* hm = head_begin + (((head_end - head_begin) / 2) & ~(int64_t)3);
    auto sum_c2o = ReduceOp<decltype(GE::make(0, 0, 0, 0, 0, opt, 0))>{
        ws + o2, nz3, 64, Conv2::K + 1,
        GE::make(g->conv2_w, g->conv2_b, Conv2::K, p->conv2_w, p->conv2_b, opt, 0)};
    auto sum_c1o = ReduceOp<decltype(GE::make(0, 0, 0, 0, 0, opt, 0))>{
        ws + o1, nz1, 32, Conv1::K + 1,
        GE::make(g->conv1_w, g->conv1_b, Conv1::K, p->conv1_w, p->conv1_b, opt, 1)};
    group(c, dW_c3, dX_c3, part(head_begin, hm));
    group(c, dW_c2, subpix_op<0, 0>(p, a, d, B), subpix_op<0, 1>(p, a, d, B),
          subpix_op<1, 0>(p, a, d, B), subpix_op<1, 1>(p, a, d, B), sum_c3,
          part(hm, head_end));
    group(c, dW_c1, sum_c2o, part(p->conv3_w, head_begin));
    group(c, sum_c1o);
  }
}

// Backward in 7 grouped launches (numbered 0..6 below):
//   0: dh                      (fc2 input grad)
//   1: dW fc2     | da3        (fc1 input grad)
//   2: dW fc1     | da2        (conv3 input grad)              [+ Adam fc2]
//   3: dW conv3 slabs | da1    (conv2 input grad, 4 sub-pixel GEMMs) [+ Adam fc1, 1st third]
//   4: sum conv3 slabs | dW conv2 slabs                        [+ Adam fc1, 2nd third]
//   5: sum conv2 slabs | dW conv1 slabs                        [+ Adam fc1, 3rd third]
//   6: sum conv1 slabs                                         [+ Adam conv2, conv3]
// or, kHeadFrom = 5, in 6 (the Rainbow fast path starts at 1, dh coming from the loss):
//   4: sum conv3 slabs | dW conv2 slabs | dW conv1 slabs       [+ Adam fc1, 2nd third]
//   5: sum conv2 slabs | sum conv1 slabs               [+ Adam fc1, 3rd third, conv3]
// With kOpt (1 TF1 Adam, 2 TF1 RMSProp) the optimizer step is spread as bracketed: float4
// AdamOps / RmsOps over ranges
// whose gradients are final and whose weights have had their last read; conv1's
// split-K sum applies it in its epilogue (and advances the beta powers).  The
// optimizer's 47 MB of traffic then overlaps the latency-bound GEMM launches
// instead of running as an 18 us launch of its own.
// Each GEMM writes its gradient/activation exactly as the per-layer form does
// (same tiles, same summation order), so the two are bitwise identical.
// kHeadFrom: the launch of the head network's conv1 (3: conv1..conv3 and the fc1
// slabs in launches 3..6; 4: conv1..conv3 in launches 4..6, its fc1 slabs left to
// forward_fused; 5: conv1, conv2 in launches 4, 5 of the six-launch schedule, conv3
// and the fc1 slabs left to forward_fused).  Riders are numbered from launch `first`: rider i rides in launch
// first + i.
template <int kOpt, int kHeadFrom = 3>
void backward_grouped(Ctx& c, const dq_cnn_params* p, const dq_cnn_params* g, int B,
                      const float* x, const dq_cnn_acts* a, const float* dout, dq_cnn_acts* d,
                      const AdamHost& opt, int first = 0, int last = 7,
                      const RiderDesc* riders = nullptr, int n_riders = 0,
                      const FwdOps* head = nullptr) {
  const int NO = p->n_out;
  using GE = GradEpi<kOpt>;
  using W16 = Tile<1, 1, 16>;
  // workspace regions (ops of one launch never share one)
  const int K3 = B * 121, K1 = B * 441;
  const int ch3 = split_chunk(K3, kSplitConvW, W16::BKT), nz3 = (K3 + ch3 - 1) / ch3;
  const int ch1 = split_chunk(K1, kSplitConv1W, W16::BKT), nz1 = (K1 + ch1 - 1) / ch1;
  const size_t o3 = c.take((size_t)nz3 * 64 * (Conv3::K + 1));
  const size_t o2 = c.take((size_t)nz3 * 64 * (Conv2::K + 1));
  const size_t o1 = c.take((size_t)nz1 * 32 * (Conv1::K + 1));
  float* ws = c.ws;
  if (c.dry) return;
  auto dX_fc2 = gemm_op<1, 1, 16>(RowKScalar{dout, NO}, ColK{p->fc2_w, kHidden},
                                  EpiMask{d->h, a->h, kHidden}, B, kHidden, NO, NO);
  auto dW_fc2 = gemm_op<4, 4, 1>(ColKScalar{dout, NO}, ColKOnes{a->h, kHidden},
                                 EpiGrad{g->fc2_w, g->fc2_b, kHidden},
                                 NO, kHidden + 1, B, B);
  auto dX_fc1 = gemm_op<1, 1, 16, kB1Late>(RowK{d->h, kHidden}, ColK{p->fc1_w, kFlat},
                                  EpiMask{d->a3, a->a3, kFlat}, B, kFlat, kHidden, kHidden);
  auto dW_fc1 = gemm_op<4, 4, 1>(ColK{d->h, kHidden}, ColKOnes{a->a3, kFlat},
                                 EpiGrad{g->fc1_w, g->fc1_b, kFlat},
                                 kHidden, kFlat + 1, B, B);
  auto dX_c3 = gemm_op<1, 1, 16>(Col2im<Conv3>{d->a3}, WeightT<Conv3>{p->conv3_w},
                                 EpiMask{d->a2, a->a2, 64}, K3, 64, Conv3::K, Conv3::K);
  auto dW_c3 = gemm_op<1, 1, 16>(DyT<64>{d->a3}, Im2colT<Conv3>{a->a2},
                                 EpiPartial{ws + o3, 64, Conv3::K + 1}, 64, Conv3::K + 1, K3, ch3);
  // two of the 8-wave sub-pixel tiles per 16-wave block of the grouped launch (+0.7%)
  auto sp_op = [](auto op) { return PairOp<decltype(op)>{op}; };
  auto sp00 = sp_op(subpix_op<0, 0>(p, a, d, B));
  auto sp01 = sp_op(subpix_op<0, 1>(p, a, d, B));
  auto sp10 = sp_op(subpix_op<1, 0>(p, a, d, B));
  auto sp11 = sp_op(subpix_op<1, 1>(p, a, d, B));
  auto sum_c3 = ReduceOp<EpiGrad>{ws + o3, nz3, 64, Conv3::K + 1,
                                  EpiGrad{g->conv3_w, g->conv3_b, Conv3::K}};
  auto dW_c2 = gemm_op<1, 1, 16>(DyT<64>{d->a2}, Im2colT<Conv2>{a->a1},
                                 EpiPartial{ws + o2, 64, Conv2::K + 1}, 64, Conv2::K + 1, K3, ch3);
  auto sum_c2 = ReduceOp<EpiGrad>{ws + o2, nz3, 64, Conv2::K + 1,
                                  EpiGrad{g->conv2_w, g->conv2_b, Conv2::K}};
  auto dW_c1 = gemm_op<1, 1, 16>(DyT<32>{d->a1}, Im2colT<Conv1>{x},
                                 EpiPartial{ws + o1, 32, Conv1::K + 1}, 32, Conv1::K + 1, K1, ch1);
  auto sum_c1 = ReduceOp<decltype(GE::make(0, 0, 0, 0, 0, opt, 0))>{
      ws + o1, nz1, 32, Conv1::K + 1,
      GE::make(g->conv1_w, g->conv1_b, Conv1::K, p->conv1_w, p->conv1_b, opt, 1)};
  auto in = [&](int i) { return first <= i && i < last; };
  auto rd = [&](int i) {   // rider of launch i
    return i >= first && i - first < n_riders ? riders + (i - first) : nullptr;
  };
  if constexpr (kOpt != 0) {
    {
      // The optimizer spread over the launches after each gradient is final and each
      // weight's last read.
      auto part = [&](float* w0, float* w1) { return OptPart<kOpt>::make(p, g, opt.a, w0, w1); };
      float* f0 = p->fc1_w;
      float* f3 = p->fc2_w;                          // fc1_w .. fc1_b (+ pad)
      // fc1's range op split points (kHeadFrom < 5), in 24ths of the range: thirds
      float* f1 = f0 + (((f3 - f0) * 8 / 24) & ~(int64_t)3);
      float* f2 = f0 + (((f3 - f0) * 16 / 24) & ~(int64_t)3);
      if constexpr (kHeadFrom >= 5) {
        // fc1 and fc2: TF1 Adam / RMSProp in their weight-gradient GEMMs' vector epilogues,
        // launch 2 (fc1's instead of range ops over fc1 in launches 3-5 reading the stored
        // gradient back: +0.6-1.2%; fc2's moved there from launch 1 so launch 1 keeps only
        // dX fc1 (+ rider), one round of blocks: +0.8%).  conv2 and conv1 in
        // their split-K sums' epilogues, conv3 as a range op in the last launch.
        auto dW_fc1a = gemm_op<4, 4, 1>(ColK{d->h, kHidden}, ColKOnes{a->a3, kFlat},
                                        Fc1EpiOpt<kOpt>::make(p, g, opt.a), kHidden, kFlat + 1,
                                        B, B);
        auto dW_fc2a = gemm_op<4, 4, 1>(ColKScalar{dout, NO}, ColKOnes{a->h, kHidden},
                                        Fc2EpiOpt<kOpt>::make(p, g, opt.a), NO, kHidden + 1, B, B);
        auto sum_c2a = ReduceOp<decltype(GE::make(0, 0, 0, 0, 0, opt, 0))>{
            ws + o2, nz3, 64, Conv2::K + 1,
            GE::make(g->conv2_w, g->conv2_b, Conv2::K, p->conv2_w, p->conv2_b, opt, 0)};
        if (in(0)) group_r(c, rd(0), dX_fc2);
        if (in(1)) group_r(c, rd(1), dX_fc1);
        if (in(2)) group_r(c, rd(2), dW_fc1a, dX_c3, dW_fc2a);
        if (kHeadFrom == 6) {
          // conv2's weight-gradient slabs (they need only da2) beside conv3's in launch 3
          // (+0.9%), the head's conv1 in launch 5, its conv2 and conv3 in the next forward.
          // (Launch 3 with the sub-pixel tiles first: 19.6 instead of 17.0 us -- conv3's last
          // slabs then wait for the sub-pixel tiles' slots, tools/group_stamps.py)
          if (in(3)) group_r(c, rd(3), dW_c3, sp00, sp01, sp10, sp11, dW_c2);
          if (in(4)) group_r(c, rd(4), sum_c3, dW_c1);
          if (in(5)) {
            if (head)
              group_r(c, rd(5), sum_c2a, sum_c1, part(p->conv3_w, p->fc1_w), head->conv1());
            else
              group_r(c, rd(5), sum_c2a, sum_c1, part(p->conv3_w, p->fc1_w));
          }
          return;
        }
        // five launches: conv2's input gradient by sub-pixel class needs only da2, so conv1's
        // weight-gradient slabs join launch 4 and the split-K sums end the backward in launch 5
        if (in(3)) group_r(c, rd(3), dW_c3, sp00, sp01, sp10, sp11);
        if (head) {
          if (in(4)) group_r(c, rd(4), sum_c3, dW_c2, dW_c1, head->conv1());
          if (in(5))
            group_r(c, rd(5), sum_c2a, sum_c1, part(p->conv3_w, p->fc1_w), head->conv2());
        } else {
          if (in(4)) group_r(c, rd(4), sum_c3, dW_c2, dW_c1);
          if (in(5)) group_r(c, rd(5), sum_c2a, sum_c1, part(p->conv3_w, p->fc1_w));
        }
        return;
      }
      if (in(0)) group_r(c, rd(0), dX_fc2);
      if (in(1)) group_r(c, rd(1), dW_fc2, dX_fc1);
      if (in(2)) group_r(c, rd(2), dW_fc1, dX_c3, part(p->fc2_w, p->fc2_b + NO));
      if (head) {
if constexpr (kHeadFrom == 4) {
          if (in(3)) group_r(c, rd(3), dW_c3, sp00, sp01, sp10, sp11, part(f0, f1));
          if (in(4)) group_r(c, rd(4), sum_c3, dW_c2, part(f1, f2), head->conv1());
          if (in(5)) group_r(c, rd(5), sum_c2, dW_c1, part(f2, f3), head->conv2());
          if (in(6)) group_r(c, rd(6), sum_c1, part(p->conv2_w, p->fc1_w), head->conv3<kB6Late>());
        } else {
          if (in(3)) group_r(c, rd(3), dW_c3, sp00, sp01, sp10, sp11, part(f0, f1), head->conv1());
          if (in(4)) group_r(c, rd(4), sum_c3, dW_c2, part(f1, f2), head->conv2());
          if (in(5)) group_r(c, rd(5), sum_c2, dW_c1, part(f2, f3), head->conv3());
          if (in(6)) group_r(c, rd(6), sum_c1, part(p->conv2_w, p->fc1_w), head->fc1());
        }
        return;
      }
      if (in(3)) group_r(c, rd(3), dW_c3, sp00, sp01, sp10, sp11, part(f0, f1));
      if (in(4)) group_r(c, rd(4), sum_c3, dW_c2, part(f1, f2));
      if (in(5)) group_r(c, rd(5), sum_c2, dW_c1, part(f2, f3));
      if (in(6)) group_r(c, rd(6), sum_c1, part(p->conv2_w, p->fc1_w));
      return;
    }
  }
  if (in(0)) group_r(c, rd(0), dX_fc2);
  if (in(1)) group_r(c, rd(1), dW_fc2, dX_fc1);
  if (in(2)) group_r(c, rd(2), dW_fc1, dX_c3);
  if constexpr (kHeadFrom >= 5) {
    if (kHeadFrom == 6) {            // as the Adam form: conv2's dW slabs in launch 3
      if (in(3)) group_r(c, rd(3), dW_c3, sp00, sp01, sp10, sp11, dW_c2);
      if (in(4)) group_r(c, rd(4), sum_c3, dW_c1);
      if (in(5)) {
        if (head)
          group_r(c, rd(5), sum_c2, sum_c1, head->conv1());
        else
          group_r(c, rd(5), sum_c2, sum_c1);
      }
      return;
    }
    if (in(3)) group_r(c, rd(3), dW_c3, sp00, sp01, sp10, sp11);
    if (head) {
      if (in(4)) group_r(c, rd(4), sum_c3, dW_c2, dW_c1, head->conv1());
      if (in(5)) group_r(c, rd(5), sum_c2, sum_c1, head->conv2());
    } else {
      if (in(4)) group_r(c, rd(4), sum_c3, dW_c2, dW_c1);
      if (in(5)) group_r(c, rd(5), sum_c2, sum_c1);
    }
    return;
  }
  if (head) {
    if constexpr (kHeadFrom == 4) {
      if (in(3)) group_r(c, rd(3), dW_c3, sp00, sp01, sp10, sp11);
      if (in(4)) group_r(c, rd(4), sum_c3, dW_c2, head->conv1());
      if (in(5)) group_r(c, rd(5), sum_c2, dW_c1, head->conv2());
      if (in(6)) group_r(c, rd(6), sum_c1, head->conv3());
    } else {
      if (in(3)) group_r(c, rd(3), dW_c3, sp00, sp01, sp10, sp11, head->conv1());
      if (in(4)) group_r(c, rd(4), sum_c3, dW_c2, head->conv2());
      if (in(5)) group_r(c, rd(5), sum_c2, dW_c1, head->conv3());
      if (in(6)) group_r(c, rd(6), sum_c1, head->fc1());
    }
    return;
  }
  if (in(3)) group_r(c, rd(3), dW_c3, sp00, sp01, sp10, sp11);
  if (in(4)) group_r(c, rd(4), sum_c3, dW_c2);
  if (in(5)) group_r(c, rd(5), sum_c2, dW_c1);
  if (in(6)) group_r(c, rd(6), sum_c1);
}

// The fused Rainbow schedule's backward (backward_grouped<1, 6>, first 1) with the data-
// parallel exchange over peer memory (dq_peer) in place of the fused optimizer's fc and conv
// updates -- the gradients are stored, the reduce-scatter + Adam of this rank's slice rides
// in launches 3 and 4, the parameter publication in launch 5, and one launch more (6) holds
// the conv bucket's exchange + Adam and the all-gather.  Same tiles and summation orders as
// backward_grouped: with world 1 the parameters, moments and gradients are bitwise those of
// the single learner's fused step.
void backward_peer(Ctx& c, const dq_cnn_params* p, const dq_cnn_params* g, int B, const float* x,
                   const dq_cnn_acts* a, const float* dout, dq_cnn_acts* d, const dq_adam_args* oa,
                   const RiderDesc* riders, int n_riders, const FwdOps* head, const dq_peer& P,
                   bool defer_ag) {
  const int NO = p->n_out;
  using W16 = Tile<1, 1, 16>;
  const int K3 = B * 121, K1 = B * 441;
  const int ch3 = split_chunk(K3, kSplitConvW, W16::BKT), nz3 = (K3 + ch3 - 1) / ch3;
  const int ch1 = split_chunk(K1, kSplitConv1W, W16::BKT), nz1 = (K1 + ch1 - 1) / ch1;
  const size_t o3 = c.take((size_t)nz3 * 64 * (Conv3::K + 1));
  const size_t o2 = c.take((size_t)nz3 * 64 * (Conv2::K + 1));
  const size_t o1 = c.take((size_t)nz1 * 32 * (Conv1::K + 1));
  float* ws = c.ws;
  if (c.dry) return;
  auto dX_fc1 = gemm_op<1, 1, 16, kB1Late>(RowK{d->h, kHidden}, ColK{p->fc1_w, kFlat},
                                           EpiMask{d->a3, a->a3, kFlat}, B, kFlat, kHidden, kHidden);
  auto dW_fc1 = gemm_op<4, 4, 1>(ColK{d->h, kHidden}, ColKOnes{a->a3, kFlat},
                                 EpiGrad{g->fc1_w, g->fc1_b, kFlat}, kHidden, kFlat + 1, B, B);
  auto dW_fc2 = gemm_op<4, 4, 1>(ColKScalar{dout, NO}, ColKOnes{a->h, kHidden},
                                 EpiGrad{g->fc2_w, g->fc2_b, kHidden}, NO, kHidden + 1, B, B);
  auto dX_c3 = gemm_op<1, 1, 16>(Col2im<Conv3>{d->a3}, WeightT<Conv3>{p->conv3_w},
                                 EpiMask{d->a2, a->a2, 64}, K3, 64, Conv3::K, Conv3::K);
  auto dW_c3 = gemm_op<1, 1, 16>(DyT<64>{d->a3}, Im2colT<Conv3>{a->a2},
                                 EpiPartial{ws + o3, 64, Conv3::K + 1}, 64, Conv3::K + 1, K3, ch3);
  auto sp_op = [](auto op) { return PairOp<decltype(op)>{op}; };
  auto sp00 = sp_op(subpix_op<0, 0>(p, a, d, B));
  auto sp01 = sp_op(subpix_op<0, 1>(p, a, d, B));
  auto sp10 = sp_op(subpix_op<1, 0>(p, a, d, B));
  auto sp11 = sp_op(subpix_op<1, 1>(p, a, d, B));
  auto sum_c3 = ReduceOp<EpiGrad>{ws + o3, nz3, 64, Conv3::K + 1,
                                  EpiGrad{g->conv3_w, g->conv3_b, Conv3::K}};
  auto dW_c2 = gemm_op<1, 1, 16>(DyT<64>{d->a2}, Im2colT<Conv2>{a->a1},
                                 EpiPartial{ws + o2, 64, Conv2::K + 1}, 64, Conv2::K + 1, K3, ch3);
  auto sum_c2 = ReduceOp<EpiGrad>{ws + o2, nz3, 64, Conv2::K + 1,
                                  EpiGrad{g->conv2_w, g->conv2_b, Conv2::K}};
  auto dW_c1 = gemm_op<1, 1, 16>(DyT<32>{d->a1}, Im2colT<Conv1>{x},
                                 EpiPartial{ws + o1, 32, Conv1::K + 1}, 32, Conv1::K + 1, K1, ch1);
  auto sum_c1 = ReduceOp<EpiGrad>{ws + o1, nz1, 32, Conv1::K + 1,
                                  EpiGrad{g->conv1_w, g->conv1_b, Conv1::K}};
  const AdamDev od{oa->state, oa->slot, oa->lr, oa->beta1, oa->beta2, oa->epsilon, 1};
  // this rank's slice of [lo, n), halves in launches 3 and 4; one float4 per thread
  const int64_t S = (P.n - P.lo) / P.world;
  const int64_t s0 = P.lo + (int64_t)P.rank * S, sm = s0 + ((S / 2) & ~(int64_t)3), s1 = s0 + S;
  auto blocks_for = [](int64_t floats, int per_thread) {
    return (int)std::min<int64_t>(kPeerMaxBlocks,
                                  std::max<int64_t>(1, (floats / 4 + per_thread * kGroupT - 1) /
                                                           (per_thread * kGroupT)));
  };
  auto rs = [&](int64_t b0, int64_t b1) {
    return PeerRsAdamOp{P, od, oa->var, oa->m, oa->v, b0, b1, blocks_for(b1 - b0, 2)};
  };
  const int nc = std::max(kPubBlocks, blocks_for(P.lo, 2));   // its first blocks publish
  const int na = blocks_for((P.n - P.lo) * (P.world - 1) / P.world, 4);
  auto rd = [&](int i) { return i >= 1 && i - 1 < n_riders ? riders + (i - 1) : nullptr; };
  group_r(c, rd(1), dX_fc1);
  group_r(c, rd(2), dW_fc1, dX_c3, dW_fc2);
  group_r(c, rd(3), PeerPubOp{P, kPeerGrad}, dW_c3, sp00, sp01, sp10, sp11, dW_c2, rs(s0, sm));
  group_r(c, rd(4), sum_c3, dW_c1, rs(sm, s1));
  // launch 5: this rank's slice published, the others' gathered (world 1: nothing to gather;
  // defer_ag: the head of the range (AgParts), the rest by the next forward's conv launches)
  const PeerAgOp ag = defer_ag ? AgParts{&P, oa->var}.head()
                               : PeerAgOp{P, oa->var, na, 0, 0, INT64_MAX};
  if (P.world > 1)
    group_r(c, rd(5), PeerPubOp{P, kPeerParam}, sum_c2, sum_c1, ag);
  else
    group_r(c, rd(5), PeerPubOp{P, kPeerParam}, sum_c2, sum_c1);
  // launch 6: the exchange's blocks first (they publish, then wait), the target head's conv1
  // beside them -- it reads only the target parameters and the batch gathered in launch 4,
  // so its tiles fill the CUs while the exchange waits for the other learners
  if (head)
    group(c, PeerExchOp{P, od, oa->var, oa->m, oa->v, nc}, head->conv1());
  else
    group(c, PeerExchOp{P, od, oa->var, oa->m, oa->v, nc});
}

// backward_grouped with the runtime head_from (7: the whole target head runs in the next
// forward, so the five-launch schedule carries none of it)
template <int kOpt>
void backward_head_from(Ctx& c, const dq_cnn_params* p, const dq_cnn_params* g, int B,
                        const float* x, const dq_cnn_acts* a, const float* dout, dq_cnn_acts* d,
                        const AdamHost& opt, int first, int last, const RiderDesc* r, int n_riders,
                        const FwdOps* hp, int head_from) {
  if (head_from == 7)
    backward_grouped<kOpt, 5>(c, p, g, B, x, a, dout, d, opt, first, last, r, n_riders, nullptr);
  else if (head_from == 6)
    backward_grouped<kOpt, 6>(c, p, g, B, x, a, dout, d, opt, first, last, r, n_riders, hp);
  else if (head_from == 5)
    backward_grouped<kOpt, 5>(c, p, g, B, x, a, dout, d, opt, first, last, r, n_riders, hp);
  else if (head_from == 4)
    backward_grouped<kOpt, 4>(c, p, g, B, x, a, dout, d, opt, first, last, r, n_riders, hp);
  else
    backward_grouped<kOpt>(c, p, g, B, x, a, dout, d, opt, first, last, r, n_riders, hp);
}

}  // namespace cnn
}  // namespace dq

using namespace dq;
using namespace dq::cnn;

// the fused optimizer needs the parameters (and gradients) in one flat buffer, in
// conv1..fc2 order, with the float4 Adam range 16-byte aligned
static int check_adam(const dq_cnn_params* p, const dq_cnn_params* g, const dq_adam_args* opt) {
  DQ_CHECK_ARG(opt->kind == DQ_OPT_ADAM || opt->kind == DQ_OPT_RMSPROP, "unknown optimizer kind");
  if (opt->kind == DQ_OPT_ADAM)
    DQ_CHECK_ARG(opt->var && opt->m && opt->v && opt->state && (opt->slot == 0 || opt->slot == 1),
                 "adam args: var, m, v, state and slot 0/1 required");
  else
    DQ_CHECK_ARG(opt->var && opt->m && opt->v && (!opt->centered || opt->mg),
                 "rmsprop args: var, ms (m), mom (v) and, centered, mg required");
  const float* w[10] = {p->conv1_w, p->conv1_b, p->conv2_w, p->conv2_b, p->conv3_w,
                        p->conv3_b, p->fc1_w,  p->fc1_b,  p->fc2_w,  p->fc2_b};
  const float* gw[10] = {g->conv1_w, g->conv1_b, g->conv2_w, g->conv2_b, g->conv3_w,
                         g->conv3_b, g->fc1_w,  g->fc1_b,  g->fc2_w,  g->fc2_b};
  for (int i = 0; i < 10; ++i) {
    DQ_CHECK_ARG(w[i] >= opt->var && (i == 0 || w[i] > w[i - 1]),
                 "parameters must live in the flat buffer opt->var in conv1..fc2 order");
    DQ_CHECK_ARG(gw[i] - g->conv1_w == w[i] - p->conv1_w,
                 "gradients must have the parameters' flat layout");
  }
  DQ_CHECK_ARG(((p->conv2_w - opt->var) & 3) == 0 && ((g->conv2_w - g->conv1_w) & 3) == 0,
               "16-byte aligned parameter views required");
  return DQ_OK;
}

extern "C" {

int dq_cnn_forward(const dq_cnn_params* p, int32_t batch, const float* x, dq_cnn_acts* a,
                   float* ws, void* stream) {
  DQ_CHECK_ARG(p && a && x && ws && batch >= 1, "null argument");
  DQ_CHECK_ARG(p->in_channels == 4 && p->n_out >= 1, "the Nature CNN takes 84x84x4 NHWC input");
  Ctx c{(hipStream_t)stream, ws, false, 0};
  forward(c, p, batch, x, a);
  DQ_CHECK_LAUNCH("dq_cnn_forward");
  return DQ_OK;
}

int dq_cnn_forward_pair(const dq_cnn_params* p0, const float* x0, dq_cnn_acts* a0, float* ws0,
                        const dq_cnn_params* p1, const float* x1, dq_cnn_acts* a1, float* ws1,
                        int32_t batch, void* stream) {
  DQ_CHECK_ARG(p0 && a0 && x0 && ws0 && p1 && a1 && x1 && ws1 && batch >= 1, "null argument");
  DQ_CHECK_ARG(p0->in_channels == 4 && p1->in_channels == 4 && p0->n_out >= 1 && p1->n_out >= 1,
               "the Nature CNN takes 84x84x4 NHWC input");
  DQ_CHECK_ARG(ws0 != ws1, "the two networks need separate workspaces");
  Ctx c0{(hipStream_t)stream, ws0, false, 0}, c1{(hipStream_t)stream, ws1, false, 0};
  forward_pair(c0, c1, p0, x0, a0, p1, x1, a1, batch);
  DQ_CHECK_LAUNCH("dq_cnn_forward_pair");
  return DQ_OK;
}

int dq_cnn_forward_head(const dq_cnn_params* p, int32_t batch, const float* x, dq_cnn_acts* a,
                        float* ws, void* stream) {
  DQ_CHECK_ARG(p && a && x && ws && batch >= 1, "null argument");
  DQ_CHECK_ARG(p->in_channels == 4 && p->n_out >= 1, "the Nature CNN takes 84x84x4 NHWC input");
  Ctx c{(hipStream_t)stream, ws, false, 0};
  forward_head(c, FwdOps{p, x, a, ws, batch});
  DQ_CHECK_LAUNCH("dq_cnn_forward_head");
  return DQ_OK;
}

int dq_cnn_forward_with_tail(const dq_cnn_params* p0, const float* x0, dq_cnn_acts* a0, float* ws0,
                             const dq_cnn_params* p1, dq_cnn_acts* a1, float* ws1, int32_t batch,
                             void* stream) {
  DQ_CHECK_ARG(p0 && a0 && x0 && ws0 && p1 && a1 && ws1 && batch >= 1, "null argument");
  DQ_CHECK_ARG(p0->in_channels == 4 && p1->in_channels == 4 && p0->n_out >= 1 && p1->n_out >= 1,
               "the Nature CNN takes 84x84x4 NHWC input");
  DQ_CHECK_ARG(ws0 != ws1, "the two networks need separate workspaces");
  Ctx c0{(hipStream_t)stream, ws0, false, 0}, c1{(hipStream_t)stream, ws1, false, 0};
  forward_with_tail(c0, c1, FwdOps{p0, x0, a0, ws0, batch}, FwdOps{p1, nullptr, a1, ws1, batch});
  DQ_CHECK_LAUNCH("dq_cnn_forward_with_tail");
  return DQ_OK;
}

int dq_cnn_forward_fused(const dq_cnn_params* p0, const float* x0, dq_cnn_acts* a0, float* ws0,
                         const dq_cnn_params* p1, const float* x1, dq_cnn_acts* a1, float* ws1,
                         int32_t batch, int32_t fc1_1, void* stream) {
  DQ_CHECK_ARG(p0 && a0 && x0 && ws0 && p1 && a1 && ws1 && batch >= 1, "null argument");
  DQ_CHECK_ARG(p0->in_channels == 4 && p1->in_channels == 4 && p0->n_out >= 1 && p1->n_out >= 1,
               "the Nature CNN takes 84x84x4 NHWC input");
  DQ_CHECK_ARG(ws0 != ws1, "the two networks need separate workspaces");
  Ctx c0{(hipStream_t)stream, ws0, false, 0}, c1{(hipStream_t)stream, ws1, false, 0};
  DQ_CHECK_ARG((fc1_1 & 12) != 12, "flags 4 (convs only) and 8 (fc layers only) exclude each other");
  DQ_CHECK_ARG(!(fc1_1 & 32) || x1, "flag 32 (net 1's conv1) needs x1");
  forward_fused(c0, c1, FwdOps{p0, x0, a0, ws0, batch}, FwdOps{p1, x1, a1, ws1, batch},
                (fc1_1 & 1) != 0, (fc1_1 & 2) != 0, (fc1_1 & 8) == 0, (fc1_1 & 4) == 0,
                (fc1_1 & 16) != 0, (fc1_1 & 32) != 0);
  DQ_CHECK_LAUNCH("dq_cnn_forward_fused");
  return DQ_OK;
}

size_t dq_cnn_fc2_parts_offset(int32_t batch) { return FwdOps::part_offset(batch); }

int dq_cnn_forward_fused_c51(const dq_cnn_params* p0, const float* x0, dq_cnn_acts* a0, float* ws0,
                             const dq_cnn_params* p1, dq_cnn_acts* a1, float* ws1, int32_t batch,
                             const dq_c51_target* c51, int32_t flags, void* stream) {
  DQ_CHECK_ARG(p0 && a0 && x0 && ws0 && p1 && a1 && ws1 && c51 && batch >= 1, "null argument");
  DQ_CHECK_ARG(p0->in_channels == 4 && p1->in_channels == 4 && p0->n_out >= 1 && p1->n_out >= 1,
               "the Nature CNN takes 84x84x4 NHWC input");
  DQ_CHECK_ARG(ws0 != ws1, "the two networks need separate workspaces");
  DQ_CHECK_ARG((flags & 12) != 12, "flags 4 (convs only) and 8 (fc layers only) exclude each other");
  DQ_CHECK_ARG(c51->rewards && c51->terminals && c51->support && c51->m_out, "null C51 argument");
  DQ_CHECK_ARG(c51->num_atoms >= 2 && c51->num_atoms <= 64 && p1->n_out % c51->num_atoms == 0,
               "n_out must be num_actions * num_atoms, 2 <= num_atoms <= 64");
  const int A = p1->n_out / c51->num_atoms;
  DQ_CHECK_ARG(A <= 4 * kC51TgtMaxWaveRows, "the riding C51 target half takes at most 16 actions");
  Ctx c0{(hipStream_t)stream, ws0, false, 0}, c1{(hipStream_t)stream, ws1, false, 0};
  const FwdOps f0{p0, x0, a0, ws0, batch}, f1{p1, nullptr, a1, ws1, batch};
  const int NO = p1->n_out;
  C51Target t{LogitsParts{ws1 + FwdOps::part_offset(batch), p1->fc2_b, (int64_t)batch * NO,
                          FcHeadOp::kBands, NO},
              c51->rewards, c51->terminals, c51->support, batch, A, c51->num_atoms,
              c51->cumulative_gamma, c51->m_out, c51->target_logits_out};
  forward_fused_c51(c0, c1, f0, f1, t, (flags & 8) == 0, (flags & 4) == 0);
  DQ_CHECK_LAUNCH("dq_cnn_forward_fused_c51");
  return DQ_OK;
}


int dq_cnn_backward(const dq_cnn_params* p, const dq_cnn_params* g, int32_t batch, const float* x,
                    const dq_cnn_acts* a, const float* dout, dq_cnn_acts* d, float* ws,
                    void* stream) {
  DQ_CHECK_ARG(p && g && a && d && x && dout && ws && batch >= 1, "null argument");
  DQ_CHECK_ARG(p->in_channels == 4 && p->n_out >= 1, "the Nature CNN takes 84x84x4 NHWC input");
  Ctx c{(hipStream_t)stream, ws, false, 0};
  backward_grouped<0>(c, p, g, batch, x, a, dout, d, AdamHost{nullptr});
  DQ_CHECK_LAUNCH("dq_cnn_backward");
  return DQ_OK;
}

int dq_cnn_backward_adam(const dq_cnn_params* p, const dq_cnn_params* g, int32_t batch,
                         const float* x, const dq_cnn_acts* a, const float* dout, dq_cnn_acts* d,
                         float* ws, const dq_adam_args* opt, void* stream) {
  DQ_CHECK_ARG(p && g && a && d && x && dout && ws && opt && batch >= 1, "null argument");
  DQ_CHECK_ARG(p->in_channels == 4 && p->n_out >= 1, "the Nature CNN takes 84x84x4 NHWC input");
  const int rc = check_adam(p, g, opt);
  if (rc != DQ_OK) return rc;
  Ctx c{(hipStream_t)stream, ws, false, 0};
  if (opt->kind == DQ_OPT_RMSPROP)
    backward_grouped<2>(c, p, g, batch, x, a, dout, d, AdamHost{opt});
  else
    backward_grouped<1>(c, p, g, batch, x, a, dout, d, AdamHost{opt});
  DQ_CHECK_LAUNCH("dq_cnn_backward_adam");
  return DQ_OK;
}

int dq_cnn_backward_groups(const dq_cnn_params* p, const dq_cnn_params* g, int32_t batch,
                           const float* x, const dq_cnn_acts* a, const float* dout,
                           dq_cnn_acts* d, float* ws, int32_t first, int32_t last, void* stream) {
  DQ_CHECK_ARG(p && g && a && d && x && dout && ws && batch >= 1, "null argument");
  DQ_CHECK_ARG(p->in_channels == 4 && p->n_out >= 1, "the Nature CNN takes 84x84x4 NHWC input");
  DQ_CHECK_ARG(0 <= first && first <= last && last <= 7, "groups must satisfy 0 <= first <= last <= 7");
  Ctx c{(hipStream_t)stream, ws, false, 0};
  backward_grouped<0>(c, p, g, batch, x, a, dout, d, AdamHost{nullptr}, first, last);
  DQ_CHECK_LAUNCH("dq_cnn_backward_groups");
  return DQ_OK;
}

int dq_cnn_backward_riders(const dq_cnn_params* p, const dq_cnn_params* g, int32_t batch,
                           const float* x, const dq_cnn_acts* a, const float* dout,
                           dq_cnn_acts* d, float* ws, const dq_rider* riders, int32_t n_riders,
                           const dq_adam_args* opt, const dq_cnn_net* head, int32_t head_from,
                           int32_t first, int32_t last, void* stream) {
  DQ_CHECK_ARG(p && g && a && d && x && dout && ws && batch >= 1, "null argument");
  DQ_CHECK_ARG(p->in_channels == 4 && p->n_out >= 1, "the Nature CNN takes 84x84x4 NHWC input");
  DQ_CHECK_ARG(0 <= n_riders && n_riders <= 7 && (riders || n_riders == 0),
               "at most one rider per grouped launch (7)");
  DQ_CHECK_ARG(0 <= first && first <= last && last <= 7, "groups must satisfy 0 <= first <= last <= 7");
  DQ_CHECK_ARG(!opt || (first <= 1 && last == 7), "the fused optimizer needs the whole backward");
  DQ_CHECK_ARG(head_from >= 3 && head_from <= 7, "head_from must be in [3, 7]");
  RiderDesc r[7];
  for (int i = 0; i < n_riders; ++i) {
    memcpy(&r[i], &riders[i], sizeof(RiderDesc));
    DQ_CHECK_ARG(r[i].kind >= kRiderNone && r[i].kind <= kRiderSetSample, "corrupt rider");
  }
  FwdOps hf{};
  if (head) {
    DQ_CHECK_ARG(head->p && head->x && head->a && head->ws, "null head network field");
    DQ_CHECK_ARG(head->p->in_channels == 4, "the Nature CNN takes 84x84x4 NHWC input");
    DQ_CHECK_ARG(head->ws != ws, "the head network needs its own workspace");
    hf = FwdOps{head->p, head->x, head->a, head->ws, batch};
  }
  Ctx c{(hipStream_t)stream, ws, false, 0};
  const FwdOps* hp = head ? &hf : nullptr;
  if (opt) {
    const int rc = check_adam(p, g, opt);
    if (rc != DQ_OK) return rc;
    if (opt->kind == DQ_OPT_RMSPROP)
      backward_head_from<2>(c, p, g, batch, x, a, dout, d, AdamHost{opt}, first, last, r, n_riders,
                            hp, head_from);
    else
      backward_head_from<1>(c, p, g, batch, x, a, dout, d, AdamHost{opt}, first, last, r, n_riders,
                            hp, head_from);
  } else {
    backward_head_from<0>(c, p, g, batch, x, a, dout, d, AdamHost{nullptr}, first, last, r,
                          n_riders, hp, head_from);
  }
  DQ_CHECK_LAUNCH("dq_cnn_backward_riders");
  return DQ_OK;
}

int dq_cnn_backward_peer(const dq_cnn_params* p, const dq_cnn_params* g, int32_t batch,
                         const float* x, const dq_cnn_acts* a, const float* dout,
                         dq_cnn_acts* d, float* ws, const dq_rider* riders, int32_t n_riders,
                         const dq_adam_args* opt, const dq_cnn_net* head, const dq_peer* peer,
                         int32_t defer_ag, void* stream) {
  DQ_CHECK_ARG(p && g && a && d && x && dout && ws && opt && peer && batch >= 1, "null argument");
  DQ_CHECK_ARG(p->in_channels == 4 && p->n_out >= 1, "the Nature CNN takes 84x84x4 NHWC input");
  DQ_CHECK_ARG(opt->kind == DQ_OPT_ADAM, "the peer exchange applies TF1 Adam");
  DQ_CHECK_ARG(0 <= n_riders && n_riders <= 5 && (riders || n_riders == 0),
               "at most one rider per grouped launch 1..5");
  const int rc = check_adam(p, g, opt);
  if (rc != DQ_OK) return rc;
  const dq_peer& P = *peer;
  DQ_CHECK_ARG(P.world >= 1 && P.world <= DQ_PEER_MAX && P.rank >= 0 && P.rank < P.world,
               "peer: 1 <= world <= DQ_PEER_MAX, 0 <= rank < world");
  DQ_CHECK_ARG(P.lo >= 0 && P.lo % 4 == 0 && P.n > P.lo && (P.n - P.lo) % (4 * P.world) == 0,
               "peer: lo % 4 == 0 and (n - lo) % (4 world) == 0");
  DQ_CHECK_ARG(P.n >= (int64_t)(p->fc2_b + p->n_out - opt->var),
               "peer: [lo, n) must reach the end of the flat parameter buffer");
  // exactly the fc bucket: a head of fc1 floats in the conv bucket would be read by the peers
  // in launch 6 after this rank may have rewritten it in the next step's launch 2 (the conv
  // gradients proper are rewritten only after the next step's launch-3 wait)
  DQ_CHECK_ARG(P.lo == (int64_t)(p->fc1_w - opt->var),
               "peer: the sharded range is exactly the fc bucket [fc1_w, n) (pad the flat buffer "
               "so that its length divides into 4 world-float slices)");
  DQ_CHECK_ARG(P.param[P.rank] == opt->var && P.grad[P.rank] == g->conv1_w - (p->conv1_w - opt->var),
               "peer: this rank's buffers must be opt->var and the gradient of its layout");
  for (int q = 0; q < P.world; ++q)
    DQ_CHECK_ARG(P.grad[q] && P.param[q] && P.flags[q], "peer: null rank buffer");
  DQ_CHECK_ARG(P.max_polls > 0, "peer: max_polls must be positive");
  DQ_CHECK_ARG(P.xcds >= 0 && P.xcds <= 8, "peer: 0 <= xcds <= 8");
  RiderDesc r[5];
  for (int i = 0; i < n_riders; ++i) {
    memcpy(&r[i], &riders[i], sizeof(RiderDesc));
    DQ_CHECK_ARG(r[i].kind >= kRiderNone && r[i].kind <= kRiderSetSample, "corrupt rider");
  }
  FwdOps hf{};
  if (head) {
    DQ_CHECK_ARG(head->p && head->x && head->a && head->ws, "null head network field");
    DQ_CHECK_ARG(head->p->in_channels == 4, "the Nature CNN takes 84x84x4 NHWC input");
    DQ_CHECK_ARG(head->ws != ws, "the head network needs its own workspace");
    hf = FwdOps{head->p, head->x, head->a, head->ws, batch};
  }
  Ctx c{(hipStream_t)stream, ws, false, 0};
  backward_peer(c, p, g, batch, x, a, dout, d, opt, r, n_riders, head ? &hf : nullptr, P,
                defer_ag != 0);
  DQ_CHECK_LAUNCH("dq_cnn_backward_peer");
  return DQ_OK;
}

static int check_peer(const dq_peer* peer, const float* var) {
  DQ_CHECK_ARG(peer && var, "null argument");
  const dq_peer& P = *peer;
  DQ_CHECK_ARG(P.world >= 1 && P.world <= DQ_PEER_MAX && P.rank >= 0 && P.rank < P.world,
               "peer: 1 <= world <= DQ_PEER_MAX, 0 <= rank < world");
  DQ_CHECK_ARG(P.lo >= 0 && P.lo % 4 == 0 && P.n > P.lo && (P.n - P.lo) % (4 * P.world) == 0,
               "peer: lo % 4 == 0 and (n - lo) % (4 world) == 0");
  DQ_CHECK_ARG(P.param[P.rank] == var, "peer: var must be this rank's parameter buffer");
  for (int q = 0; q < P.world; ++q)
    DQ_CHECK_ARG(P.grad[q] && P.param[q] && P.flags[q], "peer: null rank buffer");
  DQ_CHECK_ARG(P.max_polls > 0, "peer: max_polls must be positive");
  DQ_CHECK_ARG(P.xcds >= 0 && P.xcds <= 8, "peer: 0 <= xcds <= 8");
  return DQ_OK;
}

int dq_peer_all_gather(const dq_peer* peer, float* var, void* stream) {
  const int rc = check_peer(peer, var);
  if (rc != DQ_OK) return rc;
  const dq_peer& P = *peer;
  if (P.world > 1) {
    Ctx c{(hipStream_t)stream, nullptr, false, 0};
    group(c, AgParts{peer, var}.part(0), AgParts{peer, var}.part(1), AgParts{peer, var}.part(2));
  }
  DQ_CHECK_LAUNCH("dq_peer_all_gather");
  return DQ_OK;
}

#ifdef DQ_GROUP_PROF
// the grouped launches' stamp ring (tools/group_stamps.py): reset the counter; read it back
int dq_debug_group_reset(void) {
  static unsigned z[dq::cnn::kGrpPos];
  return hipMemcpyToSymbol(HIP_SYMBOL(dq::cnn::g_grp_seq), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
// the exchange launch's phase stamps: recs 16 x kPeerPhRing x 5 u64, seq 16 counters
int dq_debug_peer_phases(void* recs, unsigned* seq) {
  if (hipMemcpyFromSymbol(seq, HIP_SYMBOL(dq::cnn::g_peer_ph_seq), sizeof(dq::cnn::g_peer_ph_seq)) !=
      hipSuccess)
    return -1;
  return hipMemcpyFromSymbol(recs, HIP_SYMBOL(dq::cnn::g_peer_ph), sizeof(dq::cnn::g_peer_ph)) ==
                 hipSuccess ? 0 : -1;
}
// recs: kGrpPos x kGrpRing records; seq: kGrpPos counters; dims: {kGrpPos, kGrpRing}
int dq_debug_group_read(void* recs, unsigned* seq, unsigned* dims) {
  dims[0] = dq::cnn::kGrpPos;
  dims[1] = dq::cnn::kGrpRing;
  if (hipMemcpyFromSymbol(seq, HIP_SYMBOL(dq::cnn::g_grp_seq), sizeof(dq::cnn::g_grp_seq)) !=
      hipSuccess)
    return -1;
  return hipMemcpyFromSymbol(recs, HIP_SYMBOL(dq::cnn::g_grp_rec), sizeof(dq::cnn::g_grp_rec)) ==
                 hipSuccess ? 0 : -1;
}
#endif

int dq_peer_selftest(const dq_peer* peer, uint32_t tag, int32_t* mismatches_out, void* stream) {
  DQ_CHECK_ARG(peer && mismatches_out, "null argument");
  const dq_peer& P = *peer;
  const int rc = check_peer(peer, P.param[P.rank]);
  if (rc != DQ_OK) return rc;
  DQ_CHECK_ARG(P.n % 4 == 0 && P.n / 4 < (int64_t)1 << 27, "peer: n % 4 == 0, buffers < 2 GB");
  Ctx c{(hipStream_t)stream, nullptr, false, 0};
  group(c, SelfTestFillOp{P, tag, 2048});                      // 8 blocks per CU, every XCD
  group(c, PeerPubOp{P, kPeerTest});
  group(c, SelfTestCheckOp{P, tag, mismatches_out, kPeerMaxBlocks});
  DQ_CHECK_LAUNCH("dq_peer_selftest");
  return DQ_OK;
}

int dq_cnn_forward_fused_peer(const dq_cnn_params* p0, const float* x0, dq_cnn_acts* a0, float* ws0,
                              const dq_cnn_params* p1, const float* x1, dq_cnn_acts* a1, float* ws1,
                              int32_t batch, int32_t fc1_1, const dq_peer* peer, float* var,
                              void* stream) {
  DQ_CHECK_ARG(p0 && a0 && x0 && ws0 && p1 && a1 && ws1 && batch >= 1, "null argument");
  DQ_CHECK_ARG(p0->in_channels == 4 && p1->in_channels == 4 && p0->n_out >= 1 && p1->n_out >= 1,
               "the Nature CNN takes 84x84x4 NHWC input");
  DQ_CHECK_ARG(ws0 != ws1, "the two networks need separate workspaces");
  DQ_CHECK_ARG((fc1_1 & (4 | 8 | 32)) == 0 && (fc1_1 & 16),
               "the deferred gather rides in the head_from 6 schedule's conv launches (flag 16)");
  const int rc = check_peer(peer, var);
  if (rc != DQ_OK) return rc;
  Ctx c0{(hipStream_t)stream, ws0, false, 0}, c1{(hipStream_t)stream, ws1, false, 0};
  const AgParts ag{peer, var};
  forward_fused(c0, c1, FwdOps{p0, x0, a0, ws0, batch}, FwdOps{p1, x1, a1, ws1, batch},
                (fc1_1 & 1) != 0, (fc1_1 & 2) != 0, true, true, true, false,
                peer->world > 1 ? &ag : nullptr);
  DQ_CHECK_LAUNCH("dq_cnn_forward_fused_peer");
  return DQ_OK;
}

int dq_cnn_forward_torso(const dq_cnn_params* p, int32_t batch, const float* x, dq_cnn_acts* a,
                         float* ws, void* stream) {
  DQ_CHECK_ARG(p && a && x && ws && batch >= 1, "null argument");
  DQ_CHECK_ARG(p->in_channels == 4, "the Nature CNN takes 84x84x4 NHWC input");
  Ctx c{(hipStream_t)stream, ws, false, 0};
  const FwdOps f{p, x, a, ws, batch};
  group(c, f.conv1<false>());
  group(c, f.conv2<false>());
  group(c, f.conv3<false>());
  DQ_CHECK_LAUNCH("dq_cnn_forward_torso");
  return DQ_OK;
}

int dq_cnn_backward_torso(const dq_cnn_params* p, const dq_cnn_params* g, int32_t batch,
                          const float* x, const dq_cnn_acts* a, dq_cnn_acts* d, float* ws,
                          void* stream) {
  DQ_CHECK_ARG(p && g && a && d && x && ws && batch >= 1, "null argument");
  DQ_CHECK_ARG(p->in_channels == 4, "the Nature CNN takes 84x84x4 NHWC input");
  Ctx c{(hipStream_t)stream, ws, false, 0};
  backward_torso_grouped(c, p, g, batch, x, a, d);
  DQ_CHECK_LAUNCH("dq_cnn_backward_torso");
  return DQ_OK;
}

int dq_cnn_backward_torso_opt(const dq_cnn_params* p, const dq_cnn_params* g, int32_t batch,
                              const float* x, const dq_cnn_acts* a, dq_cnn_acts* d, float* ws,
                              const dq_adam_args* opt, float* head_begin, float* head_end,
                              void* stream) {
  DQ_CHECK_ARG(p && g && a && d && x && ws && opt && batch >= 1, "null argument");
  DQ_CHECK_ARG(p->in_channels == 4, "the Nature CNN takes 84x84x4 NHWC input");
  const int rc = check_adam(p, g, opt);
  if (rc) return rc;
  DQ_CHECK_ARG(head_begin && head_end && head_begin >= p->conv3_b + 64 && head_end > head_begin &&
                   ((head_begin - opt->var) & 3) == 0 && ((p->conv3_w - opt->var) & 3) == 0,
               "head range: 16-byte aligned, after conv3 in opt->var");
  Ctx c{(hipStream_t)stream, ws, false, 0};
  if (opt->kind == DQ_OPT_RMSPROP)
    backward_torso_grouped<2>(c, p, g, batch, x, a, d, AdamHost{opt}, head_begin, head_end);
  else
    backward_torso_grouped<1>(c, p, g, batch, x, a, d, AdamHost{opt}, head_begin, head_end);
  DQ_CHECK_LAUNCH("dq_cnn_backward_torso_opt");
  return DQ_OK;
}

int dq_cnn_backward_layer(const dq_cnn_params* p, const dq_cnn_params* g, int32_t batch,
                          const float* x, const dq_cnn_acts* a, const float* dout, dq_cnn_acts* d,
                          float* ws, int32_t layer, int32_t part, void* stream) {
  DQ_CHECK_ARG(p && g && a && d && x && dout && ws && batch >= 1, "null argument");
  DQ_CHECK_ARG(p->in_channels == 4 && p->n_out >= 1, "the Nature CNN takes 84x84x4 NHWC input");
  Ctx c{(hipStream_t)stream, ws, false, 0};
  DQ_CHECK_ARG((part == 0 || part == 1) && backward_layer(c, p, g, batch, x, a, dout, d, layer, part),
               "layer must be 0..4 (fc2, fc1, conv3, conv2, conv1), part 0 (input grad, not conv1) "
               "or 1 (weight grad)");
  DQ_CHECK_LAUNCH("dq_cnn_backward_layer");
  return DQ_OK;
}

size_t dq_cnn_workspace_floats(int32_t batch, int32_t n_out) {
  dq_cnn_params p = {};
  dq_cnn_acts a = {};
  p.in_channels = 4;
  p.n_out = n_out;
  size_t need = 0;
  Ctx f{nullptr, nullptr, true, 0};
  forward(f, &p, batch, nullptr, &a);
  need = f.need > need ? f.need : need;
  for (int layer = 0; layer < 5; ++layer)
    for (int part = 0; part < 2; ++part) {
      Ctx l{nullptr, nullptr, true, 0};
      backward_layer(l, &p, &p, batch, nullptr, &a, nullptr, &a, layer, part);
      need = l.need > need ? l.need : need;
    }
  Ctx g{nullptr, nullptr, true, 0};
  backward_grouped<0>(g, &p, &p, batch, nullptr, &a, nullptr, &a, AdamHost{nullptr});
  need = g.need > need ? g.need : need;
  Ctx t{nullptr, nullptr, true, 0};
  backward_torso_grouped(t, &p, &p, batch, nullptr, &a, &a);
  need = t.need > need ? t.need : need;
  Ctx f0{nullptr, nullptr, true, 0}, f1{nullptr, nullptr, true, 0};
  forward_fused(f0, f1, FwdOps{&p, nullptr, &a, nullptr, batch}, FwdOps{&p, nullptr, &a, nullptr, batch},
                true);
  return f0.need > need ? f0.need : need;
}

}  // extern "C"
