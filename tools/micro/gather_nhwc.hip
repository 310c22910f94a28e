// Micro-benchmark of NHWC frame-stack gather variants at the bench shape (1M x 84x84 u8
// frames, B = 32, n = 3, PER probabilities), each launch on a FRESH random index batch
// (400 launches per hipGraph, > the 256 MB Infinity Cache of frames) as bench.py times it.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I dopamine_amd/csrc \
//         -o tools/micro/gather_nhwc.bin tools/micro/gather_nhwc.hip
// Variants:
//   prod      the product kernel body (gather_nhwc4_body<1, true>), 7 x 2B blocks of 256
//   prod_sc1  the same with write-through (sc1) float4 stores
//   prod_nt   the same with nt float4 stores
//   fat<W,P>  dwordx4 frame loads (16 pixels of each of the 4 frames per lane), byte
//             transpose in registers, W waves per block, store policy P; pixel rows
//             exchanged through LDS so every store instruction writes 1 KiB contiguous
//   fatd<W,P> the same without the LDS exchange (each lane stores its own 256 B)
//   empty     launch floor with the prod grid
//   storeonly the prod grid writing zeros (no loads)
#include "replay_dev.h"

#include <cstdlib>
#include <vector>

namespace dq {
void set_error(const std::string&) {}
}  // namespace dq

using namespace dq;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1);} } while (0)

enum { PLAIN = 0, NT = 2, SC1 = 16 };

__device__ __forceinline__ __amdgpu_buffer_rsrc_t out_rsrc(void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(p, 0, 0x7fffffff, 0x00020000);
}

// product body with a store policy: copy of gather_nhwc4_body<1, true> (replay_dev.h)
template <int P>
__global__ __launch_bounds__(256) void k_prod(ReplayView v, GatherOut g) {
  const int bx = blockIdx.x, slot = blockIdx.y, tid = threadIdx.x;
  const int b = slot >> 1, which = slot & 1;
  const bool scal = bx == 0 && which == 0 && tid < 64;
  float* dst_base = (float*)(which ? g.next_state : g.state);
  const int64_t nd = v.obs_bytes >> 2;
  const int lane = tid & 63;
  const int64_t w0 = ((int64_t)bx * 256 + (tid & ~63));
  if (w0 >= nd) {
    if (scal) write_scalars_wave(v, g, b, pymod((int64_t)g.indices[b], v.C));
    return;
  }
  const int64_t idx = pymod((int64_t)g.indices[b], v.C);
  uint32_t w[4];
  auto load = [&](int64_t base) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t* fr = (const uint32_t*)(v.frames + pymod(base - 3 + k, v.C) * v.obs_bytes);
      const int64_t d = w0 + lane;
      w[k] = d < nd ? fr[d] : 0u;
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
    if (scal) write_scalars_wave(v, g, b, idx);
  }
  const int sh = 8 * (lane & 3);
  float4* dst = (float4*)(dst_base + (int64_t)b * 4 * v.obs_bytes) + 4 * w0;
  const __amdgpu_buffer_rsrc_t rs = out_rsrc(dst);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int src = 16 * j + (lane >> 2);
    float4 o;
    o.x = u8_unit((__shfl(w[0], src) >> sh) & 0xffu);
    o.y = u8_unit((__shfl(w[1], src) >> sh) & 0xffu);
    o.z = u8_unit((__shfl(w[2], src) >> sh) & 0xffu);
    o.w = u8_unit((__shfl(w[3], src) >> sh) & 0xffu);
    if (4 * w0 + 64 * j + lane < 4 * nd) {
      if constexpr (P == PLAIN)
        dst[64 * j + lane] = o;
      else
        __builtin_amdgcn_raw_buffer_store_b128(*(const uint32_t __attribute__((ext_vector_type(4)))*)&o,
                                               rs, (64 * j + lane) * 16, 0, P);
    }
  }
}

typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float4 px_to_f4(uint32_t p) {
  float4 o;
  o.x = u8_unit(p & 0xffu);
  o.y = u8_unit((p >> 8) & 0xffu);
  o.z = u8_unit((p >> 16) & 0xffu);
  o.w = u8_unit(p >> 24);
  return o;
}

// 4x4 byte transpose: a[k] = 4 pixels of frame k -> p[i] = pixel i's 4 channel bytes
__device__ __forceinline__ void byte_t4(uint32_t a0, uint32_t a1, uint32_t a2, uint32_t a3, uint32_t* p) {
  const uint32_t l01 = __builtin_amdgcn_perm(a1, a0, 0x05010400u);
  const uint32_t h01 = __builtin_amdgcn_perm(a1, a0, 0x07030602u);
  const uint32_t l23 = __builtin_amdgcn_perm(a3, a2, 0x05010400u);
  const uint32_t h23 = __builtin_amdgcn_perm(a3, a2, 0x07030602u);
  p[0] = __builtin_amdgcn_perm(l23, l01, 0x05040100u);
  p[1] = __builtin_amdgcn_perm(l23, l01, 0x07060302u);
  p[2] = __builtin_amdgcn_perm(h23, h01, 0x05040100u);
  p[3] = __builtin_amdgcn_perm(h23, h01, 0x07060302u);
}

// W waves per block; wave gw (of 7 per stack) covers pixels [1024 gw, 1024 gw + 1024)
template <int W, int P, bool LDSX>
__global__ __launch_bounds__(64 * W) void k_fat(ReplayView v, GatherOut g) {
  __shared__ uint32_t s_px[W][1024];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int gw = blockIdx.x * W + wv;
  const int slot = blockIdx.y, b = slot >> 1, which = slot & 1;
  const int64_t npx = v.obs_bytes;               // pixels per frame (u8)
  const bool scal = gw == 0 && which == 0;
  const int64_t p0 = (int64_t)gw * 1024;
  if (p0 >= npx) return;                         // wave-uniform
  const int64_t idx = pymod((int64_t)g.indices[b], v.C);
  const int64_t lp = p0 + 16 * lane;             // this lane's 16 pixels
  const bool live = lp < npx;
  u32x4_t w[4];
  auto load = [&](int64_t base) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint8_t* fr = v.frames + pymod(base - 3 + k, v.C) * v.obs_bytes;
      w[k] = live ? *(const u32x4_t*)(fr + lp) : u32x4_t{0, 0, 0, 0};
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
    if (scal) write_scalars_wave(v, g, b, idx);
  }
  uint32_t px[16];
#pragma unroll
  for (int q = 0; q < 4; ++q) byte_t4(w[0][q], w[1][q], w[2][q], w[3][q], px + 4 * q);
  float* dst_base = (float*)(which ? g.next_state : g.state) + (int64_t)b * 4 * npx;
  float4* dst = (float4*)dst_base + p0;         // pixel p -> float4 p
  const __amdgpu_buffer_rsrc_t rs = out_rsrc(dst);
  if constexpr (LDSX) {
    uint32_t* s = s_px[wv];
#pragma unroll
    for (int q = 0; q < 4; ++q)
      *(u32x4_t*)(s + 16 * lane + 4 * q) = u32x4_t{px[4 * q], px[4 * q + 1], px[4 * q + 2], px[4 * q + 3]};
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int p = 64 * j + lane;
      const float4 o = px_to_f4(s[p]);
      if (p0 + p < npx) {
        if constexpr (P == PLAIN)
          dst[p] = o;
        else
          __builtin_amdgcn_raw_buffer_store_b128(*(const u32x4_t*)&o, rs, p * 16, 0, P);
      }
    }
  } else {
    if (live) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const float4 o = px_to_f4(px[i]);
        const int p = 16 * lane + i;
        if constexpr (P == PLAIN)
          dst[p] = o;
        else
          __builtin_amdgcn_raw_buffer_store_b128(*(const u32x4_t*)&o, rs, p * 16, 0, P);
      }
    }
  }
}

__global__ __launch_bounds__(256) void k_empty(ReplayView v, GatherOut g) {
  if (threadIdx.x == 1023) ((float*)g.state)[0] = 0.f;
}

__global__ __launch_bounds__(256) void k_storeonly(ReplayView v, GatherOut g) {
  const int bx = blockIdx.x, slot = blockIdx.y, tid = threadIdx.x;
  const int b = slot >> 1, which = slot & 1;
  const int64_t nd = v.obs_bytes >> 2;
  const int64_t w0 = ((int64_t)bx * 256 + (tid & ~63));
  if (w0 >= nd) return;
  float4* dst = (float4*)((float*)(which ? g.next_state : g.state) + (int64_t)b * 4 * v.obs_bytes) + 4 * w0;
  const int lane = tid & 63;
#pragma unroll
  for (int j = 0; j < 4; ++j)
    if (4 * w0 + 64 * j + lane < 4 * nd) dst[64 * j + lane] = float4{0.f, 0.f, 0.f, 0.f};
}

// decomposition: (a) index load -> dependent zero stores (no frame loads)
__global__ __launch_bounds__(256) void k_idxstore(ReplayView v, GatherOut g) {
  const int bx = blockIdx.x, slot = blockIdx.y, tid = threadIdx.x;
  const int b = slot >> 1, which = slot & 1;
  const int64_t nd = v.obs_bytes >> 2;
  const int64_t w0 = ((int64_t)bx * 256 + (tid & ~63));
  if (w0 >= nd) return;
  const int64_t idx = pymod((int64_t)g.indices[b], v.C);
  const float z = (float)(idx >> 40);   // 0, but depends on the load
  float4* dst = (float4*)((float*)(which ? g.next_state : g.state) + (int64_t)b * 4 * v.obs_bytes) + 4 * w0;
  const int lane = tid & 63;
#pragma unroll
  for (int j = 0; j < 4; ++j)
    if (4 * w0 + 64 * j + lane < 4 * nd) dst[64 * j + lane] = float4{z, z, z, z};
}

// (b) random frames with NO index dependency (frame address from a hash of the launch
// number and the block), converted and stored as prod does
__global__ __launch_bounds__(256) void k_nodep(ReplayView v, GatherOut g, int launch, int64_t region) {
  const int bx = blockIdx.x, slot = blockIdx.y, tid = threadIdx.x;
  const int b = slot >> 1, which = slot & 1;
  const int64_t nd = v.obs_bytes >> 2;
  const int lane = tid & 63;
  const int64_t w0 = ((int64_t)bx * 256 + (tid & ~63));
  if (w0 >= nd) return;
  uint64_t hsh = ((uint64_t)launch * 0x9E3779B97F4A7C15ull) ^ ((uint64_t)(slot + 1) * 0xBF58476D1CE4E5B9ull);
  hsh ^= hsh >> 31; hsh *= 0x94D049BB133111EBull; hsh ^= hsh >> 29;
  const int64_t base = 10 + (int64_t)(hsh % (uint64_t)(region - 20));
  uint32_t w[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint32_t* fr = (const uint32_t*)(v.frames + (base - 3 + k) * v.obs_bytes);
    const int64_t d = w0 + lane;
    w[k] = d < nd ? fr[d] : 0u;
  }
  const int sh = 8 * (lane & 3);
  float4* dst = (float4*)((float*)(which ? g.next_state : g.state) + (int64_t)b * 4 * v.obs_bytes) + 4 * w0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int src = 16 * j + (lane >> 2);
    float4 o;
    o.x = u8_unit((__shfl(w[0], src) >> sh) & 0xffu);
    o.y = u8_unit((__shfl(w[1], src) >> sh) & 0xffu);
    o.z = u8_unit((__shfl(w[2], src) >> sh) & 0xffu);
    o.w = u8_unit((__shfl(w[3], src) >> sh) & 0xffu);
    if (4 * w0 + 64 * j + lane < 4 * nd) dst[64 * j + lane] = o;
  }
}

// (c) prod without the scalars wave and with next_state = state's stack (one dependent level)
__global__ __launch_bounds__(256) void k_oneLevel(ReplayView v, GatherOut g) {
  const int bx = blockIdx.x, slot = blockIdx.y, tid = threadIdx.x;
  const int b = slot >> 1, which = slot & 1;
  const int64_t nd = v.obs_bytes >> 2;
  const int lane = tid & 63;
  const int64_t w0 = ((int64_t)bx * 256 + (tid & ~63));
  if (w0 >= nd) return;
  const int64_t idx = pymod((int64_t)g.indices[b] + which * v.n, v.C);
  uint32_t w[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint32_t* fr = (const uint32_t*)(v.frames + pymod(idx - 3 + k, v.C) * v.obs_bytes);
    const int64_t d = w0 + lane;
    w[k] = d < nd ? fr[d] : 0u;
  }
  const int sh = 8 * (lane & 3);
  float4* dst = (float4*)((float*)(which ? g.next_state : g.state) + (int64_t)b * 4 * v.obs_bytes) + 4 * w0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int src = 16 * j + (lane >> 2);
    float4 o;
    o.x = u8_unit((__shfl(w[0], src) >> sh) & 0xffu);
    o.y = u8_unit((__shfl(w[1], src) >> sh) & 0xffu);
    o.z = u8_unit((__shfl(w[2], src) >> sh) & 0xffu);
    o.w = u8_unit((__shfl(w[3], src) >> sh) & 0xffu);
    if (4 * w0 + 64 * j + lane < 4 * nd) dst[64 * j + lane] = o;
  }
}

// prod with the per-sample scalars on their own block column (bx == nbx - 1)
template <int P>
__global__ __launch_bounds__(256) void k_sep(ReplayView v, GatherOut g) {
  const int bx = blockIdx.x, slot = blockIdx.y, tid = threadIdx.x;
  const int b = slot >> 1, which = slot & 1;
  if (bx == (int)gridDim.x - 1) {
    if (which == 0 && tid < 64) write_scalars_wave(v, g, b, pymod((int64_t)g.indices[b], v.C));
    return;
  }
  float* dst_base = (float*)(which ? g.next_state : g.state);
  const int64_t nd = v.obs_bytes >> 2;
  const int lane = tid & 63;
  const int64_t w0 = ((int64_t)bx * 256 + (tid & ~63));
  if (w0 >= nd) return;
  const int64_t idx = pymod((int64_t)g.indices[b], v.C);
  uint32_t w[4];
  auto load = [&](int64_t base) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t* fr = (const uint32_t*)(v.frames + pymod(base - 3 + k, v.C) * v.obs_bytes);
      const int64_t d = w0 + lane;
      w[k] = d < nd ? fr[d] : 0u;
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
  }
  const int sh = 8 * (lane & 3);
  float4* dst = (float4*)(dst_base + (int64_t)b * 4 * v.obs_bytes) + 4 * w0;
  const __amdgpu_buffer_rsrc_t rs = out_rsrc(dst);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int src = 16 * j + (lane >> 2);
    float4 o;
    o.x = u8_unit((__shfl(w[0], src) >> sh) & 0xffu);
    o.y = u8_unit((__shfl(w[1], src) >> sh) & 0xffu);
    o.z = u8_unit((__shfl(w[2], src) >> sh) & 0xffu);
    o.w = u8_unit((__shfl(w[3], src) >> sh) & 0xffu);
    if (4 * w0 + 64 * j + lane < 4 * nd) {
      if constexpr (P == PLAIN)
        dst[64 * j + lane] = o;
      else
        __builtin_amdgcn_raw_buffer_store_b128(*(const uint32_t __attribute__((ext_vector_type(4)))*)&o,
                                               rs, (64 * j + lane) * 16, 0, P);
    }
  }
}

int main(int argc, char** argv) {
  const int64_t C = 1000000, OBS = 84 * 84;
  const int B = argc > 1 ? atoi(argv[1]) : 32;
  const int iters = 400;
  uint8_t *frames, *term;
  int32_t *act, *idx_all;
  float *rew, *disc, *st, *nst, *o_rew, *o_nrew, *o_prob;
  int32_t *o_act, *o_nact, *o_idx;
  uint8_t* o_term;
  double* tree;
  CK(hipMalloc(&frames, C * OBS));
  CK(hipMalloc(&term, C));
  CK(hipMalloc(&act, C * 4));
  CK(hipMalloc(&rew, C * 4));
  CK(hipMalloc(&disc, 64));
  CK(hipMalloc(&tree, (int64_t)8 << 21));
  CK(hipMalloc(&idx_all, (int64_t)iters * B * 4));
  CK(hipMalloc(&st, (int64_t)B * 4 * OBS * 4));
  CK(hipMalloc(&nst, (int64_t)B * 4 * OBS * 4));
  CK(hipMalloc(&o_rew, B * 4)); CK(hipMalloc(&o_nrew, B * 4)); CK(hipMalloc(&o_prob, B * 4));
  CK(hipMalloc(&o_act, B * 4)); CK(hipMalloc(&o_nact, B * 4)); CK(hipMalloc(&o_idx, B * 4));
  CK(hipMalloc(&o_term, B));
  {
    std::vector<uint8_t> hf(OBS * 1024);
    srand(1);
    for (auto& x : hf) x = rand() & 255;
    for (int64_t i = 0; i < C; i += 1024) {
      const int64_t n = std::min<int64_t>(1024, C - i);
      CK(hipMemcpy(frames + i * OBS, hf.data(), n * OBS, hipMemcpyHostToDevice));
    }
    std::vector<uint8_t> ht(C);
    for (auto& x : ht) x = (rand() % 500) == 0;
    CK(hipMemcpy(term, ht.data(), C, hipMemcpyHostToDevice));
    CK(hipMemset(act, 0, C * 4)); CK(hipMemset(rew, 0, C * 4)); CK(hipMemset(tree, 0, (int64_t)8 << 21));
    float hd[3] = {1.f, 0.99f, 0.9801f};
    CK(hipMemcpy(disc, hd, 12, hipMemcpyHostToDevice));
    std::vector<int32_t> hi((int64_t)iters * B);
    for (auto& x : hi) x = 10 + (int32_t)(((int64_t)rand() * 7919 + rand()) % (C - 20));
    CK(hipMemcpy(idx_all, hi.data(), hi.size() * 4, hipMemcpyHostToDevice));
  }
  ReplayView v{C, OBS, 4, 3, 20, 1000, frames, act, rew, term, tree, nullptr, nullptr, disc};
  auto gout = [&](int i) {
    return GatherOut{idx_all + (int64_t)i * B, st, nst, o_act, o_rew, o_nact, o_nrew, o_term, o_idx, o_prob};
  };
  hipStream_t s;
  CK(hipStreamCreate(&s));
  const double bytes = (double)B * (2 * 4 * OBS + 2 * 4 * OBS * 4);
  auto run = [&](const char* name, auto launch) {
    for (int i = 0; i < 5; ++i) launch(i);
    CK(hipStreamSynchronize(s));
    hipGraph_t gr;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    for (int i = 0; i < iters; ++i) launch(i);
    CK(hipStreamEndCapture(s, &gr));
    CK(hipGraphInstantiate(&ge, gr, nullptr, nullptr, 0));
    CK(hipGraphLaunch(ge, s));
    CK(hipStreamSynchronize(s));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    float tot = 0.f, best = 1e30f;
    for (int rep = 0; rep < 5; ++rep) {
      CK(hipEventRecord(e0, s));
      CK(hipGraphLaunch(ge, s));
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      tot += ms;
      best = std::min(best, ms);
    }
    const double us = tot / 5 * 1e3 / iters, ub = best * 1e3 / iters;
    printf("%-30s mean %6.3f  best %6.3f us/launch   frac %.3f\n", name, us, ub, bytes / us * 1e-6 / 8.0);
    fflush(stdout);
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(gr));
  };
  std::vector<float> ref;
  auto snap = [&](std::vector<float>& out) {
    CK(hipStreamSynchronize(s));
    out.resize((size_t)B * 4 * OBS * 2);
    CK(hipMemcpy(out.data(), st, (size_t)B * 4 * OBS * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(out.data() + (size_t)B * 4 * OBS, nst, (size_t)B * 4 * OBS * 4, hipMemcpyDeviceToHost));
  };
  auto check = [&](const char* name) {
    std::vector<float> got;
    snap(got);
    if (ref.empty()) { ref = got; return; }
    size_t bad = 0;
    for (size_t i = 0; i < ref.size(); ++i) bad += ref[i] != got[i];
    if (bad) printf("  !! %s differs from prod in %zu floats\n", name, bad);
  };
  const dim3 pg(7, 2 * B);
  auto fatgrid = [&](int W) { return dim3((7 + W - 1) / W, 2 * B); };
#define ONE(name, K, grid, blk)                                                          \
  do {                                                                                   \
    hipLaunchKernelGGL(K, grid, blk, 0, s, v, gout(3));                                  \
    check(name);                                                                         \
    run(name, [&](int i) { hipLaunchKernelGGL(K, grid, blk, 0, s, v, gout(i)); });      \
  } while (0)
  ONE("prod (plain)", k_prod<PLAIN>, pg, dim3(256));
  ONE("prod sc1", k_prod<SC1>, pg, dim3(256));
  ONE("prod nt", k_prod<NT>, pg, dim3(256));
  ONE("sep scalars plain", k_sep<PLAIN>, dim3(8, 2 * B), dim3(256));
  ONE("sep scalars nt", k_sep<NT>, dim3(8, 2 * B), dim3(256));
  {
    GatherOut g0 = gout(3); g0.probs = nullptr;
    auto gnp = [&](int i) { GatherOut q = gout(i); q.probs = nullptr; return q; };
    run("sep scalars nt, no probs", [&](int i) { hipLaunchKernelGGL(k_sep<NT>, dim3(8, 2 * B), dim3(256), 0, s, v, gnp(i)); });
    run("prod nt, no probs", [&](int i) { hipLaunchKernelGGL(k_prod<NT>, pg, dim3(256), 0, s, v, gnp(i)); });
  }
  ONE("fat W1 ldsx plain", (k_fat<1, PLAIN, true>), fatgrid(1), dim3(64));
  ONE("fat W1 ldsx sc1", (k_fat<1, SC1, true>), fatgrid(1), dim3(64));
  ONE("fat W1 ldsx nt", (k_fat<1, NT, true>), fatgrid(1), dim3(64));
  ONE("fat W7 ldsx plain", (k_fat<7, PLAIN, true>), fatgrid(7), dim3(448));
  ONE("fat W7 ldsx sc1", (k_fat<7, SC1, true>), fatgrid(7), dim3(448));
  ONE("fat W4 ldsx sc1", (k_fat<4, SC1, true>), fatgrid(4), dim3(256));
  ONE("fat W1 direct plain", (k_fat<1, PLAIN, false>), fatgrid(1), dim3(64));
  ONE("fat W1 direct sc1", (k_fat<1, SC1, false>), fatgrid(1), dim3(64));
  run("idx -> zero stores", [&](int i) { hipLaunchKernelGGL(k_idxstore, pg, dim3(256), 0, s, v, gout(i)); });
  for (int64_t region : {(int64_t)C, (int64_t)300000, (int64_t)150000, (int64_t)36000, (int64_t)4500}) {
    char nm[64];
    snprintf(nm, sizeof nm, "no idx dep, region %.2f GB", region * OBS / 1e9);
    run(nm, [&](int i) { hipLaunchKernelGGL(k_nodep, pg, dim3(256), 0, s, v, gout(i), i, region); });
  }
  // scattered 4 KB pages: frame f -> f * 293 (mod C): same page count as region 4500 x 293
  // ...
  run("one level (no scal/term)", [&](int i) { hipLaunchKernelGGL(k_oneLevel, pg, dim3(256), 0, s, v, gout(i)); });
  run("empty (prod grid)", [&](int i) { hipLaunchKernelGGL(k_empty, pg, dim3(256), 0, s, v, gout(i)); });
  run("empty (64 x 64-thr)", [&](int i) { hipLaunchKernelGGL(k_empty, dim3(7, 2 * B), dim3(64), 0, s, v, gout(i)); });
  run("store only (prod grid)", [&](int i) { hipLaunchKernelGGL(k_storeonly, pg, dim3(256), 0, s, v, gout(i)); });
  return 0;
}
