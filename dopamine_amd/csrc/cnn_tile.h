// The fp32 matrix-core tile engine shared by the Nature-CNN (nature_cnn.hip) and the
// IQN quantile heads (iqn.hip): loaders producing 16-byte operand groups, epilogues,
// the templated tile kernel igemm_block in two forms -- exact f32
// (v_mfma_f32_32x32x2_f32) and split-bf16 "x6" (fp32 to rounding on
// v_mfma_f32_32x32x16_bf16, X6Img below) -- the ordered split-K sum and the host-side
// launch context.  See nature_cnn.hip's header for the design.
#pragma once
#include <type_traits>

#include "common.h"
#include "replay_dev.h"

namespace dq {
namespace cnn {

typedef float f32x16 __attribute__((ext_vector_type(16)));

// ----------------------------------------------------------------- geometry
template <int H_, int W_, int CI_, int KH_, int KW_, int S_, int PT_, int PL_, int OH_, int OW_, int CO_>
struct Conv {
  static constexpr int H = H_, W = W_, CI = CI_, KH = KH_, KW = KW_, S = S_, PT = PT_, PL = PL_;
  static constexpr int OH = OH_, OW = OW_, CO = CO_;
  static constexpr int K = KH * KW * CI;     // im2col depth
  static_assert(CI % 4 == 0 && CO % 4 == 0, "16-byte operand groups need CI, CO % 4 == 0");
};
// TF SAME: conv1 84 -> 21 (pad 2/2), conv2 21 -> 11 (pad 1/2), conv3 11 -> 11 (pad 1/1)
using Conv1 = Conv<84, 84, 4, 8, 8, 4, 2, 2, 21, 21, 32>;
using Conv2 = Conv<21, 21, 32, 4, 4, 2, 1, 1, 11, 11, 64>;
using Conv3 = Conv<11, 11, 64, 3, 3, 1, 1, 1, 11, 11, 64>;
constexpr int kFlat = 11 * 11 * 64;   // 7744
constexpr int kHidden = 512;

__device__ __forceinline__ float4 zero4() { return make_float4(0.0f, 0.0f, 0.0f, 0.0f); }
__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }

// ------------------------------------------------------------------ loaders
// get(r, k, rlim, klim): the 16-byte group of 4 consecutive operand elements
// along the contiguous dimension (k when kFast, else r) at (r, k), zero outside
// [0, rlim) x [0, klim) and in conv padding.  Branch-free by construction: the
// address is clamped to a valid one, the load always issues and a select zeroes
// it, so the loads of a whole K slice stay in flight together (a divergent
// fallback branch would make the compiler drain vmcnt at every join).
// Vector loaders need the ragged dimension to be a multiple of 4 (a group is
// wholly in or out); the scalar ones (ld = n_out) pay 4 loads per group.

__device__ __forceinline__ float4 sel4(bool ok, float4 v) { return ok ? v : zero4(); }

// Raw buffer loads: an offset at or past num_records reads as zero in hardware,
// so an out-of-range group costs one offset select instead of a clamped 64-bit
// address and four data selects.  Valid byte offsets are < 2 GB here.
constexpr int kOOB = 0x7ffffff0;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const float* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), 0, kOOB, 0x00020000);
}
__device__ __forceinline__ float4 bload4(const float* base, int off, bool ok) {   // off in floats
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rsrc(base), ok ? off * 4 : kOOB, 0, 0);
  return make_float4(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z),
                     __uint_as_float(v.w));
}
__device__ __forceinline__ float bload1(const float* base, int off, bool ok) {
  return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rsrc(base), ok ? off * 4 : kOOB, 0, 0));
}

// forward im2col of an NHWC input: rows = output pixels, k = (kh, kw, ci).
// CI % 4 == 0, so a 16-byte group never straddles a (kh, kw) tap.
template <class G>
struct Im2col {
  static constexpr bool kFast = true;
  static constexpr bool kConvFwd = true;   // the forward convolutions (cnn_x6)
  const float* x;
  __device__ __forceinline__ int offset(int m, int k) const {   // -1 in the padding
    const int b = m / (G::OH * G::OW), p = m - b * (G::OH * G::OW);
    const int oh = p / G::OW, ow = p - oh * G::OW;
    const int kk = k / G::CI, ci = k - kk * G::CI;
    const int kh = kk / G::KW, kw = kk - kh * G::KW;
    const int ih = oh * G::S - G::PT + kh, iw = ow * G::S - G::PL + kw;
    if (ih < 0 || ih >= G::H || iw < 0 || iw >= G::W) return -1;
    return ((b * G::H + ih) * G::W + iw) * G::CI + ci;
  }
  __device__ __forceinline__ float4 get(int m, int k, int mlim, int klim) const {
    const int o = offset(m, k);
    return bload4(x, o, m < mlim && k < klim && o >= 0);
  }
};

// im2col as the B operand of a weight gradient: rows k = pixels, cols n = (kh,kw,ci);
// column n == G::K is the bias "ones" column (K % 4 == 0: its group is (1, 0, 0, 0)).
template <class G>
struct Im2colT {
  static constexpr bool kFast = false;
  const float* x;
  __device__ __forceinline__ float4 get(int n, int k, int, int klim) const {
    const float4 v = Im2col<G>{x}.get(k, n, klim, G::K);
    return (n == G::K && k < klim) ? make_float4(1.0f, 0.0f, 0.0f, 0.0f) : v;
  }
};

// stride-1 conv input gradient (transposed conv): rows m = input pixels, k = (kh, kw, co)
template <class G>
struct Col2im {
  static_assert(G::S == 1, "strided input gradients go through the sub-pixel classes (SubPix)");
  static constexpr bool kFast = true;
  const float* dy;
  __device__ __forceinline__ float4 get(int m, int k, int mlim, int klim) const {
    const int b = m / (G::H * G::W), p = m - b * (G::H * G::W);
    const int ih = p / G::W, iw = p - ih * G::W;
    const int kk = k / G::CO, co = k - kk * G::CO;
    const int kh = kk / G::KW, kw = kk - kh * G::KW;
    const int oh = ih + G::PT - kh, ow = iw + G::PL - kw;
    const bool ok = m < mlim && k < klim && oh >= 0 && ow >= 0 && oh < G::OH && ow < G::OW;
    return bload4(dy, ((b * G::OH + oh) * G::OW + ow) * G::CO + co, ok);
  }
};

// conv weights as B of the transposed conv: B(n = ci, k = (kh, kw, co)) = W[co][kh][kw][ci]
template <class G>
struct WeightT {
  static constexpr bool kFast = false;
  const float* w;
  __device__ __forceinline__ float4 get(int n, int k, int nlim, int klim) const {
    const int kk = k / G::CO, co = k - kk * G::CO;
    return bload4(w, (co * (G::KH * G::KW) + kk) * G::CI + n, n < nlim && k < klim);
  }
};

// Stride-S conv input gradient by sub-pixel class: the input pixels with
// (ih % S, iw % S) == (PY, PX) receive exactly the taps kh = (PY + PT) mod S + S*th,
// kw = (PX + PL) mod S + S*tw, so the transposed conv is S*S dense GEMMs (rows = that
// class's pixels, k = (th, tw, co)) with no stride holes and no dcol round trip.
template <class G, int PY, int PX>
struct SubPix {
  static_assert(G::KH % G::S == 0 && G::KW % G::S == 0, "taps split evenly over the classes");
  static constexpr int NY = (G::H - PY + G::S - 1) / G::S, NX = (G::W - PX + G::S - 1) / G::S;
  static constexpr int TW = G::KW / G::S, K = (G::KH / G::S) * TW * G::CO;
  static constexpr int KH0 = (PY + G::PT) % G::S, KW0 = (PX + G::PL) % G::S;
  __device__ static __forceinline__ int pixel(int m) {      // NHWC pixel index of class row m
    const int b = m / (NY * NX), q = m - b * (NY * NX);
    const int i = q / NX, j = q - i * NX;
    return (b * G::H + PY + G::S * i) * G::W + PX + G::S * j;
  }
  __device__ static __forceinline__ void tap(int k, int& kh, int& kw, int& co) {
    const int t = k / G::CO;
    co = k - t * G::CO;
    const int th = t / TW;
    kh = KH0 + G::S * th;
    kw = KW0 + G::S * (t - th * TW);
  }
};
// A: dy of the taps landing on class row m, k = (th, tw, co) with co contiguous
template <class G, int PY, int PX>
struct SubPixDy {
  using SP = SubPix<G, PY, PX>;
  static constexpr bool kFast = true;
  const float* dy;
  __device__ __forceinline__ float4 get(int m, int k, int mlim, int klim) const {
    const int b = m / (SP::NY * SP::NX), q = m - b * (SP::NY * SP::NX);
    const int i = q / SP::NX, j = q - i * SP::NX;
    int kh, kw, co;
    SP::tap(k, kh, kw, co);
    const int th = PY + G::S * i + G::PT - kh, tw = PX + G::S * j + G::PL - kw;   // even
    const int oh = th / G::S, ow = tw / G::S;
    const bool ok = m < mlim && k < klim && th >= 0 && tw >= 0 && oh < G::OH && ow < G::OW;
    return bload4(dy, ((b * G::OH + oh) * G::OW + ow) * G::CO + co, ok);
  }
};
// B: W[co][kh][kw][ci] as B(n = ci, k = (th, tw, co)), ci contiguous
template <class G, int PY, int PX>
struct SubPixW {
  using SP = SubPix<G, PY, PX>;
  static constexpr bool kFast = false;
  const float* w;
  __device__ __forceinline__ float4 get(int n, int k, int nlim, int klim) const {
    int kh, kw, co;
    SP::tap(k, kh, kw, co);
    return bload4(w, ((co * G::KH + kh) * G::KW + kw) * G::CI + n, n < nlim && k < klim);
  }
};

// plain row-major [rows][ld], k contiguous (x of an FC layer, weights [N][K]); ld % 4 == 0
struct RowK {
  static constexpr bool kFast = true;
  const float* p;
  int ld;
  __device__ __forceinline__ float4 get(int r, int k, int rlim, int klim) const {
    return bload4(p, r * ld + k, r < rlim && k < klim);
  }
};
// [k][rows] with rows contiguous: dy^T of FC dW (A), W of FC dX as B(n = in, k = out); ld % 4 == 0
struct ColK {
  static constexpr bool kFast = false;
  const float* p;
  int ld;
  __device__ __forceinline__ float4 get(int r, int k, int rlim, int klim) const {
    return bload4(p, k * ld + r, r < rlim && k < klim);
  }
};
// RowK over rows taken b-major: GEMM row m = b * nq + q reads row q * B + b of p (the IQN
// quantile rows are q-major), so a tile of 128 rows holds whole samples (nq | 128)
struct RowKQ {
  static constexpr bool kFast = true;
  const float* p;
  int ld, B, nq;
  __device__ __forceinline__ float4 get(int m, int k, int rlim, int klim) const {
    const int b = m / nq, r = (m - b * nq) * B + b;
    return bload4(p, r * ld + k, m < rlim && k < klim);
  }
};
// FC dW's B operand: B(n, k = batch) = x[k][n], with the bias ones-column at n == ld
struct ColKOnes {
  static constexpr bool kFast = false;
  const float* p;
  int ld;
  __device__ __forceinline__ float4 get(int n, int k, int, int klim) const {
    const float4 v = bload4(p, k * ld + n, n < ld && k < klim);
    return (n == ld && k < klim) ? make_float4(1.0f, 0.0f, 0.0f, 0.0f) : v;
  }
};
// conv dW's A operand: A(m = co, k = pixel) = dy[pixel][co]
template <int CO>
struct DyT {
  static constexpr bool kFast = false;
  const float* dy;
  __device__ __forceinline__ float4 get(int m, int k, int mlim, int klim) const {
    return bload4(dy, k * CO + m, m < mlim && k < klim);
  }
};
// scalar forms of RowK / ColK for a leading dimension that is not a multiple of 4
// (the n_out-wide output gradient): 4 clamped loads + selects per group
struct RowKScalar {
  static constexpr bool kFast = true;
  const float* p;
  int ld;
  __device__ __forceinline__ float4 get(int r, int k, int rlim, int klim) const {
    float v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      v[j] = bload1(p, r * ld + k + j, r < rlim && k + j < klim);
    }
    return make_float4(v[0], v[1], v[2], v[3]);
  }
};
struct ColKScalar {
  static constexpr bool kFast = false;
  const float* p;
  int ld;
  __device__ __forceinline__ float4 get(int r, int k, int rlim, int klim) const {
    float v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      v[j] = bload1(p, k * ld + r + j, r + j < rlim && k < klim);
    }
    return make_float4(v[0], v[1], v[2], v[3]);
  }
};

// ---------------------------------------------------------------- epilogues
// Epilogues with kPrefetch read one input per output element (bias, ReLU mask)
// that does not depend on the product: the tile kernel issues pf() before its K
// loop and hands the value to apply(), so that load's latency hides under the
// operand fetches instead of following the reduction (same arithmetic).
struct EpiBiasAct {          // out[m][n] = act(acc + bias[n])
  float* out;
  const float* bias;
  int ld;
  bool relu;
  static constexpr bool kPrefetch = true;
  __device__ __forceinline__ float pf(int, int n) const { return bias[n]; }
  __device__ __forceinline__ void apply(int m, int n, float v, float b) const {
    v = __fadd_rn(v, b);
    out[(int64_t)m * ld + n] = relu ? fmaxf(v, 0.0f) : v;
  }
  __device__ __forceinline__ void operator()(int m, int n, float v, int) const {
    apply(m, n, v, pf(m, n));
  }
};
struct EpiMask {             // out[m][n] = acc * (act[m][n] > 0)   (ReLU backward)
  float* out;
  const float* act;
  int ld;
  static constexpr bool kPrefetch = true;
  __device__ __forceinline__ float pf(int m, int n) const { return act[(int64_t)m * ld + n]; }
  __device__ __forceinline__ void apply(int m, int n, float v, float a) const {
    out[(int64_t)m * ld + n] = a > 0.0f ? v : 0.0f;
  }
  __device__ __forceinline__ void operator()(int m, int n, float v, int) const {
    apply(m, n, v, pf(m, n));
  }
};
template <class SP, int C>
struct EpiMaskPix {          // EpiMask on a sub-pixel class: row m -> its NHWC pixel
  float* out;
  const float* act;
  static constexpr bool kPrefetch = true;
  __device__ __forceinline__ float pf(int m, int n) const {
    return act[(int64_t)SP::pixel(m) * C + n];
  }
  __device__ __forceinline__ void apply(int m, int n, float v, float a) const {
    out[(int64_t)SP::pixel(m) * C + n] = a > 0.0f ? v : 0.0f;
  }
  __device__ __forceinline__ void operator()(int m, int n, float v, int) const {
    apply(m, n, v, pf(m, n));
  }
};
struct EpiStore {            // out[m][n] = acc
  float* out;
  int ld;
  __device__ __forceinline__ void operator()(int m, int n, float v, int) const {
    out[(int64_t)m * ld + n] = v;
  }
};
struct EpiPartial {          // split-K slab z
  float* ws;
  int M, N;
  __device__ __forceinline__ void operator()(int m, int n, float v, int z) const {
    ws[((int64_t)z * M + m) * N + n] = v;
  }
};
struct EpiGrad {             // n < nw: dW[m][n]; n == nw: db[m]
  float* gw;
  float* gb;
  int nw;
  __device__ __forceinline__ void operator()(int m, int n, float v, int) const {
    if (n < nw) gw[(int64_t)m * nw + n] = v;
    else gb[m] = v;
  }
};

// gradient + TF1 Adam in one pass: the element's gradient is final here, so the
// optimizer update (same arithmetic as dq_adam_tf1) is applied where it is made.
struct AdamDev {
  float* state;
  int slot;
  float lr, b1, b2, eps;
  int store_grad;          // fused epilogues: also write the gradient (dq_adam_args.no_grad_store)
};
struct EpiGradAdam {
  float* gw;
  float* gb;
  int nw;
  float *w, *mw, *vw;      // parameter / moment slices at the same offsets as gw
  float *b, *mb, *vb;      // ... and as gb
  AdamDev o;
  int bump;                // this epilogue advances the beta powers (one per step)
  // two-phase form: pre() issues the element's loads, commit() updates and stores,
  // so a thread's loads for ALL its elements are in flight before the first store
  // (the stores may alias later loads as far as the compiler knows)
  static constexpr bool kPre = true;
  struct Pre {
    float w, m, v;
  };
  __device__ __forceinline__ Pre pre(int m, int n) const {
    if (n < nw) {
      const int64_t i = (int64_t)m * nw + n;
      return Pre{w[i], mw[i], vw[i]};
    }
    return Pre{b[m], mb[m], vb[m]};
  }
  __device__ __forceinline__ void commit(int m, int n, float g, Pre q) const {
    const float alpha = adam_alpha_of(o.state, o.slot, o.lr);
    const float omb1 = __fsub_rn(1.0f, o.b1), omb2 = __fsub_rn(1.0f, o.b2);
    adam1(q.w, g, q.m, q.v, alpha, omb1, omb2, o.eps);
    if (n < nw) {
      const int64_t i = (int64_t)m * nw + n;
      if (o.store_grad) gw[i] = g;
      w[i] = q.w;
      mw[i] = q.m;
      vw[i] = q.v;
    } else {
      if (o.store_grad) gb[m] = g;
      b[m] = q.w;
      mb[m] = q.m;
      vb[m] = q.v;
    }
    if (bump && m == 0 && n == 0) adam_bump(o.state, o.slot, o.b1, o.b2);
  }
  __device__ __forceinline__ void operator()(int m, int n, float g, int) const {
    commit(m, n, g, pre(m, n));
  }
};

// gradient + TF1 Adam in the vector (kVec) epilogue form, 4 consecutive columns per call
// (16-B loads and stores of the gradient, parameter and moments): fc1's weight gradient
// (512 x 7744 + the bias column) updates fc1 where each tile's gradient is made, instead of
// storing it for Adam riders in the following launches to read back.  Same arithmetic as
// EpiGradAdam / k_adam (adam1), element by element.
struct EpiGradAdamVec {
  float* gw;
  float* gb;
  int nw;                  // nw % 4 == 0 (the column groups never straddle the bias column)
  float *w, *mw, *vw;
  float *b, *mb, *vb;
  AdamDev o;
  static constexpr bool kVec = true;
  __device__ __forceinline__ void scalar(int m, int n, float g) const {
    const float alpha = adam_alpha_of(o.state, o.slot, o.lr);
    const float omb1 = __fsub_rn(1.0f, o.b1), omb2 = __fsub_rn(1.0f, o.b2);
    if (n < nw) {
      const int64_t i = (int64_t)m * nw + n;
      float pw = w[i], pm = mw[i], pv = vw[i];
      adam1(pw, g, pm, pv, alpha, omb1, omb2, o.eps);
      if (o.store_grad) gw[i] = g;
      w[i] = pw;
      mw[i] = pm;
      vw[i] = pv;
    } else if (n == nw) {
      float pw = b[m], pm = mb[m], pv = vb[m];
      adam1(pw, g, pm, pv, alpha, omb1, omb2, o.eps);
      if (o.store_grad) gb[m] = g;
      b[m] = pw;
      mb[m] = pm;
      vb[m] = pv;
    }
  }
  __device__ __forceinline__ void operator()(int m, int n, float g, int) const { scalar(m, n, g); }
  // the same epilogue over rows [r0, ...) of the weight (a row range of the GEMM)
  EpiGradAdamVec rows_from(int r0) const {
    EpiGradAdamVec e = *this;
    const int64_t o = (int64_t)r0 * nw;
    e.gw += o; e.w += o; e.mw += o; e.vw += o;
    e.gb += r0; e.b += r0; e.mb += r0; e.vb += r0;
    return e;
  }
  // two-phase vector form (kVecPre): the next row group's parameter / moment loads are
  // issued before this group's stores (the compiler cannot tell the rows apart and would
  // otherwise serialise each group's loads behind the previous group's stores)
  static constexpr bool kVecPre = true;
  struct VPre {
    float4 w, m, v;
  };
  // the streamed state's loads / stores with the default cache policy (non-temporal stores,
  // or loads and stores, measured no faster in round 4)
  __device__ static __forceinline__ float4 ldst(const float* p) { return ld4(p); }
  __device__ static __forceinline__ void stst(float* p, float4 v) {
    *reinterpret_cast<float4*>(p) = v;
  }
  __device__ __forceinline__ VPre vpre(int m, int n) const {
    if (n >= nw) return VPre{zero4(), zero4(), zero4()};
    const int64_t i = (int64_t)m * nw + n;
    return VPre{ldst(w + i), ldst(mw + i), ldst(vw + i)};
  }
  __device__ __forceinline__ void vcommit(int m, int n, float4 g, const VPre& p) const {
    if (n >= nw) {                 // the bias column (and the tile's padding past it)
      scalar(m, n, g.x);
      return;
    }
    const int64_t i = (int64_t)m * nw + n;
    float4 pw = p.w, pm = p.m, pv = p.v;
    const float alpha = adam_alpha_of(o.state, o.slot, o.lr);
    const float omb1 = __fsub_rn(1.0f, o.b1), omb2 = __fsub_rn(1.0f, o.b2);
    adam1(pw.x, g.x, pm.x, pv.x, alpha, omb1, omb2, o.eps);
    adam1(pw.y, g.y, pm.y, pv.y, alpha, omb1, omb2, o.eps);
    adam1(pw.z, g.z, pm.z, pv.z, alpha, omb1, omb2, o.eps);
    adam1(pw.w, g.w, pm.w, pv.w, alpha, omb1, omb2, o.eps);
    if (o.store_grad) *reinterpret_cast<float4*>(gw + i) = g;
    stst(w + i, pw);
    stst(mw + i, pm);
    stst(vw + i, pv);
  }
  __device__ __forceinline__ void vec4(int m, int n, float4 g) const {
    if (n >= nw) {                 // the bias column (and the tile's padding past it)
      scalar(m, n, g.x);
      return;
    }
    const int64_t i = (int64_t)m * nw + n;
    float4 pw = ld4(w + i), pm = ld4(mw + i), pv = ld4(vw + i);
    const float alpha = adam_alpha_of(o.state, o.slot, o.lr);
    const float omb1 = __fsub_rn(1.0f, o.b1), omb2 = __fsub_rn(1.0f, o.b2);
    adam1(pw.x, g.x, pm.x, pv.x, alpha, omb1, omb2, o.eps);
    adam1(pw.y, g.y, pm.y, pv.y, alpha, omb1, omb2, o.eps);
    adam1(pw.z, g.z, pm.z, pv.z, alpha, omb1, omb2, o.eps);
    adam1(pw.w, g.w, pm.w, pv.w, alpha, omb1, omb2, o.eps);
    if (o.store_grad) *reinterpret_cast<float4*>(gw + i) = g;
    *reinterpret_cast<float4*>(w + i) = pw;
    *reinterpret_cast<float4*>(mw + i) = pm;
    *reinterpret_cast<float4*>(vw + i) = pv;
  }
};

// gradient + TF1 RMSProp in one pass (dq_rmsprop_tf1's arithmetic, rms1): m = ms,
// v = mom, g2 = mg (centered only)
struct RmsDev {
  float lr, omr, mu, eps;
  int centered;
  int store_grad;          // as AdamDev::store_grad
};
__host__ inline RmsDev rms_dev(const dq_adam_args* a) {
  // 1 - rho in host float32 arithmetic: the value k_rmsprop's __fsub_rn forms
  return RmsDev{a->lr, 1.0f - a->decay, a->momentum, a->epsilon, a->centered != 0,
                a->no_grad_store == 0};
}
struct EpiGradRms {
  float* gw;
  float* gb;
  int nw;
  float *w, *mw, *vw, *gw2;   // parameter / ms / mom / mg slices at the same offsets as gw
  float *b, *mb, *vb, *gb2;   // ... and as gb
  RmsDev o;
  static constexpr bool kPre = true;
  struct Pre {
    float w, m, v, g2;
  };
  __device__ __forceinline__ Pre pre(int m, int n) const {
    if (n < nw) {
      const int64_t i = (int64_t)m * nw + n;
      return Pre{w[i], mw[i], vw[i], o.centered ? gw2[i] : 0.0f};
    }
    return Pre{b[m], mb[m], vb[m], o.centered ? gb2[m] : 0.0f};
  }
  __device__ __forceinline__ void commit(int m, int n, float g, Pre q) const {
    rms1(q.w, g, q.m, q.g2, q.v, o.lr, o.omr, o.mu, o.eps, o.centered != 0);
    if (n < nw) {
      const int64_t i = (int64_t)m * nw + n;
      if (o.store_grad) gw[i] = g;
      w[i] = q.w;
      mw[i] = q.m;
      vw[i] = q.v;
      if (o.centered) gw2[i] = q.g2;
    } else {
      if (o.store_grad) gb[m] = g;
      b[m] = q.w;
      mb[m] = q.m;
      vb[m] = q.v;
      if (o.centered) gb2[m] = q.g2;
    }
  }
  __device__ __forceinline__ void operator()(int m, int n, float g, int) const {
    commit(m, n, g, pre(m, n));
  }
};

// EpiGradRms as a vector (kVec) epilogue with the two-phase loads of EpiGradAdamVec:
// fc1's centered RMSProp (ms, mom, mg) applied in its weight-gradient GEMM
struct EpiGradRmsVec {
  EpiGradRms s;            // the scalar form: pointers, constants, the bias column
  static constexpr bool kVec = true;
  static constexpr bool kVecPre = true;
  EpiGradRmsVec rows_from(int r0) const {
    EpiGradRmsVec e = *this;
    const int64_t o = (int64_t)r0 * s.nw;
    e.s.gw += o; e.s.w += o; e.s.mw += o; e.s.vw += o; e.s.gw2 += o;
    e.s.gb += r0; e.s.b += r0; e.s.mb += r0; e.s.vb += r0; e.s.gb2 += r0;
    return e;
  }
  struct VPre {
    float4 w, m, v, g2;
  };
  __device__ __forceinline__ void operator()(int m, int n, float g, int) const { s(m, n, g, 0); }
  __device__ __forceinline__ VPre vpre(int m, int n) const {
    if (n >= s.nw) return VPre{zero4(), zero4(), zero4(), zero4()};
    const int64_t i = (int64_t)m * s.nw + n;
    return VPre{ld4(s.w + i), ld4(s.mw + i), ld4(s.vw + i), s.o.centered ? ld4(s.gw2 + i) : zero4()};
  }
  __device__ __forceinline__ void vcommit(int m, int n, float4 g, const VPre& p) const {
    if (n >= s.nw) {               // the bias column (and the tile's padding past it)
      s(m, n, g.x, 0);
      return;
    }
    const int64_t i = (int64_t)m * s.nw + n;
    float4 pw = p.w, pm = p.m, pv = p.v, p2 = p.g2;
    const bool ce = s.o.centered != 0;
    rms1(pw.x, g.x, pm.x, p2.x, pv.x, s.o.lr, s.o.omr, s.o.mu, s.o.eps, ce);
    rms1(pw.y, g.y, pm.y, p2.y, pv.y, s.o.lr, s.o.omr, s.o.mu, s.o.eps, ce);
    rms1(pw.z, g.z, pm.z, p2.z, pv.z, s.o.lr, s.o.omr, s.o.mu, s.o.eps, ce);
    rms1(pw.w, g.w, pm.w, p2.w, pv.w, s.o.lr, s.o.omr, s.o.mu, s.o.eps, ce);
    if (s.o.store_grad) *reinterpret_cast<float4*>(s.gw + i) = g;
    *reinterpret_cast<float4*>(s.w + i) = pw;
    *reinterpret_cast<float4*>(s.mw + i) = pm;
    *reinterpret_cast<float4*>(s.vw + i) = pv;
    if (ce) *reinterpret_cast<float4*>(s.gw2 + i) = p2;
  }
  __device__ __forceinline__ void vec4(int m, int n, float4 g) const { vcommit(m, n, g, vpre(m, n)); }
};

template <class EP, class = void>
struct HasPf {
  static constexpr bool value = false;
};
template <class EP>
struct HasPf<EP, decltype((void)EP::kPrefetch)> {
  static constexpr bool value = EP::kPrefetch;
};

template <class EP, class = void>
struct HasPre {
  static constexpr bool value = false;
};
template <class EP>
struct HasPre<EP, decltype((void)EP::kPre)> {
  static constexpr bool value = EP::kPre;
};
template <class EP, class = void>
struct PreOf {
  using type = int;
};
template <class EP>
struct PreOf<EP, decltype((void)sizeof(typename EP::Pre))> {
  using type = typename EP::Pre;
};

// EP::kVec: the epilogue takes 4 consecutive columns at a time (E.vec4(m, n, float4)),
// so its loads and stores are 16 B per lane: igemm_block passes each wave's 32 x 32
// accumulator tile through LDS (WK == 1 only; N % 4 == 0).
template <class EP, class = void>
struct HasVecPre {
  static constexpr bool value = false;
};
template <class EP>
struct HasVecPre<EP, decltype((void)EP::kVecPre)> {
  static constexpr bool value = EP::kVecPre;
};

template <class EP, class = void>
struct HasVec {
  static constexpr bool value = false;
};
template <class EP>
struct HasVec<EP, decltype((void)EP::kVec)> {
  static constexpr bool value = EP::kVec;
};

// EP::kBlock: the epilogue takes the block's whole (32 WM) x (32 WN) accumulator tile from
// LDS (E.block(tile, ld, m0, n0, M, N), all threads), e.g. to reduce across rows
template <class EP, class = void>
struct HasBlock {
  static constexpr bool value = false;
};
template <class EP>
struct HasBlock<EP, decltype((void)EP::kBlock)> {
  static constexpr bool value = EP::kBlock;
};
template <class EP, class = void>
struct BlockExtra {
  static constexpr int value = 0;
};
template <class EP>
struct BlockExtra<EP, decltype((void)EP::kBlockExtra)> {
  static constexpr int value = EP::kBlockExtra;
};

// host-side: EpiGrad, or EpiGradAdam / EpiGradRms with the optimizer slots of the same
// parameter.  kOpt: 0 none, 1 TF1 Adam, 2 TF1 RMSProp (a compile-time choice, so each
// optimizer's kernels are exactly its own code)
struct AdamHost {
  const dq_adam_args* a;
};
template <int kOpt>
struct GradEpi;
template <>
struct GradEpi<0> {
  static EpiGrad make(float* gw, float* gb, int nw, float*, float*, const AdamHost&, int) {
    return EpiGrad{gw, gb, nw};
  }
};
template <>
struct GradEpi<1> {
  static EpiGradAdam make(float* gw, float* gb, int nw, float* w, float* b, const AdamHost& h,
                          int bump) {
    const dq_adam_args* a = h.a;
    const ptrdiff_t ow = w - a->var, ob = b - a->var;
    return EpiGradAdam{gw, gb, nw, w, a->m + ow, a->v + ow, b, a->m + ob, a->v + ob,
                       AdamDev{a->state, a->slot, a->lr, a->beta1, a->beta2, a->epsilon,
                               a->no_grad_store == 0},
                       bump};
  }
};
template <>
struct GradEpi<2> {
  static EpiGradRms make(float* gw, float* gb, int nw, float* w, float* b, const AdamHost& h, int) {
    const dq_adam_args* a = h.a;
    const ptrdiff_t ow = w - a->var, ob = b - a->var;
    float* mg = a->centered ? a->mg : a->m;    // never null: the (unused) loads stay valid
    return EpiGradRms{gw, gb, nw, w, a->m + ow, a->v + ow, mg + ow,
                      b, a->m + ob, a->v + ob, mg + ob, rms_dev(a)};
  }
};

// ------------------------------------------------------------- tile kernel
// 16-byte group g of an R x BKT operand slice -> (row rr, k offset kk).
// kFast: 8 consecutive lanes cover 128 contiguous bytes of one row, then rows,
// then the next 32-wide k band.  Otherwise lanes walk the rows 4 at a time.
template <bool kFast, int R, int BKT>
__device__ __forceinline__ void group_coord(int g, int& rr, int& kk) {
  if (kFast) {
    kk = 4 * ((g & 7) + 8 * (g / (8 * R)));
    rr = (g >> 3) % R;
  } else {
    kk = g / (R / 4);
    rr = 4 * (g % (R / 4));
  }
}

// Block = WM x WN x WK waves.  The WM x WN output tiles are 32x32 (one MFMA
// accumulator each); each K slice of BKT = 32*WK is split WK ways, one 32-wide
// k band per wave, so a block with many waves covers a small GEMM's whole K in
// one or two slices and keeps several waves per SIMD (address math of one wave
// overlaps the MFMAs of another).  The next slice's operands are fetched into
// registers while the MFMAs of the current one run.  The WK partial
// accumulators are then summed through LDS by all threads, each output element
// in wave order (deterministic), and handed to the epilogue with consecutive
// threads on consecutive columns.

template <int WM, int WN, int WK>
struct Tile {
  static constexpr int T = 64 * WM * WN * WK;
  static constexpr int BM = 32 * WM, BN = 32 * WN, BKT = 32 * WK;
  // one wave per k band (WM = WN = 1): each wave stages only its own band, 16 k at a time
  static constexpr bool kPrivate = WM == 1 && WN == 1 && WK > 1;
  template <class AL, class BL>
  static constexpr int lds() {      // operand slices, or the WK > 1 reduction scratch
    const int sa = BM + (AL::kFast ? 1 : 4), sb = BN + (BL::kFast ? 1 : 4);
    const int pa = AL::kFast ? 32 * 16 : 16 * 36, pb = BL::kFast ? 32 * 16 : 16 * 36;
    const int tile = kPrivate ? WK * (pa + pb) : BKT * sa + BKT * sb;
    const int red = WK > 1 ? WK * WM * WN * 1024 : 0;
    return tile > red ? tile : red;
  }
};

// ---------------------------------------------- split-bf16 ("x6") matrix-core form
// fp32 operands as exact sums of three bf16 pieces, a = hi + mid + lo (round to
// nearest at each stage: a - hi and (a - hi) - mid are exact in fp32, and the last
// remainder has <= 8 significant bits, so lo holds it exactly), multiplied by
// v_mfma_f32_32x32x16_bf16 (bf16 x bf16 products are exact in fp32, fp32
// accumulate) over the six piece pairs whose weight reaches 2^-16:
//   hi.hi + hi.mid + mid.hi + hi.lo + mid.mid + lo.hi.
// The three dropped pairs are below 2^-25 |a b| (each piece is at most 2^-9 of the
// one above), under fp32's own rounding of the product, so the result is an fp32
// GEMM to rounding -- not a bf16 one -- at 6 x 32 cycles per 32x32x16 step instead
// of 8 x 64 for v_mfma_f32_32x32x2_f32 (2.7x the f32 matrix rate).
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));
typedef float f32x2v __attribute__((ext_vector_type(2)));
// two fp32 -> their hi / mid / lo bf16 pieces, each pair packed (element 0 low)
__device__ __forceinline__ void split_x3(float a, float b, unsigned& h, unsigned& m, unsigned& l) {
  const unsigned hu = __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2v){a, b}, bf16x2v));
  const float ra = a - __uint_as_float(hu << 16), rb = b - __uint_as_float(hu & 0xffff0000u);
  const unsigned mu = __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2v){ra, rb}, bf16x2v));
  const float sa = ra - __uint_as_float(mu << 16), sb = rb - __uint_as_float(mu & 0xffff0000u);
  h = hu;
  m = mu;
  l = __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2v){sa, sb}, bf16x2v));
}

// eight fp32 operands of one lane (k = 8h + j of its row) -> the three bf16x8 pieces
__device__ __forceinline__ void split_x3_8(const float* v, bf16x8& h, bf16x8& m, bf16x8& l) {
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  u32x4 hu, mu, lu;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    unsigned a, b, c;
    split_x3(v[2 * i], v[2 * i + 1], a, b, c);
    hu[i] = a;
    mu[i] = b;
    lu[i] = c;
  }
  h = __builtin_bit_cast(bf16x8, hu);
  m = __builtin_bit_cast(bf16x8, mu);
  l = __builtin_bit_cast(bf16x8, lu);
}
// acc += A B over one 16-k step from the pieces, smallest pairs first.
// -DDQ_X6_PAIRS=1 (throughput experiments, NOT fp32): hi.hi only -- a plain bf16 GEMM.
#ifndef DQ_X6_PAIRS
#define DQ_X6_PAIRS 6
#endif
__device__ __forceinline__ f32x16 mfma_x6(const bf16x8& ah, const bf16x8& am, const bf16x8& al,
                                          const bf16x8& bh, const bf16x8& bm, const bf16x8& bl,
                                          f32x16 acc) {
  if (DQ_X6_PAIRS == 1) return __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bm, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bh, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bm, acc, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh, acc, 0, 0, 0);
}
// one bf16x8 piece of eight fp32 values (round to nearest), the remainders left in v
__device__ __forceinline__ bf16x8 peel8(float* v) {
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  u32x4 p;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const unsigned u = __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2v){v[2 * i], v[2 * i + 1]}, bf16x2v));
    v[2 * i] -= __uint_as_float(u << 16);
    v[2 * i + 1] -= __uint_as_float(u & 0xffff0000u);
    p[i] = u;
  }
  return __builtin_bit_cast(bf16x8, p);
}
// mfma_x6 with B split as it goes (fewer live registers: B's pieces one at a time), the
// same six pairs, the large one last: al.bh, am.bh, am.bm, ah.bm, ah.bl, ah.bh
__device__ __forceinline__ f32x16 mfma_x6_lazy(const bf16x8& ah, const bf16x8& am, const bf16x8& al,
                                               float* bv, f32x16 acc) {
  const bf16x8 bh = peel8(bv);
  // the bf16 throughput build: one product, as mfma_x6 (am / al are then dead code)
  if (DQ_X6_PAIRS == 1) return __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bh, acc, 0, 0, 0);
  {
    const bf16x8 bm = peel8(bv);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bm, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bm, acc, 0, 0, 0);
  }
  const bf16x8 bl = peel8(bv);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl, acc, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh, acc, 0, 0, 0);
}

// The x6 staging image of one operand slice: 3 planes (hi, mid, lo) of [rows][BKT]
// bf16, 16-byte k chunks XOR-swizzled by row so a 32x32x16 operand read (row r, 8
// consecutive k) is one ds_read_b128 and 8 consecutive rows hit distinct banks.
template <int ROWS, int BKT>
struct X6Img {
  static constexpr int RB = 2 * BKT;               // bytes per row per plane
  static constexpr int PLANE = ROWS * RB;          // bytes per plane
  static constexpr int BYTES = 3 * PLANE;
  __device__ static __forceinline__ int off(int row, int k) {   // byte offset of element (row, k)
    return row * RB + 16 * ((k >> 3) ^ ((row >> 2) & 3)) + 2 * (k & 7);
  }
  // the 16-byte group of a loader (4 consecutive k of row rr when kFast, else 4
  // consecutive rows at k) split and written into the three planes
  __device__ static __forceinline__ void put(char* img, bool kfast, int rr, int kk, float4 v) {
    unsigned h0, m0, l0, h1, m1, l1;
    split_x3(v.x, v.y, h0, m0, l0);
    split_x3(v.z, v.w, h1, m1, l1);
    if (kfast) {                                   // kk % 4 == 0: one 8-byte write per plane
      char* p = img + off(rr, kk);
      *reinterpret_cast<uint2*>(p) = make_uint2(h0, h1);
      *reinterpret_cast<uint2*>(p + PLANE) = make_uint2(m0, m1);
      *reinterpret_cast<uint2*>(p + 2 * PLANE) = make_uint2(l0, l1);
    } else {                                       // rr % 4 == 0: one swizzle for the 4 rows
      const unsigned hs[4] = {h0 & 0xffffu, h0 >> 16, h1 & 0xffffu, h1 >> 16};
      const unsigned ms[4] = {m0 & 0xffffu, m0 >> 16, m1 & 0xffffu, m1 >> 16};
      const unsigned ls[4] = {l0 & 0xffffu, l0 >> 16, l1 & 0xffffu, l1 >> 16};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        char* p = img + off(rr + i, kk);
        *reinterpret_cast<unsigned short*>(p) = (unsigned short)hs[i];
        *reinterpret_cast<unsigned short*>(p + PLANE) = (unsigned short)ms[i];
        *reinterpret_cast<unsigned short*>(p + 2 * PLANE) = (unsigned short)ls[i];
      }
    }
  }
  // the 32x32x16 operand of rows base.. base+31, k = kb .. kb+15: lane (r, h) gets row
  // base + r, k = kb + 8h + j in element j -- one ds_read_b128 per plane
  __device__ static __forceinline__ void get(const char* img, int base, int kb, int lane, bf16x8& h,
                                             bf16x8& m, bf16x8& l) {
    const char* p = img + off(base + (lane & 31), kb + 8 * (lane >> 5));
    h = *reinterpret_cast<const bf16x8*>(p);
    m = *reinterpret_cast<const bf16x8*>(p + PLANE);
    l = *reinterpret_cast<const bf16x8*>(p + 2 * PLANE);
  }
};

// The x6 image of a row-contiguous operand (loader groups = 4 consecutive rows at one
// k): planes [k][rows] bf16, so each group lands as one 8-byte write per plane, and
// the k-contiguous MFMA operand comes back through gfx950's transposing LDS read
// (ds_read_b64_tr_b16: per 16-lane group, lane 4q + p addresses image row q, columns
// 4p .. 4p+3 of a 4 x 16 block and lane i receives column i, row q in element q).
// Row stride 2*ROWS (+ 64 B when that is a multiple of 128) puts the four image rows
// of a read in distinct 64-B bank windows: the 32 lanes of a half read 256 distinct
// bytes, conflict-free.
typedef short s16x4v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4v lds_s16x4v;
template <int ROWS, int BKT>
struct X6ImgT {
  static constexpr int RS = 2 * ROWS + ((2 * ROWS) % 128 == 0 ? 64 : 0);   // bytes per k row
  static constexpr int PLANE = BKT * RS;
  static constexpr int BYTES = 3 * PLANE;
  __device__ static __forceinline__ int off(int row, int k) { return k * RS + 2 * row; }
  __device__ static __forceinline__ void put(char* img, bool, int rr, int kk, float4 v) {
    unsigned h0, m0, l0, h1, m1, l1;
    split_x3(v.x, v.y, h0, m0, l0);
    split_x3(v.z, v.w, h1, m1, l1);
    char* p = img + off(rr, kk);                   // rr % 4 == 0: 8-byte aligned
    *reinterpret_cast<uint2*>(p) = make_uint2(h0, h1);
    *reinterpret_cast<uint2*>(p + PLANE) = make_uint2(m0, m1);
    *reinterpret_cast<uint2*>(p + 2 * PLANE) = make_uint2(l0, l1);
  }
  __device__ static __forceinline__ bf16x8 tr8(const char* p) {   // k = q and 4 + q
    typedef short s16x8 __attribute__((ext_vector_type(8)));
    const s16x4v a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4v*)(p));
    const s16x4v b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4v*)(p + 4 * RS));
    const s16x8 v = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
    return __builtin_bit_cast(bf16x8, v);
  }
  // same operand map as X6Img::get (EXEC must be all ones: the read gathers across lanes)
  __device__ static __forceinline__ void get(const char* img, int base, int kb, int lane, bf16x8& h,
                                             bf16x8& m, bf16x8& l) {
    const int g = lane >> 4, q = (lane >> 2) & 3, p4 = lane & 3;
    const char* p = img + off(base + 16 * (g & 1) + 4 * p4, kb + 8 * (g >> 1) + q);
    h = tr8(p);
    m = tr8(p + PLANE);
    l = tr8(p + 2 * PLANE);
  }
};
template <bool kFast, int ROWS, int BKT>
using X6Of = typename std::conditional<kFast, X6Img<ROWS, BKT>, X6ImgT<ROWS, BKT>>::type;

// kLate: issue each half-band fetch after the previous half's MFMAs (<= 64 VGPRs,
// for launches with several rounds of blocks, two 16-wave blocks per CU); else
// while they run (one more fetch in flight, for single-round launches).
// kX6: the split-bf16 matrix-core form (block-shared staging only).
template <int WM, int WN, int WK, class AL, class BL, class EP, bool kLate = true, bool kX6 = false>
__device__ __forceinline__ void igemm_block(const AL& A, const BL& B, const EP& E, int M, int N,
                                            int K, int kchunk, int bx, int by, int bz,
                                            float* smem, int tid_base = 0) {
  using TL = Tile<WM, WN, WK>;
  constexpr int T = TL::T, BM = TL::BM, BN = TL::BN, BKT = TL::BKT;
  constexpr int SA = BM + (AL::kFast ? 1 : 4), SB = BN + (BL::kFast ? 1 : 4);
  constexpr int NA = BM * BKT / 4 / T, NB = BN * BKT / 4 / T;
  static_assert(NA >= 1 && NB >= 1 && NA * 4 * T == BM * BKT && NB * 4 * T == BN * BKT, "tile/threads");
  constexpr int OUT = WM * WN * 1024;     // output elements per block
  float* As = smem;
  float* Bs = smem + BKT * SA;

  // tid_base: the tile's first thread (several tiles sharing a block, PairOp)
  const int tid = (int)threadIdx.x - tid_base, lane = tid & 63, wave = tid >> 6;
  const int wm = wave % WM, wn = (wave / WM) % WN, wk = wave / (WM * WN);
  const int m0 = bx * BM, n0 = by * BN;
  const int kbeg = bz * kchunk;
  const int kend = min(K, kbeg + kchunk);
  float4 ra[NA], rb[NB];

  auto load = [&](int k0) {
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      int rr, kk;
      group_coord<AL::kFast, BM, BKT>(i * T + tid, rr, kk);
      ra[i] = A.get(m0 + rr, k0 + kk, M, kend);
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      int rr, kk;
      group_coord<BL::kFast, BN, BKT>(i * T + tid, rr, kk);
      rb[i] = B.get(n0 + rr, k0 + kk, N, kend);
    }
  };
  auto put = [](float* S, int stride, bool kfast, int rr, int kk, float4 v) {
    if (kfast) {
      S[(kk + 0) * stride + rr] = v.x;
      S[(kk + 1) * stride + rr] = v.y;
      S[(kk + 2) * stride + rr] = v.z;
      S[(kk + 3) * stride + rr] = v.w;
    } else {
      *reinterpret_cast<float4*>(S + kk * stride + rr) = v;
    }
  };
  auto stash = [&]() {
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      int rr, kk;
      group_coord<AL::kFast, BM, BKT>(i * T + tid, rr, kk);
      put(As, SA, AL::kFast, rr, kk, ra[i]);
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      int rr, kk;
      group_coord<BL::kFast, BN, BKT>(i * T + tid, rr, kk);
      put(Bs, SB, BL::kFast, rr, kk, rb[i]);
    }
  };

  // the epilogue's product-independent input (bias / ReLU mask) of this thread's
  // reduction elements, loaded now (clamped, never branching); see kPrefetch
  constexpr int NE = (OUT + T - 1) / T;
  constexpr bool kPf = WK > 1 && HasPf<EP>::value && NE <= 2;
  float pfv[NE];
  if constexpr (kPf) {
#pragma unroll
    for (int i = 0; i < NE; ++i) {
      const int e = min(tid + i * T, OUT - 1);
      const int tile = e >> 10, r = (e >> 6) & 15, l = e & 63;
      const int m = m0 + (tile % WM) * 32 + (r & 3) + 8 * (r >> 2) + 4 * (l >> 5);
      const int n = n0 + (tile / WM) * 32 + (l & 31);
      pfv[i] = E.pf(min(m, M - 1), min(n, N - 1));
    }
  }
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.0f;
  if constexpr (kX6 && !TL::kPrivate) {
    // Block-shared staging as below, the slice split into bf16 pieces as it is
    // written to LDS (each element once, whichever waves read it), then per 16-k
    // step six 32x32x16 bf16 MFMAs, smallest pairs first.
    using IA = X6Of<AL::kFast, BM, BKT>;
    using IB = X6Of<BL::kFast, BN, BKT>;
    char* ia = reinterpret_cast<char*>(smem);
    char* ib = ia + IA::BYTES;
    load(kbeg);
    for (int k0 = kbeg; k0 < kend; k0 += BKT) {
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        int rr, kk;
        group_coord<AL::kFast, BM, BKT>(i * T + tid, rr, kk);
        IA::put(ia, AL::kFast, rr, kk, ra[i]);
      }
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        int rr, kk;
        group_coord<BL::kFast, BN, BKT>(i * T + tid, rr, kk);
        IB::put(ib, BL::kFast, rr, kk, rb[i]);
      }
      __syncthreads();
      if (k0 + BKT < kend) load(k0 + BKT);
      if (k0 + wk * 32 < kend) {              // wave-uniform: bands past the end are all zero
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          bf16x8 ah, am, al, bh, bm, bl;
          IA::get(ia, wm * 32, wk * 32 + 16 * s, lane, ah, am, al);
          IB::get(ib, wn * 32, wk * 32 + 16 * s, lane, bh, bm, bl);
          acc = mfma_x6(ah, am, al, bh, bm, bl, acc);
        }
      }
      __syncthreads();
    }
  } else if constexpr (TL::kPrivate) {
    // Wave-private staging: wave wk fetches its own 32-wide k band (the same
    // coalesced 128-byte row segments as the shared layout) and transposes it
    // through its own LDS window, 16 k at a time -- no block barrier until the
    // reduction, and about half the LDS of a block-shared slice.
    // MFMA step s of a half takes k = s from lanes 0-31 and k = 8 + s from lanes
    // 32-63, so a lane's 8 operands of the half are contiguous in k: a k-contiguous
    // operand is kept [row][16 k] (float4 slots XOR-swizzled by row, conflict-free
    // 128-bit writes and reads), a row-contiguous one [k][row] (stride 36: its
    // 128-bit writes and the two half-waves' scalar reads hit disjoint banks).
    constexpr int WA = AL::kFast ? 32 * 16 : 16 * 36, WB = BL::kFast ? 32 * 16 : 16 * 36;
    float* Aw = smem + wave * (WA + WB);
    float* Bw = Aw + WA;
    auto st = [](float* W, bool kfast, int rr, int kl, float4 v) {   // kl in [0, 16)
      float* q = kfast ? W + rr * 16 + 4 * ((kl >> 2) ^ ((rr >> 2) & 3)) : W + kl * 36 + rr;
      *reinterpret_cast<float4*>(q) = v;
    };
    const int r = lane & 31, hh = lane >> 5;
    auto operands = [&](const float* W, bool kfast, float* o) {   // o[s] = element (r, 8 hh + s)
      if (kfast) {
        const float4 x0 = *reinterpret_cast<const float4*>(W + r * 16 + 4 * ((2 * hh) ^ ((r >> 2) & 3)));
        const float4 x1 =
            *reinterpret_cast<const float4*>(W + r * 16 + 4 * ((2 * hh + 1) ^ ((r >> 2) & 3)));
        o[0] = x0.x; o[1] = x0.y; o[2] = x0.z; o[3] = x0.w;
        o[4] = x1.x; o[5] = x1.y; o[6] = x1.z; o[7] = x1.w;
      } else {
#pragma unroll
        for (int s = 0; s < 8; ++s) o[s] = W[(8 * hh + s) * 36 + r];
      }
    };
    // Half-band fetch: 16 k per fetch (2 float4 per operand per lane), the second
    // half's loads issued behind the first half's MFMAs: 16 fewer live registers
    // (66-69 VGPRs instead of 88-91) than fetching the whole band at once, which
    // lets small blocks share the CU with a 16-wave one (+7% per step, measured).
    float4 qa[2], qb[2];
    auto hcoord = [&](bool kfast, int h, int j, int& rr, int& kk) {
      if (kfast) {
        rr = 16 * j + (lane >> 2);
        kk = 32 * wk + 16 * h + 4 * (lane & 3);
      } else {
        rr = 4 * (lane & 7);
        kk = 32 * wk + 16 * h + 8 * j + (lane >> 3);
      }
    };
    auto fetch_h = [&](int k0, int h) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        int rr, kk;
        hcoord(AL::kFast, h, j, rr, kk);
        qa[j] = A.get(m0 + rr, k0 + kk, M, kend);
        hcoord(BL::kFast, h, j, rr, kk);
        qb[j] = B.get(n0 + rr, k0 + kk, N, kend);
      }
    };
    auto stage_h = [&](int h) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        int rr, kk;
        hcoord(AL::kFast, h, j, rr, kk);
        st(Aw, AL::kFast, rr, kk - 32 * wk - 16 * h, qa[j]);
        hcoord(BL::kFast, h, j, rr, kk);
        st(Bw, BL::kFast, rr, kk - 32 * wk - 16 * h, qb[j]);
      }
    };
    fetch_h(kbeg, 0);
    for (int k0 = kbeg; k0 < kend; k0 += BKT) {
      const bool live = k0 + wk * 32 < kend;   // wave-uniform: bands past the end are all zero
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        stage_h(h);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        if constexpr (!kLate) {
          if (h == 0) fetch_h(k0, 1);
          else if (k0 + BKT < kend) fetch_h(k0 + BKT, 0);
        }
        if (live) {
          float av[8], bv[8];
          operands(Aw, AL::kFast, av);
          operands(Bw, BL::kFast, bv);
          if constexpr (kX6) {
            // each staged element is this lane's alone (one 32 x 32 tile per wave):
            // split as read, one 16-k step of six bf16 MFMAs for the half
            bf16x8 ah, am, al;
            split_x3_8(av, ah, am, al);
            acc = mfma_x6_lazy(ah, am, al, bv, acc);
          } else {
#pragma unroll
            for (int s = 0; s < 8; ++s)
              acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av[s], bv[s], acc, 0, 0, 0);
          }
        }
        if constexpr (kLate) {
          if (h == 0) fetch_h(k0, 1);
          else if (k0 + BKT < kend) fetch_h(k0 + BKT, 0);
        }
      }
    }
    __syncthreads();                 // staging windows are reused as reduction scratch
  } else {
  load(kbeg);
  const float* pa = As + (wk * 32 + (lane >> 5)) * SA + wm * 32 + (lane & 31);
  const float* pb = Bs + (wk * 32 + (lane >> 5)) * SB + wn * 32 + (lane & 31);
  for (int k0 = kbeg; k0 < kend; k0 += BKT) {
    stash();
    __syncthreads();
    if (k0 + BKT < kend) load(k0 + BKT);
    if (k0 + wk * 32 < kend) {              // wave-uniform: bands past the end are all zero
#pragma unroll
      for (int s = 0; s < 32; s += 2)
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(pa[s * SA], pb[s * SB], acc, 0, 0, 0);
    }
    __syncthreads();
  }
  }
  // C/D layout of the 32x32 f32 MFMA: col = lane & 31, row = (r&3) + 8(r>>2) + 4(lane>>5)
  if constexpr (HasBlock<EP>::value) {
    static_assert(WK == 1, "block epilogues take whole tiles (WK == 1)");
    // the block's tile -> LDS [BM][BN + 1] (the K loop's last barrier freed the staging)
    constexpr int LDT = BN + 1;
#pragma unroll
    for (int r = 0; r < 16; ++r)
      smem[(wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5)) * LDT + wn * 32 + (lane & 31)] = acc[r];
    __syncthreads();
    E.block(smem, LDT, m0, n0, M, N);
    return;
  }
  if constexpr (HasVec<EP>::value) {
    static_assert(WK == 1, "vector epilogues take whole tiles (WK == 1)");
    // the wave's tile -> its own LDS window (rows padded to 33), then 8 lanes per row
    // read 4 consecutive columns each: 16-B epilogue loads and stores, 8 rows per
    // instruction.  The K loop's last barrier has freed the staging slices.
    float* W = smem + wave * (32 * 33);
#pragma unroll
    for (int r = 0; r < 16; ++r) W[((r & 3) + 8 * (r >> 2) + 4 * (lane >> 5)) * 33 + (lane & 31)] = acc[r];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if constexpr (HasVecPre<EP>::value) {
      const int c = 4 * (lane & 7), n = n0 + wn * 32 + c;
      auto mrow = [&](int it) { return m0 + wm * 32 + 8 * it + (lane >> 3); };
      // one row group's loads ahead (all four, or three, ahead measured slower)
      typename EP::VPre p = E.vpre(min(mrow(0), M - 1), n);
#pragma unroll
      for (int it = 0; it < 4; ++it) {
        typename EP::VPre nx = p;
        if (it < 3) nx = E.vpre(min(mrow(it + 1), M - 1), n);   // clamped: loads never branch
        const float* q = W + (8 * it + (lane >> 3)) * 33 + c;
        const int m = mrow(it);
        if (m < M && n < N) E.vcommit(m, n, make_float4(q[0], q[1], q[2], q[3]), p);
        p = nx;
      }
      return;
    }
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int row = 8 * it + (lane >> 3), c = 4 * (lane & 7);
      const float* q = W + row * 33 + c;
      const int m = m0 + wm * 32 + row, n = n0 + wn * 32 + c;
      if (m < M && n < N) E.vec4(m, n, make_float4(q[0], q[1], q[2], q[3]));
    }
    return;
  }
  if (WK == 1) {
    const int n = n0 + wn * 32 + (lane & 31);
    if constexpr (HasPre<EP>::value) {      // all loads first, then updates + stores
      typename EP::Pre q[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        q[r] = E.pre(min(m, M - 1), min(n, N - 1));     // clamped: loads never branch
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        if (m < M && n < N) E.commit(m, n, acc[r], q[r]);
      }
    } else {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        if (m < M && n < N) E(m, n, acc[r], bz);
      }
    }
    return;
  }
  // partials -> LDS [wk][tile][r][lane]
  {
    float* red = smem + (wk * WM * WN + wm + WM * wn) * 1024 + lane;
#pragma unroll
    for (int r = 0; r < 16; ++r) red[r * 64] = acc[r];
  }
  __syncthreads();
  if constexpr (kPf) {
#pragma unroll
    for (int i = 0; i < NE; ++i) {
      const int e = tid + i * T;
      if (e >= OUT) break;
      float v = smem[e];
#pragma unroll
      for (int j = 1; j < WK; ++j) v = __fadd_rn(v, smem[j * OUT + e]);
      const int tile = e >> 10, r = (e >> 6) & 15, l = e & 63;
      const int m = m0 + (tile % WM) * 32 + (r & 3) + 8 * (r >> 2) + 4 * (l >> 5);
      const int n = n0 + (tile / WM) * 32 + (l & 31);
      if (m < M && n < N) E.apply(m, n, v, pfv[i]);
    }
    return;
  }
  for (int e = tid; e < OUT; e += T) {
    float v = smem[e];
#pragma unroll
    for (int j = 1; j < WK; ++j) v = __fadd_rn(v, smem[j * OUT + e]);
    const int tile = e >> 10, r = (e >> 6) & 15, l = e & 63;
    const int m = m0 + (tile % WM) * 32 + (r & 3) + 8 * (r >> 2) + 4 * (l >> 5);
    const int n = n0 + (tile / WM) * 32 + (l & 31);
    if (m < M && n < N) E(m, n, v, bz);
  }
}

template <int WM, int WN, int WK, class AL, class BL, class EP, bool kX6 = false>
__global__ __launch_bounds__(64 * WM * WN * WK) void k_igemm(AL A, BL B, EP E, int M, int N, int K,
                                                             int kchunk) {
  constexpr int kTile0 = Tile<WM, WN, WK>::template lds<AL, BL>();
  // the block-shared x6 planes, floats (the wave-private form splits as it reads)
  constexpr int kX6Img = kX6 && !Tile<WM, WN, WK>::kPrivate
                             ? (X6Of<AL::kFast, 32 * WM, 32 * WK>::BYTES +
                                X6Of<BL::kFast, 32 * WN, 32 * WK>::BYTES) / 4
                             : 0;
  constexpr int kTile = kTile0 > kX6Img ? kTile0 : kX6Img;
  constexpr int kVecW = HasVec<EP>::value ? WM * WN * WK * 32 * 33 : 0;   // vector epilogue windows
  // block epilogue tile (+ EP::kBlockExtra floats of scratch after it)
  constexpr int kBlkW = HasBlock<EP>::value ? 32 * WM * (32 * WN + 1) + BlockExtra<EP>::value : 0;
  constexpr int kEpi = kVecW > kBlkW ? kVecW : kBlkW;
  __shared__ __attribute__((aligned(16))) float smem[kTile > kEpi ? kTile : kEpi];
  // (an XCD-aware tile order measured slower for IQN: the operands sit in the Infinity
  // Cache and the fp32 tiles are matrix-core bound)
  igemm_block<WM, WN, WK, AL, BL, EP, true, kX6>(A, B, E, M, N, K, kchunk, blockIdx.x, blockIdx.y,
                                                blockIdx.z, smem);
}

// ordered split-K sum + epilogue: element i of the (M x N) result, slab loads in flight together
template <class EP>
__device__ __forceinline__ void splitk_sum(const float* ws, int splits, int M, int N, const EP& E,
                                           int64_t i) {
  if (i >= (int64_t)M * N) return;
  const int64_t MN = (int64_t)M * N;
  // 8 slab loads in flight per memory round (16, or an optimizer epilogue's parameter /
  // moment loads issued before the sum, measured slower in round 4)
  constexpr int kBatch = 8;
  float s = ws[i];
  for (int z0 = 1; z0 < splits; z0 += kBatch) {
    float v[kBatch];
#pragma unroll
    for (int u = 0; u < kBatch; ++u) v[u] = ws[(int64_t)min(z0 + u, splits - 1) * MN + i];
#pragma unroll
    for (int u = 0; u < kBatch; ++u) s = z0 + u < splits ? __fadd_rn(s, v[u]) : s;
  }
    E((int)(i / N), (int)(i % N), s, 0);
}

template <class EP>
__global__ __launch_bounds__(256) void k_splitk_reduce(const float* ws, int splits, int M, int N, EP E) {
  splitk_sum(ws, splits, M, N, E, (int64_t)blockIdx.x * blockDim.x + threadIdx.x);
}

// the same sums 4 elements per thread with 16-B slab loads (M * N % 4 == 0); each element
// still goes through the epilogue on its own, in the same slab order
// kU slab loads in flight per round, summed in slab order
template <int kU>
__device__ __forceinline__ void splitk_sum4(const float* ws, int splits, int64_t MN, int64_t i,
                                            float4& s) {
  for (int z0 = 1; z0 < splits; z0 += kU) {
    float4 v[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) v[u] = ld4(ws + (int64_t)min(z0 + u, splits - 1) * MN + i);
#pragma unroll
    for (int u = 0; u < kU; ++u)
      if (z0 + u < splits) {
        s.x = __fadd_rn(s.x, v[u].x);
        s.y = __fadd_rn(s.y, v[u].y);
        s.z = __fadd_rn(s.z, v[u].z);
        s.w = __fadd_rn(s.w, v[u].w);
      }
  }
}

template <class EP>
__global__ __launch_bounds__(256) void k_splitk_reduce4(const float* ws, int splits, int M, int N, EP E) {
  const int64_t i = 4 * ((int64_t)blockIdx.x * blockDim.x + threadIdx.x);
  const int64_t MN = (int64_t)M * N;
  if (i >= MN) return;
  float4 s = ld4(ws + i);
  // few slabs (IQN's FC1 / dW1: 4 / 2): no clamped duplicate loads of the last slab
  switch (splits) {
    case 1: break;
    case 2: splitk_sum4<1>(ws, splits, MN, i, s); break;
    case 3: splitk_sum4<2>(ws, splits, MN, i, s); break;
    case 4: splitk_sum4<3>(ws, splits, MN, i, s); break;
    case 5: splitk_sum4<4>(ws, splits, MN, i, s); break;
    default: splitk_sum4<8>(ws, splits, MN, i, s); break;
  }
  const float r[4] = {s.x, s.y, s.z, s.w};
  int m = (int)(i / N), n = (int)(i - (int64_t)m * N);   // one division, then step along the row
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    E(m, n, r[u], 0);
    if (++n == N) {
      n = 0;
      ++m;
    }
  }
}


struct Ctx {
  hipStream_t s;
  float* ws;       // split-K slabs
  bool dry;
  size_t need;
  size_t take(size_t n) {        // carve a private workspace region (grouped ops run together)
    const size_t o = need;
    need += (n + 3) / 4 * 4;
    return o;
  }
};

// K slice per split (multiple of the block's K slice)
inline int split_chunk(int K, int splits, int bkt) {
  return ((K + splits - 1) / splits + bkt - 1) / bkt * bkt;
}

template <int WM, int WN, int WK, bool kX6, class AL, class BL, class EP>
void gemm_form(Ctx& c, AL a, BL b, EP e, int M, int N, int K, int splits) {
  constexpr int BKT = 32 * WK, T = 64 * WM * WN * WK;
  const unsigned gx = (M + 32 * WM - 1) / (32 * WM), gy = (N + 32 * WN - 1) / (32 * WN);
  const int kchunk = splits > 1 ? split_chunk(K, splits, BKT) : K;
  const int nz = splits > 1 ? (K + kchunk - 1) / kchunk : 1;
  if (nz > 1) {
    const size_t need = (size_t)nz * M * N;
    c.need = need > c.need ? need : c.need;
  }
  if (c.dry) return;
  if (nz == 1) {
    hipLaunchKernelGGL((k_igemm<WM, WN, WK, AL, BL, EP, kX6>), dim3(gx, gy, 1), dim3(T), 0, c.s, a, b,
                       e, M, N, K, K);
    return;
  }
  hipLaunchKernelGGL((k_igemm<WM, WN, WK, AL, BL, EpiPartial, kX6>), dim3(gx, gy, nz), dim3(T), 0, c.s,
                     a, b, EpiPartial{c.ws, M, N}, M, N, K, kchunk);
  const int64_t total = (int64_t)M * N;
  if (total % 4 == 0)
    hipLaunchKernelGGL((k_splitk_reduce4<EP>), dim3((unsigned)((total / 4 + 255) / 256)), dim3(256),
                       0, c.s, c.ws, nz, M, N, e);
  else
    hipLaunchKernelGGL((k_splitk_reduce<EP>), dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                       c.s, c.ws, nz, M, N, e);
}

// The Nature-CNN's form: exact-fp32 MFMA (v_mfma_f32_32x32x2_f32); -DDQ_CNN_X6=1 builds
// the wave-private tiles (one 32 x 32 tile per wave, split as read) on the split-bf16
// form for A/B runs.  One rule for gemm() and the grouped launches' GemmOp, so the
// per-layer and grouped schedules stay bitwise equal.
#ifndef DQ_CNN_X6
#define DQ_CNN_X6 0
#endif
template <class L, class = void>
struct IsConvFwd : std::false_type {};
template <class L>
struct IsConvFwd<L, std::void_t<decltype(L::kConvFwd)>> : std::integral_constant<bool, L::kConvFwd> {};
// DQ_CNN_X6: 1 = every wave-private tile, 2 = only the forward convolutions' (Im2col A)
template <int WM, int WN, int WK, class AL>
constexpr bool cnn_x6() {
  return Tile<WM, WN, WK>::kPrivate && (DQ_CNN_X6 == 1 || (DQ_CNN_X6 == 2 && IsConvFwd<AL>::value));
}
template <int WM, int WN, int WK, class AL, class BL, class EP>
void gemm(Ctx& c, AL a, BL b, EP e, int M, int N, int K, int splits = 1) {
  gemm_form<WM, WN, WK, cnn_x6<WM, WN, WK, AL>()>(c, a, b, e, M, N, K, splits);
}
// split-bf16 MFMA (X6Img): fp32 to rounding at 2.7x the f32 matrix rate
template <int WM, int WN, int WK, class AL, class BL, class EP>
void gemm_x6(Ctx& c, AL a, BL b, EP e, int M, int N, int K, int splits = 1) {
  gemm_form<WM, WN, WK, true>(c, a, b, e, M, N, K, splits);
}


}  // namespace cnn
}  // namespace dq
