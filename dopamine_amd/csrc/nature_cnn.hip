// The Nature-CNN (atari_lib.py:85-144: conv 32@8x8/4, 64@4x4/2, 64@3x3/1 with TF
// "SAME" padding, ReLU, flatten 7744 in NHWC order, FC 512 + ReLU, FC n_out)
// forward and backward as implicit-GEMM kernels on the exact-fp32 matrix cores
// (v_mfma_f32_32x32x2_f32: bit-for-bit a k-ordered fp32 FMA chain).
//
// One templated tile kernel serves every product; operands are produced by
// loaders (implicit im2col with compile-time geometry, transposed-conv gathers
// with the ReLU mask fused, plain row-major) and results consumed by
// epilogues (bias + ReLU, ReLU-mask, split-K partial slabs).  Split-K partials
// are summed in slab order by a separate reduce kernel (deterministic), which
// also routes weight/bias gradients (the bias gradient is the GEMM's extra
// "ones" column) straight into the flat gradient buffer.
//
// Activations are NHWC fp32; weights live in the flat parameter buffer as
// conv (out, kh, kw, in) and FC (out, in) -- the GEMM's natural [M][K] layouts.
#include "common.h"

namespace dq {
namespace cnn {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int BK = 32;

// ----------------------------------------------------------------- geometry
template <int H_, int W_, int CI_, int KH_, int KW_, int S_, int PT_, int PL_, int OH_, int OW_, int CO_>
struct Conv {
  static constexpr int H = H_, W = W_, CI = CI_, KH = KH_, KW = KW_, S = S_, PT = PT_, PL = PL_;
  static constexpr int OH = OH_, OW = OW_, CO = CO_;
  static constexpr int K = KH * KW * CI;     // im2col depth
};
// TF SAME: conv1 84 -> 21 (pad 2/2), conv2 21 -> 11 (pad 1/2), conv3 11 -> 11 (pad 1/1)
using Conv1 = Conv<84, 84, 4, 8, 8, 4, 2, 2, 21, 21, 32>;
using Conv2 = Conv<21, 21, 32, 4, 4, 2, 1, 1, 11, 11, 64>;
using Conv3 = Conv<11, 11, 64, 3, 3, 1, 1, 1, 11, 11, 64>;
constexpr int kFlat = 11 * 11 * 64;   // 7744
constexpr int kHidden = 512;
// split-K factors (enough K-slices to put >= ~250 blocks on the 256 CUs)
constexpr int kSplitFc1 = 16, kSplitFc2 = 8, kSplitConvW = 24, kSplitConv1W = 32;

// ------------------------------------------------------------------ loaders
// A(m, k) / B(n, k) element producers.  kFast = true: consecutive threads walk k
// (k contiguous in memory); false: they walk m / n.

// forward im2col of an NHWC input: rows = output pixels, k = (kh, kw, ci)
template <class G>
struct Im2col {
  static constexpr bool kFast = true;
  const float* x;
  __device__ __forceinline__ float operator()(int m, int k) const {
    const int b = m / (G::OH * G::OW), p = m - b * (G::OH * G::OW);
    const int oh = p / G::OW, ow = p - oh * G::OW;
    const int kk = k / G::CI, ci = k - kk * G::CI;
    const int kh = kk / G::KW, kw = kk - kh * G::KW;
    const int ih = oh * G::S - G::PT + kh, iw = ow * G::S - G::PL + kw;
    if (ih < 0 || ih >= G::H || iw < 0 || iw >= G::W) return 0.0f;
    return x[((b * G::H + ih) * G::W + iw) * G::CI + ci];
  }
};

// im2col as the B operand of a weight gradient: rows k = pixels, cols n = (kh,kw,ci);
// column n == G::K is the bias "ones" column.
template <class G>
struct Im2colT {
  static constexpr bool kFast = false;   // n (ci innermost) contiguous
  const float* x;
  __device__ __forceinline__ float operator()(int n, int k) const {
    if (n == G::K) return 1.0f;
    Im2col<G> f{x};
    return f(k, n);
  }
};

// gradient of a conv input (transposed conv): rows m = input pixels (b, ih, iw),
// k = (kh, kw, co); dy is NHWC (B, OH, OW, CO).
template <class G>
struct Col2im {
  static constexpr bool kFast = true;
  const float* dy;
  __device__ __forceinline__ float operator()(int m, int k) const {
    const int b = m / (G::H * G::W), p = m - b * (G::H * G::W);
    const int ih = p / G::W, iw = p - ih * G::W;
    const int kk = k / G::CO, co = k - kk * G::CO;
    const int kh = kk / G::KW, kw = kk - kh * G::KW;
    const int th = ih + G::PT - kh, tw = iw + G::PL - kw;   // = oh * S, ow * S
    if (th < 0 || tw < 0) return 0.0f;
    const int oh = th / G::S, ow = tw / G::S;
    if (oh * G::S != th || ow * G::S != tw || oh >= G::OH || ow >= G::OW) return 0.0f;
    return dy[((b * G::OH + oh) * G::OW + ow) * G::CO + co];
  }
};

// conv weights as B of the transposed conv: B(n = ci, k = (kh, kw, co)) = W[co][kh][kw][ci]
template <class G>
struct WeightT {
  static constexpr bool kFast = false;   // n = ci contiguous
  const float* w;
  __device__ __forceinline__ float operator()(int n, int k) const {
    const int kk = k / G::CO, co = k - kk * G::CO;
    return w[(co * (G::KH * G::KW) + kk) * G::CI + n];
  }
};

// plain row-major [rows][ld], k contiguous (x of an FC layer, weights [N][K])
struct RowK {
  static constexpr bool kFast = true;
  const float* p;
  int ld;
  __device__ __forceinline__ float operator()(int r, int k) const { return p[(int64_t)r * ld + k]; }
};
// [k][rows] with rows contiguous: dy^T of FC dW (A), and W of FC dX as B(n = in, k = out)
struct ColK {
  static constexpr bool kFast = false;
  const float* p;
  int ld;
  __device__ __forceinline__ float operator()(int r, int k) const { return p[(int64_t)k * ld + r]; }
};
// FC dW's B operand: B(n, k = batch) = x[k][n], with the bias ones-column at n == ld
struct ColKOnes {
  static constexpr bool kFast = false;
  const float* p;
  int ld;
  __device__ __forceinline__ float operator()(int n, int k) const {
    return n == ld ? 1.0f : p[(int64_t)k * ld + n];
  }
};
// conv dW's A operand: A(m = co, k = pixel) = dy[pixel][co]
template <int CO>
struct DyT {
  static constexpr bool kFast = false;
  const float* dy;
  __device__ __forceinline__ float operator()(int m, int k) const { return dy[(int64_t)k * CO + m]; }
};

// ---------------------------------------------------------------- epilogues
struct EpiBiasAct {          // out[m][n] = act(acc + bias[n])
  float* out;
  const float* bias;
  int ld;
  bool relu;
  __device__ __forceinline__ void operator()(int m, int n, float v, int) const {
    v = __fadd_rn(v, bias[n]);
    out[(int64_t)m * ld + n] = relu ? fmaxf(v, 0.0f) : v;
  }
};
struct EpiMask {             // out[m][n] = acc * (act[m][n] > 0)   (ReLU backward)
  float* out;
  const float* act;
  int ld;
  __device__ __forceinline__ void operator()(int m, int n, float v, int) const {
    const int64_t i = (int64_t)m * ld + n;
    out[i] = act[i] > 0.0f ? v : 0.0f;
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

// ------------------------------------------------------------- tile kernel
// Block = WM x WN waves, each owning a 32x32 output tile; K swept in BK = 32 slices
// staged through LDS ([k][m] / [k][n], padded), next slice prefetched into
// registers while the MFMAs of the current one run.  grid.z = split-K slices.
template <int WM, int WN, class AL, class BL, class EP>
__global__ __launch_bounds__(64 * WM * WN) void k_igemm(AL A, BL B, EP E, int M, int N, int K,
                                                        int kchunk) {
  constexpr int BM = 32 * WM, BN = 32 * WN, T = 64 * WM * WN;
  constexpr int NA = BM * BK / T, NB = BN * BK / T;
  __shared__ float As[BK][BM + 1];
  __shared__ float Bs[BK][BN + 1];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave % WM, wn = wave / WM;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
  const int kbeg = blockIdx.z * kchunk;
  const int kend = min(K, kbeg + kchunk);
  float ra[NA], rb[NB];

  auto load = [&](int k0) {
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int e = i * T + tid;
      int mm, kk;
      if (AL::kFast) { mm = e / BK; kk = e - mm * BK; } else { kk = e / BM; mm = e - kk * BM; }
      const int m = m0 + mm, k = k0 + kk;
      ra[i] = (m < M && k < kend) ? A(m, k) : 0.0f;
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int e = i * T + tid;
      int nn, kk;
      if (BL::kFast) { nn = e / BK; kk = e - nn * BK; } else { kk = e / BN; nn = e - kk * BN; }
      const int n = n0 + nn, k = k0 + kk;
      rb[i] = (n < N && k < kend) ? B(n, k) : 0.0f;
    }
  };
  auto stash = [&]() {
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int e = i * T + tid;
      int mm, kk;
      if (AL::kFast) { mm = e / BK; kk = e - mm * BK; } else { kk = e / BM; mm = e - kk * BM; }
      As[kk][mm] = ra[i];
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int e = i * T + tid;
      int nn, kk;
      if (BL::kFast) { nn = e / BK; kk = e - nn * BK; } else { kk = e / BN; nn = e - kk * BN; }
      Bs[kk][nn] = rb[i];
    }
  };

  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.0f;
  if (kbeg < kend) load(kbeg);
  for (int k0 = kbeg; k0 < kend; k0 += BK) {
    stash();
    __syncthreads();
    if (k0 + BK < kend) load(k0 + BK);
    const int ar = wm * 32 + (lane & 31), bc = wn * 32 + (lane & 31), kh = lane >> 5;
#pragma unroll
    for (int s = 0; s < BK; s += 2)
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(As[s + kh][ar], Bs[s + kh][bc], acc, 0, 0, 0);
    __syncthreads();
  }
  // C/D layout of the 32x32 f32 MFMA: col = lane & 31, row = (r&3) + 8(r>>2) + 4(lane>>5)
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int m = m0 + wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
    const int n = n0 + wn * 32 + (lane & 31);
    if (m < M && n < N) E(m, n, acc[r], blockIdx.z);
  }
}

// ordered split-K sum + epilogue
template <class EP>
__global__ __launch_bounds__(256) void k_splitk_reduce(const float* ws, int splits, int M, int N, EP E) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)M * N) return;
  float s = ws[i];
  for (int z = 1; z < splits; ++z) s = __fadd_rn(s, ws[(int64_t)z * M * N + i]);
  E((int)(i / N), (int)(i % N), s, 0);
}

// K slice per split (multiple of BK) and the resulting number of slabs
inline int split_chunk(int K, int splits) { return ((K + splits - 1) / splits + BK - 1) / BK * BK; }
inline int split_count(int K, int splits) { const int c = split_chunk(K, splits); return (K + c - 1) / c; }

template <int WM, int WN, class AL, class BL, class EP>
void launch(AL a, BL b, EP e, int M, int N, int K, int splits, float* ws, hipStream_t s) {
  const unsigned gx = (M + 32 * WM - 1) / (32 * WM), gy = (N + 32 * WN - 1) / (32 * WN);
  if (splits == 1) {
    hipLaunchKernelGGL((k_igemm<WM, WN, AL, BL, EP>), dim3(gx, gy, 1), dim3(64 * WM * WN), 0, s, a,
                       b, e, M, N, K, K);
    return;
  }
  const int kchunk = split_chunk(K, splits), nz = split_count(K, splits);
  EpiPartial p{ws, M, N};
  hipLaunchKernelGGL((k_igemm<WM, WN, AL, BL, EpiPartial>), dim3(gx, gy, nz), dim3(64 * WM * WN), 0,
                     s, a, b, p, M, N, K, kchunk);
  const int64_t total = (int64_t)M * N;
  hipLaunchKernelGGL((k_splitk_reduce<EP>), dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s,
                     ws, nz, M, N, e);
}

}  // namespace cnn
}  // namespace dq

using namespace dq;
using namespace dq::cnn;

extern "C" {

int dq_cnn_forward(const dq_cnn_params* p, int32_t batch, const float* x, dq_cnn_acts* a,
                   float* ws, void* stream) {
  DQ_CHECK_ARG(p && a && x && ws && batch >= 1, "null argument");
  DQ_CHECK_ARG(p->in_channels == 4 && p->n_out >= 1, "the Nature CNN takes 84x84x4 NHWC input");
  hipStream_t s = (hipStream_t)stream;
  const int B = batch;
  // conv1 / conv2 / conv3 + bias + ReLU  (implicit GEMM: M = pixels, N = out channels)
  launch<1, 1>(Im2col<Conv1>{x}, RowK{p->conv1_w, Conv1::K}, EpiBiasAct{a->a1, p->conv1_b, 32, true},
               B * 441, 32, Conv1::K, 1, ws, s);
  launch<1, 1>(Im2col<Conv2>{a->a1}, RowK{p->conv2_w, Conv2::K}, EpiBiasAct{a->a2, p->conv2_b, 64, true},
               B * 121, 64, Conv2::K, 1, ws, s);
  launch<1, 1>(Im2col<Conv3>{a->a2}, RowK{p->conv3_w, Conv3::K}, EpiBiasAct{a->a3, p->conv3_b, 64, true},
               B * 121, 64, Conv3::K, 1, ws, s);
  // fc1 (7744 -> 512) + ReLU: weight-streaming, split-K over the 7744 inputs
  launch<1, 1>(RowK{a->a3, kFlat}, RowK{p->fc1_w, kFlat}, EpiBiasAct{a->h, p->fc1_b, kHidden, true},
               B, kHidden, kFlat, kSplitFc1, ws, s);
  // fc2 (512 -> n_out), no activation
  launch<1, 1>(RowK{a->h, kHidden}, RowK{p->fc2_w, kHidden}, EpiBiasAct{a->out, p->fc2_b, p->n_out, false},
               B, p->n_out, kHidden, kSplitFc2, ws, s);
  DQ_CHECK_LAUNCH("dq_cnn_forward");
  return DQ_OK;
}

int dq_cnn_backward(const dq_cnn_params* p, const dq_cnn_params* g, int32_t batch, const float* x,
                    const dq_cnn_acts* a, const float* dout, dq_cnn_acts* d, float* ws,
                    void* stream) {
  DQ_CHECK_ARG(p && g && a && d && x && dout && ws && batch >= 1, "null argument");
  hipStream_t s = (hipStream_t)stream;
  const int B = batch, NO = p->n_out;
  // fc2: dW2|db2 = dout^T [h | 1];  dh = (dout W2) * (h > 0)
  launch<2, 2>(ColK{dout, NO}, ColKOnes{a->h, kHidden}, EpiGrad{g->fc2_w, g->fc2_b, kHidden},
               NO, kHidden + 1, B, 1, ws, s);
  launch<1, 1>(RowK{dout, NO}, ColK{p->fc2_w, kHidden}, EpiMask{d->h, a->h, kHidden},
               B, kHidden, NO, kSplitFc2, ws, s);
  // fc1: dW1|db1 = dh^T [a3 | 1];  da3 = (dh W1) * (a3 > 0)
  launch<2, 2>(ColK{d->h, kHidden}, ColKOnes{a->a3, kFlat}, EpiGrad{g->fc1_w, g->fc1_b, kFlat},
               kHidden, kFlat + 1, B, 1, ws, s);
  launch<1, 1>(RowK{d->h, kHidden}, ColK{p->fc1_w, kFlat}, EpiMask{d->a3, a->a3, kFlat},
               B, kFlat, kHidden, 1, ws, s);
  // conv3: dW3|db3 = da3^T [im2col(a2) | 1];  da2 = col2im(da3, W3) * (a2 > 0)
  launch<2, 2>(DyT<64>{d->a3}, Im2colT<Conv3>{a->a2}, EpiGrad{g->conv3_w, g->conv3_b, Conv3::K},
               64, Conv3::K + 1, B * 121, kSplitConvW, ws, s);
  launch<1, 1>(Col2im<Conv3>{d->a3}, WeightT<Conv3>{p->conv3_w}, EpiMask{d->a2, a->a2, 64},
               B * 121, 64, 9 * 64, 1, ws, s);
  // conv2: dW2|db2 = da2^T [im2col(a1) | 1];  da1 = col2im(da2, W2) * (a1 > 0)
  launch<2, 2>(DyT<64>{d->a2}, Im2colT<Conv2>{a->a1}, EpiGrad{g->conv2_w, g->conv2_b, Conv2::K},
               64, Conv2::K + 1, B * 121, kSplitConvW, ws, s);
  launch<1, 1>(Col2im<Conv2>{d->a2}, WeightT<Conv2>{p->conv2_w}, EpiMask{d->a1, a->a1, 32},
               B * 441, 32, 16 * 64, 1, ws, s);
  // conv1: dW1|db1 = da1^T [im2col(x) | 1]   (no input gradient needed)
  launch<1, 1>(DyT<32>{d->a1}, Im2colT<Conv1>{x}, EpiGrad{g->conv1_w, g->conv1_b, Conv1::K},
               32, Conv1::K + 1, B * 441, kSplitConv1W, ws, s);
  DQ_CHECK_LAUNCH("dq_cnn_backward");
  return DQ_OK;
}

size_t dq_cnn_workspace_floats(int32_t batch, int32_t n_out) {
  // largest split-K slab set among the launches above
  size_t m = 0;
  auto upd = [&](int K, int splits, size_t MN) {
    const size_t v = (size_t)split_count(K, splits) * MN;
    m = v > m ? v : m;
  };
  upd(kFlat, kSplitFc1, (size_t)batch * kHidden);
  upd(kHidden, kSplitFc2, (size_t)batch * n_out);
  upd(n_out, kSplitFc2, (size_t)batch * kHidden);
  upd(batch * 121, kSplitConvW, (size_t)64 * (Conv3::K + 1));
  upd(batch * 121, kSplitConvW, (size_t)64 * (Conv2::K + 1));
  upd(batch * 441, kSplitConv1W, (size_t)32 * (Conv1::K + 1));
  return m;
}

}  // extern "C"
