// How v_mfma_f32_32x32x16_bf16 rounds its fp32 accumulation, against the f32 form
// (v_mfma_f32_32x32x2_f32, documented as an fmaf chain) and float64 on the host.
// One wave, one 32 x 32 tile, a long K chain of operands that are exact in bf16 (so
// every product is exact and only the accumulation rounds); all-positive operands
// expose a rounding bias (truncation drifts linearly with K, round-to-nearest does not).
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/mfma_acc tools/micro/mfma_acc.hip && /tmp/mfma_acc
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

// A [32][K], B [K][32] fp32 (bf16-exact values); out[2][32][32]: bf16 MFMA, f32 MFMA
__global__ void k_acc(const float* A, const float* B, int K, float* out) {
  const int lane = threadIdx.x, r = lane & 31, h = lane >> 5;
  f32x16 c1, c2;
  for (int i = 0; i < 16; ++i) c1[i] = c2[i] = 0.0f;
  for (int k0 = 0; k0 < K; k0 += 16) {
    bf16x8 a, b;
    for (int j = 0; j < 8; ++j) {
      a[j] = (__bf16)A[r * K + k0 + 8 * h + j];
      b[j] = (__bf16)B[(k0 + 8 * h + j) * 32 + r];
    }
    c1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c1, 0, 0, 0);
  }
  for (int k0 = 0; k0 < K; k0 += 2)
    c2 = __builtin_amdgcn_mfma_f32_32x32x2f32(A[r * K + k0 + h], B[(k0 + h) * 32 + r], c2, 0, 0, 0);
  for (int i = 0; i < 16; ++i) {
    const int row = (i & 3) + 8 * (i >> 2) + 4 * h;
    out[row * 32 + r] = c1[i];
    out[1024 + row * 32 + r] = c2[i];
  }
}

static float bf16_round(float x) {   // round to a bf16-exact float (nearest even)
  unsigned u;
  memcpy(&u, &x, 4);
  u = (u + 0x7fff + ((u >> 16) & 1)) & 0xffff0000u;
  float y;
  memcpy(&y, &u, 4);
  return y;
}

int main() {
  for (int sign = 0; sign < 2; ++sign) {
    for (int K : {512, 4096}) {
      std::vector<float> A(32 * K), B(K * 32);
      srand(7 + K + sign);
      for (auto& v : A) v = bf16_round((float)rand() / RAND_MAX * (sign ? 2.0f : 1.0f) - (sign ? 1.0f : 0.0f) + 0.001f);
      for (auto& v : B) v = bf16_round((float)rand() / RAND_MAX * (sign ? 2.0f : 1.0f) - (sign ? 1.0f : 0.0f) + 0.001f);
      float *dA, *dB, *dO;
      hipMalloc(&dA, A.size() * 4);
      hipMalloc(&dB, B.size() * 4);
      hipMalloc(&dO, 2048 * 4);
      hipMemcpy(dA, A.data(), A.size() * 4, hipMemcpyHostToDevice);
      hipMemcpy(dB, B.data(), B.size() * 4, hipMemcpyHostToDevice);
      hipLaunchKernelGGL(k_acc, dim3(1), dim3(64), 0, 0, dA, dB, K, dO);
      std::vector<float> O(2048);
      hipMemcpy(O.data(), dO, 2048 * 4, hipMemcpyDeviceToHost);
      double e1 = 0, e2 = 0, b1 = 0, b2 = 0, scale = 0;
      for (int i = 0; i < 32; ++i)
        for (int j = 0; j < 32; ++j) {
          double s = 0, sa = 0;
          for (int k = 0; k < K; ++k) {
            s += (double)A[i * K + k] * B[k * 32 + j];
            sa += fabs((double)A[i * K + k] * B[k * 32 + j]);
          }
          scale += sa / 1024;
          const double d1 = O[i * 32 + j] - s, d2 = O[1024 + i * 32 + j] - s;
          e1 = fmax(e1, fabs(d1) / sa);
          e2 = fmax(e2, fabs(d2) / sa);
          b1 += d1 / sa / 1024;
          b2 += d2 / sa / 1024;
        }
      printf("%s K=%d  bf16 mfma: max |err|/sum|ab| %.3e mean signed %.3e   f32 mfma: %.3e %.3e\n",
             sign ? "mixed-sign" : "positive", K, e1, b1, e2, b2);
      hipFree(dA);
      hipFree(dB);
      hipFree(dO);
    }
  }
  return 0;
}
