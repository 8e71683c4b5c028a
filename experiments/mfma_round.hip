// Debug: rounding behaviour of v_mfma_f32_32x32x16_bf16 accumulation on gfx950.
// Each lane-row computes D = C + sum_k A[m][k] B[k][n]; compare with the exact (double) value.
//   case 0: C = 1.0, products tiny (exact sum needs more bits than fp32): C-add rounding
//   case 1: C = 0, products of mixed magnitude: internal sum rounding
//   case 2: C = 1.0, one product 2^-25 (half ulp of 1.0) and 2^-26 ... ties
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
#include <vector>
#include <random>
#include <cstring>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

__global__ void mfma_kernel(const float *A, const float *B, const float *C, float *D) {
  // A: 32x16 row-major, B: 16x32 (k-major), C/D: 32x32 row-major; one wave
  const int lane = threadIdx.x;
  bf16x8 a, b;
  for (int i = 0; i < 8; ++i) {
    a[i] = (__bf16)A[(lane & 31) * 16 + 8 * (lane >> 5) + i];
    b[i] = (__bf16)B[(8 * (lane >> 5) + i) * 32 + (lane & 31)];
  }
  floatx16 c;
  for (int r = 0; r < 16; ++r) c[r] = C[((r & 3) + 8 * (r >> 2) + 4 * (lane >> 5)) * 32 + (lane & 31)];
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
  for (int r = 0; r < 16; ++r) D[((r & 3) + 8 * (r >> 2) + 4 * (lane >> 5)) * 32 + (lane & 31)] = c[r];
}

static float bf(float v) {  // exactly representable in bf16 (truncate mantissa)
  uint32_t u;
  std::memcpy(&u, &v, 4);
  u &= 0xffff0000u;
  std::memcpy(&v, &u, 4);
  return v;
}

int main() {
  std::mt19937 rng(1);
  std::uniform_real_distribution<float> U(0.f, 1.f);
  float *dA, *dB, *dC, *dD;
  hipMalloc(&dA, 32 * 16 * 4); hipMalloc(&dB, 16 * 32 * 4); hipMalloc(&dC, 32 * 32 * 4); hipMalloc(&dD, 32 * 32 * 4);
  for (int cs = 0; cs < 4; ++cs) {
    double bias = 0, rms = 0;
    int trials = 200, cnt = 0, below = 0, above = 0;
    for (int t = 0; t < trials; ++t) {
      std::vector<float> A(512), B(512), C(1024), D(1024);
      for (int i = 0; i < 512; ++i) {
        float sa = cs == 1 ? std::ldexp(1.f, -(int)(U(rng) * 12)) : std::ldexp(1.f, -12);
        A[i] = bf(sa * (0.5f + U(rng)));
        B[i] = bf((cs == 3 ? (U(rng) - 0.5f) : 1.f) * (0.5f + U(rng)) * std::ldexp(1.f, -8));
      }
      for (int i = 0; i < 1024; ++i) C[i] = cs == 1 ? 0.f : (cs == 3 ? (U(rng) - 0.5f) : 1.f + U(rng));
      hipMemcpy(dA, A.data(), 2048, hipMemcpyHostToDevice);
      hipMemcpy(dB, B.data(), 2048, hipMemcpyHostToDevice);
      hipMemcpy(dC, C.data(), 4096, hipMemcpyHostToDevice);
      hipLaunchKernelGGL(mfma_kernel, dim3(1), dim3(64), 0, 0, dA, dB, dC, dD);
      hipMemcpy(D.data(), dD, 4096, hipMemcpyDeviceToHost);
      for (int m = 0; m < 32; ++m)
        for (int n = 0; n < 32; ++n) {
          double ex = C[m * 32 + n];
          for (int k = 0; k < 16; ++k) ex += (double)A[m * 16 + k] * (double)B[k * 32 + n];
          const double ulp = std::ldexp(1.0, std::ilogb(ex) - 23);
          const double e = (D[m * 32 + n] - ex) / ulp;
          bias += e; rms += e * e; ++cnt;
          const float rn = (float)ex;  // round-to-nearest reference
          if (D[m * 32 + n] < rn) ++below;
          if (D[m * 32 + n] > rn) ++above;
        }
    }
    printf("case %d: mean err %+.3f ulp, rms %.3f ulp; vs RNE fp32: %d below, %d above of %d\n", cs, bias / cnt,
           std::sqrt(rms / cnt), below, above, cnt);
  }
  return 0;
}
