// Shared helpers for the adaptseg gfx950 kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string>
#include "../../include/adaptseg.h"

namespace adaptseg {

void set_error(const char *fmt, ...);

#define AS_CHECK_ARG(cond, ...)                                                              \
  do {                                                                                       \
    if (!(cond)) {                                                                           \
      ::adaptseg::set_error(__VA_ARGS__);                                                    \
      return ADAPTSEG_ERR_ARG;                                                               \
    }                                                                                        \
  } while (0)

#define AS_CHECK_LAUNCH(name)                                                                \
  do {                                                                                       \
    hipError_t e_ = hipGetLastError();                                                       \
    if (e_ != hipSuccess) {                                                                  \
      ::adaptseg::set_error("%s: %s", name, hipGetErrorString(e_));                          \
      return ADAPTSEG_ERR_HIP;                                                               \
    }                                                                                        \
  } while (0)

inline hipStream_t as_stream(adaptseg_stream_t s) { return reinterpret_cast<hipStream_t>(s); }

// Unsigned division by a runtime constant: q = (umulhi(n, m) + n) >> s, valid for n < 2^31.
struct FastDiv {
  uint32_t d, m, s;
};

inline FastDiv make_fastdiv(uint32_t d) {
  FastDiv f;
  f.d = d;
  uint32_t s = 0;
  while ((1ull << s) < d) ++s;
  f.s = s;
  uint64_t num = ((1ull << 32) * ((1ull << s) - d));
  f.m = (uint32_t)(num / d + 1);
  if (d == 1) f.m = 0;  // (0 + n) >> 0 == n
  return f;
}

__device__ __forceinline__ uint32_t fdiv(uint32_t n, const FastDiv &f) {
  uint32_t hi = __umulhi(n, f.m);
  return (hi + n) >> f.s;
}

constexpr int kWave = 64;

// Fused conv epilogue activations: LEAKY (slope 0.2, discriminator) or RELU (slope 0, VGG);
// the *_GRAD forms scale a data gradient by the activation's derivative at aux (the
// activation OUTPUT, whose sign equals the pre-activation's).
__device__ __forceinline__ float epi_act(float v, int flags) {
  if (flags & ADAPTSEG_EPI_LEAKY) v = v > 0.f ? v : 0.2f * v;
  if (flags & ADAPTSEG_EPI_RELU) v = v > 0.f ? v : 0.f * v;
  return v;
}
__device__ __forceinline__ float epi_act_grad(float v, float a, int flags) {
  if (flags & ADAPTSEG_EPI_LEAKY_GRAD) v = a > 0.f ? v : 0.2f * v;
  if (flags & ADAPTSEG_EPI_RELU_GRAD) v = a > 0.f ? v : 0.f;
  return v;
}
constexpr int kEpiActGrad = ADAPTSEG_EPI_LEAKY_GRAD | ADAPTSEG_EPI_RELU_GRAD;

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

// Live timing (adaptseg_timing_*, conv_igemm.hip): hipEvent pair around one launch; `units` are
// algorithmic FLOPs (conv kernels, ids < kTimingMemBase) or algorithmic HBM bytes (ids >= it).
constexpr int kTimingMemBase = 1000;
enum TimingMemId {
  kTUpsampleFwd = 1000, kTUpsampleBwd = 1001, kTSoftmaxFwd = 1002, kTSoftmaxBwd = 1003,
  kTCeFwd = 1004, kTCeBwd = 1005, kTBnApply = 1006, kTBnBwdApply = 1007,
  kTUp2Fwd = 1008, kTUp2Bwd = 1009, kTWarpFwd = 1010, kTWarpDflow = 1011, kTWarpScatter = 1012,
  kTBnReduceStats = 1013, kTBnReduceBwd = 1014, kTSplitkReduce = 1015
};
void timing_begin(int kernel_id, hipStream_t s, double units, int *slot);
void timing_end(int slot, hipStream_t s);

}  // namespace adaptseg
