// Shared helpers for the adaptseg gfx950 kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
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

// The train-mode BatchNorm affine, (x - mean) * invstd * w + b: one expression for every kernel
// that evaluates it (bn.hip's apply passes and mask recomputation, the conv kernels' operand-BN
// gathers), so their results agree bit for bit
__device__ __forceinline__ float bn_affine(float v, float m, float is, float w, float b) {
  return (v - m) * is * w + b;
}
// bn_apply2d_kernel's BN + ReLU output of one element (no residual): fwd_act(affine + 0, ReLU)
__device__ __forceinline__ float bn_relu(float v, float m, float is, float w, float b) {
  return fmaxf(bn_affine(v, m, is, w, b) + 0.f, 0.f);
}

// F32X3 operand split: v = hi + mid + lo EXACTLY, each term the RNE bf16 of what is left
// (3 x 8 significant bits cover fp32's 24; bf16 has fp32's exponent range).  The conv kernels
// split their staged operands with it and the BatchNorm passes write the term images the
// LDS-DMA F32X3 kernels read (conv_x3.hpp, conv_x3r.hpp) with it, so both give the same bits.
typedef float floatx2v __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

// (a, b) -> packed bf16 pair (RNE, one v_cvt_pk_bf16_f32) and the two values it rounds to
__device__ __forceinline__ uint32_t rne2(float a, float b, float &ra, float &rb) {
  const floatx2v f = {a, b};
  const uint32_t u = __builtin_bit_cast(uint32_t, __builtin_convertvector(f, bf16x2));
  ra = __uint_as_float(u << 16);
  rb = __uint_as_float(u & 0xffff0000u);
  return u;
}

// v = hi + mid + lo exactly (each term RNE to bf16), for a pair of values: packed bf16 pairs.
// The subtractions are scalar on purpose: beside MFMAs a v_pk_add_f32 costs more issue cycles
// than two v_add_f32 (MI355X_MICROARCH.md, per-instruction constants), and the kernels that
// split in-kernel are built with -fno-slp-vectorize so the compiler does not pack them either.
__device__ __forceinline__ void split3_2(float a, float b, uint32_t &hi, uint32_t &mid, uint32_t &lo) {
  float ha, hb, ma, mb;
  hi = rne2(a, b, ha, hb);
  a -= ha;
  b -= hb;
  mid = rne2(a, b, ma, mb);
  const float la = a - ma, lb = b - mb;
  const floatx2v r = {la, lb};
  lo = __builtin_bit_cast(uint32_t, __builtin_convertvector(r, bf16x2));
}

// four elements -> three packed 4 x bf16
__device__ __forceinline__ void split3(float4 v, uint2 &hi, uint2 &mid, uint2 &lo) {
  split3_2(v.x, v.y, hi.x, mid.x, lo.x);
  split3_2(v.z, v.w, hi.y, mid.y, lo.y);
}

// four elements back from their three term images (hi + mid is exact, + lo gives v exactly)
__device__ __forceinline__ float4 join3(uint2 h, uint2 m, uint2 l) {
  auto f = [](uint32_t u, bool up) { return __uint_as_float(up ? (u & 0xffff0000u) : (u << 16)); };
  return make_float4((f(h.x, false) + f(m.x, false)) + f(l.x, false), (f(h.x, true) + f(m.x, true)) + f(l.x, true),
                     (f(h.y, false) + f(m.y, false)) + f(l.y, false), (f(h.y, true) + f(m.y, true)) + f(l.y, true));
}

int conv_math();   // process-wide conv arithmetic (adaptseg_conv_set_math)
int x3h_mode();        // ADAPTSEG_OPT_X3H (adaptseg_conv_set_option, conv_igemm.hip)
int g16_wide_mode();   // ADAPTSEG_OPT_G16_WIDE
// Operand copies of the _x entry points are three exact bf16 term images [3][rows][C] under the
// F32X3 maths (one bf16 RNE image under the BF16 maths)
inline bool copies_are_terms() {
  return conv_math() == ADAPTSEG_MATH_F32X3 || conv_math() == ADAPTSEG_MATH_F32X3_PRESPLIT;
}

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
// Execution-time form for the conv GEMMs: the slot's events are handed to the next launch_k
// of this thread, which launches through hipExtLaunchKernel with them, so they time the
// kernel's own execution (what rocprofv3 reports) rather than its stream time.  With stream
// timing on (adaptseg_timing_enable_stream) a second event pair brackets the stream time too.
void timing_begin_exec(int kernel_id, hipStream_t s, double units, int *slot);
bool timing_take_exec(hipEvent_t &start, hipEvent_t &stop);

// Launch a kernel; a pending execution-timed slot (timing_begin_exec) gets its events.
template <typename... P, typename... A>
inline void launch_k(void (*kern)(P...), dim3 grid, dim3 block, hipStream_t s, A... args) {
  hipEvent_t e0, e1;
  if (timing_take_exec(e0, e1)) hipExtLaunchKernelGGL(kern, grid, block, 0, s, e0, e1, 0, args...);
  else hipLaunchKernelGGL(kern, grid, block, 0, s, args...);
}

}  // namespace adaptseg
