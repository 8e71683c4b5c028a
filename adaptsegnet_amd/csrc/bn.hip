// BatchNorm2d (train mode, batch statistics) for NHWC activations [rows][C] on gfx950.
// Reference: nn.BatchNorm2d(affine, frozen) + ReLU + residual add in
// model/deeplab_multi.py:65-101 (Bottleneck), :130-134 (stem), :160-162 (downsample).
//
// Forward = stats pass (per-block shifted sums -> fp64 combine, one deterministic finalize
// that also updates running_mean / running_var with the unbiased variance, as torch does)
// + one fused apply pass y = relu(xhat*w + b + res).  Backward = one reduction pass
// (sum g, sum g*(x-mean), with g = dy * [y > 0] when the forward had a ReLU) + one apply
// pass that also emits the residual gradient.  All passes are float4-vectorised and
// HBM-bound.
#include "common.hpp"
#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <initializer_list>
#include <type_traits>

namespace adaptseg {

// ReLU mask without reading y: y > 0  <=>  (x - mean)*invstd*w + b > 0, evaluated with the
// same expression bn_apply2d_kernel uses (bn_affine, common.hpp; valid for BNs without a
// residual input).
__device__ __forceinline__ float4 relu_mask_from_x(float4 g, float4 v, float4 m, float4 is, float4 w, float4 b) {
  g.x = bn_affine(v.x, m.x, is.x, w.x, b.x) > 0.f ? g.x : 0.f;
  g.y = bn_affine(v.y, m.y, is.y, w.y, b.y) > 0.f ? g.y : 0.f;
  g.z = bn_affine(v.z, m.z, is.z, w.z, b.z) > 0.f ? g.z : 0.f;
  g.w = bn_affine(v.w, m.w, is.w, w.w, b.w) > 0.f ? g.w : 0.f;
  return g;
}

// Activation-derivative mask of the backward (rmode): 0 none; 1 ReLU, sign from the saved output
// y (`o`, loaded by the caller); 2 ReLU, sign recomputed from x; 3 LeakyReLU(0.2), sign from y;
// 4 LeakyReLU(0.2), sign from x.  LeakyReLU keeps the sign, so its output is as good a mask
// source as ReLU's.
__device__ __forceinline__ float4 act_mask_o(float4 g, int rmode, float4 o, float4 v, float4 m, float4 is,
                                             float4 w, float4 b) {
  if (rmode == 2 || rmode == 4) {
    o.x = bn_affine(v.x, m.x, is.x, w.x, b.x);
    o.y = bn_affine(v.y, m.y, is.y, w.y, b.y);
    o.z = bn_affine(v.z, m.z, is.z, w.z, b.z);
    o.w = bn_affine(v.w, m.w, is.w, w.w, b.w);
  }
  const float k = rmode <= 2 ? 0.f : 0.2f;
  g.x = o.x > 0.f ? g.x : k * g.x;
  g.y = o.y > 0.f ? g.y : k * g.y;
  g.z = o.z > 0.f ? g.z : k * g.z;
  g.w = o.w > 0.f ? g.w : k * g.w;
  return g;
}

// Activation operands (x, the residual, the saved output y) are fp32 or — under the bf16 conv
// math with bf16 activation storage (config c5) — bf16: four of them as a float4.
__device__ __forceinline__ float4 lda4(const float *p) { return *reinterpret_cast<const float4 *>(p); }
__device__ __forceinline__ float4 lda4(const __bf16 *p) {
  const uint2 u = *reinterpret_cast<const uint2 *>(p);
  return make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u), __uint_as_float(u.y << 16),
                     __uint_as_float(u.y & 0xffff0000u));
}
__device__ __forceinline__ float lda1(const float *p) { return *p; }
__device__ __forceinline__ float lda1(const __bf16 *p) { return (float)*p; }

// Under the F32X3 conv maths an operand copy holds the three bf16 terms of each fp32 value
// (common.hpp split3), pixel-interleaved: [rows][3][C] (x3_off) — a row's three term rows are
// adjacent, so a pass that writes or reads them streams one region.  The residual and the
// saved output (the ReLU mask source) of a BN may then be stored as terms only, read back as
// hi + mid + lo (join3).  X3 tags that storage; its pointer is the copy's base.
struct X3 {};
template <typename T> struct Act { typedef const T *ptr; };
template <> struct Act<X3> { typedef const __bf16 *ptr; };
__device__ __forceinline__ int64_t x3_off(int64_t row, int c, int C) { return row * 3 * C + c; }
template <typename T>
__device__ __forceinline__ float4 ldr4(typename Act<T>::ptr p, int64_t row, int c, int C) {
  if constexpr (std::is_same<T, X3>::value) {
    const __bf16 *q = p + x3_off(row, c, C);
    return join3(*reinterpret_cast<const uint2 *>(q), *reinterpret_cast<const uint2 *>(q + C),
                 *reinterpret_cast<const uint2 *>(q + 2 * C));
  } else {
    return lda4(p + row * C + c);
  }
}
// The ReLU / LeakyReLU mask source: only its sign is used.  From terms the hi term alone has it:
// hi = RNE_bf16(v) is nonzero with v's sign unless |v| < 2^-134, and then mid and lo round to
// zero as well, so the stored value (hi + mid + lo) is 0 too — hi > 0 <=> stored value > 0.
template <typename T>
__device__ __forceinline__ float4 ldm4(typename Act<T>::ptr p, int64_t row, int c, int C) {
  if constexpr (std::is_same<T, X3>::value)
    return lda4(p + x3_off(row, c, C));
  else
    return lda4(p + row * C + c);
}

// A thread owns QN channel quads (4*QN consecutive channels) of a row: QN = 1 for fp32
// storage, 2 for bf16 storage (one 16-B load of 8 bf16 — at one quad per thread the bf16 passes
// issue as many memory instructions as the fp32 ones for half the bytes, and measured no faster
// per launch: l3.bn3 apply 74 us bf16 vs 69 us fp32, tools/bn_bench.py)
__device__ __forceinline__ float4 bf4(unsigned a, unsigned b) {
  return make_float4(__uint_as_float(a << 16), __uint_as_float(a & 0xffff0000u), __uint_as_float(b << 16),
                     __uint_as_float(b & 0xffff0000u));
}
template <int QN> __device__ __forceinline__ void ldq(const float *p, float4 (&o)[QN]) {
#pragma unroll
  for (int h = 0; h < QN; ++h) o[h] = *reinterpret_cast<const float4 *>(p + 4 * h);
}
template <int QN> __device__ __forceinline__ void ldq(const __bf16 *p, float4 (&o)[QN]) {
  if constexpr (QN == 2) {
    const uint4 u = *reinterpret_cast<const uint4 *>(p);
    o[0] = bf4(u.x, u.y);
    o[1] = bf4(u.z, u.w);
  } else {
#pragma unroll
    for (int h = 0; h < QN; ++h) o[h] = lda4(p + 4 * h);
  }
}
// the residual (TR) / the mask source y (TY) of a row: plain storage or F32X3 term images
template <typename T, int QN>
__device__ __forceinline__ void ldrq(typename Act<T>::ptr p, int64_t row, int c, int C, float4 (&o)[QN]) {
  if constexpr (std::is_same<T, X3>::value) {
#pragma unroll
    for (int h = 0; h < QN; ++h) o[h] = ldr4<X3>(p, row, c + 4 * h, C);
  } else {
    ldq<QN>(p + row * C + c, o);
  }
}
template <typename T, int QN>
__device__ __forceinline__ void ldmq(typename Act<T>::ptr p, int64_t row, int c, int C, float4 (&o)[QN]) {
  if constexpr (std::is_same<T, X3>::value) {
#pragma unroll
    for (int h = 0; h < QN; ++h) o[h] = ldm4<X3>(p, row, c + 4 * h, C);
  } else {
    ldq<QN>(p + row * C + c, o);
  }
}
template <int QN> __device__ __forceinline__ void zq(float4 (&o)[QN]) {
#pragma unroll
  for (int h = 0; h < QN; ++h) o[h] = make_float4(0, 0, 0, 0);
}
template <int QN> __device__ __forceinline__ void ldpq(const float *p, int c, float4 (&o)[QN], float dflt) {
#pragma unroll
  for (int h = 0; h < QN; ++h)
    o[h] = p ? *reinterpret_cast<const float4 *>(p + c + 4 * h) : make_float4(dflt, dflt, dflt, dflt);
}

constexpr int kReduceUnroll = 4;
// rows in flight per thread of the bf16-storage passes (two quads a row): 2 rows at <= 128
// VGPRs beat 4 rows at ~200 (c5 40.90 / 40.95 vs 40.57 / 40.63 images/s, one quad x 4 rows
// 38.06 / 38.21; experiments/ab_bn_bf16.sh)
constexpr int kBf16Rows = 2;
// The BN passes run beside the weight-gradient GEMMs of the side stream.  A term-image F32X3
// block (conv_x3r.hpp: 8 waves at ~200 VGPRs, one per CU) leaves 96 VGPRs per SIMD free, so
// under the F32X3_PRESPLIT program the BN blocks fit beside it only at <= 96 VGPRs
// (min 5 blocks with x2 unrolled rows: 26.79 vs 26.50 images/s there).  The default program
// runs faster with the x4-unrolled passes at their natural ~126 VGPRs: 27.44 vs 27.18 images/s
// (profiles/r3/x3_copies_ab.txt).
constexpr int kBnMinBlocks = 1;
// ~2 blocks per CU for the reduce and apply passes: they share the chip with the weight-gradient
// GEMMs of the side stream (2048 blocks measured -0.3 % at c2 with the F32X3 kernels)
constexpr int kReduceBlocks = 512, kApplyBlocks = 512;
// the forward apply passes run without the weight-gradient stream beside them: 1024 blocks
// (c5 +2.0 %, c2 +0.5 %; 2048: +1.9 / +0.2 %; the backward passes at 1024: c5 -1.2 %,
// profiles/r4/bn_grids_ab.txt)
constexpr int kApplyBlocksFwd = 1024;

// Forward activation: 0 none, 1 ReLU, 2 LeakyReLU(0.2) (model/custom_layers.py:83-96).
__device__ __forceinline__ float fwd_act(float v, int act) {
  if (act == 1) return fmaxf(v, 0.f);
  if (act == 2) return v > 0.f ? v : 0.2f * v;
  return v;
}

// ReLU mask bitmaps [rows][C / 32] (C % 32 == 0): bit c % 32 of word (row, c / 32) is set when a
// BN+ReLU output is > 0.  The forward apply writes it beside y, and the backward reads 1 bit per
// element for the mask instead of the stored y (4 B fp32 / 2 B bf16): the Bottleneck's BN3,
// whose mask gates the residual gradient as well (model/deeplab_multi.py:96-103).  The lanes of an
// aligned 32-channel group — 8 lanes of one quad (QN 1) or 4 lanes of two quads (QN 2), always
// consecutive lanes of one row in these kernels — merge their bits with xor-shuffles, and the
// group's first lane stores the word.
template <int QN>
__device__ __forceinline__ void store_mask_bits(uint32_t *bits, int64_t row, int c, int C, const float4 (&o)[QN]) {
  uint32_t v = 0;
#pragma unroll
  for (int h = 0; h < QN; ++h)
    v |= ((o[h].x > 0.f ? 1u : 0u) | (o[h].y > 0.f ? 2u : 0u) | (o[h].z > 0.f ? 4u : 0u) | (o[h].w > 0.f ? 8u : 0u))
         << (4 * h);
  v <<= (c & 31);
#pragma unroll
  for (int m = 1; m < 8 / QN; m <<= 1) v |= __shfl_xor(v, m);
  if ((c & 31) == 0) bits[row * (C >> 5) + (c >> 5)] = v;
}
// this thread's 4*QN mask bits of (row, c..): the word shifted so bit 0 is channel c
__device__ __forceinline__ uint32_t load_mask_bits(const uint32_t *bits, int64_t row, int c, int C) {
  return bits[row * (C >> 5) + (c >> 5)] >> (c & 31);
}
__device__ __forceinline__ float4 mask_quad(float4 g, uint32_t w) {
  g.x = (w & 1u) ? g.x : 0.f;
  g.y = (w & 2u) ? g.y : 0.f;
  g.z = (w & 4u) ? g.z : 0.f;
  g.w = (w & 8u) ? g.w : 0.f;
  return g;
}

// Block = 256 threads laid out as TC channel groups (QN quads each) x TR row lanes (TC*TR =
// 256).  Grid = (ceil(C / (4*QN*TC)), splits).  Partial sums land in ws[2][C][splits] (float).
// TD: storage of the incoming gradient dy (fp32, or bf16 under bf16 gradient storage)
template <int MODE, typename TX, typename TY = TX, int QN = 1, typename TD = float>  // MODE 0: stats (shifted by pivot x[0][c]), 1: backward sums
__global__ void __launch_bounds__(256, kBnMinBlocks)
bn_reduce_kernel(int64_t rows, int C, int tc, const TX *__restrict__ x, const TD *__restrict__ dy,
                 typename Act<TY>::ptr __restrict__ y, const float *__restrict__ mean, const float *__restrict__ invstd,
                 const float *__restrict__ w, const float *__restrict__ b, int relu,
                 int64_t rows_per_split, float *__restrict__ partial, const uint32_t *__restrict__ dbits = nullptr) {
  const int tr = 256 / tc;
  const int cq = threadIdx.x % tc;   // channel group within block
  const int rl = threadIdx.x / tc;   // row lane
  const int c0 = (blockIdx.x * tc + cq) * 4 * QN;
  const bool cok = c0 < C;
  const int64_t r0 = blockIdx.y * rows_per_split;
  const int64_t r1 = min(rows, r0 + rows_per_split);
  float4 s1[QN], s2[QN], piv[QN], is[QN], ww[QN], bb[QN];
  zq<QN>(s1);
  zq<QN>(s2);
  zq<QN>(is);
  zq<QN>(ww);
  zq<QN>(bb);
  if (cok) {
    if (MODE == 0) ldq<QN>(x + c0, piv);
    else ldpq<QN>(mean, c0, piv, 0.f);
    if (MODE == 1 && (relu == 2 || relu == 4)) {
      ldpq<QN>(invstd, c0, is, 0.f);
      ldpq<QN>(w, c0, ww, 1.f);
      ldpq<QN>(b, c0, bb, 0.f);
    }
    // rows unrolled with every load issued before any use (memory-level parallelism: one
    // float4 per tensor in flight per thread measured 3-4 TB/s); tail rows re-read row r and
    // are masked out of the sums
    constexpr int U = QN == 2 ? kBf16Rows : kReduceUnroll;
    for (int64_t r = r0 + rl; r < r1; r += U * tr) {
      float4 v[U][QN], g[U][QN], o[U][QN];
      uint32_t mb[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t ru = r + (int64_t)u * tr;
        const int64_t row = ru < r1 ? ru : r, e = row * C + c0;
        ldq<QN>(x + e, v[u]);
        if (MODE == 1) {
          ldq<QN>(dy + e, g[u]);
          if (relu == 1 || relu == 3) ldmq<TY, QN>(y, row, c0, C, o[u]);
          mb[u] = dbits ? load_mask_bits(dbits, row, c0, C) : ~0u;
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (r + (int64_t)u * tr >= r1) break;
#pragma unroll
        for (int h = 0; h < QN; ++h) {
          const float4 vv = v[u][h], pv = piv[h];
          const float4 d = make_float4(vv.x - pv.x, vv.y - pv.y, vv.z - pv.z, vv.w - pv.w);
          float4 &a1 = s1[h], &a2 = s2[h];
          if (MODE == 0) {
            a1.x += d.x; a1.y += d.y; a1.z += d.z; a1.w += d.w;
            a2.x += d.x * d.x; a2.y += d.y * d.y; a2.z += d.z * d.z; a2.w += d.w * d.w;
          } else {
            float4 gg = g[u][h];
            if (dbits) gg = mask_quad(gg, mb[u] >> (4 * h));
            if (relu == 2) gg = relu_mask_from_x(gg, vv, pv, is[h], ww[h], bb[h]);
            else if (relu) gg = act_mask_o(gg, relu, o[u][h], vv, pv, is[h], ww[h], bb[h]);
            a1.x += gg.x; a1.y += gg.y; a1.z += gg.z; a1.w += gg.w;
            a2.x += gg.x * d.x; a2.y += gg.y * d.y; a2.z += gg.z * d.z; a2.w += gg.w * d.w;
          }
        }
      }
    }
  }
  __shared__ float4 red1[QN][256], red2[QN][256];
#pragma unroll
  for (int h = 0; h < QN; ++h) {
    red1[h][threadIdx.x] = s1[h];
    red2[h][threadIdx.x] = s2[h];
  }
  __syncthreads();
  if (rl == 0 && cok) {
    const size_t S = gridDim.y, sp = blockIdx.y;
#pragma unroll
    for (int h = 0; h < QN; ++h) {
      float4 a = red1[h][threadIdx.x], b2 = red2[h][threadIdx.x];
      for (int i = 1; i < tr; ++i) {
        float4 u = red1[h][threadIdx.x + i * tc], v = red2[h][threadIdx.x + i * tc];
        a.x += u.x; a.y += u.y; a.z += u.z; a.w += u.w;
        b2.x += v.x; b2.y += v.y; b2.z += v.z; b2.w += v.w;
      }
      // transposed [2][C][splits]: a channel's partials are contiguous for the finalize wave
      const int c = c0 + 4 * h;
      float *p1 = partial + (size_t)c * S + sp, *p2 = partial + ((size_t)C + c) * S + sp;
      p1[0] = a.x; p1[S] = a.y; p1[2 * S] = a.z; p1[3 * S] = a.w;
      p2[0] = b2.x; p2[S] = b2.y; p2[2 * S] = b2.z; p2[3 * S] = b2.w;
    }
  }
}

// One wave64 per channel sums that channel's `splits` partials (contiguous) in fp64.
__device__ __forceinline__ void wave_sum2(const float *p1, const float *p2, int splits, double &s1, double &s2) {
  const int lane = threadIdx.x & 63;
  s1 = 0.0;
  s2 = 0.0;
  for (int i = lane; i < splits; i += 64) {
    s1 += p1[i];
    s2 += p2[i];
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    s1 += __shfl_xor(s1, o);
    s2 += __shfl_xor(s2, o);
  }
}

// Finalise forward statistics: mean, invstd, running-stat update.  Block = 256 = 4 channels.
template <typename TX>
__global__ void bn_stats_final_kernel(int64_t rows, int C, int splits, const TX *__restrict__ x,
                                      const float *__restrict__ partial, float *mean_out,
                                      float *invstd_out, float *running_mean, float *running_var,
                                      float momentum, float eps) {
  const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (c >= C) return;
  double s1, s2;
  wave_sum2(partial + (size_t)c * splits, partial + ((size_t)C + c) * splits, splits, s1, s2);
  if ((threadIdx.x & 63) != 0) return;
  double n = (double)rows;
  double dm = s1 / n;
  double var = s2 / n - dm * dm;
  if (var < 0) var = 0;
  double mean = (double)lda1(x + c) + dm;
  mean_out[c] = (float)mean;
  invstd_out[c] = (float)(1.0 / sqrt(var + (double)eps));
  if (running_mean) running_mean[c] = (float)((1.0 - momentum) * running_mean[c] + momentum * mean);
  if (running_var) {
    double unb = rows > 1 ? var * n / (n - 1.0) : var;
    running_var[c] = (float)((1.0 - momentum) * running_var[c] + momentum * unb);
  }
}

// Finalise forward statistics from row-tile (count, mean, M2) triples (conv epilogue):
// lanes merge their tiles sequentially, then a fixed shuffle tree — Chan et al.'s pairwise
// update in fp64, deterministic.
__device__ __forceinline__ void chan_merge(double &n, double &m, double &q, double nb, double mb, double qb) {
  const double nn = n + nb;
  if (nb == 0.0) return;
  if (n == 0.0) {
    n = nb; m = mb; q = qb;
    return;
  }
  const double d = mb - m;
  m += d * nb / nn;
  q += qb + d * d * n * nb / nn;
  n = nn;
}

__global__ void bn_tiles_final_kernel(int C, int ntiles, const float *__restrict__ stats, float *mean_out,
                                      float *invstd_out, float *running_mean, float *running_var,
                                      float momentum, float eps) {
  const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (c >= C) return;
  const float *cnt = stats, *mu = stats + ntiles + (size_t)c * ntiles;
  const float *m2 = stats + ntiles + ((size_t)C + c) * ntiles;
  double n = 0, m = 0, q = 0;
  for (int t = lane; t < ntiles; t += 64) chan_merge(n, m, q, cnt[t], mu[t], m2[t]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const double nb = __shfl_xor(n, o), mb = __shfl_xor(m, o), qb = __shfl_xor(q, o);
    if (lane & o) {  // the upper lane merges into a copy of the lower one's order: keep the
      double n2 = nb, m2v = mb, q2 = qb;  // same (lower, upper) operand order on both lanes
      chan_merge(n2, m2v, q2, n, m, q);
      n = n2; m = m2v; q = q2;
    } else {
      chan_merge(n, m, q, nb, mb, qb);
    }
  }
  if (lane != 0) return;
  const double var = n > 0 ? q / n : 0.0;
  mean_out[c] = (float)m;
  invstd_out[c] = (float)(1.0 / sqrt(var + (double)eps));
  if (running_mean) running_mean[c] = (float)((1.0 - momentum) * running_mean[c] + momentum * m);
  if (running_var) {
    const double unb = n > 1 ? q / (n - 1.0) : var;
    running_var[c] = (float)((1.0 - momentum) * running_var[c] + momentum * unb);
  }
}

// Finalise backward sums: store mean(g) and mean(g*xhat) per channel.
// With dweight / dbias (trainable affine BN, the warper's): dbias += sum(g),
// dweight += sum(g * xhat) — torch's AccumulateGrad.
__global__ void bn_bwd_final_kernel(int64_t rows, int C, int splits, const float *__restrict__ partial,
                                    const float *__restrict__ invstd, float *coef, float *dweight = nullptr,
                                    float *dbias = nullptr) {
  const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (c >= C) return;
  double s1, s2;
  wave_sum2(partial + (size_t)c * splits, partial + ((size_t)C + c) * splits, splits, s1, s2);
  if ((threadIdx.x & 63) != 0) return;
  double n = (double)rows;
  coef[c] = (float)(s1 / n);                          // mean(g)
  coef[C + c] = (float)(s2 / n * (double)invstd[c]);  // mean(g * xhat)
  if (dbias) dbias[c] += (float)s1;
  if (dweight) dweight[c] += (float)(s2 * (double)invstd[c]);
}

// four floats -> four bf16 (RNE) in 8 bytes: the bf16 operand copy a BN pass writes beside its
// fp32 output for the bf16-operand convs (conv math BF16) that consume it
__device__ __forceinline__ uint2 bf16x4_rne(float4 v) {
  typedef float f4v __attribute__((ext_vector_type(4)));
  typedef __bf16 b4v __attribute__((ext_vector_type(4)));
  const f4v f = {v.x, v.y, v.z, v.w};
  return __builtin_bit_cast(uint2, __builtin_convertvector(f, b4v));
}

// The operand copy of the four outputs (row, c .. c+3): one bf16 RNE image [rows][C] (BF16
// maths) or their three terms in the pixel-interleaved [rows][3][C] copy (terms, F32X3 maths)
__device__ __forceinline__ void store_copy(uint2 *yb, int64_t row, int c, int C, float4 o, bool terms) {
  if (terms) {
    uint2 h, m, l;
    split3(o, h, m, l);
    const int64_t k = x3_off(row, c, C) >> 2;
    yb[k] = h;
    yb[k + (C >> 2)] = m;
    yb[k + (C >> 1)] = l;
  } else {
    yb[(row * C + c) >> 2] = bf16x4_rne(o);
  }
}

template <typename TX, typename TR = TX>
__global__ void bn_infer_apply_kernel(int64_t total4, int C, const TX *__restrict__ x,
                                      const float *__restrict__ rm, const float *__restrict__ rv, float eps,
                                      const float *__restrict__ w, const float *__restrict__ b,
                                      typename Act<TR>::ptr __restrict__ res, float *__restrict__ y, uint2 *yb, int relu,
                                      bool terms = false, uint32_t *mbits = nullptr) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total4;
       i += (int64_t)gridDim.x * blockDim.x) {
    int c = (int)((i * 4) % C);
    const int64_t row = i * 4 / C;
    float4 v = lda4(x + 4 * i);
    float o[4] = {v.x, v.y, v.z, v.w};
    float r4[4] = {0, 0, 0, 0};
    if (res) {
      float4 r = ldr4<TR>(res, row, c, C);
      r4[0] = r.x; r4[1] = r.y; r4[2] = r.z; r4[3] = r.w;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float is = 1.0f / sqrtf(rv[c + j] + eps);
      float t = (o[j] - rm[c + j]) * is * (w ? w[c + j] : 1.f) + (b ? b[c + j] : 0.f) + r4[j];
      o[j] = fwd_act(t, relu);
    }
    if (y) reinterpret_cast<float4 *>(y)[i] = make_float4(o[0], o[1], o[2], o[3]);
    if (yb) store_copy(yb, row, c, C, make_float4(o[0], o[1], o[2], o[3]), terms);
    if (mbits) {   // (C % 32 == 0: the 8 quads of a word are 8 consecutive lanes of this loop)
      const float4 oq[1] = {make_float4(o[0], o[1], o[2], o[3])};
      store_mask_bits<1>(mbits, row, c, C, oq);
    }
  }
}

// Channel-major apply passes: a block is tc channel quads x (256/tc) row lanes, so a thread
// loads its channels' parameters once and walks rows (no per-element channel modulo); rows
// are unrolled x4 with all loads issued before any store (dx / dres / y may alias dy / x:
// every element is still read before it is written, by the same thread).
constexpr int kApplyUnroll = 4;

__device__ __forceinline__ float4 ld4c(const float *p) { return *reinterpret_cast<const float4 *>(p); }
__device__ __forceinline__ void st4(float *p, float4 v) { *reinterpret_cast<float4 *>(p) = v; }
// a gradient quad stored fp32, or bf16 (RNE) under bf16 gradient storage
__device__ __forceinline__ void stg4(float *p, float4 v) { st4(p, v); }
__device__ __forceinline__ void stg4(__bf16 *p, float4 v) { *reinterpret_cast<uint2 *>(p) = bf16x4_rne(v); }

template <int QN> __device__ __forceinline__ void stq(float *p, const float4 (&v)[QN]) {
#pragma unroll
  for (int h = 0; h < QN; ++h) st4(p + 4 * h, v[h]);
}
// the operand copy of a thread's 4*QN outputs of a row: one 16-B store of eight bf16 (QN 2) or
// store_copy per quad (bf16 image or F32X3 term images)
template <int QN>
__device__ __forceinline__ void store_copyq(uint2 *yb, int64_t row, int c, int C, const float4 (&o)[QN], bool terms) {
  if constexpr (QN == 2) {
    if (!terms) {
      const uint2 lo = bf16x4_rne(o[0]), hi = bf16x4_rne(o[1]);
      *reinterpret_cast<uint4 *>(yb + ((row * C + c) >> 2)) = make_uint4(lo.x, lo.y, hi.x, hi.y);
      return;
    }
  }
#pragma unroll
  for (int h = 0; h < QN; ++h) store_copy(yb, row, c + 4 * h, C, o[h], terms);
}

template <typename TX, int QN> constexpr int apply_rows() { return QN == 2 ? kBf16Rows : kApplyUnroll; }

template <typename TX, typename TR = TX, int QN = 1>
__global__ void __launch_bounds__(256, kBnMinBlocks)
bn_apply2d_kernel(int64_t rows, int C, int tc, int64_t per, const TX *x, const float *__restrict__ mean,
                  const float *__restrict__ invstd, const float *__restrict__ w, const float *__restrict__ b,
                  typename Act<TR>::ptr res, float *y, uint2 *yb, int act, bool terms = false,
                  uint32_t *mbits = nullptr) {
  const int tr = 256 / tc;
  const int cq = threadIdx.x % tc, rl = threadIdx.x / tc;
  const int c0 = (blockIdx.x * tc + cq) * 4 * QN;
  if (c0 >= C) return;
  const int64_t r0 = blockIdx.y * per, r1 = min(rows, r0 + per);
  float4 m[QN], is[QN], ww[QN], bb[QN];
  ldpq<QN>(mean, c0, m, 0.f);
  ldpq<QN>(invstd, c0, is, 0.f);
  ldpq<QN>(w, c0, ww, 1.f);
  ldpq<QN>(b, c0, bb, 0.f);
  constexpr int U = apply_rows<TX, QN>();
  for (int64_t r = r0 + rl; r < r1; r += U * tr) {
    float4 v[U][QN], q[U][QN];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t ru = r + (int64_t)u * tr;
      const bool ok = ru < r1;
      const int64_t row = ok ? ru : r, e = row * C + c0;
      ldq<QN>(x + e, v[u]);
      if (res) ldrq<TR, QN>(res, row, c0, C, q[u]);
      else zq<QN>(q[u]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t ru = r + (int64_t)u * tr;
      if (ru >= r1) break;
      float4 o[QN];
#pragma unroll
      for (int h = 0; h < QN; ++h) {
        o[h].x = fwd_act(bn_affine(v[u][h].x, m[h].x, is[h].x, ww[h].x, bb[h].x) + q[u][h].x, act);
        o[h].y = fwd_act(bn_affine(v[u][h].y, m[h].y, is[h].y, ww[h].y, bb[h].y) + q[u][h].y, act);
        o[h].z = fwd_act(bn_affine(v[u][h].z, m[h].z, is[h].z, ww[h].z, bb[h].z) + q[u][h].z, act);
        o[h].w = fwd_act(bn_affine(v[u][h].w, m[h].w, is[h].w, ww[h].w, bb[h].w) + q[u][h].w, act);
      }
      if (y) stq<QN>(y + ru * C + c0, o);
      if (yb) store_copyq<QN>(yb, ru, c0, C, o, terms);
      if (mbits) store_mask_bits<QN>(mbits, ru, c0, C, o);
    }
  }
}

template <typename TX, typename TY = TX, int QN = 1, typename TD = float>
__global__ void __launch_bounds__(256, kBnMinBlocks)
bn_bwd_apply2d_kernel(int64_t rows, int C, int tc, int64_t per, const TD *dy, typename Act<TY>::ptr y,
                      const TX *x, const float *__restrict__ w, const float *__restrict__ b,
                      const float *__restrict__ mean, const float *__restrict__ invstd, const float *__restrict__ coef,
                      float *dx, uint2 *dxb, TD *dres, int rmode, int train, bool terms = false,
                      const uint32_t *__restrict__ dbits = nullptr) {
  if constexpr (QN == 1) {   // (the grouped body below takes 130 VGPRs here: 3 waves per SIMD)
    const int tr = 256 / tc;
    const int cq = threadIdx.x % tc, rl = threadIdx.x / tc;
    const int c0 = (blockIdx.x * tc + cq) * 4;
    if (c0 >= C) return;
    const int64_t r0 = blockIdx.y * per, r1 = min(rows, r0 + per);
    const float4 z4 = make_float4(0, 0, 0, 0);
    const float4 is = ld4c(invstd + c0);
    const float4 ww = w ? ld4c(w + c0) : make_float4(1, 1, 1, 1);
    const float4 m = train ? ld4c(mean + c0) : z4;
    const float4 mg = train ? ld4c(coef + c0) : z4, mgx = train ? ld4c(coef + C + c0) : z4;
    const float4 bb = ((rmode == 2 || rmode == 4) && b) ? ld4c(b + c0) : z4;
    const bool need_y = rmode == 1 || rmode == 3;
    constexpr int U = apply_rows<TX, 1>();
    for (int64_t r = r0 + rl; r < r1; r += U * tr) {
      float4 g[U], v[U], o4[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t ru = r + (int64_t)u * tr;
        const int64_t row = ru < r1 ? ru : r, e = row * C + c0;
        g[u] = lda4(dy + e);
        v[u] = train ? lda4(x + e) : z4;
        o4[u] = need_y ? ldm4<TY>(y, row, c0, C) : z4;
        if (dbits) g[u] = mask_quad(g[u], load_mask_bits(dbits, row, c0, C));
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t ru = r + (int64_t)u * tr;
        if (ru >= r1) break;
        const int64_t e = ru * C + c0;
        float4 gg = g[u];
        if (rmode) {
          float4 o;
          if (need_y) {
            o = o4[u];
          } else {
            o.x = bn_affine(v[u].x, m.x, is.x, ww.x, bb.x);
            o.y = bn_affine(v[u].y, m.y, is.y, ww.y, bb.y);
            o.z = bn_affine(v[u].z, m.z, is.z, ww.z, bb.z);
            o.w = bn_affine(v[u].w, m.w, is.w, ww.w, bb.w);
          }
          const float k = rmode <= 2 ? 0.f : 0.2f;
          gg.x = o.x > 0.f ? gg.x : k * gg.x;
          gg.y = o.y > 0.f ? gg.y : k * gg.y;
          gg.z = o.z > 0.f ? gg.z : k * gg.z;
          gg.w = o.w > 0.f ? gg.w : k * gg.w;
        }
        if (dres) stg4(dres + e, gg);
        float4 out;
        if (train) {
          out.x = ww.x * is.x * (gg.x - mg.x - (v[u].x - m.x) * is.x * mgx.x);
          out.y = ww.y * is.y * (gg.y - mg.y - (v[u].y - m.y) * is.y * mgx.y);
          out.z = ww.z * is.z * (gg.z - mg.z - (v[u].z - m.z) * is.z * mgx.z);
          out.w = ww.w * is.w * (gg.w - mg.w - (v[u].w - m.w) * is.w * mgx.w);
        } else {
          out.x = gg.x * ww.x * is.x; out.y = gg.y * ww.y * is.y; out.z = gg.z * ww.z * is.z; out.w = gg.w * ww.w * is.w;
        }
        if (dx) st4(dx + e, out);
        if (dxb) store_copy(dxb, ru, c0, C, out, terms);
      }
    }
  } else {
    const int tr = 256 / tc;
    const int cq = threadIdx.x % tc, rl = threadIdx.x / tc;
    const int c0 = (blockIdx.x * tc + cq) * 4 * QN;
    if (c0 >= C) return;
    const int64_t r0 = blockIdx.y * per, r1 = min(rows, r0 + per);
    float4 is[QN], ww[QN], m[QN], mg[QN], mgx[QN], bb[QN];
    ldpq<QN>(invstd, c0, is, 0.f);
    ldpq<QN>(w, c0, ww, 1.f);
    ldpq<QN>(train ? mean : nullptr, c0, m, 0.f);
    ldpq<QN>(train ? coef : nullptr, c0, mg, 0.f);
    ldpq<QN>(train ? coef + C : nullptr, c0, mgx, 0.f);
    ldpq<QN>((rmode == 2 || rmode == 4) ? b : nullptr, c0, bb, 0.f);
    const bool need_y = rmode == 1 || rmode == 3;
    constexpr int U = apply_rows<TX, QN>();
    for (int64_t r = r0 + rl; r < r1; r += U * tr) {
      float4 g[U][QN], v[U][QN], o4[U][QN];
  #pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t ru = r + (int64_t)u * tr;
        const int64_t row = ru < r1 ? ru : r, e = row * C + c0;
        ldq<QN>(dy + e, g[u]);
        if (dbits) {
          const uint32_t mw = load_mask_bits(dbits, row, c0, C);
#pragma unroll
          for (int h = 0; h < QN; ++h) g[u][h] = mask_quad(g[u][h], mw >> (4 * h));
        }
        if (train) ldq<QN>(x + e, v[u]);
        else zq<QN>(v[u]);
        if (need_y) ldmq<TY, QN>(y, row, c0, C, o4[u]);
        else zq<QN>(o4[u]);
      }
  #pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t ru = r + (int64_t)u * tr;
        if (ru >= r1) break;
        const int64_t e = ru * C + c0;
        float4 out[QN];
  #pragma unroll
        for (int h = 0; h < QN; ++h) {
          float4 gg = g[u][h];
          const float4 vv = v[u][h];
          if (rmode) {
            float4 o;
            if (need_y) {
              o = o4[u][h];
            } else {
              o.x = bn_affine(vv.x, m[h].x, is[h].x, ww[h].x, bb[h].x);
              o.y = bn_affine(vv.y, m[h].y, is[h].y, ww[h].y, bb[h].y);
              o.z = bn_affine(vv.z, m[h].z, is[h].z, ww[h].z, bb[h].z);
              o.w = bn_affine(vv.w, m[h].w, is[h].w, ww[h].w, bb[h].w);
            }
            const float k = rmode <= 2 ? 0.f : 0.2f;
            gg.x = o.x > 0.f ? gg.x : k * gg.x;
            gg.y = o.y > 0.f ? gg.y : k * gg.y;
            gg.z = o.z > 0.f ? gg.z : k * gg.z;
            gg.w = o.w > 0.f ? gg.w : k * gg.w;
          }
          if (dres) stg4(dres + e + 4 * h, gg);
          const float4 W = ww[h], I = is[h], M = m[h], G = mg[h], X = mgx[h];
          if (train) {
            out[h].x = W.x * I.x * (gg.x - G.x - (vv.x - M.x) * I.x * X.x);
            out[h].y = W.y * I.y * (gg.y - G.y - (vv.y - M.y) * I.y * X.y);
            out[h].z = W.z * I.z * (gg.z - G.z - (vv.z - M.z) * I.z * X.z);
            out[h].w = W.w * I.w * (gg.w - G.w - (vv.w - M.w) * I.w * X.w);
          } else {
            out[h].x = gg.x * W.x * I.x; out[h].y = gg.y * W.y * I.y; out[h].z = gg.z * W.z * I.z; out[h].w = gg.w * W.w * I.w;
          }
          if (dx) st4(dx + e + 4 * h, out[h]);
        }
        if (dxb) store_copyq<QN>(dxb, ru, c0, C, out, terms);
      }
    }
  }
}

struct ApplyPlan {
  int tc, cblocks, rsplits;
  int64_t per;
};

static ApplyPlan apply_plan(int64_t rows, int C, int qn = 1, int blocks = kApplyBlocks) {
  ApplyPlan a;
  const int groups = C / (4 * qn);   // channel groups of qn quads
  a.tc = std::min(groups, 64);
  if (a.tc < 1) a.tc = 1;
  while (256 % a.tc) --a.tc;
  a.cblocks = (int)ceil_div(groups, a.tc);
  const int tr = 256 / a.tc;
  // ~2 blocks per CU: the apply passes run beside the weight-gradient GEMMs; 512 blocks measured
  // +0.8 % at c2 over 2048 (c3 equal), 256 -0.6 % (two runs each)
  const int want = std::max(1, blocks / a.cblocks);
  const int64_t maxs = std::max<int64_t>(1, ceil_div(rows, (int64_t)tr * (qn == 2 ? kBf16Rows : kApplyUnroll)));
  a.rsplits = (int)std::min<int64_t>(want, maxs);
  a.per = ceil_div(rows, a.rsplits);
  a.rsplits = (int)ceil_div(rows, a.per);
  return a;
}

struct ReducePlan {
  int tc, cblocks, splits;
  int64_t per;
};

static ReducePlan reduce_plan(int64_t rows, int C, int qn = 1) {
  ReducePlan r;
  const int groups = C / (4 * qn);
  r.tc = std::min(groups, 64);
  if (r.tc < 1) r.tc = 1;
  // tc must divide 256
  while (256 % r.tc) --r.tc;
  r.cblocks = (int)ceil_div(groups, r.tc);
  // 512 blocks: 256 / 1024 measured -2 % / -4.5 % at c2 — the reduction shares the chip with
  // the weight-gradient GEMMs, more blocks take CUs from them
  int want = std::max(1, kReduceBlocks / r.cblocks);
  int tr = 256 / r.tc;
  int64_t max_splits = std::max<int64_t>(1, ceil_div(rows, (int64_t)tr * 8));
  r.splits = (int)std::min<int64_t>(want, max_splits);
  r.per = ceil_div(rows, r.splits);
  r.splits = (int)ceil_div(rows, r.per);
  return r;
}

// bf16 storage with 8-channel groups: C % 8 and 16-B aligned operands (else one quad a thread)
static int bf16_qn(int C, std::initializer_list<const void *> ptrs) {
  if (C % 8) return 1;
  for (const void *p : ptrs)
    if (reinterpret_cast<uintptr_t>(p) % 16) return 1;
  return 2;
}

// The reductions take 8-channel groups only on wide tensors: at C = 256 the halved block
// count cost more than the wider loads gained (l3.bn2 backward sums 13.2 -> 15.9 us, l3.bn3
// 62.9 -> 58.9 us; statistics 34.2 -> 25.1 us at C = 1024, tools/bn_bench.py --bf16)
static int reduce_qn(int qn, int C) { return qn == 2 && C >= 512 ? 2 : 1; }

static size_t bn_ws_bytes(int64_t rows, int C) {
  // partial [2][C][splits] + coef [2][C], for either channel grouping
  const int splits = std::max(reduce_plan(rows, C, 1).splits, C % 8 ? 0 : reduce_plan(rows, C, 2).splits);
  return ((size_t)splits * 2 * C + 2 * (size_t)C) * sizeof(float);
}

static int grid_for(int64_t total4) { return (int)std::min<int64_t>(ceil_div(total4, 256), 8192); }

}  // namespace adaptseg

namespace adaptseg {

template <typename TX, typename TY, int QN, typename TD>
static void bn_bwd_kernels(int64_t rows, int c, const TD *dy, typename Act<TY>::ptr y, const TX *x,
                           const float *weight, const float *bias, const float *save_mean, const float *save_invstd,
                           float *dx, uint16_t *dx_bf16, TD *dres, int rmode, int train, float *dweight,
                           float *dbias, float *partial, float *coef, double reduce_bytes, double apply_bytes,
                           bool dterms, const uint32_t *dbits, hipStream_t s, const float *sums, int sum_tiles) {
  int slot;
  if (train && sums) {   // the reduction fused into the producing data gradient's epilogue
    bn_bwd_final_kernel<<<(unsigned)ceil_div(c, 4), 256, 0, s>>>(rows, c, sum_tiles, sums, save_invstd, coef, dweight,
                                                                   dbias);
  } else if (train) {
    const int rqn = reduce_qn(QN, c);
    const ReducePlan r = reduce_plan(rows, c, rqn);
    timing_begin(kTBnReduceBwd, s, reduce_bytes, &slot);
    if (rqn == 2)
      bn_reduce_kernel<1, TX, TY, QN, TD><<<dim3(r.cblocks, r.splits), 256, 0, s>>>(
          rows, c, r.tc, x, dy, y, save_mean, save_invstd, weight, bias, rmode, r.per, partial, dbits);
    else
      bn_reduce_kernel<1, TX, TY, 1, TD><<<dim3(r.cblocks, r.splits), 256, 0, s>>>(
          rows, c, r.tc, x, dy, y, save_mean, save_invstd, weight, bias, rmode, r.per, partial, dbits);
    timing_end(slot, s);
    bn_bwd_final_kernel<<<(unsigned)ceil_div(c, 4), 256, 0, s>>>(rows, c, r.splits, partial, save_invstd, coef,
                                                                   dweight, dbias);
  }
  timing_begin(kTBnBwdApply, s, apply_bytes, &slot);
  const ApplyPlan ap = apply_plan(rows, c, QN);
  bn_bwd_apply2d_kernel<TX, TY, QN, TD><<<dim3(ap.cblocks, ap.rsplits), 256, 0, s>>>(
      rows, c, ap.tc, ap.per, dy, y, x, weight, bias, save_mean, save_invstd, coef, dx,
      reinterpret_cast<uint2 *>(dx_bf16), dres, rmode, train, dterms, dbits);
  timing_end(slot, s);
}

template <typename TX, typename TY = TX, typename TD = float>
int bn_bwd_launch(int64_t rows, int c, const TD *dy, typename Act<TY>::ptr y, const TX *x, const float *weight,
                         const float *bias, const float *save_mean, const float *save_invstd, float *dx,
                         uint16_t *dx_bf16, TD *dres, int rmode, int train, float *dweight, float *dbias, void *ws,
                         size_t ws_bytes, hipStream_t s, const uint32_t *dbits = nullptr, const float *sums = nullptr,
                         int sum_tiles = 0) {
  float *partial = reinterpret_cast<float *>(ws), *coef = nullptr;
  const double eb = sizeof(TX);   // bytes per activation element (x)
  const bool terms = std::is_same<TY, X3>::value;   // y stored as F32X3 term images
  const double ebt = terms ? 2.0 : eb;               // ... bytes per element of y (terms: the hi term, ldm4)
  const bool dterms = copies_are_terms() && dx_bf16;
  const int qn = (sizeof(TX) == 2 && !terms && !dterms) ? bf16_qn(c, {dy, y, x, dx, dx_bf16, dres}) : 1;
  if (train) {
    size_t need = bn_ws_bytes(rows, c);
    if (!ws || ws_bytes < need) {
      set_error("bn_bwd: workspace %zu < %zu", ws_bytes, need);
      return ADAPTSEG_ERR_WORKSPACE;
    }
    coef = partial + (size_t)reduce_plan(rows, c, reduce_qn(qn, c)).splits * 2 * c;
  }
  // reduce: dy, x (+ y for the mask from y) in; apply: dy, x (train), y (mask from y) in; dx,
  // dres out
  const double db = sizeof(TD);    // bytes per gradient element (dy, dres)
  const double mb = dbits ? 0.125 : 0.0;   // bytes per element of a mask bitmap
  const double reduce_bytes = sums ? 0.0 : (db + eb + mb + ((rmode == 1 || rmode == 3) ? ebt : 0.0)) * rows * c;
  const double apply_bytes = (db * (1 + (dres ? 1 : 0)) + 4.0 * (dx ? 1 : 0) + eb * (train ? 1 : 0) + mb +
                              ((rmode == 1 || rmode == 3) ? ebt : 0.0)) * rows * c +
                             (dx_bf16 ? (dterms ? 6.0 : 2.0) * rows * c : 0.0);
  if constexpr (sizeof(TX) == 2 && !std::is_same<TY, X3>::value) {
    if (qn == 2) {
      bn_bwd_kernels<TX, TY, 2, TD>(rows, c, dy, y, x, weight, bias, save_mean, save_invstd, dx, dx_bf16, dres, rmode,
                                    train, dweight, dbias, partial, coef, reduce_bytes, apply_bytes, dterms, dbits,
                                    s, sums, sum_tiles);
      AS_CHECK_LAUNCH("bn_bwd");
      return ADAPTSEG_OK;
    }
  }
  bn_bwd_kernels<TX, TY, 1, TD>(rows, c, dy, y, x, weight, bias, save_mean, save_invstd, dx, dx_bf16, dres, rmode,
                                train, dweight, dbias, partial, coef, reduce_bytes, apply_bytes, dterms, dbits, s,
                                sums, sum_tiles);
  AS_CHECK_LAUNCH("bn_bwd");
  return ADAPTSEG_OK;
}

}  // namespace adaptseg

using namespace adaptseg;

extern "C" {

int adaptseg_bn_workspace_size(int64_t rows, int c, size_t *bytes) {
  AS_CHECK_ARG(bytes && rows > 0 && c > 0, "bn_workspace_size: bad args");
  *bytes = bn_ws_bytes(rows, c);
  return ADAPTSEG_OK;
}

// Shared checks and apply launch of the forward entry points.  Storage: x fp32 or bf16 (bf16
// activation storage, BF16 maths); the residual stored like x — or, under the F32X3 maths, as
// the three term images of an fp32 residual (res_bf16) beside an fp32 x.  Outputs y (fp32) and
// / or its operand copy y_bf16 (bf16 RNE image, or the three term images under F32X3).
static int check_fwd_storage(const char *who, const float *x, const uint16_t *x_bf16, const float *res,
                             const uint16_t *res_bf16, const float *y, const uint16_t *y_bf16) {
  AS_CHECK_ARG((x != nullptr) != (x_bf16 != nullptr) && (y || y_bf16), "%s: exactly one of x / x_bf16, and y or y_bf16",
               who);
  AS_CHECK_ARG(!(res && res_bf16), "%s: one residual pointer", who);
  if (copies_are_terms())
    AS_CHECK_ARG(x, "%s: under the F32X3 conv maths x is fp32 (its copies are term images of fp32 tensors)", who);
  else
    AS_CHECK_ARG(x ? !res_bf16 : !res, "%s: the residual must be stored like x (fp32 or bf16)", who);
  return ADAPTSEG_OK;
}

static double fwd_apply_bytes(int64_t rows, int c, const float *x, const float *res, const uint16_t *res_bf16,
                              const float *y, const uint16_t *y_bf16) {
  const bool terms = copies_are_terms();
  const double copyb = terms ? 6.0 : 2.0;
  return ((x ? 4.0 : 2.0) + (res ? 4.0 : res_bf16 ? copyb : 0.0) + (y ? 4.0 : 0.0) + (y_bf16 ? copyb : 0.0)) *
         (double)rows * c;
}

static void launch_apply(int64_t rows, int c, const float *x, const uint16_t *x_bf16, const float *mean,
                         const float *invstd, const float *weight, const float *bias, const float *res,
                         const uint16_t *res_bf16, float *y, uint16_t *y_bf16, int relu, hipStream_t s,
                         uint32_t *mbits = nullptr) {
  const bool terms = copies_are_terms() && y_bf16;
  uint2 *yb = reinterpret_cast<uint2 *>(y_bf16);
  const __bf16 *rb = reinterpret_cast<const __bf16 *>(res_bf16);
  const int qn = (!x && !terms) ? bf16_qn(c, {x_bf16, res_bf16, y, y_bf16}) : 1;
  const ApplyPlan ap = apply_plan(rows, c, qn, kApplyBlocksFwd);
  const dim3 g(ap.cblocks, ap.rsplits);
  if (x && rb)
    bn_apply2d_kernel<float, X3><<<g, 256, 0, s>>>(rows, c, ap.tc, ap.per, x, mean, invstd, weight, bias, rb, y, yb,
                                                   relu, terms, mbits);
  else if (x)
    bn_apply2d_kernel<float, float><<<g, 256, 0, s>>>(rows, c, ap.tc, ap.per, x, mean, invstd, weight, bias, res, y,
                                                      yb, relu, terms, mbits);
  else if (qn == 2)
    bn_apply2d_kernel<__bf16, __bf16, 2><<<g, 256, 0, s>>>(rows, c, ap.tc, ap.per,
                                                           reinterpret_cast<const __bf16 *>(x_bf16), mean, invstd,
                                                           weight, bias, rb, y, yb, relu, terms, mbits);
  else
    bn_apply2d_kernel<__bf16, __bf16><<<g, 256, 0, s>>>(rows, c, ap.tc, ap.per,
                                                        reinterpret_cast<const __bf16 *>(x_bf16), mean, invstd,
                                                        weight, bias, rb, y, yb, relu, terms, mbits);
}

static constexpr const float *kNoDy = nullptr;   // the statistics pass reads no gradient

static int bn_fwd_train_impl(int64_t rows, int c, const float *x, const uint16_t *x_bf16, const float *weight,
                             const float *bias, float *running_mean, float *running_var, float momentum, float eps,
                             float *save_mean, float *save_invstd, const float *res, const uint16_t *res_bf16,
                             float *y, uint16_t *y_bf16, uint32_t *relu_bits, int relu, void *ws, size_t ws_bytes,
                             adaptseg_stream_t stream) {
  AS_CHECK_ARG(!relu_bits || c % 32 == 0, "bn_fwd_train: a mask bitmap needs C %% 32 == 0 (C=%d)", c);
  AS_CHECK_ARG(rows > 0 && c > 0 && c % 4 == 0, "bn_fwd_train: rows>0, C%%4==0 required (C=%d)", c);
  AS_CHECK_ARG(rows > 1, "bn_fwd_train: expected more than 1 value per channel when training");
  AS_CHECK_ARG(relu >= 0 && relu <= 2, "bn_fwd_train: activation %d (0 none, 1 ReLU, 2 LeakyReLU)", relu);
  AS_CHECK_ARG(save_mean && save_invstd, "bn_fwd_train: null statistics output");
  int st = check_fwd_storage("bn_fwd_train", x, x_bf16, res, res_bf16, y, y_bf16);
  if (st) return st;
  size_t need = bn_ws_bytes(rows, c);
  if (!ws || ws_bytes < need) {
    set_error("bn_fwd_train: workspace %zu < %zu", ws_bytes, need);
    return ADAPTSEG_ERR_WORKSPACE;
  }
  hipStream_t s = as_stream(stream);
  ReducePlan r = reduce_plan(rows, c), r2 = {0, 0, 0, 0};
  if (!x && reduce_qn(bf16_qn(c, {x_bf16}), c) == 2) r2 = reduce_plan(rows, c, 2);   // bf16 x: 8-channel groups
  float *partial = reinterpret_cast<float *>(ws);
  const double eb = x ? 4.0 : 2.0;   // bytes per activation element read
  int slot;  // x in
  timing_begin(kTBnReduceStats, s, eb * rows * c, &slot);
  const __bf16 *xb = reinterpret_cast<const __bf16 *>(x_bf16);
  if (x)
    bn_reduce_kernel<0, float><<<dim3(r.cblocks, r.splits), 256, 0, s>>>(rows, c, r.tc, x, kNoDy, nullptr, nullptr,
                                                                       nullptr, nullptr, nullptr, 0, r.per, partial);
  else if (r2.splits)
    bn_reduce_kernel<0, __bf16, __bf16, 2><<<dim3(r2.cblocks, r2.splits), 256, 0, s>>>(
        rows, c, r2.tc, xb, kNoDy, nullptr, nullptr, nullptr, nullptr, nullptr, 0, r2.per, partial);
  else
    bn_reduce_kernel<0, __bf16><<<dim3(r.cblocks, r.splits), 256, 0, s>>>(rows, c, r.tc, xb, kNoDy, nullptr, nullptr,
                                                                        nullptr, nullptr, nullptr, 0, r.per, partial);
  timing_end(slot, s);
  AS_CHECK_LAUNCH("bn_reduce<stats>");
  if (x)
    bn_stats_final_kernel<<<(unsigned)ceil_div(c, 4), 256, 0, s>>>(rows, c, r.splits, x, partial, save_mean, save_invstd,
                                                                   running_mean, running_var, momentum, eps);
  else
    bn_stats_final_kernel<<<(unsigned)ceil_div(c, 4), 256, 0, s>>>(rows, c, r2.splits ? r2.splits : r.splits, xb, partial, save_mean,
                                                                   save_invstd, running_mean, running_var, momentum, eps);
  AS_CHECK_LAUNCH("bn_stats_final");
  timing_begin(kTBnApply, s, fwd_apply_bytes(rows, c, x, res, res_bf16, y, y_bf16), &slot);
  launch_apply(rows, c, x, x_bf16, save_mean, save_invstd, weight, bias, res, res_bf16, y, y_bf16, relu, s,
               relu_bits);
  timing_end(slot, s);
  AS_CHECK_LAUNCH("bn_apply");
  return ADAPTSEG_OK;
}

int adaptseg_bn_fwd_train_x(int64_t rows, int c, const float *x, const uint16_t *x_bf16, const float *weight,
                            const float *bias, float *running_mean, float *running_var, float momentum, float eps,
                            float *save_mean, float *save_invstd, const float *res, const uint16_t *res_bf16,
                            float *y, uint16_t *y_bf16, int relu, void *ws, size_t ws_bytes,
                            adaptseg_stream_t stream) {
  return bn_fwd_train_impl(rows, c, x, x_bf16, weight, bias, running_mean, running_var, momentum, eps, save_mean,
                           save_invstd, res, res_bf16, y, y_bf16, nullptr, relu, ws, ws_bytes, stream);
}

int adaptseg_bn_fwd_train_xm(int64_t rows, int c, const float *x, const uint16_t *x_bf16, const float *weight,
                             const float *bias, float *running_mean, float *running_var, float momentum, float eps,
                             float *save_mean, float *save_invstd, const float *res, const uint16_t *res_bf16,
                             float *y, uint16_t *y_bf16, uint32_t *relu_bits, int relu, void *ws, size_t ws_bytes,
                             adaptseg_stream_t stream) {
  return bn_fwd_train_impl(rows, c, x, x_bf16, weight, bias, running_mean, running_var, momentum, eps, save_mean,
                           save_invstd, res, res_bf16, y, y_bf16, relu_bits, relu, ws, ws_bytes, stream);
}

int adaptseg_bn_fwd_train(int64_t rows, int c, const float *x, const float *weight, const float *bias,
                          float *running_mean, float *running_var, float momentum, float eps,
                          float *save_mean, float *save_invstd, const float *res, float *y, int relu,
                          void *ws, size_t ws_bytes, adaptseg_stream_t stream) {
  return adaptseg_bn_fwd_train_x(rows, c, x, nullptr, weight, bias, running_mean, running_var, momentum, eps,
                                 save_mean, save_invstd, res, nullptr, y, nullptr, relu, ws, ws_bytes, stream);
}

int adaptseg_bn_fwd_train_tiles_xm(int64_t rows, int c, const float *stats, int ntiles, const float *x,
                                   const uint16_t *x_bf16, const float *weight, const float *bias,
                                   float *running_mean, float *running_var, float momentum, float eps,
                                   float *save_mean, float *save_invstd, const float *res, const uint16_t *res_bf16,
                                   float *y, uint16_t *y_bf16, uint32_t *relu_bits, int relu, adaptseg_stream_t stream) {
  AS_CHECK_ARG(!relu_bits || c % 32 == 0, "bn_fwd_train_tiles: a mask bitmap needs C %% 32 == 0 (C=%d)", c);
  AS_CHECK_ARG(rows > 1 && c > 0 && c % 4 == 0, "bn_fwd_train_tiles: rows>1, C%%4==0 required (C=%d)", c);
  AS_CHECK_ARG(stats && ntiles > 0 && save_mean && save_invstd, "bn_fwd_train_tiles: null pointer");
  AS_CHECK_ARG(relu >= 0 && relu <= 2, "bn_fwd_train_tiles: activation %d", relu);
  int st = check_fwd_storage("bn_fwd_train_tiles", x, x_bf16, res, res_bf16, y, y_bf16);
  if (st) return st;
  hipStream_t s = as_stream(stream);
  bn_tiles_final_kernel<<<(unsigned)ceil_div(c, 4), 256, 0, s>>>(c, ntiles, stats, save_mean, save_invstd,
                                                                   running_mean, running_var, momentum, eps);
  AS_CHECK_LAUNCH("bn_tiles_final");
  int slot;  // x (+res) in, y out
  timing_begin(kTBnApply, s, fwd_apply_bytes(rows, c, x, res, res_bf16, y, y_bf16), &slot);
  launch_apply(rows, c, x, x_bf16, save_mean, save_invstd, weight, bias, res, res_bf16, y, y_bf16, relu, s,
               relu_bits);
  timing_end(slot, s);
  AS_CHECK_LAUNCH("bn_apply");
  return ADAPTSEG_OK;
}

int adaptseg_bn_fwd_train_tiles_stats(int64_t rows, int c, const float *stats, int ntiles, float *running_mean,
                                      float *running_var, float momentum, float eps, float *save_mean,
                                      float *save_invstd, adaptseg_stream_t stream) {
  AS_CHECK_ARG(rows > 1 && c > 0 && c % 4 == 0, "bn_fwd_train_tiles_stats: rows>1, C%%4==0 required (C=%d)", c);
  AS_CHECK_ARG(stats && ntiles > 0 && save_mean && save_invstd, "bn_fwd_train_tiles_stats: null pointer");
  hipStream_t s = as_stream(stream);
  bn_tiles_final_kernel<<<(unsigned)ceil_div(c, 4), 256, 0, s>>>(c, ntiles, stats, save_mean, save_invstd,
                                                                   running_mean, running_var, momentum, eps);
  AS_CHECK_LAUNCH("bn_tiles_final");
  return ADAPTSEG_OK;
}

int adaptseg_bn_fwd_train_tiles_x(int64_t rows, int c, const float *stats, int ntiles, const float *x,
                                  const uint16_t *x_bf16, const float *weight, const float *bias,
                                  float *running_mean, float *running_var, float momentum, float eps,
                                  float *save_mean, float *save_invstd, const float *res, const uint16_t *res_bf16,
                                  float *y, uint16_t *y_bf16, int relu, adaptseg_stream_t stream) {
  return adaptseg_bn_fwd_train_tiles_xm(rows, c, stats, ntiles, x, x_bf16, weight, bias, running_mean, running_var,
                                        momentum, eps, save_mean, save_invstd, res, res_bf16, y, y_bf16, nullptr, relu,
                                        stream);
}

int adaptseg_bn_fwd_train_tiles(int64_t rows, int c, const float *stats, int ntiles, const float *x,
                                const float *weight, const float *bias, float *running_mean, float *running_var,
                                float momentum, float eps, float *save_mean, float *save_invstd, const float *res,
                                float *y, int relu, adaptseg_stream_t stream) {
  return adaptseg_bn_fwd_train_tiles_x(rows, c, stats, ntiles, x, nullptr, weight, bias, running_mean, running_var,
                                       momentum, eps, save_mean, save_invstd, res, nullptr, y, nullptr, relu, stream);
}

int adaptseg_bn_fwd_infer_xm(int64_t rows, int c, const float *x, const uint16_t *x_bf16, const float *weight,
                             const float *bias, const float *running_mean, const float *running_var, float eps,
                             const float *res, const uint16_t *res_bf16, float *y, uint16_t *y_bf16,
                             uint32_t *relu_bits, int relu, adaptseg_stream_t stream) {
  AS_CHECK_ARG(!relu_bits || c % 32 == 0, "bn_fwd_infer: a mask bitmap needs C %% 32 == 0 (C=%d)", c);
  AS_CHECK_ARG(rows > 0 && c > 0 && c % 4 == 0, "bn_fwd_infer: C%%4==0 required");
  AS_CHECK_ARG(running_mean && running_var, "bn_fwd_infer: null running statistics");
  AS_CHECK_ARG(relu >= 0 && relu <= 2, "bn_fwd_infer: activation %d", relu);
  int st = check_fwd_storage("bn_fwd_infer", x, x_bf16, res, res_bf16, y, y_bf16);
  if (st) return st;
  hipStream_t s = as_stream(stream);
  const int64_t total4 = rows * c / 4;
  const bool terms = copies_are_terms() && y_bf16;
  uint2 *yb = reinterpret_cast<uint2 *>(y_bf16);
  const __bf16 *rb = reinterpret_cast<const __bf16 *>(res_bf16);
  if (x && rb)
    bn_infer_apply_kernel<float, X3><<<grid_for(total4), 256, 0, s>>>(total4, c, x, running_mean, running_var, eps,
                                                                      weight, bias, rb, y, yb, relu, terms, relu_bits);
  else if (x)
    bn_infer_apply_kernel<float, float><<<grid_for(total4), 256, 0, s>>>(total4, c, x, running_mean, running_var, eps,
                                                                         weight, bias, res, y, yb, relu, terms, relu_bits);
  else
    bn_infer_apply_kernel<__bf16, __bf16><<<grid_for(total4), 256, 0, s>>>(
        total4, c, reinterpret_cast<const __bf16 *>(x_bf16), running_mean, running_var, eps, weight, bias, rb, y, yb,
        relu, terms, relu_bits);
  AS_CHECK_LAUNCH("bn_infer_apply");
  return ADAPTSEG_OK;
}

int adaptseg_bn_fwd_infer_x(int64_t rows, int c, const float *x, const uint16_t *x_bf16, const float *weight,
                            const float *bias, const float *running_mean, const float *running_var, float eps,
                            const float *res, const uint16_t *res_bf16, float *y, uint16_t *y_bf16, int relu,
                            adaptseg_stream_t stream) {
  return adaptseg_bn_fwd_infer_xm(rows, c, x, x_bf16, weight, bias, running_mean, running_var, eps, res, res_bf16, y,
                                  y_bf16, nullptr, relu, stream);
}

int adaptseg_bn_fwd_infer(int64_t rows, int c, const float *x, const float *weight, const float *bias,
                          const float *running_mean, const float *running_var, float eps, const float *res,
                          float *y, int relu, adaptseg_stream_t stream) {
  return adaptseg_bn_fwd_infer_x(rows, c, x, nullptr, weight, bias, running_mean, running_var, eps, res, nullptr, y,
                                 nullptr, relu, stream);
}

static int bn_bwd_impl(int64_t rows, int c, const float *dy, const uint16_t *dy_bf16, const float *y,
                       const uint16_t *y_bf16, const float *x, const uint16_t *x_bf16, const float *weight,
                       const float *bias, const float *save_mean, const float *save_invstd, float *dx, uint16_t *dx_bf16,
                       float *dres, uint16_t *dres_bf16, int relu, int train, float *dweight, float *dbias, void *ws,
                       size_t ws_bytes, adaptseg_stream_t stream, const uint32_t *dy_bits = nullptr,
                       const float *sums = nullptr, int sum_tiles = 0) {
  AS_CHECK_ARG(rows > 0 && c > 0 && c % 4 == 0, "bn_bwd: C%%4==0 required");
  const bool xb = x_bf16 != nullptr, terms = copies_are_terms();
  AS_CHECK_ARG((dy != nullptr) != (dy_bf16 != nullptr), "bn_bwd: exactly one of dy / dy_bf16");
  AS_CHECK_ARG((dx || dx_bf16) && save_invstd && (!train || ((x || x_bf16) && save_mean)), "bn_bwd: null pointer");
  AS_CHECK_ARG(!(x && x_bf16) && !(y && y_bf16), "bn_bwd: one pointer each for the saved x and y");
  // bf16 gradient storage: dres is stored like dy; only with bf16 activation storage
  AS_CHECK_ARG(dy ? !dres_bf16 : !dres, "bn_bwd: dres is stored like dy (fp32 or bf16)");
  AS_CHECK_ARG(!dy_bf16 || (!terms && (xb || (!x && y_bf16))),
               "bn_bwd: a bf16 dy needs bf16 activation storage (BF16 conv maths)");
  if (terms)   // F32X3 maths: x fp32, y fp32 or its three term images
    AS_CHECK_ARG(!xb, "bn_bwd: under the F32X3 conv maths x is fp32 (y may be term images)");
  else
    AS_CHECK_ARG(xb ? !y : !y_bf16, "bn_bwd: the saved x and y are both fp32 or both bf16 (one pointer each)");
  AS_CHECK_ARG(relu >= 0 && relu <= 2, "bn_bwd: activation %d (0 none, 1 ReLU, 2 LeakyReLU)", relu);
  AS_CHECK_ARG(!relu || y || y_bf16 || train, "bn_bwd: activation without y needs train mode (mask from x)");
  AS_CHECK_ARG(train || (!dweight && !dbias), "bn_bwd: affine gradients need train mode");
  AS_CHECK_ARG(!dy_bits || c % 32 == 0, "bn_bwd: a mask bitmap needs C %% 32 == 0 (C=%d)", c);
  // mask mode: ReLU 1 (from the saved output y) / 2 (recomputed from x, y == NULL);
  // LeakyReLU 3 (from y) / 4 (from x)
  const bool has_y = y || y_bf16;
  const int rmode = relu == 0 ? 0 : relu == 1 ? (has_y ? 1 : 2) : (has_y ? 3 : 4);
  hipStream_t s = as_stream(stream);
  if (terms && y_bf16)
    return bn_bwd_launch<float, X3>(rows, c, dy, reinterpret_cast<const __bf16 *>(y_bf16), x, weight, bias,
                                    save_mean, save_invstd, dx, dx_bf16, dres, rmode, train, dweight, dbias, ws,
                                    ws_bytes, s, dy_bits, sums, sum_tiles);
  if (xb || (!x && y_bf16)) {
    const __bf16 *yb = reinterpret_cast<const __bf16 *>(y_bf16), *xbb = reinterpret_cast<const __bf16 *>(x_bf16);
    if (dy_bf16)
      return bn_bwd_launch<__bf16, __bf16, __bf16>(rows, c, reinterpret_cast<const __bf16 *>(dy_bf16), yb, xbb, weight,
                                                   bias, save_mean, save_invstd, dx, dx_bf16,
                                                   reinterpret_cast<__bf16 *>(dres_bf16), rmode, train, dweight, dbias,
                                                   ws, ws_bytes, s, dy_bits, sums, sum_tiles);
    return bn_bwd_launch<__bf16>(rows, c, dy, yb, xbb, weight, bias, save_mean, save_invstd, dx, dx_bf16, dres, rmode,
                                 train, dweight, dbias, ws, ws_bytes, s, dy_bits, sums, sum_tiles);
  }
  return bn_bwd_launch<float>(rows, c, dy, y, x, weight, bias, save_mean, save_invstd, dx, dx_bf16, dres, rmode, train,
                              dweight, dbias, ws, ws_bytes, s, dy_bits, sums, sum_tiles);
}

int adaptseg_bn_bwd(int64_t rows, int c, const float *dy, const float *y, const float *x, const float *weight,
                    const float *bias, const float *save_mean, const float *save_invstd, float *dx, float *dres,
                    int relu, int train, void *ws, size_t ws_bytes, adaptseg_stream_t stream) {
  return bn_bwd_impl(rows, c, dy, nullptr, y, nullptr, x, nullptr, weight, bias, save_mean, save_invstd, dx, nullptr,
                     dres, nullptr, relu, train, nullptr, nullptr, ws, ws_bytes, stream);
}

int adaptseg_bn_bwd_x(int64_t rows, int c, const float *dy, const float *y, const uint16_t *y_bf16, const float *x,
                      const uint16_t *x_bf16, const float *weight, const float *bias, const float *save_mean,
                      const float *save_invstd, float *dx, uint16_t *dx_bf16, float *dres, int relu, int train,
                      void *ws, size_t ws_bytes, adaptseg_stream_t stream) {
  return bn_bwd_impl(rows, c, dy, nullptr, y, y_bf16, x, x_bf16, weight, bias, save_mean, save_invstd, dx, dx_bf16, dres,
                     nullptr, relu, train, nullptr, nullptr, ws, ws_bytes, stream);
}

int adaptseg_bn_bwd_xg(int64_t rows, int c, const float *dy, const uint16_t *dy_bf16, const uint32_t *dy_bits,
                       const float *y, const uint16_t *y_bf16, const float *x, const uint16_t *x_bf16,
                       const float *weight, const float *bias, const float *save_mean, const float *save_invstd,
                       float *dx, uint16_t *dx_bf16, float *dres, uint16_t *dres_bf16, int relu, int train, void *ws,
                       size_t ws_bytes, adaptseg_stream_t stream) {
  return bn_bwd_impl(rows, c, dy, dy_bf16, y, y_bf16, x, x_bf16, weight, bias, save_mean, save_invstd, dx, dx_bf16,
                     dres, dres_bf16, relu, train, nullptr, nullptr, ws, ws_bytes, stream, dy_bits);
}

int adaptseg_bn_bwd_sums(int64_t rows, int c, const float *dy, const uint16_t *dy_bf16, const uint32_t *dy_bits,
                         const float *y, const uint16_t *y_bf16, const float *x, const uint16_t *x_bf16,
                         const float *weight, const float *bias, const float *save_mean, const float *save_invstd,
                         float *dx, uint16_t *dx_bf16, float *dres, uint16_t *dres_bf16, int relu,
                         const float *partial, int ntiles, void *ws, size_t ws_bytes, adaptseg_stream_t stream) {
  AS_CHECK_ARG(partial && ntiles > 0, "bn_bwd_sums: null partial sums / ntiles %d", ntiles);
  return bn_bwd_impl(rows, c, dy, dy_bf16, y, y_bf16, x, x_bf16, weight, bias, save_mean, save_invstd, dx, dx_bf16,
                     dres, dres_bf16, relu, 1, nullptr, nullptr, ws, ws_bytes, stream, dy_bits, partial, ntiles);
}

int adaptseg_bn_bwd_affine(int64_t rows, int c, const float *dy, const float *y, const float *x,
                           const float *weight, const float *bias, const float *save_mean,
                           const float *save_invstd, float *dx, float *dres, int act, float *dweight,
                           float *dbias, void *ws, size_t ws_bytes, adaptseg_stream_t stream) {
  AS_CHECK_ARG(dweight || dbias, "bn_bwd_affine: no affine gradient requested");
  return bn_bwd_impl(rows, c, dy, nullptr, y, nullptr, x, nullptr, weight, bias, save_mean, save_invstd, dx, nullptr,
                     dres, nullptr, act, 1, dweight, dbias, ws, ws_bytes, stream);
}

}  // extern "C"

