// The fork's Warper on gfx950: the decoder's ReLU -> x2 bilinear
// upsample -> skip concatenation as one HBM pass each way, and the prediction warp
// (tanh + linspace grid, clamp, grid_sample) forward and backward.
//
// Reference (file:line in /root/reference):
//   SkipConnectionDecode.forward  torch.cat((skip, out), 1)      model/warper.py:130-144
//   DecoderInput / UpConvolution / DecoderOutput (non-transpose): ReLU(inplace) ->
//     nn.Upsample(scale_factor=2, mode='bilinear') (align_corners=False)
//                                                                 model/custom_layers.py:117-188
//   ResNetMulti.warp                                             model/deeplab_multi.py:238-255
//
// Layouts: activations NHWC fp32; the warp field NHWC [n][h][w][fc] (the warper's conv output).
// Determinism: every reduction has a fixed order; the grid_sample input gradient — a scatter
// whose targets depend on the data — accumulates in 64-bit fixed point (integer atomics are
// associative), scaled per call from max|dy| so no sum can overflow; see grid_scatter_kernel.
#include "common.hpp"
#include <algorithm>

#pragma clang fp contract(off)   // match the reference's separately rounded float ops

namespace adaptseg {
namespace {

inline int grid1d(int64_t total, int threads = 256, int64_t cap = 16384) {
  return (int)std::max<int64_t>(1, std::min<int64_t>(ceil_div(total, threads), cap));
}

// nn.Upsample(scale_factor=2, bilinear, align_corners=False): output index o of an axis of
// input length L reads src = max(0.5*(o+0.5)-0.5, 0): i0 = floor(src), i1 = min(i0+1, L-1),
// lambda = src - i0 (0, 0.25 or 0.75: exact in float).
__device__ __forceinline__ void up2_src(int o, int L, int &i0, int &i1, float &lam) {
  float src = 0.5f * ((float)o + 0.5f) - 0.5f;
  if (src < 0.f) src = 0.f;
  i0 = (int)src;
  i1 = i0 < L - 1 ? i0 + 1 : i0;
  lam = src - (float)i0;
}

__device__ __forceinline__ float4 relu4(float4 v) {
  return make_float4(fmaxf(v.x, 0.f), fmaxf(v.y, 0.f), fmaxf(v.z, 0.f), fmaxf(v.w, 0.f));
}

// out[b][Y][X][c] = up2(relu(cat(s, d)))[c]; one thread per (output pixel, channel quad).
__global__ void __launch_bounds__(256)
up2_relu_cat_fwd_kernel(int n, int h, int w, int cs, int cd, const float *__restrict__ s,
                        const float *__restrict__ d, float *__restrict__ out) {
  const int C = cs + cd, q4 = C >> 2, OH = 2 * h, OW = 2 * w;
  const int64_t total = (int64_t)n * OH * OW * q4;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int q = (int)(i % q4);
    const int64_t pix = i / q4;
    const int X = (int)(pix % OW);
    const int64_t t = pix / OW;
    const int Y = (int)(t % OH), b = (int)(t / OH);
    int y0, y1, x0, x1;
    float ly, lx;
    up2_src(Y, h, y0, y1, ly);
    up2_src(X, w, x0, x1, lx);
    int c = q * 4;
    const float *src;
    int cc;
    if (c < cs) { src = s; cc = cs; }
    else { src = d; cc = cd; c -= cs; }
    const float *base = src + (int64_t)b * h * w * cc + c;
    const float4 v00 = relu4(*reinterpret_cast<const float4 *>(base + ((int64_t)y0 * w + x0) * cc));
    const float4 v01 = relu4(*reinterpret_cast<const float4 *>(base + ((int64_t)y0 * w + x1) * cc));
    const float4 v10 = relu4(*reinterpret_cast<const float4 *>(base + ((int64_t)y1 * w + x0) * cc));
    const float4 v11 = relu4(*reinterpret_cast<const float4 *>(base + ((int64_t)y1 * w + x1) * cc));
    const float h0 = 1.f - ly, h1 = ly, w0 = 1.f - lx, w1 = lx;
    float4 o;
    o.x = h0 * (w0 * v00.x + w1 * v01.x) + h1 * (w0 * v10.x + w1 * v11.x);
    o.y = h0 * (w0 * v00.y + w1 * v01.y) + h1 * (w0 * v10.y + w1 * v11.y);
    o.z = h0 * (w0 * v00.z + w1 * v01.z) + h1 * (w0 * v10.z + w1 * v11.z);
    o.w = h0 * (w0 * v00.w + w1 * v01.w) + h1 * (w0 * v10.w + w1 * v11.w);
    reinterpret_cast<float4 *>(out)[i] = o;
  }
}

// Weight of input index i in output index o (0 when o does not read i).
__device__ __forceinline__ float up2_weight(int o, int i, int L) {
  int i0, i1;
  float lam;
  up2_src(o, L, i0, i1, lam);
  return (i0 == i ? 1.f - lam : 0.f) + (i1 == i ? lam : 0.f);
}

// Adjoint: per input pixel and channel quad, gather the <= 4x4 output pixels that read it (a
// fixed order), then the ReLU mask of the concatenated source and the split into ds / dd.
__global__ void __launch_bounds__(256)
up2_relu_cat_bwd_kernel(int n, int h, int w, int cs, int cd, const float *__restrict__ s,
                        const float *__restrict__ d, const float *__restrict__ dout,
                        float *__restrict__ ds, float *__restrict__ dd) {
  const int C = cs + cd, q4 = C >> 2, OH = 2 * h, OW = 2 * w;
  const int64_t total = (int64_t)n * h * w * q4;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int q = (int)(i % q4);
    const int64_t pix = i / q4;
    const int x = (int)(pix % w);
    const int64_t t = pix / w;
    const int y = (int)(t % h), b = (int)(t / h);
    const int c = q * 4;
    float wy[4], wx[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int Y = 2 * y - 1 + k, X = 2 * x - 1 + k;
      wy[k] = (Y >= 0 && Y < OH) ? up2_weight(Y, y, h) : 0.f;
      wx[k] = (X >= 0 && X < OW) ? up2_weight(X, x, w) : 0.f;
    }
    const float *g = dout + (int64_t)b * OH * OW * C + c;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int ky = 0; ky < 4; ++ky) {
      if (wy[ky] == 0.f) continue;
      const int Y = 2 * y - 1 + ky;
      float4 r = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int kx = 0; kx < 4; ++kx) {
        if (wx[kx] == 0.f) continue;
        const int X = 2 * x - 1 + kx;
        const float4 v = *reinterpret_cast<const float4 *>(g + ((int64_t)Y * OW + X) * C);
        r.x += wx[kx] * v.x; r.y += wx[kx] * v.y; r.z += wx[kx] * v.z; r.w += wx[kx] * v.w;
      }
      acc.x += wy[ky] * r.x; acc.y += wy[ky] * r.y; acc.z += wy[ky] * r.z; acc.w += wy[ky] * r.w;
    }
    const float *src;
    float *dst;
    int cc, c2;
    if (c < cs) { src = s; dst = ds; cc = cs; c2 = c; }
    else { src = d; dst = dd; cc = cd; c2 = c - cs; }
    const int64_t off = pix * cc + c2;
    const float4 v = *reinterpret_cast<const float4 *>(src + off);
    acc.x = v.x > 0.f ? acc.x : 0.f;
    acc.y = v.y > 0.f ? acc.y : 0.f;
    acc.z = v.z > 0.f ? acc.z : 0.f;
    acc.w = v.w > 0.f ? acc.w : 0.f;
    *reinterpret_cast<float4 *>(dst + off) = acc;
  }
}

// float32(np.linspace(-1, 1, L)[j]): j*step + start in double (two roundings, as numpy),
// the last sample exactly 1, a single sample -1.
__device__ __forceinline__ float linspace_pm1(int j, int L) {
  if (L == 1) return -1.f;
  if (j == L - 1) return 1.f;
  const double step = 2.0 / (double)(L - 1);
  return (float)__dadd_rn(__dmul_rn((double)j, step), -1.0);
}

struct Tap {
  float ix, iy, nw, ne, sw, se;
  int x0, y0;
  float gx_pre, gy_pre, tx, ty;  // pre-clamp grid and tanh values (for the backward)
};

// sampler = clamp(tanh(flow[last pair]) + base, -1, 1); grid_sample's unnormalize
// ((g + 1) * size - 1) / 2 (align_corners=False) and bilinear corner weights.
__device__ __forceinline__ Tap warp_tap(const float *flow, int fc, int64_t pix, int y, int x, int h, int w) {
  Tap t;
  const float *f = flow + pix * fc + (fc / 2 - 1) * 2;
  t.tx = tanhf(f[0]);
  t.ty = tanhf(f[1]);
  t.gx_pre = t.tx + linspace_pm1(x, w);
  t.gy_pre = t.ty + linspace_pm1(y, h);
  const float gx = fminf(fmaxf(t.gx_pre, -1.f), 1.f);
  const float gy = fminf(fmaxf(t.gy_pre, -1.f), 1.f);
  t.ix = ((gx + 1.f) * (float)w - 1.f) / 2.f;
  t.iy = ((gy + 1.f) * (float)h - 1.f) / 2.f;
  const float fx = floorf(t.ix), fy = floorf(t.iy);
  t.x0 = (int)fx;
  t.y0 = (int)fy;
  const float ix_se = fx + 1.f, iy_se = fy + 1.f;
  t.nw = (ix_se - t.ix) * (iy_se - t.iy);
  t.ne = (t.ix - fx) * (iy_se - t.iy);
  t.sw = (ix_se - t.ix) * (t.iy - fy);
  t.se = (t.ix - fx) * (t.iy - fy);
  return t;
}

__device__ __forceinline__ bool inb(int y, int x, int h, int w) { return y >= 0 && y < h && x >= 0 && x < w; }

// Per-block cache of the sample taps of floor(256 / C) consecutive pixels: computed once per
// pixel (two tanh and the double-precision linspace) instead of once per channel.
struct TapCache {
  float nw[256], ne[256], sw[256], se[256];
  int x0[256], y0[256], b[256];
};

__device__ __forceinline__ void fill_taps(TapCache &tc, int pb, int64_t base, int64_t total, const float *flow,
                                          int fc, int h, int w) {
  if (threadIdx.x < pb && base + threadIdx.x < total) {
    const int64_t pix = base + threadIdx.x;
    const int x = (int)(pix % w);
    const int64_t t2 = pix / w;
    const int y = (int)(t2 % h);
    const Tap t = warp_tap(flow, fc, pix, y, x, h, w);
    tc.nw[threadIdx.x] = t.nw;
    tc.ne[threadIdx.x] = t.ne;
    tc.sw[threadIdx.x] = t.sw;
    tc.se[threadIdx.x] = t.se;
    tc.x0[threadIdx.x] = t.x0;
    tc.y0[threadIdx.x] = t.y0;
    tc.b[threadIdx.x] = (int)(t2 / h);
  }
}

// y[b][Y][X][c] = bilinear sample of x at the warped point (zeros outside); a block handles
// floor(256 / C) pixels, one thread per (pixel, channel), both heads (x1 may be NULL).
__global__ void __launch_bounds__(256)
grid_warp_fwd_kernel(int n, int C, int h, int w, int fc, const float *__restrict__ flow,
                     const float *__restrict__ x1, const float *__restrict__ x2, float *__restrict__ y1,
                     float *__restrict__ y2) {
  __shared__ TapCache tc;
  const int pb = 256 / C;
  const int j = threadIdx.x / C, c = threadIdx.x - (threadIdx.x / C) * C;
  const int64_t total = (int64_t)n * h * w;
  for (int64_t base = (int64_t)blockIdx.x * pb; base < total; base += (int64_t)gridDim.x * pb) {
    fill_taps(tc, pb, base, total, flow, fc, h, w);
    __syncthreads();
    const int64_t pix = base + j;
    if (j < pb && pix < total) {
      const int x0 = tc.x0[j], y0 = tc.y0[j];
      const bool bnw = inb(y0, x0, h, w), bne = inb(y0, x0 + 1, h, w);
      const bool bsw = inb(y0 + 1, x0, h, w), bse = inb(y0 + 1, x0 + 1, h, w);
      const int64_t pnw = (((int64_t)tc.b[j] * h + y0) * w + x0) * C + c;
      const int64_t i = pix * C + c;
      for (int head = 0; head < 2; ++head) {
        const float *xp = head ? x2 : x1;
        float *yp = head ? y2 : y1;
        if (!xp) continue;
        float o = 0.f;
        if (bnw) o += xp[pnw] * tc.nw[j];
        if (bne) o += xp[pnw + C] * tc.ne[j];
        if (bsw) o += xp[pnw + (int64_t)w * C] * tc.sw[j];
        if (bse) o += xp[pnw + (int64_t)(w + 1) * C] * tc.se[j];
        yp[i] = o;
      }
    }
    __syncthreads();
  }
}

// Gradient of the warp field: per pixel, sum over channels (and both heads) of dy times the
// derivative of the bilinear sample, times size/2 (unnormalize), the clamp mask (pass where
// -1 <= pre <= 1, as torch's clamp backward) and tanh' = 1 - tanh^2.  A block handles
// floor(256 / C) pixels with one thread per (pixel, channel) — coalesced dy and corner reads —
// and one thread per pixel then sums its C channel terms from LDS in channel order.
__global__ void __launch_bounds__(256)
grid_warp_dflow_kernel(int n, int C, int h, int w, int fc, const float *__restrict__ flow,
                       const float *__restrict__ x1, const float *__restrict__ x2,
                       const float *__restrict__ dy1, const float *__restrict__ dy2,
                       float *__restrict__ dflow) {
  __shared__ float rx[256], ry[256];
  const int pb = 256 / C;                     // pixels per block iteration
  const int j = threadIdx.x / C, c = threadIdx.x - (threadIdx.x / C) * C;
  const int64_t total = (int64_t)n * h * w;
  for (int64_t base = (int64_t)blockIdx.x * pb; base < total; base += (int64_t)gridDim.x * pb) {
    const int64_t pix = base + j;
    float gix = 0.f, giy = 0.f;
    if (j < pb && pix < total) {
      const int x = (int)(pix % w);
      const int64_t t2 = pix / w;
      const int y = (int)(t2 % h), b = (int)(t2 / h);
      const Tap t = warp_tap(flow, fc, pix, y, x, h, w);
      const bool bnw = inb(t.y0, t.x0, h, w), bne = inb(t.y0, t.x0 + 1, h, w);
      const bool bsw = inb(t.y0 + 1, t.x0, h, w), bse = inb(t.y0 + 1, t.x0 + 1, h, w);
      const int64_t pnw = (((int64_t)b * h + t.y0) * w + t.x0) * C + c;
      const float fx = (float)t.x0, fy = (float)t.y0;
      const float ix_se = fx + 1.f, iy_se = fy + 1.f;
      for (int head = 0; head < 2; ++head) {
        const float *xp = head ? x2 : x1;
        const float *gp = head ? dy2 : dy1;
        if (!xp || !gp) continue;
        const float go = gp[pix * C + c];
        if (bnw) {
          const float v = xp[pnw];
          gix -= v * (iy_se - t.iy) * go;
          giy -= v * (ix_se - t.ix) * go;
        }
        if (bne) {
          const float v = xp[pnw + C];
          gix += v * (iy_se - t.iy) * go;
          giy -= v * (t.ix - fx) * go;
        }
        if (bsw) {
          const float v = xp[pnw + (int64_t)w * C];
          gix -= v * (t.iy - fy) * go;
          giy += v * (ix_se - t.ix) * go;
        }
        if (bse) {
          const float v = xp[pnw + (int64_t)(w + 1) * C];
          gix += v * (t.iy - fy) * go;
          giy += v * (t.ix - fx) * go;
        }
      }
    }
    rx[threadIdx.x] = gix;
    ry[threadIdx.x] = giy;
    __syncthreads();
    const int64_t op = base + threadIdx.x;
    if (threadIdx.x < pb && op < total) {
      float sx = 0.f, sy = 0.f;
      for (int k = 0; k < C; ++k) {
        sx += rx[threadIdx.x * C + k];
        sy += ry[threadIdx.x * C + k];
      }
      const int x = (int)(op % w);
      const int64_t t2 = op / w;
      const int y = (int)(t2 % h);
      const Tap t = warp_tap(flow, fc, op, y, x, h, w);
      float dgx = sx * ((float)w / 2.f), dgy = sy * ((float)h / 2.f);
      dgx = (t.gx_pre >= -1.f && t.gx_pre <= 1.f) ? dgx : 0.f;
      dgy = (t.gy_pre >= -1.f && t.gy_pre <= 1.f) ? dgy : 0.f;
      float *o = dflow + op * fc;
      for (int k = 0; k < fc - 2; ++k) o[k] = 0.f;
      o[fc - 2] = dgx * (1.f - t.tx * t.tx);
      o[fc - 1] = dgy * (1.f - t.ty * t.ty);
    }
    __syncthreads();
  }
}

// max |dy| as float bits (non-negative floats order like their bit patterns: the atomic max is
// order-independent).
__global__ void __launch_bounds__(256)
absmax_kernel(int64_t total, const float *__restrict__ a, unsigned int *out) {
  float m = 0.f;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x)
    m = fmaxf(m, fabsf(a[i]));
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  if ((threadIdx.x & 63) == 0 && m > 0.f) atomicMax(out, __float_as_uint(m));
}

// Fixed-point exponent: every contribution w*dy has |w*dy| <= max|dy| < 2^e, and one input
// pixel receives at most one contribution per output pixel of its image (2^b >= h*w of them),
// so |sum| * 2^k < 2^(e+b+k) = 2^62 with k = 62 - b - e: no overflow, and each contribution is
// rounded to 2^-(k+1) = 2^(b+e-63), i.e. ~2^-42 of max|dy| at 1024x2048.
__device__ __forceinline__ int fixed_exp(unsigned int mbits, int hw) {
  int e;
  frexpf(__uint_as_float(mbits), &e);   // max = m * 2^e, m in [0.5, 1)
  int b = 0;
  while ((1ll << b) < (long long)hw) ++b;
  return 62 - b - e;
}

// Scatter dy * corner weight into the int64 accumulators of the 4 corners (zeros padding:
// out-of-range corners dropped).  One thread per dy element: a wave's atomics hit consecutive
// channels of the same corner pixels.
__global__ void __launch_bounds__(256)
grid_scatter_kernel(int n, int C, int h, int w, int fc, const float *__restrict__ flow,
                    const float *__restrict__ dy, const unsigned int *__restrict__ mbits,
                    unsigned long long *__restrict__ acc) {
  __shared__ TapCache tc;
  const unsigned int mb = *mbits;
  if (mb == 0u) return;  // dy == 0: nothing to scatter (uniform over the grid)
  const double scale = ldexp(1.0, fixed_exp(mb, h * w));
  const int pb = 256 / C;
  const int j = threadIdx.x / C, c = threadIdx.x - (threadIdx.x / C) * C;
  const int64_t total = (int64_t)n * h * w;
  for (int64_t base = (int64_t)blockIdx.x * pb; base < total; base += (int64_t)gridDim.x * pb) {
    fill_taps(tc, pb, base, total, flow, fc, h, w);
    __syncthreads();
    const int64_t pix = base + j;
    const float go = (j < pb && pix < total) ? dy[pix * C + c] : 0.f;
    if (go != 0.f) {
      const int x0 = tc.x0[j], y0 = tc.y0[j];
      const int64_t pnw = (((int64_t)tc.b[j] * h + y0) * w + x0) * C + c;
      if (inb(y0, x0, h, w))
        atomicAdd(acc + pnw, (unsigned long long)llrint((double)(go * tc.nw[j]) * scale));
      if (inb(y0, x0 + 1, h, w))
        atomicAdd(acc + pnw + C, (unsigned long long)llrint((double)(go * tc.ne[j]) * scale));
      if (inb(y0 + 1, x0, h, w))
        atomicAdd(acc + pnw + (int64_t)w * C, (unsigned long long)llrint((double)(go * tc.sw[j]) * scale));
      if (inb(y0 + 1, x0 + 1, h, w))
        atomicAdd(acc + pnw + (int64_t)(w + 1) * C, (unsigned long long)llrint((double)(go * tc.se[j]) * scale));
    }
    __syncthreads();
  }
}

__global__ void __launch_bounds__(256)
fixed_to_float_kernel(int64_t total, int hw, const unsigned long long *__restrict__ acc,
                      const unsigned int *__restrict__ mbits, float *__restrict__ dx) {
  const unsigned int mb = *mbits;
  const double inv = mb ? ldexp(1.0, -fixed_exp(mb, hw)) : 0.0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x)
    dx[i] = (float)((double)(long long)acc[i] * inv);
}

}  // namespace
}  // namespace adaptseg

using namespace adaptseg;

extern "C" {

int adaptseg_up2_relu_cat_fwd(int n, int h, int w, int cs, int cd, const float *s, const float *d, float *out,
                              adaptseg_stream_t stream) {
  AS_CHECK_ARG(n > 0 && h > 0 && w > 0 && cs >= 0 && cd > 0 && cs % 4 == 0 && cd % 4 == 0,
               "up2_relu_cat_fwd: bad shape (cs=%d cd=%d: multiples of 4, cd > 0)", cs, cd);
  AS_CHECK_ARG(d && out && (cs == 0 || s), "up2_relu_cat_fwd: null pointer");
  const int64_t total = (int64_t)n * 4 * h * w * ((cs + cd) / 4);
  int slot;  // inputs once, the 4x output once
  timing_begin(kTUp2Fwd, as_stream(stream), 20.0 * n * h * w * (cs + cd), &slot);
  up2_relu_cat_fwd_kernel<<<grid1d(total), 256, 0, as_stream(stream)>>>(n, h, w, cs, cd, s, d, out);
  timing_end(slot, as_stream(stream));
  AS_CHECK_LAUNCH("up2_relu_cat_fwd");
  return ADAPTSEG_OK;
}

int adaptseg_up2_relu_cat_bwd(int n, int h, int w, int cs, int cd, const float *s, const float *d,
                              const float *dout, float *ds, float *dd, adaptseg_stream_t stream) {
  AS_CHECK_ARG(n > 0 && h > 0 && w > 0 && cs >= 0 && cd > 0 && cs % 4 == 0 && cd % 4 == 0,
               "up2_relu_cat_bwd: bad shape (cs=%d cd=%d)", cs, cd);
  AS_CHECK_ARG(d && dout && dd && (cs == 0 || (s && ds)), "up2_relu_cat_bwd: null pointer");
  const int64_t total = (int64_t)n * h * w * ((cs + cd) / 4);
  int slot;  // dout (4x) + the mask sources in, ds/dd out
  timing_begin(kTUp2Bwd, as_stream(stream), 24.0 * n * h * w * (cs + cd), &slot);
  up2_relu_cat_bwd_kernel<<<grid1d(total), 256, 0, as_stream(stream)>>>(n, h, w, cs, cd, s, d, dout, ds, dd);
  timing_end(slot, as_stream(stream));
  AS_CHECK_LAUNCH("up2_relu_cat_bwd");
  return ADAPTSEG_OK;
}

int adaptseg_grid_warp_fwd(int n, int c, int h, int w, int fc, const float *flow, const float *x1,
                           const float *x2, float *y1, float *y2, adaptseg_stream_t stream) {
  AS_CHECK_ARG(n > 0 && c > 0 && c <= 256 && h > 0 && w > 0 && fc >= 2 && fc % 2 == 0,
               "grid_warp_fwd: bad shape (1 <= c <= 256)");
  AS_CHECK_ARG((int64_t)h * w < (1ll << 30), "grid_warp_fwd: h*w too large");
  AS_CHECK_ARG(flow && (x1 || x2) && (!x1 || y1) && (!x2 || y2), "grid_warp_fwd: null pointer");
  const int64_t total = (int64_t)n * h * w * c;
  int slot;  // the field, each head's input and output once
  timing_begin(kTWarpFwd, as_stream(stream), 4.0 * n * h * w * (2 + 2 * c * ((x1 ? 1 : 0) + (x2 ? 1 : 0))), &slot);
  grid_warp_fwd_kernel<<<grid1d(total), 256, 0, as_stream(stream)>>>(n, c, h, w, fc, flow, x1, x2, y1, y2);
  timing_end(slot, as_stream(stream));
  AS_CHECK_LAUNCH("grid_warp_fwd");
  return ADAPTSEG_OK;
}

int adaptseg_grid_warp_bwd_workspace_size(int n, int c, int h, int w, size_t *bytes) {
  AS_CHECK_ARG(bytes && n > 0 && c > 0 && h > 0 && w > 0, "grid_warp_bwd_workspace_size: bad args");
  *bytes = 256 + (size_t)n * h * w * c * sizeof(unsigned long long);
  return ADAPTSEG_OK;
}

int adaptseg_grid_warp_bwd(int n, int c, int h, int w, int fc, const float *flow, const float *x1,
                           const float *x2, const float *dy1, const float *dy2, float *dflow, float *dx1,
                           float *dx2, void *ws, size_t ws_bytes, adaptseg_stream_t stream) {
  AS_CHECK_ARG(n > 0 && c > 0 && c <= 256 && h > 0 && w > 0 && fc >= 2 && fc % 2 == 0,
               "grid_warp_bwd: bad shape (1 <= c <= 256)");
  AS_CHECK_ARG((int64_t)h * w < (1ll << 30), "grid_warp_bwd: h*w too large");
  AS_CHECK_ARG(flow && (dy1 || dy2), "grid_warp_bwd: null pointer");
  AS_CHECK_ARG(!dflow || ((!dy1 || x1) && (!dy2 || x2)), "grid_warp_bwd: dflow needs the sampled inputs");
  AS_CHECK_ARG((!dx1 || dy1) && (!dx2 || dy2), "grid_warp_bwd: dx needs its dy");
  hipStream_t s = as_stream(stream);
  const int64_t total = (int64_t)n * h * w * c;
  if (dflow) {
    int slot;  // field in and out, x and dy of each head once
    timing_begin(kTWarpDflow, s, 4.0 * n * h * w * (4 + 2 * c * ((dy1 ? 1 : 0) + (dy2 ? 1 : 0))), &slot);
    grid_warp_dflow_kernel<<<grid1d((int64_t)n * h * w * c), 256, 0, s>>>(n, c, h, w, fc, flow, x1, x2, dy1, dy2,
                                                                           dflow);
    timing_end(slot, s);
    AS_CHECK_LAUNCH("grid_warp_dflow");
  }
  if (dx1 || dx2) {
    size_t need = 0;
    adaptseg_grid_warp_bwd_workspace_size(n, c, h, w, &need);
    if (!ws || ws_bytes < need) {
      set_error("grid_warp_bwd: workspace %zu < %zu", ws_bytes, need);
      return ADAPTSEG_ERR_WORKSPACE;
    }
    unsigned int *mbits = reinterpret_cast<unsigned int *>(ws);
    unsigned long long *acc = reinterpret_cast<unsigned long long *>(reinterpret_cast<char *>(ws) + 256);
    for (int head = 0; head < 2; ++head) {
      const float *dy = head ? dy2 : dy1;
      float *dx = head ? dx2 : dx1;
      if (!dx) continue;
      int slot;  // algorithmic: the field and dy in, dx out (accumulator passes not counted)
      timing_begin(kTWarpScatter, s, 4.0 * n * h * w * (2 + 2 * c), &slot);
      if (hipMemsetAsync(ws, 0, need, s) != hipSuccess) {
        set_error("grid_warp_bwd: hipMemsetAsync failed");
        return ADAPTSEG_ERR_HIP;
      }
      absmax_kernel<<<grid1d(total, 256, 2048), 256, 0, s>>>(total, dy, mbits);
      AS_CHECK_LAUNCH("grid_warp_absmax");
      grid_scatter_kernel<<<grid1d(total), 256, 0, s>>>(n, c, h, w, fc, flow, dy, mbits, acc);
      AS_CHECK_LAUNCH("grid_warp_scatter");
      fixed_to_float_kernel<<<grid1d(total), 256, 0, s>>>(total, h * w, acc, mbits, dx);
      timing_end(slot, s);
      AS_CHECK_LAUNCH("grid_warp_fixed_to_float");
    }
  }
  return ADAPTSEG_OK;
}

}  // extern "C"
