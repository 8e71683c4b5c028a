// Thin convolutions on gfx950: convs with Cout <= 4 (the warper's 2-channel output conv,
// model/custom_layers.py:171-188; the discriminator's 1-channel classifier,
// model/discriminator.py:19).  The implicit GEMM pads their 1-4 wide output dimension (fwd N,
// wgrad M) or reduction (dgrad K = taps*Cout) to 32-wide MFMA tiles and wastes >= 7/8 of every
// MFMA; these ops are HBM-bound, so they run here on the vector ALUs with coalesced channel-
// quad loads:
//   fwd    a group of 16 lanes owns an output pixel, each lane a strided set of input-channel
//          quads; KO partial dot products reduced across the 16 lanes (fixed butterfly order);
//   dgrad  a lane owns one (input pixel, channel quad) and gathers its <= taps*KO terms (stride 1);
//   wgrad  a lane owns a weight column quad (tap, 4 input channels) and a strided set of the
//          chunk's pixels; the 4 pixel lanes are summed in LDS, the chunks in a fixed-order
//          second pass that writes (or accumulates into) dW.
// Weights stay in LDS (KO * taps * C floats).  Same epilogue flags and order as the igemm
// kernels: + bias, (+ out), (+ res), activation / activation gradient.
#include "common.hpp"
#include "conv_thin.hpp"
#include <algorithm>

namespace adaptseg {
namespace {

constexpr int kThinMaxW = 16384;  // LDS weight floats (64 KB)

struct ThinGeo {
  int n, c, h, w, k, oh, ow, kh, kw, stride, pad, dil;
  int64_t sxn, sxh, sxw;  // input strides (channel stride 1)
};

__device__ __forceinline__ float4 ld4(const float *p) { return *reinterpret_cast<const float4 *>(p); }

__device__ __forceinline__ float dot4(float4 a, float4 b) { return a.x * b.x + a.y * b.y + a.z * b.z + a.w * b.w; }

// A work item = one output row slice of 16 pixels x 16 lanes; blocks stride over them.
template <int KO>
__global__ void __launch_bounds__(256) thin_fwd_kernel(ThinGeo g, const float *__restrict__ x, const float *__restrict__ wt,
                                                       const float *__restrict__ bias, const float *res, float *out,
                                                       int flags) {
  extern __shared__ __attribute__((aligned(16))) float sw[];
  const int nw = KO * g.kh * g.kw * g.c;
  for (int i = threadIdx.x; i < nw; i += blockDim.x) sw[i] = wt[i];
  __syncthreads();
  const int lane = threadIdx.x & 15;
  const int q4 = g.c >> 2, taps = g.kh * g.kw;
  const int slices = (g.ow + 15) >> 4, nwork = g.n * g.oh * slices;
  for (int wk = blockIdx.x; wk < nwork; wk += gridDim.x) {   // LDS weights amortised over rows
  const int row = wk / slices;  // b * oh + oh
  const int ow = (wk - row * slices) * 16 + (threadIdx.x >> 4);
  if (ow >= g.ow) continue;
  const int oh = row % g.oh, b = row / g.oh;
  float acc[KO];
#pragma unroll
  for (int o = 0; o < KO; ++o) acc[o] = 0.f;
  const float *xb = x + (int64_t)b * g.sxn;
  for (int kh = 0; kh < g.kh; ++kh) {
    const int iy = oh * g.stride + kh * g.dil - g.pad;
    if ((unsigned)iy >= (unsigned)g.h) continue;
    for (int kw = 0; kw < g.kw; ++kw) {
      const int ix = ow * g.stride + kw * g.dil - g.pad;
      if ((unsigned)ix >= (unsigned)g.w) continue;
      const float *xp = xb + iy * g.sxh + ix * g.sxw;
      const float *wp = sw + (kh * g.kw + kw) * g.c;
      for (int q = lane; q < q4; q += 16) {
        const float4 v = ld4(xp + 4 * q);
#pragma unroll
        for (int o = 0; o < KO; ++o)
          acc[o] += dot4(v, *reinterpret_cast<const float4 *>(wp + o * taps * g.c + 4 * q));
      }
    }
  }
#pragma unroll
  for (int o = 0; o < KO; ++o)
#pragma unroll
    for (int s = 8; s > 0; s >>= 1) acc[o] += __shfl_xor(acc[o], s, 16);
  if (lane < KO) {
    float v = acc[0];
#pragma unroll
    for (int o = 1; o < KO; ++o) v = lane == o ? acc[o] : v;
    const int64_t idx = ((int64_t)row * g.ow + ow) * KO + lane;
    if (bias) v += bias[lane];
    if (flags & ADAPTSEG_EPI_ACCUMULATE) v += out[idx];
    if (flags & ADAPTSEG_EPI_RESIDUAL) v += res[idx];
    out[idx] = epi_act(v, flags);
  }
  }
}

// dx[b][iy][ix][c..c+3] = sum_{kh,kw} dY[b][iy+pad-kh*dil][ix+pad-kw*dil][:] . W[:][kh][kw][c..c+3]
// A work item = a slice of one input row, lanes over (ix, quad); blocks stride over them.
template <int KO>
__global__ void __launch_bounds__(256) thin_dgrad_kernel(ThinGeo g, const float *__restrict__ dy,
                                                         const float *__restrict__ wt, const float *res,
                                                         const float *aux, float *dx, int flags) {
  extern __shared__ __attribute__((aligned(16))) float sw[];
  const int nw = KO * g.kh * g.kw * g.c;
  for (int i = threadIdx.x; i < nw; i += blockDim.x) sw[i] = wt[i];
  __syncthreads();
  const int q4 = g.c >> 2, taps = g.kh * g.kw;
  const int slices = (g.w * q4 + 255) >> 8, nwork = g.n * g.h * slices;
  for (int wk = blockIdx.x; wk < nwork; wk += gridDim.x) {   // LDS weights amortised over rows
  const int row = wk / slices;  // b * h + iy
  const int t = (wk - row * slices) * 256 + threadIdx.x;
  if (t >= g.w * q4) continue;
  const int ix = t / q4, q = t - ix * q4;
  const int iy = row % g.h, b = row / g.h;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int kh = 0; kh < g.kh; ++kh) {
    const int oy = iy + g.pad - kh * g.dil;
    if ((unsigned)oy >= (unsigned)g.oh) continue;
    for (int kw = 0; kw < g.kw; ++kw) {
      const int ox = ix + g.pad - kw * g.dil;
      if ((unsigned)ox >= (unsigned)g.ow) continue;
      const float *gp = dy + (((int64_t)b * g.oh + oy) * g.ow + ox) * KO;
      const float *wp = sw + (kh * g.kw + kw) * g.c + 4 * q;
#pragma unroll
      for (int o = 0; o < KO; ++o) {
        const float gv = gp[o];
        const float4 wv = *reinterpret_cast<const float4 *>(wp + o * taps * g.c);
        acc.x += gv * wv.x;
        acc.y += gv * wv.y;
        acc.z += gv * wv.z;
        acc.w += gv * wv.w;
      }
    }
  }
  const int64_t e = ((int64_t)row * g.w + ix) * g.c + 4 * q;
  float v[4] = {acc.x, acc.y, acc.z, acc.w};
  if (flags & ADAPTSEG_EPI_ACCUMULATE) {
    const float4 o = ld4(dx + e);
    v[0] += o.x; v[1] += o.y; v[2] += o.z; v[3] += o.w;
  }
  if (flags & ADAPTSEG_EPI_RESIDUAL) {
    const float4 r = ld4(res + e);
    v[0] += r.x; v[1] += r.y; v[2] += r.z; v[3] += r.w;
  }
  if (flags & kEpiActGrad) {
    const float4 a = ld4(aux + e);
    v[0] = epi_act_grad(v[0], a.x, flags);
    v[1] = epi_act_grad(v[1], a.y, flags);
    v[2] = epi_act_grad(v[2], a.z, flags);
    v[3] = epi_act_grad(v[3], a.w, flags);
  }
  *reinterpret_cast<float4 *>(dx + e) = make_float4(v[0], v[1], v[2], v[3]);
  }
}

// Pass 1: partial[chunk][o][col] over the chunk's pixels; block = 64 column quads x 4 pixel
// lanes; the pixel position advances incrementally (no per-pixel division).
template <int KO>
__global__ void __launch_bounds__(256) thin_wgrad_partial_kernel(ThinGeo g, const float *__restrict__ dy,
                                                                 const float *__restrict__ x, int per,
                                                                 float *__restrict__ partial) {
  __shared__ float4 red[4][KO][64];
  const int cq = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int q4 = g.c >> 2, taps = g.kh * g.kw;
  const int ncol4 = taps * q4;
  const int col4 = blockIdx.x * 64 + cq;
  const bool cok = col4 < ncol4;
  const int tap = cok ? col4 / q4 : 0, q = cok ? col4 - tap * q4 : 0;
  const int kh = tap / g.kw, kw = tap - kh * g.kw;
  const int dyo = kh * g.dil - g.pad, dxo = kw * g.dil - g.pad;
  const int M = g.n * g.oh * g.ow;
  const int m0 = blockIdx.y * per, m1 = min(M, m0 + per);
  float4 acc[KO];
#pragma unroll
  for (int o = 0; o < KO; ++o) acc[o] = make_float4(0.f, 0.f, 0.f, 0.f);
  if (cok && m0 + rl < m1) {
    int m = m0 + rl;
    int ow = m % g.ow, t = m / g.ow;
    int oh = t % g.oh, b = t / g.oh;
    for (; m < m1; m += 4) {
      const int iy = oh * g.stride + dyo, ix = ow * g.stride + dxo;
      if ((unsigned)iy < (unsigned)g.h && (unsigned)ix < (unsigned)g.w) {
        const float4 v = ld4(x + (int64_t)b * g.sxn + iy * g.sxh + ix * g.sxw + 4 * q);
        const float *gp = dy + (int64_t)m * KO;
#pragma unroll
        for (int o = 0; o < KO; ++o) {
          const float gv = gp[o];
          acc[o].x += gv * v.x;
          acc[o].y += gv * v.y;
          acc[o].z += gv * v.z;
          acc[o].w += gv * v.w;
        }
      }
      ow += 4;
      while (ow >= g.ow) {
        ow -= g.ow;
        if (++oh == g.oh) {
          oh = 0;
          ++b;
        }
      }
    }
  }
#pragma unroll
  for (int o = 0; o < KO; ++o) red[rl][o][cq] = acc[o];
  __syncthreads();
  if (rl == 0 && cok) {
#pragma unroll
    for (int o = 0; o < KO; ++o) {
      float4 s = red[0][o][cq];
#pragma unroll
      for (int r = 1; r < 4; ++r) {
        const float4 u = red[r][o][cq];
        s.x += u.x; s.y += u.y; s.z += u.z; s.w += u.w;
      }
      // partial [chunk][o][taps*C]: the weight's own [co][kh][kw][ci] order
      *reinterpret_cast<float4 *>(partial + ((size_t)blockIdx.y * KO + o) * (size_t)taps * g.c + 4 * col4) = s;
    }
  }
}

// Pass 2: dW[col] (+)= sum over chunks; block = 16 columns x 16 chunk lanes, lanes summed in a
// fixed shuffle order.
__global__ void __launch_bounds__(256) thin_wgrad_final_kernel(int nchunks, int ncol, const float *__restrict__ partial,
                                                               float *dw, int accumulate) {
  const int col = blockIdx.x * 16 + (threadIdx.x & 15), cl = threadIdx.x >> 4;
  float s = 0.f;
  if (col < ncol)
    for (int c = cl; c < nchunks; c += 16) s += partial[(size_t)c * ncol + col];
  // lanes cl = 0..15 of one column sit 16 apart: threadIdx = cl*16 + col%16
  __shared__ float red[16][17];
  red[cl][threadIdx.x & 15] = s;
  __syncthreads();
  if (cl == 0 && col < ncol) {
    float t = red[0][threadIdx.x];
#pragma unroll
    for (int r = 1; r < 16; ++r) t += red[r][threadIdx.x];
    dw[col] = accumulate ? dw[col] + t : t;
  }
}

ThinGeo thin_geo(const adaptseg_conv_desc *d) {
  ThinGeo g;
  g.n = d->n; g.c = d->c; g.h = d->h; g.w = d->w; g.k = d->k; g.oh = d->oh; g.ow = d->ow;
  g.kh = d->kh; g.kw = d->kw; g.stride = d->stride; g.pad = d->pad[0]; g.dil = d->dil[0];
  g.sxn = d->in_stride[0]; g.sxh = d->in_stride[2]; g.sxw = d->in_stride[3];
  return g;
}

void wgrad_chunks(const adaptseg_conv_desc *d, int *colblocks, int *chunks, int *per) {
  const int64_t M = (int64_t)d->n * d->oh * d->ow;
  *colblocks = (int)ceil_div((int64_t)d->kh * d->kw * (d->c / 4), 64);
  const int want = std::max(1, 2048 / *colblocks);
  const int64_t maxc = std::max<int64_t>(1, M / 256);   // >= 256 pixels (64 per lane) per chunk
  int nc = (int)std::min<int64_t>(want, maxc);
  *per = (int)ceil_div(M, nc);
  *chunks = (int)ceil_div(M, *per);
}

inline bool al16(const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

}  // namespace

bool thin_eligible(const adaptseg_conv_desc *d, int op) {
  if (d->k < 1 || d->k > 4 || d->nseg != 1 || d->c % 4 != 0) return false;
  if (d->in_stride[1] != 1 || d->in_stride[0] % 4 || d->in_stride[2] % 4 || d->in_stride[3] % 4) return false;
  if ((int64_t)d->k * d->kh * d->kw * d->c > kThinMaxW) return false;
  if ((int64_t)d->n * d->h * d->w * d->c >= (1ll << 31) || (int64_t)d->n * d->oh * d->ow * d->c >= (1ll << 31))
    return false;
  if (op == ADAPTSEG_CONV_BWD_DATA && d->stride != 1) return false;
  return true;
}

size_t thin_workspace(const adaptseg_conv_desc *d, int op) {
  if (op != ADAPTSEG_CONV_BWD_WEIGHT) return 0;
  int cb, chunks, per;
  wgrad_chunks(d, &cb, &chunks, &per);
  return (size_t)chunks * d->k * d->kh * d->kw * d->c * sizeof(float);
}

double thin_flops(const adaptseg_conv_desc *d) {
  return 2.0 * d->n * d->oh * d->ow * d->k * d->c * d->kh * d->kw;
}

#define THIN_DISPATCH(KO_EXPR, CALL)            \
  switch (KO_EXPR) {                            \
    case 1: { constexpr int KO = 1; CALL; break; } \
    case 2: { constexpr int KO = 2; CALL; break; } \
    case 3: { constexpr int KO = 3; CALL; break; } \
    default: { constexpr int KO = 4; CALL; break; } \
  }

int thin_fwd(const adaptseg_conv_desc *d, const float *x, const float *w, const float *bias, const float *res,
             float *y, int flags, hipStream_t s) {
  if (!al16(x)) return ADAPTSEG_ERR_ARG;   // caller falls back
  const ThinGeo g = thin_geo(d);
  const unsigned grid = (unsigned)std::min<int64_t>(ceil_div(d->ow, 16) * d->n * d->oh, 4096);
  const size_t shm = (size_t)d->k * d->kh * d->kw * d->c * sizeof(float);
  int slot;
  timing_begin(thin_kernel_id(ADAPTSEG_CONV_FWD), s, thin_flops(d), &slot);
  THIN_DISPATCH(d->k, (thin_fwd_kernel<KO><<<grid, 256, shm, s>>>(g, x, w, bias, res, y, flags)));
  timing_end(slot, s);
  AS_CHECK_LAUNCH("thin_fwd");
  return ADAPTSEG_OK;
}

int thin_dgrad(const adaptseg_conv_desc *d, const float *dy, const float *w, const float *res, const float *aux,
               float *dx, int flags, hipStream_t s) {
  if (!al16(dx) || (res && !al16(res)) || (aux && !al16(aux))) return ADAPTSEG_ERR_ARG;
  const ThinGeo g = thin_geo(d);
  const unsigned grid = (unsigned)std::min<int64_t>(ceil_div((int64_t)d->w * (d->c / 4), 256) * d->n * d->h, 4096);
  const size_t shm = (size_t)d->k * d->kh * d->kw * d->c * sizeof(float);
  int slot;
  timing_begin(thin_kernel_id(ADAPTSEG_CONV_BWD_DATA), s, thin_flops(d), &slot);
  THIN_DISPATCH(d->k, (thin_dgrad_kernel<KO><<<grid, 256, shm, s>>>(g, dy, w, res, aux, dx, flags)));
  timing_end(slot, s);
  AS_CHECK_LAUNCH("thin_dgrad");
  return ADAPTSEG_OK;
}

int thin_wgrad(const adaptseg_conv_desc *d, const float *dy, const float *x, float *dw, int flags, void *ws,
               size_t ws_bytes, hipStream_t s) {
  if (!al16(x) || !al16(ws)) return ADAPTSEG_ERR_ARG;
  const size_t need = thin_workspace(d, ADAPTSEG_CONV_BWD_WEIGHT);
  if (!ws || ws_bytes < need) {
    set_error("thin wgrad: workspace %zu < %zu", ws_bytes, need);
    return ADAPTSEG_ERR_WORKSPACE;
  }
  const ThinGeo g = thin_geo(d);
  int cb, chunks, per;
  wgrad_chunks(d, &cb, &chunks, &per);
  float *partial = reinterpret_cast<float *>(ws);
  const int ncol = d->k * d->kh * d->kw * d->c;
  int slot;
  timing_begin(thin_kernel_id(ADAPTSEG_CONV_BWD_WEIGHT), s, thin_flops(d), &slot);
  // (An input-stationary variant — x read once, every tap's dY gathered per input pixel —
  // measured 2x slower than this tap-stationary one, which re-reads x per tap from L2.)
  THIN_DISPATCH(d->k, (thin_wgrad_partial_kernel<KO><<<dim3(cb, chunks), 256, 0, s>>>(g, dy, x, per, partial)));
  thin_wgrad_final_kernel<<<(unsigned)ceil_div(ncol, 16), 256, 0, s>>>(chunks, ncol, partial, dw,
                                                                        (flags & ADAPTSEG_EPI_ACCUMULATE) ? 1 : 0);
  timing_end(slot, s);
  AS_CHECK_LAUNCH("thin_wgrad");
  return ADAPTSEG_OK;
}

}  // namespace adaptseg
