// HBM-bound kernels of the AdaptSegNet step on gfx950 (NHWC fp32 activations):
//   max-pool fwd/bwd           model/deeplab_multi.py:135,178
//   bilinear upsample fwd/bwd  model/deeplab_multi.py:188-189 (align_corners=True)
//   channel softmax fwd/bwd    train_gta2cityscapes_multi.py:423,442,454,617-618
//   cross entropy (ignore 255) utils/loss.py:14-36, train_gta2cityscapes_multi.py:359,546
//   BCE-with-logits / MSE vs a constant target   train_gta2cityscapes_multi.py:542-545
//   SGD(momentum, wd) / Adam   train_gta2cityscapes_multi.py:532-540
// Every reduction is block-partial + one ordered finalize (no float atomics), so results
// are bitwise reproducible run to run.
#include "common.hpp"
#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstring>

namespace adaptseg {

static thread_local char g_err[512] = "";

void set_error(const char *fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

static int grid1d(int64_t n, int per_block = 256, int cap = 8192) {
  return (int)std::max<int64_t>(1, std::min<int64_t>(ceil_div(n, per_block), cap));
}

// ------------------------------------------------------------------------------------
// MaxPool2d NHWC.  argmax stores the window position (kh*k + kw) of the first maximum
// in (kh, kw) scan order — the torch CPU tie rule.  Padding acts as -inf.
// ------------------------------------------------------------------------------------
__global__ void maxpool_fwd_kernel(int n, int C, int H, int W, int OH, int OW, int k, int s, int p,
                                   const float *__restrict__ x, float *__restrict__ y,
                                   uint8_t *__restrict__ am) {
  const int64_t total = (int64_t)n * OH * OW * C;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    int c = (int)(i % C);
    int64_t t = i / C;
    int ow = (int)(t % OW); t /= OW;
    int oh = (int)(t % OH);
    int b = (int)(t / OH);
    float best = -INFINITY;
    int bi = -1;
    for (int kh = 0; kh < k; ++kh) {
      int ih = oh * s - p + kh;
      if ((unsigned)ih >= (unsigned)H) continue;
      for (int kw = 0; kw < k; ++kw) {
        int iw = ow * s - p + kw;
        if ((unsigned)iw >= (unsigned)W) continue;
        float v = x[(((int64_t)b * H + ih) * W + iw) * C + c];
        if (bi < 0) bi = kh * k + kw;
        if (v > best || isnan(v)) {
          best = v;
          bi = kh * k + kw;
        }
      }
    }
    y[i] = best;
    am[i] = (uint8_t)bi;
  }
}

__global__ void maxpool_bwd_kernel(int n, int C, int H, int W, int OH, int OW, int k, int s, int p,
                                   const float *__restrict__ dy, const uint8_t *__restrict__ am,
                                   float *__restrict__ dx) {
  const int64_t total = (int64_t)n * H * W * C;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    int c = (int)(i % C);
    int64_t t = i / C;
    int iw = (int)(t % W); t /= W;
    int ih = (int)(t % H);
    int b = (int)(t / H);
    // output rows whose window covers ih: oh*s - p <= ih <= oh*s - p + k - 1
    int oh_lo = std::max(0, (ih + p - (k - 1) + s - 1) / s);
    if (ih + p - (k - 1) < 0) oh_lo = 0;
    int oh_hi = std::min(OH - 1, (ih + p) / s);
    int ow_lo = std::max(0, (iw + p - (k - 1) + s - 1) / s);
    if (iw + p - (k - 1) < 0) ow_lo = 0;
    int ow_hi = std::min(OW - 1, (iw + p) / s);
    float acc = 0.f;
    for (int oh = oh_lo; oh <= oh_hi; ++oh) {
      int kh = ih + p - oh * s;
      if (kh < 0 || kh >= k) continue;
      for (int ow = ow_lo; ow <= ow_hi; ++ow) {
        int kw = iw + p - ow * s;
        if (kw < 0 || kw >= k) continue;
        int64_t o = (((int64_t)b * OH + oh) * OW + ow) * C + c;
        if (am[o] == kh * k + kw) acc += dy[o];
      }
    }
    dx[i] = acc;
  }
}

// Four channels per thread (C % 4 == 0, 16-B aligned tensors, < 2^31 float4 per tensor): the
// same scan order, tie rule and NaN rule as the kernels above, one float4 load per window tap and
// one float4 + uchar4 store (the scalar kernels issue a 4-B access and a 64-bit index division per
// element: DeeplabVGG's 2x2 pools took 1.1 ms per backward launch at c4, 4x their HBM time).
__global__ void __launch_bounds__(256) maxpool_fwd4_kernel(int n, int C4, int H, int W, int OH, int OW, int k, int s,
                                                           int p, FastDiv fd_c4, FastDiv fd_ow, FastDiv fd_oh,
                                                           const float4 *__restrict__ x, float4 *__restrict__ y,
                                                           uchar4 *__restrict__ am, uint2 *__restrict__ yt) {
  const uint32_t total = (uint32_t)n * OH * OW * C4;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const uint32_t t = fdiv(i, fd_c4);
    const int c4 = (int)(i - t * C4);
    const uint32_t t2 = fdiv(t, fd_ow);
    const int ow = (int)(t - t2 * OW);
    const uint32_t b = fdiv(t2, fd_oh);
    const int oh = (int)(t2 - b * OH);
    float best[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
    int bi[4] = {-1, -1, -1, -1};
    for (int kh = 0; kh < k; ++kh) {
      const int ih = oh * s - p + kh;
      if ((unsigned)ih >= (unsigned)H) continue;
      for (int kw = 0; kw < k; ++kw) {
        const int iw = ow * s - p + kw;
        if ((unsigned)iw >= (unsigned)W) continue;
        const float4 v4 = x[((b * H + ih) * W + iw) * C4 + c4];
        const float v[4] = {v4.x, v4.y, v4.z, v4.w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          if (bi[q] < 0) bi[q] = kh * k + kw;
          if (v[q] > best[q] || isnan(v[q])) {
            best[q] = v[q];
            bi[q] = kh * k + kw;
          }
        }
      }
    }
    const float4 yv = make_float4(best[0], best[1], best[2], best[3]);
    y[i] = yv;
    am[i] = make_uchar4((unsigned char)bi[0], (unsigned char)bi[1], (unsigned char)bi[2], (unsigned char)bi[3]);
    if (yt) {   // the pooled value's F32X3 term images [pixel][3][C] (the next conv's operand)
      uint2 h, m, l;
      split3(yv, h, m, l);
      uint2 *o = yt + t * 3 * C4 + c4;
      o[0] = h;
      o[C4] = m;
      o[2 * C4] = l;
    }
  }
}

__global__ void __launch_bounds__(256) maxpool_bwd4_kernel(int n, int C4, int H, int W, int OH, int OW, int k, int s,
                                                           int p, FastDiv fd_c4, FastDiv fd_w, FastDiv fd_h,
                                                           const float4 *__restrict__ dy, const uchar4 *__restrict__ am,
                                                           float4 *__restrict__ dx, uint2 *__restrict__ dxt) {
  const uint32_t total = (uint32_t)n * H * W * C4;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const uint32_t t = fdiv(i, fd_c4);
    const int c4 = (int)(i - t * C4);
    const uint32_t t2 = fdiv(t, fd_w);
    const int iw = (int)(t - t2 * W);
    const uint32_t b = fdiv(t2, fd_h);
    const int ih = (int)(t2 - b * H);
    int oh_lo = (ih + p - (k - 1) + s - 1) / s;
    if (ih + p - (k - 1) < 0) oh_lo = 0;
    const int oh_hi = min(OH - 1, (ih + p) / s);
    int ow_lo = (iw + p - (k - 1) + s - 1) / s;
    if (iw + p - (k - 1) < 0) ow_lo = 0;
    const int ow_hi = min(OW - 1, (iw + p) / s);
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    for (int oh = max(0, oh_lo); oh <= oh_hi; ++oh) {
      const int kh = ih + p - oh * s;
      if (kh < 0 || kh >= k) continue;
      for (int ow = max(0, ow_lo); ow <= ow_hi; ++ow) {
        const int kw = iw + p - ow * s;
        if (kw < 0 || kw >= k) continue;
        const uint32_t o = ((b * OH + oh) * OW + ow) * C4 + c4;
        const uchar4 a = am[o];
        const float4 g = dy[o];
        const unsigned char pos = (unsigned char)(kh * k + kw);
        acc[0] += a.x == pos ? g.x : 0.f;
        acc[1] += a.y == pos ? g.y : 0.f;
        acc[2] += a.z == pos ? g.z : 0.f;
        acc[3] += a.w == pos ? g.w : 0.f;
      }
    }
    const float4 g = make_float4(acc[0], acc[1], acc[2], acc[3]);
    dx[i] = g;
    if (dxt) {   // the routed gradient's term images (the producing conv's weight / data gradients)
      uint2 h, m, l;
      split3(g, h, m, l);
      uint2 *o = dxt + t * 3 * C4 + c4;
      o[0] = h;
      o[C4] = m;
      o[2 * C4] = l;
    }
  }
}

static bool pool_vec(int c, int64_t elems, const void *a, const void *b, const void *am, const void *terms) {
  return c % 4 == 0 && elems / 4 < (1ll << 31) / 3 && !(reinterpret_cast<uintptr_t>(a) & 15) &&
         !(reinterpret_cast<uintptr_t>(b) & 15) && !(reinterpret_cast<uintptr_t>(am) & 3) &&
         !(reinterpret_cast<uintptr_t>(terms) & 7);
}

// ------------------------------------------------------------------------------------
// Bilinear upsample, align_corners=True (torch area_pixel_compute_scale semantics).
// ------------------------------------------------------------------------------------
__device__ __forceinline__ float ac_scale(int in, int out) {
  return out > 1 ? (float)(in - 1) / (float)(out - 1) : 0.f;
}

__device__ __forceinline__ void ac_src(float scale, int dst, int in, int &i0, int &i1, float &l1) {
  float src = scale * (float)dst;
  i0 = (int)src;
  i1 = i0 + ((i0 < in - 1) ? 1 : 0);
  l1 = src - (float)i0;
}

// One thread per output pixel: the bilinear taps are computed once and applied to all C
// channels; the block's 256 pixels x C outputs are staged in LDS (stride C: conflict-free for
// odd C) and written back as one contiguous, coalesced run (NHWC rows are contiguous across
// pixels).  32-bit index math (64-bit division per element made this ALU-bound).
constexpr int kUpPix = 256;
__global__ void __launch_bounds__(kUpPix) upsample_fwd_kernel(int n, int C, int h, int w, int OH, int OW,
                                                              const float *__restrict__ x, float *__restrict__ y) {
  extern __shared__ float so[];
  const float sh = ac_scale(h, OH), sw = ac_scale(w, OW);
  const int npix = n * OH * OW;
  for (int p0 = blockIdx.x * kUpPix; p0 < npix; p0 += gridDim.x * kUpPix) {
    const int p = p0 + (int)threadIdx.x;
    const int cnt = min(kUpPix, npix - p0);
    if (p < npix) {
      const int X = p % OW, t = p / OW;
      const int Y = t % OH, b = t / OH;
      int y0, y1, x0, x1;
      float ly, lx;
      ac_src(sh, Y, h, y0, y1, ly);
      ac_src(sw, X, w, x0, x1, lx);
      const float *base = x + (size_t)b * h * w * C;
      const float *r00 = base + ((size_t)y0 * w + x0) * C, *r01 = base + ((size_t)y0 * w + x1) * C;
      const float *r10 = base + ((size_t)y1 * w + x0) * C, *r11 = base + ((size_t)y1 * w + x1) * C;
      float *o = so + threadIdx.x * C;
      for (int c = 0; c < C; ++c)
        o[c] = (1.f - ly) * ((1.f - lx) * r00[c] + lx * r01[c]) + ly * ((1.f - lx) * r10[c] + lx * r11[c]);
    }
    __syncthreads();
    float *dst = y + (size_t)p0 * C;
    for (int i = threadIdx.x; i < cnt * C; i += kUpPix) dst[i] = so[i];
    __syncthreads();
  }
}

// Candidate range of destination indices D whose source taps can touch index `v`.
__device__ __forceinline__ void ac_range(float scale, int v, int out, int &lo, int &hi) {
  if (scale <= 0.f) {
    lo = 0;
    hi = out - 1;
    return;
  }
  lo = (int)floorf((float)(v - 1) / scale) - 2;
  hi = (int)ceilf((float)(v + 1) / scale) + 2;
  lo = std::max(lo, 0);
  hi = std::min(hi, out - 1);
}

// pass 1: tmp[b][Y][x][c] = sum_X wx(X -> x) * dy[b][Y][X][c].  One thread per element, so a
// wave reads whole NHWC pixel rows of dy (consecutive c, then x) — coalesced; 32-bit index
// math (the caller guarantees n*OH*OW*C < 2^31).
__global__ void upsample_bwd_x_kernel(int n, int C, int w, int OH, int OW, const float *__restrict__ dy,
                                      float *__restrict__ tmp) {
  const float sw = ac_scale(w, OW);
  const int total = n * OH * w * C;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int c = i % C, t = i / C;
    const int xx = t % w, row = t / w;  // row = b*OH + Y
    int lo, hi;
    ac_range(sw, xx, OW, lo, hi);
    const float *g = dy + (size_t)row * OW * C + c;
    float acc = 0.f;
    for (int X = lo; X <= hi; ++X) {
      int x0, x1;
      float lx;
      ac_src(sw, X, w, x0, x1, lx);
      const float wt = (x0 == xx ? 1.f - lx : 0.f) + (x1 == xx ? lx : 0.f);
      if (wt != 0.f) acc += wt * g[X * C];
    }
    tmp[i] = acc;
  }
}

// pass 2: dx[b][y][x][c] (+)= sum_Y wy(Y -> y) * tmp[b][Y][x][c]
__global__ void upsample_bwd_y_kernel(int n, int C, int h, int w, int OH, const float *__restrict__ tmp,
                                      float *__restrict__ dx, int accumulate) {
  const float sh = ac_scale(h, OH);
  const int64_t total = (int64_t)n * h * w * C;
  const int wc = w * C;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int t = (int)(i / wc);            // one 64-bit division (by a loop-invariant)
    const int inner = (int)(i - (int64_t)t * wc);  // x*C + c
    const int yy = t % h, b = t / h;
    int lo, hi;
    ac_range(sh, yy, OH, lo, hi);
    const float *g = tmp + (int64_t)b * OH * w * C + inner;
    float acc = 0.f;
    for (int Y = lo; Y <= hi; ++Y) {
      int y0, y1;
      float ly;
      ac_src(sh, Y, h, y0, y1, ly);
      float wt = (y0 == yy ? 1.f - ly : 0.f) + (y1 == yy ? ly : 0.f);
      if (wt != 0.f) acc += wt * g[(int64_t)Y * w * C];
    }
    dx[i] = accumulate ? dx[i] + acc : acc;
  }
}

// ------------------------------------------------------------------------------------
// Channel softmax over contiguous rows of C.
// ------------------------------------------------------------------------------------
__global__ void softmax_fwd_kernel(int64_t rows, int C, const float *__restrict__ x, float *__restrict__ y) {
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < rows;
       r += (int64_t)gridDim.x * blockDim.x) {
    const float *xr = x + r * C;
    float m = -INFINITY;
    for (int c = 0; c < C; ++c) m = fmaxf(m, xr[c]);
    float s = 0.f;
    for (int c = 0; c < C; ++c) s += __expf(xr[c] - m);
    float inv = 1.f / s;
    float *yr = y + r * C;
    for (int c = 0; c < C; ++c) yr[c] = __expf(xr[c] - m) * inv;
  }
}

__global__ void softmax_bwd_kernel(int64_t rows, int C, const float *__restrict__ y, const float *__restrict__ dy,
                                   float *dx, int accumulate) {
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < rows;
       r += (int64_t)gridDim.x * blockDim.x) {
    const float *yr = y + r * C;
    const float *gr = dy + r * C;
    float dot = 0.f;
    for (int c = 0; c < C; ++c) dot += yr[c] * gr[c];
    float *dr = dx + r * C;
    for (int c = 0; c < C; ++c) {
      float v = yr[c] * (gr[c] - dot);
      dr[c] = accumulate ? dr[c] + v : v;
    }
  }
}

// ------------------------------------------------------------------------------------
// Softmax cross entropy with ignore label.
// ------------------------------------------------------------------------------------
__device__ __forceinline__ bool ce_valid(int64_t lab, int ignore, int C) {
  return lab >= 0 && lab != ignore && lab < C;
}

__global__ void __launch_bounds__(256) ce_fwd_partial_kernel(int64_t rows, int C, const float *__restrict__ logits,
                                                             const int64_t *__restrict__ labels, int ignore,
                                                             const float *__restrict__ cw, float *partial) {
  float num = 0.f, den = 0.f;
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < rows;
       r += (int64_t)gridDim.x * blockDim.x) {
    int64_t lab = labels[r];
    if (!ce_valid(lab, ignore, C)) continue;
    const float *xr = logits + r * C;
    float m = -INFINITY;
    for (int c = 0; c < C; ++c) m = fmaxf(m, xr[c]);
    float s = 0.f;
    for (int c = 0; c < C; ++c) s += __expf(xr[c] - m);
    float nll = m + __logf(s) - xr[lab];
    float wt = cw ? cw[lab] : 1.f;
    num += wt * nll;
    den += wt;
  }
  __shared__ float sn[256], sd[256];
  sn[threadIdx.x] = num;
  sd[threadIdx.x] = den;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) {
      sn[threadIdx.x] += sn[threadIdx.x + o];
      sd[threadIdx.x] += sd[threadIdx.x + o];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    partial[2 * blockIdx.x] = sn[0];
    partial[2 * blockIdx.x + 1] = sd[0];
  }
}

__global__ void pair_final_kernel(const float *partial, int nparts, float *out, int mode, double scale) {
  // mode 0: out[0] = num/den, out[1] = den (CE);  mode 1: out[0] = num*scale (mean losses).
  // One wave: lanes take strided partials (independent loads, fp64), then a fixed shuffle
  // tree — deterministic (a single serial thread spent ~36 us on 2048 dependent loads).
  const int lane = threadIdx.x & 63;
  if (threadIdx.x >= 64 || blockIdx.x != 0) return;
  double num = 0, den = 0;
  for (int i = lane; i < nparts; i += 64) {
    num += partial[2 * i];
    den += partial[2 * i + 1];
  }
  for (int o = 32; o > 0; o >>= 1) {
    num += __shfl_xor(num, o);
    den += __shfl_xor(den, o);
  }
  if (lane != 0) return;
  if (mode == 0) {
    out[0] = (float)(num / den);
    out[1] = (float)den;
  } else {
    out[0] = (float)(num * scale);
  }
}

__global__ void ce_bwd_kernel(int64_t rows, int C, const float *__restrict__ logits, const int64_t *__restrict__ labels,
                              int ignore, const float *__restrict__ cw, const float *__restrict__ out,
                              const float *__restrict__ grad_loss, float *dl, int accumulate) {
  const float scale = grad_loss[0] / out[1];
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < rows;
       r += (int64_t)gridDim.x * blockDim.x) {
    int64_t lab = labels[r];
    float *dr = dl + r * C;
    if (!ce_valid(lab, ignore, C)) {
      if (!accumulate)
        for (int c = 0; c < C; ++c) dr[c] = 0.f;
      continue;
    }
    const float *xr = logits + r * C;
    float m = -INFINITY;
    for (int c = 0; c < C; ++c) m = fmaxf(m, xr[c]);
    float s = 0.f;
    for (int c = 0; c < C; ++c) s += __expf(xr[c] - m);
    float inv = 1.f / s;
    float k = scale * (cw ? cw[lab] : 1.f);
    for (int c = 0; c < C; ++c) {
      float v = k * (__expf(xr[c] - m) * inv - (c == lab ? 1.f : 0.f));
      dr[c] = accumulate ? dr[c] + v : v;
    }
  }
}

// ------------------------------------------------------------------------------------
// LDS-tiled row kernels for C <= kRowTileMaxC (the 19-class maps of the hot path).  A block
// stages kRowTile consecutive rows (kRowTile*C contiguous floats) with coalesced loads, each
// thread then owns one row in LDS (stride C odd -> conflict-free for C = 19), and the result is
// written back through LDS with coalesced stores.  Per-thread-row global access (76-byte
// strided rows) was ~10x off the HBM roofline.
// ------------------------------------------------------------------------------------
constexpr int kRowTile = 256;
constexpr int kRowTileMaxC = 32;

// Tile copies HBM <-> LDS.  (A float4 / 8-deep batched variant measured slower here:
// softmax fwd 74 -> 108 us, CE bwd 72 -> 117 us at c2.)
__device__ __forceinline__ void tile_load(float *sm, const float *__restrict__ src, int n) {
  for (int i = threadIdx.x; i < n; i += blockDim.x) sm[i] = src[i];
}

__device__ __forceinline__ void tile_store(float *dst, const float *sm, int n, int accumulate) {
  if (accumulate)
    for (int i = threadIdx.x; i < n; i += blockDim.x) dst[i] += sm[i];
  else
    for (int i = threadIdx.x; i < n; i += blockDim.x) dst[i] = sm[i];
}

__global__ void __launch_bounds__(kRowTile) softmax_fwd_tiled_kernel(int64_t rows, int C, const float *__restrict__ x,
                                                                  float *__restrict__ y) {
  extern __shared__ float sm[];
  for (int64_t r0 = (int64_t)blockIdx.x * kRowTile; r0 < rows; r0 += (int64_t)gridDim.x * kRowTile) {
    const int nr = (int)min<int64_t>(kRowTile, rows - r0);
    const int n = nr * C;
    tile_load(sm, x + r0 * C, n);
    __syncthreads();
    if ((int)threadIdx.x < nr) {
      float *v = sm + threadIdx.x * C;
      float m = -INFINITY;
      for (int c = 0; c < C; ++c) m = fmaxf(m, v[c]);
      float s = 0.f;
      for (int c = 0; c < C; ++c) {
        const float e = __expf(v[c] - m);
        v[c] = e;
        s += e;
      }
      const float inv = 1.f / s;
      for (int c = 0; c < C; ++c) v[c] *= inv;
    }
    __syncthreads();
    tile_store(y + r0 * C, sm, n, 0);
    __syncthreads();
  }
}

__global__ void __launch_bounds__(kRowTile) softmax_bwd_tiled_kernel(int64_t rows, int C, const float *__restrict__ y,
                                                                  const float *__restrict__ dy, float *dx,
                                                                  int accumulate) {
  extern __shared__ float sm[];
  float *sg = sm + kRowTile * C;
  for (int64_t r0 = (int64_t)blockIdx.x * kRowTile; r0 < rows; r0 += (int64_t)gridDim.x * kRowTile) {
    const int nr = (int)min<int64_t>(kRowTile, rows - r0);
    const int n = nr * C;
    tile_load(sm, y + r0 * C, n);
    tile_load(sg, dy + r0 * C, n);
    __syncthreads();
    if ((int)threadIdx.x < nr) {
      float *yv = sm + threadIdx.x * C;
      const float *gv = sg + threadIdx.x * C;
      float dot = 0.f;
      for (int c = 0; c < C; ++c) dot += yv[c] * gv[c];
      for (int c = 0; c < C; ++c) yv[c] = yv[c] * (gv[c] - dot);
    }
    __syncthreads();
    tile_store(dx + r0 * C, sm, n, accumulate);
    __syncthreads();
  }
}

__global__ void __launch_bounds__(kRowTile) ce_fwd_tiled_kernel(int64_t rows, int C, const float *__restrict__ logits,
                                                             const int64_t *__restrict__ labels, int ignore,
                                                             const float *__restrict__ cw, float *partial) {
  extern __shared__ float sm[];
  __shared__ float sn[kRowTile / 64], sd[kRowTile / 64];
  float num = 0.f, den = 0.f;
  for (int64_t r0 = (int64_t)blockIdx.x * kRowTile; r0 < rows; r0 += (int64_t)gridDim.x * kRowTile) {
    const int nr = (int)min<int64_t>(kRowTile, rows - r0);
    tile_load(sm, logits + r0 * C, nr * C);
    const int64_t lab = (int)threadIdx.x < nr ? labels[r0 + threadIdx.x] : -1;
    __syncthreads();
    if ((int)threadIdx.x < nr && ce_valid(lab, ignore, C)) {
      const float *v = sm + threadIdx.x * C;
      float m = -INFINITY;
      for (int c = 0; c < C; ++c) m = fmaxf(m, v[c]);
      float s = 0.f;
      for (int c = 0; c < C; ++c) s += __expf(v[c] - m);
      const float wt = cw ? cw[lab] : 1.f;
      num += wt * (m + __logf(s) - v[lab]);
      den += wt;
    }
    __syncthreads();
  }
  for (int o = 32; o > 0; o >>= 1) {
    num += __shfl_xor(num, o);
    den += __shfl_xor(den, o);
  }
  if ((threadIdx.x & 63) == 0) {
    sn[threadIdx.x >> 6] = num;
    sd[threadIdx.x >> 6] = den;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float a = 0.f, b = 0.f;
    for (int i = 0; i < kRowTile / 64; ++i) {
      a += sn[i];
      b += sd[i];
    }
    partial[2 * blockIdx.x] = a;
    partial[2 * blockIdx.x + 1] = b;
  }
}

__global__ void __launch_bounds__(kRowTile) ce_bwd_tiled_kernel(int64_t rows, int C, const float *__restrict__ logits,
                                                             const int64_t *__restrict__ labels, int ignore,
                                                             const float *__restrict__ cw, const float *__restrict__ out,
                                                             const float *__restrict__ grad_loss, float *dl,
                                                             int accumulate) {
  extern __shared__ float sm[];
  const float scale = grad_loss[0] / out[1];
  for (int64_t r0 = (int64_t)blockIdx.x * kRowTile; r0 < rows; r0 += (int64_t)gridDim.x * kRowTile) {
    const int nr = (int)min<int64_t>(kRowTile, rows - r0);
    const int n = nr * C;
    tile_load(sm, logits + r0 * C, n);
    const int64_t lab = (int)threadIdx.x < nr ? labels[r0 + threadIdx.x] : -1;
    __syncthreads();
    if ((int)threadIdx.x < nr) {
      float *v = sm + threadIdx.x * C;
      if (!ce_valid(lab, ignore, C)) {
        for (int c = 0; c < C; ++c) v[c] = 0.f;
      } else {
        float m = -INFINITY;
        for (int c = 0; c < C; ++c) m = fmaxf(m, v[c]);
        float s = 0.f;
        for (int c = 0; c < C; ++c) {
          const float e = __expf(v[c] - m);
          v[c] = e;
          s += e;
        }
        const float k = scale * (cw ? cw[lab] : 1.f) / s;
        const float kl = scale * (cw ? cw[lab] : 1.f);
        for (int c = 0; c < C; ++c) v[c] = v[c] * k - (c == lab ? kl : 0.f);
      }
    }
    __syncthreads();
    tile_store(dl + r0 * C, sm, n, accumulate);
    __syncthreads();
  }
}

// ------------------------------------------------------------------------------------
// Adversarial losses vs constant target t.
// ------------------------------------------------------------------------------------
__device__ __forceinline__ float adv_elem(float x, float t, int kind) {
  if (kind == 0) {
    // BCEWithLogits: (1-t)*x + max(-x,0) + log(exp(-max(-x,0)) + exp(-x-max(-x,0)))
    float mv = fmaxf(-x, 0.f);
    return (1.f - t) * x + mv + __logf(__expf(-mv) + __expf(-x - mv));
  }
  float d = x - t;
  return d * d;
}

__global__ void __launch_bounds__(256) adv_fwd_partial_kernel(int64_t n, const float *__restrict__ x, float t,
                                                              int kind, float *partial) {
  float s = 0.f;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    s += adv_elem(x[i], t, kind);
  __shared__ float sh[256];
  sh[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) sh[threadIdx.x] += sh[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    partial[2 * blockIdx.x] = sh[0];
    partial[2 * blockIdx.x + 1] = 0.f;
  }
}

__global__ void adv_bwd_kernel(int64_t n, const float *__restrict__ x, float t, int kind,
                               const float *__restrict__ grad_loss, float *dx, int accumulate) {
  const float g = grad_loss[0] / (float)n;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    float xi = x[i];
    float d = kind == 0 ? (1.f / (1.f + __expf(-xi)) - t) : 2.f * (xi - t);
    float v = g * d;
    dx[i] = accumulate ? dx[i] + v : v;
  }
}

// ------------------------------------------------------------------------------------
// Optimisers over flat arenas.
// ------------------------------------------------------------------------------------
__global__ void sgd_kernel(int64_t n, float *__restrict__ p, const float *__restrict__ g, float *__restrict__ buf,
                           float lr, float mom, float wd, float gs, int mult, int first) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    float pi = p[i];
    const float gi = g[i] * gs;
    float b = buf[i];
    for (int r = 0; r < mult; ++r) {
      float d = gi + wd * pi;         // grad.add(param, alpha=wd)
      b = first ? d : b * mom + d;    // clone on first step, else buf.mul_(m).add_(d)
      pi = pi - lr * b;               // param.add_(buf, alpha=-lr)
    }
    buf[i] = b;
    p[i] = pi;
  }
}

__global__ void adam_kernel(int64_t n, float *__restrict__ p, const float *__restrict__ g, float *__restrict__ m,
                            float *__restrict__ v, float b1, float b2, float eps, float step_size, float bc2_sqrt,
                            float gs) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    float gi = g[i] * gs;
    float mi = m[i];
    mi = mi + (1.f - b1) * (gi - mi);  // torch lerp_ (weight < 0.5 branch)
    float vi = v[i] * b2 + (1.f - b2) * gi * gi;
    m[i] = mi;
    v[i] = vi;
    float denom = sqrtf(vi) / bc2_sqrt + eps;
    p[i] = p[i] - step_size * (mi / denom);
  }
}

// ------------------------------------------------------------------------------------
// Plumbing.
// ------------------------------------------------------------------------------------
struct Strides4 {
  int64_t s[4];
};

// dst[b][y][x][c] (Cd channels, Cd >= C) = c < C ? src(b, c, y, x) : 0, (+ dst with ACC)
template <bool ACC>
__global__ void to_nhwc_kernel(int n, int C, int Cd, int H, int W, Strides4 st, const float *__restrict__ src,
                               float *__restrict__ dst) {
  const int64_t total = (int64_t)n * Cd * H * W;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    int c = (int)(i % Cd);
    int64_t t = i / Cd;
    int x = (int)(t % W); t /= W;
    int y = (int)(t % H);
    int b = (int)(t / H);
    const float v = c < C ? src[b * st.s[0] + c * st.s[1] + y * st.s[2] + x * st.s[3]] : 0.f;
    dst[i] = ACC ? dst[i] + v : v;
  }
}

// Same transform, c_dst % 4 == 0: a block row per (image, y), a thread per (x, 4 output channels)
// (one float4 store, 32-bit index math) — the thin convs' input pads run on this one.
template <bool ACC>
__global__ void to_nhwc4_kernel(int C, int Cd, int H, int W, Strides4 st, const float *__restrict__ src,
                                float *__restrict__ dst) {
  const int Q = Cd >> 2;
  const int row = blockIdx.y, b = row / H, y = row - b * H;
  const int64_t base_row = (int64_t)b * st.s[0] + (int64_t)y * st.s[2];
  float4 *drow = reinterpret_cast<float4 *>(dst) + (int64_t)row * W * Q;
  for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < W * Q; t += gridDim.x * blockDim.x) {
    const int x = t / Q, q = t - x * Q;
    const float *sp = src + base_row + (int64_t)x * st.s[3];
    float v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = 4 * q + j;
      v[j] = c < C ? sp[(int64_t)c * st.s[1]] : 0.f;
    }
    float4 o = make_float4(v[0], v[1], v[2], v[3]);
    if (ACC) {
      const float4 d = drow[t];
      o.x += d.x; o.y += d.y; o.z += d.z; o.w += d.w;
    }
    drow[t] = o;
  }
}

__global__ void add_i64_kernel(int64_t *p, int64_t n, int64_t v) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    p[i] += v;
}

__global__ void axpy_kernel(int64_t n, float a, const float *__restrict__ src, float *dst, int accumulate) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    dst[i] = accumulate ? dst[i] + a * src[i] : a * src[i];
}

// ------------------------------------------------------------------------------------
// Evaluation (evaluate_cityscapes.py:153-169, compute_iou.py:15-28).
// ------------------------------------------------------------------------------------
// interp(logits) to OHxOW (align_corners=True) fused with the class argmax: one thread per
// output pixel interpolates its C class scores from the 4 source rows (L2-resident: the
// low-res map is ~2.5 MB) and writes one byte.  First maximal class wins; a NaN score wins
// over numbers (torch.argmax / np.argmax semantics).
__global__ void upsample_argmax_kernel(int n, int C, int h, int w, int OH, int OW, const float *__restrict__ x,
                                       uint8_t *__restrict__ out) {
  const float sh = ac_scale(h, OH), sw = ac_scale(w, OW);
  const int64_t total = (int64_t)n * OH * OW;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int X = (int)(i % OW);
    const int64_t t = i / OW;
    const int Y = (int)(t % OH), b = (int)(t / OH);
    int y0, y1, x0, x1;
    float ly, lx;
    ac_src(sh, Y, h, y0, y1, ly);
    ac_src(sw, X, w, x0, x1, lx);
    const float *base = x + (int64_t)b * h * w * C;
    const float *r00 = base + ((int64_t)y0 * w + x0) * C, *r01 = base + ((int64_t)y0 * w + x1) * C;
    const float *r10 = base + ((int64_t)y1 * w + x0) * C, *r11 = base + ((int64_t)y1 * w + x1) * C;
    float best = 0.f;
    int arg = 0;
    for (int c = 0; c < C; ++c) {
      const float v = (1.f - ly) * ((1.f - lx) * r00[c] + lx * r01[c]) + ly * ((1.f - lx) * r10[c] + lx * r11[c]);
      if (c == 0 || (!isnan(best) && (v > best || isnan(v)))) {
        best = v;
        arg = c;
      }
    }
    out[i] = (uint8_t)arg;
  }
}

// hist[gt][pred] += 1 over pixels whose (LUT-mapped) label is in [0, n): compute_iou's
// label_mapping + fast_hist.  Per-block LDS bins, then one 64-bit atomic per non-zero bin
// (integer adds: the result is exact and order-independent).
__global__ void __launch_bounds__(256) confusion_hist_kernel(int64_t npix, const uint8_t *__restrict__ gt,
                                                             const int *__restrict__ lut,
                                                             const uint8_t *__restrict__ pred, int n,
                                                             unsigned long long *hist) {
  extern __shared__ unsigned int bins[];
  const int nb = n * n;
  for (int j = threadIdx.x; j < nb; j += blockDim.x) bins[j] = 0u;
  __syncthreads();
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < npix;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int a = lut ? lut[gt[i]] : (int)gt[i];
    const int b = pred[i];
    if (a >= 0 && a < n && b < n) atomicAdd(&bins[a * n + b], 1u);
  }
  __syncthreads();
  for (int j = threadIdx.x; j < nb; j += blockDim.x)
    if (bins[j]) atomicAdd(&hist[j], (unsigned long long)bins[j]);
}

}  // namespace adaptseg

using namespace adaptseg;

extern "C" {

int adaptseg_upsample_argmax(int n, int c, int h, int w, int oh, int ow, const float *x, uint8_t *out,
                             adaptseg_stream_t stream) {
  AS_CHECK_ARG(n > 0 && c > 0 && c <= 256 && h > 0 && w > 0 && oh > 0 && ow > 0 && x && out,
               "upsample_argmax: bad args");
  const int64_t total = (int64_t)n * oh * ow;
  upsample_argmax_kernel<<<grid1d(total), 256, 0, as_stream(stream)>>>(n, c, h, w, oh, ow, x, out);
  AS_CHECK_LAUNCH("upsample_argmax");
  return ADAPTSEG_OK;
}

int adaptseg_confusion_hist(int64_t npix, const uint8_t *gt, const int32_t *lut, const uint8_t *pred, int ncls,
                            int64_t *hist, adaptseg_stream_t stream) {
  AS_CHECK_ARG(npix >= 0 && ncls > 0 && ncls <= 128 && hist && (npix == 0 || (gt && pred)),
               "confusion_hist: bad args");
  if (npix == 0) return ADAPTSEG_OK;
  const int blocks = grid1d(npix, 256 * 16, 1024);
  confusion_hist_kernel<<<blocks, 256, (size_t)ncls * ncls * sizeof(unsigned int), as_stream(stream)>>>(
      npix, gt, lut, pred, ncls, reinterpret_cast<unsigned long long *>(hist));
  AS_CHECK_LAUNCH("confusion_hist");
  return ADAPTSEG_OK;
}


const char *adaptseg_last_error(void) { return g_err; }
const char *adaptseg_version(void) { return "adaptseg 0.5 gfx950"; }

int adaptseg_maxpool2d_fwd(int n, int c, int h, int w, int oh, int ow, int k, int s, int p, const float *x,
                           float *y, uint8_t *argmax, adaptseg_stream_t stream) {
  return adaptseg_maxpool2d_fwd_x(n, c, h, w, oh, ow, k, s, p, x, y, argmax, nullptr, stream);
}

int adaptseg_maxpool2d_fwd_x(int n, int c, int h, int w, int oh, int ow, int k, int s, int p, const float *x,
                             float *y, uint8_t *argmax, uint16_t *y_terms, adaptseg_stream_t stream) {
  AS_CHECK_ARG(n > 0 && c > 0 && h > 0 && w > 0 && oh > 0 && ow > 0 && k > 0 && k * k <= 255 && s > 0 && p >= 0,
               "maxpool_fwd: bad geometry");
  AS_CHECK_ARG(x && y && argmax, "maxpool_fwd: null pointer");
  AS_CHECK_ARG((h + 2 * p - k) / s + 1 == oh && (w + 2 * p - k) / s + 1 == ow, "maxpool_fwd: output size mismatch");
  int64_t total = (int64_t)n * oh * ow * c;
  const bool vec = pool_vec(c, std::max<int64_t>(total, (int64_t)n * h * w * c), x, y, argmax, y_terms);
  AS_CHECK_ARG(vec || !y_terms, "maxpool_fwd: term images need C %% 4 == 0 and aligned tensors");
  if (vec) {
    const int c4 = c / 4;
    maxpool_fwd4_kernel<<<grid1d(total / 4, 256, 16384), 256, 0, as_stream(stream)>>>(
        n, c4, h, w, oh, ow, k, s, p, make_fastdiv(c4), make_fastdiv(ow), make_fastdiv(oh),
        reinterpret_cast<const float4 *>(x), reinterpret_cast<float4 *>(y), reinterpret_cast<uchar4 *>(argmax),
        reinterpret_cast<uint2 *>(y_terms));
  } else {
    maxpool_fwd_kernel<<<grid1d(total), 256, 0, as_stream(stream)>>>(n, c, h, w, oh, ow, k, s, p, x, y, argmax);
  }
  AS_CHECK_LAUNCH("maxpool_fwd");
  return ADAPTSEG_OK;
}

int adaptseg_maxpool2d_bwd(int n, int c, int h, int w, int oh, int ow, int k, int s, int p, const float *dy,
                           const uint8_t *argmax, float *dx, adaptseg_stream_t stream) {
  return adaptseg_maxpool2d_bwd_x(n, c, h, w, oh, ow, k, s, p, dy, argmax, dx, nullptr, stream);
}

int adaptseg_maxpool2d_bwd_x(int n, int c, int h, int w, int oh, int ow, int k, int s, int p, const float *dy,
                             const uint8_t *argmax, float *dx, uint16_t *dx_terms, adaptseg_stream_t stream) {
  AS_CHECK_ARG(n > 0 && c > 0 && h > 0 && w > 0 && oh > 0 && ow > 0 && k > 0 && s > 0 && p >= 0,
               "maxpool_bwd: bad geometry");
  AS_CHECK_ARG(dy && argmax && dx, "maxpool_bwd: null pointer");
  int64_t total = (int64_t)n * h * w * c;
  const bool vec = pool_vec(c, total, dy, dx, argmax, dx_terms);
  AS_CHECK_ARG(vec || !dx_terms, "maxpool_bwd: term images need C %% 4 == 0 and aligned tensors");
  if (vec) {
    const int c4 = c / 4;
    maxpool_bwd4_kernel<<<grid1d(total / 4, 256, 16384), 256, 0, as_stream(stream)>>>(
        n, c4, h, w, oh, ow, k, s, p, make_fastdiv(c4), make_fastdiv(w), make_fastdiv(h),
        reinterpret_cast<const float4 *>(dy), reinterpret_cast<const uchar4 *>(argmax), reinterpret_cast<float4 *>(dx),
        reinterpret_cast<uint2 *>(dx_terms));
  } else {
    maxpool_bwd_kernel<<<grid1d(total), 256, 0, as_stream(stream)>>>(n, c, h, w, oh, ow, k, s, p, dy, argmax, dx);
  }
  AS_CHECK_LAUNCH("maxpool_bwd");
  return ADAPTSEG_OK;
}

int adaptseg_upsample_workspace_size(int n, int c, int h, int w, int oh, int ow, size_t *bytes) {
  AS_CHECK_ARG(bytes && n > 0 && c > 0 && h > 0 && w > 0 && oh > 0 && ow > 0, "upsample_workspace_size: bad args");
  *bytes = (size_t)n * oh * w * c * sizeof(float);
  return ADAPTSEG_OK;
}

int adaptseg_upsample_bilinear_fwd(int n, int c, int h, int w, int oh, int ow, const float *x, float *y,
                                   adaptseg_stream_t stream) {
  AS_CHECK_ARG(n > 0 && c > 0 && h > 0 && w > 0 && oh > 0 && ow > 0, "upsample_fwd: bad geometry");
  AS_CHECK_ARG(c <= 64, "upsample_fwd: at most 64 channels (class-score maps); got %d", c);
  AS_CHECK_ARG((int64_t)n * oh * ow < (1ll << 31), "upsample_fwd: too many output pixels");
  AS_CHECK_ARG(x && y, "upsample_fwd: null pointer");
  int64_t total = (int64_t)n * oh * ow * c;
  int slot;
  timing_begin(kTUpsampleFwd, as_stream(stream), 4.0 * n * c * ((double)h * w + (double)oh * ow), &slot);
  (void)total;
  const int npix = n * oh * ow;
  upsample_fwd_kernel<<<grid1d(npix, kUpPix, 8192), kUpPix, kUpPix * c * sizeof(float), as_stream(stream)>>>(
      n, c, h, w, oh, ow, x, y);
  timing_end(slot, as_stream(stream));
  AS_CHECK_LAUNCH("upsample_fwd");
  return ADAPTSEG_OK;
}

int adaptseg_upsample_bilinear_bwd(int n, int c, int h, int w, int oh, int ow, const float *dy, float *dx, int flags,
                                   void *ws, size_t ws_bytes, adaptseg_stream_t stream) {
  AS_CHECK_ARG(n > 0 && c > 0 && h > 0 && w > 0 && oh > 0 && ow > 0, "upsample_bwd: bad geometry");
  AS_CHECK_ARG(c <= 64, "upsample_bwd: at most 64 channels (class-score maps); got %d", c);
  AS_CHECK_ARG((int64_t)n * oh * ow * c < (1ll << 31), "upsample_bwd: tensor too large for 32-bit indexing");
  AS_CHECK_ARG(dy && dx, "upsample_bwd: null pointer");
  size_t need = (size_t)n * oh * w * c * sizeof(float);
  if (!ws || ws_bytes < need) {
    set_error("upsample_bwd: workspace %zu < %zu", ws_bytes, need);
    return ADAPTSEG_ERR_WORKSPACE;
  }
  hipStream_t s = as_stream(stream);
  float *tmp = reinterpret_cast<float *>(ws);
  int64_t t1 = (int64_t)n * oh * w * c;
  int slot;  // algorithmic bytes: read dy, write dx (the row pass's intermediate is not counted)
  timing_begin(kTUpsampleBwd, s, 4.0 * n * c * ((double)h * w + (double)oh * ow), &slot);
  upsample_bwd_x_kernel<<<grid1d(t1), 256, 0, s>>>(n, c, w, oh, ow, dy, tmp);
  AS_CHECK_LAUNCH("upsample_bwd_x");
  int64_t t2 = (int64_t)n * h * w * c;
  upsample_bwd_y_kernel<<<grid1d(t2), 256, 0, s>>>(n, c, h, w, oh, tmp, dx,
                                                    (flags & ADAPTSEG_EPI_ACCUMULATE) ? 1 : 0);
  timing_end(slot, s);
  AS_CHECK_LAUNCH("upsample_bwd_y");
  return ADAPTSEG_OK;
}

int adaptseg_softmax_fwd(int64_t rows, int c, const float *x, float *y, adaptseg_stream_t stream) {
  AS_CHECK_ARG(rows > 0 && c > 0 && x && y, "softmax_fwd: bad args");
  int slot;
  timing_begin(kTSoftmaxFwd, as_stream(stream), 8.0 * rows * c, &slot);
  if (c <= kRowTileMaxC)
    softmax_fwd_tiled_kernel<<<grid1d(rows, kRowTile, 8192), kRowTile, kRowTile * c * sizeof(float),
                               as_stream(stream)>>>(rows, c, x, y);
  else
    softmax_fwd_kernel<<<grid1d(rows), 256, 0, as_stream(stream)>>>(rows, c, x, y);
  timing_end(slot, as_stream(stream));
  AS_CHECK_LAUNCH("softmax_fwd");
  return ADAPTSEG_OK;
}

int adaptseg_softmax_bwd(int64_t rows, int c, const float *y, const float *dy, float *dx, int flags,
                         adaptseg_stream_t stream) {
  AS_CHECK_ARG(rows > 0 && c > 0 && y && dy && dx, "softmax_bwd: bad args");
  int slot;
  timing_begin(kTSoftmaxBwd, as_stream(stream), 12.0 * rows * c, &slot);
  if (c <= kRowTileMaxC)
    softmax_bwd_tiled_kernel<<<grid1d(rows, kRowTile, 8192), kRowTile, 2 * kRowTile * c * sizeof(float),
                               as_stream(stream)>>>(rows, c, y, dy, dx, (flags & ADAPTSEG_EPI_ACCUMULATE) ? 1 : 0);
  else
    softmax_bwd_kernel<<<grid1d(rows), 256, 0, as_stream(stream)>>>(rows, c, y, dy, dx,
                                                                    (flags & ADAPTSEG_EPI_ACCUMULATE) ? 1 : 0);
  timing_end(slot, as_stream(stream));
  AS_CHECK_LAUNCH("softmax_bwd");
  return ADAPTSEG_OK;
}

static int ce_parts(int64_t rows) { return grid1d(rows, 256 * 4, 2048); }

int adaptseg_ce_workspace_size(int64_t rows, size_t *bytes) {
  AS_CHECK_ARG(bytes && rows > 0, "ce_workspace_size: bad args");
  *bytes = (size_t)ce_parts(rows) * 2 * sizeof(float);
  return ADAPTSEG_OK;
}

int adaptseg_softmax_ce_fwd(int64_t rows, int c, const float *logits, const int64_t *labels, int ignore,
                            const float *class_weight, float *out, void *ws, size_t ws_bytes,
                            adaptseg_stream_t stream) {
  AS_CHECK_ARG(rows > 0 && c > 0 && logits && labels && out, "softmax_ce_fwd: bad args");
  int parts = ce_parts(rows);
  if (!ws || ws_bytes < (size_t)parts * 2 * sizeof(float)) {
    set_error("softmax_ce_fwd: workspace too small");
    return ADAPTSEG_ERR_WORKSPACE;
  }
  hipStream_t s = as_stream(stream);
  float *partial = reinterpret_cast<float *>(ws);
  int slot;  // logits + int64 labels
  timing_begin(kTCeFwd, s, 4.0 * rows * c + 8.0 * rows, &slot);
  if (c <= kRowTileMaxC)
    ce_fwd_tiled_kernel<<<parts, kRowTile, kRowTile * c * sizeof(float), s>>>(rows, c, logits, labels, ignore,
                                                                            class_weight, partial);
  else
    ce_fwd_partial_kernel<<<parts, 256, 0, s>>>(rows, c, logits, labels, ignore, class_weight, partial);
  AS_CHECK_LAUNCH("ce_fwd_partial");
  pair_final_kernel<<<1, 64, 0, s>>>(partial, parts, out, 0, 1.0);
  timing_end(slot, s);
  AS_CHECK_LAUNCH("ce_final");
  return ADAPTSEG_OK;
}

int adaptseg_softmax_ce_bwd(int64_t rows, int c, const float *logits, const int64_t *labels, int ignore,
                            const float *class_weight, const float *out, const float *grad_loss, float *dlogits,
                            int flags, adaptseg_stream_t stream) {
  AS_CHECK_ARG(rows > 0 && c > 0 && logits && labels && out && grad_loss && dlogits, "softmax_ce_bwd: bad args");
  int slot;  // logits + labels in, dlogits out
  timing_begin(kTCeBwd, as_stream(stream), 8.0 * rows * c + 8.0 * rows, &slot);
  if (c <= kRowTileMaxC)
    ce_bwd_tiled_kernel<<<grid1d(rows, kRowTile, 8192), kRowTile, kRowTile * c * sizeof(float),
                          as_stream(stream)>>>(rows, c, logits, labels, ignore, class_weight, out, grad_loss,
                                               dlogits, (flags & ADAPTSEG_EPI_ACCUMULATE) ? 1 : 0);
  else
    ce_bwd_kernel<<<grid1d(rows), 256, 0, as_stream(stream)>>>(rows, c, logits, labels, ignore, class_weight, out,
                                                               grad_loss, dlogits,
                                                               (flags & ADAPTSEG_EPI_ACCUMULATE) ? 1 : 0);
  timing_end(slot, as_stream(stream));
  AS_CHECK_LAUNCH("ce_bwd");
  return ADAPTSEG_OK;
}

static int adv_parts(int64_t n) { return grid1d(n, 256 * 4, 256); }

int adaptseg_adv_workspace_size(int64_t n, size_t *bytes) {
  AS_CHECK_ARG(bytes && n > 0, "adv_workspace_size: bad args");
  *bytes = (size_t)adv_parts(n) * 2 * sizeof(float);
  return ADAPTSEG_OK;
}

int adaptseg_adv_loss_fwd(int64_t n, const float *x, float target, int kind, float *loss, void *ws,
                          size_t ws_bytes, adaptseg_stream_t stream) {
  AS_CHECK_ARG(n > 0 && x && loss && (kind == 0 || kind == 1), "adv_loss_fwd: bad args");
  int parts = adv_parts(n);
  if (!ws || ws_bytes < (size_t)parts * 2 * sizeof(float)) {
    set_error("adv_loss_fwd: workspace too small");
    return ADAPTSEG_ERR_WORKSPACE;
  }
  hipStream_t s = as_stream(stream);
  float *partial = reinterpret_cast<float *>(ws);
  adv_fwd_partial_kernel<<<parts, 256, 0, s>>>(n, x, target, kind, partial);
  AS_CHECK_LAUNCH("adv_fwd_partial");
  pair_final_kernel<<<1, 64, 0, s>>>(partial, parts, loss, 1, 1.0 / (double)n);
  AS_CHECK_LAUNCH("adv_final");
  return ADAPTSEG_OK;
}

int adaptseg_adv_loss_bwd(int64_t n, const float *x, float target, int kind, const float *grad_loss, float *dx,
                          int flags, adaptseg_stream_t stream) {
  AS_CHECK_ARG(n > 0 && x && grad_loss && dx && (kind == 0 || kind == 1), "adv_loss_bwd: bad args");
  adv_bwd_kernel<<<grid1d(n), 256, 0, as_stream(stream)>>>(n, x, target, kind, grad_loss, dx,
                                                           (flags & ADAPTSEG_EPI_ACCUMULATE) ? 1 : 0);
  AS_CHECK_LAUNCH("adv_bwd");
  return ADAPTSEG_OK;
}

int adaptseg_sgd_step(int64_t n, float *param, const float *grad, float *mom, float lr, float momentum,
                      float weight_decay, float grad_scale, int multiplicity, int first_step,
                      adaptseg_stream_t stream) {
  AS_CHECK_ARG(n >= 0 && (n == 0 || (param && grad && mom)) && multiplicity >= 1, "sgd_step: bad args");
  if (n == 0) return ADAPTSEG_OK;
  sgd_kernel<<<grid1d(n), 256, 0, as_stream(stream)>>>(n, param, grad, mom, lr, momentum, weight_decay, grad_scale,
                                                       multiplicity, first_step ? 1 : 0);
  AS_CHECK_LAUNCH("sgd");
  return ADAPTSEG_OK;
}

int adaptseg_adam_step(int64_t n, float *param, const float *grad, float *exp_avg, float *exp_avg_sq, float lr,
                       float beta1, float beta2, float eps, int step, float grad_scale, adaptseg_stream_t stream) {
  AS_CHECK_ARG(n >= 0 && step >= 1 && (n == 0 || (param && grad && exp_avg && exp_avg_sq)), "adam_step: bad args");
  if (n == 0) return ADAPTSEG_OK;
  double bc1 = 1.0 - std::pow((double)beta1, step);
  double bc2 = 1.0 - std::pow((double)beta2, step);
  float step_size = (float)((double)lr / bc1);
  float bc2_sqrt = (float)std::sqrt(bc2);
  adam_kernel<<<grid1d(n), 256, 0, as_stream(stream)>>>(n, param, grad, exp_avg, exp_avg_sq, beta1, beta2, eps,
                                                        step_size, bc2_sqrt, grad_scale);
  AS_CHECK_LAUNCH("adam");
  return ADAPTSEG_OK;
}

int adaptseg_zero(void *ptr, size_t bytes, adaptseg_stream_t stream) {
  if (bytes == 0) return ADAPTSEG_OK;
  AS_CHECK_ARG(ptr, "zero: null pointer");
  hipError_t e = hipMemsetAsync(ptr, 0, bytes, as_stream(stream));
  if (e != hipSuccess) {
    set_error("zero: %s", hipGetErrorString(e));
    return ADAPTSEG_ERR_HIP;
  }
  return ADAPTSEG_OK;
}

int adaptseg_to_nhwc(int n, int c, int h, int w, const int64_t *src_stride, const float *src, float *dst,
                     adaptseg_stream_t stream) {
  return adaptseg_to_nhwc_pad(n, c, h, w, src_stride, src, c, dst, 0, stream);
}

int adaptseg_to_nhwc_pad(int n, int c, int h, int w, const int64_t *src_stride, const float *src, int c_dst,
                         float *dst, int flags, adaptseg_stream_t stream) {
  AS_CHECK_ARG(n > 0 && c > 0 && h > 0 && w > 0 && c_dst >= c && src_stride && src && dst,
               "to_nhwc_pad: bad args (c %d, c_dst %d)", c, c_dst);
  Strides4 st;
  for (int i = 0; i < 4; ++i) st.s[i] = src_stride[i];
  const int64_t total = (int64_t)n * c_dst * h * w;
  const bool acc = flags & ADAPTSEG_EPI_ACCUMULATE;
  if (c_dst % 4 == 0 && ((uintptr_t)dst & 15) == 0 && (int64_t)n * h < 65536 && (int64_t)w * c_dst < (1 << 30)) {
    const dim3 grid((unsigned)std::min<int64_t>(ceil_div((int64_t)w * (c_dst / 4), 256), 64), (unsigned)(n * h));
    if (acc) to_nhwc4_kernel<true><<<grid, 256, 0, as_stream(stream)>>>(c, c_dst, h, w, st, src, dst);
    else to_nhwc4_kernel<false><<<grid, 256, 0, as_stream(stream)>>>(c, c_dst, h, w, st, src, dst);
  } else if (acc)
    to_nhwc_kernel<true><<<grid1d(total), 256, 0, as_stream(stream)>>>(n, c, c_dst, h, w, st, src, dst);
  else
    to_nhwc_kernel<false><<<grid1d(total), 256, 0, as_stream(stream)>>>(n, c, c_dst, h, w, st, src, dst);
  AS_CHECK_LAUNCH("to_nhwc_pad");
  return ADAPTSEG_OK;
}

int adaptseg_axpy(int64_t n, float alpha, const float *src, float *dst, int flags, adaptseg_stream_t stream) {
  AS_CHECK_ARG(n >= 0 && (n == 0 || (src && dst)), "axpy: bad args");
  if (n == 0) return ADAPTSEG_OK;
  axpy_kernel<<<grid1d(n), 256, 0, as_stream(stream)>>>(n, alpha, src, dst, (flags & ADAPTSEG_EPI_ACCUMULATE) ? 1 : 0);
  AS_CHECK_LAUNCH("axpy");
  return ADAPTSEG_OK;
}

int adaptseg_add_i64(int64_t *p, int64_t n, int64_t v, adaptseg_stream_t stream) {
  AS_CHECK_ARG(n >= 0 && (n == 0 || p), "add_i64: bad args");
  if (n == 0) return ADAPTSEG_OK;
  add_i64_kernel<<<grid1d(n), 256, 0, as_stream(stream)>>>(p, n, v);
  AS_CHECK_LAUNCH("add_i64");
  return ADAPTSEG_OK;
}

}  // extern "C"
