// GTA5 / Cityscapes input pipeline on the GPU: the arithmetic of
// GTA5DataSet.__getitem__ (reference dataset/gta5_dataset.py:47-71) after file decode,
//   image.resize(crop, BICUBIC); label.resize(crop, NEAREST); id -> trainId (255 elsewhere);
//   RGB -> BGR; -= IMG_MEAN (float32); HWC -> CHW
// reproduced bit-exactly.  The resize is Pillow's 8-bpc separable resampler (the library the
// reference calls): per output pixel a window [xmin, xmin+n) and n weights of the bicubic
// kernel (a = -0.5) stretched by the downscale factor, normalised in double and rounded to
// 22-bit fixed point; a horizontal pass then a vertical pass, each accumulating in int32 from
// 2^21 and clamping (acc >> 22) to uint8.  NEAREST takes floor((x + 0.5) * scale) with the
// coordinate accumulated in double, as Pillow's affine transform does.
//
// Kernels: resize_coeff_kernel builds the weight tables on the device in double with FP
// contraction off (so they equal the host's / Pillow's); resize_h_kernel (uint8 RGB ->
// uint8 [n][in_h][out_w][3]); resize_v_bgr_kernel (-> float NCHW BGR - mean); label_kernel.
// All byte/integer work, HBM-bound: one read of the source image and labels, one write of
// the float image and int64 labels (plus the out_w-wide uint8 intermediate).
#include "common.hpp"
#include <algorithm>
#include <cmath>

namespace adaptseg {

constexpr int kPrecisionBits = 32 - 8 - 2;
constexpr int kMaxKsize = 64;  // ceil(2 * downscale) * 2 + 1 <= 64: downscale up to 15x

#pragma clang fp contract(off)
__device__ double bicubic_filter(double x) {
  const double a = -0.5;
  if (x < 0.0) x = -x;
  if (x < 1.0) return ((a + 2.0) * x - (a + 3.0)) * x * x + 1;
  if (x < 2.0) return (((x - 5) * x + 8) * x - 4) * a;
  return 0.0;
}

struct ResizeTables {
  int ksx, ksy;        // taps per output pixel (x, y)
  int *bx, *by;        // [out][2] = (first source index, count)
  int *kx, *ky;        // [out][ks] fixed-point weights
  int *nx, *ny;        // nearest source index per output column / row
};

__device__ void coeffs_one(int in_size, int out_size, int o, int ks, int *bounds, int *kk) {
  const double scale = (double)in_size / (double)out_size;
  const double filterscale = scale < 1.0 ? 1.0 : scale;
  const double support = 2.0 * filterscale;
  const double ss = 1.0 / filterscale;
  const double center = ((double)o + 0.5) * scale;
  int xmin = (int)(center - support + 0.5);
  if (xmin < 0) xmin = 0;
  int xmax = (int)(center + support + 0.5);
  if (xmax > in_size) xmax = in_size;
  xmax -= xmin;
  // two passes over the (deterministic) filter instead of a per-thread weight array, which
  // would live in scratch: the sum first, then each normalised weight
  double ww = 0.0;
  for (int x = 0; x < xmax; ++x) ww += bicubic_filter(((double)(x + xmin) - center + 0.5) * ss);
  for (int x = 0; x < ks; ++x) {
    const double w = x < xmax ? bicubic_filter(((double)(x + xmin) - center + 0.5) * ss) : 0.0;
    const double v = ww != 0.0 ? w / ww : w;
    kk[(size_t)o * ks + x] = v < 0 ? (int)(-0.5 + v * (double)(1 << kPrecisionBits))
                                   : (int)(0.5 + v * (double)(1 << kPrecisionBits));
  }
  bounds[2 * o] = xmin;
  bounds[2 * o + 1] = xmax;
}

// threads [0, out_w) -> x weights, [out_w, out_w + out_h) -> y weights; the last two
// threads walk the NEAREST coordinates (a sequential double accumulation, as Pillow).
__global__ void resize_coeff_kernel(int in_h, int in_w, int out_h, int out_w, ResizeTables t) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < out_w) coeffs_one(in_w, out_w, i, t.ksx, t.bx, t.kx);
  else if (i < out_w + out_h) coeffs_one(in_h, out_h, i - out_w, t.ksy, t.by, t.ky);
  else if (i == out_w + out_h || i == out_w + out_h + 1) {
    const bool xs = i == out_w + out_h;
    const int in = xs ? in_w : in_h, out = xs ? out_w : out_h;
    int *dst = xs ? t.nx : t.ny;
    const double scale = (double)in / (double)out;
    double v = 0.5 * scale;
    for (int o = 0; o < out; ++o) {
      const int s = (int)v;
      dst[o] = s < in - 1 ? s : in - 1;
      v += scale;
    }
  }
}
#pragma clang fp contract(on)

__device__ __forceinline__ unsigned clip8(int acc) {
  const int v = acc >> kPrecisionBits;
  return (unsigned)(v < 0 ? 0 : v > 255 ? 255 : v);
}

// Horizontal pass: src [n][in_h][in_w][3] -> tmp [n][in_h][out_w][3] (uint8, Pillow-rounded).
__global__ void resize_h_kernel(int n, int in_h, int in_w, int out_w, const uint8_t *__restrict__ src,
                                ResizeTables t, uint8_t *__restrict__ tmp) {
  const int64_t total = (int64_t)n * in_h * out_w;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int xo = (int)(i % out_w);
    const int64_t row = i / out_w;  // n * in_h + y
    const int x0 = t.bx[2 * xo], cnt = t.bx[2 * xo + 1];
    const int *k = t.kx + (size_t)xo * t.ksx;
    const uint8_t *s = src + (row * in_w + x0) * 3;
    int a0 = 1 << (kPrecisionBits - 1), a1 = a0, a2 = a0;
    for (int j = 0; j < cnt; ++j) {
      const int w = k[j];
      a0 += s[3 * j] * w;
      a1 += s[3 * j + 1] * w;
      a2 += s[3 * j + 2] * w;
    }
    uint8_t *d = tmp + i * 3;
    d[0] = (uint8_t)clip8(a0);
    d[1] = (uint8_t)clip8(a1);
    d[2] = (uint8_t)clip8(a2);
  }
}

// Vertical pass + BGR + mean + CHW: tmp [n][in_h][out_w][3] -> out [n][3][out_h][out_w] with
// out[c'] = float(rgb[2 - c']) - mean[c'] (float32, as image -= IMG_MEAN).
__global__ void resize_v_bgr_kernel(int n, int in_h, int out_h, int out_w, const uint8_t *__restrict__ tmp,
                                    ResizeTables t, float m0, float m1, float m2, float *__restrict__ out) {
  const int64_t total = (int64_t)n * out_h * out_w;
  const int64_t plane = (int64_t)out_h * out_w;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int xo = (int)(i % out_w);
    const int64_t r = i / out_w;
    const int yo = (int)(r % out_h);
    const int b = (int)(r / out_h);
    const int y0 = t.by[2 * yo], cnt = t.by[2 * yo + 1];
    const int *k = t.ky + (size_t)yo * t.ksy;
    const uint8_t *s = tmp + (((int64_t)b * in_h + y0) * out_w + xo) * 3;
    const int64_t stride = (int64_t)out_w * 3;
    int a0 = 1 << (kPrecisionBits - 1), a1 = a0, a2 = a0;
    for (int j = 0; j < cnt; ++j) {
      const int w = k[j];
      a0 += s[j * stride] * w;
      a1 += s[j * stride + 1] * w;
      a2 += s[j * stride + 2] * w;
    }
    float *o = out + (int64_t)b * 3 * plane + (int64_t)yo * out_w + xo;
    o[0] = (float)clip8(a2) - m0;  // B
    o[plane] = (float)clip8(a1) - m1;  // G
    o[2 * plane] = (float)clip8(a0) - m2;  // R
  }
}

// labels [n][in_h][in_w] uint8 ids -> [n][out_h][out_w] int64 trainIds (lut[256], int32).
__global__ void label_kernel(int n, int in_h, int in_w, int out_h, int out_w, const uint8_t *__restrict__ ids,
                             ResizeTables t, const int32_t *__restrict__ lut, int64_t *__restrict__ out) {
  const int64_t total = (int64_t)n * out_h * out_w;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int xo = (int)(i % out_w);
    const int64_t r = i / out_w;
    const int yo = (int)(r % out_h);
    const int b = (int)(r / out_h);
    const uint8_t id = ids[((int64_t)b * in_h + t.ny[yo]) * in_w + t.nx[xo]];
    out[i] = lut ? (int64_t)lut[id] : (int64_t)id;
  }
}

static int ksize_for(int in_size, int out_size) {
  const double scale = (double)in_size / (double)out_size;
  const double support = 2.0 * (scale < 1.0 ? 1.0 : scale);
  return (int)std::ceil(support) * 2 + 1;
}

static size_t a256(size_t b) { return (b + 255) / 256 * 256; }

struct WsLayout {
  size_t bx, kx, by, ky, nx, ny, tmp, total;
};

static WsLayout ws_layout(int n, int in_h, int in_w, int out_h, int out_w) {
  WsLayout l;
  const int ksx = ksize_for(in_w, out_w), ksy = ksize_for(in_h, out_h);
  size_t o = 0;
  l.bx = o; o += a256((size_t)out_w * 2 * 4);
  l.kx = o; o += a256((size_t)out_w * ksx * 4);
  l.by = o; o += a256((size_t)out_h * 2 * 4);
  l.ky = o; o += a256((size_t)out_h * ksy * 4);
  l.nx = o; o += a256((size_t)out_w * 4);
  l.ny = o; o += a256((size_t)out_h * 4);
  l.tmp = o; o += a256((size_t)n * in_h * out_w * 3);
  l.total = o;
  return l;
}

static int grid_for(int64_t total) { return (int)std::max<int64_t>(1, std::min<int64_t>(ceil_div(total, 256), 16384)); }

}  // namespace adaptseg

using namespace adaptseg;

extern "C" {

int adaptseg_preprocess_workspace_size(int n, int in_h, int in_w, int out_h, int out_w, size_t *bytes) {
  AS_CHECK_ARG(bytes && n > 0 && in_h > 0 && in_w > 0 && out_h > 0 && out_w > 0, "preprocess_workspace_size: bad args");
  AS_CHECK_ARG(ksize_for(in_w, out_w) <= kMaxKsize && ksize_for(in_h, out_h) <= kMaxKsize,
               "preprocess: downscale factor above 15 not supported");
  *bytes = ws_layout(n, in_h, in_w, out_h, out_w).total;
  return ADAPTSEG_OK;
}

int adaptseg_gta5_preprocess(int n, int in_h, int in_w, int out_h, int out_w, const uint8_t *rgb, float mean_b,
                             float mean_g, float mean_r, float *image, const uint8_t *label_ids, const int32_t *lut,
                             int64_t *labels, void *ws, size_t ws_bytes, adaptseg_stream_t stream) {
  AS_CHECK_ARG(n > 0 && in_h > 0 && in_w > 0 && out_h > 0 && out_w > 0, "gta5_preprocess: bad sizes");
  AS_CHECK_ARG(rgb && image, "gta5_preprocess: null image pointer");
  AS_CHECK_ARG(!label_ids == !labels, "gta5_preprocess: label_ids and labels go together");
  AS_CHECK_ARG((int64_t)n * in_h * in_w * 3 < (1ll << 40), "gta5_preprocess: input too large");
  AS_CHECK_ARG(ksize_for(in_w, out_w) <= kMaxKsize && ksize_for(in_h, out_h) <= kMaxKsize,
               "gta5_preprocess: downscale factor above 15 not supported");
  const WsLayout l = ws_layout(n, in_h, in_w, out_h, out_w);
  if (!ws || ws_bytes < l.total) {
    set_error("gta5_preprocess: workspace %zu < required %zu", ws_bytes, l.total);
    return ADAPTSEG_ERR_WORKSPACE;
  }
  char *base = reinterpret_cast<char *>(ws);
  ResizeTables t;
  t.ksx = ksize_for(in_w, out_w);
  t.ksy = ksize_for(in_h, out_h);
  t.bx = reinterpret_cast<int *>(base + l.bx);
  t.kx = reinterpret_cast<int *>(base + l.kx);
  t.by = reinterpret_cast<int *>(base + l.by);
  t.ky = reinterpret_cast<int *>(base + l.ky);
  t.nx = reinterpret_cast<int *>(base + l.nx);
  t.ny = reinterpret_cast<int *>(base + l.ny);
  uint8_t *tmp = reinterpret_cast<uint8_t *>(base + l.tmp);
  hipStream_t s = as_stream(stream);
  resize_coeff_kernel<<<(unsigned)ceil_div(out_w + out_h + 2, 64), 64, 0, s>>>(in_h, in_w, out_h, out_w, t);
  AS_CHECK_LAUNCH("resize_coeff");
  // Pillow skips a pass whose size is unchanged; the identity table (one tap of 2^22) gives
  // the same bytes, so both passes always run.
  resize_h_kernel<<<grid_for((int64_t)n * in_h * out_w), 256, 0, s>>>(n, in_h, in_w, out_w, rgb, t, tmp);
  AS_CHECK_LAUNCH("resize_h");
  resize_v_bgr_kernel<<<grid_for((int64_t)n * out_h * out_w), 256, 0, s>>>(n, in_h, out_h, out_w, tmp, t, mean_b,
                                                                           mean_g, mean_r, image);
  AS_CHECK_LAUNCH("resize_v_bgr");
  if (label_ids) {
    label_kernel<<<grid_for((int64_t)n * out_h * out_w), 256, 0, s>>>(n, in_h, in_w, out_h, out_w, label_ids, t,
                                                                      lut, labels);
    AS_CHECK_LAUNCH("label");
  }
  return ADAPTSEG_OK;
}

}  // extern "C"
