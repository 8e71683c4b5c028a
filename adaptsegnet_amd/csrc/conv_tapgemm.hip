// Tap-GEMM path for stride-1 convolutions with few output channels (the ASPP classifier:
// Classifier_Module, model/deeplab_multi.py:106-121, 4 dilated 3x3 branches, Cout = 19).
//
// The direct implicit GEMM has N = Cout = 19, so every 32-wide MFMA column tile wastes 13/32 of
// its work.  Instead the taps are moved into the GEMM's N dimension:
//
//   fwd    Z[q][n]  = sum_ci X[q][ci] * W'[n][ci],          n = (seg*taps + t)*Cout + co
//          y[p][co] = sum_seg b_seg[co] + sum_{seg,t} Z[p + off(seg,t)][n(seg,t,co)]
//   bwd    G[q][n]  = dY[q - off(seg,t)][co]                (0 outside the image)
//          dX       = G * W'         (a 1x1 data-gradient GEMM, K = Nz)
//          dW'      = G^T * X        (a 1x1 weight-gradient GEMM, M' = Nz), unpacked into W_seg
//
// W' is the segments' weights re-packed as [Nz][Cin] (Nz = nseg*taps*Cout rounded up to 32,
// zero rows in the pad) — every GEMM is then a dense 1x1 problem on the FAST vector kernels
// (Nz = 704 for the 684 ASPP columns: 97 % useful MFMA work instead of 59 %).  Z / G cost one
// extra write + read of M x Nz floats (~90 MB at c2), a few percent of the GEMM time.
#include "conv_kernels.hpp"

namespace adaptseg {

constexpr int kTapAlign = 32;

static int tap_cols(const adaptseg_conv_desc *d) { return d->nseg * d->kh * d->kw * d->k; }
static int tap_nz(const adaptseg_conv_desc *d) { return (int)ceil_div(tap_cols(d), kTapAlign) * kTapAlign; }

bool tapgemm_eligible(const adaptseg_conv_desc *d) {
  if (!d || d->stride != 1 || d->k > 32 || d->c % 32 != 0 || d->in_stride[1] != 1) return false;
  if (d->oh != d->h || d->ow != d->w) return false;  // 'same' convolutions only (ASPP)
  if (tap_cols(d) < 128) return false;                // not worth the Z round trip
  const int64_t m = (int64_t)d->n * d->h * d->w;
  return m * tap_nz(d) < (1ll << 31) && (int64_t)tap_nz(d) * d->c < (1ll << 31);
}

// the dense 1x1 problem: (n, h, w) pixels, Cin -> Nz channels
static adaptseg_conv_desc inner_desc(const adaptseg_conv_desc *d) {
  adaptseg_conv_desc e;
  memset(&e, 0, sizeof(e));
  e.n = d->n; e.c = d->c; e.h = d->h; e.w = d->w;
  e.in_stride[0] = (int64_t)d->h * d->w * d->c; e.in_stride[1] = 1;
  e.in_stride[2] = (int64_t)d->w * d->c; e.in_stride[3] = d->c;
  e.k = tap_nz(d); e.oh = d->h; e.ow = d->w; e.kh = 1; e.kw = 1; e.stride = 1; e.nseg = 1;
  e.pad[0] = 0; e.dil[0] = 1;
  return e;
}

struct SegPtrs {
  const float *w[4];
};
struct SegOut {
  float *w[4];
};

// W'[n][ci] = W_seg[co][t][ci] for n = (seg*taps + t)*Cout + co; pad rows are 0.  float4 over ci.
__global__ void tap_pack_kernel(SegPtrs ws, int taps, int cout, int cin, int ncols, int nz, float *wp) {
  const int c4 = cin / 4;
  const int64_t total = (int64_t)nz * c4;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int n = (int)(i / c4), cq = (int)(i - (int64_t)n * c4);
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (n < ncols) {
      const int seg = n / (taps * cout), r = n - seg * taps * cout;
      const int t = r / cout, co = r - t * cout;
      const float *src = seg == 0 ? ws.w[0] : seg == 1 ? ws.w[1] : seg == 2 ? ws.w[2] : ws.w[3];
      v = reinterpret_cast<const float4 *>(src + ((size_t)co * taps + t) * cin)[cq];
    }
    reinterpret_cast<float4 *>(wp)[i] = v;
  }
}

// dW_seg[co][t][ci] (+)= dW'[n][ci]
__global__ void tap_unpack_kernel(const float *dwp, int taps, int cout, int cin, int ncols, SegOut out,
                                  int accumulate) {
  const int c4 = cin / 4;
  const int64_t total = (int64_t)ncols * c4;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int n = (int)(i / c4), cq = (int)(i - (int64_t)n * c4);
    const int seg = n / (taps * cout), r = n - seg * taps * cout;
    const int t = r / cout, co = r - t * cout;
    float *dst = seg == 0 ? out.w[0] : seg == 1 ? out.w[1] : seg == 2 ? out.w[2] : out.w[3];
    float4 *o = reinterpret_cast<float4 *>(dst + ((size_t)co * taps + t) * cin) + cq;
    float4 v = reinterpret_cast<const float4 *>(dwp)[i];
    if (accumulate) {
      const float4 a = *o;
      v.x += a.x; v.y += a.y; v.z += a.z; v.w += a.w;
    }
    *o = v;
  }
}

struct TapGeo {
  int n, h, w, cout, ntaps, nz;
  short dy[kMaxTaps], dx[kMaxTaps];
  const float *bias[4];
  int nseg;
};

// y[p][co] = sum bias + sum_{tap} Z[p + off(tap)][tap*Cout + co]  (+ the conv epilogue flags)
__global__ void tap_gather_sum_kernel(const TapGeo g, const float *__restrict__ z, float *y,
                                      const float *__restrict__ res, int flags) {
  const int64_t total = (int64_t)g.n * g.h * g.w * g.cout;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int co = (int)(i % g.cout);
    const int64_t p = i / g.cout;
    const int x = (int)(p % g.w);
    const int64_t t2 = p / g.w;
    const int yy = (int)(t2 % g.h);
    float v = 0.f;
    for (int s = 0; s < g.nseg; ++s)
      if (g.bias[s]) v += g.bias[s][co];
    for (int t = 0; t < g.ntaps; ++t) {
      const int sy = yy + g.dy[t], sx = x + g.dx[t];
      if ((unsigned)sy < (unsigned)g.h && (unsigned)sx < (unsigned)g.w) {
        const int64_t q = p + (int64_t)g.dy[t] * g.w + g.dx[t];
        v += z[q * g.nz + t * g.cout + co];
      }
    }
    if (flags & ADAPTSEG_EPI_ACCUMULATE) v += y[i];
    if (flags & ADAPTSEG_EPI_RESIDUAL) v += res[i];
    y[i] = epi_act(v, flags);
  }
}

// G[q][tap*Cout + co] = dY[q - off(tap)][co] (0 outside; pad columns 0)
__global__ void tap_scatter_grad_kernel(const TapGeo g, const float *__restrict__ dy, float *gbuf) {
  const int64_t total = (int64_t)g.n * g.h * g.w * g.nz;
  const int ncols = g.ntaps * g.cout;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int n = (int)(i % g.nz);
    const int64_t q = i / g.nz;
    float v = 0.f;
    if (n < ncols) {
      const int t = n / g.cout, co = n - t * g.cout;
      const int x = (int)(q % g.w);
      const int yy = (int)((q / g.w) % g.h);
      const int sy = yy - g.dy[t], sx = x - g.dx[t];
      if ((unsigned)sy < (unsigned)g.h && (unsigned)sx < (unsigned)g.w)
        v = dy[(q - (int64_t)g.dy[t] * g.w - g.dx[t]) * g.cout + co];
    }
    gbuf[i] = v;
  }
}

static TapGeo tap_geo(const adaptseg_conv_desc *d) {
  TapGeo g;
  memset(&g, 0, sizeof(g));
  g.n = d->n; g.h = d->h; g.w = d->w; g.cout = d->k;
  g.nseg = d->nseg;
  g.ntaps = d->nseg * d->kh * d->kw;
  g.nz = tap_nz(d);
  int t = 0;
  for (int s = 0; s < d->nseg; ++s)
    for (int kh = 0; kh < d->kh; ++kh)
      for (int kw = 0; kw < d->kw; ++kw, ++t) {
        g.dy[t] = (short)(kh * d->dil[s] - d->pad[s]);
        g.dx[t] = (short)(kw * d->dil[s] - d->pad[s]);
      }
  return g;
}

static int grid_for(int64_t n) { return (int)std::max<int64_t>(1, std::min<int64_t>(ceil_div(n, 256), 8192)); }

static size_t align256(size_t b) { return (b + 255) / 256 * 256; }

// Inner 1x1 plan for `op`; its FLOPs are reported as the outer conv's algorithmic FLOPs.
static int inner_plan(const adaptseg_conv_desc *d, int op, Plan &pl) {
  adaptseg_conv_desc e = inner_desc(d);
  int st = make_plan(&e, op, pl);
  if (st) return st;
  set_splits(pl);
  pl.flops = conv_flops(d);
  return ADAPTSEG_OK;
}

size_t tapgemm_workspace(const adaptseg_conv_desc *d, int op) {
  const size_t m = (size_t)d->n * d->h * d->w, nz = tap_nz(d);
  const size_t mn = align256(m * nz * sizeof(float)), wn = align256(nz * d->c * sizeof(float));
  Plan pl;
  if (inner_plan(d, op, pl)) return 0;
  return mn + wn + pl.slab_bytes;
}

int tapgemm_kernel_id(const adaptseg_conv_desc *d, int op, int *kid, int *splits) {
  Plan pl;
  int st = inner_plan(d, op, pl);
  if (st) return st;
  *kid = kernel_id(pl, op);
  *splits = pl.p.splits;
  return ADAPTSEG_OK;
}

// The inner GEMM reads only x's bf16 copy, so the _x forms accept x == NULL: forward and weight
// gradient on an LDS-DMA inner kernel.  The data gradient's tap scatter reads dY in fp32.
bool tapgemm_copy_only(const adaptseg_conv_desc *d, int op) {
  Plan pl;
  if (op == ADAPTSEG_CONV_BWD_DATA || inner_plan(d, op, pl)) return false;
  return pl.g16;
}

static int need_ws(const adaptseg_conv_desc *d, int op, size_t ws_bytes, void *ws) {
  const size_t need = tapgemm_workspace(d, op);
  if (!ws || ws_bytes < need) {
    set_error("conv (tap-GEMM): workspace %zu < required %zu", ws_bytes, need);
    return ADAPTSEG_ERR_WORKSPACE;
  }
  return ADAPTSEG_OK;
}

int tapgemm_fwd(const adaptseg_conv_desc *d, const float *x, const uint16_t *x_bf16, const float *const *w,
                const float *const *bias, const float *res, float *y, int flags, void *ws, size_t ws_bytes,
                hipStream_t s) {
  int st = need_ws(d, ADAPTSEG_CONV_FWD, ws_bytes, ws);
  if (st) return st;
  const size_t m = (size_t)d->n * d->h * d->w, nz = tap_nz(d);
  char *base = reinterpret_cast<char *>(ws);
  float *z = reinterpret_cast<float *>(base);
  float *wp = reinterpret_cast<float *>(base + align256(m * nz * sizeof(float)));
  void *gws = base + align256(m * nz * sizeof(float)) + align256(nz * d->c * sizeof(float));
  size_t gws_bytes = ws_bytes - (size_t)(reinterpret_cast<char *>(gws) - base);
  SegPtrs sp{};
  for (int i = 0; i < d->nseg; ++i) sp.w[i] = w[i];
  const int taps = d->kh * d->kw;
  tap_pack_kernel<<<grid_for((int64_t)nz * d->c / 4), 256, 0, s>>>(sp, taps, d->k, d->c, tap_cols(d), (int)nz, wp);
  AS_CHECK_LAUNCH("tap_pack");
  Plan pl;
  st = inner_plan(d, ADAPTSEG_CONV_FWD, pl);
  if (st) return st;
  pl.p.x = x;
  // the operand copy: read by the bf16 LDS-DMA kernels (BF16 maths) and, under F32X3_PRESPLIT,
  // as the term images of x by the inner x3r kernel (which then skips its per-call split)
  pl.act_ext = (reinterpret_cast<uintptr_t>(x_bf16) & 15) ? nullptr : x_bf16;
  AS_CHECK_ARG(x || (pl.g16 && pl.act_ext), "conv fwd (tap-GEMM): x is NULL and the inner GEMM needs it");
  pl.p.wt[0] = wp;
  pl.p.out = z;
  pl.p.flags = 0;
  st = run_plan(pl, MODE_FWD, gws, gws_bytes, s);
  if (st) return st;
  TapGeo g = tap_geo(d);
  for (int i = 0; i < d->nseg; ++i) g.bias[i] = bias ? bias[i] : nullptr;
  tap_gather_sum_kernel<<<grid_for((int64_t)m * d->k), 256, 0, s>>>(g, z, y, res, flags);
  AS_CHECK_LAUNCH("tap_gather_sum");
  return ADAPTSEG_OK;
}

int tapgemm_bwd_data(const adaptseg_conv_desc *d, const float *dy, const float *const *w, const float *res,
                     const float *aux, float *dx, int flags, void *ws, size_t ws_bytes, hipStream_t s) {
  int st = need_ws(d, ADAPTSEG_CONV_BWD_DATA, ws_bytes, ws);
  if (st) return st;
  const size_t m = (size_t)d->n * d->h * d->w, nz = tap_nz(d);
  char *base = reinterpret_cast<char *>(ws);
  float *gbuf = reinterpret_cast<float *>(base);
  float *wp = reinterpret_cast<float *>(base + align256(m * nz * sizeof(float)));
  void *gws = base + align256(m * nz * sizeof(float)) + align256(nz * d->c * sizeof(float));
  size_t gws_bytes = ws_bytes - (size_t)(reinterpret_cast<char *>(gws) - base);
  SegPtrs sp{};
  for (int i = 0; i < d->nseg; ++i) sp.w[i] = w[i];
  tap_pack_kernel<<<grid_for((int64_t)nz * d->c / 4), 256, 0, s>>>(sp, d->kh * d->kw, d->k, d->c, tap_cols(d),
                                                                   (int)nz, wp);
  AS_CHECK_LAUNCH("tap_pack");
  TapGeo g = tap_geo(d);
  tap_scatter_grad_kernel<<<grid_for((int64_t)m * nz), 256, 0, s>>>(g, dy, gbuf);
  AS_CHECK_LAUNCH("tap_scatter_grad");
  Plan pl;
  st = inner_plan(d, ADAPTSEG_CONV_BWD_DATA, pl);
  if (st) return st;
  pl.p.dy = gbuf;
  pl.p.wt[0] = wp;
  pl.p.out = dx;
  pl.p.res = res;
  pl.p.aux = aux;
  pl.p.flags = flags;
  return run_plan(pl, MODE_DGRAD, gws, gws_bytes, s);
}

int tapgemm_bwd_weight(const adaptseg_conv_desc *d, const float *dy, const float *x, const uint16_t *x_bf16,
                       float *const *dw, int flags, void *ws, size_t ws_bytes, hipStream_t s) {
  int st = need_ws(d, ADAPTSEG_CONV_BWD_WEIGHT, ws_bytes, ws);
  if (st) return st;
  const size_t m = (size_t)d->n * d->h * d->w, nz = tap_nz(d);
  char *base = reinterpret_cast<char *>(ws);
  float *gbuf = reinterpret_cast<float *>(base);
  float *dwp = reinterpret_cast<float *>(base + align256(m * nz * sizeof(float)));
  void *gws = base + align256(m * nz * sizeof(float)) + align256(nz * d->c * sizeof(float));
  size_t gws_bytes = ws_bytes - (size_t)(reinterpret_cast<char *>(gws) - base);
  TapGeo g = tap_geo(d);
  tap_scatter_grad_kernel<<<grid_for((int64_t)m * nz), 256, 0, s>>>(g, dy, gbuf);
  AS_CHECK_LAUNCH("tap_scatter_grad");
  Plan pl;
  st = inner_plan(d, ADAPTSEG_CONV_BWD_WEIGHT, pl);
  if (st) return st;
  pl.p.dy = gbuf;
  pl.p.x = x;
  pl.act_ext2 = (reinterpret_cast<uintptr_t>(x_bf16) & 15) ? nullptr : x_bf16;   // x's copy; dY's is made here
  AS_CHECK_ARG(x || (pl.g16 && pl.act_ext2), "conv bwd_weight (tap-GEMM): x is NULL and the inner GEMM needs it");
  pl.p.dw[0] = dwp;
  pl.p.flags = 0;
  st = run_plan(pl, MODE_WGRAD, gws, gws_bytes, s);
  if (st) return st;
  SegOut so{};
  for (int i = 0; i < d->nseg; ++i) so.w[i] = dw[i];
  tap_unpack_kernel<<<grid_for((int64_t)tap_cols(d) * d->c / 4), 256, 0, s>>>(
      dwp, d->kh * d->kw, d->k, d->c, tap_cols(d), so, (flags & ADAPTSEG_EPI_ACCUMULATE) ? 1 : 0);
  AS_CHECK_LAUNCH("tap_unpack");
  return ADAPTSEG_OK;
}

}  // namespace adaptseg
