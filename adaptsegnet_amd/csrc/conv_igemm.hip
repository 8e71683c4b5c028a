// Implicit-GEMM convolution for gfx950 (MI355X) on fp32 MFMA (v_mfma_f32_32x32x2_f32).
//
// One kernel template serves the three convolution products of the AdaptSegNet step
// (reference: every nn.Conv2d of model/deeplab_multi.py and model/discriminator.py):
//
//   FWD    C[m=(n,oh,ow)][co]       = sum_{k=(tap,ci)}  X[n, oh*s+dy(tap), ow*s+dx(tap), ci] * W[co][tap][ci]
//   DGRAD  C[m=(n,ih,iw)][ci]       = sum_{k=(tap,co)}  dY[n, (ih-dy)/s, (iw-dx)/s, co]       * W[co][tap][ci]
//   WGRAD  C[co][(tap,ci)]          = sum_{k=(n,oh,ow)} dY[n,oh,ow,co] * X[n, oh*s+dy, ow*s+dx, ci]
//
// A "tap" is one (kh, kw) position of one segment; (dy, dx) = (kh*dil - pad, kw*dil - pad).
// ASPP (Classifier_Module, model/deeplab_multi.py:106-121) is nseg = 4 segments whose
// taps are concatenated along K, so the four dilated 3x3 branches and their sum are a
// single GEMM.  Activations are NHWC; weights [Cout][KH][KW][Cin] per segment.
//
// Tiling: 256 threads (4 wave64s), block tile BM x BN, K step 16, two LDS stages with
// register staging (global loads of step k+1 are in flight while step k runs on the
// MFMA pipe).  LDS holds both operands k-major ([16][BM+pad]); each lane feeds the
// 32x32x2 MFMA with one ds_read_b32 per operand, which is conflict-free.  Small GEMM
// grids are split along K into fp32 slabs that a deterministic reduce kernel sums.
#include "common.hpp"
#include <algorithm>
#include <cstring>
#include <mutex>
#include <vector>

namespace adaptseg {

typedef float floatx16 __attribute__((ext_vector_type(16)));

enum { MODE_FWD = 0, MODE_DGRAD = 1, MODE_WGRAD = 2 };
constexpr int kMaxTaps = 64;
constexpr int BK = 16;

struct ConvParams {
  int M, N, K;                 // GEMM extents
  int n, c, h, w;              // conv input geometry
  int sxn, sxc, sxh, sxw;      // conv input strides (elements) — FWD/WGRAD gather
  int k, oh, ow;               // conv output geometry (dY is NHWC contiguous)
  int stride;
  int ntaps, taps_per_seg, nseg;
  int kseg;                    // FWD: taps_per_seg*c ; DGRAD: taps_per_seg*c (row length of W)
  int ktiles_per_split, splits;
  FastDiv fd_c, fd_k, fd_ow, fd_oh, fd_ohw, fd_hw, fd_w, fd_nseg_k;
  const float *x;              // conv input (FWD, WGRAD)
  const float *dy;             // grad of conv output (DGRAD, WGRAD)
  const float *wt[4];          // weights per segment (FWD, DGRAD)
  float *out;                  // final output (splits == 1) or slab base (splits > 1)
  float *dw[4];                // WGRAD outputs per segment
  const float *bias[4];        // FWD bias per segment (nullable)
  const float *res;            // residual (nullable)
  const float *aux;            // leaky-grad source (nullable)
  int flags;
  int kw_, kh_;                // kernel width / height (tap -> kh, kw)
  int pad_[4], dil_[4];        // per-segment padding / dilation
  FastDiv fd_taps, fd_kw;
  short tap_dy[kMaxTaps], tap_dx[kMaxTaps];
};

// ------------------------------------------------------------------------------------
// Operand gathers.  Each returns 4 consecutive elements along the operand's contiguous
// dimension (k for k-contiguous operands, m/n for mn-contiguous ones).
// ------------------------------------------------------------------------------------

__device__ __forceinline__ float4 ld4(const float *p) { return *reinterpret_cast<const float4 *>(p); }

// FWD A: element (m, k).  Row info (precomputed): base offset of image, ih0, iw0, valid.
struct RowInfo {
  int base;   // n*sxn (FWD) or n index (DGRAD)
  int y0, x0; // oh*s, ow*s (FWD) or ih, iw (DGRAD)
  bool ok;
};

__device__ __forceinline__ RowInfo fwd_row_info(const ConvParams &p, int m) {
  RowInfo r;
  r.ok = m < p.M;
  int mm = r.ok ? m : 0;
  uint32_t t = fdiv((uint32_t)mm, p.fd_ow);
  int ow = mm - (int)t * p.ow;
  uint32_t b = fdiv(t, p.fd_oh);
  int oh = (int)t - (int)b * p.oh;
  r.base = (int)b * p.sxn;
  r.y0 = oh * p.stride;
  r.x0 = ow * p.stride;
  return r;
}

__device__ __forceinline__ float fwd_a_elem(const ConvParams &p, const short *tdy, const short *tdx,
                                            const RowInfo &r, int k) {
  if (!r.ok || k >= p.K) return 0.f;
  int tap = (int)fdiv((uint32_t)k, p.fd_c);
  int ci = k - tap * p.c;
  int ih = r.y0 + tdy[tap], iw = r.x0 + tdx[tap];
  if ((unsigned)ih >= (unsigned)p.h || (unsigned)iw >= (unsigned)p.w) return 0.f;
  return p.x[r.base + ih * p.sxh + iw * p.sxw + ci * p.sxc];
}

template <bool VEC>
__device__ __forceinline__ float4 fwd_a_load(const ConvParams &p, const short *tdy, const short *tdx,
                                             const RowInfo &r, int k) {
  if constexpr (VEC) {
    // c % 4 == 0 and sxc == 1: the 4 elements share one tap and are contiguous.
    if (!r.ok || k >= p.K) return make_float4(0.f, 0.f, 0.f, 0.f);
    int tap = (int)fdiv((uint32_t)k, p.fd_c);
    int ci = k - tap * p.c;
    int ih = r.y0 + tdy[tap], iw = r.x0 + tdx[tap];
    if ((unsigned)ih >= (unsigned)p.h || (unsigned)iw >= (unsigned)p.w)
      return make_float4(0.f, 0.f, 0.f, 0.f);
    return ld4(p.x + r.base + ih * p.sxh + iw * p.sxw + ci);
  } else {
    return make_float4(fwd_a_elem(p, tdy, tdx, r, k), fwd_a_elem(p, tdy, tdx, r, k + 1),
                       fwd_a_elem(p, tdy, tdx, r, k + 2), fwd_a_elem(p, tdy, tdx, r, k + 3));
  }
}

// Weight pointer of segment `seg` (nseg <= 4; seg is uniform or nearly so).
__device__ __forceinline__ const float *seg_ptr(const ConvParams &p, int seg) {
  return seg == 0 ? p.wt[0] : seg == 1 ? p.wt[1] : seg == 2 ? p.wt[2] : p.wt[3];
}

// FWD B: element (k, n) = W[seg][n][k - seg*kseg], k-contiguous rows of length kseg.
__device__ __forceinline__ float fwd_b_elem(const ConvParams &p, int n, int k) {
  if (n >= p.N || k >= p.K) return 0.f;
  int seg = (int)fdiv((uint32_t)k, p.fd_nseg_k);
  int kk = k - seg * p.kseg;
  return seg_ptr(p, seg)[n * p.kseg + kk];
}

template <bool VEC>
__device__ __forceinline__ float4 fwd_b_load(const ConvParams &p, int n, int k) {
  if constexpr (VEC) {
    if (n >= p.N || k >= p.K) return make_float4(0.f, 0.f, 0.f, 0.f);
    int seg = (int)fdiv((uint32_t)k, p.fd_nseg_k);
    int kk = k - seg * p.kseg;
    return ld4(seg_ptr(p, seg) + n * p.kseg + kk);
  } else {
    return make_float4(fwd_b_elem(p, n, k), fwd_b_elem(p, n, k + 1), fwd_b_elem(p, n, k + 2),
                       fwd_b_elem(p, n, k + 3));
  }
}

// DGRAD A: element (m=(b,ih,iw), k=(tap,co)) = dY[b, (ih-dy)/s, (iw-dx)/s, co].
__device__ __forceinline__ RowInfo dgrad_row_info(const ConvParams &p, int m) {
  RowInfo r;
  r.ok = m < p.M;
  int mm = r.ok ? m : 0;
  uint32_t t = fdiv((uint32_t)mm, p.fd_w);
  int iw = mm - (int)t * p.w;
  uint32_t b = fdiv(t, p.fd_hw);  // fd_hw holds h here
  int ih = (int)t - (int)b * p.h;
  r.base = (int)b;
  r.y0 = ih;
  r.x0 = iw;
  return r;
}

__device__ __forceinline__ bool dgrad_src(const ConvParams &p, int v, int d, int lim, int &o) {
  int num = v - d;
  if (p.stride == 1) {
    o = num;
  } else {
    if (num < 0 || (num % p.stride) != 0) return false;
    o = num / p.stride;
  }
  return (unsigned)o < (unsigned)lim;
}

__device__ __forceinline__ float dgrad_a_elem(const ConvParams &p, const short *tdy, const short *tdx,
                                              const RowInfo &r, int k) {
  if (!r.ok || k >= p.K) return 0.f;
  int tap = (int)fdiv((uint32_t)k, p.fd_k);
  int co = k - tap * p.k;
  int oh, ow;
  if (!dgrad_src(p, r.y0, tdy[tap], p.oh, oh) || !dgrad_src(p, r.x0, tdx[tap], p.ow, ow)) return 0.f;
  return p.dy[((r.base * p.oh + oh) * p.ow + ow) * p.k + co];
}

template <bool VEC>
__device__ __forceinline__ float4 dgrad_a_load(const ConvParams &p, const short *tdy, const short *tdx,
                                               const RowInfo &r, int k) {
  if constexpr (VEC) {
    if (!r.ok || k >= p.K) return make_float4(0.f, 0.f, 0.f, 0.f);
    int tap = (int)fdiv((uint32_t)k, p.fd_k);
    int co = k - tap * p.k;
    int oh, ow;
    if (!dgrad_src(p, r.y0, tdy[tap], p.oh, oh) || !dgrad_src(p, r.x0, tdx[tap], p.ow, ow))
      return make_float4(0.f, 0.f, 0.f, 0.f);
    return ld4(p.dy + ((r.base * p.oh + oh) * p.ow + ow) * p.k + co);
  } else {
    return make_float4(dgrad_a_elem(p, tdy, tdx, r, k), dgrad_a_elem(p, tdy, tdx, r, k + 1),
                       dgrad_a_elem(p, tdy, tdx, r, k + 2), dgrad_a_elem(p, tdy, tdx, r, k + 3));
  }
}

// DGRAD B: element (k=(tap,co), n=ci) = W[seg][co][tap_in_seg][ci]; rows k, n contiguous.
__device__ __forceinline__ const float *dgrad_b_row(const ConvParams &p, int k) {
  int tap = (int)fdiv((uint32_t)k, p.fd_k);
  int co = k - tap * p.k;
  int seg = tap / p.taps_per_seg;
  int t = tap - seg * p.taps_per_seg;
  return seg_ptr(p, seg) + (co * p.taps_per_seg + t) * p.c;
}

template <bool VEC>
__device__ __forceinline__ float4 dgrad_b_load(const ConvParams &p, int k, int n) {
  float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
  if (k >= p.K) return v;
  const float *row = dgrad_b_row(p, k);
  if constexpr (VEC) {
    if (n < p.N) v = ld4(row + n);  // N % 4 == 0
  } else {
    if (n < p.N) v.x = row[n];
    if (n + 1 < p.N) v.y = row[n + 1];
    if (n + 2 < p.N) v.z = row[n + 2];
    if (n + 3 < p.N) v.w = row[n + 3];
  }
  return v;
}

// WGRAD A: element (m'=co, k'=m) = dY[m][co]; rows k', m' contiguous.
template <bool VEC>
__device__ __forceinline__ float4 wgrad_a_load(const ConvParams &p, int kk, int mcol) {
  float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
  if (kk >= p.K) return v;
  const float *row = p.dy + (size_t)kk * p.k;
  if constexpr (VEC) {
    if (mcol < p.M) v = ld4(row + mcol);
  } else {
    if (mcol < p.M) v.x = row[mcol];
    if (mcol + 1 < p.M) v.y = row[mcol + 1];
    if (mcol + 2 < p.M) v.z = row[mcol + 2];
    if (mcol + 3 < p.M) v.w = row[mcol + 3];
  }
  return v;
}

// WGRAD B: element (k'=m=(b,oh,ow), n'=(tap,ci)) = X[b, oh*s+dy, ow*s+dx, ci].
struct ColInfo {
  int dy, dx, ci;
  bool ok;
};

__device__ __forceinline__ ColInfo wgrad_col_info(const ConvParams &p, const short *tdy,
                                                  const short *tdx, int nn) {
  ColInfo c;
  c.ok = nn < p.N;
  int n2 = c.ok ? nn : 0;
  int tap = (int)fdiv((uint32_t)n2, p.fd_c);
  c.ci = n2 - tap * p.c;
  c.dy = tdy[tap];
  c.dx = tdx[tap];
  return c;
}

struct PixInfo {
  int base, y0, x0;
  bool ok;
};

__device__ __forceinline__ PixInfo wgrad_pix(const ConvParams &p, int kk) {
  PixInfo q;
  q.ok = kk < p.K;
  int m = q.ok ? kk : 0;
  uint32_t t = fdiv((uint32_t)m, p.fd_ow);
  int ow = m - (int)t * p.ow;
  uint32_t b = fdiv(t, p.fd_oh);
  int oh = (int)t - (int)b * p.oh;
  q.base = (int)b * p.sxn;
  q.y0 = oh * p.stride;
  q.x0 = ow * p.stride;
  return q;
}

__device__ __forceinline__ float wgrad_b_elem(const ConvParams &p, const PixInfo &q, const ColInfo &c) {
  if (!q.ok || !c.ok) return 0.f;
  int ih = q.y0 + c.dy, iw = q.x0 + c.dx;
  if ((unsigned)ih >= (unsigned)p.h || (unsigned)iw >= (unsigned)p.w) return 0.f;
  return p.x[q.base + ih * p.sxh + iw * p.sxw + c.ci * p.sxc];
}

// ------------------------------------------------------------------------------------
// Kernel
// ------------------------------------------------------------------------------------
template <int MODE, int BM, int BN, int WAVES_M, int WAVES_N, bool VA, bool VB>
__global__ void __launch_bounds__(256) igemm_kernel(const ConvParams p) {
  constexpr int WTM = BM / WAVES_M, WTN = BN / WAVES_N;
  constexpr int TM = WTM / 32, TN = WTN / 32;
  static_assert(WAVES_M * WAVES_N == 4, "4 waves per block");
  static_assert(TM >= 1 && TN >= 1, "wave tile >= 32x32");
  constexpr bool A_KC = MODE != MODE_WGRAD;  // A stored k-contiguous in global memory
  constexpr bool B_KC = MODE == MODE_FWD;
  constexpr int SA = A_KC ? BM + 2 : BM + 4;  // LDS row stride (floats); rows are k
  constexpr int SB = B_KC ? BN + 2 : BN + 4;
  constexpr int STAGE = BK * SA + BK * SB;
  // float4 staging slots per thread
  constexpr int QA = BM * BK / 4, QB = BN * BK / 4;
  constexpr int NQA = (QA + 255) / 256, NQB = (QB + 255) / 256;

  __shared__ __attribute__((aligned(16))) float lds[2 * STAGE];
  __shared__ short s_tdy[kMaxTaps], s_tdx[kMaxTaps];

  const int tid = threadIdx.x;
  if (tid < kMaxTaps) {
    s_tdy[tid] = p.tap_dy[tid];
    s_tdx[tid] = p.tap_dx[tid];
  }

  // Tile coordinates: blockIdx.x over (M tiles x N tiles), N fastest; blockIdx.y = split.
  const int ntn = (p.N + BN - 1) / BN;
  const int tm = blockIdx.x / ntn, tn = blockIdx.x - tm * ntn;
  const int bm = tm * BM, bn = tn * BN;
  const int split = blockIdx.y;
  const int nkt = (p.K + BK - 1) / BK;
  const int kt0 = split * p.ktiles_per_split;
  const int kt1 = min(nkt, kt0 + p.ktiles_per_split);

  __syncthreads();

  // Per-slot static info.
  RowInfo arow[NQA];
  int ak[NQA];     // k offset within tile (k-contig) or k row (mn-contig)
  int acol[NQA];   // row (k-contig) or column (mn-contig) within tile
  bool aact[NQA];
#pragma unroll
  for (int i = 0; i < NQA; ++i) {
    int q = tid + 256 * i;
    aact[i] = q < QA;
    if constexpr (A_KC) {
      acol[i] = q >> 2;          // row m within tile
      ak[i] = (q & 3) * 4;       // k offset
      if constexpr (MODE == MODE_FWD) arow[i] = fwd_row_info(p, bm + acol[i]);
      else arow[i] = dgrad_row_info(p, bm + acol[i]);
    } else {
      ak[i] = q / (BM / 4);
      acol[i] = (q % (BM / 4)) * 4;
    }
  }
  int bk_[NQB], bcol[NQB];
  bool bact[NQB];
  ColInfo bci[NQB][VB ? 1 : 4];
#pragma unroll
  for (int i = 0; i < NQB; ++i) {
    int q = tid + 256 * i;
    bact[i] = q < QB;
    if constexpr (B_KC) {
      bcol[i] = q >> 2;
      bk_[i] = (q & 3) * 4;
    } else {
      bk_[i] = q / (BN / 4);
      bcol[i] = (q % (BN / 4)) * 4;
      if constexpr (MODE == MODE_WGRAD) {
#pragma unroll
        for (int j = 0; j < (VB ? 1 : 4); ++j)
          bci[i][j] = wgrad_col_info(p, s_tdy, s_tdx, bn + bcol[i] + j);
      }
    }
  }

  float4 ra[NQA], rb[NQB];

  auto load_tile = [&](int kt) {
    const int kbase = kt * BK;
#pragma unroll
    for (int i = 0; i < NQA; ++i) {
      if (!aact[i]) continue;
      if constexpr (MODE == MODE_FWD) ra[i] = fwd_a_load<VA>(p, s_tdy, s_tdx, arow[i], kbase + ak[i]);
      else if constexpr (MODE == MODE_DGRAD) ra[i] = dgrad_a_load<VA>(p, s_tdy, s_tdx, arow[i], kbase + ak[i]);
      else ra[i] = wgrad_a_load<VA>(p, kbase + ak[i], bm + acol[i]);
    }
#pragma unroll
    for (int i = 0; i < NQB; ++i) {
      if (!bact[i]) continue;
      if constexpr (MODE == MODE_FWD) {
        rb[i] = fwd_b_load<VB>(p, bn + bcol[i], kbase + bk_[i]);
      } else if constexpr (MODE == MODE_DGRAD) {
        rb[i] = dgrad_b_load<VB>(p, kbase + bk_[i], bn + bcol[i]);
      } else {
        PixInfo q = wgrad_pix(p, kbase + bk_[i]);
        if constexpr (VB) {
          const ColInfo &c = bci[i][0];
          float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
          if (q.ok && c.ok) {
            int ih = q.y0 + c.dy, iw = q.x0 + c.dx;
            if ((unsigned)ih < (unsigned)p.h && (unsigned)iw < (unsigned)p.w)
              v = ld4(p.x + q.base + ih * p.sxh + iw * p.sxw + c.ci);
          }
          rb[i] = v;
        } else {
          rb[i] = make_float4(wgrad_b_elem(p, q, bci[i][0]), wgrad_b_elem(p, q, bci[i][1]),
                              wgrad_b_elem(p, q, bci[i][2]), wgrad_b_elem(p, q, bci[i][3]));
        }
      }
    }
  };

  auto store_tile = [&](int buf) {
    float *As = lds + buf * STAGE;
    float *Bs = As + BK * SA;
#pragma unroll
    for (int i = 0; i < NQA; ++i) {
      if (!aact[i]) continue;
      if constexpr (A_KC) {
        float *d = As + ak[i] * SA + acol[i];
        d[0] = ra[i].x;
        d[SA] = ra[i].y;
        d[2 * SA] = ra[i].z;
        d[3 * SA] = ra[i].w;
      } else {
        *reinterpret_cast<float4 *>(As + ak[i] * SA + acol[i]) = ra[i];
      }
    }
#pragma unroll
    for (int i = 0; i < NQB; ++i) {
      if (!bact[i]) continue;
      if constexpr (B_KC) {
        float *d = Bs + bk_[i] * SB + bcol[i];
        d[0] = rb[i].x;
        d[SB] = rb[i].y;
        d[2 * SB] = rb[i].z;
        d[3 * SB] = rb[i].w;
      } else {
        *reinterpret_cast<float4 *>(Bs + bk_[i] * SB + bcol[i]) = rb[i];
      }
    }
  };

  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WAVES_N, wn = wave - wm * WAVES_N;
  const int l32 = lane & 31, hh = lane >> 5;

  floatx16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  if (kt0 < kt1) {
    load_tile(kt0);
    store_tile(0);
    __syncthreads();
    int cur = 0;
    for (int kt = kt0; kt < kt1; ++kt) {
      const bool more = kt + 1 < kt1;
      if (more) load_tile(kt + 1);
      const float *As = lds + cur * STAGE + wm * WTM + l32;
      const float *Bs = lds + cur * STAGE + BK * SA + wn * WTN + l32;
#pragma unroll
      for (int kk = 0; kk < BK; kk += 2) {
        float a[TM], b[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) a[i] = As[(kk + hh) * SA + i * 32];
#pragma unroll
        for (int j = 0; j < TN; ++j) b[j] = Bs[(kk + hh) * SB + j * 32];
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i], b[j], acc[i][j], 0, 0, 0);
      }
      if (more) store_tile(cur ^ 1);
      __syncthreads();
      cur ^= 1;
    }
  }

  // ---------------- epilogue ----------------
  // acc[i][j][r] -> row = (r&3) + 8*(r>>2) + 4*hh, col = l32 within the 32x32 tile.
  if (p.splits > 1) {
    float *slab = p.out + (size_t)split * p.M * p.N;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        int col = bn + wn * WTN + j * 32 + l32;
        if (col >= p.N) continue;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          int row = bm + wm * WTM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
          if (row < p.M) slab[(size_t)row * p.N + col] = acc[i][j][r];
        }
      }
    return;
  }

  if constexpr (MODE == MODE_WGRAD) {
    const bool accum = p.flags & ADAPTSEG_EPI_ACCUMULATE;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      int col = bn + wn * WTN + j * 32 + l32;
      if (col >= p.N) continue;
      int seg = (int)fdiv((uint32_t)col, p.fd_nseg_k);
      int cc = col - seg * p.kseg;
      float *dst = seg == 0 ? p.dw[0] : seg == 1 ? p.dw[1] : seg == 2 ? p.dw[2] : p.dw[3];
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          int row = bm + wm * WTM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
          if (row >= p.M) continue;
          float *o = dst + (size_t)row * p.kseg + cc;
          float v = acc[i][j][r];
          *o = accum ? *o + v : v;
        }
    }
  } else {
    const int flags = p.flags;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      int col = bn + wn * WTN + j * 32 + l32;
      if (col >= p.N) continue;
      float bsum = 0.f;
      if constexpr (MODE == MODE_FWD) {
        for (int s = 0; s < p.nseg; ++s) {
          const float *bp = s == 0 ? p.bias[0] : s == 1 ? p.bias[1] : s == 2 ? p.bias[2] : p.bias[3];
          if (bp) bsum += bp[col];
        }
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          int row = bm + wm * WTM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
          if (row >= p.M) continue;
          size_t idx = (size_t)row * p.N + col;
          float v = acc[i][j][r] + bsum;
          if (flags & ADAPTSEG_EPI_ACCUMULATE) v += p.out[idx];
          if (flags & ADAPTSEG_EPI_RESIDUAL) v += p.res[idx];
          if (flags & ADAPTSEG_EPI_LEAKY) v = v > 0.f ? v : 0.2f * v;
          if (flags & ADAPTSEG_EPI_LEAKY_GRAD) v = p.aux[idx] > 0.f ? v : 0.2f * v;
          p.out[idx] = v;
        }
    }
  }
}

// ------------------------------------------------------------------------------------
// FAST path.  Preconditions (checked on the host): every BK-deep K tile of the A operand
// lies inside ONE tap (FWD: C % BK == 0; DGRAD: Cout % BK == 0 and stride 1), operands are
// NHWC with 16-B aligned float4 rows.  Then tap, channel offset and weight segment are
// tile-uniform scalars, and each lane's gather is one clamped, branch-free float4 load:
//   FWD A   x[b*sxn + (oh*s+dy)*sxh + (ow*s+dx)*sxw + ci0 + kq]   (pix_slot + s_off)
//   FWD B   w_seg[n*kseg + kk0 + kq]
//   DGRAD A dy[((b*OH+ih-dy)*OW + iw-dx)*Cout + co0 + kq]
//   DGRAD B w_seg[((co0+r)*taps + t)*C + n]
//   WGRAD A dy[m*Cout + co],   WGRAD B x[b, oh*s+dy, ow*s+dx, ci]  (per-column tap)
// ------------------------------------------------------------------------------------
__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }

__device__ __forceinline__ float4 sel4(bool ok, float4 v) {
  return ok ? v : make_float4(0.f, 0.f, 0.f, 0.f);
}

template <int MODE, int BM, int BN, int WAVES_M, int WAVES_N, int BK, bool S2>
__global__ void __launch_bounds__(256) igemm_fast_kernel(const ConvParams p) {
  constexpr int WTM = BM / WAVES_M, WTN = BN / WAVES_N;
  constexpr int TM = WTM / 32, TN = WTN / 32;
  static_assert(WAVES_M * WAVES_N == 4, "4 waves per block");
  static_assert(TM >= 1 && TN >= 1, "wave tile >= 32x32");
  constexpr bool A_KC = MODE != MODE_WGRAD;
  constexpr bool B_KC = MODE == MODE_FWD;
  constexpr int SA = A_KC ? BM + 2 : BM + 4;
  constexpr int SB = B_KC ? BN + 2 : BN + 4;
  constexpr int STAGE = BK * SA + BK * SB;
  constexpr int QA = BM * BK / 4, QB = BN * BK / 4;
  constexpr int NQA = (QA + 255) / 256, NQB = (QB + 255) / 256;
  constexpr int KQ = BK / 4;  // float4 per k-contiguous row
  static_assert(QA % 256 == 0 && QB % 256 == 0, "every thread stages whole float4 slots");

  __shared__ __attribute__((aligned(16))) float lds[2 * STAGE];

  const int tid = threadIdx.x;
  const int ntn = (p.N + BN - 1) / BN;
  const int tm = blockIdx.x / ntn, tn = blockIdx.x - tm * ntn;
  const int bm = tm * BM, bn = tn * BN;
  const int split = blockIdx.y;

  // Stride-2 data gradient: blockIdx.z = output-pixel parity class (py, px).  The class's
  // pixels (2i+py, 2j+px) form a dense (Hc x Wc) grid that only the taps kh = kh0 + 2u,
  // kw = kw0 + 2v reach (dil 1), at dY row i + (py+pad-kh)/2: a stride-1 problem with
  // K = nkh*nkw*Cout and no zero-stuffed work.
  int M = p.M, K = p.K, Hc = p.h, Wc = p.w, py = 0, px = 0, kh0 = 0, kw0 = 0, nkw = p.kw_;
  if constexpr (S2) {
    py = blockIdx.z >> 1;
    px = blockIdx.z & 1;
    Hc = (p.h - py + 1) >> 1;
    Wc = (p.w - px + 1) >> 1;
    kh0 = (py + p.pad_[0]) & 1;
    kw0 = (px + p.pad_[0]) & 1;
    const int nkh = (p.kh_ - kh0 + 1) >> 1;
    nkw = (p.kw_ - kw0 + 1) >> 1;
    M = p.n * Hc * Wc;
    K = nkh * nkw * p.k;
    if (bm >= M) return;
  }
  const int nkt = (K + BK - 1) / BK;
  const int kt0 = split * p.ktiles_per_split;
  const int kt1 = min(nkt, kt0 + p.ktiles_per_split);

  // ---- per-slot constants ----
  int a_pix[NQA], a_y[NQA], a_x[NQA], a_col[NQA], a_k[NQA];
  bool a_ok[NQA];
#pragma unroll
  for (int i = 0; i < NQA; ++i) {
    const int q = tid + 256 * i;
    if constexpr (A_KC) {
      const int row = q / KQ;
      a_col[i] = row;
      a_k[i] = (q % KQ) * 4;
      const int m = bm + row;
      a_ok[i] = m < M;
      const int mm = min(m, M - 1);
      if constexpr (S2) {
        const int j = mm % Wc, t2 = mm / Wc;
        const int ii = t2 % Hc, b = t2 / Hc;
        a_y[i] = ii;
        a_x[i] = j;
        a_pix[i] = ((b * p.oh + ii) * p.ow + j) * p.k + a_k[i];
      } else if constexpr (MODE == MODE_FWD) {
        uint32_t t = fdiv((uint32_t)mm, p.fd_ow);
        const int ow = mm - (int)t * p.ow;
        uint32_t b = fdiv(t, p.fd_oh);
        const int oh = (int)t - (int)b * p.oh;
        a_y[i] = oh * p.stride;
        a_x[i] = ow * p.stride;
        a_pix[i] = (int)b * p.sxn + a_y[i] * p.sxh + a_x[i] * p.sxw + a_k[i];
      } else {  // DGRAD, stride 1
        uint32_t t = fdiv((uint32_t)mm, p.fd_w);
        const int iw = mm - (int)t * p.w;
        uint32_t b = fdiv(t, p.fd_hw);
        const int ih = (int)t - (int)b * p.h;
        a_y[i] = ih;
        a_x[i] = iw;
        a_pix[i] = (((int)b * p.oh + ih) * p.ow + iw) * p.k + a_k[i];
      }
    } else {  // WGRAD A': rows k' = pixel, columns = output channel
      a_k[i] = q / (BM / 4);
      a_col[i] = (q % (BM / 4)) * 4;
      const int col = bm + a_col[i];
      a_ok[i] = col < p.M;
      a_pix[i] = a_ok[i] ? col : 0;
    }
  }
  int b_off[NQB], b_col[NQB], b_k[NQB], b_dy[NQB], b_dx[NQB];
  bool b_ok[NQB];
#pragma unroll
  for (int i = 0; i < NQB; ++i) {
    const int q = tid + 256 * i;
    if constexpr (B_KC) {  // FWD B: rows n, k contiguous
      const int row = q / KQ;
      b_col[i] = row;
      b_k[i] = (q % KQ) * 4;
      const int n = bn + row;
      b_ok[i] = n < p.N;
      b_off[i] = min(n, p.N - 1) * p.kseg + b_k[i];
    } else {
      b_k[i] = q / (BN / 4);
      b_col[i] = (q % (BN / 4)) * 4;
      const int n = bn + b_col[i];
      b_ok[i] = n < p.N;
      const int nn = b_ok[i] ? n : 0;
      if constexpr (MODE == MODE_DGRAD) {
        b_off[i] = b_k[i] * p.taps_per_seg * p.c + nn;
      } else {  // WGRAD B': column (tap, ci)
        const int tap = (int)fdiv((uint32_t)nn, p.fd_c);
        const int ci = nn - tap * p.c;
        const int seg = (int)fdiv((uint32_t)tap, p.fd_taps);
        const int t = tap - seg * p.taps_per_seg;
        const int kh = (int)fdiv((uint32_t)t, p.fd_kw);
        const int kw = t - kh * p.kw_;
        const int dil = seg == 0 ? p.dil_[0] : seg == 1 ? p.dil_[1] : seg == 2 ? p.dil_[2] : p.dil_[3];
        const int pad = seg == 0 ? p.pad_[0] : seg == 1 ? p.pad_[1] : seg == 2 ? p.pad_[2] : p.pad_[3];
        b_dy[i] = kh * dil - pad;
        b_dx[i] = kw * dil - pad;
        b_off[i] = ci;
      }
    }
  }

  float4 ra[NQA], rb[NQB];
  bool ma[NQA], mb[NQB];  // validity, applied when the staged tile is written to LDS

  // Tile-uniform tap -> (segment, dy, dx) on the scalar unit.
  auto tap_geom = [&](int tap, int &seg, int &t, int &dy, int &dx) {
    seg = uni((int)fdiv((uint32_t)tap, p.fd_taps));
    t = tap - seg * p.taps_per_seg;
    const int kh = (int)fdiv((uint32_t)t, p.fd_kw);
    const int kw = t - kh * p.kw_;
    const int dil = seg == 0 ? p.dil_[0] : seg == 1 ? p.dil_[1] : seg == 2 ? p.dil_[2] : p.dil_[3];
    const int pad = seg == 0 ? p.pad_[0] : seg == 1 ? p.pad_[1] : seg == 2 ? p.pad_[2] : p.pad_[3];
    dy = uni(kh * dil - pad);
    dx = uni(kw * dil - pad);
  };

  auto load_tile = [&](int kt) {
    const int kbase = kt * BK;
    if constexpr (MODE == MODE_FWD) {
      const int tap = uni((int)fdiv((uint32_t)kbase, p.fd_c));
      int seg, t, dy, dx;
      tap_geom(tap, seg, t, dy, dx);
      const int soff = uni(dy * p.sxh + dx * p.sxw + kbase - tap * p.c);
#pragma unroll
      for (int i = 0; i < NQA; ++i) {
        ma[i] = a_ok[i] && (unsigned)(a_y[i] + dy) < (unsigned)p.h &&
                (unsigned)(a_x[i] + dx) < (unsigned)p.w;
        ra[i] = ld4(p.x + (ma[i] ? a_pix[i] + soff : 0));
      }
      const float *wp = seg_ptr(p, seg) + (kbase - seg * p.kseg);
#pragma unroll
      for (int i = 0; i < NQB; ++i) {
        mb[i] = b_ok[i];
        rb[i] = ld4(wp + b_off[i]);
      }
    } else if constexpr (MODE == MODE_DGRAD) {
      const int tap = uni((int)fdiv((uint32_t)kbase, p.fd_k));
      const int co0 = kbase - tap * p.k;
      int seg, t, dy, dx;
      if constexpr (S2) {
        const int u = tap / nkw, v = tap - u * nkw;
        const int kh = kh0 + 2 * u, kw = kw0 + 2 * v;
        seg = 0;
        t = uni(kh * p.kw_ + kw);
        dy = uni(-((py + p.pad_[0] - kh) >> 1));  // dY row = i - dy
        dx = uni(-((px + p.pad_[0] - kw) >> 1));
      } else {
        tap_geom(tap, seg, t, dy, dx);
      }
      const int soff = uni(co0 - (dy * p.ow + dx) * p.k);
#pragma unroll
      for (int i = 0; i < NQA; ++i) {
        ma[i] = a_ok[i] && (unsigned)(a_y[i] - dy) < (unsigned)p.oh &&
                (unsigned)(a_x[i] - dx) < (unsigned)p.ow;
        ra[i] = ld4(p.dy + (ma[i] ? a_pix[i] + soff : 0));
      }
      const float *wp = seg_ptr(p, seg) + (co0 * p.taps_per_seg + t) * p.c;
#pragma unroll
      for (int i = 0; i < NQB; ++i) {
        mb[i] = b_ok[i];
        rb[i] = ld4(wp + b_off[i]);
      }
    } else {  // WGRAD
#pragma unroll
      for (int i = 0; i < NQA; ++i) {
        const int m = kbase + a_k[i];
        ma[i] = a_ok[i] && m < p.K;
        ra[i] = ld4(p.dy + (size_t)(ma[i] ? m : 0) * p.k + a_pix[i]);
      }
#pragma unroll
      for (int i = 0; i < NQB; ++i) {
        const int m = kbase + b_k[i];
        const int mm = min(m, p.K - 1);
        uint32_t t = fdiv((uint32_t)mm, p.fd_ow);
        const int ow = mm - (int)t * p.ow;
        uint32_t b = fdiv(t, p.fd_oh);
        const int oh = (int)t - (int)b * p.oh;
        const int iy = oh * p.stride + b_dy[i], ix = ow * p.stride + b_dx[i];
        mb[i] = b_ok[i] && m < p.K && (unsigned)iy < (unsigned)p.h && (unsigned)ix < (unsigned)p.w;
        rb[i] = ld4(p.x + (mb[i] ? (int)b * p.sxn + iy * p.sxh + ix * p.sxw + b_off[i] : 0));
      }
    }
  };

  auto store_tile = [&](int buf) {
    float *As = lds + buf * STAGE;
    float *Bs = As + BK * SA;
#pragma unroll
    for (int i = 0; i < NQA; ++i) {
      const float4 v = sel4(ma[i], ra[i]);
      if constexpr (A_KC) {
        float *d = As + a_k[i] * SA + a_col[i];
        d[0] = v.x;
        d[SA] = v.y;
        d[2 * SA] = v.z;
        d[3 * SA] = v.w;
      } else {
        *reinterpret_cast<float4 *>(As + a_k[i] * SA + a_col[i]) = v;
      }
    }
#pragma unroll
    for (int i = 0; i < NQB; ++i) {
      const float4 v = sel4(mb[i], rb[i]);
      if constexpr (B_KC) {
        float *d = Bs + b_k[i] * SB + b_col[i];
        d[0] = v.x;
        d[SB] = v.y;
        d[2 * SB] = v.z;
        d[3 * SB] = v.w;
      } else {
        *reinterpret_cast<float4 *>(Bs + b_k[i] * SB + b_col[i]) = v;
      }
    }
  };

  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WAVES_N, wn = wave - wm * WAVES_N;
  const int l32 = lane & 31, hh = lane >> 5;

  floatx16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  if (kt0 < kt1) {
    load_tile(kt0);
    store_tile(0);
    __syncthreads();
    int cur = 0;
    for (int kt = kt0; kt < kt1; ++kt) {
      const bool more = kt + 1 < kt1;
      if (more) load_tile(kt + 1);
      const float *As = lds + cur * STAGE + wm * WTM + l32;
      const float *Bs = lds + cur * STAGE + BK * SA + wn * WTN + l32;
#pragma unroll
      for (int kk = 0; kk < BK; kk += 2) {
        float a[TM], b[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) a[i] = As[(kk + hh) * SA + i * 32];
#pragma unroll
        for (int j = 0; j < TN; ++j) b[j] = Bs[(kk + hh) * SB + j * 32];
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i], b[j], acc[i][j], 0, 0, 0);
      }
      if (more) store_tile(cur ^ 1);
      __syncthreads();
      cur ^= 1;
    }
  }

  // ---- epilogue ----
  const bool full = (bm + BM <= M) && (bn + BN <= p.N);
  // output row of GEMM row `row` (S2: scatter the parity class back into the NHWC image)
  auto out_row = [&](int row) -> size_t {
    if constexpr (S2) {
      const int j = row % Wc, t2 = row / Wc;
      const int ii = t2 % Hc, b = t2 / Hc;
      return ((size_t)(b * p.h + 2 * ii + py) * p.w + 2 * j + px);
    } else {
      return (size_t)row;
    }
  };
  if (p.splits > 1) {
    float *slab = p.out + (size_t)split * p.M * p.N;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int col = bn + wn * WTN + j * 32 + l32;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = bm + wm * WTM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
          if (full || (row < p.M && col < p.N)) slab[(size_t)row * p.N + col] = acc[i][j][r];
        }
      }
    return;
  }
  if constexpr (MODE == MODE_WGRAD) {
    const bool accum = p.flags & ADAPTSEG_EPI_ACCUMULATE;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int col = bn + wn * WTN + j * 32 + l32;
      if (!full && col >= p.N) continue;
      const int seg = (int)fdiv((uint32_t)col, p.fd_nseg_k);
      const int cc = col - seg * p.kseg;
      float *dst = (seg == 0 ? p.dw[0] : seg == 1 ? p.dw[1] : seg == 2 ? p.dw[2] : p.dw[3]) + cc;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = bm + wm * WTM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
          if (!full && row >= p.M) continue;
          float *o = dst + (size_t)row * p.kseg;
          const float v = acc[i][j][r];
          *o = accum ? *o + v : v;
        }
    }
  } else {
    const int flags = p.flags;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int col = bn + wn * WTN + j * 32 + l32;
      if (!full && col >= p.N) continue;
      float bsum = 0.f;
      if constexpr (MODE == MODE_FWD) {
        for (int s = 0; s < p.nseg; ++s) {
          const float *bp = s == 0 ? p.bias[0] : s == 1 ? p.bias[1] : s == 2 ? p.bias[2] : p.bias[3];
          if (bp) bsum += bp[col];
        }
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = bm + wm * WTM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
          if (!full && row >= M) continue;
          const size_t idx = out_row(row) * p.N + col;
          float v = acc[i][j][r] + bsum;
          if (flags & ADAPTSEG_EPI_ACCUMULATE) v += p.out[idx];
          if (flags & ADAPTSEG_EPI_RESIDUAL) v += p.res[idx];
          if (flags & ADAPTSEG_EPI_LEAKY) v = v > 0.f ? v : 0.2f * v;
          if (flags & ADAPTSEG_EPI_LEAKY_GRAD) v = p.aux[idx] > 0.f ? v : 0.2f * v;
          p.out[idx] = v;
        }
    }
  }
}

// Split-K reduction + epilogue.  One thread per output element, slabs summed in order.
__global__ void splitk_reduce_kernel(const ConvParams p, const float *slab, int mode) {
  const size_t total = (size_t)p.M * p.N;
  for (size_t idx = blockIdx.x * (size_t)blockDim.x + threadIdx.x; idx < total;
       idx += (size_t)gridDim.x * blockDim.x) {
    float v = 0.f;
    for (int s = 0; s < p.splits; ++s) v += slab[(size_t)s * total + idx];
    int row = (int)(idx / p.N);
    int col = (int)(idx - (size_t)row * p.N);
    if (mode == MODE_WGRAD) {
      int seg = (int)fdiv((uint32_t)col, p.fd_nseg_k);
      int cc = col - seg * p.kseg;
      float *dst = seg == 0 ? p.dw[0] : seg == 1 ? p.dw[1] : seg == 2 ? p.dw[2] : p.dw[3];
      float *o = dst + (size_t)row * p.kseg + cc;
      *o = (p.flags & ADAPTSEG_EPI_ACCUMULATE) ? *o + v : v;
    } else {
      if (mode == MODE_FWD) {
        for (int s = 0; s < p.nseg; ++s) {
          const float *bp = s == 0 ? p.bias[0] : s == 1 ? p.bias[1] : s == 2 ? p.bias[2] : p.bias[3];
          if (bp) v += bp[col];
        }
      }
      if (p.flags & ADAPTSEG_EPI_ACCUMULATE) v += p.out[idx];
      if (p.flags & ADAPTSEG_EPI_RESIDUAL) v += p.res[idx];
      if (p.flags & ADAPTSEG_EPI_LEAKY) v = v > 0.f ? v : 0.2f * v;
      if (p.flags & ADAPTSEG_EPI_LEAKY_GRAD) v = p.aux[idx] > 0.f ? v : 0.2f * v;
      p.out[idx] = v;
    }
  }
}

// Bias gradient: db[seg][co] (+)= sum_m dY[m][co].  One block per 64-channel strip x row split.
__global__ void bias_grad_partial_kernel(const float *dy, int rows, int cout, int rows_per_split,
                                         float *partial) {
  // block: 256 threads = 64 channels x 4 row lanes
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int rl = threadIdx.x >> 6;
  const int r0 = blockIdx.y * rows_per_split;
  const int r1 = min(rows, r0 + rows_per_split);
  float s = 0.f;
  if (c < cout)
    for (int r = r0 + rl; r < r1; r += 4) s += dy[(size_t)r * cout + c];
  __shared__ float red[256];
  red[threadIdx.x] = s;
  __syncthreads();
  if (rl == 0 && c < cout) {
    float t = red[threadIdx.x] + red[threadIdx.x + 64] + red[threadIdx.x + 128] + red[threadIdx.x + 192];
    partial[(size_t)blockIdx.y * cout + c] = t;
  }
}

struct BiasOut {
  float *db[4];
};

__global__ void bias_grad_final_kernel(const float *partial, int splits, int cout, BiasOut o, int nseg,
                                       int accumulate) {
  int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= cout) return;
  double s = 0.0;
  for (int i = 0; i < splits; ++i) s += partial[(size_t)i * cout + c];
  for (int g = 0; g < nseg; ++g) {
    float *d = o.db[g];
    if (!d) continue;
    d[c] = accumulate ? d[c] + (float)s : (float)s;
  }
}

// ------------------------------------------------------------------------------------
// Live timing (benchmark roofline): hipEvent pairs around selected launches.
// ------------------------------------------------------------------------------------
struct TimingState {
  std::mutex mu;
  bool enabled = false;
  int selector = -1;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> events;
  std::vector<double> flops;
  size_t used = 0;
};
static TimingState g_timing;

static void timing_begin(int kernel_id, hipStream_t s, double fl, int *slot) {
  *slot = -1;
  if (!g_timing.enabled) return;
  if (g_timing.selector >= 0 && g_timing.selector != kernel_id) return;
  std::lock_guard<std::mutex> lk(g_timing.mu);
  if (g_timing.used == g_timing.events.size()) {
    hipEvent_t a, b;
    if (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess) return;
    g_timing.events.push_back({a, b});
    g_timing.flops.push_back(0.0);
  }
  *slot = (int)g_timing.used++;
  g_timing.flops[*slot] = fl;
  (void)hipEventRecord(g_timing.events[*slot].first, s);
}

static void timing_end(int slot, hipStream_t s) {
  if (slot < 0) return;
  (void)hipEventRecord(g_timing.events[slot].second, s);
}

// ------------------------------------------------------------------------------------
// Host side
// ------------------------------------------------------------------------------------
struct Plan {
  ConvParams p;
  int cfg;        // 0: 128x128 (2x2), 1: 256x32 (4x1), 2: 32x256 (1x4), 3: 64x256 (1x4)
  bool va, vb;
  bool fast;
  bool s2;     // stride-2 data gradient by output-pixel parity class (grid.z = 4)
  int bk;
  int mode;
  int tiles;
  size_t slab_bytes;
  double flops;  // algorithmic FLOPs of the conv product this plan computes
};

static int validate(const adaptseg_conv_desc *d) {
  AS_CHECK_ARG(d, "null conv desc");
  AS_CHECK_ARG(d->n > 0 && d->c > 0 && d->h > 0 && d->w > 0 && d->k > 0, "conv: bad input/output dims");
  AS_CHECK_ARG(d->oh > 0 && d->ow > 0 && d->kh > 0 && d->kw > 0 && d->stride > 0, "conv: bad geometry");
  AS_CHECK_ARG(d->nseg >= 1 && d->nseg <= 4, "conv: nseg must be 1..4");
  AS_CHECK_ARG(d->nseg * d->kh * d->kw <= kMaxTaps, "conv: too many taps (%d)", d->nseg * d->kh * d->kw);
  for (int s = 0; s < d->nseg; ++s) {
    AS_CHECK_ARG(d->dil[s] >= 1 && d->pad[s] >= 0, "conv: bad pad/dil");
    int eh = (d->h + 2 * d->pad[s] - d->dil[s] * (d->kh - 1) - 1) / d->stride + 1;
    int ew = (d->w + 2 * d->pad[s] - d->dil[s] * (d->kw - 1) - 1) / d->stride + 1;
    AS_CHECK_ARG(eh == d->oh && ew == d->ow, "conv: output size %dx%d != expected %dx%d (seg %d)", d->oh,
                 d->ow, eh, ew, s);
  }
  int64_t in_elems = (int64_t)d->n * d->c * d->h * d->w;
  int64_t out_elems = (int64_t)d->n * d->k * d->oh * d->ow;
  AS_CHECK_ARG(in_elems < (1ll << 31) && out_elems < (1ll << 31), "conv: tensor too large for int32 indexing");
  return ADAPTSEG_OK;
}

static void fill_common(ConvParams &p, const adaptseg_conv_desc *d) {
  memset(&p, 0, sizeof(p));
  p.n = d->n; p.c = d->c; p.h = d->h; p.w = d->w;
  p.sxn = (int)d->in_stride[0]; p.sxc = (int)d->in_stride[1];
  p.sxh = (int)d->in_stride[2]; p.sxw = (int)d->in_stride[3];
  p.k = d->k; p.oh = d->oh; p.ow = d->ow;
  p.stride = d->stride;
  p.taps_per_seg = d->kh * d->kw;
  p.nseg = d->nseg;
  p.ntaps = p.taps_per_seg * d->nseg;
  int t = 0;
  for (int s = 0; s < d->nseg; ++s)
    for (int i = 0; i < d->kh; ++i)
      for (int j = 0; j < d->kw; ++j, ++t) {
        p.tap_dy[t] = (short)(i * d->dil[s] - d->pad[s]);
        p.tap_dx[t] = (short)(j * d->dil[s] - d->pad[s]);
      }
  p.kw_ = d->kw;
  p.kh_ = d->kh;
  for (int s = 0; s < 4; ++s) {
    p.pad_[s] = s < d->nseg ? d->pad[s] : 0;
    p.dil_[s] = s < d->nseg ? d->dil[s] : 1;
  }
  p.fd_taps = make_fastdiv(p.taps_per_seg);
  p.fd_kw = make_fastdiv(d->kw);
  p.fd_c = make_fastdiv(d->c);
  p.fd_k = make_fastdiv(d->k);
  p.fd_ow = make_fastdiv(d->ow);
  p.fd_oh = make_fastdiv(d->oh);
  p.fd_w = make_fastdiv(d->w);
  p.fd_hw = make_fastdiv(d->h);
}

static double conv_flops(const adaptseg_conv_desc *d) {
  return 2.0 * d->n * d->oh * d->ow * (double)d->k * d->c * d->kh * d->kw * d->nseg;
}

// tile configs: 0 = 128x128 (2x2 waves), 1 = 256x32 (4x1), 2 = 32x256 (1x4), 3 = 64x256 (1x4),
// 4 = 256x64 (4x1).  Every wave owns a 64x64, 64x32 or 32x64 block of 32x32x2 MFMA tiles.
static const int kCfgBM[5] = {128, 256, 32, 64, 256};
static const int kCfgBN[5] = {128, 32, 256, 256, 64};
// K step of the FAST kernel per config (LDS: 2 stages x BK x (BM+BN+pad) floats)
static int fast_bk(int cfg) { return cfg == 4 ? 16 : 32; }

// Grid decomposition: tiles, then split K until the grid has ~2 blocks per CU while keeping
// >= 8 K-steps per split.  Depends on the K step of the chosen kernel (pl.bk).
static void set_splits(Plan &pl) {
  ConvParams &p = pl.p;
  const int bm = kCfgBM[pl.cfg], bn = kCfgBN[pl.cfg];
  pl.bk = pl.fast ? fast_bk(pl.cfg) : BK;
  if (!pl.fast) pl.s2 = false;
  if (pl.s2) {  // rows of the largest parity class; K of the largest tap subset; no K split
    p.M = p.n * ((p.h + 1) / 2) * ((p.w + 1) / 2);
    p.K = ((p.kh_ + 1) / 2) * ((p.kw_ + 1) / 2) * p.k;
  } else if (pl.mode == MODE_DGRAD) {
    p.M = p.n * p.h * p.w;
    p.K = p.ntaps * p.k;
  }
  pl.tiles = (int)(ceil_div(p.M, bm) * ceil_div(p.N, bn));
  const int nkt = (int)ceil_div(p.K, pl.bk);
  // fwd / data-grad: ~2 blocks per CU; weight-grad (K = every output pixel, few tiles): ~4.
  // >= 4 K-steps per split keeps the slab traffic small next to the GEMM.
  const int target = pl.mode == MODE_WGRAD ? 1024 : 512;
  int splits = 1;
  if (pl.tiles < target && !pl.s2) {
    splits = (int)ceil_div(target, pl.tiles);
    splits = std::min(splits, std::max(1, nkt / 4));
    splits = std::min(splits, 256);
  }
  int per = (int)ceil_div(nkt, splits);
  splits = (int)ceil_div(nkt, per);
  p.splits = splits;
  p.ktiles_per_split = per;
  pl.slab_bytes = splits > 1 ? (size_t)splits * p.M * p.N * sizeof(float) : 0;
}

static int make_plan(const adaptseg_conv_desc *d, int op, Plan &pl) {
  int st = validate(d);
  if (st) return st;
  ConvParams &p = pl.p;
  fill_common(p, d);
  pl.mode = op;
  const bool nhwc_in = d->in_stride[1] == 1;
  if (op == ADAPTSEG_CONV_FWD) {
    p.M = d->n * d->oh * d->ow;
    p.N = d->k;
    p.K = p.ntaps * d->c;
    p.kseg = p.taps_per_seg * d->c;
    pl.va = nhwc_in && d->c % 4 == 0;
    pl.vb = d->c % 4 == 0;
    pl.cfg = p.N <= 32 ? 1 : (p.N <= 64 ? 4 : 0);
  } else if (op == ADAPTSEG_CONV_BWD_DATA) {
    p.M = d->n * d->h * d->w;
    p.N = d->c;
    p.K = p.ntaps * d->k;
    p.kseg = p.taps_per_seg * d->c;
    pl.va = d->k % 4 == 0;
    pl.vb = d->c % 4 == 0;
    pl.cfg = p.N <= 32 ? 1 : (p.N <= 64 ? 4 : 0);
  } else if (op == ADAPTSEG_CONV_BWD_WEIGHT) {
    p.M = d->k;
    p.N = p.ntaps * d->c;
    p.K = d->n * d->oh * d->ow;
    p.kseg = p.taps_per_seg * d->c;
    pl.va = d->k % 4 == 0;
    pl.vb = nhwc_in && d->c % 4 == 0;
    pl.cfg = p.M <= 32 ? 2 : (p.M <= 64 ? 3 : 0);
  } else {
    set_error("conv: bad op %d", op);
    return ADAPTSEG_ERR_ARG;
  }
  p.fd_nseg_k = make_fastdiv(p.kseg);
  pl.flops = conv_flops(d);
  // FAST path eligibility (alignment re-checked at launch)
  const int fbk = fast_bk(pl.cfg);
  pl.s2 = false;
  if (op == ADAPTSEG_CONV_FWD) {
    pl.fast = nhwc_in && d->c % fbk == 0;
  } else if (op == ADAPTSEG_CONV_BWD_DATA) {
    pl.s2 = d->stride == 2 && d->nseg == 1 && d->dil[0] == 1;
    pl.fast = (d->stride == 1 || pl.s2) && d->k % fbk == 0 && d->c % 4 == 0;
  } else {
    pl.fast = nhwc_in && d->c % 4 == 0 && d->k % 4 == 0;
  }
  set_splits(pl);
  return ADAPTSEG_OK;
}

template <int MODE>
static hipError_t launch_cfg(const Plan &pl, hipStream_t s) {
  dim3 grid(pl.tiles, pl.p.splits, pl.s2 ? 4 : 1), block(256);
#define AS_LAUNCH(BM_, BN_, WM_, WN_, FBK_)                                                                  \
  do {                                                                                                       \
    if (pl.fast && pl.s2) {                                                                                  \
      if constexpr (MODE == MODE_DGRAD)                                                                      \
        igemm_fast_kernel<MODE, BM_, BN_, WM_, WN_, FBK_, true><<<grid, block, 0, s>>>(pl.p);               \
    } else if (pl.fast) {                                                                                    \
      igemm_fast_kernel<MODE, BM_, BN_, WM_, WN_, FBK_, false><<<grid, block, 0, s>>>(pl.p);                \
    } else if (pl.va && pl.vb) {                                                                             \
      igemm_kernel<MODE, BM_, BN_, WM_, WN_, true, true><<<grid, block, 0, s>>>(pl.p);                       \
    } else if (pl.va) {                                                                                      \
      igemm_kernel<MODE, BM_, BN_, WM_, WN_, true, false><<<grid, block, 0, s>>>(pl.p);                      \
    } else if (pl.vb) {                                                                                      \
      igemm_kernel<MODE, BM_, BN_, WM_, WN_, false, true><<<grid, block, 0, s>>>(pl.p);                      \
    } else {                                                                                                 \
      igemm_kernel<MODE, BM_, BN_, WM_, WN_, false, false><<<grid, block, 0, s>>>(pl.p);                     \
    }                                                                                                        \
  } while (0)
  switch (pl.cfg) {
    case 0: AS_LAUNCH(128, 128, 2, 2, 32); break;
    case 1: AS_LAUNCH(256, 32, 4, 1, 32); break;
    case 2: AS_LAUNCH(32, 256, 1, 4, 32); break;
    case 3: AS_LAUNCH(64, 256, 1, 4, 32); break;
    default: AS_LAUNCH(256, 64, 4, 1, 16); break;
  }
#undef AS_LAUNCH
  return hipGetLastError();
}

static int kernel_id(const Plan &pl, int mode) {
  return 100 * mode + 10 * pl.cfg + (pl.fast ? (pl.s2 ? 5 : 4) : (pl.va ? 2 : 0) + (pl.vb ? 1 : 0));
}

static int run_plan(Plan &pl, int mode, void *ws, size_t ws_bytes, hipStream_t s) {
  float *final_out = pl.p.out;
  if (pl.p.splits > 1) {
    if (!ws || ws_bytes < pl.slab_bytes) {
      set_error("conv: workspace %zu < required %zu", ws_bytes, pl.slab_bytes);
      return ADAPTSEG_ERR_WORKSPACE;
    }
    pl.p.out = reinterpret_cast<float *>(ws);
  }
  hipError_t e;
  int slot;
  timing_begin(kernel_id(pl, mode), s, pl.flops, &slot);
  if (mode == MODE_FWD) e = launch_cfg<MODE_FWD>(pl, s);
  else if (mode == MODE_DGRAD) e = launch_cfg<MODE_DGRAD>(pl, s);
  else e = launch_cfg<MODE_WGRAD>(pl, s);
  timing_end(slot, s);
  if (e != hipSuccess) {
    set_error("igemm launch: %s", hipGetErrorString(e));
    return ADAPTSEG_ERR_HIP;
  }
  if (pl.p.splits > 1) {
    const float *slab = reinterpret_cast<const float *>(ws);
    ConvParams q = pl.p;
    q.out = final_out;
    size_t total = (size_t)q.M * q.N;
    int blocks = (int)std::min<size_t>(ceil_div(total, 256), 4096);
    splitk_reduce_kernel<<<blocks, 256, 0, s>>>(q, slab, mode);
    AS_CHECK_LAUNCH("splitk_reduce");
  }
  return ADAPTSEG_OK;
}


}  // namespace adaptseg

using namespace adaptseg;

extern "C" {

int adaptseg_conv2d_workspace_size(const adaptseg_conv_desc *d, int op, size_t *bytes) {
  AS_CHECK_ARG(bytes, "null bytes");
  Plan pl;
  int st = make_plan(d, op, pl);
  if (st) return st;
  size_t b = pl.slab_bytes;
  if (pl.fast) {  // an unaligned operand at launch time falls back to the generic kernel
    Plan g = pl;
    g.fast = false;
    set_splits(g);
    b = std::max(b, g.slab_bytes);
  }
  if (op == ADAPTSEG_CONV_BWD_WEIGHT) {
    // bias-gradient partials
    int rows = d->n * d->oh * d->ow;
    int splits = (int)std::min<int64_t>(ceil_div(rows, 2048), 256);
    b = std::max(b, (size_t)splits * d->k * sizeof(float));
  }
  *bytes = b;
  return ADAPTSEG_OK;
}

int adaptseg_conv2d_kernel_id(const adaptseg_conv_desc *d, int op, int *kernel_id, int *splits) {
  AS_CHECK_ARG(kernel_id && splits, "conv2d_kernel_id: null");
  Plan pl;
  int st = make_plan(d, op, pl);
  if (st) return st;
  // alignment-dependent downgrades are not known here; report the aligned choice
  *kernel_id = ::adaptseg::kernel_id(pl, op);
  *splits = pl.p.splits;
  return ADAPTSEG_OK;
}

int adaptseg_conv2d_fwd(const adaptseg_conv_desc *d, const float *x, const float *const *w,
                        const float *const *bias, const float *res, float *y, int flags, void *ws,
                        size_t ws_bytes, adaptseg_stream_t stream) {
  Plan pl;
  int st = make_plan(d, ADAPTSEG_CONV_FWD, pl);
  if (st) return st;
  AS_CHECK_ARG(x && w && y, "conv fwd: null pointer");
  AS_CHECK_ARG(!(flags & (ADAPTSEG_EPI_LEAKY_GRAD)), "conv fwd: LEAKY_GRAD not valid");
  AS_CHECK_ARG(!(flags & ADAPTSEG_EPI_RESIDUAL) || res, "conv fwd: residual flag without res");
  ConvParams &p = pl.p;
  p.x = x;
  for (int s = 0; s < d->nseg; ++s) {
    AS_CHECK_ARG(w[s], "conv fwd: null weight %d", s);
    p.wt[s] = w[s];
    p.bias[s] = bias ? bias[s] : nullptr;
    if (reinterpret_cast<uintptr_t>(w[s]) & 15) pl.vb = pl.fast = false;
  }
  if (reinterpret_cast<uintptr_t>(x) & 15) pl.va = pl.fast = false;
  set_splits(pl);
  p.out = y;
  p.res = res;
  p.flags = flags;
  return run_plan(pl, MODE_FWD, ws, ws_bytes, as_stream(stream));
}

int adaptseg_conv2d_bwd_data(const adaptseg_conv_desc *d, const float *dy, const float *const *w,
                             const float *res, const float *aux, float *dx, int flags, void *ws,
                             size_t ws_bytes, adaptseg_stream_t stream) {
  Plan pl;
  int st = make_plan(d, ADAPTSEG_CONV_BWD_DATA, pl);
  if (st) return st;
  AS_CHECK_ARG(dy && w && dx, "conv bwd_data: null pointer");
  AS_CHECK_ARG(!(flags & ADAPTSEG_EPI_LEAKY), "conv bwd_data: LEAKY not valid");
  AS_CHECK_ARG(!(flags & ADAPTSEG_EPI_RESIDUAL) || res, "conv bwd_data: residual flag without res");
  AS_CHECK_ARG(!(flags & ADAPTSEG_EPI_LEAKY_GRAD) || aux, "conv bwd_data: LEAKY_GRAD without aux");
  ConvParams &p = pl.p;
  p.dy = dy;
  for (int s = 0; s < d->nseg; ++s) {
    AS_CHECK_ARG(w[s], "conv bwd_data: null weight %d", s);
    p.wt[s] = w[s];
    if (reinterpret_cast<uintptr_t>(w[s]) & 15) pl.vb = pl.fast = false;
  }
  if (reinterpret_cast<uintptr_t>(dy) & 15) pl.va = pl.fast = false;
  set_splits(pl);
  p.out = dx;
  p.res = res;
  p.aux = aux;
  p.flags = flags;
  return run_plan(pl, MODE_DGRAD, ws, ws_bytes, as_stream(stream));
}

int adaptseg_conv2d_bwd_weight(const adaptseg_conv_desc *d, const float *dy, const float *x,
                               float *const *dw, float *const *db, int flags, void *ws,
                               size_t ws_bytes, adaptseg_stream_t stream) {
  Plan pl;
  int st = make_plan(d, ADAPTSEG_CONV_BWD_WEIGHT, pl);
  if (st) return st;
  AS_CHECK_ARG(dy && x && dw, "conv bwd_weight: null pointer");
  ConvParams &p = pl.p;
  p.dy = dy;
  p.x = x;
  for (int s = 0; s < d->nseg; ++s) {
    AS_CHECK_ARG(dw[s], "conv bwd_weight: null dw %d", s);
    p.dw[s] = dw[s];
  }
  if (reinterpret_cast<uintptr_t>(dy) & 15) pl.va = pl.fast = false;
  if (reinterpret_cast<uintptr_t>(x) & 15) pl.vb = pl.fast = false;
  set_splits(pl);
  p.flags = flags & ADAPTSEG_EPI_ACCUMULATE;
  hipStream_t s = as_stream(stream);
  st = run_plan(pl, MODE_WGRAD, ws, ws_bytes, s);
  if (st) return st;
  if (db) {
    bool any = false;
    BiasOut o;
    for (int g = 0; g < 4; ++g) o.db[g] = g < d->nseg ? db[g] : nullptr;
    for (int g = 0; g < d->nseg; ++g) any |= db[g] != nullptr;
    if (any) {
      int rows = d->n * d->oh * d->ow;
      int splits = (int)std::min<int64_t>(ceil_div(rows, 2048), 256);
      int per = (int)ceil_div(rows, splits);
      size_t need = (size_t)splits * d->k * sizeof(float);
      if (!ws || ws_bytes < need) {
        set_error("conv bias grad: workspace too small");
        return ADAPTSEG_ERR_WORKSPACE;
      }
      float *partial = reinterpret_cast<float *>(ws);
      dim3 g((unsigned)ceil_div(d->k, 64), splits);
      bias_grad_partial_kernel<<<g, 256, 0, s>>>(dy, rows, d->k, per, partial);
      AS_CHECK_LAUNCH("bias_grad_partial");
      bias_grad_final_kernel<<<(unsigned)ceil_div(d->k, 256), 256, 0, s>>>(
          partial, splits, d->k, o, d->nseg, (flags & ADAPTSEG_EPI_ACCUMULATE) ? 1 : 0);
      AS_CHECK_LAUNCH("bias_grad_final");
    }
  }
  return ADAPTSEG_OK;
}

int adaptseg_timing_enable(int enable, int selector) {
  std::lock_guard<std::mutex> lk(g_timing.mu);
  g_timing.enabled = enable != 0;
  g_timing.selector = selector;
  if (enable) g_timing.used = 0;  // disabling keeps the recorded launches readable
  return ADAPTSEG_OK;
}

int adaptseg_timing_read(double *total_ms, double *total_flops, int64_t *launches) {
  AS_CHECK_ARG(total_ms && total_flops && launches, "timing_read: null");
  std::lock_guard<std::mutex> lk(g_timing.mu);
  double ms = 0, fl = 0;
  for (size_t i = 0; i < g_timing.used; ++i) {
    float t = 0.f;
    if (hipEventElapsedTime(&t, g_timing.events[i].first, g_timing.events[i].second) != hipSuccess) {
      set_error("timing_read: event query failed (synchronise first)");
      return ADAPTSEG_ERR_HIP;
    }
    ms += t;
    fl += g_timing.flops[i];
  }
  *total_ms = ms;
  *total_flops = fl;
  *launches = (int64_t)g_timing.used;
  return ADAPTSEG_OK;
}

}  // extern "C"
