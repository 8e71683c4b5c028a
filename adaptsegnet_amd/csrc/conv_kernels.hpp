// Implicit-GEMM convolution for gfx950 (MI355X): the fp32-input MFMA kernels
// (v_mfma_f32_32x32x2_f32, conv math F32) and the host side of every conv family (F32X3 on the
// bf16 MFMA, conv_x3.hpp / conv_x3r.hpp, the library default; bf16, conv_bf16*.hpp).
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
// Implicit-GEMM convolution kernels for gfx950 (shared by the per-op launch units).
#pragma once
#include "common.hpp"
#include <algorithm>
#include <cstring>

namespace adaptseg {


typedef float floatx16 __attribute__((ext_vector_type(16)));

enum { MODE_FWD = 0, MODE_DGRAD = 1, MODE_WGRAD = 2 };
constexpr int kMaxTaps = 64;
constexpr int BK = 16;
constexpr int kX3BK = 16;
constexpr int kX3rBK = 32;   // K step of the 256x128 F32X3 kernels (conv_x3r.hpp)
// F32X3 kernel block: 128x128 tiles; 4 waves of 64x64 for the weight gradient, 8 waves of 64x32
// for the K-contiguous products (FWD / DGRAD)
constexpr int x3_bn(int mode) { return 128; }
constexpr int x3_threads(int mode) { return 512; }  // K step of the F32X3 kernel (conv_x3.hpp)

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
  const __bf16 *resb;          // ... or the residual stored in bf16 (bf16 gradient storage; then res is NULL)
  const uint32_t *resbits;     // optional mask bitmap of the residual [rows][N / 32]: res counts where the bit is set
  const float *aux;            // leaky-grad source (nullable)
  int flags;
  int kw_, kh_;                // kernel width / height (tap -> kh, kw)
  int pad_[4], dil_[4];        // per-segment padding / dilation
  FastDiv fd_taps, fd_kw;
  __bf16 *outb;                // FWD / DGRAD: optional bf16 (RNE) copy of the final output (NULL: none)
  int outb_terms;              //   ... or (1) its F32X3 term images [rows][3][N] (the _x forms' copies)
  float *stats;                // FWD (splits == 1, no epilogue flags): per-row-tile BN statistics
  int stats_ntiles;            //   [ntiles] counts, [N][ntiles] means, [N][ntiles] M2
  // DGRAD (splits == 1, no parity scatter): the backward sums of the BatchNorm whose incoming
  // gradient this output is — per row tile tm and column c, s1 = sum g', s2 = sum g' (x - mean)
  // into bs_part[c][tm] / bs_part[N + c][tm], g' = the output value masked (bs_mask 1: ReLU of the
  // BN output, recomputed from its input x; 2: the bitmap bs_bits [rows][N / 32]; 0: none)
  float *bs_part;              //   NULL: none
  const float *bs_x;           //   the BN input x [M][N]: fp32, or ...
  const __bf16 *bs_xb;         //   ... bf16 (bf16 activation storage)
  const float *bs_mean, *bs_is, *bs_w, *bs_b;
  const uint32_t *bs_bits;
  int bs_mask, bs_ntiles;
  short tap_dy[kMaxTaps], tap_dx[kMaxTaps];
  // operand BatchNorm + ReLU (adaptseg_operand_bn): the activation operand x is a train-mode BN's
  // input and the conv reads relu((x - mean) * invstd * w + b) — the forward's A operand on
  // igemm_x3h_kernel, the weight gradient's x operand on igemm_x3_kernel (NULL abn_m: none)
  const float *abn_m, *abn_is, *abn_w, *abn_b;
};
constexpr int kAbnMaxC = 512;   // channels of an operand BN (staged in LDS)

// The epilogue's read-modify-write operands under either storage: the accumulate target (the
// fp32 output, or — bf16 gradient storage, p.out NULL — its bf16 image) and the residual (fp32,
// or bf16 in p.resb)
__device__ __forceinline__ float epi_prev(const ConvParams &p, size_t idx) {
  return p.out ? p.out[idx] : (float)p.outb[idx];
}
// The operand copy of output element (row, col): a bf16 RNE image, or its three exact bf16
// terms pixel-interleaved [row][3][N] (F32X3: the consumer conv's term-image operand)
__device__ __forceinline__ void epi_outb(const ConvParams &p, size_t row, int col, float v) {
  if (p.outb_terms) {
    uint32_t h, m, l;
    split3_2(v, 0.f, h, m, l);
    __bf16 *o = p.outb + row * 3 * p.N + col;
    o[0] = __builtin_bit_cast(__bf16, (uint16_t)h);
    o[p.N] = __builtin_bit_cast(__bf16, (uint16_t)m);
    o[2 * p.N] = __builtin_bit_cast(__bf16, (uint16_t)l);
  } else {
    p.outb[row * p.N + col] = (__bf16)v;
  }
}
__device__ __forceinline__ float epi_res(const ConvParams &p, size_t idx) {
  const float r = p.resb ? (float)p.resb[idx] : p.res[idx];
  // (N % 32 == 0: element idx = row * N + col has bit col % 32 of word row * N / 32 + col / 32)
  return (!p.resbits || ((p.resbits[idx >> 5] >> (idx & 31)) & 1u)) ? r : 0.f;
}

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
__global__ void __launch_bounds__(64 * WAVES_M * WAVES_N) igemm_kernel(const ConvParams p) {
  constexpr int NT = 64 * WAVES_M * WAVES_N;
  constexpr int WTM = BM / WAVES_M, WTN = BN / WAVES_N;
  constexpr int TM = WTM / 32, TN = WTN / 32;
  static_assert(NT == 256 || NT == 512, "4 or 8 waves per block");
  static_assert(TM >= 1 && TN >= 1, "wave tile >= 32x32");
  constexpr bool A_KC = MODE != MODE_WGRAD;  // A stored k-contiguous in global memory
  constexpr bool B_KC = MODE == MODE_FWD;
  constexpr int SA = A_KC ? BM + 2 : BM + 4;  // LDS row stride (floats); rows are k
  constexpr int SB = B_KC ? BN + 2 : BN + 4;
  constexpr int STAGE = BK * SA + BK * SB;
  // float4 staging slots per thread
  constexpr int QA = BM * BK / 4, QB = BN * BK / 4;
  constexpr int NQA = (QA + NT - 1) / NT, NQB = (QB + NT - 1) / NT;

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
    int q = tid + NT * i;
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
    int q = tid + NT * i;
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
      // LDS operands are read one k-pair ahead of the MFMAs that consume them, so the
      // ds_read latency hides behind the previous pair's MFMAs instead of stalling issue.
      float a[2][TM], b[2][TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) a[0][i] = As[hh * SA + i * 32];
#pragma unroll
      for (int j = 0; j < TN; ++j) b[0][j] = Bs[hh * SB + j * 32];
#pragma unroll
      for (int kk = 0; kk < BK; kk += 2) {
        const int cb = (kk >> 1) & 1;
        if (kk + 2 < BK) {
#pragma unroll
          for (int i = 0; i < TM; ++i) a[cb ^ 1][i] = As[(kk + 2 + hh) * SA + i * 32];
#pragma unroll
          for (int j = 0; j < TN; ++j) b[cb ^ 1][j] = Bs[(kk + 2 + hh) * SB + j * 32];
        }
        __builtin_amdgcn_sched_barrier(0);  // keep the prefetch ahead of this pair's MFMAs
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[cb][i], b[cb][j], acc[i][j], 0, 0, 0);
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
          if (flags & ADAPTSEG_EPI_ACCUMULATE) v += epi_prev(p, idx);
          if (flags & ADAPTSEG_EPI_RESIDUAL) v += epi_res(p, idx);
          v = epi_act(v, flags);
          if (flags & kEpiActGrad) v = epi_act_grad(v, p.aux[idx], flags);
          if (p.out) p.out[idx] = v;   // NULL: bf16 storage, only the copy below
          if (p.outb) epi_outb(p, row, col, v);
        }
    }
  }
}

// ------------------------------------------------------------------------------------
// FAST path: branch-free register-prefetched gathers, validity masks applied when the
// staged tile is written to LDS (so no load is ever waited on before the MFMAs run).
//
// Vector operands (AE/BE = false) need every BK-deep K tile of A inside ONE tap (FWD:
// C % BK == 0; DGRAD: Cout % BK == 0) and NHWC float4 rows; tap, channel offset and weight
// segment are then tile-uniform scalars and each lane's gather is one clamped float4 load:
//   FWD A   x[b*sxn + (oh*s+dy)*sxh + (ow*s+dx)*sxw + ci0 + kq]   (pix_slot + s_off)
//   FWD B   w_seg[n*kseg + kk0 + kq]
//   DGRAD A dy[((b*OH+ih-dy)*OW + iw-dx)*Cout + co0 + kq]
//   DGRAD B w_seg[((co0+r)*taps + t)*C + n]
//   WGRAD A dy[m*Cout + co],   WGRAD B x[b, oh*s+dy, ow*s+dx, ci]  (per-column tap)
// Per-element operands (AE / BE = true) cover the odd channel counts of the step (stem
// Cin = 3 read straight from the NCHW input, discriminator Cin = 19, ASPP / classifier
// Cout = 19 / 1): four scalar loads per slot with per-element tap decode and masks.
// ------------------------------------------------------------------------------------
__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }

// XCD-aware tile order.  The dispatcher places workgroup b on XCD b % 8 (8 XCDs, each with
// its own 4 MB L2); renumber so every XCD walks a CONTIGUOUS run of tiles (row-tile major):
// the column tiles of one row-tile and the tap halos of neighbouring row-tiles then hit the
// same L2 instead of being fetched once per XCD.
__device__ __forceinline__ int xcd_tile(int b, int nb) {
  const int x = b & 7, j = b >> 3;
  const int q = nb >> 3, r = nb & 7;
  return x * q + min(x, r) + j;
}

// Split-K grids: the dispatcher's XCD is (blockIdx.y * gridDim.x + blockIdx.x) % 8, so the
// remap runs over the flattened (split, tile) space — each XCD then walks whole splits, and
// the K slice of both operands that a split's tiles share is fetched into ONE L2.
__device__ __forceinline__ void xcd_tile_split(int &tile, int &split) {
  if (gridDim.y == 1) {
    tile = xcd_tile(blockIdx.x, gridDim.x);
    split = 0;
    return;
  }
  const int w = xcd_tile(blockIdx.y * gridDim.x + blockIdx.x, gridDim.x * gridDim.y);
  split = w / gridDim.x;
  tile = w - split * gridDim.x;
}

__device__ __forceinline__ float4 mask4(int m, float4 v) {
  return make_float4((m & 1) ? v.x : 0.f, (m & 2) ? v.y : 0.f, (m & 4) ? v.z : 0.f, (m & 8) ? v.w : 0.f);
}

// Per-segment dilation / padding / weight pointer held in SGPRs for the whole kernel.  A
// select chain over p.dil_[seg] directly compiles to an indexed kernarg s_load inside the
// K loop, whose lgkmcnt(0) wait then stalls every K tile; readfirstlane'd copies cannot be
// rematerialised as loads.
struct SegRegs {
  int dilpack, padpack;          // byte s = dilation / padding of segment s (<= 255)
  uint32_t wlo, whi;             // lane s (s < 4) holds the weight pointer of segment s
};

__device__ __forceinline__ SegRegs seg_regs(const ConvParams &p) {
  SegRegs r;
  r.dilpack = __builtin_amdgcn_readfirstlane(p.dil_[0] | (p.dil_[1] << 8) | (p.dil_[2] << 16) | (p.dil_[3] << 24));
  r.padpack = __builtin_amdgcn_readfirstlane(p.pad_[0] | (p.pad_[1] << 8) | (p.pad_[2] << 16) | (p.pad_[3] << 24));
  // lane s < 4 <- p.wt[s] through a select: a per-lane dynamic index into the kernarg struct
  // makes the compiler copy the whole ConvParams to scratch and turn every load flat
  const int l3 = threadIdx.x & 3;
  const uint64_t w = (uint64_t)(l3 == 0 ? p.wt[0] : l3 == 1 ? p.wt[1] : l3 == 2 ? p.wt[2] : p.wt[3]);
  r.wlo = (uint32_t)w;
  r.whi = (uint32_t)(w >> 32);
  return r;
}

// Uniform segment -> weight pointer with two v_readlane_b32 (no memory access in the K loop:
// a select chain over p.wt[] compiles to an indexed kernarg / LDS table load whose
// lgkmcnt(0) wait stalls every K tile).  The pointer is rebuilt through an explicit global
// (addrspace 1) pointer so its loads stay global_load: a flat load would also count against
// lgkmcnt and serialise the LDS waits of the MFMA loop.
__device__ __forceinline__ const float *seg_ptr(const SegRegs &r, int seg) {
  typedef const float __attribute__((address_space(1))) gfloat;
  const uint32_t lo = __builtin_amdgcn_readlane(r.wlo, seg);
  const uint32_t hi = __builtin_amdgcn_readlane(r.whi, seg);
  return (const float *)(gfloat *)(((uint64_t)hi << 32) | lo);
}

__device__ __forceinline__ void seg_geom(const ConvParams &p, const SegRegs &sr, int tap, int &seg, int &t,
                                         int &dy, int &dx) {
  seg = (int)fdiv((uint32_t)tap, p.fd_taps);
  t = tap - seg * p.taps_per_seg;
  const int kh = (int)fdiv((uint32_t)t, p.fd_kw);
  const int kw = t - kh * p.kw_;
  const int dil = (sr.dilpack >> (8 * seg)) & 255;
  const int pad = (sr.padpack >> (8 * seg)) & 255;
  dy = kh * dil - pad;
  dx = kw * dil - pad;
}

// ---- epilogue stores and read-backs ----------------------------------------------------
// The per-element path read the residual / accumulate target between stores; a store may alias
// them (the in-place residual), so each load waited out the full memory latency once per element
// (the layer-3 conv1 data gradient took 405 us per launch for the FLOPs of its 131-us conv3 twin,
// profiles/r4).  The LDS-transposed paths below load a whole 32x32 block's read-backs as 16-B
// rows before its first store.  Read-back kinds (uniform per launch):
enum { EK_PLAIN = 0, EK_RES_F32 = 1, EK_RES_BF16 = 2, EK_ACC_F32 = 3, EK_ACC_BF16 = 4, EK_GENERAL = 5,
       EK_ACTGRAD = 6 };   // (EK_ACTGRAD: an activation gradient from aux, the fp32 path only)

__device__ __forceinline__ float bf16_bits_to_float(uint32_t u) { return __uint_as_float(u << 16); }

__device__ __forceinline__ bool bit_of(uint32_t word, uint32_t e) { return (word >> (e & 31)) & 1u; }

// Element e (< 2^30, the caller checks) of a uniform base pointer through a 32-bit byte offset: the
// load / store takes the SGPR-base + VGPR-offset form, one VGPR per address instead of two.
template <typename T> __device__ __forceinline__ T ld_e(const void *base, uint32_t e) {
  return *reinterpret_cast<const T *>(reinterpret_cast<const char *>(base) + e * (uint32_t)sizeof(T));
}
template <typename T> __device__ __forceinline__ void st_e(void *base, uint32_t e, T v) {
  *reinterpret_cast<T *>(reinterpret_cast<char *>(base) + e * (uint32_t)sizeof(T)) = v;
}
__device__ __forceinline__ uint32_t ld_word(const uint32_t *bits, uint32_t e) {
  return *reinterpret_cast<const uint32_t *>(reinterpret_cast<const char *>(bits) + ((e >> 5) << 2));
}

__device__ __forceinline__ bool has_bias(const ConvParams &p) {
  return p.bias[0] || (p.nseg > 1 && (p.bias[1] || (p.nseg > 2 && (p.bias[2] || (p.nseg > 3 && p.bias[3])))));
}

// ---- fused BatchNorm backward sums (ConvParams::bs_part) ---------------------------------
// The BN input of four consecutive columns at element e (e % 4 == 0), stored fp32 or bf16
__device__ __forceinline__ float4 bs_x4(const ConvParams &p, uint32_t e) {
  if (p.bs_x) return ld_e<float4>(p.bs_x, e >> 2);
  const uint2 u = ld_e<uint2>(p.bs_xb, e >> 2);
  return make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u), __uint_as_float(u.y << 16),
                     __uint_as_float(u.y & 0xffff0000u));
}
__device__ __forceinline__ float bs_x1(const ConvParams &p, size_t idx) {
  return p.bs_x ? p.bs_x[idx] : (float)p.bs_xb[idx];
}
// The per-channel constants of four columns: mean, invstd, weight, bias (absent affine: 1, 0)
struct BsCol4 {
  float4 m, is, w, b;
};
__device__ __forceinline__ BsCol4 bs_col4(const ConvParams &p, int col) {
  BsCol4 c;
  c.m = *reinterpret_cast<const float4 *>(p.bs_mean + col);
  c.is = *reinterpret_cast<const float4 *>(p.bs_is + col);
  c.w = p.bs_w ? *reinterpret_cast<const float4 *>(p.bs_w + col) : make_float4(1.f, 1.f, 1.f, 1.f);
  c.b = p.bs_b ? *reinterpret_cast<const float4 *>(p.bs_b + col) : make_float4(0.f, 0.f, 0.f, 0.f);
  return c;
}
// g' of one element: the output value v masked as the BN backward masks its incoming gradient —
// mask 1: the BN's ReLU, recomputed from x with bn.hip's bn_affine expression (so the bit is the
// forward's); 2: the bitmap bit
__device__ __forceinline__ float bs_gate(int mask, float v, float x, float m, float is, float w, float b, uint32_t bit) {
  if (mask == 1) return (x - m) * is * w + b > 0.f ? v : 0.f;
  if (mask == 2) return bit ? v : 0.f;
  return v;
}
// s1 += g', s2 += g' (x - mean) over four columns; bits = the mask word shifted to column 0
__device__ __forceinline__ void bs_acc4(const ConvParams &p, const BsCol4 &c, float4 v, float4 x, uint32_t bits,
                                        float4 &s1, float4 &s2) {
  const int mk = p.bs_mask;
  const float gx = bs_gate(mk, v.x, x.x, c.m.x, c.is.x, c.w.x, c.b.x, bits & 1u);
  const float gy = bs_gate(mk, v.y, x.y, c.m.y, c.is.y, c.w.y, c.b.y, bits & 2u);
  const float gz = bs_gate(mk, v.z, x.z, c.m.z, c.is.z, c.w.z, c.b.z, bits & 4u);
  const float gw = bs_gate(mk, v.w, x.w, c.m.w, c.is.w, c.w.w, c.b.w, bits & 8u);
  s1.x += gx; s1.y += gy; s1.z += gz; s1.w += gw;
  s2.x += gx * (x.x - c.m.x); s2.y += gy * (x.y - c.m.y);
  s2.z += gz * (x.z - c.m.z); s2.w += gw * (x.w - c.m.w);
}

// bf16-only outputs (bf16 activation / gradient storage, config c5; no bias) of a full tile: each wave
// stages one 32x32 accumulator block at a time through its own 4.2 KB of LDS and writes rows of
// eight bf16 per lane (16 B), reading the bf16 residual / accumulate target the same way —
// instead of a 2-B store and a 2-B read-back per element, which left the memory-bound bf16
// layer-1/2 data gradients at 1.6-3 TB/s alone (profiles/r4/c5_dgrad_pmc.txt).  No block barrier:
// the LDS region is the wave's own (LDS operations of a wave complete in order).
template <int EK, int MODE, int TM, int TN>
__device__ __forceinline__ void epi_store_bf16x8(const ConvParams &p, const floatx16 (&acc)[TM][TN], int bm, int bn,
                                                 int wm, int wn, int wtm, int wtn, int lane, int wave, float *lds) {
  constexpr int LS = 33;                       // padded row stride (floats) of the staging block
  float *w = lds + wave * (32 * LS);
  const int l32 = lane & 31, hh = lane >> 5;
  const int c8 = (lane & 3) * 8;               // this lane's 8-column chunk ...
  const int rr = lane >> 2;                    // ... of rows rr and rr + 16
  const uint32_t N = (uint32_t)p.N;
  const int flags = p.flags;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int gcol = bn + wn * wtn + j * 32 + c8;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      __builtin_amdgcn_sched_barrier(0);   // one block's operands live at a time
      const int grow = bm + wm * wtm + i * 32 + rr;
      uint4 rd[2];
      if constexpr (EK != EK_PLAIN) {   // the read-backs first (16 B per lane and row)
        const __bf16 *src = EK == EK_RES_BF16 ? p.resb : p.outb;
#pragma unroll
        for (int h = 0; h < 2; ++h)
          rd[h] = *reinterpret_cast<const uint4 *>(src + (size_t)((uint32_t)(grow + 16 * h) * N + gcol));
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) w[((r & 3) + 8 * (r >> 2) + 4 * hh) * LS + l32] = acc[i][j][r];
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the wave's stores land before its reads
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        float v[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] = w[(rr + 16 * h) * LS + c8 + q];
        if constexpr (EK != EK_PLAIN) {
          const uint32_t u[4] = {rd[h].x, rd[h].y, rd[h].z, rd[h].w};
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            v[2 * q] += __uint_as_float(u[q] << 16);
            v[2 * q + 1] += __uint_as_float(u[q] & 0xffff0000u);
          }
        }
        uint32_t o[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float a = epi_act(v[2 * q], flags), b = epi_act(v[2 * q + 1], flags);
          o[q] = (uint32_t)__builtin_bit_cast(uint16_t, (__bf16)a) |
                 ((uint32_t)__builtin_bit_cast(uint16_t, (__bf16)b) << 16);
        }
        *reinterpret_cast<uint4 *>(p.outb + (size_t)((uint32_t)(grow + 16 * h) * N + gcol)) =
            make_uint4(o[0], o[1], o[2], o[3]);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // reads done before the next block's staging
    }
  }
}

// fp32 outputs of a full tile (F32X3 / fp32 kernels; no bias, no bf16 copy): each wave stages one
// 32x32 accumulator block at a time through its own 4.6 KB of LDS and writes rows of four fp32
// per lane (16 B), reading the residual (+ its bitmap word) / accumulate target the same way —
// a quarter of the per-element path's memory instructions.
// With fused BN sums (p.bs_part) each lane also accumulates its four columns' s1 / s2 over its
// rows; on return lanes 0..7 of the wave hold them (column chunk wn * wtn + j * 32 + 4 lane).
template <int EK, int MODE, int TM, int TN, bool S2>
__device__ __forceinline__ void epi_store_f32x4(const ConvParams &p, const floatx16 (&acc)[TM][TN], int bm, int bn,
                                                int wm, int wn, int wtm, int wtn, int lane, int wave, float *lds,
                                                int Hc, int Wc, int py, int px, float4 (&bs1)[TN], float4 (&bs2)[TN]) {
  // output row of GEMM row `row` (S2: the parity class's pixel back in the NHWC image; a pixel's
  // channels stay contiguous, so the 16-B rows hold)
  auto orow = [&](int row) -> uint32_t {
    if constexpr (S2) {
      const int jj = row % Wc, t2 = row / Wc;
      const int ii = t2 % Hc, b = t2 / Hc;
      return (uint32_t)((b * p.h + 2 * ii + py) * p.w + 2 * jj + px);
    } else {
      return (uint32_t)row;
    }
  };
  constexpr int LS = 36;                       // padded row stride: 16-B aligned rows for ds_read_b128
  float *w = lds + wave * (32 * LS);
  const int l32 = lane & 31, hh = lane >> 5;
  const int c4 = (lane & 7) * 4;               // this lane's 4-column chunk ...
  const int rr = lane >> 3;                    // ... of rows rr + 8 h, h = 0..3
  const uint32_t N = (uint32_t)p.N;
  const int flags = p.flags;
  // (fused BN sums on the plain store only: beside the residual / accumulate read-backs the
  // register-staged F32X3 build, 128 VGPRs, spills; those tiles take the general path)
  const bool bs = MODE == MODE_DGRAD && EK == EK_PLAIN && p.bs_part;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int gcol = bn + wn * wtn + j * 32 + c4;
    bs1[j] = bs2[j] = make_float4(0.f, 0.f, 0.f, 0.f);
    BsCol4 bc;
    if (bs) bc = bs_col4(p, gcol);
    float4 bsum = make_float4(0.f, 0.f, 0.f, 0.f);   // the summed segment biases of these 4 columns
    if constexpr (MODE == MODE_FWD) {
      for (int sg = 0; sg < p.nseg; ++sg) {
        const float *bp = sg == 0 ? p.bias[0] : sg == 1 ? p.bias[1] : sg == 2 ? p.bias[2] : p.bias[3];
        if (bp) {
          const float4 b4 = *reinterpret_cast<const float4 *>(bp + gcol);
          bsum.x += b4.x; bsum.y += b4.y; bsum.z += b4.z; bsum.w += b4.w;
        }
      }
    }
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      __builtin_amdgcn_sched_barrier(0);   // one block's operands live at a time
      const int grow = bm + wm * wtm + i * 32 + rr;
      float4 rd[4];
      uint32_t rb[4];
      if constexpr (EK != EK_PLAIN) {   // the read-backs first (16 B per lane and row)
        const float *src = EK == EK_RES_F32 ? p.res : EK == EK_ACTGRAD ? p.aux : p.out;
#pragma unroll
        for (int h = 0; h < 4; ++h) {
          const uint32_t e = orow(grow + 8 * h) * N + gcol;
          rd[h] = ld_e<float4>(src, e >> 2);
          rb[h] = (EK == EK_RES_F32 && p.resbits) ? ld_word(p.resbits, e) : ~0u;
        }
      }
      float4 xv[4];   // the BN input of these rows (fused BN sums)
      uint32_t xw[4];
      if (bs) {
#pragma unroll
        for (int h = 0; h < 4; ++h) {
          const uint32_t e = orow(grow + 8 * h) * N + gcol;
          xv[h] = bs_x4(p, e);
          xw[h] = p.bs_mask == 2 ? ld_word(p.bs_bits, e) >> (e & 31) : ~0u;
        }
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) w[((r & 3) + 8 * (r >> 2) + 4 * hh) * LS + l32] = acc[i][j][r];
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the wave's stores land before its reads
#pragma unroll
      for (int h = 0; h < 4; ++h) {
        const uint32_t orw = orow(grow + 8 * h);
        const uint32_t e = orw * N + gcol;
        float4 v = *reinterpret_cast<const float4 *>(w + (rr + 8 * h) * LS + c4);
        if constexpr (MODE == MODE_FWD) {
          v.x += bsum.x; v.y += bsum.y; v.z += bsum.z; v.w += bsum.w;
        }
        if constexpr (EK == EK_ACC_F32) {
          v.x += rd[h].x; v.y += rd[h].y; v.z += rd[h].z; v.w += rd[h].w;
        }
        if constexpr (EK == EK_RES_F32) {
          const uint32_t m = rb[h] >> (e & 31);
          v.x += (m & 1u) ? rd[h].x : 0.f;
          v.y += (m & 2u) ? rd[h].y : 0.f;
          v.z += (m & 4u) ? rd[h].z : 0.f;
          v.w += (m & 8u) ? rd[h].w : 0.f;
        }
        v.x = epi_act(v.x, flags); v.y = epi_act(v.y, flags);
        v.z = epi_act(v.z, flags); v.w = epi_act(v.w, flags);
        if constexpr (EK == EK_ACTGRAD) {
          v.x = epi_act_grad(v.x, rd[h].x, flags); v.y = epi_act_grad(v.y, rd[h].y, flags);
          v.z = epi_act_grad(v.z, rd[h].z, flags); v.w = epi_act_grad(v.w, rd[h].w, flags);
        }
        if (bs) bs_acc4(p, bc, v, xv[h], xw[h], bs1[j], bs2[j]);
        if (p.out) st_e<float4>(p.out, e >> 2, v);
        if (p.outb) {   // the term images [row][3][N] (outb_terms; < 2^31 elements, the host checks)
          uint2 th, tm, tl;
          split3(v, th, tm, tl);
          const uint32_t e3 = orw * 3 * N + gcol;
          st_e<uint2>(p.outb, e3 >> 2, th);
          st_e<uint2>(p.outb, (e3 + N) >> 2, tm);
          st_e<uint2>(p.outb, (e3 + 2 * N) >> 2, tl);
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // reads done before the next block's staging
    }
  }
  if (bs) {   // the 8 lanes of a column chunk (rows rr = lane >> 3) -> lanes 0..7
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int o = 8; o < 64; o <<= 1) {
        bs1[j].x += __shfl_xor(bs1[j].x, o); bs1[j].y += __shfl_xor(bs1[j].y, o);
        bs1[j].z += __shfl_xor(bs1[j].z, o); bs1[j].w += __shfl_xor(bs1[j].w, o);
        bs2[j].x += __shfl_xor(bs2[j].x, o); bs2[j].y += __shfl_xor(bs2[j].y, o);
        bs2[j].z += __shfl_xor(bs2[j].z, o); bs2[j].w += __shfl_xor(bs2[j].w, o);
      }
  }
}

// The general store (stride-2 parity scatter, activation gradients, accumulate + residual, or
// outputs of >= 2^30 elements): per-element read-backs.  Fused BN sums (p.bs_part; never with the
// parity scatter): on return lanes 0..31 hold their column's s1 / s2 over the wave's rows.
template <int MODE, int TM, int TN, typename ROWF, bool BS = true>
__device__ __forceinline__ void epi_store_general(const ConvParams &p, floatx16 (&acc)[TM][TN], int bm, int bn,
                                                  int wm, int wn, int wtm, int wtn, int hh, int l32, bool full, int M,
                                                  ROWF out_row, float (&gs1)[TN], float (&gs2)[TN]) {
  const int flags = p.flags;
  const bool bs = BS && MODE == MODE_DGRAD && p.bs_part;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = bn + wn * wtn + j * 32 + l32;
    gs1[j] = gs2[j] = 0.f;
    if (!full && col >= p.N) continue;
    float bm1 = 0.f, bi1 = 0.f, bw1 = 1.f, bb1 = 0.f;
    if (bs) {
      bm1 = p.bs_mean[col];
      bi1 = p.bs_is[col];
      if (p.bs_w) bw1 = p.bs_w[col];
      if (p.bs_b) bb1 = p.bs_b[col];
    }
    float bsum = 0.f;
    if constexpr (MODE == MODE_FWD) {
      for (int s = 0; s < p.nseg; ++s) {
        const float *bp = s == 0 ? p.bias[0] : s == 1 ? p.bias[1] : s == 2 ? p.bias[2] : p.bias[3];
        if (bp) bsum += bp[col];
      }
    }
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      // the BN input of the block's 16 rows, loaded before its first store (a store may alias it
      // for all the compiler knows, which would serialise each load behind the previous store)
      float xs[16];
      uint32_t xb[16];
      if (bs) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = min(bm + wm * wtm + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh, M - 1);
          const size_t idx = (size_t)row * p.N + col;
          xs[r] = bs_x1(p, idx);
          xb[r] = p.bs_mask == 2 ? (p.bs_bits[idx >> 5] >> (idx & 31)) & 1u : 1u;
        }
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = bm + wm * wtm + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
        if (!full && row >= M) continue;
        const size_t idx = out_row(row) * p.N + col;
        float v = acc[i][j][r] + bsum;
        if (flags & ADAPTSEG_EPI_ACCUMULATE) v += epi_prev(p, idx);
        if (flags & ADAPTSEG_EPI_RESIDUAL) v += epi_res(p, idx);
        v = epi_act(v, flags);
        if (flags & kEpiActGrad) v = epi_act_grad(v, p.aux[idx], flags);
        if (bs) {
          const float g = bs_gate(p.bs_mask, v, xs[r], bm1, bi1, bw1, bb1, xb[r]);
          gs1[j] += g;
          gs2[j] += g * (xs[r] - bm1);
        }
        if (p.out) p.out[idx] = v;   // NULL: bf16 storage, only the copy below
        if (p.outb) epi_outb(p, out_row(row), col, v);
      }
    }
  }
  if (bs) {   // lanes l32 and l32 + 32 hold the same column
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      gs1[j] += __shfl_xor(gs1[j], 32);
      gs2[j] += __shfl_xor(gs2[j], 32);
    }
  }
}

// The fused BN sums of the block's row tile tm (igemm_epilogue, after the stores): each wave's
// per-lane column sums (f32x4 layout: lanes 0..7 x 4 columns; general layout: lanes 0..31) are
// summed over the WAVES_M waves of a column range through LDS and written to bs_part[c][tm],
// bs_part[N + c][tm].  The LDS must be free of the stores' staging (a barrier first).
template <int BM, int BN, int WAVES_M, int WAVES_N, int TN>
__device__ __forceinline__ void bs_finish(const ConvParams &p, bool vec, const float4 (&bs1)[TN],
                                          const float4 (&bs2)[TN], const float (&gs1)[TN], const float (&gs2)[TN],
                                          int bn, int tm, int wm, int wn, int lane, float *lds) {
  constexpr int WTN = BN / WAVES_N;
  float *red1 = lds, *red2 = lds + WAVES_M * BN;
  __syncthreads();
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int cl = wn * WTN + j * 32;
    if (vec) {
      if (lane < 8) {
        *reinterpret_cast<float4 *>(red1 + wm * BN + cl + 4 * lane) = bs1[j];
        *reinterpret_cast<float4 *>(red2 + wm * BN + cl + 4 * lane) = bs2[j];
      }
    } else if (lane < 32) {
      red1[wm * BN + cl + lane] = gs1[j];
      red2[wm * BN + cl + lane] = gs2[j];
    }
  }
  __syncthreads();
  const int nt = p.bs_ntiles;
  for (int c = threadIdx.x; c < BN; c += 64 * WAVES_M * WAVES_N) {
    const int col = bn + c;
    if (col >= p.N) continue;
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int q = 0; q < WAVES_M; ++q) {
      s1 += red1[q * BN + c];
      s2 += red2[q * BN + c];
    }
    p.bs_part[(size_t)col * nt + tm] = s1;
    p.bs_part[((size_t)p.N + col) * nt + tm] = s2;
  }
}

// Epilogue shared by the fp32 (igemm_fast_kernel) and bf16 (igemm_bf16_kernel) MFMA paths:
// both accumulate 32x32 tiles whose C layout is row = (r&3) + 8*(r>>2) + 4*(lane>>5),
// col = lane&31 (dtype-independent on gfx950).  Split-K slabs, the weight-gradient store
// (per segment, optional accumulate) and the fwd / data-grad epilogue (bias, accumulate,
// residual, activation and its gradient, stride-2 parity scatter, fused BN statistics).
// `lds` must hold WAVES_M * BN floats and be free (the caller's main loop ended on a barrier).
// VEC: the LDS-transposed 16-B stores of full tiles — 1: bf16 outputs (epi_store_bf16x8, the
// bf16-output LDS-DMA kernels), 2: fp32 outputs (epi_store_f32x4, the F32X3 kernels); the
// kernel's LDS holds WAVES_M * WAVES_N * 4.6 KB.  Every other tile and kernel (VEC 0: the
// fp32-MFMA and register-staged bf16 kernels) takes the per-element path.  (Round 4's batched
// per-element read-back kinds took those kernels from 82-97 to 184-217 VGPRs — the stem's
// forward kernel from three waves per SIMD to one, c4 −1.3 % against round 3 on one box,
// profiles/r4/c4_r3_ab.txt — and were removed.)
template <int MODE, int BM, int BN, int WAVES_M, int WAVES_N, bool S2, int VEC = 0>
__device__ __forceinline__ void igemm_epilogue(const ConvParams &p, floatx16 (&acc)[BM / WAVES_M / 32][BN / WAVES_N / 32],
                                               int bm, int bn, int tm, int tn, int split, int M, int Hc,
                                               int Wc, int py, int px, float *lds) {
  constexpr int WTM = BM / WAVES_M, WTN = BN / WAVES_N;
  constexpr int TM = WTM / 32, TN = WTN / 32;
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WAVES_N, wn = wave - wm * WAVES_N;
  const int l32 = lane & 31, hh = lane >> 5;
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
    // the LDS-transposed kinds: stride 1, < 2^30 output elements (32-bit byte offsets)
    int ek = EK_GENERAL;
    // (S2 and activation gradients: the fp32 path only; S2 scatters into the whole image)
    const uint64_t oelems = S2 ? (uint64_t)p.n * p.h * p.w * p.N : (uint64_t)p.M * p.N;
    if (VEC > 0 && (!S2 || VEC == 2) && oelems < (1ull << 30) && (!(flags & kEpiActGrad) || VEC == 2)) {
      const int rf = flags & (ADAPTSEG_EPI_ACCUMULATE | ADAPTSEG_EPI_RESIDUAL);
      if (flags & kEpiActGrad) ek = rf == 0 ? EK_ACTGRAD : EK_GENERAL;
      else if (rf == 0) ek = EK_PLAIN;
      else if (rf == ADAPTSEG_EPI_RESIDUAL) ek = p.resb ? EK_RES_BF16 : EK_RES_F32;
      else if (rf == ADAPTSEG_EPI_ACCUMULATE) ek = p.out ? EK_ACC_F32 : EK_ACC_BF16;
    }
    bool vec = false;
    float4 bs1[TN], bs2[TN];   // fused BN sums, per lane (epi_store_f32x4 / epi_store_general)
    float gs1[TN], gs2[TN];
    if constexpr (VEC == 1 && !S2) {
      // (fused BN sums: the general path)
      vec = full && !p.out && p.outb && !p.resbits && !p.bs_part && (p.N & 7) == 0 && (MODE != MODE_FWD || !has_bias(p)) &&
            (ek == EK_PLAIN || ek == EK_RES_BF16 || ek == EK_ACC_BF16) &&
            !(reinterpret_cast<uintptr_t>(p.outb) & 15) && (ek != EK_RES_BF16 || !(reinterpret_cast<uintptr_t>(p.resb) & 15));
      if (vec) {
        if (ek == EK_PLAIN) epi_store_bf16x8<EK_PLAIN, MODE, TM, TN>(p, acc, bm, bn, wm, wn, WTM, WTN, lane, wave, lds);
        else if (ek == EK_RES_BF16)
          epi_store_bf16x8<EK_RES_BF16, MODE, TM, TN>(p, acc, bm, bn, wm, wn, WTM, WTN, lane, wave, lds);
        else epi_store_bf16x8<EK_ACC_BF16, MODE, TM, TN>(p, acc, bm, bn, wm, wn, WTM, WTN, lane, wave, lds);
      }
    }
    if constexpr (VEC == 2) {
      // (fp32 output and / or its term images; biases as 16-B rows)
      vec = full && (p.out || p.outb_terms) && (!p.outb || p.outb_terms) && (p.N & 3) == 0 &&
            (ek == EK_PLAIN || ek == EK_RES_F32 || ek == EK_ACC_F32 || ek == EK_ACTGRAD) &&
            !(reinterpret_cast<uintptr_t>(p.out) & 15) && !(reinterpret_cast<uintptr_t>(p.outb) & 7) &&
            (MODE != MODE_FWD || ((!p.bias[0] || !(reinterpret_cast<uintptr_t>(p.bias[0]) & 15)) &&
                                  (p.nseg < 2 || !p.bias[1] || !(reinterpret_cast<uintptr_t>(p.bias[1]) & 15)) &&
                                  (p.nseg < 3 || !p.bias[2] || !(reinterpret_cast<uintptr_t>(p.bias[2]) & 15)) &&
                                  (p.nseg < 4 || !p.bias[3] || !(reinterpret_cast<uintptr_t>(p.bias[3]) & 15)))) &&
            (ek != EK_RES_F32 || !(reinterpret_cast<uintptr_t>(p.res) & 15)) &&
            (ek != EK_ACTGRAD || !(reinterpret_cast<uintptr_t>(p.aux) & 15)) && (ek == EK_PLAIN || !p.bs_part);
      if (vec) {
#define AS_F32X4(EK_) \
  epi_store_f32x4<EK_, MODE, TM, TN, S2>(p, acc, bm, bn, wm, wn, WTM, WTN, lane, wave, lds, Hc, Wc, py, px, bs1, bs2)
        if (ek == EK_PLAIN) AS_F32X4(EK_PLAIN);
        else if (ek == EK_RES_F32) AS_F32X4(EK_RES_F32);
        else if (ek == EK_ACC_F32) AS_F32X4(EK_ACC_F32);
        else AS_F32X4(EK_ACTGRAD);
#undef AS_F32X4
      }
    }
    // (the fused BN sums are compiled out of the bf16-output LDS-DMA kernels, VEC 1: the host
    // plans them for no such product — bnsum_plan_tiles — and they would spill the BK-32 builds)
    constexpr bool BS = MODE == MODE_DGRAD && !S2 && VEC != 1;
    if (!vec)
      epi_store_general<MODE, TM, TN, decltype(out_row), BS>(p, acc, bm, bn, wm, wn, WTM, WTN, hh, l32, full, M, out_row,
                                                              gs1, gs2);
    if constexpr (BS) {
      if (p.bs_part) bs_finish<BM, BN, WAVES_M, WAVES_N, TN>(p, vec, bs1, bs2, gs1, gs2, bn, tm, wm, wn, lane, lds);
    }
    if constexpr (MODE == MODE_FWD && !S2) {
      // BatchNorm statistics of this row tile, straight from the accumulators (the BN that
      // consumes this conv then skips its statistics pass over y): per column the tile's
      // mean and sum of squared deviations (two passes over registers, Chan-mergeable in fp64
      // by bn_fwd_train_tiles).  Only with flags == 0 and no bias: y == acc.
      if (p.stats) {
        __syncthreads();  // the LDS stages are free (the main loop ended on a barrier)
        float *red = lds;  // [WAVES_M][BN]
        const int nvalid = min(BM, M - bm);
        float mean[TN];
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          float s = 0.f;
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              const int rl = wm * WTM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
              s += rl < nvalid ? acc[i][j][r] : 0.f;
            }
          s += __shfl_xor(s, 32);
          if (hh == 0) red[wm * BN + wn * WTN + j * 32 + l32] = s;
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          float s = 0.f;
#pragma unroll
          for (int q = 0; q < WAVES_M; ++q) s += red[q * BN + wn * WTN + j * 32 + l32];
          mean[j] = s / (float)nvalid;
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          float s = 0.f;
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              const int rl = wm * WTM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
              const float dv = acc[i][j][r] - mean[j];
              s += rl < nvalid ? dv * dv : 0.f;
            }
          s += __shfl_xor(s, 32);
          if (hh == 0) red[wm * BN + wn * WTN + j * 32 + l32] = s;
        }
        __syncthreads();
        const int nt = p.stats_ntiles;
        if (wm == 0 && hh == 0) {
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            const int col = bn + wn * WTN + j * 32 + l32;
            if (col >= p.N) continue;
            float m2 = 0.f;
#pragma unroll
            for (int q = 0; q < WAVES_M; ++q) m2 += red[q * BN + wn * WTN + j * 32 + l32];
            p.stats[nt + (size_t)col * nt + tm] = mean[j];
            p.stats[nt + ((size_t)p.N + col) * nt + tm] = m2;
          }
        }
        if (tid == 0 && tn == 0) p.stats[tm] = (float)nvalid;
      }
    }
  }
}

template <int MODE, int BM, int BN, int WAVES_M, int WAVES_N, int BK, bool S2, bool AE, bool BE, int MINB = 1>
__global__ void __launch_bounds__(64 * WAVES_M * WAVES_N, MINB) igemm_fast_kernel(const ConvParams p) {
  constexpr int NT = 64 * WAVES_M * WAVES_N;  // threads per block (4 or 8 waves)
  constexpr int WTM = BM / WAVES_M, WTN = BN / WAVES_N;
  constexpr int TM = WTM / 32, TN = WTN / 32;
  static_assert(NT == 256 || NT == 512, "4 or 8 waves per block");
  static_assert(TM >= 1 && TN >= 1, "wave tile >= 32x32");
  constexpr bool A_KC = MODE != MODE_WGRAD;
  constexpr bool B_KC = MODE == MODE_FWD;
  constexpr int SA = A_KC ? BM + 2 : BM + 4;
  constexpr int SB = B_KC ? BN + 2 : BN + 4;
  constexpr int STAGE = BK * SA + BK * SB;
  constexpr int QA = BM * BK / 4, QB = BN * BK / 4;
  constexpr int NQA = QA / NT, NQB = QB / NT;
  constexpr int KQ = BK / 4;  // float4 per k-contiguous row
  static_assert(QA % NT == 0 && QB % NT == 0, "every thread stages whole float4 slots");

  __shared__ __attribute__((aligned(16))) float lds[2 * STAGE];

  const int tid = threadIdx.x;
  const int ntn = (p.N + BN - 1) / BN;
  int tile, split;
  xcd_tile_split(tile, split);
  const int tm = tile / ntn, tn = tile - tm * ntn;
  const int bm = tm * BM, bn = tn * BN;
  const SegRegs sr = seg_regs(p);

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
    const int q = tid + NT * i;
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
        // vector: pixel base incl. this slot's k offset; per-element: image base only
        a_pix[i] = AE ? (int)b * p.sxn : (int)b * p.sxn + a_y[i] * p.sxh + a_x[i] * p.sxw + a_k[i];
      } else {  // DGRAD, stride 1
        uint32_t t = fdiv((uint32_t)mm, p.fd_w);
        const int iw = mm - (int)t * p.w;
        uint32_t b = fdiv(t, p.fd_hw);
        const int ih = (int)t - (int)b * p.h;
        a_y[i] = ih;
        a_x[i] = iw;
        a_pix[i] = (((int)b * p.oh + ih) * p.ow + iw) * p.k + (AE ? 0 : a_k[i]);
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
  int b_pk[BE && MODE == MODE_WGRAD ? NQB : 1][4], b_ci[BE && MODE == MODE_WGRAD ? NQB : 1][4];
  bool b_ok[NQB];
#pragma unroll
  for (int i = 0; i < NQB; ++i) {
    const int q = tid + NT * i;
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
      } else if constexpr (!BE) {  // WGRAD B': column (tap, ci), 4 channels of one tap
        const int tap = (int)fdiv((uint32_t)nn, p.fd_c);
        const int ci = nn - tap * p.c;
        int seg, t;
        seg_geom(p, sr, tap, seg, t, b_dy[i], b_dx[i]);
        b_off[i] = ci;
      } else {  // WGRAD B' per element: pack (dy, dx) and the channel offset per column
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int ne = n + e;
          const int tap = (int)fdiv((uint32_t)min(ne, p.N - 1), p.fd_c);
          const int ci = min(ne, p.N - 1) - tap * p.c;
          int seg, t, dy, dx;
          seg_geom(p, sr, tap, seg, t, dy, dx);
          b_pk[i][e] = (dy + 32768) | ((dx + 32768) << 16);
          b_ci[i][e] = ne < p.N ? ci * p.sxc : -1;
        }
      }
    }
  }

  float4 ra[NQA], rb[NQB];
  int ma[NQA], mb[NQB];  // 4-bit validity masks, applied when the tile is written to LDS

  auto load_tile = [&](int kt) {
    const int kbase = kt * BK;
    if constexpr (MODE == MODE_FWD) {
      if constexpr (!AE) {
        const int tap = uni((int)fdiv((uint32_t)kbase, p.fd_c));
        int seg, t, dy, dx;
        seg_geom(p, sr, tap, seg, t, dy, dx);
        dy = uni(dy);
        dx = uni(dx);
        const int soff = uni(dy * p.sxh + dx * p.sxw + kbase - tap * p.c);
#pragma unroll
        for (int i = 0; i < NQA; ++i) {
          const bool v = a_ok[i] && (unsigned)(a_y[i] + dy) < (unsigned)p.h &&
                         (unsigned)(a_x[i] + dx) < (unsigned)p.w;
          ma[i] = v ? 15 : 0;
          ra[i] = ld4(p.x + (v ? a_pix[i] + soff : 0));
        }
      } else {  // per-element tap decode (nseg == 1)
#pragma unroll
        for (int i = 0; i < NQA; ++i) {
          float vv[4];
          int msk = 0;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int k = kbase + a_k[i] + e;
            const int tap = (int)fdiv((uint32_t)k, p.fd_c);
            const int ci = k - tap * p.c;
            const int kh = (int)fdiv((uint32_t)tap, p.fd_kw);
            const int kw = tap - kh * p.kw_;
            const int iy = a_y[i] + kh * p.dil_[0] - p.pad_[0];
            const int ix = a_x[i] + kw * p.dil_[0] - p.pad_[0];
            const bool v = a_ok[i] && k < K && (unsigned)iy < (unsigned)p.h && (unsigned)ix < (unsigned)p.w;
            msk |= v ? (1 << e) : 0;
            vv[e] = p.x[v ? a_pix[i] + iy * p.sxh + ix * p.sxw + ci * p.sxc : 0];
          }
          ma[i] = msk;
          ra[i] = make_float4(vv[0], vv[1], vv[2], vv[3]);
        }
      }
      if constexpr (!BE) {
        const int seg = uni((int)fdiv((uint32_t)kbase, p.fd_nseg_k));
        const float *wp = seg_ptr(sr, seg) + (kbase - seg * p.kseg);
#pragma unroll
        for (int i = 0; i < NQB; ++i) {
          mb[i] = b_ok[i] ? 15 : 0;
          rb[i] = ld4(wp + b_off[i]);
        }
      } else {  // rows of length kseg % 4 != 0 (nseg == 1): per-element K mask
#pragma unroll
        for (int i = 0; i < NQB; ++i) {
          float vv[4];
          int msk = 0;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const bool v = b_ok[i] && kbase + b_k[i] + e < K;
            msk |= v ? (1 << e) : 0;
            vv[e] = seg_ptr(sr, 0)[v ? b_off[i] + kbase + e : 0];
          }
          mb[i] = msk;
          rb[i] = make_float4(vv[0], vv[1], vv[2], vv[3]);
        }
      }
    } else if constexpr (MODE == MODE_DGRAD) {
      if constexpr (!AE) {
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
          seg_geom(p, sr, tap, seg, t, dy, dx);
          seg = uni(seg);
          t = uni(t);
          dy = uni(dy);
          dx = uni(dx);
        }
        const int soff = uni(co0 - (dy * p.ow + dx) * p.k);
#pragma unroll
        for (int i = 0; i < NQA; ++i) {
          const bool v = a_ok[i] && (unsigned)(a_y[i] - dy) < (unsigned)p.oh &&
                         (unsigned)(a_x[i] - dx) < (unsigned)p.ow;
          ma[i] = v ? 15 : 0;
          ra[i] = ld4(p.dy + (v ? a_pix[i] + soff : 0));
        }
        const float *wp = seg_ptr(sr, seg) + (co0 * p.taps_per_seg + t) * p.c;
#pragma unroll
        for (int i = 0; i < NQB; ++i) {
          if constexpr (!BE) {
            mb[i] = b_ok[i] ? 15 : 0;
            rb[i] = ld4(wp + b_off[i]);
          } else {
            const int n = bn + b_col[i];
            float vv[4];
            int msk = 0;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const bool v = n + e < p.N;
              msk |= v ? (1 << e) : 0;
              vv[e] = wp[v ? b_off[i] + e : 0];
            }
            mb[i] = msk;
            rb[i] = make_float4(vv[0], vv[1], vv[2], vv[3]);
          }
        }
      } else {  // per-element (tap, co) decode: Cout % BK != 0 (ASPP: 19), stride 1
#pragma unroll
        for (int i = 0; i < NQA; ++i) {
          float vv[4];
          int msk = 0;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int k = kbase + a_k[i] + e;
            const int kc = min(k, K - 1);
            const int tap = (int)fdiv((uint32_t)kc, p.fd_k);
            const int co = kc - tap * p.k;
            int seg, t, dy, dx;
            seg_geom(p, sr, tap, seg, t, dy, dx);
            const bool v = a_ok[i] && k < K && (unsigned)(a_y[i] - dy) < (unsigned)p.oh &&
                           (unsigned)(a_x[i] - dx) < (unsigned)p.ow;
            msk |= v ? (1 << e) : 0;
            vv[e] = p.dy[v ? a_pix[i] + co - (dy * p.ow + dx) * p.k : 0];
          }
          ma[i] = msk;
          ra[i] = make_float4(vv[0], vv[1], vv[2], vv[3]);
        }
#pragma unroll
        for (int i = 0; i < NQB; ++i) {  // B row k = kbase + r: per-slot (seg, co, t)
          const int k = kbase + b_k[i];
          const bool rv = k < K;
          const int kc = min(k, K - 1);  // rows past K still form an in-bounds address
          const int tap = (int)fdiv((uint32_t)kc, p.fd_k);
          const int co = kc - tap * p.k;
          int seg, t, dy, dx;
          seg_geom(p, sr, tap, seg, t, dy, dx);
          const float *row = seg_ptr(p, seg) + (co * p.taps_per_seg + t) * p.c;
          const int n = bn + b_col[i];
          if constexpr (!BE) {
            mb[i] = (rv && b_ok[i]) ? 15 : 0;
            rb[i] = ld4(row + (b_ok[i] ? n : 0));
          } else {
            float vv[4];
            int msk = 0;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const bool v = rv && n + e < p.N;
              msk |= v ? (1 << e) : 0;
              vv[e] = row[v ? n + e : 0];
            }
            mb[i] = msk;
            rb[i] = make_float4(vv[0], vv[1], vv[2], vv[3]);
          }
        }
      }
    } else {  // WGRAD
#pragma unroll
      for (int i = 0; i < NQA; ++i) {
        const int m = kbase + a_k[i];
        const bool rv = m < K;
        const float *row = p.dy + (size_t)(rv ? m : 0) * p.k;
        if constexpr (!AE) {
          ma[i] = (rv && a_ok[i]) ? 15 : 0;
          ra[i] = ld4(row + a_pix[i]);
        } else {
          const int col = bm + a_col[i];
          float vv[4];
          int msk = 0;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const bool v = rv && col + e < p.M;
            msk |= v ? (1 << e) : 0;
            vv[e] = row[v ? col + e : 0];
          }
          ma[i] = msk;
          ra[i] = make_float4(vv[0], vv[1], vv[2], vv[3]);
        }
      }
#pragma unroll
      for (int i = 0; i < NQB; ++i) {
        const int m = kbase + b_k[i];
        const int mm = min(m, K - 1);
        uint32_t t = fdiv((uint32_t)mm, p.fd_ow);
        const int ow = mm - (int)t * p.ow;
        uint32_t b = fdiv(t, p.fd_oh);
        const int oh = (int)t - (int)b * p.oh;
        const int y0 = oh * p.stride, x0 = ow * p.stride;
        if constexpr (!BE) {
          const int iy = y0 + b_dy[i], ix = x0 + b_dx[i];
          const bool v = b_ok[i] && m < K && (unsigned)iy < (unsigned)p.h && (unsigned)ix < (unsigned)p.w;
          mb[i] = v ? 15 : 0;
          rb[i] = ld4(p.x + (v ? (int)b * p.sxn + iy * p.sxh + ix * p.sxw + b_off[i] : 0));
        } else {
          float vv[4];
          int msk = 0;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int iy = y0 + (b_pk[i][e] & 0xffff) - 32768;
            const int ix = x0 + (int)((unsigned)b_pk[i][e] >> 16) - 32768;
            const bool v = b_ci[i][e] >= 0 && m < K && (unsigned)iy < (unsigned)p.h &&
                           (unsigned)ix < (unsigned)p.w;
            msk |= v ? (1 << e) : 0;
            vv[e] = p.x[v ? (int)b * p.sxn + iy * p.sxh + ix * p.sxw + b_ci[i][e] : 0];
          }
          mb[i] = msk;
          rb[i] = make_float4(vv[0], vv[1], vv[2], vv[3]);
        }
      }
    }
  };

  auto store_tile = [&](int buf) {
    float *As = lds + buf * STAGE;
    float *Bs = As + BK * SA;
#pragma unroll
    for (int i = 0; i < NQA; ++i) {
      const float4 v = mask4(ma[i], ra[i]);
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
      const float4 v = mask4(mb[i], rb[i]);
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
      // LDS operands are read one k-pair ahead of the MFMAs that consume them, so the
      // ds_read latency hides behind the previous pair's MFMAs instead of stalling issue.
      float a[2][TM], b[2][TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) a[0][i] = As[hh * SA + i * 32];
#pragma unroll
      for (int j = 0; j < TN; ++j) b[0][j] = Bs[hh * SB + j * 32];
      // MFMA issue outranks the co-resident wave's loads / LDS stores while this tile's
      // products run (s_setprio is scalar: the same for every lane)
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int kk = 0; kk < BK; kk += 2) {
        const int cb = (kk >> 1) & 1;
        if (kk + 2 < BK) {
#pragma unroll
          for (int i = 0; i < TM; ++i) a[cb ^ 1][i] = As[(kk + 2 + hh) * SA + i * 32];
#pragma unroll
          for (int j = 0; j < TN; ++j) b[cb ^ 1][j] = Bs[(kk + 2 + hh) * SB + j * 32];
        }
        __builtin_amdgcn_sched_barrier(0);  // keep the prefetch ahead of this pair's MFMAs
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[cb][i], b[cb][j], acc[i][j], 0, 0, 0);
      }
      __builtin_amdgcn_s_setprio(0);
      if (more) store_tile(cur ^ 1);
      __syncthreads();
      cur ^= 1;
    }
  }

  // ---- epilogue ----
  igemm_epilogue<MODE, BM, BN, WAVES_M, WAVES_N, S2>(p, acc, bm, bn, tm, tn, split, M, Hc, Wc, py, px, lds);
}


struct Plan {
  ConvParams p;
  int cfg;        // index into kCfgBM / kCfgBN
  bool va, vb;
  bool fast;
  bool s2;     // stride-2 data gradient by output-pixel parity class (grid.z = 4)
  bool bf16;   // bf16-MFMA path (conv_bf16.hpp): 128x{128,256}x64 tiles, packed bf16 weights
  bool x3;     // F32X3 path (conv_x3.hpp): fp32 via exact 3-term bf16 splits, 128x128x16 tiles
  bool x3g;    // ... on pre-split term images by LDS-DMA (the caller's or made per call); with x3r
  bool x3r;    // ... the 256x128x32 one-block-per-CU term-image kernel (conv_x3r.hpp)
  int x3r_bm;  // its row tile (256; weight gradients with Cout < 256: 128)
  bool x3r_ok; // F32X3 product the x3r kernel covers (a 32-deep step inside one tap, 16-B chunks)
  bool x3ext;  // x3r on the caller's term images (F32X3 maths): no per-call split copies
  bool x3h;    // ... x3r's 256x128x32 tile with the fp32 activation split in-kernel (igemm_x3h_kernel)
  int bf16_bn; // its tile width: 256 for forward / data-grad products with N >= 256, else 128
  bool g16;    // bf16 LDS-DMA kernel (conv_bf16g.hpp): bf16 activation copy, g16_bm x g16_bn x 64
  int g16_bm, g16_bn, g16_bk;
  const void *act_ext;  // caller's bf16 copy of the activation operand (g16; NULL: copied per call)
  const void *act_ext2; // weight gradient: the caller's bf16 copy of x (act_ext: of dY)
  const void *wpack_ext;  // caller-built weight pack (adaptseg_conv2d_wpack; NULL: packed per call)
  bool ae, be; // FAST per-element gathers for the A / B operand
  int bk;
  int mode;
  int tiles;
  size_t slab_bytes;  // workspace need: [bf16 weight pack, 256-B aligned] + split-K slabs
  double flops;  // algorithmic FLOPs of the conv product this plan computes
};

// tile configs: 0 = 128x128 (2x2 waves), 1 = 256x32 (4x1), 2 = 32x256 (1x4), 3 = 64x256 (1x4),
// 4 = 256x64 (4x1), 5 = 64x64 (2x2, small weight gradients), 6 = 128x128 with BK 16
// (33 KB of LDS: three blocks per CU), 7 = 256x128 with 8 waves (4x2, 512 threads).  Every wave owns a 64x64, 64x32 or 32x64 block of 32x32x2 MFMA tiles.
// 8 = 128x128 with BK 16 compiled for 3 blocks per CU (__launch_bounds__ min-blocks 3: the
// accumulators move from AGPRs into the VGPR budget, 117 registers, so 3-4 waves per SIMD).
static const int kCfgBM[9] = {128, 256, 32, 64, 256, 64, 128, 256, 128};
static const int kCfgBN[9] = {128, 32, 256, 256, 64, 64, 128, 128, 128};
static const int kCfgThreads[9] = {256, 256, 256, 256, 256, 256, 256, 512, 256};
// K step of the FAST kernel per config (LDS: 2 stages x BK x (BM+BN+pad) floats)
static int fast_bk(int cfg) { return (cfg == 4 || cfg == 6 || cfg == 8) ? 16 : 32; }


// Planning and execution (conv_igemm.hip), shared with the tap-GEMM path (conv_tapgemm.hip).
double conv_flops(const adaptseg_conv_desc *d);
void set_splits(Plan &pl);
int make_plan(const adaptseg_conv_desc *d, int op, Plan &pl);
int kernel_id(const Plan &pl, int mode);
// defer: a weight gradient whose plan splits K leaves its sum pending on stream s
// (adaptseg_splitk_flush) instead of launching it
int run_plan(Plan &pl, int mode, void *ws, size_t ws_bytes, hipStream_t s, bool defer = false);

// Tap-GEMM path for stride-1 'same' convs with Cout <= 32 (ASPP): conv_tapgemm.hip.
bool tapgemm_eligible(const adaptseg_conv_desc *d);
bool tapgemm_copy_only(const adaptseg_conv_desc *d, int op);
size_t tapgemm_workspace(const adaptseg_conv_desc *d, int op);
int tapgemm_kernel_id(const adaptseg_conv_desc *d, int op, int *kid, int *splits);
// x_bf16: optional bf16 copy of x (contiguous NHWC, 16-B aligned) for the inner GEMM's bf16 kernel
int tapgemm_fwd(const adaptseg_conv_desc *d, const float *x, const uint16_t *x_bf16, const float *const *w,
                const float *const *bias, const float *res, float *y, int flags, void *ws, size_t ws_bytes,
                hipStream_t s);
int tapgemm_bwd_data(const adaptseg_conv_desc *d, const float *dy, const float *const *w, const float *res,
                     const float *aux, float *dx, int flags, void *ws, size_t ws_bytes, hipStream_t s);
int tapgemm_bwd_weight(const adaptseg_conv_desc *d, const float *dy, const float *x, const uint16_t *x_bf16,
                       float *const *dw, int flags, void *ws, size_t ws_bytes, hipStream_t s);

hipError_t launch_fwd(const Plan &pl, hipStream_t s);
// bf16 conv math (adaptseg_conv_set_math): weight-pack bytes and launcher (conv_launch_bf16.hip)
int conv_math();
size_t bf16_wpack_bytes(const Plan &pl);
size_t bf16_pre_bytes(const Plan &pl);   // workspace ahead of the slabs: weight pack (+ activation copy)
hipError_t prep_bf16(Plan &pl, void *ws, hipStream_t s);   // the weight pack (unless wpack_ext) + copies
hipError_t prep_bf16_wpack(const Plan &pl, void *pack, hipStream_t s);   // the weight pack alone
hipError_t launch_bf16(const Plan &pl, void *ws, hipStream_t s);
// F32X3 conv math: three-image weight-pack bytes and launcher (conv_launch_x3.hip)
size_t x3_wpack_bytes(const Plan &pl);
int plan_bm(const Plan &pl);
size_t x3_pre_bytes(const Plan &pl);   // workspace ahead of the slabs: weight pack + per-call term images
hipError_t prep_x3(const Plan &pl, void *wpack, hipStream_t s);    // the weight pack (unless wpack_ext) + copies
hipError_t prep_x3_wpack(const Plan &pl, void *pack, hipStream_t s);  // the weight pack alone
hipError_t launch_x3(const Plan &pl, void *wpack, hipStream_t s);  // the GEMM
hipError_t launch_dgrad(const Plan &pl, hipStream_t s);
hipError_t launch_wgrad(const Plan &pl, hipStream_t s);

}  // namespace adaptseg
