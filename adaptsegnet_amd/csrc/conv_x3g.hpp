// F32X3 convolution fed by LDS-DMA from PRE-SPLIT operands ("x3g").
//
// igemm_x3_kernel (conv_x3.hpp) gathers every fp32 activation into registers and splits it into
// its three bf16 terms (v = hi + mid + lo exactly) while staging it into LDS; the weight
// gradient splits BOTH operands that way.  PMC on l3.conv2 (profiles/r2/pmc/x3_l3conv2_counters.txt):
// MFMA utilisation 0.52 / 0.55 / 0.37 (fwd / data-grad / weight-grad), the weight gradient
// issuing twice the forward's VALU.  Here the split is done ONCE per tensor, by whoever
// produces it (or by one x3_split_copy pass per call): the operand lives in HBM as three bf16
// NHWC images [3][n][h][w][c] (hi, mid, lo), and every K step is LDS-DMA only —
// global_load_lds_dwordx4 into a 3-stage LDS ring, two steps in flight across one raw
// s_barrier per step (counted vmcnt), the loop body ds_read + the six MFMA products.  It is
// conv_bf16g.hpp's pipeline with three term images per operand; the six products and the two
// accumulators (a0*b0 alone, the five cross terms in the second) are conv_x3.hpp's, so the
// arithmetic — and the results — are bitwise those of igemm_x3_kernel.
//
// Status: conv math ADAPTSEG_MATH_F32X3_PRESPLIT, not the default.  Measured per c2 shape
// (tools/conv_bench.py, kernel time, profiles/r3/conv_shapes_presplit_kernel.txt vs
// conv_shapes_x3_staged.txt): the weight
// gradients run 8-11 % faster than the staged kernel (l3.conv2 161.6 vs 146.0 TF/s
// fp32-equivalent, l4.conv2 135.9 vs 125.3), the forward / data gradients within -10..+1 %
// (l3.conv2 181.7 vs 180.1 forward) — so the in-kernel split VALU does NOT bound the
// forward; both kernels stall on the same per-step structure.  The term images cost 6 B per
// element where the fp32 operand costs 4: made per call they cost more than the weight
// gradient gains (conv time per c2 step 148.9 vs 126.7 ms with the copies), and written by the
// producing BatchNorm passes they add ~4-5 ms of HBM traffic per c2 step against ~3-4 ms of
// weight-gradient time saved.
// Tile 128x128x16, 8 waves of 64x32 (2x1 MFMA tiles of 32x32x16), ring 3 x 24 KB (two blocks
// per CU).  Per K step a stage holds A hi/mid/lo and B hi/mid/lo, 4 KB each; waves 0-3 load
// A (one 32-row block each, its three terms: 3 instructions), waves 4-7 load B.
//   FWD / DGRAD: K-contiguous 128 x 16 images (conv_x3.hpp's kc16 layout: 32-B rows, chunk
//     swizzled by row bit 3, conflict-free ds_read_b128).  A is gathered per row (two lanes
//     per 32-B row; the swizzle goes on the source chunk); B is conv_wpack_x3v_kernel's pack,
//     already in LDS byte order, so each B instruction copies 1 KB linearly.
//   WGRAD: k = output pixel, M/N-contiguous [16 k][128] images (conv_bf16.hpp's mc layout,
//     read with ds_read_b64_tr_b16); dY rows are contiguous, x columns per-lane gathers (each
//     16-B chunk = 8 input channels of one tap: Cin % 8 == 0).
#pragma once
#include "conv_bf16g.hpp"
#include "conv_x3.hpp"

namespace adaptseg {

constexpr int kX3gStage = 6 * kX3Img;   // A and B, three term images of 128 x 16 bf16 each

// conv_x3.hpp's six products of one 16-deep step: a0*b0 into acc, the five cross terms into accs
template <int TM, int TN>
__device__ __forceinline__ void x3_products(const bf16x8 (&a)[3][TM], const bf16x8 (&b)[3][TN], floatx16 (&acc)[TM][TN],
                                            floatx16 (&accs)[TM][TN]) {
  constexpr int TA[6] = {0, 0, 1, 0, 1, 2};
  constexpr int TB[6] = {0, 1, 0, 2, 1, 0};
#pragma unroll
  for (int u = 0; u < 6; ++u)
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        if (u == 0) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][i], b[0][j], acc[i][j], 0, 0, 0);
        else accs[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[TA[u]][i], b[TB[u]][j], accs[i][j], 0, 0, 0);
      }
}

// Measured and rejected: K step 32 (48 KB stages, one block per CU, the second 16-deep half's
// fragments read during the first half's MFMAs) — slower on every c2 shape (l3.conv2 weight
// gradient 151.6 vs 161.6 TF/s, 1x1 products up to -25 %): two blocks per CU hide more.
template <int MODE, bool S2>
__global__ void __launch_bounds__(512, 2) igemm_x3g_kernel(const ConvParams p, const __bf16 *__restrict__ a3,
                                                           uint32_t aimg, const __bf16 *__restrict__ wb) {
  static_assert(MODE == MODE_FWD || MODE == MODE_DGRAD, "K-contiguous products");
  static_assert(!S2 || MODE == MODE_DGRAD, "parity classes: data gradient only");
  constexpr int BM = 128, BN = 128, BK = kX3BK, IMG = kX3Img, STAGE = kX3gStage;
  constexpr int WAVES_M = 2, WAVES_N = 4, WTM = 64, WTN = 32, TM = 2, TN = 1;
  __shared__ __attribute__((aligned(16))) char lds[kG16Stages * STAGE];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ntn = (p.N + BN - 1) / BN;
  int tile, split;
  xcd_tile_split(tile, split);
  const int tm = tile / ntn, tn = tile - tm * ntn;
  const int bm = tm * BM, bn = tn * BN;
  const SegRegs sr = seg_regs(p);

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
  const int ktot = p.ntaps * (MODE == MODE_FWD ? p.c : p.k);  // packed weight row length
  const int ca = MODE == MODE_FWD ? p.c : p.k;                 // channels of the activation images

  const bool loads_a = wave < 4;   // wave-uniform role
  const int blk = wave & 3;        // the 32-row block (A) / 1-KB quarter (B) this wave loads
  // A: row r of the tile = 32 blk + lane/2, LDS slot lane&1; its source chunk is the one whose
  // swizzled slot (kc16_off) is the lane's
  const int ra = 32 * blk + (lane >> 1);
  const int chs = ((lane & 1) ^ ((ra >> 3) & 1)) * 8;
  int a_pix = 0, a_y = 0, a_x = 0;
  bool a_ok = false;
  {
    const int m = bm + ra;
    a_ok = m < M;
    const int mm = min(m, M - 1);
    if constexpr (S2) {
      const int j = mm % Wc, t2 = mm / Wc;
      const int ii = t2 % Hc, b = t2 / Hc;
      a_y = ii;
      a_x = j;
      a_pix = ((b * p.oh + ii) * p.ow + j) * ca + chs;
    } else if constexpr (MODE == MODE_FWD) {
      uint32_t t = fdiv((uint32_t)mm, p.fd_ow);
      const int ow = mm - (int)t * p.ow;
      uint32_t b = fdiv(t, p.fd_oh);
      const int oh = (int)t - (int)b * p.oh;
      a_y = oh * p.stride;
      a_x = ow * p.stride;
      a_pix = (((int)b * p.h + a_y) * p.w + a_x) * ca + chs;
    } else {
      uint32_t t = fdiv((uint32_t)mm, p.fd_w);
      const int iw = mm - (int)t * p.w;
      uint32_t b = fdiv(t, p.fd_hw);
      const int ih = (int)t - (int)b * p.h;
      a_y = ih;
      a_x = iw;
      a_pix = (((int)b * p.oh + ih) * p.ow + iw) * ca + chs;
    }
  }
  // B: the packed tiles of this column tile, [K step][term][4 KB image]; this wave's quarter
  const char *wtile = reinterpret_cast<const char *>(wb) + (size_t)tn * ktot / kX3BK * 3 * IMG + blk * 1024 + lane * 16;
  const __bf16 *zero = reinterpret_cast<const __bf16 *>(g_bf16g_zero);
  const uint32_t lds0 = (uint32_t)(uintptr_t)lds;

  auto issue = [&](int kt, int st) {
    const int kbase = kt * BK;
    const uint32_t sbase = uni((int)(lds0 + st * STAGE + blk * 1024));
    if (loads_a) {
      int soff, dy, dx;
      if constexpr (MODE == MODE_FWD) {
        const int tap = uni((int)fdiv((uint32_t)kbase, p.fd_c));
        int seg, t;
        seg_geom(p, sr, tap, seg, t, dy, dx);
        dy = uni(dy);
        dx = uni(dx);
        soff = uni((dy * p.w + dx) * ca + kbase - tap * p.c);
      } else if constexpr (S2) {
        const int tap = uni((int)fdiv((uint32_t)kbase, p.fd_k));
        const int co0 = kbase - tap * p.k;
        const int u = tap / nkw, v = tap - u * nkw;
        const int kh = kh0 + 2 * u, kw = kw0 + 2 * v;
        dy = uni((py + p.pad_[0] - kh) >> 1);
        dx = uni((px + p.pad_[0] - kw) >> 1);
        soff = uni((dy * p.ow + dx) * ca + co0);
      } else {
        const int tap = uni((int)fdiv((uint32_t)kbase, p.fd_k));
        int seg, t;
        seg_geom(p, sr, tap, seg, t, dy, dx);
        dy = uni(-dy);
        dx = uni(-dx);
        soff = uni((dy * p.ow + dx) * ca + kbase - tap * p.k);
      }
      bool v;
      if constexpr (MODE == MODE_FWD)
        v = a_ok & ((unsigned)(a_y + dy) < (unsigned)p.h) & ((unsigned)(a_x + dx) < (unsigned)p.w);
      else
        v = a_ok & ((unsigned)(a_y + dy) < (unsigned)p.oh) & ((unsigned)(a_x + dx) < (unsigned)p.ow);
      const __bf16 *src = a3 + a_pix + soff;
#pragma unroll
      for (int t = 0; t < 3; ++t) glds16(v ? src + (size_t)t * aimg : zero, sbase + t * IMG);
    } else {
      int wkt = kt;   // packed 16-deep step
      if constexpr (S2) {   // packed row offset of (tap, co0) of the parity class
        const int tap = uni((int)fdiv((uint32_t)kbase, p.fd_k));
        const int co0 = kbase - tap * p.k;
        const int u = tap / nkw, v = tap - u * nkw;
        const int kh = kh0 + 2 * u, kw = kw0 + 2 * v;
        wkt = uni(((kh * p.kw_ + kw) * p.k + co0) / kX3BK);
      }
#pragma unroll
      for (int t = 0; t < 3; ++t) glds16(wtile + (size_t)(wkt * 3 + t) * IMG, sbase + (3 + t) * IMG);
    }
  };

  const int wm = wave / WAVES_N, wn = wave - wm * WAVES_N;
  floatx16 acc[TM][TN], accs[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = accs[i][j][r] = 0.f;

  auto compute = [&](int st) {
    const char *As = lds + st * STAGE;
    const char *Bs = As + 3 * IMG;
    bf16x8 a[3][TM], b[3][TN];
#pragma unroll
    for (int s = 0; s < 3; ++s) {
#pragma unroll
      for (int i = 0; i < TM; ++i) a[s][i] = kc16_frag(As + s * IMG, wm * WTM + i * 32, lane);
#pragma unroll
      for (int j = 0; j < TN; ++j) b[s][j] = kc16_frag(Bs + s * IMG, wn * WTN + j * 32, lane);
    }
    x3_products(a, b, acc, accs);
  };

  if (kt0 < kt1) {
    // 3-stage ring, two K steps in flight (conv_bf16g.hpp): step kt lives in stage
    // (kt - kt0) % 3; loads past the last step re-read it into a stage nobody reads again, so
    // every wave always has exactly 3 instructions per step outstanding
    const int klast = kt1 - 1;
    issue(kt0, 0);
    issue(min(kt0 + 1, klast), 1);
    int st = 0;
    for (int kt = kt0; kt < kt1; ++kt) {
      asm volatile("s_waitcnt vmcnt(3)" ::: "memory");   // this wave's DMAs of step kt landed
      __builtin_amdgcn_s_barrier();                       // ... everyone's; stage st-1 is free
      asm volatile("" ::: "memory");
      issue(min(kt + 2, klast), st == 0 ? 2 : st - 1);
      compute(st);
      st = st == 2 ? 0 : st + 1;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();   // the epilogue reuses the LDS
  }
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] += accs[i][j];
  igemm_epilogue<MODE, BM, BN, WAVES_M, WAVES_N, S2>(p, acc, bm, bn, tm, tn, split, M, Hc, Wc, py, px,
                                                      reinterpret_cast<float *>(lds));
}

// Weight gradient: dW[co][tap, ci] = sum_pix dY[pix][co] x[pix + tap][ci] on the pre-split
// images of both operands.  K step = 16 output pixels; a stage holds dY hi/mid/lo and x
// hi/mid/lo as [16 k][128] M/N-contiguous images (4 KB, 4 LDS-DMA instructions each: one
// instruction = 4 k-rows of 256 B).  Waves 0-3 load dY k-rows 4w..4w+3 (3 terms), waves 4-7
// the x k-rows; each lane's x chunk (8 channels) has its own tap.
__global__ void __launch_bounds__(512, 2) igemm_x3g_wgrad_kernel(const ConvParams p, const __bf16 *__restrict__ dy3,
                                                                  uint32_t dyimg, const __bf16 *__restrict__ x3,
                                                                  uint32_t ximg) {
  constexpr int BM = 128, BN = 128, BKP = 16, IMG = BKP * 256, STAGE = 6 * IMG;
  constexpr int WAVES_M = 2, WAVES_N = 4, WTM = 64, WTN = 32, TM = 2, TN = 1;
  __shared__ __attribute__((aligned(16))) char lds[kG16Stages * STAGE];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ntn = (p.N + BN - 1) / BN;
  int tile, split;
  xcd_tile_split(tile, split);
  const int tm = tile / ntn, tn = tile - tm * ntn;
  const int bm = tm * BM, bn = tn * BN;
  const SegRegs sr = seg_regs(p);
  const int K = p.K;   // output pixels
  const int nkt = (K + BKP - 1) / BKP;
  const int kt0 = split * p.ktiles_per_split;
  const int kt1 = min(nkt, kt0 + p.ktiles_per_split);

  const bool loads_a = wave < 4;
  const int blk = wave & 3;
  const int kr = 4 * blk + (lane >> 4);   // this lane's k-row (pixel within the step)
  const int chs = ((lane & 15) ^ (((kr & 3) << 2) | ((kr >> 2) & 3))) * 8;   // mc_off's source chunk
  const bool a_col = bm + chs < p.M;      // Cout % 8 == 0
  const bool b_col = bn + chs < p.N;
  const int ncol = b_col ? bn + chs : 0;
  const int tap = (int)fdiv((uint32_t)ncol, p.fd_c);
  int seg, t, tdy, tdx;
  seg_geom(p, sr, tap, seg, t, tdy, tdx);
  const int ci = ncol - tap * p.c;
  const __bf16 *zero = reinterpret_cast<const __bf16 *>(g_bf16g_zero);
  const uint32_t lds0 = (uint32_t)(uintptr_t)lds;

  auto issue = [&](int kt, int st) {
    const uint32_t sbase = uni((int)(lds0 + st * STAGE + blk * 1024));
    const int m = kt * BKP + kr;
    const bool rv = m < K;
    const int mm = rv ? m : 0;
    if (loads_a) {
      const __bf16 *src = dy3 + (size_t)mm * p.k + bm + chs;
      const bool v = rv & a_col;
#pragma unroll
      for (int q = 0; q < 3; ++q) glds16(v ? src + (size_t)q * dyimg : zero, sbase + q * IMG);
    } else {
      uint32_t qq = fdiv((uint32_t)mm, p.fd_ow);
      const int ow = mm - (int)qq * p.ow;
      uint32_t b = fdiv(qq, p.fd_oh);
      const int oh = (int)qq - (int)b * p.oh;
      const int iy = oh * p.stride + tdy, ix = ow * p.stride + tdx;
      const bool v = rv & b_col & ((unsigned)iy < (unsigned)p.h) & ((unsigned)ix < (unsigned)p.w);
      const __bf16 *src = x3 + (((int)b * p.h + iy) * p.w + ix) * p.c + ci;
#pragma unroll
      for (int q = 0; q < 3; ++q) glds16(v ? src + (size_t)q * ximg : zero, sbase + (3 + q) * IMG);
    }
  };

  const int wm = wave / WAVES_N, wn = wave - wm * WAVES_N;
  floatx16 acc[TM][TN], accs[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = accs[i][j][r] = 0.f;

  auto compute = [&](int st) {
    const char *As = lds + st * STAGE;
    const char *Bs = As + 3 * IMG;
    bf16x8 a[3][TM], b[3][TN];
#pragma unroll
    for (int s = 0; s < 3; ++s) {
#pragma unroll
      for (int i = 0; i < TM; ++i) a[s][i] = mc_frag(As + s * IMG, wm * WTM + i * 32, 0, lane);
#pragma unroll
      for (int j = 0; j < TN; ++j) b[s][j] = mc_frag(Bs + s * IMG, wn * WTN + j * 32, 0, lane);
    }
    x3_products(a, b, acc, accs);
  };

  if (kt0 < kt1) {
    const int klast = kt1 - 1;
    issue(kt0, 0);
    issue(min(kt0 + 1, klast), 1);
    int st = 0;
    for (int kt = kt0; kt < kt1; ++kt) {
      asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      issue(min(kt + 2, klast), st == 0 ? 2 : st - 1);
      compute(st);
      st = st == 2 ? 0 : st + 1;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] += accs[i][j];
  igemm_epilogue<MODE_WGRAD, BM, BN, WAVES_M, WAVES_N, false>(p, acc, bm, bn, tm, tn, split, p.M, p.h, p.w, 0, 0,
                                                              reinterpret_cast<float *>(lds));
}

// fp32 NHWC (pixel strides sxn / sxh / sxw, unit channel stride) -> the three exact bf16 term
// images [3][n][h][w][c] (contiguous NHWC each, `img` elements apart), 8 channels per thread:
// the operand images of the x3g kernels when the caller supplied none.
__global__ void __launch_bounds__(256) x3_split_copy_kernel(const float *__restrict__ x, int n, int h, int w, int c8,
                                                            int sxn, int sxh, int sxw, uint4 *__restrict__ out,
                                                            int64_t img8) {
  const int64_t total = (int64_t)n * h * w * c8;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int cq = (int)(i % c8);
    const int64_t pix = i / c8;
    const int xx = (int)(pix % w);
    const int64_t t = pix / w;
    const int yy = (int)(t % h), b = (int)(t / h);
    const float *src = x + (int64_t)b * sxn + (int64_t)yy * sxh + (int64_t)xx * sxw + 8 * cq;
    const float4 v0 = ld4(src), v1 = ld4(src + 4);
    uint2 h0, m0, l0, h1, m1, l1;
    split3(v0, h0, m0, l0);
    split3(v1, h1, m1, l1);
    out[i] = make_uint4(h0.x, h0.y, h1.x, h1.y);
    out[i + img8] = make_uint4(m0.x, m0.y, m1.x, m1.y);
    out[i + 2 * img8] = make_uint4(l0.x, l0.y, l1.x, l1.y);
  }
}

}  // namespace adaptseg
