// F32X3 convolution on 256x128 tiles with 32-deep K steps, fed by LDS-DMA from pre-split
// operands ("x3r").
//
// Same arithmetic as igemm_x3_kernel (conv_x3.hpp): every fp32
// operand is three exact bf16 terms (hi + mid + lo), six products a0b0, a0b1, a1b0, a0b2, a1b1,
// a2b0 per 16-deep K sub-step, a0b0 in one accumulator and the five cross terms in a second one,
// summed once in the epilogue — so the results are bitwise those of the register-staged kernel
// wherever neither splits K (same products, same per-accumulator k order).  The schedule differs:
//
//   * igemm_x3_kernel (128x128x16, 16 waves per CU) meets a barrier every 12 MFMAs per wave and
//     splits its activation operand in-kernel (weight gradients: both operands);
//     PMC on l3.conv2 (profiles/r2/pmc/x3_l3conv2_counters.txt): MFMA busy 0.52 / 0.55 / 0.37;
//   * here a block is 8 waves of 64x64 (2x2 MFMA tiles of 32x32x16, 128 accumulator VGPRs) on a
//     256x128 tile, one block per CU, and a K step is 32 deep: 48 MFMAs per wave between two
//     barriers (4x the work per barrier), half the LDS fragment reads per MFMA (a 64x64 wave
//     tile reuses each fragment twice), and no operand passes through registers — each step is
//     LDS-DMA only (global_load_lds_dwordx4 from the three term images in HBM) into a 2-stage
//     ring of 72 KB: step kt+1 is issued right after the barrier that opens step kt and has the
//     whole of step kt's MFMAs (~3,000 cycles per SIMD) to land.
//
// Operand term images are pixel-interleaved, [n][h][w][3][C] (the BatchNorm passes write them so,
// bn.hip x3_off): element (pixel, c) of term t at pixel * 3C + t * C + c.
// FWD / DGRAD (K-contiguous): a stage holds, per term t, the A image [256 rows][32 k] (64-B rows,
// conv_bf16g.hpp's g16_off<32> swizzle: conflict-free ds_read_b128 fragments) and, per 16-deep
// sub-step s, the B image [128 rows][16 k] (kc16 layout, conv_x3.hpp).  A rows are gathered per
// tap from the activation's term images, 16 rows x 64 B per LDS-DMA instruction (four lanes per
// row; the swizzle goes on the source chunk); the 32-deep step stays inside one tap (C % 32 == 0
// for the forward, Cout % 32 == 0 for the data gradient).  B is conv_wpack_x3v_kernel's pack, whose two consecutive 16-deep
// steps are 24 contiguous KB in exactly the stage's B byte order.
// WGRAD (k = output pixel, both operands M/N-contiguous [32 k][128] images, conv_bf16.hpp's mc
// layout read with ds_read_b64_tr_b16): dY rows contiguous, x columns per-lane gathers (each 16-B
// chunk = 8 input channels of one tap: Cin % 8 == 0, Cout % 8 == 0).  BM 256 (Cout >= 256: dY
// two images per term) or 128.
#pragma once
#include "conv_bf16g.hpp"
#include "conv_x3.hpp"

namespace adaptseg {

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

constexpr int kX3rStages = 2;
constexpr int x3r_stage_bytes(int bm) { return 3 * (bm + 128) * kX3rBK * 2; }   // 72 KB at BM 256

template <int MODE, bool S2>
__global__ void __launch_bounds__(512, 1) igemm_x3r_kernel(const ConvParams p, const __bf16 *__restrict__ a3,
                                                           const __bf16 *__restrict__ wb) {
  static_assert(MODE == MODE_FWD || MODE == MODE_DGRAD, "K-contiguous products");
  static_assert(!S2 || MODE == MODE_DGRAD, "parity classes: data gradient only");
  constexpr int BM = 256, BN = 128, BK = kX3rBK;
  constexpr int WAVES_M = 4, WAVES_N = 2, WTM = 64, WTN = 64, TM = 2, TN = 2;
  constexpr int IMGA = BM * BK * 2;                // one A term image [256 rows][32 k]: 16 KB
  constexpr int IMGB = BN * 16 * 2;                // one B term image of one 16-deep sub-step: 4 KB
  constexpr int BOFF = 3 * IMGA;                   // B images after the three A images
  constexpr int STAGE = x3r_stage_bytes(BM);
  __shared__ __attribute__((aligned(16))) char lds[kX3rStages * STAGE];

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
  const int ps = 3 * ca;                                       // pixel stride of its term images

  // A: wave w loads rows 32w .. 32w+31 of every A image (64-B rows of 32 k, g16_off<32>'s
  // swizzle), 16 rows per instruction: lane -> row 32w + 16h + lane/4, LDS slot lane&3, whose
  // source chunk is the one g16_off swizzles into that slot (h = 0, 1: the two instructions)
  const int ra = 32 * wave + (lane >> 2);
  const int chs = ((lane & 3) ^ ((ra >> 2) & 3)) * 8;   // (ra + 16) >> 2 & 3 is the same
  int a_pix[2], a_y[2], a_x[2];
  bool a_ok[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int m = bm + ra + 16 * h;
    a_ok[h] = m < M;
    const int mm = min(m, M - 1);
    if constexpr (S2) {
      const int j = mm % Wc, t2 = mm / Wc;
      const int ii = t2 % Hc, b = t2 / Hc;
      a_y[h] = ii;
      a_x[h] = j;
      a_pix[h] = ((b * p.oh + ii) * p.ow + j) * ps + chs;
    } else if constexpr (MODE == MODE_FWD) {
      uint32_t t = fdiv((uint32_t)mm, p.fd_ow);
      const int ow = mm - (int)t * p.ow;
      uint32_t b = fdiv(t, p.fd_oh);
      const int oh = (int)t - (int)b * p.oh;
      a_y[h] = oh * p.stride;
      a_x[h] = ow * p.stride;
      a_pix[h] = (((int)b * p.h + a_y[h]) * p.w + a_x[h]) * ps + chs;
    } else {
      uint32_t t = fdiv((uint32_t)mm, p.fd_w);
      const int iw = mm - (int)t * p.w;
      uint32_t b = fdiv(t, p.fd_hw);
      const int ih = (int)t - (int)b * p.h;
      a_y[h] = ih;
      a_x[h] = iw;
      a_pix[h] = (((int)b * p.oh + ih) * p.ow + iw) * ps + chs;
    }
  }
  // B: the packed tiles of this column tile, [16-deep step][term][4 KB image]; two 16-deep steps
  // are 24 contiguous KB — wave w copies KB w, w+8, w+16 of them
  const char *wtile = reinterpret_cast<const char *>(wb) + (size_t)tn * ktot / kX3BK * 3 * IMGB + wave * 1024 + lane * 16;
  const __bf16 *zero = reinterpret_cast<const __bf16 *>(g_bf16g_zero);
  const uint32_t lds0 = (uint32_t)(uintptr_t)lds;

  auto issue = [&](int kt, int st) {
    const int kbase = kt * BK;
    const uint32_t sbase = uni((int)(lds0 + st * STAGE));
    int soff, dy, dx, wkt;
    if constexpr (MODE == MODE_FWD) {
      const int tap = uni((int)fdiv((uint32_t)kbase, p.fd_c));
      int seg, t;
      seg_geom(p, sr, tap, seg, t, dy, dx);
      dy = uni(dy);
      dx = uni(dx);
      soff = uni((dy * p.w + dx) * ps + kbase - tap * p.c);
      wkt = 2 * kt;
    } else if constexpr (S2) {
      const int tap = uni((int)fdiv((uint32_t)kbase, p.fd_k));
      const int co0 = kbase - tap * p.k;
      const int u = tap / nkw, v = tap - u * nkw;
      const int kh = kh0 + 2 * u, kw = kw0 + 2 * v;
      dy = uni((py + p.pad_[0] - kh) >> 1);
      dx = uni((px + p.pad_[0] - kw) >> 1);
      soff = uni((dy * p.ow + dx) * ps + co0);
      wkt = uni(((kh * p.kw_ + kw) * p.k + co0) / kX3BK);   // packed 16-deep step of (tap, co0)
    } else {
      const int tap = uni((int)fdiv((uint32_t)kbase, p.fd_k));
      int seg, t;
      seg_geom(p, sr, tap, seg, t, dy, dx);
      dy = uni(-dy);
      dx = uni(-dx);
      soff = uni((dy * p.ow + dx) * ps + kbase - tap * p.k);
      wkt = 2 * kt;
    }
    bool v[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      if constexpr (MODE == MODE_FWD)
        v[h] = a_ok[h] & ((unsigned)(a_y[h] + dy) < (unsigned)p.h) & ((unsigned)(a_x[h] + dx) < (unsigned)p.w);
      else
        v[h] = a_ok[h] & ((unsigned)(a_y[h] + dy) < (unsigned)p.oh) & ((unsigned)(a_x[h] + dx) < (unsigned)p.ow);
    }
    const uint32_t adst = uni((int)(sbase + wave * 2048));
    const uint32_t bdst = uni((int)(sbase + BOFF + wave * 1024));
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const __bf16 *src = a3 + a_pix[h] + soff;
#pragma unroll
      for (int t = 0; t < 3; ++t) glds16(v[h] ? src + t * ca : zero, adst + t * IMGA + h * 1024);
    }
    const char *bsrc = wtile + (size_t)wkt * 3 * IMGB;
#pragma unroll
    for (int q = 0; q < 3; ++q) glds16(bsrc + q * 8 * 1024, bdst + q * 8 * 1024);
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
    const char *S = lds + st * STAGE;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 a[3][TM], b[3][TN];
#pragma unroll
      for (int t = 0; t < 3; ++t) {
#pragma unroll
        for (int i = 0; i < TM; ++i)
          a[t][i] = as_bf16x8(*reinterpret_cast<const uint4 *>(
              S + t * IMGA + g16_off<32>(wm * WTM + i * 32 + (lane & 31), 2 * s + (lane >> 5))));
#pragma unroll
        for (int j = 0; j < TN; ++j) b[t][j] = kc16_frag(S + BOFF + (s * 3 + t) * IMGB, wn * WTN + j * 32, lane);
      }
      x3_products(a, b, acc, accs);
    }
  };

  if (kt0 < kt1) {
    // 2-stage ring, one K step in flight: step kt lives in stage (kt - kt0) & 1
    issue(kt0, 0);
    int st = 0;
    for (int kt = kt0; kt < kt1; ++kt) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's DMAs of step kt landed
      __builtin_amdgcn_s_barrier();                       // ... everyone's; stage st^1 is free
      asm volatile("" ::: "memory");
      if (kt + 1 < kt1) issue(kt + 1, st ^ 1);
      compute(st);
      st ^= 1;
    }
    __syncthreads();   // the epilogue reuses the LDS
  }
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] += accs[i][j];
  static_assert(sizeof(lds) >= WAVES_M * WAVES_N * 32 * 36 * 4, "LDS for the f32x4 epilogue");
  igemm_epilogue<MODE, BM, BN, WAVES_M, WAVES_N, S2, 2>(p, acc, bm, bn, tm, tn, split, M, Hc, Wc, py, px,
                                                      reinterpret_cast<float *>(lds));
}

// Weight gradient: dW[co][tap, ci] = sum_pix dY[pix][co] x[pix + tap][ci] on the pre-split
// images of both operands, K step = 32 output pixels.  A stage holds, per term, BM/128 dY images
// and one x image of [32 k][128] (8 KB each, mc layout): wave w fills k-rows 4w .. 4w+3 of every
// image (one LDS-DMA instruction each, 16 lanes per 256-B k-row).  Waves: BM 256 -> 4x2 of
// 64x64; BM 128 -> 2x4 of 64x32.
template <int BM>
__global__ void __launch_bounds__(512, 1) igemm_x3r_wgrad_kernel(const ConvParams p, const __bf16 *__restrict__ dy3,
                                                                 const __bf16 *__restrict__ x3) {
  constexpr int BN = 128, BKP = kX3rBK, IMG = BKP * 256;
  constexpr int NA = BM / 128;                                    // dY images per term
  constexpr int WAVES_M = BM / 64, WAVES_N = 8 / WAVES_M;
  constexpr int WTM = 64, WTN = BN / WAVES_N, TM = 2, TN = WTN / 32;
  constexpr int STAGE = x3r_stage_bytes(BM);                      // 3 (NA + 1) images
  static_assert(STAGE == 3 * (NA + 1) * IMG, "stage layout");
  __shared__ __attribute__((aligned(16))) char lds[kX3rStages * STAGE];

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

  const int kr = 4 * wave + (lane >> 4);   // this lane's k-row (pixel within the step)
  const int chs = ((lane & 15) ^ (((kr & 3) << 2) | ((kr >> 2) & 3))) * 8;   // mc_off's source chunk
  bool a_col[NA];
#pragma unroll
  for (int i = 0; i < NA; ++i) a_col[i] = bm + 128 * i + chs < p.M;   // Cout % 8 == 0
  const bool b_col = bn + chs < p.N;
  const int ncol = b_col ? bn + chs : 0;
  const int tap = (int)fdiv((uint32_t)ncol, p.fd_c);
  int seg, t, tdy, tdx;
  seg_geom(p, sr, tap, seg, t, tdy, tdx);
  const int ci = ncol - tap * p.c;
  const __bf16 *zero = reinterpret_cast<const __bf16 *>(g_bf16g_zero);
  const uint32_t lds0 = (uint32_t)(uintptr_t)lds;

  // stage layout: [term][dY image 0 .. NA-1, x image], 8 KB each
  auto issue = [&](int kt, int st) {
    const uint32_t sbase = uni((int)(lds0 + st * STAGE + wave * 1024));
    const int m = kt * BKP + kr;
    const bool rv = m < K;
    const int mm = rv ? m : 0;
    uint32_t qq = fdiv((uint32_t)mm, p.fd_ow);
    const int ow = mm - (int)qq * p.ow;
    uint32_t b = fdiv(qq, p.fd_oh);
    const int oh = (int)qq - (int)b * p.oh;
    const int iy = oh * p.stride + tdy, ix = ow * p.stride + tdx;
    const bool bv = rv & b_col & ((unsigned)iy < (unsigned)p.h) & ((unsigned)ix < (unsigned)p.w);
    const __bf16 *asrc = dy3 + (size_t)mm * 3 * p.k + bm + chs;
    const __bf16 *bsrc = x3 + (size_t)(((int)b * p.h + iy) * p.w + ix) * 3 * p.c + ci;
#pragma unroll
    for (int q = 0; q < 3; ++q) {
#pragma unroll
      for (int i = 0; i < NA; ++i)
        glds16((rv & a_col[i]) ? asrc + q * p.k + 128 * i : zero, sbase + (q * (NA + 1) + i) * IMG);
      glds16(bv ? bsrc + q * p.c : zero, sbase + (q * (NA + 1) + NA) * IMG);
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
    const char *S = lds + st * STAGE;
    const int ai = (wm * WTM) / 128, ar = (wm * WTM) % 128;   // this wave's dY image and rows
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 a[3][TM], b[3][TN];
#pragma unroll
      for (int q = 0; q < 3; ++q) {
#pragma unroll
        for (int i = 0; i < TM; ++i) a[q][i] = mc_frag(S + (q * (NA + 1) + ai) * IMG, ar + i * 32, ks, lane);
#pragma unroll
        for (int j = 0; j < TN; ++j) b[q][j] = mc_frag(S + (q * (NA + 1) + NA) * IMG, wn * WTN + j * 32, ks, lane);
      }
      x3_products(a, b, acc, accs);
    }
  };

  if (kt0 < kt1) {
    issue(kt0, 0);
    int st = 0;
    for (int kt = kt0; kt < kt1; ++kt) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (kt + 1 < kt1) issue(kt + 1, st ^ 1);
      compute(st);
      st ^= 1;
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] += accs[i][j];
  igemm_epilogue<MODE_WGRAD, BM, BN, WAVES_M, WAVES_N, false>(p, acc, bm, bn, tm, tn, split, p.M, p.h, p.w, 0, 0,
                                                              reinterpret_cast<float *>(lds));
}

// fp32 NHWC (pixel strides sxn / sxh / sxw, unit channel stride) -> its pixel-interleaved term
// images [n][h][w][3][c], 8 channels per thread: the operand copy of the x3r kernels when the
// caller supplied none (F32X3_PRESPLIT).
__global__ void __launch_bounds__(256) x3_split_copy_kernel(const float *__restrict__ x, int n, int h, int w, int c8,
                                                            int sxn, int sxh, int sxw, uint4 *__restrict__ out) {
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
    uint4 *o = out + pix * 3 * c8 + cq;
    o[0] = make_uint4(h0.x, h0.y, h1.x, h1.y);
    o[c8] = make_uint4(m0.x, m0.y, m1.x, m1.y);
    o[2 * c8] = make_uint4(l0.x, l0.y, l1.x, l1.y);
  }
}

}  // namespace adaptseg
