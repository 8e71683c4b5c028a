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

// ---------------------------------------------------------------------------------------------
// "x3h": igemm_x3r_kernel's 256x128x32 tile, 8 waves of 64x64 and LDS layout, with the fp32
// activation operand split in-kernel as igemm_x3_kernel does — so it needs no term images (no
// per-call split copy, no 6-byte copies written by the producing pass) and still meets one
// barrier per 48 MFMAs per wave (the register-staged kernel: one per 12).
//
// Per 32-deep K step a thread gathers four fp32 float4 of the A tile (rows tid/8 + 64 i, k
// 4 (tid & 7) .. +3: eight lanes per 128-B row) into one of two register sets, and splits + stores
// the set loaded one step earlier into the other LDS stage between the MFMAs of this step
// (sched_group_barrier: the split's VALU and the ds_write_b64s fill the MFMA gaps).  B is the
// conv_wpack_x3v pack by LDS-DMA, as in igemm_x3r_kernel.  The A gathers are inline-asm
// global_load_dwordx4 like the DMA: the compiler counts neither, and the loop waits for both with
// one s_waitcnt vmcnt(0) per step whose operands tie the loaded registers (no use of them can
// move above it).  Issue order in step kt (stage st = kt & 1):
//     wait vmcnt(0) [B(kt) DMA, A(kt+1) registers]; lgkmcnt(0) [A(kt) terms stored]; barrier;
//     B(kt+1) DMA -> st^1; A(kt+2) gathers -> the free register set;
//     MFMAs of stage st, interleaved with the split + store of A(kt+1) -> st^1.
// Both loads of a step have the whole of that step's MFMAs (~3,000 cycles per SIMD) to land.
// The products, their order per accumulator and the epilogue are igemm_x3r_kernel's, so the
// results are bitwise that kernel's (and igemm_x3_kernel's where neither splits K).
typedef float f32x4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4v x3h_ld16(const float *src) {
  f32x4v r;
  asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(r) : "v"(src) : "memory");
  return r;
}

// s_waitcnt vmcnt(0) that the four registers of a set depend on
__device__ __forceinline__ void x3h_wait(f32x4v (&r)[4]) {
  asm volatile("s_waitcnt vmcnt(0)" : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]) : : "memory");
}

// ABN (operand BatchNorm, the forward only): the activation operand is a BN's input x_pre and
// the conv reads relu(bn_affine(x_pre)) — bn_apply2d_kernel's expression (common.hpp bn_relu), so
// the products equal the unfused conv's on the BN pass's output bit for bit, and taps outside the
// image read 0 as before.  The BN's per-channel mean / invstd / weight / bias (C <= kAbnMaxC) are
// staged in LDS at the start; the split of each gathered float4 applies them first.
template <int MODE, bool S2, bool ABN>
__device__ __forceinline__ void x3h_body(const ConvParams &p, const __bf16 *__restrict__ wb) {
  static_assert(MODE == MODE_FWD || MODE == MODE_DGRAD, "K-contiguous products");
  static_assert(!S2 || MODE == MODE_DGRAD, "parity classes: data gradient only");
  static_assert(!ABN || MODE == MODE_FWD, "operand BN: the forward's activation operand");
  constexpr int BM = 256, BN = 128, BK = kX3rBK;
  constexpr int WAVES_M = 4, WAVES_N = 2, WTM = 64, WTN = 64, TM = 2, TN = 2;
  constexpr int IMGA = BM * BK * 2;                // one A term image [256 rows][32 k]: 16 KB
  constexpr int IMGB = BN * 16 * 2;                // one B term image of one 16-deep sub-step: 4 KB
  constexpr int BOFF = 3 * IMGA;
  constexpr int STAGE = x3r_stage_bytes(BM);
  constexpr int ABN_BYTES = ABN ? 4 * kAbnMaxC * 4 : 0;   // [mean | invstd | weight | bias][kAbnMaxC]
  __shared__ __attribute__((aligned(16))) char lds[2 * STAGE + ABN_BYTES];

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
  const int ktot = p.ntaps * (MODE == MODE_FWD ? p.c : p.k);

  // A rows of this thread: tid/8 + 64 i, float4 q of the row's 32 k
  const int q = tid & 7;
  int a_pix[4], a_yx[4];   // element offset of the row's k-quad; (y << 16) | x of its pixel
  bool a_ok[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = bm + (tid >> 3) + 64 * i;
    a_ok[i] = m < M;
    const int mm = min(m, M - 1);
    int y, x;
    if constexpr (S2) {
      const int j = mm % Wc, t2 = mm / Wc;
      const int ii = t2 % Hc, b = t2 / Hc;
      y = ii;
      x = j;
      a_pix[i] = ((b * p.oh + ii) * p.ow + j) * p.k + 4 * q;
    } else if constexpr (MODE == MODE_FWD) {
      uint32_t t = fdiv((uint32_t)mm, p.fd_ow);
      const int ow = mm - (int)t * p.ow;
      uint32_t b = fdiv(t, p.fd_oh);
      const int oh = (int)t - (int)b * p.oh;
      y = oh * p.stride;
      x = ow * p.stride;
      a_pix[i] = (int)b * p.sxn + y * p.sxh + x * p.sxw + 4 * q;
    } else {
      uint32_t t = fdiv((uint32_t)mm, p.fd_w);
      const int iw = mm - (int)t * p.w;
      uint32_t b = fdiv(t, p.fd_hw);
      const int ih = (int)t - (int)b * p.h;
      y = ih;
      x = iw;
      a_pix[i] = (((int)b * p.oh + ih) * p.ow + iw) * p.k + 4 * q;
    }
    a_yx[i] = (y << 16) | x;
  }
  // LDS byte offset of this thread's 8 B of each A term image (g16_off<32> swizzle): row
  // tid/8 + 64 i, 16-B chunk q/2, half q&1 — the swizzle depends on row bits 2-3 only, the same
  // for the four rows
  const uint32_t a_st = (uint32_t)(g16_off<32>(tid >> 3, q >> 1) + 8 * (q & 1));
  const char *wtile = reinterpret_cast<const char *>(wb) + (size_t)tn * ktot / kX3BK * 3 * IMGB + wave * 1024 + lane * 16;
  const float *zero4 = g_x3_zero4;
  const float *src = MODE == MODE_FWD ? p.x : p.dy;
  const uint32_t lds0 = (uint32_t)(uintptr_t)lds;

  // per K step: A source offset / tap shift, B pack step
  int cbase = 0;   // FWD: the input channel of the step's first k (the operand BN's channel)
  auto geom = [&](int kt, int &soff, int &dy, int &dx, int &wkt) {
    const int kbase = kt * BK;
    if constexpr (MODE == MODE_FWD) {
      const int tap = uni((int)fdiv((uint32_t)kbase, p.fd_c));
      int seg, t;
      seg_geom(p, sr, tap, seg, t, dy, dx);
      dy = uni(dy);
      dx = uni(dx);
      cbase = uni(kbase - tap * p.c);
      soff = uni(dy * p.sxh + dx * p.sxw + cbase);
      wkt = 2 * kt;
    } else if constexpr (S2) {
      const int tap = uni((int)fdiv((uint32_t)kbase, p.fd_k));
      const int co0 = kbase - tap * p.k;
      const int u = tap / nkw, v = tap - u * nkw;
      const int kh = kh0 + 2 * u, kw = kw0 + 2 * v;
      dy = uni((py + p.pad_[0] - kh) >> 1);
      dx = uni((px + p.pad_[0] - kw) >> 1);
      soff = uni((dy * p.ow + dx) * p.k + co0);
      wkt = uni(((kh * p.kw_ + kw) * p.k + co0) / kX3BK);
    } else {
      const int tap = uni((int)fdiv((uint32_t)kbase, p.fd_k));
      int seg, t;
      seg_geom(p, sr, tap, seg, t, dy, dx);
      dy = uni(-dy);
      dx = uni(-dx);
      soff = uni((dy * p.ow + dx) * p.k + kbase - tap * p.k);
      wkt = 2 * kt;
    }
  };
  // load_a's `meta` (ABN): (channel of the thread's float4 << 4) | the four rows' tap-valid bits
  auto load_a = [&](int kt, f32x4v (&r)[4], int &meta) {
    int soff, dy, dx, wkt;
    geom(kt, soff, dy, dx, wkt);
    const int hh = MODE == MODE_FWD ? p.h : p.oh, ww = MODE == MODE_FWD ? p.w : p.ow;
    int vb = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const bool v = a_ok[i] & ((unsigned)((a_yx[i] >> 16) + dy) < (unsigned)hh) &
                     ((unsigned)((a_yx[i] & 0xffff) + dx) < (unsigned)ww);
      vb |= (int)v << i;
      r[i] = x3h_ld16(v ? src + a_pix[i] + soff : zero4);
    }
    meta = ABN ? ((cbase + 4 * q) << 4) | vb : 0;
  };
  auto issue_b = [&](int kt, int st) {
    int soff, dy, dx, wkt;
    geom(kt, soff, dy, dx, wkt);
    const uint32_t bdst = uni((int)(lds0 + st * STAGE + BOFF + wave * 1024));
    const char *bsrc = wtile + (size_t)wkt * 3 * IMGB;
#pragma unroll
    for (int j = 0; j < 3; ++j) glds16(bsrc + j * 8 * 1024, bdst + j * 8 * 1024);
  };
  auto store_a = [&](const f32x4v (&r)[4], int meta, auto st_c) {
    constexpr int st = decltype(st_c)::value;
    char *As = lds + st * STAGE + a_st;
    float4 bm4, bi4, bw4, bb4;
    if constexpr (ABN) {
      const float *L = reinterpret_cast<const float *>(lds + 2 * STAGE) + (meta >> 4);
      bm4 = *reinterpret_cast<const float4 *>(L);
      bi4 = *reinterpret_cast<const float4 *>(L + kAbnMaxC);
      bw4 = *reinterpret_cast<const float4 *>(L + 2 * kAbnMaxC);
      bb4 = *reinterpret_cast<const float4 *>(L + 3 * kAbnMaxC);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      uint2 h, m, l;
      float4 v = make_float4(r[i].x, r[i].y, r[i].z, r[i].w);
      if constexpr (ABN) {
        const bool ok = (meta >> i) & 1;
        v.x = ok ? bn_relu(v.x, bm4.x, bi4.x, bw4.x, bb4.x) : 0.f;
        v.y = ok ? bn_relu(v.y, bm4.y, bi4.y, bw4.y, bb4.y) : 0.f;
        v.z = ok ? bn_relu(v.z, bm4.z, bi4.z, bw4.z, bb4.z) : 0.f;
        v.w = ok ? bn_relu(v.w, bm4.w, bi4.w, bw4.w, bb4.w) : 0.f;
      }
      split3(v, h, m, l);
      *reinterpret_cast<uint2 *>(As + i * 64 * 64) = h;
      *reinterpret_cast<uint2 *>(As + IMGA + i * 64 * 64) = m;
      *reinterpret_cast<uint2 *>(As + 2 * IMGA + i * 64 * 64) = l;
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

  // the MFMAs of stage st with the split + store of `r` (the next step's A) into stage st^1
  auto compute = [&](auto st_c, const f32x4v (&r)[4], int meta) {
    constexpr int st = decltype(st_c)::value;
    const char *S = lds + st * STAGE;
    __builtin_amdgcn_s_setprio(1);
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
    store_a(r, meta, std::integral_constant<int, st ^ 1>{});
    // 48 MFMAs; ~100 VALU and 12 ds_write_b64 of the split: two VALU after each MFMA, one
    // store after every fourth
#pragma unroll
    for (int g = 0; g < 12; ++g) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);
    }
    __builtin_amdgcn_s_setprio(0);
  };
  auto step_open = [&](f32x4v (&r)[4]) {
    x3h_wait(r);                                         // B(kt) DMA and A(kt+1) gathers landed
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // this wave's A(kt) terms are in LDS
    __builtin_amdgcn_s_barrier();                        // ... everyone's; stage st^1 is free
    asm volatile("" ::: "memory");
  };

  if constexpr (ABN) {   // the operand BN's channel parameters (weight / bias NULL: 1 / 0)
    float *L = reinterpret_cast<float *>(lds + 2 * STAGE);
    for (int c = tid; c < p.c; c += 512) {
      L[c] = p.abn_m[c];
      L[kAbnMaxC + c] = p.abn_is[c];
      L[2 * kAbnMaxC + c] = p.abn_w ? p.abn_w[c] : 1.f;
      L[3 * kAbnMaxC + c] = p.abn_b ? p.abn_b[c] : 0.f;
    }
    __syncthreads();
  }
  if (kt0 < kt1) {
    // past the last step the loads re-read step kt1-1 into the stage nobody reads again
    const int klast = kt1 - 1;
    f32x4v ra[4], rb[4];
    int ma, mb;
    load_a(kt0, ra, ma);
    x3h_wait(ra);
    store_a(ra, ma, std::integral_constant<int, 0>{});
    issue_b(kt0, 0);
    load_a(min(kt0 + 1, klast), rb, mb);
    for (int kt = kt0; kt < kt1; kt += 2) {
      step_open(rb);                    // stage 0 holds step kt; rb = A(kt+1)
      issue_b(min(kt + 1, klast), 1);
      load_a(min(kt + 2, klast), ra, ma);
      compute(std::integral_constant<int, 0>{}, rb, mb);
      if (kt + 1 >= kt1) break;
      step_open(ra);                    // stage 1 holds step kt+1; ra = A(kt+2)
      issue_b(min(kt + 2, klast), 0);
      load_a(min(kt + 3, klast), rb, mb);
      compute(std::integral_constant<int, 1>{}, ra, ma);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the DMAs / gathers past the last step
    __syncthreads();                                     // the epilogue reuses the LDS
  }
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] += accs[i][j];
  static_assert(sizeof(lds) >= WAVES_M * WAVES_N * 32 * 36 * 4, "LDS for the f32x4 epilogue");
  igemm_epilogue<MODE, BM, BN, WAVES_M, WAVES_N, S2, 2>(p, acc, bm, bn, tm, tn, split, M, Hc, Wc, py, px,
                                                      reinterpret_cast<float *>(lds));
}

template <int MODE, bool S2>
__global__ void __launch_bounds__(512, 1) igemm_x3h_kernel(const ConvParams p, const __bf16 *__restrict__ wb) {
  x3h_body<MODE, S2, false>(p, wb);
}
// the forward with the operand BN (ConvParams::abn_*)
__global__ void __launch_bounds__(512, 1) igemm_x3h_abn_kernel(const ConvParams p, const __bf16 *__restrict__ wb) {
  x3h_body<MODE_FWD, false, true>(p, wb);
}

// Weight gradient on the x3r_wgrad tiles ({256,128} x 128, K step = 32 output pixels, mc layout),
// both fp32 operands gathered into registers and split in-kernel (no term images).  Thread t
// holds pixels t/32 and t/32 + 16 of a step and the column quad 4 (t & 31) of every image (dY:
// BM/128 images of Cout columns; x: one image of (tap, Cin) columns, the tap fixed per thread).
// No LDS-DMA here: every load is a compiler-visible global_load, so the compiler's own vmcnt
// waits are exact (the split + store of set kt+1 waits only for its own loads, not for the set
// kt+2 loads issued after them).  Step order as igemm_x3h_kernel: wait, barrier, gathers of
// step kt+2 into the free register set, MFMAs of stage st interleaved with the split + store of
// step kt+1 into stage st^1.  Products and epilogue: igemm_x3r_wgrad_kernel's (bitwise its results
// on the same plan).
template <int BM>
__global__ void __launch_bounds__(512, 1) igemm_x3hw_kernel(const ConvParams p) {
  constexpr int BN = 128, BKP = kX3rBK, IMG = BKP * 256;
  constexpr int NA = BM / 128;                                    // dY images per term
  constexpr int WAVES_M = BM / 64, WAVES_N = 8 / WAVES_M;
  constexpr int WTM = 64, WTN = BN / WAVES_N, TM = 2, TN = WTN / 32;
  constexpr int STAGE = x3r_stage_bytes(BM);                      // 3 (NA + 1) images
  constexpr int NF = 2 * (NA + 1);                                // float4 per thread and step
  __shared__ __attribute__((aligned(16))) char lds[2 * STAGE];

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

  const int krow = tid >> 5, col = 4 * (tid & 31);
  bool a_col[NA];
#pragma unroll
  for (int i = 0; i < NA; ++i) a_col[i] = bm + 128 * i + col < p.M;   // Cout % 4 == 0
  const bool b_col = bn + col < p.N;
  const int ncol = b_col ? bn + col : 0;
  const int tap = (int)fdiv((uint32_t)ncol, p.fd_c);
  int seg, t, tdy, tdx;
  seg_geom(p, sr, tap, seg, t, tdy, tdx);
  const int ci = ncol - tap * p.c;
  // mc_off's swizzle depends on k-row bits 0-3 only: row krow + 16 is 16 rows (4 KB) further
  const uint32_t st_off = (uint32_t)(mc_off(krow, col >> 3) + 8 * ((col >> 2) & 1));
  const float *zero4 = g_x3_zero4;

  auto load = [&](int kt, float4 (&r)[NF]) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int m = kt * BKP + krow + 16 * h;
      const bool rv = m < K;
      const int mm = rv ? m : 0;
      uint32_t qq = fdiv((uint32_t)mm, p.fd_ow);
      const int ow = mm - (int)qq * p.ow;
      uint32_t b = fdiv(qq, p.fd_oh);
      const int oh = (int)qq - (int)b * p.oh;
#pragma unroll
      for (int i = 0; i < NA; ++i) r[h * (NA + 1) + i] = ld4((rv & a_col[i]) ? p.dy + mm * p.k + bm + 128 * i + col : zero4);
      const int iy = oh * p.stride + tdy, ix = ow * p.stride + tdx;
      const bool bv = rv & b_col & ((unsigned)iy < (unsigned)p.h) & ((unsigned)ix < (unsigned)p.w);
      r[h * (NA + 1) + NA] = ld4(bv ? p.x + (int)b * p.sxn + iy * p.sxh + ix * p.sxw + ci : zero4);
    }
  };
  auto store = [&](const float4 (&r)[NF], auto st_c) {
    constexpr int st = decltype(st_c)::value;
    char *S = lds + st * STAGE + st_off;
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int j = 0; j <= NA; ++j) {
        uint2 hi, mi, lo;
        split3(r[h * (NA + 1) + j], hi, mi, lo);
        *reinterpret_cast<uint2 *>(S + (0 * (NA + 1) + j) * IMG + h * 4096) = hi;
        *reinterpret_cast<uint2 *>(S + (1 * (NA + 1) + j) * IMG + h * 4096) = mi;
        *reinterpret_cast<uint2 *>(S + (2 * (NA + 1) + j) * IMG + h * 4096) = lo;
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

  auto compute = [&](auto st_c, const float4 (&r)[NF]) {
    constexpr int st = decltype(st_c)::value;
    const char *S = lds + st * STAGE;
    const int ai = (wm * WTM) / 128, ar = (wm * WTM) % 128;
    __builtin_amdgcn_s_setprio(1);
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
    store(r, std::integral_constant<int, st ^ 1>{});
    if constexpr (BM == 256) {   // 48 MFMAs, 18 ds_write_b64, ~180 VALU
#pragma unroll
      for (int g = 0; g < 6; ++g) {
#pragma unroll
        for (int u = 0; u < 3; ++u) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);
          __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);
        }
#pragma unroll
        for (int u = 0; u < 5; ++u) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);
        }
      }
    } else {                     // 24 MFMAs, 12 ds_write_b64, ~120 VALU
#pragma unroll
      for (int g = 0; g < 12; ++g) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, 5, 0);
        __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, 5, 0);
      }
    }
    __builtin_amdgcn_s_setprio(0);
  };
  auto step_open = [&]() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // this wave's stores of the step are in LDS
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };

  if (kt0 < kt1) {
    const int klast = kt1 - 1;
    float4 ra[NF], rb[NF];
    load(kt0, ra);
    store(ra, std::integral_constant<int, 0>{});
    load(min(kt0 + 1, klast), rb);
    for (int kt = kt0; kt < kt1; kt += 2) {
      step_open();                                    // stage 0 holds step kt; rb = step kt+1
      load(min(kt + 2, klast), ra);
      compute(std::integral_constant<int, 0>{}, rb);
      if (kt + 1 >= kt1) break;
      step_open();                                    // stage 1 holds step kt+1; ra = step kt+2
      load(min(kt + 3, klast), rb);
      compute(std::integral_constant<int, 1>{}, ra);
    }
    __syncthreads();   // the epilogue reuses the LDS
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
