// fp32 convolution on the bf16 matrix cores: "F32X3" conv math (adaptseg_conv_set_math).
//
// gfx950 runs fp32-input MFMA (v_mfma_f32_32x32x2_f32) at 1/16 of the bf16 MFMA rate.  Every
// fp32 operand v splits EXACTLY into three bf16 terms, v = v0 + v1 + v2 (round-to-nearest-even
// each: v0 = bf16(v), v1 = bf16(v - v0), v2 = v - v0 - v1; 3 x 8 significant bits cover fp32's
// 24, and bf16 has fp32's exponent range), so
//     a * b = sum_{i+j<=2} a_i b_j  +  (a1 b2 + a2 b1 + a2 b2)
// where the dropped terms are below 2^-23 |a b| — the size of one fp32 rounding.  The six kept
// products a0b0, a0b1, a1b0, a0b2, a1b1, a2b0 are exact in the bf16 MFMA (8 x 8 bit
// significands) and accumulate in fp32, so the conv keeps fp32 accuracy (the fp64-oracle parity
// tests hold it to the same 2e-5 * max|ref| as the fp32 MFMA path) at 6 bf16 MFMAs per 16-deep
// K step instead of 8 fp32 MFMAs of 4x the cycles: 768 vs 2048 MFMA cycles per 64x64 wave tile.
//
// Two accumulators per output tile: a0*b0 into acc, the five cross terms (2^-8 and 2^-16 of it)
// into accs, summed once in the epilogue (one fp32 RNE add).  The bf16 MFMA's internal sum does
// not round to nearest: products far below the largest addend (accumulator included) lose their
// low bits, a downward bias of a few hundredths of an ulp per instruction (measured: mean -0.028
// ulp, 14398 results below vs 8734 above round-to-nearest of 204800, tools/dbg/mfma_round.hip).
// Fed into one accumulator, the small cross terms always sit ~2^8 below it and the bias piles up
// over K to ~-1e-8 * max|y| (systematic, unlike fp32 MFMA's +-1e-10); in their own accumulator
// they are the largest addends and the residual bias drops to the fp32 MFMA's level (measured on
// a 256->256 3x3 conv: mean signed error <= 2e-10 * max|y|, rms 2e-8 vs fp32 MFMA's 5.5e-8).
// The cost is 64 more accumulator VGPRs (occupancy 3 -> 2), which the measured per-product
// throughput does not show (conv step 141 -> 143 TF/s fp32-equivalent).
//
// Same products, gathers, tile order, split-K and epilogue as igemm_fast_kernel; the operand path
// is the bf16 kernel's (conv_bf16.hpp) with three LDS images per operand:
//   * activations are gathered in fp32 and split into their three bf16 images while staged;
//   * FWD / DGRAD weights are split once per call into three bf16 images packed in the exact
//     byte order of the LDS tiles ([column tile][K step][term][128 x 16, swizzled], zero rows past
//     N), so staging B is a contiguous 12 KB copy per K step (conv_wpack_x3_kernel);
//   * K-contiguous activation rows are gathered 64 B (16 fp32) per row by four lanes, so one
//     load instruction covers 16 whole rows;
//   * K-contiguous images are 32-B rows (16 k) with the 16-B chunk XOR-swizzled by row bit 3
//     (conflict-free ds_read_b128 fragments); M/N-contiguous images (weight gradient) are the
//     bf16 kernel's 256-B k-rows read with ds_read_b64_tr_b16.
// Block tile 128x128x16, 48 KB of LDS (two stages).  FWD / DGRAD: 8 waves (2x4) of 64x32 wave
// tiles (2x1 MFMA tiles, x2 accumulators: 124-126 VGPRs, two blocks = 16 waves per CU), the
// next K step's split and LDS stores interleaved with this step's MFMAs (T14 order: staged
// registers hold step kt+1, reloaded with kt+2 right after the stores) — measured +4.4 % c2 /
// +5.3 % c3 over 4 waves of 64x64 (staging after the MFMAs, which spilled at 256 VGPRs when
// interleaved).  A / B decomposition on l3.conv2 (tools/dbg): dropping the global loads saves
// 22 % of the time, dropping the split + stores with them the same — what is left is bound by
// the gathered loads, not the MFMAs.  WGRAD: 4 waves (2x2) of 64x64, staging after the MFMAs
// with raised priority (its M/N-contiguous images are 128 wide).
#pragma once
#include "conv_bf16.hpp"


namespace adaptseg {

constexpr int kX3Img = 128 * kX3BK * 2;  // bytes of one bf16 operand image (128 x 16)

__device__ __forceinline__ int kc16_off(int r, int ch) { return r * 32 + ((ch ^ ((r >> 3) & 1)) << 4); }

__device__ __forceinline__ bf16x8 kc16_frag(const char *img, int r0, int lane) {
  return as_bf16x8(*reinterpret_cast<const uint4 *>(img + kc16_off(r0 + (lane & 31), lane >> 5)));
}

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
// 16 zero bytes: the source of every operand float4 outside the image (padding taps, rows past
// M / K), so the staged values need no mask before they are split and stored
static __device__ __attribute__((aligned(16))) float g_x3_zero4[4];
// the exact three-term split (rne2 / split3_2 / split3) lives in common.hpp: the BatchNorm
// passes that write F32X3 term images use the same arithmetic

// ABN (the weight gradient only): its x operand is a train-mode BN's input and the product reads
// relu(bn_affine(x)) (common.hpp bn_relu: bn_apply2d_kernel's expression, so bitwise the unfused
// weight gradient on the BN pass's output); pixels outside the image / past K read 0.  The BN's
// channel parameters (Cin <= kAbnMaxC) are staged in LDS at the start.
template <int MODE, bool S2, bool ABN>
__device__ __forceinline__ void x3_body(const ConvParams &p, const __bf16 *__restrict__ wb) {
  static_assert(!ABN || MODE == MODE_WGRAD, "operand BN: the weight gradient's x operand");
  constexpr bool MC = MODE == MODE_WGRAD;   // both operands M/N-contiguous (k = output pixel)
  constexpr int BM = 128, BN = 128, BK = kX3BK, NT = x3_threads(MODE);
  constexpr int WAVES_M = 2, WAVES_N = NT / 128;        // 2x2 (WGRAD) or 2x4 waves
  constexpr int WTM = BM / WAVES_M, WTN = BN / WAVES_N;  // wave tile 64x64 / 64x32
  constexpr int TM = WTM / 32, TN = WTN / 32;
  constexpr int IMG = kX3Img;               // A term image: 128 rows x 16 k bf16
  constexpr int IMGB = BN * kX3BK * 2;      // B term image
  constexpr int BPT = IMGB / NT;            // packed-B bytes per thread and term (16 or 8)
  constexpr int STAGE = 3 * IMG + 3 * IMGB; // A hi/mid/lo, B hi/mid/lo
  constexpr int ABN_BYTES = ABN ? 4 * kAbnMaxC * 4 : 0;

  __shared__ __attribute__((aligned(16))) char lds[2 * STAGE + ABN_BYTES];

  const int tid = threadIdx.x;
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

  // ---- per-slot constants ----
  // K-contiguous A: slot i = row (tid>>2) + 64*i, float4 (tid&3) of its 16 k.
  // M/N-contiguous: slot q = tid + 256*i: k-row q>>5, columns 4*(q&31) .. +3.
  constexpr int NQ = 1;
  int a_pix[NQ], a_y[NQ], a_x[NQ];
  bool a_ok[NQ];
  int b_off[NQ], b_dy[NQ], b_dx[NQ];
  bool b_ok[NQ];
  const int sj = tid & 3;
#pragma unroll
  for (int i = 0; i < NQ; ++i) {
    if constexpr (!MC) {
      const int m = bm + (tid >> 2) + 64 * i;
      a_ok[i] = m < M;
      const int mm = min(m, M - 1);
      if constexpr (S2) {
        const int j = mm % Wc, t2 = mm / Wc;
        const int ii = t2 % Hc, b = t2 / Hc;
        a_y[i] = ii;
        a_x[i] = j;
        a_pix[i] = ((b * p.oh + ii) * p.ow + j) * p.k + 4 * sj;
      } else if constexpr (MODE == MODE_FWD) {
        uint32_t t = fdiv((uint32_t)mm, p.fd_ow);
        const int ow = mm - (int)t * p.ow;
        uint32_t b = fdiv(t, p.fd_oh);
        const int oh = (int)t - (int)b * p.oh;
        a_y[i] = oh * p.stride;
        a_x[i] = ow * p.stride;
        a_pix[i] = (int)b * p.sxn + a_y[i] * p.sxh + a_x[i] * p.sxw + 4 * sj;
      } else {
        uint32_t t = fdiv((uint32_t)mm, p.fd_w);
        const int iw = mm - (int)t * p.w;
        uint32_t b = fdiv(t, p.fd_hw);
        const int ih = (int)t - (int)b * p.h;
        a_y[i] = ih;
        a_x[i] = iw;
        a_pix[i] = (((int)b * p.oh + ih) * p.ow + iw) * p.k + 4 * sj;
      }
    } else {
      const int q = tid + NT * i;
      const int col = 4 * (q & 31);
      a_ok[i] = bm + col < p.M;                    // Cout % 4 == 0
      a_pix[i] = a_ok[i] ? bm + col : 0;
      const int n = bn + col;
      b_ok[i] = n < p.N;
      const int nn = b_ok[i] ? n : 0;
      const int tap = (int)fdiv((uint32_t)nn, p.fd_c);
      int seg, t;
      seg_geom(p, sr, tap, seg, t, b_dy[i], b_dx[i]);
      b_off[i] = nn - tap * p.c;                   // input channel of the column
    }
  }
  // packed B tiles of this column tile: [K step][term][IMGB]
  const char *wtile = reinterpret_cast<const char *>(wb) + (size_t)tn * ktot / BK * 3 * IMGB + BPT * tid;
  typedef typename std::conditional<BPT == 16, u32x4, uint2>::type BChunk;

  float4 ra[NQ];           // A: one float4 per slot
  float4 rbf[MC ? NQ : 1]; // MC: B float4 per slot
  bool rbv = false;        // ABN: rbf[0] is a real pixel (else the zero fill)
  BChunk rbh[MC ? 1 : 3];  // K-contiguous B: this thread's BPT bytes of each packed term image
  const float *zero4 = g_x3_zero4;

  // WGRAD: this thread's output pixel m = 16 kt + krow0 walks forward one K step at a time, its
  // (image, row, column) and element offsets advanced incrementally instead of two divisions and
  // a 3-term address per step (the weight gradient splits both operands in-kernel: its VALU,
  // not its MFMA, sets its pace — profiles/r2/pmc/x3_l3conv2_counters.txt)
  int w_kt = kt0;          // the K step the walk stands at (first load: kt0)
  int w_pos = 0;           // (output row << 16) | output column of this thread's pixel
  int w_tap = 0;           // (tap row offset << 16) + tap column offset of this thread's x column
  int w_dy = 0, w_x = 0;   // element offsets of this thread's dY and x float4s (column included)
  const int w_dcol = p.stride * p.sxw;                     // x offset per output column
  const int w_drow = p.stride * p.sxh - p.ow * w_dcol;     // ... at a row wrap
  const int w_dimg = p.sxn - p.oh * p.stride * p.sxh;      // ... at an image wrap
  if constexpr (MC) {
    w_tap = b_dy[0] * 65536 + b_dx[0];
    const int m = kt0 * BK + (tid >> 5);
    uint32_t t = fdiv((uint32_t)m, p.fd_ow);
    const int ow = m - (int)t * p.ow;
    uint32_t b = fdiv(t, p.fd_oh);
    const int oh = (int)t - (int)b * p.oh;
    w_pos = (oh << 16) | ow;
    w_dy = m * p.k + a_pix[0];
    w_x = (int)b * p.sxn + oh * p.stride * p.sxh + ow * w_dcol + b_dy[0] * p.sxh + b_dx[0] * p.sxw + b_off[0];
  }

  auto load_tile = [&](int kt) {
    const int kbase = kt * BK;
    if constexpr (MODE == MODE_FWD) {
      const int tap = uni((int)fdiv((uint32_t)kbase, p.fd_c));
      int seg, t, dy, dx;
      seg_geom(p, sr, tap, seg, t, dy, dx);
      dy = uni(dy);
      dx = uni(dx);
      const int soff = uni(dy * p.sxh + dx * p.sxw + kbase - tap * p.c);
#pragma unroll
      for (int i = 0; i < NQ; ++i) {
        const bool v = a_ok[i] && (unsigned)(a_y[i] + dy) < (unsigned)p.h && (unsigned)(a_x[i] + dx) < (unsigned)p.w;
        ra[i] = ld4(v ? p.x + a_pix[i] + soff : zero4);
      }
#pragma unroll
      for (int s = 0; s < 3; ++s) rbh[s] = *reinterpret_cast<const BChunk *>(wtile + (size_t)(kt * 3 + s) * IMGB);
    } else if constexpr (MODE == MODE_DGRAD) {
      const int tap = uni((int)fdiv((uint32_t)kbase, p.fd_k));
      const int co0 = kbase - tap * p.k;
      int dy, dx, wk;
      if constexpr (S2) {
        const int u = tap / nkw, v = tap - u * nkw;
        const int kh = kh0 + 2 * u, kw = kw0 + 2 * v;
        dy = uni(-((py + p.pad_[0] - kh) >> 1));
        dx = uni(-((px + p.pad_[0] - kw) >> 1));
        wk = uni((kh * p.kw_ + kw) * p.k + co0);   // packed row offset of (tap, co0)
      } else {
        int seg, t;
        seg_geom(p, sr, tap, seg, t, dy, dx);
        dy = uni(dy);
        dx = uni(dx);
        wk = kbase;
      }
      const int soff = uni(co0 - (dy * p.ow + dx) * p.k);
#pragma unroll
      for (int i = 0; i < NQ; ++i) {
        const bool v = a_ok[i] && (unsigned)(a_y[i] - dy) < (unsigned)p.oh && (unsigned)(a_x[i] - dx) < (unsigned)p.ow;
        ra[i] = ld4(v ? p.dy + a_pix[i] + soff : zero4);
      }
      const int wkt = wk / BK;
#pragma unroll
      for (int s = 0; s < 3; ++s) rbh[s] = *reinterpret_cast<const BChunk *>(wtile + (size_t)(wkt * 3 + s) * IMGB);
    } else {  // WGRAD: k = output pixel
      static_assert(NQ == 1 && NT == 512, "one slot: k-row tid / 32 of a 16-deep step");
      if (kt != w_kt) {   // kt == w_kt + 1 (kt == w_kt: the re-read of the last step, T14 order below)
        {                 // 16 pixels on (images are < 2^15 pixels wide and high)
          w_dy += BK * p.k;
          w_pos += BK;
          w_x += BK * w_dcol;
          while ((w_pos & 0xffff) >= p.ow) {
            w_pos += (1 << 16) - p.ow;
            w_x += w_drow;
            if ((w_pos >> 16) == p.oh) {   // next image: row 0, same column
              w_pos &= 0xffff;
              w_x += w_dimg;
            }
          }
        }
        w_kt = kt;
      }
      const bool rv = kbase + (tid >> 5) < K;
      ra[0] = ld4(rv && a_ok[0] ? p.dy + w_dy : zero4);
      const int iy = (w_pos >> 16) * p.stride + ((w_tap + 32768) >> 16);
      const int ix = (w_pos & 0xffff) * p.stride + (int)(short)(w_tap & 0xffff);
      const bool v = b_ok[0] && rv && (unsigned)iy < (unsigned)p.h && (unsigned)ix < (unsigned)p.w;
      rbf[0] = ld4(v ? p.x + w_x : zero4);
      rbv = v;
    }
  };

  auto store_tile = [&](auto buf_c) {
    constexpr int buf = decltype(buf_c)::value;
    char *As = lds + buf * STAGE;
    char *Bs = As + 3 * IMG;
    if constexpr (!MC) {
#pragma unroll
      for (int i = 0; i < NQ; ++i) {
        const int o = kc16_off((tid >> 2) + 64 * i, sj >> 1) + 8 * (sj & 1);
        uint2 h, m, l;
        split3(ra[i], h, m, l);
        *reinterpret_cast<uint2 *>(As + o) = h;
        *reinterpret_cast<uint2 *>(As + IMG + o) = m;
        *reinterpret_cast<uint2 *>(As + 2 * IMG + o) = l;
      }
#pragma unroll
      for (int s = 0; s < 3; ++s) *reinterpret_cast<BChunk *>(Bs + s * IMGB + BPT * tid) = rbh[s];
    } else {
#pragma unroll
      for (int i = 0; i < NQ; ++i) {
        const int q = tid + NT * i;
        const int kr = q >> 5, col = 4 * (q & 31);
        const int o = mc_off(kr, col >> 3) + 8 * ((col >> 2) & 1);
        uint2 h, m, l;
        split3(ra[i], h, m, l);
        *reinterpret_cast<uint2 *>(As + o) = h;
        *reinterpret_cast<uint2 *>(As + IMG + o) = m;
        *reinterpret_cast<uint2 *>(As + 2 * IMG + o) = l;
        split3(rbf[i], h, m, l);
        *reinterpret_cast<uint2 *>(Bs + o) = h;
        *reinterpret_cast<uint2 *>(Bs + IMGB + o) = m;
        *reinterpret_cast<uint2 *>(Bs + 2 * IMGB + o) = l;
      }
    }
  };

  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WAVES_N, wn = wave - wm * WAVES_N;
  // M/N-contiguous images: each lane's two transposed-read offsets per fragment (conv_bf16.hpp
  // mc_frag) within one image, computed once; a read adds only the compile-time stage / term
  // image base, which the DS offset field absorbs
  uint32_t mca[MC ? TM : 1][2], mcb[MC ? TN : 1][2];
  if constexpr (MC) {
    const int g = lane >> 4, i16 = lane & 15, q = i16 >> 2, pp = i16 & 3;
    const int kb = 8 * (g >> 1);
    auto offs = [&](int c0, uint32_t (&o)[2]) {
      const int ch = ((c0 + 16 * (g & 1)) >> 3) + (pp >> 1);
      o[0] = (uint32_t)(mc_off(kb + q, ch) + 8 * (pp & 1));
      o[1] = (uint32_t)(mc_off(kb + 4 + q, ch) + 8 * (pp & 1));
    };
#pragma unroll
    for (int i = 0; i < TM; ++i) offs(wm * WTM + i * 32, mca[i]);
#pragma unroll
    for (int j = 0; j < TN; ++j) offs(wn * WTN + j * 32, mcb[j]);
  }
  const uint32_t lds_u32 = (uint32_t)(uintptr_t)lds;
  auto mc_read = [&](uint32_t img_base, const uint32_t (&o)[2]) -> bf16x8 {
    const bf16x4 t0 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4 *)(uintptr_t)(img_base + o[0]));
    const bf16x4 t1 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4 *)(uintptr_t)(img_base + o[1]));
    return __builtin_shufflevector(t0, t1, 0, 1, 2, 3, 4, 5, 6, 7);
  };

  floatx16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  // a0*b0 accumulates in acc, the five smaller cross terms in accs (see header comment)
  floatx16 accs[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) accs[i][j][r] = 0.f;

  // Wave priority: FWD / DGRAD raise it over their MFMAs (the waves holding MFMA work issue
  // first); WGRAD, whose staging splits both operands (twice the vector work), raises it over
  // the split + LDS stores instead, so a staging wave is not starved behind the other wave's
  // MFMAs (measured: FWD 152.5 vs 148.6 TF/s with the WGRAD choice, WGRAD 142.0 vs 131.8 with
  // the FWD one, tools/dbg/ab_libs.sh).
  // One 16-deep K step from LDS buffer `cur` (a compile-time stage: the loop below is unrolled
  // by two, so every fragment and staging address is a loop-invariant VGPR plus an immediate
  // offset — with a runtime stage the weight gradient spent ~30 v_add_u32 per step rebuilding its
  // 18 transposed-read addresses): the six split products of every 32x32 tile, term-major so
  // consecutive MFMAs write different accumulators.  The kernels then split + store the NEXT
  // step's staged registers into LDS buffer cur^1 in the same basic block, and the scheduler
  // interleaves that vector / LDS work between the MFMAs (one MFMA, three VALU, one LDS store)
  // instead of running it after them.
  // ABN: the staged x float4 (loaded one step earlier) through the operand BN, in place, before
  // this step's fragments are live (inside the MFMA-interleaved split below it spilled)
  auto abn_x = [&]() {
    if constexpr (ABN) {
      const float *L = reinterpret_cast<const float *>(lds + 2 * STAGE) + b_off[0];
      const float4 bm4 = *reinterpret_cast<const float4 *>(L);
      const float4 bi4 = *reinterpret_cast<const float4 *>(L + kAbnMaxC);
      const float4 bw4 = *reinterpret_cast<const float4 *>(L + 2 * kAbnMaxC);
      const float4 bb4 = *reinterpret_cast<const float4 *>(L + 3 * kAbnMaxC);
      float4 &xv = rbf[0];
      xv.x = rbv ? bn_relu(xv.x, bm4.x, bi4.x, bw4.x, bb4.x) : 0.f;
      xv.y = rbv ? bn_relu(xv.y, bm4.y, bi4.y, bw4.y, bb4.y) : 0.f;
      xv.z = rbv ? bn_relu(xv.z, bm4.z, bi4.z, bw4.z, bb4.z) : 0.f;
      xv.w = rbv ? bn_relu(xv.w, bm4.w, bi4.w, bw4.w, bb4.w) : 0.f;
    }
  };
  auto compute = [&](auto cur_c) {
    constexpr int cur = decltype(cur_c)::value;
    const char *As = lds + cur * STAGE;
    const char *Bs = As + 3 * IMG;
    abn_x();
    bf16x8 a[3][TM], b[3][TN];
#pragma unroll
    for (int s = 0; s < 3; ++s) {
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        if constexpr (MC) a[s][i] = mc_read(lds_u32 + cur * STAGE + s * IMG, mca[i]);
        else a[s][i] = kc16_frag(As + s * IMG, wm * WTM + i * 32, lane);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        if constexpr (MC) b[s][j] = mc_read(lds_u32 + cur * STAGE + 3 * IMG + s * IMGB, mcb[j]);
        else b[s][j] = kc16_frag(Bs + s * IMGB, wn * WTN + j * 32, lane);
      }
    }
    constexpr int TA[6] = {0, 0, 1, 0, 1, 2};
    constexpr int TB[6] = {0, 1, 0, 2, 1, 0};
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int u = 0; u < 6; ++u)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          if (u == 0) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][i], b[0][j], acc[i][j], 0, 0, 0);
          else accs[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[TA[u]][i], b[TB[u]][j], accs[i][j], 0, 0, 0);
        }
    store_tile(std::integral_constant<int, cur ^ 1>{});
#pragma unroll
    for (int q = 0; q < 6 * TM * TN; ++q) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // 1 MFMA
      __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);   // 3 VALU
      __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);   // 1 LDS store
    }
    __builtin_amdgcn_s_setprio(0);
  };

  if constexpr (ABN) {   // the operand BN's channel parameters (weight / bias NULL: 1 / 0)
    float *L = reinterpret_cast<float *>(lds + 2 * STAGE);
    for (int c = tid; c < p.c; c += NT) {
      L[c] = p.abn_m[c];
      L[kAbnMaxC + c] = p.abn_is[c];
      L[2 * kAbnMaxC + c] = p.abn_w ? p.abn_w[c] : 1.f;
      L[3 * kAbnMaxC + c] = p.abn_b ? p.abn_b[c] : 0.f;
    }
    __syncthreads();
  }
  if (kt0 < kt1) {
    // T14 order with unconditional staging (past the last step it re-reads step kt1-1 into
    // the LDS buffer nobody reads again): registers hold step kt+1 while step kt computes
    const int klast = kt1 - 1;
    load_tile(kt0);
    abn_x();
    store_tile(std::integral_constant<int, 0>{});
    load_tile(min(kt0 + 1, klast));
    __syncthreads();
    for (int kt = kt0; kt < kt1; kt += 2) {
      compute(std::integral_constant<int, 0>{});
      load_tile(min(kt + 2, klast));
      __syncthreads();
      if (kt + 1 >= kt1) break;
      compute(std::integral_constant<int, 1>{});
      load_tile(min(kt + 3, klast));
      __syncthreads();
    }
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
__global__ void __launch_bounds__(x3_threads(MODE), 4) igemm_x3_kernel(const ConvParams p, const __bf16 *__restrict__ wb) {
  x3_body<MODE, S2, false>(p, wb);
}
// the weight gradient with the operand BN on x (ConvParams::abn_*)
__global__ void __launch_bounds__(x3_threads(MODE_WGRAD), 4) igemm_x3_abn_kernel(const ConvParams p,
                                                                               const __bf16 *__restrict__ wb) {
  x3_body<MODE_WGRAD, false, true>(p, wb);
}

// Weight pack: the three bf16 terms of every weight of the GEMM's B operand (FWD: row n = Cout,
// k = (seg, tap, ci); DGRAD: row n = Cin, k = (tap, co)) at the byte the kernel's LDS tile
// wants: [n / 128][k / 16][term][kc16 image of 128 rows x 16 k]; rows >= N are zeros.
// One thread per (row, 8-k chunk): eight weights gathered (FWD: two float4 of
// a K-contiguous row; DGRAD: eight scalars, consecutive lanes on consecutive input channels
// so every load is coalesced), split, and stored as one 16-B chunk per term image — a wave
// writes 1 KB contiguous per term instead of 2-B elements 32 B apart.  grid = (rows_pad / 128,
// ktot / 16), 256 threads: thread t -> row t >> 1, chunk t & 1.
template <int MODE>
__global__ void __launch_bounds__(256) conv_wpack_x3v_kernel(const ConvParams p, char *out, int ktot) {
  constexpr int TR = x3_bn(MODE), IMGB = TR * kX3BK * 2;
  const int r = threadIdx.x >> 1, ch = threadIdx.x & 1;
  const int n = blockIdx.x * TR + r;
  const int ks = blockIdx.y, k0 = ks * kX3BK + 8 * ch;
  float v[8];
  if constexpr (MODE == MODE_FWD) {   // W_seg[co][tk], k = seg * kseg + tk (kseg % 16 == 0)
    if (n < p.k) {
      const int seg = k0 / p.kseg;
      const float *src = seg_ptr(p, seg) + (size_t)n * p.kseg + (k0 - seg * p.kseg);
      const float4 a = ld4(src), b = ld4(src + 4);
      v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = 0.f;
    }
  } else {   // W_seg(tap)[co][t][ci], k = tap * Cout + co (Cout % 16 == 0), row n = ci
    const int tap = k0 / p.k, co = k0 - tap * p.k;
    const int seg = tap / p.taps_per_seg, t = tap - seg * p.taps_per_seg;
    const float *src = seg_ptr(p, seg) + ((size_t)co * p.taps_per_seg + t) * p.c + n;
    const size_t cs = (size_t)p.taps_per_seg * p.c;   // stride between consecutive co
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = n < p.c ? src[j * cs] : 0.f;
  }
  uint4 h, m, l;
  split3_2(v[0], v[1], h.x, m.x, l.x);
  split3_2(v[2], v[3], h.y, m.y, l.y);
  split3_2(v[4], v[5], h.z, m.z, l.z);
  split3_2(v[6], v[7], h.w, m.w, l.w);
  const int nkt = ktot / kX3BK;
  char *dst = out + ((size_t)blockIdx.x * nkt + ks) * 3 * IMGB + kc16_off(r, ch);
  *reinterpret_cast<uint4 *>(dst) = h;
  *reinterpret_cast<uint4 *>(dst + IMGB) = m;
  *reinterpret_cast<uint4 *>(dst + 2 * IMGB) = l;
}

}  // namespace adaptseg
