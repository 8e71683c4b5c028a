// bf16 implicit-GEMM convolution fed by LDS-DMA (global_load_lds_dwordx4) — the forward and
// stride-1 data-gradient products of the bf16 conv math (config c5) whose operands are bf16 in
// HBM: the activation operand is a bf16 NHWC copy (written once per call by bf16_copy_kernel,
// conv_launch_bf16.hip), the weights the K-contiguous bf16 pack of conv_bf16.hpp.
//
// Why a second bf16 kernel: igemm_bf16_kernel gathers the fp32 activations into registers and
// rounds them while staging.  Its PMC (profiles/r2/pmc/bf16_l3conv2_counters.txt): 163 VALU per
// 16 MFMAs per wave and K step, 30 % of wave time waiting on loads, MFMA busy 0.25 — one K step
// of prefetch (one register set; a second one does not fit) does not cover the gather latency,
// and every step moves twice the bytes the MFMA consumes.  Here no operand passes through
// registers: each K step is 6 LDS-DMA instructions per wave into a 3-deep LDS ring, two tiles
// stay in flight across each barrier (counted vmcnt, raw s_barrier — a __syncthreads() would
// drain them), and the loop body is ds_read + MFMA only.
//
// Tile BM x BN x 64 (128x256 or 256x128), 8 waves of 64x64 (2x2 MFMA tiles of 32x32x16), LDS
// 3 x 48 KB (one block per CU).  The LDS images are conv_bf16.hpp's K-contiguous [row][64 k]
// images with the 16-B chunk of row r at (ch ^ (r>>1 & 7)): an LDS-DMA instruction writes its
// 64 lanes' 16 B linearly (8 whole 128-B rows), so the swizzle goes on the SOURCE address —
// lane l of the instruction loads chunk (l&7) ^ (r>>1 & 7) of its row r.  Rows outside the
// image (padding taps, m >= M, n >= N) load from a 16-B zero block instead.
#pragma once
#include "conv_bf16.hpp"

namespace adaptseg {

// 16 zero bytes: the source of every padded operand row
static __device__ __attribute__((aligned(16))) unsigned int g_bf16g_zero[4];

// One LDS-DMA wave instruction: lane l's 16 source bytes land at LDS byte lds_dst + 16 l.  In
// inline asm, not __builtin_amdgcn_global_load_lds: hipcc (ROCm 7.2) cannot tell the DMA's LDS
// writes from the ring stages the ds_reads use and waits vmcnt(0) before the first ds_read of
// every K step, draining the two steps in flight.  The kernel counts these loads itself
// (s_waitcnt vmcnt(N) + raw s_barrier); M0 is written and restored in the same statement.
__device__ __forceinline__ void glds16(const void *src, uint32_t lds_dst) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(src), "s"(lds_dst)
               : "memory");
}

constexpr int kG16Stages = 3;

// s_waitcnt vmcnt(N): this wave's LDS-DMA loads but the last N have landed
template <int N> __device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt field");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
constexpr int g16_stage_bytes(int bm, int bn, int bk) { return (bm + bn) * bk * 2; }

// Byte offset of 16-B chunk ch of row r in a K-contiguous image of BK bf16 per row.  BK 64:
// conv_bf16.hpp's kc_off (128-B rows, ch ^ (r>>1 & 7)); BK 32: 64-B rows, ch ^ (r>>2 & 3) —
// conflict-free for the ds_read_b128 lane groups of the 32x32x16 fragment reads.
template <int BK>
__device__ __forceinline__ int g16_off(int r, int ch) {
  if constexpr (BK == 64) return r * 128 + ((ch ^ ((r >> 1) & 7)) << 4);
  else return r * 64 + ((ch ^ ((r >> 2) & 3)) << 4);
}

// BK 64: one block per CU (3 x 48 KB ring); BK 32: two (3 x 24 KB), so one block's epilogue and
// prologue overlap the other's K loop (short-K 1x1 products).
// S2: the stride-2 data gradient by output-pixel parity class (blockIdx.z = 2 py + px), each a
// dense stride-1 GEMM over its subgrid with only its taps, as igemm_x3_kernel / igemm_bf16_kernel.
// 256x256 (BK 32 only: a 3 x 32 KB ring): 8 waves of 64x128, 128 accumulator VGPRs, one block per
// CU — half the operand bytes per MFMA of the 128x256 tile, for products whose M x N fills the
// chip with such tiles.
// NST: LDS stages.  3 (the default): two K steps in flight across each barrier.  2 (256x256x64,
// "wide"): 2 x 64 KB, one step in flight — issued right after the barrier that opens the step
// before it, so it has that step's MFMAs (16 waves x 16, 2,048 cycles per SIMD) to land; twice
// the MFMA cycles per SIMD per barrier of the 128x256x64 tile and 2/3 of its operand bytes per
// MFMA.
template <int MODE, int BM, int BN, int BK, bool S2 = false, int NST = kG16Stages>
__global__ void __launch_bounds__(NST == 2 ? 1024 : 512, (BK == 32 && BM * BN < 65536) || NST == 2 ? 4 : 2)
igemm_bf16g_kernel(const ConvParams p,
                                                                              const __bf16 *__restrict__ ab,
                                                                              const __bf16 *__restrict__ wb) {
  static_assert(MODE == MODE_FWD || MODE == MODE_DGRAD, "K-contiguous products only");
  static_assert(!S2 || MODE == MODE_DGRAD, "parity classes: data gradient only");
  static_assert(BK == 64 || BK == 32, "K step");
  static_assert(NST == 3 || NST == 2, "ring depth");
  // 8 waves; the two-stage 256x256 tile: 16 waves of 64x64 (4 per SIMD, the 64x64 wave code
  // and its <= 128 registers: 64x128 wave tiles spill at two waves per SIMD)
  constexpr int NW = NST == 2 ? 16 : 8, NT = 64 * NW;
  constexpr int WAVES_M = BM / 64, WAVES_N = NW / WAVES_M;  // 64 x (BN / WAVES_N) wave tiles
  static_assert(WAVES_M * WAVES_N == NW && BN % (32 * WAVES_N) == 0, "wave grid");
  static_assert(BM * BN < 65536 || BK == 32 || NST == 2, "256x256 tiles: K step 32, or 64 on two stages");
  constexpr int WTM = 64, WTN = BN / WAVES_N, TM = 2, TN = WTN / 32;
  constexpr int LPR = BK / 8;                          // lanes per image row (16 B each)
  constexpr int RPI = 64 / LPR;                        // rows per LDS-DMA instruction
  constexpr int NA = BM / (NW * RPI), NB = BN / (NW * RPI);  // instructions per wave and K step
  constexpr int IMGA = BM * BK * 2;
  constexpr int STAGE = g16_stage_bytes(BM, BN, BK);
  (void)NT;

  __shared__ __attribute__((aligned(16))) char lds[NST * STAGE];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
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
  // bf16 copy of the activation operand: NHWC contiguous, channel count ca
  const int ca = MODE == MODE_FWD ? p.c : p.k;

  // ---- per-lane rows: instruction i of wave w covers image rows 8 RPI i + RPI w .. +RPI-1 ----
  const int rsub = wave * RPI + lane / LPR;                 // row within an NW RPI-row group
  // source chunk (elements) of this lane: the one whose swizzled slot is the lane's (lane % LPR)
  const int chs = (BK == 64 ? ((lane & 7) ^ ((rsub >> 1) & 7)) : ((lane & 3) ^ ((rsub >> 2) & 3))) * 8;
  int a_pix[NA], a_y[NA], a_x[NA];
  bool a_ok[NA];
#pragma unroll
  for (int i = 0; i < NA; ++i) {
    const int m = bm + NW * RPI * i + rsub;
    a_ok[i] = m < M;
    const int mm = min(m, M - 1);
    if constexpr (S2) {   // row = (b, i, j) of the parity class's subgrid
      const int j = mm % Wc, t2 = mm / Wc;
      const int ii = t2 % Hc, b = t2 / Hc;
      a_y[i] = ii;
      a_x[i] = j;
      a_pix[i] = ((b * p.oh + ii) * p.ow + j) * ca + chs;
    } else if constexpr (MODE == MODE_FWD) {
      uint32_t t = fdiv((uint32_t)mm, p.fd_ow);
      const int ow = mm - (int)t * p.ow;
      uint32_t b = fdiv(t, p.fd_oh);
      const int oh = (int)t - (int)b * p.oh;
      a_y[i] = oh * p.stride;
      a_x[i] = ow * p.stride;
      a_pix[i] = (((int)b * p.h + a_y[i]) * p.w + a_x[i]) * ca + chs;
    } else {
      uint32_t t = fdiv((uint32_t)mm, p.fd_w);
      const int iw = mm - (int)t * p.w;
      uint32_t b = fdiv(t, p.fd_hw);
      const int ih = (int)t - (int)b * p.h;
      a_y[i] = ih;
      a_x[i] = iw;
      a_pix[i] = (((int)b * p.oh + ih) * p.ow + iw) * ca + chs;
    }
  }
  int b_off[NB];
  bool b_ok[NB];
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    const int n = bn + NW * RPI * j + rsub;
    b_ok[j] = n < p.N;
    b_off[j] = min(n, p.N - 1) * ktot + chs;
  }
  const __bf16 *zero = reinterpret_cast<const __bf16 *>(g_bf16g_zero);

  // LDS-DMA of K step kt into ring stage st: NA + NB instructions per wave
  auto issue = [&](int kt, int st) {
    const int kbase = kt * BK;
    const uint32_t As = uni((int)((uint32_t)(uintptr_t)lds + st * STAGE + wave * 1024));
    const uint32_t Bs = As + IMGA;
    int soff, wk, dy, dx;
    if constexpr (MODE == MODE_FWD) {
      const int tap = uni((int)fdiv((uint32_t)kbase, p.fd_c));
      int seg, t;
      seg_geom(p, sr, tap, seg, t, dy, dx);
      dy = uni(dy);
      dx = uni(dx);
      soff = uni((dy * p.w + dx) * ca + kbase - tap * p.c);
      wk = kbase;
    } else if constexpr (S2) {   // tap (u, v) of the class: kernel row kh0 + 2u, column kw0 + 2v
      const int tap = uni((int)fdiv((uint32_t)kbase, p.fd_k));
      const int co0 = kbase - tap * p.k;
      const int u = tap / nkw, v = tap - u * nkw;
      const int kh = kh0 + 2 * u, kw = kw0 + 2 * v;
      dy = uni((py + p.pad_[0] - kh) >> 1);   // dY row offset from subgrid row ii
      dx = uni((px + p.pad_[0] - kw) >> 1);
      soff = uni((dy * p.ow + dx) * ca + co0);
      wk = uni((kh * p.kw_ + kw) * p.k + co0);   // packed row offset of (tap, co0)
    } else {
      const int tap = uni((int)fdiv((uint32_t)kbase, p.fd_k));
      int seg, t;
      seg_geom(p, sr, tap, seg, t, dy, dx);
      dy = uni(-dy);   // the data gradient reads dY at (ih - dy, iw - dx)
      dx = uni(-dx);
      soff = uni((dy * p.ow + dx) * ca + kbase - tap * p.k);
      wk = kbase;
    }
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      bool v;
      if constexpr (MODE == MODE_FWD)
        v = a_ok[i] & ((unsigned)(a_y[i] + dy) < (unsigned)p.h) & ((unsigned)(a_x[i] + dx) < (unsigned)p.w);
      else
        v = a_ok[i] & ((unsigned)(a_y[i] + dy) < (unsigned)p.oh) & ((unsigned)(a_x[i] + dx) < (unsigned)p.ow);
      glds16(v ? ab + a_pix[i] + soff : zero, As + i * NW * 1024);
    }
#pragma unroll
    for (int j = 0; j < NB; ++j) glds16(b_ok[j] ? wb + b_off[j] + wk : zero, Bs + j * NW * 1024);
  };

  const int wm = wave / WAVES_N, wn = wave - wm * WAVES_N;
  floatx16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  auto compute = [&](int st) {
    const char *As = lds + st * STAGE;
    const char *Bs = As + IMGA;
    bf16x8 a[2][TM], b[2][TN];
    auto read_frags = [&](int ks, int slot) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
        a[slot][i] = as_bf16x8(*reinterpret_cast<const uint4 *>(
            As + g16_off<BK>(wm * WTM + i * 32 + (lane & 31), 2 * ks + (lane >> 5))));
#pragma unroll
      for (int j = 0; j < TN; ++j)
        b[slot][j] = as_bf16x8(*reinterpret_cast<const uint4 *>(
            Bs + g16_off<BK>(wn * WTN + j * 32 + (lane & 31), 2 * ks + (lane >> 5))));
    };
    read_frags(0, 0);
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
      const int cb = ks & 1;
      if (ks + 1 < BK / 16) read_frags(ks + 1, cb ^ 1);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[cb][i], b[cb][j], acc[i][j], 0, 0, 0);
    }
  };

  if constexpr (NST == 2) {
   if (kt0 < kt1) {
    // two stages, one K step in flight: step kt lives in stage (kt - kt0) & 1
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
  } else if (kt0 < kt1) {
    // Ring of 3 stages, two K steps in flight: step kt lives in stage (kt - kt0) % 3.  The loads
    // past the last step re-read it into a stage nobody reads again, so every wave always has
    // exactly NA + NB instructions per step outstanding and the counted wait stays constant.
    const int klast = kt1 - 1;
    issue(kt0, 0);
    issue(min(kt0 + 1, klast), 1);
    int st = 0;
    for (int kt = kt0; kt < kt1; ++kt) {
      // this wave's DMAs of step kt are done (step kt+1's NA + NB stay in flight) ...
      static_assert(NST == 2 || NA + NB == 6 || NA + NB == 4 || NA + NB == 3,
                    "vmcnt below counts 6, 4 or 3 instructions per step");
      if constexpr (NA + NB == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      else if constexpr (NA + NB == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
      // ... and after the barrier every wave's are, and every wave has finished reading the
      // stage that step kt+2 overwrites (step kt-1's)
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");   // no LDS access moves above the barrier
      const int st2 = st == 0 ? 2 : st - 1;  // (st + 2) % 3
      issue(min(kt + 2, klast), st2);
      compute(st);
      st = st == 2 ? 0 : st + 1;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // the epilogue reuses the LDS
  }

  static_assert(NST * STAGE >= WAVES_M * WAVES_N * 32 * 33 * 4, "LDS for the bf16x8 epilogue");
  igemm_epilogue<MODE, BM, BN, WAVES_M, WAVES_N, S2, 1>(p, acc, bm, bn, tm, tn, split, M, Hc, Wc, py, px,
                                                      reinterpret_cast<float *>(lds));
}

// Weight gradient on the same LDS-DMA ring: dW[co][tap, ci] = sum_pix dY[pix][co] x[pix+tap][ci]
// with both operands bf16 copies in HBM (dY: the producing BN backward's copy, x: the forward
// BN's).  k = output pixel, so both images are M/N-contiguous [32 k][128] (conv_bf16.hpp's
// 256-B rows, read with ds_read_b64_tr_b16; BM 256 = two A images); one LDS-DMA instruction
// fills 4 k-rows, so a K step of 32 pixels is BM/128 A and one B instruction per wave.  Each
// lane's 16-B column chunk (8 input channels, Cin % 8 == 0) has its own tap, so a 128-column
// tile may span taps (Cin 64: two); a chunk of a tap outside the image loads zeros.  BM 256 (Cout >= 256) reads dY once per column
// tile instead of twice; 8 waves of 64x32 (BM 128) or 64x64 (BM 256); 3-stage ring of 16 / 24
// KB, two blocks per CU.  BN 256 (with BM 256): two B images, 8 waves of 64x128, a 3 x 32 KB ring
// and one block per CU — half the operand bytes per MFMA of 256x128.
// NS: LDS ring depth, NS - 1 K steps in flight across each barrier (3: two).  NS 2 with 256x256
// ("wide", ADAPTSEG_OPT_G16_WIDE): 16 waves of 64x64 and K steps of 64 pixels (each wave DMAs four
// k-rows of every image), two 64 KB stages, one step in flight — 16 MFMAs per wave and 2,048
// MFMA cycles per SIMD between barriers (the 256x128 tile: 8 and 512) and half its operand bytes
// per MFMA.
constexpr int g16w_waves(int bm, int bn, int ns) { return (bm == 256 && bn == 256 && ns == 2) ? 16 : 8; }
template <int BM, int BN = 128, int NS = kG16Stages>
__global__ void __launch_bounds__(64 * g16w_waves(BM, BN, NS), g16w_waves(BM, BN, NS) == 16 ? 4 : (BN == 256 || NS > 4) ? 1 : 2)
igemm_bf16g_wgrad_kernel(const ConvParams p, const __bf16 *__restrict__ dyb, const __bf16 *__restrict__ xb) {
  constexpr int NW = g16w_waves(BM, BN, NS);
  constexpr int BKP = 4 * NW;                 // pixels per K step: four k-rows per wave
  static_assert(BN == 128 || (BN == 256 && BM == 256), "wgrad tiles 128x128, 256x128, 256x256");
  constexpr int WAVES_M = BM / 64, WAVES_N = NW / WAVES_M;
  constexpr int WTM = 64, WTN = BN / WAVES_N, TM = 2, TN = WTN / 32;
  constexpr int NA = BM / 128;                // A images / instructions per wave and K step
  constexpr int NB = BN / 128;                // B images
  constexpr int IMG = BKP * 256;              // one [32 k][128] bf16 image
  constexpr int STAGE = (NA + NB) * IMG;
  // (a 4- / 6-deep ring measured no faster, profiles/r5/g16_wgrad_ring_ab.txt: the K loop is
  // unrolled over exactly three stages)
  static_assert((NS == 3 || (NS == 2 && NW == 16)) && NS * STAGE <= 160 * 1024, "ring depth");

  __shared__ __attribute__((aligned(16))) char lds[NS * STAGE];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int ntn = (p.N + BN - 1) / BN;
  int tile, split;
  xcd_tile_split(tile, split);
  const int tm = tile / ntn, tn = tile - tm * ntn;
  const int bm = tm * BM, bn = tn * BN;
  const SegRegs sr = seg_regs(p);

  const int K = p.K;                          // output pixels
  const int nkt = (K + BKP - 1) / BKP;
  const int kt0 = split * p.ktiles_per_split;
  const int kt1 = min(nkt, kt0 + p.ktiles_per_split);

  // this lane's k-row (pixel within the step) and 16-B slot; the source chunk whose swizzled
  // position (mc_off) is that slot
  const int kr = 4 * wave + (lane >> 4);
  const int chs = ((lane & 15) ^ (((kr & 3) << 2) | ((kr >> 2) & 3))) * 8;
  bool a_col[NA];
#pragma unroll
  for (int i = 0; i < NA; ++i) a_col[i] = bm + 128 * i + chs < p.M;   // Cout % 8 == 0
  // this lane's column chunk of each B image: its tap (per lane: with Cin % 128 != 0 a tile
  // spans taps) and input channel
  bool b_col[NB];
  int tdy[NB], tdx[NB], ci[NB];
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    b_col[j] = bn + 128 * j + chs < p.N;
    const int ncol = b_col[j] ? bn + 128 * j + chs : 0;
    const int tap = (int)fdiv((uint32_t)ncol, p.fd_c);
    int seg, t;
    seg_geom(p, sr, tap, seg, t, tdy[j], tdx[j]);
    ci[j] = ncol - tap * p.c;
  }
  const __bf16 *zero = reinterpret_cast<const __bf16 *>(g_bf16g_zero);
  // x element offset of each B chunk's tap and channel, relative to its pixel's (oh s, ow s)
  int xo[NB];
#pragma unroll
  for (int j = 0; j < NB; ++j) xo[j] = (tdy[j] * p.w + tdx[j]) * p.c + ci[j];

  // This lane's pixel walk: the pixel m = kt BKP + kr it loads, its output row / column and the
  // element offsets of its dY row (column bm + chs) and of its x pixel, advanced one K step at a
  // time (issue() sees non-decreasing kt: the re-reads past the last step repeat it) instead of
  // two divisions and a 64-bit multiply per step.  32-bit offsets: the host plans this kernel
  // only for operands of < 2^31 elements (g16_wgrad_fits).
  int w_kt = kt0, w_m = kt0 * BKP + kr, w_ow, w_oh, w_a, w_x;
  {
    const uint32_t q = fdiv((uint32_t)w_m, p.fd_ow);
    w_ow = w_m - (int)q * p.ow;
    const uint32_t b = fdiv(q, p.fd_oh);
    w_oh = (int)q - (int)b * p.oh;
    w_a = w_m * p.k + bm + chs;
    w_x = (((int)b * p.h + w_oh * p.stride) * p.w + w_ow * p.stride) * p.c;
  }
  const int x_col = p.stride * p.c;                              // x offset per output column
  const int x_row = (p.stride * p.w - p.ow * p.stride) * p.c;     // ... at a row wrap
  const int x_img = (p.h - p.oh * p.stride) * p.w * p.c;         // ... at an image wrap

  auto issue = [&](int kt, int st) {
    if (kt != w_kt) {   // kt == w_kt + 1
      w_kt = kt;
      w_m += BKP;
      w_a += BKP * p.k;
      w_ow += BKP;
      w_x += BKP * x_col;
      while (w_ow >= p.ow) {
        w_ow -= p.ow;
        w_x += x_row;
        if (++w_oh == p.oh) {
          w_oh = 0;
          w_x += x_img;
        }
      }
    }
    const uint32_t As = uni((int)((uint32_t)(uintptr_t)lds + st * STAGE + wave * 1024));
    const bool rv = w_m < K;
#pragma unroll
    for (int i = 0; i < NA; ++i) glds16((rv & a_col[i]) ? dyb + (w_a + 128 * i) : zero, As + i * IMG);
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const int iy = w_oh * p.stride + tdy[j], ix = w_ow * p.stride + tdx[j];
      const bool bv = rv & b_col[j] & ((unsigned)iy < (unsigned)p.h) & ((unsigned)ix < (unsigned)p.w);
      glds16(bv ? xb + (w_x + xo[j]) : zero, As + (NA + j) * IMG);
    }
  };

  const int wm = wave / WAVES_N, wn = wave - wm * WAVES_N;
  floatx16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // Every fragment read's per-lane byte offset within a ring stage (mc_frag's two transposed
  // reads, image base included), computed once: a read adds only the compile-time stage base,
  // which the DS offset field absorbs (the K loop below is unrolled over the NS stages).  Sub-step
  // ks + 1 is 16 k-rows (4 KB) further with the same swizzle (mc_off: k-row bits 0-3): only the
  // ks = 0 offsets are kept.
  constexpr int KS = BKP / 16;
  uint32_t oa[TM][1][2], ob[TN][1][2];
  {
    const int g = lane >> 4, i16 = lane & 15, q = i16 >> 2, pp = i16 & 3;
    auto offs = [&](int img, int c0, int ks, uint32_t (&o)[2]) {
      const int ch = ((c0 + 16 * (g & 1)) >> 3) + (pp >> 1);
      const int kb = 16 * ks + 8 * (g >> 1);
      o[0] = (uint32_t)(img + mc_off(kb + q, ch) + 8 * (pp & 1));
      o[1] = (uint32_t)(img + mc_off(kb + 4 + q, ch) + 8 * (pp & 1));
    };
    const int ia = (wm * WTM / 128) * IMG, ib = (NA + (wn * WTN) / 128) * IMG;   // this wave's A / B image
    const int ar = (wm * WTM) % 128, bc = (wn * WTN) % 128;
#pragma unroll
    for (int i = 0; i < TM; ++i) offs(ia, ar + i * 32, 0, oa[i][0]);
#pragma unroll
    for (int j = 0; j < TN; ++j) offs(ib, bc + j * 32, 0, ob[j][0]);
  }
  const uint32_t lds_u32 = (uint32_t)(uintptr_t)lds;
  auto rd = [&](uint32_t base, const uint32_t (&o)[2]) -> bf16x8 {
    const bf16x4 t0 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4 *)(uintptr_t)(base + o[0]));
    const bf16x4 t1 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4 *)(uintptr_t)(base + o[1]));
    return __builtin_shufflevector(t0, t1, 0, 1, 2, 3, 4, 5, 6, 7);
  };

  auto compute = [&](auto st_c) {
    constexpr int st = decltype(st_c)::value;
    const uint32_t sb = lds_u32 + st * STAGE;
    bf16x8 a[2][TM], b[2][TN];
    auto read_frags = [&](int ks, int slot) {
#pragma unroll
      for (int i = 0; i < TM; ++i) a[slot][i] = rd(sb + 4096 * ks, oa[i][0]);
#pragma unroll
      for (int j = 0; j < TN; ++j) b[slot][j] = rd(sb + 4096 * ks, ob[j][0]);
    };
    read_frags(0, 0);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int cb = ks & 1;
      if (ks + 1 < KS) read_frags(ks + 1, cb ^ 1);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[cb][i], b[cb][j], acc[i][j], 0, 0, 0);
    }
  };

  if constexpr (NS == 2) {
    if (kt0 < kt1) {   // two stages, one step in flight (issued after the barrier opening the step before)
      issue(kt0, 0);
      for (int kt = kt0; kt < kt1; kt += 2) {
        wait_vmcnt<0>();
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (kt + 1 < kt1) issue(kt + 1, 1);
        compute(std::integral_constant<int, 0>{});
        if (kt + 1 >= kt1) break;
        wait_vmcnt<0>();
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (kt + 2 < kt1) issue(kt + 2, 0);
        compute(std::integral_constant<int, 1>{});
      }
      __syncthreads();
    }
  } else if (kt0 < kt1) {
    // step kt lives in stage (kt - kt0) % NS; steps past the last re-read it into stages nobody
    // reads again, so every wave always has NS - 2 steps' NA + NB instructions outstanding
    const int klast = kt1 - 1;
#pragma unroll
    for (int i = 0; i < NS - 1; ++i) issue(min(kt0 + i, klast), i);
    auto step = [&](auto st_c, int kt) {
      constexpr int st = decltype(st_c)::value;
      // step kt landed (steps kt+1 .. kt+NS-2 in flight) ...
      wait_vmcnt<(NS - 2) * (NA + NB)>();
      // ... in every wave after the barrier, which also retires every wave's reads of step kt-1's
      // stage, the one step kt+NS-1 overwrites
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");   // no LDS access moves above the barrier
      issue(min(kt + NS - 1, klast), (st + NS - 1) % NS);
      compute(st_c);
    };
    for (int kt = kt0; kt < kt1; kt += 3) {   // (NS == 3: one unrolled pass per ring turn)
      step(std::integral_constant<int, 0>{}, kt);
      if (kt + 1 >= kt1) break;
      step(std::integral_constant<int, 1>{}, kt + 1);
      if (kt + 2 >= kt1) break;
      step(std::integral_constant<int, 2>{}, kt + 2);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  igemm_epilogue<MODE_WGRAD, BM, BN, WAVES_M, WAVES_N, false>(p, acc, bm, bn, tm, tn, split, p.M, p.h, p.w, 0, 0,
                                                              reinterpret_cast<float *>(lds));
}

}  // namespace adaptseg
