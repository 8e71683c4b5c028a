// Implicit-GEMM convolution on bf16 MFMA (v_mfma_f32_32x32x16_bf16, fp32 accumulate) for
// gfx950 — the "bf16" conv math of BASELINE config c5 (adaptseg_conv_set_math).
//
// Same three products, gathers, tile order, split-K and epilogue as igemm_fast_kernel
// (conv_kernels.hpp); what changes is the operand path:
//   * activations stay fp32 in HBM; each K tile is gathered as fp32 and rounded to bf16
//     (round-to-nearest-even, v_cvt_pk_bf16_f32) on its way into LDS;
//   * weights are packed once per call into bf16 K-contiguous rows (FWD: Wf[co][seg,tap,ci],
//     DGRAD: Wd[ci][seg,tap,co]) by conv_wpack_*_kernel, so the B operand of FWD and DGRAD is a
//     plain 16-byte load straight into LDS;
//   * LDS images: a K-contiguous operand is [row][64 k] (128-B rows, 16-B chunk ch of row r at
//     (ch ^ (r>>1 & 7)) — conflict-free for the ds_read_b128 fragment reads and the
//     ds_write_b128 stores); an M/N-contiguous operand (both WGRAD operands: k = output pixel)
//     is [64 k][128 m] (256-B rows, chunk ch at ch ^ ((r&3)<<2 | (r>>2)&3)) read with the
//     ds_read_b64_tr_b16 transpose, so neither operand is transposed through registers.
// Block tile 128x128x64.  FWD / DGRAD: 8 waves (2x4) of 64x32 wave tiles, 114-116 VGPRs (two
// blocks per CU), the next K step's conversion + LDS stores interleaved with this step's MFMAs
// in T14 order (+6 % on the c2-shape bf16 products over 4 waves of 64x64 with staging after
// the MFMAs).  WGRAD: 4 waves (2x2) of 64x64.
#pragma once
#include "conv_kernels.hpp"
#include <type_traits>

namespace adaptseg {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float floatx4v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;

constexpr int kB16BK = 64;
// threads per block: 4 waves (2x2 of 64x64) for the weight gradient, 8 waves (2x4) for the
// K-contiguous products
constexpr int bf16_threads(int mode) { return mode == MODE_WGRAD ? 256 : 512; }

// 128-B row (64 bf16 along k), 16-B chunk ch (8 k) of row r
__device__ __forceinline__ int kc_off(int r, int ch) { return r * 128 + ((ch ^ ((r >> 1) & 7)) << 4); }
// 256-B row (128 bf16 along m/n), 16-B chunk ch (8 m) of k-row r
__device__ __forceinline__ int mc_off(int r, int ch) {
  return r * 256 + ((ch ^ (((r & 3) << 2) | ((r >> 2) & 3))) << 4);
}

__device__ __forceinline__ uint2 cvt4_bf16(float4 v) {
  floatx4v f = {v.x, v.y, v.z, v.w};
  bf16x4 h = __builtin_convertvector(f, bf16x4);
  return __builtin_bit_cast(uint2, h);
}

__device__ __forceinline__ bf16x8 as_bf16x8(uint4 v) { return __builtin_bit_cast(bf16x8, v); }

// Transposed fragment of an M/N-contiguous image: lane l gets column c0 + (l&31), k rows
// 16*ks + 8*(l>>5) + 0..7 (the MFMA operand map), in two ds_read_b64_tr_b16.
__device__ __forceinline__ bf16x8 mc_frag(const char *img, int c0, int ks, int lane) {
  const int g = lane >> 4, i16 = lane & 15, q = i16 >> 2, pp = i16 & 3;
  const int cb = c0 + 16 * (g & 1);
  const int kb = 16 * ks + 8 * (g >> 1);
  const int ch = (cb >> 3) + (pp >> 1);
  const int o0 = mc_off(kb + q, ch) + 8 * (pp & 1);
  const int o1 = mc_off(kb + 4 + q, ch) + 8 * (pp & 1);
  const uint32_t base = (uint32_t)(uintptr_t)img;
  bf16x4 t0 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4 *)(uintptr_t)(base + o0));
  bf16x4 t1 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4 *)(uintptr_t)(base + o1));
  return __builtin_shufflevector(t0, t1, 0, 1, 2, 3, 4, 5, 6, 7);
}

// K-contiguous fragment: lane l gets row r0 + (l&31), k 16*ks + 8*(l>>5) + 0..7.
__device__ __forceinline__ bf16x8 kc_frag(const char *img, int r0, int ks, int lane) {
  return as_bf16x8(*reinterpret_cast<const uint4 *>(img + kc_off(r0 + (lane & 31), 2 * ks + (lane >> 5))));
}

// BN_ = 128 (4 waves, 2x2) or 256 (8 waves, 2x4; K-contiguous products only): the wider tile
// halves the refetch of the gathered fp32 A operand, which bounds this kernel.
// ABF (forward only): the activation operand is a bf16 NHWC copy `ab` (bf16 activation storage,
// the fp32 x may not exist): each slot loads its 8 bf16 as one 16-B load, no conversion.
template <int MODE, bool S2, int BN_ = 128, bool ABF = false>
__global__ void __launch_bounds__(bf16_threads(MODE), 2) igemm_bf16_kernel(const ConvParams p, const __bf16 *__restrict__ wb,
                                                                            const __bf16 *__restrict__ ab = nullptr) {
  static_assert(!ABF || MODE == MODE_FWD, "bf16 activation copies: forward products");
  constexpr bool MC = MODE == MODE_WGRAD;      // both operands M/N-contiguous
  constexpr int BM = 128, BN = BN_, BK = kB16BK, NT = bf16_threads(MODE);
  constexpr int WAVES_M = 2, WAVES_N = NT / 128;  // 2x2 (WGRAD) or 2x4 waves
  constexpr int WTM = BM / WAVES_M, WTN = BN / WAVES_N;
  constexpr int TM = WTM / 32, TN = WTN / 32;
  static_assert(!MC || BN_ == 128, "weight-gradient images are 128 wide");
  constexpr int IMGA = BM * BK * 2, IMGB = BN * BK * 2;  // bytes per operand image (bf16)
  constexpr int STAGE = IMGA + IMGB;
  constexpr int NQ = MC ? BM * BK / 4 / NT : BM * BK / 8 / NT;  // A slots per thread: 8 / 4 (2 at BN 256)
  constexpr int NQB = MC ? NQ : BN * BK / 8 / NT;                // B slots per thread
  static_assert(NQ * NT * (MC ? 4 : 8) == BM * BK && NQB * NT * (MC ? 4 : 8) == BN * BK, "slots cover the tile");

  __shared__ __attribute__((aligned(16))) char lds[2 * STAGE];

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
  // K-contiguous slot q: row q>>3, chunk q&7 (8 k).  M/N-contiguous slot q: k-row q>>5,
  // columns 4*(q&31) .. +3.
  int a_pix[NQ], a_y[NQ], a_x[NQ];
  bool a_ok[NQ];
  int b_off[NQB], b_dy[NQB], b_dx[NQB];
  bool b_ok[NQB];
  if constexpr (!MC) {
#pragma unroll
    for (int i = 0; i < NQB; ++i) {
      const int q = tid + NT * i;
      const int row = q >> 3, ch = q & 7;
      const int n = bn + row;
      b_ok[i] = n < p.N;
      b_off[i] = min(n, p.N - 1) * ktot + 8 * ch;
    }
  }
#pragma unroll
  for (int i = 0; i < NQ; ++i) {
    const int q = tid + NT * i;
    if constexpr (!MC) {
      const int row = q >> 3, ch = q & 7;
      const int m = bm + row;
      a_ok[i] = m < M;
      const int mm = min(m, M - 1);
      if constexpr (S2) {
        const int j = mm % Wc, t2 = mm / Wc;
        const int ii = t2 % Hc, b = t2 / Hc;
        a_y[i] = ii;
        a_x[i] = j;
        a_pix[i] = ((b * p.oh + ii) * p.ow + j) * p.k + 8 * ch;
      } else if constexpr (MODE == MODE_FWD) {
        uint32_t t = fdiv((uint32_t)mm, p.fd_ow);
        const int ow = mm - (int)t * p.ow;
        uint32_t b = fdiv(t, p.fd_oh);
        const int oh = (int)t - (int)b * p.oh;
        a_y[i] = oh * p.stride;
        a_x[i] = ow * p.stride;
        a_pix[i] = ABF ? (((int)b * p.h + a_y[i]) * p.w + a_x[i]) * p.c + 8 * ch   // contiguous NHWC copy
                       : (int)b * p.sxn + a_y[i] * p.sxh + a_x[i] * p.sxw + 8 * ch;
      } else {
        uint32_t t = fdiv((uint32_t)mm, p.fd_w);
        const int iw = mm - (int)t * p.w;
        uint32_t b = fdiv(t, p.fd_hw);
        const int ih = (int)t - (int)b * p.h;
        a_y[i] = ih;
        a_x[i] = iw;
        a_pix[i] = (((int)b * p.oh + ih) * p.ow + iw) * p.k + 8 * ch;
      }
    } else {
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

  // Register staging sets.  With two, the loads for tile kt+2 are issued while tile kt+1
  // (already in the other set) waits to be written to LDS: two K steps of latency budget.
  // Measured: two sets made fwd / data-grad 5-8 % SLOWER (register pressure at occupancy 2),
  // and the weight-gradient build would spill — so one set; the two-set schedule stays below
  // for A/B (flip the constant).
  constexpr int NSETS = 1;
  float4 ra[NSETS][MC ? NQ : 2 * NQ];
  float4 rbf[NSETS][MC ? NQ : 1];
  uint4 rbh[NSETS][MC ? 1 : NQB];
  bool ma[NSETS][NQ], mb[NSETS][NQB];

  auto load_tile = [&](int kt, auto set_) {
    constexpr int S = decltype(set_)::value;
    const int kbase = kt * BK;
    if constexpr (MODE == MODE_FWD) {
      const int tap = uni((int)fdiv((uint32_t)kbase, p.fd_c));
      int seg, t, dy, dx;
      seg_geom(p, sr, tap, seg, t, dy, dx);
      dy = uni(dy);
      dx = uni(dx);
      const int soff = ABF ? uni((dy * p.w + dx) * p.c + kbase - tap * p.c)
                           : uni(dy * p.sxh + dx * p.sxw + kbase - tap * p.c);
#pragma unroll
      for (int i = 0; i < NQ; ++i) {
        const bool v = a_ok[i] & ((unsigned)(a_y[i] + dy) < (unsigned)p.h) & ((unsigned)(a_x[i] + dx) < (unsigned)p.w);
        ma[S][i] = v;
        if constexpr (ABF) {   // 8 bf16 in the two float4 registers' bits (no conversion at the store)
          const uint4 q = *reinterpret_cast<const uint4 *>(ab + (v ? a_pix[i] + soff : 0));
          ra[S][2 * i] = make_float4(__uint_as_float(q.x), __uint_as_float(q.y), __uint_as_float(q.z),
                                     __uint_as_float(q.w));
        } else {
          const float *src = p.x + (v ? a_pix[i] + soff : 0);
          ra[S][2 * i] = ld4(src);
          ra[S][2 * i + 1] = ld4(src + 4);
        }
      }
#pragma unroll
      for (int i = 0; i < NQB; ++i) {
        mb[S][i] = b_ok[i];
        rbh[S][i] = *reinterpret_cast<const uint4 *>(wb + b_off[i] + kbase);
      }
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
        const bool v = a_ok[i] & ((unsigned)(a_y[i] - dy) < (unsigned)p.oh) & ((unsigned)(a_x[i] - dx) < (unsigned)p.ow);
        ma[S][i] = v;
        const float *src = p.dy + (v ? a_pix[i] + soff : 0);
        ra[S][2 * i] = ld4(src);
        ra[S][2 * i + 1] = ld4(src + 4);
      }
#pragma unroll
      for (int i = 0; i < NQB; ++i) {
        mb[S][i] = b_ok[i];
        rbh[S][i] = *reinterpret_cast<const uint4 *>(wb + b_off[i] + wk);
      }
    } else {  // WGRAD: k = output pixel
      const int krow0 = tid >> 5;
#pragma unroll
      for (int i = 0; i < NQ; ++i) {
        const int m = kbase + krow0 + (NT / 32) * i;
        const bool rv = m < K;
        ma[S][i] = rv && a_ok[i];
        ra[S][i] = ld4(p.dy + (size_t)(rv ? m : 0) * p.k + a_pix[i]);
        const int mm = min(m, K - 1);
        uint32_t t = fdiv((uint32_t)mm, p.fd_ow);
        const int ow = mm - (int)t * p.ow;
        uint32_t b = fdiv(t, p.fd_oh);
        const int oh = (int)t - (int)b * p.oh;
        const int iy = oh * p.stride + b_dy[i], ix = ow * p.stride + b_dx[i];
        const bool v = b_ok[i] && rv && (unsigned)iy < (unsigned)p.h && (unsigned)ix < (unsigned)p.w;
        mb[S][i] = v;
        rbf[S][i] = ld4(p.x + (v ? (int)b * p.sxn + iy * p.sxh + ix * p.sxw + b_off[i] : 0));
      }
    }
  };

  auto store_tile = [&](int buf, auto set_) {
    constexpr int S = decltype(set_)::value;
    char *As = lds + buf * STAGE;
    char *Bs = As + IMGA;
    if constexpr (!MC) {
#pragma unroll
      for (int i = 0; i < NQB; ++i) {
        const int q = tid + NT * i;
        *reinterpret_cast<uint4 *>(Bs + kc_off(q >> 3, q & 7)) = mb[S][i] ? rbh[S][i] : make_uint4(0, 0, 0, 0);
      }
    }
#pragma unroll
    for (int i = 0; i < NQ; ++i) {
      const int q = tid + NT * i;
      if constexpr (!MC) {
        const int row = q >> 3, ch = q & 7;
        uint4 av;
        if constexpr (ABF) {
          const float4 r = ra[S][2 * i];
          av = make_uint4(__float_as_uint(r.x), __float_as_uint(r.y), __float_as_uint(r.z), __float_as_uint(r.w));
        } else {
          const uint2 lo = cvt4_bf16(ra[S][2 * i]), hi = cvt4_bf16(ra[S][2 * i + 1]);
          av = make_uint4(lo.x, lo.y, hi.x, hi.y);
        }
        av = ma[S][i] ? av : make_uint4(0, 0, 0, 0);
        *reinterpret_cast<uint4 *>(As + kc_off(row, ch)) = av;
      } else {
        const int kr = q >> 5, col = 4 * (q & 31);
        const int o = mc_off(kr, col >> 3) + 8 * ((col >> 2) & 1);
        const uint2 av = cvt4_bf16(ra[S][i]), bv = cvt4_bf16(rbf[S][i]);
        *reinterpret_cast<uint2 *>(As + o) = ma[S][i] ? av : make_uint2(0, 0);
        *reinterpret_cast<uint2 *>(Bs + o) = mb[S][i] ? bv : make_uint2(0, 0);
      }
    }
  };

  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WAVES_N, wn = wave - wm * WAVES_N;

  floatx16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, NSETS - 1>;
  int cur = 0;
  // MFMAs of one K step from LDS buffer `cur`
  auto compute = [&](auto with_store) {
    const char *As = lds + cur * STAGE;
    const char *Bs = As + IMGA;
    bf16x8 a[2][TM], b[2][TN];
    auto read_frags = [&](int ks, int slot) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
        a[slot][i] = MC ? mc_frag(As, wm * WTM + i * 32, ks, lane) : kc_frag(As, wm * WTM + i * 32, ks, lane);
#pragma unroll
      for (int j = 0; j < TN; ++j)
        b[slot][j] = MC ? mc_frag(Bs, wn * WTN + j * 32, ks, lane) : kc_frag(Bs, wn * WTN + j * 32, ks, lane);
    };
    read_frags(0, 0);
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
      const int cb = ks & 1;
      if (ks + 1 < BK / 16) read_frags(ks + 1, cb ^ 1);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[cb][i], b[cb][j], acc[i][j], 0, 0, 0);
    }
    if constexpr (decltype(with_store)::value) {
      // the next K step's registers converted and stored into the other LDS buffer in the
      // MFMAs' shadow (same basic block: the scheduler interleaves them)
      store_tile(cur ^ 1, I0{});
#pragma unroll
      for (int q = 0; q < (BK / 16) * TM * TN; ++q) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // 1 MFMA
        __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);   // 4 VALU
        __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);   // 1 LDS store
      }
    }
  };
  if (kt0 < kt1) {
    load_tile(kt0, I0{});
    store_tile(0, I0{});
    if constexpr (NSETS == 2) {
      if (kt0 + 1 < kt1) load_tile(kt0 + 1, I1{});
      __syncthreads();
      // one K step; `held` = the register set holding tile kt+1
      auto kstep = [&](int kt, auto held) {
        constexpr int H = decltype(held)::value;
        using Free = std::integral_constant<int, 1 - H>;
        if (kt + 2 < kt1) load_tile(kt + 2, Free{});
        compute(std::false_type{});
        if (kt + 1 < kt1) store_tile(cur ^ 1, held);
        __syncthreads();
        cur ^= 1;
      };
      for (int kt = kt0; kt < kt1; kt += 2) {
        kstep(kt, I1{});
        if (kt + 1 < kt1) kstep(kt + 1, I0{});
      }
    } else if constexpr (!MC) {
      // K-contiguous products (8 waves): T14 order with unconditional staging — registers hold
      // step kt+1 while step kt computes and stores them; past the last step the loads re-read
      // step kt1-1 into the LDS buffer nobody reads again
      const int klast = kt1 - 1;
      load_tile(min(kt0 + 1, klast), I0{});
      __syncthreads();
      for (int kt = kt0; kt < kt1; ++kt) {
        compute(std::true_type{});
        load_tile(min(kt + 2, klast), I0{});
        __syncthreads();
        cur ^= 1;
      }
    } else {
      __syncthreads();
      for (int kt = kt0; kt < kt1; ++kt) {
        const bool more = kt + 1 < kt1;
        if (more) load_tile(kt + 1, I0{});
        compute(std::false_type{});
        if (more) store_tile(cur ^ 1, I0{});
        __syncthreads();
        cur ^= 1;
      }
    }
  }

  igemm_epilogue<MODE, BM, BN, WAVES_M, WAVES_N, S2>(p, acc, bm, bn, tm, tn, split, M, Hc, Wc, py, px,
                                                      reinterpret_cast<float *>(lds));
}

}  // namespace adaptseg
