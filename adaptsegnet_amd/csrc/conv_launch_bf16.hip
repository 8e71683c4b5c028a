// Kernel instantiations and host launchers of the bf16-MFMA conv path (conv_bf16.hpp).
#include "conv_bf16.hpp"
#include "conv_bf16g.hpp"

namespace adaptseg {

// bf16 weight packing (once per conv call; weights are small next to the activations).
// FWD: out[co][seg*kseg + tk] = W_seg[co][tk], tk = tap*Cin + ci  (K-contiguous rows).
__global__ void conv_wpack_fwd_kernel(const ConvParams p, __bf16 *out) {
  const int ktot = p.nseg * p.kseg;
  const int64_t n = (int64_t)p.k * ktot;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int co = (int)(i / ktot), kk = (int)(i - (int64_t)co * ktot);
    const int seg = kk / p.kseg, tk = kk - seg * p.kseg;
    out[i] = (__bf16)seg_ptr(p, seg)[(size_t)co * p.kseg + tk];
  }
}

// DGRAD: out[ci][tap*Cout + co] = W_seg(tap)[co][t][ci]  (tap over all segments): a 64x64
// (co, ci) tile per block transposed through LDS, so both the read (along ci) and the write
// (along co) are coalesced.  grid = (ceil(C/64), ceil(Cout/64), ntaps), 256 threads.
__global__ void __launch_bounds__(256) conv_wpack_dgrad_kernel(const ConvParams p, __bf16 *out) {
  __shared__ float tile[64][65];
  const int ci0 = blockIdx.x * 64, co0 = blockIdx.y * 64, tap = blockIdx.z;
  const int seg = tap / p.taps_per_seg, t = tap - seg * p.taps_per_seg;
  const float *w = seg_ptr(p, seg);
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int r = ty; r < 64; r += 4) {
    const int co = co0 + r, ci = ci0 + tx;
    tile[r][tx] = (co < p.k && ci < p.c) ? w[((size_t)co * p.taps_per_seg + t) * p.c + ci] : 0.f;
  }
  __syncthreads();
  const size_t ktot = (size_t)p.ntaps * p.k;
  for (int r = ty; r < 64; r += 4) {
    const int ci = ci0 + r, co = co0 + tx;
    if (ci < p.c && co < p.k) out[(size_t)ci * ktot + (size_t)tap * p.k + co] = (__bf16)tile[tx][r];
  }
}

// Vector forms (the step's convs: kseg % 8 == 0 / Cin % 4 == 0 and Cout % 8 == 0, 16-B aligned
// weights): every load a float4 and every store a 16-B chunk of eight bf16, 32-bit indexing.
// FWD: one thread per 8-k chunk of a row, consecutive threads on consecutive chunks.
__global__ void __launch_bounds__(256) conv_wpack_fwd_v_kernel(const ConvParams p, uint4 *__restrict__ out,
                                                               uint32_t cpr, uint32_t total) {
  for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < total; i += gridDim.x * 256u) {
    const uint32_t co = i / cpr, k0 = (i - co * cpr) * 8;
    int seg = 0;
    uint32_t tk = k0;
    while (tk >= (uint32_t)p.kseg) { tk -= p.kseg; ++seg; }
    const float *src = seg_ptr(p, seg) + (size_t)co * p.kseg + tk;
    const uint2 lo = cvt4_bf16(ld4(src)), hi = cvt4_bf16(ld4(src + 4));
    out[i] = make_uint4(lo.x, lo.y, hi.x, hi.y);
  }
}

// DGRAD: the 64 (co) x 64 (ci) tile of one tap read as float4 along ci, written as 16-B chunks
// along co.  grid = (ceil(C/64), ceil(Cout/64), ntaps), 256 threads.
__global__ void __launch_bounds__(256) conv_wpack_dgrad_v_kernel(const ConvParams p, __bf16 *out) {
  __shared__ float tile[64][65];
  const int ci0 = blockIdx.x * 64, co0 = blockIdx.y * 64, tap = blockIdx.z;
  const int seg = tap / p.taps_per_seg, t = tap - seg * p.taps_per_seg;
  const float *w = seg_ptr(p, seg);
  const int f = threadIdx.x & 15, r0 = threadIdx.x >> 4;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int r = r0 + 16 * j, co = co0 + r, ci = ci0 + 4 * f;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (co < p.k && ci < p.c) v = ld4(w + ((size_t)co * p.taps_per_seg + t) * p.c + ci);
    tile[r][4 * f] = v.x; tile[r][4 * f + 1] = v.y; tile[r][4 * f + 2] = v.z; tile[r][4 * f + 3] = v.w;
  }
  __syncthreads();
  const size_t ktot = (size_t)p.ntaps * p.k;
  const int c = threadIdx.x & 7, co = co0 + 8 * c;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int rl = (threadIdx.x >> 3) + 32 * j, ci = ci0 + rl;
    if (ci >= p.c || co >= p.k) continue;
    const float *col = &tile[8 * c][rl];
    const uint2 lo = cvt4_bf16(make_float4(col[0], col[65], col[130], col[195]));
    const uint2 hi = cvt4_bf16(make_float4(col[260], col[325], col[390], col[455]));
    *reinterpret_cast<uint4 *>(out + (size_t)ci * ktot + (size_t)tap * p.k + co) = make_uint4(lo.x, lo.y, hi.x, hi.y);
  }
}

// fp32 NHWC activations (pixel strides sxn / sxh / sxw, unit channel stride) -> contiguous
// NHWC bf16 (RNE), 8 channels per thread: the activation operand of the LDS-DMA kernel.
__global__ void bf16_copy_kernel(const float *__restrict__ x, int n, int h, int w, int c8, int sxn, int sxh,
                                 int sxw, uint4 *__restrict__ out) {
  const int64_t total = (int64_t)n * h * w * c8;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int cq = (int)(i % c8);
    const int64_t pix = i / c8;
    const int xx = (int)(pix % w);
    const int64_t t = pix / w;
    const int yy = (int)(t % h), b = (int)(t / h);
    const float *src = x + (int64_t)b * sxn + (int64_t)yy * sxh + (int64_t)xx * sxw + 8 * cq;
    const uint2 lo = cvt4_bf16(ld4(src)), hi = cvt4_bf16(ld4(src + 4));
    out[i] = make_uint4(lo.x, lo.y, hi.x, hi.y);
  }
}

// elements of the LDS-DMA kernel's bf16 activation copy (FWD: x, DGRAD: dY)
// (weight gradient: dY's copy, then x's)
static size_t g16_act_elems(const Plan &pl) {
  const ConvParams &p = pl.p;
  if (!pl.g16) return 0;
  return pl.mode == MODE_FWD ? (size_t)p.n * p.h * p.w * p.c : (size_t)p.n * p.oh * p.ow * p.k;
}
static size_t g16_act2_elems(const Plan &pl) {
  const ConvParams &p = pl.p;
  return pl.g16 && pl.mode == MODE_WGRAD ? (size_t)p.n * p.h * p.w * p.c : 0;
}
static size_t al256(size_t b) { return (b + 255) / 256 * 256; }

size_t bf16_pre_bytes(const Plan &pl) {
  return al256(bf16_wpack_bytes(pl)) + al256(g16_act_elems(pl) * sizeof(__bf16)) +
         al256(g16_act2_elems(pl) * sizeof(__bf16));
}

size_t bf16_wpack_bytes(const Plan &pl) {
  const ConvParams &p = pl.p;
  if (pl.mode == MODE_FWD) return (size_t)p.k * p.nseg * p.kseg * sizeof(__bf16);
  if (pl.mode == MODE_DGRAD) return (size_t)p.c * p.ntaps * p.k * sizeof(__bf16);
  return 0;
}

// Weight pack (untimed: the bench's roofline times the GEMM alone)
hipError_t prep_bf16_wpack(const Plan &pl, void *pack, hipStream_t s) {
  const ConvParams &p = pl.p;
  __bf16 *wb = reinterpret_cast<__bf16 *>(pack);
  bool wal = true;   // weights 16-B aligned (the vector forms' float4 loads)
  for (int g = 0; g < p.nseg; ++g) wal = wal && (reinterpret_cast<uintptr_t>(p.wt[g]) & 15) == 0;
  if (pl.mode == MODE_FWD) {
    const int64_t n = (int64_t)p.k * p.nseg * p.kseg;
    if (wal && p.kseg % 8 == 0 && n / 8 < (int64_t)1 << 31) {
      const uint32_t total = (uint32_t)(n / 8);
      conv_wpack_fwd_v_kernel<<<(unsigned)std::min<int64_t>(ceil_div(total, 256), 4096), 256, 0, s>>>(
          p, reinterpret_cast<uint4 *>(wb), (uint32_t)(p.nseg * p.kseg / 8), total);
    } else {
      conv_wpack_fwd_kernel<<<(unsigned)std::min<int64_t>(ceil_div(n, 256), 4096), 256, 0, s>>>(p, wb);
    }
  } else if (pl.mode == MODE_DGRAD) {
    dim3 g((unsigned)ceil_div(p.c, 64), (unsigned)ceil_div(p.k, 64), (unsigned)p.ntaps);
    if (wal && p.c % 4 == 0 && p.k % 8 == 0) conv_wpack_dgrad_v_kernel<<<g, 256, 0, s>>>(p, wb);
    else conv_wpack_dgrad_kernel<<<g, 256, 0, s>>>(p, wb);
  }
  return hipGetLastError();
}

hipError_t prep_bf16(Plan &pl, void *wpack, hipStream_t s) {
  const ConvParams &p = pl.p;
  if (!pl.wpack_ext) {
    const hipError_t e = prep_bf16_wpack(pl, wpack, s);
    if (e != hipSuccess) return e;
  }
  // the activation operands' bf16 copies the caller did not supply, after the (256-B aligned) weight pack
  if (pl.g16) {
    char *base = reinterpret_cast<char *>(wpack) + al256(bf16_wpack_bytes(pl));
    uint4 *act = reinterpret_cast<uint4 *>(base);
    const int64_t n8 = (int64_t)g16_act_elems(pl) / 8;
    const unsigned blocks = (unsigned)std::min<int64_t>(ceil_div(n8, 256), 8192);
    if (!pl.act_ext) {
      if (pl.mode == MODE_FWD)
        bf16_copy_kernel<<<blocks, 256, 0, s>>>(p.x, p.n, p.h, p.w, p.c / 8, p.sxn, p.sxh, p.sxw, act);
      else
        bf16_copy_kernel<<<blocks, 256, 0, s>>>(p.dy, p.n, p.oh, p.ow, p.k / 8, p.oh * p.ow * p.k, p.ow * p.k,
                                                p.k, act);
    }
    if (pl.mode == MODE_WGRAD && !pl.act_ext2) {
      uint4 *act2 = reinterpret_cast<uint4 *>(base + al256(g16_act_elems(pl) * sizeof(__bf16)));
      const int64_t m8 = (int64_t)g16_act2_elems(pl) / 8;
      bf16_copy_kernel<<<(unsigned)std::min<int64_t>(ceil_div(m8, 256), 8192), 256, 0, s>>>(
          p.x, p.n, p.h, p.w, p.c / 8, p.sxn, p.sxh, p.sxw, act2);
    }
  }
  return hipGetLastError();
}

hipError_t launch_bf16(const Plan &pl, void *wpack, hipStream_t s) {
  const ConvParams &p = pl.p;
  const __bf16 *wb = reinterpret_cast<const __bf16 *>(pl.wpack_ext ? pl.wpack_ext : wpack);
  if (pl.g16) {
    const char *base = reinterpret_cast<const char *>(wpack) + al256(bf16_wpack_bytes(pl));
    const __bf16 *act = pl.act_ext ? reinterpret_cast<const __bf16 *>(pl.act_ext)
                                   : reinterpret_cast<const __bf16 *>(base);
    dim3 grid(pl.tiles, p.splits, pl.s2 ? 4 : 1), block(512);
    if (pl.s2) {   // stride-2 data gradient: parity classes on grid.z, K step 32
      if (pl.g16_bn == 256) launch_k(igemm_bf16g_kernel<MODE_DGRAD, 128, 256, 32, true>, grid, block, s, p, act, wb);
      else launch_k(igemm_bf16g_kernel<MODE_DGRAD, 256, 128, 32, true>, grid, block, s, p, act, wb);
      return hipGetLastError();
    }
    if (pl.mode == MODE_WGRAD) {
      const __bf16 *act2 = pl.act_ext2 ? reinterpret_cast<const __bf16 *>(pl.act_ext2)
                                       : reinterpret_cast<const __bf16 *>(
                                             base + al256(g16_act_elems(pl) * sizeof(__bf16)));
      // (a 6-deep ring for the 256x128 tile, 4-deep for 128x128 — five / three steps in flight
      // instead of two: per shape within +-3 %, c5 -0.6 %, profiles/r5/g16_wgrad_ring_ab.txt)
      if (pl.g16_bn == 256) launch_k(igemm_bf16g_wgrad_kernel<256, 256, 2>, grid, dim3(1024), s, p, act, act2);
      else if (pl.g16_bm == 256) launch_k(igemm_bf16g_wgrad_kernel<256>, grid, block, s, p, act, act2);
      else launch_k(igemm_bf16g_wgrad_kernel<128>, grid, block, s, p, act, act2);
      return hipGetLastError();
    }
#define G16_LAUNCH(MODE_, BK_)                                                                  \
  do {                                                                                          \
    if (pl.g16_bm == 256 && pl.g16_bn == 256)                                                   \
      launch_k(igemm_bf16g_kernel<MODE_, 256, 256, 64, false, 2>, grid, dim3(1024), s, p, act, wb); \
    else if (pl.g16_bn == 256) launch_k(igemm_bf16g_kernel<MODE_, 128, 256, BK_>, grid, block, s, p, act, wb); \
    else launch_k(igemm_bf16g_kernel<MODE_, 256, 128, BK_>, grid, block, s, p, act, wb);          \
  } while (0)
    if (pl.mode == MODE_FWD) {
      if (pl.g16_bk == 64) G16_LAUNCH(MODE_FWD, 64);
      else G16_LAUNCH(MODE_FWD, 32);
    } else {
      if (pl.g16_bk == 64) G16_LAUNCH(MODE_DGRAD, 64);
      else G16_LAUNCH(MODE_DGRAD, 32);
    }
#undef G16_LAUNCH
    return hipGetLastError();
  }
  const bool w256 = pl.bf16_bn == 256 && pl.mode != MODE_WGRAD;
  dim3 grid(pl.tiles, p.splits, pl.s2 ? 4 : 1), block(bf16_threads(pl.mode));
  if (pl.mode == MODE_FWD && pl.act_ext) {   // the caller's bf16 activation copy (bf16 activation storage)
    const __bf16 *act = reinterpret_cast<const __bf16 *>(pl.act_ext);
    if (w256) launch_k(igemm_bf16_kernel<MODE_FWD, false, 256, true>, grid, block, s, p, wb, act);
    else launch_k(igemm_bf16_kernel<MODE_FWD, false, 128, true>, grid, block, s, p, wb, act);
  } else if (pl.mode == MODE_FWD) {
    if (w256) launch_k(igemm_bf16_kernel<MODE_FWD, false, 256>, grid, block, s, p, wb, (const __bf16 *)nullptr);
    else launch_k(igemm_bf16_kernel<MODE_FWD, false, 128>, grid, block, s, p, wb, (const __bf16 *)nullptr);
  } else if (pl.mode == MODE_DGRAD && pl.s2) {
    if (w256) launch_k(igemm_bf16_kernel<MODE_DGRAD, true, 256>, grid, block, s, p, wb, (const __bf16 *)nullptr);
    else launch_k(igemm_bf16_kernel<MODE_DGRAD, true, 128>, grid, block, s, p, wb, (const __bf16 *)nullptr);
  } else if (pl.mode == MODE_DGRAD) {
    if (w256) launch_k(igemm_bf16_kernel<MODE_DGRAD, false, 256>, grid, block, s, p, wb, (const __bf16 *)nullptr);
    else launch_k(igemm_bf16_kernel<MODE_DGRAD, false, 128>, grid, block, s, p, wb, (const __bf16 *)nullptr);
  } else {
    launch_k(igemm_bf16_kernel<MODE_WGRAD, false, 128>, grid, block, s, p, wb, (const __bf16 *)nullptr);
  }
  return hipGetLastError();
}

}  // namespace adaptseg
