// Kernel instantiations and host launchers of the bf16-MFMA conv path (conv_bf16.hpp).
#include "conv_bf16.hpp"

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


size_t bf16_wpack_bytes(const Plan &pl) {
  const ConvParams &p = pl.p;
  if (pl.mode == MODE_FWD) return (size_t)p.k * p.nseg * p.kseg * sizeof(__bf16);
  if (pl.mode == MODE_DGRAD) return (size_t)p.c * p.ntaps * p.k * sizeof(__bf16);
  return 0;
}

// Weight pack (untimed: the bench's roofline times the GEMM alone)
hipError_t prep_bf16(Plan &pl, void *wpack, hipStream_t s) {
  const ConvParams &p = pl.p;
  __bf16 *wb = reinterpret_cast<__bf16 *>(wpack);
  if (pl.mode == MODE_FWD) {
    const int64_t n = (int64_t)p.k * p.nseg * p.kseg;
    conv_wpack_fwd_kernel<<<(unsigned)std::min<int64_t>(ceil_div(n, 256), 4096), 256, 0, s>>>(p, wb);
  } else if (pl.mode == MODE_DGRAD) {
    dim3 g((unsigned)ceil_div(p.c, 64), (unsigned)ceil_div(p.k, 64), (unsigned)p.ntaps);
    conv_wpack_dgrad_kernel<<<g, 256, 0, s>>>(p, wb);
  }
  return hipGetLastError();
}

hipError_t launch_bf16(const Plan &pl, void *wpack, hipStream_t s) {
  const ConvParams &p = pl.p;
  const __bf16 *wb = reinterpret_cast<const __bf16 *>(wpack);
  const bool w256 = pl.bf16_bn == 256 && pl.mode != MODE_WGRAD;
  dim3 grid(pl.tiles, p.splits, pl.s2 ? 4 : 1), block(bf16_threads(pl.mode));
  if (pl.mode == MODE_FWD) {
    if (w256) igemm_bf16_kernel<MODE_FWD, false, 256><<<grid, block, 0, s>>>(p, wb);
    else igemm_bf16_kernel<MODE_FWD, false, 128><<<grid, block, 0, s>>>(p, wb);
  } else if (pl.mode == MODE_DGRAD && pl.s2) {
    if (w256) igemm_bf16_kernel<MODE_DGRAD, true, 256><<<grid, block, 0, s>>>(p, wb);
    else igemm_bf16_kernel<MODE_DGRAD, true, 128><<<grid, block, 0, s>>>(p, wb);
  } else if (pl.mode == MODE_DGRAD) {
    if (w256) igemm_bf16_kernel<MODE_DGRAD, false, 256><<<grid, block, 0, s>>>(p, wb);
    else igemm_bf16_kernel<MODE_DGRAD, false, 128><<<grid, block, 0, s>>>(p, wb);
  } else {
    igemm_bf16_kernel<MODE_WGRAD, false, 128><<<grid, block, 0, s>>>(p, wb);
  }
  return hipGetLastError();
}

}  // namespace adaptseg
