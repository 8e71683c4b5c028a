// Kernel instantiations and host launchers of the bf16-MFMA conv path (conv_bf16.hpp).
#include "conv_bf16.hpp"

namespace adaptseg {

size_t bf16_wpack_bytes(const Plan &pl) {
  const ConvParams &p = pl.p;
  if (pl.mode == MODE_FWD) return (size_t)p.k * p.nseg * p.kseg * sizeof(__bf16);
  if (pl.mode == MODE_DGRAD) return (size_t)p.c * p.ntaps * p.k * sizeof(__bf16);
  return 0;
}

hipError_t launch_bf16(const Plan &pl, void *wpack, hipStream_t s) {
  const ConvParams &p = pl.p;
  __bf16 *wb = reinterpret_cast<__bf16 *>(wpack);
  if (pl.mode == MODE_FWD) {
    const int64_t n = (int64_t)p.k * p.nseg * p.kseg;
    conv_wpack_fwd_kernel<<<(unsigned)std::min<int64_t>(ceil_div(n, 256), 4096), 256, 0, s>>>(p, wb);
  } else if (pl.mode == MODE_DGRAD) {
    dim3 g((unsigned)ceil_div(p.c, 64), (unsigned)ceil_div(p.k, 64), (unsigned)p.ntaps);
    conv_wpack_dgrad_kernel<<<g, 256, 0, s>>>(p, wb);
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const bool w256 = pl.bf16_bn == 256 && pl.mode != MODE_WGRAD;
  dim3 grid(pl.tiles, p.splits, pl.s2 ? 4 : 1), block(w256 ? 512 : 256);
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
