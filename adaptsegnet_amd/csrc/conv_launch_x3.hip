// Kernel instantiations and host launcher of the F32X3 conv math (conv_x3.hpp): fp32 convs on
// the bf16 MFMA through exact three-term bf16 splits.
#include "conv_x3.hpp"

namespace adaptseg {

// packed B operand: rows padded to whole column tiles (x3_bn), three bf16 terms per weight
static void x3_pack_dims(const Plan &pl, int &rows_pad, int &ktot) {
  const ConvParams &p = pl.p;
  rows_pad = ktot = 0;
  if (pl.mode == MODE_FWD) {
    rows_pad = (int)ceil_div(p.k, x3_bn(MODE_FWD)) * x3_bn(MODE_FWD);
    ktot = p.nseg * p.kseg;
  } else if (pl.mode == MODE_DGRAD) {
    rows_pad = (int)ceil_div(p.c, x3_bn(MODE_DGRAD)) * x3_bn(MODE_DGRAD);
    ktot = p.ntaps * p.k;
  }
}

size_t x3_wpack_bytes(const Plan &pl) {
  int rows_pad, ktot;
  x3_pack_dims(pl, rows_pad, ktot);
  return 3 * (size_t)rows_pad * ktot * sizeof(__bf16);
}

hipError_t prep_x3(const Plan &pl, void *wpack, hipStream_t s) {
  const ConvParams &p = pl.p;
  int rows_pad, ktot;
  x3_pack_dims(pl, rows_pad, ktot);
  // one thread per (row, 8-k chunk), 16-B stores (conv_wpack_x3v_kernel)
  const dim3 pg((unsigned)(rows_pad / x3_bn(pl.mode)), (unsigned)(ktot / kX3BK));
  if (pl.mode == MODE_FWD) conv_wpack_x3v_kernel<MODE_FWD><<<pg, 256, 0, s>>>(p, (char *)wpack, ktot);
  else if (pl.mode == MODE_DGRAD) conv_wpack_x3v_kernel<MODE_DGRAD><<<pg, 256, 0, s>>>(p, (char *)wpack, ktot);
  return hipGetLastError();
}

hipError_t launch_x3(const Plan &pl, void *wpack, hipStream_t s) {
  const ConvParams &p = pl.p;
  __bf16 *wb = reinterpret_cast<__bf16 *>(wpack);
  dim3 grid(pl.tiles, p.splits, pl.s2 ? 4 : 1), block(x3_threads(pl.mode));
  if (pl.mode == MODE_FWD) igemm_x3_kernel<MODE_FWD, false><<<grid, block, 0, s>>>(p, wb);
  else if (pl.mode == MODE_DGRAD && pl.s2) igemm_x3_kernel<MODE_DGRAD, true><<<grid, block, 0, s>>>(p, wb);
  else if (pl.mode == MODE_DGRAD) igemm_x3_kernel<MODE_DGRAD, false><<<grid, block, 0, s>>>(p, wb);
  else igemm_x3_kernel<MODE_WGRAD, false><<<grid, block, 0, s>>>(p, wb);
  return hipGetLastError();
}

}  // namespace adaptseg
