// Kernel instantiations and host launcher of the F32X3 conv math (conv_x3.hpp, conv_x3r.hpp):
// fp32 convs on the bf16 MFMA through exact three-term bf16 splits.
#include "conv_x3r.hpp"

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

// elements of the x3r kernel's activation operand (FWD: x, DGRAD / WGRAD: dY) and, for the
// weight gradient, of x: their term images (made per call when the caller supplies none) are
// three times that many bf16
size_t x3g_act_elems(const Plan &pl) {
  const ConvParams &p = pl.p;
  if (!pl.x3g) return 0;   // (x3ext: the caller's images have this size too, see launch_x3)
  return pl.mode == MODE_FWD ? (size_t)p.n * p.h * p.w * p.c : (size_t)p.n * p.oh * p.ow * p.k;
}
size_t x3g_act2_elems(const Plan &pl) {
  const ConvParams &p = pl.p;
  return pl.x3g && pl.mode == MODE_WGRAD ? (size_t)p.n * p.h * p.w * p.c : 0;
}
static size_t al256(size_t b) { return (b + 255) / 256 * 256; }

// workspace ahead of the split-K slabs: [weight pack][three term images of the activation
// operand (+ of x for the weight gradient) when the caller supplied none]
size_t x3_pre_bytes(const Plan &pl) {
  if (pl.x3ext && pl.x3r) return al256(x3_wpack_bytes(pl));   // the caller's term images
  return al256(x3_wpack_bytes(pl)) + al256(3 * x3g_act_elems(pl) * sizeof(__bf16)) +
         al256(3 * x3g_act2_elems(pl) * sizeof(__bf16));
}

static void split_copy(const float *x, int n, int h, int w, int c, int sxn, int sxh, int sxw, void *out,
                       hipStream_t s) {
  const int64_t n8 = (int64_t)n * h * w * c / 8;
  x3_split_copy_kernel<<<(unsigned)std::min<int64_t>(ceil_div(n8, 256), 8192), 256, 0, s>>>(
      x, n, h, w, c / 8, sxn, sxh, sxw, reinterpret_cast<uint4 *>(out));
}

hipError_t prep_x3_wpack(const Plan &pl, void *pack, hipStream_t s) {
  const ConvParams &p = pl.p;
  int rows_pad, ktot;
  x3_pack_dims(pl, rows_pad, ktot);
  // one thread per (row, 8-k chunk), 16-B stores (conv_wpack_x3v_kernel)
  const dim3 pg((unsigned)(rows_pad / x3_bn(pl.mode)), (unsigned)(ktot / kX3BK));
  if (pl.mode == MODE_FWD) conv_wpack_x3v_kernel<MODE_FWD><<<pg, 256, 0, s>>>(p, (char *)pack, ktot);
  else if (pl.mode == MODE_DGRAD) conv_wpack_x3v_kernel<MODE_DGRAD><<<pg, 256, 0, s>>>(p, (char *)pack, ktot);
  return hipGetLastError();
}

hipError_t prep_x3(const Plan &pl, void *wpack, hipStream_t s) {
  const ConvParams &p = pl.p;
  if (!pl.wpack_ext) {
    const hipError_t e = prep_x3_wpack(pl, wpack, s);
    if (e != hipSuccess) return e;
  }
  if (pl.x3g) {   // the operands' term images the caller did not supply
    char *base = reinterpret_cast<char *>(wpack) + al256(x3_wpack_bytes(pl));
    if (!pl.act_ext) {
      if (pl.mode == MODE_FWD) split_copy(p.x, p.n, p.h, p.w, p.c, p.sxn, p.sxh, p.sxw, base, s);
      else split_copy(p.dy, p.n, p.oh, p.ow, p.k, p.oh * p.ow * p.k, p.ow * p.k, p.k, base, s);
    }
    if (pl.mode == MODE_WGRAD && !pl.act_ext2)
      split_copy(p.x, p.n, p.h, p.w, p.c, p.sxn, p.sxh, p.sxw, base + al256(3 * x3g_act_elems(pl) * sizeof(__bf16)),
                 s);
  }
  return hipGetLastError();
}

hipError_t launch_x3(const Plan &pl, void *wpack, hipStream_t s) {
  const ConvParams &p = pl.p;
  const __bf16 *wb = reinterpret_cast<const __bf16 *>(pl.wpack_ext ? pl.wpack_ext : wpack);
  dim3 grid(pl.tiles, p.splits, pl.s2 ? 4 : 1), block(x3_threads(pl.mode));
  if (pl.x3r) {
    const char *base = reinterpret_cast<const char *>(wpack) + al256(x3_wpack_bytes(pl));
    const __bf16 *act = pl.act_ext ? reinterpret_cast<const __bf16 *>(pl.act_ext) : reinterpret_cast<const __bf16 *>(base);
    if (pl.mode == MODE_FWD) launch_k(igemm_x3r_kernel<MODE_FWD, false>, grid, 512, s, p, act, wb);
    else if (pl.mode == MODE_DGRAD && pl.s2) launch_k(igemm_x3r_kernel<MODE_DGRAD, true>, grid, 512, s, p, act, wb);
    else if (pl.mode == MODE_DGRAD) launch_k(igemm_x3r_kernel<MODE_DGRAD, false>, grid, 512, s, p, act, wb);
    else {
      const __bf16 *act2 = pl.act_ext2 ? reinterpret_cast<const __bf16 *>(pl.act_ext2)
                                       : reinterpret_cast<const __bf16 *>(base + al256(3 * x3g_act_elems(pl) * sizeof(__bf16)));
      if (pl.x3r_bm == 256) launch_k(igemm_x3r_wgrad_kernel<256>, grid, 512, s, p, act, act2);
      else launch_k(igemm_x3r_wgrad_kernel<128>, grid, 512, s, p, act, act2);
    }
    return hipGetLastError();
  }
  if (pl.x3h) {
    // (the 256-row weight-gradient tile needs two register sets of six float4 beside its 128
    // accumulators: it spills, so the weight gradient runs the 128-row tile)
    if (pl.mode == MODE_WGRAD) launch_k(igemm_x3hw_kernel<128>, grid, 512, s, p);
    else if (pl.mode == MODE_FWD && p.abn_m) launch_k(igemm_x3h_abn_kernel, grid, 512, s, p, wb);
    else if (pl.mode == MODE_FWD) launch_k(igemm_x3h_kernel<MODE_FWD, false>, grid, 512, s, p, wb);
    else if (pl.s2) launch_k(igemm_x3h_kernel<MODE_DGRAD, true>, grid, 512, s, p, wb);
    else launch_k(igemm_x3h_kernel<MODE_DGRAD, false>, grid, 512, s, p, wb);
    return hipGetLastError();
  }
  if (pl.mode == MODE_FWD) launch_k(igemm_x3_kernel<MODE_FWD, false>, grid, block, s, p, wb);
  else if (pl.mode == MODE_DGRAD && pl.s2) launch_k(igemm_x3_kernel<MODE_DGRAD, true>, grid, block, s, p, wb);
  else if (pl.mode == MODE_DGRAD) launch_k(igemm_x3_kernel<MODE_DGRAD, false>, grid, block, s, p, wb);
  else if (p.abn_m) launch_k(igemm_x3_abn_kernel, grid, block, s, p, wb);
  else launch_k(igemm_x3_kernel<MODE_WGRAD, false>, grid, block, s, p, wb);
  return hipGetLastError();
}

}  // namespace adaptseg
