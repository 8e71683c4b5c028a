#define LAUNCH_NAME launch_wgrad
#define LAUNCH_MODE MODE_WGRAD
// Kernel instantiations for one conv product (compiled as its own translation unit).
#include "conv_kernels.hpp"

namespace adaptseg {

#define AS_FAST(BM_, BN_, WM_, WN_, FBK_, S2_, AE_, BE_) \
  igemm_fast_kernel<MODE, BM_, BN_, WM_, WN_, FBK_, S2_, AE_, BE_><<<grid, block, 0, s>>>(pl.p)

#define AS_LAUNCH(BM_, BN_, WM_, WN_, FBK_)                                                  \
  do {                                                                                       \
    if (pl.fast) {                                                                           \
      const int v = (pl.s2 ? 4 : 0) | (pl.ae ? 2 : 0) | (pl.be ? 1 : 0);                     \
      switch (v) {                                                                           \
        case 0: AS_FAST(BM_, BN_, WM_, WN_, FBK_, false, false, false); break;              \
        case 1: AS_FAST(BM_, BN_, WM_, WN_, FBK_, false, false, true); break;               \
        case 2: AS_FAST(BM_, BN_, WM_, WN_, FBK_, false, true, false); break;               \
        case 3: AS_FAST(BM_, BN_, WM_, WN_, FBK_, false, true, true); break;                \
        case 4: if constexpr (MODE == MODE_DGRAD) AS_FAST(BM_, BN_, WM_, WN_, FBK_, true, false, false); break; \
        case 5: if constexpr (MODE == MODE_DGRAD) AS_FAST(BM_, BN_, WM_, WN_, FBK_, true, false, true); break;  \
        default: break;                                                                      \
      }                                                                                      \
    } else if (pl.va && pl.vb) {                                                             \
      igemm_kernel<MODE, BM_, BN_, WM_, WN_, true, true><<<grid, block, 0, s>>>(pl.p);       \
    } else if (pl.va) {                                                                      \
      igemm_kernel<MODE, BM_, BN_, WM_, WN_, true, false><<<grid, block, 0, s>>>(pl.p);      \
    } else if (pl.vb) {                                                                      \
      igemm_kernel<MODE, BM_, BN_, WM_, WN_, false, true><<<grid, block, 0, s>>>(pl.p);      \
    } else {                                                                                 \
      igemm_kernel<MODE, BM_, BN_, WM_, WN_, false, false><<<grid, block, 0, s>>>(pl.p);     \
    }                                                                                        \
  } while (0)

template <int MODE>
static hipError_t launch_cfg(const Plan &pl, hipStream_t s) {
  dim3 grid(pl.tiles, pl.p.splits, pl.s2 ? 4 : 1), block(256);
  switch (pl.cfg) {
    case 0: AS_LAUNCH(128, 128, 2, 2, 32); break;
    case 1: AS_LAUNCH(256, 32, 4, 1, 32); break;
    case 2: AS_LAUNCH(32, 256, 1, 4, 32); break;
    case 3: AS_LAUNCH(64, 256, 1, 4, 32); break;
    default: AS_LAUNCH(256, 64, 4, 1, 16); break;
  }
  return hipGetLastError();
}

hipError_t LAUNCH_NAME(const Plan &pl, hipStream_t s) { return launch_cfg<LAUNCH_MODE>(pl, s); }

}  // namespace adaptseg
