// Thin convolutions (Cout <= 4) on the vector ALUs: see conv_thin.hip.
#pragma once
#include "common.hpp"

namespace adaptseg {

// Cout <= 4, one segment, NHWC input with Cin % 4 == 0, weights fit LDS; data gradient stride 1.
bool thin_eligible(const adaptseg_conv_desc *d, int op);
size_t thin_workspace(const adaptseg_conv_desc *d, int op);
inline int thin_kernel_id(int op) { return 100 * op + 80; }
// Return ADAPTSEG_ERR_ARG (nothing launched) when an operand is not 16-byte aligned: the caller
// then takes the implicit-GEMM path.
int thin_fwd(const adaptseg_conv_desc *d, const float *x, const float *w, const float *bias, const float *res,
             float *y, int flags, hipStream_t s);
int thin_dgrad(const adaptseg_conv_desc *d, const float *dy, const float *w, const float *res, const float *aux,
               float *dx, int flags, hipStream_t s);
int thin_wgrad(const adaptseg_conv_desc *d, const float *dy, const float *x, float *dw, int flags, void *ws,
               size_t ws_bytes, hipStream_t s);

}  // namespace adaptseg
