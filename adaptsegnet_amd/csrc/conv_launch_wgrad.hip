// Kernel instantiations for the WGRAD conv product (its own translation unit).
#define LAUNCH_NAME launch_wgrad
#define LAUNCH_MODE MODE_WGRAD
#include "conv_kernels.hpp"
#include "conv_launch_body.inc"
