// Kernel instantiations for the DGRAD conv product (its own translation unit).
#define LAUNCH_NAME launch_dgrad
#define LAUNCH_MODE MODE_DGRAD
#include "conv_kernels.hpp"
#include "conv_launch_body.inc"
