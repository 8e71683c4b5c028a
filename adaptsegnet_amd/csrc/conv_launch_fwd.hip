// Kernel instantiations for the FWD conv product (its own translation unit).
#define LAUNCH_NAME launch_fwd
#define LAUNCH_MODE MODE_FWD
#include "conv_kernels.hpp"
#include "conv_launch_body.inc"
