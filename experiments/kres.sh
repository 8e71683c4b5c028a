#!/bin/bash
# Register / LDS / spill usage of the kernels in one built object: bash experiments/kres.sh conv_launch_x3 [name-regex]
set -e
OBJ=$(dirname "$0")/../adaptsegnet_amd/csrc/build/$1.o
D=$(mktemp -d)
LLVM=/opt/rocm/lib/llvm/bin
$LLVM/llvm-objcopy --dump-section=.hip_fatbin=$D/fat.bin "$OBJ"
$LLVM/clang-offload-bundler --unbundle --type=o --input=$D/fat.bin --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=$D/k.co
$LLVM/llvm-readelf --notes $D/k.co | grep -E "^ +\.name:|\.vgpr_count|\.agpr_count|spill_count|group_segment_fixed" \
  | paste - - - - - - | sed 's/ \+/ /g' | grep -E "${2:-.}"
rm -rf $D
