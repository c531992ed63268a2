#!/bin/bash
# Per-kernel VGPRs / scratch / VGPR spills of the built engine (code-object
# metadata of build/kernels.o; no GPU needed).
set -eu
R=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
B=/opt/rocm/lib/llvm/bin
$B/llvm-objcopy --dump-section=.hip_fatbin=$T/fat.bin "$R/coraza-kubernetes-operator_amd/build/kernels.o"
$B/clang-offload-bundler --unbundle --type=o --input=$T/fat.bin --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=$T/k.co
$B/llvm-readelf --notes $T/k.co | grep -E "^ +\.name:|\.private_segment_fixed_size|\.vgpr_count|\.vgpr_spill_count" |
  paste - - - - | sed 's/  */ /g'
rm -rf "$T"
