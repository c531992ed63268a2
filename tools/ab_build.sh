#!/bin/bash
# A/B variant of libgpuinspect.so: kernels.hip rebuilt with extra -D flags,
# linked with the in-tree host objects -> ab/<name>/libgpuinspect.so (load it
# with GI_LIB=ab/<name>/libgpuinspect.so).  Prints the variant's k_scan /
# k_eval / k_detect register and scratch usage.
#   tools/ab_build.sh <name> "<flags>"
set -eu
cd "$(dirname "$0")/.."
N=$1; F=${2:-}
S=${SRC:-coraza-kubernetes-operator_amd/csrc/kernels.hip}  # another kernels source (same directory) for the variant
D=ab/$N; mkdir -p $D
M=coraza-kubernetes-operator_amd
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function \
  -D__HIP_DEFINE_EXTENDED_HOST_MIN_MAX__=1 -mllvm -amdgpu-spill-vgpr-to-agpr=0 $F \
  -Rpass-analysis=kernel-resource-usage -c $S -o $D/kernels.o 2> $D/resources.txt
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $D/libgpuinspect.so $D/kernels.o \
  $M/build/runtime.o $M/build/compile.o $M/build/regex.o $M/build/dfa.o $M/build/pike.o $M/build/artifact.o
python3 tools/kernel_res.py $D/resources.txt
