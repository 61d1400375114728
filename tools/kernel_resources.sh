#!/bin/bash
# Registers, spills and scratch of every kernel in the built library, read from the embedded gfx950
# code object (no recompile): bash tools/kernel_resources.sh [lib.so] [name regex]
LIB=${1:-$(dirname $0)/../cartpoleplusplus_amd/libcartpole_hip.so}
PAT=${2:-step_kernel|reset_kernel|rollout}
T=$(mktemp -d)
objcopy -O binary --only-section=.hip_fatbin "$LIB" $T/fatbin.bin || exit 1
/opt/rocm/lib/llvm/bin/clang-offload-bundler --unbundle --type=o --targets=hipv4-amdgcn-amd-amdhsa--gfx950 \
    --input=$T/fatbin.bin --output=$T/co.elf || exit 1
/opt/rocm/lib/llvm/bin/llvm-readelf --notes $T/co.elf | grep -E "\.name:|\.vgpr_count|\.private_segment_fixed_size|\.sgpr_spill|\.vgpr_spill" \
    | paste - - - - - | grep -E "$PAT" | sed 's/  */ /g; s/ \.name: / /; s/\.private_segment_fixed_size/scratch/; s/\.sgpr_spill_count/sgpr_spill/; s/\.vgpr_count/vgpr/; s/\.vgpr_spill_count/vgpr_spill/'
rm -rf $T
