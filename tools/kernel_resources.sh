#!/bin/bash
# Registers, spills and scratch of every kernel in the built library, read from the embedded gfx950
# code objects (one bundle per translation unit; no recompile):
#   bash tools/kernel_resources.sh [lib.so] [name regex]
LIB=${1:-$(dirname $0)/../cartpoleplusplus_amd/libcartpole_hip.so}
PAT=${2:-step_kernel|reset_kernel|rollout}
T=$(mktemp -d)
objcopy -O binary --only-section=.hip_fatbin "$LIB" $T/fatbin.bin || exit 1
python3 - "$T" <<'PY'
import sys
d = sys.argv[1]
b = open(f"{d}/fatbin.bin", "rb").read()
m = b"__CLANG_OFFLOAD_BUNDLE__"
starts = [i for i in range(len(b)) if b.startswith(m, i)]
for k, s in enumerate(starts):
    e = starts[k + 1] if k + 1 < len(starts) else len(b)
    open(f"{d}/bundle{k}.bin", "wb").write(b[s:e])
PY
for f in $T/bundle*.bin; do
  /opt/rocm/lib/llvm/bin/clang-offload-bundler --unbundle --type=o --targets=hipv4-amdgcn-amd-amdhsa--gfx950 \
      --input=$f --output=$f.elf 2>/dev/null || continue
  /opt/rocm/lib/llvm/bin/llvm-readelf --notes $f.elf | grep -E "\.name:|\.vgpr_count|\.private_segment_fixed_size|\.sgpr_spill|\.vgpr_spill" \
      | paste - - - - - | grep -E "$PAT" | sed 's/  */ /g; s/ \.name: / /; s/\.private_segment_fixed_size/scratch/; s/\.sgpr_spill_count/sgpr_spill/; s/\.vgpr_count/vgpr/; s/\.vgpr_spill_count/vgpr_spill/'
done
rm -rf $T
