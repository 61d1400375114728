#!/bin/bash
# Where does hipcc spill?  Prints scratch loads/stores per source line of the discrete step kernel.
# usage: bash tools/spills.sh [extra hipcc flags, e.g. -DCP_WAVES_PER_EU=2]
OUT=/tmp/cp_spills.s
/opt/rocm/bin/hipcc -O3 -gline-tables-only --offload-arch=gfx950 -std=c++17 -ffp-contract=off -fno-slp-vectorize -S --cuda-device-only "$@" \
    $(dirname $0)/../cartpoleplusplus_amd/csrc/cp_kernels.hip -o $OUT 2>/dev/null || exit 1
awk '/^_ZN2cp14cp_step_kernelILi1/,/s_endpgm/' $OUT > $OUT.k
grep "\.file" $OUT | awk '{print $2, $4}' | tr -d '"' > $OUT.files
awk 'NR==FNR {f[$1]=$2; next} /\.loc/ {loc=f[$2]":"$3} /scratch_(store|load)/ {print loc}' $OUT.files $OUT.k | sort | uniq -c | sort -rn | head -${N:-25}
