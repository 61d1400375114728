#!/bin/bash
# Device-only compile of ONE env kernel instantiation (seconds instead of the library's minutes), for
# reading its register use and loops:  bash tools/isa_one.sh 'cp_reset_kernel<true>' out.s [-DFLAG ...]
#   python3 tools/isa_loops.py out.s    (loop sizes, AGPR moves, LDS ops per loop)
set -e
K=$1; OUT=$2; shift 2
ARGS=${ARGS:-o}  # the kernel arguments after (cfg, b): step kernels ARGS="v, o, o, d, o, o, 0, lq"
R=$(cd $(dirname $0)/.. && pwd)
T=$(mktemp -d)
cat > $T/one.hip <<SRC
#include <hip/hip_runtime.h>
#include <type_traits>
#include "$R/include/cartpole_amd.h"
#include "$R/cartpoleplusplus_amd/csrc/cp_common.h"
#define CP_KERNELS_ONLY
#define CP_NS ${NS:-cp}
#define CP_REAL ${REAL:-float}
#include "$R/cartpoleplusplus_amd/csrc/cp_math.h"
#include "$R/cartpoleplusplus_amd/csrc/cp_physics.h"
#include "$R/cartpoleplusplus_amd/csrc/cp_env.h"
__global__ void one_entry(cp_config cfg, cpc::Bufs b, float* o) { (void)cfg; (void)b; (void)o; }
void one_launch(cp_config cfg, cpc::Bufs b, void* v, float* o, uint8_t* d, cpc::Lqr lq) {
    (void)v; (void)d; (void)lq;
    hipLaunchKernelGGL((${NS:-cp}::$K), dim3(1), dim3(64), 0, 0, cfg, b, $ARGS);
}
SRC
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -ffp-contract=off -fno-slp-vectorize \
    -mllvm -amdgpu-sched-strategy=iterative-ilp --cuda-device-only -c "$@" -o $T/one.o $T/one.hip
/opt/rocm/lib/llvm/bin/clang-offload-bundler --unbundle --type=o --targets=hipv4-amdgcn-amd-amdhsa--gfx950 \
    --input=$T/one.o --output=$T/one.elf
/opt/rocm/lib/llvm/bin/llvm-readelf --notes $T/one.elf | grep -E "\.name:|\.vgpr_count|\.agpr_count|\.private_segment_fixed_size|\.vgpr_spill" | grep -v one_entry || true
/opt/rocm/lib/llvm/bin/llvm-objdump -d --no-show-raw-insn $T/one.elf > $OUT
rm -rf $T
