// cp_kernels64.hip — the fp64 instantiation of the env kernels (cp_env.h over real =
// double, namespace cp64): the parity variant of cp_config.precision == CP_PRECISION_F64,
// bit-exact against the oracle's fp64 build (tests/test_gpu_f64.py).  Its
// launchers are called from the C-ABI in cp_kernels.hip (cp_common.h declares them).
#include <hip/hip_runtime.h>

#include "../../include/cartpole_amd.h"
#include "cp_common.h"

#define CP_NS cp64
#define CP_REAL double
#include "cp_math.h"
#include "cp_physics.h"
#include "cp_env.h"
#undef CP_NS
#undef CP_REAL
