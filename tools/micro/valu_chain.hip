// Microbenchmark (diagnostic, not part of the library): cycles per instruction of one wave alone on
// its SIMD for dependent and independent fp32 VALU chains, the instruction mix of the PGS row chain.
// hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/micro/valu_chain.hip -o /tmp/valu_chain
#include <hip/hip_runtime.h>
#include <cstdio>

#define N 1024

template <int MODE>
__global__ void __launch_bounds__(64) chain(float* out, float a, float b, unsigned long long* cyc) {
    float x = a + threadIdx.x, y = b, z = a * 0.5f, w = b * 0.25f;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
    for (int it = 0; it < 8; ++it) {
#pragma unroll
        for (int k = 0; k < N / 8; ++k) {
            if constexpr (MODE == 0) {         // dependent fma chain
                x = __builtin_fmaf(x, y, z);
            } else if constexpr (MODE == 1) {  // 4 independent fma chains interleaved
                x = __builtin_fmaf(x, y, 1.0f); z = __builtin_fmaf(z, y, 1.0f);
                w = __builtin_fmaf(w, y, 1.0f); y = __builtin_fmaf(y, 0.999f, 0.001f);
            } else if constexpr (MODE == 2) {  // dependent mul / add / sub / max mix (the row chain's shape)
                x = x * y; x = x + z; x = w - x; x = __builtin_fmaxf(x, 0.0f);
            } else if constexpr (MODE == 3) {  // dependent chain with a compare into a mask per 4 ops
                x = x * y; x = x + z; x = w - x; x = __builtin_fmaxf(x, 0.0f);
                z = (__builtin_fabsf(x) > 1e-3f) ? z + 1.0f : z;
            }
        }
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = x + y + z + w;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

int main() {
    float* out; unsigned long long* cyc;
    hipMalloc(&out, 64 * sizeof(float)); hipMalloc(&cyc, 8);
    const char* names[4] = {"dependent fma", "4 independent fma chains", "dependent mul/add/sub/max",
                            "dependent + compare/select"};
    const double ops[4] = {N, 4.0 * N, 4.0 * N, 6.0 * N};
    for (int m = 0; m < 4; ++m) {
        for (int rep = 0; rep < 3; ++rep) {
            if (m == 0) hipLaunchKernelGGL(chain<0>, dim3(1), dim3(64), 0, 0, out, 1.0f, 0.999f, cyc);
            if (m == 1) hipLaunchKernelGGL(chain<1>, dim3(1), dim3(64), 0, 0, out, 1.0f, 0.999f, cyc);
            if (m == 2) hipLaunchKernelGGL(chain<2>, dim3(1), dim3(64), 0, 0, out, 1.0f, 0.999f, cyc);
            if (m == 3) hipLaunchKernelGGL(chain<3>, dim3(1), dim3(64), 0, 0, out, 1.0f, 0.999f, cyc);
            hipDeviceSynchronize();
        }
        unsigned long long c = 0;
        hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
        printf("%-30s %8llu cycles for %6.0f source ops = %.2f cycles/op\n", names[m], c, ops[m], c / ops[m]);
    }
    return 0;
}
