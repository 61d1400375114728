// Microbenchmark (diagnostic, not part of the library): the latency-shaped kernels' settle-structure PGS
// sweep (cp_physics.h sweeps_c44: 4 +z ground rows, then 4 cart-pole rows, fast form) run by one wave
// alone on its SIMD, on synthetic rows; cycles per sweep (s_memtime) vs the same wave count spread.
// hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-slp-vectorize -DCP_STAMPS \
//     -mllvm -amdgpu-sched-strategy=iterative-ilp tools/micro/sweep_c44.hip -o tools/micro/sweep_c44
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../include/cartpole_amd.h"
#include "../../cartpoleplusplus_amd/csrc/cp_common.h"
#define CP_NS cpm
#define CP_REAL float
#include "../../cartpoleplusplus_amd/csrc/cp_math.h"
#include "../../cartpoleplusplus_amd/csrc/cp_physics.h"

namespace cpm {
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(1, 1)))
bench_c44(const float* in, float* out, unsigned long long* cyc, int nsweeps) {
    const int t = blockIdx.x * 64 + threadIdx.x;
    const float* p = in + (size_t)t * 128;
    int k = 0;
    auto nx = [&]() { return p[k++]; };
    Ctx c;
    FastIsl F;
    Stamps ST;
    c.I.d1.v = mk(nx(), nx(), nx()); c.I.d1.w = mk(nx(), nx(), nx());
    c.I.d2.v = mk(nx(), nx(), nx()); c.I.d2.w = mk(nx(), nx(), nx());
    c.I.im1 = 1.0f; c.I.im2 = 0.2f;
    c.T.n[2] = mk(nx(), nx(), 1.0f);
    for (int r = 0; r < 4; ++r) {
        F.g0[r].rbt = mk(nx(), nx(), 0.0f); F.g0[r].ib = mk(nx(), nx(), nx());
        F.g0[r].ie = nx(); F.g0[r].tg = nx(); F.g0[r].lam = nx();
        F.c2[r].rbt = mk(nx(), nx(), nx()); F.c2[r].ib = mk(nx(), nx(), nx());
        F.c2[r].rat = mk(nx(), nx(), nx()); F.c2[r].ia = mk(nx(), nx(), nx());
        F.c2[r].ie = nx(); F.c2[r].tg = nx(); F.c2[r].lam = nx();
    }
    c.active = true;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    sweeps_c44(c, F, 0.0f, 0, nsweeps, ST);
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    float acc = c.I.d1.v.x + c.I.d1.w.y + c.I.d2.v.z + c.I.d2.w.x;
    for (int r = 0; r < 4; ++r) acc += F.g0[r].lam + F.c2[r].lam;
    out[t] = acc;
    if (threadIdx.x == 0) {
        cyc[blockIdx.x * 2] = t1 - t0;
        cyc[blockIdx.x * 2 + 1] = ST.sweeps;
    }
}
}  // namespace cpm

int main(int argc, char** argv) {
    const int waves_list[3] = {1, 11, 340};
    std::vector<float> h(340 * 64 * 128);
    srand(1);
    for (size_t i = 0; i < h.size(); ++i) {
        const int f = (int)(i % 128);
        float u = (float)rand() / RAND_MAX - 0.5f;
        // ie ~ 0.3..0.8, lam ~ 0..2, velocities / lever terms small
        h[i] = (f >= 13) ? u * 0.1f : u * 0.01f;
    }
    for (size_t e = 0; e < h.size() / 128; ++e) {   // effective masses and impulses positive
        float* p = &h[e * 128];
        int k = 15;
        for (int r = 0; r < 4; ++r) {
            k += 5; p[k++] = 0.5f; p[k++] = -0.001f; p[k++] = 1.0f;        // ground row ie, tg, lam
            k += 12; p[k++] = 0.3f; p[k++] = -0.0005f; p[k++] = 2.0f;      // cart-pole row ie, tg, lam
        }
    }
    float *d_in, *d_out; unsigned long long* d_cyc;
    hipMalloc(&d_in, h.size() * 4); hipMalloc(&d_out, 340 * 64 * 4); hipMalloc(&d_cyc, 340 * 16);
    hipMemcpy(d_in, h.data(), h.size() * 4, hipMemcpyHostToDevice);
    for (int wi = 0; wi < 3; ++wi) {
        const int W = waves_list[wi];
        for (int rep = 0; rep < 3; ++rep) {
            hipLaunchKernelGGL(cpm::bench_c44, dim3(W), dim3(64), 0, 0, d_in, d_out, d_cyc, 50);
            hipDeviceSynchronize();
        }
        std::vector<unsigned long long> c(W * 2);
        hipMemcpy(c.data(), d_cyc, W * 16, hipMemcpyDeviceToHost);
        double sum = 0, sw = 0;
        for (int w = 0; w < W; ++w) { sum += c[2 * w]; sw += c[2 * w + 1]; }
        printf("waves %4d: %.0f cycles per wave, %.1f sweeps, %.0f cycles per sweep\n", W, sum / W, sw / W,
               sum / sw);
    }
    return 0;
}
