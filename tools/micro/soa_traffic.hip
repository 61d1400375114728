// soa_traffic.hip -- calibrate rocprofv3's FETCH_SIZE / WRITE_SIZE on the step kernel's exact HBM access
// shape: is the guide's x2 FETCH_SIZE correction (MI355X_MICROARCH.md, measured for
// 16-B/lane streaming loads) right for 4-B/lane buffer loads over the state SoA, and what do the
// kernel's stores count as?  Each kernel moves a known number of bytes; run under
//   rocprofv3 --kernel-trace --pmc FETCH_SIZE -- ./soa_traffic      (then a second run with WRITE_SIZE)
// and divide the per-launch counter by the kernel's byte count (printed by the program).
//
// Shapes (B = 65,536 envs, 2 lanes per env as in cp_step_kernel, state SoA [123][B] float through a
// buffer resource with an SGPR field offset and a VGPR env offset -- cpc::SoaT, the kernel's own code):
//   rd16        16-B/lane coalesced streaming read of the 32.2 MB SoA (the guide's calibration case)
//   rd_pair     both lanes of each env load all 123 fields (4 B/lane, the pair reads one column)
//   wr_lead     the pair's first lane stores 119 fields (the step kernel's store_sim + steps + caches)
//   step_shape  the step kernel's pattern: both lanes load the 60 body / force / counter fields, each
//               lane its island's 25 warm-start fields; the first lane stores 59 fields, each lane its
//               island's 25 cache fields; the first lane writes 168 B of obs + reward + done
//   obs_rows    the first lane of each pair writes its env's 42 obs floats (env-major rows, 168 B)
// Every read kernel folds what it loads into one float per env written to a sink (B * 4 B, counted).
// build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -I ../../cartpoleplusplus_amd/csrc -I ../../include
//        soa_traffic.hip -o soa_traffic
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "cartpole_amd.h"
#include "cp_common.h"

using cpc::SoaT;
using Soa = SoaT<float>;
constexpr int B = 65536, F = CP_STATE_FIELDS, WAVE = 64;

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                   \
            std::exit(1);                                                                  \
        }                                                                                  \
    } while (0)

__global__ void __launch_bounds__(256) rd16(const float4* __restrict__ s, float* sink, int n4) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    float acc = 0.f;
    for (int k = t; k < n4; k += gridDim.x * blockDim.x) {
        const float4 v = s[k];
        acc += v.x + v.y + v.z + v.w;
    }
    if (acc == 1234.5f) sink[t] = acc;   // never true on the zero-filled input: no stores
}

__global__ void __launch_bounds__(WAVE) rd_pair(void* state, float* sink) {
    const int t = blockIdx.x * WAVE + threadIdx.x, i = t >> 1;
    const Soa st = Soa::make(state, B, F);
    const uint32_t o = Soa::eoff(i);
    float acc = 0.f;
#pragma unroll 8
    for (int f = 0; f < F; ++f) acc += st.ld(f, o);
    if ((t & 1) == 0) sink[i] = acc;
}

__global__ void __launch_bounds__(WAVE) wr_lead(void* state) {
    const int t = blockIdx.x * WAVE + threadIdx.x, i = t >> 1;
    if (t & 1) return;
    const Soa st = Soa::make(state, B, F);
    const uint32_t o = Soa::eoff(i);
#pragma unroll 8
    for (int f = 0; f < 119; ++f) st.st(f, o, (float)f);
}

__global__ void __launch_bounds__(WAVE) step_shape(void* state, float* obs, float* rew, uint8_t* done) {
    const int t = blockIdx.x * WAVE + threadIdx.x, i = t >> 1, isl = t & 1;
    const Soa st = Soa::make(state, B, F);
    const uint32_t o = Soa::eoff(i);
    const uint32_t wo = o + (uint32_t)(isl * CP_ISLAND_PAIRS) * st.fstride;      // Mem::woff
    const uint32_t lo = o + (uint32_t)(isl * 4 * CP_ISLAND_PAIRS) * st.fstride;  // Mem::loff
    float v[60];
#pragma unroll
    for (int f = 0; f < 60; ++f) v[f] = st.ld(f, o);                            // bodies, forces, steps, done
    float acc = 0.f;
#pragma unroll
    for (int j = 0; j < CP_ISLAND_PAIRS; ++j) {
        acc += st.ld(CP_SF_WS_ID(0, j), wo);
#pragma unroll
        for (int k = 0; k < 4; ++k) acc += st.ld(CP_SF_WS_LAM(0, j, k), lo);
    }
#pragma unroll
    for (int f = 0; f < 60; ++f) v[f] += acc;
#pragma unroll
    for (int j = 0; j < CP_ISLAND_PAIRS; ++j) {
        st.st(CP_SF_WS_ID(0, j), wo, acc);
#pragma unroll
        for (int k = 0; k < 4; ++k) st.st(CP_SF_WS_LAM(0, j, k), lo, acc + (float)k);
    }
    if (isl) return;
#pragma unroll
    for (int f = 0; f < 59; ++f) st.st(f, o, v[f]);
    float* ob = obs + (size_t)i * 42;
#pragma unroll
    for (int f = 0; f < 42; ++f) ob[f] = v[f % 60];
    rew[i] = 1.f;
    done[i] = 0;
}

__global__ void __launch_bounds__(WAVE) obs_rows(float* obs) {
    const int t = blockIdx.x * WAVE + threadIdx.x, i = t >> 1;
    if (t & 1) return;
    float* ob = obs + (size_t)i * 42;
#pragma unroll
    for (int f = 0; f < 42; ++f) ob[f] = (float)f;
}

int main(int argc, char** argv) {
    const int reps = argc > 1 ? std::atoi(argv[1]) : 20;
    void* state;
    float *sink, *obs, *rew;
    uint8_t* done;
    CK(hipMalloc(&state, (size_t)F * B * 4));
    CK(hipMalloc(&sink, (size_t)B * 8));
    CK(hipMalloc(&obs, (size_t)B * 42 * 4));
    CK(hipMalloc(&rew, (size_t)B * 4));
    CK(hipMalloc(&done, (size_t)B));
    CK(hipMemset(state, 0, (size_t)F * B * 4));
    const dim3 g2(2 * B / WAVE), w(WAVE);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timeit = [&](const char* name, double rd, double wr, auto&& launch) {
        launch();
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        for (int r = 0; r < reps; ++r) launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms = 0.f;
        CK(hipEventElapsedTime(&ms, e0, e1));
        std::printf("{\"kernel\": \"%s\", \"alg_read_bytes\": %.0f, \"alg_write_bytes\": %.0f, \"avg_us\": %.2f, "
                    "\"launches\": %d}\n", name, rd, wr, 1e3 * ms / reps, reps + 1);
    };
    const double S = (double)F * B * 4;
    timeit("rd16", S, 0, [&] { hipLaunchKernelGGL(rd16, dim3(1024), dim3(256), 0, 0, (const float4*)state, sink, (int)(S / 16)); });
    timeit("rd_pair", S, B * 4.0, [&] { hipLaunchKernelGGL(rd_pair, g2, w, 0, 0, state, sink); });
    timeit("wr_lead", 0, 119.0 * B * 4, [&] { hipLaunchKernelGGL(wr_lead, g2, w, 0, 0, state); });
    timeit("step_shape", (60.0 + 50.0) * B * 4, (59.0 + 50.0) * B * 4 + B * (168.0 + 4 + 1),
           [&] { hipLaunchKernelGGL(step_shape, g2, w, 0, 0, state, obs, rew, done); });
    timeit("obs_rows", 0, 168.0 * B, [&] { hipLaunchKernelGGL(obs_rows, g2, w, 0, 0, obs); });
    CK(hipDeviceSynchronize());
    return 0;
}
