// cp_common.h — pieces of the cartpole kernels that do not depend on the real type.
//
// The physics (cp_math.h, cp_physics.h, cp_env.h) is written once over `real` and
// instantiated twice: namespace cp (real = float, the product path) and namespace cp64
// (real = double, the fp64 parity variant).  The overloads here give both
// instantiations the same source: every fused multiply-add is an explicit fma_ (v_fma_f32
// / v_fma_f64), the library is compiled with -ffp-contract=off, and division / sqrt are the
// IEEE-correct defaults, so each instantiation rounds exactly like the oracle's build of
// the same type (oracle/cp_oracle.c, real = float or double).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/cartpole_amd.h"

#define CP_DEV __device__ __forceinline__

// CP_MODEL_PERSISTENT: per lane (island) and local pair, the persistent manifold: count, then for
// the 4 cache slots the local point on A (3), on B (3), the normal (3), the separation (1) and the
// applied normal impulse (1) -- buffer Bufs::pman, one column per lane (cp_physics.h PMan)
#define CP_PM_PAIR_FIELDS 45
#define CP_PM_FIELDS (CP_ISLAND_PAIRS * CP_PM_PAIR_FIELDS)

// Scratch SoA (Bufs::scratch), one column per lane: rows [0, CP_SCR_HDR_FIELDS) are reserved (the
// manifold headers of a diagnostic build until round 5; the headers live in registers); rows
// [CP_SCR_RC_BASE, CP_SCR_FIELDS) hold cp_rollout's per-lane state machine (RC_* in cp_env.h), kept
// across substeps.
#define CP_SCR_HDR_FIELDS (4 * CP_ISLAND_PAIRS)
#define CP_SCR_RC_BASE CP_SCR_HDR_FIELDS
#define CP_SCR_RC_FIELDS 10
#define CP_SCR_FIELDS (CP_SCR_RC_BASE + CP_SCR_RC_FIELDS)

namespace cpc {

CP_DEV float fma_(float a, float b, float c) { return __builtin_fmaf(a, b, c); }
CP_DEV double fma_(double a, double b, double c) { return __builtin_fma(a, b, c); }
CP_DEV float fmaf_(float a, float b, float c) { return __builtin_fmaf(a, b, c); }  // fp32-only code (raster)
CP_DEV float sqrt_(float x) { return sqrtf(x); }
CP_DEV double sqrt_(double x) { return sqrt(x); }
CP_DEV float abs_(float x) { return fabsf(x); }
CP_DEV double abs_(double x) { return fabs(x); }

// Friction clamp to [-b, b] for b > 0: one v_med3_f32 in fp32 (the same value as the
// oracle's compare chain for every non-NaN l); fp64 has no med3, so the compare chain itself.
CP_DEV float clamp_sym(float l, float b) { return __builtin_amdgcn_fmed3f(l, -b, b); }
CP_DEV double clamp_sym(double l, double b) { return l > b ? b : (l < -b ? -b : l); }

// The partner lane of a lane pair (DPP quad_perm [1,0,3,2]).  Only where both lanes of
// the pair are active: a DPP read of an inactive lane returns garbage.
CP_DEV uint32_t partner_u(uint32_t x) { return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xF, 0xF, false); }
CP_DEV float partner(float x) { return __uint_as_float(partner_u(__float_as_uint(x))); }
CP_DEV double partner(double x) {
    const uint64_t u = (uint64_t)__double_as_longlong(x);
    const uint64_t lo = partner_u((uint32_t)u), hi = partner_u((uint32_t)(u >> 32));
    return __longlong_as_double((long long)(lo | (hi << 32)));
}
// Island ISL's lane of the pair, read by both lanes (DPP quad_perm [0,0,2,2] / [1,1,3,3]): one move where
// "own value on one lane, the partner's on the other" took a partner read and a select.  Same rule.
template <int ISL>
CP_DEV uint32_t lane_of_u(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, ISL ? 0xF5 : 0xA0, 0xF, 0xF, false);
}
template <int ISL>
CP_DEV float lane_of(float x) { return __uint_as_float(lane_of_u<ISL>(__float_as_uint(x))); }
template <int ISL>
CP_DEV double lane_of(double x) {
    const uint64_t u = (uint64_t)__double_as_longlong(x);
    const uint64_t lo = lane_of_u<ISL>((uint32_t)u), hi = lane_of_u<ISL>((uint32_t)(u >> 32));
    return __longlong_as_double((long long)(lo | (hi << 32)));
}

// Integer fields (steps, episode, done, warm-start ids, packed headers) kept in a
// real-typed array: the int32 bits in the first 4 bytes; an fp64 field's high word is 0
// (the oracle's fp64 build stores them the same way: memcpy of 4 bytes into a zeroed double).
template <typename R> CP_DEV R bits_to(uint32_t v);
template <> CP_DEV float bits_to<float>(uint32_t v) { return __uint_as_float(v); }
template <> CP_DEV double bits_to<double>(uint32_t v) { return __longlong_as_double((long long)(uint64_t)v); }
CP_DEV uint32_t to_bits(float x) { return __float_as_uint(x); }
CP_DEV uint32_t to_bits(double x) { return (uint32_t)(uint64_t)__double_as_longlong(x); }

// SoA field access through a buffer resource: the field base is a wave-uniform SGPR
// soffset (f * B * sizeof(T)) and the env is a 32-bit VGPR voffset (i * sizeof(T)), so
// each env keeps one offset register instead of a 64-bit address per field (the flat form
// made the compiler hoist and spill ~100 of them).  Limits one SoA array to 4 GiB:
// B * fields * sizeof(T) < 2^32 (checked at cp_create).
// The SoA buffer accesses use the default cache policy (aux 0): streaming the state past L2 (nt) was
// measured slower.

template <typename T>
struct SoaT {
    __amdgpu_buffer_rsrc_t r;
    uint32_t fstride;  // B * sizeof(T) bytes
    CP_DEV static SoaT make(void* base, int B, int fields) {
        SoaT s;
        s.r = __builtin_amdgcn_make_buffer_rsrc(base, (short)0,
                                                (int)((uint32_t)B * (uint32_t)sizeof(T) * (uint32_t)fields), 0x00020000);
        s.fstride = (uint32_t)B * (uint32_t)sizeof(T);
        return s;
    }
    CP_DEV static uint32_t eoff(int i) { return (uint32_t)i * (uint32_t)sizeof(T); }
    CP_DEV T ld(int f, uint32_t off) const {
        if constexpr (sizeof(T) == 4) {
            return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, (int)off, (int)((uint32_t)f * fstride), 0));
        } else {
            const auto v = __builtin_amdgcn_raw_buffer_load_b64(r, (int)off, (int)((uint32_t)f * fstride), 0);
            return __longlong_as_double((long long)(((uint64_t)(uint32_t)v[1] << 32) | (uint32_t)v[0]));
        }
    }
    CP_DEV void st(int f, uint32_t off, T x) const {
        if constexpr (sizeof(T) == 4) {
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(x), r, (int)off, (int)((uint32_t)f * fstride), 0);
        } else {
            const uint64_t u = (uint64_t)__double_as_longlong(x);
            __attribute__((ext_vector_type(2))) unsigned int v = {(unsigned int)u, (unsigned int)(u >> 32)};
            __builtin_amdgcn_raw_buffer_store_b64(v, r, (int)off, (int)((uint32_t)f * fstride), 0);
        }
    }
};

// closed-loop LQR policy arguments (random_action_agent.py:60-135)
struct Lqr {
    const float* gains;  // [B or 1][2 pairs][2 (fx, fy)][8]
    int per_env;
    float* state8;       // [B][2][R][S][8] or null
    float done_pos;      // _check_done thresholds (:108-119); <= 0: no bounds termination
    float done_angle;
};

// Per-handle device buffers.  `state` and `scratch` hold the handle's real type.
struct Bufs {
    void* state;       // [CP_STATE_FIELDS][B] real
    float* term_obs;   // [R*14][B]
    void* bumps;       // [B][ifs][2][2] of the handle's real type (float, or double for fp64 handles)
    float* ret_acc;    // [B]
    float* last_ret;   // [B]
    int32_t* last_len; // [B]
    int32_t* overflow; // [B]
    int32_t* nonfinite;  // [B] steps / resets that ended with a non-finite body state
    int32_t* list;     // [B] reset list
    int32_t* count;    // reset list length (one of the handle's two counters, by step parity)
    int32_t* count_next;  // the other counter: zeroed by the step and reset kernels for the next call
    void* scratch;     // [CP_SCR_FIELDS][2B] real: reserved rows, cp_rollout state
    uint64_t* stamps;  // [waves][8] diagnostic phase cycles (CP_STAMPS builds only)
    float* rposes;     // [B][R][4][7] repeat-end poses for the raster obs (NULL: raster off)
    float4* rtable;    // [C][H*W] (d, t_ground) then [C][H*W] uint8 ground class (cp_raster_table_kernel)
    int32_t* rlist;    // [B] envs to render after the step kernel
    int32_t* rcount;   // [1]
    uint8_t* stepped;  // [B] 1 = simulated by the last cp_step (event log: done-before envs are not logged)
    void* pman;        // [CP_PM_FIELDS][2B] real: persistent manifolds (CP_MODEL_PERSISTENT handles only)
    int32_t npar;      // CP_AUTORESET_NEXT_STEP: the reset list this call appends to (0 / 1); a finishing
                       // env's done field becomes 2 + npar until the next call returns its reset obs
    int32_t keep_done; // reset kernel: leave the done field (NEXT_STEP's in-flight reset; the fixup clears it)
    int32_t nlo, nhi;  // reset kernel: serve a list of length n only if nlo < n <= nhi (nhi 0: no upper bound;
                       // CP_SHAPE_LIST's launches, one per layout)
};

}  // namespace cpc

// Launches of one real type's kernels (cp_env.h), defined in that instantiation's translation
// unit: cp_kernels.hip (fp32, namespace cp) and cp_kernels64.hip (fp64, namespace cp64).
#define CP_DECLARE_LAUNCHES(NS)                                                                                  \
    namespace NS {                                                                                               \
    void launch_init(const cp_config& cfg, const cpc::Bufs& b, hipStream_t st);                                  \
    void launch_reset(int shape, const cp_config& cfg, const cpc::Bufs& b, float* obs_out, hipStream_t st);     \
    void launch_nextstep_fixup(const cp_config& cfg, const cpc::Bufs& b, const int32_t* list, const int32_t* count, \
                               int q, const float* nobs, float* obs_out, float* reward_out, uint8_t* done_out,    \
                               hipStream_t st);                                                                    \
    void launch_nextstep_resolve(const cp_config& cfg, const cpc::Bufs& b, const uint8_t* mask, const float* nobs, \
                                 float* obs_out, hipStream_t st);                                                  \
    void launch_step(int shape, int kind, const cp_config& cfg, const cpc::Bufs& b, const void* actions,         \
                     float* obs_out, float* reward_out, uint8_t* done_out, float* term_out, float* readback,    \
                     int rb_bug, const cpc::Lqr& lq, hipStream_t st);                                            \
    void launch_rollout(bool lat, int kind, const cp_config& cfg, const cpc::Bufs& b, int steps,                 \
                        const void* actions, float* obs_out, float* reward_out, uint8_t* done_out,              \
                        float* term_out, const cpc::Lqr& lq, hipStream_t st);                                   \
    }
CP_DECLARE_LAUNCHES(cp)
CP_DECLARE_LAUNCHES(cp64)
