// cp_kernels.hip — batched cartpole++ env on MI355X (gfx950): kernels + C-ABI.
//
// Replaces bullet_cartpole.py's hot path (BulletCartpole.step/reset and the
// pybullet calls behind them) for B independent envs, two lanes per env (lane
// 2e+p owns contact island p; cp_physics.h).
//
//   cp_step_kernel   R x S substeps fused in one launch; force applied after each
//                    substep (bullet_cartpole.py:199-207); obs at each repeat end
//                    (:237 -> :298-311); steps/done/reward (:239-260).  Finishing
//                    envs are appended to a reset list by wave ballot compaction.
//   cp_reset_kernel  spawn poses, 100 settle + 30 bump substeps (:313-346), over a
//                    compacted list of env ids (dense waves, no idle lanes).
//
// Memory: per-env state is SoA float32 [CP_STATE_FIELDS][B] in HBM (coalesced
// per field); inside a launch the env lives in VGPRs and its contact rows in a
// 20 KiB-per-wave LDS pool (8 waves per CU = 160 KiB).  DESIGN.md §Kernels.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "../../include/cartpole_amd.h"
#include "cp_physics.h"
#include "cp_raster.h"
#include "cp_replay.h"

namespace cp {

// occupancy target of the physics kernels (waves per SIMD); the register budget follows
#ifndef CP_WAVES_PER_EU
#define CP_WAVES_PER_EU 2
#endif
#define CP_PHYS_ATTR __launch_bounds__(WAVE) __attribute__((amdgpu_waves_per_eu(CP_WAVES_PER_EU, CP_WAVES_PER_EU)))

__constant__ float kDiscrete[CP_NUM_DISCRETE][2] = {{0.f, 0.f}, {-1.f, 0.f}, {1.f, 0.f}, {0.f, 1.f}, {0.f, -1.f}};

struct Bufs {
    float* state;      // [CP_STATE_FIELDS][B]
    float* term_obs;   // [R*14][B]
    float* bumps;      // [B][ifs][2][2]
    float* ret_acc;    // [B]
    float* last_ret;   // [B]
    int32_t* last_len; // [B]
    int32_t* overflow; // [B]
    int32_t* list;     // [B] reset list
    int32_t* count;    // reset list length (one of the handle's two counters, by step parity)
    int32_t* count_next;  // the other counter: zeroed by the reset kernel for the next call
    float* scratch;    // [4*CP_ISLAND_PAIRS][2B] manifold headers of the current substep, per lane
    uint64_t* stamps;  // [waves][8] diagnostic phase cycles (CP_STAMPS builds only)
    float* rposes;     // [B][R][4][7] repeat-end poses for the raster obs (NULL: raster off)
    float4* rtable;    // [C][H*W] (d, t_ground) then [C][H*W] uint8 ground class (cp_raster_table_kernel)
    int32_t* rlist;    // [B] envs to render after the step kernel
    int32_t* rcount;   // [1]
    uint8_t* stepped;  // [B] 1 = simulated by the last cp_step (event log: done-before envs are not logged)
};

// raster obs: the repeat-end pose of the 4 bodies (xyz, quat xyzw) for the render kernel
CP_DEV void write_rposes(const Sim& S, float* dst) {
#pragma unroll
    for (int d = 0; d < CP_NUM_DYN; ++d) {
        float* o = dst + d * 7;
        o[0] = S.b[d].x.x; o[1] = S.b[d].x.y; o[2] = S.b[d].x.z;
        o[3] = S.b[d].q[0]; o[4] = S.b[d].q[1]; o[5] = S.b[d].q[2]; o[6] = S.b[d].q[3];
    }
}

// per-wave stamp accumulation into b.stamps (lane 0 writes; CP_STAMPS builds only)
CP_DEV void flush_stamps(const Stamps& ST, uint64_t* dst, uint64_t total) {
#ifdef CP_STAMPS
    if ((threadIdx.x & (WAVE - 1)) == 0) {
        atomicAdd((unsigned long long*)&dst[0], (unsigned long long)ST.narrow);
        atomicAdd((unsigned long long*)&dst[1], (unsigned long long)ST.vel);
        atomicAdd((unsigned long long*)&dst[2], (unsigned long long)ST.solve);
        atomicAdd((unsigned long long*)&dst[3], (unsigned long long)ST.integ);
        atomicAdd((unsigned long long*)&dst[4], (unsigned long long)ST.sweeps);
        atomicAdd((unsigned long long*)&dst[5], (unsigned long long)ST.substeps);
        atomicAdd((unsigned long long*)&dst[6], (unsigned long long)total);
        atomicAdd((unsigned long long*)&dst[7], 1ull);
        if (ST.bb) {  // narrowphase split into the spare slots 8-10
            atomicAdd((unsigned long long*)&dst[8], (unsigned long long)ST.sel);
            atomicAdd((unsigned long long*)&dst[9], (unsigned long long)ST.bb);
            atomicAdd((unsigned long long*)&dst[10], (unsigned long long)ST.rows);
        }
    }
#else
    (void)ST; (void)dst; (void)total;
#endif
}


CP_DEV uint32_t boff(int i) { return (uint32_t)i * 4u; }

CP_DEV void load_sim(Sim& S, const Soa& st, uint32_t o) {
#pragma unroll
    for (int d = 0; d < CP_NUM_DYN; ++d) {
        S.b[d].x = mk(st.ld(CP_SF_BODY(d, 0), o), st.ld(CP_SF_BODY(d, 1), o), st.ld(CP_SF_BODY(d, 2), o));
#pragma unroll
        for (int k = 0; k < 4; ++k) S.b[d].q[k] = st.ld(CP_SF_BODY(d, 3 + k), o);
        S.b[d].v = mk(st.ld(CP_SF_BODY(d, 7), o), st.ld(CP_SF_BODY(d, 8), o), st.ld(CP_SF_BODY(d, 9), o));
        S.b[d].w = mk(st.ld(CP_SF_BODY(d, 10), o), st.ld(CP_SF_BODY(d, 11), o), st.ld(CP_SF_BODY(d, 12), o));
    }
    S.f0 = mk(st.ld(CP_SF_PENDING(0, 0), o), st.ld(CP_SF_PENDING(0, 1), o), st.ld(CP_SF_PENDING(0, 2), o));
    S.f2 = mk(st.ld(CP_SF_PENDING(1, 0), o), st.ld(CP_SF_PENDING(1, 1), o), st.ld(CP_SF_PENDING(1, 2), o));
}

CP_DEV void store_sim(const Sim& S, const Soa& st, uint32_t o) {
#pragma unroll
    for (int d = 0; d < CP_NUM_DYN; ++d) {
        st.st(CP_SF_BODY(d, 0), o, S.b[d].x.x);
        st.st(CP_SF_BODY(d, 1), o, S.b[d].x.y);
        st.st(CP_SF_BODY(d, 2), o, S.b[d].x.z);
#pragma unroll
        for (int k = 0; k < 4; ++k) st.st(CP_SF_BODY(d, 3 + k), o, S.b[d].q[k]);
        st.st(CP_SF_BODY(d, 7), o, S.b[d].v.x);
        st.st(CP_SF_BODY(d, 8), o, S.b[d].v.y);
        st.st(CP_SF_BODY(d, 9), o, S.b[d].v.z);
        st.st(CP_SF_BODY(d, 10), o, S.b[d].w.x);
        st.st(CP_SF_BODY(d, 11), o, S.b[d].w.y);
        st.st(CP_SF_BODY(d, 12), o, S.b[d].w.z);
    }
    st.st(CP_SF_PENDING(0, 0), o, S.f0.x);
    st.st(CP_SF_PENDING(0, 1), o, S.f0.y);
    st.st(CP_SF_PENDING(0, 2), o, S.f0.z);
    st.st(CP_SF_PENDING(1, 0), o, S.f2.x);
    st.st(CP_SF_PENDING(1, 1), o, S.f2.y);
    st.st(CP_SF_PENDING(1, 2), o, S.f2.z);
}

CP_DEV int32_t ldi(const Soa& st, int f, uint32_t o) { return __float_as_int(st.ld(f, o)); }
CP_DEV void sti(const Soa& st, int f, uint32_t o, int32_t v) { st.st(f, o, __int_as_float(v)); }

CP_DEV void write_obs_row(const Sim& S, float* dst) {
    dst[0] = S.b[0].x.x; dst[1] = S.b[0].x.y; dst[2] = S.b[0].x.z;
    dst[3] = S.b[0].q[0]; dst[4] = S.b[0].q[1]; dst[5] = S.b[0].q[2]; dst[6] = S.b[0].q[3];
    dst[7] = S.b[1].x.x; dst[8] = S.b[1].x.y; dst[9] = S.b[1].x.z;
    dst[10] = S.b[1].q[0]; dst[11] = S.b[1].q[1]; dst[12] = S.b[1].q[2]; dst[13] = S.b[1].q[3];
}

// 12-state pole readback (bullet_cartpole.py:212-229)
template <int POLE, int VEL>
CP_DEV void readback_pole(const Sim& S, float* dst) {
    const Body& p = S.b[POLE];
    const Body& vb = S.b[VEL];
    V3 rpy = quat_euler(p.q[0], p.q[1], p.q[2], p.q[3]);
    dst[0] = p.x.x; dst[1] = p.x.y; dst[2] = p.x.z;
    dst[3] = rpy.x; dst[4] = rpy.y; dst[5] = rpy.z;
    dst[6] = vb.v.x; dst[7] = vb.v.y; dst[8] = vb.v.z;
    dst[9] = vb.w.x; dst[10] = vb.w.y; dst[11] = vb.w.z;
}

// ---- closed-loop LQR policy (random_action_agent.py:60-135)
struct Lqr {
    const float* gains;  // [B or 1][2 pairs][2 (fx, fy)][8]
    int per_env;
    float* state8;       // [B][2][R][S][8] or null
    float done_pos;      // _check_done thresholds (:108-119); <= 0: no bounds termination
    float done_angle;
};

// pole 8-state of pair P (:121-135): x - x0, x', y, y', roll, roll', pitch, pitch'
template <int P>
CP_DEV void pole_state8(const Sim& S, float x0, float s[8]) {
    const Body& p = S.b[2 * P + 1];
    const V3 rpy = quat_euler(p.q[0], p.q[1], p.q[2], p.q[3]);
    s[0] = p.x.x - x0; s[1] = p.v.x; s[2] = p.x.y; s[3] = p.v.y;
    s[4] = rpy.x; s[5] = p.w.x; s[6] = rpy.y; s[7] = p.w.y;
}

// u = -K s (:92-95, lqr zero point 0), accumulated k = 0..7 with fma
CP_DEV void lqr_u(const float* K, const float s[8], float& ux, float& uy) {
    float ax = 0.0f, ay = 0.0f;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        ax = fmaf_(K[k], s[k], ax);
        ay = fmaf_(K[8 + k], s[k], ay);
    }
    ux = -ax;
    uy = -ay;
}

CP_DEV bool lqr_out_of_bounds(const float s[8], float pos, float ang) {
    return fabsf(s[0]) > pos || fabsf(s[2]) > pos || fabsf(s[4]) > ang || fabsf(s[6]) > ang;
}

// 8-states of both pairs -> next forces; true if both pairs are out of bounds (:908)
CP_DEV bool lqr_observe(const Sim& S, const cp_config& cfg, const Lqr& q, const float* K, float u[2][2],
                        float* s8_out) {
    float s[8];
    pole_state8<0>(S, cfg.phys.spawn_pos[CP_BODY_POLE][0], s);
    if (s8_out)
        for (int k = 0; k < 8; ++k) s8_out[k] = s[k];
    lqr_u(K, s, u[0][0], u[0][1]);
    const bool out0 = lqr_out_of_bounds(s, q.done_pos, q.done_angle);
    pole_state8<1>(S, cfg.phys.spawn_pos[CP_BODY_POLE2][0], s);
    if (s8_out)
        for (int k = 0; k < 8; ++k) s8_out[k + 8] = s[k];
    lqr_u(K + 16, s, u[1][0], u[1][1]);
    const bool out1 = lqr_out_of_bounds(s, q.done_pos, q.done_angle);
    return q.done_pos > 0.0f && out0 && out1;
}

// commented-out bounds check of the reference (:243-253), on the pole pose
CP_DEV bool bounds_exceeded(const Sim& S, const cp_config& cfg) {
    const Body& p = S.b[1];
    if (fabsf(p.x.x) > cfg.pos_threshold || fabsf(p.x.y) > cfg.pos_threshold) return true;
    float qx = p.q[0], qy = p.q[1], qz = p.q[2], qw = p.q[3];
    float Y = 2.0f * fmaf_(qy, qz, qw * qx);
    float X = ((qw * qw - qx * qx) - qy * qy) + qz * qz;
    bool roll_out = (X > 0.0f) ? (fabsf(Y) > X * cfg.tan_angle_threshold) : !(X == 0.0f && Y == 0.0f);
    float sarg = -2.0f * fmaf_(qx, qz, -(qw * qy));
    bool pitch_out = fabsf(sarg) > cfg.sin_angle_threshold;
    return roll_out || pitch_out;
}

// Bump force k on cart C (LINK frame), bullet_cartpole.py:354-359
CP_DEV void bump_force(const cp_config& cfg, const float* bumps, int i, int episode, int k, int c, float& fx,
                       float& fy) {
    if (cfg.bump_mode == CP_BUMP_HOST) {
        const float* f = bumps + (((size_t)i * cfg.initial_force_steps + k) * 2 + c) * 2;
        fx = f[0];
        fy = f[1];
        return;
    }
    const float F = cfg.initial_force;
    if (!cfg.random_theta) {
        fx = F;
        fy = F * 0.0f;
        return;
    }
    uint32_t idx = (uint32_t)(2 * k + c);
    uint64_t gid = (uint64_t)(cfg.env_id_offset + i);
    uint32_t w = philox_word(idx >> 2, (uint32_t)episode, (uint32_t)gid, (uint32_t)(gid >> 32), (uint32_t)cfg.seed,
                             (uint32_t)(cfg.seed >> 32), (int)(idx & 3u));
    float u = (float)(w >> 8) * 5.9604644775390625e-08f;
    float s, co;
    sincos_turns(u, s, co);
    fx = F * co;
    fy = F * s;
}

// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) cp_init_kernel(cp_config cfg, Bufs b) {
    const int B = cfg.num_envs;
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= B) return;
    const Soa st = Soa::make(b.state, B, CP_STATE_FIELDS);
    const uint32_t o = boff(i);
    for (int f = 0; f < CP_STATE_FIELDS; ++f) st.st(f, o, 0.0f);
#pragma unroll
    for (int d = 0; d < CP_NUM_DYN; ++d) {
#pragma unroll
        for (int k = 0; k < 3; ++k) st.st(CP_SF_BODY(d, k), o, cfg.phys.spawn_pos[d + 1][k]);
        st.st(CP_SF_BODY(d, 6), o, 1.0f);
    }
#pragma unroll
    for (int p = 0; p < CP_NUM_ISLANDS; ++p)
#pragma unroll
        for (int j = 0; j < CP_ISLAND_PAIRS; ++j) sti(st, CP_SF_WS_ID(p, j), o, -1);
    sti(st, CP_SF_DONE, o, 1);  // not reset yet: reference raises, batched API reports done
    b.ret_acc[i] = 0.0f;
    b.last_ret[i] = 0.0f;
    b.last_len[i] = 0;
    b.overflow[i] = 0;
}

// env_mask -> compacted list (wave ballot + one atomic per wave)
__global__ void __launch_bounds__(256) cp_mask_to_list_kernel(int B, const uint8_t* mask, int32_t* list,
                                                               int32_t* count) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    bool want = i < B && (mask == nullptr || mask[i] != 0);
    uint64_t bal = __ballot(want);
    int lane = threadIdx.x & (WAVE - 1);
    int n = __popcll(bal);
    int base = 0;
    if (lane == 0 && n) base = atomicAdd(count, n);
    base = __shfl(base, 0);
    if (want) list[base + __popcll(bal & ((1ull << lane) - 1ull))] = i;
}

// LAT = false: the throughput shape of the step kernel (2 waves per SIMD), for reset bursts
// (fixed-length episodes end together).  LAT = true: one wave per SIMD with 512 registers and
// fast-form rows, for the short lists of desynchronised episodes (bounds termination), where
// the 130 serial substeps of one wave are the whole latency of the step.
template <bool LAT>
__global__ void __launch_bounds__(WAVE)
__attribute__((amdgpu_waves_per_eu(LAT ? 1 : CP_WAVES_PER_EU, LAT ? 1 : CP_WAVES_PER_EU)))
cp_reset_kernel(cp_config cfg, Bufs b, float* obs_out) {
    __shared__ float lds_pool[POOL_FLOATS * WAVE];
    const int B = cfg.num_envs;
    const int t = blockIdx.x * WAVE + threadIdx.x;
    if (t == 0 && b.count_next) *b.count_next = 0;  // the next cp_step's list starts empty
    const int n = *b.count;
    if ((t >> 1) >= n) return;  // lane pairs past the compacted list
    const int isl = t & 1;
    const bool lead = isl == 0;
    const int i = b.list[t >> 1];
    float* pool = lds_pool + threadIdx.x;
    float* pool0 = lds_pool + (threadIdx.x & ~1u);
    const Mem G = Mem::make(b.state, b.scratch, B, i, isl);
    const Lane L = Lane::make(isl, cfg.phys);
    Stamps ST;
    Sim S;
    load_sim(S, G.st, G.off);  // pending forces survive the reset (pybullet keeps them)
    const int episode = ldi(G.st, CP_SF_EPISODE, G.off);
#pragma unroll
    for (int d = 0; d < CP_NUM_DYN; ++d) {
        S.b[d].x = mk(cfg.phys.spawn_pos[d + 1][0], cfg.phys.spawn_pos[d + 1][1], cfg.phys.spawn_pos[d + 1][2]);
        S.b[d].q[0] = 0.0f; S.b[d].q[1] = 0.0f; S.b[d].q[2] = 0.0f; S.b[d].q[3] = 1.0f;
        S.b[d].v = mk(0.0f, 0.0f, 0.0f);
        S.b[d].w = mk(0.0f, 0.0f, 0.0f);
    }
#pragma unroll
    for (int j = 0; j < CP_ISLAND_PAIRS; ++j) {  // the lane's island's warm-start cache
        G.sw(CP_SF_WS_ID(0, j), __int_as_float(-1));
#pragma unroll
        for (int k = 0; k < 4; ++k) G.sl(CP_SF_WS_LAM(0, j, k), 0.0f);
    }
    int ov = 0;
    const int nsub = cfg.settle_steps + cfg.initial_force_steps;
    for (int s = 0; s < nsub; ++s) {
        substep<LAT>(S, cfg.phys, L, pool, pool0, ov, G, ST);
        const int k = s - cfg.settle_steps;
        if (k >= 0) {
            float fx, fy;
            bump_force(cfg, b.bumps, i, episode, k, 0, fx, fy);
            apply_force_link<0>(S, fx, fy);
            bump_force(cfg, b.bumps, i, episode, k, 1, fx, fy);
            apply_force_link<1>(S, fx, fy);
        }
    }
    ov += (int)partner_u((uint32_t)ov);
    if (!lead) return;
    store_sim(S, G.st, G.off);
    b.overflow[i] += ov;
    float row[14];
    write_obs_row(S, row);
    const int R = cfg.action_repeats;
    if (b.rposes)  // every repeat slot shows the reset pose (bullet_cartpole.py:342-345)
        for (int r = 0; r < R; ++r) write_rposes(S, b.rposes + ((size_t)i * R + r) * CP_NUM_DYN * 7);
    float* o = obs_out + (size_t)i * R * 14;
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int f = 0; f < 14; ++f) o[r * 14 + f] = row[f];
    sti(G.st, CP_SF_STEPS, G.off, 0);
    sti(G.st, CP_SF_DONE, G.off, 0);
    sti(G.st, CP_SF_EPISODE, G.off, episode + 1);
    b.ret_acc[i] = 0.0f;
}

// LAT: the latency shape of cp_reset_kernel<true> (1 wave per SIMD, 512 registers, fast-form
// rows) for batches whose waves all get a SIMD of their own (<= 32,768 envs)
template <int KIND, bool LQR, bool LAT>
__global__ void __launch_bounds__(WAVE)
__attribute__((amdgpu_waves_per_eu(LAT ? 1 : CP_WAVES_PER_EU, LAT ? 1 : CP_WAVES_PER_EU)))
cp_step_kernel(cp_config cfg, Bufs b, const void* actions, float* obs_out, float* reward_out, uint8_t* done_out,
               float* term_out, float* readback, int rb_bug, Lqr lq) {
    __shared__ float lds_pool[POOL_FLOATS * WAVE];
    const int B = cfg.num_envs;
    const int t = blockIdx.x * WAVE + threadIdx.x;
    const int i = t >> 1, isl = t & 1;
    const bool lead = isl == 0;  // lane 0 of the pair writes the env's outputs
    const bool inb = i < B;
    const int R = cfg.action_repeats, SR = cfg.steps_per_repeat;
    float* pool = lds_pool + threadIdx.x;
    float* pool0 = lds_pool + (threadIdx.x & ~1u);
    bool want_reset = false;
    bool render_me = false;  // simulated this step: its frames go to the render kernel
    Stamps ST;
    CP_STAMP(k0);
    if (inb) {
        const Mem G = Mem::make(b.state, b.scratch, B, i, isl);
        const Lane L = Lane::make(isl, cfg.phys);
        const Soa term = Soa::make(b.term_obs, B, R * 14);
        float* obs = obs_out + (size_t)i * R * 14;
        const bool was_done = ldi(G.st, CP_SF_DONE, G.off) != 0;
        if (lead) b.stepped[i] = was_done ? 0 : 1;
        if (was_done) {  // step after done (bullet_cartpole.py:179-181)
            if (lead) {
                for (int f = 0; f < R * 14; ++f) obs[f] = term.ld(f, G.off);
                reward_out[i] = 0.0f;
                done_out[i] = 1;
            }
        } else {
            float a00, a01, a10, a11;
            if constexpr (KIND == CP_ACTION_CONTINUOUS) {
                const float4 a = reinterpret_cast<const float4*>(actions)[i];
                a00 = a.x; a01 = a.y; a10 = a.z; a11 = a.w;
            } else {
                const char2 a = reinterpret_cast<const char2*>(actions)[i];
                int k0 = a.x, k1 = a.y;
                k0 = (k0 < 0 || k0 >= CP_NUM_DISCRETE) ? 0 : k0;
                k1 = (k1 < 0 || k1 >= CP_NUM_DISCRETE) ? 0 : k1;
                a00 = kDiscrete[k0][0]; a01 = kDiscrete[k0][1];
                a10 = kDiscrete[k1][0]; a11 = kDiscrete[k1][1];
            }
            const float F = cfg.action_force;
            const float f00 = a00 * F, f01 = a01 * F, f10 = a10 * F, f11 = a11 * F;
            Sim S;
            load_sim(S, G.st, G.off);
            int ov = 0;
            float u[2][2] = {{0.0f, 0.0f}, {0.0f, 0.0f}};  // LQR forces from the last observed state
            bool lqr_done = false;
            const float* K = nullptr;
            if constexpr (LQR) {
                K = lq.gains + (lq.per_env ? (size_t)i * 32 : 0);
                lqr_observe(S, cfg, lq, K, u, nullptr);
            }
            for (int r = 0; r < R; ++r) {
                for (int s = 0; s < SR; ++s) {
                    substep<LAT>(S, cfg.phys, L, pool, pool0, ov, G, ST);
                    if constexpr (LQR) {  // disturbance + control (:897-901), control from the pre-step state
                        apply_force_link<0>(S, f00 + u[0][0], f01 + u[0][1]);
                        apply_force_link<1>(S, f10 + u[1][0], f11 + u[1][1]);
                        float* s8 = (lq.state8 && lead) ? lq.state8 + (((size_t)i * R + r) * SR + s) * 16 : nullptr;
                        lqr_done |= lqr_observe(S, cfg, lq, K, u, s8);
                    } else {
                        apply_force_link<0>(S, f00, f01);
                        apply_force_link<1>(S, f10, f11);
                    }
                    if (readback && lead) {
                        float* rb = readback + (size_t)i * 2 * R * SR * 12;
                        readback_pole<1, 1>(S, rb + ((size_t)(0 * R + r) * SR + s) * 12);
                        if (rb_bug) readback_pole<3, 1>(S, rb + ((size_t)(1 * R + r) * SR + s) * 12);
                        else readback_pole<3, 3>(S, rb + ((size_t)(1 * R + r) * SR + s) * 12);
                    }
                }
                if (lead) {
                    float row[14];
                    write_obs_row(S, row);
#pragma unroll
                    for (int f = 0; f < 14; ++f) obs[r * 14 + f] = row[f];
                    if (b.rposes) write_rposes(S, b.rposes + ((size_t)i * R + r) * CP_NUM_DYN * 7);
                }
            }
            render_me = lead && b.rposes != nullptr;
            ov += (int)partner_u((uint32_t)ov);
            if (ov && lead) b.overflow[i] += ov;
            const int steps = ldi(G.st, CP_SF_STEPS, G.off) + 1;
            bool done = steps >= cfg.max_episode_len;
            if (cfg.done_on_bounds && bounds_exceeded(S, cfg)) done = true;
            if (LQR && lqr_done) done = true;
            if (lead) {
                store_sim(S, G.st, G.off);
                sti(G.st, CP_SF_STEPS, G.off, steps);
                reward_out[i] = 1.0f;  // bullet_cartpole.py:260
                done_out[i] = done ? 1 : 0;
                const float ret = b.ret_acc[i] + 1.0f;
                if (done) {
                    b.last_ret[i] = ret;
                    b.last_len[i] = steps;
                    b.ret_acc[i] = 0.0f;
                    for (int f = 0; f < R * 14; ++f) term.st(f, G.off, obs[f]);
                    if (term_out)
                        for (int f = 0; f < R * 14; ++f) term_out[(size_t)i * R * 14 + f] = obs[f];
                    sti(G.st, CP_SF_DONE, G.off, 1);
                    want_reset = cfg.autoreset != 0;
                } else {
                    b.ret_acc[i] = ret;
                }
            }
        }
    }
#ifdef CP_STAMPS
    CP_STAMP(k1);
    flush_stamps(ST, b.stamps, k1 - k0);
#endif
    if (cfg.autoreset) {
        // wave ballot compaction of the finishing envs into the reset list
        const uint64_t bal = __ballot(want_reset);
        const int lane = threadIdx.x;  // want_reset is set on lead lanes only
        const int n = __popcll(bal);
        int base = 0;
        if (lane == 0 && n) base = atomicAdd(b.count, n);
        base = __shfl(base, 0);
        if (want_reset) b.list[base + __popcll(bal & ((1ull << lane) - 1ull))] = i;
    }
    if (b.rposes) {
        const uint64_t bal = __ballot(render_me);
        const int lane = threadIdx.x & (WAVE - 1);
        const int n = __popcll(bal);
        int base = 0;
        if (lane == 0 && n) base = atomicAdd(b.rcount, n);
        base = __shfl(base, 0);
        if (render_me) b.rlist[base + __popcll(bal & ((1ull << lane) - 1ull))] = i;
    }
}

// ---------------------------------------------------------------------------
// Event log records (protobuf wire format of event.proto; see cp_encode_events).
CP_DEV void put_u8(uint8_t*& p, uint32_t v) { *p++ = (uint8_t)v; }
CP_DEV void put_varint(uint8_t*& p, uint32_t v) {
    while (v >= 0x80u) { put_u8(p, (v & 0x7Fu) | 0x80u); v >>= 7; }
    put_u8(p, v);
}
CP_DEV void put_f32(uint8_t*& p, uint32_t key, float x) {  // fixed32 field, little endian
    put_u8(p, key);
    const uint32_t u = __float_as_uint(x);
    put_u8(p, u); put_u8(p, u >> 8); put_u8(p, u >> 16); put_u8(p, u >> 24);
}
__host__ __device__ inline int varint_len(uint32_t v) { int n = 1; while (v >= 0x80u) { v >>= 7; ++n; } return n; }
__host__ __device__ inline int event_len(int kind, int R, int with_action) {
    // State: 7 cart_pose + 7 pole_pose fixed32 fields = 70 B, wrapped (tag, len 70) = 72 B
    return (with_action ? (kind == CP_ACTION_CONTINUOUS ? 4 : 2) * 5 + 5 : 0) + R * 72;
}
__host__ __device__ inline int record_len(int kind, int R, int with_action) {
    const int n = event_len(kind, R, with_action);
    return 1 + varint_len((uint32_t)n) + n;
}
// one Episode.event entry: tag 1 (length-delimited), Event { action*, state*, reward }
CP_DEV void put_record(uint8_t* p, int kind, int R, bool with_action, const void* actions, int i, const float* obs,
                       float reward) {
    put_u8(p, 0x0A);
    put_varint(p, (uint32_t)event_len(kind, R, with_action ? 1 : 0));
    if (with_action) {
        if (kind == CP_ACTION_CONTINUOUS) {
            const float* a = reinterpret_cast<const float*>(actions) + (size_t)i * 4;
            for (int k = 0; k < 4; ++k) put_f32(p, 0x0D, a[k]);
        } else {
            const int8_t* a = reinterpret_cast<const int8_t*>(actions) + (size_t)i * 2;
            put_f32(p, 0x0D, (float)a[0]);
            put_f32(p, 0x0D, (float)a[1]);
        }
    }
    for (int r = 0; r < R; ++r) {
        put_u8(p, 0x12);
        put_u8(p, 70);
        const float* o = obs + ((size_t)i * R + r) * 14;
        for (int k = 0; k < 7; ++k) put_f32(p, 0x0D, o[k]);       // cart_pose = 1
        for (int k = 0; k < 7; ++k) put_f32(p, 0x15, o[7 + k]);   // pole_pose = 2
    }
    if (with_action) put_f32(p, 0x1D, reward);                    // reward = 3
}

__global__ void __launch_bounds__(256) cp_event_kernel(int B, int R, int mode, int kind, int autoreset,
                                                        const void* actions, const float* obs, const float* term,
                                                        const float* reward, const uint8_t* done,
                                                        const uint8_t* mask, const uint8_t* stepped,
                                                        uint8_t* step_rec, uint8_t* reset_rec, uint8_t* flags) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= B) return;
    const int sb = record_len(kind, R, 1), rb = record_len(kind, R, 0);
    uint8_t fl = 0;
    if (mode == 0) {
        if (stepped[i]) {
            fl = 1;
            const bool fresh = autoreset && done[i];   // finished and auto-reset in that cp_step
            put_record(step_rec + (size_t)i * sb, kind, R, true, actions, i, fresh && term ? term : obs,
                       reward[i]);
            if (fresh && reset_rec) {
                fl |= 2;
                put_record(reset_rec + (size_t)i * rb, kind, R, false, nullptr, i, obs, 0.0f);
            }
        }
    } else if (!mask || mask[i]) {
        fl = 2;
        put_record(reset_rec + (size_t)i * rb, kind, R, false, nullptr, i, obs, 0.0f);
    }
    flags[i] = fl;
}

__global__ void __launch_bounds__(256) cp_copy_kernel(const float* src, float* dst, size_t n) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) dst[i] = src[i];
}

}  // namespace cp

// ============================================================================ C-ABI
struct cp_timing {
    int cap = 0;                             // event pairs per kind
    int nstep = 0, nreset = 0, nrender = 0;  // pairs recorded
    int stride[3] = {1, 1, 1};               // record every stride-th launch of a kind
    int seen[3] = {0, 0, 0};                 // launches of a kind since cp_timing_begin
    double render_ms = 0.0;                  // summed by cp_timing_end
    int render_launches = 0;
    std::vector<hipEvent_t> ev;  // [0, 2cap): step pairs, [2cap, 4cap): reset, [4cap, 6cap): render
};

struct cp_handle {
    cp_config cfg;
    int device;
    cp::Bufs b;
    float* readback;
    int readback_bug;
    cp::Lqr lqr;
    cp_timing timing;
    cp_raster_config raster;
    uint16_t* pixels;  // raster obs output (NULL: raster off)
    int32_t* count2;   // [2] reset-list counters, alternating by call: each reset launch zeroes the other one
    int par;           // counter the next call appends to
    int reset_lat;     // 1: latency-shaped autoreset kernel (episodes end at different steps)
    int step_lat;      // 1: latency-shaped step kernel (every wave gets a SIMD of its own)
    std::string err;
};

static void choose_reset_shape(cp_handle* h);

static void timing_free(cp_timing& t) {
    for (hipEvent_t e : t.ev) (void)hipEventDestroy(e);
    t.ev.clear();
    t.cap = t.nstep = t.nreset = t.nrender = 0;
    for (int k = 0; k < 3; ++k) t.stride[k] = 1, t.seen[k] = 0;
}
// returns the event pair to record around a launch of `kind` (0 step, 1 reset, 2 render), or nullptr
static hipEvent_t* timing_slot(cp_handle* h, int kind) {
    cp_timing& t = h->timing;
    if (t.cap == 0) return nullptr;
    if (t.seen[kind]++ % t.stride[kind] != 0) return nullptr;
    int& n = kind == 0 ? t.nstep : (kind == 1 ? t.nreset : t.nrender);
    if (n >= (kind == 2 ? 2 * t.cap : t.cap)) return nullptr;  // up to 2 render launches per step
    hipEvent_t* p = &t.ev[(size_t)(kind * t.cap + n) * 2];
    ++n;
    return p;
}

static thread_local std::string g_err;

static int fail(cp_handle* h, const std::string& msg) {
    if (h) h->err = msg;
    g_err = msg;
    return -1;
}
static int check(cp_handle* h, hipError_t e, const char* what) {
    if (e != hipSuccess) return fail(h, std::string(what) + ": " + hipGetErrorString(e));
    return 0;
}
#define CP_TRY(h, call)                                   \
    do {                                                  \
        if (check((h), (call), #call)) return -1;         \
    } while (0)

static inline unsigned grid_for(int n, int block) { return (unsigned)((n + block - 1) / block); }

extern "C" {

int cp_abi_version(void) { return CP_ABI_VERSION; }

void cp_default_config(cp_config* c) {
    std::memset(c, 0, sizeof(*c));
    c->num_envs = 1;
    c->action_repeats = 2;       // bullet_cartpole.py:23
    c->steps_per_repeat = 1;     // :25
    c->max_episode_len = 200;    // :31
    c->action_force = 50.0f;     // :18
    c->initial_force = 200.0f;   // :20
    c->random_theta = 1;         // :22
    c->initial_force_steps = 30; // :76
    c->settle_steps = 100;       // :326
    c->done_on_bounds = 0;       // :243-253 are commented out in the fork
    c->pos_threshold = 3.0f;     // :58
    c->angle_threshold = 0.35f;  // :62
    c->tan_angle_threshold = (float)std::tan((double)0.35f);
    c->sin_angle_threshold = (float)std::sin((double)0.35f);
    c->autoreset = 0;
    c->bump_mode = CP_BUMP_PHILOX;
    c->seed = 0;
    c->env_id_offset = 0;
    cp_physics* p = &c->phys;
    p->dt = (float)(1.0 / 240.0);
    p->inv_dt = 240.0f;
    p->gravity[0] = 0.0f;
    p->gravity[1] = 0.0f;
    p->gravity[2] = -9.81f;  // :152
    p->lin_damping = 0.04f;
    p->ang_damping = 0.04f;
    p->erp = 0.2f;
    p->contact_margin = 0.02f;
    p->residual_threshold = 1e-7f;
    p->solver_iterations = 50;
    p->edge_bias = 1e-4f;
    p->max_angular_step = (float)(0.25 * 3.141592653589793);
    p->warmstart = 0.85f;
    // models/ground.urdf, cart.urdf, pole.urdf, cart2.urdf, pole2.urdf
    static const double he[5][3] = {{1.5, 1.5, 0.05}, {0.1, 0.1, 0.025}, {0.005, 0.005, 0.25},
                                    {0.1, 0.1, 0.025}, {0.005, 0.005, 0.25}};
    static const double mass[5] = {0.0, 1.0, 5.0, 1.0, 5.0};
    static const double inert[5][3] = {{0, 0, 0},
                                       {0.0035416666666, 0.0035416666666, 0.0066666666666},
                                       {0.104208333333333, 0.104208333333333, 0.00008333333333},
                                       {0.0035416666666, 0.0035416666666, 0.0066666666666},
                                       {0.104208333333333, 0.104208333333333, 0.00008333333333}};
    static const double mu[5] = {0.5, 0.0, 1.0, 0.0, 1.0};
    static const double spawn[5][3] = {{0, 0, 0}, {0, 0, 0.08}, {0, 0, 0.35}, {1, 0, 0.08}, {1, 0, 0.35}};
    for (int b = 0; b < 5; ++b) {
        for (int k = 0; k < 3; ++k) {
            p->half_extents[b][k] = (float)he[b][k];
            p->inertia[b][k] = (float)inert[b][k];
            p->inv_inertia[b][k] = inert[b][k] > 0 ? (float)(1.0 / inert[b][k]) : 0.0f;
            p->spawn_pos[b][k] = (float)spawn[b][k];
        }
        p->inv_mass[b] = mass[b] > 0 ? (float)(1.0 / mass[b]) : 0.0f;
        p->friction[b] = (float)mu[b];
    }
}

const char* cp_last_error(const cp_handle* h) { return h ? h->err.c_str() : g_err.c_str(); }

int cp_create(const cp_config* cfg, int device, cp_handle** out) {
    if (!cfg || !out) return fail(nullptr, "cp_create: null argument");
    if (cfg->num_envs <= 0) return fail(nullptr, "cp_create: num_envs must be > 0");
    if (cfg->action_repeats <= 0 || cfg->steps_per_repeat <= 0)
        return fail(nullptr, "cp_create: action_repeats and steps_per_repeat must be > 0");
    if (cfg->initial_force_steps < 0 || cfg->settle_steps < 0)
        return fail(nullptr, "cp_create: negative step counts");
    if (cfg->phys.solver_iterations < 0) return fail(nullptr, "cp_create: negative solver_iterations");
    // host-computed derived fields must agree with their sources (the kernels use both)
    if (!(cfg->phys.dt > 0.0f) || std::fabs((double)cfg->phys.dt * (double)cfg->phys.inv_dt - 1.0) > 1e-6)
        return fail(nullptr, "cp_create: phys.inv_dt must be 1 / phys.dt (recompute it when dt changes)");
    if (std::fabs((double)cfg->tan_angle_threshold - std::tan((double)cfg->angle_threshold)) > 1e-6 ||
        std::fabs((double)cfg->sin_angle_threshold - std::sin((double)cfg->angle_threshold)) > 1e-6)
        return fail(nullptr, "cp_create: tan/sin_angle_threshold must be tan/sin(angle_threshold)");
    if (!(cfg->phys.residual_threshold >= 0.0f)) return fail(nullptr, "cp_create: negative residual_threshold");
    if ((unsigned long long)cfg->num_envs * CP_STATE_FIELDS * 4ull >= (1ull << 32) ||
        (unsigned long long)cfg->num_envs * cfg->action_repeats * 14ull * 4ull >= (1ull << 32))
        return fail(nullptr, "cp_create: num_envs too large for one handle (SoA arrays must stay below 4 GiB)");
    cp_handle* h = new (std::nothrow) cp_handle();
    if (!h) return fail(nullptr, "cp_create: out of memory");
    h->cfg = *cfg;
    h->device = device;
    h->readback = nullptr;
    h->readback_bug = 1;
    h->lqr = cp::Lqr{nullptr, 0, nullptr, 0.0f, 0.0f};
    h->pixels = nullptr;
    choose_reset_shape(h);
    cp_default_raster_config(&h->raster);
    std::memset(&h->b, 0, sizeof(h->b));
    const size_t B = (size_t)cfg->num_envs;
    const int R = cfg->action_repeats;
    auto fail_free = [&](hipError_t e, const char* what) {
        std::string msg = std::string(what) + ": " + hipGetErrorString(e);
        cp_destroy(h);
        return fail(nullptr, msg);
    };
    hipError_t e = hipSetDevice(device);
    if (e != hipSuccess) return fail_free(e, "hipSetDevice");
#define CP_ALLOC(ptr, bytes)                                   \
    e = hipMalloc((void**)&(ptr), (bytes));                    \
    if (e != hipSuccess) return fail_free(e, "hipMalloc " #ptr);
    CP_ALLOC(h->b.state, (size_t)CP_STATE_FIELDS * B * sizeof(float));
    CP_ALLOC(h->b.term_obs, (size_t)R * 14 * B * sizeof(float));
    CP_ALLOC(h->b.bumps, B * (size_t)(cfg->initial_force_steps > 0 ? cfg->initial_force_steps : 1) * 4 * sizeof(float));
    CP_ALLOC(h->b.ret_acc, B * sizeof(float));
    CP_ALLOC(h->b.last_ret, B * sizeof(float));
    CP_ALLOC(h->b.last_len, B * sizeof(int32_t));
    CP_ALLOC(h->b.overflow, B * sizeof(int32_t));
    CP_ALLOC(h->b.list, B * sizeof(int32_t));
    CP_ALLOC(h->count2, 2 * sizeof(int32_t));
    CP_ALLOC(h->b.scratch, (size_t)4 * CP_ISLAND_PAIRS * 2 * B * sizeof(float));
    CP_ALLOC(h->b.stamps, 16 * sizeof(uint64_t));
    CP_ALLOC(h->b.stepped, B * sizeof(uint8_t));
#undef CP_ALLOC
    e = hipMemset(h->count2, 0, 2 * sizeof(int32_t));
    if (e != hipSuccess) return fail_free(e, "hipMemset");
    h->b.count = h->count2;
    h->b.count_next = nullptr;
    e = hipMemset(h->b.stepped, 0, B * sizeof(uint8_t));
    if (e != hipSuccess) return fail_free(e, "hipMemset");
    e = hipMemset(h->b.stamps, 0, 16 * sizeof(uint64_t));
    if (e != hipSuccess) return fail_free(e, "hipMemset");
    e = hipMemset(h->b.term_obs, 0, (size_t)R * 14 * B * sizeof(float));
    if (e != hipSuccess) return fail_free(e, "hipMemset");
    e = hipMemset(h->b.bumps, 0, B * (size_t)(cfg->initial_force_steps > 0 ? cfg->initial_force_steps : 1) * 4 * sizeof(float));
    if (e != hipSuccess) return fail_free(e, "hipMemset");
    hipLaunchKernelGGL(cp::cp_init_kernel, dim3(grid_for((int)B, 256)), dim3(256), 0, 0, h->cfg, h->b);
    e = hipGetLastError();
    if (e != hipSuccess) return fail_free(e, "cp_init_kernel");
    e = hipDeviceSynchronize();
    if (e != hipSuccess) return fail_free(e, "hipDeviceSynchronize");
    *out = h;
    return 0;
}

void cp_destroy(cp_handle* h) {
    if (!h) return;
    (void)hipSetDevice(h->device);
    timing_free(h->timing);
    (void)hipFree(h->b.state);
    (void)hipFree(h->b.term_obs);
    (void)hipFree(h->b.bumps);
    (void)hipFree(h->b.ret_acc);
    (void)hipFree(h->b.last_ret);
    (void)hipFree(h->b.last_len);
    (void)hipFree(h->b.overflow);
    (void)hipFree(h->b.list);
    (void)hipFree(h->count2);
    (void)hipFree(h->b.scratch);
    (void)hipFree(h->b.stamps);
    (void)hipFree(h->b.stepped);
    (void)hipFree(h->b.rposes);
    (void)hipFree(h->b.rlist);
    (void)hipFree(h->b.rcount);
    (void)hipFree(h->b.rtable);
    delete h;
}

// raster obs of the envs in list[0 .. *count) (a device count: the grid covers B)
static int launch_render(cp_handle* h, const int32_t* list, const int32_t* count, hipStream_t st) {
    hipEvent_t* ev = timing_slot(h, 2);
    if (ev) CP_TRY(h, hipEventRecord(ev[0], st));
    const int C = h->raster.num_cameras, R = h->cfg.action_repeats, npx = h->raster.width * h->raster.height;
    const uint8_t* cls = reinterpret_cast<const uint8_t*>(h->b.rtable + (size_t)C * npx);
    const size_t small = (size_t)cp::render_small_lds(C, R, npx).total;
    if (small <= (size_t)cp::SMALL_LDS_MAX) {  // one block per env, dense ray tests
        hipLaunchKernelGGL(cp::cp_render_small_kernel, dim3((unsigned)h->cfg.num_envs),
                           dim3(cp::RENDER_WAVES * cp::WAVE_R), small, st, h->raster, h->cfg.phys, R, list, count,
                           h->b.rposes, h->b.rtable, cls, h->pixels);
    } else {  // large frames: one wave per env
        const size_t lds = (size_t)cp::RENDER_WAVES * cp::render_lds(C, R).total;
        const unsigned grid = (unsigned)((h->cfg.num_envs + cp::RENDER_WAVES - 1) / cp::RENDER_WAVES);
        hipLaunchKernelGGL(cp::cp_render_kernel, dim3(grid), dim3(cp::RENDER_WAVES * cp::WAVE_R), lds, st, h->raster,
                           h->cfg.phys, R, list, count, h->b.rposes, h->b.rtable, cls, h->pixels);
    }
    if (check(h, hipGetLastError(), "cp_render_kernel")) return -1;
    if (ev) CP_TRY(h, hipEventRecord(ev[1], st));
    return 0;
}

// the reset list's counter for this call: the one the previous call's reset launch zeroed
static void use_counter(cp_handle* h) {
    h->b.count = h->count2 + h->par;
    h->b.count_next = h->count2 + (h->par ^ 1);
    h->par ^= 1;
}

// Which autoreset kernel shape (cp_reset_kernel<LAT>): episodes that can end early (bounds
// termination, LQR done thresholds) end at different steps, so every step resets a short list
// and its latency is the step's; fixed-length episodes end together in bursts (throughput),
// except in batches small enough that a burst fits one wave per SIMD.
// The step kernel has the same two shapes, chosen by batch size alone.  CP_RESET_LATENCY=0/1 and
// CP_STEP_LATENCY=0/1 override (diagnostics).
static void choose_reset_shape(cp_handle* h) {
    const bool lqr_done = h->lqr.gains && (h->lqr.done_pos > 0.0f || h->lqr.done_angle > 0.0f);
    // up to 32,768 envs every wave gets a SIMD of its own even in a full burst (1,024 SIMDs), so
    // the latency shape is never the slower one there
    const bool small = h->cfg.num_envs <= 32768;
    const char* e = std::getenv("CP_RESET_LATENCY");
    h->reset_lat = (e && (e[0] == '0' || e[0] == '1')) ? e[0] == '1' : (h->cfg.done_on_bounds || lqr_done || small);
    const char* es = std::getenv("CP_STEP_LATENCY");
    h->step_lat = (es && (es[0] == '0' || es[0] == '1')) ? es[0] == '1' : small;
}

static int launch_reset_from_list(cp_handle* h, float* obs_out, hipStream_t st, bool render) {
    const int B = h->cfg.num_envs;
    hipEvent_t* ev = timing_slot(h, 1);
    if (ev) CP_TRY(h, hipEventRecord(ev[0], st));
    if (h->reset_lat)
        hipLaunchKernelGGL(cp::cp_reset_kernel<true>, dim3(grid_for(2 * B, cp::WAVE)), dim3(cp::WAVE), 0, st, h->cfg,
                           h->b, obs_out);
    else
        hipLaunchKernelGGL(cp::cp_reset_kernel<false>, dim3(grid_for(2 * B, cp::WAVE)), dim3(cp::WAVE), 0, st, h->cfg,
                           h->b, obs_out);
    if (check(h, hipGetLastError(), "cp_reset_kernel")) return -1;
    if (ev) CP_TRY(h, hipEventRecord(ev[1], st));
    if (render && h->pixels) return launch_render(h, h->b.list, h->b.count, st);
    return 0;
}

int cp_reset(cp_handle* h, const uint8_t* env_mask, float* obs_out, void* stream) {
    if (!h || !obs_out) return fail(h, "cp_reset: null argument");
    hipStream_t st = (hipStream_t)stream;
    const int B = h->cfg.num_envs;
    CP_TRY(h, hipSetDevice(h->device));
    use_counter(h);
    CP_TRY(h, hipMemsetAsync(h->b.count, 0, sizeof(int32_t), st));
    hipLaunchKernelGGL(cp::cp_mask_to_list_kernel, dim3(grid_for(B, 256)), dim3(256), 0, st, B, env_mask, h->b.list,
                       h->b.count);
    CP_TRY(h, hipGetLastError());
    return launch_reset_from_list(h, obs_out, st, true);
}

int cp_step(cp_handle* h, const void* actions, int action_kind, float* obs_out, float* reward_out,
            uint8_t* done_out, float* terminal_obs_out, void* stream) {
    if (!h || !actions || !obs_out || !reward_out || !done_out) return fail(h, "cp_step: null argument");
    if (action_kind != CP_ACTION_CONTINUOUS && action_kind != CP_ACTION_DISCRETE)
        return fail(h, "cp_step: action_kind must be CP_ACTION_CONTINUOUS or CP_ACTION_DISCRETE");
    hipStream_t st = (hipStream_t)stream;
    const int B = h->cfg.num_envs;
    CP_TRY(h, hipSetDevice(h->device));
    if (h->cfg.autoreset) use_counter(h);  // zeroed by the previous call's reset launch
    if (h->pixels) CP_TRY(h, hipMemsetAsync(h->b.rcount, 0, sizeof(int32_t), st));
    dim3 grid(grid_for(2 * B, cp::WAVE)), block(cp::WAVE);  // two lanes per env
    hipEvent_t* ev = timing_slot(h, 0);
    if (ev) CP_TRY(h, hipEventRecord(ev[0], st));
    const bool lqr = h->lqr.gains != nullptr;
#define CP_LAUNCH_STEP(K, Q)                                                                                    \
    do {                                                                                                        \
        if (h->step_lat)                                                                                        \
            hipLaunchKernelGGL((cp::cp_step_kernel<K, Q, true>), grid, block, 0, st, h->cfg, h->b, actions,     \
                               obs_out, reward_out, done_out, terminal_obs_out, h->readback, h->readback_bug,    \
                               h->lqr);                                                                         \
        else                                                                                                    \
            hipLaunchKernelGGL((cp::cp_step_kernel<K, Q, false>), grid, block, 0, st, h->cfg, h->b, actions,    \
                               obs_out, reward_out, done_out, terminal_obs_out, h->readback, h->readback_bug,    \
                               h->lqr);                                                                         \
    } while (0)
    if (action_kind == CP_ACTION_CONTINUOUS) {
        if (lqr) CP_LAUNCH_STEP(CP_ACTION_CONTINUOUS, true);
        else CP_LAUNCH_STEP(CP_ACTION_CONTINUOUS, false);
    } else {
        if (lqr) CP_LAUNCH_STEP(CP_ACTION_DISCRETE, true);
        else CP_LAUNCH_STEP(CP_ACTION_DISCRETE, false);
    }
#undef CP_LAUNCH_STEP
    CP_TRY(h, hipGetLastError());
    if (ev) CP_TRY(h, hipEventRecord(ev[1], st));
    // autoreset envs were simulated this step, so they are in the render list; the reset
    // kernel rewrites their poses first, and the one render launch draws the new episode
    if (h->cfg.autoreset && launch_reset_from_list(h, obs_out, st, false)) return -1;
    if (h->pixels) return launch_render(h, h->b.rlist, h->b.rcount, st);
    return 0;
}

int cp_set_readback(cp_handle* h, float* readback_out, int reference_bug) {
    if (!h) return fail(h, "cp_set_readback: null handle");
    h->readback = readback_out;
    h->readback_bug = reference_bug ? 1 : 0;
    return 0;
}

int cp_set_lqr(cp_handle* h, const float* gains, int per_env, float* state8_out, float done_pos,
               float done_angle) {
    if (!h) return fail(h, "cp_set_lqr: null handle");
    if (!gains && state8_out) return fail(h, "cp_set_lqr: the 8-state readback needs the LQR policy on");
    h->lqr.gains = gains;
    h->lqr.per_env = per_env ? 1 : 0;
    h->lqr.state8 = state8_out;
    h->lqr.done_pos = done_pos;
    h->lqr.done_angle = done_angle;
    choose_reset_shape(h);
    return 0;
}

int cp_set_bump_forces(cp_handle* h, const float* forces, void* stream) {
    if (!h || !forces) return fail(h, "cp_set_bump_forces: null argument");
    CP_TRY(h, hipSetDevice(h->device));
    size_t n = (size_t)h->cfg.num_envs * h->cfg.initial_force_steps * 4;
    CP_TRY(h, hipMemcpyAsync(h->b.bumps, forces, n * sizeof(float), hipMemcpyDeviceToDevice, (hipStream_t)stream));
    return 0;
}

int cp_get_state(cp_handle* h, float* state_out, void* stream) {
    if (!h || !state_out) return fail(h, "cp_get_state: null argument");
    CP_TRY(h, hipSetDevice(h->device));
    size_t n = (size_t)CP_STATE_FIELDS * h->cfg.num_envs;
    CP_TRY(h, hipMemcpyAsync(state_out, h->b.state, n * sizeof(float), hipMemcpyDeviceToDevice, (hipStream_t)stream));
    return 0;
}

int cp_set_state(cp_handle* h, const float* state_in, void* stream) {
    if (!h || !state_in) return fail(h, "cp_set_state: null argument");
    CP_TRY(h, hipSetDevice(h->device));
    size_t n = (size_t)CP_STATE_FIELDS * h->cfg.num_envs;
    CP_TRY(h, hipMemcpyAsync(h->b.state, state_in, n * sizeof(float), hipMemcpyDeviceToDevice, (hipStream_t)stream));
    return 0;
}

int cp_episode_returns(cp_handle* h, float* returns_out, int32_t* lengths_out, void* stream) {
    if (!h) return fail(h, "cp_episode_returns: null handle");
    CP_TRY(h, hipSetDevice(h->device));
    size_t B = (size_t)h->cfg.num_envs;
    hipStream_t st = (hipStream_t)stream;
    if (returns_out) CP_TRY(h, hipMemcpyAsync(returns_out, h->b.last_ret, B * sizeof(float), hipMemcpyDeviceToDevice, st));
    if (lengths_out)
        CP_TRY(h, hipMemcpyAsync(lengths_out, h->b.last_len, B * sizeof(int32_t), hipMemcpyDeviceToDevice, st));
    return 0;
}

int cp_overflow_counts(cp_handle* h, int32_t* out, void* stream) {
    if (!h || !out) return fail(h, "cp_overflow_counts: null argument");
    CP_TRY(h, hipSetDevice(h->device));
    CP_TRY(h, hipMemcpyAsync(out, h->b.overflow, (size_t)h->cfg.num_envs * sizeof(int32_t), hipMemcpyDeviceToDevice,
                             (hipStream_t)stream));
    return 0;
}

int cp_debug_stamps(cp_handle* h, uint64_t* out16, int reset) {
    if (!h || !out16) return fail(h, "cp_debug_stamps: null argument");
    CP_TRY(h, hipSetDevice(h->device));
    CP_TRY(h, hipDeviceSynchronize());
    CP_TRY(h, hipMemcpy(out16, h->b.stamps, 16 * sizeof(uint64_t), hipMemcpyDeviceToHost));
    if (reset) CP_TRY(h, hipMemset(h->b.stamps, 0, 16 * sizeof(uint64_t)));
#ifdef CP_STAMPS
    return 1;
#else
    return 0;
#endif
}

int cp_timing_begin(cp_handle* h, int max_launches) {
    if (!h || max_launches <= 0) return fail(h, "cp_timing_begin: bad argument");
    CP_TRY(h, hipSetDevice(h->device));
    timing_free(h->timing);
    h->timing.ev.resize((size_t)max_launches * 8);
    for (auto& e : h->timing.ev) CP_TRY(h, hipEventCreate(&e));
    h->timing.cap = max_launches;
    return 0;
}

int cp_timing_stride(cp_handle* h, int step_stride, int reset_stride) {
    if (!h || step_stride <= 0 || reset_stride <= 0) return fail(h, "cp_timing_stride: bad argument");
    h->timing.stride[0] = step_stride;
    h->timing.stride[1] = reset_stride;
    return 0;
}

int cp_timing_end(cp_handle* h, double* step_ms, int32_t* step_launches, double* reset_ms,
                  int32_t* reset_launches) {
    if (!h) return fail(h, "cp_timing_end: null handle");
    cp_timing& t = h->timing;
    double sums[3] = {0.0, 0.0, 0.0};
    int counts[3] = {t.nstep, t.nreset, t.nrender};
    for (int kind = 0; kind < 3; ++kind) {
        for (int n = 0; n < counts[kind]; ++n) {
            hipEvent_t a = t.ev[(size_t)(kind * t.cap + n) * 2], b = t.ev[(size_t)(kind * t.cap + n) * 2 + 1];
            CP_TRY(h, hipEventSynchronize(b));
            float ms = 0.0f;
            CP_TRY(h, hipEventElapsedTime(&ms, a, b));
            sums[kind] += ms;
        }
    }
    if (step_ms) *step_ms = sums[0];
    if (step_launches) *step_launches = counts[0];
    if (reset_ms) *reset_ms = sums[1];
    if (reset_launches) *reset_launches = counts[1];
    timing_free(t);
    t.render_ms = sums[2];
    t.render_launches = counts[2];
    return 0;
}

int cp_event_record_bytes(int action_kind, int repeats, int with_action) {
    if ((action_kind != CP_ACTION_CONTINUOUS && action_kind != CP_ACTION_DISCRETE) || repeats <= 0)
        return fail(nullptr, "cp_event_record_bytes: bad action kind or repeats");
    return cp::record_len(action_kind, repeats, with_action ? 1 : 0);
}

int cp_encode_events(cp_handle* h, int mode, const void* actions, int action_kind, const float* obs,
                     const float* terminal_obs, const float* reward, const uint8_t* done, const uint8_t* env_mask,
                     uint8_t* step_records, uint8_t* reset_records, uint8_t* flags, void* stream) {
    if (!h || !obs || !flags) return fail(h, "cp_encode_events: null argument");
    if (action_kind != CP_ACTION_CONTINUOUS && action_kind != CP_ACTION_DISCRETE)
        return fail(h, "cp_encode_events: bad action kind");
    if (mode == 0 && (!actions || !reward || !done || !step_records))
        return fail(h, "cp_encode_events: mode 0 needs actions, reward, done and step_records");
    if (mode == 1 && !reset_records) return fail(h, "cp_encode_events: mode 1 needs reset_records");
    if (mode != 0 && mode != 1) return fail(h, "cp_encode_events: mode must be 0 (step) or 1 (reset)");
    CP_TRY(h, hipSetDevice(h->device));
    const int B = h->cfg.num_envs;
    hipLaunchKernelGGL(cp::cp_event_kernel, dim3(grid_for(B, 256)), dim3(256), 0, (hipStream_t)stream, B,
                       h->cfg.action_repeats, mode, action_kind, h->cfg.autoreset, actions, obs, terminal_obs, reward,
                       done, env_mask, h->b.stepped, step_records, reset_records, flags);
    CP_TRY(h, hipGetLastError());
    return 0;
}

int cp_timing_render(cp_handle* h, double* render_ms, int32_t* render_launches) {
    if (!h) return fail(h, "cp_timing_render: null handle");
    if (render_ms) *render_ms = h->timing.render_ms;
    if (render_launches) *render_launches = h->timing.render_launches;
    return 0;
}

void cp_default_raster_config(cp_raster_config* rc) {
    std::memset(rc, 0, sizeof(*rc));
    rc->width = 50;        // --render-width, bullet_cartpole.py:35
    rc->height = 50;       // --render-height, :37
    rc->num_cameras = 1;   // --num-cameras, :27
    const float temp = 0.75f;  // :278-279
    rc->eye[0][0] = 0.0f; rc->eye[0][1] = temp; rc->eye[0][2] = temp;
    rc->eye[1][0] = temp; rc->eye[1][1] = 0.0f; rc->eye[1][2] = temp;
    rc->target[0] = 0.0f; rc->target[1] = 0.0f; rc->target[2] = 0.3f;  // :280
    rc->up[0] = 0.0f; rc->up[1] = 0.0f; rc->up[2] = 1.0f;              // :281
    rc->tan_half_fov = (float)std::tan(0.5 * 30.0 * 3.141592653589793 / 180.0);  // fov 30, :283
    rc->far_plane = 20.0f;                                             // :282
    // light from above and in front of camera 0 (unpinned: TinyRenderer's is not available)
    const double l[3] = {0.3, 0.5, 1.0};
    const double ln = std::sqrt(l[0] * l[0] + l[1] * l[1] + l[2] * l[2]);
    for (int k = 0; k < 3; ++k) rc->light[k] = (float)(l[k] / ln);
    rc->ambient = 0.6f;
    rc->diffuse = 0.4f;
    rc->background[0] = 1.0f; rc->background[1] = 1.0f; rc->background[2] = 1.0f;
    static const float col[5][3] = {{0.3f, 0.3f, 0.0f},   // ground.urdf:15
                                    {0.9f, 0.2f, 0.1f},   // cart.urdf:25
                                    {0.2f, 0.7f, 0.1f},   // pole.urdf:30
                                    {0.2f, 0.9f, 0.1f},   // cart2.urdf:25
                                    {0.7f, 0.2f, 0.7f}};  // pole2.urdf:24
    std::memcpy(rc->color, col, sizeof(col));
}

int cp_set_raster(cp_handle* h, const cp_raster_config* rc, uint16_t* pixels_out) {
    if (!h) return fail(h, "cp_set_raster: null handle");
    CP_TRY(h, hipSetDevice(h->device));
    if (!pixels_out) {
        h->pixels = nullptr;
        (void)hipFree(h->b.rposes);
        (void)hipFree(h->b.rlist);
        (void)hipFree(h->b.rcount);
        (void)hipFree(h->b.rtable);
        h->b.rposes = nullptr;
        h->b.rlist = h->b.rcount = nullptr;
        h->b.rtable = nullptr;
        return 0;
    }
    if (!rc) return fail(h, "cp_set_raster: null config");
    const int R = h->cfg.action_repeats;
    if (rc->width <= 0 || rc->height <= 0 || rc->width > 4096 || rc->height > 4096)
        return fail(h, "cp_set_raster: width and height must be in 1..4096");
    if (rc->num_cameras != 1 && rc->num_cameras != 2) return fail(h, "--num-cameras must be 1 or 2");
    if (rc->num_cameras * R > cp::RMAX_FRAMES)
        return fail(h, "cp_set_raster: num_cameras * action_repeats must be <= 16");
    h->raster = *rc;
    h->pixels = pixels_out;
    if (!h->b.rposes) {
        const size_t B = (size_t)h->cfg.num_envs;
        hipError_t e = hipMalloc((void**)&h->b.rposes, B * R * CP_NUM_DYN * 7 * sizeof(float));
        if (e == hipSuccess) e = hipMalloc((void**)&h->b.rlist, B * sizeof(int32_t));
        if (e == hipSuccess) e = hipMalloc((void**)&h->b.rcount, sizeof(int32_t));
        if (e != hipSuccess) {
            (void)hipFree(h->b.rposes);
            (void)hipFree(h->b.rlist);
            h->b.rposes = nullptr;
            h->b.rlist = nullptr;
            h->pixels = nullptr;
            return check(h, e, "cp_set_raster: hipMalloc");
        }
    }
    // per-camera ray table for this configuration (synchronous: a setup call)
    (void)hipFree(h->b.rtable);
    h->b.rtable = nullptr;
    const int npx = rc->width * rc->height;
    CP_TRY(h, hipMalloc((void**)&h->b.rtable, (size_t)rc->num_cameras * npx * 2 * sizeof(float4)));
    hipLaunchKernelGGL(cp::cp_raster_table_kernel, dim3(grid_for(npx, cp::RT), rc->num_cameras), dim3(cp::RT), 0, 0,
                       h->raster, h->cfg.phys, h->b.rtable,
                       reinterpret_cast<uint8_t*>(h->b.rtable + (size_t)rc->num_cameras * npx));
    CP_TRY(h, hipGetLastError());
    CP_TRY(h, hipDeviceSynchronize());
    return 0;
}

// ---------------------------------------------------------------- event log writer
}  // extern "C"

struct cp_eventlog {
    FILE* f = nullptr;
    std::vector<std::vector<uint8_t>> ep;  // open episode per env (encoded Episode body)
};

static int eventlog_flush(cp_eventlog* log, std::vector<uint8_t>& ep) {
    if (ep.empty()) return 0;
    const int32_t n = (int32_t)ep.size();  // struct.pack('=l', len(buff)), event_log.py:54
    if (std::fwrite(&n, sizeof(n), 1, log->f) != 1 || std::fwrite(ep.data(), 1, ep.size(), log->f) != ep.size())
        return fail(nullptr, "cp_eventlog: write failed");
    ep.clear();
    return 0;
}

extern "C" {

int cp_eventlog_open(const char* path, int num_envs, cp_eventlog** out) {
    if (!path || !out || num_envs <= 0) return fail(nullptr, "cp_eventlog_open: bad argument");
    cp_eventlog* log = new (std::nothrow) cp_eventlog();
    if (!log) return fail(nullptr, "cp_eventlog_open: out of memory");
    log->f = std::fopen(path, "ab");  // appends, as event_log.py:45
    if (!log->f) {
        delete log;
        return fail(nullptr, std::string("cp_eventlog_open: cannot open ") + path);
    }
    log->ep.resize((size_t)num_envs);
    *out = log;
    return 0;
}

int cp_eventlog_write(cp_eventlog* log, const uint8_t* flags, const uint8_t* step_records, int step_bytes,
                      const uint8_t* reset_records, int reset_bytes) {
    if (!log || !flags) return fail(nullptr, "cp_eventlog_write: null argument");
    for (size_t i = 0; i < log->ep.size(); ++i) {
        const uint8_t fl = flags[i];
        if ((fl & 1) && step_records) {
            const uint8_t* r = step_records + i * (size_t)step_bytes;
            log->ep[i].insert(log->ep[i].end(), r, r + step_bytes);
        }
        if ((fl & 2) && reset_records) {  // EventLog.reset + add_just_state (bullet_cartpole.py:342-344)
            if (eventlog_flush(log, log->ep[i])) return -1;
            const uint8_t* r = reset_records + i * (size_t)reset_bytes;
            log->ep[i].assign(r, r + reset_bytes);
        }
    }
    std::fflush(log->f);
    return 0;
}

int cp_eventlog_close(cp_eventlog* log) {
    if (!log) return fail(nullptr, "cp_eventlog_close: null handle");
    int rc = 0;
    for (auto& ep : log->ep)
        if (eventlog_flush(log, ep)) rc = -1;
    if (std::fclose(log->f) != 0) rc = fail(nullptr, "cp_eventlog_close: close failed");
    delete log;
    return rc;
}

int cp_get_stepped(cp_handle* h, uint8_t* out, void* stream) {
    if (!h || !out) return fail(h, "cp_get_stepped: null argument");
    CP_TRY(h, hipSetDevice(h->device));
    CP_TRY(h, hipMemcpyAsync(out, h->b.stepped, h->cfg.num_envs, hipMemcpyDeviceToDevice, (hipStream_t)stream));
    return 0;
}

/* ---- replay memory (cp_replay.h) ---- */
static int replay_ok(const cp_replay* rm, const char* what) {
    if (!rm || !rm->state || !rm->state_1_idx || !rm->action || !rm->reward || !rm->terminal_mask ||
        !rm->state_2_idx || !rm->free_slots || !rm->ctrl || !rm->plan || !rm->scan)
        return fail(nullptr, std::string(what) + ": null replay buffer");
    if (rm->buffer_size < 1 || rm->state_dim < 1 || rm->action_dim < 1 ||
        rm->state_buffer_size < rm->buffer_size + rm->buffer_size / 2)
        return fail(nullptr, std::string(what) + ": bad sizes (state_buffer_size must be >= int(1.5 * buffer_size))");
    return 0;
}

int cp_replay_init(const cp_replay* rm, int32_t* cur, int rows, void* stream) {
    if (replay_ok(rm, "cp_replay_init")) return -1;
    if (rows < 0 || (rows > 0 && !cur)) return fail(nullptr, "cp_replay_init: bad rows / cur");
    const int64_t n = std::max<int64_t>(std::max<int64_t>(rm->state_buffer_size, rows), CP_RM_CTRL);
    hipLaunchKernelGGL(cprm::init_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       *rm, cur, rows);
    CP_TRY(nullptr, hipGetLastError());
    return 0;
}

int cp_replay_add(const cp_replay* rm, int32_t* cur, int rows, const uint8_t* valid, const void* actions,
                  int action_kind, const float* reward, const uint8_t* done, const uint8_t* restart,
                  const void* next_states, const void* terminal_states, int state_kind, void* stream) {
    if (replay_ok(rm, "cp_replay_add")) return -1;
    if (rows < 0 || rows > rm->buffer_size) return fail(nullptr, "cp_replay_add: rows must be in [0, buffer_size]");
    if (rows == 0) return 0;
    if (!cur) return fail(nullptr, "cp_replay_add: null cur");
    if (valid && (!actions || !reward || !done || !next_states))
        return fail(nullptr, "cp_replay_add: events need actions, reward, done and next_states");
    if (restart && !next_states) return fail(nullptr, "cp_replay_add: restarts need next_states");
    if (action_kind != CP_ACTION_CONTINUOUS && action_kind != CP_ACTION_DISCRETE)
        return fail(nullptr, "cp_replay_add: bad action kind");
    if (state_kind != CP_STATES_F32 && state_kind != CP_STATES_F16)
        return fail(nullptr, "cp_replay_add: bad state kind");
    if (!valid && !restart) return 0;
    const hipStream_t st = (hipStream_t)stream;
    const dim3 nb((unsigned)((rows + cprm::PLAN_THREADS - 1) / cprm::PLAN_THREADS)), nt(cprm::PLAN_THREADS);
    hipLaunchKernelGGL(cprm::count_kernel, nb, nt, 0, st, *rm, rows, valid);
    hipLaunchKernelGGL(cprm::free_count_kernel, nb, nt, 0, st, *rm, rows, valid, restart);
    hipLaunchKernelGGL(cprm::plan_kernel, nb, nt, 0, st, *rm, rows, valid, restart);
    switch (cprm::vec_for(rm->state_dim, state_kind)) {
        case 8: cprm::launch_write<8>(rm, rows, cur, actions, action_kind, reward, done, restart, next_states,
                                       terminal_states, state_kind, st); break;
        case 4: cprm::launch_write<4>(rm, rows, cur, actions, action_kind, reward, done, restart, next_states,
                                       terminal_states, state_kind, st); break;
        case 2: cprm::launch_write<2>(rm, rows, cur, actions, action_kind, reward, done, restart, next_states,
                                       terminal_states, state_kind, st); break;
        default: cprm::launch_write<1>(rm, rows, cur, actions, action_kind, reward, done, restart, next_states,
                                        terminal_states, state_kind, st);
    }
    CP_TRY(nullptr, hipGetLastError());
    return 0;
}

int cp_replay_sample(const cp_replay* rm, int n, const int32_t* idxs, uint64_t seed, uint64_t counter,
                     const cp_replay_batch* out, void* stream) {
    if (replay_ok(rm, "cp_replay_sample")) return -1;
    if (n < 0 || !out) return fail(nullptr, "cp_replay_sample: bad n / null out");
    if (n == 0) return 0;
    const int vec = cprm::vec_for(rm->state_dim, CP_STATES_F16);
    const int64_t threads = (int64_t)n * (rm->state_dim / vec);
    const dim3 grid((unsigned)((threads + 255) / 256));
    const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32), c1 = (uint32_t)counter,
                   c2 = (uint32_t)(counter >> 32);
    const hipStream_t st = (hipStream_t)stream;
    switch (vec) {
        case 8: hipLaunchKernelGGL(cprm::sample_kernel<8>, grid, dim3(256), 0, st, *rm, n, idxs, k0, k1, c1, c2, *out); break;
        case 4: hipLaunchKernelGGL(cprm::sample_kernel<4>, grid, dim3(256), 0, st, *rm, n, idxs, k0, k1, c1, c2, *out); break;
        case 2: hipLaunchKernelGGL(cprm::sample_kernel<2>, grid, dim3(256), 0, st, *rm, n, idxs, k0, k1, c1, c2, *out); break;
        default: hipLaunchKernelGGL(cprm::sample_kernel<1>, grid, dim3(256), 0, st, *rm, n, idxs, k0, k1, c1, c2, *out);
    }
    CP_TRY(nullptr, hipGetLastError());
    return 0;
}

}  // extern "C"
