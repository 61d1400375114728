// Replay memory kernels (C-ABI in include/cartpole_amd.h).
//
// The reference (replay_memory.py:76-118) adds events one at a time: free the
// clobbered event's state slots (append), write the event, pop a slot for
// state_2.  For a batch of rows the slot bookkeeping is a pure prefix-sum
// problem: row j's event lands at insert + (valid rows before j), its frees are
// appended at tail + (frees before j) and its pops read head + (pops before j).
// So three short scan passes over blocks of 1024 rows (count valid rows; count frees
// and pops; fix every position and push the freed slots) plan the batch, and a wide
// kernel then does the HBM work (state rows, event fields) for all rows in parallel.  The result is identical to the
// sequential reference order, FIFO contents included.
#pragma once

#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>

namespace cprm {

constexpr int PLAN_THREADS = 1024;
constexpr int PLAN_WAVES = PLAN_THREADS / 64;

// block-wide exclusive scan of a 64-bit value; returns the block total in *total
__device__ inline int64_t block_exclusive_scan(int64_t x, int64_t* total, int64_t* lds) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    int64_t inc = x;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        int64_t y = __shfl_up(inc, o, 64);
        if (lane >= o) inc += y;
    }
    if (lane == 63) lds[wave] = inc;
    __syncthreads();
    if (wave == 0) {
        int64_t w = lane < PLAN_WAVES ? lds[lane] : 0, wi = w;
#pragma unroll
        for (int o = 1; o < PLAN_WAVES; o <<= 1) {
            int64_t y = __shfl_up(wi, o, 64);
            if (lane >= o) wi += y;
        }
        if (lane < PLAN_WAVES) lds[PLAN_WAVES + lane] = wi - w;  // exclusive wave offsets
        if (lane == PLAN_WAVES - 1) lds[2 * PLAN_WAVES] = wi;
    }
    __syncthreads();
    const int64_t r = lds[PLAN_WAVES + wave] + inc - x;
    *total = lds[2 * PLAN_WAVES];
    __syncthreads();  // lds reused by the next call
    return r;
}

// sum of a[0..n) over the block (every thread gets it)
__device__ inline int64_t block_sum(const int64_t* a, int n, int64_t* lds) {
    int64_t x = 0;
    for (int k = threadIdx.x; k < n; k += PLAN_THREADS) x += a[k];
    int64_t tot;
    block_exclusive_scan(x, &tot, lds);
    return tot;
}

// Three passes over blocks of 1024 rows; scan[] = blockV[nb] | blockFP[nb] | ctrl snapshot.
// Pass 1: valid rows per block, and the ctrl snapshot the later passes read (pass 3
// rewrites ctrl).
__global__ void __launch_bounds__(PLAN_THREADS) count_kernel(cp_replay rm, int rows, const uint8_t* valid) {
    __shared__ int64_t lds[2 * PLAN_WAVES + 1];
    const int nb = (rows + PLAN_THREADS - 1) / PLAN_THREADS;
    const int j = blockIdx.x * PLAN_THREADS + threadIdx.x;
    const int v = (j < rows && valid && valid[j]) ? 1 : 0;
    int64_t tot;
    block_exclusive_scan(v, &tot, lds);
    if (threadIdx.x == 0) rm.scan[blockIdx.x] = tot;
    if (blockIdx.x == 0 && threadIdx.x < CP_RM_CTRL) rm.scan[2 * nb + threadIdx.x] = rm.ctrl[threadIdx.x];
}

struct RowPlan {
    int v, r, f, p;
    int64_t pos;
};

// row j's event position and free / pop counts (needs the global valid prefix)
__device__ inline RowPlan row_plan(const cp_replay& rm, int rows, const uint8_t* valid, const uint8_t* restart,
                                   int64_t* lds) {
    const int nb = (rows + PLAN_THREADS - 1) / PLAN_THREADS;
    const int64_t* snap = rm.scan + 2 * nb;
    const int64_t N = rm.buffer_size, insert = snap[CP_RM_INSERT];
    const bool full = snap[CP_RM_FULL] != 0;
    const int j = blockIdx.x * PLAN_THREADS + threadIdx.x;
    RowPlan q;
    q.v = (j < rows && valid && valid[j]) ? 1 : 0;
    q.r = (j < rows && restart && restart[j]) ? 1 : 0;
    const int64_t Kb = block_sum(rm.scan, blockIdx.x, lds);
    int64_t kv;
    const int64_t k = Kb + block_exclusive_scan(q.v, &kv, lds);
    q.pos = -1;
    q.f = 0;
    if (q.v) {
        const int64_t g = insert + k;  // < 2N: rows <= N
        q.pos = g >= N ? g - N : g;
        if (full || g >= N) q.f = rm.terminal_mask[q.pos] == 0.f ? 2 : 1;  // :80-91
    }
    q.p = q.v + q.r;
    return q;
}

// Pass 2: frees and pops per block (packed f | p << 32).
__global__ void __launch_bounds__(PLAN_THREADS) free_count_kernel(cp_replay rm, int rows, const uint8_t* valid,
                                                                  const uint8_t* restart) {
    __shared__ int64_t lds[2 * PLAN_WAVES + 1];
    const int nb = (rows + PLAN_THREADS - 1) / PLAN_THREADS;
    const RowPlan q = row_plan(rm, rows, valid, restart, lds);
    int64_t tot;
    block_exclusive_scan((int64_t)q.f | ((int64_t)q.p << 32), &tot, lds);
    if (threadIdx.x == 0) rm.scan[nb + blockIdx.x] = tot;
}

// Pass 3: plan[2j] = event position of row j (-1: no event), plan[2j+1] = its first
// pop's free-ring position (-1: no pop); the freed slots are pushed here, before any
// pop reads them (write_kernel).  The last block publishes the new ctrl.
__global__ void __launch_bounds__(PLAN_THREADS) plan_kernel(cp_replay rm, int rows, const uint8_t* valid,
                                                            const uint8_t* restart) {
    __shared__ int64_t lds[2 * PLAN_WAVES + 1];
    const int nb = (rows + PLAN_THREADS - 1) / PLAN_THREADS;
    const int64_t* snap = rm.scan + 2 * nb;
    const int64_t S = rm.state_buffer_size, head = snap[CP_RM_HEAD], tail = snap[CP_RM_TAIL];
    const RowPlan q = row_plan(rm, rows, valid, restart, lds);
    const int j = blockIdx.x * PLAN_THREADS + threadIdx.x;
    const int64_t FPb = block_sum(rm.scan + nb, blockIdx.x, lds);
    int64_t tot;
    const int64_t ex = FPb + block_exclusive_scan((int64_t)q.f | ((int64_t)q.p << 32), &tot, lds);
    const int64_t fj = ex & 0xffffffffll, pj = ex >> 32;
    if (q.f) {
        const int64_t a = tail + fj;
        rm.free_slots[a % S] = rm.state_1_idx[q.pos];
        if (q.f == 2) rm.free_slots[(a + 1) % S] = rm.state_2_idx[q.pos];
    }
    // sequential order: row j's pops come after its own frees
    if (q.p && head + pj + q.p > tail + fj + q.f) atomicOr((unsigned long long*)&rm.ctrl[CP_RM_ERROR], 1ull);
    if (j < rows) {
        rm.plan[2 * j] = (int32_t)q.pos;
        rm.plan[2 * j + 1] = q.p ? (int32_t)((head + pj) % S) : -1;
    }
    int64_t e2;
    block_exclusive_scan(q.f == 2 ? 1 : 0, &e2, lds);
    if (threadIdx.x == 0 && e2) atomicAdd((unsigned long long*)&rm.ctrl[CP_RM_EVICTED_S2], (unsigned long long)e2);
    if (blockIdx.x == nb - 1) {
        const int64_t K = block_sum(rm.scan, nb, lds), FP = block_sum(rm.scan + nb, nb, lds);
        if (threadIdx.x == 0) {
            const int64_t N = rm.buffer_size, insert = snap[CP_RM_INSERT];
            rm.ctrl[CP_RM_INSERT] = (insert + K) % N;
            rm.ctrl[CP_RM_FULL] = (snap[CP_RM_FULL] || insert + K >= N) ? 1 : 0;
            rm.ctrl[CP_RM_HEAD] = head + (FP >> 32);
            rm.ctrl[CP_RM_TAIL] = tail + (FP & 0xffffffffll);
            rm.ctrl[CP_RM_ADDS] = snap[CP_RM_ADDS] + K;
        }
    }
}

template <int VEC>
struct alignas(2 * VEC) HalfVec {
    __half h[VEC];
};

// copy unit u (VEC elements) of a state row into slot `slot` of the state buffer
template <int VEC, bool F16>
__device__ inline void put_state(const cp_replay& rm, int64_t slot, const void* src, int64_t row, int u) {
    const int64_t D = rm.state_dim;
    HalfVec<VEC> o;
    if (F16) {
        o = reinterpret_cast<const HalfVec<VEC>*>(static_cast<const uint16_t*>(src) + row * D)[u];
    } else {
        const float* s = static_cast<const float*>(src) + row * D + (int64_t)u * VEC;
#pragma unroll
        for (int e = 0; e < VEC; ++e) o.h[e] = __float2half_rn(s[e]);  // numpy f32 -> f16 (RNE)
    }
    reinterpret_cast<HalfVec<VEC>*>(rm.state + slot * D)[u] = o;
}

template <int VEC, bool F16>
__global__ void __launch_bounds__(256) write_kernel(cp_replay rm, int rows, int32_t* cur, const void* actions,
                                                    int action_kind, const float* reward, const uint8_t* done,
                                                    const uint8_t* restart, const void* next_states,
                                                    const void* terminal_states) {
    const int units = rm.state_dim / VEC;
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t j = t / units;
    const int u = (int)(t - j * units);
    if (j >= rows) return;
    const int32_t pos = rm.plan[2 * j], pb = rm.plan[2 * j + 1];
    if (pb < 0) return;
    const int64_t S = rm.state_buffer_size;
    const bool r = restart && restart[j];
    int32_t s2 = -1, slot = -1;
    if (pos >= 0) {
        s2 = rm.free_slots[pb];
        const void* src = (r && terminal_states) ? terminal_states : next_states;
        put_state<VEC, F16>(rm, s2, src, j, u);
        if (u == 0) {
            const int32_t s1 = cur[j];
            if (s1 < 0) atomicOr((unsigned long long*)&rm.ctrl[CP_RM_ERROR], 2ull);
            const int A = rm.action_dim;
            rm.state_1_idx[pos] = s1;
            for (int a = 0; a < A; ++a)
                rm.action[(int64_t)pos * A + a] = action_kind == CP_ACTION_DISCRETE
                                                      ? (float)static_cast<const int8_t*>(actions)[j * A + a]
                                                      : static_cast<const float*>(actions)[j * A + a];
            rm.reward[pos] = reward[j];
            rm.terminal_mask[pos] = done[j] ? 0.f : 1.f;  // :99-100
            rm.state_2_idx[pos] = s2;
        }
    }
    if (r) {
        slot = rm.free_slots[(pb + (pos >= 0 ? 1 : 0)) % S];
        put_state<VEC, F16>(rm, slot, next_states, j, u);
    }
    if (u == 0) cur[j] = r ? slot : s2;
}

template <int VEC>
__global__ void __launch_bounds__(256) sample_kernel(cp_replay rm, int n, const int32_t* idxs, uint32_t k0,
                                                     uint32_t k1, uint32_t c1, uint32_t c2, cp_replay_batch out) {
    const int64_t D = rm.state_dim;
    const int units = (int)(D / VEC);
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t j = t / units;
    const int u = (int)(t - j * units);
    if (j >= n) return;
    const int64_t size = rm.ctrl[CP_RM_FULL] ? rm.buffer_size : rm.ctrl[CP_RM_INSERT];  // size(), :117-118
    int64_t idx;
    if (idxs) {
        idx = idxs[j];
    } else {
        const uint32_t w = cp::philox_word((uint32_t)j, c1, c2, 0x52504c59u, k0, k1, 0);
        idx = size ? (int64_t)(((uint64_t)w * (uint64_t)size) >> 32) : -1;
    }
    if (idx < 0 || idx >= size) {
        if (u == 0) {
            if (idxs) atomicOr((unsigned long long*)&rm.ctrl[CP_RM_ERROR], 4ull);
            if (out.idx) out.idx[j] = -1;
        }
        return;
    }
    const int32_t s1 = rm.state_1_idx[idx], s2 = rm.state_2_idx[idx];
    if (s1 < 0 || s1 >= rm.state_buffer_size || s2 < 0 || s2 >= rm.state_buffer_size) return;  // error bit 2 set
    using V = HalfVec<VEC>;
    if (out.state_1) reinterpret_cast<V*>(out.state_1 + j * D)[u] = reinterpret_cast<const V*>(rm.state + s1 * D)[u];
    if (out.state_2) reinterpret_cast<V*>(out.state_2 + j * D)[u] = reinterpret_cast<const V*>(rm.state + s2 * D)[u];
    if (u == 0) {
        if (out.idx) out.idx[j] = (int32_t)idx;
        const int A = rm.action_dim;
        if (out.action)
            for (int a = 0; a < A; ++a) out.action[j * A + a] = rm.action[idx * A + a];
        if (out.reward) out.reward[j] = rm.reward[idx];
        if (out.terminal_mask) out.terminal_mask[j] = rm.terminal_mask[idx];
        if (out.state_1_idx) out.state_1_idx[j] = s1;
        if (out.state_2_idx) out.state_2_idx[j] = s2;
    }
}

__global__ void init_kernel(cp_replay rm, int32_t* cur, int rows) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t < rm.state_buffer_size) rm.free_slots[t] = (int32_t)t;
    if (t < rows) cur[t] = -1;
    if (t < CP_RM_CTRL) rm.ctrl[t] = t == CP_RM_TAIL ? rm.state_buffer_size : 0;
}

// widest element group (<= 16 bytes of float16) dividing the state row
inline int vec_for(int D, int state_kind) {
    const int cap = state_kind == CP_STATES_F16 ? 8 : 4;
    for (int v = cap; v > 1; v >>= 1)
        if (D % v == 0) return v;
    return 1;
}

template <int VEC>
inline void launch_write(const cp_replay* rm, int rows, int32_t* cur, const void* actions, int action_kind,
                                const float* reward, const uint8_t* done, const uint8_t* restart,
                                const void* next_states, const void* terminal_states, int state_kind,
                                hipStream_t st) {
    const int64_t threads = (int64_t)rows * (rm->state_dim / VEC);
    const dim3 grid((unsigned)((threads + 255) / 256));
    if (state_kind == CP_STATES_F16)
        hipLaunchKernelGGL((write_kernel<VEC, true>), grid, dim3(256), 0, st, *rm, rows, cur, actions,
                           action_kind, reward, done, restart, next_states, terminal_states);
    else
        hipLaunchKernelGGL((write_kernel<VEC, false>), grid, dim3(256), 0, st, *rm, rows, cur, actions,
                           action_kind, reward, done, restart, next_states, terminal_states);
}

}  // namespace cprm
