// cp_raster.h — in-kernel raster observation (--use-raw-pixels).
//
// Replaces render_rgb + set_state_element_for_repeat (bullet_cartpole.py:277-306):
// for every env, repeat r and camera c, an H x W RGB image of the 5 boxes, written
// as float16 [H][W][3][C][R] per env, the reference's state layout (:299-306).
//
// One wave per env (taken from a compacted env list).  The wave stages the env's R
// poses in LDS, projects every box to a conservative screen rectangle per (camera,
// repeat) and tabulates the shaded colour of every face; the per-pixel ray
// directions and the static ground's hits come from a per-camera table built once
// (cp_raster_table_kernel).  Strips of 64 consecutive pixels are contiguous in the
// output: most pixels meet no box rectangle and take a static colour, so the kernel
// is a stream of 16-byte stores with the ray tests confined to the boxes' rectangles.
//
// The per-pixel arithmetic is the oracle's (oracle/cp_oracle.c, raster section),
// operation for operation; the rectangles only skip boxes a ray cannot hit.
#pragma once
#include <hip/hip_fp16.h>

#include "../../include/cartpole_amd.h"
// (uses namespace cp's fp32 math: included after the fp32 instantiation of cp_math.h)

namespace cp {

constexpr int RT = 256;           // threads per table block
constexpr int WAVE_R = 64;        // lanes per wave
constexpr int RMAX_FRAMES = 16;   // C * R frames per env staged in LDS (checked at cp_set_raster)

struct Cam {
    V3 eye, f, r, u;
};

// camera basis (oracle: raster_camera)
CP_DEV Cam make_cam(const cp_raster_config& rc, int c) {
    Cam k;
    k.eye = mk(rc.eye[c][0], rc.eye[c][1], rc.eye[c][2]);
    const V3 F = sub(mk(rc.target[0], rc.target[1], rc.target[2]), k.eye);
    const float lf = sqrtf(dot(F, F));
    k.f = mk(F.x / lf, F.y / lf, F.z / lf);
    const V3 rr = cross(k.f, mk(rc.up[0], rc.up[1], rc.up[2]));
    const float lr = sqrtf(dot(rr, rr));
    k.r = mk(rr.x / lr, rr.y / lr, rr.z / lr);
    k.u = cross(k.r, k.f);
    return k;
}

// float16 bits of float32(u8) / 255 rounded to nearest even (numpy float16 division, :294)
CP_DEV uint16_t u8_to_half(int v) {
    return __half_as_ushort(__float2half_rn((float)v / 255.0f));
}
CP_DEV int to_u8(float x) {
    x = x > 1.0f ? 1.0f : (x < 0.0f ? 0.0f : x);
    return (int)(x * 255.0f + 0.5f);
}

// conservative pixel rectangle of box (centre cc, axes A, half h) seen by camera k.  FAST: the
// perspective divisions by the hardware reciprocal (v_rcp_f32, <= 1 ulp) instead of IEEE division:
// the rectangle only decides which ray tests run (every pixel value comes from ray_box_o's exact
// arithmetic, as the oracle's), and its +-1 pixel margin covers the ~1e-5 px an edge can move
template <bool FAST = false>
CP_DEV void box_rect(const Cam& k, V3 cc, const Axes& A, V3 h, float sxk, float syk, int W, int H, int16_t* out) {
    float x0 = 1e30f, x1 = -1e30f, y0 = 1e30f, y1 = -1e30f;
    bool behind = false, all_behind = true;
#pragma unroll
    for (int n = 0; n < 8; ++n) {
        V3 P = cc;
        P = madd(P, A.a0, (n & 1) ? h.x : -h.x);
        P = madd(P, A.a1, (n & 2) ? h.y : -h.y);
        P = madd(P, A.a2, (n & 4) ? h.z : -h.z);
        const V3 v = sub(P, k.eye);
        const float z = dot(v, k.f);
        behind = behind || z < 1e-3f;
        all_behind = all_behind && z < -1e-3f;
        float xs, ys;
        if constexpr (FAST) {
            xs = dot(v, k.r) * __builtin_amdgcn_rcpf(z * sxk);
            ys = dot(v, k.u) * __builtin_amdgcn_rcpf(z * syk);
        } else {
            xs = dot(v, k.r) / (z * sxk);
            ys = dot(v, k.u) / (z * syk);
        }
        const float px = (xs + 1.0f) * 0.5f * (float)W - 0.5f, py = (1.0f - ys) * 0.5f * (float)H - 0.5f;
        x0 = fminf(x0, px); x1 = fmaxf(x1, px); y0 = fminf(y0, py); y1 = fmaxf(y1, py);
    }
    if (all_behind) {  // a ray point at t > 0 has depth t * (d . f) = t > 0: no hit possible
        out[0] = 32000; out[1] = -32000; out[2] = 32000; out[3] = -32000;
        return;
    }
    if (behind || !(x0 == x0) || !(y0 == y0)) {  // straddles the eye plane: no culling
        out[0] = -32000; out[1] = 32000; out[2] = -32000; out[3] = 32000;
        return;
    }
    const float lim = 30000.0f;
    // a pixel centre k is hit only if k lies in [x0, x1] up to rounding (~1e-4 px):
    // floor / ceil plus one pixel covers it
    out[0] = (int16_t)fmaxf(-lim, floorf(x0) - 1.0f);
    out[1] = (int16_t)fminf(lim, ceilf(x1) + 1.0f);
    out[2] = (int16_t)fmaxf(-lim, floorf(y0) - 1.0f);
    out[3] = (int16_t)fminf(lim, ceilf(y1) + 1.0f);
}

// 1.0f / x, correctly rounded (the oracle's 1.0f / d): the hardware reciprocal and one FMA Newton
// step, which is the correctly rounded result for every x whose biased exponent lies in [1, 252]
// (checked for all 2^32 floats on gfx950: tools/micro/rcp_exact.hip, profiles/rd4e_rcp_exact.json);
// other x (zero, denormal, |x| >= 2^126, inf, NaN) take the IEEE division.  3 VALU instead of ~10.
constexpr unsigned RCP_EXP_LO = 1, RCP_EXP_HI = 252;
CP_DEV float rcp_rn(float x) {
    const unsigned ex = (__float_as_uint(x) >> 23) & 0xFFu;
    if (ex - RCP_EXP_LO <= RCP_EXP_HI - RCP_EXP_LO) {
        const float y = __builtin_amdgcn_rcpf(x);
        return __builtin_fmaf(__builtin_fmaf(-x, y, 1.0f), y, y);
    }
    return 1.0f / x;
}

// Ray (eye + t d) against a box with axes A and half extents h, given the origin-side
// dot products o_i = (eye - c) . a_i (oracle: ray_box computes them per ray; the same
// values): slab test, entry t, its axis and the face sign.  Returns false on a miss.
CP_DEV bool ray_box_o(V3 d, const float o[3], const Axes& A, V3 h, float& t, int& axis, float& sgn) {
    float lo[3], hi[3], dd[3];
    const V3 ax[3] = {A.a0, A.a1, A.a2};
    const float hh[3] = {h.x, h.y, h.z};
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        dd[i] = dot(d, ax[i]);
        const float inv = rcp_rn(dd[i]);
        const float t1 = (-hh[i] - o[i]) * inv, t2 = (hh[i] - o[i]) * inv;
        const bool lt = t1 < t2;
        lo[i] = lt ? t1 : t2;
        hi[i] = lt ? t2 : t1;
    }
    float tmin = lo[0];
    int a = 0;
    if (lo[1] > tmin) { tmin = lo[1]; a = 1; }
    if (lo[2] > tmin) { tmin = lo[2]; a = 2; }
    float tmax = hi[0] < hi[1] ? hi[0] : hi[1];
    tmax = tmax < hi[2] ? tmax : hi[2];
    t = tmin;
    axis = a;
    const float da = a == 0 ? dd[0] : (a == 1 ? dd[1] : dd[2]);
    sgn = da > 0.0f ? -1.0f : 1.0f;
    return tmin <= tmax && tmin > 0.0f;
}

// Per camera and pixel, the ray direction and the static ground's hit: the same for
// every env, computed once per raster configuration (cp_set_raster) with the render
// kernel's own arithmetic.  tabd [C][H*W] float4 (d.xyz, t of the ground hit or
// far_plane); cls [C][H*W] uint8: the ground face hit (axis * 2 + (sign > 0)), or 6 =
// background.  A pixel no dynamic box can reach shows its class's colour.
__global__ void __launch_bounds__(RT) cp_raster_table_kernel(cp_raster_config rc, cp_physics P, float4* tabd,
                                                              uint8_t* cls) {
    const int W = rc.width, H = rc.height, npx = W * H;
    const int p = blockIdx.x * RT + threadIdx.x, cam = blockIdx.y;
    if (p >= npx) return;
    const Cam k = make_cam(rc, cam);
    const float syk = rc.tan_half_fov;
    const float sxk = rc.tan_half_fov * ((float)W / (float)H);
    const int py = p / W, px = p - py * W;
    const float sx = ((2.0f * ((float)px + 0.5f)) / (float)W - 1.0f) * sxk;
    const float sy = (1.0f - (2.0f * ((float)py + 0.5f)) / (float)H) * syk;
    const V3 d = mk(fmaf_(sy, k.u.x, fmaf_(sx, k.r.x, k.f.x)), fmaf_(sy, k.u.y, fmaf_(sx, k.r.y, k.f.y)),
                    fmaf_(sy, k.u.z, fmaf_(sx, k.r.z, k.f.z)));
    const Axes I3 = {mk(1.0f, 0.0f, 0.0f), mk(0.0f, 1.0f, 0.0f), mk(0.0f, 0.0f, 1.0f)};
    const V3 oc = sub(k.eye, mk(0.0f, 0.0f, 0.0f));
    const float o[3] = {dot(oc, I3.a0), dot(oc, I3.a1), dot(oc, I3.a2)};
    float best = rc.far_plane;
    int face = 6;
    float t, sg;
    int ax;
    if (ray_box_o(d, o, I3, mk(P.half_extents[0][0], P.half_extents[0][1], P.half_extents[0][2]), t, ax, sg) &&
        t < best) {
        best = t;
        face = ax * 2 + (sg > 0.0f ? 1 : 0);
    }
    tabd[(size_t)cam * npx + p] = make_float4(d.x, d.y, d.z, best);
    cls[(size_t)cam * npx + p] = (uint8_t)face;
}

// Per-wave LDS carve-up of the render kernel (byte offsets, 16-byte aligned), for C
// cameras and R repeats.
struct RenderLds {
    int ax, c, oloc, rect, face, stage, total;
};
__host__ __device__ inline RenderLds render_lds(int C, int R) {
    RenderLds w;
    int o = 0;
    auto al = [](int x) { return (x + 15) & ~15; };
    w.ax = o;    o = al(o + R * CP_NUM_DYN * 9 * 4);          // body axes (columns) per repeat
    w.c = o;     o = al(o + R * CP_NUM_DYN * 3 * 4);          // body centres per repeat
    w.oloc = o;  o = al(o + C * R * CP_NUM_DYN * 3 * 4);      // (eye - c) . a_i per camera, repeat, body
    w.rect = o;  o = al(o + C * R * CP_NUM_DYN * 4 * 2);      // screen rectangle x0 x1 y0 y1
    w.face = o;  o = al(o + R * CP_NUM_BODIES * 6 * 3 * 2);   // shaded face colours, float16 bits
    w.stage = o; o = al(o + (WAVE_R * 3 * C * R + 8) * 2);    // one strip of 64 pixels (+ alignment slack)
    w.total = o;
    return w;
}

// 16-byte streaming (non-temporal) store: the frames are written once and read by the
// consumer much later
CP_DEV void store_stream(uint4* dst, uint4 q) {
    typedef unsigned int v4u __attribute__((ext_vector_type(4)));
    v4u v = {q.x, q.y, q.z, q.w};
    __builtin_nontemporal_store(v, reinterpret_cast<v4u*>(dst));
}

CP_DEV void wave_sync() {  // LDS written by some lanes, then read by others of the same wave
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

constexpr int RENDER_WAVES = 4;  // envs (one per wave) per render block

// poses [B][R][4][7] (xyz, quat xyzw) -> pixels float16 [B][H][W][3][C][R] for the envs
// in list[0 .. *count), one env per wave.  Per (camera, repeat, body) the ray-independent
// terms and a conservative screen rectangle go to the wave's LDS; the image is rendered
// in strips of 64 consecutive pixels (one per lane), which are contiguous in the output:
// a pixel outside every rectangle takes its static class colour, the others test the
// boxes whose rectangle holds them in body order against the ground's t (the oracle
// evaluates the same expressions per frame, so the images agree bit for bit).  Each
// strip is staged in LDS in the reference's (3, C, R) pixel order at the output's
// alignment and stored with 16-byte writes.
__global__ void __launch_bounds__(RENDER_WAVES * WAVE_R) cp_render_kernel(
    cp_raster_config rc, cp_physics P, int R, const int32_t* list, const int32_t* count, const float* poses,
    const float4* tabd, const uint8_t* cls, uint16_t* pixels) {
    extern __shared__ __align__(16) unsigned char render_lds_raw[];
    const int wave = threadIdx.x / WAVE_R, lane = threadIdx.x % WAVE_R;
    const int slot = blockIdx.x * RENDER_WAVES + wave;
    if (slot >= *count) return;  // wave-uniform; the kernel has no block barriers
    const int env = list[slot];
    const int W = rc.width, H = rc.height, C = rc.num_cameras, npx = W * H;
    const int per_px = 3 * C * R, F = C * R;
    const RenderLds L = render_lds(C, R);
    unsigned char* base = render_lds_raw + wave * L.total;
    float* sax = reinterpret_cast<float*>(base + L.ax);
    float* sc = reinterpret_cast<float*>(base + L.c);
    float* soloc = reinterpret_cast<float*>(base + L.oloc);
    int16_t* srect = reinterpret_cast<int16_t*>(base + L.rect);
    uint16_t* sface = reinterpret_cast<uint16_t*>(base + L.face);
    uint16_t* stage = reinterpret_cast<uint16_t*>(base + L.stage);

    const float* pe = poses + (size_t)env * R * CP_NUM_DYN * 7;
    if (lane < R * CP_NUM_DYN) {
        const float* q = pe + lane * 7;
        const Axes A = quat_axes(q[3], q[4], q[5], q[6]);
        float* a9 = sax + lane * 9;
        a9[0] = A.a0.x; a9[1] = A.a0.y; a9[2] = A.a0.z;
        a9[3] = A.a1.x; a9[4] = A.a1.y; a9[5] = A.a1.z;
        a9[6] = A.a2.x; a9[7] = A.a2.y; a9[8] = A.a2.z;
        sc[lane * 3 + 0] = q[0]; sc[lane * 3 + 1] = q[1]; sc[lane * 3 + 2] = q[2];
    }
    wave_sync();
    const float syk = rc.tan_half_fov;
    const float sxk = rc.tan_half_fov * ((float)W / (float)H);
    if (lane < F * CP_NUM_DYN) {  // item (cam, r, dyn body)
        const int cam = lane / (R * CP_NUM_DYN), rb = lane % (R * CP_NUM_DYN), b = rb % CP_NUM_DYN;
        const Cam k = make_cam(rc, cam);
        const float* a9 = sax + rb * 9;
        Axes A;
        A.a0 = mk(a9[0], a9[1], a9[2]); A.a1 = mk(a9[3], a9[4], a9[5]); A.a2 = mk(a9[6], a9[7], a9[8]);
        const V3 c = mk(sc[rb * 3 + 0], sc[rb * 3 + 1], sc[rb * 3 + 2]);
        const V3 oc = sub(k.eye, c);
        soloc[lane * 3 + 0] = dot(oc, A.a0);  // (the oracle's ray_box computes these per ray)
        soloc[lane * 3 + 1] = dot(oc, A.a1);
        soloc[lane * 3 + 2] = dot(oc, A.a2);
        box_rect(k, c, A, mk(P.half_extents[b + 1][0], P.half_extents[b + 1][1], P.half_extents[b + 1][2]), sxk,
                 syk, W, H, srect + lane * 4);
    }
    const V3 light = mk(rc.light[0], rc.light[1], rc.light[2]);
    for (int it = lane; it < R * CP_NUM_BODIES * 6; it += WAVE_R) {  // [r][body][face]
        const int r = it / (CP_NUM_BODIES * 6), b = (it / 6) % CP_NUM_BODIES, fc = it % 6;
        const int ax = fc >> 1;
        const float sg = (fc & 1) ? 1.0f : -1.0f;
        V3 an;
        if (b == 0) {
            an = ax == 0 ? mk(1.0f, 0.0f, 0.0f) : (ax == 1 ? mk(0.0f, 1.0f, 0.0f) : mk(0.0f, 0.0f, 1.0f));
        } else {
            const float* a9 = sax + (r * CP_NUM_DYN + b - 1) * 9 + 3 * ax;
            an = mk(a9[0], a9[1], a9[2]);
        }
        const float ndl = dot(scl(an, sg), light);
        const float sh = fmaf_(rc.diffuse, ndl > 0.0f ? ndl : 0.0f, rc.ambient);
        sface[it * 3 + 0] = u8_to_half(to_u8(rc.color[b][0] * sh));
        sface[it * 3 + 1] = u8_to_half(to_u8(rc.color[b][1] * sh));
        sface[it * 3 + 2] = u8_to_half(to_u8(rc.color[b][2] * sh));
    }
    const uint16_t bg0 = u8_to_half(to_u8(rc.background[0])), bg1 = u8_to_half(to_u8(rc.background[1])),
                   bg2 = u8_to_half(to_u8(rc.background[2]));
    wave_sync();

    uint16_t* out = pixels + (size_t)env * npx * per_px;
    const int RB = R * CP_NUM_DYN;  // near bits per camera
    const uint64_t cam_mask = RB >= 64 ? ~0ull : ((1ull << RB) - 1ull);
    for (int p0 = 0; p0 < npx; p0 += WAVE_R) {
        const int p = p0 + lane;
        const bool valid = p < npx;
        const int pl = valid ? p : npx - 1;
        const int py = pl / W, px = pl - py * W;
        const int last = (p0 + WAVE_R - 1 < npx ? p0 + WAVE_R - 1 : npx - 1);
        const int yA = p0 / W, yB = last / W;
        const int xA = yA == yB ? p0 - yA * W : 0, xB = yA == yB ? last - yB * W : W - 1;
        // (camera, repeat, body) items whose rectangle meets the strip: one bit each
        bool ov = false;
        if (lane < F * CP_NUM_DYN) {
            const int16_t* q = srect + lane * 4;
            ov = q[0] <= xB && q[1] >= xA && q[2] <= yB && q[3] >= yA;
        }
        const uint64_t near = __ballot(ov);
        uint16_t* dst = out + (size_t)p0 * per_px;
        const int sh = (int)((reinterpret_cast<uintptr_t>(dst) & 15) >> 1);  // halves before dst in its 16 B
        uint16_t* sp = stage + sh + lane * per_px;
        for (int cam = 0; cam < C; ++cam) {
            const int cl = cls[(size_t)cam * npx + pl];
            const uint64_t nc = (near >> (cam * RB)) & cam_mask;
            bool need = false;
            if (nc) {  // wave-uniform
                for (int k = 0; k < RB; ++k) {
                    if (!((nc >> k) & 1ull)) continue;
                    const int16_t* q = srect + (cam * RB + k) * 4;
                    need = need || (px >= q[0] && px <= q[1] && py >= q[2] && py <= q[3]);
                }
            }
            float4 t0 = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            if (need) t0 = tabd[(size_t)cam * npx + pl];
            for (int r = 0; r < R; ++r) {
                int hit = cl < 6 ? 0 : -1, fc = cl;
                const uint32_t nr = (uint32_t)(nc >> (r * CP_NUM_DYN)) & 15u;
                if (nr && need) {
                    const V3 d = mk(t0.x, t0.y, t0.z);
                    float best = t0.w;
#pragma unroll
                    for (int b = 1; b < CP_NUM_BODIES; ++b) {
                        if (!((nr >> (b - 1)) & 1u)) continue;
                        const int item = (cam * R + r) * CP_NUM_DYN + b - 1;
                        const int16_t* q = srect + item * 4;
                        if (px < q[0] || px > q[1] || py < q[2] || py > q[3]) continue;
                        const float* a9 = sax + (r * CP_NUM_DYN + b - 1) * 9;
                        Axes A;
                        A.a0 = mk(a9[0], a9[1], a9[2]); A.a1 = mk(a9[3], a9[4], a9[5]);
                        A.a2 = mk(a9[6], a9[7], a9[8]);
                        const V3 h = mk(P.half_extents[b][0], P.half_extents[b][1], P.half_extents[b][2]);
                        float t, sg;
                        int ax;
                        if (ray_box_o(d, soloc + item * 3, A, h, t, ax, sg) && t < best) {
                            best = t;
                            hit = b;
                            fc = ax * 2 + (sg > 0.0f ? 1 : 0);
                        }
                    }
                }
                uint16_t h0 = bg0, h1 = bg1, h2 = bg2;
                if (hit >= 0) {
                    const uint16_t* fh = sface + ((r * CP_NUM_BODIES + hit) * 6 + fc) * 3;
                    h0 = fh[0];
                    h1 = fh[1];
                    h2 = fh[2];
                }
                if (valid) {
                    sp[cam * R + r] = h0;
                    sp[F + cam * R + r] = h1;
                    sp[2 * F + cam * R + r] = h2;
                }
            }
        }
        wave_sync();
        // copy the strip: 16-byte blocks of the aligned span, partial blocks by halves
        const int nh = ((npx - p0) < WAVE_R ? (npx - p0) : WAVE_R) * per_px;
        const int tot = sh + nh;
        uint4* d4 = reinterpret_cast<uint4*>(dst - sh);
        const uint4* s4 = reinterpret_cast<const uint4*>(stage);
        for (int k = lane; k * 8 < tot; k += WAVE_R) {
            const int h0 = k * 8;
            if (h0 >= sh && h0 + 8 <= tot) {
                store_stream(&d4[k], s4[k]);
            } else {
                for (int e = (h0 > sh ? h0 : sh); e < (h0 + 8 < tot ? h0 + 8 : tot); ++e) dst[e - sh] = stage[e];
            }
        }
        wave_sync();
    }
}

// ---- small frames (the reference's 50 x 50): one block per env, dense ray tests ----
// Per frame an LDS code buffer holds, per pixel, what it shows: the static ground
// class (face 0..5, or 30 = background) to start with, then body b's face f as
// b * 6 + f once a box is nearer, with its depth in a depth buffer.  Every box is
// tested only over its own screen rectangle, densely (thread k of the block takes the
// rectangle's k-th pixel), one body after another in body order: the sequential
// "t < best" scan of the oracle with the pixels of one body in parallel (a pixel still
// showing the ground compares against the ground's t from the table).  The output
// pass maps codes to colours through a per-repeat LUT and streams strips of 64
// pixels out as cp_render_kernel does.
constexpr int CODE_BG = 30;  // background; codes 0..29 = body * 6 + face (body 0 = ground)
struct SmallLds {
    int lut, best, code, stage, total;
    RenderLds w;  // the scene part (its own face / stage fields unused)
};
__host__ __device__ inline SmallLds render_small_lds(int C, int R, int npx) {
    SmallLds s;
    s.w = render_lds(C, R);
    int o = s.w.face;  // the scene arrays before the face table are shared with RenderLds
    s.lut = o;   o = (o + R * 32 * 8 + 15) & ~15;  // [R][32] x 4 float16 (3 used)
    s.best = o;  o = (o + npx * 4 + 15) & ~15;
    s.code = o;  o = (o + C * R * npx + 15) & ~15;
    s.stage = o; o = (o + RENDER_WAVES * (WAVE_R * 3 * C * R + 8) * 2 + 15) & ~15;
    s.total = o;
    return s;
}
constexpr int SMALL_LDS_MAX = 48 * 1024;  // keeps >= 3 blocks (12 waves) per CU

__global__ void __launch_bounds__(RENDER_WAVES * WAVE_R) cp_render_small_kernel(
    cp_raster_config rc, cp_physics P, int R, const int32_t* list, const int32_t* count, const float* poses,
    const float4* tabd, const uint8_t* cls, uint16_t* pixels) {
    extern __shared__ __align__(16) unsigned char render_lds_raw[];
    if ((int)blockIdx.x >= *count) return;  // block-uniform
    const int env = list[blockIdx.x];
    const int tid = threadIdx.x, wave = tid / WAVE_R, lane = tid % WAVE_R;
    constexpr int NT = RENDER_WAVES * WAVE_R;
    const int W = rc.width, H = rc.height, C = rc.num_cameras, npx = W * H;
    const int per_px = 3 * C * R, F = C * R;
    const SmallLds L = render_small_lds(C, R, npx);
    unsigned char* base = render_lds_raw;
    float* sax = reinterpret_cast<float*>(base + L.w.ax);
    float* sc = reinterpret_cast<float*>(base + L.w.c);
    float* soloc = reinterpret_cast<float*>(base + L.w.oloc);
    int16_t* srect = reinterpret_cast<int16_t*>(base + L.w.rect);
    uint2* slut = reinterpret_cast<uint2*>(base + L.lut);
    float* sbest = reinterpret_cast<float*>(base + L.best);
    uint8_t* scode = reinterpret_cast<uint8_t*>(base + L.code);
    uint16_t* stage = reinterpret_cast<uint16_t*>(base + L.stage) + wave * (WAVE_R * per_px + 8);

    const float* pe = poses + (size_t)env * R * CP_NUM_DYN * 7;
    if (tid < R * CP_NUM_DYN) {
        const float* q = pe + tid * 7;
        const Axes A = quat_axes(q[3], q[4], q[5], q[6]);
        float* a9 = sax + tid * 9;
        a9[0] = A.a0.x; a9[1] = A.a0.y; a9[2] = A.a0.z;
        a9[3] = A.a1.x; a9[4] = A.a1.y; a9[5] = A.a1.z;
        a9[6] = A.a2.x; a9[7] = A.a2.y; a9[8] = A.a2.z;
        sc[tid * 3 + 0] = q[0]; sc[tid * 3 + 1] = q[1]; sc[tid * 3 + 2] = q[2];
    }
    // every frame starts as the static ground / background (class 6 -> CODE_BG)
    for (int cam = 0; cam < C; ++cam) {
        if ((npx & 3) == 0) {  // 4 pixels per thread and step (class 6 -> 30: add 24 to bytes >= 6)
            const uint32_t* c4 = reinterpret_cast<const uint32_t*>(cls + (size_t)cam * npx);
            for (int k = tid; k < npx / 4; k += NT) {
                uint32_t v = c4[k];
                const uint32_t ge6 = ((v | 0x80808080u) - 0x06060606u) & 0x80808080u;  // per byte: v >= 6
                v += (ge6 >> 7) * 24u;
                for (int r = 0; r < R; ++r) reinterpret_cast<uint32_t*>(scode + (cam * R + r) * npx)[k] = v;
            }
        } else {
            for (int p = tid; p < npx; p += NT) {
                const int cl = cls[(size_t)cam * npx + p];
                for (int r = 0; r < R; ++r) scode[(cam * R + r) * npx + p] = (uint8_t)(cl < 6 ? cl : CODE_BG);
            }
        }
    }
    __syncthreads();
    const float syk = rc.tan_half_fov;
    const float sxk = rc.tan_half_fov * ((float)W / (float)H);
    if (tid < F * CP_NUM_DYN) {
        const int cam = tid / (R * CP_NUM_DYN), rb = tid % (R * CP_NUM_DYN), b = rb % CP_NUM_DYN;
        const Cam k = make_cam(rc, cam);
        const float* a9 = sax + rb * 9;
        Axes A;
        A.a0 = mk(a9[0], a9[1], a9[2]); A.a1 = mk(a9[3], a9[4], a9[5]); A.a2 = mk(a9[6], a9[7], a9[8]);
        const V3 c = mk(sc[rb * 3 + 0], sc[rb * 3 + 1], sc[rb * 3 + 2]);
        const V3 oc = sub(k.eye, c);
        soloc[tid * 3 + 0] = dot(oc, A.a0);
        soloc[tid * 3 + 1] = dot(oc, A.a1);
        soloc[tid * 3 + 2] = dot(oc, A.a2);
        int16_t q[4];
        box_rect(k, c, A, mk(P.half_extents[b + 1][0], P.half_extents[b + 1][1], P.half_extents[b + 1][2]), sxk,
                 syk, W, H, q);
        // clipped to the image (empty: x0 > x1)
        srect[tid * 4 + 0] = q[0] < 0 ? 0 : q[0];
        srect[tid * 4 + 1] = q[1] > W - 1 ? (int16_t)(W - 1) : q[1];
        srect[tid * 4 + 2] = q[2] < 0 ? 0 : q[2];
        srect[tid * 4 + 3] = q[3] > H - 1 ? (int16_t)(H - 1) : q[3];
    }
    const V3 light = mk(rc.light[0], rc.light[1], rc.light[2]);
    for (int it = tid; it < R * 32; it += NT) {  // colour LUT [r][code]
        const int r = it / 32, code = it % 32;
        uint16_t h[3];
        if (code < CP_NUM_BODIES * 6) {
            const int b = code / 6, fc = code % 6, ax = fc >> 1;
            const float sg = (fc & 1) ? 1.0f : -1.0f;
            V3 an;
            if (b == 0) {
                an = ax == 0 ? mk(1.0f, 0.0f, 0.0f) : (ax == 1 ? mk(0.0f, 1.0f, 0.0f) : mk(0.0f, 0.0f, 1.0f));
            } else {
                const float* a9 = sax + (r * CP_NUM_DYN + b - 1) * 9 + 3 * ax;
                an = mk(a9[0], a9[1], a9[2]);
            }
            const float ndl = dot(scl(an, sg), light);
            const float sh = fmaf_(rc.diffuse, ndl > 0.0f ? ndl : 0.0f, rc.ambient);
            for (int ch = 0; ch < 3; ++ch) h[ch] = u8_to_half(to_u8(rc.color[b][ch] * sh));
        } else {
            for (int ch = 0; ch < 3; ++ch) h[ch] = u8_to_half(to_u8(rc.background[ch]));
        }
        slut[it] = make_uint2((uint32_t)h[0] | ((uint32_t)h[1] << 16), (uint32_t)h[2]);
    }
    __syncthreads();

    // dense ray tests: frame by frame, body by body
    for (int f = 0; f < F; ++f) {
        const int cam = f / R, r = f % R;
        uint8_t* cf = scode + f * npx;
        for (int b = 1; b < CP_NUM_BODIES; ++b) {
            const int item = f * CP_NUM_DYN + b - 1;
            const int x0 = srect[item * 4 + 0], x1 = srect[item * 4 + 1];
            const int y0 = srect[item * 4 + 2], y1 = srect[item * 4 + 3];
            if (x0 > x1 || y0 > y1) continue;  // block-uniform
            const int rw = x1 - x0 + 1, area = rw * (y1 - y0 + 1);
            const float inv_rw = 1.0f / (float)rw;
            const float* a9 = sax + (r * CP_NUM_DYN + b - 1) * 9;
            Axes A;
            A.a0 = mk(a9[0], a9[1], a9[2]); A.a1 = mk(a9[3], a9[4], a9[5]); A.a2 = mk(a9[6], a9[7], a9[8]);
            const V3 h = mk(P.half_extents[b][0], P.half_extents[b][1], P.half_extents[b][2]);
            const float* ol = soloc + item * 3;
            for (int k = tid; k < area; k += NT) {
                int yy = (int)((float)k * inv_rw), xx = k - yy * rw;  // k / rw, corrected
                if (xx < 0) { --yy; xx += rw; }
                if (xx >= rw) { ++yy; xx -= rw; }
                const int p = (y0 + yy) * W + x0 + xx;
                const float4 t0 = tabd[(size_t)cam * npx + p];
                float t, sg;
                int ax;
                if (ray_box_o(mk(t0.x, t0.y, t0.z), ol, A, h, t, ax, sg)) {
                    const int cur = cf[p];
                    const float best = (cur < 6 || cur == CODE_BG) ? t0.w : sbest[p];
                    if (t < best) {
                        sbest[p] = t;
                        cf[p] = (uint8_t)(b * 6 + ax * 2 + (sg > 0.0f ? 1 : 0));
                    }
                }
            }
            __syncthreads();  // the next body compares against this one's hits
        }
    }

    // colours, strips of 64 pixels per wave
    uint16_t* out = pixels + (size_t)env * npx * per_px;
    for (int p0 = wave * WAVE_R; p0 < npx; p0 += RENDER_WAVES * WAVE_R) {
        const int p = p0 + lane;
        const bool valid = p < npx;
        const int pl = valid ? p : npx - 1;
        uint16_t* dst = out + (size_t)p0 * per_px;
        const int sh = (int)((reinterpret_cast<uintptr_t>(dst) & 15) >> 1);
        uint16_t* sp = stage + sh + lane * per_px;
        for (int f = 0; f < F; ++f) {
            const uint2 c = slut[(f % R) * 32 + scode[f * npx + pl]];
            if (valid) {
                sp[f] = (uint16_t)c.x;
                sp[F + f] = (uint16_t)(c.x >> 16);
                sp[2 * F + f] = (uint16_t)c.y;
            }
        }
        wave_sync();
        const int nh = ((npx - p0) < WAVE_R ? (npx - p0) : WAVE_R) * per_px;
        const int tot = sh + nh;
        uint4* d4 = reinterpret_cast<uint4*>(dst - sh);
        const uint4* s4 = reinterpret_cast<const uint4*>(stage);
        for (int k = lane; k * 8 < tot; k += WAVE_R) {
            const int h0 = k * 8;
            if (h0 >= sh && h0 + 8 <= tot) {
                store_stream(&d4[k], s4[k]);
            } else {
                for (int e = (h0 > sh ? h0 : sh); e < (h0 + 8 < tot ? h0 + 8 : tot); ++e) dst[e - sh] = stage[e];
            }
        }
        wave_sync();
    }
}

// ---- small frames, v2 (round 4): the same images as cp_render_small_kernel, fewer instructions.
// For NF = C * R frames known at compile time: the code buffer holds one word per pixel with the
// pixel's NF codes in 5-bit fields (frame f at bits 5 f, seeded with the static class; 16 bits for
// NF <= 3, 32 for NF <= 6), so the colour pass reads a pixel's codes with one load and no class
// lookup, and the buffer (5 KB at 50 x 50, NF = 3) leaves room for 8 blocks (32 waves) per CU; the
// pixel's 3 * NF float16 values are assembled in registers and staged with dword writes (one 16-bit
// write at an odd start) instead of 3 * NF 16-bit writes; the box rectangles use the hardware
// reciprocal (box_rect<true>).  The dense ray tests, the colour LUT and the strip stores are
// cp_render_small_kernel's.
struct Small2Lds {
    int lut, best, code, stage, total;
    RenderLds w;
};
template <bool SHORT> struct CodeWordT { using T = uint32_t; };
template <> struct CodeWordT<true> { using T = uint16_t; };
template <int NF> using CodeWord = typename CodeWordT<(NF <= 3)>::T;
// per wave: the strip's 512 values between two 24-value margins (a pixel's 3 * NF <= 24 values overhang a
// strip edge by less than that; 16-byte multiples)
template <int NF>
__host__ __device__ constexpr int small2_stage_halves() { return 24 + WAVE_R * 8 + 24; }
constexpr int SMALL2_SPT = 2;  // strips per trip of the colour pass (independent chains between syncs)
template <int NF>
__host__ __device__ inline Small2Lds render_small2_lds(int C, int R, int npx) {
    static_assert(NF <= 6, "five-bit code fields: at most 6 frames in a word");
    Small2Lds s;
    s.w = render_lds(C, R);
    int o = s.w.face;
    s.lut = o;   o = (o + R * 32 * 8 + 15) & ~15;
    // the dense pass's depth buffer and, after it, the colour pass's stages (two strips per wave) share
    // one region: they are never live together
    const int stage_bytes = RENDER_WAVES * SMALL2_SPT * small2_stage_halves<NF>() * 2;
    s.best = o;
    s.stage = o; o = (o + (npx * 4 > stage_bytes ? npx * 4 : stage_bytes) + 15) & ~15;
    s.code = o;  o = (o + npx * (int)sizeof(CodeWord<NF>) + 15) & ~15;
    s.total = o;
    return s;
}

template <int CC, int RR>
__global__ void __launch_bounds__(RENDER_WAVES * WAVE_R) cp_render_small2_kernel(
    cp_raster_config rc, cp_physics P, const int32_t* list, const int32_t* count, const float* poses,
    const float4* tabd, const uint8_t* cls, uint16_t* pixels) {
    constexpr int R = RR, NF = CC * RR;  // cameras and repeats at compile time (the launcher checks them)
    constexpr int PP = 3 * NF, NT = RENDER_WAVES * WAVE_R;
    using CWord = CodeWord<NF>;
    extern __shared__ __align__(16) unsigned char render_lds_raw[];
    if ((int)blockIdx.x >= *count) return;  // block-uniform
    const int env = list[blockIdx.x];
    const int tid = threadIdx.x, wave = tid / WAVE_R, lane = tid % WAVE_R;
    constexpr int C = CC;
    const int W = rc.width, H = rc.height, npx = W * H;
    const Small2Lds L = render_small2_lds<NF>(C, R, npx);
    unsigned char* base = render_lds_raw;
    float* sax = reinterpret_cast<float*>(base + L.w.ax);
    float* soloc = reinterpret_cast<float*>(base + L.w.oloc);
    int16_t* srect = reinterpret_cast<int16_t*>(base + L.w.rect);
    uint2* slut = reinterpret_cast<uint2*>(base + L.lut);
    float* sbest = reinterpret_cast<float*>(base + L.best);
    CWord* scw = reinterpret_cast<CWord*>(base + L.code);
    uint16_t* stage = reinterpret_cast<uint16_t*>(base + L.stage) + wave * SMALL2_SPT * small2_stage_halves<NF>();

    // the scene in one phase (one barrier): wave 0 the box axes for the dense pass, wave 1 the camera-space
    // terms and screen rectangles, waves 2-3 (then 0-1) the colour LUT, all threads the class seeding;
    // the rectangle and LUT threads take their boxes' axes from the poses themselves (quat_axes, the
    // same arithmetic as wave 0's, so the same bits) instead of waiting for wave 0's LDS writes
    const float* pe = poses + (size_t)env * R * CP_NUM_DYN * 7;
    if (tid < R * CP_NUM_DYN) {
        const float* q = pe + tid * 7;
        const Axes A = quat_axes(q[3], q[4], q[5], q[6]);
        float* a9 = sax + tid * 9;
        a9[0] = A.a0.x; a9[1] = A.a0.y; a9[2] = A.a0.z;
        a9[3] = A.a1.x; a9[4] = A.a1.y; a9[5] = A.a1.z;
        a9[6] = A.a2.x; a9[7] = A.a2.y; a9[8] = A.a2.z;
    }
    // every frame starts as its static class (the ground face the pixel's ray hits, or the background;
    // cls, L1-resident): field f of pixel p = class of p in camera f / R.  The dense pass compares a
    // pixel whose field still holds a static class against the ground's t from the table
    auto seed_word = [&](uint32_t c0, uint32_t c1) -> uint32_t {
        c0 = c0 < 6 ? c0 : CODE_BG;
        c1 = c1 < 6 ? c1 : CODE_BG;
        uint32_t w = 0;
#pragma unroll
        for (int f = 0; f < NF; ++f) w |= (f < R ? c0 : c1) << (5 * f);
        return w;
    };
    if ((npx & 3) == 0) {  // four pixels per class load (both cameras' rows 4-byte aligned), one LDS write
        const uint32_t* c32 = reinterpret_cast<const uint32_t*>(cls);
        for (int k = tid; k < (npx >> 2); k += NT) {
            const uint32_t a0 = c32[k], a1 = C > 1 ? c32[(npx >> 2) + k] : a0;
            uint32_t w[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) w[j] = seed_word((a0 >> (8 * j)) & 0xFFu, (a1 >> (8 * j)) & 0xFFu);
            if constexpr (sizeof(CWord) == 2) {
                reinterpret_cast<uint2*>(scw)[k] = make_uint2(w[0] | (w[1] << 16), w[2] | (w[3] << 16));
            } else {
                reinterpret_cast<uint4*>(scw)[k] = make_uint4(w[0], w[1], w[2], w[3]);
            }
        }
    } else {
#pragma unroll 4
        for (int k = tid; k < npx; k += NT) {
            const uint32_t c0 = cls[k];
            scw[k] = (CWord)seed_word(c0, C > 1 ? cls[(size_t)npx + k] : c0);
        }
    }
    const float syk = rc.tan_half_fov;
    const float sxk = rc.tan_half_fov * ((float)W / (float)H);
    static_assert(NF * CP_NUM_DYN <= WAVE_R, "one rectangle per lane of wave 1");
    if (tid >= WAVE_R && tid < WAVE_R + NF * CP_NUM_DYN) {
        const int item = tid - WAVE_R;
        const int cam = item / (R * CP_NUM_DYN), rb = item % (R * CP_NUM_DYN), b = rb % CP_NUM_DYN;
        const Cam k = make_cam(rc, cam);
        const float* qp = pe + rb * 7;
        const Axes A = quat_axes(qp[3], qp[4], qp[5], qp[6]);
        const V3 c = mk(qp[0], qp[1], qp[2]);
        const V3 oc = sub(k.eye, c);
        soloc[item * 3 + 0] = dot(oc, A.a0);
        soloc[item * 3 + 1] = dot(oc, A.a1);
        soloc[item * 3 + 2] = dot(oc, A.a2);
        int16_t q[4];
        box_rect<true>(k, c, A, mk(P.half_extents[b + 1][0], P.half_extents[b + 1][1], P.half_extents[b + 1][2]),
                       sxk, syk, W, H, q);
        srect[item * 4 + 0] = q[0] < 0 ? 0 : q[0];
        srect[item * 4 + 1] = q[1] > W - 1 ? (int16_t)(W - 1) : q[1];
        srect[item * 4 + 2] = q[2] < 0 ? 0 : q[2];
        srect[item * 4 + 3] = q[3] > H - 1 ? (int16_t)(H - 1) : q[3];
    }
    const V3 light = mk(rc.light[0], rc.light[1], rc.light[2]);
    for (int it = (tid + 2 * WAVE_R) % NT; it < R * 32; it += NT) {  // colour LUT [r][code] (cp_render_small_kernel's)
        const int r = it / 32, code = it % 32;
        uint16_t h[3];
        if (code < CP_NUM_BODIES * 6) {
            const int b = code / 6, fc = code % 6, ax = fc >> 1;
            const float sg = (fc & 1) ? 1.0f : -1.0f;
            V3 an;
            if (b == 0) {
                an = ax == 0 ? mk(1.0f, 0.0f, 0.0f) : (ax == 1 ? mk(0.0f, 1.0f, 0.0f) : mk(0.0f, 0.0f, 1.0f));
            } else {
                const float* qp = pe + (r * CP_NUM_DYN + b - 1) * 7;
                const Axes A = quat_axes(qp[3], qp[4], qp[5], qp[6]);
                an = ax == 0 ? A.a0 : (ax == 1 ? A.a1 : A.a2);
            }
            const float ndl = dot(scl(an, sg), light);
            const float sh = fmaf_(rc.diffuse, ndl > 0.0f ? ndl : 0.0f, rc.ambient);
            for (int ch = 0; ch < 3; ++ch) h[ch] = u8_to_half(to_u8(rc.color[b][ch] * sh));
        } else {
            for (int ch = 0; ch < 3; ++ch) h[ch] = u8_to_half(to_u8(rc.background[ch]));
        }
        slut[it] = make_uint2((uint32_t)h[0] | ((uint32_t)h[1] << 16), (uint32_t)h[2]);
    }
    __syncthreads();

    // dense ray tests: frame by frame, body by body (cp_render_small_kernel's, pixel-major codes)
#pragma unroll 1
    for (int f = 0; f < NF; ++f) {
        const int cam = f / R, r = f % R;
        for (int b = 1; b < CP_NUM_BODIES; ++b) {
            const int item = f * CP_NUM_DYN + b - 1;
            const int x0 = srect[item * 4 + 0], x1 = srect[item * 4 + 1];
            const int y0 = srect[item * 4 + 2], y1 = srect[item * 4 + 3];
            if (x0 > x1 || y0 > y1) continue;  // block-uniform
            const int rw = x1 - x0 + 1, area = rw * (y1 - y0 + 1);
            const float inv_rw = 1.0f / (float)rw;
            const float* a9 = sax + (r * CP_NUM_DYN + b - 1) * 9;
            Axes A;
            A.a0 = mk(a9[0], a9[1], a9[2]); A.a1 = mk(a9[3], a9[4], a9[5]); A.a2 = mk(a9[6], a9[7], a9[8]);
            const V3 h = mk(P.half_extents[b][0], P.half_extents[b][1], P.half_extents[b][2]);
            const float* ol = soloc + item * 3;
            for (int k = tid; k < area; k += NT) {
                int yy = (int)((float)k * inv_rw), xx = k - yy * rw;  // k / rw, corrected
                if (xx < 0) { --yy; xx += rw; }
                if (xx >= rw) { ++yy; xx -= rw; }
                const int p = (y0 + yy) * W + x0 + xx;
                const float4 t0 = tabd[(size_t)cam * npx + p];
                float t, sg;
                int ax;
                if (ray_box_o(mk(t0.x, t0.y, t0.z), ol, A, h, t, ax, sg)) {
                    const uint32_t w = scw[p];
                    const int cur = (int)((w >> (5 * f)) & 31u);
                    const float best = (cur < 6 || cur == CODE_BG) ? t0.w : sbest[p];
                    if (t < best) {
                        sbest[p] = t;
                        const uint32_t c = (uint32_t)(b * 6 + ax * 2 + (sg > 0.0f ? 1 : 0));
                        scw[p] = (CWord)((w & ~(31u << (5 * f))) | (c << (5 * f)));
                    }
                }
            }
            __syncthreads();  // the next body compares against this one's hits
        }
    }

    // colours, in strips of 64 output chunks: chunk q is the 16 bytes at out + 16 q - (out mod 16), so
    // every strip is 16-byte aligned and each lane stores one whole chunk; the pixels overlapping the
    // strip's 512 values (<= 59) are computed one per lane (a pixel cut by a strip edge is computed by
    // both strips), their 3 * NF values assembled in registers and staged with dword writes at their
    // position relative to the strip; only the env's first and last chunks are written by halves
    uint16_t* out = pixels + (size_t)env * npx * PP;
    const int N = npx * PP;                                             // the env's values
    const int sh = (int)((reinterpret_cast<uintptr_t>(out) & 15) >> 1);  // values before out in its chunk
    const int Q = (N + sh + 7) >> 3;                                     // chunks touched
    constexpr int M = 24;                                                // stage margin (>= PP, 16-byte multiple)
    static_assert(PP <= M, "small2_stage_halves: the margins must hold a pixel's values");
    uint4* d4 = reinterpret_cast<uint4*>(out - sh);
    constexpr int SH = small2_stage_halves<NF>();
    // two strips per trip (stage u = 0, 1): two independent load / LUT / stage chains between syncs;
    // wave w takes strips w, w + 4, w + 8, ... (in units of 64 chunks)
    for (int s0 = wave * WAVE_R; s0 < Q; s0 += SMALL2_SPT * RENDER_WAVES * WAVE_R) {
#pragma unroll
        for (int u = 0; u < SMALL2_SPT; ++u) {
            const int sa = s0 + u * RENDER_WAVES * WAVE_R;
            if (sa >= Q) break;  // wave-uniform
            uint16_t* st = stage + u * SH;
            const int g0 = sa * 8 - sh;                                 // the strip's first value (env-relative)
            const int glo = g0 > 0 ? g0 : 0;
            const int ghi = (g0 + WAVE_R * 8 < N ? g0 + WAVE_R * 8 : N) - 1;
            const int plo = glo / PP, np = ghi / PP - plo + 1;          // pixels overlapping the strip
            for (int i = lane; i < np; i += WAVE_R) {                   // one pass for 3 * NF >= 9
                const int p = plo + i;
                const uint32_t cw = scw[p];
                // the pixel's static class per camera (ground face or background), shown where no body is
                uint16_t hv[PP];
#pragma unroll
                for (int f = 0; f < NF; ++f) {
                    const int code = (int)((cw >> (5 * f)) & 31u);
                    const uint2 c = slut[(f % R) * 32 + code];
                    hv[f] = (uint16_t)c.x;
                    hv[NF + f] = (uint16_t)(c.x >> 16);
                    hv[2 * NF + f] = (uint16_t)c.y;
                }
                const int o = M + p * PP - g0;                          // in (M - PP, M + 512)
                // the PP values at st[o ..): without a branch on the parity a = o & 1 (PP is odd when
                // NF is, so neighbouring lanes differ): the full dwords hold values (2k + a, 2k + 1 + a)
                // at dword (o + a) / 2 + k; what is left over is one value (odd PP: the last one if a = 0,
                // the first if a = 1) or, for even PP and a = 1, the first and the last
                const int a = o & 1;
                uint32_t* s32 = reinterpret_cast<uint32_t*>(st) + ((o + a) >> 1);
                constexpr int NFULL = (PP - 1) / 2;
#pragma unroll
                for (int k = 0; k < NFULL; ++k) {
                    const uint32_t e = (uint32_t)hv[2 * k] | ((uint32_t)hv[2 * k + 1] << 16);
                    const uint32_t d = (uint32_t)hv[2 * k + 1] | ((uint32_t)hv[2 * k + 2] << 16);
                    s32[k] = a ? d : e;
                }
                if constexpr (PP & 1) {
                    st[a ? o : o + PP - 1] = a ? hv[0] : hv[PP - 1];
                } else {  // even PP: a = 0 leaves one more full pair, a = 1 the first and the last value
                    if (a) {
                        st[o] = hv[0];
                        st[o + PP - 1] = hv[PP - 1];
                    } else {
                        s32[NFULL] = (uint32_t)hv[PP - 2] | ((uint32_t)hv[PP - 1] << 16);
                    }
                }
            }
        }
        wave_sync();
#pragma unroll
        for (int u = 0; u < SMALL2_SPT; ++u) {
            const int q = s0 + u * RENDER_WAVES * WAVE_R + lane;
            const int e0 = q * 8 - sh;                                  // the chunk's first value
            if (q < Q) {
                const uint16_t* src = stage + u * SH + M + lane * 8;
                if (e0 >= 0 && e0 + 8 <= N) {
                    store_stream(&d4[q], *reinterpret_cast<const uint4*>(src));
                } else {  // the env's first / last chunk: its values only (the neighbour env owns the rest)
                    for (int e = 0; e < 8; ++e)
                        if (e0 + e >= 0 && e0 + e < N) out[e0 + e] = src[e];
                }
            }
        }
        wave_sync();
    }
}

}  // namespace cp
