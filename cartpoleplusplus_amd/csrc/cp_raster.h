// cp_raster.h — in-kernel raster observation (--use-raw-pixels).
//
// Replaces render_rgb + set_state_element_for_repeat (bullet_cartpole.py:277-306):
// for every env, repeat r and camera c, an H x W RGB image of the 5 boxes, written
// as float16 [H][W][3][C][R] per env, the reference's state layout (:299-306).
//
// One 256-thread block per env (taken from a compacted env list).  The block
// stages the env's R poses and the cameras in LDS, projects every box to a
// conservative screen rectangle per (camera, repeat) and tabulates the shaded
// colour of every face; the per-pixel ray directions and the static ground's hits
// come from a per-camera table built once (cp_raster_table_kernel).  Each wave
// renders an 8 x 8 pixel tile (a thin pole's rectangle diverges few waves) for all
// C x R frames; an 8-row band is staged in LDS in the reference's pixel order and
// stored with 4-byte stores.
//
// The per-pixel arithmetic is the oracle's (oracle/cp_oracle.c, raster section),
// operation for operation; the rectangles only skip boxes a ray cannot hit.
#pragma once
#include <hip/hip_fp16.h>

#include "../../include/cartpole_amd.h"
#include "cp_math.h"

namespace cp {

constexpr int RT = 256;           // threads per render block
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

// LDS layout of one env's scene
struct Scene {
    Cam cam[2];                             // camera bases
    float ax[RMAX_FRAMES][CP_NUM_DYN][9];   // per repeat r (index < R) the body axes (columns)
    float c[RMAX_FRAMES][CP_NUM_DYN][3];    // and centres
    int16_t rect[2][RMAX_FRAMES][CP_NUM_BODIES][4];  // per camera, repeat, box: x0 x1 y0 y1 (pixels)
};

// conservative pixel rectangle of box (centre cc, axes A, half h) seen by camera k
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
        const float xs = dot(v, k.r) / (z * sxk), ys = dot(v, k.u) / (z * syk);
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
    out[0] = (int16_t)fmaxf(-lim, floorf(x0) - 2.0f);
    out[1] = (int16_t)fminf(lim, ceilf(x1) + 2.0f);
    out[2] = (int16_t)fmaxf(-lim, floorf(y0) - 2.0f);
    out[3] = (int16_t)fminf(lim, ceilf(y1) + 2.0f);
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
        const float inv = 1.0f / dd[i];
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
// kernel's own arithmetic.  table [C][H*W][2] float4: (d.xyz, t_ground), (hit, face).
__global__ void __launch_bounds__(RT) cp_raster_table_kernel(cp_raster_config rc, cp_physics P, float4* table) {
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
    int hit = -1, face = 0;
    float t, sg;
    int ax;
    if (ray_box_o(d, o, I3, mk(P.half_extents[0][0], P.half_extents[0][1], P.half_extents[0][2]), t, ax, sg) &&
        t < best) {
        best = t;
        hit = 0;
        face = ax * 2 + (sg > 0.0f ? 1 : 0);
    }
    table[((size_t)cam * npx + p) * 2 + 0] = make_float4(d.x, d.y, d.z, best);
    table[((size_t)cam * npx + p) * 2 + 1] = make_float4(__int_as_float(hit), __int_as_float(face), 0.0f, 0.0f);
}

// poses [B][R][4][7] (xyz, quat xyzw) -> pixels float16 [B][H][W][3][C][R] for the envs
// in list[0 .. *count).  Per pixel and camera the ground (static) is tested once and
// reused for every repeat; per (camera, repeat, body) the ray-independent terms are
// precomputed in LDS.  The oracle evaluates the same expressions per frame, so the
// images agree bit for bit.
__global__ void __launch_bounds__(RT) cp_render_kernel(cp_raster_config rc, cp_physics P, int R, const int32_t* list,
                                                        const int32_t* count, const float* poses, const float4* table,
                                                        uint16_t* pixels) {
    __shared__ Scene sc;
    __shared__ float oloc[2][RMAX_FRAMES][CP_NUM_DYN][3];  // (eye - c) . a_i per camera, repeat, body
    __shared__ uint16_t lut[256];                          // u8 -> float16 bits (:289-294)
    // shaded colour of every face: [repeat][box][axis * 2 + (sign > 0)][channel] as float16
    // bits (flat shading depends on the face only; same arithmetic as per pixel)
    __shared__ uint16_t face[RMAX_FRAMES][CP_NUM_BODIES][6][3];
    __shared__ uint16_t chunk[RT * 3 * RMAX_FRAMES];
    if ((int)blockIdx.x >= *count) return;  // block-uniform
    const int env = list[blockIdx.x];
    const int W = rc.width, H = rc.height, C = rc.num_cameras;
    const int per_px = 3 * C * R;           // halves per pixel
    const float* pe = poses + (size_t)env * R * CP_NUM_DYN * 7;
    const int tid = threadIdx.x;
    lut[tid] = u8_to_half(tid);
    if (tid < R * CP_NUM_DYN) {
        const int r = tid / CP_NUM_DYN, b = tid % CP_NUM_DYN;
        const float* q = pe + (r * CP_NUM_DYN + b) * 7;
        const Axes A = quat_axes(q[3], q[4], q[5], q[6]);
        float* a9 = sc.ax[r][b];
        a9[0] = A.a0.x; a9[1] = A.a0.y; a9[2] = A.a0.z;
        a9[3] = A.a1.x; a9[4] = A.a1.y; a9[5] = A.a1.z;
        a9[6] = A.a2.x; a9[7] = A.a2.y; a9[8] = A.a2.z;
        sc.c[r][b][0] = q[0]; sc.c[r][b][1] = q[1]; sc.c[r][b][2] = q[2];
    }
    if (tid < C) sc.cam[tid] = make_cam(rc, tid);
    __syncthreads();
    const float syk = rc.tan_half_fov;
    const float sxk = rc.tan_half_fov * ((float)W / (float)H);
    if (tid < C * R * CP_NUM_BODIES) {
        const int cam = tid / (R * CP_NUM_BODIES), r = (tid / CP_NUM_BODIES) % R, b = tid % CP_NUM_BODIES;
        const Cam k = sc.cam[cam];
        V3 cc;
        Axes A;
        if (b == 0) {
            cc = mk(0.0f, 0.0f, 0.0f);
            A.a0 = mk(1.0f, 0.0f, 0.0f); A.a1 = mk(0.0f, 1.0f, 0.0f); A.a2 = mk(0.0f, 0.0f, 1.0f);
        } else {
            const float* a9 = sc.ax[r][b - 1];
            cc = mk(sc.c[r][b - 1][0], sc.c[r][b - 1][1], sc.c[r][b - 1][2]);
            A.a0 = mk(a9[0], a9[1], a9[2]); A.a1 = mk(a9[3], a9[4], a9[5]); A.a2 = mk(a9[6], a9[7], a9[8]);
            const V3 oc = sub(k.eye, cc);
            oloc[cam][r][b - 1][0] = dot(oc, A.a0);  // (the oracle's ray_box computes these per ray)
            oloc[cam][r][b - 1][1] = dot(oc, A.a1);
            oloc[cam][r][b - 1][2] = dot(oc, A.a2);
        }
        box_rect(k, cc, A, mk(P.half_extents[b][0], P.half_extents[b][1], P.half_extents[b][2]), sxk, syk, W, H,
                 sc.rect[cam][r][b]);
    }
    const V3 light = mk(rc.light[0], rc.light[1], rc.light[2]);
    for (int it = tid; it < R * CP_NUM_BODIES * 6; it += RT) {
        const int r = it / (CP_NUM_BODIES * 6), b = (it / 6) % CP_NUM_BODIES, fc = it % 6;
        const int ax = fc >> 1;
        const float sg = (fc & 1) ? 1.0f : -1.0f;
        V3 an;
        if (b == 0) {
            an = ax == 0 ? mk(1.0f, 0.0f, 0.0f) : (ax == 1 ? mk(0.0f, 1.0f, 0.0f) : mk(0.0f, 0.0f, 1.0f));
        } else {
            const float* a9 = sc.ax[r][b - 1] + 3 * ax;
            an = mk(a9[0], a9[1], a9[2]);
        }
        const float ndl = dot(scl(an, sg), light);
        const float sh = fmaf_(rc.diffuse, ndl > 0.0f ? ndl : 0.0f, rc.ambient);
        face[r][b][fc][0] = u8_to_half(to_u8(rc.color[b][0] * sh));
        face[r][b][fc][1] = u8_to_half(to_u8(rc.color[b][1] * sh));
        face[r][b][fc][2] = u8_to_half(to_u8(rc.color[b][2] * sh));
    }
    __syncthreads();
    const uint16_t bgh0 = lut[to_u8(rc.background[0])], bgh1 = lut[to_u8(rc.background[1])],
                   bgh2 = lut[to_u8(rc.background[2])];
    const int npx = W * H;
    uint16_t* out = pixels + (size_t)env * npx * per_px;
    const bool words = (npx * per_px) % 2 == 0 && ((size_t)env * npx * per_px) % 2 == 0;

    // all C x R frames of pixel (px, py) -> dst[(ch * C + cam) * R + r] (the reference's
    // (3, C, R) order within a pixel)
    auto render_px = [&](int px, int py, uint64_t near, uint16_t* dst) {
        for (int cam = 0; cam < C; ++cam) {
            // ray direction and the static ground's hit, from the per-camera table
            const float4 t0 = table[((size_t)cam * npx + py * W + px) * 2 + 0];
            const float4 t1 = table[((size_t)cam * npx + py * W + px) * 2 + 1];
            const V3 d = mk(t0.x, t0.y, t0.z);
            const float best0 = t0.w;
            const int hit0 = __float_as_int(t1.x), face0 = __float_as_int(t1.y);
            for (int r = 0; r < R; ++r) {
                float best = best0;
                int hit = hit0, fc = face0;
#pragma unroll
                for (int b = 1; b < CP_NUM_BODIES; ++b) {
                    if (!((near >> ((cam * R + r) * 4 + b - 1)) & 1ull)) continue;  // wave-uniform
                    const int16_t* rect = sc.rect[cam][r][b];
                    if (px < rect[0] || px > rect[1] || py < rect[2] || py > rect[3]) continue;
                    const float* a9 = sc.ax[r][b - 1];
                    Axes A;
                    A.a0 = mk(a9[0], a9[1], a9[2]); A.a1 = mk(a9[3], a9[4], a9[5]); A.a2 = mk(a9[6], a9[7], a9[8]);
                    const V3 h = mk(P.half_extents[b][0], P.half_extents[b][1], P.half_extents[b][2]);
                    float t, sg;
                    int ax;
                    if (ray_box_o(d, oloc[cam][r][b - 1], A, h, t, ax, sg) && t < best) {
                        best = t;
                        hit = b;
                        fc = ax * 2 + (sg > 0.0f ? 1 : 0);
                    }
                }
                uint16_t h0 = bgh0, h1 = bgh1, h2 = bgh2;
                if (hit >= 0) {
                    const uint16_t* fh = face[r][hit][fc];
                    h0 = fh[0];
                    h1 = fh[1];
                    h2 = fh[2];
                }
                uint16_t* o = dst + cam * R + r;
                o[0] = h0;
                o[C * R] = h1;
                o[2 * C * R] = h2;
            }
        }
    };
    // copy `n` staged halves to out[first ...] (a contiguous span of the image)
    auto flush = [&](size_t first, int n) {
        if (words) {
            const uint32_t* src = reinterpret_cast<const uint32_t*>(chunk);
            uint32_t* dst = reinterpret_cast<uint32_t*>(out + first);
            for (int w = tid; w < n / 2; w += RT) dst[w] = src[w];
        } else {
            for (int w = tid; w < n; w += RT) out[first + w] = chunk[w];
        }
    };
    constexpr int TW = 8, TH = 8;  // one wave = an 8 x 8 pixel tile: a thin pole's rectangle
                                   // then diverges few waves, where a row strip hits them all
    constexpr int CHUNK = RT * 3 * RMAX_FRAMES;
    if (TH * W * per_px <= CHUNK) {
        // 8-row bands; per pass the 4 waves take 4 tiles side by side
        const int wv = tid / WAVE_R, ln = tid % WAVE_R;
        for (int y0 = 0; y0 < H; y0 += TH) {
            const int rows = H - y0 < TH ? H - y0 : TH;
            for (int x0 = 0; x0 < W; x0 += (RT / WAVE_R) * TW) {
                const int tx = x0 + wv * TW;
                const int px = tx + ln % TW, py = y0 + ln / TW;
                // bodies whose rectangle meets this wave's tile, one bit per (camera, repeat,
                // body): lane l tests item l, a ballot gathers them
                bool ov = false;
                if (ln < C * R * 4) {
                    const int16_t* rect = sc.rect[ln / (R * 4)][(ln / 4) % R][ln % 4 + 1];
                    ov = rect[0] <= tx + TW - 1 && rect[1] >= tx && rect[2] <= y0 + TH - 1 && rect[3] >= y0;
                }
                const uint64_t near = __ballot(ov);
                if (px < W && py < H) render_px(px, py, near, chunk + ((py - y0) * W + px) * per_px);
            }
            __syncthreads();
            flush((size_t)y0 * W * per_px, rows * W * per_px);
            __syncthreads();
        }
    } else {
        // wide images: row-major chunks of RT pixels
        for (int base = 0; base < npx; base += RT) {
            const int p = base + tid;
            if (p < npx) {
                const int py = p / W;
                render_px(p - py * W, py, ~0ull, chunk + tid * per_px);
            }
            __syncthreads();
            flush((size_t)base * per_px, (npx - base < RT ? npx - base : RT) * per_px);
            __syncthreads();
        }
    }
}

}  // namespace cp
