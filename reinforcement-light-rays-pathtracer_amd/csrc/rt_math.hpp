// rt_math.hpp — scalar math shared by the host scene builder and the gfx950
// kernels.  Every function is written so that host (x86-64, SSE) and device
// (gfx950) evaluate the same IEEE-754 binary32 operations in the same order:
// build with -ffp-contract=off, correctly-rounded division and sqrt (hipcc's
// default), no fast-math.  The operation orders follow GLM 0.9.9.3 as vendored
// by the reference (glm/glm/detail/func_geometric.inl:48-89,
// func_matrix.inl:210-220) because the reference computes with GLM.
#pragma once

#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define RT_HD __host__ __device__ __forceinline__
#else
#include <math.h>
#define RT_HD inline
#endif

namespace rt {

struct f3 {
    float x, y, z;
};

RT_HD f3 make3(float x, float y, float z) {
    f3 r;
    r.x = x; r.y = y; r.z = z;
    return r;
}

// glm compute_dot<vec3>: tmp = a*b; (tmp.x + tmp.y) + tmp.z
RT_HD float dot(f3 a, f3 b) {
    float tx = a.x * b.x;
    float ty = a.y * b.y;
    float tz = a.z * b.z;
    return (tx + ty) + tz;
}

#if defined(__HIPCC__)
// Correctly rounded 1/x.  For |x| in [2^-125, 2^125], v_rcp_f32 (<= 1 ulp)
// refined by one Newton step in FMA; the result equals IEEE 1.0f/x bit for bit
// (verified over every float by rt_selftest(RT_SELFTEST_RCP), a GPU test).  Other
// inputs take hipcc's IEEE division sequence.
__device__ __forceinline__ float rcp_rn_from(float x, float r0) {
    const float ax = fabsf(x);
    const float e = fmaf(-x, r0, 1.0f);
    float r = fmaf(e, r0, r0);
    const bool out_of_range = !(ax >= 0x1p-125f && ax <= 0x1p125f);
    if (__builtin_amdgcn_ballot_w64(out_of_range) != 0ull) {  // wave-uniform, rare
        const float q = 1.0f / x;
        r = out_of_range ? q : r;
    }
    return r;
}
__device__ __forceinline__ float rcp_rn(float x) { return rcp_rn_from(x, __builtin_amdgcn_rcpf(x)); }

// x / 12 for x = +0 or |x| in [2^-100, 2^100]: q = RN(x c), c = RN(1/12), corrected
// by one FMA residual step; equal to IEEE x / 12.0f over that whole range (checked
// exhaustively over every float on the host, tools/check_div12.c; -0 gives +0).
// The grid coordinates gx = cell + jitter are +0 or in [2^-24, 12].
__device__ __forceinline__ float div12(float x) {
    const float c = 1.0f / 12.0f;
    const float q = x * c;
    const float r = fmaf(-q, 12.0f, x);
    return fmaf(r, c, q);
}
#endif

#if defined(__HIPCC__)
// x / RHO, RHO = RN(1 / (2 RN(pi))) (GPU/constants/image_settings.h:14): q = RN(x c),
// c = RN(1/RHO), corrected by one FMA residual step; equal to IEEE x / RHO for every
// float x = +-0 or |x| in [2^-100, 2^100] (checked exhaustively on the host,
// tools/check_divrho.c: 0 mismatches; zeros pass through so -0 keeps its sign).  Other
// inputs (rare; wave-uniform test) take the division.
__device__ __forceinline__ float div_rho(float x) {
    constexpr float rho = 1.0f / (2.0f * 3.14159265358979323846f);
    constexpr float c = 1.0f / rho;
    const float q = x * c;
    const float r = fmaf(-q, rho, x);
    float y = (x == 0.0f) ? x : fmaf(r, c, q);
    const float ax = fabsf(x);
    const bool out_of_range = !(ax >= 0x1p-100f && ax <= 0x1p100f) && (x != 0.0f);
    if (__builtin_amdgcn_ballot_w64(out_of_range) != 0ull) {
        const float d = x / rho;
        y = out_of_range ? d : y;
    }
    return y;
}
#endif

// glm normalize: v * inversesqrt(dot(v, v)), inversesqrt(x) = 1 / sqrt(x)
// (device: the reciprocal by rcp_rn, bit-identical to the division)
RT_HD f3 normalize(f3 v) {
#if defined(__HIP_DEVICE_COMPILE__)
    const float inv = rcp_rn(sqrtf(dot(v, v)));
#else
    const float inv = 1.0f / sqrtf(dot(v, v));
#endif
    return make3(v.x * inv, v.y * inv, v.z * inv);
}

// glm compute_cross
RT_HD f3 cross(f3 x, f3 y) {
    return make3(x.y * y.z - y.y * x.z, x.z * y.x - y.z * x.x, x.x * y.y - y.x * x.y);
}

#ifndef RT_XOR3
#define RT_XOR3 1
#endif
// a ^ b ^ c: one v_bitop3_b32 on gfx950 (the compiler emits two v_xor_b32 for it)
#if defined(__HIP_DEVICE_COMPILE__) && RT_XOR3
#define RT_XOR3F(a, b, c) __builtin_amdgcn_bitop3_b32((a), (b), (c), 0x96)
#else
#define RT_XOR3F(a, b, c) ((a) ^ (b) ^ (c))
#endif

// Philox4x32-10 (Salmon, Moraes, Dror, Shaw, SC'11).  Counter
// (pixel, sample, event, 0), key (seed_lo, seed_hi): DESIGN.md §3.
RT_HD void philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0,
                         uint32_t k1, uint32_t out[4]) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        uint64_t p0 = (uint64_t)0xD2511F53u * (uint64_t)c0;
        uint64_t p1 = (uint64_t)0xCD9E8D57u * (uint64_t)c2;
        uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        uint32_t n0 = RT_XOR3F(hi1, c1, k0);
        uint32_t n2 = RT_XOR3F(hi0, c3, k1);
        c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

// Philox4x32-10 blocks that differ only in the last counter word c3 (the DQN sampler's 47
// blocks of one ray: pixel, sample and event fixed, c3 = the draw): rounds 1-3 hold five
// products and xors that do not depend on c3, computed once (philox_shared) instead of per
// block; philox_from finishes a block -- the same words as philox4x32_10, bit for bit.
struct PhiloxShared {
    uint32_t r1_n0, r1_lo1, r1_x, r1_lo0;  // after round 1: (n0, lo1, n2 = r1_x ^ c3, lo0)
    uint32_t r2_hi0, r2_lo0;               // round 2's product of the shared word n0
    uint32_t k0, k1;                       // the key
};
RT_HD PhiloxShared philox_shared(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t k0, uint32_t k1) {
    PhiloxShared s;
    const uint64_t p0 = (uint64_t)0xD2511F53u * (uint64_t)c0;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * (uint64_t)c2;
    s.r1_n0 = RT_XOR3F((uint32_t)(p1 >> 32), c1, k0);
    s.r1_lo1 = (uint32_t)p1;
    s.r1_x = (uint32_t)(p0 >> 32) ^ k1;
    s.r1_lo0 = (uint32_t)p0;
    const uint64_t q0 = (uint64_t)0xD2511F53u * (uint64_t)s.r1_n0;
    s.r2_hi0 = (uint32_t)(q0 >> 32);
    s.r2_lo0 = (uint32_t)q0;
    s.k0 = k0;
    s.k1 = k1;
    return s;
}
RT_HD void philox_from(const PhiloxShared& s, uint32_t c3, uint32_t out[4]) {
    uint32_t k0 = s.k0 + 0x9E3779B9u, k1 = s.k1 + 0xBB67AE85u;
    // round 2: (n0, lo1, n2, lo0) of round 1 with n2 = r1_x ^ c3
    const uint32_t n2 = s.r1_x ^ c3;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * (uint64_t)n2;
    uint32_t c0 = RT_XOR3F((uint32_t)(p1 >> 32), s.r1_lo1, k0);
    uint32_t c1 = (uint32_t)p1;
    uint32_t c2 = RT_XOR3F(s.r2_hi0, s.r1_lo0, k1);
    uint32_t c3w = s.r2_lo0;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
#pragma unroll
    for (int r = 2; r < 10; ++r) {
        const uint64_t q0 = (uint64_t)0xD2511F53u * (uint64_t)c0;
        const uint64_t q1 = (uint64_t)0xCD9E8D57u * (uint64_t)c2;
        const uint32_t n0 = RT_XOR3F((uint32_t)(q1 >> 32), c1, k0);
        const uint32_t m2 = RT_XOR3F((uint32_t)(q0 >> 32), c3w, k1);
        c0 = n0;
        c1 = (uint32_t)q1;
        c2 = m2;
        c3w = (uint32_t)q0;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    out[0] = c0;
    out[1] = c1;
    out[2] = c2;
    out[3] = c3w;
}

// 24-bit uniform in [0, 1)
RT_HD float u01(uint32_t x) { return (float)(x >> 8) * 0x1p-24f; }
// the two 16-bit uniforms of one Philox word, k/2^16 in [0, 1) (the DQN sampler's cell
// jitters: 4 cells per draw)
RT_HD float u16lo(uint32_t x) { return (float)(x & 0xffffu) * 0x1p-16f; }
RT_HD float u16hi(uint32_t x) { return (float)(x >> 16) * 0x1p-16f; }
// 24-bit uniform in (0, 1], the range of curand_uniform (the SARSA sector draws: r = 0
// would select sector 0 of an all-zero-mass CDF prefix, which curand cannot)
RT_HD float u01_oc(uint32_t x) { return (float)((x >> 8) + 1u) * 0x1p-24f; }

// sin(2*pi*r), cos(2*pi*r) by quarter-turn reduction (exact) and Taylor
// polynomials of sin(pi/2 f), cos(pi/2 f) on f in [-1/2, 1/2] (Horner, no FMA).
RT_HD void sincos_turn(float r, float* s_out, float* c_out) {
    const float S1 = 1.57079632679489662f, S3 = -0.645964097506246254f,
                S5 = 0.0796926262461670451f, S7 = -0.00468175413531868810f,
                S9 = 0.000160441184757112456f;
    const float C2 = -1.23370055013616983f, C4 = 0.253669507901048014f,
                C6 = -0.0208634807633529609f, C8 = 0.000919260274839426046f,
                C10 = -0.0000252020423730606054f;
    float x = r * 4.0f;
    float q = rintf(x);
    float f = x - q;
    int qi = ((int)q) & 3;
    float f2 = f * f;
    float sp = S9;
    sp = sp * f2; sp = sp + S7;
    sp = sp * f2; sp = sp + S5;
    sp = sp * f2; sp = sp + S3;
    sp = sp * f2; sp = sp + S1;
    sp = sp * f;
    float cp = C10;
    cp = cp * f2; cp = cp + C8;
    cp = cp * f2; cp = cp + C6;
    cp = cp * f2; cp = cp + C4;
    cp = cp * f2; cp = cp + C2;
    cp = cp * f2; cp = cp + 1.0f;
    float s = (qi == 0) ? sp : (qi == 1) ? cp : (qi == 2) ? -sp : -cp;
    float c = (qi == 0) ? cp : (qi == 1) ? -sp : (qi == 2) ? -cp : sp;
    *s_out = s;
    *c_out = c;
}

// create_normal_coordinate_system (CPU/utils/hemisphere_helpers.cpp:26-39)
RT_HD void normal_frame(f3 n, f3* T, f3* B) {
    if (fabsf(n.x) > fabsf(n.y)) {
        *T = normalize(make3(n.z, 0.0f, -n.x));
    } else {
        *T = normalize(make3(0.0f, -n.z, n.y));
    }
    *B = cross(n, *T);
}

constexpr float kPi = 3.14159265358979323846f;  // (float)M_PI
constexpr float kEps = 1e-5f;                   // EPS / the 0.00001f offsets
constexpr int kGridRes = 12;                    // GRID_RESOLUTION (GPU/constants/radiance_volumes_settings.h:9)

// Chiu's square -> hemisphere map (GPU/utils/hemisphere_helpers.cu:123-226),
// restated in turns: cos(theta) = 1 - xx^2, sin(theta) = xx*sqrt(2 - xx^2),
// phi = offset + (yy/xx)/8 turns (the same angles; no acos/sin/cos of radians).
RT_HD void chiu_map(float x, float y, float* xr, float* yr, float* zr) {
    x = 2.0f * x - 1.0f;
    y = 2.0f * y - 1.0f;
    float xx, yy, off;
    bool origin = false;
    if (y > -x) {
        if (y < x) {
            xx = x;
            if (y > 0.0f) { off = 0.0f; yy = y; }
            else { off = 0.875f; yy = x + y; }
        } else {
            xx = y;
            if (x > 0.0f) { off = 0.125f; yy = y - x; }
            else { off = 0.25f; yy = -x; }
        }
    } else {
        if (y > x) {
            xx = -x;
            if (y > 0.0f) { off = 0.375f; yy = -x - y; }
            else { off = 0.5f; yy = -y; }
        } else {
            xx = -y;
            if (x > 0.0f) { off = 0.75f; yy = x; }
            else if (y != 0.0f) { off = 0.625f; yy = x - y; }
            else { origin = true; xx = 1.0f; yy = 0.0f; off = 0.0f; }
        }
    }
    const float c = 1.0f - xx * xx;
    const float s = xx * sqrtf(2.0f - xx * xx);
    const float phi = off + 0.125f * (yy / xx);
    float sp, cp;
    sincos_turn(phi, &sp, &cp);
    *xr = origin ? 0.0f : s * cp;
    *yr = origin ? 1.0f : c;
    *zr = origin ? 0.0f : s * sp;
}

// cos(theta) of the Chiu-map direction of grid point (gx, gy): the map's y component
// 1 - xx^2 with xx = max(|2x - 1|, |2y - 1|) (chiu_map's octant branches select exactly
// that), the origin giving 1.  The reference takes dot(N, normalize(M v - p)) of the
// world direction, the same angle up to float rounding.
RT_HD float chiu_cos(float gx, float gy) {
#if defined(__HIP_DEVICE_COMPILE__)
    // gx, gy in [0, 12]; 2 div12(g) is exact, so fma(2, d, -1) rounds once, as 2 d - 1 does
    const float x = fmaf(2.0f, div12(gx), -1.0f), y = fmaf(2.0f, div12(gy), -1.0f);
#else
    const float x = 2.0f * (gx / (float)kGridRes) - 1.0f, y = 2.0f * (gy / (float)kGridRes) - 1.0f;
#endif
    const float xx = fmaxf(fabsf(x), fabsf(y));
    return 1.0f - xx * xx;
}

// convert_grid_pos_to_direction(_random) (hemisphere_helpers.cu:95-121): map(gx/12, gy/12),
// world = mat4(T, N, B, pos) * (xh, yh, zh, 1) in glm order, direction = normalize(world - pos)
RT_HD f3 grid_direction(float gx, float gy, f3 N, f3 T, f3 B, f3 pos) {
    float xh, yh, zh;
#if defined(__HIP_DEVICE_COMPILE__)
    chiu_map(div12(gx), div12(gy), &xh, &yh, &zh);  // gx, gy in [0, 12]
#else
    chiu_map(gx / (float)kGridRes, gy / (float)kGridRes, &xh, &yh, &zh);
#endif
    const f3 w = make3((T.x * xh + N.x * yh) + (B.x * zh + pos.x * 1.0f),
                       (T.y * xh + N.y * yh) + (B.y * zh + pos.y * 1.0f),
                       (T.z * xh + N.z * yh) + (B.z * zh + pos.z * 1.0f));
    return normalize(make3(w.x - pos.x, w.y - pos.y, w.z - pos.z));
}

}  // namespace rt
