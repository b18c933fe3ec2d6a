// rt_trace.hpp — device-side building blocks shared by the path-trace
// megakernel (rt_kernels.hip) and the DQN wavefront kernels (rt_dqn.hip):
// the closest-hit loop with the reference's two hit predicates, the
// correctly-rounded reciprocal, and the Philox draws.
#pragma once

#include <float.h>

#include "rt_cull.hpp"
#include "rt_internal.hpp"

namespace rt {

// One pixel's RGB as a single 12-B store (global_store_dwordx3): three dword stores of a
// lone lane are three partial-line writes in the memory system's count
typedef float rgb3 __attribute__((ext_vector_type(3), aligned(4)));
__device__ __forceinline__ void store_rgb(float* dst, float r, float g, float b) {
    rgb3 v;
    v.x = r;
    v.y = g;
    v.z = b;
    *reinterpret_cast<rgb3*>(dst) = v;
}

constexpr float kRho = 1.0f / (2.0f * kPi);  // RHO: GPU/constants/image_settings.h:14

// Triangle records are read-only for a launch: loads through the constant address
// space are selected as scalar loads (SGPR broadcast) whenever the address is
// wave-uniform, even in kernels with global stores or atomics in the loop (the
// compiler otherwise falls back to per-lane vector loads of the same address there).
typedef float __attribute__((ext_vector_type(4))) f32x4_t;
typedef __attribute__((address_space(4))) const f32x4_t cfloat4;
__device__ __forceinline__ cfloat4* as_const(const float4* p) { return (cfloat4*)p; }
__device__ __forceinline__ float4 ldc(cfloat4* p) {
    const f32x4_t v = *p;
    return make_float4(v.x, v.y, v.z, v.w);
}

struct Hit {
    float t;
    int tri;
};

// Closest hit over the triangle soup.  D = dir * t_scale, A = [-D | e1 | e2],
// x = (t,u,v) by Cramer's rule with GLM's determinant order
// (glm/glm/detail/func_matrix.inl:214-217):
//   det(c0,c1,c2) = (c0.x*(c1.y*c2.z - c2.y*c1.z) - c1.x*(c0.y*c2.z - c2.y*c0.z))
//                   + c2.x*(c0.y*c1.z - c1.y*c0.z)
// The minors shared between detA, det_t, det_u and det_v are evaluated once
// (same operands, same order, so the same bits).
// RULE 0 = CPU triangle.cpp.o predicate (inv = 1/detA; accept t>=0, u>=0, v>=0,
//          u+v<=1, t < best+1e-5, t > 1e-5; best starts at FLT_MAX)
// RULE 1 = GPU/rays/ray.cu:63-64 (true divisions; t < best; best starts 999999)
// Build-time knobs (A/B experiments; defaults are the shipped configuration):
//   RT_HIT_MODE 0: exact; u/v behind a branch on the t test (skipped per wave)
//               1: exact, branch-free
//               2: conservative approximate rejection (v_rcp_f32) first; the
//                  exact IEEE test runs only for lanes it cannot reject
//   RT_UNROLL   unroll factor of the triangle loop
#ifndef RT_HIT_MODE
#define RT_HIT_MODE 2  // 7% faster than 0 on Cornell 512^2/256 spp, same image (profiles/r1_ab3.json)
#endif
#ifndef RT_UNROLL
#define RT_UNROLL 1
#endif
//   RT_FAST_RCP 1: 1/detA by rcp_rn (v_rcp_f32 + Newton, exhaustively verified)
#ifndef RT_FAST_RCP
#define RT_FAST_RCP 1
#endif
#if RT_FAST_RCP
#define RT_RCP(x) rcp_rn(x)
#else
#define RT_RCP(x) (1.0f / (x))
#endif

// rcp_rn / rcp_rn_from: rt_math.hpp

// Exact hit test of one triangle (the reference's arithmetic, see above).
template <int RULE>
__device__ __forceinline__ void exact_test_inv(float detA, float inv, float det_t, float det_u,
                                               float det_v, int i, Hit& h) {
    // RULE 0 with inv = RN(1/detA) already computed
    const float t = det_t * inv;
    const float u = det_u * inv;
    const float v = det_v * inv;
    if ((detA != 0.0f) && (t >= 0.0f) && (u >= 0.0f) && (v >= 0.0f) && ((u + v) <= 1.0f) &&
        (t < h.t + kEps) && (t > kEps)) {
        h.t = t;
        h.tri = i;
    }
}

template <int RULE>
__device__ __forceinline__ void exact_test(float detA, float det_t, float det_u, float det_v, int i,
                                           Hit& h) {
    if (RULE == 0) {
        const float inv = RT_RCP(detA);
        const float t = det_t * inv;
        const float u = det_u * inv;
        const float v = det_v * inv;
        if ((detA != 0.0f) && (t >= 0.0f) && (u >= 0.0f) && (v >= 0.0f) && ((u + v) <= 1.0f) &&
            (t < h.t + kEps) && (t > kEps)) {
            h.t = t;
            h.tri = i;
        }
    } else {
        const float t = det_t / detA;
        const float u = det_u / detA;
        const float v = det_v / detA;
        if ((detA != 0.0f) && (t >= 0.0f) && (u >= 0.0f) && (v >= 0.0f) && ((u + v) <= 1.0f) &&
            (t < h.t)) {
            h.t = t;
            h.tri = i;
        }
    }
}

template <int RULE>
__device__ __forceinline__ Hit closest_hit(const float4* __restrict__ tri_g, int n_tri, f3 o, f3 d,
                                           float t_scale) {
    cfloat4* __restrict__ tri = as_const(tri_g);
    const float nDx = -(d.x * t_scale);
    const float nDy = -(d.y * t_scale);
    const float nDz = -(d.z * t_scale);
    Hit h;
    h.t = (RULE == 0) ? FLT_MAX : 999999.0f;
    h.tri = -1;
#if RT_HIT_MODE == 2
    // upper bound of the t window, widened by 2^-18 (RULE 0: best + eps)
    float hi = ((RULE == 0) ? (h.t + kEps) : h.t) * (1.0f + 0x1p-18f);
#endif
#pragma unroll RT_UNROLL
    for (int i = 0; i < n_tri; ++i) {
        const float4 A = ldc(tri + i * kIsectF4 + 0);
        const float4 E1 = ldc(tri + i * kIsectF4 + 1);
        const float4 E2 = ldc(tri + i * kIsectF4 + 2);
        const float bx = o.x - A.x, by = o.y - A.y, bz = o.z - A.z;
        // detA = det(-D, e1, e2)
        const float s1 = nDy * E2.z - E2.y * nDz;
        const float s2 = nDy * E1.z - E1.y * nDz;
        const float detA = (nDx * A.w - E1.x * s1) + E2.x * s2;
        // det_t = det(b, e1, e2)
        const float s3 = by * E2.z - E2.y * bz;
        const float s4 = by * E1.z - E1.y * bz;
        const float det_t = (bx * A.w - E1.x * s3) + E2.x * s4;
#if RT_HIT_MODE == 0
        bool tpass;
        float inv = 0.0f;
        if (RULE == 0) {
            inv = RT_RCP(detA);
            const float t = det_t * inv;
            tpass = (detA != 0.0f) && (t >= 0.0f) && (t < h.t + kEps) && (t > kEps);
        } else {
            const float t = det_t / detA;
            tpass = (detA != 0.0f) && (t >= 0.0f) && (t < h.t);
        }
        if (tpass) {
            // det_u = det(-D, b, e2), det_v = det(-D, e1, b)
            const float s5 = nDy * bz - by * nDz;
            const float s6 = E1.y * bz - by * E1.z;
            const float det_u = (nDx * s3 - bx * s1) + E2.x * s5;
            const float det_v = (nDx * s6 - E1.x * s5) + bx * s2;
            exact_test<RULE>(detA, det_t, det_u, det_v, i, h);
        }
#else
        const float s5 = nDy * bz - by * nDz;
        const float s6 = E1.y * bz - by * E1.z;
        const float det_u = (nDx * s3 - bx * s1) + E2.x * s5;
        const float det_v = (nDx * s6 - E1.x * s5) + bx * s2;
#if RT_HIT_MODE == 1
        exact_test<RULE>(detA, det_t, det_u, det_v, i, h);
#else
        // Conservative rejection: with |detA| in [2^-100, 2^100], v_rcp_f32 is
        // within 1 ulp, so ta/ua/va differ from the exact t/u/v by < 2^-21
        // relative.  A lane is rejected only if the exact test must fail:
        //   ta < eps(1-2^-18) (RULE 0) or ta < -2^-90 (RULE 1)  =>  t fails
        //   ta > hi = (best [+eps]) (1+2^-18)                   =>  t fails
        //   ua or va < -2^-90 (no underflow to -0 possible)     =>  u/v fail
        //   ua + va > 1 + 2^-18 (with ua, va >= -2^-90)         =>  u+v > 1
        // NaN/inf or out-of-range detA never rejects.
        const float r = __builtin_amdgcn_rcpf(detA);
        const float ta = det_t * r, ua = det_u * r, va = det_v * r;
        const float ad = fabsf(detA);
        const float lo = (RULE == 0) ? kEps * (1.0f - 0x1p-18f) : -0x1p-90f;
        const bool sure_miss = (ad >= 0x1p-100f) && (ad <= 0x1p100f) &&
                               ((ta < lo) || (ta > hi) || (ua < -0x1p-90f) || (va < -0x1p-90f) ||
                                ((ua + va) > 1.0f + 0x1p-18f));
        if (!sure_miss) {
#if RT_FAST_RCP
            if (RULE == 0)
                exact_test_inv<RULE>(detA, rcp_rn_from(detA, r), det_t, det_u, det_v, i, h);
            else
                exact_test<RULE>(detA, det_t, det_u, det_v, i, h);
#else
            exact_test<RULE>(detA, det_t, det_u, det_v, i, h);
#endif
            hi = ((RULE == 0) ? (h.t + kEps) : h.t) * (1.0f + 0x1p-18f);
        }
#endif
#endif
    }
    return h;
}

// Exact test of triangle i, record loaded by this lane: the operations of
// closest_hit (same operands, same order), so the same bits.
template <int RULE>
__device__ __forceinline__ void exact_one(const float4* __restrict__ tri, int i, f3 o, float nDx,
                                          float nDy, float nDz, Hit& h) {
    const float4 A = tri[i * kIsectF4 + 0];
    const float4 E1 = tri[i * kIsectF4 + 1];
    const float4 E2 = tri[i * kIsectF4 + 2];
    const float bx = o.x - A.x, by = o.y - A.y, bz = o.z - A.z;
    const float s1 = nDy * E2.z - E2.y * nDz;
    const float s2 = nDy * E1.z - E1.y * nDz;
    const float detA = (nDx * A.w - E1.x * s1) + E2.x * s2;
    const float s3 = by * E2.z - E2.y * bz;
    const float s4 = by * E1.z - E1.y * bz;
    const float det_t = (bx * A.w - E1.x * s3) + E2.x * s4;
    const float s5 = nDy * bz - by * nDz;
    const float s6 = E1.y * bz - by * E1.z;
    const float det_u = (nDx * s3 - bx * s1) + E2.x * s5;
    const float det_v = (nDx * s6 - E1.x * s5) + bx * s2;
    exact_test<RULE>(detA, det_t, det_u, det_v, i, h);
}

// exact_one with a wave-uniform triangle index: the record arrives by scalar loads
// (same operands, same order, so the same bits).
template <int RULE>
__device__ __forceinline__ void exact_one_c(cfloat4* __restrict__ tri, int i, f3 o, float nDx,
                                            float nDy, float nDz, Hit& h) {
    const float4 A = ldc(tri + i * kIsectF4 + 0);
    const float4 E1 = ldc(tri + i * kIsectF4 + 1);
    const float4 E2 = ldc(tri + i * kIsectF4 + 2);
    const float bx = o.x - A.x, by = o.y - A.y, bz = o.z - A.z;
    const float s1 = nDy * E2.z - E2.y * nDz;
    const float s2 = nDy * E1.z - E1.y * nDz;
    const float detA = (nDx * A.w - E1.x * s1) + E2.x * s2;
    const float s3 = by * E2.z - E2.y * bz;
    const float s4 = by * E1.z - E1.y * bz;
    const float det_t = (bx * A.w - E1.x * s3) + E2.x * s4;
    const float s5 = nDy * bz - by * nDz;
    const float s6 = E1.y * bz - by * E1.z;
    const float det_u = (nDx * s3 - bx * s1) + E2.x * s5;
    const float det_v = (nDx * s6 - E1.x * s5) + bx * s2;
    exact_test<RULE>(detA, det_t, det_u, det_v, i, h);
}

// ---- Primary-ray culling (k_render_ps) ----
// A camera ray through pixel (px, py) with jitter (r1, r2) in [0, 1)^2 has direction
// d = Rf p / |p| (+ rounding), p = (px + r1 - W/2, py + r2 - H/2, H), Rf the camera's float
// rotation (camera_ray).  Over a pixel rectangle every filter quantity of
// closest_hit_filtered is a linear form a.d (or a constant): Ad = N.d, U = (o x e2 - G2).d,
// V = (-(o x e1) + G1).d, T = w0 - o.N, with o the camera position.  A triangle is culled
// for the rectangle when, for every such d, the filter's rejection holds with twice its
// margins -- the filter's float evaluation differs from these real values by at most
// 18u S (record and evaluation rounding), below the margins' c S = 256u S, so the filter
// would reject every one of these rays, and the filter rejects only pairs whose exact
// test fails (build_filter, rt_capi.cpp).  So a culled triangle cannot be the hit of any
// primary ray of the rectangle, and testing the others in index order gives the
// reference's hit bit for bit.
// CamRect, rect_cull: rt_cull.hpp (shared with the host for tests)

// Two-phase closest hit: the same Hit as closest_hit, bit for bit.
//
// The reference's predicate is the exact float Cramer test of every triangle in
// index order, each accepted hit narrowing the t window of the next.  Its result
// depends only on the triangles that pass the geometric part of the test
// (detA != 0, u >= 0, v >= 0, u + v <= 1, t > eps [RULE 0] / t >= 0 [RULE 1]),
// taken in index order.  Phase 1 (wave-uniform loop, records in SGPRs) evaluates
// the same quantities with 18 FMAs instead of 43 unfused operations, scaled by
// 1/t_scale and with the sign of the determinant folded in:
//   Ad = d.N,  T = w0 - o.N,  U = e2.R - d.G2,  V = -e1.R + d.G1   (R = d x o)
//   u = U/Ad,  v = V/Ad,  t = T/(t_scale Ad)
// and rejects a pair only when it is farther from the decision boundary than the
// combined rounding error of both evaluations (the per-triangle bounds eA, EW, ET
// of build_filter, rt_capi.cpp); the survivors set a bit of the lane's candidate
// mask.  Phase 2 runs the exact test (exact_one) on the candidates in index order.
// NaN/inf inputs never reject (the comparisons fail), and a zero direction leaves
// |Ad| <= eA, which never rejects either.
// Phase-1 quantities of one (ray, triangle) pair against filter record `f`,
// returned as three floats whose sign bits say "certain to fail":
//   x1 = eA - |Ad|        < 0  <=>  |Ad| > eA   (the sign of Ad is certain)
//   x2 = min(u,v,w) + EW  < 0  <=>  a barycentric test certainly fails
//   x3 = tm + ET          < 0  <=>  the t test certainly fails
// The exact test certainly fails iff x1 < 0 and (x2 < 0 or x3 < 0).  The sums are
// exact in sign (a nonzero exact sum never rounds to zero under gradual underflow,
// and an exact zero is +0), so each sign bit equals the comparison it stands for.
// Finite inputs only (the caller keeps every triangle of a non-finite ray).
template <int RULE>
__device__ __forceinline__ void filter_eval(cfloat4* __restrict__ f, f3 o, f3 d, float Rx,
                                            float Ry, float Rz, float ets, float* x1, float* x2,
                                            float* x3) {
    const float4 F0 = ldc(f + 0), F1 = ldc(f + 1), F2 = ldc(f + 2), F3 = ldc(f + 3), F4 = ldc(f + 4);
    const float ad = fmaf(d.x, F0.x, fmaf(d.y, F0.y, d.z * F0.z));
    const float tt = fmaf(-o.x, F0.x, fmaf(-o.y, F0.y, fmaf(-o.z, F0.z, F0.w)));
    const float uu = fmaf(F1.x, Rx, fmaf(F1.y, Ry, fmaf(F1.z, Rz,
                     fmaf(d.x, F2.x, fmaf(d.y, F2.y, d.z * F2.z)))));
    const float vv = fmaf(F3.x, Rx, fmaf(F3.y, Ry, fmaf(F3.z, Rz,
                     fmaf(d.x, F4.x, fmaf(d.y, F4.y, d.z * F4.z)))));
    const uint32_t sg = __float_as_uint(ad) & 0x80000000u;
    const float su = __uint_as_float(__float_as_uint(uu) ^ sg);
    const float sv = __uint_as_float(__float_as_uint(vv) ^ sg);
    const float st = __uint_as_float(__float_as_uint(tt) ^ sg);
    const float aa = fabsf(ad);
    const float w = (aa - su) - sv;
    const float m = fminf(fminf(su, sv), w);
    const float tm = (RULE == 0) ? fmaf(-ets, aa, st) : st;
    *x1 = F1.w - aa;
    *x2 = m + F2.w;
    *x3 = tm + F3.w;
}

// keep bit (bit 31) of one pair: NOT (x1 & (x2 | x3)) on the sign bits
__device__ __forceinline__ uint32_t keep_bit(float x1, float x2, float x3) {
    return ~(__float_as_uint(x1) & (__float_as_uint(x2) | __float_as_uint(x3)));
}

// Phase 1 over triangles [0, cnt) of one 32-triangle block `f`, in pairs (records
// padded to an even count), branch-free and all-VALU: each keep bit is shifted in
// at bit 0 (v_alignbit), so triangle j ends at bit cnt-1-j (the pad falls off the
// bottom).  `finite`: false for a ray with a non-finite component (keep all).
template <int RULE>
__device__ __forceinline__ uint32_t filter_block(cfloat4* __restrict__ f, int cnt, bool finite,
                                                 f3 o, f3 d, float Rx, float Ry, float Rz,
                                                 float ets) {
    uint32_t mask = 0u;
    const int cnt2 = (cnt + 1) & ~1;
#pragma clang loop vectorize(disable) unroll(disable)
    for (int j = 0; j < cnt2; j += 2) {
        float a1, a2, a3, b1, b2, b3;
        filter_eval<RULE>(f + j * kFiltF4, o, d, Rx, Ry, Rz, ets, &a1, &a2, &a3);
        filter_eval<RULE>(f + (j + 1) * kFiltF4, o, d, Rx, Ry, Rz, ets, &b1, &b2, &b3);
        mask = __builtin_amdgcn_alignbit(mask, keep_bit(a1, a2, a3), 31);
        mask = __builtin_amdgcn_alignbit(mask, keep_bit(b1, b2, b3), 31);
    }
    mask >>= (cnt2 - cnt);
    const uint32_t all = (cnt >= 32) ? 0xffffffffu : ((1u << cnt) - 1u);
    return finite ? mask : all;
}

template <int RULE>
__device__ __forceinline__ Hit closest_hit_filtered(const float4* __restrict__ filt,
                                                    const float4* __restrict__ tri, int n_tri, f3 o,
                                                    f3 d, float t_scale) {
    const float nDx = -(d.x * t_scale);
    const float nDy = -(d.y * t_scale);
    const float nDz = -(d.z * t_scale);
    const float Rx = fmaf(d.y, o.z, -(d.z * o.y));
    const float Ry = fmaf(d.z, o.x, -(d.x * o.z));
    const float Rz = fmaf(d.x, o.y, -(d.y * o.x));
    const float ets = kEps * t_scale;
    const bool finite = __builtin_isfinite(o.x) & __builtin_isfinite(o.y) & __builtin_isfinite(o.z) &
                        __builtin_isfinite(d.x) & __builtin_isfinite(d.y) & __builtin_isfinite(d.z);
    Hit h;
    h.t = (RULE == 0) ? FLT_MAX : 999999.0f;
    h.tri = -1;
    // 64 triangles per round: both masks first, then ONE divergent phase-2 loop over a
    // lane's candidates of the round in index order (the wave iterates the max over
    // lanes of the round's total instead of the sum of two per-block maxima; rounds of
    // 128 with a two-word mask measured slower).  Triangle base + i sits at bit
    // (c0 + c1 - 1 - i) of (m0 << c1 | m1).
    for (int base = 0; base < n_tri; base += 64) {
        const int c0 = min(32, n_tri - base);
        const int c1 = min(32, n_tri - base - 32);
        const uint32_t m0 =
            filter_block<RULE>(as_const(filt) + (size_t)base * kFiltF4, c0, finite, o, d, Rx, Ry, Rz, ets);
        uint32_t m1 = 0u;
        if (c1 > 0)
            m1 = filter_block<RULE>(as_const(filt) + (size_t)(base + 32) * kFiltF4, c1, finite, o, d, Rx, Ry,
                                    Rz, ets);
        uint64_t mm = ((uint64_t)m0 << (c1 > 0 ? c1 : 0)) | (uint64_t)m1;
        const int top = base + c0 + (c1 > 0 ? c1 : 0) - 1;
        while (mm != 0ull) {
            const int b = 63 - __builtin_clzll(mm);
            mm ^= 1ull << b;
            exact_one<RULE>(tri, top - b, o, nDx, nDy, nDz, h);
        }
    }
    return h;
}

// ---- The filter on the matrix cores (rays from surface points) ----
// closest_hit_filtered spends 31 VALU instructions per (ray, triangle) pair, 18 of them
// the four dot products A, T, U, V.  closest_hit_mf evaluates those on
// v_mfma_f32_16x16x32_bf16 (features and rows split into bf16 hi + lo, three products
// per term: rt_internal.hpp, kMfRound) and keeps 10 VALU instructions per pair for
// the tests, at margins 16x wider (c = 2^-12) than the fp32 filter's, folded into the
// rows' scale (build_mf_rows in rt_capi.cpp): no per-triangle margin loads.  Wave-level: every lane of the wave calls it
// (`active` false: a lane whose result is not used; it gets no candidates).
typedef __bf16 mf_bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 mf_bf16x2 __attribute__((ext_vector_type(2)));
typedef float mf_f32x4 __attribute__((ext_vector_type(4)));
typedef float mf_f32x2 __attribute__((ext_vector_type(2)));

// x, y -> bf16x2 hi (RNE) and bf16x2 lo = RNE(x - hi) (x - hi is exact)
__device__ __forceinline__ void mf_split2(float x, float y, uint32_t* hi, uint32_t* lo) {
    const mf_f32x2 v = {x, y};
    const uint32_t hb = __builtin_bit_cast(uint32_t, __builtin_convertvector(v, mf_bf16x2));
    const mf_f32x2 r = {x - __uint_as_float(hb << 16), y - __uint_as_float(hb & 0xffff0000u)};
    *hi = hb;
    *lo = __builtin_bit_cast(uint32_t, __builtin_convertvector(r, mf_bf16x2));
}

// 4x4 transpose of the 16-lane rows: in, x_p at row r = M[r][p]; out, x_c at row r = M[c][r]
__device__ __forceinline__ void mf_transpose(uint32_t& x0, uint32_t& x1, uint32_t& x2, uint32_t& x3) {
    auto a = __builtin_amdgcn_permlane32_swap(x0, x2, false, false);  // rows 2,3 of x0 <-> rows 0,1 of x2
    auto b = __builtin_amdgcn_permlane32_swap(x1, x3, false, false);
    auto c = __builtin_amdgcn_permlane16_swap(a[0], b[0], false, false);  // odd rows of x0 <-> even rows of x1
    auto d = __builtin_amdgcn_permlane16_swap(a[1], b[1], false, false);
    x0 = c[0];
    x1 = c[1];
    x2 = d[0];
    x3 = d[1];
}

typedef uint32_t mf_u32x4 __attribute__((ext_vector_type(4)));

// A 16-B global load the compiler cannot move or merge (closest_hit_mf's prefetch), and
// the waits that make its result usable: vmcnt(1) = every load but the newest landed
// (the other fragment may still be in flight; extra loads of the compiler's only make it
// stricter), vmcnt(0) = all landed.  The fragments pass through the waits' asm as
// in/out operands, so no use of them can be scheduled above the wait.  No memory clobber:
// the image is read-only, and the compiler's own loads need no ordering against these
// (its waits count only its loads, so ours can only make them wait longer).
__device__ __forceinline__ mf_u32x4 mf_load(const uint4* p) {
    mf_u32x4 v;
    asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(v) : "v"(p));
    return v;
}
__device__ __forceinline__ void mf_wait1(mf_u32x4& v) { asm volatile("s_waitcnt vmcnt(1)" : "+v"(v)); }
__device__ __forceinline__ void mf_wait0(mf_u32x4& a, mf_u32x4& b) {
    asm volatile("s_waitcnt vmcnt(0)" : "+v"(a), "+v"(b));
}

__device__ __forceinline__ mf_bf16x8 mf_frag(uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    const u32x4 v = {a, b, c, d};
    return __builtin_bit_cast(mf_bf16x8, v);
}

// drop bit (bit 31) of one pair from the scaled row values A, T', U, V (build_mf_rows:
// margins 1, sign-test threshold rho): set iff the exact test must fail, i.e. |A| > rho and
// one of s U, s V, s W (W = A - U - V), s T' is below -1, s = sign A.  s X + 1 < 0 is tested
// as the sign of fma(X, A, |A|) = |A| (s X + 1), which one rounding cannot flip (an exact
// 0 gives +0: keep); W's two subtractions round as the fp32 filter's (aa - su) - sv do.
__device__ __forceinline__ uint32_t mf_drop(mf_f32x4 q, float rho) {
    const float A = q[0], aa = fabsf(q[0]);
    const float w = (A - q[2]) - q[3];
    const float xu = fmaf(q[2], A, aa), xv = fmaf(q[3], A, aa);
    const float xw = fmaf(w, A, aa), xt = fmaf(q[1], A, aa);
    const float mn = fminf(fminf(xu, xv), fminf(xw, xt));
    return __float_as_uint(rho - aa) & __float_as_uint(mn);
}

// groups of the image that hold triangles (all rounds but the last are full)
__host__ __device__ inline int mf_groups(int n_tri) {
    if (n_tri <= 0) return 0;
    const int rounds = (n_tri + kMfRound - 1) / kMfRound;
    const int last = n_tri - (rounds - 1) * kMfRound;
    return (rounds - 1) * kMfGroupsPerRound + (last + 3) / 4;
}

// The exact test of triangle i without the t window: t if the triangle passes
// (detA != 0, t >= 0, u, v >= 0, u + v <= 1, t > eps for RULE 0), else +inf; the
// operations of exact_one (same operands, same order, so the same bits).  Accepting t
// when t < best + eps (RULE 0) / t < best (RULE 1), in index order, is exact_one's
// result (+inf, like a NaN, never passes either window).
template <int RULE>
__device__ __forceinline__ float exact_tv(const float4* __restrict__ tri, int i, f3 o, float nDx, float nDy,
                                          float nDz) {
    const float4 A = tri[i * kIsectF4 + 0];
    const float4 E1 = tri[i * kIsectF4 + 1];
    const float4 E2 = tri[i * kIsectF4 + 2];
    const float bx = o.x - A.x, by = o.y - A.y, bz = o.z - A.z;
    const float s1 = nDy * E2.z - E2.y * nDz;
    const float s2 = nDy * E1.z - E1.y * nDz;
    const float detA = (nDx * A.w - E1.x * s1) + E2.x * s2;
    const float s3 = by * E2.z - E2.y * bz;
    const float s4 = by * E1.z - E1.y * bz;
    const float det_t = (bx * A.w - E1.x * s3) + E2.x * s4;
    const float s5 = nDy * bz - by * nDz;
    const float s6 = E1.y * bz - by * E1.z;
    const float det_u = (nDx * s3 - bx * s1) + E2.x * s5;
    const float det_v = (nDx * s6 - E1.x * s5) + bx * s2;
    float t, u, v;
    if (RULE == 0) {
        const float inv = RT_RCP(detA);
        t = det_t * inv;
        u = det_u * inv;
        v = det_v * inv;
    } else {
        t = det_t / detA;
        u = det_u / detA;
        v = det_v / detA;
    }
    const bool ok = (detA != 0.0f) && (t >= 0.0f) && (u >= 0.0f) && (v >= 0.0f) && ((u + v) <= 1.0f) &&
                    (RULE != 0 || t > kEps);
    return ok ? t : __builtin_inff();
}

#ifndef RT_PROF
#define RT_PROF 0  // 1: k_render_ps sums per-phase s_memtime cycles into RenderLaunch::prof
#endif
#ifndef RT_MF_PINGPONG
#define RT_MF_PINGPONG 1  // 0: one operand set prefetched a group ahead (copied each group)
#endif
#ifndef RT_MF_RHO_GROUP
#define RT_MF_RHO_GROUP 1  // one sign-test threshold per 4-triangle group, the largest (0: per slot, 2: 1/2; 1 measured fastest, profiles/r3i)
#endif
#ifndef RT_MF_FIRST_OWN
// 1: with one 64-triangle block (NB == 1) each lane tests its first candidate itself, the
// rest shared (Cornell 512^2 x 256: 3.92 vs 4.00 ms; on complex_light_room's four blocks it
// measured 314 vs 310 ms, so wider scenes share every pair: profiles/r3q/)
#define RT_MF_FIRST_OWN 1
#endif
#ifndef RT_MF_COOP
#define RT_MF_COOP 1  // 0: each lane runs its own candidates' exact tests (A/B builds)
#endif

// LDS of one wave for the shared exact phase: rays [6][64] (o, -D), pairs [cap] u16
// (lane << 6 | triangle of the block); the tests' t values stay in registers
#ifndef RT_MF_PAIR_CAP
#define RT_MF_PAIR_CAP 256
#endif
#ifndef RT_MF_TV_LDS
#define RT_MF_TV_LDS 1  // 0: t values by cross-lane reads (Cornell 512^2 x 256: 4.19 vs 3.96 ms)
#endif
constexpr int kMfPairCap = RT_MF_PAIR_CAP;
constexpr int kMfWaveFloats = 6 * 64 + kMfPairCap / 2 + (RT_MF_TV_LDS ? kMfPairCap : 0);
static_assert(kMfWaveFloats >= 11 * 64, "cand_exact_min's LDS (rays, first, mask, key) fits a wave's block");
// The table-route kernel k_render_ps<.., CT> (RULE 0): about 3 candidates per ray of which the
// lane tests its first RT_CTAB_OWN itself, so the shared phase lists a few dozen pairs per wave;
// a smaller list block (with RT_PS_CT_SHADE_LDS) lets one more workgroup fit a CU's LDS
#ifndef RT_PS_CT_PAIR_CAP
#define RT_PS_CT_PAIR_CAP 96  // (64 / 96 / 128 / 256: 2.37 / 2.33 / 2.34 / 2.63 ms with the shading records in L1/L2)
#endif
constexpr int kCtPairCap = RT_PS_CT_PAIR_CAP;
__host__ __device__ constexpr int mf_wave_floats(int cap, int rule) {
    return (rule == 1 && 6 * 64 + cap / 2 + (RT_MF_TV_LDS ? cap : 0) < 11 * 64) ? 11 * 64
                                                                              : 6 * 64 + cap / 2 + (RT_MF_TV_LDS ? cap : 0);
}

__device__ __forceinline__ void wave_lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// The exact phase of one 64-triangle block (triangles tri0 + bit of F) shared by the
// wave: the lanes' candidate pairs are listed in LDS in (lane, index) order and tested
// 64 at a time by all lanes, then each lane folds its own results in index order.  The
// trip count is (candidates of the wave) / 64 instead of the largest per-lane count.
template <int RULE, int CAP = kMfPairCap>
__device__ __forceinline__ void mf_exact_wave(const float4* __restrict__ isect, int tri0, uint64_t F, f3 o,
                                              float nDx, float nDy, float nDz, float* wl, int lane, Hit& h) {
    const int cnt = __builtin_popcountll(F);  // 0..64: 7 bits
    // exclusive prefix sum over the lanes, bit-sliced through ballots (no LDS round trips,
    // unlike a shuffle scan: the cross-lane permutes were a dependent chain of 6)
    int excl = 0, total = 0;
#pragma unroll
    for (int b = 0; b < 7; ++b) {
        const uint64_t bm = __ballot((cnt >> b) & 1);
        excl += (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(bm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bm, 0u)) << b;
        total += __builtin_popcountll(bm) << b;
    }
    if (total == 0) return;
    const float* ray = wl;  // (o, -D) of every lane: written by closest_hit_mf before its masks
    uint16_t* pr = reinterpret_cast<uint16_t*>(wl + 6 * 64);
    // the lane's pairs not yet folded (lowest bit first) and the list position of the next
    uint64_t R = F;
    int pos = excl;
    for (int cb = 0; cb < total; cb += CAP) {
        {
            uint64_t G = F;
            int p = excl - cb;
            while (G != 0ull) {
                const int b = __builtin_ctzll(G);
                G &= G - 1ull;
                if (p >= 0 && p < CAP) pr[p] = (uint16_t)((lane << 6) | b);
                ++p;
            }
        }
        wave_lds_sync();
        const int nb = min(CAP, total - cb);
#if RT_MF_TV_LDS
        float* tv = wl + 6 * 64 + CAP / 2;
        for (int k = lane; k < nb; k += 64) {
            const uint32_t q = pr[k];
            const int rl = (int)(q >> 6);
            const f3 ro = make3(ray[0 * 64 + rl], ray[1 * 64 + rl], ray[2 * 64 + rl]);
            tv[k] = exact_tv<RULE>(isect, tri0 + (int)(q & 63u), ro, ray[3 * 64 + rl], ray[4 * 64 + rl],
                                   ray[5 * 64 + rl]);
        }
        wave_lds_sync();
        {
            uint64_t G = F;
            int p = excl - cb;
            while (G != 0ull) {
                const int b = __builtin_ctzll(G);
                G &= G - 1ull;
                if (p >= 0 && p < CAP) {
                    const float t = tv[p];
                    if ((RULE == 0) ? (t < h.t + kEps) : (t < h.t)) {
                        h.t = t;
                        h.tri = tri0 + b;
                    }
                }
                ++p;
            }
        }
        (void)R;
        (void)pos;
#else
        for (int sb = 0; sb < nb; sb += 64) {
            // 64 pairs at a time: lane k tests pair sb + k; each lane then takes its own pairs'
            // results from the testing lanes' registers (ds_bpermute: no LDS array for them)
            float tr = __builtin_inff();
            const int k = sb + lane;
            if (k < nb) {
                const uint32_t q = pr[k];
                const int rl = (int)(q >> 6);
                const f3 ro = make3(ray[0 * 64 + rl], ray[1 * 64 + rl], ray[2 * 64 + rl]);
                tr = exact_tv<RULE>(isect, tri0 + (int)(q & 63u), ro, ray[3 * 64 + rl], ray[4 * 64 + rl],
                                    ray[5 * 64 + rl]);
            }
            // The fold, one pair per lane and step, with the whole wave active: a cross-lane
            // read (ds_bpermute) from a lane that is switched off returns 0, not its value,
            // so the read must not sit in a lane-divergent loop.  A lane's next pair is in
            // this window iff pos < base + 64 (earlier windows consumed those before it).
            const int base = cb + sb;
            for (;;) {
                const bool has = (R != 0ull) && (pos < base + 64);
                if (__ballot(has) == 0ull) break;
                const float t = __shfl(tr, has ? pos - base : 0, 64);
                if (has) {
                    const int b = __builtin_ctzll(R);
                    R &= R - 1ull;
                    ++pos;
                    if ((RULE == 0) ? (t < h.t + kEps) : (t < h.t)) {
                        h.t = t;
                        h.tri = tri0 + b;
                    }
                }
            }
        }
#endif
        wave_lds_sync();  // the pair list is read before the next window overwrites it
    }
}

// s.mf_frag may point to a workgroup's LDS copy of the image (k_render_ps);
// wl: the wave's LDS for the shared exact phase (kMfWaveFloats floats)
// NB: 64-triangle blocks per super-block (1: scenes of <= 64 triangles, fewer registers)
// ovr (wave-uniform, kRenderCullWords 64-triangle masks) with use_ovr: the lane's candidates
// are ovr's instead of the filter's (k_render's camera rays: the wave's primary-ray cull,
// rt_cull.hpp, when the camera lies outside mf_bound); they join the shared exact phase.
template <int RULE, bool COUNT = false, int NB = 4>
__device__ __forceinline__ Hit closest_hit_mf(const DeviceScene& s, f3 o, f3 d, float t_scale, bool active,
                                              float* wl, int* n_cand = nullptr, uint64_t* t_mask_end = nullptr,
                                              const uint64_t* ovr = nullptr, bool use_ovr = false) {
    const float nDx = -(d.x * t_scale);
    const float nDy = -(d.y * t_scale);
    const float nDz = -(d.z * t_scale);
    const bool finite = __builtin_isfinite(o.x) & __builtin_isfinite(o.y) & __builtin_isfinite(o.z) &
                        __builtin_isfinite(d.x) & __builtin_isfinite(d.y) & __builtin_isfinite(d.z);
    const float om = fmaxf(fmaxf(fabsf(o.x), fabsf(o.y)), fabsf(o.z));
    const float dm = fmaxf(fmaxf(fabsf(d.x), fabsf(d.y)), fabsf(d.z));
    const bool keep_all = !(finite && om <= s.mf_bound && dm <= kMfDirBound);
    const int lane = threadIdx.x & 63;
    // the lane's ray for the shared exact phase, parked in LDS now: o and -D are not held in
    // registers through the masks (the caller may read them back: wl rows 0-5)
    wl[0 * 64 + lane] = o.x;
    wl[1 * 64 + lane] = o.y;
    wl[2 * 64 + lane] = o.z;
    wl[3 * 64 + lane] = nDx;
    wl[4 * 64 + lane] = nDy;
    wl[5 * 64 + lane] = nDz;
    const uint4* __restrict__ frag = s.mf_frag;
    [[maybe_unused]] const int slot = lane >> 4;  // the lane's slot of the MFMA output
    const mf_f32x4 zero = {0.0f, 0.0f, 0.0f, 0.0f};

    Hit h;
    h.t = (RULE == 0) ? FLT_MAX : 999999.0f;
    h.tri = -1;
    const int n_tri = s.n_tri;
    // super-blocks of 256 triangles: the masks of all 8 rounds first (the ray operands
    // die there), then the exact phase of each 64-triangle block
    for (int sb = 0; sb < n_tri; sb += 2 * NB * kMfRound) {
        uint64_t F0 = 0ull, F1 = 0ull, F2 = 0ull, F3 = 0ull;
        {
            const float Rx = fmaf(d.y, o.z, -(d.z * o.y));
            const float Ry = fmaf(d.z, o.x, -(d.x * o.z));
            const float Rz = fmaf(d.x, o.y, -(d.y * o.x));
            const float ets = (RULE == 0) ? kEps * t_scale : 0.0f;
            const float px = fmaf(-ets, d.x, -o.x), py = fmaf(-ets, d.y, -o.y), pz = fmaf(-ets, d.z, -o.z);
            // features f = (d, o', R, 1) as bf16 pairs: h_k = (fh_2k, fh_2k+1), l_k likewise
            uint32_t h0, h1, h2, h3, h4, l0, l1, l2, l3, l4;
            mf_split2(d.x, d.y, &h0, &l0);
            mf_split2(d.z, px, &h1, &l1);
            mf_split2(py, pz, &h2, &l2);
            mf_split2(Rx, Ry, &h3, &l3);
            mf_split2(Rz, 1.0f, &h4, &l4);
            // the four K parts of the lane's ray, then across the rows: B operand of ray block c
            uint32_t b00 = h0, b01 = h1, b02 = h2, b03 = h3;  // k  0.. 7
            uint32_t b10 = h4, b11 = l0, b12 = l1, b13 = l2;  // k  8..15
            uint32_t b20 = l3, b21 = l4, b22 = h0, b23 = h1;  // k 16..23
            uint32_t b30 = h2, b31 = h3, b32 = h4, b33 = 0u;  // k 24..31
            mf_transpose(b00, b10, b20, b30);
            mf_transpose(b01, b11, b21, b31);
            mf_transpose(b02, b12, b22, b32);
            mf_transpose(b03, b13, b23, b33);
            const mf_bf16x8 B0 = mf_frag(b00, b01, b02, b03), B1 = mf_frag(b10, b11, b12, b13);
            const mf_bf16x8 B2 = mf_frag(b20, b21, b22, b23), B3 = mf_frag(b30, b31, b32, b33);
            const int n_rounds = min(2 * NB, (n_tri - sb + kMfRound - 1) / kMfRound);
#pragma clang loop unroll(disable)
            for (int rr = 0; rr < n_rounds; ++rr) {
                const int r = sb / kMfRound + rr;
                const int cnt = min(kMfRound, n_tri - r * kMfRound);
                const int G = (cnt + 3) >> 2;
                uint32_t m0 = 0u, m1 = 0u, m2 = 0u, m3 = 0u;
                const int gi0 = r * kMfGroupsPerRound;
                // one 4-triangle group: 4 MFMAs (ray blocks 0..3), drop bits shifted in
                auto group = [&](const mf_u32x4 af) {
                    // the slots' sign-test thresholds, stored in the fragment's unused K entries
                    // (build_mf_image: lane 48 + 4 s, dword 3)
#if RT_MF_RHO_GROUP == 2
                    const float rho = 0.5f;  // the bound of every threshold (loosest)
#elif RT_MF_RHO_GROUP == 1
                    // the group's largest (one scalar per group: a looser test for its smaller triangles)
                    const float rho = __int_as_float(__builtin_amdgcn_readlane((int)af[3], 49));
#else
                    const float t0 = __int_as_float(__builtin_amdgcn_readlane((int)af[3], 48));
                    const float t1 = __int_as_float(__builtin_amdgcn_readlane((int)af[3], 52));
                    const float t2 = __int_as_float(__builtin_amdgcn_readlane((int)af[3], 56));
                    const float t3 = __int_as_float(__builtin_amdgcn_readlane((int)af[3], 60));
                    const float rho = (slot & 2) ? ((slot & 1) ? t3 : t2) : ((slot & 1) ? t1 : t0);
#endif
                    const mf_bf16x8 A = __builtin_bit_cast(mf_bf16x8, af);
                    const mf_f32x4 q0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A, B0, zero, 0, 0, 0);
                    const mf_f32x4 q1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A, B1, zero, 0, 0, 0);
                    const mf_f32x4 q2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A, B2, zero, 0, 0, 0);
                    const mf_f32x4 q3 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A, B3, zero, 0, 0, 0);
                    m0 = __builtin_amdgcn_alignbit(m0, mf_drop(q0, rho), 31);
                    m1 = __builtin_amdgcn_alignbit(m1, mf_drop(q1, rho), 31);
                    m2 = __builtin_amdgcn_alignbit(m2, mf_drop(q2, rho), 31);
                    m3 = __builtin_amdgcn_alignbit(m3, mf_drop(q3, rho), 31);
                };
#if RT_MF_PINGPONG
                // two operand sets in flight: group g + 2's fragment is loaded right after
                // group g's MFMAs have read theirs, a whole group of work before its use.
                // The loads are inline asm with explicit waits: written as plain loads, the
                // optimizer proves the prefetched value equals a load at the top of the
                // next trip and moves it there, waiting on it at once.  mf_wait1 returns
                // the fragment (tied through the asm), so its MFMAs cannot move above it.
                // An odd G starts with a pad group (index G < 8: zero rows, so its drop bit
                // is 0 and lands at bit G of the slot mask, where the next slot's bit 0 is
                // or-ed in).  The prefetches past the end reload group G - 1 (in range).
                const uint4* __restrict__ fr = frag + (size_t)gi0 * 64 + lane;
                const int gs = -(G & 1);
                mf_u32x4 fa = mf_load(fr + (gs < 0 ? G : 0) * 64);
                mf_u32x4 fb = mf_load(fr + (gs + 1) * 64);
                for (int g = gs; g < G; g += 2) {
                    const int n2 = min(g + 2, G - 1), n3 = min(g + 3, G - 1);
                    mf_wait1(fa);
                    group(fa);
                    fa = mf_load(fr + n2 * 64);
                    mf_wait1(fb);
                    group(fb);
                    fb = mf_load(fr + n3 * 64);
                }
                mf_wait0(fa, fb);  // the last (unused) loads land before their registers are reused
#else
                uint4 afn = frag[gi0 * 64 + lane];
                for (int g = 0; g < G; ++g) {
                    const uint4 af = afn;
                    if (g + 1 < G) afn = frag[(gi0 + g + 1) * 64 + lane];  // the next group's operand ahead
                    const mf_u32x4 v = {af.x, af.y, af.z, af.w};
                    group(v);
                }
#endif
                // lane (slot s, ray q) holds m_c for ray 16 c + q; after the transpose lane
                // (c, q) holds the masks of slots 0..3 of its own ray: bit j of slot s's mask
                // is triangle s G + j of the round
                mf_transpose(m0, m1, m2, m3);
                const uint32_t Dr = m0 | (m1 << G) | (m2 << (2 * G)) | (m3 << (3 * G));  // drop bits
                const uint32_t all = (cnt >= 32) ? 0xffffffffu : ((1u << cnt) - 1u);
                const uint32_t Fr = keep_all ? all : (~Dr & all);
                const uint64_t Fs = (uint64_t)Fr << (32 * (rr & 1));  // wave-uniform word select
                const int w = rr >> 1;
                F0 |= (w == 0) ? Fs : 0ull;
                if (NB > 1) {
                    F1 |= (w == 1) ? Fs : 0ull;
                    F2 |= (w == 2) ? Fs : 0ull;
                    F3 |= (w == 3) ? Fs : 0ull;
                }
            }
        }
#if RT_PROF
        if (t_mask_end) *t_mask_end = __builtin_amdgcn_s_memtime();
#endif
#pragma unroll
        for (int w = 0; w < NB; ++w) {
            const int tri0 = sb + 64 * w;
            if (tri0 >= n_tri) break;
            uint64_t Fw = active ? (w == 0 ? F0 : w == 1 ? F1 : w == 2 ? F2 : F3) : 0ull;
            if (ovr != nullptr) {
                const int g = (sb >> 6) + w;
                Fw = use_ovr ? ((active && g < 4) ? ovr[g < 4 ? g : 0] : 0ull) : Fw;
            }
            if (COUNT) *n_cand += __builtin_popcountll(Fw);
#if RT_MF_COOP
#if RT_MF_FIRST_OWN
            // the lane's first candidate on its own lane (its own ray, no pair list: every live
            // lane has one, usually its hit), then the rest (≈ 0.3 per ray) shared by the wave
            if (NB == 1 && Fw != 0ull) {
                const int b = __builtin_ctzll(Fw);
                const float t = exact_tv<RULE>(s.isect, tri0 + b, o, nDx, nDy, nDz);
                if ((RULE == 0) ? (t < h.t + kEps) : (t < h.t)) {
                    h.t = t;
                    h.tri = tri0 + b;
                }
                Fw &= Fw - 1ull;
            }
#endif
            mf_exact_wave<RULE>(s.isect, tri0, Fw, o, nDx, nDy, nDz, wl, lane, h);
#else
            uint64_t G = Fw;
            while (G != 0ull) {
                const int b = __builtin_ctzll(G);
                G &= G - 1ull;
                exact_one<RULE>(s.isect, tri0 + b, o, nDx, nDy, nDz, h);
            }
#endif
        }
    }
    return h;
}

// The candidates of a bounce ray leaving surface `surf` (rt_ctab.cpp) from the table T of the
// launch's hit rule: the mask of its (origin patch, direction bin) OR that of its grazing bin
// OR, for a direction within T.cop_th of the surface's plane (always, under rule 1), the
// triangles coplanar with it -- every other triangle fails the exact test for this ray -- or
// every triangle where the table does not apply (origin off the surface's plane or grid, a
// direction off its hemisphere, non-unit or non-finite).  F: NW >= T.words mask words (the
// rest 0).  rt_ctab.cpp ctab_lookup is the same lookup on the host.
template <int NW>
__device__ __forceinline__ void ctab_candidates(const CtabDev& T, int n_tri, int n_surf, int surf, f3 o, f3 d,
                                                uint64_t (&F)[NW]) {
    const int W = T.words;
#pragma unroll
    for (int w = 0; w < NW; ++w) F[w] = (w < W) ? ((n_tri - 64 * w >= 64) ? ~0ull : ((1ull << (n_tri - 64 * w)) - 1ull)) : 0ull;
    if (surf < 0 || surf >= n_surf) return;
    const float4 R0 = T.tri[surf * 4 + 0], R1 = T.tri[surf * 4 + 1];
    const float4 R2 = T.tri[surf * 4 + 2], R3 = T.tri[surf * 4 + 3];
    const float bx = o.x - R0.x, by = o.y - R0.y, bz = o.z - R0.z;
    const float w = (bx * R3.x + by * R3.y) + bz * R3.z;
    const float pu = ((bx * R1.x + by * R1.y) + bz * R1.z) * R0.w;
    const float pv = ((bx * R2.x + by * R2.y) + bz * R2.z) * R0.w;
    const int nu = __float_as_int(R1.w), nv = __float_as_int(R2.w), base = __float_as_int(R3.w);
    const float len2 = fmaf(d.x, d.x, fmaf(d.y, d.y, d.z * d.z));
    const float cn = (d.x * R3.x + d.y * R3.y) + d.z * R3.z;  // R3: the surface's shading normal
    const bool in = (fabsf(w) <= T.h) & (pu >= 0.0f) & (pu < (float)nu) & (pv >= 0.0f) & (pv < (float)nv) &
                    (len2 >= 1.0f - 0x1p-20f) & (len2 <= 1.0f + 0x1p-20f) & (cn >= -kCtabHemi);
    if (!in) return;
    // cube-map face: the axis of the largest |d_i| (x before y before z on ties), u, v the next two
    const float ax = fabsf(d.x), ay = fabsf(d.y), az = fabsf(d.z);
    const bool fx = (ax >= ay) & (ax >= az), fy = !fx & (ay >= az);
    const float dm = fx ? d.x : (fy ? d.y : d.z);
    const float da = fx ? d.y : (fy ? d.z : d.x);
    const float db = fx ? d.z : (fy ? d.x : d.y);
    const int f = (fx ? 0 : (fy ? 2 : 4)) + (dm < 0.0f ? 1 : 0);
    const float r = __builtin_amdgcn_rcpf(fabsf(dm));
    const float u1 = da * r + 1.0f, v1 = db * r + 1.0f;  // (the build contracts nothing: two roundings)
    const int iu = min(kCtabBins - 1, max(0, (int)(u1 * (0.5f * kCtabBins))));
    const int iv = min(kCtabBins - 1, max(0, (int)(v1 * (0.5f * kCtabBins))));
    const int gu = min(kCtabGraze - 1, max(0, (int)(u1 * (0.5f * kCtabGraze))));
    const int gv = min(kCtabGraze - 1, max(0, (int)(v1 * (0.5f * kCtabGraze))));
    const int patch = base + (int)pu * nv + (int)pv;
    const unsigned long long* mm = T.masks + ((size_t)patch * (6 * kCtabBins * kCtabBins) + (f * kCtabBins + iu) * kCtabBins + iv) * W;
    const int gi = (f * kCtabGraze + gu) * kCtabGraze + gv;
    // the triangles coplanar with the surface join near its plane's great circle (rule 0) or always (rule 1)
    const bool cp = fabsf(cn) < T.cop_th;
    if (T.gflag) {
        // the grazing fold (rt_ctab.cpp): the entry holds its bin's grazing mask unless bit 63 of
        // its last word asks for the lookup -- one dependent access for most rays, not three
        uint64_t m[NW];
#pragma unroll
        for (int k = 0; k < NW; ++k) m[k] = (k < W) ? mm[k] : 0ull;
        uint64_t last = 0ull;
#pragma unroll
        for (int k = 0; k < NW; ++k)
            if (k == W - 1) last = m[k];
        const bool look = (last & kCtabGflagBit) != 0ull;
        const unsigned long long* gg = look ? T.gdict + (size_t)T.gid[gi] * W : nullptr;
#pragma unroll
        for (int k = 0; k < NW; ++k)
            if (k < W)
                F[k] = (m[k] & (k == W - 1 ? ~kCtabGflagBit : ~0ull)) | (look ? gg[k] : 0ull) |
                       (cp ? T.cop[surf * W + k] : 0ull);
        return;
    }
    const unsigned long long* gg = T.gdict + (size_t)T.gid[gi] * W;
#pragma unroll
    for (int k = 0; k < NW; ++k)
        if (k < W) F[k] = mm[k] | gg[k] | (cp ? T.cop[surf * W + k] : 0ull);
}

#ifndef RT_CTAB_OWN
#define RT_CTAB_OWN 3  // candidates each lane tests on its own lane before the shared exact phase (Cornell
                       // 512^2 x 256: 1 / 3 / 5 -> 3.04 / 2.90 / 2.96 ms with 8x8 bins, profiles/r5t)
#endif
// the table usable for a launch: built with this build's dimensions, for its t_scale
__device__ __forceinline__ bool ctab_usable(const CtabDev& T, float t_scale) {
    return T.masks != nullptr && T.bins == kCtabBins && T.graze_n == kCtabGraze && t_scale >= T.ts_min;
}
// closest_hit_mf's result for a ray whose candidates are given, F (NW mask words): every other
// triangle fails the exact test for the lane's ray, so testing F in index order gives the scan's
// hit.  The lane's first RT_CTAB_OWN candidates on its own lane, the rest shared by the wave
// (mf_exact_wave, per 64-triangle block).  Wave-level like closest_hit_mf (a lane without a ray:
// F = 0).  closest_hit_ctab: F from the table T for a bounce ray leaving surface `surf`.
#ifndef RT_CAND_MIN
#define RT_CAND_MIN 1  // 0: RULE 1's shared exact phase folds as RULE 0's (per-lane list walks)
#endif
#ifndef RT_CAND_OWN_MIN
#define RT_CAND_OWN_MIN 0  // RT_CTAB_OWN of the min-fold phase (complex_light_room 512^2 x 64: 0 / 1 -> 50.9 / 66.8 ms)
#endif

// RULE 1's window (accept t < best, in index order, from best = 999999, tri -1) picks the
// lexicographic minimum of (t, index) over the passing candidates and the start: a 64-bit key,
// |t|'s bits above the index + 1 (0: the start, which wins a tie at its t) and t's sign bit
// (a pass can be -0: ordered as +0, returned as it was)
__device__ __forceinline__ uint64_t min_key(float t, int tri) {
    const uint32_t b = __float_as_uint(t);
    return ((uint64_t)(b & 0x7fffffffu) << 32) | ((uint64_t)(uint32_t)(tri + 1) << 1) | (uint64_t)(b >> 31);
}
__device__ __forceinline__ void min_unkey(uint64_t k, Hit& h) {
    const uint32_t hi = (uint32_t)(k >> 32), lo = (uint32_t)k;
    h.t = __uint_as_float(hi | (lo << 31));
    h.tri = (int)(lo >> 1) - 1;
}
// position of the j-th (from 0) set bit of x (j < popcount(x))
__device__ __forceinline__ int select_bit(uint64_t x, int j) {
    uint32_t w = (uint32_t)x;
    int pos = 0, c = __builtin_popcount(w);
    if (j >= c) {
        j -= c;
        w = (uint32_t)(x >> 32);
        pos = 32;
    }
#pragma unroll
    for (int sh = 16; sh >= 1; sh >>= 1) {
        c = __builtin_popcount(w & ((1u << sh) - 1u));
        if (j >= c) {
            j -= c;
            w >>= sh;
            pos += sh;
        }
    }
    return pos;
}
// The shared exact phase of one 64-triangle block under RULE 1, folded by minimum: the wave's
// (lane, candidate) pairs are numbered lane-major, and lane k of each round of 64 finds pair
// cb + k's lane (binary search over the lanes' first pair numbers) and triangle (the j-th set
// bit of that lane's mask), tests it and folds its t into that lane's key with an LDS atomic
// minimum.  No lane walks its own list: a round costs the same whatever the lanes' counts.
// LDS (wl, after the rays' 6 x 64 floats): first[64] int, mask[64] u64, key[64] u64.
__device__ __forceinline__ void cand_exact_min(const float4* __restrict__ isect, int tri0, uint64_t F, float* wl,
                                               int lane, unsigned long long* key) {
    const int cnt = __builtin_popcountll(F);
    int excl = 0, total = 0;
#pragma unroll
    for (int b = 0; b < 7; ++b) {
        const uint64_t bm = __ballot((cnt >> b) & 1);
        excl += (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(bm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bm, 0u)) << b;
        total += __builtin_popcountll(bm) << b;
    }
    if (total == 0) return;
    int* first = reinterpret_cast<int*>(wl + 6 * 64);
    unsigned long long* mask = reinterpret_cast<unsigned long long*>(wl + 7 * 64);
    first[lane] = excl;
    mask[lane] = F;
    wave_lds_sync();
    const float* ray = wl;
    for (int cb = 0; cb < total; cb += 64) {
        const int k = cb + lane;
        if (k < total) {
            int r = 0;
#pragma unroll
            for (int st = 32; st >= 1; st >>= 1)
                if (first[r + st] <= k) r += st;
            const int i = tri0 + select_bit(mask[r], k - first[r]);
            const f3 ro = make3(ray[0 * 64 + r], ray[1 * 64 + r], ray[2 * 64 + r]);
            const float t = exact_tv<1>(isect, i, ro, ray[3 * 64 + r], ray[4 * 64 + r], ray[5 * 64 + r]);
            if (t < 999999.0f) atomicMin(key + r, (unsigned long long)min_key(t, i));
        }
    }
    wave_lds_sync();
}

template <int RULE, int NW, int CAP = kMfPairCap>
__device__ __forceinline__ Hit closest_hit_cand(const DeviceScene& s, uint64_t (&F)[NW], f3 o, f3 d, float t_scale,
                                                float* wl) {
    const float nDx = -(d.x * t_scale);
    const float nDy = -(d.y * t_scale);
    const float nDz = -(d.z * t_scale);
    const int lane = threadIdx.x & 63;
    // the lane's ray for the shared exact phase (rows 0-5 of wl, as closest_hit_mf parks it)
    wl[0 * 64 + lane] = o.x;
    wl[1 * 64 + lane] = o.y;
    wl[2 * 64 + lane] = o.z;
    wl[3 * 64 + lane] = nDx;
    wl[4 * 64 + lane] = nDy;
    wl[5 * 64 + lane] = nDz;
    Hit h;
    h.t = (RULE == 0) ? FLT_MAX : 999999.0f;
    h.tri = -1;
    constexpr bool kMin = RULE == 1 && RT_CAND_MIN;
    // the lane's first candidates (in index order) on its own lane
#pragma unroll
    for (int k = 0; k < (kMin ? RT_CAND_OWN_MIN : RT_CTAB_OWN); ++k) {
        int wsel = -1;
#pragma unroll
        for (int w = NW - 1; w >= 0; --w)
            if (F[w] != 0ull) wsel = w;
        if (wsel >= 0) {
            uint64_t fw = 0ull;
#pragma unroll
            for (int w = 0; w < NW; ++w)
                if (w == wsel) fw = F[w];
            const int b = 64 * wsel + __builtin_ctzll(fw);
            const float t = exact_tv<RULE>(s.isect, b, o, nDx, nDy, nDz);
            if ((RULE == 0) ? (t < h.t + kEps) : (t < h.t)) {
                h.t = t;
                h.tri = b;
            }
#pragma unroll
            for (int w = 0; w < NW; ++w)
                if (w == wsel) F[w] &= F[w] - 1ull;
        }
    }
    if constexpr (kMin) {
        unsigned long long* key = reinterpret_cast<unsigned long long*>(wl + 9 * 64);
        key[lane] = min_key(h.t, h.tri);
#pragma unroll
        for (int w = 0; w < NW; ++w)
            if (64 * w < s.n_tri) cand_exact_min(s.isect, 64 * w, F[w], wl, lane, key);
        wave_lds_sync();
        min_unkey(key[lane], h);
    } else {
#pragma unroll
        for (int w = 0; w < NW; ++w)
            if (64 * w < s.n_tri) mf_exact_wave<RULE, CAP>(s.isect, 64 * w, F[w], o, nDx, nDy, nDz, wl, lane, h);
    }
    return h;
}
template <int RULE, int NW, int CAP = kMfPairCap>
__device__ __forceinline__ Hit closest_hit_ctab(const DeviceScene& s, const CtabDev& T, int surf, f3 o, f3 d,
                                                float t_scale, bool active, float* wl) {
    uint64_t F[NW];
    if (active) {
        ctab_candidates<NW>(T, s.n_tri, s.n_surf, surf, o, d, F);
    } else {
#pragma unroll
        for (int k = 0; k < NW; ++k) F[k] = 0ull;
    }
    return closest_hit_cand<RULE, NW, CAP>(s, F, o, d, t_scale, wl);
}

#ifndef RT_FILTER
#define RT_FILTER 1  // 0: always the single-phase scan (A/B builds)
#endif
#ifndef RT_MF
#define RT_MF 1  // 0: the bounce casts of k_render_ps on the fp32 filter (A/B builds)
#endif
#ifndef RT_PS_SCENE_LDS
#define RT_PS_SCENE_LDS 1  // k_render_ps<MF>: the scene's isect/shade records in LDS (0: global)
#endif
#ifndef RT_PS_SHADE_LDS
#define RT_PS_SHADE_LDS 1  // 0: with RT_PS_SCENE_LDS, only the isect records in LDS (shading from L1/L2)
#endif
#ifndef RT_PS_CT_DICT_LDS
#define RT_PS_CT_DICT_LDS 0  // 1: the table route's grazing dictionary in LDS (when it has <= kPsCtDictLds words)
#endif
constexpr int kPsCtDictLds = 64;
#ifndef RT_PS_CT_TRI_LDS
#define RT_PS_CT_TRI_LDS 0  // 1: the table route's surface patch frames (CtabDev::tri) in LDS
#endif
#ifndef RT_PS_CT_SHADE_LDS
// the table-route kernel's shading records: from L1/L2 (0) -- with the shorter pair list it keeps
// the workgroup at 29.4 KB of LDS, five per CU (Cornell 512^2 x 256: 2.33 ms, in LDS 2.37-2.40;
// the 35.6-KB layout of round 5 held four per CU: 2.63 ms, profiles/r6f/ab.log)
#define RT_PS_CT_SHADE_LDS 0
#endif
#ifndef RT_MF_LDS
#define RT_MF_LDS 0  // 1: k_render_ps reads the image from a workgroup copy in LDS (0: global)
#endif

template <int RULE>
__device__ __forceinline__ Hit closest_hit_sel(const DeviceScene& s, int use_filter, f3 o, f3 d,
                                               float t_scale) {
#if RT_FILTER
    if (use_filter) return closest_hit_filtered<RULE>(s.filt, s.isect, s.n_tri, o, d, t_scale);
#endif
    return closest_hit<RULE>(s.isect, s.n_tri, o, d, t_scale);
}

// ---- Exact BVH path (large scenes; rt_bvh.cpp has the proof obligations) ----
// Rule-1 result: the smallest t below 999999, ties to the smallest index (the scan's
// strict t < best in index order).  Rule 0 (t < best + eps, ties to the later index)
// depends on the order, but only through the triangles with t below tmin + 2 eps: the
// first triangle with t = tmin resets the scan's best to tmin, and after it a triangle
// is accepted only below best + eps.  Those few are kept (index, t), sorted by index
// and folded as the scan folds them; if the fold's best could reach the cut, or more
// than kBvhCand arrive, the ray takes the exact scan.
struct BvhCand {
    float tmin, cut;               // rule 0: smallest t, fl(fl(tmin + eps) + eps)
    float ct[kBvhCand];
    int ci[kBvhCand];
    int nc;
    bool overflow;
    float bt;                      // rule 1: best t, index
    int bi;
};

template <int RULE>
__device__ __forceinline__ void bvh_insert(BvhCand& c, float t, int idx) {
    if (RULE == 1) {
        if (t < c.bt || (t == c.bt && idx < c.bi)) {
            c.bt = t;
            c.bi = idx;
        }
        return;
    }
    if (!(t < c.cut)) return;
#pragma unroll
    for (int k = 0; k < kBvhCand; ++k)
        if (k < c.nc && c.ci[k] == idx) return;  // listed already (BVH leaf and grazing list)
    if (c.nc == kBvhCand) {
        c.overflow = true;
        return;
    }
#pragma unroll
    for (int k = 0; k < kBvhCand; ++k)
        if (k == c.nc) {
            c.ct[k] = t;
            c.ci[k] = idx;
        }
    ++c.nc;
    if (t < c.tmin) {
        c.tmin = t;
        c.cut = (t + kEps) + kEps;
    }
}

// the window of the traversal in ray-parameter units (lambda = t * t_scale): a regular
// pair passing the exact test with t below the cut has lambda <= (cut ts + a) / (1 - b)
template <int RULE>
__device__ __forceinline__ float bvh_lam_hi(const BvhCand& c, const DeviceScene& s, float t_scale) {
    const float cut = (RULE == 0) ? c.cut : c.bt;
    return ((cut * t_scale + s.bvh_sig_a) / (1.0f - s.bvh_sig_b)) * 1.0000002f;
}

// stk: the lane's LDS stack (kBvhMaxDepth entries), STRIDE ints apart.
template <int RULE, int STRIDE = 256>
__device__ Hit closest_hit_bvh(const DeviceScene& s, f3 o, f3 d, float t_scale, int* stk) {
    const float nDx = -(d.x * t_scale), nDy = -(d.y * t_scale), nDz = -(d.z * t_scale);
    const float om = fmaxf(fmaxf(fabsf(o.x), fabsf(o.y)), fabsf(o.z));
    const float dm = fmaxf(fmaxf(fabsf(d.x), fabsf(d.y)), fabsf(d.z));
    // outside the bounds the records were built for (non-finite included): the scan
    if (!(om <= s.origin_bound && dm <= kMfDirBound && t_scale > 0.0f && t_scale <= kFiltMaxTScale))
        return closest_hit<RULE>(s.isect, s.n_tri, o, d, t_scale);
    BvhCand c;
    c.tmin = FLT_MAX;
    c.cut = FLT_MAX;
    c.nc = 0;
    c.overflow = false;
    c.bt = 999999.0f;
    c.bi = -1;
#pragma unroll
    for (int k = 0; k < kBvhCand; ++k) {
        c.ct[k] = 0.0f;
        c.ci[k] = 0;
    }
    // slab test: directions clamped away from 0 by 2^-100 (the node padding covers it)
    auto safe = [](float x) { return (fabsf(x) < 7.8886091e-31f) ? copysignf(7.8886091e-31f, x) : x; };
    const float ix = 1.0f / safe(d.x), iy = 1.0f / safe(d.y), iz = 1.0f / safe(d.z);
    const float lam_lo = -2.0f * s.bvh_sig_a - 1e-6f;
    const float4* __restrict__ nodes = s.bvh_nodes;
    const float4* __restrict__ tris = s.bvh_tris;
    auto slab = [&](int n, float lam_hi, float* entry) -> bool {
        const float4 lo = nodes[2 * n], hi = nodes[2 * n + 1];
        const float x0 = (lo.x - o.x) * ix, x1 = (hi.x - o.x) * ix;
        const float y0 = (lo.y - o.y) * iy, y1 = (hi.y - o.y) * iy;
        const float z0 = (lo.z - o.z) * iz, z1 = (hi.z - o.z) * iz;
        const float tn = fmaxf(fmaxf(fminf(x0, x1), fminf(y0, y1)), fmaxf(fminf(z0, z1), lam_lo));
        const float tf = fminf(fminf(fmaxf(x0, x1), fmaxf(y0, y1)), fminf(fmaxf(z0, z1), lam_hi));
        *entry = tn;
        return tn <= tf;
    };
    int sp = 0;
    int node = 0;
    for (;;) {
        const float4 hi = nodes[2 * node + 1];
        const int cnt = __float_as_int(hi.w);
        const int link = __float_as_int(nodes[2 * node].w);
        if (cnt > 0) {
            for (int j = link; j < link + cnt; ++j) {
                const float t = exact_tv<RULE>(tris, j, o, nDx, nDy, nDz);
                if (t <= FLT_MAX) bvh_insert<RULE>(c, t, __float_as_int(tris[j * kIsectF4 + 1].w));
            }
        } else {
            const float lh = bvh_lam_hi<RULE>(c, s, t_scale);
            float e0, e1;
            const bool h0 = slab(link, lh, &e0);
            const bool h1 = slab(link + 1, lh, &e1);
            if (h0 && h1) {
                const bool first0 = e0 <= e1;
                stk[(sp++) * STRIDE] = first0 ? link + 1 : link;
                node = first0 ? link : link + 1;
                continue;
            }
            if (h0 || h1) {
                node = h0 ? link : link + 1;
                continue;
            }
        }
        if (sp == 0) break;
        node = stk[(--sp) * STRIDE];
    }
    // grazing pairs (rt_bvh.cpp): the list of the ray's cube-map cell of directions, each
    // triangle tested for |d.N~| <= alpha B + beta and, with a window lambda, for its plane
    // within PA B + PB + (alpha B + beta) lambda of the origin (N units)
#ifdef RT_BVH_TIMING_TRAVERSAL_ONLY
    {  // timing-only build (wrong hits): the traversal alone
        Hit hh;
        hh.t = (RULE == 0) ? c.tmin : c.bt;
        hh.tri = (RULE == 0) ? (c.nc ? c.ci[0] : -1) : c.bi;
        return hh;
    }
#endif
    {
        const float cut = (RULE == 0) ? c.cut : c.bt;
        const float lam_cut = cut * t_scale * 1.0000002f;
        const bool bounded = lam_cut <= 3.0e38f;
#ifdef RT_BVH_TIMING_SKIP_UNBOUNDED
        if (!bounded) goto resolve;  // timing-only build (wrong hits)
#endif
        const float B = om * 1.000001f;
        // the cube-map cell of d (the host lists hold for any direction of the cell, plus
        // the rounding of this choice)
        const float ax = fabsf(d.x), ay = fabsf(d.y), az = fabsf(d.z);
        int f;
        float u, v, m;
        if (ax >= ay && ax >= az) {
            f = d.x >= 0.0f ? 0 : 1; m = ax; u = d.y; v = d.z;
        } else if (ay >= az) {
            f = d.y >= 0.0f ? 2 : 3; m = ay; u = d.z; v = d.x;
        } else {
            f = d.z >= 0.0f ? 4 : 5; m = az; u = d.x; v = d.y;
        }
        const float G = (float)kBvhDirGrid;
        const int iu = min(kBvhDirGrid - 1, max(0, (int)((u / m + 1.0f) * 0.5f * G)));
        const int iv = min(kBvhDirGrid - 1, max(0, (int)((v / m + 1.0f) * 0.5f * G)));
        const int cell = (f * kBvhDirGrid + iu) * kBvhDirGrid + iv;
        const bool cam = !(B <= s.bvh_B_lists);
        const int32_t* st = s.bvh_dstart + (cam ? 6 * kBvhDirGrid * kBvhDirGrid + 1 : 0);
        const int32_t* __restrict__ dl = cam ? s.bvh_dlist_cam : s.bvh_dlist;
        const float4* __restrict__ gr = s.bvh_grec;
        const int j0 = st[cell], j1 = st[cell + 1];
        for (int j = j0; j < j1; ++j) {
            const int i = dl[j];
            const float4 g = gr[2 * i];
            const float a = fmaf(d.z, g.z, fmaf(d.y, g.y, d.x * g.x));
            const float4 q = gr[2 * i + 1];
            const float thr = fmaf(g.w, B, q.x) * 1.000001f;
            bool cand = fabsf(a) <= thr;
            if (cand && bounded) {
                const float w = fmaf(o.z, g.z, fmaf(o.y, g.y, o.x * g.x)) - q.y;
                cand = fabsf(w) <= fmaf(thr, lam_cut, fmaf(q.z, B, q.w)) * 1.00001f;
            }
            if (cand) {
                const float t = exact_tv<RULE>(s.isect, i, o, nDx, nDy, nDz);
                if (t <= FLT_MAX) bvh_insert<RULE>(c, t, i);
            }
        }
    }
#ifdef RT_BVH_TIMING_SKIP_UNBOUNDED
resolve:
#endif
    Hit h;
    if (RULE == 1) {
        h.t = c.bt;
        h.tri = c.bi;
        return h;
    }
    if (c.overflow) return closest_hit<RULE>(s.isect, s.n_tri, o, d, t_scale);
    // the listed triangles below the final cut, in index order (insertion sort)
    float ft[kBvhCand];
    int fi[kBvhCand];
    int m = 0;
#pragma unroll
    for (int k = 0; k < kBvhCand; ++k) {
        ft[k] = 0.0f;
        fi[k] = 0x7fffffff;
    }
#pragma unroll
    for (int k = 0; k < kBvhCand; ++k) {
        if (k < c.nc && c.ct[k] < c.cut) {
            float t = c.ct[k];
            int i = c.ci[k];
#pragma unroll
            for (int j = 0; j < kBvhCand; ++j) {  // keep fi ascending: swap the larger one on
                if (j <= m && i < fi[j]) {
                    const float tt = ft[j];
                    const int ii = fi[j];
                    ft[j] = t;
                    fi[j] = i;
                    t = tt;
                    i = ii;
                }
            }
            ++m;
        }
    }
    h.t = FLT_MAX;
    h.tri = -1;
    bool seen = false;
    float bmax = 0.0f;
#pragma unroll
    for (int k = 0; k < kBvhCand; ++k) {
        if (k < m) {
            if (ft[k] < h.t + kEps) {
                h.t = ft[k];
                h.tri = fi[k];
            }
            if (ft[k] == c.tmin) seen = true;
            if (seen) bmax = fmaxf(bmax, h.t);
        }
    }
    if (m > 0 && !(bmax + kEps <= c.cut)) return closest_hit<RULE>(s.isect, s.n_tri, o, d, t_scale);
    return h;
}

// two uniforms of event `ev` of sample `smp` of pixel `pix`
__device__ __forceinline__ void draw2(uint32_t pix, uint32_t smp, uint32_t ev, uint32_t k0,
                                      uint32_t k1, float* a, float* b) {
#ifdef RT_TIMING_CHEAP_RNG
    // timing-only build (wrong images): what the Philox rounds cost
    const uint32_t h = (pix * 0x9E3779B9u) ^ (smp * 0x85EBCA6Bu) ^ (ev * 0xC2B2AE35u) ^ k0;
    *a = u01(h * 0x27D4EB2Fu);
    *b = u01((h ^ (h >> 15)) * 0x165667B1u);
    return;
#endif
    uint32_t o[4];
    philox4x32_10(pix, smp, ev, 0u, k0, k1, o);
    *a = u01(o[0]);
    *b = u01(o[1]);
}

// Camera ray through (px+r1, py+r2): default_path_tracing.cpp:25-34, Ray::Ray
// (ray.cpp:7-11), rotate_ray (ray.cpp:47-52; GPU/rays/ray.cu:161-172), with
// glm's mat4*vec4 order (m0*v0 + m1*v1) + (m2*v2 + m3*v3).
template <int PRESET>
__device__ __forceinline__ void camera_ray(const RenderLaunch& a, int px, int py, float r1, float r2,
                                           f3* d_out) {
    const float x = (float)px + r1;
    const float y = (float)py + r2;
    f3 dir = make3(x - (float)a.width / 2.0f, y - (float)a.height / 2.0f, (float)a.height);
    dir = normalize(dir);
    const float w = 1.0f;
    f3 r;
    r.x = (a.cos_y * dir.x + 0.0f * dir.y) + (-a.sin_y * dir.z + 0.0f * w);
    r.y = (0.0f * dir.x + 1.0f * dir.y) + (0.0f * dir.z + 0.0f * w);
    r.z = (a.sin_y * dir.x + 0.0f * dir.y) + (a.cos_y * dir.z + 0.0f * w);
    if (PRESET == 1) {
        const float rw = (0.0f * dir.x + 0.0f * dir.y) + (0.0f * dir.z + 1.0f * w);
        f3 q;
        q.x = (1.0f * r.x + 0.0f * r.y) + (0.0f * r.z + 0.0f * rw);
        q.y = (0.0f * r.x + a.cos_x * r.y) + (a.sin_x * r.z + 0.0f * rw);
        q.z = (0.0f * r.x + -a.sin_x * r.y) + (a.cos_x * r.z + 0.0f * rw);
        r = q;
    }
    *d_out = r;
}

__device__ __forceinline__ unsigned wave_sum(unsigned v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

}  // namespace rt
