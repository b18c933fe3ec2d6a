// rt_bounds.hpp — real-value bounds of the exact hit test, shared by the host builds of the
// exact BVH (rt_bvh.cpp) and the bounce-ray candidate table (rt_ctab.cpp).
//
// For the real values of a (ray, triangle) pair (build_filter's quantities, rt_capi.cpp:
// A = d.N, U = e2.R - d.G2, V = -e1.R + d.G1, W = A - U - V, T = w0 - o.N, R = d x o):
//   exact test passes  =>  s U >= -EW, s V >= -EW, s W >= -EW, s T >= -ET  (s = sign A)
// with EW, ET bounds on the two evaluations' rounding (16u scale x 4: c = 2^-19) for
// directions |d_i| <= kMfDirBound, origins |o_i| <= B and t_scale <= kFiltMaxTScale.
// U / A, V / A, W / A are the barycentrics of the plane crossing X = o + lambda d,
// lambda = T / A, so a pass with |A| >= a puts X in the triangle grown to barycentrics
// >= -EW / a, at lambda >= -ET / a.
#pragma once

#include <cfloat>
#include <cmath>

#include "rt_internal.hpp"

namespace rt {
namespace bnd {

constexpr double kU = 1.0 / 16777216.0;  // 2^-24
constexpr double kC = 1.0 / 524288.0;    // 2^-19: 2x the 16u of both evaluations

inline float down(double x) {
    float f = (float)x;
    return ((double)f <= x) ? f : nextafterf(f, -INFINITY);
}
inline float up(double x) {
    float f = (float)x;
    return ((double)f >= x) ? f : nextafterf(f, INFINITY);
}

// build_filter's per-triangle sums of one hit record {v0, c0}, {e1}, {e2}
struct TriAlg {
    double N[3] = {0, 0, 0}, w0 = 0, nlen = 0;
    double M = 0, n1 = 0, n2 = 0;  // sum |e1_j e2_k| + |e1_k e2_j|, |e1|_1, |e2|_1
    double vmax = 0;               // max |v0_i|
};
inline TriAlg tri_alg(const float4& P0, const float4& P1, const float4& P2) {
    TriAlg t;
    const double v0[3] = {P0.x, P0.y, P0.z}, a[3] = {P1.x, P1.y, P1.z}, b[3] = {P2.x, P2.y, P2.z};
    for (int k = 0; k < 3; ++k) {
        const int j = (k + 1) % 3, l = (k + 2) % 3;
        t.N[k] = a[j] * b[l] - a[l] * b[j];
        t.M += fabs(a[j] * b[l]) + fabs(a[l] * b[j]);
        t.n1 += fabs(a[k]);
        t.n2 += fabs(b[k]);
        t.vmax = fmax(t.vmax, fabs(v0[k]));
    }
    t.w0 = v0[0] * t.N[0] + v0[1] * t.N[1] + v0[2] * t.N[2];
    t.nlen = sqrt(t.N[0] * t.N[0] + t.N[1] * t.N[1] + t.N[2] * t.N[2]);
    return t;
}

struct Bounds {
    double eA, EW, ET;
};
// error bounds of one triangle for origins within B (build_filter's structure)
inline Bounds bounds_for(const TriAlg& t, double B) {
    const double dinf = (double)kMfDirBound;
    const double F = ldexp(1.0, -90);
    Bounds b;
    b.eA = kC * dinf * t.M + F;
    b.EW = 2.0 * (kC * 2.0 * dinf * B * t.n2 + kC * 2.0 * dinf * B * t.n1 + b.eA) + F;
    b.ET = kC * (B + t.vmax) * t.M + 2.0 * 1e-5 * (double)kFiltMaxTScale * b.eA + F;
    return b;
}

// unit direction of the cube-map point (face f, u, v): axis f / 2 with sign (f & 1 ? -1 : +1),
// u along axis (f / 2 + 1) % 3, v along (f / 2 + 2) % 3
inline void face_dir(int f, double u, double v, double out[3]) {
    const int ax = f >> 1;
    double p[3];
    p[ax] = (f & 1) ? -1.0 : 1.0;
    p[(ax + 1) % 3] = u;
    p[(ax + 2) % 3] = v;
    const double l = sqrt(p[0] * p[0] + p[1] * p[1] + p[2] * p[2]);
    for (int k = 0; k < 3; ++k) out[k] = p[k] / l;
}

// centre direction of the cube-map cell [u0, u1] x [v0, v1] of face f and a bound on the
// distance of any unit direction of the cell from it (its image is a spherical quad
// bounded by great-circle arcs, farthest from the centre at a corner), widened for the
// kernels' rounding of the cell choice
inline double cell_chord(int f, double u0, double u1, double v0, double v1, double dc[3]) {
    face_dir(f, 0.5 * (u0 + u1), 0.5 * (v0 + v1), dc);
    double chord = 0.0, q[3];
    const double us[2] = {u0, u1}, vs[2] = {v0, v1};
    for (int ku = 0; ku < 2; ++ku)
        for (int kv = 0; kv < 2; ++kv) {
            face_dir(f, us[ku], vs[kv], q);
            chord = fmax(chord, sqrt((q[0] - dc[0]) * (q[0] - dc[0]) + (q[1] - dc[1]) * (q[1] - dc[1]) +
                                     (q[2] - dc[2]) * (q[2] - dc[2])));
        }
    return chord * (1.0 + 1e-6) + 1e-6;
}

}  // namespace bnd
}  // namespace rt
