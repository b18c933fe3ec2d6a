// rt_cull.hpp — the primary-ray cull of k_render_ps, host and device alike: the render
// kernel evaluates it per wave (and k_cull_ps for the diagnostic rt_cull_masks_device),
// the host in rt_rect_candidates (the C ABI's check of the cull against the CPU
// restatement).  Single precision, no division, no fused operations (-ffp-contract=off
// on host and device): host and device compute the same masks.
//
// A camera ray through pixel (px, py) with jitter (r1, r2) in [0, 1)^2 has direction
// d = Rf p / |p| (+ rounding), p = (px + r1 - W/2, py + r2 - H/2, H), Rf the camera's float
// rotation (camera_ray).  Over a pixel rectangle every filter quantity of
// closest_hit_filtered is a linear form a.d (or a constant): Ad = N.d, U = (o x e2 - G2).d,
// V = (-(o x e1) + G1).d, T = w0 - o.N, with o the camera position.  A triangle is culled
// for the rectangle when, for every such d, the filter's rejection holds with twice its
// margins.  The filter's float evaluation differs from these real values by at most
// 18u S (record and evaluation rounding; u = 2^-24), and the bounds below enclose the real
// values: every rounding of this file is covered by an explicit slack term (`rnd` below,
// <= 2^-19 S, an eighth of a margin).  So the filter would reject every one of these
// rays, and the filter rejects only pairs whose exact test fails (build_filter,
// rt_capi.cpp): a culled triangle cannot be the hit of any primary ray of the rectangle,
// and testing the others in index order gives the reference's hit bit for bit.
#pragma once

#include "rt_internal.hpp"

namespace rt {

struct CamRect {
    float ox, oy, oz;         // camera position
    float cy, sy;             // d = R p, R = [[cy, 0, -sy], [0, 1, 0], [sy, 0, cy]] (camera_ray, PRESET 0)
    float x0, x1, y0, y1;     // p.x in [x0, x1], p.y in [y0, y1], p.z = H over the rectangle (exact)
    float H, inv_H_hi;        // H and an upper bound of 1/H
    float inv_pmax;           // a lower bound of 1 / max |p| over the rectangle (|p| >= H)
    float delta;              // bound of |d_float - R p/|p|| per component
    float rnd;                // rounding slack of form_bounds per unit of |a|_1 (16u (X + Y + H) / H)
    float ets;                // eps * t_scale as the filter computes it (RULE 0)
};

// bounds of a.d over the rectangle (a in world space), widened by `ea`, a bound of the
// rounding error of a's own evaluation.  a.(R p) = b.p with b = R^T a; over the corner set
// {x0, x1} x {y0, y1} x {H} the extremes of b.p separate per axis.
RT_HD void form_bounds(const CamRect& c, float ax, float ay, float az, float ea, float* lo, float* hi) {
    const float bx = c.cy * ax + c.sy * az;
    const float by = ay;
    const float bz = c.cy * az - c.sy * ax;
    const float ex0 = bx * c.x0, ex1 = bx * c.x1, ey0 = by * c.y0, ey1 = by * c.y1, ez = bz * c.H;
    const float l = (fminf(ex0, ex1) + fminf(ey0, ey1)) + ez;
    const float h = (fmaxf(ex0, ex1) + fmaxf(ey0, ey1)) + ez;
    const float n1 = (fabsf(ax) + fabsf(ay)) + fabsf(az);
    const float slack = (c.delta + c.rnd) * n1 + ea;
    *lo = l * (l >= 0.0f ? c.inv_pmax : c.inv_H_hi) - slack;
    *hi = h * (h >= 0.0f ? c.inv_H_hi : c.inv_pmax) + slack;
}

// true if filter record `f` certainly rejects every camera ray of the rectangle.
// Straight-line code (every test evaluated, combined at the end): no divergent returns.
template <int RULE>
RT_HD bool rect_cull(const float4* __restrict__ f, const CamRect& c) {
    constexpr float u4 = 0x1p-22f;  // 4u: bound of the rounding of a 3-term sum of products
    const float4 F0 = f[0], F1 = f[1], F2 = f[2], F3 = f[3], F4 = f[4];
    const float eA = 2.0f * F1.w, EW = 2.0f * F2.w, ET = 2.0f * F3.w;
    const float nx = F0.x, ny = F0.y, nz = F0.z;
    float alo, ahi;
    form_bounds(c, nx, ny, nz, 0.0f, &alo, &ahi);
    const bool pos = alo > eA, neg = ahi < -eA;  // the sign of the determinant is certain
    // t <= eps (RULE 0) / t < 0 (RULE 1): tm = sg (T - ets Ad), T = w0 - o.N
    const float on = (c.ox * nx + c.oy * ny) + c.oz * nz;
    const float eT = u4 * ((fabsf(F0.w) + fabsf(c.ox * nx)) + (fabsf(c.oy * ny) + fabsf(c.oz * nz)));
    const float cT = F0.w - on;
    const float tmax = (RULE == 0) ? (pos ? (cT - c.ets * alo) : (c.ets * ahi - cT)) : (pos ? cT : -cT);
    const float etm = eT + ((RULE == 0) ? u4 * (fabsf(cT) + c.ets * fmaxf(fabsf(alo), fabsf(ahi))) : 0.0f);
    // U = (o x e2 + F2).d, e2 = F1;  V = (o x F3 + F4).d, F3 = -e1
    const float ux = (c.oy * F1.z - c.oz * F1.y) + F2.x;
    const float uy = (c.oz * F1.x - c.ox * F1.z) + F2.y;
    const float uz = (c.ox * F1.y - c.oy * F1.x) + F2.z;
    const float vx = (c.oy * F3.z - c.oz * F3.y) + F4.x;
    const float vy = (c.oz * F3.x - c.ox * F3.z) + F4.y;
    const float vz = (c.ox * F3.y - c.oy * F3.x) + F4.z;
    // rounding of the coefficient vectors, summed over the components (|d_i| <= 1 + delta)
    const float eu = u4 * (((fabsf(c.oy * F1.z) + fabsf(c.oz * F1.y)) + (fabsf(c.oz * F1.x) + fabsf(c.ox * F1.z))) +
                           ((fabsf(c.ox * F1.y) + fabsf(c.oy * F1.x)) + ((fabsf(F2.x) + fabsf(F2.y)) + fabsf(F2.z))));
    const float ev = u4 * (((fabsf(c.oy * F3.z) + fabsf(c.oz * F3.y)) + (fabsf(c.oz * F3.x) + fabsf(c.ox * F3.z))) +
                           ((fabsf(c.ox * F3.y) + fabsf(c.oy * F3.x)) + ((fabsf(F4.x) + fabsf(F4.y)) + fabsf(F4.z))));
    const float wx = (nx - ux) - vx, wy = (ny - uy) - vy, wz = (nz - uz) - vz;
    const float ew = (eu + ev) + u4 * ((fabsf(wx) + fabsf(wy)) + fabsf(wz)) * 2.0f;
    float ulo, uhi, vlo, vhi, wlo, whi;
    form_bounds(c, ux, uy, uz, eu, &ulo, &uhi);
    form_bounds(c, vx, vy, vz, ev, &vlo, &vhi);
    form_bounds(c, wx, wy, wz, ew, &wlo, &whi);
    const bool u_neg = (pos ? uhi : -ulo) < -EW;  // u < 0
    const bool v_neg = (pos ? vhi : -vlo) < -EW;  // v < 0
    const bool w_neg = (pos ? whi : -wlo) < -EW;  // u + v > 1
    const bool t_out = tmax + etm < -ET;
    return (pos || neg) && (t_out || u_neg || v_neg || w_neg);
}

// The rectangle of pixels [px0, px1] x [py0, py1] (inclusive) of a width x height
// image seen from the camera at (cx, cy, cz) with yaw (cos_y, sin_y) (PRESET 0).
RT_HD CamRect make_cam_rect(float cx, float cyp, float cz, float cos_y, float sin_y, int width, int height,
                            float t_scale, int px0, int px1, int py0, int py1) {
    CamRect c;
    c.ox = cx; c.oy = cyp; c.oz = cz;
    c.cy = cos_y; c.sy = sin_y;
    const float W = (float)width, H = (float)height;
    // pixel coordinates and half sizes are integers or halves below 2^23: exact
    c.x0 = (float)px0 - 0.5f * W;
    c.x1 = (float)(px1 + 1) - 0.5f * W;
    c.y0 = (float)py0 - 0.5f * H;
    c.y1 = (float)(py1 + 1) - 0.5f * H;
    c.H = H;
    const float mx = fmaxf(fabsf(c.x0), fabsf(c.x1)), my = fmaxf(fabsf(c.y0), fabsf(c.y1));
    // bounds of the reciprocals (one rounding each, moved out by 2^-20)
    c.inv_H_hi = (1.0f / H) * (1.0f + 0x1p-20f);
    const float pmax = sqrtf((mx * mx + my * my) + H * H) * (1.0f + 0x1p-20f);
    c.inv_pmax = (1.0f / pmax) * (1.0f - 0x1p-20f);
    c.delta = 0x1p-24f * (64.0f + 8.0f * (W + H) / H);
    c.rnd = 0x1p-20f * ((mx + my) + H) / H;
    c.ets = kEps * t_scale;
    return c;
}

}  // namespace rt
