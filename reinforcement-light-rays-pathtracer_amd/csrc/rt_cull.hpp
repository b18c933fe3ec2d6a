// rt_cull.hpp — the primary-ray cull of k_render_ps (see the comment above
// CamRect), host and device alike: the kernels use it in k_cull_ps, the host in
// rt_rect_candidates (the C ABI's check of the cull against the CPU restatement).
#pragma once

#include "rt_internal.hpp"

namespace rt {

struct CamRect {
    double ox, oy, oz;        // camera position
    double cy, sy;            // d = R p, R = [[cy, 0, -sy], [0, 1, 0], [sy, 0, cy]] (camera_ray, PRESET 0)
    double x0, x1, y0, y1;    // p.x in [x0, x1], p.y in [y0, y1], p.z = H over the rectangle
    double H;
    double pmax;              // max |p| over the rectangle (|p| >= H)
    double delta;             // bound of |d_float - R p/|p|| per component
    double ets;               // eps * t_scale as the filter computes it (RULE 0)
};

// bounds of a.d over the rectangle (a in world space).  a.(R p) = b.p with b = R^T a;
// over the corner set {x0, x1} x {y0, y1} x {H} the extremes of b.p separate per axis.
RT_HD void form_bounds(const CamRect& c, double ax, double ay, double az, double* lo,
                                            double* hi) {
    const double bx = c.cy * ax + c.sy * az;
    const double by = ay;
    const double bz = c.cy * az - c.sy * ax;
    const double ex0 = bx * c.x0, ex1 = bx * c.x1, ey0 = by * c.y0, ey1 = by * c.y1, ez = bz * c.H;
    const double l = (fmin(ex0, ex1) + fmin(ey0, ey1)) + ez;
    const double h = (fmax(ex0, ex1) + fmax(ey0, ey1)) + ez;
    const double slack = c.delta * (fabs(ax) + fabs(ay) + fabs(az));
    *lo = l / (l >= 0.0 ? c.pmax : c.H) - slack;
    *hi = h / (h >= 0.0 ? c.H : c.pmax) + slack;
}

// true if filter record `f` certainly rejects every camera ray of the rectangle.
// Straight-line code (every test evaluated, combined at the end): no divergent returns.
template <int RULE>
RT_HD bool rect_cull(const float4* __restrict__ f, const CamRect& c) {
    const float4 F0 = f[0], F1 = f[1], F2 = f[2], F3 = f[3], F4 = f[4];
    const double eA = 2.0 * (double)F1.w, EW = 2.0 * (double)F2.w, ET = 2.0 * (double)F3.w;
    const double nx = F0.x, ny = F0.y, nz = F0.z;
    double alo, ahi;
    form_bounds(c, nx, ny, nz, &alo, &ahi);
    const bool pos = alo > eA, neg = ahi < -eA;  // the sign of the determinant is certain
    const double sg = pos ? 1.0 : -1.0;
    // t <= eps (RULE 0) / t < 0 (RULE 1): tm = sg (T - ets Ad), T = w0 - o.N
    const double cT = (double)F0.w - (c.ox * nx + c.oy * ny + c.oz * nz);
    const double tmax = (RULE == 0) ? (pos ? cT - c.ets * alo : -cT + c.ets * ahi) : sg * cT;
    // U = (o x e2 + F2).d, e2 = F1;  V = (o x F3 + F4).d, F3 = -e1
    const double ux = (c.oy * F1.z - c.oz * F1.y) + F2.x;
    const double uy = (c.oz * F1.x - c.ox * F1.z) + F2.y;
    const double uz = (c.ox * F1.y - c.oy * F1.x) + F2.z;
    const double vx = (c.oy * F3.z - c.oz * F3.y) + F4.x;
    const double vy = (c.oz * F3.x - c.ox * F3.z) + F4.y;
    const double vz = (c.ox * F3.y - c.oy * F3.x) + F4.z;
    double ulo, uhi, vlo, vhi, wlo, whi;
    form_bounds(c, ux, uy, uz, &ulo, &uhi);
    form_bounds(c, vx, vy, vz, &vlo, &vhi);
    form_bounds(c, nx - ux - vx, ny - uy - vy, nz - uz - vz, &wlo, &whi);
    const bool u_neg = (pos ? uhi : -ulo) < -EW;  // u < 0
    const bool v_neg = (pos ? vhi : -vlo) < -EW;  // v < 0
    const bool w_neg = (pos ? whi : -wlo) < -EW;  // u + v > 1
    const bool t_out = tmax < -ET;
    return (pos || neg) && (t_out || u_neg || v_neg || w_neg);
}

// The rectangle of pixels [px0, px1] x [py0, py1] (inclusive) of a width x height
// image seen from the camera at (cx, cy, cz) with yaw (cos_y, sin_y) (PRESET 0).
RT_HD CamRect make_cam_rect(float cx, float cyp, float cz, float cos_y, float sin_y, int width, int height,
                            float t_scale, int px0, int px1, int py0, int py1) {
    CamRect c;
    c.ox = cx; c.oy = cyp; c.oz = cz;
    c.cy = cos_y; c.sy = sin_y;
    const double W = width, H = height;
    c.x0 = (double)px0 - 0.5 * W;
    c.x1 = (double)(px1 + 1) - 0.5 * W;
    c.y0 = (double)py0 - 0.5 * H;
    c.y1 = (double)(py1 + 1) - 0.5 * H;
    c.H = H;
    const double mx = fmax(fabs(c.x0), fabs(c.x1)), my = fmax(fabs(c.y0), fabs(c.y1));
    c.pmax = sqrt(mx * mx + my * my + H * H) * (1.0 + 0x1p-40);
    c.delta = 0x1p-24 * (64.0 + 8.0 * (W + H) / H);
    c.ets = (double)(kEps * t_scale);
    return c;
}

}  // namespace rt
