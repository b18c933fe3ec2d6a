// rt_ctab.cpp — host build of the bounce-ray candidate table (rt_internal.hpp CtabHost,
// rt_trace.hpp closest_hit_ctab): both hit rules -- the CPU engine's (rule 0, t_scale >=
// CtabHost::ts_min) and the GPU engine's (rule 1, any t_scale) -- for scenes of at most 256
// triangles (1-4 mask words per entry).  Default size: kCtabPatches = 16,384 patches over the
// scene x 6 x 16 x 16 direction bins, one 8-B word per entry and mask word: about 200 MB per mask
// word (Cornell 201 MB, complex_light_room 600 MB at 3 words), built in about 1-5 s on the host's
// threads on the first render that takes it (rt_scene_ctab_info reports both).
//
// The reference tests every triangle for every ray (Ray::closest_intersection,
// CPU/rays/ray.cpp:14-28); its hit depends only on the triangles that pass the geometric
// test (Triangle::intersects), taken in index order.  A bounce ray
// starts on the surface it last hit, 1e-5 along its direction: its origin lies in a patch
// of a 2D grid over that triangle's plane (a thin parallelepiped), and its direction in a
// bin of a cube map.  For every (surface, patch, direction bin) the table holds the
// triangles that some ray from the patch with a direction in the bin may pass the exact
// test of; every other triangle fails it for every such ray.  The kernel ORs the mask of its
// ray's (patch, bin) with the mask of its fine grazing bin and runs the exact test on those
// candidates in index order: the scan's hit bit for bit.
//
// Why a triangle can be left out (rt_bounds.hpp): a pass with |A| = |d.N| >= a puts the
// plane crossing X = o + lambda d in the triangle grown to barycentrics >= -EW / a, and the
// Cramer t within (ET + |lambda| eA) / (|A| - eA) of lambda / t_scale; rule 0 passes only
// t > 1e-5, so lambda >= lambda_min = (1e-5 ts_min - ET / (a - eA)) / (1 + eA / (a - eA)).
// Three kinds of directions, by |A|:
//  * grazing, |A| < K EW (K = kBvhK): the grazing bins (kCtabGraze per face edge) list every
//    triangle whose plane such a direction can run along, whatever the origin;
//  * band, K EW <= |A| < a_g = theta_g |N|: X lies in the triangle grown by 1/K, so lambda <=
//    lam (the farthest point of that from the patch) and |T| = |lambda A| <= lam a_g (or ET
//    behind the origin): the triangle is a candidate of the coarse bins holding such
//    directions only for patches within lam theta_g + ET / |N| of its plane;
//  * regular, |A| >= a_g: X lies in the triangle grown by sigma = EW / a_g at lambda >=
//    lambda_min, so the direction of the ray is a direction of the convex set
//    P = {x - o : x in the grown triangle, o in the patch}, of length >= lambda_min: the bins
//    the central projection of P covers on each cube face (the bounding rectangle of its 24
//    projected vertices where P lies in front of the face; a P straddling the face's plane is
//    tested bin by bin against the bin's four bounding planes and split, pieces inside the
//    ball of radius lambda_min dropped).  A triangle whose plane passes within D of the whole
//    patch (the origin's own plane: D ~ 1e-5) is crossed at lambda >= lambda_min only along
//    directions with |d.n| <= D / lambda_min < theta_g: band directions, so it has no regular
//    bins.
// Rule 1 (t >= 0, no lower bound): lambda_min is 0, so the triangles coplanar with the origin's
// surface join every ray leaving it (cop, cop_th = infinity) and the rest follows with lambda >= 0.
// Origins: the kernel's patch choice (float dot products) and its check |o.n - c| <= h are
// covered by widening the patch; directions by widening the bins beyond the kernel's
// rounding of the cube-map coordinates.  A ray that is outside the table (origin off its
// surface's plane or grid, a non-finite or non-unit direction) keeps every triangle.
// Everything is computed in double.
#include <algorithm>
#include <atomic>
#include <bitset>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <unordered_map>
#include <vector>

#include "rt_bounds.hpp"
#include "rt_internal.hpp"

namespace rt {

namespace {

constexpr double kK = kBvhK;
#ifndef RT_CTAB_GFOLD
#define RT_CTAB_GFOLD 1  // 0: no grazing fold (A/B builds)
#endif
constexpr int kNc = kCtabBins;    // coarse direction bins per face edge
constexpr int kNg = kCtabGraze;   // grazing bins per face edge
using Bins = std::bitset<kNc * kNc>;  // the coarse bins of one face, bit iu * kNc + iv
constexpr double kThetaG = 0.02;  // the band |d.n| < theta_g (head comment)
constexpr int kSplitDepth = 12;   // subdivisions of a P straddling a face's plane
constexpr double kMuDir = 4e-6;   // > the kernel's rounding of u = d_a / |d_m| (and of (u + 1) kNc / 2)

// a parallelepiped: centre and three half-edge vectors
struct Ppd {
    double c[3], h[3][3];
};

void corners(const Ppd& b, double out[8][3]) {
    for (int j = 0; j < 8; ++j)
        for (int k = 0; k < 3; ++k)
            out[j][k] = b.c[k] + ((j & 1) ? b.h[0][k] : -b.h[0][k]) + ((j & 2) ? b.h[1][k] : -b.h[1][k]) +
                        ((j & 4) ? b.h[2][k] : -b.h[2][k]);
}

double len3d(const double* v) { return sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]); }

// bins [i0, i1] x [j0, j1] of one face
Bins bin_rect(int i0, int i1, int j0, int j1) {
    Bins m;
    for (int i = i0; i <= i1; ++i)
        for (int j = j0; j <= j1; ++j) m.set(i * kNc + j);
    return m;
}

// coarse bins of u over [lo, hi] (widened by kMuDir, clipped to the face)
void bin_range(double lo, double hi, int* i0, int* i1) {
    lo = std::max(-1.0, lo - kMuDir);
    hi = std::min(1.0, hi + kMuDir);
    *i0 = std::min(kNc - 1, std::max(0, (int)floor((lo + 1.0) * (kNc / 2.0))));
    *i1 = std::min(kNc - 1, std::max(0, (int)floor((hi + 1.0) * (kNc / 2.0))));
}

// The coarse bins of face f that a direction w = x - o (x in the triangle t, o in the
// parallelepiped b, |w| >= lam_min) can fall in, OR-ed into *bins.  cand: the bins still
// open.  P = {x - o} is the hull of the 24 vertex differences.
void sweep(const double t[3][3], const Ppd& b, double lam_min, int f, int depth, Bins cand, Bins* bins) {
    cand &= ~*bins;
    if (cand.none()) return;
    const int m = f >> 1, a = (m + 1) % 3, bb = (m + 2) % 3;
    const double sg = (f & 1) ? -1.0 : 1.0;
    double co[8][3];
    corners(b, co);
    double W[24][3];  // (w_m, w_a, w_b)
    double wm_min = INFINITY, wm_max = -INFINITY, wlen = 0.0, wabs = 0.0;
    double s1 = -INFINITY, s2 = -INFINITY, s3 = -INFINITY, s4 = -INFINITY;  // max of w_m -+ w_a, w_m -+ w_b
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 8; ++j) {
            double* w = W[i * 8 + j];
            const double d3[3] = {t[i][0] - co[j][0], t[i][1] - co[j][1], t[i][2] - co[j][2]};
            w[0] = sg * d3[m];
            w[1] = d3[a];
            w[2] = d3[bb];
            wlen = std::max(wlen, len3d(d3));
            wabs = std::max(wabs, std::max(fabs(w[0]), std::max(fabs(w[1]), fabs(w[2]))));
            wm_min = std::min(wm_min, w[0]);
            wm_max = std::max(wm_max, w[0]);
            s1 = std::max(s1, w[0] - w[1]);
            s2 = std::max(s2, w[0] + w[1]);
            s3 = std::max(s3, w[0] - w[2]);
            s4 = std::max(s4, w[0] + w[2]);
        }
    // the piece inside the ball |w| < lam_min (its hull is, the ball being convex)
    if (wlen * (1.0 + 1e-9) < lam_min) return;
    // P outside the face's cone {w_m >= |w_a|, w_m >= |w_b|}: a linear form negative on it
    // (beyond the rounding of the differences)
    const double ew = 1e-12 * wabs;
    if (wm_max < -ew || s1 < -ew || s2 < -ew || s3 < -ew || s4 < -ew) return;
    if (wm_min > 0.0) {
        // in front of the face: the projection of P is the hull H of its projected vertices;
        // a bin is hit iff its rectangle meets H (separating axes: H's edge normals and the
        // rectangle's own axes, the latter by the bounding rectangle)
        double pu[24], pv[24];
        double umin = INFINITY, umax = -INFINITY, vmin = INFINITY, vmax = -INFINITY;
        for (int k = 0; k < 24; ++k) {
            pu[k] = W[k][1] / W[k][0];
            pv[k] = W[k][2] / W[k][0];
            umin = std::min(umin, pu[k]);
            umax = std::max(umax, pu[k]);
            vmin = std::min(vmin, pv[k]);
            vmax = std::max(vmax, pv[k]);
        }
        const double rel = 1e-12;
        int i0, i1, j0, j1;
        bin_range(umin - rel * fabs(umin), umax + rel * fabs(umax), &i0, &i1);
        bin_range(vmin - rel * fabs(vmin), vmax + rel * fabs(vmax), &j0, &j1);
        // the hull (monotone chain), counter-clockwise
        int idx[24];
        for (int k = 0; k < 24; ++k) idx[k] = k;
        std::sort(idx, idx + 24, [&](int x, int y) { return pu[x] < pu[y] || (pu[x] == pu[y] && pv[x] < pv[y]); });
        int hull[50], nh = 0;
        auto cross2 = [&](int o, int a2, int b2) {
            return (pu[a2] - pu[o]) * (pv[b2] - pv[o]) - (pv[a2] - pv[o]) * (pu[b2] - pu[o]);
        };
        for (int k = 0; k < 24; ++k) {
            while (nh >= 2 && cross2(hull[nh - 2], hull[nh - 1], idx[k]) <= 0.0) --nh;
            hull[nh++] = idx[k];
        }
        for (int k = 22, lo2 = nh + 1; k >= 0; --k) {
            while (nh >= lo2 && cross2(hull[nh - 2], hull[nh - 1], idx[k]) <= 0.0) --nh;
            hull[nh++] = idx[k];
        }
        --nh;  // the last point repeats the first
        const double scale = 1.0 + std::max(std::max(fabs(umin), fabs(umax)), std::max(fabs(vmin), fabs(vmax)));
        for (int iu = i0; iu <= i1; ++iu)
            for (int iv = j0; iv <= j1; ++iv) {
                const int q = iu * kNc + iv;
                if (!cand.test(q)) continue;
                bool sep = false;
                if (nh >= 3) {
                    const double ru0 = -1.0 + 2.0 * iu / kNc - kMuDir, ru1 = -1.0 + 2.0 * (iu + 1) / kNc + kMuDir;
                    const double rv0 = -1.0 + 2.0 * iv / kNc - kMuDir, rv1 = -1.0 + 2.0 * (iv + 1) / kNc + kMuDir;
                    const double cu[4] = {ru0, ru1, ru1, ru0}, cv[4] = {rv0, rv0, rv1, rv1};
                    for (int e = 0; e < nh && !sep; ++e) {
                        const int a2 = hull[e], b2 = hull[(e + 1) % nh];
                        const double eu = pu[b2] - pu[a2], ev = pv[b2] - pv[a2];
                        // outward normal of a counter-clockwise edge: (ev, -eu)
                        const double len = sqrt(eu * eu + ev * ev);
                        if (!(len > 0.0)) continue;
                        const double slack = 1e-9 * scale * len;
                        bool out = true;
                        for (int c = 0; c < 4 && out; ++c)
                            out = (ev * (cu[c] - pu[a2]) - eu * (cv[c] - pv[a2])) > slack;
                        sep = out;
                    }
                }
                if (!sep) bins->set(q);
            }
        return;
    }
    {
        // straddling: keep the bins whose cone {u0 w_m <= w_a <= u1 w_m, v0 w_m <= w_b <= v1 w_m}
        // no bounding plane separates from P
        Bins open;
        const double eps = 4.0 * ew;
        for (int q = 0; q < kNc * kNc; ++q) {
            if (!cand.test(q)) continue;
            const int iu = q / kNc, iv = q % kNc;
            const double u0 = -1.0 + 2.0 * iu / kNc - kMuDir, u1 = -1.0 + 2.0 * (iu + 1) / kNc + kMuDir;
            const double v0 = -1.0 + 2.0 * iv / kNc - kMuDir, v1 = -1.0 + 2.0 * (iv + 1) / kNc + kMuDir;
            double m1 = -INFINITY, m2 = -INFINITY, m3 = -INFINITY, m4 = -INFINITY;
            for (const auto& w : W) {
                m1 = std::max(m1, w[1] - u0 * w[0]);
                m2 = std::max(m2, u1 * w[0] - w[1]);
                m3 = std::max(m3, w[2] - v0 * w[0]);
                m4 = std::max(m4, v1 * w[0] - w[2]);
            }
            if (m1 >= -eps && m2 >= -eps && m3 >= -eps && m4 >= -eps) open.set(q);
        }
        if (open.none()) return;
        if (depth >= kSplitDepth) {
            *bins |= open;
            return;
        }
        cand = open;
    }
    // split the larger of the two generators
    double lt = 0.0;
    for (int i = 0; i < 3; ++i) {
        const double e[3] = {t[(i + 1) % 3][0] - t[i][0], t[(i + 1) % 3][1] - t[i][1], t[(i + 1) % 3][2] - t[i][2]};
        lt = std::max(lt, len3d(e));
    }
    int bax = 0;
    double lb = 0.0;
    for (int k = 0; k < 3; ++k)
        if (2.0 * len3d(b.h[k]) > lb) {
            lb = 2.0 * len3d(b.h[k]);
            bax = k;
        }
    if (lt >= lb) {
        double mid[3][3];  // mid[i]: the midpoint of edge (i, i + 1)
        for (int i = 0; i < 3; ++i)
            for (int k = 0; k < 3; ++k) mid[i][k] = 0.5 * (t[i][k] + t[(i + 1) % 3][k]);
        const double* parts[4][3] = {{t[0], mid[0], mid[2]}, {mid[0], t[1], mid[1]},
                                     {mid[2], mid[1], t[2]}, {mid[0], mid[1], mid[2]}};
        for (const auto& p : parts) {
            double s[3][3];
            for (int q = 0; q < 3; ++q)
                for (int k = 0; k < 3; ++k) s[q][k] = p[q][k];
            sweep(s, b, lam_min, f, depth + 1, cand, bins);
        }
    } else {
        Ppd h1 = b, h2 = b;
        for (int k = 0; k < 3; ++k) {
            h1.h[bax][k] = h2.h[bax][k] = 0.5 * b.h[bax][k];
            h1.c[k] = b.c[k] - 0.5 * b.h[bax][k];
            h2.c[k] = b.c[k] + 0.5 * b.h[bax][k];
        }
        sweep(t, h1, lam_min, f, depth + 1, cand, bins);
        sweep(t, h2, lam_min, f, depth + 1, cand, bins);
    }
}

// inverse of the 3x3 matrix with rows r[0..2]
bool inv3(const double r[3][3], double inv[3][3]) {
    const double det = r[0][0] * (r[1][1] * r[2][2] - r[1][2] * r[2][1]) -
                       r[0][1] * (r[1][0] * r[2][2] - r[1][2] * r[2][0]) +
                       r[0][2] * (r[1][0] * r[2][1] - r[1][1] * r[2][0]);
    if (!(fabs(det) > 1e-6)) return false;
    inv[0][0] = (r[1][1] * r[2][2] - r[1][2] * r[2][1]) / det;
    inv[0][1] = (r[0][2] * r[2][1] - r[0][1] * r[2][2]) / det;
    inv[0][2] = (r[0][1] * r[1][2] - r[0][2] * r[1][1]) / det;
    inv[1][0] = (r[1][2] * r[2][0] - r[1][0] * r[2][2]) / det;
    inv[1][1] = (r[0][0] * r[2][2] - r[0][2] * r[2][0]) / det;
    inv[1][2] = (r[0][2] * r[1][0] - r[0][0] * r[1][2]) / det;
    inv[2][0] = (r[1][0] * r[2][1] - r[1][1] * r[2][0]) / det;
    inv[2][1] = (r[0][1] * r[2][0] - r[0][0] * r[2][1]) / det;
    inv[2][2] = (r[0][0] * r[1][1] - r[0][1] * r[1][0]) / det;
    return true;
}

// does the 2D triangle (p[3][2]) meet the rectangle [x0, x1] x [y0, y1]?  (separating axes)
bool tri_rect_2d(const double p[3][2], double x0, double x1, double y0, double y1) {
    double mn[2] = {INFINITY, INFINITY}, mx[2] = {-INFINITY, -INFINITY};
    for (int i = 0; i < 3; ++i)
        for (int k = 0; k < 2; ++k) {
            mn[k] = std::min(mn[k], p[i][k]);
            mx[k] = std::max(mx[k], p[i][k]);
        }
    if (mn[0] > x1 || mx[0] < x0 || mn[1] > y1 || mx[1] < y0) return false;
    const double rx[4] = {x0, x1, x1, x0}, ry[4] = {y0, y0, y1, y1};
    for (int i = 0; i < 3; ++i) {
        const double ex = p[(i + 1) % 3][0] - p[i][0], ey = p[(i + 1) % 3][1] - p[i][1];
        const double nx = -ey, ny = ex;  // edge normal
        double tmin = INFINITY, tmax = -INFINITY;
        for (int q = 0; q < 3; ++q) {
            const double s = nx * p[q][0] + ny * p[q][1];
            tmin = std::min(tmin, s);
            tmax = std::max(tmax, s);
        }
        double rmin = INFINITY, rmax = -INFINITY;
        for (int q = 0; q < 4; ++q) {
            const double s = nx * rx[q] + ny * ry[q];
            rmin = std::min(rmin, s);
            rmax = std::max(rmax, s);
        }
        const double slack = 1e-9 * (fabs(tmin) + fabs(tmax) + fabs(rmin) + fabs(rmax));
        if (rmin > tmax + slack || rmax < tmin - slack) return false;
    }
    return true;
}

}  // namespace

// Builds the candidate table of a scene of n <= 64 triangles (isect: their kIsectF4
// records, the first n_surf surfaces); B: a bound on |o_i| of the rays it serves
// (DeviceScene::mf_bound; raised to every origin the patch grids accept); ts_min: the
// smallest t_scale it serves.  Returns false if the scene is out of the filter's ranges or
// too large.
bool ctab_build(const float4* isect, int n, int n_surf, double B, int rule, double ts_min, CtabHost* out) {
    if (n <= 0 || n > 64 * kCtabMaxWords || n_surf <= 0 || n_surf > n || !(B < ldexp(1.0, 20))) return false;
    if (rule != 0 && rule != 1) return false;
    const int W = (n + 63) / 64;  // mask words per entry
    std::vector<bnd::TriAlg> ta((size_t)n);
    std::vector<double> vt((size_t)n * 9);
    double vmax = 0.0;
    for (int i = 0; i < n; ++i) {
        const float4 P0 = isect[(size_t)i * 3], P1 = isect[(size_t)i * 3 + 1], P2 = isect[(size_t)i * 3 + 2];
        ta[(size_t)i] = bnd::tri_alg(P0, P1, P2);
        if (!(ta[(size_t)i].M < ldexp(1.0, 36)) || !(ta[(size_t)i].nlen > 0.0)) return false;
        const double v0[3] = {P0.x, P0.y, P0.z}, e1[3] = {P1.x, P1.y, P1.z}, e2[3] = {P2.x, P2.y, P2.z};
        for (int k = 0; k < 3; ++k) {
            // the geometric triangle of the record: v0 + u e1 + v e2
            vt[(size_t)i * 9 + k] = v0[k];
            vt[(size_t)i * 9 + 3 + k] = v0[k] + e1[k];
            vt[(size_t)i * 9 + 6 + k] = v0[k] + e2[k];
            for (int q = 0; q < 3; ++q) vmax = std::max(vmax, fabs(vt[(size_t)i * 9 + 3 * q + k]));
        }
    }
    CtabHost& h = *out;
    h = CtabHost();
    h.n_tri = n;
    h.n_surf = n_surf;
    h.words = W;
    h.rule = rule;
    h.ts_min = rule == 0 ? (float)ts_min : 0.0f;
    // the origin slab: 1e-5 |sd| off the surface (|sd| = 1 to float precision) plus the
    // rounding of the hit point and of the kernel's frame (a few 1e-7 at these coordinates)
    h.h_run = bnd::up(1.1e-5 + 1e-6 * (1.0 + vmax));
    const double mu = 2e-6 * (1.0 + vmax);  // > the rounding of the kernel's dot products with the frame
    const double h_slab = (double)h.h_run + mu;

    // the surfaces' patch grids: frame (O', U, V, N) in float, cell size c
    double area = 0.0;
    struct Frame {
        float O[3], U[3], V[3], N[3];
        double p2[3][2];  // the triangle in (u, v)
    };
    std::vector<Frame> fr((size_t)n_surf);
    for (int s = 0; s < n_surf; ++s) {
        const double* v = &vt[(size_t)s * 9];
        double e1[3], n3[3];
        for (int k = 0; k < 3; ++k) {
            e1[k] = v[3 + k] - v[k];
            n3[k] = -ta[(size_t)s].N[k] / ta[(size_t)s].nlen;  // the shading normal, cross(e2, e1)
        }
        const double l1 = len3d(e1);
        double U[3], V[3];
        for (int k = 0; k < 3; ++k) U[k] = e1[k] / l1;
        V[0] = n3[1] * U[2] - n3[2] * U[1];
        V[1] = n3[2] * U[0] - n3[0] * U[2];
        V[2] = n3[0] * U[1] - n3[1] * U[0];
        Frame& F = fr[(size_t)s];
        for (int k = 0; k < 3; ++k) {
            F.U[k] = (float)U[k];
            F.V[k] = (float)V[k];
            F.N[k] = (float)n3[k];
        }
        double lo[2] = {INFINITY, INFINITY}, hi[2] = {-INFINITY, -INFINITY};
        for (int q = 0; q < 3; ++q) {
            double p[2] = {0, 0};
            for (int k = 0; k < 3; ++k) {
                p[0] += (v[q * 3 + k] - v[k]) * (double)F.U[k];
                p[1] += (v[q * 3 + k] - v[k]) * (double)F.V[k];
            }
            for (int k = 0; k < 2; ++k) {
                lo[k] = std::min(lo[k], p[k]);
                hi[k] = std::max(hi[k], p[k]);
            }
        }
        const double pad = 4.0 * mu;
        for (int k = 0; k < 3; ++k)
            F.O[k] = (float)(v[k] + (lo[0] - pad) * (double)F.U[k] + (lo[1] - pad) * (double)F.V[k]);
        area += (hi[0] - lo[0] + 2 * pad) * (hi[1] - lo[1] + 2 * pad);
    }
    const double c = std::max(sqrt(area / (double)kCtabPatches), 1e-6);
    const float inv_c = (float)(1.0 / c);
    const double cr = 1.0 / (double)inv_c;  // the cell size the kernel's float inv_c gives
    h.tri.resize((size_t)n_surf * 4);
    int n_patch = 0;
    std::vector<int> nu((size_t)n_surf), nv((size_t)n_surf), base((size_t)n_surf);
    for (int s = 0; s < n_surf; ++s) {
        Frame& F = fr[(size_t)s];
        const double* v = &vt[(size_t)s * 9];
        double ext[2] = {0, 0};
        for (int q = 0; q < 3; ++q) {
            double p[2] = {0, 0};
            for (int k = 0; k < 3; ++k) {
                p[0] += (v[q * 3 + k] - (double)F.O[k]) * (double)F.U[k];
                p[1] += (v[q * 3 + k] - (double)F.O[k]) * (double)F.V[k];
            }
            F.p2[q][0] = p[0];
            F.p2[q][1] = p[1];
            ext[0] = std::max(ext[0], p[0]);
            ext[1] = std::max(ext[1], p[1]);
        }
        nu[(size_t)s] = std::max(1, (int)ceil((ext[0] + 4.0 * mu) / cr));
        nv[(size_t)s] = std::max(1, (int)ceil((ext[1] + 4.0 * mu) / cr));
        base[(size_t)s] = n_patch;
        n_patch += nu[(size_t)s] * nv[(size_t)s];
        if (n_patch > (1 << 22)) return false;
        int32_t bits[3] = {nu[(size_t)s], nv[(size_t)s], base[(size_t)s]};
        float fb[3];
        memcpy(fb, bits, sizeof fb);
        h.tri[(size_t)s * 4 + 0] = make_float4(F.O[0], F.O[1], F.O[2], inv_c);
        h.tri[(size_t)s * 4 + 1] = make_float4(F.U[0], F.U[1], F.U[2], fb[0]);
        h.tri[(size_t)s * 4 + 2] = make_float4(F.V[0], F.V[1], F.V[2], fb[1]);
        h.tri[(size_t)s * 4 + 3] = make_float4(F.N[0], F.N[1], F.N[2], fb[2]);
    }
    // the bound on |o_i| the filter's margins are taken at: every origin the kernel accepts
    // lies in some surface's patch grid
    for (int s = 0; s < n_surf; ++s) {
        const Frame& F = fr[(size_t)s];
        const double R[3][3] = {{F.U[0], F.U[1], F.U[2]}, {F.V[0], F.V[1], F.V[2]}, {F.N[0], F.N[1], F.N[2]}};
        double Ri[3][3];
        if (!inv3(R, Ri)) return false;
        for (int j = 0; j < 8; ++j) {
            const double uvw[3] = {(j & 1) ? nu[(size_t)s] * cr + mu : -mu, (j & 2) ? nv[(size_t)s] * cr + mu : -mu,
                                   (j & 4) ? h_slab : -h_slab};
            for (int k = 0; k < 3; ++k)
                B = std::max(B, fabs((double)F.O[k] + Ri[k][0] * uvw[0] + Ri[k][1] * uvw[1] + Ri[k][2] * uvw[2]) *
                                    (1.0 + 1e-9));
        }
    }
    if (!(B < ldexp(1.0, 20))) return false;
    // per triangle: the regular directions' growth sigma and lambda_min, ET / |N|, the unit
    // normal; per triangle, face and bin: does the bin hold a band direction (|d.n| < theta_g)?
    std::vector<double> sig((size_t)n), lmin((size_t)n), et_n((size_t)n), un((size_t)n * 3);
    std::vector<Bins> band((size_t)n * 6);
    for (int i = 0; i < n; ++i) {
        const bnd::TriAlg& t = ta[(size_t)i];
        const bnd::Bounds bo = bnd::bounds_for(t, B);
        const double ag = std::max(kK * bo.EW, kThetaG * t.nlen * (1.0 - 1e-6));
        if (!(ag > 2.0 * bo.eA)) return false;
        sig[(size_t)i] = bo.EW / ag * (1.0 + 1e-9);
        const double den = ag - bo.eA;
        // rule 0 passes t > 1e-5f (= 9.99999975e-6 > 0.99999e-5); rule 1 passes t >= 0 (no bound
        // away from the origin)
        lmin[(size_t)i] = rule == 0 ? std::max(0.0, (0.99999e-5 * ts_min - bo.ET / den) / (1.0 + bo.eA / den)) *
                                          (1.0 - 1e-6)
                                    : 0.0;
        et_n[(size_t)i] = bo.ET / t.nlen;
        for (int k = 0; k < 3; ++k) un[(size_t)i * 3 + k] = t.N[k] / t.nlen;
        for (int f = 0; f < 6; ++f)
            for (int iu = 0; iu < kNc; ++iu)
                for (int iv = 0; iv < kNc; ++iv) {
                    const double u0 = -1.0 + 2.0 * iu / kNc - kMuDir, u1 = -1.0 + 2.0 * (iu + 1) / kNc + kMuDir;
                    const double v0 = -1.0 + 2.0 * iv / kNc - kMuDir, v1 = -1.0 + 2.0 * (iv + 1) / kNc + kMuDir;
                    double dc[3];
                    const double chord = bnd::cell_chord(f, u0, u1, v0, v1, dc);
                    const double mn = fabs(dc[0] * un[(size_t)i * 3] + dc[1] * un[(size_t)i * 3 + 1] +
                                           dc[2] * un[(size_t)i * 3 + 2]) - chord;
                    if (mn < kThetaG) band[(size_t)i * 6 + f].set(iu * kNc + iv);
                }
    }
    const int per_patch = 6 * kNc * kNc * W;  // mask words per patch
    auto all_word = [&](int w) { return (n - 64 * w >= 64) ? ~0ull : ((1ull << (n - 64 * w)) - 1ull); };
    h.masks.assign((size_t)n_patch * per_patch, 0ull);
    h.cop.assign((size_t)n_surf * W, 0ull);
    // the surfaces' patches, one surface per task on the host's threads
    std::vector<double> cop_th_s((size_t)n_surf, 0.0);
    std::vector<int> whole_s((size_t)n_surf, 0);
    std::vector<char> ok_s((size_t)n_surf, 1);
    auto build_surface = [&](int s) -> bool {
        const Frame& F = fr[(size_t)s];
        double& cop_th = cop_th_s[(size_t)s];
        // the triangles coplanar with s: crossed at lambda >= lambda_min from anywhere on s
        // only along directions with |d.n| < theta_j (their plane within D of every patch of
        // s, D / lambda_min < theta_g); the kernel adds them where |d.N_s| < cop_th instead
        // of through the patches' bins
        std::vector<uint64_t> cop((size_t)W, 0ull);
        {
            // the corners of s's whole patch grid
            const double R[3][3] = {{F.U[0], F.U[1], F.U[2]}, {F.V[0], F.V[1], F.V[2]}, {F.N[0], F.N[1], F.N[2]}};
            double Ri[3][3];
            if (!inv3(R, Ri)) return false;
            double gc[8][3];
            for (int j = 0; j < 8; ++j) {
                const double uvw[3] = {(j & 1) ? nu[(size_t)s] * cr + mu : -mu, (j & 2) ? nv[(size_t)s] * cr + mu : -mu,
                                       (j & 4) ? h_slab : -h_slab};
                for (int k = 0; k < 3; ++k)
                    gc[j][k] = (double)F.O[k] + Ri[k][0] * uvw[0] + Ri[k][1] * uvw[1] + Ri[k][2] * uvw[2];
            }
            for (int i = 0; i < n; ++i) {
                const double* v = &vt[(size_t)i * 9];
                const double* nn = &un[(size_t)i * 3];
                const double pc = v[0] * nn[0] + v[1] * nn[1] + v[2] * nn[2];
                double dmax = 0.0;
                for (const auto& x : gc) dmax = std::max(dmax, fabs(x[0] * nn[0] + x[1] * nn[1] + x[2] * nn[2] - pc));
                const double D = dmax * (1.0 + 1e-9) + 1e-12 * (1.0 + fabs(pc));
                const double lm = lmin[(size_t)i];
                if (rule == 1) {
                    // rule 1 (t >= 0): the plane of s, up to rounding, may be passed right at the
                    // origin in any direction -- a candidate of every ray leaving s
                    if (D <= 1e-4 * (1.0 + vmax)) {
                        cop[(size_t)(i >> 6)] |= 1ull << (i & 63);
                        cop_th = 4.0;
                    }
                    continue;
                }
                if (!(lm > 0.0 && D / lm < kThetaG * (1.0 - 1e-6))) continue;
                cop[(size_t)(i >> 6)] |= 1ull << (i & 63);
                const bnd::Bounds bo = bnd::bounds_for(ta[(size_t)i], B);
                const double th_j = std::max(std::max(kK * bo.EW, kThetaG * ta[(size_t)i].nlen) / ta[(size_t)i].nlen,
                                             kThetaG) * (1.0 + 1e-5);
                // |d.N_s| >= |d.n_j| - |d| |N_s -+ n_j|
                const double Ns[3] = {F.N[0], F.N[1], F.N[2]};
                const double sgn = (Ns[0] * nn[0] + Ns[1] * nn[1] + Ns[2] * nn[2]) < 0.0 ? -1.0 : 1.0;
                const double dn[3] = {Ns[0] - sgn * nn[0], Ns[1] - sgn * nn[1], Ns[2] - sgn * nn[2]};
                cop_th = std::max(cop_th, th_j + len3d(dn) * 1.001 + 1e-6);
            }
        }
        for (int w = 0; w < W; ++w) h.cop[(size_t)s * W + w] = cop[(size_t)w];
        // the bins holding a direction of s's hemisphere (d.N_s >= -kCtabHemi: the kernel keeps
        // every triangle for the others); the rest stay empty
        Bins hemi[6];
        for (int f = 0; f < 6; ++f)
            for (int iu = 0; iu < kNc; ++iu)
                for (int iv = 0; iv < kNc; ++iv) {
                    const double u0 = -1.0 + 2.0 * iu / kNc - kMuDir, u1 = -1.0 + 2.0 * (iu + 1) / kNc + kMuDir;
                    const double v0 = -1.0 + 2.0 * iv / kNc - kMuDir, v1 = -1.0 + 2.0 * (iv + 1) / kNc + kMuDir;
                    double dc[3];
                    const double chord = bnd::cell_chord(f, u0, u1, v0, v1, dc);
                    const double dn = dc[0] * F.N[0] + dc[1] * F.N[1] + dc[2] * F.N[2];
                    if (dn + chord * 1.001 >= -2.0 * (double)kCtabHemi - 1e-6) hemi[f].set(iu * kNc + iv);
                }
        // (u, v, w) -> x = O' + Ri (u, v, w): Ri inverts the float frame's rows
        const double R[3][3] = {{F.U[0], F.U[1], F.U[2]}, {F.V[0], F.V[1], F.V[2]}, {F.N[0], F.N[1], F.N[2]}};
        double Ri[3][3];
        if (!inv3(R, Ri)) return false;
        for (int iu = 0; iu < nu[(size_t)s]; ++iu)
            for (int iv = 0; iv < nv[(size_t)s]; ++iv) {
                uint64_t* cm = &h.masks[(size_t)(base[(size_t)s] + iu * nv[(size_t)s] + iv) * per_patch];
                const double u0 = iu * cr - mu, u1 = (iu + 1) * cr + mu;
                const double v0 = iv * cr - mu, v1 = (iv + 1) * cr + mu;
                if (!tri_rect_2d(F.p2, u0 - 4.0 * mu, u1 + 4.0 * mu, v0 - 4.0 * mu, v1 + 4.0 * mu)) {
                    for (int q = 0; q < per_patch; ++q) cm[q] = all_word(q % W);  // off the triangle
                    ++whole_s[(size_t)s];
                    continue;
                }
                // the patch's origins: a parallelepiped
                Ppd P;
                const double mid[3] = {0.5 * (u0 + u1), 0.5 * (v0 + v1), 0.0};
                const double half[3] = {0.5 * (u1 - u0), 0.5 * (v1 - v0), h_slab};
                for (int k = 0; k < 3; ++k) {
                    P.c[k] = (double)F.O[k] + Ri[k][0] * mid[0] + Ri[k][1] * mid[1] + Ri[k][2] * mid[2];
                    for (int e = 0; e < 3; ++e) P.h[e][k] = Ri[k][e] * half[e];
                }
                double co[8][3];
                corners(P, co);
                for (int i = 0; i < n; ++i) {
                    if ((cop[(size_t)(i >> 6)] >> (i & 63)) & 1ull) continue;  // the kernel's |d.N_s| test
                    const double* v = &vt[(size_t)i * 9];
                    const double* nn = &un[(size_t)i * 3];
                    const double pc = (v[0] * nn[0] + v[1] * nn[1] + v[2] * nn[2]);
                    // the patch's distances to the triangle's plane
                    double dmin = INFINITY, dmax = -INFINITY;
                    for (const auto& x : co) {
                        const double dd = x[0] * nn[0] + x[1] * nn[1] + x[2] * nn[2] - pc;
                        dmin = std::min(dmin, dd);
                        dmax = std::max(dmax, dd);
                    }
                    const double dabs = std::max(fabs(dmin), fabs(dmax)) * (1.0 + 1e-9) + 1e-12 * (1.0 + fabs(pc));
                    const double dist = (dmin > 0.0 || dmax < 0.0) ? std::min(fabs(dmin), fabs(dmax)) : 0.0;
                    // band: the farthest point of the triangle grown by 1/K from the patch
                    double lam = 0.0;
                    const double g = 1.0 / kK;
                    for (int q = 0; q < 3; ++q) {
                        double x[3];
                        for (int k = 0; k < 3; ++k)
                            x[k] = v[q * 3 + k] +
                                   g * (2.0 * v[q * 3 + k] - v[((q + 1) % 3) * 3 + k] - v[((q + 2) % 3) * 3 + k]);
                        for (const auto& o : co) {
                            const double w[3] = {x[0] - o[0], x[1] - o[1], x[2] - o[2]};
                            lam = std::max(lam, len3d(w));
                        }
                    }
                    lam = lam / (1.0 - 1e-6);  // |d| >= 1 - 1e-6
                    const double reach = (lam * kThetaG + et_n[(size_t)i]) * (1.0 + 1e-6) + 1e-9 * (1.0 + fabs(pc));
                    const bool band_near = dist * (1.0 - 1e-9) <= reach;
                    // regular: none when the plane passes within D of the whole patch with
                    // D / lambda_min < theta_g (those crossings need band directions)
                    const double lm = lmin[(size_t)i];
                    const bool regular = !(lm > 0.0 && dabs / lm < kThetaG * (1.0 - 1e-6));
                    double tg[3][3];
                    const double sgm = sig[(size_t)i];
                    for (int q = 0; q < 3; ++q)
                        for (int k = 0; k < 3; ++k)
                            tg[q][k] = v[q * 3 + k] +
                                       sgm * (2.0 * v[q * 3 + k] - v[((q + 1) % 3) * 3 + k] - v[((q + 2) % 3) * 3 + k]);
                    for (int f = 0; f < 6; ++f) {
                        Bins bins;
                        if (regular) sweep(tg, P, lm, f, 0, hemi[f], &bins);
                        if (band_near) bins |= band[(size_t)i * 6 + f] & hemi[f];
                        for (int q = 0; q < kNc * kNc; ++q)
                            if (bins.test(q)) cm[(size_t)(f * kNc * kNc + q) * W + (i >> 6)] |= 1ull << (i & 63);
                    }
                }
            }
        return true;
    };
    {
        std::atomic<int> next(0);
        const int n_thr = std::max(1, std::min(16, (int)std::thread::hardware_concurrency()));
        std::vector<std::thread> pool;
        for (int k = 0; k < n_thr; ++k)
            pool.emplace_back([&]() {
                for (int s = next++; s < n_surf; s = next++) ok_s[(size_t)s] = build_surface(s) ? 1 : 0;
            });
        for (auto& th : pool) th.join();
    }
    double cop_th = 0.0;
    for (int s = 0; s < n_surf; ++s) {
        if (!ok_s[(size_t)s]) return false;
        cop_th = std::max(cop_th, cop_th_s[(size_t)s]);
        h.patches_all += whole_s[(size_t)s];
    }

    // grazing bins: every triangle a direction of the bin can run along (|d.N| < K EW)
    h.graze.assign((size_t)6 * kNg * kNg * W, 0ull);
    for (int f = 0; f < 6; ++f)
        for (int iu = 0; iu < kNg; ++iu)
            for (int iv = 0; iv < kNg; ++iv) {
                const double u0 = -1.0 + 2.0 * iu / kNg - kMuDir, u1 = -1.0 + 2.0 * (iu + 1) / kNg + kMuDir;
                const double v0 = -1.0 + 2.0 * iv / kNg - kMuDir, v1 = -1.0 + 2.0 * (iv + 1) / kNg + kMuDir;
                double dc[3];
                const double chord = bnd::cell_chord(f, u0, u1, v0, v1, dc);
                uint64_t* m = &h.graze[((size_t)(f * kNg + iu) * kNg + iv) * W];
                for (int i = 0; i < n; ++i) {
                    const bnd::TriAlg& t = ta[(size_t)i];
                    const bnd::Bounds bo = bnd::bounds_for(t, B);
                    const double dn = fabs(dc[0] * t.N[0] + dc[1] * t.N[1] + dc[2] * t.N[2]) / t.nlen;
                    // |d.N| >= (1 - 1e-6) |N| (dn - chord) for every direction of the bin
                    if ((dn - chord) * (1.0 - 1e-6) * t.nlen < kK * bo.EW * 1.01) m[i >> 6] |= 1ull << (i & 63);
                }
            }
    h.n_patch = n_patch;
    h.cop_th = bnd::up(cop_th);
    // the grazing bins' dictionary (16-bit indices: a table with more is not built)
    {
        struct Key {
            uint64_t w[kCtabMaxWords];
            bool operator==(const Key& o) const { return memcmp(w, o.w, sizeof w) == 0; }
        };
        struct KeyHash {
            size_t operator()(const Key& k) const {
                uint64_t x = 0x9e3779b97f4a7c15ull;
                for (uint64_t v : k.w) x = (x ^ v) * 0xff51afd7ed558ccdull ^ (x >> 29);
                return (size_t)x;
            }
        };
        std::unordered_map<Key, uint32_t, KeyHash> ids;
        h.gid.resize(h.graze.size() / (size_t)W);
        for (size_t e = 0; e < h.gid.size(); ++e) {
            Key k;
            memset(k.w, 0, sizeof k.w);
            for (int w = 0; w < W; ++w) k.w[w] = h.graze[e * (size_t)W + (size_t)w];
            auto it = ids.find(k);
            if (it == ids.end()) {
                if (ids.size() > 0xffffu) return false;
                it = ids.emplace(k, (uint32_t)ids.size()).first;
                for (int w = 0; w < W; ++w) h.gdict.push_back(k.w[w]);
            }
            h.gid[e] = (uint16_t)it->second;
        }
        std::vector<uint64_t>().swap(h.graze);
        // The grazing fold (scenes whose triangle count is not a multiple of 64: bit 63 of the
        // last mask word is free).  A coarse bin (f, iu, iv) holds the fine grazing bins (f, gu, gv)
        // with gu / r = iu, gv / r = iv (kNg = r kNc, r a power of two: the kernel's bin indices are
        // floor(u1 kN / 2) of the same u1, so a fine bin's coarse bin is its index / r).  Where they
        // all share one grazing mask, that mask is OR-ed into every patch's entry of the bin -- the
        // lookup's F = mm | gg is unchanged -- and elsewhere bit 63 of the entries' last word is set:
        // look the grazing mask up.  A ray in a folded bin then needs one dependent memory access
        // (its entry), not two.
        h.gflag = 0;
        if (RT_CTAB_GFOLD && n < 64 * W && kNg % kNc == 0) {
            const int sh = kNg / kNc;
            size_t folded = 0;
            std::vector<int32_t> fold(6 * kNc * kNc, -1);
            for (int f = 0; f < 6; ++f)
                for (int iu = 0; iu < kNc; ++iu)
                    for (int iv = 0; iv < kNc; ++iv) {
                        const uint16_t g0 = h.gid[(size_t)(f * kNg + iu * sh) * kNg + iv * sh];
                        bool same = true;
                        for (int a = 0; a < sh && same; ++a)
                            for (int b = 0; b < sh && same; ++b)
                                same = h.gid[(size_t)(f * kNg + iu * sh + a) * kNg + iv * sh + b] == g0;
                        if (same) {
                            fold[(size_t)(f * kNc + iu) * kNc + iv] = g0;
                            ++folded;
                        }
                    }
            const size_t per = (size_t)6 * kNc * kNc;
            const size_t entries = h.masks.size() / (size_t)W;
            for (size_t e = 0; e < entries; ++e) {
                const int32_t g = fold[e % per];
                uint64_t* m = &h.masks[e * (size_t)W];
                if (g >= 0) {
                    for (int w = 0; w < W; ++w) m[w] |= h.gdict[(size_t)g * W + w];
                } else {
                    m[W - 1] |= kCtabGflagBit;
                }
            }
            h.gflag = 1;
            if (getenv("RT_CTAB_VERBOSE"))
                fprintf(stderr, "rtmi: candidate table: %zu of %zu coarse bins folded\n", folded, per);
        }
        if (getenv("RT_CTAB_VERBOSE"))
            fprintf(stderr, "rtmi: candidate table: %d triangles, rule %d, %d patches (%.1f MB), %zu distinct grazing masks\n",
                    n, rule, n_patch, h.masks.size() * 8e-6, ids.size());
    }
    return true;
}

// The kernel's lookup (rt_trace.hpp ctab_candidates) on the host, with the same float
// operations: the candidate mask (h.words words into out) of the ray (o, d) leaving surface
// s, or every triangle where the table does not apply.
void ctab_lookup(const CtabHost& h, int s, const float o[3], const float d[3], uint64_t* out) {
    const int W = h.words;
    for (int w = 0; w < W; ++w) out[w] = (h.n_tri - 64 * w >= 64) ? ~0ull : ((1ull << (h.n_tri - 64 * w)) - 1ull);
    if (s < 0 || s >= h.n_surf) return;
    const float4 R0 = h.tri[(size_t)s * 4], R1 = h.tri[(size_t)s * 4 + 1], R2 = h.tri[(size_t)s * 4 + 2],
                 R3 = h.tri[(size_t)s * 4 + 3];
    const float bx = o[0] - R0.x, by = o[1] - R0.y, bz = o[2] - R0.z;
    const float w = (bx * R3.x + by * R3.y) + bz * R3.z;
    const float pu = ((bx * R1.x + by * R1.y) + bz * R1.z) * R0.w;
    const float pv = ((bx * R2.x + by * R2.y) + bz * R2.z) * R0.w;
    int32_t nu, nv, base;
    memcpy(&nu, &R1.w, 4);
    memcpy(&nv, &R2.w, 4);
    memcpy(&base, &R3.w, 4);
    if (!(fabsf(w) <= h.h_run) || !(pu >= 0.0f) || !(pu < (float)nu) || !(pv >= 0.0f) || !(pv < (float)nv)) return;
    const float len2 = fmaf(d[0], d[0], fmaf(d[1], d[1], d[2] * d[2]));
    if (!(len2 >= 1.0f - 0x1p-20f) || !(len2 <= 1.0f + 0x1p-20f)) return;
    const float cn = (d[0] * R3.x + d[1] * R3.y) + d[2] * R3.z;
    if (!(cn >= -kCtabHemi)) return;
    const float ax = fabsf(d[0]), ay = fabsf(d[1]), az = fabsf(d[2]);
    const int m = (ax >= ay && ax >= az) ? 0 : (ay >= az ? 1 : 2);
    const float dm = d[m];
    const int f = 2 * m + (dm < 0.0f ? 1 : 0);
    const float r = 1.0f / fabsf(dm);  // (the kernel: v_rcp_f32, within 1 ulp of this)
    const float u1 = d[(m + 1) % 3] * r + 1.0f, v1 = d[(m + 2) % 3] * r + 1.0f;
    auto bin = [](float x1, int nb) { return std::min(nb - 1, std::max(0, (int)(x1 * (0.5f * (float)nb)))); };
    const int patch = base + (int)pu * nv + (int)pv;
    const bool cp = fabsf(cn) < h.cop_th;
    const uint64_t* mm = &h.masks[((size_t)patch * 6 * kNc * kNc + (size_t)(f * kNc + bin(u1, kNc)) * kNc + bin(v1, kNc)) * W];
    const uint64_t* gg = &h.gdict[(size_t)h.gid[(size_t)(f * kNg + bin(u1, kNg)) * kNg + bin(v1, kNg)] * W];
    if (h.gflag) {  // the grazing fold: the bin's grazing mask is in the entry unless flagged
        const bool look = (mm[W - 1] & kCtabGflagBit) != 0;
        for (int k = 0; k < W; ++k)
            out[k] = (mm[k] & (k == W - 1 ? ~kCtabGflagBit : ~0ull)) | (look ? gg[k] : 0ull) |
                     (cp ? h.cop[(size_t)s * W + k] : 0ull);
        return;
    }
    for (int k = 0; k < W; ++k) out[k] = mm[k] | gg[k] | (cp ? h.cop[(size_t)s * W + k] : 0ull);
}

}  // namespace rt
