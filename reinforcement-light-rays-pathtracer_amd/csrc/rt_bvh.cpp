// rt_bvh.cpp — host build of the exact BVH path for large triangle soups
// (Models/bunny.obj, Medieval_House.obj; the reference scans
// every triangle, Ray::closest_intersection CPU/rays/ray.cpp:14-28, GPU/rays/ray.cu:16-141).
//
// The device traversal (rt_trace.hpp, closest_hit_bvh) must return the brute-force
// scan's hit bit for bit, so every box test is a proof that the exact float test of the
// triangles inside fails.  With the real values of the filter quantities of a (ray,
// triangle) pair (build_filter, rt_capi.cpp: A = d.N, U, V, W = A - U - V, T = w0 - o.N,
// lambda = T / A the ray parameter of the plane crossing X):
//   exact test passes  =>  s U >= -EW, s V >= -EW, s W >= -EW, s T >= -ET  (s = sign A)
// with EW, ET bounds on the two evaluations' rounding (here at 16u scale x 4, c = 2^-18,
// for unit directions and origins within `B`).  Two cases:
//  * regular, |A| >= K EW: the barycentrics of X are >= -1/K, so X lies in the triangle
//    grown by 2/K of its extent per axis (the padded box), and the Cramer t of the test
//    satisfies |t ts - lambda| <= a + b |lambda| (a = ET / (K EW - eA), b = eA / (...));
//    a ray whose slab interval misses the padded box (or enters it beyond the t window)
//    cannot pass the exact test of any triangle inside;
//  * grazing, |A| < K EW: X can be anywhere (the ray runs nearly in the plane), but a
//    pass with t within the window lambda needs |T| <= lambda (K EW + eA) + ET, i.e. the
//    origin within p + s lambda of the triangle's plane, and |d.N| <= K EW + slack, i.e.
//    the unit normal within s of the great circle normal to d.  A second BVH, over the
//    planes (n, w) of the triangles, finds every triangle meeting both conditions for the
//    window the first traversal left (only the second for a ray that hit nothing); the
//    kernel runs the exact test on those.
// K = 4.  Everything is computed in double and rounded outward to float.
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "rt_bounds.hpp"
#include "rt_internal.hpp"

namespace rt {

namespace {

using bnd::Bounds;
using bnd::bounds_for;
using bnd::down;
using bnd::kC;
using bnd::kU;
using bnd::up;
constexpr double kK = kBvhK;
constexpr int kLeafMax = 4;
constexpr int kBins = 16;

// build_filter's sums (bnd::TriAlg) and the padded box of one triangle
struct TriInfo : bnd::TriAlg {
    double lo[3], hi[3];  // padded box
    double c[3];          // centroid of the padded box
};

struct Box {
    double lo[3] = {DBL_MAX, DBL_MAX, DBL_MAX}, hi[3] = {-DBL_MAX, -DBL_MAX, -DBL_MAX};
    void grow(const double* l, const double* h) {
        for (int i = 0; i < 3; ++i) {
            lo[i] = std::min(lo[i], l[i]);
            hi[i] = std::max(hi[i], h[i]);
        }
    }
    double area() const {
        if (lo[0] > hi[0]) return 0.0;
        const double x = hi[0] - lo[0], y = hi[1] - lo[1], z = hi[2] - lo[2];
        return 2.0 * (x * y + y * z + z * x);
    }
};

// threshold of the kernel's |d.N~| test (N~ the float normal): K EW + eA + evaluation slack
float graze_threshold(const TriInfo& t, const Bounds& b) {
    return up((kK * b.EW + b.eA + 8.0 * kU * (double)kMfDirBound * t.M) * (1.0 + 1e-9));
}

struct Builder {
    const std::vector<TriInfo>& ti;
    std::vector<int> idx;
    std::vector<Box> nodes;
    std::vector<int> left, first, count;
    int depth = 0;

    explicit Builder(const std::vector<TriInfo>& t) : ti(t) {}

    int make_node() {
        nodes.emplace_back();
        left.push_back(0);
        first.push_back(0);
        count.push_back(0);
        return (int)nodes.size() - 1;
    }

    // node covering idx[b, e); children allocated as a pair
    void build(int node, int b, int e, int level) {
        depth = std::max(depth, level);
        Box box, cbox;
        for (int k = b; k < e; ++k) {
            const TriInfo& t = ti[idx[k]];
            box.grow(t.lo, t.hi);
            cbox.grow(t.c, t.c);
        }
        nodes[node] = box;
        const int n = e - b;
        if (n <= kLeafMax || level >= kBvhMaxDepth - 1) {
            first[node] = b;
            count[node] = n;
            return;
        }
        // binned SAH over the padded-box centroids
        double best = DBL_MAX;
        int best_axis = -1, best_split = 0;
        for (int ax = 0; ax < 3; ++ax) {
            const double lo = cbox.lo[ax], hi = cbox.hi[ax];
            if (!(hi > lo)) continue;
            Box bb[kBins];
            int bc[kBins] = {0};
            const double sc = kBins / (hi - lo);
            for (int k = b; k < e; ++k) {
                const TriInfo& t = ti[idx[k]];
                int j = (int)((t.c[ax] - lo) * sc);
                j = std::min(kBins - 1, std::max(0, j));
                bb[j].grow(t.lo, t.hi);
                ++bc[j];
            }
            Box lb[kBins], rb[kBins];
            int lc[kBins], rc[kBins];
            Box acc;
            int cnt = 0;
            for (int j = 0; j < kBins; ++j) {
                if (bc[j]) acc.grow(bb[j].lo, bb[j].hi);
                cnt += bc[j];
                lb[j] = acc;
                lc[j] = cnt;
            }
            acc = Box();
            cnt = 0;
            for (int j = kBins - 1; j >= 0; --j) {
                if (bc[j]) acc.grow(bb[j].lo, bb[j].hi);
                cnt += bc[j];
                rb[j] = acc;
                rc[j] = cnt;
            }
            for (int j = 0; j < kBins - 1; ++j) {
                if (lc[j] == 0 || rc[j + 1] == 0) continue;
                const double cost = lb[j].area() * lc[j] + rb[j + 1].area() * rc[j + 1];
                if (cost < best) {
                    best = cost;
                    best_axis = ax;
                    best_split = j;
                }
            }
        }
        int mid;
        if (best_axis < 0) {  // coincident centroids: split the list in half
            mid = b + n / 2;
        } else {
            const double lo = cbox.lo[best_axis], sc = kBins / (cbox.hi[best_axis] - lo);
            auto part = std::partition(idx.begin() + b, idx.begin() + e, [&](int i) {
                int j = (int)((ti[i].c[best_axis] - lo) * sc);
                j = std::min(kBins - 1, std::max(0, j));
                return j <= best_split;
            });
            mid = (int)(part - idx.begin());
            if (mid == b || mid == e) mid = b + n / 2;
        }
        const int l = make_node();
        make_node();
        left[node] = l;
        count[node] = 0;
        build(l, b, mid, level + 1);
        build(l + 1, mid, e, level + 1);
    }
};

}  // namespace

// Builds the BVH path of a scene (isect: the kIsectF4 records of its n triangles).
// Returns false if the scene is out of the filter's ranges.
bool bvh_build(const float4* isect, int n, BvhHost* out) {
    if (n <= 0) return false;
    std::vector<TriInfo> ti((size_t)n);
    double vmax_scene = 0.0;
    for (int i = 0; i < n; ++i) {
        const float4 P0 = isect[(size_t)i * 3], P1 = isect[(size_t)i * 3 + 1], P2 = isect[(size_t)i * 3 + 2];
        const double v0[3] = {P0.x, P0.y, P0.z}, a[3] = {P1.x, P1.y, P1.z}, b[3] = {P2.x, P2.y, P2.z};
        for (int k = 0; k < 3; ++k) {
            // the vertices as the reference's records give them: v0, v0 + e1, v0 + e2
            vmax_scene = std::max(vmax_scene, std::max(fabs(v0[k]), std::max(fabs(v0[k] + a[k]), fabs(v0[k] + b[k]))));
        }
    }
    // origins of bounce rays: surface points + the 1e-5 offset, plus slack
    const double B_s = vmax_scene * (1.0 + ldexp(1.0, -10)) + ldexp(1.0, -10);
    const double obound = std::max(8.0, 2.0 * vmax_scene + 1.0);  // filter_origin_bound
    // a hit point lies in the scene's box and a surface origin near it: the window of a
    // ray that hit something is below the box diagonal (x 2 for slack)
    // the ray parameter of a point of the scene seen from any origin within obound
    const double lam_max = 2.0 * sqrt(3.0) * obound;
    const double mu = ldexp(1.0, -18) * (obound + lam_max);  // slab-test rounding (>= 4u |coords|)
    for (int i = 0; i < n; ++i) {
        const float4 P0 = isect[(size_t)i * 3], P1 = isect[(size_t)i * 3 + 1], P2 = isect[(size_t)i * 3 + 2];
        const double v0[3] = {P0.x, P0.y, P0.z}, a[3] = {P1.x, P1.y, P1.z}, b[3] = {P2.x, P2.y, P2.z};
        TriInfo& t = ti[(size_t)i];
        static_cast<bnd::TriAlg&>(t) = bnd::tri_alg(P0, P1, P2);
        for (int k = 0; k < 3; ++k) {
            const double x0 = v0[k], x1 = v0[k] + a[k], x2 = v0[k] + b[k];
            const double lo = std::min(x0, std::min(x1, x2)), hi = std::max(x0, std::max(x1, x2));
            const double pad = 2.0 / kK * (hi - lo) + mu;
            t.lo[k] = lo - pad;
            t.hi[k] = hi + pad;
            t.c[k] = 0.5 * (t.lo[k] + t.hi[k]);
        }
        if (!(t.M < ldexp(1.0, 36)) || !(obound < ldexp(1.0, 20))) return false;
    }
    // t-window slack over the regular pairs, for origins within obound (camera included)
    double sa = 0.0, sb = 0.0;
    for (const TriInfo& t : ti) {
        const Bounds bo = bounds_for(t, obound);
        const double den = kK * bo.EW - bo.eA;
        sa = std::max(sa, bo.ET / den);
        sb = std::max(sb, bo.eA / den + 4.0 * kU);
    }
    if (!(sb < 0.25)) return false;

    Builder bld(ti);
    bld.idx.resize((size_t)n);
    for (int i = 0; i < n; ++i) bld.idx[(size_t)i] = i;
    bld.make_node();
    bld.build(0, 0, n, 0);

    BvhHost& h = *out;
    h = BvhHost();
    const size_t nn = bld.nodes.size();
    h.nodes.resize(nn * 2);
    for (size_t k = 0; k < nn; ++k) {
        const Box& bx = bld.nodes[k];
        const int32_t link = bld.count[k] > 0 ? bld.first[k] : bld.left[k];
        float4 lo, hi;
        lo.x = down(bx.lo[0]); lo.y = down(bx.lo[1]); lo.z = down(bx.lo[2]);
        hi.x = up(bx.hi[0]); hi.y = up(bx.hi[1]); hi.z = up(bx.hi[2]);
        memcpy(&lo.w, &link, 4);
        const int32_t cnt = bld.count[k];
        memcpy(&hi.w, &cnt, 4);
        h.nodes[k * 2] = lo;
        h.nodes[k * 2 + 1] = hi;
    }
    h.tris.resize((size_t)n * 3);
    for (int k = 0; k < n; ++k) {
        const int i = bld.idx[(size_t)k];
        h.tris[(size_t)k * 3 + 0] = isect[(size_t)i * 3 + 0];
        h.tris[(size_t)k * 3 + 1] = isect[(size_t)i * 3 + 1];
        h.tris[(size_t)k * 3 + 2] = isect[(size_t)i * 3 + 2];
        memcpy(&h.tris[(size_t)k * 3 + 1].w, &i, 4);  // original index (the record's w is 0)
    }
    // grazing data: the normal as a float (w: the threshold for origins within the scene
    // box, informational; the kernel uses grec)
    h.graze.resize((size_t)n);
    for (int i = 0; i < n; ++i) {
        const TriInfo& t = ti[(size_t)i];
        float4 g;
        g.x = (float)t.N[0]; g.y = (float)t.N[1]; g.z = (float)t.N[2];
        g.w = graze_threshold(t, bounds_for(t, B_s));
        h.graze[(size_t)i] = g;
    }
    // Direction-binned index of the grazing pairs.  Triangle i can pass the exact test
    // outside its padded box only when (1) |d.N~_i| <= thr_i(B) = alpha_i B + beta_i
    // (B >= the ray's max |o_j|; K EW is affine in B): its unit normal n within
    // s_i(B) = (thr_i(B) + 4u dinf M) / |N| of the great circle normal to d; and (2) for a
    // pass with t below the window lambda, |T| <= lambda (K EW + eA) + ET: in N units
    // |N~.o - W| <= (PA B + PB) + thr_i(B) lambda (W = N.v0, PA/PB: ET affine in B plus
    // the float evaluation's rounding).  The directions are cut into the cells of a cube
    // map (6 x G x G); cell c lists every triangle with |d_c.n| <= s_i(B_L) + chord_c
    // (d_c the cell's centre direction, chord_c >= |d - d_c| over the cell: its image is a
    // spherical quad bounded by great-circle arcs, farthest from d_c at a corner).  Two
    // list sets: B_L = the scene box (bounce rays) and B_L = obound (camera rays).  The
    // kernel walks the ray's cell list and applies (1) and (2) exactly per triangle.
    {
        const double dinf = (double)kMfDirBound;
        h.grec.resize((size_t)n * 2);
        std::vector<double> s_a((size_t)n), s_b((size_t)n), un((size_t)n * 3);
        for (int i = 0; i < n; ++i) {
            const TriInfo& t = ti[(size_t)i];
            const Bounds b0 = bounds_for(t, 0.0);
            const double a = kK * 2.0 * (kC * 2.0 * dinf * (t.n1 + t.n2)) * (1.0 + 1e-9);
            const double bb = (kK * b0.EW + b0.eA + 8.0 * kU * dinf * t.M) * (1.0 + 1e-9);
            const double n1 = fabs(t.N[0]) + fabs(t.N[1]) + fabs(t.N[2]);
            const float Wf = (float)t.w0;
            // ET(B) = c (B + vmax) M + 2 eps ts_max eA + F, plus the rounding of N~.o - W
            const double PA = (kC * t.M + 8.0 * kU * n1) * (1.0 + 1e-6);
            const double PB = (kC * t.vmax * t.M + 2.0 * 1e-5 * (double)kFiltMaxTScale * b0.eA + ldexp(1.0, -90) +
                               8.0 * kU * fabs((double)Wf) + fabs((double)Wf - t.w0)) * (1.0 + 1e-6) + ldexp(1.0, -100);
            float4 r0, r1;
            r0.x = h.graze[(size_t)i].x; r0.y = h.graze[(size_t)i].y; r0.z = h.graze[(size_t)i].z; r0.w = up(a);
            r1.x = up(bb); r1.y = Wf; r1.z = up(PA); r1.w = up(PB);
            h.grec[(size_t)i * 2] = r0;
            h.grec[(size_t)i * 2 + 1] = r1;
            s_a[(size_t)i] = (double)r0.w / t.nlen * (1.0 + 1e-6);
            s_b[(size_t)i] = ((double)r1.x + 8.0 * kU * dinf * t.M) / t.nlen * (1.0 + 1e-6);
            for (int k = 0; k < 3; ++k) un[(size_t)i * 3 + k] = t.N[k] / t.nlen;
        }
        const int G = kBvhDirGrid;
        const int cells = 6 * G * G;
        const double BL[2] = {B_s, obound};
        for (int set = 0; set < 2; ++set) {
            std::vector<int32_t>& start = set ? h.dstart_cam : h.dstart;
            std::vector<int32_t>& list = set ? h.dlist_cam : h.dlist;
            start.assign((size_t)cells + 1, 0);
            list.clear();
            for (int c = 0; c < cells; ++c) {
                const int f = c / (G * G), iu = (c / G) % G, iv = c % G;
                const double u0 = -1.0 + 2.0 * iu / G, u1 = -1.0 + 2.0 * (iu + 1) / G;
                const double v0 = -1.0 + 2.0 * iv / G, v1 = -1.0 + 2.0 * (iv + 1) / G;
                double dc[3];
                const double chord = bnd::cell_chord(f, u0, u1, v0, v1, dc);
                for (int i = 0; i < n; ++i) {
                    const double* nn3 = &un[(size_t)i * 3];
                    const double dn = fabs(dc[0] * nn3[0] + dc[1] * nn3[1] + dc[2] * nn3[2]);
                    // (|d| >= 1 - 2^-10 for the ray's unit-length direction: 0.2% on s)
                    if (dn <= (s_a[(size_t)i] * BL[set] + s_b[(size_t)i]) * 1.002 + chord) list.push_back(i);
                }
                start[(size_t)c + 1] = (int32_t)list.size();
            }
        }
        h.B_lists = down(B_s);
    }
    h.n_nodes = (int)nn;
    h.depth = bld.depth;
    h.sig_a = up(sa * (1.0 + 1e-6));
    h.sig_b = up(sb * (1.0 + 1e-6));
    return true;
}

// Invariants of a host build (rt_bvh_check, CPU tests): every triangle in exactly one
// leaf of each tree; each node's box holds its children's / its triangles' (vertices +
// padding); each triangle's folded plane (n, w) inside its plane-space leaf.  Returns an
// empty string or the first violation.
std::string bvh_check(const float4* isect, int n, const BvhHost& h) {
    char buf[160];
    std::vector<int> seen((size_t)n, 0);
    auto node_lo = [&](int k, int a) { return (&h.nodes[(size_t)k * 2].x)[a]; };
    auto node_hi = [&](int k, int a) { return (&h.nodes[(size_t)k * 2 + 1].x)[a]; };
    for (int k = 0; k < h.n_nodes; ++k) {
        int link, cnt;
        memcpy(&link, &h.nodes[(size_t)k * 2].w, 4);
        memcpy(&cnt, &h.nodes[(size_t)k * 2 + 1].w, 4);
        if (cnt > 0) {
            for (int j = link; j < link + cnt; ++j) {
                int i;
                memcpy(&i, &h.tris[(size_t)j * 3 + 1].w, 4);
                if (i < 0 || i >= n) return "leaf index out of range";
                ++seen[(size_t)i];
                const float4 P0 = isect[(size_t)i * 3], P1 = isect[(size_t)i * 3 + 1], P2 = isect[(size_t)i * 3 + 2];
                const double v[3][3] = {{P0.x, P0.y, P0.z},
                                        {P0.x + (double)P1.x, P0.y + (double)P1.y, P0.z + (double)P1.z},
                                        {P0.x + (double)P2.x, P0.y + (double)P2.y, P0.z + (double)P2.z}};
                for (int a = 0; a < 3; ++a)
                    for (int q = 0; q < 3; ++q)
                        if (!(node_lo(k, a) < v[q][a] && v[q][a] < node_hi(k, a))) {
                            snprintf(buf, sizeof buf, "triangle %d outside leaf %d", i, k);
                            return buf;
                        }
            }
        } else {
            if (link <= k || link + 1 >= h.n_nodes) return "bad child link";
            for (int c = link; c <= link + 1; ++c)
                for (int a = 0; a < 3; ++a)
                    if (node_lo(c, a) < node_lo(k, a) || node_hi(c, a) > node_hi(k, a)) {
                        snprintf(buf, sizeof buf, "node %d outside its parent %d", c, k);
                        return buf;
                    }
        }
    }
    for (int i = 0; i < n; ++i)
        if (seen[(size_t)i] != 1) {
            snprintf(buf, sizeof buf, "triangle %d in %d leaves", i, seen[(size_t)i]);
            return buf;
        }
    // the direction lists: sorted, in range, the start arrays monotone
    for (int set = 0; set < 2; ++set) {
        const std::vector<int32_t>& start = set ? h.dstart_cam : h.dstart;
        const std::vector<int32_t>& list = set ? h.dlist_cam : h.dlist;
        if (start.empty() || start.back() != (int32_t)list.size()) return "direction list bounds";
        for (size_t c = 0; c + 1 < start.size(); ++c) {
            if (start[c] > start[c + 1]) return "direction list starts";
            for (int32_t j = start[c]; j < start[c + 1]; ++j)
                if (list[(size_t)j] < 0 || list[(size_t)j] >= n || (j > start[c] && list[(size_t)j] <= list[(size_t)j - 1]))
                    return "direction list entries";
        }
    }
    return std::string();
}

}  // namespace rt
