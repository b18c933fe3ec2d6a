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
//    pass with t within the window lambda_win needs |T| <= lambda_win (K EW + eA) + ET,
//    i.e. the origin within r = (lambda_max (K EW + eA) + ET) / |N| of the triangle's
//    plane.  Per origin region (the surface triangle a bounce ray starts from, grown by
//    the bounce offset; the camera, per launch) the list of triangles whose plane passes
//    that close is precomputed; the kernel tests |d.N| against K EW + slack for each and
//    runs the exact test on those that qualify.  An origin outside its region, or a ray
//    whose window exceeds lambda_max, scans every triangle's |d.N| instead.
// K = 8.  Everything is computed in double and rounded outward to float.
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "rt_internal.hpp"

namespace rt {

namespace {

constexpr double kU = 1.0 / 16777216.0;   // 2^-24
constexpr double kC = 1.0 / 524288.0;     // 2^-19: 2x the 16u of both evaluations
constexpr double kK = kBvhK;
constexpr int kLeafMax = 4;
constexpr int kBins = 16;

float down(double x) {
    float f = (float)x;
    return ((double)f <= x) ? f : nextafterf(f, -INFINITY);
}
float up(double x) {
    float f = (float)x;
    return ((double)f >= x) ? f : nextafterf(f, INFINITY);
}

struct TriInfo {
    double lo[3], hi[3];  // padded box
    double c[3];          // centroid of the padded box
    double N[3], w0, nlen;
    double M, n1, n2;     // build_filter's sums
    double vmax;
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

// error bounds of one triangle for origins within B (build_filter's structure)
struct Bounds {
    double eA, EW, ET;
};
Bounds bounds_for(const TriInfo& t, double B) {
    const double dinf = (double)kMfDirBound;
    const double F = ldexp(1.0, -90);
    Bounds b;
    b.eA = kC * dinf * t.M + F;
    b.EW = 2.0 * (kC * 2.0 * dinf * B * t.n2 + kC * 2.0 * dinf * B * t.n1 + b.eA) + F;
    b.ET = kC * (B + t.vmax) * t.M + 2.0 * 1e-5 * (double)kFiltMaxTScale * b.eA + F;
    return b;
}

// threshold of the kernel's |d.N~| test (N~ the float normal): K EW + eA + evaluation slack
float graze_threshold(const TriInfo& t, const Bounds& b) {
    return up((kK * b.EW + b.eA + 8.0 * kU * (double)kMfDirBound * t.M) * (1.0 + 1e-9));
}

// the plane's distance to box [lo, hi] (0 if it cuts the box), in world units
double plane_box_dist(const TriInfo& t, const double* lo, const double* hi) {
    double c = 0.0, r = 0.0;
    for (int i = 0; i < 3; ++i) {
        const double m = 0.5 * (lo[i] + hi[i]), h = 0.5 * (hi[i] - lo[i]);
        c += t.N[i] * m;
        r += fabs(t.N[i]) * h;
    }
    return std::max(0.0, fabs(c - t.w0) - r) / t.nlen;
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
// `vmax` bounds the scene's coordinates; surface-region origins are within vmax + the
// bounce offset.  Returns false if the scene is out of the filter's ranges.
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
    const double lam_max = 2.0 * sqrt(3.0) * B_s * 1.01 + 1e-3;
    const double mu = ldexp(1.0, -18) * (obound + lam_max);  // slab-test rounding (>= 4u |coords|)
    for (int i = 0; i < n; ++i) {
        const float4 P0 = isect[(size_t)i * 3], P1 = isect[(size_t)i * 3 + 1], P2 = isect[(size_t)i * 3 + 2];
        const double v0[3] = {P0.x, P0.y, P0.z}, a[3] = {P1.x, P1.y, P1.z}, b[3] = {P2.x, P2.y, P2.z};
        TriInfo& t = ti[(size_t)i];
        t.M = t.n1 = t.n2 = t.vmax = 0.0;
        for (int k = 0; k < 3; ++k) {
            const int j = (k + 1) % 3, l = (k + 2) % 3;
            t.N[k] = a[j] * b[l] - a[l] * b[j];
            t.M += fabs(a[j] * b[l]) + fabs(a[l] * b[j]);
            t.n1 += fabs(a[k]);
            t.n2 += fabs(b[k]);
            t.vmax = std::max(t.vmax, fabs(v0[k]));
            const double x0 = v0[k], x1 = v0[k] + a[k], x2 = v0[k] + b[k];
            const double lo = std::min(x0, std::min(x1, x2)), hi = std::max(x0, std::max(x1, x2));
            const double pad = 2.0 / kK * (hi - lo) + mu;
            t.lo[k] = lo - pad;
            t.hi[k] = hi + pad;
            t.c[k] = 0.5 * (t.lo[k] + t.hi[k]);
        }
        t.w0 = v0[0] * t.N[0] + v0[1] * t.N[1] + v0[2] * t.N[2];
        t.nlen = sqrt(t.N[0] * t.N[0] + t.N[1] * t.N[1] + t.N[2] * t.N[2]);
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
    // grazing data: the normal as a float, the threshold for surface origins (within B_s)
    // and, apart, the one for any origin within obound (the full scan)
    h.graze.resize((size_t)n);
    h.graze_full.resize((size_t)n);
    for (int i = 0; i < n; ++i) {
        const TriInfo& t = ti[(size_t)i];
        float4 g;
        g.x = (float)t.N[0]; g.y = (float)t.N[1]; g.z = (float)t.N[2];
        g.w = graze_threshold(t, bounds_for(t, B_s));
        h.graze[(size_t)i] = g;
        h.graze_full[(size_t)i] = graze_threshold(t, bounds_for(t, obound));
    }
    // origin regions: each triangle's box grown by the padding, the offset of the
    // bounce origin (1e-5 x |sd| <= 1.02e-5) and the error of the hit position
    // (a + b lambda_max along the ray, plus rounding).  A triangle i can be grazed from a
    // region within window lambda only if its plane passes within p_i + q_i lambda of it
    // (p = ET / |N|, q = (K EW + eA) / |N|), i.e. from lambda_crit = (dist - p) / q on.
    // Each region lists its triangles by lambda_crit up to kBvhListMax entries (all with
    // lambda_crit <= lambda_max if fewer); the last listed lambda_crit bound, `lam_k`,
    // is stored with the region: a ray whose window exceeds it scans every triangle.
    h.region.resize((size_t)n * 2);
    h.gstart.assign((size_t)n + 1, 0);
    h.glist.clear();
    std::vector<double> p_s((size_t)n), q_s((size_t)n);
    for (int i = 0; i < n; ++i) {
        const TriInfo& t = ti[(size_t)i];
        const Bounds bs = bounds_for(t, B_s);
        p_s[(size_t)i] = bs.ET / t.nlen * (1.0 + 1e-6) + ldexp(1.0, -40);
        q_s[(size_t)i] = (kK * bs.EW + bs.eA) / t.nlen * (1.0 + 1e-6);
    }
    std::vector<std::pair<double, int>> cand;
    for (int k = 0; k < n; ++k) {
        const TriInfo& t = ti[(size_t)k];
        double lo[3], hi[3];
        // the hit position on triangle k is off the exact crossing by a_k + b_k lambda
        const Bounds bk = bounds_for(t, obound);
        const double den = kK * bk.EW - bk.eA;
        const double g = 1.02e-5 + bk.ET / den + (bk.eA / den + 4.0 * kU) * lam_max + mu;
        for (int a = 0; a < 3; ++a) {  // within the box the B_s thresholds hold for
            lo[a] = std::max(t.lo[a] - g, -B_s);
            hi[a] = std::min(t.hi[a] + g, B_s);
        }
        cand.clear();
        for (int i = 0; i < n; ++i) {
            const double dist = plane_box_dist(ti[(size_t)i], lo, hi);
            const double lc = std::max(0.0, (dist - p_s[(size_t)i]) / q_s[(size_t)i]);
            if (lc <= lam_max) cand.emplace_back(lc, i);
        }
        std::sort(cand.begin(), cand.end());
        double lam_k = lam_max;
        if ((int)cand.size() > kBvhListMax) {
            lam_k = cand[(size_t)kBvhListMax].first;  // complete below the first one left out
            cand.resize((size_t)kBvhListMax);
        }
        float4 L, H;
        L.x = down(lo[0]); L.y = down(lo[1]); L.z = down(lo[2]); L.w = down(lam_k);
        H.x = up(hi[0]); H.y = up(hi[1]); H.z = up(hi[2]); H.w = 0.0f;
        h.region[(size_t)k * 2] = L;
        h.region[(size_t)k * 2 + 1] = H;
        for (const auto& c : cand) {
            int2 e;
            e.x = c.second;
            const float lcf = down(c.first);
            memcpy(&e.y, &lcf, 4);
            h.glist.push_back(e);
        }
        // each list starts 16-B aligned and is readable 4 entries past its end (the
        // kernel's 4-wide steps): pad with entries that end any walk
        const int2 stop = {0, 0x7f800000};  // lambda_crit = +inf
        while (h.glist.size() % 2 != 0) h.glist.push_back(stop);
        h.gstart[(size_t)k + 1] = (int32_t)h.glist.size();
    }
    for (int k = 0; k < 4; ++k) h.glist.push_back({0, 0x7f800000});
    // Normal-space index of the full grazing test (rays with no usable list: escaping
    // rays, unknown regions).  Triangle i qualifies when |d.N~_i| <= thr_i(B) = alpha_i B
    // + beta_i (B >= the ray's max |o_j|: K EW is affine in B), i.e. only if its unit
    // normal lies in the band |d.n| <= s_i(B) = (thr_i(B) + 4u dinf M) / |N| around the
    // great circle normal to d.  A BVH over the normals (folded to one hemisphere, the
    // test being symmetric) with per-node maxima of alpha / |N| and beta' / |N| turns the
    // scan of every triangle into a slab query.
    {
        const double dinf = (double)kMfDirBound;
        std::vector<double> al((size_t)n), be((size_t)n), pt((size_t)n * 3);
        h.gcoef.resize((size_t)n);
        for (int i = 0; i < n; ++i) {
            const TriInfo& t = ti[(size_t)i];
            const Bounds b0 = bounds_for(t, 0.0);
            // EW(B) = 2 (4 c dinf B (n1 + n2) / 2 ... ) : build_filter's form, affine in B
            const double a = kK * 2.0 * (kC * 2.0 * dinf * (t.n1 + t.n2)) * (1.0 + 1e-9);
            const double b = (kK * b0.EW + b0.eA + 8.0 * kU * dinf * t.M) * (1.0 + 1e-9);
            float2 g;
            g.x = up(a);
            g.y = up(b);
            h.gcoef[(size_t)i] = g;
            al[(size_t)i] = (double)g.x / t.nlen * (1.0 + 1e-6);
            be[(size_t)i] = ((double)g.y + 8.0 * kU * dinf * t.M) / t.nlen * (1.0 + 1e-6) + 1e-6;
            double nn3[3] = {t.N[0] / t.nlen, t.N[1] / t.nlen, t.N[2] / t.nlen};
            const bool flip = nn3[2] < 0.0 || (nn3[2] == 0.0 && (nn3[1] < 0.0 || (nn3[1] == 0.0 && nn3[0] < 0.0)));
            for (int a3 = 0; a3 < 3; ++a3) pt[(size_t)i * 3 + a3] = flip ? -nn3[a3] : nn3[a3];
        }
        std::vector<int> id((size_t)n);
        for (int i = 0; i < n; ++i) id[(size_t)i] = i;
        h.nnodes.clear();
        h.nleaf.clear();
        // iterative median build: node record {c, alpha'}, {h, link|count, beta'} as 3 float4
        struct Job { int node, b, e; };
        std::vector<Job> jobs;
        auto alloc = [&]() {
            h.nnodes.resize(h.nnodes.size() + 3);
            return (int)(h.nnodes.size() / 3) - 1;
        };
        jobs.push_back({alloc(), 0, n});
        int nd = 0;
        while (!jobs.empty()) {
            const Job j = jobs.back();
            jobs.pop_back();
            double lo[3] = {DBL_MAX, DBL_MAX, DBL_MAX}, hi[3] = {-DBL_MAX, -DBL_MAX, -DBL_MAX}, am = 0.0, bm = 0.0;
            for (int k = j.b; k < j.e; ++k) {
                const int i = id[(size_t)k];
                for (int a3 = 0; a3 < 3; ++a3) {
                    lo[a3] = std::min(lo[a3], pt[(size_t)i * 3 + a3]);
                    hi[a3] = std::max(hi[a3], pt[(size_t)i * 3 + a3]);
                }
                am = std::max(am, al[(size_t)i]);
                bm = std::max(bm, be[(size_t)i]);
            }
            float4 r0, r1, r2;
            r0.x = (float)(0.5 * (lo[0] + hi[0])); r0.y = (float)(0.5 * (lo[1] + hi[1]));
            r0.z = (float)(0.5 * (lo[2] + hi[2])); r0.w = up(am);
            // half extents from the float centre, rounded up, + slack for the float test
            r1.x = up(std::max(hi[0] - r0.x, r0.x - lo[0]) + 1e-6);
            r1.y = up(std::max(hi[1] - r0.y, r0.y - lo[1]) + 1e-6);
            r1.z = up(std::max(hi[2] - r0.z, r0.z - lo[2]) + 1e-6);
            r2.x = 0.0f; r2.y = 0.0f; r2.z = up(bm);
            const int cnt = j.e - j.b;
            int link, cw;
            if (cnt <= 4) {
                link = (int)h.nleaf.size();
                for (int k = j.b; k < j.e; ++k) h.nleaf.push_back(id[(size_t)k]);
                cw = cnt;
            } else {
                int ax = 0;
                for (int a3 = 1; a3 < 3; ++a3)
                    if (hi[a3] - lo[a3] > hi[ax] - lo[ax]) ax = a3;
                const int mid = j.b + cnt / 2;
                std::nth_element(id.begin() + j.b, id.begin() + mid, id.begin() + j.e,
                                 [&](int x, int y) { return pt[(size_t)x * 3 + ax] < pt[(size_t)y * 3 + ax]; });
                link = alloc();
                alloc();
                jobs.push_back({link + 1, mid, j.e});
                jobs.push_back({link, j.b, mid});
                cw = 0;
            }
            memcpy(&r1.w, &link, 4);
            memcpy(&r2.w, &cw, 4);
            h.nnodes[(size_t)j.node * 3] = r0;
            h.nnodes[(size_t)j.node * 3 + 1] = r1;
            h.nnodes[(size_t)j.node * 3 + 2] = r2;
            ++nd;
        }
        // depth of a median tree over n points: ceil(log2(n / 4)) + 1 < kBvhMaxDepth
        if ((int)(h.nnodes.size() / 3) > 0 && n > (1 << (kBvhMaxDepth - 2)) * 4) return false;
    }
    h.n_nodes = (int)nn;
    h.depth = bld.depth;
    h.sig_a = up(sa * (1.0 + 1e-6));
    h.sig_b = up(sb * (1.0 + 1e-6));
    h.lam_max = down(lam_max);
    h.B_s = B_s;
    h.obound = obound;
    h.ti_cache.resize((size_t)n * 8);
    for (int i = 0; i < n; ++i) {
        const TriInfo& t = ti[(size_t)i];
        double* c = &h.ti_cache[(size_t)i * 8];
        c[0] = t.N[0]; c[1] = t.N[1]; c[2] = t.N[2]; c[3] = t.w0; c[4] = t.nlen;
        c[5] = t.M; c[6] = t.n1 + t.n2; c[7] = t.vmax;
    }
    return true;
}

// The grazing list of rays from a camera at (cx, cy, cz) (lambda_max: the camera's
// distance to the far corner of the scene box, x 2).
float bvh_camera_list(const BvhHost& h, int n, float cx, float cy, float cz, std::vector<int4>* out) {
    out->clear();
    const double cam[3] = {cx, cy, cz};
    const double vm = h.B_s;
    double lam = 0.0;
    for (int k = 0; k < 8; ++k) {
        const double p[3] = {(k & 1) ? vm : -vm, (k & 2) ? vm : -vm, (k & 4) ? vm : -vm};
        lam = std::max(lam, sqrt((p[0] - cam[0]) * (p[0] - cam[0]) + (p[1] - cam[1]) * (p[1] - cam[1]) +
                                 (p[2] - cam[2]) * (p[2] - cam[2])));
    }
    lam = 1.01 * lam + 1e-3;
    const double B = std::max(h.B_s, std::max(fabs(cam[0]), std::max(fabs(cam[1]), fabs(cam[2])))) + 1e-6;
    std::vector<std::pair<double, int>> cand;
    std::vector<float> thr((size_t)n);
    for (int i = 0; i < n; ++i) {
        const double* c = &h.ti_cache[(size_t)i * 8];
        TriInfo t;
        t.N[0] = c[0]; t.N[1] = c[1]; t.N[2] = c[2]; t.w0 = c[3]; t.nlen = c[4];
        t.M = c[5]; t.n1 = c[6]; t.n2 = 0.0; t.vmax = c[7];
        const Bounds b = bounds_for(t, B);
        const double p = b.ET / t.nlen * (1.0 + 1e-6) + ldexp(1.0, -40);
        const double q = (kK * b.EW + b.eA) / t.nlen * (1.0 + 1e-6);
        const double d = fabs(t.N[0] * cam[0] + t.N[1] * cam[1] + t.N[2] * cam[2] - t.w0) / t.nlen;
        const double lc = std::max(0.0, (d - p) / q);
        if (lc <= lam) cand.emplace_back(lc, i);
        thr[(size_t)i] = graze_threshold(t, b);
    }
    std::sort(cand.begin(), cand.end());
    if ((int)cand.size() > kBvhListMax) {
        lam = cand[(size_t)kBvhListMax].first;
        cand.resize((size_t)kBvhListMax);
    }
    for (const auto& c : cand) {
        int4 e;
        e.x = c.second;
        memcpy(&e.y, &thr[(size_t)c.second], 4);
        const float lcf = down(c.first);
        memcpy(&e.z, &lcf, 4);
        e.w = 0;
        out->push_back(e);
    }
    return down(lam);
}

// Invariants of a host build (rt_bvh_check, CPU tests): every triangle in exactly one
// leaf; each node's box holds its children's / its triangles' (vertices + padding);
// each region's box holds its triangle, its list is sorted by lambda_crit and lists the
// triangle itself at 0.  Returns an empty string or the first violation.
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
    // the normal-space index: every triangle in one leaf, its unit normal in the box
    std::fill(seen.begin(), seen.end(), 0);
    const int nn = (int)(h.nnodes.size() / 3);
    for (int k = 0; k < nn; ++k) {
        const float4 r0 = h.nnodes[(size_t)k * 3], r1 = h.nnodes[(size_t)k * 3 + 1], r2 = h.nnodes[(size_t)k * 3 + 2];
        int link, cnt;
        memcpy(&link, &r1.w, 4);
        memcpy(&cnt, &r2.w, 4);
        for (int j = link; cnt > 0 && j < link + cnt; ++j) {
            const int i = h.nleaf[(size_t)j];
            if (i < 0 || i >= n) return "normal leaf index out of range";
            ++seen[(size_t)i];
            const float4 E1 = isect[(size_t)i * 3 + 1], E2 = isect[(size_t)i * 3 + 2];
            double N[3] = {(double)E1.y * E2.z - (double)E1.z * E2.y, (double)E1.z * E2.x - (double)E1.x * E2.z,
                           (double)E1.x * E2.y - (double)E1.y * E2.x};
            const double l = sqrt(N[0] * N[0] + N[1] * N[1] + N[2] * N[2]);
            const double c[3] = {r0.x, r0.y, r0.z}, hh[3] = {r1.x, r1.y, r1.z};
            bool in_p = true, in_m = true;
            for (int a = 0; a < 3; ++a) {
                in_p = in_p && fabs(N[a] / l - c[a]) <= hh[a];
                in_m = in_m && fabs(-N[a] / l - c[a]) <= hh[a];
            }
            if (!(in_p || in_m)) {
                snprintf(buf, sizeof buf, "normal of triangle %d outside its leaf %d", i, k);
                return buf;
            }
        }
    }
    for (int i = 0; i < n; ++i)
        if (seen[(size_t)i] != 1) {
            snprintf(buf, sizeof buf, "triangle %d in %d normal leaves", i, seen[(size_t)i]);
            return buf;
        }
    for (int k = 0; k < n; ++k) {
        const float4 L = h.region[(size_t)k * 2], H = h.region[(size_t)k * 2 + 1];
        const float4 P0 = isect[(size_t)k * 3];
        if (!(L.x <= P0.x && P0.x <= H.x && L.y <= P0.y && P0.y <= H.y && L.z <= P0.z && P0.z <= H.z)) {
            snprintf(buf, sizeof buf, "region %d misses its triangle", k);
            return buf;
        }
        float prev = -1.0f;
        bool self = false;
        for (int j = h.gstart[(size_t)k]; j < h.gstart[(size_t)k + 1]; ++j) {
            float lc;
            memcpy(&lc, &h.glist[(size_t)j].y, 4);
            if (lc < prev) return "grazing list not sorted";
            prev = lc;
            if (h.glist[(size_t)j].x == k && lc == 0.0f) self = true;
        }
        if (!self) {
            snprintf(buf, sizeof buf, "region %d does not list its own triangle", k);
            return buf;
        }
    }
    return std::string();
}

}  // namespace rt
