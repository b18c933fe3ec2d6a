// rt_sarsa_host.cpp — C ABI of the Expected-SARSA path (BASELINE config 3):
// radiance-volume placement (RadianceMap::get_radiance_volumes_count /
// uniformly_sample_radiance_volumes, GPU/radiance_volumes/radiance_map.cu:57-84),
// the radiance volume's initial state (RadianceVolume::initialise_*,
// radiance_volume.cu:46-89), the KD tree and its array form (RadianceTree,
// radiance_tree.cu:10-246), and the frame driver (GPU/main.cu:296-350: render,
// then update_radiance_volume_distributions).
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <array>
#include <fstream>
#include <map>
#include <sstream>
#include <string>
#include <vector>

#include "../../include/rtmi.h"
#include "rt_internal.hpp"

namespace rt {
int set_error(int code, const char* msg);
int ctx_device(const rt_ctx* ctx);
const DeviceScene& scene_device(const rt_scene* s);
void scene_host(const rt_scene* s, const float** tri, const float** normals, const float** albedo,
                const float** emission, int* n_surf, int* n_light);
int ctx_blocks(rt_ctx* ctx, const int32_t* tiles, int n_tiles, int tile_size, int width, int height,
               const BlockDesc** d_blocks, int* n_blocks);
RenderLaunch render_launch(const rt_scene* scene, const rt_camera* cam, const rt_params* p);
int scene_ensure_ctab(const rt_scene* scene, int rule, float t_scale, bool wanted);
bool ctab_wanted(const rt_scene* sc, const rt_camera* cam, const rt_params* p, int user);

// read_hemisphere_locations_and_normals (GPU/utils/hemisphere_helpers.cu:230-278): one
// "x y z nx ny nz" per line, tokens split on ' ' and read with std::stof, the first
// three the location, the rest the normal
int read_locations(const char* path, std::vector<float>* loc_out, std::vector<float>* nrm_out) {
    std::ifstream in(path);
    if (!in.is_open()) return set_error(RT_E_IO, (std::string("cannot read ") + path).c_str());
    std::string line;
    try {
        while (std::getline(in, line)) {
            float loc[3] = {0.f, 0.f, 0.f}, nrm[3] = {0.f, 0.f, 0.f};
            size_t pos;
            int idx = 0;
            while ((pos = line.find(' ')) != std::string::npos) {
                const float v = std::stof(line.substr(0, pos));
                if (idx < 3) loc[idx] = v;
                else nrm[idx % 3] = v;
                ++idx;
                line.erase(0, pos + 1);
            }
            nrm[idx % 3] = std::stof(line);
            loc_out->insert(loc_out->end(), loc, loc + 3);
            nrm_out->insert(nrm_out->end(), nrm, nrm + 3);
        }
    } catch (const std::exception&) {
        return set_error(RT_E_IO, (std::string("malformed location line in ") + path).c_str());
    }
    return RT_OK;
}
}  // namespace rt

namespace {

int err(int code, const std::string& m) { return rt::set_error(code, m.c_str()); }

#define RT_HIPE(expr)                                                                          \
    do {                                                                                       \
        hipError_t e_ = (expr);                                                                \
        if (e_ != hipSuccess) return err(RT_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

constexpr float kAreaPerSample = 0.001f;  // AREA_PER_SAMPLE (radiance_volumes_settings.h:12)
constexpr float kInitialRadiance = (1.f / ((float)rt::kGridRes * (float)rt::kGridRes)) * 100.f;  // :16
constexpr uint32_t kPlacementEvent = 0xFFFF0001u;  // RNG counter word 2 of volume placement
constexpr int kMaxKdDepth = rt::kKdStack - 1;    // the traversal stack holds depth + 1 entries

// Triangle::compute_area (GPU/objects/triangle.cu:17-27): float lengths and
// cosine; 1 - pow(cos, 2) and its sqrt in double (host pow promotes).
float triangle_area(const float* v) {
    using rt::f3;
    const f3 a = rt::make3(v[3] - v[0], v[4] - v[1], v[5] - v[2]);
    const f3 b = rt::make3(v[6] - v[0], v[7] - v[1], v[8] - v[2]);
    const float e01_e02 = sqrtf(rt::dot(a, a)) * sqrtf(rt::dot(b, b));
    const float c = rt::dot(a, b) / e01_e02;
    const float s = (float)sqrt(1.0 - (double)c * (double)c);
    return 0.5f * e01_e02 * s;
}

// Material::Material / AreaLight luminance (objects/material.cu:13, lights/area_light.cu:22)
float luminance(const float* rgb) {
    const float mx = std::max(rgb[0], std::max(rgb[1], rgb[2]));
    const float mn = std::min(rgb[0], std::min(rgb[1], rgb[2]));
    return 0.5f * (mx + mn);
}

struct Tree {
    const std::vector<float>* pos;  // [n][4]
    std::vector<rt::KdNode> nodes;
    int max_depth = 0;

    struct Sub {  // one RadianceTree node before flattening
        int dim;
        float median;
        int vol = -1;  // leaf
        int left = -1, right = -1;
    };
    std::vector<Sub> subs;

    // RadianceTree::RadianceTree (radiance_tree.cu:10-60): std::sort on the split
    // dimension (the reference's comparator: position[dim] <), left = [0, median_index].
    int build(std::vector<int>& v, int dim, int depth) {
        max_depth = std::max(max_depth, depth);
        const int me = (int)subs.size();
        subs.push_back(Sub());
        subs[me].dim = dim;
        const int n = (int)v.size();
        const std::vector<float>& P = *pos;
        if (n == 1) {
            subs[me].median = P[4 * v[0] + dim];
            subs[me].vol = v[0];
            return me;
        }
        std::sort(v.begin(), v.end(), [&](int l, int r) { return P[4 * l + dim] < P[4 * r + dim]; });
        int mi;
        if (n % 2 == 0) {
            mi = n / 2 - 1;
            subs[me].median = (P[4 * v[mi] + dim] + P[4 * v[mi + 1] + dim]) / 2;
        } else {
            mi = n / 2;
            subs[me].median = P[4 * v[mi] + dim];
        }
        std::vector<int> L(v.begin(), v.begin() + mi + 1), R(v.begin() + mi + 1, v.end());
        const int nd = (dim + 1) % 3;
        const int l = build(L, nd, depth + 1);
        const int r = build(R, nd, depth + 1);
        subs[me].left = l;
        subs[me].right = r;
        return me;
    }

    // RadianceTree::convert_to_array / traverse_and_insert (radiance_tree.cu:181-246):
    // the root first, then each internal node appends its two children and
    // recurses left before right; a leaf overwrites its own slot.
    void flatten(int root, const std::vector<float>& nrm) {
        rt::KdNode r;
        memset(&r, 0, sizeof(r));
        r.dim = subs[root].dim;
        r.data = subs[root].median;
        nodes.push_back(r);
        insert(root, 0, nrm);
    }
    void insert(int s, int slot, const std::vector<float>& nrm) {
        const int last = (int)nodes.size() - 1;
        const Sub& u = subs[s];
        if (u.vol >= 0) {
            rt::KdNode& e = nodes[slot];
            memset(&e, 0, sizeof(e));
            e.dim = u.dim;
            e.leaf = 1;
            e.data = (float)u.vol;
            e.vol = u.vol;
            e.px = (*pos)[4 * u.vol];
            e.py = (*pos)[4 * u.vol + 1];
            e.pz = (*pos)[4 * u.vol + 2];
            e.nx = nrm[3 * u.vol];
            e.ny = nrm[3 * u.vol + 1];
            e.nz = nrm[3 * u.vol + 2];
            return;
        }
        nodes[slot].left = last + 1;
        nodes[slot].right = last + 2;
        rt::KdNode c;
        memset(&c, 0, sizeof(c));
        c.dim = (u.dim + 1) % 3;
        c.data = subs[u.left].median;
        nodes.push_back(c);
        c.data = subs[u.right].median;
        nodes.push_back(c);
        insert(u.left, last + 1, nrm);
        insert(u.right, last + 2, nrm);
    }
};

// Exact fast path of find_closest_radiance_volume_iterative (rt_sarsa.hip
// sarsa_nearest_grid).  The KD search visits a leaf L iff, at every ancestor whose
// split separates the query q from L, (q_k - split)^2 < MAX_DIST; the split lies
// between q_k and L_k (left subtrees hold coordinates <= the median, right ones >=),
// so a leaf whose float distance to q is below h = sqrt(MAX_DIST) * 0.999 is always
// visited.  Hence when the nearest same-normal volume is closer than h and unique in
// float distance, it is the search's result (against the initial volume 0 at the
// distance of element 0); otherwise the kernel runs the KD search itself.  Every
// leaf closer than h lies in the 3x3x3 cells around q in a grid of cell size 1.01 h
// over the volumes of q's normal class; each cell stores that whole neighbourhood
// as one contiguous candidate list (27 copies of every volume position), so a query
// reads one range.  The grid has one padding cell per side (queries are clamped
// into it; a clamped query has no volume within h and falls back).
struct NearestGrid {
    std::vector<int32_t> tri_class;  // [n_surf]
    std::vector<float4> org, nrm;    // [n_class]
    std::vector<int4> dim;           // [n_class] padded cells per axis
    std::vector<uint32_t> start;     // [cells + 1]
    std::vector<float4> leaf;        // [27 n]
    float inv_cs = 0.f, cs = 0.f, h = 0.f;
};

constexpr size_t kMaxGridCells = (size_t)1 << 26;

inline bool finite3(const float* v) { return std::isfinite(v[0]) && std::isfinite(v[1]) && std::isfinite(v[2]); }

// class key of a normal under float ==: -0 and +0 compare equal
std::array<uint32_t, 3> normal_key(const float* v) {
    std::array<uint32_t, 3> k;
    for (int c = 0; c < 3; ++c) {
        const float x = (v[c] == 0.0f) ? 0.0f : v[c];
        memcpy(&k[c], &x, 4);
    }
    return k;
}

// padded cell of coordinate p along one axis (the kernel's float operations and clamp)
inline int grid_cell(float p, float o, float inv_cs, int n) {
    return (int)floorf(fminf(fmaxf((p - o) * inv_cs, 0.0f), (float)(n - 1)));
}

bool build_nearest_grid(const std::vector<float>& pos, const std::vector<float>& nrm, int n,
                        const float* normals, int n_surf, float max_dist, NearestGrid* g) {
    g->h = sqrtf(max_dist) * 0.999f;
    const float cs = g->h * 1.01f;
    g->cs = cs;
    g->inv_cs = 1.0f / cs;
    std::map<std::array<uint32_t, 3>, int> cls;
    std::vector<int> vc(n, -1);
    for (int i = 0; i < n; ++i) {
        if (!finite3(&nrm[3 * i])) continue;  // never equal to any query normal
        auto it = cls.emplace(normal_key(&nrm[3 * i]), (int)cls.size()).first;
        vc[i] = it->second;
    }
    const int nc = (int)cls.size();
    if (nc == 0) return false;
    g->nrm.assign(nc, make_float4(0.f, 0.f, 0.f, 0.f));
    for (const auto& kv : cls) {
        float v[3];
        memcpy(v, kv.first.data(), 12);
        g->nrm[kv.second] = make_float4(v[0], v[1], v[2], 0.f);
    }
    g->tri_class.assign(n_surf, -1);
    for (int j = 0; j < n_surf; ++j) {
        if (!finite3(normals + 3 * j)) continue;
        auto it = cls.find(normal_key(normals + 3 * j));
        if (it != cls.end()) g->tri_class[j] = it->second;
    }
    std::vector<float> lo((size_t)nc * 3, INFINITY), hi((size_t)nc * 3, -INFINITY);
    for (int i = 0; i < n; ++i) {
        if (vc[i] < 0) continue;
        for (int c = 0; c < 3; ++c) {
            lo[(size_t)vc[i] * 3 + c] = std::min(lo[(size_t)vc[i] * 3 + c], pos[4 * i + c]);
            hi[(size_t)vc[i] * 3 + c] = std::max(hi[(size_t)vc[i] * 3 + c], pos[4 * i + c]);
        }
    }
    g->org.resize(nc);
    g->dim.resize(nc);
    size_t cells = 0;
    for (int k = 0; k < nc; ++k) {
        int d[3];
        float o[3];
        for (int c = 0; c < 3; ++c) {
            const float l = lo[(size_t)k * 3 + c], h = hi[(size_t)k * 3 + c];
            if (!std::isfinite(l) || !std::isfinite(h) || !((h - l) * g->inv_cs < 1e6f)) return false;
            o[c] = l - 1.5f * cs;  // a padding cell below (volumes bin to cells >= 1)
            d[c] = (int)floorf((h - o[c]) * g->inv_cs) + 2;  // ... and at least one above
        }
        const uint32_t base = (uint32_t)cells;
        float basef;
        memcpy(&basef, &base, 4);
        g->org[k] = make_float4(o[0], o[1], o[2], basef);
        g->dim[k] = make_int4(d[0], d[1], d[2], 0);
        cells += (size_t)d[0] * d[1] * d[2];
        if (cells > kMaxGridCells) return false;
    }
    // volumes binned per cell
    std::vector<uint32_t> cell_of(n, 0xFFFFFFFFu), cnt(cells + 1, 0);
    for (int i = 0; i < n; ++i) {
        if (vc[i] < 0) continue;
        const float4 o = g->org[vc[i]];
        const int4 d = g->dim[vc[i]];
        uint32_t base;
        memcpy(&base, &o.w, 4);
        const int x = grid_cell(pos[4 * i], o.x, g->inv_cs, d.x), y = grid_cell(pos[4 * i + 1], o.y, g->inv_cs, d.y),
                  z = grid_cell(pos[4 * i + 2], o.z, g->inv_cs, d.z);
        if (x < 1 || y < 1 || z < 1 || x > d.x - 2 || y > d.y - 2 || z > d.z - 2) return false;
        cell_of[i] = base + (uint32_t)((z * d.y + y) * d.x + x);
        ++cnt[cell_of[i] + 1];
    }
    std::vector<uint32_t> own(cells + 1, 0);
    for (size_t c = 0; c < cells; ++c) own[c + 1] = own[c] + cnt[c + 1];
    std::vector<uint32_t> fill(own.begin(), own.end() - 1), vol_in(own[cells]);
    for (int i = 0; i < n; ++i)
        if (cell_of[i] != 0xFFFFFFFFu) vol_in[fill[cell_of[i]]++] = (uint32_t)i;
    // neighbourhood lists
    g->start.assign(cells + 1, 0);
    g->leaf.clear();
    g->leaf.reserve((size_t)27 * own[cells]);
    for (int k = 0; k < nc; ++k) {
        const int4 d = g->dim[k];
        uint32_t base;
        memcpy(&base, &g->org[k].w, 4);
        for (int z = 0; z < d.z; ++z)
            for (int y = 0; y < d.y; ++y)
                for (int x = 0; x < d.x; ++x) {
                    const uint32_t c = base + (uint32_t)((z * d.y + y) * d.x + x);
                    g->start[c] = (uint32_t)g->leaf.size();
                    for (int zz = std::max(z - 1, 0); zz <= std::min(z + 1, d.z - 1); ++zz)
                        for (int yy = std::max(y - 1, 0); yy <= std::min(y + 1, d.y - 1); ++yy)
                            for (int xx = std::max(x - 1, 0); xx <= std::min(x + 1, d.x - 1); ++xx) {
                                const uint32_t nb = base + (uint32_t)((zz * d.y + yy) * d.x + xx);
                                for (uint32_t t = own[nb]; t < own[nb + 1]; ++t) {
                                    const int v = (int)vol_in[t];
                                    float vf;
                                    memcpy(&vf, &v, 4);
                                    g->leaf.push_back(make_float4(pos[4 * v], pos[4 * v + 1], pos[4 * v + 2], vf));
                                }
                            }
                    // ascending distance to the cell centre (the kernel's float centre):
                    // the search stops at the first candidate that cannot beat its best
                    const float cx = g->org[k].x + ((float)x + 0.5f) * cs;
                    const float cy = g->org[k].y + ((float)y + 0.5f) * cs;
                    const float cz = g->org[k].z + ((float)z + 0.5f) * cs;
                    auto dc = [&](const float4& L) {
                        const double dx = (double)L.x - cx, dy = (double)L.y - cy, dz = (double)L.z - cz;
                        return dx * dx + dy * dy + dz * dz;
                    };
                    std::stable_sort(g->leaf.begin() + g->start[c], g->leaf.end(),
                                     [&](const float4& a, const float4& b) { return dc(a) < dc(b); });
                    if (g->leaf.size() > ((size_t)1 << 31)) return false;
                }
    }
    g->start[cells] = (uint32_t)g->leaf.size();
    return true;
}


}  // namespace

struct rt_sarsa {
    int device = 0;
    int n_vol = 0;
    uint32_t frames = 0;      // frames rendered so far (RNG sample base = frames * spp)
    uint64_t seed = 0;
    std::vector<float> pos;   // [n][4]
    std::vector<float> nrm;   // [n][3]
    std::vector<int32_t> surf;  // [n] surface index
    std::vector<rt::KdNode> kd;
    std::vector<float> lum;         // [n] luminance of the volume's surface
    std::vector<float> cos_center;  // [n*144] (rt_sarsa_load_q's irradiance)
    int64_t grid_cells = 0;   // nearest-volume grid (0: none, every search walks the KD tree)
    rt::SarsaMap m;
    std::vector<void*> allocs;
    // k_sarsa_render_pq's chunk sums and work counter (grown on demand)
    float* d_csum = nullptr;
    size_t csum_cap = 0;
    unsigned long long* d_work = nullptr;
    // the camera rays' rectangle masks of its table route (four 16x4 rectangles per block)
    unsigned long long* d_cull = nullptr;
    size_t cull_cap = 0;
    ~rt_sarsa() {
        (void)hipSetDevice(device);
        for (void* p : allocs) (void)hipFree(p);
        if (d_csum) (void)hipFree(d_csum);
        if (d_cull) (void)hipFree(d_cull);
        if (d_work) (void)hipFree(d_work);
        if (m.prof) (void)hipFree(m.prof);
    }
    template <class T>
    hipError_t alloc(T** p, size_t count) {
        void* q = nullptr;
        hipError_t e = hipMalloc(&q, sizeof(T) * (count ? count : 1));
        if (e == hipSuccess) allocs.push_back(q);
        *p = (T*)q;
        return e;
    }
};

namespace {

// initialise_radiance_grid (radiance_volume.cu:46-63): cos * (luminance / M_PI) * Q in
// double, summed in float
float initial_irradiance(const float* cc, const float* q, float lum) {
    float irr = 0.f;
    for (int k = 0; k < rt::kSarsaSectors; ++k)
        irr = (float)((double)irr + ((double)cc[k] * ((double)lum / M_PI)) * (double)q[k]);
    return irr;
}

int check_sarsa_params(const rt_params* p) {
    if (!p) return err(RT_E_INVALID, "params is NULL");
    if (p->width <= 0 || p->height <= 0 || p->spp <= 0) return err(RT_E_INVALID, "bad image size / spp");
    if (p->max_bounces < 1) return err(RT_E_INVALID, "max_bounces must be >= 1");
    if (p->preset != RT_PRESET_GPU)
        return err(RT_E_UNSUPPORTED, "the SARSA renderer implements the GPU-engine preset");
    if (p->hit_rule != RT_HIT_RULE_CPU && p->hit_rule != RT_HIT_RULE_GPU) return err(RT_E_INVALID, "bad hit_rule");
    const int split = p->spp_split <= 0 ? 1 : p->spp_split;
    if (split > 64 || (split & (split - 1)) != 0)
        return err(RT_E_INVALID, "spp_split must be a power of two <= 64");
    if (p->spp % split != 0) return err(RT_E_INVALID, "spp_split does not divide spp");
    if ((int64_t)p->width * (int64_t)p->height > (int64_t)1 << 31) return err(RT_E_INVALID, "image too large");
    return RT_OK;
}

int render_frame(rt_sarsa* sa, const rt_scene* scene, const rt_camera* cam, const rt_params* p,
                 const rt::BlockDesc* d_blocks, int n_blocks, int clip_x1, int clip_y1, int out_pitch,
                 float* d_out, unsigned long long* d_casts, hipStream_t stream, bool apply) {
    const int rc = rt::scene_ensure_ctab(scene, p->hit_rule, p->t_scale, rt::ctab_wanted(scene, cam, p, rt::kCtabForSarsa));
    if (rc != RT_OK) return rc;
    rt::RenderLaunch a = rt::render_launch(scene, cam, p);
    a.blocks = d_blocks;
    a.n_blocks = n_blocks;
    a.clip_x1 = clip_x1;
    a.clip_y1 = clip_y1;
    a.out_pitch = out_pitch;
    a.out = d_out;
    a.casts = d_casts;
    a.sample_base = sa->frames * (uint32_t)p->spp;
    // the persistent kernel's chunk sums (float4 per (pixel, chunk)) and work counter
    const size_t nc = (size_t)n_blocks * 256 * (size_t)a.split * 4;
    if (nc > sa->csum_cap) {
        if (sa->d_csum) (void)hipFree(sa->d_csum);
        sa->d_csum = nullptr;
        sa->csum_cap = 0;
        RT_HIPE(hipMalloc(&sa->d_csum, sizeof(float) * nc));
        sa->csum_cap = nc;
    }
    if (!sa->d_work) RT_HIPE(hipMalloc(&sa->d_work, sizeof(unsigned long long)));
    a.csum = sa->d_csum;
    a.work = sa->d_work;
    const size_t ncull = (size_t)n_blocks * 4 * rt::kRenderCullWords;
    if (ncull > sa->cull_cap) {
        if (sa->d_cull) (void)hipFree(sa->d_cull);
        sa->d_cull = nullptr;
        sa->cull_cap = 0;
        RT_HIPE(hipMalloc(&sa->d_cull, sizeof(unsigned long long) * ncull));
        sa->cull_cap = ncull;
    }
    a.cull = sa->d_cull;
    RT_HIPE(hipMemsetAsync(sa->m.stats, 0, 2 * sizeof(unsigned long long), stream));
    // RT_SARSA_PROF (with an RT_SARSA_PROF=1 kernel build): the render's per-phase cycles to stderr.
    // On a default build the counters are never written: warn once, and do not synchronise.
    static const bool prof_env = getenv("RT_SARSA_PROF") != nullptr;
    static const bool prof = prof_env && rt::sarsa_prof_compiled();
    static bool warned = false;
    if (prof_env && !prof && !warned) {
        warned = true;
        fprintf(stderr, "rtmi: RT_SARSA_PROF is set, but rt_sarsa.hip was built without -DRT_SARSA_PROF=1: ignored\n");
    }
    if (prof && !sa->m.prof) RT_HIPE(hipMalloc(&sa->m.prof, 8 * sizeof(unsigned long long)));
    if (prof) RT_HIPE(hipMemsetAsync(sa->m.prof, 0, 8 * sizeof(unsigned long long), stream));
    RT_HIPE(rt::launch_sarsa_render(a, sa->m, stream));
    if (prof) {
        unsigned long long v[8];
        RT_HIPE(hipStreamSynchronize(stream));
        RT_HIPE(hipMemcpy(v, sa->m.prof, sizeof(v), hipMemcpyDeviceToHost));
        fprintf(stderr, "{\"sarsa_prof\": {\"trace\": %llu, \"grid\": %llu, \"walks\": %llu, \"step\": %llu, "
                        "\"trips\": %llu, \"active_lanes\": %llu}}\n", v[0], v[1], v[2], v[3], v[4], v[5]);
    }
    if (apply) RT_HIPE(rt::launch_sarsa_apply(sa->m, stream));
    sa->frames += 1;
    return RT_OK;
}

}  // namespace

extern "C" {

int rt_sarsa_create(rt_ctx* ctx, const rt_scene* scene, uint64_t seed, rt_sarsa** out) {
    return rt_sarsa_create_density(ctx, scene, seed, kAreaPerSample, out);
}

int rt_sarsa_create_density(rt_ctx* ctx, const rt_scene* scene, uint64_t seed, float area_per_sample,
                            rt_sarsa** out) {
    if (!ctx || !scene || !out) return err(RT_E_INVALID, "NULL argument");
    *out = nullptr;
    if (!(area_per_sample > 0.f) || !isfinite(area_per_sample))
        return err(RT_E_INVALID, "area_per_sample must be a finite float > 0");
    {
        // the map takes ~4.7 KB of device memory per volume: refuse densities beyond 2^24 volumes
        const float *tri0, *nrm0, *alb0, *em0;
        int ns0, nl0;
        rt::scene_host(scene, &tri0, &nrm0, &alb0, &em0, &ns0, &nl0);
        double total = 0;
        for (int j = 0; j < ns0; ++j) total += floor((double)(triangle_area(tri0 + 9 * j) / area_per_sample));
        if (!(total <= (double)(1 << 24)))
            return err(RT_E_UNSUPPORTED, "area_per_sample gives more than 2^24 radiance volumes");
    }
    const float *tri, *normals, *albedo, *emission;
    int n_surf, n_light;
    rt::scene_host(scene, &tri, &normals, &albedo, &emission, &n_surf, &n_light);
    const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
    rt_sarsa* sa = new rt_sarsa();
    sa->device = rt::ctx_device(ctx);
    sa->seed = seed;
    // get_radiance_volumes_count + uniformly_sample_radiance_volumes: per surface,
    // floor(area / AREA_PER_SAMPLE) points by rejection (a1 + a2 <= 1), drawn from
    // Philox counter (volume, attempt, kPlacementEvent, 0) in place of rand().
    for (int j = 0; j < n_surf; ++j) {
        const float* v = tri + 9 * j;
        const int cnt = (int)floorf(triangle_area(v) / area_per_sample);
        for (int i = 0; i < cnt; ++i) {
            const uint32_t x = (uint32_t)sa->pos.size() / 4;
            float a1, a2;
            uint32_t attempt = 0;
            do {
                uint32_t r[4];
                rt::philox4x32_10(x, attempt++, kPlacementEvent, 0u, k0, k1, r);
                a1 = rt::u01(r[0]);
                a2 = rt::u01(r[1]);
            } while (a1 + a2 > 1.f);
            for (int c = 0; c < 3; ++c) {
                const float p0 = v[c], p1 = v[3 + c], p2 = v[6 + c];
                sa->pos.push_back((p0 + a1 * (p1 - p0)) + a2 * (p2 - p0));
            }
            sa->pos.push_back(1.f);
            for (int c = 0; c < 3; ++c) sa->nrm.push_back(normals[3 * j + c]);
            sa->surf.push_back(j);
        }
    }
    const int n = (int)sa->surf.size();
    sa->n_vol = n;
    if (n == 0) {
        delete sa;
        return err(RT_E_INVALID, "scene has no radiance volumes (total surface area < AREA_PER_SAMPLE)");
    }
    // RadianceVolume frames and per-sector cosines (cell centres for the CDF,
    // cell corners for expected_sarsa_irradiance), the initial Q / CDF / irradiance.
    const int S = rt::kSarsaSectors;
    std::vector<float> frame((size_t)n * 12), brdf(n), cc((size_t)n * S), ck((size_t)n * S), Q((size_t)n * S),
        cdf((size_t)n * S), accum(n);
    for (int i = 0; i < n; ++i) {
        const rt::f3 N = rt::make3(sa->nrm[3 * i], sa->nrm[3 * i + 1], sa->nrm[3 * i + 2]);
        const rt::f3 P = rt::make3(sa->pos[4 * i], sa->pos[4 * i + 1], sa->pos[4 * i + 2]);
        rt::f3 T, B;
        rt::normal_frame(N, &T, &B);
        const float f[12] = {N.x, N.y, N.z, P.x, T.x, T.y, T.z, P.y, B.x, B.y, B.z, P.z};
        memcpy(&frame[(size_t)12 * i], f, sizeof(f));
        const float lum = luminance(albedo + 3 * sa->surf[i]);
        brdf[i] = lum / rt::kPi;
        for (int x = 0; x < rt::kGridRes; ++x)
            for (int y = 0; y < rt::kGridRes; ++y) {
                const int k = x * rt::kGridRes + y;
                const rt::f3 dc = rt::grid_direction((float)x + 0.5f, (float)y + 0.5f, N, T, B, P);
                const rt::f3 dk = rt::grid_direction((float)x, (float)y, N, T, B, P);
                cc[(size_t)i * S + k] = rt::dot(dc, N);
                ck[(size_t)i * S + k] = rt::dot(dk, N);
                Q[(size_t)i * S + k] = kInitialRadiance;
                cdf[(size_t)i * S + k] = (float)k * (1.f / ((float)rt::kGridRes * (float)rt::kGridRes));
            }
        accum[i] = initial_irradiance(&cc[(size_t)i * S], &Q[(size_t)i * S], lum);
    }
    sa->lum.resize(n);
    for (int i = 0; i < n; ++i) sa->lum[i] = luminance(albedo + 3 * sa->surf[i]);
    sa->cos_center = cc;
    std::vector<float> tri_lum(n_surf + n_light);
    for (int j = 0; j < n_surf; ++j) tri_lum[j] = luminance(albedo + 3 * j);
    for (int j = 0; j < n_light; ++j) tri_lum[n_surf + j] = luminance(emission + 3 * j);
    // KD tree over the volume positions
    Tree t;
    t.pos = &sa->pos;
    std::vector<int> idx(n);
    for (int i = 0; i < n; ++i) idx[i] = i;
    const int root = t.build(idx, 0, 0);
    if (t.max_depth > kMaxKdDepth) {
        delete sa;
        return err(RT_E_UNSUPPORTED, "radiance tree deeper than the traversal stack allows");
    }
    t.flatten(root, sa->nrm);
    sa->kd = t.nodes;
    NearestGrid grid;
    const bool have_grid = build_nearest_grid(sa->pos, sa->nrm, n, normals, n_surf, sa->m.max_dist, &grid);

    hipError_t e = hipSetDevice(sa->device);
    float4 *d_pos = nullptr, *d_frame = nullptr;
    float *d_brdf = nullptr, *d_cc = nullptr, *d_ck = nullptr, *d_lum = nullptr, *d_Q = nullptr, *d_cdf = nullptr,
          *d_acc = nullptr;
    uint32_t *d_vis = nullptr, *d_cnt = nullptr;
    unsigned long long* d_sum = nullptr;
    uint4* d_kd = nullptr;
    std::vector<uint4> kd4(sa->kd.size());
    for (size_t i = 0; i < sa->kd.size(); ++i) {
        const rt::KdNode& k = sa->kd[i];
        if (k.leaf) {
            memcpy(&kd4[i].x, &k.px, 4);
            memcpy(&kd4[i].y, &k.py, 4);
            memcpy(&kd4[i].z, &k.pz, 4);
            kd4[i].w = (uint32_t)k.vol;
        } else {
            memcpy(&kd4[i].x, &k.data, 4);
            kd4[i].y = (uint32_t)k.left;
            kd4[i].z = (uint32_t)k.dim;
            kd4[i].w = 0xFFFFFFFFu;
        }
    }
    const size_t nS = (size_t)n * S;
    if (e == hipSuccess) e = sa->alloc(&d_pos, n);
    if (e == hipSuccess) e = sa->alloc(&d_frame, (size_t)n * 3);
    if (e == hipSuccess) e = sa->alloc(&d_brdf, n);
    if (e == hipSuccess) e = sa->alloc(&d_cc, nS);
    if (e == hipSuccess) e = sa->alloc(&d_ck, nS);
    if (e == hipSuccess) e = sa->alloc(&d_lum, tri_lum.size());
    if (e == hipSuccess) e = sa->alloc(&d_Q, nS);
    if (e == hipSuccess) e = sa->alloc(&d_cdf, nS);
    float4* d_top = nullptr;
    if (e == hipSuccess) e = sa->alloc(&d_top, (size_t)n * 4);
    if (e == hipSuccess) e = sa->alloc(&d_acc, n);
    if (e == hipSuccess) e = sa->alloc(&d_vis, nS);
    if (e == hipSuccess) e = sa->alloc(&d_cnt, nS);
    if (e == hipSuccess) e = sa->alloc(&d_sum, nS);
    if (e == hipSuccess) e = sa->alloc(&d_kd, sa->kd.size());
    int32_t* d_tcls = nullptr;
    float4 *d_corg = nullptr, *d_cnrm = nullptr, *d_leaf = nullptr;
    int4* d_cdim = nullptr;
    uint32_t* d_cstart = nullptr;
    unsigned long long* d_fb = nullptr;
    uint2* d_crange = nullptr;
    float4* d_tgrid = nullptr;
    float4* d_chead = nullptr;

    if (e == hipSuccess) e = sa->alloc(&d_fb, 1);
    unsigned long long* d_stats = nullptr;
    int32_t* d_qmax = nullptr;
    if (e == hipSuccess) e = sa->alloc(&d_stats, 2);
    if (e == hipSuccess) e = sa->alloc(&d_qmax, n);
    if (have_grid) {
        if (e == hipSuccess) e = sa->alloc(&d_tcls, grid.tri_class.size());
        if (e == hipSuccess) e = sa->alloc(&d_corg, grid.org.size());
        if (e == hipSuccess) e = sa->alloc(&d_cnrm, grid.nrm.size());
        if (e == hipSuccess) e = sa->alloc(&d_cdim, grid.dim.size());
        if (e == hipSuccess) e = sa->alloc(&d_cstart, grid.start.size());
        if (e == hipSuccess) e = sa->alloc(&d_leaf, grid.leaf.size());
        if (e == hipSuccess) e = sa->alloc(&d_crange, grid.start.size() - 1);
        if (e == hipSuccess) e = sa->alloc(&d_chead, 4 * (grid.start.size() - 1));
        if (e == hipSuccess) e = sa->alloc(&d_tgrid, 2 * grid.tri_class.size());
    }

    auto up = [&](void* d, const void* h, size_t bytes) {
        if (e == hipSuccess && bytes) e = hipMemcpy(d, h, bytes, hipMemcpyHostToDevice);
    };
    up(d_pos, sa->pos.data(), sizeof(float) * 4 * n);
    up(d_frame, frame.data(), sizeof(float) * frame.size());
    up(d_brdf, brdf.data(), sizeof(float) * n);
    up(d_cc, cc.data(), sizeof(float) * nS);
    up(d_ck, ck.data(), sizeof(float) * nS);
    up(d_lum, tri_lum.data(), sizeof(float) * tri_lum.size());
    up(d_Q, Q.data(), sizeof(float) * nS);
    up(d_cdf, cdf.data(), sizeof(float) * nS);
    {
        std::vector<float> top((size_t)n * 16, 0.f);
        for (int i = 0; i < n; ++i) {
            top[(size_t)16 * i] = cdf[(size_t)i * S];
            for (int x = 0; x < rt::kGridRes; ++x)
                top[(size_t)16 * i + 1 + x] = cdf[(size_t)i * S + x * rt::kGridRes + rt::kGridRes - 1];
        }
        up(d_top, top.data(), sizeof(float) * top.size());
    }
    up(d_acc, accum.data(), sizeof(float) * n);
    up(d_kd, kd4.data(), sizeof(uint4) * kd4.size());
    if (have_grid) {
        up(d_tcls, grid.tri_class.data(), sizeof(int32_t) * grid.tri_class.size());
        up(d_corg, grid.org.data(), sizeof(float4) * grid.org.size());
        up(d_cnrm, grid.nrm.data(), sizeof(float4) * grid.nrm.size());
        up(d_cdim, grid.dim.data(), sizeof(int4) * grid.dim.size());
        up(d_cstart, grid.start.data(), sizeof(uint32_t) * grid.start.size());
        up(d_leaf, grid.leaf.data(), sizeof(float4) * grid.leaf.size());
        std::vector<uint2> range(grid.start.size() - 1);
        for (size_t c = 0; c + 1 < grid.start.size(); ++c) range[c] = make_uint2(grid.start[c], grid.start[c + 1]);
        up(d_crange, range.data(), sizeof(uint2) * range.size());
        // per cell: its range and first three candidates in one 64-B record (the search's
        // first load then already holds them: one dependent round trip less)
        std::vector<float4> head(4 * range.size(), make_float4(0.f, 0.f, 0.f, 0.f));
        for (size_t c = 0; c < range.size(); ++c) {
            float fx, fy;
            memcpy(&fx, &range[c].x, 4);
            memcpy(&fy, &range[c].y, 4);
            head[4 * c] = make_float4(fx, fy, 0.f, 0.f);
            for (uint32_t u = 0; u < 3 && range[c].x + u < range[c].y; ++u) head[4 * c + 1 + u] = grid.leaf[range[c].x + u];
        }
        up(d_chead, head.data(), sizeof(float4) * head.size());
        // per surface: its class's grid descriptor (the kernel's one-step lookup)
        std::vector<float4> tg(2 * grid.tri_class.size(), make_float4(0.f, 0.f, 0.f, 0.f));
        for (size_t j = 0; j < grid.tri_class.size(); ++j) {
            const int k = grid.tri_class[j];
            int4 d = make_int4(0, 0, 0, -1);
            if (k >= 0) {
                tg[2 * j] = grid.org[k];
                d = make_int4(grid.dim[k].x, grid.dim[k].y, grid.dim[k].z, k);
            }
            memcpy(&tg[2 * j + 1], &d, sizeof(d));
        }
        up(d_tgrid, tg.data(), sizeof(float4) * tg.size());
    }

    if (e == hipSuccess) e = hipMemset(d_fb, 0, sizeof(unsigned long long));
    if (e == hipSuccess) e = hipMemset(d_stats, 0, 2 * sizeof(unsigned long long));
    if (e == hipSuccess) e = hipMemset(d_qmax, 0, sizeof(int32_t) * n);  // every Q equal: sector 0
    if (e == hipSuccess) e = hipMemset(d_vis, 0, sizeof(uint32_t) * nS);
    if (e == hipSuccess) e = hipMemset(d_cnt, 0, sizeof(uint32_t) * nS);
    if (e == hipSuccess) e = hipMemset(d_sum, 0, sizeof(unsigned long long) * nS);
    if (e != hipSuccess) {
        delete sa;
        return err(RT_E_HIP, std::string("rt_sarsa_create: ") + hipGetErrorString(e));
    }
    rt::SarsaMap& m = sa->m;
    m.n_vol = n;
    m.vol_pos = d_pos;
    m.vol_frame = d_frame;
    m.vol_brdf = d_brdf;
    m.cos_center = d_cc;
    m.cos_corner = d_ck;
    m.tri_lum = d_lum;
    m.Q = d_Q;
    m.cdf = d_cdf;
    m.cdf_top = d_top;
    m.visits = d_vis;
    m.accum = d_acc;
    m.acc_sum = d_sum;
    m.acc_cnt = d_cnt;
    m.kd4 = d_kd;
    m.n_kd = (int)sa->kd.size();
    m.root_x = sa->kd[0].px;
    m.root_y = sa->kd[0].py;
    m.root_z = sa->kd[0].pz;
    if (have_grid) {
        m.use_grid = 1;
        m.n_class = (int)grid.org.size();
        m.tri_class = d_tcls;
        m.class_org = d_corg;
        m.class_dim = d_cdim;
        m.class_nrm = d_cnrm;
        m.cell_start = d_cstart;
        m.grid_leaf = d_leaf;
        m.cell_range = d_crange;
        m.cell_head = d_chead;
        m.tri_grid = d_tgrid;

        m.grid_inv_cs = grid.inv_cs;
        m.grid_cs = grid.cs;
        m.grid_h = grid.h;
        sa->grid_cells = (int64_t)grid.start.size() - 1;
    }
    m.grid_fallbacks = d_fb;
    m.stats = d_stats;
    m.qmax = d_qmax;
    *out = sa;
    return RT_OK;
}

int rt_sarsa_destroy(rt_sarsa* sarsa) {
    delete sarsa;
    return RT_OK;
}

int rt_sarsa_info(const rt_sarsa* sa, int32_t* n_volumes, int32_t* n_nodes, uint32_t* frames) {
    if (!sa) return err(RT_E_INVALID, "NULL argument");
    if (n_volumes) *n_volumes = sa->n_vol;
    if (n_nodes) *n_nodes = (int32_t)sa->kd.size();
    if (frames) *frames = sa->frames;
    return RT_OK;
}

int rt_sarsa_set_search(rt_sarsa* sa, int mode) {
    if (!sa) return err(RT_E_INVALID, "NULL argument");
    if (mode != RT_SARSA_SEARCH_KD && mode != RT_SARSA_SEARCH_GRID) return err(RT_E_INVALID, "bad search mode");
    sa->m.use_grid = (mode == RT_SARSA_SEARCH_GRID && sa->grid_cells > 0) ? 1 : 0;
    return RT_OK;
}

int rt_sarsa_search_stats(const rt_sarsa* sa, int32_t* mode, int32_t* n_classes, int64_t* grid_cells,
                          uint64_t* kd_fallbacks) {
    if (!sa) return err(RT_E_INVALID, "NULL argument");
    if (mode) *mode = sa->m.use_grid ? RT_SARSA_SEARCH_GRID : RT_SARSA_SEARCH_KD;
    if (n_classes) *n_classes = sa->m.n_class;
    if (grid_cells) *grid_cells = sa->grid_cells;
    if (kd_fallbacks) {
        unsigned long long v = 0;
        (void)hipSetDevice(sa->device);
        RT_HIPE(hipMemcpy(&v, sa->m.grid_fallbacks, sizeof(v), hipMemcpyDeviceToHost));
        *kd_fallbacks = v;
    }
    return RT_OK;
}

int rt_sarsa_volumes(const rt_sarsa* sa, float* pos, float* normal, int32_t* surface, float* kd_nodes) {
    if (!sa) return err(RT_E_INVALID, "NULL argument");
    const int n = sa->n_vol;
    if (pos)
        for (int i = 0; i < n; ++i) memcpy(pos + 3 * i, &sa->pos[4 * i], sizeof(float) * 3);
    if (normal) memcpy(normal, sa->nrm.data(), sizeof(float) * 3 * n);
    if (surface) memcpy(surface, sa->surf.data(), sizeof(int32_t) * n);
    if (kd_nodes) memcpy(kd_nodes, sa->kd.data(), sizeof(rt::KdNode) * sa->kd.size());
    return RT_OK;
}

int rt_sarsa_read(const rt_sarsa* sa, float* q, float* cdf, uint32_t* visits, float* irradiance) {
    if (!sa) return err(RT_E_INVALID, "NULL argument");
    RT_HIPE(hipSetDevice(sa->device));
    const size_t nS = (size_t)sa->n_vol * rt::kSarsaSectors;
    RT_HIPE(hipDeviceSynchronize());
    if (q) RT_HIPE(hipMemcpy(q, sa->m.Q, sizeof(float) * nS, hipMemcpyDeviceToHost));
    if (cdf) RT_HIPE(hipMemcpy(cdf, sa->m.cdf, sizeof(float) * nS, hipMemcpyDeviceToHost));
    if (visits) RT_HIPE(hipMemcpy(visits, sa->m.visits, sizeof(uint32_t) * nS, hipMemcpyDeviceToHost));
    if (irradiance) RT_HIPE(hipMemcpy(irradiance, sa->m.accum, sizeof(float) * sa->n_vol, hipMemcpyDeviceToHost));
    return RT_OK;
}

int rt_sarsa_nearest(rt_ctx* ctx, const rt_sarsa* sa, const float* pos, const float* normal, int n, int32_t* out) {
    if (!ctx || !sa || (n > 0 && (!pos || !normal || !out))) return err(RT_E_INVALID, "NULL argument");
    if (n < 0) return err(RT_E_INVALID, "n < 0");
    if (n == 0) return RT_OK;
    RT_HIPE(hipSetDevice(sa->device));
    float *d_p = nullptr, *d_n = nullptr;
    int32_t* d_o = nullptr;
    const size_t b3 = sizeof(float) * 3 * (size_t)n;
    hipError_t e = hipMalloc(&d_p, b3);
    if (e == hipSuccess) e = hipMalloc(&d_n, b3);
    if (e == hipSuccess) e = hipMalloc(&d_o, sizeof(int32_t) * n);
    if (e == hipSuccess) e = hipMemcpy(d_p, pos, b3, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(d_n, normal, b3, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = rt::launch_sarsa_nearest(sa->m, d_p, d_n, n, d_o, 0);
    if (e == hipSuccess) e = hipMemcpy(out, d_o, sizeof(int32_t) * n, hipMemcpyDeviceToHost);
    (void)hipFree(d_p);
    (void)hipFree(d_n);
    (void)hipFree(d_o);
    if (e != hipSuccess) return err(RT_E_HIP, std::string("rt_sarsa_nearest: ") + hipGetErrorString(e));
    return RT_OK;
}

int rt_sarsa_save_q(const rt_sarsa* sa, const char* path) {
    if (!sa || !path) return err(RT_E_INVALID, "NULL argument");
    const int S = rt::kSarsaSectors;
    std::vector<float> q((size_t)sa->n_vol * S);
    int rc = rt_sarsa_read(sa, q.data(), nullptr, nullptr, nullptr);
    if (rc != RT_OK) return rc;
    // RadianceMap::save_q_vals_to_file: ostream defaults (6 significant digits)
    std::ofstream f(path);
    if (!f.is_open()) return err(RT_E_IO, std::string("cannot write ") + path);
    f << S << "\n";
    for (int i = 0; i < sa->n_vol; ++i) {
        f << sa->pos[4 * i] << " " << sa->pos[4 * i + 1] << " " << sa->pos[4 * i + 2];
        for (int k = 0; k < S; ++k) f << " " << q[(size_t)i * S + k];
        f << "\n";
    }
    f.close();
    if (f.fail()) return err(RT_E_IO, std::string("write failed: ") + path);
    return RT_OK;
}

int rt_sarsa_load_q(rt_sarsa* sa, const char* path) {
    if (!sa || !path) return err(RT_E_INVALID, "NULL argument");
    const int S = rt::kSarsaSectors;
    FILE* f = fopen(path, "r");
    if (!f) return err(RT_E_IO, std::string("cannot open ") + path);
    std::vector<float> q((size_t)sa->n_vol * S);
    int rc = RT_OK;
    int actions = 0;
    if (fscanf(f, "%d", &actions) != 1 || actions != S) rc = err(RT_E_IO, "first line must be the action count 144");
    char tok[64];
    auto next = [&](float* v) {  // std::stof semantics
        if (fscanf(f, "%63s", tok) != 1) return false;
        char* end = nullptr;
        *v = strtof(tok, &end);
        return end != tok && *end == '\0';
    };
    for (int i = 0; rc == RT_OK && i < sa->n_vol; ++i) {
        for (int c = 0; c < 3 && rc == RT_OK; ++c) {
            float v;
            if (!next(&v)) {
                rc = err(RT_E_IO, "truncated or malformed Q-table file");
                break;
            }
            // the position must be this map's volume i as save_q prints it
            std::ostringstream os;
            os << sa->pos[4 * i + c];
            if (strtof(os.str().c_str(), nullptr) != v)
                rc = err(RT_E_INVALID, "volume " + std::to_string(i) + ": position differs from this map's "
                                       "(another scene or seed)");
        }
        for (int k = 0; k < S && rc == RT_OK; ++k)
            if (!next(&q[(size_t)i * S + k])) rc = err(RT_E_IO, "truncated or malformed Q-table file");
    }
    if (rc == RT_OK && fscanf(f, "%63s", tok) == 1) rc = err(RT_E_INVALID, "more volumes in the file than in the map");
    fclose(f);
    if (rc != RT_OK) return rc;
    std::vector<float> accum(sa->n_vol);
    for (int i = 0; i < sa->n_vol; ++i)
        accum[i] = initial_irradiance(&sa->cos_center[(size_t)i * S], &q[(size_t)i * S], sa->lum[i]);
    RT_HIPE(hipSetDevice(sa->device));
    RT_HIPE(hipDeviceSynchronize());
    RT_HIPE(hipMemcpy(sa->m.Q, q.data(), sizeof(float) * q.size(), hipMemcpyHostToDevice));
    RT_HIPE(hipMemcpy(sa->m.accum, accum.data(), sizeof(float) * accum.size(), hipMemcpyHostToDevice));
    RT_HIPE(rt::launch_sarsa_rebuild(sa->m, 0));
    RT_HIPE(hipDeviceSynchronize());
    return RT_OK;
}

int rt_sarsa_set_sampling(rt_sarsa* sa, int mode) {
    if (!sa) return err(RT_E_INVALID, "NULL argument");
    if (mode != RT_SARSA_SAMPLE_CDF && mode != RT_SARSA_SAMPLE_MAX) return err(RT_E_INVALID, "bad sampling mode");
    sa->m.sample_max = mode == RT_SARSA_SAMPLE_MAX;
    return RT_OK;
}

int rt_sarsa_set_td_mode(rt_sarsa* sa, int mode) {
    if (!sa) return err(RT_E_INVALID, "NULL argument");
    if (mode != RT_SARSA_TD_FRAME && mode != RT_SARSA_TD_INFRAME) return err(RT_E_INVALID, "bad TD mode");
    sa->m.td_inframe = mode == RT_SARSA_TD_INFRAME;
    return RT_OK;
}

int rt_sarsa_set_inframe_lanes(rt_sarsa* sa, int lanes) {
    if (!sa) return err(RT_E_INVALID, "NULL argument");
    if (lanes < 0) return err(RT_E_INVALID, "lanes must be >= 0");
    sa->m.max_wgs = lanes == 0 ? 0 : (int)(((int64_t)lanes + 255) / 256);
    return RT_OK;
}

int rt_sarsa_get_td_mode(const rt_sarsa* sa, int* mode) {
    if (!sa || !mode) return err(RT_E_INVALID, "NULL argument");
    *mode = sa->m.td_inframe ? RT_SARSA_TD_INFRAME : RT_SARSA_TD_FRAME;
    return RT_OK;
}

int rt_sarsa_frame_stats(const rt_sarsa* sa, uint64_t* path_floor_sum, uint64_t* zero_paths) {
    if (!sa) return err(RT_E_INVALID, "NULL argument");
    unsigned long long v[2] = {0, 0};
    RT_HIPE(hipSetDevice(sa->device));
    RT_HIPE(hipDeviceSynchronize());
    RT_HIPE(hipMemcpy(v, sa->m.stats, sizeof(v), hipMemcpyDeviceToHost));
    if (path_floor_sum) *path_floor_sum = v[0];
    if (zero_paths) *zero_paths = v[1];
    return RT_OK;
}

int rt_sarsa_save_selected(rt_ctx* ctx, const rt_sarsa* sa, const char* to_select_path, const char* out_path) {
    if (!ctx || !sa || !to_select_path || !out_path) return err(RT_E_INVALID, "NULL argument");
    std::vector<float> qp, qn;
    int rc = rt::read_locations(to_select_path, &qp, &qn);
    if (rc != RT_OK) return rc;
    const int n = (int)qp.size() / 3;
    std::vector<int32_t> idx(n);
    rc = rt_sarsa_nearest(ctx, sa, qp.data(), qn.data(), n, idx.data());
    if (rc != RT_OK) return rc;
    const int S = rt::kSarsaSectors;
    std::vector<float> cdf((size_t)sa->n_vol * S);
    rc = rt_sarsa_read(sa, nullptr, cdf.data(), nullptr, nullptr);
    if (rc != RT_OK) return rc;
    // the file is replaced, then each volume appended (write_volume_to_file,
    // radiance_volume.cu:338-365) with its distribution: convert_radiance_distribution
    // (:332-336) differences the CDF, sector 0 keeps cdf[0]
    std::ofstream f(out_path);
    if (!f.is_open()) return err(RT_E_IO, std::string("cannot write ") + out_path);
    for (int i = 0; i < n; ++i) {
        const int v = idx[i];
        const float* c = &cdf[(size_t)v * S];
        f << sa->pos[4 * v] << " " << sa->pos[4 * v + 1] << " " << sa->pos[4 * v + 2];
        f << " " << sa->nrm[3 * v] << " " << sa->nrm[3 * v + 1] << " " << sa->nrm[3 * v + 2];
        for (int k = 0; k < S; ++k) f << " " << (k == 0 ? c[0] : c[k] - c[k - 1]);
        f << "\n";
    }
    f.close();
    if (f.fail()) return err(RT_E_IO, std::string("write failed: ") + out_path);
    return RT_OK;
}

int rt_render_sarsa(rt_ctx* ctx, const rt_scene* scene, rt_sarsa* sa, const rt_camera* cam,
                    const rt_params* params, int frames, float* out_rgb, uint64_t* out_ray_casts) {
    if (!ctx || !scene || !sa || !cam || !out_rgb) return err(RT_E_INVALID, "NULL argument");
    int rc = check_sarsa_params(params);
    if (rc != RT_OK) return rc;
    if (frames < 1) return err(RT_E_INVALID, "frames must be >= 1");
    if (sa->device != rt::ctx_device(ctx)) return err(RT_E_INVALID, "radiance map belongs to another device");
    RT_HIPE(hipSetDevice(sa->device));
    const int W = params->width, H = params->height;
    std::vector<rt::BlockDesc> blocks;
    for (int by = 0; by < H; by += 16)
        for (int bx = 0; bx < W; bx += 16) blocks.push_back({bx, by, bx, by});
    rt::BlockDesc* d_blocks = nullptr;
    float* d_out = nullptr;
    unsigned long long* d_casts = nullptr;
    const size_t ob = sizeof(float) * 3 * (size_t)W * H;
    hipError_t e = hipMalloc(&d_blocks, sizeof(rt::BlockDesc) * blocks.size());
    if (e == hipSuccess) e = hipMalloc(&d_out, ob);
    if (e == hipSuccess) e = hipMalloc(&d_casts, sizeof(unsigned long long));
    if (e == hipSuccess) e = hipMemset(d_casts, 0, sizeof(unsigned long long));
    if (e == hipSuccess)
        e = hipMemcpy(d_blocks, blocks.data(), sizeof(rt::BlockDesc) * blocks.size(), hipMemcpyHostToDevice);
    rc = RT_OK;
    for (int f = 0; e == hipSuccess && rc == RT_OK && f < frames; ++f)
        rc = render_frame(sa, scene, cam, params, d_blocks, (int)blocks.size(), W, H, W, d_out, d_casts, 0, true);
    if (rc == RT_OK && e == hipSuccess) e = hipDeviceSynchronize();
    unsigned long long casts = 0;
    if (rc == RT_OK && e == hipSuccess) e = hipMemcpy(out_rgb, d_out, ob, hipMemcpyDeviceToHost);
    if (rc == RT_OK && e == hipSuccess) e = hipMemcpy(&casts, d_casts, sizeof(casts), hipMemcpyDeviceToHost);
    (void)hipFree(d_blocks);
    (void)hipFree(d_out);
    (void)hipFree(d_casts);
    if (rc != RT_OK) return rc;
    if (e != hipSuccess) return err(RT_E_HIP, std::string("rt_render_sarsa: ") + hipGetErrorString(e));
    if (out_ray_casts) *out_ray_casts = casts;
    return RT_OK;
}

int rt_render_sarsa_tiles_device(rt_ctx* ctx, const rt_scene* scene, rt_sarsa* sa, const rt_camera* cam,
                                 const rt_params* params, const int32_t* tiles, int n_tiles, int tile_size,
                                 float* d_out, uint64_t* d_casts, int apply, void* stream) {
    if (!ctx || !scene || !sa || !cam) return err(RT_E_INVALID, "NULL argument");
    int rc = check_sarsa_params(params);
    if (rc != RT_OK) return rc;
    if (n_tiles < 0 || (n_tiles > 0 && (!tiles || !d_out))) return err(RT_E_INVALID, "bad tiles/out");
    if (sa->device != rt::ctx_device(ctx)) return err(RT_E_INVALID, "radiance map belongs to another device");
    if (!apply && sa->m.td_inframe)
        return err(RT_E_UNSUPPORTED, "in-frame TD mode: the frame's TD is applied in place, nothing to exchange");
    RT_HIPE(hipSetDevice(sa->device));
    const rt::BlockDesc* d_blocks = nullptr;
    int n_blocks = 0;
    if (n_tiles > 0) {
        rc = rt::ctx_blocks(ctx, tiles, n_tiles, tile_size, params->width, params->height, &d_blocks, &n_blocks);
        if (rc != RT_OK) return rc;
    }
    return render_frame(sa, scene, cam, params, d_blocks, n_blocks, params->width, params->height, tile_size, d_out,
                        reinterpret_cast<unsigned long long*>(d_casts), (hipStream_t)stream, apply != 0);
}

int rt_sarsa_td_device(rt_sarsa* sa, void** d_sum, void** d_count, int64_t* n_entries) {
    if (!sa) return err(RT_E_INVALID, "NULL argument");
    if (sa->m.td_inframe)
        return err(RT_E_UNSUPPORTED, "in-frame TD mode: no frame TD sums (the map is updated in place)");
    if (d_sum) *d_sum = sa->m.acc_sum;
    if (d_count) *d_count = sa->m.acc_cnt;
    if (n_entries) *n_entries = (int64_t)sa->n_vol * rt::kSarsaSectors;
    return RT_OK;
}

int rt_sarsa_apply(rt_sarsa* sa, void* stream) {
    if (!sa) return err(RT_E_INVALID, "NULL argument");
    RT_HIPE(hipSetDevice(sa->device));
    RT_HIPE(rt::launch_sarsa_apply(sa->m, (hipStream_t)stream));
    return RT_OK;
}

}  // extern "C"
