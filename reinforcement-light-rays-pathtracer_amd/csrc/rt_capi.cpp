// rt_capi.cpp — the C ABI (include/rtmi.h): contexts, device scenes,
// launches.  Host-only code; the kernels live in rt_kernels.hip.
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdarg.h>
#include <stdlib.h>

#include <cmath>
#include <stdio.h>
#include <string.h>

#include <atomic>
#include <chrono>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/rtmi.h"
#include "rt_cull.hpp"
#include "rt_internal.hpp"

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

#define RT_HIP(expr)                                                                    \
    do {                                                                                \
        hipError_t e_ = (expr);                                                         \
        if (e_ != hipSuccess)                                                           \
            return fail(RT_E_HIP, "%s failed: %s", #expr, hipGetErrorString(e_));       \
    } while (0)

}  // namespace

namespace rt {
int set_error(int code, const char* msg) {
    g_err = msg;
    return code;
}
}  // namespace rt

struct rt_ctx {
    int device = 0;
    // cached block list for rt_render_tiles_device
    std::vector<int32_t> tiles_key;
    int tiles_size = 0, tiles_w = 0, tiles_h = 0;
    rt::BlockDesc* d_blocks = nullptr;
    int n_blocks = 0;
    int blocks_cap = 0;
    // per-wave candidate masks of rt_cull_masks_device (RenderLaunch::cull)
    unsigned long long* d_cull = nullptr;
    size_t cull_cap = 0;
    // the GPU preset's chunk sums and work counter (RenderLaunch::csum / work, k_render_pq)
    float* d_csum = nullptr;
    size_t csum_cap = 0;
    unsigned long long* d_work = nullptr;
};

struct rt_scene {
    rt_ctx* ctx = nullptr;
    rt::DeviceScene dev;
    int n_surf = 0, n_light = 0;
    std::vector<float> normals;  // host copy, n_tri x 3
    std::vector<float> tri;      // host copy, n_tri x 9 (surfaces then lights)
    std::vector<float> albedo;   // n_surf x 3
    std::vector<float> emission; // n_light x 3
    // exact BVH path (rt_bvh.cpp): built for scenes above RT_BVH_AUTO_MIN triangles or on
    // request (rt_scene_set_accel)
    int accel = RT_ACCEL_AUTO;
    bool has_bvh = false;
    rt::BvhHost bvh;
    float4* d_bvh[4] = {nullptr, nullptr, nullptr, nullptr};  // nodes, tris, graze, grec
    int32_t* d_dir[3] = {nullptr, nullptr, nullptr};           // starts (2 sets), list, camera list
    // bounce-ray candidate table (rt_ctab.cpp): built on the first render that can use it
    // (scene_ensure_ctab), its device arrays in dev.ctab*
    bool ctab_tried[2] = {false, false};  // per hit rule
    std::mutex ctab_mu;                    // (renders of one scene from several threads)
    double ctab_build_s[2] = {0.0, 0.0};   // host build + upload, seconds (rt_scene_ctab_info)
    uint64_t ctab_bytes[2] = {0, 0};       // device bytes of the table
};

namespace {
// the BVH's device arrays, or nothing
void scene_free_bvh(rt_scene* sc);

// (on any failure every partial allocation is released: has_bvh stays false and the
// pointers null, so a later call starts clean)
int scene_build_bvh(rt_scene* sc) {
    if (sc->has_bvh) return RT_OK;
    scene_free_bvh(sc);
    std::vector<float4> isect((size_t)sc->dev.n_tri * rt::kIsectF4);
    if (hipMemcpy(isect.data(), sc->dev.isect, sizeof(float4) * isect.size(), hipMemcpyDeviceToHost) != hipSuccess)
        return RT_E_HIP;
    if (!rt::bvh_build(isect.data(), sc->dev.n_tri, &sc->bvh)) return RT_E_UNSUPPORTED;
    const rt::BvhHost& b = sc->bvh;
    hipError_t e = hipSuccess;
    auto put = [&](auto** dst, const auto& v) {
        if (e != hipSuccess) return;
        e = hipMalloc(dst, sizeof(v[0]) * std::max<size_t>(1, v.size()));
        if (e == hipSuccess && !v.empty()) e = hipMemcpy(*dst, v.data(), sizeof(v[0]) * v.size(), hipMemcpyHostToDevice);
    };
    put(&sc->d_bvh[0], b.nodes);
    put(&sc->d_bvh[1], b.tris);
    put(&sc->d_bvh[2], b.graze);
    put(&sc->d_bvh[3], b.grec);
    std::vector<int32_t> starts(b.dstart);
    starts.insert(starts.end(), b.dstart_cam.begin(), b.dstart_cam.end());
    put(&sc->d_dir[0], starts);
    put(&sc->d_dir[1], b.dlist);
    put(&sc->d_dir[2], b.dlist_cam);
    if (e != hipSuccess) {
        scene_free_bvh(sc);
        return RT_E_HIP;
    }
    sc->has_bvh = true;
    return RT_OK;
}

void scene_free_bvh(rt_scene* sc) {
    for (auto& p : sc->d_bvh) {
        if (p) (void)hipFree(p);
        p = nullptr;
    }
    for (auto& p : sc->d_dir) {
        if (p) (void)hipFree(p);
        p = nullptr;
    }
    sc->has_bvh = false;
}

bool scene_uses_bvh(const rt_scene* sc) {
    if (!sc->has_bvh) return false;
    if (sc->accel == RT_ACCEL_BVH) return true;
    return sc->accel == RT_ACCEL_AUTO && sc->dev.n_tri > RT_BVH_AUTO_MIN;
}

// the device view of the scene for a launch (BVH fields set when the BVH path is on, or
// whenever the BVH exists with force_bvh: RT_ISECT_BVH, without touching the scene's mode)
rt::DeviceScene launch_scene(const rt_scene* sc, bool force_bvh = false) {
    rt::DeviceScene d = sc->dev;
    if (force_bvh ? !sc->has_bvh : !scene_uses_bvh(sc)) return d;
    d.bvh_nodes = sc->d_bvh[0];
    d.bvh_tris = sc->d_bvh[1];
    d.bvh_graze = sc->d_bvh[2];
    d.bvh_grec = sc->d_bvh[3];
    d.bvh_dstart = sc->d_dir[0];
    d.bvh_dlist = sc->d_dir[1];
    d.bvh_dlist_cam = sc->d_dir[2];
    d.bvh_B_lists = sc->bvh.B_lists;
    d.bvh_sig_a = sc->bvh.sig_a;
    d.bvh_sig_b = sc->bvh.sig_b;
    return d;
}
}  // namespace

namespace rt {
void release_dqn_workspace(const rt_ctx* ctx);
int ctx_device(const rt_ctx* ctx) { return ctx->device; }
const DeviceScene& scene_device(const rt_scene* s) { return s->dev; }
// the device view a render launch takes (the BVH fields set when the scene's BVH path is on)
DeviceScene scene_launch_view(const rt_scene* s) { return launch_scene(s); }
void scene_host(const rt_scene* s, const float** tri, const float** normals, const float** albedo,
                const float** emission, int* n_surf, int* n_light) {
    *tri = s->tri.data();
    *normals = s->normals.data();
    *albedo = s->albedo.data();
    *emission = s->emission.data();
    *n_surf = s->n_surf;
    *n_light = s->n_light;
}
int ensure_blocks_impl(rt_ctx* ctx, const std::vector<BlockDesc>& blocks);
// Device block list (16x16 pixel blocks) of a tile list, cached per context.
int ctx_blocks(rt_ctx* ctx, const int32_t* tiles, int n_tiles, int tile_size, int width, int height,
               const BlockDesc** d_blocks, int* n_blocks) {
    if (tile_size <= 0 || tile_size % 16 != 0)
        return set_error(RT_E_INVALID, "tile_size must be a positive multiple of 16");
    for (int k = 0; k < n_tiles; ++k) {
        const int tx = tiles[2 * k], ty = tiles[2 * k + 1];
        if (tx < 0 || ty < 0 || tx >= width || ty >= height)
            return set_error(RT_E_INVALID, "tile origin outside the image");
    }
    const bool same = ctx->tiles_size == tile_size && ctx->tiles_w == width && ctx->tiles_h == height &&
                      (int)ctx->tiles_key.size() == 2 * n_tiles &&
                      memcmp(ctx->tiles_key.data(), tiles, sizeof(int32_t) * 2 * n_tiles) == 0;
    if (!same) {
        std::vector<BlockDesc> blocks;
        const int per = tile_size / 16;
        for (int k = 0; k < n_tiles; ++k)
            for (int sy = 0; sy < per; ++sy)
                for (int sx = 0; sx < per; ++sx)
                    blocks.push_back({tiles[2 * k] + 16 * sx, tiles[2 * k + 1] + 16 * sy, 16 * sx,
                                      k * tile_size + 16 * sy});
        int rc = ensure_blocks_impl(ctx, blocks);
        if (rc != RT_OK) return rc;
        ctx->tiles_key.assign(tiles, tiles + 2 * n_tiles);
        ctx->tiles_size = tile_size;
        ctx->tiles_w = width;
        ctx->tiles_h = height;
    }
    *d_blocks = ctx->d_blocks;
    *n_blocks = ctx->n_blocks;
    return RT_OK;
}
}  // namespace rt

namespace {

int set_device(rt_ctx* ctx) {
    RT_HIP(hipSetDevice(ctx->device));
    return RT_OK;
}

}  // namespace

namespace rt {
// The cull workspace of a render launch (grown on demand, kept by the context).
int ctx_cull(rt_ctx* ctx, RenderLaunch* a) {
    const size_t words = (size_t)a->n_blocks * (size_t)a->split * 4 * kRenderCullWords;
    if (words > ctx->cull_cap) {
        if (ctx->d_cull) RT_HIP(hipFree(ctx->d_cull));
        ctx->d_cull = nullptr;
        ctx->cull_cap = 0;
        RT_HIP(hipMalloc(&ctx->d_cull, sizeof(unsigned long long) * words));
        ctx->cull_cap = words;
    }
    a->cull = ctx->d_cull;
    return RT_OK;
}

// The GPU preset's chunk-queue workspace (k_render_pq): one float3 per (pixel, chunk) of the
// launch, the work counter and the camera-ray masks (grown on demand, kept by the context)
int ctx_chunks(rt_ctx* ctx, RenderLaunch* a) {
    if (a->preset != RT_PRESET_GPU) return RT_OK;
    const size_t n = (size_t)a->n_blocks * 256 * (size_t)a->split * 3;
    if (n > ctx->csum_cap) {
        if (ctx->d_csum) RT_HIP(hipFree(ctx->d_csum));
        ctx->d_csum = nullptr;
        ctx->csum_cap = 0;
        RT_HIP(hipMalloc(&ctx->d_csum, sizeof(float) * n));
        ctx->csum_cap = n;
    }
    if (!ctx->d_work) RT_HIP(hipMalloc(&ctx->d_work, sizeof(unsigned long long)));
    a->csum = ctx->d_csum;
    a->work = ctx->d_work;
    // the camera rays' rectangle masks of k_render_pq's table route: four 16x4 rectangles per block
    const size_t words = (size_t)a->n_blocks * 4 * kRenderCullWords;
    if (words > ctx->cull_cap) {
        if (ctx->d_cull) RT_HIP(hipFree(ctx->d_cull));
        ctx->d_cull = nullptr;
        ctx->cull_cap = 0;
        RT_HIP(hipMalloc(&ctx->d_cull, sizeof(unsigned long long) * words));
        ctx->cull_cap = words;
    }
    a->cull = ctx->d_cull;
    return RT_OK;
}
}  // namespace rt

int rt::ensure_blocks_impl(rt_ctx* ctx, const std::vector<rt::BlockDesc>& blocks) {
    if ((int)blocks.size() > ctx->blocks_cap) {
        if (ctx->d_blocks) RT_HIP(hipFree(ctx->d_blocks));
        ctx->d_blocks = nullptr;
        ctx->blocks_cap = 0;
        RT_HIP(hipMalloc(&ctx->d_blocks, sizeof(rt::BlockDesc) * blocks.size()));
        ctx->blocks_cap = (int)blocks.size();
    }
    if (!blocks.empty())
        RT_HIP(hipMemcpy(ctx->d_blocks, blocks.data(), sizeof(rt::BlockDesc) * blocks.size(),
                         hipMemcpyHostToDevice));
    ctx->n_blocks = (int)blocks.size();
    return RT_OK;
}

namespace {

int check_params(const rt_params* p) {
    if (!p) return fail(RT_E_INVALID, "params is NULL");
    if (p->width <= 0 || p->height <= 0) return fail(RT_E_INVALID, "bad image size %dx%d", p->width, p->height);
    if (p->spp <= 0) return fail(RT_E_INVALID, "spp must be > 0");
    if (p->max_bounces < 0) return fail(RT_E_INVALID, "max_bounces must be >= 0");
    if (p->preset != RT_PRESET_CPU && p->preset != RT_PRESET_GPU) return fail(RT_E_INVALID, "bad preset %d", p->preset);
    if (p->sampler != RT_SAMPLER_UNIFORM && p->sampler != RT_SAMPLER_COSINE)
        return fail(RT_E_INVALID, "bad sampler %d", p->sampler);
    if (p->hit_rule != RT_HIT_RULE_CPU && p->hit_rule != RT_HIT_RULE_GPU)
        return fail(RT_E_INVALID, "bad hit_rule %d", p->hit_rule);
    if (p->preset == RT_PRESET_CPU && p->max_bounces > 2)
        return fail(RT_E_UNSUPPORTED, "CPU preset supports max_bounces <= 2 (got %d)", p->max_bounces);
    if (p->preset == RT_PRESET_GPU && p->max_bounces < 1)
        return fail(RT_E_INVALID, "GPU preset needs max_bounces >= 1");
    const int split = p->spp_split <= 0 ? 1 : p->spp_split;
    if (split > 64 || (split & (split - 1)) != 0)
        return fail(RT_E_INVALID, "spp_split must be a power of two <= 64 (got %d)", p->spp_split);
    if (p->spp % split != 0) return fail(RT_E_INVALID, "spp_split %d does not divide spp %d", split, p->spp);
    if ((int64_t)p->width * (int64_t)p->height > (int64_t)1 << 31)
        return fail(RT_E_INVALID, "image too large");
    return RT_OK;
}


void isect_record(const float* v, float4* out);

// The bounce-ray candidate table of a scene for hit rule `rule` (rt_ctab.cpp), built and
// uploaded once, on the first render that will take it (ctab_wanted: the launchers' own
// predicates); rule 0 serves t_scale >= kCtabTsMin.  A lazily built cache of the scene
// (hence the const_cast), guarded by the scene's mutex.  RT_CTAB=0 leaves the bounce casts on
// the image's masks (A/B builds).  The table is an accelerator, never required: a scene it
// cannot be built or uploaded for (host build refused, device memory short) keeps the image,
// and the render goes on (RT_CTAB_TEST_FAIL=1 forces the upload failure, for the tests).
}  // namespace
namespace rt {
bool ctab_wanted(const rt_scene* sc, const rt_camera* cam, const rt_params* p, int user) {
    const DeviceScene& d = sc->dev;
    if (d.mf_frag == nullptr || d.n_surf <= 0 || d.n_tri > 64 * kCtabMaxWords || scene_uses_bvh(sc)) return false;
    if (!filter_usable(d, cam->pos[0], cam->pos[1], cam->pos[2], p->t_scale)) return false;
    const float cb = d.mf_bound;
    const bool cam_in = fabsf(cam->pos[0]) <= cb && fabsf(cam->pos[1]) <= cb && fabsf(cam->pos[2]) <= cb;
    const bool t_ok = p->t_scale > 0.0f && p->t_scale <= kFiltMaxTScale;
    // the launch's pitch rotation is the identity (make_launch's cos_x / sin_x)
    const bool pitch0 = (float)cos((double)cam->yaw_x) == 1.0f && (float)sin((double)cam->yaw_x) == 0.0f;
    switch (user) {
        case kCtabForRender:  // launch_render_t: k_render_ps<.., CT> (CPU preset), k_render_pq<.., CT> (GPU)
            if (p->preset == RT_PRESET_CPU) return d.n_tri <= 64;
            return cam_in && t_ok && pitch0;
        case kCtabForDqn:  // launch_dqn_bounce: dqn_mf > 0
            return cam_in && t_ok;
        case kCtabForSarsa:  // k_sarsa_render_pq<.., CT> (built, off by default: RT_SARSA_CTAB)
            return sarsa_ctab_compiled() && t_ok;
    }
    return false;
}

int scene_ensure_ctab(const rt_scene* scene, int rule, float t_scale, bool wanted) {
    rt_scene* sc = const_cast<rt_scene*>(scene);
    if (rule != 0 && rule != 1) return RT_OK;
    if (!wanted || (rule == 0 && !(t_scale >= kCtabTsMin))) return RT_OK;
    std::lock_guard<std::mutex> lock(sc->ctab_mu);
    if (sc->ctab_tried[rule]) return RT_OK;
    sc->ctab_tried[rule] = true;
    static const bool ctab_on = getenv("RT_CTAB") == nullptr || atoi(getenv("RT_CTAB")) != 0;
    const int n = sc->dev.n_tri, n_surf = sc->dev.n_surf;
    if (!ctab_on || sc->dev.mf_frag == nullptr || n > 64 * kCtabMaxWords || n_surf <= 0) return RT_OK;
    std::vector<float4> isect((size_t)n * kIsectF4);
    for (int i = 0; i < n; ++i) isect_record(sc->tri.data() + (size_t)i * 9, &isect[(size_t)i * 3]);
    CtabHost ct;
    const auto t0 = std::chrono::steady_clock::now();
    if (!ctab_build(isect.data(), n, n_surf, (double)sc->dev.mf_bound, rule, kCtabTsMin, &ct)) return RT_OK;
    int rc = set_device(sc->ctx);
    if (rc != RT_OK) return rc;
    unsigned long long *dm = nullptr, *dd = nullptr, *dc = nullptr;
    uint16_t* dg = nullptr;
    float4* dt = nullptr;
    const char* force = getenv("RT_CTAB_TEST_FAIL");
    hipError_t e = (force && atoi(force) != 0) ? hipErrorOutOfMemory : hipSuccess;
    if (e == hipSuccess) e = hipMalloc(&dm, sizeof(uint64_t) * ct.masks.size());
    if (e == hipSuccess) e = hipMalloc(&dd, sizeof(uint64_t) * ct.gdict.size());
    if (e == hipSuccess) e = hipMalloc(&dg, sizeof(uint16_t) * ct.gid.size());
    if (e == hipSuccess) e = hipMalloc(&dc, sizeof(uint64_t) * ct.cop.size());
    if (e == hipSuccess) e = hipMalloc(&dt, sizeof(float4) * ct.tri.size());
    if (e == hipSuccess) e = hipMemcpy(dm, ct.masks.data(), sizeof(uint64_t) * ct.masks.size(), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(dd, ct.gdict.data(), sizeof(uint64_t) * ct.gdict.size(), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(dg, ct.gid.data(), sizeof(uint16_t) * ct.gid.size(), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(dc, ct.cop.data(), sizeof(uint64_t) * ct.cop.size(), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(dt, ct.tri.data(), sizeof(float4) * ct.tri.size(), hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        if (dd) (void)hipFree(dd);
        if (dm) (void)hipFree(dm);
        if (dg) (void)hipFree(dg);
        if (dc) (void)hipFree(dc);
        if (dt) (void)hipFree(dt);
        (void)hipGetLastError();  // the failed allocation must not fail the render's own launches
        static std::atomic<bool> warned{false};
        if (!warned.exchange(true))
            fprintf(stderr, "rtmi: candidate table upload failed (%s); the bounce casts stay on the matrix-core image\n",
                    hipGetErrorString(e));
        return RT_OK;
    }
    CtabDev& t = sc->dev.ctab[rule];
    t.masks = dm;
    t.gdict = dd;
    t.gid = dg;
    t.cop = dc;
    t.tri = dt;
    t.h = ct.h_run;
    t.ts_min = ct.ts_min;
    t.cop_th = ct.cop_th;
    t.words = ct.words;
    t.bins = kCtabBins;
    t.graze_n = kCtabGraze;
    t.gflag = ct.gflag;
    t.n_gdict = (int)(ct.gdict.size() / (size_t)ct.words);
    sc->ctab_build_s[rule] = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    sc->ctab_bytes[rule] = sizeof(uint64_t) * (ct.masks.size() + ct.gdict.size() + ct.cop.size()) +
                           sizeof(uint16_t) * ct.gid.size() + sizeof(float4) * ct.tri.size();
    return RT_OK;
}
}  // namespace rt
namespace {

rt::RenderLaunch make_launch(const rt_scene* scene, const rt_camera* cam, const rt_params* p) {
    rt::RenderLaunch a;
    memset(&a, 0, sizeof(a));
    a.scene = launch_scene(scene);
    a.width = p->width;
    a.height = p->height;
    a.spp = p->spp;
    a.max_bounces = p->max_bounces;
    a.split = p->spp_split <= 0 ? 1 : p->spp_split;
    a.split_log2 = 0;
    while ((1 << a.split_log2) < a.split) ++a.split_log2;
    a.per_chunk = p->spp / a.split;
    a.preset = p->preset;
    a.sampler = p->sampler;
    a.hit_rule = p->hit_rule;
    a.seed_lo = (uint32_t)p->seed;
    a.seed_hi = (uint32_t)(p->seed >> 32);
    a.t_scale = p->t_scale;
    a.env_light = p->env_light;
    a.cam_x = cam->pos[0];
    a.cam_y = cam->pos[1];
    a.cam_z = cam->pos[2];
    // Ray::rotate_ray's cos(yaw)/sin(yaw): evaluated once per frame on the host
    a.cos_y = (float)cos((double)cam->yaw_y);
    a.sin_y = (float)sin((double)cam->yaw_y);
    a.cos_x = (float)cos((double)cam->yaw_x);
    a.sin_x = (float)sin((double)cam->yaw_x);
    a.use_filter = rt::filter_usable(a.scene, a.cam_x, a.cam_y, a.cam_z, a.t_scale);
    return a;
}

// Hit-test record of one triangle (v = v0, v1, v2): {v0, c0}, {e1, 0}, {e2, 0} with
// c0 = m11*m22 - m21*m12 of [-D | e1 | e2] (rt_internal.hpp, kIsectF4).
void isect_record(const float* v, float4* out) {
    const float e1x = v[3] - v[0], e1y = v[4] - v[1], e1z = v[5] - v[2];
    const float e2x = v[6] - v[0], e2y = v[7] - v[1], e2z = v[8] - v[2];
    const float c0 = e1y * e2z - e2y * e1z;
    out[0] = make_float4(v[0], v[1], v[2], c0);
    out[1] = make_float4(e1x, e1y, e1z, 0.0f);
    out[2] = make_float4(e2x, e2y, e2z, 0.0f);
}

// Origin bound of the filter records of a scene: every surface point, plus room for a
// camera outside the scene (a camera beyond it gets the single-phase scan).
double filter_origin_bound(const float* v, size_t n_floats) {
    double vmax = 0.0;
    for (size_t k = 0; k < n_floats; ++k) vmax = fmax(vmax, fabs((double)v[k]));
    return fmax(8.0, 2.0 * vmax + 1.0);
}

// float >= x (x finite, >= 0)
float round_up(double x) {
    const float f = (float)x;
    return ((double)f >= x) ? f : nextafterf(f, INFINITY);
}

// Filter record of one triangle for closest_hit_filtered (rt_trace.hpp; layout in
// rt_internal.hpp).  The filter may reject a (ray, triangle) pair only if the exact
// test must fail, so its margins bound the difference between the two evaluations of
// each quantity, for |d_i| <= 2, |o_i| <= obound, t_scale <= kFiltMaxTScale.  With
// u = 2^-24, both the exact float Cramer evaluation (GLM order, incl. the rounding of
// b = o - v0 and of -t_scale*d) and the FMA evaluation on the double-rounded records
// are within 16u of the sum of the absolute values of the products involved:
//   A = d.N:           S_A = 2 M,            M = sum_i |e1_j e2_k| + |e1_k e2_j|
//   T = w0 - o.N:      S_T = B M,            B = obound + max_i |v0_i|
//   U = e2.R - d.G2:   S_U = 2 * 2 B |e2|_1  (R = d x o)
//   V = -e1.R + d.G1:  S_V = 2 * 2 B |e1|_1
// (all scaled by 1/t_scale where the exact evaluation carries t_scale).  The margins
// use c = 2^-16 = 256u, 16x that, plus an absolute floor F = 2^-90 that keeps a
// rejected u, v, t away from the underflow to -0 (which would pass ">= 0"):
//   eA = c S_A + F                          sign of A certain when |A~| > eA
//   EW = 2 (c S_U + c S_V + eA) + F         u < 0, v < 0 or u + v > 1 certain
//   ET = c S_T + 2 eps kFiltMaxTScale eA + F  t <= eps (RULE 0) / t < 0 certain
// Returns false outside the ranges where F stays negligible (huge coordinates).
bool build_filter(const float4& P0, const float4& P1, const float4& P2, double obound, float4* out) {
    const double v0[3] = {P0.x, P0.y, P0.z};
    const double a[3] = {P1.x, P1.y, P1.z};  // e1
    const double b[3] = {P2.x, P2.y, P2.z};  // e2
    double N[3], G1[3], G2[3], M = 0.0, vmax = 0.0, n1 = 0.0, n2 = 0.0;
    for (int i = 0; i < 3; ++i) {
        const int j = (i + 1) % 3, k = (i + 2) % 3;
        N[i] = a[j] * b[k] - a[k] * b[j];
        M += fabs(a[j] * b[k]) + fabs(a[k] * b[j]);
        G1[i] = v0[j] * a[k] - v0[k] * a[j];
        G2[i] = v0[j] * b[k] - v0[k] * b[j];
        vmax = fmax(vmax, fabs(v0[i]));
        n1 += fabs(a[i]);
        n2 += fabs(b[i]);
    }
    const float Nf[3] = {(float)N[0], (float)N[1], (float)N[2]};
    const double w0 = v0[0] * Nf[0] + v0[1] * Nf[1] + v0[2] * Nf[2];
    const double B = obound + vmax;
    const double c = ldexp(1.0, -16), F = ldexp(1.0, -90), dinf = 2.0;
    const double eA = c * dinf * M + F;
    const double EW = 2.0 * (c * 2.0 * dinf * B * n2 + c * 2.0 * dinf * B * n1 + eA) + F;
    const double ET = c * B * M + 2.0 * 1e-5 * (double)rt::kFiltMaxTScale * eA + F;
    if (!(M < ldexp(1.0, 36)) || !(B < ldexp(1.0, 20)) || !std::isfinite(EW) || !std::isfinite(ET))
        return false;
    out[0] = make_float4(Nf[0], Nf[1], Nf[2], (float)w0);
    out[1] = make_float4(P2.x, P2.y, P2.z, round_up(eA));
    out[2] = make_float4((float)-G2[0], (float)-G2[1], (float)-G2[2], round_up(EW));
    out[3] = make_float4(-P1.x, -P1.y, -P1.z, round_up(ET));
    out[4] = make_float4((float)G1[0], (float)G1[1], (float)G1[2], 0.0f);
    return true;
}

// ---- matrix-core filter image (rt_internal.hpp, kMfRound; rt_trace.hpp, closest_hit_mf) ----

uint16_t bf16_rne(float f) {
    uint32_t u;
    memcpy(&u, &f, 4);
    u += 0x7fffu + ((u >> 16) & 1u);
    return (uint16_t)(u >> 16);
}

double bf16_value(uint16_t h) {
    const uint32_t u = (uint32_t)h << 16;
    float f;
    memcpy(&f, &u, 4);
    return (double)f;
}

// x = hi + lo + r with |r| <= 2^-16 (1 + 2^-7) |x|
void bf16_split(double x, uint16_t* hi, uint16_t* lo) {
    *hi = bf16_rne((float)x);
    *lo = bf16_rne((float)(x - bf16_value(*hi)));
}

// The four rows of one triangle over the features (d, o', R, 1), each scaled so that its
// margin is 1.  Error of the matrix-core evaluation of a row against its real value: the
// split drops at most 3.1 * 2^-16 of sum |f_i b_i| (hi*lo, lo*hi kept; lo*lo and the split
// remainders dropped), the fp32 accumulation of the 30 products adds <= 2^-18 of it
// (measured 5.3 * 2^-24, profiles/probe/r2_mfma_split_probe.log), the rounding of R and o'
// a few u: under 3.5 * 2^-16 S.  The exact float test is within 16u S = 2^-20 S
// (build_filter).  The margins are build_filter's at c = 2^-12 >= 4.5x their sum, with
// |d_i| <= dinf = kMfDirBound, B = mf_bound + max |v0_i| and the t test folded into
// T' = T - ets A (|o'_i| <= mf_bound + dinf ets_max, ets_max = eps kFiltMaxTScale):
//   S_A = dinf M,  S_U = 2 dinf B |e2|_1,  S_V = 2 dinf B |e1|_1,  S_T' <= (B + dinf ets_max) M
//   eA = c S_A + F,  EW = 2 (c S_U + c S_V + eA) + F,  ET = c S_T' + 2 ets_max eA + F
// Every error bound is relative to the row's own sum of |products|, so it scales with the
// row: A, U, V are scaled by alpha < 1/EW (W = A - U - V then too) and T' by beta < 1/ET,
// which puts the barycentric and t margins at (below) 1.  The sign test of A keeps its own
// threshold *rho >= alpha eA (<= 1/2, since EW >= 2 eA): one float per triangle, carried in
// the fragment's unused K entries (build_mf_image; closest_hit_mf, mf_drop).  A constant 1/2 in its place doubled
// the exact tests on complex_light_room, whose small triangles have eA << EW.
bool build_mf_rows(const float4& P0, const float4& P1, const float4& P2, double mf_bound, double rows[4][10],
                   float* rho) {
    const double v0[3] = {P0.x, P0.y, P0.z};
    const double a[3] = {P1.x, P1.y, P1.z};  // e1
    const double b[3] = {P2.x, P2.y, P2.z};  // e2
    double N[3], G1[3], G2[3], M = 0.0, vmax = 0.0, n1 = 0.0, n2 = 0.0;
    for (int i = 0; i < 3; ++i) {
        const int j = (i + 1) % 3, k = (i + 2) % 3;
        N[i] = a[j] * b[k] - a[k] * b[j];
        M += fabs(a[j] * b[k]) + fabs(a[k] * b[j]);
        G1[i] = v0[j] * a[k] - v0[k] * a[j];
        G2[i] = v0[j] * b[k] - v0[k] * b[j];
        vmax = fmax(vmax, fabs(v0[i]));
        n1 += fabs(a[i]);
        n2 += fabs(b[i]);
    }
    const double w0 = v0[0] * N[0] + v0[1] * N[1] + v0[2] * N[2];
    for (int r = 0; r < 4; ++r)
        for (int k = 0; k < 10; ++k) rows[r][k] = 0.0;
    for (int i = 0; i < 3; ++i) {
        rows[0][i] = N[i];          // A  = d.N
        rows[1][3 + i] = N[i];      // T' = o'.N + w0
        rows[2][i] = -G2[i];        // U  = -G2.d + e2.R
        rows[2][6 + i] = b[i];
        rows[3][i] = G1[i];         // V  = G1.d - e1.R
        rows[3][6 + i] = -a[i];
    }
    rows[1][9] = w0;
    const double B = mf_bound + vmax;
    const double c = ldexp(1.0, -12), F = ldexp(1.0, -90), dinf = (double)rt::kMfDirBound;
    const double ets_max = 1e-5 * (double)rt::kFiltMaxTScale;
    const double eA = c * dinf * M + F;
    const double EW = 2.0 * (c * 2.0 * dinf * B * n2 + c * 2.0 * dinf * B * n1 + eA) + F;
    const double ET = c * (B + dinf * ets_max) * M + 2.0 * ets_max * eA + F;
    if (!(M < ldexp(1.0, 36)) || !(B < ldexp(1.0, 20)) || !std::isfinite(EW) || !std::isfinite(ET)) return false;
    // (1 - 2^-20: the double rounding of the scale and the products stays below 1)
    const double alpha = (1.0 / EW) * (1.0 - ldexp(1.0, -20)), beta = (1.0 / ET) * (1.0 - ldexp(1.0, -20));
    if (!(alpha * eA <= 0.5) || !(alpha * EW < 1.0) || !(beta * ET < 1.0)) return false;
    *rho = round_up(alpha * eA * (1.0 + ldexp(1.0, -20)));
    for (int k = 0; k < 10; ++k) {
        rows[0][k] *= alpha;
        rows[1][k] *= beta;
        rows[2][k] *= alpha;
        rows[3][k] *= alpha;
    }
    return true;
}

// Device image of the matrix-core filter: frag (8 * rounds groups x 64 lanes x 8 bf16) and
// rho (8 * rounds groups x 4 slots); layout in rt_internal.hpp.
bool build_mf_image(const std::vector<float4>& isect, int n, double mf_bound, std::vector<uint16_t>* frag,
                    std::vector<float>* rho) {
    const int rounds = (n + rt::kMfRound - 1) / rt::kMfRound;
    const size_t groups = (size_t)rounds * rt::kMfGroupsPerRound;
    frag->assign(groups * 64 * 8, 0);
    rho->assign(groups * 4, 0.0f);
    for (int r = 0; r < rounds; ++r) {
        const int base = r * rt::kMfRound;
        const int cnt = std::min(rt::kMfRound, n - base);
        const int G = (cnt + 3) / 4;
        for (int g = 0; g < G; ++g) {
            const size_t gi = (size_t)r * rt::kMfGroupsPerRound + g;
            for (int s = 0; s < 4; ++s) {
                const int tl = s * G + (G - 1 - g);
                if (tl >= cnt) continue;  // pad slot: zero rows (masked off)
                const int t = base + tl;
                double rows[4][10];
                if (!build_mf_rows(isect[(size_t)t * 3], isect[(size_t)t * 3 + 1], isect[(size_t)t * 3 + 2],
                                   mf_bound, rows, &(*rho)[gi * 4 + s]))
                    return false;
                for (int i = 0; i < 4; ++i) {
                    uint16_t bh[10], bl[10];
                    for (int k = 0; k < 10; ++k) bf16_split(rows[i][k], &bh[k], &bl[k]);
                    // the K order of the ray operand (rt_internal.hpp)
                    const uint16_t kv[32] = {bh[0], bh[1], bh[2], bh[3], bh[4], bh[5], bh[6], bh[7],
                                             bh[8], bh[9], bh[0], bh[1], bh[2], bh[3], bh[4], bh[5],
                                             bh[6], bh[7], bh[8], bh[9], bl[0], bl[1], bl[2], bl[3],
                                             bl[4], bl[5], bl[6], bl[7], bl[8], bl[9], 0, 0};
                    const int row = 4 * s + i;
                    for (int p = 0; p < 4; ++p) {
                        const int lane = 16 * p + row;
                        for (int j = 0; j < 8; ++j) (*frag)[(gi * 64 + lane) * 8 + j] = kv[8 * p + j];
                    }
                }
                // the slot's sign-test threshold rides in the fragment's unused k = 30, 31 of
                // row 4 s (lane 48 + 4 s, its 4th dword; the ray operand is 0 there, so the
                // MFMA ignores it): closest_hit_mf reads it with v_readlane
                uint32_t rb;
                memcpy(&rb, &(*rho)[gi * 4 + s], 4);
                (*frag)[(gi * 64 + 48 + 4 * s) * 8 + 6] = (uint16_t)(rb & 0xffffu);
                (*frag)[(gi * 64 + 48 + 4 * s) * 8 + 7] = (uint16_t)(rb >> 16);
            }
            // and the group's largest threshold (lane 49: RT_MF_RHO_GROUP builds)
            float gmax = 0.0f;
            for (int s = 0; s < 4; ++s) gmax = std::max(gmax, (*rho)[gi * 4 + s]);
            uint32_t gb;
            memcpy(&gb, &gmax, 4);
            (*frag)[(gi * 64 + 49) * 8 + 6] = (uint16_t)(gb & 0xffffu);
            (*frag)[(gi * 64 + 49) * 8 + 7] = (uint16_t)(gb >> 16);
        }
    }
    return true;
}

}  // namespace

namespace rt {
// shared with the SARSA host code (rt_sarsa_host.cpp)
RenderLaunch render_launch(const rt_scene* scene, const rt_camera* cam, const rt_params* p) {
    return make_launch(scene, cam, p);
}
}  // namespace rt

extern "C" {

const char* rt_last_error(void) { return g_err.c_str(); }

int rt_params_default(int preset, rt_params* p) {
    if (!p) return fail(RT_E_INVALID, "params is NULL");
    memset(p, 0, sizeof(*p));
    if (preset == RT_PRESET_CPU) {
        p->width = 512; p->height = 512; p->spp = 16; p->max_bounces = 2;
        p->hit_rule = RT_HIT_RULE_CPU;
    } else if (preset == RT_PRESET_GPU) {
        p->width = 720; p->height = 720; p->spp = 32; p->max_bounces = 80;
        p->hit_rule = RT_HIT_RULE_GPU;
    } else {
        return fail(RT_E_INVALID, "bad preset %d", preset);
    }
    p->preset = preset;
    p->sampler = RT_SAMPLER_UNIFORM;
    p->spp_split = 1;
    p->seed = 1984;
    p->env_light = 0.0f;
    p->t_scale = (float)p->height;
    return RT_OK;
}

int rt_ctx_create(int device_ordinal, rt_ctx** out) {
    if (!out) return fail(RT_E_INVALID, "out is NULL");
    *out = nullptr;
    int n = 0;
    RT_HIP(hipGetDeviceCount(&n));
    if (device_ordinal < 0 || device_ordinal >= n)
        return fail(RT_E_INVALID, "device %d out of range (%d devices)", device_ordinal, n);
    rt_ctx* c = new (std::nothrow) rt_ctx();
    if (!c) return fail(RT_E_NOMEM, "out of host memory");
    c->device = device_ordinal;
    int rc = set_device(c);
    if (rc != RT_OK) {
        delete c;
        return rc;
    }
    *out = c;
    return RT_OK;
}

int rt_ctx_destroy(rt_ctx* ctx) {
    if (!ctx) return RT_OK;
    (void)hipSetDevice(ctx->device);
    rt::release_dqn_workspace(ctx);
    if (ctx->d_blocks) (void)hipFree(ctx->d_blocks);
    if (ctx->d_cull) (void)hipFree(ctx->d_cull);
    if (ctx->d_csum) (void)hipFree(ctx->d_csum);
    if (ctx->d_work) (void)hipFree(ctx->d_work);
    delete ctx;
    return RT_OK;
}

int rt_scene_create(rt_ctx* ctx, const float* tri_v, const float* albedo, int n_surf,
                    const float* light_v, const float* emission, const int32_t* light_group,
                    int n_light, rt_scene** out) {
    using rt::f3;
    using rt::make3;
    if (!ctx || !out) return fail(RT_E_INVALID, "ctx/out is NULL");
    *out = nullptr;
    if (n_surf < 0 || n_light < 0 || n_surf + n_light <= 0) return fail(RT_E_INVALID, "empty scene");
    if ((n_surf > 0 && (!tri_v || !albedo)) || (n_light > 0 && (!light_v || !emission || !light_group)))
        return fail(RT_E_INVALID, "missing scene arrays");
    if (n_surf + n_light > (1 << 24)) return fail(RT_E_INVALID, "too many triangles");
    int rc = set_device(ctx);
    if (rc != RT_OK) return rc;
    const int n = n_surf + n_light;
    std::vector<float4> isect((size_t)n * rt::kIsectF4);
    std::vector<float4> shade((size_t)n * rt::kShadeF4);
    std::vector<int32_t> code_cpu(n), code_gpu(n);
    rt_scene* sc = new (std::nothrow) rt_scene();
    if (!sc) return fail(RT_E_NOMEM, "out of host memory");
    sc->ctx = ctx;
    sc->n_surf = n_surf;
    sc->n_light = n_light;
    sc->normals.resize((size_t)n * 3);
    sc->tri.resize((size_t)n * 9);
    if (n_surf > 0) {
        memcpy(sc->tri.data(), tri_v, sizeof(float) * 9 * (size_t)n_surf);
        sc->albedo.assign(albedo, albedo + 3 * (size_t)n_surf);
    }
    if (n_light > 0) {
        memcpy(sc->tri.data() + 9 * (size_t)n_surf, light_v, sizeof(float) * 9 * (size_t)n_light);
        sc->emission.assign(emission, emission + 3 * (size_t)n_light);
    }
    for (int i = 0; i < n; ++i) {
        const bool is_light = i >= n_surf;
        const int j = is_light ? i - n_surf : i;
        const float* v = is_light ? light_v + (size_t)j * 9 : tri_v + (size_t)j * 9;
        isect_record(v, &isect[(size_t)i * 3]);
        const f3 v0 = make3(v[0], v[1], v[2]);
        const f3 e1 = make3(isect[(size_t)i * 3 + 1].x, isect[(size_t)i * 3 + 1].y, isect[(size_t)i * 3 + 1].z);
        const f3 e2 = make3(isect[(size_t)i * 3 + 2].x, isect[(size_t)i * 3 + 2].y, isect[(size_t)i * 3 + 2].z);
        (void)v0;
        // Triangle::compute_and_set_normal: normalize(cross(e2, e1))
        const f3 N = rt::normalize(rt::cross(e2, e1));
        f3 T, B;
        rt::normal_frame(N, &T, &B);
        sc->normals[(size_t)i * 3 + 0] = N.x;
        sc->normals[(size_t)i * 3 + 1] = N.y;
        sc->normals[(size_t)i * 3 + 2] = N.z;
        shade[(size_t)i * 5 + 0] = make_float4(N.x, N.y, N.z, 0.0f);
        shade[(size_t)i * 5 + 1] = make_float4(T.x, T.y, T.z, 0.0f);
        shade[(size_t)i * 5 + 2] = make_float4(B.x, B.y, B.z, 0.0f);
        if (is_light) {
            const float* e = emission + (size_t)j * 3;
            shade[(size_t)i * 5 + 3] = make_float4(e[0], e[1], e[2], 0.0f);
            shade[(size_t)i * 5 + 4] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            code_cpu[i] = (int32_t)((RT_HIT_TYPE_LIGHT << 30) | (uint32_t)light_group[j]);
            code_gpu[i] = (int32_t)((RT_HIT_TYPE_LIGHT << 30) | (uint32_t)j);
        } else {
            const float* al = albedo + (size_t)j * 3;
            // BRDF = reflectance / M_PI (default_path_tracing.cpp:95)
            shade[(size_t)i * 5 + 3] = make_float4(al[0] / rt::kPi, al[1] / rt::kPi, al[2] / rt::kPi, 0.0f);
            shade[(size_t)i * 5 + 4] = make_float4(al[0], al[1], al[2], 0.0f);
            code_cpu[i] = code_gpu[i] = (int32_t)((RT_HIT_TYPE_SURFACE << 30) | (uint32_t)j);
        }
    }
    // Filter records (two-phase hit test).  Origin bound: every surface point, plus room
    // for a camera outside the scene (a camera beyond it gets the single-phase scan).
    const double obound = filter_origin_bound(sc->tri.data(), sc->tri.size());
    // padded to an even triangle count (phase 1 runs in pairs; the pad is masked off)
    std::vector<float4> filt((size_t)((n + 1) & ~1) * rt::kFiltF4, make_float4(0.0f, 0.0f, 0.0f, 0.0f));
    bool filt_ok = true;
    for (int i = 0; i < n && filt_ok; ++i)
        filt_ok = build_filter(isect[(size_t)i * 3 + 0], isect[(size_t)i * 3 + 1], isect[(size_t)i * 3 + 2],
                               obound, &filt[(size_t)i * rt::kFiltF4]);
    // matrix-core filter of rays from surface points: origins within the scene's box + 1
    double vmax_scene = 0.0;
    for (float x : sc->tri) vmax_scene = fmax(vmax_scene, fabs((double)x));
    // the kernel compares with this float; the margins are built for it
    const double mf_bound = (double)round_up(vmax_scene * (1.0 + ldexp(1.0, -10)) + ldexp(1.0, -10));
    std::vector<uint16_t> mf_frag;
    std::vector<float> mf_rho;
    const bool mf_ok = filt_ok && build_mf_image(isect, n, mf_bound, &mf_frag, &mf_rho);
    sc->dev.n_surf = n_surf;
    sc->dev.n_tri = n;
    sc->dev.origin_bound = (float)obound;
    sc->dev.mf_bound = (float)mf_bound;
    auto cleanup = [&]() {
        if (sc->dev.isect) (void)hipFree(sc->dev.isect);
        if (sc->dev.shade) (void)hipFree(sc->dev.shade);
        if (sc->dev.filt) (void)hipFree(sc->dev.filt);
        if (sc->dev.mf_frag) (void)hipFree(sc->dev.mf_frag);
        if (sc->dev.code_cpu) (void)hipFree(sc->dev.code_cpu);
        if (sc->dev.code_gpu) (void)hipFree(sc->dev.code_gpu);
        delete sc;
    };
    hipError_t e = hipMalloc(&sc->dev.isect, sizeof(float4) * isect.size());
    if (e == hipSuccess) e = hipMalloc(&sc->dev.shade, sizeof(float4) * shade.size());
    if (e == hipSuccess) e = hipMalloc(&sc->dev.code_cpu, sizeof(int32_t) * n);
    if (e == hipSuccess) e = hipMalloc(&sc->dev.code_gpu, sizeof(int32_t) * n);
    if (e == hipSuccess) e = hipMemcpy(sc->dev.isect, isect.data(), sizeof(float4) * isect.size(), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(sc->dev.shade, shade.data(), sizeof(float4) * shade.size(), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(sc->dev.code_cpu, code_cpu.data(), sizeof(int32_t) * n, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(sc->dev.code_gpu, code_gpu.data(), sizeof(int32_t) * n, hipMemcpyHostToDevice);
    if (e == hipSuccess && filt_ok) {
        e = hipMalloc(&sc->dev.filt, sizeof(float4) * filt.size());
        if (e == hipSuccess)
            e = hipMemcpy(sc->dev.filt, filt.data(), sizeof(float4) * filt.size(), hipMemcpyHostToDevice);
    }
    if (e == hipSuccess && mf_ok) {
        e = hipMalloc(&sc->dev.mf_frag, sizeof(uint16_t) * mf_frag.size());
        if (e == hipSuccess)
            e = hipMemcpy(sc->dev.mf_frag, mf_frag.data(), sizeof(uint16_t) * mf_frag.size(), hipMemcpyHostToDevice);

    }
    if (e != hipSuccess) {
        cleanup();
        return fail(RT_E_HIP, "scene upload failed: %s", hipGetErrorString(e));
    }
    // large scenes: the exact BVH path (a scene it cannot be built for keeps the scan)
    if (n > RT_BVH_AUTO_MIN && scene_build_bvh(sc) != RT_OK) scene_free_bvh(sc);
    *out = sc;
    return RT_OK;
}

int rt_scene_destroy(rt_scene* scene) {
    if (!scene) return RT_OK;
    (void)hipSetDevice(scene->ctx->device);
    (void)hipFree(scene->dev.isect);
    (void)hipFree(scene->dev.shade);
    (void)hipFree(scene->dev.code_cpu);
    (void)hipFree(scene->dev.code_gpu);
    if (scene->dev.filt) (void)hipFree(scene->dev.filt);
    if (scene->dev.mf_frag) (void)hipFree(scene->dev.mf_frag);
    for (const rt::CtabDev& t : scene->dev.ctab) {
        if (t.masks) (void)hipFree(const_cast<unsigned long long*>(t.masks));
        if (t.gdict) (void)hipFree(const_cast<unsigned long long*>(t.gdict));
        if (t.gid) (void)hipFree(const_cast<uint16_t*>(t.gid));
        if (t.cop) (void)hipFree(const_cast<unsigned long long*>(t.cop));
        if (t.tri) (void)hipFree(const_cast<float4*>(t.tri));
    }
    scene_free_bvh(scene);
    delete scene;
    return RT_OK;
}

int rt_scene_ctab_info(const rt_scene* scene, int hit_rule, int* built, double* build_s, uint64_t* bytes) {
    if (!scene) return fail(RT_E_INVALID, "scene is NULL");
    if (hit_rule != RT_HIT_RULE_CPU && hit_rule != RT_HIT_RULE_GPU) return fail(RT_E_INVALID, "bad hit_rule %d", hit_rule);
    std::lock_guard<std::mutex> lock(const_cast<rt_scene*>(scene)->ctab_mu);
    const bool on = scene->dev.ctab[hit_rule].masks != nullptr;
    if (built) *built = on ? 1 : 0;
    if (build_s) *build_s = on ? scene->ctab_build_s[hit_rule] : 0.0;
    if (bytes) *bytes = on ? scene->ctab_bytes[hit_rule] : 0;
    return RT_OK;
}

int rt_scene_set_accel(rt_scene* scene, int mode) {
    if (!scene) return fail(RT_E_INVALID, "scene is NULL");
    if (mode != RT_ACCEL_AUTO && mode != RT_ACCEL_SCAN && mode != RT_ACCEL_BVH)
        return fail(RT_E_INVALID, "bad accel mode %d", mode);
    int rc = set_device(scene->ctx);
    if (rc != RT_OK) return rc;
    if (mode == RT_ACCEL_BVH || (mode == RT_ACCEL_AUTO && scene->dev.n_tri > RT_BVH_AUTO_MIN)) {
        rc = scene_build_bvh(scene);
        if (rc != RT_OK) return fail(rc, "BVH build failed (scene outside the filter's ranges?)");
    }
    scene->accel = mode;
    return RT_OK;
}

int rt_ctab_candidates(const float* tri_v, int n, int n_surf, int hit_rule, const int32_t* surf, const float* orig,
                       const float* dir, int n_rays, uint64_t* masks, int64_t* stats) {
    if (!tri_v || n <= 0 || n > 64 * rt::kCtabMaxWords || n_surf <= 0 || n_surf > n)
        return fail(RT_E_INVALID, "need 1 to %d triangles", 64 * rt::kCtabMaxWords);
    if (hit_rule != RT_HIT_RULE_CPU && hit_rule != RT_HIT_RULE_GPU) return fail(RT_E_INVALID, "bad hit rule %d", hit_rule);
    if (n_rays < 0 || (n_rays > 0 && (!surf || !orig || !dir || !masks))) return fail(RT_E_INVALID, "missing ray arrays");
    std::vector<float4> isect((size_t)n * rt::kIsectF4);
    double vmax = 0.0;
    for (int i = 0; i < n; ++i) isect_record(tri_v + (size_t)i * 9, &isect[(size_t)i * 3]);
    for (int k = 0; k < n * 9; ++k) vmax = fmax(vmax, fabs((double)tri_v[k]));
    // the scene's origin bound, as rt_scene_create gives the matrix-core image and the table
    const double mf_bound = (double)round_up(vmax * (1.0 + ldexp(1.0, -10)) + ldexp(1.0, -10));
    rt::CtabHost h;
    if (!rt::ctab_build(isect.data(), n, n_surf, mf_bound, hit_rule, rt::kCtabTsMin, &h))
        return fail(RT_E_UNSUPPORTED, "candidate table build failed");
    for (int r = 0; r < n_rays; ++r)
        rt::ctab_lookup(h, surf[r], orig + (size_t)r * 3, dir + (size_t)r * 3, masks + (size_t)r * h.words);
    if (stats) {
        std::vector<int64_t> pc(h.gdict.size() / (size_t)h.words, 0);  // bits of each grazing dictionary mask
        for (size_t e = 0; e < h.gdict.size(); ++e) pc[e / (size_t)h.words] += __builtin_popcountll(h.gdict[e]);
        int64_t bits = 0;
        for (uint64_t m : h.masks) bits += __builtin_popcountll(m);
        int64_t gbits = 0;
        for (uint16_t i : h.gid) gbits += pc[i];
        stats[0] = h.n_patch;
        stats[1] = h.patches_all;
        stats[2] = bits;
        stats[3] = gbits;
    }
    return RT_OK;
}

int rt_bvh_check(const float* tri_v, int n, int64_t* stats) {
    if (!tri_v || n <= 0) return fail(RT_E_INVALID, "no triangles");
    std::vector<float4> isect((size_t)n * rt::kIsectF4);
    for (int i = 0; i < n; ++i) isect_record(tri_v + (size_t)i * 9, &isect[(size_t)i * 3]);
    rt::BvhHost h;
    if (!rt::bvh_build(isect.data(), n, &h)) return fail(RT_E_UNSUPPORTED, "BVH build failed");
    const std::string err = rt::bvh_check(isect.data(), n, h);
    if (stats) {
        int64_t leaves = 0;
        for (int k = 0; k < h.n_nodes; ++k) {
            int cnt;
            memcpy(&cnt, &h.nodes[(size_t)k * 2 + 1].w, 4);
            leaves += cnt > 0;
        }
        stats[0] = h.n_nodes;
        stats[1] = h.depth;
        stats[2] = (int64_t)h.dlist.size();
        stats[3] = leaves;
    }
    if (!err.empty()) return fail(RT_E_INTERNAL, "BVH invariant: %s", err.c_str());
    return RT_OK;
}

int rt_scene_accel_info(const rt_scene* scene, int* n_nodes, int* depth, int64_t* dir_entries) {
    if (!scene) return fail(RT_E_INVALID, "scene is NULL");
    if (n_nodes) *n_nodes = scene->has_bvh ? scene->bvh.n_nodes : 0;
    if (depth) *depth = scene->has_bvh ? scene->bvh.depth : 0;
    if (dir_entries) *dir_entries = scene->has_bvh ? (int64_t)scene->bvh.dlist.size() : 0;
    return RT_OK;
}

// RT_ISECT_BVH of rt_intersect_method: the BVH path whatever the scene's mode
static int intersect_bvh_host(rt_ctx* ctx, const rt_scene* scene, const float* orig, const float* dir, int n,
                              float t_scale, int hit_rule, float* out_t, int32_t* out_hit) {
    int rc = set_device(ctx);
    if (rc != RT_OK) return rc;
    // builds the BVH once if the scene has none yet (kept for later calls; rt_scene_set_accel
    // builds it up front); the scene's accel mode is not touched
    rc = scene_build_bvh(const_cast<rt_scene*>(scene));
    if (rc != RT_OK) return fail(rc, "BVH build failed");
    const rt::DeviceScene ds = launch_scene(scene, /*force_bvh=*/true);
    float *d_o = nullptr, *d_d = nullptr, *d_t = nullptr;
    int32_t* d_h = nullptr;
    const size_t b3 = sizeof(float) * 3 * (size_t)n;
    hipError_t e = hipMalloc(&d_o, b3);
    if (e == hipSuccess) e = hipMalloc(&d_d, b3);
    if (e == hipSuccess) e = hipMalloc(&d_t, sizeof(float) * (size_t)n);
    if (e == hipSuccess) e = hipMalloc(&d_h, sizeof(int32_t) * (size_t)n);
    if (e == hipSuccess) e = hipMemcpy(d_o, orig, b3, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(d_d, dir, b3, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = rt::launch_intersect_bvh(ds, d_o, d_d, n, t_scale, hit_rule, d_t, d_h, 0);
    if (e == hipSuccess) e = hipMemcpy(out_t, d_t, sizeof(float) * (size_t)n, hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(out_hit, d_h, sizeof(int32_t) * (size_t)n, hipMemcpyDeviceToHost);
    (void)hipFree(d_o);
    (void)hipFree(d_d);
    (void)hipFree(d_t);
    (void)hipFree(d_h);
    if (e != hipSuccess) return fail(RT_E_HIP, "rt_intersect_method(BVH): %s", hipGetErrorString(e));
    return RT_OK;
}

int rt_scene_normals(const rt_scene* scene, float* out) {
    if (!scene || !out) return fail(RT_E_INVALID, "scene/out is NULL");
    memcpy(out, scene->normals.data(), sizeof(float) * scene->normals.size());
    return RT_OK;
}

int rt_intersect_device(rt_ctx* ctx, const rt_scene* scene, const float* d_orig, const float* d_dir,
                        int n, float t_scale, int hit_rule, float* d_t, int32_t* d_hit, void* stream) {
    if (!ctx || !scene) return fail(RT_E_INVALID, "ctx/scene is NULL");
    if (n < 0) return fail(RT_E_INVALID, "n < 0");
    if (n > 0 && (!d_orig || !d_dir || !d_t || !d_hit)) return fail(RT_E_INVALID, "NULL buffer");
    if (hit_rule != RT_HIT_RULE_CPU && hit_rule != RT_HIT_RULE_GPU) return fail(RT_E_INVALID, "bad hit_rule");
    int rc = set_device(ctx);
    if (rc != RT_OK) return rc;
    if (scene_uses_bvh(scene)) {  // the BVH path checks each ray's range itself
        RT_HIP(rt::launch_intersect_bvh(launch_scene(scene), d_orig, d_dir, n, t_scale, hit_rule, d_t, d_hit,
                                        (hipStream_t)stream));
        return RT_OK;
    }
    // device rays of unknown range: the single-phase scan (no filter bounds to rely on)
    RT_HIP(rt::launch_intersect(scene->dev, d_orig, d_dir, n, t_scale, hit_rule, 0, d_t, d_hit,
                                (hipStream_t)stream));
    return RT_OK;
}

int rt_intersect(rt_ctx* ctx, const rt_scene* scene, const float* orig, const float* dir, int n,
                 float t_scale, int hit_rule, float* out_t, int32_t* out_hit) {
    if (!ctx || !scene) return fail(RT_E_INVALID, "ctx/scene is NULL");
    if (n < 0) return fail(RT_E_INVALID, "n < 0");
    if (n == 0) return RT_OK;
    if (!orig || !dir || !out_t || !out_hit) return fail(RT_E_INVALID, "NULL buffer");
    if (hit_rule != RT_HIT_RULE_CPU && hit_rule != RT_HIT_RULE_GPU) return fail(RT_E_INVALID, "bad hit_rule");
    int rc = set_device(ctx);
    if (rc != RT_OK) return rc;
    float *d_o = nullptr, *d_d = nullptr, *d_t = nullptr;
    int32_t* d_h = nullptr;
    const size_t b3 = sizeof(float) * 3 * (size_t)n;
    hipError_t e = hipMalloc(&d_o, b3);
    if (e == hipSuccess) e = hipMalloc(&d_d, b3);
    if (e == hipSuccess) e = hipMalloc(&d_t, sizeof(float) * (size_t)n);
    if (e == hipSuccess) e = hipMalloc(&d_h, sizeof(int32_t) * (size_t)n);
    if (e == hipSuccess) e = hipMemcpy(d_o, orig, b3, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(d_d, dir, b3, hipMemcpyHostToDevice);
    // the two-phase hit test when every ray is inside the filter's bounds
    float omax = 0.0f, dmax = 0.0f;
    for (size_t k = 0; k < 3 * (size_t)n; ++k) {
        omax = fmaxf(omax, fabsf(orig[k]));  // NaN: fmaxf keeps omax; NaN rays never reject
        dmax = fmaxf(dmax, fabsf(dir[k]));
    }
    const int use_filter = (dmax <= 2.0f) ? rt::filter_usable(scene->dev, omax, 0.0f, 0.0f, t_scale) : 0;
    if (e == hipSuccess) {
        if (scene_uses_bvh(scene))
            e = rt::launch_intersect_bvh(launch_scene(scene), d_o, d_d, n, t_scale, hit_rule, d_t, d_h, 0);
        else
            e = rt::launch_intersect(scene->dev, d_o, d_d, n, t_scale, hit_rule, use_filter, d_t, d_h, 0);
    }
    if (e == hipSuccess) e = hipMemcpy(out_t, d_t, sizeof(float) * (size_t)n, hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(out_hit, d_h, sizeof(int32_t) * (size_t)n, hipMemcpyDeviceToHost);
    (void)hipFree(d_o);
    (void)hipFree(d_d);
    (void)hipFree(d_t);
    (void)hipFree(d_h);
    if (e != hipSuccess) return fail(RT_E_HIP, "rt_intersect: %s", hipGetErrorString(e));
    return RT_OK;
}

int rt_intersect_method(rt_ctx* ctx, const rt_scene* scene, const float* orig, const float* dir, int n,
                        float t_scale, int hit_rule, int method, float* out_t, int32_t* out_hit,
                        int32_t* out_cand) {
    if (!ctx || !scene) return fail(RT_E_INVALID, "ctx/scene is NULL");
    if (n < 0) return fail(RT_E_INVALID, "n < 0");
    if (n == 0) return RT_OK;
    if (!orig || !dir || !out_t || !out_hit) return fail(RT_E_INVALID, "NULL buffer");
    if (hit_rule != RT_HIT_RULE_CPU && hit_rule != RT_HIT_RULE_GPU) return fail(RT_E_INVALID, "bad hit_rule");
    if (method == RT_ISECT_BVH) {
        if (out_cand) return fail(RT_E_INVALID, "out_cand needs RT_ISECT_MFMA");
        return intersect_bvh_host(ctx, scene, orig, dir, n, t_scale, hit_rule, out_t, out_hit);
    }
    if (method != RT_ISECT_SCAN && method != RT_ISECT_FILTER && method != RT_ISECT_MFMA)
        return fail(RT_E_INVALID, "bad method %d", method);
    if (out_cand && method != RT_ISECT_MFMA) return fail(RT_E_INVALID, "out_cand needs RT_ISECT_MFMA");
    if (method == RT_ISECT_MFMA && (!scene->dev.mf_frag || !(t_scale > 0.0f && t_scale <= rt::kFiltMaxTScale)))
        return fail(RT_E_UNSUPPORTED, "no matrix-core filter image for this scene / t_scale");
    if (method == RT_ISECT_FILTER) {
        float omax = 0.0f, dmax = 0.0f;
        for (size_t k = 0; k < 3 * (size_t)n; ++k) {
            omax = fmaxf(omax, fabsf(orig[k]));
            dmax = fmaxf(dmax, fabsf(dir[k]));
        }
        if (!(dmax <= 2.0f) || !rt::filter_usable(scene->dev, omax, 0.0f, 0.0f, t_scale))
            return fail(RT_E_UNSUPPORTED, "rays outside the filter's bounds");
    }
    int rc = set_device(ctx);
    if (rc != RT_OK) return rc;
    float *d_o = nullptr, *d_d = nullptr, *d_t = nullptr;
    int32_t *d_h = nullptr, *d_c = nullptr;
    const size_t b3 = sizeof(float) * 3 * (size_t)n;
    hipError_t e = hipMalloc(&d_o, b3);
    if (e == hipSuccess) e = hipMalloc(&d_d, b3);
    if (e == hipSuccess) e = hipMalloc(&d_t, sizeof(float) * (size_t)n);
    if (e == hipSuccess) e = hipMalloc(&d_h, sizeof(int32_t) * (size_t)n);
    if (e == hipSuccess && out_cand) e = hipMalloc(&d_c, sizeof(int32_t) * (size_t)n);
    if (e == hipSuccess) e = hipMemcpy(d_o, orig, b3, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(d_d, dir, b3, hipMemcpyHostToDevice);
    if (e == hipSuccess) {
        if (method == RT_ISECT_MFMA)
            e = rt::launch_intersect_mf(scene->dev, d_o, d_d, n, t_scale, hit_rule, d_t, d_h, d_c, 0);
        else
            e = rt::launch_intersect(scene->dev, d_o, d_d, n, t_scale, hit_rule, method == RT_ISECT_FILTER ? 1 : 0,
                                     d_t, d_h, 0);
    }
    if (e == hipSuccess) e = hipMemcpy(out_t, d_t, sizeof(float) * (size_t)n, hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(out_hit, d_h, sizeof(int32_t) * (size_t)n, hipMemcpyDeviceToHost);
    if (e == hipSuccess && out_cand) e = hipMemcpy(out_cand, d_c, sizeof(int32_t) * (size_t)n, hipMemcpyDeviceToHost);
    (void)hipFree(d_o);
    (void)hipFree(d_d);
    (void)hipFree(d_t);
    (void)hipFree(d_h);
    if (d_c) (void)hipFree(d_c);
    if (e != hipSuccess) return fail(RT_E_HIP, "rt_intersect_method: %s", hipGetErrorString(e));
    return RT_OK;
}

int rt_render(rt_ctx* ctx, const rt_scene* scene, const rt_camera* cam, const rt_params* params,
              int x0, int y0, int w, int h, float* out_rgb, uint64_t* out_ray_casts) {
    if (!ctx || !scene || !cam || !out_rgb) return fail(RT_E_INVALID, "NULL argument");
    int rc = check_params(params);
    if (rc != RT_OK) return rc;
    if (w <= 0 || h <= 0 || x0 < 0 || y0 < 0 || x0 + w > params->width || y0 + h > params->height)
        return fail(RT_E_INVALID, "rectangle outside the image");
    rc = set_device(ctx);
    if (rc != RT_OK) return rc;
    std::vector<rt::BlockDesc> blocks;
    for (int by = 0; by < h; by += 16)
        for (int bx = 0; bx < w; bx += 16) blocks.push_back({x0 + bx, y0 + by, bx, by});
    rt::BlockDesc* d_blocks = nullptr;
    float* d_out = nullptr;
    unsigned long long* d_casts = nullptr;
    const size_t out_bytes = sizeof(float) * 3 * (size_t)w * (size_t)h;
    rc = rt::scene_ensure_ctab(scene, params->hit_rule, params->t_scale,
                               rt::ctab_wanted(scene, cam, params, rt::kCtabForRender));
    if (rc != RT_OK) return rc;
    hipError_t e = hipMalloc(&d_blocks, sizeof(rt::BlockDesc) * blocks.size());
    if (e == hipSuccess) e = hipMalloc(&d_out, out_bytes);
    if (e == hipSuccess) e = hipMalloc(&d_casts, sizeof(unsigned long long));
    if (e == hipSuccess) e = hipMemset(d_casts, 0, sizeof(unsigned long long));
    if (e == hipSuccess)
        e = hipMemcpy(d_blocks, blocks.data(), sizeof(rt::BlockDesc) * blocks.size(), hipMemcpyHostToDevice);
    if (e == hipSuccess) {
        rt::RenderLaunch a = make_launch(scene, cam, params);
        a.blocks = d_blocks;
        a.n_blocks = (int)blocks.size();
        a.clip_x1 = x0 + w;
        a.clip_y1 = y0 + h;
        a.out_pitch = w;
        a.out = d_out;
        a.casts = d_casts;
        if (rt::ctx_chunks(ctx, &a) != RT_OK) e = hipErrorOutOfMemory;
        if (e == hipSuccess) e = rt::launch_render(a, 0);
    }
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e == hipSuccess) e = hipMemcpy(out_rgb, d_out, out_bytes, hipMemcpyDeviceToHost);
    unsigned long long casts = 0;
    if (e == hipSuccess) e = hipMemcpy(&casts, d_casts, sizeof(casts), hipMemcpyDeviceToHost);
    (void)hipFree(d_blocks);
    (void)hipFree(d_out);
    (void)hipFree(d_casts);
    if (e != hipSuccess) return fail(RT_E_HIP, "rt_render: %s", hipGetErrorString(e));
    if (out_ray_casts) *out_ray_casts = casts;
    return RT_OK;
}

int rt_render_tiles_device(rt_ctx* ctx, const rt_scene* scene, const rt_camera* cam,
                           const rt_params* params, const int32_t* tiles, int n_tiles, int tile_size,
                           float* d_out, uint64_t* d_casts, void* stream) {
    if (!ctx || !scene || !cam) return fail(RT_E_INVALID, "NULL argument");
    int rc = check_params(params);
    if (rc != RT_OK) return rc;
    if (n_tiles < 0) return fail(RT_E_INVALID, "n_tiles < 0");
    if (n_tiles == 0) return RT_OK;
    if (!tiles || !d_out) return fail(RT_E_INVALID, "NULL tiles/out");
    if (tile_size <= 0 || tile_size % 16 != 0) return fail(RT_E_INVALID, "tile_size must be a positive multiple of 16");
    for (int k = 0; k < n_tiles; ++k) {
        const int tx = tiles[2 * k], ty = tiles[2 * k + 1];
        if (tx < 0 || ty < 0 || tx >= params->width || ty >= params->height)
            return fail(RT_E_INVALID, "tile %d origin (%d,%d) outside the image", k, tx, ty);
    }
    rc = set_device(ctx);
    if (rc != RT_OK) return rc;
    const rt::BlockDesc* d_blocks = nullptr;
    int n_blocks = 0;
    rc = rt::ctx_blocks(ctx, tiles, n_tiles, tile_size, params->width, params->height, &d_blocks, &n_blocks);
    if (rc != RT_OK) return rc;
    rc = rt::scene_ensure_ctab(scene, params->hit_rule, params->t_scale,
                               rt::ctab_wanted(scene, cam, params, rt::kCtabForRender));
    if (rc != RT_OK) return rc;
    rt::RenderLaunch a = make_launch(scene, cam, params);
    a.blocks = d_blocks;
    a.n_blocks = n_blocks;
    a.clip_x1 = params->width;
    a.clip_y1 = params->height;
    a.out_pitch = tile_size;
    a.out = d_out;
    a.casts = reinterpret_cast<unsigned long long*>(d_casts);
    rc = rt::ctx_chunks(ctx, &a);
    if (rc != RT_OK) return rc;
    // RT_PS_PROF (with an RT_PROF=1 kernel build): k_render_ps's per-phase cycle sums to stderr
    static const bool prof = getenv("RT_PS_PROF") != nullptr;
    if (prof) RT_HIP(hipMalloc(&a.prof, 8 * sizeof(unsigned long long)));
    if (prof) RT_HIP(hipMemsetAsync(a.prof, 0, 8 * sizeof(unsigned long long), (hipStream_t)stream));
    RT_HIP(rt::launch_render(a, (hipStream_t)stream));
    if (prof) {
        unsigned long long v[8];
        RT_HIP(hipStreamSynchronize((hipStream_t)stream));
        RT_HIP(hipMemcpy(v, a.prof, sizeof(v), hipMemcpyDeviceToHost));
        RT_HIP(hipFree(a.prof));
        fprintf(stderr, "{\"ps_prof\": {\"primary\": %llu, \"shade\": %llu, \"masks\": %llu, \"exact\": %llu, "
                        "\"bounce_total\": %llu, \"trips\": %llu}}\n", v[0], v[1], v[2], v[3], v[4], v[5]);
    }
    return RT_OK;
}

int rt_selftest(rt_ctx* ctx, int which, uint64_t* result) {
    if (!ctx || !result) return fail(RT_E_INVALID, "NULL argument");
    if (which != RT_SELFTEST_RCP && which != RT_SELFTEST_DIV12 && which != RT_SELFTEST_DIVRHO)
        return fail(RT_E_INVALID, "unknown self-test %d", which);
    int rc = set_device(ctx);
    if (rc != RT_OK) return rc;
    unsigned long long* d_m = nullptr;
    unsigned* d_f = nullptr;
    hipError_t e = hipMalloc(&d_m, sizeof(unsigned long long));
    if (e == hipSuccess) e = hipMalloc(&d_f, sizeof(unsigned));
    if (e == hipSuccess) e = hipMemset(d_m, 0, sizeof(unsigned long long));
    if (e == hipSuccess) e = hipMemset(d_f, 0xff, sizeof(unsigned));
    if (e == hipSuccess) e = rt::launch_selftest(which, d_m, d_f, 0);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    unsigned long long m = 0;
    unsigned f = 0;
    if (e == hipSuccess) e = hipMemcpy(&m, d_m, sizeof(m), hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(&f, d_f, sizeof(f), hipMemcpyDeviceToHost);
    (void)hipFree(d_m);
    (void)hipFree(d_f);
    if (e != hipSuccess) return fail(RT_E_HIP, "rt_selftest: %s", hipGetErrorString(e));
    result[0] = m;
    result[1] = f;
    return RT_OK;
}


// ---- checks of the primary-ray cull (k_cull_ps) on the host ----

int rt_filter_build(const float* tri_v, int n, float* out_filt) {
    if (!tri_v || !out_filt || n <= 0) return fail(RT_E_INVALID, "bad arguments");
    const double obound = filter_origin_bound(tri_v, (size_t)n * 9);
    for (int i = 0; i < n; ++i) {
        float4 rec[3];
        isect_record(tri_v + (size_t)i * 9, rec);
        float4 f[rt::kFiltF4];
        if (!build_filter(rec[0], rec[1], rec[2], obound, f))
            return fail(RT_E_UNSUPPORTED, "no filter record for triangle %d (coordinates too large)", i);
        memcpy(out_filt + (size_t)i * 4 * rt::kFiltF4, f, sizeof(f));
    }
    return RT_OK;
}

int rt_cull_masks_device(rt_ctx* ctx, const rt_scene* scene, const rt_camera* cam, const rt_params* params,
                         int x0, int y0, int w, int h, uint64_t* out, int64_t* n_words) {
    if (!ctx || !scene || !cam || !out || !n_words) return fail(RT_E_INVALID, "NULL argument");
    int rc = check_params(params);
    if (rc != RT_OK) return rc;
    if (w <= 0 || h <= 0 || x0 < 0 || y0 < 0 || x0 + w > params->width || y0 + h > params->height)
        return fail(RT_E_INVALID, "rectangle outside the image");
    rc = set_device(ctx);
    if (rc != RT_OK) return rc;
    std::vector<rt::BlockDesc> blocks;
    for (int by = 0; by < h; by += 16)
        for (int bx = 0; bx < w; bx += 16) blocks.push_back({x0 + bx, y0 + by, bx, by});
    // k_cull_ps covers what k_render_ps's launch condition covers: the CPU preset, scenes of
    // <= 64 * kRenderCullWords triangles (wider scenes would get truncated masks)
    if (params->preset != RT_PRESET_CPU) return fail(RT_E_UNSUPPORTED, "the primary-ray cull is CPU-preset only");
    if (scene->dev.n_tri > 64 * rt::kRenderCullWords)
        return fail(RT_E_UNSUPPORTED, "the primary-ray cull covers scenes of <= %d triangles (this one has %d)",
                    64 * rt::kRenderCullWords, scene->dev.n_tri);
    rt::RenderLaunch a = make_launch(scene, cam, params);
    if (!a.use_filter) return fail(RT_E_UNSUPPORTED, "no filter records for this scene and camera");
    a.n_blocks = (int)blocks.size();
    a.clip_x1 = x0 + w;
    a.clip_y1 = y0 + h;
    const int64_t words = (int64_t)a.n_blocks * a.split * 4 * rt::kRenderCullWords;
    if (*n_words < words) {
        const long long cap = (long long)*n_words;
        *n_words = words;
        return fail(RT_E_INVALID, "out holds %lld words, %lld needed", cap, (long long)words);
    }
    rt::BlockDesc* d_blocks = nullptr;
    hipError_t e = hipMalloc(&d_blocks, sizeof(rt::BlockDesc) * blocks.size());
    if (e == hipSuccess)
        e = hipMemcpy(d_blocks, blocks.data(), sizeof(rt::BlockDesc) * blocks.size(), hipMemcpyHostToDevice);
    if (e == hipSuccess) {
        a.blocks = d_blocks;
        rc = rt::ctx_cull(ctx, &a);
        if (rc != RT_OK) e = hipErrorOutOfMemory;
    }
    if (e == hipSuccess) e = rt::launch_cull(a, 0);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e == hipSuccess) e = hipMemcpy(out, a.cull, sizeof(uint64_t) * (size_t)words, hipMemcpyDeviceToHost);
    (void)hipFree(d_blocks);
    if (e != hipSuccess) return fail(RT_E_HIP, "rt_cull_masks_device: %s", hipGetErrorString(e));
    *n_words = words;
    return RT_OK;
}

int rt_rect_candidates(const float* filt, int n_tri, const rt_camera* cam, const rt_params* p, int px0, int py0,
                       int px1, int py1, uint64_t* masks) {
    if (!filt || !cam || !p || !masks || n_tri <= 0) return fail(RT_E_INVALID, "bad arguments");
    if (p->preset != RT_PRESET_CPU) return fail(RT_E_UNSUPPORTED, "the primary-ray phase is CPU-preset only");
    if (px0 > px1 || py0 > py1) return fail(RT_E_INVALID, "empty rectangle");
    const rt::CamRect c = rt::make_cam_rect(cam->pos[0], cam->pos[1], cam->pos[2], (float)cos((double)cam->yaw_y),
                                            (float)sin((double)cam->yaw_y), p->width, p->height, p->t_scale,
                                            px0, px1, py0, py1);
    const float4* f = reinterpret_cast<const float4*>(filt);
    for (int g = 0; g < (n_tri + 63) / 64; ++g) masks[g] = 0;
    for (int i = 0; i < n_tri; ++i) {
        const bool cull = (p->hit_rule == RT_HIT_RULE_CPU) ? rt::rect_cull<0>(f + (size_t)i * rt::kFiltF4, c)
                                                           : rt::rect_cull<1>(f + (size_t)i * rt::kFiltF4, c);
        if (!cull) masks[i / 64] |= 1ull << (i % 64);
    }
    return RT_OK;
}

}  // extern "C"
