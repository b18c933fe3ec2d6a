// rt_internal.hpp — types shared by the C-ABI layer and the gfx950 kernels.
#pragma once

#include <string>
#include <vector>

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rt_math.hpp"

namespace rt {

// Kernel timing (rt_ktime.cpp; rt_ktime_enable / rt_ktime_read in rtmi.h): while enabled,
// a KernelTimer scope records a HIP event pair on the launch stream around the launches
// it encloses, per kernel family.  Off by default (one relaxed atomic load per launch).
enum KtimeKernel {
    KT_RENDER_PS = 0,   // k_render_ps (CPU preset, the bench kernel)
    KT_RENDER = 1,      // k_render (GPU preset / no primary phase)
    KT_SARSA_RENDER = 2,
    KT_SARSA_APPLY = 3,
    KT_DQN_MLP = 4,
    KT_DQN_BOUNCE = 5,
    KT_DQN_CAMERA = 6,
    KT_COUNT = 7
};
struct KernelTimer {
    int kernel = -1;  // -1: not timing
    hipStream_t stream = nullptr;
    hipEvent_t ev_a = nullptr, ev_b = nullptr;  // owned by this scope until its end is recorded
    KernelTimer(int kernel, hipStream_t s);
    ~KernelTimer();
    KernelTimer(const KernelTimer&) = delete;
    KernelTimer& operator=(const KernelTimer&) = delete;
};

// CUs of the current device (persistent-grid launch sizes), cached per device ordinal;
// safe to call from several host threads (rt_ktime.cpp)
int device_cu_count();

// Device layout of one triangle for the hit test: 3 x float4 = 48 B
//   [0] = {v0.x, v0.y, v0.z, c0}   c0 = e1.y*e2.z - e2.y*e1.z (the determinant
//                                   minor that depends on the triangle only)
//   [1] = {e1.x, e1.y, e1.z, 0}     e1 = v1 - v0
//   [2] = {e2.x, e2.y, e2.z, 0}     e2 = v2 - v0
// Surfaces come first, then light triangles (the reference's test order:
// CPU/rays/ray.cpp:17-27).
constexpr int kIsectF4 = 3;

// Device layout of one triangle for shading: 5 x float4 = 80 B
//   [0] = normal N (CPU/objects/triangle.cpp:73-82)
//   [1] = tangent T, [2] = bitangent B (CPU/utils/hemisphere_helpers.cpp:26-39,
//         a per-triangle constant, so computed once on the host)
//   [3] = BRDF = albedo / pi (surfaces) or emission (lights)
//   [4] = albedo (surfaces)
constexpr int kShadeF4 = 5;

// Device layout of one triangle for the candidate filter of the two-phase hit
// test (rt_trace.hpp, closest_hit_filtered): 5 x float4 = 80 B, built in double
// on the host (rt_capi.cpp, build_filter) with N = e1 x e2, G1 = v0 x e1,
// G2 = v0 x e2:
//   [0] = {N, w0 = v0.N}
//   [1] = {e2, eA}    eA: error bound of the determinant A = d.N
//   [2] = {-G2, EW}   EW: error bound of the barycentric tests
//   [3] = {-e1, ET}   ET: error bound of the t test
//   [4] = {G1, 0}
// The bounds hold for |d_i| <= 2, |o_i| <= DeviceScene::origin_bound and
// t_scale <= kFiltMaxTScale (the host checks the last two per launch).
constexpr int kFiltF4 = 5;
constexpr float kFiltMaxTScale = 16384.0f;

// Matrix-core form of the same filter for rays from surface points (rt_trace.hpp,
// closest_hit_mf; built by rt_capi.cpp, build_mf_image).  Per ray the ten features
// f = (d, o', R = d x o, 1), o' = -o - ets d (RULE 0) or -o (RULE 1); per triangle four
// rows over f: A = d.N, T' = w0 + o'.N, U = e2.R - G2.d, V = -e1.R + G1.d (double,
// split into bf16 hi + lo).  One v_mfma_f32_16x16x32_bf16 evaluates
// sum fh bh + fl bh + fh bl for 4 triangles x 16 rays, K = 32:
//   k  0.. 7: fh0..fh7 | bh0..bh7      k 16..23: fl6..fl9, fh0..fh3 | bh6..bh9, bl0..bl3
//   k  8..15: fh8, fh9, fl0..fl5 | bh8, bh9, bh0..bh5    k 24..31: fh4..fh9, 0, 0 | bl4..bl9, 0, 0
// Triangles go in rounds of 32 (round r: triangles 32 r .., G = ceil(count / 4) groups);
// group g of a round holds triangle s G + (G - 1 - g) in slot s = 0..3 (rows 4 s + i,
// i = A, T', U, V).  Device image per group (index 8 r + g):
//   frag: 64 lanes x 8 bf16 (lane l: row l & 15, k = 8 (l >> 4) ..), the A operand
//   (lane 48 + 4 s, dword 3 = k 30, 31 of row 4 s, where the ray operand is 0: slot s's
//    threshold of the sign test |A| > rho, fp32 bits; 0 for a pad slot)
// Each row is scaled so that the filter's barycentric and t margins at c = 2^-12 become
// the constant 1 (U, V, W = A - U - V, T'): build_mf_rows.  The margins hold
// for |d_i| <= kMfDirBound (unit directions), |o_i| <= mf_bound (the scene's box, widened
// by 2^-10 relative + 2^-10: surface points and the bounce loop's 1e-5 offset) and
// t_scale <= kFiltMaxTScale; a lane outside keeps every triangle.
constexpr int kMfRound = 32;
constexpr int kMfGroupsPerRound = 8;
constexpr float kMfDirBound = 1.0009765625f;  // 1 + 2^-10

// Exact BVH path for large scenes (rt_bvh.cpp, rt_trace.hpp closest_hit_bvh).
//   nodes:  2 float4 per node {lo.xyz, link}, {hi.xyz, count} (int bits in w): count > 0 a
//           leaf of tris [link, link + count), else children link, link + 1
//   tris:   the kIsectF4 records in leaf order, [1].w = the original index (int bits)
//   graze:  per triangle {N (float), the grazing threshold at the scene box}
//   grec:   per triangle the grazing tests, 2 float4 {N~, alpha}, {beta, W, PA, PB}:
//           |d.N~| <= alpha B + beta, |N~.o - W| <= PA B + PB + (alpha B + beta) lambda
//   dstart/dlist: per cube-map cell of directions (6 x G x G), the triangles a ray in it
//           may graze (origins within the scene box); dstart_cam/dlist_cam: any origin
//           within obound
#ifndef RT_BVH_K
#define RT_BVH_K 4
#endif
#ifndef RT_BVH_PLANE_LEAF
#define RT_BVH_PLANE_LEAF 4
#endif
constexpr int kBvhK = RT_BVH_K;   // regular pairs: |A| >= K EW (barycentrics >= -1/K)
#ifndef RT_BVH_DIR_GRID
#define RT_BVH_DIR_GRID 48
#endif
constexpr int kBvhDirGrid = RT_BVH_DIR_GRID;  // cube-map cells per face edge
constexpr int kBvhMaxDepth = 24;  // traversal stack entries per lane (tree depth < 24)
constexpr int kBvhCand = 4;       // rule-0 candidates kept per ray (overflow: exact scan)
struct BvhHost {
    std::vector<float4> nodes, tris, graze, grec;
    std::vector<int32_t> dstart, dlist, dstart_cam, dlist_cam;
    float B_lists = 0.f;
    int n_nodes = 0, depth = 0;
    float sig_a = 0.f, sig_b = 0.f;
};
bool bvh_build(const float4* isect, int n, BvhHost* out);
std::string bvh_check(const float4* isect, int n, const BvhHost& h);

// Bounce-ray candidate table (rt_ctab.cpp, rt_trace.hpp closest_hit_ctab): hit rule 0 (t_scale >=
// ts_min) and hit rule 1 (any t_scale), scenes of at most 256 triangles (words = 1-4 mask words per
// entry).  A bounce ray leaving surface s from origin o in
// direction d: the patch of o in the 2D grid over s (its frame tri[4 s .. 4 s + 3]:
// {O', 1 / cell}, {U, n_u}, {V, n_v}, {N, first patch}; |N.(o - O')| <= h_run) and the cube-map
// bin of d (6 x kCtabBins^2; d in s's hemisphere, d.N >= -kCtabHemi) -> masks[patch][face][iu][iv], the
// triangles the ray may pass the
// exact test of; OR-ed with graze[face][gu][gv] (6 x kCtabGraze^2, as gid indices into gdict) and, where |d.N| < cop_th,
// with cop[s] (the triangles coplanar with s).  About kCtabPatches patches over the scene: at the
// default 16,384, about 200 MB of masks per mask word (Cornell 201 MB, built in about 1 s).
#ifndef RT_CTAB_PATCHES
#define RT_CTAB_PATCHES 16384  // 4,096 / 16,384 / 32,768: complex_light_room 2048^2 x 64 687 / 640 / 679 ms, Cornell 512^2 x 256 2.69 / 2.66 ms
#endif
#ifndef RT_CTAB_BINS
#define RT_CTAB_BINS 16
#endif
#ifndef RT_CTAB_GRAZE
#define RT_CTAB_GRAZE 256
#endif
constexpr int kCtabPatches = RT_CTAB_PATCHES;
constexpr int kCtabBins = RT_CTAB_BINS;
constexpr int kCtabGraze = RT_CTAB_GRAZE;
constexpr float kCtabTsMin = 256.0f;  // the smallest t_scale the table serves
constexpr float kCtabHemi = 2e-6f;    // directions with d.N_s < -kCtabHemi (off s's hemisphere) keep every triangle
constexpr int kCtabMaxWords = 4;  // mask words per entry: scenes of at most 256 triangles
constexpr uint64_t kCtabGflagBit = 1ull << 63;  // (gflag tables: scenes of at most 63 triangles)
// the render paths that may take the table (rt_capi.cpp ctab_wanted)
constexpr int kCtabForRender = 0, kCtabForDqn = 1, kCtabForSarsa = 2;
struct CtabHost {
    int n_tri = 0, n_surf = 0, n_patch = 0;
    int words = 1;        // ceil(n_tri / 64): masks, graze and cop hold that many words per entry
    int rule = 0;         // the hit rule it serves (0: ts_min applies; 1: any t_scale)
    int patches_all = 0;  // patches off their triangle (every triangle kept)
    float ts_min = 0.f, h_run = 0.f;
    float cop_th = 0.f;           // |d.N_s| below which the triangles coplanar with s join
    std::vector<float4> tri;      // [n_surf][4]
    std::vector<uint64_t> cop;    // [n_surf][words]: the triangles coplanar with s
    std::vector<uint64_t> masks;  // [patch][face][iu][iv][words]
    // the grazing bins' masks as 16-bit indices into a dictionary of their distinct masks (a few
    // hundred: 0.8 MB of indices instead of 9.4 MB of masks at 3 words, resident in L2)
    std::vector<uint64_t> gdict;  // [n_gdict][words]
    std::vector<uint16_t> gid;    // [face][gu][gv]
    std::vector<uint64_t> graze;  // the build's uncompressed grazing bins (emptied once indexed)
    int gflag = 0;                // the grazing fold (rt_ctab.cpp): masks hold their bin's grazing mask
                                  // unless bit 63 (kCtabGflagBit) says to look it up
};
bool ctab_build(const float4* isect, int n, int n_surf, double B, int rule, double ts_min, CtabHost* out);
void ctab_lookup(const CtabHost& h, int s, const float o[3], const float d[3], uint64_t* out);

// a candidate table on the device (CtabHost's arrays and constants)
struct CtabDev {
    const unsigned long long* masks = nullptr;  // [patch][face][iu][iv][words]
    const unsigned long long* gdict = nullptr;  // [n_gdict][words]
    const uint16_t* gid = nullptr;              // [face][gu][gv] -> gdict
    const unsigned long long* cop = nullptr;    // [n_surf][words]
    const float4* tri = nullptr;                // [n_surf][4]: the surfaces' patch frames
    float h = 0.0f, ts_min = 0.0f, cop_th = 0.0f;
    int words = 0;
    int bins = 0, graze_n = 0;  // the build's kCtabBins / kCtabGraze (kernels use the table only if theirs agree)
    int gflag = 0;              // CtabHost::gflag
    int n_gdict = 0;            // entries of gdict (words each)
};

struct DeviceScene {
    float4* isect = nullptr;   // n_tri * kIsectF4
    float4* shade = nullptr;   // n_tri * kShadeF4
    float4* filt = nullptr;    // n_tri * kFiltF4 (nullptr: no filter records for this scene)
    uint4* mf_frag = nullptr;  // matrix-core filter image (above; nullptr: none)
    float mf_bound = 0.0f;     // |o_i| bound of the matrix-core margins
    float origin_bound = 0.0f; // |o_i| bound the filter records were built for
    int32_t* code_cpu = nullptr;  // n_tri packed hit codes under hit rule CPU
    int32_t* code_gpu = nullptr;  // ... under hit rule GPU
    // BVH path (nullptr: none)
    const float4* bvh_nodes = nullptr;
    const float4* bvh_tris = nullptr;
    const float4* bvh_graze = nullptr;
    const float4* bvh_grec = nullptr;
    const int32_t* bvh_dstart = nullptr;      // [2][cells + 1]: scene-box origins, any origin
    const int32_t* bvh_dlist = nullptr;
    const int32_t* bvh_dlist_cam = nullptr;
    float bvh_B_lists = 0.0f;
    float bvh_sig_a = 0.0f, bvh_sig_b = 0.0f;
    // bounce-ray candidate tables (CtabHost), one per hit rule (masks nullptr: none)
    CtabDev ctab[2];
    int n_surf = 0;
    int n_tri = 0;
};

// One 16x16 pixel block of work: pixel origin and output origin.  It is
// rendered by `split` workgroups of 256 threads; each pixel by `split` lanes.
struct BlockDesc {
    int px0, py0, ox0, oy0;
};

struct RenderLaunch {
    DeviceScene scene;
    int width, height, spp, max_bounces;
    int split, split_log2, per_chunk;  // lanes per pixel, log2, samples per lane
    int preset, sampler, hit_rule;
    uint32_t seed_lo, seed_hi;
    float t_scale, env_light;
    float cam_x, cam_y, cam_z;
    float cos_y, sin_y, cos_x, sin_x;
    const BlockDesc* blocks;
    int n_blocks;
    int clip_x1, clip_y1;
    int out_pitch;
    float* out;
    unsigned long long* casts;
    uint32_t sample_base;  // first RNG sample index (SARSA: frame * spp); 0 elsewhere
    int use_filter;        // 1: two-phase closest hit (filter records valid for this launch)
    // k_render<MF> (GPU preset): 1 = camera rays take the wave's primary-ray candidate set
    // (rt_cull.hpp) instead of the matrix-core filter -- set by the launcher when the camera
    // lies outside the image's origin bound (every camera ray would keep every triangle)
    int cam_cull;
    // k_cull_ps (diagnostic): kRenderCullWords 64-bit candidate masks per wave
    // (n_blocks * split * 4 waves); unused by the renders
    unsigned long long* cull;
    // RT_PROF builds only: per-phase s_memtime cycle sums of k_render_ps (8 counters)
    unsigned long long* prof;
    // GPU preset, persistent chunk queue (k_render_pq): the chunk sums [n_blocks * 256 *
    // split][3] and the work counter (zeroed by the launcher); null: the per-pixel kernels
    float* csum;
    unsigned long long* work;
};
constexpr int kRenderCullWords = 4;  // candidate masks per wave: scenes of <= 256 triangles

// 1 if the filter records of `s` hold for rays from a camera at (cx, cy, cz) (and
// from surface points) at this t_scale.  Host side, once per launch.
inline int filter_usable(const DeviceScene& s, float cx, float cy, float cz, float t_scale) {
    if (s.filt == nullptr) return 0;
    const float m = fmaxf(fabsf(cx), fmaxf(fabsf(cy), fabsf(cz)));
    return (m <= s.origin_bound && t_scale > 0.0f && t_scale <= kFiltMaxTScale) ? 1 : 0;
}

// ---- DQN Q-value network (dq_network/fc_layer) and its wavefront renderer ----
// Four ReLU layers n_in -> h1 -> h2 -> h3 -> n_out (NN_Builders/dq_network.cu:8-33).
// Layer 0's input is x = Scene::vertices - p, the vertices relative to the ray
// position p (nn_rendering_helpers.cu:280-298), so W1 x + b1 = (W1 v + b1) - S p
// with S[o][c] = sum over the vertices of W1[o][3v + c]: an affine map of the 3
// coordinates of p.  The host folds it once per network in double
// (rt_dqn_create); the kernel evaluates it in fp32 (an exact f32 MFMA, the
// reference's own precision) instead of a K = n_in bf16 contraction.  Layers 1-3 run on MFMA:
// device weights bf16, zero padded, stored in MFMA B-fragment order.
constexpr int kDqnActions = 144;  // GRID_RESOLUTION^2 (GPU/constants/radiance_volumes_settings.h:9)
constexpr int kDqnGrid = 12;

constexpr int kMlpStationary = 2;  // RT_DQN_MLP_STATIONARY
struct DqnNet {
    // layer 0 folded: [N[0]] x {-S0, -S1, -S2, c0}; h1 = ReLU(c0 - fma(S2, z, fma(S1, y, S0 x)))
    const float4* l0 = nullptr;
    // layers 1-3: bf16 bits in fragment order [N/16][K/32][lane 64][8], lane = kq*16 + r
    // holding W[nt*16 + r][ks*32 + kq*8 .. +7] -- a wave's fragment load is one contiguous 1 KB
    const uint16_t* W[4] = {nullptr, nullptr, nullptr, nullptr};
    const float* b[4] = {nullptr, nullptr, nullptr, nullptr};      // fp32, padded (b[0] unused)
    int K[4] = {0, 0, 0, 0};      // padded input width of each layer (K[0] = n_in, unpadded)
    int N[4] = {0, 0, 0, 0};      // padded output width of each layer (multiple of 32; last = 144)
    int mlp_mode = 0;             // RT_DQN_MLP_* (rtmi.h rt_dqn_set_mlp)
};

// Ray state of the DQN wavefront renderer (SoA over the rays of a frame part).
// Several samples are in flight at once: ray id = slot * n_pix + pixel index, slot k
// tracing sample s0 + k, so late bounces (few surviving paths per sample) still fill
// the GPU; the per-pixel totals add the slots in sample order (the sequential order).
struct DqnRays {
    float* loc = nullptr;   // [n][3] current position (GPU: ray_locations_device)
    float* dir = nullptr;   // [n][3]
    float* tp = nullptr;    // [n][3] throughput
    float* total = nullptr; // [n_pix][3] sum over samples
    int32_t* tri = nullptr; // [n] triangle of the last surface hit (normal / frame)
    uint32_t* pix = nullptr;   // [n_pix] global pixel id (RNG key)
    int32_t* list[2] = {nullptr, nullptr};  // active ray lists (ping-pong)
    int32_t* count = nullptr;  // [2 + 1] list sizes, [2] = ray casts of this call (low 32 bits unused)
    unsigned long long* casts = nullptr;
    float* q = nullptr;     // [144][ldq] Q values of the active list, action-major (list order)
    int n = 0;              // rays of the current pass: n_pix * samples in flight
    int n_pix = 0;          // pixel slots (16x16 blocks x 256)
    int s0 = 0;             // sample of slot 0
    int ldq = 0;            // leading dimension of q: ray capacity rounded up to whole MLP tiles and 64
};

struct DqnLaunch {
    DeviceScene scene;
    DqnNet net;
    DqnRays rays;
    int width, height, spp, max_bounces;
    uint32_t seed_lo, seed_hi;
    float t_scale, env_light;
    float cam_x, cam_y, cam_z;
    float cos_y, sin_y, cos_x, sin_x;
    const BlockDesc* blocks;   // 16x16 pixel blocks (ray id = block * 256 + y*16 + x)
    int n_blocks;
    int clip_x1, clip_y1;
    int out_pitch;
    float* out;
    int use_filter;  // as RenderLaunch::use_filter
};

// Neural-Q training renderer (GPU/deep_learning/neural_q_pathtracer.cu:226-600): one ray
// per pixel (id = y * width + x) through all bounces of a sample, in the reference's
// per-ray arrays (SoA, device).
struct NqRays {
    int n = 0;                     // rays = pixels
    float* loc = nullptr;          // [n][3] position (S_{t+1} after a trace)
    float* prev = nullptr;         // [n][3] position before the trace (S_t of the learning rule)
    float* dir = nullptr;          // [n][3] direction to trace next
    float* tp = nullptr;           // [n][3] throughput
    float* total = nullptr;        // [n][3] throughput summed over the frame's samples
    int32_t* tri = nullptr;        // [n] surface of the position (its frame: shade N, T, B)
    uint32_t* state = nullptr;     // [n] 0 active, 1 terminal, 2 restarted (learning only)
    float* reward = nullptr;       // [n]
    float* discount = nullptr;     // [n]
    uint32_t* bounces = nullptr;   // [n] bounce of termination (MAX_RAY_BOUNCES if none)
    int32_t* action = nullptr;     // [n] sampled cell (the learning rule's a_t)
    int32_t* terminal = nullptr;   // [n] state == 1 (compute_td_targets' test)
    uint32_t* pix = nullptr;       // [n] pixel ids (RNG keys; = ray ids)
    int32_t* flag = nullptr;       // [1] 1 = every path has terminated (rays_finished)
    const float* surf_v = nullptr;  // [n_surf][9] surface vertices (restarts)
    const float* tri_lum = nullptr; // [n_tri] Material / AreaLight luminance 0.5 (max + min)
    unsigned long long* stats = nullptr;  // [3] sum of bounces, zero-contribution paths, ray casts
};
hipError_t launch_nq_init(const DqnLaunch& a, const NqRays& r, int sample, hipStream_t stream);
hipError_t launch_nq_sample(const DqnLaunch& a, const NqRays& r, float* q, float eps, int sample, int bounce,
                            hipStream_t stream);
hipError_t launch_nq_trace(const DqnLaunch& a, const NqRays& r, int bounce, hipStream_t stream);
hipError_t launch_nq_restart(const DqnLaunch& a, const NqRays& r, int sample, int bounce, hipStream_t stream);
hipError_t launch_nq_end_sample(const DqnLaunch& a, const NqRays& r, hipStream_t stream);
hipError_t launch_nq_image(const DqnLaunch& a, const NqRays& r, float* out, int spp, hipStream_t stream);

// rays per k_dqn_mlp workgroup (an action-major q's ldq covers whole tiles)
int dqn_mlp_tile_rows();
// q layout: ldq == 0 -> [row][144] (the C ABI's); ldq > 0 -> action-major q[a * ldq + row],
// ldq a multiple of 64 covering every launched row (whole MLP tiles; the renderer's, coalesced per action)
hipError_t launch_dqn_mlp(const DqnNet& net, const float* loc, const int32_t* list,
                          const int32_t* count, int max_rows, float* q, int ldq, hipStream_t stream);
// weight-stationary forward (rt_dqn_ws.hip): one workgroup per CU, the 200-300-200 shape
bool dqn_mlp_ws_fits(const DqnNet& net);
hipError_t launch_dqn_mlp_ws(const DqnNet& net, const float* loc, const int32_t* list, const int32_t* count,
                             int max_rows, float* q, int ldq, int n_cu, bool qb, hipStream_t stream);
hipError_t launch_dqn_frame_begin(const DqnLaunch& a, hipStream_t stream);
hipError_t launch_dqn_camera(const DqnLaunch& a, hipStream_t stream);  // samples s0 .. s0 + n/n_pix - 1
hipError_t launch_dqn_bounce(const DqnLaunch& a, int bounce, hipStream_t stream);
hipError_t launch_dqn_accumulate(const DqnLaunch& a, hipStream_t stream);
hipError_t launch_dqn_finish(const DqnLaunch& a, hipStream_t stream);
// sampler alone (parity): rows i < n, Q [n][144] (overwritten with Q*cos), pixel/tri/loc per row
hipError_t launch_dqn_sample_only(const DeviceScene& s, const float* q, const float* loc,
                                  const int32_t* tri, const uint32_t* pix, int n, int sample,
                                  int bounce, uint32_t seed_lo, uint32_t seed_hi, float* tp,
                                  float* dir_out, int32_t* action, hipStream_t stream);

// ---- Expected-SARSA radiance volumes (BASELINE config 3) ----
// Flattened KD tree of GPU/radiance_volumes/radiance_tree.cuh:19-27 (48 B per node):
// the host/export form.  The device form is 16 B per node in the same order (kd4), so
// a subtree's nodes, leaf positions included, are contiguous (the reference's layout
// appends a node's two children together, then the left subtree, then the right):
//   internal: {median bits, left child (right = left + 1), split dimension, 0xFFFFFFFF}
//   leaf:     {x, y, z (float bits), volume index}; its normal is vol_frame[3 * volume].
struct KdNode {
    int dim, leaf, left, right;
    float data;          // split median (internal) or volume index (leaf, as float like the reference)
    float px, py, pz;    // leaf position (0 for internal nodes)
    float nx, ny, nz;    // leaf normal
    int vol;             // leaf volume index
};

constexpr int kSarsaSectors = 144;

struct SarsaMap {
    int n_vol = 0;
    const float4* vol_pos = nullptr;    // [n] sampled position
    const float4* vol_frame = nullptr;  // [n*3] N, T, B (create_transformation_matrix); w: position x, y, z
    const float* vol_brdf = nullptr;    // [n] luminance/pi of the volume's surface
    const float* cos_center = nullptr;  // [n*144] cos of the cell-centre directions
    const float* cos_corner = nullptr;  // [n*144] cos of the cell-corner directions
    const float* tri_lum = nullptr;     // [n_tri] Material/AreaLight luminance 0.5*(max+min)
    float* Q = nullptr;                 // [n*144] radiance_grid
    float* cdf = nullptr;               // [n*144] radiance_distribution
    float4* cdf_top = nullptr;          // [n*4] {cdf[0], cdf[11], cdf[23], .., cdf[143], 0, 0, 0}: row ends
    uint32_t* visits = nullptr;         // [n*144]
    float* accum = nullptr;             // [n] irradiance_accum
    unsigned long long* acc_sum = nullptr;  // [n*144] frame TD targets, fixed point 2^-32
    uint32_t* acc_cnt = nullptr;            // [n*144] frame TD target count
    const uint4* kd4 = nullptr;         // [n_kd] device KD array (above)
    int n_kd = 0;
    float root_x = 0.f, root_y = 0.f, root_z = 0.f;  // position of KD element 0 (0 if internal)
    float max_dist = 0.003f;            // MAX_DIST (compared with delta^2)
    int max_wgs = 0;                    // host: cap on the persistent render's workgroups (0: none)
    // Exact fast path of the nearest-volume search (rt_sarsa.hip sarsa_nearest_grid):
    // per normal class (volumes whose normals compare equal), a uniform grid of cell
    // size >= grid_h over the class's volume positions.
    int use_grid = 0;
    int n_class = 0;
    const int32_t* tri_class = nullptr;    // [n_surf] class of each surface's normal, -1: none
    const float4* class_org = nullptr;     // [n_class] grid origin, w = first cell (int bits)
    const int4* class_dim = nullptr;       // [n_class] cells per axis
    const float4* class_nrm = nullptr;     // [n_class] the class normal
    const uint32_t* cell_start = nullptr;  // [cells + 1] first grid_leaf of each cell
    const uint2* cell_range = nullptr;     // [cells] {first, end} grid_leaf of each cell (one load)
    const float4* cell_head = nullptr;     // [cells][4] {first, end (bits)} + the cell's first 3 grid_leaf entries (one 64-B line)
    const float4* tri_grid = nullptr;      // [n_surf][2] the surface's class grid: {org, first cell (bits)},
                                           // {dims (int bits), class (int bits, -1: none)}
    const float4* grid_leaf = nullptr;     // [n] volume positions by (class, cell), w = volume (int bits)
    float grid_inv_cs = 0.f;               // 1 / cell size
    float grid_cs = 0.f;                   // cell size (cell centres: org + (i + 0.5) cs)
    float grid_h = 0.f;                    // accept radius: sqrt(MAX_DIST) * 0.999
    unsigned long long* grid_fallbacks = nullptr;  // optional count of KD fallbacks
    // sampling rule: 0 = the CDF (sample_direction_from_radiance_distribution), 1 = the
    // sector of largest Q (sample_max_direction_from_radiance_distribution)
    int sample_max = 0;
    // TD rule: 0 = frame-synchronous sums folded by k_sarsa_apply (deterministic), 1 = the
    // reference's in-frame update of Q, visits and irradiance at each event (racy)
    int td_inframe = 0;
    int32_t* qmax = nullptr;               // [n] first sector of largest Q (k_sarsa_apply)
    unsigned long long* stats = nullptr;   // [2] launch: sum of per-pixel int(mean path length), zero paths
    unsigned long long* prof = nullptr;    // [8] RT_SARSA_PROF builds: per-phase s_memtime cycles (rt_sarsa.hip)
};
#ifndef RT_KD_STACK
// 30: the SARSA render's 256-lane workgroup then takes 30 KB of LDS and five fit a CU (32 KB held
// it to four: door_room 512^2 x 256 frames 1-4 108.6 -> 104.9 ms, profiles/r6r/); supports trees
// of depth 29 (2^29 volumes; rt_sarsa_create_density caps maps at 2^24)
#define RT_KD_STACK 30
#endif
constexpr int kKdStack = RT_KD_STACK;  // traversal stack entries per lane (LDS); tree depth <= kKdStack - 1

hipError_t launch_sarsa_render(const RenderLaunch& r, const SarsaMap& m, hipStream_t stream);
hipError_t launch_sarsa_apply(const SarsaMap& m, hipStream_t stream);
bool sarsa_prof_compiled();  // rt_sarsa.hip was built with RT_SARSA_PROF=1 (per-phase cycle counters)
bool sarsa_ctab_compiled();  // rt_sarsa.hip was built with RT_SARSA_CTAB=1 (the table route of its persistent kernel)
hipError_t launch_sarsa_rebuild(const SarsaMap& m, hipStream_t stream);  // CDF + argmax from Q
hipError_t launch_sarsa_nearest(const SarsaMap& m, const float* pos, const float* nrm, int n, int32_t* out,
                                hipStream_t stream);

hipError_t launch_intersect(const DeviceScene& s, const float* orig, const float* dir, int n,
                            float t_scale, int hit_rule, int use_filter, float* out_t,
                            int32_t* out_hit, hipStream_t stream);
// the exact BVH path on caller rays
hipError_t launch_intersect_bvh(const DeviceScene& s, const float* orig, const float* dir, int n, float t_scale,
                                int hit_rule, float* out_t, int32_t* out_hit, hipStream_t stream);
// the matrix-core filter (closest_hit_mf) on caller rays; cand: optional candidates per ray
hipError_t launch_intersect_mf(const DeviceScene& s, const float* orig, const float* dir, int n, float t_scale,
                               int hit_rule, float* out_t, int32_t* out_hit, int32_t* cand, hipStream_t stream);

// exhaustive rcp_rn == 1.0f/x check over all 2^32 floats (4096 x 256 threads x 4096)
hipError_t launch_selftest(int which, unsigned long long* mism, unsigned* first, hipStream_t stream);

// "x y z nx ny nz" location files (to_select.txt); RT_OK or RT_E_IO (rt_sarsa_host.cpp)
int read_locations(const char* path, std::vector<float>* loc, std::vector<float>* nrm);

// returns hipErrorInvalidValue for combinations the kernels do not instantiate
hipError_t launch_render(const RenderLaunch& a, hipStream_t stream);
// k_cull_ps alone (the primary-ray candidate masks into a.cull)
hipError_t launch_cull(const RenderLaunch& a, hipStream_t stream);

}  // namespace rt
