// rt_kernels.hip — gfx950 kernels of the path tracer's hot path.
//
//  k_intersect : Ray::closest_intersection over a batch of rays (one lane per
//                ray) — the reference's innermost loop (CPU/rays/ray.cpp:14-28,
//                GPU/rays/ray.cu:16-141) as a standalone kernel.
//  k_render    : the per-pixel trace loop (pixel -> SPP -> bounce) as one
//                megakernel: camera ray, closest hit, uniform-hemisphere
//                sampling, Lambertian estimator, SPP mean
//                (CPU/path_tracing/default_path_tracing.cpp:5-101,
//                GPU/path_tracing/default_path_tracing.cu:7-88).
//
// CDNA4 mapping:
//  * one lane = one (pixel, sample chunk); a pixel's `split` chunks sit in
//    adjacent lanes and are folded with wave shuffles in a fixed order; a
//    16x16 pixel block is `split` workgroups of 256 threads.  A lane runs its
//    chunk's samples in order and
//    regenerates a camera ray the moment its path ends, so every lane casts a
//    ray on every loop trip until its pixel is done (no idle lanes waiting
//    for the longest path of the wave); the loop exit is a wave ballot.
//  * the triangle loop index is wave-uniform: the triangle records are
//    fetched with scalar loads (s_load_dwordx4) into SGPRs and broadcast as
//    VALU operands — no LDS round trip and no per-lane address math.
//  * per-pixel sums are kept in registers in sample order, so the image is
//    bit-identical to the CPU restatement (oracle/) and to any tiling.
//
// Numerics: built with -ffp-contract=off and hipcc's default correctly
// rounded fp32 division / sqrt; no fast-math (see rt_math.hpp).

#include <float.h>

#include "rt_trace.hpp"

namespace rt {

namespace {

template <int RULE>
__global__ __launch_bounds__(256) void k_intersect(const DeviceScene s, int use_filter,
                                                   const int32_t* __restrict__ code,
                                                   const float* __restrict__ orig,
                                                   const float* __restrict__ dir, int n,
                                                   float t_scale, float* __restrict__ out_t,
                                                   int32_t* __restrict__ out_hit) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    const f3 o = make3(orig[3 * r + 0], orig[3 * r + 1], orig[3 * r + 2]);
    const f3 d = make3(dir[3 * r + 0], dir[3 * r + 1], dir[3 * r + 2]);
    const Hit h = closest_hit_sel<RULE>(s, use_filter, o, d, t_scale);
    out_t[r] = (h.tri >= 0) ? h.t : __builtin_inff();
    out_hit[r] = (h.tri >= 0) ? code[h.tri] : -1;
}

// The matrix-core filter on caller rays (rt_intersect_method): every lane of a wave
// takes part, lanes past n cast a dummy ray with no candidates.  cand (optional): the
// candidates of each ray that reached the exact test.
template <int RULE>
__global__ __launch_bounds__(256) void k_intersect_mf(const DeviceScene s, const int32_t* __restrict__ code,
                                                      const float* __restrict__ orig,
                                                      const float* __restrict__ dir, int n, float t_scale,
                                                      float* __restrict__ out_t, int32_t* __restrict__ out_hit,
                                                      int32_t* __restrict__ cand) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    const bool in = r < n;
    const f3 o = in ? make3(orig[3 * r + 0], orig[3 * r + 1], orig[3 * r + 2]) : make3(0.0f, 0.0f, 0.0f);
    const f3 d = in ? make3(dir[3 * r + 0], dir[3 * r + 1], dir[3 * r + 2]) : make3(0.0f, 0.0f, 1.0f);
    __shared__ float wls[4][kMfWaveFloats];
    int nc = 0;
    const Hit h = closest_hit_mf<RULE, true>(s, o, d, t_scale, in, wls[threadIdx.x >> 6], &nc);
    if (!in) return;
    out_t[r] = (h.tri >= 0) ? h.t : __builtin_inff();
    out_hit[r] = (h.tri >= 0) ? code[h.tri] : -1;
    if (cand != nullptr) cand[r] = nc;
}

// The exact BVH path on caller rays (large scenes).
template <int RULE>
__global__ __launch_bounds__(256) void k_intersect_bvh(const DeviceScene s, const int32_t* __restrict__ code,
                                                       const float* __restrict__ orig, const float* __restrict__ dir,
                                                       int n, float t_scale, float* __restrict__ out_t,
                                                       int32_t* __restrict__ out_hit) {
    __shared__ int stk[kBvhMaxDepth * 256];
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    const f3 o = make3(orig[3 * r + 0], orig[3 * r + 1], orig[3 * r + 2]);
    const f3 d = make3(dir[3 * r + 0], dir[3 * r + 1], dir[3 * r + 2]);
    const Hit h = closest_hit_bvh<RULE>(s, o, d, t_scale, stk + threadIdx.x);
    out_t[r] = (h.tri >= 0) ? h.t : __builtin_inff();
    out_hit[r] = (h.tri >= 0) ? code[h.tri] : -1;
}




// PRESET 0: CPU engine recursion (a path's value is folded from the light
// back to the camera: L_k = ((L_{k+1} * brdf_k) * cos_k) / rho), cap <= 2.
// PRESET 1: GPU engine iterative throughput.
//
// STEAL: the lanes of a pixel share its samples instead of owning fixed chunks: a lane
// whose path ends claims the pixel's next unclaimed sample (ballot + mbcnt rank), so
// no lane idles while another finishes a long chunk (with fixed chunks the wave runs
// for the longest chunk: ~90% lane use at 4 samples per lane).  Each sample's value
// goes to LDS; at the end lane c sums samples [c m, (c + 1) m) in order, exactly the
// chunk sum of the fixed assignment, so the image is bit-identical.
//
// BVH: large scenes cast through closest_hit_bvh (the exact BVH path: same hits as the
// scan).
//
// MF (> 0: 64-triangle blocks per super-block): every cast on the matrix-core filter
// (closest_hit_mf, wave-level: lanes without a live sample take part with no
// candidates), as the bounce casts of k_render_ps; the launcher picks it when the camera
// lies inside the image's origin bound (else every camera ray would keep every triangle).
// the bits of 64-triangle group g that are triangles of an n-triangle scene
__device__ __forceinline__ uint64_t tri_mask(int n, int g) {
    const int k = n - 64 * g;
    return k >= 64 ? ~0ull : (k <= 0 ? 0ull : ((1ull << k) - 1ull));
}

// The candidate triangles of the wave's camera rays: bit i of cm[i / 64] = triangle i may
// be the hit of a camera ray through one of the wave's pixels (the pixel rectangle's cull,
// rect_cull in rt_cull.hpp; wave-uniform).  k_render_ps phase P, k_render<MF> camera rays.
template <int RULE>
__device__ __forceinline__ void wave_candidates(const RenderLaunch& a, bool valid, int px, int py, int lane,
                                                uint64_t* cm) {
    int x0 = valid ? px : 0x7fffffff, x1 = valid ? px : -1;
    int y0 = valid ? py : 0x7fffffff, y1 = valid ? py : -1;
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        x0 = min(x0, __shfl_xor(x0, off, 64));
        x1 = max(x1, __shfl_xor(x1, off, 64));
        y0 = min(y0, __shfl_xor(y0, off, 64));
        y1 = max(y1, __shfl_xor(y1, off, 64));
    }
    const CamRect c = make_cam_rect(a.cam_x, a.cam_y, a.cam_z, a.cos_y, a.sin_y, a.width, a.height, a.t_scale,
                                    __builtin_amdgcn_readfirstlane(x0), __builtin_amdgcn_readfirstlane(x1),
                                    __builtin_amdgcn_readfirstlane(y0), __builtin_amdgcn_readfirstlane(y1));
    const int n_tri = a.scene.n_tri;
#pragma unroll
    for (int g = 0; g < kRenderCullWords; ++g) {
        if (g * 64 >= n_tri) {  // (wave-uniform) no triangle in this word
            cm[g] = 0ull;
            continue;
        }
        const int i = g * 64 + lane;
        const bool in_range = i < n_tri;
#ifdef RT_TIMING_NO_CULL
        const bool keep = in_range;
#else
        // every lane tests a real record (triangle 0 past the end), the range masks after
        const bool cull = rect_cull<RULE>(a.scene.filt + (size_t)(in_range ? i : 0) * kFiltF4, c);
        const bool keep = in_range && !cull;
#endif
        cm[g] = __ballot(keep) & tri_mask(n_tri, g);
    }
}

template <int PRESET, int SAMPLER, int RULE, bool STEAL, bool BVH, int MF = 0>
#ifndef RT_MIN_WAVES
#define RT_MIN_WAVES 1
#endif
#ifndef RT_MF_RENDER_WAVES
#define RT_MF_RENDER_WAVES 4  // occupancy floor of the MF variants (<= 128 VGPRs; 1: the compiler's 142-150)
#endif
__global__ __launch_bounds__(256, MF > 0 ? RT_MF_RENDER_WAVES : RT_MIN_WAVES) void k_render(const RenderLaunch a) {
    extern __shared__ float s_val[];  // STEAL: [pixel of the workgroup][spp][3]
    __shared__ int s_stk[BVH ? kBvhMaxDepth * 256 : 1];
    __shared__ float s_mfw[MF > 0 ? 4 * kMfWaveFloats : 1];  // MF: the waves' exact-phase LDS
    // workgroup -> (16x16 block, part); lane -> (pixel of the block, sample chunk)
    const int lg = a.split_log2;
    const BlockDesc blk = a.blocks[blockIdx.x >> lg];
    const int part = blockIdx.x & (a.split - 1);
    const int q = (part << (8 - lg)) + ((int)threadIdx.x >> lg);
    const int chunk = threadIdx.x & (a.split - 1);
    const int lane = threadIdx.x & 63;
    const int lx = q & 15;
    const int ly = q >> 4;
    const int px = blk.px0 + lx;
    const int py = blk.py0 + ly;
    const bool valid = (px < a.clip_x1) && (py < a.clip_y1);
    const uint32_t pix = (uint32_t)py * (uint32_t)a.width + (uint32_t)px;
    const float4* __restrict__ shade = a.scene.shade;
    const int n_surf = a.scene.n_surf;
    const int s_end = STEAL ? a.spp : (chunk + 1) * a.per_chunk;
    float* const pvals = STEAL ? s_val + (size_t)((int)threadIdx.x >> lg) * a.spp * 3 : nullptr;
    const int gbase = lane & ~(a.split - 1);  // first lane of this pixel's group
    const unsigned long long gmask = (a.split == 64) ? ~0ull : ((1ull << a.split) - 1ull);
    int next = a.split;                       // STEAL: the pixel's next unclaimed sample

    int s = valid ? (STEAL ? chunk : chunk * a.per_chunk) : s_end;  // current sample
    int depth = 0;              // surface bounces so far on this path
    f3 o = make3(a.cam_x, a.cam_y, a.cam_z);
    f3 d = make3(0.0f, 0.0f, 1.0f);
    f3 acc = make3(0.0f, 0.0f, 0.0f);
    f3 tp = make3(1.0f, 1.0f, 1.0f);     // PRESET 1 throughput
    int f_tri0 = 0, f_tri1 = 0;          // PRESET 0 factors (cap <= 2)
    float f_cos0 = 0.0f, f_cos1 = 0.0f;
    unsigned n_casts = 0;

    if (s < s_end) {
        float r1, r2;
        draw2(pix, (uint32_t)s, 0u, a.seed_lo, a.seed_hi, &r1, &r2);
        camera_ray<PRESET>(a, px, py, r1, r2, &d);
    }
    // MF with the camera outside the image's bound: camera rays take the wave's cull
    uint64_t cm[kRenderCullWords] = {0ull, 0ull, 0ull, 0ull};
    if (MF > 0 && a.cam_cull && __ballot(valid) != 0ull) wave_candidates<RULE>(a, valid, px, py, lane, cm);

    for (;;) {
        const bool active = s < s_end;
        if (__ballot(active) == 0ull) break;
        Hit h;
        if constexpr (MF > 0) {
            h = closest_hit_mf<RULE, false, MF>(a.scene, o, d, a.t_scale, active,
                                                s_mfw + ((int)threadIdx.x >> 6) * kMfWaveFloats, nullptr, nullptr,
                                                a.cam_cull ? cm : nullptr, depth == 0);
            if (!active) continue;
        } else {
            if (!active) continue;
            h = BVH ? closest_hit_bvh<RULE>(a.scene, o, d, a.t_scale, s_stk + threadIdx.x)
                    : closest_hit_sel<RULE>(a.scene, a.use_filter, o, d, a.t_scale);
        }
        ++n_casts;

        bool terminal = false;
        f3 L = make3(0.0f, 0.0f, 0.0f);
        if (h.tri < 0) {
            terminal = true;
            if (PRESET == 1) L = make3(tp.x * a.env_light, tp.y * a.env_light, tp.z * a.env_light);
        } else if (h.tri >= n_surf) {
            terminal = true;
            const float4 e = shade[h.tri * kShadeF4 + 3];
            if (PRESET == 0) {
                L = make3(e.x, e.y, e.z);
                if (depth >= 2) {
                    const float4 c = shade[f_tri1 * kShadeF4 + (SAMPLER == 0 ? 3 : 4)];
                    if (SAMPLER == 0) {
                        L.x = div_rho((L.x * c.x) * f_cos1);
                        L.y = div_rho((L.y * c.y) * f_cos1);
                        L.z = div_rho((L.z * c.z) * f_cos1);
                    } else {
                        L = make3(L.x * c.x, L.y * c.y, L.z * c.z);
                    }
                }
                if (depth >= 1) {
                    const float4 c = shade[f_tri0 * kShadeF4 + (SAMPLER == 0 ? 3 : 4)];
                    if (SAMPLER == 0) {
                        L.x = div_rho((L.x * c.x) * f_cos0);
                        L.y = div_rho((L.y * c.y) * f_cos0);
                        L.z = div_rho((L.z * c.z) * f_cos0);
                    } else {
                        L = make3(L.x * c.x, L.y * c.y, L.z * c.z);
                    }
                }
            } else {
                L = make3(tp.x * e.x, tp.y * e.y, tp.z * e.z);
            }
        } else if (PRESET == 0 && depth == a.max_bounces) {
            terminal = true;  // bounces == MAX_RAY_BOUNCES -> vec3(0)
        } else {
            // surface: position, sample a direction, update the estimator
            const float Dx = d.x * a.t_scale, Dy = d.y * a.t_scale, Dz = d.z * a.t_scale;
            const f3 pos = make3(o.x + h.t * Dx, o.y + h.t * Dy, o.z + h.t * Dz);
            const float4 N = shade[h.tri * kShadeF4 + 0];
            const float4 T = shade[h.tri * kShadeF4 + 1];
            const float4 B = shade[h.tri * kShadeF4 + 2];
            float r1, r2;
            draw2(pix, (uint32_t)s, 1u + (uint32_t)depth, a.seed_lo, a.seed_hi, &r1, &r2);
            float cos_theta, sin_theta;
            if (SAMPLER == 0) {
                cos_theta = r1;
                sin_theta = sqrtf(1.0f - r1 * r1);
            } else {
                cos_theta = sqrtf(r1);
                sin_theta = sqrtf(1.0f - r1);
            }
            float sphi, cphi;
            sincos_turn(r2, &sphi, &cphi);
            const float sx = sin_theta * cphi, sz = sin_theta * sphi;
            const f3 sd = make3((sx * B.x + cos_theta * N.x) + sz * T.x,
                                (sx * B.y + cos_theta * N.y) + sz * T.y,
                                (sx * B.z + cos_theta * N.z) + sz * T.z);
            if (PRESET == 0) {
                if (depth == 0) {
                    f_tri0 = h.tri;
                    f_cos0 = cos_theta;
                } else {
                    f_tri1 = h.tri;
                    f_cos1 = cos_theta;
                }
            } else {
                if (SAMPLER == 0) {
                    const float4 c = shade[h.tri * kShadeF4 + 3];
                    tp.x = div_rho((tp.x * c.x) * cos_theta);
                    tp.y = div_rho((tp.y * c.y) * cos_theta);
                    tp.z = div_rho((tp.z * c.z) * cos_theta);
                } else {
                    const float4 c = shade[h.tri * kShadeF4 + 4];
                    tp = make3(tp.x * c.x, tp.y * c.y, tp.z * c.z);
                }
            }
            o = make3(pos.x + kEps * sd.x, pos.y + kEps * sd.y, pos.z + kEps * sd.z);
            d = normalize(sd);
            ++depth;
            if (PRESET == 1 && depth == a.max_bounces) terminal = true;  // loop exhausted -> 0
        }

        if (STEAL) {
            const unsigned long long m = (__ballot(terminal) >> gbase) & gmask;
            if (terminal) {
                pvals[s * 3 + 0] = L.x;
                pvals[s * 3 + 1] = L.y;
                pvals[s * 3 + 2] = L.z;
                s = next + __popcll(m & ((1ull << chunk) - 1ull));
            }
            next += __popcll(m);
        }
        if (terminal) {
            if (!STEAL) {
                acc.x = acc.x + L.x;
                acc.y = acc.y + L.y;
                acc.z = acc.z + L.z;
                ++s;
            }
            depth = 0;
            tp = make3(1.0f, 1.0f, 1.0f);
            o = make3(a.cam_x, a.cam_y, a.cam_z);
            if (s < s_end) {
                float r1, r2;
                draw2(pix, (uint32_t)s, 0u, a.seed_lo, a.seed_hi, &r1, &r2);
                camera_ray<PRESET>(a, px, py, r1, r2, &d);
            }
        }
    }

    if (STEAL) {
        // every sample of the pixel was computed by a lane of this wave
        __syncthreads();
        if (valid) {
            for (int k = chunk * a.per_chunk; k < (chunk + 1) * a.per_chunk; ++k) {
                acc.x = acc.x + pvals[k * 3 + 0];
                acc.y = acc.y + pvals[k * 3 + 1];
                acc.z = acc.z + pvals[k * 3 + 2];
            }
        }
    }
    // fold the chunk sums of a pixel in chunk order: ((P0 + P1) + P2) + ...
    const int base = gbase;
    f3 tot = acc;
    for (int k = 1; k < a.split; ++k) {
        const float vx = __shfl(acc.x, base + k, 64);
        const float vy = __shfl(acc.y, base + k, 64);
        const float vz = __shfl(acc.z, base + k, 64);
        tot.x = tot.x + vx;
        tot.y = tot.y + vy;
        tot.z = tot.z + vz;
    }
    if (valid && chunk == 0) {
        const float fs = (float)a.spp;
        float* dst = a.out + ((size_t)(blk.oy0 + ly) * (size_t)a.out_pitch + (size_t)(blk.ox0 + lx)) * 3;
        store_rgb(dst, tot.x / fs, tot.y / fs, tot.z / fs);
    }
    if (a.casts != nullptr) {
        const unsigned total = wave_sum(n_casts);
        if (lane == 0) atomicAdd(a.casts, (unsigned long long)total);
    }
}

// ---- GPU preset: a persistent grid over a queue of (pixel, chunk) work items ----
// k_render gives each wave a fixed set of pixels: once their samples are out, the wave's
// lanes idle until its longest path (up to 80 casts) ends -- 3.21 MFMAs per cast against
// the 2.63 of full waves on complex_light_room, and sample stealing within the wave does
// not help.  Here a lane claims a chunk (pixel p, chunk c: samples
// [c m, (c + 1) m), m = spp / split) from a launch-wide queue, traces its samples one after
// another summing their values in sample order (k_render's fixed-chunk sum, bit for bit),
// stores the chunk sum and claims the next; lanes idle only at the end of the whole launch.
// k_fold_chunks then adds each pixel's chunk sums in chunk order (((P0 + P1) + P2) + ...)
// and divides by spp, as k_render's fold does.  The wave takes items 64 at a time from the
// global counter (one atomic per 64 chunks) and hands them to its lanes by ballot rank.
// Camera inside the matrix-core image's bound, MF > 0.
// CT: the casts take their candidates from tables instead of the matrix-core filter -- a
// camera ray the cull of its pixel's 16x4 rectangle (rect_cull, k_cull_ps over the launch's
// blocks, a.cull), a bounce ray the candidate table of the surface it leaves (ctab_candidates,
// rt_ctab.cpp) -- and closest_hit_cand tests them in index order: the same hit.
#ifndef RT_PQ_CT_WAVES
#define RT_PQ_CT_WAVES 8  // waves per SIMD of the table route's persistent grid (complex_light_room 2048^2 x 64: 4 / 6 / 8 -> 640 / 536 / 517 ms: its lookups' latency)
#endif
template <int SAMPLER, int RULE, int MF, bool CT = false>
__global__ __launch_bounds__(256, CT ? RT_PQ_CT_WAVES : RT_MF_RENDER_WAVES) void k_render_pq(const RenderLaunch a) {
    __shared__ __attribute__((aligned(16))) float s_mfw[4 * kMfWaveFloats];
    float* const wl = s_mfw + ((int)threadIdx.x >> 6) * kMfWaveFloats;
    const int lane = threadIdx.x & 63;
    const float4* __restrict__ shade = a.scene.shade;
    const int n_surf = a.scene.n_surf;
    const long long total = (long long)a.n_blocks * 256 * a.split;
    const f3 cam = make3(a.cam_x, a.cam_y, a.cam_z);
    long long qb = 0, qe = 0;  // wave-uniform: the wave's claimed, not yet handed out items
    bool exhausted = false;     // wave-uniform: the launch's queue is empty
    bool have = false;          // the lane holds a chunk
    long long item = 0;
    int s = 0, s_end = 0, px = 0, py = 0;
    uint32_t pix = 0;
    int depth = 0;
    int surf = -1, cidx = 0;  // CT: the surface the ray leaves; the pixel's rectangle in a.cull
    f3 o = cam, d = make3(0.0f, 0.0f, 1.0f), tp = make3(1.0f, 1.0f, 1.0f), acc = make3(0.0f, 0.0f, 0.0f);
    unsigned n_casts = 0;
    auto camera = [&]() {
        float r1, r2;
        draw2(pix, (uint32_t)s, 0u, a.seed_lo, a.seed_hi, &r1, &r2);
        camera_ray<1>(a, px, py, r1, r2, &d);
        o = cam;
        tp = make3(1.0f, 1.0f, 1.0f);
        depth = 0;
    };
    for (;;) {
        // lanes without a chunk take the next items of the queue
        if (!exhausted) {
            const uint64_t need = __ballot(!have);
            if (need != 0ull) {
                const int n_need = __builtin_popcountll(need);
                const int rank = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(need >> 32),
                                                                __builtin_amdgcn_mbcnt_lo((uint32_t)need, 0u));
                const long long avail = qe - qb;
                long long nb = 0;
                if (n_need > avail) {  // (wave-uniform) 64 more items
                    unsigned long long v = 0;
                    if (lane == 0) v = atomicAdd(a.work, 64ull);
                    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
                    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
                    nb = (long long)(((unsigned long long)hi << 32) | lo);
                }
                if (!have) {
                    const long long j = rank < avail ? qb + rank : nb + (rank - avail);
                    if (j < total) {
                        item = j;
                        const long long p = j >> a.split_log2;
                        const int c = (int)(j & (a.split - 1));
                        const BlockDesc blk = a.blocks[p >> 8];
                        const int q = (int)(p & 255);
                        px = blk.px0 + (q & 15);
                        py = blk.py0 + (q >> 4);
                        if (px < a.clip_x1 && py < a.clip_y1) {  // (a clipped pixel's chunks: nothing)
                            pix = (uint32_t)py * (uint32_t)a.width + (uint32_t)px;
                            cidx = (int)(p >> 8) * 4 + (q >> 6);
                            s = c * a.per_chunk;
                            s_end = s + a.per_chunk;
                            acc = make3(0.0f, 0.0f, 0.0f);
                            have = true;
                            camera();
                        }
                    }
                }
                if (n_need > avail) {
                    qb = nb + (n_need - avail);
                    qe = nb + 64;
                } else {
                    qb += n_need;
                }
                if (qb >= total) exhausted = true;
            }
        }
        const bool active = have;
        if (__ballot(active) == 0ull) {
            if (exhausted) break;
            continue;  // (every claimed item was a clipped pixel's)
        }
        Hit h;
        if constexpr (CT) {
            constexpr int NW = MF;
            uint64_t F[NW];
#pragma unroll
            for (int k = 0; k < NW; ++k) F[k] = 0ull;
            if (active && depth == 0) {
#pragma unroll
                for (int k = 0; k < NW; ++k)
                    F[k] = (k < kRenderCullWords) ? a.cull[(size_t)cidx * kRenderCullWords + k] : 0ull;
            } else if (active) {
                ctab_candidates<NW>(a.scene.ctab[RULE], a.scene.n_tri, n_surf, surf, o, d, F);
            }
            h = closest_hit_cand<RULE, NW>(a.scene, F, o, d, a.t_scale, wl);
        } else {
            h = closest_hit_mf<RULE, false, MF>(a.scene, o, d, a.t_scale, active, wl);
        }
        if (!active) continue;
        ++n_casts;
        bool terminal = false;
        f3 L = make3(0.0f, 0.0f, 0.0f);
        if (h.tri < 0) {
            terminal = true;
            L = make3(tp.x * a.env_light, tp.y * a.env_light, tp.z * a.env_light);
        } else if (h.tri >= n_surf) {
            terminal = true;
            const float4 e = shade[h.tri * kShadeF4 + 3];
            L = make3(tp.x * e.x, tp.y * e.y, tp.z * e.z);
        } else {
            // as k_render<1, ...>: position, sample a direction, update the throughput
            const float Dx = d.x * a.t_scale, Dy = d.y * a.t_scale, Dz = d.z * a.t_scale;
            const f3 pos = make3(o.x + h.t * Dx, o.y + h.t * Dy, o.z + h.t * Dz);
            const float4 N = shade[h.tri * kShadeF4 + 0];
            const float4 T = shade[h.tri * kShadeF4 + 1];
            const float4 B = shade[h.tri * kShadeF4 + 2];
            float r1, r2;
            draw2(pix, (uint32_t)s, 1u + (uint32_t)depth, a.seed_lo, a.seed_hi, &r1, &r2);
            float cos_theta, sin_theta;
            if (SAMPLER == 0) {
                cos_theta = r1;
                sin_theta = sqrtf(1.0f - r1 * r1);
            } else {
                cos_theta = sqrtf(r1);
                sin_theta = sqrtf(1.0f - r1);
            }
            float sphi, cphi;
            sincos_turn(r2, &sphi, &cphi);
            const float sx = sin_theta * cphi, sz = sin_theta * sphi;
            const f3 sd = make3((sx * B.x + cos_theta * N.x) + sz * T.x, (sx * B.y + cos_theta * N.y) + sz * T.y,
                                (sx * B.z + cos_theta * N.z) + sz * T.z);
            if (SAMPLER == 0) {
                const float4 c = shade[h.tri * kShadeF4 + 3];
                tp.x = div_rho((tp.x * c.x) * cos_theta);
                tp.y = div_rho((tp.y * c.y) * cos_theta);
                tp.z = div_rho((tp.z * c.z) * cos_theta);
            } else {
                const float4 c = shade[h.tri * kShadeF4 + 4];
                tp = make3(tp.x * c.x, tp.y * c.y, tp.z * c.z);
            }
            o = make3(pos.x + kEps * sd.x, pos.y + kEps * sd.y, pos.z + kEps * sd.z);
            d = normalize(sd);
            surf = h.tri;
            ++depth;
            if (depth == a.max_bounces) terminal = true;  // loop exhausted -> 0
        }
        if (terminal) {
            acc.x = acc.x + L.x;
            acc.y = acc.y + L.y;
            acc.z = acc.z + L.z;
            ++s;
            if (s < s_end) {
                camera();
            } else {
                store_rgb(a.csum + (size_t)item * 3, acc.x, acc.y, acc.z);
                have = false;
            }
        }
    }
    if (a.casts != nullptr) {
        const unsigned tot = wave_sum(n_casts);
        if (lane == 0) atomicAdd(a.casts, (unsigned long long)tot);
    }
}

// the pixels of k_render_pq's launch: chunk sums in chunk order, / spp (k_render's fold)
__global__ __launch_bounds__(256) void k_fold_chunks(const RenderLaunch a) {
    const long long p = (long long)blockIdx.x * 256 + threadIdx.x;
    if (p >= (long long)a.n_blocks * 256) return;
    const BlockDesc blk = a.blocks[p >> 8];
    const int q = (int)(p & 255), lx = q & 15, ly = q >> 4;
    if (blk.px0 + lx >= a.clip_x1 || blk.py0 + ly >= a.clip_y1) return;
    const float* c = a.csum + (size_t)p * a.split * 3;
    f3 tot = make3(c[0], c[1], c[2]);
    for (int k = 1; k < a.split; ++k) {
        tot.x = tot.x + c[3 * k + 0];
        tot.y = tot.y + c[3 * k + 1];
        tot.z = tot.z + c[3 * k + 2];
    }
    const float fs = (float)a.spp;
    float* dst = a.out + ((size_t)(blk.oy0 + ly) * (size_t)a.out_pitch + (size_t)(blk.ox0 + lx)) * 3;
    store_rgb(dst, tot.x / fs, tot.y / fs, tot.z / fs);
}

#ifndef RT_PQ_CTAB
#define RT_PQ_CTAB 1  // 0: k_render_pq's casts always on the matrix-core filter (A/B)
#endif
#ifndef RT_RENDER_PQ
#define RT_RENDER_PQ 1  // 0: the GPU preset's matrix-core renders keep the per-pixel k_render (A/B)
#endif

// k_render_ps: the CPU-engine preset (PRESET 0) in two phases per wave.
//
// Primary rays are a known family: the camera position and the pixel rectangle of the
// wave bound every direction, so a triangle whose filter certainly rejects all of them
// (rect_cull, rt_trace.hpp) cannot be hit by any of them.  Phase P traces every sample's
// primary ray of the lane against the few remaining candidates only (exact test, index
// order: the reference's hit bit for bit) and parks the result in LDS: the direction and
// hit of a path that continues, or the value of one that ends at its first cast.  Phase S
// is the bounce loop of k_render without camera rays: when a path ends, the lane takes
// its next sample's primary hit from LDS (adding the values of samples that ended at the
// first cast on the way, in sample order) and shades it, so every trip casts a secondary
// ray on every live lane.  The image, the ray casts and the sum order are those of
// k_render<0, ...> (oracle/ parity); PRESET 0 paths are 1-3 casts, so about 37% of the
// casts of the frame move from the full-scene scan to a few exact tests.
//
// LDS: per wave and sample slot k, three 64-lane float rows (lane-contiguous: conflict-free)
// and one int16 row of hit codes:
//   continuing: the hit point x, y, z, triangle;  ended: L.x, L.y, L.z, -1.
// (int16 codes: 13 KB of slots per 256-lane workgroup at 4 samples per lane instead of 16 KB --
// with the table route's pair list that is 25.6 KB per workgroup, six per CU)
#ifndef RT_PS_CODE16
#define RT_PS_CODE16 1  // the slots' hit codes as int16 beside three float rows (0: a fourth float row)
#endif
constexpr int kPsFields = RT_PS_CODE16 ? 3 : 4;  // float rows per sample slot

#ifndef RT_PS_PRIM_BATCH
#define RT_PS_PRIM_BATCH 4  // samples per candidate pass of phase P (1: one sample at a time)
#endif
#ifndef RT_PS_STEAL
#define RT_PS_STEAL 1  // 0: each lane bounces only its own samples (A/B builds)
#endif
#ifndef RT_PS_CTAB
#define RT_PS_CTAB 1  // 0: k_render_ps's bounce casts on the matrix-core image even with a candidate table (A/B)
#endif
#ifndef RT_PS_LIGHT_SPLIT
#define RT_PS_LIGHT_SPLIT 1  // 0: terminal casts always run the full closest hit (A/B builds)
#endif
constexpr int kPsSplitLights = 8;  // the light pre-test runs when the scene has at most this many light triangles
// floats of LDS per wave: the sample slots, then (RT_PS_STEAL) the wave's queue of
// continuing samples, one u16 (k << 6 | lane) per slot
__host__ __device__ constexpr int ps_wave_floats(int pc) {
    return pc * kPsFields * 64 + (RT_PS_CODE16 ? pc * 32 : 0) + (RT_PS_STEAL ? pc * 32 : 0);
}


// Candidate masks of the primary-ray phase: wave w of workgroup b writes
// cull[(b * 4 + w) * kRenderCullWords + g], bit j = triangle 64 g + j may be the hit of a
// camera ray through the wave's pixel rectangle (rect_cull, rt_trace.hpp).  Same grid
// and lane -> pixel mapping as k_render_ps.
// Candidate masks of the wave's pixel rectangle (the valid lanes' pixels): bit j of
// cm[g] = triangle 64 g + j may be the hit of a camera ray through the rectangle
// (rect_cull); never a bit past the scene.  All lanes of the wave take part.
// The masks alone, as k_render_ps computes them, into a.cull (wave w of workgroup b at
// words (b * 4 + w) * kRenderCullWords ..): the diagnostic rt_cull_masks_device.
template <int RULE>
__global__ __launch_bounds__(256) void k_cull_ps(const RenderLaunch a) {
    const int lg = a.split_log2;
    const BlockDesc blk = a.blocks[blockIdx.x >> lg];
    const int part = blockIdx.x & (a.split - 1);
    const int q = (part << (8 - lg)) + ((int)threadIdx.x >> lg);
    const int lane = threadIdx.x & 63;
    const int px = blk.px0 + (q & 15);
    const int py = blk.py0 + (q >> 4);
    const bool valid = (px < a.clip_x1) && (py < a.clip_y1);
    uint64_t cm[kRenderCullWords];
    if (__ballot(valid) == 0ull) {
        for (int g = 0; g < kRenderCullWords; ++g) cm[g] = 0ull;
    } else {
        wave_candidates<RULE>(a, valid, px, py, lane, cm);
    }
    unsigned long long* w = a.cull + ((size_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * kRenderCullWords;
    if (lane < kRenderCullWords) {
        uint64_t v = cm[0];
#pragma unroll
        for (int g = 1; g < kRenderCullWords; ++g) v = (lane == g) ? cm[g] : v;
        w[lane] = v;
    }
}

// the work of k_render_ps for one wave with at least one pixel; returns the lane's casts.
// CT: the bounce casts from the scene's candidate table (the launcher checked it serves this
// launch) -- the matrix-core path is not compiled in, so the kernel's registers allow more waves
template <int SAMPLER, int RULE, int MF, bool CT = false>
__device__ __forceinline__ unsigned ps_body(const RenderLaunch& a, const DeviceScene& ms, float* wl,
                                            const BlockDesc& blk, int q, int chunk, int lane, int lx, int ly, int px,
                                            int py, bool valid) {
    extern __shared__ float s_ps[];
    const uint32_t pix = (uint32_t)py * (uint32_t)a.width + (uint32_t)px;
    const float4* __restrict__ shade = ms.shade;  // (RT_PS_SCENE_LDS: the workgroup's LDS copy)
    const int n_surf = a.scene.n_surf;
    const int pc = a.per_chunk;
    float* const wslots = s_ps + (size_t)(threadIdx.x >> 6) * ps_wave_floats(pc);
    float* const slots = wslots + lane;
    // a slot's hit code: the triangle a continuing path's primary hit is on, or -1 (ended)
#if RT_PS_CODE16
    int16_t* const wcodes = reinterpret_cast<int16_t*>(wslots + pc * kPsFields * 64);
    auto code_at = [&](int kk, int ln) -> int { return (int)wcodes[kk * 64 + ln]; };
    auto set_code_at = [&](int kk, int ln, int c) { wcodes[kk * 64 + ln] = (int16_t)c; };
#else
    auto code_at = [&](int kk, int ln) -> int { return __float_as_int(wslots[(kk * kPsFields + 3) * 64 + ln]); };
    auto set_code_at = [&](int kk, int ln, int c) { wslots[(kk * kPsFields + 3) * 64 + ln] = __int_as_float(c); };
#endif
    const f3 cam = make3(a.cam_x, a.cam_y, a.cam_z);

    // ---- candidate triangles of the wave's pixel rectangle (rect_cull, rt_cull.hpp) ----
    uint64_t cm[kRenderCullWords];
    wave_candidates<RULE>(a, valid, px, py, lane, cm);

    // ---- phase P: primary rays of the lane's samples ----
    unsigned n_casts = 0;
#if RT_PROF
    uint64_t pt[6] = {0, 0, 0, 0, 0, 0};  // P, shade, filter masks, exact, post, loops
    uint64_t t0 = __builtin_amdgcn_s_memtime();
#endif
    const float nts = a.t_scale;
    cfloat4* __restrict__ isect = as_const(a.scene.isect);
    // parks sample k's primary result (the shading's pos = cam + t D, or the final value)
    auto park = [&](int k, const f3& d, const Hit& h) {
        n_casts += valid ? 1u : 0u;
        // a continuing path parks its hit point (the same operations the bounce loop's
        // shading used to apply to (cam, t, d): D = d t_scale, pos = cam + t D)
        float v0 = cam.x + h.t * (d.x * a.t_scale), v1 = cam.y + h.t * (d.y * a.t_scale),
              v2 = cam.z + h.t * (d.z * a.t_scale);
        int code = h.tri;
        if (h.tri < 0) {
            v0 = v1 = v2 = 0.0f;  // PRESET 0: a miss contributes 0
            code = -1;
        } else if (h.tri >= n_surf) {
            const float4 e = shade[h.tri * kShadeF4 + 3];
            v0 = e.x; v1 = e.y; v2 = e.z;  // the light's emission, no surface bounce to fold
            code = -1;
        } else if (a.max_bounces == 0) {
            v0 = v1 = v2 = 0.0f;
            code = -1;
        }
        float* sl = slots + k * kPsFields * 64;
        sl[0 * 64] = v0;
        sl[1 * 64] = v1;
        sl[2 * 64] = v2;
        set_code_at(k, lane, code);
    };
#if RT_PS_PRIM_BATCH > 1
    // The primary rays all start at the camera, so the cofactors of the exact test that
    // involve only b = cam - v0 and the edges (s3, s4, s6, det_t) are the same for every
    // sample of the wave: computed once per candidate for a batch of samples, each sample
    // then runs the direction-dependent rest (exact_one_c's operations on the same
    // operands in the same order: the same bits).  Samples of a batch fold the candidates
    // in index order each, as before.
    constexpr int PB = RT_PS_PRIM_BATCH;
    for (int k0 = 0; k0 < pc; k0 += PB) {
        f3 dd[PB];
        float nx[PB], ny[PB], nz[PB];
        Hit hh[PB];
#pragma unroll
        for (int j = 0; j < PB; ++j) {
            const int s = chunk * pc + min(k0 + j, pc - 1);
            float r1, r2;
            draw2(pix, (uint32_t)s, 0u, a.seed_lo, a.seed_hi, &r1, &r2);
            camera_ray<0>(a, px, py, r1, r2, &dd[j]);
            nx[j] = -(dd[j].x * nts);
            ny[j] = -(dd[j].y * nts);
            nz[j] = -(dd[j].z * nts);
            hh[j].t = (RULE == 0) ? FLT_MAX : 999999.0f;
            hh[j].tri = -1;
        }
#pragma unroll
        for (int g = 0; g < kRenderCullWords; ++g) {
            uint64_t m = cm[g];
            while (m != 0ull) {
                const int b = __builtin_ctzll(m);
                m &= m - 1ull;
                const int i = g * 64 + b;
                const float4 A = ldc(isect + i * kIsectF4 + 0);
                const float4 E1 = ldc(isect + i * kIsectF4 + 1);
                const float4 E2 = ldc(isect + i * kIsectF4 + 2);
                const float bx = cam.x - A.x, by = cam.y - A.y, bz = cam.z - A.z;
                const float s3 = by * E2.z - E2.y * bz;
                const float s4 = by * E1.z - E1.y * bz;
                const float det_t = (bx * A.w - E1.x * s3) + E2.x * s4;
                const float s6 = E1.y * bz - by * E1.z;
#pragma unroll
                for (int j = 0; j < PB; ++j) {
                    const float s1 = ny[j] * E2.z - E2.y * nz[j];
                    const float s2 = ny[j] * E1.z - E1.y * nz[j];
                    const float detA = (nx[j] * A.w - E1.x * s1) + E2.x * s2;
                    const float s5 = ny[j] * bz - by * nz[j];
                    const float det_u = (nx[j] * s3 - bx * s1) + E2.x * s5;
                    const float det_v = (nx[j] * s6 - E1.x * s5) + bx * s2;
                    exact_test<RULE>(detA, det_t, det_u, det_v, i, hh[j]);
                }
            }
        }
#pragma unroll
        for (int j = 0; j < PB; ++j)
            if (k0 + j < pc) park(k0 + j, dd[j], hh[j]);
    }
#else
    for (int k = 0; k < pc; ++k) {
        const int s = chunk * pc + k;
        float r1, r2;
        draw2(pix, (uint32_t)s, 0u, a.seed_lo, a.seed_hi, &r1, &r2);
        f3 d;
        camera_ray<0>(a, px, py, r1, r2, &d);
        const float nDx = -(d.x * nts), nDy = -(d.y * nts), nDz = -(d.z * nts);
        Hit h;
        h.t = (RULE == 0) ? FLT_MAX : 999999.0f;
        h.tri = -1;
#pragma unroll
        for (int g = 0; g < kRenderCullWords; ++g) {
            uint64_t m = cm[g];
            while (m != 0ull) {
                const int b = __builtin_ctzll(m);
                m &= m - 1ull;
                exact_one_c<RULE>(isect, g * 64 + b, cam, nDx, nDy, nDz, h);
            }
        }
        park(k, d, h);
    }
#endif

    // ---- phase S: bounces ----
#if RT_PROF
    const uint64_t t_s = __builtin_amdgcn_s_memtime();
    pt[0] += t_s - t0;
#endif
    f3 acc = make3(0.0f, 0.0f, 0.0f);
    int k = 0;          // next slot
    int cur = 0;        // sample of the live path
    int depth = 0;      // surface bounces of the live path so far
    f3 o = cam, d = make3(0.0f, 0.0f, 1.0f);
    f3 pos = cam;       // the live path's surface hit to shade next, and its triangle
    int hit_tri = 0;
    int f_tri0 = 0;
    float f_cos0 = 0.0f;
#if RT_PS_STEAL
    // The wave's continuing samples form one queue (slot-major: k, then lane), so a lane
    // whose path ends takes the next queued sample of any lane of the wave instead of
    // only its own: the wave runs ceil(casts / 64) trips instead of its busiest lane's.
    // A finished sample's value goes back into its slot; every lane then sums its own
    // slots in sample order (the fixed-chunk sum: the image is unchanged).
    uint16_t* const queue = reinterpret_cast<uint16_t*>(wslots + pc * kPsFields * 64 + (RT_PS_CODE16 ? pc * 32 : 0));
    int q_total = 0;
    for (int kk = 0; kk < pc; ++kk) {
        const bool cont = valid && code_at(kk, lane) >= 0;
        const uint64_t m = __ballot(cont);
        if (cont) queue[q_total + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                      __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u))] = (uint16_t)((kk << 6) | lane);
        q_total += __builtin_popcountll(m);
    }
    int q_next = 0;       // wave-uniform: next queue entry
    float* own = slots;   // slot of the live path's sample (any lane's)
    uint32_t lpix = pix;  // its pixel (RNG key)
    bool live = false;
    auto claim = [&]() {  // wave-level: lanes without a path take the next queued samples
        const uint64_t need = __ballot(!live);
        if (need == 0ull || q_next >= q_total) return;
        const int j = q_next + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(need >> 32),
                                                              __builtin_amdgcn_mbcnt_lo((uint32_t)need, 0u));
        if (!live && j < q_total) {
            const uint32_t e = queue[j];
            const int ol = (int)(e & 63u), kk = (int)(e >> 6);
            own = wslots + kk * kPsFields * 64 + ol;
            pos = make3(own[0 * 64], own[1 * 64], own[2 * 64]);
            hit_tri = code_at(kk, ol);
            depth = 0;
            const int oq = q - (lane >> a.split_log2) + (ol >> a.split_log2);  // the lane's pixel
            lpix = (uint32_t)(blk.py0 + (oq >> 4)) * (uint32_t)a.width + (uint32_t)(blk.px0 + (oq & 15));
            cur = (ol & (a.split - 1)) * pc + kk;
            live = true;
        }
        q_next = min(q_total, q_next + __builtin_popcountll(need));
    };
#endif
    // next continuing sample of the lane (adding the values of the ended ones in order)
    auto fetch = [&]() -> bool {
        while (k < pc) {
            const float* sl = slots + k * kPsFields * 64;
            const int code = code_at(k, lane);
            if (code < 0) {
                acc.x = acc.x + sl[0 * 64];
                acc.y = acc.y + sl[1 * 64];
                acc.z = acc.z + sl[2 * 64];
                ++k;
                continue;
            }
            pos = make3(sl[0 * 64], sl[1 * 64], sl[2 * 64]);
            hit_tri = code;
            depth = 0;
            cur = chunk * pc + k;
            ++k;
            return true;
        }
        return false;
    };
#if RT_PS_STEAL
    (void)fetch;
#else
    bool live = valid && fetch();
#endif
    // the bounce casts on the matrix cores when the scene has the image (wave-uniform)
    const bool use_mf = MF > 0;  // the launcher: MF = 64-triangle blocks of the scene (image present), else 0
    // scenes of at most 64 triangles: the candidates from the scene's table (rt_ctab.cpp) instead
    // of the image's masks (wave-uniform)
    constexpr bool use_ctab = CT && MF == 1;
    // the next direction from the surface hit (pos, hit_tri) at bounce depth dep: cos theta
    // and the ray (o = pos + eps sd, d = normalize(sd)), sampled with the path's Philox draw
    auto shade_hit = [&](int dep, float* cos_out, f3* o_out, f3* d_out) {
        const float4 N = shade[hit_tri * kShadeF4 + 0];
        const float4 T = shade[hit_tri * kShadeF4 + 1];
        const float4 B = shade[hit_tri * kShadeF4 + 2];
        float r1, r2;
#if RT_PS_STEAL
        draw2(lpix, (uint32_t)cur, 1u + (uint32_t)dep, a.seed_lo, a.seed_hi, &r1, &r2);
#else
        draw2(pix, (uint32_t)cur, 1u + (uint32_t)dep, a.seed_lo, a.seed_hi, &r1, &r2);
#endif
        float cos_theta, sin_theta;
        if (SAMPLER == 0) {
            cos_theta = r1;
            sin_theta = sqrtf(1.0f - r1 * r1);
        } else {
            cos_theta = sqrtf(r1);
            sin_theta = sqrtf(1.0f - r1);
        }
        float sphi, cphi;
        sincos_turn(r2, &sphi, &cphi);
        const float sx = sin_theta * cphi, sz = sin_theta * sphi;
        const f3 sd = make3((sx * B.x + cos_theta * N.x) + sz * T.x,
                            (sx * B.y + cos_theta * N.y) + sz * T.y,
                            (sx * B.z + cos_theta * N.z) + sz * T.z);
        *cos_out = cos_theta;
        *o_out = make3(pos.x + kEps * sd.x, pos.y + kEps * sd.y, pos.z + kEps * sd.z);
        *d_out = normalize(sd);
    };
    // Light pre-test (RT_PS_LIGHT_SPLIT).  The terminal cast of a path (the one at depth
    // max_bounces) adds light only if its closest hit is a light triangle; a surface or a miss
    // there gives 0.  If no light triangle passes the exact test without its t window
    // (exact_tv: the full test's own operations), the closest hit cannot be a light, and the
    // cast's value is 0 whatever the surfaces are.  So when a cast leaves a path whose next
    // cast is terminal, the lane samples that next ray at once and tests only the light
    // triangles: no pass -> the path ends with 0 (the terminal cast counted); a pass (a few
    // percent of rays) -> the path stays live and the next trip traces the same ray (same
    // Philox draw) in full.  Terminal casts thus stop taking slots of the matrix-core trips:
    // the image and the ray casts are k_render's bit for bit.
    const bool split = RT_PS_LIGHT_SPLIT && use_mf && a.max_bounces >= 1 &&
                       (a.scene.n_tri - n_surf) <= kPsSplitLights;
    // the pre-test of the terminal ray from (pos, hit_tri) at depth dep = max_bounces - 1
    auto light_pass = [&](int dep) -> bool {
        float c;
        f3 lo, ld;
        shade_hit(dep, &c, &lo, &ld);
        const float nDx = -(ld.x * a.t_scale), nDy = -(ld.y * a.t_scale), nDz = -(ld.z * a.t_scale);
        bool pass = false;
        for (int j = n_surf; j < a.scene.n_tri; ++j)
            pass |= exact_tv<RULE>(ms.isect, j, lo, nDx, nDy, nDz) != __builtin_inff();
        return pass;
    };
    for (;;) {
#if RT_PS_STEAL
        claim();
#endif
        if (__ballot(live) == 0ull) break;
        if (!use_mf && !live) continue;
#if RT_PROF
        const uint64_t ta = __builtin_amdgcn_s_memtime();
        pt[5] += 1;
#endif
        int s_tri = 0;
        float s_cos = 0.0f;
        if (live) {
            // shade the live path's surface hit (depth < max_bounces by construction)
            s_tri = hit_tri;
            shade_hit(depth, &s_cos, &o, &d);
            if (depth == 0) {
                f_tri0 = s_tri;
                f_cos0 = s_cos;
            }
            ++depth;
        }
        // every lane of the wave takes part in the matrix-core filter; a lane without a
        // live path casts its stale (finite) ray with no candidates
#if RT_PROF
        const uint64_t tb = __builtin_amdgcn_s_memtime();
        uint64_t tm = tb;
#endif
        Hit h;
        if constexpr (use_ctab)
            h = closest_hit_ctab<RULE, 1, kCtPairCap>(ms, ms.ctab[RULE], s_tri, o, d, a.t_scale, live, wl);
        else if (use_mf)
#if RT_PROF
            h = closest_hit_mf<RULE, false, (MF > 0 ? MF : 1)>(ms, o, d, a.t_scale, live, wl, nullptr, &tm);
#else
            h = closest_hit_mf<RULE, false, (MF > 0 ? MF : 1)>(ms, o, d, a.t_scale, live, wl);
#endif
        else
            h = closest_hit_sel<RULE>(a.scene, 1, o, d, a.t_scale);
#if RT_PROF
        const uint64_t tc = __builtin_amdgcn_s_memtime();
        pt[1] += tb - ta;
        pt[2] += tm - tb;
        pt[3] += tc - tm;
#endif
        if (!live) continue;
        ++n_casts;

        bool terminal = true;
        f3 L = make3(0.0f, 0.0f, 0.0f);
        if (h.tri < 0) {
            // miss: 0
        } else if (h.tri >= n_surf) {
            const float4 e = shade[h.tri * kShadeF4 + 3];
            L = make3(e.x, e.y, e.z);
            // fold back through the surface bounces: depth 2 (this shading), then depth 1
            if (depth >= 2) {
                const float4 c = shade[s_tri * kShadeF4 + (SAMPLER == 0 ? 3 : 4)];
                if (SAMPLER == 0) {
                    L.x = div_rho((L.x * c.x) * s_cos);
                    L.y = div_rho((L.y * c.y) * s_cos);
                    L.z = div_rho((L.z * c.z) * s_cos);
                } else {
                    L = make3(L.x * c.x, L.y * c.y, L.z * c.z);
                }
            }
            {
                const float4 c = shade[f_tri0 * kShadeF4 + (SAMPLER == 0 ? 3 : 4)];
                if (SAMPLER == 0) {
                    L.x = div_rho((L.x * c.x) * f_cos0);
                    L.y = div_rho((L.y * c.y) * f_cos0);
                    L.z = div_rho((L.z * c.z) * f_cos0);
                } else {
                    L = make3(L.x * c.x, L.y * c.y, L.z * c.z);
                }
            }
        } else if (depth == a.max_bounces) {
            // bounces == MAX_RAY_BOUNCES -> vec3(0)
        } else {
            terminal = false;  // shade the hit on the next trip
            pos = make3(o.x + h.t * (d.x * a.t_scale), o.y + h.t * (d.y * a.t_scale), o.z + h.t * (d.z * a.t_scale));
            hit_tri = h.tri;
            if (split && depth + 1 == a.max_bounces && !light_pass(depth)) {
                ++n_casts;  // the terminal cast: no light triangle can be its hit
                terminal = true;
            }
        }
        if (terminal) {
#if RT_PS_STEAL
            own[0 * 64] = L.x;
            own[1 * 64] = L.y;
            own[2 * 64] = L.z;
            live = false;
#else
            acc.x = acc.x + L.x;
            acc.y = acc.y + L.y;
            acc.z = acc.z + L.z;
            live = fetch();
#endif
        }
    }
#if RT_PS_STEAL
    // the lane's own samples in order: ended ones hold their value in fields 0..2
    for (int kk = 0; kk < pc; ++kk) {
        const float* sl = slots + kk * kPsFields * 64;
        acc.x = acc.x + sl[0 * 64];
        acc.y = acc.y + sl[1 * 64];
        acc.z = acc.z + sl[2 * 64];
    }
#endif

#if RT_PROF
    pt[4] = __builtin_amdgcn_s_memtime() - t_s;  // the whole bounce phase
    if (a.prof != nullptr && lane == 0) {
        for (int i = 0; i < 6; ++i) atomicAdd(a.prof + i, (unsigned long long)pt[i]);
    }
#endif
    // fold the chunk sums of a pixel in chunk order: ((P0 + P1) + P2) + ...
    const int base = lane & ~(a.split - 1);
    f3 tot = acc;
    for (int kk = 1; kk < a.split; ++kk) {
        const float vx = __shfl(acc.x, base + kk, 64);
        const float vy = __shfl(acc.y, base + kk, 64);
        const float vz = __shfl(acc.z, base + kk, 64);
        tot.x = tot.x + vx;
        tot.y = tot.y + vy;
        tot.z = tot.z + vz;
    }
    if (valid && chunk == 0) {
        const float fs = (float)a.spp;
        float* dst = a.out + ((size_t)(blk.oy0 + ly) * (size_t)a.out_pitch + (size_t)(blk.ox0 + lx)) * 3;
        store_rgb(dst, tot.x / fs, tot.y / fs, tot.z / fs);
    }
    return n_casts;
}

#ifndef RT_PS_MIN_WAVES
#define RT_PS_MIN_WAVES 4  // the matrix-core filter's operands: ~99 VGPRs
#endif
#ifndef RT_PS_CT_WAVES
// occupancy floor of the table-route variant: 6 (80 VGPRs, 7 spilled) -- with the int16 slot codes
// its workgroup takes 26.7 KB of LDS and six fit a CU (Cornell 512^2 x 256: 2.39 -> 2.24 ms,
// profiles/r6v/; at the 28.7-KB layout LDS held it to five and 6 only added spills)
#define RT_PS_CT_WAVES 6
#endif
template <int SAMPLER, int RULE, int MF, bool CT = false>
__global__ __launch_bounds__(256, CT ? RT_PS_CT_WAVES : RT_PS_MIN_WAVES) void k_render_ps(const RenderLaunch a) {
    const int lg = a.split_log2;
    const BlockDesc blk = a.blocks[blockIdx.x >> lg];
    // XCD-aware parts: workgroups go to the 8 XCDs round-robin by blockIdx, so the
    // workgroups of one XCD take consecutive parts (whole pixel rows of the block) and a
    // row's output lines are written through one XCD's L2 instead of eight
    int part = blockIdx.x & (a.split - 1);
    if (a.split >= 8) part = ((part & 7) << (lg - 3)) | (part >> 3);
    const int q = (part << (8 - lg)) + ((int)threadIdx.x >> lg);
    const int chunk = threadIdx.x & (a.split - 1);
    const int lane = threadIdx.x & 63;
    const int lx = q & 15;
    const int ly = q >> 4;
    const int px = blk.px0 + lx;
    const int py = blk.py0 + ly;
    const bool valid = (px < a.clip_x1) && (py < a.clip_y1);
    const uint64_t vmask = __ballot(valid);
    // ray casts: one atomic per workgroup (a wave's count through LDS, one barrier at the
    // end; every wave reaches it, a wave without pixels contributes 0): one atomic per
    // wave put 16 MB per launch of atomic write traffic on a 3 MB frame
    __shared__ unsigned wg_casts[4];
    // LDS after the sample slots (launch_render_t sizes it): the waves' exact-phase
    // regions, then (RT_MF_LDS) the matrix-core filter's image
    DeviceScene ms = a.scene;
    float* wl = nullptr;
    if (MF > 0) {
        extern __shared__ float s_ps[];
        float* const mf_base = s_ps + (size_t)4 * ps_wave_floats(a.per_chunk);
        // (the table route's wave blocks hold a shorter pair list: mf_wave_floats)
        constexpr int wf = CT ? mf_wave_floats(kCtPairCap, RULE) : kMfWaveFloats;
        wl = mf_base + (size_t)(threadIdx.x >> 6) * wf;
        float* next = mf_base + 4 * wf;
#if RT_PS_SCENE_LDS
        // hit-test and shading records of the scene (divergent per-lane reads: LDS latency
        // instead of L1/L2)
        {
            const int n = a.scene.n_tri;
            float4* li = reinterpret_cast<float4*>(next);
            float4* ls = li + (size_t)n * kIsectF4;
            for (int i = threadIdx.x; i < n * kIsectF4; i += 256) li[i] = a.scene.isect[i];
            ms.isect = li;
            constexpr bool shade_lds = RT_PS_SHADE_LDS && (!CT || RT_PS_CT_SHADE_LDS);
            if (shade_lds) {
                for (int i = threadIdx.x; i < n * kShadeF4; i += 256) ls[i] = a.scene.shade[i];
                ms.shade = ls;
            }
            next = reinterpret_cast<float*>(ls + (shade_lds ? (size_t)n * kShadeF4 : 0));
        }
#endif
#if RT_PS_CT_TRI_LDS
        // the table's surface patch frames (the first link of every bounce cast's lookup chain:
        // frame -> patch and bin -> mask words): from LDS instead of L1/L2
        if constexpr (CT) {
            float4* lt = reinterpret_cast<float4*>(next);
            const int m = a.scene.n_surf * 4;
            for (int i = threadIdx.x; i < m; i += 256) lt[i] = a.scene.ctab[RULE].tri[i];
            ms.ctab[RULE].tri = lt;
            next = reinterpret_cast<float*>(lt + m);
        }
#endif
#if RT_PS_CT_DICT_LDS
        // the grazing masks' dictionary (a few dozen words): the last link of the lookup chain in LDS
        if constexpr (CT) {
            const CtabDev& T = a.scene.ctab[RULE];
            if (T.n_gdict <= kPsCtDictLds) {
                unsigned long long* ld = reinterpret_cast<unsigned long long*>(next);
                for (int i = threadIdx.x; i < T.n_gdict; i += 256) ld[i] = T.gdict[i];
                ms.ctab[RULE].gdict = ld;
            }
            next += 2 * kPsCtDictLds;
        }
#endif
#if RT_MF_LDS
        if (!CT) {
            const int ng = mf_groups(a.scene.n_tri);
            uint4* lf = reinterpret_cast<uint4*>(next);
            for (int i = threadIdx.x; i < ng * 64; i += 256) lf[i] = a.scene.mf_frag[i];
            ms.mf_frag = lf;
        }
#endif
        if (RT_PS_SCENE_LDS || (RT_MF_LDS && !CT) || ((RT_PS_CT_TRI_LDS || RT_PS_CT_DICT_LDS) && CT)) __syncthreads();
    }
    const unsigned n_casts =
        (vmask == 0ull) ? 0u : ps_body<SAMPLER, RULE, MF, CT>(a, ms, wl, blk, q, chunk, lane, lx, ly, px, py, valid);
    if (a.casts != nullptr) {
        const unsigned total = wave_sum(n_casts);
        if (lane == 0) wg_casts[threadIdx.x >> 6] = total;
        __syncthreads();
        if (threadIdx.x == 0)
            atomicAdd(a.casts, (unsigned long long)((wg_casts[0] + wg_casts[1]) + (wg_casts[2] + wg_casts[3])));
    }
}

// Exhaustive check of rcp_rn against IEEE division: thread g covers the
// 4096 bit patterns [g*4096, (g+1)*4096).  Counts mismatches (ignoring NaN
// payloads) and keeps the smallest mismatching pattern.
// WHICH = RT_SELFTEST_RCP: rcp_rn(x) vs IEEE 1.0f / x over all 2^32 floats;
// RT_SELFTEST_DIV12: div12(x) vs x / 12.0f over its domain (+0, |x| in [2^-100, 2^100]);
// RT_SELFTEST_DIVRHO: div_rho(x) vs x / RHO over all 2^32 floats (its fallback included).
// NaNs compare equal to NaNs.
constexpr int kSelfRcp = 1, kSelfDiv12 = 2, kSelfDivRho = 3;  // RT_SELFTEST_* (rtmi.h)

template <int WHICH>
__global__ __launch_bounds__(256) void k_selftest(unsigned long long* mism, unsigned* first) {
    const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    unsigned bad = 0;
    for (uint32_t k = 0; k < 4096u; ++k) {
        const uint32_t bits = (uint32_t)(g * 4096u + k);
        const float x = __uint_as_float(bits);
        float a, b;
        if constexpr (WHICH == kSelfRcp) {
            a = rcp_rn(x);
            b = 1.0f / x;
        } else if constexpr (WHICH == kSelfDiv12) {
            const float ax = fabsf(x);
            if (!(bits == 0u || (ax >= 0x1p-100f && ax <= 0x1p100f))) continue;
            a = div12(x);
            b = x / 12.0f;
        } else {
            constexpr float rho = 1.0f / (2.0f * 3.14159265358979323846f);
            a = div_rho(x);
            b = x / rho;
        }
        const bool same = (__float_as_uint(a) == __float_as_uint(b)) || (a != a && b != b);
        if (!same) {
            ++bad;
            atomicMin(first, bits);
        }
    }
    if (bad) atomicAdd(mism, (unsigned long long)bad);
}

}  // namespace

hipError_t launch_selftest(int which, unsigned long long* mism, unsigned* first, hipStream_t stream) {
    if (which == kSelfRcp)
        hipLaunchKernelGGL(k_selftest<kSelfRcp>, dim3(4096), dim3(256), 0, stream, mism, first);
    else if (which == kSelfDiv12)
        hipLaunchKernelGGL(k_selftest<kSelfDiv12>, dim3(4096), dim3(256), 0, stream, mism, first);
    else if (which == kSelfDivRho)
        hipLaunchKernelGGL(k_selftest<kSelfDivRho>, dim3(4096), dim3(256), 0, stream, mism, first);
    else
        return hipErrorInvalidValue;
    return hipGetLastError();
}

hipError_t launch_intersect(const DeviceScene& s, const float* orig, const float* dir, int n,
                            float t_scale, int hit_rule, int use_filter, float* out_t,
                            int32_t* out_hit, hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    const dim3 block(256);
    const dim3 grid((unsigned)((n + 255) / 256));
    if (hit_rule == 0) {
        hipLaunchKernelGGL(k_intersect<0>, grid, block, 0, stream, s, use_filter, s.code_cpu, orig, dir,
                           n, t_scale, out_t, out_hit);
    } else {
        hipLaunchKernelGGL(k_intersect<1>, grid, block, 0, stream, s, use_filter, s.code_gpu, orig, dir,
                           n, t_scale, out_t, out_hit);
    }
    return hipGetLastError();
}

hipError_t launch_intersect_bvh(const DeviceScene& s, const float* orig, const float* dir, int n, float t_scale,
                                int hit_rule, float* out_t, int32_t* out_hit, hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    if (s.bvh_nodes == nullptr) return hipErrorInvalidValue;
    const dim3 block(256), grid((unsigned)((n + 255) / 256));
    if (hit_rule == 0)
        hipLaunchKernelGGL(k_intersect_bvh<0>, grid, block, 0, stream, s, s.code_cpu, orig, dir, n, t_scale, out_t,
                           out_hit);
    else
        hipLaunchKernelGGL(k_intersect_bvh<1>, grid, block, 0, stream, s, s.code_gpu, orig, dir, n, t_scale, out_t,
                           out_hit);
    return hipGetLastError();
}

hipError_t launch_intersect_mf(const DeviceScene& s, const float* orig, const float* dir, int n, float t_scale,
                               int hit_rule, float* out_t, int32_t* out_hit, int32_t* cand, hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    if (s.mf_frag == nullptr || !(t_scale > 0.0f && t_scale <= kFiltMaxTScale))
        return hipErrorInvalidValue;
    const dim3 block(256);
    const dim3 grid((unsigned)((n + 255) / 256));
    if (hit_rule == 0)
        hipLaunchKernelGGL(k_intersect_mf<0>, grid, block, 0, stream, s, s.code_cpu, orig, dir, n, t_scale, out_t,
                           out_hit, cand);
    else
        hipLaunchKernelGGL(k_intersect_mf<1>, grid, block, 0, stream, s, s.code_gpu, orig, dir, n, t_scale, out_t,
                           out_hit, cand);
    return hipGetLastError();
}

#ifndef RT_MF_RENDER
#define RT_MF_RENDER 1  // 0: the GPU preset's casts on the fp32 filter (A/B builds)
#endif
#ifndef RT_CAM_CULL
#define RT_CAM_CULL 1  // 0: a camera outside the image's bound keeps the fp32 filter (A/B builds)
#endif
#ifndef RT_STEAL_MAX_LDS
#define RT_STEAL_MAX_LDS (64 * 1024)  // sample stealing when its LDS fits (0: never)
#endif

// Sample stealing pays where path lengths vary (GPU preset, up to 80 casts: Cornell
// +24%, complex_light_room +32%); with the CPU preset's cap of 3 casts the lanes stay
// in step and it costs 1%, so that preset keeps the fixed chunks.
#ifndef RT_PS
#define RT_PS 1  // 0: the CPU preset without the primary-ray phase (A/B builds)
#endif
#ifndef RT_PS_MAX_LDS
#define RT_PS_MAX_LDS (40 * 1024)  // per workgroup: 8 samples per lane
#endif

template <int PRESET, int SAMPLER, int RULE>
static void launch_render_t(const RenderLaunch& a, hipStream_t stream) {
    if (PRESET == 0 && RT_PS && a.use_filter && a.scene.n_tri <= 64 * kRenderCullWords &&
        a.scene.bvh_nodes == nullptr) {
        const size_t ps_lds = (size_t)4 * ps_wave_floats(a.per_chunk) * sizeof(float);
        if (ps_lds <= (size_t)RT_PS_MAX_LDS) {
            // the bounce casts from the scene's candidate table (rt_ctab.cpp) when it serves this
            // launch: one mask word, this build's bins, t_scale >= its ts_min
            const CtabDev& T = a.scene.ctab[RULE];
            const bool ct = RT_PS_CTAB && RT_MF && a.scene.mf_frag != nullptr && a.scene.n_tri <= 64 &&
                            T.masks != nullptr && T.bins == kCtabBins && T.graze_n == kCtabGraze &&
                            a.t_scale >= T.ts_min && T.words == 1;
            size_t mf_lds = 0;
            if (RT_MF && a.scene.mf_frag != nullptr) {
                mf_lds = (size_t)4 * (ct ? mf_wave_floats(kCtPairCap, RULE) : kMfWaveFloats) * sizeof(float);
                if (RT_PS_SCENE_LDS)
                    mf_lds += (size_t)a.scene.n_tri *
                              (kIsectF4 + (RT_PS_SHADE_LDS && (!ct || RT_PS_CT_SHADE_LDS) ? kShadeF4 : 0)) * sizeof(float4);
                if (RT_MF_LDS && !ct) mf_lds += (size_t)mf_groups(a.scene.n_tri) * 64 * sizeof(uint4);
                if (RT_PS_CT_TRI_LDS && ct) mf_lds += (size_t)a.scene.n_surf * 4 * sizeof(float4);
                if (RT_PS_CT_DICT_LDS && ct) mf_lds += (size_t)kPsCtDictLds * sizeof(uint64_t);
            }
            const dim3 grid((unsigned)(a.n_blocks * a.split));
            KernelTimer kt(KT_RENDER_PS, stream);
            if (ct)
                hipLaunchKernelGGL((k_render_ps<SAMPLER, RULE, 1, true>), grid, dim3(256), ps_lds + mf_lds, stream, a);
            else if (mf_lds > 0 && a.scene.n_tri <= 64)
                hipLaunchKernelGGL((k_render_ps<SAMPLER, RULE, 1>), grid, dim3(256), ps_lds + mf_lds, stream, a);
            else if (mf_lds > 0)
                hipLaunchKernelGGL((k_render_ps<SAMPLER, RULE, 4>), grid, dim3(256), ps_lds + mf_lds, stream, a);
            else
                hipLaunchKernelGGL((k_render_ps<SAMPLER, RULE, 0>), grid, dim3(256), ps_lds, stream, a);
            return;
        }
    }
    const size_t lds = (size_t)(256 / a.split) * (size_t)a.spp * 3 * sizeof(float);
    const dim3 grid((unsigned)(a.n_blocks * a.split));
    const bool steal = PRESET == 1 && lds <= (size_t)RT_STEAL_MAX_LDS;
    KernelTimer kt(KT_RENDER, stream);
    // the GPU preset's casts on the matrix-core filter: when the scene has the image and
    // the camera is inside its origin bound (camera rays then get real masks)
    const float cb = a.scene.mf_bound;
    const bool mf_base = PRESET == 1 && RT_MF_RENDER && a.use_filter && a.scene.mf_frag != nullptr &&
                         a.scene.bvh_nodes == nullptr && a.t_scale > 0.0f && a.t_scale <= kFiltMaxTScale;
    const bool cam_in = fabsf(a.cam_x) <= cb && fabsf(a.cam_y) <= cb && fabsf(a.cam_z) <= cb;
    // a camera outside the bound: its rays take the wave's primary-ray cull (rt_cull.hpp),
    // which models the CPU preset's camera -- the GPU preset's is the same ray when the
    // pitch is 0 (camera_ray: the second rotation is the identity, exactly)
    const bool cam_cull = !cam_in && RT_CAM_CULL && a.scene.n_tri <= 64 * kRenderCullWords &&
                          a.cos_x == 1.0f && a.sin_x == 0.0f;
    const bool mf = mf_base && (cam_in || cam_cull);
    if (mf) {
        if (PRESET == 1) {  // (the CPU preset runs k_render_ps)
            RenderLaunch b = a;
            b.cam_cull = cam_in ? 0 : 1;
            const bool one = a.scene.n_tri <= 64;
            if (RT_RENDER_PQ && cam_in && a.csum != nullptr && a.work != nullptr) {
                (void)hipMemsetAsync(a.work, 0, sizeof(unsigned long long), stream);
                // a persistent grid: as many workgroups as the device holds at 4 waves per SIMD
                const unsigned wgs = (unsigned)min(a.n_blocks * a.split, RT_MF_RENDER_WAVES * device_cu_count());
                // the table route (k_render_pq CT): the scene's candidate table for this hit rule and
                // t_scale, and the camera rays' rectangle cull -- CPU-preset camera geometry, i.e.
                // pitch 0 (camera_ray: the second rotation is then the identity, exactly)
                const CtabDev& T = a.scene.ctab[RULE];
                const bool ct = RT_PQ_CTAB && a.cull != nullptr && a.cos_x == 1.0f && a.sin_x == 0.0f &&
                                a.scene.n_tri <= 64 * kRenderCullWords && T.masks != nullptr && T.bins == kCtabBins &&
                                T.graze_n == kCtabGraze && a.t_scale >= T.ts_min && T.words <= (one ? 1 : 4);
                if (ct) {
                    RenderLaunch c = b;  // one workgroup per 16x16 block: the masks of its four 16x4 rectangles
                    c.split = 1;
                    c.split_log2 = 0;
                    hipLaunchKernelGGL((k_cull_ps<RULE>), dim3((unsigned)a.n_blocks), dim3(256), 0, stream, c);
                    const unsigned wct = (unsigned)min(a.n_blocks * a.split, RT_PQ_CT_WAVES * device_cu_count());
                    if (one)
                        hipLaunchKernelGGL((k_render_pq<SAMPLER, RULE, 1, true>), dim3(wct), dim3(256), 0, stream, b);
                    else
                        hipLaunchKernelGGL((k_render_pq<SAMPLER, RULE, 4, true>), dim3(wct), dim3(256), 0, stream, b);
                } else if (one)
                    hipLaunchKernelGGL((k_render_pq<SAMPLER, RULE, 1>), dim3(wgs), dim3(256), 0, stream, b);
                else
                    hipLaunchKernelGGL((k_render_pq<SAMPLER, RULE, 4>), dim3(wgs), dim3(256), 0, stream, b);
                hipLaunchKernelGGL(k_fold_chunks, dim3((unsigned)a.n_blocks), dim3(256), 0, stream, b);
                return;
            }
            if (steal && one)
                hipLaunchKernelGGL((k_render<PRESET, SAMPLER, RULE, true, false, 1>), grid, dim3(256), lds, stream, b);
            else if (steal)
                hipLaunchKernelGGL((k_render<PRESET, SAMPLER, RULE, true, false, 4>), grid, dim3(256), lds, stream, b);
            else if (one)
                hipLaunchKernelGGL((k_render<PRESET, SAMPLER, RULE, false, false, 1>), grid, dim3(256), 0, stream, b);
            else
                hipLaunchKernelGGL((k_render<PRESET, SAMPLER, RULE, false, false, 4>), grid, dim3(256), 0, stream, b);
        }
        return;
    }
    if (a.scene.bvh_nodes != nullptr) {
        if (steal)
            hipLaunchKernelGGL((k_render<PRESET, SAMPLER, RULE, true, true>), grid, dim3(256), lds, stream, a);
        else
            hipLaunchKernelGGL((k_render<PRESET, SAMPLER, RULE, false, true>), grid, dim3(256), 0, stream, a);
    } else if (steal) {
        hipLaunchKernelGGL((k_render<PRESET, SAMPLER, RULE, true, false>), grid, dim3(256), lds, stream, a);
    } else {
        hipLaunchKernelGGL((k_render<PRESET, SAMPLER, RULE, false, false>), grid, dim3(256), 0, stream, a);
    }
}

hipError_t launch_cull(const RenderLaunch& a, hipStream_t stream) {
    if (a.n_blocks <= 0 || a.cull == nullptr || a.scene.filt == nullptr) return hipErrorInvalidValue;
    if (a.hit_rule == 0)
        hipLaunchKernelGGL((k_cull_ps<0>), dim3((unsigned)(a.n_blocks * a.split)), dim3(256), 0, stream, a);
    else
        hipLaunchKernelGGL((k_cull_ps<1>), dim3((unsigned)(a.n_blocks * a.split)), dim3(256), 0, stream, a);
    return hipGetLastError();
}

hipError_t launch_render(const RenderLaunch& a, hipStream_t stream) {
    if (a.n_blocks <= 0) return hipSuccess;
    if (a.preset == 0 && a.max_bounces > 2) return hipErrorInvalidValue;
    if (a.split < 1 || a.split > 64 || (a.split & (a.split - 1)) != 0 || (1 << a.split_log2) != a.split ||
        a.per_chunk * a.split != a.spp)
        return hipErrorInvalidValue;
    const int key = a.preset * 4 + a.sampler * 2 + a.hit_rule;
    switch (key) {
        case 0: launch_render_t<0, 0, 0>(a, stream); break;
        case 1: launch_render_t<0, 0, 1>(a, stream); break;
        case 2: launch_render_t<0, 1, 0>(a, stream); break;
        case 3: launch_render_t<0, 1, 1>(a, stream); break;
        case 4: launch_render_t<1, 0, 0>(a, stream); break;
        case 5: launch_render_t<1, 0, 1>(a, stream); break;
        case 6: launch_render_t<1, 1, 0>(a, stream); break;
        case 7: launch_render_t<1, 1, 1>(a, stream); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace rt
