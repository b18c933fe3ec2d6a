// rt_internal.hpp — types shared by the C-ABI layer and the gfx950 kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rt_math.hpp"

namespace rt {

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

struct DeviceScene {
    float4* isect = nullptr;   // n_tri * kIsectF4
    float4* shade = nullptr;   // n_tri * kShadeF4
    int32_t* code_cpu = nullptr;  // n_tri packed hit codes under hit rule CPU
    int32_t* code_gpu = nullptr;  // ... under hit rule GPU
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
};

hipError_t launch_intersect(const DeviceScene& s, const float* orig, const float* dir, int n,
                            float t_scale, int hit_rule, float* out_t, int32_t* out_hit,
                            hipStream_t stream);

// returns hipErrorInvalidValue for combinations the kernels do not instantiate
hipError_t launch_render(const RenderLaunch& a, hipStream_t stream);

}  // namespace rt
