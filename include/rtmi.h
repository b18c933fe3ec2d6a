/*
 * rtmi.h — C ABI of the MI355X-native path tracer (librtmi.so).
 *
 * The reference (callumPearce/Reinforcement-Light-Rays-Pathtracer) has no
 * FFI; its drop-in boundary for the hot path is the C++ scene-loader /
 * Camera / SDL frame-buffer API plus the render entry point.  Each entry
 * point below names the reference interface it replaces (paths relative to
 * the reference root; CPU/ = Old_CPU_Rendering_Engine/Source,
 * GPU/ = GPU_Rendering_Engine/Source).  The C++ facade in
 * reinforcement-light-rays-pathtracer_amd/host/ restores the reference's
 * class/function names on top of this ABI; Python binds it with ctypes.
 *
 * Conventions
 *  - every function returns RT_OK (0) or a negative RT_E* code; nothing
 *    throws across the ABI; rt_last_error() holds a thread-local message.
 *  - host pointers are caller-owned; device memory is owned by rt_ctx /
 *    rt_scene.  Functions named *_device take device pointers and a
 *    hipStream_t passed as void* and are asynchronous on that stream.
 *  - one host thread per rt_ctx; contexts on different GPUs may run
 *    concurrently (one process per GPU is the supported multi-GPU model).
 */
#ifndef RTMI_H
#define RTMI_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RT_OK 0
#define RT_E_INVALID (-1)     /* bad argument */
#define RT_E_HIP (-2)         /* HIP runtime error */
#define RT_E_NOMEM (-3)       /* allocation failed */
#define RT_E_IO (-4)          /* file could not be opened / parsed */
#define RT_E_UNSUPPORTED (-5) /* valid request this build does not implement */
#define RT_E_INTERNAL (-6)    /* a self-check of the library failed */

#define RT_HIT_NONE (-1)
#define RT_HIT_TYPE_LIGHT 1u   /* enum IntersectionType AREA_LIGHT(_PLANE) */
#define RT_HIT_TYPE_SURFACE 2u /* enum IntersectionType SURFACE */

/* semantic presets */
#define RT_PRESET_CPU 0 /* Old_CPU_Rendering_Engine: recursive estimator, bounce cap semantics of
                           CPU/path_tracing/default_path_tracing.cpp:46-101 */
#define RT_PRESET_GPU 1 /* GPU_Rendering_Engine: iterative throughput,
                           GPU/path_tracing/default_path_tracing.cu:36-88 */

#define RT_HIT_RULE_CPU 0 /* predicate of the prebuilt CPU triangle.cpp.o (t > 1e-5, t < dist + 1e-5) */
#define RT_HIT_RULE_GPU 1 /* GPU/rays/ray.cu:38-141 (t < dist, dist starts at 999999) */

#define RT_SAMPLER_UNIFORM 0 /* the reference's sampler: cos(theta) = r1, pdf 1/(2*pi) */
#define RT_SAMPLER_COSINE 1  /* cosine-weighted: cos(theta) = sqrt(r1), pdf cos/pi */

typedef struct rt_ctx rt_ctx;
typedef struct rt_scene rt_scene;

/* Camera: CPU/camera.h:11-42 (position, yaw) and GPU/camera.cuh:11-36 (yaw_y, yaw_x). */
typedef struct {
    float pos[4];
    float yaw_y; /* CPU engine "yaw" */
    float yaw_x; /* GPU engine only; 0 for the CPU preset */
} rt_camera;

/* Render parameters: the reference's compile-time constants
 * (CPU/constants/ and GPU/constants/ headers) as a runtime struct. */
typedef struct {
    int32_t width, height; /* SCREEN_WIDTH / SCREEN_HEIGHT; FOCAL_LENGTH = height */
    int32_t spp;           /* SAMPLES_PER_PIXEL */
    int32_t max_bounces;   /* MAX_RAY_BOUNCES */
    int32_t sampler;       /* RT_SAMPLER_* */
    int32_t preset;        /* RT_PRESET_* */
    int32_t hit_rule;      /* RT_HIT_RULE_* */
    int32_t spp_split;     /* sample chunks per pixel (1,2,4,...,64; divides spp; 0 = 1).  Chunk c
                              sums samples [c*spp/S, (c+1)*spp/S) in order; the pixel is
                              (((P0 + P1) + P2) + ...) / spp.  Part of the result's definition:
                              keep it fixed across GPU counts for bit-identical images. */
    uint64_t seed;         /* Philox key; the reference's curand seed is 1984 */
    float env_light;       /* ENVIRONMENT_LIGHT (GPU preset) */
    float t_scale;         /* direction scale in the hit test (= SCREEN_HEIGHT in the reference) */
} rt_params;

/* Fill *p with the reference defaults of a preset:
 *   CPU: 512x512, 16 spp, cap 2, hit rule CPU   (CPU/constants/image_settings.h:9-12,
 *                                                monte_carlo_settings.h:8-9)
 *   GPU: 720x720, 32 spp, cap 80, hit rule GPU  (GPU/constants/image_settings.h:9-12,
 *                                                monte_carlo_settings.h:8-10)
 * seed 1984 (GPU/utils/cuda_helpers.cu:24). */
int rt_params_default(int preset, rt_params* p);

/* ---- context ---------------------------------------------------------- */
/* Replaces the device setup of GPU/main.cu:150-198 (cudaMalloc + pointer patching). */
int rt_ctx_create(int device_ordinal, rt_ctx** out);
int rt_ctx_destroy(rt_ctx* ctx);
const char* rt_last_error(void);

/* ---- scene construction (host side, no GPU) --------------------------- */
/* get_cornell_shapes: CPU/scenes/cornell_box_scene.cpp:3-205 (variant RT_PRESET_CPU:
 * one light plane, emission 1*(1,1,0.9)) and GPU/scenes/cornell_box_scene.cu:4 (variant
 * RT_PRESET_GPU: two AreaLights, emission 14*(0.9,0.9,0.9)).
 * Arrays must hold 36 surfaces / 2 lights (rt_cornell_counts). */
int rt_cornell_counts(int* n_surf, int* n_light);
int rt_cornell_geometry(int variant, float* tri_v /* n_surf x 9 */, float* albedo /* n_surf x 3 */,
                        float* light_v /* n_light x 9 */, float* emission /* n_light x 3 */,
                        int32_t* light_group /* n_light */);

/* load_scene for OBJ files with the GPU engine's semantics:
 * GPU/objects/object_importer.cu:8-412 (scale 2, (v1,v3,v2) order, per-scene materials and
 * lights, lights_in_obj for complex_light_room).  `scene_kind` selects the hard-coded
 * material/light block: 0 generic (white 0.75, no lights), 1 door_room, 2 archway,
 * 3 complex_light_room.  Two-pass: call with NULL arrays to get counts.
 * door_room variants: scene_kind = 1 | (bits << 8), the blocks the reference comments in
 * and out by hand (object_importer.cu).  0 = the door-room lights of :214-237, the red
 * material of :152-155 on triangles 24-35 and the blue of :161-163 on 12-23: the scene of
 * the thesis's door-room comparison renders (Images/door_room/default_128spp_50avg.png:
 * image mean and average path length match, tools/door_variants.py).  RT_DOOR_WHITE_DOOR
 * drops the red material (commented at HEAD), RT_DOOR_NO_BLUE the blue (active at HEAD),
 * RT_DOOR_ARCHWAY_LIGHTS uses the lights active at HEAD (:240-271, the archway's, outside
 * this room: a black image) instead of the door-room lights (commented at HEAD). */
#define RT_DOOR_WHITE_DOOR 1
#define RT_DOOR_NO_BLUE 2
#define RT_DOOR_ARCHWAY_LIGHTS 4
int rt_obj_geometry(const char* path, int scene_kind, float* tri_v, float* albedo, int* n_surf,
                    float* light_v, float* emission, int32_t* light_group, int* n_light,
                    float* nn_vertices /* Scene::vertices order, may be NULL */, int* n_nn_floats);

/* ---- device scene ------------------------------------------------------ */
/* Scene::load_* + the H2D copies of GPU/main.cu:160-180.  Copies the host arrays;
 * computes normals (CPU/objects/triangle.cpp:73-82) and per-triangle tangent frames. */
int rt_scene_create(rt_ctx* ctx, const float* tri_v, const float* albedo, int n_surf,
                    const float* light_v, const float* emission, const int32_t* light_group,
                    int n_light, rt_scene** out);
int rt_scene_destroy(rt_scene* scene);
/* Host copy of the normals the scene computed, (n_surf+n_light) x 3. */
int rt_scene_normals(const rt_scene* scene, float* out);

/* ---- the hot path -------------------------------------------------------- */
/* Ray::closest_intersection over a ray batch (CPU/rays/ray.cpp:14-28 + the hit predicate;
 * GPU/rays/ray.cu:16-141).  dir must be normalised (Ray::Ray does it).  out_t = hit distance
 * in t_scale units (+inf on miss); out_hit = (type<<30)|index, RT_HIT_NONE on miss; light
 * index = plane index (hit_rule CPU) or light-triangle index (hit_rule GPU). Host arrays. */
int rt_intersect(rt_ctx* ctx, const rt_scene* scene, const float* orig /* n x 3 */,
                 const float* dir /* n x 3 */, int n, float t_scale, int hit_rule,
                 float* out_t, int32_t* out_hit);
/* Same, device pointers, asynchronous on `stream` (hipStream_t). */
int rt_intersect_device(rt_ctx* ctx, const rt_scene* scene, const float* d_orig,
                        const float* d_dir, int n, float t_scale, int hit_rule, float* d_t,
                        int32_t* d_hit, void* stream);
/* Diagnostic: rt_intersect by a chosen hit-test method.  Every method returns the same
 * bits (the exact test decides; the filters only skip triangles it must reject):
 *   RT_ISECT_SCAN    the single-phase exact scan of every triangle
 *   RT_ISECT_FILTER  the fp32 two-phase filter (rays within the scene's filter bounds,
 *                    else RT_E_UNSUPPORTED)
 *   RT_ISECT_MFMA    the matrix-core filter of k_render_ps's bounce casts (a ray whose
 *                    origin is outside the scene's box + 1 keeps every triangle)
 * out_cand (optional, MFMA only): per ray, the triangles that reached the exact test. */
#define RT_ISECT_SCAN 0
#define RT_ISECT_FILTER 1
#define RT_ISECT_MFMA 2
#define RT_ISECT_BVH 3 /* the exact BVH path: built on first use if the scene has none, and kept
                          (this call may allocate); the scene's accel mode is not changed */
int rt_intersect_method(rt_ctx* ctx, const rt_scene* scene, const float* orig, const float* dir, int n,
                        float t_scale, int hit_rule, int method, float* out_t, int32_t* out_hit,
                        int32_t* out_cand);

/* ---- acceleration structure for large scenes ----
 * The reference scans every triangle per ray (CPU/rays/ray.cpp:14-28, GPU/rays/ray.cu:
 * 16-141) and has no acceleration structure; Models/bunny.obj (4,968 triangles) and
 * Medieval_House.obj (2,663) make that scan the whole cost.  The BVH path returns the
 * scan's hit bit for bit (both hit rules): padded boxes that prove the exact test fails,
 * and a second BVH over the triangles' planes for the pairs a ray could graze (rt_bvh.cpp).  RT_ACCEL_AUTO (the
 * default) builds and uses it for scenes above RT_BVH_AUTO_MIN triangles; RT_ACCEL_SCAN
 * never uses it; RT_ACCEL_BVH builds it for any scene (A/B).  The default-sampler renders
 * (rt_render, rt_render_tiles_device), the Expected-SARSA, DQN and Neural-Q renders
 * (their trace kernels take the BVH when the scene's mode turns it on) and rt_intersect /
 * rt_intersect_device follow the mode. */
#define RT_ACCEL_AUTO 0
#define RT_ACCEL_SCAN 1
#define RT_ACCEL_BVH 2
#define RT_BVH_AUTO_MIN 256
int rt_scene_set_accel(rt_scene* scene, int mode);
/* nodes of the triangle BVH, its depth, nodes of the plane-space BVH (out pointers may
 * be NULL; zeros when the scene has no BVH) */
int rt_scene_accel_info(const rt_scene* scene, int* n_nodes, int* depth, int64_t* plane_nodes);
/* The bounce-ray candidate table of hit rule `hit_rule` (no reference counterpart: the
 * scene's preprocessing, like a BVH build): built on the first render that takes it.
 * built: 1 once on the device; build_s: host build + upload seconds; bytes: device bytes.
 * Out pointers may be NULL; zeros before the build or when no render took it. */
int rt_scene_ctab_info(const rt_scene* scene, int hit_rule, int* built, double* build_s, uint64_t* bytes);
/* Host only (no GPU): build the BVH of n triangles (n x 9 vertices, the rt_scene_create
 * order) and check its invariants (every triangle in one leaf of each tree, boxes nested
 * and holding their triangles, planes inside their plane-space leaves).  stats
 * (optional, 4 entries): nodes, depth, plane-space nodes, leaves.  RT_E_INTERNAL with
 * rt_last_error() naming the first violation. */
int rt_bvh_check(const float* tri_v, int n, int64_t* stats);

/* draw_default_path_tracing (CPU/path_tracing/default_path_tracing.cpp:5-18;
 * GPU kernel GPU/path_tracing/default_path_tracing.cu:7-34): render the rectangle
 * [x0,x0+w) x [y0,y0+h) of the params->width x params->height image.
 * out_rgb: w*h*3 floats, row-major (row = y-y0).  Synchronous; host memory. */
int rt_render(rt_ctx* ctx, const rt_scene* scene, const rt_camera* cam, const rt_params* params,
              int x0, int y0, int w, int h, float* out_rgb, uint64_t* out_ray_casts);

/* Tile-list render for image-tile partitioning across GPUs.  tiles: n_tiles x 2 int32
 * (host) pixel origins of tile_size x tile_size tiles (tile_size a multiple of 16).
 * d_out: device, n_tiles*tile_size*tile_size*3 floats, [tile][y][x][rgb].
 * d_casts: device uint64 (accumulated into, may be NULL).  Asynchronous on `stream`. */
int rt_render_tiles_device(rt_ctx* ctx, const rt_scene* scene, const rt_camera* cam,
                           const rt_params* params, const int32_t* tiles, int n_tiles,
                           int tile_size, float* d_out, uint64_t* d_casts, void* stream);

/* ---- DQN Q-value sampling (BASELINE config 4) ---------------------------- */
typedef struct rt_dqn rt_dqn;

/* DyNet TextFileSaver format reader (the reference loads RMD/<scene>.model with
 * dynet::TextFileLoader, GPU/deep_learning/pre_trained_pathtracer.cu:45-53).  Parameters in
 * file order; each returned row-major [rows][cols] (DyNet stores column-major); a vector
 * ("{rows}" header) is returned with cols = 0 and holds rows values.  Call with values = NULL
 * to size: *n_params, *n_values. */
int rt_dynet_read(const char* path, int max_params, int32_t* rows, int32_t* cols, float* values,
                  int* n_params, int64_t* n_values);

/* DyNet TextFileSaver format writer (the reference saves its trained networks with
 * dynet::TextFileSaver, GPU_Rendering_Engine/Source/deep_learning/neural_q_pathtracer.cu:193 and
 * NN_Q_Value_Trainer/Source/main.cu:290, into Radiance_Map_Data/<name>.model):
 * "#Parameter# /_<k> {rows,cols} <bytes> ZERO_GRAD" (vectors "{rows}") then one line of
 * column-major "%+.8e " values; <bytes> counts that line with its newline.  values: the
 * n_params parameters concatenated, each row-major [rows][cols] (the rt_dynet_read layout;
 * cols = 0: a vector of rows values, "{rows}" header; cols = 1: an (rows, 1) matrix), so a
 * write -> read round trip returns the same floats and shapes bit for bit.  Non-finite
 * values are refused (RT_E_INVALID): DyNet's loader cannot parse them. */
int rt_dynet_write(const char* path, int n_params, const int32_t* rows, const int32_t* cols,
                   const float* values);

/* DQNetwork::initialize + the parameters it loads (NN_Builders/dq_network.cu:8-33,
 * fc_layer.cu:29-35): ReLU(W x + b) x 4, n_in -> hidden[0] -> hidden[1] -> hidden[2] -> n_out.
 * W[l]: row-major [out][in] fp32, b[l]: [out].  nn_vertices: Scene::vertices (n_in floats);
 * the network input is nn_vertices - ray position (nn_rendering_helpers.cu:280-298).
 * Stored on the device as bf16 for the MFMA forward.  n_out must be 144. */
int rt_dqn_create(rt_ctx* ctx, const float* nn_vertices, int n_in, const int32_t* hidden /* 3 */,
                  int n_out, const float* const* W /* 4 */, const float* const* b /* 4 */,
                  rt_dqn** out);
int rt_dqn_destroy(rt_dqn* dqn);
/* Kernel of the forward pass (same Q bit for bit; A/B measurement):
 * RT_DQN_MLP_AUTO (default) and RT_DQN_MLP_STREAM: the weight-streaming kernel (64 rays per
 * workgroup, weight fragments from L2); RT_DQN_MLP_STATIONARY: the weight-stationary one
 * (weights resident in registers, one workgroup per CU) for the reference's 200-300-200
 * shape, the streaming one otherwise. */
#define RT_DQN_MLP_AUTO 0
#define RT_DQN_MLP_STREAM 1
#define RT_DQN_MLP_STATIONARY 2
int rt_dqn_set_mlp(rt_dqn* dqn, int mode);
/* DQNetwork::network_inference on n ray positions (host arrays): q = n x 144. */
int rt_dqn_forward(rt_ctx* ctx, const rt_dqn* dqn, const float* loc /* n x 3 */, int n, float* q);
/* Same on device buffers, asynchronous on `stream`. */
int rt_dqn_forward_device(rt_ctx* ctx, const rt_dqn* dqn, const float* d_loc, int n, float* d_q,
                          void* stream);
/* save_selected_radiance_volumes_vals_nn / write_q_values_for_position
 * (GPU/deep_learning/q_value_extractor.cu:18-125): for each "x y z nx ny nz" line of
 * to_select_path, the network's Q values at x (rt_dqn_forward) normalised by their sum,
 * written as "x y z nx ny nz q0 .. q143" (selected_deep.txt); out_path is replaced. */
int rt_dqn_save_selected(rt_ctx* ctx, const rt_dqn* dqn, const char* to_select_path, const char* out_path);
/* importance_sample_direction (nn_rendering_helpers.cu:391-489) for n rays given their Q
 * values (host arrays; q is overwritten with Q*cos as in the reference).  tri: surface the
 * ray sits on; pix: global pixel id (RNG key); tp updated in place; action -1 = none. */
int rt_dqn_sample(rt_ctx* ctx, const rt_scene* scene, uint64_t seed, float* q, const float* loc,
                  const int32_t* tri, const uint32_t* pix, int n, int sample, int bounce, float* tp,
                  float* dir_out, int32_t* action);
/* PretrainedPathtracer::render_frame (pre_trained_pathtracer.cu:188-376), GPU-engine preset:
 * rectangle render into host memory, and tile-list render into device memory (stream-ordered;
 * synchronises the stream every few bounces to stop once all paths have ended).  Between the
 * forward and the sampler each ray's 144 Q values are kept in bf16 (round to nearest even of
 * the forward's fp32 Q, within the forward's own bf16 tolerance): the per-bounce Q buffer's
 * HBM round trip is half the bytes (the sampler itself is rt_dqn_sample's, on those values). */
int rt_render_dqn(rt_ctx* ctx, const rt_scene* scene, const rt_dqn* dqn, const rt_camera* cam,
                  const rt_params* params, int x0, int y0, int w, int h, float* out_rgb,
                  uint64_t* out_ray_casts);
int rt_render_dqn_tiles_device(rt_ctx* ctx, const rt_scene* scene, const rt_dqn* dqn,
                               const rt_camera* cam, const rt_params* params, const int32_t* tiles,
                               int n_tiles, int tile_size, float* d_out, uint64_t* d_casts,
                               void* stream);

/* ---- Neural-Q training ---------------------------
 * The learning rule of NeuralQPathtracer::render_frame
 * (GPU/deep_learning/neural_q_pathtracer.cu:420-513), which the reference runs through
 * DyNet on the host, on device buffers in fp32: parameters, gradients and Adam moments
 * live on the device; rt_dqn_trainer_params copies the weights out (row-major, the
 * rt_dqn_create layout) to rebuild the bf16 inference network. */
typedef struct rt_dqn_trainer rt_dqn_trainer;
/* DQNetwork::initialize (NN_Builders/dq_network.cu:8-33) with the given parameters +
 * dynet::AdamTrainer(model) (neural_q_pathtracer.cu:47): DyNet defaults beta1 0.9,
 * beta2 0.999, eps 1e-8, global gradient-norm clipping at 5; learning_rate (DyNet 1e-3). */
int rt_dqn_trainer_create(rt_ctx* ctx, const float* nn_vertices, int n_in, const int32_t* hidden /* 3 */,
                          int n_out, const float* const* W /* 4 */, const float* const* b /* 4 */,
                          float learning_rate, rt_dqn_trainer** out);
int rt_dqn_trainer_destroy(rt_dqn_trainer* trainer);
int rt_dqn_trainer_params(const rt_dqn_trainer* trainer, float* const* W /* 4 */, float* const* b /* 4 */);
/* Steps 5-7 of the training loop (neural_q_pathtracer.cu:478-513) on n rays: forward on the
 * current states (network input nn_vertices - loc), pick the taken actions, loss =
 * sum (target - q_a)^2 (sum_batches), backward, trainer.update().  Device arrays:
 * d_loc n x 3, d_action n (an action outside [0, n_out) contributes nothing), d_target n.
 * loss_out / grad_norm_out (host, optional; either one synchronises the stream): the loss
 * and the gradient L2 norm before clipping. */
int rt_dqn_train_step_device(rt_ctx* ctx, rt_dqn_trainer* trainer, const float* d_loc, const int32_t* d_action,
                             const float* d_target, int n, float* loss_out, float* grad_norm_out, void* stream);
/* compute_td_targets (GPU/deep_learning/nn_rendering_helpers.cu:91-140): target =
 * reward + max_a(Q(s',a) cos_a) * discount, reward alone where terminal == 1; action 0 is
 * not cosine-weighted (as in the reference); cos_a of a jittered direction in cell a
 * (Philox: pixel, sample, event 1 + bounce).  d_next_q: n x 144 row-major. */
int rt_dqn_td_targets_device(rt_ctx* ctx, uint64_t seed, const float* d_next_q, const int32_t* d_terminal,
                             const float* d_reward, const float* d_discount, const uint32_t* d_pix, int sample,
                             int bounce, int n, float* d_target, void* stream);

/* NeuralQPathtracer (GPU/deep_learning/neural_q_pathtracer.cu:226-600): renders while
 * training `trainer`'s network, on the device.  Per sample: initialise_ray (:604-643); per
 * bounce b until no path is bouncing or max_bounces: (b > 0) the network's Q at every ray's
 * position and sample_batch_ray_directions_epsilon_greedy (nn_rendering_helpers.cu:330-389:
 * importance_sample_direction with probability 1 - epsilon, else a uniform cell), trace_ray
 * (:646-745: rewards 0 / light luminance x 200, discount = the surface's luminance,
 * throughput on contributing paths), (b > 0) the learning rule per batch of batch_size rays
 * (compute_td_targets on the new positions, trainer.update on the old ones with the sampled
 * actions, neural_q_pathtracer.cu:420-513), sample_random_scene_pos_for_terminated_rays
 * (:241-277, restarted rays learn but no longer contribute; the point is stored with y and
 * z exchanged, as the reference stores it).  After a sample epsilon = max(epsilon -
 * decay, min) (:543-546).  The frame is the throughput summed over the samples / spp.
 * Reference settings: batch 4096, epsilon 0.05 / 0.05 / 0.01 (deep_learning_settings.h).
 * stats (optional, spp x 3 floats): per sample the nn_training_stats.txt values (:553-583):
 * average path length (sum of termination bounces / pixels), loss (summed over batches),
 * zero-contribution paths ((r + g + b) / 3 < THROUGHPUT_THRESHOLD).  out_rgb: W x H x 3 or
 * NULL.  Pixel ids key the RNG (Philox; seed = params->seed); successive frames continue
 * the sample sequence. */
typedef struct rt_neuralq rt_neuralq;
int rt_neuralq_create(rt_ctx* ctx, const rt_scene* scene, rt_dqn_trainer* trainer, int batch_size,
                      float epsilon_start, float epsilon_min, float epsilon_decay, rt_neuralq** out);
int rt_neuralq_destroy(rt_neuralq* nq);
int rt_neuralq_epsilon(const rt_neuralq* nq, float* epsilon);
int rt_neuralq_render_frame(rt_ctx* ctx, rt_neuralq* nq, const rt_camera* cam, const rt_params* params,
                            float* out_rgb, float* stats, uint64_t* out_ray_casts);

/* ---- Expected-SARSA radiance volumes (BASELINE config 3) ------------------ */
typedef struct rt_sarsa rt_sarsa;

/* RadianceMap::RadianceMap (GPU/radiance_volumes/radiance_map.cu:8-55): floor(area/0.001)
 * radiance volumes per surface, placed by rejection point picking (Philox stream of `seed`
 * in place of rand()), each with Q = 100/144 per sector, CDF k/144 and the irradiance of
 * initialise_radiance_grid (radiance_volume.cu:46-89); the KD tree of radiance_tree.cu in
 * its array form.  The map lives on the context's device. */
int rt_sarsa_create(rt_ctx* ctx, const rt_scene* scene, uint64_t seed, rt_sarsa** out);
/* The same with the volume density as an argument: floor(area / area_per_sample) volumes per
 * surface -- AREA_PER_SAMPLE (GPU/constants/radiance_volumes_settings.h:12), a compile-time
 * constant of the reference (0.001f) that its thesis runs varied (Images/door_room/
 * sarsa_128_344_volumes.bmp, 4_critical_evaluation.tex:240-245).  area_per_sample must be a
 * finite float > 0; rt_sarsa_create(...) is rt_sarsa_create_density(..., 0.001f, ...). */
int rt_sarsa_create_density(rt_ctx* ctx, const rt_scene* scene, uint64_t seed, float area_per_sample,
                            rt_sarsa** out);
int rt_sarsa_destroy(rt_sarsa* sarsa);
/* sizes: volumes, KD array elements, frames rendered so far (any pointer may be NULL) */
int rt_sarsa_info(const rt_sarsa* sarsa, int32_t* n_volumes, int32_t* n_nodes, uint32_t* frames);
/* Nearest-volume search of find_closest_radiance_volume_iterative
 * (GPU/radiance_volumes/radiance_map.cu:149-203).  Both modes return the same volume
 * for every query: RT_SARSA_SEARCH_KD walks the reference's KD array;
 * RT_SARSA_SEARCH_GRID (default) answers from a per-normal uniform grid when the
 * nearest same-normal volume is provably a leaf the KD walk visits and is unique,
 * and walks the KD array otherwise (counted in kd_fallbacks). */
#define RT_SARSA_SEARCH_KD 0
#define RT_SARSA_SEARCH_GRID 1
int rt_sarsa_set_search(rt_sarsa* sarsa, int mode);
/* Direction sampling at a surface with a radiance volume:
 * RT_SARSA_SAMPLE_CDF (default) RadianceVolume::sample_direction_from_radiance_distribution
 *   (radiance_volume.cu:191-244), the CDF by inverse transform;
 * RT_SARSA_SAMPLE_MAX sample_max_direction_from_radiance_distribution (:246-278): the first
 *   sector of largest Q (of the previous frame), uniform within it, pdf = RHO x its CDF step
 *   / GRID_RHO -- 0 for sector 0, as the reference computes it (the path's throughput is
 *   then infinite).  TD learning is the same in both modes. */
#define RT_SARSA_SAMPLE_CDF 0
#define RT_SARSA_SAMPLE_MAX 1
int rt_sarsa_set_sampling(rt_sarsa* sarsa, int mode);
/* TD learning rule (replaces the reference's in-kernel update,
 * GPU/radiance_volumes/radiance_volume.cu:282-301 temporal_difference_update and :93-112
 * expected_sarsa_irradiance, called from radiance_map.cu:90-146):
 * RT_SARSA_TD_FRAME (default) every TD target of a frame goes into a per-sector
 *   fixed-point sum and count; the frame end folds them into Q in closed form (the running
 *   mean alpha = 1/(1 + visits) gives) -- deterministic, bit-exact against oracle/, the same
 *   on any GPU count;
 * RT_SARSA_TD_INFRAME the reference's own rule: each event updates the sector's Q, visits
 *   and the volume's irradiance in place while the frame renders (later targets of the same
 *   frame see it; concurrent updates race as in the reference).  The CDFs still change only
 *   at the frame end (update_radiance_volume_distributions).  SAMPLE_MAX then scans the
 *   live Q at every sample, as the reference's scan of its radiance grid does.  Not
 *   reproducible run to run (a launch with one active lane is: the events then run in the
 *   restatement's order); one GPU only: rt_sarsa_td_device and a tile render with apply = 0
 *   return RT_E_UNSUPPORTED in this mode. */
#define RT_SARSA_TD_FRAME 0
#define RT_SARSA_TD_INFRAME 1
int rt_sarsa_set_td_mode(rt_sarsa* sarsa, int mode);
int rt_sarsa_get_td_mode(const rt_sarsa* sarsa, int* mode);
/* Paths in flight of the in-frame rule's render.  Its races -- and with them how fast a frame
 * learns -- depend on how many paths update the table at once: the reference's GTX 1070 Ti
 * holds at most 19 SMs x 2048 threads = 38,912.  lanes > 0 caps the render's persistent grid
 * at ceil(lanes / 256) workgroups of 256 lanes (the image and its statistics are then
 * rendered by fewer lanes, each taking more work items); 0 (default): the device's full
 * occupancy.  No effect on the frame-synchronous rule's results. */
int rt_sarsa_set_inframe_lanes(rt_sarsa* sarsa, int lanes);
/* Training statistics of the last frame rendered (GPU/main.cu:321-339, one line of
 * Radiance_Map_Data/sarsa_training_stats.txt per frame): path_floor_sum = the sum over the
 * frame's pixels of int(path lengths / spp) (path_trace_reinforcement,
 * reinforcement_path_tracing.cu:27-44; a path's length is its ray casts), zero_paths = the
 * paths whose mean radiance (r + g + b) / 3 < THROUGHPUT_THRESHOLD.  The reference's line is
 * "<path_floor_sum / pixels, integer division> 0 <zero_paths>".  For rt_render_sarsa_tiles_device
 * the sums cover the call's tiles (add them over ranks). */
int rt_sarsa_frame_stats(const rt_sarsa* sarsa, uint64_t* path_floor_sum, uint64_t* zero_paths);
/* On-disk formats of the reference's Q-tables.
 * rt_sarsa_save_q: RadianceMap::save_q_vals_to_file (GPU/radiance_volumes/radiance_map.cu:236-266):
 *   "144\n", then one line per volume in map order: "x y z Q0 .. Q143" (ostream defaults,
 *   6 significant digits).
 * rt_sarsa_save_selected: RadianceMap::save_selected_radiance_volumes_vals (radiance_map.cu:270-301):
 *   for each "x y z nx ny nz" line of to_select_path (RMD/selected_radiance_volumes/to_select.txt),
 *   the nearest volume (rt_sarsa_nearest) as "px py pz nx ny nz d0 .. d143" with its sector
 *   distribution (the CDF differenced: convert_radiance_distribution, radiance_volume.cu:332-336);
 *   out_path is replaced.  Both return RT_E_IO on file errors. */
int rt_sarsa_save_q(const rt_sarsa* sarsa, const char* path);
/* The Q-table back into a map: a file of rt_sarsa_save_q / save_q_vals_to_file, whose
 * volume positions must be this map's (same scene and seed: RT_E_INVALID otherwise).  Q is
 * set from the file (std::stof of the printed values), the irradiance estimate recomputed
 * as initialise_radiance_grid does for a Q grid (radiance_volume.cu:46-63), the CDF as
 * update_radiance_distribution (:148-188); visits are kept.  The reference reads its
 * per-volume files back only to draw them (read_radiance_volumes_from_file,
 * radiance_volume.cu:377-440); this resumes training or renders from a saved map.
 * save_q -> load_q -> save_q reproduces the file byte for byte. */
int rt_sarsa_load_q(rt_sarsa* sarsa, const char* path);
int rt_sarsa_save_selected(rt_ctx* ctx, const rt_sarsa* sarsa, const char* to_select_path,
                           const char* out_path);
int rt_sarsa_search_stats(const rt_sarsa* sarsa, int32_t* mode, int32_t* n_classes, int64_t* grid_cells,
                          uint64_t* kd_fallbacks);
/* host copies: pos n x 3, normal n x 3, surface index n, KD array n_nodes x 12 words
 * {dim, leaf, left, right (int32), data, px, py, pz, nx, ny, nz (float), vol (int32)} */
int rt_sarsa_volumes(const rt_sarsa* sarsa, float* pos, float* normal, int32_t* surface,
                     float* kd_nodes);
/* Q-table (radiance_grid), CDF (radiance_distribution), visits (n x 144, sector x*12+y) and
 * irradiance_accum (n) after the last applied frame; NULL pointers are skipped. */
int rt_sarsa_read(const rt_sarsa* sarsa, float* q, float* cdf, uint32_t* visits,
                  float* irradiance);
/* RadianceMap::find_closest_radiance_volume_iterative (radiance_map.cu:149-203), n queries. */
int rt_sarsa_nearest(rt_ctx* ctx, const rt_sarsa* sarsa, const float* pos, const float* normal,
                     int n, int32_t* out);
/* draw_reinforcement_path_tracing + update_radiance_volume_distributions per frame
 * (reinforcement_path_tracing.cu:6-120, GPU/main.cu:296-350), GPU-engine preset: `frames`
 * frames of params->spp samples, each frame learning from the previous frame's Q-table;
 * out_rgb = the last frame (W x H x 3), out_ray_casts = casts of all frames. */
int rt_render_sarsa(rt_ctx* ctx, const rt_scene* scene, rt_sarsa* sarsa, const rt_camera* cam,
                    const rt_params* params, int frames, float* out_rgb, uint64_t* out_ray_casts);
/* One frame over a tile list into device memory (stream-ordered).  apply = 0 leaves the
 * frame's TD sums in the map's accumulators (rt_sarsa_td_device: int64 fixed-point sums,
 * uint32 counts, n x 144 each) for a cross-GPU sum before rt_sarsa_apply. */
int rt_render_sarsa_tiles_device(rt_ctx* ctx, const rt_scene* scene, rt_sarsa* sarsa,
                                 const rt_camera* cam, const rt_params* params,
                                 const int32_t* tiles, int n_tiles, int tile_size, float* d_out,
                                 uint64_t* d_casts, int apply, void* stream);
int rt_sarsa_td_device(rt_sarsa* sarsa, void** d_sum, void** d_count, int64_t* n_entries);
int rt_sarsa_apply(rt_sarsa* sarsa, void* stream);

/* Device self-tests of numeric building blocks (no reference counterpart): every
 * bit-exact claim against oracle/ rests on them.  result[0] = mismatches, result[1] = the
 * lowest mismatching input bits (0xffffffff: none).
 * RT_SELFTEST_RCP: the kernels' correctly-rounded reciprocal (Cramer's 1/detA, normalize)
 *   vs IEEE 1.0f / x over all 2^32 floats;
 * RT_SELFTEST_DIV12: the grid-coordinate x / 12 (Chiu map) vs IEEE over its domain,
 *   +0 and |x| in [2^-100, 2^100];
 * RT_SELFTEST_DIVRHO: the estimator's x / RHO vs IEEE over all 2^32 floats. */
#define RT_SELFTEST_RCP 1
#define RT_SELFTEST_DIV12 2
#define RT_SELFTEST_DIVRHO 3
int rt_selftest(rt_ctx* ctx, int which, uint64_t* result /* 2 */);

/* Host-side checks of the CPU-preset primary-ray cull (k_cull_ps; no GPU needed).
 * rt_filter_build: the per-triangle filter records of the two-phase hit test
 * (5 x float4 per triangle, layout rt_internal.hpp kFiltF4) for the triangle soup
 * tri_v (n x 9, surfaces then lights: the rt_scene_create order).
 * rt_rect_candidates: bit i of masks[i / 64] = triangle i may be the hit of a camera
 * ray through a pixel of [px0, px1] x [py0, py1] (inclusive); the other triangles
 * certainly fail the exact test for every such ray (RT_PRESET_CPU parameters).
 * Replaces no reference interface: it exposes the kernel's own cull so tests can check
 * it against the CPU restatement's hits (Ray::closest_intersection, CPU/rays/ray.cpp:14-28). */
int rt_filter_build(const float* tri_v, int n, float* out_filt /* n x 20 */);
int rt_rect_candidates(const float* filt, int n_tri, const rt_camera* cam, const rt_params* params,
                       int px0, int py0, int px1, int py1, uint64_t* masks /* ceil(n_tri / 64) */);
/* The same masks computed by the kernel (k_cull_ps) for the launch rt_render would make
 * for the rectangle (x0, y0, w, h): 4 words per wave, waves in launch order (16x16 blocks
 * row-major, `spp_split` workgroups each, 4 waves per workgroup).  *n_words: capacity of
 * out on entry, words written on return. */
int rt_cull_masks_device(rt_ctx* ctx, const rt_scene* scene, const rt_camera* cam, const rt_params* params,
                         int x0, int y0, int w, int h, uint64_t* out, int64_t* n_words);
/* Host-side check of the bounce-ray candidate table (rt_ctab.cpp): a render builds it on first
 * use for a scene of at most 256 triangles -- hit rule RT_HIT_RULE_CPU (k_render_ps's bounce
 * casts, t_scale >= 256) or RT_HIT_RULE_GPU (the GPU-engine renders' and the DQN renderer's
 * bounce casts; the GPU-engine renders' camera rays take the cull of their 16x4 pixel
 * rectangle) -- and the bounce casts take their candidates from it (RT_CTAB=0 in the
 * environment: never built).  For the triangle soup tri_v (n <= 256, the first n_surf
 * surfaces: the rt_scene_create order) build the table of `hit_rule` and look up each ray
 * (surf: the surface its origin lies on, orig, dir: n_rays x 3, dir unit length) as the kernels
 * do: bit i % 64 of masks[r * words + i / 64] (words = ceil(n / 64)) = triangle i is a
 * candidate of ray r; every other triangle fails the exact test under that rule (rule CPU:
 * t_scale >= 256) for it (rays the table does not cover get every triangle).  stats (optional,
 * 4 entries): patches, patches kept whole, candidate bits over all (patch, bin) entries,
 * grazing-table bits.  Replaces no reference interface: tests check it against the CPU
 * restatement's pass sets of Triangle::intersects (CPU/rays/ray.cpp:14-28; GPU/rays/ray.cu:63-64). */
int rt_ctab_candidates(const float* tri_v, int n, int n_surf, int hit_rule, const int32_t* surf, const float* orig,
                       const float* dir, int n_rays, uint64_t* masks, int64_t* stats);

/* Live kernel timing (no reference counterpart; bench.py's roofline): while enabled, every
 * launch of the kernel families below is bracketed by a HIP event pair on its own launch
 * stream.  rt_ktime_enable(1) clears the totals and starts, rt_ktime_enable(0) stops;
 * rt_ktime_read waits for the recorded launches and returns the total milliseconds and the
 * launch count of one family since the last enable. */
#define RT_KT_RENDER_PS 0     /* k_render_ps: CPU preset (configs 1-2, the bench kernel) */
#define RT_KT_RENDER 1        /* k_render: GPU preset (config 5) */
#define RT_KT_SARSA_RENDER 2  /* k_sarsa_render (config 3) */
#define RT_KT_SARSA_APPLY 3   /* k_sarsa_apply */
#define RT_KT_DQN_MLP 4       /* k_dqn_mlp: the Q-network forward (config 4) */
#define RT_KT_DQN_BOUNCE 5    /* k_dqn_bounce: Q.cos sampling + trace */
#define RT_KT_DQN_CAMERA 6    /* k_dqn_camera */
#define RT_KT_COUNT 7
int rt_ktime_enable(int on);
int rt_ktime_read(int kernel, double* total_ms, int64_t* launches);
const char* rt_ktime_name(int kernel);

/* SDLScreen::PutPixelSDL pack rule (CPU/sdl/sdl_screen.cpp:100-112). Host arrays. */
int rt_pack_argb(const float* rgb, int n, uint32_t* out_argb);

/* SDLScreen::SDL_SaveImage replacement: 32-bit BMP of an ARGB buffer (headless). */
int rt_save_bmp(const char* path, const uint32_t* argb, int width, int height);
/* The same frame as an 8-bit RGB PNG (the thesis images, Images/<scene>/reference.png;
 * SURVEY.md §8(f) item 4); stored deflate blocks, no compression. */
int rt_save_png(const char* path, const uint32_t* argb, int width, int height);

#ifdef __cplusplus
}
#endif

#endif /* RTMI_H */
