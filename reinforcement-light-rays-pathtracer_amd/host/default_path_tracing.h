// default_path_tracing.h — draw_default_path_tracing with the reference's
// signatures (CPU/path_tracing/default_path_tracing.h:28 and the GPU engine's
// host loop GPU/main.cu:190-245), running on an MI355X through the C ABI.
//
//   rtmi::PathTracer keeps the rt_ctx and device scene alive across frames
//   (the reference re-copies the camera each frame and keeps the scene on the
//   device: GPU/main.cu:160-218).
#pragma once

#include <stdio.h>

#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/rtmi.h"
#include "camera.h"
#include "scene.h"
#include "sdl_screen.h"

namespace rtmi {

class PathTracer {
   public:
    explicit PathTracer(int device = 0) {
        if (rt_ctx_create(device, &ctx_) != RT_OK) throw std::runtime_error(rt_last_error());
    }
    ~PathTracer() {
        if (scene_) rt_scene_destroy(scene_);
        if (ctx_) rt_ctx_destroy(ctx_);
    }
    PathTracer(const PathTracer&) = delete;
    PathTracer& operator=(const PathTracer&) = delete;

    void set_scene(const SceneArrays& a) {
        if (scene_) rt_scene_destroy(scene_);
        scene_ = nullptr;
        if (rt_scene_create(ctx_, a.tri.data(), a.albedo.data(), a.n_surf(), a.light.data(), a.emission.data(),
                            a.light_group.data(), a.n_light(), &scene_) != RT_OK)
            throw std::runtime_error(rt_last_error());
        ++uploads_;
    }

    // renders the whole frame into screen.buffer; returns the number of ray casts
    uint64_t draw(SDLScreen& screen, const Camera& camera, const rt_params& params) {
        if (!scene_) throw std::runtime_error("PathTracer: no scene");
        rgb_.resize((size_t)screen.width * screen.height * 3);
        const rt_camera cam = camera.to_rt();
        uint64_t casts = 0;
        if (rt_render(ctx_, scene_, &cam, &params, 0, 0, screen.width, screen.height, rgb_.data(), &casts) != RT_OK)
            throw std::runtime_error(rt_last_error());
        screen.PutFrame(rgb_.data());
        return casts;
    }

    const std::vector<float>& radiance() const { return rgb_; }
    int scene_uploads() const { return uploads_; }

   private:
    rt_ctx* ctx_ = nullptr;
    rt_scene* scene_ = nullptr;
    std::vector<float> rgb_;
    int uploads_ = 0;
};

// The CPU engine's entry point: CPU preset semantics (cap 2, emission of the plane,
// hit rule of the CPU object), SAMPLES_PER_PIXEL 16, FOCAL_LENGTH = screen height.
// The reference calls it once per frame (CPU/main.cpp:85-131, `while NoQuitMessageSDL`):
// one PathTracer (context + device scene) lives for the process and the scene is
// uploaded again only when the surfaces or lights passed in change.
inline PathTracer& default_path_tracer() {
    // never destroyed: a device context must not outlive the HIP runtime's own teardown
    static PathTracer* pt = new PathTracer(0);
    return *pt;
}

inline void draw_default_path_tracing(SDLScreen screen, Camera& camera, std::vector<AreaLightPlane*> light_planes,
                                      std::vector<Surface*> surfaces, int spp = 16) {
    static SceneArrays uploaded;
    static bool have_scene = false;
    PathTracer& pt = default_path_tracer();
    SceneArrays a = flatten(surfaces, light_planes);
    if (!have_scene || !a.same_as(uploaded)) {
        pt.set_scene(a);
        uploaded = std::move(a);
        have_scene = true;
    }
    rt_params p;
    rt_params_default(RT_PRESET_CPU, &p);
    p.width = screen.width;
    p.height = screen.height;
    p.t_scale = (float)screen.height;
    p.spp = spp;
    pt.draw(screen, camera, p);  // screen shares its buffer pointer with the caller's copy
}

}  // namespace rtmi
