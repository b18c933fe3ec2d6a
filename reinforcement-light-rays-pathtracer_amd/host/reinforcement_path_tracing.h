// reinforcement_path_tracing.h — the GPU engine's learned-sampling renderers with
// the reference's names, on an MI355X through the C ABI:
//
//   RadianceMap + draw_reinforcement_path_tracing + update_radiance_volume_distributions
//     Expected SARSA (GPU/radiance_volumes/radiance_map.cuh, GPU/path_tracing/
//     reinforcement_path_tracing.cuh:1-30, host loop GPU/main.cu:260-350)
//   PretrainedPathtracer::render_frame
//     DQN Q-value sampling (GPU/deep_learning/pre_trained_pathtracer.cuh, main.cu:420-470)
//   NeuralQPathtracer::render_frame
//     rendering while training the network (GPU/deep_learning/neural_q_pathtracer.cuh)
//
// The reference's draw kernel learns while it renders and the distribution update
// runs after it; here draw_reinforcement_path_tracing renders one frame and folds
// the frame's TD targets, so update_radiance_volume_distributions
// is already part of it and kept as a no-op for source compatibility.
#pragma once

#include <algorithm>
#include <fstream>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/rtmi.h"
#include "camera.h"
#include "scene.h"
#include "sdl_screen.h"

namespace rtmi {

namespace detail {
inline void check(int rc) {
    if (rc != RT_OK) throw std::runtime_error(rt_last_error());
}
}  // namespace detail

// Owns the device context and scene used by the learned renderers.
class DeviceScene {
   public:
    explicit DeviceScene(const Scene& scene, int device = 0) {
        detail::check(rt_ctx_create(device, &ctx_));
        const SceneArrays a = flatten(scene.surfaces, scene.area_lights);
        if (rt_scene_create(ctx_, a.tri.data(), a.albedo.data(), a.n_surf(), a.light.data(), a.emission.data(),
                            a.light_group.data(), a.n_light(), &scene_) != RT_OK) {
            const std::string e = rt_last_error();
            rt_ctx_destroy(ctx_);
            throw std::runtime_error(e);
        }
        vertices_ = scene.vertices;
    }
    ~DeviceScene() {
        if (scene_) rt_scene_destroy(scene_);
        if (ctx_) rt_ctx_destroy(ctx_);
    }
    DeviceScene(const DeviceScene&) = delete;
    DeviceScene& operator=(const DeviceScene&) = delete;
    rt_ctx* ctx() const { return ctx_; }
    rt_scene* scene() const { return scene_; }
    const std::vector<float>& vertices() const { return vertices_; }

   private:
    rt_ctx* ctx_ = nullptr;
    rt_scene* scene_ = nullptr;
    std::vector<float> vertices_;
};

// GPU/radiance_volumes/radiance_map.cuh: sampled radiance volumes, Q-table, KD tree.
class RadianceMap {
   public:
    // area_per_sample: AREA_PER_SAMPLE (GPU/constants/radiance_volumes_settings.h:12), the volume density
    explicit RadianceMap(DeviceScene& ds, uint64_t seed = 1984, float area_per_sample = 0.001f) : ds_(ds) {
        detail::check(rt_sarsa_create_density(ds.ctx(), ds.scene(), seed, area_per_sample, &map_));
        detail::check(rt_sarsa_info(map_, &radiance_volumes_count, &radiance_array_size, nullptr));
    }
    ~RadianceMap() {
        if (map_) rt_sarsa_destroy(map_);
    }
    RadianceMap(const RadianceMap&) = delete;
    RadianceMap& operator=(const RadianceMap&) = delete;

    // Q-values (radiance_grid) of every volume, sector x*12+y (save_q_vals_to_file's content)
    std::vector<float> q_vals() const {
        std::vector<float> q((size_t)radiance_volumes_count * 144);
        detail::check(rt_sarsa_read(map_, q.data(), nullptr, nullptr, nullptr));
        return q;
    }

    // RadianceMap::save_q_vals_to_file (radiance_map.cu:236-266) to `path`
    void save_q_vals_to_file(const std::string& path) const { detail::check(rt_sarsa_save_q(map_, path.c_str())); }
    // a saved Q-table back into this map (same scene and seed): resume training / render greedily
    void read_q_vals_from_file(const std::string& path) { detail::check(rt_sarsa_load_q(map_, path.c_str())); }
    // sample_max_direction_from_radiance_distribution (radiance_volume.cu:246-278) instead of the CDF
    void set_sample_max_direction(bool on) {
        detail::check(rt_sarsa_set_sampling(map_, on ? RT_SARSA_SAMPLE_MAX : RT_SARSA_SAMPLE_CDF));
    }
    // the reference's racy in-frame TD update (radiance_volume.cu:282-301) instead of the
    // deterministic frame-synchronous fold (one GPU)
    void set_in_frame_td(bool on) {
        detail::check(rt_sarsa_set_td_mode(map_, on ? RT_SARSA_TD_INFRAME : RT_SARSA_TD_FRAME));
    }
    // paths in flight of the in-frame rule (its races depend on it; the reference's GTX 1070 Ti
    // held about 4,864: the setting its training logs are matched at); 0: the whole device
    void set_in_frame_lanes(int lanes) { detail::check(rt_sarsa_set_inframe_lanes(map_, lanes)); }
    // GPU/main.cu:321-339 after a frame: the average path length as the reference computes it
    // (int(sum over pixels of int(path lengths / spp)) / pixels)) and the zero-contribution
    // paths; append_training_stats writes its "avg 0 zero" line.
    void frame_stats(int pixels, float* avg_path_length, uint64_t* zero_paths) const {
        uint64_t paths = 0;
        detail::check(rt_sarsa_frame_stats(map_, &paths, zero_paths));
        *avg_path_length = (float)(paths / (uint64_t)pixels);
    }
    void append_training_stats(const std::string& path, int pixels) const {
        float avg = 0.f;
        uint64_t zero = 0;
        frame_stats(pixels, &avg, &zero);
        std::ofstream f(path, std::ios::app);
        f << avg << " " << 0.0 << " " << zero << "\n";
        if (!f) throw std::runtime_error("cannot append to " + path);
    }

    int radiance_volumes_count = 0;
    int radiance_array_size = 0;
    rt_sarsa* handle() const { return map_; }
    DeviceScene& device_scene() const { return ds_; }

   private:
    DeviceScene& ds_;
    rt_sarsa* map_ = nullptr;
};

inline rt_params gpu_engine_params(const SDLScreen& screen, int spp) {
    rt_params p;
    rt_params_default(RT_PRESET_GPU, &p);
    p.width = screen.width;
    p.height = screen.height;
    p.t_scale = (float)screen.height;
    p.spp = spp;
    return p;
}

// draw_reinforcement_path_tracing (GPU/path_tracing/reinforcement_path_tracing.cu:15-24) for one
// frame of SAMPLES_PER_PIXEL samples; the frame's radiance goes to the screen buffer.
// Returns the frame's ray casts (sum of the per-pixel path lengths).
inline uint64_t draw_reinforcement_path_tracing(SDLScreen& screen, const Camera& camera, RadianceMap& map,
                                                int spp = 32) {
    const rt_params p = gpu_engine_params(screen, spp);
    const rt_camera cam = camera.to_rt();
    std::vector<float> rgb((size_t)screen.width * screen.height * 3);
    uint64_t casts = 0;
    detail::check(rt_render_sarsa(map.device_scene().ctx(), map.device_scene().scene(), map.handle(), &cam, &p, 1,
                                  rgb.data(), &casts));
    screen.PutFrame(rgb.data());
    return casts;
}

// update_radiance_volume_distributions (reinforcement_path_tracing.cu:6-13): folded into the draw.
inline void update_radiance_volume_distributions(RadianceMap&) {}

// GPU/deep_learning/pre_trained_pathtracer.cuh: a trained DyNet Q-network loaded from the
// reference's text model (Radiance_Map_Data/<scene>_12_12.model) and its frame renderer.
// a DQNetwork's parameters as dynet::TextFileLoader reads them (rt_dynet_read)
struct DqnModel {
    std::vector<int32_t> rows, cols;
    std::vector<float> values;
    const float* W[4];
    const float* b[4];
    int32_t hidden[3];
    int n_in = 0, n_out = 0;
    explicit DqnModel(const std::string& path) {
        int n_params = 0;
        int64_t n_values = 0;
        detail::check(rt_dynet_read(path.c_str(), 0, nullptr, nullptr, nullptr, &n_params, &n_values));
        if (n_params != 8) throw std::runtime_error("expected 4 fully connected layers (8 parameters)");
        rows.resize(n_params);
        cols.resize(n_params);
        values.resize((size_t)n_values);
        detail::check(rt_dynet_read(path.c_str(), n_params, rows.data(), cols.data(), values.data(), &n_params,
                                    &n_values));
        size_t off = 0;
        for (int l = 0; l < 4; ++l) {
            W[l] = values.data() + off;
            off += (size_t)rows[2 * l] * std::max(cols[2 * l], 1);  // cols 0: a vector
            b[l] = values.data() + off;
            off += (size_t)rows[2 * l + 1] * std::max(cols[2 * l + 1], 1);
        }
        for (int l = 0; l < 3; ++l) hidden[l] = rows[2 * l];
        n_in = cols[0];
        n_out = rows[6];
    }
};

class PretrainedPathtracer {
   public:
    PretrainedPathtracer(DeviceScene& ds, const std::string& model_path) : ds_(ds) {
        const DqnModel m(model_path);
        const std::vector<float>& v = ds.vertices();
        detail::check(rt_dqn_create(ds.ctx(), v.data(), (int)v.size(), m.hidden, m.n_out, m.W, m.b, &net_));
    }
    ~PretrainedPathtracer() {
        if (net_) rt_dqn_destroy(net_);
    }
    PretrainedPathtracer(const PretrainedPathtracer&) = delete;
    PretrainedPathtracer& operator=(const PretrainedPathtracer&) = delete;

    // render_frame (pre_trained_pathtracer.cu:188-376): returns the frame's ray casts
    uint64_t render_frame(SDLScreen& screen, const Camera& camera, int spp = 32) {
        const rt_params p = gpu_engine_params(screen, spp);
        const rt_camera cam = camera.to_rt();
        std::vector<float> rgb((size_t)screen.width * screen.height * 3);
        uint64_t casts = 0;
        detail::check(rt_render_dqn(ds_.ctx(), ds_.scene(), net_, &cam, &p, 0, 0, screen.width, screen.height,
                                    rgb.data(), &casts));
        screen.PutFrame(rgb.data());
        return casts;
    }

   private:
    DeviceScene& ds_;
    rt_dqn* net_ = nullptr;
};

// GPU/deep_learning/neural_q_pathtracer.cuh: renders while training the Q-network
// (NeuralQPathtracer, main.cu:114-124: batch 4096), starting from a saved model (the
// reference's LOAD_MODEL path, neural_q_pathtracer.cu:54-59); each sample's statistics
// go to nn_training_stats.txt (:577-583) and save_model writes the trained network in
// the reference's format (dynet::TextFileSaver, :193).
class NeuralQPathtracer {
   public:
    NeuralQPathtracer(DeviceScene& ds, const std::string& model_path, unsigned batch_size = 4096,
                      const std::string& stats_path = "nn_training_stats.txt")
        : ds_(ds), stats_path_(stats_path) {
        const DqnModel m(model_path);
        const std::vector<float>& v = ds.vertices();
        shapes_.assign(m.rows.begin(), m.rows.end());
        n_in_ = m.n_in;
        detail::check(rt_dqn_trainer_create(ds.ctx(), v.data(), (int)v.size(), m.hidden, m.n_out, m.W, m.b, 1e-3f,
                                            &trainer_));
        // EPSILON_START / EPSILON_MIN / EPSILON_DECAY (constants/deep_learning_settings.h:5-7)
        detail::check(rt_neuralq_create(ds.ctx(), ds.scene(), trainer_, (int)batch_size, 0.05f, 0.05f, 0.01f, &nq_));
    }
    ~NeuralQPathtracer() {
        if (nq_) rt_neuralq_destroy(nq_);
        if (trainer_) rt_dqn_trainer_destroy(trainer_);
    }
    NeuralQPathtracer(const NeuralQPathtracer&) = delete;
    NeuralQPathtracer& operator=(const NeuralQPathtracer&) = delete;

    // render_frame (neural_q_pathtracer.cu:226-600): returns the frame's ray casts
    uint64_t render_frame(SDLScreen& screen, const Camera& camera, int spp = 32) {
        const rt_params p = gpu_engine_params(screen, spp);
        const rt_camera cam = camera.to_rt();
        std::vector<float> rgb((size_t)screen.width * screen.height * 3), stats((size_t)spp * 3);
        uint64_t casts = 0;
        detail::check(rt_neuralq_render_frame(ds_.ctx(), nq_, &cam, &p, rgb.data(), stats.data(), &casts));
        screen.PutFrame(rgb.data());
        std::ofstream f(stats_path_, std::ios::app);
        for (int s = 0; s < spp; ++s)
            f << stats[3 * s] << " " << stats[3 * s + 1] << " " << (long long)stats[3 * s + 2] << "\n";
        if (!f) throw std::runtime_error("cannot append to " + stats_path_);
        return casts;
    }

    float epsilon() const {
        float e = 0.f;
        detail::check(rt_neuralq_epsilon(nq_, &e));
        return e;
    }

    // the trained network in the reference's DyNet text format
    void save_model(const std::string& path) const {
        std::vector<std::vector<float>> W(4), b(4);
        float* Wp[4];
        float* bp[4];
        int32_t rows[8], cols[8];
        int in = n_in_;
        for (int l = 0; l < 4; ++l) {
            const int out = shapes_[2 * l];
            W[l].resize((size_t)out * in);
            b[l].resize((size_t)out);
            Wp[l] = W[l].data();
            bp[l] = b[l].data();
            rows[2 * l] = out;
            cols[2 * l] = in;
            rows[2 * l + 1] = out;
            cols[2 * l + 1] = 0;  // a vector
            in = out;
        }
        detail::check(rt_dqn_trainer_params(trainer_, Wp, bp));
        std::vector<float> flat;
        for (int l = 0; l < 4; ++l) {
            flat.insert(flat.end(), W[l].begin(), W[l].end());
            flat.insert(flat.end(), b[l].begin(), b[l].end());
        }
        detail::check(rt_dynet_write(path.c_str(), 8, rows, cols, flat.data()));
    }

   private:
    DeviceScene& ds_;
    std::string stats_path_;
    std::vector<int32_t> shapes_;
    int n_in_ = 0;
    rt_dqn_trainer* trainer_ = nullptr;
    rt_neuralq* nq_ = nullptr;
};

}  // namespace rtmi
