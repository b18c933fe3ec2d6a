// reinforcement_main.cpp — the GPU engine's learned-sampling main loops
// (GPU/main.cu:260-350 Expected SARSA, :420-470 pre-trained DQN) written against
// the drop-in facade: load a scene, render frames, log the per-frame statistics and
// append them to sarsa_training_stats.txt (the format of Radiance_Map_Data/sarsa_*.txt),
// save the Q-table (radiance_map_data.txt) and the last frame, in the working directory.
//
//   ./build/reinforcement_demo sarsa <scene.obj> <kind> [frames] [spp] [out.bmp]
//   ./build/reinforcement_demo dqn <scene.obj> <kind> <model> [frames] [spp] [out.bmp]
//   ./build/reinforcement_demo neuralq <scene.obj> <kind> <model> [frames] [spp] [out.bmp]
//     (trains from <model>; writes nn_training_stats.txt and trained.model)
//   (kind: 1 door_room, 2 archway, 3 complex_light_room; scene "cornell" = the Cornell box)
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>

#include "../host/camera.h"
#include "../host/reinforcement_path_tracing.h"
#include "../host/scene.h"
#include "../host/sdl_screen.h"

using namespace rtmi;

static vec4 camera_for(int kind) {  // GPU/main.cu:100-104
    switch (kind) {
        case 1: return vec4(0.f, 0.5f, -0.9f, 1.f);
        case 2: return vec4(-1.f, 0.2f, -0.99f, 1.f);
        case 3: return vec4(-1.f, -1.f, -0.4f, 1.f);
        default: return vec4(0.f, 0.f, -3.f, 1.f);
    }
}

int main(int argc, char** argv) {
    if (argc < 4) {
        fprintf(stderr, "usage: %s sarsa|dqn <scene.obj|cornell> <kind> [model] [frames] [spp] [out.bmp]\n", argv[0]);
        return 2;
    }
    const bool nq = strcmp(argv[1], "neuralq") == 0;
    const bool dqn = nq || strcmp(argv[1], "dqn") == 0;
    const int kind = atoi(argv[3]);
    int a = 4;
    const char* model = dqn ? (argc > a ? argv[a++] : "") : "";
    const int frames = argc > a ? atoi(argv[a++]) : 4;
    const int spp = argc > a ? atoi(argv[a++]) : 32;
    const char* out = argc > a ? argv[a++] : "render.bmp";
    Scene scene;
    if (strcmp(argv[2], "cornell") == 0) scene.load_cornell_box_scene();
    else if (!scene.load_custom_scene_kind(argv[2], kind)) {
        fprintf(stderr, "cannot load %s\n", argv[2]);
        return 1;
    }
    SDLScreen screen(512, 512, false);
    Camera camera(camera_for(kind));
    try {
        DeviceScene ds(scene);
        if (nq) {
            NeuralQPathtracer pt(ds, model);
            for (int f = 0; f < frames; ++f) {
                const uint64_t casts = pt.render_frame(screen, camera, spp);
                printf("frame %d: %llu ray casts, epsilon %.3f\n", f, (unsigned long long)casts, pt.epsilon());
            }
            pt.save_model("trained.model");
        } else if (dqn) {
            PretrainedPathtracer pt(ds, model);
            for (int f = 0; f < frames; ++f) {
                const uint64_t casts = pt.render_frame(screen, camera, spp);
                printf("frame %d: average path length %.3f\n", f,
                       (double)casts / ((double)screen.width * screen.height * spp));
            }
        } else {
            RadianceMap map(ds);
            printf("radiance volumes: %d (KD array %d)\n", map.radiance_volumes_count, map.radiance_array_size);
            for (int f = 0; f < frames; ++f) {
                const uint64_t casts = draw_reinforcement_path_tracing(screen, camera, map, spp);
                printf("frame %d: average path length %.3f\n", f,
                       (double)casts / ((double)screen.width * screen.height * spp));
                // GPU/main.cu:321-339: the logged statistics and the training-stats line
                float avg = 0.f;
                uint64_t zero = 0;
                map.frame_stats(screen.width * screen.height, &avg, &zero);
                printf("Average Path Length: %.3f\n", avg);
                printf("Zero contribution light paths: %llu\n", (unsigned long long)zero);
                map.append_training_stats("sarsa_training_stats.txt", screen.width * screen.height);
                update_radiance_volume_distributions(map);
            }
            map.save_q_vals_to_file("radiance_map_data.txt");  // SAVE_RADIANCE_MAP (main.cu:353-369)
        }
    } catch (const std::exception& e) {
        fprintf(stderr, "render failed: %s\n", e.what());
        return 1;
    }
    screen.SDL_Renderframe();
    screen.SDL_SaveImage(out);
    screen.kill_screen();
    printf("wrote %s\n", out);
    return 0;
}
