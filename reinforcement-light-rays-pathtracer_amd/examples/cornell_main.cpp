// cornell_main.cpp — the CPU engine's main (CPU/main.cpp:63-153, method 3 =
// default path tracing) written against the drop-in facade: Cornell box,
// Camera(0,0,-3,1), draw_default_path_tracing, SDL_SaveImage.
//
//   ./build/cornell_demo [out.bmp] [spp] [frames]
// With frames > 1 the frame loop of CPU/main.cpp:85-131 runs that many times (same
// camera): the facade keeps one context and device scene for all of them.
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#include "../host/camera.h"
#include "../host/default_path_tracing.h"
#include "../host/scene.h"
#include "../host/sdl_screen.h"

using namespace rtmi;

int main(int argc, char** argv) {
    const char* out = argc > 1 ? argv[1] : "render.bmp";
    const int spp = argc > 2 ? atoi(argv[2]) : 16;
    const int frames = argc > 3 ? atoi(argv[3]) : 1;
    SDLScreen screen(512, 512, false);

    std::vector<Surface> surfaces_load;
    std::vector<AreaLightPlane> light_planes_load;
    get_cornell_shapes(surfaces_load, light_planes_load);
    Camera camera(vec4(0, 0, -3, 1));

    std::vector<Surface*> surfaces;
    for (auto& s : surfaces_load) surfaces.push_back(&s);
    std::vector<AreaLightPlane*> light_planes;
    for (auto& l : light_planes_load) light_planes.push_back(&l);

    try {
        for (int f = 0; f < frames && screen.NoQuitMessageSDL(); ++f) {
            draw_default_path_tracing(screen, camera, light_planes, surfaces, spp);
            screen.SDL_Renderframe();
        }
    } catch (const std::exception& e) {
        fprintf(stderr, "render failed: %s\n", e.what());
        return 1;
    }
    printf("frames %d, scene uploads %d\n", screen.frames_presented, default_path_tracer().scene_uploads());
    screen.SDL_SaveImage(out);
    screen.kill_screen();
    printf("wrote %s\n", out);
    return 0;
}
