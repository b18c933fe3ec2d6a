// sdl_screen.h — SDLScreen with the reference's interface (CPU/sdl/sdl_screen.h:11-30),
// headless: the ARGB buffer, PutPixelSDL's pack rule and a BMP writer.
// SDL2 is absent on the build and GPU hosts, so there is no window; a
// front end that has SDL can blit `buffer` itself.
#pragma once

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/rtmi.h"
#include "rt_vec.hpp"

namespace rtmi {

class SDLScreen {
   public:
    uint32_t* buffer;
    int height;
    int width;
    int frames_presented = 0;

    SDLScreen(int w, int h, bool fullscreen = false) : height(h), width(w) {
        (void)fullscreen;
        buffer = new uint32_t[(size_t)w * (size_t)h];
        memset(buffer, 0, sizeof(uint32_t) * (size_t)w * (size_t)h);
    }

    bool NoQuitMessageSDL() { return true; }

    // CPU/sdl/sdl_screen.cpp:100-112
    void PutPixelSDL(int x, int y, vec3 colour) {
        if (x < 0 || x >= width || y < 0 || y >= height) return;
        const float rgb[3] = {colour.r, colour.g, colour.b};
        rt_pack_argb(rgb, 1, &buffer[(size_t)y * width + x]);
    }

    // whole-frame form used by the renderer: rgb is height*width*3, row-major
    void PutFrame(const float* rgb) { rt_pack_argb(rgb, width * height, buffer); }

    void SDL_Renderframe() { ++frames_presented; }

    void SDL_SaveImage(const char* filename) {
        if (rt_save_bmp(filename, buffer, width, height) != RT_OK)
            fprintf(stderr, "SDL_SaveImage: %s\n", rt_last_error());
    }

    void kill_screen() {
        delete[] buffer;
        buffer = nullptr;
    }
};

}  // namespace rtmi
