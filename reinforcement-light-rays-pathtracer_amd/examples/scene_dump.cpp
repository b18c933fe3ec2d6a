// scene_dump.cpp — the reference's scene set-up call (GPU/main.cu:110-111,
// `scene.load_custom_scene("../Models/archway.obj", false)`) against the drop-in facade,
// with the loaded Scene written out so the tests can compare it with the C ABI.
//
//   ./build/scene_dump <scene.obj> <0|1 = lights_in_obj> <out.bin>
//
// out.bin: int32 counts (surfaces, area lights, vertices), then per surface v0,v1,v2 (xyz)
// and the diffuse colour (12 floats), per area light v0,v1,v2 and diffuse_p (12 floats),
// then the NN vertex list (3 floats per vertex).  Host only: no GPU is touched.
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#include "../host/scene.h"

using namespace rtmi;

static void put_tri(std::vector<float>& o, const Triangle& t, vec3 c) {
    for (const vec4& v : {t.v0, t.v1, t.v2}) o.insert(o.end(), {v.x, v.y, v.z});
    o.insert(o.end(), {c.x, c.y, c.z});
}

int main(int argc, char** argv) {
    if (argc < 4) {
        fprintf(stderr, "usage: %s <scene.obj> <lights_in_obj 0|1> <out.bin>\n", argv[0]);
        return 2;
    }
    const bool lights_in_obj = atoi(argv[2]) != 0;
    Scene scene;
    if (!scene.load_custom_scene(argv[1], lights_in_obj)) {
        fprintf(stderr, "cannot load %s\n", argv[1]);
        return 1;
    }
    std::vector<float> body;
    for (const Surface& s : scene.surfaces) put_tri(body, s, s.material.diffuse_c);
    for (const AreaLight& l : scene.area_lights) put_tri(body, l, l.diffuse_p);
    body.insert(body.end(), scene.vertices.begin(), scene.vertices.end());
    const int32_t counts[3] = {scene.surfaces_count, scene.area_light_count, scene.vertices_count};
    FILE* f = fopen(argv[3], "wb");
    if (!f) return 1;
    const bool ok = fwrite(counts, sizeof(int32_t), 3, f) == 3 &&
                    fwrite(body.data(), sizeof(float), body.size(), f) == body.size();
    if (fclose(f) != 0 || !ok) return 1;
    printf("surfaces %d, area lights %d, vertices %d\n", counts[0], counts[1], counts[2]);
    return 0;
}
