// scene.h — scene types and loaders with the reference's names:
//   Material / Triangle / Surface / AreaLight / AreaLightPlane
//     (CPU/objects/*.h, CPU/lights/*.h, GPU/objects/*.cuh, GPU/lights/*.cuh)
//   get_cornell_shapes  (CPU/scenes/cornell_box_scene.h:15, GPU/scenes/cornell_box_scene.cu:4)
//   load_scene          (GPU/objects/object_importer.cuh:15-16; bool lights_in_obj as at HEAD)
//   Scene               (GPU/scenes/scene.cuh:27-47)
// The geometry is produced by the C ABI (rt_cornell_geometry, rt_obj_geometry).
#pragma once

#include <stdint.h>

#include <string>
#include <vector>

#include "../../include/rtmi.h"
#include "rt_vec.hpp"

namespace rtmi {

struct Material {
    vec3 diffuse_c;
    explicit Material(vec3 c = vec3(0)) : diffuse_c(c) {}
    vec3 get_diffuse_c() const { return diffuse_c; }
};

struct Triangle {
    vec4 v0, v1, v2, normal;
    Triangle(vec4 a, vec4 b, vec4 c) : v0(a), v1(b), v2(c) { compute_and_set_normal(); }
    // CPU/objects/triangle.cpp:73-82
    void compute_and_set_normal() {
        const vec3 e1(v1.x - v0.x, v1.y - v0.y, v1.z - v0.z);
        const vec3 e2(v2.x - v0.x, v2.y - v0.y, v2.z - v0.z);
        normal = vec4(normalize(cross(e2, e1)), 1.0f);
    }
    vec4 getV0() const { return v0; }
    vec4 getV1() const { return v1; }
    vec4 getV2() const { return v2; }
    vec4 getNormal() const { return normal; }
};

struct Surface : Triangle {
    Material material;
    Surface(vec4 a, vec4 b, vec4 c, Material m) : Triangle(a, b, c), material(m) {}
    Material get_material() const { return material; }
};

struct AreaLight : Triangle {
    vec3 diffuse_p;
    AreaLight(vec4 a, vec4 b, vec4 c, vec3 e) : Triangle(a, b, c), diffuse_p(e) {}
    vec3 get_diffuse_p() const { return diffuse_p; }
};

// CPU engine light: a polygon fanned into AreaLights (CPU/lights/area_light_plane.cpp:4-22)
struct AreaLightPlane {
    std::vector<AreaLight> area_lights;
    vec3 diffuse_p;
    AreaLightPlane(const std::vector<vec4>& vertices, vec3 e) : diffuse_p(e) {
        for (size_t i = 1; i + 1 < vertices.size(); ++i)
            area_lights.emplace_back(vertices[0], vertices[i], vertices[i + 1], e);
    }
    std::vector<AreaLight> get_area_lights() const { return area_lights; }
    vec3 get_diffuse_p() const { return diffuse_p; }
};

namespace detail {
inline vec4 vtx(const float* p, int k) { return vec4(p[3 * k], p[3 * k + 1], p[3 * k + 2], 1.0f); }
}  // namespace detail

// CPU-engine signature: one light plane, emission 1*(1,1,0.9)
inline bool get_cornell_shapes(std::vector<Surface>& surfaces, std::vector<AreaLightPlane>& planes) {
    int ns = 0, nl = 0;
    rt_cornell_counts(&ns, &nl);
    std::vector<float> tri((size_t)ns * 9), alb((size_t)ns * 3), lv((size_t)nl * 9), em((size_t)nl * 3);
    std::vector<int32_t> grp(nl);
    if (rt_cornell_geometry(RT_PRESET_CPU, tri.data(), alb.data(), lv.data(), em.data(), grp.data()) != RT_OK)
        return false;
    for (int i = 0; i < ns; ++i)
        surfaces.emplace_back(detail::vtx(&tri[i * 9], 0), detail::vtx(&tri[i * 9], 1), detail::vtx(&tri[i * 9], 2),
                              Material(vec3(alb[i * 3], alb[i * 3 + 1], alb[i * 3 + 2])));
    // the fan (K,I,J), (K,J,L) of the polygon K, I, J, L
    std::vector<vec4> poly = {detail::vtx(&lv[0], 0), detail::vtx(&lv[0], 1), detail::vtx(&lv[0], 2),
                              detail::vtx(&lv[9], 2)};
    planes.emplace_back(poly, vec3(em[0], em[1], em[2]));
    return true;
}

// Flattened scene arrays in the C ABI's layout
struct SceneArrays {
    std::vector<float> tri, albedo, light, emission, vertices;
    std::vector<int32_t> light_group;
    int n_surf() const { return (int)(tri.size() / 9); }
    int n_light() const { return (int)(light.size() / 9); }
    bool same_as(const SceneArrays& o) const {
        return tri == o.tri && albedo == o.albedo && light == o.light && emission == o.emission &&
               light_group == o.light_group;
    }
};

inline void push_tri(std::vector<float>& dst, const Triangle& t) {
    const vec4 v[3] = {t.v0, t.v1, t.v2};
    for (const vec4& p : v) {
        dst.push_back(p.x);
        dst.push_back(p.y);
        dst.push_back(p.z);
    }
}

inline SceneArrays flatten(const std::vector<Surface*>& surfaces, const std::vector<AreaLightPlane*>& planes) {
    SceneArrays a;
    for (const Surface* s : surfaces) {
        push_tri(a.tri, *s);
        a.albedo.insert(a.albedo.end(), {s->material.diffuse_c.x, s->material.diffuse_c.y, s->material.diffuse_c.z});
    }
    for (size_t p = 0; p < planes.size(); ++p)
        for (const AreaLight& l : planes[p]->area_lights) {
            push_tri(a.light, l);
            a.emission.insert(a.emission.end(), {l.diffuse_p.x, l.diffuse_p.y, l.diffuse_p.z});
            a.light_group.push_back((int32_t)p);
        }
    return a;
}

inline SceneArrays flatten(const std::vector<Surface>& surfaces, const std::vector<AreaLight>& lights) {
    SceneArrays a;
    for (const Surface& s : surfaces) {
        push_tri(a.tri, s);
        a.albedo.insert(a.albedo.end(), {s.material.diffuse_c.x, s.material.diffuse_c.y, s.material.diffuse_c.z});
    }
    for (size_t i = 0; i < lights.size(); ++i) {
        push_tri(a.light, lights[i]);
        a.emission.insert(a.emission.end(), {lights[i].diffuse_p.x, lights[i].diffuse_p.y, lights[i].diffuse_p.z});
        a.light_group.push_back((int32_t)i);
    }
    return a;
}

// GPU-engine signature: two AreaLights, emission 14*(0.9,0.9,0.9), NN vertex list
inline bool get_cornell_shapes(std::vector<Surface>& surfaces, std::vector<AreaLight>& lights,
                               std::vector<float>& vertices) {
    int ns = 0, nl = 0;
    rt_cornell_counts(&ns, &nl);
    std::vector<float> tri((size_t)ns * 9), alb((size_t)ns * 3), lv((size_t)nl * 9), em((size_t)nl * 3);
    std::vector<int32_t> grp(nl);
    if (rt_cornell_geometry(RT_PRESET_GPU, tri.data(), alb.data(), lv.data(), em.data(), grp.data()) != RT_OK)
        return false;
    for (int i = 0; i < ns; ++i) {
        surfaces.emplace_back(detail::vtx(&tri[i * 9], 0), detail::vtx(&tri[i * 9], 1), detail::vtx(&tri[i * 9], 2),
                              Material(vec3(alb[i * 3], alb[i * 3 + 1], alb[i * 3 + 2])));
        vertices.insert(vertices.end(), &tri[i * 9], &tri[i * 9] + 9);
    }
    for (int j = 0; j < nl; ++j) {
        lights.emplace_back(detail::vtx(&lv[j * 9], 0), detail::vtx(&lv[j * 9], 1), detail::vtx(&lv[j * 9], 2),
                            vec3(em[j * 3], em[j * 3 + 1], em[j * 3 + 2]));
        vertices.insert(vertices.end(), &lv[j * 9], &lv[j * 9] + 9);
    }
    return true;
}

// The OBJ importer with an explicit scene kind (rt_obj_geometry): the reference's
// hard-coded material/light blocks, 0 generic (white, no lights), 1 door_room, 2 archway,
// 3 complex_light_room, plus RT_DOOR_* variant bits << 8 for the door room.  Not a
// reference name: the reference's own signature is load_scene(..., bool) below.
inline bool load_scene_kind(const char* path, std::vector<Surface>& surfaces, std::vector<AreaLight>& lights,
                            std::vector<float>& vertices, int kind) {
    int ns = 0, nl = 0, nn = 0;
    if (rt_obj_geometry(path, kind, nullptr, nullptr, &ns, nullptr, nullptr, nullptr, &nl, nullptr, &nn) != RT_OK)
        return false;
    std::vector<float> tri((size_t)ns * 9), alb((size_t)ns * 3), lv((size_t)nl * 9), em((size_t)nl * 3),
        nnv((size_t)nn);
    std::vector<int32_t> grp(nl);
    if (rt_obj_geometry(path, kind, tri.data(), alb.data(), &ns, lv.data(), em.data(), grp.data(), &nl,
                        nnv.data(), &nn) != RT_OK)
        return false;
    for (int i = 0; i < ns; ++i)
        surfaces.emplace_back(detail::vtx(&tri[i * 9], 0), detail::vtx(&tri[i * 9], 1), detail::vtx(&tri[i * 9], 2),
                              Material(vec3(alb[i * 3], alb[i * 3 + 1], alb[i * 3 + 2])));
    for (int j = 0; j < nl; ++j)
        lights.emplace_back(detail::vtx(&lv[j * 9], 0), detail::vtx(&lv[j * 9], 1), detail::vtx(&lv[j * 9], 2),
                            vec3(em[j * 3], em[j * 3 + 1], em[j * 3 + 2]));
    vertices.insert(vertices.end(), nnv.begin(), nnv.end());
    return true;
}

// GPU/objects/object_importer.cu:8-89 load_scene, the reference's signature and HEAD
// semantics (:83-88):
//   lights_in_obj == true  -> build_surfaces_and_lights (:318-412): the complex_light_room
//                             blocks, the OBJ's own light triangles      == kind 3;
//   lights_in_obj == false -> build_surfaces (:93-185, HEAD materials: red i > 80, blue
//                             11 < i < 24) + build_area_lights (:210-314, HEAD: the archway
//                             lights, emission 8)                         == kind 2.
// (The reference's `main` calls scene.load_custom_scene("../Models/archway.obj", false),
// GPU/main.cu:111.)  Returns false when the file cannot be opened or parsed.
inline bool load_scene(const char* path, std::vector<Surface>& surfaces, std::vector<AreaLight>& lights,
                       std::vector<float>& vertices, bool lights_in_obj) {
    return load_scene_kind(path, surfaces, lights, vertices, lights_in_obj ? 3 : 2);
}
// Only bool selects the reference's blocks: an int (a scene kind) does not convert silently.
template <class T>
bool load_scene(const char*, std::vector<Surface>&, std::vector<AreaLight>&, std::vector<float>&, T) = delete;

// GPU/scenes/scene.cuh:27-47 (owning flat arrays; no new[]/delete[] by the caller)
struct Scene {
    std::vector<Surface> surfaces;
    std::vector<AreaLight> area_lights;
    std::vector<float> vertices;
    int surfaces_count = 0, area_light_count = 0, vertices_count = 0;

    void load_cornell_box_scene() {
        get_cornell_shapes(surfaces, area_lights, vertices);
        counts();
    }
    // GPU/scenes/scene.cu:33-39 (lights_in_obj as in load_scene above)
    bool load_custom_scene(const char* filename, bool lights_in_obj) {
        const bool ok = load_scene(filename, surfaces, area_lights, vertices, lights_in_obj);
        counts();
        return ok;
    }
    template <class T>
    bool load_custom_scene(const char*, T) = delete;
    // explicit scene kind (load_scene_kind)
    bool load_custom_scene_kind(const char* filename, int kind) {
        const bool ok = load_scene_kind(filename, surfaces, area_lights, vertices, kind);
        counts();
        return ok;
    }

   private:
    void counts() {
        surfaces_count = (int)surfaces.size();
        area_light_count = (int)area_lights.size();
        vertices_count = (int)(vertices.size() / 3);
    }
};

}  // namespace rtmi
