// rt_scene_build.cpp — host-side scene construction and frame-buffer helpers
// of the C ABI: the Cornell box builders, the OBJ importer with the GPU
// engine's semantics, the PutPixelSDL pack rule and a headless BMP writer.
// No GPU code here.
#include <ctype.h>
#include <errno.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <vector>

#include "../../include/rtmi.h"

// rt_last_error plumbing lives in rt_capi.cpp; reuse it through this hook.
extern "C" const char* rt_last_error(void);
namespace rt {
int set_error(int code, const char* msg);
}

namespace {

struct V4 {
    float x, y, z, w;
};

V4 v4(float x, float y, float z, float w = 1.0f) { return V4{x, y, z, w}; }
V4 operator*(V4 a, float s) { return V4{a.x * s, a.y * s, a.z * s, a.w * s}; }
V4 operator-(V4 a, V4 b) { return V4{a.x - b.x, a.y - b.y, a.z - b.z, a.w - b.w}; }
V4 operator+(V4 a, V4 b) { return V4{a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w}; }
V4 operator*(V4 a, V4 b) { return V4{a.x * b.x, a.y * b.y, a.z * b.z, a.w * b.w}; }

// Cornell / light placement transform: v * (2/l) - (1,1,1,1); x,y negated; w = 1
// (CPU/scenes/cornell_box_scene.cpp:161-199, GPU/scenes/cornell_box_scene.cu:163-240,
//  GPU/objects/object_importer.cu:274-299)
V4 box_to_world(V4 v, float l) {
    V4 r = v * (2.0f / l);
    r = r - v4(1, 1, 1, 1);
    r.x *= -1.0f;
    r.y *= -1.0f;
    r.w = 1.0f;
    return r;
}

void put(float* dst, V4 a, V4 b, V4 c) {
    const float f[9] = {a.x, a.y, a.z, b.x, b.y, b.z, c.x, c.y, c.z};
    memcpy(dst, f, sizeof(f));
}

struct Tri {
    V4 a, b, c;
    float col[3];
};

void cornell_surfaces(std::vector<Tri>& out, V4* K, V4* I, V4* J, V4* L) {
    const float blue[3] = {0.15f, 0.15f, 0.75f}, white[3] = {0.75f, 0.75f, 0.75f},
                red[3] = {0.75f, 0.15f, 0.15f}, green[3] = {0.15f, 0.75f, 0.15f},
                yellow[3] = {0.75f, 0.75f, 0.15f}, cyan[3] = {0.15f, 0.75f, 0.75f};
    const float l = 555;
    auto add = [&](V4 a, V4 b, V4 c, const float* m) {
        Tri t{a, b, c, {m[0], m[1], m[2]}};
        out.push_back(t);
    };
    // room
    V4 A = v4(l, 0, 0), B = v4(0, 0, 0), C = v4(l, 0, l), D = v4(0, 0, l);
    V4 E = v4(l, l, 0), F = v4(0, l, 0), G = v4(l, l, l), H = v4(0, l, l);
    *I = v4(l / 3, l, (2 * l) / 3);
    *J = v4((2 * l) / 3, l, (2 * l) / 3);
    *K = v4(l / 3, l, l / 3);
    *L = v4((2 * l) / 3, l, l / 3);
    add(C, B, A, green); add(C, D, B, green);                      // floor
    add(A, E, C, white); add(C, E, G, white);                      // left wall
    add(F, B, D, white); add(H, F, D, white);                      // right wall
    add(F, H, *I, cyan); add(F, *I, *K, cyan); add(F, *K, E, cyan); // ceiling around the light
    add(*K, *L, E, cyan); add(*L, G, E, cyan); add(*L, *J, G, cyan);
    add(*I, G, *J, cyan); add(H, G, *I, cyan);
    add(G, D, C, yellow); add(G, H, D, yellow);                    // back wall
    // short block
    {
        V4 a = v4(240, 0, 234), b = v4(80, 0, 185), c = v4(190, 0, 392), d = v4(32, 0, 345);
        V4 e = v4(240, 165, 234), f = v4(80, 165, 185), g = v4(190, 165, 392), h = v4(32, 165, 345);
        add(e, b, a, blue); add(e, f, b, blue); add(f, d, b, blue); add(f, h, d, blue);
        add(h, c, d, blue); add(h, g, c, blue); add(g, e, c, blue); add(e, a, c, blue);
        add(g, f, e, blue); add(g, h, f, blue);
    }
    // tall block
    {
        V4 a = v4(443, 0, 247), b = v4(285, 0, 296), c = v4(492, 0, 406), d = v4(334, 0, 456);
        V4 e = v4(443, 330, 247), f = v4(285, 330, 296), g = v4(492, 330, 406), h = v4(334, 330, 456);
        add(e, b, a, red); add(e, f, b, red); add(f, d, b, red); add(f, h, d, red);
        add(h, c, d, red); add(h, g, c, red); add(g, e, c, red); add(e, a, c, red);
        add(g, f, e, red); add(g, h, f, red);
    }
}

// ---- OBJ import (GPU/objects/object_importer.cu:8-89) ----------------------

struct ObjData {
    std::vector<float> v;   // xyz per vertex
    std::vector<int> face;  // 3 one-based indices per fan triangle
};

// The reference reads the file word by word (fscanf "%s"); a word "v" is
// followed by three floats, a word "f" by the rest of its line, which is
// split on spaces and fan-triangulated; only the vertex index of "a/b/c" is
// used.  Every other word is skipped.
int parse_obj(const char* path, ObjData* out) {
    FILE* f = fopen(path, "r");
    if (!f) return rt::set_error(RT_E_IO, "File could not be opened");
    char word[128];
    int rc = RT_OK;
    while (fscanf(f, "%127s", word) == 1) {
        if (strcmp(word, "v") == 0) {
            float x, y, z;
            if (fscanf(f, "%f %f %f", &x, &y, &z) != 3) {
                rc = rt::set_error(RT_E_IO, "malformed vertex line");
                break;
            }
            out->v.push_back(x);
            out->v.push_back(y);
            out->v.push_back(z);
        } else if (strcmp(word, "f") == 0) {
            char line[256];
            if (!fgets(line, sizeof(line), f)) break;
            std::vector<int> idx;
            const char* p = line;
            while (*p) {
                while (*p && isspace((unsigned char)*p)) ++p;
                if (!*p) break;
                char* end = nullptr;
                errno = 0;
                long k = strtol(p, &end, 10);
                if (end == p || errno != 0) {
                    rc = rt::set_error(RT_E_IO, "malformed face line");
                    break;
                }
                idx.push_back((int)k);
                p = end;
                while (*p && !isspace((unsigned char)*p)) ++p;  // skip "/vt/vn"
            }
            if (rc != RT_OK) break;
            for (size_t i = 1; i + 1 < idx.size(); ++i) {
                out->face.push_back(idx[0]);
                out->face.push_back(idx[i]);
                out->face.push_back(idx[i + 1]);
            }
        }
    }
    fclose(f);
    if (rc != RT_OK) return rc;
    const int nv = (int)(out->v.size() / 3);
    for (int k : out->face)
        if (k < 1 || k > nv) return rt::set_error(RT_E_IO, "face index out of range");
    return RT_OK;
}

struct Built {
    std::vector<float> tri, albedo, light, emission, nn;
    std::vector<int32_t> group;
};

void push3(std::vector<float>& dst, V4 a) {
    dst.push_back(a.x);
    dst.push_back(a.y);
    dst.push_back(a.z);
}

void add_light(Built& b, V4 p, V4 q, V4 r, float e) {
    const size_t n = b.light.size();
    b.light.resize(n + 9);
    put(&b.light[n], p, q, r);
    b.emission.push_back(e);
    b.emission.push_back(e);
    b.emission.push_back(e);
    b.group.push_back((int32_t)b.group.size());
}

// build_surfaces / build_area_lights / build_surfaces_and_lights
// (GPU/objects/object_importer.cu:93-185, 210-314, 318-412)
// kind: 0 generic, 1 door_room, 2 archway, 3 complex_light_room; for door_room the bits
// of `variant` select among the blocks the reference leaves commented or active at HEAD
// (RT_DOOR_* in rtmi.h).
int build_obj(const ObjData& o, int kind, int variant, Built* b) {
    const int nv = (int)(o.v.size() / 3);
    float max_pos[3] = {0.f, 0.f, 0.f}, min_pos[3] = {0.f, 0.f, 0.f};  // start at 0 as the reference
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < nv; ++j) {
            const float c = o.v[(size_t)j * 3 + i];
            if (c > max_pos[i]) max_pos[i] = c;
            if (c < min_pos[i]) min_pos[i] = c;
        }
    const float scale = 2.f;
    const float dx = -1.f - (min_pos[0] * scale), dy = -1.f - (min_pos[1] * scale),
                dz = -1.f - (min_pos[2] * scale);
    const V4 rot = v4(-1.f, -1.f, 1.f, 1.f);
    const int nt = (int)(o.face.size() / 3);
    auto vert = [&](int k) {
        const float* p = &o.v[(size_t)(k - 1) * 3];
        V4 r = v4(p[0], p[1], p[2], 1.f) * scale;
        r = r + v4(dx, dy, dz, 0.f);
        r = r * rot;
        r.w = 1.f;
        return r;
    };
    for (int i = 0; i < nt; ++i) {
        const V4 v1 = vert(o.face[(size_t)i * 3 + 0]);
        const V4 v2 = vert(o.face[(size_t)i * 3 + 1]);
        const V4 v3 = vert(o.face[(size_t)i * 3 + 2]);
        if (kind == 3 && ((i > 23 && i < 36) || (i > 50 && i < 63))) {
            add_light(*b, v1, v3, v2, 12.f * 1.f);
        } else {
            float col[3] = {0.75f, 0.75f, 0.75f};
            if (kind == 2) {  // archway materials active at HEAD (:157-163)
                if (i > 80) { col[0] = 0.75f; col[1] = 0.15f; col[2] = 0.15f; }
                if (11 < i && i < 24) { col[0] = 0.15f; col[1] = 0.15f; col[2] = 0.75f; }
            } else if (kind == 1) {  // door_room
                // red door (:152-155, commented at HEAD), then the blue block (:161-163, active).
                // Both on: the scene of the thesis's 128-spp comparison renders
                // (Images/door_room/default_128spp_50avg.png: mean and path length match).
                if (!(variant & RT_DOOR_WHITE_DOOR) && i > 23 && i < 36) {
                    col[0] = 0.75f; col[1] = 0.15f; col[2] = 0.15f;
                }
                if (!(variant & RT_DOOR_NO_BLUE) && 11 < i && i < 24) {
                    col[0] = 0.15f; col[1] = 0.15f; col[2] = 0.75f;
                }
            } else if (kind == 3) {  // complex_light_room (:382-389)
                col[0] = col[1] = col[2] = 0.9f;
                if (i >= 0 && i <= 7) col[0] = col[1] = col[2] = 0.1f;
                else if (i > 133 && i < 142) { col[0] = 0.75f; col[1] = 0.15f; col[2] = 0.15f; }
            }
            const size_t n = b->tri.size();
            b->tri.resize(n + 9);
            put(&b->tri[n], v1, v3, v2);  // Surface(v1, v3, v2, mat)
            b->albedo.insert(b->albedo.end(), col, col + 3);
        }
        // Scene::vertices keeps OBJ order v1, v2, v3
        push3(b->nn, v1);
        push3(b->nn, v2);
        push3(b->nn, v3);
    }
    if (kind == 1 || kind == 2) {
        const float l = 2.f;
        std::vector<V4> quad;
        if (kind == 1 && !(variant & RT_DOOR_ARCHWAY_LIGHTS)) {  // door room block, commented at HEAD (:216-237)
            V4 I = v4((6.3f * l) / 8, (l * 6.f) / 8, 1.499f * l);
            V4 J = v4((6.3f * l) / 8, 0, 1.499f * l);
            V4 K = v4((2.58f * l) / 8, (l * 6.f) / 8, 1.499f * l);
            V4 L = v4((2.58f * l) / 8, 0, 1.499f * l);
            quad = {K, I, J, K, J, L};
        } else {  // archway (:240-271)
            V4 I = v4(l + 1.99f, l, (float)(2.5 * l));
            V4 J = v4(l + 1.99f, (l * 4.f) / 8, 2.5f * l);
            V4 K = v4(l + 1.99f, l, 2.f * l);
            V4 L = v4(l + 1.99f, (l * 4.f) / 8, 2.f * l);
            V4 M = v4(l - 1.99f, l, 2.5f * l);
            V4 N = v4(l - 1.99f, (l * 4.f) / 8, 2.5f * l);
            V4 O = v4(l - 1.99f, l, 2.0f * l);
            V4 P = v4(l - 1.99f, (l * 4.f) / 8, 2.0f * l);
            V4 Q = v4(l - 0.5f, l, 2.99f * l);
            V4 R = v4(l - 0.5f, l * 0.5f, 2.99f * l);
            V4 S = v4(l + 0.5f, l, 2.99f * l);
            V4 T = v4(l + 0.5f, l * 0.5f, 2.99f * l);
            quad = {K, I, J, K, J, L, O, M, N, O, N, P, S, Q, R, S, R, T};
        }
        for (size_t k = 0; k < quad.size(); k += 3) {
            const V4 a = box_to_world(quad[k], l), c = box_to_world(quad[k + 1], l),
                     d = box_to_world(quad[k + 2], l);
            add_light(*b, a, c, d, 8.f * 1.f);
            push3(b->nn, a);
            push3(b->nn, c);
            push3(b->nn, d);
        }
    }
    return RT_OK;
}

uint32_t chan8(float c) {
    // uint32_t(glm::clamp(255*c, 0.f, 255.f)); glm::clamp = min(max(x, lo), hi)
    float v = 255.0f * c;
    v = (v < 0.0f) ? 0.0f : v;
    v = (255.0f < v) ? 255.0f : v;
    return (uint32_t)v;
}

}  // namespace

extern "C" {

int rt_cornell_counts(int* n_surf, int* n_light) {
    if (!n_surf || !n_light) return rt::set_error(RT_E_INVALID, "NULL argument");
    *n_surf = 36;
    *n_light = 2;
    return RT_OK;
}

int rt_cornell_geometry(int variant, float* tri_v, float* albedo, float* light_v, float* emission,
                        int32_t* light_group) {
    if (variant != RT_PRESET_CPU && variant != RT_PRESET_GPU)
        return rt::set_error(RT_E_INVALID, "bad Cornell variant");
    if (!tri_v || !albedo || !light_v || !emission || !light_group)
        return rt::set_error(RT_E_INVALID, "NULL argument");
    const float l = 555;
    std::vector<Tri> tris;
    V4 K, I, J, L;
    cornell_surfaces(tris, &K, &I, &J, &L);
    for (size_t i = 0; i < tris.size(); ++i) {
        put(tri_v + i * 9, box_to_world(tris[i].a, l), box_to_world(tris[i].b, l), box_to_world(tris[i].c, l));
        memcpy(albedo + i * 3, tris[i].col, sizeof(float) * 3);
    }
    const V4 k = box_to_world(K, l), ii = box_to_world(I, l), j = box_to_world(J, l), ll = box_to_world(L, l);
    put(light_v, k, ii, j);      // fan of plane (K,I,J,L): (K,I,J), (K,J,L)
    put(light_v + 9, k, j, ll);
    for (int q = 0; q < 2; ++q) {
        if (variant == RT_PRESET_CPU) {  // 1.f * vec3(1, 1, 0.9): one plane, index 0
            emission[q * 3 + 0] = 1.f * 1.f;
            emission[q * 3 + 1] = 1.f * 1.f;
            emission[q * 3 + 2] = 1.f * 0.9f;
            light_group[q] = 0;
        } else {  // 14.f * vec3(0.9, 0.9, 0.9): two AreaLights
            emission[q * 3 + 0] = 14.f * 0.9f;
            emission[q * 3 + 1] = 14.f * 0.9f;
            emission[q * 3 + 2] = 14.f * 0.9f;
            light_group[q] = q;
        }
    }
    return RT_OK;
}

int rt_obj_geometry(const char* path, int scene_kind, float* tri_v, float* albedo, int* n_surf,
                    float* light_v, float* emission, int32_t* light_group, int* n_light,
                    float* nn_vertices, int* n_nn_floats) {
    if (!path || !n_surf || !n_light) return rt::set_error(RT_E_INVALID, "NULL argument");
    const int kind = scene_kind & 0xff, variant = scene_kind >> 8;
    if (kind < 0 || kind > 3) return rt::set_error(RT_E_INVALID, "bad scene_kind");
    if (variant != 0 && (kind != 1 || (variant & ~7) != 0)) return rt::set_error(RT_E_INVALID, "bad variant bits");
    ObjData o;
    int rc = parse_obj(path, &o);
    if (rc != RT_OK) return rc;
    Built b;
    rc = build_obj(o, kind, variant, &b);
    if (rc != RT_OK) return rc;
    const int ns = (int)(b.tri.size() / 9), nl = (int)(b.light.size() / 9);
    if (tri_v || albedo || light_v || emission || light_group) {
        if (*n_surf < ns || *n_light < nl) return rt::set_error(RT_E_INVALID, "arrays too small");
        if (tri_v) memcpy(tri_v, b.tri.data(), sizeof(float) * b.tri.size());
        if (albedo) memcpy(albedo, b.albedo.data(), sizeof(float) * b.albedo.size());
        if (light_v) memcpy(light_v, b.light.data(), sizeof(float) * b.light.size());
        if (emission) memcpy(emission, b.emission.data(), sizeof(float) * b.emission.size());
        if (light_group) memcpy(light_group, b.group.data(), sizeof(int32_t) * b.group.size());
    }
    if (nn_vertices) {
        if (!n_nn_floats || *n_nn_floats < (int)b.nn.size())
            return rt::set_error(RT_E_INVALID, "nn_vertices too small");
        memcpy(nn_vertices, b.nn.data(), sizeof(float) * b.nn.size());
    }
    if (n_nn_floats) *n_nn_floats = (int)b.nn.size();
    *n_surf = ns;
    *n_light = nl;
    return RT_OK;
}

int rt_pack_argb(const float* rgb, int n, uint32_t* out_argb) {
    if (n < 0) return rt::set_error(RT_E_INVALID, "n < 0");
    if (n > 0 && (!rgb || !out_argb)) return rt::set_error(RT_E_INVALID, "NULL argument");
    for (int i = 0; i < n; ++i)
        out_argb[i] = (128u << 24) + (chan8(rgb[3 * i]) << 16) + (chan8(rgb[3 * i + 1]) << 8) +
                      chan8(rgb[3 * i + 2]);
    return RT_OK;
}

int rt_save_bmp(const char* path, const uint32_t* argb, int width, int height) {
    if (!path || !argb || width <= 0 || height <= 0) return rt::set_error(RT_E_INVALID, "bad argument");
    FILE* f = fopen(path, "wb");
    if (!f) return rt::set_error(RT_E_IO, "cannot open output file");
    const uint32_t img = (uint32_t)width * (uint32_t)height * 4u;
    unsigned char h[54] = {0};
    auto w32 = [&](int off, uint32_t v) {
        h[off] = (unsigned char)v; h[off + 1] = (unsigned char)(v >> 8);
        h[off + 2] = (unsigned char)(v >> 16); h[off + 3] = (unsigned char)(v >> 24);
    };
    h[0] = 'B'; h[1] = 'M';
    w32(2, 54u + img); w32(10, 54u); w32(14, 40u);
    w32(18, (uint32_t)width); w32(22, (uint32_t)(-height));  // top-down rows
    h[26] = 1; h[28] = 32;
    w32(34, img);
    int ok = fwrite(h, 1, 54, f) == 54;
    for (int y = 0; ok && y < height; ++y)  // little-endian ARGB = B,G,R,A bytes
        ok = fwrite(argb + (size_t)y * width, 4, (size_t)width, f) == (size_t)width;
    ok = (fclose(f) == 0) && ok;
    return ok ? RT_OK : rt::set_error(RT_E_IO, "write failed");
}

// 8-bit RGB PNG of the frame buffer (the thesis images are
// PNGs, Images/*/reference.png).  No zlib in the image: the IDAT stream is zlib with
// stored (uncompressed) deflate blocks of <= 65535 bytes, filter type 0 per row,
// CRC-32 per chunk and Adler-32 over the raw rows.  RGB from the ARGB packing of
// PutPixelSDL (alpha dropped).
int rt_save_png(const char* path, const uint32_t* argb, int width, int height) {
    if (!path || !argb || width <= 0 || height <= 0 || width > (1 << 24) || height > (1 << 24))
        return rt::set_error(RT_E_INVALID, "bad argument");
    static uint32_t crc_tab[256];
    static bool crc_init = false;
    if (!crc_init) {
        for (uint32_t n = 0; n < 256; ++n) {
            uint32_t c = n;
            for (int k = 0; k < 8; ++k) c = (c & 1u) ? 0xedb88320u ^ (c >> 1) : c >> 1;
            crc_tab[n] = c;
        }
        crc_init = true;
    }
    auto crc = [&](uint32_t c, const unsigned char* b, size_t n) {
        for (size_t i = 0; i < n; ++i) c = crc_tab[(c ^ b[i]) & 0xffu] ^ (c >> 8);
        return c;
    };
    const size_t row = (size_t)width * 3 + 1;
    std::vector<unsigned char> raw(row * (size_t)height);
    for (int y = 0; y < height; ++y) {
        unsigned char* r = raw.data() + (size_t)y * row;
        r[0] = 0;  // filter: none
        for (int x = 0; x < width; ++x) {
            const uint32_t v = argb[(size_t)y * width + x];
            r[1 + 3 * x] = (unsigned char)(v >> 16);
            r[2 + 3 * x] = (unsigned char)(v >> 8);
            r[3 + 3 * x] = (unsigned char)v;
        }
    }
    std::vector<unsigned char> z;
    z.reserve(raw.size() + raw.size() / 65535 * 5 + 16);
    z.push_back(0x78);
    z.push_back(0x01);
    uint32_t a1 = 1, a2 = 0;
    for (size_t off = 0; off < raw.size() || off == 0; ) {
        const size_t n = std::min<size_t>(65535, raw.size() - off);
        const bool last = off + n >= raw.size();
        z.push_back(last ? 1 : 0);
        z.push_back((unsigned char)n);
        z.push_back((unsigned char)(n >> 8));
        z.push_back((unsigned char)~n);
        z.push_back((unsigned char)(~n >> 8));
        z.insert(z.end(), raw.begin() + off, raw.begin() + off + n);
        for (size_t i = off; i < off + n; ++i) {
            a1 = (a1 + raw[i]) % 65521u;
            a2 = (a2 + a1) % 65521u;
        }
        off += n;
        if (last) break;
    }
    const uint32_t adler = (a2 << 16) | a1;
    for (int k = 3; k >= 0; --k) z.push_back((unsigned char)(adler >> (8 * k)));
    FILE* f = fopen(path, "wb");
    if (!f) return rt::set_error(RT_E_IO, "cannot open output file");
    bool ok = true;
    auto put32 = [&](unsigned char* b, uint32_t v) {
        b[0] = (unsigned char)(v >> 24); b[1] = (unsigned char)(v >> 16);
        b[2] = (unsigned char)(v >> 8); b[3] = (unsigned char)v;
    };
    auto chunk = [&](const char* type, const unsigned char* data, size_t n) {
        unsigned char hd[8];
        put32(hd, (uint32_t)n);
        memcpy(hd + 4, type, 4);
        uint32_t c = crc(0xffffffffu, hd + 4, 4);
        c = crc(c, data, n) ^ 0xffffffffu;
        unsigned char tl[4];
        put32(tl, c);
        ok = ok && fwrite(hd, 1, 8, f) == 8 && (n == 0 || fwrite(data, 1, n, f) == n) && fwrite(tl, 1, 4, f) == 4;
    };
    static const unsigned char sig[8] = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1a, '\n'};
    ok = fwrite(sig, 1, 8, f) == 8;
    unsigned char ihdr[13];
    put32(ihdr, (uint32_t)width);
    put32(ihdr + 4, (uint32_t)height);
    ihdr[8] = 8; ihdr[9] = 2; ihdr[10] = 0; ihdr[11] = 0; ihdr[12] = 0;  // 8-bit RGB
    chunk("IHDR", ihdr, 13);
    chunk("IDAT", z.data(), z.size());
    chunk("IEND", nullptr, 0);
    ok = (fclose(f) == 0) && ok;
    return ok ? RT_OK : rt::set_error(RT_E_IO, "write failed");
}

}  // extern "C"
