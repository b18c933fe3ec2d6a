// rt_dqn_host.cpp — C ABI of the DQN path (BASELINE config 4): the DyNet text
// model reader (TextFileLoader of GPU/deep_learning/pre_trained_pathtracer.cu:45-53),
// the device network (DQNetwork::initialize, NN_Builders/dq_network.cu:8-33),
// and the wavefront render driver (PretrainedPathtracer::render_frame,
// pre_trained_pathtracer.cu:188-376).
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <fstream>

#include <string>
#include <vector>

#include "../../include/rtmi.h"
#include "rt_internal.hpp"

namespace rt {
int set_error(int code, const char* msg);
int ctx_device(const rt_ctx* ctx);
const DeviceScene& scene_device(const rt_scene* s);
DeviceScene scene_launch_view(const rt_scene* s);
int scene_ensure_ctab(const rt_scene* scene, int rule, float t_scale, bool wanted);
bool ctab_wanted(const rt_scene* sc, const rt_camera* cam, const rt_params* p, int user);
int ctx_blocks(rt_ctx* ctx, const int32_t* tiles, int n_tiles, int tile_size, int width, int height,
               const BlockDesc** d_blocks, int* n_blocks);
}  // namespace rt

namespace {

int err(int code, const std::string& m) { return rt::set_error(code, m.c_str()); }

#define RT_HIPE(expr)                                                                          \
    do {                                                                                       \
        hipError_t e_ = (expr);                                                                \
        if (e_ != hipSuccess) return err(RT_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

uint16_t to_bf16(float f) {  // round to nearest even (NaN stays NaN)
    uint32_t u;
    memcpy(&u, &f, 4);
    if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40u);
    u += 0x7fffu + ((u >> 16) & 1u);
    return (uint16_t)(u >> 16);
}

int pad32(int x) { return (x + 31) / 32 * 32; }

}  // namespace

struct rt_dqn {
    int device = 0;
    int n_in = 0, n_out = 0, h[3] = {0, 0, 0};
    rt::DqnNet net;
    std::vector<void*> allocs;
    ~rt_dqn() {
        (void)hipSetDevice(device);
        for (void* p : allocs) (void)hipFree(p);
    }
};

extern "C" {

int rt_dynet_read(const char* path, int max_params, int32_t* rows, int32_t* cols, float* values,
                  int* n_params, int64_t* n_values) {
    if (!path || !n_params || !n_values) return err(RT_E_INVALID, "NULL argument");
    FILE* f = fopen(path, "r");
    if (!f) return err(RT_E_IO, std::string("cannot open ") + path);
    int np = 0;
    int64_t nv = 0;
    int rc = RT_OK;
    char head[512];
    while (fgets(head, sizeof(head), f)) {
        if (strncmp(head, "#Parameter#", 11) != 0 && strncmp(head, "#LookupParameter#", 17) != 0) continue;
        const char* br = strchr(head, '{');
        int r = 0, c = 1;
        if (!br || sscanf(br, "{%d,%d}", &r, &c) < 1) {
            rc = err(RT_E_IO, "bad #Parameter# header");
            break;
        }
        const bool vec = !strchr(br, ',') || strchr(br, ',') > strchr(br, '}');  // vector {r}
        if (vec) c = 1;
        if (r <= 0 || c <= 0) {
            rc = err(RT_E_IO, "bad parameter shape");
            break;
        }
        const int64_t cnt = (int64_t)r * c;
        if (values && np < max_params) {
            // DyNet/Eigen store column-major: value[j*rows + i] = W[i][j]; return row-major
            float* dst = values + nv;
            for (int64_t k = 0; k < cnt; ++k) {
                float v;
                if (fscanf(f, "%f", &v) != 1) {
                    rc = err(RT_E_IO, "truncated parameter values");
                    break;
                }
                const int64_t i = k % r, j = k / r;
                dst[i * c + j] = v;
            }
            if (rc != RT_OK) break;
        } else {
            for (int64_t k = 0; k < cnt; ++k) {
                float v;
                if (fscanf(f, "%f", &v) != 1) {
                    rc = err(RT_E_IO, "truncated parameter values");
                    break;
                }
            }
            if (rc != RT_OK) break;
        }
        if (rows && np < max_params) rows[np] = r;
        if (cols && np < max_params) cols[np] = vec ? 0 : c;  // 0: a vector of r values
        ++np;
        nv += cnt;
    }
    fclose(f);
    if (rc != RT_OK) return rc;
    *n_params = np;
    *n_values = nv;
    return RT_OK;
}

int rt_dynet_write(const char* path, int n_params, const int32_t* rows, const int32_t* cols,
                   const float* values) {
    if (!path || n_params < 0 || (n_params > 0 && (!rows || !cols || !values)))
        return err(RT_E_INVALID, "NULL argument");
    int64_t total = 0;
    for (int p = 0; p < n_params; ++p) {
        if (rows[p] <= 0 || cols[p] < 0) return err(RT_E_INVALID, "bad parameter shape");
        total += (int64_t)rows[p] * (cols[p] ? cols[p] : 1);
    }
    // DyNet's loader reads values with operator>>(float), which cannot parse nan/inf
    for (int64_t k = 0; k < total; ++k)
        if (!std::isfinite(values[k])) return err(RT_E_INVALID, "non-finite parameter value");
    FILE* f = fopen(path, "w");
    if (!f) return err(RT_E_IO, std::string("cannot open ") + path);
    std::string line;
    const float* src = values;
    for (int p = 0; p < n_params && f; ++p) {
        const bool vec = cols[p] == 0;
        const int r = rows[p], c = vec ? 1 : cols[p];
        // values line first: the header carries its byte count (newline included)
        line.clear();
        char num[32];
        for (int64_t k = 0; k < (int64_t)r * c; ++k) {
            const int64_t i = k % r, j = k / r;  // column-major, as Eigen stores it
            snprintf(num, sizeof(num), "%+.8e ", (double)src[i * c + j]);
            line += num;
        }
        line += '\n';
        if (vec)
            fprintf(f, "#Parameter# /_%d {%d} %zu ZERO_GRAD\n", p, r, line.size());
        else
            fprintf(f, "#Parameter# /_%d {%d,%d} %zu ZERO_GRAD\n", p, r, c, line.size());
        fputs(line.c_str(), f);
        src += (int64_t)r * c;
    }
    const bool bad = ferror(f) != 0;
    if (fclose(f) != 0 || bad) return err(RT_E_IO, std::string("write failed: ") + path);
    return RT_OK;
}

int rt_dqn_create(rt_ctx* ctx, const float* nn_vertices, int n_in, const int32_t* hidden, int n_out,
                  const float* const* W, const float* const* b, rt_dqn** out) {
    if (!ctx || !nn_vertices || !hidden || !W || !b || !out) return err(RT_E_INVALID, "NULL argument");
    *out = nullptr;
    if (n_in <= 0 || n_in % 3 != 0) return err(RT_E_INVALID, "n_in must be a positive multiple of 3");
    if (n_out != rt::kDqnActions) return err(RT_E_UNSUPPORTED, "n_out must be 144 (12x12 grid)");
    const int dims[5] = {n_in, hidden[0], hidden[1], hidden[2], n_out};
    const int limits[3] = {224, 320, 224};
    for (int l = 0; l < 3; ++l)
        if (hidden[l] <= 0 || pad32(hidden[l]) > limits[l])
            return err(RT_E_UNSUPPORTED, "hidden widths must be <= 224, 320, 224");
    for (int l = 0; l < 4; ++l)
        if (!W[l] || !b[l]) return err(RT_E_INVALID, "NULL layer parameters");
    RT_HIPE(hipSetDevice(rt::ctx_device(ctx)));
    rt_dqn* d = new (std::nothrow) rt_dqn();
    if (!d) return err(RT_E_NOMEM, "out of host memory");
    d->device = rt::ctx_device(ctx);
    d->n_in = n_in;
    d->n_out = n_out;
    for (int l = 0; l < 3; ++l) d->h[l] = hidden[l];
    d->net.K[0] = n_in;
    d->net.N[0] = pad32(dims[1]);
    d->net.K[1] = d->net.N[0];
    d->net.N[1] = pad32(dims[2]);
    d->net.K[2] = d->net.N[1];
    d->net.N[2] = pad32(dims[3]);
    d->net.K[3] = d->net.N[2];
    d->net.N[3] = n_out;
    auto upload = [&](const void* src, size_t bytes, void** dst) -> int {
        void* p = nullptr;
        hipError_t e = hipMalloc(&p, bytes);
        if (e == hipSuccess) e = hipMemcpy(p, src, bytes, hipMemcpyHostToDevice);
        if (e != hipSuccess) {
            if (p) (void)hipFree(p);
            return err(RT_E_HIP, std::string("dqn upload: ") + hipGetErrorString(e));
        }
        d->allocs.push_back(p);
        *dst = p;
        return RT_OK;
    };
    // layer 0 folded (rt_internal.hpp): c0 = W1 v + b1, S[.][c] = column sums of W1 per coordinate
    std::vector<float4> l0((size_t)d->net.N[0], make_float4(0.0f, 0.0f, 0.0f, 0.0f));
    for (int o = 0; o < dims[1]; ++o) {
        const float* w = W[0] + (size_t)o * n_in;
        double c0 = (double)b[0][o], S[3] = {0.0, 0.0, 0.0};
        for (int i = 0; i < n_in; ++i) {
            c0 += (double)w[i] * (double)nn_vertices[i];
            S[i % 3] += (double)w[i];
        }
        l0[o] = make_float4(-(float)S[0], -(float)S[1], -(float)S[2], (float)c0);  // MFMA A operand
    }
    void* p = nullptr;
    int rc = upload(l0.data(), l0.size() * sizeof(float4), &p);
    if (rc != RT_OK) { delete d; return rc; }
    d->net.l0 = (const float4*)p;
    for (int l = 1; l < 4; ++l) {
        const int Kp = d->net.K[l], Np = d->net.N[l], in = dims[l], outd = dims[l + 1];
        std::vector<uint16_t> w((size_t)Np * Kp, 0);
        std::vector<float> bias((size_t)Np, 0.0f);
        for (int o = 0; o < outd; ++o) {
            for (int i = 0; i < in; ++i) w[(size_t)o * Kp + i] = to_bf16(W[l][(size_t)o * in + i]);
            bias[o] = b[l][o];
        }
        // fragment order (rt_internal.hpp DqnNet::W): one 16x32 B-fragment = 1 KB contiguous
        std::vector<uint16_t> wf((size_t)Np * Kp, 0);
        const int KS = Kp / 32;
        for (int nt = 0; nt < Np / 16; ++nt)
            for (int ks = 0; ks < KS; ++ks)
                for (int ln = 0; ln < 64; ++ln)
                    for (int e = 0; e < 8; ++e)
                        wf[(((size_t)nt * KS + ks) * 64 + ln) * 8 + e] =
                            w[(size_t)(nt * 16 + (ln & 15)) * Kp + ks * 32 + (ln >> 4) * 8 + e];
        rc = upload(wf.data(), wf.size() * sizeof(uint16_t), &p);
        if (rc != RT_OK) { delete d; return rc; }
        d->net.W[l] = (const uint16_t*)p;
        rc = upload(bias.data(), bias.size() * sizeof(float), &p);
        if (rc != RT_OK) { delete d; return rc; }
        d->net.b[l] = (const float*)p;
    }
    *out = d;
    return RT_OK;
}

int rt_dqn_destroy(rt_dqn* dqn) {
    delete dqn;
    return RT_OK;
}

static_assert(RT_DQN_MLP_STATIONARY == rt::kMlpStationary, "MLP mode constants");

int rt_dqn_set_mlp(rt_dqn* dqn, int mode) {
    if (!dqn) return err(RT_E_INVALID, "NULL argument");
    if (mode != RT_DQN_MLP_AUTO && mode != RT_DQN_MLP_STREAM && mode != RT_DQN_MLP_STATIONARY)
        return err(RT_E_INVALID, "bad MLP kernel mode");
    dqn->net.mlp_mode = mode;
    return RT_OK;
}

int rt_dqn_forward(rt_ctx* ctx, const rt_dqn* dqn, const float* loc, int n, float* q) {
    if (!ctx || !dqn || (n > 0 && (!loc || !q))) return err(RT_E_INVALID, "NULL argument");
    if (n < 0) return err(RT_E_INVALID, "n < 0");
    if (n == 0) return RT_OK;
    RT_HIPE(hipSetDevice(rt::ctx_device(ctx)));
    float *d_loc = nullptr, *d_q = nullptr;
    hipError_t e = hipMalloc(&d_loc, sizeof(float) * 3 * (size_t)n);
    if (e == hipSuccess) e = hipMalloc(&d_q, sizeof(float) * rt::kDqnActions * (size_t)n);
    if (e == hipSuccess) e = hipMemcpy(d_loc, loc, sizeof(float) * 3 * (size_t)n, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = rt::launch_dqn_mlp(dqn->net, d_loc, nullptr, nullptr, n, d_q, 0, 0);
    if (e == hipSuccess) e = hipMemcpy(q, d_q, sizeof(float) * rt::kDqnActions * (size_t)n, hipMemcpyDeviceToHost);
    (void)hipFree(d_loc);
    (void)hipFree(d_q);
    if (e != hipSuccess) return err(RT_E_HIP, std::string("rt_dqn_forward: ") + hipGetErrorString(e));
    return RT_OK;
}

int rt_dqn_forward_device(rt_ctx* ctx, const rt_dqn* dqn, const float* d_loc, int n, float* d_q,
                          void* stream) {
    if (!ctx || !dqn || (n > 0 && (!d_loc || !d_q))) return err(RT_E_INVALID, "NULL argument");
    if (n < 0) return err(RT_E_INVALID, "n < 0");
    RT_HIPE(hipSetDevice(rt::ctx_device(ctx)));
    RT_HIPE(rt::launch_dqn_mlp(dqn->net, d_loc, nullptr, nullptr, n, d_q, 0, (hipStream_t)stream));
    return RT_OK;
}

int rt_dqn_save_selected(rt_ctx* ctx, const rt_dqn* dqn, const char* to_select_path, const char* out_path) {
    if (!ctx || !dqn || !to_select_path || !out_path) return err(RT_E_INVALID, "NULL argument");
    std::vector<float> loc, nrm;
    int rc = rt::read_locations(to_select_path, &loc, &nrm);
    if (rc != RT_OK) return rc;
    const int n = (int)loc.size() / 3;
    std::vector<float> q((size_t)n * rt::kDqnActions);
    if (n > 0) {
        rc = rt_dqn_forward(ctx, dqn, loc.data(), n, q.data());
        if (rc != RT_OK) return rc;
    }
    // write_q_values_for_position (q_value_extractor.cu:18-71): Q normalised by its sum
    std::ofstream f(out_path);
    if (!f.is_open()) return err(RT_E_IO, std::string("cannot write ") + out_path);
    for (int i = 0; i < n; ++i) {
        const float* qi = &q[(size_t)i * rt::kDqnActions];
        float sum = 0.f;
        for (int a = 0; a < rt::kDqnActions; ++a) sum += qi[a];
        f << loc[3 * i] << " " << loc[3 * i + 1] << " " << loc[3 * i + 2];
        f << " " << nrm[3 * i] << " " << nrm[3 * i + 1] << " " << nrm[3 * i + 2];
        for (int a = 0; a < rt::kDqnActions; ++a) f << " " << qi[a] / sum;
        f << "\n";
    }
    f.close();
    if (f.fail()) return err(RT_E_IO, std::string("write failed: ") + out_path);
    return RT_OK;
}

int rt_dqn_sample(rt_ctx* ctx, const rt_scene* scene, uint64_t seed, float* q, const float* loc,
                  const int32_t* tri, const uint32_t* pix, int n, int sample, int bounce, float* tp,
                  float* dir_out, int32_t* action) {
    if (!ctx || !scene || (n > 0 && (!q || !loc || !tri || !pix || !tp || !dir_out || !action)))
        return err(RT_E_INVALID, "NULL argument");
    if (n <= 0) return n == 0 ? RT_OK : err(RT_E_INVALID, "n < 0");
    const rt::DeviceScene& s = rt::scene_device(scene);
    for (int i = 0; i < n; ++i)
        if (tri[i] < 0 || tri[i] >= s.n_surf) return err(RT_E_INVALID, "tri must index a surface");
    RT_HIPE(hipSetDevice(rt::ctx_device(ctx)));
    const size_t nq = sizeof(float) * rt::kDqnActions * (size_t)n, n3 = sizeof(float) * 3 * (size_t)n;
    float *d_q = nullptr, *d_loc = nullptr, *d_tp = nullptr, *d_dir = nullptr;
    int32_t *d_tri = nullptr, *d_act = nullptr;
    uint32_t* d_pix = nullptr;
    hipError_t e = hipMalloc(&d_q, nq);
    if (e == hipSuccess) e = hipMalloc(&d_loc, n3);
    if (e == hipSuccess) e = hipMalloc(&d_tp, n3);
    if (e == hipSuccess) e = hipMalloc(&d_dir, n3);
    if (e == hipSuccess) e = hipMalloc(&d_tri, sizeof(int32_t) * n);
    if (e == hipSuccess) e = hipMalloc(&d_act, sizeof(int32_t) * n);
    if (e == hipSuccess) e = hipMalloc(&d_pix, sizeof(uint32_t) * n);
    if (e == hipSuccess) e = hipMemcpy(d_q, q, nq, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(d_loc, loc, n3, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(d_tp, tp, n3, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(d_tri, tri, sizeof(int32_t) * n, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(d_pix, pix, sizeof(uint32_t) * n, hipMemcpyHostToDevice);
    if (e == hipSuccess)
        e = rt::launch_dqn_sample_only(s, d_q, d_loc, d_tri, d_pix, n, sample, bounce, (uint32_t)seed,
                                       (uint32_t)(seed >> 32), d_tp, d_dir, d_act, 0);
    if (e == hipSuccess) e = hipMemcpy(q, d_q, nq, hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(tp, d_tp, n3, hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(dir_out, d_dir, n3, hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(action, d_act, sizeof(int32_t) * n, hipMemcpyDeviceToHost);
    for (void* p : {(void*)d_q, (void*)d_loc, (void*)d_tp, (void*)d_dir, (void*)d_tri, (void*)d_act, (void*)d_pix})
        (void)hipFree(p);
    if (e != hipSuccess) return err(RT_E_HIP, std::string("rt_dqn_sample: ") + hipGetErrorString(e));
    return RT_OK;
}

}  // extern "C"

namespace {

// the action-major Q buffer's leading dimension: the ray capacity rounded up to whole MLP
// workgroup tiles (every launched row is written) and to 64
int dqn_ldq(int n) {
    const int t = rt::dqn_mlp_tile_rows();
    return ((n + t - 1) / t * t + 63) / 64 * 64;
}

struct Workspace {
    rt::DqnRays r;
    std::vector<void*> allocs;
    int cap = 0;
    int device = 0;
    void release() {
        for (void* p : allocs) (void)hipFree(p);
        allocs.clear();
        cap = 0;
    }
    ~Workspace() { release(); }
    int ensure(int n) {
        if (n <= cap) {
            r.n = n;
            return RT_OK;
        }
        release();
        auto alloc = [&](size_t bytes, void** p) -> bool {
            if (hipMalloc(p, bytes) != hipSuccess) return false;
            allocs.push_back(*p);
            return true;
        };
        const size_t n3 = sizeof(float) * 3 * (size_t)n;
        bool ok = alloc(n3, (void**)&r.loc) && alloc(n3, (void**)&r.dir) && alloc(n3, (void**)&r.tp) &&
                  alloc(n3, (void**)&r.total) && alloc(sizeof(int32_t) * n, (void**)&r.tri) &&
                  alloc(sizeof(uint32_t) * n, (void**)&r.pix) && alloc(sizeof(int32_t) * n, (void**)&r.list[0]) &&
                  alloc(sizeof(int32_t) * n, (void**)&r.list[1]) && alloc(sizeof(int32_t) * 4, (void**)&r.count) &&
                  alloc(sizeof(unsigned long long), (void**)&r.casts) &&
                  alloc(sizeof(float) * rt::kDqnActions * (size_t)dqn_ldq(n), (void**)&r.q);
        if (!ok) {
            release();
            return err(RT_E_NOMEM, "DQN workspace allocation failed");
        }
        cap = n;
        r.n = n;
        r.ldq = dqn_ldq(n);
        return RT_OK;
    }
};

Workspace* g_ws_for(rt_ctx* ctx);

constexpr int kRaysInFlight = 1 << 22;  // DQN wavefront size (q: 2.4 GB at 4 M rays)

int run_dqn(rt_ctx* ctx, const rt_scene* scene, const rt_dqn* dqn, const rt_camera* cam, const rt_params* p,
            const rt::BlockDesc* d_blocks, int n_blocks, int clip_x1, int clip_y1, int out_pitch, float* d_out,
            uint64_t* d_casts, hipStream_t stream) {
    Workspace* ws = g_ws_for(ctx);
    // samples in flight: about kRaysInFlight rays per pass (all of spp for small frames)
    const int n_pix = n_blocks * 256;
    int rays_in_flight = kRaysInFlight;
    if (const char* env = getenv("RTMI_DQN_RAYS_IN_FLIGHT")) rays_in_flight = std::max(1, atoi(env));  // tests
    const int in_flight = std::max(1, std::min(p->spp, rays_in_flight / n_pix));
    int rc = ws->ensure(n_pix * in_flight);
    if (rc != RT_OK) return rc;
    // the bounce casts' candidate table (rule 1: the GPU engine's hit rule), built on the first render
    rc = rt::scene_ensure_ctab(scene, 1, p->t_scale, rt::ctab_wanted(scene, cam, p, rt::kCtabForDqn));
    if (rc != RT_OK) return rc;
    rt::DqnLaunch a;
    memset(&a, 0, sizeof(a));
    a.scene = rt::scene_launch_view(scene);  // (large scenes: the exact BVH, dqn_trace<kMfBvh>)
    a.net = dqn->net;
    a.rays = ws->r;
    if (d_casts) a.rays.casts = reinterpret_cast<unsigned long long*>(d_casts);
    else RT_HIPE(hipMemsetAsync(a.rays.casts, 0, sizeof(unsigned long long), stream));
    a.width = p->width;
    a.height = p->height;
    a.spp = p->spp;
    a.max_bounces = p->max_bounces;
    a.seed_lo = (uint32_t)p->seed;
    a.seed_hi = (uint32_t)(p->seed >> 32);
    a.t_scale = p->t_scale;
    a.env_light = p->env_light;
    a.cam_x = cam->pos[0];
    a.cam_y = cam->pos[1];
    a.cam_z = cam->pos[2];
    a.cos_y = (float)cos((double)cam->yaw_y);
    a.sin_y = (float)sin((double)cam->yaw_y);
    a.cos_x = (float)cos((double)cam->yaw_x);
    a.sin_x = (float)sin((double)cam->yaw_x);
    a.blocks = d_blocks;
    a.n_blocks = n_blocks;
    a.clip_x1 = clip_x1;
    a.clip_y1 = clip_y1;
    a.out_pitch = out_pitch;
    a.out = d_out;
    a.use_filter = rt::filter_usable(a.scene, a.cam_x, a.cam_y, a.cam_z, a.t_scale);
    int32_t* h_count = nullptr;
    RT_HIPE(hipHostMalloc((void**)&h_count, sizeof(int32_t), hipHostMallocDefault));
    a.rays.n_pix = n_pix;
    a.rays.n = n_pix;
    hipError_t e = rt::launch_dqn_frame_begin(a, stream);
    for (int s = 0; e == hipSuccess && s < p->spp; s += in_flight) {
        a.rays.s0 = s;
        a.rays.n = n_pix * std::min(in_flight, p->spp - s);
        e = hipMemsetAsync(a.rays.count, 0, sizeof(int32_t) * 2, stream);
        if (e == hipSuccess) e = rt::launch_dqn_camera(a, stream);
        for (int b = 1; e == hipSuccess && b < p->max_bounces; ++b) {
            e = hipMemsetAsync(a.rays.count + (b & 1), 0, sizeof(int32_t), stream);
            if (e == hipSuccess) e = rt::launch_dqn_bounce(a, b, stream);
            if (e == hipSuccess && (b % 4 == 0 || b == 1)) {  // stop once every path has ended
                e = hipMemcpyAsync(h_count, a.rays.count + (b & 1), sizeof(int32_t), hipMemcpyDeviceToHost, stream);
                if (e == hipSuccess) e = hipStreamSynchronize(stream);
                if (e == hipSuccess && *h_count == 0) break;
            }
        }
        if (e == hipSuccess) e = rt::launch_dqn_accumulate(a, stream);
    }
    if (e == hipSuccess) e = rt::launch_dqn_finish(a, stream);
    (void)hipHostFree(h_count);
    if (e != hipSuccess) return err(RT_E_HIP, std::string("DQN render: ") + hipGetErrorString(e));
    return RT_OK;
}

int check_dqn_params(const rt_params* p) {
    if (!p) return err(RT_E_INVALID, "params is NULL");
    if (p->width <= 0 || p->height <= 0 || p->spp <= 0) return err(RT_E_INVALID, "bad image size / spp");
    if (p->max_bounces < 1) return err(RT_E_INVALID, "max_bounces must be >= 1");
    if (p->preset != RT_PRESET_GPU || p->hit_rule != RT_HIT_RULE_GPU)
        return err(RT_E_UNSUPPORTED, "the DQN renderer implements the GPU-engine preset (hit rule GPU)");
    return RT_OK;
}

}  // namespace

extern "C" {

int rt_render_dqn_tiles_device(rt_ctx* ctx, const rt_scene* scene, const rt_dqn* dqn, const rt_camera* cam,
                               const rt_params* params, const int32_t* tiles, int n_tiles, int tile_size,
                               float* d_out, uint64_t* d_casts, void* stream) {
    if (!ctx || !scene || !dqn || !cam) return err(RT_E_INVALID, "NULL argument");
    int rc = check_dqn_params(params);
    if (rc != RT_OK) return rc;
    if (n_tiles == 0) return RT_OK;
    if (!tiles || !d_out || n_tiles < 0) return err(RT_E_INVALID, "bad tiles/out");
    RT_HIPE(hipSetDevice(rt::ctx_device(ctx)));
    const rt::BlockDesc* d_blocks = nullptr;
    int n_blocks = 0;
    rc = rt::ctx_blocks(ctx, tiles, n_tiles, tile_size, params->width, params->height, &d_blocks, &n_blocks);
    if (rc != RT_OK) return rc;
    return run_dqn(ctx, scene, dqn, cam, params, d_blocks, n_blocks, params->width, params->height, tile_size,
                   d_out, d_casts, (hipStream_t)stream);
}

int rt_render_dqn(rt_ctx* ctx, const rt_scene* scene, const rt_dqn* dqn, const rt_camera* cam,
                  const rt_params* params, int x0, int y0, int w, int h, float* out_rgb, uint64_t* out_ray_casts) {
    if (!ctx || !scene || !dqn || !cam || !out_rgb) return err(RT_E_INVALID, "NULL argument");
    int rc = check_dqn_params(params);
    if (rc != RT_OK) return rc;
    if (w <= 0 || h <= 0 || x0 < 0 || y0 < 0 || x0 + w > params->width || y0 + h > params->height)
        return err(RT_E_INVALID, "rectangle outside the image");
    RT_HIPE(hipSetDevice(rt::ctx_device(ctx)));
    std::vector<rt::BlockDesc> blocks;
    for (int by = 0; by < h; by += 16)
        for (int bx = 0; bx < w; bx += 16) blocks.push_back({x0 + bx, y0 + by, bx, by});
    rt::BlockDesc* d_blocks = nullptr;
    float* d_out = nullptr;
    uint64_t* d_casts = nullptr;
    const size_t ob = sizeof(float) * 3 * (size_t)w * h;
    hipError_t e = hipMalloc(&d_blocks, sizeof(rt::BlockDesc) * blocks.size());
    if (e == hipSuccess) e = hipMalloc(&d_out, ob);
    if (e == hipSuccess) e = hipMalloc(&d_casts, sizeof(uint64_t));
    if (e == hipSuccess) e = hipMemset(d_casts, 0, sizeof(uint64_t));
    if (e == hipSuccess)
        e = hipMemcpy(d_blocks, blocks.data(), sizeof(rt::BlockDesc) * blocks.size(), hipMemcpyHostToDevice);
    if (e == hipSuccess) {
        rc = run_dqn(ctx, scene, dqn, cam, params, d_blocks, (int)blocks.size(), x0 + w, y0 + h, w, d_out, d_casts, 0);
        if (rc == RT_OK) e = hipDeviceSynchronize();
    }
    uint64_t casts = 0;
    if (rc == RT_OK && e == hipSuccess) e = hipMemcpy(out_rgb, d_out, ob, hipMemcpyDeviceToHost);
    if (rc == RT_OK && e == hipSuccess) e = hipMemcpy(&casts, d_casts, sizeof(casts), hipMemcpyDeviceToHost);
    (void)hipFree(d_blocks);
    (void)hipFree(d_out);
    (void)hipFree(d_casts);
    if (rc != RT_OK) return rc;
    if (e != hipSuccess) return err(RT_E_HIP, std::string("rt_render_dqn: ") + hipGetErrorString(e));
    if (out_ray_casts) *out_ray_casts = casts;
    return RT_OK;
}

}  // extern "C"

// one workspace per context (contexts are single-threaded by contract)
#include <map>
#include <memory>
#include <mutex>
namespace {
std::mutex g_ws_mu;
std::map<const rt_ctx*, std::unique_ptr<Workspace>> g_ws;
Workspace* g_ws_for(rt_ctx* ctx) {
    std::lock_guard<std::mutex> lk(g_ws_mu);
    auto& w = g_ws[ctx];
    if (!w) w.reset(new Workspace());
    return w.get();
}
}  // namespace

namespace rt {
void release_dqn_workspace(const rt_ctx* ctx) {
    std::lock_guard<std::mutex> lk(g_ws_mu);
    g_ws.erase(ctx);
}
}  // namespace rt
