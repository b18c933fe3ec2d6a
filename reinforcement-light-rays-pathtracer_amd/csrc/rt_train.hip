// rt_train.hip — Neural-Q training: the learning rule of
// NeuralQPathtracer::render_frame (GPU/deep_learning/neural_q_pathtracer.cu:420-513)
// that the reference runs through DyNet on the host, on device buffers:
//   compute_td_targets (GPU/deep_learning/nn_rendering_helpers.cu:91-140)
//     target = reward + max_a(Q(s', a) cos_a) * discount   (reward alone when terminal)
//   loss = sum_b (target_b - Q(s_b, a_b))^2    (dynet::pick + pow + sum_batches)
//   backward through the four ReLU layers of DQNetwork (NN_Builders/dq_network.cu:8-49,
//     fc_layer.cu:40-72: b + W x, rectify, no dropout)
//   dynet::AdamTrainer::update (neural_q_pathtracer.cu:47, :512) with DyNet's defaults:
//     global gradient-norm clipping at 5, beta1 0.9, beta2 0.999, eps 1e-8.
// DyNet is an un-vendored dependency; the rule is restated from its
// published algorithm, so this path's parity is against the fp64 restatement in
// oracle/oracle.py (dqn_train_step_ref), not against DyNet output: parity unpinned.
//
// MI355X mapping: fp32 throughout (the reference trains in fp32): every product is an
// LDS-tiled fp32 GEMM (64x64 tile per 256-thread workgroup, 4x4 outputs per lane,
// k-ordered fmaf, so results do not depend on the launch) with the bias + ReLU or the
// ReLU-derivative mask fused in the epilogue; the parameters, gradients and Adam moments
// are four flat device arrays so clipping and the update are two elementwise passes;
// reductions (loss, gradient norm) go through per-block partials summed in a fixed
// order (deterministic).  The inference network (rt_dqn, bf16 MFMA) is rebuilt from
// rt_dqn_trainer_params when the caller wants to render with the trained weights.
#include <hip/hip_runtime.h>

#include <math.h>
#include <string.h>

#include <algorithm>
#include <cmath>
#include <new>
#include <string>
#include <vector>

#include "../../include/rtmi.h"
#include "rt_internal.hpp"

namespace rt {
int set_error(int code, const char* msg);
int ctx_device(const rt_ctx* ctx);
const DeviceScene& scene_device(const rt_scene* s);
}  // namespace rt

namespace {

using rt::f3;

constexpr int kT = 64;   // GEMM output tile (rows and columns)
constexpr int kTK = 16;  // GEMM k step
constexpr int kRedBlocks = 256;

// C[M][N] = op(A)[M][K] * op(B)[K][N], row-major storage:
//   TA = 0: A[m * lda + k]   TA = 1: A[k * lda + m]
//   TB = 0: B[k * ldb + n]   TB = 1: B[n * ldb + k]
// EPI 0: C = acc;  1: C = max(acc + bias[n], 0) (fc_layer + rectify);
//     2: C = mask[m * ldm + n] > 0 ? acc : 0  (rectify's derivative, y > 0)
template <int TA, int TB, int EPI>
__global__ __launch_bounds__(256) void k_gemm(int M, int N, int K, const float* __restrict__ A, int lda,
                                              const float* __restrict__ B, int ldb, float* __restrict__ C,
                                              int ldc, const float* __restrict__ bias,
                                              const float* __restrict__ mask, int ldm) {
    __shared__ float As[kTK][kT + 4];
    __shared__ float Bs[kTK][kT + 4];
    const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
    const int m0 = blockIdx.y * kT, n0 = blockIdx.x * kT;
    // split K (gridDim.z > 1, EPI 0 only): slice z covers [z kc, (z + 1) kc) and writes the
    // partial product to C + z M ldc; k_sum_slices adds the slices in order
    const int kc = (K + (int)gridDim.z - 1) / (int)gridDim.z;
    const int kb = (int)blockIdx.z * kc, ke = min(K, kb + kc);
    C += (size_t)blockIdx.z * M * ldc;
    float acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = 0.0f;
    // tiles staged with the stored matrix's contiguous index fastest (coalesced); the
    // next k step's elements are loaded into registers while this step computes
    constexpr int kPer = kT * kTK / 256;  // tile elements per thread
    float ra[kPer], rb[kPer];
    auto load = [&](int k0) {
#pragma unroll
        for (int u = 0; u < kPer; ++u) {
            const int e = (int)threadIdx.x + 256 * u;
            const int mm = TA ? (e % kT) : (e / kTK);
            const int kk = TA ? (e / kT) : (e % kTK);
            const int gm = m0 + mm, gk = k0 + kk;
            ra[u] = (gm < M && gk < ke) ? (TA ? A[(size_t)gk * lda + gm] : A[(size_t)gm * lda + gk]) : 0.0f;
            const int nn = TB ? (e / kTK) : (e % kT);
            const int kb2 = TB ? (e % kTK) : (e / kT);
            const int gn = n0 + nn, gk2 = k0 + kb2;
            rb[u] = (gn < N && gk2 < ke) ? (TB ? B[(size_t)gn * ldb + gk2] : B[(size_t)gk2 * ldb + gn]) : 0.0f;
        }
    };
    if (kb < ke) load(kb);
    for (int k0 = kb; k0 < ke; k0 += kTK) {
#pragma unroll
        for (int u = 0; u < kPer; ++u) {
            const int e = (int)threadIdx.x + 256 * u;
            As[TA ? (e / kT) : (e % kTK)][TA ? (e % kT) : (e / kTK)] = ra[u];
            Bs[TB ? (e % kTK) : (e / kT)][TB ? (e / kTK) : (e % kT)] = rb[u];
        }
        __syncthreads();
        if (k0 + kTK < ke) load(k0 + kTK);
#pragma unroll
        for (int kk = 0; kk < kTK; ++kk) {
            float a[4], b[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) a[i] = As[kk][ty + 16 * i];
#pragma unroll
            for (int j = 0; j < 4; ++j) b[j] = Bs[kk][tx + 16 * j];
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[i][j] = fmaf(a[i], b[j], acc[i][j]);
        }
        __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int gm = m0 + ty + 16 * i;
        if (gm >= M) continue;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int gn = n0 + tx + 16 * j;
            if (gn >= N) continue;
            float v = acc[i][j];
            if (EPI == 1) {
                v = v + bias[gn];
                v = v > 0.0f ? v : 0.0f;
            } else if (EPI == 2) {
                v = mask[(size_t)gm * ldm + gn] > 0.0f ? v : 0.0f;
            }
            C[(size_t)gm * ldc + gn] = v;
        }
    }
}

// network input x = Scene::vertices - ray position (nn_rendering_helpers.cu:280-298)
__global__ __launch_bounds__(256) void k_build_x(const float* __restrict__ verts, int n_in,
                                                 const float* __restrict__ loc, int n, float* __restrict__ X) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= (size_t)n * n_in) return;
    const int b = (int)(i / n_in), j = (int)(i - (size_t)b * n_in);
    X[i] = verts[j] - loc[(size_t)b * 3 + (j % 3)];
}

// dynet::pick(Q, action) + pow(target - q, 2): the output gradient row of each ray is
// zero except d loss / d q_a = -2 (target - q_a), passed by the output ReLU when q_a > 0.
// Per-block partial sums of the squared errors (summed in a fixed order later).
__global__ __launch_bounds__(256) void k_loss_grad(const float* __restrict__ q, int n_out,
                                                   const int32_t* __restrict__ action,
                                                   const float* __restrict__ target, int n,
                                                   float* __restrict__ dq, float* __restrict__ partial) {
    __shared__ float red[256];
    const int b = blockIdx.x * 256 + threadIdx.x;
    float e2 = 0.0f;
    if (b < n) {
        const int a = action[b];
        if (a >= 0 && a < n_out) {
            const float qa = q[(size_t)b * n_out + a];
            const float diff = target[b] - qa;
            e2 = diff * diff;
            dq[(size_t)b * n_out + a] = qa > 0.0f ? -2.0f * diff : 0.0f;
        }
    }
    red[threadIdx.x] = e2;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
        __syncthreads();
    }
    if (threadIdx.x == 0) partial[blockIdx.x] = red[0];
}

// bias gradient: column sums of the layer's output gradient.  Stage 1: chunk y of the
// rows (in order) per column -> part[y][c]; stage 2 (k_sum_slices): the chunks in order.
__global__ __launch_bounds__(256) void k_colsum(const float* __restrict__ d, int n, int cols, int rows_per,
                                                float* __restrict__ part) {
    const int c = blockIdx.x * 256 + threadIdx.x;
    if (c >= cols) return;
    const int r0 = blockIdx.y * rows_per, r1 = min(n, r0 + rows_per);
    float s = 0.0f;
    for (int b = r0; b < r1; ++b) s += d[(size_t)b * cols + c];
    part[(size_t)blockIdx.y * cols + c] = s;
}

// out[i] = sum_z slices[z][i], z in order (split-K and column-sum partials)
__global__ __launch_bounds__(256) void k_sum_slices(const float* __restrict__ slices, int n_slices, size_t len,
                                                    float* __restrict__ out) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= len) return;
    float s = slices[i];
    for (int z = 1; z < n_slices; ++z) s += slices[(size_t)z * len + i];
    out[i] = s;
}

// per-block partial sums of squares of the flat gradient (grid-stride, fixed order)
__global__ __launch_bounds__(256) void k_sumsq(const float* __restrict__ g, size_t n, float* __restrict__ partial) {
    __shared__ float red[256];
    float s = 0.0f;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
        s = fmaf(g[i], g[i], s);
    red[threadIdx.x] = s;
    __syncthreads();
    for (int k = 128; k > 0; k >>= 1) {
        if ((int)threadIdx.x < k) red[threadIdx.x] += red[threadIdx.x + k];
        __syncthreads();
    }
    if (threadIdx.x == 0) partial[blockIdx.x] = red[0];
}

// scal[0] = loss, scal[1] = gradient L2 norm, scal[2] = clip scale
// (dynet::Trainer::clip_gradients: clip_threshold / ||g|| when ||g|| > clip_threshold)
__global__ void k_finalize(const float* __restrict__ loss_part, int n_loss, const float* __restrict__ g_part,
                           int n_g, float clip, float* __restrict__ scal) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    float l = 0.0f, gg = 0.0f;
    for (int i = 0; i < n_loss; ++i) l += loss_part[i];
    for (int i = 0; i < n_g; ++i) gg += g_part[i];
    gg = sqrtf(gg);
    scal[0] = l;
    scal[1] = gg;
    scal[2] = (clip > 0.0f && gg > clip) ? clip / gg : 1.0f;
}

// dynet::AdamTrainer::update_rule:
//   m = m b1 + g (1 - b1) s;  v = v b2 + g^2 (1 - b2) s^2;  x -= m / (sqrt(v) + eps) lr_t
__global__ __launch_bounds__(256) void k_adam(float* __restrict__ x, const float* __restrict__ g,
                                              float* __restrict__ m, float* __restrict__ v, size_t n,
                                              const float* __restrict__ scal, float b1, float b2, float eps,
                                              float lr_t) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const float s = scal[2];
    const float gi = g[i];
    const float mi = m[i] * b1 + gi * ((1.0f - b1) * s);
    const float vi = v[i] * b2 + (gi * gi) * ((1.0f - b2) * (s * s));
    m[i] = mi;
    v[i] = vi;
    x[i] = x[i] - (mi / (sqrtf(vi) + eps)) * lr_t;
}

// compute_td_targets (nn_rendering_helpers.cu:91-140) for rays in state s' on surface
// tri: max over actions of Q(s', a) * cos_a, where action 0 keeps its raw Q (the
// reference starts the max at next_qs[0] and weights actions 1.. only) and cos_a is the
// cosine of a jittered direction in cell a (sample_ray_for_grid_index), here the Chiu
// map's cos(theta) with the sampler's Philox jitters: pixel, sample,
// event 1 + bounce, counter word 1 + a/2.
__global__ __launch_bounds__(256) void k_td_targets(const float* __restrict__ next_q,
                                                    const int32_t* __restrict__ terminal,
                                                    const float* __restrict__ reward,
                                                    const float* __restrict__ discount,
                                                    const uint32_t* __restrict__ pix, uint32_t sample,
                                                    uint32_t ev, uint32_t k0, uint32_t k1, int n,
                                                    float* __restrict__ target) {
    const int b = blockIdx.x * 256 + threadIdx.x;
    if (b >= n) return;
    if (terminal[b] == 1) {
        target[b] = reward[b];
        return;
    }
    const float* q = next_q + (size_t)b * rt::kDqnActions;
    float best = q[0];
    uint32_t o[4];
    for (int a2 = 0; a2 < rt::kDqnActions; a2 += 2) {
        rt::philox4x32_10(pix[b], sample, ev, 1u + (uint32_t)(a2 >> 1), k0, k1, o);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int a = a2 + h;
            if (a == 0) continue;
            const int gxi = a / rt::kDqnGrid, gyi = a - gxi * rt::kDqnGrid;
            const float c = rt::chiu_cos((float)gxi + rt::u01(o[2 * h]), (float)gyi + rt::u01(o[2 * h + 1]));
            const float t = q[a] * c;
            if (best < t) best = t;
        }
    }
    target[b] = reward[b] + best * discount[b];
}

int err(int code, const std::string& m) { return rt::set_error(code, m.c_str()); }

#define RT_HIPE(expr)                                                                                   \
    do {                                                                                                \
        hipError_t e_ = (expr);                                                                         \
        if (e_ != hipSuccess) return err(RT_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

unsigned blocks_for(size_t n) { return (unsigned)((n + 255) / 256); }

template <int TA, int TB, int EPI>
hipError_t gemm(hipStream_t st, int M, int N, int K, const float* A, int lda, const float* B, int ldb, float* C,
                int ldc, const float* bias = nullptr, const float* mask = nullptr, int ldm = 0, int split = 1) {
    const dim3 grid((unsigned)((N + kT - 1) / kT), (unsigned)((M + kT - 1) / kT), (unsigned)split);
    hipLaunchKernelGGL((k_gemm<TA, TB, EPI>), grid, dim3(256), 0, st, M, N, K, A, lda, B, ldb, C, ldc, bias, mask,
                       ldm);
    return hipGetLastError();
}

}  // namespace

struct rt_dqn_trainer {
    int device = 0;
    int dims[5] = {0, 0, 0, 0, 0};  // n_in, h1, h2, h3, n_out
    size_t w_off[4] = {0, 0, 0, 0}, b_off[4] = {0, 0, 0, 0}, n_par = 0;
    float *P = nullptr, *G = nullptr, *Mo = nullptr, *Vo = nullptr;  // flat [W0 b0 W1 b1 ...]
    float* verts = nullptr;
    float lr = 1e-3f, b1 = 0.9f, b2 = 0.999f, eps = 1e-8f, clip = 5.0f;
    long long updates = 0;
    // workspace (rays): X, H1..H4, dH (two ping-pong gradient buffers), partials, scalars
    int cap = 0;
    float *X = nullptr, *H[4] = {nullptr, nullptr, nullptr, nullptr}, *D[2] = {nullptr, nullptr};
    float *part_loss = nullptr, *part_g = nullptr, *scal = nullptr;
    float* slices = nullptr;  // split-K partial products of the weight gradients
    size_t slice_cap = 0;
    void free_ws() {
        for (float* p : {X, H[0], H[1], H[2], H[3], D[0], D[1], part_loss, slices}) (void)hipFree(p);
        X = D[0] = D[1] = part_loss = slices = nullptr;
        slice_cap = 0;
        for (auto& h : H) h = nullptr;
        cap = 0;
    }
    ~rt_dqn_trainer() {
        (void)hipSetDevice(device);
        free_ws();
        for (float* p : {P, G, Mo, Vo, verts, part_g, scal}) (void)hipFree(p);
    }
};

namespace {

constexpr int kColChunks = 256;  // most row chunks of the bias-gradient column sums

// K slices of a weight-gradient GEMM (M x N tiles over a batch of K rays): enough
// workgroups to fill the 256 CUs, slices of at least 256 rays
int split_for(int M, int N, int K) {
    const int tiles = ((M + kT - 1) / kT) * ((N + kT - 1) / kT);
    int s = (1024 + tiles - 1) / tiles;
    s = std::min(s, std::max(1, K / 256));
    return std::max(1, std::min(s, 64));
}

int ensure_ws(rt_dqn_trainer* t, int n) {
    if (n <= t->cap) return RT_OK;
    t->free_ws();
    const int cap = ((n + 255) / 256) * 256;
    int widest = 0;
    for (int l = 1; l < 5; ++l) widest = std::max(widest, t->dims[l]);
    RT_HIPE(hipMalloc(&t->X, sizeof(float) * (size_t)cap * t->dims[0]));
    for (int l = 0; l < 4; ++l) RT_HIPE(hipMalloc(&t->H[l], sizeof(float) * (size_t)cap * t->dims[l + 1]));
    for (int k = 0; k < 2; ++k) RT_HIPE(hipMalloc(&t->D[k], sizeof(float) * (size_t)cap * widest));
    RT_HIPE(hipMalloc(&t->part_loss, sizeof(float) * (size_t)(cap / 256)));
    size_t sl = 0;
    for (int l = 0; l < 4; ++l) {
        const int s = split_for(t->dims[l + 1], t->dims[l], cap);
        sl = std::max(sl, (size_t)s * t->dims[l + 1] * t->dims[l]);
        sl = std::max(sl, (size_t)kColChunks * t->dims[l + 1]);
    }
    RT_HIPE(hipMalloc(&t->slices, sizeof(float) * sl));
    t->slice_cap = sl;
    t->cap = cap;
    return RT_OK;
}

}  // namespace

extern "C" {

int rt_dqn_trainer_create(rt_ctx* ctx, const float* nn_vertices, int n_in, const int32_t* hidden, int n_out,
                          const float* const* W, const float* const* b, float learning_rate,
                          rt_dqn_trainer** out) {
    if (!ctx || !nn_vertices || !hidden || !W || !b || !out) return err(RT_E_INVALID, "NULL argument");
    *out = nullptr;
    if (n_in <= 0 || n_in % 3 != 0) return err(RT_E_INVALID, "n_in must be a positive multiple of 3");
    if (n_out <= 0 || hidden[0] <= 0 || hidden[1] <= 0 || hidden[2] <= 0)
        return err(RT_E_INVALID, "layer widths must be positive");
    if (!(learning_rate > 0.0f) || !std::isfinite(learning_rate)) return err(RT_E_INVALID, "bad learning rate");
    for (int l = 0; l < 4; ++l)
        if (!W[l] || !b[l]) return err(RT_E_INVALID, "NULL layer parameters");
    RT_HIPE(hipSetDevice(rt::ctx_device(ctx)));
    rt_dqn_trainer* t = new (std::nothrow) rt_dqn_trainer();
    if (!t) return err(RT_E_NOMEM, "out of host memory");
    t->device = rt::ctx_device(ctx);
    t->lr = learning_rate;
    const int d[5] = {n_in, hidden[0], hidden[1], hidden[2], n_out};
    memcpy(t->dims, d, sizeof(d));
    size_t off = 0;
    for (int l = 0; l < 4; ++l) {
        t->w_off[l] = off;
        off += (size_t)d[l + 1] * d[l];
        t->b_off[l] = off;
        off += (size_t)d[l + 1];
    }
    t->n_par = off;
    std::vector<float> flat(off);
    for (int l = 0; l < 4; ++l) {
        memcpy(flat.data() + t->w_off[l], W[l], sizeof(float) * (size_t)d[l + 1] * d[l]);
        memcpy(flat.data() + t->b_off[l], b[l], sizeof(float) * (size_t)d[l + 1]);
    }
    auto fail = [&](hipError_t e) {
        delete t;
        return err(RT_E_HIP, std::string("trainer alloc: ") + hipGetErrorString(e));
    };
    hipError_t e = hipSuccess;
    for (float** p : {&t->P, &t->G, &t->Mo, &t->Vo})
        if (e == hipSuccess) e = hipMalloc(p, sizeof(float) * off);
    if (e == hipSuccess) e = hipMalloc(&t->verts, sizeof(float) * (size_t)n_in);
    if (e == hipSuccess) e = hipMalloc(&t->part_g, sizeof(float) * kRedBlocks);
    if (e == hipSuccess) e = hipMalloc(&t->scal, sizeof(float) * 4);
    if (e == hipSuccess) e = hipMemcpy(t->P, flat.data(), sizeof(float) * off, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(t->verts, nn_vertices, sizeof(float) * (size_t)n_in, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemset(t->Mo, 0, sizeof(float) * off);
    if (e == hipSuccess) e = hipMemset(t->Vo, 0, sizeof(float) * off);
    if (e != hipSuccess) return fail(e);
    *out = t;
    return RT_OK;
}

int rt_dqn_trainer_destroy(rt_dqn_trainer* t) {
    delete t;
    return RT_OK;
}

int rt_dqn_trainer_params(const rt_dqn_trainer* t, float* const* W, float* const* b) {
    if (!t || !W || !b) return err(RT_E_INVALID, "NULL argument");
    RT_HIPE(hipSetDevice(t->device));
    std::vector<float> flat(t->n_par);
    RT_HIPE(hipMemcpy(flat.data(), t->P, sizeof(float) * t->n_par, hipMemcpyDeviceToHost));
    for (int l = 0; l < 4; ++l) {
        if (!W[l] || !b[l]) return err(RT_E_INVALID, "NULL layer buffer");
        memcpy(W[l], flat.data() + t->w_off[l], sizeof(float) * (size_t)t->dims[l + 1] * t->dims[l]);
        memcpy(b[l], flat.data() + t->b_off[l], sizeof(float) * (size_t)t->dims[l + 1]);
    }
    return RT_OK;
}

int rt_dqn_train_step_device(rt_ctx* ctx, rt_dqn_trainer* t, const float* d_loc, const int32_t* d_action,
                             const float* d_target, int n, float* loss_out, float* grad_norm_out, void* stream) {
    if (!ctx || !t || !d_loc || !d_action || !d_target) return err(RT_E_INVALID, "NULL argument");
    if (n <= 0) return err(RT_E_INVALID, "empty batch");
    RT_HIPE(hipSetDevice(t->device));
    int rc = ensure_ws(t, n);
    if (rc != RT_OK) return rc;
    hipStream_t st = (hipStream_t)stream;
    const int* d = t->dims;
    // forward, activations kept: H[l] = ReLU(H[l-1] W_l^T + b_l), H[-1] = X
    hipLaunchKernelGGL(k_build_x, dim3(blocks_for((size_t)n * d[0])), dim3(256), 0, st, t->verts, d[0], d_loc, n,
                       t->X);
    RT_HIPE(hipGetLastError());
    const float* in = t->X;
    for (int l = 0; l < 4; ++l) {
        RT_HIPE((gemm<0, 1, 1>(st, n, d[l + 1], d[l], in, d[l], t->P + t->w_off[l], d[l], t->H[l], d[l + 1],
                               t->P + t->b_off[l])));
        in = t->H[l];
    }
    // loss and the output-layer gradient
    RT_HIPE(hipMemsetAsync(t->D[0], 0, sizeof(float) * (size_t)n * d[4], st));
    const unsigned nb = blocks_for((size_t)n);
    hipLaunchKernelGGL(k_loss_grad, dim3(nb), dim3(256), 0, st, t->H[3], d[4], d_action, d_target, n, t->D[0],
                       t->part_loss);
    RT_HIPE(hipGetLastError());
    // backward: dW_l = dH_l^T H_{l-1}, db_l = column sums, dH_{l-1} = (dH_l W_l) * [H_{l-1} > 0]
    int cur = 0;
    for (int l = 3; l >= 0; --l) {
        const float* prev = (l == 0) ? t->X : t->H[l - 1];
        const int sk = split_for(d[l + 1], d[l], n);
        const size_t wlen = (size_t)d[l + 1] * d[l];
        if (sk == 1) {
            RT_HIPE((gemm<1, 0, 0>(st, d[l + 1], d[l], n, t->D[cur], d[l + 1], prev, d[l], t->G + t->w_off[l], d[l])));
        } else {
            RT_HIPE((gemm<1, 0, 0>(st, d[l + 1], d[l], n, t->D[cur], d[l + 1], prev, d[l], t->slices, d[l], nullptr,
                                   nullptr, 0, sk)));
            hipLaunchKernelGGL(k_sum_slices, dim3(blocks_for(wlen)), dim3(256), 0, st, t->slices, sk, wlen,
                               t->G + t->w_off[l]);
            RT_HIPE(hipGetLastError());
        }
        // chunks of >= 64 rows, at most kColChunks of them (measured: 4096 rays -> 64 chunks,
        // 65536 rays -> 256 chunks balance the two stages)
        const int rows_per = std::max(64, (n + kColChunks - 1) / kColChunks);
        const int chunks = (n + rows_per - 1) / rows_per;
        hipLaunchKernelGGL(k_colsum, dim3(blocks_for((size_t)d[l + 1]), (unsigned)chunks), dim3(256), 0, st,
                           t->D[cur], n, d[l + 1], rows_per, t->slices);
        RT_HIPE(hipGetLastError());
        hipLaunchKernelGGL(k_sum_slices, dim3(blocks_for((size_t)d[l + 1])), dim3(256), 0, st, t->slices,
                           chunks, (size_t)d[l + 1], t->G + t->b_off[l]);
        RT_HIPE(hipGetLastError());
        if (l > 0) {
            RT_HIPE((gemm<0, 0, 2>(st, n, d[l], d[l + 1], t->D[cur], d[l + 1], t->P + t->w_off[l], d[l],
                                   t->D[cur ^ 1], d[l], nullptr, t->H[l - 1], d[l])));
            cur ^= 1;
        }
    }
    // clipping scale and Adam
    hipLaunchKernelGGL(k_sumsq, dim3(kRedBlocks), dim3(256), 0, st, t->G, t->n_par, t->part_g);
    RT_HIPE(hipGetLastError());
    hipLaunchKernelGGL(k_finalize, dim3(1), dim3(64), 0, st, t->part_loss, (int)nb, t->part_g, kRedBlocks, t->clip,
                       t->scal);
    RT_HIPE(hipGetLastError());
    const double u = (double)(t->updates + 1);
    const float lr_t = (float)((double)t->lr * sqrt(1.0 - pow((double)t->b2, u)) / (1.0 - pow((double)t->b1, u)));
    hipLaunchKernelGGL(k_adam, dim3(blocks_for(t->n_par)), dim3(256), 0, st, t->P, t->G, t->Mo, t->Vo, t->n_par,
                       t->scal, t->b1, t->b2, t->eps, lr_t);
    RT_HIPE(hipGetLastError());
    t->updates++;
    if (loss_out || grad_norm_out) {
        float h[4];
        RT_HIPE(hipMemcpyAsync(h, t->scal, sizeof(h), hipMemcpyDeviceToHost, st));
        RT_HIPE(hipStreamSynchronize(st));
        if (loss_out) *loss_out = h[0];
        if (grad_norm_out) *grad_norm_out = h[1];
    }
    return RT_OK;
}

int rt_dqn_td_targets_device(rt_ctx* ctx, uint64_t seed, const float* d_next_q, const int32_t* d_terminal,
                             const float* d_reward, const float* d_discount, const uint32_t* d_pix, int sample,
                             int bounce, int n, float* d_target, void* stream) {
    if (!ctx || !d_next_q || !d_terminal || !d_reward || !d_discount || !d_pix || !d_target)
        return err(RT_E_INVALID, "NULL argument");
    if (n < 0 || sample < 0 || bounce < 0) return err(RT_E_INVALID, "negative count");
    if (n == 0) return RT_OK;
    RT_HIPE(hipSetDevice(rt::ctx_device(ctx)));
    hipLaunchKernelGGL(k_td_targets, dim3(blocks_for((size_t)n)), dim3(256), 0, (hipStream_t)stream, d_next_q,
                       d_terminal, d_reward, d_discount, d_pix, (uint32_t)sample, 1u + (uint32_t)bounce,
                       (uint32_t)seed, (uint32_t)(seed >> 32), n, d_target);
    RT_HIPE(hipGetLastError());
    return RT_OK;
}

}  // extern "C"
