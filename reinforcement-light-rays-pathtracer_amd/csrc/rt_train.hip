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
// Layer 0 is folded, as in the inference network: its input vertices - p makes it an
// affine map of the ray position, so the n x n_in input matrix is never built and the
// layer's forward is c0 - S p (k_fold0 / k_layer0_fwd, in double), its weight gradient
// g v^T - T spread over the coordinates (k_colsum4 / k_grad0, sums in double): the two largest
// GEMMs of the step (K or N = n_in = 918) disappear; the arithmetic is the same map.
// MI355X mapping: fp32 throughout (the reference trains in fp32): every product is an
// LDS-tiled fp32 GEMM on the f32 MFMA (v_mfma_f32_16x16x4_f32, 64x64 tile per 256-thread
// workgroup, k-ordered fmaf chains, so results do not depend on the launch) with the bias + ReLU or the
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
DeviceScene scene_launch_view(const rt_scene* s);
void scene_host(const rt_scene* s, const float** tri, const float** normals, const float** albedo,
                const float** emission, int* n_surf, int* n_light);
}  // namespace rt

namespace {

using rt::f3;

constexpr int kT = 64;   // GEMM output tile (rows and columns)
constexpr int kTK = 16;  // GEMM k step
constexpr int kRedBlocks = 256;

typedef __attribute__((ext_vector_type(4))) float f32x4;
constexpr int kPadS = 16;  // LDS row padding: lanes l and l + 16 of a ds_read_b32 half hit other banks

// C[M][N] = op(A)[M][K] * op(B)[K][N], row-major storage:
//   TA = 0: A[m * lda + k]   TA = 1: A[k * lda + m]
//   TB = 0: B[k * ldb + n]   TB = 1: B[n * ldb + k]
// EPI 0: C = acc;  1: C = max(acc + bias[n], 0) (fc_layer + rectify);
//     2: C = mask[m * ldm + n] > 0 ? acc : 0  (rectify's derivative, y > 0)
// On v_mfma_f32_16x16x4_f32 (exact f32 in and out: each instruction is the k-ordered fmaf
// chain of its 4 products, MI355X_MICROARCH.md § Matrix cores): a 64x64 tile per
// workgroup, wave w owns rows 32(w/2) .. +31 and columns 32(w%2) .. +31 as 2x2 tiles of
// 16x16, four independent accumulators per wave (the instruction's 40-cycle dependent
// latency against its 32-cycle issue).  Every output is fmaf(a_K-1, b_K-1, .. fmaf(a_0,
// b_0, 0)) in k order, as the VALU kernel it replaces computed it: the same bits.
template <int TA, int TB, int EPI>
__global__ __launch_bounds__(256) void k_gemm(int M, int N, int K, const float* __restrict__ A, int lda,
                                              const float* __restrict__ B, int ldb, float* __restrict__ C,
                                              int ldc, const float* __restrict__ bias,
                                              const float* __restrict__ mask, int ldm) {
    __shared__ float As[kTK][kT + kPadS];
    __shared__ float Bs[kTK][kT + kPadS];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int wr = (wave >> 1) * 32, wc = (wave & 1) * 32;  // the wave's 32x32 quarter
    const int r16 = lane & 15, kq = lane >> 4;
    const int m0 = blockIdx.y * kT, n0 = blockIdx.x * kT;
    // split K (gridDim.z > 1, EPI 0 only): slice z covers [z kc, (z + 1) kc) and writes the
    // partial product to C + z M ldc; k_sum_slices adds the slices in order
    const int kc = (K + (int)gridDim.z - 1) / (int)gridDim.z;
    const int kb = (int)blockIdx.z * kc, ke = min(K, kb + kc);
    C += (size_t)blockIdx.z * M * ldc;
    f32x4 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
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
        // zero-padded past ke: the padded products are fmaf(0, b, acc) steps, as in the
        // VALU kernel this replaces (same chain, same bits)
#pragma unroll
        for (int s4 = 0; s4 < kTK; s4 += 4) {
            float a[2], b[2];
#pragma unroll
            for (int i = 0; i < 2; ++i) a[i] = As[s4 + kq][wr + 16 * i + r16];  // A[m = lane & 15][k = lane >> 4]
#pragma unroll
            for (int j = 0; j < 2; ++j) b[j] = Bs[s4 + kq][wc + 16 * j + r16];  // B[k = lane >> 4][n = lane & 15]
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i], b[j], acc[i][j], 0, 0, 0);
        }
        __syncthreads();
    }
    // lane holds rows 4 (lane >> 4) + r of column lane & 15 of each 16x16 tile
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int gn = n0 + wc + 16 * j + r16;
            if (gn >= N) continue;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int gm = m0 + wr + 16 * i + 4 * kq + r;
                if (gm >= M) continue;
                float v = acc[i][j][r];
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

// Layer 0 folded (as the inference network folds it, rt_internal.hpp DqnNet): its input
// x = Scene::vertices - p (nn_rendering_helpers.cu:280-298) makes W0 x + b0 an affine map
// of the ray position p: c0 - S p with c0 = W0 v + b0 and S[o][c] = sum_v W0[o][3v + c].
// One wave per output o, products and sums in double, combined in a fixed order.
__global__ __launch_bounds__(64) void k_fold0(const float* __restrict__ W0, const float* __restrict__ b0,
                                              const float* __restrict__ verts, int n_in,
                                              double4* __restrict__ fold) {
    const int o = blockIdx.x, lane = threadIdx.x;
    double c = 0.0, s0 = 0.0, s1 = 0.0, s2 = 0.0;
    const float* w = W0 + (size_t)o * n_in;
    for (int v = lane; v < n_in / 3; v += 64) {
        const double w0 = w[3 * v], w1 = w[3 * v + 1], w2 = w[3 * v + 2];
        c += (w0 * verts[3 * v] + w1 * verts[3 * v + 1]) + w2 * verts[3 * v + 2];
        s0 += w0;
        s1 += w1;
        s2 += w2;
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        c += __shfl_xor(c, off, 64);
        s0 += __shfl_xor(s0, off, 64);
        s1 += __shfl_xor(s1, off, 64);
        s2 += __shfl_xor(s2, off, 64);
    }
    if (lane == 0) fold[o] = make_double4(s0, s1, s2, c + (double)b0[o]);
}

// H0[b][o] = ReLU(c0 - S p) in double, rounded once: c0 and S p are each of the size of
// the whole sum while their difference may be much smaller, so single precision here
// would lose the digits the explicit fp32 contraction keeps
__global__ __launch_bounds__(256) void k_layer0_fwd(const double4* __restrict__ fold, int n_out,
                                                    const float* __restrict__ loc, int n, float* __restrict__ H) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= (size_t)n * n_out) return;
    const int b = (int)(i / n_out), o = (int)(i - (size_t)b * n_out);
    const double4 f = fold[o];
    const double x = loc[(size_t)b * 3], y = loc[(size_t)b * 3 + 1], z = loc[(size_t)b * 3 + 2];
    const float h = (float)(f.w - ((f.x * x + f.y * y) + f.z * z));
    H[i] = h > 0.0f ? h : 0.0f;
}

// Layer 0's gradients from the output gradient d (n x n_out): db0[o] = g[o] = sum_b d[b][o]
// and dW0[o][j] = sum_b d[b][o] (v_j - p_b[j % 3]) = g[o] v_j - T[o][j % 3], T[o][c] =
// sum_b d[b][o] p_b[c].  Stage 1: per chunk of rows, per column, the four sums in double
// (4 row groups of the block, combined in a fixed order) -> part[chunk][o].
__global__ __launch_bounds__(256) void k_colsum4(const float* __restrict__ d, int n, int cols, int rows_per,
                                                 const float* __restrict__ loc, double4* __restrict__ part) {
    __shared__ double4 red[4][64];
    const int c = blockIdx.x * 64 + (threadIdx.x & 63), rg = threadIdx.x >> 6;
    const int r0 = blockIdx.y * rows_per, r1 = min(n, r0 + rows_per);
    double s = 0.0, sx = 0.0, sy = 0.0, sz = 0.0;
    if (c < cols)
        for (int b = r0 + rg; b < r1; b += 4) {
            const double v = d[(size_t)b * cols + c];
            s += v;
            sx += v * (double)loc[(size_t)b * 3];
            sy += v * (double)loc[(size_t)b * 3 + 1];
            sz += v * (double)loc[(size_t)b * 3 + 2];
        }
    red[rg][threadIdx.x & 63] = make_double4(s, sx, sy, sz);
    __syncthreads();
    if (rg == 0 && c < cols) {
        double4 t = red[0][threadIdx.x];
        for (int k = 1; k < 4; ++k) {
            const double4 u = red[k][threadIdx.x];
            t.x += u.x;
            t.y += u.y;
            t.z += u.z;
            t.w += u.w;
        }
        part[(size_t)blockIdx.y * cols + c] = t;
    }
}

// Stage 2: the chunks in order (one thread per output) -> part[0][o]
__global__ __launch_bounds__(256) void k_sum4(double4* __restrict__ part, int chunks, int cols) {
    const int o = blockIdx.x * 256 + threadIdx.x;
    if (o >= cols) return;
    double4 t = part[o];
    for (int k = 1; k < chunks; ++k) {
        const double4 u = part[(size_t)k * cols + o];
        t.x += u.x;
        t.y += u.y;
        t.z += u.z;
        t.w += u.w;
    }
    part[o] = t;
}

// Stage 3: db0 and dW0 (one thread per weight)
__global__ __launch_bounds__(256) void k_grad0(const double4* __restrict__ tot, int cols, int n_in,
                                               const float* __restrict__ verts, float* __restrict__ dW,
                                               float* __restrict__ db) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= (size_t)cols * n_in) return;
    const int o = (int)(i / n_in), j = (int)(i - (size_t)o * n_in);
    const double4 t = tot[o];
    const double T = (j % 3 == 0) ? t.y : ((j % 3 == 1) ? t.z : t.w);
    dW[i] = (float)(t.x * (double)verts[j] - T);
    if (j == 0) db[o] = (float)t.x;
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
// rows per column -> part[y][c], its 4 row groups (rows = rg mod 4) combined in a fixed
// order; stage 2 (k_sum_slices): the chunks in order.
__global__ __launch_bounds__(256) void k_colsum(const float* __restrict__ d, int n, int cols, int rows_per,
                                                float* __restrict__ part) {
    __shared__ float red[4][64];
    const int c = blockIdx.x * 64 + (threadIdx.x & 63), rg = threadIdx.x >> 6;
    const int r0 = blockIdx.y * rows_per, r1 = min(n, r0 + rows_per);
    float s = 0.0f;
    if (c < cols)
        for (int b = r0 + rg; b < r1; b += 4) s += d[(size_t)b * cols + c];
    red[rg][threadIdx.x & 63] = s;
    __syncthreads();
    if (rg == 0 && c < cols)
        part[(size_t)blockIdx.y * cols + c] = ((red[0][threadIdx.x] + red[1][threadIdx.x]) + red[2][threadIdx.x]) +
                                              red[3][threadIdx.x];
}

// out[i] = sum_z slices[z][i], z in order (split-K and column-sum partials); 4 outputs
// per thread (16-B loads) and 8 slices' loads in flight before their in-order adds
__global__ __launch_bounds__(256) void k_sum_slices(const float* __restrict__ slices, int n_slices, size_t len,
                                                    float* __restrict__ out) {
    const size_t i = ((size_t)blockIdx.x * 256 + threadIdx.x) * 4;
    if (i >= len) return;
    if (i + 4 <= len && (len & 3) == 0) {
        float4 s = *reinterpret_cast<const float4*>(slices + i);
        int z = 1;
        for (; z + 8 <= n_slices; z += 8) {
            float4 v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = *reinterpret_cast<const float4*>(slices + (size_t)(z + u) * len + i);
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                s.x += v[u].x;
                s.y += v[u].y;
                s.z += v[u].z;
                s.w += v[u].w;
            }
        }
        for (; z < n_slices; ++z) {
            const float4 v = *reinterpret_cast<const float4*>(slices + (size_t)z * len + i);
            s.x += v.x;
            s.y += v.y;
            s.z += v.z;
            s.w += v.w;
        }
        *reinterpret_cast<float4*>(out + i) = s;
        return;
    }
    for (size_t k = i; k < len && k < i + 4; ++k) {
        float s = slices[k];
        for (int z = 1; z < n_slices; ++z) s += slices[(size_t)z * len + k];
        out[k] = s;
    }
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
// (dynet::Trainer::clip_gradients: clip_threshold / ||g|| when ||g|| > clip_threshold).
// One wave: lane l sums partials l, l + 64, .. in order, then a fixed xor-shuffle tree.
__global__ __launch_bounds__(64) void k_finalize(const float* __restrict__ loss_part, int n_loss,
                                                 const float* __restrict__ g_part, int n_g, float clip,
                                                 float* __restrict__ scal) {
    const int lane = threadIdx.x;
    float l = 0.0f, gg = 0.0f;
    for (int i = lane; i < n_loss; i += 64) l += loss_part[i];
    for (int i = lane; i < n_g; i += 64) gg += g_part[i];
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        l += __shfl_xor(l, off, 64);
        gg += __shfl_xor(gg, off, 64);
    }
    if (lane != 0) return;
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
    const rt::PhiloxShared ph = rt::philox_shared(pix[b], sample, ev, k0, k1);  // 72 draws, one (pixel, sample, event)
    for (int a2 = 0; a2 < rt::kDqnActions; a2 += 2) {
        rt::philox_from(ph, 1u + (uint32_t)(a2 >> 1), o);
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

// the learning rule's loss summed over a sample's batches (neural_q_pathtracer.cu:509)
__global__ void k_acc_loss(const float* __restrict__ scal, double* __restrict__ acc) {
    if (threadIdx.x == 0 && blockIdx.x == 0) acc[0] += (double)scal[0];
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
    float *H[4] = {nullptr, nullptr, nullptr, nullptr}, *D[2] = {nullptr, nullptr};
    double4* fold = nullptr;   // layer 0 folded: {S0, S1, S2, c0} per output (k_fold0)
    double4* part4 = nullptr;  // layer-0 gradient chunk sums (k_colsum4)
    float *part_loss = nullptr, *part_g = nullptr, *scal = nullptr;
    float* slices = nullptr;  // split-K partial products of the weight gradients
    size_t slice_cap = 0;
    void free_ws() {
        for (float* p : {H[0], H[1], H[2], H[3], D[0], D[1], part_loss, slices}) (void)hipFree(p);
        (void)hipFree(part4);
        D[0] = D[1] = part_loss = slices = nullptr;
        part4 = nullptr;
        slice_cap = 0;
        for (auto& h : H) h = nullptr;
        cap = 0;
    }
    ~rt_dqn_trainer() {
        (void)hipSetDevice(device);
        free_ws();
        for (float* p : {P, G, Mo, Vo, verts, part_g, scal}) (void)hipFree(p);
        (void)hipFree(fold);
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
    RT_HIPE(hipMalloc(&t->part4, sizeof(double4) * (size_t)kColChunks * t->dims[1]));
    for (int l = 0; l < 4; ++l) RT_HIPE(hipMalloc(&t->H[l], sizeof(float) * (size_t)cap * t->dims[l + 1]));
    for (int k = 0; k < 2; ++k) RT_HIPE(hipMalloc(&t->D[k], sizeof(float) * (size_t)cap * widest));
    RT_HIPE(hipMalloc(&t->part_loss, sizeof(float) * (size_t)(cap / 256)));
    size_t sl = 0;
    for (int l = 1; l < 4; ++l) {
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
    if (e == hipSuccess) e = hipMalloc(&t->fold, sizeof(double4) * (size_t)hidden[0]);
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

}  // extern "C"

namespace {

// forward with the activations kept (H[0..3]; Q = H[3], n x n_out row-major)
int trainer_forward(rt_dqn_trainer* t, const float* d_loc, int n, hipStream_t st) {
    const int* d = t->dims;
    // forward, activations kept: H[l] = ReLU(H[l-1] W_l^T + b_l); layer 0 folded (its input
    // vertices - p is never built: k_fold0 / k_layer0_fwd)
    hipLaunchKernelGGL(k_fold0, dim3((unsigned)d[1]), dim3(64), 0, st, t->P + t->w_off[0], t->P + t->b_off[0],
                       t->verts, d[0], t->fold);
    RT_HIPE(hipGetLastError());
    hipLaunchKernelGGL(k_layer0_fwd, dim3(blocks_for((size_t)n * d[1])), dim3(256), 0, st, t->fold, d[1], d_loc, n,
                       t->H[0]);
    RT_HIPE(hipGetLastError());
    const float* in = t->H[0];
    for (int l = 1; l < 4; ++l) {
        RT_HIPE((gemm<0, 1, 1>(st, n, d[l + 1], d[l], in, d[l], t->P + t->w_off[l], d[l], t->H[l], d[l + 1],
                               t->P + t->b_off[l])));
        in = t->H[l];
    }
    return RT_OK;
}

// steps 5-7 of the learning rule on n rays (forward, loss, backward, clipping, Adam)
int trainer_step(rt_dqn_trainer* t, const float* d_loc, const int32_t* d_action, const float* d_target, int n,
                 hipStream_t st) {
    int rc = trainer_forward(t, d_loc, n, st);
    if (rc != RT_OK) return rc;
    const int* d = t->dims;
    // loss and the output-layer gradient
    RT_HIPE(hipMemsetAsync(t->D[0], 0, sizeof(float) * (size_t)n * d[4], st));
    const unsigned nb = blocks_for((size_t)n);
    hipLaunchKernelGGL(k_loss_grad, dim3(nb), dim3(256), 0, st, t->H[3], d[4], d_action, d_target, n, t->D[0],
                       t->part_loss);
    RT_HIPE(hipGetLastError());
    // backward: dW_l = dH_l^T H_{l-1}, db_l = column sums, dH_{l-1} = (dH_l W_l) * [H_{l-1} > 0]
    int cur = 0;
    // chunks of >= 64 rows, at most kColChunks of them (measured: 4096 rays -> 64 chunks,
    // 65536 rays -> 256 chunks balance the two stages)
    const int rows_per = std::max(64, (n + kColChunks - 1) / kColChunks);
    const int chunks = (n + rows_per - 1) / rows_per;
    for (int l = 3; l >= 1; --l) {
        const float* prev = t->H[l - 1];
        const int sk = split_for(d[l + 1], d[l], n);
        const size_t wlen = (size_t)d[l + 1] * d[l];
        if (sk == 1) {
            RT_HIPE((gemm<1, 0, 0>(st, d[l + 1], d[l], n, t->D[cur], d[l + 1], prev, d[l], t->G + t->w_off[l], d[l])));
        } else {
            RT_HIPE((gemm<1, 0, 0>(st, d[l + 1], d[l], n, t->D[cur], d[l + 1], prev, d[l], t->slices, d[l], nullptr,
                                   nullptr, 0, sk)));
            hipLaunchKernelGGL(k_sum_slices, dim3(blocks_for((wlen + 3) / 4)), dim3(256), 0, st, t->slices, sk, wlen,
                               t->G + t->w_off[l]);
            RT_HIPE(hipGetLastError());
        }
        hipLaunchKernelGGL(k_colsum, dim3((unsigned)((d[l + 1] + 63) / 64), (unsigned)chunks), dim3(256), 0, st,
                           t->D[cur], n, d[l + 1], rows_per, t->slices);
        RT_HIPE(hipGetLastError());
        hipLaunchKernelGGL(k_sum_slices, dim3(blocks_for(((size_t)d[l + 1] + 3) / 4)), dim3(256), 0, st, t->slices,
                           chunks, (size_t)d[l + 1], t->G + t->b_off[l]);
        RT_HIPE(hipGetLastError());
        RT_HIPE((gemm<0, 0, 2>(st, n, d[l], d[l + 1], t->D[cur], d[l + 1], t->P + t->w_off[l], d[l],
                               t->D[cur ^ 1], d[l], nullptr, t->H[l - 1], d[l])));
        cur ^= 1;
    }
    // layer 0 (folded): db0 and dW0 from the chunk sums of d, d p_x, d p_y, d p_z
    hipLaunchKernelGGL(k_colsum4, dim3((unsigned)((d[1] + 63) / 64), (unsigned)chunks), dim3(256), 0, st,
                       t->D[cur], n, d[1], rows_per, d_loc, t->part4);
    RT_HIPE(hipGetLastError());
    hipLaunchKernelGGL(k_sum4, dim3(blocks_for((size_t)d[1])), dim3(256), 0, st, t->part4, chunks, d[1]);
    RT_HIPE(hipGetLastError());
    hipLaunchKernelGGL(k_grad0, dim3(blocks_for((size_t)d[1] * d[0])), dim3(256), 0, st, t->part4, d[1], d[0],
                       t->verts, t->G + t->w_off[0], t->G + t->b_off[0]);
    RT_HIPE(hipGetLastError());
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
    return RT_OK;
}

}  // namespace

extern "C" {

int rt_dqn_train_step_device(rt_ctx* ctx, rt_dqn_trainer* t, const float* d_loc, const int32_t* d_action,
                             const float* d_target, int n, float* loss_out, float* grad_norm_out, void* stream) {
    if (!ctx || !t || !d_loc || !d_action || !d_target) return err(RT_E_INVALID, "NULL argument");
    if (n <= 0) return err(RT_E_INVALID, "empty batch");
    RT_HIPE(hipSetDevice(t->device));
    int rc = ensure_ws(t, n);
    if (rc != RT_OK) return rc;
    hipStream_t st = (hipStream_t)stream;
    rc = trainer_step(t, d_loc, d_action, d_target, n, st);
    if (rc != RT_OK) return rc;
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

// ---------------------------------------------------------------------------
// Neural-Q training renderer: NeuralQPathtracer::render_frame
// (GPU/deep_learning/neural_q_pathtracer.cu:226-600) on device buffers.  Per sample:
// initialise_ray; per bounce: (b > 0) Q of every ray's position -> epsilon-greedy
// directions; trace_ray; (b > 0) per batch of ray_batch_size rays the learning rule
// (next Q at the new positions -> compute_td_targets -> trainer.update on the old
// positions and the sampled actions); restarts of terminated rays; until no path is
// still bouncing or MAX_RAY_BOUNCES.  Then epsilon decays and the sample's statistics
// (nn_training_stats.txt: average path length, loss, zero-contribution paths) are kept.
// ---------------------------------------------------------------------------
struct rt_neuralq {
    int device = 0;
    rt_dqn_trainer* tr = nullptr;
    const rt_scene* scene = nullptr;
    int batch = 4096;
    float eps = 0.05f, eps_min = 0.05f, eps_decay = 0.01f;
    uint32_t frames = 0;
    int cap = 0;
    rt::NqRays r;
    float* targets = nullptr;
    double* loss_acc = nullptr;
    float* img = nullptr;
    int32_t* h_flag = nullptr;  // pinned
    std::vector<void*> allocs;   // per-size buffers
    std::vector<void*> fixed;    // scene buffers
    void free_rays() {
        for (void* p : allocs) (void)hipFree(p);
        allocs.clear();
        cap = 0;
    }
    ~rt_neuralq() {
        (void)hipSetDevice(device);
        free_rays();
        for (void* p : fixed) (void)hipFree(p);
        if (h_flag) (void)hipHostFree(h_flag);
    }
};

namespace {

int nq_ensure(rt_neuralq* q, int n) {
    if (n <= q->cap) return RT_OK;
    q->free_rays();
    auto al = [&](void** p, size_t bytes) -> hipError_t {
        hipError_t e = hipMalloc(p, bytes);
        if (e == hipSuccess) q->allocs.push_back(*p);
        return e;
    };
    rt::NqRays& r = q->r;
    const size_t f3b = sizeof(float) * 3 * (size_t)n, wb = sizeof(int32_t) * (size_t)n;
    hipError_t e = hipSuccess;
    for (float** f : {&r.loc, &r.prev, &r.dir, &r.tp, &r.total, &q->img})
        if (e == hipSuccess) e = al((void**)f, f3b);
    for (float** f : {&r.reward, &r.discount, &q->targets})
        if (e == hipSuccess) e = al((void**)f, sizeof(float) * (size_t)n);
    for (int32_t** w : {&r.tri, &r.action, &r.terminal})
        if (e == hipSuccess) e = al((void**)w, wb);
    for (uint32_t** w : {&r.state, &r.bounces, &r.pix})
        if (e == hipSuccess) e = al((void**)w, wb);
    if (e != hipSuccess) {
        q->free_rays();
        return err(RT_E_HIP, std::string("neural-q buffers: ") + hipGetErrorString(e));
    }
    q->cap = n;
    return RT_OK;
}

}  // namespace

extern "C" {

int rt_neuralq_create(rt_ctx* ctx, const rt_scene* scene, rt_dqn_trainer* trainer, int batch_size,
                      float epsilon_start, float epsilon_min, float epsilon_decay, rt_neuralq** out) {
    if (!ctx || !scene || !trainer || !out) return err(RT_E_INVALID, "NULL argument");
    *out = nullptr;
    if (batch_size <= 0) return err(RT_E_INVALID, "batch_size must be positive");
    if (!(epsilon_start >= 0.0f && epsilon_start <= 1.0f) || !(epsilon_min >= 0.0f && epsilon_min <= 1.0f) ||
        !(epsilon_decay >= 0.0f))
        return err(RT_E_INVALID, "epsilon values must lie in [0, 1] (decay >= 0)");
    if (trainer->dims[4] != rt::kDqnActions) return err(RT_E_UNSUPPORTED, "the network must have 144 outputs");
    if (trainer->device != rt::ctx_device(ctx)) return err(RT_E_INVALID, "trainer belongs to another device");
    const float *tri, *normals, *albedo, *emission;
    int n_surf, n_light;
    rt::scene_host(scene, &tri, &normals, &albedo, &emission, &n_surf, &n_light);
    if (n_surf <= 0) return err(RT_E_INVALID, "scene has no surfaces");
    RT_HIPE(hipSetDevice(rt::ctx_device(ctx)));
    rt_neuralq* q = new (std::nothrow) rt_neuralq();
    if (!q) return err(RT_E_NOMEM, "out of host memory");
    q->device = rt::ctx_device(ctx);
    q->tr = trainer;
    q->scene = scene;
    q->batch = batch_size;
    q->eps = epsilon_start;
    q->eps_min = epsilon_min;
    q->eps_decay = epsilon_decay;
    // surface vertices (restarts) and luminance per triangle (rewards, discounts)
    std::vector<float> lum((size_t)(n_surf + n_light));
    auto lum3 = [](const float* c) {
        const float mx = std::max(std::max(c[0], c[1]), c[2]), mn = std::min(std::min(c[0], c[1]), c[2]);
        return 0.5f * (mx + mn);
    };
    for (int j = 0; j < n_surf; ++j) lum[j] = lum3(albedo + 3 * j);
    for (int j = 0; j < n_light; ++j) lum[n_surf + j] = lum3(emission + 3 * j);
    float *d_v = nullptr, *d_lum = nullptr;
    unsigned long long* d_stats = nullptr;
    int32_t* d_flag = nullptr;
    double* d_loss = nullptr;
    hipError_t e = hipMalloc(&d_v, sizeof(float) * 9 * (size_t)n_surf);
    if (e == hipSuccess) q->fixed.push_back(d_v), e = hipMalloc(&d_lum, sizeof(float) * lum.size());
    if (e == hipSuccess) q->fixed.push_back(d_lum), e = hipMalloc(&d_stats, sizeof(unsigned long long) * 3);
    if (e == hipSuccess) q->fixed.push_back(d_stats), e = hipMalloc(&d_flag, sizeof(int32_t));
    if (e == hipSuccess) q->fixed.push_back(d_flag), e = hipMalloc(&d_loss, sizeof(double));
    if (e == hipSuccess) q->fixed.push_back(d_loss), e = hipHostMalloc((void**)&q->h_flag, sizeof(int32_t));
    if (e == hipSuccess) e = hipMemcpy(d_v, tri, sizeof(float) * 9 * (size_t)n_surf, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(d_lum, lum.data(), sizeof(float) * lum.size(), hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        delete q;
        return err(RT_E_HIP, std::string("rt_neuralq_create: ") + hipGetErrorString(e));
    }
    q->r.surf_v = d_v;
    q->r.tri_lum = d_lum;
    q->r.stats = d_stats;
    q->r.flag = d_flag;
    q->loss_acc = d_loss;
    *out = q;
    return RT_OK;
}

int rt_neuralq_destroy(rt_neuralq* q) {
    delete q;
    return RT_OK;
}

int rt_neuralq_epsilon(const rt_neuralq* q, float* epsilon) {
    if (!q || !epsilon) return err(RT_E_INVALID, "NULL argument");
    *epsilon = q->eps;
    return RT_OK;
}

int rt_neuralq_render_frame(rt_ctx* ctx, rt_neuralq* q, const rt_camera* cam, const rt_params* p, float* out_rgb,
                            float* stats, uint64_t* out_ray_casts) {
    if (!ctx || !q || !cam || !p) return err(RT_E_INVALID, "NULL argument");
    if (p->width <= 0 || p->height <= 0 || p->spp <= 0 || p->max_bounces < 1)
        return err(RT_E_INVALID, "bad image size / spp / max_bounces");
    if (p->preset != RT_PRESET_GPU) return err(RT_E_UNSUPPORTED, "the Neural-Q renderer implements the GPU-engine preset");
    if ((int64_t)p->width * p->height > (int64_t)1 << 26) return err(RT_E_INVALID, "image too large");
    if (q->device != rt::ctx_device(ctx)) return err(RT_E_INVALID, "renderer belongs to another device");
    RT_HIPE(hipSetDevice(q->device));
    const int n = p->width * p->height;
    int rc = nq_ensure(q, n);
    if (rc == RT_OK) rc = ensure_ws(q->tr, n);
    if (rc != RT_OK) return rc;
    hipStream_t st = 0;
    rt::DqnLaunch a;
    memset(&a, 0, sizeof(a));
    a.scene = rt::scene_launch_view(q->scene);  // (large scenes: k_nq_trace<true> on the exact BVH)
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
    a.use_filter = 0;  // restarted rays may start outside the box the filter records assume
    rt::NqRays& r = q->r;
    r.n = n;
    rt_dqn_trainer* t = q->tr;
    RT_HIPE(hipMemsetAsync(r.total, 0, sizeof(float) * 3 * (size_t)n, st));
    RT_HIPE(hipMemsetAsync(r.stats + 2, 0, sizeof(unsigned long long), st));
    const uint32_t base = q->frames * (uint32_t)p->spp;
    for (int s = 0; s < p->spp; ++s) {
        const int smp = (int)(base + (uint32_t)s);
        RT_HIPE(hipMemsetAsync(r.stats, 0, 2 * sizeof(unsigned long long), st));
        RT_HIPE(hipMemsetAsync(q->loss_acc, 0, sizeof(double), st));
        RT_HIPE(rt::launch_nq_init(a, r, smp, st));
        for (int b = 0; b < p->max_bounces; ++b) {
            if (b > 0) {
                rc = trainer_forward(t, r.loc, n, st);
                if (rc != RT_OK) return rc;
                RT_HIPE(rt::launch_nq_sample(a, r, t->H[3], q->eps, smp, b, st));
            }
            RT_HIPE(hipMemsetAsync(r.flag, 0x01, 1, st));  // flag = 1 (little-endian low byte)
            RT_HIPE(hipMemsetAsync(reinterpret_cast<char*>(r.flag) + 1, 0, 3, st));
            RT_HIPE(rt::launch_nq_trace(a, r, b, st));
            if (b > 0) {
                for (int b0 = 0; b0 < n; b0 += q->batch) {
                    const int nb = std::min(q->batch, n - b0);
                    rc = trainer_forward(t, r.loc + (size_t)3 * b0, nb, st);
                    if (rc != RT_OK) return rc;
                    hipLaunchKernelGGL(k_td_targets, dim3(blocks_for((size_t)nb)), dim3(256), 0, st, t->H[3],
                                       r.terminal + b0, r.reward + b0, r.discount + b0, r.pix + b0, (uint32_t)smp,
                                       0x4000u + (uint32_t)b, a.seed_lo, a.seed_hi, nb, q->targets + b0);
                    RT_HIPE(hipGetLastError());
                    rc = trainer_step(t, r.prev + (size_t)3 * b0, r.action + b0, q->targets + b0, nb, st);
                    if (rc != RT_OK) return rc;
                    hipLaunchKernelGGL(k_acc_loss, dim3(1), dim3(64), 0, st, t->scal, q->loss_acc);
                    RT_HIPE(hipGetLastError());
                }
            }
            RT_HIPE(rt::launch_nq_restart(a, r, smp, b, st));
            RT_HIPE(hipMemcpyAsync(q->h_flag, r.flag, sizeof(int32_t), hipMemcpyDeviceToHost, st));
            RT_HIPE(hipStreamSynchronize(st));
            if (*q->h_flag == 1) break;
        }
        RT_HIPE(rt::launch_nq_end_sample(a, r, st));
        unsigned long long h_stats[2];
        double h_loss = 0.0;
        RT_HIPE(hipMemcpyAsync(h_stats, r.stats, sizeof(h_stats), hipMemcpyDeviceToHost, st));
        RT_HIPE(hipMemcpyAsync(&h_loss, q->loss_acc, sizeof(double), hipMemcpyDeviceToHost, st));
        RT_HIPE(hipStreamSynchronize(st));
        q->eps = std::max(q->eps - q->eps_decay, q->eps_min);
        if (stats) {
            stats[3 * s + 0] = (float)h_stats[0] / ((float)p->height * (float)p->width);
            stats[3 * s + 1] = (float)h_loss;
            stats[3 * s + 2] = (float)h_stats[1];
        }
    }
    q->frames += 1;
    RT_HIPE(rt::launch_nq_image(a, r, q->img, p->spp, st));
    unsigned long long casts = 0;
    if (out_rgb) RT_HIPE(hipMemcpyAsync(out_rgb, q->img, sizeof(float) * 3 * (size_t)n, hipMemcpyDeviceToHost, st));
    RT_HIPE(hipMemcpyAsync(&casts, r.stats + 2, sizeof(casts), hipMemcpyDeviceToHost, st));
    RT_HIPE(hipStreamSynchronize(st));
    if (out_ray_casts) *out_ray_casts = casts;
    return RT_OK;
}

}  // extern "C"
