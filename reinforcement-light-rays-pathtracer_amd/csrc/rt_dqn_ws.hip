// rt_dqn_ws.hip — the Q-network forward (k_dqn_mlp's contraction) with the weights held
// in registers: BASELINE config 4's dense hot spot.
//
// Reference: NN_Builders/dq_network.cu:36-49 (DQNetwork::network_inference, four ReLU
// affine layers), fc_layer.cu:40-72; the input x = vertices - p of
// nn_rendering_helpers.cu:280-298, folded to an affine map of p (rt_internal.hpp DqnNet).
//
// Why weight-stationary: k_dqn_mlp streams every bf16 weight fragment of layers 1-3 from
// L2 once per 64 rays (≈ 300 KB per workgroup, 1 KB per fragment feeding 4 MFMAs), which
// needs ≈ 128 B/clk per CU against the ≈ 64 B/clk a CU gets from L2: the MFMA pipe idles
// half the time.  Here one workgroup per CU (4 waves, one per SIMD) loads its share of
// the weights ONCE into registers — 343 fragments of 1 KB, 79-89 per wave (316-356
// VGPR/AGPRs of the 512 a lone wave may hold) — and then loops over 64-ray tiles of the
// active list: per tile the only memory traffic is 12 B of ray position in and 576 B of
// Q out per ray; activations stay in LDS (bf16) between the layers.
//
// N-tiles per wave (16 features each): layer 1 (320 = 20 tiles) w, w+4, .. (5 each);
// layer 2 (224 = 14) w, w+4, w+8 [, w+12] (4, 4, 3, 3); layer 3 (144 = 9) 3-w, 7-w [, 8]
// (2, 2, 2, 3): 89, 89, 79, 86 fragments.  MFMA v_mfma_f32_16x16x32_bf16, weights as the
// A operand, activations as B, fp32 accumulation in the same K order as k_dqn_mlp, so
// both kernels give the same Q bit for bit.
//
// LDS rows are XOR-swizzled at 16-B granularity (slot ^ ((row >> 2) & 7)) on strides of
// 336 / 272 bf16: the B-operand ds_read_b128 of a 16-lane group hits 16 distinct 16-B
// slots (conflict-free), the 8-B epilogue stores are 2-way (tools: the bank rule of
// MI355X_MICROARCH.md §LDS, brute-forced over the layouts).
#include "rt_trace.hpp"

namespace rt {

namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;

constexpr int kRows = 32;        // rays per tile (2 M-tiles of 16)
constexpr int kMT = kRows / 16;
constexpr int kWsThreads = 256;  // 4 waves, one per SIMD
constexpr int kStrA = 336;       // bufA row stride (K up to 320), bf16 elements
constexpr int kStrB = 272;       // bufB row stride (K up to 224)
constexpr int kQStage = kDqnActions + 1;  // fp32 Q staging rows (in bufA)
static_assert(kRows * kQStage * 4 <= kRows * kStrA * 2, "Q staging tile exceeds bufA");
// the padded shape this kernel is built for (hidden 200, 300, 200: dq_network.cu:14-17)
constexpr int kK1 = 224, kK2 = 320, kK3 = 224;
constexpr int kKs1 = kK1 / 32, kKs2 = kK2 / 32, kKs3 = kK3 / 32;
constexpr int kNt1 = 20, kNt2 = 14, kNt3 = 9;

// acc += W-fragment x activation fragment with the weights read from AGPRs: a lone wave
// holds up to 256 VGPRs and 256 AGPRs, and the stationary weights (316-356 registers) only
// fit across both files: layer 1's in VGPRs (140), layers 2-3's in AGPRs (200-244).
// gfx950 MFMAs take src A from either file, but the compiler's own MFMA forms want it in
// VGPRs (it then shuttles every fragment AGPR -> VGPR), so this one instruction is
// written out; the accumulator stays a VGPR operand.
__device__ __forceinline__ void mfma_w(f32x4& acc, const bf16x8& w, const bf16x8& x) {
    asm("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(acc) : "a"(w), "v"(x));
}

// Workgroup barrier for LDS traffic only: __syncthreads() also waits for every outstanding
// global access (vmcnt(0)), which would put the Q stores and the next tile's position
// loads on every barrier; a lone workgroup per CU has no other waves to cover that.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// element offset of (row, k) in a swizzled activation buffer
__device__ __forceinline__ int swz(int row, int k, int stride) {
    return row * stride + ((((k >> 3) ^ ((row >> 2) & 7))) << 3) + (k & 7);
}

// N-tile of slot j of wave w in layer L (see the header)
template <int L>
__device__ __forceinline__ int tile_of(int w, int j) {
    return (L < 3) ? w + 4 * j : ((j < 2) ? (3 - w) + 4 * j : 8);
}

template <int L, int NT, int KS>
__device__ __forceinline__ void load_weights(const uint16_t* __restrict__ W, int K, int wave,
                                             int lane, bf16x8 (&w)[NT][KS]) {
#pragma unroll
    for (int j = 0; j < NT; ++j) {
        const int nt = tile_of<L>(wave, j);
        const uint16_t* p = W + ((size_t)nt * (K >> 5) * 64 + lane) * 8;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) w[j][ks] = *reinterpret_cast<const bf16x8*>(p + (size_t)ks * 512);
    }
}

// One layer over the tile: acc[m][j] = sum_k W[tile j][k] act[m rows][k], then bias + ReLU
// into the next buffer (bf16, swizzled) or, for the last layer, the fp32 Q stage.
template <int L, int NT, int KS, bool LAST, bool WA>
__device__ __forceinline__ void ws_layer(const bf16x8 (&w)[NT][KS], int wave, int lane,
                                         const float* __restrict__ bias, const __bf16* in, int in_stride,
                                         __bf16* out, int out_stride) {
    const int r16 = lane & 15, kq = lane >> 4;
    f32x4 acc[kMT][NT];
#pragma unroll
    for (int m = 0; m < kMT; ++m)
#pragma unroll
        for (int j = 0; j < NT; ++j) acc[m][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    bf16x8 a[2][kMT];
#pragma unroll
    for (int m = 0; m < kMT; ++m) a[0][m] = *reinterpret_cast<const bf16x8*>(in + swz(m * 16 + r16, kq * 8, in_stride));
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
        const int cur = ks & 1;
        if (ks + 1 < KS) {
#pragma unroll
            for (int m = 0; m < kMT; ++m)
                a[cur ^ 1][m] =
                    *reinterpret_cast<const bf16x8*>(in + swz(m * 16 + r16, (ks + 1) * 32 + kq * 8, in_stride));
        }
#pragma unroll
        for (int j = 0; j < NT; ++j)
#pragma unroll
            for (int m = 0; m < kMT; ++m)
                if (WA)
                    mfma_w(acc[m][j], w[j][ks], a[cur][m]);
                else
                    acc[m][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[j][ks], a[cur][m], acc[m][j], 0, 0, 0);
    }
    // the accumulators are read by VALU next: the MFMA -> VALU read-after-write wait
    // (the compiler cannot see through the asm above): 2 x 8 idle cycles, once per layer
    if (WA) asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");
#pragma unroll
    for (int j = 0; j < NT; ++j) {
        const int col = tile_of<L>(wave, j) * 16 + kq * 4;
        const float4 bj = *reinterpret_cast<const float4*>(bias + col);
        const float bb[4] = {bj.x, bj.y, bj.z, bj.w};
#pragma unroll
        for (int m = 0; m < kMT; ++m) {
            const int row = m * 16 + r16;
            float v[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                v[r] = acc[m][j][r] + bb[r];
                v[r] = v[r] > 0.0f ? v[r] : 0.0f;
            }
            if (LAST) {
                float* st = reinterpret_cast<float*>(out) + row * kQStage + col;
                st[0] = v[0];
                st[1] = v[1];
                st[2] = v[2];
                st[3] = v[3];
            } else {
                bf16x4 h;
#pragma unroll
                for (int r = 0; r < 4; ++r) h[r] = (__bf16)v[r];
                *reinterpret_cast<bf16x4*>(out + swz(row, col, out_stride)) = h;
            }
        }
    }
}

// layer 0 (folded, exact fp32 MFMA; see rt_dqn.hip mlp_layer0) into bufB
__device__ __forceinline__ void ws_layer0(const DqnNet& net, const float4* __restrict__ l0, const float* __restrict__ locs,
                                          __bf16* out, int wave, int lane) {
    const int r16 = lane & 15, kq = lane >> 4;
    float b[kMT];
#pragma unroll
    for (int m = 0; m < kMT; ++m) b[m] = (kq < 3) ? locs[(m * 16 + r16) * 3 + kq] : 1.0f;
    const int n_tiles = net.N[0] >> 4;
#pragma unroll
    for (int j = 0; j < 4; ++j) {  // 224 features = 14 tiles over 4 waves
        const int nt = wave + 4 * j;
        if (nt >= n_tiles) continue;  // wave-uniform
        const float a = reinterpret_cast<const float*>(l0 + nt * 16 + r16)[kq];
#pragma unroll
        for (int m = 0; m < kMT; ++m) {
            const f32x4 d = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b[m], f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
            bf16x4 h;
#pragma unroll
            for (int r = 0; r < 4; ++r) h[r] = (__bf16)(d[r] > 0.0f ? d[r] : 0.0f);
            *reinterpret_cast<bf16x4*>(out + swz(m * 16 + r16, nt * 16 + kq * 4, kStrB)) = h;
        }
    }
}

// the rows' ray ids: list order, or the rows themselves
__device__ __forceinline__ int row_id(const int32_t* __restrict__ list, int row, int n_rows) {
    if (row >= n_rows) return -1;
    return (list != nullptr) ? list[row] : row;
}

template <int NT1, int NT2, int NT3>
__device__ void ws_wave(const DqnNet& net, const float* __restrict__ loc, const int32_t* __restrict__ list,
                        int n_rows, float* __restrict__ q, int ldq, bool qb, __bf16* bufA, __bf16* bufB, float* locs,
                        const float4* l0s, const float* bias1, const float* bias2, const float* bias3, int wave,
                        int lane) {
    bf16x8 w1[NT1][kKs1], w2[NT2][kKs2], w3[NT3][kKs3];
    load_weights<1, NT1, kKs1>(net.W[1], kK1, wave, lane, w1);
    load_weights<2, NT2, kKs2>(net.W[2], kK2, wave, lane, w2);
    load_weights<3, NT3, kKs3>(net.W[3], kK3, wave, lane, w3);
    const int n_tiles = (n_rows + kRows - 1) / kRows;
    // ray positions one tile ahead (threads < kRows): the id load is issued at the top of
    // a tile, the position loads after its layer 1, the LDS store at the next tile's top
    const bool loader = threadIdx.x < kRows;
    int t = blockIdx.x;
    int nid = loader ? row_id(list, t * kRows + (int)threadIdx.x, n_rows) : -1;
    float px = 0.0f, py = 0.0f, pz = 0.0f;
    if (nid >= 0) {
        px = loc[(size_t)nid * 3 + 0];
        py = loc[(size_t)nid * 3 + 1];
        pz = loc[(size_t)nid * 3 + 2];
    }
    for (; t < n_tiles; t += gridDim.x) {  // block-uniform trip count
        const int row0 = t * kRows;
        const int rows_valid = min(kRows, n_rows - row0);
        if (loader) {
            const int row = threadIdx.x;
            locs[row * 3 + 0] = px;
            locs[row * 3 + 1] = py;
            locs[row * 3 + 2] = pz;
            nid = row_id(list, (t + (int)gridDim.x) * kRows + row, n_rows);
        }
        lds_barrier();
        ws_layer0(net, l0s, locs, bufB, wave, lane);
        lds_barrier();
        ws_layer<1, NT1, kKs1, false, false>(w1, wave, lane, bias1, bufB, kStrB, bufA, kStrA);
        px = py = pz = 0.0f;
        if (nid >= 0) {
            px = loc[(size_t)nid * 3 + 0];
            py = loc[(size_t)nid * 3 + 1];
            pz = loc[(size_t)nid * 3 + 2];
        }
        lds_barrier();
        ws_layer<2, NT2, kKs2, false, true>(w2, wave, lane, bias2, bufA, kStrA, bufB, kStrB);
        lds_barrier();
        ws_layer<3, NT3, kKs3, true, true>(w3, wave, lane, bias3, bufB, kStrB, bufA, 0);
        lds_barrier();
        // the Q tile from LDS in 16-B stores (as k_dqn_mlp): rows, or action-major columns
        const float* stage = reinterpret_cast<const float*>(bufA);
        if (ldq == 0) {
            float* dst = q + (size_t)row0 * kDqnActions;
            for (int i = threadIdx.x; i < rows_valid * (kDqnActions / 4); i += kWsThreads) {
                const int r = i / (kDqnActions / 4), c = (i - r * (kDqnActions / 4)) * 4;
                const float* sp = stage + r * kQStage + c;
                *reinterpret_cast<float4*>(dst + (size_t)r * kDqnActions + c) = make_float4(sp[0], sp[1], sp[2], sp[3]);
            }
        } else if (qb) {  // the renderer's bf16 Q (k_dqn_mlp<.., QB>'s layout): q2[j * ldq + ray]
            typedef float f32x2 __attribute__((ext_vector_type(2)));
            typedef __bf16 b16x2 __attribute__((ext_vector_type(2)));
            uint32_t* const q2 = reinterpret_cast<uint32_t*>(q);
            for (int i = threadIdx.x; i < (kDqnActions / 2) * (kRows / 4); i += kWsThreads) {
                const int j = i / (kRows / 4), r = (i - j * (kRows / 4)) * 4;
                const float* sp = stage + r * kQStage + 2 * j;
                uint32_t w[4];
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const f32x2 v = {sp[k * kQStage], sp[k * kQStage + 1]};
                    w[k] = __builtin_bit_cast(uint32_t, __builtin_convertvector(v, b16x2));
                }
                *reinterpret_cast<uint4*>(q2 + (size_t)j * ldq + row0 + r) = make_uint4(w[0], w[1], w[2], w[3]);
            }
        } else {
            for (int i = threadIdx.x; i < kDqnActions * (kRows / 4); i += kWsThreads) {
                const int c = i / (kRows / 4), r = (i - c * (kRows / 4)) * 4;
                const float* sp = stage + r * kQStage + c;
                *reinterpret_cast<float4*>(q + (size_t)c * ldq + row0 + r) =
                    make_float4(sp[0], sp[kQStage], sp[2 * kQStage], sp[3 * kQStage]);
            }
        }
        // the next tile's first LDS writes (locs, then bufB after a barrier) do not touch
        // the Q stage these stores read; bufA is next written after two barriers
    }
}

__global__ __launch_bounds__(kWsThreads, 1) void k_dqn_mlp_ws(const DqnNet net, const float* __restrict__ loc,
                                                              const int32_t* __restrict__ list,
                                                              const int32_t* __restrict__ count, int max_rows,
                                                              float* __restrict__ q, int ldq, int qb) {
    __shared__ __attribute__((aligned(16))) __bf16 bufA[kRows * kStrA];
    __shared__ __attribute__((aligned(16))) __bf16 bufB[kRows * kStrB];
    __shared__ float locs[kRows * 3];
    // the layers' biases and the folded layer 0, read every tile: LDS copies
    __shared__ __attribute__((aligned(16))) float4 l0s[kK1];
    __shared__ __attribute__((aligned(16))) float bias1[kNt1 * 16];
    __shared__ __attribute__((aligned(16))) float bias2[kNt2 * 16];
    __shared__ __attribute__((aligned(16))) float bias3[kNt3 * 16];
    const int n_rows = (count != nullptr) ? min(*count, max_rows) : max_rows;
    if ((int)blockIdx.x * kRows >= n_rows) return;  // no tile for this workgroup: skip the weight loads
    for (int i = threadIdx.x; i < kK1; i += kWsThreads) l0s[i] = net.l0[i];
    for (int i = threadIdx.x; i < kNt1 * 16; i += kWsThreads) bias1[i] = net.b[1][i];
    for (int i = threadIdx.x; i < kNt2 * 16; i += kWsThreads) bias2[i] = net.b[2][i];
    for (int i = threadIdx.x; i < kNt3 * 16; i += kWsThreads) bias3[i] = net.b[3][i];
    // (visible after the first tile's barrier)
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    switch (wave) {  // the per-wave tile counts are compile-time (register arrays)
        case 0:
            ws_wave<5, 4, 2>(net, loc, list, n_rows, q, ldq, qb != 0, bufA, bufB, locs, l0s, bias1, bias2, bias3, wave, lane);
            break;
        case 1:
            ws_wave<5, 4, 2>(net, loc, list, n_rows, q, ldq, qb != 0, bufA, bufB, locs, l0s, bias1, bias2, bias3, wave, lane);
            break;
        case 2:
            ws_wave<5, 3, 2>(net, loc, list, n_rows, q, ldq, qb != 0, bufA, bufB, locs, l0s, bias1, bias2, bias3, wave, lane);
            break;
        default:
            ws_wave<5, 3, 3>(net, loc, list, n_rows, q, ldq, qb != 0, bufA, bufB, locs, l0s, bias1, bias2, bias3, wave, lane);
            break;
    }
}

}  // namespace

bool dqn_mlp_ws_fits(const DqnNet& net) {
    return net.K[1] == kK1 && net.N[1] == kNt1 * 16 && net.K[2] == kK2 && net.N[2] == kNt2 * 16 &&
           net.K[3] == kK3 && net.N[3] == kNt3 * 16 && net.N[0] == kK1;
}

hipError_t launch_dqn_mlp_ws(const DqnNet& net, const float* loc, const int32_t* list, const int32_t* count,
                             int max_rows, float* q, int ldq, int n_cu, bool qb, hipStream_t stream) {
    if (max_rows <= 0) return hipSuccess;
    const int tiles = (max_rows + kRows - 1) / kRows;
    if (ldq != 0 && (ldq < tiles * kRows || ldq % 4 != 0)) return hipErrorInvalidValue;
    const int blocks = min(tiles, n_cu);
    hipLaunchKernelGGL(k_dqn_mlp_ws, dim3((unsigned)blocks), dim3(kWsThreads), 0, stream, net, loc, list, count,
                       max_rows, q, ldq, (int)(qb && ldq != 0));
    return hipGetLastError();
}

}  // namespace rt
