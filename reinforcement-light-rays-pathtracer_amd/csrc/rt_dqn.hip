// rt_dqn.hip — the pretrained-DQN path tracer (BASELINE config 4) on gfx950.
//
// Reference: GPU/deep_learning/pre_trained_pathtracer.cu:188-491 (wavefront
// driver, initialise_ray, trace_ray), GPU/deep_learning/nn_rendering_helpers.cu
// (:143-172 accumulation, :280-298 NN input, :391-489 importance sampling),
// GPU/utils/hemisphere_helpers.cu:95-226 (grid cell -> direction, Chiu's map),
// NN_Builders/dq_network.cu + fc_layer.cu (4 ReLU affine layers).
//
// MI355X mapping:
//  * k_dqn_mlp — the dense contraction.  One workgroup = 96 active rays (M = MT * 16),
//    4 waves; each wave owns every M-tile and a quarter of the N-tiles, so each
//    weight byte is fetched once per workgroup (from L2; 0.4-0.7 MB per net).
//    v_mfma_f32_16x16x32_bf16 with fp32 accumulation; bias + ReLU fused in the
//    epilogue; activations stay in LDS (bf16) between the four layers, so
//    nothing but Q touches HBM.  The input x = vertices - ray_position is built
//    in registers straight into the A fragments (never materialised; the
//    reference writes W*H*n_in floats per bounce and ships them to DyNet on the
//    host).  Features are ordered coordinate-major so a 32-deep K step needs
//    one coordinate of the ray position.
//  * k_dqn_bounce — per active ray: Q*cos over the 144 grid cells (Chiu map,
//    one Philox draw per two cells), CDF walk, jittered direction, throughput,
//    then the closest hit of the new ray; surviving rays are appended to the
//    next active list (stream compaction with one atomic per wave).
//  * rays that end are dropped from the list, so later bounces (mean path
//    length ~24 in the thesis renders) only pay for live rays.

#include <float.h>

#include "rt_trace.hpp"

namespace rt {

namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

#ifndef RT_MLP_MT
#define RT_MLP_MT 6  // 16-row M-tiles per MLP workgroup (96 rays; 4 with the two-buffer layout)
#endif
constexpr int kTileM = RT_MLP_MT * 16;  // rays per MLP workgroup
#ifndef RT_MLP_WAVES
#define RT_MLP_WAVES 4  // waves per MLP workgroup (each owns every M-tile, 1/W of the N-tiles)
#endif
constexpr int kMlpWaves = RT_MLP_WAVES;
constexpr int kMlpThreads = 64 * kMlpWaves;
static_assert(kTileM <= kMlpThreads, "one ray position per thread at load");
// N-tile slots per wave for the widest accepted layers (out 224 | 320, 224, 144)
constexpr int slots(int tiles) { return (tiles + kMlpWaves - 1) / kMlpWaves; }
// MT = 8 (one 142 KB workgroup per CU) is 1.4x slower; a single flattened weight
// stream over layers 1-3 with a 2-4 deep register ring was 2x slower (round-1 A/B,
// DESIGN.md §4).
// LDS activation rows (bf16) are XOR-swizzled at 16-B granularity, slot ^ ((row >> 2) & 7),
// on strides of 336 / 272 elements: the B-operand ds_read_b128 of each 16-lane group then
// hits 16 distinct 16-B slots (conflict-free; the padded 328 / 232 rows were 2-way) and
// the 8-B epilogue stores are 2-way (bank rule of MI355X_MICROARCH.md §LDS, brute-forced
// over strides and swizzles)
#ifndef RT_MLP_RING_VGPRS
#define RT_MLP_RING_VGPRS 60  // VGPRs of the weight-fragment ring (60: 3 K steps of layer 1's 5 fragments)
#endif
constexpr int kMlpRingVgprs = RT_MLP_RING_VGPRS;
#ifndef RT_MLP_XPF
// 1: each layer's first weight fragments prefetched during the previous layer (archway
// 512^2 x 16 with MT = 4: 110.4 vs 111.2 ms; with MT = 6 it spills: 119.8 ms, profiles/r4p)
#define RT_MLP_XPF 0
#endif
#ifndef RT_MLP_A_DB
#define RT_MLP_A_DB 0  // 1: the next K step's activations double-buffered in registers (MT = 4: 234 VGPRs)
#endif
#ifndef RT_DQN_NT_LOAD
#define RT_DQN_NT_LOAD 1  // the sampler's reads of the bf16 Q non-temporal (read once: archway 512^2 x 16 with the NT stores: 104.6 vs 106.4 ms, profiles/r4af)
#endif
#ifndef RT_MLP_NT_STORE
#define RT_MLP_NT_STORE 1  // the renderer's bf16 Q stored non-temporally (106.4 vs 107.4 ms, profiles/r4af)
#endif
#ifndef RT_MLP_EPI2
#define RT_MLP_EPI2 1  // packed epilogue (bias pairs, ReLU on bf16 pairs; archway 1024^2 x 16: 409.7 vs 417.0 ms, profiles/r4ao)
#endif
#ifndef RT_MLP_T_NOEPI  // timing-only knobs (wrong Q): the layers' epilogues, the ray loads, the Q stores
#define RT_MLP_T_NOEPI 0
#endif
#ifndef RT_MLP_T_NOLOC
#define RT_MLP_T_NOLOC 0
#endif
#ifndef RT_MLP_T_NOSTORE
#define RT_MLP_T_NOSTORE 0
#endif
#ifndef RT_MLP_SKIP_PAD
#define RT_MLP_SKIP_PAD 0
#endif
#ifndef RT_MLP_PROLOGUE_GROUP
#define RT_MLP_PROLOGUE_GROUP 1
#endif
typedef float mlp_f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 mlp_bf16x2 __attribute__((ext_vector_type(2)));
constexpr int kStrideA = 336;
constexpr int kStrideB = 272;
#ifndef RT_MLP_INPLACE
// 1: one activation buffer (stride 336) that every layer reads and then overwrites (a
// barrier between the K loop and the epilogue; the accumulators hold the layer's outputs
// meanwhile): 2 * 336 * 2 B per row instead of (336 + 272) * 2, so MT = 7 (112 rays, 75 KB)
// still fits two workgroups per CU, and each weight fragment feeds 7 MFMAs instead of 4
#define RT_MLP_INPLACE 1  // archway 512^2 x 16: 107.4 (MT = 6) vs 110.5 ms (two buffers, MT = 4), profiles/r4o
#endif
__device__ __forceinline__ int swz(int row, int k, int stride) {
    return row * stride + (((k >> 3) ^ ((row >> 2) & 7)) << 3) + (k & 7);
}
constexpr int kStageStride = kDqnActions + 1;  // fp32 Q staging rows (in bufA)
// bf16 Q staging (RT_MLP_EPI2, the renderer's QB forward): [72 cell pairs][kQPairStride rows]
// dwords; 2 * 104 = 16 mod 64 banks, so a wave's pair-row writes hit 64 distinct banks
constexpr int kQPairStride = kTileM <= 104 ? 104 : kTileM + 8;
// the sampler's fixed sum order: kSampBlocks blocks of kSampCells cells (sample_from_q)
constexpr int kSampBlocks = 4;
constexpr int kSampCells = kDqnActions / kSampBlocks;  // 36 = 9 Philox draws
static_assert(kTileM * kStageStride * 4 <= kTileM * kStrideA * 2, "Q staging tile exceeds bufA");
// the fused sampler maps a thread to a (ray, block): 64 rays on kSampBlocks waves
constexpr bool kFusedFits = kTileM == 64 && kMlpThreads == 64 * kSampBlocks && !RT_MLP_INPLACE;
constexpr float kGridRho = 1.0f / ((float)kDqnGrid * (float)kDqnGrid);  // GRID_RHO

__device__ __forceinline__ unsigned wave_sum_u(unsigned v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

// Append `rid` to a list with one atomic per wave (order inside the list is
// irrelevant: every ray's result depends only on its own data).
__device__ __forceinline__ void list_append(bool keep, int32_t rid, int32_t* list, int32_t* count) {
    const unsigned long long m = __ballot(keep);
    if (m == 0ull) return;
    const int lane = threadIdx.x & 63;
    const int leader = __ffsll((long long)m) - 1;
    int base = 0;
    if (lane == leader) base = atomicAdd(count, __popcll(m));
    base = __shfl(base, leader, 64);
    if (keep) {
        const int rank = __popcll(m & ((1ull << lane) - 1ull));
        list[base + rank] = rid;
    }
}

// ---------------------------------------------------------------------------
// Layer 0, folded to an affine map of the ray position (rt_internal.hpp DqnNet):
// h1 = ReLU(c0 - fma(S2, z, fma(S1, y, S0 x))) as one fp32 MFMA per 16x16 tile,
// v_mfma_f32_16x16x4_f32 with A = {-S0, -S1, -S2, c0} per feature and B = (x, y, z, 1)
// per ray, C = 0: the instruction is the k-ordered fmaf chain, bit for bit
// (MI355X_MICROARCH.md, Matrix cores), i.e. exactly the expression above.  Lane l
// gets features 4(l/16)..+3 of ray l%16: one 8-B bf16 LDS store.
// ---------------------------------------------------------------------------
template <int MT>
__device__ __forceinline__ void mlp_layer0(const DqnNet& net, const float* __restrict__ loc_lds,
                                           __bf16* out_lds, int out_stride) {
    typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int r16 = lane & 15, kq = lane >> 4;
    const int n_tiles = net.N[0] >> 4;
    float b[MT];
#pragma unroll
    for (int m = 0; m < MT; ++m) b[m] = (kq < 3) ? loc_lds[(m * 16 + r16) * 3 + kq] : 1.0f;
#pragma unroll
    for (int j = 0; j < slots(14); ++j) {  // 224 features = 14 tiles: slots wave, wave + W, ..
        const int nt = wave + kMlpWaves * j;
        if (nt >= n_tiles) continue;  // wave-uniform
        const float* c = reinterpret_cast<const float*>(net.l0 + nt * 16 + r16);
        const float a = c[kq];
#pragma unroll
        for (int m = 0; m < MT; ++m) {
            const f32x4 d = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b[m], f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
            bf16x4 h;
#pragma unroll
            for (int r = 0; r < 4; ++r) h[r] = (__bf16)(d[r] > 0.0f ? d[r] : 0.0f);
            *reinterpret_cast<bf16x4*>(out_lds + swz(m * 16 + r16, nt * 16 + kq * 4, out_stride)) = h;
        }
    }
}

// ---------------------------------------------------------------------------
// MLP layers 1-3: MT*16 rows on 4 waves, A (bf16) from LDS.  Wave w owns every
// M-tile and the N-tiles w, w+4, .., w+4(NT-1) (NT = 5, 4, 3 for the widest accepted
// layers 320, 224, 144), so a weight fragment (one contiguous 1 KB load) feeds MT
// MFMAs; the fragments of K step k+32 are in flight while the MFMAs of step k run.
// Slots past the layer's last tile recompute that tile (their MFMAs are
// unconditional: a conditional MFMA makes the compiler shuttle every accumulator
// between AGPRs and VGPRs each K step) and are not stored.
// ---------------------------------------------------------------------------
// the weight-fragment ring depth of a layer with NT N-tile slots per wave
constexpr int mlp_ring(int nt) { return (kMlpRingVgprs / (4 * nt)) < 2 ? 2 : (kMlpRingVgprs / (4 * nt)); }

// wave's weight fragments of layer L, K steps 0 .. PS-1 (the layer's ring prologue), into
// pre[s * NT + j]: issued ahead (the previous layer's tail, or layer 0 for layer 1) so a
// layer starts with its first fragments in registers instead of an L2 round trip
template <int NT, int PS>
__device__ __forceinline__ void mlp_prefetch(const DqnNet& net, int L, bf16x8* pre) {
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int n_tiles = net.N[L] >> 4;
    const uint16_t* __restrict__ W = net.W[L];
#pragma unroll
    for (int j = 0; j < NT; ++j) {
        const uint16_t* wr = W + ((size_t)min(wave + kMlpWaves * j, n_tiles - 1) * (net.K[L] >> 5) * 64 + lane) * 8;
#pragma unroll
        for (int s = 0; s < PS; ++s) pre[s * NT + j] = *reinterpret_cast<const bf16x8*>(wr + s * 32 * 16);
    }
}

// PRE_IN: the ring prologue (mlp_ring(NT) - 1 steps) arrives in pre_in (mlp_prefetch);
// NTN > 0: the next layer's prologue (NTN slots, mlp_ring(NTN) - 1 steps) is issued into
// pre_out once this layer's own weight loads are done (KS > 0 only)
template <int NT, bool LAST, int MT, int KS = 0, bool INPLACE = false, bool PRE_IN = false, int NTN = 0>
__device__ __forceinline__ void mlp_layer(const DqnNet& net, int L, const __bf16* in_lds, int in_stride,
                                          __bf16* out_lds, int out_stride, const bf16x8* pre_in = nullptr,
                                          bf16x8* pre_out = nullptr) {
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int K = net.K[L];
    const int n_tiles = net.N[L] >> 4;
    const uint16_t* __restrict__ W = net.W[L];
    const float* __restrict__ bias = net.b[L];
    const int r16 = lane & 15;
    const int kg = (lane >> 4) * 8;
    const uint16_t* wrow[NT];
#pragma unroll
    for (int j = 0; j < NT; ++j)
        wrow[j] = W + ((size_t)min(wave + kMlpWaves * j, n_tiles - 1) * (K >> 5) * 64 + lane) * 8;
    f32x4 acc[MT][NT];
    // (RT_MLP_EPI2 with K known: the first K step's MFMAs take C = 0 as an inline constant,
    // no zeroing moves)
    if (!(RT_MLP_EPI2 && KS > 0)) {
#pragma unroll
        for (int m = 0; m < MT; ++m)
#pragma unroll
            for (int j = 0; j < NT; ++j) acc[m][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    if constexpr (KS > 0) {
        // K known at compile time (the reference's 200-300-200 shape): the weight
        // fragments of steps k+1 .. k+R-1 and the activations of step k+1 are in flight
        // while the MFMAs of step k run (an R-deep register ring, fully unrolled: no
        // copies).  R is set by the register budget: the kernel is held to two waves per
        // SIMD by its LDS anyway, so VGPRs up to 256 are free, and an L2 fragment load
        // (~1 us under load) needs several K steps of MFMAs (NT*MT*16 clk each) to hide.
        constexpr int R = mlp_ring(NT);
        // the activations of step k + 1 in flight during step k's MFMAs (RT_MLP_A_DB), or
        // read at the top of their own step (MT * 4 fewer VGPRs: the wider tiles)
        constexpr int AB = RT_MLP_A_DB ? 2 : 1;
        bf16x8 bw[R][NT], a[AB][MT];
#pragma unroll
        for (int s = 0; s < R - 1; ++s) {
            if (s < KS) {
#pragma unroll
                for (int j = 0; j < NT; ++j)
                    bw[s][j] = PRE_IN ? pre_in[s * NT + j] : *reinterpret_cast<const bf16x8*>(wrow[j] + s * 32 * 16);
            }
        }
#pragma unroll
        for (int m = 0; m < MT; ++m)
            a[0][m] = *reinterpret_cast<const bf16x8*>(in_lds + swz(m * 16 + r16, kg, in_stride));
#if RT_MLP_PROLOGUE_GROUP
        // the prologue's loads as their own groups: each step's groups below then claim
        // that step's own loads (without this the scheduler pairs step k's MFMAs with the
        // prologue's second step, and the ring is one step shallower than written)
        if (!PRE_IN) __builtin_amdgcn_sched_group_barrier(0x020, (R - 1 < KS ? R - 1 : KS) * NT, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, MT, 0);
#endif
        constexpr int PN = NTN > 0 ? mlp_ring(NTN) - 1 : 0;  // next layer's prologue steps
        const bool last_valid = __builtin_amdgcn_readfirstlane(wave) + kMlpWaves * (NT - 1) < n_tiles;
        constexpr int KP = KS - R + 1 > 0 ? KS - R + 1 : 0;  // first step without own loads
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            if (ks + R - 1 < KS) {
#pragma unroll
                for (int j = 0; j < NT; ++j)
                    bw[(ks + R - 1) % R][j] = *reinterpret_cast<const bf16x8*>(wrow[j] + (ks + R - 1) * 32 * 16);
            }
            if (AB == 2 && ks + 1 < KS) {
#pragma unroll
                for (int m = 0; m < MT; ++m)
                    a[(ks + 1) % AB][m] =
                        *reinterpret_cast<const bf16x8*>(in_lds + swz(m * 16 + r16, (ks + 1) * 32 + kg, in_stride));
            }
            if (AB == 1 && ks > 0) {
#pragma unroll
                for (int m = 0; m < MT; ++m)
                    a[0][m] = *reinterpret_cast<const bf16x8*>(in_lds + swz(m * 16 + r16, ks * 32 + kg, in_stride));
            }
            if (PN > 0 && ks == KP) mlp_prefetch<(NTN > 0 ? NTN : 1), PN>(net, L + 1, pre_out);
#pragma unroll
            for (int j = 0; j < NT; ++j) {
                // (RT_MLP_SKIP_PAD: the wave's last slot, past the layer's tiles for some waves,
                // skipped by a wave-uniform branch instead of recomputing the last tile)
                if (RT_MLP_SKIP_PAD && j == NT - 1 && !last_valid) continue;
#pragma unroll
                for (int m = 0; m < MT; ++m)
                    acc[m][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                        bw[ks % R][j], a[ks % AB][m], (RT_MLP_EPI2 && ks == 0) ? f32x4{0.f, 0.f, 0.f, 0.f} : acc[m][j],
                        0, 0, 0);
            }
#if RT_MLP_PROLOGUE_GROUP
            if (ks + R - 1 < KS) __builtin_amdgcn_sched_group_barrier(0x020, NT, 0);  // VMEM reads
            if (PN > 0 && ks == KP) __builtin_amdgcn_sched_group_barrier(0x020, PN * (NTN > 0 ? NTN : 1), 0);
            if (AB == 2 ? ks + 1 < KS : ks > 0) __builtin_amdgcn_sched_group_barrier(0x100, MT, 0);  // LDS reads
#else
            __builtin_amdgcn_sched_group_barrier(0x020, NT, 0);
            __builtin_amdgcn_sched_group_barrier(0x100, MT, 0);
#endif
            __builtin_amdgcn_sched_group_barrier(0x008, NT * MT, 0);  // MFMA
        }
    } else {
    // weight fragments ping-pong between b0 and b1 (no register copies, which would
    // make the loads of step k+1 wait inside step k): step k's MFMAs run while step
    // k+1's fragments are in flight; sched_group_barrier keeps the order
    // loads -> A reads -> MFMAs (the scheduler otherwise sinks each load to its use)
    bf16x8 b0[NT], b1[NT];
#pragma unroll
    for (int j = 0; j < NT; ++j) b0[j] = *reinterpret_cast<const bf16x8*>(wrow[j]);
    auto step = [&](int k0, const bf16x8 (&bw)[NT]) {
        bf16x8 a[MT];
#pragma unroll
        for (int m = 0; m < MT; ++m)
            a[m] = *reinterpret_cast<const bf16x8*>(in_lds + swz(m * 16 + r16, k0 + kg, in_stride));
#pragma unroll
        for (int j = 0; j < NT; ++j)
#pragma unroll
            for (int m = 0; m < MT; ++m)  // D^T = W * act^T: lane holds 4 features of one ray
                acc[m][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw[j], a[m], acc[m][j], 0, 0, 0);
    };
    int k0 = 0;
    for (; k0 + 32 < K; k0 += 64) {
#pragma unroll
        for (int j = 0; j < NT; ++j) b1[j] = *reinterpret_cast<const bf16x8*>(wrow[j] + (k0 + 32) * 16);
        step(k0, b0);
        __builtin_amdgcn_sched_group_barrier(0x020, NT, 0);       // VMEM reads
        __builtin_amdgcn_sched_group_barrier(0x100, MT, 0);       // LDS reads
        __builtin_amdgcn_sched_group_barrier(0x008, NT * MT, 0);  // MFMA
        const int kn = min(k0 + 64, K - 32);
#pragma unroll
        for (int j = 0; j < NT; ++j) b0[j] = *reinterpret_cast<const bf16x8*>(wrow[j] + kn * 16);
        step(k0 + 32, b1);
        __builtin_amdgcn_sched_group_barrier(0x020, NT, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, MT, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, NT * MT, 0);
    }
    if (k0 < K) step(k0, b0);  // odd number of K steps
    }
    if constexpr (INPLACE) __syncthreads();  // every wave has read the layer's input
    // epilogue: bias + ReLU (fc_layer.cu:40-72, dynet::rectify)
#if RT_MLP_T_NOEPI  // timing only: no epilogue (wrong Q)
    if (acc[0][0][0] != 12345.0f) return;
#endif
    // (the weights are the MFMA's A operand, the activations its B operand, so a lane
    // holds 4 consecutive features of one ray: one 8-B (bf16) or 16-B (fp32) LDS store)
#pragma unroll
    for (int j = 0; j < NT; ++j) {
        const int nt = wave + kMlpWaves * j;
        if (nt >= n_tiles) continue;  // wave-uniform
        const int col = nt * 16 + (lane >> 4) * 4;
        const float4 bj = *reinterpret_cast<const float4*>(bias + col);
        const float bb[4] = {bj.x, bj.y, bj.z, bj.w};
#pragma unroll
        for (int m = 0; m < MT; ++m) {
            const int row = m * 16 + r16;
#if RT_MLP_EPI2
            if (!LAST || out_stride != 0) {
                // bias in packed adds (the same IEEE sums), then RNE to bf16 and the ReLU on the
                // bf16 pairs as a signed 16-bit max with 0: RN is monotone with RN(0) = 0, so
                // max(RN(v), 0) = RN(max(v, 0)) for every finite v (a negative bf16 is a
                // negative int16; -0 becomes +0 as the fp32 ReLU gives)
                const mlp_f32x2 s01 = mlp_f32x2{acc[m][j][0], acc[m][j][1]} + mlp_f32x2{bb[0], bb[1]};
                const mlp_f32x2 s23 = mlp_f32x2{acc[m][j][2], acc[m][j][3]} + mlp_f32x2{bb[2], bb[3]};
                typedef short mlp_i16x2 __attribute__((ext_vector_type(2)));
                const mlp_i16x2 z = {0, 0};
                mlp_i16x2 h01 = __builtin_bit_cast(mlp_i16x2, __builtin_convertvector(s01, mlp_bf16x2));
                mlp_i16x2 h23 = __builtin_bit_cast(mlp_i16x2, __builtin_convertvector(s23, mlp_bf16x2));
                h01 = h01 > z ? h01 : z;
                h23 = h23 > z ? h23 : z;
                if (LAST) {  // the renderer's bf16 Q: cell pairs staged action-major, [pair][row]
                    uint32_t* const st2 = reinterpret_cast<uint32_t*>(out_lds);
                    st2[(col >> 1) * out_stride + row] = __builtin_bit_cast(uint32_t, h01);
                    st2[((col >> 1) + 1) * out_stride + row] = __builtin_bit_cast(uint32_t, h23);
                    continue;
                }
                uint2 w;
                w.x = __builtin_bit_cast(uint32_t, h01);
                w.y = __builtin_bit_cast(uint32_t, h23);
                *reinterpret_cast<uint2*>(out_lds + swz(row, col, out_stride)) = w;
                continue;
            }
#endif
            float v[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                v[r] = acc[m][j][r] + bb[r];
                v[r] = v[r] > 0.0f ? v[r] : 0.0f;
            }
            if (LAST) {  // fp32 Q tile staged in LDS, written out coalesced by the caller
                float* st = reinterpret_cast<float*>(out_lds) + row * kStageStride + col;
                st[0] = v[0];
                st[1] = v[1];
                st[2] = v[2];
                st[3] = v[3];
            } else {
                typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
                bf16x4 h;
#pragma unroll
                for (int r = 0; r < 4; ++r) h[r] = (__bf16)v[r];
                *reinterpret_cast<bf16x4*>(out_lds + swz(row, col, out_stride)) = h;
            }
        }
    }
}


// The fused Q.cos sampler's per-ray inputs (k_dqn_mlp<MT, true>): the rays' pixel keys and
// sample (ray id = slot * n_pix + pixel slot, as k_dqn_bounce), the Philox event and key.
struct MlpSample {
    const uint32_t* pix = nullptr;
    int n_pix = 0, s0 = 0;
    uint32_t ev = 0, k0 = 0, k1 = 0;
};

__device__ __forceinline__ float chiu_cos_cell(int a, float r1, float r2) {
    const int gxi = a / kDqnGrid;
    const int gyi = a - gxi * kDqnGrid;
    return chiu_cos((float)gxi + r1, (float)gyi + r2);  // cos of the jittered cell direction
}
// the same for the cell's two 16-bit jitters in one Philox word (u16lo / u16hi): the grid
// coordinate cell + k 2^-16 as one fma -- both terms and their sum exact, so the same
// float as u16lo's product then the add (the build does not contract them itself)
__device__ __forceinline__ float chiu_cos_cell_w(int a, uint32_t w) {
    const int gxi = a / kDqnGrid;
    const int gyi = a - gxi * kDqnGrid;
    return chiu_cos(fmaf((float)(w & 0xffffu), 0x1p-16f, (float)gxi), fmaf((float)(w >> 16), 0x1p-16f, (float)gyi));
}

// One workgroup = MT*16 rays (LDS: MT = 6 in place -> 66 KB, two workgroups per CU).
// FUSED: instead of writing Q out, the workgroup runs importance_sample_direction's
// selection (nn_rendering_helpers.cu:391-489) on its LDS tile in sample_from_q's blocked
// order, one thread per (ray, block of 36 cells): Q*cos and the block sums, then the total,
// the block prefixes and the walks of the reached blocks, the first block's cell winning -- and
// writes the chosen cell and its normalised Q*cos per ray (q[i] = action bits,
// q[ldq + i] = qd), 8 B instead of 576 B of Q per ray; k_dqn_bounce<MF, true> finishes the
// direction.  Q never leaves the chip.
template <int MT, bool FUSED = false, bool QB = false>
#ifndef RT_MLP_MIN_WAVES
#define RT_MLP_MIN_WAVES 2  // waves per SIMD: the workgroups per CU that its LDS admits (3: MT = 4 in place)
#endif
__global__ __launch_bounds__(kMlpThreads, RT_MLP_MIN_WAVES) void k_dqn_mlp(const DqnNet net, const float* __restrict__ loc,
                                                 const int32_t* __restrict__ list,
                                                 const int32_t* __restrict__ count, int max_rows,
                                                 float* __restrict__ q, int ldq, const MlpSample smp) {
    constexpr int kRows = MT * 16;
    __shared__ __attribute__((aligned(16))) __bf16 bufA[kRows * kStrideA];
    __shared__ __attribute__((aligned(16))) __bf16 bufB[RT_MLP_INPLACE ? 8 : kRows * kStrideB];
    __shared__ float locs[kRows * 3];
    const int n_rows = (count != nullptr) ? min(*count, max_rows) : max_rows;
    const int row0 = blockIdx.x * kRows;
    if (row0 >= n_rows) return;
    const int rows_valid = min(kRows, n_rows - row0);
    // layer 1's first weight fragments in flight during the ray loads and layer 0
    const bool ref_net = net.K[1] == 224 && net.K[2] == 320 && net.K[3] == 224;
    bf16x8 p1[RT_MLP_XPF ? (mlp_ring(slots(20)) - 1) * slots(20) : 1];
    if constexpr (RT_MLP_XPF != 0) {
        if (ref_net) mlp_prefetch<slots(20), mlp_ring(slots(20)) - 1>(net, 1, p1);
    }
    if (threadIdx.x < kRows) {
        const int row = threadIdx.x;
        float x = 0.0f, y = 0.0f, z = 0.0f;
        if (row < rows_valid && !RT_MLP_T_NOLOC) {  // (RT_MLP_T_NOLOC: timing only, positions 0)
            const int rid = (list != nullptr) ? list[row0 + row] : (row0 + row);
            x = loc[(size_t)rid * 3 + 0];
            y = loc[(size_t)rid * 3 + 1];
            z = loc[(size_t)rid * 3 + 2];
        }
        locs[row * 3 + 0] = x;
        locs[row * 3 + 1] = y;
        locs[row * 3 + 2] = z;
    }
    __syncthreads();
#if RT_MLP_INPLACE
    mlp_layer0<MT>(net, locs, bufA, kStrideA);
    __syncthreads();
    if (ref_net) {  // the reference's 200-300-200 net
        bf16x8 p2[RT_MLP_XPF ? (mlp_ring(slots(14)) - 1) * slots(14) : 1];
        bf16x8 p3[RT_MLP_XPF ? (mlp_ring(slots(9)) - 1) * slots(9) : 1];
        mlp_layer<slots(20), false, MT, 7, true, RT_MLP_XPF, RT_MLP_XPF ? slots(14) : 0>(net, 1, bufA, kStrideA, bufA,
                                                                                      kStrideA, p1, p2);
        __syncthreads();
        mlp_layer<slots(14), false, MT, 10, true, RT_MLP_XPF, RT_MLP_XPF ? slots(9) : 0>(net, 2, bufA, kStrideA, bufA,
                                                                                      kStrideA, p2, p3);
        __syncthreads();
        mlp_layer<slots(9), true, MT, 7, true, RT_MLP_XPF>(net, 3, bufA, kStrideA, bufA, (RT_MLP_EPI2 && QB) ? kQPairStride : 0,
                                                          p3);
    } else {
        mlp_layer<slots(20), false, MT, 0, true>(net, 1, bufA, kStrideA, bufA, kStrideA);  // N <= 320
        __syncthreads();
        mlp_layer<slots(14), false, MT, 0, true>(net, 2, bufA, kStrideA, bufA, kStrideA);  // N <= 224
        __syncthreads();
        mlp_layer<slots(9), true, MT, 0, true>(net, 3, bufA, kStrideA, bufA, (RT_MLP_EPI2 && QB) ? kQPairStride : 0);
    }
    (void)bufB;
#else
#ifndef RT_MLP_SKIP_L0  // timing only: layer 0 not evaluated (wrong Q)
    mlp_layer0<MT>(net, locs, bufB, kStrideB);
#endif
    __syncthreads();
    if (ref_net) {  // the reference's 200-300-200 net
        bf16x8 p2[RT_MLP_XPF ? (mlp_ring(slots(14)) - 1) * slots(14) : 1];
        bf16x8 p3[RT_MLP_XPF ? (mlp_ring(slots(9)) - 1) * slots(9) : 1];
        mlp_layer<slots(20), false, MT, 7, false, RT_MLP_XPF, RT_MLP_XPF ? slots(14) : 0>(net, 1, bufB, kStrideB, bufA,
                                                                                       kStrideA, p1, p2);
        __syncthreads();
        mlp_layer<slots(14), false, MT, 10, false, RT_MLP_XPF, RT_MLP_XPF ? slots(9) : 0>(net, 2, bufA, kStrideA, bufB,
                                                                                       kStrideB, p2, p3);
        __syncthreads();
        mlp_layer<slots(9), true, MT, 7, false, RT_MLP_XPF>(net, 3, bufB, kStrideB, bufA, 0, p3);
    } else {
        mlp_layer<slots(20), false, MT>(net, 1, bufB, kStrideB, bufA, kStrideA);  // N <= 320
        __syncthreads();
        mlp_layer<slots(14), false, MT>(net, 2, bufA, kStrideA, bufB, kStrideB);  // N <= 224
        __syncthreads();
        mlp_layer<slots(9), true, MT>(net, 3, bufB, kStrideB, bufA, 0);           // N = 144
    }
#endif
    __syncthreads();
    if constexpr (FUSED && kFusedFits) {
        static_assert(kRows == 64 && kMlpThreads == 64 * kSampBlocks, "the fused sampler maps a thread to a block");
        float* const stage = reinterpret_cast<float*>(bufA);  // [row][kStageStride]: Q -> Q*cos
        float* const bsum = reinterpret_cast<float*>(bufB);   // [row][block] B_w (bufB is free after layer 3)
        const int r = threadIdx.x & 63, w = threadIdx.x >> 6;  // ray, block (sample_from_q's order)
        const bool live = r < rows_valid;
        uint32_t pixid = 0, sample = 0;
        if (live) {
            const int rid = list[row0 + r];
            const int slot = rid / smp.n_pix;
            pixid = smp.pix[rid - slot * smp.n_pix];
            sample = (uint32_t)(smp.s0 + slot);
        }
        float* const srow = stage + r * kStageStride;
        // (1) Q*cos of the block's cells (one Philox draw per four cells, counter 1 + a/4), B_w
        const PhiloxShared ph = philox_shared(pixid, sample, smp.ev, smp.k0, smp.k1);
        if (live) {
            const int c0 = w * kSampCells;
            float b = 0.0f;
#pragma unroll 3
            for (int a = c0; a < c0 + kSampCells; a += 4) {
                uint32_t o[4];
                philox_from(ph, 1u + (uint32_t)(a >> 2), o);
#pragma unroll
                for (int h = 0; h < 4; ++h) {
                    const float qc = srow[a + h] * chiu_cos_cell_w(a + h, o[h]);
                    srow[a + h] = qc;
                    b = b + qc;
                }
            }
            bsum[r * kSampBlocks + w] = b;
        }
        __syncthreads();
        // (2) every (ray, block) thread: the total and its block's prefixes; the block is walked
        // iff it is reached (P_{w+1} > rv) -- in parallel, the first reached block that finds
        // a cell winning (sample_from_q walks them in order and stops there: the same cell)
        int* const hit = reinterpret_cast<int*>(bsum + kRows * kSampBlocks);  // [row][block]
        float* const hq = reinterpret_cast<float*>(hit + kRows * kSampBlocks);
        if (live) {
            uint32_t o[4];
            philox_from(ph, 0u, o);
            const float rv = u01(o[0]);
            float bs[kSampBlocks];
            float total = 0.0f;
#pragma unroll
            for (int k = 0; k < kSampBlocks; ++k) {
                bs[k] = bsum[r * kSampBlocks + k];
                total = total + bs[k];
            }
            float P = 0.0f, Pn = 0.0f;
#pragma unroll
            for (int k = 0; k < kSampBlocks; ++k) {
                Pn = P + bs[k] / total;
                if (k == w) break;
                P = Pn;
            }
            int act = -1;
            float qsel = 0.0f;
            if (Pn > rv) {
                float cum = P;
                for (int a = w * kSampCells; a < (w + 1) * kSampCells && act < 0; ++a) {
                    const float qd = srow[a] / total;
                    cum = cum + qd;
                    if (cum > rv && qd > 0.0f) {
                        act = a;
                        qsel = qd;
                    }
                }
            }
            hit[r * kSampBlocks + w] = act;
            hq[r * kSampBlocks + w] = qsel;
        }
        __syncthreads();
        if (w == 0 && live) {
            int act = -1;
            float qsel = 0.0f;
#pragma unroll
            for (int k = 0; k < kSampBlocks; ++k) {
                const int h = hit[r * kSampBlocks + k];
                if (act < 0 && h >= 0) {
                    act = h;
                    qsel = hq[r * kSampBlocks + k];
                }
            }
            q[row0 + r] = __int_as_float(act);
            q[(size_t)ldq + row0 + r] = qsel;
        }
        return;
    }
    // Q tile [kRows][144] from LDS (odd row stride: conflict-free column reads) in
    // 16-B stores: row-major rows are one contiguous run, action-major columns runs
    // of kRows rows (ldq covers every launched row, so padding rows may be written).
    const float* stage = reinterpret_cast<const float*>(bufA);
#if RT_MLP_T_NOSTORE  // timing only: Q not written
    if (stage[threadIdx.x] != 12345.0f) return;
#endif
    if (ldq == 0) {
        float* dst = q + (size_t)row0 * kDqnActions;
        for (int t = threadIdx.x; t < rows_valid * (kDqnActions / 4); t += kMlpThreads) {
            const int r = t / (kDqnActions / 4), c = (t - r * (kDqnActions / 4)) * 4;
            const float* sp = stage + r * kStageStride + c;
            *reinterpret_cast<float4*>(dst + (size_t)r * kDqnActions + c) = make_float4(sp[0], sp[1], sp[2], sp[3]);
        }
    } else if constexpr (QB) {
        // the renderer's Q in bf16 (RNE), cells 2j and 2j + 1 of a ray in one dword (low,
        // high): q2[j * ldq + ray], 16-B runs of four rays -- half the bytes of the fp32 tile
        uint32_t* const q2 = reinterpret_cast<uint32_t*>(q);
#if RT_MLP_EPI2 && RT_MLP_INPLACE
        static_assert(kRows <= kQPairStride && (kDqnActions / 2) * kQPairStride * 4 <= kRows * kStrideA * 2,
                      "the bf16 Q staging fits bufA");
        const uint32_t* const st2 = reinterpret_cast<const uint32_t*>(bufA);
        for (int t = threadIdx.x; t < (kDqnActions / 2) * (kRows / 4); t += kMlpThreads) {
            const int j = t / (kRows / 4), r = (t - j * (kRows / 4)) * 4;
            const uint4 v = *reinterpret_cast<const uint4*>(st2 + j * kQPairStride + r);
#if RT_MLP_NT_STORE
            typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));
            const u32x4v wv = {v.x, v.y, v.z, v.w};
            __builtin_nontemporal_store(wv, reinterpret_cast<u32x4v*>(q2 + (size_t)j * ldq + row0 + r));
#else
            *reinterpret_cast<uint4*>(q2 + (size_t)j * ldq + row0 + r) = v;
#endif
        }
        if (true) return;
#endif
        for (int t = threadIdx.x; t < (kDqnActions / 2) * (kRows / 4); t += kMlpThreads) {
            const int j = t / (kRows / 4), r = (t - j * (kRows / 4)) * 4;
            const float* sp = stage + r * kStageStride + 2 * j;
            uint32_t w[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const mlp_f32x2 v = {sp[k * kStageStride], sp[k * kStageStride + 1]};
                w[k] = __builtin_bit_cast(uint32_t, __builtin_convertvector(v, mlp_bf16x2));
            }
#if RT_MLP_NT_STORE
            // streamed past the caches: the weights the other workgroups re-read stay in L2
            typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));
            const u32x4v wv = {w[0], w[1], w[2], w[3]};
            __builtin_nontemporal_store(wv, reinterpret_cast<u32x4v*>(q2 + (size_t)j * ldq + row0 + r));
#else
            *reinterpret_cast<uint4*>(q2 + (size_t)j * ldq + row0 + r) = make_uint4(w[0], w[1], w[2], w[3]);
#endif
        }
    } else {
        for (int t = threadIdx.x; t < kDqnActions * (kRows / 4); t += kMlpThreads) {
            const int c = t / (kRows / 4), r = (t - c * (kRows / 4)) * 4;
            const float* sp = stage + r * kStageStride + c;
            *reinterpret_cast<float4*>(q + (size_t)c * ldq + row0 + r) =
                make_float4(sp[0], sp[kStageStride], sp[2 * kStageStride], sp[3 * kStageStride]);
        }
    }
}

struct SampleOut {
    int action;   // -1: no cell selected (the reference then traces a zero direction: a miss)
    f3 dir;
};

// the chosen cell's jittered direction (Philox counter 1 + 72) and the throughput update
// cos / pdf, pdf = RHO * (qd / GRID_RHO) -- the end of importance_sample_direction
__device__ __forceinline__ SampleOut sample_finish(int action, float qd_sel, f3 N, f3 T, f3 B, f3 pos,
                                                   const PhiloxShared& ph, f3* tp, bool update_tp) {
    SampleOut res;
    res.action = action;
    res.dir = make3(0.0f, 0.0f, 0.0f);
    if (action >= 0) {
        uint32_t o[4];
        philox_from(ph, 1u + kDqnActions / 2, o);
        const int gxi = action / kDqnGrid;
        const int gyi = action - gxi * kDqnGrid;
        res.dir = grid_direction((float)gxi + u01(o[0]), (float)gyi + u01(o[1]), N, T, B, pos);
        if (update_tp) {
            const float c = dot(N, res.dir);
            const float pdf = kRho * (qd_sel / kGridRho);
            tp->x = (tp->x * c) / pdf;
            tp->y = (tp->y * c) / pdf;
            tp->z = (tp->z * c) / pdf;
        }
    }
    return res;
}

// importance_sample_direction (nn_rendering_helpers.cu:391-489) for one ray, on its 144 Q
// values q[a * qs] (qs = 1 for a [row][144] buffer, ldq for the action-major one).
// The sums run in a fixed blocked order (kSampBlocks blocks of kSampCells consecutive
// cells; the fused k_dqn_mlp<.., true> gives each block its own thread, the oracle's
// dqn_sample adds the same way):
//   qc = Q * cos (the cell's jittered direction), B_w = sum of qc over block w in cell
//   order, total = ((B_0 + B_1) + B_2) + B_3, P_0 = 0, P_{w+1} = P_w + B_w / total;
//   the walk starts in the first block w with P_{w+1} > rv: cum = P_w, then cell by cell
//   cum = cum + qc / total, taking the first cell with cum > rv and qd = qc / total > 0
//   (on into the next block if rounding leaves the block without one).
// Inside the chosen block this is the reference's own walk (cum = q_sum + qd per cell);
// the block sums only change the association of the float sums.  Only one block's cells
// are divided and walked.  WB: q is overwritten with Q * cos, as the reference does in
// place (rt_dqn_sample, the Neural-Q sampler); without it the walk recomputes its block's
// Q * cos (the same operations, so the same bits) instead of a 576-B store and reload.
// QB: q holds the renderer's bf16 Q (k_dqn_mlp<.., QB>): cells 2j, 2j + 1 in dword j * qs
template <bool WB, bool QB = false>
__device__ __forceinline__ SampleOut sample_from_q(float* __restrict__ q, size_t qs, f3 N, f3 T, f3 B, f3 pos,
                                                   uint32_t pix, uint32_t smp, uint32_t ev,
                                                   uint32_t k0, uint32_t k1, f3* tp, bool update_tp) {
    static_assert(!(WB && QB), "the in-place Q*cos store needs the fp32 buffer");
    // every draw of the ray shares (pixel, sample, event): rounds 1-3's shared part once
    const PhiloxShared ph = philox_shared(pix, smp, ev, k0, k1);
    uint32_t o[4];
    philox_from(ph, 0u, o);
    const float rv = u01(o[0]);
    // Q is read in groups of kQGroup cells (all loads of a group in flight at once:
    // one-at-a-time loads put an HBM round trip on every cell)
    constexpr int kQGroup = 12;
    static_assert(kSampCells % kQGroup == 0, "groups tile the blocks");
    // Q*cos of the group of cells g .. g + kQGroup - 1 into qv (q holds Q, or Q*cos if done)
    auto qcos = [&](int g, float* qv, bool stored) {
        if constexpr (QB) {
            const uint32_t* q2 = reinterpret_cast<const uint32_t*>(q);
#pragma unroll
            for (int u = 0; u < kQGroup; u += 2) {
#if RT_DQN_NT_LOAD
                const uint32_t w = stored ? q2[(size_t)((g + u) >> 1) * qs]
                                          : __builtin_nontemporal_load(q2 + (size_t)((g + u) >> 1) * qs);
#else
                const uint32_t w = q2[(size_t)((g + u) >> 1) * qs];
#endif
                qv[u] = __uint_as_float(w << 16);
                qv[u + 1] = __uint_as_float(w & 0xffff0000u);
            }
        } else {
#pragma unroll
            for (int u = 0; u < kQGroup; ++u) qv[u] = q[(size_t)(g + u) * qs];
        }
        if (stored) return;
#pragma unroll
        for (int u4 = 0; u4 < kQGroup; u4 += 4) {
            uint32_t r[4];
            philox_from(ph, 1u + (uint32_t)((g + u4) >> 2), r);
#pragma unroll
            for (int h = 0; h < 4; ++h) qv[u4 + h] = qv[u4 + h] * chiu_cos_cell_w(g + u4 + h, r[h]);
        }
    };
    float bs[kSampBlocks];
#pragma unroll
    for (int w = 0; w < kSampBlocks; ++w) {
        float b = 0.0f;
        for (int g = w * kSampCells; g < (w + 1) * kSampCells; g += kQGroup) {
            float qv[kQGroup];
            qcos(g, qv, false);
#pragma unroll
            for (int u = 0; u < kQGroup; ++u) {
                if (WB) q[(size_t)(g + u) * qs] = qv[u];
                b = b + qv[u];
            }
        }
        bs[w] = b;
    }
    float total = 0.0f;
#pragma unroll
    for (int w = 0; w < kSampBlocks; ++w) total = total + bs[w];
    SampleOut res;
    res.action = -1;
    res.dir = make3(0.0f, 0.0f, 0.0f);
    float qd_sel = 0.0f;
    float P = 0.0f;  // P_w
    for (int w = 0; w < kSampBlocks && res.action < 0; ++w) {
        const float Pn = P + bs[w] / total;
        if (Pn > rv) {
            float cum = P;
            for (int g = w * kSampCells; g < (w + 1) * kSampCells && res.action < 0; g += kQGroup) {
                float qv[kQGroup];
                qcos(g, qv, WB);
#pragma unroll
                for (int u = 0; u < kQGroup; ++u) {
                    const float qd = qv[u] / total;
                    cum = cum + qd;
                    if (res.action < 0 && cum > rv && qd > 0.0f) {
                        res.action = g + u;
                        qd_sel = qd;
                    }
                }
            }
        }
        P = Pn;
    }
    return sample_finish(res.action, qd_sel, N, T, B, pos, ph, tp, update_tp);
}

// trace_ray (pre_trained_pathtracer.cu:413-491): Ray(pos + dir*1e-5, dir), GPU hit rule.
// Returns true if the ray continues (hit a surface).
// MF > 0: the cast on the matrix-core filter (closest_hit_mf: every lane of the wave
// calls, `active` false for a lane without a ray, which then returns false untouched).
// MF < 0: the exact BVH (large scenes, closest_hit_bvh), wl = the lane's LDS stack column.
// BOUNCE (MF > 0): a bounce ray leaving surface `surf`, its candidates from the scene's rule-1
// candidate table when it has one (closest_hit_ctab, rt_ctab.cpp; wave-uniform choice)
#ifndef RT_DQN_CTAB
#define RT_DQN_CTAB 1  // 0: the bounce casts on the matrix-core image even with a candidate table (A/B)
#endif
template <int MF, bool BOUNCE = false, bool CT = false>
__device__ __forceinline__ bool dqn_trace(const DqnLaunch& a, f3 pos, f3 dir, bool active, float* wl, f3* loc_out,
                                          int* tri_out, f3* tp, int surf = -1) {
    const f3 o = make3(pos.x + dir.x * kEps, pos.y + dir.y * kEps, pos.z + dir.z * kEps);
    const f3 d = normalize(dir);
    Hit h;
    if constexpr (MF > 0) {
        // CT: the launcher checked the table serves this launch (no matrix-core path compiled in)
        if constexpr (CT)
            h = closest_hit_ctab<1, MF>(a.scene, a.scene.ctab[1], surf, o, d, a.t_scale, active, wl);
        else if (BOUNCE && RT_DQN_CTAB && ctab_usable(a.scene.ctab[1], a.t_scale) && a.scene.ctab[1].words <= MF)
            h = closest_hit_ctab<1, MF>(a.scene, a.scene.ctab[1], surf, o, d, a.t_scale, active, wl);
        else
            h = closest_hit_mf<1, false, MF>(a.scene, o, d, a.t_scale, active, wl);
        if (!active) return false;
    } else if constexpr (MF < 0) {
        if (!active) return false;
        h = closest_hit_bvh<1, 256>(a.scene, o, d, a.t_scale, reinterpret_cast<int*>(wl));
    } else {
        if (!active) return false;
        h = closest_hit_sel<1>(a.scene, a.use_filter, o, d, a.t_scale);
    }
    if (h.tri < 0) {
        *tp = make3(tp->x * a.env_light, tp->y * a.env_light, tp->z * a.env_light);
        return false;
    }
    const float4 c = a.scene.shade[h.tri * kShadeF4 + 3];
    if (h.tri >= a.scene.n_surf) {
        *tp = make3(tp->x * c.x, tp->y * c.y, tp->z * c.z);
        return false;
    }
    const float Dx = d.x * a.t_scale, Dy = d.y * a.t_scale, Dz = d.z * a.t_scale;
    *loc_out = make3(o.x + h.t * Dx, o.y + h.t * Dy, o.z + h.t * Dz);
    *tri_out = h.tri;
    *tp = make3(tp->x * c.x, tp->y * c.y, tp->z * c.z);  // *= BRDF
    return true;
}

#ifndef RT_DQN_NT_STATE
#define RT_DQN_NT_STATE 0  // 1: the per-ray state (position, throughput) loaded and stored non-temporally (A/B)
#endif
__device__ __forceinline__ f3 ld3(const float* p, int i) {
#if RT_DQN_NT_STATE
    return make3(__builtin_nontemporal_load(p + (size_t)i * 3), __builtin_nontemporal_load(p + (size_t)i * 3 + 1),
                 __builtin_nontemporal_load(p + (size_t)i * 3 + 2));
#else
    return make3(p[(size_t)i * 3], p[(size_t)i * 3 + 1], p[(size_t)i * 3 + 2]);
#endif
}
__device__ __forceinline__ void st3(float* p, int i, f3 v) {
#if RT_DQN_NT_STATE
    __builtin_nontemporal_store(v.x, p + (size_t)i * 3);
    __builtin_nontemporal_store(v.y, p + (size_t)i * 3 + 1);
    __builtin_nontemporal_store(v.z, p + (size_t)i * 3 + 2);
#else
    p[(size_t)i * 3] = v.x;
    p[(size_t)i * 3 + 1] = v.y;
    p[(size_t)i * 3 + 2] = v.z;
#endif
}

// ray id -> pixel of the tile list
__device__ __forceinline__ bool ray_pixel(const DqnLaunch& a, int rid, int* px, int* py) {
    const BlockDesc blk = a.blocks[rid >> 8];
    const int q = rid & 255;
    *px = blk.px0 + (q & 15);
    *py = blk.py0 + (q >> 4);
    return (*px < a.clip_x1) && (*py < a.clip_y1);
}

__global__ __launch_bounds__(256) void k_dqn_frame_begin(const DqnLaunch a) {
    const int rid = blockIdx.x * 256 + threadIdx.x;  // pixel slot
    if (rid >= a.rays.n_pix) return;
    int px, py;
    const bool valid = ray_pixel(a, rid, &px, &py);
    a.rays.pix[rid] = valid ? (uint32_t)py * (uint32_t)a.width + (uint32_t)px : 0u;
    st3(a.rays.total, rid, make3(0.0f, 0.0f, 0.0f));
}

// Ray::sample_ray_through_pixel's direction for the jittered pixel position (x, y)
__device__ __forceinline__ f3 dqn_camera_dir(const DqnLaunch& a, float x, float y) {
    const f3 dir = normalize(make3(x - (float)a.width / 2.0f, y - (float)a.height / 2.0f, (float)a.height));
    const float w = 1.0f;
    f3 r;
    r.x = (a.cos_y * dir.x + 0.0f * dir.y) + (-a.sin_y * dir.z + 0.0f * w);
    r.y = (0.0f * dir.x + 1.0f * dir.y) + (0.0f * dir.z + 0.0f * w);
    r.z = (a.sin_y * dir.x + 0.0f * dir.y) + (a.cos_y * dir.z + 0.0f * w);
    const float rw = (0.0f * dir.x + 0.0f * dir.y) + (0.0f * dir.z + 1.0f * w);
    f3 d;
    d.x = (1.0f * r.x + 0.0f * r.y) + (0.0f * r.z + 0.0f * rw);
    d.y = (0.0f * r.x + a.cos_x * r.y) + (a.sin_x * r.z + 0.0f * rw);
    d.z = (0.0f * r.x + -a.sin_x * r.y) + (a.cos_x * r.z + 0.0f * rw);
    return d;
}

// the trace's LDS: MF > 0 the filter's per-wave scratch, MF < 0 the BVH stacks (a column per lane)
__host__ __device__ constexpr int dqn_lds_floats(int mf) {
    return mf > 0 ? 4 * kMfWaveFloats : (mf < 0 ? kBvhMaxDepth * 256 : 1);
}
template <int MF>
__device__ __forceinline__ float* dqn_lane_ws(float* s) {
    return MF < 0 ? s + threadIdx.x : s + ((int)threadIdx.x >> 6) * kMfWaveFloats;
}

// initialise_ray + the first trace_ray (bounce 0: no Q evaluation)
#ifndef RT_MF_DQN_WAVES
#define RT_MF_DQN_WAVES 4  // occupancy floor of the MF variants
#endif
template <int MF>
__global__ __launch_bounds__(256, MF > 0 ? RT_MF_DQN_WAVES : 1) void k_dqn_camera(const DqnLaunch a) {
    __shared__ float s_mfw[dqn_lds_floats(MF)];
    const int rid = blockIdx.x * 256 + threadIdx.x;
    bool keep = false;
    unsigned casts = 0;
    bool valid = false;
    f3 d = make3(0.0f, 0.0f, 1.0f), tp = make3(0.0f, 0.0f, 0.0f);
    if (rid < a.rays.n) {
        const int slot = rid / a.rays.n_pix, pi = rid - slot * a.rays.n_pix;
        const int sample = a.rays.s0 + slot;
        int px, py;
        valid = ray_pixel(a, pi, &px, &py);
        tp = make3(valid ? 1.0f : 0.0f, valid ? 1.0f : 0.0f, valid ? 1.0f : 0.0f);
        if (valid) {
            float r1, r2;
            draw2(a.rays.pix[pi], (uint32_t)sample, 0u, a.seed_lo, a.seed_hi, &r1, &r2);
            const float x = (float)px + r1, y = (float)py + r2;
            d = dqn_camera_dir(a, x, y);
            casts = 1;
        }
    }
    f3 loc;
    int tri = 0;
    keep = dqn_trace<MF>(a, make3(a.cam_x, a.cam_y, a.cam_z), d, valid, dqn_lane_ws<MF>(s_mfw),
                         &loc, &tri, &tp);
    if (rid < a.rays.n) {
        if (keep) {
            st3(a.rays.loc, rid, loc);
            a.rays.tri[rid] = tri;
        }
        st3(a.rays.tp, rid, tp);
    }
    list_append(keep, rid, a.rays.list[0], a.rays.count + 0);
    const unsigned tot = wave_sum_u(casts);
    if ((threadIdx.x & 63) == 0 && tot) atomicAdd(a.rays.casts, (unsigned long long)tot);
}

// one bounce >= 1 for the rays of list[cur]: sample (Q already in a.rays.q), trace
// FUSED: the cell was chosen by k_dqn_mlp<MT, true> (q[i] = its index bits, q[ldq + i] = qd)
#ifndef RT_DQN_CT_WAVES
#define RT_DQN_CT_WAVES 4  // occupancy floor of the table-route bounce kernel (archway 1024^2 x 16: 4 / 6 / 8 waves 375.5 / 417.7 / 416.3 ms per frame)
#endif
template <int MF, bool FUSED = false, bool QB = false, bool CT = false>
__global__ __launch_bounds__(256, CT ? RT_DQN_CT_WAVES : (MF > 0 ? RT_MF_DQN_WAVES : 1)) void k_dqn_bounce(const DqnLaunch a, int bounce) {
    __shared__ float s_mfw[dqn_lds_floats(MF)];
    const int cur = (bounce - 1) & 1, nxt = bounce & 1;
    const int i = blockIdx.x * 256 + threadIdx.x;
    const int n_act = a.rays.count[cur];
    if ((int)(blockIdx.x * 256) >= n_act) return;  // uniform
    bool keep = false;
    unsigned casts = 0;
    int rid = 0;
    bool want = false;  // the lane casts a ray (wave-level filter below)
    f3 pos = make3(0.0f, 0.0f, 0.0f), dir = make3(0.0f, 0.0f, 1.0f), tp = make3(0.0f, 0.0f, 0.0f);
    f3 loc = pos;
    int ntri = 0;
    if (i < n_act) {
        rid = a.rays.list[cur][i];
        const int slot = rid / a.rays.n_pix;
        const int sample = a.rays.s0 + slot;
        const uint32_t pixid = a.rays.pix[rid - slot * a.rays.n_pix];
        const int tri = a.rays.tri[rid];
        pos = ld3(a.rays.loc, rid);
        tp = ld3(a.rays.tp, rid);
        const float4 N4 = a.scene.shade[tri * kShadeF4 + 0];
        const float4 T4 = a.scene.shade[tri * kShadeF4 + 1];
        const float4 B4 = a.scene.shade[tri * kShadeF4 + 2];
        const SampleOut so =
            FUSED ? sample_finish(__float_as_int(a.rays.q[i]), a.rays.q[(size_t)a.rays.ldq + i], make3(N4.x, N4.y, N4.z),
                                  make3(T4.x, T4.y, T4.z), make3(B4.x, B4.y, B4.z), pos,
                                  philox_shared(pixid, (uint32_t)sample, 1u + (uint32_t)bounce, a.seed_lo, a.seed_hi),
                                  &tp, true)
                  : sample_from_q<false, QB>(a.rays.q + i, (size_t)a.rays.ldq, make3(N4.x, N4.y, N4.z), make3(T4.x, T4.y, T4.z),
                                  make3(B4.x, B4.y, B4.z), pos, pixid, (uint32_t)sample,
                                  1u + (uint32_t)bounce, a.seed_lo, a.seed_hi, &tp, true);
        casts = 1;
        loc = pos;
        ntri = tri;
        if (so.action >= 0) {
            want = true;
            dir = so.dir;
        } else {
            // zero direction: the reference's ray is NaN and hits nothing
            tp = make3(tp.x * a.env_light, tp.y * a.env_light, tp.z * a.env_light);
        }
    }
    keep = dqn_trace<MF, true, CT>(a, pos, dir, want, dqn_lane_ws<MF>(s_mfw), &loc, &ntri, &tp, want ? ntri : -1);
    if (i < n_act) {
        if (keep) {
            st3(a.rays.loc, rid, loc);
            a.rays.tri[rid] = ntri;
        }
        st3(a.rays.tp, rid, tp);
    }
    list_append(keep, rid, a.rays.list[nxt], a.rays.count + nxt);
    const unsigned tot = wave_sum_u(casts);
    if ((threadIdx.x & 63) == 0 && tot) atomicAdd(a.rays.casts, (unsigned long long)tot);
}

// update_total_throughput (nn_rendering_helpers.cu:143-156)
__global__ __launch_bounds__(256) void k_dqn_accumulate(const DqnLaunch a) {
    const int pi = blockIdx.x * 256 + threadIdx.x;
    if (pi >= a.rays.n_pix) return;
    f3 t = ld3(a.rays.total, pi);
    for (int rid = pi; rid < a.rays.n; rid += a.rays.n_pix) {  // slots in sample order
        const f3 p = ld3(a.rays.tp, rid);
        t = make3(t.x + p.x, t.y + p.y, t.z + p.z);
    }
    st3(a.rays.total, pi, t);
}

// update_device_buffer (nn_rendering_helpers.cu:159-172): total / SPP into the tile output
__global__ __launch_bounds__(256) void k_dqn_finish(const DqnLaunch a) {
    const int rid = blockIdx.x * 256 + threadIdx.x;  // pixel slot
    if (rid >= a.rays.n_pix) return;
    int px, py;
    if (!ray_pixel(a, rid, &px, &py)) return;
    const BlockDesc blk = a.blocks[rid >> 8];
    const int q = rid & 255;
    const f3 t = ld3(a.rays.total, rid);
    const float fs = (float)a.spp;
    float* dst = a.out + ((size_t)(blk.oy0 + (q >> 4)) * (size_t)a.out_pitch + (size_t)(blk.ox0 + (q & 15))) * 3;
    dst[0] = t.x / fs;
    dst[1] = t.y / fs;
    dst[2] = t.z / fs;
}

__global__ __launch_bounds__(256) void k_dqn_sample_only(const DeviceScene s, float* q, const float* loc,
                                                         const int32_t* tri, const uint32_t* pix, int n,
                                                         int sample, int bounce, uint32_t k0, uint32_t k1,
                                                         float* tp, float* dir_out, int32_t* action) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const int t = tri[i];
    const float4 N4 = s.shade[t * kShadeF4 + 0];
    const float4 T4 = s.shade[t * kShadeF4 + 1];
    const float4 B4 = s.shade[t * kShadeF4 + 2];
    f3 tpv = ld3(tp, i);
    const SampleOut so = sample_from_q<true>(q + (size_t)i * kDqnActions, 1, make3(N4.x, N4.y, N4.z),
                                       make3(T4.x, T4.y, T4.z), make3(B4.x, B4.y, B4.z), ld3(loc, i),
                                       pix[i], (uint32_t)sample, 1u + (uint32_t)bounce, k0, k1, &tpv, true);
    st3(tp, i, tpv);
    st3(dir_out, i, so.dir);
    action[i] = so.action;
}

// ---------------------------------------------------------------------------
// Neural-Q training renderer (NeuralQPathtracer::render_frame,
// GPU/deep_learning/neural_q_pathtracer.cu:226-600): every ray of the frame steps through
// every bounce of a sample (terminated rays are restarted on the scene and keep feeding
// the learning rule), the network being trained between bounces (rt_train.hip).
// Philox events (pixel id, sample, event, counter): 0 camera jitter, 1 + b the Q-weighted
// sampler of bounce b, kNqEvGreedy + b the epsilon draw / exploration cell and jitters,
// kNqEvRestart + b and kNqEvRestartPos + b a restart's surface and position.
// ---------------------------------------------------------------------------
constexpr uint32_t kNqEvGreedy = 0x1000u, kNqEvRestart = 0x2000u, kNqEvRestartPos = 0x3000u;
constexpr float kThroughputThreshold = 0.0001f;  // THROUGHPUT_THRESHOLD (constants/monte_carlo_settings.h:11)

// initialise_ray (neural_q_pathtracer.cu:604-643)
__global__ __launch_bounds__(256) void k_nq_init(const DqnLaunch a, const NqRays r, int sample) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= r.n) return;
    const int px = i % a.width, py = i / a.width;
    float r1, r2;
    draw2((uint32_t)i, (uint32_t)sample, 0u, a.seed_lo, a.seed_hi, &r1, &r2);
    const f3 d = dqn_camera_dir(a, (float)px + r1, (float)py + r2);
    const f3 cam = make3(a.cam_x, a.cam_y, a.cam_z);
    st3(r.loc, i, cam);
    st3(r.prev, i, cam);
    st3(r.dir, i, d);
    st3(r.tp, i, make3(1.0f, 1.0f, 1.0f));
    r.tri[i] = -1;
    r.state[i] = 0u;
    r.reward[i] = 0.0f;
    r.discount[i] = 1.0f;
    r.bounces[i] = (uint32_t)a.max_bounces;
    r.action[i] = 0;
    r.pix[i] = (uint32_t)i;
}

// sample_batch_ray_directions_epsilon_greedy (nn_rendering_helpers.cu:330-389): with
// probability 1 - eps importance_sample_direction on Q (sample_from_q; a ray whose Q admits
// no cell keeps its direction, the reference's loop finding nothing), else a uniformly
// chosen cell, (u - 0.0001) * 144, jittered (sample_ray_for_grid_index, :4-35:
// throughput * cos / RHO).  q: [n][144], overwritten with Q * cos on the greedy rows.
__global__ __launch_bounds__(256) void k_nq_sample(const DqnLaunch a, const NqRays r, float* q, float eps,
                                                   int sample, int bounce) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= r.n) return;
    const int tri = r.tri[i];
    const float4 N4 = a.scene.shade[tri * kShadeF4 + 0];
    const float4 T4 = a.scene.shade[tri * kShadeF4 + 1];
    const float4 B4 = a.scene.shade[tri * kShadeF4 + 2];
    const f3 N = make3(N4.x, N4.y, N4.z), T = make3(T4.x, T4.y, T4.z), B = make3(B4.x, B4.y, B4.z);
    const f3 pos = ld3(r.loc, i);
    f3 tp = ld3(r.tp, i);
    const bool live = r.state[i] == 0u;
    uint32_t o[4];
    philox4x32_10(r.pix[i], (uint32_t)sample, kNqEvGreedy + (uint32_t)bounce, 0u, a.seed_lo, a.seed_hi, o);
    const float rv = u01_oc(o[0]);
    if (rv > eps) {
        const SampleOut so = sample_from_q<true>(q + (size_t)i * kDqnActions, 1, N, T, B, pos, r.pix[i], (uint32_t)sample,
                                           1u + (uint32_t)bounce, a.seed_lo, a.seed_hi, &tp, live);
        if (so.action >= 0) {
            st3(r.dir, i, so.dir);
            r.action[i] = so.action;
        } else {
            r.action[i] = 0;
        }
    } else {
        const float u = u01_oc(o[1]) - 0.0001f;
        int idx = (int)(u * (float)kDqnActions);
        idx = idx < 0 ? 0 : (idx > kDqnActions - 1 ? kDqnActions - 1 : idx);
        const int gx = idx / kDqnGrid, gy = idx - gx * kDqnGrid;
        const f3 d = grid_direction((float)gx + u01(o[2]), (float)gy + u01(o[3]), N, T, B, pos);
        if (live) {
            const float c = dot(N, d);
            tp = make3((tp.x * c) / kRho, (tp.y * c) / kRho, (tp.z * c) / kRho);
        }
        st3(r.dir, i, d);
        r.action[i] = idx;
    }
    st3(r.tp, i, tp);
}

// trace_ray (neural_q_pathtracer.cu:646-745): Ray(pos + dir * 1e-5, dir), GPU hit rule;
// miss: reward 0, terminal; light: reward = its luminance x 200, terminal; surface: the
// new state, discount = the material's luminance.  Throughputs and path lengths change
// only for paths still contributing (state 0).  The position before the trace is the
// learning rule's S_t.  BVH: the scene's exact BVH (large scenes), a stack column per lane.
template <bool BVH>
__global__ __launch_bounds__(256) void k_nq_trace(const DqnLaunch a, const NqRays r, int bounce) {
    __shared__ int s_stk[BVH ? kBvhMaxDepth * 256 : 1];
    const int i = blockIdx.x * 256 + threadIdx.x;
    unsigned casts = 0;
    if (i < r.n) {
        const f3 pos = ld3(r.loc, i), dir = ld3(r.dir, i);
        st3(r.prev, i, pos);
        const f3 o = make3(pos.x + dir.x * kEps, pos.y + dir.y * kEps, pos.z + dir.z * kEps);
        const f3 d = normalize(dir);
        Hit h;
        if constexpr (BVH)
            h = closest_hit_bvh<1, 256>(a.scene, o, d, a.t_scale, s_stk + threadIdx.x);
        else
            h = closest_hit_sel<1>(a.scene, a.use_filter, o, d, a.t_scale);
        casts = 1;
        const uint32_t st = r.state[i];
        f3 tp = ld3(r.tp, i);
        if (h.tri < 0 || h.tri >= a.scene.n_surf) {
            const bool light = h.tri >= 0;
            r.reward[i] = light ? r.tri_lum[h.tri] * 200.0f : 0.0f;
            r.discount[i] = 0.0f;
            if (st == 0u) {
                if (light) {
                    const float4 e = a.scene.shade[h.tri * kShadeF4 + 3];
                    tp = make3(tp.x * e.x, tp.y * e.y, tp.z * e.z);
                } else {
                    tp = make3(tp.x * a.env_light, tp.y * a.env_light, tp.z * a.env_light);
                }
                r.bounces[i] = (uint32_t)bounce;
            }
            r.state[i] = 1u;
            r.terminal[i] = 1;
        } else {
            const float Dx = d.x * a.t_scale, Dy = d.y * a.t_scale, Dz = d.z * a.t_scale;
            st3(r.loc, i, make3(o.x + h.t * Dx, o.y + h.t * Dy, o.z + h.t * Dz));
            r.tri[i] = h.tri;
            if (st == 0u) {
                const float4 c = a.scene.shade[h.tri * kShadeF4 + 3];  // diffuse_c / pi
                tp = make3(tp.x * c.x, tp.y * c.y, tp.z * c.z);
                r.flag[0] = 0;  // a path still bounces (a vector store; every writer stores 0)
            }
            r.reward[i] = 0.0f;
            r.discount[i] = r.tri_lum[h.tri];
            r.terminal[i] = 0;
        }
        st3(r.tp, i, tp);
    }
    const unsigned tot = wave_sum_u(casts);
    if ((threadIdx.x & 63) == 0 && tot) atomicAdd(&r.stats[2], (unsigned long long)tot);
}

// sample_random_scene_pos_for_terminated_rays (nn_rendering_helpers.cu:241-277): a random
// surface, floor(surfaces_count * u), a point on it by rejection (Triangle::
// sample_position_on_plane), stored with its y and z exchanged as the reference stores
// it (ray_locations[i*3+2] = pos.y, [i*3+1] = pos.z); its normal; state 2.
__global__ __launch_bounds__(256) void k_nq_restart(const DqnLaunch a, const NqRays r, int sample, int bounce) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= r.n || r.state[i] != 1u) return;
    uint32_t o[4];
    philox4x32_10(r.pix[i], (uint32_t)sample, kNqEvRestart + (uint32_t)bounce, 0u, a.seed_lo, a.seed_hi, o);
    int s = (int)((float)a.scene.n_surf * u01_oc(o[0]));
    s = s < a.scene.n_surf ? s : a.scene.n_surf - 1;
    const float* v = r.surf_v + (size_t)s * 9;
    float a1, a2;
    uint32_t attempt = 0;
    do {
        philox4x32_10(r.pix[i], (uint32_t)sample, kNqEvRestartPos + (uint32_t)bounce, attempt++, a.seed_lo, a.seed_hi,
                      o);
        a1 = u01_oc(o[0]);
        a2 = u01_oc(o[1]);
    } while (a1 + a2 > 1.0f && attempt < 64u);
    if (a1 + a2 > 1.0f) {  // (probability 2^-64: keep the point on the triangle)
        a1 = 1.0f - a1;
        a2 = 1.0f - a2;
    }
    float p[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) p[c] = (v[c] + a1 * (v[3 + c] - v[c])) + a2 * (v[6 + c] - v[c]);
    st3(r.loc, i, make3(p[0], p[2], p[1]));
    r.tri[i] = s;
    r.state[i] = 2u;
}

// end of a sample: update_total_throughput (every ray's throughput, as the reference adds
// it), sum_path_lengths and sum_zero_contribution_light_paths (nn_rendering_helpers.cu)
__global__ __launch_bounds__(256) void k_nq_end_sample(const DqnLaunch a, const NqRays r) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    unsigned b = 0, z = 0;
    if (i < r.n) {
        const f3 tp = ld3(r.tp, i);
        const f3 t = ld3(r.total, i);
        st3(r.total, i, make3(t.x + tp.x, t.y + tp.y, t.z + tp.z));
        b = r.bounces[i];
        // every channel below THROUGHPUT_THRESHOLD (sum_zero_contribution_light_paths,
        // nn_rendering_helpers.cu:556-568; the Expected-SARSA count tests the channels' mean,
        // reinforcement_path_tracing.cu:36-42); a NaN channel is not below it
        z = (tp.x < kThroughputThreshold && tp.y < kThroughputThreshold && tp.z < kThroughputThreshold) ? 1u : 0u;
    }
    const unsigned sb = wave_sum_u(b), sz = wave_sum_u(z);
    if ((threadIdx.x & 63) == 0) {
        atomicAdd(&r.stats[0], (unsigned long long)sb);
        atomicAdd(&r.stats[1], (unsigned long long)sz);
    }
}

// update_device_buffer (nn_rendering_helpers.cu:159-172): the frame = total / SPP
__global__ __launch_bounds__(256) void k_nq_image(const DqnLaunch a, const NqRays r, float* out, int spp) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= r.n) return;
    const f3 t = ld3(r.total, i);
    const float fs = (float)spp;
    st3(out, i, make3(t.x / fs, t.y / fs, t.z / fs));
}

}  // namespace

static hipError_t launch_dqn_mlp_fused(const DqnNet& net, const float* loc, const int32_t* list,
                                       const int32_t* count, int max_rows, float* q, int ldq, const MlpSample* smp,
                                       bool qb, hipStream_t stream);

hipError_t launch_dqn_mlp(const DqnNet& net, const float* loc, const int32_t* list, const int32_t* count,
                          int max_rows, float* q, int ldq, hipStream_t stream) {
    return launch_dqn_mlp_fused(net, loc, list, count, max_rows, q, ldq, nullptr, false, stream);
}

// fused (smp != nullptr): the sampler runs in the forward kernel (k_dqn_mlp<MT, true>)
static hipError_t launch_dqn_mlp_fused(const DqnNet& net, const float* loc, const int32_t* list, const int32_t* count,
                                int max_rows, float* q, int ldq, const MlpSample* smp, bool qb, hipStream_t stream) {
    if (max_rows <= 0) return hipSuccess;
    KernelTimer kt(KT_DQN_MLP, stream);
    // this file's weight-streaming kernel; the weight-stationary one (rt_dqn_ws.hip) when
    // asked (rt_dqn_set_mlp) and the network has the 200-300-200 shape
    if (net.mlp_mode == kMlpStationary && dqn_mlp_ws_fits(net)) {
        int dev = 0, n_cu = 0;
        hipError_t e = hipGetDevice(&dev);
        if (e == hipSuccess) e = hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev);
        if (e != hipSuccess) return e;
        return launch_dqn_mlp_ws(net, loc, list, count, max_rows, q, ldq, n_cu, qb, stream);
    }
    const int blocks = (max_rows + kTileM - 1) / kTileM;
    if (ldq != 0 && (ldq < blocks * kTileM || ldq % 4 != 0)) return hipErrorInvalidValue;
    if (smp != nullptr) {
        if constexpr (kFusedFits)
            hipLaunchKernelGGL((k_dqn_mlp<RT_MLP_MT, true>), dim3((unsigned)blocks), dim3(kMlpThreads), 0, stream, net,
                               loc, list, count, max_rows, q, ldq, *smp);
        else
            return hipErrorInvalidValue;
    } else if (qb && ldq != 0)
        hipLaunchKernelGGL((k_dqn_mlp<RT_MLP_MT, false, true>), dim3((unsigned)blocks), dim3(kMlpThreads), 0, stream, net,
                           loc, list, count, max_rows, q, ldq, MlpSample());
    else
        hipLaunchKernelGGL((k_dqn_mlp<RT_MLP_MT, false>), dim3((unsigned)blocks), dim3(kMlpThreads), 0, stream, net, loc,
                           list, count, max_rows, q, ldq, MlpSample());
    return hipGetLastError();
}

int dqn_mlp_tile_rows() { return kTileM; }

static unsigned ray_blocks(const DqnLaunch& a) { return (unsigned)((a.rays.n + 255) / 256); }
static unsigned pix_blocks(const DqnLaunch& a) { return (unsigned)((a.rays.n_pix + 255) / 256); }

hipError_t launch_dqn_frame_begin(const DqnLaunch& a, hipStream_t stream) {
    hipLaunchKernelGGL(k_dqn_frame_begin, dim3(pix_blocks(a)), dim3(256), 0, stream, a);
    return hipGetLastError();
}

#ifndef RT_MF_DQN
#define RT_MF_DQN 1  // 0: the casts on the fp32 filter (archway 512^2 x 16: 125.2 vs 120.9 ms, profiles/r3q)
#endif
// 64-triangle blocks of the matrix-core filter for this launch (0: the fp32 filter): the
// image present and the camera inside its origin bound (as launch_render_t); -1: the
// scene's exact BVH (large scenes, the launch view carries it)
static int dqn_mf(const DqnLaunch& a) {
    if (a.scene.bvh_nodes != nullptr) return -1;
    const float cb = a.scene.mf_bound;
    const bool mf = RT_MF_DQN && a.use_filter && a.scene.mf_frag != nullptr && a.t_scale > 0.0f &&
                    a.t_scale <= kFiltMaxTScale && fabsf(a.cam_x) <= cb && fabsf(a.cam_y) <= cb &&
                    fabsf(a.cam_z) <= cb;
    return mf ? (a.scene.n_tri <= 64 ? 1 : 4) : 0;
}

hipError_t launch_dqn_camera(const DqnLaunch& a, hipStream_t stream) {
    KernelTimer kt(KT_DQN_CAMERA, stream);
    switch (dqn_mf(a)) {
        case 1: hipLaunchKernelGGL(k_dqn_camera<1>, dim3(ray_blocks(a)), dim3(256), 0, stream, a); break;
        case 4: hipLaunchKernelGGL(k_dqn_camera<4>, dim3(ray_blocks(a)), dim3(256), 0, stream, a); break;
        case -1: hipLaunchKernelGGL(k_dqn_camera<-1>, dim3(ray_blocks(a)), dim3(256), 0, stream, a); break;
        default: hipLaunchKernelGGL(k_dqn_camera<0>, dim3(ray_blocks(a)), dim3(256), 0, stream, a); break;
    }
    return hipGetLastError();
}

#ifndef RT_DQN_QBF16
#define RT_DQN_QBF16 1  // the renderer's Q between the forward and the sampler in bf16 (0: fp32; archway 512^2 x 16: 110.7 vs 121.0 ms, profiles/r4c)
#endif
#ifndef RT_DQN_FUSED
#define RT_DQN_FUSED 0  // 1: the sampler inside k_dqn_mlp (measured slower: 143.9 vs 131.8 ms, archway 512^2 x 16)
#endif

hipError_t launch_dqn_bounce(const DqnLaunch& a, int bounce, hipStream_t stream) {
    const int cur = (bounce - 1) & 1;
    // the fused sampler: the streaming forward (the weight-stationary A/B kernel writes Q)
    const bool fused = RT_DQN_FUSED && kFusedFits && !(a.net.mlp_mode == kMlpStationary && dqn_mlp_ws_fits(a.net)) &&
                       a.net.N[3] == kDqnActions && a.rays.ldq >= 2;
    MlpSample smp;
    smp.pix = a.rays.pix;
    smp.n_pix = a.rays.n_pix;
    smp.s0 = a.rays.s0;
    smp.ev = 1u + (uint32_t)bounce;
    smp.k0 = a.seed_lo;
    smp.k1 = a.seed_hi;
    // the renderer's Q in bf16 (either forward kernel writes it)
    const bool qb = RT_DQN_QBF16 && !fused && a.net.N[3] == kDqnActions;
    hipError_t e = launch_dqn_mlp_fused(a.net, a.rays.loc, a.rays.list[cur], a.rays.count + cur, a.rays.n,
                                        a.rays.q, a.rays.ldq, fused ? &smp : nullptr, qb, stream);
    if (e != hipSuccess) return e;
    KernelTimer kt(KT_DQN_BOUNCE, stream);
    const dim3 grid(ray_blocks(a));
    const CtabDev& T = a.scene.ctab[1];
    const int mf = dqn_mf(a);
    const bool ct = RT_DQN_CTAB && qb && mf > 0 && T.masks != nullptr && T.bins == kCtabBins &&
                    T.graze_n == kCtabGraze && a.t_scale >= T.ts_min && T.words <= mf;
    if (ct) {
        if (mf == 1)
            hipLaunchKernelGGL((k_dqn_bounce<1, false, true, true>), grid, dim3(256), 0, stream, a, bounce);
        else
            hipLaunchKernelGGL((k_dqn_bounce<4, false, true, true>), grid, dim3(256), 0, stream, a, bounce);
        return hipGetLastError();
    }
    if (qb) {
        switch (dqn_mf(a)) {
            case 1: hipLaunchKernelGGL((k_dqn_bounce<1, false, true>), grid, dim3(256), 0, stream, a, bounce); break;
            case 4: hipLaunchKernelGGL((k_dqn_bounce<4, false, true>), grid, dim3(256), 0, stream, a, bounce); break;
            case -1: hipLaunchKernelGGL((k_dqn_bounce<-1, false, true>), grid, dim3(256), 0, stream, a, bounce); break;
            default: hipLaunchKernelGGL((k_dqn_bounce<0, false, true>), grid, dim3(256), 0, stream, a, bounce); break;
        }
        return hipGetLastError();
    }
    switch (dqn_mf(a) * 2 + (fused ? 1 : 0)) {
        case 2: hipLaunchKernelGGL((k_dqn_bounce<1, false>), grid, dim3(256), 0, stream, a, bounce); break;
        case 3: hipLaunchKernelGGL((k_dqn_bounce<1, true>), grid, dim3(256), 0, stream, a, bounce); break;
        case 8: hipLaunchKernelGGL((k_dqn_bounce<4, false>), grid, dim3(256), 0, stream, a, bounce); break;
        case 9: hipLaunchKernelGGL((k_dqn_bounce<4, true>), grid, dim3(256), 0, stream, a, bounce); break;
        case -2: hipLaunchKernelGGL((k_dqn_bounce<-1, false>), grid, dim3(256), 0, stream, a, bounce); break;
        case -1: hipLaunchKernelGGL((k_dqn_bounce<-1, true>), grid, dim3(256), 0, stream, a, bounce); break;
        case 1: hipLaunchKernelGGL((k_dqn_bounce<0, true>), grid, dim3(256), 0, stream, a, bounce); break;
        default: hipLaunchKernelGGL((k_dqn_bounce<0, false>), grid, dim3(256), 0, stream, a, bounce); break;
    }
    return hipGetLastError();
}

hipError_t launch_dqn_accumulate(const DqnLaunch& a, hipStream_t stream) {
    hipLaunchKernelGGL(k_dqn_accumulate, dim3(pix_blocks(a)), dim3(256), 0, stream, a);
    return hipGetLastError();
}

hipError_t launch_dqn_finish(const DqnLaunch& a, hipStream_t stream) {
    hipLaunchKernelGGL(k_dqn_finish, dim3(pix_blocks(a)), dim3(256), 0, stream, a);
    return hipGetLastError();
}

hipError_t launch_dqn_sample_only(const DeviceScene& s, const float* q, const float* loc, const int32_t* tri,
                                  const uint32_t* pix, int n, int sample, int bounce, uint32_t seed_lo,
                                  uint32_t seed_hi, float* tp, float* dir_out, int32_t* action,
                                  hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_dqn_sample_only, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, s,
                       const_cast<float*>(q), loc, tri, pix, n, sample, bounce, seed_lo, seed_hi, tp, dir_out,
                       action);
    return hipGetLastError();
}

static unsigned nq_blocks(const NqRays& r) { return (unsigned)((r.n + 255) / 256); }

hipError_t launch_nq_init(const DqnLaunch& a, const NqRays& r, int sample, hipStream_t stream) {
    hipLaunchKernelGGL(k_nq_init, dim3(nq_blocks(r)), dim3(256), 0, stream, a, r, sample);
    return hipGetLastError();
}
hipError_t launch_nq_sample(const DqnLaunch& a, const NqRays& r, float* q, float eps, int sample, int bounce,
                            hipStream_t stream) {
    hipLaunchKernelGGL(k_nq_sample, dim3(nq_blocks(r)), dim3(256), 0, stream, a, r, q, eps, sample, bounce);
    return hipGetLastError();
}
hipError_t launch_nq_trace(const DqnLaunch& a, const NqRays& r, int bounce, hipStream_t stream) {
    if (a.scene.bvh_nodes != nullptr)
        hipLaunchKernelGGL(k_nq_trace<true>, dim3(nq_blocks(r)), dim3(256), 0, stream, a, r, bounce);
    else
        hipLaunchKernelGGL(k_nq_trace<false>, dim3(nq_blocks(r)), dim3(256), 0, stream, a, r, bounce);
    return hipGetLastError();
}
hipError_t launch_nq_restart(const DqnLaunch& a, const NqRays& r, int sample, int bounce, hipStream_t stream) {
    hipLaunchKernelGGL(k_nq_restart, dim3(nq_blocks(r)), dim3(256), 0, stream, a, r, sample, bounce);
    return hipGetLastError();
}
hipError_t launch_nq_end_sample(const DqnLaunch& a, const NqRays& r, hipStream_t stream) {
    hipLaunchKernelGGL(k_nq_end_sample, dim3(nq_blocks(r)), dim3(256), 0, stream, a, r);
    return hipGetLastError();
}
hipError_t launch_nq_image(const DqnLaunch& a, const NqRays& r, float* out, int spp, hipStream_t stream) {
    hipLaunchKernelGGL(k_nq_image, dim3(nq_blocks(r)), dim3(256), 0, stream, a, r, out, spp);
    return hipGetLastError();
}

}  // namespace rt
