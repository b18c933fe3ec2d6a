// rt_sarsa.hip — Expected-SARSA radiance-volume path tracer (BASELINE config 3).
//
// Reference: GPU/path_tracing/reinforcement_path_tracing.cu:6-120 (render
// kernel, per-frame distribution update), GPU/radiance_volumes/radiance_map.cu
// (:90-146 sampling + TD update dispatch, :149-203 nearest volume),
// GPU/radiance_volumes/radiance_volume.cu (:93-112 expected_sarsa_irradiance,
// :148-188 update_radiance_distribution, :191-244 CDF sampling,
// :282-307 temporal_difference_update, irradiance estimate).
//
// Determinism: the reference updates the Q-table racily while
// it renders (non-atomic read-modify-write + atomicExch).  Here a frame reads
// the Q-table, irradiance and CDFs of the previous frame, and every TD target
// is added to a per-(volume, sector) fixed-point sum (2^-32 units, integer
// atomics: order-independent) with a visit count; k_sarsa_apply then folds
// the frame's targets into Q in closed form — the running mean that
// alpha = 1/(1 + visits) produces — and rebuilds the CDFs.  Same frames, same
// seed: bit-identical Q-table and image on any GPU count, and against oracle/.
#include <float.h>

#include "rt_trace.hpp"

// A/B knobs (timing / statistics builds only; all but SCAN_STATS change results):
// RT_SARSA_NO_TD drops the TD atomics, RT_SARSA_NO_KD replaces the nearest-volume
// search by volume 0, RT_SARSA_FIRST_ONLY takes the first candidate of the grid list
// (same normal class: frame-0 paths keep their statistics), RT_SARSA_SCAN_STATS
// counts the grid scan steps (4 candidates each) in grid_fallbacks
#ifndef RT_SARSA_NO_TD
#define RT_SARSA_NO_TD 0
#endif
#ifndef RT_SARSA_PROF
#define RT_SARSA_PROF 0  // 1: k_sarsa_render_pq sums per-phase s_memtime cycles into SarsaMap::prof (timing builds)
#endif
#ifndef RT_SARSA_NO_KD
#define RT_SARSA_NO_KD 0
#endif
#ifndef RT_SARSA_SCAN_STATS
#define RT_SARSA_SCAN_STATS 0
#endif
#ifndef RT_SARSA_FIRST_ONLY
#define RT_SARSA_FIRST_ONLY 0
#endif
#ifndef RT_SARSA_NO_FALLBACK  // grid answer even where the KD walk is needed (timing only)
#define RT_SARSA_NO_FALLBACK 0
#endif

namespace rt {

namespace {

constexpr float kGridRhoS = 1.0f / ((float)kGridRes * (float)kGridRes);             // GRID_RHO
constexpr float kRadianceThreshold = (1.f / ((float)kGridRes * (float)kGridRes)) * 0.8f;  // RADIANCE_THRESHOLD
constexpr float kIrrScale = (2.f * kPi) / ((float)(kGridRes * kGridRes));          // get_irradiance_estimate
constexpr float kThroughputThreshold = 0.0001f;  // THROUGHPUT_THRESHOLD (constants/monte_carlo_settings.h:11)

__device__ __forceinline__ float len3(float x, float y, float z) { return sqrtf((x * x + y * y) + z * z); }

// find_closest_radiance_volume_iterative (radiance_map.cu:149-203): explicit-stack
// KD descent; a far child is visited when delta^2 < MAX_DIST; leaves need an
// identical normal; the search starts from volume 0 at the distance of element 0's
// position (the origin for an internal root).  The stack lives in LDS, one column per
// lane of the wave's own block (st[k * 64], kd_stack_of); its depth is bounded by the
// tree depth (host-checked).
// the k-d stack column of this lane: each wave owns a contiguous kKdStack x 64 block (the
// exact phase of the matrix-core filter reuses it between searches: k_sarsa_render<MF>)
__device__ __forceinline__ int* kd_stack_of(int* kd_stack) {
    return kd_stack + ((int)threadIdx.x >> 6) * (kKdStack * 64) + ((int)threadIdx.x & 63);
}

__device__ int sarsa_nearest(const SarsaMap& m, f3 pos, f3 nrm, int* st) {
    if (RT_SARSA_NO_KD) return 0;
    const uint4* __restrict__ kd = m.kd4;
    int best = 0;
    float best_d = len3(pos.x - m.root_x, pos.y - m.root_y, pos.z - m.root_z);
    st[0] = 0;
    int sp = 1;
    while (sp > 0) {
        --sp;
        const uint4 nd = kd[st[sp * 64]];
        if (nd.w != 0xFFFFFFFFu) {  // leaf
            const float d = len3(__uint_as_float(nd.x) - pos.x, __uint_as_float(nd.y) - pos.y,
                                 __uint_as_float(nd.z) - pos.z);
            if (d < best_d) {
                const float4 n4 = m.vol_frame[nd.w * 3];
                if (nrm.x == n4.x && nrm.y == n4.y && nrm.z == n4.z) {
                    best = (int)nd.w;
                    best_d = d;
                }
            }
        } else {
            const float pc = (nd.z == 0u) ? pos.x : ((nd.z == 1u) ? pos.y : pos.z);
            const float delta = pc - __uint_as_float(nd.x);
            const bool near_split = (delta * delta) < m.max_dist;
            const int left = (int)nd.y;
            const int nearc = delta < 0.0f ? left : left + 1;
            if (near_split) st[(sp++) * 64] = (left + left + 1) - nearc;
            st[(sp++) * 64] = nearc;
        }
    }
    return best;
}

// The same volume as sarsa_nearest, from the per-normal grid when that is provably
// equal (rt_sarsa_host.cpp NearestGrid): the nearest same-normal volume among the
// 3x3x3 cells around pos, if its distance is below grid_h (so the KD walk visits it)
// and no other candidate has the same float distance (the KD walk's order would
// break the tie).  cls: normal class of the hit surface (-1: no volume has its
// normal, the KD walk keeps volume 0).  Otherwise kNeedWalk: the KD walk decides
// (sarsa_resolve_walks).
constexpr int kNeedWalk = -2;  // sarsa_nearest_grid: only the KD walk decides this query

#ifndef RT_SARSA_HEAD
#define RT_SARSA_HEAD 1  // the cell's range and first three candidates as one 64-B record (0: range, then leaves)
#endif
#ifndef RT_SARSA_TRIREC
#define RT_SARSA_TRIREC 1  // 0: class -> grid descriptor -> cell start / end as four dependent loads (A/B)
#endif
// G, D: the class grid's origin (w: first cell, bits) and cells per axis
__device__ int sarsa_nearest_grid_gd(const SarsaMap& m, float4 G, int4 D, f3 pos) {
    {
        const float ic = m.grid_inv_cs;
        // padded cell of the query (rt_sarsa_host.cpp grid_cell): its list holds every
        // class volume of the 3x3x3 neighbourhood
        const int ix = (int)floorf(fminf(fmaxf((pos.x - G.x) * ic, 0.0f), (float)(D.x - 1)));
        const int iy = (int)floorf(fminf(fmaxf((pos.y - G.y) * ic, 0.0f), (float)(D.y - 1)));
        const int iz = (int)floorf(fminf(fmaxf((pos.z - G.z) * ic, 0.0f), (float)(D.z - 1)));
        const uint32_t c = __float_as_uint(G.w) + (uint32_t)((iz * D.y + iy) * D.x + ix);
        uint32_t k0, e;
#if RT_SARSA_HEAD
        const float4* hp = m.cell_head + (size_t)c * 4;
        const float4 h0 = hp[0];
        const float4 H[3] = {hp[1], hp[2], hp[3]};
        k0 = __float_as_uint(h0.x);
        e = __float_as_uint(h0.y);
#else
        if (RT_SARSA_TRIREC) {
            const uint2 r = m.cell_range[c];
            k0 = r.x;
            e = r.y;
        } else {
            k0 = m.cell_start[c];
            e = m.cell_start[c + 1];
        }
#endif
        // The list is sorted by distance to the cell centre C: d(q, L) >= d(C, L) - d(q, C),
        // so once d(C, L) exceeds best + d(q, C) (with a 2^-12 margin: such a candidate's
        // float distance is strictly above the best, no tie either) no later one can win.
        const float cx = G.x + ((float)ix + 0.5f) * m.grid_cs;
        const float cy = G.y + ((float)iy + 0.5f) * m.grid_cs;
        const float cz = G.z + ((float)iz + 0.5f) * m.grid_cs;
        const float qx = pos.x - cx, qy = pos.y - cy, qz = pos.z - cz;
        const float dq = __builtin_sqrtf((qx * qx + qy * qy) + qz * qz);
        float b1 = INFINITY, b2 = INFINITY;
        int bv = -1;
#if RT_SARSA_SCAN_STATS  // statistics builds only: grid_fallbacks counts scan steps instead
        uint32_t steps = 0;
#endif
#if RT_SARSA_FIRST_ONLY  // timing only: the first listed candidate (wrong volumes)
        if (k0 < e) return __float_as_int(m.grid_leaf[k0].w);
#endif
        uint32_t kb = k0;
#if RT_SARSA_HEAD
        // the cell record's own first three candidates (no break test before the first
        // candidates: the limit is infinite there); the scan goes on from the fourth.  Where
        // the scan's batches start does not change its answer: the break only skips
        // candidates that can neither win nor tie.
#pragma unroll
        for (int u = 0; u < 3; ++u) {
            const float dx = H[u].x - pos.x, dy = H[u].y - pos.y, dz = H[u].z - pos.z;
            const float s = (dx * dx + dy * dy) + dz * dz;  // len3's sum
            if (k0 + (uint32_t)u < e) {
                if (s < b1) {
                    b2 = b1;
                    b1 = s;
                    bv = __float_as_int(H[u].w);
                } else if (s < b2) {
                    b2 = s;
                }
            }
        }
        kb = k0 + 3;
#endif
        for (uint32_t k = kb; k < e; k += 4) {  // 4 candidate loads in flight
#if RT_SARSA_SCAN_STATS
            ++steps;
#endif
            float4 L[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) L[u] = m.grid_leaf[min(k + (uint32_t)u, e - 1u)];
            {
                const float lim = (__builtin_sqrtf(b1) + dq) * (1.0f + 0x1p-12f) + 1e-6f;
                const float ex = L[0].x - cx, ey = L[0].y - cy, ez = L[0].z - cz;
                if ((ex * ex + ey * ey) + ez * ez > lim * lim) break;
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const float dx = L[u].x - pos.x, dy = L[u].y - pos.y, dz = L[u].z - pos.z;
                const float s = (dx * dx + dy * dy) + dz * dz;  // len3's sum
                if (k + (uint32_t)u < e) {
                    if (s < b1) {
                        b2 = b1;
                        b1 = s;
                        bv = __float_as_int(L[u].w);
                    } else if (s < b2) {
                        b2 = s;
                    }
                }
            }
        }
#if RT_SARSA_SCAN_STATS
        atomicAdd(m.grid_fallbacks, (unsigned long long)steps);
#endif
        const float d = sqrtf(b1);
        if (bv >= 0 && d < m.grid_h && sqrtf(b2) != d) {
            const float d0 = len3(pos.x - m.root_x, pos.y - m.root_y, pos.z - m.root_z);
            return d < d0 ? bv : 0;
        }
        if (m.grid_fallbacks != nullptr) atomicAdd(m.grid_fallbacks, 1ull);
        if (RT_SARSA_NO_FALLBACK) return bv >= 0 ? bv : 0;
    }
    return kNeedWalk;
}

// cls: normal class of the query (-1: no volume has its normal -- the KD walk keeps volume 0)
__device__ int sarsa_nearest_grid(const SarsaMap& m, int cls, f3 pos, f3 nrm) {
    (void)nrm;
    if (RT_SARSA_NO_KD) return 0;
    if (cls < 0) return 0;
    return sarsa_nearest_grid_gd(m, m.class_org[cls], m.class_dim[cls], pos);
}

// the same for a hit on surface tri: its class's grid descriptor in one per-surface record
// (two independent loads instead of the class, then its descriptor)
__device__ int sarsa_nearest_grid_tri(const SarsaMap& m, int tri, f3 pos, f3 nrm) {
    if (RT_SARSA_NO_KD) return 0;
    if (!RT_SARSA_TRIREC) return sarsa_nearest_grid(m, m.tri_class[tri], pos, nrm);
    const float4 G = m.tri_grid[2 * tri];
    const float4 Df = m.tri_grid[2 * tri + 1];
    const int4 D = make_int4(__float_as_int(Df.x), __float_as_int(Df.y), __float_as_int(Df.z), __float_as_int(Df.w));
    if (D.w < 0) return 0;
    return sarsa_nearest_grid_gd(m, G, D, pos);
}

#ifndef RT_SARSA_COOP_KD
#define RT_SARSA_COOP_KD 1  // 0: a grid miss walks the k-d tree on its own lane (A/B builds)
#endif
constexpr int kKdFront = kKdStack * 32;  // frontier entries per buffer: two fill a wave's stack block

// sarsa_nearest for ONE query (pos, nrm: wave-uniform values) walked by the whole wave.
// The walk of sarsa_nearest visits a node iff every ancestor's split lets it through
// ((q_k - split)^2 < MAX_DIST for the far child), which does not depend on the best found
// so far: the visited leaves are a fixed set.  Here the wave expands that set level by
// level (breadth first, one node per lane and step, the frontier in the wave's LDS block)
// instead of one dependent load per visited node on one lane.  The walk's answer is the
// first leaf in its visit order with the smallest distance (same len3) and the query's
// normal, if that distance is below the start distance d0, else volume 0: equal here
// unless two visited leaves share the smallest distance (then the order decides) -- *ok is
// false then, on a frontier overflow and for a non-finite query, and the caller walks.
// All lanes of the wave take part; blk = the wave's kKdStack x 64 block.
__device__ int sarsa_nearest_wave(const SarsaMap& m, f3 pos, f3 nrm, int* blk, int lane, bool* ok) {
    const uint4* __restrict__ kd = m.kd4;
    *ok = false;
    if (!(__builtin_isfinite(pos.x) && __builtin_isfinite(pos.y) && __builtin_isfinite(pos.z))) return 0;
    int* cur = blk;
    int* nxt = blk + kKdFront;
    wave_lds_sync();  // the block's previous use (stack, exact phase) is done
    if (lane == 0) cur[0] = 0;
    wave_lds_sync();
    int n = 1;
    float best_d = INFINITY;
    int best = -1;
    bool tie = false;
    while (n > 0) {
        int m_next = 0;
        for (int base = 0; base < n; base += 64) {
            const int i = base + lane;
            int c0 = -1, c1 = -1;
            if (i < n) {
                const uint4 nd = kd[cur[i]];
                if (nd.w != 0xFFFFFFFFu) {  // leaf
                    const float d = len3(__uint_as_float(nd.x) - pos.x, __uint_as_float(nd.y) - pos.y,
                                         __uint_as_float(nd.z) - pos.z);
                    if (d <= best_d) {
                        const float4 n4 = m.vol_frame[nd.w * 3];
                        if (nrm.x == n4.x && nrm.y == n4.y && nrm.z == n4.z) {
                            tie = (d == best_d);
                            if (d < best_d) {
                                best_d = d;
                                best = (int)nd.w;
                            }
                        }
                    }
                } else {
                    const float pc = (nd.z == 0u) ? pos.x : ((nd.z == 1u) ? pos.y : pos.z);
                    const float delta = pc - __uint_as_float(nd.x);
                    const int left = (int)nd.y;
                    c0 = delta < 0.0f ? left : left + 1;
                    if ((delta * delta) < m.max_dist) c1 = (left + left + 1) - c0;
                }
            }
            // append the children: exclusive prefix of the lanes' counts (0..2) by ballots
            const int cnt = (c0 >= 0 ? 1 : 0) + (c1 >= 0 ? 1 : 0);
            const uint64_t b0 = __ballot(cnt & 1), b1 = __ballot(cnt >> 1);
            const int excl = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(b0 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b0, 0u)) +
                             2 * (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(b1 >> 32),
                                                                __builtin_amdgcn_mbcnt_lo((uint32_t)b1, 0u));
            const int tot = __builtin_popcountll(b0) + 2 * __builtin_popcountll(b1);
            if (m_next + tot > kKdFront) return 0;  // (wave-uniform) overflow: the caller walks
            if (c0 >= 0) nxt[m_next + excl] = c0;
            if (c1 >= 0) nxt[m_next + excl + 1] = c1;
            m_next += tot;
        }
        wave_lds_sync();  // the next level is written before any lane reads it
        int* t = cur;
        cur = nxt;
        nxt = t;
        n = m_next;
    }
    // the smallest distance over the wave, and whether it is unique
    float g = best_d;
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) g = fminf(g, __shfl_xor(g, off, 64));
    const bool at_min = best >= 0 && best_d == g;
    const uint64_t holders = __ballot(at_min), ties = __ballot(at_min && tie);
    wave_lds_sync();  // the frontier reads are done before the block's next use
    if (holders == 0ull) {  // no visited leaf has the normal: the start volume
        *ok = true;
        return 0;
    }
    if (__builtin_popcountll(holders) > 1 || ties != 0ull) return 0;  // the visit order decides
    const int src = __builtin_ctzll(holders);
    const int v = __shfl(best, src, 64);
    const float d0 = len3(pos.x - m.root_x, pos.y - m.root_y, pos.z - m.root_z);
    *ok = true;
    return g < d0 ? v : 0;
}

// every lane with *rv == kNeedWalk gets sarsa_nearest's volume: the wave walks the queries
// one after another (sarsa_nearest_wave), a lane whose query it cannot settle walks alone.
// All lanes take part.
__device__ void sarsa_resolve_walks(const SarsaMap& m, f3 pos, f3 nrm, int* rv, int* blk, int* st, int lane) {
#if RT_SARSA_COOP_KD
    uint64_t need = __ballot(*rv == kNeedWalk);
    while (need != 0ull) {
        const int L = __builtin_ctzll(need);
        need &= need - 1ull;
        const f3 q = make3(__shfl(pos.x, L, 64), __shfl(pos.y, L, 64), __shfl(pos.z, L, 64));
        const f3 qn = make3(__shfl(nrm.x, L, 64), __shfl(nrm.y, L, 64), __shfl(nrm.z, L, 64));
        bool ok;
        const int v = sarsa_nearest_wave(m, q, qn, blk, lane, &ok);
        if (lane == L && ok) *rv = v;
    }
#else
    (void)blk;
    (void)lane;
#endif
    if (*rv == kNeedWalk) *rv = sarsa_nearest(m, pos, nrm, st);
}

// normal class of a query normal (queries without a surface index)
__device__ int sarsa_class_of(const SarsaMap& m, f3 nrm) {
    for (int c = 0; c < m.n_class; ++c) {
        const float4 n4 = m.class_nrm[c];
        if (nrm.x == n4.x && nrm.y == n4.y && nrm.z == n4.z) return c;
    }
    return -1;
}

// The sampling volume's per-frame data, loaded as soon as the volume is known (sarsa_step):
// its CDF row ends (one 64-B line) and its frame (N, T, B with the position)
struct VolPre {
    float4 t0, t1, t2, t3;
    float4 N4, T4, B4;
};
__device__ __forceinline__ VolPre vol_load(const SarsaMap& m, int rv) {
    VolPre v;
    const float4* tp = m.cdf_top + (size_t)rv * 4;
    v.t0 = tp[0];
    v.t1 = tp[1];
    v.t2 = tp[2];
    v.t3 = tp[3];
    v.N4 = m.vol_frame[rv * 3 + 0];
    v.T4 = m.vol_frame[rv * 3 + 1];
    v.B4 = m.vol_frame[rv * 3 + 2];
    return v;
}

// sample_direction_from_radiance_distribution (radiance_volume.cu:191-244); vp: vol_load(m, rv)
__device__ bool sarsa_sample(const SarsaMap& m, int rv, const VolPre& vp, float r, float rx, float ry, int* sector,
                             f3* dir, float* pdf) {
    const float* __restrict__ cdf = m.cdf + (size_t)rv * kSarsaSectors;
    int found = -1;
    float mv = 0.0f, pv = 0.0f;
    // The CDF is non-decreasing, so the reference's binary search returns i0, the first
    // sector with cdf > r, unless one of its probes meets cdf[k] == r (it then turns
    // left of i0 and fails), which requires cdf[i0 - 1] == r.  i0 from two rounds of
    // independent loads (the 12 row ends, then one 12-sector row) instead of 8
    // dependent probes; the rare equal / NaN cases run the search itself.
    bool exact = false;
    const float4 t0 = vp.t0, t1 = vp.t1, t2 = vp.t2, t3 = vp.t3;  // one 64-B line: cdf[0] and the row ends
    const float c0 = t0.x;
    if (r <= c0) {
        found = 0;
        mv = c0;
    } else {
        const float top[kGridRes] = {t0.y, t0.z, t0.w, t1.x, t1.y, t1.z, t1.w, t2.x, t2.y, t2.z, t2.w, t3.x};
        int row = 0;
        bool nan = false;
#pragma unroll
        for (int x = 0; x < kGridRes; ++x) {
            row += (top[x] <= r) ? 1 : 0;
            nan |= (top[x] != top[x]);
        }
        if (row < kGridRes && !nan) {
            const float4* rp = reinterpret_cast<const float4*>(cdf + row * kGridRes);
            const float4 q0 = rp[0], q1 = rp[1], q2 = rp[2];
            const float v[kGridRes] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w, q2.x, q2.y, q2.z, q2.w};
            int j = 0;
            float prev = (row > 0) ? top[row - 1] : 0.0f;
#pragma unroll
            for (int k = 0; k < kGridRes; ++k) {
                const bool le = v[k] <= r;
                j += le ? 1 : 0;
                prev = le ? v[k] : prev;
                nan |= (v[k] != v[k]);
            }
            // j < 12: the row's last value is top[row] > r
            if (nan || prev == r) {
                exact = true;
            } else {
                found = row * kGridRes + j;
                mv = v[j < kGridRes ? j : kGridRes - 1];
                pv = prev;
            }
        } else {
            exact = nan;  // row == 12: no sector has cdf > r, the search fails
        }
    }
    if (exact) {
        int start = 0, end = kSarsaSectors - 1;
        while (start <= end) {
            const int mid = (end + start) / 2;
            const float mval = cdf[mid];
            const float pval = (mid > 0) ? cdf[mid - 1] : 0.0f;
            if (r < mval && pval <= r) {
                found = mid;
                mv = mval;
                pv = pval;
                break;
            } else if (mval < r) {
                start = mid + 1;
            } else {
                end = mid - 1;
            }
        }
    }
    if (found < 0) return false;
    const int sx = found / kGridRes;
    const int sy = found - sx * kGridRes;
    *sector = found;
    *pdf = kRho * ((found == 0 ? mv : (mv - pv)) / kGridRhoS);
    const float4 N4 = vp.N4, T4 = vp.T4, B4 = vp.B4;
    *dir = grid_direction((float)sx + rx, (float)sy + ry, make3(N4.x, N4.y, N4.z), make3(T4.x, T4.y, T4.z),
                          make3(B4.x, B4.y, B4.z), make3(N4.w, T4.w, B4.w));
    return true;
}

// a live value of the in-frame TD mode's shared state (Q, irradiance): read at device scope,
// past this CU's L1, so a lane sees the other lanes' (and its own earlier) atomicExch writes
__device__ __forceinline__ float live_load(const float* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// sample_max_direction_from_radiance_distribution (radiance_volume.cu:246-278): the first
// sector of largest Q, uniform within it; the pdf is the CDF step of that sector, 0 for
// sector 0 (the reference's last_pdf is cdf[0] there, :274).  Frame-synchronous TD: Q is
// fixed within the frame, so its argmax (qmax) is kept by k_sarsa_apply; in-frame TD
// (TD = 1): the reference's scan of the live radiance grid at every sample (:251-257), the
// CDF still the frame's (update_radiance_volume_distributions runs between frames).
template <int TD>
__device__ void sarsa_sample_max(const SarsaMap& m, int rv, const VolPre& vp, float rx, float ry, int* sector, f3* dir,
                                 float* pdf) {
    const float* __restrict__ cdf = m.cdf + (size_t)rv * kSarsaSectors;
    int mi;
    if constexpr (TD == 1) {
        const float* q = m.Q + (size_t)rv * kSarsaSectors;
        mi = 0;
        float mq = live_load(q);
        // the reference's scan (radiance_volume.cu:251-257) starts at i = 0 with grid[0] already
        // loaded; its plain (non-volatile) loads let the compiler read grid[0] once, so the
        // k = 0 step (mq < q[0] with mq = q[0]) is skipped: 144 device-scope loads, not 145
        for (int k = 1; k < kSarsaSectors; ++k) {
            const float v = live_load(q + k);
            if (mq < v) {
                mq = v;
                mi = k;
            }
        }
    } else {
        mi = m.qmax[rv];
    }
    const float mv = cdf[mi];
    const float last = cdf[mi > 0 ? mi - 1 : 0];
    const int sx = mi / kGridRes;
    const int sy = mi - sx * kGridRes;
    *sector = mi;
    *pdf = kRho * ((mv - last) / kGridRhoS);
    const float4 N4 = vp.N4, T4 = vp.T4, B4 = vp.B4;
    *dir = grid_direction((float)sx + rx, (float)sy + ry, make3(N4.x, N4.y, N4.z), make3(T4.x, T4.y, T4.z),
                          make3(B4.x, B4.y, B4.z), make3(N4.w, T4.w, B4.w));
}

// temporal_difference_update + expected_sarsa_irradiance as the reference runs them
// (radiance_volume.cu:282-301, :93-112): read-modify-write of the sector's Q and the
// volume's irradiance while other lanes do the same -- a lost update is the reference's own
// race.  The visit count comes from the atomic's return (the reference reads it first).
__device__ __forceinline__ void td_event_inframe(const SarsaMap& m, int rv, int sector, float target) {
    const size_t k = (size_t)rv * kSarsaSectors + sector;
    const uint32_t vs = atomicAdd(&m.visits[k], 1u);
    const float alpha = 1.f / (1.f + (float)vs);
    const float q_old = live_load(&m.Q[k]);
    float upd = ((1.f - alpha) * q_old) + (alpha * target);
    upd = upd > kRadianceThreshold ? upd : kRadianceThreshold;
    const float cc = m.cos_corner[k];
    const float brdf = m.vol_brdf[rv];
    const float acc = live_load(&m.accum[rv]);
    const float acc_new = (acc - ((q_old * cc) * brdf)) + ((upd * cc) * brdf);
    atomicExch(&m.Q[k], upd);
    atomicExch(&m.accum[rv], acc_new);
}

template <int TD>
__device__ __forceinline__ void td_event(const SarsaMap& m, int rv, int sector, float target) {
    if (RT_SARSA_NO_TD) return;
    if constexpr (TD == 1) {
        td_event_inframe(m, rv, sector, target);
        return;
    }
    const long long v = __float2ll_rn(target * 4294967296.0f);
    const size_t k = (size_t)rv * kSarsaSectors + sector;
    atomicAdd(&m.acc_sum[k], (unsigned long long)v);
    atomicAdd(&m.acc_cnt[k], 1u);
}

// The path's state between casts (k_sarsa_render, k_sarsa_render_pq)
struct SarsaPath {
    f3 o, d, tp;
    int depth, cur_rv, cur_sector;
    float cur_brdf;
    bool null_ray;  // set by sarsa_step: the path ended by tracing the zero direction
};

// One cast of path_trace_reinforcement_iterative after its closest hit h and the volume
// rv at a surface hit: the TD event of the previous step, then light / miss / the next
// direction from the volume's distribution.  Returns true when the path ends, with its
// value in *L (n_casts counts the reference's extra cast of a zero direction).
template <int TD>
__device__ __forceinline__ bool sarsa_step(const RenderLaunch& a, const SarsaMap& m, const Hit& h, bool is_surf,
                                           f3 pos, f3 nrm, int rv, bool td, uint32_t pix, int s, SarsaPath& P,
                                           unsigned& n_casts, f3* L_out) {
    const float4* __restrict__ shade = a.scene.shade;
    // the volume this hit samples from, and its data loaded now: in flight with the TD
    // target's irradiance load, the TD atomics and the Philox block
    const int sv = (td || (P.depth == 0 && is_surf)) ? rv : P.cur_rv;
    VolPre vp;
    if (is_surf && sv >= 0) vp = vol_load(m, sv);
    if (td) {
        float target;
        if (h.tri < 0) {
            target = P.cur_brdf * a.env_light;
        } else if (!is_surf) {
            target = P.cur_brdf * m.tri_lum[h.tri];
        } else {
            target = ((TD == 1 ? live_load(&m.accum[rv]) : m.accum[rv]) * kIrrScale) * P.cur_brdf;
        }
        td_event<TD>(m, P.cur_rv, P.cur_sector, target);
        P.cur_rv = rv;
        P.cur_sector = -1;
    } else if (P.depth == 0 && is_surf) {
        P.cur_rv = rv;
    }
    bool terminal = false;
    f3 L = make3(0.f, 0.f, 0.f);
    if (h.tri < 0) {
        terminal = true;
        L = make3(P.tp.x * a.env_light, P.tp.y * a.env_light, P.tp.z * a.env_light);
    } else if (!is_surf) {
        terminal = true;
        const float4 e = shade[h.tri * kShadeF4 + 3];
        L = make3(P.tp.x * e.x, P.tp.y * e.y, P.tp.z * e.z);
    } else {
        uint32_t rn[4];
        philox4x32_10(pix, a.sample_base + (uint32_t)s, 1u + (uint32_t)P.depth, 0u, a.seed_lo, a.seed_hi, rn);
        f3 sd;
        float pdf;
        bool ok = true;
        if (P.cur_rv < 0) {  // no volume: uniform hemisphere, pdf = RHO
            const float4 T4 = shade[h.tri * kShadeF4 + 1], B4 = shade[h.tri * kShadeF4 + 2];
            const float c = u01(rn[0]);
            const float st = sqrtf(1.0f - c * c);
            float sphi, cphi;
            sincos_turn(u01(rn[1]), &sphi, &cphi);
            const float sx = st * cphi, sz = st * sphi;
            sd = make3((sx * B4.x + c * nrm.x) + sz * T4.x, (sx * B4.y + c * nrm.y) + sz * T4.y,
                       (sx * B4.z + c * nrm.z) + sz * T4.z);
            pdf = kRho;
        } else if (m.sample_max) {
            sarsa_sample_max<TD>(m, P.cur_rv, vp, u01_oc(rn[1]), u01_oc(rn[2]), &P.cur_sector, &sd, &pdf);
        } else {
            ok = sarsa_sample(m, P.cur_rv, vp, u01_oc(rn[0]), u01_oc(rn[1]), u01_oc(rn[2]), &P.cur_sector, &sd, &pdf);
        }
        if (!ok) {
            // no sector: the reference traces the zero direction it returns, which
            // hits nothing (one more cast; its radiance there is NaN, here the miss value)
            terminal = true;
            if (P.depth + 1 < a.max_bounces) {
                ++n_casts;
                L = make3(P.tp.x * a.env_light, P.tp.y * a.env_light, P.tp.z * a.env_light);
                // the reference's throughput is (BRDF * 0) / pdf 0 = NaN here: its radiance is
                // NaN, which its zero-contribution test (NaN < threshold) does not count
                P.null_ray = true;
            }
        } else {
            const float4 brdf = shade[h.tri * kShadeF4 + 3];
            const float cos_theta = dot(nrm, sd);
            P.cur_brdf = m.tri_lum[h.tri] / kPi;
            P.tp.x = P.tp.x * ((brdf.x * cos_theta) / pdf);
            P.tp.y = P.tp.y * ((brdf.y * cos_theta) / pdf);
            P.tp.z = P.tp.z * ((brdf.z * cos_theta) / pdf);
            P.o = make3(pos.x + sd.x * kEps, pos.y + sd.y * kEps, pos.z + sd.z * kEps);
            P.d = normalize(sd);
            ++P.depth;
            if (P.depth == a.max_bounces) terminal = true;
        }
    }
    *L_out = L;
    return terminal;
}

// path_trace_reinforcement_iterative (reinforcement_path_tracing.cu:50-120), GPU preset
// MF > 0: every cast on the matrix-core filter (closest_hit_mf, wave-level; the launcher
// picks it as launch_render_t does for k_render: image present, camera inside its bound)
// MF: the exact phase's LDS is the wave's own block of the k-d stack (free between searches;
// wave_lds_sync orders the two uses), so the workgroup needs the stack's 32 KB only; scenes
// of <= 64 triangles held to 4 waves per SIMD (<= 128 VGPRs without spills; the 4-block
// variant would spill there and keeps the compiler's 3 waves).
#ifndef RT_MF_SARSA_WAVES
#define RT_MF_SARSA_WAVES 4
#endif
template <int RULE, int MF, int TD>
__global__ __launch_bounds__(256, MF == 1 ? RT_MF_SARSA_WAVES : 1) void k_sarsa_render(const RenderLaunch a,
                                                                                     const SarsaMap m) {
    const int lg = a.split_log2;
    const BlockDesc blk = a.blocks[blockIdx.x >> lg];
    const int part = blockIdx.x & (a.split - 1);
    const int q = (part << (8 - lg)) + ((int)threadIdx.x >> lg);
    const int chunk = threadIdx.x & (a.split - 1);
    const int lane = threadIdx.x & 63;
    const int lx = q & 15, ly = q >> 4;
    const int px = blk.px0 + lx, py = blk.py0 + ly;
    const bool valid = (px < a.clip_x1) && (py < a.clip_y1);
    const uint32_t pix = (uint32_t)py * (uint32_t)a.width + (uint32_t)px;
    const float4* __restrict__ shade = a.scene.shade;
    const int n_surf = a.scene.n_surf;
    const int s_end = (chunk + 1) * a.per_chunk;
    __shared__ int kd_stack[kKdStack * 256];
    int* const st = kd_stack_of(kd_stack);
    static_assert(kKdStack * 64 >= kMfWaveFloats, "the exact phase's LDS fits a wave's stack block");
    float* const wl = reinterpret_cast<float*>(kd_stack + ((int)threadIdx.x >> 6) * (kKdStack * 64));

    int s = valid ? chunk * a.per_chunk : s_end;
    int depth = 0;
    int cur_rv = -1, cur_sector = -1;
    float cur_brdf = 0.0f;
    f3 o = make3(a.cam_x, a.cam_y, a.cam_z), d = make3(0.f, 0.f, 1.f);
    f3 tp = make3(1.f, 1.f, 1.f), acc = make3(0.f, 0.f, 0.f);
    unsigned n_casts = 0, n_zero = 0;
    if (s < s_end) {
        float r1, r2;
        draw2(pix, a.sample_base + (uint32_t)s, 0u, a.seed_lo, a.seed_hi, &r1, &r2);
        camera_ray<1>(a, px, py, r1, r2, &d);
    }
    for (;;) {
        const bool active = s < s_end;
        if (__ballot(active) == 0ull) break;
        Hit h;
        h.t = 0.0f;
        h.tri = -1;
        if constexpr (MF > 0) {
            wave_lds_sync();  // the previous search's stack accesses stay before the exact phase
            h = closest_hit_mf<RULE, false, MF>(a.scene, o, d, a.t_scale, active, wl);
            wave_lds_sync();  // and its LDS traffic before the next search
        } else if (active) {
            h = closest_hit_sel<RULE>(a.scene, a.use_filter, o, d, a.t_scale);
        }
        // (inactive lanes go on to the volume search, which the whole wave runs, with no query)
        if (active) ++n_casts;
        const bool is_surf = active && (h.tri >= 0) && (h.tri < n_surf);
        f3 pos = o;
        f3 nrm = make3(0.f, 0.f, 0.f);
        if (is_surf) {
            const float Dx = d.x * a.t_scale, Dy = d.y * a.t_scale, Dz = d.z * a.t_scale;
            pos = make3(o.x + h.t * Dx, o.y + h.t * Dy, o.z + h.t * Dz);
            const float4 N4 = shade[h.tri * kShadeF4 + 0];
            nrm = make3(N4.x, N4.y, N4.z);
        }
        // temporal_difference_update_radiance_volume_sector at every bounce after a
        // sampled sector; the volume at a surface hit serves both the TD target and
        // the next sampling step (one search call site: the search is divergent)
        const bool td = active && depth > 0 && cur_rv >= 0 && cur_sector >= 0;
        int rv = -1;
        if (is_surf && (depth == 0 || td))
            rv = m.use_grid ? sarsa_nearest_grid_tri(m, h.tri, pos, nrm) : kNeedWalk;
        if (m.use_grid)  // the grid's few undecided queries: walked by the whole wave
            sarsa_resolve_walks(m, pos, nrm, &rv, kd_stack + ((int)threadIdx.x >> 6) * (kKdStack * 64), st, lane);
        else if (rv == kNeedWalk)
            rv = sarsa_nearest(m, pos, nrm, st);
        if (!active) continue;
        SarsaPath P{o, d, tp, depth, cur_rv, cur_sector, cur_brdf, false};
        f3 L;
        const bool terminal = sarsa_step<TD>(a, m, h, is_surf, pos, nrm, rv, td, pix, s, P, n_casts, &L);
        o = P.o;
        d = P.d;
        tp = P.tp;
        depth = P.depth;
        cur_rv = P.cur_rv;
        cur_sector = P.cur_sector;
        cur_brdf = P.cur_brdf;
        if (terminal) {
            acc.x = acc.x + L.x;
            acc.y = acc.y + L.y;
            acc.z = acc.z + L.z;
            // a zero-contribution light path (reinforcement_path_tracing.cu:36-40)
            n_zero += (!P.null_ray && (L.x + L.y + L.z) / 3.f < kThroughputThreshold) ? 1u : 0u;
            ++s;
            depth = 0;
            cur_rv = -1;
            cur_sector = -1;
            tp = make3(1.f, 1.f, 1.f);
            o = make3(a.cam_x, a.cam_y, a.cam_z);
            if (s < s_end) {
                float r1, r2;
                draw2(pix, a.sample_base + (uint32_t)s, 0u, a.seed_lo, a.seed_hi, &r1, &r2);
                camera_ray<1>(a, px, py, r1, r2, &d);
            }
        }
    }
    const int base = lane & ~(a.split - 1);
    f3 tot = acc;
    unsigned pix_casts = n_casts;  // a sample's path length is its ray casts
    for (int k = 1; k < a.split; ++k) {
        const float vx = __shfl(acc.x, base + k, 64);
        const float vy = __shfl(acc.y, base + k, 64);
        const float vz = __shfl(acc.z, base + k, 64);
        pix_casts += (unsigned)__shfl((int)n_casts, base + k, 64);
        tot.x = tot.x + vx;
        tot.y = tot.y + vy;
        tot.z = tot.z + vz;
    }
    if (m.stats != nullptr) {
        // main.cu:321-339 statistics: int(total_path_lengths / SAMPLES_PER_PIXEL) per pixel
        const unsigned pf = (valid && chunk == 0) ? pix_casts / (unsigned)a.spp : 0u;
        const unsigned sp = wave_sum(pf), sz = wave_sum(n_zero);
        if (lane == 0) {
            atomicAdd(&m.stats[0], (unsigned long long)sp);
            atomicAdd(&m.stats[1], (unsigned long long)sz);
        }
    }
    if (valid && chunk == 0) {
        const float fs = (float)a.spp;
        float* dst = a.out + ((size_t)(blk.oy0 + ly) * (size_t)a.out_pitch + (size_t)(blk.ox0 + lx)) * 3;
        store_rgb(dst, tot.x / fs, tot.y / fs, tot.z / fs);
    }
    if (a.casts != nullptr) {
        const unsigned total = wave_sum(n_casts);
        if (lane == 0) atomicAdd(a.casts, (unsigned long long)total);
    }
}

// k_sarsa_render on a persistent grid over a launch-wide (pixel, chunk) queue, as
// k_render_pq does for the GPU preset (rt_kernels.hip): a lane claims a chunk (the samples
// [c m, (c + 1) m) of pixel p), traces them one after another with k_sarsa_render's
// per-cast work (sarsa_step) and its fixed-chunk sum, stores the chunk's value sum and ray
// casts, and claims the next, so lanes idle only at the end of the frame instead of at
// each wave's longest path (frame 0: 41 casts per path on door_room, up to 80).
// k_sarsa_fold adds each pixel's chunks in chunk order and takes its path-length statistic.
// The volume search still runs with every lane of the wave (the walks of the grid's
// undecided queries, sarsa_resolve_walks).  csum: float4 per chunk {r, g, b, casts (bits)}.
#ifndef RT_SARSA_WAVES
#define RT_SARSA_WAVES 5  // waves per SIMD of the persistent render (its grid: that many workgroups per CU)
#endif
// BVH: scenes with the exact BVH (large models, rt_scene_set_accel): the casts through
// closest_hit_bvh, its stack in the lane's k-d stack column (free until the volume search)
// CT > 0: the casts take their candidates from tables (CT mask words; k_render_pq's CT route:
// a camera ray the cull of its pixel's 16x4 rectangle in a.cull, a bounce ray the candidate
// table of the surface it leaves) and closest_hit_cand tests them in index order
template <int RULE, int MF, int TD, bool BVH = false, int CT = 0>
#ifndef RT_SARSA_BVH_WAVES
#define RT_SARSA_BVH_WAVES 4  // the BVH variant's traversal state: 128 VGPRs, no spills (96 at 5 waves spilled)
#endif
__global__ __launch_bounds__(256, BVH ? RT_SARSA_BVH_WAVES : (MF == 1 ? RT_MF_SARSA_WAVES : RT_SARSA_WAVES)) void k_sarsa_render_pq(const RenderLaunch a,
                                                                                        const SarsaMap m) {
    __shared__ __attribute__((aligned(16))) int kd_stack[kKdStack * 256];
    static_assert(kKdStack * 64 >= kMfWaveFloats, "the exact phase's LDS fits a wave's stack block");
    int* const st = kd_stack_of(kd_stack);
    int* const blk_ws = kd_stack + ((int)threadIdx.x >> 6) * (kKdStack * 64);  // the wave's block
    float* const wl = reinterpret_cast<float*>(blk_ws);
    const int lane = threadIdx.x & 63;
    const float4* __restrict__ shade = a.scene.shade;
    const int n_surf = a.scene.n_surf;
    const long long total = (long long)a.n_blocks * 256 * a.split;
    const f3 cam = make3(a.cam_x, a.cam_y, a.cam_z);
    long long qb = 0, qe = 0;  // wave-uniform: the wave's claimed, not yet handed out items
    bool exhausted = false;
    bool have = false;
    long long item = 0;
    int s = 0, s_end = 0, px = 0, py = 0;
    uint32_t pix = 0;
    int surf = -1, cidx = 0;  // CT: the surface the ray leaves; the pixel's rectangle in a.cull
    SarsaPath P{cam, make3(0.f, 0.f, 1.f), make3(1.f, 1.f, 1.f), 0, -1, -1, 0.0f, false};
    f3 acc = make3(0.f, 0.f, 0.f);
    unsigned n_casts = 0, n_zero = 0, casts0 = 0;
#if RT_SARSA_PROF
    uint64_t pr[6] = {0, 0, 0, 0, 0, 0};  // trace, grid search, walks, step (TD + sampling), trips, active lanes
#endif
    auto camera = [&]() {
        float r1, r2;
        draw2(pix, a.sample_base + (uint32_t)s, 0u, a.seed_lo, a.seed_hi, &r1, &r2);
        camera_ray<1>(a, px, py, r1, r2, &P.d);
        P.o = cam;
        P.tp = make3(1.f, 1.f, 1.f);
        P.depth = 0;
        P.cur_rv = -1;
        P.cur_sector = -1;
        P.null_ray = false;
    };
    for (;;) {
        if (!exhausted) {
            const uint64_t need = __ballot(!have);
            if (need != 0ull) {
                const int n_need = __builtin_popcountll(need);
                const int rank = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(need >> 32),
                                                                __builtin_amdgcn_mbcnt_lo((uint32_t)need, 0u));
                const long long avail = qe - qb;
                long long nb = 0;
                if (n_need > avail) {  // (wave-uniform) 64 more items
                    unsigned long long v = 0;
                    if (lane == 0) v = atomicAdd(a.work, 64ull);
                    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
                    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
                    nb = (long long)(((unsigned long long)hi << 32) | lo);
                }
                if (!have) {
                    const long long j = rank < avail ? qb + rank : nb + (rank - avail);
                    if (j < total) {
                        item = j;
                        const long long p = j >> a.split_log2;
                        const int c = (int)(j & (a.split - 1));
                        const BlockDesc blk = a.blocks[p >> 8];
                        const int q = (int)(p & 255);
                        px = blk.px0 + (q & 15);
                        py = blk.py0 + (q >> 4);
                        if (px < a.clip_x1 && py < a.clip_y1) {
                            pix = (uint32_t)py * (uint32_t)a.width + (uint32_t)px;
                            cidx = (int)(p >> 8) * 4 + (q >> 6);
                            s = c * a.per_chunk;
                            s_end = s + a.per_chunk;
                            acc = make3(0.f, 0.f, 0.f);
                            casts0 = n_casts;
                            have = true;
                            camera();
                        }
                    }
                }
                if (n_need > avail) {
                    qb = nb + (n_need - avail);
                    qe = nb + 64;
                } else {
                    qb += n_need;
                }
                if (qb >= total) exhausted = true;
            }
        }
        const bool active = have;
        if (__ballot(active) == 0ull) {
            if (exhausted) break;
            continue;
        }
#if RT_SARSA_PROF
        const uint64_t pt0 = __builtin_amdgcn_s_memtime();
        pr[5] += (uint64_t)__builtin_popcountll(__ballot(active));
#endif
        Hit h;
        h.t = 0.0f;
        h.tri = -1;
        if constexpr (BVH) {
            static_assert(kKdStack >= kBvhMaxDepth, "the BVH stack fits the k-d stack column");
            if (active) h = closest_hit_bvh<RULE, 64>(a.scene, P.o, P.d, a.t_scale, st);
        } else if constexpr (CT > 0) {
            uint64_t F[CT];
#pragma unroll
            for (int k = 0; k < CT; ++k) F[k] = 0ull;
            if (active && P.depth == 0) {
#pragma unroll
                for (int k = 0; k < CT; ++k)
                    F[k] = (k < kRenderCullWords) ? a.cull[(size_t)cidx * kRenderCullWords + k] : 0ull;
            } else if (active) {
                ctab_candidates<CT>(a.scene.ctab[RULE], a.scene.n_tri, n_surf, surf, P.o, P.d, F);
            }
            wave_lds_sync();
            h = closest_hit_cand<RULE, CT>(a.scene, F, P.o, P.d, a.t_scale, wl);
            wave_lds_sync();
        } else if constexpr (MF > 0) {
            wave_lds_sync();
            h = closest_hit_mf<RULE, false, MF>(a.scene, P.o, P.d, a.t_scale, active, wl);
            wave_lds_sync();
        } else if (active) {
            h = closest_hit_sel<RULE>(a.scene, a.use_filter, P.o, P.d, a.t_scale);
        }
#if RT_SARSA_PROF
        const uint64_t pt1 = __builtin_amdgcn_s_memtime();
#endif
        if (active) ++n_casts;
        const bool is_surf = active && (h.tri >= 0) && (h.tri < n_surf);
        f3 pos = P.o;
        f3 nrm = make3(0.f, 0.f, 0.f);
        if (is_surf) {
            const float Dx = P.d.x * a.t_scale, Dy = P.d.y * a.t_scale, Dz = P.d.z * a.t_scale;
            pos = make3(P.o.x + h.t * Dx, P.o.y + h.t * Dy, P.o.z + h.t * Dz);
            const float4 N4 = shade[h.tri * kShadeF4 + 0];
            nrm = make3(N4.x, N4.y, N4.z);
        }
        const bool td = active && P.depth > 0 && P.cur_rv >= 0 && P.cur_sector >= 0;
        int rv = -1;
        if (is_surf && (P.depth == 0 || td))
            rv = m.use_grid ? sarsa_nearest_grid_tri(m, h.tri, pos, nrm) : kNeedWalk;
#if RT_SARSA_PROF
        const uint64_t pt2 = __builtin_amdgcn_s_memtime();
#endif
        if (m.use_grid)
            sarsa_resolve_walks(m, pos, nrm, &rv, blk_ws, st, lane);
        else if (rv == kNeedWalk)
            rv = sarsa_nearest(m, pos, nrm, st);
#if RT_SARSA_PROF
        const uint64_t pt3 = __builtin_amdgcn_s_memtime();
        f3 L;
        const bool term = active && sarsa_step<TD>(a, m, h, is_surf, pos, nrm, rv, td, pix, s, P, n_casts, &L);
        surf = h.tri;
        const uint64_t pt4 = __builtin_amdgcn_s_memtime();
        pr[0] += pt1 - pt0;
        pr[1] += pt2 - pt1;
        pr[2] += pt3 - pt2;
        pr[3] += pt4 - pt3;
        pr[4] += 1;
        if (!active) continue;
        if (term) {
#else
        if (!active) continue;
        f3 L;
        const bool term = sarsa_step<TD>(a, m, h, is_surf, pos, nrm, rv, td, pix, s, P, n_casts, &L);
        surf = h.tri;  // (a continuing path leaves the surface it hit)
        if (term) {
#endif
            acc.x = acc.x + L.x;
            acc.y = acc.y + L.y;
            acc.z = acc.z + L.z;
            n_zero += (!P.null_ray && (L.x + L.y + L.z) / 3.f < kThroughputThreshold) ? 1u : 0u;
            ++s;
            if (s < s_end) {
                camera();
            } else {
                reinterpret_cast<float4*>(a.csum)[item] = make_float4(acc.x, acc.y, acc.z, __uint_as_float(n_casts - casts0));
                have = false;
            }
        }
    }
    if (m.stats != nullptr) {
        const unsigned sz = wave_sum(n_zero);
        if (lane == 0) atomicAdd(&m.stats[1], (unsigned long long)sz);
    }
    if (a.casts != nullptr) {
        const unsigned tot = wave_sum(n_casts);
        if (lane == 0) atomicAdd(a.casts, (unsigned long long)tot);
    }
#if RT_SARSA_PROF
    if (m.prof != nullptr && lane == 0)
        for (int i = 0; i < 6; ++i) atomicAdd(m.prof + i, (unsigned long long)pr[i]);
#endif
}

// the pixels of k_sarsa_render_pq's launch: the chunk sums in chunk order / spp, and the
// per-pixel statistic int(path lengths / SAMPLES_PER_PIXEL) (main.cu:321-339)
__global__ __launch_bounds__(256) void k_sarsa_fold(const RenderLaunch a, const SarsaMap m) {
    const long long p = (long long)blockIdx.x * 256 + threadIdx.x;
    const BlockDesc blk = a.blocks[blockIdx.x];
    const int q = threadIdx.x, lx = q & 15, ly = q >> 4;
    const bool valid = (blk.px0 + lx < a.clip_x1) && (blk.py0 + ly < a.clip_y1);
    unsigned pf = 0;
    if (valid) {
        const float4* c = reinterpret_cast<const float4*>(a.csum) + (size_t)p * a.split;
        float4 v = c[0];
        f3 tot = make3(v.x, v.y, v.z);
        unsigned pix_casts = __float_as_uint(v.w);
        for (int k = 1; k < a.split; ++k) {
            v = c[k];
            tot.x = tot.x + v.x;
            tot.y = tot.y + v.y;
            tot.z = tot.z + v.z;
            pix_casts += __float_as_uint(v.w);
        }
        pf = pix_casts / (unsigned)a.spp;
        const float fs = (float)a.spp;
        float* dst = a.out + ((size_t)(blk.oy0 + ly) * (size_t)a.out_pitch + (size_t)(blk.ox0 + lx)) * 3;
        store_rgb(dst, tot.x / fs, tot.y / fs, tot.z / fs);
    }
    if (m.stats != nullptr) {
        const unsigned sp = wave_sum(pf);
        if ((threadIdx.x & 63) == 0) atomicAdd(&m.stats[0], (unsigned long long)sp);
    }
}

// update_radiance_distribution (radiance_volume.cu:148-188) of volume v, its row ends, and
// the first sector of largest Q (the max-direction sampler's scan, radiance_volume.cu:251-257)
__device__ void rebuild_volume(const SarsaMap& m, int v) {
    const size_t b = (size_t)v * kSarsaSectors;
    float total = 0.0000000001f;
    for (int k = 0; k < kSarsaSectors; ++k) {
        float t = m.Q[b + k] * m.cos_center[b + k];
        t = t > 0.0f ? t : 0.0f;
        total += t;
    }
    float prev = 0.0f;
    float* top = reinterpret_cast<float*>(m.cdf_top + (size_t)v * 4);
    for (int k = 0; k < kSarsaSectors; ++k) {
        float t = m.Q[b + k] * m.cos_center[b + k];
        t = t > 0.0f ? t : 0.0f;
        const float rad = t / total + prev;
        m.cdf[b + k] = rad;
        if (k == 0) top[0] = rad;
        if (k % kGridRes == kGridRes - 1) top[1 + k / kGridRes] = rad;
        prev = rad;
    }
    int mi = 0;
    float mq = m.Q[b];
    for (int k = 0; k < kSarsaSectors; ++k) {
        const float q = m.Q[b + k];
        if (mq < q) {
            mq = q;
            mi = k;
        }
    }
    m.qmax[v] = mi;
}

// End of frame, one lane per volume: fold the frame's TD targets (the running
// mean of alpha = 1/(1+visits), clamped at RADIANCE_THRESHOLD), update the
// irradiance with expected_sarsa_irradiance's increments (cell corners), and
// rebuild the CDF from Q*cos(cell centre) (update_radiance_distribution).
__global__ __launch_bounds__(256) void k_sarsa_apply(const SarsaMap m) {
    const int v = blockIdx.x * 256 + threadIdx.x;
    if (v >= m.n_vol) return;
    const size_t b = (size_t)v * kSarsaSectors;
    const float brdf = m.vol_brdf[v];
    float accum = m.accum[v];
    for (int k = 0; k < kSarsaSectors; ++k) {
        const uint32_t n = m.acc_cnt[b + k];
        if (n == 0u) continue;
        const long long S = (long long)m.acc_sum[b + k];
        const float sum = (float)((double)S * 2.3283064365386962890625e-10);
        const uint32_t vis = m.visits[b + k];
        const float q_old = m.Q[b + k];
        float q_new = (q_old * (float)vis + sum) / (float)(vis + n);
        q_new = q_new > kRadianceThreshold ? q_new : kRadianceThreshold;
        const float cc = m.cos_corner[b + k];
        accum = (accum - ((q_old * cc) * brdf)) + ((q_new * cc) * brdf);
        m.Q[b + k] = q_new;
        m.visits[b + k] = vis + n;
        m.acc_cnt[b + k] = 0u;
        m.acc_sum[b + k] = 0ull;
    }
    m.accum[v] = accum;
    rebuild_volume(m, v);
}

// CDF and argmax of Q after a load (rt_sarsa_load_q)
__global__ __launch_bounds__(256) void k_sarsa_rebuild(const SarsaMap m) {
    const int v = blockIdx.x * 256 + threadIdx.x;
    if (v >= m.n_vol) return;
    rebuild_volume(m, v);
}

// nearest-volume queries alone (KD parity): pos/nrm [n][3]
__global__ __launch_bounds__(256) void k_sarsa_nearest(const SarsaMap m, const float* __restrict__ pos,
                                                       const float* __restrict__ nrm, int n, int32_t* out) {
    __shared__ int kd_stack[kKdStack * 256];
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (blockIdx.x * 256 + (threadIdx.x & ~63) >= n) return;  // (whole waves past the end)
    const bool in = i < n;
    const f3 p = in ? make3(pos[3 * i], pos[3 * i + 1], pos[3 * i + 2]) : make3(0.f, 0.f, 0.f);
    const f3 nr = in ? make3(nrm[3 * i], nrm[3 * i + 1], nrm[3 * i + 2]) : make3(0.f, 0.f, 0.f);
    int v = -1;
    if (m.use_grid) {  // as k_sarsa_render searches
        if (in) v = RT_SARSA_NO_KD ? 0 : sarsa_nearest_grid(m, sarsa_class_of(m, nr), p, nr);
        sarsa_resolve_walks(m, p, nr, &v, kd_stack + ((int)threadIdx.x >> 6) * (kKdStack * 64), kd_stack_of(kd_stack),
                            threadIdx.x & 63);
    } else if (in) {
        v = sarsa_nearest(m, p, nr, kd_stack_of(kd_stack));
    }
    if (in) out[i] = v;
}

}  // namespace

hipError_t launch_sarsa_nearest(const SarsaMap& m, const float* pos, const float* nrm, int n, int32_t* out,
                                hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_sarsa_nearest, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, m, pos, nrm, n, out);
    return hipGetLastError();
}

#ifndef RT_MF_SARSA
#define RT_MF_SARSA 0  // 1: the casts on the matrix-core filter (measured slower: DESIGN.md §4)
#endif

#ifndef RT_SARSA_CTAB
#define RT_SARSA_CTAB 0  // 1: k_sarsa_render_pq's casts from the candidate tables (door_room 512^2 x 256: 110.3 vs 92.1 ms per frame)
#endif

#ifndef RT_SARSA_PQ
#define RT_SARSA_PQ 1  // 0: the per-pixel k_sarsa_render (A/B builds)
#endif

namespace {

// the render launch of one TD rule (TD: k_sarsa_render's template argument, so the default
// frame-synchronous kernel carries no in-frame branch)
template <int TD>
hipError_t launch_sarsa_render_t(const RenderLaunch& a, const SarsaMap& m, hipStream_t stream) {
    const float cb = a.scene.mf_bound;
    const bool mf = RT_MF_SARSA && a.scene.bvh_nodes == nullptr && a.use_filter && a.scene.mf_frag != nullptr && a.t_scale > 0.0f &&
                    a.t_scale <= kFiltMaxTScale && fabsf(a.cam_x) <= cb && fabsf(a.cam_y) <= cb &&
                    fabsf(a.cam_z) <= cb;
    const bool one = a.scene.n_tri <= 64;
    // the table route (k_sarsa_render_pq CT): as k_render_pq's -- the scene's candidate table for
    // this hit rule and t_scale, the camera rays' rectangle cull (pitch 0, filter records valid
    // for the camera)
    const CtabDev& T = a.scene.ctab[a.hit_rule == 0 ? 0 : 1];
    const bool ct = !mf && RT_SARSA_CTAB && a.scene.bvh_nodes == nullptr && a.cull != nullptr && a.use_filter &&
                    a.cos_x == 1.0f && a.sin_x == 0.0f && a.scene.n_tri <= 64 * kRenderCullWords &&
                    T.masks != nullptr && T.bins == kCtabBins && T.graze_n == kCtabGraze && a.t_scale >= T.ts_min &&
                    T.words <= (one ? 1 : 4);
    if constexpr (RT_SARSA_PQ) {
        if (a.csum == nullptr || a.work == nullptr) return hipErrorInvalidValue;
        (void)hipMemsetAsync(a.work, 0, sizeof(unsigned long long), stream);
        // as many workgroups as fit: RT_SARSA_WAVES per CU (registers and the k-d stack's LDS)
        const int per_cu = a.scene.bvh_nodes != nullptr ? RT_SARSA_BVH_WAVES : (mf ? RT_MF_SARSA_WAVES : RT_SARSA_WAVES);
        int wgs = min(a.n_blocks * a.split, per_cu * device_cu_count());
        if (m.max_wgs > 0) wgs = min(wgs, m.max_wgs);  // rt_sarsa_set_inframe_lanes
        const dim3 grid((unsigned)wgs);
        if constexpr (RT_MF_SARSA) {
            if (mf) {
                if (a.hit_rule == 0 && one)
                    hipLaunchKernelGGL((k_sarsa_render_pq<0, 1, TD>), grid, dim3(256), 0, stream, a, m);
                else if (a.hit_rule == 0)
                    hipLaunchKernelGGL((k_sarsa_render_pq<0, 4, TD>), grid, dim3(256), 0, stream, a, m);
                else if (one)
                    hipLaunchKernelGGL((k_sarsa_render_pq<1, 1, TD>), grid, dim3(256), 0, stream, a, m);
                else
                    hipLaunchKernelGGL((k_sarsa_render_pq<1, 4, TD>), grid, dim3(256), 0, stream, a, m);
            }
        }
        if (a.scene.bvh_nodes != nullptr) {  // the exact BVH (large scenes)
            if (a.hit_rule == 0)
                hipLaunchKernelGGL((k_sarsa_render_pq<0, 0, TD, true>), grid, dim3(256), 0, stream, a, m);
            else
                hipLaunchKernelGGL((k_sarsa_render_pq<1, 0, TD, true>), grid, dim3(256), 0, stream, a, m);
        } else if (ct) {
            RenderLaunch c = a;  // one workgroup per 16x16 block: the masks of its four 16x4 rectangles
            c.split = 1;
            c.split_log2 = 0;
            (void)launch_cull(c, stream);
            if (a.hit_rule == 0) {
                if (one)
                    hipLaunchKernelGGL((k_sarsa_render_pq<0, 0, TD, false, 1>), grid, dim3(256), 0, stream, a, m);
                else
                    hipLaunchKernelGGL((k_sarsa_render_pq<0, 0, TD, false, 4>), grid, dim3(256), 0, stream, a, m);
            } else {
                if (one)
                    hipLaunchKernelGGL((k_sarsa_render_pq<1, 0, TD, false, 1>), grid, dim3(256), 0, stream, a, m);
                else
                    hipLaunchKernelGGL((k_sarsa_render_pq<1, 0, TD, false, 4>), grid, dim3(256), 0, stream, a, m);
            }
        } else if (!mf) {
            if (a.hit_rule == 0)
                hipLaunchKernelGGL((k_sarsa_render_pq<0, 0, TD>), grid, dim3(256), 0, stream, a, m);
            else
                hipLaunchKernelGGL((k_sarsa_render_pq<1, 0, TD>), grid, dim3(256), 0, stream, a, m);
        }
        hipLaunchKernelGGL(k_sarsa_fold, dim3((unsigned)a.n_blocks), dim3(256), 0, stream, a, m);
        return hipGetLastError();
    } else {
        const dim3 grid((unsigned)(a.n_blocks * a.split));
        if constexpr (RT_MF_SARSA) {
            if (mf) {
                if (a.hit_rule == 0 && one)
                    hipLaunchKernelGGL((k_sarsa_render<0, 1, TD>), grid, dim3(256), 0, stream, a, m);
                else if (a.hit_rule == 0)
                    hipLaunchKernelGGL((k_sarsa_render<0, 4, TD>), grid, dim3(256), 0, stream, a, m);
                else if (one)
                    hipLaunchKernelGGL((k_sarsa_render<1, 1, TD>), grid, dim3(256), 0, stream, a, m);
                else
                    hipLaunchKernelGGL((k_sarsa_render<1, 4, TD>), grid, dim3(256), 0, stream, a, m);
            }
        }
        if (!mf) {
            if (a.hit_rule == 0)
                hipLaunchKernelGGL((k_sarsa_render<0, 0, TD>), grid, dim3(256), 0, stream, a, m);
            else
                hipLaunchKernelGGL((k_sarsa_render<1, 0, TD>), grid, dim3(256), 0, stream, a, m);
        }
        return hipGetLastError();
    }
}

}  // namespace

hipError_t launch_sarsa_render(const RenderLaunch& a, const SarsaMap& m, hipStream_t stream) {
    if (a.n_blocks <= 0) return hipSuccess;
    KernelTimer kt(KT_SARSA_RENDER, stream);
    return m.td_inframe ? launch_sarsa_render_t<1>(a, m, stream) : launch_sarsa_render_t<0>(a, m, stream);
}

hipError_t launch_sarsa_rebuild(const SarsaMap& m, hipStream_t stream) {
    if (m.n_vol <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_sarsa_rebuild, dim3((unsigned)((m.n_vol + 255) / 256)), dim3(256), 0, stream, m);
    return hipGetLastError();
}

bool sarsa_prof_compiled() { return RT_SARSA_PROF != 0; }
bool sarsa_ctab_compiled() { return RT_SARSA_CTAB != 0; }

hipError_t launch_sarsa_apply(const SarsaMap& m, hipStream_t stream) {
    if (m.n_vol <= 0) return hipSuccess;
    KernelTimer kt(KT_SARSA_APPLY, stream);
    hipLaunchKernelGGL(k_sarsa_apply, dim3((unsigned)((m.n_vol + 255) / 256)), dim3(256), 0, stream, m);
    return hipGetLastError();
}

}  // namespace rt
