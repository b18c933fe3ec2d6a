// rt_ktime.cpp — per-kernel-family launch timing with HIP events on the launch stream
// (bench.py's live kernel durations for the roofline of every workload; rt_ktime_* in
// rtmi.h).  Disabled: a KernelTimer costs one atomic load.  Enabled: one event pair per
// timed launch, recycled through a pool; rt_ktime_read waits for the recorded pairs and
// folds them into per-family totals.
#include <atomic>
#include <mutex>
#include <vector>

#include "../../include/rtmi.h"
#include "rt_internal.hpp"

namespace rt {
int set_error(int code, const char* msg);
}

namespace {

struct Rec {
    int kernel;
    hipEvent_t a, b;
};

std::atomic<bool> g_on{false};
std::mutex g_mu;
std::vector<Rec> g_pending;
std::vector<std::pair<hipEvent_t, hipEvent_t>> g_pool;
double g_ms[rt::KT_COUNT];
int64_t g_n[rt::KT_COUNT];
int g_errors = 0;

const char* const kNames[rt::KT_COUNT] = {"k_render_ps", "k_render", "k_sarsa_render", "k_sarsa_apply",
                                          "k_dqn_mlp", "k_dqn_bounce", "k_dqn_camera"};

// fold every recorded pair into the totals (caller holds g_mu)
void drain(bool keep) {
    for (const Rec& r : g_pending) {
        float ms = 0.f;
        if (hipEventSynchronize(r.b) == hipSuccess && hipEventElapsedTime(&ms, r.a, r.b) == hipSuccess) {
            if (keep) {
                g_ms[r.kernel] += ms;
                g_n[r.kernel] += 1;
            }
        } else {
            ++g_errors;
        }
        g_pool.emplace_back(r.a, r.b);
    }
    g_pending.clear();
}

}  // namespace

namespace rt {

KernelTimer::KernelTimer(int k, hipStream_t s) : stream(s) {
    if (!g_on.load(std::memory_order_relaxed) || k < 0 || k >= KT_COUNT) return;
    hipEvent_t a = nullptr, b = nullptr;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        if (!g_pool.empty()) {
            a = g_pool.back().first;
            b = g_pool.back().second;
            g_pool.pop_back();
        }
    }
    if (a == nullptr && (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess)) {
        // the first event may exist when the second failed: do not leak it
        if (a != nullptr) (void)hipEventDestroy(a);
        a = b = nullptr;
        std::lock_guard<std::mutex> lk(g_mu);
        ++g_errors;
        return;
    }
    if (hipEventRecord(a, s) != hipSuccess) {
        std::lock_guard<std::mutex> lk(g_mu);
        g_pool.emplace_back(a, b);
        ++g_errors;
        return;
    }
    kernel = k;
    ev_a = a;
    ev_b = b;
}

// the pair joins the pending list only once both events are recorded, so a concurrent
// rt_ktime_read / rt_ktime_enable never recycles the events of an open scope
KernelTimer::~KernelTimer() {
    if (kernel < 0) return;
    const bool ok = hipEventRecord(ev_b, stream) == hipSuccess;
    std::lock_guard<std::mutex> lk(g_mu);
    if (ok) {
        g_pending.push_back(Rec{kernel, ev_a, ev_b});
    } else {
        ++g_errors;
        g_pool.emplace_back(ev_a, ev_b);
    }
}

int device_cu_count() {
    constexpr int kMaxDev = 64;
    static std::atomic<int> cache[kMaxDev];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0) return 256;
    if (dev < kMaxDev) {
        const int c = cache[dev].load(std::memory_order_relaxed);
        if (c > 0) return c;
    }
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    if (dev < kMaxDev) cache[dev].store(n, std::memory_order_relaxed);
    return n;
}

}  // namespace rt

extern "C" {

int rt_ktime_enable(int on) {
    std::lock_guard<std::mutex> lk(g_mu);
    drain(false);
    for (int k = 0; k < rt::KT_COUNT; ++k) {
        g_ms[k] = 0.0;
        g_n[k] = 0;
    }
    g_errors = 0;
    g_on.store(on != 0);
    return RT_OK;
}

int rt_ktime_read(int kernel, double* total_ms, int64_t* launches) {
    if (kernel < 0 || kernel >= rt::KT_COUNT) return rt::set_error(RT_E_INVALID, "bad kernel id");
    std::lock_guard<std::mutex> lk(g_mu);
    drain(true);
    if (g_errors) return rt::set_error(RT_E_HIP, "kernel timing: a HIP event call failed");
    if (total_ms) *total_ms = g_ms[kernel];
    if (launches) *launches = g_n[kernel];
    return RT_OK;
}

const char* rt_ktime_name(int kernel) {
    return (kernel >= 0 && kernel < rt::KT_COUNT) ? kNames[kernel] : nullptr;
}

}  // extern "C"
