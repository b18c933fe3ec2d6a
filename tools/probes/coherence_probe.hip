// Cross-kernel visibility probe: is a buffer rewritten between kernels (by an H2D copy,
// by a kernel, or after free/realloc) read fresh by every XCD's workgroups?
// hipcc --offload-arch=gfx950 -O2 tools/probes/coherence_probe.hip -o /tmp/coherence_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

constexpr int kWords = 1024;

__global__ void k_read(const unsigned* __restrict__ b, unsigned* __restrict__ out) {
    unsigned s = 0;
    for (int i = threadIdx.x; i < kWords; i += blockDim.x) s += b[i] * (unsigned)(i + 1);
    __shared__ unsigned red[256];
    red[threadIdx.x] = s;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
        __syncthreads();
    }
    if (threadIdx.x == 0) out[blockIdx.x] = red[0];
}
__global__ void k_write(unsigned* b, unsigned v) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < kWords; i += gridDim.x * blockDim.x) b[i] = v + i;
}
__global__ void k_read_scalar(const unsigned* __restrict__ b, unsigned* __restrict__ out) {
    // uniform addresses: scalar loads through the scalar cache
    typedef __attribute__((address_space(4))) const unsigned cu;
    cu* p = (cu*)b;
    unsigned s = 0;
    for (int i = 0; i < kWords; ++i) s += p[i] * (unsigned)(i + 1);
    if (threadIdx.x == 0) out[blockIdx.x] = s;
}

static unsigned expect(const std::vector<unsigned>& h) {
    unsigned s = 0;
    for (int i = 0; i < kWords; ++i) s += h[i] * (unsigned)(i + 1);
    return s;
}

int main() {
    const int nwg = 2048;
    unsigned *b, *out;
    CK(hipMalloc(&b, kWords * 4));
    CK(hipMalloc(&out, nwg * 4));
    std::vector<unsigned> h(kWords), o(nwg);
    auto check = [&](const char* what, unsigned want, bool scalar) {
        if (scalar) hipLaunchKernelGGL(k_read_scalar, dim3(nwg), dim3(64), 0, 0, b, out);
        else hipLaunchKernelGGL(k_read, dim3(nwg), dim3(256), 0, 0, b, out);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(o.data(), out, nwg * 4, hipMemcpyDeviceToHost));
        int bad = 0;
        for (int i = 0; i < nwg; ++i) bad += o[i] != want;
        printf("%-48s %s stale workgroups: %d of %d\n", what, scalar ? "scalar" : "vector", bad, nwg);
    };
    for (int scalar = 0; scalar < 2; ++scalar) {
        for (int i = 0; i < kWords; ++i) h[i] = 1000 + i;
        CK(hipMemcpy(b, h.data(), kWords * 4, hipMemcpyHostToDevice));
        check("H2D pattern 1", expect(h), scalar);
        for (int i = 0; i < kWords; ++i) h[i] = 2000 + 3 * i;
        CK(hipMemcpy(b, h.data(), kWords * 4, hipMemcpyHostToDevice));
        check("H2D pattern 2 over cached pattern 1", expect(h), scalar);
        hipLaunchKernelGGL(k_write, dim3(1), dim3(64), 0, 0, b, 7000u);
        for (int i = 0; i < kWords; ++i) h[i] = 7000 + i;
        check("kernel write (1 WG) over cached pattern 2", expect(h), scalar);
        std::vector<unsigned> back(kWords);
        CK(hipMemcpy(back.data(), b, kWords * 4, hipMemcpyDeviceToHost));
        hipLaunchKernelGGL(k_write, dim3(1), dim3(64), 0, 0, b, 9000u);
        for (int i = 0; i < kWords; ++i) h[i] = 9000 + i;
        check("D2H read, then kernel write (1 WG)", expect(h), scalar);
        CK(hipMemcpy(back.data(), b, kWords * 4, hipMemcpyDeviceToHost));
        CK(hipFree(b));
        CK(hipMalloc(&b, kWords * 4));
        for (int i = 0; i < kWords; ++i) h[i] = 5000 + 7 * i;
        CK(hipMemcpy(b, h.data(), kWords * 4, hipMemcpyHostToDevice));
        check("D2H read, free, malloc, H2D", expect(h), scalar);
        CK(hipMemcpy(back.data(), b, kWords * 4, hipMemcpyDeviceToHost));
        CK(hipFree(b));
        CK(hipMalloc(&b, kWords * 4));
        hipLaunchKernelGGL(k_write, dim3(1), dim3(64), 0, 0, b, 11000u);
        for (int i = 0; i < kWords; ++i) h[i] = 11000 + i;
        check("D2H read, free, malloc, kernel write", expect(h), scalar);
    }
    return 0;
}
