// Probe (run once on the GPU box): (1) v_permlane32_swap / v_permlane16_swap lane
// semantics; (2) error of a 10-term f32 dot product evaluated as three bf16 products
// (hi*hi + lo*hi + hi*lo, K = 32) on v_mfma_f32_16x16x32_bf16, relative to the sum
// of the absolute values of the products, against a double evaluation.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include <random>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ void k_perm(unsigned* out) {
    const unsigned l = threadIdx.x;
    auto r = __builtin_amdgcn_permlane32_swap(l, 100u + l, false, false);
    out[l] = r[0];
    out[64 + l] = r[1];
    auto s = __builtin_amdgcn_permlane16_swap(l, 100u + l, false, false);
    out[128 + l] = s[0];
    out[192 + l] = s[1];
}

// A: 16 rows x 32 k (bf16, row-major), B: 32 k x 16 cols (bf16, col-major) per problem
__global__ void k_mm(const __bf16* A, const __bf16* B, float* C, int nprob) {
    const int p = blockIdx.x;
    if (p >= nprob) return;
    const int l = threadIdx.x;
    bf16x8 a, b;
    for (int j = 0; j < 8; ++j) {
        a[j] = A[(size_t)p * 512 + (l & 15) * 32 + 8 * (l >> 4) + j];
        b[j] = B[(size_t)p * 512 + (l & 15) * 32 + 8 * (l >> 4) + j];
    }
    f32x4 c = {0.f, 0.f, 0.f, 0.f};
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
    for (int i = 0; i < 4; ++i) C[(size_t)p * 256 + ((l >> 4) * 4 + i) * 16 + (l & 15)] = c[i];
}

static uint16_t bf16_bits(float x) {  // round to nearest even
    uint32_t u;
    std::memcpy(&u, &x, 4);
    u += 0x7fff + ((u >> 16) & 1);
    return (uint16_t)(u >> 16);
}
static float bf16_val(uint16_t h) {
    uint32_t u = (uint32_t)h << 16;
    float f;
    std::memcpy(&f, &u, 4);
    return f;
}

int main() {
    unsigned* dp;
    hipMalloc(&dp, 256 * 4);
    hipLaunchKernelGGL(k_perm, dim3(1), dim3(64), 0, 0, dp);
    unsigned hp[256];
    hipMemcpy(hp, dp, sizeof(hp), hipMemcpyDeviceToHost);
    const char* nm[4] = {"p32 r0", "p32 r1", "p16 r0", "p16 r1"};
    for (int t = 0; t < 4; ++t) {
        printf("%s:", nm[t]);
        for (int l = 0; l < 64; l += 8) printf(" [%d]=%u", l, hp[t * 64 + l]);
        printf("\n");
    }
    const int nprob = 4096;
    std::mt19937 rng(7);
    std::uniform_real_distribution<float> U(-1.f, 1.f);
    std::vector<uint16_t> A((size_t)nprob * 512), B((size_t)nprob * 512);
    std::vector<float> fa((size_t)nprob * 16 * 10), fb((size_t)nprob * 16 * 10);
    for (int p = 0; p < nprob; ++p) {
        for (int r = 0; r < 16; ++r)
            for (int k = 0; k < 10; ++k) {
                const float sa = std::ldexp(1.0f, (int)(rng() % 12) - 6);
                const float sb = std::ldexp(1.0f, (int)(rng() % 12) - 6);
                fa[((size_t)p * 16 + r) * 10 + k] = U(rng) * sa;
                fb[((size_t)p * 16 + r) * 10 + k] = U(rng) * sb;
            }
        for (int r = 0; r < 16; ++r) {
            uint16_t h[10], lo[10], hb[10], lb[10];
            for (int k = 0; k < 10; ++k) {
                const float x = fa[((size_t)p * 16 + r) * 10 + k];
                h[k] = bf16_bits(x);
                lo[k] = bf16_bits(x - bf16_val(h[k]));
                const float y = fb[((size_t)p * 16 + r) * 10 + k];
                hb[k] = bf16_bits(y);
                lb[k] = bf16_bits(y - bf16_val(hb[k]));
            }
            uint16_t* ar = &A[(size_t)p * 512 + r * 32];
            uint16_t* bc = &B[(size_t)p * 512 + r * 32];
            for (int k = 0; k < 32; ++k) ar[k] = bc[k] = 0;
            for (int k = 0; k < 10; ++k) {
                ar[k] = h[k];       bc[k] = hb[k];
                ar[10 + k] = lo[k]; bc[10 + k] = hb[k];
                ar[20 + k] = h[k];  bc[20 + k] = lb[k];
            }
        }
    }
    __bf16 *dA, *dB;
    float* dC;
    hipMalloc(&dA, A.size() * 2);
    hipMalloc(&dB, B.size() * 2);
    hipMalloc(&dC, (size_t)nprob * 256 * 4);
    hipMemcpy(dA, A.data(), A.size() * 2, hipMemcpyHostToDevice);
    hipMemcpy(dB, B.data(), B.size() * 2, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_mm, dim3(nprob), dim3(64), 0, 0, dA, dB, dC, nprob);
    std::vector<float> C((size_t)nprob * 256);
    hipMemcpy(C.data(), dC, C.size() * 4, hipMemcpyDeviceToHost);
    double worst = 0.0, worst_trunc = 0.0;
    for (int p = 0; p < nprob; ++p)
        for (int r = 0; r < 16; ++r)
            for (int c = 0; c < 16; ++c) {
                double ex = 0.0, ab = 0.0, em = 0.0;
                for (int k = 0; k < 10; ++k) {
                    const double x = fa[((size_t)p * 16 + r) * 10 + k], y = fb[((size_t)p * 16 + c) * 10 + k];
                    ex += x * y;
                    ab += fabs(x * y);
                }
                // the exact value of the three bf16 products (what a perfect accumulator gives)
                for (int k = 0; k < 32; ++k)
                    em += (double)bf16_val(A[(size_t)p * 512 + r * 32 + k]) * (double)bf16_val(B[(size_t)p * 512 + c * 32 + k]);
                const double got = C[(size_t)p * 256 + r * 16 + c];
                worst = fmax(worst, fabs(got - ex) / ab);
                worst_trunc = fmax(worst_trunc, fabs(got - em) / ab);
            }
    printf("max |mfma - exact| / sum|a b| = %.3e (= %.2f * 2^-16)\n", worst, worst * 65536.0);
    printf("max |mfma - exact bf16 products| / sum|a b| = %.3e (= %.2f * 2^-24)\n", worst_trunc,
           worst_trunc * 16777216.0);
    return 0;
}
