/* Exhaustive host check of div12 (rt_math.hpp): x / 12 by one multiplication and one FMA
 * residual step, compared with IEEE x / 12.0f for every float of its domain, x = +0 or
 * |x| in [2^-100, 2^100] (the grid coordinates cell + jitter are +0 or in [2^-24, 12]).
 * The device form of the same check: rt_selftest(RT_SELFTEST_DIV12).
 *   gcc -O2 -fopenmp -ffp-contract=off tools/check_div12.c -o /tmp/check_div12 -lm */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
int main(void) {
    const float c = 1.0f / 12.0f;
    unsigned long long bad = 0, tested = 0;
#pragma omp parallel for reduction(+ : bad, tested) schedule(static)
    for (long long b = 0; b < (1ll << 32); ++b) {
        uint32_t u = (uint32_t)b;
        float x;
        memcpy(&x, &u, 4);
        if (x != x) continue;
        if (!(u == 0u || (fabsf(x) >= 0x1p-100f && fabsf(x) <= 0x1p100f))) continue;
        const float ref = x / 12.0f;
        const float q = x * c;
        const float r = fmaf(-q, 12.0f, x);
        const float q2 = fmaf(r, c, q);
        uint32_t a1, a2;
        memcpy(&a1, &ref, 4);
        memcpy(&a2, &q2, 4);
        ++tested;
        if (a1 != a2) ++bad;
    }
    printf("tested %llu  mismatches %llu\n", tested, bad);
    return bad != 0;
}
