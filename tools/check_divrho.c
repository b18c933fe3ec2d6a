/* Exhaustive host check of div_rho (rt_math.hpp): x / RHO by one multiplication and
 * one FMA residual step (zeros passed through), RHO = RN(1 / (2 RN(pi))) (GPU/constants/image_settings.h:14).
 * Compares with IEEE x / RHO for every float x = +-0 or |x| in [2^-100, 2^100].
 *   gcc -O2 -fopenmp -ffp-contract=off tools/check_divrho.c -o /tmp/check_divrho -lm */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
int main(void) {
    const float rho = 1.0f / (2.0f * 3.14159265358979323846f);
    const float c = 1.0f / rho;
    unsigned long long bad = 0, tested = 0;
#pragma omp parallel for reduction(+ : bad, tested) schedule(static)
    for (long long b = 0; b < (1ll << 32); ++b) {
        uint32_t u = (uint32_t)b;
        float x;
        memcpy(&x, &u, 4);
        if (x != x) continue;
        if (!(fabsf(x) >= 0x1p-100f && fabsf(x) <= 0x1p100f) && x != 0.0f) continue;
        const float ref = x / rho;
        const float q = x * c;
        const float r = fmaf(-q, rho, x);
        const float q2 = (x == 0.0f) ? x : fmaf(r, c, q);  /* -0 keeps its sign */
        uint32_t a1, a2;
        memcpy(&a1, &ref, 4);
        memcpy(&a2, &q2, 4);
        ++tested;
        if (a1 != a2) { ++bad; printf("x=%a ref=%a got=%a\n", x, ref, q2); }
    }
    printf("rho %a  1/rho %a  tested %llu  mismatches %llu\n", rho, c, tested, bad);
    return bad != 0;
}
