#include <stdio.h>
#include <math.h>
#include <stdint.h>
#include <string.h>
int main(void){
  const float c = 1.0f/12.0f;
  unsigned long long bad = 0; uint32_t first = 0;
  for (uint64_t b = 0; b < (1ull<<32); ++b) {
    uint32_t u = (uint32_t)b; float x; memcpy(&x,&u,4);
    if (x != x) continue; if (!(fabsf(x) >= 0x1p-100f && fabsf(x) <= 0x1p100f) && x != 0.0f) continue;
    float ref = x / 12.0f;
    float q = x * c;
    float r = fmaf(-q, 12.0f, x);
    float q2 = fmaf(r, c, q);
    uint32_t a1, a2; memcpy(&a1,&ref,4); memcpy(&a2,&q2,4);
    if (a1 != a2) { if (!bad) first = u; ++bad; }
  }
  printf("mismatches %llu first %08x\n", bad, first);
  return 0;
}
