/* Exhaustive check (every float bit pattern, every V in 1..VMAX) that the FMA division by a small integer
 *   q0 = a * r,  e = fma(-q0, V, a),  q = fma(e, r, q0),   r = (float)(1.0 / V)
 * returns exactly the IEEE quotient a / V (round to nearest even), so the fused warp's mean may divide by the
 * camera count with three f32 operations (Markstein's correction step).  Build + run:
 *   gcc -O2 -mfma -fopenmp -ffp-contract=off tools/verify_div_markstein.c -o /tmp/vdm && /tmp/vdm 64
 * Prints the V for which it holds for ALL inputs (NaN: both NaN). */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static inline float bits2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static inline uint32_t f2bits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }

int main(int argc, char **argv) {
    int vmax = argc > 1 ? atoi(argv[1]) : 64;
    for (int V = 1; V <= vmax; ++V) {
        const float vf = (float)V, r = (float)(1.0 / (double)V);
        long long bad = 0;
        uint32_t first_bad = 0;
#pragma omp parallel for reduction(+ : bad) schedule(static)
        for (long long k = 0; k < (1ll << 32); ++k) {
            const float a = bits2f((uint32_t)k);
            const float ref = a / vf;
            const float q0 = a * r;
            const float e = fmaf(-q0, vf, a);
            const float q = fmaf(e, r, q0);
            const int ok = (isnan(ref) && isnan(q)) || f2bits(ref) == f2bits(q);
            if (!ok) {
                bad++;
                first_bad = (uint32_t)k;
            }
        }
        printf("V=%d %s (%lld mismatches%s%08x)\n", V, bad ? "FAILS" : "exact", bad, bad ? ", e.g. 0x" : " ",
               bad ? first_bad : 0u);
        fflush(stdout);
    }
    return 0;
}
