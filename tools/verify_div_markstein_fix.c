/* Exhaustive check (every float bit pattern, V = 1..VMAX) of the mean division the fused warp uses:
 *   q0 = a * r,  e = fma(-q0, V, a),  q = fma(e, r, q0),  q = (q is NaN) ? q0 : q,   r = (float)(1.0 / V)
 * against the IEEE quotient a / V (round to nearest even).  The NaN fix-up covers a = +-inf (e is NaN there; q0 is
 * the exact +-inf) and a = NaN.  The one remaining difference, a = -0 (q = +0), never reaches the division: the view
 * sum starts at +0 and x + y is -0 only when both are -0.  Prints, per V, the mismatches other than a = -0, and at
 * the end the bit mask of the V for which there are none (the kernel's table).  Build + run:
 *   gcc -O2 -mfma -fopenmp -ffp-contract=off tools/verify_div_markstein_fix.c -o /tmp/vdmf && /tmp/vdmf 64 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static inline float bits2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static inline uint32_t f2bits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }

int main(int argc, char **argv) {
    const int vmax = argc > 1 ? atoi(argv[1]) : 64;
    uint64_t good = 0;
    for (int V = 1; V <= vmax; ++V) {
        const float vf = (float)V, r = (float)(1.0 / (double)V);
        long long bad = 0;
#pragma omp parallel for reduction(+ : bad) schedule(static)
        for (long long k = 0; k < (1ll << 32); ++k) {
            if ((uint32_t)k == 0x80000000u) continue;  /* -0: see above */
            const float a = bits2f((uint32_t)k);
            const float ref = a / vf;
            const float q0 = a * r;
            const float e = fmaf(-q0, vf, a);
            float q = fmaf(e, r, q0);
            if (q != q) q = q0;
            if (!((isnan(ref) && isnan(q)) || f2bits(ref) == f2bits(q))) bad++;
        }
        printf("V=%d %s (%lld mismatches)\n", V, bad ? "FAILS" : "exact", bad);
        fflush(stdout);
        if (!bad) good |= 1ull << (V - 1);
    }
    printf("mask of exact V (bit V-1): 0x%016llx\n", (unsigned long long)good);
    return 0;
}
