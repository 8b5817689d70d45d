/* Randomized host check of cell_ixy's division (bev_geometry.h): u0 / ws as IEEE fp32 versus
 *   rws = rcp(ws) refined by two Newton steps in double, q = (float)((double)u0 * rws).
 * v_rcp_f64's approximation is emulated by 1.0 / ws perturbed by a random relative error of up to 2^-20 (the
 * hardware's is far smaller); the two Newton steps take any such start to within ~2^-53.  Samples: |ws| from 1e-6
 * to 1e6 (log-uniform, both signs), u0 log-uniform over 1e-45..3e38 (both signs; subnormal, overflowing and subnormal-input cases included), plus zeros.  Any mismatch is
 * printed; exit status 1 if one is found.   gcc -O2 -o /tmp/vrw tools/verify_div_rcp_ws.c -lm && /tmp/vrw 200000000
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static uint64_t s = 0x9e3779b97f4a7c15ull;
static uint64_t nx(void) {
    s ^= s << 13;
    s ^= s >> 7;
    s ^= s << 17;
    return s;
}
static double unif(void) { return (double)(nx() >> 11) * (1.0 / 9007199254740992.0); }

int main(int argc, char **argv) {
    const long n = argc > 1 ? atol(argv[1]) : 100000000L;
    long bad = 0;
    for (long i = 0; i < n; ++i) {
        const float ws = (float)((nx() & 1 ? -1.0 : 1.0) * pow(10.0, -6.0 + 12.0 * unif()));
        float u0 = (float)((nx() & 1 ? -1.0 : 1.0) * pow(10.0, -45.0 + 83.5 * unif()));
        if ((i & 1023) == 0) u0 = 0.0f;
        if (fabsf(ws) < 1e-6f) continue;
        const double wd = (double)ws;
        double r = (1.0 / wd) * (1.0 + (unif() - 0.5) * 0x1p-19);  /* emulated rcp: error up to 2^-20 */
        r = fma(r, fma(-wd, r, 1.0), r);
        r = fma(r, fma(-wd, r, 1.0), r);
        const float q = (float)((double)u0 * r);
        const float ref = u0 / ws;
        if (memcmp(&q, &ref, 4) != 0 && !(q != q && ref != ref)) {
            if (bad < 10) printf("mismatch u0=%a ws=%a q=%a ref=%a\n", u0, ws, q, ref);
            ++bad;
        }
    }
    printf("%ld samples, %ld mismatches\n", n, bad);
    return bad != 0;
}
