/* Exhaustive check of the division-by-constant sequence used by the HIP march
 * (DESIGN.md §5): for a divisor a with y = RN(1/a),
 *   q0 = RN(d*y); r0 = fma(-q0,a,d); q1 = fma(r0,y,q0); r1 = fma(-q1,a,d); q2 = fma(r1,y,q1)
 * must equal the IEEE quotient RN(d/a) for every float d in [1e-4, 1.0002].
 * The one-correction quotient q1 is counted too (the kernels use q1 since
 * this check found it exact: Markstein's theorem with y = RN(1/a), q0
 * faithful).  Divisors: a few fixed, 32 adversarial mantissas, then random.
 * Build: gcc -O2 -mfma -ffp-contract=off -fopenmp markstein_check.c -lm */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static float u2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static uint32_t f2u(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }

int main(int argc, char **argv) {
    int ndiv = argc > 1 ? atoi(argv[1]) : 64;
    uint32_t lo = f2u(1e-4f), hi = f2u(1.0002f);
    unsigned long long bad_total = 0, bad1_total = 0, n_total = 0;
    srand(12345);
    for (int k = 0; k < ndiv; k++) {
        float a;
        if (k == 0) a = 0.7287353f; else if (k == 1) a = 0.42073548f; else if (k == 2) a = 0.5403023f;
        else if (k == 3) a = 1.0f; else if (k == 4) a = 0.5f; else if (k == 5) a = u2f(0x3f7fffff);
        else if (k == 6) a = u2f(0x3f000001); else if (k == 7) a = 1e-3f; else if (k == 8) a = 3e-7f;
        /* adversarial mantissas: all ones, one ulp above/below powers of two, alternating bits */
        else if (k < 9 + 32) {
            static const uint32_t m[8] = {0x7fffff, 0x000001, 0x7ffffe, 0x000002, 0x555555, 0x2aaaaa, 0x400000, 0x3fffff};
            a = u2f(((uint32_t)(100 + (k - 9) / 8 * 7) << 23) | m[(k - 9) % 8]);
        }
        else a = u2f(0x30000000u + (uint32_t)(((unsigned long long)rand() * 2654435761ull) % 0x0f800000u));
        float y = 1.0f / a;
        unsigned long long bad = 0, bad1 = 0, n = 0;
#pragma omp parallel for reduction(+ : bad, bad1, n) schedule(static)
        for (long long u = lo; u <= (long long)hi; u++) {
            float d = u2f((uint32_t)u);
            float q = d / a;
            float q0 = d * y;
            float r0 = fmaf(-q0, a, d);
            float q1 = fmaf(r0, y, q0);
            float r1 = fmaf(-q1, a, d);
            float q2 = fmaf(r1, y, q1);
            bad += f2u(q2) != f2u(q);
            bad1 += f2u(q1) != f2u(q);
            n++;
        }
        bad_total += bad; bad1_total += bad1; n_total += n;
        if (bad) printf("divisor %a: %llu mismatches (two-step)\n", a, bad);
    }
    printf("divisors %d, quotients %llu, two-step mismatches %llu, one-step mismatches %llu\n", ndiv, n_total,
           bad_total, bad1_total);
    return bad_total != 0;
}
