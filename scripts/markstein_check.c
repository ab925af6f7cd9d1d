/* Checks the sequential FGS solver's division (stereo_depth_ruler_amd/csrc/sdr_wls.hip div_by):
 *   q0 = x * r,  rem = -fma(q0, den, -x),  q = fma(rem, r, q0)      (r = 1/den, correctly rounded)
 * against the IEEE quotient x / den, for den >= 1 (every FGS pivot is) and |q0| >= 2^-96 (the
 * kernel redoes a chunk with real divisions when some 0 < |q0| < 2^-96).  Random den over
 * [1, 2^102) (every pivot the accepted lambdas reach: den <= 1 + 2 lambda, lambda <= 2^100), random x of either sign (subnormals included) with |x / den| from 2^-150 to 2^100;
 * counts, separately, the mismatches below the threshold (the inputs the redo exists for).
 * Optional second argument: the threshold's exponent (default -96); third: den's exponent range
 * (default 102; round 5 checked 60).
 *   gcc -O2 -mfma -o /tmp/markstein scripts/markstein_check.c -lm && /tmp/markstein 2000000000
 * (-mfma: fmaf must be the fused instruction; x86-64 with FMA3.)  Round 5 result: no mismatch at
 * or above the threshold in 2e9 pairs with den < 2^60 (x from the subnormal range up, zeros of both
 * signs); round 6 the same over den < 2^102: profiles/r6_markstein_check.txt. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static uint64_t s = 88172645463325252ull;
static inline uint64_t rnd(void) {
    s ^= s << 13;
    s ^= s >> 7;
    s ^= s << 17;
    return s;
}
static inline float fbits(uint32_t u) {
    float f;
    memcpy(&f, &u, 4);
    return f;
}
static inline uint32_t ubits(float f) {
    uint32_t u;
    memcpy(&u, &f, 4);
    return u;
}

int main(int argc, char** argv) {
    const long n = argc > 1 ? atol(argv[1]) : 100000000L;
    const float thr = argc > 2 ? ldexpf(1.0f, atoi(argv[2])) : 0x1p-96f;  /* the redo threshold */
    const int dmax = argc > 3 ? atoi(argv[3]) : 102;
    long bad = 0, below = 0, below_bad = 0;
    for (long i = 0; i < n; i++) {
        const int de = (int)(rnd() % (uint64_t)dmax);         /* den in [2^de, 2^(de+1)) */
        const float den = fbits((uint32_t)(127 + de) << 23 | (uint32_t)(rnd() & 0x7fffff));
        const int qe = -150 + (int)(rnd() % 250);             /* |x / den| ~ 2^qe */
        const int xe = qe + de;
        if (xe < -149 || xe > 127) continue;
        /* x: normal, or subnormal (a random multiple of 2^-149 below 2^(xe+1)) */
        const float x = xe >= -126
            ? fbits((uint32_t)(rnd() & 1) << 31 | (uint32_t)(127 + xe) << 23 | (uint32_t)(rnd() & 0x7fffff))
            : fbits((uint32_t)(rnd() & 1) << 31 | (uint32_t)(rnd() & ((1u << (xe + 150)) - 1)));
        const volatile float r = 1.0f / den;
        const float q0 = x * r;
        /* (volatile: gcc folds -fma(a, b, -c) into fnmadd, -(a b) + c, which loses the sign of a
         * zero remainder; the kernel's fma with a negated addend and a negated first operand
         * keeps it) */
        const volatile float e = fmaf(q0, den, -x);
        const float rem = -e;
        const float q = fmaf(rem, r, q0);
        const volatile float ref = x / den;
        const int tiny = fabsf(q0) < thr && q0 != 0.0f;
        if (tiny) below++;
        if (ubits(q) != ubits(ref)) {
            if (tiny) below_bad++;
            else {
                if (bad < 10) printf("mismatch x=%a den=%a ref=%a got=%a\n", x, den, ref, q);
                bad++;
            }
        }
    }
    printf("n=%ld mismatches(|q0| >= threshold)=%ld  below the threshold: %ld pairs, %ld mismatches\n", n, bad, below,
           below_bad);
    return bad != 0;
}
