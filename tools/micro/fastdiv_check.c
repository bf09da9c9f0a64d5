// Exhaustive-by-sampling check of division by a precomputed reciprocal:
//   y = RN(1/b); q0 = RN(a*y); e0 = fma(-q0, b, a); q1 = fma(e0, y, q0);
//   e1 = fma(-q1, b, a); q2 = fma(e1, y, q1)            (q2 claimed == RN(a/b))
// Markstein: if y is within 1/2 ulp of 1/b and q1 is faithful, RN(q1 + (a - b q1) y) = RN(a/b).
// Counts mismatches of q1 (one correction) and q2 (two) against IEEE a/b.
//   gcc -O2 -mfma -ffp-contract=off fastdiv_check.c -lm && ./a.out N seed
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static uint64_t s[2];
static uint64_t nxt(void) {  // xorshift128+
    uint64_t x = s[0], y = s[1];
    s[0] = y; x ^= x << 23; s[1] = x ^ y ^ (x >> 17) ^ (y >> 26);
    return s[1] + y;
}
static double bits(uint64_t u) { double d; memcpy(&d, &u, 8); return d; }
static uint64_t ub(double d) { uint64_t u; memcpy(&u, &d, 8); return u; }
// random double with exponent in [e0, e1] and random sign
static double rnd(int e0, int e1) {
    uint64_t m = nxt() & ((1ull << 52) - 1);
    int e = e0 + (int)(nxt() % (uint64_t)(e1 - e0 + 1));
    uint64_t sg = nxt() & 1;
    return bits((sg << 63) | ((uint64_t)(e + 1023) << 52) | m);
}

int main(int argc, char** argv) {
    long long n = argc > 1 ? atoll(argv[1]) : 100000000LL;
    s[0] = 0x9E3779B97F4A7C15ull ^ (argc > 2 ? atoll(argv[2]) : 1); s[1] = 0xD1B54A32D192ED03ull;
    long long bad1 = 0, bad2 = 0, bad0 = 0;
    for (long long i = 0; i < n; ++i) {
        double a, b;
        switch (i & 3) {
            case 0: a = rnd(-60, 60); b = rnd(-60, 60); break;         // general
            case 1: a = rnd(-40, 4); b = fabs(rnd(-30, 4)); break;       // grid-like spans
            case 2: {  // a close to a multiple of b (quotients near simple values)
                b = fabs(rnd(-20, 4));
                double q = (double)(int64_t)(nxt() % 4096) / 64.0 + bits(ub(1.0) + (nxt() % 64)) - 1.0;
                a = q * b;
                a = bits(ub(a) + (int64_t)(nxt() % 5) - 2);
                break;
            }
            default: {  // b with many trailing ones / zeros in the significand
                uint64_t m = (nxt() & 1) ? ((1ull << 52) - 1) ^ (nxt() & 0xFF) : (nxt() & 0xFF);
                b = bits(((uint64_t)(1023 + (int)(nxt() % 8) - 4) << 52) | m);
                a = rnd(-10, 10);
            }
        }
        if (b == 0.0 || !isfinite(a) || !isfinite(b)) continue;
        double ref = a / b;
        double y = 1.0 / b;
        double q0 = a * y;
        double e0 = fma(-q0, b, a);
        double q1 = fma(e0, y, q0);
        double e1 = fma(-q1, b, a);
        double q2 = fma(e1, y, q1);
        if (ub(q0) != ub(ref)) ++bad0;
        if (ub(q1) != ub(ref)) ++bad1;
        if (ub(q2) != ub(ref)) {
            if (bad2 < 10) printf("MISMATCH a=%a b=%a ref=%a q2=%a\n", a, b, ref, q2);
            ++bad2;
        }
    }
    printf("n=%lld  q0(RN(a*y)) mismatches %lld  one correction %lld  two corrections %lld\n", n,
           bad0, bad1, bad2);
    return bad2 != 0;
}
