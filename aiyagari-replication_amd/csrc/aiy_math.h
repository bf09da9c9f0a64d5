// Portable scalar math shared by the HIP kernels and the CPU oracle, so that every kernel
// reproduces the oracle bit for bit — including control flow that branches on function values
// (MATLAB fminbnd inside Krusell_Smith_VFI.m:164) and the EGM inversion RHS.^(-1/sigma),
// whose ulp-level differences the fine asset grid would otherwise amplify.
//
// aiy_log is the classic fdlibm __ieee754_log algorithm (argument reduction to [sqrt(2)/2,
// sqrt(2)), s = f/(2+f), degree-14 odd polynomial in s), written with plain IEEE double
// operations only.  Compiled with -ffp-contract=off on both sides it is bit-identical on
// host and device, and within 1 ulp of a correctly rounded log.
#ifndef AIY_MATH_H
#define AIY_MATH_H
#include <stdint.h>
#include <string.h>

#if defined(__HIPCC__)
#define AIY_HD __host__ __device__ __forceinline__
#else
#define AIY_HD static inline
#endif

AIY_HD uint64_t aiy_dbits(double x) {
    uint64_t u;
    memcpy(&u, &x, sizeof u);
    return u;
}
AIY_HD double aiy_bitsd(uint64_t u) {
    double x;
    memcpy(&x, &u, sizeof x);
    return x;
}

AIY_HD double aiy_log(double x) {
    const double ln2_hi = 6.93147180369123816490e-01;
    const double ln2_lo = 1.90821492927058770002e-10;
    const double two54 = 1.80143985094819840000e+16;
    const double Lg1 = 6.666666666666735130e-01;
    const double Lg2 = 3.999999999940941908e-01;
    const double Lg3 = 2.857142874366239149e-01;
    const double Lg4 = 2.222219843214978396e-01;
    const double Lg5 = 1.818357216161805012e-01;
    const double Lg6 = 1.531383769920937332e-01;
    const double Lg7 = 1.479819860511658591e-01;
    uint64_t u = aiy_dbits(x);
    int32_t hx = (int32_t)(u >> 32);
    uint32_t lx = (uint32_t)u;
    int32_t k = 0;
    if (hx < 0x00100000) {
        if (((hx & 0x7fffffff) | lx) == 0) return -__builtin_inf();
        if (hx < 0) return __builtin_nan("");
        k -= 54;
        x *= two54;
        u = aiy_dbits(x);
        hx = (int32_t)(u >> 32);
    }
    if (hx >= 0x7ff00000) return x + x;
    k += (hx >> 20) - 1023;
    hx &= 0x000fffff;
    int32_t i = (hx + 0x95f64) & 0x100000;
    u = aiy_dbits(x);
    u = ((uint64_t)(uint32_t)(hx | (i ^ 0x3ff00000)) << 32) | (u & 0xffffffffull);
    x = aiy_bitsd(u);
    k += (i >> 20);
    double f = x - 1.0;
    double dk;
    if ((0x000fffff & (2 + hx)) < 3) {
        if (f == 0.0) {
            if (k == 0) return 0.0;
            dk = (double)k;
            return dk * ln2_hi + dk * ln2_lo;
        }
        double R = f * f * (0.5 - 0.33333333333333333 * f);
        if (k == 0) return f - R;
        dk = (double)k;
        return dk * ln2_hi - ((R - dk * ln2_lo) - f);
    }
    double s = f / (2.0 + f);
    dk = (double)k;
    double z = s * s;
    i = hx - 0x6147a;
    double w = z * z;
    int32_t j = 0x6b851 - hx;
    double t1 = w * (Lg2 + w * (Lg4 + w * Lg6));
    double t2 = z * (Lg1 + w * (Lg3 + w * (Lg5 + w * Lg7)));
    i |= j;
    double R = t2 + t1;
    if (i > 0) {
        double hfsq = 0.5 * f * f;
        if (k == 0) return f - (hfsq - s * (hfsq + R));
        return dk * ln2_hi - ((hfsq - (s * (hfsq + R) + dk * ln2_lo)) - f);
    }
    if (k == 0) return f - s * (f - R);
    return dk * ln2_hi - ((s * (f - R) - dk * ln2_lo) - f);
}

// fdlibm __ieee754_exp: reduction x = k ln2 + r, |r| <= ln2/2, rational approximation of
// r(e^r+1)/(e^r-1) (Remez, degree 5), then scaling by 2^k.  Plain IEEE operations only.
AIY_HD double aiy_exp(double x) {
    const double o_threshold = 7.09782712893383973096e+02;
    const double u_threshold = -7.45133219101941108420e+02;
    const double ln2HI = 6.93147180369123816490e-01;
    const double ln2LO = 1.90821492927058770002e-10;
    const double invln2 = 1.44269504088896338700e+00;
    const double P1 = 1.66666666666666019037e-01;
    const double P2 = -2.77777777770155933842e-03;
    const double P3 = 6.61375632143793436117e-05;
    const double P4 = -1.65339022054652515390e-06;
    const double P5 = 4.13813679705723846039e-08;
    const double twom1000 = 9.33263618503218878990e-302;
    uint64_t u = aiy_dbits(x);
    uint32_t hx = (uint32_t)(u >> 32);
    int xsb = (int)((hx >> 31) & 1);
    hx &= 0x7fffffff;
    if (hx >= 0x40862E42) {
        if (hx >= 0x7ff00000) {
            if (((hx & 0xfffff) | (uint32_t)u) != 0) return x + x;
            return xsb == 0 ? x : 0.0;
        }
        if (x > o_threshold) return __builtin_inf();
        if (x < u_threshold) return 0.0;
    }
    double hi = 0.0, lo = 0.0;
    int k = 0;
    if (hx > 0x3fd62e42) {
        if (hx < 0x3FF0A2B2) {
            hi = xsb ? x + ln2HI : x - ln2HI;
            lo = xsb ? -ln2LO : ln2LO;
            k = 1 - xsb - xsb;
        } else {
            k = (int)(invln2 * x + (xsb ? -0.5 : 0.5));
            double t = (double)k;
            hi = x - t * ln2HI;
            lo = t * ln2LO;
        }
        x = hi - lo;
    } else if (hx < 0x3e300000) {
        return 1.0 + x;
    }
    double t = x * x;
    double c = x - t * (P1 + t * (P2 + t * (P3 + t * (P4 + t * P5))));
    if (k == 0) return 1.0 - ((x * c) / (c - 2.0) - x);
    double y = 1.0 - ((lo - (x * c) / (2.0 - c)) - hi);
    uint64_t yb = aiy_dbits(y);
    if (k >= -1021) {
        yb += (uint64_t)((int64_t)k * (int64_t)4503599627370496ll);  // k << 52
        return aiy_bitsd(yb);
    }
    yb += (uint64_t)((int64_t)(k + 1000) * (int64_t)4503599627370496ll);
    return aiy_bitsd(yb) * twom1000;
}

// c^n for integer n >= 1, MSB-first binary powering (the sequence np_oracle.ipow uses).
AIY_HD double aiy_ipow(double c, int n) {
    int top = 31 - __builtin_clz((unsigned)n);
    double r = c;
    for (int b = top - 1; b >= 0; --b) {
        r = r * r;
        if ((n >> b) & 1) r = r * c;
    }
    return r;
}

// x^y for the real powers the scripts use (c.^(1-sigma), RHS.^(-1/sigma), L.^(1+eta), ...):
// y == 1 → x; integer-valued y → binary powering (1/x^|y| for y < 0); otherwise
// exp(y·log x) for x > 0 (NaN for x < 0, as pow).  Identical on host and device.
AIY_HD double aiy_pow(double x, double y) {
    if (y == 1.0) return x;
    if (y == 0.0) return 1.0;
    double ay = y < 0 ? -y : y;
    if (ay < 64.0 && (double)(int)ay == ay) {
        double r = aiy_ipow(x, (int)ay);
        return y < 0 ? 1.0 / r : r;
    }
    if (x != x || y != y) return x + y;
    if (x == 0.0) return y < 0 ? __builtin_inf() : 0.0;
    if (x < 0.0) return __builtin_nan("");
    return aiy_exp(y * aiy_log(x));
}

#endif
