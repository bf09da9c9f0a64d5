// MATLAB pchip on the device (pchip.m slopes: Fritsch–Butland weighted harmonic mean, 3-point
// end rule; pwch coefficients + ppval Horner), shared by the KS VFI and KS EGM kernels.  The C
// oracle (oracle/aiy_oracle.c) uses the same formulas in the same order (-ffp-contract=off).
#pragma once
#include <hip/hip_runtime.h>

namespace aiy {

__device__ __forceinline__ int sgn_dev(double x) { return (x > 0) - (x < 0); }

// RN(a / b) for b > 0 from rb = RN(1 / b): q = RN(a·rb), then two residual corrections
// q += fma(−q, b, a)·rb (Markstein: with rb correctly rounded and q faithful, the corrected
// quotient is the correctly rounded one — no overflow or underflow here: grid spans and value
// differences; tools/micro/fastdiv_check.c: 2·10⁸ random and adversarial pairs, one correction
// misses 1, two miss 0).  A zero numerator keeps its sign, as IEEE a / b does for b > 0.  Five
// dependent fp64 operations instead of the eleven of the IEEE division sequence.
__device__ __forceinline__ double div_by_rcp(double a, double b, double rb) {
    double q = a * rb;
    double e = __builtin_fma(-q, b, a);
    q = __builtin_fma(e, rb, q);
    e = __builtin_fma(-q, b, a);
    q = __builtin_fma(e, rb, q);
    return a == 0.0 ? a : q;
}

// pchip slope at point q of a column (x = k_grid), MATLAB pchipslopes.  y is anything
// indexable by the column's node index: a column pointer, or a window staged in LDS (LdsCol).
template <class Y>
__device__ inline double pchip_slope_t(const double* __restrict__ x, const Y& y, int n, int q) {
    if (q == 0 || q == n - 1) {
        double h0, h1, e0, e1;
        if (q == 0) {
            h0 = x[1] - x[0];
            h1 = x[2] - x[1];
            e0 = (y[1] - y[0]) / h0;
            e1 = (y[2] - y[1]) / h1;
        } else {
            h0 = x[n - 1] - x[n - 2];
            h1 = x[n - 2] - x[n - 3];
            e0 = (y[n - 1] - y[n - 2]) / h0;
            e1 = (y[n - 2] - y[n - 3]) / h1;
        }
        double d = ((2 * h0 + h1) * e0 - h0 * e1) / (h0 + h1);
        if (sgn_dev(d) != sgn_dev(e0)) d = 0.0;
        else if (sgn_dev(e0) != sgn_dev(e1) && fabs(d) > fabs(3 * e0)) d = 3 * e0;
        return d;
    }
    int k = q - 1;
    double h1 = x[k + 1] - x[k], h2 = x[k + 2] - x[k + 1];
    double d1 = (y[k + 1] - y[k]) / h1, d2 = (y[k + 2] - y[k + 1]) / h2;
    if (sgn_dev(d1) * sgn_dev(d2) > 0) {
        double hs = h1 + h2;
        double w1 = (h1 + hs) / (3 * hs);
        double w2 = (hs + h2) / (3 * hs);
        double dmax = fmax(fabs(d1), fabs(d2));
        double dmin = fmin(fabs(d1), fabs(d2));
        return dmin / (w1 * (d1 / dmax) + w2 * (d2 / dmax));
    }
    return 0.0;
}
__device__ inline double pchip_slope(const double* __restrict__ x, const double* __restrict__ y,
                                     int n, int q) {
    return pchip_slope_t(x, y, n, q);
}

// the grid's slope tables (ks_grid_tables): rcp[i] = RN(1 / (x[i+1] − x[i])), i < n − 1, then
// w[2q], w[2q + 1] = the interior weights (h1 + hs) / (3·hs), (hs + h2) / (3·hs) of node q — the
// values pchip_slope_t computes, computed once per grid
__device__ __forceinline__ void pchip_grid_tables(const double* __restrict__ x, int n, int q,
                                                  double* __restrict__ tab) {
    if (q < n - 1) tab[q] = 1.0 / (x[q + 1] - x[q]);
    if (q >= 1 && q < n - 1) {
        const int k = q - 1;
        double h1 = x[k + 1] - x[k], h2 = x[k + 2] - x[k + 1];
        double hs = h1 + h2;
        tab[n + 2 * q] = (h1 + hs) / (3 * hs);
        tab[n + 2 * q + 1] = (hs + h2) / (3 * hs);
    }
}
// pchip_slope_t with the grid tables: the two interval slopes divide by the tabled reciprocals
// (div_by_rcp, correctly rounded), the weights are read, and of d1/dmax, d2/dmax the one whose
// magnitude is dmax is ±1 exactly — three IEEE divisions instead of seven, the same values
template <class Y>
__device__ inline double pchip_slope_tab(const double* __restrict__ x, const Y& y, int n, int q,
                                         const double* __restrict__ tab) {
    if (q == 0 || q == n - 1) return pchip_slope_t(x, y, n, q);
    int k = q - 1;
    double h1 = x[k + 1] - x[k], h2 = x[k + 2] - x[k + 1];
    double d1 = div_by_rcp(y[k + 1] - y[k], h1, tab[k]);
    double d2 = div_by_rcp(y[k + 2] - y[k + 1], h2, tab[k + 1]);
    if (sgn_dev(d1) * sgn_dev(d2) > 0) {
        const double w1 = tab[n + 2 * q], w2 = tab[n + 2 * q + 1];
        double dmax = fmax(fabs(d1), fabs(d2));
        double dmin = fmin(fabs(d1), fabs(d2));
        const double t1 = fabs(d1) == dmax ? copysign(1.0, d1) : d1 / dmax;
        const double t2 = fabs(d2) == dmax ? copysign(1.0, d2) : d2 / dmax;
        return dmin / (w1 * t1 + w2 * t2);
    }
    return 0.0;
}
// nodes [lo, lo + len) of a column staged in LDS, indexed by node
struct LdsCol {
    const double* p;
    int lo;
    __device__ double operator[](int i) const { return p[i - lo]; }
};

// a column element: plain load, or (SC1) an L1-bypassing agent-scope load — the consumer side
// of an in-kernel hand-off whose producer stored the bytes sc1 (MI355X_MICROARCH.md, the
// inter-workgroup visibility table's first row)
template <bool SC1>
__device__ __forceinline__ double col_ld(const double* p) {
    if constexpr (SC1)
        return __builtin_bit_cast(double, __hip_atomic_load(
            reinterpret_cast<const unsigned long long*>(p), __ATOMIC_RELAXED,
            __HIP_MEMORY_SCOPE_AGENT));
    else
        return *p;
}

// pwch coefficients + ppval Horner on segment i; rh = RN(1 / h) of the segment (the forecast
// queries of one node share the segment: one IEEE division for all of them)
template <bool SC1 = false>
__device__ __forceinline__ double pchip_at(const double* __restrict__ x,
                                           const double* __restrict__ y,
                                           const double* __restrict__ d, int i, double xq,
                                           double h, double rh) {
    const double y0 = col_ld<SC1>(y + i), y1 = col_ld<SC1>(y + i + 1);
    const double d0 = col_ld<SC1>(d + i), d1 = col_ld<SC1>(d + i + 1);
    double dl = div_by_rcp(y1 - y0, h, rh);
    double dzzdx = div_by_rcp(dl - d0, h, rh);
    double dzdxdx = div_by_rcp(d1 - dl, h, rh);
    double c3 = div_by_rcp(dzdxdx - dzzdx, h, rh);
    double c2 = 2 * dzzdx - dzdxdx;
    double sx = xq - x[i];
    double v = c3;
    v = sx * v + c2;
    v = sx * v + d0;
    v = sx * v + y0;
    return v;
}

// slope at point q of a (possibly two-point) knot set: MATLAB pchip is linear for n == 2
__device__ inline double pchip_slope_n(const double* __restrict__ x, const double* __restrict__ y,
                                       int n, int q) {
    if (n == 2) return (y[1] - y[0]) / (x[1] - x[0]);
    return pchip_slope(x, y, n, q);
}

// value of the pchip interpolant of (x, y) at xq on segment i, slopes computed locally
__device__ inline double pchip_local(const double* __restrict__ x, const double* __restrict__ y,
                                     int n, int i, double xq) {
    double d[2] = {pchip_slope_n(x, y, n, i), pchip_slope_n(x, y, n, i + 1)};
    double h = x[i + 1] - x[i];
    double dl = (y[i + 1] - y[i]) / h;
    double dzzdx = (dl - d[0]) / h;
    double dzdxdx = (d[1] - dl) / h;
    double c3 = (dzdxdx - dzzdx) / h;
    double c2 = 2 * dzzdx - dzdxdx;
    double sx = xq - x[i];
    double v = c3;
    v = sx * v + c2;
    v = sx * v + d[0];
    v = sx * v + y[i];
    return v;
}

}  // namespace aiy
