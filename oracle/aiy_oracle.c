/* C restatement of kostastril/Aiyagari-Replication's hot-path loops — TEST INFRASTRUCTURE.
 * See aiy_oracle.h for the status line ("parity unpinned against MATLAB") and layouts.
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off -fopenmp).  Every function follows the
 * MATLAB evaluation order of the cited lines; OpenMP only distributes independent states. */
#include "aiy_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#include "../aiyagari-replication_amd/csrc/aiy_math.h" /* aiy_log (KS only), aiy_ipow */

int orc_num_threads(int n) {
#ifdef _OPENMP
    if (n > 0) omp_set_num_threads(n);
    return omp_get_max_threads();
#else
    (void)n;
    return 1;
#endif
}


/* Powers and logs use the portable aiy_pow / aiy_log (aiy_math.h, shared with the kernels):
 * integer exponents by binary powering, otherwise exp(y*log x) in plain IEEE operations, so
 * the restatement and the HIP kernels agree bit for bit.  MATLAB's own libm is unpinned. */
/* c.^(1-sigma)  (Aiyagari_VFI.m:77) */
static double crra_p(double c, double sigma) { return aiy_pow(c, 1.0 - sigma); }
/* c.^(-sigma)  (Aiyagari_EGM.m:68) */
static double uprime(double c, double sigma) { return aiy_pow(c, -sigma); }

/* (beta*P(i,:))*v_old(:,k), m ascending (Aiyagari_VFI.m:79) */
static void ev_rows(int64_t N, int64_t Na, const double* P, const double* V, double beta,
                    double* EV) {
#pragma omp parallel for schedule(static)
    for (int64_t ik = 0; ik < N * Na; ++ik) {
        int64_t i = ik / Na, k = ik % Na;
        double acc = 0.0;
        for (int64_t m = 0; m < N; ++m) acc = acc + (beta * P[i * N + m]) * V[m * Na + k];
        EV[ik] = acc;
    }
}

/* ------------------------------------------------------------------ A1 / A2 */
int orc_vfi_sweep(int64_t N, int64_t Na, const double* v_old, const double* a_grid,
                  const double* s, const double* P, double r, double w, double beta,
                  double sigma, double* v_new, int32_t* idx, double* policy_k,
                  double* policy_c) {
    double* EV = (double*)malloc(sizeof(double) * N * Na);
    if (!EV) return 1;
    ev_rows(N, Na, P, v_old, beta, EV);
#pragma omp parallel for schedule(dynamic, 16)
    for (int64_t ij = 0; ij < N * Na; ++ij) {
        int64_t i = ij / Na, j = ij % Na;
        const double* ev = EV + i * Na;
        double coh = (1 + r) * a_grid[j] + w * s[i]; /* :72 */
        double best = NAN;
        int64_t bk = -1;
        for (int64_t k = 0; k < Na; ++k) {
            double c = coh - a_grid[k];
            if (c <= 0) continue; /* :73 NaN, ignored by max */
            double u = (sigma == 1.0) ? aiy_log(c) : (crra_p(c, sigma) - 1) / (1 - sigma);
            double val = u + ev[k];
            if (isnan(val)) continue;
            if (bk < 0 || val > best) { /* first maximiser */
                best = val;
                bk = k;
            }
        }
        if (bk < 0) bk = 0; /* max of all-NaN: NaN, index 1 */
        v_new[ij] = best;
        idx[ij] = (int32_t)bk;
        policy_k[ij] = a_grid[bk];            /* :80 */
        policy_c[ij] = ((1 + r) * a_grid[j] + w * s[i]) - policy_k[ij]; /* :81 */
    }
    free(EV);
    return 0;
}

static double nanmax_absdiff(int64_t n, const double* a, const double* b) {
    double m = NAN;
    for (int64_t i = 0; i < n; ++i) {
        double d = fabs(a[i] - b[i]);
        if (isnan(d)) continue;
        if (isnan(m) || d > m) m = d;
    }
    return m;
}

int orc_vfi_solve(int64_t N, int64_t Na, double* v_old, const double* a_grid, const double* s,
                  const double* P, double r, double w, double beta, double sigma, double tol,
                  int64_t max_iter, double* v_new, int32_t* idx, double* policy_k,
                  double* policy_c, int64_t* iters) {
    int64_t it = 0;
    for (it = 1; it <= max_iter; ++it) {
        orc_vfi_sweep(N, Na, v_old, a_grid, s, P, r, w, beta, sigma, v_new, idx, policy_k,
                      policy_c);
        double d = nanmax_absdiff(N * Na, v_new, v_old);
        if (d < tol) break;                        /* :85-86 */
        memcpy(v_old, v_new, sizeof(double) * N * Na); /* :88 */
    }
    if (it > max_iter) it = max_iter;
    *iters = it;
    return 0;
}

/* ------------------------------------------------------------------ A3 */
int orc_labor_vfi_sweep(int64_t N, int64_t Na, int64_t Nl, const double* v_old,
                        const double* a_grid, const double* s, const double* P,
                        const double* L, double r, double w, double beta, double sigma,
                        double psi, double eta, double* v_new, double* policy_k,
                        double* policy_l, double* policy_c, int32_t* lin) {
    double* EV = (double*)malloc(sizeof(double) * N * Na);
    double* dis = (double*)malloc(sizeof(double) * Nl);
    if (!EV || !dis) return 1;
    ev_rows(N, Na, P, v_old, beta, EV); /* :69 EV = beta*P*v_old */
    for (int64_t l = 0; l < Nl; ++l) {
        double e1 = 1 + eta;
        double Lp = aiy_pow(L[l], e1);
        dis[l] = psi * Lp / (1 + eta); /* :96 */
    }
#pragma omp parallel for schedule(dynamic, 16)
    for (int64_t ij = 0; ij < N * Na; ++ij) {
        int64_t i = ij / Na, j = ij % Na;
        const double* ev = EV + i * Na;
        double x = (1 + r) * a_grid[j];
        double y = w * s[i];
        double best = 0, bc = 0;
        int64_t bq = -1;
        int any = 0;
        for (int64_t k = 0; k < Na; ++k) {          /* column-major scan: k outer, l inner */
            for (int64_t l = 0; l < Nl; ++l) {
                double c = (x + y * L[l]) - a_grid[k]; /* :81 */
                double val;
                if (c > 0) {
                    any = 1;
                    /* :95 has no sigma == 1 branch (0/0 = NaN there, as in MATLAB) */
                    double u = (crra_p(c, sigma) - 1) / (1 - sigma);
                    val = (u - dis[l]) + ev[k];        /* :95-99 */
                } else {
                    val = -INFINITY + ev[k];           /* utility = -Inf */
                }
                if (isnan(val)) continue;
                if (bq < 0 || val > best) {
                    best = val;
                    bq = l + Nl * k;
                    bc = c;
                }
            }
        }
        if (!any) continue; /* :85 keep previous values */
        if (bq < 0) bq = 0;
        int64_t li = bq % Nl, ki = bq / Nl;
        policy_l[ij] = L[li];
        policy_k[ij] = a_grid[ki];
        policy_c[ij] = bc;
        lin[ij] = (int32_t)bq;
        v_new[ij] = best;
    }
    free(EV);
    free(dis);
    return 0;
}

int orc_labor_vfi_solve(int64_t N, int64_t Na, int64_t Nl, double* v_old, const double* a_grid,
                        const double* s, const double* P, const double* L, double r, double w,
                        double beta, double sigma, double psi, double eta, double tol,
                        int64_t max_iter, double* v_new, double* policy_k, double* policy_l,
                        double* policy_c, int32_t* lin, int64_t* iters) {
    int64_t it;
    for (it = 1; it <= max_iter; ++it) {
        orc_labor_vfi_sweep(N, Na, Nl, v_old, a_grid, s, P, L, r, w, beta, sigma, psi, eta,
                            v_new, policy_k, policy_l, policy_c, lin);
        if (nanmax_absdiff(N * Na, v_new, v_old) < tol) break;
        memcpy(v_old, v_new, sizeof(double) * N * Na);
    }
    if (it > max_iter) it = max_iter;
    *iters = it;
    return 0;
}

/* ------------------------------------------------------------------ interp1 */
static int64_t seg_of(int64_t n, const double* x, double q) {
    /* largest i with x[i] <= q, clamped to [0, n-2] */
    int64_t lo = 0, hi = n; /* first index with x > q */
    while (lo < hi) {
        int64_t mid = (lo + hi) >> 1;
        if (x[mid] <= q) lo = mid + 1;
        else hi = mid;
    }
    int64_t i = lo - 1;
    if (i < 0) i = 0;
    if (i > n - 2) i = n - 2;
    return i;
}
static double interp_one(int64_t n, const double* x, const double* y, int64_t ystride,
                         double q) {
    int64_t i = seg_of(n, x, q);
    double t = (q - x[i]) / (x[i + 1] - x[i]);
    double y0 = y[i * ystride], y1 = y[(i + 1) * ystride];
    return y0 + t * (y1 - y0);
}
void orc_interp1(int64_t n, const double* x, const double* y, int64_t nq, const double* xq,
                 double* out) {
    for (int64_t q = 0; q < nq; ++q) out[q] = interp_one(n, x, y, 1, xq[q]);
}

/* ------------------------------------------------------------------ A4 / A5 */
static void egm_rhs(int64_t N, int64_t Na, const double* c, const double* P, double r,
                    double beta, double sigma, double* RHS) {
#pragma omp parallel for schedule(static)
    for (int64_t ja = 0; ja < N * Na; ++ja) {
        int64_t j = ja / Na, a = ja % Na;
        double acc = 0.0;
        for (int64_t m = 0; m < N; ++m)
            acc = acc + ((beta * (1 + r)) * P[j * N + m]) * uprime(c[m * Na + a], sigma);
        RHS[ja] = acc;
    }
}

int orc_egm_step(int64_t N, int64_t Na, const double* pc, const double* a_grid,
                 const double* s, const double* P, double r, double w, double beta,
                 double sigma, double amin, double* pcn, double* pk, double* dist) {
    double* RHS = (double*)malloc(sizeof(double) * N * Na);
    double* ah = (double*)malloc(sizeof(double) * N * Na);
    if (!RHS || !ah) return 1;
    egm_rhs(N, Na, pc, P, r, beta, sigma, RHS);
    for (int64_t ja = 0; ja < N * Na; ++ja) {
        int64_t j = ja / Na, a = ja % Na;
        double cn = aiy_pow(RHS[ja], -1.0 / sigma);       /* :88 */
        ah[ja] = ((cn + a_grid[a]) - w * s[j]) / (1 + r);  /* :92 */
    }
#pragma omp parallel for schedule(static)
    for (int64_t ja = 0; ja < N * Na; ++ja) {
        int64_t j = ja / Na, a = ja % Na;
        double g = interp_one(Na, ah + j * Na, a_grid, 1, a_grid[a]); /* :95 */
        if (g < amin) g = amin;                                          /* :98 */
        pk[ja] = g;
        pcn[ja] = ((1 + r) * a_grid[a] + w * s[j]) - g;                 /* :102 */
    }
    *dist = nanmax_absdiff(N * Na, pcn, pc);
    free(RHS);
    free(ah);
    return 0;
}

int orc_egm_solve(int64_t N, int64_t Na, double* pc, const double* a_grid, const double* s,
                  const double* P, double r, double w, double beta, double sigma, double amin,
                  double tol, int64_t max_iter, double* pk, double* dist, int64_t* iters) {
    double* nxt = (double*)malloc(sizeof(double) * N * Na);
    if (!nxt) return 1;
    double d = 1.0;
    int64_t it = 0;
    while (d > tol && it < max_iter) {
        ++it;
        orc_egm_step(N, Na, pc, a_grid, s, P, r, w, beta, sigma, amin, nxt, pk, &d);
        memcpy(pc, nxt, sizeof(double) * N * Na);
    }
    free(nxt);
    *dist = d;
    *iters = it;
    return 0;
}

static double labor_of(double c, double ws, double sigma, double phi, double theta) {
    double x = (ws * uprime(c, sigma)) / phi;
    return (1.0 / theta == 1.0) ? x : aiy_pow(x, 1.0 / theta);
}

int orc_labor_egm_step(int64_t N, int64_t Na, const double* pc, const double* a_grid,
                       const double* s, const double* P, double r, double w, double beta,
                       double sigma, double phi, double theta, double amin, double* pcn,
                       double* pk, double* pl, double* dist) {
    double* RHS = (double*)malloc(sizeof(double) * N * Na);
    double* ah = (double*)malloc(sizeof(double) * N * Na);
    double* cn = (double*)malloc(sizeof(double) * N * Na);
    if (!RHS || !ah || !cn) return 1;
    egm_rhs(N, Na, pc, P, r, beta, sigma, RHS);
    for (int64_t ja = 0; ja < N * Na; ++ja) {
        int64_t j = ja / Na, a = ja % Na;
        double ws = w * s[j];
        cn[ja] = aiy_pow(RHS[ja], -1.0 / sigma);                    /* :82 */
        double ls = labor_of(cn[ja], ws, sigma, phi, theta);          /* :86 */
        ah[ja] = ((cn[ja] + a_grid[a]) - ws * ls) / (1 + r);          /* :87 */
    }
#pragma omp parallel for schedule(static)
    for (int64_t ja = 0; ja < N * Na; ++ja) {
        int64_t j = ja / Na, a = ja % Na;
        double ws = w * s[j];
        double g = interp_one(Na, ah + j * Na, cn + j * Na, 1, a_grid[a]); /* :90 */
        if (a_grid[a] < amin) g = amin;                                       /* :91 */
        pcn[ja] = g;
        pl[ja] = labor_of(g, ws, sigma, phi, theta);                          /* :95 */
        double k = ((1 + r) * a_grid[a] + ws * pl[ja]) - g;                   /* :98 */
        pk[ja] = (k < 0) ? 0.0 : k;                                           /* :99 */
    }
    *dist = nanmax_absdiff(N * Na, pcn, pc);
    free(RHS);
    free(ah);
    free(cn);
    return 0;
}

int orc_labor_egm_solve(int64_t N, int64_t Na, double* pc, const double* a_grid,
                        const double* s, const double* P, double r, double w, double beta,
                        double sigma, double phi, double theta, double amin, double tol,
                        int64_t max_iter, double* pk, double* pl, double* dist,
                        int64_t* iters) {
    double* nxt = (double*)malloc(sizeof(double) * N * Na);
    if (!nxt) return 1;
    double d = 1.0;
    int64_t it = 0;
    while (d > tol && it < max_iter) {
        ++it;
        orc_labor_egm_step(N, Na, pc, a_grid, s, P, r, w, beta, sigma, phi, theta, amin, nxt,
                           pk, pl, &d);
        memcpy(pc, nxt, sizeof(double) * N * Na);
    }
    free(nxt);
    *dist = d;
    *iters = it;
    return 0;
}

/* ------------------------------------------------------------------ A9 */
int orc_sim_capital(int64_t N, int64_t Na, const double* pol, int64_t zs, int64_t as,
                    const double* a_grid, const double* P, int64_t z1, double k1, int64_t T,
                    const double* U, double* mean_k, double* sim_k) {
    double* cs = (double*)malloc(sizeof(double) * N * N);
    if (!cs) return 1;
    for (int64_t z = 0; z < N; ++z) {
        double acc = 0.0;
        for (int64_t m = 0; m < N; ++m) {
            acc = acc + P[z * N + m];
            cs[z * N + m] = acc;
        }
    }
    int64_t z = z1;
    double k = k1, sum = k1;
    if (sim_k) sim_k[0] = k1;
    for (int64_t t = 1; t < T; ++t) {
        double u = U[t - 1];
        int64_t zn = -1;
        for (int64_t m = 0; m < N; ++m)
            if (u < cs[z * N + m]) { zn = m; break; }
        if (zn < 0) { free(cs); return 2; } /* find() empty → MATLAB assignment error */
        z = zn;
        k = interp_one(Na, a_grid, pol + z * zs, as, k); /* :113 */
        if (sim_k) sim_k[t] = k;
        sum += k;
    }
    *mean_k = sum / (double)T;
    free(cs);
    return 0;
}

/* ------------------------------------------------------------------ A10 (new) */
/* A10 (new; no reference code).  The mass of destination (i,k) is the sum of the terms that
 * land there, in ascending source j, summed sequentially in chunks of ORC_DIST_CHUNK terms with
 * the chunk sums summed sequentially (the definition the HIP kernels follow,
 * csrc/dist.hpp kDistChunk): runs of <= 32 terms are the plain sequential scatter. */
#define ORC_DIST_CHUNK 32
typedef struct { double *tot, *part; int* cnt; } orc_mass_acc;
static int mass_acc_init(orc_mass_acc* m, int64_t n) {
    m->tot = (double*)calloc((size_t)n, sizeof(double));
    m->part = (double*)calloc((size_t)n, sizeof(double));
    m->cnt = (int*)calloc((size_t)n, sizeof(int));
    return !(m->tot && m->part && m->cnt);
}
static void mass_acc_add(orc_mass_acc* m, int64_t q, double x) {
    m->part[q] = m->part[q] + x;
    if (++m->cnt[q] == ORC_DIST_CHUNK) {
        m->tot[q] = m->tot[q] + m->part[q];
        m->part[q] = 0.0;
        m->cnt[q] = 0;
    }
}
/* finish the chunks and project: out(m,k) = sum_i P(i,m) mass(i,k), i ascending */
static void mass_acc_project(orc_mass_acc* m, int64_t N, int64_t Na, const double* P,
                             double* out) {
#pragma omp parallel for schedule(static)
    for (int64_t q = 0; q < N * Na; ++q)
        if (m->cnt[q]) m->tot[q] = m->tot[q] + m->part[q];
#pragma omp parallel for schedule(static)
    for (int64_t c = 0; c < N; ++c)
        for (int64_t k = 0; k < Na; ++k) {
            double acc = 0.0;
            for (int64_t i = 0; i < N; ++i) acc = acc + P[i * N + c] * m->tot[i * Na + k];
            out[c * Na + k] = acc;
        }
}
static void mass_acc_free(orc_mass_acc* m) {
    free(m->tot);
    free(m->part);
    free(m->cnt);
}

int orc_dist_update_ongrid(int64_t N, int64_t Na, const double* lam, const int32_t* idx,
                           const double* P, double* out) {
    orc_mass_acc m;
    if (mass_acc_init(&m, N * Na)) { mass_acc_free(&m); return 1; }
    /* rows are independent (source row i lands in destination row i): threads over rows keep
     * every destination's term order */
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < N; ++i)
        for (int64_t j = 0; j < Na; ++j) mass_acc_add(&m, i * Na + idx[i * Na + j], lam[i * Na + j]);
    mass_acc_project(&m, N, Na, P, out);
    mass_acc_free(&m);
    return 0;
}

int orc_dist_update_lottery(int64_t N, int64_t Na, const double* lam, const double* kp,
                            const double* a_grid, const double* P, double* out) {
    orc_mass_acc m;
    if (mass_acc_init(&m, N * Na)) { mass_acc_free(&m); return 1; }
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < N; ++i)
        for (int64_t j = 0; j < Na; ++j) {
            double x = kp[i * Na + j];
            if (x < a_grid[0]) x = a_grid[0];
            if (x > a_grid[Na - 1]) x = a_grid[Na - 1];
            int64_t k = seg_of(Na, a_grid, x);
            double wr = (x - a_grid[k]) / (a_grid[k + 1] - a_grid[k]);
            mass_acc_add(&m, i * Na + k, lam[i * Na + j] * (1 - wr));
            mass_acc_add(&m, i * Na + k + 1, lam[i * Na + j] * wr);
        }
    mass_acc_project(&m, N, Na, P, out);
    mass_acc_free(&m);
    return 0;
}

int orc_dist_stationary(int64_t N, int64_t Na, const int32_t* idx, const double* kp,
                        const double* a_grid, const double* P, double tol, int64_t max_iter,
                        double* lam, double* K, int64_t* iters, double* dist) {
    double* nxt = (double*)malloc(sizeof(double) * N * Na);
    if (!nxt) return 1;
    int64_t it;
    double d = NAN;
    for (it = 1; it <= max_iter; ++it) {
        if (idx) orc_dist_update_ongrid(N, Na, lam, idx, P, nxt);
        else orc_dist_update_lottery(N, Na, lam, kp, a_grid, P, nxt);
        d = nanmax_absdiff(N * Na, nxt, lam);
        memcpy(lam, nxt, sizeof(double) * N * Na);
        if (d < tol) break;
    }
    if (it > max_iter) it = max_iter;
    double acc = 0.0;
    for (int64_t i = 0; i < N; ++i)
        for (int64_t j = 0; j < Na; ++j) acc = acc + lam[i * Na + j] * a_grid[j];
    *K = acc;
    *iters = it;
    *dist = d;
    free(nxt);
    return 0;
}

/* ------------------------------------------------------------------ A6 / A7 */
static int sgn(double x) { return (x > 0) - (x < 0); }

void orc_pchip_slopes(int64_t n, const double* x, const double* y, double* d) {
    for (int64_t k = 0; k + 2 < n; ++k) {
        double h1 = x[k + 1] - x[k], h2 = x[k + 2] - x[k + 1];
        double d1 = (y[k + 1] - y[k]) / h1, d2 = (y[k + 2] - y[k + 1]) / h2;
        double dk = 0.0;
        if (sgn(d1) * sgn(d2) > 0) {
            double hs = h1 + h2;
            double w1 = (h1 + hs) / (3 * hs);
            double w2 = (hs + h2) / (3 * hs);
            double dmax = fmax(fabs(d1), fabs(d2));
            double dmin = fmin(fabs(d1), fabs(d2));
            dk = dmin / (w1 * (d1 / dmax) + w2 * (d2 / dmax));
        }
        d[k + 1] = dk;
    }
    double h0 = x[1] - x[0], h1 = x[2] - x[1];
    double e0 = (y[1] - y[0]) / h0, e1 = (y[2] - y[1]) / h1;
    double d0 = ((2 * h0 + h1) * e0 - h0 * e1) / (h0 + h1);
    if (sgn(d0) != sgn(e0)) d0 = 0.0;
    else if (sgn(e0) != sgn(e1) && fabs(d0) > fabs(3 * e0)) d0 = 3 * e0;
    d[0] = d0;
    double hn = x[n - 1] - x[n - 2], hm = x[n - 2] - x[n - 3];
    double en = (y[n - 1] - y[n - 2]) / hn, em = (y[n - 2] - y[n - 3]) / hm;
    double dn = ((2 * hn + hm) * en - hn * em) / (hn + hm);
    if (sgn(dn) != sgn(en)) dn = 0.0;
    else if (sgn(en) != sgn(em) && fabs(dn) > fabs(3 * en)) dn = 3 * en;
    d[n - 1] = dn;
}

double orc_pchip_eval(int64_t n, const double* x, const double* y, const double* d,
                      double xq) {
    int64_t i = seg_of(n, x, xq);
    double h = x[i + 1] - x[i];
    double dl = (y[i + 1] - y[i]) / h;
    double dzzdx = (dl - d[i]) / h;
    double dzdxdx = (d[i + 1] - dl) / h;
    double c3 = (dzdxdx - dzzdx) / h;
    double c2 = 2 * dzzdx - dzdxdx;
    double sx = xq - x[i];
    double v = c3;
    v = sx * v + c2;
    v = sx * v + d[i];
    v = sx * v + y[i];
    return v;
}

/* bellman_value (Krusell_Smith_VFI.m:329-364).  V,dV column-major k x K x S. */
double orc_ks_bellman(const orc_ks_params* p, int64_t nk, int64_t nK, const double* k_grid,
                      const double* K_grid, const double* V, const double* dV, const double* B,
                      const double* P, double kp, int64_t k_i, int64_t K_i, int64_t s_i) {
    double z = p->z_grid[(s_i + 1 <= 2) ? 1 : 0]; /* :332 flipped */
    double K = K_grid[K_i], k = k_grid[k_i];
    double Kp;
    if (z == p->z_grid[0]) Kp = exp(B[0] + B[1] * log(fmax(K, 1e-8)));
    else Kp = exp(B[2] + B[3] * log(fmax(K, 1e-8)));
    Kp = fmax(fmin(Kp, K_grid[nK - 1]), K_grid[0]);
    int64_t Kp_idx = 0;
    double bd = fabs(K_grid[0] - Kp);
    for (int64_t q = 1; q < nK; ++q) {
        double dd = fabs(K_grid[q] - Kp);
        if (dd < bd) { bd = dd; Kp_idx = q; }
    }
    double expec = 0;
    double kq = fmax(fmin(kp, k_grid[nk - 1]), k_grid[0]);
    for (int64_t sn = 0; sn < 4; ++sn) {
        const double* col = V + (sn * nK + Kp_idx) * nk;
        const double* dcol = dV + (sn * nK + Kp_idx) * nk;
        expec = expec + P[s_i * 4 + sn] * orc_pchip_eval(nk, k_grid, col, dcol, kq);
    }
    double L = p->l_bar * (1 - p->ug * (double)(z == p->z_grid[0]) -
                           p->ub * (double)(z == p->z_grid[1]));
    double r_val = p->alpha * z * pow(K, p->alpha - 1) * pow(L, 1 - p->alpha);
    double w_val = (1 - p->alpha) * z * pow(K, p->alpha) * pow(L, -p->alpha);
    double eps = (s_i % 2 == 0) ? p->eps_grid[0] : p->eps_grid[1]; /* s_grid(s_i,2) */
    double c = (r_val + 1 - p->delta) * k + w_val * (eps * p->l_bar) - kp;
    c = fmax(c, 1e-10);
    return aiy_log(c) + p->beta * expec;
}

double orc_fminbnd_ks(const orc_ks_params* p, int64_t nk, int64_t nK, const double* k_grid,
                      const double* K_grid, const double* V, const double* dV, const double* B,
                      const double* P, int64_t k_i, int64_t K_i, int64_t s_i, double ax,
                      double bx, int32_t* nfev) {
#define F(X) (-orc_ks_bellman(p, nk, nK, k_grid, K_grid, V, dV, B, P, (X), k_i, K_i, s_i))
    const double seps = sqrt(2.220446049250313e-16), tolx = 1e-4;
    const double cg = 0.5 * (3.0 - sqrt(5.0));
    double a = ax, b = bx, v = a + cg * (b - a), w = v, xf = v, d = 0, e = 0, x = xf;
    double fx = F(x);
    int num = 1, it = 0;
    double fv = fx, fw = fx, xm = 0.5 * (a + b);
    double tol1 = seps * fabs(xf) + tolx / 3.0, tol2 = 2.0 * tol1;
    while (fabs(xf - xm) > (tol2 - 0.5 * (b - a))) {
        int gs = 1;
        if (fabs(e) > tol1) {
            gs = 0;
            double r = (xf - w) * (fx - fv);
            double q = (xf - v) * (fx - fw);
            double pp = (xf - v) * q - (xf - w) * r;
            q = 2.0 * (q - r);
            if (q > 0.0) pp = -pp;
            q = fabs(q);
            r = e;
            e = d;
            if (fabs(pp) < fabs(0.5 * q * r) && pp > q * (a - xf) && pp < q * (b - xf)) {
                d = pp / q;
                x = xf + d;
                if ((x - a) < tol2 || (b - x) < tol2) {
                    double si = sgn(xm - xf) + ((xm - xf) == 0);
                    d = tol1 * si;
                }
            } else {
                gs = 1;
            }
        }
        if (gs) {
            e = (xf >= xm) ? (a - xf) : (b - xf);
            d = cg * e;
        }
        double si = sgn(d) + (d == 0);
        x = xf + si * fmax(fabs(d), tol1);
        double fu = F(x);
        ++num;
        ++it;
        if (fu <= fx) {
            if (x >= xf) a = xf;
            else b = xf;
            v = w; fv = fw;
            w = xf; fw = fx;
            xf = x; fx = fu;
        } else {
            if (x < xf) a = x;
            else b = x;
            if (fu <= fw || w == xf) {
                v = w; fv = fw;
                w = x; fw = fu;
            } else if (fu <= fv || v == xf || v == w) {
                v = x; fv = fu;
            }
        }
        xm = 0.5 * (a + b);
        tol1 = seps * fabs(xf) + tolx / 3.0;
        tol2 = 2.0 * tol1;
        if (num >= 500 || it >= 500) break;
    }
    if (nfev) *nfev = num;
    return xf;
#undef F
}

static void ks_all_slopes(int64_t nk, int64_t nK, const double* k_grid, const double* V,
                          double* dV) {
    for (int64_t c = 0; c < 4 * nK; ++c) orc_pchip_slopes(nk, k_grid, V + c * nk, dV + c * nk);
}

int orc_ks_policy_improve(const orc_ks_params* p, int64_t nk, int64_t nK, const double* k_grid,
                          const double* K_grid, const double* V, const double* B,
                          const double* P, const double* s_grid, double* k_opt,
                          int32_t* nfev) {
    (void)s_grid;
    double* dV = (double*)malloc(sizeof(double) * nk * nK * 4);
    if (!dV) return 1;
    ks_all_slopes(nk, nK, k_grid, V, dV);
#pragma omp parallel for schedule(dynamic, 4)
    for (int64_t n = 0; n < nk * nK * 4; ++n) {
        int64_t k_i = n % nk, K_i = (n / nk) % nK, s_i = n / (nk * nK);
        double zt = (s_i < 2) ? p->z_grid[0] : p->z_grid[1]; /* s_grid(s_i,1), :19-20 */
        double eps = (s_i % 2 == 0) ? p->eps_grid[0] : p->eps_grid[1];
        double K = K_grid[K_i];
        double L = p->l_bar * (1 - p->ug * (double)(zt == p->z_grid[0]) -
                               p->ub * (double)(zt == p->z_grid[1])); /* :112 */
        double wt = (1 - p->alpha) * zt * pow(K, p->alpha) * pow(L, -p->alpha);
        double rt = p->alpha * zt * pow(K, p->alpha - 1) * pow(L, 1 - p->alpha);
        double res = (rt + 1 - p->delta) * k_grid[k_i] +
                     wt * (eps * p->l_bar + (1 - eps) * p->mu); /* :152-153 */
        double kpmax = fmin(res, p->k_max);                       /* :159 */
        int32_t nf = 0;
        k_opt[n] = orc_fminbnd_ks(p, nk, nK, k_grid, K_grid, V, dV, B, P, k_i, K_i, s_i,
                                  p->k_min, kpmax, &nf);          /* :164 */
        if (nfev) nfev[n] = nf;
    }
    free(dV);
    return 0;
}

int orc_ks_howard(const orc_ks_params* p, int64_t nk, int64_t nK, const double* k_grid,
                  const double* K_grid, double* V, const double* k_opt, const double* B,
                  const double* P, int64_t steps) {
    int64_t n_all = nk * nK * 4;
    double* dV = (double*)malloc(sizeof(double) * n_all);
    double* Vn = (double*)malloc(sizeof(double) * n_all);
    if (!dV || !Vn) return 1;
    for (int64_t h = 0; h < steps; ++h) { /* :172-192, Jacobi */
        ks_all_slopes(nk, nK, k_grid, V, dV);
#pragma omp parallel for schedule(static)
        for (int64_t n = 0; n < n_all; ++n) {
            int64_t k_i = n % nk, K_i = (n / nk) % nK, s_i = n / (nk * nK);
            Vn[n] = orc_ks_bellman(p, nk, nK, k_grid, K_grid, V, dV, B, P, k_opt[n], k_i, K_i,
                                   s_i);
        }
        memcpy(V, Vn, sizeof(double) * n_all);
    }
    free(dV);
    free(Vn);
    return 0;
}

/* ------------------------------------------------------------------ A8 (KS EGM) */
/* Per (s_i, K_i) scalars, Krusell_Smith_EGM.m:101-112, :139-175 (libm pow/exp/log).
 * s_grid = [Z(:), Eps(:)] of meshgrid(z_grid, eps_grid): s = (z1,e1), (z1,e2), (z2,e1), (z2,e2). */
void orc_ks_egm_pairs(const orc_ks_params* p, int64_t nK, const double* K_grid, const double* B,
                      orc_ks_egm_pair* out) {
    const double* zg = p->z_grid;
    const double* eg = p->eps_grid;
    const double a = p->alpha, dl = p->delta, lb = p->l_bar;
    for (int64_t s_i = 0; s_i < 4; ++s_i) {
        double z = zg[s_i < 2 ? 0 : 1], e = eg[s_i % 2];
        for (int64_t K_i = 0; K_i < nK; ++K_i) {
            orc_ks_egm_pair* q = out + s_i * nK + K_i;
            double K = K_grid[K_i];
            double L = lb * (1 - p->ug * (double)(z == zg[0]) - p->ub * (double)(z == zg[1]));
            double r = a * z * pow(K, a - 1) * pow(L, 1 - a);
            double w = (1 - a) * z * pow(K, a) * pow(L, -a);
            double Kp = (z == zg[0]) ? exp(B[0] + B[1] * log(K)) : exp(B[2] + B[3] * log(K));
            for (int s_j = 0; s_j < 4; ++s_j) {
                double zn = zg[s_j < 2 ? 0 : 1], en = eg[s_j % 2];
                double Kd = (zn == zg[0]) ? exp(B[0] + B[1] * log(Kp)) : exp(B[2] + B[3] * log(Kp));
                int64_t idx = 0;
                double bd = fabs(K_grid[0] - Kd);
                for (int64_t m = 1; m < nK; ++m) {
                    double dd = fabs(K_grid[m] - Kd);
                    if (dd < bd) { bd = dd; idx = m; }
                }
                double Ln = lb * (1 - p->ug * (double)(zn == zg[0]) - p->ub * (double)(zn == zg[1]));
                double rn = a * zn * pow(Kd, a - 1) * pow(Ln, 1 - a);
                double wn = (1 - a) * zn * pow(Kd, a) * pow(Ln, -a);
                q->kd[s_j] = (int32_t)idx;
                q->Rn[s_j] = (1 + rn) - dl;
                q->Wn[s_j] = (wn * en) * lb;
            }
            q->R = (1 + r) - dl;
            q->We = (w * e) * lb;
        }
    }
}

/* pchip slopes for n >= 2 (pchip.m: n == 2 is linear) */
static void pchip_slopes_n(int64_t n, const double* x, const double* y, double* d) {
    if (n == 2) {
        d[0] = d[1] = (y[1] - y[0]) / (x[1] - x[0]);
        return;
    }
    orc_pchip_slopes(n, x, y, d);
}

/* One Gauss-Seidel sweep (Krusell_Smith_EGM.m:133-200); k_opt k x K x S column-major. */
/* One sweep over the (s_i, K_i) pairs reading the next-period policy from `src` and writing
 * each pair's column of `dst`: src == dst is the script's Gauss-Seidel order
 * (Krusell_Smith_EGM.m:199 overwrites k_opt in place); src = a copy of the sweep's input is the
 * Jacobi variant (F1, not the reference's result). */
static int ks_egm_sweep2(const orc_ks_params* p, int64_t nk, int64_t nK, const double* k_grid,
                         const orc_ks_egm_pair* pairs, const double* P, const double* src,
                         double* dst);
int orc_ks_egm_sweep(const orc_ks_params* p, int64_t nk, int64_t nK, const double* k_grid,
                     const orc_ks_egm_pair* pairs, const double* P, double* k_opt) {
    return ks_egm_sweep2(p, nk, nK, k_grid, pairs, P, k_opt, k_opt);
}
static int ks_egm_sweep2(const orc_ks_params* p, int64_t nk, int64_t nK, const double* k_grid,
                         const orc_ks_egm_pair* pairs, const double* P, const double* src,
                         double* k_opt) {
    double* d4 = (double*)malloc(sizeof(double) * 4 * nk);
    double* kc = (double*)malloc(sizeof(double) * nk);
    int64_t* ord = (int64_t*)malloc(sizeof(int64_t) * nk);
    double* xs = (double*)malloc(sizeof(double) * nk);
    double* ys = (double*)malloc(sizeof(double) * nk);
    double* dd = (double*)malloc(sizeof(double) * nk);
    int rc = 0;
    for (int64_t s_i = 0; s_i < 4 && rc == 0; ++s_i)
        for (int64_t K_i = 0; K_i < nK && rc == 0; ++K_i) {
            const orc_ks_egm_pair* q = pairs + s_i * nK + K_i;
            const double* col[4];
            for (int s_j = 0; s_j < 4; ++s_j) {
                col[s_j] = src + ((int64_t)s_j * nK + q->kd[s_j]) * nk;
                orc_pchip_slopes(nk, k_grid, col[s_j], d4 + s_j * nk);
            }
            for (int64_t t = 0; t < nk; ++t) {
                double kp = k_grid[t], em = 0.0;
                for (int s_j = 0; s_j < 4; ++s_j) {
                    double kpn = orc_pchip_eval(nk, k_grid, col[s_j], d4 + s_j * nk, kp);
                    double cn = (q->Rn[s_j] * kp + q->Wn[s_j]) - kpn;
                    cn = fmax(cn, 1e-8); /* MATLAB max ignores NaN, as fmax */
                    em = em + (P[s_i * 4 + s_j] * q->Rn[s_j]) / cn;
                }
                double c = 1 / (p->beta * em);
                kc[t] = ((c + kp) - q->We) / q->R;
            }
            /* stable ascending sort, NaN last (MATLAB sort) */
            for (int64_t t = 0; t < nk; ++t) ord[t] = t;
            for (int64_t t = 1; t < nk; ++t) {
                int64_t v = ord[t];
                int64_t u = t;
                while (u > 0) {
                    double a0 = kc[ord[u - 1]], b0 = kc[v];
                    int gt = (a0 != a0) ? (b0 == b0) : (b0 == b0 && a0 > b0);
                    if (!gt) break;
                    ord[u] = ord[u - 1];
                    --u;
                }
                ord[u] = v;
            }
            int64_t nv = 0;
            for (int64_t t = 0; t < nk; ++t) {
                double x = kc[ord[t]];
                if (x >= p->k_min && x <= p->k_max) {
                    xs[nv] = x;
                    ys[nv] = k_grid[ord[t]];
                    ++nv;
                }
            }
            if (nv < 2) {
                rc = -2;
                break;
            }
            pchip_slopes_n(nv, xs, ys, dd);
            double* out = k_opt + (s_i * nK + K_i) * nk;
            for (int64_t t = 0; t < nk; ++t) {
                double kq = k_grid[t], v;
                if (kq < xs[0]) v = ys[0];
                else if (kq > xs[nv - 1]) v = ys[nv - 1];
                else v = orc_pchip_eval(nv, xs, ys, dd, kq);
                v = fmin(v, p->k_max);
                out[t] = fmax(v, p->k_min);
            }
        }
    free(d4); free(kc); free(ord); free(xs); free(ys); free(dd);
    return rc;
}

int orc_ks_egm_solve(const orc_ks_params* p, int64_t nk, int64_t nK, const double* k_grid,
                     const double* K_grid, const double* B, const double* P, double tol,
                     int64_t max_iter, double* k_opt, int64_t* iters, double* diff) {
    orc_ks_egm_pair* pairs = (orc_ks_egm_pair*)malloc(sizeof(orc_ks_egm_pair) * 4 * nK);
    double* old = (double*)malloc(sizeof(double) * nk * nK * 4);
    orc_ks_egm_pairs(p, nK, K_grid, B, pairs);
    int rc = 0;
    int64_t it;
    double dmax = NAN;
    for (it = 1; it <= max_iter; ++it) {
        memcpy(old, k_opt, sizeof(double) * nk * nK * 4);
        rc = orc_ks_egm_sweep(p, nk, nK, k_grid, pairs, P, k_opt);
        if (rc) break;
        dmax = NAN;
        for (int64_t n = 0; n < nk * nK * 4; ++n) {
            double d = fabs(k_opt[n] - old[n]);
            if (d == d && !(dmax >= d)) dmax = d;
        }
        if (dmax < tol) break;
    }
    if (it > max_iter) it = max_iter;
    *iters = it;
    *diff = dmax;
    free(pairs);
    free(old);
    return rc;
}

/* F1: the Jacobi variant of the KS EGM iteration (every pair of a sweep reads the previous
 * sweep's k_opt) — NOT the reference's result (the script is Gauss-Seidel, :199); same stop
 * rule (:204-207). */
int orc_ks_egm_solve_jacobi(const orc_ks_params* p, int64_t nk, int64_t nK, const double* k_grid,
                            const double* K_grid, const double* B, const double* P, double tol,
                            int64_t max_iter, double* k_opt, int64_t* iters, double* diff) {
    orc_ks_egm_pair* pairs = (orc_ks_egm_pair*)malloc(sizeof(orc_ks_egm_pair) * 4 * nK);
    double* old = (double*)malloc(sizeof(double) * nk * nK * 4);
    orc_ks_egm_pairs(p, nK, K_grid, B, pairs);
    int rc = 0;
    int64_t it;
    double dmax = NAN;
    for (it = 1; it <= max_iter; ++it) {
        memcpy(old, k_opt, sizeof(double) * nk * nK * 4);
        rc = ks_egm_sweep2(p, nk, nK, k_grid, pairs, P, old, k_opt);
        if (rc) break;
        dmax = NAN;
        for (int64_t n = 0; n < nk * nK * 4; ++n) {
            double d = fabs(k_opt[n] - old[n]);
            if (d == d && !(dmax >= d)) dmax = d;
        }
        if (dmax < tol) break;
    }
    if (it > max_iter) it = max_iter;
    *iters = it;
    *diff = dmax;
    free(pairs);
    free(old);
    return rc;
}
