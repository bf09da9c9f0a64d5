/* C restatement of the reference's hot-path loops (kostastril/Aiyagari-Replication).
 *
 * TEST INFRASTRUCTURE ONLY: linked by tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg, never by the product library.  Parity against MATLAB is UNPINNED (no
 * MATLAB/Octave in the image, no fixtures in the reference); this restatement is pinned by
 * the independent numpy restatement (oracle/np_oracle.py) through tests/golden/.
 *
 * Layouts (row-major C arrays):
 *   VFI arrays  v[i*Na + j]   = v_old(i+1, j+1)          (N x Na)
 *   EGM arrays  c[j*Na + a]   = policy_c(a+1, j+1)       (Na x N column-major == [N][Na])
 *   P[i*N + m]                = P(i+1, m+1)
 *   KS value    V[(s*K + Ki)*k + ki] = value(ki+1, Ki+1, s+1)   (column-major k x K x S)
 * Indices returned are 0-based.
 */
#ifndef AIY_ORACLE_H
#define AIY_ORACLE_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

int orc_num_threads(int n); /* set OpenMP threads (0 = leave); returns active count */

/* A1: Aiyagari_VFI.m:70-83 */
int orc_vfi_sweep(int64_t N, int64_t Na, const double* v_old, const double* a_grid,
                  const double* s, const double* P, double r, double w, double beta,
                  double sigma, double* v_new, int32_t* idx, double* policy_k,
                  double* policy_c);
/* A2: Aiyagari_VFI.m:65-90 (v_old in/out = previous iterate at the break) */
int orc_vfi_solve(int64_t N, int64_t Na, double* v_old, const double* a_grid, const double* s,
                  const double* P, double r, double w, double beta, double sigma, double tol,
                  int64_t max_iter, double* v_new, int32_t* idx, double* policy_k,
                  double* policy_c, int64_t* iters);

/* A3: Aiyagari_Endogenous_Labor_VFI.m:69-112.  v_new/policies in/out (kept where no choice
 * is feasible).  lin = 0-based column-major index l + Nl*k. */
int orc_labor_vfi_sweep(int64_t N, int64_t Na, int64_t Nl, const double* v_old,
                        const double* a_grid, const double* s, const double* P,
                        const double* labor_choice, double r, double w, double beta,
                        double sigma, double psi, double eta, double* v_new, double* policy_k,
                        double* policy_l, double* policy_c, int32_t* lin);
int orc_labor_vfi_solve(int64_t N, int64_t Na, int64_t Nl, double* v_old, const double* a_grid,
                        const double* s, const double* P, const double* labor_choice, double r,
                        double w, double beta, double sigma, double psi, double eta, double tol,
                        int64_t max_iter, double* v_new, double* policy_k, double* policy_l,
                        double* policy_c, int32_t* lin, int64_t* iters);

/* interp1(x, y, xq, 'linear', 'extrap') */
void orc_interp1(int64_t n, const double* x, const double* y, int64_t nq, const double* xq,
                 double* out);

/* A4: Aiyagari_EGM.m:75-107 (one step) and :71-110 (solve).  [N][Na] layout. */
int orc_egm_step(int64_t N, int64_t Na, const double* policy_c, const double* a_grid,
                 const double* s, const double* P, double r, double w, double beta,
                 double sigma, double amin, double* policy_c_next, double* policy_k,
                 double* dist);
int orc_egm_solve(int64_t N, int64_t Na, double* policy_c, const double* a_grid,
                  const double* s, const double* P, double r, double w, double beta,
                  double sigma, double amin, double tol, int64_t max_iter, double* policy_k,
                  double* dist, int64_t* iters);
/* A5: Aiyagari_Endogenous_Labor_EGM.m:68-104 */
int orc_labor_egm_step(int64_t N, int64_t Na, const double* policy_c, const double* a_grid,
                       const double* s, const double* P, double r, double w, double beta,
                       double sigma, double phi, double theta, double amin,
                       double* policy_c_next, double* policy_k, double* policy_l,
                       double* dist);
int orc_labor_egm_solve(int64_t N, int64_t Na, double* policy_c, const double* a_grid,
                        const double* s, const double* P, double r, double w, double beta,
                        double sigma, double phi, double theta, double amin, double tol,
                        int64_t max_iter, double* policy_k, double* policy_l, double* dist,
                        int64_t* iters);

/* A9: Aiyagari_VFI.m:104-129.  policy rows: pol[z*Na + j] (row_stride = Na, col_stride = 1)
 * or EGM layout via strides.  z1 0-based.  T-1 uniforms.  sim_k may be NULL. */
int orc_sim_capital(int64_t N, int64_t Na, const double* policy, int64_t z_stride,
                    int64_t a_stride, const double* a_grid, const double* P, int64_t z1,
                    double k1, int64_t T, const double* uniforms, double* mean_k,
                    double* sim_k);

/* A10 (new): one histogram push λ -> λ' for an on-grid (idx) or off-grid (kp) policy.  The
 * mass of a destination sums its terms in ascending source j in chunks of 32 (chunk sums summed
 * in order) — the order the HIP gather kernel follows (csrc/dist.hpp kDistChunk); runs of up
 * to 32 terms are the plain sequential scatter. */
int orc_dist_update_ongrid(int64_t N, int64_t Na, const double* lam, const int32_t* idx,
                           const double* P, double* lam_out);
int orc_dist_update_lottery(int64_t N, int64_t Na, const double* lam, const double* kp,
                            const double* a_grid, const double* P, double* lam_out);

/* A10: iterate to max|Δλ| < tol; K = Σ λ(i,j)·a_j (sequential, i-major). */
int orc_dist_stationary(int64_t N, int64_t Na, const int32_t* idx, const double* kp,
                        const double* a_grid, const double* P, double tol, int64_t max_iter,
                        double* lam, double* K, int64_t* iters, double* dist);

/* A6/A7 Krusell-Smith (Krusell_Smith_VFI.m:148-192, bellman_value :329-364). */
typedef struct {
    double beta, alpha, delta, k_min, k_max, ug, ub, l_bar, mu;
    double z_grid[2];
    double eps_grid[2];
} orc_ks_params;
void orc_pchip_slopes(int64_t n, const double* x, const double* y, double* d);
double orc_pchip_eval(int64_t n, const double* x, const double* y, const double* d, double xq);
double orc_ks_bellman(const orc_ks_params* p, int64_t nk, int64_t nK, const double* k_grid,
                      const double* K_grid, const double* V, const double* dV, const double* B,
                      const double* P, double kp, int64_t k_i, int64_t K_i, int64_t s_i);
double orc_fminbnd_ks(const orc_ks_params* p, int64_t nk, int64_t nK, const double* k_grid,
                      const double* K_grid, const double* V, const double* dV, const double* B,
                      const double* P, int64_t k_i, int64_t K_i, int64_t s_i, double ax,
                      double bx, int32_t* nfev);
int orc_ks_policy_improve(const orc_ks_params* p, int64_t nk, int64_t nK, const double* k_grid,
                          const double* K_grid, const double* V, const double* B,
                          const double* P, const double* s_grid, double* k_opt,
                          int32_t* nfev);
int orc_ks_howard(const orc_ks_params* p, int64_t nk, int64_t nK, const double* k_grid,
                  const double* K_grid, double* V, const double* k_opt, const double* B,
                  const double* P, int64_t steps);

/* A8 Krusell-Smith EGM (Krusell_Smith_EGM.m:101-112, :129-209).  P row-major [s_i*4 + s_j]
 * (as orc_ks_*); k_opt k x K x S column-major, updated Gauss-Seidel in (s_i outer, K_i inner)
 * order.  Returns 0, or -2 when an (s, K) pair has fewer than 2 valid EGM points. */
typedef struct {
    int32_t kd[4];  /* K''_idx per s_j */
    double Rn[4];   /* (1 + r_next) - delta */
    double Wn[4];   /* w_next * eps_next * l_bar */
    double R;       /* (1 + r) - delta */
    double We;      /* w * eps * l_bar */
} orc_ks_egm_pair;
void orc_ks_egm_pairs(const orc_ks_params* p, int64_t nK, const double* K_grid, const double* B,
                      orc_ks_egm_pair* out);
int orc_ks_egm_sweep(const orc_ks_params* p, int64_t nk, int64_t nK, const double* k_grid,
                     const orc_ks_egm_pair* pairs, const double* P, double* k_opt);
int orc_ks_egm_solve(const orc_ks_params* p, int64_t nk, int64_t nK, const double* k_grid,
                     const double* K_grid, const double* B, const double* P, double tol,
                     int64_t max_iter, double* k_opt, int64_t* iters, double* diff);
int orc_ks_egm_solve_jacobi(const orc_ks_params* p, int64_t nk, int64_t nK, const double* k_grid,
                     const double* K_grid, const double* B, const double* P, double tol,
                     int64_t max_iter, double* k_opt, int64_t* iters, double* diff);

#ifdef __cplusplus
}
#endif
#endif
