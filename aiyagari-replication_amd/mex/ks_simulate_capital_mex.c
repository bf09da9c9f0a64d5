/* [K_ts, k_population] = ks_simulate_capital_mex(k_opt, k_grid, K_grid, zi_shock, epsi_shock,
 *                                                k_population)
 * Replaces the capital path simulation of Krusell_Smith_VFI.m:206-248 (Krusell_Smith_EGM.m
 * :211-253).  k_opt: k_size x K_size x 4; zi_shock T (0/1); epsi_shock T x population (1/2);
 * k_population: population x 1 (the script keeps it across ALM iterations, :101). */
#include "mexcommon.h"
void mexFunction(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    aiy_nargs(nrhs, 6, 6, nlhs, 2, "[K_ts,k_population] = ks_simulate_capital_mex(k_opt,k_grid,K_grid,zi_shock,epsi_shock,k_population)");
    mwSize nk = 0, nK = 0, T = 0, pop = 0;
    const double* kg = aiy_vec(prhs[1], "k_grid", 0, &nk);
    const double* Kg = aiy_vec(prhs[2], "K_grid", 0, &nK);
    if (mxGetNumberOfElements(prhs[0]) != nk * nK * 4)
        aiy_err("aiy:shape", "k_opt must be k_size x K_size x 4");
    const double* ko = aiy_in(prhs[0], "k_opt", 0, 0);
    const double* zi = aiy_vec(prhs[3], "zi_shock", 0, &T);
    const double* ep = aiy_in(prhs[4], "epsi_shock", T, 0);
    const double* kp = aiy_vec(prhs[5], "k_population", 0, &pop);
    if (mxGetN(prhs[4]) != pop)
        aiy_err("aiy:shape", "epsi_shock must be numel(zi_shock) x numel(k_population)");
    mxArray* K_ts = aiy_out(T, 1);
    mxArray* kout = aiy_out(pop, 1);
    memcpy(mxGetPr(kout), kp, sizeof(double) * pop);
    aiy_begin();
    int rc = ks_simulate_capital(ko, kg, Kg, (int64_t)nk, (int64_t)nK, zi, ep, (int64_t)T,
                                 (int64_t)pop, mxGetPr(kout), mxGetPr(K_ts));
    if (rc != AIY_OK) {
        mxDestroyArray(K_ts);
        mxDestroyArray(kout);
    }
    aiy_check(rc);
    plhs[0] = K_ts;
    if (nlhs > 1) plhs[1] = kout;
    else mxDestroyArray(kout);
}
