/* [zi_shock, epsi_shock] = ks_shocks_mex(T, population, uniforms, params)
 * Replaces the shock simulation of Krusell_Smith_VFI.m:57-94.  uniforms: the script's rand
 * draws in its order, (T-1) + population + (T-1)*population values (e.g. rand(n,1) in a fresh
 * session).  zi_shock: T x 1 in {0 good, 1 bad} (after :68); epsi_shock: T x population in
 * {1, 2}.  params: the 13 KS doubles (ug = params(6), ub = params(7)). */
#include "mexcommon.h"
void mexFunction(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    aiy_nargs(nrhs, 4, 4, nlhs, 2, "[zi_shock,epsi_shock] = ks_shocks_mex(T,population,uniforms,params)");
    double Td = aiy_scalar(prhs[0], "T"), popd = aiy_scalar(prhs[1], "population");
    if (!(Td >= 1 && popd >= 1) || Td != (double)(int64_t)Td || popd != (double)(int64_t)popd)
        aiy_err("aiy:shape", "T and population must be positive integers");
    int64_t T = (int64_t)Td, pop = (int64_t)popd;
    const double* U = aiy_vec(prhs[2], "uniforms", (mwSize)ks_shock_draws(T, pop), NULL);
    const double* prm = aiy_vec(prhs[3], "params", 13, NULL);
    mxArray* zi = aiy_out((mwSize)T, 1);
    mxArray* ep = aiy_out((mwSize)T, (mwSize)pop);
    aiy_begin();
    int rc = ks_shocks(T, pop, U, prm, mxGetPr(zi), mxGetPr(ep));
    if (rc != AIY_OK) {
        mxDestroyArray(zi);
        mxDestroyArray(ep);
    }
    aiy_check(rc);
    plhs[0] = zi;
    if (nlhs > 1) plhs[1] = ep;
    else mxDestroyArray(ep);
}
