/* [value, k_opt, iter, rel_diff] = ks_vfi_solve_mex(value, k_opt, k_grid, K_grid, B, P, params,
 *                                                   howard_steps, tol_vfi, max_vfi, n_devices
 *                                                   [, depth])
 * Replaces the Howard-accelerated VFI loop of Krusell_Smith_VFI.m:141-204 for the current B.
 * n_devices > 1: (K, Z) slices over the visible devices, `depth` Howard sweeps per exchange
 * (default 4; ks_vfi_solve_sharded).
 * value, k_opt: k_size x K_size x 4.  params = [beta alpha delta k_min k_max ug ub l_bar mu
 * z_grid(1) z_grid(2) eps_grid(1) eps_grid(2)]. */
#include "mexcommon.h"
void mexFunction(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    aiy_nargs(nrhs, 11, 12, nlhs, 4, "[value,k_opt,iter,rel_diff] = ks_vfi_solve_mex(value,k_opt,k_grid,K_grid,B,P,params,howard_steps,tol_vfi,max_vfi,n_devices[,depth])");
    mwSize nk = 0, nK = 0;
    const double* kg = aiy_vec(prhs[2], "k_grid", 0, &nk);
    const double* Kg = aiy_vec(prhs[3], "K_grid", 0, &nK);
    if (mxGetNumberOfElements(prhs[0]) != nk * nK * 4 || mxGetNumberOfElements(prhs[1]) != nk * nK * 4)
        aiy_err("aiy:shape", "value and k_opt must be k_size x K_size x 4");
    aiy_in(prhs[0], "value", 0, 0);
    aiy_in(prhs[1], "k_opt", 0, 0);
    const double* B = aiy_vec(prhs[4], "B", 4, NULL);
    const double* P = aiy_in(prhs[5], "P", 4, 4);
    const double* prm = aiy_vec(prhs[6], "params", 13, NULL);
    int64_t H = (int64_t)aiy_scalar(prhs[7], "howard_steps");
    double tol = aiy_scalar(prhs[8], "tol_vfi");
    int64_t maxv = (int64_t)aiy_scalar(prhs[9], "max_vfi");
    int nd = (int)aiy_scalar(prhs[10], "n_devices");
    int depth = nrhs > 11 ? (int)aiy_scalar(prhs[11], "depth") : 4;
    mwSize dims[3] = {nk, nK, 4};
    plhs[0] = mxCreateNumericArray(3, dims, mxDOUBLE_CLASS, mxREAL);
    mxArray* ko = mxCreateNumericArray(3, dims, mxDOUBLE_CLASS, mxREAL);
    memcpy(mxGetPr(plhs[0]), mxGetPr(prhs[0]), sizeof(double) * nk * nK * 4);
    memcpy(mxGetPr(ko), mxGetPr(prhs[1]), sizeof(double) * nk * nK * 4);
    int64_t it = 0;
    double rel = 0;
    aiy_begin();
    if (nd > 1)
        aiy_check(ks_vfi_solve_sharded(mxGetPr(plhs[0]), mxGetPr(ko), kg, Kg, B, P, prm,
                                       (int64_t)nk, (int64_t)nK, H, tol, maxv, nd, depth, &it,
                                       &rel));
    else
        aiy_check(ks_vfi_solve(mxGetPr(plhs[0]), mxGetPr(ko), kg, Kg, B, P, prm, (int64_t)nk,
                               (int64_t)nK, H, tol, maxv, nd, &it, &rel));
    if (nlhs > 1) plhs[1] = ko; else mxDestroyArray(ko);
    if (nlhs > 2) plhs[2] = mxCreateDoubleScalar((double)it);
    if (nlhs > 3) plhs[3] = mxCreateDoubleScalar(rel);
}
