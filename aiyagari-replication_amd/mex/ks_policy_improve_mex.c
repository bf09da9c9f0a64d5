/* [k_opt, nfev] = ks_policy_improve_mex(value, k_grid, K_grid, B, P, params)
 * Replaces the policy-improvement step of Krusell_Smith_VFI.m:148-168 (fminbnd on -bellman_value
 * over [k_min, min(resources, k_max)] per node; MaxFunEvals = MaxIter = 500, TolX = 1e-4) for the
 * current ALM coefficients B.  value: k_size x K_size x 4; k_opt (and nfev, the function
 * evaluations per node) come back in the same shape.  params = [beta alpha delta k_min k_max
 * ug ub l_bar mu z_grid(1) z_grid(2) eps_grid(1) eps_grid(2)]. */
#include "mexcommon.h"
void mexFunction(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    aiy_nargs(nrhs, 6, 6, nlhs, 2, "[k_opt,nfev] = ks_policy_improve_mex(value,k_grid,K_grid,B,P,params)");
    mwSize nk = 0, nK = 0;
    const double* kg = aiy_vec(prhs[1], "k_grid", 0, &nk);
    const double* Kg = aiy_vec(prhs[2], "K_grid", 0, &nK);
    if (mxGetNumberOfElements(prhs[0]) != nk * nK * 4)
        aiy_err("aiy:shape", "value must be k_size x K_size x 4");
    const double* V = aiy_in(prhs[0], "value", 0, 0);
    const double* B = aiy_vec(prhs[3], "B", 4, NULL);
    const double* P = aiy_in(prhs[4], "P", 4, 4);
    const double* prm = aiy_vec(prhs[5], "params", 13, NULL);
    mwSize dims[3] = {nk, nK, 4};
    mxArray* ko = mxCreateNumericArray(3, dims, mxDOUBLE_CLASS, mxREAL);
    int32_t* nf = nlhs > 1 ? (int32_t*)malloc(sizeof(int32_t) * nk * nK * 4) : NULL;
    aiy_begin();
    int rc = ks_policy_improve(V, kg, Kg, B, P, prm, (int64_t)nk, (int64_t)nK, mxGetPr(ko), nf);
    if (rc == AIY_OK && nf) {
        plhs[1] = mxCreateNumericArray(3, dims, mxDOUBLE_CLASS, mxREAL);
        for (mwSize q = 0; q < nk * nK * 4; ++q) mxGetPr(plhs[1])[q] = nf[q];
    }
    free(nf);
    if (rc != AIY_OK) mxDestroyArray(ko);
    aiy_check(rc);
    plhs[0] = ko;
}
