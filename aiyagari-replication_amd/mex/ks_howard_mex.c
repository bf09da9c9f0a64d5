/* value = ks_howard_mex(value, k_opt, k_grid, K_grid, B, P, params, steps)
 * Replaces the Howard policy-evaluation loop of Krusell_Smith_VFI.m:172-192: `steps` Jacobi
 * sweeps value <- bellman_value(k_opt) with the pchip slopes rebuilt from each sweep's values
 * (the .Values refresh of :186-191).  value, k_opt: k_size x K_size x 4.  params: as
 * ks_policy_improve_mex. */
#include "mexcommon.h"
void mexFunction(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    aiy_nargs(nrhs, 8, 8, nlhs, 1, "value = ks_howard_mex(value,k_opt,k_grid,K_grid,B,P,params,steps)");
    mwSize nk = 0, nK = 0;
    const double* kg = aiy_vec(prhs[2], "k_grid", 0, &nk);
    const double* Kg = aiy_vec(prhs[3], "K_grid", 0, &nK);
    if (mxGetNumberOfElements(prhs[0]) != nk * nK * 4 || mxGetNumberOfElements(prhs[1]) != nk * nK * 4)
        aiy_err("aiy:shape", "value and k_opt must be k_size x K_size x 4");
    aiy_in(prhs[0], "value", 0, 0);
    const double* ko = aiy_in(prhs[1], "k_opt", 0, 0);
    const double* B = aiy_vec(prhs[4], "B", 4, NULL);
    const double* P = aiy_in(prhs[5], "P", 4, 4);
    const double* prm = aiy_vec(prhs[6], "params", 13, NULL);
    double steps_d = aiy_scalar(prhs[7], "steps");
    if (!(steps_d >= 0) || steps_d != floor(steps_d)) aiy_err("aiy:BAD_ARG", "steps must be a non-negative integer");
    mwSize dims[3] = {nk, nK, 4};
    plhs[0] = mxCreateNumericArray(3, dims, mxDOUBLE_CLASS, mxREAL);
    memcpy(mxGetPr(plhs[0]), mxGetPr(prhs[0]), sizeof(double) * nk * nK * 4);
    aiy_begin();
    aiy_check(ks_howard(mxGetPr(plhs[0]), ko, kg, Kg, B, P, prm, (int64_t)nk, (int64_t)nK,
                        (int64_t)steps_d));
}
