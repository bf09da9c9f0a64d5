/* [k_opt, iter, diff] = ks_egm_solve_mex(k_opt, k_grid, K_grid, B, P, params, tol_egm, max_egm
 *                                         [, jacobi])
 * Replaces the EGM policy-iteration loop of Krusell_Smith_EGM.m:129-209 for the current B
 * (Gauss-Seidel over (s, K), each column overwritten as soon as it is computed).  jacobi = 1
 * selects the F1 variant (every pair reads the previous sweep; NOT the script's path — same
 * fixed point within tol, different sweep count), ks_egm_solve_jacobi in the C ABI.
 * k_opt: k_size x K_size x 4.  params = [beta alpha delta k_min k_max ug ub l_bar mu
 * z_grid(1) z_grid(2) eps_grid(1) eps_grid(2)] (mu unused). */
#include "mexcommon.h"
void mexFunction(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    aiy_nargs(nrhs, 8, 9, nlhs, 3, "[k_opt,iter,diff] = ks_egm_solve_mex(k_opt,k_grid,K_grid,B,P,params,tol_egm,max_egm[,jacobi])");
    mwSize nk = 0, nK = 0;
    const double* kg = aiy_vec(prhs[1], "k_grid", 0, &nk);
    const double* Kg = aiy_vec(prhs[2], "K_grid", 0, &nK);
    if (mxGetNumberOfElements(prhs[0]) != nk * nK * 4)
        aiy_err("aiy:shape", "k_opt must be k_size x K_size x 4");
    aiy_in(prhs[0], "k_opt", 0, 0);
    const double* B = aiy_vec(prhs[3], "B", 4, NULL);
    const double* P = aiy_in(prhs[4], "P", 4, 4);
    const double* prm = aiy_vec(prhs[5], "params", 13, NULL);
    double tol = aiy_scalar(prhs[6], "tol_egm");
    int64_t maxe = (int64_t)aiy_scalar(prhs[7], "max_egm");
    double jac = nrhs > 8 ? aiy_scalar(prhs[8], "jacobi") : 0.0;
    if (jac != 0.0 && jac != 1.0) aiy_err("aiy:type", "jacobi must be 0 or 1");
    mwSize dims[3] = {nk, nK, 4};
    plhs[0] = mxCreateNumericArray(3, dims, mxDOUBLE_CLASS, mxREAL);
    memcpy(mxGetPr(plhs[0]), mxGetPr(prhs[0]), sizeof(double) * nk * nK * 4);
    int64_t it = 0;
    double diff = 0;
    aiy_begin();
    if (jac == 1.0)
        aiy_check(ks_egm_solve_jacobi(mxGetPr(plhs[0]), kg, Kg, B, P, prm, (int64_t)nk,
                                      (int64_t)nK, tol, maxe, &it, &diff));
    else
        aiy_check(ks_egm_solve(mxGetPr(plhs[0]), kg, Kg, B, P, prm, (int64_t)nk, (int64_t)nK,
                               tol, maxe, &it, &diff));
    if (nlhs > 1) plhs[1] = mxCreateDoubleScalar((double)it);
    if (nlhs > 2) plhs[2] = mxCreateDoubleScalar(diff);
}
