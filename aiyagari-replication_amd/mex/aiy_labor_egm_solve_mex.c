/* [policy_c, policy_k, policy_l, dist, iter] = aiy_labor_egm_solve_mex(policy_c, a_grid, s, P,
 *     r, w, beta, sigma, phi, theta, amin, tol, max_iter)
 * Replaces Aiyagari_Endogenous_Labor_EGM.m:64-107 (GE copy :169-214). */
#include "mexcommon.h"
void mexFunction(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    aiy_nargs(nrhs, 13, 13, nlhs, 5, "[policy_c,policy_k,policy_l,dist,iter] = aiy_labor_egm_solve_mex(policy_c,a_grid,s,P,r,w,beta,sigma,phi,theta,amin,tol,max_iter)");
    mwSize Na = mxGetM(prhs[0]), N = mxGetN(prhs[0]);
    aiy_in(prhs[0], "policy_c", 0, 0);
    const double* a = aiy_vec(prhs[1], "a_grid", Na, NULL);
    const double* s = aiy_vec(prhs[2], "s", N, NULL);
    const double* P = aiy_in(prhs[3], "P", N, N);
    double r = aiy_scalar(prhs[4], "r"), w = aiy_scalar(prhs[5], "w");
    double beta = aiy_scalar(prhs[6], "beta"), sigma = aiy_scalar(prhs[7], "sigma");
    double phi = aiy_scalar(prhs[8], "phi"), theta = aiy_scalar(prhs[9], "theta");
    double amin = aiy_scalar(prhs[10], "amin"), tol = aiy_scalar(prhs[11], "tol");
    int64_t max_iter = (int64_t)aiy_scalar(prhs[12], "max_iter");
    plhs[0] = aiy_copy(prhs[0]);
    mxArray* pk = aiy_out(Na, N);
    mxArray* pl = aiy_out(Na, N);
    double dist = 0;
    int64_t it = 0;
    aiy_begin();
    aiy_check(aiy_labor_egm_solve(mxGetPr(plhs[0]), a, s, P, (int64_t)N, (int64_t)Na, r, w, beta,
                                  sigma, phi, theta, amin, tol, max_iter, mxGetPr(pk), mxGetPr(pl),
                                  &dist, &it));
    if (nlhs > 1) plhs[1] = pk; else mxDestroyArray(pk);
    if (nlhs > 2) plhs[2] = pl; else mxDestroyArray(pl);
    if (nlhs > 3) plhs[3] = mxCreateDoubleScalar(dist);
    if (nlhs > 4) plhs[4] = mxCreateDoubleScalar((double)it);
}
