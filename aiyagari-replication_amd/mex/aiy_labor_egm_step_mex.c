/* [policy_c_next, policy_k, policy_l, dist] =
 *     aiy_labor_egm_step_mex(policy_c, a_grid, s, P, r, w, beta, sigma, phi, theta, amin)
 * One pass of the labour EGM loop body, Aiyagari_Endogenous_Labor_EGM.m:70-104 (GE copy
 * :176-211): the Euler RHS, the intratemporal FOC for labour (:86, :95), interp1 of
 * consumption on the endogenous grid (:90), a' = (1+r)a + w s l - c clamped at 0 (:98-99), and
 * dist = max|policy_c_next - policy_c| (:103).  Arrays Na x N (the script's layout). */
#include "mexcommon.h"
void mexFunction(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    aiy_nargs(nrhs, 11, 11, nlhs, 4, "[policy_c_next,policy_k,policy_l,dist] = aiy_labor_egm_step_mex(policy_c,a_grid,s,P,r,w,beta,sigma,phi,theta,amin)");
    mwSize Na = mxGetM(prhs[0]), N = mxGetN(prhs[0]);
    const double* c = aiy_in(prhs[0], "policy_c", 0, 0);
    const double* a = aiy_vec(prhs[1], "a_grid", Na, NULL);
    const double* s = aiy_vec(prhs[2], "s", N, NULL);
    const double* P = aiy_in(prhs[3], "P", N, N);
    double r = aiy_scalar(prhs[4], "r"), w = aiy_scalar(prhs[5], "w");
    double beta = aiy_scalar(prhs[6], "beta"), sigma = aiy_scalar(prhs[7], "sigma");
    double phi = aiy_scalar(prhs[8], "phi"), theta = aiy_scalar(prhs[9], "theta");
    double amin = aiy_scalar(prhs[10], "amin");
    plhs[0] = aiy_out(Na, N);
    mxArray* pk = aiy_out(Na, N);
    mxArray* pl = aiy_out(Na, N);
    double dist = 0;
    aiy_begin();
    aiy_check(aiy_labor_egm_step(c, a, s, P, (int64_t)N, (int64_t)Na, r, w, beta, sigma, phi,
                                 theta, amin, mxGetPr(plhs[0]), mxGetPr(pk), mxGetPr(pl), &dist));
    if (nlhs > 1) plhs[1] = pk; else mxDestroyArray(pk);
    if (nlhs > 2) plhs[2] = pl; else mxDestroyArray(pl);
    if (nlhs > 3) plhs[3] = mxCreateDoubleScalar(dist);
}
