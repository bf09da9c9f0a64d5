/* [v_new, v_old, policy_k, policy_c, iter, idx] =
 *     aiy_vfi_solve_mex(v_old, a_grid, s, P, r, w, beta, sigma, tol, max_iter)
 * Replaces Aiyagari_VFI.m:65-90 (and the GE copy :147-171).  Break semantics kept: v_new is
 * the converged iterate, v_old the previous one (the GE loop warm-starts from it).  idx
 * (optional) is the last sweep's argmax, 1-based as `max` returns it (:79-80), so
 * policy_k == a_grid(idx). */
#include "mexcommon.h"
void mexFunction(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    aiy_nargs(nrhs, 10, 10, nlhs, 6, "[v_new,v_old,policy_k,policy_c,iter,idx] = aiy_vfi_solve_mex(v_old,a_grid,s,P,r,w,beta,sigma,tol,max_iter)");
    mwSize N = mxGetM(prhs[0]), Na = mxGetN(prhs[0]);
    aiy_in(prhs[0], "v_old", 0, 0);
    const double* a = aiy_vec(prhs[1], "a_grid", Na, NULL);
    const double* s = aiy_vec(prhs[2], "s", N, NULL);
    const double* P = aiy_in(prhs[3], "P", N, N);
    double r = aiy_scalar(prhs[4], "r"), w = aiy_scalar(prhs[5], "w");
    double beta = aiy_scalar(prhs[6], "beta"), sigma = aiy_scalar(prhs[7], "sigma");
    double tol = aiy_scalar(prhs[8], "tol");
    int64_t max_iter = (int64_t)aiy_scalar(prhs[9], "max_iter");
    mxArray* vo = aiy_copy(prhs[0]); /* inputs are read-only: work on a copy */
    plhs[0] = aiy_out(N, Na);
    mxArray* pk = aiy_out(N, Na);
    mxArray* pc = aiy_out(N, Na);
    int64_t it = 0;
    int32_t* idx = nlhs > 5 ? (int32_t*)malloc(sizeof(int32_t) * N * Na) : NULL;
    aiy_begin();
    int rc = aiy_vfi_solve(mxGetPr(vo), a, s, P, (int64_t)N, (int64_t)Na, r, w, beta, sigma, tol,
                           max_iter, mxGetPr(plhs[0]), mxGetPr(pk), mxGetPr(pc), idx, &it);
    if (rc == AIY_OK && idx) {
        plhs[5] = aiy_out(N, Na);
        double* o = mxGetPr(plhs[5]);
        for (mwSize q = 0; q < N * Na; ++q) o[q] = idx[q];
    }
    free(idx);
    aiy_check(rc);
    if (nlhs > 1) plhs[1] = vo; else mxDestroyArray(vo);
    if (nlhs > 2) plhs[2] = pk; else mxDestroyArray(pk);
    if (nlhs > 3) plhs[3] = pc; else mxDestroyArray(pc);
    if (nlhs > 4) plhs[4] = mxCreateDoubleScalar((double)it);
}
