/* [k_supply, k_demand, iters] = aiy_ge_batch_mex(r, v_old, a_grid, s, P, alpha, delta, beta,
 *                                                 sigma, labor, tol, max_iter, z1, k1, uniforms,
 *                                                 n_devices)
 * Config 4 / SURVEY §8(b) B2: the body of one GE step of Aiyagari_VFI.m:147-195 at every
 * candidate rate r(c) at once — the VFI from v_old (N x Na, the common warm start), the
 * Monte-Carlo capital supply from (z1, k1) with the c-th column of `uniforms` ((T-1) x C, the
 * rand draws that step would consume) and K_d = labor*(alpha/(r+delta))^(1/(1-alpha)).  The
 * candidates are spread over n_devices GPUs.  The script keeps its bracket logic (:196-204),
 * e.g. evaluating every midpoint of the next levels of the bisection tree in one call. */
#include "mexcommon.h"
void mexFunction(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    aiy_nargs(nrhs, 16, 16, nlhs, 3, "[k_supply,k_demand,iters] = aiy_ge_batch_mex(r,v_old,a_grid,s,P,alpha,delta,beta,sigma,labor,tol,max_iter,z1,k1,uniforms,n_devices)");
    mwSize C = 0;
    const double* r = aiy_vec(prhs[0], "r", 0, &C);
    mwSize N = mxGetM(prhs[1]), Na = mxGetN(prhs[1]);
    const double* v = aiy_in(prhs[1], "v_old", 0, 0);
    const double* a = aiy_vec(prhs[2], "a_grid", Na, NULL);
    const double* s = aiy_vec(prhs[3], "s", N, NULL);
    const double* P = aiy_in(prhs[4], "P", N, N);
    double alpha = aiy_scalar(prhs[5], "alpha"), delta = aiy_scalar(prhs[6], "delta");
    double beta = aiy_scalar(prhs[7], "beta"), sigma = aiy_scalar(prhs[8], "sigma");
    double labor = aiy_scalar(prhs[9], "labor"), tol = aiy_scalar(prhs[10], "tol");
    double mi = aiy_scalar(prhs[11], "max_iter"), z1 = aiy_scalar(prhs[12], "z1");
    double k1 = aiy_scalar(prhs[13], "k1");
    const double* U = aiy_in(prhs[14], "uniforms", 0, C);
    int64_t T = (int64_t)mxGetM(prhs[14]) + 1;
    double nd = aiy_scalar(prhs[15], "n_devices");
    if (mi != (double)(int64_t)mi || z1 != (double)(int64_t)z1 || nd != (double)(int)nd)
        aiy_err("aiy:type", "max_iter, z1 and n_devices must be integers");
    mxArray* ks = aiy_out(C, 1);
    mxArray* kd = aiy_out(C, 1);
    int64_t* it = (int64_t*)malloc(sizeof(int64_t) * (C ? C : 1));
    aiy_begin();
    int rc = aiy_ge_batch(r, (int64_t)C, v, a, s, P, (int64_t)N, (int64_t)Na, alpha, delta, beta,
                          sigma, labor, tol, (int64_t)mi, (int64_t)z1, k1, T, U, (int)nd,
                          mxGetPr(ks), mxGetPr(kd), it);
    if (rc != AIY_OK) {
        free(it);
        mxDestroyArray(ks);
        mxDestroyArray(kd);
    }
    aiy_check(rc);
    plhs[0] = ks;
    if (nlhs > 1) plhs[1] = kd;
    else mxDestroyArray(kd);
    if (nlhs > 2) {
        plhs[2] = aiy_out(C, 1);
        for (mwSize q = 0; q < C; ++q) mxGetPr(plhs[2])[q] = (double)it[q];
    }
    free(it);
}
