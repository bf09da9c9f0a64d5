/* Minimal stand-in for MATLAB's mex.h / matrix.h — ONLY for compile- and unit-testing the
 * gateways in this image (no MATLAB or Octave here).  A real build uses the headers that ship
 * with MATLAB (`mex`) or Octave (`mkoctfile --mex`); nothing here is linked into those builds.
 * The subset declared is exactly what the gateways use, with MATLAB's signatures. */
#ifndef AIY_STUB_MEX_H
#define AIY_STUB_MEX_H
#include <stddef.h>
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif
typedef size_t mwSize;
typedef size_t mwIndex;
typedef struct mxArray_tag mxArray;
typedef enum { mxUNKNOWN_CLASS = 0, mxDOUBLE_CLASS = 6, mxINT32_CLASS = 12 } mxClassID;
typedef enum { mxREAL = 0, mxCOMPLEX = 1 } mxComplexity;

mxArray* mxCreateDoubleMatrix(mwSize m, mwSize n, mxComplexity c);
mxArray* mxCreateDoubleScalar(double v);
mxArray* mxCreateNumericArray(mwSize ndim, const mwSize* dims, mxClassID cls, mxComplexity c);
void mxDestroyArray(mxArray* a);
double* mxGetPr(const mxArray* a);
void* mxGetData(const mxArray* a);
mwSize mxGetM(const mxArray* a);
mwSize mxGetN(const mxArray* a);
mwSize mxGetNumberOfElements(const mxArray* a);
mwSize mxGetNumberOfDimensions(const mxArray* a);
const mwSize* mxGetDimensions(const mxArray* a);
int mxIsDouble(const mxArray* a);
int mxIsComplex(const mxArray* a);
int mxIsSparse(const mxArray* a);
double mxGetScalar(const mxArray* a);
void mexErrMsgIdAndTxt(const char* id, const char* fmt, ...);
int mexAtExit(void (*fn)(void));
void mexLock(void);
void mexUnlock(void);
#ifdef __cplusplus
}
#endif
#endif
