/*
 * mex.h -- TEST-ONLY stand-in for MATLAB's MEX API (no MATLAB in this image).
 * It declares exactly the subset matlab/ccsc_mex.c and matlab/ccsc_solve_mex.c use, with MATLAB's
 * signatures (R2018a interleaved-complex API), so the gateway compiles with
 * -Wall -Werror here and runs under tests/mex_stub/mexstub.c, a minimal
 * column-major mxArray implementation driven from Python (tests/test_mex.py).
 * It is not a MATLAB replacement and is never linked into libccsc.
 */
#ifndef CCSC_TEST_MEX_H_
#define CCSC_TEST_MEX_H_

#include <stddef.h>

typedef size_t mwSize;
typedef enum { mxUNKNOWN_CLASS = 0, mxCHAR_CLASS = 4, mxDOUBLE_CLASS = 6, mxSTRUCT_CLASS = 2 } mxClassID;
typedef enum { mxREAL = 0, mxCOMPLEX = 1 } mxComplexity;
typedef struct mxArray_tag mxArray;

#ifdef __cplusplus
extern "C" {
#endif
/* provided by the gateway */
void mexFunction(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]);

double mxGetScalar(const mxArray* a);
int mxIsDouble(const mxArray* a);
int mxIsComplex(const mxArray* a);
int mxIsEmpty(const mxArray* a);
double* mxGetDoubles(const mxArray* a);
size_t mxGetNumberOfElements(const mxArray* a);
const mwSize* mxGetDimensions(const mxArray* a);
mwSize mxGetNumberOfDimensions(const mxArray* a);
int mxGetString(const mxArray* a, char* buf, mwSize buflen);
mxArray* mxCreateNumericArray(mwSize nd, const mwSize* dims, mxClassID cls, mxComplexity cx);
mxArray* mxCreateDoubleMatrix(mwSize m, mwSize n, mxComplexity cx);
mxArray* mxCreateDoubleScalar(double v);
mxArray* mxCreateStructMatrix(mwSize m, mwSize n, int nfields, const char** names);
void mxSetField(mxArray* s, size_t i, const char* name, mxArray* v);
void mxSetN(mxArray* a, mwSize n);
void mxDestroyArray(mxArray* a);
void* mxCalloc(size_t n, size_t size);
void mxFree(void* ptr);
void mexErrMsgIdAndTxt(const char* id, const char* fmt, ...);
int mexPrintf(const char* fmt, ...);
int mexEvalString(const char* cmd);
int mexAtExit(void (*fn)(void));
#ifdef __cplusplus
}
#endif
#endif
