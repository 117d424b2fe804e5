/*
 * mexstub.c -- TEST-ONLY minimal MEX runtime (see mex.h): column-major double
 * arrays, char arrays, 1x1 structs, mexErrMsgIdAndTxt as a longjmp back to
 * hx_call().  Lets tests/test_mex.py run matlab/ccsc_mex.c's mexFunction on
 * the GPU box exactly as MATLAB would call it, minus MATLAB.
 */
#include "mex.h"

#include <setjmp.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

struct mxArray_tag {
  mxClassID cls;
  mwSize nd;
  mwSize dims[8];
  double* data;
  char* str;
  int nfields;
  char** fnames;
  mxArray** fvals;
};

static jmp_buf g_jmp;
static char g_err[2048];
static void (*g_exit)(void) = NULL;

static mwSize numel(const mxArray* a) {
  mwSize n = 1;
  for (mwSize i = 0; i < a->nd; ++i) n *= a->dims[i];
  return n;
}
double mxGetScalar(const mxArray* a) { return a->data && numel(a) ? a->data[0] : 0.0; }
int mxIsDouble(const mxArray* a) { return a->cls == mxDOUBLE_CLASS; }
int mxIsComplex(const mxArray* a) { (void)a; return 0; }
int mxIsEmpty(const mxArray* a) { return numel(a) == 0; }
double* mxGetDoubles(const mxArray* a) { return a->cls == mxDOUBLE_CLASS ? a->data : NULL; }
size_t mxGetNumberOfElements(const mxArray* a) { return numel(a); }
const mwSize* mxGetDimensions(const mxArray* a) { return a->dims; }
mwSize mxGetNumberOfDimensions(const mxArray* a) { return a->nd; }
int mxGetString(const mxArray* a, char* buf, mwSize len) {
  if (a->cls != mxCHAR_CLASS || !len) return 1;
  snprintf(buf, len, "%s", a->str);
  return 0;
}
mxArray* mxCreateNumericArray(mwSize nd, const mwSize* dims, mxClassID cls, mxComplexity cx) {
  (void)cx;
  mxArray* a = (mxArray*)calloc(1, sizeof *a);
  a->cls = cls;
  a->nd = nd < 2 ? 2 : nd;
  a->dims[0] = a->dims[1] = 1;
  for (mwSize i = 0; i < nd; ++i) a->dims[i] = dims[i];
  a->data = (double*)calloc(numel(a) ? numel(a) : 1, sizeof(double));
  return a;
}
mxArray* mxCreateDoubleMatrix(mwSize m, mwSize n, mxComplexity cx) {
  const mwSize d[2] = {m, n};
  return mxCreateNumericArray(2, d, mxDOUBLE_CLASS, cx);
}
mxArray* mxCreateDoubleScalar(double v) {
  mxArray* a = mxCreateDoubleMatrix(1, 1, mxREAL);
  a->data[0] = v;
  return a;
}
mxArray* mxCreateStructMatrix(mwSize m, mwSize n, int nf, const char** names) {
  mxArray* a = (mxArray*)calloc(1, sizeof *a);
  a->cls = mxSTRUCT_CLASS;
  a->nd = 2;
  a->dims[0] = m;
  a->dims[1] = n;
  a->nfields = nf;
  a->fnames = (char**)calloc(nf, sizeof(char*));
  a->fvals = (mxArray**)calloc(nf, sizeof(mxArray*));
  for (int i = 0; i < nf; ++i) a->fnames[i] = strdup(names[i]);
  return a;
}
void mxSetField(mxArray* s, size_t i, const char* name, mxArray* v) {
  (void)i;
  for (int f = 0; f < s->nfields; ++f)
    if (!strcmp(s->fnames[f], name)) s->fvals[f] = v;
}
void mxSetN(mxArray* a, mwSize n) { a->dims[1] = n; }
void mxDestroyArray(mxArray* a) {
  if (!a) return;
  for (int f = 0; f < a->nfields; ++f) {
    free(a->fnames[f]);
    mxDestroyArray(a->fvals[f]);
  }
  free(a->fnames);
  free(a->fvals);
  free(a->data);
  free(a->str);
  free(a);
}
void mexErrMsgIdAndTxt(const char* id, const char* fmt, ...) {
  int k = snprintf(g_err, sizeof g_err, "%s: ", id);
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err + k, sizeof g_err - (size_t)k, fmt, ap);
  va_end(ap);
  longjmp(g_jmp, 1);
}
int mexPrintf(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  const int r = vprintf(fmt, ap);
  va_end(ap);
  return r;
}
int mexEvalString(const char* cmd) { (void)cmd; return 0; }
int mexAtExit(void (*fn)(void)) { g_exit = fn; return 0; }

/* ---- harness entry points (ctypes) ---- */
mxArray* hx_double(const double* src, int nd, const int64_t* dims) {
  mwSize d[8];
  for (int i = 0; i < nd; ++i) d[i] = (mwSize)dims[i];
  mxArray* a = mxCreateNumericArray((mwSize)nd, d, mxDOUBLE_CLASS, mxREAL);
  if (src) memcpy(a->data, src, numel(a) * sizeof(double));
  return a;
}
mxArray* hx_string(const char* s) {
  mxArray* a = (mxArray*)calloc(1, sizeof *a);
  a->cls = mxCHAR_CLASS;
  a->nd = 2;
  a->dims[0] = 1;
  a->dims[1] = strlen(s);
  a->str = strdup(s);
  return a;
}
int hx_ndims(const mxArray* a) { return (int)a->nd; }
int64_t hx_dim(const mxArray* a, int i) { return (int64_t)a->dims[i]; }
const double* hx_data(const mxArray* a) { return a->data; }
mxArray* hx_field(const mxArray* s, const char* name) {
  for (int f = 0; f < s->nfields; ++f)
    if (!strcmp(s->fnames[f], name)) return s->fvals[f];
  return NULL;
}
void* mxCalloc(size_t n, size_t size) { return calloc(n ? n : 1, size); }
void mxFree(void* ptr) { free(ptr); }
void hx_free(mxArray* a) { mxDestroyArray(a); }
/* 0 on success; else the mexErrMsgIdAndTxt message in err */
int hx_call(int nlhs, mxArray** plhs, int nrhs, mxArray** prhs, char* err, size_t errlen) {
  for (int i = 0; i < nlhs; ++i) plhs[i] = NULL;
  if (setjmp(g_jmp)) {
    snprintf(err, errlen, "%s", g_err);
    return 1;
  }
  mexFunction(nlhs, plhs, nrhs, (const mxArray**)prhs);
  return 0;
}
void hx_exit(void) {
  if (g_exit) g_exit();
  g_exit = NULL;
}
