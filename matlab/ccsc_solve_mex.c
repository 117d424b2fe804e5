/*
 * ccsc_solve_mex.c -- MEX gateway of the reconstruction solvers over libccsc
 * (ccsc_solve, include/ccsc.h).  Thin by design: marshal the column-major mxArrays
 * into the C-ABI and back.  Build on a MATLAB host with:
 *   mex -R2018a ccsc_solve_mex.c -I../include -L../ccsc_code_iccv2017_amd -lccsc
 *
 * Called by the .m wrappers in this directory, which keep the reference signatures:
 *   [z, res] = ccsc_solve_mex(variant, b, kernels, mask, lambda_residual, lambda_prior,
 *                             max_it, tol, verbose, smooth_init, psf, x_orig, device)
 *   variant 0  admm_solve_conv2D_weighted_sampling   2D/Inpainting/...:1-4
 *           1  admm_solve_conv_poisson               2D/Poisson_deconv/...:1-2
 *           2  admm_solve_conv23D_weighted_sampling  2-3D/Demosaicing/...:1-2
 *              (and admm_solve_conv_weighted_sampling_lf, 4D/ViewSynthesis)
 *           3  admm_solve_video_weighted_sampling    3D/Deblurring/...:1-2
 * Empty smooth_init / psf / x_orig mean "not given".  res is only formed when the
 * caller takes it (nargout).  verbose 'brief' / 'all' prints the reference's per-iterate
 * line (objective, PSNR where x_orig is given, relative change) after the solve.
 */
#include "mex.h"
#include "ccsc.h"

#include <math.h>
#include <string.h>

static ccsc_ctx* g_sctx = NULL;
static int32_t g_sdev = -1;

static void solve_cleanup(void) {
  if (g_sctx) ccsc_destroy(g_sctx);
  g_sctx = NULL;
  g_sdev = -1;
}

static ccsc_ctx* solve_context(int32_t dev, char* err, size_t errlen) {
  if (g_sctx && g_sdev == dev) return g_sctx;
  solve_cleanup();
  g_sctx = ccsc_create(dev, 0, 1, NULL, err, errlen);
  if (!g_sctx) mexErrMsgIdAndTxt("ccsc:hip", "%s", err);
  g_sdev = dev;
  mexAtExit(solve_cleanup);
  return g_sctx;
}

static const double* opt(const mxArray* a) { return mxIsEmpty(a) ? NULL : mxGetDoubles(a); }

void mexFunction(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
  char err[1024] = {0};
  if (nrhs < 13) mexErrMsgIdAndTxt("ccsc:args", "ccsc_solve_mex needs 13 arguments");
  for (int i = 1; i < 13; ++i)
    if (i != 8 && !mxIsEmpty(prhs[i]) && (!mxIsDouble(prhs[i]) || mxIsComplex(prhs[i])))
      mexErrMsgIdAndTxt("ccsc:args", "argument %d must be real double", i + 1);
  const int variant = (int)mxGetScalar(prhs[0]);
  const mxArray* b = prhs[1];
  const mxArray* k = prhs[2];
  const mwSize* bd = mxGetDimensions(b);
  const mwSize bn = mxGetNumberOfDimensions(b);
  const mwSize* kd = mxGetDimensions(k);
  const mwSize kn = mxGetNumberOfDimensions(k);

  ccsc_solve_problem p;
  memset(&p, 0, sizeof p);
  p.variant = variant;
  const int v3 = variant == CCSC_SOLVE_VIDEO3D, mc = variant == CCSC_SOLVE_MULTICH;
  p.sb[0] = (int64_t)bd[0];
  p.sb[1] = (int64_t)(bn > 1 ? bd[1] : 1);
  p.sb[2] = (int64_t)(v3 && bn > 2 ? bd[2] : 1);
  p.nch = mc ? (int32_t)(bn > 2 ? bd[2] : 1) : 1;
  p.n = 1;
  /* kernels: [k,k,K] (2D), [k,k,W,K] (2-3D / 4D), [k,k,k,K] (3D) */
  const mwSize kdim = v3 ? 3 : 2;
  for (mwSize i = 0; i < 3; ++i) p.ksize[i] = (int32_t)(i < kdim && i < kn ? kd[i] : 1);
  const mwSize lead = kdim + (mc ? 1 : 0);
  p.K = (int32_t)(kn > lead ? kd[kn - 1] : 1);
  if (v3) {
    const mxArray* ps = prhs[10];
    const mwSize* pd = mxGetDimensions(ps);
    const mwSize pn = mxGetNumberOfDimensions(ps);
    for (mwSize i = 0; i < 3; ++i) p.psf_size[i] = (int32_t)(i < pn ? pd[i] : 1);
  }
  p.lambda_residual = mxGetScalar(prhs[4]);
  p.lambda_prior = mxGetScalar(prhs[5]);
  p.max_it = (int32_t)mxGetScalar(prhs[6]);
  p.tol = mxGetScalar(prhs[7]);
  {
    char v[16] = {0};
    if (mxGetString(prhs[8], v, sizeof v) != 0) v[0] = 0;
    p.verbose = !strcmp(v, "all") ? CCSC_VERBOSE_ALL : !strcmp(v, "brief") ? CCSC_VERBOSE_BRIEF
                                                                           : CCSC_VERBOSE_NONE;
  }
  /* the library copies exactly numel(b) doubles of mask and smooth_init, numel(b)/W of
   * x_orig and prod(size(psf)) of psf: a wrong size is an error here, as MATLAB's own
   * size checks would raise in the reference */
  if (mxGetNumberOfElements(prhs[3]) != mxGetNumberOfElements(b))
    mexErrMsgIdAndTxt("ccsc:args", "mask must have the size of b");
  if (!mxIsEmpty(prhs[9]) && mxGetNumberOfElements(prhs[9]) != mxGetNumberOfElements(b))
    mexErrMsgIdAndTxt("ccsc:args", "smooth_init must have the size of b");
  if (!mxIsEmpty(prhs[11]) &&
      mxGetNumberOfElements(prhs[11]) != mxGetNumberOfElements(b) / (mwSize)p.nch)
    mexErrMsgIdAndTxt("ccsc:args", "x_orig must have the size of one channel of b");
  if (v3 && mxIsEmpty(prhs[10]))
    mexErrMsgIdAndTxt("ccsc:args", "the video solver needs the blur psf");
  if (ccsc_solve_supported(&p, err, sizeof err)) mexErrMsgIdAndTxt("ccsc:invalid", "%s", err);
  ccsc_ctx* ctx = solve_context((int32_t)mxGetScalar(prhs[12]), err, sizeof err);

  ccsc_solve_inputs in;
  memset(&in, 0, sizeof in);
  in.b = mxGetDoubles(b);
  in.kernels = mxGetDoubles(k);
  in.mask = mxGetDoubles(prhs[3]);
  in.smooth_init = opt(prhs[9]);
  in.psf = opt(prhs[10]);
  in.x_orig = opt(prhs[11]);

  /* z: the padded code grid incl. the dirac channel of SP (last) / SV (first) */
  const int rx = mc ? 0 : p.ksize[0] / 2, ry = mc ? 0 : p.ksize[1] / 2;
  const int rt = v3 ? p.ksize[2] / 2 : 0;
  const mwSize Kc = (mwSize)p.K + ((variant == CCSC_SOLVE_POISSON2D || v3) ? 1 : 0);
  mwSize zd[4], rd[3];
  mwSize nzd = 0, nrd = 0;
  zd[nzd++] = (mwSize)(p.sb[0] + 2 * rx);
  zd[nzd++] = (mwSize)(p.sb[1] + 2 * ry);
  if (v3) zd[nzd++] = (mwSize)(p.sb[2] + 2 * rt);
  zd[nzd++] = Kc;
  rd[nrd++] = (mwSize)p.sb[0];
  rd[nrd++] = (mwSize)p.sb[1];
  if (v3) rd[nrd++] = (mwSize)p.sb[2];
  if (mc) rd[nrd++] = (mwSize)p.nch;
  ccsc_solve_outputs out;
  memset(&out, 0, sizeof out);
  plhs[0] = mxCreateNumericArray(nzd, zd, mxDOUBLE_CLASS, mxREAL);
  out.z = mxGetDoubles(plhs[0]);
  if (nlhs > 1) {
    plhs[1] = mxCreateNumericArray(nrd, rd, mxDOUBLE_CLASS, mxREAL);
    out.res = mxGetDoubles(plhs[1]);
  }

  const int cap = p.max_it + 1;
  int32_t iters = 0;
  mxArray* tr = mxCreateDoubleMatrix(3, (mwSize)cap, mxREAL);   /* obj, psnr, diff rows */
  double* t = mxGetDoubles(tr);
  double* obj = (double*)mxCalloc((size_t)cap, sizeof(double));
  double* psnr = (double*)mxCalloc((size_t)cap, sizeof(double));
  double* diff = (double*)mxCalloc((size_t)cap, sizeof(double));
  ccsc_solvelog lg;
  memset(&lg, 0, sizeof lg);
  lg.capacity = cap;
  lg.iters = &iters;
  lg.obj = obj;
  lg.psnr = psnr;
  lg.diff = diff;
  const int rc = ccsc_solve(ctx, &p, &in, &out, &lg, err, sizeof err);
  if (rc) {
    mxFree(obj);
    mxFree(psnr);
    mxFree(diff);
    mxDestroyArray(tr);
    mexErrMsgIdAndTxt("ccsc:solve", "%s (code %d)", err, rc);
  }
  if (p.verbose != CCSC_VERBOSE_NONE) {
    /* the reference's per-iterate lines (SI:69,124; SD:49,81) */
    const int has_psnr = (variant == CCSC_SOLVE_INPAINT2D || variant == CCSC_SOLVE_POISSON2D) &&
                         in.x_orig != NULL;
    for (int i = 0; i <= iters; ++i) {
      if (has_psnr)
        mexPrintf("Iter %d, Obj %3.3g, PSNR %2.2f, Diff %5.5g\n", i, obj[i], psnr[i], diff[i]);
      else
        mexPrintf("Iter %d, Obj %3.3g, Diff %5.5g\n", i, obj[i], diff[i]);
    }
  }
  for (int i = 0; i < cap; ++i) {
    t[3 * i] = obj[i];
    t[3 * i + 1] = psnr[i];
    t[3 * i + 2] = diff[i];
  }
  mxFree(obj);
  mxFree(psnr);
  mxFree(diff);
  if (nlhs > 2) {
    mxSetN(tr, (mwSize)iters + 1);
    plhs[2] = tr;   /* extra output: the trace [obj; psnr; diff] per iterate */
  } else {
    mxDestroyArray(tr);
  }
}
