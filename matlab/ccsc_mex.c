/*
 * ccsc_mex.c -- MEX gateway over libccsc (include/ccsc.h).  Thin by design:
 * marshal mxArrays (already column-major float64) into the C-ABI and back.
 * NOT compiled in this repository (no MATLAB / mex.h here); build on a MATLAB
 * host with:   mex -R2018a ccsc_mex.c -I../include -L../ccsc_code_iccv2017_amd -lccsc
 *
 * Called by the .m wrappers in this directory, which keep the reference
 * signatures (2D/admm_learn_conv2D_large_dParallel.m:1-4 etc.):
 *   [d_res, iter, z_res, DZ, obj_val] = ccsc_mex(variant, b, kernel_size,
 *        lambda_residual, lambda_prior, max_it, tol, verbose, d0, z0, devices
 *        [, smooth_init])                      (smooth_init: 2-3D learner only)
 * Outputs are ordered so that the wrappers pass their own nargout through:
 * z_res / DZ / obj_val are only allocated and copied when asked for (z_res is
 * ~97 GB at C2).  `devices` is a vector of GPU indices (ccsc_device.m): more
 * than one runs the learner over those GPUs from this one call
 * (ccsc_create_multi: one host thread per device, RCCL over xGMI).
 * Output shapes per variant (what the library writes, include/ccsc.h):
 *   dP / dZ  d_res [s,s,K]      z_res [X,Y,K,n]      DZ [X,Y,1,n]
 *   3D       d_res [s,s,s,K]    z_res [X,Y,T,K,n]    DZ [X,Y,T,n]
 *   4D       d_res [s,s,U,V,K]  z_res [X,Y,1,1,K,n]  DZ [x,y,U,V,n] (cropped, L4:205-206)
 *   2-3D     d_res [s,s,W,K]    z_res [X,Y,K,n]      DZ [X,Y,W,n]   (incl. smoothinit)
 */
#include "mex.h"
#include "ccsc.h"

#include <string.h>

#define CCSC_MEX_MAXDEV 64
static ccsc_ctx* g_ctx = NULL;
static int32_t g_devs[CCSC_MEX_MAXDEV];
static int g_ndev = 0;

static void cleanup(void) {
  if (g_ctx) ccsc_destroy(g_ctx);
  g_ctx = NULL;
  g_ndev = 0;
}

/* the cached context when it serves the same device list, else a new one */
static ccsc_ctx* context_for(const mxArray* a, int first_only, char* err, size_t errlen) {
  const mwSize nd = first_only && mxGetNumberOfElements(a) > 0 ? 1 : mxGetNumberOfElements(a);
  if (nd < 1 || nd > CCSC_MEX_MAXDEV)
    mexErrMsgIdAndTxt("ccsc:devices", "devices must list 1..%d GPU indices", CCSC_MEX_MAXDEV);
  int32_t devs[CCSC_MEX_MAXDEV];
  const double* dv = mxGetDoubles(a);
  for (mwSize i = 0; i < nd; ++i) devs[i] = (int32_t)dv[i];
  if (g_ctx && g_ndev == (int)nd && !memcmp(g_devs, devs, nd * sizeof(int32_t))) return g_ctx;
  cleanup();
  g_ctx = ccsc_create_multi(devs, (int32_t)nd, err, errlen);
  if (!g_ctx) mexErrMsgIdAndTxt("ccsc:hip", "%s", err);
  memcpy(g_devs, devs, nd * sizeof(int32_t));
  g_ndev = (int)nd;
  mexAtExit(cleanup);
  return g_ctx;
}

static void progress(void* user, int32_t it, double od, double oz, double t) {
  (void)user;
  mexPrintf("Iter %d, Obj %3.3g / %3.3g, %.2f s\n", it, od, oz, t);  /* calling thread only */
  mexEvalString("drawnow;");
}

static mxArray* zeros_nd(mwSize nd, const mwSize* d) {
  return mxCreateNumericArray(nd, d, mxDOUBLE_CLASS, mxREAL);
}

void mexFunction(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
  char err[1024] = {0};
  if (nrhs < 11) mexErrMsgIdAndTxt("ccsc:args", "ccsc_mex needs 11 arguments (12 for 2-3D)");
  const int variant = (int)mxGetScalar(prhs[0]);
  const mxArray* b = prhs[1];
  if (!mxIsDouble(b) || mxIsComplex(b)) mexErrMsgIdAndTxt("ccsc:b", "b must be real double");
  const double* ks = mxGetDoubles(prhs[2]);
  const mwSize nks = mxGetNumberOfElements(prhs[2]);
  const mwSize* bd = mxGetDimensions(b);
  const mwSize bn = mxGetNumberOfDimensions(b);

  ccsc_problem p;
  memset(&p, 0, sizeof p);
  p.variant = variant;
  p.ndim = (variant == CCSC_L3D) ? 3 : 2;
  for (int i = 0; i < p.ndim; ++i) p.sb[i] = (int64_t)bd[i];
  p.views[0] = p.views[1] = 1;
  if (variant == CCSC_L4D && nks == 5) { p.views[0] = (int32_t)ks[2]; p.views[1] = (int32_t)ks[3]; }
  if (variant == CCSC_HS23 && nks == 4) p.views[0] = (int32_t)ks[2];
  /* n = size(b, end): b is [sb..., (U,V | W), n] */
  const mwSize lead = (mwSize)p.ndim + (variant == CCSC_L4D ? 2 : variant == CCSC_HS23 ? 1 : 0);
  p.n = (int64_t)(bn > lead ? bd[bn - 1] : 1);
  p.K = (int32_t)ks[nks - 1];
  p.psf = (int32_t)ks[0];
  p.lambda_residual = mxGetScalar(prhs[3]);
  p.lambda_prior = mxGetScalar(prhs[4]);
  p.max_it = (int32_t)mxGetScalar(prhs[5]);
  p.tol = mxGetScalar(prhs[6]);
  {
    char v[16] = {0};
    mxGetString(prhs[7], v, sizeof v);
    p.verbose = !strcmp(v, "all") ? CCSC_VERBOSE_ALL : !strcmp(v, "brief") ? CCSC_VERBOSE_BRIEF
                                                                           : CCSC_VERBOSE_NONE;
  }
  p.precision = CCSC_FP64;
  if (ccsc_resolve(&p, err, sizeof err)) mexErrMsgIdAndTxt("ccsc:invalid", "%s", err);

  const double* smooth = NULL;
  if (variant == CCSC_HS23) {
    if (nrhs < 12 || mxGetNumberOfElements(prhs[11]) != mxGetNumberOfElements(b))
      mexErrMsgIdAndTxt("ccsc:args", "the 2-3D learner needs smooth_init of size(b)");
    smooth = mxGetDoubles(prhs[11]);
  }

  if (!mxIsDouble(prhs[10])) mexErrMsgIdAndTxt("ccsc:devices", "devices must be double");
  const double* d0 = mxIsEmpty(prhs[8]) ? NULL : mxGetDoubles(prhs[8]);
  const double* z0 = mxIsEmpty(prhs[9]) ? NULL : mxGetDoubles(prhs[9]);

  /* outputs: allocate only what nargout asks for (z_res is ~97 GB at C2) */
  const int64_t r = p.psf / 2;
  const mwSize s = (mwSize)p.psf, K = (mwSize)p.K, n = (mwSize)p.n;
  const mwSize X = (mwSize)(p.sb[0] + 2 * r), Y = (mwSize)(p.sb[1] + 2 * r);
  const mwSize T = (mwSize)(p.ndim == 3 ? p.sb[2] + 2 * r : 1);
  const mwSize U = (mwSize)p.views[0], V = (mwSize)p.views[1];
  /* the library copies exactly these many doubles from init.d / init.z: a wrong size
   * is an error here, as MATLAB's own size checks would raise in the reference */
  {
    const mwSize nd0 = s * s * (p.ndim == 3 ? s : 1) * (variant == CCSC_L4D ? U * V : 1) * K;
    const mwSize nz0 = X * Y * T * K * (variant == CCSC_DZPAR ? (mwSize)p.ni : n);
    if (d0 && mxGetNumberOfElements(prhs[8]) != nd0)
      mexErrMsgIdAndTxt("ccsc:args", "init.d must have %d elements", (int)nd0);
    if (z0 && mxGetNumberOfElements(prhs[9]) != nz0)
      mexErrMsgIdAndTxt("ccsc:args", "init.z must have %.0f elements", (double)nz0);
    if ((d0 && (!mxIsDouble(prhs[8]) || mxIsComplex(prhs[8]))) ||
        (z0 && (!mxIsDouble(prhs[9]) || mxIsComplex(prhs[9]))))
      mexErrMsgIdAndTxt("ccsc:args", "init.d / init.z must be real double");
  }
  /* the 2-3D learner runs on one GPU (its d-solve couples every image per frequency) */
  ccsc_ctx* ctx = context_for(prhs[10], variant == CCSC_HS23, err, sizeof err);
  mwSize dd[5], zd[6], xd[5];
  mwSize ndd, nzd, nxd;
  switch (variant) {
    case CCSC_L3D:
      ndd = 4; dd[0] = s; dd[1] = s; dd[2] = s; dd[3] = K;
      nzd = 5; zd[0] = X; zd[1] = Y; zd[2] = T; zd[3] = K; zd[4] = n;
      nxd = 4; xd[0] = X; xd[1] = Y; xd[2] = T; xd[3] = n;
      break;
    case CCSC_L4D:
      ndd = 5; dd[0] = s; dd[1] = s; dd[2] = U; dd[3] = V; dd[4] = K;
      nzd = 6; zd[0] = X; zd[1] = Y; zd[2] = 1; zd[3] = 1; zd[4] = K; zd[5] = n;
      nxd = 5; xd[0] = (mwSize)p.sb[0]; xd[1] = (mwSize)p.sb[1]; xd[2] = U; xd[3] = V; xd[4] = n;
      break;
    case CCSC_HS23:
      ndd = 4; dd[0] = s; dd[1] = s; dd[2] = U; dd[3] = K;
      nzd = 4; zd[0] = X; zd[1] = Y; zd[2] = K; zd[3] = n;
      nxd = 4; xd[0] = X; xd[1] = Y; xd[2] = U; xd[3] = n;
      break;
    default:
      ndd = 3; dd[0] = s; dd[1] = s; dd[2] = K;
      nzd = 4; zd[0] = X; zd[1] = Y; zd[2] = K; zd[3] = n;
      nxd = 4; xd[0] = X; xd[1] = Y; xd[2] = 1; xd[3] = n;
  }
  ccsc_outputs out;
  memset(&out, 0, sizeof out);
  plhs[0] = zeros_nd(ndd, dd);
  out.d_res = mxGetDoubles(plhs[0]);
  if (nlhs > 2) {
    plhs[2] = zeros_nd(nzd, zd);
    out.z_res = mxGetDoubles(plhs[2]);
  }
  if (nlhs > 3) {
    plhs[3] = zeros_nd(nxd, xd);
    out.DZ = mxGetDoubles(plhs[3]);
  }
  double obj = 0;
  if (nlhs > 4) out.obj_val = &obj;

  const int cap = p.max_it + 1;
  mxArray* od = mxCreateDoubleMatrix(1, cap, mxREAL);
  mxArray* oz = mxCreateDoubleMatrix(1, cap, mxREAL);
  mxArray* tv = mxCreateDoubleMatrix(1, cap, mxREAL);
  ccsc_iterlog lg;
  memset(&lg, 0, sizeof lg);
  lg.capacity = cap;
  lg.obj_vals_d = mxGetDoubles(od);
  lg.obj_vals_z = mxGetDoubles(oz);
  lg.tim_vals = mxGetDoubles(tv);

  ccsc_cb cb = p.verbose == CCSC_VERBOSE_NONE ? NULL : progress;
  const int rc = variant == CCSC_HS23
                     ? ccsc_learn_hs23(ctx, &p, mxGetDoubles(b), smooth, d0, z0, &out, &lg, cb,
                                       NULL, err, sizeof err)
                     : ccsc_learn(ctx, &p, mxGetDoubles(b), d0, z0, &out, &lg, cb, NULL, err,
                                  sizeof err);
  if (rc) mexErrMsgIdAndTxt("ccsc:learn", "%s (code %d)", err, rc);
  mxSetN(od, lg.count);
  mxSetN(oz, lg.count);
  mxSetN(tv, lg.count);
  if (nlhs > 4) plhs[4] = mxCreateDoubleScalar(obj);
  if (nlhs > 1) {
    const char* f[] = {"obj_vals_d", "obj_vals_z", "tim_vals"};
    plhs[1] = mxCreateStructMatrix(1, 1, 3, f);
    mxSetField(plhs[1], 0, "obj_vals_d", od);
    mxSetField(plhs[1], 0, "obj_vals_z", oz);
    mxSetField(plhs[1], 0, "tim_vals", tv);
  } else {
    mxDestroyArray(od);
    mxDestroyArray(oz);
    mxDestroyArray(tv);
  }
}
