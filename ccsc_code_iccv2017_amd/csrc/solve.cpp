// libccsc reconstruction solvers: planning, the ADMM schedule and the C-ABI
// ccsc_solve (kernels in recon.hip).
//
// Per iteration (SI:81-139 and its siblings), one launch each:
//   rows(codes)  C2R of zhat -> z (tol partials) -> ProxSparse / dual -> R2C x-lines of xi2
//   rows(data)   C2R of sum_k dhat zhat -> v1 (objective partials) -> data prox / dual
//                -> R2C x-lines of xi1
//   cols fwd     y (and t) lines of both spectrum sets
//   solve        Sherman-Morrison (SI, SP) or the diagonal form (SD, SL, SV) per bin,
//                plus the synthesis sum_k dhat zhat that becomes the next v1
//   cols inv
// The partial sums are read back only when the tol test or the verbose trace needs
// them; the reconstruction is formed after the last iteration from z (fft2(z) ==
// zhat for the Hermitian iterates of these real problems).
#include "host.hpp"
#include "recon.hpp"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <functional>
#include <limits>

namespace ccsc {

static const int kNativeRad[] = {11, 10, 8, 7, 5, 4, 3, 2};   // fft_pass_dispatch

static bool native_rad(int R) {
  for (int r : kNativeRad)
    if (r == R) return true;
  return false;
}

static int64_t gen_tasks(int n, int nlines, int R) {
  return (int64_t)nlines * (n / R) * (((R - 1) / 2 + kGenericQP - 1) / kGenericQP);
}

// Line plan of length n for `nlines` lines per workgroup: fewest passes (<= kPlanSlots),
// then fewest generic passes.  Native radices need (n/R) * nlines butterflies within
// the register budget; any other odd factor runs as a generic pass (fft_pass_generic,
// one task per thread).  Lengths with an even factor outside {2,4,8,10} beyond the
// native set, e.g. 2^5 * 3 = 96 = 8 * 4 * 3, still plan.
static bool plan_line(int n, int nlines, Plan1D& out) {
  if (n == 1) {
    out = Plan1D{};
    out.n = 1;
    return true;
  }
  Plan1D best{};
  int best_np = 99, best_ng = 99;
  std::vector<int> cur;
  std::function<void(int, int)> dfs = [&](int rem, int ng) {
    if (rem == 1) {
      const int np = (int)cur.size();
      if (np < best_np || (np == best_np && ng < best_ng)) {
        best_np = np;
        best_ng = ng;
        best = Plan1D{};
        best.n = n;
        best.npass = np;
        for (int i = 0; i < np; ++i) best.rad[i] = cur[i];
      }
      return;
    }
    if ((int)cur.size() >= kPlanSlots || (int)cur.size() + 1 > best_np) return;
    for (int R : kNativeRad) {
      if (rem % R) continue;
      if ((int64_t)(n / R) * nlines > (int64_t)maxb_for_radix(R) * kLineBS * kLineNT) continue;
      cur.push_back(R);
      dfs(rem / R, ng);
      cur.pop_back();
    }
    for (int R = 3; R <= rem; R += 2) {
      if (rem % R || native_rad(R)) continue;
      if (gen_tasks(n, nlines, R) > (int64_t)kLineGT * kLineNT) continue;
      cur.push_back(R);
      dfs(rem / R, ng + 1);
      cur.pop_back();
    }
  };
  dfs(n, 0);
  if (best_np == 99) return false;
  out = best;
  return true;
}

// twiddle tables of one plan, appended to t (offsets into t in p.twoff)
static void add_twiddles(Plan1D& p, std::vector<cpx<double>>& t) {
  const long double pi = 3.141592653589793238462643383279502884L;
  int Ns = 1;
  for (int s = 0; s < p.npass; ++s) {
    const int R = p.rad[s];
    p.twoff[s] = (int)t.size();
    for (int r = 1; r < R; ++r)
      for (int k = 0; k < Ns; ++k) {
        const long double a = -2.0L * pi * (long double)(r * k) / (long double)(Ns * R);
        t.push_back({(double)cosl(a), (double)sinl(a)});
      }
    if (!native_rad(R))
      for (int m = 0; m < R; ++m) {
        const long double a = -2.0L * pi * (long double)m / (long double)R;
        t.push_back({(double)cosl(a), (double)sinl(a)});
      }
    Ns *= R;
  }
}

// LDS budget of one line-kernel workgroup (four or more per CU)
static size_t line_lds() { return (size_t)40 * 1024; }

static int twiddle_count(const Plan1D& p) {
  int n = 0, Ns = 1;
  for (int s = 0; s < p.npass; ++s) {
    n += (p.rad[s] - 1) * Ns + (native_rad(p.rad[s]) ? 0 : p.rad[s]);
    Ns *= p.rad[s];
  }
  return std::max(n, 1);
}

static bool plan_rows(int X, int rows, RowGeom& rg) {
  rg = RowGeom{};
  Grid2D& G = rg.G;
  G.X = X;
  G.Xh = X / 2 + 1;
  G.RS = 2 * G.Xh;
  while (G.RS % 16 != 6) G.RS += 2;   // column-pair lines off the same LDS banks (engine.cpp)
  rg.rows = rows;
  for (int L = (rows + 1) / 2; L >= 1; --L) {
    rg.L = L;
    if (!plan_line(X, L, G.px)) continue;
    rg.ntw = twiddle_count(G.px);
    if (rows_smem_bytes(rg, sizeof(double)) > line_lds()) continue;
    rg.groups = (rows + 2 * L - 1) / (2 * L);
    return true;
  }
  return false;
}

static bool plan_cols(int n, int Xh, ColGeom& cg) {
  cg = ColGeom{};
  cg.n = n;
  cg.Xh = Xh;
  for (int TC = std::min(32, Xh); TC >= 1; --TC) {
    cg.TC = TC;
    if (!plan_line(n, TC, cg.p)) continue;
    cg.ntw = twiddle_count(cg.p);
    if (cols_smem_bytes(cg, sizeof(double)) > line_lds()) continue;
    cg.xtiles = (Xh + TC - 1) / TC;
    return true;
  }
  return false;
}

bool gfft_plan(int X, int Y, RowGeom& rg, ColGeom& cy, std::vector<cpx<double>>& tw_rows,
               std::vector<cpx<double>>& tw_cy) {
  if (!plan_rows(X, Y, rg) || !plan_cols(Y, X / 2 + 1, cy)) return false;
  const int Xh = X / 2 + 1;
  cy.es = Xh;
  cy.ninner = 1;
  cy.sin = 0;
  cy.sout = (int64_t)Xh * Y;
  tw_rows.clear();
  tw_cy.clear();
  add_twiddles(rg.G.px, tw_rows);
  add_twiddles(cy.p, tw_cy);
  return true;
}

// 3D grids X x Y x T (the 3D learner's slices past one CU's LDS or past the t-tile
// kernels): rows over the Y T rows of a slice, y-lines per plane, t-lines over the Y rows
// of a slice (the video solver's passes, resolve_solve)
bool gfft_plan3(int X, int Y, int Tn, RowGeom& rg, ColGeom& cy, ColGeom& ct,
                std::vector<cpx<double>>& tw_rows, std::vector<cpx<double>>& tw_cy,
                std::vector<cpx<double>>& tw_ct) {
  if (!plan_rows(X, Y * Tn, rg) || !plan_cols(Y, X / 2 + 1, cy) || !plan_cols(Tn, X / 2 + 1, ct))
    return false;
  const int Xh = X / 2 + 1;
  cy.es = Xh;
  cy.ninner = 1;
  cy.sin = 0;
  cy.sout = (int64_t)Xh * Y;
  ct.es = (int64_t)Xh * Y;
  ct.ninner = Y;
  ct.sin = Xh;
  ct.sout = (int64_t)Xh * Y * Tn;
  tw_rows.clear();
  tw_cy.clear();
  tw_ct.clear();
  add_twiddles(rg.G.px, tw_rows);
  add_twiddles(cy.p, tw_cy);
  add_twiddles(ct.p, tw_ct);
  return true;
}

// ---------------------------------------------------------------------------
// problem resolution
// ---------------------------------------------------------------------------
struct SolveSpec {
  ccsc_solve_problem p;
  int nd = 2;              // transform dims
  int X = 0, Y = 0, Tn = 1;
  int rx = 0, ry = 0, rt = 0;
  int Kc = 0;              // code channels (incl. the dirac of SP / SV)
  int W = 1;               // data channels
  int64_t P = 0, F = 0;    // voxels / half-spectrum bins per slice
  double c_gamma = 0;      // gamma_heuristic = c_gamma * lambda / max(b)
  double g1_div = 1;       // gamma(1) = gamma_heuristic / g1_div
  double rho = 0;          // z-solve rho
  RowGeom rg{};
  ColGeom cy{}, ct{};
  std::vector<cpx<double>> tw_rows, tw_cy, tw_ct;
};

static void resolve_solve(const ccsc_solve_problem& pin, SolveSpec& S) {
  S.p = pin;
  ccsc_solve_problem& p = S.p;
  if (p.variant < CCSC_SOLVE_INPAINT2D || p.variant > CCSC_SOLVE_VIDEO3D)
    throw Err(CCSC_E_INVALID, "unknown solver variant");
  const bool v3 = p.variant == CCSC_SOLVE_VIDEO3D;
  S.nd = v3 ? 3 : 2;
  if (!v3) p.sb[2] = 1;
  for (int i = 0; i < S.nd; ++i)
    if (p.sb[i] <= 0) throw Err(CCSC_E_INVALID, "image extent must be positive");
  if (p.n <= 0) throw Err(CCSC_E_INVALID, "n must be positive");
  if (p.K <= 0) throw Err(CCSC_E_INVALID, "K must be positive");
  if (p.max_it < 0) throw Err(CCSC_E_INVALID, "max_it must be >= 0");
  if (p.verbose < CCSC_VERBOSE_NONE || p.verbose > CCSC_VERBOSE_ALL)
    throw Err(CCSC_E_INVALID, "bad verbose");
  if (!v3) p.ksize[2] = 1;
  for (int i = 0; i < S.nd; ++i)
    if (p.ksize[i] <= 0) throw Err(CCSC_E_INVALID, "filter extent must be positive");
  if (p.variant == CCSC_SOLVE_MULTICH) {
    if (p.nch <= 0) throw Err(CCSC_E_INVALID, "MULTICH needs the channel count W = size(b, 3)");
    S.W = p.nch;
  } else {
    p.nch = 1;
  }
  if (v3)
    for (int i = 0; i < 3; ++i)
      if (p.psf_size[i] <= 0) throw Err(CCSC_E_INVALID, "VIDEO3D needs the psf extent");
  // psf_radius = floor(size(kmat)/2) and the padded grid (SI:10-11, SP:10-11, SV:10-11);
  // SD/SL do not pad (psf_radius = [0 0], SD:5)
  if (p.variant != CCSC_SOLVE_MULTICH) {
    S.rx = p.ksize[0] / 2;
    S.ry = p.ksize[1] / 2;
    S.rt = v3 ? p.ksize[2] / 2 : 0;
  }
  S.X = (int)(p.sb[0] + 2 * S.rx);
  S.Y = (int)(p.sb[1] + 2 * S.ry);
  S.Tn = v3 ? (int)(p.sb[2] + 2 * S.rt) : 1;
  if (p.variant == CCSC_SOLVE_MULTICH && (p.ksize[0] > S.X || p.ksize[1] > S.Y))
    throw Err(CCSC_E_INVALID, "filters larger than the image (psf2otf)");
  if (v3 && (p.psf_size[0] > S.X || p.psf_size[1] > S.Y || p.psf_size[2] > S.Tn))
    throw Err(CCSC_E_INVALID, "psf larger than the padded grid (psf2otf)");
  for (int i = 0; i < S.nd; ++i) {
    const int r = i == 0 ? S.rx : (i == 1 ? S.ry : S.rt);
    if (r > p.sb[i]) throw Err(CCSC_E_INVALID, "symmetric padding wider than the image");
  }
  S.Kc = p.K + ((p.variant == CCSC_SOLVE_POISSON2D || v3) ? 1 : 0);
  S.P = (int64_t)S.X * S.Y * S.Tn;
  S.F = (int64_t)(S.X / 2 + 1) * S.Y * S.Tn;
  switch (p.variant) {
    case CCSC_SOLVE_INPAINT2D: S.c_gamma = 60; S.g1_div = 100; S.rho = 100; break;   // SI:36-37,178
    case CCSC_SOLVE_POISSON2D: S.c_gamma = 20; S.g1_div = 5; S.rho = 5; break;       // SP:34-35,179
    case CCSC_SOLVE_MULTICH: S.c_gamma = 60; S.g1_div = 1; S.rho = S.W; break;        // SD:31-32,126
    case CCSC_SOLVE_VIDEO3D: S.c_gamma = 500; S.g1_div = 1; S.rho = S.Tn; break;      // SV:36-37,149
  }
  if (!(p.lambda_prior > 0)) throw Err(CCSC_E_INVALID, "lambda_prior must be positive (gamma heuristic)");
  // transform plans
  if (!plan_rows(S.X, S.Y * S.Tn, S.rg))
    throw Err(CCSC_E_UNSUPPORTED, "grid length " + std::to_string(S.X) + " has no line plan");
  if (!plan_cols(S.Y, S.X / 2 + 1, S.cy))
    throw Err(CCSC_E_UNSUPPORTED, "grid length " + std::to_string(S.Y) + " has no line plan");
  const int Xh = S.X / 2 + 1;
  S.cy.es = Xh;
  S.cy.ninner = 1;
  S.cy.sin = 0;
  S.cy.sout = (int64_t)Xh * S.Y;
  add_twiddles(S.rg.G.px, S.tw_rows);
  add_twiddles(S.cy.p, S.tw_cy);
  if (v3) {
    if (!plan_cols(S.Tn, Xh, S.ct))
      throw Err(CCSC_E_UNSUPPORTED, "grid length " + std::to_string(S.Tn) + " has no line plan");
    S.ct.es = (int64_t)Xh * S.Y;
    S.ct.ninner = S.Y;
    S.ct.sin = Xh;
    S.ct.sout = (int64_t)Xh * S.Y * S.Tn;
    add_twiddles(S.ct.p, S.tw_ct);
  }
  if (S.F > INT32_MAX / 2 || (int64_t)S.Kc * S.W > 65535 * 4)
    throw Err(CCSC_E_UNSUPPORTED, "spectrum too large for the per-bin kernels");
  if (p.n > 65535) throw Err(CCSC_E_UNSUPPORTED, "more than 65535 images in one call");
}

// ---------------------------------------------------------------------------
// the solver session (one call)
// ---------------------------------------------------------------------------
struct Solver {
  SolveSpec S;
  hipStream_t st;
  int64_t n;
  DevBuf tw_r, tw_y, tw_t;
  DevBuf dhat, dhat_res, senergy;
  DevBuf Sz, Sx, Z, D2, D1, M, Mb, SM, XO;
  DevBuf part, sums, theta1, theta2, active;
  std::vector<double> h_theta1, h_theta2;

  Solver(ccsc_ctx* ctx, const ccsc_solve_problem& p) : st(ctx->stream) {
    resolve_solve(p, S);
    n = S.p.n;
  }

  template <typename X> static X* ptr(DevBuf& b) { return b.as<X>(); }
  cpx<double>* tw(DevBuf& b) { return b.as<cpx<double>>(); }

  void upload_tw(DevBuf& b, const std::vector<cpx<double>>& t) {
    b.alloc(std::max<size_t>(t.size(), 1) * 16);
    if (!t.empty()) HIPCHK(hipMemcpyAsync(b.p, t.data(), t.size() * 16, hipMemcpyHostToDevice, st));
  }

  // forward transform of `count` real grid slices (src) into spectra (dst)
  void fwd(const double* src, cpx<double>* dst, int64_t count) {
    RowArgs<double> a{};
    a.S = dst;
    a.src = src;
    a.per_img = 1;
    HIPCHK(launch_rows<double>(kRowFwd, a, count, S.rg, tw(tw_r), st));
    cols(dst, -1, count);
  }
  void cols(cpx<double>* sp, int sign, int64_t count) {
    if (sign < 0) {
      HIPCHK(launch_cols<double>(sp, -1, count * S.Tn, S.cy, tw(tw_y), st));
      if (S.nd == 3) HIPCHK(launch_cols<double>(sp, -1, count * S.Y, S.ct, tw(tw_t), st));
    } else {
      if (S.nd == 3) HIPCHK(launch_cols<double>(sp, +1, count * S.Y, S.ct, tw(tw_t), st));
      HIPCHK(launch_cols<double>(sp, +1, count * S.Tn, S.cy, tw(tw_y), st));
    }
  }

  // both spectrum sets (codes, data) in one launch per line direction
  void cols2(int sign, int64_t nz, int64_t nx) {
    cpx<double>* a = Sz.as<cpx<double>>();
    cpx<double>* b = Sx.as<cpx<double>>();
    if (sign < 0) {
      HIPCHK(launch_cols<double>(a, -1, nz * S.Tn, S.cy, tw(tw_y), st, b, nx * S.Tn));
      if (S.nd == 3) HIPCHK(launch_cols<double>(a, -1, nz * S.Y, S.ct, tw(tw_t), st, b, nx * S.Y));
    } else {
      if (S.nd == 3) HIPCHK(launch_cols<double>(a, +1, nz * S.Y, S.ct, tw(tw_t), st, b, nx * S.Y));
      HIPCHK(launch_cols<double>(a, +1, nz * S.Tn, S.cy, tw(tw_y), st, b, nx * S.Tn));
    }
  }

  void setup(const ccsc_solve_inputs& in) {
    const ccsc_solve_problem& p = S.p;
    if (!in.b || !in.kernels || !in.mask) throw Err(CCSC_E_INVALID, "b, kernels and mask are required");
    const bool v3 = p.variant == CCSC_SOLVE_VIDEO3D;
    const bool has_sm = p.variant != CCSC_SOLVE_POISSON2D;
    if (has_sm && !in.smooth_init) throw Err(CCSC_E_INVALID, "smooth_init is required");
    if (v3 && !in.psf) throw Err(CCSC_E_INVALID, "VIDEO3D needs the psf");
    const bool psnr = in.x_orig && (p.variant == CCSC_SOLVE_INPAINT2D ||
                                    p.variant == CCSC_SOLVE_POISSON2D);
    upload_tw(tw_r, S.tw_rows);
    upload_tw(tw_y, S.tw_cy);
    upload_tw(tw_t, S.tw_ct);
    const int64_t P = S.P, F = S.F;
    const int Kc = S.Kc, W = S.W;
    // ---- filter spectra (psf2otf of every filter; SI:155-162, SD:100-115, SV:121-138)
    const int kx = p.ksize[0], ky = p.ksize[1], kt = v3 ? p.ksize[2] : 1;
    const int64_t kvol = (int64_t)kx * ky * kt;
    const int64_t nfilt = (int64_t)Kc * W;
    std::vector<double> hk((size_t)(kvol * nfilt), 0.0);
    const int64_t nlearn = (int64_t)p.K * W;
    const int64_t koff = v3 ? kvol : 0;   // SV prepends the dirac (SV:7), SP appends it (SP:7)
    std::memcpy(hk.data() + koff, in.kernels, (size_t)(kvol * nlearn) * 8);
    if (p.variant == CCSC_SOLVE_POISSON2D || v3) {
      double* dk = hk.data() + (v3 ? 0 : kvol * nlearn);
      dk[(int64_t)(kt / 2) * kx * ky + (int64_t)(ky / 2) * kx + kx / 2] = 1.0;   // SP:6, SV:6
    }
    {
      DevBuf kd, grid;
      kd.alloc(hk.size() * 8);
      HIPCHK(hipMemcpyAsync(kd.p, hk.data(), kd.bytes, hipMemcpyHostToDevice, st));
      grid.alloc((size_t)(nfilt * P) * 8);
      HIPCHK(hipMemsetAsync(grid.p, 0, grid.bytes, st));
      HIPCHK(launch_embed_kernels<double>(kd.as<double>(), grid.as<double>(), kx, ky, kt,
                                          (int)nfilt, S.X, S.Y, S.Tn, st));
      dhat.alloc((size_t)(nfilt * F) * 16);
      fwd(grid.as<double>(), dhat.as<cpx<double>>(), nfilt);
      if (v3) {
        // dhat = psf_hat .* dhat_k (SV:131); the reconstruction keeps dhat_k (SV:109)
        dhat_res.alloc(dhat.bytes);
        HIPCHK(hipMemcpyAsync(dhat_res.p, dhat.p, dhat.bytes, hipMemcpyDeviceToDevice, st));
        const int64_t pvol = (int64_t)p.psf_size[0] * p.psf_size[1] * p.psf_size[2];
        DevBuf pd, pg, ph;
        pd.alloc((size_t)pvol * 8);
        HIPCHK(hipMemcpyAsync(pd.p, in.psf, pd.bytes, hipMemcpyHostToDevice, st));
        pg.alloc((size_t)P * 8);
        HIPCHK(hipMemsetAsync(pg.p, 0, pg.bytes, st));
        HIPCHK(launch_embed_kernels<double>(pd.as<double>(), pg.as<double>(), p.psf_size[0],
                                            p.psf_size[1], p.psf_size[2], 1, S.X, S.Y, S.Tn, st));
        ph.alloc((size_t)F * 16);
        fwd(pg.as<double>(), ph.as<cpx<double>>(), 1);
        HIPCHK(launch_spec_mul<double>(dhat.as<cpx<double>>(), ph.as<cpx<double>>(), F, (int)nfilt, st));
        HIPCHK(hipStreamSynchronize(st));
      }
      HIPCHK(hipStreamSynchronize(st));
    }
    // s = sum |dhat|^2 (SI:166); the diagonal solves keep invP / (rho + s) (SD:132, SV:155)
    senergy.alloc((size_t)F * 8);
    const bool diag = p.variant == CCSC_SOLVE_MULTICH || v3;
    HIPCHK(launch_spec_energy<double>(dhat.as<cpx<double>>(), senergy.as<double>(), F, (int)nfilt,
                                      diag ? 1 : 0, S.rho, 1.0 / (double)P, st));
    // ---- per-image data on the padded grid
    const int64_t sbv = p.sb[0] * p.sb[1] * p.sb[2];
    const int64_t nd = n * W;   // data slices
    {
      DevBuf b, mk, sm, xo;
      b.alloc((size_t)(nd * sbv) * 8);
      mk.alloc(b.bytes);
      HIPCHK(hipMemcpyAsync(b.p, in.b, b.bytes, hipMemcpyHostToDevice, st));
      HIPCHK(hipMemcpyAsync(mk.p, in.mask, mk.bytes, hipMemcpyHostToDevice, st));
      if (has_sm) {
        sm.alloc(b.bytes);
        HIPCHK(hipMemcpyAsync(sm.p, in.smooth_init, sm.bytes, hipMemcpyHostToDevice, st));
      }
      if (psnr) {
        xo.alloc((size_t)(n * sbv) * 8);
        HIPCHK(hipMemcpyAsync(xo.p, in.x_orig, xo.bytes, hipMemcpyHostToDevice, st));
      }
      M.alloc((size_t)(nd * P) * 8);
      Mb.alloc(M.bytes);
      if (has_sm) SM.alloc(M.bytes);
      if (psnr) XO.alloc(M.bytes);
      HIPCHK(launch_pad_inputs<double>(b.as<double>(), mk.as<double>(), sm.as<double>(),
                                       xo.as<double>(), M.as<double>(), Mb.as<double>(),
                                       SM.as<double>(), XO.as<double>(), nd, (int)p.sb[0],
                                       (int)p.sb[1], (int)p.sb[2], S.rx, S.ry, S.rt, S.X, S.Y,
                                       S.Tn, st));
      // gamma_heuristic = c * lambda / max(b(:)) per image (SI:36)
      DevBuf scratch, mx;
      scratch.alloc(2 * kNormParts * 8);
      mx.alloc((size_t)n * 8);
      for (int64_t i = 0; i < n; ++i)
        HIPCHK(launch_max<double>(b.as<double>() + i * W * sbv, W * sbv, scratch.as<double>(),
                                  mx.as<double>() + i, st));
      std::vector<double> hmax((size_t)n);
      HIPCHK(hipMemcpyAsync(hmax.data(), mx.p, mx.bytes, hipMemcpyDeviceToHost, st));
      HIPCHK(hipStreamSynchronize(st));
      h_theta1.resize((size_t)n);
      h_theta2.resize((size_t)n);
      for (int64_t i = 0; i < n; ++i) {
        const double gh = S.c_gamma * p.lambda_prior / hmax[(size_t)i];
        h_theta1[(size_t)i] = p.lambda_residual / (gh / S.g1_div);   // lambda(1)/gamma(1) (SI:88)
        h_theta2[(size_t)i] = p.lambda_prior / gh;                   // lambda(2)/gamma(2) (SI:89)
      }
    }
    theta1.alloc((size_t)n * 8);
    theta2.alloc((size_t)n * 8);
    HIPCHK(hipMemcpyAsync(theta1.p, h_theta1.data(), theta1.bytes, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(theta2.p, h_theta2.data(), theta2.bytes, hipMemcpyHostToDevice, st));
    // ---- state
    Sz.alloc((size_t)(n * Kc * F) * 16);
    Sx.alloc((size_t)(nd * F) * 16);
    Z.alloc((size_t)(n * Kc * P) * 8);
    D2.alloc(Z.bytes);
    D1.alloc((size_t)(nd * P) * 8);
    HIPCHK(hipMemsetAsync(Z.p, 0, Z.bytes, st));
    HIPCHK(hipMemsetAsync(D2.p, 0, D2.bytes, st));
    HIPCHK(hipMemsetAsync(D1.p, 0, D1.bytes, st));
    part.alloc((size_t)(n * (Kc + W) * S.rg.groups * kRowParts) * 8);
    sums.alloc((size_t)(n * kRowParts) * 8);
    active.alloc((size_t)n * 4);
    std::vector<int> ones((size_t)n, 1);
    HIPCHK(hipMemcpyAsync(active.p, ones.data(), active.bytes, hipMemcpyHostToDevice, st));
    HIPCHK(hipStreamSynchronize(st));
  }

  RowArgs<double> code_args(bool first) {
    RowArgs<double> a{};
    a.S = Sz.as<cpx<double>>();
    a.Z = Z.as<double>();
    a.D = D2.as<double>();
    a.part = part.as<double>();
    a.part_slices = S.Kc + S.W;
    a.part_off = 0;
    a.active = active.as<int>();
    a.theta = theta2.as<double>();
    a.per_img = S.Kc;
    a.first = first ? 1 : 0;
    a.prox = S.p.variant == CCSC_SOLVE_POISSON2D ? 1 : 0;
    a.Y = S.Y;
    return a;
  }
  RowArgs<double> data_args(bool first) {
    const ccsc_solve_problem& p = S.p;
    RowArgs<double> a{};
    a.S = Sx.as<cpx<double>>();
    a.D = D1.as<double>();
    a.M = M.as<double>();
    a.Mb = Mb.as<double>();
    a.SM = SM.p ? SM.as<double>() : nullptr;
    a.XO = XO.p ? XO.as<double>() : nullptr;
    a.part = part.as<double>();
    a.part_slices = S.Kc + S.W;
    a.part_off = S.Kc;
    a.theta = theta1.as<double>();
    a.per_img = S.W;
    a.first = first ? 1 : 0;
    a.prox = p.variant == CCSC_SOLVE_POISSON2D ? 1 : 0;
    a.mtm_sq = p.variant == CCSC_SOLVE_INPAINT2D ? 1 : 0;
    a.obj_sm = (p.variant == CCSC_SOLVE_MULTICH || p.variant == CCSC_SOLVE_VIDEO3D) ? 1 : 0;
    a.psnr_sm = p.variant == CCSC_SOLVE_INPAINT2D ? 1 : 0;
    // PSNR window: psnr_pad = psf_radius inside the cropped image (SI:59-60)
    a.px0 = 2 * S.rx;
    a.px1 = S.X - 2 * S.rx;
    a.py0 = 2 * S.ry;
    a.py1 = S.Y - 2 * S.ry;
    a.Y = S.Y;
    return a;
  }

  void solve_bins() {
    const ccsc_solve_problem& p = S.p;
    const double invP = 1.0 / (double)S.P;
    if (p.variant == CCSC_SOLVE_INPAINT2D || p.variant == CCSC_SOLVE_POISSON2D) {
      HIPCHK(launch_solve_sm<double>(Sz.as<cpx<double>>(), Sx.as<cpx<double>>(),
                                     dhat.as<cpx<double>>(), senergy.as<double>(), S.rho, invP,
                                     (int)S.F, S.Kc, n, p.variant == CCSC_SOLVE_POISSON2D ? 1 : 0,
                                     S.X, S.Y, S.X / 2 + 1, st));
    } else {
      // zhat_k = (sum_w conj(dhat_wk) xi1_w + rho xi2_k) * invP / (rho + s), then
      // v1_w = sum_k dhat_wk zhat_k: the per-bin GEMMs of hs23.hip (dhat [K][W][F])
      HIPCHK(launch_hs_analysis<double>(dhat.as<cpx<double>>(), Sx.as<cpx<double>>(),
                                        Sz.as<cpx<double>>(), senergy.as<double>(), S.rho,
                                        Sz.as<cpx<double>>(), (int)S.F, S.W, S.Kc, (int)n, st));
      HIPCHK(launch_hs_synth<double>(dhat.as<cpx<double>>(), Sz.as<cpx<double>>(),
                                     Sx.as<cpx<double>>(), (int)S.F, S.W, S.Kc, (int)n, st));
    }
  }

  void run(ccsc_solve_outputs* out, ccsc_solvelog* log) {
    const ccsc_solve_problem& p = S.p;
    const int max_it = p.max_it;
    const bool want_trace = p.verbose != CCSC_VERBOSE_NONE && log &&
                            (log->obj || log->psnr || log->diff);
    const bool need_sums = p.tol > 0 || want_trace;
    if (log && (log->obj || log->psnr || log->diff) && log->capacity < max_it + 1)
      throw Err(CCSC_E_INVALID, "solvelog capacity < max_it + 1");
    std::vector<int> iters((size_t)n, 0), act((size_t)n, 1);
    std::vector<double> hs((size_t)(n * kRowParts));
    const double nan = std::numeric_limits<double>::quiet_NaN();
    auto put = [&](double* arr, int64_t img, int it, double v) {
      if (arr && want_trace) arr[img * log->capacity + it] = v;
    };
    const double psnr_count = (double)(p.sb[0] - 2 * S.rx) * (double)(p.sb[1] - 2 * S.ry);
    const int64_t nz = n * S.Kc, nx = n * S.W;
    hipEvent_t e0, e1;
    HIPCHK(hipEventCreate(&e0));
    HIPCHK(hipEventCreate(&e1));
    HIPCHK(hipEventRecord(e0, st));
    int live = (int)n;
    for (int i = 0; i <= max_it && live > 0; ++i) {
      const bool last = i == max_it;
      HIPCHK(launch_rows_pair<double>(last ? kRowFinalZ : kRowIterZ, code_args(i == 0), nz,
                                      data_args(i == 0), nx, S.rg, tw(tw_r), st));
      if (need_sums) {
        HIPCHK(launch_reduce_parts<double>(part.as<double>(), sums.as<double>(), n, S.Kc + S.W,
                                           S.rg.groups, st));
        HIPCHK(hipMemcpyAsync(hs.data(), sums.p, sums.bytes, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        bool changed = false;
        for (int64_t m = 0; m < n; ++m) {
          if (!act[(size_t)m]) continue;
          const double* q = hs.data() + m * kRowParts;
          const double diff = i == 0 ? 0.0 : std::sqrt(q[0]) / std::sqrt(q[1]);   // SI:124
          iters[(size_t)m] = i;
          put(log ? log->diff : nullptr, m, i, diff);
          put(log ? log->obj : nullptr, m, i,
              p.lambda_residual * 0.5 * q[3] + p.lambda_prior * q[2]);          // SI:196-200
          if (log && log->psnr) {
            double ps = nan;
            if (XO.p) {
              const double mse = q[4] / psnr_count;                            // SI:61-66
              ps = mse > std::numeric_limits<double>::epsilon() ? 10.0 * std::log10(1.0 / mse)
                                                                : std::numeric_limits<double>::infinity();
            }
            put(log->psnr, m, i, ps);
          }
          if (i > 0 && p.tol > 0 && diff < p.tol) {                              // SI:136
            act[(size_t)m] = 0;
            --live;
            changed = true;
          }
        }
        if (changed)
          HIPCHK(hipMemcpyAsync(active.p, act.data(), active.bytes, hipMemcpyHostToDevice, st));
      } else {
        for (auto& it : iters) it = i;
      }
      if (last || live == 0) break;
      cols2(-1, nz, nx);
      solve_bins();
      cols2(+1, nz, nx);
    }
    HIPCHK(hipEventRecord(e1, st));
    HIPCHK(hipEventSynchronize(e1));
    float ms = 0;
    HIPCHK(hipEventElapsedTime(&ms, e0, e1));
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    if (log) {
      if (log->iters)
        for (int64_t m = 0; m < n; ++m) log->iters[m] = iters[(size_t)m];
      if (log->seconds) log->seconds[0] = ms * 1e-3;
    }
    // ---- outputs: z, and res = crop(real(ifft(sum_k dhat_k fft(z))) + smoothinit)
    if (out && out->z)
      HIPCHK(hipMemcpyAsync(out->z, Z.p, Z.bytes, hipMemcpyDeviceToHost, st));
    if (out && out->res) {
      fwd(Z.as<double>(), Sz.as<cpx<double>>(), nz);
      const cpx<double>* dres = dhat_res.p ? dhat_res.as<cpx<double>>() : dhat.as<cpx<double>>();
      HIPCHK(launch_hs_synth<double>(dres, Sz.as<cpx<double>>(), Sx.as<cpx<double>>(), (int)S.F,
                                     S.W, S.Kc, (int)n, st));
      cols(Sx.as<cpx<double>>(), +1, nx);
      RowArgs<double> a{};
      a.S = Sx.as<cpx<double>>();
      a.SM = SM.p ? SM.as<double>() : nullptr;
      a.per_img = S.W;
      a.Y = S.Y;
      a.sbx = (int)p.sb[0];
      a.sby = (int)p.sb[1];
      a.sbt = (int)p.sb[2];
      a.rx = S.rx;
      a.ry = S.ry;
      a.rt = S.rt;
      a.clamp0 = p.variant == CCSC_SOLVE_POISSON2D ? 1 : 0;   // SP:131
      a.scale = 1.0 / (double)S.P;
      DevBuf res;
      res.alloc((size_t)(nx * p.sb[0] * p.sb[1] * p.sb[2]) * 8);
      a.res = res.as<double>();
      HIPCHK(launch_rows<double>(kRowRes, a, nx, S.rg, tw(tw_r), st));
      HIPCHK(hipMemcpyAsync(out->res, res.p, res.bytes, hipMemcpyDeviceToHost, st));
      HIPCHK(hipStreamSynchronize(st));
    }
    HIPCHK(hipStreamSynchronize(st));
  }
};

}  // namespace ccsc

using namespace ccsc;

extern "C" {

int32_t ccsc_solve_supported(const ccsc_solve_problem* p, char* err, size_t errlen) {
  return guarded(err, errlen, [&] {
    if (!p) throw Err(CCSC_E_INVALID, "NULL problem");
    SolveSpec S;
    resolve_solve(*p, S);
  });
}

int32_t ccsc_solve(ccsc_ctx* ctx, const ccsc_solve_problem* p, const ccsc_solve_inputs* in,
                   ccsc_solve_outputs* out, ccsc_solvelog* log, char* err, size_t errlen) {
  return guarded(err, errlen, [&] {
    if (!ctx || !p || !in) throw Err(CCSC_E_INVALID, "NULL ctx/problem/inputs");
    if (!ctx->subs.empty())
      throw Err(CCSC_E_UNSUPPORTED, "the solvers run on a one-device context");
    HIPCHK(hipSetDevice(ctx->device));
    Solver s(ctx, *p);
    s.setup(*in);
    s.run(out, log);
  });
}

int32_t ccsc_local_cn_dev(ccsc_ctx* ctx, const double* in, double* out, int64_t n, int32_t H,
                          int32_t W, char* err, size_t errlen) {
  return guarded(err, errlen, [&] {
    if (!ctx || !in || !out || n < 0) throw Err(CCSC_E_INVALID, "bad arguments");
    if (!local_cn_ok(H, W))
      throw Err(CCSC_E_UNSUPPORTED, "local_cn: images must be 7x7 .. 12288 pixels and fit the LDS");
    HIPCHK(hipSetDevice(ctx->device));
    HIPCHK(launch_local_cn(in, out, n, H, W, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
  });
}

int32_t ccsc_local_cn(ccsc_ctx* ctx, const double* in, double* out, int64_t n, int32_t H,
                      int32_t W, char* err, size_t errlen) {
  return guarded(err, errlen, [&] {
    if (!ctx || !in || !out || n < 0) throw Err(CCSC_E_INVALID, "bad arguments");
    if (!local_cn_ok(H, W))
      throw Err(CCSC_E_UNSUPPORTED, "local_cn: images must be 7x7 .. 12288 pixels and fit the LDS");
    HIPCHK(hipSetDevice(ctx->device));
    const int64_t per = (int64_t)H * W;
    const int64_t chunk = std::max<int64_t>(1, std::min<int64_t>(n, (256LL << 20) / (per * 8)));
    DevBuf a, b;
    a.alloc((size_t)(chunk * per) * 8);
    b.alloc(a.bytes);
    for (int64_t i0 = 0; i0 < n; i0 += chunk) {
      const int64_t m = std::min(chunk, n - i0);
      HIPCHK(hipMemcpyAsync(a.p, in + i0 * per, (size_t)(m * per) * 8, hipMemcpyHostToDevice,
                            ctx->stream));
      HIPCHK(launch_local_cn(a.as<double>(), b.as<double>(), m, H, W, ctx->stream));
      HIPCHK(hipMemcpyAsync(out + i0 * per, b.p, (size_t)(m * per) * 8, hipMemcpyDeviceToHost,
                            ctx->stream));
    }
    HIPCHK(hipStreamSynchronize(ctx->stream));
  });
}

}  // extern "C"
