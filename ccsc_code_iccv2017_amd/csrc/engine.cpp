// libccsc host engine: problem resolution, memory plan, the outer ADMM
// schedule of the consensus learners, RCCL consensus, and the C-ABI.
//
// Schedule of one outer iteration (dP:89-190; dZ:90-194), per rank:
//   precompute  for each local block: R2C of its z slices -> Zh;
//               gram+cholesky -> L_f, h_f                       (dP:95-99)
//   d-loop      dual+R2C -> C ; dsolve -> Dhat ; C2R -> D, support(D+y)
//               -> local sum -> RCCL all-reduce -> projection u (dP:103-134)
//   z-prep      dhat = Dhat of global block 1 (RCCL broadcast), sden  (dP:143)
//   z-loop      fused z-iteration kernel over the local patches   (dP:147-168)
#include "../../include/ccsc.h"
#include "host.hpp"
#include "recon.hpp"

#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <mutex>
#include <thread>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <limits>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace ccsc {

// ---------------------------------------------------------------------------
// FFT planning (host)
// ---------------------------------------------------------------------------
static const int kRadices[] = {11, 10, 8, 7, 5, 4, 3, 2};  // fft_pass_dispatch

static bool is_native_radix(int R) {
  for (int r : kRadices)
    if (r == R) return true;
  return false;
}

// Fewest passes over the native (unrolled) radices; lengths they cannot factor take
// generic passes (fft_pass_generic: any odd prime length, one task of kGenericQP conjugate
// output pairs per thread, inputs streamed from LDS, roots from the twiddle table) for
// their other prime factors -- primes above 11 of any size (131 of a 262 grid) and several
// of them (13 x 17) -- after the native passes: fewest generic passes, then fewest passes
// (e.g. 74 = 2 * 37, the prime-factor pfa pass).  Register budget: a native pass holds
// n/R butterflies per line (<= kMaxButterflies), a generic pass one task per thread.
static int64_t generic_tasks(int n, int nlines, int p) {
  return (int64_t)nlines * (n / p) * (((p - 1) / 2 + kGenericQP - 1) / kGenericQP);
}

static bool is_prime(int p) {
  if (p < 2) return false;
  for (int d = 2; d * d <= p; ++d)
    if (p % d == 0) return false;
  return true;
}

static bool plan1d(int n, int nlines, Plan1D& out) {
  if (n == 1) {
    out = Plan1D{1, 0, {0}, {0}};
    return true;
  }
  constexpr int nrad = (int)(sizeof(kRadices) / sizeof(int));
  Plan1D best{};
  best.npass = 99;
  int best_ng = 99;
  std::vector<int> nat, gen;
  // natives in kRadices order from `start`, generic primes non-decreasing
  std::function<void(int, int, bool)> dfs = [&](int rem, int start, bool allow_gen) {
    const int np = (int)(nat.size() + gen.size()), ng = (int)gen.size();
    if (rem == 1) {
      if (ng < best_ng || (ng == best_ng && np < best.npass)) {
        best_ng = ng;
        best = Plan1D{};
        best.n = n;
        best.npass = np;
        for (int i = 0; i < (int)nat.size(); ++i) best.rad[i] = nat[i];
        for (int i = 0; i < ng; ++i) best.rad[nat.size() + i] = gen[i];
      }
      return;
    }
    if (np >= kMaxPass) return;
    if (ng > best_ng || (ng == best_ng && np + 1 >= best.npass)) return;
    for (int i = start; i < nrad; ++i) {
      const int R = kRadices[i];
      if (rem % R) continue;
      if ((int64_t)(n / R) * nlines > (int64_t)maxb_for_radix(R) * kNT) continue;  // registers
      nat.push_back(R);
      dfs(rem / R, i, allow_gen);
      nat.pop_back();
    }
    if (!allow_gen) return;
    for (int R = gen.empty() ? 13 : gen.back(); R <= rem; ++R) {
      if (rem % R || !is_prime(R)) continue;
      if (generic_tasks(n, nlines, R) > kNT) continue;
      gen.push_back(R);
      dfs(rem / R, start, true);
      gen.pop_back();
    }
  };
  dfs(n, 0, false);   // native radices only (every plan of earlier rounds stays as it was)
  if (best.npass == 99) dfs(n, 0, true);
  if (best.npass == 99) return false;
  // 2 * kPfaM: the prime-factor pass with immediate roots (fft_pass_pfa)
  best.pfa = (n == 2 * kPfaM && best.npass == 2 && best.rad[0] == 2 && best.rad[1] == kPfaM &&
              pfa_slots(nlines, kPfaM, kPfaQP) <= kNT);
  out = best;
  return true;
}

static bool make_grid2d(int X, int Y, Grid2D& G, std::string& why) {
  G.X = X;
  G.Y = Y;
  G.Xh = X / 2 + 1;
  // LDS row stride (units of T): >= 2*Xh, even (16-B complex alignment), and
  // 4*RS = 24 (mod 64) dwords so the column-pair lines of the x passes do not
  // alias onto the same LDS banks (measured: 6e9 conflict cycles per z-step
  // launch with RS = 2*Xh = 112).
  G.RS = 2 * G.Xh;
  while (G.RS % 16 != 6) G.RS += 2;
  G.Yp = Y + (Y & 1);
  G.F = G.Xh * Y;
  if (!plan1d(X, G.Yp / 2, G.px)) {
    why = "grid length " + std::to_string(X) +
          " has no radix plan within kMaxPass passes and the per-thread task budget";
    return false;
  }
  if (!plan1d(Y, G.Xh, G.py)) {
    why = "grid length " + std::to_string(Y) +
          " has no radix plan within kMaxPass passes and the per-thread task budget";
    return false;
  }
  // per-pass twiddle tables, x passes then y passes
  int off = 0;
  for (Plan1D* p : {&G.px, &G.py}) {
    int Ns = 1;
    for (int s = 0; s < p->npass; ++s) {
      p->twoff[s] = off;
      off += (p->rad[s] - 1) * Ns + (is_native_radix(p->rad[s]) ? 0 : p->rad[s]);
      Ns *= p->rad[s];
    }
  }
  G.ntw = std::max(off, 1);
  const size_t lds = fused_smem_bytes(G, sizeof(double), 3);
  if (lds > 160 * 1024) {
    why = "padded slice " + std::to_string(X) + "x" + std::to_string(Y) +
          " does not fit one CU's LDS in fp64";
    return false;
  }
  if (pick_nb(G.F) < 0) {
    why = "half spectrum too large for the register-resident z-solve";
    return false;
  }
  return true;
}

// Tile of the t-direction FFT of the 3D learner: Tn rows of Xh complex lines
// (plan in Gt.py; Gt.px unused).
static bool make_gridt(int Tn, int Xh, Grid2D& Gt, std::string& why) {
  Gt = Grid2D{};
  Gt.Y = Gt.Yp = Tn;
  Gt.Xh = Xh;
  Gt.RS = 2 * Xh;  // lanes run along x' (lines): 16-B consecutive, conflict-free
  Gt.F = Xh * Tn;
  Gt.px = Plan1D{1, 0, {0}, {0}};
  if (!plan1d(Tn, Xh, Gt.py)) {
    why = "grid length " + std::to_string(Tn) + " has no radix plan for the t-direction FFT";
    return false;
  }
  int off = 0, Ns = 1;
  for (int s = 0; s < Gt.py.npass; ++s) {
    Gt.py.twoff[s] = off;
    off += (Gt.py.rad[s] - 1) * Ns + (is_native_radix(Gt.py.rad[s]) ? 0 : Gt.py.rad[s]);
    Ns *= Gt.py.rad[s];
  }
  Gt.ntw = std::max(off, 1);
  if (tfft_smem_bytes(Gt, sizeof(double)) > 160 * 1024) {
    why = "t-direction tile does not fit one CU's LDS";
    return false;
  }
  return true;
}

static std::vector<cpx<double>> make_twiddles(const Grid2D& G) {
  std::vector<cpx<double>> t(G.ntw, cpx<double>{1.0, 0.0});
  const long double pi = 3.141592653589793238462643383279502884L;
  for (const Plan1D* p : {&G.px, &G.py}) {
    int Ns = 1;
    for (int s = 0; s < p->npass; ++s) {
      const int R = p->rad[s];
      for (int r = 1; r < R; ++r)
        for (int k = 0; k < Ns; ++k) {
          const long double a = -2.0L * pi * (long double)(r * k) / (long double)(Ns * R);
          t[p->twoff[s] + (r - 1) * Ns + k] = {(double)cosl(a), (double)sinl(a)};
        }
      if (!is_native_radix(R))
        for (int m = 0; m < R; ++m) {
          const long double a = -2.0L * pi * (long double)m / (long double)R;
          t[p->twoff[s] + (R - 1) * Ns + m] = {(double)cosl(a), (double)sinl(a)};
        }
      Ns *= R;
    }
  }
  return t;
}

// ---------------------------------------------------------------------------
// Problem resolution (Appendix A of SURVEY.md)
// ---------------------------------------------------------------------------
static void resolve_problem(ccsc_problem& p) {
  if (p.variant < CCSC_DPAR || p.variant > CCSC_HS23) throw Err(CCSC_E_INVALID, "unknown variant");
  const bool is3 = p.variant == CCSC_L3D;
  const bool isHS = p.variant == CCSC_HS23;
  const int want_ndim = is3 ? 3 : 2;
  if (p.ndim == 0) p.ndim = want_ndim;
  if (p.ndim != want_ndim) throw Err(CCSC_E_INVALID, "ndim does not match the variant");
  for (int i = 0; i < p.ndim; ++i)
    if (p.sb[i] <= 0) throw Err(CCSC_E_INVALID, "spatial size of b must be positive");
  if (isHS) {
    // W wavelengths = kernel_size(3) = size(b, 3) (L23:6-15); they play the role of views
    if (p.views[0] <= 0)
      throw Err(CCSC_E_INVALID, "2-3D learner needs the wavelength count W (kernel_size(3)) in views[0]");
    p.views[1] = 1;
    if (!(p.lambda_prior > 0))
      throw Err(CCSC_E_INVALID, "2-3D learner needs lambda_prior > 0 (gamma_heuristic = 60*lambda/max(b), L23:36)");
  } else if (p.variant != CCSC_L4D) {
    p.views[0] = p.views[1] = 1;
  } else if (p.views[0] <= 0 || p.views[1] <= 0 || p.views[0] != p.views[1]) {
    throw Err(CCSC_E_INVALID, "4D needs equal positive view counts U == V (L4:9-10, Q9)");
  }
  if (p.n <= 0) throw Err(CCSC_E_INVALID, "n must be positive");
  if (p.K <= 0) throw Err(CCSC_E_INVALID, "K must be positive");
  if (p.psf <= 0 || (p.psf & 1) == 0) throw Err(CCSC_E_INVALID, "psf size must be odd and positive");
  if (p.max_it < 0) throw Err(CCSC_E_INVALID, "max_it must be >= 0");
  // variant constants
  int ni = 100, mid = 10, miz = 10;
  double rd = 500, rz = 50, td = 50;
  switch (p.variant) {
    case CCSC_DPAR: break;                                     // dP:11,75-76,98,150,153
    case CCSC_DZPAR: mid = 5; rd = 5000; rz = 1; td = 1; break;  // dZ:75,99,151,154
    case CCSC_L3D:
    case CCSC_L4D: {
      const int64_t s = (int64_t)std::llround(std::sqrt((double)p.n));
      if (s * s != p.n)
        throw Err(CCSC_E_INVALID, "3D/4D learners need n to be a perfect square (ni = sqrt(n), L3:11)");
      ni = (int)s;
      if (p.variant == CCSC_L3D) { rd = 5000; rz = 1; td = 1; }  // L3:109,168,175
      break;                                                      // L4:105,159,162
    }
    case CCSC_HS23:
      // one non-consensus ADMM over all images; rho_D = gamma_D(2)/gamma_D(1) = 5000
      // (L23:37,93), rho_Z = W gamma_Z(2)/gamma_Z(1) = 500 W (L23:38,311); the prox
      // thresholds follow from gamma_heuristic at run time (engine: SessionHS)
      if (p.n > INT32_MAX) throw Err(CCSC_E_INVALID, "n too large");
      ni = (int)p.n;
      rd = 5000;
      rz = 500.0 * p.views[0];
      td = 1;
      break;
  }
  if (p.ni <= 0) p.ni = ni;
  if (p.max_it_d <= 0) p.max_it_d = mid;
  if (p.max_it_z <= 0) p.max_it_z = miz;
  if (!(p.rho_d > 0)) p.rho_d = rd;
  if (!(p.rho_z > 0)) p.rho_z = rz;
  if (!(p.theta_div > 0)) p.theta_div = td;
  if (p.n % p.ni != 0)
    throw Err(CCSC_E_INVALID, "n (" + std::to_string(p.n) + ") must be a multiple of ni (" +
                                  std::to_string(p.ni) + "); the reference floors n/ni silently (Q13)");
  if (p.verbose < CCSC_VERBOSE_NONE || p.verbose > CCSC_VERBOSE_ALL)
    throw Err(CCSC_E_INVALID, "bad verbose");
  if (p.precision == CCSC_FP32)
    throw Err(CCSC_E_UNSUPPORTED, "CCSC_FP32 was never built and is deprecated (ABI 7): use CCSC_FP64");
  if (p.precision != CCSC_FP64) throw Err(CCSC_E_INVALID, "precision must be CCSC_FP64 (double, as the reference)");
  if (p.dfactor < CCSC_DFACTOR_AUTO || p.dfactor > CCSC_DFACTOR_WOODBURY)
    throw Err(CCSC_E_INVALID, "bad dfactor");
  // AUTO resolves to the form the consensus learners will run (observable through
  // ccsc_resolve): the ni x ni Woodbury factor for blocks of few patches, else K x K
  if (p.variant != CCSC_HS23 && p.dfactor == CCSC_DFACTOR_AUTO)
    p.dfactor = (woodbury_fits(p.K, p.ni) || (p.K > 400 && wbig_ok(p.K, p.ni)))
                    ? CCSC_DFACTOR_WOODBURY
                    : CCSC_DFACTOR_CHOLESKY;
  const int r = p.psf / 2;
  for (int i = 0; i < p.ndim; ++i)
    if (p.sb[i] + 2 * r < p.psf) throw Err(CCSC_E_INVALID, "grid smaller than the filter");
}

// Transform geometry of one slice: the (x, y) plane grid and, for the 3D
// learner, the t-direction tile (Tn = 1 otherwise).
struct Geom {
  Grid2D G{};
  Grid2D Gt{};
  int Tn = 1;
  // 2D slices past one CU's LDS (or past the slice planner): transforms as the global
  // line passes of recon.hip, the elementwise stages in gslice.hip (G holds X, Y, Xh, F)
  bool gp = false;
  int64_t P() const { return (int64_t)G.X * G.Y * Tn; }   // voxels per slice
  int64_t F() const { return (int64_t)G.F * Tn; }         // half-spectrum bins per slice
};

// engine capability check (separate from validity: valid reference inputs we
// do not run yet return CCSC_E_UNSUPPORTED)
static void check_supported(const ccsc_problem& p, Geom* Gout) {
  // (right-hand sides past the Gram kernels' budget, K * views > 2048 or views > 16, are
  // formed by the per-bin GEMM of hs23.hip instead, Session2D::h_sep)
  if ((int64_t)p.K * p.views[0] * p.views[1] > (int64_t)1 << 20)
    throw Err(CCSC_E_UNSUPPORTED, "K * views > 2^20 filter slices");
  // K <= 192: the register-resident MFMA factor (gramchol.hip); 192 < K <= 400: the
  // HBM-resident Gram + left-looking Cholesky of gramchol_big.hip (consensus learners);
  // K > 400 (consensus) and K > 192 (2-3D): the reference's Woodbury form on the ni x ni
  // (n x n) factor (wbig.hip), for ni <= 100 and ni K + ni^2 <= K (K + 1) / 2
  if (p.K > 400 && p.variant != CCSC_HS23 &&
      !(p.dfactor == CCSC_DFACTOR_WOODBURY && wbig_ok(p.K, p.ni)))
    throw Err(CCSC_E_UNSUPPORTED, "K > 400 runs the Woodbury D-factor only, which needs ni <= 100 and "
                                  "ni K + ni^2 <= K (K + 1) / 2");
  if (p.K > 192 && p.variant == CCSC_HS23 && (p.n > INT32_MAX || !wbig_ok(p.K, (int)p.n)))
    throw Err(CCSC_E_UNSUPPORTED, "the 2-3D learner past K = 192 runs the n x n Woodbury factor "
                                  "(L23:290), which needs n <= 100 and n K + n^2 <= K (K + 1) / 2");
  if (p.dfactor == CCSC_DFACTOR_WOODBURY &&
      (p.variant == CCSC_HS23 || !(woodbury_ok(p.K, p.ni) || wbig_ok(p.K, p.ni))))
    throw Err(CCSC_E_UNSUPPORTED, "the Woodbury D-factor needs ni <= 100 and ni K + ni^2 <= K (K + 1) / 2 "
                                  "(consensus learners only)");
  const int r = p.psf / 2;
  Geom g;
  std::string why;
  const int X = (int)(p.sb[0] + 2 * r), Y = (int)(p.sb[1] + 2 * r);
  const bool is3 = p.variant == CCSC_L3D;
  const int Tn = is3 ? (int)(p.sb[2] + 2 * r) : 1;
  bool fits = make_grid2d(X, Y, g.G, why);
  // 3D: the plane kernels also need a t-tile plan (k_tfft / k_tsolve3 hold whole t-columns)
  if (fits && is3 && !make_gridt(Tn, g.G.Xh, g.Gt, why)) fits = false;
  if (!fits) {
    // every learner on any grid the reference accepts (dP:16,23-24; L3:16,23-26;
    // L23:12-26): slices past one CU's LDS (or 3D t-columns past the t-tile kernels) take
    // the global line passes
    const bool gp_ok = p.variant == CCSC_DPAR || p.variant == CCSC_DZPAR ||
                       p.variant == CCSC_L4D || is3 || p.variant == CCSC_HS23;
    RowGeom rg{};
    ColGeom cy{}, ct{};
    std::vector<cpx<double>> t1, t2, t3;
    if (!gp_ok) throw Err(CCSC_E_UNSUPPORTED, why);
    if (is3 ? !gfft_plan3(X, Y, Tn, rg, cy, ct, t1, t2, t3) : !gfft_plan(X, Y, rg, cy, t1, t2))
      throw Err(CCSC_E_UNSUPPORTED, why + "; no global line plan either");
    g.gp = true;
    g.G = Grid2D{};
    g.G.X = X;
    g.G.Y = Y;
    g.G.Xh = X / 2 + 1;
    g.G.Yp = Y + (Y & 1);
    g.G.F = g.G.Xh * Y;
    g.G.ntw = 1;   // (the slice twiddle table is unused)
    g.Gt = Grid2D{};
    if ((int64_t)g.G.F * 16 > INT32_MAX / 2) throw Err(CCSC_E_UNSUPPORTED, "2D half spectrum too large");
  }
  if (is3) {
    g.Tn = Tn;
    if (g.F() > INT32_MAX / 2 || g.P() > INT32_MAX / 2)
      throw Err(CCSC_E_UNSUPPORTED, "3D half spectrum too large");
  }
  if (Gout) *Gout = g;
}

// (the 2-3D learner has one block of all n images, L23: its shards are runs of images)
static void shard(const ccsc_problem& p, int rank, int nranks, int64_t& b0, int64_t& nb) {
  if (nranks <= 0 || rank < 0 || rank >= nranks) throw Err(CCSC_E_INVALID, "bad rank/nranks");
  const int64_t N = p.variant == CCSC_HS23 ? p.n : p.n / p.ni;
  if (N < nranks) throw Err(CCSC_E_INVALID, "fewer blocks than ranks");
  const int64_t base = N / nranks, rem = N % nranks;
  nb = base + (rank < rem ? 1 : 0);
  b0 = rank * base + std::min<int64_t>(rank, rem);
}

}  // namespace ccsc

using namespace ccsc;


namespace ccsc {

// the register-line z-step serves the 110 grid (k_zsplit every other 2D grid)
static bool zline_usable(const Grid2D& G) { return zline_grid(G); }

// memory plan shared by ccsc_plan_bytes and the session
struct Plan2D {
  int64_t np, nbl, b0;
  size_t z, yz, cbuf, W, dhw, D, yD, Bhat, b, L, h, Ch, Dh, Zh, E, zl, big, misc, gr, cg;
  size_t total() const {
    return z + yz + cbuf + W + dhw + D + yD + Bhat + b + L + h + Ch + Dh + Zh + E + zl + big + misc +
           gr + cg;
  }
};

static Plan2D plan2d(const ccsc_problem& p, const Geom& g, int rank, int nranks) {
  Plan2D m{};
  shard(p, rank, nranks, m.b0, m.nbl);
  m.np = m.nbl * p.ni;
  const Grid2D& G = g.G;
  const size_t P = g.P(), F = g.F(), K = p.K;
  const size_t NV = (size_t)p.views[0] * p.views[1];
  const size_t Kp = K * (K + 1) / 2;
  const size_t s = p.psf;
  const size_t SS = s * s * (g.Tn > 1 ? s : 1);   // filter support (2r+1)^ndim
  const bool is4 = p.variant == CCSC_L4D, is3 = p.variant == CCSC_L3D;
  m.z = m.np * K * P * 8;
  m.yz = m.z;
  // 2D split z-state (zsplit.hip): w per patch + the filter spectrum it was
  // solved with; with tol > 0 a u buffer so z_old survives for the tol test
  // (the 4D and 3D z-steps compare per slice/plane; the register-line z-step of
  // the 110 grid keeps z_old in the y buffer, zline.hip)
  const bool gp = g.gp;
  const bool zline = !is4 && !is3 && !gp && zline_usable(G);
  m.cbuf = (p.tol > 0 && !is4 && !is3 && !gp && !zline) ? m.z : 0;
  m.W = (!is4 && !is3 && !gp) ? m.np * F * 16 : 0;
  m.dhw = (!is4 && !is3 && !gp) ? K * F * 16 : 0;
  // global-pass 2D slices: a real scratch of the largest transform batch (the z-step's
  // np K slices, the D-step's nbl K, the precompute's ni K), the z-step spectra (E)
  m.gr = gp ? (size_t)std::max<int64_t>({m.np * (int64_t)K, m.nbl * (int64_t)(K * NV),
                                         (int64_t)(p.ni * K), m.np * (int64_t)NV}) * P * 8
             : 0;
  m.D = m.nbl * K * NV * P * 8;
  m.yD = m.D;
  m.Bhat = m.np * NV * F * 16;
  m.b = m.np * NV * (size_t)p.sb[0] * p.sb[1] * (is3 ? (size_t)p.sb[2] : 1) * 8;
  m.L = m.nbl * F * Kp * 16;
  m.h = m.nbl * F * NV * K * 16;
  m.Ch = m.nbl * K * NV * F * 16;
  m.Dh = m.Ch;
  m.Zh = (size_t)p.ni * K * F * 16;
  // K > 192 (gramchol_big.hip): the block's code spectra transposed frequency-major
  // (and the Woodbury form past k_gram_wb's ni <= 8, wbig.hip: the same frequency-major slabs)
  m.big = ((K > 192 && p.dfactor != CCSC_DFACTOR_WOODBURY) ||
           (p.dfactor == CCSC_DFACTOR_WOODBURY && !woodbury_ok((int)K, p.ni)))
              ? m.Zh
              : 0;
  // 4D: view correlations E; 3D: spectra of the z-step's plane/t transforms, in the
  // t-minor tile order when k_tsolve3 runs (padded to whole tiles: sized for TC = 4),
  // with B^, the filter spectrum and sden in that order (misc)
  const size_t F3t = is3 && !gp ? (size_t)std::max<int64_t>(ttile_bins(g.Tn, G.Y, G.Xh, 4),
                                                     ttile_bins(g.Tn, G.Y, G.Xh, 2))
                         : 0;
  m.E = is4 || gp ? m.np * K * F * 16 : is3 ? m.np * K * std::max(F, F3t) * 16 : 0;
  // 4D on global-pass slices: E keeps the view correlations, the z-step spectra go to cg
  m.cg = is4 && gp ? m.np * K * F * 16 : 0;
  // register-line z-step (zline.hip, 110 grid): B^ and the two filter spectra in
  // bin-slot order, sden in bin-slot order
  m.zl = zline ? m.np * F * 16 + 2 * K * F * 16 + F * 8 : 0;
  // + the second precompute workspace (the R2C of block j+1 beside the Gram of block j)
  if (zline) m.zl += m.Zh;
  m.misc = (2 * K * NV * F) * 16 + F * 8 + (m.nbl + 2) * K * NV * SS * 8 * 2 +
           (4 * m.np * NV * g.Tn + 4 * K * NV * g.Tn + 64) * 8 + (size_t)(G.ntw + g.Gt.ntw) * 16 +
           (is3 ? F * 16 + P * 8 + (m.np + K) * F3t * 16 + F3t * 8 : 0) +
           (gp ? NV * (F * 16 + P * 8) + 64 * 1024 : 0);   // objective scratch, line twiddles
  return m;
}

static const char* kKernelNames[5] = {"zstep", "gram_chol", "dsolve", "dual_r2c", "c2r_dout"};

// Wait for a non-blocking communicator's pending call (ncclInProgress); with `abort`,
// give up as soon as the group aborted (the enqueue may be waiting on a failed rank).
static void wait_comm(ncclComm_t c, const std::atomic<bool>* abort) {
  ncclResult_t st = ncclInProgress;
  for (;;) {
    NCCLCHK(ncclCommGetAsyncError(c, &st));
    if (st != ncclInProgress) break;
    if (abort && abort->load())
      throw Err(CCSC_E_RCCL, "host communicator aborted: another rank of this context failed");
    std::this_thread::yield();
  }
  if (st != ncclSuccess)
    throw Err(CCSC_E_RCCL, std::string("RCCL communicator error: ") + ncclGetErrorString(st));
}

// The communicators of a device-list context (rank i on devices[i]), created
// non-blocking so that no collective call can stall inside RCCL: abort_group relies on
// it to abort them only while no rank is inside a call.
static void init_group_comms(std::vector<ncclComm_t>& comms, const int32_t* devices, int nd) {
  // NCCL_COMM_BLOCKING=1 overrides cfg.blocking = 0 per communicator: a surviving rank could
  // then block inside a collective waiting on a failed one and abort_group would wait on it
  // forever -- refuse it instead of deadlocking later
  if (const char* b = std::getenv("NCCL_COMM_BLOCKING"))
    if (std::atoi(b) != 0)
      throw Err(CCSC_E_INVALID,
                "NCCL_COMM_BLOCKING=1 is not supported for multi-device contexts: their RCCL "
                "communicators must be non-blocking so a failed rank can be aborted");
  ncclUniqueId id;
  NCCLCHK(ncclGetUniqueId(&id));
  ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
  cfg.blocking = 0;
  auto ok = [](ncclResult_t r) { return r == ncclSuccess || r == ncclInProgress; };
  if (!ok(ncclGroupStart())) throw Err(CCSC_E_RCCL, "ncclGroupStart failed");
  for (int i = 0; i < nd; ++i) {
    HIPCHK(hipSetDevice(devices[i]));
    const ncclResult_t r = ncclCommInitRankConfig(&comms[i], nd, id, i, &cfg);
    if (!ok(r)) {
      ncclGroupEnd();
      throw Err(CCSC_E_RCCL, std::string("ncclCommInitRankConfig failed: ") + ncclGetErrorString(r));
    }
  }
  const ncclResult_t r = ncclGroupEnd();
  if (!ok(r)) throw Err(CCSC_E_RCCL, std::string("ncclGroupEnd failed: ") + ncclGetErrorString(r));
  for (int i = 0; i < nd; ++i) wait_comm(comms[i], nullptr);
}

// ---------------------------------------------------------------------------
// Session: 2D consensus learners (dP / dZ)
// ---------------------------------------------------------------------------
// ---- collectives of a rank context ------------------------------------------
// The transport is chosen by what the context was created with (a host callback or
// an RCCL communicator), never by a communicator pointer an abort may have cleared;
// in a multi-device group every collective first checks that no rank has failed.
static void host_exchange(ccsc_ctx* ctx, hipStream_t st, int op, double* buf, size_t count) {
  ctx->stage.resize(count);
  HIPCHK(hipMemcpyAsync(ctx->stage.data(), buf, count * 8, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  if (ctx->hostfn(ctx->hostuser, op, ctx->stage.data(), (int64_t)count) != 0)
    throw Err(CCSC_E_RCCL, "host communicator callback failed");
  HIPCHK(hipMemcpyAsync(buf, ctx->stage.data(), count * 8, hipMemcpyHostToDevice, st));
  HIPCHK(hipStreamSynchronize(st));
}
static void ctx_collective(ccsc_ctx* ctx, hipStream_t st, int op, double* buf, size_t count) {
  if (ctx->nranks <= 1 && !ctx->rccl_self) return;
  if (ctx->hostfn) {   // the exchange itself returns an error once the group aborted
    host_exchange(ctx, st, op, buf, count);
    return;
  }
  CommGroup* g = ctx->grp.get();
  if (g) g->inflight.fetch_add(1);
  struct Leave {
    CommGroup* g;
    ~Leave() {
      if (g) g->inflight.fetch_sub(1);
    }
  } leave{g};
  if (g && g->aborted.load())
    throw Err(CCSC_E_RCCL, "host communicator aborted: another rank of this context failed");
  if (!ctx->comm) throw Err(CCSC_E_STATE, "multi-rank context without a communicator");
  const ncclResult_t r = op == CCSC_COMM_ALLREDUCE_SUM
                             ? ncclAllReduce(buf, buf, count, ncclDouble, ncclSum, ctx->comm, st)
                             : ncclBroadcast(buf, buf, count, ncclDouble, 0, ctx->comm, st);
  // a device-list group's communicators are non-blocking (init_group_comms): the enqueue
  // may still be connecting; wait for it here, giving up once the group aborted, so no
  // rank stays inside RCCL on a communicator abort_group is about to abort
  if (r == ncclInProgress) wait_comm(ctx->comm, g ? &g->aborted : nullptr);
  else if (r != ncclSuccess)
    throw Err(CCSC_E_RCCL, std::string("RCCL collective failed: ") + ncclGetErrorString(r));
}

// Session of every consensus learner: dP, dZ, the 4D light-field learner (2D
// spatial convolution, NV = U*V views share the codes, L4:18-21) and the 3D
// learner (Tn > 1: plane transforms + t-direction FFT, L3).
struct Session2D {
  ccsc_ctx* ctx;
  ccsc_problem p;
  Geom g;
  Grid2D G;     // plane grid (g.G)
  Plan2D m;
  int r, s, K, ni, P, F, Kp;   // P, F: voxels / half-spectrum bins per slice (all dims)
  int SS;       // filter support size (2r+1)^ndim
  int Tn;       // 3D: t extent of the padded grid (1 otherwise)
  int NV, KG;   // views, filter slices per block (K * NV)
  bool is4, is3;
  bool woodbury;   // D-factor in Woodbury form (p.dfactor; AUTO: woodbury_fits, ni << K)
  bool wbig = false;   // ... past k_gram_wb's ni <= 8 (wbig.hip; K > 400 resolves to it)
  bool gram_mf;    // Gram + Cholesky on the matrix cores (gramchol.hip; else the VALU form)
  bool dtile = false;   // tile d-solve on a factor with inverted diagonal tiles (dstep.hip)
  bool gram_big = false;   // K > 192: HBM-resident Gram + Cholesky (gramchol_big.hip), X its workspace
  // right-hand sides h = A^H b past what the Gram kernels hold (K NV > 2048 or NV > 16 for
  // gramchol.hip, K NV > 8192 for gramchol_big.hip): the Gram runs with NV = 0 and the
  // per-bin GEMM of hs23.hip forms h (its Zh^H Xi, L23:289-295), same [F][NV][K] layout
  bool h_sep = false;
  bool wb_stage = true;    // CCSC_WB_STAGE (A/B: 0 keeps k_dsolve_wbv), read once per session
  DevBuf Xbig;
  // the diagonal-tile inversion of block j runs on st2 beside block j+1's precompute R2C
  hipStream_t st2 = nullptr;
  hipEvent_t ev_g = nullptr, ev_i = nullptr;
  // 110 grid: block j+1's precompute R2C (k_zhat_line, into the other of Zh / Zh2) runs on
  // st3 beside block j's Gram/Cholesky, filling that kernel's last partial round
  hipStream_t st3 = nullptr;
  hipEvent_t ev_s = nullptr, ev_z = nullptr, ev_gz[2] = {nullptr, nullptr};
  // 110 grid, tol = 0, >= 512 patches: a z-phase's launches split over two streams (patches [0, np/2) on st,
  // the rest on st3, idle during the z-phase), so each stream's next launch starts as soon as
  // its own half is done and fills the other's partial last round of workgroups (a C2 launch
  // is 39.06 rounds of one workgroup per CU); the halves couple only at the phase ends
  bool zsplit_open = false;
  hipEvent_t zsp_a = nullptr;
  int zsp_n = 0;
  DevBuf Zh2;
  int64_t N, nbl, b0, np;
  bool owner0;
  double theta;
  hipStream_t st;

  DevBuf tw, bdev, Bhat, z, yz, cbuf, D, yD, Usup, ssum, supp, Ch, Dh, L, h, Zh, dhat, dtmp, sden,
      dnorm, znorm, part, pair, E;
  // 2D z-phase state (zsplit.hip): zmode 0 = (z, y) materialised in `z`, `yz`;
  // zmode 1 = `z` holds the pre-threshold state a = z + y, W the last w and `dw`
  // the filter spectrum w was solved with (dhat, or dhatw after the next z-prep
  // replaced dhat); `yz` is then stale until materialize_z().
  DevBuf W, dhatw;
  int zmode = 0;
  const cpx<double>* dw = nullptr;
  // zmode 2 = register-line z-step (zline.hip, the 110 grid with tol = 0): `z` holds a
  // in state order, W the last w in bin-slot order solved with dws (dhs or dhws);
  // Bhs / dhs / sdens: B^, the current filter spectrum and sden in bin-slot order.
  bool zl_on = false;
  DevBuf Bhs, dhs, dhws, sdens;
  const cpx<double>* dws = nullptr;
  // tol > 0 with the register-line z-step: what `yz` holds (state order) while the
  // state is in zmode 2 -- ZT_PREV: the z of the iterate before the current one
  // (the next launch measures the current iterate against it), ZT_CUR: the
  // current iterate's z (its test is done), ZT_NONE: nothing (y, or stale).
  enum { ZT_NONE, ZT_PREV, ZT_CUR };
  int zt = ZT_NONE;
  DevBuf twt, oacc, odz;   // 3D: t-FFT twiddles, objective scratch (also the global path's)
  // 2D slices past one CU's LDS (Geom::gp): global line passes (recon.hip), their
  // twiddles, and the real scratch the elementwise stages (gslice.hip) read and write
  bool gp = false;
  RowGeom grg{};
  ColGeom gcy{}, gct{};   // gct: the 3D learner's t-lines
  DevBuf gtwr, gtwc, gtwt, gR, Cg;
  int tsolve_tc = 0;       // 3D: x' columns per k_tsolve3 workgroup (0: three-kernel z-solve)
  Grid2D gt2{};            //     its t plan (K * tsolve_tc lines) and twiddles
  DevBuf twt2;
  DevBuf BhatT, dhatT, sdenT;   // B^, the filter spectrum, sden in k_tsolve3's tile order
  int tsolve_ppw = 16;          // patches per k_tsolve3 workgroup
  bool c_ready = false;         // 3D: the z-step spectrum C already holds the next forward

  // host-side log
  int outer_done = 0;
  bool finished = false;
  double last_d = std::numeric_limits<double>::infinity();
  double last_z = std::numeric_limits<double>::infinity();
  double obj_filter = std::numeric_limits<double>::quiet_NaN();
  double obj_z = std::numeric_limits<double>::quiet_NaN();
  std::vector<double> v_obj_d, v_obj_z, v_tim, tr_od, tr_oz, tr_dd, tr_zd;
  std::vector<int32_t> v_nd, v_nz;

  // profiling
  bool prof = false;
  struct Rec { int id; hipEvent_t a, b; int n = 1; };   // n launches between a and b
  std::vector<Rec> recs;
  std::vector<hipEvent_t> pool;
  int64_t k_launch[5] = {0, 0, 0, 0, 0};
  double k_ms[5] = {0, 0, 0, 0, 0};

  hipEvent_t get_event() {
    if (!pool.empty()) {
      hipEvent_t e = pool.back();
      pool.pop_back();
      return e;
    }
    hipEvent_t e;
    HIPCHK(hipEventCreate(&e));
    return e;
  }
  template <typename Fn>
  void timed(int id, Fn&& fn) {
    if (!prof) {
      fn();
      return;
    }
    Rec rc{id, get_event(), get_event()};
    HIPCHK(hipEventRecord(rc.a, st));
    fn();
    HIPCHK(hipEventRecord(rc.b, st));
    recs.push_back(rc);
  }
  void drain_records() {
    for (auto& rc : recs) {
      float ms = 0;
      HIPCHK(hipEventSynchronize(rc.b));
      HIPCHK(hipEventElapsedTime(&ms, rc.a, rc.b));
      k_launch[rc.id] += rc.n;
      k_ms[rc.id] += ms;
      pool.push_back(rc.a);
      pool.push_back(rc.b);
    }
    recs.clear();
  }

  ~Session2D() {
    if (st) hipStreamSynchronize(st);
    if (st2) {
      hipStreamSynchronize(st2);
      hipStreamDestroy(st2);
    }
    if (ev_g) hipEventDestroy(ev_g);
    if (ev_i) hipEventDestroy(ev_i);
    if (st3) {
      hipStreamSynchronize(st3);
      hipStreamDestroy(st3);
    }
    for (hipEvent_t e : {ev_s, ev_z, ev_gz[0], ev_gz[1]})
      if (e) hipEventDestroy(e);
    for (auto& rc : recs) {
      hipEventDestroy(rc.a);
      hipEventDestroy(rc.b);
    }
    for (auto e : pool) hipEventDestroy(e);
  }

  bool verbose_refresh_d() const {
    if (p.variant == CCSC_DPAR) return p.verbose == CCSC_VERBOSE_BRIEF;  // dP:126
    if (p.variant == CCSC_L4D) return p.verbose == CCSC_VERBOSE_ALL;     // L4:135
    if (p.variant == CCSC_L3D) return p.verbose == CCSC_VERBOSE_ALL;     // L3:145
    return p.verbose != CCSC_VERBOSE_NONE;                               // dZ:127
  }
  bool verbose_refresh_z() const {
    if (p.variant == CCSC_DPAR) return p.verbose == CCSC_VERBOSE_BRIEF;  // dP:161
    if (p.variant == CCSC_L4D) return p.verbose == CCSC_VERBOSE_ALL;     // L4:170
    if (p.variant == CCSC_L3D) return p.verbose == CCSC_VERBOSE_ALL;     // L3:185
    return p.verbose != CCSC_VERBOSE_NONE;                               // dZ:165
  }

  Session2D(ccsc_ctx* c, const ccsc_problem& pin, const double* b, const double* d0,
            const double* z0)
      : ctx(c), p(pin), st(c->stream) {
    resolve_problem(p);
    check_supported(p, &g);
    G = g.G;
    m = plan2d(p, g, ctx->rank, ctx->nranks);
    r = p.psf / 2;
    s = p.psf;
    K = p.K;
    ni = p.ni;
    Tn = g.Tn;
    P = (int)g.P();
    F = (int)g.F();
    SS = s * s * (Tn > 1 ? s : 1);
    Kp = K * (K + 1) / 2;
    woodbury = p.dfactor == CCSC_DFACTOR_WOODBURY ||
               (p.dfactor == CCSC_DFACTOR_AUTO && woodbury_fits(K, ni));
    wbig = woodbury && !woodbury_ok(K, ni);
    NV = p.views[0] * p.views[1];
    KG = K * NV;
    {
      const char* ew = std::getenv("CCSC_WB_STAGE");
      wb_stage = !(ew && ew[0] == '0');
      h_sep = !woodbury && (K > 192 ? !gram_big_ok(K, NV) : !gram_chol_mf_ok(K, NV));
      const int NVg = h_sep ? 0 : NV;
      gram_mf = gram_chol_mf_ok(K, NVg);
      gram_big = !woodbury && K > 192 && gram_big_ok(K, NVg);
      // tile d-solve (one read of the factor per solve) on the MFMA factor with inverted
      // diagonal tiles; CCSC_DS_TILE=0 keeps the two-sweep k_dsolve
      const char* et = std::getenv("CCSC_DS_TILE");
      dtile = gram_mf && !woodbury && dsolve_tile_ok(K, NV) && !(et && et[0] == '0');
      if (dtile) {
        HIPCHK(hipStreamCreateWithFlags(&st2, hipStreamNonBlocking));
        HIPCHK(hipEventCreateWithFlags(&ev_g, hipEventDisableTiming));
        HIPCHK(hipEventCreateWithFlags(&ev_i, hipEventDisableTiming));
      }
    }
    is4 = p.variant == CCSC_L4D;
    is3 = p.variant == CCSC_L3D;
    gp = g.gp;
    N = p.n / ni;
    nbl = m.nbl;
    b0 = m.b0;
    np = m.np;
    owner0 = (b0 == 0);
    theta = p.lambda_prior / p.theta_div;
    if (!b) throw Err(CCSC_E_INVALID, "b must not be NULL");

    size_t freeb = 0, totalb = 0;
    HIPCHK(hipMemGetInfo(&freeb, &totalb));
    if (m.total() > freeb)
      throw Err(CCSC_E_NOMEM, "device plan needs " + std::to_string(m.total() >> 20) +
                                  " MiB, " + std::to_string(freeb >> 20) + " MiB free" +
                                  (p.tol > 0 ? " (tol > 0 adds a z-sized buffer)" : ""));
    auto tws = make_twiddles(G);
    tw.alloc(tws.size() * sizeof(cpx<double>));
    HIPCHK(hipMemcpy(tw.p, tws.data(), tw.bytes, hipMemcpyHostToDevice));
    if (is3 && !gp) {
      auto twts = make_twiddles(g.Gt);
      twt.alloc(twts.size() * sizeof(cpx<double>));
      HIPCHK(hipMemcpy(twt.p, twts.data(), twt.bytes, hipMemcpyHostToDevice));
      oacc.alloc((size_t)F * 16);
      odz.alloc((size_t)P * 8);
      // fused t-FFT + z-solve (k_tsolve3): TC x' columns per workgroup; C4 (74x74x42,
      // K = 49) measured 0.432 s per outer iteration at TC = 2, 0.456 at TC = 4 and with
      // the three-kernel form, 0.587 at TC = 1; the three-kernel form serves what k_tsolve3
      // cannot hold
      {
        std::string why2;
        // (C4 itself runs TC = 1 on narrow workgroups when kernels3d.hip builds that form:
        // two workgroups per CU, tsolve3_nt)
        const bool narrow = tsolve3_nt(Tn, K, 1) != kNT;
        for (int tc : narrow ? std::initializer_list<int>{1, 2, 4} : std::initializer_list<int>{2, 4, 1}) {
          Grid2D Gt2{};
          if (!tsolve3_ok(Tn, K, tc) || !make_gridt(Tn, K * tc, Gt2, why2)) continue;
          if (tsolve3_smem_bytes(Gt2, K, tc, sizeof(double)) > 160 * 1024) continue;
          tsolve_tc = tc;
          gt2 = Gt2;
          auto t2 = make_twiddles(gt2);
          twt2.alloc(t2.size() * sizeof(cpx<double>));
          HIPCHK(hipMemcpy(twt2.p, t2.data(), twt2.bytes, hipMemcpyHostToDevice));
          break;
        }
      }
    }
    if (gp) {
      std::vector<cpx<double>> t1, t2, t3;
      if (is3 ? !gfft_plan3(G.X, G.Y, Tn, grg, gcy, gct, t1, t2, t3)
              : !gfft_plan(G.X, G.Y, grg, gcy, t1, t2))
        throw Err(CCSC_E_UNSUPPORTED, "no global line plan");
      gtwr.alloc(t1.size() * sizeof(cpx<double>));
      gtwc.alloc(t2.size() * sizeof(cpx<double>));
      HIPCHK(hipMemcpy(gtwr.p, t1.data(), gtwr.bytes, hipMemcpyHostToDevice));
      HIPCHK(hipMemcpy(gtwc.p, t2.data(), gtwc.bytes, hipMemcpyHostToDevice));
      if (is3) {
        gtwt.alloc(std::max<size_t>(t3.size(), 1) * sizeof(cpx<double>));
        HIPCHK(hipMemcpy(gtwt.p, t3.data(), t3.size() * sizeof(cpx<double>), hipMemcpyHostToDevice));
      }
      gR.alloc(m.gr);
      oacc.alloc((size_t)NV * F * 16);
      odz.alloc((size_t)NV * P * 8);
      if (m.cg) Cg.alloc(m.cg);
    }
    const size_t KP = (size_t)K * P;
    bdev.alloc(m.b);
    Bhat.alloc(m.Bhat);
    z.alloc(m.z);
    yz.alloc(m.yz);
    if (m.cbuf) cbuf.alloc(m.cbuf);
    if (m.W) W.alloc(m.W);
    if (m.dhw) dhatw.alloc(m.dhw);
    zl_on = m.zl != 0;
    if (zl_on) {
      Zh2.alloc(m.Zh);
      HIPCHK(hipStreamCreateWithFlags(&st3, hipStreamNonBlocking));
      for (hipEvent_t* e : {&ev_s, &ev_z, &ev_gz[0], &ev_gz[1]})
        HIPCHK(hipEventCreateWithFlags(e, hipEventDisableTiming));
      Bhs.alloc((size_t)np * F * 16);
      dhs.alloc((size_t)K * F * 16);
      dhws.alloc((size_t)K * F * 16);
      sdens.alloc((size_t)F * 8);
    }
    D.alloc(m.D);
    yD.alloc(m.yD);
    Usup.alloc((size_t)KG * SS * 8);
    ssum.alloc((size_t)KG * SS * 8);
    supp.alloc((size_t)nbl * KG * SS * 8);
    Ch.alloc(m.Ch);
    Dh.alloc(m.Dh);
    L.alloc(m.L);
    h.alloc(m.h);
    Zh.alloc(m.Zh);
    if (gram_big || wbig) Xbig.alloc(m.big);
    dhat.alloc((size_t)KG * F * 16);
    dtmp.alloc((size_t)KG * F * 16);
    sden.alloc((size_t)F * 8);
    dnorm.alloc((size_t)2 * KG * Tn * 8);
    znorm.alloc((size_t)2 * std::max<int64_t>(np * K * Tn, 1) * 8);
    part.alloc((size_t)2 * std::max<int64_t>(np * NV, 1) * 8);
    pair.alloc(4 * 8);
    if (m.E) E.alloc(m.E);

    // data: b (rank-local, [sbx, sby(, sbt), np] column-major) and its padded spectrum
    HIPCHK(hipMemcpy(bdev.p, b, m.b, hipMemcpyHostToDevice));
    fwd_embed(bdev.as<double>(), (int)p.sb[0], (int)p.sb[1], is3 ? (int)p.sb[2] : 1, r,
              Bhat.as<cpx<double>>(), np * NV);
    if (zl_on)
      HIPCHK(launch_to_slots<double>(Bhat.as<cpx<double>>(), Bhs.as<cpx<double>>(), np, st));
    if (tsolve_tc) {
      const size_t F3t = (size_t)ttile_bins(Tn, G.Y, G.Xh, tsolve_tc);
      BhatT.alloc((size_t)np * F3t * 16);
      dhatT.alloc((size_t)K * F3t * 16);
      sdenT.alloc(F3t * 8);
      HIPCHK(launch_to_ttiles<double>(Bhat.as<cpx<double>>(), BhatT.as<cpx<double>>(), Tn, G.Y,
                                      G.Xh, tsolve_tc, np, st));
    }
    // filters: init.d or device RNG (dP:38-39; 4D: [psf,psf,U,V,K], L4:39-40; 3D: psf^3, L3:39-40)
    DevBuf d0dev;
    const size_t nd0 = (size_t)SS * KG;
    d0dev.alloc(nd0 * 8);
    if (d0) HIPCHK(hipMemcpy(d0dev.p, d0, nd0 * 8, hipMemcpyHostToDevice));
    else HIPCHK(launch_randn<double>(d0dev.as<double>(), (int64_t)nd0, p.seed ^ 0xd0d0d0d0ULL, 0, st));
    HIPCHK(launch_embed_filters<double>(d0dev.as<double>(), D.as<double>(), (int)nbl, KG, s, G, Tn,
                                        st));
    HIPCHK(hipMemsetAsync(yD.p, 0, m.yD, st));
    HIPCHK(hipMemsetAsync(Usup.p, 0, Usup.bytes, st));  // u = Pi(0) = 0 (Q2)
    HIPCHK(hipMemsetAsync(yz.p, 0, m.yz, st));
    // codes: init.z or device RNG (dP:45; dZ:44-47 replicates one z0 per block)
    if (p.variant == CCSC_DZPAR) {
      const size_t nz0 = (size_t)ni * KP;
      if (z0) HIPCHK(hipMemcpy(z.p, z0, nz0 * 8, hipMemcpyHostToDevice));
      else HIPCHK(launch_randn<double>(z.as<double>(), (int64_t)nz0, p.seed, 0, st));
      if (nbl > 1)
        HIPCHK(launch_replicate<double>(z.as<double>(), z.as<double>() + nz0, (int64_t)nz0,
                                        (int)nbl - 1, st));
    } else {
      if (z0) HIPCHK(hipMemcpy(z.p, z0, m.z, hipMemcpyHostToDevice));
      else
        HIPCHK(launch_randn<double>(z.as<double>(), (int64_t)(np * KP), p.seed,
                                    (uint64_t)(b0 * ni) * KP, st));
    }
    // 3D / 4D / global-pass 2D: `yz` holds the z-step state a = z + y (kernels3d.hip,
    // zstep.hip, gslice.hip), y = 0
    if (is4 || is3 || gp) HIPCHK(hipMemcpyAsync(yz.p, z.p, m.z, hipMemcpyDeviceToDevice, st));
    // dhat = fft2(d) of the initial filters (all blocks share d0, dP:41-42)
    fwd_embed(D.as<double>(), G.X, G.Y, Tn, 0, dhat.as<cpx<double>>(), KG);
    HIPCHK(hipStreamSynchronize(st));

    v_obj_d.push_back(std::numeric_limits<double>::quiet_NaN());
    v_obj_z.push_back(std::numeric_limits<double>::quiet_NaN());
    v_tim.push_back(0.0);
    if (p.verbose != CCSC_VERBOSE_NONE || p.trace_objective) {
      const double o = objective(dhat.as<cpx<double>>(), nullptr);  // dP:56
      obj_filter = obj_z = o;
      v_obj_d[0] = o;
      v_obj_z[0] = o;
    }
  }

  // ---- collectives (ctx_collective) -------------------------------------------
  void allreduce(double* buf, size_t count) { ctx_collective(ctx, st, CCSC_COMM_ALLREDUCE_SUM, buf, count); }
  void bcast0(double* buf, size_t count) { ctx_collective(ctx, st, CCSC_COMM_BCAST0, buf, count); }
  void pair_to_host(double* out2) {
    HIPCHK(hipMemcpyAsync(out2, pair.p, 2 * sizeof(double), hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
  }

  // ---- transforms ------------------------------------------------------------
  // global-pass 2D slices: real [count][Y][X] -> half spectra [count][Y][Xh], and back
  // (unnormalised; src is overwritten by the inverse column pass)
  // (3D: slices of Tn planes, [count][t][y][x] -> [count][t][y][x']; y-lines per plane,
  // then t-lines over the Y rows of each slice)
  void g_r2c(const double* src, cpx<double>* dst, int64_t count) {
    RowArgs<double> a{};
    a.S = dst;
    a.src = src;
    a.per_img = 1;
    HIPCHK(launch_rows<double>(kRowFwd, a, count, grg, gtwr.as<cpx<double>>(), st));
    HIPCHK(launch_cols<double>(dst, -1, count * Tn, gcy, gtwc.as<cpx<double>>(), st));
    if (Tn > 1) HIPCHK(launch_cols<double>(dst, -1, count * G.Y, gct, gtwt.as<cpx<double>>(), st));
  }
  void g_c2r(cpx<double>* src, double* dst, int64_t count) {
    if (Tn > 1) HIPCHK(launch_cols<double>(src, +1, count * G.Y, gct, gtwt.as<cpx<double>>(), st));
    HIPCHK(launch_cols<double>(src, +1, count * Tn, gcy, gtwc.as<cpx<double>>(), st));
    RowArgs<double> a{};
    a.S = src;
    a.Z = dst;
    a.per_img = 1;
    HIPCHK(launch_rows<double>(kRowFinalZ, a, count, grg, gtwr.as<cpx<double>>(), st));
  }
  // dst[count][F] = R2C of the zero-padded [sx, sy, st] sub-volumes of src placed at
  // offset o in every dimension (o = r: padarray of b, dP:23 / L3:23; o = 0: full grid)
  void fwd_embed(const double* src, int sx, int sy, int stt, int o, cpx<double>* dst,
                 int64_t count) {
    const auto* twc = tw.as<cpx<double>>();
    if (gp) {
      if (sx == G.X && sy == G.Y && stt == Tn && o == 0) {
        g_r2c(src, dst, count);
        return;
      }
      HIPCHK(launch_gp_prolog<double>(0, src, nullptr, nullptr, sx, sy, o, 0.0, 1, r,
                                      gR.as<double>(), G.X, G.Y, count, st, Tn, stt,
                                      Tn > 1 ? o : 0));
      g_r2c(gR.as<double>(), dst, count);
      return;
    }
    if (!is3) {
      HIPCHK(launch_r2c_embed<double>(src, (int64_t)sx * sy, sx, sy, o, o, dst, F, count, twc, G,
                                      st));
      return;
    }
    HIPCHK(launch_plane_fwd<double>(0, src, nullptr, nullptr, sx, sy, stt, o, 0.0, 1, 0, dst,
                                    count, Tn, twc, G, st));
    HIPCHK(launch_tfft<double>(dst, dst, count, G.Y, G.F, -1, twt.as<cpx<double>>(), g.Gt, st));
  }
  // D-step dual + R2C of (u - y) into Ch (dP:107-111)
  void dual_fwd() {
    const auto* twc = tw.as<cpx<double>>();
    if (gp) {
      HIPCHK(launch_gp_prolog<double>(2, D.as<double>(), yD.as<double>(), Usup.as<double>(), 0, 0,
                                      0, 0.0, KG, r, gR.as<double>(), G.X, G.Y, nbl * KG, st, Tn));
      g_r2c(gR.as<double>(), Ch.as<cpx<double>>(), nbl * KG);
      return;
    }
    if (!is3) {
      HIPCHK(launch_dual_r2c<double>(D.as<double>(), yD.as<double>(), Usup.as<double>(),
                                     Ch.as<cpx<double>>(), nbl * KG, twc, G, KG, r, st));
      return;
    }
    HIPCHK(launch_plane_fwd<double>(2, D.as<double>(), yD.as<double>(), Usup.as<double>(), 0, 0, 0,
                                    0, 0.0, KG, r, Ch.as<cpx<double>>(), nbl * KG, Tn, twc, G, st));
    HIPCHK(launch_tfft<double>(Ch.as<cpx<double>>(), Ch.as<cpx<double>>(), nbl * KG, G.Y, G.F, -1,
                               twt.as<cpx<double>>(), g.Gt, st));
  }
  // C2R of Dh -> D, support of D + y, d-norms of block 1 (dP:112-121)
  void inv_dout() {
    const auto* twc = tw.as<cpx<double>>();
    if (gp) {   // Dh stays intact (block 1's spectrum feeds the z-step): the inverse runs on Ch
      HIPCHK(hipMemcpyAsync(Ch.p, Dh.p, (size_t)nbl * KG * F * 16, hipMemcpyDeviceToDevice, st));
      g_c2r(Ch.as<cpx<double>>(), gR.as<double>(), nbl * KG);
      HIPCHK(launch_gp_epilog<double>(2, gR.as<double>(), D.as<double>(), yD.as<double>(),
                                      supp.as<double>(), dnorm.as<double>(), owner0 ? KG : 0,
                                      1.0 / (double)P, r, G.X, G.Y, nbl * KG, nullptr, 0.0, 0, st, Tn));
      return;
    }
    if (!is3) {
      HIPCHK(launch_c2r_dout<double>(Dh.as<cpx<double>>(), D.as<double>(), yD.as<double>(),
                                     supp.as<double>(), dnorm.as<double>(), owner0 ? KG : 0,
                                     nbl * KG, twc, G, r, st));
      return;
    }
    // Dh stays intact (block 1's spectrum feeds the z-step): t-inverse into Ch
    HIPCHK(launch_tfft<double>(Dh.as<cpx<double>>(), Ch.as<cpx<double>>(), nbl * KG, G.Y, G.F, +1,
                               twt.as<cpx<double>>(), g.Gt, st));
    HIPCHK(launch_plane_inv<double>(2, Ch.as<cpx<double>>(), D.as<double>(), yD.as<double>(),
                                    supp.as<double>(), dnorm.as<double>(), owner0 ? KG : 0,
                                    1.0 / (double)P, r, nbl * KG, Tn, twc, G, st));
  }
  // what a z-step launch left for the tol test (register-line z-step, zline.hip):
  // `lagged` the test of the iterate it started from (zpart, one launch late: the
  // launch was speculative), `form` the test of the iterate it produced (fpart)
  struct ZTests {
    bool lagged = false, form = false;
  };
  double* zpart() { return znorm.as<double>(); }
  double* fpart() { return znorm.as<double>() + 2 * np; }
  // one z-iteration over the local patches (dP:147-157; 4D L4:163-167; 3D L3:164-178).
  // The other z-steps leave the test of the produced iterate in znorm when tol_on.
  bool zsplit_ok(bool tol_on) const {
    const char* e = std::getenv("CCSC_ZSPLIT2");   // A/B: CCSC_ZSPLIT2=0 keeps one stream
    const bool on = !(e && e[0] == '0');
    return on && zl_on && !tol_on && zmode == 2 && st3 && np >= 512;
  }
  // both halves of a split z-phase done before anything else reads the state on st
  void zsplit_join() {
    if (!zsplit_open) return;
    hipEvent_t e = get_event(), b = get_event();
    HIPCHK(hipEventRecord(e, st3));
    HIPCHK(hipStreamWaitEvent(st, e, 0));
    HIPCHK(hipEventRecord(b, st));
    pool.push_back(e);
    if (prof) {
      recs.push_back(Rec{0, zsp_a, b, zsp_n});
    } else {
      pool.push_back(zsp_a);
      pool.push_back(b);
    }
    zsplit_open = false;
  }

  // write_z: the 3D / 4D z-steps store z only for the iterations whose z is read (the last
  // of the phase -- the D-precompute's -- the objective's, the tol test's); `yz` holds
  // their state a = z + y (kernels3d.hip, zstep.hip)
  // more: another z-iteration follows directly (3D: its forward plane transform is fused
  // into this one's inverse, c_ready)
  ZTests zstep_iter(bool tol_on, bool write_z = true, bool more = false) {
    const auto* twc = tw.as<cpx<double>>();
    if (is4 && !gp) {
      HIPCHK(launch_zstep_diag<double>(z.as<double>(), yz.as<double>(), E.as<cpx<double>>(),
                                       sden.as<double>(), np * K, twc, G, theta, p.rho_z,
                                       znorm.as<double>(), tol_on, write_z || tol_on, st));
    } else if (is3 && !gp) {
      cpx<double>* C = E.as<cpx<double>>();
      const auto* twtc = twt.as<cpx<double>>();
      // the state a = z + y lives in `yz` (modes 3, kernels3d.hip)
      if (!c_ready)
        HIPCHK(launch_plane_fwd<double>(3, z.as<double>(), yz.as<double>(), nullptr, 0, 0, 0, 0,
                                        theta, 1, r, C, np * K, Tn, twc, G, st, tsolve_tc));
      if (tsolve_tc) {
        HIPCHK(launch_tsolve3<double>(C, BhatT.as<cpx<double>>(), dhatT.as<cpx<double>>(),
                                      sdenT.as<double>(), np, K, G.Y, G.Xh, tsolve_tc,
                                      1.0 / (double)P, twt2.as<cpx<double>>(), gt2, st,
                                      tsolve_ppw));
      } else {
        HIPCHK(launch_tfft<double>(C, C, np * K, G.Y, G.F, -1, twtc, g.Gt, st));
        HIPCHK(launch_zsolve3<double>(C, Bhat.as<cpx<double>>(), dhat.as<cpx<double>>(),
                                      sden.as<double>(), F, np, K, 1.0 / (double)P, st));
        HIPCHK(launch_tfft<double>(C, C, np * K, G.Y, G.F, +1, twtc, g.Gt, st));
      }
      HIPCHK(launch_plane_inv<double>(3, C, z.as<double>(), nullptr, nullptr,
                                      tol_on ? znorm.as<double>() : nullptr, 0, 1.0, r, np * K,
                                      Tn, twc, G, st, tsolve_tc, yz.as<double>(), theta,
                                      write_z || tol_on, more ? C : nullptr));
      c_ready = more;
    } else if (gp) {
      // global-pass 2D slices: c = a - 2 clamp(a) -> R2C -> closed-form solve per bin
      // (k_zsolve3, the 1/P folded in) -> C2R -> a' = z' + clamp(a), z' when it is read
      // (4D: the diagonal solve (E + rho c) sden against the view correlations, L4:327-347)
      cpx<double>* C = is4 ? Cg.as<cpx<double>>() : E.as<cpx<double>>();
      HIPCHK(launch_gp_prolog<double>(3, nullptr, yz.as<double>(), nullptr, 0, 0, 0, theta, 1, r,
                                      gR.as<double>(), G.X, G.Y, np * K, st, Tn));
      g_r2c(gR.as<double>(), C, np * K);
      if (is4)
        HIPCHK(launch_gp_zdiag<double>(C, E.as<cpx<double>>(), sden.as<double>(), p.rho_z, (int)F,
                                       np * K, st));
      else
        HIPCHK(launch_zsolve3<double>(C, Bhat.as<cpx<double>>(), dhat.as<cpx<double>>(),
                                      sden.as<double>(), F, np, K, 1.0 / (double)P, st));
      g_c2r(C, gR.as<double>(), np * K);
      HIPCHK(launch_gp_epilog<double>(3, gR.as<double>(), z.as<double>(), nullptr, nullptr,
                                      tol_on ? znorm.as<double>() : nullptr, 0, 1.0, r, G.X, G.Y,
                                      np * K, yz.as<double>(), theta, write_z || tol_on, st, Tn));
    } else if (zl_on) {
      // register-line z-step (zline.hip): mode 0 reads (z, y) and leaves a in state order.
      // tol > 0: a launch whose starting w was solved with the current filters measures
      // the iterate it produces in place (Form); otherwise (the first z-iteration after a
      // d-phase, or a materialised state) it stores the z it starts from in `yz`, and the
      // next launch measures that iterate against it (Cmp, one launch late)
      const int mode = zmode == 2 ? 2 : 0;
      if (zsplit_ok(tol_on)) {
        if (!zsplit_open) {
          zsp_a = get_event();
          HIPCHK(hipEventRecord(zsp_a, st));
          HIPCHK(hipStreamWaitEvent(st3, zsp_a, 0));
          zsplit_open = true;
          zsp_n = 0;
        }
        const int64_t na = np / 2;
        const int64_t zo = na * K * (int64_t)P, wo = na * (int64_t)F;
        HIPCHK(launch_zline<double>(z.as<double>(), z.as<double>(), z.as<double>(), yz.as<double>(),
                                    W.as<cpx<double>>(), Bhs.as<cpx<double>>(), dws,
                                    dhs.as<cpx<double>>(), sdens.as<double>(), na, K, theta,
                                    p.rho_z, 2, st, 0, nullptr, nullptr, nullptr));
        HIPCHK(launch_zline<double>(z.as<double>() + zo, z.as<double>() + zo, z.as<double>() + zo,
                                    yz.as<double>() + zo, W.as<cpx<double>>() + wo,
                                    Bhs.as<cpx<double>>() + wo, dws, dhs.as<cpx<double>>(),
                                    sdens.as<double>(), np - na, K, theta, p.rho_z, 2, st3, 0,
                                    nullptr, nullptr, nullptr));
        ++zsp_n;
        dws = dhs.as<cpx<double>>();
        return ZTests{};
      }
      const bool same = mode == 2 && dws == dhs.as<cpx<double>>();
      int tolv = 0;
      if (tol_on) {
        if (!same) tolv = kZlTolStore;
        else if (zt == ZT_PREV) tolv = kZlTolStore | kZlTolCmp | kZlTolForm;
        else tolv = kZlTolForm;
      }
      HIPCHK(launch_zline<double>(z.as<double>(), z.as<double>(), z.as<double>(), yz.as<double>(),
                                  W.as<cpx<double>>(), Bhs.as<cpx<double>>(),
                                  zmode == 2 ? dws : dhs.as<cpx<double>>(), dhs.as<cpx<double>>(),
                                  sdens.as<double>(), np, K, theta, p.rho_z, mode, st, tolv,
                                  yz.as<double>(), zpart(), fpart()));
      zmode = 2;
      dws = dhs.as<cpx<double>>();
      // `yz` holds the z before the current iterate only after a lone Store launch; after a
      // Cmp launch it holds the iterate the test covered (kept for zl_rollback only)
      if (tol_on) zt = (tolv == kZlTolStore) ? ZT_PREV : ZT_NONE;
      ZTests r;
      r.lagged = (tolv & kZlTolCmp) != 0;
      r.form = (tolv & kZlTolForm) != 0;
      return r;
    } else if (!tol_on) {
      // one pass per patch over the pre-threshold state a (zsplit.hip): `z` holds a
      HIPCHK(launch_zsplit<double>(z.as<double>(), z.as<double>(), yz.as<double>(),
                                   W.as<cpx<double>>(), Bhat.as<cpx<double>>(), dw,
                                   dhat.as<cpx<double>>(), sden.as<double>(), np, twc, G, K,
                                   theta, zmode, st));
      zmode = 1;
      dw = dhat.as<cpx<double>>();
    } else {
      // tol test (dP:156-157): a into cbuf so z_old stays in z, then (z, y) from a
      // and ifft2(conj(d) w) with the per-slice change norms
      HIPCHK(launch_zsplit<double>(z.as<double>(), cbuf.as<double>(), yz.as<double>(),
                                   W.as<cpx<double>>(), Bhat.as<cpx<double>>(), dw,
                                   dhat.as<cpx<double>>(), sden.as<double>(), np, twc, G, K,
                                   theta, zmode, st));
      HIPCHK(launch_zmat<double>(cbuf.as<double>(), yz.as<double>(), W.as<cpx<double>>(),
                                 dhat.as<cpx<double>>(), z.as<double>(), z.as<double>(),
                                 znorm.as<double>(), np, twc, G, K, theta, st));
      zmode = 0;
    }
    return ZTests{};
  }
  // register-line state + tol: the test of the current iterate against the z before it
  // (in `yz`, ZT_PREV) without advancing (end of a z-phase)
  void zl_finalize() {
    HIPCHK(launch_zline<double>(z.as<double>(), z.as<double>(), z.as<double>(), yz.as<double>(),
                                W.as<cpx<double>>(), Bhs.as<cpx<double>>(), dws,
                                dhs.as<cpx<double>>(), sdens.as<double>(), np, K, theta, p.rho_z,
                                3, st, kZlTolStore | kZlTolCmp, yz.as<double>(), zpart(),
                                fpart()));
    zt = ZT_CUR;
  }
  // register-line state + tol: materialise (z, y) of the current iterate and measure it
  // against the z before it (`yz`, ZT_PREV): both slices to natural order in place, then
  // k_zmat with z_old = yz (read before it is overwritten by y)
  void zl_materialize_tol() {
    HIPCHK(launch_state_to_nat_inplace<double>(z.as<double>(), np * K, st));
    HIPCHK(launch_state_to_nat_inplace<double>(yz.as<double>(), np * K, st));
    HIPCHK(launch_zmat<double>(z.as<double>(), yz.as<double>(), W.as<cpx<double>>(), dws,
                               z.as<double>(), yz.as<double>(), znorm.as<double>(), np,
                               tw.as<cpx<double>>(), G, K, theta, st, true));
    zmode = 0;
    zt = ZT_NONE;
  }
  // register-line state + tol: the launch just made was one iteration past the break
  // (its test of the iterate it started from fired).  That iterate is intact: `yz` holds
  // its z and `z` its pre-threshold value a = z + y (the launch's state write); the
  // launch's w is dropped.  (z, y) natural <- (yz, z - yz).
  void zl_rollback() {
    HIPCHK(launch_state_to_nat_inplace<double>(z.as<double>(), np * K, st));
    HIPCHK(launch_state_to_nat_inplace<double>(yz.as<double>(), np * K, st));
    HIPCHK(launch_sub_inplace<double>(z.as<double>(), yz.as<double>(), np * K * (int64_t)P, st));
    std::swap(z.p, yz.p);   // z <- z, yz <- y
    zmode = 0;
    zt = ZT_NONE;
  }
  // state a -> (z, y) materialised in place (objective, outputs)
  void materialize_z() {
    if (zmode == 0) return;
    zt = ZT_NONE;   // `yz` receives y
    if (zmode == 2) {   // state order -> natural a in yz, then (z, y) from it
      HIPCHK(launch_state_to_nat<double>(z.as<double>(), yz.as<double>(), np * K, st));
      HIPCHK(launch_zmat<double>(yz.as<double>(), yz.as<double>(), W.as<cpx<double>>(), dws,
                                 z.as<double>(), nullptr, nullptr, np, tw.as<cpx<double>>(), G, K,
                                 theta, st, true));
      zmode = 0;
      return;
    }
    HIPCHK(launch_zmat<double>(z.as<double>(), yz.as<double>(), W.as<cpx<double>>(), dw,
                               z.as<double>(), nullptr, nullptr, np, tw.as<cpx<double>>(), G, K,
                               theta, st));
    zmode = 0;
  }

  // 3D objective (L3:342-355), patch by patch through the z-step's spectrum buffer
  void objective3_parts(const cpx<double>* dsp, double* DZdev) {
    const auto* twc = tw.as<cpx<double>>();
    const auto* twtc = twt.as<cpx<double>>();
    cpx<double>* C = E.as<cpx<double>>();
    const int sbx = (int)p.sb[0], sby = (int)p.sb[1], sbt = (int)p.sb[2];
    HIPCHK(hipMemsetAsync(pair.p, 0, 2 * sizeof(double), st));
    for (int64_t q = 0; q < np; ++q) {
      const double* zq = z.as<double>() + (size_t)q * K * P;
      double* dzq = DZdev ? DZdev + (size_t)q * P : odz.as<double>();
      HIPCHK(launch_plane_fwd<double>(0, zq, nullptr, nullptr, G.X, G.Y, Tn, 0, 0.0, 1, 0, C, K,
                                      Tn, twc, G, st));
      HIPCHK(launch_tfft<double>(C, C, K, G.Y, G.F, -1, twtc, g.Gt, st));
      HIPCHK(launch_corr_sum<double>(C, dsp, oacc.as<cpx<double>>(), F, K, st));
      HIPCHK(launch_tfft<double>(oacc.as<cpx<double>>(), oacc.as<cpx<double>>(), 1, G.Y, G.F, +1,
                                 twtc, g.Gt, st));
      HIPCHK(launch_plane_inv<double>(0, oacc.as<cpx<double>>(), dzq, nullptr, nullptr, nullptr, 0,
                                      1.0 / (double)P, r, 1, Tn, twc, G, st));
      HIPCHK(launch_crop_sq<double>(dzq, bdev.as<double>() + (size_t)q * sbx * sby * sbt, sbx, sby,
                                    sbt, r, r, G.X, G.Y, zq, (int64_t)K * P, pair.as<double>(), st));
    }
  }


  // objective with filter spectrum `dsp` (valid on every rank); DZ optional.
  // global-pass 2D objective (dP:305-324), patch by patch through the z-step's spectra
  // (4D, L4:349-369: every view of the patch from the same code spectra, DZ cropped per view)
  void objective_gp_parts(const cpx<double>* dsp, double* DZdev) {
    cpx<double>* C = is4 ? Cg.as<cpx<double>>() : E.as<cpx<double>>();
    const int sbx = (int)p.sb[0], sby = (int)p.sb[1];
    HIPCHK(hipMemsetAsync(pair.p, 0, 2 * sizeof(double), st));
    if (is4) {
      const size_t vb = (size_t)sbx * sby;
      for (int64_t q = 0; q < np; ++q) {
        const double* zq = z.as<double>() + (size_t)q * K * P;
        g_r2c(zq, C, K);
        HIPCHK(launch_gp_views<double>(C, dsp, oacc.as<cpx<double>>(), (int)F, K, NV, st));
        g_c2r(oacc.as<cpx<double>>(), gR.as<double>(), NV);
        HIPCHK(launch_gp_crop<double>(gR.as<double>(), bdev.as<double>() + (size_t)q * NV * vb,
                                      DZdev ? DZdev + (size_t)q * NV * vb : nullptr, sbx, sby, r,
                                      G.X, G.Y, 1.0 / (double)P, pair.as<double>(), NV, st));
        // sum |z| of the patch (no crop term: sx = sy = 0)
        HIPCHK(launch_crop_sq<double>(gR.as<double>(), bdev.as<double>(), 0, 0, 1, r, 0, G.X, G.Y, zq,
                                      (int64_t)K * P, pair.as<double>(), st));
      }
      return;
    }
    for (int64_t q = 0; q < np; ++q) {
      const double* zq = z.as<double>() + (size_t)q * K * P;
      double* dzq = DZdev ? DZdev + (size_t)q * P : odz.as<double>();
      g_r2c(zq, C, K);
      HIPCHK(launch_corr_sum<double>(C, dsp, oacc.as<cpx<double>>(), F, K, st));
      g_c2r(oacc.as<cpx<double>>(), gR.as<double>(), 1);
      HIPCHK(launch_gp_epilog<double>(0, gR.as<double>(), dzq, nullptr, nullptr, nullptr, 0,
                                      1.0 / (double)P, r, G.X, G.Y, 1, nullptr, 0.0, 0, st, Tn));
      // (3D: the crop of L3:351 in t as well)
      const int sbt = Tn > 1 ? (int)p.sb[2] : 1;
      HIPCHK(launch_crop_sq<double>(dzq, bdev.as<double>() + (size_t)q * sbx * sby * sbt, sbx, sby,
                                    sbt, r, Tn > 1 ? r : 0, G.X, G.Y, zq, (int64_t)K * P,
                                    pair.as<double>(), st));
    }
  }

  double objective(const cpx<double>* dsp, double* DZdev) {
    if (is3 || gp) {
      if (gp) objective_gp_parts(dsp, DZdev);
      else objective3_parts(dsp, DZdev);
      allreduce(pair.as<double>(), 2);
      double h2[2];
      pair_to_host(h2);
      return p.lambda_residual * 0.5 * h2[0] + p.lambda_prior * h2[1];
    }
    materialize_z();
    HIPCHK(launch_objective<double>(z.as<double>(), dsp, bdev.as<double>(), (int)p.sb[0],
                                    (int)p.sb[1], r, DZdev, part.as<double>(), np,
                                    tw.as<cpx<double>>(), G, K, NV, st));
    HIPCHK(launch_sum_pairs<double>(part.as<double>(), (int)(np * NV), pair.as<double>(), st));
    allreduce(pair.as<double>(), 2);
    double h2[2];
    pair_to_host(h2);
    return p.lambda_residual * 0.5 * h2[0] + p.lambda_prior * h2[1];
  }
  // current filter spectrum of global block 1 into dtmp on every rank
  const cpx<double>* current_dhat() {
    if (owner0)
      HIPCHK(hipMemcpyAsync(dtmp.p, Dh.p, (size_t)KG * F * 16, hipMemcpyDeviceToDevice, st));
    bcast0(dtmp.as<double>(), (size_t)2 * KG * F);
    return dtmp.as<cpx<double>>();
  }

  // ---- one outer iteration --------------------------------------------------
  void outer_iteration() {
    const int it = outer_done;
    hipEvent_t e0 = get_event(), e1 = get_event();
    double obj_ms = 0;
    auto objective_timed = [&](const cpx<double>* dsp) {
      hipEvent_t a = get_event(), b = get_event();
      HIPCHK(hipEventRecord(a, st));
      const double o = objective(dsp, nullptr);
      HIPCHK(hipEventRecord(b, st));
      HIPCHK(hipEventSynchronize(b));
      float ms = 0;
      HIPCHK(hipEventElapsedTime(&ms, a, b));
      obj_ms += ms;
      pool.push_back(a);
      pool.push_back(b);
      return o;
    };
    HIPCHK(hipEventRecord(e0, st));

    // ---- D precompute (dP:95-99) ----
    // 110 grid: block j+1's R2C on st3 beside block j's Gram on st (same-box A/B at
    // 8ff8b2a: 949 vs 957.7 ms per C2 step in series, profiles/r03j/preov_ab.txt)
    const bool ovz = zmode == 2 && st3;
    if (ovz) {   // st3's R2C passes read the state the z-phase left on st
      HIPCHK(hipEventRecord(ev_s, st));
      HIPCHK(hipStreamWaitEvent(st3, ev_s, 0));
    }
    for (int64_t jl = 0; jl < nbl; ++jl) {
      cpx<double>* Zc = (ovz && (jl & 1)) ? Zh2.as<cpx<double>>() : Zh.as<cpx<double>>();
      if (ovz) {   // the same on the lanes (zline.hip), on st3 (see st3)
        if (jl >= 2) HIPCHK(hipStreamWaitEvent(st3, ev_gz[jl & 1], 0));   // Gram(jl-2) read Zc
        HIPCHK(launch_zhat_line<double>(z.as<double>() + (size_t)jl * ni * K * P,
                                        W.as<cpx<double>>() + (size_t)jl * ni * F, dws, Zc, ni,
                                        K, theta, st3));
        HIPCHK(hipEventRecord(ev_z, st3));
        HIPCHK(hipStreamWaitEvent(st, ev_z, 0));
      } else if (zmode == 2)
        HIPCHK(launch_zhat_line<double>(z.as<double>() + (size_t)jl * ni * K * P,
                                        W.as<cpx<double>>() + (size_t)jl * ni * F, dws,
                                        Zh.as<cpx<double>>(), ni, K, theta, st));
      else if (zmode)  // fft2(z) of the state a: fft2(u - y) + XY conj(dw) w, u = soft(a)
        HIPCHK(launch_zhat_split<double>(z.as<double>() + (size_t)jl * ni * K * P,
                                         W.as<cpx<double>>() + (size_t)jl * ni * F,
                                         zmode == 2 ? dws : dw, Zh.as<cpx<double>>(), ni,
                                         tw.as<cpx<double>>(), G, K, theta, st, zmode == 2));
      else
        fwd_embed(z.as<double>() + (size_t)jl * ni * K * P, G.X, G.Y, Tn, 0,
                  Zh.as<cpx<double>>(), (int64_t)ni * K);
      timed(1, [&] {
        const cpx<double>* Bj = Bhat.as<cpx<double>>() + (size_t)jl * ni * NV * F;
        cpx<double>* Lj = L.as<cpx<double>>() + (size_t)jl * F * Kp;
        cpx<double>* hj = h.as<cpx<double>>() + (size_t)jl * F * NV * K;
        const int NVg = h_sep ? 0 : NV;
        if (h_sep)
          HIPCHK(launch_hs_corr<double>(Zc, Bj, hj, F, NV, K, ni, st));
        if (wbig)
          HIPCHK(launch_wbig_gram(Zc, Bj, Xbig.as<cpx<double>>(), Lj, hj, F, K, ni, p.rho_d, NV, st));
        else if (woodbury)
          HIPCHK(launch_gram_wb<double>(Zc, Bj, Lj, hj, F, K, ni, p.rho_d, NV, wb_stage, st));
        else if (gram_big)
          HIPCHK(launch_gram_big(Zc, Bj, Xbig.as<cpx<double>>(), Lj, hj, F, K, ni, p.rho_d, NVg, st));
        else if (gram_mf) {
          HIPCHK(launch_gram_chol_mf(Zc, Bj, Lj, hj, F, K, ni, p.rho_d, NVg, st));
          if (dtile) {
            HIPCHK(hipEventRecord(ev_g, st));
            HIPCHK(hipStreamWaitEvent(st2, ev_g, 0));
            HIPCHK(launch_invert_diag(Lj, F, K, st2));
          }
        }
        else
          HIPCHK(launch_gram_chol<double>(Zc, Bj, Lj, hj, F, K, ni, p.rho_d, NVg, st));
      });
      if (ovz) HIPCHK(hipEventRecord(ev_gz[jl & 1], st));
    }
    if (dtile) {   // every block's inverted diagonal tiles before the first d-solve
      HIPCHK(hipEventRecord(ev_i, st2));
      HIPCHK(hipStreamWaitEvent(st, ev_i, 0));
    }
    // ---- D iterations (dP:103-134) ----
    const bool tol_on = p.tol > 0;
    const bool want_od = verbose_refresh_d() || p.trace_objective;
    int nd = 0;
    for (int id = 0; id < p.max_it_d; ++id) {
      timed(3, [&] { dual_fwd(); });
      timed(2, [&] {
        if (wbig)
          HIPCHK(launch_wbig_solve(L.as<cpx<double>>(), h.as<cpx<double>>(), Ch.as<cpx<double>>(),
                                   Dh.as<cpx<double>>(), (int)nbl, F, K, ni, p.rho_d, NV, st));
        else if (woodbury)
          HIPCHK(launch_dsolve_wb<double>(L.as<cpx<double>>(), h.as<cpx<double>>(),
                                          Ch.as<cpx<double>>(), Dh.as<cpx<double>>(), (int)nbl, F,
                                          K, ni, p.rho_d, NV, wb_stage, st));
        else if (dtile)
          HIPCHK(launch_dsolve_tile(L.as<cpx<double>>(), h.as<cpx<double>>(),
                                    Ch.as<cpx<double>>(), Dh.as<cpx<double>>(), (int)nbl, F, K,
                                    p.rho_d, NV, st));
        else
          HIPCHK(launch_dsolve<double>(L.as<cpx<double>>(), h.as<cpx<double>>(),
                                       Ch.as<cpx<double>>(), Dh.as<cpx<double>>(), (int)nbl, F, K,
                                       p.rho_d, NV, st));
      });
      timed(4, [&] { inv_dout(); });
      HIPCHK(launch_supp_reduce<double>(supp.as<double>(), ssum.as<double>(), (int)nbl, KG * SS,
                                        st));
      allreduce(ssum.as<double>(), (size_t)KG * SS);
      // Pi normalises per filter (2D, dP:212-213; 3D, L3:245-252) / per (u,v,k) slice
      // (4D, L4:224-225)
      HIPCHK(launch_project<double>(ssum.as<double>(), Usup.as<double>(), KG, SS,
                                    1.0 / (double)N, st));
      ++nd;
      double dd = std::numeric_limits<double>::quiet_NaN();
      if (tol_on) {
        if (owner0)
          // (the plane kernels leave one pair per (slice, t); the global-pass epilogue per slice)
          HIPCHK(launch_sum_pairs<double>(dnorm.as<double>(), gp ? KG : KG * Tn, pair.as<double>(), st));
        else HIPCHK(hipMemsetAsync(pair.p, 0, 2 * sizeof(double), st));
        allreduce(pair.as<double>(), 2);
        double h2[2];
        pair_to_host(h2);
        dd = std::sqrt(h2[0]) / std::sqrt(h2[1]);
        last_d = dd;
        tr_dd[(size_t)it * p.max_it_d + id] = dd;
      }
      if (want_od) {
        const double o = objective_timed(current_dhat());
        if (verbose_refresh_d()) obj_filter = o;
        if (p.trace_objective) tr_od[(size_t)it * p.max_it_d + id] = o;
      }
      if (tol_on && dd < p.tol) break;  // dP:130-132
    }
    // ---- Z precompute (dP:143-144): d = Dhat of block 1 ----
    if (zmode == 1 && dw == dhat.as<cpx<double>>()) {  // keep the spectrum w was solved with
      std::swap(dhat.p, dhatw.p);
      dw = dhatw.as<cpx<double>>();
    }
    if (zmode == 2 && dws == dhs.as<cpx<double>>()) {
      std::swap(dhs.p, dhws.p);
      dws = dhws.as<cpx<double>>();
    }
    if (owner0) HIPCHK(hipMemcpyAsync(dhat.p, Dh.p, (size_t)KG * F * 16, hipMemcpyDeviceToDevice, st));
    bcast0(dhat.as<double>(), (size_t)2 * KG * F);
    // s(f) = sum over filters (and views, L4:277,330) of |dhat|^2
    HIPCHK(launch_sden<double>(dhat.as<cpx<double>>(), sden.as<double>(), F, KG, p.rho_z,
                               1.0 / (double)P, st));
    if (zl_on) {
      HIPCHK(launch_to_slots<double>(dhat.as<cpx<double>>(), dhs.as<cpx<double>>(), K, st));
      HIPCHK(launch_to_slots_real<double>(sden.as<double>(), sdens.as<double>(), st));
    }
    if (tsolve_tc) {
      HIPCHK(launch_to_ttiles<double>(dhat.as<cpx<double>>(), dhatT.as<cpx<double>>(), Tn, G.Y,
                                      G.Xh, tsolve_tc, K, st));
      HIPCHK(launch_to_ttiles_real<double>(sden.as<double>(), sdenT.as<double>(), Tn, G.Y, G.Xh,
                                           tsolve_tc, st));
    }
    if (is4)   // L4:327 first term, constant over the z-iterations
      HIPCHK(launch_view_corr<double>(dhat.as<cpx<double>>(), Bhat.as<cpx<double>>(),
                                      E.as<cpx<double>>(), np, F, K, NV, st));
    // ---- Z iterations (dP:147-168) ----
    const bool want_oz = verbose_refresh_z() || p.trace_objective;
    int nz = 0;
    // z_diff of iteration iz (dP:156-157, dZ:163-164) from `count` partial pairs
    // (||z - z_old||^2, ||z||^2); the Parseval form of zline.hip may round a vanishing
    // difference to a tiny negative sum
    auto z_test = [&](int iz, const double* parts, int64_t count) {
      HIPCHK(launch_sum_pairs<double>(parts, (int)count, pair.as<double>(), st));
      allreduce(pair.as<double>(), 2);
      double h2[2];
      pair_to_host(h2);
      const double zd = std::sqrt(std::max(h2[0], 0.0)) / std::sqrt(h2[1]);
      last_z = zd;
      tr_zd[(size_t)it * p.max_it_z + iz] = zd;
      return zd;
    };
    // register-line z-step with tol (zline.hip): a launch measures the iterate it
    // produces (ZTests::form) once its starting w was solved with the current filters;
    // after a d-phase the first launch stores its starting z and the second measures
    // that iterate one launch late (ZTests::lagged; the second launch was speculative
    // when the test fires: zl_rollback); the objective's materialisation measures
    // without the lag (zl_materialize_tol)
    const bool zl_tol = zl_on && tol_on;
    bool zbreak = false;
    c_ready = false;
    for (int iz = 0; iz < p.max_it_z; ++iz) {
      ZTests zt_done;
      const bool wz = want_oz || iz + 1 == p.max_it_z;
      // the objective (want_oz) reuses the spectrum buffer between iterations
      const bool more = iz + 1 < p.max_it_z && !want_oz;
      if (zsplit_ok(tol_on))
        zt_done = zstep_iter(tol_on, wz, more);   // timed as one phase record by zsplit_join
      else
        timed(0, [&] { zt_done = zstep_iter(tol_on, wz, more); });
      ++nz;
      if (zt_done.lagged && z_test(iz - 1, zpart(), np) < p.tol) {   // dP:165-167 for iz - 1
        zl_rollback();
        --nz;
        zbreak = true;
        break;
      }
      double zd = std::numeric_limits<double>::quiet_NaN();
      if (zl_tol && want_oz) {
        zl_materialize_tol();
        zd = z_test(iz, znorm.as<double>(), np * K);
      } else if (zt_done.form) {
        zd = z_test(iz, fpart(), np);
      } else if (tol_on && !zl_tol) {
        zd = z_test(iz, znorm.as<double>(), gp ? np * K : np * K * Tn);
      }
      if (want_oz) {
        zsplit_join();
        const double o = objective_timed(dhat.as<cpx<double>>());
        if (verbose_refresh_z()) obj_z = o;
        if (p.trace_objective) tr_oz[(size_t)it * p.max_it_z + iz] = o;
      }
      if (tol_on && zd < p.tol) {  // dP:165-167
        zbreak = true;
        break;
      }
    }
    zsplit_join();
    if (zl_tol && !zbreak && zt == ZT_PREV) {   // the last iteration's test
      zl_finalize();
      z_test(nz - 1, zpart(), np);
    }
    HIPCHK(hipEventRecord(e1, st));
    HIPCHK(hipEventSynchronize(e1));
    float ms = 0;
    HIPCHK(hipEventElapsedTime(&ms, e0, e1));
    pool.push_back(e0);
    pool.push_back(e1);
    drain_records();
    const double secs = (ms - obj_ms) * 1e-3;
    v_obj_d.push_back(obj_filter);  // dP:174-176
    v_obj_z.push_back(obj_z);
    v_tim.push_back(v_tim.back() + secs);
    v_nd.push_back(nd);
    v_nz.push_back(nz);
    ++outer_done;
    if (tol_on && last_z < p.tol && last_d < p.tol) finished = true;  // dP:186-188
  }

  void ensure_trace_capacity(int total_outer) {
    const size_t nd = (size_t)total_outer * p.max_it_d, nz = (size_t)total_outer * p.max_it_z;
    const double nan = std::numeric_limits<double>::quiet_NaN();
    if (tr_od.size() < nd) tr_od.resize(nd, nan);
    if (tr_dd.size() < nd) tr_dd.resize(nd, nan);
    if (tr_oz.size() < nz) tr_oz.resize(nz, nan);
    if (tr_zd.size() < nz) tr_zd.resize(nz, nan);
  }

  void step(int n_outer, int32_t* done) {
    ensure_trace_capacity(outer_done + n_outer);
    for (int i = 0; i < n_outer && !finished; ++i) outer_iteration();
    if (done) *done = finished ? 1 : 0;
  }

  void results(ccsc_outputs* out) {
    if (!out) return;
    if (out->d_res) {
      // D1 lives on rank 0 (block 1); broadcast so every rank returns it.
      std::vector<double> D1((size_t)KG * P);
      DevBuf tmp;
      tmp.alloc((size_t)KG * P * 8);
      if (owner0) HIPCHK(hipMemcpyAsync(tmp.p, D.p, tmp.bytes, hipMemcpyDeviceToDevice, st));
      bcast0(tmp.as<double>(), (size_t)KG * P);
      HIPCHK(hipMemcpyAsync(D1.data(), tmp.p, tmp.bytes, hipMemcpyDeviceToHost, st));
      HIPCHK(hipStreamSynchronize(st));
      // d_res = circshift(D1, +r)(1:psf, 1:psf(, 1:psf), :)  (dP:195-196; 4D L4:208-209:
      // per view; 3D L3:226-227)
      const int st3 = Tn > 1 ? s : 1;
      for (int k = 0; k < KG; ++k)
        for (int l = 0; l < st3; ++l)
          for (int j = 0; j < s; ++j)
            for (int i = 0; i < s; ++i) {
              const int x = (i - r + G.X) % G.X, y = (j - r + G.Y) % G.Y;
              const int t = Tn > 1 ? (l - r + Tn) % Tn : 0;
              out->d_res[i + (size_t)s * (j + (size_t)s * (l + (size_t)st3 * k))] =
                  D1[(size_t)k * P + ((size_t)t * G.Y + y) * G.X + x];
            }
    }
    if (out->z_res) {
      materialize_z();
      HIPCHK(hipStreamSynchronize(st));   // st is non-blocking: hipMemcpy does not order after it
      HIPCHK(hipMemcpy(out->z_res, z.p, m.z, hipMemcpyDeviceToHost));
    }
    if (out->DZ) {
      // DZ = real(ifft2(sum_k zhat .* dup{1}))  (dP:193), uncropped [X,Y,1,n]
      DevBuf dz;
      dz.alloc(is4 ? (size_t)np * NV * p.sb[0] * p.sb[1] * 8 : (size_t)np * P * 8);
      objective(dhat.as<cpx<double>>(), dz.as<double>());
      HIPCHK(hipMemcpy(out->DZ, dz.p, dz.bytes, hipMemcpyDeviceToHost));
    }
    if (out->obj_val) *out->obj_val = objective(dhat.as<cpx<double>>(), nullptr);
  }

  void iterlog(ccsc_iterlog* lg) {
    if (!lg) return;
    const int cnt = std::min<int>(lg->capacity, (int)v_tim.size());
    lg->count = cnt;
    for (int i = 0; i < cnt; ++i) {
      if (lg->obj_vals_d) lg->obj_vals_d[i] = v_obj_d[i];
      if (lg->obj_vals_z) lg->obj_vals_z[i] = v_obj_z[i];
      if (lg->tim_vals) lg->tim_vals[i] = v_tim[i];
    }
    const int no = std::min<int>(lg->capacity, outer_done);
    for (int i = 0; i < no; ++i) {
      if (lg->n_d) lg->n_d[i] = v_nd[i];
      if (lg->n_z) lg->n_z[i] = v_nz[i];
      if (lg->flags) lg->flags[i] = 0;
      for (int t = 0; t < p.max_it_d; ++t) {
        const size_t q = (size_t)i * p.max_it_d + t;
        if (lg->trace_obj_d) lg->trace_obj_d[q] = q < tr_od.size() ? tr_od[q] : NAN;
        if (lg->trace_d_diff) lg->trace_d_diff[q] = q < tr_dd.size() ? tr_dd[q] : NAN;
      }
      for (int t = 0; t < p.max_it_z; ++t) {
        const size_t q = (size_t)i * p.max_it_z + t;
        if (lg->trace_obj_z) lg->trace_obj_z[q] = q < tr_oz.size() ? tr_oz[q] : NAN;
        if (lg->trace_z_diff) lg->trace_z_diff[q] = q < tr_zd.size() ? tr_zd[q] : NAN;
      }
    }
  }

  double alg_bytes(int id) const {
    const double Pd = P, Fd = F, Kd = K;
    switch (id) {
      case 0:  // z-iteration, SURVEY.md §8(d): n K (4 s P + 4 c F) + n c F V  (s = 8, c = 16):
               // prox+dual+R2C, solve, C2R stages each reading/writing their operands once
        return (double)np * Kd * (4.0 * 8.0 * Pd + 4.0 * 16.0 * Fd) + (double)np * NV * 16.0 * Fd;
      case 1:  // gram+chol per block: read A (ni x K x F) + b, write L, h
        return (double)ni * Kd * Fd * 16.0 + ni * Fd * 16.0 + Fd * Kp * 16.0 + Fd * Kd * 16.0;
      case 2:  // dsolve over local blocks: read L, h, C; write Dhat
        return (double)nbl * Fd * (Kp + 3.0 * Kd) * 16.0;
      case 3:  // dual+R2C: read D, y; write y, C
        return (double)nbl * Kd * (3.0 * 8.0 * Pd + 16.0 * Fd);
      case 4:  // C2R + support: read Dhat, write D
        return (double)nbl * Kd * (16.0 * Fd + 8.0 * Pd);
    }
    return 0;
  }
};

// ---------------------------------------------------------------------------
// Session: 2-3D hyperspectral learner (L23 = 2-3D/DictionaryLearning/admm_learn.m)
// ---------------------------------------------------------------------------
// One non-consensus ADMM over all n images (one block).  It runs on one rank:
// its d-solve sums over every image per frequency, so sharding images needs an
// all-reduce of K x K Grams ("replicas only at first").
// Device state (hs23.hip):
//   real     [X,Y,W,n]  v = H z (= Dz - smoothinit), eD = d_D{1}, eZ = d_Z{1}, smp = smoothinit
//            [X,Y,W,K]  D, yD = -d_D{2} (the consensus kernels' sign), Dold
//            [X,Y,K,n]  z, eZ2 = d_Z{2}, zold
//   spectra  Zh [n][K][F] (zhat; xi_Z{2} in place), Xi [n][W][F] (xi{1}, also H zhat),
//            Ch [K][W][F] (xi_D{2}), Dh, Dhold [K][W][F] (d_hat), h [F][W][K],
//            L [F][K(K+1)/2] (Cholesky of Z'Z + rho I per bin)
struct PlanHS {
  size_t b, vwn, dwk, zkn, Zh, Xi, dspec, L, h, misc, gr, wx;
  size_t total() const {
    return b + 4 * vwn + 3 * dwk + 3 * zkn + Zh + Xi + 3 * dspec + L + h + misc + gr + wx;
  }
};

// n_local: the rank's images (shard(); the whole problem on one rank)
static PlanHS plan_hs(const ccsc_problem& p, const Geom& g, int64_t n_local, bool dist) {
  PlanHS m{};
  const size_t P = g.P(), F = g.F(), K = p.K, W = p.views[0], n = (size_t)n_local;
  const size_t SS = (size_t)p.psf * p.psf;
  m.b = (size_t)p.sb[0] * p.sb[1] * W * n * 8;
  m.vwn = P * W * n * 8;
  m.dwk = P * W * K * 8;
  m.zkn = P * K * n * 8;
  m.Zh = F * K * n * 16;
  m.Xi = F * W * n * 16;
  m.dspec = F * W * K * 16;
  m.L = F * (K * (K + 1) / 2) * 16;
  m.h = F * W * K * 16;
  // smooth_init staging, sden, support/projection, d0 staging, reduction scratch, twiddles
  m.misc = m.b + F * 8 + 2 * W * K * SS * 8 + 2 * W * K * 8 + (SS * K + SS * W * K) * 8 +
           (2 * std::max<size_t>(std::max(W * n, K * n), kNormParts) + 8) * 8 +
           (size_t)g.G.ntw * 16 + (g.gp ? 64 * 1024 : 0);
  // global-pass slices: the real scratch of the largest transform batch
  m.gr = g.gp ? std::max({W * n, K * n, W * K}) * P * 8 : 0;
  // K > 192: the n x n Woodbury factor (wbig.hip) and its frequency-major workspace; several
  // ranks: the same workspace for the per-rank Gram (gramchol_big.hip, summed over the ranks)
  m.wx = (K > 192 || dist) ? m.Zh : 0;
  return m;
}

struct SessionHS {
  ccsc_ctx* ctx;
  ccsc_problem p;
  Geom g;
  Grid2D G;
  PlanHS m;
  int r, s, SS, K, W, KG, P, F, sbx, sby;
  int n;
  hipStream_t st;
  double th_D1 = 0, th_Z1 = 0, th_Z2 = 0, gamma_h = 0;

  DevBuf tw, bdev, smp, v, eD, eZ, D, yD, Dold, z, eZ2, zold, Zh, Xi, Ch, Dh, Dhold, L, h, sden,
      Usup, supp, dnorm, part, pair;
  // slices past one CU's LDS (Geom::gp): the global line passes of recon.hip with the
  // elementwise halves of the fused slice kernels in gslice.hip over the real scratch gR
  bool gp = false;
  RowGeom grg{};
  ColGeom gcy{};
  DevBuf gtwr, gtwc, gR;

  int outer_done = 0;
  bool finished = false;
  // 64 < K <= 112: the tile d-solve over the W wavelengths on a factor with inverted
  // diagonal tiles (dstep.hip; CCSC_DS_TILE=0 keeps the two-sweep k_dsolve)
  bool hs_dtile = false;
  // K > 192: the reference's own n x n Woodbury form of opt_f (L23:290; wbig.hip)
  bool hs_wbig = false;
  DevBuf Xw;
  // several ranks (one process per GPU, images sharded in contiguous runs, shard()): the
  // d-solve couples every image per frequency (L23:289-295), so each rank forms the Gram of
  // its images (gramchol_big.hip, rho on rank 0 only) and the right-hand sides Z^H xi1 of its
  // images, both are summed over the ranks (allreduce), and every rank factors and solves the
  // same system; the objective's sums, the z change norms and max(b) (L23:36) are reduced too
  bool dist = false;
  int64_t i0 = 0;   // first image of this rank
  double obj = std::numeric_limits<double>::quiet_NaN();
  double obj_filter = obj, obj_z = obj;
  std::vector<double> v_obj_d, v_obj_z, v_tim, tr_od, tr_oz, tr_dd, tr_zd;
  std::vector<int32_t> v_nd, v_nz, v_flags;

  SessionHS(ccsc_ctx* c, const ccsc_problem& pin, const double* b, const double* smooth_init,
            const double* d0, const double* z0)
      : ctx(c), p(pin), st(c->stream) {
    resolve_problem(p);
    if (p.variant != CCSC_HS23) throw Err(CCSC_E_INVALID, "SessionHS runs the 2-3D learner only");
    check_supported(p, &g);
    dist = ctx->nranks > 1 || ctx->rccl_self;
    if (dist && p.K > 192)
      throw Err(CCSC_E_UNSUPPORTED, "the 2-3D learner past K = 192 (the n x n Woodbury factor "
                                    "couples every image) runs on one rank");
    int64_t nloc = p.n;
    shard(p, ctx->rank, ctx->nranks, i0, nloc);
    {
      const char* et = std::getenv("CCSC_DS_TILE");
      hs_dtile = dsolve_tile_ok(p.K, p.views[0]) && !(et && et[0] == '0');
      hs_wbig = p.K > 192;
      if (hs_wbig) hs_dtile = false;
    }
    if (!b || !smooth_init) throw Err(CCSC_E_INVALID, "b and smooth_init must not be NULL");
    G = g.G;
    gp = g.gp;
    m = plan_hs(p, g, nloc, dist);
    r = p.psf / 2;
    s = p.psf;
    SS = s * s;
    K = p.K;
    W = p.views[0];
    KG = K * W;
    P = G.X * G.Y;
    F = G.F;
    sbx = (int)p.sb[0];
    sby = (int)p.sb[1];
    n = (int)nloc;   // this rank's images
    if (r > sbx || r > sby)
      throw Err(CCSC_E_UNSUPPORTED, "symmetric padding wider than the image (L23:19)");

    size_t freeb = 0, totalb = 0;
    HIPCHK(hipMemGetInfo(&freeb, &totalb));
    if (m.total() > freeb)
      throw Err(CCSC_E_NOMEM, "device plan needs " + std::to_string(m.total() >> 20) + " MiB, " +
                                  std::to_string(freeb >> 20) + " MiB free");
    auto tws = make_twiddles(G);
    tw.alloc(tws.size() * sizeof(cpx<double>));
    HIPCHK(hipMemcpy(tw.p, tws.data(), tw.bytes, hipMemcpyHostToDevice));
    if (gp) {
      std::vector<cpx<double>> t1, t2;
      if (!gfft_plan(G.X, G.Y, grg, gcy, t1, t2)) throw Err(CCSC_E_UNSUPPORTED, "no global line plan");
      gtwr.alloc(t1.size() * sizeof(cpx<double>));
      gtwc.alloc(t2.size() * sizeof(cpx<double>));
      HIPCHK(hipMemcpy(gtwr.p, t1.data(), gtwr.bytes, hipMemcpyHostToDevice));
      HIPCHK(hipMemcpy(gtwc.p, t2.data(), gtwc.bytes, hipMemcpyHostToDevice));
      gR.alloc(m.gr);
    }
    const size_t vwn = (size_t)P * W * n, dwk = (size_t)P * KG, zkn = (size_t)P * K * n;
    bdev.alloc(m.b);
    smp.alloc(vwn * 8);
    v.alloc(vwn * 8);
    eD.alloc(vwn * 8);
    eZ.alloc(vwn * 8);
    D.alloc(dwk * 8);
    yD.alloc(dwk * 8);
    Dold.alloc(dwk * 8);
    z.alloc(zkn * 8);
    eZ2.alloc(zkn * 8);
    zold.alloc(zkn * 8);
    Zh.alloc(m.Zh);
    if (m.wx) Xw.alloc(m.wx);
    Xi.alloc(m.Xi);
    Ch.alloc(m.dspec);
    Dh.alloc(m.dspec);
    Dhold.alloc(m.dspec);
    L.alloc(m.L);
    h.alloc(m.h);
    sden.alloc((size_t)F * 8);
    Usup.alloc((size_t)KG * SS * 8);
    supp.alloc((size_t)KG * SS * 8);
    dnorm.alloc((size_t)2 * KG * 8);
    part.alloc((size_t)2 * std::max<int64_t>(std::max<int64_t>((int64_t)W * n, (int64_t)K * n),
                                             kNormParts) * 8);
    pair.alloc(12 * 8);

    // data: b and smoothinit = padarray(smooth_init, [r r 0 0], 'symmetric') (L23:19)
    HIPCHK(hipMemcpy(bdev.p, b, m.b, hipMemcpyHostToDevice));
    {
      DevBuf stage;
      stage.alloc(m.b);
      HIPCHK(hipMemcpy(stage.p, smooth_init, m.b, hipMemcpyHostToDevice));
      HIPCHK(launch_pad_symmetric<double>(stage.as<double>(), smp.as<double>(), sbx, sby, r, G.X,
                                          G.Y, (int64_t)W * n, st));
      HIPCHK(hipStreamSynchronize(st));
    }
    // gammas (L23:35-38): gamma_heuristic = 60 lambda / max(b(:))
    HIPCHK(launch_max<double>(bdev.as<double>(), (int64_t)((size_t)sbx * sby * W * n),
                              part.as<double>(), pair.as<double>(), st));
    double bmax = 0;
    HIPCHK(hipMemcpyAsync(&bmax, pair.p, sizeof(double), hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    if (dist) {   // max over the ranks through the sum collective: one slot per rank
      std::vector<double> mx((size_t)ctx->nranks, 0.0);
      mx[(size_t)ctx->rank] = bmax;
      DevBuf rm;
      rm.alloc(mx.size() * 8);
      HIPCHK(hipMemcpy(rm.p, mx.data(), rm.bytes, hipMemcpyHostToDevice));
      ctx_collective(ctx, st, CCSC_COMM_ALLREDUCE_SUM, rm.as<double>(), mx.size());
      HIPCHK(hipMemcpyAsync(mx.data(), rm.p, rm.bytes, hipMemcpyDeviceToHost, st));
      HIPCHK(hipStreamSynchronize(st));
      bmax = *std::max_element(mx.begin(), mx.end());
    }
    if (!(bmax > 0)) throw Err(CCSC_E_INVALID, "max(b(:)) must be positive (L23:36)");
    gamma_h = 60.0 * p.lambda_prior / bmax;
    const double gD1 = gamma_h / p.rho_d;                // gammas_D = [gh/5000, gh]  (L23:37)
    const double gZ1 = gamma_h * W / p.rho_z;            // gammas_Z = [gh/500, gh]   (L23:38)
    th_D1 = p.lambda_residual / gD1;                     // lambda(1)/gammas_D(1)     (L23:112)
    th_Z1 = p.lambda_residual / gZ1;                     // lambda(1)/gammas_Z(1)     (L23:175)
    th_Z2 = p.lambda_prior / gamma_h;                    // lambda(2)/gammas_Z(2)     (L23:176)

    // filters: d0 [s,s,K] replicated over W, embedded at circshift(-r) (L23:54-56)
    {
      DevBuf d0dev, d0w;
      d0dev.alloc((size_t)SS * K * 8);
      d0w.alloc((size_t)SS * KG * 8);
      if (d0) HIPCHK(hipMemcpy(d0dev.p, d0, d0dev.bytes, hipMemcpyHostToDevice));
      else HIPCHK(launch_randn<double>(d0dev.as<double>(), (int64_t)SS * K, p.seed ^ 0xd0d0d0d0ULL, 0, st));
      HIPCHK(launch_rep_filters<double>(d0dev.as<double>(), d0w.as<double>(), SS, W, K, st));
      HIPCHK(launch_embed_filters<double>(d0w.as<double>(), D.as<double>(), 1, KG, s, G, 1, st));
      HIPCHK(hipStreamSynchronize(st));
    }
    HIPCHK(hipMemsetAsync(yD.p, 0, yD.bytes, st));
    HIPCHK(hipMemsetAsync(eD.p, 0, eD.bytes, st));
    HIPCHK(hipMemsetAsync(eZ.p, 0, eZ.bytes, st));
    HIPCHK(hipMemsetAsync(eZ2.p, 0, eZ2.bytes, st));
    // codes z = randn(size_z) (L23:69)
    if (z0) HIPCHK(hipMemcpy(z.p, z0, z.bytes, hipMemcpyHostToDevice));
    else HIPCHK(launch_randn<double>(z.as<double>(), (int64_t)zkn, p.seed, 0, st));
    // d_hat = fft2(d) (L23:57); u_D{2} of the first d-iteration = Pi(d - 0) (L23:113)
    r2c_full(D.as<double>(), Dh.as<cpx<double>>(), KG);
    HIPCHK(launch_gather_support<double>(D.as<double>(), yD.as<double>(), supp.as<double>(), KG, r,
                                         G.X, G.Y, st));
    HIPCHK(launch_project<double>(supp.as<double>(), Usup.as<double>(), KG, SS, 1.0, st));
    obj = objective_fresh();                              // L23:72
    obj_filter = obj_z = obj;                             // L23:82-83
    v_obj_d.push_back(obj);
    v_obj_z.push_back(obj);
    v_tim.push_back(0.0);
  }

  // ---- slice transforms: the fused LDS slice kernels, or on global-pass slices the line
  // passes of recon.hip around gslice.hip's elementwise halves.  On global passes the
  // inverse consumes its input spectrum (the column pass runs in place): Xi and Zh are dead
  // after their C2R here; Dh is copied to Ch (free between its d-solve and the next dual).
  void g_r2c(const double* src, cpx<double>* dst, int64_t count) {
    RowArgs<double> a{};
    a.S = dst;
    a.src = src;
    a.per_img = 1;
    HIPCHK(launch_rows<double>(kRowFwd, a, count, grg, gtwr.as<cpx<double>>(), st));
    HIPCHK(launch_cols<double>(dst, -1, count, gcy, gtwc.as<cpx<double>>(), st));
  }
  void g_c2r(cpx<double>* src, double* dst, int64_t count) {
    HIPCHK(launch_cols<double>(src, +1, count, gcy, gtwc.as<cpx<double>>(), st));
    RowArgs<double> a{};
    a.S = src;
    a.Z = dst;
    a.per_img = 1;
    HIPCHK(launch_rows<double>(kRowFinalZ, a, count, grg, gtwr.as<cpx<double>>(), st));
  }
  // fft2 of whole real slices (L23:57,100,158,234)
  void r2c_full(const double* src, cpx<double>* dst, int64_t count) {
    if (gp) g_r2c(src, dst, count);
    else
      HIPCHK(launch_r2c_embed<double>(src, P, G.X, G.Y, 0, 0, dst, F, count, tw.as<cpx<double>>(),
                                      G, st));
  }
  // v = real(ifft2(Xi)), DZ (nullable), the objective's data parts (k_hs_c2r_v)
  void c2r_v(double* DZ) {
    const int64_t cnt = (int64_t)W * n;
    if (!gp) {
      HIPCHK(launch_hs_c2r_v<double>(Xi.as<cpx<double>>(), v.as<double>(), bdev.as<double>(),
                                     smp.as<double>(), DZ, part.as<double>(), cnt,
                                     tw.as<cpx<double>>(), G, r, sbx, sby, st));
      return;
    }
    g_c2r(Xi.as<cpx<double>>(), gR.as<double>(), cnt);
    HIPCHK(launch_gp_hs_epilog<double>(kHsV, gR.as<double>(), v.as<double>(), bdev.as<double>(),
                                       smp.as<double>(), DZ, part.as<double>(), G.X, G.Y, r, sbx,
                                       sby, 1.0 / (double)P, cnt, st));
  }
  // masked-data split with dual e, into Xi (k_hs_data_r2c)
  void data_r2c(DevBuf& e, double theta) {
    const int64_t cnt = (int64_t)W * n;
    if (!gp) {
      HIPCHK(launch_hs_data_r2c<double>(v.as<double>(), e.as<double>(), bdev.as<double>(),
                                        smp.as<double>(), Xi.as<cpx<double>>(), cnt,
                                        tw.as<cpx<double>>(), G, r, sbx, sby, theta, st));
      return;
    }
    HIPCHK(launch_gp_hs_prolog<double>(kHsData, v.as<double>(), e.as<double>(), bdev.as<double>(),
                                       smp.as<double>(), gR.as<double>(), G.X, G.Y, r, sbx, sby,
                                       theta, cnt, st));
    g_r2c(gR.as<double>(), Xi.as<cpx<double>>(), cnt);
  }
  // kernel-constraint split of the D-phase, into Ch (k_dual_r2c)
  void dual_r2c() {
    if (!gp) {
      HIPCHK(launch_dual_r2c<double>(D.as<double>(), yD.as<double>(), Usup.as<double>(),
                                     Ch.as<cpx<double>>(), KG, tw.as<cpx<double>>(), G, KG, r, st));
      return;
    }
    HIPCHK(launch_gp_prolog<double>(2, D.as<double>(), yD.as<double>(), Usup.as<double>(), 0, 0, 0,
                                    0.0, KG, r, gR.as<double>(), G.X, G.Y, KG, st));
    g_r2c(gR.as<double>(), Ch.as<cpx<double>>(), KG);
  }
  // d = real(ifft2(d_hat)), the support of d + y (k_c2r_dout); Dh stays intact
  void c2r_dout() {
    if (!gp) {
      HIPCHK(launch_c2r_dout<double>(Dh.as<cpx<double>>(), D.as<double>(), yD.as<double>(),
                                     supp.as<double>(), dnorm.as<double>(), 0, KG,
                                     tw.as<cpx<double>>(), G, r, st));
      return;
    }
    HIPCHK(hipMemcpyAsync(Ch.p, Dh.p, Dh.bytes, hipMemcpyDeviceToDevice, st));
    g_c2r(Ch.as<cpx<double>>(), gR.as<double>(), KG);
    HIPCHK(launch_gp_epilog<double>(2, gR.as<double>(), D.as<double>(), yD.as<double>(),
                                    supp.as<double>(), dnorm.as<double>(), 0, 1.0 / (double)P, r,
                                    G.X, G.Y, KG, nullptr, 0.0, 0, st));
  }
  // sparsity split of the Z-phase with dual eZ2, into Zh (k_hs_z_r2c)
  void z_r2c() {
    const int64_t cnt = (int64_t)K * n;
    if (!gp) {
      HIPCHK(launch_hs_z_r2c<double>(z.as<double>(), eZ2.as<double>(), Zh.as<cpx<double>>(), cnt,
                                     tw.as<cpx<double>>(), G, th_Z2, st));
      return;
    }
    HIPCHK(launch_gp_hs_prolog<double>(kHsSparse, z.as<double>(), eZ2.as<double>(),
                                       bdev.as<double>(), smp.as<double>(), gR.as<double>(), G.X,
                                       G.Y, r, sbx, sby, th_Z2, cnt, st));
    g_r2c(gR.as<double>(), Zh.as<cpx<double>>(), cnt);
  }
  // z = real(ifft2(zhat)), sum |z| per slice (k_hs_c2r_z)
  void c2r_z() {
    const int64_t cnt = (int64_t)K * n;
    if (!gp) {
      HIPCHK(launch_hs_c2r_z<double>(Zh.as<cpx<double>>(), z.as<double>(), part.as<double>(), cnt,
                                     tw.as<cpx<double>>(), G, st));
      return;
    }
    g_c2r(Zh.as<cpx<double>>(), gR.as<double>(), cnt);
    HIPCHK(launch_gp_hs_epilog<double>(kHsZ, gR.as<double>(), z.as<double>(), bdev.as<double>(),
                                       smp.as<double>(), nullptr, part.as<double>(), G.X, G.Y, r,
                                       sbx, sby, 1.0 / (double)P, cnt, st));
  }
  // D = real(ifft2(Dh)) (the rollback); Dh stays intact
  void c2r_plain_D() {
    if (!gp) {
      HIPCHK(launch_c2r_plain<double>(Dh.as<cpx<double>>(), F, D.as<double>(), P, KG,
                                      tw.as<cpx<double>>(), G, 1.0 / (double)P, st));
      return;
    }
    HIPCHK(hipMemcpyAsync(Ch.p, Dh.p, Dh.bytes, hipMemcpyDeviceToDevice, st));
    g_c2r(Ch.as<cpx<double>>(), gR.as<double>(), KG);
    HIPCHK(launch_gp_epilog<double>(0, gR.as<double>(), D.as<double>(), nullptr, nullptr, nullptr,
                                    0, 1.0 / (double)P, r, G.X, G.Y, KG, nullptr, 0.0, 0, st));
  }

  // v = real(ifft2(H zhat)) from Xi (= H zhat) and the objective of (z, d_hat)
  // (objectiveFunction, L23:326-343); pair[2] must hold sum |z|.
  double finish_objective() {
    c2r_v(nullptr);
    HIPCHK(launch_sum_pairs<double>(part.as<double>(), W * n, pair.as<double>(), st));
    // the data term and sum |z| over every rank's images, reduced in a copy: pair[2] (this
    // rank's sum |z|) serves every objective of a d-phase
    const double* ps = pair.as<double>();
    if (dist) {
      HIPCHK(hipMemcpyAsync(pair.as<double>() + 8, ps, 4 * sizeof(double), hipMemcpyDeviceToDevice, st));
      ctx_collective(ctx, st, CCSC_COMM_ALLREDUCE_SUM, pair.as<double>() + 8, 4);
      ps = pair.as<double>() + 8;
    }
    double h4[4];
    HIPCHK(hipMemcpyAsync(h4, ps, sizeof h4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    return p.lambda_residual * 0.5 * h4[0] + p.lambda_prior * W * h4[2];   // g_z: z repeated W times (L23:332,338)
  }
  // zhat = fft2(z) (L23:100,158,234), sum |z|, v = H z and the objective
  double objective_fresh() {
    r2c_full(z.as<double>(), Zh.as<cpx<double>>(), (int64_t)K * n);
    HIPCHK(launch_norms<double>(z.as<double>(), nullptr, (int64_t)z.bytes / 8, part.as<double>(),
                                pair.as<double>() + 2, st));
    HIPCHK(launch_hs_synth<double>(Dh.as<cpx<double>>(), Zh.as<cpx<double>>(),
                                   Xi.as<cpx<double>>(), F, W, K, n, st));
    return finish_objective();
  }
  // global: a and b are rank-local (z; D is the same on every rank)
  double rel_change(const DevBuf& a, const DevBuf& b, bool global = false) {
    HIPCHK(launch_norms<double>(a.as<double>(), b.as<double>(), (int64_t)a.bytes / 8,
                                part.as<double>(), pair.as<double>() + 4, st));
    if (global && dist) ctx_collective(ctx, st, CCSC_COMM_ALLREDUCE_SUM, pair.as<double>() + 4, 2);
    double h2[2];
    HIPCHK(hipMemcpyAsync(h2, pair.as<double>() + 4, sizeof h2, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    return std::sqrt(h2[0]) / std::sqrt(h2[1]);
  }

  void ensure_trace_capacity(int total_outer) {
    const double nan = std::numeric_limits<double>::quiet_NaN();
    const size_t nd = (size_t)total_outer * p.max_it_d, nz = (size_t)total_outer * p.max_it_z;
    if (tr_od.size() < nd) tr_od.resize(nd, nan);
    if (tr_dd.size() < nd) tr_dd.resize(nd, nan);
    if (tr_oz.size() < nz) tr_oz.resize(nz, nan);
    if (tr_zd.size() < nz) tr_zd.resize(nz, nan);
  }

  // ---- one outer iteration (L23:86-226) ---------------------------------------
  void outer_iteration() {
    const int it = outer_done;
    const auto t0 = std::chrono::steady_clock::now();
    const double obj_min = std::min(obj_filter, obj_z);   // L23:94
    HIPCHK(hipMemcpyAsync(Dold.p, D.p, D.bytes, hipMemcpyDeviceToDevice, st));    // d_old (L23:95)
    HIPCHK(hipMemcpyAsync(Dhold.p, Dh.p, Dh.bytes, hipMemcpyDeviceToDevice, st)); // d_hat_old
    // z_hat = fft2(z) (L23:100) and v_D{1} = H z of the first d-iteration (L23:108)
    objective_fresh();
    // opt_f = (Z_f' Z_f + rho I)^-1 as a Cholesky factor per bin (L23:290)
    // on the matrix cores (gramchol.hip, K <= 192; no right-hand side here: NV = 0)
    if (hs_wbig) {
      HIPCHK(launch_wbig_gram(Zh.as<cpx<double>>(), Zh.as<cpx<double>>(), Xw.as<cpx<double>>(),
                              L.as<cpx<double>>(), h.as<cpx<double>>(), F, K, n, p.rho_d, 0, st));
    } else if (dist) {
      // the Gram of this rank's images (rho I on rank 0 only), summed over the ranks, then
      // the same Cholesky on every rank
      HIPCHK(launch_gram_big(Zh.as<cpx<double>>(), Zh.as<cpx<double>>(), Xw.as<cpx<double>>(),
                             L.as<cpx<double>>(), h.as<cpx<double>>(), F, K, n,
                             ctx->rank == 0 ? p.rho_d : 0.0, 0, st, false));
      ctx_collective(ctx, st, CCSC_COMM_ALLREDUCE_SUM, L.as<double>(),
                     (size_t)2 * F * (K * (K + 1) / 2));
      HIPCHK(launch_chol_big(L.as<cpx<double>>(), F, K, st));
    } else
      HIPCHK(launch_gram_chol_mf(Zh.as<cpx<double>>(), Zh.as<cpx<double>>(), L.as<cpx<double>>(),
                                 h.as<cpx<double>>(), F, K, n, p.rho_d, 0, st));
    // 64 < K <= 112: the tile d-solve over the W wavelengths (factor read once per solve)
    if (hs_dtile) HIPCHK(launch_invert_diag(L.as<cpx<double>>(), F, K, st));
    for (int id = 0; id < p.max_it_d; ++id) {                                    // L23:102
      // c = 1: masked data split (L23:112, 117, 120-121)
      data_r2c(eD, th_D1);
      // c = 2: kernel constraint split, y = -d_D{2} (L23:113, 117, 120-121)
      dual_r2c();
      // d_hat = opt (Z' xi1 + rho xi2) per (bin, wavelength)  (L23:125, 289-295)
      HIPCHK(launch_hs_corr<double>(Zh.as<cpx<double>>(), Xi.as<cpx<double>>(),
                                    h.as<cpx<double>>(), F, W, K, n, st));
      if (dist) ctx_collective(ctx, st, CCSC_COMM_ALLREDUCE_SUM, h.as<double>(), (size_t)2 * F * W * K);
      if (hs_wbig)
        HIPCHK(launch_wbig_solve(L.as<cpx<double>>(), h.as<cpx<double>>(), Ch.as<cpx<double>>(),
                                 Dh.as<cpx<double>>(), 1, F, K, n, p.rho_d, W, st));
      else if (hs_dtile)
        HIPCHK(launch_dsolve_tile(L.as<cpx<double>>(), h.as<cpx<double>>(), Ch.as<cpx<double>>(),
                                  Dh.as<cpx<double>>(), 1, F, K, p.rho_d, W, st));
      else
        HIPCHK(launch_dsolve<double>(L.as<cpx<double>>(), h.as<cpx<double>>(), Ch.as<cpx<double>>(),
                                     Dh.as<cpx<double>>(), 1, F, K, p.rho_d, W, st));
      // d = real(ifft2(d_hat)) (L23:126); support of d - d_D{2} -> u_D{2} of the next d-iteration
      c2r_dout();
      HIPCHK(launch_project<double>(supp.as<double>(), Usup.as<double>(), KG, SS, 1.0, st));
      // objective (L23:132); its H z is v_D{1} of the next d-iteration (z is fixed here)
      HIPCHK(launch_hs_synth<double>(Dh.as<cpx<double>>(), Zh.as<cpx<double>>(),
                                     Xi.as<cpx<double>>(), F, W, K, n, st));
      obj = finish_objective();
      tr_od[(size_t)it * p.max_it_d + id] = obj;
    }
    obj_filter = obj;                                                            // L23:139
    const double d_diff = rel_change(D, Dold);                                   // L23:142-146
    tr_dd[(size_t)it * p.max_it_d] = d_diff;

    // ---- Z-phase (L23:149-200) ----
    // 1 / (rho + sum_{w,k} |d_hat|^2) per bin (L23:262-268, 317)
    HIPCHK(launch_sden<double>(Dh.as<cpx<double>>(), sden.as<double>(), F, KG, p.rho_z, 1.0, st));
    HIPCHK(hipMemcpyAsync(zold.p, z.p, z.bytes, hipMemcpyDeviceToDevice, st));  // z_old (L23:159)
    // v = H z is current: the last D objective used z_hat = fft2(z) (L23:158)
    for (int iz = 0; iz < p.max_it_z; ++iz) {                                    // L23:165
      data_r2c(eZ, th_Z1);                                                       // L23:175,180,183-184
      z_r2c();                                                                   // L23:176,180,183-184
      HIPCHK(launch_hs_analysis<double>(Dh.as<cpx<double>>(), Xi.as<cpx<double>>(),
                                        Zh.as<cpx<double>>(), sden.as<double>(), p.rho_z,
                                        Zh.as<cpx<double>>(), F, W, K, n, st));  // L23:188, 302-324
      // objective (L23:195); H zhat is v_Z{1} of the next z-iteration (L23:171) -- formed
      // before the C2R of zhat, which consumes Zh on global-pass slices
      HIPCHK(launch_hs_synth<double>(Dh.as<cpx<double>>(), Zh.as<cpx<double>>(),
                                     Xi.as<cpx<double>>(), F, W, K, n, st));
      c2r_z();                                                                   // L23:189
      HIPCHK(launch_sum_pairs<double>(part.as<double>(), K * n, pair.as<double>() + 2, st));
      obj = finish_objective();
      tr_oz[(size_t)it * p.max_it_z + iz] = obj;
    }
    obj_z = obj;                                                                 // L23:202
    int flags = 0;
    if (obj_min <= obj_filter && obj_min <= obj_z) {                             // L23:204-213 (Q16)
      // roll back to the iterate before this outer iteration and stop
      HIPCHK(hipMemcpyAsync(z.p, zold.p, z.bytes, hipMemcpyDeviceToDevice, st));
      HIPCHK(hipMemcpyAsync(Dh.p, Dhold.p, Dh.bytes, hipMemcpyDeviceToDevice, st));
      c2r_plain_D();
      obj = objective_fresh();
      finished = true;
      flags |= 1;
    } else {
      const double z_diff = rel_change(z, zold, true);                           // L23:216-220
      tr_zd[(size_t)it * p.max_it_z] = z_diff;
      if (z_diff < p.tol && d_diff < p.tol) finished = true;                     // L23:223
    }
    HIPCHK(hipStreamSynchronize(st));
    const double secs =
        std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    v_obj_d.push_back(obj_filter);
    v_obj_z.push_back(obj_z);
    v_tim.push_back(v_tim.back() + secs);
    v_nd.push_back(p.max_it_d);
    v_nz.push_back(p.max_it_z);
    v_flags.push_back(flags);
    ++outer_done;
  }

  void step(int n_outer, int32_t* done) {
    ensure_trace_capacity(outer_done + n_outer);
    for (int i = 0; i < n_outer && !finished; ++i) outer_iteration();
    if (done) *done = finished ? 1 : 0;
  }

  void results(ccsc_outputs* out) {
    if (!out) return;
    if (out->d_res) {
      // d_res = circshift(d, [r r 0 0])(1:2r+1, 1:2r+1, :, :)  (L23:231-232)
      std::vector<double> Dh_((size_t)KG * P);
      HIPCHK(hipMemcpy(Dh_.data(), D.p, D.bytes, hipMemcpyDeviceToHost));
      for (int gI = 0; gI < KG; ++gI)
        for (int j = 0; j < s; ++j)
          for (int i = 0; i < s; ++i) {
            const int x = (i - r + G.X) % G.X, y = (j - r + G.Y) % G.Y;
            out->d_res[i + (size_t)s * (j + (size_t)s * gI)] = Dh_[(size_t)gI * P + (size_t)y * G.X + x];
          }
    }
    if (out->z_res) HIPCHK(hipMemcpy(out->z_res, z.p, z.bytes, hipMemcpyDeviceToHost));
    if (out->DZ) {
      // Dz = real(ifft2(sum_k d_hat .* fft2(z))) + smoothinit  (L23:234-235)
      DevBuf dz;
      dz.alloc(v.bytes);
      r2c_full(z.as<double>(), Zh.as<cpx<double>>(), (int64_t)K * n);
      HIPCHK(launch_hs_synth<double>(Dh.as<cpx<double>>(), Zh.as<cpx<double>>(),
                                     Xi.as<cpx<double>>(), F, W, K, n, st));
      c2r_v(dz.as<double>());
      HIPCHK(hipStreamSynchronize(st));   // st is non-blocking: hipMemcpy does not order after it
      HIPCHK(hipMemcpy(out->DZ, dz.p, dz.bytes, hipMemcpyDeviceToHost));
    }
    if (out->obj_val) *out->obj_val = obj;   // the last objective the learner evaluated
  }

  void iterlog(ccsc_iterlog* lg) {
    if (!lg) return;
    const int cnt = std::min<int>(lg->capacity, (int)v_tim.size());
    lg->count = cnt;
    for (int i = 0; i < cnt; ++i) {
      if (lg->obj_vals_d) lg->obj_vals_d[i] = v_obj_d[i];
      if (lg->obj_vals_z) lg->obj_vals_z[i] = v_obj_z[i];
      if (lg->tim_vals) lg->tim_vals[i] = v_tim[i];
    }
    const int no = std::min<int>(lg->capacity, outer_done);
    for (int i = 0; i < no; ++i) {
      if (lg->n_d) lg->n_d[i] = v_nd[i];
      if (lg->n_z) lg->n_z[i] = v_nz[i];
      if (lg->flags) lg->flags[i] = v_flags[i];
      for (int t = 0; t < p.max_it_d; ++t) {
        const size_t q = (size_t)i * p.max_it_d + t;
        if (lg->trace_obj_d) lg->trace_obj_d[q] = q < tr_od.size() ? tr_od[q] : NAN;
        if (lg->trace_d_diff) lg->trace_d_diff[q] = q < tr_dd.size() ? tr_dd[q] : NAN;
      }
      for (int t = 0; t < p.max_it_z; ++t) {
        const size_t q = (size_t)i * p.max_it_z + t;
        if (lg->trace_obj_z) lg->trace_obj_z[q] = q < tr_oz.size() ? tr_oz[q] : NAN;
        if (lg->trace_z_diff) lg->trace_z_diff[q] = q < tr_zd.size() ? tr_zd[q] : NAN;
      }
    }
  }
};

}  // namespace ccsc

struct ccsc_session {
  std::unique_ptr<ccsc::Session2D> s2;
  std::unique_ptr<ccsc::SessionHS> hs;
  ccsc_ctx* ctx() const { return s2 ? s2->ctx : hs->ctx; }
};

namespace ccsc {
// One rank of a multi-device context failed: mark the group aborted (once, whichever
// threads fail), wake the in-process exchange, wait until no rank is inside a collective
// call, then abort every RCCL communicator so the other ranks' kernels waiting on the
// failed rank return (see CommGroup).  The wait has no time limit and needs none: the
// group's communicators are non-blocking (init_group_comms), so an enqueue returns at
// once and collective()'s poll loop leaves as soon as `aborted` is set -- a communicator
// is never aborted (freed) while another thread is inside RCCL with it, and a rank that
// enters collective() later sees `aborted` (set before the wait) before it reads `comm`.
static void abort_group(ccsc_ctx* ctx) {
  CommGroup* g = ctx->grp.get();
  std::lock_guard<std::mutex> lk(g->mu);
  if (g->aborted.exchange(true)) return;
  if (ctx->hg) ctx->hg->abort();
  while (g->inflight.load() > 0) std::this_thread::sleep_for(std::chrono::microseconds(50));
  for (ccsc_ctx* u : ctx->subs)
    if (u->comm) {
      ncclCommAbort(u->comm);
      u->comm = nullptr;
    }
}

// Before a learn on a multi-device context whose previous learn failed: fresh
// communicators (RCCL: ncclCommInitAll over the device list; repeated devices: a new
// in-process exchange), so a failure does not leave the (MEX-cached) context unusable.
static void reset_group(ccsc_ctx* ctx) {
  CommGroup* g = ctx->grp.get();
  if (!g || !g->aborted.load()) return;
  std::lock_guard<std::mutex> lk(g->mu);
  const int nd = (int)ctx->subs.size();
  if (ctx->hg) {
    ctx->hg.reset(new HostGroup(nd));
    for (int i = 0; i < nd; ++i) ctx->hg_ranks[i] = HostGroupRank{ctx->hg.get(), i};
  } else {
    std::vector<ncclComm_t> comms(nd, nullptr);
    init_group_comms(comms, ctx->devices.data(), nd);
    for (int i = 0; i < nd; ++i) ctx->subs[i]->comm = comms[i];
    HIPCHK(hipSetDevice(ctx->device));
  }
  g->aborted.store(false);
}

// Test-only fault injection (failure detection): CCSC_TEST_FAIL_RANK =
// "rank:outer" makes that rank of a multi-device learn throw before outer iteration
// `outer`, while the other ranks run into their next collective.
static bool injected_fault(int rank, int outer) {
  const char* ev = std::getenv("CCSC_TEST_FAIL_RANK");
  int r = -1, o = -1;
  return ev && std::sscanf(ev, "%d:%d", &r, &o) == 2 && r == rank && o == outer;
}

// ccsc_learn on a multi-device context: the caller's whole problem (b, z0, outputs
// over all n patches) is split at the block boundaries of ccsc_shard; rank i runs
// on sub-context i in its own host thread, the calling thread drives rank 0 and is
// the only one that calls back (include/ccsc.h threading rule).  Collectives
// inside the sessions (RCCL, or the in-process exchange) keep the ranks in step.
static void learn_group(ccsc_ctx* ctx, const ccsc_problem& pin, const double* b, const double* d0,
                        const double* z0, ccsc_outputs* out, ccsc_iterlog* log, ccsc_cb cb,
                        void* user) {
  reset_group(ctx);
  ccsc_problem q = pin;
  resolve_problem(q);
  Geom g;
  check_supported(q, &g);
  const int nd = (int)ctx->subs.size();
  const bool is4 = q.variant == CCSC_L4D, is3 = q.variant == CCSC_L3D;
  const int64_t NV = (int64_t)q.views[0] * q.views[1];
  const int64_t bpatch = q.sb[0] * q.sb[1] * (is3 ? q.sb[2] : 1) * NV;   // b [sb.., (U,V), n]
  const int64_t zpatch = (int64_t)q.K * (int64_t)g.P();                  // z [X,Y,(T),K, n]
  const int64_t xpatch = is4 ? NV * q.sb[0] * q.sb[1] : (int64_t)g.P();  // DZ per patch
  const int64_t KG = (int64_t)q.K * NV;
  const int64_t SS = (int64_t)q.psf * q.psf * (is3 ? q.psf : 1);
  std::vector<std::vector<double>> dscr(nd), oscr(nd);
  std::vector<std::string> errs(nd);
  std::vector<int> codes(nd, CCSC_OK);
  auto run = [&](int i) {
    // the session outlives the catch: a failed rank aborts the group BEFORE its stream is
    // drained, so no rank waits on a collective whose peer has stopped
    std::unique_ptr<Session2D> Sp;
    try {
      ccsc_ctx* u = ctx->subs[i];
      HIPCHK(hipSetDevice(u->device));
      int64_t b0 = 0, nb = 0;
      shard(q, i, nd, b0, nb);
      const int64_t p0 = b0 * q.ni;
      const double* zi = z0 ? (q.variant == CCSC_DZPAR ? z0 : z0 + p0 * zpatch) : nullptr;
      Sp.reset(new Session2D(u, q, b + p0 * bpatch, d0, zi));
      Session2D& S = *Sp;
      S.ensure_trace_capacity(S.p.max_it);
      for (int it = 0; it < S.p.max_it && !S.finished; ++it) {
        if (injected_fault(i, it))
          throw Err(CCSC_E_INVALID, "injected fault (CCSC_TEST_FAIL_RANK) before outer iteration " +
                                        std::to_string(it));
        S.outer_iteration();
        if (i == 0 && cb) cb(user, S.outer_done, S.v_obj_d.back(), S.v_obj_z.back(), S.v_tim.back());
      }
      ccsc_outputs o{};
      if (out) {
        // d_res and obj_val are collectives: every rank asks when the caller does
        if (out->d_res) {
          dscr[i].resize(i == 0 ? 0 : (size_t)(KG * SS));
          o.d_res = i == 0 ? out->d_res : dscr[i].data();
        }
        if (out->obj_val) {
          oscr[i].resize(1);
          o.obj_val = i == 0 ? out->obj_val : oscr[i].data();
        }
        if (out->z_res) o.z_res = out->z_res + p0 * zpatch;
        if (out->DZ) o.DZ = out->DZ + p0 * xpatch;
      }
      S.results(out ? &o : nullptr);
      if (i == 0) S.iterlog(log);
    } catch (const Err& e) {
      errs[i] = e.what();
      codes[i] = e.code;
      abort_group(ctx);
    } catch (const std::exception& e) {
      errs[i] = e.what();
      codes[i] = CCSC_E_INVALID;
      abort_group(ctx);
    }
    try {
      Sp.reset();
    } catch (...) {
    }
  };
  std::vector<std::thread> th;
  for (int i = 1; i < nd; ++i) th.emplace_back(run, i);
  run(0);
  for (auto& t : th) t.join();
  HIPCHK(hipSetDevice(ctx->device));
  for (int i = 0; i < nd; ++i)   // the first failure (others are its consequences)
    if (codes[i] != CCSC_OK && !errs[i].empty() && errs[i].find("host communicator") == std::string::npos)
      throw Err(codes[i], "device " + std::to_string(ctx->subs[i]->device) + " (rank " +
                              std::to_string(i) + "): " + errs[i]);
  for (int i = 0; i < nd; ++i)
    if (codes[i] != CCSC_OK) throw Err(codes[i], "rank " + std::to_string(i) + ": " + errs[i]);
}
}  // namespace ccsc

// ===========================================================================
// C-ABI
// ===========================================================================
extern "C" {

int32_t ccsc_abi_version(void) { return CCSC_ABI_VERSION; }

int32_t ccsc_resolve(ccsc_problem* p, char* err, size_t errlen) {
  return guarded(err, errlen, [&] {
    if (!p) throw Err(CCSC_E_INVALID, "problem is NULL");
    resolve_problem(*p);
  });
}

int32_t ccsc_supported(const ccsc_problem* p, char* err, size_t errlen) {
  return guarded(err, errlen, [&] {
    if (!p) throw Err(CCSC_E_INVALID, "problem is NULL");
    ccsc_problem q = *p;
    resolve_problem(q);
    check_supported(q, nullptr);
  });
}

int32_t ccsc_shard(const ccsc_problem* p, int32_t rank, int32_t nranks, int64_t* block_begin,
                   int64_t* block_count, char* err, size_t errlen) {
  return guarded(err, errlen, [&] {
    if (!p || !block_begin || !block_count) throw Err(CCSC_E_INVALID, "NULL argument");
    ccsc_problem q = *p;
    resolve_problem(q);
    shard(q, rank, nranks, *block_begin, *block_count);
  });
}

int32_t ccsc_plan_bytes(const ccsc_problem* p, int32_t rank, int32_t nranks, uint64_t* bytes,
                        char* err, size_t errlen) {
  return guarded(err, errlen, [&] {
    if (!p || !bytes) throw Err(CCSC_E_INVALID, "NULL argument");
    ccsc_problem q = *p;
    resolve_problem(q);
    Geom g;
    check_supported(q, &g);
    if (q.variant == CCSC_HS23) {
      int64_t i0 = 0, nl = 0;
      shard(q, rank, nranks, i0, nl);
      *bytes = plan_hs(q, g, nl, nranks > 1).total();
    } else {
      *bytes = plan2d(q, g, rank, nranks).total();
    }
  });
}

int32_t ccsc_device_count(int32_t* count, char* err, size_t errlen) {
  return guarded(err, errlen, [&] {
    int c = 0;
    HIPCHK(hipGetDeviceCount(&c));
    *count = c;
  });
}

int32_t ccsc_get_unique_id(uint8_t* uid128, char* err, size_t errlen) {
  return guarded(err, errlen, [&] {
    static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
    ncclUniqueId id;
    NCCLCHK(ncclGetUniqueId(&id));
    std::memcpy(uid128, &id, 128);
  });
}

ccsc_ctx* ccsc_create(int32_t device, int32_t rank, int32_t nranks, const uint8_t* uid128,
                      char* err, size_t errlen) {
  ccsc_ctx* ctx = nullptr;
  const int rc = guarded(err, errlen, [&] {
    if (nranks < 1 || rank < 0 || rank >= nranks) throw Err(CCSC_E_INVALID, "bad rank/nranks");
    std::unique_ptr<ccsc_ctx> c(new ccsc_ctx());
    c->device = device;
    c->rank = rank;
    c->nranks = nranks;
    HIPCHK(hipSetDevice(device));
    HIPCHK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    if (nranks > 1) {
      if (!uid128) throw Err(CCSC_E_INVALID, "multi-rank context needs the RCCL unique id");
      ncclUniqueId id;
      std::memcpy(&id, uid128, 128);
      NCCLCHK(ncclCommInitRank(&c->comm, nranks, id, rank));
    }
    ctx = c.release();
  });
  return rc == CCSC_OK ? ctx : nullptr;
}

ccsc_ctx* ccsc_create_hostcomm(int32_t device, int32_t rank, int32_t nranks, ccsc_comm_fn fn,
                               void* user, char* err, size_t errlen) {
  ccsc_ctx* ctx = nullptr;
  const int rc = guarded(err, errlen, [&] {
    if (nranks < 1 || rank < 0 || rank >= nranks) throw Err(CCSC_E_INVALID, "bad rank/nranks");
    if (nranks > 1 && !fn) throw Err(CCSC_E_INVALID, "host communicator needs a callback");
    std::unique_ptr<ccsc_ctx> c(new ccsc_ctx());
    c->device = device;
    c->rank = rank;
    c->nranks = nranks;
    c->hostfn = fn;
    c->hostuser = user;
    HIPCHK(hipSetDevice(device));
    HIPCHK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    ctx = c.release();
  });
  return rc == CCSC_OK ? ctx : nullptr;
}

ccsc_ctx* ccsc_create_multi(const int32_t* devices, int32_t ndev, char* err, size_t errlen) {
  ccsc_ctx* ctx = nullptr;
  const int rc = guarded(err, errlen, [&] {
    if (!devices || ndev < 1) throw Err(CCSC_E_INVALID, "empty device list");
    int count = 0;
    HIPCHK(hipGetDeviceCount(&count));
    for (int i = 0; i < ndev; ++i)
      if (devices[i] < 0 || devices[i] >= count)
        throw Err(CCSC_E_INVALID, "device " + std::to_string(devices[i]) + " out of range (" +
                                      std::to_string(count) + " visible)");
    // every object is owned by `c` (subs, their streams and communicators) the moment it
    // exists, so an error at any step releases all of it through ccsc_destroy
    struct Guard {
      ccsc_ctx* c;
      ~Guard() {
        if (c) ccsc_destroy(c);
      }
    } guard{new ccsc_ctx()};
    ccsc_ctx* c = guard.c;
    c->device = devices[0];
    c->nranks = ndev;
    c->devices.assign(devices, devices + ndev);
    HIPCHK(hipSetDevice(devices[0]));
    HIPCHK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    const char* self_ev = std::getenv("CCSC_TEST_RCCL_SELF");
    const bool rccl_self = ndev == 1 && self_ev && std::atoi(self_ev) != 0;
    if (ndev > 1 || rccl_self) {
      bool distinct = true;
      for (int i = 0; i < ndev; ++i)
        for (int j = 0; j < i; ++j) distinct = distinct && devices[i] != devices[j];
      c->grp = std::make_shared<CommGroup>();
      if (!distinct) {
        c->hg.reset(new HostGroup(ndev));
        c->hg_ranks.resize(ndev);
      }
      for (int i = 0; i < ndev; ++i) {
        c->subs.push_back(new ccsc_ctx());
        ccsc_ctx* u = c->subs.back();
        u->device = devices[i];
        u->rank = i;
        u->nranks = ndev;
        u->rccl_self = rccl_self;
        u->grp = c->grp;
        if (c->hg) {
          c->hg_ranks[i] = HostGroupRank{c->hg.get(), i};
          u->hostfn = host_group_fn;
          u->hostuser = &c->hg_ranks[i];
        }
      }
      if (distinct) {
        std::vector<ncclComm_t> comms(ndev, nullptr);
        init_group_comms(comms, devices, ndev);
        for (int i = 0; i < ndev; ++i) c->subs[i]->comm = comms[i];
      }
      for (int i = 0; i < ndev; ++i) {
        HIPCHK(hipSetDevice(devices[i]));
        HIPCHK(hipStreamCreateWithFlags(&c->subs[i]->stream, hipStreamNonBlocking));
      }
      HIPCHK(hipSetDevice(devices[0]));
    }
    ctx = c;
    guard.c = nullptr;
  });
  return rc == CCSC_OK ? ctx : nullptr;
}

int32_t ccsc_comm_ranks(ccsc_ctx* ctx, int32_t* ranks, int32_t* transport, char* err,
                        size_t errlen) {
  return guarded(err, errlen, [&] {
    if (!ctx || !ranks) throw Err(CCSC_E_INVALID, "NULL argument");
    // a multi-device context reports the communicator of its rank 0
    const ccsc_ctx* u = ctx->subs.empty() ? ctx : ctx->subs[0];
    int32_t t = CCSC_TRANSPORT_NONE, n = 1;
    if (u->nranks > 1 && u->hostfn) {
      t = CCSC_TRANSPORT_HOST;
      n = u->nranks;
    } else if (u->nranks > 1 || u->rccl_self) {
      if (!u->comm) throw Err(CCSC_E_STATE, "the communicator was aborted (a rank failed)");
      int c = 0;
      NCCLCHK(ncclCommCount(u->comm, &c));
      t = CCSC_TRANSPORT_RCCL;
      n = c;
    }
    *ranks = n;
    if (transport) *transport = t;
  });
}

void ccsc_destroy(ccsc_ctx* ctx) {
  if (!ctx) return;
  for (ccsc_ctx* u : ctx->subs) ccsc_destroy(u);
  ctx->subs.clear();
  hipSetDevice(ctx->device);
  if (ctx->stream) hipStreamSynchronize(ctx->stream);
  if (ctx->comm) ncclCommDestroy(ctx->comm);
  if (ctx->stream) hipStreamDestroy(ctx->stream);
  delete ctx;
}

ccsc_session* ccsc_session_create(ccsc_ctx* ctx, const ccsc_problem* p, const double* b,
                                  const double* d0, const double* z0, char* err, size_t errlen) {
  ccsc_session* out = nullptr;
  guarded(err, errlen, [&] {
    if (!ctx || !p) throw Err(CCSC_E_INVALID, "NULL ctx/problem");
    if (p->variant == CCSC_HS23)
      throw Err(CCSC_E_INVALID, "the 2-3D learner takes smooth_init: use ccsc_session_create_hs23");
    if (!ctx->subs.empty())
      throw Err(CCSC_E_UNSUPPORTED, "sessions run on a one-device context (one per rank); a "
                                    "multi-device context serves ccsc_learn");
    HIPCHK(hipSetDevice(ctx->device));
    std::unique_ptr<ccsc_session> s(new ccsc_session());
    s->s2.reset(new Session2D(ctx, *p, b, d0, z0));
    out = s.release();
  });
  return out;
}

ccsc_session* ccsc_session_create_hs23(ccsc_ctx* ctx, const ccsc_problem* p, const double* b,
                                       const double* smooth_init, const double* d0,
                                       const double* z0, char* err, size_t errlen) {
  ccsc_session* out = nullptr;
  guarded(err, errlen, [&] {
    if (!ctx || !p) throw Err(CCSC_E_INVALID, "NULL ctx/problem");
    if (!ctx->subs.empty())
      throw Err(CCSC_E_UNSUPPORTED, "the 2-3D learner runs one process per GPU (a rank context of "
                                    "ccsc_create / ccsc_create_hostcomm), not on a device list");
    HIPCHK(hipSetDevice(ctx->device));
    std::unique_ptr<ccsc_session> s(new ccsc_session());
    s->hs.reset(new SessionHS(ctx, *p, b, smooth_init, d0, z0));
    out = s.release();
  });
  return out;
}

static void need_session(const ccsc_session* s) {
  if (!s || (!s->s2 && !s->hs)) throw Err(CCSC_E_STATE, "no session");
}

int32_t ccsc_session_step(ccsc_session* s, int32_t n_outer, int32_t* done, char* err,
                          size_t errlen) {
  return guarded(err, errlen, [&] {
    need_session(s);
    HIPCHK(hipSetDevice(s->ctx()->device));
    if (s->hs) s->hs->step(n_outer, done);
    else s->s2->step(n_outer, done);
  });
}

int32_t ccsc_session_objective(ccsc_session* s, double* obj, char* err, size_t errlen) {
  return guarded(err, errlen, [&] {
    need_session(s);
    if (!obj) throw Err(CCSC_E_INVALID, "NULL obj");
    HIPCHK(hipSetDevice(s->ctx()->device));
    if (s->hs) *obj = s->hs->objective_fresh();
    else *obj = s->s2->objective(s->s2->dhat.as<cpx<double>>(), nullptr);
  });
}

int32_t ccsc_session_results(ccsc_session* s, ccsc_outputs* out, char* err, size_t errlen) {
  return guarded(err, errlen, [&] {
    need_session(s);
    HIPCHK(hipSetDevice(s->ctx()->device));
    if (s->hs) s->hs->results(out);
    else s->s2->results(out);
  });
}

int32_t ccsc_session_iterlog(ccsc_session* s, ccsc_iterlog* log, char* err, size_t errlen) {
  return guarded(err, errlen, [&] {
    need_session(s);
    if (s->hs) s->hs->iterlog(log);
    else s->s2->iterlog(log);
  });
}

int32_t ccsc_session_set_profiling(ccsc_session* s, int32_t on) {
  if (!s || !s->s2) return s && s->hs ? CCSC_OK : CCSC_E_STATE;  // 2-3D: no per-kernel timers
  s->s2->prof = on != 0;
  return CCSC_OK;
}

int32_t ccsc_session_kernel_stats(ccsc_session* s, int32_t id, int64_t* launches,
                                  double* total_ms, double* alg_bytes_per_launch, char* err,
                                  size_t errlen) {
  return guarded(err, errlen, [&] {
    need_session(s);
    if (id < 0 || id > 4) throw Err(CCSC_E_INVALID, "kernel id out of range");
    const bool t = (bool)s->s2;
    if (launches) *launches = t ? s->s2->k_launch[id] : 0;
    if (total_ms) *total_ms = t ? s->s2->k_ms[id] : 0.0;
    if (alg_bytes_per_launch) *alg_bytes_per_launch = t ? s->s2->alg_bytes(id) : 0.0;
    (void)kKernelNames;
  });
}

void ccsc_session_destroy(ccsc_session* s) {
  if (!s) return;
  if (s->s2 || s->hs) hipSetDevice(s->ctx()->device);
  delete s;
}

int32_t ccsc_learn_hs23(ccsc_ctx* ctx, const ccsc_problem* p, const double* b,
                        const double* smooth_init, const double* d0, const double* z0,
                        ccsc_outputs* out, ccsc_iterlog* log, ccsc_cb cb, void* user, char* err,
                        size_t errlen) {
  return guarded(err, errlen, [&] {
    if (!ctx || !p) throw Err(CCSC_E_INVALID, "NULL ctx/problem");
    if (!ctx->subs.empty())
      throw Err(CCSC_E_UNSUPPORTED, "the 2-3D learner runs one process per GPU (a rank context of "
                                    "ccsc_create / ccsc_create_hostcomm), not on a device list");
    HIPCHK(hipSetDevice(ctx->device));
    SessionHS S(ctx, *p, b, smooth_init, d0, z0);
    S.ensure_trace_capacity(S.p.max_it);
    for (int i = 0; i < S.p.max_it && !S.finished; ++i) {
      S.outer_iteration();
      if (cb) cb(user, S.outer_done, S.v_obj_d.back(), S.v_obj_z.back(), S.v_tim.back());
    }
    S.results(out);
    S.iterlog(log);
  });
}

int32_t ccsc_learn(ccsc_ctx* ctx, const ccsc_problem* p, const double* b, const double* d0,
                   const double* z0, ccsc_outputs* out, ccsc_iterlog* log, ccsc_cb cb,
                   void* user, char* err, size_t errlen) {
  return guarded(err, errlen, [&] {
    if (!ctx || !p) throw Err(CCSC_E_INVALID, "NULL ctx/problem");
    if (p->variant == CCSC_HS23)
      throw Err(CCSC_E_INVALID, "the 2-3D learner takes smooth_init: use ccsc_learn_hs23");
    if (!ctx->subs.empty()) {
      learn_group(ctx, *p, b, d0, z0, out, log, cb, user);
      return;
    }
    HIPCHK(hipSetDevice(ctx->device));
    Session2D S(ctx, *p, b, d0, z0);
    S.ensure_trace_capacity(S.p.max_it);
    for (int i = 0; i < S.p.max_it && !S.finished; ++i) {
      S.outer_iteration();
      if (cb) cb(user, S.outer_done, S.v_obj_d.back(), S.v_obj_z.back(), S.v_tim.back());
    }
    S.results(out);
    S.iterlog(log);
  });
}

int32_t ccsc_test_fft2d(ccsc_ctx* ctx, int32_t X, int32_t Y, int32_t count, const double* in,
                        double* out_halfspec, double* roundtrip, char* err, size_t errlen) {
  return guarded(err, errlen, [&] {
    if (!ctx || !in || count <= 0) throw Err(CCSC_E_INVALID, "bad arguments");
    HIPCHK(hipSetDevice(ctx->device));
    Grid2D G{};
    std::string why;
    if (!make_grid2d(X, Y, G, why)) throw Err(CCSC_E_UNSUPPORTED, why);
    auto tws = make_twiddles(G);
    DevBuf tw, a, hs, rt;
    tw.alloc(tws.size() * 16);
    HIPCHK(hipMemcpy(tw.p, tws.data(), tw.bytes, hipMemcpyHostToDevice));
    const size_t P = (size_t)X * Y;
    a.alloc(P * count * 8);
    hs.alloc((size_t)G.F * count * 16);
    rt.alloc(P * count * 8);
    HIPCHK(hipMemcpy(a.p, in, a.bytes, hipMemcpyHostToDevice));
    hipStream_t st = ctx->stream;
    HIPCHK(launch_r2c_embed<double>(a.as<double>(), P, X, Y, 0, 0, hs.as<cpx<double>>(), G.F,
                                    count, tw.as<cpx<double>>(), G, st));
    HIPCHK(launch_c2r_plain<double>(hs.as<cpx<double>>(), G.F, rt.as<double>(), P, count,
                                    tw.as<cpx<double>>(), G, 1.0 / (double)P, st));
    HIPCHK(hipStreamSynchronize(st));
    if (out_halfspec) HIPCHK(hipMemcpy(out_halfspec, hs.p, hs.bytes, hipMemcpyDeviceToHost));
    if (roundtrip) HIPCHK(hipMemcpy(roundtrip, rt.p, rt.bytes, hipMemcpyDeviceToHost));
  });
}

}  // extern "C"
