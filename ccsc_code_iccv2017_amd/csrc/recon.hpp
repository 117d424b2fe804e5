// Reconstruction solvers: the device side of ccsc_solve.
//
// The solvers reconstruct ONE image per problem from learned filters (inpainting,
// Poisson deconvolution, demosaicing, view synthesis, video deblurring).  Their
// grids are whole images (266 x 266 for the 256^2 inpainting test set, 522 x 394 for
// the Poisson set), too large for the LDS-resident slice transforms of the learners,
// so every 2D/3D transform here is a sequence of global line passes:
//   rows     x-direction R2C / C2R of row pairs (two-for-one), one workgroup per
//            group of row pairs of one slice, with the ADMM prox/dual updates fused
//            between the inverse and the forward transform (k_rows)
//   columns  strided complex FFTs along y (and t) over tiles of TC half-spectrum
//            columns (k_cols)
// and the per-bin z-solves in between.  Spectra are half spectra [slice][t][y][x'].
#pragma once

#include "kernels.hpp"

#include <vector>

namespace ccsc {

// Row-pass geometry: G.X, G.Xh, G.RS (LDS row stride, units of T), G.px (plan of the
// x lines for L row pairs); rows = Y * T rows per slice, L row pairs per workgroup.
struct RowGeom {
  Grid2D G;
  int rows;
  int L;
  int groups;
  int ntw;     // twiddle table length (complex), staged into LDS
};

// Column-pass geometry: lines of length n with element stride es (complex units),
// TC consecutive x' columns per workgroup; workgroup o of a launch starts at
// (o % ninner) * sin + (o / ninner) * sout.
struct ColGeom {
  Plan1D p;
  int n, TC, Xh, xtiles, ninner;
  int ntw;     // twiddle table length (complex), staged into LDS
  int64_t es, sin, sout;
};

// Line kernels run 256-thread workgroups (several per CU: their LDS tiles are small) and
// hold up to kLineGT generic-radix tasks per thread across a pass barrier.  Two, not four:
// the generic tasks' accumulators set the kernels' registers (~160 VGPRs at four, ~100 at
// two), so two allow four workgroups per CU, as many as the 40 KB LDS tiles do -- same-box
// solver bench: inpainting 0.587 -> 0.532, Poisson 2.40 -> 2.13, video 0.713 -> 0.643 ms per
// iteration (profiles/r05/solver_gt_ab.txt)
constexpr int kLineNT = 256;
constexpr int kLineGT = 2;
constexpr int kLineBS = 1;   // native-pass butterflies per thread: maxb_for_radix * BS

constexpr int kRowParts = 5;   // partial sums per row workgroup (see RowArgs)

enum RowMode : int {
  kRowFwd = 0,     // real src slices -> half spectra
  kRowIterZ = 1,   // code slices: C2R -> z (+ tol partials) -> sparsity prox/dual -> R2C of xi2
  kRowIterX = 2,   // data slices: C2R -> v1 (+ objective partials) -> data prox/dual -> R2C of xi1
  kRowFinalZ = 3,  // code slices: C2R -> z (+ partials), no update
  kRowRes = 4,     // data slices: C2R * scale + smoothinit, crop (+ clamp) -> res
};

template <typename T>
struct RowArgs {
  cpx<T>* S;            // spectra [slice][rows][Xh]
  const T* src;         // kRowFwd input [slice][rows][X]
  T* Z;                 // codes [slice][rows][X]
  T* D;                 // dual of the slice's split (d2 codes, d1 data) [slice][rows][X]
  const T* M;           // data slices: padded mask, pad(mask .* b), padded smoothinit,
  const T* Mb;          //   padded x_orig (nullable)         [slice][rows][X]
  const T* SM;
  const T* XO;
  T* res;               // kRowRes output, cropped [slice][st][sy][sx]
  T* part;              // [img][part_slices][group][kRowParts]; this launch's slices of an
  int part_slices;      //   image start at slice part_off of the image's region
  int part_off;
  const int* active;    // per image: 0 = converged, z is final (nullable = all active)
  const T* theta;       // per image prox parameter (lambda / gamma)
  int per_img;          // slices per image in this launch
  int first;            // iteration 0: z = 0, v1 = 0 (no input spectrum)
  int prox;             // codes: 0 soft threshold on every channel, 1 channel 0 skips it (SP:84)
                        // data: 0 quadratic (Mtb + u/th) / (MtM + 1/th), 1 Poisson (SP:193-205)
  int mtm_sq;           // data: MtM = M .* M (SI:151) instead of M
  int obj_sm;           // data: objective residual uses Dz + smoothinit (SD, SV)
  int psnr_sm;          // data: PSNR uses Dz + smoothinit (SI)
  int px0, px1, py0, py1;  // PSNR window in padded-grid coordinates (2D)
  int Y;                // rows per t-plane
  int sbx, sby, sbt;    // kRowRes crop extent
  int rx, ry, rt;       // crop offsets
  int clamp0;           // kRowRes: res(res < 0) = 0 (SP:131)
  T scale;              // kRowRes: C2R scale
};

// LDS offset (units of T, 16-B aligned) of the row kernel's twiddle table: past the
// 2L rows of the slice and the reduction scratch
__host__ __device__ inline size_t rows_tw_off(const RowGeom& rg) {
  return ((size_t)(2 * rg.L) * rg.G.RS + 16 + kLineNT / 64 + 1) & ~(size_t)1;
}
size_t rows_smem_bytes(const RowGeom& rg, size_t tsize);
size_t cols_smem_bytes(const ColGeom& cg, size_t tsize);

template <typename T>
hipError_t launch_rows(int mode, const RowArgs<T>& a, int64_t nslices, const RowGeom& rg,
                       const cpx<T>* tw, hipStream_t st);
// code slices (a, code_mode kRowIterZ / kRowFinalZ) and data slices (b, kRowIterX) in one launch
template <typename T>
hipError_t launch_rows_pair(int code_mode, const RowArgs<T>& a, int64_t nz, const RowArgs<T>& b,
                            int64_t nx, const RowGeom& rg, const cpx<T>* tw, hipStream_t st);
// nouter line sets of S, then (optionally) nouter2 of S2, in one launch
template <typename T>
hipError_t launch_cols(cpx<T>* S, int sign, int64_t nouter, const ColGeom& cg, const cpx<T>* tw,
                       hipStream_t st, cpx<T>* S2 = nullptr, int64_t nouter2 = 0);

// Plans of the global 2D transforms of an X x Y grid (row pass over row pairs + y-line
// column pass, solve.cpp), shared with the consensus learners' slices past one CU's LDS
// (engine.cpp); false if a length has no line plan.
bool gfft_plan(int X, int Y, RowGeom& rg, ColGeom& cy, std::vector<cpx<double>>& tw_rows,
               std::vector<cpx<double>>& tw_cy);
// X x Y x T grids: + the t-line pass (ct) over the Y rows of each slice
bool gfft_plan3(int X, int Y, int Tn, RowGeom& rg, ColGeom& cy, ColGeom& ct,
                std::vector<cpx<double>>& tw_rows, std::vector<cpx<double>>& tw_cy,
                std::vector<cpx<double>>& tw_ct);

// Sherman-Morrison z-solve of SI / SP per (image, bin), in place:
//   xi2 [n][K][F] -> zhat * invP, xi1 [n][F] -> sum_k dhat_k zhat_k (the next v1);
//   tg: SP's smoothness weight on channel 0 (2D grid X x Y), else 0.
template <typename T>
hipError_t launch_solve_sm(cpx<T>* Sz, cpx<T>* Sx, const cpx<T>* dhat, const T* s, T rho, T invP,
                           int F, int K, int64_t n, int tg, int X, int Y, int Xh,
                           hipStream_t st);
// Embed column-major filters [kx, ky, (kt), count] into zeroed grid slices
// [count][T][Y][X] at circshift(-floor(k/2)) (psf2otf's centring).
template <typename T>
hipError_t launch_embed_kernels(const T* k, T* dst, int kx, int ky, int kt, int count, int X, int Y,
                                int Tn, hipStream_t st);
// Padded data-slice inputs of count (image, channel) slices: M = pad0(mask),
// Mb = pad0(mask .* b), SM = padsym(smooth) (nullable), XO = pad0(x_orig) (nullable).
template <typename T>
hipError_t launch_pad_inputs(const T* b, const T* mask, const T* smooth, const T* xo, T* M, T* Mb,
                             T* SM, T* XO, int64_t count, int sbx, int sby, int sbt, int rx,
                             int ry, int rt, int X, int Y, int Tn, hipStream_t st);
// s_f = sum over `count` spectra of |dhat|^2; diag != 0: out = invP / (rho + s_f).
template <typename T>
hipError_t launch_spec_energy(const cpx<T>* dhat, T* out, int64_t F, int count, int diag, T rho,
                              T invP, hipStream_t st);
// a[c][f] *= m[f] for count spectra
template <typename T>
hipError_t launch_spec_mul(cpx<T>* a, const cpx<T>* m, int64_t F, int count, hipStream_t st);
// out[img][j] = sum of part[(img * per_img + s) * groups + g][j] over s, g (fixed order)
template <typename T>
hipError_t launch_reduce_parts(const T* part, T* out, int64_t n, int per_img, int groups,
                               hipStream_t st);

}  // namespace ccsc
