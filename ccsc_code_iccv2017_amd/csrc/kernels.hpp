// Host-visible launchers of the libccsc device kernels.
#pragma once

#include "fft.hpp"

namespace ccsc {

size_t slice_smem_bytes(const Grid2D& G, size_t tsize);
size_t fused_smem_bytes(const Grid2D& G, size_t tsize, int nbl);  // + NBL*kNT accumulator bins
int pick_nb(int F);

// ---- kernels2d.hip -------------------------------------------------------
template <typename T>
hipError_t launch_r2c_embed(const T* src, int64_t src_slice, int sx, int sy, int ox, int oy,
                            cpx<T>* dst, int64_t dst_slice, int64_t count, const cpx<T>* tw,
                            const Grid2D& G, hipStream_t st);
template <typename T>
hipError_t launch_c2r_plain(const cpx<T>* src, int64_t src_slice, T* dst, int64_t dst_slice,
                            int64_t count, const cpx<T>* tw, const Grid2D& G, T scale,
                            hipStream_t st);
template <typename T>
hipError_t launch_dual_r2c(const T* D, T* yD, const T* Usup, cpx<T>* Ch, int64_t nslices,
                           const cpx<T>* tw, const Grid2D& G, int K, int r, hipStream_t st);
template <typename T>
hipError_t launch_c2r_dout(const cpx<T>* Dh, T* D, const T* yD, T* supp, T* dnorm, int nfirst,
                           int64_t nslices, const cpx<T>* tw, const Grid2D& G, int r,
                           hipStream_t st);
template <typename T>
hipError_t launch_supp_reduce(const T* supp, T* ssum, int nbl, int per_block, hipStream_t st);
template <typename T>
hipError_t launch_project(const T* ssum, T* Usup, int ngroups, int glen, T invN,
                          hipStream_t st);
template <typename T>
hipError_t launch_sden(const cpx<T>* dhat, T* sden, int F, int K, T rho, T invP,
                       hipStream_t st);
template <typename T>
hipError_t launch_objective(const T* z, const cpx<T>* dhat, const T* b, int sbx, int sby, int r,
                            T* DZ, T* part, int64_t npatch, const cpx<T>* tw, const Grid2D& G,
                            int K, int NV, hipStream_t st);
template <typename T>
hipError_t launch_zstep_diag(T* z, T* as, const cpx<T>* E, const T* sden, int64_t nslices,
                             const cpx<T>* tw, const Grid2D& G, T theta, T rho, T* znorm,
                             bool tol, bool write_z, hipStream_t st);
template <typename T>
hipError_t launch_view_corr(const cpx<T>* dhat, const cpx<T>* Bhat, cpx<T>* E, int64_t npatch,
                            int F, int K, int NV, hipStream_t st);
template <typename T>
hipError_t launch_sum_pairs(const T* part, int count, T* out, hipStream_t st);

// ---- zsplit.hip: the 2D learners' z-iteration on the pre-threshold state ----
// a = z + y per slice + w per patch: u = soft(a), y = a - u, z = u - y +
// ifft2(conj(dcorr) w); see zsplit.hip.
size_t zsplit_smem_bytes(const Grid2D& G);
template <typename T>
hipError_t launch_zsplit(const T* A, T* Ao, const T* Yz, cpx<T>* W, const cpx<T>* Bhat,
                         const cpx<T>* dcorr, const cpx<T>* dhat, const T* sden, int64_t npatch,
                         const cpx<T>* tw, const Grid2D& G, int K, T theta, int mode,
                         hipStream_t st);
// wslot: W and dcorr in bin-slot order (zline state); astate: A in state order.
template <typename T>
hipError_t launch_zmat(const T* As, T* Yz, const cpx<T>* W, const cpx<T>* dcorr, T* Zd,
                       const T* zold, T* znorm, int64_t npatch, const cpx<T>* tw, const Grid2D& G,
                       int K, T theta, hipStream_t st, bool wslot = false);
template <typename T>
hipError_t launch_zhat_split(const T* A, const cpx<T>* W, const cpx<T>* dcorr, cpx<T>* dst,
                             int64_t npatch, const cpx<T>* tw, const Grid2D& G, int K, T theta,
                             hipStream_t st, bool zline_order = false);

// ---- zline.hip: register-line z-iteration on the 110 x 110 grid -------------
// State a in "state order" and w, B^, d^, sden in "bin-slot order" (zline.hpp).
// mode 0: (z, y) materialised in Zn / Yn (natural layout); mode 2: state in A.
bool zline_grid(const Grid2D& G);
size_t zline_smem_bytes();
// tol (kZlTol* bits): Store: z of the starting iterate -> Zt (state order); Cmp: also the
// patch sums of ||z - Zt||^2, ||z||^2 -> zpart[2p..2p+1]; Form: the patch sums of
// ||z_new - z||^2, ||z_new||^2 of the produced iterate -> fpart[2p..2p+1] (needs
// dcorr == dhat); mode 3 = finalize (Store | Cmp, no advance).
template <typename T>
hipError_t launch_zline(const T* A, T* Ao, const T* Zn, const T* Yn, cpx<T>* W, const cpx<T>* Bs,
                        const cpx<T>* dcorr, const cpx<T>* dhat, const T* sden, int64_t npatch,
                        int K, T theta, T rho, int mode, hipStream_t st, int tol = 0,
                        T* Zt = nullptr, T* zpart = nullptr, T* fpart = nullptr);
// tol bits of launch_zline (zline.hip): store z_cur / compare with the stored z / the
// Parseval test of the produced iterate
constexpr int kZlTolStore = 1, kZlTolCmp = 2, kZlTolForm = 4;
template <typename T>
hipError_t launch_state_to_nat_inplace(T* a, int64_t count, hipStream_t st);
// fft2(z) of the register-line state for the D-precompute (k_zhat_split's result in
// natural order, the transforms on the lanes): dst [npatch][K][F]
template <typename T>
hipError_t launch_zhat_line(const T* A, const cpx<T>* W, const cpx<T>* dcorr, cpx<T>* dst,
                            int64_t npatch, int K, T theta, hipStream_t st);
template <typename T>
hipError_t launch_to_slots(const cpx<T>* src, cpx<T>* dst, int64_t count, hipStream_t st);
template <typename T>
hipError_t launch_to_slots_real(const T* src, T* dst, hipStream_t st);
template <typename T>
hipError_t launch_state_to_nat(const T* st_, T* nat, int64_t count, hipStream_t st);

// ---- dstep.hip ------------------------------------------------------------
// Per frequency f of one block: G = A^H A + rho I (A = ni x K code spectra),
// h = A^H b, Cholesky G = L L^H; L packed lower column-major per f.
// NV views: h [F][NV][K], B [ni][NV][F] (NV = 1 in 2D).
template <typename T>
hipError_t launch_gram_chol(const cpx<T>* Zh, const cpx<T>* Bh, cpx<T>* L, cpx<T>* h, int F,
                            int K, int ni, T rho, int NV, hipStream_t st);
// The same outputs on the matrix cores (gramchol.hip): fp64 MFMA Gram and blocked
// Cholesky, K <= 112, K * NV <= 2048.
bool gram_chol_mf_ok(int K, int NV);
hipError_t launch_gram_chol_mf(const cpx<double>* Zh, const cpx<double>* Bh, cpx<double>* L,
                               cpx<double>* h, int F, int K, int ni, double rho, int NV,
                               hipStream_t st);
// The same outputs for 192 < K <= 400 (gramchol_big.hip): the block's code spectra
// transposed into X ([F][ni][K], ni K F complex of workspace), the Gram on the matrix
// cores into the packed slots of L, then a left-looking Cholesky in place.
bool gram_big_ok(int K, int NV);
// X[f][r] = Z[r][f] for the R = ni K rows of a block's code spectra (frequency-major slabs)
hipError_t launch_zh_fmajor(const cpx<double>* Z, cpx<double>* X, int R, int F, hipStream_t st);
// The reference's Woodbury form past the packed K x K kernels (wbig.hip): per f the slot of
// K(K+1)/2 complex holds A_f (ni x K) and the Cholesky factor of M_f = rho I + A_f A_f^H
// (ni x ni), as k_gram_wb's layout; X is the ni K F complex frequency-major workspace.
constexpr int kWgMaxNi = 100;
bool wbig_ok(int K, int ni);
size_t wbig_workspace(int K, int ni, int F);
hipError_t launch_wbig_gram(const cpx<double>* Zh, const cpx<double>* Bh, cpx<double>* X,
                            cpx<double>* L, cpx<double>* h, int F, int K, int ni, double rho, int NV,
                            hipStream_t st);
hipError_t launch_wbig_solve(const cpx<double>* L, const cpx<double>* h, const cpx<double>* Ch,
                             cpx<double>* Dh, int nblocks, int F, int K, int ni, double rho, int NV,
                             hipStream_t st);
hipError_t launch_gram_big(const cpx<double>* Zh, const cpx<double>* Bh, cpx<double>* X,
                           cpx<double>* L, cpx<double>* h, int F, int K, int ni, double rho, int NV,
                           hipStream_t st, bool factor = true);
// the Cholesky of launch_gram_big alone, in place on packed lower Grams (factor = false above,
// e.g. after a sum of per-rank Grams)
hipError_t launch_chol_big(cpx<double>* L, int F, int K, hipStream_t st);
// x_{f,uv} = (L L^H)^{-1} (h_{f,uv} + rho * C_{f,uv}) for every (block, f, view);
// C and Dh are [blk][K][NV][F].
template <typename T>
hipError_t launch_dsolve(const cpx<T>* L, const cpx<T>* h, const cpx<T>* Ch, cpx<T>* Dh,
                         int nblocks, int F, int K, T rho, int NV, hipStream_t st);
// The same solve (NV = 1, 64 < K <= 112) on a factor whose diagonal 16 x 16 tiles hold
// L_jj^-1 (launch_invert_diag, in place after the Gram/Cholesky kernel): one workgroup
// per (block, f) holds the factor's
// 16 x 16 tiles in registers and both sweeps are tile matrix-vector products, so L is
// read once per solve instead of twice.
bool dsolve_tile_ok(int K, int NV);
hipError_t launch_invert_diag(cpx<double>* L, int F, int K, hipStream_t st);
hipError_t launch_dsolve_tile(const cpx<double>* L, const cpx<double>* h, const cpx<double>* Ch,
                              cpx<double>* Dh, int nblocks, int F, int K, double rho, int NV,
                              hipStream_t st);
// Woodbury form for blocks of few patches (woodbury_fits): per f the slot of
// Kp = K(K+1)/2 complex holds A (ni x K, row-major) and the Cholesky factor of
// M = rho I + A A^H (ni x ni dense, row-major, zeros above the diagonal);
// (A^H A + rho I)^{-1} = (I - A^H M^{-1} A) / rho.  Same h, C, Dh layouts.
// woodbury_ok: the kernels can hold the form (lanes over k, ni <= 8 rows of A,
// A and L_M within the K(K+1)/2 slot); woodbury_fits: the AUTO choice, blocks
// of few patches (ni <= K/4) where the form saves bytes and flops.  The form is
// the reference's pinv(rho I + A A^H) (dP:230-236); its solve loses digits when
// ||A||^2 >> rho, which CCSC_DFACTOR_CHOLESKY avoids.
constexpr int kWbMaxNi = 8;
inline bool woodbury_ok(int K, int ni) {
  return ni <= kWbMaxNi && K <= 128 && ni * K + ni * ni <= K * (K + 1) / 2;
}
inline bool woodbury_fits(int K, int ni) { return woodbury_ok(K, ni) && 4 * ni <= K; }
template <typename T>
hipError_t launch_gram_wb(const cpx<T>* Zh, const cpx<T>* Bh, cpx<T>* L, cpx<T>* h, int F, int K,
                          int ni, T rho, int NV, bool staged, hipStream_t st);
// staged: the session's choice of the staged many-view solve (CCSC_WB_STAGE, read once);
// the same value must reach launch_gram_wb and launch_dsolve_wb (it sets h's layout)
template <typename T>
hipError_t launch_dsolve_wb(const cpx<T>* L, const cpx<T>* h, const cpx<T>* Ch, cpx<T>* Dh,
                            int nblocks, int F, int K, int ni, T rho, int NV, bool staged,
                            hipStream_t st);

// ---- kernels3d.hip: the 3D learner's factored transforms -------------------
// Spectra [slice][t][F2]; P2 = X*Y plane voxels.  Modes: see kernels3d.hip.
size_t tfft_smem_bytes(const Grid2D& Gt, size_t tsize);
// tc > 0: the plane spectra go to / come from the t-minor tile order of k_tsolve3
// ([slice][y][x'/tc][t][tc], ttile_bins per slice) instead of [slice][t][F2]
template <typename T>
hipError_t launch_plane_fwd(int mode, const T* a, T* b, const T* usup, int sx, int sy, int st,
                            int o, T theta, int KG, int r, cpx<T>* dst, int64_t nslices, int Tn,
                            const cpx<T>* tw, const Grid2D& G, hipStream_t stream, int tc = 0);
int64_t ttile_bins(int Tn, int Yn, int Xh, int tc);
template <typename T>
hipError_t launch_to_ttiles(const cpx<T>* src, cpx<T>* dst, int Tn, int Yn, int Xh, int tc,
                            int64_t count, hipStream_t stream);
template <typename T>
hipError_t launch_to_ttiles_real(const T* src, T* dst, int Tn, int Yn, int Xh, int tc,
                                 hipStream_t stream);
template <typename T>
hipError_t launch_tfft(const cpx<T>* src, cpx<T>* dst, int64_t nslices, int Yn, int F2, int sign,
                       const cpx<T>* tw, const Grid2D& Gt, hipStream_t stream);
template <typename T>
hipError_t launch_plane_inv(int mode, const cpx<T>* src, T* dst, const T* yv, T* supp, T* norms,
                            int64_t nfirst, T scale, int r, int64_t nslices, int Tn,
                            const cpx<T>* tw, const Grid2D& G, hipStream_t stream, int tc = 0,
                            T* state = nullptr, T theta = 0, bool wz = true,
                            cpx<T>* nxt = nullptr);
// fused t-FFT + z-solve + inverse t-FFT over (patch, y, TC x' columns) tiles; Gt2 plans
// the t lines of K * TC columns (make_gridt with Xh = K * TC); C, Bhat, dhat, sden in the
// t-minor tile order of tile width TC; ppw patches per workgroup (the filter-spectrum
// columns of a block stay in L2 across them)
bool tsolve3_ok(int Tn, int K, int TC);
int tsolve3_nt(int Tn, int K, int TC);   // threads per k_tsolve3 workgroup
size_t tsolve3_smem_bytes(const Grid2D& Gt2, int K, int TC, size_t tsize, bool dl = false);
template <typename T>
hipError_t launch_tsolve3(cpx<T>* C, const cpx<T>* Bhat, const cpx<T>* dhat, const T* sden,
                          int64_t npatch, int K, int Yn, int Xh, int TC, T invP3,
                          const cpx<T>* tw, const Grid2D& Gt2, hipStream_t stream, int ppw);
template <typename T>
hipError_t launch_zsolve3(cpx<T>* C, const cpx<T>* Bhat, const cpx<T>* dhat, const T* sden,
                          int64_t F3, int64_t npatch, int K, T invP3, hipStream_t stream);
template <typename T>
hipError_t launch_corr_sum(const cpx<T>* Zh, const cpx<T>* dhat, cpx<T>* out, int64_t F3, int K,
                           hipStream_t stream);
template <typename T>
hipError_t launch_crop_sq(const T* Dz, const T* b, int sx, int sy, int st, int r, int rt, int X,
                          int Y, const T* z, int64_t zcount, T* part, hipStream_t stream);

// ---- gslice.hip: elementwise stages of 2D slices past one CU's LDS (global-pass path) ----
template <typename T>
hipError_t launch_gp_zdiag(cpx<T>* C, const cpx<T>* E, const T* sden, T rho, int F, int64_t count,
                           hipStream_t st);
template <typename T>
hipError_t launch_gp_views(const cpx<T>* Z, const cpx<T>* dhat, cpx<T>* out, int F, int K, int NV,
                           hipStream_t st);
template <typename T>
hipError_t launch_gp_crop(const T* R, const T* b, T* DZ, int sbx, int sby, int r, int X, int Y,
                          T scale, T* part, int count, hipStream_t st);
template <typename T>
hipError_t launch_gp_prolog(int mode, const T* a, T* b, const T* usup, int sx, int sy, int o,
                            T theta, int KG, int r, T* R, int X, int Y, int64_t count,
                            hipStream_t st, int Tn = 1, int sst = 1, int ot = 0);
template <typename T>
hipError_t launch_gp_epilog(int mode, const T* R, T* dst, const T* yv, T* supp, T* norms,
                            int64_t nfirst, T scale, int r, int X, int Y, int64_t count,
                            T* state, T theta, int wz, hipStream_t st, int Tn = 1);
// the 2-3D learner's slices past one CU's LDS: prologues (masked data prox / sparsity prox +
// dual into R) and epilogues (v or z from the C2R output + the objective's per-slice parts)
enum GpHsMode : int { kHsData = 0, kHsSparse = 1, kHsV = 2, kHsZ = 3 };
template <typename T>
hipError_t launch_gp_hs_prolog(int mode, const T* a, T* e, const T* b, const T* sm, T* R, int X,
                               int Y, int r, int sbx, int sby, T theta, int64_t count,
                               hipStream_t st);
template <typename T>
hipError_t launch_gp_hs_epilog(int mode, const T* R, T* dst, const T* b, const T* sm, T* DZ,
                               T* part, int X, int Y, int r, int sbx, int sby, T invP,
                               int64_t count, hipStream_t st);

// ---- hs23.hip: the 2-3D hyperspectral learner (L23) ----------------------------
// Spectra slice-major [slice][F]: dhat [K][W], zhat [n][K], Xi1 / Yv [n][W]; h [F][W][K].
template <typename T>
hipError_t launch_hs_synth(const cpx<T>* dhat, const cpx<T>* zhat, cpx<T>* Yv, int F, int W,
                           int K, int n, hipStream_t st);
template <typename T>
hipError_t launch_hs_analysis(const cpx<T>* dhat, const cpx<T>* Xi1, const cpx<T>* Xi2,
                              const T* sden, T rho, cpx<T>* zhat, int F, int W, int K, int n,
                              hipStream_t st);
template <typename T>
hipError_t launch_hs_corr(const cpx<T>* zhat, const cpx<T>* Xi1, cpx<T>* h, int F, int W, int K,
                          int n, hipStream_t st);
template <typename T>
hipError_t launch_hs_c2r_v(const cpx<T>* Ys, T* v, const T* b, const T* sm, T* DZ, T* part,
                           int64_t nslices, const cpx<T>* tw, const Grid2D& G, int r, int sbx,
                           int sby, hipStream_t st);
template <typename T>
hipError_t launch_hs_data_r2c(const T* v, T* e, const T* b, const T* sm, cpx<T>* Xi,
                              int64_t nslices, const cpx<T>* tw, const Grid2D& G, int r, int sbx,
                              int sby, T theta, hipStream_t st);
template <typename T>
hipError_t launch_hs_z_r2c(const T* z, T* e, cpx<T>* Xi, int64_t nslices, const cpx<T>* tw,
                           const Grid2D& G, T theta, hipStream_t st);
template <typename T>
hipError_t launch_hs_c2r_z(const cpx<T>* Zh, T* z, T* part, int64_t nslices, const cpx<T>* tw,
                           const Grid2D& G, hipStream_t st);
template <typename T>
hipError_t launch_pad_symmetric(const T* a, T* out, int sbx, int sby, int r, int X, int Y,
                                int64_t nslices, hipStream_t st);
template <typename T>
hipError_t launch_rep_filters(const T* d0, T* out, int SS, int W, int K, hipStream_t st);
template <typename T>
hipError_t launch_gather_support(const T* D, const T* y, T* supp, int KG, int r, int X, int Y,
                                 hipStream_t st);
constexpr int kNormParts = 1024;  // scratch pairs of launch_norms / launch_max
template <typename T>
hipError_t launch_norms(const T* a, const T* b, int64_t count, T* part, T* out2, hipStream_t st);
template <typename T>
hipError_t launch_max(const T* a, int64_t count, T* part, T* out, hipStream_t st);

// ---- localcn.hip: CreateImages.m:299-369 'local_cn' + ZERO_MEAN (:652-657) ---------
// n column-major [H, W] fp64 images (device pointers), one workgroup per image.
bool local_cn_ok(int H, int W);
hipError_t launch_local_cn(const double* in, double* out, int64_t n, int H, int W,
                           hipStream_t st);

// ---- util.hip ---------------------------------------------------------------
template <typename T>
hipError_t launch_randn(T* out, int64_t count, uint64_t seed, uint64_t offset, hipStream_t st);
// Embed [psf,psf,K] (Tn == 1) or [psf,psf,psf,K] filters (column-major) into nrep
// copies of the [K][Tn][Y][X] grid at circshift(-r) positions (dP:38-39, L3:39-40).
template <typename T>
hipError_t launch_embed_filters(const T* d0, T* D, int nrep, int K, int psf, const Grid2D& G,
                                int Tn, hipStream_t st);
template <typename T>
hipError_t launch_replicate(const T* src, T* dst, int64_t n, int nrep, hipStream_t st);
template <typename T>
hipError_t launch_sub_inplace(T* a, const T* b, int64_t n, hipStream_t st);

}  // namespace ccsc
