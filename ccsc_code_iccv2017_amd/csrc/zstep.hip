// Fused z-iteration kernel (gfx950): the byte-dominant stage of the learner
// (91-95% of the HBM traffic of an outer iteration at the 2D configs,
// SURVEY.md §3 "Hot loops").
#include "slice.hpp"

namespace ccsc {

// ---------------------------------------------------------------------------
// Fused z-iteration, one workgroup per patch (dP:150-154 with the
// Sherman-Morrison solve of dP:278-303 in its simplified form):
//
//   u = soft(z + y, theta);  y += z - u;  c = u - y;  C_k = fft2(c_k)
//   w = (B - sum_k d_k C_k) / (rho + sum_k |d_k|^2)              (per bin)
//   z_k = c_k + ifft2(conj(d_k) * w)
//
// which equals the reference's  zhat_k = b_k/rho - conj(d_k)(d^T b)/(rho(rho+s)),
// b_k = conj(d_k) B + rho C_k  (algebra in DESIGN.md §4).  w lives in
// registers (NB bins per thread); the slice lives in LDS.  Pass 1 stores c
// over z (or into cbuf when the tol test needs z_old), pass 2 rebuilds z.
// ---------------------------------------------------------------------------
template <typename T, int NB>
__global__ __launch_bounds__(kNT) void k_zstep(T* __restrict__ z, T* __restrict__ yz,
                                               T* __restrict__ cbuf,
                                               const cpx<T>* __restrict__ Bhat,
                                               const cpx<T>* __restrict__ dhat,
                                               const T* __restrict__ sden,
                                               const cpx<T>* __restrict__ twg, Grid2D G, int K,
                                               T theta, T* __restrict__ znorm, int TOL) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  Smem<T> S = carve<T>(smem, G);
  load_twiddles(S.tw, twg, G.X + G.Y);
  const int p = blockIdx.x;
  const int P = G.X * G.Y;
  const int F = G.F;
  cpx<T> acc[NB];
#pragma unroll
  for (int i = 0; i < NB; ++i) acc[i] = {(T)0, (T)0};

  // ---- pass 1: prox + dual + R2C + accumulate sum_k d_k C_k ----
  for (int k = 0; k < K; ++k) {
    const int64_t off = ((int64_t)p * K + k) * P;
    __syncthreads();
    for (int e = threadIdx.x; e < P; e += kNT) {
      const int y = e / G.X, x = e - y * G.X;
      const T zv = z[off + e];
      const T yv = yz[off + e];
      const T a = zv + yv;
      const T aa = fabs(a);
      const T sh = (aa > theta) ? (T)1 - theta / aa : (T)0;   // max(0, 1 - theta/|a|)
      const T u = sh * a;
      const T yn = yv + zv - u;
      const T c = u - yn;
      yz[off + e] = yn;
      if (TOL) cbuf[off + e] = c;
      else z[off + e] = c;
      S.slice[y * G.RS + x] = c;
    }
    zero_pad_row(S.slice, G);
    slice_r2c<T, 2>(S.slice, G, S.tw);
    const cpx<T>* dk = dhat + (int64_t)k * F;
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int f = threadIdx.x + i * kNT;
      if (f < F) {
        const cpx<T> c = {S.slice[2 * f], S.slice[2 * f + 1]};
        acc[i] = cadd(acc[i], cmul(dk[f], c));
      }
    }
  }
  // ---- w = (B - acc) * sden ----
  const cpx<T>* Bp = Bhat + (int64_t)p * F;
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const int f = threadIdx.x + i * kNT;
    if (f < F) acc[i] = cscale(csub(Bp[f], acc[i]), sden[f]);
  }
  // ---- pass 2: z_k = c_k + C2R(conj(d_k) w) ----
  T nd = 0, nz = 0;
  for (int k = 0; k < K; ++k) {
    const int64_t off = ((int64_t)p * K + k) * P;
    const cpx<T>* dk = dhat + (int64_t)k * F;
    __syncthreads();
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int f = threadIdx.x + i * kNT;
      if (f < F) {
        const cpx<T> v = cmulc(dk[f], acc[i]);
        S.slice[2 * f] = v.x;
        S.slice[2 * f + 1] = v.y;
      }
    }
    slice_c2r<T, 2>(S.slice, G, S.tw);
    for (int e = threadIdx.x; e < P; e += kNT) {
      const int y = e / G.X, x = e - y * G.X;
      const T c = TOL ? cbuf[off + e] : z[off + e];
      const T zn = c + S.slice[y * G.RS + x];
      if (TOL) {
        const T zo = z[off + e];
        nd += (zn - zo) * (zn - zo);
        nz += zn * zn;
      }
      z[off + e] = zn;
    }
  }
  if (TOL) {
    nd = block_sum(nd, S.red);
    nz = block_sum(nz, S.red);
    if (threadIdx.x == 0) {
      znorm[2 * p] = nd;
      znorm[2 * p + 1] = nz;
    }
  }
}

template <typename T>
hipError_t launch_zstep(T* z, T* yz, T* cbuf, const cpx<T>* Bhat, const cpx<T>* dhat,
                        const T* sden, int64_t npatch, const cpx<T>* tw, const Grid2D& G, int K,
                        T theta, T* znorm, bool tol, hipStream_t st) {
  if (npatch <= 0) return hipSuccess;
  const size_t sm = slice_smem_bytes(G, sizeof(T));
  const int nbv = pick_nb(G.F);
  const int t = tol ? 1 : 0;
  CCSC_NB_SWITCH(nbv, hipLaunchKernelGGL((k_zstep<T, NB>), dim3((unsigned)npatch), dim3(kNT), sm,
                                         st, z, yz, cbuf, Bhat, dhat, sden, tw, G, K, theta,
                                         znorm, t));
  return hipGetLastError();
}

template hipError_t launch_zstep<double>(double*, double*, double*, const cpx<double>*,
                                         const cpx<double>*, const double*, int64_t,
                                         const cpx<double>*, const Grid2D&, int, double, double*,
                                         bool, hipStream_t);

}  // namespace ccsc
