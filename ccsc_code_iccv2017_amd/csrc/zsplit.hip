// Single-pass z-iteration of the 2D learners (gfx950): the byte-dominant
// stage of an outer iteration (95% of the algorithmic bytes of
// C2).
//
// Reference (dP:150-154 with solve_conv_term_Z, dP:278-303; dZ:151-157,
// 283-308):
//   u = soft(z + y, theta);  y += z - u;  C_k = fft2(u - y)
//   zhat_k = b_k/rho - conj(d_k) (d^T b)/(rho (rho + s)),  b_k = conj(d_k) B + rho C_k
//   z = real(ifft2(zhat))
// Closed form: z_k = c_k + ifft2(conj(d_k) w),
//   w = (B - sum_k d_k C_k) / (rho + s),   c_k = u_k - y_k.
//
// The per-bin reduction over k makes a z-iteration need every filter slice of
// a patch before any new z_k exists, which costs a fused kernel a second pass
// over the patch (6 slice-sized HBM transfers per (patch, filter) instead of
// the 4 of the state itself: read z, y; write z, y).  The engine therefore
// keeps the z-phase state *split*: (u_k, y_k) per slice plus w per patch (1/K
// of a slice), with
//     z_k = u_k - y_k + ifft2(conj(dw_k) w)                        (*)
// (dw = the filter spectrum w was solved with).  One z-iteration is then ONE
// pass per patch, each slice read once and written once:
//     z_k   <- (*)                       C2R of conj(dw_k) w, LDS-resident
//     u, y  <- prox / dual of z_k        stored back over (u_k, y_k)
//     C_k    = fft2(u - y)               R2C, LDS-resident
//     acc   += d_k C_k                   registers + spare LDS
//   w <- (B - acc) / ((rho + s) X Y)     stored for the next iteration.
// In exact arithmetic this is the reference's iteration; rounding matches the
// two-pass form operation for operation ((u - y) + ifft2(...) is how z_k was
// formed there too).  k_zmat materialises z (objective, outputs, tol tests);
// k_zhat_split gives the D-precompute its fft2(z) from the split state.
#include "fft_fixed.hpp"
#include "slice.hpp"

#include <type_traits>

namespace ccsc {

// element pairs per thread whose loads are issued before the C2R (the rest
// after it): the prefetch hides HBM latency under the transform, bounded by
// the 128-VGPR budget of a 1024-thread workgroup.
#ifndef CCSC_ZS_PREFETCH
#define CCSC_ZS_PREFETCH 4
#endif
constexpr int kZsPrefetch = CCSC_ZS_PREFETCH;

// 16-B global access at a 32-bit byte offset from a uniform base: lowers to
// the saddr form (SGPR base + one VGPR offset) instead of a 64-bit VGPR
// address per access.
template <typename V>
__device__ __forceinline__ V ld16(const void* base, uint32_t boff) {
  return *reinterpret_cast<const V*>(reinterpret_cast<const char*>(base) + boff);
}
template <typename V>
__device__ __forceinline__ void st16(void* base, uint32_t boff, V v) {
  *reinterpret_cast<V*>(reinterpret_cast<char*>(base) + boff) = v;
}

template <typename T>
__device__ __forceinline__ T soft_dual(T zv, T yv, T theta, T& yn) {
  const T a = zv + yv;
  const T aa = fabs(a);
  const T u = ((aa > theta) ? (T)1 - theta / aa : (T)0) * a;  // max(0, 1-theta/|a|) a  (dP:32)
  yn = a - u;                                                  // y + z - u  (dP:151)
  return u;
}

// One workgroup (NT threads) per patch.  mode 0: U holds z (materialised
// state); mode 1: U holds u and W the previous w (solved with dcorr).
// Outputs: Uo <- u (Uo may alias U), Yz <- y, W <- w.  NBR + NBL accumulator
// bins per thread (registers + spare LDS), NPR element pairs per thread.
template <typename T, int NBR, int NBL, class FG, int NT>
__global__ __launch_bounds__(NT) void k_zsplit(const T* U, T* Uo, T* __restrict__ Yz,
                                               cpx<T>* __restrict__ W,
                                               const cpx<T>* __restrict__ Bhat,
                                               const cpx<T>* __restrict__ dcorr,
                                               const cpx<T>* __restrict__ dhat,
                                               const T* __restrict__ sden,
                                               const cpx<T>* __restrict__ twg, Grid2D Gd, int K,
                                               T theta, int mode) {
  using GO = GridOps<FG, NT>;
  using V2 = typename vec2_t<T>::type;
  constexpr int NB = NBR + NBL;
  constexpr int NPR = FG::P == 0 ? NB : (FG::P / 2 + NT - 1) / NT;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  Smem<T> S = carve<T>(smem, Gd);
  load_twiddles<T, NT>(S.tw, twg, GO::ntw(Gd));
  const int p = blockIdx.x;
  const int X = GO::X(Gd), Yd = GO::Y(Gd), RS = GO::RS(Gd), F = GO::F(Gd);
  const int P = X * Yd;
  const int P2 = P / 2;
  BinAcc<T, NBR, NBL, NT> acc;
  acc.init(S.acc);
  cpx<T>* Wp = W + (int64_t)p * F;

  for (int k = 0; k < K; ++k) {
    const int64_t off = ((int64_t)p * K + k) * P;
    int tid = threadIdx.x;
    asm volatile("" : "+v"(tid));  // per-thread index math stays inside the K loop (LICM)
    const bool vec = (X & 1) == 0;  // element pairs never straddle a row: 16-B accesses
    const V2* U2 = reinterpret_cast<const V2*>(U + off);
    V2* Uo2 = reinterpret_cast<V2*>(Uo + off);
    V2* Y2 = reinterpret_cast<V2*>(Yz + off);
    V2 uv[NPR], yv[NPR];
    if (vec) {
      // first kZsPrefetch pairs: issued before the C2R so their latency hides under it
#pragma unroll
      for (int i = 0; i < kZsPrefetch && i < NPR; ++i) {
        const int e2 = tid + i * NT;
        if (e2 < P2) {
#ifndef CCSC_ABL_NOMEM
          uv[i] = ld16<V2>(U2, (uint32_t)e2 * 16u);
          yv[i] = ld16<V2>(Y2, (uint32_t)e2 * 16u);
#else
          uv[i].x = uv[i].y = (T)e2;
          yv[i].x = yv[i].y = (T)k;
#endif
        }
      }
    }
    lds_sync();  // previous slice's spectrum reads are done
    if (mode) {  // LDS <- conj(dw_k) w, C2R: the ifft2 term of (*)
      const cpx<T>* dk = dcorr + (int64_t)k * F;
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        const int f = tid + i * NT;
        if (f < F) {
          const int y = f / GO::Xh(Gd);
          lds_cpx_store(S.slice + y * RS + 2 * (f - y * GO::Xh(Gd)), 1, cmulc(dk[f], Wp[f]));
        }
      }
#ifndef CCSC_ABL_NOFFT
      GO::c2r(S.slice, Gd, S.tw, tid);
#endif
    }
    asm volatile("" : "+v"(tid));  // elementwise index math after the C2R, not live across it
    if (vec) {
#pragma unroll
      for (int i = kZsPrefetch; i < NPR; ++i) {
        const int e2 = tid + i * NT;
        if (e2 < P2) {
#ifndef CCSC_ABL_NOMEM
          uv[i] = ld16<V2>(U2, (uint32_t)e2 * 16u);
          yv[i] = ld16<V2>(Y2, (uint32_t)e2 * 16u);
#else
          uv[i].x = uv[i].y = (T)e2;
          yv[i].x = yv[i].y = (T)k;
#endif
        }
      }
#pragma unroll
      for (int i = 0; i < NPR; ++i) {
        const int e2 = tid + i * NT;
        if (e2 < P2) {
          const int e = 2 * e2;
          const int y = e / X;
          T* q = S.slice + y * RS + (e - y * X);
          V2 zv = uv[i];
          if (mode) {
            const V2 c = *reinterpret_cast<const V2*>(q);
            zv.x = (uv[i].x - yv[i].x) + c.x;
            zv.y = (uv[i].y - yv[i].y) + c.y;
          }
          V2 un, yn, cn;
          un.x = soft_dual(zv.x, yv[i].x, theta, yn.x);
          un.y = soft_dual(zv.y, yv[i].y, theta, yn.y);
          cn.x = un.x - yn.x;
          cn.y = un.y - yn.y;
#ifndef CCSC_ABL_NOMEM
          st16<V2>(Uo2, (uint32_t)e2 * 16u, un);
          st16<V2>(Y2, (uint32_t)e2 * 16u, yn);
#else
          if (un.x == (T)-1.2345) st16<V2>(Uo2, (uint32_t)e2 * 16u, un);
#endif
          *reinterpret_cast<V2*>(q) = cn;
        }
      }
    } else {
      // odd X (test grids only): scalar elements
      for (int e = tid; e < P; e += NT) {
        const int y = e / X, x = e - y * X;
        const T uu = U[off + e], yy = Yz[off + e];
        const T zv = mode ? (uu - yy) + S.slice[y * RS + x] : uu;
        T yn;
        const T un = soft_dual(zv, yy, theta, yn);
        Uo[off + e] = un;
        Yz[off + e] = yn;
        S.slice[y * RS + x] = un - yn;
      }
    }
    if (GO::Yp(Gd) != GO::Y(Gd))
      for (int x = tid; x < RS; x += NT) S.slice[Yd * RS + x] = (T)0;
#ifndef CCSC_ABL_NOFFT
    GO::r2c(S.slice, Gd, S.tw, tid);
#else
    lds_sync();
#endif
    const cpx<T>* dk = dhat + (int64_t)k * F;
    acc.each(F, [&](int f, cpx<T>& a) {
      const int y = f / GO::Xh(Gd);
      const cpx<T> c = lds_cpx(S.slice + y * RS + 2 * (f - y * GO::Xh(Gd)), 1);
      a = cadd(a, cmul(dk[f], c));
    });
  }
  // w = (B - acc) * sden   (sden = 1/((rho + s) X Y)); every thread reads and
  // writes only its own bins of W, so no barrier is needed after the last
  // C2R's reads of w.
  const cpx<T>* Bp = Bhat + (int64_t)p * F;
  acc.each(F, [&](int f, cpx<T>& a) { Wp[f] = cscale(csub(Bp[f], a), sden[f]); });
}

// Materialise z from the split state, one workgroup per (patch, filter) slice:
//   Zd = Us - Yz + ifft2(conj(dcorr_k) w_p)          (*)
// Zd may alias Us.  With zold != NULL also ||Zd - zold||^2, ||Zd||^2 per slice
// (the tol test, dP:156-157; zold may alias Zd, read before written).
template <typename T, class FG>
__global__ __launch_bounds__(kNT) void k_zmat(const T* Us, const T* __restrict__ Yz,
                                              const cpx<T>* __restrict__ W,
                                              const cpx<T>* __restrict__ dcorr, T* Zd,
                                              const T* zold, T* __restrict__ znorm,
                                              const cpx<T>* __restrict__ twg, Grid2D Gd, int K) {
  using GO = GridOps<FG>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  Smem<T> S = carve<T>(smem, Gd);
  load_twiddles(S.tw, twg, GO::ntw(Gd));
  const int64_t slice = blockIdx.x;
  const int64_t p = slice / K;
  const int k = (int)(slice - p * K);
  const int X = GO::X(Gd), RS = GO::RS(Gd), F = GO::F(Gd);
  const int P = X * GO::Y(Gd);
  const int tid = threadIdx.x;
  const cpx<T>* dk = dcorr + (int64_t)k * F;
  const cpx<T>* Wp = W + p * F;
  for (int f = tid; f < F; f += kNT) {
    const int y = f / GO::Xh(Gd);
    lds_cpx_store(S.slice + y * RS + 2 * (f - y * GO::Xh(Gd)), 1, cmulc(dk[f], Wp[f]));
  }
  GO::c2r(S.slice, Gd, S.tw, tid);
  const int64_t off = slice * P;
  T nd = 0, nz = 0;
  for (int e = tid; e < P; e += kNT) {
    const int y = e / X, x = e - y * X;
    const T zn = (Us[off + e] - Yz[off + e]) + S.slice[y * RS + x];
    if (zold) {
      const T zo = zold[off + e];
      nd += (zn - zo) * (zn - zo);
      nz += zn * zn;
    }
    Zd[off + e] = zn;
  }
  if (zold) {
    nd = block_sum(nd, S.red);
    nz = block_sum(nz, S.red);
    if (tid == 0) {
      znorm[2 * slice] = nd;
      znorm[2 * slice + 1] = nz;
    }
  }
}

// fft2(z) from the split state for the D-precompute (dP:97 uses zhat), one
// workgroup per slice: fft2(u - y) + X*Y conj(dcorr_k) w_p  (fft2 of (*)).
// Slices s = 0..count-1 of patches starting at U/Yz/W (K slices per patch).
template <typename T, class FG>
__global__ __launch_bounds__(kNT) void k_zhat_split(const T* __restrict__ U,
                                                    const T* __restrict__ Yz,
                                                    const cpx<T>* __restrict__ W,
                                                    const cpx<T>* __restrict__ dcorr,
                                                    cpx<T>* __restrict__ dst,
                                                    const cpx<T>* __restrict__ twg, Grid2D Gd,
                                                    int K) {
  using GO = GridOps<FG>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  Smem<T> S = carve<T>(smem, Gd);
  load_twiddles(S.tw, twg, GO::ntw(Gd));
  const int64_t slice = blockIdx.x;
  const int64_t p = slice / K;
  const int k = (int)(slice - p * K);
  const int X = GO::X(Gd), Yd = GO::Y(Gd), RS = GO::RS(Gd), F = GO::F(Gd);
  const int P = X * Yd;
  const int tid = threadIdx.x;
  const int64_t off = slice * P;
  for (int e = tid; e < P; e += kNT) {
    const int y = e / X, x = e - y * X;
    S.slice[y * RS + x] = U[off + e] - Yz[off + e];
  }
  if (GO::Yp(Gd) != Yd)
    for (int x = tid; x < RS; x += kNT) S.slice[Yd * RS + x] = (T)0;
  GO::r2c(S.slice, Gd, S.tw, tid);
  const cpx<T>* dk = dcorr + (int64_t)k * F;
  const cpx<T>* Wp = W + p * F;
  cpx<T>* out = dst + slice * F;
  const T sc = (T)P;
  for (int f = tid; f < F; f += kNT) {
    const int y = f / GO::Xh(Gd);
    const cpx<T> c = lds_cpx(S.slice + y * RS + 2 * (f - y * GO::Xh(Gd)), 1);
    const cpx<T> q = cmulc(dk[f], Wp[f]);
    out[f] = {c.x + sc * q.x, c.y + sc * q.y};
  }
}

// ---------------------------------------------------------------------------
// Host launchers: the fixed 110x110 plan when the grid is C1/C2's, the
// runtime plan otherwise.
// ---------------------------------------------------------------------------
// Workgroup of the fixed-grid z-iteration: 12 waves (3 per SIMD) leave 168
// VGPRs per lane for the transform, the accumulator bins and the prefetch
// (16 waves cap a lane at 128 and spill); every FFT pass of the 110 grid has
// <= 616 butterflies, so one butterfly per thread still covers a pass.
#ifndef CCSC_ZS_NT
#define CCSC_ZS_NT 768
#endif
#ifndef CCSC_ZS_NBR
#define CCSC_ZS_NBR 6
#endif
constexpr int kZsNT = CCSC_ZS_NT;
constexpr int kZsNB = (Grid110::F + kZsNT - 1) / kZsNT;
constexpr int kZsNBR = CCSC_ZS_NBR < kZsNB ? CCSC_ZS_NBR : kZsNB;
constexpr int kZsNBL = kZsNB - kZsNBR;

size_t zsplit_smem_bytes(const Grid2D& G) {
  if (grid_is<Grid110>(G))
    return slice_smem_bytes(G, sizeof(double)) + (size_t)kZsNBL * kZsNT * 2 * sizeof(double);
  return fused_smem_bytes(G, sizeof(double), 3);
}

template <typename T>
hipError_t launch_zsplit(const T* U, T* Uo, T* Yz, cpx<T>* W, const cpx<T>* Bhat,
                         const cpx<T>* dcorr, const cpx<T>* dhat, const T* sden, int64_t npatch,
                         const cpx<T>* tw, const Grid2D& G, int K, T theta, int mode,
                         hipStream_t st) {
  if (npatch <= 0) return hipSuccess;
  if (grid_is<Grid110>(G)) {
    const size_t sm = slice_smem_bytes(G, sizeof(T)) + (size_t)kZsNBL * kZsNT * 2 * sizeof(T);
    hipLaunchKernelGGL((k_zsplit<T, kZsNBR, kZsNBL, Grid110, kZsNT>), dim3((unsigned)npatch),
                       dim3(kZsNT), sm, st, U, Uo, Yz, W, Bhat, dcorr, dhat, sden, tw, G, K,
                       theta, mode);
    return hipGetLastError();
  }
  const int nbv = pick_nb(G.F);
  if (nbv < 0 || (int64_t)(G.X * G.Y / 2) > (int64_t)nbv * kNT) return hipErrorInvalidValue;
  CCSC_NB_SWITCH(nbv, hipLaunchKernelGGL((k_zsplit<T, NBR, NBL, DynGrid, kNT>),
                                         dim3((unsigned)npatch), dim3(kNT),
                                         fused_smem_bytes(G, sizeof(T), NBL), st, U, Uo, Yz, W,
                                         Bhat, dcorr, dhat, sden, tw, G, K, theta, mode));
  return hipGetLastError();
}

template <typename T>
hipError_t launch_zmat(const T* Us, const T* Yz, const cpx<T>* W, const cpx<T>* dcorr, T* Zd,
                       const T* zold, T* znorm, int64_t npatch, const cpx<T>* tw, const Grid2D& G,
                       int K, hipStream_t st) {
  if (npatch <= 0) return hipSuccess;
  const dim3 grid((unsigned)(npatch * K));
  const size_t sm = slice_smem_bytes(G, sizeof(T));
  if (grid_is<Grid110>(G))
    hipLaunchKernelGGL((k_zmat<T, Grid110>), grid, dim3(kNT), sm, st, Us, Yz, W, dcorr, Zd, zold,
                       znorm, tw, G, K);
  else
    hipLaunchKernelGGL((k_zmat<T, DynGrid>), grid, dim3(kNT), sm, st, Us, Yz, W, dcorr, Zd, zold,
                       znorm, tw, G, K);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_zhat_split(const T* U, const T* Yz, const cpx<T>* W, const cpx<T>* dcorr,
                             cpx<T>* dst, int64_t npatch, const cpx<T>* tw, const Grid2D& G,
                             int K, hipStream_t st) {
  if (npatch <= 0) return hipSuccess;
  const dim3 grid((unsigned)(npatch * K));
  const size_t sm = slice_smem_bytes(G, sizeof(T));
  if (grid_is<Grid110>(G))
    hipLaunchKernelGGL((k_zhat_split<T, Grid110>), grid, dim3(kNT), sm, st, U, Yz, W, dcorr, dst,
                       tw, G, K);
  else
    hipLaunchKernelGGL((k_zhat_split<T, DynGrid>), grid, dim3(kNT), sm, st, U, Yz, W, dcorr, dst,
                       tw, G, K);
  return hipGetLastError();
}

template hipError_t launch_zsplit<double>(const double*, double*, double*, cpx<double>*,
                                          const cpx<double>*, const cpx<double>*,
                                          const cpx<double>*, const double*, int64_t,
                                          const cpx<double>*, const Grid2D&, int, double, int,
                                          hipStream_t);
template hipError_t launch_zmat<double>(const double*, const double*, const cpx<double>*,
                                        const cpx<double>*, double*, const double*, double*,
                                        int64_t, const cpx<double>*, const Grid2D&, int,
                                        hipStream_t);
template hipError_t launch_zhat_split<double>(const double*, const double*, const cpx<double>*,
                                              const cpx<double>*, cpx<double>*, int64_t,
                                              const cpx<double>*, const Grid2D&, int, hipStream_t);

}  // namespace ccsc
