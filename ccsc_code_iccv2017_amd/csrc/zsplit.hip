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
// State.  The prox and the dual update are functions of the pre-threshold
// value a = z + y alone (dP:150-151):
//     u = soft(a, theta),   y_new = y + z - u = a - u   (= clip(a, -theta, theta)),
// and the next iteration's pre-threshold value is
//     a' = z' + y_new = (u - y_new + corr) + y_new = u + corr,   corr = ifft2(conj(dw_k) w)
// (dw = the filter spectrum w was solved with).  So the z-phase state is ONE
// array a per (patch, filter) slice plus w per patch (1/K of a slice): a
// z-iteration streams 2 slice transfers (read a, write a') instead of the 4 of
// (z, y), in one pass per patch:
//     a  <- soft(a) + corr               C2R of conj(dw_k) w, LDS-resident
//     u = soft(a), y = a - u, C_k = fft2(u - y)     R2C, LDS-resident
//     acc += d_k C_k                     registers + spare LDS
//   w <- (B - acc) / ((rho + s) X Y)     stored for the next iteration.
// In exact arithmetic this is the reference's iteration.  k_zmat materialises
// z = u - y + corr and y (objective, outputs, tol tests); k_zhat_split gives
// the D-precompute fft2(z) from the state.  Mode 0 (z, y materialised: session
// start, after an objective) forms a = z + y on the fly.
#include "fft_fixed.hpp"
#include "slice.hpp"
#include "zline.hpp"

#include <type_traits>

namespace ccsc {

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

// ProxSparse = max(0, 1 - theta/|a|) a  (dP:32) = a - theta sign(a) for |a| > theta,
// else 0: the division-free form (equal up to one rounding; the fp64 divide
// expands to ~12 VALU ops and ran twice per element per iteration, a quarter of
// the z-iteration's VALU instructions).
template <typename T>
__device__ __forceinline__ T soft(T a, T theta) {
  return (fabs(a) > theta) ? a - copysign(theta, a) : (T)0;
}

// half-spectrum bins of a compile-time grid (0 for the runtime-planned one)
template <class FG>
__device__ constexpr int fixed_bins() {
  if constexpr (FG::P == 0) return 0;
  else return FG::F;
}

// One workgroup (NT threads) per patch.  mode 0: A holds z and Yz holds y
// (materialised state); mode 1: A holds the previous pre-threshold state and
// W the previous w (solved with dcorr).  Outputs: Ao <- a (may alias A),
// W <- w.  NBR + NBL accumulator bins per thread (registers + spare LDS), NPR
// element pairs per thread; the next slice's state is loaded while this
// slice's R2C, accumulation and the next C2R run.
template <typename T, int NBR, int NBL, class FG, int NT>
__global__ __launch_bounds__(NT) void k_zsplit(const T* A, T* Ao, const T* __restrict__ Yz,
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
  // element pairs / bins per thread that are in range for every thread (fixed
  // grids): straight-line code without exec-mask branches, which would make
  // the waitcnt pass fence every global access
  constexpr int PFULL = FG::P == 0 ? 0 : (FG::P / 2) / NT;
  constexpr int BFULL = fixed_bins<FG>() / NT;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  Smem<T> S = carve<T>(smem, Gd);
  load_twiddles<T, NT>(S.tw, twg, GO::ntw(Gd));
  const int p = blockIdx.x;
  const int X = GO::X(Gd), Yd = GO::Y(Gd), RS = GO::RS(Gd), F = GO::F(Gd);
  const int P = X * Yd;
  const int P2 = P / 2;
  const bool vec = (X & 1) == 0;  // element pairs never straddle a row: 16-B accesses
  BinAcc<T, NBR, NBL, NT> acc;
  acc.init(S.acc);
  cpx<T>* Wp = W + (int64_t)p * F;

  V2 av[NPR];
  auto load_state = [&](int k) {
    int tid = threadIdx.x;
    asm volatile("" : "+v"(tid));
    const V2* A2 = reinterpret_cast<const V2*>(A + ((int64_t)p * K + k) * P);
#pragma unroll
    for (int i = 0; i < NPR; ++i) {
      const int e2 = tid + i * NT;
      if (i < PFULL || e2 < P2) av[i] = ld16<V2>(A2, (uint32_t)e2 * 16u);
    }
  };
  if (vec) load_state(0);

  for (int k = 0; k < K; ++k) {
    const int64_t off = ((int64_t)p * K + k) * P;
    int tid = threadIdx.x;
    asm volatile("" : "+v"(tid));  // per-thread index math stays inside the K loop (LICM)
    lds_sync();  // previous slice's spectrum reads are done
    if (mode) {  // LDS <- conj(dw_k) w, C2R: the corr term
      const cpx<T>* dk = dcorr + (int64_t)k * F;
      cpx<T> dv[NB], wv[NB];
#pragma unroll
      for (int i = 0; i < NB; ++i) {  // all loads in flight before the first use
        const int f = tid + i * NT;
        if (i < BFULL || f < F) {
          dv[i] = dk[f];
          wv[i] = Wp[f];
        }
      }
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        const int f = tid + i * NT;
        if (i < BFULL || f < F) {
          const int y = f / GO::Xh(Gd);
          lds_cpx_store(S.slice + y * RS + 2 * (f - y * GO::Xh(Gd)), 1, cmulc(dv[i], wv[i]));
        }
      }
      GO::c2r(S.slice, Gd, S.tw, tid);
    }
    asm volatile("" : "+v"(tid));  // elementwise index math after the C2R, not live across it
    if (vec) {
      V2* Ao2 = reinterpret_cast<V2*>(Ao + off);
      const V2* Y2 = reinterpret_cast<const V2*>(Yz + off);
      // all state values are consumed before the first store: on gfx9 vmcnt
      // counts stores too, so a use of a prefetched value after a store waits
      // for that store's completion (the interleaved form stalled once per pair)
#pragma unroll
      for (int i = 0; i < NPR; ++i) {
        const int e2 = tid + i * NT;
        if (i < PFULL || e2 < P2) {
          const int e = 2 * e2;
          const int y = e / X;
          T* q = S.slice + y * RS + (e - y * X);
          V2 a = av[i];
          if (mode) {
            const V2 c = *reinterpret_cast<const V2*>(q);
            a.x = soft(a.x, theta) + c.x;
            a.y = soft(a.y, theta) + c.y;
          } else {
            const V2 yv = ld16<V2>(Y2, (uint32_t)e2 * 16u);
            a.x += yv.x;
            a.y += yv.y;
          }
          av[i] = a;
          const T ux = soft(a.x, theta), uy = soft(a.y, theta);
          V2 cn;
          cn.x = ux - (a.x - ux);   // u - y_new
          cn.y = uy - (a.y - uy);
          *reinterpret_cast<V2*>(q) = cn;
        }
      }
#pragma unroll
      for (int i = 0; i < NPR; ++i) {
        const int e2 = tid + i * NT;
        if (i < PFULL || e2 < P2) st16<V2>(Ao2, (uint32_t)e2 * 16u, av[i]);
      }
    } else {
      // odd X (test grids only): scalar elements
      for (int e = tid; e < P; e += NT) {
        const int y = e / X, x = e - y * X;
        const T av0 = A[off + e];
        const T a = mode ? soft(av0, theta) + S.slice[y * RS + x] : av0 + Yz[off + e];
        Ao[off + e] = a;
        const T u = soft(a, theta);
        S.slice[y * RS + x] = u - (a - u);
      }
    }
    if (GO::Yp(Gd) != GO::Y(Gd))
      for (int x = tid; x < RS; x += NT) S.slice[Yd * RS + x] = (T)0;
    GO::r2c(S.slice, Gd, S.tw, tid);
    // next slice's state: issued after the R2C, when this slice's stores (whose
    // data registers the loads overwrite) have drained; it lands under the
    // accumulation and the next C2R
    if (vec && k + 1 < K) load_state(k + 1);
    const cpx<T>* dk = dhat + (int64_t)k * F;
    acc.template each<BFULL>(F, [&](int f, cpx<T>& a) {
      const int y = f / GO::Xh(Gd);
      const cpx<T> c = lds_cpx(S.slice + y * RS + 2 * (f - y * GO::Xh(Gd)), 1);
      a = cadd(a, cmul(dk[f], c));
    });
  }
  // w = (B - acc) * sden   (sden = 1/((rho + s) X Y)); every thread reads and
  // writes only its own bins of W, so no barrier is needed after the last
  // C2R's reads of w.
  const cpx<T>* Bp = Bhat + (int64_t)p * F;
  acc.template each<BFULL>(F, [&](int f, cpx<T>& a) { Wp[f] = cscale(csub(Bp[f], a), sden[f]); });
}

// Materialise (z, y) from the state, one workgroup per (patch, filter) slice:
//   u = soft(a), y = a - u, z = (u - y) + ifft2(conj(dcorr_k) w_p)
// Zd may alias As (each element read, then written, by one thread).  With
// zold != NULL also ||Zd - zold||^2, ||Zd||^2 per slice (the tol test,
// dP:156-157; zold may alias Zd or Yz: each element is read before it is written,
// by the same thread).
// WSLOT: W and dcorr in the bin-slot order of zline.hip (110 grid only).
template <typename T, class FG, bool WSLOT = false>
__global__ __launch_bounds__(kNT) void k_zmat(const T* As, T* Yz,
                                              const cpx<T>* __restrict__ W,
                                              const cpx<T>* __restrict__ dcorr, T* Zd,
                                              const T* zold, T* __restrict__ znorm,
                                              const cpx<T>* __restrict__ twg, Grid2D Gd, int K,
                                              T theta) {
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
    const int fw = WSLOT ? zl::bin_slot(f) : f;
    lds_cpx_store(S.slice + y * RS + 2 * (f - y * GO::Xh(Gd)), 1, cmulc(dk[fw], Wp[fw]));
  }
  GO::c2r(S.slice, Gd, S.tw, tid);
  const int64_t off = slice * P;
  T nd = 0, nz = 0;
  for (int e = tid; e < P; e += kNT) {
    const int y = e / X, x = e - y * X;
    const T a = As[off + e];
    const T u = soft(a, theta);
    const T yv = a - u;
    const T zn = (u - yv) + S.slice[y * RS + x];
    if (zold) {
      const T zo = zold[off + e];
      nd += (zn - zo) * (zn - zo);
      nz += zn * zn;
    }
    Yz[off + e] = yv;
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

// fft2(z) from the state for the D-precompute (dP:97 uses zhat), one
// workgroup per slice: fft2(u - y) + X*Y conj(dcorr_k) w_p  with u = soft(a),
// y = a - u.  Slices s = 0..count-1 of patches starting at A/W (K per patch).
// ZL: A in the state order and W, dcorr in the bin-slot order of zline.hip.
template <typename T, class FG, bool ZL = false>
__global__ __launch_bounds__(kNT) void k_zhat_split(const T* __restrict__ A,
                                                    const cpx<T>* __restrict__ W,
                                                    const cpx<T>* __restrict__ dcorr,
                                                    cpx<T>* __restrict__ dst,
                                                    const cpx<T>* __restrict__ twg, Grid2D Gd,
                                                    int K, T theta) {
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
    const T a = A[off + (ZL ? zl::state_off(e) : e)];
    const T u = soft(a, theta);
    S.slice[y * RS + x] = u - (a - u);
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
    const int fw = ZL ? zl::bin_slot(f) : f;
    const cpx<T> q = cmulc(dk[fw], Wp[fw]);
    out[f] = {c.x + sc * q.x, c.y + sc * q.y};
  }
}

// ---------------------------------------------------------------------------
// Host launchers: the fixed 110x110 plan when the grid is C1/C2's, the
// runtime plan otherwise.
// ---------------------------------------------------------------------------
// Workgroup of the fixed-grid z-iteration: 12 waves (3 per SIMD) leave 168
// VGPRs per lane for the transform, the accumulator bins and the one-slice
// state prefetch (16 waves cap a lane at 128 and spill); the wave-local line
// transforms of the 110 grid need 11 (x) and 12 (y) waves.
constexpr int kZsNT = 768;
constexpr int kZsNB = (Grid110::F + kZsNT - 1) / kZsNT;
constexpr int kZsNBR = 6 < kZsNB ? 6 : kZsNB;
constexpr int kZsNBL = kZsNB - kZsNBR;

size_t zsplit_smem_bytes(const Grid2D& G) {
  if (grid_is<Grid110>(G))
    return slice_smem_bytes(G, sizeof(double)) + (size_t)kZsNBL * kZsNT * 2 * sizeof(double);
  return fused_smem_bytes(G, sizeof(double), 3);
}

template <typename T>
hipError_t launch_zsplit(const T* U, T* Uo, const T* Yz, cpx<T>* W, const cpx<T>* Bhat,
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
hipError_t launch_zmat(const T* As, T* Yz, const cpx<T>* W, const cpx<T>* dcorr, T* Zd,
                       const T* zold, T* znorm, int64_t npatch, const cpx<T>* tw, const Grid2D& G,
                       int K, T theta, hipStream_t st, bool wslot) {
  if (npatch <= 0) return hipSuccess;
  const dim3 grid((unsigned)(npatch * K));
  const size_t sm = slice_smem_bytes(G, sizeof(T));
  if (wslot && !grid_is<Grid110>(G)) return hipErrorInvalidValue;
  if (wslot)
    hipLaunchKernelGGL((k_zmat<T, Grid110, true>), grid, dim3(kNT), sm, st, As, Yz, W, dcorr, Zd,
                       zold, znorm, tw, G, K, theta);
  else if (grid_is<Grid110>(G))
    hipLaunchKernelGGL((k_zmat<T, Grid110>), grid, dim3(kNT), sm, st, As, Yz, W, dcorr, Zd, zold,
                       znorm, tw, G, K, theta);
  else
    hipLaunchKernelGGL((k_zmat<T, DynGrid>), grid, dim3(kNT), sm, st, As, Yz, W, dcorr, Zd, zold,
                       znorm, tw, G, K, theta);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_zhat_split(const T* A, const cpx<T>* W, const cpx<T>* dcorr, cpx<T>* dst,
                             int64_t npatch, const cpx<T>* tw, const Grid2D& G, int K, T theta,
                             hipStream_t st, bool zline_order) {
  if (npatch <= 0) return hipSuccess;
  const dim3 grid((unsigned)(npatch * K));
  const size_t sm = slice_smem_bytes(G, sizeof(T));
  if (zline_order && !grid_is<Grid110>(G)) return hipErrorInvalidValue;
  if (zline_order)
    hipLaunchKernelGGL((k_zhat_split<T, Grid110, true>), grid, dim3(kNT), sm, st, A, W, dcorr, dst,
                       tw, G, K, theta);
  else if (grid_is<Grid110>(G))
    hipLaunchKernelGGL((k_zhat_split<T, Grid110>), grid, dim3(kNT), sm, st, A, W, dcorr, dst, tw,
                       G, K, theta);
  else
    hipLaunchKernelGGL((k_zhat_split<T, DynGrid>), grid, dim3(kNT), sm, st, A, W, dcorr, dst, tw,
                       G, K, theta);
  return hipGetLastError();
}

template hipError_t launch_zsplit<double>(const double*, double*, const double*, cpx<double>*,
                                          const cpx<double>*, const cpx<double>*,
                                          const cpx<double>*, const double*, int64_t,
                                          const cpx<double>*, const Grid2D&, int, double, int,
                                          hipStream_t);
template hipError_t launch_zmat<double>(const double*, double*, const cpx<double>*,
                                        const cpx<double>*, double*, const double*, double*,
                                        int64_t, const cpx<double>*, const Grid2D&, int, double,
                                        hipStream_t, bool);
template hipError_t launch_zhat_split<double>(const double*, const cpx<double>*,
                                              const cpx<double>*, cpx<double>*, int64_t,
                                              const cpx<double>*, const Grid2D&, int, double,
                                              hipStream_t, bool);

}  // namespace ccsc
