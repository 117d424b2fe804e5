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
template <typename T, int NBR, int NBL>
__global__ __launch_bounds__(kNT) void k_zstep(T* __restrict__ z, T* __restrict__ yz,
                                               T* __restrict__ cbuf,
                                               const cpx<T>* __restrict__ Bhat,
                                               const cpx<T>* __restrict__ dhat,
                                               const T* __restrict__ sden,
                                               const cpx<T>* __restrict__ twg, Grid2D G, int K,
                                               T theta, T* __restrict__ znorm, int TOL) {
  using V2 = typename vec2_t<T>::type;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  Smem<T> S = carve<T>(smem, G);
  load_twiddles(S.tw, twg, G.ntw);
  const int p = blockIdx.x;
  const int P = G.X * G.Y;
  const int P2 = P / 2;
  const int F = G.F;
  const bool vec = (G.X & 1) == 0;  // element pairs never straddle a row
  BinAcc<T, NBR, NBL> acc;
  acc.init(S.acc);

  auto prox = [&](T zv, T yv, T& yn) {
    const T a = zv + yv;
    const T aa = fabs(a);
    const T u = ((aa > theta) ? (T)1 - theta / aa : (T)0) * a;  // max(0, 1-theta/|a|) a
    yn = yv + zv - u;
    return u - yn;                                               // c = u - y_new
  };
  auto lds_pair = [&](int e2) -> T* {
    const int e = 2 * e2;
    const int y = e / G.X;
    return S.slice + y * G.RS + (e - y * G.X);
  };

  // ---- pass 1: prox + dual + R2C + accumulate sum_k d_k C_k ----
  for (int k = 0; k < K; ++k) {
    const int64_t off = ((int64_t)p * K + k) * P;
    T* cdst = (TOL ? cbuf : z) + off;
    int tid = threadIdx.x;
    asm volatile("" : "+v"(tid));  // keep per-thread index math inside the K loop (LICM)
    lds_sync();
    if (vec) {
      const V2* z2 = reinterpret_cast<const V2*>(z + off);
      V2* y2 = reinterpret_cast<V2*>(yz + off);
      V2* c2 = reinterpret_cast<V2*>(cdst);
      for (int base = 0; base < P2; base += kPairBatch * kNT) {
        V2 zv[kPairBatch], yv[kPairBatch];
#pragma unroll
        for (int i = 0; i < kPairBatch; ++i) {
          const int e2 = base + tid + i * kNT;
          if (e2 < P2) {
#ifndef CCSC_ABL_NOMEM
            zv[i] = z2[e2];
            yv[i] = y2[e2];
#else
            zv[i].x = zv[i].y = (T)e2;
            yv[i].x = yv[i].y = (T)k;
#endif
          }
        }
#pragma unroll
        for (int i = 0; i < kPairBatch; ++i) {
          const int e2 = base + tid + i * kNT;
          if (e2 < P2) {
            V2 yn, c;
            c.x = prox(zv[i].x, yv[i].x, yn.x);
            c.y = prox(zv[i].y, yv[i].y, yn.y);
#ifndef CCSC_ABL_NOMEM
            y2[e2] = yn;
            c2[e2] = c;
#endif
            *reinterpret_cast<V2*>(lds_pair(e2)) = c;
          }
        }
      }
    } else {
      for (int e = tid; e < P; e += kNT) {
        const int y = e / G.X, x = e - y * G.X;
        T yn;
        const T c = prox(z[off + e], yz[off + e], yn);
        yz[off + e] = yn;
        cdst[e] = c;
        S.slice[y * G.RS + x] = c;
      }
    }
    zero_pad_row(S.slice, G);
#ifndef CCSC_ABL_NOFFT
    slice_r2c<T, kMaxB>(S.slice, G, S.tw);
#else
    lds_sync();
#endif
    const cpx<T>* dk = dhat + (int64_t)k * F;
    acc.each(F, [&](int f, cpx<T>& a) {
      const cpx<T> c = lds_cpx(S.slice + bin_off(f, G), 1);
      a = cadd(a, cmul(dk[f], c));
    });
  }
  // ---- w = (B - acc) * sden ----
  const cpx<T>* Bp = Bhat + (int64_t)p * F;
  acc.each(F, [&](int f, cpx<T>& a) { a = cscale(csub(Bp[f], a), sden[f]); });
  // ---- pass 2: z_k = c_k + C2R(conj(d_k) w) ----
  T nd = 0, nz = 0;
  for (int k = 0; k < K; ++k) {
    const int64_t off = ((int64_t)p * K + k) * P;
    const T* csrc = (TOL ? cbuf : z) + off;
    const cpx<T>* dk = dhat + (int64_t)k * F;
    int tid = threadIdx.x;
    asm volatile("" : "+v"(tid));  // keep per-thread index math inside the K loop (LICM)
    lds_sync();
    acc.each(F, [&](int f, cpx<T>& a) {
      lds_cpx_store(S.slice + bin_off(f, G), 1, cmulc(dk[f], a));
    });
#ifndef CCSC_ABL_NOFFT
    slice_c2r<T, kMaxB>(S.slice, G, S.tw);
#else
    lds_sync();
#endif
    if (vec) {
      V2* z2 = reinterpret_cast<V2*>(z + off);
      const V2* c2 = reinterpret_cast<const V2*>(csrc);
      for (int base = 0; base < P2; base += kPairBatch * kNT) {
        V2 cv[kPairBatch], zo[kPairBatch];
#pragma unroll
        for (int i = 0; i < kPairBatch; ++i) {
          const int e2 = base + tid + i * kNT;
          if (e2 < P2) {
#ifndef CCSC_ABL_NOMEM
            cv[i] = c2[e2];
            if (TOL) zo[i] = z2[e2];
#else
            cv[i].x = cv[i].y = (T)e2;
#endif
          }
        }
#pragma unroll
        for (int i = 0; i < kPairBatch; ++i) {
          const int e2 = base + tid + i * kNT;
          if (e2 < P2) {
            const V2 q = *reinterpret_cast<const V2*>(lds_pair(e2));
            V2 zn;
            zn.x = cv[i].x + q.x;
            zn.y = cv[i].y + q.y;
            if (TOL) {
              nd += (zn.x - zo[i].x) * (zn.x - zo[i].x) + (zn.y - zo[i].y) * (zn.y - zo[i].y);
              nz += zn.x * zn.x + zn.y * zn.y;
            }
#ifndef CCSC_ABL_NOMEM
            z2[e2] = zn;
#else
            if (zn.x == (T)-1.2345) z2[e2] = zn;
#endif
          }
        }
      }
    } else {
      for (int e = tid; e < P; e += kNT) {
        const int y = e / G.X, x = e - y * G.X;
        const T zn = csrc[e] + S.slice[y * G.RS + x];
        if (TOL) {
          const T zo = z[off + e];
          nd += (zn - zo) * (zn - zo);
          nz += zn * zn;
        }
        z[off + e] = zn;
      }
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

// ---------------------------------------------------------------------------
// 4D z-iteration (L4:159-164 with the diagonal solve of L4:310-347): the
// reference's z-solve has no coupling across filters,
//   zhat = (sum_uv conj(d_uv) B_uv + rho C) / (rho + sum_{uv,k} |d_uv,k|^2),
// so one workgroup per (patch, filter) slice: prox + dual + R2C, scale, C2R.
// E = sum_uv conj(d) B is precomputed once per outer iteration (k_view_corr);
// sden = 1/((rho + s) X Y).  z stays real (Q8: the reference's imaginary part
// is round-off).  Traffic per slice: read z, y, E; write y, z.
// ---------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(kNT) void k_zstep_diag(T* __restrict__ z, T* __restrict__ yz,
                                                    const cpx<T>* __restrict__ E,
                                                    const T* __restrict__ sden,
                                                    const cpx<T>* __restrict__ twg, Grid2D G,
                                                    T theta, T rho, T* __restrict__ znorm,
                                                    int TOL) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  Smem<T> S = carve<T>(smem, G);
  load_twiddles(S.tw, twg, G.ntw);
  const int64_t slice = blockIdx.x;
  const int P = G.X * G.Y;
  const int F = G.F;
  const int64_t off = slice * P;
  lds_sync();
  for (int e = threadIdx.x; e < P; e += kNT) {
    const int y = e / G.X, x = e - y * G.X;
    const T zv = z[off + e], yv = yz[off + e];
    const T a = zv + yv;
    const T aa = fabs(a);
    const T u = ((aa > theta) ? (T)1 - theta / aa : (T)0) * a;
    const T yn = yv + zv - u;
    yz[off + e] = yn;
    S.slice[y * G.RS + x] = u - yn;
  }
  zero_pad_row(S.slice, G);
  slice_r2c<T, kMaxB>(S.slice, G, S.tw);
  const cpx<T>* Es = E + slice * F;
  for (int f = threadIdx.x; f < F; f += kNT) {
    T* q = S.slice + bin_off(f, G);
    const cpx<T> c = lds_cpx(q, 1);
    const cpx<T> e = Es[f];
    const T sc = sden[f];
    lds_cpx_store(q, 1, cpx<T>{(e.x + rho * c.x) * sc, (e.y + rho * c.y) * sc});
  }
  slice_c2r<T, kMaxB>(S.slice, G, S.tw);
  T nd = 0, nz = 0;
  for (int e = threadIdx.x; e < P; e += kNT) {
    const int y = e / G.X, x = e - y * G.X;
    const T zn = S.slice[y * G.RS + x];
    if (TOL) {
      const T zo = z[off + e];
      nd += (zn - zo) * (zn - zo);
      nz += zn * zn;
    }
    z[off + e] = zn;
  }
  if (TOL) {
    nd = block_sum(nd, S.red);
    nz = block_sum(nz, S.red);
    if (threadIdx.x == 0) {
      znorm[2 * slice] = nd;
      znorm[2 * slice + 1] = nz;
    }
  }
}

template <typename T>
hipError_t launch_zstep_diag(T* z, T* yz, const cpx<T>* E, const T* sden, int64_t nslices,
                             const cpx<T>* tw, const Grid2D& G, T theta, T rho, T* znorm,
                             bool tol, hipStream_t st) {
  if (nslices <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_zstep_diag<T>, dim3((unsigned)nslices), dim3(kNT),
                     slice_smem_bytes(G, sizeof(T)), st, z, yz, E, sden, tw, G, theta, rho,
                     znorm, tol ? 1 : 0);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_zstep(T* z, T* yz, T* cbuf, const cpx<T>* Bhat, const cpx<T>* dhat,
                        const T* sden, int64_t npatch, const cpx<T>* tw, const Grid2D& G, int K,
                        T theta, T* znorm, bool tol, hipStream_t st) {
  if (npatch <= 0) return hipSuccess;
  const int nbv = pick_nb(G.F);
  const int t = tol ? 1 : 0;
  CCSC_NB_SWITCH(nbv, hipLaunchKernelGGL((k_zstep<T, NBR, NBL>), dim3((unsigned)npatch),
                                         dim3(kNT), fused_smem_bytes(G, sizeof(T), NBL), st, z,
                                         yz, cbuf, Bhat, dhat, sden, tw, G, K, theta, znorm, t));
  return hipGetLastError();
}

template hipError_t launch_zstep_diag<double>(double*, double*, const cpx<double>*,
                                              const double*, int64_t, const cpx<double>*,
                                              const Grid2D&, double, double, double*, bool,
                                              hipStream_t);
template hipError_t launch_zstep<double>(double*, double*, double*, const cpx<double>*,
                                         const cpx<double>*, const double*, int64_t,
                                         const cpx<double>*, const Grid2D&, int, double, double*,
                                         bool, hipStream_t);

}  // namespace ccsc
