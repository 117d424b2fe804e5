// 2D slice kernels of the consensus-ADMM CSC engine (gfx950).
//
// Each kernel owns one X*Y slice (or one patch = K slices) per workgroup and
// keeps it LDS-resident between the elementwise prologue, the R2C/C2R FFT and
// the per-frequency epilogue, so every slice crosses HBM once per stage.
//
// Reference cross-walk (paths relative to the reference):
//   k_r2c_embed   fft2(padarray(b)) (dP:23-24), fft2(z) for the D-precompute
//                 (dP:97 uses z_hat), fft2 of D1 (dP:143)
//   k_dual_r2c    d_D += D - u ; fft2(u - d_D)                      (dP:109-110)
//   k_c2r_dout    D = real(ifft2(dup)) + support gather of D + d_D  (dP:112,114-121,208-209)
//   k_zstep       ProxSparse; dual; fft2; solve_conv_term_Z; real(ifft2)
//                                                                   (dP:150-154, 278-303)
//   k_objective   objectiveFunction / DZ                            (dP:305-324, dP:193)
#include "slice.hpp"

namespace ccsc {

// ---------------------------------------------------------------------------
// Batched R2C of real slices embedded (zero padded) into the X*Y grid.
// src slice s: sx*sy values (x fastest) placed at offset (ox, oy).
// ---------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(kNT) void k_r2c_embed(const T* __restrict__ src, int64_t src_slice,
                                                   int sx, int sy, int ox, int oy,
                                                   cpx<T>* __restrict__ dst, int64_t dst_slice,
                                                   const cpx<T>* __restrict__ twg, Grid2D G) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  Smem<T> S = carve<T>(smem, G);
  load_twiddles(S.tw, twg, G.ntw);
  const T* in = src + (int64_t)blockIdx.x * src_slice;
  const bool full = (sx == G.X && sy == G.Y);
  if (!full)
    for (int e = threadIdx.x; e < G.Yp * G.RS; e += kNT) S.slice[e] = (T)0;
  __syncthreads();
  batched_loop<3>(sx * sy, [&](int e) { return in[e]; }, [&](int e, T v) {
    const int y = e / sx, x = e - y * sx;
    S.slice[(y + oy) * G.RS + x + ox] = v;
  });
  if (full) zero_pad_row(S.slice, G);
  slice_r2c<T, kMaxB>(S.slice, G, S.tw);
  cpx<T>* out = dst + (int64_t)blockIdx.x * dst_slice;
  for (int f = threadIdx.x; f < G.F; f += kNT) { const int o = bin_off(f, G); out[f] = {S.slice[o], S.slice[o + 1]}; }
}

// Batched C2R (scaled): half spectra -> real X*Y slices.
template <typename T>
__global__ __launch_bounds__(kNT) void k_c2r_plain(const cpx<T>* __restrict__ src,
                                                   int64_t src_slice, T* __restrict__ dst,
                                                   int64_t dst_slice,
                                                   const cpx<T>* __restrict__ twg, Grid2D G,
                                                   T scale) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  Smem<T> S = carve<T>(smem, G);
  load_twiddles(S.tw, twg, G.ntw);
  const cpx<T>* in = src + (int64_t)blockIdx.x * src_slice;
  batched_loop<3>(G.F, [&](int f) { return in[f]; }, [&](int f, cpx<T> v) {
    const int o = bin_off(f, G);
    S.slice[o] = v.x;
    S.slice[o + 1] = v.y;
  });
  slice_c2r<T, kMaxB>(S.slice, G, S.tw);
  T* out = dst + (int64_t)blockIdx.x * dst_slice;
  const int P = G.X * G.Y;
  for (int e = threadIdx.x; e < P; e += kNT) {
    const int y = e / G.X, x = e - y * G.X;
    out[e] = S.slice[y * G.RS + x] * scale;
  }
}

// ---------------------------------------------------------------------------
// D-step, part 1 (dP:109-110): y_j += D_j - u ; C_j = fft2(u - y_j).
// u is zero off the (2r+1)^2 support; Usup holds its support values
// [KG][s][s] with support coordinate (x + r) mod X (KernelConstraintProj layout).
// slice = jl*KG + g over the local blocks; g = k*NV + uv (KG = K*NV filter
// slices per block: NV = 1 in 2D, the U*V views in 4D).
// ---------------------------------------------------------------------------
template <typename T, int RM>
__global__ __launch_bounds__(kNT) __attribute__((amdgpu_waves_per_eu(slice_waves<RM>())))
void k_dual_r2c(const T* __restrict__ D, T* __restrict__ yD,
                                                  const T* __restrict__ Usup,
                                                  cpx<T>* __restrict__ Ch,
                                                  const cpx<T>* __restrict__ twg, Grid2D G,
                                                  int K, int r) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  Smem<T> S = carve<T>(smem, G);
  using Q = SG<RM>;
  const int GX = Q::X(G), GY = Q::Y(G), GF = Q::F(G);
  if constexpr (!Q::fixed) load_twiddles(S.tw, twg, G.ntw);
  const int slice = blockIdx.x;
  const int g = slice % K;   // K here = KG filter slices per block
  const int s = 2 * r + 1;
  const int P = GX * GY;
  const int64_t off = (int64_t)slice * P;
  const T* u = Usup + (int64_t)g * s * s;
  batched_loop<3>(
      P, [&](int e) { return Pair2<T>{yD[off + e], D[off + e]}; },
      [&](int e, Pair2<T> yd) {
        const int y = e / GX, x = e - y * GX;
        const int xr = x + r, yr = y + r;
        const int sxx = xr >= GX ? xr - GX : xr, syy = yr >= GY ? yr - GY : yr;   // (x + r) mod X
        const T uv = (sxx < s && syy < s) ? u[syy * s + sxx] : (T)0;
        const T yv = yd.a + yd.b - uv;
        yD[off + e] = yv;
        S.slice[Q::px(x, y, G)] = uv - yv;
      });
  zero_pad_row(S.slice, G);
  slice_r2c_rm<T, RM>(S.slice, G, S.tw);
  cpx<T>* out = Ch + (int64_t)slice * GF;
  for (int f = threadIdx.x; f < GF; f += kNT) { const int o = Q::bin(f, G); out[f] = {S.slice[o], S.slice[o + 1]}; }
}

// ---------------------------------------------------------------------------
// D-step, part 3 (dP:112, 114-121): D_j = real(ifft2(Dhat_j)); gather the
// support values of D_j + y_j for the consensus sum (only the support is read
// by KernelConstraintProj, dP:208-209).  Slices of global block 1 (the first
// `nfirst` slices of the launch, or none) also accumulate ||D1 - D1_old||^2
// and ||D1||^2 for the tol test (dP:125-131).
// ---------------------------------------------------------------------------
template <typename T, int RM>
__global__ __launch_bounds__(kNT) __attribute__((amdgpu_waves_per_eu(slice_waves<RM>())))
void k_c2r_dout(const cpx<T>* __restrict__ Dh,
                                                  T* __restrict__ D, const T* __restrict__ yD,
                                                  T* __restrict__ supp, T* __restrict__ dnorm,
                                                  int nfirst, const cpx<T>* __restrict__ twg,
                                                  Grid2D G, int r, T invP) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  Smem<T> S = carve<T>(smem, G);
  using Q = SG<RM>;
  const int GX = Q::X(G), GY = Q::Y(G), GF = Q::F(G);
  if constexpr (!Q::fixed) load_twiddles(S.tw, twg, G.ntw);
  const int slice = blockIdx.x;
  const cpx<T>* in = Dh + (int64_t)slice * GF;
  batched_loop<3>(GF, [&](int f) { return in[f]; }, [&](int f, cpx<T> v) {
    const int o = Q::bin(f, G);
    S.slice[o] = v.x;
    S.slice[o + 1] = v.y;
  });
  slice_c2r_rm<T, RM>(S.slice, G, S.tw);
  const int P = GX * GY;
  const int64_t off = (int64_t)slice * P;
  const bool first = slice < nfirst;
  T acc_d = 0, acc_n = 0;
  batched_loop<3>(P, [&](int e) { return first ? D[off + e] : (T)0; }, [&](int e, T o) {
    const int y = e / GX, x = e - y * GX;
    const T v = S.slice[Q::px(x, y, G)] * invP;
    if (first) {
      acc_d += (v - o) * (v - o);
      acc_n += v * v;
    }
    D[off + e] = v;
  });
  const int s = 2 * r + 1;
  T* sp = supp + (int64_t)slice * s * s;
  for (int q = threadIdx.x; q < s * s; q += kNT) {
    const int sy = q / s, sx = q - sy * s;
    const int x = (sx - r + GX) % GX, y = (sy - r + GY) % GY;
    sp[q] = S.slice[Q::px(x, y, G)] * invP + yD[off + y * GX + x];
  }
  if (first) {
    acc_d = block_sum(acc_d, S.red);
    acc_n = block_sum(acc_n, S.red);
    if (threadIdx.x == 0) {
      dnorm[2 * slice] = acc_d;
      dnorm[2 * slice + 1] = acc_n;
    }
  }
}

// consensus: ssum[q] = sum over local blocks of supp[jl][q]   (q over K*s*s)
template <typename T>
__global__ void k_supp_reduce(const T* __restrict__ supp, T* __restrict__ ssum, int nbl,
                              int per_block) {
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= per_block) return;
  T a = 0;
  for (int j = 0; j < nbl; ++j) a += supp[(int64_t)j * per_block + q];
  ssum[q] = a;
}

// u = KernelConstraintProj((1/N) * sum_j (D_j + y_j))   (dP:106, 201-219).
// One workgroup per normalisation group (a filter in 2D/3D; a (u,v,k) slice in
// 4D, L4:224-225), group = `glen` consecutive support values.
template <typename T>
__global__ __launch_bounds__(256) void k_project(const T* __restrict__ ssum, T* __restrict__ Usup,
                                                 int glen, T invN) {
  __shared__ T red[4];
  const T* in = ssum + (int64_t)blockIdx.x * glen;
  T* out = Usup + (int64_t)blockIdx.x * glen;
  T a = 0;
  for (int q = threadIdx.x; q < glen; q += 256) {
    const T v = in[q] * invN;
    a += v * v;
  }
  a = wave_sum(a);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = a;
  __syncthreads();
  const T nrm = red[0] + red[1] + red[2] + red[3];
  const T sc = (nrm >= (T)1) ? (T)1 / sqrt(nrm) : (T)1;
  for (int q = threadIdx.x; q < glen; q += 256) out[q] = in[q] * invN * sc;
}

// sden[f] = 1 / ((rho + sum_k |dhat_k(f)|^2) * X*Y)   (dP:239-250, folded with
// the 1/(XY) of the inverse FFT).
template <typename T>
__global__ __launch_bounds__(1024) void k_sden(const cpx<T>* __restrict__ dhat,
                                               T* __restrict__ sden, int F, int K, T rho,
                                               T invP) {
  // 64 bins per workgroup, the 16 waves split the K slices (k = w mod 16) and meet in LDS in
  // a fixed order: one thread per bin looping over all slices left C3 (K W = 3100 slices,
  // 6160 bins: 24 workgroups) and C5 (1225 slices, 2812 bins) at 0.2 TB/s
  __shared__ T part[16][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int f = blockIdx.x * 64 + lane;
  T s = 0;
  if (f < F)
    for (int k = w; k < K; k += 16) s += cabs2(dhat[(int64_t)k * F + f]);
  part[w][lane] = s;
  __syncthreads();
  if (w == 0 && f < F) {
    T t = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) t += part[i][lane];
    sden[f] = invP / (rho + t);
  }
}

// 4D z-step precompute (L4:327 first term): E[p][k][f] = sum_uv conj(d[k][uv][f]) B[p][uv][f]
template <typename T>
__global__ void k_view_corr(const cpx<T>* __restrict__ dhat, const cpx<T>* __restrict__ Bhat,
                            cpx<T>* __restrict__ E, int F, int K, int NV) {
  // patch fastest: the workgroups in flight share one bin block's filter spectra in L2
  const int f = blockIdx.y * blockDim.x + threadIdx.x;
  const int p = blockIdx.x;
  if (f >= F) return;
  const cpx<T>* Bp = Bhat + (int64_t)p * NV * F + f;
  for (int k = 0; k < K; ++k) {
    cpx<T> a = {(T)0, (T)0};
    const cpx<T>* dk = dhat + (int64_t)k * NV * F + f;
    for (int uv = 0; uv < NV; ++uv) a = cadd(a, cmulc(dk[(int64_t)uv * F], Bp[(int64_t)uv * F]));
    E[((int64_t)p * K + k) * F + f] = a;
  }
}

// sum of pairs: out[0] = sum part[2i], out[1] = sum part[2i+1]  (one block)
template <typename T>
__global__ __launch_bounds__(256) void k_sum_pairs(const T* __restrict__ part, int count,
                                                   T* __restrict__ out) {
  __shared__ T red[2][4];
  T a = 0, b = 0;
  for (int i = threadIdx.x; i < count; i += 256) {
    a += part[2 * i];
    b += part[2 * i + 1];
  }
  a = wave_sum(a);
  b = wave_sum(b);
  if ((threadIdx.x & 63) == 0) {
    red[0][threadIdx.x >> 6] = a;
    red[1][threadIdx.x >> 6] = b;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    out[0] = red[0][0] + red[0][1] + red[0][2] + red[0][3];
    out[1] = red[1][0] + red[1][1] + red[1][2] + red[1][3];
  }
}

// ---------------------------------------------------------------------------
// Host launchers
// ---------------------------------------------------------------------------
size_t slice_smem_bytes(const Grid2D& G, size_t tsize) {
  return (size_t)G.ntw * 2 * tsize + (size_t)G.Yp * G.RS * tsize + 16 * tsize;
}
size_t fused_smem_bytes(const Grid2D& G, size_t tsize, int nbl) {
  return slice_smem_bytes(G, tsize) + (size_t)nbl * kNT * 2 * tsize;
}

template <typename T>
hipError_t launch_r2c_embed(const T* src, int64_t src_slice, int sx, int sy, int ox, int oy,
                            cpx<T>* dst, int64_t dst_slice, int64_t count, const cpx<T>* tw,
                            const Grid2D& G, hipStream_t st) {
  if (count <= 0) return hipSuccess;
  const size_t sm = slice_smem_bytes(G, sizeof(T));
  hipLaunchKernelGGL(k_r2c_embed<T>, dim3((unsigned)count), dim3(kNT), sm, st, src, src_slice,
                     sx, sy, ox, oy, dst, dst_slice, tw, G);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_c2r_plain(const cpx<T>* src, int64_t src_slice, T* dst, int64_t dst_slice,
                            int64_t count, const cpx<T>* tw, const Grid2D& G, T scale,
                            hipStream_t st) {
  if (count <= 0) return hipSuccess;
  const size_t sm = slice_smem_bytes(G, sizeof(T));
  hipLaunchKernelGGL(k_c2r_plain<T>, dim3((unsigned)count), dim3(kNT), sm, st, src, src_slice,
                     dst, dst_slice, tw, G, scale);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_dual_r2c(const T* D, T* yD, const T* Usup, cpx<T>* Ch, int64_t nslices,
                           const cpx<T>* tw, const Grid2D& G, int K, int r, hipStream_t st) {
  if (nslices <= 0) return hipSuccess;
  const size_t sm = slice_smem_bytes(G, sizeof(T));
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3((unsigned)nslices), dim3(kNT), sm, st, D, yD, Usup, Ch, tw, G,
                       K, r);
  };
  if (grid_is74(G)) go(k_dual_r2c<T, kRm74F>);   // the 74 grid (C5): 2 slices per CU
  else if (slice_fits(kRm74, G)) go(k_dual_r2c<T, kRm74>);
  else go(k_dual_r2c<T, kRmAll>);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_c2r_dout(const cpx<T>* Dh, T* D, const T* yD, T* supp, T* dnorm, int nfirst,
                           int64_t nslices, const cpx<T>* tw, const Grid2D& G, int r,
                           hipStream_t st) {
  if (nslices <= 0) return hipSuccess;
  const size_t sm = slice_smem_bytes(G, sizeof(T));
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3((unsigned)nslices), dim3(kNT), sm, st, Dh, D, yD, supp, dnorm,
                       nfirst, tw, G, r, (T)1 / (T)(G.X * G.Y));
  };
  if (grid_is74(G)) go(k_c2r_dout<T, kRm74F>);
  else if (slice_fits(kRm74, G)) go(k_c2r_dout<T, kRm74>);
  else go(k_c2r_dout<T, kRmAll>);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_supp_reduce(const T* supp, T* ssum, int nbl, int per_block, hipStream_t st) {
  hipLaunchKernelGGL(k_supp_reduce<T>, dim3((per_block + 255) / 256), dim3(256), 0, st, supp,
                     ssum, nbl, per_block);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_project(const T* ssum, T* Usup, int ngroups, int glen, T invN,
                          hipStream_t st) {
  hipLaunchKernelGGL(k_project<T>, dim3(ngroups), dim3(256), 0, st, ssum, Usup, glen, invN);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_sden(const cpx<T>* dhat, T* sden, int F, int K, T rho, T invP,
                       hipStream_t st) {
  hipLaunchKernelGGL(k_sden<T>, dim3((F + 63) / 64), dim3(1024), 0, st, dhat, sden, F, K, rho,
                     invP);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_view_corr(const cpx<T>* dhat, const cpx<T>* Bhat, cpx<T>* E, int64_t npatch,
                            int F, int K, int NV, hipStream_t st) {
  if (npatch <= 0) return hipSuccess;
  if (npatch > 0x7fffffff) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_view_corr<T>, dim3((unsigned)npatch, (F + 255) / 256), dim3(256), 0, st,
                     dhat, Bhat, E, F, K, NV);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_sum_pairs(const T* part, int count, T* out, hipStream_t st) {
  hipLaunchKernelGGL(k_sum_pairs<T>, dim3(1), dim3(256), 0, st, part, count, out);
  return hipGetLastError();
}

#define CCSC_INST2D(T)                                                                          \
  template hipError_t launch_r2c_embed<T>(const T*, int64_t, int, int, int, int, cpx<T>*,        \
                                          int64_t, int64_t, const cpx<T>*, const Grid2D&,        \
                                          hipStream_t);                                          \
  template hipError_t launch_c2r_plain<T>(const cpx<T>*, int64_t, T*, int64_t, int64_t,          \
                                          const cpx<T>*, const Grid2D&, T, hipStream_t);         \
  template hipError_t launch_dual_r2c<T>(const T*, T*, const T*, cpx<T>*, int64_t,               \
                                         const cpx<T>*, const Grid2D&, int, int, hipStream_t);   \
  template hipError_t launch_c2r_dout<T>(const cpx<T>*, T*, const T*, T*, T*, int, int64_t,      \
                                         const cpx<T>*, const Grid2D&, int, hipStream_t);        \
  template hipError_t launch_supp_reduce<T>(const T*, T*, int, int, hipStream_t);               \
  template hipError_t launch_project<T>(const T*, T*, int, int, T, hipStream_t);                \
  template hipError_t launch_sden<T>(const cpx<T>*, T*, int, int, T, T, hipStream_t);           \
  template hipError_t launch_sum_pairs<T>(const T*, int, T*, hipStream_t);                       \
  template hipError_t launch_view_corr<T>(const cpx<T>*, const cpx<T>*, cpx<T>*, int64_t, int,   \
                                          int, int, hipStream_t);

CCSC_INST2D(double)

}  // namespace ccsc
