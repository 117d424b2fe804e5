// Objective / DZ kernel (reporting only; excluded from tim_vals like the
// reference, dP:122 vs dP:127).
#include "slice.hpp"

namespace ccsc {

int pick_nb(int F) {
  const int need = (F + kNT - 1) / kNT;
  const int opts[] = {1, 2, 4, 7};
  for (int o : opts)
    if (o >= need) return o;
  return -1;
}

// ---------------------------------------------------------------------------
// Objective / DZ, one workgroup per patch (dP:305-324, dP:193):
//   Dz = real(ifft2(sum_k fft2(z_k) .* dhat_k));
//   part[p] = { ||crop(Dz) - b_p||^2, sum |z_p| }
// b: [np][sby][sbx]; DZ (nullable): [np][Y][X] uncropped.
// ---------------------------------------------------------------------------
// grid (npatch, NV): view uv of patch p (NV = 1 in 2D; 4D: L4:349-369 with the
// same codes z for every view).  DZ: 2D uncropped [p][Y][X] (dP:193), 4D
// cropped [p][uv][sby][sbx] (L4:205-206).  |z|_1 is counted by view 0 only.
template <typename T, int NBR, int NBL>
__global__ __launch_bounds__(kNT) void k_objective(const T* __restrict__ z,
                                                   const cpx<T>* __restrict__ dhat,
                                                   const T* __restrict__ b, int sbx, int sby,
                                                   int r, T* __restrict__ DZ,
                                                   T* __restrict__ part,
                                                   const cpx<T>* __restrict__ twg, Grid2D G,
                                                   int K, int NV) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  Smem<T> S = carve<T>(smem, G);
  load_twiddles(S.tw, twg, G.ntw);
  const int p = blockIdx.x;
  const int uv = blockIdx.y;
  const int P = G.X * G.Y;
  const int F = G.F;
  BinAcc<T, NBR, NBL> acc;
  acc.init(S.acc);
  T l1 = 0;
  for (int k = 0; k < K; ++k) {
    const int64_t off = ((int64_t)p * K + k) * P;
    lds_sync();
    for (int e = threadIdx.x; e < P; e += kNT) {
      const int y = e / G.X, x = e - y * G.X;
      const T v = z[off + e];
      l1 += fabs(v);
      S.slice[y * G.RS + x] = v;
    }
    zero_pad_row(S.slice, G);
    slice_r2c<T, kMaxB>(S.slice, G, S.tw);
    const cpx<T>* dk = dhat + ((int64_t)k * NV + uv) * F;
    acc.each(F, [&](int f, cpx<T>& a) {
      a = cadd(a, cmul(dk[f], lds_cpx(S.slice + bin_off(f, G), 1)));
    });
  }
  __syncthreads();
  acc.each(F, [&](int f, cpx<T>& a) { lds_cpx_store(S.slice + bin_off(f, G), 1, a); });
  slice_c2r<T, kMaxB>(S.slice, G, S.tw);
  const T invP = (T)1 / (T)P;
  if (DZ && NV == 1) {
    T* o = DZ + (int64_t)p * P;
    for (int e = threadIdx.x; e < P; e += kNT) {
      const int y = e / G.X, x = e - y * G.X;
      o[e] = S.slice[y * G.RS + x] * invP;
    }
  } else if (DZ) {
    T* o = DZ + ((int64_t)p * NV + uv) * sbx * sby;
    for (int e = threadIdx.x; e < sbx * sby; e += kNT) {
      const int y = e / sbx, x = e - y * sbx;
      o[e] = S.slice[(y + r) * G.RS + x + r] * invP;
    }
  }
  if (uv != 0) l1 = 0;
  T sq = 0;
  const T* bp = b + ((int64_t)p * NV + uv) * sbx * sby;
  for (int e = threadIdx.x; e < sbx * sby; e += kNT) {
    const int y = e / sbx, x = e - y * sbx;
    const T d = S.slice[(y + r) * G.RS + x + r] * invP - bp[e];
    sq += d * d;
  }
  sq = block_sum(sq, S.red);
  l1 = block_sum(l1, S.red);
  if (threadIdx.x == 0) {
    part[2 * ((int64_t)p * NV + uv)] = sq;
    part[2 * ((int64_t)p * NV + uv) + 1] = l1;
  }
}

template <typename T>
hipError_t launch_objective(const T* z, const cpx<T>* dhat, const T* b, int sbx, int sby, int r,
                            T* DZ, T* part, int64_t npatch, const cpx<T>* tw, const Grid2D& G,
                            int K, int NV, hipStream_t st) {
  if (npatch <= 0) return hipSuccess;
  const int nbv = pick_nb(G.F);
  CCSC_NB_SWITCH(nbv, hipLaunchKernelGGL((k_objective<T, NBR, NBL>),
                                         dim3((unsigned)npatch, (unsigned)NV), dim3(kNT),
                                         fused_smem_bytes(G, sizeof(T), NBL), st, z, dhat, b,
                                         sbx, sby, r, DZ, part, tw, G, K, NV));
  return hipGetLastError();
}

template hipError_t launch_objective<double>(const double*, const cpx<double>*, const double*,
                                             int, int, int, double*, double*, int64_t,
                                             const cpx<double>*, const Grid2D&, int, int,
                                             hipStream_t);

}  // namespace ccsc
