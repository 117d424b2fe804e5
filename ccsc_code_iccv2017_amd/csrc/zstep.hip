// 4D z-iteration kernel (gfx950).  The 2D learners' z-iteration is in
// zsplit.hip.
#include "slice.hpp"

namespace ccsc {

// ---------------------------------------------------------------------------
// 4D z-iteration (L4:159-164 with the diagonal solve of L4:310-347): the
// reference's z-solve has no coupling across filters,
//   zhat = (sum_uv conj(d_uv) B_uv + rho C) / (rho + sum_{uv,k} |d_uv,k|^2),
// so one workgroup per (patch, filter) slice: prox + dual + R2C, scale, C2R.
// E = sum_uv conj(d) B is precomputed once per outer iteration (k_view_corr);
// sden = 1/((rho + s) X Y).  z stays real (Q8: the reference's imaginary part
// is round-off).
// The slice state is a = z + y (the pre-threshold value, as the 2D z-step keeps it):
// u = soft(a) = a - clamp(a), y' = a - u = clamp(a), c = u - y' = a - 2 clamp(a), and
// after the solve a' = z' + y' = z' + clamp(a) -- a read once (re-read from L2 for the
// last step) and written once per iteration; z' is stored only when WZ (the iteration
// whose z the D-precompute, the objective or the tol test reads).  Traffic per slice:
// read a, E; write a' (+ z').
// ---------------------------------------------------------------------------
template <typename T, int RM>
__global__ __launch_bounds__(kNT) __attribute__((amdgpu_waves_per_eu(slice_waves<RM>())))
void k_zstep_diag(T* __restrict__ z, T* __restrict__ as,
                                                    const cpx<T>* __restrict__ E,
                                                    const T* __restrict__ sden,
                                                    const cpx<T>* __restrict__ twg, Grid2D G,
                                                    T theta, T rho, T* __restrict__ znorm,
                                                    int TOL, int WZ) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  Smem<T> S = carve<T>(smem, G);
  using Q = SG<RM>;
  const int GX = Q::X(G);
  if constexpr (!Q::fixed) load_twiddles(S.tw, twg, G.ntw);
  const int64_t slice = blockIdx.x;
  const int P = GX * Q::Y(G);
  const int F = Q::F(G);
  const int64_t off = slice * P;
  theta = __builtin_canonicalize(theta);
  lds_sync();
  // (loads batched: common.hpp batched_loop)
  batched_loop<3>(P, [&](int e) { return as[off + e]; }, [&](int e, T a) {
    const int y = e / GX, x = e - y * GX;
    S.slice[Q::px(x, y, G)] = fma((T)-2, fmax(-theta, fmin(a, theta)), a);
  });
  zero_pad_row(S.slice, G);
  slice_r2c_rm<T, RM>(S.slice, G, S.tw);
  const cpx<T>* Es = E + slice * F;
  struct ES {
    cpx<T> e;
    T sc;
  };
  batched_loop<3>(F, [&](int f) { return ES{Es[f], sden[f]}; }, [&](int f, ES es) {
    T* q = S.slice + Q::bin(f, G);
    const cpx<T> c = lds_cpx(q, 1);
    lds_cpx_store(q, 1, cpx<T>{(es.e.x + rho * c.x) * es.sc, (es.e.y + rho * c.y) * es.sc});
  });
  slice_c2r_rm<T, RM>(S.slice, G, S.tw);
  T nd = 0, nz = 0;
  batched_loop<3>(
      P, [&](int e) { return Pair2<T>{TOL ? z[off + e] : (T)0, as[off + e]}; },
      [&](int e, Pair2<T> za) {
        const int y = e / GX, x = e - y * GX;
        const T zn = S.slice[Q::px(x, y, G)];
        if (TOL) {
          nd += (zn - za.a) * (zn - za.a);
          nz += zn * zn;
        }
        as[off + e] = zn + fmax(-theta, fmin(za.b, theta));
        if (WZ) z[off + e] = zn;
      });
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
hipError_t launch_zstep_diag(T* z, T* as, const cpx<T>* E, const T* sden, int64_t nslices,
                             const cpx<T>* tw, const Grid2D& G, T theta, T rho, T* znorm,
                             bool tol, bool write_z, hipStream_t st) {
  if (nslices <= 0) return hipSuccess;
  if (tol && !write_z) return hipErrorInvalidValue;   // the test reads the z it replaces
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3((unsigned)nslices), dim3(kNT), slice_smem_bytes(G, sizeof(T)),
                       st, z, as, E, sden, tw, G, theta, rho, znorm, tol ? 1 : 0, write_z ? 1 : 0);
  };
  if (grid_is74(G)) go(k_zstep_diag<T, kRm74F>);   // the 74 grid (C5): 2 slices per CU
  else if (slice_fits(kRm74, G)) go(k_zstep_diag<T, kRm74>);
  else go(k_zstep_diag<T, kRmAll>);
  return hipGetLastError();
}

template hipError_t launch_zstep_diag<double>(double*, double*, const cpx<double>*,
                                              const double*, int64_t, const cpx<double>*,
                                              const Grid2D&, double, double, double*, bool,
                                              bool, hipStream_t);

}  // namespace ccsc
