// 2-3D hyperspectral learner (L23 = 2-3D/DictionaryLearning/admm_learn.m) on gfx950.
//
// L23 learns one 2D filter per wavelength and atom, d [X,Y,W,K], and codes z
// [X,Y,K,n] shared by the W wavelengths of an image:
//     b(:,:,w,p) ~ crop( sum_k d(:,:,w,k) (*) z(:,:,k,p) ) + smoothinit
// with ONE (non-consensus) ADMM over all n images whose two phases each split
// v1 = H x (masked data prox, L23:26) and v2 = x (kernel constraint in the
// D-phase, sparsity in the Z-phase).
//
// Spectra are slice-major half spectra [slice][F] (F = (X/2+1) Y bins, bins
// contiguous), exactly what the slice transforms produce.  The couplings across
// wavelengths w, atoms k and images p are per-bin complex GEMMs; k_bin_gemm runs
// its lanes along f, so every operand load is a coalesced 16-B-per-lane stream
// and each thread keeps a TM x TN register tile of one bin:
//   synth     Yv(f)[w][p] = sum_k dhat(f)[w][k] zhat(f)[k][p]   (L23:108, 171, 334)
//   analysis  zhat(f)[k][p] = (sum_w conj(dhat(f)[w][k]) Xi1(f)[w][p]
//                              + rho Xi2(f)[k][p]) / (rho + s(f)) (L23:314-319, Q7)
//   corr      h(f)[w][k] = sum_p conj(zhat(f)[k][p]) Xi1(f)[w][p]   (L23:293, Z'*xi1)
// The slice kernels fuse each prox/dual update with its transform, one
// workgroup per slice held in LDS (the 2D machinery of fft.hpp):
//   k_hs_c2r_v     v = real(ifft2(Yv)) + the objective's crop residual (L23:108, 336)
//   k_hs_data_r2c  u = ProxDataMasked(v - e); e -= v - u; fft2(u + e)  (L23:112-121, 175-184)
//   k_hs_z_r2c     u = ProxSparse(z - e);     e -= z - u; fft2(u + e)  (L23:176-184)
//   k_hs_c2r_z     z = real(ifft2(zhat)) + sum|z| of the slice        (L23:189, 338)
// The D-phase kernel-constraint split reuses the consensus kernels with one
// block (k_dual_r2c / k_c2r_dout / k_project on y = -d_D{2}), and the d-solve
// the Cholesky path of dstep.hip with the W wavelengths as right-hand sides.
#include "slice.hpp"

namespace ccsc {

// ---------------------------------------------------------------------------
// Per-bin complex GEMM.  For every bin f of F:
//   C(f)[m][q] = alpha(f) * ( sum_j opA(A(f)[m][j]) B(f)[j][q] + beta E(f)[m][q] )
// with X(f)[a][b] = X[f + a*sa + b*sb] (element strides, units of cpx) and the
// output at C[f*cf + m*cm + q*cq].  opA = conj when CONJA.
// ---------------------------------------------------------------------------
constexpr int kBgNT = 256;

template <typename T>
struct BinGemm {
  const cpx<T>* A;
  int64_t am, aj;
  const cpx<T>* B;
  int64_t bj, bq;
  cpx<T>* C;
  int64_t cf, cm, cq;
  const cpx<T>* E;  // nullable
  int64_t em, eq;
  const T* alpha;   // nullable (1)
  T beta;
  int M, N, Kd, F, mtiles, ntiles;
};

// Workgroup order: bin block slowest, (m, q) tile fastest, so the workgroups in flight at
// any time cover few bin blocks and all tiles -- every tile re-reads the same A rows / B
// columns of those bins from L2 / MALL instead of HBM (the other order streamed A once per
// q tile and B once per m tile from HBM: ~10 GB per C3 synthesis launch for 1.1 GB of
// operands)
template <typename T, int TM, int TN, bool CONJA>
__global__ __launch_bounds__(kBgNT) void k_bin_gemm(BinGemm<T> g) {
  const int nt = g.mtiles * g.ntiles;
  const int tile = (int)(blockIdx.x % nt), fblk = (int)(blockIdx.x / nt);
  const int f = fblk * kBgNT + threadIdx.x;
  if (f >= g.F) return;
  const int m0 = (tile % g.mtiles) * TM;
  const int q0 = (tile / g.mtiles) * TN;
  const int mv = min(TM, g.M - m0), qv = min(TN, g.N - q0);
  cpx<T> acc[TM][TN];
#pragma unroll
  for (int u = 0; u < TM; ++u)
#pragma unroll
    for (int v = 0; v < TN; ++v) acc[u][v] = {(T)0, (T)0};
  const cpx<T>* a = g.A + f + (int64_t)m0 * g.am;
  const cpx<T>* b = g.B + f + (int64_t)q0 * g.bq;
  for (int j = 0; j < g.Kd; ++j) {
    cpx<T> av[TM], bv[TN];
#pragma unroll
    for (int t = 0; t < TM; ++t) av[t] = t < mv ? a[t * g.am] : cpx<T>{(T)0, (T)0};
#pragma unroll
    for (int t = 0; t < TN; ++t) bv[t] = t < qv ? b[t * g.bq] : cpx<T>{(T)0, (T)0};
#pragma unroll
    for (int u = 0; u < TM; ++u)
#pragma unroll
      for (int v = 0; v < TN; ++v)
        acc[u][v] = cadd(acc[u][v], CONJA ? cmulc(av[u], bv[v]) : cmul(av[u], bv[v]));
    a += g.aj;
    b += g.bj;
  }
  const T al = g.alpha ? g.alpha[f] : (T)1;
#pragma unroll
  for (int u = 0; u < TM; ++u)
#pragma unroll
    for (int v = 0; v < TN; ++v) {
      if (u < mv && v < qv) {
        cpx<T> c = acc[u][v];
        if (g.E) {
          const cpx<T> e = g.E[f + (int64_t)(m0 + u) * g.em + (int64_t)(q0 + v) * g.eq];
          c.x += g.beta * e.x;
          c.y += g.beta * e.y;
        }
        g.C[(int64_t)f * g.cf + (int64_t)(m0 + u) * g.cm + (int64_t)(q0 + v) * g.cq] =
            cscale(c, al);
      }
    }
}

// ---------------------------------------------------------------------------
// Slice kernels (one workgroup of kNT threads per X*Y slice).
// Image-support test: the crop region [r, r+sbx) x [r, r+sby) of the padded grid
// (M = 1 there, 0 on the padding, L23:255-258).
// ---------------------------------------------------------------------------
__device__ __forceinline__ bool hs_inside(int x, int y, int r, int sbx, int sby) {
  return x >= r && x < r + sbx && y >= r && y < r + sby;
}

template <typename T>
__device__ __forceinline__ void lds_from_spectrum(T* lds, const cpx<T>* __restrict__ in,
                                                  const Grid2D& G) {
  batched_loop<3>(G.F, [&](int f) { return in[f]; }, [&](int f, cpx<T> c) {
    const int o = bin_off(f, G);
    lds[o] = c.x;
    lds[o + 1] = c.y;
  });
}

template <typename T>
__device__ __forceinline__ void lds_to_spectrum(const T* lds, cpx<T>* __restrict__ out,
                                                const Grid2D& G) {
  for (int f = threadIdx.x; f < G.F; f += kNT) {
    const int o = bin_off(f, G);
    out[f] = {lds[o], lds[o + 1]};
  }
}

// v = real(ifft2(Yv)) for (w, p) slices (1/XY folded in); DZ (nullable) =
// v + smoothinit (L23:235); part[2s] = ||crop(v + smoothinit) - b||^2 of the
// slice (the data term of objectiveFunction, L23:334-337).
template <typename T>
__global__ __launch_bounds__(kNT) void k_hs_c2r_v(const cpx<T>* __restrict__ Ys,
                                                  T* __restrict__ v, const T* __restrict__ b,
                                                  const T* __restrict__ sm, T* __restrict__ DZ,
                                                  T* __restrict__ part,
                                                  const cpx<T>* __restrict__ twg, Grid2D G, int r,
                                                  int sbx, int sby, T invP) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  Smem<T> S = carve<T>(smem, G);
  load_twiddles(S.tw, twg, G.ntw);
  const int64_t s = blockIdx.x;
  lds_from_spectrum(S.slice, Ys + s * G.F, G);
  slice_c2r<T, kMaxB>(S.slice, G, S.tw);
  const int P = G.X * G.Y;
  const int64_t off = s * P;
  const T* bs = b + s * (int64_t)sbx * sby;
  T acc = 0;
  batched_loop<3>(P, [&](int e) { return sm[off + e]; }, [&](int e, T smv) {
    const int y = e / G.X, x = e - y * G.X;
    const T val = S.slice[y * G.RS + x] * invP;
    v[off + e] = val;
    if (DZ) DZ[off + e] = val + smv;
    if (hs_inside(x, y, r, sbx, sby)) {
      const T d = (val + smv) - bs[(y - r) * sbx + (x - r)];
      acc += d * d;
    }
  });
  acc = block_sum(acc, S.red);
  if (threadIdx.x == 0) {
    part[2 * s] = acc;
    part[2 * s + 1] = (T)0;
  }
}

// Masked-data split of either phase (D: L23:112,117,120-121; Z: L23:175,180,183-184):
//   u = ProxDataMasked(v - e, theta) = (Mtb + (v - e)/theta) ./ (M + 1/theta),
//   Mtb = M .* (padarray(b) - smoothinit);   e <- e - (v - u);   Xi = fft2(u + e)
template <typename T>
__global__ __launch_bounds__(kNT) void k_hs_data_r2c(const T* __restrict__ v, T* __restrict__ e,
                                                     const T* __restrict__ b,
                                                     const T* __restrict__ sm,
                                                     cpx<T>* __restrict__ Xi,
                                                     const cpx<T>* __restrict__ twg, Grid2D G,
                                                     int r, int sbx, int sby, T invtheta) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  Smem<T> S = carve<T>(smem, G);
  load_twiddles(S.tw, twg, G.ntw);
  const int64_t s = blockIdx.x;
  const int P = G.X * G.Y;
  const int64_t off = s * P;
  const T* bs = b + s * (int64_t)sbx * sby;
  struct In {
    T v, e, sm;
  };
  batched_loop<3>(P, [&](int i) { return In{v[off + i], e[off + i], sm[off + i]}; }, [&](int i, In ve) {
    const int y = i / G.X, x = i - y * G.X;
    const T vv = ve.v, ev = ve.e;
    T m = 0, mtb = 0;
    if (hs_inside(x, y, r, sbx, sby)) {
      m = (T)1;
      mtb = bs[(y - r) * sbx + (x - r)] - ve.sm;
    }
    const T u = (mtb + invtheta * (vv - ev)) / (m + invtheta);
    const T en = ev - (vv - u);
    e[off + i] = en;
    S.slice[y * G.RS + x] = u + en;
  });
  zero_pad_row(S.slice, G);
  slice_r2c<T, kMaxB>(S.slice, G, S.tw);
  lds_to_spectrum(S.slice, Xi + s * G.F, G);
}

// Sparsity split of the Z-phase (L23:176,180,183-184):
//   u = ProxSparse(z - e, theta) = max(0, 1 - theta/|z - e|) (z - e)
//   e <- e - (z - u);   Xi = fft2(u + e)
template <typename T>
__global__ __launch_bounds__(kNT) void k_hs_z_r2c(const T* __restrict__ z, T* __restrict__ e,
                                                  cpx<T>* __restrict__ Xi,
                                                  const cpx<T>* __restrict__ twg, Grid2D G,
                                                  T theta) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  Smem<T> S = carve<T>(smem, G);
  load_twiddles(S.tw, twg, G.ntw);
  const int64_t s = blockIdx.x;
  const int P = G.X * G.Y;
  const int64_t off = s * P;
  batched_loop<3>(P, [&](int i) { return Pair2<T>{z[off + i], e[off + i]}; }, [&](int i, Pair2<T> ze) {
    const int y = i / G.X, x = i - y * G.X;
    const T zv = ze.a, ev = ze.b;
    const T a = zv - ev;
    const T aa = fabs(a);
    const T u = ((aa > theta) ? (T)1 - theta / aa : (T)0) * a;
    const T en = ev - (zv - u);
    e[off + i] = en;
    S.slice[y * G.RS + x] = u + en;
  });
  zero_pad_row(S.slice, G);
  slice_r2c<T, kMaxB>(S.slice, G, S.tw);
  lds_to_spectrum(S.slice, Xi + s * G.F, G);
}

// z = real(ifft2(zhat)) per (k, p) slice (L23:189); part[2s] = sum |z| (L23:338).
template <typename T>
__global__ __launch_bounds__(kNT) void k_hs_c2r_z(const cpx<T>* __restrict__ Zh,
                                                  T* __restrict__ z, T* __restrict__ part,
                                                  const cpx<T>* __restrict__ twg, Grid2D G,
                                                  T invP) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  Smem<T> S = carve<T>(smem, G);
  load_twiddles(S.tw, twg, G.ntw);
  const int64_t s = blockIdx.x;
  lds_from_spectrum(S.slice, Zh + s * G.F, G);
  slice_c2r<T, kMaxB>(S.slice, G, S.tw);
  const int P = G.X * G.Y;
  const int64_t off = s * P;
  T acc = 0;
  for (int i = threadIdx.x; i < P; i += kNT) {
    const int y = i / G.X, x = i - y * G.X;
    const T val = S.slice[y * G.RS + x] * invP;
    z[off + i] = val;
    acc += fabs(val);
  }
  acc = block_sum(acc, S.red);
  if (threadIdx.x == 0) {
    part[2 * s] = acc;
    part[2 * s + 1] = (T)0;
  }
}

// ---------------------------------------------------------------------------
// Small helpers: symmetric padding of smoothinit, filter replication over the
// wavelengths, the support gather that seeds the first projection, and
// grid-wide reductions.
// ---------------------------------------------------------------------------
// padarray(a, [r r 0 0], 'symmetric', 'both') (L23:19): mirror incl. the edge sample.
template <typename T>
__global__ void k_pad_symmetric(const T* __restrict__ a, T* __restrict__ out, int sbx, int sby,
                                int r, int X, int Y, int64_t nslices) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t P = (int64_t)X * Y;
  if (i >= P * nslices) return;
  const int64_t s = i / P;
  const int e = (int)(i - s * P);
  const int y = e / X, x = e - y * X;
  int xi = x - r, yi = y - r;
  if (xi < 0) xi = -xi - 1;
  if (xi >= sbx) xi = 2 * sbx - xi - 1;
  if (yi < 0) yi = -yi - 1;
  if (yi >= sby) yi = 2 * sby - yi - 1;
  out[i] = a[s * (int64_t)sbx * sby + (int64_t)yi * sbx + xi];
}

// d0 [s,s,K] -> [s,s,W,K]: the same filter for every wavelength (L23:56).
template <typename T>
__global__ void k_rep_filters(const T* __restrict__ d0, T* __restrict__ out, int SS, int W, int K) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= SS * W * K) return;
  const int q = i % SS, g = i / SS, k = g / W;
  out[i] = d0[k * SS + q];
}

// supp[g][q] = D + y at support sample q of filter slice g (the values
// KernelConstraintProj reads, L23:242-243).
template <typename T>
__global__ void k_gather_support(const T* __restrict__ D, const T* __restrict__ y,
                                 T* __restrict__ supp, int KG, int r, int X, int Y) {
  const int s = 2 * r + 1, SS = s * s;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= KG * SS) return;
  const int g = i / SS, q = i - g * SS;
  const int sy = q / s, sx = q - sy * s;
  const int x = (sx - r + X) % X, yy = (sy - r + Y) % Y;
  const int64_t o = (int64_t)g * X * Y + (int64_t)yy * X + x;
  supp[i] = D[o] + y[o];
}

constexpr int kRedBlocks = kNormParts;

// mode 0: (sum (a-b)^2, sum a^2); mode 1: (sum |a|, 0); per-block pairs
template <typename T>
__global__ __launch_bounds__(256) void k_norm_parts(const T* __restrict__ a,
                                                    const T* __restrict__ b, int64_t count,
                                                    int mode, T* __restrict__ part) {
  __shared__ T red[2][4];
  T s0 = 0, s1 = 0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < count;
       i += (int64_t)gridDim.x * 256) {
    const T av = a[i];
    if (mode == 0) {
      const T d = av - b[i];
      s0 += d * d;
      s1 += av * av;
    } else {
      s0 += fabs(av);
    }
  }
  s0 = wave_sum(s0);
  s1 = wave_sum(s1);
  if ((threadIdx.x & 63) == 0) {
    red[0][threadIdx.x >> 6] = s0;
    red[1][threadIdx.x >> 6] = s1;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x] = red[0][0] + red[0][1] + red[0][2] + red[0][3];
    part[2 * blockIdx.x + 1] = red[1][0] + red[1][1] + red[1][2] + red[1][3];
  }
}

template <typename T>
__device__ __forceinline__ T wave_max(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
  return v;
}

// out[blockIdx.x] = max over this block's grid-stride share of a
template <typename T>
__global__ __launch_bounds__(256) void k_max_parts(const T* __restrict__ a, int64_t count,
                                                   T* __restrict__ out) {
  __shared__ T red[4];
  T m = -INFINITY;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < count;
       i += (int64_t)gridDim.x * 256)
    m = fmax(m, a[i]);
  m = wave_max(m);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = fmax(fmax(red[0], red[1]), fmax(red[2], red[3]));
}

// ---------------------------------------------------------------------------
// Host launchers
// ---------------------------------------------------------------------------
// register tile TM x TN per thread: 4 x 8 where N allows (C3: 4 x 4 0.0977, 8 x 4 0.0930,
// 4 x 8 0.0919 s per outer iteration, profiles/r05/bin_gemm_tile_ab.txt), 4 x 4 for the
// solvers' one-image GEMMs (N < 8)
template <typename T, bool CONJA, int TM, int TN>
static hipError_t bin_gemm_t(BinGemm<T> g, hipStream_t st) {
  g.mtiles = (g.M + TM - 1) / TM;
  g.ntiles = (g.N + TN - 1) / TN;
  const int64_t nwg = (int64_t)((g.F + kBgNT - 1) / kBgNT) * g.mtiles * g.ntiles;
  if (nwg >= ((int64_t)1 << 31)) return hipErrorInvalidValue;
  const dim3 grid((unsigned)nwg);
  hipLaunchKernelGGL((k_bin_gemm<T, TM, TN, CONJA>), grid, dim3(kBgNT), 0, st, g);
  return hipGetLastError();
}
template <typename T, bool CONJA>
static hipError_t bin_gemm(BinGemm<T> g, hipStream_t st) {
  if (g.M <= 0 || g.N <= 0 || g.F <= 0) return hipSuccess;
  return g.N >= 8 ? bin_gemm_t<T, CONJA, 4, 8>(g, st) : bin_gemm_t<T, CONJA, 4, 4>(g, st);
}

// Yv [n][W][F] = sum_k dhat [K][W][F] * zhat [n][K][F]
template <typename T>
hipError_t launch_hs_synth(const cpx<T>* dhat, const cpx<T>* zhat, cpx<T>* Yv, int F, int W,
                           int K, int n, hipStream_t st) {
  BinGemm<T> g{};
  g.A = dhat; g.am = F; g.aj = (int64_t)W * F;            // A(f)[w][k]
  g.B = zhat; g.bj = F; g.bq = (int64_t)K * F;            // B(f)[k][p]
  g.C = Yv; g.cf = 1; g.cm = F; g.cq = (int64_t)W * F;    // C(f)[w][p]
  g.M = W; g.N = n; g.Kd = K; g.F = F;
  return bin_gemm<T, false>(g, st);
}

// zhat [n][K][F] = (sum_w conj(dhat [K][W][F]) Xi1 [n][W][F] + rho Xi2 [n][K][F]) * sden;
// zhat may alias Xi2 (each element is read and written by the same thread).
template <typename T>
hipError_t launch_hs_analysis(const cpx<T>* dhat, const cpx<T>* Xi1, const cpx<T>* Xi2,
                              const T* sden, T rho, cpx<T>* zhat, int F, int W, int K, int n,
                              hipStream_t st) {
  BinGemm<T> g{};
  g.A = dhat; g.am = (int64_t)W * F; g.aj = F;            // A(f)[k][w]
  g.B = Xi1; g.bj = F; g.bq = (int64_t)W * F;             // B(f)[w][p]
  g.C = zhat; g.cf = 1; g.cm = F; g.cq = (int64_t)K * F;  // C(f)[k][p]
  g.E = Xi2; g.em = F; g.eq = (int64_t)K * F;
  g.beta = rho;
  g.alpha = sden;
  g.M = K; g.N = n; g.Kd = W; g.F = F;
  return bin_gemm<T, true>(g, st);
}

// h [F][W][K] = sum_p conj(zhat [n][K][F]) Xi1 [n][W][F]  (the d-solve's A'*xi1 per wavelength)
template <typename T>
hipError_t launch_hs_corr(const cpx<T>* zhat, const cpx<T>* Xi1, cpx<T>* h, int F, int W, int K,
                          int n, hipStream_t st) {
  BinGemm<T> g{};
  g.A = zhat; g.am = F; g.aj = (int64_t)K * F;            // A(f)[k][p]
  g.B = Xi1; g.bj = (int64_t)W * F; g.bq = F;             // B(f)[p][w]
  g.C = h; g.cf = (int64_t)W * K; g.cm = 1; g.cq = K;     // C(f)[k][w] at h[f][w][k]
  g.M = K; g.N = W; g.Kd = n; g.F = F;
  return bin_gemm<T, true>(g, st);
}

template <typename T>
hipError_t launch_hs_c2r_v(const cpx<T>* Ys, T* v, const T* b, const T* sm, T* DZ, T* part,
                           int64_t nslices, const cpx<T>* tw, const Grid2D& G, int r, int sbx,
                           int sby, hipStream_t st) {
  if (nslices <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_hs_c2r_v<T>, dim3((unsigned)nslices), dim3(kNT),
                     slice_smem_bytes(G, sizeof(T)), st, Ys, v, b, sm, DZ, part, tw, G, r, sbx,
                     sby, (T)1 / (T)(G.X * G.Y));
  return hipGetLastError();
}

template <typename T>
hipError_t launch_hs_data_r2c(const T* v, T* e, const T* b, const T* sm, cpx<T>* Xi,
                              int64_t nslices, const cpx<T>* tw, const Grid2D& G, int r, int sbx,
                              int sby, T theta, hipStream_t st) {
  if (nslices <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_hs_data_r2c<T>, dim3((unsigned)nslices), dim3(kNT),
                     slice_smem_bytes(G, sizeof(T)), st, v, e, b, sm, Xi, tw, G, r, sbx, sby,
                     (T)1 / theta);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_hs_z_r2c(const T* z, T* e, cpx<T>* Xi, int64_t nslices, const cpx<T>* tw,
                           const Grid2D& G, T theta, hipStream_t st) {
  if (nslices <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_hs_z_r2c<T>, dim3((unsigned)nslices), dim3(kNT),
                     slice_smem_bytes(G, sizeof(T)), st, z, e, Xi, tw, G, theta);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_hs_c2r_z(const cpx<T>* Zh, T* z, T* part, int64_t nslices, const cpx<T>* tw,
                           const Grid2D& G, hipStream_t st) {
  if (nslices <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_hs_c2r_z<T>, dim3((unsigned)nslices), dim3(kNT),
                     slice_smem_bytes(G, sizeof(T)), st, Zh, z, part, tw, G,
                     (T)1 / (T)(G.X * G.Y));
  return hipGetLastError();
}

template <typename T>
hipError_t launch_pad_symmetric(const T* a, T* out, int sbx, int sby, int r, int X, int Y,
                                int64_t nslices, hipStream_t st) {
  const int64_t total = (int64_t)X * Y * nslices;
  if (total <= 0) return hipSuccess;
  if (r > sbx || r > sby) return hipErrorInvalidValue;  // one mirror reflection only
  hipLaunchKernelGGL(k_pad_symmetric<T>, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st,
                     a, out, sbx, sby, r, X, Y, nslices);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_rep_filters(const T* d0, T* out, int SS, int W, int K, hipStream_t st) {
  const int total = SS * W * K;
  hipLaunchKernelGGL(k_rep_filters<T>, dim3((total + 255) / 256), dim3(256), 0, st, d0, out, SS,
                     W, K);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_gather_support(const T* D, const T* y, T* supp, int KG, int r, int X, int Y,
                                 hipStream_t st) {
  const int total = KG * (2 * r + 1) * (2 * r + 1);
  hipLaunchKernelGGL(k_gather_support<T>, dim3((total + 255) / 256), dim3(256), 0, st, D, y, supp,
                     KG, r, X, Y);
  return hipGetLastError();
}

// out2 <- (sum (a-b)^2, sum a^2) (b != NULL) or (sum |a|, 0); part holds 2*kRedBlocks
template <typename T>
hipError_t launch_norms(const T* a, const T* b, int64_t count, T* part, T* out2,
                        hipStream_t st) {
  hipLaunchKernelGGL(k_norm_parts<T>, dim3(kRedBlocks), dim3(256), 0, st, a, b, count,
                     b ? 0 : 1, part);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  return launch_sum_pairs<T>(part, kRedBlocks, out2, st);
}

// out[0] = max(a); part holds kRedBlocks
template <typename T>
hipError_t launch_max(const T* a, int64_t count, T* part, T* out, hipStream_t st) {
  hipLaunchKernelGGL(k_max_parts<T>, dim3(kRedBlocks), dim3(256), 0, st, a, count, part);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_max_parts<T>, dim3(1), dim3(256), 0, st, part, (int64_t)kRedBlocks, out);
  return hipGetLastError();
}

#define CCSC_INSTHS(T)                                                                          \
  template hipError_t launch_hs_synth<T>(const cpx<T>*, const cpx<T>*, cpx<T>*, int, int, int,  \
                                         int, hipStream_t);                                     \
  template hipError_t launch_hs_analysis<T>(const cpx<T>*, const cpx<T>*, const cpx<T>*,        \
                                            const T*, T, cpx<T>*, int, int, int, int,           \
                                            hipStream_t);                                       \
  template hipError_t launch_hs_corr<T>(const cpx<T>*, const cpx<T>*, cpx<T>*, int, int, int,   \
                                        int, hipStream_t);                                      \
  template hipError_t launch_hs_c2r_v<T>(const cpx<T>*, T*, const T*, const T*, T*, T*,        \
                                         int64_t, const cpx<T>*, const Grid2D&, int, int, int,  \
                                         hipStream_t);                                          \
  template hipError_t launch_hs_data_r2c<T>(const T*, T*, const T*, const T*, cpx<T>*,          \
                                            int64_t, const cpx<T>*, const Grid2D&, int, int,    \
                                            int, T, hipStream_t);                               \
  template hipError_t launch_hs_z_r2c<T>(const T*, T*, cpx<T>*, int64_t, const cpx<T>*,         \
                                         const Grid2D&, T, hipStream_t);                        \
  template hipError_t launch_hs_c2r_z<T>(const cpx<T>*, T*, T*, int64_t, const cpx<T>*,         \
                                         const Grid2D&, hipStream_t);                           \
  template hipError_t launch_pad_symmetric<T>(const T*, T*, int, int, int, int, int, int64_t,   \
                                              hipStream_t);                                     \
  template hipError_t launch_rep_filters<T>(const T*, T*, int, int, int, hipStream_t);          \
  template hipError_t launch_gather_support<T>(const T*, const T*, T*, int, int, int, int,      \
                                               hipStream_t);                                    \
  template hipError_t launch_norms<T>(const T*, const T*, int64_t, T*, T*, hipStream_t);        \
  template hipError_t launch_max<T>(const T*, int64_t, T*, T*, hipStream_t);

CCSC_INSTHS(double)

}  // namespace ccsc
