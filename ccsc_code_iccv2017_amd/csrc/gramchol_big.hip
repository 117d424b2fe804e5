// D-step precompute for filter counts past the register-resident factor of
// gramchol.hip (192 < K <= 400): the same outputs -- per frequency f of a block
// G_f = A_f^H A_f + rho I, h_f = A_f^H b_f and the Cholesky factor L_f, packed lower
// column-major (reference precompute_H_hat_D, dP:221-237, which inverts G_f through
// pinv for any kernel_size, dP:7-8) -- with G_f held in HBM instead of registers:
//   k_zh_fmajor  the block's code spectra [p][k][F] -> [F][p][k] (LDS-tiled transpose),
//                so one frequency's A_f is a contiguous ni x K row-major slab;
//   k_gram_big   one workgroup per (f, tile column J): the lower tiles (I >= J, J) of G_f
//                on v_mfma_f64_16x16x4f64 (four waves, up to seven tiles each), written
//                packed with rho on the diagonal; the J = 0 workgroup also forms h_f;
//   k_chol_big   one workgroup (8 waves) per f, left-looking over 16-column panels in
//                place on the packed matrix: panel j's tiles (I, j) lose
//                sum_{J' < j} L_IJ' L_jJ'^H on the matrix cores (L read back from HBM/L2),
//                then the panel is factored in registers exactly as k_gram_chol_mf's
//                panel (pivots by v_readlane, 1/sqrt by v_rsq_f64 + Newton).
// The d-solve of these factors is k_dsolve (dstep.hip, up to seven rows per lane).
#include "kernels.hpp"

namespace ccsc {

typedef double d4b __attribute__((ext_vector_type(4)));

constexpr int kBgMaxT = 25;             // tiles per dimension: K <= 400
constexpr int kBgTS = 17;               // LDS tile column stride (complex)
constexpr int kBgTSZ = 16 * kBgTS;      // complex per LDS tile
constexpr int kBgGramTW = 7;            // Gram tiles per wave (4 waves, T - J <= 25 tiles)
constexpr int kBgCholNT = 512;          // 8 waves
constexpr int kBgCholTW = 4;            // panel tiles per wave (8 waves, T - j <= 25 tiles)

__device__ __forceinline__ d4b mfma_b(double a, double b, d4b c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ double rdl_b(double v, int l) {
  return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), l),
                          __builtin_amdgcn_readlane(__double2loint(v), l));
}

__device__ __forceinline__ int64_t pk_b(int j, int K) { return (int64_t)j * K - ((int64_t)j * (j - 1)) / 2; }

// X[f][r] = Z[r][f] for r = p K + k over rows [0, R): 64 x 64 complex tiles through LDS
__global__ __launch_bounds__(256) void k_zh_fmajor(const cpx<double>* __restrict__ Z,
                                                   cpx<double>* __restrict__ X, int R, int F) {
  __shared__ cpx<double> t[64][65];
  const int r0 = blockIdx.y * 64, f0 = blockIdx.x * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int i = ty; i < 64; i += 4)
    if (r0 + i < R && f0 + tx < F) t[i][tx] = Z[(int64_t)(r0 + i) * F + f0 + tx];
  __syncthreads();
  for (int i = ty; i < 64; i += 4)
    if (f0 + i < F && r0 + tx < R) X[(int64_t)(f0 + i) * R + r0 + tx] = t[tx][i];
}

// lower tiles (I, J), I = J + w + 4 s, of G_f; X_f = A_f row-major (ni x K)
__global__ __launch_bounds__(256) void k_gram_big(const cpx<double>* __restrict__ X,
                                                  const cpx<double>* __restrict__ Bh,
                                                  cpx<double>* __restrict__ L,
                                                  cpx<double>* __restrict__ h, int F, int K,
                                                  int ni, double rho, int NV) {
  const int T = (K + 15) >> 4;
  const int f = blockIdx.x / T, J = blockIdx.x - f * T;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const cpx<double>* Xf = X + (int64_t)f * ni * K;
  const cpx<double> zero = {0.0, 0.0};
  d4b gr[kBgGramTW], gi[kBgGramTW];
#pragma unroll
  for (int s = 0; s < kBgGramTW; ++s) gr[s] = gi[s] = (d4b){0.0, 0.0, 0.0, 0.0};
  const int c = lane & 15, pq = lane >> 4;
  for (int p0 = 0; p0 < ni; p0 += 4) {
    const int p = p0 + pq;
    const cpx<double>* row = Xf + (int64_t)p * K;
    const cpx<double> b = (p < ni && 16 * J + c < K) ? row[16 * J + c] : zero;
#pragma unroll
    for (int s = 0; s < kBgGramTW; ++s) {
      const int I = J + w + 4 * s;
      if (I < T) {
        const cpx<double> a = (p < ni && 16 * I + c < K) ? row[16 * I + c] : zero;
        // conj(a) b: the (I, J) tile of A^H A
        gr[s] = mfma_b(a.x, b.x, gr[s]);
        gr[s] = mfma_b(a.y, b.y, gr[s]);
        gi[s] = mfma_b(a.x, b.y, gi[s]);
        gi[s] = mfma_b(-a.y, b.x, gi[s]);
      }
    }
  }
  cpx<double>* Lf = L + (int64_t)f * (K * (K + 1) / 2);
  // accumulator layout: lane l holds row (l >> 4) + 4 i, column l & 15 of the tile
#pragma unroll
  for (int s = 0; s < kBgGramTW; ++s) {
    const int I = J + w + 4 * s;
    if (I < T) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = 16 * I + pq + 4 * i, cc = 16 * J + c;
        if (r < K && cc < K && r >= cc)
          Lf[pk_b(cc, K) + r - cc] = (r == cc) ? cpx<double>{gr[s][i] + rho, 0.0}
                                               : cpx<double>{gr[s][i], gi[s][i]};
      }
    }
  }
  if (J == 0) {   // h_f = A_f^H b_f, q = uv K + k
    const int KV = K * NV;
    for (int q = threadIdx.x; q < KV; q += 256) {
      const int uv = q / K, k = q - uv * K;
      cpx<double> acc = zero;
      for (int pp = 0; pp < ni; ++pp)
        acc = cadd(acc, cmulc(Xf[(int64_t)pp * K + k], Bh[((int64_t)pp * NV + uv) * F + f]));
      h[(int64_t)f * KV + q] = acc;
    }
  }
}

// element (r, k), r >= k, of the packed lower factor; zero past the matrix
__device__ __forceinline__ cpx<double> lget(const cpx<double>* Lf, int r, int k, int K) {
  return (r < K) ? Lf[pk_b(k, K) + r - k] : cpx<double>{0.0, 0.0};
}

__global__ __launch_bounds__(kBgCholNT) void k_chol_big(cpx<double>* __restrict__ L, int F, int K) {
  const int f = blockIdx.x;
  if (f >= F) return;
  __shared__ cpx<double> P[kBgMaxT * kBgTSZ];   // panel j's tiles (I, j), element (row, col) at col * TS + row
  const int T = (K + 15) >> 4;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  cpx<double>* Lf = L + (int64_t)f * (K * (K + 1) / 2);
  const int row16 = lane & 15, c4 = lane >> 4;
  for (int j = 0; j < T; ++j) {
    // ---- panel update: tiles (I, j), I = j + wave + 8 s ----
#pragma unroll
    for (int s = 0; s < kBgCholTW; ++s) {
      const int I = j + wave + 8 * s;
      if (I < T) {
        d4b gr, gi;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int r = 16 * I + c4 + 4 * i, cc = 16 * j + row16;
          cpx<double> v = {0.0, 0.0};
          if (r < K && r >= cc) v = Lf[pk_b(cc, K) + r - cc];   // cc < K as r >= cc
          else if (r == cc) v = {1.0, 0.0};                     // padding rows: identity
          gr[i] = v.x;
          gi[i] = v.y;
        }
        for (int Jp = 0; Jp < j; ++Jp) {
#pragma unroll
          for (int kk = 0; kk < 4; ++kk) {
            const int k = 16 * Jp + 4 * kk + c4;
            const cpx<double> a = lget(Lf, 16 * I + row16, k, K);   // L_IJ' (row16, k)
            const cpx<double> b = lget(Lf, 16 * j + row16, k, K);   // L_jJ' (row16, k)
            gr = mfma_b(-a.x, b.x, gr);
            gr = mfma_b(-a.y, b.y, gr);
            gi = mfma_b(-a.y, b.x, gi);
            gi = mfma_b(a.x, b.y, gi);
          }
        }
        cpx<double>* dst = P + I * kBgTSZ;
#pragma unroll
        for (int i = 0; i < 4; ++i) dst[row16 * kBgTS + c4 + 4 * i] = {gr[i], gi[i]};
      }
    }
    __syncthreads();   // panel j's updated tiles are in P
    // ---- panel factor (POTRF of (j, j) + TRSM below), right-looking in registers ----
    {
      const bool diag = lane < 16;
      const int q = wave * 48 + lane - 16;
      const int ti = diag ? j : j + 1 + (q >> 4);
      const int row = diag ? lane : (q & 15);
      const bool mine = diag || ti < T;
      cpx<double> x[16];
#pragma unroll
      for (int c = 0; c < 16; ++c)
        x[c] = mine ? P[ti * kBgTSZ + c * kBgTS + row] : cpx<double>{1.0, 0.0};
#pragma unroll
      for (int c = 0; c < 16; ++c) {
        const double a = rdl_b(x[c].x, c);
        double y = __builtin_amdgcn_rsq(a);
        const double hh = 0.5 * a;
        y = fma(y, fma(-hh * y, y, 0.5), y);
        y = fma(y, fma(-hh * y, y, 0.5), y);
        x[c] = (lane == c) ? cpx<double>{a * y, 0.0} : cscale(x[c], y);
#pragma unroll
        for (int c2 = c + 1; c2 < 16; ++c2) {
          const double lx = rdl_b(x[c].x, c2), ly = rdl_b(x[c].y, c2);   // L[c2][c]
          x[c2].x -= x[c].x * lx + x[c].y * ly;
          x[c2].y -= x[c].y * lx - x[c].x * ly;
        }
      }
      const int gr_ = 16 * ti + row;
      if (mine && (!diag || wave == 0) && gr_ < K) {
#pragma unroll
        for (int c = 0; c < 16; ++c) {
          const int gc = 16 * j + c;
          if (gc < K && (!diag || row >= c)) Lf[pk_b(gc, K) + gr_ - gc] = x[c];
        }
      }
    }
    __syncthreads();   // column panel j of L is in HBM (workgroup-visible) before the next update
  }
}

hipError_t launch_zh_fmajor(const cpx<double>* Z, cpx<double>* X, int R, int F, hipStream_t st) {
  hipLaunchKernelGGL(k_zh_fmajor, dim3((F + 63) / 64, (R + 63) / 64), dim3(256), 0, st, Z, X, R, F);
  return hipGetLastError();
}

bool gram_big_ok(int K, int NV) { return K > 0 && K <= 16 * kBgMaxT && K * NV <= 8192; }

hipError_t launch_gram_big(const cpx<double>* Zh, const cpx<double>* Bh, cpx<double>* X,
                           cpx<double>* L, cpx<double>* h, int F, int K, int ni, double rho, int NV,
                           hipStream_t st, bool factor) {
  if (!gram_big_ok(K, NV)) return hipErrorInvalidValue;
  const int R = ni * K;
  hipLaunchKernelGGL(k_zh_fmajor, dim3((F + 63) / 64, (R + 63) / 64), dim3(256), 0, st, Zh, X, R, F);
  const int T = (K + 15) / 16;
  // (J, f): the T workgroups of one frequency are dispatched together, so its slab of
  // code spectra is read from HBM once and re-read from L2
  hipLaunchKernelGGL(k_gram_big, dim3(T * F), dim3(256), 0, st, X, Bh, L, h, F, K, ni, rho, NV);
  if (factor) hipLaunchKernelGGL(k_chol_big, dim3(F), dim3(kBgCholNT), 0, st, L, F, K);
  return hipGetLastError();
}

hipError_t launch_chol_big(cpx<double>* L, int F, int K, hipStream_t st) {
  if (!gram_big_ok(K, 0)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_chol_big, dim3(F), dim3(kBgCholNT), 0, st, L, F, K);
  return hipGetLastError();
}

}  // namespace ccsc
