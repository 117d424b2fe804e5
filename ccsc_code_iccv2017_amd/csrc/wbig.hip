// D-factor in the reference's own Woodbury form for filter counts past the packed K x K
// Cholesky kernels (K > 400 in the consensus learners, K > 192 in the 2-3D learner): per
// frequency f of a block of ni patches (images)
//   (A_f^H A_f + rho I)^-1 = (I - A_f^H M_f^-1 A_f) / rho,   M_f = rho I + A_f A_f^H (ni x ni)
// -- precompute_H_hat_D's pinv branch (dP:230-236; L23:290 inverts the n x n form for every
// kernel_size), with M_f factored M_f = L_M L_M^H instead of inverted.  The per-f slot of
// K(K+1)/2 complex holds A_f (ni x K row-major) then L_M (ni x ni row-major, zeros above the
// diagonal), the layout of k_gram_wb (dstep.hip) for ni <= 8; here ni <= kWgMaxNi.
//   k_wbig_gram   one workgroup per f: A_f from the frequency-major slab of k_zh_fmajor
//                 (gramchol_big.hip) into the slot, M_f's lower triangle accumulated in LDS
//                 over column chunks of A_f staged through LDS, its Cholesky in LDS
//                 (right-looking, one column per step), h_f = A_f^H b_f when NV > 0;
//   k_wbig_solve  one workgroup per (block, f), per view: r = h + rho C, t = A r (wave rows,
//                 lane-strided columns, wave sums), L_M L_M^H s = t (one wave), x = (r - A^H s)/rho.
// Both are L2/latency-bound generality paths (few frequencies per CU at these K), not the
// benchmark's: the headline K = 100 block runs gramchol.hip + k_dsolve_tile.
#include "kernels.hpp"

namespace ccsc {

constexpr int kWgNT = 256;
constexpr int kWgKC = 16;   // A_f columns per LDS chunk of the Gram

__device__ __forceinline__ int tri_idx(int p, int q) { return p * (p + 1) / 2 + q; }   // q <= p

// wave sum of a double (every lane gets the total)
__device__ __forceinline__ double wg_wave_sum(double v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__global__ __launch_bounds__(kWgNT) void k_wbig_gram(const cpx<double>* __restrict__ X,
                                                     const cpx<double>* __restrict__ Bh,
                                                     cpx<double>* __restrict__ L,
                                                     cpx<double>* __restrict__ h, int F, int K,
                                                     int ni, double rho, int NV, int64_t Kp) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  cpx<double>* sM = reinterpret_cast<cpx<double>*>(smem);          // lower triangle of M_f
  cpx<double>* sA = sM + kWgMaxNi * (kWgMaxNi + 1) / 2;              // [ni][kWgKC] chunk
  const int f = blockIdx.x;
  const int tid = threadIdx.x;
  const int nt = ni * (ni + 1) / 2;
  const cpx<double>* A = X + (int64_t)f * ni * K;                    // A_f row-major
  cpx<double>* slot = L + (int64_t)f * Kp;
  for (int e = tid; e < ni * K; e += kWgNT) slot[e] = A[e];
  for (int e = tid; e < nt; e += kWgNT) sM[e] = {0.0, 0.0};
  for (int k0 = 0; k0 < K; k0 += kWgKC) {
    __syncthreads();
    for (int e = tid; e < ni * kWgKC; e += kWgNT) {
      const int p = e / kWgKC, c = e - p * kWgKC;
      sA[e] = (k0 + c < K) ? A[(int64_t)p * K + k0 + c] : cpx<double>{0.0, 0.0};
    }
    __syncthreads();
    // M[p][q] += sum_k A[p][k] conj(A[q][k]) (each entry owned by one thread)
    for (int e = tid; e < nt; e += kWgNT) {
      int p = (int)((sqrt(8.0 * e + 1.0) - 1.0) * 0.5);
      while (tri_idx(p, 0) > e) --p;
      while (tri_idx(p + 1, 0) <= e) ++p;
      const int q = e - tri_idx(p, 0);
      cpx<double> acc = sM[e];
#pragma unroll
      for (int c = 0; c < kWgKC; ++c) acc = cmacc(acc, sA[q * kWgKC + c], sA[p * kWgKC + c]);
      sM[e] = acc;
    }
  }
  __syncthreads();
  for (int p = tid; p < ni; p += kWgNT) sM[tri_idx(p, p)] = {sM[tri_idx(p, p)].x + rho, 0.0};
  // right-looking Cholesky of M_f in LDS
  for (int j = 0; j < ni; ++j) {
    __syncthreads();
    const double d = sqrt(sM[tri_idx(j, j)].x);
    const double inv = 1.0 / d;
    __syncthreads();
    if (tid == 0) sM[tri_idx(j, j)] = {d, 0.0};
    for (int i = j + 1 + tid; i < ni; i += kWgNT) sM[tri_idx(i, j)] = cscale(sM[tri_idx(i, j)], inv);
    __syncthreads();
    const int m = ni - j - 1;   // trailing triangle rows j+1..ni-1
    for (int e = tid; e < m * (m + 1) / 2; e += kWgNT) {
      int a = (int)((sqrt(8.0 * e + 1.0) - 1.0) * 0.5);
      while (tri_idx(a, 0) > e) --a;
      while (tri_idx(a + 1, 0) <= e) ++a;
      const int b = e - tri_idx(a, 0);
      const int i = j + 1 + a, q = j + 1 + b;   // q <= i
      const cpx<double> lij = sM[tri_idx(i, j)], lqj = sM[tri_idx(q, j)];
      sM[tri_idx(i, q)] = cmsub(sM[tri_idx(i, q)], lij, cpx<double>{lqj.x, -lqj.y});
    }
  }
  __syncthreads();
  for (int e = tid; e < ni * ni; e += kWgNT) {
    const int p = e / ni, q = e - p * ni;
    slot[(int64_t)ni * K + e] = q <= p ? sM[tri_idx(p, q)] : cpx<double>{0.0, 0.0};
  }
  // h[f][uv][k] = sum_p conj(A[p][k]) B[p][uv][f]
  for (int e = tid; e < NV * K; e += kWgNT) {
    const int uv = e / K, k = e - uv * K;
    cpx<double> acc = {0.0, 0.0};
    for (int p = 0; p < ni; ++p)
      acc = cmacc(acc, A[(int64_t)p * K + k], Bh[((int64_t)p * NV + uv) * F + f]);
    h[((int64_t)f * NV + uv) * K + k] = acc;
  }
}

__global__ __launch_bounds__(kWgNT) void k_wbig_solve(const cpx<double>* __restrict__ L,
                                                      const cpx<double>* __restrict__ h,
                                                      const cpx<double>* __restrict__ Ch,
                                                      cpx<double>* __restrict__ Dh, int F, int K,
                                                      int ni, double rho, int NV, int64_t Kp) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  cpx<double>* sL = reinterpret_cast<cpx<double>*>(smem);   // L_M lower triangle
  cpx<double>* sT = sL + kWgMaxNi * (kWgMaxNi + 1) / 2;     // t, then y, then s (ni)
  cpx<double>* sR = sT + kWgMaxNi;                          // r (K)
  const int64_t blk = blockIdx.x / F;
  const int f = (int)(blockIdx.x - blk * F);
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const cpx<double>* slot = L + (blk * F + f) * Kp;
  const cpx<double>* A = slot;
  for (int e = tid; e < ni * (ni + 1) / 2; e += kWgNT) {
    int p = (int)((sqrt(8.0 * e + 1.0) - 1.0) * 0.5);
    while (tri_idx(p, 0) > e) --p;
    while (tri_idx(p + 1, 0) <= e) ++p;
    const int q = e - tri_idx(p, 0);
    sL[e] = slot[(int64_t)ni * K + p * ni + q];
  }
  const int64_t cs = (int64_t)NV * F;   // C / Dh: [blk][k][uv][F]
  const cpx<double>* Cb = Ch + blk * K * cs;
  cpx<double>* Db = Dh + blk * K * cs;
  const cpx<double>* hb = h + (blk * F + f) * (int64_t)NV * K;
  for (int uv = 0; uv < NV; ++uv) {
    __syncthreads();
    for (int k = tid; k < K; k += kWgNT) {
      const cpx<double> c = Cb[(int64_t)k * cs + (int64_t)uv * F + f], hv = hb[(int64_t)uv * K + k];
      sR[k] = {hv.x + rho * c.x, hv.y + rho * c.y};
    }
    __syncthreads();
    // t_p = sum_k A[p][k] r_k: rows over the waves, columns over the lanes
    for (int p = wave; p < ni; p += kWgNT / 64) {
      double tx = 0.0, ty = 0.0;
      for (int k = lane; k < K; k += 64) {
        const cpx<double> a = A[(int64_t)p * K + k], r = sR[k];
        tx = fma(a.x, r.x, fma(-a.y, r.y, tx));
        ty = fma(a.x, r.y, fma(a.y, r.x, ty));
      }
      tx = wg_wave_sum(tx);
      ty = wg_wave_sum(ty);
      if (lane == 0) sT[p] = {tx, ty};
    }
    __syncthreads();
    // L_M y = t, L_M^H s = y on wave 0 (column-oriented, lanes over rows i, i + 64)
    if (wave == 0) {
      for (int j = 0; j < ni; ++j) {
        const cpx<double> yj = cscale(sT[j], 1.0 / sL[tri_idx(j, j)].x);
        __builtin_amdgcn_wave_barrier();
        if (lane == 0) sT[j] = yj;
        for (int i = j + 1 + lane; i < ni; i += 64) sT[i] = cmsub(sT[i], sL[tri_idx(i, j)], yj);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      }
      for (int j = ni - 1; j >= 0; --j) {
        const cpx<double> sj = cscale(sT[j], 1.0 / sL[tri_idx(j, j)].x);
        __builtin_amdgcn_wave_barrier();
        if (lane == 0) sT[j] = sj;
        // rows i < j lose conj(L[j][i]) s_j
        for (int i = lane; i < j; i += 64) {
          const cpx<double> l = sL[tri_idx(j, i)];
          sT[i] = cmsub(sT[i], cpx<double>{l.x, -l.y}, sj);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      }
    }
    __syncthreads();
    // x_k = (r_k - sum_p conj(A[p][k]) s_p) / rho
    const double irho = 1.0 / rho;
    for (int k = tid; k < K; k += kWgNT) {
      cpx<double> acc = sR[k];
      for (int p = 0; p < ni; ++p) acc = cmsubc(acc, A[(int64_t)p * K + k], sT[p]);
      Db[(int64_t)k * cs + (int64_t)uv * F + f] = cscale(acc, irho);
    }
  }
}

bool wbig_ok(int K, int ni) {
  return K > 0 && ni >= 1 && ni <= kWgMaxNi && K <= 4096 &&
         (int64_t)ni * K + (int64_t)ni * ni <= (int64_t)K * (K + 1) / 2;
}

size_t wbig_workspace(int K, int ni, int F) { return (size_t)ni * K * F * sizeof(cpx<double>); }

hipError_t launch_wbig_gram(const cpx<double>* Zh, const cpx<double>* Bh, cpx<double>* X,
                            cpx<double>* L, cpx<double>* h, int F, int K, int ni, double rho, int NV,
                            hipStream_t st) {
  if (!wbig_ok(K, ni)) return hipErrorInvalidValue;
  const hipError_t e = launch_zh_fmajor(Zh, X, ni * K, F, st);
  if (e != hipSuccess) return e;
  const size_t smem = ((size_t)kWgMaxNi * (kWgMaxNi + 1) / 2 + (size_t)kWgMaxNi * kWgKC) * 16;
  hipLaunchKernelGGL(k_wbig_gram, dim3(F), dim3(kWgNT), smem, st, X, Bh, L, h, F, K, ni, rho, NV,
                     (int64_t)K * (K + 1) / 2);
  return hipGetLastError();
}

hipError_t launch_wbig_solve(const cpx<double>* L, const cpx<double>* h, const cpx<double>* Ch,
                             cpx<double>* Dh, int nblocks, int F, int K, int ni, double rho, int NV,
                             hipStream_t st) {
  if (nblocks <= 0) return hipSuccess;
  if (!wbig_ok(K, ni)) return hipErrorInvalidValue;
  const size_t smem = ((size_t)kWgMaxNi * (kWgMaxNi + 1) / 2 + kWgMaxNi + (size_t)K) * 16;
  if (smem > 160 * 1024) return hipErrorInvalidValue;
  if ((int64_t)nblocks * F >= ((int64_t)1 << 31)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_wbig_solve, dim3((unsigned)((int64_t)nblocks * F)), dim3(kWgNT), smem, st, L,
                     h, Ch, Dh, F, K, ni, rho, NV, (int64_t)K * (K + 1) / 2);
  return hipGetLastError();
}

}  // namespace ccsc
