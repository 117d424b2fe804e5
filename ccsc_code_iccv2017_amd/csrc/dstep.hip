// D-step per-frequency solves (gfx950).
//
// Reference: precompute_H_hat_D (dP:221-237) forms, for every frequency f of
// a block, Sinv_f = 1/rho*I - 1/rho*A'*pinv(rho*I + A*A')*A  (A = ni x K code
// spectra) == (A'A + rho I)^-1, and solve_conv_term_D (dP:252-276) applies
// x_f = Sinv_f (A'b_f + rho c_f) once per d-iteration.
//
// Here the precompute builds G_f = A'A + rho I and h_f = A'b_f in fp64 and
// stores the Cholesky factor L_f (packed lower, column-major, K(K+1)/2
// complex); every d-iteration streams L_f once and does the two triangular
// solves.  Only the half spectrum is solved: for real data S_{-f} = conj(S_f).
#include "kernels.hpp"
#include <algorithm>
#include <cstdlib>

namespace ccsc {

constexpr int kGramNT = 256;
constexpr int kGramTS = 5;   // register tile (rows x cols) of G per thread
constexpr int kGramPC = 16;  // patches staged in LDS per chunk

__device__ __forceinline__ int pk_off(int j, int K) { return j * K - (j * (j - 1)) / 2; }

// ---------------------------------------------------------------------------
// Blocked right-looking Cholesky G = L L^H of the packed lower Hermitian G in LDS
// (column-major, pk_off), in place, K <= 128, by one workgroup of kGramNT threads.
// Panels of kCholNB columns are factored by wave 0 in registers (rows over the
// lanes, pivot rows by shuffles: no workgroup barrier inside a panel); then every
// wave applies the rank-kCholNB update to the trailing lower triangle with
// kCholT x kCholT register tiles, one LDS read-modify-write per element per
// panel.  Two barriers per panel instead of two per column: the column-by-column
// form spent its time in LDS latency chains (measured 2.9 of 4.2 ms per block
// launch at K = 100).
// ---------------------------------------------------------------------------
constexpr int kCholNB = 8;
constexpr int kCholT = 2;

// broadcast of lane `l` (wave-uniform) through v_readlane: a scalar-register
// hop of a few cycles, where a shuffle is an LDS-crossbar round trip
__device__ __forceinline__ double readlane(double v, int l) {
  return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), l),
                          __builtin_amdgcn_readlane(__double2loint(v), l));
}
template <typename T>
__device__ __forceinline__ cpx<T> readlane_c(cpx<T> v, int l) {
  return {readlane(v.x, l), readlane(v.y, l)};
}

// Full-wave fp64 sum through DPP (VALU lane moves, no LDS): quad swaps, then
// half-row and row mirrors leave each 16-lane row's sum in all its lanes; the
// four row sums are combined through v_readlane.  Result in every lane.  The
// xor-shuffle form (wave_sum) costs 12 ds_bpermute round trips per double.
// (mov_dpp: every control used here gives each lane a valid source, so the old value is
// dead -- update_dpp(0, ...) spent a v_mov of the zero per DPP move)
template <int CTRL>
__device__ __forceinline__ double dpp_mov(double v) {
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xF, 0xF, true);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xF, 0xF, true);
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double wave_sum_dpp(double v) {
  v += dpp_mov<0xB1>(v);    // quad_perm [1,0,3,2]
  v += dpp_mov<0x4E>(v);    // quad_perm [2,3,0,1]
  v += dpp_mov<0x141>(v);   // row_half_mirror
  v += dpp_mov<0x140>(v);   // row_mirror
  return (readlane(v, 0) + readlane(v, 16)) + (readlane(v, 32) + readlane(v, 48));
}

template <typename T>
__device__ __forceinline__ void chol_blocked(cpx<T>* sG, int K) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int j0 = 0; j0 < K; j0 += kCholNB) {
    const int jb = min(kCholNB, K - j0);
    if (wave == 0) {
      cpx<T> P[2][kCholNB];  // rows r = j0 + lane + 64 t of the panel columns j0 .. j0+jb-1
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int r = j0 + lane + 64 * t;
#pragma unroll
        for (int c = 0; c < kCholNB; ++c) {
          const int j = j0 + c;
          P[t][c] = ldc_if(c < jb && r < K && r >= j, sG + pk_off(j, K) + r - j);
        }
      }
#pragma unroll
      for (int c = 0; c < kCholNB; ++c) {
        if (c < jb) {
          const int j = j0 + c;
          const T djj = sqrt(readlane(P[0][c].x, c));  // row j sits in lane c
          const T inv = (T)1 / djj;
#pragma unroll
          for (int t = 0; t < 2; ++t) {
            const int r = j0 + lane + 64 * t;
            if (r > j) P[t][c] = cscale(P[t][c], inv);
            else if (r == j) P[t][c] = {djj, (T)0};
          }
          // G[r][j0+c2] -= G[r][j] conj(G[j0+c2][j]) inside the panel
#pragma unroll
          for (int c2 = c + 1; c2 < kCholNB; ++c2) {
            if (c2 < jb) {
              const cpx<T> g = readlane_c(P[0][c], c2);
#pragma unroll
              for (int t = 0; t < 2; ++t) {
                const int r = j0 + lane + 64 * t;
                if (r >= j0 + c2) {
                  P[t][c2].x -= P[t][c].x * g.x + P[t][c].y * g.y;
                  P[t][c2].y -= P[t][c].y * g.x - P[t][c].x * g.y;
                }
              }
            }
          }
        }
      }
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int r = j0 + lane + 64 * t;
#pragma unroll
        for (int c = 0; c < kCholNB; ++c) {
          const int j = j0 + c;
          if (c < jb && r < K && r >= j) sG[pk_off(j, K) + r - j] = P[t][c];
        }
      }
    }
    __syncthreads();
    // trailing update G[i][l] -= sum_c G[i][j0+c] conj(G[l][j0+c]),  b0 <= l <= i < K
    const int b0 = j0 + jb;
    const int mt = K - b0;
    if (mt > 0) {
      const int nt = (mt + kCholT - 1) / kCholT;
      const int ntiles = nt * (nt + 1) / 2;
      for (int q = tid; q < ntiles; q += kGramNT) {
        int I = (int)((sqrt(8.0 * q + 1.0) - 1.0) * 0.5);
        while ((I + 1) * (I + 2) / 2 <= q) ++I;
        while (I * (I + 1) / 2 > q) --I;
        const int J = q - I * (I + 1) / 2;
        const int i0 = b0 + I * kCholT, l0 = b0 + J * kCholT;
        cpx<T> acc[kCholT][kCholT];
#pragma unroll
        for (int a = 0; a < kCholT; ++a)
#pragma unroll
          for (int b = 0; b < kCholT; ++b) acc[a][b] = {(T)0, (T)0};
        for (int c = 0; c < jb; ++c) {
          const int j = j0 + c;
          const cpx<T>* col = sG + pk_off(j, K) - j;   // col[r] = G[r][j]
          cpx<T> ai[kCholT], bl[kCholT];
#pragma unroll
          for (int a = 0; a < kCholT; ++a) {
            ai[a] = (i0 + a < K) ? col[i0 + a] : cpx<T>{(T)0, (T)0};
            bl[a] = (l0 + a < K) ? col[l0 + a] : cpx<T>{(T)0, (T)0};
          }
#pragma unroll
          for (int a = 0; a < kCholT; ++a)
#pragma unroll
            for (int b = 0; b < kCholT; ++b) {
              acc[a][b].x += ai[a].x * bl[b].x + ai[a].y * bl[b].y;
              acc[a][b].y += ai[a].y * bl[b].x - ai[a].x * bl[b].y;
            }
        }
#pragma unroll
        for (int b = 0; b < kCholT; ++b) {
          const int l = l0 + b;
          if (l < K) {
            cpx<T>* cl = sG + pk_off(l, K) - l;
#pragma unroll
            for (int a = 0; a < kCholT; ++a) {
              const int i = i0 + a;
              if (i < K && i >= l) cl[i] = csub(cl[i], acc[a][b]);
            }
          }
        }
      }
    }
    __syncthreads();
  }
}

// one workgroup per frequency (XCD-aware: consecutive f share an XCD's L2)
constexpr int kGramHPT = 8;  // (view, filter) right-hand-side entries per thread

// h[f][uv][k] = sum_p conj(A[p][k]) B[p][uv][f] for NV views (4D: the same A_f
// serves every view, L4:252 replicates it, so one Cholesky per spatial f).
template <typename T>
__global__ __launch_bounds__(kGramNT) void k_gram_chol(const cpx<T>* __restrict__ Zh,
                                                       const cpx<T>* __restrict__ Bh,
                                                       cpx<T>* __restrict__ L,
                                                       cpx<T>* __restrict__ h, int F, int K,
                                                       int ni, T rho, int NV) {
  const int per = gridDim.x >> 3;
  const int f = (blockIdx.x & 7) * per + (blockIdx.x >> 3);
  if (f >= F) return;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  cpx<T>* sG = reinterpret_cast<cpx<T>*>(smem);           // packed G, Kp entries
  const int Kp = K * (K + 1) / 2;
  cpx<T>* sA = sG;                                          // chunk [PC][K] (aliases sG)
  cpx<T>* sB = sA + kGramPC * K;                            // [PC][NV]
  const int tid = threadIdx.x;
  const int Kt = (K + kGramTS - 1) / kGramTS;
  const int ntiles = Kt * (Kt + 1) / 2;
  const bool act = tid < ntiles;
  int I = 0, J = 0;
  if (act) {
    I = (int)((sqrt(8.0 * tid + 1.0) - 1.0) * 0.5);
    while ((I + 1) * (I + 2) / 2 <= tid) ++I;
    while (I * (I + 1) / 2 > tid) --I;
    J = tid - I * (I + 1) / 2;
  }
  cpx<T> acc[kGramTS][kGramTS];
#pragma unroll
  for (int a = 0; a < kGramTS; ++a)
#pragma unroll
    for (int b = 0; b < kGramTS; ++b) acc[a][b] = {(T)0, (T)0};
  cpx<T> hacc[kGramHPT];
#pragma unroll
  for (int i = 0; i < kGramHPT; ++i) hacc[i] = {(T)0, (T)0};
  const int KV = K * NV;

  for (int p0 = 0; p0 < ni; p0 += kGramPC) {
    const int pc = min(kGramPC, ni - p0);
    __syncthreads();
    for (int idx = tid; idx < pc * K; idx += kGramNT) {
      const int pp = idx / K, k = idx - pp * K;
      sA[idx] = Zh[((int64_t)(p0 + pp) * K + k) * F + f];
    }
    for (int q = tid; q < pc * NV; q += kGramNT)
      sB[q] = Bh[(int64_t)(p0 * NV + q) * F + f];   // B[p][uv][f], q = pp*NV + uv
    __syncthreads();
    if (act) {
      for (int pp = 0; pp < pc; ++pp) {
        const cpx<T>* a = sA + pp * K;
        cpx<T> ai[kGramTS], aj[kGramTS];
#pragma unroll
        for (int t = 0; t < kGramTS; ++t) {
          const int ri = I * kGramTS + t, cj = J * kGramTS + t;
          ai[t] = (ri < K) ? a[ri] : cpx<T>{(T)0, (T)0};
          aj[t] = (cj < K) ? a[cj] : cpx<T>{(T)0, (T)0};
        }
#pragma unroll
        for (int u = 0; u < kGramTS; ++u)
#pragma unroll
          for (int v = 0; v < kGramTS; ++v) acc[u][v] = cmacc(acc[u][v], ai[u], aj[v]);
      }
    }
#pragma unroll
    for (int i = 0; i < kGramHPT; ++i) {
      const int q = tid + i * kGramNT;   // q = uv*K + k
      if (q < KV) {
        const int uv = q / K, k = q - uv * K;
        for (int pp = 0; pp < pc; ++pp)
          hacc[i] = cmacc(hacc[i], sA[pp * K + k], sB[pp * NV + uv]);
      }
    }
  }
  __syncthreads();  // chunk buffer (aliasing sG) no longer read
  if (act) {
#pragma unroll
    for (int u = 0; u < kGramTS; ++u)
#pragma unroll
      for (int v = 0; v < kGramTS; ++v) {
        const int row = I * kGramTS + u, col = J * kGramTS + v;
        if (row < K && col <= row) {
          cpx<T> g = acc[u][v];
          if (row == col) {
            g.x += rho;
            g.y = (T)0;
          }
          sG[pk_off(col, K) + row - col] = g;
        }
      }
  }
#pragma unroll
  for (int i = 0; i < kGramHPT; ++i) {
    const int q = tid + i * kGramNT;
    if (q < KV) h[(int64_t)f * KV + q] = hacc[i];
  }
  __syncthreads();

  chol_blocked(sG, K);
  cpx<T>* Lf = L + (int64_t)f * Kp;
  for (int q = tid; q < Kp; q += kGramNT) Lf[q] = sG[q];
}

template <typename T>
hipError_t launch_gram_chol(const cpx<T>* Zh, const cpx<T>* Bh, cpx<T>* L, cpx<T>* h, int F,
                            int K, int ni, T rho, int NV, hipStream_t st) {
  const int Kt = (K + kGramTS - 1) / kGramTS;
  if (Kt * (Kt + 1) / 2 > kGramNT) return hipErrorInvalidValue;
  if (K * NV > kGramHPT * kGramNT) return hipErrorInvalidValue;
  if (K > 128) return hipErrorInvalidValue;  // chol_blocked: two panel rows per lane
  const int Kp = K * (K + 1) / 2;
  size_t sm = (size_t)Kp * sizeof(cpx<T>);
  const size_t sm2 = (size_t)(kGramPC * K + kGramPC * NV) * sizeof(cpx<T>);
  if (sm2 > sm) sm = sm2;
  const int grid = ((F + 7) / 8) * 8;
  hipLaunchKernelGGL(k_gram_chol<T>, dim3(grid), dim3(kGramNT), sm, st, Zh, Bh, L, h, F, K, ni,
                     rho, NV);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// d-solve: one wave per (block, f); rows of the K-vector are spread over the
// 64 lanes (RPL rows per lane).  Both triangular solves are column axpys with
// the pivot broadcast by v_readlane: forward with the contiguous packed column
// (coalesced), backward with each lane's own column (L^H's row).
// ---------------------------------------------------------------------------
template <typename T>
__device__ __forceinline__ cpx<T> shfl_c(cpx<T> v, int src) {
  return {__shfl(v.x, src, 64), __shfl(v.y, src, 64)};
}

// NV right-hand sides per (block, f) share one factor (4D views, L4:281-308;
// the W wavelengths of the 2-3D learner, L23:293).  They are solved NVB at a
// time in one sweep over the factor, so L is streamed ceil(NV/NVB) times
// instead of NV times.  The factor's columns are read in blocks of kDsJB per
// wave (one load batch per block, address-independent of the solve) so their
// latency is paid once per block instead of once per column.
constexpr int kDsJB = 6;

// x[u] for a wave-uniform u < RPL (unrolled selects: no runtime register indexing)
template <typename T, int RPL>
__device__ __forceinline__ cpx<T> pick_reg(const cpx<T> (&x)[RPL], int u) {
  cpx<T> r = x[0];
#pragma unroll
  for (int q = 1; q < RPL; ++q)
    if (u == q) r = x[q];
  return r;
}
template <typename T, int RPL>
__device__ __forceinline__ void put_reg(cpx<T> (&x)[RPL], int u, cpx<T> v) {
#pragma unroll
  for (int q = 0; q < RPL; ++q)
    if (u == q) x[q] = v;
}

template <typename T, int RPL, int NVB>
__global__ __launch_bounds__(256) void k_dsolve(const cpx<T>* __restrict__ L,
                                                const cpx<T>* __restrict__ h,
                                                const cpx<T>* __restrict__ Ch,
                                                cpx<T>* __restrict__ Dh, int F, int K, T rho,
                                                int fgroups, int NV) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int blk = blockIdx.x / fgroups;
  const int f = (blockIdx.x - blk * fgroups) * 4 + wave;
  if (f >= F) return;
  const int Kp = K * (K + 1) / 2;
  const cpx<T>* Lf = L + ((int64_t)blk * F + f) * Kp;
  const cpx<T> zero = {(T)0, (T)0};
  // lane row l = lane + 64u (clamped into the matrix): packed column l starts at
  // coff[u] + l (entry L[p][l] at coff[u] + p, p >= l)
  int il[RPL], coff[RPL];
#pragma unroll
  for (int u = 0; u < RPL; ++u) {
    il[u] = min(lane + 64 * u, K - 1);
    coff[u] = il[u] * K - (il[u] * (il[u] - 1)) / 2 - il[u];
  }
  for (int uv0 = 0; uv0 < NV; uv0 += NVB) {
  // views past NV solve a zero right-hand side (uniform, no divergence) and are not stored
  const int nvc = min(NVB, NV - uv0);
  cpx<T> x[NVB][RPL];
#pragma unroll
  for (int v = 0; v < NVB; ++v) {
    const int uv = uv0 + v;
    const cpx<T>* hf = h + (((int64_t)blk * F + f) * NV + uv) * K;
    const cpx<T>* Cb = Ch + (int64_t)blk * K * NV * F + (int64_t)uv * F;   // [blk][k][uv][F]
#pragma unroll
    for (int t = 0; t < RPL; ++t) {
      const int i = lane + 64 * t;
      if (v < nvc && i < K) {
        const cpx<T> c = Cb[(int64_t)i * NV * F + f];
        const cpx<T> hh = hf[i];
        x[v][t] = {hh.x + rho * c.x, hh.y + rho * c.y};
      } else {
        x[v][t] = zero;
      }
    }
  }
  // forward: L y = rhs (column axpy)
  for (int j0 = 0; j0 < K; j0 += kDsJB) {
    cpx<T> lc[kDsJB][RPL];
    T dg[kDsJB];
#pragma unroll
    for (int jj = 0; jj < kDsJB; ++jj) {
      const int j = min(j0 + jj, K - 1);
      const cpx<T>* col = Lf + (j * K - (j * (j - 1)) / 2) - j;   // col[i] = L[i][j]
      dg[jj] = col[j].x;
#pragma unroll
      for (int u = 0; u < RPL; ++u) lc[jj][u] = col[min(lane + 64 * u, K - 1)];
    }
#pragma unroll
    for (int jj = 0; jj < kDsJB; ++jj) {
      const int j = j0 + jj;
      if (j < K) {
        const int src = j & 63, tj = j >> 6;
        const T inv = (T)1 / dg[jj];
#pragma unroll
        for (int v = 0; v < NVB; ++v) {
          const cpx<T> xj = cscale(readlane_c(pick_reg<T, RPL>(x[v], tj), src), inv);
          if (lane == src) put_reg<T, RPL>(x[v], tj, xj);
#pragma unroll
          for (int u = 0; u < RPL; ++u) {
            const int i = lane + 64 * u;
            if (i > j && i < K) x[v][u] = cmsub(x[v][u], lc[jj][u], xj);
          }
        }
      }
    }
  }
  // backward, one right-hand side: column dot products (coalesced reads of
  // column p), wave-reduced.  With several right-hand sides per sweep the
  // reductions dominate and the column-axpy form below is faster; with one the
  // latter's per-lane column walk (64 lines per load) costs more than the
  // reductions (C2: 22 vs 42 ms per launch, with shuffle reductions).
  if constexpr (NVB == 1) {
  for (int j1 = K - 1; j1 >= 0; j1 -= kDsJB) {
    cpx<T> lc[kDsJB][RPL];
    T dg[kDsJB];
#pragma unroll
    for (int jj = 0; jj < kDsJB; ++jj) {
      const int j = max(j1 - jj, 0);
      const cpx<T>* col = Lf + (j * K - (j * (j - 1)) / 2) - j;
      dg[jj] = col[j].x;
#pragma unroll
      for (int u = 0; u < RPL; ++u) lc[jj][u] = col[min(lane + 64 * u, K - 1)];
    }
#pragma unroll
    for (int jj = 0; jj < kDsJB; ++jj) {
      const int j = j1 - jj;
      if (j >= 0) {
        const int src = j & 63, tj = j >> 6;
        const T inv = (T)1 / dg[jj];
#pragma unroll
        for (int v = 0; v < NVB; ++v) {
          cpx<T> part = zero;
#pragma unroll
          for (int u = 0; u < RPL; ++u) {
            const int i = lane + 64 * u;
            if (i > j && i < K) part = cmacc(part, lc[jj][u], x[v][u]);
          }
          part.x = wave_sum_dpp(part.x);
          part.y = wave_sum_dpp(part.y);
          if (lane == src) put_reg<T, RPL>(x[v], tj, cscale(csub(pick_reg<T, RPL>(x[v], tj), part), inv));
        }
      }
    }
  }
  } else {
  // backward: L^H x = y, also as column axpys: once x_p is final, every row
  // l < p loses conj(L[p][l]) x_p.  L[p][l] sits in column l, so lane l walks
  // its own packed column upwards (8 consecutive entries per block = one
  // 128-B line per lane); no cross-lane reductions.
  for (int j1 = K - 1; j1 >= 0; j1 -= kDsJB) {
    cpx<T> lr[kDsJB][RPL];
    T dg[kDsJB];
#pragma unroll
    for (int jj = 0; jj < kDsJB; ++jj) {
      const int p = max(j1 - jj, 0);
      dg[jj] = Lf[p * K - (p * (p - 1)) / 2].x;                  // L[p][p]
#pragma unroll
      for (int u = 0; u < RPL; ++u) lr[jj][u] = Lf[coff[u] + max(p, il[u])];   // L[p][l]
    }
#pragma unroll
    for (int jj = 0; jj < kDsJB; ++jj) {
      const int p = j1 - jj;
      if (p >= 0) {
        const int src = p & 63, tp = p >> 6;
        const T inv = (T)1 / dg[jj];
#pragma unroll
        for (int v = 0; v < NVB; ++v) {
          const cpx<T> xp = cscale(readlane_c(pick_reg<T, RPL>(x[v], tp), src), inv);
          if (lane == src) put_reg<T, RPL>(x[v], tp, xp);
#pragma unroll
          for (int u = 0; u < RPL; ++u)
            if (lane + 64 * u < p) x[v][u] = cmsubc(x[v][u], lr[jj][u], xp);
        }
      }
    }
  }
  }
#pragma unroll
  for (int v = 0; v < NVB; ++v) {
    if (v < nvc) {
      cpx<T>* Db = Dh + (int64_t)blk * K * NV * F + (int64_t)(uv0 + v) * F;
#pragma unroll
      for (int t = 0; t < RPL; ++t) {
        const int i = lane + 64 * t;
        if (i < K) Db[(int64_t)i * NV * F + f] = x[v][t];
      }
    }
  }
  }  // view groups
}

template <typename T, int RPL, int NVB>
static void dsolve_go(dim3 grid, hipStream_t st, const cpx<T>* L, const cpx<T>* h,
                      const cpx<T>* Ch, cpx<T>* Dh, int F, int K, T rho, int fgroups, int NV) {
  hipLaunchKernelGGL((k_dsolve<T, RPL, NVB>), grid, dim3(256), 0, st, L, h, Ch,
                     Dh, F, K, rho, fgroups, NV);
}

template <typename T>
hipError_t launch_dsolve(const cpx<T>* L, const cpx<T>* h, const cpx<T>* Ch, cpx<T>* Dh,
                         int nblocks, int F, int K, T rho, int NV, hipStream_t st) {
  if (nblocks <= 0) return hipSuccess;
  const int fgroups = (F + 3) / 4;
  const dim3 grid((unsigned)(nblocks * fgroups));
  if (K <= 64) {
    if (NV == 1) dsolve_go<T, 1, 1>(grid, st, L, h, Ch, Dh, F, K, rho, fgroups, NV);
    else if (NV <= 4) dsolve_go<T, 1, 4>(grid, st, L, h, Ch, Dh, F, K, rho, fgroups, NV);
    else dsolve_go<T, 1, 8>(grid, st, L, h, Ch, Dh, F, K, rho, fgroups, NV);
  } else if (K <= 128) {
    // many right-hand sides (L23's W = 31 wavelengths): 8 per sweep over the factor
    if (NV == 1) dsolve_go<T, 2, 1>(grid, st, L, h, Ch, Dh, F, K, rho, fgroups, NV);
    else if (NV <= 4) dsolve_go<T, 2, 4>(grid, st, L, h, Ch, Dh, F, K, rho, fgroups, NV);
    else dsolve_go<T, 2, 8>(grid, st, L, h, Ch, Dh, F, K, rho, fgroups, NV);
  } else if (K <= 192) {
    if (NV == 1) dsolve_go<T, 3, 1>(grid, st, L, h, Ch, Dh, F, K, rho, fgroups, NV);
    else dsolve_go<T, 3, 4>(grid, st, L, h, Ch, Dh, F, K, rho, fgroups, NV);
  } else if (K <= 256) {   // factors of gramchol_big.hip
    if (NV == 1) dsolve_go<T, 4, 1>(grid, st, L, h, Ch, Dh, F, K, rho, fgroups, NV);
    else dsolve_go<T, 4, 4>(grid, st, L, h, Ch, Dh, F, K, rho, fgroups, NV);
  } else if (K <= 320) {
    if (NV == 1) dsolve_go<T, 5, 1>(grid, st, L, h, Ch, Dh, F, K, rho, fgroups, NV);
    else dsolve_go<T, 5, 4>(grid, st, L, h, Ch, Dh, F, K, rho, fgroups, NV);
  } else if (K <= 400) {
    if (NV == 1) dsolve_go<T, 7, 1>(grid, st, L, h, Ch, Dh, F, K, rho, fgroups, NV);
    else dsolve_go<T, 7, 4>(grid, st, L, h, Ch, Dh, F, K, rho, fgroups, NV);
  } else {
    return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Tile d-solve for the 2D headline block shape (NV = 1, 64 < K <= 112; C1/C2:
// K = 100, dP:252-276).  The factor's diagonal 16 x 16 tiles hold M_JJ = L_JJ^-1
// (k_invert_diag, once per precompute), so with r = h + rho C
//   forward   y_J = M_JJ (r_J - sum_{J' < J} L_JJ' y_J')
//   backward  x_J = M_JJ^H (y_J - sum_{I > J} L_IJ^H x_I)
// are tile matrix-vector products with no serial chain inside a tile.  One
// workgroup (4 waves) per (block, f) holds the T(T+1)/2 lower tiles in registers
// (lane (row = l & 15, cg = l >> 4) holds L[row][4 cg + q], q < 4), reads them once
// and runs both sweeps from registers: the factor crosses HBM once per solve where
// k_dsolve streams it twice.  Tile ownership (kDtMap) puts (J+1, J) on the wave that
// owns (J+1, J+1), so each sweep step is one phase between barriers:
//   forward phase J:  owners of (I, J), I > J+1: r_I -= L_IJ y_J;  the owner of
//                     (J+1, J): y_{J+1} = M (r_{J+1} - L_{J+1,J} y_J)
//   backward phase J: the owner of (J, J): x_J = M^H (y_J - sum_I P_IJ), then
//                     P_{J,J-1} = L_{J,J-1}^H x_J;  owners of (I, J-1), I > J: P_{I,J-1}
// (P double-buffered by phase parity): T + 1 barriers per sweep pair instead of 4T.
// ---------------------------------------------------------------------------
constexpr int kDtT = 7;                          // tiles per dimension (K <= 112)
constexpr int kDtTW = kDtT * (kDtT + 1) / 8;     // 7 tiles per wave
// (I, J) of wave w's tile s, packed I * 8 + J (see above: pairs (J+1, J), (J+1, J+1)
// share a wave; every column's off-diagonal tiles spread over the waves)
__constant__ const unsigned char kDtMap[4][kDtTW] = {
    {1 * 8 + 0, 1 * 8 + 1, 5 * 8 + 4, 5 * 8 + 5, 4 * 8 + 1, 4 * 8 + 2, 6 * 8 + 3},
    {2 * 8 + 1, 2 * 8 + 2, 6 * 8 + 5, 6 * 8 + 6, 4 * 8 + 0, 5 * 8 + 3, 6 * 8 + 4},
    {3 * 8 + 2, 3 * 8 + 3, 0 * 8 + 0, 2 * 8 + 0, 6 * 8 + 0, 5 * 8 + 1, 6 * 8 + 2},
    {4 * 8 + 3, 4 * 8 + 4, 3 * 8 + 0, 5 * 8 + 0, 3 * 8 + 1, 6 * 8 + 1, 5 * 8 + 2}};

// sum over the four 16-lane rows (lanes row, row + 16, row + 32, row + 48) through the
// gfx950 row-swap moves (VALU; the xor shuffles they replace were LDS bpermute round trips
// on the sweeps' serial chain): permlane16_swap pairs rows 0/1 and 2/3, permlane32_swap
// the two halves; each add sees the same two operands as v + shfl_xor(v, 16 | 32)
__device__ __forceinline__ double pl_pair_sum(double v, bool r32) {
  const int lo = __double2loint(v), hi = __double2hiint(v);
  if (r32) {
    const auto l = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
    const auto h = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
    return __hiloint2double(h[0], l[0]) + __hiloint2double(h[1], l[1]);
  }
  const auto l = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
  const auto h = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
  return __hiloint2double(h[0], l[0]) + __hiloint2double(h[1], l[1]);
}
__device__ __forceinline__ double xrow_sum(double v) {
  return pl_pair_sum(pl_pair_sum(v, false), true);
}
// Row sums of four complex values p[0..3] over each 16-lane row, reduce-scatter form:
// the eight doubles halve at each DPP level (ror 8, half-mirror, xor 2) and the last
// level sums one value (xor 1) -- 26 DPP moves and 15 adds instead of the 64 and 32 of
// eight row16_sums.  Lane r of the row ends with the sum of double (r >> 1) & 7, i.e.
// component (r >> 1) & 1 of p[r >> 2]; the even lanes store it to out[r >> 2].
__device__ __forceinline__ void row16_sum4_store(const cpx<double> (&p)[4], int r,
                                                 cpx<double>* out) {
  double v[8];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    v[2 * q] = p[q].x;
    v[2 * q + 1] = p[q].y;
  }
  const bool b3 = (r & 8) != 0, b2 = (r & 4) != 0, b1 = (r & 2) != 0;
  double w1[4], w2[2];
#pragma unroll
  for (int k = 0; k < 4; ++k) {   // partner r ^ 8
    const double keep = b3 ? v[k + 4] : v[k], send = b3 ? v[k] : v[k + 4];
    w1[k] = keep + dpp_mov<0x128>(send);   // row_ror:8
  }
#pragma unroll
  for (int k = 0; k < 2; ++k) {   // partner (r & 8) | (7 - (r & 7)): bit 2 flipped
    const double keep = b2 ? w1[k + 2] : w1[k], send = b2 ? w1[k] : w1[k + 2];
    w2[k] = keep + dpp_mov<0x141>(send);   // row_half_mirror
  }
  double w3;
  {                               // partner r ^ 2
    const double keep = b1 ? w2[1] : w2[0], send = b1 ? w2[0] : w2[1];
    w3 = keep + dpp_mov<0x4E>(send);       // quad_perm [2,3,0,1]
  }
  w3 += dpp_mov<0xB1>(w3);                 // quad_perm [1,0,3,2]
  if ((r & 1) == 0) reinterpret_cast<double*>(out)[r >> 1] = w3;
}
__device__ __forceinline__ void wave_sync_lds() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

// NV right-hand sides per (block, f) -- the 4D views, L23's W wavelengths -- are solved one
// after the other against the factor tiles the workgroup loaded once (k_dsolve streams the
// factor twice per group of up to 8 right-hand sides); layouts [blk][k][uv][F] (Ch, Dh) and
// [blk][f][uv][k] (h)
bool dsolve_tile_ok(int K, int NV) { return NV >= 1 && NV <= 64 && K > 64 && K <= 16 * kDtT; }

// NB right-hand sides share each barrier phase (NB = 1 for the single-view headline)
template <int NB>
__global__ __launch_bounds__(256) void k_dsolve_tile(const cpx<double>* __restrict__ L,
                                                     const cpx<double>* __restrict__ h,
                                                     const cpx<double>* __restrict__ Ch,
                                                     cpx<double>* __restrict__ Dh, int F, int K,
                                                     double rho, int NV) {
  __shared__ cpx<double> sr[NB][16 * kDtT], sy[NB][16 * kDtT], sx[NB][16 * kDtT],
      sp[2][NB][kDtT][16];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int row = lane & 15, cg = lane >> 4;
  // XCD-aware: workgroups i, i + 8, ... (one XCD) take neighbouring f, so the [blk][K][F]
  // right-hand sides and solutions they read and write share 128-B lines in one L2
  const int per = (F + 7) >> 3;
  const int blk = blockIdx.x / (8 * per), r8 = blockIdx.x - blk * 8 * per;
  const int f = (r8 & 7) * per + (r8 >> 3);
  if (f >= F) return;
  const int Tn = (K + 15) >> 4;
  const cpx<double>* Lf = L + ((int64_t)blk * F + f) * (K * (K + 1) / 2);
  const cpx<double> zero = {0.0, 0.0};
  int tI[kDtTW], tJ[kDtTW];   // wave-uniform; tiles past the grid get I = -1
#pragma unroll
  for (int s = 0; s < kDtTW; ++s) {
    const int m = kDtMap[wave][s];
    tI[s] = (m >> 3) < Tn ? (m >> 3) : -1;
    tJ[s] = m & 7;
  }
  cpx<double> Lt[kDtTW][4];
#pragma unroll
  for (int s = 0; s < kDtTW; ++s) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int R = 16 * tI[s] + row, C = 16 * tJ[s] + 4 * cg + q;
      Lt[s][q] = ldc_if(tI[s] >= 0 && R < K && C <= R, Lf + C * K - (C * (C - 1)) / 2 + R - C);
    }
  }
  // right-hand side uv: r = h + rho C (thread tid < K holds row tid), prefetched one batch ahead
  auto rhs = [&](int uv) {
    cpx<double> v = zero;
    if (tid < K && uv < NV) {
      const cpx<double> c = Ch[(((int64_t)blk * K + tid) * NV + uv) * F + f];
      const cpx<double> hh = h[(((int64_t)blk * F + f) * NV + uv) * K + tid];
      v = {hh.x + rho * c.x, hh.y + rho * c.y};
    }
    return v;
  };
  cpx<double> vn[NB];
#pragma unroll
  for (int b = 0; b < NB; ++b) vn[b] = rhs(b);
  // y = M v for the diagonal tile in slot s, v[i] in vbuf (LDS, this wave's own writes)
  auto diag_fwd = [&](const cpx<double> (&Mt)[4], const cpx<double>* vbuf, cpx<double>* ybuf) {
    cpx<double> v = zero;
#pragma unroll
    for (int q = 0; q < 4; ++q) v = cmac(v, Mt[q], vbuf[4 * cg + q]);
    v = {xrow_sum(v.x), xrow_sum(v.y)};
    if (cg == 0) ybuf[row] = v;
  };
  for (int uv0 = 0; uv0 < NV; uv0 += NB) {
    if (tid < 16 * Tn) {
#pragma unroll
      for (int b = 0; b < NB; ++b) sr[b][tid] = vn[b];
    }
    __syncthreads();
#pragma unroll
    for (int b = 0; b < NB; ++b) vn[b] = rhs(uv0 + NB + b);
    // ---- forward ----
#pragma unroll
    for (int s = 0; s < kDtTW; ++s)
      if (tI[s] == 0 && tJ[s] == 0) {
#pragma unroll
        for (int b = 0; b < NB; ++b) diag_fwd(Lt[s], sr[b], sy[b]);
      }
    __syncthreads();
    for (int J = 0; J + 1 < Tn; ++J) {
#pragma unroll
      for (int s = 0; s < kDtTW; ++s) {
        if (tJ[s] == J && tI[s] > J) {
#pragma unroll
          for (int b = 0; b < NB; ++b) {
            const cpx<double>* yJ = sy[b] + 16 * J;
            cpx<double> v = zero;
#pragma unroll
            for (int q = 0; q < 4; ++q) v = cmac(v, Lt[s][q], yJ[4 * cg + q]);
            v = {xrow_sum(v.x), xrow_sum(v.y)};
            cpx<double>* rI = sr[b] + 16 * tI[s];
            if (cg == 0) rI[row] = csub(rI[row], v);
          }
          if (tI[s] == J + 1) {
            // this wave also owns (J+1, J+1) (slot s + 1 by construction of kDtMap)
            wave_sync_lds();
#pragma unroll
            for (int b = 0; b < NB; ++b)
              diag_fwd(Lt[s + 1 < kDtTW ? s + 1 : s], sr[b] + 16 * tI[s], sy[b] + 16 * (J + 1));
          }
        }
      }
      __syncthreads();
    }
    // ---- backward ----
    for (int J = Tn - 1; J >= 0; --J) {
      const int pb = J & 1;   // partials P_IJ were written in the previous phase into sp[pb]
#pragma unroll
      for (int s = 0; s < kDtTW; ++s) {
        if (tI[s] == J && tJ[s] == J) {
#pragma unroll
          for (int b = 0; b < NB; ++b) {
            cpx<double> v = sy[b][16 * J + row];
            for (int I = J + 1; I < Tn; ++I) v = csub(v, sp[pb][b][I][row]);
            cpx<double> p[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) p[q] = cmulc(Lt[s][q], v);   // conj(M[row][c]) v[row]
            row16_sum4_store(p, row, sx[b] + 16 * J + 4 * cg);
          }
          wave_sync_lds();
        }
      }
      if (J == 0) break;
      // partials for column block J - 1 (x_I known for I >= J after the step above)
#pragma unroll
      for (int s = 0; s < kDtTW; ++s) {
        if (tJ[s] == J - 1 && tI[s] >= J) {
#pragma unroll
          for (int b = 0; b < NB; ++b) {
            const cpx<double> xr = sx[b][16 * tI[s] + row];
            cpx<double> p[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) p[q] = cmulc(Lt[s][q], xr);   // conj(L[row][c]) x[row]
            row16_sum4_store(p, row, &sp[pb ^ 1][b][tI[s]][4 * cg]);
          }
        }
      }
      __syncthreads();
    }
    __syncthreads();
    if (tid < K) {
#pragma unroll
      for (int b = 0; b < NB; ++b)
        if (uv0 + b < NV) Dh[(((int64_t)blk * K + tid) * NV + uv0 + b) * F + f] = sx[b][tid];
    }
  }
}

hipError_t launch_dsolve_tile(const cpx<double>* L, const cpx<double>* h, const cpx<double>* Ch,
                              cpx<double>* Dh, int nblocks, int F, int K, double rho, int NV,
                              hipStream_t st) {
  if (nblocks <= 0) return hipSuccess;
  if (!dsolve_tile_ok(K, NV)) return hipErrorInvalidValue;
  const dim3 grid((unsigned)(nblocks * 8 * ((F + 7) / 8)));
  // three right-hand sides per barrier phase (C3: one 0.1211, two 0.1165 -> three (163 VGPRs)
  // 0.0910 -> 0.0896 s per outer iteration after the GEMM changes; four: 169 VGPRs, two waves
  // per SIMD, 0.1217 s)
  if (NV == 1)
    hipLaunchKernelGGL(k_dsolve_tile<1>, grid, dim3(256), 0, st, L, h, Ch, Dh, F, K, rho, NV);
  else
    hipLaunchKernelGGL(k_dsolve_tile<3>, grid, dim3(256), 0, st, L, h, Ch, Dh, F, K, rho, NV);
  return hipGetLastError();
}

// In place: the diagonal 16 x 16 tiles of one block's F packed factors <- their
// inverses (the form k_dsolve_tile reads), once per precompute.  One wave per
// (f, tile J) item: L_JJ staged in LDS, lane c & 15 forms column c of M = L_JJ^-1 by
// forward substitution into the wave's LDS copy of M (each lane reads back only its
// own column; the four lanes of a column write the same values):
//   M[r][c] = (delta_rc - sum_{k<r} L[r][k] M[k][c]) / L[r][r],
// a row's 2r broadcast reads issued together.
__global__ __launch_bounds__(256) void k_invert_diag(cpx<double>* __restrict__ L, int F, int K,
                                                     int Tn) {
  __shared__ cpx<double> sL[4][16 * 17], sM[4][16 * 17];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, c = lane & 15;
  const int64_t item = (int64_t)blockIdx.x * 4 + wave;   // f * Tn + J
  if (item >= (int64_t)F * Tn) return;                   // wave-uniform
  const int f = (int)(item / Tn), J = (int)(item - (int64_t)f * Tn);
  cpx<double>* Lf = L + (int64_t)f * (K * (K + 1) / 2);
  cpx<double>* Lw = sL[wave];
  cpx<double>* Mw = sM[wave];
  for (int e = lane; e < 256; e += 64) {
    const int r = e & 15, cc = e >> 4, R = 16 * J + r, C = 16 * J + cc;
    Lw[cc * 17 + r] = (r >= cc && R < K) ? Lf[C * K - (C * (C - 1)) / 2 + R - C]
                                         : cpx<double>{(r == cc) ? 1.0 : 0.0, 0.0};
  }
  wave_sync_lds();
  for (int r = 0; r < 16; ++r) {
    cpx<double> s0 = {(r == c) ? 1.0 : 0.0, 0.0}, s1 = {0.0, 0.0};
#pragma unroll
    for (int k = 0; k < 15; ++k) {
      if (k < r) {
        const cpx<double> p = cmul(Lw[k * 17 + r], Mw[k * 17 + c]);
        if (k & 1) s1 = csub(s1, p);
        else s0 = csub(s0, p);
      }
    }
    Mw[r * 17 + c] = cscale(cadd(s0, s1), 1.0 / Lw[r * 17 + r].x);
  }
  if (lane < 16) {
    const int C = 16 * J + c;
    for (int r = c; r < 16 && 16 * J + r < K; ++r)
      Lf[C * K - (C * (C - 1)) / 2 + 16 * J + r - C] = Mw[r * 17 + c];
  }
}

hipError_t launch_invert_diag(cpx<double>* L, int F, int K, hipStream_t st) {
  const int Tn = (K + 15) >> 4;
  if (F <= 0 || Tn > kDtT) return hipErrorInvalidValue;
  const int64_t items = (int64_t)F * Tn;
  hipLaunchKernelGGL(k_invert_diag, dim3((unsigned)((items + 3) / 4)), dim3(256), 0, st, L, F, K,
                     Tn);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Woodbury form for blocks of ni << K patches (3D/4D: ni = sqrt(n) = 8, K = 49):
// (A^H A + rho I)^{-1} = (I - A^H M^{-1} A) / rho, M = rho I + A A^H (ni x ni) --
// the reference's own pinv(rho I + A A^H) form (dP:230-236, L3/L4 precompute),
// with M factored instead of inverted.  Per f: ni K + ni^2 complex instead of
// the K(K+1)/2 of the K x K factor, no K^3 factorisation, and a solve of
// 2 ni K + ni^2 complex MACs per right-hand side instead of K^2.
// One wave per f, lanes over k (RPL rows per lane); row p of M / L_M lives in
// lane p.
// ---------------------------------------------------------------------------
// The spectra the Woodbury kernels read and write are [.][k][..][F] (lanes over k stride
// F), so a wave's access touches one 16-B piece of K lines: the kWbWG waves of a workgroup
// take consecutive f (the neighbouring pieces of the same lines), and consecutive
// workgroups of one XCD (ids i, i + 8, ...) the next f's, so the lines are read and
// written whole from one L2 instead of piecewise from several.
constexpr int kWbWG = 8;
__device__ __forceinline__ int xcd_group(int ntot) {
  const int per = (int)((gridDim.x + 7) >> 3);
  const int g = (int)(blockIdx.x & 7) * per + (int)(blockIdx.x >> 3);
  return g < ntot ? g : -1;
}

// HT: h in the [k][uv][F] layout of Ch (block-local), which k_dsolve_wbs stages through LDS
// with the right-hand sides; else [f][uv][k]
template <typename T, int RPL, bool HT = false>
__global__ __launch_bounds__(64 * kWbWG) void k_gram_wb(const cpx<T>* __restrict__ Zh,
                                                        const cpx<T>* __restrict__ Bh,
                                                        cpx<T>* __restrict__ L,
                                                        cpx<T>* __restrict__ h, int F, int K,
                                                        int ni, T rho, int NV, int Kp) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int g = xcd_group((F + kWbWG - 1) / kWbWG);
  const int f = g * kWbWG + wave;
  if (g < 0 || f >= F) return;
  const cpx<T> zero = {(T)0, (T)0};
  cpx<T> a[kWbMaxNi][RPL];
#pragma unroll
  for (int p = 0; p < kWbMaxNi; ++p)
#pragma unroll
    for (int u = 0; u < RPL; ++u) {
      const int i = lane + 64 * u;
      a[p][u] = ldc_if(p < ni && i < K, Zh + ((int64_t)p * K + i) * F + f);
    }
  cpx<T>* slot = L + (int64_t)f * Kp;
#pragma unroll
  for (int p = 0; p < kWbMaxNi; ++p)
#pragma unroll
    for (int u = 0; u < RPL; ++u) {
      const int i = lane + 64 * u;
      if (p < ni && i < K) slot[p * K + i] = a[p][u];
    }
  // M[p][q] = rho delta_pq + sum_k A[p][k] conj(A[q][k]), q <= p (wave sums,
  // staged through LDS so that lane p picks up row p with static indices)
  __shared__ cpx<T> sM[kWbWG][kWbMaxNi * kWbMaxNi];
#pragma unroll
  for (int p = 0; p < kWbMaxNi; ++p)
#pragma unroll
    for (int q = 0; q <= p; ++q) {
      if (p < ni) {
        cpx<T> part = zero;
#pragma unroll
        for (int u = 0; u < RPL; ++u) part = cmacc(part, a[q][u], a[p][u]);
        cpx<T> v = {wave_sum_dpp(part.x), wave_sum_dpp(part.y)};
        if (p == q) v = {v.x + rho, (T)0};
        if (lane == 0) sM[wave][p * kWbMaxNi + q] = v;
      }
    }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  cpx<T> m[kWbMaxNi];
#pragma unroll
  for (int q = 0; q < kWbMaxNi; ++q)
    m[q] = ldc_if(lane < ni && q <= lane, &sM[wave][min(lane, kWbMaxNi - 1) * kWbMaxNi + q]);
  // right-looking Cholesky M = L_M L_M^H across the lanes
#pragma unroll
  for (int j = 0; j < kWbMaxNi; ++j) {
    if (j < ni) {
      const T d = sqrt(readlane(m[j].x, j));
      const T inv = (T)1 / d;
      if (lane == j) m[j] = {d, (T)0};
      if (lane > j && lane < ni) m[j] = cscale(m[j], inv);           // L[lane][j]
#pragma unroll
      for (int q = 0; q < kWbMaxNi; ++q) {
        if (q > j && q < ni) {
          const cpx<T> lq = readlane_c(m[j], q);                      // L[q][j]
          if (lane >= q && lane < ni) m[q] = cmsub(m[q], m[j], cpx<T>{lq.x, -lq.y});
        }
      }
    }
  }
  if (lane < ni) {
#pragma unroll
    for (int q = 0; q < kWbMaxNi; ++q)
      if (q < ni) {
        cpx<T> v = zero;
        if (q <= lane) v = m[q];
        slot[ni * K + lane * ni + q] = v;
      }
  }
  // h[f][uv][k] = sum_p conj(A[p][k]) B[p][uv][f]
  for (int uv = 0; uv < NV; ++uv) {
    cpx<T> acc[RPL];
#pragma unroll
    for (int u = 0; u < RPL; ++u) acc[u] = zero;
#pragma unroll
    for (int p = 0; p < kWbMaxNi; ++p) {
      if (p < ni) {
        const cpx<T> b = Bh[((int64_t)p * NV + uv) * F + f];
#pragma unroll
        for (int u = 0; u < RPL; ++u) acc[u] = cmacc(acc[u], a[p][u], b);
      }
    }
#pragma unroll
    for (int u = 0; u < RPL; ++u) {
      const int i = lane + 64 * u;
      if (i < K) h[HT ? ((int64_t)i * NV + uv) * F + f : ((int64_t)f * NV + uv) * K + i] = acc[u];
    }
  }
}

// One wave per (block, f), kWbWG consecutive f per workgroup (see k_gram_wb).
template <typename T, int RPL, int NVB>
__global__ __launch_bounds__(64 * kWbWG) void k_dsolve_wb(const cpx<T>* __restrict__ L,
                                                          const cpx<T>* __restrict__ h,
                                                          const cpx<T>* __restrict__ Ch,
                                                          cpx<T>* __restrict__ Dh, int F, int K,
                                                          T rho, int fgroups, int ntot, int NV,
                                                          int ni, int Kp) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int g = xcd_group(ntot);
  const int blk = g / fgroups;
  const int f = (g - blk * fgroups) * kWbWG + wave;
  if (g < 0 || f >= F) return;
  const cpx<T> zero = {(T)0, (T)0};
  const cpx<T>* slot = L + ((int64_t)blk * F + f) * Kp;
  cpx<T> a[kWbMaxNi][RPL];
#pragma unroll
  for (int p = 0; p < kWbMaxNi; ++p)
#pragma unroll
    for (int u = 0; u < RPL; ++u) {
      const int i = lane + 64 * u;
      a[p][u] = ldc_if(p < ni && i < K, slot + p * K + i);
    }
  // lane p: row p and column p of L_M, 1 / L_M[p][p]
  const cpx<T>* lm = slot + ni * K;
  cpx<T> lrow[kWbMaxNi], lcol[kWbMaxNi];
  const bool lp = lane < ni;
#pragma unroll
  for (int q = 0; q < kWbMaxNi; ++q) {
    lrow[q] = ldc_if(lp && q < ni, lm + lane * ni + q);
    lcol[q] = ldc_if(lp && q < ni, lm + q * ni + lane);
  }
  const T dinv = lp ? (T)1 / lm[lane * ni + lane].x : (T)0;
  const T irho = (T)1 / rho;
  for (int uv0 = 0; uv0 < NV; uv0 += NVB) {
    const int nvc = min(NVB, NV - uv0);
    cpx<T> r[NVB][RPL], t[NVB];
#pragma unroll
    for (int v = 0; v < NVB; ++v) {
      const int uv = uv0 + v;
      const cpx<T>* hf = h + (((int64_t)blk * F + f) * NV + uv) * K;
      const cpx<T>* Cb = Ch + (int64_t)blk * K * NV * F + (int64_t)uv * F;   // [blk][k][uv][F]
#pragma unroll
      for (int u = 0; u < RPL; ++u) {
        const int i = lane + 64 * u;
        if (v < nvc && i < K) {
          const cpx<T> c = Cb[(int64_t)i * NV * F + f];
          const cpx<T> hh = hf[i];
          r[v][u] = {hh.x + rho * c.x, hh.y + rho * c.y};
        } else {
          r[v][u] = zero;
        }
      }
      t[v] = zero;
    }
    // t = A r (lane p keeps t_p)
#pragma unroll
    for (int p = 0; p < kWbMaxNi; ++p) {
      if (p < ni) {
#pragma unroll
        for (int v = 0; v < NVB; ++v) {
          cpx<T> part = zero;
#pragma unroll
          for (int u = 0; u < RPL; ++u) part = cmac(part, a[p][u], r[v][u]);
          const cpx<T> s = {wave_sum_dpp(part.x), wave_sum_dpp(part.y)};
          if (lane == p) t[v] = s;
        }
      }
    }
    // M s = t: forward L_M y = t, backward L_M^H s = y (pivots via v_readlane)
#pragma unroll
    for (int j = 0; j < kWbMaxNi; ++j) {
      if (j < ni) {
        const T dj = readlane(dinv, j);
#pragma unroll
        for (int v = 0; v < NVB; ++v) {
          const cpx<T> yj = cscale(readlane_c(t[v], j), dj);
          if (lane == j) t[v] = yj;
          if (lane > j && lane < ni) t[v] = cmsub(t[v], lrow[j], yj);
        }
      }
    }
#pragma unroll
    for (int j = kWbMaxNi - 1; j >= 0; --j) {
      if (j < ni) {
        const T dj = readlane(dinv, j);
#pragma unroll
        for (int v = 0; v < NVB; ++v) {
          const cpx<T> sj = cscale(readlane_c(t[v], j), dj);
          if (lane == j) t[v] = sj;
          if (lane < j) t[v] = cmsubc(t[v], lcol[j], sj);         // conj(L_M[j][lane])
        }
      }
    }
    // x = (r - A^H s) / rho
#pragma unroll
    for (int p = 0; p < kWbMaxNi; ++p) {
      if (p < ni) {
#pragma unroll
        for (int v = 0; v < NVB; ++v) {
          const cpx<T> sp = readlane_c(t[v], p);
#pragma unroll
          for (int u = 0; u < RPL; ++u) r[v][u] = cmsubc(r[v][u], a[p][u], sp);
        }
      }
    }
#pragma unroll
    for (int v = 0; v < NVB; ++v) {
      if (v < nvc) {
        cpx<T>* Db = Dh + (int64_t)blk * K * NV * F + (int64_t)(uv0 + v) * F;
#pragma unroll
        for (int u = 0; u < RPL; ++u) {
          const int i = lane + 64 * u;
          if (i < K) Db[(int64_t)i * NV * F + f] = cscale(r[v][u], irho);
        }
      }
    }
  }
}

// Many right-hand sides per f (4D: the NV = U V views share A_f, L4 precompute): one wave
// per (block, f) with lanes over the views instead of k.  A_f and L_M are wave-uniform:
// copied once into the wave's LDS slice (the slot is contiguous) and read as broadcasts,
// so each lane runs t = A r, M s = t and x = (r - A^H s) / rho for its own view with no
// wave reductions -- the lanes-over-k form spends 2 ni NV of them per f on t.  With
// NV <= 32 the two half-waves take the two halves of the k range (H = 2: lane = 32 hh + v,
// rows hh KH .. hh KH + KH - 1, KH = ceil(K / 2)): half the rows of r per lane, and the
// half sums of t meet through v_permlane32_swap.  r stays in registers (KR >= KH rows).
constexpr int kWbvMaxNV = 64;
constexpr int kWbvCH = 8;   // rows of r per load chunk
constexpr int kWbvPad = 64;   // zero complex past a wave's slot in LDS (row reads past K)
__device__ __forceinline__ double half_swap_sum(double v) {
  // v(lanes l mod 32) + v(lanes 32 + l mod 32) in every lane, the same order in both halves
  const auto lo = __builtin_amdgcn_permlane32_swap(__double2loint(v), __double2loint(v), false, false);
  const auto hi = __builtin_amdgcn_permlane32_swap(__double2hiint(v), __double2hiint(v), false, false);
  return __hiloint2double(hi[0], lo[0]) + __hiloint2double(hi[1], lo[1]);
}
template <typename T, int KR, int H>
__global__ __launch_bounds__(64 * kWbWG) __attribute__((amdgpu_waves_per_eu(KR <= 8 ? 4 : 2))) void k_dsolve_wbv(const cpx<T>* __restrict__ L,
                                                           const cpx<T>* __restrict__ h,
                                                           const cpx<T>* __restrict__ Ch,
                                                           cpx<T>* __restrict__ Dh, int F, int K,
                                                           T rho, int fgroups, int ntot, int NV,
                                                           int ni, int Kp) {
  static_assert(H == 1 || H == 2, "row segments");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int g = xcd_group(ntot);
  const int blk = g / fgroups;
  const int f = (g - blk * fgroups) * kWbWG + wave;
  if (g < 0 || f >= F) return;   // wave-uniform; the waves never meet at a barrier
  const int sz = ni * K + ni * ni;   // + kWbvPad zeros: row reads past K stay finite
  cpx<T>* sA = reinterpret_cast<cpx<T>*>(smem) + wave * (sz + kWbvPad);
  const cpx<T>* slot = L + ((int64_t)blk * F + f) * Kp;
  for (int i = lane; i < sz + kWbvPad; i += 64) sA[i] = i < sz ? slot[i] : cpx<T>{(T)0, (T)0};
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  const cpx<T> zero = {(T)0, (T)0};
  constexpr int VL = 64 / H;   // view lanes per row segment
  const int v = lane & (VL - 1), hh = H == 1 ? 0 : lane / VL;
  const int KH = (K + H - 1) / H;
  const int k0 = hh * KH;   // the lane's first row
  // branch-free body: rows k >= K and views >= NV load a clamped valid address and are
  // zeroed (r) or not stored; rows p >= ni of A contribute through t[p] = 0
  const int lv = min(v, NV - 1);
  // wave-uniform 64-bit bases + 32-bit lane offsets (global_load saddr form: no 64-bit
  // per-lane address per row; the host keeps a block's K NV F spectra under 4 GB)
  const int64_t cs = (int64_t)NV * F;   // k stride of Ch / Dh ([blk][k][uv][F])
  const cpx<T>* hf = h + ((int64_t)blk * F + f) * NV * K;   // [blk][f][uv][k]
  const cpx<T>* Cb = Ch + (int64_t)blk * K * cs + f;
  auto at = [](const cpx<T>* base, uint32_t boff) -> const cpx<T>& {
    return *reinterpret_cast<const cpx<T>*>(reinterpret_cast<const char*>(base) + boff);
  };
  // row i of the lane's segment is k = min(k0 + i, K - 1) (rows past K are clamped and
  // zeroed); the wave-uniform base takes row u = min(i, K - 1) and the lane offset the
  // difference k - u >= 0 (min is monotone and k0 >= 0), so the 32-bit offset never wraps
  auto urow = [&](int i) { return min(i, K - 1); };
  auto offh = [&](int i) {
    return (uint32_t)(lv * K + min(k0 + i, K - 1) - urow(i)) * (uint32_t)sizeof(cpx<T>);
  };
  auto offc = [&](int i) {
    return (uint32_t)(lv * F + (min(k0 + i, K - 1) - urow(i)) * cs) * (uint32_t)sizeof(cpx<T>);
  };
  // r = h + rho c in chunks of kWbvCH rows (sched_barrier: the compiler would otherwise
  // hoist every load of r to the top, 8 KR registers in flight)
  constexpr int NCH = (KR + kWbvCH - 1) / kWbvCH;
  cpx<T> r[NCH * kWbvCH];
  cpx<T> t[kWbMaxNi];
#pragma unroll
  for (int p = 0; p < kWbMaxNi; ++p) t[p] = zero;
  // row p of A in LDS (clamped to ni - 1; its t is discarded); columns k >= K read the
  // next row or the zero pad, times r[k] = 0
  int ar[kWbMaxNi];
#pragma unroll
  for (int p = 0; p < kWbMaxNi; ++p) ar[p] = min(p, ni - 1) * K + k0;
  // chunk ch + 1's loads are issued before chunk ch's products (double buffer)
  cpx<T> hb[kWbvCH], cb[kWbvCH];
  auto load = [&](int ch) {
#pragma unroll
    for (int i = 0; i < kWbvCH; ++i) {
      const int ii = ch * kWbvCH + i;
      cb[i] = at(Cb + urow(ii) * cs, offc(ii));
      hb[i] = at(hf + urow(ii), offh(ii));
    }
  };
  load(0);
#pragma unroll
  for (int ch = 0; ch < NCH; ++ch) {
#pragma unroll
    for (int i = 0; i < kWbvCH; ++i) {
      const int ii = ch * kWbvCH + i;
      const bool ok = ii < KH && k0 + ii < K;
      r[ii] = {ok ? fma(rho, cb[i].x, hb[i].x) : (T)0, ok ? fma(rho, cb[i].y, hb[i].y) : (T)0};
      asm volatile("" : "+v"(r[ii].x), "+v"(r[ii].y));
    }
    if (ch + 1 < NCH) load(ch + 1);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int p = 0; p < kWbMaxNi; ++p) {
#pragma unroll
      for (int i = 0; i < kWbvCH; ++i) {
        const int ii = ch * kWbvCH + i;
        const cpx<T> a = sA[ar[p] + ii];
        t[p].x = fma(a.x, r[ii].x, fma(-a.y, r[ii].y, t[p].x));
        t[p].y = fma(a.x, r[ii].y, fma(a.y, r[ii].x, t[p].y));
      }
      // pin the chunk's products here (LLVM otherwise sinks them to the solve, keeping
      // every loaded operand live)
      asm volatile("" : "+v"(t[p].x), "+v"(t[p].y));
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  if constexpr (H == 2) {
#pragma unroll
    for (int p = 0; p < kWbMaxNi; ++p) t[p] = {half_swap_sum(t[p].x), half_swap_sum(t[p].y)};
  }
  // M s = t: forward L_M y = t, backward L_M^H s = y (ni wave-uniform)
  const cpx<T>* lm = sA + ni * K;
  T dinv[kWbMaxNi];
#pragma unroll
  for (int j = 0; j < kWbMaxNi; ++j) dinv[j] = (T)1 / lm[min(j, ni - 1) * (ni + 1)].x;
#pragma unroll
  for (int j = 0; j < kWbMaxNi; ++j) {
    if (j < ni) {
      t[j] = cscale(t[j], dinv[j]);
#pragma unroll
      for (int q = j + 1; q < kWbMaxNi; ++q)
        if (q < ni) t[q] = cmsub(t[q], lm[q * ni + j], t[j]);
    }
  }
#pragma unroll
  for (int j = kWbMaxNi - 1; j >= 0; --j) {
    if (j < ni) {
      t[j] = cscale(t[j], dinv[j]);
#pragma unroll
      for (int q = 0; q < j; ++q) t[q] = cmsubc(t[q], lm[j * ni + q], t[j]);   // conj(L_M[j][q])
    }
  }
#pragma unroll
  for (int p = 0; p < kWbMaxNi; ++p)
    if (p >= ni) t[p] = zero;
  // x = (r - A^H s) / rho; A re-read from LDS through an opaque base (kept from the t loop,
  // 8 KR complex would not fit the registers)
  int xo = wave * (sz + kWbvPad);
  asm volatile("" : "+s"(xo));
  const cpx<T>* sA2 = reinterpret_cast<const cpx<T>*>(smem) + xo;
  const T irho = (T)1 / rho;
  cpx<T>* Db = Dh + (int64_t)blk * K * cs + f;
  if (v < NV) {
#pragma unroll
    for (int ii = 0; ii < KR; ++ii) {
      if (ii < KH && k0 + ii < K) {
        cpx<T> x = r[ii];
#pragma unroll
        for (int p = 0; p < kWbMaxNi; ++p) {   // x -= conj(A[p][k]) s_p
          const cpx<T> a = sA2[ar[p] + ii];
          x.x = fma(-a.x, t[p].x, fma(-a.y, t[p].y, x.x));
          x.y = fma(-a.x, t[p].y, fma(a.y, t[p].x, x.y));
        }
        __builtin_amdgcn_sched_barrier(0);
        *reinterpret_cast<cpx<T>*>(reinterpret_cast<char*>(Db + urow(ii) * cs) + offc(ii)) = cscale(x, irho);
      }
    }
  }
}

// k_dsolve_wbv with the views' right-hand sides r = h + rho C staged through LDS (NV <= 32, two row
// segments; C5: 0.809 -> 0.754 ms per launch, 19.8 -> 19.3 ms per outer iteration,
// profiles/r05/c5_wbs_ab.txt): Ch and Dh are [blk][k][uv][F], so a lane's own (view, k) element is one
// 16-B piece of a line F apart from its neighbour view's -- every load and store
// instruction of k_dsolve_wbv touched ~50 lines (C5: the texture-address unit 76% busy,
// 3.3 GB of L2 read requests for 1 GB of data).  Here the workgroup's 8 waves (8
// consecutive f) move a chunk of kWbsCH rows per segment cooperatively: consecutive
// threads take consecutive f of one (k, uv) row, 128 contiguous bytes, into an LDS tile
// [row][f][uv] (uv padded to 33: each wave then reads its f's views conflict-free), and the
// solutions leave the same way.  The next chunk's loads are in flight (registers) under the
// current chunk's products.  Waves past F run along (clamped operands, nothing stored) so
// every wave meets the barriers.
constexpr int kWbsCH = 4;   // rows per segment and chunk (2: 20.07, 8: 19.91, 4: 19.33 ms per C5 iteration)
constexpr int kWbsLD = 33;
// waves (consecutive f) per workgroup: 4, so two workgroups share a CU (two waves per SIMD at
// these registers either way) and one's chunk barriers overlap the other's work (C5: 8 per
// workgroup 17.1, 4 per workgroup 16.5 ms per outer iteration, profiles/r05/c5_wbs_wg_ab.txt)
constexpr int kWbsWG = 4;
__host__ __device__ constexpr size_t wbs_stage_elems() { return (size_t)2 * kWbsCH * kWbsWG * kWbsLD; }
template <typename T, int KR>
__global__ __launch_bounds__(64 * kWbsWG) __attribute__((amdgpu_waves_per_eu(2))) void k_dsolve_wbs(
    const cpx<T>* __restrict__ L, const cpx<T>* __restrict__ h, const cpx<T>* __restrict__ Ch,
    cpx<T>* __restrict__ Dh, int F, int K, T rho, int fgroups, int ntot, int NV, int ni, int Kp) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int g = xcd_group(ntot);
  if (g < 0) return;   // the whole workgroup
  const int blk = g / fgroups;
  const int fb = (g - blk * fgroups) * kWbsWG;
  const int f = min(fb + wave, F - 1);   // waves past F: clamped, results not stored
  const int sz = ni * K + ni * ni;
  cpx<T>* sA = reinterpret_cast<cpx<T>*>(smem) + wave * (sz + kWbvPad);
  cpx<T>* SB = reinterpret_cast<cpx<T>*>(smem) + kWbsWG * (sz + kWbvPad);
  const cpx<T>* slot = L + ((int64_t)blk * F + f) * Kp;
  for (int i = lane; i < sz + kWbvPad; i += 64) sA[i] = i < sz ? slot[i] : cpx<T>{(T)0, (T)0};
  const cpx<T> zero = {(T)0, (T)0};
  const int v = lane & 31, hh = lane >> 5;
  const int KH = (K + 1) / 2, k0 = hh * KH;
  const int64_t cs = (int64_t)NV * F;   // k stride of Ch / Dh
  const cpx<T>* Hblk = h + (int64_t)blk * K * cs;   // [blk][k][uv][F] (k_gram_wb<HT>)
  const cpx<T>* Cblk = Ch + (int64_t)blk * K * cs;
  cpx<T>* Dblk = Dh + (int64_t)blk * K * cs;
  constexpr int NCH = (KR + kWbsCH - 1) / kWbsCH;
  constexpr int EPT = (int)(2 * kWbsCH * 32 * kWbsWG / (64 * kWbsWG));   // staged elements per thread
  constexpr int FB = kWbsWG == 8 ? 3 : kWbsWG == 4 ? 2 : 1;   // log2(kWbsWG)
  // element e of a chunk: f offset fl = e mod kWbsWG, view uv = (e / kWbsWG) mod 32, tile row kk
  // (segment kk / kWbsCH, row c kWbsCH + kk % kWbsCH of it)
  auto rowk = [&](int c, int kk) {
    const int i = c * kWbsCH + (kk % kWbsCH);
    return i < KH ? (kk / kWbsCH) * KH + i : K;   // K: past the segment
  };
  auto sbi = [](int kk, int fl, int uv) { return (kk * kWbsWG + fl) * kWbsLD + uv; };
  cpx<T> pre[EPT];
  auto gload = [&](int c) {
#pragma unroll
    for (int j = 0; j < EPT; ++j) {
      const int e = tid + j * 64 * kWbsWG;
      const int fl = e & (kWbsWG - 1), uv = (e >> FB) & 31, kk = e >> (FB + 5);
      const int k = rowk(c, kk), ff = fb + fl;
      const bool ok = k < K && uv < NV && ff < F;
      const int64_t o = (int64_t)k * cs + (int64_t)uv * F + ff;
      const cpx<T> cv = ldc_if(ok, Cblk + o), hv = ldc_if(ok, Hblk + o);
      pre[j] = {fma(rho, cv.x, hv.x), fma(rho, cv.y, hv.y)};   // r = h + rho c
    }
  };
  auto sput = [&]() {
#pragma unroll
    for (int j = 0; j < EPT; ++j) {
      const int e = tid + j * 64 * kWbsWG;
      SB[sbi(e >> (FB + 5), e & (kWbsWG - 1), (e >> FB) & 31)] = pre[j];
    }
  };
  cpx<T> r[KR];   // rows past KR >= KH are zero: skipped at compile time
  cpx<T> t[kWbMaxNi];
#pragma unroll
  for (int p = 0; p < kWbMaxNi; ++p) t[p] = zero;
  int ar[kWbMaxNi];
#pragma unroll
  for (int p = 0; p < kWbMaxNi; ++p) ar[p] = min(p, ni - 1) * K + k0;
  gload(0);
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    __syncthreads();   // the previous chunk's tile reads are done (and sA is written)
    sput();
    __syncthreads();
    if (c + 1 < NCH) gload(c + 1);
#pragma unroll
    for (int i = 0; i < kWbsCH; ++i) {
      const int ii = c * kWbsCH + i;
      if (ii >= KR) break;
      const bool ok = ii < KH && k0 + ii < K;
      const cpx<T> rv = SB[sbi(hh * kWbsCH + i, wave, v)];
      r[ii] = {ok ? rv.x : (T)0, ok ? rv.y : (T)0};
      asm volatile("" : "+v"(r[ii].x), "+v"(r[ii].y));
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int p = 0; p < kWbMaxNi; ++p) {
#pragma unroll
      for (int i = 0; i < kWbsCH; ++i) {
        const int ii = c * kWbsCH + i;
        if (ii >= KR) break;
        const cpx<T> a = sA[ar[p] + ii];
        t[p].x = fma(a.x, r[ii].x, fma(-a.y, r[ii].y, t[p].x));
        t[p].y = fma(a.x, r[ii].y, fma(a.y, r[ii].x, t[p].y));
      }
      asm volatile("" : "+v"(t[p].x), "+v"(t[p].y));
      __builtin_amdgcn_sched_barrier(0);
    }
  }
#pragma unroll
  for (int p = 0; p < kWbMaxNi; ++p) t[p] = {half_swap_sum(t[p].x), half_swap_sum(t[p].y)};
  // M s = t (as k_dsolve_wbv)
  const cpx<T>* lm = sA + ni * K;
  T dinv[kWbMaxNi];
#pragma unroll
  for (int j = 0; j < kWbMaxNi; ++j) dinv[j] = (T)1 / lm[min(j, ni - 1) * (ni + 1)].x;
#pragma unroll
  for (int j = 0; j < kWbMaxNi; ++j) {
    if (j < ni) {
      t[j] = cscale(t[j], dinv[j]);
#pragma unroll
      for (int q = j + 1; q < kWbMaxNi; ++q)
        if (q < ni) t[q] = cmsub(t[q], lm[q * ni + j], t[j]);
    }
  }
#pragma unroll
  for (int j = kWbMaxNi - 1; j >= 0; --j) {
    if (j < ni) {
      t[j] = cscale(t[j], dinv[j]);
#pragma unroll
      for (int q = 0; q < j; ++q) t[q] = cmsubc(t[q], lm[j * ni + q], t[j]);
    }
  }
#pragma unroll
  for (int p = 0; p < kWbMaxNi; ++p)
    if (p >= ni) t[p] = zero;
  // x = (r - A^H s) / rho, staged out chunk by chunk
  int xo = wave * (sz + kWbvPad);
  asm volatile("" : "+s"(xo));
  const cpx<T>* sA2 = reinterpret_cast<const cpx<T>*>(smem) + xo;
  const T irho = (T)1 / rho;
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    __syncthreads();   // the tile is free
#pragma unroll
    for (int i = 0; i < kWbsCH; ++i) {
      const int ii = c * kWbsCH + i;
      if (ii >= KR) break;
      cpx<T> x = r[ii];
#pragma unroll
      for (int p = 0; p < kWbMaxNi; ++p) {   // x -= conj(A[p][k]) s_p
        const cpx<T> a = sA2[ar[p] + ii];
        x.x = fma(-a.x, t[p].x, fma(-a.y, t[p].y, x.x));
        x.y = fma(-a.x, t[p].y, fma(a.y, t[p].x, x.y));
      }
      SB[sbi(hh * kWbsCH + i, wave, v)] = cscale(x, irho);
      __builtin_amdgcn_sched_barrier(0);
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < EPT; ++j) {
      const int e = tid + j * 64 * kWbsWG;
      const int fl = e & (kWbsWG - 1), uv = (e >> FB) & 31, kk = e >> (FB + 5);
      const int k = rowk(c, kk), ff = fb + fl;
      if (k < K && uv < NV && ff < F) Dblk[(int64_t)k * cs + (int64_t)uv * F + ff] = SB[sbi(kk, fl, uv)];
    }
  }
}

// the many-view d-solve runs staged (k_dsolve_wbs) and then reads h in Ch's layout.
// `allow` is the session's choice (CCSC_WB_STAGE, read once at session creation), passed to
// both launchers so the Gram's h layout and the solve's reads cannot disagree
static bool wb_staged(int K, int NV, int F, bool allow) {
  return allow && NV > 1 && NV <= 32 && K <= 64 &&
         (int64_t)K * NV * F * (int64_t)sizeof(cpx<double>) < ((int64_t)1 << 32);
}

template <typename T>
hipError_t launch_gram_wb(const cpx<T>* Zh, const cpx<T>* Bh, cpx<T>* L, cpx<T>* h, int F, int K,
                          int ni, T rho, int NV, bool staged, hipStream_t st) {
  if (!woodbury_ok(K, ni)) return hipErrorInvalidValue;
  const int Kp = K * (K + 1) / 2;
  const dim3 grid((unsigned)((((F + kWbWG - 1) / kWbWG + 7) / 8) * 8));   // whole XCD rounds
  if (wb_staged(K, NV, F, staged))
    hipLaunchKernelGGL((k_gram_wb<T, 1, true>), grid, dim3(64 * kWbWG), 0, st, Zh, Bh, L, h, F, K,
                       ni, rho, NV, Kp);
  else if (K <= 64)
    hipLaunchKernelGGL((k_gram_wb<T, 1>), grid, dim3(64 * kWbWG), 0, st, Zh, Bh, L, h, F, K, ni,
                       rho, NV, Kp);
  else
    hipLaunchKernelGGL((k_gram_wb<T, 2>), grid, dim3(64 * kWbWG), 0, st, Zh, Bh, L, h, F, K, ni,
                       rho, NV, Kp);
  return hipGetLastError();
}

template <typename T, int RPL, int NVB>
static void dsolve_wb_go(dim3 grid, hipStream_t st, const cpx<T>* L, const cpx<T>* h,
                         const cpx<T>* Ch, cpx<T>* Dh, int F, int K, T rho, int fgroups, int NV,
                         int ni) {
  const int ntot = (int)grid.y * fgroups;   // grid.y carries the block count (see launcher)
  hipLaunchKernelGGL((k_dsolve_wb<T, RPL, NVB>), dim3(grid.x), dim3(64 * kWbWG), 0, st, L, h, Ch,
                     Dh, F, K, rho, fgroups, ntot, NV, ni, K * (K + 1) / 2);
}

template <typename T>
hipError_t launch_dsolve_wb(const cpx<T>* L, const cpx<T>* h, const cpx<T>* Ch, cpx<T>* Dh,
                            int nblocks, int F, int K, int ni, T rho, int NV, bool staged,
                            hipStream_t st) {
  if (nblocks <= 0) return hipSuccess;
  if (!woodbury_ok(K, ni)) return hipErrorInvalidValue;
  const int fgroups = (F + kWbWG - 1) / kWbWG;
  const int n = nblocks * fgroups;
  const dim3 grid((unsigned)(((n + 7) / 8) * 8), (unsigned)nblocks);   // whole XCD rounds
  if (NV > 1 && NV <= kWbvMaxNV && K <= 64 &&
      (int64_t)K * NV * F * (int64_t)sizeof(cpx<T>) < ((int64_t)1 << 32)) {   // lanes over the views
    const size_t smem = (size_t)kWbWG * (ni * K + ni * ni + kWbvPad) * sizeof(cpx<T>);
    auto go = [&](auto kern) {
      hipLaunchKernelGGL(kern, dim3(grid.x), dim3(64 * kWbWG), smem, st, L, h, Ch, Dh, F, K, rho,
                         fgroups, n, NV, ni, K * (K + 1) / 2);
    };
    if (wb_staged(K, NV, F, staged)) {   // staged views (k_dsolve_wbs; h in Ch's layout, k_gram_wb)
      const int kh = (K + 1) / 2;
      const size_t smem2 = (size_t)kWbsWG * (ni * K + ni * ni + kWbvPad) * sizeof(cpx<T>) +
                           wbs_stage_elems() * sizeof(cpx<T>);
      const int fg2 = (F + kWbsWG - 1) / kWbsWG, n2 = nblocks * fg2;
      auto go2 = [&](auto kern) {
        hipLaunchKernelGGL(kern, dim3((unsigned)(((n2 + 7) / 8) * 8)), dim3(64 * kWbsWG), smem2, st,
                           L, h, Ch, Dh, F, K, rho, fg2, n2, NV, ni, K * (K + 1) / 2);
      };
      if (kh <= 8) go2(k_dsolve_wbs<T, 8>);
      else if (kh <= 16) go2(k_dsolve_wbs<T, 16>);
      else if (kh <= 24) go2(k_dsolve_wbs<T, 24>);
      else if (kh <= 28) go2(k_dsolve_wbs<T, 28>);
      else go2(k_dsolve_wbs<T, 32>);
    } else if (NV <= 32) {   // two row segments of KH = ceil(K / 2) <= 32
      const int kh = (K + 1) / 2;
      if (kh <= 8) go(k_dsolve_wbv<T, 8, 2>);
      else if (kh <= 16) go(k_dsolve_wbv<T, 16, 2>);
      else if (kh <= 24) go(k_dsolve_wbv<T, 24, 2>);
      else if (kh <= 28) go(k_dsolve_wbv<T, 28, 2>);
      else go(k_dsolve_wbv<T, 32, 2>);
    } else {
      if (K <= 16) go(k_dsolve_wbv<T, 16, 1>);
      else if (K <= 32) go(k_dsolve_wbv<T, 32, 1>);
      else if (K <= 48) go(k_dsolve_wbv<T, 48, 1>);
      else if (K <= 56) go(k_dsolve_wbv<T, 56, 1>);
      else go(k_dsolve_wbv<T, 64, 1>);
    }
    return hipGetLastError();
  }
  if (K <= 64) {
    if (NV == 1) dsolve_wb_go<T, 1, 1>(grid, st, L, h, Ch, Dh, F, K, rho, fgroups, NV, ni);
    else dsolve_wb_go<T, 1, 4>(grid, st, L, h, Ch, Dh, F, K, rho, fgroups, NV, ni);
  } else {
    if (NV == 1) dsolve_wb_go<T, 2, 1>(grid, st, L, h, Ch, Dh, F, K, rho, fgroups, NV, ni);
    else dsolve_wb_go<T, 2, 4>(grid, st, L, h, Ch, Dh, F, K, rho, fgroups, NV, ni);
  }
  return hipGetLastError();
}

template hipError_t launch_gram_wb<double>(const cpx<double>*, const cpx<double>*, cpx<double>*,
                                           cpx<double>*, int, int, int, double, int, bool,
                                           hipStream_t);
template hipError_t launch_dsolve_wb<double>(const cpx<double>*, const cpx<double>*,
                                             const cpx<double>*, cpx<double>*, int, int, int, int,
                                             double, int, bool, hipStream_t);
template hipError_t launch_gram_chol<double>(const cpx<double>*, const cpx<double>*,
                                             cpx<double>*, cpx<double>*, int, int, int, double,
                                             int, hipStream_t);
template hipError_t launch_dsolve<double>(const cpx<double>*, const cpx<double>*,
                                          const cpx<double>*, cpx<double>*, int, int, int,
                                          double, int, hipStream_t);

}  // namespace ccsc
