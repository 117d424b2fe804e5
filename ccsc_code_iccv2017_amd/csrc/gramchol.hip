// D-step precompute on the matrix cores (gfx950): per frequency f of a block,
// G_f = A_f^H A_f + rho I (A_f = ni x K code spectra, K <= 112), h_f = A_f^H b_f,
// and the Cholesky factor L_f of G_f, packed lower column-major -- the same
// outputs as k_gram_chol (dstep.hip; reference precompute_H_hat_D, dP:221-237:
// Sinv_f = (A^H A + rho I)^-1 through pinv, here factored instead of inverted).
//
// G is held as 16 x 16 tiles (T = ceil(K / 16) <= 7 per dimension, the T(T+1)/2
// lower tiles dealt round-robin to the four waves) in v_mfma_f64_16x16x4_f64
// accumulators for the whole kernel:
//   Gram     per 4 patches and tile (I, J): Re G = Ar_I^T Ar_J + Ai_I^T Ai_J,
//            Im G = Ar_I^T Ai_J - Ai_I^T Ar_J from three real products (Gauss, 3 MFMAs,
//            gram_kstep); the code spectra are
//            staged through LDS in chunks of 16 patches, double-buffered, the next
//            chunk's (strided) global loads in flight under the current chunk's MFMAs;
//   Cholesky blocked right-looking over the T tile columns j:
//            POTRF of tile (j, j) by wave 0 (rows on lanes, pivots by v_readlane),
//            TRSM of the tiles below by every wave (one row per lane, L_jj read as
//            LDS broadcasts), trailing update A_ik -= L_ij L_kj^H of every tile
//            k > j on the matrix cores by its owner (16 MFMAs per tile).
// L goes from the POTRF/TRSM registers straight to HBM (for a fixed column,
// consecutive lanes hold consecutive rows: coalesced).  LDS: the staging chunks
// (58 KB) or two column panels (61 KB), so two workgroups share a CU and one's
// VALU phases (POTRF, TRSM) run beside the other's MFMA phases.
#include "kernels.hpp"

#include <utility>

namespace ccsc {

typedef double d4 __attribute__((ext_vector_type(4)));

constexpr int kGcNT = 256;                  // 4 waves
// TM = tiles per dimension, K <= 16 TM: TM = 7 (K <= 112, the headline K = 100) runs two
// workgroups per CU; TM = 8, 10, 12 (K <= 192) hold up to 20 accumulator tiles per wave
// (320 of the 512 registers) at one workgroup per CU
template <int TM>
struct GcShape {
  static constexpr int Tiles = TM * (TM + 1) / 2;
  static constexpr int TW = (Tiles + 3) / 4;   // tiles per wave
  static constexpr int KP = 16 * TM;           // padded filter count of a staged row
  static constexpr int LD = KP + 1;            // staged row stride (complex)
  static constexpr int WGS = TM <= 7 ? 2 : 1;  // workgroups per CU
  // the third accumulator set of the Gauss Gram fits the registers up to TM = 8
  static constexpr bool Gauss = TM <= 8;
};
constexpr int kGcMaxTM = 12;
constexpr int kGcPC = 16;                   // patches per staged chunk
constexpr int kGcTS = 17;                   // column stride (complex) of an LDS tile
constexpr int kGcTSZ = 16 * kGcTS;          // complex per LDS tile
constexpr int kGcHPT = 8;                   // right-hand-side entries of h per thread

__device__ __forceinline__ d4 mfma(double a, double b, d4 c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ double rdl(double v, int l) {
  return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), l),
                          __builtin_amdgcn_readlane(__double2loint(v), l));
}

__device__ __forceinline__ int gc_pk(int j, int K) { return j * K - (j * (j - 1)) / 2; }

// tile t of the T(T+1)/2 lower tiles -> (I, J); wave w owns tiles w, w + 4, ...
__device__ __forceinline__ void gc_tile(int t, int& I, int& J) {
  I = (int)((sqrt(8.0 * t + 1.0) - 1.0) * 0.5);
  while ((I + 1) * (I + 2) / 2 <= t) ++I;
  while (I * (I + 1) / 2 > t) --I;
  J = t - I * (I + 1) / 2;
}

// the same map at compile time: the per-wave instantiations of the kernel body
// (gram_chol_body<TM, HP, W>) see tile coordinates and LDS offsets as constants -- no
// per-tile index arithmetic or branches in the MFMA loops (1.82 -> 1.70 ms per C2 block,
// profiles/r05/gram_ct_ab.txt)
constexpr int ct_I(int t) {
  int I = 0;
  while ((I + 1) * (I + 2) / 2 <= t) ++I;
  return I;
}
constexpr int ct_J(int t) { return t - ct_I(t) * (ct_I(t) + 1) / 2; }

// Gram MFMAs of tile S of wave W for one k-step (see gram_kstep)
template <int TM, int W, int S>
__device__ __forceinline__ void gram_tile_w(const cpx<double>* row, int Tn,
                                            d4 (&t1)[GcShape<TM>::TW], d4 (&t2)[GcShape<TM>::TW],
                                            d4 (&t3)[GcShape<TM>::Gauss ? GcShape<TM>::TW : 1]) {
  constexpr int t = W + 4 * S;
  if constexpr (t < GcShape<TM>::Tiles) {
    constexpr int I = ct_I(t), J = ct_J(t);
    if (I < Tn) {
      const cpx<double> a = row[16 * I + (threadIdx.x & 15)];
      const cpx<double> b = I == J ? a : row[16 * J + (threadIdx.x & 15)];
      if constexpr (GcShape<TM>::Gauss) {
        t1[S] = mfma(a.x, b.x, t1[S]);
        t2[S] = mfma(a.y, b.y, t2[S]);
        t3[S] = mfma(a.x - a.y, b.x + b.y, t3[S]);
      } else {
        t1[S] = mfma(a.x, b.x, t1[S]);
        t1[S] = mfma(a.y, b.y, t1[S]);
        t2[S] = mfma(a.x, b.y, t2[S]);
        t2[S] = mfma(-a.y, b.x, t2[S]);
      }
    }
  }
  // one tile's operands at a time (hoisting the next tiles' LDS reads spills)
  __builtin_amdgcn_sched_barrier(0);
}
template <int TM, int W, int... S>
__device__ __forceinline__ void gram_kstep_seq(const cpx<double>* row, int Tn,
                                               d4 (&t1)[GcShape<TM>::TW], d4 (&t2)[GcShape<TM>::TW],
                                               d4 (&t3)[GcShape<TM>::Gauss ? GcShape<TM>::TW : 1],
                                               std::integer_sequence<int, S...>) {
  (gram_tile_w<TM, W, S>(row, Tn, t1, t2, t3), ...);
}
// the k-steps of one staged chunk (kvalid of kGcPC / 4), wave W
template <int TM, int W>
__device__ __forceinline__ void gram_chunk_w(const cpx<double>* row0, int kvalid, int Tn,
                                             d4 (&t1)[GcShape<TM>::TW], d4 (&t2)[GcShape<TM>::TW],
                                             d4 (&t3)[GcShape<TM>::Gauss ? GcShape<TM>::TW : 1]) {
#pragma unroll
  for (int kk = 0; kk < kGcPC / 4; ++kk)
    if (kk < kvalid)
      gram_kstep_seq<TM, W>(row0 + 4 * kk * GcShape<TM>::LD, Tn, t1, t2, t3,
                            std::make_integer_sequence<int, GcShape<TM>::TW>{});
}

// Gram MFMAs of wave w for one k-step (4 patches: lane l takes patch l >> 4 of the
// step and filter 16 T + (l & 15) of tile row/column T).  Tile coordinates are
// wave-uniform runtime values: operands are loaded per tile from LDS, so no
// register array is indexed at run time.  Three real products per complex tile
// (Gauss): t1 = sum ax bx, t2 = sum ay by, t3 = sum (ax - ay)(bx + by), so that
// Re G = t1 + t2 and Im G = sum (ax by - ay bx) = t3 - t1 + t2 (gram_gauss_fold) --
// 3 MFMAs per tile and k-step instead of 4 (the Gram is matrix-core bound).
template <int TM>
__device__ __forceinline__ void gram_kstep(const cpx<double>* row, int w, int Tn,
                                           d4 (&t1)[GcShape<TM>::TW], d4 (&t2)[GcShape<TM>::TW],
                                           d4 (&t3)[GcShape<TM>::Gauss ? GcShape<TM>::TW : 1]) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int s = 0; s < GcShape<TM>::TW; ++s) {
    const int t = w + 4 * s;
    int I, J;
    gc_tile(t, I, J);
    if (t < GcShape<TM>::Tiles && I < Tn) {
      const cpx<double> a = row[16 * I + (lane & 15)];
      const cpx<double> b = row[16 * J + (lane & 15)];
      if constexpr (GcShape<TM>::Gauss) {
        t1[s] = mfma(a.x, b.x, t1[s]);
        t2[s] = mfma(a.y, b.y, t2[s]);
        t3[s] = mfma(a.x - a.y, b.x + b.y, t3[s]);
      } else {   // Re, Im directly (4 MFMAs; t1 = Re, t2 = Im)
        t1[s] = mfma(a.x, b.x, t1[s]);
        t1[s] = mfma(a.y, b.y, t1[s]);
        t2[s] = mfma(a.x, b.y, t2[s]);
        t2[s] = mfma(-a.y, b.x, t2[s]);
      }
    }
  }
}
template <int TM>
__device__ __forceinline__ void gram_gauss_fold(d4 (&t1)[GcShape<TM>::TW], d4 (&t2)[GcShape<TM>::TW],
                                                const d4 (&t3)[GcShape<TM>::Gauss ? GcShape<TM>::TW : 1]) {
  if constexpr (!GcShape<TM>::Gauss) return;
#pragma unroll
  for (int s = 0; s < GcShape<TM>::TW; ++s) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const double re = t1[s][r] + t2[s][r];
      const double im = (t3[s][r] - t1[s][r]) + t2[s][r];
      t1[s][r] = re;
      t2[s][r] = im;
    }
  }
}

// store an accumulator tile (C/D layout: lane l holds row (l >> 4) + 4 r, column l & 15)
// into an LDS tile (element (row, col) at col * kGcTS + row)
__device__ __forceinline__ void tile_to_lds(cpx<double>* dst, const d4& re, const d4& im) {
  const int lane = threadIdx.x & 63;
  const int col = lane & 15;
#pragma unroll
  for (int r = 0; r < 4; ++r) dst[col * kGcTS + (lane >> 4) + 4 * r] = {re[r], im[r]};
}

// trailing update of wave w's tiles (i, k), k > j: A_ik -= L_ij L_kj^H, the panel
// tiles L_.j in P (P[i * kGcTSZ + col * kGcTS + row]); then the tiles of column
// j + 1 to the next panel buffer Pn
template <int TM>
__device__ __forceinline__ void trail_step(const cpx<double>* P, cpx<double>* Pn, int j, int w,
                                           int Tn, d4 (&gr)[GcShape<TM>::TW],
                                           d4 (&gi)[GcShape<TM>::TW]) {
  const int lane = threadIdx.x & 63;
  const int row = lane & 15, c4 = lane >> 4;
#pragma unroll
  for (int s = 0; s < GcShape<TM>::TW; ++s) {
    const int t = w + 4 * s;
    int I, J;
    gc_tile(t, I, J);
    if (t < GcShape<TM>::Tiles && I < Tn && J > j) {
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        const int col = 4 * kk + c4;
        const cpx<double> a = P[I * kGcTSZ + col * kGcTS + row];   // L_ij (row, col)
        const cpx<double> b = P[J * kGcTSZ + col * kGcTS + row];   // L_kj (row, col)
        gr[s] = mfma(-a.x, b.x, gr[s]);
        gr[s] = mfma(-a.y, b.y, gr[s]);
        gi[s] = mfma(-a.y, b.x, gi[s]);
        gi[s] = mfma(a.x, b.y, gi[s]);
      }
      if (J == j + 1) tile_to_lds(Pn + I * kGcTSZ, gr[s], gi[s]);
    }
  }
}

// trail_step with wave W's tile coordinates as constants
template <int TM, int W>
__device__ __forceinline__ void trail_step_w(const cpx<double>* P, cpx<double>* Pn, int j, int Tn,
                                             d4 (&gr)[GcShape<TM>::TW], d4 (&gi)[GcShape<TM>::TW]) {
  const int lane = threadIdx.x & 63;
  const int row = lane & 15, c4 = lane >> 4;
#pragma unroll
  for (int s = 0; s < GcShape<TM>::TW; ++s) {
    const int t = W + 4 * s;
    const int I = ct_I(t), J = ct_J(t);
    if (t < GcShape<TM>::Tiles && I < Tn && J > j) {
      if constexpr (TM <= 10) {
        // three real products per tile and column step (Gauss, as the Gram): 12 MFMAs
        // instead of 16 (1.694 -> 1.675 ms per C2 block; TM = 12 would spill the third set)
        d4 u1 = {0.0, 0.0, 0.0, 0.0}, u2 = u1, u3 = u1;
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
          const int col = 4 * kk + c4;
          const cpx<double> a = P[I * kGcTSZ + col * kGcTS + row];
          const cpx<double> b = P[J * kGcTSZ + col * kGcTS + row];
          u1 = mfma(a.x, b.x, u1);
          u2 = mfma(a.y, b.y, u2);
          u3 = mfma(a.x - a.y, b.x + b.y, u3);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          gr[s][r] -= u1[r] + u2[r];
          gi[s][r] += (u3[r] - u1[r]) + u2[r];
        }
      } else {
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
          const int col = 4 * kk + c4;
          const cpx<double> a = P[I * kGcTSZ + col * kGcTS + row];
          const cpx<double> b = P[J * kGcTSZ + col * kGcTS + row];
          gr[s] = mfma(-a.x, b.x, gr[s]);
          gr[s] = mfma(-a.y, b.y, gr[s]);
          gi[s] = mfma(-a.y, b.x, gi[s]);
          gi[s] = mfma(a.x, b.y, gi[s]);
        }
      }
      if (J == j + 1) tile_to_lds(Pn + I * kGcTSZ, gr[s], gi[s]);
    }
  }
}

template <int TM>
__device__ __forceinline__ void first_panel(cpx<double>* P, int w, int Tn,
                                            const d4 (&gr)[GcShape<TM>::TW],
                                            const d4 (&gi)[GcShape<TM>::TW]) {
#pragma unroll
  for (int s = 0; s < GcShape<TM>::TW; ++s) {
    const int t = w + 4 * s;
    int I, J;
    gc_tile(t, I, J);
    if (t < GcShape<TM>::Tiles && I < Tn && J == 0) tile_to_lds(P + I * kGcTSZ, gr[s], gi[s]);
  }
}

// rho on the diagonal (exactly real), identity on the padding rows K..16 Tn - 1
template <int TM>
__device__ __forceinline__ void fix_diag(int w, int K, int Tn, double rho,
                                         d4 (&gr)[GcShape<TM>::TW], d4 (&gi)[GcShape<TM>::TW]) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int s = 0; s < GcShape<TM>::TW; ++s) {
    const int t = w + 4 * s;
    int I, J;
    gc_tile(t, I, J);
    if (t < GcShape<TM>::Tiles && I < Tn && I == J) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int rr = (lane >> 4) + 4 * r, cc = lane & 15;
        if (rr == cc) {
          gr[s][r] = (16 * I + rr < K) ? gr[s][r] + rho : 1.0;
          gi[s][r] = 0.0;
        }
      }
    }
  }
}

// HP: right-hand-side entries of h per thread (1 when K NV <= kGcNT: the headline's one);
// WV: the wave index as a template constant (0..3), or -1 for the run-time index (the
// TM = 7, HP = 8 shape, whose per-wave instantiations spill)
template <int TM, int HP, int WV>
__device__ __forceinline__ void gram_chol_body(const cpx<double>* __restrict__ Zh,
                                               const cpx<double>* __restrict__ Bh,
                                               cpx<double>* __restrict__ L,
                                               cpx<double>* __restrict__ h, int F, int K, int ni,
                                               double rho, int NV, int f, char* smem) {
  using S = GcShape<TM>;
  constexpr int kGcTW = S::TW, kGcKP = S::KP, kGcLD = S::LD, kGcTM = TM;
  cpx<double>* sA = reinterpret_cast<cpx<double>*>(smem);      // [2][kGcPC][kGcLD]
  cpx<double>* sB = sA + 2 * kGcPC * kGcLD;                    // [2][kGcPC][NV]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = WV >= 0 ? WV : __builtin_amdgcn_readfirstlane(tid >> 6);
  int Tn = (K + 15) >> 4;
  const int KV = K * NV;

  d4 gr[kGcTW], gi[kGcTW], g3[S::Gauss ? kGcTW : 1];   // Gram: Gauss products t1, t2, t3
#pragma unroll
  for (int s = 0; s < kGcTW; ++s) gr[s] = gi[s] = (d4){0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int s = 0; s < (S::Gauss ? kGcTW : 1); ++s) g3[s] = (d4){0.0, 0.0, 0.0, 0.0};
  cpx<double> hacc[HP];
#pragma unroll
  for (int i = 0; i < HP; ++i) hacc[i] = {0.0, 0.0};

  // ---- Gram + h: chunks of kGcPC patches, double-buffered ----
  constexpr int kPer = (kGcPC * kGcKP + kGcNT - 1) / kGcNT;   // staged values per thread
  cpx<double> pre[kPer];
  cpx<double> preb = {0.0, 0.0};
  auto fetch = [&](int p0) {
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int idx = tid + i * kGcNT;
      const int pp = idx / kGcKP, k = idx - pp * kGcKP;
      pre[i] = (pp < kGcPC && k < K && p0 + pp < ni)
                   ? Zh[((int64_t)(p0 + pp) * K + k) * F + f]
                   : cpx<double>{0.0, 0.0};
    }
    if (tid < kGcPC * NV) {
      const int pp = tid / NV;
      preb = (p0 + pp < ni) ? Bh[(int64_t)(p0 * NV + tid) * F + f] : cpx<double>{0.0, 0.0};
    }
  };
  auto stage = [&](int buf) {
    cpx<double>* a = sA + buf * kGcPC * kGcLD;
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int idx = tid + i * kGcNT;
      const int pp = idx / kGcKP, k = idx - pp * kGcKP;
      if (pp < kGcPC) a[pp * kGcLD + k] = pre[i];
    }
    if (tid < kGcPC * NV) sB[buf * kGcPC * NV + tid] = preb;
  };
  const int nch = (ni + kGcPC - 1) / kGcPC;
  fetch(0);
  stage(0);
  __syncthreads();
  for (int c = 0; c < nch; ++c) {
    const int buf = c & 1;
    if (c + 1 < nch) fetch((c + 1) * kGcPC);
    const cpx<double>* a = sA + buf * kGcPC * kGcLD;
    // k-steps past the last patch (the zero padding of a partial last chunk: ni = 100 is
    // 6.25 chunks) are skipped -- adding their zero products changes nothing
    const int kvalid = (ni - c * kGcPC + 3) >> 2;
    if constexpr (WV >= 0) {
      gram_chunk_w<TM, (WV >= 0 ? WV : 0)>(a + (lane >> 4) * kGcLD, kvalid, Tn, gr, gi, g3);
    } else {
#pragma unroll
      for (int kk = 0; kk < kGcPC / 4; ++kk) {
        const cpx<double>* row = a + (4 * kk + (lane >> 4)) * kGcLD;
        if (kk < kvalid) gram_kstep<TM>(row, wave, Tn, gr, gi, g3);
      }
    }
    const cpx<double>* b = sB + buf * kGcPC * NV;
#pragma unroll
    for (int i = 0; i < HP; ++i) {
      const int q = tid + i * kGcNT;   // q = uv * K + k
      if (q < KV) {
        const int uv = q / K, k = q - uv * K;
        const int pv = min(kGcPC, ni - c * kGcPC);
#pragma unroll 4
        for (int pp = 0; pp < pv; ++pp)
          hacc[i] = cmacc(hacc[i], a[pp * kGcLD + k], b[pp * NV + uv]);
      }
    }
    if (c + 1 < nch) stage(buf ^ 1);
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < HP; ++i) {
    const int q = tid + i * kGcNT;
    if (q < KV) h[(int64_t)f * KV + q] = hacc[i];
  }
  gram_gauss_fold<TM>(gr, gi, g3);   // gr, gi <- Re G, Im G
  fix_diag<TM>(wave, K, Tn, rho, gr, gi);

  // ---- blocked Cholesky over the tile columns ----
  cpx<double>* Pbuf = reinterpret_cast<cpx<double>*>(smem);   // [2][kGcTM][kGcTSZ]
  cpx<double>* Lf = L + (int64_t)f * (K * (K + 1) / 2);
  first_panel<TM>(Pbuf, wave, Tn, gr, gi);
  for (int j = 0; j < Tn; ++j) {
    cpx<double>* P = Pbuf + (j & 1) * kGcTM * kGcTSZ;
    cpx<double>* Pn = Pbuf + ((j + 1) & 1) * kGcTM * kGcTSZ;
    __syncthreads();   // column j's tiles are in P
    // Panel j (POTRF of tile (j, j) + TRSM of the tiles below) in one sweep over its 16
    // columns, on as few waves as hold its rows: lanes 0..15 hold the rows of tile (j, j)
    // (redundantly on each such wave, so none waits for another), lanes 16..63 RW = 48 of
    // the panel's other rows -- waves 0 and 1 at K = 100 until j = 3, wave 0 alone after
    // (the other waves go to the barrier and leave the SIMDs to the CU's other workgroup;
    // every wave with 4 (TM - 1) rows: 1.89 ms per C2 block, this form 1.82).  Column c
    // of row r:
    //   s = a[r][c] - sum_{k < c} L[r][k] conj(L[c][k]);  L[c][c] = sqrt(s of row c),
    //   L[r][c] = s / L[c][c]  (the POTRF and TRSM formulas coincide).
    if (wave == 0 || wave * 48 < 16 * (Tn - 1 - j)) {
      const bool diag = lane < 16;
      constexpr int RW = 48;
      static_assert(16 + RW <= 64, "panel rows per wave");
      const int q = wave * RW + lane - 16;
      const int ti = diag ? j : j + 1 + (q >> 4);
      const int row = diag ? lane : (q & 15);
      const bool mine = diag || (lane < 16 + RW && ti < Tn);
      cpx<double> x[16];
#pragma unroll
      for (int c = 0; c < 16; ++c)
        x[c] = mine ? ldc_if(true, P + ti * kGcTSZ + c * kGcTS + row) : cpx<double>{1.0, 0.0};
      // right-looking in registers: once column c is final, every row r loses
      // L[r][c] conj(L[c2][c]) from its column c2 > c, L[c2][c] broadcast from lane c2 by
      // v_readlane -- no LDS round trip on the column-to-column chain; 1/sqrt of the
      // pivot by v_rsq_f64 and one Newton step (error ~1.5 e0^2; a second one measured
      // 1.4% of the kernel, profiles/r03j/gram_newton_ab.txt) instead of sqrt and a division
#pragma unroll
      for (int c = 0; c < 16; ++c) {
        const double a = rdl(x[c].x, c);
        double y = __builtin_amdgcn_rsq(a);
        const double hh = 0.5 * a;
        y = fma(y, fma(-hh * y, y, 0.5), y);
        x[c] = (lane == c) ? cpx<double>{a * y, 0.0} : cscale(x[c], y);
#pragma unroll
        for (int c2 = c + 1; c2 < 16; ++c2) {
          const double lx = rdl(x[c].x, c2), ly = rdl(x[c].y, c2);   // L[c2][c]
          // x[c2] -= x[c] conj(L[c2][c]) as four FMAs (the expression form compiled to
          // mul + fma + add per component)
          x[c2].x = fma(-x[c].x, lx, fma(-x[c].y, ly, x[c2].x));
          x[c2].y = fma(-x[c].y, lx, fma(x[c].x, ly, x[c2].y));
        }
      }
      const int gr_ = 16 * ti + row;
      if (mine && (!diag || wave == 0) && gr_ < K) {
#pragma unroll
        for (int c = 0; c < 16; ++c) {
          const int gc = 16 * j + c;
          if (!diag || row >= c) Lf[gc_pk(gc, K) + gr_ - gc] = x[c];
        }
      }
      if (mine && !diag) {
#pragma unroll
        for (int c = 0; c < 16; ++c) P[ti * kGcTSZ + c * kGcTS + row] = x[c];
      }
    }
    __syncthreads();   // the panel L_.j is in P
    if (j + 1 < Tn) {
      if constexpr (WV >= 0) trail_step_w<TM, (WV >= 0 ? WV : 0)>(P, Pn, j, Tn, gr, gi);
      else trail_step<TM>(P, Pn, j, wave, Tn, gr, gi);
    }
  }
}

template <int TM, int HP>
__global__ __launch_bounds__(kGcNT, GcShape<TM>::WGS) void k_gram_chol_mf(const cpx<double>* __restrict__ Zh,
                                                           const cpx<double>* __restrict__ Bh,
                                                           cpx<double>* __restrict__ L,
                                                           cpx<double>* __restrict__ h, int F,
                                                           int K, int ni, double rho, int NV) {
  const int per = gridDim.x >> 3;
  const int f = (blockIdx.x & 7) * per + (blockIdx.x >> 3);   // XCD-aware: neighbours share L2
  if (f >= F) return;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  if constexpr (TM == 7 && HP > 1) {
    gram_chol_body<TM, HP, -1>(Zh, Bh, L, h, F, K, ni, rho, NV, f, smem);
  } else {
    // every wave runs the same barriers in its own instantiation
    switch (__builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6)) {
      case 0: gram_chol_body<TM, HP, 0>(Zh, Bh, L, h, F, K, ni, rho, NV, f, smem); break;
      case 1: gram_chol_body<TM, HP, 1>(Zh, Bh, L, h, F, K, ni, rho, NV, f, smem); break;
      case 2: gram_chol_body<TM, HP, 2>(Zh, Bh, L, h, F, K, ni, rho, NV, f, smem); break;
      default: gram_chol_body<TM, HP, 3>(Zh, Bh, L, h, F, K, ni, rho, NV, f, smem); break;
    }
  }
}

static int gc_tm(int K) { const int t = (K + 15) / 16; return t <= 7 ? 7 : t <= 8 ? 8 : t <= 10 ? 10 : 12; }

bool gram_chol_mf_ok(int K, int NV) {
  return K <= 16 * kGcMaxTM && K * NV <= kGcHPT * kGcNT && NV <= 16;
}

size_t gram_chol_mf_smem(int NV, int K) {
  const int tm = gc_tm(K);
  const size_t stage = (size_t)2 * kGcPC * (16 * tm + 1) * 16 + (size_t)2 * kGcPC * NV * 16;
  const size_t chol = (size_t)2 * tm * kGcTSZ * 16;   // two column panels
  return stage > chol ? stage : chol;
}

template <int TM, int HP>
static void gram_chol_mf_go(const cpx<double>* Zh, const cpx<double>* Bh, cpx<double>* L,
                            cpx<double>* h, int F, int K, int ni, double rho, int NV,
                            hipStream_t st) {
  const int grid = ((F + 7) / 8) * 8;
  hipLaunchKernelGGL((k_gram_chol_mf<TM, HP>), dim3(grid), dim3(kGcNT), gram_chol_mf_smem(NV, K), st,
                     Zh, Bh, L, h, F, K, ni, rho, NV);
}

hipError_t launch_gram_chol_mf(const cpx<double>* Zh, const cpx<double>* Bh, cpx<double>* L,
                               cpx<double>* h, int F, int K, int ni, double rho, int NV,
                               hipStream_t st) {
  if (!gram_chol_mf_ok(K, NV)) return hipErrorInvalidValue;
  switch (gc_tm(K)) {
    case 7:
      if (K * NV <= kGcNT) gram_chol_mf_go<7, 1>(Zh, Bh, L, h, F, K, ni, rho, NV, st);
      else gram_chol_mf_go<7, kGcHPT>(Zh, Bh, L, h, F, K, ni, rho, NV, st);
      break;
    case 8: gram_chol_mf_go<8, kGcHPT>(Zh, Bh, L, h, F, K, ni, rho, NV, st); break;
    case 10: gram_chol_mf_go<10, kGcHPT>(Zh, Bh, L, h, F, K, ni, rho, NV, st); break;
    default: gram_chol_mf_go<12, kGcHPT>(Zh, Bh, L, h, F, K, ni, rho, NV, st); break;
  }
  return hipGetLastError();
}

}  // namespace ccsc
