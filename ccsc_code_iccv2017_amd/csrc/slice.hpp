// Shared LDS carve-up and helpers of the slice-resident kernels.
#pragma once

#include "kernels.hpp"
#include "fft_fixed.hpp"

namespace ccsc {

// Waves per SIMD a slice kernel of pass mask RM is compiled for: the masked 74-point
// instantiations fit 64 VGPRs, so two 1024-thread workgroups (two slices) share a CU
// and one's barriers and HBM waits overlap the other's passes; the all-radix build
// needs ~95-127 VGPRs (one workgroup per CU).
// (the fixed-geometry 74 build, kRm74F, needs ~70 and spills a little at 64: still
// faster than one workgroup per CU, C4 0.247 vs 0.307 s per outer iteration, round 4)
constexpr int kRm74Fbit = 1 << 14;
template <int RM>
constexpr int slice_waves() { return RM == kRmAll ? 4 : 8; }

// the slice kernels' x passes run Yp/2 column-pair lines, the y passes Xh columns
__host__ inline bool slice_fits(int rm, const Grid2D& G) {
  return rm_fits(rm, G.px, G.Yp / 2) && rm_fits(rm, G.py, G.Xh);
}

template <typename T>
struct Smem {
  cpx<T>* tw;
  T* slice;
  T* red;       // kNT/64 scratch for block reductions
  cpx<T>* acc;  // per-thread spill-free accumulator bins (fused per-patch kernels)
};

template <typename T>
__device__ __forceinline__ Smem<T> carve(char* smem, const Grid2D& G) {
  Smem<T> s;
  s.tw = reinterpret_cast<cpx<T>*>(smem);
  s.slice = reinterpret_cast<T*>(s.tw + G.ntw);
  s.red = s.slice + G.Yp * G.RS;
  s.acc = reinterpret_cast<cpx<T>*>(s.red + 16);
  return s;
}

template <typename T, int NT = kNT>
__device__ __forceinline__ void load_twiddles(cpx<T>* s_tw, const cpx<T>* __restrict__ tw,
                                              int count) {
  for (int i = threadIdx.x; i < count; i += NT) s_tw[i] = tw[i];
}

// Zero the padding row of an odd-height grid (the partner of the last row in
// the x-direction two-for-one transform).
template <typename T>
__device__ __forceinline__ void zero_pad_row(T* lds, const Grid2D& G) {
  if (G.Yp != G.Y)
    for (int x = threadIdx.x; x < G.RS; x += kNT) lds[G.Y * G.RS + x] = (T)0;
}

// LDS offset (units of T) of dense half-spectrum bin f = y*Xh + x'.
__device__ __forceinline__ int bin_off(int f, const Grid2D& G) {
  const int y = f / G.Xh;
  return y * G.RS + 2 * (f - y * G.Xh);
}

// ---- the 74 x 74 grid of the C4 / C5 configs (64 + 2 * 5), compile-time ----------
// Planned as a radix-2 pass then the 37-point prime-factor pass per direction (no
// twiddles).  kRm74F instantiations run on exactly this grid: geometry and the radix-2
// passes are compile-time (fft_fixed.hpp fpass; the runtime pass's arithmetic, bit for
// bit), so the element / bin index divisions of the slice kernels fold to multiplies
// and the pass geometry to immediates.
using Grid74 = FixedGrid<2, kPfaM, 2, kPfaM>;
constexpr int kRm74F = kRm74 | kRm74Fbit;

__host__ inline bool grid_is74(const Grid2D& G) {
  auto plan_ok = [](const Plan1D& p) {
    return p.n == Grid74::X && p.npass == 2 && p.rad[0] == 2 && p.rad[1] == kPfaM && p.pfa;
  };
  return G.X == Grid74::X && G.Y == Grid74::Y && G.RS == Grid74::RS && G.Yp == Grid74::Yp &&
         plan_ok(G.px) && plan_ok(G.py);
}

// slice geometry of an instantiation: compile-time for kRm74F, else the runtime grid
template <int RM>
struct SG {
  static constexpr bool fixed = RM == kRm74F;
  __device__ static int X(const Grid2D& G) { if constexpr (fixed) return Grid74::X; else return G.X; }
  __device__ static int Y(const Grid2D& G) { if constexpr (fixed) return Grid74::Y; else return G.Y; }
  __device__ static int Xh(const Grid2D& G) { if constexpr (fixed) return Grid74::Xh; else return G.Xh; }
  __device__ static int RS(const Grid2D& G) { if constexpr (fixed) return Grid74::RS; else return G.RS; }
  __device__ static int Yp(const Grid2D& G) { if constexpr (fixed) return Grid74::Yp; else return G.Yp; }
  __device__ static int F(const Grid2D& G) { if constexpr (fixed) return Grid74::F; else return G.F; }
  // LDS offset of the real plane's (x, y): line-minor on the fixed 74 grid (the layout
  // its x passes read and write, fpass LM), natural rows otherwise
  __device__ static int px(int x, int y, const Grid2D& G) {
    if constexpr (fixed) return x * Grid74::Yp + y;
    else return y * RS(G) + x;
  }
  __device__ static int bin(int f, const Grid2D& G) {
    const int y = f / Xh(G);
    return y * RS(G) + 2 * (f - y * Xh(G));
  }
};

// the x passes read and write the line-minor layout (fpass LM): the forward one for the
// split-to-half y pass, the inverse one, the last pass of the C2R, for the kernels' real
// planes (SG<kRm74F>::px)
// The radix-2 passes store the prime pass's symmetric input pairs already formed
// (fpass2_pairs, fft_pass_pfa<PRE = true>; the plain radix-2 pass measured slower,
// profiles/r05/pfa_pre_ab.txt).
// PK (a template parameter of the slice transforms, chosen per kernel): the prime pass with
// dense lanes (fft_pass_pfa_packed) -- the 3D plane kernels (C4 0.1884 -> 0.1836 s per outer
// iteration); the 4D kernels keep the plain form (C5 0.0157 -> 0.0159 with it,
// profiles/r05/pfa_pack_ab.txt).  QP: conjugate output pairs per prime-pass task (the 3D
// plane kernels 2, the others kPfaQP).  Every choice is a template parameter, so one
// mangled name never gets different bodies in different translation units.
// the 37 roots of the packed pass's lane-varying tasks, one LDS copy per workgroup
template <typename T>
__device__ __forceinline__ cpx<T>* pfa74_roots() {
  __shared__ __attribute__((aligned(16))) cpx<T> roots[kPfaM];
  return roots;
}
template <typename T, bool PK>
__device__ __forceinline__ void pfa74_fill_roots(int tid) {
  if constexpr (PK) {
    static constexpr double tab[kPfaM][2] = {
#define CCSC_R(m) {TC<kPfaM, m>::c, TC<kPfaM, m>::s}
        CCSC_R(0),  CCSC_R(1),  CCSC_R(2),  CCSC_R(3),  CCSC_R(4),  CCSC_R(5),  CCSC_R(6),
        CCSC_R(7),  CCSC_R(8),  CCSC_R(9),  CCSC_R(10), CCSC_R(11), CCSC_R(12), CCSC_R(13),
        CCSC_R(14), CCSC_R(15), CCSC_R(16), CCSC_R(17), CCSC_R(18), CCSC_R(19), CCSC_R(20),
        CCSC_R(21), CCSC_R(22), CCSC_R(23), CCSC_R(24), CCSC_R(25), CCSC_R(26), CCSC_R(27),
        CCSC_R(28), CCSC_R(29), CCSC_R(30), CCSC_R(31), CCSC_R(32), CCSC_R(33), CCSC_R(34),
        CCSC_R(35), CCSC_R(36)};
#undef CCSC_R
    if (tid < kPfaM) pfa74_roots<T>()[tid] = {(T)tab[tid][0], (T)tab[tid][1]};
  }
}
template <typename T, int SIGN, bool PK, int QP>
__device__ __forceinline__ void pfa74(T* lds, bool xdir) {
  using FG = Grid74;
  constexpr LineGeom gy = {FG::Xh, 2, FG::RS, 1};
  constexpr LineGeom gxi = {FG::Yp / 2, 2, FG::Yp, 1};   // line-minor
  if constexpr (PK) {
    if (xdir)
      fft_pass_pfa_packed<T, kPfaM, SIGN, QP, kNT, FG::Yp / 2>(lds, gxi, gxi, pfa74_roots<T>());
    else
      fft_pass_pfa_packed<T, kPfaM, SIGN, QP, kNT, FG::Xh>(lds, gy, gy, pfa74_roots<T>());
  } else {
    if (xdir) fft_pass_pfa<T, kPfaM, SIGN, QP, kNT, true>(lds, gxi, gxi);
    else fft_pass_pfa<T, kPfaM, SIGN, QP, kNT, true>(lds, gy, gy);
  }
}
// the radix-2 pass of a 74-point direction ahead of pfa74
template <typename T, bool XD, int SIGN, int MODE, int LM>
__device__ __forceinline__ void rad2_74(T* lds, const cpx<T>* tw, int tid) {
  fpass2_pairs<T, Grid74, kNT, XD, MODE, LM>(lds, tid);
}

// slice_r2c / slice_c2r of instantiation RM (fft.hpp), the fixed passes on kRm74F
template <typename T, int RM, bool PK = false, int QP = kPfaQP>
__device__ __forceinline__ void slice_r2c_rm(T* lds, const Grid2D& G, const cpx<T>* tw) {
  if constexpr (RM == kRm74F) {
    const int tid = threadIdx.x;
    pfa74_fill_roots<T, PK>(tid);
    lds_sync();
    rad2_74<T, true, -1, kModePlain, kLmIn | kLmOut>(lds, tw, tid);
    pfa74<T, -1, PK, QP>(lds, true);
    rad2_74<T, false, -1, kModeSplitToHalf, kLmIn>(lds, tw, tid);
    pfa74<T, -1, PK, QP>(lds, false);
  } else {
    slice_r2c<T, kMaxB, RM>(lds, G, tw);
  }
}
template <typename T, int RM, bool PK = false, int QP = kPfaQP>
__device__ __forceinline__ void slice_c2r_rm(T* lds, const Grid2D& G, const cpx<T>* tw) {
  if constexpr (RM == kRm74F) {
    const int tid = threadIdx.x;
    pfa74_fill_roots<T, PK>(tid);
    lds_sync();
    rad2_74<T, false, +1, kModePlain, 0>(lds, tw, tid);
    pfa74<T, +1, PK, QP>(lds, false);
    rad2_74<T, true, +1, kModeHermPair, kLmOut>(lds, tw, tid);
    pfa74<T, +1, PK, QP>(lds, true);
  } else {
    slice_c2r<T, kMaxB, RM>(lds, G, tw);
  }
}

// Register budget of the per-bin accumulators (bins per thread) of the fused
// per-patch kernels.
// The fused kernels keep NBR bins per thread in registers and NBL more in the
// LDS left over by the slice (kNT = 1024: NBR + NBL = 7 covers F <= 7168;
// 110x110 -> F = 6160 uses 4 + 3, i.e. 48 KB of LDS, no VGPR spill).
#define CCSC_NB_SWITCH(NBV, CALL)                                            \
  switch (NBV) {                                                             \
    case 1: { constexpr int NBR = 1, NBL = 0; CALL; } break;                 \
    case 2: { constexpr int NBR = 2, NBL = 0; CALL; } break;                 \
    case 4: { constexpr int NBR = 4, NBL = 0; CALL; } break;                 \
    case 7: { constexpr int NBR = 4, NBL = 3; CALL; } break;                 \
    default: return hipErrorInvalidValue;                                    \
  }

// Accumulator bins of one thread: NBR in registers, NBL in its private LDS
// slots (workgroups of NT threads).
template <typename T, int NBR, int NBL, int NT = kNT>
struct BinAcc {
  cpx<T> r[NBR > 0 ? NBR : 1];
  cpx<T>* l;  // S.acc + threadIdx.x, stride NT
  __device__ __forceinline__ void init(cpx<T>* lds_acc) {
    l = lds_acc + threadIdx.x;
#pragma unroll
    for (int i = 0; i < NBR; ++i) r[i] = {(T)0, (T)0};
#pragma unroll
    for (int i = 0; i < NBL; ++i) l[i * NT] = {(T)0, (T)0};
  }
  // apply fn(bin f, acc&) to every bin f = threadIdx.x + i*NT < F; the first
  // NFULL bins are known in range (compile-time grids): no guard, no branch
  template <int NFULL = 0, typename Fn>
  __device__ __forceinline__ void each(int F, Fn&& fn) {
    int tid = threadIdx.x;
    asm volatile("" : "+v"(tid));  // bin index math stays at the use (LICM)
#pragma unroll
    for (int i = 0; i < NBR; ++i) {
      const int f = tid + i * NT;
      if (i < NFULL || f < F) fn(f, r[i]);
    }
#pragma unroll
    for (int i = 0; i < NBL; ++i) {
      const int f = tid + (NBR + i) * NT;
      if (NBR + i < NFULL || f < F) {
        cpx<T> a = l[i * NT];
        fn(f, a);
        l[i * NT] = a;
      }
    }
  }
};

// Element-pair batches of one slice per thread, loaded before use so a slice
// costs one global-memory round trip instead of one per loop iteration.
constexpr int kPairBatch = 1;

}  // namespace ccsc
