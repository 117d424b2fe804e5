// Compile-time-planned slice transforms for the learners' hot grid.
//
// The 2D configs C1/C2 pose every solve on the (100 + 2*5)^2 = 110 x 110 grid
// (dP:16), planned as two radix passes per direction,
// 110 = 11 * 10.  With the radices, line counts, strides and twiddle offsets
// known at compile time every index division becomes a constant multiply and
// the per-pass radix switch of fft.hpp disappears (that switch is what drives
// the SGPR/VGPR spills of the runtime-planned kernels).  The arithmetic is
// exactly fft.hpp's (same dft_sink butterflies, same twiddle tables, same
// pass order), so the fixed and runtime transforms agree bit for bit.
#pragma once

#include "fft.hpp"

namespace ccsc {

// LDS row stride rule of make_grid2d (engine.cpp): >= 2*Xh, 4*RS = 24 (mod 64) dwords.
constexpr int lds_row_stride(int Xh) {
  int rs = 2 * Xh;
  while (rs % 16 != 6) rs += 2;
  return rs;
}

// Grid X = RX0*RX1, Y = RY0*RY1, two passes per direction (x passes, then y
// passes, twiddle tables laid out as in make_twiddles).
template <int RX0, int RX1, int RY0, int RY1>
struct FixedGrid {
  static constexpr int X = RX0 * RX1, Y = RY0 * RY1;
  static constexpr int Xh = X / 2 + 1;
  static constexpr int RS = lds_row_stride(Xh);
  static constexpr int Yp = Y + (Y & 1);
  static constexpr int F = Xh * Y;
  static constexpr int P = X * Y;
  static constexpr int TWX0 = 0;
  static constexpr int TWX1 = TWX0 + (RX0 - 1);
  static constexpr int TWY0 = TWX1 + (RX1 - 1) * RX0;
  static constexpr int TWY1 = TWY0 + (RY0 - 1);
  static constexpr int NTW = TWY1 + (RY1 - 1) * RY0;
  static constexpr int rx0 = RX0, rx1 = RX1, ry0 = RY0, ry1 = RY1;
};

// The grid of C1/C2 (and of every 100x100-patch 2D learner with 11x11 filters).
using Grid110 = FixedGrid<11, 10, 11, 10>;

// Element load of a fixed-geometry pass (modes as fft.hpp's load_elem).
template <typename T, class FG, bool XD, int MODE, bool XPERM = false>
__device__ __forceinline__ cpx<T> fload(const T* lds, int line, int e) {
  if constexpr (MODE == kModePlain) {
    if constexpr (XD && XPERM) {   // the line-minor layout: (x, y) at Yp x + y
      return lds_cpx(lds + e * FG::Yp + 2 * line, 1);
    } else if constexpr (XD) {  // row pair: re in row 2j, im in row 2j+1
      const T* p = lds + line * (2 * FG::RS) + e;
      return {p[0], p[FG::RS]};
    } else {             // interleaved complex column
      return lds_cpx(lds + line * 2 + e * FG::RS, 1);
    }
  } else if constexpr (MODE == kModeSplitToHalf) {
    const int j = e >> 1;
    const int x1 = line;
    const int x2 = (line == 0) ? 0 : FG::X - line;
    cpx<T> z1, z2;
    if constexpr (XPERM) {   // row pair j, column x at 2 (NL x + j) (fpass XPERM)
      z1 = lds_cpx(lds + x1 * FG::Yp + 2 * j, 1);
      z2 = lds_cpx(lds + x2 * FG::Yp + 2 * j, 1);
    } else {
      const T* r0 = lds + (2 * j) * FG::RS;
      const T* r1 = r0 + FG::RS;
      z1 = {r0[x1], r1[x1]};
      z2 = {r0[x2], r1[x2]};
    }
    if ((e & 1) == 0) return {(T)0.5 * (z1.x + z2.x), (T)0.5 * (z1.y - z2.y)};
    return {(T)0.5 * (z1.y + z2.y), (T)-0.5 * (z1.x - z2.x)};
  } else {  // kModeHermPair
    const int j = line;
    const bool hi = e >= FG::Xh;
    const int c = hi ? FG::X - e : e;
    const T* r0 = lds + (2 * j) * FG::RS + 2 * c;
    cpx<T> a = lds_cpx(r0, 1);
    cpx<T> b = {(T)0, (T)0};
    if ((FG::Y & 1) == 0 || 2 * j + 1 < FG::Y) b = lds_cpx(r0 + FG::RS, 1);
    if (hi) {
      a.y = -a.y;
      b.y = -b.y;
    }
    return {a.x - b.y, a.y + b.x};
  }
}

// One in-place Stockham radix-R pass over all lines of one direction.
// XD: x direction (row-pair lines, consecutive lanes -> consecutive
// butterflies of a line); else y direction (interleaved columns, consecutive
// lanes -> consecutive lines).  `tid` is the caller's laundered thread index.
// LM (the line-minor layout: element e of row-pair line l as interleaved complex at
// 2 (NL e + l), i.e. the real plane's (x, y) at Yp x + y): bit kLmIn, the inputs are read
// from it (x passes in plain mode, the split-to-half y pass); bit kLmOut, an x pass
// stores its outputs there.  A next pass whose lanes run over the row-pair lines
// (fft_pass_pfa) then reads lane-contiguous: the natural layout puts those lanes 2 RS
// apart, a 4-way LDS bank conflict on each of its 37 reads per task.  An x pass with
// both bits runs its lanes over the lines (as the y passes): contiguous reads and stores.
constexpr int kLmIn = 1, kLmOut = 2;
template <typename T, class FG, int NT, bool XD, int R, int NS, int SIGN, int MODE, int LM = 0>
__device__ __forceinline__ void fpass(T* lds, const cpx<T>* __restrict__ tw, int tid) {
  constexpr int N = XD ? FG::X : FG::Y;
  constexpr int NL = XD ? FG::Yp / 2 : FG::Xh;
  constexpr int NB = N / R;
  constexpr int TOTAL = NL * NB;
  constexpr int MAXB = (TOTAL + NT - 1) / NT;
  constexpr int LSTR = XD ? 2 * FG::RS : 2;
  constexpr int ESTR = XD ? 1 : FG::RS;
  static_assert(NB * R == N, "radix does not divide the line length");
  constexpr bool IPERM = (LM & kLmIn) != 0, OPERM = (LM & kLmOut) != 0;
  static_assert(!IPERM || (XD ? MODE == kModePlain : MODE == kModeSplitToHalf),
                "line-minor inputs: the plain x pass or the split-to-half y pass");
  static_assert(!OPERM || XD, "line-minor outputs: x passes");
  constexpr int OLSTR = OPERM ? 2 : LSTR;
  constexpr int OESTR = OPERM ? 2 * NL : ESTR;
  // a fresh opaque copy of the thread index per pass: the pass's index math
  // cannot be scheduled ahead of the previous pass's barrier and kept live
  asm volatile("" : "+v"(tid));
  cpx<T> v[MAXB][R];
  int outbase[MAXB];
#pragma unroll
  for (int b = 0; b < MAXB; ++b) {
    const int bf = tid + b * NT;
    outbase[b] = -1;
    if (bf < TOTAL) {
      int line, j;
      if constexpr (XD && !(IPERM && OPERM)) {
        line = bf / NB;
        j = bf - line * NB;
      } else {
        j = bf / NL;
        line = bf - j * NL;
      }
      const int k = j % NS;
      outbase[b] = line * OLSTR + ((j - k) * R + k) * OESTR;
      v[b][0] = fload<T, FG, XD, MODE, IPERM>(lds, line, j);
#pragma unroll
      for (int r = 1; r < R; ++r) {
        const cpx<T> x = fload<T, FG, XD, MODE, IPERM>(lds, line, j + r * NB);
        if constexpr (NS > 1) {
          cpx<T> w = tw[(r - 1) * NS + k];
          if (SIGN > 0) w.y = -w.y;
          v[b][r] = cmul(x, w);
        } else {
          v[b][r] = x;
        }
      }
    }
  }
  lds_sync();
#pragma unroll
  for (int b = 0; b < MAXB; ++b) {
    if (outbase[b] >= 0) {
      T* base = lds + outbase[b];
      dft_sink<T, R, SIGN>(v[b], [&](int q, cpx<T> val) {
        if constexpr (XD && !OPERM) {
          base[q * NS * ESTR] = val.x;
          base[q * NS * ESTR + FG::RS] = val.y;
        } else {
          lds_cpx_store(base + q * NS * OESTR, 1, val);
        }
      });
    }
  }
  lds_sync();
}

// The radix-2 Stockham pass (NS = 1) of a length N = 2 M line ahead of fft_pass_pfa<PRE>:
// one task per line and input pair r of the M-point pass -- the butterflies j = 2 r and
// M - 2 r (r = 0: butterfly 0 alone) -- storing the pairs the prime pass sums over,
//   k1 = 0: out[4r] +- out[2(M-2r)],  k1 = 1: out[4r+1] -+ out[2(M-2r)+1]
// (out[2j] = x_j + x_{j+M}, out[2j+1] = x_j - x_{j+M}; the k1 = 1 partner enters the prime
// pass negated, fft_pass_pfa) at elements pfa_pre_slot: the same adds, formed once per line
// here instead of once per output group there, and H + 1 tasks per line instead of M.
// Loads as fpass (MODE, kLmIn); stores line-minor for x passes (kLmOut required),
// interleaved columns for y passes.
template <typename T, class FG, int NT, bool XD, int MODE, int LM = 0>
__device__ __forceinline__ void fpass2_pairs(T* lds, int tid) {
  constexpr int N = XD ? FG::X : FG::Y;
  constexpr int M = N / 2;
  constexpr int H = (M - 1) / 2;
  constexpr int NL = XD ? FG::Yp / 2 : FG::Xh;
  constexpr int NP = H + 1;
  constexpr int TOTAL = NL * NP;
  constexpr int MAXB = (TOTAL + NT - 1) / NT;
  constexpr bool IPERM = (LM & kLmIn) != 0, OPERM = (LM & kLmOut) != 0;
  static_assert(N == 2 * M && (M & 1), "a 2 x odd line");
  static_assert(!XD || OPERM, "x passes store line-minor");
  constexpr int OESTR = XD ? 2 * NL : FG::RS;
  asm volatile("" : "+v"(tid));
  cpx<T> v[MAXB][4];
  int ob[MAXB], rr[MAXB];
#pragma unroll
  for (int b = 0; b < MAXB; ++b) {
    const int bf = tid + b * NT;
    ob[b] = -1;
    rr[b] = 0;
    if (bf < TOTAL) {
      int line, r;
      if constexpr (XD && !IPERM) {   // lanes over a line's pairs (the HermPair x pass)
        line = bf / NP;
        r = bf - line * NP;
      } else {                        // lanes over the lines
        r = bf / NL;
        line = bf - r * NL;
      }
      ob[b] = 2 * line;
      rr[b] = r;
      const int j = 2 * r;
      v[b][0] = fload<T, FG, XD, MODE, IPERM>(lds, line, j);
      v[b][1] = fload<T, FG, XD, MODE, IPERM>(lds, line, j + M);
      if (r > 0) {
        v[b][2] = fload<T, FG, XD, MODE, IPERM>(lds, line, M - j);
        v[b][3] = fload<T, FG, XD, MODE, IPERM>(lds, line, N - j);
      }
    }
  }
  lds_sync();
#pragma unroll
  for (int b = 0; b < MAXB; ++b) {
    if (ob[b] >= 0) {
      T* base = lds + ob[b];
      const cpx<T> e0 = cadd(v[b][0], v[b][1]), o0 = csub(v[b][0], v[b][1]);
      const int r = rr[b];
      if (r == 0) {
        lds_cpx_store(base + pfa_pre_slot<M>(0, 0, 0) * OESTR, 1, e0);
        lds_cpx_store(base + pfa_pre_slot<M>(0, 1, 0) * OESTR, 1, o0);
      } else {
        const cpx<T> e1 = cadd(v[b][2], v[b][3]), o1 = csub(v[b][2], v[b][3]);
        T* p = base + pfa_pre_slot<M>(r, 0, 0) * OESTR;
        lds_cpx_store(p, 1, cadd(e0, e1));
        lds_cpx_store(p + OESTR, 1, csub(e0, e1));
        lds_cpx_store(p + 2 * OESTR, 1, csub(o0, o1));
        lds_cpx_store(p + 3 * OESTR, 1, cadd(o0, o1));
      }
    }
  }
  lds_sync();
}

// Forward 2D R2C (MATLAB fft2) of the real slice in LDS rows [y*RS, y*RS+X);
// result: interleaved half spectrum, bin (x', y) at lds[y*RS + 2x'].
// (A wave-local variant -- each 110-point line owned by 11 lanes of one wave,
// its two radix stages exchanging through the line's own LDS slots, 3 barriers
// per 2D transform instead of 9 -- measured 5% slower on the C2 z-iteration:
// these passes are LDS/VALU-throughput bound, not barrier bound.)
template <typename T, class FG, int NT>
__device__ __forceinline__ void fslice_r2c(T* lds, const cpx<T>* tw, int tid) {
  lds_sync();
  fpass<T, FG, NT, true, FG::rx0, 1, -1, kModePlain>(lds, tw + FG::TWX0, tid);
  fpass<T, FG, NT, true, FG::rx1, FG::rx0, -1, kModePlain>(lds, tw + FG::TWX1, tid);
  fpass<T, FG, NT, false, FG::ry0, 1, -1, kModeSplitToHalf>(lds, tw + FG::TWY0, tid);
  fpass<T, FG, NT, false, FG::ry1, FG::ry0, -1, kModePlain>(lds, tw + FG::TWY1, tid);
}

// Inverse 2D C2R (unnormalised) of the interleaved half spectrum in LDS.
template <typename T, class FG, int NT>
__device__ __forceinline__ void fslice_c2r(T* lds, const cpx<T>* tw, int tid) {
  lds_sync();
  fpass<T, FG, NT, false, FG::ry0, 1, +1, kModePlain>(lds, tw + FG::TWY0, tid);
  fpass<T, FG, NT, false, FG::ry1, FG::ry0, +1, kModePlain>(lds, tw + FG::TWY1, tid);
  fpass<T, FG, NT, true, FG::rx0, 1, +1, kModeHermPair>(lds, tw + FG::TWX0, tid);
  fpass<T, FG, NT, true, FG::rx1, FG::rx0, +1, kModePlain>(lds, tw + FG::TWX1, tid);
}

// Runtime-planned grids (every other size): the same slice kernels, with
// geometry from Grid2D and the transforms of fft.hpp.
struct DynGrid {
  static constexpr int P = 0;  // runtime size (Grid2D)
};

template <class FG, int NT = kNT>
struct GridOps {
  static constexpr int kThreads = NT;
  __device__ static constexpr int X(const Grid2D&) { return FG::X; }
  __device__ static constexpr int Y(const Grid2D&) { return FG::Y; }
  __device__ static constexpr int Xh(const Grid2D&) { return FG::Xh; }
  __device__ static constexpr int RS(const Grid2D&) { return FG::RS; }
  __device__ static constexpr int Yp(const Grid2D&) { return FG::Yp; }
  __device__ static constexpr int F(const Grid2D&) { return FG::F; }
  __device__ static constexpr int ntw(const Grid2D&) { return FG::NTW; }
  template <typename T>
  __device__ __forceinline__ static void r2c(T* lds, const Grid2D&, const cpx<T>* tw, int tid) {
    fslice_r2c<T, FG, NT>(lds, tw, tid);
  }
  template <typename T>
  __device__ __forceinline__ static void c2r(T* lds, const Grid2D&, const cpx<T>* tw, int tid) {
    fslice_c2r<T, FG, NT>(lds, tw, tid);
  }
};

template <>
struct GridOps<DynGrid, kNT> {
  static constexpr int kThreads = kNT;
  __device__ static int X(const Grid2D& G) { return G.X; }
  __device__ static int Y(const Grid2D& G) { return G.Y; }
  __device__ static int Xh(const Grid2D& G) { return G.Xh; }
  __device__ static int RS(const Grid2D& G) { return G.RS; }
  __device__ static int Yp(const Grid2D& G) { return G.Yp; }
  __device__ static int F(const Grid2D& G) { return G.F; }
  __device__ static int ntw(const Grid2D& G) { return G.ntw; }
  template <typename T>
  __device__ __forceinline__ static void r2c(T* lds, const Grid2D& G, const cpx<T>* tw, int) {
    slice_r2c<T, kMaxB>(lds, G, tw);
  }
  template <typename T>
  __device__ __forceinline__ static void c2r(T* lds, const Grid2D& G, const cpx<T>* tw, int) {
    slice_c2r<T, kMaxB>(lds, G, tw);
  }
};

// Host: does the runtime plan of G equal the fixed grid FG (plans, stride,
// twiddle layout)?
template <class FG>
inline bool grid_is(const Grid2D& G) {
  return G.X == FG::X && G.Y == FG::Y && G.RS == FG::RS && G.ntw == FG::NTW &&
         G.px.npass == 2 && G.px.rad[0] == FG::rx0 && G.px.rad[1] == FG::rx1 &&
         G.py.npass == 2 && G.py.rad[0] == FG::ry0 && G.py.rad[1] == FG::ry1 &&
         G.px.twoff[0] == FG::TWX0 && G.px.twoff[1] == FG::TWX1 && G.py.twoff[0] == FG::TWY0 &&
         G.py.twoff[1] == FG::TWY1;
}

}  // namespace ccsc
