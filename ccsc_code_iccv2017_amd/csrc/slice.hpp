// Shared LDS carve-up and helpers of the slice-resident kernels.
#pragma once

#include "kernels.hpp"

namespace ccsc {

// Waves per SIMD a slice kernel of pass mask RM is compiled for: the masked 74-point
// instantiations fit 64 VGPRs, so two 1024-thread workgroups (two slices) share a CU
// and one's barriers and HBM waits overlap the other's passes; the all-radix build
// needs ~95-127 VGPRs (one workgroup per CU).
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
