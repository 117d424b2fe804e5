// Shared LDS carve-up and helpers of the slice-resident kernels.
#pragma once

#include "kernels.hpp"

namespace ccsc {

template <typename T>
struct Smem {
  cpx<T>* tw;
  T* slice;
  T* red;  // kNT/64 scratch for block reductions
};

template <typename T>
__device__ __forceinline__ Smem<T> carve(char* smem, const Grid2D& G) {
  Smem<T> s;
  s.tw = reinterpret_cast<cpx<T>*>(smem);
  s.slice = reinterpret_cast<T*>(s.tw + G.X + G.Y);
  s.red = s.slice + G.Yp * G.RS;
  return s;
}

template <typename T>
__device__ __forceinline__ void load_twiddles(cpx<T>* s_tw, const cpx<T>* __restrict__ tw,
                                              int count) {
  for (int i = threadIdx.x; i < count; i += kNT) s_tw[i] = tw[i];
}

// Zero the padding row of an odd-height grid (the partner of the last row in
// the x-direction two-for-one transform).
template <typename T>
__device__ __forceinline__ void zero_pad_row(T* lds, const Grid2D& G) {
  if (G.Yp != G.Y)
    for (int x = threadIdx.x; x < G.RS; x += kNT) lds[G.Y * G.RS + x] = (T)0;
}

// Register budget of the per-bin accumulators (bins per thread) of the fused
// per-patch kernels: NB in {2, 6, 13} covers F <= 6656 (110x110 -> F = 6160).
#define CCSC_NB_SWITCH(NBV, CALL)                      \
  switch (NBV) {                                       \
    case 2: { constexpr int NB = 2; CALL; } break;     \
    case 6: { constexpr int NB = 6; CALL; } break;     \
    case 13: { constexpr int NB = 13; CALL; } break;   \
    default: return hipErrorInvalidValue;              \
  }

}  // namespace ccsc
