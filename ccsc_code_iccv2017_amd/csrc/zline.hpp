// Geometry and HBM orders of the register-line z-step (zline.hip) on the 110 x 110
// grid of C1/C2; shared with the kernels that read its state (zsplit.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>

namespace ccsc {

namespace zl {
constexpr int X = 110, Y = 110, Xh = 56, F = 6160, P = 12100;
constexpr int RS = 57;                 // T row stride in complex: 4*57 = 228 dwords, bank-spread
constexpr int NT = 768, NW = 12;       // 12 waves, five lines each
constexpr int TSZ = Y * RS;            // complex slots of T
constexpr int NTW = 110;               // W_110^m, m = 0..109
constexpr size_t kSmem = (size_t)(TSZ + NTW) * 16;
__host__ __device__ constexpr int bin_slot(int f) {
  const int y = f / Xh, c = f - y * Xh;
  return (y / 11) * 616 + c * 11 + (y % 11);
}
__host__ __device__ constexpr int state_off(int e) {
  const int y = e / X, x = e - y * X;
  return 2 * ((x / 10) * 550 + (y >> 1) * 10 + (x % 10)) + (y & 1);
}
}  // namespace zl

}  // namespace ccsc
