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
constexpr size_t kSmem = (size_t)TSZ * 16;
// Prime-factor (Good-Thomas) maps of 110 = 10 x 11 (coprime, no twiddles):
//   layout A (lane n1 < 10, register n2 < 11): element (11 n1 + 10 n2) mod 110,
//     inverse n1 = e mod 10, n2 = 10 e mod 11;
//   layout B (lane k2 < 11, register k1 < 10): element (11 k1 + 100 k2) mod 110,
//     inverse k1 = e mod 10, k2 = e mod 11.
__host__ __device__ constexpr int elem_a(int n1, int n2) { return (11 * n1 + 10 * n2) % 110; }
__host__ __device__ constexpr int elem_b(int k2, int k1) { return (11 * k1 + 100 * k2) % 110; }
// bin (x' = c, y) of a 6160-bin half spectrum -> its bin slot k1*616 + c*11 + k2 (layout B of
// column c: lane k2, register k1)
__host__ __device__ constexpr int bin_slot(int f) {
  const int y = f / Xh, c = f - y * Xh;
  return (y % 10) * 616 + c * 11 + (y % 11);
}
// pixel e = y*110 + x of a slice -> its offset in state order: pair n2*550 + (y>>1)*10 + n1
// (layout A of row pair y>>1: lane n1, register n2), row parity in the pair
__host__ __device__ constexpr int state_off(int e) {
  const int y = e / X, x = e - y * X;
  return 2 * (((10 * x) % 11) * 550 + (y >> 1) * 10 + (x % 10)) + (y & 1);
}
}  // namespace zl

}  // namespace ccsc
