// Common device/host helpers for libccsc (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstddef>

namespace ccsc {

// 16-B aligned (fp64): every complex array of the engine starts 16-B aligned with
// complex-sized elements, so one 16-B access per element instead of two 8-B ones
template <typename T> struct alignas(2 * sizeof(T)) cpx { T x, y; };
// predicated complex load as one 16-B access (a `c ? p[i] : zero` select is split by the
// compiler into two 8-B loads)
template <typename T>
__device__ __forceinline__ cpx<T> ldc_if(bool c, const cpx<T>* p) {
  cpx<T> v = {(T)0, (T)0};
  if (c) v = *p;
  return v;
}
template <typename T> struct vec2_t;
template <> struct vec2_t<double> { using type = double2; };
template <> struct vec2_t<float> { using type = float2; };

template <typename T>
__host__ __device__ __forceinline__ cpx<T> cmul(cpx<T> a, cpx<T> b) {
  return {a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x};
}
// conj(a) * b
template <typename T>
__host__ __device__ __forceinline__ cpx<T> cmulc(cpx<T> a, cpx<T> b) {
  return {a.x * b.x + a.y * b.y, a.x * b.y - a.y * b.x};
}
template <typename T>
__host__ __device__ __forceinline__ cpx<T> cadd(cpx<T> a, cpx<T> b) { return {a.x + b.x, a.y + b.y}; }
// acc + a b and acc + conj(a) b as four FMAs (cadd(acc, cmul(a, b)) compiles to a mul, an FMA
// and an add per component: the sum cannot be reassociated into the product)
template <typename T>
__host__ __device__ __forceinline__ cpx<T> cmac(cpx<T> acc, cpx<T> a, cpx<T> b) {
  return {fma(a.x, b.x, fma(-a.y, b.y, acc.x)), fma(a.x, b.y, fma(a.y, b.x, acc.y))};
}
template <typename T>
__host__ __device__ __forceinline__ cpx<T> cmacc(cpx<T> acc, cpx<T> a, cpx<T> b) {
  return {fma(a.x, b.x, fma(a.y, b.y, acc.x)), fma(a.x, b.y, fma(-a.y, b.x, acc.y))};
}
// acc - a b and acc - conj(a) b, likewise
template <typename T>
__host__ __device__ __forceinline__ cpx<T> cmsub(cpx<T> acc, cpx<T> a, cpx<T> b) {
  return {fma(-a.x, b.x, fma(a.y, b.y, acc.x)), fma(-a.x, b.y, fma(-a.y, b.x, acc.y))};
}
template <typename T>
__host__ __device__ __forceinline__ cpx<T> cmsubc(cpx<T> acc, cpx<T> a, cpx<T> b) {
  return {fma(-a.x, b.x, fma(-a.y, b.y, acc.x)), fma(-a.x, b.y, fma(a.y, b.x, acc.y))};
}
template <typename T>
__host__ __device__ __forceinline__ cpx<T> csub(cpx<T> a, cpx<T> b) { return {a.x - b.x, a.y - b.y}; }
template <typename T>
__host__ __device__ __forceinline__ cpx<T> cscale(cpx<T> a, T s) { return {a.x * s, a.y * s}; }
template <typename T>
__host__ __device__ __forceinline__ T cabs2(cpx<T> a) { return a.x * a.x + a.y * a.y; }

// Block size of every slice-resident kernel: 16 waves of 64 lanes (one
// workgroup per CU holds a whole fp64 slice in LDS, so the waves of that one
// workgroup are all the latency hiding the CU gets).
constexpr int kNT = 1024;
// Butterflies per FFT pass that the threads hold in registers at once (the
// in-place pass needs every butterfly of the pass live between its read and
// write barriers); MAXB = kMaxButterflies / kNT per thread.
constexpr int kMaxButterflies = 1024;
constexpr int kMaxB = kMaxButterflies / kNT;
// Small radices cost few registers per butterfly, so a thread may hold more of
// them (needed e.g. by the radix-2 pass of the 74-point grids: 37 x 37 = 1369).
__host__ __device__ constexpr int maxb_for_radix(int R) {
  return (R <= 4 ? 4 : (R <= 8 ? 2 : 1)) * kMaxB;
}

// Workgroup barrier for LDS hand-offs only.  __syncthreads() also waits
// vmcnt(0), i.e. it drains every outstanding global load/store of the wave at
// each of the ~20 barriers of a slice transform; this one waits only for the
// wave's LDS ops, so global stores keep draining (and loads stay in flight)
// underneath the FFT.  The "memory" clobber keeps the compiler from moving
// memory ops across it; register dependences on pending global loads are
// still guarded by the compiler's own vmcnt waits.
__device__ __forceinline__ void lds_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// Wave-level sum (64 lanes) via shuffles.
template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Block-level sum of one value per thread; result valid in every thread.
// `scratch` must hold kNT/64 elements and not alias live data.
template <typename T>
__device__ __forceinline__ T block_sum(T v, T* scratch) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) scratch[w] = v;
  __syncthreads();
  T s = 0;
#pragma unroll
  for (int i = 0; i < kNT / 64; ++i) s += scratch[i];
  __syncthreads();
  return s;
}

// A block-strided loop (NT threads) over n elements whose global loads are issued B at a
// time before any is used: one memory round trip per batch instead of per element.  As plain
// `for (e = tid; e < n; e += NT)` loops the compiler waits vmcnt(0) for every iteration's own
// load (the 3D plane kernels made 3 and 6 dependent HBM round trips per plane and thread, the
// line passes of recon.hip ~10 per workgroup).  ld(e) loads, use(e, v) consumes.
template <int B, int NT = kNT, typename Ld, typename Use>
__device__ __forceinline__ void batched_loop(int n, Ld&& ld, Use&& use) {
  using V = decltype(ld(0));
  for (int base = threadIdx.x; base < n; base += B * NT) {
    V v[B];
#pragma unroll
    for (int i = 0; i < B; ++i) {
      const int e = base + i * NT;
      if (e < n) v[i] = ld(e);
    }
#pragma unroll
    for (int i = 0; i < B; ++i) {
      const int e = base + i * NT;
      if (e < n) use(e, v[i]);
    }
  }
}
template <typename T>
struct Pair2 {
  T a, b;
};

}  // namespace ccsc
