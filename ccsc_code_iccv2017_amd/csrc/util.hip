// Initialisation kernels: device RNG for d0/z0 when `init` is empty (the
// reference draws randn with MATLAB's global stream, dP:38,45; it is not
// reproducible, Q11), filter embedding (dP:38-39) and block replication
// (dZ:44-47 gives every block the same z0, Q4).
#include "kernels.hpp"

#include <algorithm>

namespace ccsc {

__device__ __forceinline__ uint64_t mix64(uint64_t x) {
  x ^= x >> 30;
  x *= 0xbf58476d1ce4e5b9ULL;
  x ^= x >> 27;
  x *= 0x94d049bb133111ebULL;
  x ^= x >> 31;
  return x;
}

// Counter-based N(0,1): element i depends only on (seed, offset + i), so a
// sharded draw equals the single-GPU draw.
template <typename T>
__global__ void k_randn(T* __restrict__ out, int64_t count, uint64_t seed, uint64_t offset) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  const uint64_t g = offset + (uint64_t)i;
  const uint64_t q = g >> 1;
  const uint64_t h1 = mix64(seed ^ mix64(2 * q + 1));
  const uint64_t h2 = mix64(h1 + 0x9e3779b97f4a7c15ULL);
  const double u1 = ((double)(h1 >> 11) + 1.0) * 0x1.0p-53;  // (0, 1]
  const double u2 = (double)(h2 >> 11) * 0x1.0p-53;          // [0, 1)
  const double rr = sqrt(-2.0 * log(u1));
  double s, c;
  sincospi(2.0 * u2, &s, &c);
  out[i] = (T)((g & 1) ? rr * s : rr * c);
}

template <typename T>
hipError_t launch_randn(T* out, int64_t count, uint64_t seed, uint64_t offset, hipStream_t st) {
  // chunks of 2^30 elements: one dispatch holds at most 2^32 work-items (dP's z0 at
  // C2 is 1.2e10 values)
  constexpr int64_t kChunk = int64_t(1) << 30;
  for (int64_t c0 = 0; c0 < count; c0 += kChunk) {
    const int64_t n = count - c0 < kChunk ? count - c0 : kChunk;
    hipLaunchKernelGGL(k_randn<T>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, out + c0,
                       n, seed, offset + (uint64_t)c0);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

// D[rep][k][y][x] = d0(i, j, k) at x = (i - r) mod X, y = (j - r) mod Y; zero elsewhere.
template <typename T>
__global__ void k_embed(const T* __restrict__ d0, T* __restrict__ D, int nrep, int K, int psf,
                        int X, int Y, int Tn) {
  const int64_t P = (int64_t)X * Y * Tn;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t total = (int64_t)nrep * K * P;
  if (i >= total) return;
  const int64_t e = i % P;
  const int k = (int)((i / P) % K);
  const int x = (int)(e % X), y = (int)((e / X) % Y), t = (int)(e / ((int64_t)X * Y));
  const int r = psf / 2;
  const int ii = (x + r) % X, jj = (y + r) % Y, tt = (Tn == 1) ? 0 : (t + r) % Tn;
  const int pt = (Tn == 1) ? 1 : psf;  // 3D filters are psf^3 (L3:39-40)
  T v = (T)0;
  if (ii < psf && jj < psf && tt < pt) v = d0[ii + psf * (jj + psf * (tt + pt * (int64_t)k))];
  D[i] = v;
}

template <typename T>
hipError_t launch_embed_filters(const T* d0, T* D, int nrep, int K, int psf, const Grid2D& G,
                                int Tn, hipStream_t st) {
  const int64_t total = (int64_t)nrep * K * G.X * G.Y * Tn;
  hipLaunchKernelGGL(k_embed<T>, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, d0, D,
                     nrep, K, psf, G.X, G.Y, Tn);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_replicate(const T* src, T* dst, int64_t n, int nrep, hipStream_t st) {
  for (int r = 0; r < nrep; ++r) {
    hipError_t e = hipMemcpyAsync(dst + (int64_t)r * n, src, n * sizeof(T),
                                  hipMemcpyDeviceToDevice, st);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

// a <- a - b over n elements (grid-stride: z-sized arrays exceed 2^32 work-items)
template <typename T>
__global__ void k_sub_inplace(T* __restrict__ a, const T* __restrict__ b, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    a[i] -= b[i];
}

template <typename T>
hipError_t launch_sub_inplace(T* a, const T* b, int64_t n, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  const int64_t want = (n + 255) / 256;
  const unsigned grid = (unsigned)std::min<int64_t>(want, 256 * 64);
  hipLaunchKernelGGL(k_sub_inplace<T>, dim3(grid), dim3(256), 0, st, a, b, n);
  return hipGetLastError();
}

template hipError_t launch_sub_inplace<double>(double*, const double*, int64_t, hipStream_t);
template hipError_t launch_randn<double>(double*, int64_t, uint64_t, uint64_t, hipStream_t);
template hipError_t launch_embed_filters<double>(const double*, double*, int, int, int,
                                                 const Grid2D&, int, hipStream_t);
template hipError_t launch_replicate<double>(const double*, double*, int64_t, int, hipStream_t);

}  // namespace ccsc
