// Issue-rate probe for the two fp64 pipes the D-precompute can use on gfx950:
// v_mfma_f64_16x16x4_f64 (matrix cores) and v_fma_f64 (VALU).  Each wave runs
// independent accumulator chains (enough to cover the pipe latency) for N iterations;
// the whole grid fills every SIMD with `wpe` waves.  Prints Tflop/s and cycles per
// wave-instruction per SIMD at the measured clock.
//   hipcc -O3 --offload-arch=gfx950 tools/rate_probe.hip -o build/rate_probe
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double d4 __attribute__((ext_vector_type(4)));

template <int CH>
__global__ __launch_bounds__(256) void k_mfma(double* out, int n, double a0) {
  d4 acc[CH];
  for (int c = 0; c < CH; ++c) acc[c] = (d4){0, 0, 0, 0};
  double a = a0 + threadIdx.x * 1e-9, b = a0 - threadIdx.x * 1e-9;
  for (int i = 0; i < n; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) acc[c] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[c], 0, 0, 0);
  }
  double s = 0;
  for (int c = 0; c < CH; ++c) s += acc[c][0] + acc[c][1] + acc[c][2] + acc[c][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int CH>
__global__ __launch_bounds__(256) void k_fma(double* out, int n, double a0) {
  double acc[CH];
  for (int c = 0; c < CH; ++c) acc[c] = c;
  const double a = a0 + threadIdx.x * 1e-9, b = 1.0 - 1e-12;
  for (int i = 0; i < n; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) acc[c] = fma(acc[c], b, a);
  }
  double s = 0;
  for (int c = 0; c < CH; ++c) s += acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  const int cus = p.multiProcessorCount;
  double* out;
  hipMalloc(&out, (size_t)cus * 8 * 256 * 8);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const double clk = p.clockRate * 1e3;   // Hz (peak engine clock)
  for (int wpe = 1; wpe <= 2; ++wpe) {
    const int blocks = cus * wpe;   // 4 waves per WG = one per SIMD
    const int n = 20000;
    for (int rep = 0; rep < 2; ++rep) {
      hipEventRecord(e0);
      hipLaunchKernelGGL(k_mfma<8>, dim3(blocks), dim3(256), 0, 0, out, n, 1.0);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      const double inst = (double)blocks * 4 * n * 8;   // wave-level MFMAs
      const double fl = inst * 2048.0;
      if (rep)
        printf("mfma_f64_16x16x4 waves/SIMD %d: %.3f ms, %.1f TFLOP/s, %.1f cycles per MFMA per SIMD at %.0f MHz\n",
               wpe, ms, fl / ms / 1e9, (ms * 1e-3 * clk) / (inst / (cus * 4)), clk / 1e6);
    }
    for (int rep = 0; rep < 2; ++rep) {
      hipEventRecord(e0);
      hipLaunchKernelGGL(k_fma<16>, dim3(blocks), dim3(256), 0, 0, out, n, 1.0);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      const double inst = (double)blocks * 4 * n * 16;
      const double fl = inst * 64 * 2;
      if (rep)
        printf("v_fma_f64 waves/SIMD %d: %.3f ms, %.1f TFLOP/s, %.2f cycles per wave-FMA per SIMD\n", wpe,
               ms, fl / ms / 1e9, (ms * 1e-3 * clk) / (inst / (cus * 4)));
    }
  }
  hipFree(out);
  return 0;
}
