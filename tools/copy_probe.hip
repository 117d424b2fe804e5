// Achievable HBM streaming rate on this GPU for bench.py's roofline line (VERDICT r05 weak 3:
// torch's copy_ understated it): a hand-written copy with 16 B per lane, U independent 16-B
// loads in flight per thread before their stores, a grid of whole rounds of workgroups on
// every CU, in the plain and the nontemporal cache policy.  copy_probe() runs `reps` timed
// copies of each form and returns the best (read + write bytes) / time in GB/s, the form in
// *form (0 plain, 1 nontemporal).  Built by ccsc_code_iccv2017_amd/build.py into
// tools/libcopy_probe.so; the engine does not use it.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <vector>

typedef double d2 __attribute__((ext_vector_type(2)));

template <int U, bool NT>
__global__ __launch_bounds__(256) void k_copy(const d2* __restrict__ src, d2* __restrict__ dst,
                                              int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x * U;
  for (int64_t base = (int64_t)blockIdx.x * blockDim.x * U + threadIdx.x; base < n; base += stride) {
    d2 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = base + (int64_t)u * blockDim.x;
      if (i < n) v[u] = NT ? __builtin_nontemporal_load(src + i) : src[i];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = base + (int64_t)u * blockDim.x;
      if (i < n) {
        if (NT) __builtin_nontemporal_store(v[u], dst + i);
        else dst[i] = v[u];
      }
    }
  }
}

extern "C" int copy_probe(const void* src, void* dst, int64_t bytes, int reps, double* gbps,
                          int* form) {
  if (!src || !dst || bytes < 16 || reps < 1 || !gbps) return 1;
  const int64_t n = bytes / 16;
  int dev = 0, ncu = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 2;
  if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 2;
  const dim3 grid((unsigned)(ncu * 8)), block(256);   // 8 workgroups (32 waves) per CU
  hipEvent_t a, b;
  if (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess) return 2;
  double best = 0;
  int best_form = 0;
  for (int f = 0; f < 2; ++f) {
    auto go = [&] {
      if (f == 0)
        hipLaunchKernelGGL((k_copy<4, false>), grid, block, 0, 0, (const d2*)src, (d2*)dst, n);
      else
        hipLaunchKernelGGL((k_copy<4, true>), grid, block, 0, 0, (const d2*)src, (d2*)dst, n);
    };
    go();   // warm-up
    std::vector<float> ts;
    for (int r = 0; r < reps; ++r) {
      hipEventRecord(a, 0);
      go();
      hipEventRecord(b, 0);
      if (hipEventSynchronize(b) != hipSuccess) return 3;
      float ms = 0;
      hipEventElapsedTime(&ms, a, b);
      ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    const double med = ts[ts.size() / 2] * 1e-3;
    const double rate = 2.0 * (double)n * 16 / med / 1e9;
    if (rate > best) {
      best = rate;
      best_form = f;
    }
  }
  hipEventDestroy(a);
  hipEventDestroy(b);
  if (hipGetLastError() != hipSuccess) return 3;
  *gbps = best;
  if (form) *form = best_form;
  return 0;
}
