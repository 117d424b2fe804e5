// Achievable HBM streaming rate on this GPU for bench.py's roofline line (VERDICT r05 weak 3:
// torch's copy_ understated it): a hand-written copy with 16 B per lane, U independent 16-B
// loads in flight per thread before their stores, a grid of whole rounds of workgroups on
// every CU (or one pass over the buffer), in the plain and the nontemporal cache policy.
// copy_probe() runs `reps` timed copies of each form and returns the best (read + write bytes)
// / time in GB/s, the form in *form (bits: see below).  Built by ccsc_code_iccv2017_amd/build.py into
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
  hipEvent_t a, b;
  if (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess) return 2;
  double best = 0;
  int best_form = 0;
  // form = policy (bit 0: nontemporal) | loads in flight (bit 1: 8, else 4) | workgroups per
  // CU (bit 2: 16, else 8) | bit 3: one pass (a grid covering the buffer, no loop)
  for (int f = 0; f < 16; ++f) {
    const bool nt = f & 1, u8 = f & 2;
    const int U = u8 ? 8 : 4;
    const int64_t one_pass = (n + 256 * U - 1) / (256 * U);
    if ((f & 8) && (f & 4)) continue;   // one pass: the grid size is the buffer's
    if ((f & 8) && one_pass >= ((int64_t)1 << 31)) continue;
    const dim3 grid((unsigned)((f & 8) ? one_pass : ncu * ((f & 4) ? 16 : 8))), block(256);
    auto go = [&] {
      const d2* s_ = (const d2*)src;
      d2* d_ = (d2*)dst;
      if (nt && u8) hipLaunchKernelGGL((k_copy<8, true>), grid, block, 0, 0, s_, d_, n);
      else if (nt) hipLaunchKernelGGL((k_copy<4, true>), grid, block, 0, 0, s_, d_, n);
      else if (u8) hipLaunchKernelGGL((k_copy<8, false>), grid, block, 0, 0, s_, d_, n);
      else hipLaunchKernelGGL((k_copy<4, false>), grid, block, 0, 0, s_, d_, n);
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
