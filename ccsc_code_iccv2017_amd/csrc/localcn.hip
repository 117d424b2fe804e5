// Local contrast normalisation of the learners' input images:
// the 'local_cn' branch of image_helpers/CreateImages.m:299-369 followed by its
// ZERO_MEAN branch (CreateImages.m:652-657), one workgroup per image:
//
//   k      = fspecial('gaussian', [13 13], 3*1.591)                     (CI:306)
//   lmn    = rconv2(I, k), lmnsq = rconv2(I.^2, k)                       (CI:309-310)
//            rconv2 = reflection about the edge pixels (edge not repeated) then
//            conv2(..., 'valid') (image_helpers/rconv2.m:22-58)
//   lstd   = sqrt(max(lmnsq - lmn.^2, 0))                                (CI:311-313)
//   th     = median: the round(N/2)-th smallest lstd; when it is 0, the same over the
//            nonzero lstd (0 if there are none)                          (CI:334-347)
//   lstd(lstd <= th) = th; lstd(lstd == 0) = eps                         (CI:348-352)
//   I      = single((I - lmn) ./ lstd), then I - mean(I) in single       (CI:367, :655)
//
// The image (reflect-padded, (H+12) x (W+12) fp64) sits in LDS for the two 13x13
// convolutions; every thread keeps its pixels' lmn / lstd in registers; the median is
// a radix select on the IEEE bits of the non-negative stds (8 passes of 8 bits, LDS
// histograms), no sort.  Images are column-major [H, W] (MATLAB dim 1 fastest).
#include "kernels.hpp"

namespace ccsc {

constexpr int kCnNT = 1024;
constexpr int kCnR = 6;                  // 13 x 13 kernel: radius 6
constexpr int kCnMaxPix = 12;            // pixels per thread: H * W <= 12288

struct CnKernel {
  double k[13 * 13];
};

__device__ __forceinline__ int reflect_idx(int i, int n) {
  // MATLAB rconv2 reflection about the edge sample (edge not repeated), |i| < n
  if (i < 0) return -i;
  if (i >= n) return 2 * n - 2 - i;
  return i;
}

// k-th smallest (1-based) of the lanes' values v[0..cnt) (non-negative doubles: their
// bit patterns order like the values); hist: 256 ints of LDS.
__device__ uint64_t radix_select(const uint64_t (&v)[kCnMaxPix], int cnt, int64_t k, int* hist,
                                 int* shared_k) {
  uint64_t prefix = 0, mask = 0;
  for (int pass = 7; pass >= 0; --pass) {
    const int sh = pass * 8;
    for (int i = threadIdx.x; i < 256; i += kCnNT) hist[i] = 0;
    __syncthreads();
#pragma unroll
    for (int i = 0; i < kCnMaxPix; ++i)
      if (i < cnt && (v[i] & mask) == prefix) atomicAdd(&hist[(v[i] >> sh) & 255], 1);
    __syncthreads();
    if (threadIdx.x == 0) {
      int64_t acc = 0;
      int b = 0;
      for (; b < 256; ++b) {
        if (acc + hist[b] >= k) break;
        acc += hist[b];
      }
      shared_k[0] = b;
      shared_k[1] = (int)(k - acc);
    }
    __syncthreads();
    const int b = shared_k[0];
    k = shared_k[1];
    prefix |= (uint64_t)b << sh;
    mask |= (uint64_t)255 << sh;
    __syncthreads();
  }
  return prefix;
}

__global__ __launch_bounds__(kCnNT) void k_local_cn(const double* __restrict__ in,
                                                    double* __restrict__ out, int H, int W,
                                                    CnKernel kc) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int HP = H + 2 * kCnR, WP = W + 2 * kCnR;
  double* pad = reinterpret_cast<double*>(smem);                 // [WP][HP], h fastest
  int* hist = reinterpret_cast<int*>(pad + (size_t)HP * WP);     // 256 + 2
  double* red = reinterpret_cast<double*>(hist + 260);            // kCnNT / 64
  const int64_t img = blockIdx.x;
  const int N = H * W;
  const double* I = in + img * N;
  for (int e = threadIdx.x; e < HP * WP; e += kCnNT) {
    const int w = e / HP, h = e - w * HP;
    pad[e] = I[reflect_idx(w - kCnR, W) * H + reflect_idx(h - kCnR, H)];
  }
  __syncthreads();
  double lmn[kCnMaxPix], lstd[kCnMaxPix];
  uint64_t bits[kCnMaxPix];
  int cnt = 0;
#pragma unroll
  for (int i = 0; i < kCnMaxPix; ++i) {
    const int p = threadIdx.x + i * kCnNT;
    lmn[i] = 0;
    lstd[i] = 0;
    bits[i] = 0;
    if (p < N) {
      cnt = i + 1;
      const int w = p / H, h = p - w * H;
      // conv2 'valid' of the padded image with the flipped kernel (rconv2.m:58):
      // out(h, w) = sum_{u,v} pad(h + u, w + v) k(12 - u, 12 - v)
      double m = 0, q = 0;
      for (int v = 0; v < 13; ++v) {
        const double* col = pad + (w + v) * HP + h;
#pragma unroll
        for (int u = 0; u < 13; ++u) {
          const double x = col[u];
          const double kk = kc.k[(12 - v) * 13 + (12 - u)];   // k(12 - u, 12 - v), column-major
          m += x * kk;
          q += (x * x) * kk;
        }
      }
      const double var = q - m * m;
      lmn[i] = m;
      lstd[i] = sqrt(var < 0 ? 0.0 : var);
      bits[i] = (uint64_t)__double_as_longlong(lstd[i]);
    }
  }
  // ---- median floor (CI:334-347) ----
  const int64_t lq = (int64_t)floor(N / 2.0 + 0.5);
  double th = __longlong_as_double((long long)radix_select(bits, cnt, lq, hist, hist + 256));
  if (th == 0.0) {
    int z = 0;
#pragma unroll
    for (int i = 0; i < kCnMaxPix; ++i) z += (i < cnt && bits[i] == 0) ? 1 : 0;
    __syncthreads();
    if (threadIdx.x == 0) hist[258] = 0;
    __syncthreads();
    if (z) atomicAdd(&hist[258], z);
    __syncthreads();
    const int zeros = hist[258];
    const int nnz = N - zeros;
    th = 0.0;
    if (nnz > 0) {
      const int64_t lq2 = (int64_t)floor(nnz / 2.0 + 0.5);
      th = __longlong_as_double((long long)radix_select(bits, cnt, zeros + lq2, hist, hist + 256));
    }
  }
  // ---- normalise in single, zero mean in single (CI:348-367, :652-657) ----
  const double* Ip = I;
  float o[kCnMaxPix];
  double s = 0;
#pragma unroll
  for (int i = 0; i < kCnMaxPix; ++i) {
    o[i] = 0.f;
    if (i < cnt) {
      const int p = threadIdx.x + i * kCnNT;
      double sd = lstd[i] <= th ? th : lstd[i];
      if (sd == 0.0) sd = 2.220446049250313e-16;
      o[i] = (float)((Ip[p] - lmn[i]) / sd);
      s += (double)o[i];
    }
  }
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  double tot = 0;
  for (int i = 0; i < kCnNT / 64; ++i) tot += red[i];
  const float mean = (float)(tot / (double)N);
  double* O = out + img * N;
#pragma unroll
  for (int i = 0; i < kCnMaxPix; ++i)
    if (i < cnt) O[threadIdx.x + i * kCnNT] = (double)(o[i] - mean);
}

bool local_cn_ok(int H, int W) {
  if (H < 7 || W < 7) return false;          // the 13x13 reflection needs 6 samples per side
  if ((int64_t)H * W > (int64_t)kCnNT * kCnMaxPix) return false;
  const size_t lds = (size_t)(H + 12) * (W + 12) * 8 + 260 * 4 + kCnNT / 64 * 8;
  return lds <= 160 * 1024;
}

hipError_t launch_local_cn(const double* in, double* out, int64_t n, int H, int W,
                           hipStream_t st) {
  if (n <= 0) return hipSuccess;
  if (!local_cn_ok(H, W)) return hipErrorInvalidValue;
  CnKernel kc;
  // fspecial('gaussian', [13 13], 3*1.591): exp(-(x^2+y^2)/(2 sigma^2)), values below
  // eps * max set to 0, normalised to sum 1
  const double sigma = 3 * 1.591;
  double mx = 0, sum = 0;
  for (int a = 0; a < 13; ++a)
    for (int b = 0; b < 13; ++b) {
      const double x = a - 6.0, y = b - 6.0;
      kc.k[b * 13 + a] = std::exp(-(x * x + y * y) / (2 * sigma * sigma));
      mx = kc.k[b * 13 + a] > mx ? kc.k[b * 13 + a] : mx;
    }
  for (int i = 0; i < 169; ++i) {
    if (kc.k[i] < 2.220446049250313e-16 * mx) kc.k[i] = 0;
    sum += kc.k[i];
  }
  for (int i = 0; i < 169; ++i) kc.k[i] /= sum;
  const size_t lds = (size_t)(H + 12) * (W + 12) * 8 + 260 * 4 + kCnNT / 64 * 8;
  hipLaunchKernelGGL(k_local_cn, dim3((unsigned)n), dim3(kCnNT), lds, st, in, out, H, W, kc);
  return hipGetLastError();
}

}  // namespace ccsc
