// LDS-resident mixed-radix Stockham FFT building blocks for gfx950.
//
// Replaces the fft2/ifft2/fftn builtins the reference calls on every
// (filter, patch) slice (dP:24,41,46,110,112,143,152,154).
// One workgroup (kNT threads) transforms one slice held in LDS:
//
//   R2C  (forward, MATLAB fft2):  x-pass on column pairs (two real rows packed
//        as one complex line, "split" format: re in row 2j, im in row 2j+1),
//        then y-passes over the Xh = X/2+1 half-spectrum columns.  The
//        two-for-one separation is folded into the first y-pass's loads.
//   C2R  (inverse, MATLAB real(ifft2), unnormalised): y-passes, then x-passes
//        whose first load rebuilds the Hermitian pair Z = A_2j + i*A_2j+1.
//
// Lengths are the reference's own padded grids (110 = 10*11 for 2D, 74, 42,
// 60 ...), not powers of two: padding further would change the optimisation
// problem the reference solves (SURVEY.md §7 "Hard parts").
//
// Every pass is in place: each thread keeps all of its butterflies of the pass
// in registers between a "read all" and a "write all" barrier, so one slice
// needs only its own footprint of LDS (98.6 KB at 110x110 in fp64).
#pragma once

#include "common.hpp"


#include <utility>

namespace ccsc {

// ---------------------------------------------------------------------------
// compile-time trig for the in-register DFT constants
// ---------------------------------------------------------------------------
constexpr double kPi = 3.14159265358979323846264338327950288;

constexpr double series_sin(double x) {  // |x| <= pi/4
  double t = x, s = x;
  for (int i = 1; i < 14; ++i) {
    t *= -x * x / ((2 * i) * (2 * i + 1));
    s += t;
  }
  return s;
}
constexpr double series_cos(double x) {  // |x| <= pi/4
  double t = 1.0, s = 1.0;
  for (int i = 1; i < 14; ++i) {
    t *= -x * x / ((2 * i - 1) * (2 * i));
    s += t;
  }
  return s;
}
// cos / sin of 2*pi*m/R with octant reduction done in exact integer arithmetic.
constexpr void turn_cos_sin(int m, int R, double& c, double& s) {
  m %= R;
  if (m < 0) m += R;
  // t = m / R in [0,1)
  double sc = 1.0, ss = 1.0;
  int num = m, den = R;  // t = num/den
  if (2 * num > den) {   // t > 1/2: sin(t) = -sin(1-t), cos(t) = cos(1-t)
    num = den - num;
    ss = -ss;
  }
  bool swap = false;
  if (4 * num > den) {   // t in (1/4,1/2]: cos(t) = -cos(1/2-t), sin(t) = sin(1/2-t)
    num = den - 2 * num;
    den *= 2;
    sc = -sc;
  }
  if (8 * num > den) {   // t in (1/8,1/4]: swap to 1/4 - t
    num = den - 4 * num;
    den *= 4;
    swap = true;
  }
  const double x = 2.0 * kPi * (double)num / (double)den;
  const double cx = series_cos(x), sx = series_sin(x);
  c = sc * (swap ? sx : cx);
  s = ss * (swap ? cx : sx);
}

constexpr double turn_cos(int m, int R) {
  double c = 0, s = 0;
  turn_cos_sin(m, R, c, s);
  return c;
}
constexpr double turn_sin(int m, int R) {
  double c = 0, s = 0;
  turn_cos_sin(m, R, c, s);
  return s;
}
// cos/sin(2*pi*M/R) as compile-time immediates
template <int R, int M> struct TC {
  static constexpr double c = turn_cos(M, R);
  static constexpr double s = turn_sin(M, R);
};

// compile-time loop: f(std::integral_constant<int, 0..N-1>)
template <typename Fn, int... I>
__device__ __forceinline__ void sfor_impl(Fn&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename Fn>
__device__ __forceinline__ void sfor(Fn&& f) {
  sfor_impl(f, std::make_integer_sequence<int, N>{});
}

// ---------------------------------------------------------------------------
// In-register DFT of size R:  out[q] = sum_r v[r] * exp(SIGN*2*pi*i*r*q/R),
// streamed to `sink(q, out[q])` as soon as each output (pair) is formed so the
// R outputs are never live at once (a radix-11 fp64 pass at 1024 threads must
// fit in 128 VGPRs).  Odd/even pairing (r, R-r) halves the multiplies.
// ---------------------------------------------------------------------------
template <typename T, int R, int SIGN, typename Sink>
__device__ __forceinline__ void dft_sink(cpx<T> (&v)[R], Sink&& sink) {
  if constexpr (R == 1) {
    sink(0, v[0]);
  } else if constexpr (R == 2) {
    sink(0, cadd(v[0], v[1]));
    sink(1, csub(v[0], v[1]));
  } else if constexpr (R == 4) {
    const cpx<T> a0 = cadd(v[0], v[2]), a1 = csub(v[0], v[2]);
    const cpx<T> b0 = cadd(v[1], v[3]), b1 = csub(v[1], v[3]);
    const cpx<T> b1i = {-(T)SIGN * b1.y, (T)SIGN * b1.x};  // b1 * (SIGN*i)
    sink(0, cadd(a0, b0));
    sink(2, csub(a0, b0));
    sink(1, cadd(a1, b1i));
    sink(3, csub(a1, b1i));
  } else if constexpr (R % 4 == 2 && R > 2) {
    // R = 2 M, M odd: prime-factor (Good-Thomas) split, no twiddles -- input
    // n = (M n1 + 2 n2) mod R, output k = (M k1 + (M + 1) k2) mod R; M two-point
    // butterflies then two M-point DFTs (DFT-10: 92 instead of 124 flops)
    constexpr int M = R / 2;
    cpx<T> e[M], o[M];
    sfor<M>([&](auto i) {
      constexpr int n2 = decltype(i)::value;
      constexpr int ia = (2 * n2) % R, ib = (M + 2 * n2) % R;
      e[n2] = cadd(v[ia], v[ib]);
      o[n2] = csub(v[ia], v[ib]);
    });
    dft_sink<T, M, SIGN>(e, [&](int k2, cpx<T> val) { sink(((M + 1) * k2) % R, val); });
    dft_sink<T, M, SIGN>(o, [&](int k2, cpx<T> val) { sink((M + (M + 1) * k2) % R, val); });
  } else {
    constexpr int H = (R - 1) / 2;
    constexpr bool EVEN = (R % 2) == 0;
    cpx<T> a[H + 1], b[H + 1];
    sfor<H>([&](auto ri) {
      constexpr int r = decltype(ri)::value + 1;
      a[r] = cadd(v[r], v[R - r]);
      b[r] = csub(v[r], v[R - r]);
    });
    const cpx<T> v0 = v[0];
    cpx<T> vh = {(T)0, (T)0};
    if constexpr (EVEN) vh = v[R / 2];
    {
      cpx<T> s0 = v0;
      sfor<H>([&](auto ri) { s0 = cadd(s0, a[decltype(ri)::value + 1]); });
      if constexpr (EVEN) s0 = cadd(s0, vh);
      sink(0, s0);
    }
    sfor<H>([&](auto qi) {
      constexpr int q = decltype(qi)::value + 1;
      cpx<T> re = v0;
      cpx<T> im = {(T)0, (T)0};
      sfor<H>([&](auto ri) {
        constexpr int r = decltype(ri)::value + 1;
        constexpr int m = (r * q) % R;
        constexpr T c = (T)TC<R, m>::c;
        constexpr T s = (T)TC<R, m>::s;
        re.x += a[r].x * c;
        re.y += a[r].y * c;
        im.x += b[r].x * s;
        im.y += b[r].y * s;
      });
      if constexpr (EVEN) {
        if constexpr (q & 1) re = csub(re, vh);
        else re = cadd(re, vh);
      }
      const cpx<T> ii = {-(T)SIGN * im.y, (T)SIGN * im.x};  // SIGN * i * im
      sink(q, cadd(re, ii));
      sink(R - q, csub(re, ii));
    });
    if constexpr (EVEN) {
      cpx<T> s0 = v0;
      sfor<H>([&](auto ri) {
        constexpr int r = decltype(ri)::value + 1;
        if constexpr (r & 1) s0 = csub(s0, a[r]);
        else s0 = cadd(s0, a[r]);
      });
      if constexpr ((R / 2) & 1) s0 = csub(s0, vh);
      else s0 = cadd(s0, vh);
      sink(R / 2, s0);
    }
  }
}

// ---------------------------------------------------------------------------
// Geometry of a batch of lines inside the LDS slice (units of T).
// ---------------------------------------------------------------------------
struct LineGeom {
  int nlines;   // number of independent 1D transforms
  int lstride;  // distance between consecutive lines
  int estride;  // distance between consecutive elements of a line
  int imoff;    // offset of the imaginary part from the real part
};

constexpr int kMaxPass = 3;    // pass slots of the slice kernels' fft_dir
constexpr int kPlanSlots = 4;  // plan capacity (the global line kernels of recon.hip use 4)
struct Plan1D {
  int n;
  int npass;
  int rad[kPlanSlots];
  int twoff[kPlanSlots];  // offset (complex units) of pass s's twiddle table,
                        // entries (r-1)*Ns + k = exp(-2 pi i r k / (Ns R)); a
                        // generic-radix pass appends its R roots exp(-2 pi i m/R)
  int pfa;              // n = 2 M, rad = {2, M}: the M pass is fft_pass_pfa (M = kPfaM)
};
// Radices with an unrolled in-register butterfly; any other odd factor (e.g. 37 for the
// 74-point grids of the 3D/4D configs, 131 for 262 = 2 x 131, 13 and 17 for 221) runs through
// fft_pass_generic.  The planner (plan1d, engine.cpp) takes the plan with the fewest generic
// passes, then the fewest passes, within the slice kernels' per-thread task budget.
constexpr int kGenericQP = 3;      // conjugate output pairs per generic-pass task

// Per-slice description of the 2D grid (all in units of T unless noted).
struct Grid2D {
  int X, Y;     // padded grid (MATLAB dim 1 = x fastest, dim 2 = y)
  int Xh;       // X/2 + 1 half-spectrum columns
  int RS;       // LDS row stride in T = 2*Xh
  int Yp;       // rows rounded up to even (column pairs = Yp/2)
  int F;        // Xh * Y half-spectrum bins, layout [y][x'] (x' fastest)
  Plan1D px, py;
  int ntw;      // twiddle table length (complex), both directions
};

// Load-decoding modes of the first pass of a direction.
constexpr int kModePlain = 0;
constexpr int kModeSplitToHalf = 1;   // y-forward: two-for-one separation
constexpr int kModeHermPair = 2;      // x-inverse: Z = A_2j + i*A_2j+1 (Hermitian ext.)

template <typename T>
__device__ __forceinline__ cpx<T> lds_cpx(const T* p, int imoff) {
  if (imoff == 1) {  // interleaved complex: one 16-B (fp64) / 8-B (fp32) LDS access
    const auto v = *reinterpret_cast<const typename vec2_t<T>::type*>(p);
    return {v.x, v.y};
  }
  return {p[0], p[imoff]};
}
template <typename T>
__device__ __forceinline__ void lds_cpx_store(T* p, int imoff, cpx<T> v) {
  if (imoff == 1) {
    typename vec2_t<T>::type w;
    w.x = v.x;
    w.y = v.y;
    *reinterpret_cast<typename vec2_t<T>::type*>(p) = w;
  } else {
    p[0] = v.x;
    p[imoff] = v.y;
  }
}

template <typename T>
__device__ __forceinline__ cpx<T> load_elem(const T* lds, const LineGeom& g, const Grid2D& G,
                                            int mode, int line, int e) {
  if (mode == kModePlain) {
    return lds_cpx(lds + line * g.lstride + e * g.estride, g.imoff);
  } else if (mode == kModeSplitToHalf) {
    // line = x' (half-spectrum column), e = y.  Pair j = y/2 holds rows 2j, 2j+1
    // transformed together along x in split format.
    const int j = e >> 1;
    const int x1 = line;
    const int x2 = (line == 0) ? 0 : G.X - line;
    const T* r0 = lds + (2 * j) * G.RS;
    const T* r1 = r0 + G.RS;
    const cpx<T> z1 = {r0[x1], r1[x1]};
    const cpx<T> z2 = {r0[x2], r1[x2]};
    if ((e & 1) == 0) return {(T)0.5 * (z1.x + z2.x), (T)0.5 * (z1.y - z2.y)};
    // -i/2 * (z1 - conj z2)
    return {(T)0.5 * (z1.y + z2.y), (T)-0.5 * (z1.x - z2.x)};
  } else {
    // line = pair j, e = x.  Rows 2j, 2j+1 hold interleaved half spectra.
    const int j = line;
    const bool hi = e >= G.Xh;
    const int c = hi ? G.X - e : e;
    const T* r0 = lds + (2 * j) * G.RS + 2 * c;
    cpx<T> a = lds_cpx(r0, 1);
    cpx<T> b = {(T)0, (T)0};
    if (2 * j + 1 < G.Y) b = lds_cpx(r0 + G.RS, 1);
    if (hi) {
      a.y = -a.y;
      b.y = -b.y;
    }
    return {a.x - b.y, a.y + b.x};
  }
}

// One Stockham radix-R pass over all lines, in place.
// Lane mapping (LDS bank conflicts): when the elements of a line are contiguous
// (x direction, estride 1) consecutive lanes take consecutive butterflies of
// one line; when they are strided (y direction) consecutive lanes take the
// same butterfly of consecutive lines, so every access is lane-contiguous.
template <typename T, int R, int MAXB, int SIGN, int NT = kNT>
__device__ __forceinline__ void fft_pass(T* lds, int mode, const LineGeom& gin,
                                         const LineGeom& gout, const Grid2D& G, int n, int Ns,
                                         const cpx<T>* __restrict__ tw) {
  const int nb = n / R;
  const int nl = gin.nlines;
  const int total = nl * nb;
  const bool along = gin.estride == 1;
  cpx<T> v[MAXB][R];
  int outbase[MAXB];
  // read phase: load, twiddle (so no twiddle stays live across the barrier)
#pragma unroll
  for (int b = 0; b < MAXB; ++b) {
    const int bf = (int)threadIdx.x + b * NT;
    outbase[b] = -1;
    if (bf < total) {
      int line, j;
      if (along) {
        line = bf / nb;
        j = bf - line * nb;
      } else {
        j = bf / nl;
        line = bf - j * nl;
      }
      const int k = j % Ns;
      outbase[b] = line * gout.lstride + ((j - k) * R + k) * gout.estride;
      v[b][0] = load_elem<T>(lds, gin, G, mode, line, j);
#pragma unroll
      for (int r = 1; r < R; ++r) {
        const cpx<T> x = load_elem<T>(lds, gin, G, mode, line, j + r * nb);
        if (Ns > 1) {
          cpx<T> w = tw[(r - 1) * Ns + k];  // lane-contiguous in k: no bank conflicts
          if (SIGN > 0) w.y = -w.y;
          v[b][r] = cmul(x, w);
        } else {
          v[b][r] = x;
        }
      }
    }
  }
  lds_sync();
  const int ostride = Ns * gout.estride;
#pragma unroll
  for (int b = 0; b < MAXB; ++b) {
    if (outbase[b] >= 0) {
      T* base = lds + outbase[b];
      const int imoff = gout.imoff;
      dft_sink<T, R, SIGN>(v[b], [&](int q, cpx<T> val) {
        lds_cpx_store(base + q * ostride, imoff, val);
      });
    }
  }
  lds_sync();
}

// Generic odd-prime radix-R Stockham pass (R not unrolled, e.g. 37 for the
// 74-point grids):
//   out[(j-k)R + k + q Ns] = sum_r x[j + r nb] tw(r, k) w^(r q),   w = e^(SIGN 2 pi i/R).
// The R-point DFT is evaluated in conjugate output pairs.  With twiddled inputs
// x_r, s_r = x_r + x_{R-r}, d_r = x_r - x_{R-r} (r = 1..h, h = (R-1)/2) and
// theta = 2 pi r q / R:  A = x_0 + sum_r s_r cos(theta), B = -sum_r d_r sin(theta),
// X_q = A + iB and X_{R-q} = A - iB forward (swapped for the inverse).  One task
// reads its DFT's R inputs once and produces kGenericQP pairs (task 0 also the
// DC term): ~(2R + 3h)/(2 kGenericQP) LDS reads per output instead of the
// 3(R-1) of an output-per-thread R-term sum.  The host plan keeps the task
// count within one per thread (generic_tasks() in engine.cpp).
template <typename T, int SIGN, int NT = kNT, int GT = 1>
__device__ __forceinline__ void fft_pass_generic(T* lds, int R, int mode, const LineGeom& gin,
                                              const LineGeom& gout, const Grid2D& G, int n,
                                              int Ns, const cpx<T>* __restrict__ tw) {
  // GT tasks per thread (the slice kernels use 1; the global line kernels of recon.hip
  // hold up to GT tasks' accumulators across the pass barrier)
  constexpr int QP = kGenericQP;
  const int nb = n / R;
  const int nl = gin.nlines;
  const int h = (R - 1) / 2;
  const int ng = (h + QP - 1) / QP;   // tasks per DFT
  const int total = nl * nb * ng;
  const bool along = gin.estride == 1;
  const cpx<T>* roots = tw + (R - 1) * Ns;   // (cos, -sin)(2 pi m / R)
  int dst[GT], q0[GT];
  cpx<T> dc[GT], A[GT][QP], B[GT][QP];
#pragma unroll
  for (int t = 0; t < GT; ++t) {
    const int o = (int)threadIdx.x + t * NT;
    dst[t] = -1;
    q0[t] = 0;
    if (o < total) {
      int line, j, g;
      if (along) {   // lanes contiguous in j (contiguous LDS addresses)
        j = o % nb;
        const int rest = o / nb;
        g = rest % ng;
        line = rest / ng;
      } else {       // lanes contiguous in line (strided lines: one address per line)
        line = o % nl;
        const int rest = o / nl;
        j = rest % nb;
        g = rest / nb;
      }
      const int k = j % Ns;
      q0[t] = 1 + g * QP;
      int m[QP];
#pragma unroll
      for (int i = 0; i < QP; ++i) {
        A[t][i] = {(T)0, (T)0};
        B[t][i] = {(T)0, (T)0};
        m[i] = 0;
      }
      const cpx<T> x0 = load_elem<T>(lds, gin, G, mode, line, j);
      cpx<T> sdc = {(T)0, (T)0};
      for (int r = 1; r <= h; ++r) {
        cpx<T> xa = load_elem<T>(lds, gin, G, mode, line, j + r * nb);
        cpx<T> xb = load_elem<T>(lds, gin, G, mode, line, j + (R - r) * nb);
        if (Ns > 1) {
          cpx<T> wa = tw[(r - 1) * Ns + k], wb = tw[(R - r - 1) * Ns + k];
          if (SIGN > 0) {
            wa.y = -wa.y;
            wb.y = -wb.y;
          }
          xa = cmul(xa, wa);
          xb = cmul(xb, wb);
        }
        const cpx<T> sr = cadd(xa, xb), dr = csub(xa, xb);
        sdc = cadd(sdc, sr);
#pragma unroll
        for (int i = 0; i < QP; ++i) {
          m[i] += q0[t] + i;
          if (m[i] >= R) m[i] -= R;
          const cpx<T> rt = roots[m[i]];   // (cos theta, -sin theta)
          A[t][i].x += sr.x * rt.x;
          A[t][i].y += sr.y * rt.x;
          B[t][i].x += dr.x * rt.y;
          B[t][i].y += dr.y * rt.y;
        }
      }
      dc[t] = cadd(x0, sdc);
#pragma unroll
      for (int i = 0; i < QP; ++i) A[t][i] = cadd(A[t][i], x0);
      dst[t] = line * gout.lstride + ((j - k) * R + k) * gout.estride;
    }
  }
  lds_sync();
  const int ostride = Ns * gout.estride;
#pragma unroll
  for (int t = 0; t < GT; ++t) {
    if (dst[t] >= 0) {
      // forward (SIGN < 0): X_q = A + i B, X_{R-q} = A - i B; inverse: the opposite
      if (q0[t] == 1) lds_cpx_store(lds + dst[t], gout.imoff, dc[t]);
#pragma unroll
      for (int i = 0; i < QP; ++i) {
        const int q = q0[t] + i;
        if (q <= h) {
          const cpx<T> iB = {-B[t][i].y, B[t][i].x};
          const cpx<T> xq = SIGN < 0 ? cadd(A[t][i], iB) : csub(A[t][i], iB);
          const cpx<T> xr = SIGN < 0 ? csub(A[t][i], iB) : cadd(A[t][i], iB);
          lds_cpx_store(lds + dst[t] + q * ostride, gout.imoff, xq);
          lds_cpx_store(lds + dst[t] + (R - q) * ostride, gout.imoff, xr);
        }
      }
    }
  }
  lds_sync();
}

// Second pass of a length N = 2 M line (M odd prime, compile-time roots) as a
// prime-factor (Good-Thomas) split, no twiddles.  The radix-2 Stockham pass before it
// (Ns = 1) left out[2j] = x_j + x_{j+M}, out[2j+1] = x_j - x_{j+M}; with n = (M n1 +
// 2 n2) mod N and k = (M k1 + (M+1) k2) mod N,
//   X_k = sum_{n2} W_M^{n2 k2} u^{k1}_{n2},   u^{k1}_{n2} = +-out[2 j + k1], j = 2 n2 mod M
// (the minus for k1 = 1 when 2 n2 >= M: the pair is then (x_{j+M}, x_j)).  One task =
// (line, k1, output group g of QP conjugate pairs); the slots are laid out g-major then
// k1 then line, padded to whole waves, so g and k1 are wave-uniform and every root is
// an immediate (fft_pass_generic reads one per term from LDS and twiddles its inputs).
constexpr int kPfaM = 37;   // the 74-point grids of the 3D / 4D configs (74 = 64 + 2 * 5)
constexpr int kPfaQP = 3;   // conjugate output pairs per task

__host__ __device__ constexpr int pfa_slots(int nlines, int M, int QP) {
  return ((M - 1) / 2 + QP - 1) / QP * 2 * ((nlines + 63) / 64 * 64);
}

// gi: where the radix-2 pass left the inputs (the fixed 74-point x pass stores them
// line-minor so the 37 reads per task are lane-contiguous; g otherwise); g: the output.
// PRE: the radix-2 pass before (fft_fixed.hpp fpass2_pairs) stored the symmetric input
// pairs already formed -- element k1 holds u_0, element 2 + 4 (r - 1) + 2 k1 holds
// u_r + u_{M-r} and the next one u_r - u_{M-r} -- so each task reads them instead of
// forming them (the same two adds per pair, once per line instead of once per output group)
template <int M>
__host__ __device__ constexpr int pfa_pre_slot(int r, int k1, int dif) {
  return r == 0 ? k1 : 2 + 4 * (r - 1) + 2 * k1 + dif;
}
template <typename T, int M, int SIGN, int QP, int NT, bool PRE = false>
__device__ __forceinline__ void fft_pass_pfa(T* lds, const LineGeom& g, const LineGeom& gi) {
  constexpr int H = (M - 1) / 2;
  constexpr int NG = (H + QP - 1) / QP;
  const int nl = g.nlines;
  const int lpad = (nl + 63) & ~63;
  int o = (int)threadIdx.x;
  asm volatile("" : "+v"(o));
  const int grp = __builtin_amdgcn_readfirstlane(o / (2 * lpad));
  const int k1 = __builtin_amdgcn_readfirstlane((o / lpad) & 1);
  const int line = o % lpad;
  const bool on = grp < NG && line < nl;
  T* base = lds + line * g.lstride;
  const T* ibase = lds + line * gi.lstride;
  const int es = g.estride, im = g.imoff;
  cpx<T> A[QP], S[QP], dc = {(T)0, (T)0};
#pragma unroll
  for (int i = 0; i < QP; ++i) A[i] = S[i] = {(T)0, (T)0};   // (A starts at u_0)
  auto in = [&](auto n2c, auto k1c) {
    constexpr int n2 = decltype(n2c)::value, kk = decltype(k1c)::value;
    constexpr int j = (2 * n2) % M;
    cpx<T> v = lds_cpx(ibase + (2 * j + kk) * gi.estride, gi.imoff);
    if constexpr (kk == 1 && 2 * n2 >= M) v = {-v.x, -v.y};
    return v;
  };
  auto body = [&](auto gc, auto k1c) {
    constexpr int gg = decltype(gc)::value;
    constexpr int kk = decltype(k1c)::value;
    {
      cpx<T> u0;
      if constexpr (PRE) u0 = lds_cpx(ibase + pfa_pre_slot<M>(0, kk, 0) * gi.estride, gi.imoff);
      else u0 = in(std::integral_constant<int, 0>{}, k1c);
      if constexpr (gg == 0) dc = u0;
#pragma unroll
      for (int i = 0; i < QP; ++i) A[i] = u0;
    }
    // the scheduling fence per term keeps the compiler from hoisting all 2 H loads
    // (4 H VGPRs of complex) to the top: 8 waves per SIMD cover the LDS latency
    sfor<H>([&](auto ri) {
      constexpr int r = decltype(ri)::value + 1;
      cpx<T> sr, dr;
      if constexpr (PRE) {
        sr = lds_cpx(ibase + pfa_pre_slot<M>(r, kk, 0) * gi.estride, gi.imoff);
        dr = lds_cpx(ibase + pfa_pre_slot<M>(r, kk, 1) * gi.estride, gi.imoff);
      } else {
        const cpx<T> a = in(std::integral_constant<int, r>{}, k1c);
        const cpx<T> b = in(std::integral_constant<int, M - r>{}, k1c);
        sr = cadd(a, b);
        dr = csub(a, b);
      }
      if constexpr (gg == 0) dc = cadd(dc, sr);
      sfor<QP>([&](auto ii) {
        constexpr int q = gg * QP + decltype(ii)::value + 1;
        if constexpr (q <= H) {
          constexpr int m = (r * q) % M;
          constexpr T c = (T)TC<M, m>::c;
          constexpr T sn = (T)TC<M, m>::s;
          A[ii].x += sr.x * c;
          A[ii].y += sr.y * c;
          S[ii].x += dr.x * sn;
          S[ii].y += dr.y * sn;
        }
      });
      __builtin_amdgcn_sched_barrier(0);
    });
  };
  if (on) {
    sfor<NG>([&](auto gc) {
      if (grp == decltype(gc)::value) {
        if (k1 == 0) body(gc, std::integral_constant<int, 0>{});
        else body(gc, std::integral_constant<int, 1>{});
      }
    });
  }
  lds_sync();
  auto put = [&](auto gc, auto k1c) {
    constexpr int gg = decltype(gc)::value, kk = decltype(k1c)::value;
    constexpr int N = 2 * M;
    if constexpr (gg == 0) lds_cpx_store(base + ((M * kk) % N) * es, im, dc);
    sfor<QP>([&](auto ii) {
      constexpr int q = gg * QP + decltype(ii)::value + 1;
      if constexpr (q <= H) {
        // X_q = A + SIGN i S, X_{M-q} = A - SIGN i S
        const cpx<T> iS = {-(T)SIGN * S[ii].y, (T)SIGN * S[ii].x};
        constexpr int kq = (M * kk + (M + 1) * q) % N;
        constexpr int kr = (M * kk + (M + 1) * (M - q)) % N;
        lds_cpx_store(base + kq * es, im, cadd(A[ii], iS));
        lds_cpx_store(base + kr * es, im, csub(A[ii], iS));
      }
    });
  };
  if (on) {
    sfor<NG>([&](auto gc) {
      if (grp == decltype(gc)::value) {
        if (k1 == 0) put(gc, std::integral_constant<int, 0>{});
        else put(gc, std::integral_constant<int, 1>{});
      }
    });
  }
  lds_sync();
}

// fft_pass_pfa<PRE> with dense lanes, for NL = 32 .. 49 lines: the plain form runs one task
// per (output group, k1, line) with lanes over the lines, 37 or 38 of a wave's 64.  Here wave
// g < NG takes output group g of lines 0..31 for both k1 (lane = 32 k1 + line; k1 only moves
// the input slot and the output index by M); the waves after them take lines 32..NL-1, one
// task per (line, k1, conjugate output pair q), their roots read from the LDS table `roots`
// (roots[m] = exp(2 pi i m / M), lane-varying m = r q mod M).  Same products, same order.
template <typename T, int M, int SIGN, int QP, int NT, int NL>
__device__ __forceinline__ void fft_pass_pfa_packed(T* lds, const LineGeom& g, const LineGeom& gi,
                                                    const cpx<T>* roots) {
  constexpr int H = (M - 1) / 2;
  constexpr int NG = (H + QP - 1) / QP;
  constexpr int N = 2 * M;
  constexpr int NLO = NL - 32;                     // lines past the main waves
  constexpr int NLEFT = NLO * 2 * H;               // their (line, k1, q) tasks
  static_assert(NL >= 32 && NG * 64 + NLEFT <= NT, "dense prime pass: 32..49 lines");
  int o = (int)threadIdx.x;
  asm volatile("" : "+v"(o));
  const int wave = __builtin_amdgcn_readfirstlane(o >> 6);
  const int lane = o & 63;
  const int ies = gi.estride, iim = gi.imoff, es = g.estride, im = g.imoff;
  auto slot = [&](int r, int d) { return (2 + 4 * (r - 1) + d) * ies; };   // pfa_pre_slot, k1 = 0
  cpx<T> A[QP], S[QP], dc = {(T)0, (T)0};
#pragma unroll
  for (int i = 0; i < QP; ++i) A[i] = S[i] = {(T)0, (T)0};
  int kk = 0, line = 0, q = 0;
  bool on = false;
  if (wave < NG) {
    kk = lane >> 5;
    line = lane & 31;
    on = true;
    const T* ib = lds + line * gi.lstride;
    const T* ip = ib + 2 * kk * ies;
    sfor<NG>([&](auto gc) {
      constexpr int gg = decltype(gc)::value;
      if (wave == gg) {
        const cpx<T> u0 = lds_cpx(ib + kk * ies, iim);
        if constexpr (gg == 0) dc = u0;
#pragma unroll
        for (int i = 0; i < QP; ++i) A[i] = u0;
        sfor<H>([&](auto ri) {
          constexpr int r = decltype(ri)::value + 1;
          const cpx<T> sr = lds_cpx(ip + slot(r, 0), iim);
          const cpx<T> dr = lds_cpx(ip + slot(r, 1), iim);
          if constexpr (gg == 0) dc = cadd(dc, sr);
          sfor<QP>([&](auto ii) {
            constexpr int qq = gg * QP + decltype(ii)::value + 1;
            if constexpr (qq <= H) {
              constexpr int m = (r * qq) % M;
              constexpr T c = (T)TC<M, m>::c;
              constexpr T sn = (T)TC<M, m>::s;
              A[ii].x += sr.x * c;
              A[ii].y += sr.y * c;
              S[ii].x += dr.x * sn;
              S[ii].y += dr.y * sn;
            }
          });
          __builtin_amdgcn_sched_barrier(0);
        });
      }
    });
  } else {
    const int t = (wave - NG) * 64 + lane;
    if (t < NLEFT) {
      const int qi = t / (2 * NLO), rem = t - qi * (2 * NLO);
      kk = rem / NLO;
      line = 32 + rem - kk * NLO;
      q = qi + 1;
      on = true;
      const T* ib = lds + line * gi.lstride;
      const T* ip = ib + 2 * kk * ies;
      const cpx<T> u0 = lds_cpx(ib + kk * ies, iim);
      dc = u0;
      A[0] = u0;
      int m = 0;
      sfor<H>([&](auto ri) {
        constexpr int r = decltype(ri)::value + 1;
        const cpx<T> sr = lds_cpx(ip + slot(r, 0), iim);
        const cpx<T> dr = lds_cpx(ip + slot(r, 1), iim);
        dc = cadd(dc, sr);
        m += q;
        m = m >= M ? m - M : m;
        const cpx<T> w = lds_cpx(reinterpret_cast<const T*>(roots + m), 1);
        A[0].x += sr.x * w.x;
        A[0].y += sr.y * w.x;
        S[0].x += dr.x * w.y;
        S[0].y += dr.y * w.y;
        __builtin_amdgcn_sched_barrier(0);
      });
    }
  }
  lds_sync();
  if (on) {
    T* base = lds + line * g.lstride;
    const int kd = kk * M * es;   // k1 = 1 moves every output index by M (mod N)
    if (wave < NG) {
      sfor<NG>([&](auto gc) {
        constexpr int gg = decltype(gc)::value;
        if (wave == gg) {
          if constexpr (gg == 0) lds_cpx_store(base + kd, im, dc);
          sfor<QP>([&](auto ii) {
            constexpr int qq = gg * QP + decltype(ii)::value + 1;
            if constexpr (qq <= H) {
              const cpx<T> iS = {-(T)SIGN * S[ii].y, (T)SIGN * S[ii].x};
              constexpr int kq0 = ((M + 1) * qq) % N, kr0 = ((M + 1) * (M - qq)) % N;
              lds_cpx_store(base + kq0 * es + (kq0 < M ? kd : -kd), im, cadd(A[ii], iS));
              lds_cpx_store(base + kr0 * es + (kr0 < M ? kd : -kd), im, csub(A[ii], iS));
            }
          });
        }
      });
    } else {
      if (q == 1) lds_cpx_store(base + kd, im, dc);
      const cpx<T> iS = {-(T)SIGN * S[0].y, (T)SIGN * S[0].x};
      const int kq = (M * kk + (M + 1) * q) % N, kr = (M * kk + (M + 1) * (M - q)) % N;
      lds_cpx_store(base + kq * es, im, cadd(A[0], iS));
      lds_cpx_store(base + kr * es, im, csub(A[0], iS));
    }
  }
  lds_sync();
}

template <typename T, int M, int SIGN, int QP, int NT>
__device__ __forceinline__ void fft_pass_pfa(T* lds, const LineGeom& g) {
  fft_pass_pfa<T, M, SIGN, QP, NT>(lds, g, g);
}

// Pass kinds a kernel instantiation compiles (RM): bit R for the native radix R, plus the
// generic and the prime-factor pass.  A kernel holds the registers of the largest pass it
// compiles, so the slice kernels of a known grid instantiate only that grid's passes
// (the 74-point grids: radix 2 + fft_pass_pfa, ~60 instead of ~95-127 VGPRs) and the host
// checks plan_mask(plan) against the instantiation it launches (engine.cpp).
constexpr int kRmGeneric = 1 << 12, kRmPfa = 1 << 13;
constexpr int kRmAll = 0x3fff;
constexpr int kRm74 = (1 << 2) | kRmPfa;                  // 74 = 2 * 37 (C4 / C5 planes)
constexpr int kRm42 = (1 << 2) | (1 << 3) | (1 << 7);     // 42 = 2 * 3 * 7 (C4 t lines)

// butterflies per thread of a native pass: the 74-point instantiation holds the 2 its
// radix-2 pass needs (37 x 38 butterflies over kNT threads) instead of maxb_for_radix's 4
__host__ __device__ constexpr int rm_maxb(int rm, int R) {
  return rm == kRm74 ? 2 : rm == kRm42 ? (R == 2 ? 3 : R == 3 ? 2 : 1) : maxb_for_radix(R);
}

template <typename T, int MAXB, int SIGN, int NT = kNT, int GT = 1, int BS = 1, int RM = kRmAll>
__device__ __forceinline__ void fft_pass_dispatch(int R, T* lds, int mode, const LineGeom& gin,
                                                  const LineGeom& gout, const Grid2D& G, int n,
                                                  int Ns, const cpx<T>* tw) {
  switch (R) {
#define CCSC_NATIVE_PASS(RR)                                                                   \
    case RR:                                                                                   \
      if constexpr ((RM >> RR) & 1)                                                            \
        fft_pass<T, RR, rm_maxb(RM, RR) * BS, SIGN, NT>(lds, mode, gin, gout, G, n, Ns, tw);   \
      break;
    CCSC_NATIVE_PASS(2)
    CCSC_NATIVE_PASS(3)
    CCSC_NATIVE_PASS(4)
    CCSC_NATIVE_PASS(5)
    CCSC_NATIVE_PASS(7)
    CCSC_NATIVE_PASS(8)
    CCSC_NATIVE_PASS(10)
    CCSC_NATIVE_PASS(11)
#undef CCSC_NATIVE_PASS
    default:
      if constexpr ((RM & kRmGeneric) != 0)
        fft_pass_generic<T, SIGN, NT, GT>(lds, R, mode, gin, gout, G, n, Ns, tw);
      break;
  }
}

// All passes of one direction; the first pass decodes its loads with `mode0`.
// The passes are unrolled into kMaxPass guarded slots: a runtime pass loop
// around the radix switch makes the AMDGPU structurizer keep every case's
// registers live (256 VGPRs + scratch); unrolled slots compile to ~134 VGPRs.
// `n` is laundered through an empty asm: inside a caller's loop (the K loop of
// the fused kernels) LICM would otherwise hoist every pass's loop-invariant
// index math out of the loop and keep it live in registers (256 VGPRs + 5 KB
// of scratch per lane).
template <typename T, int MAXB, int SIGN, int NSLOT = kMaxPass, int NT = kNT, int GT = 1,
          int BS = 1, int RM = kRmAll>
__device__ __forceinline__ void fft_dir(T* lds, int mode0, const LineGeom& gfirst,
                                        const LineGeom& g, const Grid2D& G, const Plan1D& p,
                                        const cpx<T>* tw) {
  static_assert(NSLOT <= kPlanSlots, "plan capacity");
  int Ns = 1;
  int n = p.n;
  asm volatile("" : "+s"(n));
  sfor<NSLOT>([&](auto si) {
    constexpr int s = decltype(si)::value;
    if (s < p.npass) {
      const int R = p.rad[s];
      const cpx<T>* tws = tw + p.twoff[s];
      if constexpr (s == 0) {
        fft_pass_dispatch<T, MAXB, SIGN, NT, GT, BS, RM>(R, lds, mode0, gfirst, g, G, n, Ns, tws);
      } else if constexpr (s == 1 && NT == kNT && (RM & kRmPfa) != 0) {
        // (the prime-factor pass: plans of kNT-thread slice kernels only)
        if (p.pfa) fft_pass_pfa<T, kPfaM, SIGN, kPfaQP, NT>(lds, g);
        else fft_pass_dispatch<T, MAXB, SIGN, NT, GT, BS, RM>(R, lds, kModePlain, g, g, G, n, Ns, tws);
      } else {
        fft_pass_dispatch<T, MAXB, SIGN, NT, GT, BS, RM>(R, lds, kModePlain, g, g, G, n, Ns, tws);
      }
      Ns *= R;
    }
  });
}

__device__ __forceinline__ LineGeom geom_xsplit(const Grid2D& G) {
  return {G.Yp / 2, 2 * G.RS, 1, G.RS};
}
__device__ __forceinline__ LineGeom geom_ycols(const Grid2D& G) {
  return {G.Xh, 2, G.RS, 1};
}

// Forward 2D R2C of the real slice in LDS rows [y*RS, y*RS+X) (rows Y..Yp-1 zero).
// Result: interleaved half spectrum, bin (x', y) at lds[y*RS + 2x'].
template <typename T, int MAXB, int RM = kRmAll>
__device__ __forceinline__ void slice_r2c(T* lds, const Grid2D& G, const cpx<T>* tw) {
  const LineGeom gx = geom_xsplit(G);
  const LineGeom gy = geom_ycols(G);
  lds_sync();
  fft_dir<T, MAXB, -1, kMaxPass, kNT, 1, 1, RM>(lds, kModePlain, gx, gx, G, G.px, tw);
  fft_dir<T, MAXB, -1, kMaxPass, kNT, 1, 1, RM>(lds, kModeSplitToHalf, gy, gy, G, G.py, tw);
}

// Inverse 2D C2R (unnormalised) of the interleaved half spectrum in LDS.
// Result: real rows [y*RS, y*RS+X).
template <typename T, int MAXB, int RM = kRmAll>
__device__ __forceinline__ void slice_c2r(T* lds, const Grid2D& G, const cpx<T>* tw) {
  const LineGeom gx = geom_xsplit(G);
  const LineGeom gy = geom_ycols(G);
  lds_sync();
  fft_dir<T, MAXB, +1, kMaxPass, kNT, 1, 1, RM>(lds, kModePlain, gy, gy, G, G.py, tw);
  fft_dir<T, MAXB, +1, kMaxPass, kNT, 1, 1, RM>(lds, kModeHermPair, gx, gx, G, G.px, tw);
}

// The pass kinds a plan needs (RM bits of fft_pass_dispatch / fft_dir).
__host__ __device__ inline int plan_mask(const Plan1D& p) {
  int m = 0;
  for (int s = 0; s < p.npass; ++s) {
    const int R = p.rad[s];
    if (s == 1 && p.pfa) m |= kRmPfa;
    else if (R == 2 || R == 3 || R == 4 || R == 5 || R == 7 || R == 8 || R == 10 || R == 11)
      m |= 1 << R;
    else m |= kRmGeneric;
  }
  return m;
}
// instantiation rm runs plan p over nlines lines: it compiles every pass kind p needs
// and holds enough butterflies per thread for each native pass
__host__ __device__ inline bool rm_covers(int rm, int m) { return (m & ~rm) == 0; }
__host__ inline bool rm_fits(int rm, const Plan1D& p, int nlines) {
  if (!rm_covers(rm, plan_mask(p))) return false;
  for (int s = 0; s < p.npass; ++s) {
    const int R = p.rad[s];
    if (s == 1 && p.pfa) continue;
    if ((plan_mask(Plan1D{R, 1, {R}, {0}, 0}) & kRmGeneric) != 0) continue;
    if ((int64_t)(p.n / R) * nlines > (int64_t)rm_maxb(rm, R) * kNT) return false;
  }
  return true;
}

}  // namespace ccsc
