// Reconstruction solvers on gfx950: global line transforms with fused ADMM updates.
//
// One ADMM iteration of every solver (SI:81-139, SP:75-127, SD:53-86, SV:58-107) is
//   v1 = real(ifft(sum_k dhat_k zhat_k)), v2 = z
//   u1 = ProxData(v1 - d1), u2 = ProxSparse(z - d2); d += u - v; xi = u + d; fft(xi)
//   zhat = solve(xi_hat1, xi_hat2); z = real(ifft(zhat))
// and runs here as four passes over the half spectra of the K code slices (Sz) and
// the W data slices (Sx):
//   k_rows  (inverse x-lines of the previous column pass, the elementwise update of
//           z / v1 with its partial sums, forward x-lines of xi)      [one pass]
//   k_cols  forward y (and t) lines
//   solve   per bin (k_solve_sm, or the per-bin GEMMs of hs23.hip for the diagonal
//           solves of SD / SL / SV), 1/P folded in, and the synthesis sum_k dhat zhat
//   k_cols  inverse y (and t) lines
// so each spectrum crosses HBM four times per iteration and each real state array
// (z, d2, d1) once in each direction.
#include "recon.hpp"

namespace ccsc {

template <typename T>
__device__ __forceinline__ T soft_thr(T a, T th) {
  // max(0, 1 - th/|a|) * a without the divide (SI:32; a = 0 -> 0)
  return a > th ? a - th : (a < -th ? a + th : (T)0);
}

// block-level sum over the kLineNT threads (scratch: kLineNT / 64 elements)
template <typename T>
__device__ __forceinline__ T line_block_sum(T v, T* scratch) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) scratch[w] = v;
  __syncthreads();
  T s = 0;
#pragma unroll
  for (int i = 0; i < kLineNT / 64; ++i) s += scratch[i];
  __syncthreads();
  return s;
}

// ---------------------------------------------------------------------------
// Row pass: 2L rows (L row pairs) of one slice per workgroup.  LDS rows of RS T.
// ---------------------------------------------------------------------------
template <typename T, int MODE>
__device__ __forceinline__ void rows_body(const RowArgs<T>& a, const RowGeom& rg,
                                          const cpx<T>* __restrict__ tw, int64_t slice, T* lds) {
  Grid2D G = rg.G;
  const int X = G.X, Xh = G.Xh, RS = G.RS;
  const int g = blockIdx.y;
  const int row0 = g * 2 * rg.L;
  const int nrows = min(2 * rg.L, rg.rows - row0);
  G.Y = nrows;
  G.Yp = nrows + (nrows & 1);
  const LineGeom gx = geom_xsplit(G);
  const int64_t img = slice / a.per_img;
  const int sl = (int)(slice - img * a.per_img);
  const int64_t rbase = (slice * rg.rows + row0) * (int64_t)X;     // real arrays
  const int64_t sbase = (slice * rg.rows + row0) * (int64_t)Xh;    // spectra
  // twiddle tables in LDS (every pass reads them per butterfly)
  cpx<T>* s_tw = reinterpret_cast<cpx<T>*>(lds + rows_tw_off(rg));
  batched_loop<4, kLineNT>(rg.ntw, [&](int i) { return tw[i]; }, [&](int i, cpx<T> v) { s_tw[i] = v; });

  // ---- load (batched: every load of a batch in flight before the first LDS store) ----
  if (MODE == kRowFwd) {
    batched_loop<4, kLineNT>(
        G.Yp * X,
        [&](int i) {
          const int ry = i / X, x = i - ry * X;
          return ry < nrows ? a.src[rbase + (int64_t)ry * X + x] : (T)0;
        },
        [&](int i, T v) {
          const int ry = i / X, x = i - ry * X;
          lds[ry * RS + x] = v;
        });
  } else if (a.first) {
    for (int i = threadIdx.x; i < G.Yp * X; i += kLineNT) {
      const int ry = i / X, x = i - ry * X;
      lds[ry * RS + x] = (T)0;
    }
  } else {
    batched_loop<4, kLineNT>(
        nrows * Xh, [&](int i) { return a.S[sbase + i]; },
        [&](int i, cpx<T> c) {
          const int ry = i / Xh, xp = i - ry * Xh;
          lds[ry * RS + 2 * xp] = c.x;
          lds[ry * RS + 2 * xp + 1] = c.y;
        });
    lds_sync();
    fft_dir<T, kMaxB, +1, kPlanSlots, kLineNT, kLineGT, kLineBS>(lds, kModeHermPair, gx, gx, G, G.px, s_tw);
  }
  lds_sync();

  // ---- elementwise ----------------------------------------------------------
  T p0 = 0, p1 = 0, p2 = 0;
  if (MODE == kRowIterZ || MODE == kRowFinalZ) {
    const bool act = !a.active || a.active[img] != 0;
    const T th = a.theta ? a.theta[img] : (T)0;
    const bool ident = a.prox == 1 && sl == 0;
    batched_loop<4, kLineNT>(
        nrows * X,
        [&](int i) {
          const int64_t gi = rbase + i;   // (rows of X reals: gi = rbase + ry X + x)
          return Pair2<T>{a.Z[gi], MODE == kRowIterZ ? a.D[gi] : (T)0};
        },
        [&](int i, Pair2<T> zd) {
          const int ry = i / X, x = i - ry * X;
          const int64_t gi = rbase + i;
          const T z = lds[ry * RS + x];
          const T dz = z - zd.a;
          p0 += dz * dz;
          p1 += z * z;
          p2 += fabs(z);
          if (act) a.Z[gi] = z;
          if (MODE == kRowIterZ) {
            const T d = zd.b;
            const T av = z - d;                               // v2 - d2
            const T u = ident ? av : soft_thr(av, th);        // SI:89, SP:84
            const T dn = d - (z - u);                         // SI:93
            a.D[gi] = dn;
            lds[ry * RS + x] = u + dn;                        // xi2 (SI:96)
          }
        });
  } else if (MODE == kRowIterX) {
    const T th = a.theta[img];
    const T ith = (T)1 / th;
    struct XIn {
      T m, mb, sm, d;
    };
    batched_loop<2, kLineNT>(
        nrows * X,
        [&](int i) {
          const int64_t gi = rbase + i;
          return XIn{a.M[gi], a.Mb[gi], a.SM ? a.SM[gi] : (T)0, a.D[gi]};
        },
        [&](int i, XIn in) {
          const int ry = i / X, x = i - ry * X;
          const int64_t gi = rbase + (int64_t)ry * X + x;
          const T v = lds[ry * RS + x];
          const T m = in.m, mb = in.mb;
          const T sm = in.sm;
          // objective residual mask .* crop(Dz) - mask .* b (SI:196; SD:144 and SV:171 with
          // smoothinit); M is zero outside the image, so the whole grid is the crop
          const T e = m * (v + (a.obj_sm ? sm : (T)0)) - mb;
          p0 += e * e;
          if (a.XO) {
            const int row = row0 + ry;
            const int y = row % a.Y;
            if (x >= a.px0 && x < a.px1 && y >= a.py0 && y < a.py1) {
              const T q = a.XO[gi] - (v + (a.psnr_sm ? sm : (T)0));   // SI:60
              p1 += q * q;
            }
          }
          const T d = in.d;
          const T w = v - d;
          T u;
          if (a.prox == 1) {   // Poisson where data is present, identity elsewhere (SP:193-205)
            const T wt = w - th;
            u = m != (T)0 ? (T)0.5 * (wt + sqrt(wt * wt + (T)4 * th * mb)) : w;
          } else {             // (Mtb + w/th) / (MtM + 1/th), Mtb = M b - M smoothinit (SI:29,152)
            const T mtb = mb - m * sm;
            const T mtm = a.mtm_sq ? m * m : m;
            u = (mtb + ith * w) / (mtm + ith);
          }
          const T dn = d - (v - u);
          a.D[gi] = dn;
          lds[ry * RS + x] = u + dn;                          // xi1
        });
  } else if (MODE == kRowRes) {
    for (int i = threadIdx.x; i < nrows * X; i += kLineNT) {
      const int ry = i / X, x = i - ry * X;
      const int row = row0 + ry;
      const int y = row % a.Y, t = row / a.Y;
      const int xo = x - a.rx, yo = y - a.ry, to = t - a.rt;
      if (xo < 0 || xo >= a.sbx || yo < 0 || yo >= a.sby || to < 0 || to >= a.sbt) continue;
      const int64_t gi = rbase + (int64_t)ry * X + x;
      T v = lds[ry * RS + x] * a.scale + (a.SM ? a.SM[gi] : (T)0);
      if (a.clamp0 && v < (T)0) v = (T)0;
      a.res[((slice * a.sbt + to) * a.sby + yo) * (int64_t)a.sbx + xo] = v;
    }
  }
  if (MODE != kRowFwd && MODE != kRowRes && a.part) {
    T* scratch = lds + (size_t)G.Yp * RS + 16;   // past the slice (rows_smem_bytes)
    const T s0 = line_block_sum(p0, scratch);
    const T s1 = line_block_sum(p1, scratch);
    const T s2 = line_block_sum(p2, scratch);
    if (threadIdx.x == 0) {
      const int off = (MODE == kRowIterX) ? 3 : 0;   // codes: dz^2, z^2, |z|; data: obj, psnr
      T* pp = a.part + (((img * a.part_slices + a.part_off + sl) * rg.groups) + g) * kRowParts;
      for (int j = 0; j < kRowParts; ++j) pp[j] = (T)0;
      pp[off] = s0;
      pp[off + 1] = s1;
      if (off == 0) pp[2] = s2;
    }
  }
  if (MODE == kRowFinalZ || MODE == kRowRes) return;

  // ---- forward x lines and two-for-one separation -------------------------------
  if (G.Yp != nrows)
    for (int x = threadIdx.x; x < X; x += kLineNT) lds[nrows * RS + x] = (T)0;
  lds_sync();
  fft_dir<T, kMaxB, -1, kPlanSlots, kLineNT, kLineGT, kLineBS>(lds, kModePlain, gx, gx, G, G.px, s_tw);
  lds_sync();
  const int np = G.Yp / 2;
  for (int i = threadIdx.x; i < np * Xh; i += kLineNT) {
    const int j = i / Xh, xp = i - j * Xh;
    const int x2 = xp == 0 ? 0 : X - xp;
    const T* r0 = lds + (2 * j) * RS;
    const T* r1 = r0 + RS;
    const cpx<T> z1 = {r0[xp], r1[xp]};
    const cpx<T> z2 = {r0[x2], r1[x2]};
    a.S[sbase + (int64_t)(2 * j) * Xh + xp] = {(T)0.5 * (z1.x + z2.x), (T)0.5 * (z1.y - z2.y)};
    if (2 * j + 1 < nrows)
      a.S[sbase + (int64_t)(2 * j + 1) * Xh + xp] = {(T)0.5 * (z1.y + z2.y),
                                                    (T)-0.5 * (z1.x - z2.x)};
  }
}

template <typename T, int MODE>
__global__ __launch_bounds__(kLineNT) void k_rows(RowArgs<T> a, RowGeom rg,
                                              const cpx<T>* __restrict__ tw) {
  extern __shared__ __align__(16) unsigned char smem_raw[];
  rows_body<T, MODE>(a, rg, tw, (int64_t)blockIdx.x, reinterpret_cast<T*>(smem_raw));
}

// One launch for both slice sets of an iteration: workgroups [0, nz) run the code
// slices (MZ = kRowIterZ or kRowFinalZ) with args a, the rest the data slices
// (kRowIterX) with args b -- the single-image data launch alone would leave the GPU
// nearly idle for its whole latency.
template <typename T, int MZ>
__global__ __launch_bounds__(kLineNT) void k_rows_pair(RowArgs<T> a, RowArgs<T> b, int64_t nz,
                                                   RowGeom rg, const cpx<T>* __restrict__ tw) {
  extern __shared__ __align__(16) unsigned char smem_raw[];
  T* lds = reinterpret_cast<T*>(smem_raw);
  const int64_t s = blockIdx.x;
  if (s < nz) rows_body<T, MZ>(a, rg, tw, s, lds);
  else rows_body<T, kRowIterX>(b, rg, tw, s - nz, lds);
}

// ---------------------------------------------------------------------------
// Column pass: TC consecutive x' columns of one line set, LDS [e][c] complex.
// ---------------------------------------------------------------------------
template <typename T, int SIGN>
__global__ __launch_bounds__(kLineNT) void k_cols(cpx<T>* __restrict__ S, cpx<T>* __restrict__ S2,
                                              int64_t n1, ColGeom cg,
                                              const cpx<T>* __restrict__ tw, int64_t ntot) {
  extern __shared__ __align__(16) unsigned char smem_raw[];
  T* lds = reinterpret_cast<T*>(smem_raw);
  // XCD-aware order, tiles of one line set consecutive: logical id L = (b mod 8) per + b / 8,
  // so the neighbouring column tiles of a line set -- which share the 128-B lines their
  // TC-column row segments cut -- run on one XCD at about the same time
  const int64_t per = gridDim.x >> 3;
  const int64_t L = (int64_t)(blockIdx.x & 7) * per + (blockIdx.x >> 3);
  if (L >= ntot) return;   // the whole workgroup
  int64_t o = L / cg.xtiles;
  const int tile = (int)(L - o * cg.xtiles);
  if (o >= n1) {   // workgroups past the first set's n1 line sets run the second set
    S = S2;
    o -= n1;
  }
  const int TC = cg.TC, n = cg.n;
  const int c0 = tile * TC;
  const int nc = min(TC, cg.Xh - c0);
  cpx<T>* base = S + (o % cg.ninner) * cg.sin + (o / cg.ninner) * cg.sout + c0;
  cpx<T>* s_tw = reinterpret_cast<cpx<T>*>(lds + (size_t)2 * n * TC);
  batched_loop<4, kLineNT>(cg.ntw, [&](int i) { return tw[i]; }, [&](int i, cpx<T> v) { s_tw[i] = v; });
  // the line set's columns, four loads in flight per thread before their LDS stores
  batched_loop<4, kLineNT>(
      n * TC,
      [&](int i) {
        const int e = i / TC, c = i - e * TC;
        return c < nc ? base[(int64_t)e * cg.es + c] : cpx<T>{(T)0, (T)0};
      },
      [&](int i, cpx<T> v) {
        lds[2 * i] = v.x;
        lds[2 * i + 1] = v.y;
      });
  const LineGeom g = {TC, 2, 2 * TC, 1};
  Grid2D Gd{};
  lds_sync();
  fft_dir<T, kMaxB, SIGN, kPlanSlots, kLineNT, kLineGT, kLineBS>(lds, kModePlain, g, g, Gd, cg.p, s_tw);
  lds_sync();
  for (int i = threadIdx.x; i < n * TC; i += kLineNT) {
    const int e = i / TC, c = i - e * TC;
    if (c < nc) base[(int64_t)e * cg.es + c] = {lds[2 * i], lds[2 * i + 1]};
  }
}

// ---------------------------------------------------------------------------
// Sherman-Morrison z-solve (SI:170-190; SP:158-191 with TG on channel 0).
//   b_k = conj(d_k) xi1 + rho xi2_k,  c = sum_k d_k b_k,
//   zhat_k = (b_k - conj(d_k) c / (rho + TG_k + s)) / (rho + TG_k)
// One thread per (image, bin); two sweeps over k (b_k is recomputed, not stored).
// ---------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void k_solve_sm(cpx<T>* __restrict__ Sz, cpx<T>* __restrict__ Sx,
                                                  const cpx<T>* __restrict__ dhat,
                                                  const T* __restrict__ s, T rho, T invP, int F,
                                                  int K, int tg, int X, int Y, int Xh) {
  const int f = blockIdx.x * 256 + threadIdx.x;
  if (f >= F) return;
  const int64_t img = blockIdx.y;
  cpx<T>* z = Sz + img * K * (int64_t)F + f;
  const cpx<T> x1 = Sx[img * F + f];
  cpx<T> c = {(T)0, (T)0};
  for (int k = 0; k < K; ++k) {
    const cpx<T> d = dhat[(int64_t)k * F + f];
    const cpx<T> x2 = z[(int64_t)k * F];
    const cpx<T> b = {cmulc(d, x1).x + rho * x2.x, cmulc(d, x1).y + rho * x2.y};
    c = cadd(c, cmul(d, b));
  }
  T tgv = (T)0;
  if (tg) {
    // 0.5 (|psf2otf([1,-1])|^2 + |psf2otf([1;-1])|^2) (SP:166-175)
    const int xp = f % Xh, y = f / Xh;
    const T two_pi = (T)6.283185307179586476925286766559;
    tgv = (T)0.5 * ((T)4 - (T)2 * cos(two_pi * (T)y / (T)Y) - (T)2 * cos(two_pi * (T)xp / (T)X));
  }
  const T sf = s[f];
  cpx<T> syn = {(T)0, (T)0};
  for (int k = 0; k < K; ++k) {
    const cpx<T> d = dhat[(int64_t)k * F + f];
    const cpx<T> x2 = z[(int64_t)k * F];
    const cpx<T> b = {cmulc(d, x1).x + rho * x2.x, cmulc(d, x1).y + rho * x2.y};
    const T den = rho + (k == 0 ? tgv : (T)0);
    const T q = (T)1 / (den + sf);
    const cpx<T> dc = cmulc(d, c);          // conj(d) c
    cpx<T> zk = {(b.x - dc.x * q) / den, (b.y - dc.y * q) / den};
    zk = cscale(zk, invP);
    z[(int64_t)k * F] = zk;
    syn = cadd(syn, cmul(d, zk));
  }
  Sx[img * F + f] = syn;
}

// ---------------------------------------------------------------------------
// setup kernels
// ---------------------------------------------------------------------------
template <typename T>
__global__ void k_embed_kernels(const T* __restrict__ k, T* __restrict__ dst, int kx, int ky,
                                int kt, int64_t total, int X, int Y, int Tn) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int64_t per = (int64_t)kx * ky * kt;
  const int64_t c = i / per;
  int64_t r = i - c * per;
  const int ix = (int)(r % kx);
  r /= kx;
  const int iy = (int)(r % ky);
  const int it = (int)(r / ky);
  const int x = ((ix - kx / 2) % X + X) % X;
  const int y = ((iy - ky / 2) % Y + Y) % Y;
  const int t = ((it - kt / 2) % Tn + Tn) % Tn;
  dst[((c * Tn + t) * Y + y) * (int64_t)X + x] = k[i];
}

__device__ __forceinline__ int sym_index(int i, int n) {
  // MATLAB padarray 'symmetric' (mirror including the edge sample), |pad| <= n
  if (i < 0) return -i - 1;
  if (i >= n) return 2 * n - i - 1;
  return i;
}

template <typename T>
__global__ void k_pad_inputs(const T* __restrict__ b, const T* __restrict__ mask,
                             const T* __restrict__ smooth, const T* __restrict__ xo, T* M, T* Mb,
                             T* SM, T* XO, int64_t total, int sbx, int sby, int sbt, int rx,
                             int ry, int rt, int X, int Y, int Tn) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int64_t P = (int64_t)X * Y * Tn;
  const int64_t c = i / P;
  int64_t r = i - c * P;
  const int x = (int)(r % X);
  r /= X;
  const int y = (int)(r % Y);
  const int t = (int)(r / Y);
  const int xi = x - rx, yi = y - ry, ti = t - rt;
  const int64_t cb = c * (int64_t)sbx * sby * sbt;
  const bool in = xi >= 0 && xi < sbx && yi >= 0 && yi < sby && ti >= 0 && ti < sbt;
  const int64_t o = in ? cb + ((int64_t)ti * sby + yi) * sbx + xi : 0;
  const T m = in ? mask[o] : (T)0;
  M[i] = m;
  Mb[i] = in ? m * b[o] : (T)0;
  if (XO) XO[i] = in ? xo[o] : (T)0;
  if (SM) {
    const int xs = sym_index(xi, sbx), ys = sym_index(yi, sby), ts = sym_index(ti, sbt);
    SM[i] = smooth[cb + ((int64_t)ts * sby + ys) * sbx + xs];
  }
}

template <typename T>
__global__ void k_spec_energy(const cpx<T>* __restrict__ d, T* out, int64_t F, int count, int diag,
                              T rho, T invP) {
  const int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= F) return;
  T s = 0;
  for (int c = 0; c < count; ++c) s += cabs2(d[(int64_t)c * F + f]);
  out[f] = diag ? invP / (rho + s) : s;
}

template <typename T>
__global__ void k_spec_mul(cpx<T>* a, const cpx<T>* __restrict__ m, int64_t F, int64_t total) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  a[i] = cmul(a[i], m[i % F]);
}

template <typename T>
__global__ __launch_bounds__(256) void k_reduce_parts(const T* __restrict__ part, T* out, int per,
                                                      int groups) {
  const int64_t img = blockIdx.x;
  const int64_t cnt = (int64_t)per * groups;
  __shared__ T sh[kRowParts][256];
  T acc[kRowParts] = {};
  for (int64_t i = threadIdx.x; i < cnt; i += 256)
    for (int j = 0; j < kRowParts; ++j) acc[j] += part[(img * cnt + i) * kRowParts + j];
  for (int j = 0; j < kRowParts; ++j) sh[j][threadIdx.x] = acc[j];
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w)
      for (int j = 0; j < kRowParts; ++j) sh[j][threadIdx.x] += sh[j][threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x < kRowParts) out[img * kRowParts + threadIdx.x] = sh[threadIdx.x][0];
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
size_t rows_smem_bytes(const RowGeom& rg, size_t tsize) {
  return (rows_tw_off(rg) + 2 * (size_t)rg.ntw) * tsize;
}
size_t cols_smem_bytes(const ColGeom& cg, size_t tsize) {
  return ((size_t)cg.n * cg.TC * 2 + 2 * (size_t)cg.ntw) * tsize;
}

template <typename T>
hipError_t launch_rows(int mode, const RowArgs<T>& a, int64_t nslices, const RowGeom& rg,
                       const cpx<T>* tw, hipStream_t st) {
  if (nslices <= 0) return hipSuccess;
  const dim3 grid((unsigned)nslices, (unsigned)rg.groups);
  const size_t sm = rows_smem_bytes(rg, sizeof(T));
  switch (mode) {
    case kRowFwd: hipLaunchKernelGGL((k_rows<T, kRowFwd>), grid, dim3(kLineNT), sm, st, a, rg, tw); break;
    case kRowIterZ: hipLaunchKernelGGL((k_rows<T, kRowIterZ>), grid, dim3(kLineNT), sm, st, a, rg, tw); break;
    case kRowIterX: hipLaunchKernelGGL((k_rows<T, kRowIterX>), grid, dim3(kLineNT), sm, st, a, rg, tw); break;
    case kRowFinalZ: hipLaunchKernelGGL((k_rows<T, kRowFinalZ>), grid, dim3(kLineNT), sm, st, a, rg, tw); break;
    case kRowRes: hipLaunchKernelGGL((k_rows<T, kRowRes>), grid, dim3(kLineNT), sm, st, a, rg, tw); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

template <typename T>
hipError_t launch_cols(cpx<T>* S, int sign, int64_t nouter, const ColGeom& cg, const cpx<T>* tw,
                       hipStream_t st, cpx<T>* S2, int64_t nouter2) {
  if (nouter + nouter2 <= 0) return hipSuccess;
  const int64_t ntot = (nouter + nouter2) * (int64_t)cg.xtiles;
  if (ntot >= ((int64_t)1 << 31)) return hipErrorInvalidValue;
  const dim3 grid((unsigned)(((ntot + 7) / 8) * 8));
  const size_t sm = cols_smem_bytes(cg, sizeof(T));
  if (sign < 0)
    hipLaunchKernelGGL((k_cols<T, -1>), grid, dim3(kLineNT), sm, st, S, S2, nouter, cg, tw, ntot);
  else
    hipLaunchKernelGGL((k_cols<T, +1>), grid, dim3(kLineNT), sm, st, S, S2, nouter, cg, tw, ntot);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_rows_pair(int code_mode, const RowArgs<T>& a, int64_t nz, const RowArgs<T>& b,
                            int64_t nx, const RowGeom& rg, const cpx<T>* tw, hipStream_t st) {
  if (nz + nx <= 0) return hipSuccess;
  const dim3 grid((unsigned)(nz + nx), (unsigned)rg.groups);
  const size_t sm = rows_smem_bytes(rg, sizeof(T));
  if (code_mode == kRowIterZ)
    hipLaunchKernelGGL((k_rows_pair<T, kRowIterZ>), grid, dim3(kLineNT), sm, st, a, b, nz, rg, tw);
  else if (code_mode == kRowFinalZ)
    hipLaunchKernelGGL((k_rows_pair<T, kRowFinalZ>), grid, dim3(kLineNT), sm, st, a, b, nz, rg, tw);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

template <typename T>
hipError_t launch_solve_sm(cpx<T>* Sz, cpx<T>* Sx, const cpx<T>* dhat, const T* s, T rho, T invP,
                           int F, int K, int64_t n, int tg, int X, int Y, int Xh,
                           hipStream_t st) {
  if (n <= 0 || n > 65535) return hipErrorInvalidValue;
  const dim3 grid((unsigned)((F + 255) / 256), (unsigned)n);
  hipLaunchKernelGGL((k_solve_sm<T>), grid, dim3(256), 0, st, Sz, Sx, dhat, s, rho, invP, F, K, tg,
                     X, Y, Xh);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_embed_kernels(const T* k, T* dst, int kx, int ky, int kt, int count, int X, int Y,
                                int Tn, hipStream_t st) {
  const int64_t total = (int64_t)kx * ky * kt * count;
  if (total <= 0) return hipSuccess;
  hipLaunchKernelGGL((k_embed_kernels<T>), dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st,
                     k, dst, kx, ky, kt, total, X, Y, Tn);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_pad_inputs(const T* b, const T* mask, const T* smooth, const T* xo, T* M, T* Mb,
                             T* SM, T* XO, int64_t count, int sbx, int sby, int sbt, int rx,
                             int ry, int rt, int X, int Y, int Tn, hipStream_t st) {
  const int64_t total = count * (int64_t)X * Y * Tn;
  if (total <= 0) return hipSuccess;
  hipLaunchKernelGGL((k_pad_inputs<T>), dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, b,
                     mask, smooth, xo, M, Mb, SM, XO, total, sbx, sby, sbt, rx, ry, rt, X, Y, Tn);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_spec_energy(const cpx<T>* dhat, T* out, int64_t F, int count, int diag, T rho,
                              T invP, hipStream_t st) {
  hipLaunchKernelGGL((k_spec_energy<T>), dim3((unsigned)((F + 255) / 256)), dim3(256), 0, st, dhat,
                     out, F, count, diag, rho, invP);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_spec_mul(cpx<T>* a, const cpx<T>* m, int64_t F, int count, hipStream_t st) {
  const int64_t total = F * count;
  if (total <= 0) return hipSuccess;
  hipLaunchKernelGGL((k_spec_mul<T>), dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, a, m,
                     F, total);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_reduce_parts(const T* part, T* out, int64_t n, int per_img, int groups,
                               hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL((k_reduce_parts<T>), dim3((unsigned)n), dim3(256), 0, st, part, out, per_img,
                     groups);
  return hipGetLastError();
}

template hipError_t launch_rows<double>(int, const RowArgs<double>&, int64_t, const RowGeom&,
                                        const cpx<double>*, hipStream_t);
template hipError_t launch_cols<double>(cpx<double>*, int, int64_t, const ColGeom&,
                                        const cpx<double>*, hipStream_t, cpx<double>*, int64_t);
template hipError_t launch_rows_pair<double>(int, const RowArgs<double>&, int64_t,
                                             const RowArgs<double>&, int64_t, const RowGeom&,
                                             const cpx<double>*, hipStream_t);
template hipError_t launch_solve_sm<double>(cpx<double>*, cpx<double>*, const cpx<double>*,
                                            const double*, double, double, int, int, int64_t, int,
                                            int, int, int, hipStream_t);
template hipError_t launch_embed_kernels<double>(const double*, double*, int, int, int, int, int,
                                                 int, int, hipStream_t);
template hipError_t launch_pad_inputs<double>(const double*, const double*, const double*,
                                              const double*, double*, double*, double*, double*,
                                              int64_t, int, int, int, int, int, int, int, int, int,
                                              hipStream_t);
template hipError_t launch_spec_energy<double>(const cpx<double>*, double*, int64_t, int, int,
                                               double, double, hipStream_t);
template hipError_t launch_spec_mul<double>(cpx<double>*, const cpx<double>*, int64_t, int,
                                            hipStream_t);
template hipError_t launch_reduce_parts<double>(const double*, double*, int64_t, int, int,
                                                hipStream_t);

}  // namespace ccsc
