// 3D learner kernels (3D/admm_learn_conv3D_large.m, "L3").
//
// A 3D slice (e.g. 74 x 74 x 42 fp64 = 1.8 MB for the C4 config) does not fit
// one CU's LDS, so the reference's per-slice fftn/ifftn (L3:25,44,53,123,127,
// 172,178) is factored:  R2C = [plane R2C over (x, y) for every t] then
// [complex FFT along t]; C2R is the mirror image.  The plane kernels reuse the
// LDS-resident 2D machinery and fuse the elementwise stages (prox + dual,
// D-step dual, support gather, padding); the t kernel holds one y-row of
// lines (T x Xh complex) in LDS.  Spectra are stored [slice][t][y][x'] with
// plane bins dense (F2 = Xh * Y), F3 = F2 * T -- except between the z-step's plane
// transforms and its fused t-solve (k_tsolve3), which exchange them "t-minor":
// [slice][y][x' / TC][t][TC] (F3t = Y * ntile * T * TC, ntile = ceil(Xh / TC)), so the
// t-solve reads and writes T * TC contiguous values per filter instead of TC-complex
// segments at the plane stride, and the filter spectrum, B^ and sden it reads are
// kept in the same order (k_to_ttiles).
// the plane kernels' dense-lane 37-point pass (slice.hpp PK) with two output pairs per task:
// 9 main waves + 3-4, 0-4 spilled VGPRs instead of 16-36 at three; C4 0.1845 -> 0.1823 s per
// outer iteration, same box (profiles/r05/pfa_pack_q2_ab.txt)
#include "slice.hpp"

namespace ccsc {

constexpr int kPlaneQP = 2;   // conjugate output pairs per 37-point task of the plane kernels

// ---- plane forward: prologue -> 2D R2C -> dst[(slice*T + t)*F2 + f] --------
// mode 0: embed src sub-volume [st][sy][sx] at offset (o, o, o) (zero padding)
// mode 2: D-step dual y += D - u, c = u - y (L3:121-123), u from the (2r+1)^3 support
// mode 3: z-step on the state a = z + y in b (read only): u = a - clamp(a), y' = clamp(a),
//         c = u - y' = a - 2 clamp(a); k_plane_inv mode 3 forms a' = z' + clamp(a)
// index of bin (t, y, x') of a slice in the t-minor tile order
__device__ __forceinline__ int64_t ttile_idx(int t, int f2, int Tn, int Xh, int tc, int ntile) {
  const int y = f2 / Xh, x = f2 - y * Xh;
  const int tile = x / tc, c = x - tile * tc;
  return ((int64_t)(y * ntile + tile) * Tn + t) * tc + c;
}

// XCD-aware plane order: logical plane L = (b mod 8) per + b / 8 (per = gridDim / 8), so the
// workgroups of one XCD take consecutive planes (t) of a slice -- the t-minor spectra of
// neighbouring planes share 128-B lines (k_tsolve3's order), which one L2 then fetches and
// writes whole instead of every XCD a 32-B piece of each
__device__ __forceinline__ int64_t plane_of_block(int64_t nplanes) {
  const int64_t per = gridDim.x >> 3;
  const int64_t L = (int64_t)(blockIdx.x & 7) * per + (blockIdx.x >> 3);
  return L < nplanes ? L : -1;
}
__host__ inline unsigned plane_grid(int64_t nplanes) { return (unsigned)(((nplanes + 7) / 8) * 8); }


template <typename T, int RM>
__global__ __launch_bounds__(kNT) __attribute__((amdgpu_waves_per_eu(slice_waves<RM>())))
void k_plane_fwd(int mode, const T* __restrict__ a,
                                                   T* __restrict__ b, const T* __restrict__ usup,
                                                   int sx, int sy, int st, int o, T theta,
                                                   int KG, int r, cpx<T>* __restrict__ dst,
                                                   int Tn, const cpx<T>* __restrict__ twg,
                                                   Grid2D G, int tc, int64_t nplanes) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int64_t pl = plane_of_block(nplanes);
  if (pl < 0) return;   // the whole workgroup
  Smem<T> S = carve<T>(smem, G);
  using Q = SG<RM>;
  const int GX = Q::X(G), GY = Q::Y(G), RS = Q::RS(G), GF = Q::F(G), GXh = Q::Xh(G);
  if constexpr (!Q::fixed) load_twiddles(S.tw, twg, G.ntw);
  const int64_t slice = pl / Tn;
  const int t = (int)(pl - slice * Tn);
  const int P = GX * GY;
  const int s = 2 * r + 1;
  if (mode == 0) {
    for (int e = threadIdx.x; e < Q::Yp(G) * RS; e += kNT) S.slice[e] = (T)0;
    lds_sync();
    const int tt = t - o;
    if (tt >= 0 && tt < st) {
      const T* in = a + ((int64_t)slice * st + tt) * sx * sy;
      for (int e = threadIdx.x; e < sx * sy; e += kNT) {
        const int y = e / sx, x = e - y * sx;
        S.slice[Q::px(x + o, y + o, G)] = in[e];
      }
    }
  } else {
    const int64_t off = (slice * Tn + t) * P;
    const int st3 = (t + r) % Tn;
    const T* u = usup + (int64_t)(slice % KG) * s * s * s;
    if (mode == 3) {   // the z-step (L3:168-172) on the state a = z + y
      batched_loop<3>(
          P, [&](int e) { return b[off + e]; },
          [&](int e, T q) {
            const int y = e / GX, x = e - y * GX;
            S.slice[Q::px(x, y, G)] = fma((T)-2, fmax(-theta, fmin(q, theta)), q);
          });
    } else {
      batched_loop<3>(
          P, [&](int e) { return Pair2<T>{b[off + e], a[off + e]}; },
          [&](int e, Pair2<T> ba) {
            const int y = e / GX, x = e - y * GX;
            const int sxx = (x + r) % GX, syy = (y + r) % GY;
            const T uv = (sxx < s && syy < s && st3 < s) ? u[(st3 * s + syy) * s + sxx] : (T)0;
            const T yn = ba.a + ba.b - uv;
            b[off + e] = yn;
            S.slice[Q::px(x, y, G)] = uv - yn;
          });
    }
    zero_pad_row(S.slice, G);
  }
  slice_r2c_rm<T, RM, true, kPlaneQP>(S.slice, G, S.tw);
  if (tc > 0) {   // t-minor tiles (k_tsolve3's order)
    const int ntile = (GXh + tc - 1) / tc;
    cpx<T>* out = dst + slice * ((int64_t)GY * ntile * Tn * tc);
    for (int f = threadIdx.x; f < GF; f += kNT)
      out[ttile_idx(t, f, Tn, GXh, tc, ntile)] = lds_cpx(S.slice + Q::bin(f, G), 1);
    return;
  }
  cpx<T>* out = dst + (slice * Tn + t) * GF;
  for (int f = threadIdx.x; f < GF; f += kNT) out[f] = lds_cpx(S.slice + Q::bin(f, G), 1);
}

// ---- compile-time t transforms of C4 (T = 42 = 7 * 3 * 2 radix passes) ----------------
// The t lines of an LDS tile are interleaved complex columns (line stride 2, element stride
// RS = 2 NL): fft_fixed.hpp's y-direction pass with this geometry, index math and strides
// compile-time (the runtime fft_dir's arithmetic, bit for bit).  tline42_ok() checks the
// runtime plan (radix order, twiddle offsets) the fixed passes assume.
template <int NL>
struct TLines42 {
  static constexpr int X = 1, Y = 42, Yp = 42, Xh = NL, RS = 2 * NL;
};
__host__ inline bool tline42_ok(const Grid2D& Gt, int nl) {
  const Plan1D& p = Gt.py;
  return Gt.Y == 42 && Gt.Xh == nl && Gt.RS == 2 * nl && p.n == 42 && p.npass == 3 &&
         p.rad[0] == 7 && p.rad[1] == 3 && p.rad[2] == 2 && p.twoff[0] == 0 && p.twoff[1] == 6 &&
         p.twoff[2] == 20;
}
template <typename T, int NL, int SIGN, int NT = kNT>
__device__ __forceinline__ void tfft42(T* lds, const cpx<T>* tw) {
  using FG = TLines42<NL>;
  const int tid = threadIdx.x;
  fpass<T, FG, NT, false, 7, 1, SIGN, kModePlain>(lds, tw, tid);
  fpass<T, FG, NT, false, 3, 7, SIGN, kModePlain>(lds, tw + 6, tid);
  fpass<T, FG, NT, false, 2, 21, SIGN, kModePlain>(lds, tw + 20, tid);
}

// ---- t-direction complex FFT (src may equal dst); one workgroup per (slice, y)
// Gt describes the T x Xh tile: Gt.Y = T (plan Gt.py), Gt.Xh = lines, Gt.RS = row stride.
template <typename T, int SIGN, int RM, int FNL = 0>
__global__ __launch_bounds__(kNT) __attribute__((amdgpu_waves_per_eu(slice_waves<RM>())))
void k_tfft(const cpx<T>* src, cpx<T>* dst, int Yn, int F2,
                                              const cpx<T>* __restrict__ twg, Grid2D Gt) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  cpx<T>* s_tw = reinterpret_cast<cpx<T>*>(smem);
  T* lds = reinterpret_cast<T*>(s_tw + Gt.ntw);
  for (int i = threadIdx.x; i < Gt.ntw; i += kNT) s_tw[i] = twg[i];
  const int64_t slice = blockIdx.x / Yn;
  const int y = blockIdx.x - (int)(slice * Yn);
  const int Tn = Gt.Y, Xh = Gt.Xh;
  const int64_t base = slice * (int64_t)Tn * F2 + (int64_t)y * Xh;
  for (int e = threadIdx.x; e < Tn * Xh; e += kNT) {
    const int t = e / Xh, x = e - t * Xh;
    lds_cpx_store(lds + t * Gt.RS + 2 * x, 1, src[base + (int64_t)t * F2 + x]);
  }
  lds_sync();
  const LineGeom g = {Xh, 2, Gt.RS, 1};
  if constexpr (FNL > 0) tfft42<T, FNL, SIGN>(lds, s_tw);   // C4's 42 x 38 tiles
  else fft_dir<T, kMaxB, SIGN, kMaxPass, kNT, 1, 1, RM>(lds, kModePlain, g, g, Gt, Gt.py, s_tw);
  for (int e = threadIdx.x; e < Tn * Xh; e += kNT) {
    const int t = e / Xh, x = e - t * Xh;
    dst[base + (int64_t)t * F2 + x] = lds_cpx(lds + t * Gt.RS + 2 * x, 1);
  }
}

// ---- plane inverse: src plane spectrum -> 2D C2R -> epilogue ----------------
// mode 0: dst = plane * scale
// mode 2: D-step: D = plane * scale; support gather of D + y (L3:239-240), d-norms
// mode 3: z-step on the state a (k_plane_fwd mode 3): a' = z' + clamp(a) into `state`,
//         z' into dst only when wz (the iterations whose z is read), tol norms vs old z;
//         with nxt, also the next z-iteration's k_plane_fwd (c' = a' - 2 clamp(a'), plane
//         R2C) into nxt -- the plane's own bins of src, overwritten in place -- so the
//         state is not read back by a separate forward launch
template <typename T, int RM>
__global__ __launch_bounds__(kNT) __attribute__((amdgpu_waves_per_eu(slice_waves<RM>())))
void k_plane_inv(int mode, const cpx<T>* src,
                                                   T* __restrict__ dst, const T* __restrict__ yv,
                                                   T* __restrict__ supp, T* __restrict__ norms,
                                                   int64_t nfirst, T scale, int r, int Tn,
                                                   const cpx<T>* __restrict__ twg, Grid2D G,
                                                   int tc, T* __restrict__ state, T theta, int wz,
                                                   cpx<T>* nxt, int64_t nplanes) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int64_t pl = plane_of_block(nplanes);
  if (pl < 0) return;   // the whole workgroup
  Smem<T> S = carve<T>(smem, G);
  using Q = SG<RM>;
  const int GX = Q::X(G), GY = Q::Y(G), GF = Q::F(G), GXh = Q::Xh(G);
  if constexpr (!Q::fixed) load_twiddles(S.tw, twg, G.ntw);
  const int64_t slice = pl / Tn;
  const int t = (int)(pl - slice * Tn);
  if (tc > 0) {   // t-minor tiles (k_tsolve3's order)
    const int ntile = (GXh + tc - 1) / tc;
    const cpx<T>* in = src + slice * ((int64_t)GY * ntile * Tn * tc);
    batched_loop<3>(
        GF, [&](int f) { return in[ttile_idx(t, f, Tn, GXh, tc, ntile)]; },
        [&](int f, cpx<T> v) { lds_cpx_store(S.slice + Q::bin(f, G), 1, v); });
  } else {
    const cpx<T>* in = src + (slice * Tn + t) * GF;
    batched_loop<3>(
        GF, [&](int f) { return in[f]; },
        [&](int f, cpx<T> v) { lds_cpx_store(S.slice + Q::bin(f, G), 1, v); });
  }
  slice_c2r_rm<T, RM, true, kPlaneQP>(S.slice, G, S.tw);
  const int P = GX * GY;
  const int64_t off = (slice * Tn + t) * P;
  const bool nrm = (mode == 3 && norms) || (mode == 2 && slice < nfirst);
  T acc_d = 0, acc_n = 0;
  // the old z / D (norms) and the state of a batch are loaded before any is used
  batched_loop<3>(
      P,
      [&](int e) {
        return Pair2<T>{nrm ? dst[off + e] : (T)0, mode == 3 ? state[off + e] : (T)0};
      },
      [&](int e, Pair2<T> oq) {
        const int y = e / GX, x = e - y * GX;
        const T v = S.slice[Q::px(x, y, G)] * scale;
        if (nrm) {
          acc_d += (v - oq.a) * (v - oq.a);
          acc_n += v * v;
        }
        if (mode == 3) {
          const T an = v + fmax(-theta, fmin(oq.b, theta));
          state[off + e] = an;
          if (wz) dst[off + e] = v;
          if (nxt) S.slice[Q::px(x, y, G)] = fma((T)-2, fmax(-theta, fmin(an, theta)), an);
        } else {
          dst[off + e] = v;
        }
      });
  if (mode == 2) {
    const int s = 2 * r + 1;
    const int st3 = (t + r) % Tn;          // support plane index (L3:239-240 circshift)
    if (st3 < s) {
      T* sp = supp + (slice * s + st3) * s * s;
      for (int q = threadIdx.x; q < s * s; q += kNT) {
        const int sy = q / s, sx = q - sy * s;
        const int x = (sx - r + GX) % GX, y = (sy - r + GY) % GY;
        sp[q] = S.slice[Q::px(x, y, G)] * scale + yv[off + y * GX + x];
      }
    }
  }
  if (nrm) {
    acc_d = block_sum(acc_d, S.red);
    acc_n = block_sum(acc_n, S.red);
    if (threadIdx.x == 0) {
      norms[2 * (slice * Tn + t)] = acc_d;
      norms[2 * (slice * Tn + t) + 1] = acc_n;
    }
  }
  if (mode == 3 && nxt) {   // the next iteration's forward plane transform (k_plane_fwd mode 3)
    zero_pad_row(S.slice, G);
    slice_r2c_rm<T, RM, true, kPlaneQP>(S.slice, G, S.tw);
    if (tc > 0) {
      const int ntile = (GXh + tc - 1) / tc;
      cpx<T>* out = nxt + slice * ((int64_t)GY * ntile * Tn * tc);
      for (int f = threadIdx.x; f < GF; f += kNT)
        out[ttile_idx(t, f, Tn, GXh, tc, ntile)] = lds_cpx(S.slice + Q::bin(f, G), 1);
    } else {
      cpx<T>* out = nxt + (slice * Tn + t) * GF;
      for (int f = threadIdx.x; f < GF; f += kNT) out[f] = lds_cpx(S.slice + Q::bin(f, G), 1);
    }
  }
}

// ---- z-solve per (patch, bin) (L3:314-339, closed form as in 2D) -------------
//   w = (B - sum_k d_k C_k) * sden,  Zhat_k = C_k * (1/P3) + conj(d_k) w  (in place)
// sden = 1 / ((rho + s) P3) carries the inverse-FFT scale of both terms.
template <typename T>
__global__ void k_zsolve3(cpx<T>* __restrict__ C, const cpx<T>* __restrict__ Bhat,
                          const cpx<T>* __restrict__ dhat, const T* __restrict__ sden,
                          int64_t F3, int K, T invP3) {
  const int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t p = blockIdx.y;
  if (f >= F3) return;
  cpx<T>* Cp = C + p * K * F3 + f;
  cpx<T> acc = {(T)0, (T)0};
  for (int k = 0; k < K; ++k) acc = cmac(acc, dhat[(int64_t)k * F3 + f], Cp[(int64_t)k * F3]);
  const cpx<T> w = cscale(csub(Bhat[p * F3 + f], acc), sden[f]);
  for (int k = 0; k < K; ++k) {
    const cpx<T> c = Cp[(int64_t)k * F3];
    const cpx<T> d = dhat[(int64_t)k * F3 + f];
    Cp[(int64_t)k * F3] = cmacc(cscale(c, invP3), d, w);
  }
}

// ---- fused t-FFT + z-solve + inverse t-FFT (replaces k_tfft(-1), k_zsolve3,
// k_tfft(+1) of the 3D z-step): one workgroup per (y row, tile of TC x' columns,
// group of ppw patches) holds, per patch in turn, the K filters' T x TC plane-spectrum
// columns in LDS, layout [t][k*TC + c] (K*TC complex lines of length T), so the spectra
// cross HBM once each way per z-iteration instead of three times (L3:172-178, the
// closed form of k_zsolve3).  C, B^, dhat and sden are in the t-minor tile order (F3t
// per slice): a (slice, y, tile) block is T * TC contiguous complex.  The patch loop
// keeps the block's K filter-spectrum columns hot in L2 across the ppw patches (one
// HBM read of dhat per workgroup instead of per patch) and prefetches the next patch's
// block into registers (LD complex per thread) while the current one is transformed
// (82 KB of LDS at TC = 2: one workgroup per CU, nothing else hides the HBM reads).
// Gt2: the t plan for K*TC lines.
// DL: the block's K filter-spectrum columns (and sden) are staged in LDS once per
// workgroup -- the solve of every patch reads them there instead of from L2 (two exposed
// global round trips per patch otherwise) -- and each patch's B^ values are loaded before
// its forward t-FFT, consumed after it.
// FNL > 0: the t transforms on the compile-time 42-point plan over FNL = K TC lines (C4),
// TC = TCF; NT threads per workgroup (NT, or 512 for C4's TC = 1 form: two workgroups per CU)
template <typename T, int RM, int LD, int KMAX, bool DL, int FNL, int NT = kNT, int TCF = 2>
__global__ __launch_bounds__(NT) void k_tsolve3(cpx<T>* __restrict__ C,
                                                 const cpx<T>* __restrict__ Bhat,
                                                 const cpx<T>* __restrict__ dhat,
                                                 const T* __restrict__ sden, int K, int Yn,
                                                 int Xh, int TC, int xtiles, T invP3,
                                                 const cpx<T>* __restrict__ twg, Grid2D Gt,
                                                 int64_t npatch, int ppw) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  cpx<T>* s_tw = reinterpret_cast<cpx<T>*>(smem);
  T* lds = reinterpret_cast<T*>(s_tw + Gt.ntw);
  for (int i = threadIdx.x; i < Gt.ntw; i += NT) s_tw[i] = twg[i];
  if constexpr (FNL > 0) {   // C4: TC = TCF, T = 42, K = FNL / TCF -- the index math compile-time
    TC = TCF;
    K = FNL / TCF;
  }
  const int tile = blockIdx.x % xtiles;
  const int64_t rest = blockIdx.x / xtiles;
  const int y = (int)(rest % Yn);
  const int64_t p0 = (rest / Yn) * ppw;
  const int64_t p1 = min(npatch, p0 + ppw);
  const int Tn = FNL > 0 ? 42 : Gt.Y;
  const int nc = min(TC, Xh - tile * TC);
  const int NL = K * TC;
  const int TT = Tn * TC;                                   // one (slice, y, tile) block
  const int KT = K * TT;
  const int64_t F3t = (int64_t)Yn * xtiles * TT;
  const int64_t blk = (int64_t)(y * xtiles + tile) * TT;
  const LineGeom g = {NL, 2, 2 * NL, 1};
  // load slot j of this thread: i = threadIdx.x + j * NT < K * TT -> global offset
  // (K F3t < 2^31: checked by the host) and LDS offset; recomputed where used from a
  // laundered thread index, so the patch loop does not keep them (and every FFT pass's
  // per-thread index math) live in registers across its iterations
  auto slot = [&](int tid, int j, int& src, int& dst) {
    const int i = tid + j * NT;
    const int k = i / TT, rem = i - k * TT;
    const int t = rem / TC, c = rem - t * TC;
    src = (i < KT && c < nc) ? k * (int)F3t + rem : -1;
    dst = i < KT ? 2 * (t * NL + k * TC + c) : -1;
  };
  cpx<T> pre[LD];
  // solve-phase geometry: G = NT / (T TC) threads per bin split the k range
  const int nb = TT;
  const int G = max(1, NT / nb);
  const int kg = (K + G - 1) / G;
  cpx<T>* part = reinterpret_cast<cpx<T>*>(lds + 2 * (size_t)Tn * NL);   // [G][nb]
  cpx<T>* sD = part + (size_t)G * nb;                                    // DL: [K][nb]
  T* sS = reinterpret_cast<T*>(sD + (size_t)K * nb);                     // DL: [nb]
  if constexpr (DL) {   // visible after the patch loop's first barrier
    for (int i = threadIdx.x; i < K * nb; i += NT) {
      const int k = i / nb, bb = i - k * nb;
      sD[i] = dhat[(int64_t)k * F3t + blk + bb];
    }
    for (int i = threadIdx.x; i < nb; i += NT) sS[i] = sden[blk + i];
  }
  {
    const cpx<T>* Cp = C + p0 * K * F3t + blk;
#pragma unroll
    for (int j = 0; j < LD; ++j) {
      int src, dst;
      slot((int)threadIdx.x, j, src, dst);
      pre[j] = src >= 0 ? Cp[src] : cpx<T>{(T)0, (T)0};
    }
  }
  for (int64_t p = p0; p < p1; ++p) {
    int tid = (int)threadIdx.x;
    asm volatile("" : "+v"(tid));
    cpx<T>* Cp = C + p * K * F3t + blk;
#pragma unroll
    for (int j = 0; j < LD; ++j) {
      int src, dst;
      slot(tid, j, src, dst);
      if (dst >= 0) lds_cpx_store(lds + dst, 1, pre[j]);
    }
    lds_sync();
    if (p + 1 < p1) {   // the next patch's block, in flight across this one's transforms
      const cpx<T>* Cn = Cp + K * F3t;
#pragma unroll
      for (int j = 0; j < LD; ++j) {
        int src, dst;
        slot(tid, j, src, dst);
        pre[j] = src >= 0 ? Cn[src] : cpx<T>{(T)0, (T)0};
      }
    }
    cpx<T> bh = {(T)0, (T)0};
    if constexpr (DL) {   // this patch's B^ in flight under the forward t-FFT
      const int b = tid % nb, grp = tid / nb;
      if (grp < G && b - (b / TC) * TC < nc) bh = Bhat[p * F3t + blk + b];
    }
    if constexpr (FNL > 0) tfft42<T, FNL, -1, NT>(lds, s_tw);
    else fft_dir<T, kMaxB, -1, kMaxPass, NT, 1, 1, RM>(lds, kModePlain, g, g, Gt, Gt.py, s_tw);
    // per bin (t, c): w = (B - sum_k d_k C_k) sden, C_k <- C_k / P3 + conj(d_k) w; the
    // d_k of a thread's k range stay in registers between the two sweeps, partial sums
    // meet in LDS past the spectra
    tid = (int)threadIdx.x;
    asm volatile("" : "+v"(tid));
    const int b = tid % nb, grp = tid / nb;
    const int t = b / TC, c = b - t * TC;
    const bool on = grp < G && c < nc;
    const int64_t f3 = blk + b;                               // t * TC + c inside the block
    T* row = lds + 2 * (t * NL + c);
    cpx<T> dv[KMAX];
    cpx<T> acc = {(T)0, (T)0};
#pragma unroll
    for (int j = 0; j < KMAX; ++j) {
      const int k = grp * kg + j;
      const bool ok = on && j < kg && k < K;
      if constexpr (DL) dv[j] = ldc_if(ok, sD + k * nb + b);
      else dv[j] = ok ? dhat[(int64_t)k * F3t + f3] : cpx<T>{(T)0, (T)0};
    }
#pragma unroll
    for (int j = 0; j < KMAX; ++j) {
      const int k = grp * kg + j;
      if (on && j < kg && k < K) acc = cmac(acc, dv[j], lds_cpx(row + 2 * k * TC, 1));
    }
    if (grp < G) part[grp * nb + b] = acc;
    lds_sync();
    if (on) {
      cpx<T> tot = {(T)0, (T)0};
      for (int q = 0; q < G; ++q) tot = cadd(tot, part[q * nb + b]);
      cpx<T> w;
      if constexpr (DL) {
        w = cscale(csub(bh, tot), sS[b]);
      } else {
        w = cscale(csub(Bhat[p * F3t + f3], tot), sden[f3]);
      }
#pragma unroll
      for (int j = 0; j < KMAX; ++j) {
        const int k = grp * kg + j;
        if (j < kg && k < K) {
          const cpx<T> cv = lds_cpx(row + 2 * k * TC, 1);
          lds_cpx_store(row + 2 * k * TC, 1, cmacc(cscale(cv, invP3), dv[j], w));
        }
      }
    }
    lds_sync();
    if constexpr (FNL > 0) tfft42<T, FNL, +1, NT>(lds, s_tw);
    else fft_dir<T, kMaxB, +1, kMaxPass, NT, 1, 1, RM>(lds, kModePlain, g, g, Gt, Gt.py, s_tw);
    tid = (int)threadIdx.x;
    asm volatile("" : "+v"(tid));
#pragma unroll
    for (int j = 0; j < LD; ++j) {
      int src, dst;
      slot(tid, j, src, dst);
      if (src >= 0) Cp[src] = lds_cpx(lds + dst, 1);
    }
    lds_sync();   // (the next patch's block overwrites the LDS)
  }
}

// dst[s][t-minor tile order] = src[s][t][y][x'] (count spectra of F3 = T Y Xh bins; the
// padding columns x' >= Xh of the last tile are zero)
template <typename T, typename V>
__global__ void k_to_ttiles(const V* __restrict__ src, V* __restrict__ dst, int Tn, int Yn,
                            int Xh, int tc, int64_t count) {
  const int ntile = (Xh + tc - 1) / tc;
  const int64_t F3t = (int64_t)Yn * ntile * Tn * tc;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count * F3t) return;
  const int64_t s = i / F3t;
  int64_t r = i - s * F3t;
  const int c = (int)(r % tc);
  r /= tc;
  const int t = (int)(r % Tn);
  r /= Tn;
  const int tile = (int)(r % ntile);
  const int y = (int)(r / ntile);
  const int x = tile * tc + c;
  V v{};
  if (x < Xh) v = src[(s * Tn + t) * ((int64_t)Yn * Xh) + (int64_t)y * Xh + x];
  dst[i] = v;
}

// ---- objective helper: acc[p][f] = sum_k Zhat[p][k][f] d[k][f] --------------
template <typename T>
__global__ void k_corr_sum(const cpx<T>* __restrict__ Zh, const cpx<T>* __restrict__ dhat,
                           cpx<T>* __restrict__ out, int64_t F3, int K) {
  const int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= F3) return;
  cpx<T> acc = {(T)0, (T)0};
  for (int k = 0; k < K; ++k) acc = cmac(acc, Zh[(int64_t)k * F3 + f], dhat[(int64_t)k * F3 + f]);
  out[f] = acc;
}

// crop-diff squared sum and l1 of one patch: part[0] += ||crop(Dz) - b||^2 (over a
// [X,Y,T] volume, crop r in x and y, rt in t: 0 for a 2D slice), part[1] += sum |z| over the K slices
template <typename T>
__global__ void k_crop_sq(const T* __restrict__ Dz, const T* __restrict__ b, int sx, int sy,
                          int st, int r, int rt, int X, int Y, const T* __restrict__ z, int64_t zcount,
                          T* __restrict__ part) {
  __shared__ T red[2][4];
  T sq = 0, l1 = 0;
  const int64_t nb = (int64_t)sx * sy * st;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < nb; e += (int64_t)gridDim.x * 256) {
    const int x = (int)(e % sx), y = (int)((e / sx) % sy), t = (int)(e / ((int64_t)sx * sy));
    const T d = Dz[((int64_t)(t + rt) * Y + (y + r)) * X + (x + r)] - b[e];
    sq += d * d;
  }
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < zcount; e += (int64_t)gridDim.x * 256)
    l1 += fabs(z[e]);
  sq = wave_sum(sq);
  l1 = wave_sum(l1);
  if ((threadIdx.x & 63) == 0) {
    red[0][threadIdx.x >> 6] = sq;
    red[1][threadIdx.x >> 6] = l1;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    atomicAdd(&part[0], red[0][0] + red[0][1] + red[0][2] + red[0][3]);
    atomicAdd(&part[1], red[1][0] + red[1][1] + red[1][2] + red[1][3]);
  }
}

// ---------------------------------------------------------------------------
size_t tfft_smem_bytes(const Grid2D& Gt, size_t tsize) {
  return (size_t)Gt.ntw * 2 * tsize + (size_t)Gt.Y * Gt.RS * tsize;
}

template <typename T>
hipError_t launch_plane_fwd(int mode, const T* a, T* b, const T* usup, int sx, int sy, int st,
                            int o, T theta, int KG, int r, cpx<T>* dst, int64_t nslices, int Tn,
                            const cpx<T>* tw, const Grid2D& G, hipStream_t stream, int tc) {
  if (nslices <= 0) return hipSuccess;
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3(plane_grid(nslices * Tn)), dim3(kNT),
                       slice_smem_bytes(G, sizeof(T)), stream, mode, a, b, usup, sx, sy, st, o,
                       theta, KG, r, dst, Tn, tw, G, tc, nslices * Tn);
  };
  if (grid_is74(G)) go(k_plane_fwd<T, kRm74F>);
  else if (slice_fits(kRm74, G)) go(k_plane_fwd<T, kRm74>);
  else go(k_plane_fwd<T, kRmAll>);
  return hipGetLastError();
}

int64_t ttile_bins(int Tn, int Yn, int Xh, int tc) {
  return (int64_t)Yn * ((Xh + tc - 1) / tc) * Tn * tc;
}

template <typename T>
hipError_t launch_to_ttiles(const cpx<T>* src, cpx<T>* dst, int Tn, int Yn, int Xh, int tc,
                            int64_t count, hipStream_t stream) {
  if (count <= 0) return hipSuccess;
  const int64_t n = count * ttile_bins(Tn, Yn, Xh, tc);
  hipLaunchKernelGGL((k_to_ttiles<T, cpx<T>>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     stream, src, dst, Tn, Yn, Xh, tc, count);
  return hipGetLastError();
}
template <typename T>
hipError_t launch_to_ttiles_real(const T* src, T* dst, int Tn, int Yn, int Xh, int tc,
                                 hipStream_t stream) {
  const int64_t n = ttile_bins(Tn, Yn, Xh, tc);
  hipLaunchKernelGGL((k_to_ttiles<T, T>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream,
                     src, dst, Tn, Yn, Xh, tc, (int64_t)1);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_tfft(const cpx<T>* src, cpx<T>* dst, int64_t nslices, int Yn, int F2, int sign,
                       const cpx<T>* tw, const Grid2D& Gt, hipStream_t stream) {
  if (nslices <= 0) return hipSuccess;
  const dim3 grid((unsigned)(nslices * Yn));
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, grid, dim3(kNT), tfft_smem_bytes(Gt, sizeof(T)), stream, src, dst,
                       Yn, F2, tw, Gt);
  };
  const bool r42 = rm_fits(kRm42, Gt.py, Gt.Xh);
  const bool f38 = r42 && tline42_ok(Gt, 38);
  if (sign < 0) {
    if (f38) go(k_tfft<T, -1, kRm42, 38>);
    else if (r42) go(k_tfft<T, -1, kRm42>);
    else go(k_tfft<T, -1, kRmAll>);
  } else {
    if (f38) go(k_tfft<T, 1, kRm42, 38>);
    else if (r42) go(k_tfft<T, 1, kRm42>);
    else go(k_tfft<T, 1, kRmAll>);
  }
  return hipGetLastError();
}

// C4's narrow form: TC = 1 on 512-thread workgroups (74 KB of LDS with the filter block
// staged, two workgroups per CU).  Measured slower than TC = 2 on 1024 threads (C4 0.1843 ->
// 0.1954 s per outer iteration, profiles/r05/tsolve_narrow_ab.txt): off unless built with 1.
#ifndef CCSC_TSOLVE_NARROW
#define CCSC_TSOLVE_NARROW 0
#endif
constexpr int kTsNarrowNT = 512;
int tsolve3_nt(int Tn, int K, int TC) {
  return (CCSC_TSOLVE_NARROW != 0 && Tn == 42 && K == 49 && TC == 1) ? kTsNarrowNT : kNT;
}
// per-thread k range of the solve phase (<= 16 k values) and block load slots (<= 8)
static int tsolve3_kg(int Tn, int K, int TC) {
  const int G = std::max(1, tsolve3_nt(Tn, K, TC) / (Tn * TC));
  return (K + G - 1) / G;
}
static int tsolve3_ld(int Tn, int K, int TC) {
  const int nt = tsolve3_nt(Tn, K, TC);
  return (K * Tn * TC + nt - 1) / nt;
}

bool tsolve3_ok(int Tn, int K, int TC) {
  const int nb = Tn * TC;
  if (nb > tsolve3_nt(Tn, K, TC)) return false;
  return tsolve3_kg(Tn, K, TC) <= 16 && tsolve3_ld(Tn, K, TC) <= 8;
}

size_t tsolve3_smem_bytes(const Grid2D& Gt2, int K, int TC, size_t tsize, bool dl) {
  const int nb = Gt2.Y * TC;
  const int G = std::max(1, tsolve3_nt(Gt2.Y, K, TC) / nb);
  return (size_t)Gt2.ntw * 2 * tsize + (size_t)Gt2.Y * K * TC * 2 * tsize +
         (size_t)G * nb * 2 * tsize +                        // + the solve's partial sums
         (dl ? (size_t)K * nb * 2 * tsize + (size_t)nb * tsize : 0);   // + dhat, sden (DL)
}
// the fused t-solve's LDS with the filter block staged (DL) when it fits one CU
static bool tsolve3_dl(const Grid2D& Gt2, int K, int TC, size_t tsize) {
  return tsolve3_smem_bytes(Gt2, K, TC, tsize, true) <= 160 * 1024;
}

template <typename T>
hipError_t launch_tsolve3(cpx<T>* C, const cpx<T>* Bhat, const cpx<T>* dhat, const T* sden,
                          int64_t npatch, int K, int Yn, int Xh, int TC, T invP3,
                          const cpx<T>* tw, const Grid2D& Gt2, hipStream_t stream, int ppw) {
  if (npatch <= 0) return hipSuccess;
  if (Gt2.Xh != K * TC) return hipErrorInvalidValue;   // the plan's line count
  if (!tsolve3_ok(Gt2.Y, K, TC)) return hipErrorInvalidValue;
  const int xtiles = (Xh + TC - 1) / TC;
  if ((int64_t)K * Yn * xtiles * Gt2.Y * TC >= ((int64_t)1 << 31)) return hipErrorInvalidValue;
  ppw = std::max(1, std::min<int>(ppw, (int)npatch));
  const int64_t pgroups = (npatch + ppw - 1) / ppw;
  const dim3 grid((unsigned)(pgroups * Yn * xtiles));
  const bool dl = tsolve3_dl(Gt2, K, TC, sizeof(T));
  const size_t smem = tsolve3_smem_bytes(Gt2, K, TC, sizeof(T), dl);
  const int nt = tsolve3_nt(Gt2.Y, K, TC);
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, grid, dim3(nt), smem, stream, C, Bhat, dhat, sden, K, Yn, Xh, TC,
                       xtiles, invP3, tw, Gt2, npatch, ppw);
  };
  const bool r42 = rm_fits(kRm42, Gt2.py, Gt2.Xh);
  const bool small = tsolve3_ld(Gt2.Y, K, TC) <= 5 && tsolve3_kg(Gt2.Y, K, TC) <= 8;
  if (nt != kNT) {   // C4's narrow form, nothing else
    if (!(r42 && small && dl && TC == 1 && tline42_ok(Gt2, 49))) return hipErrorInvalidValue;
    go(k_tsolve3<T, kRm42, 5, 8, true, 49, kTsNarrowNT, 1>);
  } else if (r42 && small && dl && TC == 2 && tline42_ok(Gt2, 98)) go(k_tsolve3<T, kRm42, 5, 8, true, 98>);   // C4
  else if (r42 && small && dl) go(k_tsolve3<T, kRm42, 5, 8, true, 0>);
  else if (r42 && small) go(k_tsolve3<T, kRm42, 5, 8, false, 0>);
  else if (r42) go(k_tsolve3<T, kRm42, 8, 16, false, 0>);
  else if (small && dl) go(k_tsolve3<T, kRmAll, 5, 8, true, 0>);
  else if (small) go(k_tsolve3<T, kRmAll, 5, 8, false, 0>);
  else if (dl) go(k_tsolve3<T, kRmAll, 8, 16, true, 0>);
  else go(k_tsolve3<T, kRmAll, 8, 16, false, 0>);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_plane_inv(int mode, const cpx<T>* src, T* dst, const T* yv, T* supp, T* norms,
                            int64_t nfirst, T scale, int r, int64_t nslices, int Tn,
                            const cpx<T>* tw, const Grid2D& G, hipStream_t stream, int tc,
                            T* state, T theta, bool wz, cpx<T>* nxt) {
  if (nslices <= 0) return hipSuccess;
  if (mode == 3 && (!state || (norms && !wz))) return hipErrorInvalidValue;
  if (nxt && (mode != 3 || nxt != src)) return hipErrorInvalidValue;
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3(plane_grid(nslices * Tn)), dim3(kNT),
                       slice_smem_bytes(G, sizeof(T)), stream, mode, src, dst, yv, supp, norms,
                       nfirst, scale, r, Tn, tw, G, tc, state, theta, wz ? 1 : 0, nxt,
                       nslices * Tn);
  };
  if (grid_is74(G)) go(k_plane_inv<T, kRm74F>);
  else if (slice_fits(kRm74, G)) go(k_plane_inv<T, kRm74>);
  else go(k_plane_inv<T, kRmAll>);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_zsolve3(cpx<T>* C, const cpx<T>* Bhat, const cpx<T>* dhat, const T* sden,
                          int64_t F3, int64_t npatch, int K, T invP3, hipStream_t stream) {
  if (npatch <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_zsolve3<T>, dim3((unsigned)((F3 + 255) / 256), (unsigned)npatch),
                     dim3(256), 0, stream, C, Bhat, dhat, sden, F3, K, invP3);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_corr_sum(const cpx<T>* Zh, const cpx<T>* dhat, cpx<T>* out, int64_t F3, int K,
                           hipStream_t stream) {
  hipLaunchKernelGGL(k_corr_sum<T>, dim3((unsigned)((F3 + 255) / 256)), dim3(256), 0, stream, Zh,
                     dhat, out, F3, K);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_crop_sq(const T* Dz, const T* b, int sx, int sy, int st, int r, int rt, int X,
                          int Y, const T* z, int64_t zcount, T* part, hipStream_t stream) {
  hipLaunchKernelGGL(k_crop_sq<T>, dim3(256), dim3(256), 0, stream, Dz, b, sx, sy, st, r, rt, X, Y, z,
                     zcount, part);
  return hipGetLastError();
}

template hipError_t launch_plane_fwd<double>(int, const double*, double*, const double*, int, int,
                                             int, int, double, int, int, cpx<double>*, int64_t,
                                             int, const cpx<double>*, const Grid2D&, hipStream_t,
                                             int);
template hipError_t launch_to_ttiles<double>(const cpx<double>*, cpx<double>*, int, int, int, int,
                                             int64_t, hipStream_t);
template hipError_t launch_to_ttiles_real<double>(const double*, double*, int, int, int, int,
                                                  hipStream_t);
template hipError_t launch_tfft<double>(const cpx<double>*, cpx<double>*, int64_t, int, int, int,
                                        const cpx<double>*, const Grid2D&, hipStream_t);
template hipError_t launch_plane_inv<double>(int, const cpx<double>*, double*, const double*,
                                             double*, double*, int64_t, double, int, int64_t, int,
                                             const cpx<double>*, const Grid2D&, hipStream_t, int,
                                             double*, double, bool, cpx<double>*);
template hipError_t launch_tsolve3<double>(cpx<double>*, const cpx<double>*,
                                           const cpx<double>*, const double*, int64_t, int, int,
                                           int, int, double, const cpx<double>*, const Grid2D&,
                                           hipStream_t, int);
template hipError_t launch_zsolve3<double>(cpx<double>*, const cpx<double>*, const cpx<double>*,
                                           const double*, int64_t, int64_t, int, double,
                                           hipStream_t);
template hipError_t launch_corr_sum<double>(const cpx<double>*, const cpx<double>*, cpx<double>*,
                                            int64_t, int, hipStream_t);
template hipError_t launch_crop_sq<double>(const double*, const double*, int, int, int, int, int,
                                           int, int, const double*, int64_t, double*, hipStream_t);

}  // namespace ccsc
