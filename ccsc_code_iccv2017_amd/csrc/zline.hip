// Register-line z-iteration of the 2D learners on the 110 x 110 grid of C1/C2
// (gfx950): the same math as k_zsplit (zsplit.hip; reference dP:150-154 with
// solve_conv_term_Z dP:278-303, dZ:151-157, 283-308), re-laid out so that the
// slice transforms live in registers and LDS only carries transposes.
//
// Every 110-point line transform is the prime-factor (Good-Thomas) split
// 110 = 10 x 11 (coprime factors: no twiddle multiplies), over the lanes of one
// wave (five lines per wave):
//   layout A ("time"): 10 lanes per line, lane n1 holds elements (11 n1 + 10 n2)
//                       mod 110, n2 = 0..10 (11 complex registers);
//   layout B ("freq"): 11 lanes per line, lane k2 holds elements (11 k1 + 100 k2)
//                       mod 110, k1 = 0..9 (10 complex registers).
//   forward A -> B:  DFT-11 over the registers, a wave-local transpose through
//                    LDS, DFT-10 over the registers;
//   inverse B -> A:  the mirror image.
// A slice's 2D transforms are then y-lines (the 56 half-spectrum columns) and
// x-lines (the 55 row pairs packed as complex, two-for-one), joined by one
// workgroup-wide transpose buffer T [110 rows][57 complex] per direction change:
//
//   P1  y-C2R:  bins conj(dw_k) w (layout B, read straight from global in bin-slot
//       order) -> inverse -> T[y][x']
//   P2  barrier
//   P3  x-C2R:  Hermitian rebuild of row pair j from T -> inverse -> layout A of
//       the row pair = corr at (2j, x), (2j+1, x)
//   P4  elementwise in registers: a' = soft(a) + corr (stored), c = u - y
//   P5  x-R2C:  forward -> Z_j into T (rows 2j, 2j+1 of the pair)
//   P6  barrier
//   P7  y-R2C loads: two-for-one separation while reading the columns
//   P8  barrier
//   P9  forward of the columns -> bins C_k (layout B) -> acc += dhat_k C_k
//
// so the per-slice LDS traffic is four wave-local transposes and two
// workgroup transposes (the Stockham form of k_zsplit made ten passes through
// the slice), the elementwise stage and the bin accumulation never touch LDS,
// and a slice costs four barriers instead of nineteen.  Wave-local exchanges
// reuse the wave's own region of T (the columns of its y-lines, the rows of its
// x-lines), which no other wave touches between the barriers.
//
// Layouts in HBM (engine-internal, z-step only):
//   state a:    "state order", per (patch, filter) slice 6050 (row 2j, row 2j+1)
//               pairs, pair n2*550 + j*10 + n1 holds x = elem_a(n1, n2) (zl::state_off);
//   w, B^, d^:  "bin-slot order" per 6160-bin spectrum, slot k1*616 + c*11 + k2
//               holds bin (x' = c, y = elem_b(k2, k1)) (zl::bin_slot) -- lane-contiguous,
//               so every per-slice global access is a coalesced 16-B stream.
// k_zmat / k_zhat_split (zsplit.hip) read these orders; k_state_to_nat and
// k_to_slots convert.
#include "fft_fixed.hpp"
#include "slice.hpp"
#include "zline.hpp"


// Measured on the C2 slice (n = 1000, ms per launch): 7.98 plain, 7.75 nontemporal state,
// 8.56 resident w alone, 7.17 both (round 2); a next-slice state prefetch by the idle wave
// (LDS-DMA) and w held in registers (49 spills) were slower.

namespace ccsc {

constexpr int kZlWL = 7;   // waves whose w bins stay in LDS (35 columns x 110 bins, 61.6 KB)
constexpr size_t kZlWBytes = (size_t)kZlWL * 5 * zl::Y * 16;

// Region-major transpose buffer of k_zline (round 5).  Row pair j (rows 2j, 2j+1) owns
// region (m, r) = (j mod 5, 9j mod 11) of 112 complex slots at A(m) + r PS; inside it,
// slot (a, b) sits at TAU(a) + b:
//   * (x mod 10, x mod 11) = zslot(x) holds Z_j(x), the x-R2C of the packed pair (x->y
//     direction, written by P5), and in the y->x direction H_2j(c) at zslot(c) and
//     H_2j+1(c) at zslot(110 - c), the odd rows of the self-conjugate columns c = 0, 55 at
//     (10, 0) / (10, 1);
//   * so an x-line touches only its own region and a y-line (column c) only the slots
//     zslot(c), zslot(110 - c) (or (10, 0/1)) of every region: P3..P5 of a pair and P7,
//     P9, P1 of a column are private to their lines (their wave-local exchanges live in
//     those slots too), and a slice needs two workgroup barriers (the two transposes)
//     instead of four;
//   * every access is a per-lane base plus a compile-time register offset: a y-line's
//     layout-A lane n1 owns rows (11 n1 + 10 n2) mod 110, i.e. region (n1 >> 1, n2 + (n1 & 1))
//     (one wrap, at n2 = 10 on the odd lanes) -- no per-element row or column index math.
// PS, A and TAU come from a search over the gfx950 bank model (tools/lds_anneal.py,
// tools/lds_sim2.py): 16.0k LDS-array cycles per slice and workgroup, the same as the
// round-4 column layout (16.1k).
namespace zr {
constexpr int PS = 113;
__host__ __device__ constexpr int A(int m) { return m * 1245 + (m >= 3 ? 5 : 0) + (m >= 4 ? 29 : 0); }
__host__ __device__ constexpr int TAU(int a) { return 11 * a + 5 + (a >= 2 ? 1 : 0); }
__host__ __device__ constexpr int SL(int a, int b) { return TAU(a) + b; }
constexpr int kSize = A(4) + 10 * PS + SL(10, 1) + 1;   // complex slots
// column c's slots: H_2j(c) / Z_j(c), Z_j(110 - c) (x->y), H_2j+1(c) (y->x)
__device__ __forceinline__ int ze(int c) { return SL(c % 10, c % 11); }
__device__ __forceinline__ int zm(int c) {
  const int x = c == 0 ? 0 : 110 - c;
  return SL(x % 10, x % 11);
}
__device__ __forceinline__ int zo(int c) { return c == 0 ? SL(10, 0) : c == 55 ? SL(10, 1) : zm(c); }
__device__ __forceinline__ int region(int j) { return A(j % 5) + ((9 * j) % 11) * PS; }
// bit k1 set: bin x = elem_b(k2, k1) > 55 of an x-line's layout-B lane k2 (its P3 value
// is the swapped combination of the two slots it reads); as 64-bit lane masks of the
// wave's lane layout (five 11-lane lines, lanes 55..63 duplicating k2 = 10)
constexpr bool hi_bin(int k2, int k1) { return (11 * k1 + 100 * k2) % 110 > 55; }
constexpr unsigned long long hi_mask(int k1) {
  unsigned long long m = 0;
  for (int lane = 0; lane < 64; ++lane) {
    const int l = lane / 11 < 4 ? lane / 11 : 4;
    const int s = lane - 11 * l;
    if (hi_bin(s < 10 ? s : 10, k1)) m |= 1ull << lane;
  }
  return m;
}
// evaluated at compile time (a namespace-scope constexpr table: as a call in the kernel
// the lane loop was left to run on the scalar unit)
struct HiMasks {
  unsigned long long m[10];
};
constexpr HiMasks make_hi_masks() {
  HiMasks h{};
  for (int k1 = 0; k1 < 10; ++k1) h.m[k1] = hi_mask(k1);
  return h;
}
constexpr HiMasks kHi = make_hi_masks();
}  // namespace zr
constexpr size_t kZlSmem = (size_t)zr::kSize * 16 + kZlWBytes;
static_assert(kZlSmem <= 160 * 1024, "z-step LDS");

// clamp(a, -theta, theta): the prox and the dual update of a z-iteration are
// u = soft(a, theta) = a - clamp(a) and u - y = 2u - a = a - 2 clamp(a) (min/max + one
// add or FMA each, no compare/select chains)
// theta stays in its kernel-argument SGPRs (the VOP3 min/max read it there, negated by
// the source modifier): as a C++ fmin/fmax operand it is canonicalised into four VGPRs
// held across the slice loop, at the VGPR cap (inputs are finite: no NaN quieting needed)
__device__ __forceinline__ double clamp_t(double a, double theta) {
  double r;
  asm("v_min_f64 %0, %1, %2\n\tv_max_f64 %0, %0, -%2" : "=&v"(r) : "v"(a), "s"(theta));
  return r;
}

// the z-step's LDS as bytes (32-bit offsets: no 64-bit address arithmetic)
template <typename T>
__device__ __forceinline__ cpx<T>& lds_cpx_at(uint32_t byte_off) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  return *reinterpret_cast<cpx<T>*>(smem + byte_off);
}

template <typename T, int R, int SIGN, typename Sink>
__device__ __forceinline__ void zdft(cpx<T> (&v)[R], Sink&& sink) {
  dft_sink<T, R, SIGN>(v, sink);
}

__device__ __forceinline__ void wave_lds_fence() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Forward 110-point transform of one line, layout A (v[n2], lane n1 = s < 10)
// -> layout B (out[k1], lane k2 = s <= 10).  eb: LDS byte offset of the line's 110
// exchange slots, slot n1*11 + k2 at complex (n1*11 + k2) * ES from it (32-bit offsets:
// the slot's constant part folds into the instruction's offset field).
// Idle lanes (lane 10 of a line in layout A, lanes 55..63, the clamped lines of the
// last wave) run on clamped indices and so duplicate a real lane exactly: their
// LDS and global stores write the same value to the same address, no guards
// (k_zline masks lanes 55..63 and the clamped lines out of its phases).
// The outputs stream to sink(k1, value) as the last stage forms them.
// ODDROT: the inputs of the lanes n1 odd arrive divided by -i (the y-R2C's two-for-one
// separation of the odd rows, see P7): in layout B they are register n1 (compile time),
// so the factor -i is a free swap + negate of the DFT-10's operands.
template <typename T, int ES, bool ODDROT = false, typename Sink>
__device__ __forceinline__ void fwd_line(cpx<T> (&v)[11], uint32_t eb, int s, Sink&& sink) {
  const int sa = min(s, 9);
  const uint32_t ea = eb + (uint32_t)(sa * 11 * ES) * 16u, es = eb + (uint32_t)(s * ES) * 16u;
  zdft<T, 11, -1>(v, [&](int k2, cpx<T> val) { lds_cpx_at<T>(ea + (uint32_t)(k2 * ES * 16)) = val; });
  wave_lds_fence();
  cpx<T> in[10];
#pragma unroll
  for (int n1 = 0; n1 < 10; ++n1) {
    const cpx<T> w = lds_cpx_at<T>(es + (uint32_t)(n1 * 11 * ES * 16));
    in[n1] = (ODDROT && (n1 & 1)) ? cpx<T>{w.y, -w.x} : w;
  }
  zdft<T, 10, -1>(in, sink);
}

// Inverse (unnormalised) 110-point transform, layout B (in[k1], lane k2 = s)
// -> layout A (out[n2], lane n1 = s < 10).
template <typename T, int ES, typename Sink>
__device__ __forceinline__ void inv_line(cpx<T> (&in)[10], uint32_t eb, int s, Sink&& sink) {
  const uint32_t es = eb + (uint32_t)(s * ES) * 16u;
  zdft<T, 10, +1>(in, [&](int n1, cpx<T> val) { lds_cpx_at<T>(es + (uint32_t)(n1 * 11 * ES * 16)) = val; });
  wave_lds_fence();
  const int sa = min(s, 9);
  const uint32_t ea = eb + (uint32_t)(sa * 11 * ES) * 16u;
  cpx<T> v[11];
#pragma unroll
  for (int k2 = 0; k2 < 11; ++k2) v[k2] = lds_cpx_at<T>(ea + (uint32_t)(k2 * ES * 16));
  zdft<T, 11, +1>(v, sink);
}

// Consumption orders of the register DFTs (dft_sink): loads issued in these orders let the
// in-order vmcnt / lgkmcnt waits release each value as soon as its own load is back (issued
// 0..R-1, the DFT-11's third input -- register 10 -- waited for every load of the group).
//   DFT-11 reads its inputs as v0 then the pairs (r, 11 - r); its outputs stream 0, (q, 11 - q)
//   DFT-10 (2 x 5 prime-factor) reads the pairs (2 n2, 5 + 2 n2) mod 10
// (same-box A/B at n = 1000: 5.874 -> 5.850 ms per launch; the filter spectrum's P9 loads
// issued ahead of the DFT in its output order measured slower, 5.955)
constexpr int kOrd11[11] = {0, 1, 10, 2, 9, 3, 8, 4, 7, 5, 6};
constexpr int kOrd10in[10] = {0, 5, 2, 7, 4, 9, 6, 1, 8, 3};

// The same line transforms with the exchange slot of each register given by a caller's
// address function (byte offsets, compile-time register index): the region-major buffer
// places a y-line's 110 exchange slots over all regions, an x-line's inside its own.
template <typename T, typename WA, typename RA, typename Sink>
__device__ __forceinline__ void inv_line_r(cpx<T> (&in)[10], WA&& waddr, RA&& raddr, Sink&& sink) {
  zdft<T, 10, +1>(in, [&](int n1, cpx<T> val) { lds_cpx_at<T>(waddr(n1)) = val; });
  wave_lds_fence();
  cpx<T> v[11];
#pragma unroll
  for (int i = 0; i < 11; ++i) v[kOrd11[i]] = lds_cpx_at<T>(raddr(kOrd11[i]));
  zdft<T, 11, +1>(v, sink);
}
template <typename T, bool ODDROT, typename WA, typename RA, typename Sink>
__device__ __forceinline__ void fwd_line_r(cpx<T> (&v)[11], WA&& waddr, RA&& raddr, Sink&& sink) {
  zdft<T, 11, -1>(v, [&](int k2, cpx<T> val) { lds_cpx_at<T>(waddr(k2)) = val; });
  wave_lds_fence();
  cpx<T> in[10];
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const int n1 = kOrd10in[i];
    const cpx<T> w = lds_cpx_at<T>(raddr(n1));
    in[n1] = (ODDROT && (n1 & 1)) ? cpx<T>{w.y, -w.x} : w;
  }
  zdft<T, 10, -1>(in, sink);
}

// select between two doubles on a compile-time lane mask (two v_cndmask_b32 with the mask
// in an SGPR pair: no per-lane condition arithmetic)
__device__ __forceinline__ double lane_sel(double a_if_set, double b, unsigned long long mask) {
  const int alo = __double2loint(a_if_set), ahi = __double2hiint(a_if_set);
  const int blo = __double2loint(b), bhi = __double2hiint(b);
  int lo, hi;
  asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(lo) : "v"(blo), "v"(alo), "s"(mask));
  asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(hi) : "v"(bhi), "v"(ahi), "s"(mask));
  return __hiloint2double(hi, lo);
}

__device__ __forceinline__ void zl_sync() { lds_sync(); }

// (e mod 110) for 0 <= e < 220
__device__ __forceinline__ int mod110(int e) { return e >= 110 ? e - 110 : e; }
// slot of element x of a row pair's spectrum Z_j in layout-B order (k1*11 + k2)
__device__ __forceinline__ int zslot(int x) { return (x % 10) * 11 + (x % 11); }

// LDS bank placement (gfx950: a ds_read_b128 serves 16 lanes per cycle, one 16-B chunk of
// the 256-B bank row each; tools/lds_sim.py models every access of this kernel):
//  * T rows (P1 sink, P3 reads): column c at tcol(c) = even columns then odd ones -- the
//    P3 reads of one register all have one column parity, which on the natural order
//    leaves them 8 of the 16 chunks (modelled 2486 -> 1650 LDS cycles per slice);
//  * a wave's five x-lines exchange at line offsets 110 l + {0, 0, 11, 12, 16} and store
//    their spectra Z_j at 110 l + {0, 6, 7, 8, 11} of the wave's ten T rows (570 slots)
//    instead of 110 l / 114 l (exchanges 2068 -> 1485, P7 reads 2968 -> 1888).
// Every region a wave writes between two barriers stays inside the ten rows it alone
// reads in P3, as before.
__device__ __forceinline__ int tcol(int c) { return (c >> 1) + (c & 1) * 28; }
__device__ __forceinline__ int xoff(int l) { return 110 * l + (l < 2 ? 0 : l == 2 ? 11 : l == 3 ? 12 : 16); }
__device__ __forceinline__ int zoff(int l) { return 110 * l + (l < 1 ? 0 : l < 4 ? 5 + l : 11); }
constexpr int kZlWR = 10 * zl::RS;   // complex slots of a wave's ten T rows

// 16-B global access at a 32-bit byte offset from a wave-uniform base (saddr form:
// SGPR base + one VGPR offset, no 64-bit VGPR address per access).
template <typename V>
__device__ __forceinline__ V zld(const void* base, uint32_t boff) {
  return *reinterpret_cast<const V*>(reinterpret_cast<const char*>(base) + boff);
}
template <typename V>
__device__ __forceinline__ void zst(void* base, uint32_t boff, V v) {
  *reinterpret_cast<V*>(reinterpret_cast<char*>(base) + boff) = v;
}
// Buffer-descriptor forms of the slice loop's global loads: the wave-uniform base goes
// into a descriptor, the lane's byte offset into voffset and the register's constant
// offset into soffset (an SGPR), so no per-access 64-bit VGPR address arithmetic is
// issued (6.75 -> 6.55 ms at n = 1000, round 3).
typedef unsigned int zl_u4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t zrsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}
constexpr int kZlNT = 2;   // cache policy bit: nontemporal (gfx950 NT = SLC)
template <typename V, int AUX>
__device__ __forceinline__ V bld(const void* base, uint32_t bytes, uint32_t voff, uint32_t soff) {
  const zl_u4 u = __builtin_amdgcn_raw_buffer_load_b128(zrsrc(base, bytes), voff, soff, AUX);
  V v;
  __builtin_memcpy(&v, &u, 16);
  return v;
}
// spectrum (F complex) access: lane offset + register offset
template <typename V>
__device__ __forceinline__ V fld(const void* base, uint32_t lane, uint32_t reg) {
  return bld<V, 0>(base, zl::F * 16, lane, reg);
}
template <typename V>
__device__ __forceinline__ V wld(const void* base, uint32_t lane, uint32_t reg) {
  return bld<V, 0>(base, zl::F * 16, lane, reg);
}
// The state stream (read once, written once per launch) is nontemporal, so it does not
// evict the re-read spectra (w, dcorr, dhat) from L2.  State slice (P reals) loads:
template <typename V>
__device__ __forceinline__ V sld2(const void* base, uint32_t lane, uint32_t reg) {
  return bld<V, kZlNT>(base, zl::P * 8, lane, reg);
}
// state stores stay global stores: a buffer store carrying the register offset in soffset
// failed the mode-2 parity cases on the GPU (round 3), while the same store with the whole
// offset in voffset passes and then costs the same per-store VGPR add as a global store
typedef double nt_d2 __attribute__((ext_vector_type(2)));
template <typename V>
__device__ __forceinline__ void sst2(void* base, uint32_t lane, uint32_t reg, V v) {
  const nt_d2 r = {v.x, v.y};
  // one 32-bit offset: the saddr form (SGPR base + VGPR offset), no 64-bit address add per store
  __builtin_nontemporal_store(r, reinterpret_cast<nt_d2*>(reinterpret_cast<char*>(base) + (uint32_t)(lane + reg)));
}

// an opaque copy of a lane index: per-lane address math is redone where it is used
// instead of being hoisted out of the slice loop into (spilled) registers
__device__ __forceinline__ int fresh(int v) {
  asm volatile("" : "+v"(v));
  return v;
}

// One workgroup per patch, loop over its K filter slices.  MODE 0: Zn / Yn hold
// the materialised (z, y) in natural layout (a = z + y, no corr term); MODE 2:
// A holds the state in state order and W the previous w (bin-slot order) solved
// with dcorr.  Out: Ao <- a' (state order; Ao may alias A, or Zn in mode 0),
// W <- w.  Bs, dcorr, dhat, sden in bin-slot order.
//
// The tol test (dP:156-157 / dZ:163-169: ||z - z_old|| / ||z|| after every
// z-iteration) without a third z-sized buffer.  TOL is a set of kZt* bits:
//  kZtForm  the test of the iterate the launch PRODUCES, in the launch itself, when the
//           state's w was solved with the current filters (dcorr == dhat): the launch
//           holds c_t = 2 soft(a) - a of the iterate it starts from and c_t+1 of the one it
//           produces, and w_t, w_t+1 at its end; with z = c + ifft(conj(dhat) w_true),
//           w_true = XY w = (B - acc) / (rho + s), Parseval gives
//             ||z_t+1 - z_t||^2 = sum ||c_t+1 - c_t||^2 - XY sum_f |w_t+1 - w_t|^2 (2 rho + s)
//             ||z_t+1||^2       = sum ||c_t+1||^2 + sum_f [2 Re(w conj(acc)) + XY s |w|^2]
//           (half-spectrum bins weighted 2 but the self-conjugate columns x' = 0, 55;
//           the cross terms use acc_t+1 - acc_t = -(rho + s) XY (w_t+1 - w_t)) into
//           fpart[2p], [2p + 1] -- no z-sized stream;
//  kZtStore z_cur = (u - y)(A) + corr (mode 2) or the materialised z (mode 0), the z of
//           the iterate the launch starts from, formed in registers anyway, to Zt in state
//           order (the otherwise idle y buffer; in mode 0 Zt may alias Yn: read before
//           written) -- after a launch whose starting w came from other filters (the first
//           z-iteration of an outer iteration) or a materialised state;
//  kZtCmp   reads the z before it from Zt and adds ||z_cur - z_prev||^2, ||z_cur||^2 of the
//           patch into zpart[2p], [2p + 1] -- the test of the iterate the launch started
//           from, one launch late (the engine treats the launch as speculative, DESIGN.md
//           §4).
// MODE 3 ("finalize"): kZtStore | kZtCmp without advancing: no state write, no R2C, W
// untouched.
constexpr int kZtStore = kZlTolStore, kZtCmp = kZlTolCmp, kZtForm = kZlTolForm;
template <typename T, int MODE, int TOL>
__global__ __launch_bounds__(zl::NT) __attribute__((amdgpu_waves_per_eu(3, 3))) void k_zline(const T* A, T* Ao, const T* Zn, const T* Yn,
                                                  cpx<T>* __restrict__ W,
                                                  const cpx<T>* __restrict__ Bs,
                                                  const cpx<T>* __restrict__ dcorr,
                                                  const cpx<T>* __restrict__ dhat,
                                                  const T* __restrict__ sden, int K, T theta,
                                                  T rho, T* Zt, T* __restrict__ zpart,
                                                  T* __restrict__ fpart) {
  static_assert(MODE == 0 || MODE == 2 || MODE == 3, "zline mode");
  static_assert(TOL >= 0 && TOL <= 7 && (!(TOL & kZtCmp) || (TOL & kZtStore)) &&
                    (MODE != 0 || TOL <= kZtStore) &&
                    (MODE != 3 || TOL == (kZtStore | kZtCmp)),
                "zline tol variant");
  constexpr bool kStore = TOL & kZtStore, kCmp = TOL & kZtCmp, kForm = TOL & kZtForm;
  using V2 = typename vec2_t<T>::type;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  cpx<T>* sT = reinterpret_cast<cpx<T>*>(smem);
  const int64_t p = blockIdx.x;
  cpx<T> acc[10];
#pragma unroll
  for (int i = 0; i < 10; ++i) acc[i] = {(T)0, (T)0};
  const cpx<T>* Wp = W + p * zl::F;
  // the last wave owns one y-line and no x-line (55 row pairs = 11 waves of 5)
  const bool xwave = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6) < 11;
  T nd = (T)0, nz = (T)0;   // kCmp: ||z_cur - z_prev||^2, ||z_cur||^2 of the lanes' own elements
  T fd = (T)0, fz = (T)0;   // kForm: ||z_t+1 - z_t||^2, ||z_t+1||^2 (element, then bin terms)
  // w is the same for every slice of the patch: the y-lines of waves 0..kZlWL-1 (columns
  // 0..5 kZlWL - 1) keep their bins in the LDS left over beside T, each lane its own ten
  // (slot k1 * 385 + c * 11 + k2; written and read back by the same lane, so no barrier)
  cpx<T>* sW = sT + zr::kSize;
  if constexpr (MODE >= 2) {
    if (__builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6) < kZlWL) {
      const int lane = threadIdx.x & 63, l = min(lane / 11, 4), s = lane - 11 * l;
      const int c = 5 * (int)(threadIdx.x >> 6) + l;
      const int sb = min(s, 10);
      const uint32_t bo = (uint32_t)(c * 11 + sb) * 16u;
#pragma unroll
      for (int k1 = 0; k1 < 10; ++k1) sW[k1 * 385 + c * 11 + sb] = zld<cpx<T>>(Wp, bo + k1 * 616 * 16);
    }
  }
  constexpr uint32_t kPSB = (uint32_t)zr::PS * 16u;   // region stride per n2, bytes

  for (int k = 0; k < K; ++k) {
    // lane roles, recomputed per slice from an opaque thread index (see fresh())
    const int tid = fresh((int)threadIdx.x);
    const int wave = tid >> 6, lane = tid & 63;
    const int l = min(lane / 11, 4);   // line within the wave (lanes 55..63 alias line 4)
    const int s = lane - 11 * l;       // n1 (layout A, < 10) or k2 (layout B); >= 11 idle
    const int sb = min(s, 10), sa = min(s, 9);
    const int c = min(5 * wave + l, 55);   // y-line (column)
    const int j = min(5 * wave + l, 54);   // x-line (row pair)
    // lanes that duplicate another lane's work (55..63: line 4, k2 = 10; lines 1..4 of the last
    // wave: column 55 again) sit the phases out -- their stores only repeated a real lane's, and
    // the kernel is power-limited: 5.886 -> 5.817 ms at n = 1000
    // (profiles/r06/zline_lane_mask_ab.txt)
    const bool xlive = lane < 55;
    const bool ylive = lane < 55 && (__builtin_amdgcn_readfirstlane(wave) < zl::NW - 1 || lane < 11);
    const int64_t sl = (p * K + k) * zl::P;
    cpx<T> zc[11];   // c = u - y of the row pair (x-lines, layout A) for the R2C
    const uint32_t po = (uint32_t)(j * 10 + fresh(sa)) * 16u;   // pair n2 at po + n2*550*16
    V2 av[11];   // the state a of row pair j (layout A), mode 2
    // the y-line's exchange bases (region-major buffer, zr): DFT-10 side (lanes k2) at
    // wE / wO + A(n1 mod 5) for n1 < 5 / >= 5, DFT-11 side (lanes n1) at yX + k2 PS
    const int yzE = zr::ze(c), yzO = zr::zo(c);
    const uint32_t ywE = (uint32_t)(sb * zr::PS + yzE) * 16u, ywO = (uint32_t)(sb * zr::PS + yzO) * 16u;
    const uint32_t yX = (uint32_t)(zr::A(sa < 5 ? sa : sa - 5) + (sa < 5 ? yzE : yzO)) * 16u;
    auto yw = [&](int n1) { return (n1 < 5 ? ywE : ywO) + (uint32_t)zr::A(n1 % 5) * 16u; };
    auto yr = [&](int k2) { return yX + (uint32_t)k2 * kPSB; };
    if constexpr (MODE >= 2) {
      if (ylive) {
        // ---- P1: y-C2R of conj(dcorr_k) w from bins to column c of every region ----
        const cpx<T>* dk = dcorr + (int64_t)k * zl::F;
        const uint32_t bo = (uint32_t)(c * 11 + sb) * 16u;
        const bool wl = __builtin_amdgcn_readfirstlane(wave) < kZlWL;
        // every operand load first, then the products (sched_barrier): interleaved, the
        // scheduler waits for each load pair in turn -- ten L2 round trips per wave
        cpx<T> b[10], wv[10];
        if (wl) {
#pragma unroll
          for (int i = 0; i < 10; ++i) {
            const int k1 = kOrd10in[i];
            b[k1] = fld<cpx<T>>(dk, bo, k1 * 616 * 16);
            wv[k1] = sW[k1 * 385 + c * 11 + sb];
          }
        } else {
#pragma unroll
          for (int i = 0; i < 10; ++i) {
            const int k1 = kOrd10in[i];
            b[k1] = fld<cpx<T>>(dk, bo, k1 * 616 * 16);
            wv[k1] = wld<cpx<T>>(Wp, bo, k1 * 616 * 16);
          }
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < 10; ++i) b[kOrd10in[i]] = cmulc(b[kOrd10in[i]], wv[kOrd10in[i]]);
        // row (11 n1 + 10 n2) mod 110 of lane n1 = sa: region (sa >> 1, n2 + (sa & 1)), its
        // column slot ze (even rows) / zo (odd rows); the odd lanes wrap at n2 = 10
        const uint32_t ys = (uint32_t)(zr::A(sa >> 1) + ((sa & 1) ? zr::PS + yzO : yzE)) * 16u;
        const uint32_t ys10 = ys - ((sa & 1) ? 11u * kPSB : 0u);
        inv_line_r<T>(b, yw, yr, [&](int n2, cpx<T> val) {
          lds_cpx_at<T>((n2 == 10 ? ys10 : ys) + (uint32_t)n2 * kPSB) = val;
        });
      }
      zl_sync();   // P2
      if (xwave && xlive) {
        // ---- P3: x-C2R of row pair j from its region: Z(x) = H_2j(x) + i H_2j+1(x) ----
        const int s3 = fresh(sb);
        const int R = zr::region(j);
        const uint32_t xa = (uint32_t)(R + s3) * 16u;                  // slot (k1, s3) + TAU(k1)
        const uint32_t xb = (uint32_t)(R + (s3 == 0 ? 0 : 11 - s3)) * 16u;   // (10-k1, 11-s3)
        // lane k2 = 0's bins x = 0, 55 take their odd-row value from (10, 0) / (10, 1)
        const uint32_t xb0 = xb + (s3 == 0 ? (uint32_t)(zr::TAU(10) - zr::TAU(0)) * 16u : 0u);
        const uint32_t xb5 = xb + (s3 == 0 ? (uint32_t)(zr::SL(10, 1) - zr::TAU(5)) * 16u : 0u);
        cpx<T> zb[10], zr_[10];
        // the 20 reads first, then the combination (no pairwise lgkmcnt waits)
#pragma unroll
        for (int i = 0; i < 10; ++i) {
          const int k1 = kOrd10in[i];
          zb[k1] = lds_cpx_at<T>(xa + (uint32_t)zr::TAU(k1) * 16u);
          const uint32_t bb = k1 == 0 ? xb0 : k1 == 5 ? xb5 : xb;
          zr_[k1] = lds_cpx_at<T>(bb + (uint32_t)zr::TAU((10 - k1) % 10) * 16u);
        }
        __builtin_amdgcn_sched_barrier(0);
        // x <= 55: u + i v (u = H_2j(x), v = H_2j+1(x)); x > 55: conj(v) + i conj(u) with
        // u, v the values of column 110 - x -- the same two sums, re and im swapped
#pragma unroll
        for (int i = 0; i < 10; ++i) {
          const int k1 = kOrd10in[i];
          const T p_ = zb[k1].x - zr_[k1].y, q_ = zb[k1].y + zr_[k1].x;
          zb[k1] = {lane_sel(q_, p_, zr::kHi.m[k1]), lane_sel(p_, q_, zr::kHi.m[k1])};
        }
        // ---- P4: state (row 2j, row 2j+1) at x = elem_a(n1, n2), in flight under the C2R;
        // each corr value is consumed as the last inverse stage forms it ----
#pragma unroll
        for (int i = 0; i < 11; ++i) av[kOrd11[i]] = sld2<V2>(A + sl, po, kOrd11[i] * 550 * 16);
        V2 zo_[kCmp ? 11 : 1];
        if constexpr (kCmp) {
#pragma unroll
          for (int i = 0; i < 11; ++i) zo_[kOrd11[i]] = sld2<V2>(Zt + sl, po, kOrd11[i] * 550 * 16);
        }
        // lanes that own their elements (not a clamped duplicate) count in the norms
        const T own = (s < 10 && lane < 55) ? (T)1 : (T)0;
        const uint32_t xn = (uint32_t)(R + zr::TAU(fresh(sa))) * 16u;   // lanes n1: + k2
        inv_line_r<T>(
            zb, [&](int n1) { return xa + (uint32_t)zr::TAU(n1) * 16u; },
            [&](int k2) { return xn + (uint32_t)k2 * 16u; },
            [&](int n2, cpx<T> corr) {
              V2 a = av[n2];
              const T tx = clamp_t(a.x, theta), ty = clamp_t(a.y, theta);
              const T sx = a.x - tx, sy = a.y - ty;                          // u = soft(a)
              const T ctx = fma((T)-2, tx, a.x), cty = fma((T)-2, ty, a.y);   // c_t = u - y
              if constexpr (kStore) {   // z_cur = (u - y)(A) + corr
                V2 zn;
                zn.x = ctx + corr.x;
                zn.y = cty + corr.y;
                if constexpr (kCmp) {
                  const T ex = zn.x - zo_[n2].x, ey = zn.y - zo_[n2].y;
                  nd += own * (ex * ex + ey * ey);
                  nz += own * (zn.x * zn.x + zn.y * zn.y);
                }
                sst2<V2>(Zt + sl, po, n2 * 550 * 16, zn);
              }
              if constexpr (MODE == 2) {
                a.x = sx + corr.x;
                a.y = sy + corr.y;
                sst2<V2>(Ao + sl, po, n2 * 550 * 16, a);
                zc[n2] = {fma((T)-2, clamp_t(a.x, theta), a.x), fma((T)-2, clamp_t(a.y, theta), a.y)};
                if constexpr (kForm) {   // c_t+1 - c_t and c_t+1 of the lanes' own elements
                  const T dx = zc[n2].x - ctx, dy = zc[n2].y - cty;
                  fd += own * (dx * dx + dy * dy);
                  fz += own * (zc[n2].x * zc[n2].x + zc[n2].y * zc[n2].y);
                }
              }
            });
      }
    } else {
      // ---- P4 (mode 0): a = z + y from the materialised natural layout ----
      V2 av0[11];
      if (xwave && xlive) {
        const T* z0 = Zn + sl + 2 * j * zl::X;
        const T* y0 = Yn + sl + 2 * j * zl::X;
#pragma unroll
        for (int n2 = 0; n2 < 11; ++n2) {
          const int x = mod110(11 * sa + 10 * n2);
          av0[n2].x = z0[x] + y0[x];
          av0[n2].y = z0[zl::X + x] + y0[zl::X + x];
        }
#pragma unroll
        for (int n2 = 0; n2 < 11; ++n2) {
          const V2 a = av0[n2];
          zc[n2] = {fma((T)-2, clamp_t(a.x, theta), a.x), fma((T)-2, clamp_t(a.y, theta), a.y)};
        }
      }
      V2 zv[kStore ? 11 : 1];
      if constexpr (kStore) {
        if (xwave && xlive) {
          const T* z0 = Zn + sl + 2 * j * zl::X;
#pragma unroll
          for (int n2 = 0; n2 < 11; ++n2) {
            const int x = mod110(11 * sa + 10 * n2);
            zv[n2].x = z0[x];
            zv[n2].y = z0[zl::X + x];
          }
        }
      }
      __syncthreads();   // the slice is read in natural order before it is rewritten in state order
      if (xwave && xlive) {
#pragma unroll
        for (int n2 = 0; n2 < 11; ++n2) {
          zst<V2>(Ao + sl, po + n2 * 550 * 16, av0[n2]);
          if constexpr (kStore) zst<V2>(Zt + sl, po + n2 * 550 * 16, zv[n2]);
        }
      }
    }
    if constexpr (MODE == 3) {
      lds_sync();   // the next slice's P1 rewrites every region's column slots
      continue;
    }
    // ---- P5: x-R2C of the row pair -> Z_j(x) at slot zslot(x) of its region ----
    if (xwave && xlive) {
      const int R = zr::region(j);
      const uint32_t xa = (uint32_t)(R + fresh(sb)) * 16u;
      const uint32_t xn = (uint32_t)(R + zr::TAU(fresh(sa))) * 16u;
      fwd_line_r<T, false>(
          zc, [&](int k2) { return xn + (uint32_t)k2 * 16u; },
          [&](int n1) { return xa + (uint32_t)zr::TAU(n1) * 16u; },
          [&](int k1, cpx<T> val) { lds_cpx_at<T>(xa + (uint32_t)zr::TAU(k1) * 16u) = val; });
    }
    zl_sync();   // P6
    // ---- P7: column c, rows y = (11 n1 + 10 n2) mod 110: two-for-one separation of
    // Z_j(c), Z_j(110 - c) of pair y >> 1 (region (n1 >> 1, n2 + (n1 & 1))) ----
    if (ylive) {
      cpx<T> col[11];
      {
        const int n1 = fresh(sa);
        const T sg = (n1 & 1) ? (T)-1 : (T)1;
        const uint32_t rb = (uint32_t)(zr::A(n1 >> 1) + (n1 & 1) * zr::PS) * 16u;
        const uint32_t rb10 = rb - ((n1 & 1) ? 11u * kPSB : 0u);
        const uint32_t a1 = (uint32_t)zr::ze(c) * 16u, a2 = (uint32_t)zr::zm(c) * 16u;
        // even rows z1 + conj z2, odd rows z1 - conj z2 -- twice the row spectra (the 1/2 is
        // applied once to the patch's accumulated bins), the odd rows' times i (the -i is
        // applied in P9's DFT-10, where the odd rows are compile-time registers -- ODDROT)
        cpx<T> z1[11], z2[11];
#pragma unroll
        for (int i = 0; i < 11; ++i) {
          const int n2 = kOrd11[i];
          const uint32_t r = (n2 == 10 ? rb10 : rb) + (uint32_t)n2 * kPSB;
          z1[n2] = lds_cpx_at<T>(r + a1);
          z2[n2] = lds_cpx_at<T>(r + a2);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < 11; ++i) {
          const int n2 = kOrd11[i];
          col[n2] = {fma(sg, z2[n2].x, z1[n2].x), fma(-sg, z2[n2].y, z1[n2].y)};
        }
      }
      // no barrier: P9's exchange reuses the slots this line alone just read
      // ---- P9: y-R2C of column c -> bins, accumulate sum_k dhat_k C_k ----
      {
        const int s9 = fresh(sb);
        const cpx<T>* dk = dhat + (int64_t)k * zl::F;
        const uint32_t bo = (uint32_t)(c * 11 + s9) * 16u;
        fwd_line_r<T, true>(col, yr, yw, [&](int k1, cpx<T> cb) {
          acc[k1] = cmac(acc[k1], fld<cpx<T>>(dk, bo, k1 * 616 * 16), cb);
        });
      }
    }
  }
  // w = (B - acc) * sden  (sden = 1/((rho + s) X Y)); each lane owns its slots
  if constexpr (MODE != 3) {
#pragma unroll
    for (int i = 0; i < 10; ++i) acc[i] = cscale(acc[i], (T)0.5);   // P7's unscaled separation
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int l = lane / 11, s = lane - 11 * l, line = 5 * wave + l;
    if (l < 5 && line < 56) {
      cpx<T>* Wo = W + p * zl::F;
      const cpx<T>* Bp = Bs + p * zl::F;
      const T wt = (line == 0 || line == zl::Xh - 1) ? (T)1 : (T)2;   // self-conjugate columns
#pragma unroll
      for (int k1 = 0; k1 < 10; ++k1) {
        const int sl2 = k1 * 616 + line * 11 + s;
        const T sd = sden[sl2];
        const cpx<T> wn = cscale(csub(Bp[sl2], acc[k1]), sd);
        if constexpr (kForm) {   // the bin terms of the Parseval forms (w_t is read first)
          const cpx<T> dw = csub(wn, Wo[sl2]);
          const T rs = (T)1 / (sd * (T)zl::P);   // rho + s(f)
          fd -= wt * (T)zl::P * cabs2(dw) * (rs + rho);
          fz += wt * ((T)2 * (wn.x * acc[k1].x + wn.y * acc[k1].y) +
                      (T)zl::P * (rs - rho) * cabs2(wn));
        }
        Wo[sl2] = wn;
      }
    }
  }
  if constexpr (kCmp || kForm) {   // patch sums of the tol norms (T is free after the last slice)
    T* red = reinterpret_cast<T*>(smem);
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    nd = wave_sum(nd);
    nz = wave_sum(nz);
    fd = wave_sum(fd);
    fz = wave_sum(fz);
    lds_sync();
    if (lane == 0) {
      red[4 * wave] = nd;
      red[4 * wave + 1] = nz;
      red[4 * wave + 2] = fd;
      red[4 * wave + 3] = fz;
    }
    lds_sync();
    if (threadIdx.x == 0) {
      T sd = 0, sz = 0, sfd = 0, sfz = 0;
      for (int w = 0; w < zl::NW; ++w) {
        sd += red[4 * w];
        sz += red[4 * w + 1];
        sfd += red[4 * w + 2];
        sfz += red[4 * w + 3];
      }
      if constexpr (kCmp) {
        zpart[2 * p] = sd;
        zpart[2 * p + 1] = sz;
      }
      if constexpr (kForm) {
        fpart[2 * p] = sfd;
        fpart[2 * p + 1] = sfz;
      }
    }
  }
}

// D-precompute spectra of the register-line state (dP:95-99, the fft2(z) of
// precompute_H_hat_D's input): for the KB filter slices k0..k0+KB-1 of patch p,
//   zhat = fft2(u - y) + XY conj(dcorr_k) w,   u = soft(a), y = a - u,
// i.e. the R2C half of k_zline (P4 elementwise, P5 x-R2C, P7 separation, P9 y-R2C)
// with the correction term added as each bin forms.  Out: natural-order half spectra
// dst[(p K + k) F + y Xh + c] (the layout the Gram kernels read).  One workgroup per
// (patch, KB slices), three barriers per slice; the stores of a wave cover 5 columns x
// 11 rows per register, merged in L2.
template <typename T, int KB>
__global__ __launch_bounds__(zl::NT) void k_zhat_line(const T* __restrict__ A,
                                                      const cpx<T>* __restrict__ W,
                                                      const cpx<T>* __restrict__ dcorr,
                                                      cpx<T>* __restrict__ dst, int K, int kgroups,
                                                      T theta) {
  using V2 = typename vec2_t<T>::type;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  cpx<T>* sT = reinterpret_cast<cpx<T>*>(smem);
  const int64_t p = blockIdx.x / kgroups;
  const int k0 = (int)(blockIdx.x - p * kgroups) * KB;
  const cpx<T>* Wp = W + p * zl::F;
  const bool xwave = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6) < 11;
  const T sc = (T)zl::P;
  for (int kk = 0; kk < KB; ++kk) {
    const int k = k0 + kk;
    if (k >= K) break;   // uniform
    const int tid = fresh((int)threadIdx.x);
    const int wave = tid >> 6, lane = tid & 63;
    const int l = min(lane / 11, 4);
    const int s = lane - 11 * l;
    const int sb = min(s, 10), sa = min(s, 9);
    const int c = min(5 * wave + l, 55);
    const int j = min(5 * wave + l, 54);
    const uint32_t Ey = (uint32_t)tcol(c) * 16u;
    const uint32_t Ex = (uint32_t)(10 * min(wave, 10) * zl::RS + l * 110) * 16u;
    const int64_t sl = (p * K + k) * zl::P;
    // (masking the duplicate lanes out, as k_zline does, slowed this kernel beside the Gram:
    // 808.0 vs 790.8 ms per C2 step, profiles/r06/zline_lane_mask_ab.txt)
    if (xwave) {
      // ---- P4/P5: c = u - y of row pair j (layout A) -> x-R2C -> rows 2j, 2j+1 of T ----
      const uint32_t po = (uint32_t)(j * 10 + fresh(sa)) * 16u;
      cpx<T> zc[11];
#pragma unroll
      for (int n2 = 0; n2 < 11; ++n2) {
        const V2 a = sld2<V2>(A + sl, po, n2 * 550 * 16);
        zc[n2] = {fma((T)-2, clamp_t(a.x, theta), a.x), fma((T)-2, clamp_t(a.y, theta), a.y)};
      }
      const int s5 = fresh(sb);
      const uint32_t r0 = (uint32_t)(kZlWR * min(wave, 10) + zoff(l) + s5) * 16u;
      fwd_line<T, 1>(zc, Ex, s5, [&](int k1, cpx<T> val) { lds_cpx_at<T>(r0 + (uint32_t)(k1 * 176)) = val; });
    }
    lds_sync();
    // ---- P7: column c, rows y = n1 + 10 n2: two-for-one separation ----
    cpx<T> col[11];
    {
      const int n1 = fresh(sa);
      const int zc1 = zslot(c), zc2 = zslot((c == 0) ? 0 : zl::X - c);
      // twice the row spectra (halved at the store); odd rows times i (undone in P9, ODDROT)
      const T sg = (n1 & 1) ? (T)-1 : (T)1;
#pragma unroll
      for (int n2 = 0; n2 < 11; ++n2) {
        // row y = (11 n1 + 10 n2) mod 110: pair y >> 1 is line n1 >> 1 of wave (n1 + n2) mod 11
        const int wv = n1 + n2 >= 11 ? n1 + n2 - 11 : n1 + n2;
        const cpx<T>* r0 = sT + kZlWR * wv + zoff(n1 >> 1);
        const cpx<T> z1 = r0[zc1], z2 = r0[zc2];
        col[n2] = {fma(sg, z2.x, z1.x), fma(-sg, z2.y, z1.y)};
      }
    }
    lds_sync();
    // ---- P9: y-R2C of column c -> bins (x' = c, y = elem_b(k2, k1)) + XY conj(dcorr) w ----
    {
      const int s9 = fresh(sb);
      const cpx<T>* dk = dcorr + (int64_t)k * zl::F;
      const uint32_t bo = (uint32_t)(c * 11 + s9) * 16u;
      cpx<T>* out = dst + (p * K + k) * (int64_t)zl::F + c;
      fwd_line<T, zl::RS, true>(col, Ey, s9, [&](int k1, cpx<T> cb) {
        const cpx<T> q = cmulc(fld<cpx<T>>(dk, bo, k1 * 616 * 16), wld<cpx<T>>(Wp, bo, k1 * 616 * 16));
        out[zl::elem_b(s9, k1) * zl::Xh] = {fma((T)0.5, cb.x, sc * q.x), fma((T)0.5, cb.y, sc * q.y)};
      });
    }
    lds_sync();   // the next slice's P5 rewrites the rows of T
  }
}

// dst[b][bin_slot(f)] = src[b][f]  (complex spectra, `count` of them)
template <typename T>
__global__ void k_to_slots(const cpx<T>* __restrict__ src, cpx<T>* __restrict__ dst,
                           int64_t count) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count * zl::F) return;
  const int64_t b = i / zl::F;
  const int f = (int)(i - b * zl::F);
  dst[b * zl::F + zl::bin_slot(f)] = src[i];
}
template <typename T>
__global__ void k_to_slots_real(const T* __restrict__ src, T* __restrict__ dst) {
  const int f = blockIdx.x * blockDim.x + threadIdx.x;
  if (f < zl::F) dst[zl::bin_slot(f)] = src[f];
}
// natural[s][e] = state[s][state_off(e)], one workgroup per slice (a flat grid over
// the 1.2e10 elements of C2 would exceed the 2^32 work-items of one dispatch)
template <typename T>
__global__ void k_state_to_nat(const T* __restrict__ st, T* __restrict__ nat) {
  const int64_t b = blockIdx.x;
  for (int e = threadIdx.x; e < zl::P; e += blockDim.x)
    nat[b * zl::P + e] = st[b * zl::P + zl::state_off(e)];
}

// in place: slice <- natural order of its state-order contents (one workgroup per
// slice; the whole slice passes through LDS, 96.8 KB)
template <typename T>
__global__ __launch_bounds__(1024) void k_state_to_nat_inplace(T* a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  T* s = reinterpret_cast<T*>(smem);
  T* sl = a + (int64_t)blockIdx.x * zl::P;
  for (int q = threadIdx.x; q < zl::P; q += 1024) s[q] = sl[q];
  __syncthreads();
  for (int e = threadIdx.x; e < zl::P; e += 1024) sl[e] = s[zl::state_off(e)];
}

bool zline_grid(const Grid2D& G) { return grid_is<Grid110>(G); }

template <typename T, int MODE, int TOL>
static void zline_go(hipStream_t st, int64_t npatch, const T* A, T* Ao, const T* Zn, const T* Yn,
                     cpx<T>* W, const cpx<T>* Bs, const cpx<T>* dcorr, const cpx<T>* dhat,
                     const T* sden, int K, T theta, T rho, T* Zt, T* zpart, T* fpart) {
  hipLaunchKernelGGL((k_zline<T, MODE, TOL>), dim3((unsigned)npatch), dim3(zl::NT), kZlSmem, st,
                     A, Ao, Zn, Yn, W, Bs, dcorr, dhat, sden, K, theta, rho, Zt, zpart, fpart);
}

template <typename T>
hipError_t launch_zline(const T* A, T* Ao, const T* Zn, const T* Yn, cpx<T>* W, const cpx<T>* Bs,
                        const cpx<T>* dcorr, const cpx<T>* dhat, const T* sden, int64_t npatch,
                        int K, T theta, T rho, int mode, hipStream_t st, int tol, T* Zt,
                        T* zpart, T* fpart) {
  if (npatch <= 0) return hipSuccess;
  if ((tol & kZtStore) && !Zt) return hipErrorInvalidValue;
  if ((tol & kZtCmp) && !zpart) return hipErrorInvalidValue;
  if ((tol & kZtForm) && (!fpart || dcorr != dhat)) return hipErrorInvalidValue;
  const int v = mode * 10 + tol;
#define ZL_GO(M, TL)                                                                          \
  zline_go<T, M, TL>(st, npatch, A, Ao, Zn, Yn, W, Bs, dcorr, dhat, sden, K, theta, rho, Zt, \
                     zpart, fpart)
  switch (v) {
    case 0: ZL_GO(0, 0); break;
    case 1: ZL_GO(0, 1); break;
    case 20: ZL_GO(2, 0); break;
    case 21: ZL_GO(2, 1); break;
    case 23: ZL_GO(2, 3); break;
    case 24: ZL_GO(2, 4); break;
    case 27: ZL_GO(2, 7); break;
    case 33: ZL_GO(3, 3); break;
    default: return hipErrorInvalidValue;
  }
#undef ZL_GO
  return hipGetLastError();
}

template <typename T>
hipError_t launch_to_slots(const cpx<T>* src, cpx<T>* dst, int64_t count, hipStream_t st) {
  if (count <= 0) return hipSuccess;
  const int64_t n = count * zl::F;
  hipLaunchKernelGGL(k_to_slots<T>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, src, dst,
                     count);
  return hipGetLastError();
}
template <typename T>
hipError_t launch_to_slots_real(const T* src, T* dst, hipStream_t st) {
  hipLaunchKernelGGL(k_to_slots_real<T>, dim3((zl::F + 255) / 256), dim3(256), 0, st, src, dst);
  return hipGetLastError();
}
template <typename T>
hipError_t launch_state_to_nat(const T* st_, T* nat, int64_t count, hipStream_t st) {
  if (count <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_state_to_nat<T>, dim3((unsigned)count), dim3(256), 0, st, st_, nat);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_state_to_nat_inplace(T* a, int64_t count, hipStream_t st) {
  if (count <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_state_to_nat_inplace<T>, dim3((unsigned)count), dim3(1024),
                     (size_t)zl::P * sizeof(T), st, a);
  return hipGetLastError();
}

size_t zline_smem_bytes() { return zl::kSmem; }

constexpr int kZhKB = 4;   // filter slices per workgroup of k_zhat_line

template <typename T>
hipError_t launch_zhat_line(const T* A, const cpx<T>* W, const cpx<T>* dcorr, cpx<T>* dst,
                            int64_t npatch, int K, T theta, hipStream_t st) {
  if (npatch <= 0) return hipSuccess;
  const int kg = (K + kZhKB - 1) / kZhKB;
  hipLaunchKernelGGL((k_zhat_line<T, kZhKB>), dim3((unsigned)(npatch * kg)), dim3(zl::NT),
                     zl::kSmem, st, A, W, dcorr, dst, K, kg, theta);
  return hipGetLastError();
}

template hipError_t launch_zline<double>(const double*, double*, const double*, const double*,
                                         cpx<double>*, const cpx<double>*, const cpx<double>*,
                                         const cpx<double>*, const double*, int64_t, int, double,
                                         double, int, hipStream_t, int, double*, double*,
                                         double*);
template hipError_t launch_zhat_line<double>(const double*, const cpx<double>*,
                                             const cpx<double>*, cpx<double>*, int64_t, int,
                                             double, hipStream_t);
template hipError_t launch_to_slots<double>(const cpx<double>*, cpx<double>*, int64_t, hipStream_t);
template hipError_t launch_to_slots_real<double>(const double*, double*, hipStream_t);
template hipError_t launch_state_to_nat<double>(const double*, double*, int64_t, hipStream_t);
template hipError_t launch_state_to_nat_inplace<double>(double*, int64_t, hipStream_t);

}  // namespace ccsc
