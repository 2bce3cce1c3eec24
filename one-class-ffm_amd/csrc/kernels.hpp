// kernels.hpp — CDNA4 (gfx950) device code of the one-class FFM epoch.
//
// Every pass of the reference epoch (ffm.cpp:314-870) is a gather / dot /
// AXPY over k-vectors, bound by HBM (or Infinity-Cache) bandwidth, not by
// MFMA.  Layout: every table (W, H, P, Q, S, V, R, Hv, h) is row-major with a
// padded row stride KP = next power of two >= k (padding columns stay exactly
// zero, so results equal the unpadded math).  One lane owns VE consecutive
// elements of a row (16 bytes: float4 / double2), so LPR = KP/VE lanes cover
// a row and a 64-lane wave holds NSG = 64/LPR "subgroups".
//
// Row kernels run one row per wave: subgroups split the row's positives
// (or feature nodes), each subgroup gathers whole 16-B-per-lane row slices,
// and cross-subgroup sums use xor shuffles.  The scatter x_i (x) h_i into the
// D x k gradient / Hessian-vector buffers is done without per-thread buffers
// (the reference's nr_threads x D x k copies, ffm.cpp:557,759): a row pass
// writes h (R x k), then a feature-major (CSC) pass sums each feature's rows
// in chunks; single-chunk features are plain stores, multi-chunk features
// (low-cardinality fields) use float atomics into a buffer that the
// finalising pass zeroes again.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

namespace ocffm {

typedef float f4v __attribute__((ext_vector_type(4)));
typedef double d2v __attribute__((ext_vector_type(2)));
typedef double d4v __attribute__((ext_vector_type(4)));

// fp64 lane width: 16 B (two doubles) or, with OCFFM_F64_WIDE, 32 B (four
// doubles, two 16-B loads): a KP = 32 row then spans 8 lanes as in fp32, so
// a wave walks 8 segments at once instead of 4.
// Default wide (round 5, fp64 kkbox epoch at 10 epochs, two alternations:
// 10.04 -> 9.50 ms; gd_cross_row 186 -> 174 us, feat_hv 1.47 -> 1.23 ms per
// epoch); -DOCFFM_F64_WIDE=0 builds the 16-B layout.
#ifndef OCFFM_F64_WIDE
#define OCFFM_F64_WIDE 1
#endif
template <typename real> struct VT;
template <> struct VT<float> {
  using V = f4v;
  static constexpr int N = 4;
};
template <> struct VT<double> {
  using V = std::conditional_t<OCFFM_F64_WIDE != 0, d4v, d2v>;
  static constexpr int N = OCFFM_F64_WIDE ? 4 : 2;
};
template <typename real> using vec_t = typename VT<real>::V;

template <typename real, int KP> struct Geo {
  static constexpr int VE = VT<real>::N;
  static constexpr int LPR = KP / VE;  // lanes per row
  static constexpr int NSG = 64 / LPR; // rows (subgroups) per wave
  static_assert(LPR >= 1 && LPR <= 64, "KP out of range");
};

constexpr int BLOCK = 256;   // 4 waves
// Minimum waves per SIMD the positive-gather row passes are compiled for
// (1 = the compiler's choice); experiment builds set them with -D.
#ifndef OCFFM_HS_OCC64
#define OCFFM_HS_OCC64 1  // the fp64 build of k_hs_cross_seg (experiment builds: -D)
#endif
#ifndef OCFFM_HS_OCC
#define OCFFM_HS_OCC 1
#endif
#ifndef OCFFM_GD_GB
#define OCFFM_GD_GB 8  // partner-row gathers per round in k_gd_cross_seg (entering a block: two gathers each)
#endif
#ifndef OCFFM_GD_GB_IN
#define OCFFM_GD_GB_IN OCFFM_GD_GB  // the same in the passes with one gather per positive
#endif
#ifndef OCFFM_HS_GB
#define OCFFM_HS_GB 32  // partner-row gathers per round in k_hs_cross_seg
#endif
#ifndef OCFFM_HS_GB64
// the same in its fp64 build (wide lanes: 8 gathers of 32 B per lane, 140
// registers / 3 waves per SIMD; 16 took 202 / 2)
#define OCFFM_HS_GB64 (OCFFM_F64_WIDE ? 8 : OCFFM_HS_GB)
#endif
#ifndef OCFFM_GD_OCC
// fp32 k_gd_cross_seg: at least 3 waves per SIMD (with the MFMA T tile the
// entering pass came out at 172 + 4 registers, 2 waves; bounded: 166, no spill)
#define OCFFM_GD_OCC 3
#endif
#ifndef OCFFM_GD_OCC_IN
#define OCFFM_GD_OCC_IN OCFFM_GD_OCC  // the fp32 passes with one gather per positive (BM_IN, BM_FULL)
#endif
#ifndef OCFFM_GD_OCC64
// the fp64 build of k_gd_cross_seg: wide lanes bounded to 3 waves per SIMD
// (the entering pass: 167 registers), else the compiler's choice
#define OCFFM_GD_OCC64 (OCFFM_F64_WIDE ? 3 : 1)
#endif
#ifndef OCFFM_GD_GB64
// fp64: 4 gathers per round (3 / 4 waves per SIMD instead of 2 / 3; the
// fp64 kkbox epoch's gd_cross_row 206 -> 200 us per launch, 2 is no faster)
#define OCFFM_GD_GB64 4
#endif
constexpr int MAXCG = 20;    // ffm.cpp:761
constexpr double CG_EPS = 9e-2;  // ffm.cpp:762

// One subgroup's share of a feature pass over the feature-major (CSC) view
// of a field.  A column with <= JOB_ENT entries is one "light" job, finished
// by its subgroup.  A heavier column is cut into wave-chunks of NSG jobs
// (one wave, JOB_ENT entries per subgroup) summed across the wave; a column
// of several wave-chunks is summed by the last chunk to arrive, from the
// partial slots in chunk order (deterministic, no float atomics).
// Every subgroup issues its JOB_ENT row loads at once: one latency round.
struct Job {
  uint32_t col;     // JOB_NONE: padding
  uint32_t nparts;  // wave-chunks of the column (wave jobs), else 1
  uint32_t slot;    // wave jobs: partial slot of this wave-chunk
  uint32_t flags;   // bit 0: wave job; bits 1..: wave-chunk index in the column
  int64_t b, e;
};
constexpr uint32_t JOB_NONE = 0xffffffffu;
constexpr int JOB_ENT = 8;  // entries per job (JE) of fields with multi-entry columns; unit fields use 1

// A run of one row's positives [b, e): rows with many positives (popular
// items: the Pareto head holds ~all users) are split so that no wave walks
// tens of thousands of positives alone.  `first` marks the segment that also
// carries the row-local terms.  Row kernels write one partial per segment;
// the CSC pass sums a row's segments in order (deterministic, no atomics).
struct Seg {
  uint32_t row;
  uint32_t info;  // bit 0: first segment of the row; bits 1..: segments of the row
  int64_t b, e;
};
__device__ __forceinline__ bool seg_first(const Seg &s) { return s.info & 1u; }
__device__ __forceinline__ unsigned seg_nrow(const Seg &s) { return s.info >> 1; }

// Device-resident CG scalars (the host never reads them on the hot path).
struct CgState {
  double g2, r2, alpha, beta, vhv;
  int run[MAXCG + 2];  // run[it]: CG iteration `it` (1-based) executes
  int nr_cg;
  double scal[4];      // misc scalars (sum of a partner bias, ...)
};

template <typename real> __device__ __forceinline__ vec_t<real> vld(const real *p) {
  return *reinterpret_cast<const vec_t<real> *>(p);
}
// The same through a pointer that was itself read from memory (a table of
// tables): the cast to the global address space keeps the load a global_load
// (a flat load would make every wait also drain the LDS counter).
template <typename real> __device__ __forceinline__ vec_t<real> gvld(const real *p) {
  typedef const __attribute__((address_space(1))) vec_t<real> gvec;
  return *(gvec *)p;
}
// Stores of pass outputs.  OCFFM_NT_STORES=1 at build time makes them
// non-temporal (global_store ... nt): the bytes stream out instead of
// sitting dirty in the XCD's L2 until the kernel-end write-back, which the
// next (dependent) dispatch waits for.
#ifndef OCFFM_NT_STORES
#define OCFFM_NT_STORES 0
#endif
template <typename real> __device__ __forceinline__ void vst(real *p, vec_t<real> v) {
  if constexpr (OCFFM_NT_STORES) __builtin_nontemporal_store(v, reinterpret_cast<vec_t<real> *>(p));
  else *reinterpret_cast<vec_t<real> *>(p) = v;
}
template <typename real> __device__ __forceinline__ vec_t<real> vzero() {
  vec_t<real> v;
#pragma unroll
  for (int e = 0; e < VT<real>::N; e++) v[e] = (real)0;
  return v;
}
template <typename real> __device__ __forceinline__ real hsum(vec_t<real> v) {
  real s = v[0];
#pragma unroll
  for (int e = 1; e < VT<real>::N; e++) s += v[e];
  return s;
}
template <typename real> __device__ __forceinline__ vec_t<real> vsplat(real x) {
  vec_t<real> v;
#pragma unroll
  for (int e = 0; e < VT<real>::N; e++) v[e] = x;
  return v;
}

// ------------------------------------------------------ lane exchange ---
// DPP lane moves run on the VALU (no LDS-pipe ds_bpermute).  Controls:
// quad_perm 0x00-0xff, row_shl:n 0x100+n, row_shr:n 0x110+n,
// row_mirror 0x140, row_half_mirror 0x141, row_newbcast:n 0x150+n (gfx950).
template <int CTRL> __device__ __forceinline__ uint32_t dpp32(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, 0xF, 0xF, false);
}
struct W2 {
  uint32_t lo, hi;
};
template <int CTRL, typename T> __device__ __forceinline__ T dpp(T x) {
  static_assert(sizeof(T) == 4 || sizeof(T) == 8, "dpp: 32/64-bit values");
  if constexpr (sizeof(T) == 4) {
    return __builtin_bit_cast(T, dpp32<CTRL>(__builtin_bit_cast(uint32_t, x)));
  } else {
    W2 w = __builtin_bit_cast(W2, x);
    w.lo = dpp32<CTRL>(w.lo);
    w.hi = dpp32<CTRL>(w.hi);
    return __builtin_bit_cast(T, w);
  }
}

// Sum over the LPR lanes of one subgroup (all of them active together).
// Every lane ends with the same bits (each step adds a commuted pair).
template <int LPR, typename T> __device__ __forceinline__ T sg_sum(T x) {
  if constexpr (LPR >= 2) x += dpp<0xB1>(x);   // quad_perm [1,0,3,2]: xor 1
  if constexpr (LPR >= 4) x += dpp<0x4E>(x);   // quad_perm [2,3,0,1]: xor 2
  if constexpr (LPR >= 8) x += dpp<0x141>(x);  // half-row mirror: the other quad
  if constexpr (LPR >= 16) x += dpp<0x140>(x); // row mirror: the other half-row
  if constexpr (LPR >= 32) x += __shfl_xor(x, 16, 64);
  if constexpr (LPR >= 64) x += __shfl_xor(x, 32, 64);
  return x;
}

// Value of lane SRC of the caller's LPR-lane subgroup, in every lane of it.
template <int LPR, int SRC, typename T> __device__ __forceinline__ T sg_bcast(T x, int li) {
  if constexpr (LPR == 1) {
    return x;
  } else if constexpr (LPR == 2) {
    return dpp<(SRC | SRC << 2 | (2 + SRC) << 4 | (2 + SRC) << 6)>(x);
  } else if constexpr (LPR == 4) {
    return dpp<SRC * 0x55>(x);
  } else if constexpr (LPR == 8) {
    const T a = dpp<(SRC % 4) * 0x55>(x);  // lane SRC%4 of each quad
    if constexpr (SRC < 4) {
      const T b = dpp<0x114>(a);  // row_shr:4: the upper quad takes the lower one's
      return (li & 4) ? b : a;
    } else {
      const T b = dpp<0x104>(a);  // row_shl:4: the lower quad takes the upper one's
      return (li & 4) ? a : b;
    }
  } else if constexpr (LPR == 16) {
    return dpp<0x150 + SRC>(x);  // row_newbcast: lane SRC of each 16-lane row (no LDS-pipe bpermute)
  } else {
    return __shfl(x, (int)((threadIdx.x & 63) & ~(LPR - 1)) + SRC, 64);
  }
}

template <int... I> struct iseq {};
template <int N, int... I> struct make_iseq : make_iseq<N - 1, N - 1, I...> {};
template <int... I> struct make_iseq<0, I...> {
  using type = iseq<I...>;
};
template <typename F, int... I> __device__ __forceinline__ void sfor_impl(F &&f, iseq<I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
// Compile-time unrolled loop: f(integral_constant<int, 0..N-1>).
template <int N, typename F> __device__ __forceinline__ void sfor(F &&f) {
  sfor_impl(f, typename make_iseq<N>::type{});
}

// x M for a k-vector x spread over the subgroup (lane l holds components
// l*VE ..) and a KP x KP row-major M (LDS or global): component e of x is
// broadcast from its lane by DPP, M's row e read as one vector per lane.
template <typename real, int KP>
__device__ __forceinline__ vec_t<real> sg_vecmat(const vec_t<real> &x, const real *M, int li);

// Raw-buffer view of a table for gathers.  A load at an out-of-range offset
// returns zero without a memory access (the buffer range check), so the
// unused slots of a fixed-width gather need neither a branch nor a wait:
// all of a subgroup's loads go out in one round.  Tables < 4 GiB (host-checked).
struct BufView {
  __amdgpu_buffer_rsrc_t r;
  uint32_t oob;  // an offset past the end
};
__device__ __forceinline__ BufView buf_view(const void *p, uint64_t bytes) {
  return BufView{__builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), (short)0, (int)(uint32_t)bytes, 0x00020000),
                 (uint32_t)bytes};
}
template <typename real> __device__ __forceinline__ vec_t<real> bld(const BufView &b, uint32_t off) {
  if constexpr (sizeof(vec_t<real>) == 16) {
    return __builtin_bit_cast(vec_t<real>, __builtin_amdgcn_raw_buffer_load_b128(b.r, off, 0, 0));
  } else {  // a 32-B lane: two 16-B loads (an out-of-range offset reads zero for both)
    const d2v lo = __builtin_bit_cast(d2v, __builtin_amdgcn_raw_buffer_load_b128(b.r, off, 0, 0));
    const d2v hi = __builtin_bit_cast(d2v, __builtin_amdgcn_raw_buffer_load_b128(b.r, off == b.oob ? off : off + 16u, 0, 0));
    return vec_t<real>{lo[0], lo[1], hi[0], hi[1]};
  }
}
// the same with the sc1 bit (aux 16: the last-arriver hand-off's loads)
template <typename real> __device__ __forceinline__ vec_t<real> bld_sc1(const BufView &b, uint32_t off) {
  if constexpr (sizeof(vec_t<real>) == 16) {
    return __builtin_bit_cast(vec_t<real>, __builtin_amdgcn_raw_buffer_load_b128(b.r, off, 0, 16));
  } else {
    const d2v lo = __builtin_bit_cast(d2v, __builtin_amdgcn_raw_buffer_load_b128(b.r, off, 0, 16));
    const d2v hi = __builtin_bit_cast(d2v, __builtin_amdgcn_raw_buffer_load_b128(b.r, off == b.oob ? off : off + 16u, 0, 16));
    return vec_t<real>{lo[0], lo[1], hi[0], hi[1]};
  }
}
// bytes of one lane's share of a row (16, or 32 for wide fp64 lanes)
template <typename real> constexpr uint32_t LANE_B = (uint32_t)sizeof(vec_t<real>);
template <typename real> __device__ __forceinline__ real bld1(const BufView &b, uint32_t off);
template <> __device__ __forceinline__ float bld1<float>(const BufView &b, uint32_t off) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(b.r, off, 0, 0));
}
template <> __device__ __forceinline__ double bld1<double>(const BufView &b, uint32_t off) {
  return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(b.r, off, 0, 0));
}

template <typename real, int KP>
__device__ __forceinline__ vec_t<real> sg_vecmat(const vec_t<real> &x, const real *M, int li) {
  using G = Geo<real, KP>;
  vec_t<real> t = vzero<real>();
  sfor<KP>([&](auto E) {
    constexpr int e = decltype(E)::value;
    const real xe = sg_bcast<G::LPR, e / G::VE>(x[e % G::VE], li);
    t += vsplat<real>(xe) * vld<real>(M + (size_t)e * KP + li * G::VE);
  });
  return t;
}

// The same product as a rolled loop (a lane-index shuffle per component, a
// few rows of M in flight): for a path that runs rarely inside a kernel
// whose register budget belongs to another path (k_hs_cross_seg's hot rows).
// UNR: iterations in flight (VE rows of M each); 0 = the default for the
// hot rows of k_hs_cross_seg (2 at KP <= 32, else 1: that kernel's 4
// waves/SIMD register budget)
template <typename real, int KP, int UNR_ = 0>
__device__ __forceinline__ vec_t<real> sg_vecmat_rolled(const vec_t<real> &x, const real *M, int li) {
  using G = Geo<real, KP>;
  const int base = (int)(threadIdx.x & 63) & ~(G::LPR - 1);
  vec_t<real> t = vzero<real>();
  constexpr int UNR = UNR_ > 0 ? UNR_ : (KP <= 32 ? 2 : 1);
#pragma unroll UNR
  for (int l = 0; l < G::LPR; l++) {
#pragma unroll
    for (int c = 0; c < G::VE; c++) {
      const real xe = __shfl(x[c], base + l, 64);
      t += vsplat<real>(xe) * vld<real>(M + (size_t)(l * G::VE + c) * KP + li * G::VE);
    }
  }
  return t;
}

// Lane-local vector-matrix accumulation for t = x M summed over several M
// (fp32): lane li holds rows r = li*4 + e of x, so it adds x[e] * M[r][n] for
// ALL n into u (no cross-lane broadcast per element), column pairs in packed
// FMAs.  Mt is M in pair-transposed order, Mt[(n/2)*2KP + 2r + n%2] = M[r][n]:
// per column pair two conflict-free 16-B reads.  The subgroup sums u once at
// the end with sg_reduce_scatter.
typedef float f2v __attribute__((ext_vector_type(2)));
template <int KP>
__device__ __forceinline__ void lane_vecmat_acc(f2v (&u)[KP / 2], const f4v &x, const float *Mt, int li) {
  const f2v x0 = {x[0], x[0]}, x1 = {x[1], x[1]}, x2 = {x[2], x[2]}, x3 = {x[3], x[3]};
#pragma unroll
  for (int q = 0; q < KP / 2; q++) {
    const f4v a = *reinterpret_cast<const f4v *>(Mt + q * 2 * KP + li * 8);
    const f4v b = *reinterpret_cast<const f4v *>(Mt + q * 2 * KP + li * 8 + 4);
    f2v s = u[q];
    s += x0 * f2v{a[0], a[1]};
    s += x1 * f2v{a[2], a[3]};
    s += x2 * f2v{b[0], b[1]};
    s += x3 * f2v{b[2], b[3]};
    u[q] = s;
  }
}
__device__ __forceinline__ int mt_index(int KP, int r, int n) { return (n >> 1) * 2 * KP + 2 * r + (n & 1); }
// Subgroup reduce-scatter of u[KP]: lane li returns sum over the LPR lanes of
// u[li*VE .. li*VE+VE-1] (halving exchanges, highest lane bit first).
template <typename real, int KP>
__device__ __forceinline__ vec_t<real> sg_reduce_scatter(real (&u)[KP], int li) {
  using G = Geo<real, KP>;
  sfor<6>([&](auto S) {  // stages o = LPR/2, ..., 1 (S indexes the stage)
    constexpr int o = (G::LPR >> 1) >> decltype(S)::value;
    if constexpr (o >= 1) {
      constexpr int H = (KP * o) / G::LPR;  // elements kept after this stage
      const bool up = li & o;
#pragma unroll
      for (int m = 0; m < H; m++) {
        const real send = up ? u[m] : u[m + H];
        const real keep = up ? u[m + H] : u[m];
        u[m] = keep + __shfl_xor(send, o, 64);
      }
    }
  });
  vec_t<real> t;
#pragma unroll
  for (int e = 0; e < G::VE; e++) t[e] = u[e];
  return t;
}

// A pass over up to PW positions [p0, p0+PW) of a positive segment, spread
// over the LPR lanes of the subgroup: lane li holds the column (ycol) of
// positions p0 + li + t*LPR, t < UT, loaded in one round; position `pos`
// of the pass is then read from lane pos % LPR, slot pos / LPR.  Gathers of
// partner rows go out GB at a time through a BufView (absent positions load
// zero rows), so a 32-position segment costs 1 + 32/GB latency rounds
// instead of one per position.
constexpr uint32_t POS_NONE = 0xffffffffu;
template <typename real, int KP, int GB_ = 8, int PW_ = 32> struct PosPass {
  using G = Geo<real, KP>;
  // positions per pass (PW_: 32, or 16 for sides whose segments are short)
  static constexpr int PW = G::LPR > PW_ ? G::LPR : PW_;
  static constexpr int UT = PW / G::LPR;
  static constexpr int GB = GB_ < PW ? GB_ : PW;  // gathers per round
  static constexpr uint32_t ROWB = KP * sizeof(real);
  template <int POS, typename T> static __device__ __forceinline__ T at(const T (&v)[UT], int li) {
    return sg_bcast<G::LPR, POS % G::LPR>(v[POS / G::LPR], li);
  }
  static __device__ __forceinline__ void load_cols(const uint32_t *__restrict__ ycol, int64_t p0, int64_t e, int li,
                                                   uint32_t (&jj)[UT]) {
#pragma unroll
    for (int t = 0; t < UT; t++) {
      const int64_t q = p0 + li + t * G::LPR;
      jj[t] = q < e ? ycol[q] : POS_NONE;
    }
  }
  static __device__ __forceinline__ uint32_t row_off(uint32_t j, const BufView &b, int li) {
    return j == POS_NONE ? b.oob : j * ROWB + (uint32_t)li * LANE_B<real>;
  }
};

// Sum over the NSG subgroups of a wave (lane-wise, whole wave active).
template <int LPR, typename T> __device__ __forceinline__ T xsg_sum(T x) {
#pragma unroll
  for (int o = LPR; o < 64; o <<= 1) x += __shfl_xor(x, o, 64);
  return x;
}
template <int LPR, typename real> __device__ __forceinline__ vec_t<real> xsg_vsum(vec_t<real> v) {
#pragma unroll
  for (int e = 0; e < VT<real>::N; e++) v[e] = xsg_sum<LPR>(v[e]);
  return v;
}

__device__ __forceinline__ double wave_sum(double x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
  return x;
}

// Deterministic block sum (fixed tree), result valid in every thread.
__device__ __forceinline__ double block_sum(double v) {
  __shared__ double sh[BLOCK / 64];
  v = wave_sum(v);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) sh[w] = v;
  __syncthreads();
  double t = 0;
#pragma unroll
  for (int i = 0; i < BLOCK / 64; i++) t += sh[i];
  return t;
}

// Cross-block reduction by the last-arriving block.  Hand-off per the
// MI355X guide's measured-valid form: partials written with agent-scope
// (sc1) stores, the writing wave drains vmcnt, one agent-scope atomic add per
// block; the block whose add returns gridDim-1 reads every partial with sc1
// loads after a workgroup barrier.  No L2 write-back fence is needed.
// Partials are summed in block order: deterministic for a fixed grid.
// Grid-wide "last block" election for deterministic reductions.  Each
// block stores its NV partials (sc1), drains, and takes a ticket; the block
// that completes the grid reads every partial back (sc1) and sums them in
// block order.  Tickets go through TICK_SUB sub-counters (block % TICK_SUB,
// 256 B apart) whose last arrivals take a ticket on the top counter: one
// address serialises ~10 ns per same-address atomic, so a flat counter
// costs ~30 us for 3000 blocks.  tick: TICK_WORDS zeroed words, zero at rest.
constexpr int TICK_SUB = 32;
constexpr int TICK_STRIDE = 64;  // words
constexpr int TICK_WORDS = (TICK_SUB + 1) * TICK_STRIDE;
// extra (optional): nextra x NV more values, stored by waves of any block
// before their block's ticket (sc1 stores, drained), added to the total in
// index order by the last block.
template <int NV, int ROUND = 8>  // ROUND: blocks per thread per read-back round (registers: 2 ROUND NV)
__device__ __forceinline__ bool last_block(const double (&v)[NV], double *part, unsigned *tick, double (&tot)[NV],
                                           const double *extra = nullptr, uint32_t nextra = 0) {
  __shared__ int s_last;
  if (threadIdx.x == 0) {
#pragma unroll
    for (int k = 0; k < NV; k++)
      __hip_atomic_store(&part[(size_t)blockIdx.x * NV + k], v[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned g = blockIdx.x % TICK_SUB;
    const unsigned members = (gridDim.x - g + TICK_SUB - 1) / TICK_SUB;
    unsigned *sub = tick + (1 + g) * TICK_STRIDE;
    int last = 0;
    if (__hip_atomic_fetch_add(sub, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == members - 1) {
      __hip_atomic_store(sub, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      // the reset lands before the top ticket (a persistent grid's next
      // round takes tickets on the same words right after the release)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const unsigned groups = gridDim.x < (unsigned)TICK_SUB ? gridDim.x : (unsigned)TICK_SUB;
      last = __hip_atomic_fetch_add(tick, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == groups - 1;
    }
    s_last = last;
  }
  __syncthreads();
  if (!s_last) return false;
  // All partials in one round: sc1 buffer loads (aux 16), out-of-range
  // slots read zero; fixed summation order (thread, then round, then tree).
  const BufView pv = buf_view(part, (uint64_t)gridDim.x * NV * sizeof(double));
  double x[NV];
#pragma unroll
  for (int k = 0; k < NV; k++) x[k] = 0;
  for (unsigned b0 = 0; b0 < gridDim.x; b0 += ROUND * BLOCK) {
    double y[ROUND][NV];
#pragma unroll
    for (int u = 0; u < ROUND; u++)
#pragma unroll
      for (int k = 0; k < NV; k++) {
        const unsigned b = b0 + u * BLOCK + threadIdx.x;
        y[u][k] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(
                                                 pv.r, b < gridDim.x ? (b * NV + k) * 8u : pv.oob, 0, 16));
      }
#pragma unroll
    for (int u = 0; u < ROUND; u++)
#pragma unroll
      for (int k = 0; k < NV; k++) x[k] += y[u][k];
  }
  if (nextra) {  // the extra slots: all rounds' loads in flight, then added in
                 // a fixed order (thread, round) before the one block tree.
                 // (One dependent round per BLOCK slots had cost feature passes
                 // with ~1,000 heavy-column slots ~3 us each.)
    const BufView ev = buf_view(extra, (uint64_t)nextra * NV * sizeof(double));
    constexpr int ER = 8;
    for (uint32_t q0 = 0; q0 < nextra; q0 += ER * BLOCK) {
      double z[ER][NV];
#pragma unroll
      for (int u = 0; u < ER; u++)
#pragma unroll
        for (int k = 0; k < NV; k++) {
          const uint32_t q = q0 + u * BLOCK + threadIdx.x;
          z[u][k] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(
                                                   ev.r, q < nextra ? (q * NV + k) * 8u : ev.oob, 0, 16));
        }
#pragma unroll
      for (int u = 0; u < ER; u++)
#pragma unroll
        for (int k = 0; k < NV; k++) x[k] += z[u][k];
    }
  }
#pragma unroll
  for (int k = 0; k < NV; k++) tot[k] = block_sum(x[k]);
  if (threadIdx.x == 0) __hip_atomic_store(tick, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return true;
}

// XCD-aware block order (round 6).  Workgroups are dealt round-robin over
// the 8 XCDs (blocks b and b + 8 share one, MI355X guide §Workgroup
// dispatch), so the ngroups blocks of one row chunk — which all read that
// chunk's B rows — landed on different XCDs and each XCD's L2 fetched B
// again (config 5: 105.8 GB fetched per launch against 65.3 GB of tables).
// With the grid a multiple of 8, work item L = (b % 8) * (grid / 8) + b / 8
// gives each XCD a contiguous run of work items, so the blocks of a chunk
// run on one XCD back to back and B is fetched into one L2 once.  Work items
// past nwork (the padding) exit.
__device__ __forceinline__ unsigned xcd_work_item(unsigned b, unsigned grid) {
  return (b & 7u) * (grid >> 3) + (b >> 3);
}

#define WAVE_SETUP                                                                  \
  const int lane = threadIdx.x & 63;                                                \
  const uint64_t wave = ((uint64_t)blockIdx.x * BLOCK + threadIdx.x) >> 6;          \
  const uint64_t nwaves = ((uint64_t)gridDim.x * BLOCK) >> 6;                       \
  (void)lane;                                                                       \
  (void)nwaves;

// CG direction of iteration `it` at feature row d.  The gradient pass stores
// p_1 = r_0.  The vector update of iteration it-1 (S += a p, r -= a Hp,
// ffm.cpp:806-807) is applied lazily by the feature pass of iteration it,
// which owns row d, and every reader of p_it forms it on the fly:
//   p_it = (r - a_{it-1} Hp_{it-1}) + b_{it-1} p_{it-1}   (ffm.cpp:810-811)
// with b from |r - a Hp|^2 = r2 - 2a<r,Hp> + a^2|Hp|^2 (same reduction pass).
template <typename real, int KP>
__device__ __forceinline__ vec_t<real> cg_dir_at(const real *__restrict__ P, const real *__restrict__ Rv,
                                                 const real *__restrict__ Hv, real alpha, real beta, bool upd,
                                                 size_t off) {
  // upd is uniform over a launch: the three loads go out together, or only
  // the p row (the first CG step).  (Round 5: forming p_it once per step in
  // its own pass, so that the row passes read one row per node reference,
  // measured a net loss on every shape: the ~4.5 us launch outweighed what
  // hs_cross / hs_side saved, ~2-5 us per launch even at outbrain's three
  // nodes per ~1-positive row.)
  if (!upd) return vld<real>(P + off);
  const vec_t<real> p = vld<real>(P + off), r = vld<real>(Rv + off), hp = vld<real>(Hv + off);
  return (r - vsplat<real>(alpha) * hp) + vsplat<real>(beta) * p;
}


// ------------------------------------------------ column finalisation ---
// Arguments of the finalisation of a D x k gradient / Hessian-vector column.
template <typename real> struct Fin {
  const real *fw;  // per-feature frequency (--freq) or null
  double lam;
  const real *W;   // gradient mode: the table being solved
  real *G;         // gradient mode: G (debug copy) or null
  real *S, *P, *R, *Hp;
  real *acc;       // zero at rest; partial sums of multi-part columns
  unsigned *cnt;   // zero at rest; arrival tickets of multi-part columns
  CgState *st;
  double *part;
  unsigned *tick;  // last_block tickets (TICK_WORDS, zero at rest)
  int *run_host;
  int it;          // CG iteration (Hessian-vector mode)
  double *dots;    // non-null: the grid's dot products are this rank's partials;
                   // the last block stores them here for a cross-rank sum and
                   // k_cg_step publishes the CG scalars (owned fields)
  // column tau (k_feat<..., TAU>): the w phi_i QTQ term of hs_cross for a
  // one-node-per-row field, summed per column: w (sum_{i in col} x_i^2) p QTQ
  const real *xsq;  // per column: sum of x^2 over its rows
  double tw;        // w
  // Dot-product contributions of the columns a feature pass finalises in a
  // last-arriving chunk (heavy columns, k_feat): one slot of 3 doubles per
  // column (at its first chunk slot), summed by the grid's last block in
  // slot order.  Which block finalises such a column depends on arrival
  // order, so its terms must not enter that block's partial: the grid sum
  // would then associate differently from run to run.  nhd: slots (0: none).
  double *hdots;
  uint32_t nhd;
  // Exact residual (fp64 parity mode, OCFFM_EXACT_R2): the finalisation
  // publishes alpha only; k_cg_r2 then reduces |r - alpha Hp|^2 as a second
  // pass, as ffm.cpp:807-808 recomputes |R|^2 after R -= alpha Hv, and
  // publishes beta and the verdict.
  int exact_r2;
};

// MODE 0 (gradient, ffm.cpp:561-570, 773-779): G = lam f W + s; r = -G;
//   p = r; S = 0; ds[0] += |G|^2.
// MODE 1 (Hessian-vector, ffm.cpp:783-809): apply iteration it-1's update
//   (S += a p, r -= a Hp, p = r + b p), then Hp = lam f p + s;
//   ds += (<p,Hp>, <r,Hp>, |Hp|^2).
// The operands a column's finalisation reads (fin_load) do not depend on
// the column sum, so a kernel can issue them before its gather.
template <typename real> struct FinOps {
  vec_t<real> w_or_p, r, hp, s;
  real reg;
};
template <typename real, int KP, int MODE>
__device__ __forceinline__ FinOps<real> fin_load(const Fin<real> &f, uint32_t col, bool upd, int li) {
  using G = Geo<real, KP>;
  const size_t off = (size_t)col * KP + li * G::VE;
  FinOps<real> o;
  o.reg = (real)(f.fw ? f.lam * (double)f.fw[col] : f.lam);
  if (MODE == 0) {
    o.w_or_p = vld<real>(f.W + off);
  } else {
    o.w_or_p = vld<real>(f.P + off);
    o.r = vld<real>(f.R + off);
    if (upd) {
      o.hp = vld<real>(f.Hp + off);
      o.s = vld<real>(f.S + off);
    }
  }
  return o;
}
template <typename real, int KP, int MODE, bool TAU = false>
__device__ __forceinline__ void col_finalize(const Fin<real> &f, uint32_t col, vec_t<real> s, real alpha, real beta,
                                             bool upd, int li, double (&ds)[3], const FinOps<real> &o,
                                             const real *tq = nullptr) {
  using G = Geo<real, KP>;
  const size_t off = (size_t)col * KP + li * G::VE;
  if (MODE == 0) {
    const vec_t<real> g = vsplat<real>(o.reg) * o.w_or_p + s;
    if (f.G) vst<real>(f.G + off, g);
    vst<real>(f.R + off, -g);
    vst<real>(f.P + off, -g);
    vst<real>(f.S + off, vzero<real>());
#pragma unroll
    for (int e = 0; e < G::VE; e++) ds[0] += (double)g[e] * (double)g[e];
  } else {
    vec_t<real> rn = o.r, pe = o.w_or_p;
    if (upd) {
      rn = o.r - vsplat<real>(alpha) * o.hp;
      pe = rn + vsplat<real>(beta) * o.w_or_p;
      vst<real>(f.S + off, o.s + vsplat<real>(alpha) * o.w_or_p);
      vst<real>(f.R + off, rn);
      vst<real>(f.P + off, pe);
    }
    if constexpr (TAU) s += vsplat<real>((real)(f.tw * (double)f.xsq[col])) * sg_vecmat<real, KP>(pe, tq, li);
    const vec_t<real> hp = vsplat<real>(o.reg) * pe + s;
    vst<real>(f.Hp + off, hp);
#pragma unroll
    for (int e = 0; e < G::VE; e++) {
      ds[0] += (double)pe[e] * (double)hp[e];
      ds[1] += (double)rn[e] * (double)hp[e];
      ds[2] += (double)hp[e] * (double)hp[e];
    }
  }
}
template <typename real, int KP, int MODE>
__device__ __forceinline__ void col_finalize(const Fin<real> &f, uint32_t col, vec_t<real> s, real alpha, real beta,
                                             bool upd, int li, double (&ds)[3]) {
  col_finalize<real, KP, MODE>(f, col, s, alpha, beta, upd, li, ds, fin_load<real, KP, MODE>(f, col, upd, li));
}

// Grid-wide end of a finalising kernel.  MODE 0 publishes g2 and the first
// CG verdict; MODE 1 computes alpha = r2/<p,Hp>, the new r2 (expanded),
// beta and the verdict for iteration it+1 (ffm.cpp:780, 803-809).
// The host copy of a verdict (run_host, host-mapped, polled by the host; it
// clears the words before each half) is RUN_GO or RUN_STOP, never 0.
constexpr int RUN_GO = 1, RUN_STOP = 2;
template <typename real, int MODE>
__device__ __forceinline__ void cg_publish(const Fin<real> &f, const double (&tot)[3]) {
  CgState *st = f.st;
  if (MODE == 0) {
    st->g2 = tot[0];
    st->r2 = tot[0];
    st->nr_cg = 0;
    for (int i = 0; i <= MAXCG + 1; i++) st->run[i] = 0;
    const int go = (tot[0] * CG_EPS < tot[0]) ? 1 : 0;
    st->run[1] = go;
    if (f.run_host) __hip_atomic_store(f.run_host + 1, go ? RUN_GO : RUN_STOP, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  } else {
    const double r2 = st->r2;
    const double alpha = r2 / tot[0];
    st->vhv = tot[0];
    st->alpha = alpha;
    if (f.exact_r2) {  // beta, r2 and the verdict: k_cg_r2
      st->nr_cg = f.it;
      return;
    }
    const double r2n = r2 - 2 * alpha * tot[1] + alpha * alpha * tot[2];
    st->beta = r2n / r2;
    st->r2 = r2n;
    st->nr_cg = f.it;
    const int go = (f.it < MAXCG && st->g2 * CG_EPS < r2n) ? 1 : 0;
    st->run[f.it + 1] = go;
    if (f.run_host)
      __hip_atomic_store(f.run_host + f.it + 1, go ? RUN_GO : RUN_STOP, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

template <typename real, int MODE>
__device__ __forceinline__ void fin_blocks(const Fin<real> &f, const double (&ds)[3]) {
  double bv[3] = {block_sum(ds[0]), block_sum(ds[1]), block_sum(ds[2])}, tot[3];
  if (last_block<3>(bv, f.part, f.tick, tot, f.hdots, f.nhd) && threadIdx.x == 0) {
    if (f.dots) {
#pragma unroll
      for (int k = 0; k < 3; k++) f.dots[k] = tot[k];
    } else {
      cg_publish<real, MODE>(f, tot);
    }
  }
}

// CG scalars of an owned-field feature pass once its partial dot products
// have been summed over the ranks: one thread.
template <typename real, int MODE>
__global__ void k_cg_step(Fin<real> f) {
  if (MODE == 1 && !f.st->run[f.it]) return;
  const double tot[3] = {f.dots[0], f.dots[1], f.dots[2]};
  cg_publish<real, MODE>(f, tot);
}

// ------------------------------------------------------------------ UTX ---
// out_i = sum_{x in X_i} val * A[idx]  (ffm.cpp:314-331).  One row per subgroup.
template <typename real, int KP>
__global__ __launch_bounds__(BLOCK) void k_utx(uint64_t R, const int64_t *__restrict__ xptr,
                                               const uint32_t *__restrict__ xidx, const real *__restrict__ xval,
                                               const real *__restrict__ A, real *__restrict__ out) {
  using G = Geo<real, KP>;
  WAVE_SETUP
  const int sg = lane / G::LPR, li = lane % G::LPR;
  for (uint64_t i = wave * G::NSG + sg; i < R; i += nwaves * G::NSG) {
    vec_t<real> acc = vzero<real>();
    for (int64_t p = xptr[i]; p < xptr[i + 1]; p++)
      acc += vsplat<real>(xval[p]) * vld<real>(A + (size_t)xidx[p] * KP + li * G::VE);
    vst<real>(out + i * KP + li * G::VE, acc);
  }
}

// acc_i += <P_i, Q_i>  (add_side, ffm.cpp:352-358).  One row per subgroup.
template <typename real, int KP>
__global__ __launch_bounds__(BLOCK) void k_rowdot_add(uint64_t R, const real *__restrict__ P,
                                                      const real *__restrict__ Q, real *__restrict__ acc) {
  using G = Geo<real, KP>;
  WAVE_SETUP
  const int sg = lane / G::LPR, li = lane % G::LPR;
  for (uint64_t i = wave * G::NSG + sg; i < R; i += nwaves * G::NSG) {
    const real d = sg_sum<G::LPR>(hsum<real>(vld<real>(P + i * KP + li * G::VE) * vld<real>(Q + i * KP + li * G::VE)));
    if (li == 0) acc[i] += d;
  }
}

// out_i = sum_c <T_c[i], v_c>  (sa / sb of cache_sasb, ffm.cpp:514-535).
template <typename real, int KP>
__global__ __launch_bounds__(BLOCK) void k_rowdot_multi(uint64_t R, int C, const real *const *__restrict__ tabs,
                                                        const double *__restrict__ vecs, real *__restrict__ out) {
  using G = Geo<real, KP>;
  WAVE_SETUP
  const int sg = lane / G::LPR, li = lane % G::LPR;
  for (uint64_t i = wave * G::NSG + sg; i < R; i += nwaves * G::NSG) {
    real s = 0;
    for (int c = 0; c < C; c++) {
      const vec_t<real> t = gvld<real>(tabs[c] + i * KP + li * G::VE);
      vec_t<real> v;
#pragma unroll
      for (int e = 0; e < G::VE; e++) v[e] = (real)vecs[(size_t)c * KP + li * G::VE + e];
      s += sg_sum<G::LPR>(hsum<real>(t * v));
    }
    if (li == 0) out[i] = s;
  }
}

// y~ is kept factored: the reference maintains y~_ij = a_i + b_j +
// sum_c <P_c[i], Q_c[j]> - 1 incrementally (init_y_tilde / update_side /
// update_cross, ffm.cpp:388-465), so only base_ij = sum_c <P_c[i],Q_c[j]> - 1
// is stored (both orientations) and readers add a_i + b_j.  Side updates then
// touch no positive at all.  This kernel writes the initial base for every
// positive (ffm.cpp:388-403).  One row per wave.
template <typename real, int KP>
__global__ __launch_bounds__(BLOCK) void k_init_ytilde(uint64_t R, const int64_t *__restrict__ yptr,
                                                       const uint32_t *__restrict__ ycol, real *__restrict__ yt,
                                                       real *__restrict__ yt_other, const uint32_t *__restrict__ perm,
                                                       int C, const real *const *__restrict__ Ptabs,
                                                       const real *const *__restrict__ Qtabs,
                                                       const real *__restrict__ a, const real *__restrict__ b) {
  using G = Geo<real, KP>;
  WAVE_SETUP
  const int sg = lane / G::LPR, li = lane % G::LPR;
  for (uint64_t i = wave; i < R; i += nwaves) {
    const real ai = a[i];
    for (int64_t p = yptr[i] + sg; p < yptr[i + 1]; p += G::NSG) {
      const uint32_t j = ycol[p];
      real s = 0;
      for (int c = 0; c < C; c++)
        s += sg_sum<G::LPR>(hsum<real>(gvld<real>(Ptabs[c] + i * KP + li * G::VE) *
                                       vld<real>(Qtabs[c] + (size_t)j * KP + li * G::VE)));
      if (li == 0) {
        const real v = s - (real)1;  // base_ij; y~_ij = base_ij + a_i + b_j
        yt[p] = v;
        yt_other[perm[p]] = v;
      }
    }
  }
}

// T_i = sum_c A_c[i] M_c for every row of a side (the w T_i term of
// gd_cross, ffm.cpp:663-700, T = sum_a P_a (Q_a^T Q1)), fp32 at KP = 32 or
// 64, on MFMA, ahead of the cross gradient pass (which then loads one T row
// per row instead of C table rows and C k x k products).  In the pass, T_i
// costs C k^2 multiply-adds per row with M read from LDS (or, when the C
// Grams exceed 64 KB, from L2: at BASELINE config 5, C = 39 and k = 64, that
// is 624 KB of M per row).  Here T = [A_1 .. A_C] [M_1; ..; M_C] is a
// (R x C KP) by (C KP x KP) product on v_mfma_f32_32x32x2f32: each wave owns
// TW tiles of 32 rows x KP columns (KP/32 accumulators of 16 registers per
// tile); the K dimension (table c, column k) is taken in the order (s, s +
// KP/2) so that lane l's A operands are the KP/2 consecutive floats
// [KP/2 (l/32), +KP/2) of row l%32 (KP/8 16-B loads per table and tile, the
// next table's in flight during this table's MFMAs).  B = M_c from LDS,
// staged TG tables at a time (one block per CU, 8 waves: 512 rows share
// each staging); Ms[(c k 32 + e) NT + t] = M_c[k][32 t + e], so one
// ds_read_b64 (KP = 64) gives a lane both output tiles' operands.
constexpr int TBLOCK = 512;  // threads of a k_rows_T block
template <int KP> struct RowsT {
  static constexpr int NT = KP / 32;  // 32-column output tiles
  static constexpr int KH = KP / 2;   // K steps per table (two K values each)
  static constexpr int TW = 2;        // 32-row tiles per wave
  // tables per LDS stage: KP = 64 two (32 KB; 8 tables / 128 KB measured 8 % slower,
  // tools/mb/mb_rowsT.hip), KP = 32 all 32 of a stage (128 KB)
  static constexpr int TG = KP == 64 ? 2 : 32;
  static constexpr int ROWS = (TBLOCK / 64) * TW * 32;  // rows per block pass
};
template <int KP>
__global__ __launch_bounds__(TBLOCK) void k_rows_T(uint64_t R, int C, const float *const *__restrict__ A,
                                                   const float *__restrict__ M, float *__restrict__ T) {
  using RT = RowsT<KP>;
  constexpr int NT = RT::NT, KH = RT::KH, TW = RT::TW, TG = RT::TG;
  typedef float f16x __attribute__((ext_vector_type(16)));
  typedef float v2f __attribute__((ext_vector_type(2)));
  __shared__ __align__(16) float Ms[TG * KP * KP];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int e = lane & 31, hf = lane >> 5;
  const uint32_t rowb = KP * 4;
  for (uint64_t base = (uint64_t)blockIdx.x * RT::ROWS; base < R; base += (uint64_t)gridDim.x * RT::ROWS) {
    f16x acc[TW][NT];
#pragma unroll
    for (int t = 0; t < TW; t++)
#pragma unroll
      for (int n = 0; n < NT; n++)
#pragma unroll
        for (int r = 0; r < 16; r++) acc[t][n][r] = 0.0f;
    // rows of this wave's tiles: row (base + (w TW + t) 32 + e); past R: zero (buffer range)
    for (int g0 = 0; g0 < C; g0 += TG) {
      const int ng = C - g0 < TG ? C - g0 : TG;
      __syncthreads();  // the previous stage's readers are done
      {
        // the stage in one round of independent 16-B loads (up to TG KP^2 / 4
        // / TBLOCK per thread), then the permuted LDS stores
        // (in two halves: the staging registers are not live beside the
        // operands' double buffer)
        constexpr int PER = (TG * KP * KP / 4 + TBLOCK - 1) / TBLOCK, PH = PER / 2 > 0 ? PER / 2 : 1;
        const BufView mb = buf_view(M + (size_t)g0 * KP * KP, (uint64_t)ng * KP * KP * 4);
#pragma unroll 1
        for (int u0 = 0; u0 < PER; u0 += PH) {
          f4v mv[PH];
#pragma unroll
          for (int u = 0; u < PH; u++) mv[u] = bld<float>(mb, (uint32_t)(threadIdx.x + (u0 + u) * TBLOCK) * 16u);
#pragma unroll
          for (int u = 0; u < PH; u++) {
            const int q = (threadIdx.x + (u0 + u) * TBLOCK) * 4;
            if (q < ng * KP * KP) {
              const int c = q / (KP * KP), rem = q % (KP * KP), k = rem / KP, col = rem % KP;
#pragma unroll
              for (int x = 0; x < 4; x++)
                Ms[((c * KP + k) * 32 + ((col + x) & 31)) * NT + ((col + x) >> 5)] = mv[u][x];
            }
          }
        }
      }
      __syncthreads();
      f4v a[2][TW][KH / 4];
      auto load = [&](auto SB, int c) {
        constexpr int sb = decltype(SB)::value;
        const BufView ab = buf_view(A[g0 + c], R * rowb);
#pragma unroll
        for (int t = 0; t < TW; t++) {
          const uint64_t row = base + (uint64_t)(w * TW + t) * 32 + e;
          const uint32_t off = row < R ? (uint32_t)(row * rowb + hf * KH * 4) : ab.oob;
#pragma unroll
          for (int q = 0; q < KH / 4; q++) a[sb][t][q] = bld<float>(ab, off + q * 16);
        }
      };
      // table c on register set c % 2 (compile-time: a runtime set index
      // would put the operands in scratch memory)
      auto compute = [&](auto SB, int c) {
        constexpr int sb = decltype(SB)::value;
        const float *mc = Ms + (size_t)c * KP * KP;
#pragma unroll
        for (int s = 0; s < KH; s++) {
          const int k = s + KH * hf;
          if constexpr (NT == 2) {
            const v2f b = *reinterpret_cast<const v2f *>(mc + (k * 32 + e) * 2);
#pragma unroll
            for (int t = 0; t < TW; t++) {
              const float av = a[sb][t][s >> 2][s & 3];
              acc[t][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, b[0], acc[t][0], 0, 0, 0);
              acc[t][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, b[1], acc[t][1], 0, 0, 0);
            }
          } else {
            const float b = mc[k * 32 + e];
#pragma unroll
            for (int t = 0; t < TW; t++)
              acc[t][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[sb][t][s >> 2][s & 3], b, acc[t][0], 0, 0, 0);
          }
        }
      };
      load(std::integral_constant<int, 0>(), 0);
      for (int c = 0; c < ng; c += 2) {
        if (c + 1 < ng) load(std::integral_constant<int, 1>(), c + 1);
        compute(std::integral_constant<int, 0>(), c);
        if (c + 1 >= ng) break;
        if (c + 2 < ng) load(std::integral_constant<int, 0>(), c + 2);
        compute(std::integral_constant<int, 1>(), c + 1);
      }
    }
    // D register r of lane l: row 8(r/4) + 4(l/32) + r%4 of the tile, column l%32 (+32 n)
#pragma unroll
    for (int t = 0; t < TW; t++)
#pragma unroll
      for (int n = 0; n < NT; n++)
#pragma unroll
        for (int r = 0; r < 16; r++) {
          const uint64_t m = base + (uint64_t)(w * TW + t) * 32 + 8 * (r >> 2) + 4 * hf + (r & 3);
          if (m < R) T[m * KP + n * 32 + e] = acc[t][n][r];
        }
  }
}

// --------------------------------------------------------- gradient rows ---
// Positive-gather row kernels run ONE SEGMENT PER SUBGROUP (LPR lanes): a
// wave keeps NSG segments in flight, each walking its (<= 32) positives with
// 4 independent row gathers per step.  Item rows are short (median ~10
// positives) and their dependent chain (segment -> row nodes -> feature
// row -> partner rows) is latency-bound, so parallelism per wave is the lever.
//
// Per segment s of row i:
//   h[s] = sum_{j in seg} ((1-w) y~_ij - w (1-r)) q_j
//          + [first] w (T_i + (a_i - r) oQ + bQ),   T_i = sum_c P_c[i] M_c
// (gd_cross row body, ffm.cpp:658-700); y~ = base + a_i + b_j.  M in LDS.
enum { BM_FULL = 0, BM_IN = 1, BM_ENTER = 2 };  // base modes of k_gd_cross_seg
// Experiment builds: -DOCFFM_GD_PROBE=1 launches, ahead of every cross
// gradient pass, its PRB instantiation ("gd_probe"): the same loads (the
// positions, the stored values and the partner-row gathers of every
// position, one or two per position) without the arithmetic, the T_i term
// and the stored-value writes: the time of its gathers alone.
#ifndef OCFFM_GD_PROBE
#define OCFFM_GD_PROBE 0
#endif

// T_i = sum_c P_c[i] M_c of the cross gradient (ffm.cpp:663-670) on the
// matrix cores, inside k_gd_cross_seg (round 5).  A block iteration covers
// SB = 4 NSG consecutive segments; T of their rows (first segments only:
// the others carry no row term) is the (SB x C KP) x (C KP x KP) product
// [P_1 .. P_C]_rows [M_1; ..; M_C], cut into 16 x 16 tiles, one per wave
// (fp32: SB KP = 1024, four tiles; fp64 at KP = 32: two, waves 2, 3 idle),
// each the chain of C KP / 4 v_mfma_{f32,f64}_16x16x4 over the whole K.
// The K order inside each chunk of 16 is permuted so that lane l (row l%16,
// k-group q = l/16) loads its 4 A values as one 16-B (fp64: 32-B) row slice
// A[row][16 j + 4 q .. +3] and takes them as the K values of 4 consecutive
// MFMAs; M is staged in LDS in the matching order Bt[(k/4) KP + n][k%4], so
// the 4 B values are one 16-B (32-B) LDS read.  The tile goes to LDS (Tl)
// and each segment's subgroup reads its row back.  The VALU version read M
// from LDS once per row and table (32 ds_read_b128 per row and table at KP =
// 32): LDS-bound at ~4x the VALU time on the song-id item halves.
#ifndef OCFFM_NO_TMMA
#define OCFFM_NO_TMMA 0  // experiment builds: -DOCFFM_NO_TMMA=1 keeps T_i on the VALU
#endif
template <typename real, int KP> struct TMma {
  using G = Geo<real, KP>;
  static constexpr bool OK =
      !OCFFM_NO_TMMA && ((std::is_same<real, float>::value && (KP == 16 || KP == 32 || KP == 64)) ||
                         (std::is_same<real, double>::value && KP == 32));
  static constexpr int SB = 4 * G::NSG;                    // segments (tile rows) per block iteration
  static constexpr int TR = SB >= 16 ? SB / 16 : 1, TC = KP >= 16 ? KP / 16 : 1;
  static constexpr int NTW = TR * TC;                     // waves computing a tile
  // LDS bytes beyond M (the T tile)
  static constexpr size_t tile_bytes() { return (size_t)SB * KP * sizeof(real); }
  // output row of D register r in lane l (v_mfma_f32_16x16x4f32: lane group
  // l/16 holds 4 consecutive rows; v_mfma_f64_16x16x4f64: rows l/16 + 4 r,
  // k_gram_mfma_f64's layout)
  static __device__ __forceinline__ int drow(int l, int r) {
    if constexpr (std::is_same<real, float>::value) return 4 * (l >> 4) + r;
    else return (l >> 4) + 4 * r;
  }
  // M (C KP x KP row-major, c-major) -> Bt in LDS
  static __device__ __forceinline__ void stage(const real *__restrict__ M, int C, real *Bt) {
    const int tot = C * KP * KP;
    for (int t = threadIdx.x; t < tot; t += BLOCK) {
      const int k = t / KP, n = t % KP;
      Bt[((k >> 2) * KP + n) * 4 + (k & 3)] = M[t];
    }
  }
  // the tile of wave w (< NTW) for segments [base, base + SB) into Tl
  static __device__ __forceinline__ void tile(uint64_t base, uint64_t nseg, const Seg *__restrict__ segs,
                                              const uint32_t *__restrict__ sord, int C,
                                              const real *const *__restrict__ Ptabs, const real *Bt, real *Tl,
                                              int w, int lane) {
    const int tr = w % TR, tc = w / TR;
    const int m = lane & 15, q = lane >> 4;
    const uint64_t si = base + (uint64_t)tr * 16 + m;
    bool have = false;
    uint64_t row = 0;
    if (si < nseg) {
      const Seg s = segs[sord ? (uint64_t)sord[si] : si];
      have = seg_first(s);
      row = s.row;
    }
    const int nch = C * KP / 16;
    if constexpr (std::is_same<real, float>::value) {
      // GR independent accumulators (chunk u of a group into acc[u]): the
      // chain of C KP / 4 dependent MFMAs (40-cycle accumulator latency) cut
      // into GR interleaved ones, summed at the end
      f4v acc[4] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
      constexpr int GR = 4;  // chunks per load group (two groups in flight)
      f4v a[2][GR];
      auto load = [&](auto SB_, int j0) {
        constexpr int sb = decltype(SB_)::value;
#pragma unroll
        for (int u = 0; u < GR; u++) {
          const int j = j0 + u, k0 = 16 * j;
          a[sb][u] = (have && j < nch) ? gvld<float>(Ptabs[k0 / KP] + row * KP + (k0 % KP) + 4 * q)
                                       : f4v{0.f, 0.f, 0.f, 0.f};
        }
      };
      auto mma = [&](auto SB_, int j0) {
        constexpr int sb = decltype(SB_)::value;
#pragma unroll
        for (int u = 0; u < GR; u++) {
          const int j = j0 + u;
          if (j < nch) {
            const f4v b = *reinterpret_cast<const f4v *>(Bt + ((4 * j + q) * KP + tc * 16 + m) * 4);
#pragma unroll
            for (int s = 0; s < 4; s++)
              acc[u] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[sb][u][s], b[s], acc[u], 0, 0, 0);
          }
        }
      };
      load(std::integral_constant<int, 0>(), 0);
      for (int j0 = 0; j0 < nch; j0 += 2 * GR) {
        load(std::integral_constant<int, 1>(), j0 + GR);
        mma(std::integral_constant<int, 0>(), j0);
        if (j0 + GR >= nch) break;
        load(std::integral_constant<int, 0>(), j0 + 2 * GR);
        mma(std::integral_constant<int, 1>(), j0 + GR);
      }
      const f4v t = (acc[0] + acc[1]) + (acc[2] + acc[3]);
#pragma unroll
      for (int r = 0; r < 4; r++) Tl[(tr * 16 + drow(lane, r)) * KP + tc * 16 + m] = t[r];
    } else {
      typedef double d4 __attribute__((ext_vector_type(4)));
      d4 acc = {0.0, 0.0, 0.0, 0.0};
      constexpr int GR = 2;
      d2v a[2][GR][2];
      auto load = [&](auto SB_, int j0) {
        constexpr int sb = decltype(SB_)::value;
#pragma unroll
        for (int u = 0; u < GR; u++) {
          const int j = j0 + u, k0 = 16 * j;
          const bool ok = have && j < nch;
          const double *p = ok ? Ptabs[k0 / KP] + row * KP + (k0 % KP) + 4 * q : nullptr;
#pragma unroll
          for (int h = 0; h < 2; h++)
            a[sb][u][h] = ok ? *(const __attribute__((address_space(1))) d2v *)(p + 2 * h) : d2v{0.0, 0.0};
        }
      };
      auto mma = [&](auto SB_, int j0) {
        constexpr int sb = decltype(SB_)::value;
#pragma unroll
        for (int u = 0; u < GR; u++) {
          const int j = j0 + u;
          if (j < nch) {
            const double *bp = Bt + ((4 * j + q) * KP + tc * 16 + m) * 4;
            const d2v b0 = *reinterpret_cast<const d2v *>(bp), b1 = *reinterpret_cast<const d2v *>(bp + 2);
            acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a[sb][u][0][0], b0[0], acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a[sb][u][0][1], b0[1], acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a[sb][u][1][0], b1[0], acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a[sb][u][1][1], b1[1], acc, 0, 0, 0);
          }
        }
      };
      load(std::integral_constant<int, 0>(), 0);
      for (int j0 = 0; j0 < nch; j0 += 2 * GR) {
        load(std::integral_constant<int, 1>(), j0 + GR);
        mma(std::integral_constant<int, 0>(), j0);
        if (j0 + GR >= nch) break;
        load(std::integral_constant<int, 0>(), j0 + 2 * GR);
        mma(std::integral_constant<int, 1>(), j0 + GR);
      }
#pragma unroll
      for (int r = 0; r < 4; r++) Tl[(tr * 16 + drow(lane, r)) * KP + tc * 16 + m] = acc[r];
    }
  }
};

template <typename real, int KP, bool MLDS, int BM, bool TP = false, bool PRB = false>
__global__ __launch_bounds__(BLOCK, sizeof(real) == 8 ? OCFFM_GD_OCC64 : (BM == BM_ENTER ? OCFFM_GD_OCC : OCFFM_GD_OCC_IN)) void k_gd_cross_seg(uint64_t nseg, const Seg *__restrict__ segs,
                                                        const uint32_t *__restrict__ ycol,
                                                        real *__restrict__ yt, const real *__restrict__ Q1,
                                                        int C, const real *const *__restrict__ Ptabs,
                                                        const real *__restrict__ M, const double *__restrict__ sums,
                                                        const real *__restrict__ a1, const real *__restrict__ b1,
                                                        double w, double r, real *__restrict__ h,
                                                        uint64_t q1rows, const real *__restrict__ cur,
                                                        const real *__restrict__ drow,
                                                        const real *__restrict__ dxs,
                                                        const uint32_t *__restrict__ perm,
                                                        const real *__restrict__ Tpre,
                                                        const real *__restrict__ ytv,
                                                        const uint32_t *__restrict__ sord) {
  using G = Geo<real, KP>;
  using PP = PosPass<real, KP, sizeof(real) == 8 ? OCFFM_GD_GB64 : (BM == BM_ENTER ? OCFFM_GD_GB : OCFFM_GD_GB_IN)>;
  // TP: T_i precomputed by k_rows_T (one row load; no M in LDS)
  // ytv (BM_IN): the stored value is read from the other orientation through
  // perm (ytv[perm[q]]), so the entering pass of the block needs no refresh
  // of this orientation (solver.hip gradient)
  const BufView qb = buf_view(Q1, q1rows * KP * sizeof(real)), bb = buf_view(b1, q1rows * sizeof(real));
  const BufView xb = buf_view(dxs, dxs ? q1rows * KP * sizeof(real) : 0);
  extern __shared__ __align__(16) unsigned char smem_raw[];
  real *Ms = reinterpret_cast<real *>(smem_raw);
  const real *Mp = M;
  // TM: T_i on the matrix cores, a tile per block iteration (TMma); else
  // TL: T_i by lane-local accumulation over transposed M (fp32, KP <= 32)
  using TMM = TMma<real, KP>;
  constexpr bool TM = MLDS && !TP && TMM::OK;
  constexpr bool TL = !TM && MLDS && std::is_same<real, float>::value && KP <= 32;
  real *Tl = Ms + (TM ? (size_t)C * KP * KP : 0);
  if (TM) {
    TMM::stage(M, C, Ms);
    __syncthreads();
  } else if (MLDS && !TP) {
    const int tot = C * KP * KP;
    for (int t = threadIdx.x; t < tot; t += BLOCK) {
      if constexpr (TL) {  // pair-transposed (lane_vecmat_acc)
        const int c = t / (KP * KP), rn = t % (KP * KP);
        Ms[c * KP * KP + mt_index(KP, rn / KP, rn % KP)] = M[t];
      } else {
        Ms[t] = M[t];
      }
    }
    __syncthreads();
    Mp = Ms;
  }
  WAVE_SETUP
  const int sg = lane / G::LPR, li = lane % G::LPR;
  const real cpos = (real)(1 - w), cneg = (real)(w * (1 - r));
  vec_t<real> oQ, bQ;
#pragma unroll
  for (int e = 0; e < G::VE; e++) {
    oQ[e] = (real)sums[li * G::VE + e];
    bQ[e] = (real)sums[KP + li * G::VE + e];
  }
  // Block-excluded y~.  During the cross loop the stored value is
  // e_ij = y~_ij - <P_b[i], Q_b[j]> for the current cross block b: the halves'
  // updates of P_b / Q_b leave it untouched, and the biases (constant over the
  // cross loop) are folded in.  cur = this half's own factor of block b (its
  // partner factor is the gathered q_j).
  //   BM_FULL : base stored; y~ = base + a_i + b_j
  //   BM_IN   : inside block b; y~ = e + <cur_i, q_j>
  //   BM_ENTER: entering block b; y~ = e' + <drow_i, dxs_j> (e' of block b',
  //             drow/dxs its factors) or base + a_i + b_j (dxs null); stores
  //             e = y~ - <cur_i, q_j> here.
  constexpr bool WR = BM == BM_ENTER;
  auto body = [&](const Seg &sgm) -> vec_t<real> {
    const uint64_t i = sgm.row;
    const real ai = a1[i];
    vec_t<real> pk = vzero<real>();
    const vec_t<real> dr = (WR && dxs) ? vld<real>(drow + i * KP + li * G::VE) : vzero<real>();
    const vec_t<real> cr = BM != BM_FULL ? vld<real>(cur + i * KP + li * G::VE) : vzero<real>();
    const bool gbias = BM == BM_FULL || (WR && !dxs);
    for (int64_t p0 = sgm.b; p0 < sgm.e; p0 += PP::PW) {
      uint32_t jj[PP::UT];
      real yv[PP::UT];
      PP::load_cols(ycol, p0, sgm.e, li, jj);
#pragma unroll
      for (int t = 0; t < PP::UT; t++) {
        const int64_t q = p0 + li + t * G::LPR;
        yv[t] = q < sgm.e ? (ytv ? ytv[perm[q]] : yt[q]) : (real)0;
      }
      real yn[PP::UT];  // WR: e of this lane's positions
#pragma unroll
      for (int t = 0; t < PP::UT; t++) yn[t] = yv[t];
      sfor<PP::PW / PP::GB>([&](auto BT) {
        constexpr int bt = decltype(BT)::value * PP::GB;
        if (p0 + bt >= sgm.e) return;
        vec_t<real> qv[PP::GB], xv[WR ? PP::GB : 1];
        real yb[PP::GB];
        sfor<PP::GB>([&](auto U) {
          constexpr int u = decltype(U)::value;
          const uint32_t j = PP::template at<bt + u>(jj, li);
          yb[u] = PP::template at<bt + u>(yv, li);
          qv[u] = bld<real>(qb, PP::row_off(j, qb, li));
          if (gbias) yb[u] += ai + bld1<real>(bb, j == POS_NONE ? bb.oob : j * (uint32_t)sizeof(real));
          if constexpr (WR) {
            if (dxs) xv[u] = bld<real>(xb, PP::row_off(j, xb, li));
          }
        });
        if constexpr (PRB) {  // bound probe: the gathers and the sum, no dot products
#pragma unroll
          for (int u = 0; u < PP::GB; u++) {
            pk += qv[u];
            if constexpr (WR) pk += xv[u];
          }
          return;
        }
        if constexpr (BM != BM_FULL) {
#pragma unroll
          for (int u = 0; u < PP::GB; u++) {
            const real c = sg_sum<G::LPR>(hsum<real>(cr * qv[u]));
            if constexpr (WR) {
              if (dxs) yb[u] += sg_sum<G::LPR>(hsum<real>(dr * xv[u]));
              if ((bt + u) % G::LPR == li) yn[(bt + u) / G::LPR] = yb[u] - c;
            } else {
              yb[u] += c;
            }
          }
        }
#pragma unroll
        for (int u = 0; u < PP::GB; u++) pk += vsplat<real>(cpos * yb[u] - cneg) * qv[u];
      });
      if constexpr (WR && !PRB) {
#pragma unroll
        for (int t = 0; t < PP::UT; t++) {
          const int64_t q = p0 + li + t * G::LPR;
          if (q < sgm.e) yt[q] = yn[t];
        }
      }
    }
    if (!PRB && TP && seg_first(sgm)) {
      const real z = ai - (real)r;
      pk += vsplat<real>((real)w) * (vld<real>(Tpre + i * KP + li * G::VE) + vsplat<real>(z) * oQ + bQ);
    }
    if (!PRB && TM && seg_first(sgm)) {  // T_i from the block's MFMA tile
      const real z = ai - (real)r;
      const vec_t<real> t = vld<real>(Tl + (size_t)((threadIdx.x >> 6) * G::NSG + sg) * KP + li * G::VE);
      pk += vsplat<real>((real)w) * (t + vsplat<real>(z) * oQ + bQ);
    }
    if (!PRB && !TP && !TM && seg_first(sgm)) {
      // T_i: the C row loads are independent; issue them in batches so the
      // vector-matrix products do not wait on one HBM round trip per table
      constexpr int CB = 4;
      vec_t<real> t = vzero<real>();
      f2v ul[TL ? KP / 2 : 1];
      if constexpr (TL) {
#pragma unroll
        for (int q = 0; q < KP / 2; q++) ul[q] = f2v{0.f, 0.f};
      }
      for (int c0 = 0; c0 < C; c0 += CB) {
        vec_t<real> pc[CB];
#pragma unroll
        for (int u = 0; u < CB; u++)
          pc[u] = c0 + u < C ? gvld<real>(Ptabs[c0 + u] + i * KP + li * G::VE) : vzero<real>();
#pragma unroll
        for (int u = 0; u < CB; u++)
          if (c0 + u < C) {
            if constexpr (TL) lane_vecmat_acc<KP>(ul, pc[u], Mp + (size_t)(c0 + u) * KP * KP, li);
            else t += sg_vecmat<real, KP>(pc[u], Mp + (size_t)(c0 + u) * KP * KP, li);
          }
      }
      if constexpr (TL) {
        real uf[KP];
#pragma unroll
        for (int q = 0; q < KP / 2; q++) {
          uf[2 * q] = ul[q][0];
          uf[2 * q + 1] = ul[q][1];
        }
        t = sg_reduce_scatter<real, KP>(uf, li);
      }
      const real z = ai - (real)r;
      pk += vsplat<real>((real)w) * (t + vsplat<real>(z) * oQ + bQ);
    }
    return pk;
  };
  if constexpr (TM) {
    // block iterations over SB consecutive segments: the waves' MFMA tile,
    // a barrier, the segments (each reads its row of the tile), a barrier
    // before the next iteration rewrites the tile
    const int wv = threadIdx.x >> 6;
    for (uint64_t base = (uint64_t)blockIdx.x * TMM::SB; base < nseg; base += (uint64_t)gridDim.x * TMM::SB) {
      if (!PRB && wv < TMM::NTW) TMM::tile(base, nseg, segs, sord, C, Ptabs, Ms, Tl, wv, lane);
      __syncthreads();
      const uint64_t s = base + (uint64_t)wv * G::NSG + sg;
      if (s < nseg) {
        const uint64_t sx = sord ? (uint64_t)sord[s] : s;
        vst<real>(h + sx * KP + li * G::VE, body(segs[sx]));
      }
      __syncthreads();
    }
  } else {
    // sord (optional): processing order of the segments (longest first, as
    // in k_hs_cross_seg); h stays in segment order
    for (uint64_t s = wave * G::NSG + sg; s < nseg; s += nwaves * G::NSG) {
      const uint64_t sx = sord ? (uint64_t)sord[s] : s;
      vst<real>(h + sx * KP + li * G::VE, body(segs[sx]));
    }
  }
}

// Per segment s: ysum[s] = sum_{p in seg} (base_p + b1[ycol_p]).  A side's
// gradient passes (gd_side) need sum_{j in seg} y~_ij = ysum[s] + n_s a_i
// (y~ = base + a_i + b_j), and over the side halves of one side
// neither the base nor the partner biases b change (side updates only move
// this side's a): the solver computes ysum once per side phase and the
// gradient passes then touch no positive (k_gd_side_seg PRE).
template <typename real, int KP>
__global__ __launch_bounds__(BLOCK) void k_seg_ysum(uint64_t nseg, const Seg *__restrict__ segs,
                                                    const uint32_t *__restrict__ ycol, const real *__restrict__ yt,
                                                    const real *__restrict__ b1, uint64_t nb1,
                                                    real *__restrict__ ysum) {
  using G = Geo<real, KP>;
  using PP = PosPass<real, KP>;
  const BufView bb = buf_view(b1, nb1 * sizeof(real));
  WAVE_SETUP
  const int sg = lane / G::LPR, li = lane % G::LPR;
  for (uint64_t s = wave * G::NSG + sg; s < nseg; s += nwaves * G::NSG) {
    const Seg sgm = segs[s];
    real z = 0;
    for (int64_t p0 = sgm.b; p0 < sgm.e; p0 += PP::PW) {
      uint32_t jj[PP::UT];
      real yv[PP::UT], cb[PP::UT];
      PP::load_cols(ycol, p0, sgm.e, li, jj);
#pragma unroll
      for (int t = 0; t < PP::UT; t++) {
        const int64_t q = p0 + li + t * G::LPR;
        yv[t] = q < sgm.e ? yt[q] : (real)0;
        cb[t] = bld1<real>(bb, jj[t] == POS_NONE ? bb.oob : jj[t] * (uint32_t)sizeof(real));
      }
#pragma unroll
      for (int t = 0; t < PP::UT; t++)
        if (p0 + li + t * G::LPR < sgm.e) z += yv[t] + cb[t];
    }
    z = sg_sum<G::LPR>(z);
    if (li == 0) ysum[s] = z;
  }
}

// Per row: yrow[i] = sum of ysum over row i's segments (one wave per row,
// lanes striding its segments: the rows of popular items have hundreds),
// for the fused side half (k_cg_side_id FULL), which then reads one value
// per row.
template <typename real>
__global__ __launch_bounds__(BLOCK) void k_row_ysum(uint64_t R, const uint32_t *__restrict__ segptr,
                                                    const real *__restrict__ ysum, real *__restrict__ yrow) {
  WAVE_SETUP
  for (uint64_t i = wave; i < R; i += nwaves) {
    real z = 0;
    for (uint32_t q = segptr[i] + lane; q < segptr[i + 1]; q += 64) z += ysum[q];
    z = sg_sum<64>(z);
    if (lane == 0) yrow[i] = z;
  }
}

// Per segment: h[s] = zpart * q1_i, zpart = sum_{p in seg} ((1-w) y~ - w (1-r))
// + [first] w (n1 (a_i - r) + sum(b) + sa_i)   (gd_side row body, ffm.cpp:572-589).
// ysum non-null: the positive sum comes from k_seg_ysum (no positive pass).
template <typename real, int KP>
__global__ __launch_bounds__(BLOCK) void k_gd_side_seg(uint64_t nseg, const Seg *__restrict__ segs,
                                                       const uint32_t *__restrict__ ycol,
                                                       const real *__restrict__ yt, const real *__restrict__ Q1,
                                                       const real *__restrict__ a1, const real *__restrict__ b1,
                                                       const real *__restrict__ sa1,
                                                       const double *__restrict__ bsum, double n1, double w,
                                                       double r, real *__restrict__ h, uint64_t nb1,
                                                       const real *__restrict__ ysum) {
  using G = Geo<real, KP>;
  using PP = PosPass<real, KP>;
  const BufView bb = buf_view(b1, nb1 * sizeof(real));
  WAVE_SETUP
  const int sg = lane / G::LPR, li = lane % G::LPR;
  const real cpos = (real)(1 - w), cneg = (real)(w * (1 - r));
  const double bs = *bsum;
  auto body = [&](const Seg &sgm, uint64_t s) -> vec_t<real> {
    const uint64_t i = sgm.row;
    const real ai = a1[i];
    real z = 0;
    if (ysum) {  // sum_{p in seg} ((1-w)(base + a_i + b_j) - w(1-r)), summed once per side phase
      const real n = (real)(sgm.e - sgm.b);
      z = cpos * (ysum[s] + n * ai) - n * cneg;
    } else {
    for (int64_t p0 = sgm.b; p0 < sgm.e; p0 += PP::PW) {
      uint32_t jj[PP::UT];
      real yv[PP::UT], cb[PP::UT];
      PP::load_cols(ycol, p0, sgm.e, li, jj);
#pragma unroll
      for (int t = 0; t < PP::UT; t++) {
        const int64_t q = p0 + li + t * G::LPR;
        yv[t] = q < sgm.e ? yt[q] : (real)0;
        cb[t] = bld1<real>(bb, jj[t] == POS_NONE ? bb.oob : jj[t] * (uint32_t)sizeof(real));
      }
#pragma unroll
      for (int t = 0; t < PP::UT; t++)
        if (p0 + li + t * G::LPR < sgm.e) z += cpos * (yv[t] + ai + cb[t]) - cneg;
    }
    z = sg_sum<G::LPR>(z);
    }
    if (seg_first(sgm)) z += (real)(w * (n1 * ((double)ai - r) + bs + (double)sa1[i]));
    return vsplat<real>(z) * vld<real>(Q1 + i * KP + li * G::VE);
  };
  for (uint64_t s = wave * G::NSG + sg; s < nseg; s += nwaves * G::NSG) vst<real>(h + s * KP + li * G::VE, body(segs[s], s));
}

// ------------------------------------------------ Hessian-vector rows ---
// h_i = d_i <phi_i, q1_i> q1_i, phi_i = X_i V, d_i = (1-w)|pos(i)| + w n1
// (hs_side row body, ffm.cpp:603-624).  One row per subgroup, row-indexed h.
// SCAT (id-like field, several ranks): x_i h_i goes straight to its column's
// slot of f.acc for the all-reduce (the CSC scatter is the identity).
template <typename real, int KP, bool FUSE, bool SCAT = false>
__global__ __launch_bounds__(BLOCK) void k_hs_side_row(uint64_t R, const int64_t *__restrict__ xptr,
                                                       const uint32_t *__restrict__ xidx,
                                                       const real *__restrict__ xval, const real *__restrict__ V,
                                                       const int64_t *__restrict__ yptr,
                                                       const real *__restrict__ Q1, double w, double n1,
                                                       real *__restrict__ h, const int *__restrict__ run,
                                                       const real *__restrict__ Rv, const real *__restrict__ Hv,
                                                       const CgState *st, int it, bool one, Fin<real> f) {
  using G = Geo<real, KP>;
  if (run && !*run) return;
  const bool upd = st && it > 1;
  const real alpha = upd ? (real)st->alpha : (real)0, beta = upd ? (real)st->beta : (real)0;
  WAVE_SETUP
  const int sg = lane / G::LPR, li = lane % G::LPR;
  double dsum[3] = {0, 0, 0};
  for (uint64_t i = wave * G::NSG + sg; i < R; i += nwaves * G::NSG) {
    if (FUSE) {
      // id-like field: row i is column d's only row, so the finalisation
      // operands (p, r, Hp, S of column d) are loaded once and the row's
      // CG direction is formed from them (V = f.P, Rv = f.R, Hv = f.Hp)
      const uint32_t d = xidx[i];
      const real x = xval[i];
      const FinOps<real> ops = fin_load<real, KP, 1>(f, d, upd, li);
      const vec_t<real> q = vld<real>(Q1 + i * KP + li * G::VE);
      vec_t<real> pt = ops.w_or_p;
      if (upd) pt = (ops.r - vsplat<real>(alpha) * ops.hp) + vsplat<real>(beta) * ops.w_or_p;
      const real z = sg_sum<G::LPR>(hsum<real>(vsplat<real>(x) * pt * q));
      const real dd = (real)((1 - w) * (double)(yptr[i + 1] - yptr[i]) + w * n1);
      col_finalize<real, KP, 1>(f, d, vsplat<real>(x) * (vsplat<real>(dd * z) * q), alpha, beta, upd, li, dsum, ops);
      continue;
    }
    vec_t<real> phi = vzero<real>();
    if (one) {  // one node per row: xptr[i] == i
      phi = vsplat<real>(xval[i]) * cg_dir_at<real, KP>(V, Rv, Hv, alpha, beta, upd, (size_t)xidx[i] * KP + li * G::VE);
    } else {
      for (int64_t p = xptr[i]; p < xptr[i + 1]; p++)
        phi += vsplat<real>(xval[p]) * cg_dir_at<real, KP>(V, Rv, Hv, alpha, beta, upd, (size_t)xidx[p] * KP + li * G::VE);
    }
    const vec_t<real> q = vld<real>(Q1 + i * KP + li * G::VE);
    const real z = sg_sum<G::LPR>(hsum<real>(phi * q));
    const real d = (real)((1 - w) * (double)(yptr[i + 1] - yptr[i]) + w * n1);
    if constexpr (SCAT) {  // id-like field on several ranks: row i is column xidx[i]'s only row
      vst<real>(f.acc + (size_t)xidx[i] * KP + li * G::VE, vsplat<real>(xval[i] * d * z) * q);
    } else {
      vst<real>(h + i * KP + li * G::VE, vsplat<real>(d * z) * q);
    }
  }
  if (FUSE) fin_blocks<real, 1>(f, dsum);
}

// ------------------------------------------- per-column Grams (side) ---
// A side half over a one-node-per-row field has, per feature column c,
//   (X^T h)_c = sum_{i: idx_i = c} x_i h_i = G_c p_c,
//   G_c = sum_{i: idx_i = c} d_i x_i^2 q1_i q1_i^T  (k x k, symmetric)
// (hs_side row body, ffm.cpp:603-624, summed per column).  q1 and d are
// fixed over the half's CG steps, so G_c is built once per half and each CG
// step is one launch over D k^2 instead of a row pass plus a feature pass.
// Rows per Gram chunk: a chunk's q1 rows are staged once in 32 KB of LDS
// (the host caps OCFFM_CGRAM_CHUNK at this).  Measured at kkbox shape:
// 256-row chunks 44 us, 128 rows 32 us (default), 64 rows 34 us per build.
constexpr int cgram_rows(int kp, int rs) { return 32768 / (kp * rs) < 256 ? 32768 / (kp * rs) : 256; }

// One block per chunk (Job: col, nparts = chunks of the column, slot =
// partial slot, flags = chunk index in the column, [b, e) in the field's
// CSC, e - b <= cgram_rows): each thread sums its entries of the chunk's
// rank-n update.  A one-chunk column stores G_c.  The chunks of a longer
// column store their partials in consecutive slots (sc1), take a ticket on
// the column, and the last to arrive sums the slots in chunk order:
// deterministic, no float atomics (the guide's last-arriver hand-off: sc1
// stores, every wave drained behind a barrier, one agent-scope add per
// block, sc1 loads by the block whose add came last).
template <typename real, int KP>
__global__ __launch_bounds__(BLOCK) void k_col_gram(const Job *__restrict__ chunks, const uint32_t *__restrict__ crow,
                                                    const real *__restrict__ cval, const int64_t *__restrict__ yptr,
                                                    const real *__restrict__ Q1, double w, double n1,
                                                    real *__restrict__ G, real *__restrict__ gpart,
                                                    unsigned *__restrict__ cnt, int pw) {
  constexpr int CH = cgram_rows(KP, (int)sizeof(real));
  constexpr int KK = KP * KP;
  constexpr int NE = (KK + BLOCK - 1) / BLOCK;
  __shared__ real qs[CH * KP];
  __shared__ real cs[CH];
  __shared__ int s_last;
  const Job jb = chunks[blockIdx.x];
  const int n = (int)(jb.e - jb.b);
  for (int t = threadIdx.x; t < n * KP; t += BLOCK) qs[t] = Q1[(size_t)crow[jb.b + t / KP] * KP + t % KP];
  for (int r = threadIdx.x; r < n; r += BLOCK) {
    const uint32_t i = crow[jb.b + r];
    const real x = cval[jb.b + r];
    cs[r] = (real)((1 - w) * (double)(yptr[i + 1] - yptr[i]) + w * n1) * (pw ? x : x * x);
  }
  __syncthreads();
  real acc[NE];
#pragma unroll
  for (int e = 0; e < NE; e++) acc[e] = 0;
  for (int r = 0; r < n; r++) {
    const real c = cs[r];
#pragma unroll
    for (int e = 0; e < NE; e++) {
      const int t = threadIdx.x + e * BLOCK;
      if (t < KK) acc[e] += c * qs[r * KP + t / KP] * qs[r * KP + t % KP];
    }
  }
  real *g = G + (size_t)jb.col * KK;
  if (jb.nparts <= 1) {
#pragma unroll
    for (int e = 0; e < NE; e++) {
      const int t = threadIdx.x + e * BLOCK;
      if (t < KK) g[t] = acc[e];
    }
    return;
  }
  real *gp = gpart + (size_t)jb.slot * KK;
#pragma unroll
  for (int e = 0; e < NE; e++) {
    const int t = threadIdx.x + e * BLOCK;
    if (t < KK) __hip_atomic_store(gp + t, acc[e], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0)
    s_last = __hip_atomic_fetch_add(cnt + jb.col, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == jb.nparts - 1;
  __syncthreads();
  if (!s_last) return;
  // the column's slots, RB at a time per element (sc1 buffer loads: aux 16;
  // slots past the column read zero), summed in slot order
  constexpr int RB = NE >= 32 ? 1 : 32 / NE;
  const BufView pv = buf_view(gpart + (size_t)(jb.slot - jb.flags) * KK, (uint64_t)jb.nparts * KK * sizeof(real));
  real s[NE];
#pragma unroll
  for (int e = 0; e < NE; e++) s[e] = 0;
  for (uint32_t q0 = 0; q0 < jb.nparts; q0 += RB) {
    real y[NE][RB];
#pragma unroll
    for (int e = 0; e < NE; e++)
#pragma unroll
      for (int u = 0; u < RB; u++) {
        const int t = threadIdx.x + e * BLOCK;
        const uint32_t q = q0 + u;
        const uint32_t off = (t < KK && q < jb.nparts) ? (uint32_t)((q * KK + t) * sizeof(real)) : pv.oob;
        if constexpr (sizeof(real) == 4)
          y[e][u] = __builtin_bit_cast(real, __builtin_amdgcn_raw_buffer_load_b32(pv.r, off, 0, 16));
        else
          y[e][u] = __builtin_bit_cast(real, __builtin_amdgcn_raw_buffer_load_b64(pv.r, off, 0, 16));
      }
#pragma unroll
    for (int e = 0; e < NE; e++)
#pragma unroll
      for (int u = 0; u < RB; u++)
        if (q0 + u == 0) s[e] = y[e][u];
        else if (q0 + u < jb.nparts) s[e] += y[e][u];
  }
#pragma unroll
  for (int e = 0; e < NE; e++) {
    const int t = threadIdx.x + e * BLOCK;
    if (t < KK) g[t] = s[e];
  }
  if (threadIdx.x == 0) __hip_atomic_store(cnt + jb.col, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Per-column Grams on MFMA (fp32, KP = 32; the default where it applies).
// One WAVE per chunk of <= CGRAM32_ROWS rows of a column: lane l stages row
// l's index and weight c_l = d_i x_i^2, then each v_mfma_f32_32x32x2f32 takes
// a row pair r = 2s + l/32 (A lane l = c_r q_r[l%32], B lane l = q_r[l%32],
// the k_gram_mfma32 operand layout): the chunk's sum_r c_r q_r q_r^T builds
// up in 16 accumulator registers with no LDS.  Every q-row load of the
// chunk is issued before the first MFMA (one latency round).  A one-chunk
// column stores G_c; the chunks of a longer column store their partial
// slot (plain stores) and k_gram_slot_sum adds the slots in slot order after
// the launch (deterministic; no tickets, no in-kernel hand-off).  Replaces
// k_col_gram's one block per <= 128-row chunk, whose rank-1 updates read two
// LDS words per multiply-add (genre: 32.7 us, artist: 35.4 us per build).
constexpr int CGRAM32_ROWS = 64;
static __global__ __launch_bounds__(BLOCK) void k_col_gram32(uint64_t nchunks, const Job *__restrict__ chunks,
                                                      const uint32_t *__restrict__ crow,
                                                      const float *__restrict__ cval, const int64_t *__restrict__ yptr,
                                                      const float *__restrict__ Q1, uint64_t q1rows, double w, double n1,
                                                      float *__restrict__ G, float *__restrict__ gpart, int pw) {
  typedef float f16x __attribute__((ext_vector_type(16)));
  const int lane = threadIdx.x & 63;
  const uint64_t wv = ((uint64_t)blockIdx.x * BLOCK + threadIdx.x) >> 6;
  if (wv >= nchunks) return;
  const Job jb = chunks[wv];
  const int n = (int)(jb.e - jb.b);  // <= CGRAM32_ROWS (host)
  uint32_t il = 0;
  float cl = 0.0f;
  if (lane < n) {
    il = crow[jb.b + lane];
    const float x = cval[jb.b + lane];
    cl = (float)((1 - w) * (double)(yptr[il + 1] - yptr[il]) + w * n1) * (pw ? x : x * x);
  }
  const BufView qb = buf_view(Q1, q1rows * 128);
  const int e = lane & 31, hf = lane >> 5;
  float qv[CGRAM32_ROWS / 2], cv[CGRAM32_ROWS / 2];
#pragma unroll
  for (int s = 0; s < CGRAM32_ROWS / 2; s++) {
    const int r = 2 * s + hf;  // rows past n: weight 0, the load reads zero
    const uint32_t i = (uint32_t)__shfl((int)il, r, 64);
    cv[s] = __shfl(cl, r, 64);
    qv[s] = bld1<float>(qb, r < n ? i * 128u + (uint32_t)e * 4u : 0xffffffffu);
  }
  f16x acc;
#pragma unroll
  for (int r = 0; r < 16; r++) acc[r] = 0.0f;
  // branch-free (rows past n have weight and row zero): a per-MFMA branch
  // made the compiler copy the accumulator between AGPRs and VGPRs each time
#pragma unroll
  for (int s = 0; s < CGRAM32_ROWS / 2; s++) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(cv[s] * qv[s], qv[s], acc, 0, 0, 0);
  // D register r of lane l: element m = 8(r/4) + 4(l/32) + r%4, n = l%32
  float *out = jb.nparts <= 1 ? G + (size_t)jb.col * 1024 : gpart + (size_t)jb.slot * 1024;
#pragma unroll
  for (int r = 0; r < 16; r++) out[(8 * (r >> 2) + 4 * hf + (r & 3)) * 32 + e] = acc[r];
}

// The same in fp64 on the f64 matrix cores (v_mfma_f64_16x16x4f64, the
// k_hot_gram_mfma_f64 operand layout: four rows per MFMA as K; tiles 00, 01,
// 11 of the symmetric 32 x 32 Gram, 10 stored as 01^T); multi-chunk columns
// summed by k_hot_slot_sum<double, 32>.
static __global__ __launch_bounds__(BLOCK) void k_col_gram_f64(uint64_t nchunks, const Job *__restrict__ chunks,
                                                              const uint32_t *__restrict__ crow,
                                                              const double *__restrict__ cval,
                                                              const int64_t *__restrict__ yptr,
                                                              const double *__restrict__ Q1, uint64_t q1rows, double w,
                                                              double n1, double *__restrict__ G,
                                                              double *__restrict__ gpart, int pw) {
  typedef double d4 __attribute__((ext_vector_type(4)));
  constexpr int NG = CGRAM32_ROWS / 4;
  const int lane = threadIdx.x & 63;
  const uint64_t wv = ((uint64_t)blockIdx.x * BLOCK + threadIdx.x) >> 6;
  if (wv >= nchunks) return;
  const Job jb = chunks[wv];
  const int n = (int)(jb.e - jb.b);  // <= CGRAM32_ROWS (host)
  uint32_t il = 0;
  double cl = 0.0;
  if (lane < n) {
    il = crow[jb.b + lane];
    const double x = cval[jb.b + lane];
    cl = ((1 - w) * (double)(yptr[il + 1] - yptr[il]) + w * n1) * (pw ? x : x * x);
  }
  const BufView qb = buf_view(Q1, q1rows * 256);
  const int c16 = lane & 15, rq = lane >> 4;
  double q0[NG], q1[NG], cv[NG];
#pragma unroll
  for (int g = 0; g < NG; g++) {
    const int r = 4 * g + rq;  // rows past n: weight 0, the loads read zero
    const uint32_t i = (uint32_t)__shfl((int)il, r, 64);
    cv[g] = __shfl(cl, r, 64);
    const uint32_t off = r < n ? i * 256u + (uint32_t)c16 * 8u : 0xffffffffu;
    q0[g] = bld1<double>(qb, off);
    q1[g] = bld1<double>(qb, r < n ? off + 128u : 0xffffffffu);
  }
  d4 acc[2][3];
#pragma unroll
  for (int u = 0; u < 2; u++)
#pragma unroll
    for (int a = 0; a < 3; a++) acc[u][a] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int g = 0; g < NG; g++) {
    d4(&c)[3] = acc[g & 1];
    const double a0 = cv[g] * q0[g], a1 = cv[g] * q1[g];
    c[0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, q0[g], c[0], 0, 0, 0);
    c[1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, q1[g], c[1], 0, 0, 0);
    c[2] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, q1[g], c[2], 0, 0, 0);
  }
#pragma unroll
  for (int a = 0; a < 3; a++) acc[0][a] += acc[1][a];
  double *out = jb.nparts <= 1 ? G + (size_t)jb.col * 1024 : gpart + (size_t)jb.slot * 1024;
#pragma unroll
  for (int r = 0; r < 4; r++) {
    const int m = rq + 4 * r;
    out[m * 32 + c16] = acc[0][0][r];
    out[m * 32 + 16 + c16] = acc[0][1][r];
    out[(16 + c16) * 32 + m] = acc[0][1][r];
    out[(16 + m) * 32 + 16 + c16] = acc[0][2][r];
  }
}

// G_c = sum of the partial slots of a multi-chunk column, in slot order
// (sums: Job{col, nparts, first slot}).  One block per such column; thread t
// owns elements 4t .. 4t+3; slots are read GB at a time (loads in flight).
static __global__ __launch_bounds__(BLOCK) void k_gram_slot_sum(const Job *__restrict__ sums,
                                                         const float *__restrict__ gpart, float *__restrict__ G) {
  constexpr int GB = 8;
  const Job jb = sums[blockIdx.x];
  const f4v *src = reinterpret_cast<const f4v *>(gpart + (size_t)jb.slot * 1024) + threadIdx.x;
  f4v acc = src[0];
  for (uint32_t q0 = 1; q0 < jb.nparts; q0 += GB) {
    f4v y[GB];
#pragma unroll
    for (int u = 0; u < GB; u++) y[u] = q0 + u < jb.nparts ? src[(size_t)(q0 + u) * 256] : f4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int u = 0; u < GB; u++)
      if (q0 + u < jb.nparts) acc += y[u];
  }
  reinterpret_cast<f4v *>(G + (size_t)jb.col * 1024)[threadIdx.x] = acc;
}

// ------------------------------------------- per-row Grams (cross) ---
// Hot rows of a cross half: a row i with many positives has
//   sum_{j in Omega_i} <phi_i, q_j> q_j = G_i phi_i,  G_i = sum_{j in Omega_i} q_j q_j^T
// (hs_cross row body, ffm.cpp:715-738).  The partner table Q1 is fixed over
// the half's CG steps, so G_i is built once per half and each step reads
// k x k values for the row instead of gathering |Omega_i| partner rows (a
// popular item's ~10^4 users; a heavy user's ~10^2 items).  Chunks
// (Job: col = the row's Gram slot, nparts = chunks of the row, slot = the
// partial slot, [b, e) = a range of the row's positives) sum into G, or into
// ordered partial slots that k_hot_slot_sum adds in slot order after the
// launch (deterministic).  HOT_NONE: a segment of a row without a Gram.
constexpr uint32_t HOT_NONE = 0xffffffffu;

// Per segment: the Gram slot of its row (or HOT_NONE).
static __global__ __launch_bounds__(BLOCK) void k_hot_seg(uint64_t nseg, const Seg *__restrict__ segs,
                                                   const uint32_t *__restrict__ row_slot, uint32_t *__restrict__ out) {
  const uint64_t s = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
  if (s < nseg) out[s] = row_slot[segs[s].row];
}

// Generic build (fp64, or any KP): one block per chunk, the chunk's partner
// rows staged through LDS cgram_rows at a time, thread t owns elements
// t, t + BLOCK, ... of the k x k sum.  wts (optional): a weight per position
// (per-column cross Grams: x_i^2 of the position's row).
template <typename real, int KP>
__global__ __launch_bounds__(BLOCK) void k_hot_gram(const Job *__restrict__ chunks, const uint32_t *__restrict__ ycol,
                                                    const real *__restrict__ wts, const real *__restrict__ Q1,
                                                    real *__restrict__ G, real *__restrict__ gpart) {
  constexpr int CH = cgram_rows(KP, (int)sizeof(real));
  constexpr int KK = KP * KP;
  constexpr int NE = (KK + BLOCK - 1) / BLOCK;
  __shared__ real qs[CH * KP];
  __shared__ real ws[CH];
  const Job jb = chunks[blockIdx.x];
  real acc[NE];
#pragma unroll
  for (int e = 0; e < NE; e++) acc[e] = 0;
  for (int64_t b0 = jb.b; b0 < jb.e; b0 += CH) {
    const int n = (int)(jb.e - b0 < CH ? jb.e - b0 : CH);
    __syncthreads();
    for (int t = threadIdx.x; t < n * KP; t += BLOCK) qs[t] = Q1[(size_t)ycol[b0 + t / KP] * KP + t % KP];
    for (int t = threadIdx.x; t < n; t += BLOCK) ws[t] = wts ? wts[b0 + t] : (real)1;
    __syncthreads();
    for (int r = 0; r < n; r++) {
      const real c = ws[r];
#pragma unroll
      for (int e = 0; e < NE; e++) {
        const int t = threadIdx.x + e * BLOCK;
        if (t < KK) acc[e] += c * qs[r * KP + t / KP] * qs[r * KP + t % KP];
      }
    }
  }
  real *out = jb.nparts <= 1 ? G + (size_t)jb.col * KK : gpart + (size_t)jb.slot * KK;
#pragma unroll
  for (int e = 0; e < NE; e++) {
    const int t = threadIdx.x + e * BLOCK;
    if (t < KK) out[t] = acc[e];
  }
}

// fp32 builds on MFMA (v_mfma_f32_32x32x2f32, the k_col_gram32 operand
// layout: a row pair r = 2s + lane/32 is the K dimension, lane l holds
// w_r q_r[l % 32] as the A and q_r[l % 32] as the B operand).  One wave per
// chunk (the host cuts a long row or column into up to 64 chunks, so a
// popular item's ~10^4 positions spread over many waves); the chunk's rows
// 32 at a time: one coalesced load of their indices and weights, the row
// loads all in flight, then 16 MFMAs alternating over two accumulator sets.
// Small batches keep the kernel at ~70 VGPRs (KP = 32), so several waves
// per SIMD hide each other's load latency (a software-pipelined 64-row
// version at 232 registers ran 3x slower).  KP = 32: one 32 x 32 tile.
// KP = 64: tiles 00, 01 and 11 (G is symmetric; tile 10 is stored as the
// transpose of 01).
constexpr int HOT_CHUNK_MAX = 256;
template <int KP>
__global__ __launch_bounds__(BLOCK) void k_hot_gram_mfma(uint64_t nchunks, const Job *__restrict__ chunks,
                                                         const uint32_t *__restrict__ ycol,
                                                         const float *__restrict__ wts,
                                                         const float *__restrict__ Q1, uint64_t q1rows,
                                                         float *__restrict__ G, float *__restrict__ gpart,
                                                         const float *__restrict__ xsq, const float *__restrict__ QTQ,
                                                         float w) {
  static_assert(KP == 32 || KP == 64, "MFMA hot Grams: KP 32 or 64");
  typedef float f16x __attribute__((ext_vector_type(16)));
  constexpr int T = KP / 32, NT = T == 1 ? 1 : 3, NA = 2, HB = 32, NS = HB / 2;
  const int lane = threadIdx.x & 63;
  const uint64_t wv = ((uint64_t)blockIdx.x * BLOCK + threadIdx.x) >> 6;
  if (wv >= nchunks) return;
  const Job jb = chunks[wv];
  const BufView qb = buf_view(Q1, q1rows * KP * 4);
  const int e = lane & 31, hf = lane >> 5;
  f16x acc[NA][NT];
#pragma unroll
  for (int u = 0; u < NA; u++)
#pragma unroll
    for (int a = 0; a < NT; a++)
#pragma unroll
      for (int r = 0; r < 16; r++) acc[u][a][r] = 0.0f;
  for (int64_t b0 = jb.b; b0 < jb.e; b0 += HB) {
    const int n = (int)(jb.e - b0 < HB ? jb.e - b0 : HB);
    const uint32_t il = lane < n ? ycol[b0 + lane] : 0u;
    const float wl = lane < n ? (wts ? wts[b0 + lane] : 1.0f) : 0.0f;
    float q0[NS], q1[T == 1 ? 1 : NS], w[NS];
#pragma unroll
    for (int s = 0; s < NS; s++) {
      const int r = 2 * s + hf;  // rows past n read zero (buffer range check)
      const uint32_t i = (uint32_t)__shfl((int)il, r, 64);
      w[s] = __shfl(wl, r, 64);
      const uint32_t off = r < n ? i * (uint32_t)(KP * 4) + (uint32_t)e * 4u : 0xffffffffu;
      q0[s] = bld1<float>(qb, off);
      if constexpr (T == 2) q1[s] = bld1<float>(qb, r < n ? off + 128u : 0xffffffffu);
    }
    // branch-free: rows past n are zero (weight and row), so their MFMAs add
    // nothing (a per-MFMA branch made the compiler copy the accumulators
    // between AGPRs and VGPRs around every one of them)
#pragma unroll
    for (int s = 0; s < NS; s++) {
      f16x(&c)[NT] = acc[s % NA];
      const float a0 = w[s] * q0[s];
      c[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, q0[s], c[0], 0, 0, 0);
      if constexpr (T == 2) {
        c[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, q1[s], c[1], 0, 0, 0);
        c[2] = __builtin_amdgcn_mfma_f32_32x32x2f32(w[s] * q1[s], q1[s], c[2], 0, 0, 0);
      }
    }
  }
#pragma unroll
  for (int u = 1; u < NA; u++)
#pragma unroll
    for (int a = 0; a < NT; a++) acc[0][a] += acc[u][a];
  float *out = jb.nparts <= 1 ? G + (size_t)jb.col * KP * KP : gpart + (size_t)jb.slot * KP * KP;
  // per-column cross Grams: the column tau w xsq_c QTQ, added once (by the
  // column's first chunk; the slot sum carries it)
  const float tw = (xsq && jb.flags == 0) ? w * xsq[jb.col] : 0.0f;
  auto tau = [&](int m, int nn) { return xsq ? tw * QTQ[m * KP + nn] : 0.0f; };
  // D register r of lane l: element m = 8(r/4) + 4(l/32) + r%4, n = l%32
#pragma unroll
  for (int r = 0; r < 16; r++) {
    const int m = 8 * (r >> 2) + 4 * hf + (r & 3);
    out[m * KP + e] = acc[0][0][r] + tau(m, e);
    if constexpr (T == 2) {
      out[m * KP + 32 + e] = acc[0][1][r] + tau(m, 32 + e);               // tile 01: rows 0..31, columns 32..63
      out[(32 + e) * KP + m] = acc[0][1][r] + tau(32 + e, m);             // tile 10 = 01^T
      out[(32 + m) * KP + 32 + e] = acc[0][2][r] + tau(32 + m, 32 + e);  // tile 11
    }
  }
}

// The fp64 build at KP = 32 on the f64 matrix cores (v_mfma_f64_16x16x4f64,
// MI355X guide: A lane l = A[m = l%16][k = l/16], B lane l = B[k = l/16][n =
// l%16], D register r of lane l = element (row l/16 + 4r, column l%16)): four
// positions are the K dimension, lane l holds w_r q_r[16t + l%16] / q_r[16t +
// l%16] of position r = l/16 of the group; 32 positions per batch (one
// coalesced index / weight load), tiles 00, 01 and 11 of the symmetric 32 x 32
// Gram (10 stored as 01^T), two accumulator sets; the column tau added by the
// column's first chunk as in k_hot_gram_mfma.
static __global__ __launch_bounds__(BLOCK) void k_hot_gram_mfma_f64(uint64_t nchunks, const Job *__restrict__ chunks,
                                                            const uint32_t *__restrict__ ycol,
                                                            const double *__restrict__ wts,
                                                            const double *__restrict__ Q1, uint64_t q1rows,
                                                            double *__restrict__ G, double *__restrict__ gpart,
                                                            const double *__restrict__ xsq,
                                                            const double *__restrict__ QTQ, double w) {
  typedef double d4 __attribute__((ext_vector_type(4)));
  constexpr int KP = 32, HB = 32, NG = HB / 4, NA = 2;
  const int lane = threadIdx.x & 63;
  const uint64_t wv = ((uint64_t)blockIdx.x * BLOCK + threadIdx.x) >> 6;
  if (wv >= nchunks) return;
  const Job jb = chunks[wv];
  const BufView qb = buf_view(Q1, q1rows * KP * 8);
  const int c16 = lane & 15, rq = lane >> 4;
  d4 acc[NA][3];
#pragma unroll
  for (int u = 0; u < NA; u++)
#pragma unroll
    for (int a = 0; a < 3; a++) acc[u][a] = d4{0.0, 0.0, 0.0, 0.0};
  for (int64_t b0 = jb.b; b0 < jb.e; b0 += HB) {
    const int n = (int)(jb.e - b0 < HB ? jb.e - b0 : HB);
    const uint32_t il = lane < n ? ycol[b0 + lane] : 0u;
    const double wl = lane < n ? (wts ? wts[b0 + lane] : 1.0) : 0.0;
    double q0[NG], q1[NG], wg[NG];
#pragma unroll
    for (int g = 0; g < NG; g++) {
      const int r = 4 * g + rq;  // positions past n read zero (buffer range check)
      const uint32_t i = (uint32_t)__shfl((int)il, r, 64);
      wg[g] = __shfl(wl, r, 64);
      const uint32_t off = r < n ? i * (uint32_t)(KP * 8) + (uint32_t)c16 * 8u : 0xffffffffu;
      q0[g] = bld1<double>(qb, off);
      q1[g] = bld1<double>(qb, r < n ? off + 128u : 0xffffffffu);
    }
#pragma unroll
    for (int g = 0; g < NG; g++) {
      d4(&c)[3] = acc[g % NA];
      const double a0 = wg[g] * q0[g], a1 = wg[g] * q1[g];
      c[0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, q0[g], c[0], 0, 0, 0);
      c[1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, q1[g], c[1], 0, 0, 0);
      c[2] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, q1[g], c[2], 0, 0, 0);
    }
  }
#pragma unroll
  for (int u = 1; u < NA; u++)
#pragma unroll
    for (int a = 0; a < 3; a++) acc[0][a] += acc[u][a];
  double *out = jb.nparts <= 1 ? G + (size_t)jb.col * KP * KP : gpart + (size_t)jb.slot * KP * KP;
  const double tw = (xsq && jb.flags == 0) ? w * xsq[jb.col] : 0.0;
  auto tau = [&](int m, int nn) { return xsq ? tw * QTQ[m * KP + nn] : 0.0; };
#pragma unroll
  for (int r = 0; r < 4; r++) {
    const int m = rq + 4 * r;
    out[m * KP + c16] = acc[0][0][r] + tau(m, c16);
    out[m * KP + 16 + c16] = acc[0][1][r] + tau(m, 16 + c16);
    out[(16 + c16) * KP + m] = acc[0][1][r] + tau(16 + c16, m);
    out[(16 + m) * KP + 16 + c16] = acc[0][2][r] + tau(16 + m, 16 + c16);
  }
}

// Per-column cross Grams: C_c += w xsq_c QTQ, the column tau
// term folded in, so a CG step is C_c p_c alone (k_hv_cgram).
template <typename real, int KP>
__global__ __launch_bounds__(BLOCK) void k_gram_add_tau(uint64_t D, real *__restrict__ G, const real *__restrict__ xsq,
                                                        const real *__restrict__ QTQ, double w) {
  constexpr int KK = KP * KP;
  for (uint64_t t = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; t < D * KK; t += (uint64_t)gridDim.x * BLOCK)
    G[t] += (real)(w * (double)xsq[t / KK]) * QTQ[t % KK];
}

// Per-column cross Grams, their positions in column order (set up once per
// field): key[p] = the column of position p's row (a one-node field),
// then (after a stable sort of the keys) cpos[t] = partner row of the t-th
// position, cw[t] = (1 - w) x^2 of its row.
static __global__ __launch_bounds__(BLOCK) void k_pos_colkey(uint64_t P, const uint32_t *__restrict__ rid,
                                                      const uint32_t *__restrict__ xidx, uint32_t *__restrict__ key) {
  const uint64_t p = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
  if (p < P) key[p] = xidx[rid[p]];
}
template <typename real>
__global__ __launch_bounds__(BLOCK) void k_ccg_gather(uint64_t P, const uint32_t *__restrict__ perm,
                                                      const uint32_t *__restrict__ rid, const uint32_t *__restrict__ ycol,
                                                      const real *__restrict__ xval, double w, uint32_t *__restrict__ cpos,
                                                      real *__restrict__ cw) {
  const uint64_t t = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
  if (t >= P) return;
  const uint32_t p = perm[t];
  const double x = (double)xval[rid[p]];
  cpos[t] = ycol[p];
  cw[t] = (real)((1 - w) * x * x);
}

// G of a multi-chunk row = its partial slots summed in slot order (sums:
// Job{col = Gram slot, nparts, slot = first partial slot}); blockIdx.x: the
// Gram, blockIdx.y: a range of BLOCK of its elements (a column of a few
// hundred chunks keeps one element per thread in flight).
template <typename real, int KP>
__global__ __launch_bounds__(BLOCK) void k_hot_slot_sum(const Job *__restrict__ sums, const real *__restrict__ gpart,
                                                        real *__restrict__ G) {
  constexpr int KK = KP * KP, GB = 8;
  const Job jb = sums[blockIdx.x];
  for (int t = blockIdx.y * BLOCK + threadIdx.x; t < KK; t += gridDim.y * BLOCK) {
    const real *src = gpart + (size_t)jb.slot * KK + t;
    real acc = src[0];
    for (uint32_t q0 = 1; q0 < jb.nparts; q0 += GB) {
      real y[GB];
#pragma unroll
      for (int u = 0; u < GB; u++) y[u] = q0 + u < jb.nparts ? src[(size_t)(q0 + u) * KK] : (real)0;
#pragma unroll
      for (int u = 0; u < GB; u++)
        if (q0 + u < jb.nparts) acc += y[u];
    }
    G[(size_t)jb.col * KK + t] = acc;
  }
}

// One CG step of a Gram side half: per column, the direction p_c of
// iteration f.it (formed from r, Hp, p as col_finalize does), s = G_c p_c,
// then the Hessian-vector finalisation (MODE 1), or s stored into f.acc for
// the all-reduce of several ranks (MODE 2: the Grams are partials over this
// rank's positives and rows).  One column per subgroup.  own (an owned
// field on several ranks): this rank's columns only, whose Grams are whole
// here; the dot products go to f.dots for the all-reduce (fin_blocks).
template <typename real, int KP, int MODE = 1>
__global__ __launch_bounds__(BLOCK) void k_hv_cgram(uint64_t D, const real *__restrict__ G, Fin<real> f,
                                                    const uint8_t *__restrict__ own = nullptr) {
  using Gm = Geo<real, KP>;
  if (!f.st->run[f.it]) return;
  const bool upd = f.it > 1;
  const real alpha = upd ? (real)f.st->alpha : (real)0, beta = upd ? (real)f.st->beta : (real)0;
  WAVE_SETUP
  const int sg = lane / Gm::LPR, li = lane % Gm::LPR;
  double dsum[3] = {0, 0, 0};
  for (uint64_t c = wave * Gm::NSG + sg; c < D; c += nwaves * Gm::NSG) {
    if (own && !own[c]) continue;
    const FinOps<real> ops = fin_load<real, KP, 1>(f, (uint32_t)c, upd, li);
    vec_t<real> pt = ops.w_or_p;
    if (upd) pt = (ops.r - vsplat<real>(alpha) * ops.hp) + vsplat<real>(beta) * ops.w_or_p;
    // KP >= 64: the product rolled (16 rows of G in flight; unrolled it took
    // 624 registers at KP = 64, one wave per SIMD with spills)
    vec_t<real> s;
    if constexpr (KP >= 64) s = sg_vecmat_rolled<real, KP, 4>(pt, G + c * KP * KP, li);
    else s = sg_vecmat<real, KP>(pt, G + c * KP * KP, li);
    if constexpr (MODE == 2) vst<real>(f.acc + c * KP + li * Gm::VE, s);
    else col_finalize<real, KP, 1>(f, (uint32_t)c, s, alpha, beta, upd, li, dsum, ops);
  }
  if constexpr (MODE != 2) fin_blocks<real, 1>(f, dsum);
}

// ------------------------------------------------------- pair Grams ---
// Side halves of a low-cardinality field with several nodes per row (the
// kkbox context field: 120 features, two per row; round 5, OCFFM_PGRAM).
// The field block of the side Hessian (hs_side, ffm.cpp:594-628) is
//   (H v)_a = sum_b G_ab v_b,  G_ab = sum_{i: X_ia X_ib != 0} d_i X_ia X_ib q_i q_i^T,
// one k x k Gram per feature pair (a <= b) present in some row, built once
// per half (k_col_gram* with pair weights).  A CG step is then ONE launch
// instead of the row pass over every row plus a feature pass whose heavy
// columns (~500 rows each) cost a chain of dependent rounds (~21 us per
// step): block a sums G_ab p_b over feature a's pairs (its subgroups split
// the adjacency list, p_b formed on the fly from the read-only CG vectors),
// stores s_a (sc1, drained) and takes a ticket; the last block to arrive
// finalises every column (col_finalize: the CG vectors are written only
// once nobody reads them) and publishes the CG scalars itself.  FIN false
// (many features): s into acc only, k_fin finalises.
// QB blocks per feature split its adjacency (about one entry per subgroup:
// one round of loads), each storing its partial slot acc[a QB + q]; the last
// block sums a feature's QB slots in slot order.
template <typename real, int KP, bool FIN>
__global__ __launch_bounds__(BLOCK) void k_pg_step(uint64_t D, uint32_t QB, const int64_t *__restrict__ aptr,
                                                   const uint32_t *__restrict__ apair,
                                                   const uint32_t *__restrict__ aoth, const real *__restrict__ G,
                                                   real *__restrict__ part, Fin<real> f) {
  using Gm = Geo<real, KP>;
  if (!f.st->run[f.it]) return;
  const bool upd = f.it > 1;
  const real alpha = upd ? (real)f.st->alpha : (real)0, beta = upd ? (real)f.st->beta : (real)0;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int sg = lane / Gm::LPR, li = lane % Gm::LPR;
  const int sid = w * Gm::NSG + sg;
  __shared__ __align__(16) real red[BLOCK / 64][KP];
  for (uint64_t bq = blockIdx.x; bq < D * QB; bq += gridDim.x) {
    const uint64_t a = bq / QB;
    const int64_t t0 = aptr[a], t1 = aptr[a + 1];
    vec_t<real> s = vzero<real>();
    for (int64_t t = t0 + (int64_t)(bq % QB) * 4 * Gm::NSG + sid; t < t1; t += (int64_t)QB * 4 * Gm::NSG) {
      const uint32_t p = apair[t], b = aoth[t];
      const vec_t<real> vb = cg_dir_at<real, KP>(f.P, f.R, f.Hp, alpha, beta, upd, (size_t)b * KP + li * Gm::VE);
      const real *Gp = G + (size_t)p * KP * KP;  // symmetric: G v = v G
      if constexpr (KP >= 64) s += sg_vecmat_rolled<real, KP, 4>(vb, Gp, li);
      else s += sg_vecmat<real, KP>(vb, Gp, li);
    }
    s = xsg_vsum<Gm::LPR, real>(s);
    if (sg == 0) *reinterpret_cast<vec_t<real> *>(&red[w][li * Gm::VE]) = s;
    __syncthreads();
    if (w == 0 && sg == 0) {  // the waves' sums in wave order
      vec_t<real> t = *reinterpret_cast<const vec_t<real> *>(&red[0][li * Gm::VE]);
#pragma unroll
      for (int q = 1; q < BLOCK / 64; q++) t += *reinterpret_cast<const vec_t<real> *>(&red[q][li * Gm::VE]);
#pragma unroll
      for (int e = 0; e < Gm::VE; e++)
        __hip_atomic_store(part + bq * KP + li * Gm::VE + e, t[e], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
  }
  if (w == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this block's partial slots landed
  __syncthreads();
  const double z[1] = {0.0};
  double tz[1];
  if (!last_block<1>(z, f.part, f.tick, tz)) return;
  // the last block: each feature's slots in order, then (FIN) the
  // finalisation of every column and the CG scalars, else s into acc
  const BufView pb = buf_view(part, D * QB * KP * sizeof(real));
  double dsum[3] = {0, 0, 0};
  for (uint64_t q = threadIdx.x; q < D * Gm::LPR; q += BLOCK) {
    const uint32_t c = (uint32_t)(q / Gm::LPR);
    const int l = (int)(q % Gm::LPR);
    FinOps<real> ops;
    if constexpr (FIN) ops = fin_load<real, KP, 1>(f, c, upd, l);
    vec_t<real> sv = vzero<real>();
    for (uint32_t u = 0; u < QB; u++)
      sv += bld_sc1<real>(pb, (uint32_t)((((size_t)c * QB + u) * KP + l * Gm::VE) * sizeof(real)));
    if constexpr (FIN) col_finalize<real, KP, 1>(f, c, sv, alpha, beta, upd, l, dsum, ops);
    else vst<real>(f.acc + (size_t)c * KP + l * Gm::VE, sv);
  }
  if constexpr (FIN) {
    double tot[3] = {block_sum(dsum[0]), block_sum(dsum[1]), block_sum(dsum[2])};
    if (threadIdx.x == 0) {
      if (f.dots) {
#pragma unroll
        for (int k = 0; k < 3; k++) f.dots[k] = tot[k];
      } else {
        cg_publish<real, 1>(f, tot);
      }
    }
  }
}

// ------------------------------------------ persistent column-Gram CG ---
// Every CG step of a half whose Hessian-vector product is the D column
// Grams (k_hv_cgram: the genre / artist side halves, the column-Gram cross
// halves; ffm.cpp:761-812) in ONE launch (round 5, OCFFM_CGP): a step is
// each column's s = G_c p_c and its finalisation by the column's fixed
// owner (so no vector crosses a block), the grid's dot products by the
// last-arriving block (last_block), which publishes alpha, beta and the
// verdict (the same arithmetic as cg_publish, through agent-scope stores)
// and then releases the grid through a generation word that the other
// blocks poll (bounded spin); the next step reads the scalars with
// agent-scope loads.  No host round trip or kernel boundary between steps.
//
// Co-residency (round 6).  The host checks the grid against the occupancy
// API (at most one block per CU) and can launch it cooperatively
// (OCFFM_CGP_COOP=1: the runtime's own check, measured +0.27 ms per kkbox
// epoch of host launch cost, nothing more: a plain launch of the same grid
// has the same residency).  Neither stops another process's kernels from
// holding CUs or the queue from being time-sliced, so the barrier is made
// safe to give up: the generation word is released and aborted by
// compare-and-swap.  A
// waiter that spins past `spin_max` swaps the unreleased word for CGP_ABORT;
// the last block of the step swaps in the release.  Exactly one of the two
// wins.  Every block always finishes the step it is in and takes its
// ticket (the tickets reset themselves), and the last block publishes the
// step's scalars and verdict BEFORE its swap, so an abort at barrier `it`
// leaves every column at step `it` with the scalars of step `it` in
// CgState: exactly the state the two-launch path (k_hv_cgram) continues
// from at step it+1.  The abort is reported as it + 1 in the host-mapped
// word and as 1 in `abort_dev`, which guards the update kernels queued
// behind this launch (they return at entry); the host then resets both
// words and the generation word and finishes the solve per step.
// stall_step (tests only): the grid's last block sleeps before the column
// work of that step, long enough for the others to give up.
constexpr unsigned CGP_ABORT = 0xffffffffu;
// Memory ordering.  Everything that crosses blocks inside the launch is an
// agent-scope (sc1) atomic on both sides — the partial dot products and
// tickets (last_block), the CG scalars and verdicts (ast / ald), the
// generation word — and every storing wave drains vmcnt before its ticket
// or the release (MI355X guide, Consumer bullet conditions 1-4); the CG
// vectors are only ever touched by the block that owns the column.  So no
// L2 write-back / invalidate is needed at the barrier.  -DOCFFM_CGP_FENCE=1
// adds an agent release fence before the release and an acquire fence
// after it (for plain stores read across blocks, should any be added):
// measured +0.07 ms per kkbox epoch (a write-back of the XCD's dirty L2 per
// step).
#ifndef OCFFM_CGP_FENCE
#define OCFFM_CGP_FENCE 0
#endif
__device__ __forceinline__ void cgp_report_abort(int *err_host, int *abort_dev, int it) {
  __hip_atomic_store(abort_dev, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(err_host, it + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);  // step + 1: never 0
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
__device__ __forceinline__ double ald(const double *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int ald(const int *p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ void ast(double *p, double v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void ast(int *p, int v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
constexpr unsigned CGP_SPIN_MAX = 1u << 22;  // ~0.1 s of s_sleep 1: then the grid gives up (recoverable)
template <typename real, int KP>
__global__ __launch_bounds__(BLOCK) void k_cg_cgram(uint64_t D, const real *__restrict__ G, Fin<real> f,
                                                    unsigned *__restrict__ gen, unsigned gen0, int *__restrict__ err_host,
                                                    int *__restrict__ abort_dev, unsigned spin_max, int stall_step,
                                                    int xcd_cols) {
  using Gm = Geo<real, KP>;
  const int lane = threadIdx.x & 63;
  const int sg = lane / Gm::LPR, li = lane % Gm::LPR;
  // XCD-ordered contiguous column ranges (round 6): the blocks of an XCD own
  // consecutive columns, so an XCD's share of the Grams (artist: 20 MB over
  // the 8 L2s) is re-read from its own L2 at every step
  const unsigned L = (gridDim.x & 7u) ? blockIdx.x : xcd_work_item(blockIdx.x, gridDim.x);
  const uint64_t cpb = (D + gridDim.x - 1) / gridDim.x;  // columns per block
  const uint64_t c0 = (uint64_t)L * cpb, c1 = c0 + cpb < D ? c0 + cpb : D;
  const int sid = (threadIdx.x >> 6) * Gm::NSG + sg;
  CgState *st = f.st;
  __shared__ int s_ok;
  for (int it = 1; it <= MAXCG; it++) {
    if (!ald(&st->run[it])) return;  // the same word for every block (read after the barrier)
    const bool upd = it > 1;
    const real alpha = upd ? (real)ald(&st->alpha) : (real)0, beta = upd ? (real)ald(&st->beta) : (real)0;
    f.it = it;
    if (it == stall_step && blockIdx.x == gridDim.x - 1 && gridDim.x > 1)
      for (int q = 0; q < 4000; q++) __builtin_amdgcn_s_sleep(127);
    double dsum[3] = {0, 0, 0};
    const uint64_t cb = xcd_cols ? c0 + sid : (uint64_t)blockIdx.x * (BLOCK / Gm::LPR) + sid;
    const uint64_t ce = xcd_cols ? c1 : D, cs = xcd_cols ? BLOCK / Gm::LPR : (uint64_t)gridDim.x * (BLOCK / Gm::LPR);
    for (uint64_t c = cb; c < ce; c += cs) {
      const FinOps<real> ops = fin_load<real, KP, 1>(f, (uint32_t)c, upd, li);
      vec_t<real> pt = ops.w_or_p;
      if (upd) pt = (ops.r - vsplat<real>(alpha) * ops.hp) + vsplat<real>(beta) * ops.w_or_p;
      vec_t<real> s;
      if constexpr (KP >= 64) s = sg_vecmat_rolled<real, KP, 4>(pt, G + c * KP * KP, li);
      else s = sg_vecmat<real, KP>(pt, G + c * KP * KP, li);
      col_finalize<real, KP, 1>(f, (uint32_t)c, s, alpha, beta, upd, li, dsum, ops);
    }
    double bv[3] = {block_sum(dsum[0]), block_sum(dsum[1]), block_sum(dsum[2])}, tot[3];
    if (last_block<3>(bv, f.part, f.tick, tot)) {
      if (threadIdx.x == 0) {
        // cg_publish MODE 1 (ffm.cpp:803-809) through agent-scope stores
        const double r2 = ald(&st->r2), g2 = ald(&st->g2);
        const double a = r2 / tot[0];
        const double r2n = r2 - 2 * a * tot[1] + a * a * tot[2];
        ast(&st->vhv, tot[0]);
        ast(&st->alpha, a);
        ast(&st->beta, r2n / r2);
        ast(&st->r2, r2n);
        ast(&st->nr_cg, it);
        const int go = (it < MAXCG && g2 * CG_EPS < r2n) ? 1 : 0;
        ast(&st->run[it + 1], go);
        if (f.run_host)
          __hip_atomic_store(f.run_host + it + 1, go ? RUN_GO : RUN_STOP, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every store above (and the tickets' reset) landed
        // release by swap: fails only if a waiter already gave up on this
        // barrier (fence: see OCFFM_CGP_FENCE above)
        if constexpr (OCFFM_CGP_FENCE) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        unsigned cur = __hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        int ok = 0;
        while (cur != CGP_ABORT) {
          if (__hip_atomic_compare_exchange_strong(gen, &cur, gen0 + (unsigned)it, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_AGENT)) {
            ok = 1;
            break;
          }
        }
        if (!ok) cgp_report_abort(err_host, abort_dev, it);
        s_ok = ok;
      }
      __syncthreads();
      if (!s_ok) return;
    } else {
      if (threadIdx.x == 0) {
        int ok = 1;
        unsigned spins = 0;
        for (;;) {
          // relaxed sc1 polls (an acquire per poll would invalidate this
          // CU's L1 every time)
          unsigned cur = __hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (cur == gen0 + (unsigned)it) {  // released
            if constexpr (OCFFM_CGP_FENCE) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            break;
          }
          if (cur == CGP_ABORT) {                 // another waiter gave up
            ok = 0;
            break;
          }
          __builtin_amdgcn_s_sleep(1);
          if (++spins > spin_max &&
              __hip_atomic_compare_exchange_strong(gen, &cur, CGP_ABORT, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_AGENT)) {
            cgp_report_abort(err_host, abort_dev, it);
            ok = 0;
            break;
          }
        }
        s_ok = ok;
      }
      __syncthreads();
      if (!s_ok) return;
    }
  }
}

// The release / give-up barrier of the persistent CG kernels (k_cg_cgram
// above; k_cg_side_id below), run by every block after its share of step
// `it`: the last-arriving block publishes the CG scalars of the step
// (cg_publish MODE 1, ffm.cpp:803-809, through agent-scope stores) and
// releases the grid; the others wait (see the co-residency notes above).
// Returns false when the grid gave up (every block then leaves).
// MODE 0 (it = 0, a fused gradient): publishes g2 = r2 = |G|^2 and the
// first verdict as cg_publish MODE 0 does (ffm.cpp:773-780).
template <typename real, int MODE = 1>
__device__ __forceinline__ bool cgp_step_end(const Fin<real> &f, const double (&dsum)[3], int it, unsigned *gen,
                                             unsigned gen0, int *err_host, int *abort_dev, unsigned spin_max) {
  __shared__ int s_ok;
  CgState *st = f.st;
  double bv[3] = {block_sum(dsum[0]), block_sum(dsum[1]), block_sum(dsum[2])}, tot[3];
  if (last_block<3, 1>(bv, f.part, f.tick, tot)) {  // (a short read-back round: the caller holds state in registers)
    if (threadIdx.x == 0) {
      int go;
      if constexpr (MODE == 0) {
        ast(&st->g2, tot[0]);
        ast(&st->r2, tot[0]);
        ast(&st->nr_cg, 0);
        for (int q = 0; q <= MAXCG + 1; q++) ast(&st->run[q], 0);
        go = (tot[0] * CG_EPS < tot[0]) ? 1 : 0;
        ast(&st->run[1], go);
      } else {
        const double r2 = ald(&st->r2), g2 = ald(&st->g2);
        const double a = r2 / tot[0];
        const double r2n = r2 - 2 * a * tot[1] + a * a * tot[2];
        ast(&st->vhv, tot[0]);
        ast(&st->alpha, a);
        ast(&st->beta, r2n / r2);
        ast(&st->r2, r2n);
        ast(&st->nr_cg, it);
        go = (it < MAXCG && g2 * CG_EPS < r2n) ? 1 : 0;
        ast(&st->run[it + 1], go);
      }
      if (f.run_host)
        __hip_atomic_store(f.run_host + it + 1, go ? RUN_GO : RUN_STOP, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if constexpr (OCFFM_CGP_FENCE) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      unsigned cur = __hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      int ok = 0;
      while (cur != CGP_ABORT) {
        if (__hip_atomic_compare_exchange_strong(gen, &cur, gen0 + (unsigned)it, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT)) {
          ok = 1;
          break;
        }
      }
      if (!ok) cgp_report_abort(err_host, abort_dev, it);
      s_ok = ok;
    }
  } else if (threadIdx.x == 0) {
    int ok = 1;
    unsigned spins = 0;
    for (;;) {
      unsigned cur = __hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (cur == gen0 + (unsigned)it) {
        if constexpr (OCFFM_CGP_FENCE) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        break;
      }
      if (cur == CGP_ABORT) {
        ok = 0;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
      if (++spins > spin_max &&
          __hip_atomic_compare_exchange_strong(gen, &cur, CGP_ABORT, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT)) {
        cgp_report_abort(err_host, abort_dev, it);
        ok = 0;
        break;
      }
    }
    s_ok = ok;
  }
  __syncthreads();
  return s_ok != 0;
}

// Persistent CG of a side half over an id-like field (round 6): every
// CG step of the half in ONE launch with the CG vectors in registers.  An
// id-like field's Hessian-vector product is row-local (row i is column
// xidx[i]'s only row: hs_side, ffm.cpp:594-628, is k_hs_side_row FUSE's
// d_i <x p, q_i> x q_i), so a block that owns a set of rows owns their
// columns' p, r, Hp and S for the whole solve: the steps read no vector
// from memory, only the CG scalars.  Block L (XCD-ordered) owns rows
// [L RB, (L+1) RB), RB = SMAX 4 NSG; subgroup sid holds rows L RB + s 4 NSG
// + sid, s < SMAX: p and r in registers, Hp and S in LDS (kkbox's song-id
// rows: 100 k rows x 2 x 128 B = 25.6 MB of the chip's 40 MB of LDS), q_i
// read each step (the blocks of an XCD own contiguous rows, so an XCD's q
// rows stay in its L2).  The state is loaded once after the gradient (R = P = -g,
// S = 0) and written back when the solve stops or the grid gives up on a
// barrier (then at step `it`: the state the per-step path continues from,
// solver.hip cgp_recover).  Per step the arithmetic is k_hs_side_row FUSE's
// and col_finalize MODE 1's, expression for expression; only the grouping of
// the grid's dot products differs.
//
// FULL (round 6): the whole side half in the launch.  Step 0 is the
// gradient (k_gd_side_seg with the row's sums (k_row_ysum) + the feature
// pass's col_finalize MODE 0 for the row's one column: G = lam f W + x z q_i,
// z = (1-w)(Y_i + n_i a_i) - n_i w (1-r) + w (n1 (a_i - r) + sum(b) + sa_i)),
// published at the barrier as
// cg_publish MODE 0 does; after the last step the update
// (k_update_side_row with apply_owned_row: s = S + a p, W += s, P1_i += x s,
// a_i += <x s, q_i>, the new sum of a to sh.asum).  A grid that gives up
// (at step 0 too) writes the state back and skips the update: the host
// continues per step and runs the update itself.
template <typename real> struct SideHalf {
  const real *yrow;        // per row: sum of base + partner bias over its positives (k_row_ysum)
  real *a1;                // this side's bias (updated)
  const real *sa1;
  const double *bsum;      // sum of the partner side's bias (read)
  double *asum;            // sum of this side's new bias (written)
  real *P1;
  double r;
};
template <typename real, int KP, int SMAX, bool FULL = false>
__global__ __launch_bounds__(BLOCK, sizeof(real) * SMAX <= 16 ? 4 : 2) void k_cg_side_id(uint64_t R, const uint32_t *__restrict__ xidx,
                                                         const real *__restrict__ xval,
                                                         const int64_t *__restrict__ cnt, const real *__restrict__ Q1,
                                                         double w, double n1, Fin<real> f, unsigned *__restrict__ gen,
                                                         unsigned gen0, int *__restrict__ err_host,
                                                         int *__restrict__ abort_dev, unsigned spin_max,
                                                         int stall_step, SideHalf<real> sh) {
  using Gm = Geo<real, KP>;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int sg = lane / Gm::LPR, li = lane % Gm::LPR;
  const unsigned L = (gridDim.x & 7u) ? blockIdx.x : xcd_work_item(blockIdx.x, gridDim.x);
  const uint64_t base = (uint64_t)L * SMAX * 4 * Gm::NSG + (uint64_t)(wv * Gm::NSG + sg);
  CgState *st = f.st;
  __shared__ vec_t<real> Sl[SMAX][BLOCK], Hl[SMAX][BLOCK];
  vec_t<real> p[SMAX], r[SMAX];
  real x[SMAX], dd[SMAX], reg[SMAX];
  uint32_t col[SMAX];
  const uint64_t nval = R > base ? (R - base + 4 * Gm::NSG - 1) / (4 * Gm::NSG) : 0;  // valid slots: s < nval
#pragma unroll
  for (int s = 0; s < SMAX; s++) {
    const uint64_t i = base + (uint64_t)s * 4 * Gm::NSG;
    const uint64_t ic = (uint64_t)s < nval ? i : 0;
    col[s] = xidx[ic];
    const size_t off = (size_t)col[s] * KP + li * Gm::VE;
    x[s] = xval[ic];
    dd[s] = (real)((1 - w) * (double)(cnt[ic + 1] - cnt[ic]) + w * n1);
    reg[s] = (real)(f.fw ? f.lam * (double)f.fw[col[s]] : f.lam);
    if constexpr (!FULL) {
      p[s] = vld<real>(f.P + off);
      r[s] = vld<real>(f.R + off);
      Sl[s][threadIdx.x] = vld<real>(f.S + off);
    }
    Hl[s][threadIdx.x] = vzero<real>();
  }
  int done = 0;  // steps computed
  bool gave_up = false;
  if constexpr (FULL) {  // step 0: the gradient
    const real cpos = (real)(1 - w), cneg = (real)(w * (1 - sh.r));
    const double bs = *sh.bsum;
    double dsum[3] = {0, 0, 0};
#pragma unroll
    for (int s = 0; s < SMAX; s++) {
      p[s] = r[s] = vzero<real>();
      Sl[s][threadIdx.x] = vzero<real>();
      if ((uint64_t)s >= nval) continue;
      const uint64_t i = base + (uint64_t)s * 4 * Gm::NSG;
      const real ai = sh.a1[i], n = (real)(cnt[i + 1] - cnt[i]);
      const real z = (cpos * (sh.yrow[i] + n * ai) - n * cneg) +
                     (real)(w * (n1 * ((double)ai - sh.r) + bs + (double)sh.sa1[i]));
      const size_t off = (size_t)col[s] * KP + li * Gm::VE;
      const vec_t<real> q = vld<real>(Q1 + i * KP + li * Gm::VE);
      const vec_t<real> g = vsplat<real>(reg[s]) * vld<real>(f.W + off) + vsplat<real>(x[s]) * (vsplat<real>(z) * q);
      if (f.G) vst<real>(f.G + off, g);
      r[s] = p[s] = -g;
#pragma unroll
      for (int e = 0; e < Gm::VE; e++) dsum[0] += (double)g[e] * (double)g[e];
    }
    if (stall_step == 0 && blockIdx.x == gridDim.x - 1 && gridDim.x > 1)
      for (int u = 0; u < 4000; u++) __builtin_amdgcn_s_sleep(127);
    gave_up = !cgp_step_end<real, 0>(f, dsum, 0, gen, gen0, err_host, abort_dev, spin_max);
  }
  for (int it = 1; it <= MAXCG && !gave_up; it++) {
    if (!ald(&st->run[it])) break;  // the same word for every block (read after the barrier)
    const bool upd = it > 1;
    const real alpha = upd ? (real)ald(&st->alpha) : (real)0, beta = upd ? (real)ald(&st->beta) : (real)0;
    if (it == stall_step && blockIdx.x == gridDim.x - 1 && gridDim.x > 1)
      for (int u = 0; u < 4000; u++) __builtin_amdgcn_s_sleep(127);
    double dsum[3] = {0, 0, 0};
#pragma unroll
    for (int s = 0; s < SMAX; s++) {
      if ((uint64_t)s >= nval) continue;
      uint64_t qrow = base + (uint64_t)s * 4 * Gm::NSG;
      asm volatile("" : "+v"(qrow));  // (the address is recomputed each step, not held)
      const vec_t<real> q = vld<real>(Q1 + qrow * KP + li * Gm::VE);
      const vec_t<real> hpo = Hl[s][threadIdx.x];
      vec_t<real> pt = p[s];
      if (upd) pt = (r[s] - vsplat<real>(alpha) * hpo) + vsplat<real>(beta) * p[s];
      const real z = sg_sum<Gm::LPR>(hsum<real>(vsplat<real>(x[s]) * pt * q));
      const vec_t<real> sum = vsplat<real>(x[s]) * (vsplat<real>(dd[s] * z) * q);
      // col_finalize MODE 1
      vec_t<real> rn = r[s], pe = p[s];
      if (upd) {
        rn = r[s] - vsplat<real>(alpha) * hpo;
        pe = rn + vsplat<real>(beta) * p[s];
        Sl[s][threadIdx.x] = Sl[s][threadIdx.x] + vsplat<real>(alpha) * p[s];
        r[s] = rn;
        p[s] = pe;
      }
      const vec_t<real> hpn = vsplat<real>(reg[s]) * pe + sum;
      Hl[s][threadIdx.x] = hpn;
#pragma unroll
      for (int e = 0; e < Gm::VE; e++) {
        dsum[0] += (double)pe[e] * (double)hpn[e];
        dsum[1] += (double)rn[e] * (double)hpn[e];
        dsum[2] += (double)hpn[e] * (double)hpn[e];
      }
      __builtin_amdgcn_sched_barrier(0);  // one slot at a time (the slots' temporaries are not live together)
    }
    done = it;
    if (!cgp_step_end<real>(f, dsum, it, gen, gen0, err_host, abort_dev, spin_max)) {
      gave_up = true;
      break;
    }
  }
  if constexpr (FULL) {
    if (!gave_up) {  // the update (the final step's S + a p)
      const real alpha = ald(&st->nr_cg) >= 1 ? (real)ald(&st->alpha) : (real)0;
      double bsn = 0;
#pragma unroll
      for (int s = 0; s < SMAX; s++) {
        if ((uint64_t)s >= nval) continue;
        uint32_t c = col[s];
        asm volatile("" : "+v"(c));
        const size_t off = (size_t)c * KP + li * Gm::VE;
        const uint64_t i = base + (uint64_t)s * 4 * Gm::NSG;
        const vec_t<real> sv = Sl[s][threadIdx.x] + vsplat<real>(alpha) * p[s];
        vst<real>(const_cast<real *>(f.W) + off, vld<real>(f.W + off) + sv);
        const vec_t<real> xs = vsplat<real>(x[s]) * sv;
        vst<real>(sh.P1 + i * KP + li * Gm::VE, vld<real>(sh.P1 + i * KP + li * Gm::VE) + xs);
        const real gap = sg_sum<Gm::LPR>(hsum<real>(xs * vld<real>(Q1 + i * KP + li * Gm::VE)));
        if (li == 0) {
          const real an = sh.a1[i] + gap;
          sh.a1[i] = an;
          bsn += (double)an;
        }
      }
      const double bv[1] = {block_sum(bsn)};
      double tot[1];
      if (last_block<1>(bv, f.part, f.tick, tot) && threadIdx.x == 0) sh.asum[0] = tot[0];
      return;
    }
  }
  // the state back where the per-step path and the update read it
  if (!FULL && done == 0) return;
#pragma unroll
  for (int s = 0; s < SMAX; s++) {
    if ((uint64_t)s >= nval) continue;
    uint32_t c = col[s];
    asm volatile("" : "+v"(c));  // recompute the addresses here (else the prologue's stay live in registers)
    const size_t off = (size_t)c * KP + li * Gm::VE;
    vst<real>(f.S + off, Sl[s][threadIdx.x]);
    vst<real>(f.R + off, r[s]);
    vst<real>(f.P + off, p[s]);
    vst<real>(f.Hp + off, Hl[s][threadIdx.x]);
  }
}

// Cross Hessian-vector product of an id-like field, fused with its
// finalisation (round 6; one GPU): row i is column c = xidx[i]'s only row,
// so the feature pass of hs_cross (ffm.cpp:715-742, then 783-809) reduces
// to the row itself, as k_hs_side_row FUSE does for side halves:
//   Hp_c = lam f pt_c + x_i ((1-w) sum_{j in pos(i)} <phi, q_j> q_j + w phi QTQ),
//   phi = x_i pt_c,
// one launch per CG step instead of k_hs_cross_seg + k_feat.  The gathers
// are k_hs_cross_seg's over the row's positives; the tau term takes QTQ
// from LDS (k_feat TAU's per-column form); a hot row (hot_row[i] !=
// HOT_NONE: more positives than one gather pass) reads its Gram
// G_i = sum_j q_j q_j^T (k_hot_gram, built for the half), so no subgroup
// walks a popular item's thousands of positives.
template <typename real, int KP> constexpr bool xfuse_kp() { return KP <= 64; }  // (QTQ in LDS)
// XGB: gathers per round (8: 4 waves per SIMD at <= 128 registers; 16:
// the compiler's choice, ~166 registers)
template <typename real, int KP, int XGB = 8>
__global__ __launch_bounds__(BLOCK, XGB >= 16 ? 1 : 4) void k_hv_cross_id(
    uint64_t R, const uint32_t *__restrict__ xidx, const real *__restrict__ xval, const int64_t *__restrict__ yptr,
    const uint32_t *__restrict__ ycol, const real *__restrict__ Q1, uint64_t q1rows, const real *__restrict__ QTQ,
    double w, const uint32_t *__restrict__ hot_row, const real *__restrict__ hotG, Fin<real> f) {
  using G = Geo<real, KP>;
  using PP = PosPass<real, KP, sizeof(real) == 8 ? XGB / 2 : XGB, 32>;
  if constexpr (!xfuse_kp<real, KP>()) return;
  if (!f.st->run[f.it]) return;
  const BufView qb = buf_view(Q1, q1rows * KP * sizeof(real));
  __shared__ __align__(16) real Qs[xfuse_kp<real, KP>() ? KP * KP : 1];
  for (int t = threadIdx.x; t < KP * KP; t += BLOCK) Qs[t] = QTQ[t];
  __syncthreads();
  const bool upd = f.it > 1;
  const real alpha = upd ? (real)f.st->alpha : (real)0, beta = upd ? (real)f.st->beta : (real)0;
  const real cpos = (real)(1 - w), wr = (real)w;
  WAVE_SETUP
  const int sg = lane / G::LPR, li = lane % G::LPR;
  double dsum[3] = {0, 0, 0};
  // the next row's descriptor in flight while this one is processed (a
  // resident grid, OCFFM_ROW_FILL, walks several rows per subgroup)
  const uint64_t stride = nwaves * G::NSG;
  uint32_t nc = 0, nh = HOT_NONE;
  real nx = 0;
  int64_t nb = 0, ne = 0;
  auto fetch = [&](uint64_t q) {
    nc = xidx[q];
    nx = xval[q];
    nb = yptr[q];
    ne = yptr[q + 1];
    if (hot_row) nh = hot_row[q];
  };
  if (wave * G::NSG + sg < R) fetch(wave * G::NSG + sg);
  for (uint64_t i = wave * G::NSG + sg; i < R; i += stride) {
    const uint32_t c = nc, hs = nh;
    const real x = nx;
    const int64_t b = nb, e = ne;
    if (i + stride < R) fetch(i + stride);
    uint32_t jj[PP::UT];  // the first pass's columns go out with the finalisation operands
    if (hs == HOT_NONE) PP::load_cols(ycol, b, e, li, jj);
    // col_finalize MODE 1's update part first (it does not depend on the
    // product): S += a p, r -= a Hp, p = r + b p; then only p (= pt) and r
    // stay live across the gathers
    const size_t off = (size_t)c * KP + li * G::VE;
    const real reg = (real)(f.fw ? f.lam * (double)f.fw[c] : f.lam);
    vec_t<real> pt = vld<real>(f.P + off), rn = vld<real>(f.R + off);
    if (upd) {
      const vec_t<real> hp = vld<real>(f.Hp + off), so = vld<real>(f.S + off);
      vst<real>(f.S + off, so + vsplat<real>(alpha) * pt);
      rn = rn - vsplat<real>(alpha) * hp;
      pt = rn + vsplat<real>(beta) * pt;
      vst<real>(f.R + off, rn);
      vst<real>(f.P + off, pt);
    }
    const vec_t<real> phi = vsplat<real>(x) * pt;
    vec_t<real> ka = vzero<real>();
    if (hs != HOT_NONE) {
      ka = sg_vecmat_rolled<real, KP>(phi, hotG + (size_t)hs * KP * KP, li);
    } else {
      for (int64_t p0 = b; p0 < e; p0 += PP::PW) {
        if (p0 != b) PP::load_cols(ycol, p0, e, li, jj);
        sfor<PP::PW / PP::GB>([&](auto BT) {
          constexpr int bt = decltype(BT)::value * PP::GB;
          if (p0 + bt >= e) return;
          vec_t<real> qv[PP::GB];
          sfor<PP::GB>([&](auto U) {
            constexpr int u = decltype(U)::value;
            qv[u] = bld<real>(qb, PP::row_off(PP::template at<bt + u>(jj, li), qb, li));
          });
          real dv[PP::GB];
#pragma unroll
          for (int u = 0; u < PP::GB; u++) dv[u] = sg_sum<G::LPR>(hsum<real>(phi * qv[u]));
#pragma unroll
          for (int u = 0; u < PP::GB; u++) ka += vsplat<real>(dv[u]) * qv[u];
        });
      }
    }
    const vec_t<real> s =
        vsplat<real>(x) * (vsplat<real>(cpos) * ka + vsplat<real>(wr) * sg_vecmat_rolled<real, KP, 2>(phi, Qs, li));
    const vec_t<real> hp = vsplat<real>(reg) * pt + s;
    vst<real>(f.Hp + off, hp);
#pragma unroll
    for (int q = 0; q < G::VE; q++) {
      dsum[0] += (double)pt[q] * (double)hp[q];
      dsum[1] += (double)rn[q] * (double)hp[q];
      dsum[2] += (double)hp[q] * (double)hp[q];
    }
  }
  fin_blocks<real, 1>(f, dsum);
}

// Per segment of row i: h[s] = (1-w) sum_{j in seg} <phi_i, q_j> q_j
// + [first] w phi_i QTQ, phi_i = X_i p  (hs_cross row body, ffm.cpp:715-738;
// tau = X_i (V QTQ) = phi_i QTQ).  QTQ staged in LDS; phi_i's components
// are broadcast by DPP for the k x k product (sg_vecmat).
//
// TT (round 6; fp32, KP 16 / 32 / 64, rows with several nodes — one-node
// fields take tau per column in the feature pass instead): tau on the matrix
// cores.  The block walks SB = 4 NSG consecutive segments per iteration;
// each subgroup puts its phi (first segments; else zero) in an LDS tile and
// does its gathers, then the block's [phi rows] x QTQ product is cut into
// 16 x 16 tiles, one per wave, each a chain of KP / 4 v_mfma_f32_16x16x4f32
// (TMma's K order: A one 16-B LDS read of a phi row, B one 16-B read of QTQ
// staged as TMma::stage does), the tau tile goes back to LDS and each
// subgroup adds its row.  sg_vecmat had read QTQ once per row: KP 16-B LDS
// reads per lane and row (at k = 64 ~30 % of outbrain's user-half pass).
template <typename real, int KP> struct TauTile {
  using G = Geo<real, KP>;
  static constexpr bool OK = TMma<real, KP>::OK && std::is_same<real, float>::value;
  static constexpr int SB = 4 * G::NSG;                      // segments per block iteration
  static constexpr int TR = SB / 16, TC = KP / 16;           // 16 x 16 output tiles
  static constexpr int LD = KP + 4;                          // padded row stride (floats) of the phi / tau tiles
  static constexpr size_t bytes() { return (size_t)KP * KP * 4 + 2 * (size_t)SB * LD * 4; }
  static_assert(!OK || TR * TC <= 4 * ((TR * TC + 3) / 4), "tiles");
};
template <typename real, int KP, bool MLDS, int PW_ = 32, bool TT = false>
__global__ __launch_bounds__(BLOCK, sizeof(real) == 8 ? OCFFM_HS_OCC64 : OCFFM_HS_OCC) void k_hs_cross_seg(uint64_t nseg, const Seg *__restrict__ segs,
                                                        const int64_t *__restrict__ xptr,
                                                        const uint32_t *__restrict__ xidx,
                                                        const real *__restrict__ xval, const real *__restrict__ V,
                                                        const uint32_t *__restrict__ ycol,
                                                        const real *__restrict__ Q1, uint64_t q1rows,
                                                        const real *__restrict__ QTQ, double w, real *__restrict__ h,
                                                        const int *__restrict__ run, const real *__restrict__ Rv,
                                                        const real *__restrict__ Hv, const CgState *st, int it,
                                                        const uint32_t *__restrict__ segd,
                                                        const real *__restrict__ segx,
                                                        const uint32_t *__restrict__ hot_seg,
                                                        const real *__restrict__ hotG,
                                                        const uint32_t *__restrict__ sord) {
  using G = Geo<real, KP>;
  // gathers per round (32: one round per <= 32-positive segment); PW_ = 16
  // for sides whose segments are nearly all short (outbrain's users: ~1
  // positive each), so a round carries fewer absent slots
  using PP = PosPass<real, KP, sizeof(real) == 8 ? OCFFM_HS_GB64 : OCFFM_HS_GB, PW_>;
  const BufView qb = buf_view(Q1, q1rows * KP * sizeof(real));
  if (run && !*run) return;
  const bool upd = st && it > 1;
  const real alpha = upd ? (real)st->alpha : (real)0, beta = upd ? (real)st->beta : (real)0;
  extern __shared__ __align__(16) unsigned char smem_raw[];
  real *Qs = reinterpret_cast<real *>(smem_raw);
  const real *Qp = QTQ;
  if constexpr (TT) {
    TMma<real, KP>::stage(QTQ, 1, Qs);  // B operand layout (tau tiles)
    __syncthreads();
  } else if (MLDS) {  // QTQ null: the tau term is added per column by the feature pass (k_feat TAU)
    if (QTQ)
      for (int t = threadIdx.x; t < KP * KP; t += BLOCK) Qs[t] = QTQ[t];
    __syncthreads();
    Qp = Qs;
  }
  WAVE_SETUP
  const int sg = lane / G::LPR, li = lane % G::LPR;
  const real cpos = (real)(1 - w);
  // Per segment: phi from the row's node(s), the partner-row gathers, tau.
  // A hot row (hs != HOT_NONE) reads its Gram instead: its first segment
  // stores (1 - w) G_i phi_i (+ tau), its other segments zero.
  auto seg_out = [&](const Seg &sgm, uint32_t d1, real x1, uint32_t hs, vec_t<real> *phi_out) -> vec_t<real> {
    const uint64_t i = sgm.row;
    if (hs != HOT_NONE && !seg_first(sgm)) return vzero<real>();
    uint32_t jj[PP::UT];  // the first pass's columns go out with the phi gather
    if (hs == HOT_NONE) PP::load_cols(ycol, sgm.b, sgm.e, li, jj);
    vec_t<real> phi = vzero<real>();
    if (segd) {  // one node per row: the segment carries it (no row indirection)
      phi = vsplat<real>(x1) * cg_dir_at<real, KP>(V, Rv, Hv, alpha, beta, upd, (size_t)d1 * KP + li * G::VE);
    } else {
      for (int64_t p = xptr[i]; p < xptr[i + 1]; p++)
        phi += vsplat<real>(xval[p]) * cg_dir_at<real, KP>(V, Rv, Hv, alpha, beta, upd, (size_t)xidx[p] * KP + li * G::VE);
    }
    if (hs != HOT_NONE) {
      vec_t<real> out = vsplat<real>(cpos) * sg_vecmat_rolled<real, KP>(phi, hotG + (size_t)hs * KP * KP, li);
      if (QTQ) out += vsplat<real>((real)w) * sg_vecmat_rolled<real, KP>(phi, Qp, li);
      return out;
    }
    vec_t<real> ka = vzero<real>();
    for (int64_t p0 = sgm.b; p0 < sgm.e; p0 += PP::PW) {
      if (p0 != sgm.b) PP::load_cols(ycol, p0, sgm.e, li, jj);
      sfor<PP::PW / PP::GB>([&](auto BT) {
        constexpr int bt = decltype(BT)::value * PP::GB;
        if (p0 + bt >= sgm.e) return;
        vec_t<real> qv[PP::GB];
        sfor<PP::GB>([&](auto U) {
          constexpr int u = decltype(U)::value;
          qv[u] = bld<real>(qb, PP::row_off(PP::template at<bt + u>(jj, li), qb, li));
        });
        real dv[PP::GB];
#pragma unroll
        for (int u = 0; u < PP::GB; u++) dv[u] = sg_sum<G::LPR>(hsum<real>(phi * qv[u]));
#pragma unroll
        for (int u = 0; u < PP::GB; u++) ka += vsplat<real>(dv[u]) * qv[u];
      });
    }
    vec_t<real> out = vsplat<real>(cpos) * ka;
    if constexpr (TT) {
      if (seg_first(sgm)) *phi_out = phi;  // tau: the block's MFMA tile
    } else if (QTQ && seg_first(sgm)) {
      out += vsplat<real>((real)w) * sg_vecmat<real, KP>(phi, Qp, li);
    }
    return out;
  };
  if constexpr (TT) {
    using TTl = TauTile<real, KP>;
    constexpr int SB = TTl::SB, LD = TTl::LD;
    real *Ph = Qs + KP * KP, *Tl = Ph + SB * LD;
    const int wv = threadIdx.x >> 6, rowl = wv * G::NSG + sg;  // this subgroup's tile row
    for (uint64_t base = (uint64_t)blockIdx.x * SB; base < nseg; base += (uint64_t)gridDim.x * SB) {
      const uint64_t sx = base + rowl;
      vec_t<real> phi = vzero<real>(), out = vzero<real>();
      bool first = false;
      if (sx < nseg) {
        const Seg sgm = segs[sx];
        first = seg_first(sgm);
        out = seg_out(sgm, segd ? segd[sx] : 0u, segd ? segx[sx] : (real)0, HOT_NONE, &phi);
      }
      *reinterpret_cast<vec_t<real> *>(Ph + rowl * LD + li * G::VE) = phi;
      __syncthreads();
      // wave wv: output tiles wv, wv + 4, ... of the TR x TC grid
      for (int t = wv; t < TTl::TR * TTl::TC; t += 4) {
        const int tr = t % TTl::TR, tc = t / TTl::TR, m = lane & 15, q = lane >> 4;
        f4v acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int j = 0; j < KP / 16; j++) {
          const f4v a = *reinterpret_cast<const f4v *>(Ph + (tr * 16 + m) * LD + 16 * j + 4 * q);
          const f4v b = *reinterpret_cast<const f4v *>(Qs + ((4 * j + q) * KP + tc * 16 + m) * 4);
#pragma unroll
          for (int u = 0; u < 4; u++) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u], b[u], acc, 0, 0, 0);
        }
#pragma unroll
        for (int r = 0; r < 4; r++) Tl[(tr * 16 + 4 * q + r) * LD + tc * 16 + m] = acc[r];
      }
      __syncthreads();
      if (sx < nseg) {
        if (first) out += vsplat<real>((real)w) * *reinterpret_cast<const vec_t<real> *>(Tl + rowl * LD + li * G::VE);
        vst<real>(h + sx * KP + li * G::VE, out);
      }
    }
    return;
  }
  // Grid-stride over segments with the next segment's descriptor (and its
  // node) in flight while the current one is gathered.
  // sord (optional): the order in which the subgroups take the segments
  // (longest first: a wave's subgroups then walk similar lengths, so fewer
  // absent slots pass through the gather rounds); h stays in segment order
  const uint64_t stride = nwaves * G::NSG;
  uint64_t s = wave * G::NSG + sg;
  Seg nxt{0u, 0u, 0, 0};
  uint32_t nd = 0, nh = HOT_NONE;
  uint64_t nsx = 0;
  real nx = 0;
  auto fetch = [&](uint64_t q) {
    nsx = sord ? (uint64_t)sord[q] : q;
    nxt = segs[nsx];
    if (segd) {
      nd = segd[nsx];
      nx = segx[nsx];
    }
    if (hot_seg) nh = hot_seg[nsx];
  };
  if (s < nseg) fetch(s);
  for (; s < nseg; s += stride) {
    const Seg sgm = nxt;
    const uint32_t d1 = nd, hs = nh;
    const real x1 = nx;
    const uint64_t sx = nsx;
    if (s + stride < nseg) fetch(s + stride);
    vst<real>(h + sx * KP + li * G::VE, seg_out(sgm, d1, x1, hs, nullptr));
  }
}


// ------------------------------------------------------ feature pass ---
// acc_col = sum_{(r, x) in column} x h[r] for every feature column of a field
// (the X^T h of gd_* / hs_*, ffm.cpp:561-570, 603-624, 715-742), then
// MODE 0: gradient finalisation, MODE 1: Hessian-vector finalisation of CG
// iteration f.it (col_finalize above), MODE 2: store the column sums into
// f.acc (multi-GPU: the all-reduce and k_fin follow).
template <typename real, int KP, int MODE, int JE = JOB_ENT, bool TAU = false>
__global__ __launch_bounds__(BLOCK) void k_feat(uint64_t nwave, const Job *__restrict__ jobs,
                                                const uint32_t *__restrict__ crow, const real *__restrict__ cval,
                                                const real *__restrict__ h, uint64_t hbytes, real *__restrict__ wpart,
                                                uint64_t wbytes, Fin<real> f, const real *__restrict__ QTQ) {
  using G = Geo<real, KP>;
  if (f.it > 0 && !f.st->run[f.it]) return;
  // TAU (MODE 1, and MODE 2 on several ranks): QTQ staged in LDS for the
  // per-column tau term (MODE 2 forms the column's CG direction for it)
  extern __shared__ __align__(16) unsigned char smem_raw[];
  real *Qs = reinterpret_cast<real *>(smem_raw);
  if constexpr (TAU) {
    for (int t = threadIdx.x; t < KP * KP; t += BLOCK) Qs[t] = QTQ[t];
    __syncthreads();
  }
  const BufView hb = buf_view(h, hbytes);
  const bool upd = (MODE == 1 || (MODE == 2 && TAU)) && f.it > 1;
  const real alpha = upd ? (real)f.st->alpha : (real)0, beta = upd ? (real)f.st->beta : (real)0;
  const int lane = threadIdx.x & 63;
  const uint64_t wave = ((uint64_t)blockIdx.x * BLOCK + threadIdx.x) >> 6;
  const int sg = lane / G::LPR, li = lane % G::LPR;
  double dsum[3] = {0, 0, 0};
  bool hd_stored = false;  // this wave stored a heavy column's dot-product slot
  const uint64_t nwaves = ((uint64_t)gridDim.x * BLOCK) >> 6;
  Job nxt = wave < nwave ? jobs[wave * G::NSG + sg] : Job{JOB_NONE, 1u, 0u, 0u, 0, 0};
  for (uint64_t w = wave; w < nwave; w += nwaves) {
    const Job jb = nxt;  // this round's job; the next round's is in flight below
    if (w + nwaves < nwave) nxt = jobs[(w + nwaves) * G::NSG + sg];
    // finalisation operands first (padding jobs read column 0, unused)
    FinOps<real> ops;
    if (MODE != 2) ops = fin_load<real, KP, (MODE == 2 ? 0 : MODE)>(f, jb.col == JOB_NONE ? 0u : jb.col, upd, li);
    constexpr int U = (JE + G::LPR - 1) / G::LPR;
    // a light job is one round of <= JE entries; a wave-chunk of a heavy
    // column gives each subgroup several rounds (build_csc sizes them)
    vec_t<real> s = vzero<real>();
    int64_t b0 = jb.b;
    do {
      uint32_t rr[U];
      real vv[U];
#pragma unroll
      for (int t = 0; t < U; t++) {
        const int e = li + t * G::LPR;
        const bool ok = e < JE && b0 + e < jb.e;
        rr[t] = ok ? crow[b0 + e] : 0u;
        vv[t] = ok ? cval[b0 + e] : (real)0;
      }
      vec_t<real> hv[JE];
      sfor<JE>([&](auto E) {
        constexpr int e = decltype(E)::value;
        const uint32_t r = sg_bcast<G::LPR, e % G::LPR>(rr[e / G::LPR], li);
        const real x = sg_bcast<G::LPR, e % G::LPR>(vv[e / G::LPR], li);
        const uint32_t off = b0 + e < jb.e ? r * (uint32_t)(KP * sizeof(real)) + li * LANE_B<real> : hb.oob;
        hv[e] = vsplat<real>(x) * bld<real>(hb, off);
      });
#pragma unroll
      for (int e = 0; e < JE; e++) s += hv[e];
      b0 += JE;
    } while (b0 < jb.e);
    bool mine = jb.col != JOB_NONE;
    int64_t hslot = -1;  // a last-arriving chunk: the column's dot-product slot
    if (jb.flags & 1u) {  // wave job (wave-uniform)
      s = xsg_vsum<G::LPR, real>(s);
      mine = sg == 0;
      if (jb.nparts > 1) {
        if (sg == 0) {
#pragma unroll
          for (int e = 0; e < G::VE; e++)
            __hip_atomic_store(wpart + (size_t)jb.slot * KP + li * G::VE + e, s[e], __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        unsigned t = 0;
        if (lane == 0) t = __hip_atomic_fetch_add(f.cnt + jb.col, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        t = __shfl(t, 0, 64);
        if (t != jb.nparts - 1) {
          mine = false;
        } else {
          // the column's partial slots in chunk order, RB per subgroup in
          // flight (sc1 buffer loads: the last-arriver hand-off), then a
          // fixed tree over the subgroups: deterministic
          const uint32_t s0 = jb.slot - (jb.flags >> 1);
          const BufView pv = buf_view(wpart, wbytes);
          constexpr int RB = 8;
          vec_t<real> a = vzero<real>();
          for (uint32_t q0 = sg; q0 < jb.nparts; q0 += RB * G::NSG) {
            vec_t<real> y[RB];
#pragma unroll
            for (int u = 0; u < RB; u++) {
              const uint32_t q = q0 + u * G::NSG;
              const uint32_t off = q < jb.nparts ? (uint32_t)(((size_t)(s0 + q) * KP + li * G::VE) * sizeof(real)) : pv.oob;
              y[u] = bld_sc1<real>(pv, off);
            }
#pragma unroll
            for (int u = 0; u < RB; u++) a += y[u];
          }
          s = xsg_vsum<G::LPR, real>(a);
          hslot = s0;
          if (lane == 0) __hip_atomic_store(f.cnt + jb.col, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
    }
    if (mine) {
      if constexpr (MODE == 2) {
        if constexpr (TAU) {
          const vec_t<real> d = cg_dir_at<real, KP>(f.P, f.R, f.Hp, alpha, beta, upd, (size_t)jb.col * KP + li * G::VE);
          s += vsplat<real>((real)(f.tw * (double)f.xsq[jb.col])) * sg_vecmat<real, KP>(d, Qs, li);
        }
        vst<real>(f.acc + (size_t)jb.col * KP + li * G::VE, s);
      } else if (hslot >= 0 && f.hdots) {
        // the column's dot products into its own slot (fixed order: the
        // subgroup's lanes by DPP), not into this block's partial
        double cd[3] = {0, 0, 0};
        col_finalize<real, KP, (MODE == 2 ? 0 : MODE), TAU>(f, jb.col, s, alpha, beta, upd, li, cd, ops, Qs);
#pragma unroll
        for (int k = 0; k < 3; k++) cd[k] = sg_sum<G::LPR>(cd[k]);
        if (li == 0)
#pragma unroll
          for (int k = 0; k < 3; k++)
            __hip_atomic_store(f.hdots + (size_t)hslot * 3 + k, cd[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        hd_stored = true;
      } else col_finalize<real, KP, (MODE == 2 ? 0 : MODE), TAU>(f, jb.col, s, alpha, beta, upd, li, dsum, ops, Qs);
    }
  }
  // a wave's dot-product slot stores are drained before this block's ticket
  // (last_block); waves that stored none do not wait for their vector stores
  // (wave jobs are wave-uniform, so is the flag)
  if (__any(hd_stored)) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (MODE != 2) fin_blocks<real, (MODE == 2 ? 0 : MODE)>(f, dsum);
}

// Feature pass of a field whose columns are few and heavy (round 5; the
// kkbox context field: 120 columns of ~500 rows, ~1,300 segments): ONE
// BLOCK PER COLUMN.  Its 4 NSG subgroups take FE consecutive entries each
// per round (all their row loads in flight), the column's sum is reduced
// through LDS in a fixed order and finalised by one subgroup, whose
// finalisation operands were loaded at the start; the grid's dot products
// by the last block (fin_blocks).  k_feat instead cuts such a column into
// wave-chunks whose partial slots the last-arriving chunk sums: a chain of
// dependent rounds (~15 us per context step).  Deterministic (fixed grid).
// MODE as k_feat (no column tau).
template <typename real, int KP, int MODE>
__global__ __launch_bounds__(BLOCK) void k_feat_col(uint64_t D, const int64_t *__restrict__ cptr,
                                                    const uint32_t *__restrict__ crow, const real *__restrict__ cval,
                                                    const real *__restrict__ h, uint64_t hbytes, Fin<real> f) {
  using Gm = Geo<real, KP>;
  constexpr int FE = 8;  // entries per subgroup and round
  constexpr int U = (FE + Gm::LPR - 1) / Gm::LPR;
  if (f.it > 0 && !f.st->run[f.it]) return;
  const BufView hb = buf_view(h, hbytes);
  const bool upd = MODE == 1 && f.it > 1;
  const real alpha = upd ? (real)f.st->alpha : (real)0, beta = upd ? (real)f.st->beta : (real)0;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int sg = lane / Gm::LPR, li = lane % Gm::LPR;
  const int sid = w * Gm::NSG + sg;
  constexpr int NS = 4 * Gm::NSG;
  __shared__ __align__(16) real red[BLOCK / 64][KP];
  double dsum[3] = {0, 0, 0};
  for (uint64_t c = blockIdx.x; c < D; c += gridDim.x) {
    const bool fin = w == 0 && sg == 0;
    FinOps<real> ops;
    if (MODE != 2 && fin) ops = fin_load<real, KP, (MODE == 2 ? 0 : MODE)>(f, (uint32_t)c, upd, li);
    const int64_t b = cptr[c], e = cptr[c + 1];
    vec_t<real> s = vzero<real>();
    for (int64_t t0 = b + (int64_t)sid * FE; t0 < e; t0 += (int64_t)NS * FE) {
      uint32_t rr[U];
      real vv[U];
#pragma unroll
      for (int u = 0; u < U; u++) {
        const int64_t t = t0 + li + u * Gm::LPR;
        const bool ok = li + u * Gm::LPR < FE && t < e;
        rr[u] = ok ? crow[t] : 0u;
        vv[u] = ok ? cval[t] : (real)0;
      }
      vec_t<real> hv[FE];
      sfor<FE>([&](auto E) {
        constexpr int q = decltype(E)::value;
        const uint32_t r = sg_bcast<Gm::LPR, q % Gm::LPR>(rr[q / Gm::LPR], li);
        const real x = sg_bcast<Gm::LPR, q % Gm::LPR>(vv[q / Gm::LPR], li);
        const uint32_t off = t0 + q < e ? r * (uint32_t)(KP * sizeof(real)) + li * LANE_B<real> : hb.oob;
        hv[q] = vsplat<real>(x) * bld<real>(hb, off);
      });
#pragma unroll
      for (int q = 0; q < FE; q++) s += hv[q];
    }
    s = xsg_vsum<Gm::LPR, real>(s);
    if (sg == 0) *reinterpret_cast<vec_t<real> *>(&red[w][li * Gm::VE]) = s;
    __syncthreads();
    if (fin) {  // the waves' sums in wave order
      vec_t<real> t = *reinterpret_cast<const vec_t<real> *>(&red[0][li * Gm::VE]);
#pragma unroll
      for (int q = 1; q < BLOCK / 64; q++) t += *reinterpret_cast<const vec_t<real> *>(&red[q][li * Gm::VE]);
      if constexpr (MODE == 2) vst<real>(f.acc + c * KP + li * Gm::VE, t);
      else col_finalize<real, KP, (MODE == 2 ? 0 : MODE)>(f, (uint32_t)c, t, alpha, beta, upd, li, dsum, ops);
    }
    __syncthreads();
  }
  if (MODE != 2) fin_blocks<real, (MODE == 2 ? 0 : MODE)>(f, dsum);
}

// ------------------------------------------------- CG vector kernels ---
// All operate on n vectors of VE elements (D x KP buffers); row = v / LPR.
#define VEC_LOOP for (uint64_t v = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; v < nv; v += (uint64_t)gridDim.x * BLOCK)

// Unfused finalisation (multi-GPU: after the all-reduce of acc), the same
// col_finalize / fin_blocks as the fused feature pass with s = acc (then
// acc = 0).  MODE 0: gradient start (ffm.cpp:561-570, 773-779); MODE 1:
// Hessian-vector product of CG iteration f.it (ffm.cpp:783-809).
template <typename real, int KP, int MODE>
__global__ __launch_bounds__(BLOCK) void k_fin(uint64_t nv, Fin<real> f) {
  using G = Geo<real, KP>;
  if (MODE == 1 && !f.st->run[f.it]) return;
  const bool upd = MODE == 1 && f.it > 1;
  const real alpha = upd ? (real)f.st->alpha : (real)0, beta = upd ? (real)f.st->beta : (real)0;
  double dsum[3] = {0, 0, 0};
  VEC_LOOP {
    const vec_t<real> s = vld<real>(f.acc + v * G::VE);
    vst<real>(f.acc + v * G::VE, vzero<real>());
    col_finalize<real, KP, MODE>(f, (uint32_t)(v / G::LPR), s, alpha, beta, upd, (int)(v % G::LPR), dsum);
  }
  fin_blocks<real, MODE>(f, dsum);
}

// Exact CG residual (Fin::exact_r2): after the finalisation of iteration
// f.it has published alpha, |r - alpha Hp|^2 over the D x KP vectors in a
// fixed order (grid-stride, block tree, block order), then beta = r2n / r2
// and the verdict of iteration it+1 (ffm.cpp:807-809).  r and Hp hold
// iteration it's values here: the lazy update (cg_dir_at) applies
// r -= alpha Hp in the next feature pass, with this same rounding.
template <typename real>
__global__ __launch_bounds__(BLOCK) void k_cg_r2(uint64_t nv, Fin<real> f) {
  CgState *st = f.st;
  if (!st->run[f.it]) return;
  const real alpha = (real)st->alpha;
  double acc = 0;
  VEC_LOOP {
    const vec_t<real> rn = vld<real>(f.R + v * VT<real>::N) - vsplat<real>(alpha) * vld<real>(f.Hp + v * VT<real>::N);
#pragma unroll
    for (int e = 0; e < VT<real>::N; e++) acc += (double)rn[e] * (double)rn[e];
  }
  double bv[1] = {block_sum(acc)}, tot[1];
  if (last_block<1>(bv, f.part, f.tick, tot) && threadIdx.x == 0) {
    const double r2 = st->r2, r2n = tot[0];
    st->beta = r2n / r2;
    st->r2 = r2n;
    const int go = (f.it < MAXCG && st->g2 * CG_EPS < r2n) ? 1 : 0;
    st->run[f.it + 1] = go;
    if (f.run_host)
      __hip_atomic_store(f.run_host + f.it + 1, go ? RUN_GO : RUN_STOP, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// The step of the half: S += alpha_last p_last (the update of the last CG
// iteration, pending under the lazy scheme above), W += S  (ffm.cpp:806, 410, 441).
// own (owned fields on several ranks): only this rank's feature rows; the
// others hold another rank's stale scratch and are left alone.
template <typename real>
__global__ __launch_bounds__(BLOCK) void k_apply(uint64_t nv, const real *__restrict__ P, real *__restrict__ S,
                                                 real *__restrict__ W, const CgState *st,
                                                 const uint8_t *__restrict__ own, uint32_t lpr,
                                                 const int *__restrict__ skip) {
  if (skip && *skip) return;  // speculative update of a CG solve that went on (solver.hip finish_half)
  const real alpha = st->nr_cg >= 1 ? (real)st->alpha : (real)0;
  VEC_LOOP {
    if (own && !own[v / lpr]) continue;
    const vec_t<real> s = vld<real>(S + v * VT<real>::N) + vsplat<real>(alpha) * vld<real>(P + v * VT<real>::N);
    vst<real>(S + v * VT<real>::N, s);
    vst<real>(W + v * VT<real>::N, vld<real>(W + v * VT<real>::N) + s);
  }
}

// Zero the feature rows this rank does not own (owned fields before the
// all-reduce that makes a table whole again on every rank).
template <typename real>
__global__ __launch_bounds__(BLOCK) void k_mask_rows(uint64_t nv, real *__restrict__ T, const uint8_t *__restrict__ own,
                                                     uint32_t lpr) {
  VEC_LOOP {
    if (!own[v / lpr]) vst<real>(T + v * VT<real>::N, vzero<real>());
  }
}

// ------------------------------------------------------- update rows ---
// The CG step of an id-like field (each feature in exactly one row), with
// the work of k_apply folded in by the row that owns the feature: the last
// pending S += alpha p (ffm.cpp:806), then W += S (410, 441).  Returns S.
template <typename real, int KP>
__device__ __forceinline__ vec_t<real> apply_owned_row(const real *__restrict__ S, const real *__restrict__ Pd,
                                                       real *__restrict__ W, real alpha, size_t off) {
  const vec_t<real> s = vld<real>(S + off) + vsplat<real>(alpha) * vld<real>(Pd + off);
  vst<real>(W + off, vld<real>(W + off) + s);
  return s;
}

// k_apply's work folded into an update kernel for a field that is not
// id-like (round 6): the rows form XS from the final step S + a p
// on the fly (the same expression k_apply stores), and every thread of the
// grid then takes a stride of W += S + a p.  Nothing in the kernel reads W,
// and S is only read, so the two parts need no ordering.  nv = D KP / VE
// (0: no fold).
template <typename real>
__device__ __forceinline__ vec_t<real> final_step(const real *__restrict__ S, const real *__restrict__ Pd, real alpha,
                                                  size_t off) {
  return vld<real>(S + off) + vsplat<real>(alpha) * vld<real>(Pd + off);
}
template <typename real>
__device__ __forceinline__ void fold_apply(uint64_t nv, const real *__restrict__ S, const real *__restrict__ Pd,
                                           real *__restrict__ W, real alpha) {
  for (uint64_t v = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; v < nv; v += (uint64_t)gridDim.x * BLOCK) {
    const vec_t<real> s = final_step<real>(S, Pd, alpha, v * VT<real>::N);
    vst<real>(W + v * VT<real>::N, vld<real>(W + v * VT<real>::N) + s);
  }
}

// Per segment of row i (one segment per subgroup): XS_i = X_i S;
// [first] P_i += XS_i; base_ij += <XS_i, q_j> for the segment's positives
// (update_cross, ffm.cpp:439-465), in this side's orientation; k_gather_pos
// then refreshes the other orientation (a gather instead of a scattered
// read-modify-write per positive).
template <typename real, int KP>
__global__ __launch_bounds__(BLOCK) void k_update_cross_seg(uint64_t nseg, const Seg *__restrict__ segs,
                                                            const int64_t *__restrict__ xptr,
                                                            const uint32_t *__restrict__ xidx,
                                                            const real *__restrict__ xval,
                                                            const real *__restrict__ S, real *__restrict__ P1,
                                                            const uint32_t *__restrict__ ycol,
                                                            real *__restrict__ yt, const real *__restrict__ Q1,
                                                            uint64_t q1rows, const uint32_t *__restrict__ segd,
                                                            const real *__restrict__ segx, real *__restrict__ W,
                                                            const real *__restrict__ Pd, const CgState *st,
                                                            const real *__restrict__ XSin,
                                                            const real *__restrict__ a1,
                                                            const real *__restrict__ b1,
                                                            const int *__restrict__ skip) {
  using G = Geo<real, KP>;
  using PP = PosPass<real, KP>;
  if (skip && *skip) return;
  const BufView qb = buf_view(Q1, q1rows * KP * sizeof(real));
  WAVE_SETUP
  const int sg = lane / G::LPR, li = lane % G::LPR;
  const real alpha = (W && st->nr_cg >= 1) ? (real)st->alpha : (real)0;
  for (uint64_t s = wave * G::NSG + sg; s < nseg; s += nwaves * G::NSG) {
    const Seg sgm = segs[s];
    const uint64_t i = sgm.row;
    vec_t<real> xs = vzero<real>();
    real ai = 0;
    if (XSin) {  // flush of the block-excluded y~ (a1/b1: its biases come out)
      xs = vld<real>(XSin + i * KP + li * G::VE);
      ai = a1[i];
    } else if (W) {  // id-like field (segd set): the row's first segment does its feature's k_apply work
      const size_t off = (size_t)segd[s] * KP + li * G::VE;
      const vec_t<real> sf = seg_first(sgm) ? apply_owned_row<real, KP>(S, Pd, W, alpha, off)
                                            : vld<real>(S + off) + vsplat<real>(alpha) * vld<real>(Pd + off);
      xs = vsplat<real>(segx[s]) * sf;
    } else if (segd) {
      xs = vsplat<real>(segx[s]) * vld<real>(S + (size_t)segd[s] * KP + li * G::VE);
    } else {
      for (int64_t p = xptr[i]; p < xptr[i + 1]; p++)
        xs += vsplat<real>(xval[p]) * vld<real>(S + (size_t)xidx[p] * KP + li * G::VE);
    }
    if (seg_first(sgm) && !XSin) vst<real>(P1 + i * KP + li * G::VE, vld<real>(P1 + i * KP + li * G::VE) + xs);
    for (int64_t p0 = sgm.b; p0 < sgm.e; p0 += PP::PW) {
      uint32_t jj[PP::UT];
      PP::load_cols(ycol, p0, sgm.e, li, jj);
      real dd[PP::UT];
#pragma unroll
      for (int t = 0; t < PP::UT; t++) dd[t] = 0;
      sfor<PP::PW / PP::GB>([&](auto BT) {
        constexpr int bt = decltype(BT)::value * PP::GB;
        if (p0 + bt >= sgm.e) return;
        vec_t<real> qv[PP::GB];
        sfor<PP::GB>([&](auto U) {
          constexpr int u = decltype(U)::value;
          qv[u] = bld<real>(qb, PP::row_off(PP::template at<bt + u>(jj, li), qb, li));
        });
#pragma unroll
        for (int u = 0; u < PP::GB; u++) {
          const real d = sg_sum<G::LPR>(hsum<real>(xs * qv[u]));
          if ((bt + u) % G::LPR == li) dd[(bt + u) / G::LPR] = d;
        }
      });
      // each lane owns its positions p0 + li + t*LPR: all loads, then all stores
      real ym[PP::UT];
#pragma unroll
      for (int t = 0; t < PP::UT; t++) {
        const int64_t q = p0 + li + t * G::LPR;
        ym[t] = q < sgm.e ? yt[q] : (real)0;
        if (XSin && q < sgm.e) ym[t] -= ai + b1[jj[t]];
      }
#pragma unroll
      for (int t = 0; t < PP::UT; t++) {
        const int64_t q = p0 + li + t * G::LPR;
        if (q < sgm.e) yt[q] = ym[t] + dd[t];
      }
    }
  }
}

// The cross update without its positive pass (block-excluded base, DESIGN
// §2: the stored base does not depend on this block's factors):
// XS_i = X_i S, P_i += XS_i (and XS_i kept when XS is given).  W non-null
// (id-like field): the row also does its feature's k_apply work.
template <typename real, int KP>
__global__ __launch_bounds__(BLOCK) void k_update_cross_rows(uint64_t R, const int64_t *__restrict__ xptr,
                                                             const uint32_t *__restrict__ xidx,
                                                             const real *__restrict__ xval,
                                                             const real *__restrict__ S, real *__restrict__ P1,
                                                             real *__restrict__ XS, bool one, real *__restrict__ W,
                                                             const real *__restrict__ Pd, const CgState *st,
                                                             const int *__restrict__ skip, uint64_t nfold) {
  using G = Geo<real, KP>;
  if (skip && *skip) return;
  WAVE_SETUP
  const int sg = lane / G::LPR, li = lane % G::LPR;
  const real alpha = ((W || nfold) && st->nr_cg >= 1) ? (real)st->alpha : (real)0;
  for (uint64_t i = wave * G::NSG + sg; i < R; i += nwaves * G::NSG) {
    vec_t<real> xs = vzero<real>();
    if (nfold) {  // W is updated below (fold_apply): S + a p on the fly
      for (int64_t p = one ? (int64_t)i : xptr[i]; p < (one ? (int64_t)i + 1 : xptr[i + 1]); p++)
        xs += vsplat<real>(xval[p]) * final_step<real>(S, Pd, alpha, (size_t)xidx[p] * KP + li * G::VE);
    } else if (W) {
      xs = vsplat<real>(xval[i]) * apply_owned_row<real, KP>(S, Pd, W, alpha, (size_t)xidx[i] * KP + li * G::VE);
    } else if (one) {
      xs = vsplat<real>(xval[i]) * vld<real>(S + (size_t)xidx[i] * KP + li * G::VE);
    } else {
      for (int64_t p = xptr[i]; p < xptr[i + 1]; p++)
        xs += vsplat<real>(xval[p]) * vld<real>(S + (size_t)xidx[p] * KP + li * G::VE);
    }
    vst<real>(P1 + i * KP + li * G::VE, vld<real>(P1 + i * KP + li * G::VE) + xs);
    if (XS) vst<real>(XS + i * KP + li * G::VE, xs);
  }
  if (nfold) fold_apply<real>(nfold, S, Pd, W, alpha);
}

// dst[q] = src[idx[q]]: the other orientation of base from this one (idx =
// the other side's perm).  Four positions per thread: one 16-B index load,
// four gathers, one wide store.
template <typename real>
__global__ __launch_bounds__(BLOCK) void k_gather_pos(uint64_t n, const uint32_t *__restrict__ idx,
                                                      const real *__restrict__ src, real *__restrict__ dst,
                                                      const int *__restrict__ skip) {
  if (skip && *skip) return;
  for (uint64_t q = ((uint64_t)blockIdx.x * BLOCK + threadIdx.x) * 4; q < n; q += (uint64_t)gridDim.x * BLOCK * 4) {
    if (q + 4 <= n) {
      const uint4 ix = *reinterpret_cast<const uint4 *>(idx + q);
      const real a = src[ix.x], b = src[ix.y], c = src[ix.z], d = src[ix.w];
      dst[q] = a;
      dst[q + 1] = b;
      dst[q + 2] = c;
      dst[q + 3] = d;
    } else {
      for (uint64_t r = q; r < n; r++) dst[r] = src[idx[r]];
    }
  }
}

// XS_i = X_i S; P_i += XS_i; a_i += <XS_i, q1_i>  (update_side,
// ffm.cpp:405-437).  The reference also adds the gap to every positive of
// row i; with y~ kept factored (see k_init_ytilde) that is implied by a_i.
// One row per subgroup.  W non-null (id-like field): the row also does its
// feature's k_apply work (apply_owned_row).  The sum of the new a over the
// side (b_sum of the next gd_side, ffm.cpp:551) goes to *asum, summed in a
// fixed order (last_block).
template <typename real, int KP>
__global__ __launch_bounds__(BLOCK) void k_update_side_row(uint64_t R, const int64_t *__restrict__ xptr,
                                                           const uint32_t *__restrict__ xidx,
                                                           const real *__restrict__ xval, const real *__restrict__ S,
                                                           real *__restrict__ P1, const real *__restrict__ Q1,
                                                           real *__restrict__ a1, bool one, real *__restrict__ W,
                                                           const real *__restrict__ Pd, const CgState *st,
                                                           double *__restrict__ asum, double *part, unsigned *tick,
                                                           const int *__restrict__ skip, uint64_t nfold) {
  using G = Geo<real, KP>;
  if (skip && *skip) return;  // (every block: the last_block tickets stay untouched)
  WAVE_SETUP
  const int sg = lane / G::LPR, li = lane % G::LPR;
  const real alpha = ((W || nfold) && st->nr_cg >= 1) ? (real)st->alpha : (real)0;
  double bs = 0;
  for (uint64_t i = wave * G::NSG + sg; i < R; i += nwaves * G::NSG) {
    vec_t<real> xs = vzero<real>();
    if (nfold) {  // W is updated below (fold_apply): S + a p on the fly
      for (int64_t p = one ? (int64_t)i : xptr[i]; p < (one ? (int64_t)i + 1 : xptr[i + 1]); p++)
        xs += vsplat<real>(xval[p]) * final_step<real>(S, Pd, alpha, (size_t)xidx[p] * KP + li * G::VE);
    } else if (W) {  // id-like: one node per row, the row owns its feature
      xs = vsplat<real>(xval[i]) * apply_owned_row<real, KP>(S, Pd, W, alpha, (size_t)xidx[i] * KP + li * G::VE);
    } else if (one) {
      xs = vsplat<real>(xval[i]) * vld<real>(S + (size_t)xidx[i] * KP + li * G::VE);
    } else {
      for (int64_t p = xptr[i]; p < xptr[i + 1]; p++)
        xs += vsplat<real>(xval[p]) * vld<real>(S + (size_t)xidx[p] * KP + li * G::VE);
    }
    vst<real>(P1 + i * KP + li * G::VE, vld<real>(P1 + i * KP + li * G::VE) + xs);
    const real gap = sg_sum<G::LPR>(hsum<real>(xs * vld<real>(Q1 + i * KP + li * G::VE)));
    if (li == 0) {
      const real an = a1[i] + gap;
      a1[i] = an;
      bs += (double)an;
    }
  }
  if (nfold) fold_apply<real>(nfold, S, Pd, W, alpha);
  const double bv[1] = {block_sum(bs)};
  double tot[1];
  if (last_block<1>(bv, part, tick, tot) && threadIdx.x == 0) asum[0] = tot[0];
}

// ------------------------------------------------- partner aggregates ---
// Per-block partial sums over a range of partner rows j:
//   gram[l][e][d] = sum_j A_l[j][e] B[j][d]     (Q_c^T Q1, ffm.cpp:663-670,770)
//   col[d]        = sum_j B[j][d]               (oQ = Q1^T 1, ffm.cpp:660)
//   wcol[d]       = sum_j wv_j B[j][d]          (bQ = Q1^T b, ffm.cpp:661)
//   wsum          = sum_j wv_j                  (sum of b, ffm.cpp:551)
// Rows are staged through LDS TR at a time with 16-B cooperative loads (the
// whole block keeps many loads in flight); each thread then owns up to SPT
// 4x4 (e,d) sub-tiles and accumulates in registers.  Output layout per block:
// [L*KP*KP grams | KP col | KP wcol | 1 wsum] (doubles).
template <typename real, int KP, int SPT>
__global__ __launch_bounds__(BLOCK) void k_gram_part(uint64_t Rp, int L, const real *const *__restrict__ A,
                                                     const real *__restrict__ B, const real *__restrict__ wv,
                                                     double *__restrict__ part, uint64_t rows_per_block,
                                                     int sub_per_y) {
  constexpr int Q4 = KP / 4;
  constexpr int TR = (KP >= 64) ? 16 : 32;
  constexpr int VE = VT<real>::N;
  extern __shared__ __align__(16) unsigned char smem_raw[];
  real *sA = reinterpret_cast<real *>(smem_raw);  // [L][TR][KP]
  real *sB = sA + (size_t)L * TR * KP;            // [TR][KP]
  real *sW = sB + (size_t)TR * KP;                // [TR]
  const int t = threadIdx.x;
  const int nsub_tot = L * Q4 * Q4;
  const int sub0 = blockIdx.y * sub_per_y;
  const int nsub = max(0, min(sub_per_y, nsub_tot - sub0));
  real acc[SPT][16];
#pragma unroll
  for (int q = 0; q < SPT; q++)
#pragma unroll
    for (int x = 0; x < 16; x++) acc[q][x] = 0;
  real cs = 0, ws = 0, wtot = 0;
  const uint64_t r0 = (uint64_t)blockIdx.x * rows_per_block;
  const uint64_t r1 = min(Rp, r0 + rows_per_block);
  const bool do_cols = blockIdx.y == 0;
  const int pieces_row = KP / VE;
  const int ntab = L + (B ? 1 : 0);
  for (uint64_t j0 = r0; j0 < r1; j0 += TR) {
    const int nr = (int)min<uint64_t>(TR, r1 - j0);
    __syncthreads();
    const int tot = ntab * TR * pieces_row;
    for (int q = t; q < tot; q += BLOCK) {
      const int tab = q / (TR * pieces_row);
      const int rr = (q / pieces_row) % TR;
      const int pc = q % pieces_row;
      vec_t<real> v = vzero<real>();
      if (rr < nr) v = vld<real>((tab < L ? A[tab] : B) + (j0 + rr) * KP + pc * VE);
      vst<real>((tab < L ? sA + ((size_t)tab * TR + rr) * KP : sB + (size_t)rr * KP) + pc * VE, v);
    }
    if (wv && t < TR) sW[t] = t < nr ? wv[j0 + t] : (real)0;
    __syncthreads();
#pragma unroll
    for (int q = 0; q < SPT; q++) {
      if (t + q * BLOCK < nsub) {
        const int sub = sub0 + t + q * BLOCK;
        const int l = sub / (Q4 * Q4), eq = (sub / Q4) % Q4, dq = sub % Q4;
        const real *pa = sA + (size_t)l * TR * KP + eq * 4;
        const real *pb = sB + dq * 4;
        for (int rr = 0; rr < nr; rr++) {
          real av[4], bv[4];
#pragma unroll
          for (int x = 0; x < 4; x++) {
            av[x] = pa[rr * KP + x];
            bv[x] = pb[rr * KP + x];
          }
#pragma unroll
          for (int x = 0; x < 4; x++)
#pragma unroll
            for (int y = 0; y < 4; y++) acc[q][x * 4 + y] += av[x] * bv[y];
        }
      }
    }
    if (do_cols && t < KP && B) {
      for (int rr = 0; rr < nr; rr++) {
        const real bb = sB[rr * KP + t];
        cs += bb;
        if (wv) ws += sW[rr] * bb;
      }
    }
    if (do_cols && t == 0 && wv)
      for (int rr = 0; rr < nr; rr++) wtot += sW[rr];
  }
  const size_t NOUT = (size_t)L * KP * KP + 2 * KP + 1;
  double *out = part + (size_t)blockIdx.x * NOUT;
#pragma unroll
  for (int q = 0; q < SPT; q++) {
    if (t + q * BLOCK < nsub) {
      const int sub = sub0 + t + q * BLOCK;
      const int l = sub / (Q4 * Q4), eq = (sub / Q4) % Q4, dq = sub % Q4;
#pragma unroll
      for (int x = 0; x < 4; x++)
#pragma unroll
        for (int y = 0; y < 4; y++) out[((size_t)l * KP + eq * 4 + x) * KP + dq * 4 + y] = (double)acc[q][x * 4 + y];
    }
  }
  if (do_cols) {
    if (t < KP) {
      out[(size_t)L * KP * KP + t] = (double)cs;
      out[(size_t)L * KP * KP + KP + t] = (double)ws;
    }
    if (t == 0) out[(size_t)L * KP * KP + 2 * KP] = (double)wtot;
  }
}

// The same per-block partials as k_gram_part for fp32 rows of KP = 32, on
// MFMA (v_mfma_f32_32x32x2f32): the Gram gram[l][e][d] = sum_j A_l[j][e] B[j][d]
// is a 32 x 32 x (rows) product with the rows as the K dimension.  Operand
// layouts: A lane l = A_l[j + l/32][l%32] (m = e), B lane l = B[j + l/32][l%32]
// (n = d): each lane loads one dword per table per row pair, so a wave reads
// two whole 128-B rows per load instruction, straight into the MFMA operand
// registers (no LDS staging).  D register r of lane l is element
// m = 8(r/4) + 4(l/32) + r%4, n = l%32.  The four waves of a block take
// interleaved row pairs and are combined in wave order through LDS
// (deterministic).  Column sums ride along on the B operand.
template <int L>
__global__ __launch_bounds__(BLOCK) void k_gram_mfma32(uint64_t Rp, const float *const *__restrict__ A,
                                                      const float *__restrict__ B, const float *__restrict__ wv,
                                                      float *__restrict__ part, uint64_t rows_per_block) {
  typedef float f16x __attribute__((ext_vector_type(16)));
  constexpr int U = 4;  // row pairs per wave per round
  __shared__ float red[L][1024];
  __shared__ float redc[3][32];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int e = lane & 31, hf = lane >> 5;
  f16x acc[L];
#pragma unroll
  for (int c = 0; c < L; c++)
#pragma unroll
    for (int r = 0; r < 16; r++) acc[c][r] = 0.0f;
  // raw buffer loads (a table pointer read from memory would make the
  // compiler fall back to flat loads); rows past the end read zero
  BufView ab[L];
#pragma unroll
  for (int c = 0; c < L; c++) ab[c] = buf_view(A[c], Rp * 128);
  const BufView bb = buf_view(B, B ? Rp * 128 : 0), wb = buf_view(wv, wv ? Rp * 4 : 0);
  float cs = 0, ws = 0, wt = 0;
  const uint64_t r0 = (uint64_t)blockIdx.x * rows_per_block;
  const uint64_t r1 = min(Rp, r0 + rows_per_block);
  // two register sets: the next round's loads are in flight while this
  // round's MFMAs run (one wave per SIMD: the loop is latency-bound)
  float bv[2][U], wvv[2][U], av[2][U][L];
  auto load = [&](int sb, uint64_t j0) {
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint64_t jj = j0 + 8 * u + hf;
      const bool ok = jj < r1;
      const uint32_t off = ok ? (uint32_t)(jj * 128 + e * 4) : 0xffffffffu;
      bv[sb][u] = bld1<float>(bb, off);
      wvv[sb][u] = bld1<float>(wb, ok ? (uint32_t)(jj * 4) : 0xffffffffu);
#pragma unroll
      for (int c = 0; c < L; c++) av[sb][u][c] = bld1<float>(ab[c], off);
    }
  };
  auto step = [&](int sb) {
#pragma unroll
    for (int u = 0; u < U; u++) {
#pragma unroll
      for (int c = 0; c < L; c++) acc[c] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[sb][u][c], bv[sb][u], acc[c], 0, 0, 0);
      cs += bv[sb][u];
      ws += wvv[sb][u] * bv[sb][u];
      if (e == 0) wt += wvv[sb][u];
    }
  };
  // rows past r1 load zeros (buffer range check), so a trailing round is harmless
  for (uint64_t j0 = r0 + 2 * w; j0 < r1; j0 += 16 * U) {
    load(0, j0);
    load(1, j0 + 8 * U);
    step(0);
    step(1);
  }
  // column sums: the two half-waves hold even / odd rows of the same column
  cs += __shfl_xor(cs, 32, 64);
  ws += __shfl_xor(ws, 32, 64);
  wt += __shfl_xor(wt, 32, 64);
  for (int ww = 0; ww < BLOCK / 64; ww++) {
    if (w == ww) {
#pragma unroll
      for (int c = 0; c < L; c++)
#pragma unroll
          for (int r = 0; r < 16; r++) {
            const int m = 8 * (r >> 2) + 4 * hf + (r & 3);
            float &x = red[c][m * 32 + e];
            x = (ww == 0 ? 0.0f : x) + acc[c][r];
          }
      if (hf == 0) {
        redc[0][e] = (ww == 0 ? 0.0f : redc[0][e]) + cs;
        redc[1][e] = (ww == 0 ? 0.0f : redc[1][e]) + ws;
        if (e == 0) redc[2][0] = (ww == 0 ? 0.0f : redc[2][0]) + wt;
      }
    }
    __syncthreads();
  }
  const size_t NOUT = (size_t)L * 1024 + 2 * 32 + 1;
  float *out = part + (size_t)blockIdx.x * NOUT;  // f32 partials (k_reduce_parts<real, float>)
  for (int o = threadIdx.x; o < L * 1024; o += BLOCK) out[o] = red[o >> 10][o & 1023];
  if (threadIdx.x < 32) {
    out[(size_t)L * 1024 + threadIdx.x] = redc[0][threadIdx.x];
    out[(size_t)L * 1024 + 32 + threadIdx.x] = redc[1][threadIdx.x];
  }
  if (threadIdx.x == 0) out[(size_t)L * 1024 + 64] = redc[2][0];
}

// Cross-half aggregates at KP = 64, fp32, on MFMA (gd_cross / cg,
// ffm.cpp:660-670, 767-771): M_c = A_c^T B for every partner-side table A_c
// (k x k, c < C), oQ = sum_i B_i, bQ = sum_i wv_i B_i and sum wv, over the
// rows of block x's chunk.  Wave slot c < C owns table c (4 x 16 accumulator
// registers: the 2 x 2 tiles of 32 x 32) and walks every row of the chunk:
// v_mfma_f32_32x32x2f32 takes a row pair as the K dimension, lane l
// supplying A_c[row 2u + l/32][32 mt + l%32] and B[row][32 nt + l%32] (dword
// loads: a half-wave reads one 128-B half-row), two register sets so that
// the next round's loads are in flight.  Wave slot C computes the sums on
// the matrix cores too, as S^T B with S_i = [1, wv_i, 0, ...] (rows 0 and 1
// of its first row tile), plus sum wv: summing on the VALU in one of the
// table waves had slowed the whole launch by 14 % (f32 VALU and f32 MFMA
// share the SIMD's f32 rate; tools/mb/mb_gram64.hip).  The block's four
// waves read the same B rows (L1 hits).  Block b takes slot group b % ng and
// row chunk b / ng, so the blocks of one chunk are dispatched together and
// share its B rows in the Infinity Cache.  Partials: part[chunk][c * 4096 +
// m * 64 + n] and the sums at [C * 4096 ..) (k_reduce_parts, fixed order).
constexpr int GW64 = 1;  // tables per wave of k_gram_mfma64 (64 accumulators each)
static __global__ __launch_bounds__(BLOCK, 3) void k_gram_mfma64(uint64_t Rp, int C, const float *const *__restrict__ A,
                                                       const float *__restrict__ B, const float *__restrict__ wv,
                                                       float *__restrict__ part, uint64_t nout,
                                                       uint64_t rows_per_block, unsigned ngroups, unsigned nwork) {
  typedef float f16x __attribute__((ext_vector_type(16)));
  constexpr int U = 4;  // row pairs per round (U = 8: 9 % slower at config 5)
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int e = lane & 31, hf = lane >> 5;
  const unsigned L = (gridDim.x & 7u) ? blockIdx.x : xcd_work_item(blockIdx.x, gridDim.x);
  if (L >= nwork) return;
  const unsigned grp = L % ngroups, chunk = L / ngroups;
  const int c0 = (int)(grp * (BLOCK / 64) + w);
  if (c0 > C) return;  // no barrier below
  f16x acc[4];
#pragma unroll
  for (int t = 0; t < 4; t++)
#pragma unroll
    for (int r = 0; r < 16; r++) acc[t][r] = 0.0f;
  const BufView bb = buf_view(B, Rp * 256);
  const uint64_t r0 = (uint64_t)chunk * rows_per_block;
  const uint64_t r1 = r0 + rows_per_block < Rp ? r0 + rows_per_block : Rp;
  float *out = part + (size_t)chunk * nout;
  if (c0 == C) {  // the sums slot: S^T B, S_i = [1, wv_i, 0, ...]; rows past r1 meet B = 0
    const BufView wb = buf_view(wv, wv ? Rp * 4 : 0);
    float wt = 0;
    for (uint64_t j0 = r0; j0 < r1; j0 += 2 * U) {
      float bv[U][2], sv[U];
#pragma unroll
      for (int u = 0; u < U; u++) {
        const uint64_t jj = j0 + 2 * u + hf;
        const bool ok = jj < r1;
        const uint32_t off = ok ? (uint32_t)(jj * 256 + e * 4) : 0xffffff00u;
#pragma unroll
        for (int h = 0; h < 2; h++) bv[u][h] = bld1<float>(bb, off + h * 128);
        const float wvi = bld1<float>(wb, ok ? (uint32_t)(jj * 4) : 0xffffff00u);
        sv[u] = e == 0 ? 1.0f : (e == 1 ? wvi : 0.0f);
        if (e == 0) wt += wvi;
      }
#pragma unroll
      for (int u = 0; u < U; u++)
#pragma unroll
        for (int nt = 0; nt < 2; nt++) acc[nt] = __builtin_amdgcn_mfma_f32_32x32x2f32(sv[u], bv[u][nt], acc[nt], 0, 0, 0);
    }
    // D row m = 0 (lanes hf = 0, register 0) is sum B, row 1 (register 1) sum wv B
    wt += __shfl_xor(wt, 32, 64);  // lanes 0 and 32 hold the even / odd rows' sums
    if (hf == 0) {
#pragma unroll
      for (int nt = 0; nt < 2; nt++) {
        out[(size_t)C * 4096 + nt * 32 + e] = acc[nt][0];
        out[(size_t)C * 4096 + 64 + nt * 32 + e] = acc[nt][1];
      }
      if (e == 0) out[(size_t)C * 4096 + 128] = wt;
    }
    return;
  }
  const BufView ab = buf_view(A[c0], Rp * 256);
  float bv[2][U][2], av[2][U][2];
  auto load = [&](int sb, uint64_t j0) {
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint64_t jj = j0 + 2 * u + hf;
      const uint32_t off = jj < r1 ? (uint32_t)(jj * 256 + e * 4) : 0xffffff00u;
#pragma unroll
      for (int h = 0; h < 2; h++) {
        bv[sb][u][h] = bld1<float>(bb, off + h * 128);
        av[sb][u][h] = bld1<float>(ab, off + h * 128);
      }
    }
  };
  auto step = [&](int sb) {
#pragma unroll
    for (int u = 0; u < U; u++)
#pragma unroll
      for (int mt = 0; mt < 2; mt++)
#pragma unroll
        for (int nt = 0; nt < 2; nt++)
          acc[mt * 2 + nt] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[sb][u][mt], bv[sb][u][nt], acc[mt * 2 + nt], 0, 0, 0);
  };
  // rows past r1 load zeros (buffer range check), so a trailing round is harmless
  for (uint64_t j0 = r0; j0 < r1; j0 += 4 * U) {
    load(0, j0);
    load(1, j0 + 2 * U);
    step(0);
    step(1);
  }
#pragma unroll
  for (int t = 0; t < 4; t++)
#pragma unroll
    for (int r = 0; r < 16; r++) {
      const int m = (t >> 1) * 32 + 8 * (r >> 2) + 4 * hf + (r & 3), n = (t & 1) * 32 + e;
      out[(size_t)c0 * 4096 + m * 64 + n] = acc[t][r];
    }
}

// Cross-half aggregates at KP = 32, fp64, on the f64 matrix cores: M_c =
// A_c^T B (32 x 32) for every table c < C, oQ = sum_i B_i, bQ = sum_i wv_i
// B_i and sum wv over block x's row chunk, laid out like k_gram_part's
// partials (double; k_reduce_parts).  Wave slot c < C owns table c and walks
// the chunk four rows at a time: v_mfma_f64_16x16x4f64 takes them as the K
// dimension, lane l supplying A_c[row l/16][16 mt + l%16] and B[row l/16][16
// nt + l%16] (tiles mt, nt of the 2 x 2 grid; D register r of lane l is
// element (16 mt + l/16 + 4r, 16 nt + l%16)), two register sets in flight.
// Wave slot C sums B and wv B on the VALU.
static __global__ __launch_bounds__(BLOCK) void k_gram_mfma_f64(uint64_t Rp, int C, const double *const *__restrict__ A,
                                                               const double *__restrict__ B,
                                                               const double *__restrict__ wv, double *__restrict__ part,
                                                               uint64_t nout, uint64_t rows_per_block,
                                                               unsigned ngroups, unsigned nwork) {
  typedef double d4 __attribute__((ext_vector_type(4)));
  constexpr int U = 4;  // groups of four rows per register set
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c16 = lane & 15, rq = lane >> 4;
  const unsigned L = (gridDim.x & 7u) ? blockIdx.x : xcd_work_item(blockIdx.x, gridDim.x);  // (k_gram_mfma64)
  if (L >= nwork) return;
  const unsigned grp = L % ngroups, chunk = L / ngroups;
  const int c0 = (int)(grp * (BLOCK / 64) + w);
  if (c0 > C) return;  // no barrier below
  const uint64_t r0 = (uint64_t)chunk * rows_per_block;
  const uint64_t r1 = r0 + rows_per_block < Rp ? r0 + rows_per_block : Rp;
  double *out = part + (size_t)chunk * nout;
  const BufView bb = buf_view(B, Rp * 256);
  if (c0 == C) {  // the sums slot
    const BufView wb = buf_view(wv, wv ? Rp * 8 : 0);
    double cs[2] = {0, 0}, ws[2] = {0, 0}, wt = 0;
    for (uint64_t j0 = r0; j0 < r1; j0 += 4 * U) {
#pragma unroll
      for (int u = 0; u < U; u++) {
        const uint64_t jj = j0 + 4 * u + rq;
        const bool ok = jj < r1;
        const uint32_t off = ok ? (uint32_t)(jj * 256 + c16 * 8) : 0xffffff00u;
        const double wvi = bld1<double>(wb, ok ? (uint32_t)(jj * 8) : 0xffffff00u);
#pragma unroll
        for (int h = 0; h < 2; h++) {
          const double b = bld1<double>(bb, off + h * 128);
          cs[h] += b;
          ws[h] += wvi * b;
        }
        if (c16 == 0) wt += wvi;
      }
    }
#pragma unroll
    for (int o = 16; o < 64; o <<= 1) {
#pragma unroll
      for (int h = 0; h < 2; h++) {
        cs[h] += __shfl_xor(cs[h], o, 64);
        ws[h] += __shfl_xor(ws[h], o, 64);
      }
      wt += __shfl_xor(wt, o, 64);
    }
    if (rq == 0) {
#pragma unroll
      for (int h = 0; h < 2; h++) {
        out[(size_t)C * 1024 + h * 16 + c16] = cs[h];
        out[(size_t)C * 1024 + 32 + h * 16 + c16] = ws[h];
      }
      if (c16 == 0) out[(size_t)C * 1024 + 64] = wt;
    }
    return;
  }
  const BufView ab = buf_view(A[c0], Rp * 256);
  d4 acc[4];
#pragma unroll
  for (int t = 0; t < 4; t++) acc[t] = d4{0.0, 0.0, 0.0, 0.0};
  double av[2][U][2], bv[2][U][2];
  auto load = [&](int sb, uint64_t j0) {
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint64_t jj = j0 + 4 * u + rq;
      const uint32_t off = jj < r1 ? (uint32_t)(jj * 256 + c16 * 8) : 0xffffff00u;
#pragma unroll
      for (int h = 0; h < 2; h++) {
        av[sb][u][h] = bld1<double>(ab, off + h * 128);
        bv[sb][u][h] = bld1<double>(bb, off + h * 128);
      }
    }
  };
  auto step = [&](int sb) {
#pragma unroll
    for (int u = 0; u < U; u++)
#pragma unroll
      for (int mt = 0; mt < 2; mt++)
#pragma unroll
        for (int nt = 0; nt < 2; nt++)
          acc[mt * 2 + nt] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[sb][u][mt], bv[sb][u][nt], acc[mt * 2 + nt], 0, 0, 0);
  };
  // rows past r1 load zeros (buffer range check), so a trailing round is harmless
  for (uint64_t j0 = r0; j0 < r1; j0 += 8 * U) {
    load(0, j0);
    load(1, j0 + 4 * U);
    step(0);
    step(1);
  }
#pragma unroll
  for (int t = 0; t < 4; t++)
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const int m = (t >> 1) * 16 + rq + 4 * r, n = (t & 1) * 16 + c16;
      out[(size_t)c0 * 1024 + m * 32 + n] = acc[t][r];
    }
}

// o in [0, cnt): t = sum_b part[b][off + o]; o < split -> out_real[o] = t,
// else out_dbl[o - split] = t.  A block owns 16 consecutive outputs
// (coalesced 128-B reads) and 16 groups of partial rows; groups are combined
// in fixed order through LDS (deterministic).
// PT: the partials' type (double; float for k_gram_mfma32, whose partials
// are f32 MFMA accumulators: half the bytes, the same values).
template <typename real, typename PT = double>
__global__ __launch_bounds__(BLOCK) void k_reduce_parts(uint64_t nb, uint64_t nout, uint64_t off, uint64_t cnt,
                                                        const PT *__restrict__ part, uint64_t split,
                                                        real *__restrict__ out_real, double *__restrict__ out_dbl) {
  __shared__ double sh[16][17];
  const int to = threadIdx.x & 15, tg = threadIdx.x >> 4;
  const uint64_t o = (uint64_t)blockIdx.x * 16 + to;
  double s = 0;
  if (o < cnt) {
    const PT *p = part + off + o;
    uint64_t b = tg;
    for (; b + 48 < nb; b += 64) {
      const double x0 = p[b * nout], x1 = p[(b + 16) * nout], x2 = p[(b + 32) * nout], x3 = p[(b + 48) * nout];
      s += (x0 + x1) + (x2 + x3);
    }
    for (; b < nb; b += 16) s += p[b * nout];
  }
  sh[tg][to] = s;
  __syncthreads();
  if (tg == 0 && o < cnt) {
    double t = 0;
#pragma unroll
    for (int g = 0; g < 16; g++) t += sh[g][to];
    if (o < split) out_real[o] = (real)t;
    else out_dbl[o - split] = t;
  }
}

// out = sum_i v[i] in double (b_sum of gd_side, ffm.cpp:551): block sums,
// then the last block combines them in block order (deterministic).
template <typename real>
__global__ __launch_bounds__(BLOCK) void k_vec_sum(uint64_t n, const real *__restrict__ v, double *__restrict__ out,
                                                   double *part, unsigned *tick) {
  double s = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; i < n; i += (uint64_t)gridDim.x * BLOCK)
    s += (double)v[i];
  const double bv[1] = {block_sum(s)};
  double tot[1];
  if (last_block<1>(bv, part, tick, tot) && threadIdx.x == 0) out[0] = tot[0];
}

// Column sums of C tables at once (cache_sasb, ffm.cpp:514-535):
// part[block][c*KP + d] = sum over the block's rows j of T_c[j][d].  Rows are
// read 16 B per lane, BLOCK/LPR rows per pass; row groups are combined in
// fixed order through LDS (deterministic); k_reduce_parts sums the blocks.
template <typename real, int KP>
__global__ __launch_bounds__(BLOCK) void k_colsum_multi(uint64_t R, int C, const real *const *__restrict__ tabs,
                                                        double *__restrict__ part, uint64_t rows_per_block) {
  using G = Geo<real, KP>;
  constexpr int RG = BLOCK / G::LPR;  // row groups per pass
  __shared__ double sh[RG][KP + 1];
  const int li = threadIdx.x % G::LPR, rg = threadIdx.x / G::LPR;
  const uint64_t r0 = (uint64_t)blockIdx.x * rows_per_block;
  const uint64_t r1 = min(R, r0 + rows_per_block);
  for (int c = 0; c < C; c++) {
    const real *T = tabs[c];
    double a[G::VE];
#pragma unroll
    for (int e = 0; e < G::VE; e++) a[e] = 0;
    uint64_t j = r0 + rg;
    for (; j + 3 * RG < r1; j += 4 * RG) {
      const vec_t<real> x0 = vld<real>(T + j * KP + li * G::VE), x1 = vld<real>(T + (j + RG) * KP + li * G::VE);
      const vec_t<real> x2 = vld<real>(T + (j + 2 * RG) * KP + li * G::VE);
      const vec_t<real> x3 = vld<real>(T + (j + 3 * RG) * KP + li * G::VE);
#pragma unroll
      for (int e = 0; e < G::VE; e++) a[e] += ((double)x0[e] + (double)x1[e]) + ((double)x2[e] + (double)x3[e]);
    }
    for (; j < r1; j += RG) {
      const vec_t<real> x = vld<real>(T + j * KP + li * G::VE);
#pragma unroll
      for (int e = 0; e < G::VE; e++) a[e] += (double)x[e];
    }
    __syncthreads();
#pragma unroll
    for (int e = 0; e < G::VE; e++) sh[rg][li * G::VE + e] = a[e];
    __syncthreads();
    if (threadIdx.x < KP) {
      double t = 0;
      for (int g = 0; g < RG; g++) t += sh[g][threadIdx.x];
      part[(uint64_t)blockIdx.x * C * KP + (uint64_t)c * KP + threadIdx.x] = t;
    }
  }
}

// ------------------------------------------------------- validation ---
// z[r][j] = bt_j + sum_c <Pva_c[i], Qva_c[j]> for test row i = row0 + r
// (pred_z, ffm.cpp:915-923); cold rows (no kept feature) score by train
// popularity (ffm.cpp:975-977).
template <typename real, int KP>
__global__ __launch_bounds__(BLOCK) void k_scores(uint64_t rows, uint64_t row0, uint64_t n, int C,
                                                  const real *const *__restrict__ Pva,
                                                  const real *const *__restrict__ Qva, const real *__restrict__ bt,
                                                  const uint8_t *__restrict__ cold, const double *__restrict__ popular,
                                                  uint64_t npop, double *__restrict__ z) {
  const uint64_t r = blockIdx.y;
  const uint64_t i = row0 + r;
  double *zr = z + r * n;
  if (cold[i]) {
    for (uint64_t j = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; j < n; j += (uint64_t)gridDim.x * BLOCK)
      zr[j] = j < npop ? popular[j] : -1.0e300;
    return;
  }
  for (uint64_t j = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; j < n; j += (uint64_t)gridDim.x * BLOCK) {
    real s = bt[j];
    for (int c = 0; c < C; c++) {
      const real *p = Pva[c] + i * KP;
      const real *q = Qva[c] + j * KP;
      real d = 0;
#pragma unroll
      for (int e = 0; e < KP; e++) d += p[e] * q[e];
      s += d;
    }
    zr[j] = (double)s;
  }
}

// Per test row: ploss term, then repeated argmax over z[0:max_z) with
// z[argmax] = MIN_Z (-1000) and first-index tie-break, accumulating hits and
// DCG/IDCG at the cut-offs 5,10,20,40,80 (validate/prec_k/ndcg,
// ffm.cpp:982-1128).  One block per row.  out[r] = {ploss, hits[5], ndcg[5]}.
// forced: the reference's EBUG_nDCG build (ffm.cpp:988-993): after the
// ploss term the row's scores are replaced by z_j = n - j, j < n.
static __global__ __launch_bounds__(BLOCK) void k_rank(uint64_t rows, uint64_t row0, uint64_t n, uint64_t max_z,
                                                double *__restrict__ z, const int64_t *__restrict__ lptr,
                                                const uint32_t *__restrict__ lcol, const uint8_t *__restrict__ cold,
                                                uint64_t npop, const double *__restrict__ at,
                                                double *__restrict__ out, int forced) {
  const uint64_t r = blockIdx.x;
  const uint64_t i = row0 + r;
  double *zr = z + r * n;
  const int64_t l0 = lptr[i], l1 = lptr[i + 1];
  const uint64_t zs0 = cold[i] ? npop : n;  // size of the row's score vector (popularity: #train items)
  const uint64_t zsize = forced ? n : zs0;     // (resized to n by the forced build)
  const uint64_t mz = max_z < zsize ? max_z : zsize;
  __shared__ double s_val[BLOCK / 64];
  __shared__ uint64_t s_idx[BLOCK / 64];
  __shared__ uint64_t s_am;
  // ploss
  double pl = 0;
  for (int64_t p = l0 + threadIdx.x; p < l1; p += BLOCK) {
    const uint64_t j = lcol[p];
    if (j < zs0) {
      const double d = 1 - zr[j] - at[i];
      pl += d * d;
    }
  }
  pl = block_sum(pl);
  if (forced) {
    for (uint64_t j = threadIdx.x; j < n; j += BLOCK) zr[j] = (double)(n - j);
    __syncthreads();
  }
  const int cut[5] = {5, 10, 20, 40, 80};
  double hits[5] = {0, 0, 0, 0, 0}, dcg[5] = {0, 0, 0, 0, 0}, idcg[5] = {0, 0, 0, 0, 0};
  const uint64_t nlab = (uint64_t)(l1 - l0);
  uint64_t cnt = 0;
  for (int s = 0; s < 5; s++) {
    while (cnt < (uint64_t)cut[s]) {
      if (cnt >= mz) break;
      double bv = -1.0e308;
      uint64_t bi = ~0ULL;
      for (uint64_t j = threadIdx.x; j < mz; j += BLOCK) {
        const double v = zr[j];
        if (v > bv) {  // strided scan: keeps the lowest index among equals
          bv = v;
          bi = j;
        }
      }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        const double ov = __shfl_xor(bv, o, 64);
        const uint64_t oi = __shfl_xor(bi, o, 64);
        if (ov > bv || (ov == bv && oi < bi)) {
          bv = ov;
          bi = oi;
        }
      }
      __syncthreads();
      if ((threadIdx.x & 63) == 0) {
        s_val[threadIdx.x >> 6] = bv;
        s_idx[threadIdx.x >> 6] = bi;
      }
      __syncthreads();
      if (threadIdx.x == 0) {
        double v = s_val[0];
        uint64_t id = s_idx[0];
        for (int w2 = 1; w2 < BLOCK / 64; w2++)
          if (s_val[w2] > v || (s_val[w2] == v && s_idx[w2] < id)) {
            v = s_val[w2];
            id = s_idx[w2];
          }
        s_am = id;
        zr[id] = -1000.0;  // MIN_Z (ffm.h:40)
      }
      __syncthreads();
      const uint64_t am = s_am;
      if (threadIdx.x == 0) {
        bool hit = false;
        for (uint64_t t = 0; t < nlab; t++)
          if (lcol[l0 + t] == am) {
            hit = true;
            break;
          }
        const double g = 1.0 / log2((double)cnt + 2);
        if (hit) {
          hits[s] += 1;
          dcg[s] += g;
        }
        if (nlab > cnt) idcg[s] += g;
      }
      cnt++;
    }
  }
  if (threadIdx.x == 0) {
    for (int s = 1; s < 5; s++) {
      hits[s] += hits[s - 1];
      dcg[s] += dcg[s - 1];
      idcg[s] += idcg[s - 1];
    }
    double *o = out + r * 11;
    o[0] = pl;
    for (int s = 0; s < 5; s++) {
      o[1 + s] = hits[s];
      o[6 + s] = dcg[s] / idcg[s];
    }
  }
}

}  // namespace ocffm
