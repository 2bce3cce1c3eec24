// devbuild.hip — on-device build of the solver's data layout (see
// devbuild.h).  Every kernel is integer/byte work over the parsed rows:
// per-row counts, prefix scans (three-pass, below), stable LSD radix sorts (rocPRIM:
// equal keys keep their input order, which is what makes every array equal
// the host build's sequential loops), gathers and scatters.  HBM-bound; the
// largest input (config 5: 78 M nodes) is read a few times.
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/iterator/counting_iterator.hpp>

#include <algorithm>
#include <cstring>

#include "devbuild.h"

namespace ocffm {
namespace dev {

namespace {

constexpr int TB = 256;

unsigned grid(uint64_t n, unsigned cap = 8192) {
  const uint64_t g = (n + TB - 1) / TB;
  return (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(g, cap));
}

#define GSTRIDE(i, n) for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < (n); i += (uint64_t)gridDim.x * blockDim.x)

// ---------------------------------------------------------- split_fields
// cnt[f * (R + 1) + i + 1] = nodes of row i in field f (ffm.cpp:196-206).
__global__ void k_field_count(uint64_t R, const uint64_t *__restrict__ xptr, uint64_t x0,
                              const uint32_t *__restrict__ fid, uint32_t nf, int64_t *__restrict__ cnt) {
  GSTRIDE(i, R) {
    for (uint64_t p = xptr[i] - x0; p < xptr[i + 1] - x0; p++) {
      const uint32_t f = fid[p];
      if (f < nf) cnt[(uint64_t)f * (R + 1) + i + 1]++;
    }
  }
}

// Per-field row pointers out of the inclusive scan S of cnt.
__global__ void k_field_ptr(uint64_t R, uint32_t nf, const int64_t *__restrict__ S, int64_t *__restrict__ xptr) {
  GSTRIDE(t, (uint64_t)nf * (R + 1)) {
    const uint64_t f = t / (R + 1);
    xptr[t] = S[t] - S[f * (R + 1)];
  }
}

// Each row's nodes to its fields in row order (ffm.cpp:208-226): the row's
// cursor in field f is S[f (R+1) + i] (this thread's alone).
__global__ void k_field_scatter(uint64_t R, const uint64_t *__restrict__ xptr, uint64_t x0,
                                const uint32_t *__restrict__ fid, const uint64_t *__restrict__ idx,
                                const double *__restrict__ val, uint32_t nf, int64_t *__restrict__ S,
                                uint32_t *__restrict__ oidx, double *__restrict__ oval) {
  GSTRIDE(i, R) {
    for (uint64_t p = xptr[i] - x0; p < xptr[i + 1] - x0; p++) {
      const uint32_t f = fid[p];
      if (f >= nf) continue;
      const int64_t q = S[(uint64_t)f * (R + 1) + i]++;
      oidx[q] = (uint32_t)idx[p];
      oval[q] = val[p];
    }
  }
}

// ------------------------------------------------------------------- CSC
__global__ void k_rowid(uint64_t R, const int64_t *__restrict__ ptr, uint32_t *__restrict__ out) {
  GSTRIDE(i, R) {
    for (int64_t p = ptr[i] - ptr[0]; p < ptr[i + 1] - ptr[0]; p++) out[p] = (uint32_t)i;
  }
}

// cptr[d] = position of the first key >= d in the sorted keys (cptr[D]:
// the count of keys < D): every d is written once, no atomics (a histogram
// serialised on the popular columns' counters).
__global__ void k_bounds(uint64_t n, const uint32_t *__restrict__ keys, uint64_t D, int64_t *__restrict__ cptr) {
  GSTRIDE(q, n + 1) {
    const int64_t lo = q == 0 ? -1 : (int64_t)std::min<uint64_t>(keys[q - 1], D);
    const int64_t hi = q == n ? (int64_t)D : (int64_t)std::min<uint64_t>(keys[q], D);
    for (int64_t d = lo + 1; d <= hi; d++) cptr[d] = (int64_t)q;
  }
}

__global__ void k_csc_fill(uint64_t n, const uint32_t *__restrict__ perm, const uint32_t *__restrict__ rowid,
                           const double *__restrict__ xval, uint32_t *__restrict__ crow, double *__restrict__ cval) {
  GSTRIDE(q, n) {
    const uint32_t p = perm[q];
    crow[q] = rowid[p];
    cval[q] = xval[p];
  }
}

// Per column: light job (1), heavy jobs (np * nsg) and heavy slots (np).
__global__ void k_job_count(uint64_t D, const int64_t *__restrict__ cptr, const uint8_t *__restrict__ own, int nsg,
                            int64_t *__restrict__ lc, int64_t *__restrict__ hc, int64_t *__restrict__ sc) {
  GSTRIDE(d, D) {
    const uint64_t n = (uint64_t)(cptr[d + 1] - cptr[d]);
    const bool mine = !own || own[d];
    const bool light = n <= (uint64_t)JOB_ENT;
    lc[d] = light && mine ? 1 : 0;
    uint64_t np = 0;
    if (!light && mine) {
      const uint64_t wc = (uint64_t)nsg * JOB_ENT * heavy_rounds(n, nsg);
      np = (n + wc - 1) / wc;
    }
    hc[d] = (int64_t)(np * nsg);
    sc[d] = (int64_t)np;
  }
}

// Jobs in build_csc's order; L/H/S: inclusive scans of the counts above.
__global__ void k_job_write(uint64_t D, const int64_t *__restrict__ cptr, const uint8_t *__restrict__ own, int nsg,
                            const int64_t *__restrict__ L, const int64_t *__restrict__ H,
                            const int64_t *__restrict__ S, uint64_t nlight_pad, Job *__restrict__ jobs) {
  GSTRIDE(d, D) {
    const int64_t b = cptr[d], e = cptr[d + 1];
    const uint64_t n = (uint64_t)(e - b);
    const bool mine = !own || own[d];
    if (!mine) continue;
    if (n <= (uint64_t)JOB_ENT) {
      jobs[L[d] - 1] = Job{(uint32_t)d, 1u, 0u, 0u, b, e};
      continue;
    }
    const uint64_t sub = (uint64_t)JOB_ENT * heavy_rounds(n, nsg), wc = (uint64_t)nsg * sub;
    const uint32_t np = (uint32_t)((n + wc - 1) / wc);
    const uint64_t base = nlight_pad + (uint64_t)(H[d] - (int64_t)np * nsg);
    const uint32_t slot0 = (uint32_t)(S[d] - np);
    for (uint32_t q = 0; q < np; q++)
      for (int g = 0; g < nsg; g++) {
        const int64_t sb = std::min<int64_t>(e, b + (int64_t)(q * wc + (uint64_t)g * sub));
        const int64_t se = std::min<int64_t>(e, sb + (int64_t)sub);
        jobs[base + (uint64_t)q * nsg + g] = Job{(uint32_t)d, np, slot0 + q, 1u | (q << 1), sb, se};
      }
  }
}

__global__ void k_job_pad(uint64_t b, uint64_t e, Job *__restrict__ jobs) {
  GSTRIDE(t, e - b) jobs[b + t] = Job{JOB_NONE, 1u, 0u, 0u, 0, 0};
}

// -------------------------------------------------------- flags / sums
__global__ void k_flags(uint64_t R, const int64_t *__restrict__ xptr, uint64_t D, const int64_t *__restrict__ cptr,
                        unsigned long long *__restrict__ bad) {
  unsigned long long br = 0, bc = 0;
  GSTRIDE(i, R) br += xptr[i + 1] - xptr[i] != 1;
  GSTRIDE(d, D) bc += cptr[d + 1] - cptr[d] != 1;
  if (br) atomicAdd(&bad[0], br);
  if (bc) atomicAdd(&bad[1], bc);
}

// Sum of x^2 per column (one block per column) in the order xsq_col
// (devbuild.h) states for the host: 256 strided partials, then a fixed tree.
// (A thread per column walked a popular column's ~600 k rows serially.)
__global__ void __launch_bounds__(TB) k_xsq(uint64_t D, const int64_t *__restrict__ cptr,
                                            const double *__restrict__ cval, double *__restrict__ out) {
#pragma clang fp contract(off)
  __shared__ double lds[TB];
  const int t = threadIdx.x;
  for (uint64_t d = blockIdx.x; d < D; d += gridDim.x) {
    const int64_t b = cptr[d], e = cptr[d + 1];
    double s = 0.0;
    int64_t q = b + t;
    for (; q + 3 * TB < e; q += 4 * TB) {  // loads batched, adds in q order
      const double v0 = cval[q], v1 = cval[q + TB], v2 = cval[q + 2 * TB], v3 = cval[q + 3 * TB];
      s = s + v0 * v0;
      s = s + v1 * v1;
      s = s + v2 * v2;
      s = s + v3 * v3;
    }
    for (; q < e; q += TB) {
      const double v = cval[q];
      s = s + v * v;
    }
    lds[t] = s;
    __syncthreads();
    for (int o = TB / 2; o > 0; o >>= 1) {
      if (t < o) lds[t] = lds[t] + lds[t + o];
      __syncthreads();
    }
    if (t == 0) out[d] = lds[0];
    __syncthreads();
  }
}

__global__ void k_col_counts(uint64_t D, const int64_t *__restrict__ cptr, double *__restrict__ out) {
  GSTRIDE(d, D) out[d] = (double)(cptr[d + 1] - cptr[d]);
}

// ------------------------------------------------------------- segments
__global__ void k_seg_count(uint64_t R, const int64_t *__restrict__ yptr, uint64_t len, int64_t *__restrict__ c) {
  GSTRIDE(i, R) {
    const int64_t n = yptr[i + 1] - yptr[i];
    c[i] = std::max<int64_t>(1, (n + (int64_t)len - 1) / (int64_t)len);
  }
}

// S: inclusive scan of the per-row segment counts.
__global__ void k_seg_write(uint64_t R, const int64_t *__restrict__ yptr, uint64_t len, const int64_t *__restrict__ S,
                            Seg *__restrict__ segs, uint32_t *__restrict__ segptr) {
  GSTRIDE(i, R) {
    const int64_t b = yptr[i], e = yptr[i + 1];
    const uint32_t s0 = i ? (uint32_t)S[i - 1] : 0u, nrow = (uint32_t)(S[i] - (i ? S[i - 1] : 0));
    segptr[i] = s0;
    if (i + 1 == R) segptr[R] = (uint32_t)S[i];
    int64_t p = b;
    for (uint32_t q = 0; q < nrow; q++) {
      const int64_t pe = std::min<int64_t>(e, p + (int64_t)len);
      segs[s0 + q] = Seg{(uint32_t)i, (nrow << 1) | (q == 0 ? 1u : 0u), p, pe};
      p = pe;
    }
  }
}

__global__ void k_seg_nodes(uint64_t nseg, const Seg *__restrict__ segs, const int64_t *__restrict__ xptr,
                            int64_t *__restrict__ c) {
  GSTRIDE(s, nseg) {
    const uint32_t i = segs[s].row;
    c[s] = xptr[i + 1] - xptr[i];
  }
}

__global__ void k_seg_copy(uint64_t nseg, const Seg *__restrict__ segs, const int64_t *__restrict__ xptr,
                           const uint32_t *__restrict__ xidx, const double *__restrict__ xval,
                           const int64_t *__restrict__ sptr, uint32_t *__restrict__ oidx, double *__restrict__ oval) {
  GSTRIDE(s, nseg) {
    const uint32_t i = segs[s].row;
    int64_t q = sptr[s];
    for (int64_t p = xptr[i]; p < xptr[i + 1]; p++, q++) {
      oidx[q] = xidx[p];
      oval[q] = xval[p];
    }
  }
}

// --------------------------------------------------------------- labels
__global__ void k_rebase(uint64_t n, const uint64_t *__restrict__ in, int64_t *__restrict__ out) {
  GSTRIDE(i, n) out[i] = (int64_t)(in[i] - in[0]);
}

__global__ void k_narrow(uint64_t n, const uint64_t *__restrict__ in, uint32_t *__restrict__ out) {
  GSTRIDE(i, n) out[i] = (uint32_t)std::min<uint64_t>(in[i], 0xffffffffull);
}

// vcol[q] = local user of positive v2u[q]; u2v the inverse map.
__global__ void k_trans_fill(uint64_t np, const uint32_t *__restrict__ v2u, const uint32_t *__restrict__ rowid,
                             uint32_t *__restrict__ vcol, uint32_t *__restrict__ u2v) {
  GSTRIDE(q, np) {
    const uint32_t p = v2u[q];
    vcol[q] = rowid[p];
    u2v[p] = (uint32_t)q;
  }
}

__global__ void k_pop(uint64_t n, const int64_t *__restrict__ ptr, double total, double *__restrict__ out) {
  GSTRIDE(j, n) out[j] = (double)(ptr[j + 1] - ptr[j]) / total;
}

// ----------------------------------------------------------------- scans
// Inclusive int64 scan in three launches (tile sums, one-block scan of the
// tile sums, tile scans with their offsets).  rocPRIM's single-pass scan
// queries the device properties on every call (~ms on this runtime), which
// dominated the per-field build; these take a few microseconds each.
constexpr int SCAN_IT = 8, SCAN_TILE = TB * SCAN_IT;

__device__ int64_t block_excl_scan(int64_t v, int64_t *lds, int64_t &total) {
  const int t = threadIdx.x;
  lds[t] = v;
  __syncthreads();
  for (int o = 1; o < TB; o <<= 1) {
    const int64_t a = t >= o ? lds[t - o] : 0;
    __syncthreads();
    lds[t] += a;
    __syncthreads();
  }
  total = lds[TB - 1];
  const int64_t r = lds[t] - v;
  __syncthreads();
  return r;
}

__global__ void __launch_bounds__(TB) k_scan_tiles(uint64_t n, const int64_t *__restrict__ in,
                                                   int64_t *__restrict__ tsum) {
  __shared__ int64_t lds[TB];
  const uint64_t b = (uint64_t)blockIdx.x * SCAN_TILE + (uint64_t)threadIdx.x * SCAN_IT;
  int64_t v = 0;
  for (int k = 0; k < SCAN_IT; k++)
    if (b + k < n) v += in[b + k];
  int64_t tot;
  block_excl_scan(v, lds, tot);
  if (threadIdx.x == 0) tsum[blockIdx.x] = tot;
}

// one block: tsum := exclusive scan of tsum[0, nt)
__global__ void __launch_bounds__(TB) k_scan_top(uint64_t nt, int64_t *__restrict__ tsum) {
  __shared__ int64_t lds[TB];
  const uint64_t per = (nt + TB - 1) / TB, b = (uint64_t)threadIdx.x * per;
  int64_t v = 0;
  for (uint64_t k = 0; k < per; k++)
    if (b + k < nt) v += tsum[b + k];
  int64_t tot;
  int64_t run = block_excl_scan(v, lds, tot);
  for (uint64_t k = 0; k < per; k++)
    if (b + k < nt) {
      const int64_t x = tsum[b + k];
      tsum[b + k] = run;
      run += x;
    }
}

__global__ void __launch_bounds__(TB) k_scan_apply(uint64_t n, const int64_t *__restrict__ in,
                                                   const int64_t *__restrict__ toff, int64_t *__restrict__ out) {
  __shared__ int64_t lds[TB];
  const uint64_t b = (uint64_t)blockIdx.x * SCAN_TILE + (uint64_t)threadIdx.x * SCAN_IT;
  int64_t x[SCAN_IT], v = 0;
  for (int k = 0; k < SCAN_IT; k++) {
    x[k] = b + k < n ? in[b + k] : 0;
    v += x[k];
  }
  int64_t tot;
  int64_t run = block_excl_scan(v, lds, tot) + toff[blockIdx.x];
  for (int k = 0; k < SCAN_IT; k++) {
    run += x[k];
    if (b + k < n) out[b + k] = run;
  }
}

// --------------------------------------------------------------- init_mat
// minstd_rand0: x' = 16807 x mod (2^31 - 1), reduced without a division
__device__ __forceinline__ uint64_t lcg_mul(uint64_t x, uint64_t a) {
  const uint64_t p = x * a;  // < 2^62
  const uint64_t r = (p & 0x7fffffffull) + (p >> 31);
  return r >= 0x7fffffffull ? r - 0x7fffffffull : r;
}
__device__ __forceinline__ uint64_t lcg_pow(uint64_t e) {
  uint64_t r = 1, a = 16807;
  for (; e; e >>= 1, a = lcg_mul(a, a))
    if (e & 1) r = lcg_mul(r, a);
  return r;
}

// A wave draws DRAW_RUN consecutive values per lane, interleaved: lane l
// takes values base + l + 64 j (coalesced stores), so its engine state jumps
// 128 steps (A^128) between its values.  Value i consumes engine outputs
// 2i + 1 and 2i + 2 of the table's stream.
constexpr int DRAW_RUN = 64;
template <typename real>
__global__ void __launch_bounds__(TB) k_draw(uint64_t n, uint32_t cols, uint32_t kp, uint64_t x0, double a,
                                             double width, double r2, uint64_t a128, real *__restrict__ out) {
  const uint64_t wave = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) / 64, lane = threadIdx.x % 64;
  const uint64_t base = wave * 64 * DRAW_RUN;
  if (base >= n) return;
  uint64_t x = lcg_mul(x0, lcg_pow(2 * (base + lane)));  // state before value base + lane
  for (int j = 0; j < DRAW_RUN; j++) {
    const uint64_t i = base + lane + 64 * (uint64_t)j;
    if (i >= n) break;
    const uint64_t u1 = lcg_mul(x, 16807), u2 = lcg_mul(u1, 16807);
    const double sum = __fma_rn((double)(u2 - 1), 2147483646.0, (double)(u1 - 1));
    double c = __ddiv_rn(sum, r2);
    if (c >= 1.0) c = 0x1.fffffffffffffp-1;  // nextafter(1, 0)
    const double v = __fma_rn(c, width, a);
    out[(i / cols) * kp + (i % cols)] = (real)v;
    x = lcg_mul(x, a128);
  }
}

}  // namespace

template <typename real>
void draw_table(hipStream_t s, real *out, uint64_t rows, uint32_t cols, uint32_t kp, const TableDraw &t) {
  const uint64_t n = rows * cols;
  if (!n) return;
  uint64_t a128 = 1;
  for (int q = 0; q < 128; q++) a128 = a128 * 16807 % 0x7fffffffull;
  const uint64_t waves = (n + 64 * DRAW_RUN - 1) / (64 * DRAW_RUN);
  const uint64_t blocks = (waves * 64 + TB - 1) / TB;
  hipLaunchKernelGGL(k_draw<real>, (unsigned)blocks, TB, 0, s, n, cols, kp, t.x0, t.a, t.width, t.r2, a128, out);
  HIPCHK(hipGetLastError());
}
template void draw_table<float>(hipStream_t, float *, uint64_t, uint32_t, uint32_t, const TableDraw &);
template void draw_table<double>(hipStream_t, double *, uint64_t, uint32_t, uint32_t, const TableDraw &);

// ---------------------------------------------------------------- host side
void Builder::incl_scan(const int64_t *in, int64_t *out, uint64_t n) {
  if (!n) return;
  const uint64_t nt = (n + SCAN_TILE - 1) / SCAN_TILE;
  if (nt > 0x7fffffffull) throw Error(OCFFM_E_DATA, "scan too long");
  int64_t *ts = grow(t_tile_, nt);
  hipLaunchKernelGGL(k_scan_tiles, (unsigned)nt, TB, 0, s_, n, in, ts);
  hipLaunchKernelGGL(k_scan_top, 1, TB, 0, s_, nt, ts);
  hipLaunchKernelGGL(k_scan_apply, (unsigned)nt, TB, 0, s_, n, in, (const int64_t *)ts, out);
}

void Builder::sort_positions(const uint32_t *kin, uint32_t *kout, uint32_t *vout, uint64_t n, uint64_t maxkey) {
  if (!n) return;
  unsigned bits = 1;
  while (bits < 32 && (maxkey >> bits)) bits++;
  const rocprim::counting_iterator<uint32_t> pos(0u);
  size_t bytes = 0;
  HIPCHK(rocprim::radix_sort_pairs(nullptr, bytes, kin, kout, pos, vout, (size_t)n, 0u, bits, s_));
  HIPCHK(rocprim::radix_sort_pairs(scr_.get(bytes, s_), bytes, kin, kout, pos, vout, (size_t)n, 0u, bits, s_));
}

void Builder::rowid(const int64_t *ptr, uint64_t R, uint32_t *out) {
  if (R) hipLaunchKernelGGL(k_rowid, grid(R), TB, 0, s_, R, ptr, out);
}

void Builder::bounds(const uint32_t *sorted, uint64_t n, uint64_t D, int64_t *ptr) {
  hipLaunchKernelGGL(k_bounds, grid(n + 1), TB, 0, s_, n, sorted, D, ptr);
}

std::vector<CSR> Builder::split(const HostData &d, uint64_t r0, uint64_t r1, uint32_t nf) {
  const Rows &raw = d.raw;
  const uint64_t R = r1 - r0;
  const uint64_t x0 = raw.xptr[r0], x1 = raw.xptr[r1], nn = x1 - x0;
  DevBuf<uint64_t> xptr;
  DevBuf<uint32_t> fid;
  DevBuf<uint64_t> idx;
  DevBuf<double> val;
  xptr.upload(raw.xptr.data() + r0, R + 1);
  fid.upload(raw.fid.data() + x0, nn);
  idx.upload(raw.idx.data() + x0, nn);
  val.upload(raw.val.data() + x0, nn);
  const uint64_t cells = (uint64_t)nf * (R + 1);
  DevBuf<int64_t> cnt, S, fptr;
  cnt.alloc(std::max<uint64_t>(cells, 1));  // zeroed
  S.alloc(std::max<uint64_t>(cells, 1), false);
  fptr.alloc(std::max<uint64_t>(cells, 1), false);
  if (R && nf) hipLaunchKernelGGL(k_field_count, grid(R), TB, 0, s_, R, xptr.p, x0, fid.p, nf, cnt.p);
  incl_scan(cnt.p, S.p, cells);
  if (cells) hipLaunchKernelGGL(k_field_ptr, grid(cells), TB, 0, s_, R, nf, S.p, fptr.p);
  DevBuf<uint32_t> oidx;
  DevBuf<double> oval;
  oidx.alloc(std::max<uint64_t>(nn, 1), false);
  oval.alloc(std::max<uint64_t>(nn, 1), false);
  // field starts (before the scatter moves the cursors)
  std::vector<int64_t> fstart(nf + 1, 0);
  for (uint32_t f = 0; f < nf; f++)
    HIPCHK(hipMemcpyAsync(&fstart[f], S.p + (uint64_t)f * (R + 1), sizeof(int64_t), hipMemcpyDeviceToHost, s_));
  if (cells) HIPCHK(hipMemcpyAsync(&fstart[nf], S.p + cells - 1, sizeof(int64_t), hipMemcpyDeviceToHost, s_));
  sync();
  if (R && nf)
    hipLaunchKernelGGL(k_field_scatter, grid(R), TB, 0, s_, R, xptr.p, x0, fid.p, idx.p, val.p, nf, S.p, oidx.p, oval.p);
  std::vector<CSR> out(nf);
  for (uint32_t f = 0; f < nf; f++) {
    CSR &c = out[f];
    c.R = R;
    c.nnz = (uint64_t)(fstart[f + 1] - fstart[f]);
    c.xptr.alloc(R + 1, false);
    HIPCHK(hipMemcpyAsync(c.xptr.p, fptr.p + (uint64_t)f * (R + 1), (R + 1) * sizeof(int64_t),
                          hipMemcpyDeviceToDevice, s_));
    c.xidx.alloc(c.nnz, false);
    c.xval.alloc(c.nnz, false);
    if (c.nnz) {
      HIPCHK(hipMemcpyAsync(c.xidx.p, oidx.p + fstart[f], c.nnz * sizeof(uint32_t), hipMemcpyDeviceToDevice, s_));
      HIPCHK(hipMemcpyAsync(c.xval.p, oval.p + fstart[f], c.nnz * sizeof(double), hipMemcpyDeviceToDevice, s_));
    }
  }
  sync();
  return out;
}

void Builder::csc(const CSR &x, uint64_t D, int nsg, const uint8_t *own, CSC &out) {
  const uint64_t n = x.nnz;
  uint32_t *rid = grow(t_rid_, n), *keys = grow(t_keys_, n), *perm = grow(t_perm_, n);
  rowid(x.xptr.p, x.R, rid);
  sort_positions(x.xidx.p, keys, perm, n, D ? D - 1 : 0);
  out.crow.alloc(n, false);
  double *cval = grow(t_cval_, n);
  int64_t *cptr = grow(t_cptr_, D + 1);
  out.cval = cval;
  out.cptr = cptr;
  if (n) hipLaunchKernelGGL(k_csc_fill, grid(n), TB, 0, s_, n, perm, rid, x.xval.p, out.crow.p, cval);
  bounds(keys, n, D, cptr);
  // jobs
  int64_t *lc = grow(t_i64_[0], D), *hc = grow(t_i64_[1], D), *sc = grow(t_i64_[2], D);
  int64_t *L = grow(t_i64_[3], D), *H = grow(t_i64_[4], D), *S = grow(t_i64_[5], D);
  if (D) hipLaunchKernelGGL(k_job_count, grid(D), TB, 0, s_, D, cptr, own, nsg, lc, hc, sc);
  incl_scan(lc, L, D);
  incl_scan(hc, H, D);
  incl_scan(sc, S, D);
  int64_t tot[3] = {0, 0, 0};
  if (D) {
    HIPCHK(hipMemcpyAsync(&tot[0], L + D - 1, sizeof(int64_t), hipMemcpyDeviceToHost, s_));
    HIPCHK(hipMemcpyAsync(&tot[1], H + D - 1, sizeof(int64_t), hipMemcpyDeviceToHost, s_));
    HIPCHK(hipMemcpyAsync(&tot[2], S + D - 1, sizeof(int64_t), hipMemcpyDeviceToHost, s_));
    sync();
  }
  const uint64_t nlight = (uint64_t)tot[0], nheavy = (uint64_t)tot[1];
  out.nslot = (uint64_t)tot[2];
  const uint64_t pad = (nlight + nsg - 1) / nsg * nsg;
  out.njobs = pad + nheavy;
  out.jobs.alloc(out.njobs, false);
  if (D) hipLaunchKernelGGL(k_job_write, grid(D), TB, 0, s_, D, cptr, own, nsg, L, H, S, pad, out.jobs.p);
  if (pad > nlight) hipLaunchKernelGGL(k_job_pad, grid(pad - nlight), TB, 0, s_, nlight, pad, out.jobs.p);
}

void Builder::flags(const CSR &x, const CSC &c, uint64_t D, bool &one, bool &idlike) {
  unsigned long long *bad = (unsigned long long *)grow(t_bad_, 2);
  HIPCHK(hipMemsetAsync(bad, 0, 2 * sizeof(int64_t), s_));
  hipLaunchKernelGGL(k_flags, grid(std::max(x.R, D)), TB, 0, s_, x.R, x.xptr.p, D, c.cptr, bad);
  unsigned long long h[2];
  HIPCHK(hipMemcpyAsync(h, bad, sizeof(h), hipMemcpyDeviceToHost, s_));
  sync();
  one = x.R > 0 && x.nnz == x.R && h[0] == 0;
  idlike = one && D == x.R && h[1] == 0;
}

const double *Builder::xsq(const CSC &c, uint64_t D) {
  double *out = grow(t_dbl_, std::max<uint64_t>(D, 1));
  HIPCHK(hipMemsetAsync(out, 0, std::max<uint64_t>(D, 1) * sizeof(double), s_));
  if (D) hipLaunchKernelGGL(k_xsq, (unsigned)std::min<uint64_t>(D, 16384), TB, 0, s_, D, c.cptr, c.cval, out);
  return out;
}

const double *Builder::col_counts(const CSC &c, uint64_t D) {
  double *out = grow(t_dbl_, std::max<uint64_t>(D, 1));
  if (D) hipLaunchKernelGGL(k_col_counts, grid(D), TB, 0, s_, D, c.cptr, out);
  return out;
}

void Builder::segments(const int64_t *yptr, uint64_t R, uint64_t len, DevBuf<Seg> &segs, DevBuf<uint32_t> &segptr,
                       uint64_t &nseg) {
  DevBuf<int64_t> c, S;
  c.alloc(std::max<uint64_t>(R, 1), false);
  S.alloc(std::max<uint64_t>(R, 1), false);
  if (R) hipLaunchKernelGGL(k_seg_count, grid(R), TB, 0, s_, R, yptr, len, c.p);
  incl_scan(c.p, S.p, R);
  nseg = R ? (uint64_t)read1(S.p + R - 1) : 0;
  if (nseg > 0xffffffffull) throw Error(OCFFM_E_DATA, "too many positive segments");
  segs.alloc(nseg, false);
  segptr.alloc(R + 1);
  if (R) hipLaunchKernelGGL(k_seg_write, grid(R), TB, 0, s_, R, yptr, len, S.p, segs.p, segptr.p);
  sync();
}

const CSR &Builder::seg_expand(const int64_t *xptr, const uint32_t *xidx, const double *xval, const Seg *segs,
                               uint64_t nseg) {
  CSR &out = t_ex_;
  int64_t *c = grow(t_cnt_, nseg);
  out.R = nseg;
  int64_t *sptr = grow(out.xptr, nseg + 1);
  HIPCHK(hipMemsetAsync(sptr, 0, sizeof(int64_t), s_));
  if (nseg) hipLaunchKernelGGL(k_seg_nodes, grid(nseg), TB, 0, s_, nseg, segs, xptr, c);
  incl_scan(c, sptr + 1, nseg);
  out.nnz = nseg ? (uint64_t)read1(sptr + nseg) : 0;
  uint32_t *oidx = grow(out.xidx, out.nnz);
  double *oval = grow(out.xval, out.nnz);
  if (nseg && out.nnz)
    hipLaunchKernelGGL(k_seg_copy, grid(nseg), TB, 0, s_, nseg, segs, xptr, xidx, xval, sptr, oidx, oval);
  return out;
}

void Builder::labels(const HostData &U, uint64_t r0, uint64_t r1, DevBuf<int64_t> &yptr, DevBuf<uint32_t> &ycol) {
  const uint64_t R = r1 - r0, pb = U.yptr[r0], pe = U.yptr[r1];
  DevBuf<uint64_t> y, c;
  y.upload(U.yptr.data() + r0, R + 1);
  c.upload(U.ycol.data() + pb, pe - pb);
  yptr.alloc(R + 1, false);
  ycol.alloc(pe - pb, false);
  hipLaunchKernelGGL(k_rebase, grid(R + 1), TB, 0, s_, R + 1, y.p, yptr.p);
  if (pe > pb) hipLaunchKernelGGL(k_narrow, grid(pe - pb), TB, 0, s_, pe - pb, c.p, ycol.p);
  sync();
}

void Builder::transpose(const DevBuf<int64_t> &yptr, const DevBuf<uint32_t> &ycol, uint64_t R, uint64_t n,
                        DevBuf<int64_t> &vptr, DevBuf<uint32_t> &vcol, DevBuf<uint32_t> &v2u, DevBuf<uint32_t> &u2v) {
  const uint64_t np = ycol.n;
  uint32_t *rid = grow(t_rid_, np), *keys = grow(t_keys_, np);
  rowid(yptr.p, R, rid);
  v2u.alloc(np, false);
  vcol.alloc(np, false);
  u2v.alloc(np, false);
  sort_positions(ycol.p, keys, v2u.p, np, n ? n - 1 : 0);
  if (np) hipLaunchKernelGGL(k_trans_fill, grid(np), TB, 0, s_, np, v2u.p, rid, vcol.p, u2v.p);
  vptr.alloc(n + 1, false);
  bounds(keys, np, n, vptr.p);
  sync();
}

void Builder::label_ptr(const HostData &U, uint64_t n, DevBuf<int64_t> &ptr) {
  const uint64_t np = U.ycol.size();
  DevBuf<uint64_t> c;
  c.upload(U.ycol);
  uint32_t *c32 = grow(t_rid_, np), *keys = grow(t_keys_, np);
  if (np) hipLaunchKernelGGL(k_narrow, grid(np), TB, 0, s_, np, c.p, c32);
  if (np) {
    unsigned bits = 1;
    while (bits < 32 && ((n ? n - 1 : 0) >> bits)) bits++;
    size_t bytes = 0;
    HIPCHK(rocprim::radix_sort_keys(nullptr, bytes, c32, keys, (size_t)np, 0u, bits, s_));
    HIPCHK(rocprim::radix_sort_keys(scr_.get(bytes, s_), bytes, c32, keys, (size_t)np, 0u, bits, s_));
  }
  ptr.alloc(n + 1, false);
  bounds(keys, np, n, ptr.p);
  sync();
}

void Builder::popularity(const HostData &U, DevBuf<double> &out) {
  const uint64_t n = U.n;
  DevBuf<int64_t> ptr;
  label_ptr(U, n, ptr);
  out.alloc(n, false);
  // the host sums the counts as doubles in item order: exact integers
  const double total = (double)U.ycol.size();
  if (n) hipLaunchKernelGGL(k_pop, grid(n), TB, 0, s_, n, ptr.p, total, out.p);
  sync();
}

}  // namespace dev
}  // namespace ocffm
