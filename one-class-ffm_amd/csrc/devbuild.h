// devbuild.h — on-device construction of the solver's data layout (SURVEY
// §8f rank 2): the per-field CSR split of ImpData::split_fields
// (ffm.cpp:185-257), the item-major transpose of the labels (transY,
// ffm.cpp:259-294), the item popularity (ffm.cpp:143,172-176), and this
// repo's own derived structures (feature-major CSCs, feature-pass jobs,
// positive segments).  Integer and byte work: histograms, prefix scans,
// stable radix sorts, gathers.  Every array equals the host build's
// (solver.hip: build_csc / build_segments / build_seg_csc / build_item_side)
// bit for bit; OCFFM_HOST_BUILD=1 selects the host build, and
// tests/test_boundary_gpu.py compares the digests of every array.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <vector>

#include "common.hpp"
#include "host_data.h"
#include "kernels.hpp"

namespace ocffm {
namespace dev {

// Growable device scratch for rocPRIM temporary storage and the build's
// intermediates (released with the builder).
struct Scratch {
  DevBuf<char> tmp;
  // (a larger buffer replaces the old one only once the stream has drained)
  void *get(size_t bytes, hipStream_t s) {
    if (bytes > tmp.n) {
      HIPCHK(hipStreamSynchronize(s));
      tmp.alloc(bytes + (bytes >> 3) + 256, false);
    }
    return tmp.p;
  }
};

// One field's rows [0, R) as CSR on the device (values still fp64).
struct CSR {
  uint64_t R = 0, nnz = 0;
  DevBuf<int64_t> xptr;  // R + 1
  DevBuf<uint32_t> xidx;
  DevBuf<double> xval;
};

// Feature-major view of a CSR and its feature-pass jobs (solver.hip
// build_csc): rows increasing inside a column, light columns' jobs first
// (padded to a multiple of nsg), then the wave-chunks of heavy columns.
// crow / jobs are the caller's; cval / cptr live in the builder's scratch
// (valid until its next csc call).
struct CSC {
  DevBuf<uint32_t> crow;
  const double *cval = nullptr;
  const int64_t *cptr = nullptr;  // D + 1
  DevBuf<Job> jobs;
  uint64_t njobs = 0, nslot = 0;
};

class Builder {
 public:
  explicit Builder(hipStream_t s) : s_(s) {}

  // split_fields of rows [r0, r1) of d into nf fields (fields >= d.f or
  // absent rows: empty).  Ds: the per-field column counts (checked).
  std::vector<CSR> split(const HostData &d, uint64_t r0, uint64_t r1, uint32_t nf);

  // CSC + jobs of one CSR over D columns; own (device, D bytes) or null:
  // columns with own[d] == 0 get no job (owned fields).
  void csc(const CSR &x, uint64_t D, int nsg, const uint8_t *own, CSC &out);

  // one: every row has exactly one node; idlike: additionally D == R and
  // every column holds exactly one row (solver.hip DevField).
  void flags(const CSR &x, const CSC &c, uint64_t D, bool &one, bool &idlike);

  // One node per row: per-column sum of x^2 in the order of xsq_col (fp64,
  // no FMA); max(D, 1) values in the builder's scratch.
  const double *xsq(const CSC &c, uint64_t D);

  // Per-column entry counts as fp64 (the --freq weights of a one-rank run),
  // in the builder's scratch.
  const double *col_counts(const CSC &c, uint64_t D);

  // Positive segments of at most len positives per row (rows without
  // positives get one empty segment); yptr: R + 1 local offsets (device).
  void segments(const int64_t *yptr, uint64_t R, uint64_t len, DevBuf<Seg> &segs, DevBuf<uint32_t> &segptr,
                uint64_t &nseg);

  // The CSR over segments: each segment repeats its row's nodes.  The
  // result lives in the builder's scratch (valid until the next call).
  const CSR &seg_expand(const int64_t *xptr, const uint32_t *xidx, const double *xval, const Seg *segs,
                        uint64_t nseg);

  // Labels of rows [r0, r1) as local user-major arrays (yptr rebased,
  // ycol narrowed to 32 bits).
  void labels(const HostData &U, uint64_t r0, uint64_t r1, DevBuf<int64_t> &yptr, DevBuf<uint32_t> &ycol);

  // transY restricted to the local users: item-major positives of n items
  // (vptr n + 1, vcol = local user of each), v2u / u2v the position maps.
  void transpose(const DevBuf<int64_t> &yptr, const DevBuf<uint32_t> &ycol, uint64_t R, uint64_t n,
                 DevBuf<int64_t> &vptr, DevBuf<uint32_t> &vcol, DevBuf<uint32_t> &v2u, DevBuf<uint32_t> &u2v);

  // Per-item label counts over all rows of U as a CSR pointer (n + 1).
  void label_ptr(const HostData &U, uint64_t n, DevBuf<int64_t> &ptr);

  // Normalised label counts over all rows of U (ffm.cpp:143,172-176), U.n items.
  void popularity(const HostData &U, DevBuf<double> &out);

  void sync() { HIPCHK(hipStreamSynchronize(s_)); }

  // stable sort of (key, position) pairs: vout[q] = input position of the
  // q-th smallest key (ties in input order)
  void sort_positions(const uint32_t *kin, uint32_t *kout, uint32_t *vout, uint64_t n, uint64_t maxkey);
  // out[p] = the row of position p of a CSR pointer (R + 1)
  void rowid(const int64_t *ptr, uint64_t R, uint32_t *out);
  // CSR pointer (D + 1) of sorted keys
  void bounds(const uint32_t *sorted, uint64_t n, uint64_t D, int64_t *ptr);

 private:
  void incl_scan(const int64_t *in, int64_t *out, uint64_t n);
  // scratch buffers reused across calls (grown, never shrunk; a larger one
  // replaces the old only once the stream has drained)
  template <class T> T *grow(DevBuf<T> &b, uint64_t n) {
    if (b.n < std::max<uint64_t>(n, 1)) {
      sync();
      b.alloc(std::max<uint64_t>(n, 1) + (n >> 3), false);
    }
    return b.p;
  }
  DevBuf<uint32_t> t_rid_, t_keys_, t_perm_;
  DevBuf<int64_t> t_cnt_, t_tile_, t_cptr_, t_bad_, t_i64_[6];
  DevBuf<double> t_cval_, t_dbl_;
  CSR t_ex_;
  template <class T> T read1(const T *p) {
    T v;
    HIPCHK(hipMemcpyAsync(&v, p, sizeof(T), hipMemcpyDeviceToHost, s_));
    sync();
    return v;
  }
  hipStream_t s_;
  Scratch scr_;
};

// init_mat (ffm.cpp:71-78) on the device: table (rows x cols doubles in
// row-major draw order) into out (row stride kp, padding untouched), the
// values init_table draws on the host bit for bit (minstd_rand0 jump-ahead
// per lane; generate_canonical<double, 53> and uniform_real_distribution
// with the two FMA contractions g++ -mfma makes in host_data.cpp).
template <typename real>
void draw_table(hipStream_t s, real *out, uint64_t rows, uint32_t cols, uint32_t kp, const TableDraw &t);

// The column-tau weight of a one-node field, sum of x^2 over a column's
// entries v[0, n) (in row order), in the order k_xsq adds them: 256 strided
// partials p[t] = v[t]^2 + v[t+256]^2 + ..., then p[t] += p[t + o] for
// o = 128, 64, .., 1.  The host build computes it this way too.
inline double xsq_col(const double *v, uint64_t n) {
#pragma clang fp contract(off)
  double p[256];
  for (int t = 0; t < 256; t++) p[t] = 0.0;
  for (uint64_t q = 0; q < n; q++) p[q % 256] = p[q % 256] + v[q] * v[q];
  for (int o = 128; o > 0; o >>= 1)
    for (int t = 0; t < o; t++) p[t] = p[t] + p[t + o];
  return p[0];
}

// Rounds of JOB_ENT entries per subgroup for a heavy column of n entries
// (solver.hip build_csc): R = round(sqrt(n / (8 nsg^2 JOB_ENT))), at least 1,
// in integers so that host and device agree exactly: the largest r >= 1
// with (2r - 1)^2 * 8 nsg^2 JOB_ENT <= 4 n.
__host__ __device__ inline uint64_t heavy_rounds(uint64_t n, int nsg) {
  const uint64_t den = 8ull * (uint64_t)nsg * (uint64_t)nsg * (uint64_t)JOB_ENT;
  uint64_t r = 1;
  while (true) {
    const uint64_t t = 2 * (r + 1) - 1;
    if (t * t * den > 4 * n) break;
    r++;
  }
  return r;
}

}  // namespace dev
}  // namespace ocffm
