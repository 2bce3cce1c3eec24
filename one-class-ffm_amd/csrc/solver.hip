// solver.hip — device-resident block Newton-CG epoch and the C ABI.
//
// Host C++ owns the block schedule and the data layout; every row, feature
// and vector pass is a kernel from kernels.hpp on one HIP stream.  The CG
// loop (ffm.cpp:780) is data-dependent: its scalars live on the device and
// the host only learns the loop exit one iteration late (it enqueues
// iteration it+1 before waiting for iteration it's verdict; kernels of an
// iteration that must not run return at entry), so the GPU never idles on a
// host round trip.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <charconv>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iomanip>
#include <iostream>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <thread>
#include <tuple>
#include <unordered_map>
#include <type_traits>
#include <vector>

#include "../../include/ocffm.h"
#include "common.hpp"
#include "devbuild.h"
#include "host_data.h"
#include "kernels.hpp"

namespace ocffm {

thread_local std::string g_last_error;

static uint32_t block_index(uint32_t f1, uint32_t f2, uint32_t f) { return f2 + (f - 1) * f1 - f1 * (f1 - 1) / 2; }

static uint32_t pad_k(uint32_t k) {
  uint32_t kp = 4;
  while (kp < k) kp <<= 1;
  return kp;
}

// OCFFM_EXP_KP32 (experiment builds only, tools/build_variant.sh): fp32 at
// KP = 32 instantiated alone, so a kernel experiment compiles in a fraction
// of the full build's time.
template <class F> static void with_kp(uint32_t kp, F &&f) {
#ifdef OCFFM_EXP_KP32
  if (kp != 32) throw Error(OCFFM_E_ARG, "experiment build: k must pad to 32");
  f(std::integral_constant<int, 32>());
  return;
#endif
  switch (kp) {
    case 4: f(std::integral_constant<int, 4>()); break;
    case 8: f(std::integral_constant<int, 8>()); break;
    case 16: f(std::integral_constant<int, 16>()); break;
    case 32: f(std::integral_constant<int, 32>()); break;
    case 64: f(std::integral_constant<int, 64>()); break;
    case 128: f(std::integral_constant<int, 128>()); break;
    default: throw Error(OCFFM_E_ARG, "k must be in 1..128");
  }
}

static unsigned grid_for(uint64_t items, uint64_t per_block, unsigned cap = 4096) {
  uint64_t g = (items + per_block - 1) / per_block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (unsigned)g;
}

template <typename real> __global__ void k_to_real(uint64_t n, const double *__restrict__ in, real *__restrict__ out) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    out[i] = (real)in[i];
}

// -------------------------------------------------------------- profiling
struct KStat {
  uint64_t launches = 0;
  double ms = 0, bytes = 0, flops = 0;
};

// ------------------------------------------------------------------- data
// Item-owned CG steps of an item-id field's cross halves on several ranks
// (OCFFM_ITEM_OWNED): rank q owns the items [j0, j1) (equal
// chunks of `chunk` items) and holds ALL positives of its items (every
// rank's users), as positive segments whose partner rows index the
// all-gathered user table (Pg: rank r's users at rows [r cu, r cu + R_r)).
// Its CG steps then gather, finalise its own columns and sum only the three
// dot products, instead of all-reducing the D x k partials every step.
template <typename real> struct ItemOwned {
  uint64_t j0 = 0, j1 = 0, chunk = 0, nseg = 0;
  DevBuf<Seg> segs;
  DevBuf<uint32_t> segptr;
  DevBuf<uint32_t> ycol;  // Pg row of each positive
  DevBuf<uint32_t> segd;  // the segment's column (the item)
  DevBuf<real> segx;
  DevBuf<uint32_t> scrow;  // segment CSC over the owned columns
  DevBuf<real> scval;
  DevBuf<Job> sjobs;
  uint64_t snjw = 0, snslot = 0;
  DevBuf<double> shdots;
};

template <typename real> struct DevField {
  uint64_t D = 0, nnz = 0;
  DevBuf<int64_t> xptr;
  DevBuf<uint32_t> xidx;
  DevBuf<real> xval;
  DevBuf<uint32_t> crow;
  DevBuf<real> cval;
  DevBuf<Job> jobs;  // kernels.hpp: Job; njw waves of NSG jobs
  uint64_t njw = 0, nslot = 0;
  DevBuf<double> hdots, shdots;  // heavy columns' dot-product slots (row / segment CSC; kernels.hpp Fin::hdots)
  DevBuf<real> freqw;  // global feature frequency (for --freq)
  DevBuf<real> xsq;    // one node per row: sum of x^2 over each column's rows (column tau)
  // the same CSC over positive segments (kernels.hpp: Seg) of the side
  DevBuf<uint32_t> scrow;
  DevBuf<real> scval;
  DevBuf<Job> sjobs;
  uint64_t snjw = 0, snslot = 0;
  DevBuf<unsigned> cnt;  // per-column arrival tickets (zero at rest)
  bool idlike = false;   // one node per row and each feature in exactly one row (CSC = identity)
  bool one = false;      // exactly one node per row (xptr[i] == i)
  // Per-column Grams (kernels.hpp k_col_gram / k_hv_cgram) of a one-node-per-row
  // field with few columns: chunk jobs over the CSC and the D x k x k Grams.
  // Allocated on the first Gram half (col_grams); gpart holds the ordered
  // partial slots of multi-chunk columns (gslots of them).
  DevBuf<Job> gchunks;
  DevBuf<Job> gsums;  // MFMA build (k_col_gram32): multi-chunk columns {col, nparts, first slot}
  DevBuf<real> gram, gpart;
  uint64_t gslots = 0;
  // Owned field (several ranks): every feature is touched by the
  // rows of at most one rank.  Its CG vectors are then not all-reduced: each
  // rank finalises only the columns it owns (untouched ones go to rank 0) and
  // only the dot products are summed over the ranks.
  bool excl = false;
  std::vector<uint8_t> h_own;
  DevBuf<uint8_t> own;
  // Per-column cross Grams (one node per row, few columns): the
  // positions of the field's rows' positives in column order (partner row,
  // (1 - w) x^2 of the position's row) and their Gram build chunks.
  bool ccg_ready = false;
  DevBuf<uint32_t> cpos;
  DevBuf<real> cw;
  DevBuf<Job> cchunks, csums;
  uint64_t cslots = 0, cnpos = 0;
  DevBuf<uint32_t> segd;  // one: the node of each positive segment's row (no row indirection)
  DevBuf<real> segx;
  std::unique_ptr<ItemOwned<real>> io;  // item-owned CG steps (item-id field, several ranks)
  // Pair Grams (kernels.hpp k_pg_step; several nodes per row, few
  // features): pairs p = (pa, pb), pa <= pb, of features met in one row;
  // their entries (row, X_ia X_ib) pair-major with Gram build chunks; each
  // feature's adjacency (its pairs and the other feature of each).
  bool pg = false;
  uint64_t npair = 0;
  DevBuf<uint32_t> ppa, ppb, pgrow;
  DevBuf<real> pgval, pgram, pgpart;
  DevBuf<Job> pgchunks, pgsums;
  uint64_t pgslots = 0;
  DevBuf<unsigned> pgcnt;
  DevBuf<int64_t> paptr;  // per feature a: its pairs (pair, other feature) in papair / paoth
  DevBuf<uint32_t> papair, paoth;
  uint32_t pqb = 1;  // k_pg_step blocks per feature
  // column pointers of the row / segment CSC for the column-block feature
  // pass (k_feat_col; derived from the jobs on first use)
  DevBuf<int64_t> fcptr[2];
  int fcol[2] = {-1, -1};  // -1 not decided, 0 no, 1 yes
  // host copies kept until the segment CSC is built
  std::vector<int64_t> h_xptr;
  std::vector<uint32_t> h_xidx;
  std::vector<double> h_xval;
};

template <typename real> struct DevSide {
  uint64_t R = 0;       // local rows
  uint64_t R_glob = 0;  // global rows
  uint64_t row0 = 0;
  std::vector<std::unique_ptr<DevField<real>>> F;
  std::vector<uint64_t> Ds;
  uint64_t npos = 0;
  DevBuf<int64_t> yptr;
  DevBuf<uint32_t> ycol;
  DevBuf<real> yt;
  DevBuf<uint32_t> perm;  // position of the same positive in the other orientation
  DevBuf<real> bias;      // a (users) or b (items)
  DevBuf<real> s;         // sa or sb
  uint64_t nseg = 0;      // positive segments (kernels.hpp: Seg)
  DevBuf<Seg> segs;
  DevBuf<uint32_t> sord;  // the cross row passes' processing order of the segments (longest first)
  bool short_segs = false;  // >= 99 % of the segments hold <= 16 positives (k_hs_cross_seg's 16-position pass)
  DevBuf<uint32_t> segptr;
  // Hot rows (kernels.hpp k_hot_gram*): rows with >= hot_min positives whose
  // cross-half Hessian-vector rows read a k x k Gram of their partner rows
  // (built once per cross half) instead of gathering them every CG step.
  uint64_t nhot = 0, hslots = 0, hpos = 0;  // rows, partial slots, their positives
  DevBuf<uint32_t> hot_seg;                  // per segment: the row's Gram slot or HOT_NONE
  DevBuf<uint32_t> hot_row;                  // per row: its Gram slot or HOT_NONE
  bool xf_ok = false;                        // every row under the hot threshold, or the hot rows' Grams set up
  DevBuf<Job> hchunks, hsums;
};

// Split every row's positives into segments of at most `len` (rows without
// positives still get one, empty, segment for their row-local terms).
template <typename real> static void build_seg_csc(DevSide<real> &s, const std::vector<uint32_t> &segptr, int nsg) {
  for (auto &Fp : s.F) {
    DevField<real> &F = *Fp;
    const uint64_t R = F.h_xptr.size() - 1;
    // expand each row's nodes over its segments, then reuse the row builder
    std::vector<int64_t> xptr(segptr[R] + 1, 0);
    std::vector<uint32_t> xidx;
    std::vector<double> xval;
    uint64_t sidx = 0;
    for (uint64_t i = 0; i < R; i++)
      for (uint32_t sg = segptr[i]; sg < segptr[i + 1]; sg++, sidx++) {
        for (int64_t p = F.h_xptr[i]; p < F.h_xptr[i + 1]; p++) {
          xidx.push_back(F.h_xidx[p]);
          xval.push_back(F.h_xval[p]);
        }
        xptr[sidx + 1] = (int64_t)xidx.size();
      }
    std::vector<uint32_t> crow;
    std::vector<double> cval;
    if (F.one) {  // xidx/xval now hold one node per segment
      F.segd.upload(xidx);
      std::vector<real> sx(xval.begin(), xval.end());
      F.segx.upload(sx);
    }
    std::vector<Job> jobs;
    build_csc(sidx, F.D, xptr.data(), xidx.data(), xval.data(), nsg, crow, cval, jobs, F.snslot,
              F.excl ? F.h_own.data() : nullptr);
    F.scrow.upload(crow);
    std::vector<real> cv(cval.begin(), cval.end());
    F.scval.upload(cv);
    F.sjobs.upload(jobs);
    F.snjw = jobs.size() / nsg;
    F.shdots.alloc(std::max<uint64_t>(F.snslot, 1) * 3);
    F.h_xptr.clear();
    F.h_xptr.shrink_to_fit();
    F.h_xidx.clear();
    F.h_xidx.shrink_to_fit();
    F.h_xval.clear();
    F.h_xval.shrink_to_fit();
  }
}

template <typename real>
static void build_segments(DevSide<real> &s, const std::vector<int64_t> &yptr, uint64_t len, int nsg) {
  const uint64_t R = yptr.size() - 1;
  std::vector<Seg> segs;
  std::vector<uint32_t> segptr(R + 1, 0);
  segs.reserve(R + (uint64_t)yptr[R] / len + 1);
  for (uint64_t i = 0; i < R; i++) {
    segptr[i] = (uint32_t)segs.size();
    const int64_t b = yptr[i], e = yptr[i + 1];
    const uint32_t nrow = (uint32_t)std::max<int64_t>(1, (e - b + (int64_t)len - 1) / (int64_t)len);
    int64_t p = b;
    do {
      const int64_t q = std::min<int64_t>(e, p + (int64_t)len);
      segs.push_back(Seg{(uint32_t)i, (nrow << 1) | (p == b ? 1u : 0u), p, q});
      p = q;
    } while (p < e);
  }
  segptr[R] = (uint32_t)segs.size();
  s.nseg = segs.size();
  s.segs.upload(segs);
  s.segptr.upload(segptr);
  build_seg_csc(s, segptr, nsg);
}

struct Block {
  bool used = false;
  uint32_t f1 = 0, f2 = 0;
};

// Feature-major (CSC) view of one field's CSR and its feature-pass jobs
// (kernels.hpp: Job): light columns first, packed NSG to a wave, then the
// wave-chunks of the heavy columns.  Empty columns get a job too (their
// finalisation is lam W alone).  own (owned fields): columns of other ranks
// get no job.
static void build_csc(uint64_t R, uint64_t D, const int64_t *xptr, const uint32_t *xidx, const double *xval, int nsg,
                      std::vector<uint32_t> &crow, std::vector<double> &cval, std::vector<Job> &jobs,
                      uint64_t &nslot, const uint8_t *own) {
  const uint64_t nnz = (uint64_t)xptr[R] - (uint64_t)xptr[0];
  std::vector<uint64_t> cptr(D + 1, 0);
  for (int64_t p = xptr[0]; p < xptr[R]; p++) cptr[xidx[p] + 1]++;
  for (uint64_t d = 0; d < D; d++) cptr[d + 1] += cptr[d];
  crow.assign(nnz, 0);
  cval.assign(nnz, 0);
  std::vector<uint64_t> cur(cptr.begin(), cptr.end() - 1);
  for (uint64_t i = 0; i < R; i++)
    for (int64_t p = xptr[i]; p < xptr[i + 1]; p++) {
      const uint64_t q = cur[xidx[p]]++;
      crow[q] = (uint32_t)i;
      cval[q] = xval[p];
    }
  jobs.clear();
  for (uint64_t d = 0; d < D; d++)
    if (cptr[d + 1] - cptr[d] <= (uint64_t)JOB_ENT && (!own || own[d]))
      jobs.push_back(Job{(uint32_t)d, 1u, 0u, 0u, (int64_t)cptr[d], (int64_t)cptr[d + 1]});
  while (jobs.size() % nsg) jobs.push_back(Job{JOB_NONE, 1u, 0u, 0u, 0, 0});
  nslot = 0;
  for (uint64_t d = 0; d < D; d++) {
    const uint64_t b = cptr[d], e = cptr[d + 1];
    if (e - b <= (uint64_t)JOB_ENT || (own && !own[d])) continue;
    // A heavy column of n entries: np wave-chunks, each subgroup walking R
    // rounds of JOB_ENT entries, then the last chunk to arrive sums the np
    // slots 8 per subgroup per round (kernels.hpp k_feat).  Both are chains
    // of dependent load rounds, ~R and ~np / (8 nsg) long: with n = np R nsg
    // JOB_ENT their sum is least at R = sqrt(K / (8 nsg)), K = n / (nsg
    // JOB_ENT).  (A 400,000-row column: 632 chunks of 20 rounds instead of
    // 12,500 one-round chunks summed 4 at a time.)
    // (R = round(sqrt(K / (8 nsg))) in integers: devbuild.h heavy_rounds)
    const uint64_t R = dev::heavy_rounds(e - b, nsg);
    const uint64_t sub = (uint64_t)JOB_ENT * R, wc = (uint64_t)nsg * sub;
    const uint32_t np = (uint32_t)((e - b + wc - 1) / wc);
    for (uint32_t q = 0; q < np; q++)
      for (int g = 0; g < nsg; g++) {
        const int64_t sb = (int64_t)std::min(e, b + q * wc + (uint64_t)g * sub);
        const int64_t se = (int64_t)std::min<uint64_t>(e, (uint64_t)sb + sub);
        jobs.push_back(Job{(uint32_t)d, np, (uint32_t)(nslot + q), 1u | (q << 1), sb, se});
      }
    nslot += np;
  }
}

// ---------------------------------------------------------------- problem
struct ProblemBase {
  virtual ~ProblemBase() = default;
  virtual void init() = 0;
  virtual void one_epoch() = 0;
  virtual void solve_block(uint32_t f1, uint32_t f2) = 0;
  virtual void cache_sasb() = 0;
  virtual void validate(ocffm_metrics *m, bool forced = false, double *per_row_ndcg = nullptr, uint64_t cap = 0) = 0;
  virtual uint64_t test_rows() const = 0;
  virtual uint64_t get(char what, uint32_t b12, double *out, uint64_t cap) = 0;
  virtual void set(char what, uint32_t b12, const double *in, uint64_t len) = 0;
  virtual void grad(uint32_t f1, uint32_t f2, int half, double *out) = 0;
  virtual void hv(uint32_t f1, uint32_t f2, int half, const double *v, double *out) = 0;
  virtual void save_model(const std::string &path) = 0;
  virtual void save_binary(const std::string &path) = 0;
  virtual void load_binary(const std::string &path) = 0;
  virtual void sync() = 0;
  virtual std::vector<std::pair<std::string, uint64_t>> layout_digest() = 0;
  virtual bool has_test() const = 0;
  virtual uint32_t nr_pass() const = 0;
  virtual int rank() const = 0;
  std::vector<int32_t> cg_log;
  std::map<std::string, KStat> kstats;
  bool profiling = false;
  std::string prof_filter;
  double alg_bytes = 0;
  std::map<std::string, int64_t> counters;  // diagnostics (ocffm_problem_counter)
};

struct Comm {
  int rank = 0, nranks = 1;
  ncclComm_t nccl = nullptr;
  ocffm_allreduce_fn host_fn = nullptr;
  void *host_user = nullptr;
  bool active() const { return nranks > 1 || host_fn != nullptr || nccl != nullptr; }
};

template <typename real> class Problem final : public ProblemBase {
 public:
  Problem(const HostData &U, const HostData *Ut, const HostData &V, const ocffm_param &prm, Comm comm)
      : prm_(prm), comm_(comm), has_test_(Ut != nullptr) {
    HIPCHK(hipSetDevice(prm.device));
    HIPCHK(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
    k_ = prm.k;
    kp_ = pad_k(k_);
    if (k_ == 0 || k_ > 128) throw Error(OCFFM_E_ARG, "k must be in 1..128");
    w_ = prm.omega;
    lam_ = prm.lambda;
    r_ = prm.r;
    fu_ = (uint32_t)U.f;
    fv_ = (uint32_t)V.f;
    f_ = fu_ + fv_;
    if (!V.transposed) throw Error(OCFFM_E_STATE, "item data must go through ocffm_data_trans_y");
    for (uint64_t j : U.ycol)
      if (j >= V.m) throw Error(OCFFM_E_DATA, "train label >= number of item rows (reference: out-of-bounds read)");
    m_glob_ = U.m;
    n_ = V.m;
    if (const char *e = std::getenv("OCFFM_SEG_LEN")) seg_len_ = std::max<uint64_t>(1, std::strtoull(e, nullptr, 10));
    if (const char *e = std::getenv("OCFFM_LOOKAHEAD")) lookahead_ = std::max(1, std::atoi(e));
    if (const char *e = std::getenv("OCFFM_HS_BLOCKS")) hs_blocks_ = (unsigned)std::max(1, std::atoi(e));
    if (const char *e = std::getenv("OCFFM_FEAT_BLOCKS")) feat_blocks_ = (unsigned)std::max(1, std::atoi(e));
    if (const char *e = std::getenv("OCFFM_FUSE")) fuse_ = std::atoi(e) != 0;  // id-field side Hv rows finalise their column
    if (const char *e = std::getenv("OCFFM_NO_OWNED")) no_owned_ = std::atoi(e) != 0;  // all-reduce every field
    // shard users contiguously
    u0_ = U.m * (uint64_t)comm_.rank / (uint64_t)comm_.nranks;
    u1_ = U.m * (uint64_t)(comm_.rank + 1) / (uint64_t)comm_.nranks;
    tmark(nullptr);
    {
      // the data layout: built on the device (devbuild.h), or on the host
      // with OCFFM_HOST_BUILD=1 (the checker: identical arrays)
      dev::Builder B(stream_);
      build_user_side(U, B);
      tmark("create: user side");
      build_item_side(V, U, B);
      tmark("create: item side");
      if (Ut) build_test(*Ut, U, B);
      tmark("create: test rows");
      if (host_build_) popular_.upload(split_host(U).popular);
      else B.popularity(U, popular_);
      npop_ = U.has_label ? U.n : 0;
      B.sync();
    }
    blocks_.resize(f_ * (f_ + 1) / 2);
    W_.resize(blocks_.size());
    H_.resize(blocks_.size());
    P_.resize(blocks_.size());
    Q_.resize(blocks_.size());
    for (uint32_t f1 = 0; f1 < f_; f1++)
      for (uint32_t f2 = f1; f2 < f_; f2++) {
        Block &b = blocks_[block_index(f1, f2, f_)];
        b.f1 = f1;
        b.f2 = f2;
        b.used = prm_.self_side || (f1 < fu_ && f2 >= fu_);
      }
    // scratch
    uint64_t Dmax = 1, Rmax = std::max<uint64_t>(U_.R, V_.R);
    for (auto d : U_.Ds) Dmax = std::max(Dmax, d);
    for (auto d : V_.Ds) Dmax = std::max(Dmax, d);
    dmax_ = Dmax;
    const size_t dk = Dmax * kp_;
    acc_.alloc(dk);
    G_.alloc(dk);
    S_.alloc(dk);
    Vd_.alloc(dk);
    Rv_.alloc(dk);
    Hv_.alloc(dk);
    // h: row or segment partials
    const uint64_t nsegmax = std::max(U_.nseg, V_.nseg);
    h_.alloc(std::max<uint64_t>(std::max(Rmax, nsegmax), 1) * kp_);
    if (std::max(U_.R, V_.R) * kp_ * sizeof(real) >= (1ull << 32) - 64)  // partner-row gathers (BufView)
      throw Error(OCFFM_E_DATA, "too many rows per GPU for 32-bit gather offsets; shard over more GPUs");
    if (std::max(U_.npos, V_.npos) * 4 >= (1ull << 32) - 64)  // column reads through a BufView (k_hs_cross_w)
      throw Error(OCFFM_E_DATA, "too many positives per GPU for 32-bit offsets; shard over more GPUs");
    if (h_.bytes() >= (1ull << 32) - 64)  // kernels.hpp: BufView gathers use 32-bit offsets
      throw Error(OCFFM_E_DATA, "too many rows/segments per GPU for one partial buffer; shard over more GPUs");
    uint64_t nslot = 1;
    for (DevSide<real> *sd : {&U_, &V_})
      for (auto &F : sd->F) nslot = std::max(nslot, std::max(F->nslot, F->snslot));
    wpart_.alloc(nslot * kp_);
    tick_.alloc(TICK_WORDS);
    C_ = fu_ * fv_;
    M_.alloc(std::max<uint32_t>(C_, 1) * kp_ * kp_);
    sums_.alloc(2 * kp_ + 1);
    vecs_.alloc((size_t)std::max<uint32_t>(C_, 1) * kp_);
    part_.alloc(1 << 22, false);
    st_.alloc(1);
    tabs_.alloc(4 * std::max<uint32_t>(C_, 1) + 4);
    // (MAXCG + 2 verdict words, then the persistent CG's error word at MAXCG + 3)
    HIPCHK(hipHostMalloc((void **)&run_host_, sizeof(int) * (MAXCG + 4), hipHostMallocMapped | hipHostMallocCoherent));
    run_host_[MAXCG + 3] = 0;
    {
      int dev = 0, ncu = 0;
      HIPCHK(hipGetDevice(&dev));
      HIPCHK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
      ncu_ = (unsigned)std::max(1, ncu);
    }
    cgp_gen_buf_.alloc(1);
    cgp_abort_.alloc(1);
    {
      int dev = 0, coop = 0;
      HIPCHK(hipGetDevice(&dev));
      if (hipDeviceGetAttribute(&coop, hipDeviceAttributeCooperativeLaunch, dev) != hipSuccess) coop = 0;
      cgp_coop_ = cgp_coop_ && coop != 0;
    }
    std::memset(run_host_, 0, sizeof(int) * (MAXCG + 2));
    HIPCHK(hipHostGetDevicePointer((void **)&run_host_dev_, run_host_, 0));
    if (comm_.host_fn) HIPCHK(hipHostMalloc((void **)&stage_, Dmax * kp_ * sizeof(real), hipHostMallocDefault));
    if (comm_.host_fn) HIPCHK(hipHostMalloc((void **)&dstage_, DSTAGE * sizeof(double), hipHostMallocDefault));
    dots_.alloc(4);
    bsum_.alloc(2);
    ysum_.alloc(std::max<uint64_t>(std::max(U_.nseg, V_.nseg), 1));
    yrow_.alloc(std::max<uint64_t>(std::max(U_.R, V_.R), 1));
    // hot rows (opt-in, DESIGN §7: measured no gain at kkbox shape and a
    // loss at config 5): >= OCFFM_HOT positives, in halves whose last CG
    // count was >= OCFFM_HOT_STEPS (default 0 with OCFFM_HOT set)
    if (const char *e = std::getenv("OCFFM_HOT")) {
      hot_min_ = std::strtoull(e, nullptr, 10);
      hot_steps_ = 0;
      hot_env_ = hot_min_ > 0;
    }
    if (const char *e = std::getenv("OCFFM_HOT_STEPS")) hot_steps_ = std::atoi(e);
    // the fused cross steps of id-like fields (k_hv_cross_id) read the Grams
    // of rows with >= OCFFM_XF_HOT positives (default: more than one gather
    // pass, 33) instead of gathering them
    if (!hot_env_ && xfuse_on_ && !comm_.active()) {
      const char *e = std::getenv("OCFFM_XF_HOT");
      hot_min_ = e ? std::max<uint64_t>(1, std::strtoull(e, nullptr, 10)) : 33;
    }
    if (C_ > 0 && hot_min_ > 0) {
      hot_setup(U_);
      hot_setup(V_);
      const uint64_t nh = std::max(U_.nhot, V_.nhot), ns = std::max(U_.hslots, V_.hslots);
      if (nh) hotG_.alloc(nh * kp_ * kp_, false);
      if (ns) hotP_.alloc(ns * kp_ * kp_, false);
    }
    // per-column cross Grams: every eligible field's positions in column
    // order, set up here (device sort) rather than inside an epoch
    // (on several ranks: where every rank's shard qualifies, ccg_field_all)
    for (DevSide<real> *sd : {&U_, &V_})
      for (uint32_t fi = 0; fi < sd->F.size(); fi++)
        if (ccg_field_all(*sd->F[fi], *sd, sd == &U_, fi, U)) ccg_setup(*sd->F[fi], *sd);
    if (io_mode_ != 0 && comm_.active() && (comm_.nranks > 1 || io_mode_ == 2) && C_ > 0) io_setup(U, V);
    build_sorder(U_);
    build_sorder(V_);
    seg_shape(U_);
    seg_shape(V_);
    // pair Grams of the side halves of low-cardinality multi-node fields
    // (one GPU: every rank would otherwise have to agree on its local shard's
    // pair count, and the multi-rank path has its own partial-sum protocol)
    if (pgram_mode_ != 0 && !comm_.active() && prm_.self_side)
      for (DevSide<real> *sd : {&U_, &V_})
        for (uint32_t fi = 0; fi < sd->F.size(); fi++) pgram_setup(*sd->F[fi], *sd);
    // T pre-pass rows: the larger side that takes the pre-pass (tpre() also
    // bounds R for 32-bit buffer offsets, so test each side on its own)
    uint64_t tR = 0;
    for (const DevSide<real> *sd : {&U_, &V_})
      if (tpre(sd->R, sd->npos)) tR = std::max(tR, sd->R);
    if (tR) Tpre_.alloc(tR * kp_);
  }

  ~Problem() override {
    if (run_host_) (void)hipHostFree(run_host_);
    if (stage_) (void)hipHostFree(stage_);
    if (dstage_) (void)hipHostFree(dstage_);
    for (auto &e : ev_pool_) (void)hipEventDestroy(e);
    if (side_) (void)hipStreamSynchronize(side_);
    if (side_ev_[0]) (void)hipEventDestroy(side_ev_[0]);
    if (side_ev_[1]) (void)hipEventDestroy(side_ev_[1]);
    if (side_) (void)hipStreamDestroy(side_);
    if (stream_) (void)hipStreamDestroy(stream_);
    if (comm_.nccl) ncclCommDestroy(comm_.nccl);
  }

  bool has_test() const override { return has_test_; }
  uint64_t test_rows() const override { return has_test_ ? T_.R : 0; }
  uint32_t nr_pass() const override { return prm_.nr_pass; }
  int rank() const override { return comm_.rank; }
  void sync() override {
    side_join();
    HIPCHK(hipStreamSynchronize(stream_));
  }

  // FNV-1a digests of every array of the data layout (and its counts), in
  // a fixed order: the device build and the host build must agree on each.
  std::vector<std::pair<std::string, uint64_t>> layout_digest() override {
    sync();
    std::vector<std::pair<std::string, uint64_t>> out;
    auto fnv = [](const void *p, size_t n, uint64_t h) {
      const unsigned char *b = (const unsigned char *)p;
      for (size_t i = 0; i < n; i++) h = (h ^ b[i]) * 0x100000001b3ull;
      return h;
    };
    auto num = [&](const std::string &name, uint64_t v) { out.emplace_back(name, fnv(&v, sizeof(v), 0xcbf29ce484222325ull)); };
    auto buf = [&](const std::string &name, const auto &b) {
      using T = std::remove_pointer_t<decltype(b.p)>;
      std::vector<T> h(b.n);
      if (b.n) HIPCHK(hipMemcpy(h.data(), b.p, b.n * sizeof(T), hipMemcpyDeviceToHost));
      out.emplace_back(name, fnv(h.data(), h.size() * sizeof(T), fnv(&b.n, sizeof(b.n), 0xcbf29ce484222325ull)));
    };
    const char *sn[3] = {"U", "V", "T"};
    DevSide<real> *sd[3] = {&U_, &V_, &T_};
    for (int q = 0; q < 3; q++) {
      DevSide<real> &s = *sd[q];
      const std::string p = sn[q];
      num(p + ".R", s.R);
      num(p + ".npos", s.npos);
      num(p + ".nseg", s.nseg);
      buf(p + ".yptr", s.yptr);
      buf(p + ".ycol", s.ycol);
      buf(p + ".perm", s.perm);
      buf(p + ".segs", s.segs);
      buf(p + ".segptr", s.segptr);
      for (size_t fi = 0; fi < s.F.size(); fi++) {
        DevField<real> &F = *s.F[fi];
        const std::string f = p + ".F" + std::to_string(fi) + ".";
        num(f + "D", F.D);
        num(f + "nnz", F.nnz);
        num(f + "flags", (F.one ? 1 : 0) | (F.idlike ? 2 : 0) | (F.excl ? 4 : 0));
        num(f + "njw", F.njw);
        num(f + "nslot", F.nslot);
        num(f + "snjw", F.snjw);
        num(f + "snslot", F.snslot);
        num(f + "gslots", F.gslots);
        buf(f + "xptr", F.xptr);
        buf(f + "xidx", F.xidx);
        buf(f + "xval", F.xval);
        buf(f + "crow", F.crow);
        buf(f + "cval", F.cval);
        buf(f + "jobs", F.jobs);
        buf(f + "scrow", F.scrow);
        buf(f + "scval", F.scval);
        buf(f + "sjobs", F.sjobs);
        buf(f + "segd", F.segd);
        buf(f + "segx", F.segx);
        buf(f + "xsq", F.xsq);
        buf(f + "freqw", F.freqw);
        buf(f + "gchunks", F.gchunks);
        buf(f + "gsums", F.gsums);
        buf(f + "own", F.own);
      }
    }
    buf("popular", popular_);
    buf("gvptr", gvptr_);
    num("npop", npop_);
    return out;
  }

  // --------------------------------------------------------------- init
  // ffm.cpp:467-512.
  // OCFFM_TIMING=1: host wall time of set-up phases on stderr.
  void tmark(const char *name) {
    static const bool on = std::getenv("OCFFM_TIMING") != nullptr;
    if (!on) return;
    if (name) {
      HIPCHK(hipStreamSynchronize(stream_));
      std::fprintf(stderr, "[timing]   %-22s %9.3f ms\n", name,
                   std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tmark_t_).count());
    }
    tmark_t_ = std::chrono::steady_clock::now();
  }
  std::chrono::steady_clock::time_point tmark_t_;

  void init() override {
    ysum_dirty();
    // a previous epoch that threw inside the cross loop may have left the
    // block-excluded form on: the base is rebuilt below from scratch
    excl_ = ExclBase{};
    lazy_ok_ = false;
    // grid-reduction tickets and the persistent CG's words back at rest,
    // whatever a failed call left (every kernel resets what it takes, so
    // this only matters after an error the host reported mid-half)
    side_join();
    HIPCHK(hipMemsetAsync(tick_.p, 0, tick_.bytes(), stream_));
    HIPCHK(hipMemsetAsync(cgp_abort_.p, 0, sizeof(int), stream_));
    HIPCHK(hipMemsetAsync(cgp_gen_buf_.p, 0, sizeof(unsigned), stream_));
    cgp_gen_ = 1;
    run_host_[MAXCG + 3] = 0;
    tmark(nullptr);
    const size_t rs = sizeof(real);
    std::vector<double> host;
    for (uint32_t f1 = 0; f1 < f_; f1++)
      for (uint32_t f2 = f1; f2 < f_; f2++) {
        const uint32_t b12 = block_index(f1, f2, f_);
        if (!blocks_[b12].used) continue;
        DevSide<real> &s1 = side(f1), &s2 = side(f2);
        const uint32_t fi = fidx(f1), fj = fidx(f2);
        const uint64_t D1 = s1.Ds[fi], D2 = s2.Ds[fj];
        W_[b12].alloc(D1 * kp_);
        H_[b12].alloc(D2 * kp_);
        upload_table(W_[b12], D1);
        upload_table(H_[b12], D2);
        P_[b12].alloc(std::max<uint64_t>(s1.R, 1) * kp_);
        Q_[b12].alloc(std::max<uint64_t>(s2.R, 1) * kp_);
        utx(s1, fi, W_[b12].p, P_[b12].p);
        utx(s2, fj, H_[b12].p, Q_[b12].p);
      }
    (void)rs;
    (void)host;
    derive_state();
  }

  // Everything init() derives from W/H (ffm.cpp:490-511): P/Q are already
  // UTX'd; the cross-table lists, sa/sb, the side sums a/b (from zero), the
  // bias sums and y~.  Also the state of a loaded binary snapshot.
  void derive_state() {
    // cross-table pointer lists used by the gradient / sasb / y~ kernels
    std::vector<real *> tl(4 * std::max<uint32_t>(C_, 1) + 4, nullptr);
    uint32_t c = 0;
    for (uint32_t f1 = 0; f1 < fu_; f1++)
      for (uint32_t f2 = fu_; f2 < f_; f2++, c++) {
        const uint32_t b12 = block_index(f1, f2, f_);
        tl[c] = P_[b12].p;            // user-side cross tables
        tl[C_ + c] = Q_[b12].p;       // item-side cross tables
      }
    HIPCHK(hipMemcpy(tabs_.p, tl.data(), tl.size() * sizeof(real *), hipMemcpyHostToDevice));
    tmark("init: tables + UTX");
    cache_sasb();
    if (prm_.self_side) calc_side();
    bias_sums();
    tmark("init: sasb + side");
    init_y_tilde();
    tmark("init: y~");
    sync();
    inited_ = true;
  }

  // Binary snapshot in the layout of the reference's save_binary_model
  // (ffm.cpp:1239-1267, native little-endian): uint32 f, fu, fv, k; uint64
  // Ds of the user fields, then of the item fields; per block in (f1, f2)
  // order (cross blocks only under --ns): uint32 index_vec, uint64 |W|,
  // uint64 |H|, then W and H as doubles, D x k row-major.
  void save_binary(const std::string &path) override {
    need_init();
    std::FILE *fp = std::fopen(path.c_str(), "wb");
    if (!fp) throw Error(OCFFM_E_IO, "cannot write " + path);
    bool ok = true;
    auto put = [&](const void *v, size_t n) { ok = ok && std::fwrite(v, 1, n, fp) == n; };
    const uint32_t hd[4] = {f_, fu_, fv_, k_};
    put(hd, sizeof(hd));
    put(U_.Ds.data(), fu_ * sizeof(uint64_t));
    put(V_.Ds.data(), fv_ * sizeof(uint64_t));
    std::vector<double> w, h;
    for (uint32_t f1 = 0; f1 < f_ && ok; f1++)
      for (uint32_t f2 = f1; f2 < f_ && ok; f2++) {
        const uint32_t b12 = block_index(f1, f2, f_);
        if (!blocks_[b12].used) continue;
        const uint64_t nw = get('W', b12, nullptr, 0), nh = get('H', b12, nullptr, 0);
        w.resize(nw);
        h.resize(nh);
        get('W', b12, w.data(), nw);
        get('H', b12, h.data(), nh);
        put(&b12, sizeof(b12));
        put(&nw, sizeof(nw));
        put(&nh, sizeof(nh));
        put(w.data(), nw * sizeof(double));
        put(h.data(), nh * sizeof(double));
      }
    ok = (std::fclose(fp) == 0) && ok;
    if (!ok) throw Error(OCFFM_E_IO, "write failed: " + path);
  }

  // What the reference's load_binary_model (ffm.cpp:1269-1301) was written
  // to do (it opens an ofstream and writes instead): read the layout above,
  // check it against this problem, restore W/H and re-derive P, Q, sa/sb,
  // a/b and y~ as init does.  The result is the state init() would reach if
  // its draw had produced these tables.
  void load_binary(const std::string &path) override {
    // The whole file is read and checked into host buffers first (header,
    // field sizes, every block's table, no trailing bytes); the device
    // state is touched only after that, so a bad or short file leaves the
    // problem exactly as it was.
    std::FILE *fp = std::fopen(path.c_str(), "rb");
    if (!fp) throw Error(OCFFM_E_IO, "cannot read " + path);
    std::unique_ptr<std::FILE, int (*)(std::FILE *)> guard(fp, &std::fclose);
    auto get_ = [&](void *v, size_t n) {
      if (std::fread(v, 1, n, fp) != n) throw Error(OCFFM_E_DATA, "truncated binary model: " + path);
    };
    uint32_t hd[4];
    get_(hd, sizeof(hd));
    if (hd[0] != f_ || hd[1] != fu_ || hd[2] != fv_ || hd[3] != k_)
      throw Error(OCFFM_E_DATA, "binary model: f/fu/fv/k differ from this problem");
    std::vector<uint64_t> du(fu_), dv(fv_);
    get_(du.data(), fu_ * sizeof(uint64_t));
    get_(dv.data(), fv_ * sizeof(uint64_t));
    if (du != U_.Ds || dv != V_.Ds) throw Error(OCFFM_E_DATA, "binary model: field sizes differ from this problem");
    std::vector<std::pair<uint32_t, std::vector<double>>> tabs;  // (b12, W or H), file order
    for (uint32_t f1 = 0; f1 < f_; f1++)
      for (uint32_t f2 = f1; f2 < f_; f2++) {
        const uint32_t b12 = block_index(f1, f2, f_);
        if (!blocks_[b12].used) continue;
        uint32_t idx;
        uint64_t nw, nh;
        get_(&idx, sizeof(idx));
        get_(&nw, sizeof(nw));
        get_(&nh, sizeof(nh));
        const uint64_t D1 = side(f1).Ds[fidx(f1)], D2 = side(f2).Ds[fidx(f2)];
        if (idx != b12 || nw != D1 * k_ || nh != D2 * k_) throw Error(OCFFM_E_DATA, "binary model: block table differs");
        for (const uint64_t n : {nw, nh}) {
          tabs.emplace_back(b12, std::vector<double>(n));
          get_(tabs.back().second.data(), n * sizeof(double));
        }
      }
    if (std::fgetc(fp) != EOF) throw Error(OCFFM_E_DATA, "binary model: trailing bytes after the last block");
    ysum_dirty();
    excl_ = ExclBase{};
    lazy_ok_ = false;
    for (size_t q = 0; q < tabs.size(); q++) {
      const uint32_t b12 = tabs[q].first;
      const Block &b = blocks_[b12];
      const bool isW = q % 2 == 0;
      const uint32_t fl = isW ? b.f1 : b.f2;
      DevSide<real> &sd = side(fl);
      const uint64_t D = sd.Ds[fidx(fl)];
      const std::vector<double> &w = tabs[q].second;
      DevBuf<real> &dst = isW ? W_[b12] : H_[b12];
      if (!dst.p) dst.alloc(D * kp_);
      std::vector<real> pad(D * kp_, (real)0);
      for (uint64_t rr = 0; rr < D; rr++)
        for (uint32_t cc = 0; cc < k_; cc++) pad[rr * kp_ + cc] = (real)w[rr * k_ + cc];
      HIPCHK(hipMemcpy(dst.p, pad.data(), pad.size() * sizeof(real), hipMemcpyHostToDevice));
      DevBuf<real> &proj = isW ? P_[b12] : Q_[b12];
      if (!proj.p) proj.alloc(std::max<uint64_t>(sd.R, 1) * kp_);
      utx(sd, fidx(fl), dst.p, proj.p);
    }
    HIPCHK(hipMemsetAsync(U_.bias.p, 0, U_.bias.bytes(), stream_));
    HIPCHK(hipMemsetAsync(V_.bias.p, 0, V_.bias.bytes(), stream_));
    owned_stale_ = false;
    derive_state();
  }

  // ------------------------------------------------------------ epoch
  // ffm.cpp:852-870.
  // OCFFM_TIMING=1: per epoch, host wall time and the part of it the host
  // spent blocked on the GPU (CG verdict waits).  Blocked most of the time =
  // GPU-bound; rarely blocked = the host's launch rate is the limit.
  template <class F> auto host_wait(F &&f) {
    if (!timing_) return f();
    const auto t = std::chrono::steady_clock::now();
    auto r = f();
    wait_ms_ += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
    return r;
  }
  // Spin on the host-mapped verdict of CG iteration q until a finalising
  // kernel has published it.  Every few thousand polls the stream is
  // queried, so a faulted kernel surfaces as an error instead of a hang.
  // CGP_GAVE_UP: the persistent CG grid gave up on its barrier (the word
  // MAXCG + 3 holds the step it completed; the caller recovers, `half`).
  static constexpr int CGP_GAVE_UP = -1;
  int poll_verdict(int q) {
    for (uint64_t n = 1;; n++) {
      const int v = __atomic_load_n(&run_host_[q], __ATOMIC_ACQUIRE);
      if (v) return v;
      if (n % 4096 == 0 && __atomic_load_n(&run_host_[MAXCG + 3], __ATOMIC_ACQUIRE)) return CGP_GAVE_UP;
      if (n % 4096 == 0) {
        const hipError_t e = hipStreamQuery(stream_);
        if (e == hipSuccess) {  // stream drained: the word must be there now
          const int w = __atomic_load_n(&run_host_[q], __ATOMIC_ACQUIRE);
          if (w) return w;
          // a full synchronisation, then ~50 ms of polls before calling it lost
          HIPCHK(hipStreamSynchronize(stream_));
          if (__atomic_load_n(&run_host_[MAXCG + 3], __ATOMIC_ACQUIRE)) return CGP_GAVE_UP;
          const auto t0 = std::chrono::steady_clock::now();
          do {
            const int x = __atomic_load_n(&run_host_[q], __ATOMIC_ACQUIRE);
            if (x) return x;
            __builtin_ia32_pause();
          } while (std::chrono::steady_clock::now() - t0 < std::chrono::milliseconds(50));
          throw Error(OCFFM_E_STATE, "CG verdict " + std::to_string(q) + " never published");
        }
        if (e != hipErrorNotReady) HIPCHK(e);
      }
      __builtin_ia32_pause();
    }
  }
  bool timing_ = std::getenv("OCFFM_TIMING") != nullptr;
  double wait_ms_ = 0;

  void one_epoch() override {
    need_init();
    const auto te = std::chrono::steady_clock::now();
    wait_ms_ = 0;
    if (prm_.self_side) {
      for (uint32_t f1 = 0; f1 < fu_; f1++)
        for (uint32_t f2 = f1; f2 < fu_; f2++) solve_block(f1, f2);
      for (uint32_t f1 = fu_; f1 < f_; f1++)
        for (uint32_t f2 = f1; f2 < f_; f2++) solve_block(f1, f2);
    }
    // cross blocks on the block-excluded base, restored after the
    // last one (the side halves and the next epoch read the full base)
    lazy_ok_ = lazy_base_;
    try {
      for (uint32_t f1 = 0; f1 < fu_; f1++)
        for (uint32_t f2 = fu_; f2 < f_; f2++) {
          half(f1, f2, 0);
          half(f1, f2, 1);
        }
    } catch (...) {
      lazy_ok_ = false;
      throw;
    }
    lazy_ok_ = false;
    flush_base();
    if (prm_.self_side) cache_sasb();
    if (timing_) {
      const double host = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - te).count();
      sync();
      const double all = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - te).count();
      std::fprintf(stderr, "[timing] epoch %.3f ms: host enqueue done at %.3f ms, blocked on CG verdicts %.3f ms\n", all,
                   host, wait_ms_);
    }
    flush_prof();
  }

  void solve_block(uint32_t f1, uint32_t f2) override {
    need_init();
    if (f1 > f2 || f2 >= f_) throw Error(OCFFM_E_ARG, "bad block");
    if (!blocks_[block_index(f1, f2, f_)].used) throw Error(OCFFM_E_ARG, "block not in the model (--ns)");
    half(f1, f2, 0);
    half(f1, f2, 1);
  }

  // ffm.cpp:514-535.  Under sharding sb is this rank's partial (it only feeds
  // the item-side gradient, whose partial sums are all-reduced).
  void cache_sasb() override {
    if (C_ == 0) return;
    std::vector<double> vec((size_t)C_ * kp_);
    // sums over item rows of each Q_c -> sa ; over local user rows of P_c -> sb
    for (int sidew = 0; sidew < 2; sidew++) {
      DevSide<real> &part_side = sidew == 0 ? V_ : U_;   // rows summed
      DevSide<real> &out_side = sidew == 0 ? U_ : V_;    // rows scored
      with_kp(kp_, [&](auto K) {
        constexpr int KP = decltype(K)::value;
        using Gm = Geo<real, KP>;
        // column sums of every cross table of the summed side -> vecs_ (C x KP doubles)
        const uint64_t Rs = part_side.R, nout = (uint64_t)C_ * KP;
        uint64_t nbx = std::max<uint64_t>(1, std::min<uint64_t>((Rs + 255) / 256, 512));
        nbx = std::min<uint64_t>(nbx, std::max<uint64_t>(1, part_.n / nout));
        const uint64_t rpb = (Rs + nbx - 1) / nbx;
        prof_launch("aggregates", (double)Rs * C_ * KP * sizeof(real), [&] {
          launch(k_colsum_multi<real, KP>, (unsigned)nbx, BLOCK, 0, Rs, (int)C_,
                 (const real *const *)(tabs_.p + (sidew == 0 ? C_ : 0)), part_.p, rpb);
        });
        prof_launch("aggr_reduce", (double)nbx * nout * 8, [&] {
          launch(k_reduce_parts<real>, (unsigned)((nout + 15) / 16), BLOCK, 0, nbx, nout, (uint64_t)0, nout, part_.p,
                 (uint64_t)0, (real *)nullptr, vecs_.p);
        });
        const uint64_t R = out_side.R;
        if (R == 0) return;
        prof_launch("rowdot_multi", (double)R * (C_ * kp_ * sizeof(real) + sizeof(real)), [&] {
          launch(k_rowdot_multi<real, KP>, grid_for(R, 4 * Gm::NSG), BLOCK, 0,
              R, (int)C_, (const real *const *)(tabs_.p + (sidew == 0 ? 0 : C_)), vecs_.p, out_side.s.p);
        });
      });
    }
  }

  // ------------------------------------------------------- validation
  // forced: the reference's nDCG debug build (EBUG_nDCG, ffm.cpp:988-993):
  // after the ploss term every row's scores become z_j = n - j; per_row
  // (optional, this rank's test rows, cap doubles): nDCG@5,10,20,40,80 of
  // each row, row-major (ffm.cpp:1059-1128; that build prints the @10 one).
  void validate(ocffm_metrics *out, bool forced = false, double *per_row = nullptr, uint64_t cap = 0) override {
    need_init();
    if (per_row && cap < test_rows() * 5) throw Error(OCFFM_E_ARG, "per-row nDCG buffer too small");
    sync_owned();
    static const uint32_t cuts[5] = {5, 10, 20, 40, 80};
    for (int s = 0; s < 5; s++) out->top_k[s] = cuts[s];
    if (!has_test_) {
      out->loss = 0;
      for (int s = 0; s < 5; s++) out->prec[s] = out->ndcg[s] = 0;
      return;
    }
    // projections (ffm.cpp:932-946)
    const uint64_t mt = T_.R;
    std::vector<DevBuf<real>> Pva(blocks_.size()), Qva(blocks_.size());
    for (uint32_t f1 = 0; f1 < f_; f1++)
      for (uint32_t f2 = f1; f2 < f_; f2++) {
        const uint32_t b12 = block_index(f1, f2, f_);
        if (!blocks_[b12].used) continue;
        DevSide<real> &s1 = f1 < fu_ ? T_ : V_, &s2 = f2 < fu_ ? T_ : V_;
        Pva[b12].alloc(std::max<uint64_t>(s1.R, 1) * kp_);
        Qva[b12].alloc(std::max<uint64_t>(s2.R, 1) * kp_);
        utx(s1, fidx(f1), W_[b12].p, Pva[b12].p);
        utx(s2, fidx(f2), H_[b12].p, Qva[b12].p);
      }
    DevBuf<real> at, bt;
    at.alloc(std::max<uint64_t>(mt, 1));
    bt.alloc(std::max<uint64_t>(n_, 1));
    if (prm_.self_side)
      for (uint32_t f1 = 0; f1 < f_; f1++)
        for (uint32_t f2 = f1; f2 < f_; f2++) {
          if ((f1 < fu_) != (f2 < fu_)) continue;
          const uint32_t b12 = block_index(f1, f2, f_);
          rowdot_add(f1 < fu_ ? mt : n_, Pva[b12].p, Qva[b12].p, f1 < fu_ ? at.p : bt.p);
        }
    DevBuf<real *> vt;
    std::vector<real *> tl(2 * std::max<uint32_t>(C_, 1), nullptr);
    for (uint32_t c = 0, f1 = 0; f1 < fu_; f1++)
      for (uint32_t f2 = fu_; f2 < f_; f2++, c++) {
        tl[c] = Pva[block_index(f1, f2, f_)].p;
        tl[C_ + c] = Qva[block_index(f1, f2, f_)].p;
      }
    vt.upload(tl);
    DevBuf<double> rowout;
    rowout.alloc(std::max<uint64_t>(mt, 1) * 11);
    const uint64_t budget = 512ull << 20;
    const uint64_t chunk = std::max<uint64_t>(1, std::min<uint64_t>(mt, budget / (std::max<uint64_t>(n_, 1) * 8)));
    DevBuf<double> z;
    z.alloc(chunk * std::max<uint64_t>(n_, 1), false);
    const uint64_t max_z = npop_;
    for (uint64_t r0 = 0; r0 < mt; r0 += chunk) {
      const uint64_t rows = std::min(chunk, mt - r0);
      with_kp(kp_, [&](auto K) {
        constexpr int KP = decltype(K)::value;
        dim3 g(grid_for(n_, BLOCK, 64), (unsigned)rows);
        launch(k_scores<real, KP>, g, BLOCK, 0, rows, r0, n_, (int)C_, vt.p, vt.p + C_, bt.p, cold_.p,
                                                     popular_.p, npop_, z.p);
      });
      launch(k_rank, (unsigned)rows, BLOCK, 0, rows, r0, n_, max_z, z.p, T_.yptr.p, T_.ycol.p, cold_.p, npop_,
             at_double(at, mt), rowout.p + r0 * 11, (int)forced);
      HIPCHK(hipGetLastError());
    }
    std::vector<double> ro(mt * 11);
    if (mt) HIPCHK(hipMemcpyAsync(ro.data(), rowout.p, mt * 11 * sizeof(double), hipMemcpyDeviceToHost, stream_));
    sync();
    std::vector<double> tot(11, 0.0);
    for (uint64_t i = 0; i < mt; i++)
      for (int x = 0; x < 11; x++) tot[x] += ro[i * 11 + x];
    if (per_row)
      for (uint64_t i = 0; i < mt; i++)
        for (int s = 0; s < 5; s++) per_row[i * 5 + s] = ro[i * 11 + 6 + s];
    allreduce_host(tot.data(), tot.size());
    const double mt_glob = (double)T_.R_glob;
    out->loss = std::sqrt(tot[0] / mt_glob);
    for (int s = 0; s < 5; s++) {
      out->prec[s] = tot[1 + s] / (mt_glob * cuts[s]);
      out->ndcg[s] = tot[6 + s] / mt_glob;
    }
  }

  // ----------------------------------------------------------- access
  uint64_t get(char what, uint32_t b12, double *out, uint64_t cap) override {
    need_init();
    const real *src = nullptr;
    uint64_t rows = 0, cols = 1;
    switch (what) {
      case 'W': case 'H': case 'P': case 'Q': {
        if (b12 >= blocks_.size() || !blocks_[b12].used) throw Error(OCFFM_E_ARG, "block not in the model");
        if (what == 'W' || what == 'H') sync_owned();
        const Block &b = blocks_[b12];
        cols = k_;
        if (what == 'W') { src = W_[b12].p; rows = side(b.f1).Ds[fidx(b.f1)]; }
        if (what == 'H') { src = H_[b12].p; rows = side(b.f2).Ds[fidx(b.f2)]; }
        if (what == 'P') { src = P_[b12].p; rows = side(b.f1).R; }
        if (what == 'Q') { src = Q_[b12].p; rows = side(b.f2).R; }
        break;
      }
      case 'a': src = U_.bias.p; rows = U_.R; break;
      case 'b': src = V_.bias.p; rows = V_.R; break;
      case 's': src = U_.s.p; rows = U_.R; break;
      case 't': src = V_.s.p; rows = V_.R; break;
      case 'u':
      case 'v': return get_ytilde(what == 'u', out, cap);
      default: throw Error(OCFFM_E_ARG, "unknown state name");
    }
    const uint64_t count = rows * cols;
    if (out && cap) {
      const bool table = what == 'W' || what == 'H' || what == 'P' || what == 'Q';  // rows padded to kp_ (k = 1 too)
      const uint64_t stride = table ? kp_ : 1;
      std::vector<real> tmp(rows * stride);
      sync();
      if (rows) HIPCHK(hipMemcpy(tmp.data(), src, tmp.size() * sizeof(real), hipMemcpyDeviceToHost));
      for (uint64_t rr = 0, o = 0; rr < rows; rr++)
        for (uint64_t cc = 0; cc < cols && o < cap; cc++, o++) out[o] = (double)tmp[rr * stride + cc];
    }
    return count;
  }

  // y~ = base + a_i + b_j (the factored form, kernels.hpp k_init_ytilde), in
  // the user-major ('u') or item-major ('v') orientation of this rank.
  uint64_t get_ytilde(bool user_major, double *out, uint64_t cap) {
    DevSide<real> &s = user_major ? U_ : V_;
    const uint64_t np = s.npos;
    if (!out || !cap) return np;
    flush_base();
    sync();
    auto down = [&](auto &buf, size_t n) {
      std::vector<typename std::remove_pointer<decltype(buf.p)>::type> v(n);
      if (n) HIPCHK(hipMemcpy(v.data(), buf.p, n * sizeof(v[0]), hipMemcpyDeviceToHost));
      return v;
    };
    auto base = down(s.yt, np);
    auto ptr = down(s.yptr, s.R + 1);
    auto col = down(s.ycol, np);
    auto a = down(U_.bias, U_.R);
    auto b = down(V_.bias, V_.R);
    for (uint64_t i = 0; i < s.R; i++)
      for (int64_t p = ptr[i]; p < ptr[i + 1] && (uint64_t)p < cap; p++) {
        const uint64_t ui = user_major ? i : col[p], vj = user_major ? col[p] : i;
        out[p] = (double)base[p] + (double)a[ui] + (double)b[vj];
      }
    return np;
  }

  void set(char what, uint32_t b12, const double *in, uint64_t len) override {
    ysum_dirty();
    need_init();
    flush_base();  // restore the full base while P/Q still match it
    if (b12 >= blocks_.size() || !blocks_[b12].used) throw Error(OCFFM_E_ARG, "block not in the model");
    const Block &b = blocks_[b12];
    const bool isW = what == 'W';
    if (!isW && what != 'H') throw Error(OCFFM_E_ARG, "only W or H can be set");
    const uint32_t fl = isW ? b.f1 : b.f2;
    DevSide<real> &s = side(fl);
    const uint64_t D = s.Ds[fidx(fl)];
    if (len != D * k_) throw Error(OCFFM_E_ARG, "size mismatch");
    std::vector<real> tmp(D * kp_, (real)0);
    for (uint64_t rr = 0; rr < D; rr++)
      for (uint32_t cc = 0; cc < k_; cc++) tmp[rr * kp_ + cc] = (real)in[rr * k_ + cc];
    DevBuf<real> &dst = isW ? W_[b12] : H_[b12];
    HIPCHK(hipMemcpy(dst.p, tmp.data(), tmp.size() * sizeof(real), hipMemcpyHostToDevice));
    utx(s, fidx(fl), dst.p, isW ? P_[b12].p : Q_[b12].p);
    sync();
  }

  void grad(uint32_t f1, uint32_t f2, int half_id, double *out) override {
    need_init();
    HalfCtx hc = half_ctx(f1, f2, half_id);
    want_g_ = true;
    gradient(hc);
    want_g_ = false;
    copy_out(G_.p, hc.D, out);
  }

  void hv(uint32_t f1, uint32_t f2, int half_id, const double *v, double *out) override {
    need_init();
    HalfCtx hc = half_ctx(f1, f2, half_id);
    std::vector<real> tmp(hc.D * kp_, (real)0);
    for (uint64_t rr = 0; rr < hc.D; rr++)
      for (uint32_t cc = 0; cc < k_; cc++) tmp[rr * kp_ + cc] = (real)v[rr * k_ + cc];
    HIPCHK(hipMemcpyAsync(Vd_.p, tmp.data(), tmp.size() * sizeof(real), hipMemcpyHostToDevice, stream_));
    if (hc.cross) {  // QTQ over the partner rows (slot of this block in the Gram list)
      aggregates(hc.partner->R, (int)C_, partner_tabs(hc), hc.Q1, nullptr, M_.p);
      const uint32_t c0 = cross_slot(std::min(hc.fl, hc.fo), std::max(hc.fl, hc.fo));
      qtq_ = M_.p + (size_t)c0 * kp_ * kp_;
    }
    ccg_now_ = ccg_eligible(hc) && ccg_mode_ == 2;
    hot_now_ = hot_steps_ == 0;
    col_grams(hc);
    hot_grams(hc, xfuse(hc));
    // force iteration 1 to run
    CgState hs{};
    hs.run[1] = 1;
    hs.r2 = 1.0;
    sync();
    HIPCHK(hipMemcpy(st_.p, &hs, sizeof(CgState), hipMemcpyHostToDevice));
    hv_pass(hc, 1);
    ccg_now_ = hot_now_ = false;
    sync();
    copy_out(Hv_.p, hc.D, out);
  }

  // ffm.cpp:1163-1237: the reference's text model.  Values are formatted as
  // the reference's ostream does by default (precision 6, %g), by
  // std::to_chars(general, 6), which the standard defines as that printf
  // conversion; row ranges are formatted by parallel host threads and
  // written in order.
  void save_model(const std::string &path) override {
    need_init();
    std::FILE *fp = std::fopen(path.c_str(), "wb");
    if (!fp) throw Error(OCFFM_E_IO, "cannot write " + path);
    std::string head = std::to_string(f_) + "\n" + std::to_string(fu_) + "\n" + std::to_string(fv_) + "\n" +
                       std::to_string(k_) + "\n";
    for (uint32_t i = 0; i < fu_; i++) head += std::to_string(U_.Ds[i]) + "\n";
    for (uint32_t i = 0; i < fv_; i++) head += std::to_string(V_.Ds[i]) + "\n";
    bool ok = std::fwrite(head.data(), 1, head.size(), fp) == head.size();
    const unsigned nth = std::max(1u, std::min(32u, std::thread::hardware_concurrency()));
    std::vector<double> buf;
    std::vector<std::string> parts(nth);
    for (uint32_t fi = 0; fi < f_ && ok; fi++)
      for (uint32_t fj = fi; fj < f_ && ok; fj++) {
        const uint32_t b12 = block_index(fi, fj, f_);
        if (!blocks_[b12].used) continue;
        for (int t = 0; t < 2 && ok; t++) {
          const char c = t == 0 ? 'W' : 'H';
          const uint64_t cnt = get(c, b12, nullptr, 0);
          buf.resize(cnt);
          get(c, b12, buf.data(), cnt);
          const uint64_t rows = cnt / k_;
          const std::string pre = std::string(1, c) + "," + std::to_string(fi) + "," + std::to_string(fj) + ",";
          auto work = [&](unsigned w) {
            std::string &o = parts[w];
            o.clear();
            const uint64_t r0 = rows * w / nth, r1 = rows * (w + 1) / nth;
            char num[64];
            for (uint64_t rr = r0; rr < r1; rr++) {
              o += pre;
              auto res = std::to_chars(num, num + sizeof(num), rr);
              o.append(num, res.ptr);
              for (uint32_t e = 0; e < k_; e++) {
                o += ' ';
                res = std::to_chars(num, num + sizeof(num), buf[rr * k_ + e], std::chars_format::general, 6);
                o.append(num, res.ptr);
              }
              o += '\n';
            }
          };
          std::vector<std::thread> th;
          for (unsigned w = 1; w < nth; w++) th.emplace_back(work, w);
          work(0);
          for (auto &x : th) x.join();
          for (auto &o : parts) ok = ok && std::fwrite(o.data(), 1, o.size(), fp) == o.size();
        }
      }
    ok = (std::fclose(fp) == 0) && ok;
    if (!ok) throw Error(OCFFM_E_IO, "write failed: " + path);
  }

 private:
  // ------------------------------------------------------------ setup
  // Owned-field test over the contiguous row shards of all ranks (every rank
  // holds the whole HostData, so no communication is needed): per field, the
  // rank whose rows touch each feature (-1: none, -2: several), from one
  // pass over the parsed nodes.
  std::vector<std::vector<int32_t>> owners(const HostData &d, const std::vector<uint64_t> &Ds) {
    const Rows &r = d.raw;
    const uint64_t m = d.m, N = (uint64_t)comm_.nranks, nf = Ds.size();
    std::vector<std::vector<int32_t>> who(nf);
    for (uint64_t f = 0; f < nf; f++) who[f].assign(Ds[f], -1);
    for (uint64_t q = 0; q < N; q++) {
      const uint64_t a = m * q / N, b = m * (q + 1) / N;
      for (uint64_t p = r.xptr[a]; p < r.xptr[b]; p++) {
        if (r.fid[p] >= nf) continue;
        int32_t &w = who[r.fid[p]][r.idx[p]];
        if (w == -1) w = (int32_t)q;
        else if (w != (int32_t)q) w = -2;
      }
    }
    return who;
  }
  void ownership(DevField<real> &F, const std::vector<int32_t> &who) {
    if (no_owned_ || std::find(who.begin(), who.end(), -2) != who.end()) return;
    F.excl = true;
    F.h_own.resize(F.D);
    for (uint64_t x = 0; x < F.D; x++) F.h_own[x] = who[x] == comm_.rank || (who[x] < 0 && comm_.rank == 0);
    F.own.upload(F.h_own);
  }
  // --freq on several ranks: each field's feature counts over all rows.
  std::vector<std::vector<double>> global_counts(const HostData &d, const std::vector<uint64_t> &Ds) {
    const Rows &r = d.raw;
    std::vector<std::vector<double>> c(Ds.size());
    for (size_t f = 0; f < Ds.size(); f++) c[f].assign(Ds[f], 0.0);
    for (uint64_t p = 0; p < r.fid.size(); p++)
      if (r.fid[p] < Ds.size()) c[r.fid[p]][r.idx[p]] += 1;
    return c;
  }
  // Side halves of this one-node field run on per-column Grams.
  bool gram_field(const DevField<real> &F, uint64_t R) const {
    return F.one && !F.idlike && !F.excl && cgram_on_ && R > 0 && prm_.self_side && cgram_pays(R, F.D) &&
           F.D * kp_ * kp_ * sizeof(real) <= (1ull << 30);
  }

  // Per-field CSR, CSC + jobs, flags and column sums of rows [r0, r1) of d
  // (split_fields, ffm.cpp:185-257, and the layout of DESIGN §5), on the
  // device (devbuild.h); OCFFM_HOST_BUILD=1: on the host.  Returns (device
  // build) each field's fp64 node values, which the segment CSCs read.
  std::vector<DevBuf<double>> build_fields(DevSide<real> &s, const HostData &d, uint64_t r0, uint64_t r1,
                                           const std::vector<uint64_t> &Ds_glob, dev::Builder &B, bool owned = false) {
    s.F.clear();
    s.Ds = Ds_glob;
    const uint64_t R = r1 - r0;
    const uint32_t nf = (uint32_t)Ds_glob.size();
    std::vector<std::vector<int32_t>> who;
    if (owned) who = owners(d, Ds_glob);
    std::vector<std::vector<double>> gcnt;
    if (prm_.freq && comm_.nranks > 1) gcnt = global_counts(d, Ds_glob);
    if (host_build_) {
      build_fields_host(s, split_host(d), r0, r1, Ds_glob, who, gcnt);
      return {};
    }
    std::vector<dev::CSR> csr = B.split(d, r0, r1, nf);
    tmark("create:   split_fields");
    std::vector<DevBuf<double>> vals(nf);
    for (uint32_t fi = 0; fi < nf; fi++) {
      auto F = std::make_unique<DevField<real>>();
      F->D = Ds_glob[fi];
      dev::CSR &x = csr[fi];
      F->nnz = x.nnz;
      if (owned && fi < d.f) ownership(*F, who[fi]);
      dev::CSC c;
      B.csc(x, F->D, nsg(), F->excl ? F->own.p : nullptr, c);
      B.flags(x, c, F->D, F->one, F->idlike);
      F->xptr = std::move(x.xptr);
      F->xidx = std::move(x.xidx);
      to_real_dev(x.xval.p, x.nnz, F->xval);
      if (F->one) to_real_dev(B.xsq(c, F->D), std::max<uint64_t>(F->D, 1), F->xsq);
      F->crow = std::move(c.crow);
      to_real_dev(c.cval, F->nnz, F->cval);
      F->jobs = std::move(c.jobs);
      F->njw = c.njobs / nsg();
      F->nslot = c.nslot;
      F->hdots.alloc(std::max<uint64_t>(F->nslot, 1) * 3);
      F->cnt.alloc(std::max<uint64_t>(F->D, 1));
      if (gram_field(*F, R)) {
        std::vector<int64_t> cptr(F->D + 1);
        HIPCHK(hipMemcpyAsync(cptr.data(), c.cptr, cptr.size() * sizeof(int64_t), hipMemcpyDeviceToHost, stream_));
        B.sync();
        col_gram_chunks(*F, cptr);
      }
      if (prm_.freq && fi < d.f) {
        if (comm_.nranks > 1) {
          F->freqw.upload(to_real(gcnt[fi]));
        } else {
          to_real_dev(B.col_counts(c, F->D), F->D, F->freqw);
        }
      }
      B.sync();  // (c's buffers are freed at the end of the iteration)
      vals[fi] = std::move(x.xval);
      s.F.push_back(std::move(F));
    }
    tmark("create:   CSCs + jobs");
    return vals;
  }

  // The host build: the reference's loops restated (the checker of the
  // device build, OCFFM_HOST_BUILD=1).
  void build_fields_host(DevSide<real> &s, const HostData &d, uint64_t r0, uint64_t r1,
                         const std::vector<uint64_t> &Ds_glob, const std::vector<std::vector<int32_t>> &who,
                         const std::vector<std::vector<double>> &gcnt) {
    const uint64_t R = r1 - r0;
    for (uint64_t fi = 0; fi < Ds_glob.size(); fi++) {
      auto F = std::make_unique<DevField<real>>();
      F->D = Ds_glob[fi];
      std::vector<int64_t> xptr(R + 1, 0);
      std::vector<uint32_t> xidx;
      std::vector<double> xval;
      if (fi < d.f) {
        const int64_t base = d.xptr[fi][r0];
        for (uint64_t i = 0; i <= R; i++) xptr[i] = d.xptr[fi][r0 + i] - base;
        xidx.assign(d.xidx[fi].begin() + base, d.xidx[fi].begin() + d.xptr[fi][r1]);
        xval.assign(d.xval[fi].begin() + base, d.xval[fi].begin() + d.xptr[fi][r1]);
      }
      F->nnz = xidx.size();
      F->one = R > 0 && F->nnz == R;
      for (uint64_t i = 0; i < R && F->one; i++) F->one = xptr[i + 1] - xptr[i] == 1;
      if (F->nnz == R && F->D == R && R > 0) {
        std::vector<uint8_t> seen(F->D, 0);
        bool ok = true;
        for (uint64_t i = 0; i < R && ok; i++) {
          if (xptr[i + 1] - xptr[i] != 1 || seen[xidx[xptr[i]]]) ok = false;
          else seen[xidx[xptr[i]]] = 1;
        }
        F->idlike = ok;
      }
      if (!who.empty() && fi < d.f) ownership(*F, who[fi]);
      F->xptr.upload(xptr);
      F->xidx.upload(xidx);
      F->xval.upload(to_real(xval));
      std::vector<uint32_t> crow;
      std::vector<double> cval;
      std::vector<Job> jobs;
      build_csc(R, F->D, xptr.data(), xidx.data(), xval.data(), nsg(), crow, cval, jobs, F->nslot,
                F->excl ? F->h_own.data() : nullptr);
      if (F->one) {  // sum of x^2 per column, rows in order (devbuild.h xsq_col)
        std::vector<uint64_t> cptr(F->D + 1, 0);
        for (uint32_t c : xidx) cptr[c + 1]++;
        for (uint64_t q = 0; q < F->D; q++) cptr[q + 1] += cptr[q];
        std::vector<double> sq(std::max<uint64_t>(F->D, 1), 0.0);
        for (uint64_t q = 0; q < F->D; q++) sq[q] = dev::xsq_col(cval.data() + cptr[q], cptr[q + 1] - cptr[q]);
        F->xsq.upload(to_real(sq));
      }
      F->crow.upload(crow);
      F->cval.upload(to_real(cval));
      F->jobs.upload(jobs);
      F->njw = jobs.size() / nsg();
      F->hdots.alloc(std::max<uint64_t>(F->nslot, 1) * 3);
      F->cnt.alloc(std::max<uint64_t>(F->D, 1));
      if (gram_field(*F, R)) {
        std::vector<int64_t> cptr(F->D + 1, 0);
        for (uint32_t c : xidx) cptr[c + 1]++;
        for (uint64_t q = 0; q < F->D; q++) cptr[q + 1] += cptr[q];
        col_gram_chunks(*F, cptr);
      }
      F->h_xptr = std::move(xptr);
      F->h_xidx = std::move(xidx);
      F->h_xval = std::move(xval);
      if (prm_.freq && fi < d.f) {  // global counts (all rows, not just this shard)
        if (!gcnt.empty()) {
          F->freqw.upload(to_real(gcnt[fi]));
        } else {
          std::vector<double> fr(F->D, 0.0);
          for (uint32_t x : d.xidx[fi]) fr[x] += 1;
          F->freqw.upload(to_real(fr));
        }
      }
      s.F.push_back(std::move(F));
    }
  }

  // Segments and the segment CSCs of a side on the device (the host build:
  // build_segments).  vals: each field's fp64 node values (build_fields).
  void build_segments_dev(DevSide<real> &s, const DevBuf<int64_t> &yptr, uint64_t R, std::vector<DevBuf<double>> &vals,
                          dev::Builder &B) {
    B.segments(yptr.p, R, seg_len_, s.segs, s.segptr, s.nseg);
    for (size_t fi = 0; fi < s.F.size(); fi++) {
      DevField<real> &F = *s.F[fi];
      const dev::CSR &ex = B.seg_expand(F.xptr.p, F.xidx.p, vals[fi].p, s.segs.p, s.nseg);
      if (F.one) {  // one node per segment
        F.segd.alloc(ex.nnz, false);
        if (ex.nnz)
          HIPCHK(hipMemcpyAsync(F.segd.p, ex.xidx.p, ex.nnz * sizeof(uint32_t), hipMemcpyDeviceToDevice, stream_));
        to_real_dev(ex.xval.p, ex.nnz, F.segx);
      }
      dev::CSC c;
      B.csc(ex, F.D, nsg(), F.excl ? F.own.p : nullptr, c);
      F.scrow = std::move(c.crow);
      to_real_dev(c.cval, ex.nnz, F.scval);
      F.sjobs = std::move(c.jobs);
      F.snjw = c.njobs / nsg();
      F.snslot = c.nslot;
      F.shdots.alloc(std::max<uint64_t>(F.snslot, 1) * 3);
      B.sync();
      vals[fi].release();
    }
  }

  void build_user_side(const HostData &U, dev::Builder &B) {
    U_.R = u1_ - u0_;
    U_.R_glob = U.m;
    U_.row0 = u0_;
    auto vals = build_fields(U_, U, u0_, u1_, U.Ds, B, comm_.nranks > 1);
    const uint64_t pb = U.yptr[u0_], pe = U.yptr[u1_];
    U_.npos = pe - pb;
    if (host_build_) {
      std::vector<int64_t> yptr(U_.R + 1);
      for (uint64_t i = 0; i <= U_.R; i++) yptr[i] = (int64_t)(U.yptr[u0_ + i] - pb);
      std::vector<uint32_t> ycol(pe - pb);
      for (uint64_t p = pb; p < pe; p++) ycol[p - pb] = (uint32_t)U.ycol[p];
      build_segments(U_, yptr, seg_len_, nsg());
      U_.yptr.upload(yptr);
      U_.ycol.upload(ycol);
    } else {
      B.labels(U, u0_, u1_, U_.yptr, U_.ycol);
      build_segments_dev(U_, U_.yptr, U_.R, vals, B);
      tmark("create:   segments + CSCs");
    }
    U_.yt.alloc(std::max<uint64_t>(U_.npos, 1));
    U_.bias.alloc(std::max<uint64_t>(U_.R, 1));
    U_.s.alloc(std::max<uint64_t>(U_.R, 1));
  }

  // Item-major positives restricted to this rank's users, and the position
  // maps between the two orientations (transY order: users increasing,
  // labels in file order, ffm.cpp:259-294).
  void build_item_side(const HostData &V, const HostData &U, dev::Builder &B) {
    V_.R = V.m;
    V_.R_glob = V.m;
    V_.row0 = 0;
    auto vals = build_fields(V_, V, 0, V.m, V.Ds, B);
    V_.npos = U_.npos;
    if (!host_build_) {
      // (U_.yptr / U_.ycol: this rank's user-major labels, build_user_side)
      DevBuf<uint32_t> v2u, u2v;
      B.transpose(U_.yptr, U_.ycol, U_.R, V.m, V_.yptr, V_.ycol, v2u, u2v);
      if (comm_.active()) {  // the counts over ALL users (item side halves' CG steps, repl())
        B.label_ptr(U, V.m, gvptr_);
        gn1_ = (double)U.m;
      }
      build_segments_dev(V_, V_.yptr, V.m, vals, B);
      V_.perm = std::move(v2u);
      U_.perm = std::move(u2v);
    } else {
      std::vector<int64_t> vptr(V.m + 1, 0);
      for (uint64_t i = u0_; i < u1_; i++)
        for (uint64_t p = U.yptr[i]; p < U.yptr[i + 1]; p++) vptr[U.ycol[p] + 1]++;
      for (uint64_t j = 0; j < V.m; j++) vptr[j + 1] += vptr[j];
      const uint64_t np = (uint64_t)vptr[V.m];
      std::vector<uint32_t> vcol(np), u2v(U_.npos), v2u(np);
      std::vector<int64_t> cur(vptr.begin(), vptr.end() - 1);
      const uint64_t pb = U.yptr[u0_];
      for (uint64_t i = u0_; i < u1_; i++)
        for (uint64_t p = U.yptr[i]; p < U.yptr[i + 1]; p++) {
          const uint64_t q = (uint64_t)cur[U.ycol[p]]++;
          vcol[q] = (uint32_t)(i - u0_);
          u2v[p - pb] = (uint32_t)q;
          v2u[q] = (uint32_t)(p - pb);
        }
      if (comm_.active()) {
        std::vector<int64_t> gptr(V.m + 1, 0);
        for (uint64_t i = 0; i < U.m; i++)
          for (uint64_t p = U.yptr[i]; p < U.yptr[i + 1]; p++) gptr[U.ycol[p] + 1]++;
        for (uint64_t j = 0; j < V.m; j++) gptr[j + 1] += gptr[j];
        gvptr_.upload(gptr);
        gn1_ = (double)U.m;
      }
      build_segments(V_, vptr, seg_len_, nsg());
      V_.yptr.upload(vptr);
      V_.ycol.upload(vcol);
      V_.perm.upload(v2u);
      U_.perm.upload(u2v);
    }
    V_.yt.alloc(std::max<uint64_t>(V_.npos, 1));
    V_.bias.alloc(std::max<uint64_t>(V_.R, 1));
    V_.s.alloc(std::max<uint64_t>(V_.R, 1));
  }

  void build_test(const HostData &Ut, const HostData &U, dev::Builder &B) {
    const uint64_t t0 = Ut.m * (uint64_t)comm_.rank / (uint64_t)comm_.nranks;
    const uint64_t t1 = Ut.m * (uint64_t)(comm_.rank + 1) / (uint64_t)comm_.nranks;
    T_.R = t1 - t0;
    T_.R_glob = Ut.m;
    T_.row0 = t0;
    std::vector<uint64_t> Ds(U.Ds);  // test fields use the train Ds
    build_fields(T_, Ut, t0, t1, Ds, B);
    if (host_build_) {
      for (auto &F : T_.F) {
        F->h_xptr.clear();
        F->h_xidx.clear();
        F->h_xval.clear();
      }
      std::vector<int64_t> lptr(T_.R + 1);
      const uint64_t lb = Ut.yptr[t0];
      for (uint64_t i = 0; i <= T_.R; i++) lptr[i] = (int64_t)(Ut.yptr[t0 + i] - lb);
      std::vector<uint32_t> lcol(Ut.yptr[t1] - lb);
      for (uint64_t p = lb; p < Ut.yptr[t1]; p++)
        lcol[p - lb] = (uint32_t)std::min<uint64_t>(Ut.ycol[p], 0xffffffffu);
      T_.yptr.upload(lptr);
      T_.ycol.upload(lcol);
    } else {
      B.labels(Ut, t0, t1, T_.yptr, T_.ycol);
    }
    std::vector<uint8_t> cold(std::max<uint64_t>(T_.R, 1), 0);
    for (uint64_t i = 0; i < T_.R; i++) cold[i] = Ut.nnx[t0 + i] == 0;
    cold_.upload(cold);
  }

  // fp64 values to the solver's precision on the device (the same rounding
  // as the host's (real) cast)
  void to_real_dev(const double *in, uint64_t n, DevBuf<real> &out) {
    out.alloc(n, false);
    if (!n) return;
    if constexpr (std::is_same<real, double>::value) {
      HIPCHK(hipMemcpyAsync(out.p, in, n * sizeof(double), hipMemcpyDeviceToDevice, stream_));
    } else {
      launch(k_to_real<real>, grid_for(n, BLOCK, 8192), BLOCK, 0, n, in, out.p);
    }
  }
  void to_real_dev(const DevBuf<double> &in, DevBuf<real> &out) { to_real_dev(in.p, in.n, out); }

  std::vector<real> to_real(const std::vector<double> &v) {
    std::vector<real> o(v.size());
    for (size_t i = 0; i < v.size(); i++) o[i] = (real)v[i];
    return o;
  }

  // init_mat (ffm.cpp:71-78): drawn on the device (devbuild.h draw_table;
  // OCFFM_HOST_INIT=1: on the host and uploaded), the same values either way.
  void upload_table(DevBuf<real> &t, uint64_t D) {
    if (!host_init_) {
      dev::draw_table<real>(stream_, t.p, D, k_, kp_, table_draw(k_));
      return;
    }
    std::vector<double> host(D * k_);
    init_table(host.data(), D, k_);
    std::vector<real> pad(D * kp_, (real)0);
    for (uint64_t rr = 0; rr < D; rr++)
      for (uint32_t cc = 0; cc < k_; cc++) pad[rr * kp_ + cc] = (real)host[rr * k_ + cc];
    HIPCHK(hipMemcpy(t.p, pad.data(), pad.size() * sizeof(real), hipMemcpyHostToDevice));
  }

  void copy_out(const real *src, uint64_t D, double *out) {
    std::vector<real> tmp(D * kp_);
    sync();
    HIPCHK(hipMemcpy(tmp.data(), src, tmp.size() * sizeof(real), hipMemcpyDeviceToHost));
    for (uint64_t rr = 0; rr < D; rr++)
      for (uint32_t cc = 0; cc < k_; cc++) out[rr * k_ + cc] = (double)tmp[rr * kp_ + cc];
  }

  void need_init() const {
    if (!inited_) throw Error(OCFFM_E_STATE, "call ocffm_problem_init first");
  }

  DevSide<real> &side(uint32_t fl) { return fl < fu_ ? U_ : V_; }
  uint32_t fidx(uint32_t fl) const { return fl < fu_ ? fl : fl - fu_; }
  // cross tables: which 0 = user-side P_c, 1 = item-side Q_c (c in block order)
  real *cross_tab(int which, uint32_t c) {
    uint32_t cc = 0;
    for (uint32_t f1 = 0; f1 < fu_; f1++)
      for (uint32_t f2 = fu_; f2 < f_; f2++, cc++)
        if (cc == c) return which == 0 ? P_[block_index(f1, f2, f_)].p : Q_[block_index(f1, f2, f_)].p;
    return nullptr;
  }
  uint32_t cross_slot(uint32_t f1, uint32_t f2) const { return f1 * fv_ + (f2 - fu_); }
  // Device list of the partner side's cross tables: a user half multiplies
  // item-side Q_c (slots C..2C), an item half user-side P_c (slots 0..C).
  template <class HC> const real *const *partner_tabs(const HC &h) const {
    return (const real *const *)(tabs_.p + (h.user ? C_ : 0));
  }

  // ------------------------------------------------------ primitives
  // Kernel launches go through launch(): when prof_launch has armed an event
  // pair, the dispatch packet itself carries them (hipExtLaunchKernel: start
  // on the first dispatch of the armed region, stop after each), so the
  // recorded time is the kernels' own, as rocprofv3's kernel trace sees it.
  // Blocks of kernel k (BLOCK threads, smem bytes) resident on the whole
  // GPU at once (the occupancy API's per-CU count x CUs; cached per kernel).
  std::unordered_map<const void *, unsigned> resident_;
  template <typename... KArgs> unsigned resident(void (*k)(KArgs...), size_t smem) {
    const void *key = reinterpret_cast<const void *>(k);
    auto it = resident_.find(key);
    if (it != resident_.end()) return it->second;
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, key, BLOCK, smem) != hipSuccess || nb <= 0) nb = 1;
    const unsigned r = (unsigned)nb * std::max(1u, ncu_);
    resident_[key] = r;
    return r;
  }
  // grid capped at one resident wave of blocks (OCFFM_MISC_FILL: the side
  // gradient, update and column-Gram step passes; no LDS)
  bool misc_fill_ = !std::getenv("OCFFM_MISC_FILL") || std::atoi(std::getenv("OCFFM_MISC_FILL")) != 0;
  template <typename... KArgs> unsigned mfill(void (*k)(KArgs...), unsigned grid) {
    return misc_fill_ ? std::min(grid, resident(k, 0)) : grid;
  }
  template <typename... KArgs, typename... A>
  void launch(void (*k)(KArgs...), dim3 grid, dim3 block, size_t smem, A... a) {
    static_assert(sizeof...(KArgs) == sizeof...(A), "kernel argument count");
    hipEvent_t e0 = arm_first_ ? arm_a_ : nullptr;
    arm_first_ = false;
    hipExtLaunchKernelGGL(k, grid, block, (uint32_t)smem, stream_, e0, arm_b_, 0u, static_cast<KArgs>(a)...);
    HIPCHK(hipGetLastError());
  }
  // bytes / flops: the launch's algorithmic HBM bytes and (MFMA kernels)
  // floating-point operations, for the roofline of its family
  template <class L> void prof_launch(const char *name, double bytes, L &&body, double flops = 0) {
    if (!profiling || (!prof_filter.empty() && prof_filter != name)) {
      body();
      HIPCHK(hipGetLastError());
      return;
    }
    arm_a_ = ev();
    arm_b_ = ev();
    arm_first_ = true;
    body();
    HIPCHK(hipGetLastError());
    if (arm_first_) {  // the region launched nothing (all work empty): zero-length record
      HIPCHK(hipEventRecord(arm_a_, stream_));
      HIPCHK(hipEventRecord(arm_b_, stream_));
    }
    pending_.push_back({name, bytes, arm_a_, arm_b_, prof_tag_, flops});
    arm_a_ = arm_b_ = nullptr;
    arm_first_ = false;
  }
  hipEvent_t ev() {
    if (ev_free_.empty()) {
      hipEvent_t e;
      HIPCHK(hipEventCreate(&e));
      ev_pool_.push_back(e);
      return e;
    }
    hipEvent_t e = ev_free_.back();
    ev_free_.pop_back();
    return e;
  }
  void flush_prof() {
    if (pending_.empty()) return;
    sync();
    for (auto &p : pending_) {
      float ms = 0;
      HIPCHK(hipEventElapsedTime(&ms, p.a, p.b));
      KStat &k = kstats[p.name];
      k.launches++;
      k.ms += ms;
      k.bytes += p.bytes;
      k.flops += p.flops;
      ev_free_.push_back(p.a);
      ev_free_.push_back(p.b);
    }
    pending_.clear();
  }

  void utx(DevSide<real> &s, uint32_t fi, const real *A, real *out) {
    if (s.R == 0) return;
    DevField<real> &F = *s.F[fi];
    with_kp(kp_, [&](auto K) {
      constexpr int KP = decltype(K)::value;
      using Gm = Geo<real, KP>;
      prof_launch("utx", 0, [&] {
        launch(k_utx<real, KP>, grid_for(s.R, 4 * Gm::NSG), BLOCK, 0, s.R, F.xptr.p, F.xidx.p, F.xval.p, A, out);
      });
    });
  }

  void rowdot_add(uint64_t R, const real *P, const real *Q, real *acc) {
    if (R == 0) return;
    with_kp(kp_, [&](auto K) {
      constexpr int KP = decltype(K)::value;
      using Gm = Geo<real, KP>;
      launch(k_rowdot_add<real, KP>, grid_for(R, 4 * Gm::NSG), BLOCK, 0, R, P, Q, acc);
      HIPCHK(hipGetLastError());
    });
  }

  // bsum_ = (sum of a over this rank's users, sum of b): the b_sum term of
  // gd_side (ffm.cpp:551).  Kept current by k_update_side_row afterwards.
  void bias_sums() {
    for (int sd = 0; sd < 2; sd++) {
      DevSide<real> &s = sd ? V_ : U_;
      launch(k_vec_sum<real>, grid_for(s.R, BLOCK, 256), BLOCK, 0, (uint64_t)s.R, (const real *)s.bias.p,
             bsum_.p + sd, part_.p, tick_.p);
    }
  }

  // calc_side (ffm.cpp:360-373): a += <P,Q> over user-side blocks, b over item-side.
  void calc_side() {
    for (uint32_t f1 = 0; f1 < f_; f1++)
      for (uint32_t f2 = f1; f2 < f_; f2++) {
        if ((f1 < fu_) != (f2 < fu_)) continue;
        const uint32_t b12 = block_index(f1, f2, f_);
        DevSide<real> &s = side(f1);
        rowdot_add(s.R, P_[b12].p, Q_[b12].p, s.bias.p);
      }
  }

  void init_y_tilde() {
    if (U_.R == 0) return;
    with_kp(kp_, [&](auto K) {
      constexpr int KP = decltype(K)::value;
      launch(k_init_ytilde<real, KP>, grid_for(U_.R, 4), BLOCK, 0,
          U_.R, U_.yptr.p, U_.ycol.p, U_.yt.p, V_.yt.p, U_.perm.p, (int)C_, (const real *const *)tabs_.p,
          (const real *const *)(tabs_.p + C_), U_.bias.p, V_.bias.p);
      HIPCHK(hipGetLastError());
    });
  }

  // Partner-side aggregates over Rp rows in one pass (kernels.hpp:
  // k_gram_part): M (L x KP x KP, real) = A_l^T B for the device pointer
  // list A, and sums_ = [sum B | sum wv*B | sum wv] (doubles).  A or B or wv
  // may be absent (L = 0, B = null, wv = null).
  static constexpr int GRAM_LMAX = 8;  // tables per k_gram_mfma32 launch
  bool mfma_gram(int L) const { return std::is_same<real, float>::value && kp_ == 32 && L >= 1 && !no_mfma_; }

  void aggregates(uint64_t Rp, int L, const real *const *A, const real *B, const real *wv, real *M) {
    const size_t rs = sizeof(real);
    if (mfma_gram64(L, Rp)) {  // fp32, KP = 64: every table in one launch (k_gram_mfma64)
      gram64(Rp, L, A, B, wv, M);
      return;
    }
    if (std::is_same<real, double>::value && kp_ == 32 && L >= 1 && !no_mfma_ && B_ok(Rp) && M && B) {
      gram_f64(Rp, L, A, B, wv, M);  // fp64, KP = 32: every table in one launch (k_gram_mfma_f64)
      return;
    }
    const int TR = kp_ >= 64 ? 16 : 32;
    // tables per launch so the LDS stage fits in 64 KB (MFMA path: its register budget)
    const bool mg = mfma_gram(L) && (uint64_t)Rp * 128 < 0xffffff00ull;  // buffer-load offsets are 32-bit
    const int lmax = mg ? GRAM_LMAX
                                  : std::max<int>(1, (int)((64 * 1024 / rs - (size_t)TR * kp_ - TR) / ((size_t)TR * kp_)));
    int l0 = 0;
    bool first = true;
    do {
      const int Lc = std::min(L - l0, lmax);
      launch_aggr(Rp, Lc, A ? A + l0 : nullptr, B, first ? wv : nullptr, M ? M + (size_t)l0 * kp_ * kp_ : nullptr,
                  first, mg);
      l0 += Lc;
      first = false;
    } while (l0 < L);
  }

  // KP = 64 fp32 Grams on MFMA: gy groups of 4 GW64 tables x nbx row
  // chunks; one launch over all L tables, f32 partials per row chunk summed
  // in chunk order (k_reduce_parts).  ~1,024 blocks of 4 waves.
  bool mfma_gram64(int L, uint64_t Rp) const {
    return std::is_same<real, float>::value && kp_ == 64 && L >= 1 && !no_mfma_ && B_ok(Rp);
  }
  static bool B_ok(uint64_t Rp) { return Rp * 256 < 0xffffff00ull; }  // 32-bit buffer offsets
  void gram64(uint64_t Rp, int L, const real *const *A, const real *B, const real *wv, real *M) {
    if (!M || !B) throw Error(OCFFM_E_STATE, "gram64: Grams and partner table required");
    constexpr int TPB = (BLOCK / 64) * GW64;  // tables per block
    const unsigned gy = (unsigned)((L + 1 + TPB - 1) / TPB);  // L table slots + the sums slot
    const uint64_t nout = (uint64_t)L * 4096 + 129;
    uint64_t nbx = std::max<uint64_t>(1, std::min<uint64_t>((Rp + 63) / 64, std::max<uint64_t>(1, gram64_blocks_ / gy)));
    const uint64_t rpb = ((Rp + nbx - 1) / nbx + 15) / 16 * 16;  // whole rounds of row pairs
    nbx = std::max<uint64_t>(1, (Rp + rpb - 1) / rpb);
    if (gpart64_.n < nbx * nout) gpart64_.alloc(nbx * nout, false);
    const double abytes = (double)Rp * ((L + (B ? 1 : 0)) * 64 + (wv ? 1 : 0)) * sizeof(real);
    const unsigned nwork = (unsigned)(nbx * gy);
    const unsigned grid = xcd_order_ ? (nwork + 7) / 8 * 8 : nwork;  // whole rounds of the 8 XCDs (k_gram_mfma64)
    prof_launch("aggregates", abytes, [&] {
      launch(k_gram_mfma64, grid, BLOCK, 0, Rp, L, (const float *const *)A, (const float *)B,
             (const float *)wv, gpart64_.p, nout, rpb, gy, nwork);
    }, 2.0 * Rp * L * 64 * 64);
    const uint64_t ng = (uint64_t)L * 4096, cnt = ng + 129;
    prof_launch("aggr_reduce", (double)nbx * cnt * 4, [&] {
      launch(k_reduce_parts<real, float>, (unsigned)((cnt + 15) / 16), BLOCK, 0, nbx, nout, (uint64_t)0, cnt,
             (const float *)gpart64_.p, ng, M, sums_.p);
    });
  }

  // KP = 32 fp64 Grams on the f64 matrix cores: the gram64 grid (groups of
  // four table slots, the last slot the sums, x row chunks), double partials
  // summed in chunk order (k_reduce_parts).
  void gram_f64(uint64_t Rp, int L, const real *const *A, const real *B, const real *wv, real *M) {
    constexpr int TPB = BLOCK / 64;
    const unsigned gy = (unsigned)((L + 1 + TPB - 1) / TPB);
    const uint64_t nout = (uint64_t)L * 1024 + 65;
    uint64_t nbx = std::max<uint64_t>(1, std::min<uint64_t>((Rp + 63) / 64, std::max<uint64_t>(1, gram64_blocks_ / gy)));
    const uint64_t rpb = ((Rp + nbx - 1) / nbx + 31) / 32 * 32;  // whole rounds of 2 x 4 x 4 rows
    nbx = std::max<uint64_t>(1, (Rp + rpb - 1) / rpb);
    if (gpartd_.n < nbx * nout) gpartd_.alloc(nbx * nout, false);
    const double abytes = (double)Rp * ((L + 1) * 32 + (wv ? 1 : 0)) * sizeof(real);
    const unsigned nwork = (unsigned)(nbx * gy);
    const unsigned grid = xcd_order_ ? (nwork + 7) / 8 * 8 : nwork;
    prof_launch("aggregates", abytes, [&] {
      launch(k_gram_mfma_f64, grid, BLOCK, 0, Rp, L, (const double *const *)A, (const double *)B,
             (const double *)wv, gpartd_.p, nout, rpb, gy, nwork);
    }, 2.0 * Rp * L * 32 * 32);
    const uint64_t ng = (uint64_t)L * 1024, cnt = ng + 65;
    prof_launch("aggr_reduce", (double)nbx * cnt * 8, [&] {
      launch(k_reduce_parts<real, double>, (unsigned)((cnt + 15) / 16), BLOCK, 0, nbx, nout, (uint64_t)0, cnt,
             (const double *)gpartd_.p, ng, M, sums_.p);
    });
  }

  void launch_aggr(uint64_t Rp, int L, const real *const *A, const real *B, const real *wv, real *M, bool sums,
                   bool mg) {
    const int TR = kp_ >= 64 ? 16 : 32;
    const size_t smem = ((size_t)L * TR * kp_ + (size_t)TR * kp_ + TR) * sizeof(real);
    const uint64_t nout = (uint64_t)L * kp_ * kp_ + 2 * kp_ + 1;
    const int nsub = L * (kp_ / 4) * (kp_ / 4);
    with_kp(kp_, [&](auto K) {
      constexpr int KP = decltype(K)::value;
      constexpr int SPT = KP >= 64 ? 4 : 2;
      const int sub_per_y = SPT * BLOCK;
      const unsigned gy = (unsigned)std::max(1, (nsub + sub_per_y - 1) / sub_per_y);
      uint64_t nbx = std::max<uint64_t>(1, std::min<uint64_t>((Rp + 63) / 64, 512 / gy));
      nbx = std::min<uint64_t>(nbx, std::max<uint64_t>(1, part_.n / nout));
      const uint64_t rpb = (Rp + nbx - 1) / nbx;
      const double abytes = (double)Rp * ((L + (B ? 1 : 0)) * kp_ + (wv ? 1 : 0)) * sizeof(real);
      if (mg) {  // fp32, KP = 32: the Grams on MFMA (kernels.hpp k_gram_mfma32)
        nbx = std::max<uint64_t>(1, std::min<uint64_t>((Rp + 127) / 128, gram_blocks_));
        nbx = std::min<uint64_t>(nbx, std::max<uint64_t>(1, part_.n / nout));
        const uint64_t rpbm = (Rp + nbx - 1) / nbx;
        prof_launch("aggregates", abytes, [&] {
          auto go = [&](auto lc) {
            launch(k_gram_mfma32<decltype(lc)::value>, (unsigned)nbx, BLOCK, 0, Rp, (const float *const *)A,
                   (const float *)B, (const float *)wv, (float *)part_.p, rpbm);
          };
          switch (L) {  // the table count is a compile-time constant of the kernel
            case 1: go(std::integral_constant<int, 1>()); break;
            case 2: go(std::integral_constant<int, 2>()); break;
            case 3: go(std::integral_constant<int, 3>()); break;
            case 4: go(std::integral_constant<int, 4>()); break;
            case 5: go(std::integral_constant<int, 5>()); break;
            case 6: go(std::integral_constant<int, 6>()); break;
            case 7: go(std::integral_constant<int, 7>()); break;
            default: go(std::integral_constant<int, GRAM_LMAX>()); break;
          }
        });
      } else {
        prof_launch("aggregates", abytes, [&] {
          launch(k_gram_part<real, KP, SPT>, dim3((unsigned)nbx, gy), BLOCK, smem, Rp, L, A, B, wv, part_.p,
                                                                                        rpb, sub_per_y);
        });
      }
      // one reduction launch over [grams -> M (real) | sums -> sums_ (double)]
      const uint64_t ng = (uint64_t)L * KP * KP;
      const uint64_t gm = M ? ng : 0, off = M ? 0 : ng, cnt = gm + (sums ? 2 * KP + 1 : 0);
      if (cnt)
        prof_launch("aggr_reduce", (double)nbx * cnt * (mg ? 4 : 8), [&] {
          if (mg)  // f32 partials (k_gram_mfma32)
            launch(k_reduce_parts<real, float>, (unsigned)((cnt + 15) / 16), BLOCK, 0, nbx, nout, off, cnt,
                   (const float *)part_.p, gm, M, sums_.p);
          else
            launch(k_reduce_parts<real>, (unsigned)((cnt + 15) / 16), BLOCK, 0, nbx, nout, off, cnt,
                   (const double *)part_.p, gm, M, sums_.p);
        });
      HIPCHK(hipGetLastError());
    });
  }

  // CSC scatter of h into acc over one field, then the all-reduce (if any).
  // seg: h holds per-segment partials (use the segment CSC of the field).
  void allreduce_dev(real *buf, uint64_t count) {
    if (!comm_.active()) return;
    if (comm_.nccl) {
      NCCLCHK(ncclAllReduce(buf, buf, count, std::is_same<real, double>::value ? ncclDouble : ncclFloat, ncclSum,
                            comm_.nccl, stream_));
    } else {
      HIPCHK(hipMemcpyAsync(stage_, buf, count * sizeof(real), hipMemcpyDeviceToHost, stream_));
      sync();
      if (comm_.host_fn(stage_, count, std::is_same<real, double>::value, comm_.host_user) != 0)
        throw Error(OCFFM_E_COMM, "host all-reduce callback failed");
      HIPCHK(hipMemcpyAsync(buf, stage_, count * sizeof(real), hipMemcpyHostToDevice, stream_));
    }
  }

  void allreduce_dev_d(double *buf, uint64_t count) {
    if (!comm_.active()) return;
    if (comm_.nccl) {
      NCCLCHK(ncclAllReduce(buf, buf, count, ncclDouble, ncclSum, comm_.nccl, stream_));
    } else {
      if (count > DSTAGE) throw Error(OCFFM_E_ARG, "allreduce_dev_d: too many values");
      HIPCHK(hipMemcpyAsync(dstage_, buf, count * sizeof(double), hipMemcpyDeviceToHost, stream_));
      sync();
      if (comm_.host_fn(dstage_, count, 1, comm_.host_user) != 0)
        throw Error(OCFFM_E_COMM, "host all-reduce callback failed");
      HIPCHK(hipMemcpyAsync(buf, dstage_, count * sizeof(double), hipMemcpyHostToDevice, stream_));
    }
  }

  // Make the owned fields' tables whole on every rank (each rank keeps only
  // its own feature rows current): zero the others, sum over the ranks.
  void sync_owned() {
    if (!owned_stale_) return;
    owned_stale_ = false;
    for (uint32_t f1 = 0; f1 < f_; f1++)
      for (uint32_t f2 = f1; f2 < f_; f2++) {
        const uint32_t b12 = block_index(f1, f2, f_);
        if (!blocks_[b12].used) continue;
        for (int t = 0; t < 2; t++) {
          const uint32_t fl = t == 0 ? f1 : f2;
          DevField<real> &F = *side(fl).F[fidx(fl)];
          if (!F.excl) continue;
          real *T = t == 0 ? W_[b12].p : H_[b12].p;
          with_kp(kp_, [&](auto K) {
            constexpr int KP = decltype(K)::value;
            using Gm = Geo<real, KP>;
            const uint64_t nv = F.D * KP / Gm::VE;
            launch(k_mask_rows<real>, grid_for(nv, BLOCK, 2048), BLOCK, 0, nv, T, F.own.p, (uint32_t)Gm::LPR);
          });
          allreduce_dev(T, F.D * kp_);
        }
      }
    sync();
  }

  void allreduce_host(double *buf, uint64_t count) {
    if (!comm_.active()) return;
    if (comm_.nccl) {
      DevBuf<double> d;
      d.upload(buf, count);
      NCCLCHK(ncclAllReduce(d.p, d.p, count, ncclDouble, ncclSum, comm_.nccl, stream_));
      HIPCHK(hipMemcpyAsync(buf, d.p, count * sizeof(double), hipMemcpyDeviceToHost, stream_));
      sync();
    } else if (comm_.host_fn(buf, count, 1, comm_.host_user) != 0) {
      throw Error(OCFFM_E_COMM, "host all-reduce callback failed");
    }
  }

  const double *at_double(DevBuf<real> &at, uint64_t mt) {
    at_d_.alloc(std::max<uint64_t>(mt, 1));
    if (mt) {
      std::vector<real> t(mt);
      HIPCHK(hipMemcpyAsync(t.data(), at.p, mt * sizeof(real), hipMemcpyDeviceToHost, stream_));
      sync();
      std::vector<double> d(t.begin(), t.end());
      HIPCHK(hipMemcpy(at_d_.p, d.data(), mt * sizeof(double), hipMemcpyHostToDevice));
    }
    return at_d_.p;
  }

  // ------------------------------------------------------------- halves
  struct HalfCtx {
    uint32_t b12, fl, fo;
    bool cross, user;
    DevSide<real> *own, *partner;
    DevField<real> *F;
    uint64_t D;
    real *W1, *P1, *Q1;
    const real *fw;
  };

  HalfCtx half_ctx(uint32_t f1, uint32_t f2, int which) {
    HalfCtx h;
    h.b12 = block_index(f1, f2, f_);
    if (!blocks_[h.b12].used) throw Error(OCFFM_E_ARG, "block not in the model (--ns)");
    h.fl = which == 0 ? f1 : f2;
    h.fo = which == 0 ? f2 : f1;
    h.user = h.fl < fu_;
    h.cross = (f1 < fu_) != (f2 < fu_);
    h.own = &side(h.fl);
    h.partner = h.cross ? &side(h.fo) : h.own;
    h.F = h.own->F[fidx(h.fl)].get();
    h.D = h.F->D;
    h.W1 = which == 0 ? W_[h.b12].p : H_[h.b12].p;
    h.P1 = which == 0 ? P_[h.b12].p : Q_[h.b12].p;
    h.Q1 = which == 0 ? Q_[h.b12].p : P_[h.b12].p;
    h.fw = prm_.freq ? h.F->freqw.p : nullptr;
    return h;
  }

  // gd_side / gd_cross (ffm.cpp:537-703) -> G, and the CG start vectors.
  void gradient(HalfCtx &h) {
    DevSide<real> &own = *h.own;
    if (!(lazy_ok_ && h.cross)) flush_base();  // this half reads (or updates) the full base
    if (h.cross) ysum_dirty();                   // (entering a block rewrites the stored base)
    with_kp(kp_, [&](auto K) {
      constexpr int KP = decltype(K)::value;
      using Gm = Geo<real, KP>;
      const double rs = sizeof(real);
      if (h.cross) {
        DevSide<real> &ps = *h.partner;
        // partner aggregates: M_c = A_c^T Q1 for every cross block (A_c = partner-side tables)
        aggregates(ps.R, (int)C_, partner_tabs(h), h.Q1, ps.bias.p, M_.p);  // M_c, oQ, bQ
        const size_t msz = (size_t)C_ * KP * KP * sizeof(real);
        const bool lds = msz <= 64 * 1024;
        double bytes = (double)own.R * 8 + (double)own.npos * (4 + rs) + (double)ps.R * KP * rs +
                       (double)C_ * own.R * KP * rs + (double)own.R * rs + (double)own.R * KP * rs;
        DevField<real> &F = *h.F;
        const Fin<real> fin = make_fin(h, 0);
        // block-excluded base: enter this block (store), or read it inside
        const real *cur = nullptr, *drow = nullptr, *dxs = nullptr;
        bool enter = false;
        if (lazy_ok_) {
          cur = h.P1;
          enter = !(excl_.on && excl_.b12 == h.b12);
          if (enter && excl_.on) {  // leave the previous block in the same pass
            drow = h.user ? P_[excl_.b12].p : Q_[excl_.b12].p;  // indexed by this half's rows
            dxs = h.user ? Q_[excl_.b12].p : P_[excl_.b12].p;   // indexed by the partner
          }
          excl_ = ExclBase{true, h.b12};
        }
        // cur / drow are rows of the C tables already counted; entering stores e
        // and gathers the previous block's partner rows
        if (enter) bytes += (double)own.npos * rs + (dxs ? (double)ps.R * KP * rs : 0);
        // inside the block (BM_IN): read the stored value through perm from
        // the orientation the entering pass wrote (no refresh in between)
        const bool via = ytvia_ && cur && !enter && !side_pending_;
        // the item orientation refreshed on the side stream (side_refresh_):
        // the in-block pass reads it in order once the refresh has landed
        if (cur && !enter) side_join();
        // T_i = sum_c P_c[i] M_c on MFMA ahead of the pass (k_rows_T), where
        // the C Grams do not fit the pass's LDS (or OCFFM_TPRE=1)
        const bool tp = tpre(own.R, own.npos);
        if (tp) {
          if constexpr (std::is_same<real, float>::value && (KP == 32 || KP == 64)) {
            const uint64_t nb = (own.R + RowsT<KP>::ROWS - 1) / RowsT<KP>::ROWS;
            prof_launch("rows_T", (double)C_ * own.R * KP * rs + (double)own.R * KP * rs + (double)C_ * KP * KP * rs, [&] {
              launch(k_rows_T<KP>, (unsigned)std::min<uint64_t>(nb, tpre_blocks_), TBLOCK, 0, (uint64_t)own.R, (int)C_,
                     (const float *const *)(tabs_.p + (h.user ? 0 : C_)), (const float *)M_.p, (float *)Tpre_.p);
            }, 2.0 * own.R * C_ * KP * KP);
          }
        }
        auto go2 = [&](auto ml, auto bm) {
          constexpr bool ML = decltype(ml)::value;
          constexpr int BM = decltype(bm)::value;
          auto go3 = [&](auto tpc) {
            constexpr bool TP = decltype(tpc)::value;
            // (with T on the matrix cores the block also holds its T tile)
            constexpr bool TM = ML && !TP && TMma<real, KP>::OK;
            // one resident wave of blocks (OCFFM_GD_FILL): the grid-stride
            // loop then has no partial last wave of blocks
            const size_t gsm = TP ? 0 : (ML ? msz + (TM ? TMma<real, KP>::tile_bytes() : 0) : 0);
            unsigned grid = grid_for(own.nseg, 4 * Gm::NSG, gd_blocks_);
            if (gd_fill_) grid = std::min(grid, resident(k_gd_cross_seg<real, KP, ML, BM, TP>, gsm));
            launch(k_gd_cross_seg<real, KP, ML, BM, TP>, grid, BLOCK, gsm, own.nseg, own.segs.p, own.ycol.p, own.yt.p, h.Q1, (int)C_,
                (const real *const *)(tabs_.p + (h.user ? 0 : C_)), M_.p, sums_.p, own.bias.p, h.partner->bias.p, w_,
                r_, h_.p, (uint64_t)h.partner->R, cur, drow, dxs, (const uint32_t *)own.perm.p,
                TP ? (const real *)Tpre_.p : (const real *)nullptr,
                via ? (const real *)h.partner->yt.p : (const real *)nullptr, sord(own));
          };
          if constexpr (std::is_same<real, float>::value && (KP == 32 || KP == 64) && !ML) {
            if (tp) {
              go3(std::true_type());
              return;
            }
          }
          go3(std::false_type());
        };
        auto go = [&](auto ml) {
          if (!cur) go2(ml, std::integral_constant<int, BM_FULL>());
          else if (enter) go2(ml, std::integral_constant<int, BM_ENTER>());
          else go2(ml, std::integral_constant<int, BM_IN>());
        };
        if (tp) bytes += (double)own.R * KP * rs - (double)C_ * own.R * KP * rs;  // one T row instead of C table rows
        if constexpr (OCFFM_GD_PROBE) {  // the gathers alone (kernels.hpp PRB), timed as their own family
          auto probe = [&](auto bm) {
            constexpr int BM = decltype(bm)::value;
            launch(k_gd_cross_seg<real, KP, false, BM, false, true>, grid_for(own.nseg, 4 * Gm::NSG, gd_blocks_), BLOCK,
                   0, own.nseg, own.segs.p, own.ycol.p, own.yt.p, h.Q1, (int)C_,
                   (const real *const *)(tabs_.p + (h.user ? 0 : C_)), M_.p, sums_.p, own.bias.p, h.partner->bias.p, w_,
                   r_, h_.p, (uint64_t)h.partner->R, cur, drow, dxs, (const uint32_t *)own.perm.p,
                   (const real *)nullptr, via ? (const real *)h.partner->yt.p : (const real *)nullptr, sord(own));
          };
          prof_launch("gd_probe", bytes, [&] {
            if (!cur) probe(std::integral_constant<int, BM_FULL>());
            else if (enter) probe(std::integral_constant<int, BM_ENTER>());
            else probe(std::integral_constant<int, BM_IN>());
          });
        }
        prof_launch("gd_cross_row", bytes, [&] {
          if (lds && !tp) go(std::true_type());
          else go(std::false_type());
        });
        // the other orientation: refreshed here, or on the side stream while
        // this half's CG runs (side_refresh_: nothing reads it before the
        // block's second half), or read through perm by the block's second
        // half (ytvia_; flush_base refreshes it after the loop)
        if (enter && side_refresh_ && h.partner->npos) {
          if (!side_) {
            HIPCHK(hipStreamCreateWithFlags(&side_, hipStreamNonBlocking));
            HIPCHK(hipEventCreateWithFlags(&side_ev_[0], hipEventDisableTiming));
            HIPCHK(hipEventCreateWithFlags(&side_ev_[1], hipEventDisableTiming));
          }
          HIPCHK(hipEventRecord(side_ev_[0], stream_));
          HIPCHK(hipStreamWaitEvent(side_, side_ev_[0], 0));
          std::swap(stream_, side_);  // launch() and the profiler's events go to the stream in stream_
          refresh_other(own, *h.partner);
          std::swap(stream_, side_);
          HIPCHK(hipEventRecord(side_ev_[1], side_));
          side_pending_ = true;
        } else if (enter && !ytvia_) {
          refresh_other(own, *h.partner);
        }
        // QTQ for CG = M of this block (M_ is not rewritten before the half ends)
        const uint32_t c0 = cross_slot(std::min(h.fl, h.fo), std::max(h.fl, h.fo));
        qtq_ = M_.p + (size_t)c0 * KP * KP;
      } else {
        DevSide<real> &other = h.user ? V_ : U_;  // bsum_: sum of the other side's bias (b_sum, ffm.cpp:551)
        const double n1 = (double)other.R;
        // (with the segment sums: one sum per segment instead of the positives)
        const double bytes = (double)own.R * 8 + (ysum_on_ ? (double)own.nseg * (16 + rs) : (double)own.npos * rs) +
                             (double)own.R * KP * rs * 2 + (double)own.R * rs * 2;
        DevField<real> &F = *h.F;
        const Fin<real> fin = make_fin(h, 0);
        seg_ysum(h);
        const real *ysum = ysum_on_ ? (const real *)ysum_.p : nullptr;
        prof_launch("gd_side_row", bytes, [&] {
          launch(k_gd_side_seg<real, KP>, mfill(k_gd_side_seg<real, KP>, grid_for(own.nseg, 4 * Gm::NSG)), BLOCK, 0, own.nseg, own.segs.p, own.ycol.p,
                 own.yt.p, h.Q1, own.bias.p, other.bias.p, own.s.p, bsum_.p + (h.user ? 1 : 0), n1, w_, r_, h_.p,
                 (uint64_t)other.R, ysum);
        });
      }
      feature_pass(h, 0, true);
    });
  }

  // segment sums of base + partner bias of a side half's rows: once per
  // side phase (k_seg_ysum)
  // rows: also the per-row totals (k_row_ysum, the fused side half's input)
  void seg_ysum(const HalfCtx &h, bool rows = false) {
    DevSide<real> &own = *h.own, &other = h.user ? V_ : U_;
    const int ys = h.user ? 0 : 1;
    if (!ysum_on_ || !own.nseg) return;
    if (ysum_ok_[ys]) {
      if (rows && !yrow_ok_[ys]) row_ysum(own, ys);
      return;
    }
    with_kp(kp_, [&](auto K) {
      constexpr int KP = decltype(K)::value;
      using Gm = Geo<real, KP>;
      const double rs = sizeof(real);
      prof_launch("seg_ysum", (double)own.npos * (4 + 2 * rs) + (double)own.nseg * (16 + rs), [&] {
        launch(k_seg_ysum<real, KP>, grid_for(own.nseg, 4 * Gm::NSG), BLOCK, 0, own.nseg, own.segs.p, own.ycol.p,
               (const real *)own.yt.p, (const real *)other.bias.p, (uint64_t)other.R, ysum_.p);
      });
    });
    ysum_ok_[ys] = true;
    ysum_ok_[1 - ys] = false;  // one buffer for both sides: the other side's sums are gone
    yrow_ok_[0] = yrow_ok_[1] = false;
    if (rows) row_ysum(own, ys);
  }
  void row_ysum(DevSide<real> &own, int ys) {
    prof_launch("row_ysum", (double)own.R * 8 + (double)own.nseg * sizeof(real) + (double)own.R * sizeof(real), [&] {
      launch(k_row_ysum<real>, grid_for(own.R, BLOCK / 64, 8192), BLOCK, 0, (uint64_t)own.R, (const uint32_t *)own.segptr.p,
             (const real *)ysum_.p, yrow_.p);
    });
    yrow_ok_[ys] = true;
    yrow_ok_[1 - ys] = false;
  }

  // subgroups per wave of this problem's row geometry (kernels.hpp: Geo)
  int nsg() const { return 64 / std::max<int>(1, (int)(kp_ / VT<real>::N)); }

  // Restore the full base from the block-excluded y~:
  // base_ij = e_ij + <P_b[i], Q_b[j]> - a_i - b_j in the user orientation
  // (k_update_cross_seg with XS = P_b), then the refresh of the other one.
  // the main stream waits for a pending side-stream refresh (side_refresh_)
  void side_join() {
    if (!side_pending_) return;
    HIPCHK(hipStreamWaitEvent(stream_, side_ev_[1], 0));
    side_pending_ = false;
  }
  void flush_base() {
    side_join();
    if (!excl_.on) return;
    ysum_dirty();
    excl_.on = false;
    const Block &b = blocks_[excl_.b12];
    DevSide<real> &own = U_, &other = V_;
    DevField<real> &F = *own.F[fidx(b.f1)];
    const real *P1 = P_[excl_.b12].p, *Q1 = Q_[excl_.b12].p;
    if (own.R == 0) return;
    with_kp(kp_, [&](auto K) {
      constexpr int KP = decltype(K)::value;
      using Gm = Geo<real, KP>;
      const double rs = sizeof(real);
      prof_launch("flush_base", (double)own.R * (KP + 1) * rs + (double)own.npos * (4 + 2 * rs) + (double)other.R * (KP + 1) * rs,
                  [&] {
                    launch(k_update_cross_seg<real, KP>, grid_for(own.nseg, 4 * Gm::NSG), BLOCK, 0, own.nseg,
                           own.segs.p, F.xptr.p, F.xidx.p, F.xval.p, (const real *)S_.p, (real *)nullptr, own.ycol.p,
                           own.yt.p, Q1, (uint64_t)other.R, F.segd.p, F.segx.p,
                           (real *)nullptr, (const real *)nullptr, (const CgState *)st_.p, P1,
                           (const real *)U_.bias.p, (const real *)V_.bias.p, (const int *)nullptr);
                  });
    });
    refresh_other(own, other);
  }

  // other.yt (base in the other orientation) := own.yt through other.perm.
  void refresh_other(DevSide<real> &own, DevSide<real> &other, const int *skip = nullptr) {
    ysum_dirty();
    if (!other.npos) return;
    prof_launch("refresh_base", (double)other.npos * (4 + 2 * sizeof(real)), [&] {
      launch(k_gather_pos<real>, grid_for((other.npos + 3) / 4, BLOCK, 4096), BLOCK, 0, (uint64_t)other.npos,
             other.perm.p, own.yt.p, other.yt.p, skip);
    });
  }

  Fin<real> make_fin(const HalfCtx &h, int it) {
    Fin<real> f;
    f.fw = h.fw;
    f.lam = lam_;
    f.W = h.W1;
    f.G = want_g_ ? G_.p : nullptr;
    f.S = S_.p;
    f.P = Vd_.p;
    f.R = Rv_.p;
    f.Hp = Hv_.p;
    f.acc = acc_.p;
    f.cnt = h.F->cnt.p;
    f.st = st_.p;
    f.part = part_.p;
    f.tick = tick_.p;
    f.run_host = run_host_dev_;
    f.it = it;
    f.dots = h.F->excl ? dots_.p : nullptr;
    f.xsq = nullptr;
    f.tw = w_;
    f.hdots = nullptr;
    f.nhd = 0;
    f.exact_r2 = exact_r2(h) ? 1 : 0;
    return f;
  }
  // Gram build chunks of a list of position ranges (one Gram per range):
  // ~HOT_CHUNK_MAX positions per chunk, at most 64 chunks per Gram; the
  // chunks of a multi-chunk Gram write consecutive partial slots, summed in
  // slot order by k_hot_slot_sum (sums: {gram, nparts, first slot}).
  static void gram_chunks(const std::vector<std::pair<uint64_t, uint64_t>> &ranges, std::vector<Job> &chunks,
                          std::vector<Job> &sums, uint64_t &slots, uint64_t cmax = HOT_CHUNK_MAX,
                          uint64_t npmax = 64) {
    for (uint64_t g = 0; g < ranges.size(); g++) {
      const uint64_t b = ranges[g].first, e = ranges[g].second;
      const uint64_t np = std::max<uint64_t>(1, std::min<uint64_t>(npmax, (e - b + cmax - 1) / cmax));
      const uint64_t len = (e - b + np - 1) / std::max<uint64_t>(np, 1);
      for (uint64_t q = 0; q < np; q++)
        chunks.push_back(Job{(uint32_t)g, (uint32_t)np, np > 1 ? (uint32_t)(slots + q) : 0u, (uint32_t)q,
                             (int64_t)std::min(e, b + q * len), (int64_t)std::min(e, b + (q + 1) * len)});
      if (np > 1) {
        sums.push_back(Job{(uint32_t)g, (uint32_t)np, (uint32_t)slots, 0u, 0, 0});
        slots += np;
      }
    }
    if (slots > 0xffffffffull) throw Error(OCFFM_E_DATA, "too many Gram partial slots");
  }

  // Hot rows of a side (rows with >= hot_min_ positives): Gram slots, the
  // build chunks, and every segment's slot (k_hot_seg).
  void hot_setup(DevSide<real> &s) {
    if (!s.R || !s.npos) return;
    std::vector<int64_t> yp(s.R + 1);
    HIPCHK(hipMemcpy(yp.data(), s.yptr.p, yp.size() * sizeof(int64_t), hipMemcpyDeviceToHost));
    std::vector<uint32_t> row_slot(s.R, HOT_NONE);
    std::vector<std::pair<uint64_t, uint64_t>> ranges;
    uint64_t nhot = 0, slots = 0, hpos = 0;
    s.xf_ok = false;
    for (uint64_t i = 0; i < s.R; i++) {
      const uint64_t b = (uint64_t)yp[i], e = (uint64_t)yp[i + 1];
      if (e - b < hot_min_) continue;
      row_slot[i] = (uint32_t)nhot;
      ranges.emplace_back(b, e);
      hpos += e - b;
      nhot++;
    }
    s.xf_ok = nhot == 0;
    if (!nhot) return;
    if (!hot_env_ && 2 * hpos > s.npos) return;  // (k_hv_cross_id's gate: the Grams would replace most gathers)
    s.xf_ok = true;
    std::vector<Job> chunks, sums;
    gram_chunks(ranges, chunks, sums, slots);
    s.nhot = nhot;
    s.hslots = slots;
    s.hpos = hpos;
    s.hchunks.upload(chunks);
    s.hsums.upload(sums);
    DevBuf<uint32_t> rs;
    rs.upload(row_slot);
    s.hot_row.upload(row_slot);
    s.hot_seg.alloc(s.nseg);
    launch(k_hot_seg, (unsigned)((s.nseg + BLOCK - 1) / BLOCK), BLOCK, 0, (uint64_t)s.nseg, (const Seg *)s.segs.p,
           (const uint32_t *)rs.p, s.hot_seg.p);
    sync();
  }
  // A cross half reads hot rows' Grams when its previous CG count was at
  // least hot_steps_ (the build is one MFMA pass over the hot positives;
  // each step then saves their gathers) and it is not on column Grams.
  bool hot(const HalfCtx &h) const {
    return hot_env_ && hot_now_ && h.cross && h.own->nhot > 0 && hotG_.p && !ccg_now_;
  }

  // The hot rows' Grams G_i = sum_{j in Omega_i} q_j q_j^T over this half's
  // partner table (fixed over the half's CG steps).
  void hot_grams(const HalfCtx &h, bool force = false) {
    if (!(force ? h.own->nhot > 0 && hotG_.p : hot(h))) return;
    DevSide<real> &own = *h.own;
    with_kp(kp_, [&](auto K) {
      constexpr int KP = decltype(K)::value;
      const double rs = sizeof(real);
      const double bytes = (double)own.hpos * (4 + KP * rs) + (double)own.nhot * KP * KP * rs +
                           (double)own.hslots * KP * KP * rs * 2;
      prof_launch("hot_gram", bytes, [&] {
        bool done = false;
        if constexpr (std::is_same<real, float>::value && (KP == 32 || KP == 64)) {
          if (!no_mfma_) {
            launch(k_hot_gram_mfma<KP>, (unsigned)((own.hchunks.n + 3) / 4), BLOCK, 0, (uint64_t)own.hchunks.n,
                   (const Job *)own.hchunks.p, (const uint32_t *)own.ycol.p, (const float *)nullptr, (const float *)h.Q1,
                   (uint64_t)h.partner->R, (float *)hotG_.p, (float *)hotP_.p, (const float *)nullptr,
                   (const float *)nullptr, 0.0f);
            done = true;
          }
        }
        if constexpr (std::is_same<real, double>::value && KP == 32) {
          if (!no_mfma_) {
            launch(k_hot_gram_mfma_f64, (unsigned)((own.hchunks.n + 3) / 4), BLOCK, 0, (uint64_t)own.hchunks.n,
                   (const Job *)own.hchunks.p, (const uint32_t *)own.ycol.p, (const double *)nullptr,
                   (const double *)h.Q1, (uint64_t)h.partner->R, (double *)hotG_.p, (double *)hotP_.p,
                   (const double *)nullptr, (const double *)nullptr, 0.0);
            done = true;
          }
        }
        if (!done)
          launch(k_hot_gram<real, KP>, (unsigned)own.hchunks.n, BLOCK, 0, (const Job *)own.hchunks.p,
                 (const uint32_t *)own.ycol.p, (const real *)nullptr, (const real *)h.Q1, hotG_.p, hotP_.p);
        if (own.hsums.n)
          launch(k_hot_slot_sum<real, KP>, dim3((unsigned)own.hsums.n, (KP * KP + BLOCK - 1) / BLOCK), BLOCK, 0,
                 (const Job *)own.hsums.p, (const real *)hotP_.p, hotG_.p);
      }, 2.0 * own.hpos * KP * KP);
    });
  }

  // Gram chunks of a one-node-per-row field (build_csc's column order): each
  // column in chunks of at most cgram_rows rows (one LDS stage: larger
  // OCFFM_CGRAM_CHUNK values are capped there); empty columns get one empty
  // chunk so that their G_c is stored as zero.  The chunks of a multi-chunk
  // column get consecutive partial slots (Job.slot) and their index in the
  // column (Job.flags).  The Gram buffers are allocated by col_grams.
  void col_gram_chunks(DevField<real> &F, const std::vector<int64_t> &cptr) {
    const uint64_t ch = cgram32() ? (uint64_t)CGRAM32_ROWS
                                  : std::min<uint64_t>(cgram_chunk_, (uint64_t)cgram_rows((int)kp_, (int)sizeof(real)));
    std::vector<Job> chunks, sums;
    uint64_t slots = 0;
    for (uint64_t d = 0; d < F.D; d++) {
      const uint64_t b = cptr[d], e = cptr[d + 1];
      const uint32_t np = (uint32_t)std::max<uint64_t>(1, (e - b + ch - 1) / ch);
      for (uint32_t q = 0; q < np; q++)
        chunks.push_back(Job{(uint32_t)d, np, np > 1 ? (uint32_t)(slots + q) : 0u, q,
                             (int64_t)std::min(e, b + q * ch), (int64_t)std::min(e, b + (q + 1) * ch)});
      if (np > 1) sums.push_back(Job{(uint32_t)d, np, (uint32_t)slots, 0u, 0, 0});
      if (np > 1) slots += np;
    }
    if (slots > 0xffffffffull) throw Error(OCFFM_E_DATA, "too many Gram chunks in one field");
    F.gchunks.upload(chunks);
    if (cgram32() && !sums.empty()) F.gsums.upload(sums);
    F.gslots = slots;
  }

  // KP = 32: the Grams are built on the matrix cores (kernels.hpp
  // k_col_gram32, fp32; k_col_gram_f64, fp64)
  bool cgram32() const { return kp_ == 32 && !no_mfma_; }

  // Side half whose CG steps run on per-column Grams (several ranks: each
  // builds its partial Grams, and every CG step all-reduces G_c p_c).
  bool cgram(const HalfCtx &h) const { return h.cross ? ccg_now_ : h.F->gchunks.n > 0; }
  const real *gram_of(const HalfCtx &h) const { return h.cross ? ccgG_.p : h.F->gram.p; }

  // ---- per-column cross Grams.  A cross half over a one-node-per-row field
  // has, per column c (rows i with idx_i = c, value x_i),
  //   (X^T h)_c = sum_i x_i h_i = C_c p_c,
  //   C_c = (1 - w) sum_i x_i^2 sum_{j in Omega_i} q_j q_j^T + w (sum_i x_i^2) QTQ
  // (hs_cross, ffm.cpp:706-742, summed per column): with few columns (an
  // artist or genre field) a CG step is D k x k products (k_hv_cgram)
  // instead of a pass gathering every positive's partner row plus a
  // feature pass.  Built once per half (the partner table is fixed there)
  // where the previous epoch's CG count says it pays (OCFFM_CCG: 0 off,
  // 1 when the half ran >= 3 steps, 2 always).
  // A field whose cross halves can run on column Grams: one node per row,
  // not id-like (a column per row: the per-row Gram), columns few enough
  // that one Gram step reads less than a row pass gathers (D KP <= (P + 2R)
  // / 2: positives' partner rows plus the h round trip), the Grams within
  // 8 GB.  The positions in column order are set up once (ccg_setup).
  bool ccg_pred(uint64_t D, bool one, bool idlike, uint64_t npos, uint64_t R) const {
    const bool mfma = kp_ == 32 || (kp_ == 64 && std::is_same<real, float>::value);
    return ccg_mode_ != 0 && C_ > 0 && one && !idlike && npos > 0 && R > 0 && (ccg_mode_ == 2 || mfma) &&
           (double)D * kp_ * kp_ * sizeof(real) <= 8.0 * (1ull << 30) &&
           (ccg_mode_ == 2 || 2.0 * D * kp_ <= (double)npos + 2.0 * R);
  }
  bool ccg_field(const DevField<real> &F, const DevSide<real> &own) const {
    return ccg_pred(F.D, F.one, F.idlike, own.npos, own.R);
  }
  // On several ranks: the field qualifies on every rank's shard, which each
  // rank works out from the whole data set it holds (no communication), so
  // all ranks take the same path and meet in the same all-reduces.  The item
  // side's rows (all items) are the same on every rank; its positives and
  // the user side's rows are the shard's.
  bool ccg_field_all(const DevField<real> &F, const DevSide<real> &own, bool user, uint32_t fi,
                     const HostData &U) {
    if (!ccg_field(F, own)) return false;
    if (comm_.nranks == 1) return true;
    const uint64_t N = (uint64_t)comm_.nranks;
    if (user && shard_facts_.empty()) shard_facts_ = shard_field_facts(U, N);
    for (uint64_t q = 0; q < N; q++) {
      const uint64_t u0 = U.m * q / N, u1 = U.m * (q + 1) / N;
      const uint64_t npos = U.yptr[u1] - U.yptr[u0];
      bool one = F.one, idl = F.idlike;
      if (user) {
        const uint8_t fact = shard_facts_[q * U_.F.size() + fi];
        one = fact & 1;
        idl = (fact & 2) != 0;
      }
      if (!ccg_pred(F.D, one, idl, npos, user ? u1 - u0 : own.R)) return false;
    }
    return true;
  }
  // Per (user shard q, user field f), in ONE pass over the raw nodes: bit 0
  // = every row of the shard has exactly one node of f (and the shard has
  // rows), bit 1 = also no feature of f twice in the shard with D_f = its
  // rows (an id-like field on that shard).  O(nnz) for all fields together.
  std::vector<uint8_t> shard_field_facts(const HostData &U, uint64_t N) const {
    const Rows &raw = U.raw;
    const uint32_t nf = (uint32_t)U_.F.size();
    std::vector<uint8_t> facts(N * nf, 0);
    std::vector<uint32_t> cnt(nf, 0);
    std::vector<uint64_t> ones(nf, 0);
    std::vector<std::vector<uint8_t>> seen(nf);
    for (uint64_t q = 0; q < N; q++) {
      const uint64_t u0 = U.m * q / N, u1 = U.m * (q + 1) / N;
      std::vector<uint8_t> idl(nf, 0);
      for (uint32_t f = 0; f < nf; f++) {
        const uint64_t D = U_.F[f]->D;
        idl[f] = D == u1 - u0 && u1 > u0;
        seen[f].assign(idl[f] ? D : 0, 0);
        ones[f] = 0;
      }
      // per row: count each field's nodes, then visit the nodes again (each
      // field once: its count is reset on the first visit)
      for (uint64_t i = u0; i < u1; i++) {
        const uint64_t b = raw.xptr[i], e = raw.xptr[i + 1];
        for (uint64_t p = b; p < e; p++)
          if (raw.fid[p] < nf) cnt[raw.fid[p]]++;
        for (uint64_t p = b; p < e; p++) {
          const uint32_t f = raw.fid[p];
          if (f >= nf || cnt[f] == 0) continue;
          if (cnt[f] == 1) {
            ones[f]++;
            const uint64_t x = raw.idx[p];
            if (idl[f]) {
              if (x < seen[f].size() && !seen[f][x]) seen[f][x] = 1;
              else idl[f] = 0;
            }
          }
          cnt[f] = 0;
        }
      }
      for (uint32_t f = 0; f < nf; f++) {
        const bool one = u1 > u0 && ones[f] == u1 - u0;
        facts[q * nf + f] = (uint8_t)((one ? 1 : 0) | ((one && idl[f]) ? 2 : 0));
      }
    }
    return facts;
  }
  std::vector<uint8_t> shard_facts_;  // shard_field_facts, computed on first use
  bool ccg_eligible(const HalfCtx &h) const { return h.cross && h.F->ccg_ready; }
  void ccg_setup(DevField<real> &F, DevSide<real> &own) {
    if (F.ccg_ready) return;
    const uint64_t P = own.npos;
    dev::Builder B(stream_);
    DevBuf<uint32_t> rid, key, kout, perm;
    rid.alloc(P, false);
    key.alloc(P, false);
    kout.alloc(P, false);
    perm.alloc(P, false);
    B.rowid(own.yptr.p, own.R, rid.p);  // the row of every position
    launch(k_pos_colkey, (unsigned)((P + BLOCK - 1) / BLOCK), BLOCK, 0, P, (const uint32_t *)rid.p,
           (const uint32_t *)F.xidx.p, key.p);
    B.sort_positions(key.p, kout.p, perm.p, P, F.D);  // stable: rows in order inside a column
    DevBuf<int64_t> cptr;
    cptr.alloc(F.D + 1, false);
    B.bounds(kout.p, P, F.D, cptr.p);
    F.cpos.alloc(P, false);
    F.cw.alloc(P, false);
    launch(k_ccg_gather<real>, (unsigned)((P + BLOCK - 1) / BLOCK), BLOCK, 0, P, (const uint32_t *)perm.p,
           (const uint32_t *)rid.p, (const uint32_t *)own.ycol.p, (const real *)F.xval.p, w_, F.cpos.p, F.cw.p);
    std::vector<int64_t> cp(F.D + 1);
    HIPCHK(hipMemcpyAsync(cp.data(), cptr.p, cp.size() * sizeof(int64_t), hipMemcpyDeviceToHost, stream_));
    sync();
    std::vector<std::pair<uint64_t, uint64_t>> ranges(F.D);
    for (uint64_t c = 0; c < F.D; c++) ranges[c] = {(uint64_t)cp[c], (uint64_t)cp[c + 1]};
    std::vector<Job> chunks, sums;
    uint64_t slots = 0;
    // one chunk per column where the columns alone fill the chip (artist:
    // 5,000 columns of ~420 positions: no partial slots to sum); a Pareto
    // head column (millions of positions) in up to 256 chunks
    gram_chunks(ranges, chunks, sums, slots, F.D >= 2048 ? 1024 : HOT_CHUNK_MAX, 256);
    F.cchunks.upload(chunks);
    F.csums.upload(sums);
    F.cslots = slots;
    F.cnpos = P;
    if (F.D * kp_ * kp_ > ccgG_.n) ccgG_.alloc(F.D * kp_ * kp_, false);
    if (slots * kp_ * kp_ > ccgP_.n) ccgP_.alloc(slots * kp_ * kp_, false);
    F.ccg_ready = true;
  }
  // C_c of every column for this half (needs qtq_: gradient() sets it)
  void ccg_build(const HalfCtx &h) {
    DevField<real> &F = *h.F;
    with_kp(kp_, [&](auto K) {
      constexpr int KP = decltype(K)::value;
      const double rs = sizeof(real);
      const double bytes = (double)F.cnpos * (8 + KP * rs) + (double)F.D * KP * KP * rs * 3 +
                           (double)F.cslots * KP * KP * rs * 2;
      prof_launch("ccg_build", bytes, [&] {
        bool done = false;
        if constexpr (std::is_same<real, float>::value && (KP == 32 || KP == 64)) {
          if (!no_mfma_) {
            launch(k_hot_gram_mfma<KP>, (unsigned)((F.cchunks.n + 3) / 4), BLOCK, 0, (uint64_t)F.cchunks.n,
                   (const Job *)F.cchunks.p, (const uint32_t *)F.cpos.p, (const float *)F.cw.p,
                   (const float *)h.Q1, (uint64_t)h.partner->R, (float *)ccgG_.p, (float *)ccgP_.p,
                   (const float *)F.xsq.p, (const float *)qtq_, (float)w_);  // tau folded in
            done = true;
          }
        }
        if constexpr (std::is_same<real, double>::value && KP == 32) {
          if (!no_mfma_) {
            launch(k_hot_gram_mfma_f64, (unsigned)((F.cchunks.n + 3) / 4), BLOCK, 0, (uint64_t)F.cchunks.n,
                   (const Job *)F.cchunks.p, (const uint32_t *)F.cpos.p, (const double *)F.cw.p,
                   (const double *)h.Q1, (uint64_t)h.partner->R, (double *)ccgG_.p, (double *)ccgP_.p,
                   (const double *)F.xsq.p, (const double *)qtq_, w_);  // tau folded in
            done = true;
          }
        }
        if (!done)
          launch(k_hot_gram<real, KP>, (unsigned)F.cchunks.n, BLOCK, 0, (const Job *)F.cchunks.p,
                 (const uint32_t *)F.cpos.p, (const real *)F.cw.p, (const real *)h.Q1, ccgG_.p, ccgP_.p);
        if (F.csums.n)
          launch(k_hot_slot_sum<real, KP>, dim3((unsigned)F.csums.n, (KP * KP + BLOCK - 1) / BLOCK), BLOCK, 0,
                 (const Job *)F.csums.p, (const real *)ccgP_.p, ccgG_.p);
        if (!done)
          launch(k_gram_add_tau<real, KP>, grid_for(F.D * KP * KP, BLOCK, 2048), BLOCK, 0, (uint64_t)F.D, ccgG_.p,
                 (const real *)F.xsq.p, (const real *)qtq_, w_);
      }, 2.0 * F.cnpos * KP * KP);
    });
  }

  // Does a side half over a one-node-per-row field (R rows, D columns) pay
  // for its Grams?  Estimated time (us) of a half of `c` CG steps, from the
  // kkbox-shape measurements: ~4 TB/s effective for the
  // streamed bytes, ~4.1e6 rank-1 MACs per us for the build, dispatch
  // floors of 5 us (one launch) and 10 us (row pass + feature pass).
  //   Gram: build + c (D k^2 + 9 D k) s     rows: c (4 R k + 9 D k) s
  // OCFFM_CGRAM=2 takes the Gram path wherever the structure allows.
  bool cgram_pays(uint64_t R, uint64_t D) const {
    if (cgram_mode_ == 2) return true;
    const double k = (double)kp_, s = sizeof(real), bw = 4e6, c = 4;
    const double build = 5 + (double)R * k * k / 4.1e6 + ((double)R * k + (double)D * k * k) * s / bw;
    const double gstep = 5 + ((double)D * k * k + 9.0 * D * k) * s / bw;
    const double rstep = 10 + (4.0 * R * k + 9.0 * D * k) * s / bw;
    return build + c * gstep <= c * rstep;
  }

  // ---- pair Grams (kernels.hpp k_pg_step; OCFFM_PGRAM: 0 off, 1 where
  // the gate below passes, 2 wherever the structure allows)
  // (default off: measured 5.37 -> 5.63 ms per kkbox epoch against the
  // column-block feature pass)
  int pgram_mode_ = std::getenv("OCFFM_PGRAM") ? std::atoi(std::getenv("OCFFM_PGRAM")) : 0;
  static constexpr uint64_t PG_FIN1 = 1024;  // k_pg_step finalises in its last block up to this many features
  DevBuf<real> pgt_;                          // its per-(feature, block) partial slots
  bool pgram(const HalfCtx &h) const { return !h.cross && h.F->pg; }
  // The field's pairs, entries and CSCs from its rows (host; once).  Gate:
  // several nodes per row (one node: the per-column Grams), not owned, at
  // most PG_FIN1 features (the single-launch step), and (mode 1) a CG step reading the pair Grams
  // (npair k^2) costs at most what the row pass reads for the partner rows
  // times 8 (npair k <= 8 R): the kkbox context field has ~7,200 pairs over
  // 30,755 rows (0.93 of the bound).
  void pgram_setup(DevField<real> &F, DevSide<real> &sd) {
    const uint64_t R = sd.R;
    if (F.one || F.idlike || F.excl || R == 0 || F.nnz == 0 || F.D == 0) return;
    if (pgram_mode_ == 1 && F.D > PG_FIN1) return;
    std::vector<int64_t> xp(R + 1);
    std::vector<uint32_t> xi(F.nnz);
    std::vector<real> xv(F.nnz);
    HIPCHK(hipMemcpy(xp.data(), F.xptr.p, xp.size() * sizeof(int64_t), hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(xi.data(), F.xidx.p, xi.size() * sizeof(uint32_t), hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(xv.data(), F.xval.p, xv.size() * sizeof(real), hipMemcpyDeviceToHost));
    struct Ent {
      uint64_t key;
      uint32_t row;
      double w;
    };
    std::vector<Ent> ent;
    std::vector<std::pair<uint32_t, double>> nd;
    for (uint64_t i = 0; i < R; i++) {
      nd.clear();  // the row's vector X_i: nodes by feature, repeats summed
      for (int64_t q = xp[i]; q < xp[i + 1]; q++) nd.push_back({xi[q], (double)xv[q]});
      std::sort(nd.begin(), nd.end(), [](const auto &x, const auto &y) { return x.first < y.first; });
      size_t u = 0;
      for (size_t q = 0; q < nd.size(); q++) {
        if (u && nd[u - 1].first == nd[q].first) nd[u - 1].second += nd[q].second;
        else nd[u++] = nd[q];
      }
      nd.resize(u);
      for (size_t x = 0; x < u; x++)
        for (size_t y = x; y < u; y++)
          ent.push_back(Ent{(uint64_t)nd[x].first * F.D + nd[y].first, (uint32_t)i, nd[x].second * nd[y].second});
    }
    std::stable_sort(ent.begin(), ent.end(), [](const Ent &x, const Ent &y) { return x.key < y.key; });
    std::vector<uint32_t> pa, pb, prow;
    std::vector<double> pw;
    std::vector<int64_t> pptr{0};
    for (uint64_t q = 0; q < ent.size(); q++) {
      if (q == 0 || ent[q].key != ent[q - 1].key) {
        if (q) pptr.push_back((int64_t)q);
        pa.push_back((uint32_t)(ent[q].key / F.D));
        pb.push_back((uint32_t)(ent[q].key % F.D));
      }
      prow.push_back(ent[q].row);
      pw.push_back(ent[q].w);
    }
    pptr.push_back((int64_t)ent.size());
    const uint64_t np = pa.size();
    const double gb = (double)np * kp_ * kp_ * sizeof(real);
    if (np == 0 || np > (1ull << 24) || gb > 1.0 * (1ull << 30)) return;
    if (pgram_mode_ == 1 && (double)np * kp_ > 8.0 * (double)R) return;
    F.npair = np;
    F.ppa.upload(pa);
    F.ppb.upload(pb);
    F.pgrow.upload(prow);
    F.pgval.upload(to_real(pw));
    // Gram build chunks (col_gram_chunks' cut, over the pairs' entries)
    const uint64_t ch = cgram32() ? (uint64_t)CGRAM32_ROWS
                                  : std::min<uint64_t>(cgram_chunk_, (uint64_t)cgram_rows((int)kp_, (int)sizeof(real)));
    std::vector<Job> chunks, sums;
    uint64_t slots = 0;
    for (uint64_t d = 0; d < np; d++) {
      const uint64_t b = pptr[d], e = pptr[d + 1];
      const uint32_t n = (uint32_t)std::max<uint64_t>(1, (e - b + ch - 1) / ch);
      for (uint32_t q = 0; q < n; q++)
        chunks.push_back(Job{(uint32_t)d, n, n > 1 ? (uint32_t)(slots + q) : 0u, q, (int64_t)std::min(e, b + q * ch),
                             (int64_t)std::min(e, b + (q + 1) * ch)});
      if (n > 1) sums.push_back(Job{(uint32_t)d, n, (uint32_t)slots, 0u, 0, 0});
      if (n > 1) slots += n;
    }
    F.pgchunks.upload(chunks);
    if (cgram32() && !sums.empty()) F.pgsums.upload(sums);
    F.pgslots = slots;
    F.pgcnt.alloc(np);
    // adjacency: feature a <- (p, b) for p = (a, b), and b <- (p, a) for a != b
    std::vector<int64_t> ap(F.D + 1, 0);
    for (uint64_t d = 0; d < np; d++) {
      ap[pa[d] + 1]++;
      if (pa[d] != pb[d]) ap[pb[d] + 1]++;
    }
    for (uint64_t d = 0; d < F.D; d++) ap[d + 1] += ap[d];
    std::vector<uint32_t> apair((size_t)ap[F.D]), aoth((size_t)ap[F.D]);
    std::vector<int64_t> cur(ap.begin(), ap.end() - 1);
    for (uint64_t d = 0; d < np; d++) {
      apair[(size_t)cur[pa[d]]] = (uint32_t)d;
      aoth[(size_t)cur[pa[d]]++] = pb[d];
      if (pa[d] != pb[d]) {
        apair[(size_t)cur[pb[d]]] = (uint32_t)d;
        aoth[(size_t)cur[pb[d]]++] = pa[d];
      }
    }
    F.paptr.upload(ap);
    F.papair.upload(apair);
    F.paoth.upload(aoth);
    // blocks per feature: about one adjacency entry per subgroup
    uint64_t amax = 1;
    for (uint64_t d = 0; d < F.D; d++) amax = std::max<uint64_t>(amax, (uint64_t)(ap[d + 1] - ap[d]));
    const uint64_t per = 4 * (uint64_t)nsg();
    F.pqb = (uint32_t)std::min<uint64_t>(8, (amax + per - 1) / per);
    if (F.D * F.pqb * kp_ > pgt_.n) pgt_.alloc(F.D * F.pqb * kp_);
    F.pg = true;
  }
  // The half's pair Grams (k_col_gram* with pair weights: d_i X_ia X_ib).
  void pair_grams(const HalfCtx &h) {
    DevField<real> &F = *h.F;
    if (!F.pgram.p) F.pgram.alloc(F.npair * kp_ * kp_, false);
    if (F.pgslots && !F.pgpart.p) F.pgpart.alloc(F.pgslots * kp_ * kp_, false);
    with_kp(kp_, [&](auto K) {
      constexpr int KP = decltype(K)::value;
      const double rs = sizeof(real);
      prof_launch("pair_gram", (double)F.pgrow.n * (8 + rs + 16 + KP * rs) + (double)F.pgram.bytes(), [&] {
        if constexpr (std::is_same<real, float>::value && KP == 32) {
          if (cgram32()) {
            launch(k_col_gram32, (unsigned)((F.pgchunks.n + 3) / 4), BLOCK, 0, (uint64_t)F.pgchunks.n,
                   (const Job *)F.pgchunks.p, (const uint32_t *)F.pgrow.p, (const float *)F.pgval.p, hess_cnt(h),
                   (const float *)h.Q1, (uint64_t)h.own->R, w_, hess_n1(h), (float *)F.pgram.p, (float *)F.pgpart.p,
                   1);
            if (F.pgsums.n)
              launch(k_gram_slot_sum, (unsigned)F.pgsums.n, BLOCK, 0, (const Job *)F.pgsums.p,
                     (const float *)F.pgpart.p, (float *)F.pgram.p);
            return;
          }
        }
        if constexpr (std::is_same<real, double>::value && KP == 32) {
          if (cgram32()) {
            launch(k_col_gram_f64, (unsigned)((F.pgchunks.n + 3) / 4), BLOCK, 0, (uint64_t)F.pgchunks.n,
                   (const Job *)F.pgchunks.p, (const uint32_t *)F.pgrow.p, (const double *)F.pgval.p, hess_cnt(h),
                   (const double *)h.Q1, (uint64_t)h.own->R, w_, hess_n1(h), (double *)F.pgram.p,
                   (double *)F.pgpart.p, 1);
            if (F.pgsums.n)
              launch(k_hot_slot_sum<double, 32>, dim3((unsigned)F.pgsums.n, (1024 + BLOCK - 1) / BLOCK), BLOCK, 0,
                     (const Job *)F.pgsums.p, (const double *)F.pgpart.p, (double *)F.pgram.p);
            return;
          }
        }
        launch(k_col_gram<real, KP>, (unsigned)F.pgchunks.n, BLOCK, 0, F.pgchunks.p, F.pgrow.p, F.pgval.p,
               hess_cnt(h), h.Q1, w_, hess_n1(h), F.pgram.p, F.pgpart.p, F.pgcnt.p, 1);
      });
    });
  }
  // One CG step of a pair-Gram half: one launch (k_pg_step), or with many
  // features the pair products into acc and the unfused finalisation.
  void pair_pass(HalfCtx &h, int it) {
    DevField<real> &F = *h.F;
    with_kp(kp_, [&](auto K) {
      constexpr int KP = decltype(K)::value;
      using Gm = Geo<real, KP>;
      const double rs = sizeof(real);
      const Fin<real> fin = make_fin(h, it);
      const uint32_t QB = F.pqb;
      const unsigned grid = (unsigned)std::min<uint64_t>(F.D * QB, 8192);
      const double bytes = (double)F.paoth.n * (KP * KP * rs + 8) + (double)F.D * KP * rs * (it > 1 ? 9 : 4);
      prof_launch("pg_step", bytes, [&] {
        if (F.D <= PG_FIN1) {
          launch(k_pg_step<real, KP, true>, grid, BLOCK, 0, (uint64_t)F.D, QB, (const int64_t *)F.paptr.p,
                 (const uint32_t *)F.papair.p, (const uint32_t *)F.paoth.p, (const real *)F.pgram.p, pgt_.p, fin);
          return;
        }
        launch(k_pg_step<real, KP, false>, grid, BLOCK, 0, (uint64_t)F.D, QB, (const int64_t *)F.paptr.p,
               (const uint32_t *)F.papair.p, (const uint32_t *)F.paoth.p, (const real *)F.pgram.p, pgt_.p, fin);
        const uint64_t nv = h.D * KP / Gm::VE;
        launch(k_fin<real, KP, 1>, grid_for(nv, BLOCK, 2048), BLOCK, 0, nv, fin);
      });
    });
  }

  void col_grams(const HalfCtx &h) {
    if (pgram(h)) {
      pair_grams(h);
      return;
    }
    if (!cgram(h)) return;
    if (h.cross) {
      ccg_build(h);
      return;
    }
    DevField<real> &F = *h.F;
    DevSide<real> &other = h.user ? V_ : U_;
    if (!F.gram.p) F.gram.alloc(F.D * kp_ * kp_, false);  // every column is stored by its last chunk
    if (F.gslots && !F.gpart.p) F.gpart.alloc(F.gslots * kp_ * kp_, false);
    with_kp(kp_, [&](auto K) {
      constexpr int KP = decltype(K)::value;
      const double rs = sizeof(real);
      prof_launch("col_gram", (double)F.nnz * (8 + rs + 16 + KP * rs) + (double)F.gram.bytes(), [&] {
        if constexpr (std::is_same<real, float>::value && KP == 32) {
          if (cgram32()) {
            // (q1: the same-side partner table, one row per row of this side)
            launch(k_col_gram32, (unsigned)((F.gchunks.n + 3) / 4), BLOCK, 0, (uint64_t)F.gchunks.n,
                   (const Job *)F.gchunks.p, (const uint32_t *)F.crow.p, (const float *)F.cval.p, hess_cnt(h),
                   (const float *)h.Q1, (uint64_t)h.own->R, w_, hess_n1(h), (float *)F.gram.p, (float *)F.gpart.p, 0);
            if (F.gsums.n)
              launch(k_gram_slot_sum, (unsigned)F.gsums.n, BLOCK, 0, (const Job *)F.gsums.p,
                     (const float *)F.gpart.p, (float *)F.gram.p);
            return;
          }
        }
        if constexpr (std::is_same<real, double>::value && KP == 32) {
          if (cgram32()) {
            launch(k_col_gram_f64, (unsigned)((F.gchunks.n + 3) / 4), BLOCK, 0, (uint64_t)F.gchunks.n,
                   (const Job *)F.gchunks.p, (const uint32_t *)F.crow.p, (const double *)F.cval.p, hess_cnt(h),
                   (const double *)h.Q1, (uint64_t)h.own->R, w_, hess_n1(h), (double *)F.gram.p,
                   (double *)F.gpart.p, 0);
            if (F.gsums.n)
              launch(k_hot_slot_sum<double, 32>, dim3((unsigned)F.gsums.n, (1024 + BLOCK - 1) / BLOCK), BLOCK, 0,
                     (const Job *)F.gsums.p, (const double *)F.gpart.p, (double *)F.gram.p);
            return;
          }
        }
        launch(k_col_gram<real, KP>, (unsigned)F.gchunks.n, BLOCK, 0, F.gchunks.p, F.crow.p, F.cval.p,
               hess_cnt(h), h.Q1, w_, hess_n1(h), F.gram.p, F.gpart.p, F.cnt.p, 0);
      });
    });
  }

  // Column tau: the w phi_i QTQ term of a cross half's Hessian-vector rows,
  // for a one-node-per-row field, is w (sum_{i in col d} x_i^2) p_d QTQ per
  // column, added by the feature pass (k_feat TAU) instead of per row by
  // k_hs_cross_seg: one k x k product per column instead of per row (items
  // over artist / genre: 100,000 rows, 5,000 / 50 columns).  On several ranks
  // the term is added to the column partial sums before the all-reduce (it is
  // linear in QTQ, a partial over local users on the item halves, and in
  // sum x^2, a partial over local rows on the user halves).
  static constexpr size_t COLTAU_LDS = 32 * 1024;
  bool coltau(const HalfCtx &h) const {
    return coltau_on_ && h.cross && h.F->one &&
           (size_t)kp_ * kp_ * sizeof(real) <= COLTAU_LDS;
  }

  // The Hessian-vector row pass of an id-like field's side half finalises
  // its row's feature column itself (one row = one feature, no partial sums;
  // OCFFM_FUSE=0: a separate feature pass).  Cross halves and the gradient
  // passes walk positive segments, whose sums a feature pass assembles.
  bool fused_rows(const HalfCtx &h) const {
    return fuse_ && h.F->idlike && !h.cross && (!comm_.active() || repl(h));
  }

  // Several ranks, id-like field (replicated rows, e.g. items; never an owned
  // field): the side Hessian-vector row pass writes its column partials
  // straight into acc (k_hs_side_row SCAT), no CSC scatter launch.
  bool scat_rows(const HalfCtx &h) const {
    return comm_.active() && h.F->idlike && !h.F->excl && !h.cross && !repl(h);
  }
  // Item side half on several ranks: CG steps computed whole on every rank.
  bool repl(const HalfCtx &h) const { return comm_.active() && !h.cross && !h.user && !h.F->excl && gvptr_.p; }
  const int64_t *hess_cnt(const HalfCtx &h) const { return repl(h) ? gvptr_.p : h.own->yptr.p; }
  double hess_n1(const HalfCtx &h) const { return repl(h) ? gn1_ : (double)(h.user ? V_ : U_).R; }

  void scatter(HalfCtx &h, int it, bool seg) {
    DevField<real> &F = *h.F;
    feat_launch(h, it, seg, 2);
    allreduce_dev(acc_.p, F.D * kp_);
  }

  // One feature pass (kernels.hpp: k_feat) over the row or segment CSC of
  // the half's field.  mode 0/1 finalise (gradient / Hessian-vector of CG
  // iteration it); mode 2 stores the column sums into acc_.
  // Column-block feature pass (kernels.hpp k_feat_col): a field with few,
  // heavy columns (at most 4,096 columns of 64 entries or more on average,
  // none longer than 4,096), not owned (its CSC's unowned columns have no
  // jobs), no column tau.
  int feat_col_mode_ = std::getenv("OCFFM_FEATCOL") ? std::atoi(std::getenv("OCFFM_FEATCOL")) : 1;
  bool feat_col(HalfCtx &h, bool seg, int mode) {
    DevField<real> &F = *h.F;
    const int ix = seg ? 1 : 0;
    if (feat_col_mode_ == 0 || F.excl || (mode != 0 && coltau(h))) return false;
    if (F.fcol[ix] < 0) {
      F.fcol[ix] = 0;
      const uint64_t ent = seg ? F.scrow.n : F.crow.n;
      const uint64_t nj = (seg ? F.snjw : F.njw) * (uint64_t)nsg();
      if (F.D > 0 && F.D <= 4096 && nj && (feat_col_mode_ == 2 || ent >= 64 * F.D)) {
        std::vector<Job> jobs(nj);
        HIPCHK(hipMemcpy(jobs.data(), seg ? F.sjobs.p : F.jobs.p, nj * sizeof(Job), hipMemcpyDeviceToHost));
        std::vector<int64_t> first(F.D, INT64_MAX), last(F.D, -1), cp(F.D + 1, 0);
        for (const Job &j : jobs)
          if (j.col != JOB_NONE && j.col < F.D) {
            first[j.col] = std::min(first[j.col], j.b);
            last[j.col] = std::max(last[j.col], j.e);
          }
        bool ok = true;
        for (uint64_t c = 0; c < F.D && ok; c++) {
          if (last[c] < 0) {
            cp[c + 1] = cp[c];
          } else {
            ok = first[c] == cp[c];
            cp[c + 1] = last[c];
          }
        }
        // one block walks a whole column: only where no column is long (at
        // most 16 rounds of 256 entries; outbrain's platform columns of
        // ~83 k rows took 587 us per step this way, the job-based pass ~50)
        int64_t cmax = 0;
        for (uint64_t c = 0; c < F.D; c++) cmax = std::max<int64_t>(cmax, cp[c + 1] - cp[c]);
        if (ok && (uint64_t)cp[F.D] == ent && (feat_col_mode_ == 2 || cmax <= 4096)) {
          F.fcptr[ix].upload(cp);
          F.fcol[ix] = 1;
        }
      }
    }
    return F.fcol[ix] == 1;
  }

  void feat_launch(HalfCtx &h, int it, bool seg, int mode) {
    DevField<real> &F = *h.F;
    const uint64_t njw = seg ? F.snjw : F.njw;
    if (!njw) return;
    if (feat_col(h, seg, mode)) {
      with_kp(kp_, [&](auto K) {
        constexpr int KP = decltype(K)::value;
        const double rs = sizeof(real);
        const uint64_t ent = seg ? F.scrow.n : F.crow.n;
        const double vecs = mode == 2 ? 1 : (mode == 0 ? 5 : (it > 1 ? 8 : 3));
        const double bytes = (double)ent * (4 + rs) + (double)ent * KP * rs + (double)F.D * 8 +
                             (double)h.D * KP * rs * vecs;
        const char *name = mode == 2 ? "csc_scatter" : (mode == 0 ? "feat_grad" : "feat_hv");
        Fin<real> fin = make_fin(h, it);
        const uint32_t *crow = seg ? F.scrow.p : F.crow.p;
        const real *cval = seg ? F.scval.p : F.cval.p;
        const int64_t *cp = F.fcptr[seg ? 1 : 0].p;
        const unsigned grid = (unsigned)std::min<uint64_t>(F.D, 4096);
        prof_launch(name, bytes, [&] {
          if (mode == 0)
            launch(k_feat_col<real, KP, 0>, grid, BLOCK, 0, (uint64_t)F.D, cp, crow, cval, (const real *)h_.p,
                   (uint64_t)h_.bytes(), fin);
          else if (mode == 1)
            launch(k_feat_col<real, KP, 1>, grid, BLOCK, 0, (uint64_t)F.D, cp, crow, cval, (const real *)h_.p,
                   (uint64_t)h_.bytes(), fin);
          else
            launch(k_feat_col<real, KP, 2>, grid, BLOCK, 0, (uint64_t)F.D, cp, crow, cval, (const real *)h_.p,
                   (uint64_t)h_.bytes(), fin);
        });
      });
      return;
    }
    with_kp(kp_, [&](auto K) {
      constexpr int KP = decltype(K)::value;
      using Gm = Geo<real, KP>;
      const double rs = sizeof(real);
      const uint64_t ent = seg ? F.scrow.n : F.crow.n;
      const double vecs = mode == 2 ? 1 : (mode == 0 ? 5 : (it > 1 ? 8 : 3));
      const double bytes = (double)ent * (4 + rs) + (double)ent * KP * rs + (double)njw * Gm::NSG * sizeof(Job) +
                           (double)h.D * KP * rs * vecs;
      const unsigned grid0 = (unsigned)std::min<uint64_t>((njw + 3) / 4, feat_blocks_);  // grid-stride: fewer tickets
      // at most one resident wave of blocks (OCFFM_FEAT_FILL): fp64's
      // register count holds fewer blocks per CU than the fp32 cap assumes
      auto fill = [&](auto k, size_t sm) { return feat_fill_ ? std::min(grid0, resident(k, sm)) : grid0; };
      Fin<real> fin = make_fin(h, it);
      fin.hdots = seg ? F.shdots.p : F.hdots.p;
      fin.nhd = (uint32_t)(seg ? F.snslot : F.nslot);
      const Job *jobs = seg ? F.sjobs.p : F.jobs.p;
      const uint32_t *crow = seg ? F.scrow.p : F.crow.p;
      const real *cval = seg ? F.scval.p : F.cval.p;
      real *hb = h_.p;
      const uint64_t hbytes = h_.bytes();
      const char *name = mode == 2 ? "csc_scatter" : (mode == 0 ? "feat_grad" : "feat_hv");
      const real *nq = nullptr;
      prof_launch(name, bytes, [&] {
        constexpr size_t tq = (size_t)KP * KP * sizeof(real);
        if (mode == 0) {
          launch(k_feat<real, KP, 0>, fill(k_feat<real, KP, 0>, 0), BLOCK, 0, njw, jobs, crow, cval, hb, hbytes,
                 wpart_.p, wpart_.bytes(), fin, nq);
        } else if (mode == 1) {
          if constexpr (tq <= COLTAU_LDS) {
            if (coltau(h)) {
              fin.xsq = F.xsq.p;
              launch(k_feat<real, KP, 1, JOB_ENT, true>, fill(k_feat<real, KP, 1, JOB_ENT, true>, tq), BLOCK, tq, njw,
                     jobs, crow, cval, hb, hbytes, wpart_.p, wpart_.bytes(), fin, (const real *)qtq_);
              return;
            }
          }
          launch(k_feat<real, KP, 1>, fill(k_feat<real, KP, 1>, 0), BLOCK, 0, njw, jobs, crow, cval, hb, hbytes,
                 wpart_.p, wpart_.bytes(), fin, nq);
        } else {
          if constexpr (tq <= COLTAU_LDS) {
            if (coltau(h) && it > 0) {
              fin.xsq = F.xsq.p;
              launch(k_feat<real, KP, 2, JOB_ENT, true>, fill(k_feat<real, KP, 2, JOB_ENT, true>, tq), BLOCK, tq, njw,
                     jobs, crow, cval, hb, hbytes, wpart_.p, wpart_.bytes(), fin, (const real *)qtq_);
              return;
            }
          }
          launch(k_feat<real, KP, 2>, fill(k_feat<real, KP, 2>, 0), BLOCK, 0, njw, jobs, crow, cval, hb, hbytes,
                 wpart_.p, wpart_.bytes(), fin, nq);
        }
      });
    });
  }

  // Feature pass of a half: fused gather + finalisation on one GPU; gather,
  // all-reduce, finalisation when the partial sums must meet across ranks.
  // mode 0: gradient (it = 0), mode 1: Hessian-vector of CG iteration `it`.
  void feature_pass(HalfCtx &h, int it, bool seg, bool acc_ready = false) {
    if (!comm_.active() || (it > 0 && repl(h))) {
      feat_launch(h, it, seg, it == 0 ? 0 : 1);
      return;
    }
    if (h.F->excl) {  // owned field: local columns only, then the dot products meet
      if (!(seg ? h.F->snjw : h.F->njw)) HIPCHK(hipMemsetAsync(dots_.p, 0, 3 * sizeof(double), stream_));
      else feat_launch(h, it, seg, it == 0 ? 0 : 1);
      allreduce_dev_d(dots_.p, 3);
      const Fin<real> fin = make_fin(h, it);
      prof_launch("cg_step", 0, [&] {
        if (it == 0) launch(k_cg_step<real, 0>, 1, 64, 0, fin);
        else launch(k_cg_step<real, 1>, 1, 64, 0, fin);
      });
      return;
    }
    if (acc_ready) allreduce_dev(acc_.p, h.F->D * kp_);  // the row pass filled acc (scat_rows)
    else scatter(h, it, seg);
    with_kp(kp_, [&](auto K) {
      constexpr int KP = decltype(K)::value;
      using Gm = Geo<real, KP>;
      const double rs = sizeof(real);
      const uint64_t nv = h.D * KP / Gm::VE;
      const Fin<real> fin = make_fin(h, it);
      const unsigned grid = grid_for(nv, BLOCK, 2048);
      if (it == 0)
        prof_launch("grad_fin", (double)h.D * KP * rs * 6, [&] { launch(k_fin<real, KP, 0>, grid, BLOCK, 0, nv, fin); });
      else
        prof_launch("hv_fin", (double)h.D * KP * rs * (it > 1 ? 9 : 4),
                    [&] { launch(k_fin<real, KP, 1>, grid, BLOCK, 0, nv, fin); });
    });
  }

  // One CG step: the Hessian-vector product lam*V + H(V) into Hv_ with alpha
  // (and beta and the verdict, or those from the exact residual pass).
  void hv_pass(HalfCtx &h, int it) {
    hv_product(h, it);
    if (!exact_r2(h)) return;
    const Fin<real> fin = make_fin(h, it);
    const uint64_t nv = h.D * kp_ / VT<real>::N;
    prof_launch("cg_r2", (double)h.D * kp_ * sizeof(real) * 2,
                [&] { launch(k_cg_r2<real>, grid_for(nv, BLOCK, 1024), BLOCK, 0, nv, fin); });
  }
  // Exact residual norm (fp64 parity mode): not for owned fields
  // on several ranks, whose r / Hp rows are current on their owner only.
  bool exact_r2(const HalfCtx &h) const { return exact_r2_ && !(comm_.active() && (h.F->excl || io_half(h))); }

  // ---- item-owned CG steps (OCFFM_ITEM_OWNED=1, the default: several
  // ranks; 2: also a one-rank communicator, to run the collectives' code
  // path; 0: off, every step all-reduces the D x k partials)
  int io_mode_ = std::getenv("OCFFM_ITEM_OWNED") ? std::atoi(std::getenv("OCFFM_ITEM_OWNED")) : 1;
  DevBuf<real> Pg_, qtqg_;
  uint64_t io_cu_ = 0;  // user rows per rank slot of Pg
  bool io_half(const HalfCtx &h) const { return h.cross && !h.user && h.F->io != nullptr; }

  // In-place all-gather: rank r's `count` values at buf + r count.  RCCL:
  // ncclAllGather; the host hook (tests, rehearsals) sums the buffer with
  // every other slot zeroed (exact).
  void allgather_dev(real *buf, uint64_t count) {
    const uint64_t N = (uint64_t)comm_.nranks, r = (uint64_t)comm_.rank;
    if (comm_.nccl) {
      NCCLCHK(ncclAllGather(buf + r * count, buf, count, std::is_same<real, double>::value ? ncclDouble : ncclFloat,
                            comm_.nccl, stream_));
      return;
    }
    if (r) HIPCHK(hipMemsetAsync(buf, 0, r * count * sizeof(real), stream_));
    if (r + 1 < N) HIPCHK(hipMemsetAsync(buf + (r + 1) * count, 0, (N - r - 1) * count * sizeof(real), stream_));
    allreduce_dev(buf, N * count);
  }

  // Each item-id field of the item side (one node per item row, item j ->
  // column j) gets its owned items' positives over all users, in the order
  // one rank would hold them (users ascending per item), cut into the same
  // segments; the segment CSC's jobs cover the owned columns only.
  void io_setup(const HostData &U, const HostData &V) {
    const uint64_t N = (uint64_t)comm_.nranks, q = (uint64_t)comm_.rank, m = U.m;
    // Worth it where the user table's all-gather (m k) plus S and p (2 n k)
    // moves less than the ring all-reduces of ~8 CG steps (8 x 2 n k): m <=
    // 14 n (kkbox at N = 8: 246 k users, 100 k items; not config 5: 100 M
    // users against 250 k items), and the gathered table within the 32-bit
    // offsets of the partner-row gathers (BufView).
    if (io_mode_ == 1 && (double)m > 14.0 * (double)n_) return;
    if ((double)N * ((m + N - 1) / N) * kp_ * sizeof(real) >= (double)((1ull << 32) - 64)) return;
    io_cu_ = (m + N - 1) / N;
    const HostData &Vs = split_host(V);
    bool any = false;
    uint64_t need = 0;
    for (uint32_t fi = 0; fi < V_.F.size(); fi++) {
      DevField<real> &F = *V_.F[fi];
      if (!F.one || F.D != n_ || F.excl) continue;
      bool ident = Vs.xptr[fi].size() == n_ + 1;
      for (uint64_t j = 0; j < n_ && ident; j++) ident = Vs.xptr[fi][j + 1] - Vs.xptr[fi][j] == 1 && Vs.xidx[fi][j] == j;
      if (!ident) continue;
      auto io = std::make_unique<ItemOwned<real>>();
      io->chunk = (n_ + N - 1) / N;
      io->j0 = std::min<uint64_t>(n_, q * io->chunk);
      io->j1 = std::min<uint64_t>(n_, (q + 1) * io->chunk);
      const uint64_t R = io->j1 - io->j0;
      // item-major positives of the owned items (users ascending), as Pg rows
      std::vector<int64_t> yp(R + 1, 0);
      for (uint64_t p = 0; p < U.ycol.size(); p++) {
        const uint64_t j = U.ycol[p];
        if (j >= io->j0 && j < io->j1) yp[j - io->j0 + 1]++;
      }
      for (uint64_t r = 0; r < R; r++) yp[r + 1] += yp[r];
      std::vector<uint32_t> yc((size_t)yp[R]);
      std::vector<int64_t> cur(yp.begin(), yp.end() - 1);
      for (uint64_t rk = 0; rk < N; rk++) {
        const uint64_t g0 = m * rk / N, g1 = m * (rk + 1) / N;
        for (uint64_t g = g0; g < g1; g++)
          for (uint64_t p = U.yptr[g]; p < U.yptr[g + 1]; p++) {
            const uint64_t j = U.ycol[p];
            if (j >= io->j0 && j < io->j1) yc[(size_t)cur[j - io->j0]++] = (uint32_t)(rk * io_cu_ + (g - g0));
          }
      }
      // segments (build_segments' cut) with their node, and the CSC jobs
      std::vector<Seg> segs;
      std::vector<uint32_t> segptr(R + 1, 0), sd;
      std::vector<double> sx;
      for (uint64_t r = 0; r < R; r++) {
        segptr[r] = (uint32_t)segs.size();
        const int64_t b = yp[r], e = yp[r + 1];
        const uint32_t nrow = (uint32_t)std::max<int64_t>(1, (e - b + (int64_t)seg_len_ - 1) / (int64_t)seg_len_);
        int64_t p = b;
        do {
          const int64_t t = std::min<int64_t>(e, p + (int64_t)seg_len_);
          segs.push_back(Seg{(uint32_t)r, (nrow << 1) | (p == b ? 1u : 0u), p, t});
          sd.push_back((uint32_t)(io->j0 + r));
          sx.push_back(Vs.xval[fi][io->j0 + r]);
          p = t;
        } while (p < e);
      }
      segptr[R] = (uint32_t)segs.size();
      io->nseg = segs.size();
      std::vector<int64_t> xp(io->nseg + 1);
      for (uint64_t t = 0; t <= io->nseg; t++) xp[t] = (int64_t)t;
      std::vector<uint8_t> own(F.D, 0);
      for (uint64_t j = io->j0; j < io->j1; j++) own[j] = 1;
      std::vector<uint32_t> crow;
      std::vector<double> cval;
      std::vector<Job> jobs;
      build_csc(io->nseg, F.D, xp.data(), sd.data(), sx.data(), nsg(), crow, cval, jobs, io->snslot, own.data());
      io->segs.upload(segs);
      io->segptr.upload(segptr);
      io->ycol.upload(yc);
      io->segd.upload(sd);
      io->segx.upload(to_real(sx));
      io->scrow.upload(crow);
      io->scval.upload(to_real(cval));
      io->sjobs.upload(jobs);
      io->snjw = jobs.size() / nsg();
      io->shdots.alloc(std::max<uint64_t>(io->snslot, 1) * 3);
      need = std::max(need, io->nseg);
      if (io->snslot * kp_ > wpart_.n) wpart_.alloc(io->snslot * kp_);
      if (N * io->chunk * kp_ > S_.n) {  // the all-gathered CG vectors: N whole chunks
        S_.alloc(N * io->chunk * kp_);
        Vd_.alloc(N * io->chunk * kp_);
      }
      F.io = std::move(io);
      any = true;
    }
    if (!any) return;
    if (need * kp_ > h_.n) h_.alloc(need * kp_);
    if (h_.bytes() >= (1ull << 32) - 64)  // kernels.hpp: BufView gathers use 32-bit offsets
      throw Error(OCFFM_E_DATA, "too many item-owned segments per GPU for one partial buffer; set OCFFM_ITEM_OWNED=0");
    Pg_.alloc(N * io_cu_ * kp_);
    qtqg_.alloc((uint64_t)kp_ * kp_);
    const uint64_t st = std::max<uint64_t>(N * io_cu_, N * ((n_ + N - 1) / N)) * kp_;
    if (comm_.host_fn && st > dmax_ * kp_) {
      HIPCHK(hipHostFree(stage_));
      HIPCHK(hipHostMalloc((void **)&stage_, st * sizeof(real), hipHostMallocDefault));
    }
  }

  // Before the CG steps: every rank's rows of the partner (user) table and
  // the global Q^T Q of this half.
  void io_begin(HalfCtx &h) {
    const uint64_t r = (uint64_t)comm_.rank, R = h.partner->R;
    HIPCHK(hipMemsetAsync(Pg_.p + r * io_cu_ * kp_, 0, io_cu_ * kp_ * sizeof(real), stream_));
    if (R) HIPCHK(hipMemcpyAsync(Pg_.p + r * io_cu_ * kp_, h.Q1, R * kp_ * sizeof(real), hipMemcpyDeviceToDevice, stream_));
    allgather_dev(Pg_.p, io_cu_ * kp_);
    HIPCHK(hipMemcpyAsync(qtqg_.p, qtq_, (size_t)kp_ * kp_ * sizeof(real), hipMemcpyDeviceToDevice, stream_));
    allreduce_dev(qtqg_.p, (uint64_t)kp_ * kp_);
  }
  // After them: the owners' S and p columns on every rank (the update reads
  // S + alpha p of every column).
  void io_end(HalfCtx &h) {
    const ItemOwned<real> &io = *h.F->io;
    allgather_dev(S_.p, io.chunk * kp_);
    allgather_dev(Vd_.p, io.chunk * kp_);
  }
  // One item-owned CG step: the owned items' rows over all users' positives,
  // the owned columns' finalisation, the dot products summed over the ranks.
  void hv_io(HalfCtx &h, int it) {
    DevField<real> &F = *h.F;
    const ItemOwned<real> &io = *F.io;
    with_kp(kp_, [&](auto K) {
      constexpr int KP = decltype(K)::value;
      using Gm = Geo<real, KP>;
      const double rs = sizeof(real);
      const size_t qsz = (size_t)KP * KP * sizeof(real);
      const bool lds = qsz <= 32 * 1024;
      const bool ct = coltau(h);
      Fin<real> fin = make_fin(h, it);
      fin.dots = dots_.p;
      const int *run = &st_.p->run[it];
      if (io.nseg) {
        prof_launch("hs_cross_io", (double)io.nseg * (24 + 8 + rs) + (double)io.nseg * KP * rs * 2, [&] {
          auto go = [&](auto ml) {
            constexpr bool ML = decltype(ml)::value;
            launch(k_hs_cross_seg<real, KP, ML>, grid_for(io.nseg, 4 * Gm::NSG, hs_blocks_), BLOCK, lds ? qsz : 0,
                   io.nseg, io.segs.p, F.xptr.p, F.xidx.p, F.xval.p, Vd_.p, io.ycol.p, (const real *)Pg_.p,
                   (uint64_t)comm_.nranks * io_cu_, ct ? (const real *)nullptr : (const real *)qtqg_.p, w_, h_.p,
                   run, Rv_.p, Hv_.p, st_.p, it, io.segd.p, io.segx.p, (const uint32_t *)nullptr,
                   (const real *)nullptr, (const uint32_t *)nullptr);
          };
          if (lds) go(std::true_type());
          else go(std::false_type());
        });
      }
      if (!io.snjw) {
        HIPCHK(hipMemsetAsync(dots_.p, 0, 3 * sizeof(double), stream_));
      } else {
        fin.hdots = io.shdots.p;
        fin.nhd = (uint32_t)io.snslot;
        const unsigned grid = (unsigned)std::min<uint64_t>((io.snjw + 3) / 4, feat_blocks_);
        prof_launch("feat_hv_io", (double)io.scrow.n * (4 + rs) * 2 + (double)io.snjw * Gm::NSG * sizeof(Job), [&] {
          if constexpr ((size_t)KP * KP * sizeof(real) <= COLTAU_LDS) {
            if (ct) {
              fin.xsq = F.xsq.p;
              launch(k_feat<real, KP, 1, JOB_ENT, true>, grid, BLOCK, (size_t)KP * KP * sizeof(real), io.snjw,
                     io.sjobs.p, io.scrow.p, io.scval.p, h_.p, h_.bytes(), wpart_.p, wpart_.bytes(), fin,
                     (const real *)qtqg_.p);
              return;
            }
          }
          launch(k_feat<real, KP, 1>, grid, BLOCK, 0, io.snjw, io.sjobs.p, io.scrow.p, io.scval.p, h_.p, h_.bytes(),
                 wpart_.p, wpart_.bytes(), fin, (const real *)nullptr);
        });
      }
      allreduce_dev_d(dots_.p, 3);
      const Fin<real> f2 = fin;
      prof_launch("cg_step", 0, [&] { launch(k_cg_step<real, 1>, 1, 64, 0, f2); });
    });
  }

  // Persistent column-Gram CG (k_cg_cgram): one GPU (or a replicated half:
  // no collective inside), the plain expanded residual, not item-owned.
  // Only where the step kernel's own grid fits one block per CU (genre,
  // artist): a persistent grid is capped there, and on config 5's 250 k
  // columns that cap cost the Gram stream its occupancy (5.0 -> 5.3 s per
  // epoch with the persistent kernel on every column-Gram half).
  bool cgp_ok(const HalfCtx &h) const {
    const uint64_t per_block = 4 * (uint64_t)nsg();
    return cgp_on_ && cgram(h) && (!comm_.active() || repl(h)) && !exact_r2(h) && !io_half(h) && h.D > 0 &&
           (h.D + per_block - 1) / per_block <= ncu_;
  }
  double cgp_step_bytes(const HalfCtx &h) const {
    return (double)h.D * kp_ * kp_ * sizeof(real) + (double)h.D * kp_ * sizeof(real) * 9;
  }
  // Returns false if nothing was launched (a cooperative launch the runtime
  // refused: the caller takes the two-launch path for the whole half).
  bool cg_persist(HalfCtx &h) {
    bool ok = true;
    with_kp(kp_, [&](auto K) {
      constexpr int KP = decltype(K)::value;
      using Gm = Geo<real, KP>;
      Fin<real> fin = make_fin(h, 1);
      // at most one block per CU (co-resident unless other work holds the CUs),
      // whole rounds of the 8 XCDs where that stays within the CUs
      unsigned grid = (unsigned)std::min<uint64_t>((h.D + 4 * Gm::NSG - 1) / (4 * Gm::NSG), ncu_);
      if (cgp_xcd_ && (grid + 7) / 8 * 8 <= ncu_) grid = (grid + 7) / 8 * 8;
      if (cgp_gen_ > 0xf0000000u) {  // keep clear of CGP_ABORT
        HIPCHK(hipMemsetAsync(cgp_gen_buf_.p, 0, sizeof(unsigned), stream_));
        cgp_gen_ = 1;
      }
      unsigned g0 = cgp_gen_;
      cgp_gen_ += MAXCG + 1;
      const real *G = gram_of(h);
      uint64_t D = h.D;
      unsigned *genp = cgp_gen_buf_.p;
      int *errh = run_host_dev_ + MAXCG + 3, *abd = cgp_abort_.p;
      unsigned spin = cgp_spin_;
      int stall = cgp_stall_, xcdc = cgp_xcd_ ? 1 : 0;
      if (grid > resident(k_cg_cgram<real, KP>, 0)) {  // cannot be resident at once: per-step path
        counters["cgp_refused"]++;
        ok = false;
        return;
      }
      counters["cgp_launches"]++;
      prof_launch("cg_cgram", 0.0, [&] {
        if (!cgp_coop_) {
          launch(k_cg_cgram<real, KP>, grid, BLOCK, 0, D, G, fin, genp, g0, errh, abd, spin, stall, xcdc);
          return;
        }
        // cooperative: the runtime checks that the grid can be resident at
        // once and refuses it otherwise (then: the per-step path)
        void *args[] = {&D, (void *)&G, &fin, &genp, &g0, &errh, &abd, &spin, &stall, &xcdc};
        if (arm_first_) HIPCHK(hipEventRecord(arm_a_, stream_));
        const hipError_t e = hipLaunchCooperativeKernel(reinterpret_cast<const void *>(k_cg_cgram<real, KP>), dim3(grid),
                                                        dim3(BLOCK), args, 0u, stream_);
        if (e == hipErrorCooperativeLaunchTooLarge) {
          (void)hipGetLastError();
          counters["cgp_refused"]++;
          ok = false;
        } else {
          HIPCHK(e);
        }
        if (arm_first_) {
          HIPCHK(hipEventRecord(arm_b_, stream_));
          arm_first_ = false;
        }
      });
    });
    return ok;
  }
  // Persistent CG of an id-like side half (k_cg_side_id): the CG
  // vectors of the half's rows in registers for the whole solve.  Where the
  // fused per-step path would run (fused_rows: one GPU, or replicated rows),
  // with the plain expanded residual, and where the rows fit the resident
  // grid at <= 4 rows per subgroup (SMAX): kkbox's song-id (100 k, fp32)
  // and listener-id (30 k) side halves.
  // full: the whole half in the launch (k_cg_side_id FULL: gradient, CG
  // and update), where the gradient reads the segment sums and nothing
  // else runs between the gradient and the CG (one GPU; no Gram path).
  int sidep_smax(const HalfCtx &h, bool full = false) {
    if (!sidep_on_ || !fused_rows(h) || exact_r2(h) || h.own->R == 0 ||
        h.F->excl)
      return 0;
    if (full && (!sidef_on_ || comm_.active() || !ysum_on_ || !h.own->nseg || pgram(h) || cgram(h) || hot(h)))
      return 0;
    int smax = 0;
    with_kp(kp_, [&](auto K) {
      constexpr int KP = decltype(K)::value;
      using Gm = Geo<real, KP>;
      const uint64_t R = h.own->R;
      auto fits = [&](auto sm) {
        constexpr int SM = decltype(sm)::value;
        const unsigned res = full ? resident(k_cg_side_id<real, KP, SM, true>, 0) : resident(k_cg_side_id<real, KP, SM>, 0);
        return (R + SM * 4 * Gm::NSG - 1) / (SM * 4 * Gm::NSG) <= res;
      };
      if (fits(std::integral_constant<int, 1>())) smax = 1;
      else if (fits(std::integral_constant<int, 2>())) smax = 2;
      else if (fits(std::integral_constant<int, 4>())) smax = 4;
    });
    return smax;
  }
  bool side_persist(HalfCtx &h, int smax, bool full = false) {
    if (full) {
      flush_base();  // (gradient's work ahead of the gradient pass)
      seg_ysum(h, true);
    }
    with_kp(kp_, [&](auto K) {
      constexpr int KP = decltype(K)::value;
      using Gm = Geo<real, KP>;
      Fin<real> fin = make_fin(h, full ? 0 : 1);
      DevSide<real> &own = *h.own;
      DevField<real> &F = *h.F;
      if (cgp_gen_ > 0xf0000000u) {  // keep clear of CGP_ABORT
        HIPCHK(hipMemsetAsync(cgp_gen_buf_.p, 0, sizeof(unsigned), stream_));
        cgp_gen_ = 1;
      }
      const unsigned g0 = cgp_gen_;
      cgp_gen_ += MAXCG + 1;
      counters["cgp_launches"]++;
      counters["cgp_side_launches"]++;
      if (full) counters["cgp_side_full"]++;
      const double rs = sizeof(real);
      const double bytes = (double)own.R * KP * rs * 9 + (double)own.R * (4 + rs + 16);
      DevSide<real> &other = h.user ? V_ : U_;
      SideHalf<real> sh{(const real *)yrow_.p, own.bias.p, own.s.p,
                        bsum_.p + (h.user ? 1 : 0), bsum_.p + (h.user ? 0 : 1), h.P1, r_};
      (void)other;
      auto go = [&](auto sm) {
        constexpr int SM = decltype(sm)::value;
        auto kern = [&](auto fl) {
          constexpr bool FL = decltype(fl)::value;
          const unsigned need = (unsigned)((own.R + SM * 4 * Gm::NSG - 1) / (SM * 4 * Gm::NSG));
          const unsigned res = resident(k_cg_side_id<real, KP, SM, FL>, 0);
          const unsigned grid = (need + 7) / 8 * 8 <= res ? (need + 7) / 8 * 8 : need;  // XCD-ordered when it fits
          prof_launch(FL ? "side_half" : "cg_side", bytes, [&] {
            launch(k_cg_side_id<real, KP, SM, FL>, grid, BLOCK, 0, own.R, F.xidx.p, F.xval.p, hess_cnt(h), h.Q1, w_,
                   hess_n1(h), fin, cgp_gen_buf_.p, g0, run_host_dev_ + MAXCG + 3, cgp_abort_.p, cgp_spin_,
                   cgp_stall_, sh);
          });
        };
        if (full) kern(std::true_type());
        else kern(std::false_type());
      };
      if (smax == 1) go(std::integral_constant<int, 1>());
      else if (smax == 2) go(std::integral_constant<int, 2>());
      else go(std::integral_constant<int, 4>());
    });
    return true;
  }
  // The persistent grid gave up on a barrier (kernels.hpp k_cg_cgram): every
  // column is at step `ab` (the host word holds ab + 1; ab = 0: the fused
  // side half gave up after its gradient, k_side_id_half) with that step's
  // scalars and verdict published, and the update queued behind the launch
  // returned at entry.  Reset the abort words and the generation word, read
  // the verdicts up to ab + 1, and return the step the per-step loop
  // continues with.
  template <class Ex> int cgp_recover(Ex &examine, bool &gave_up, bool &queued) {
    HIPCHK(hipStreamSynchronize(stream_));
    const int ab = __atomic_load_n(&run_host_[MAXCG + 3], __ATOMIC_ACQUIRE) - 1;  // the word holds step + 1
    if (ab < 0 || ab > MAXCG) throw Error(OCFFM_E_STATE, "persistent CG: bad abort step " + std::to_string(ab));
    run_host_[MAXCG + 3] = 0;
    std::atomic_thread_fence(std::memory_order_seq_cst);
    HIPCHK(hipMemsetAsync(cgp_abort_.p, 0, sizeof(int), stream_));
    HIPCHK(hipMemsetAsync(cgp_gen_buf_.p, 0, sizeof(unsigned), stream_));
    cgp_gen_ = 1;
    counters["cgp_recovered"]++;
    gave_up = false;
    queued = false;
    examine(ab + 1);
    if (gave_up) throw Error(OCFFM_E_STATE, "persistent CG: verdict missing after recovery");
    return ab + 1;
  }

  // Processing order of a side's segments for the cross row passes
  // (k_gd_cross_seg, k_hs_cross_seg): by length, longest first, stable (a
  // counting sort of the lengths <= seg_len_).  A wave's subgroups take
  // consecutive entries, so they walk segments of similar length and the
  // gather rounds carry fewer absent slots (item rows: median ~10 positives
  // in 32-slot rounds).  Opt-in (OCFFM_SORDER=1): measured slower, 5.40 ->
  // 5.58 ms per kkbox epoch (gd_cross_row 72.8 -> 81.1 us: the MFMA T tile's
  // rows and the h stores lose their contiguity).
  bool sorder_on_ = std::getenv("OCFFM_SORDER") && std::atoi(std::getenv("OCFFM_SORDER")) != 0;
  const uint32_t *sord(const DevSide<real> &sd) const { return sorder_on_ && sd.sord.p ? sd.sord.p : nullptr; }
  void build_sorder(DevSide<real> &sd) {
    if (!sorder_on_ || sd.nseg == 0 || sd.nseg >= (1ull << 32)) return;
    std::vector<Seg> sg(sd.nseg);
    HIPCHK(hipMemcpy(sg.data(), sd.segs.p, sd.nseg * sizeof(Seg), hipMemcpyDeviceToHost));
    // key k = L - len in [0, L] (longest first); bucket starts by an
    // exclusive prefix sum over the L + 1 keys
    const uint64_t L = seg_len_ + 1;
    auto key = [&](const Seg &x) { return L - std::min<uint64_t>(L, (uint64_t)(x.e - x.b)); };
    std::vector<uint64_t> start(L + 2, 0);
    for (const Seg &x : sg) start[key(x) + 1]++;
    for (uint64_t k = 0; k <= L; k++) start[k + 1] += start[k];
    std::vector<uint32_t> ord(sd.nseg);
    for (uint64_t q = 0; q < sd.nseg; q++) ord[start[key(sg[q])]++] = (uint32_t)q;
    sd.sord.upload(ord);
  }

  // Segment length profile of a side (host, once): short_segs when at
  // least 99 % of its segments hold at most 16 positives (outbrain's users:
  // ~1 positive per row), where k_hs_cross_seg's passes of 16 positions
  // carry half the absent slots of the 32-position pass (OCFFM_SHORTPASS=0:
  // always 32).
  bool shortpass_on_ = !std::getenv("OCFFM_SHORTPASS") || std::atoi(std::getenv("OCFFM_SHORTPASS")) != 0;
  void seg_shape(DevSide<real> &sd) {
    sd.short_segs = false;
    if (!shortpass_on_ || sd.nseg == 0) return;
    std::vector<Seg> sg(sd.nseg);
    HIPCHK(hipMemcpy(sg.data(), sd.segs.p, sd.nseg * sizeof(Seg), hipMemcpyDeviceToHost));
    uint64_t small = 0;
    for (const Seg &x : sg) small += (x.e - x.b) <= 16 ? 1 : 0;
    sd.short_segs = (double)small >= 0.99 * (double)sd.nseg;
  }

  // Fused cross steps (k_hv_cross_id): an id-like cross half on one GPU
  // whose hot rows (Grams) hold a minority of the positives.
  bool xfuse(const HalfCtx &h) const {
    if (!xfuse_on_ || !h.cross || !h.F->idlike || comm_.active() || h.F->excl || cgram(h) || pgram(h) || ccg_now_ ||
        hot(h) || h.own->R == 0 || !qtq_ || kp_ > 64 || !h.own->xf_ok)
      return false;
    return h.own->nhot == 0 || hotG_.p;
  }
  void hv_cross_id(HalfCtx &h, int it) {
    DevSide<real> &own = *h.own;
    const bool hotr = own.nhot > 0 && hotG_.p;
    with_kp(kp_, [&](auto K) {
      constexpr int KP = decltype(K)::value;
      if constexpr (xfuse_kp<real, KP>()) {
        using Gm = Geo<real, KP>;
        const double rs = sizeof(real);
        DevField<real> &F = *h.F;
        const Fin<real> fin = make_fin(h, it);
        // (the partner table once, as k_hs_cross_seg's count: its rows are L2 / Infinity Cache hits)
        const double bytes = (double)own.R * (16 + 4 + rs + 4) + (double)(own.npos - own.hpos) * 4 +
                             (double)h.partner->R * KP * rs + (double)own.nhot * KP * KP * rs +
                             (double)h.D * KP * rs * (it > 1 ? 8 : 3);
        auto go = [&](auto gb) {
          constexpr int GB = decltype(gb)::value;
          unsigned grid = grid_for(own.R, 4 * Gm::NSG, hs_blocks_);
          // one resident wave of blocks in both precisions (~3 rows per
          // subgroup, the next row's descriptor in flight; fp32: 4.99 -> 4.78 ms)
          grid = std::min(grid, resident(k_hv_cross_id<real, KP, GB>, 0));
          launch(k_hv_cross_id<real, KP, GB>, grid, BLOCK, 0, own.R, F.xidx.p, F.xval.p, (const int64_t *)own.yptr.p,
                 (const uint32_t *)own.ycol.p, h.Q1, (uint64_t)h.partner->R, (const real *)qtq_, w_,
                 hotr ? (const uint32_t *)own.hot_row.p : (const uint32_t *)nullptr, (const real *)hotG_.p, fin);
        };
        prof_launch("hv_cross_id", bytes, [&] {
          if (xf_gb_ >= 16) go(std::integral_constant<int, 16>());
          else go(std::integral_constant<int, 8>());
        });
      }
    });
  }

  void hv_product(HalfCtx &h, int it) {
    DevSide<real> &own = *h.own;
    const int *run = &st_.p->run[it];
    if (io_half(h)) {
      hv_io(h, it);
      return;
    }
    if (xfuse(h)) {
      hv_cross_id(h, it);
      return;
    }
    if (cgram(h)) {
      with_kp(kp_, [&](auto K) {
        constexpr int KP = decltype(K)::value;
        using Gm = Geo<real, KP>;
        const double rs = sizeof(real);
        const Fin<real> fin = make_fin(h, it);
        if (!comm_.active() || repl(h)) {
          prof_launch("hv_cgram", (double)h.D * KP * KP * rs + (double)h.D * KP * rs * (it > 1 ? 9 : 4), [&] {
            launch(k_hv_cgram<real, KP>, mfill(k_hv_cgram<real, KP>, grid_for(h.D, 4 * Gm::NSG, 1024)), BLOCK, 0, (uint64_t)h.D, gram_of(h), fin,
                   (const uint8_t *)nullptr);
          });
          return;
        }
        if (h.F->excl) {  // owned field: this rank's columns are whole here; the dot products meet (feature_pass)
          prof_launch("hv_cgram", (double)h.D * KP * KP * rs + (double)h.D * KP * rs * (it > 1 ? 9 : 4), [&] {
            launch(k_hv_cgram<real, KP>, mfill(k_hv_cgram<real, KP>, grid_for(h.D, 4 * Gm::NSG, 1024)), BLOCK, 0, (uint64_t)h.D, gram_of(h), fin,
                   (const uint8_t *)h.F->own.p);
          });
          allreduce_dev_d(dots_.p, 3);
          prof_launch("cg_step", 0, [&] { launch(k_cg_step<real, 1>, 1, 64, 0, fin); });
          return;
        }
        prof_launch("hv_cgram", (double)h.D * KP * KP * rs + (double)h.D * KP * rs * 4, [&] {
          launch(k_hv_cgram<real, KP, 2>, mfill(k_hv_cgram<real, KP, 2>, grid_for(h.D, 4 * Gm::NSG, 1024)), BLOCK, 0, (uint64_t)h.D, gram_of(h), fin,
                 (const uint8_t *)nullptr);
        });
        allreduce_dev(acc_.p, h.D * kp_);
        const uint64_t nv = h.D * KP / Gm::VE;
        prof_launch("hv_fin", (double)h.D * KP * rs * (it > 1 ? 9 : 4),
                    [&] { launch(k_fin<real, KP, 1>, grid_for(nv, BLOCK, 2048), BLOCK, 0, nv, fin); });
      });
      return;
    }
    if (pgram(h)) {
      pair_pass(h, it);
      return;
    }
    const bool fz_ = fused_rows(h);
    with_kp(kp_, [&](auto K) {
      constexpr int KP = decltype(K)::value;
      using Gm = Geo<real, KP>;
      const double rs = sizeof(real);
      DevField<real> &F = *h.F;
      const Fin<real> fin = make_fin(h, it);
      if (own.R) {
        if (h.cross) {
          const size_t qsz = (size_t)KP * KP * sizeof(real);
          const bool lds = qsz <= 32 * 1024;
          const size_t smem = lds ? qsz : 0;
          const double bytes = (double)own.R * 16 + (double)F.nnz * (4 + rs) + (double)F.D * KP * rs +
                               (double)own.npos * 4 + (double)h.partner->R * KP * rs + (double)own.R * KP * rs;
          // tau on the matrix cores (kernels.hpp TauTile) where the rows take
          // it per row: fp32, QTQ in LDS, no column tau, no hot rows, segment order
          const bool tt = tau_mfma_ && TauTile<real, KP>::OK && lds && !coltau(h) && !hot(h) && !sord(own);
          auto go = [&](auto ml) {
            constexpr bool ML = decltype(ml)::value;
            auto go2 = [&](auto pw) {
              constexpr int PW = decltype(pw)::value;
              auto go3 = [&](auto ttc) {
                constexpr bool TT = decltype(ttc)::value && ML && TauTile<real, KP>::OK;
                const size_t sm = TT ? TauTile<real, KP>::bytes() : smem;
                unsigned grid = TT ? grid_for(own.nseg, TauTile<real, KP>::SB, hs_blocks_)
                                   : grid_for(own.nseg, 4 * Gm::NSG, hs_blocks_);
                if (row_fill_) grid = std::min(grid, resident(k_hs_cross_seg<real, KP, ML, PW, TT>, sm));
                launch(k_hs_cross_seg<real, KP, ML, PW, TT>, grid, BLOCK, sm,
                       own.nseg, own.segs.p, F.xptr.p, F.xidx.p, F.xval.p, Vd_.p, own.ycol.p, h.Q1,
                       (uint64_t)h.partner->R, coltau(h) ? (const real *)nullptr : (const real *)qtq_, w_, h_.p, run,
                       Rv_.p, Hv_.p, st_.p, it, F.segd.p, F.segx.p,
                       hot(h) ? (const uint32_t *)own.hot_seg.p : (const uint32_t *)nullptr, (const real *)hotG_.p,
                       sord(own));
              };
              if (tt) go3(std::true_type());
              else go3(std::false_type());
            };
            if constexpr (Gm::LPR <= 16) {
              if (own.short_segs) {
                go2(std::integral_constant<int, 16>());
                return;
              }
            }
            go2(std::integral_constant<int, 32>());
          };
          prof_launch("hs_cross_row", bytes, [&] {
            if (lds) go(std::true_type());
            else go(std::false_type());
          });
        } else {
          const double n1 = hess_n1(h);
          const double bytes = (double)own.R * 16 + (double)F.nnz * (4 + rs) + (double)F.D * KP * rs +
                               (double)own.R * KP * rs * 2;
          auto go = [&](auto fz, auto sc) {
            constexpr bool FZ = decltype(fz)::value, SC = decltype(sc)::value;
            unsigned grid = grid_for(own.R, 4 * Gm::NSG, FZ ? 2048u : 4096u);
            if (side_fill_) grid = std::min(grid, resident(k_hs_side_row<real, KP, FZ, SC>, 0));
            launch(k_hs_side_row<real, KP, FZ, SC>, grid, BLOCK, 0,
                own.R, F.xptr.p, F.xidx.p, F.xval.p, Vd_.p, hess_cnt(h), h.Q1, w_, n1, h_.p, run, Rv_.p, Hv_.p, st_.p, it,
                F.one, fin);
          };
          prof_launch(fz_ ? "hs_side_fused" : "hs_side_row", bytes, [&] {
            if (fz_) go(std::true_type(), std::false_type());
            else if (scat_rows(h)) go(std::false_type(), std::true_type());
            else go(std::false_type(), std::false_type());
          });
        }
      }
    });
    if (!fz_) feature_pass(h, it, h.cross, !h.cross && scat_rows(h));
  }

  // One half of a block: gradient, Newton-CG, update (ffm.cpp:826-832, 843-849).
  void half(uint32_t f1, uint32_t f2, int which) {
    HalfCtx h = half_ctx(f1, f2, which);
    hipEvent_t hb = nullptr;
    if (profiling && prof_filter.empty()) {
      hb = ev();
      HIPCHK(hipEventRecord(hb, stream_));
    }
    // The verdicts of this half start unknown (0); the finalising kernels
    // publish RUN_GO / RUN_STOP into the host-mapped words (kernels.hpp
    // cg_publish).  Nothing of the previous half can still write them: its
    // last verdict has been read and the iterations queued past it are no-ops.
    std::memset(run_host_, 0, sizeof(int) * (MAXCG + 2));
    std::atomic_thread_fence(std::memory_order_seq_cst);
    // CG with `lookahead_` iterations in flight (see file header): iteration
    // it is enqueued before the host waits for iteration it-L's verdict, so
    // the GPU never waits on the host.  Iterations past the real exit run as
    // no-ops.  The count of iterations that ran is the last t with run[t].
    // The host polls the verdict words instead of synchronising on events:
    // an event recorded between two CG steps cost ~5 us of GPU idle per step
    // (measured: 6.7 us vs 1.1 us at the boundaries without one).
    int nr = 0, known = 0;
    bool done = false, gave_up = false;
    auto examine = [&](int upto) {
      for (int q = known + 1; q <= upto && q <= MAXCG && !done; q++) {
        const int v = host_wait([&] { return poll_verdict(q); });
        if (v == CGP_GAVE_UP) {
          gave_up = true;
          return;
        }
        if (v != RUN_GO) done = true;
        else nr = q;
        known = q;
      }
    };
    // Speculative update (look-ahead 1): a half's CG count is
    // nearly always that of the same half in the previous epoch.  At that
    // iteration the update is queued in place of the next (usually no-op)
    // CG step, guarded on the device by run[pred+1]: it runs only if the
    // solve stopped by then, and returns at entry if the solve went on (the
    // host then sees the verdict and carries on with the CG loop).  A hit
    // saves the trailing no-op row pass + feature pass (~9 us per half).
    // The verdicts are global, so on several ranks every rank predicts and
    // queues the same sequence (the update itself has no collective).
    const size_t key = (size_t)h.b12 * 2 + (size_t)which;
    const bool io = io_half(h);  // (its update needs the all-gathered S and p: no speculative update)
    const int pred = !spec_on_ || lookahead_ != 1 || io ? 0
                     : spec_fixed_ > 0                ? spec_fixed_
                     : key < pred_.size()             ? pred_[key]
                                                      : 0;
    bool queued = false;
    const size_t pend0 = pending_.size();
    const int last = key < pred_.size() ? pred_[key] : 0;
    ccg_now_ = ccg_eligible(h) && (ccg_mode_ == 2 || last >= 3);
    hot_now_ = last >= hot_steps_;
    int it0 = 1;
    const int sfull = sidep_smax(h, true);
    if (sfull) {
      // the whole half in one launch (k_cg_side_id FULL): gradient, CG and
      // update; if the grid gave up (at the gradient's barrier too) the
      // host continues per step from the state it wrote back, and updates
      prof_tag_ = 1;
      side_persist(h, sfull, true);
      prof_tag_ = 0;
      ysum_ok_[h.user ? 1 : 0] = false;  // (the update moves this side's bias: finish_half's bookkeeping)
      examine(MAXCG);
      queued = true;
      if (gave_up) it0 = cgp_recover(examine, gave_up, queued);
      if (profiling && pending_.size() > pend0) {  // its bytes: the gradient, the steps and the update that ran
        const double rs = sizeof(real), k = (double)kp_, R = (double)h.own->R;
        const int steps = it0 > 1 ? it0 - 1 : nr;
        for (size_t q = pend0; q < pending_.size(); q++)
          if (pending_[q].name == "side_half")
            pending_[q].bytes = R * (8 + 4 + rs + 16 + 3 * rs) + (double)h.own->nseg * (16 + rs) +
                                (double)h.D * k * rs * 3 + 2 * R * k * rs + (steps + 2) * R * k * rs;
      }
    } else {
      gradient(h);
      col_grams(h);
      hot_grams(h, xfuse(h));
      if (io) io_begin(h);
    }
    const bool pcg = !sfull && cgp_ok(h);
    const int smax = pcg || sfull ? 0 : sidep_smax(h);
    if (pcg || smax) {
      // the whole CG in one persistent launch, the update queued right
      // behind it (no speculation, no host round trip inside the half); the
      // update returns at entry if the grid gave up on its barrier
      prof_tag_ = 1;
      const bool launched = pcg ? cg_persist(h) : side_persist(h, smax);
      prof_tag_ = 0;
      if (launched) {
        finish_half(h, cgp_abort_.p);
        queued = true;
        examine(MAXCG);
        if (gave_up) it0 = cgp_recover(examine, gave_up, queued);
        if (profiling && pending_.size() > pend0) {  // its bytes: the steps that ran in it
          for (size_t q = pend0; q < pending_.size(); q++)
            if (pending_[q].name == "cg_cgram")
              pending_[q].bytes = (double)(it0 > 1 ? it0 - 1 : nr) * cgp_step_bytes(h);
        }
      }
    }
    for (int it = it0; it <= MAXCG && !done && !queued; it++) {
      prof_tag_ = it;
      hv_pass(h, it);
      prof_tag_ = 0;
      const int t = it - lookahead_;
      if (t >= 1) examine(t + 1);  // upd(t) decided run[t+1]
      if (!done && it == pred && it < MAXCG) {
        prof_tag_ = -1;
        finish_half(h, &st_.p->run[it + 1]);
        prof_tag_ = 0;
        examine(it + 1);
        queued = done;  // stopped by iteration pred: the guarded update is the one that runs
      }
    }
    if (!done) examine(MAXCG);
    if (io) io_end(h);
    if (!queued) finish_half(h, nullptr);
    if (key >= pred_.size()) pred_.resize(key + 1, 0);
    pred_[key] = nr;
    // profiling: launches that returned at entry (CG steps past the exit, a
    // speculative update of a solve that went on) move no bytes; they are
    // kept apart under "<family>.noop" so a family's rate counts real work
    for (size_t q = pend0; q < pending_.size(); q++) {
      Pending &e = pending_[q];
      if (e.tag > nr || (e.tag == -1 && !queued)) e.name += ".noop";
    }
    ccg_now_ = hot_now_ = false;
    cg_log.push_back(nr);
    account_half(h, nr);
    if (hb) {
      hipEvent_t he = ev();
      HIPCHK(hipEventRecord(he, stream_));
      char name[32];
      std::snprintf(name, sizeof(name), "half(%u,%u)%c", f1, f2, which ? 'H' : 'W');
      pending_.push_back({name, 0.0, hb, he, 0, 0.0});
    }
  }

  // The end of a half: apply S (W += S, the last pending S += alpha p) and
  // update P, the biases and y~ (ffm.cpp:826-832, 843-849).  skip non-null:
  // a speculative update, whose kernels return at entry when *skip is set.
  void finish_half(HalfCtx &h, const int *skip) {
    DevSide<real> &own = *h.own;
    // a cross update moves the base; a side update moves this side's bias,
    // which the other side's segment sums hold (k_seg_ysum)
    if (h.cross) ysum_dirty();
    else ysum_ok_[h.user ? 1 : 0] = false;
    with_kp(kp_, [&](auto K) {
      constexpr int KP = decltype(K)::value;
      using Gm = Geo<real, KP>;
      const double rs = sizeof(real);
      const uint64_t nv = h.D * KP / Gm::VE;
      const bool excl = h.F->excl;
      if (excl) owned_stale_ = true;
      // id-like field: each feature's row does its k_apply work in the update
      // kernel (apply_owned_row), one launch fewer at the end of the half
      DevField<real> &F = *h.F;
      const bool fold = F.idlike && own.R > 0 && !excl && !no_fold_;
      // any other field on one rank's rows kernel: k_apply folded in too
      // (kernels.hpp fold_apply: W += S + a p by a grid stride, the rows
      // form XS from S + a p), one launch fewer per half
      const bool rows_kernel = !h.cross || (excl_.on && excl_.b12 == h.b12);
      const bool gfold = !fold && own.R > 0 && !excl && !no_fold_ && gfold_on_ && rows_kernel;
      real *Wf = (fold || gfold) ? h.W1 : nullptr;
      const uint64_t nfold = gfold ? nv : 0;
      const double fbytes = gfold ? (double)h.D * KP * rs * 4 : 0.0;
      if (!fold && !gfold)
        prof_launch("apply_step", (double)h.D * KP * rs * 5, [&] {
          launch(k_apply<real>, grid_for(nv, BLOCK, 2048), BLOCK, 0, nv, Vd_.p, S_.p, h.W1, st_.p,
                 excl ? (const uint8_t *)h.F->own.p : nullptr, (uint32_t)Gm::LPR, skip);
        });
      if (own.R == 0) return;
      if (h.cross) {
        DevSide<real> &other = *h.partner;
        if (excl_.on && excl_.b12 == h.b12) {
          // block-excluded base: the base does not depend on P1, no positive pass
          prof_launch("update_cross_rows", (double)own.R * 16 + (double)F.nnz * (4 + rs) + (double)F.D * KP * rs +
                                               (double)own.R * KP * rs * 2 + fbytes, [&] {
            launch(k_update_cross_rows<real, KP>, mfill(k_update_cross_rows<real, KP>, grid_for(own.R, 4 * Gm::NSG)), BLOCK, 0, own.R, F.xptr.p, F.xidx.p,
                   F.xval.p, (const real *)S_.p, h.P1, (real *)nullptr, F.one, Wf, (const real *)Vd_.p,
                   (const CgState *)st_.p, skip, nfold);
          });
          return;
        }
        const double bytes = (double)own.R * 16 + (double)F.nnz * (4 + rs) + (double)F.D * KP * rs +
                             (double)own.R * KP * rs * 2 + (double)own.npos * (4 + 2 * rs) +
                             (double)other.R * KP * rs;
        prof_launch("update_cross_row", bytes, [&] {
          launch(k_update_cross_seg<real, KP>, mfill(k_update_cross_seg<real, KP>, grid_for(own.nseg, 4 * Gm::NSG)), BLOCK, 0,
              own.nseg, own.segs.p, F.xptr.p, F.xidx.p, F.xval.p, S_.p, h.P1, own.ycol.p, own.yt.p, h.Q1,
              (uint64_t)other.R, F.segd.p, F.segx.p, Wf,
              (const real *)Vd_.p, (const CgState *)st_.p, (const real *)nullptr, (const real *)nullptr,
              (const real *)nullptr, skip);
        });
        refresh_other(own, other, skip);  // the other orientation by a gather through perm
      } else {
        DevSide<real> &other = h.user ? V_ : U_;
        const double bytes = (double)own.R * 16 + (double)F.nnz * (4 + rs) + (double)F.D * KP * rs +
                             (double)own.R * KP * rs * 3 + (double)own.R * rs * 2 + (double)own.npos * (4 + 4 * rs) + fbytes;
        prof_launch("update_side_row", bytes, [&] {
          launch(k_update_side_row<real, KP>, mfill(k_update_side_row<real, KP>, grid_for(own.R, 4 * Gm::NSG)), BLOCK, 0,
              own.R, F.xptr.p, F.xidx.p, F.xval.p, S_.p, h.P1, h.Q1, own.bias.p, F.one, Wf,
              (const real *)Vd_.p, (const CgState *)st_.p, bsum_.p + (h.user ? 0 : 1), part_.p, tick_.p, skip, nfold);
        });
      }
    });
  }

  // Algorithmic bytes of one half (SURVEY §8d formula, s = sizeof(real)).
  void account_half(const HalfCtx &h, int c) {
    const double s = sizeof(real), k = (double)kp_;
    const double R = (double)h.own->R, D = (double)h.D, P = (double)h.own->npos;
    const double csr = 8 * R + (double)h.F->nnz * (4 + s);
    if (!h.cross) {
      const double Rp = (double)(h.user ? V_.R : U_.R);
      const double gd = P * s + 8 * R + 2 * R * s + Rp * s + R * k * s + csr + 2 * D * k * s;
      const double hs = c * (8 * R + R * k * s + csr + 9 * D * k * s);
      const double upd = 4 * D * k * s + csr + 3 * R * k * s + 2 * R * s + 2 * P * s + 8 * R;
      alg_bytes += gd + hs + upd;
    } else {
      const double Rp = (double)h.partner->R, Cc = (double)C_;
      const double gd = (Cc + 2) * Rp * k * s + Rp * s + Cc * R * k * s + 8 * R + P * (4 + s) + R * s + csr +
                        2 * D * k * s;
      const double hs = Rp * k * s + c * (csr + 8 * R + 4 * P + Rp * k * s + 9 * D * k * s);
      const double upd = 4 * D * k * s + csr + 2 * R * k * s + 2 * P * s + 4 * P + 8 * R + Rp * k * s;
      alg_bytes += gd + hs + upd;
    }
  }

  // ------------------------------------------------------------- state
  ocffm_param prm_;
  Comm comm_;
  // Several ranks: per-item positive counts and the user count over all
  // ranks.  An item side half's Hessian is a function of these and of the
  // replicated item tables only, so its CG steps run on every rank in full
  // with no all-reduce (repl()); its gradient is still a sum over users.
  DevBuf<int64_t> gvptr_;
  double gn1_ = 0;
  bool has_test_;
  bool inited_ = false;
  hipStream_t stream_ = nullptr;
  uint32_t k_, kp_, fu_, fv_, f_, C_ = 0;
  double w_, lam_, r_;
  uint64_t m_glob_ = 0, n_ = 0, u0_ = 0, u1_ = 0, dmax_ = 0, npop_ = 0;
  // positives per segment: fp64 48 (8.99 -> 8.89 ms per kkbox epoch at the
  // 10-epoch command: fewer segments for the feature passes to sum), fp32 32
  // (48: within noise; 64: slower gradient passes)
  uint64_t seg_len_ = std::is_same<real, double>::value ? 48 : 32;

  int lookahead_ = 1;
  // speculative update at the previous epoch's CG count (OCFFM_SPEC=0: off)
  bool spec_on_ = !std::getenv("OCFFM_SPEC") || std::atoi(std::getenv("OCFFM_SPEC")) != 0;
  std::vector<int> pred_;  // per (block, half): CG count of the last solve
  // Segment sums of base + partner bias for the side gradient passes
  // (k_seg_ysum); [0] user rows, [1] item rows.  OCFFM_YSUM=0: the passes
  // walk their positives every time.
  bool ysum_on_ = !std::getenv("OCFFM_YSUM") || std::atoi(std::getenv("OCFFM_YSUM")) != 0;
  // CG residual |r|^2 recomputed by a second reduction (k_cg_r2) instead of
  // the expanded scalar of the finalisation (OCFFM_EXACT_R2=1)
  bool exact_r2_ = std::getenv("OCFFM_EXACT_R2") && std::atoi(std::getenv("OCFFM_EXACT_R2")) != 0;
  bool ysum_ok_[2] = {false, false};
  DevBuf<real> yrow_;                 // per-row totals of the segment sums (k_row_ysum)
  bool yrow_ok_[2] = {false, false};  // (valid only with ysum_ok_ of the side)
  // Cross loop: the item halves read the block-excluded value through perm
  // from the user orientation (k_gd_cross_seg ytv) instead of a refresh after
  // each entering pass.  OCFFM_YTVIA=0: refresh.
  // OCFFM_GFOLD=0: k_apply as its own launch for fields that are not id-like
  bool gfold_on_ = !std::getenv("OCFFM_GFOLD") || std::atoi(std::getenv("OCFFM_GFOLD")) != 0;
  bool ytvia_ = !std::getenv("OCFFM_YTVIA") || std::atoi(std::getenv("OCFFM_YTVIA")) != 0;
  // OCFFM_SIDE_REFRESH=1: the entering pass's refresh of the item orientation
  // runs on a second stream, overlapped with the user half's CG; the block's
  // item half then reads the stored value in order (no perm gather)
  bool side_refresh_ = std::getenv("OCFFM_SIDE_REFRESH") && std::atoi(std::getenv("OCFFM_SIDE_REFRESH")) != 0;
  hipStream_t side_ = nullptr;
  hipEvent_t side_ev_[2] = {nullptr, nullptr};
  bool side_pending_ = false;
  // T_i of the cross gradient passes precomputed on MFMA (k_rows_T; fp32,
  // KP = 32 or 64).  On where the C cross Grams exceed the pass's 64 KB of
  // LDS (BASELINE config 5: 39 Grams of 64 x 64, 624 KB: the pass would read
  // them from L2 for every row); elsewhere opt-in (OCFFM_TPRE=1): measured a
  // wash at kkbox shape (the pass gets 25 / 13 us faster per item /
  // user half, the pre-pass costs 26.8 / 10.8 us: it must read the C tables'
  // rows, 77 MB on the item half, which the pass had overlapped with its gathers).
  bool tpre_on_ = std::getenv("OCFFM_TPRE") && std::atoi(std::getenv("OCFFM_TPRE")) != 0;
  DevBuf<real> Tpre_;
  // grid cap: one 512-thread block per CU (128 KB of LDS each)
  unsigned tpre_blocks_ = std::getenv("OCFFM_TPRE_BLOCKS") ? (unsigned)std::max(1, std::atoi(std::getenv("OCFFM_TPRE_BLOCKS"))) : 256;
  // T_i as an MFMA pre-pass (k_rows_T): where the C Grams do not fit the
  // gradient pass's LDS, or where the rows carry few positives (< 4 per row
  // on average: the pass is then mostly its T_i work; outbrain's 250 k
  // users with ~1.2 each: gd_cross_row 193 -> 61 us + rows_T 71 us), or
  // OCFFM_TPRE=1
  bool tpre(uint64_t R, uint64_t npos) const {
    const bool big = (size_t)C_ * kp_ * kp_ * sizeof(real) > 64 * 1024;
    const bool few = tpre_few_ && R >= 65536 && npos < 4 * R;
    return (tpre_on_ || big || few) && std::is_same<real, float>::value && (kp_ == 32 || kp_ == 64) && C_ >= 1 &&
           R > 0 && (uint64_t)R * kp_ * sizeof(real) < 0xffffff00ull && !no_mfma_;
  }
  bool tpre_few_ = !std::getenv("OCFFM_TPRE_FEW") || std::atoi(std::getenv("OCFFM_TPRE_FEW")) != 0;
  DevBuf<real> ysum_;
  void ysum_dirty() { ysum_ok_[0] = ysum_ok_[1] = false; }
  // hot rows: positives per row from which a cross half reads a per-row
  // Gram (OCFFM_HOT, default 2 KP; 0: off), the Grams and partial slots
  uint64_t hot_min_ = 0;
  DevBuf<real> hotG_, hotP_;
  int hot_steps_ = 6;
  bool hot_env_ = false;  // OCFFM_HOT set: the per-step cross passes read hot rows' Grams
  bool hot_now_ = false;
  // default: on where the build runs on MFMA (fp32, KP 32 / 64); the fp64
  // VALU build measured slower than the steps it saves
  // (default on where the builds run on the matrix cores: fp32 at KP 32 / 64,
  // fp64 at KP 32, ccg_pred)
  int ccg_mode_ = std::getenv("OCFFM_CCG") ? std::atoi(std::getenv("OCFFM_CCG"))
                  : std::getenv("OCFFM_NO_MFMA") == nullptr ? 1 : 0;
  bool ccg_now_ = false;  // this cross half's CG steps run on per-column Grams
  DevBuf<real> ccgG_, ccgP_;  // the column Grams of the current half (max D KP^2), their partial slots
  // OCFFM_SPEC_FIXED=n (tests): predict n for every half (hits and misses of every kind)
  int spec_fixed_ = std::getenv("OCFFM_SPEC_FIXED") ? std::atoi(std::getenv("OCFFM_SPEC_FIXED")) : 0;
  bool fuse_ = true;
  // OCFFM_COLTAU=0: the tau term of cross Hessian-vector rows per row (k_hs_cross_seg)
  bool coltau_on_ = !std::getenv("OCFFM_COLTAU") || std::atoi(std::getenv("OCFFM_COLTAU")) != 0;
  // OCFFM_NO_FOLD=1: k_apply as its own launch on id-like fields too
  bool no_fold_ = std::getenv("OCFFM_NO_FOLD") != nullptr;
  // OCFFM_CGRAM: side halves of one-node-per-row fields run their CG steps
  // on per-column Grams where cgram_pays() (1, default), never (0), or
  // wherever the structure allows (2).
  int cgram_mode_ = std::getenv("OCFFM_CGRAM") ? std::atoi(std::getenv("OCFFM_CGRAM")) : 1;
  bool cgram_on_ = cgram_mode_ != 0;
  // OCFFM_CGRAM_CHUNK: rows per k_col_gram block, capped at one LDS stage
  // (cgram_rows: 256 rows at k = 32 fp32)
  uint64_t cgram_chunk_ = std::getenv("OCFFM_CGRAM_CHUNK") ? std::max(1, std::atoi(std::getenv("OCFFM_CGRAM_CHUNK"))) : 128;
  bool no_mfma_ = std::getenv("OCFFM_NO_MFMA") != nullptr;  // Grams on the VALU kernel instead
  DevBuf<float> gpart64_;  // k_gram_mfma64 partials
  DevBuf<double> gpartd_;  // k_gram_mfma_f64 partials
  // OCFFM_TAU_MFMA=0: the cross Hessian-vector row pass takes tau by sg_vecmat (VALU) instead of MFMA tiles
  bool tau_mfma_ = !std::getenv("OCFFM_TAU_MFMA") || std::atoi(std::getenv("OCFFM_TAU_MFMA")) != 0;
  // OCFFM_XCD_ORDER=0: the Gram kernels' blocks in plain order (no XCD-aware remap)
  bool xcd_order_ = !std::getenv("OCFFM_XCD_ORDER") || std::atoi(std::getenv("OCFFM_XCD_ORDER")) != 0;
  uint64_t gram64_blocks_ = std::getenv("OCFFM_GRAM64_BLOCKS") ? std::strtoull(std::getenv("OCFFM_GRAM64_BLOCKS"), nullptr, 10) : 1024;
  uint64_t gram_blocks_ = std::getenv("OCFFM_GRAM_BLOCKS") ? std::strtoull(std::getenv("OCFFM_GRAM_BLOCKS"), nullptr, 10) : 512;
  bool no_owned_ = false;
  // OCFFM_HOST_BUILD=1: the data layout built on the host (the checker of
  // the device build, devbuild.h)
  bool host_build_ = std::getenv("OCFFM_HOST_BUILD") != nullptr && std::atoi(std::getenv("OCFFM_HOST_BUILD")) != 0;
  bool host_init_ = std::getenv("OCFFM_HOST_INIT") != nullptr && std::atoi(std::getenv("OCFFM_HOST_INIT")) != 0;
  bool owned_stale_ = false;  // owned tables differ across ranks until sync_owned()
  unsigned hs_blocks_ = 4096;  // grid cap of the cross Hessian-vector row pass
  unsigned feat_blocks_ = 1024;  // grid cap of the feature pass (grid-stride over jobs)
  hipEvent_t arm_a_ = nullptr, arm_b_ = nullptr;
  bool arm_first_ = false;
  DevSide<real> U_, V_, T_;
  std::vector<Block> blocks_;
  std::vector<DevBuf<real>> W_, H_, P_, Q_;
  DevBuf<real> acc_, G_, S_, Vd_, Rv_, Hv_, h_, M_, wpart_;
  DevBuf<double> bsum_;  // sums of a and b (bias_sums)
  // Block-excluded y~: while `on`, both orientations of the
  // stored base hold y~ - <P_b12[i], Q_b12[j]>; the cross halves of block
  // b12 then update P/Q without a positive pass.  flush_base() restores it.
  struct ExclBase {
    bool on = false;
    uint32_t b12 = 0;
  } excl_;
  bool lazy_ok_ = false;  // set by one_epoch around its cross halves
  // OCFFM_LAZY_BASE=0: every cross update applies its base change at once
  bool lazy_base_ = !std::getenv("OCFFM_LAZY_BASE") || std::atoi(std::getenv("OCFFM_LAZY_BASE")) != 0;
  // grid cap of the cross gradient pass (each block stages the C aggregates M in LDS)
  unsigned gd_blocks_ = std::getenv("OCFFM_GD_BLOCKS") ? (unsigned)std::atoi(std::getenv("OCFFM_GD_BLOCKS")) : 2048u;
  bool gd_fill_ = !std::getenv("OCFFM_GD_FILL") || std::atoi(std::getenv("OCFFM_GD_FILL")) != 0;
  bool feat_fill_ = !std::getenv("OCFFM_FEAT_FILL") || std::atoi(std::getenv("OCFFM_FEAT_FILL")) != 0;
  // hs rows: fp32 (outbrain / kdd12 hs_cross -4 %, kkbox neutral); the fp64
  // hs_cross measured 1.6 % slower at its resident wave than at the cap
  bool row_fill_ = std::getenv("OCFFM_ROW_FILL") ? std::atoi(std::getenv("OCFFM_ROW_FILL")) != 0
                                                 : std::is_same<real, float>::value;
  // the side rows (k_hs_side_row): both precisions (fp64 kkbox -0.3 %)
  bool side_fill_ = !std::getenv("OCFFM_SIDE_FILL") || std::atoi(std::getenv("OCFFM_SIDE_FILL")) != 0;
  bool want_g_ = false;  // grad(): the gradient finalisation also stores G
  const real *qtq_ = nullptr;  // this cross half's Q^T Q: a slot of M_
  DevBuf<unsigned> tick_;
  DevBuf<double> sums_, vecs_, part_, at_d_, popular_;
  DevBuf<uint8_t> cold_;
  DevBuf<CgState> st_;
  DevBuf<real *> tabs_;
  int *run_host_ = nullptr, *run_host_dev_ = nullptr;
  // persistent column-Gram CG (k_cg_cgram, OCFFM_CGP): the grid's release
  // word (monotonic across launches), the CU count that bounds its grid
  DevBuf<unsigned> cgp_gen_buf_;
  DevBuf<int> cgp_abort_;  // 1: the last persistent grid gave up (guards its queued update)
  unsigned cgp_gen_ = 1, ncu_ = 256;
  bool cgp_on_ = !std::getenv("OCFFM_CGP") || std::atoi(std::getenv("OCFFM_CGP")) != 0;
  // OCFFM_CGP_XCD=0: k_cg_cgram's columns grid-strided instead of XCD-contiguous ranges
  bool cgp_xcd_ = !std::getenv("OCFFM_CGP_XCD") || std::atoi(std::getenv("OCFFM_CGP_XCD")) != 0;
  // OCFFM_SIDEP=0: id-like side halves' CG per step (k_hs_side_row FUSE) instead of k_cg_side_id
  bool sidep_on_ = !std::getenv("OCFFM_SIDEP") || std::atoi(std::getenv("OCFFM_SIDEP")) != 0;
  // OCFFM_SIDE_FULL=0: id-like side halves run gradient and update as their own launches around k_cg_side_id
  bool sidef_on_ = !std::getenv("OCFFM_SIDE_FULL") || std::atoi(std::getenv("OCFFM_SIDE_FULL")) != 0;
  // OCFFM_XFUSE=0: id-like cross halves' CG steps as k_hs_cross_seg + feature pass instead of k_hv_cross_id
  bool xfuse_on_ = !std::getenv("OCFFM_XFUSE") || std::atoi(std::getenv("OCFFM_XFUSE")) != 0;
  // gathers per round (8 or 16; fp64 moves half as many rows per round at
  // the same registers: 16 there, at ~163 registers, 8.72 -> 8.57 ms per epoch)
  int xf_gb_ = std::getenv("OCFFM_XF_GB") ? std::atoi(std::getenv("OCFFM_XF_GB")) : (sizeof(real) == 8 ? 16 : 8);
  // OCFFM_CGP_COOP=1: cooperative launch (the runtime's residency check; +0.27 ms per kkbox epoch)
  bool cgp_coop_ = std::getenv("OCFFM_CGP_COOP") && std::atoi(std::getenv("OCFFM_CGP_COOP")) != 0;
  // tests: a short spin limit and one block stalled at a given step force the give-up
  unsigned cgp_spin_ = std::getenv("OCFFM_CGP_SPIN") ? (unsigned)std::atol(std::getenv("OCFFM_CGP_SPIN")) : CGP_SPIN_MAX;
  int cgp_stall_ = std::getenv("OCFFM_CGP_STALL") ? std::atoi(std::getenv("OCFFM_CGP_STALL")) : -1;
  real *stage_ = nullptr;
  static constexpr uint64_t DSTAGE = 64;
  double *dstage_ = nullptr;  // host all-reduce stage of the owned-field dot products
  DevBuf<double> dots_;
  struct Pending {
    std::string name;
    double bytes;
    hipEvent_t a, b;
    int tag;  // CG iteration of a Hessian-vector launch, -1 a speculative update, 0 other
    double flops;
  };
  int prof_tag_ = 0;
  std::vector<Pending> pending_;
  std::vector<hipEvent_t> ev_pool_, ev_free_;
};

}  // namespace ocffm

// ====================================================================== ABI
using namespace ocffm;

struct ocffm_problem {
  std::unique_ptr<ProblemBase> p;
};

extern "C" {

void ocffm_param_default(ocffm_param *p) {
  p->omega = 0.1;
  p->lambda = 1e-5;
  p->r = -1;
  p->nr_pass = 20;
  p->k = 4;
  p->nr_threads = 1;
  p->self_side = 1;
  p->freq = 0;
  p->precision = OCFFM_FP64;
  p->device = 0;
}

const char *ocffm_last_error(void) { return g_last_error.c_str(); }

int ocffm_device_count(int *count) {
  return guarded([&] {
    int c = 0;
    hipError_t e = hipGetDeviceCount(&c);
    *count = e == hipSuccess ? c : 0;
  });
}

int ocffm_data_read(const char *path, int has_label, const uint64_t *ds, uint32_t nds, ocffm_data **out) {
  return guarded([&] {
    auto d = std::make_unique<ocffm_data>();
    build(d->d, parse_rows(path, has_label != 0, ds, nds));
    d->d.path = path;
    *out = d.release();
  });
}

int ocffm_data_from_rows(uint64_t m, const uint64_t *xptr, const uint32_t *fid, const uint64_t *idx,
                         const double *val, const uint64_t *yptr, const uint64_t *ycol, const uint64_t *ds,
                         uint32_t nds, ocffm_data **out) {
  return guarded([&] {
    Rows r;
    r.has_label = yptr != nullptr;
    const uint64_t nn = xptr[m] - xptr[0];
    for (uint64_t p = xptr[0]; p < xptr[m]; p++) r.f = std::max<uint64_t>(r.f, (uint64_t)fid[p] + 1);
    if (ds == nullptr) {  // every node kept: the arrays as given
      r.xptr.resize(m + 1);
      for (uint64_t i = 0; i <= m; i++) r.xptr[i] = xptr[i] - xptr[0];
      r.fid.assign(fid + xptr[0], fid + xptr[m]);
      r.idx.assign(idx + xptr[0], idx + xptr[m]);
      r.val.assign(val + xptr[0], val + xptr[m]);
    } else {
      r.fid.reserve(nn);
      r.idx.reserve(nn);
      r.val.reserve(nn);
      r.xptr.reserve(m + 1);
      for (uint64_t i = 0; i < m; i++) {
        for (uint64_t p = xptr[i]; p < xptr[i + 1]; p++) {
          if (fid[p] >= nds || ds[fid[p]] <= idx[p]) continue;
          r.fid.push_back(fid[p]);
          r.idx.push_back(idx[p]);
          r.val.push_back(val[p]);
        }
        r.xptr.push_back(r.fid.size());
      }
    }
    if (r.has_label) {
      r.yptr.resize(m + 1);
      for (uint64_t i = 0; i <= m; i++) r.yptr[i] = yptr[i] - yptr[0];
      r.ycol.assign(ycol + yptr[0], ycol + yptr[m]);
      for (uint64_t j : r.ycol) r.n = std::max<uint64_t>(r.n, j + 1);
    }
    auto d = std::make_unique<ocffm_data>();
    build(d->d, std::move(r));
    *out = d.release();
  });
}

int ocffm_data_trans_y(ocffm_data *V, const ocffm_data *U) {
  return guarded([&] { trans_y(V->d, U->d); });
}

int ocffm_data_get_info(const ocffm_data *d, ocffm_data_info *o) {
  return guarded([&] {
    o->m = d->d.m;
    o->n = d->d.n;
    o->f = d->d.f;
    o->nnz_x = d->d.raw.fid.size();
    o->nnz_y = d->d.ycol.size();
  });
}

int ocffm_data_get_ds(const ocffm_data *d, uint64_t *out) {
  return guarded([&] {
    for (size_t i = 0; i < d->d.Ds.size(); i++) out[i] = d->d.Ds[i];
  });
}

int ocffm_data_get_labels(const ocffm_data *d, uint64_t *yptr, uint64_t *ycol) {
  return guarded([&] {
    if (yptr) std::copy(d->d.yptr.begin(), d->d.yptr.end(), yptr);
    if (ycol) std::copy(d->d.ycol.begin(), d->d.ycol.end(), ycol);
  });
}

int ocffm_data_get_field(const ocffm_data *d, uint32_t field, int64_t *xptr, uint32_t *xidx, double *xval,
                         uint64_t *nnz) {
  return guarded([&] {
    if (field >= d->d.f) throw ocffm::Error(OCFFM_E_ARG, "no such field");
    split_host(d->d);
    if (nnz) *nnz = d->d.xidx[field].size();
    if (xptr) std::copy(d->d.xptr[field].begin(), d->d.xptr[field].end(), xptr);
    if (xidx) std::copy(d->d.xidx[field].begin(), d->d.xidx[field].end(), xidx);
    if (xval) std::copy(d->d.xval[field].begin(), d->d.xval[field].end(), xval);
  });
}

void ocffm_data_free(ocffm_data *d) { delete d; }

static int create_impl(const ocffm_data *U, const ocffm_data *Ut, const ocffm_data *V, const ocffm_param *p,
                       Comm comm, ocffm_problem **out) {
  return guarded([&] {
    if (!U || !V || !p || !out) throw Error(OCFFM_E_ARG, "null argument");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
      throw Error(OCFFM_E_HIP, "no HIP device visible (this build has no CPU fallback)");
    auto pr = std::make_unique<ocffm_problem>();
    const HostData *ut = Ut ? &Ut->d : nullptr;
    if (p->precision == OCFFM_FP32)
      pr->p = std::make_unique<Problem<float>>(U->d, ut, V->d, *p, comm);
#ifndef OCFFM_EXP_KP32
    else if (p->precision == OCFFM_FP64)
      pr->p = std::make_unique<Problem<double>>(U->d, ut, V->d, *p, comm);
#endif
    else
      throw Error(OCFFM_E_ARG, "precision must be 32 or 64");
    *out = pr.release();
  });
}

int ocffm_problem_create(const ocffm_data *U, const ocffm_data *Ut, const ocffm_data *V, const ocffm_param *p,
                         ocffm_problem **out) {
  return create_impl(U, Ut, V, p, Comm{}, out);
}

int ocffm_comm_id(void *out) {
  return guarded([&] {
    static_assert(sizeof(ncclUniqueId) <= OCFFM_COMM_ID_BYTES, "id size");
    ncclUniqueId id;
    NCCLCHK(ncclGetUniqueId(&id));
    std::memset(out, 0, OCFFM_COMM_ID_BYTES);
    std::memcpy(out, &id, sizeof(id));
  });
}

int ocffm_problem_create_dist(const ocffm_data *U, const ocffm_data *Ut, const ocffm_data *V, const ocffm_param *p,
                              int rank, int nranks, const void *comm_id, ocffm_problem **out) {
  Comm c;
  int st = guarded([&] {
    if (nranks < 1 || rank < 0 || rank >= nranks) throw Error(OCFFM_E_ARG, "bad rank/nranks");
    c.rank = rank;
    c.nranks = nranks;
    if (comm_id) {  // RCCL even for one rank: the distributed path, all-reduces included
      HIPCHK(hipSetDevice(p->device));
      ncclUniqueId id;
      std::memcpy(&id, comm_id, sizeof(id));
      NCCLCHK(ncclCommInitRank(&c.nccl, nranks, id, rank));
    }
  });
  if (st != OCFFM_OK) return st;
  st = create_impl(U, Ut, V, p, c, out);
  if (st != OCFFM_OK && c.nccl) ncclCommDestroy(c.nccl);
  return st;
}

int ocffm_problem_create_dist_host(const ocffm_data *U, const ocffm_data *Ut, const ocffm_data *V,
                                   const ocffm_param *p, int rank, int nranks, ocffm_allreduce_fn fn, void *user,
                                   ocffm_problem **out) {
  Comm c;
  c.rank = rank;
  c.nranks = nranks;
  c.host_fn = fn;
  c.host_user = user;
  if (nranks < 1 || rank < 0 || rank >= nranks || !fn) {
    g_last_error = "bad rank/nranks/callback";
    return OCFFM_E_ARG;
  }
  return create_impl(U, Ut, V, p, c, out);
}

#define PROB_CALL(body)                                    \
  return guarded([&] {                                     \
    if (!prob || !prob->p) throw Error(OCFFM_E_ARG, "null problem"); \
    body;                                                  \
  })

int ocffm_problem_init(ocffm_problem *prob) { PROB_CALL(prob->p->init()); }
int ocffm_problem_one_epoch(ocffm_problem *prob) { PROB_CALL(prob->p->one_epoch()); }
int ocffm_problem_solve_block(ocffm_problem *prob, uint32_t f1, uint32_t f2) {
  PROB_CALL(prob->p->solve_block(f1, f2));
}
int ocffm_problem_cache_sasb(ocffm_problem *prob) { PROB_CALL(prob->p->cache_sasb()); }
int ocffm_problem_validate(ocffm_problem *prob, ocffm_metrics *m) { PROB_CALL(prob->p->validate(m)); }
int ocffm_problem_validate_forced(ocffm_problem *prob, ocffm_metrics *m, double *per_row_ndcg, uint64_t cap) {
  PROB_CALL(prob->p->validate(m, true, per_row_ndcg, cap));
}
int ocffm_problem_test_rows(ocffm_problem *prob, uint64_t *m) {
  PROB_CALL(if (!m) throw Error(OCFFM_E_ARG, "null output"); *m = prob->p->test_rows());
}
int ocffm_problem_save_binary(ocffm_problem *prob, const char *path) { PROB_CALL(prob->p->save_binary(path)); }
int ocffm_problem_load_binary(ocffm_problem *prob, const char *path) { PROB_CALL(prob->p->load_binary(path)); }

int ocffm_print_header(void) {
  std::cout << "iter";
  uint32_t s = 5;
  for (int i = 0; i < 5; i++, s *= 2) {
    std::cout.width(9);
    std::cout << "( p@ " << s << ", ";
    std::cout.width(6);
    std::cout << "nDCG@" << s << " )";
  }
  std::cout.width(12);
  std::cout << "ploss" << std::endl;
  return OCFFM_OK;
}

int ocffm_print_epoch(const ocffm_metrics *m, uint32_t t) {
  std::cout.width(2);
  std::cout << t + 1;
  if (m) {
    for (int i = 0; i < 5; i++) {
      std::cout.width(9);
      std::cout << "( " << std::setprecision(3) << m->prec[i] * 100 << " ,";
      std::cout.width(6);
      std::cout << std::setprecision(3) << m->ndcg[i] * 100 << " )";
    }
    std::cout.width(13);
    std::cout << std::setprecision(3) << m->loss;
  }
  std::cout << std::endl;
  return OCFFM_OK;
}

// ffm.cpp:1147-1161.
int ocffm_problem_solve(ocffm_problem *prob) {
  PROB_CALL({
    ProblemBase &P = *prob->p;
    const bool talk = P.rank() == 0;
    if (P.has_test() && talk) ocffm_print_header();
    for (uint32_t it = 0; it < P.nr_pass(); it++) {
      P.one_epoch();
      if (P.has_test() && it % 10 == 9) {
        ocffm_metrics m;
        P.validate(&m);
        if (talk) ocffm_print_epoch(&m, it);
      }
    }
  });
}

int ocffm_problem_get(ocffm_problem *prob, char what, uint32_t b12, double *out, uint64_t cap, uint64_t *len) {
  PROB_CALL({
    uint64_t n = prob->p->get(what, b12, out, cap);
    if (len) *len = n;
  });
}
int ocffm_problem_set(ocffm_problem *prob, char what, uint32_t b12, const double *in, uint64_t len) {
  PROB_CALL(prob->p->set(what, b12, in, len));
}
int ocffm_problem_grad(ocffm_problem *prob, uint32_t f1, uint32_t f2, int half, double *out) {
  PROB_CALL(prob->p->grad(f1, f2, half, out));
}
int ocffm_problem_hv(ocffm_problem *prob, uint32_t f1, uint32_t f2, int half, const double *v, double *out) {
  PROB_CALL(prob->p->hv(f1, f2, half, v, out));
}
int ocffm_problem_save_model(ocffm_problem *prob, const char *path) { PROB_CALL(prob->p->save_model(path)); }

int ocffm_problem_cg_log(ocffm_problem *prob, int32_t *out, int cap, int *count) {
  PROB_CALL({
    auto &l = prob->p->cg_log;
    for (int i = 0; i < (int)l.size() && i < cap; i++) out[i] = l[i];
    if (count) *count = (int)l.size();
  });
}
int ocffm_problem_set_profiling(ocffm_problem *prob, int on) { PROB_CALL(prob->p->profiling = on != 0); }
int ocffm_problem_set_profile_filter(ocffm_problem *prob, const char *name) {
  PROB_CALL(prob->p->prof_filter = name ? name : "");
}
int ocffm_problem_kernel_stats(ocffm_problem *prob, ocffm_kernel_stat *out, int cap, int *count) {
  PROB_CALL({
    int i = 0;
    for (auto &kv : prob->p->kstats) {
      if (i < cap && out) {
        std::memset(&out[i], 0, sizeof(ocffm_kernel_stat));
        std::strncpy(out[i].name, kv.first.c_str(), sizeof(out[i].name) - 1);
        out[i].launches = kv.second.launches;
        out[i].total_ms = kv.second.ms;
        out[i].alg_bytes = kv.second.bytes;
        out[i].alg_flops = kv.second.flops;
      }
      i++;
    }
    if (count) *count = i;
  });
}
int ocffm_problem_reset_stats(ocffm_problem *prob) {
  PROB_CALL({
    prob->p->kstats.clear();
    prob->p->cg_log.clear();
    prob->p->alg_bytes = 0;
  });
}
int ocffm_problem_alg_bytes(ocffm_problem *prob, double *bytes) { PROB_CALL(*bytes = prob->p->alg_bytes); }
int ocffm_problem_counter(ocffm_problem *prob, const char *name, int64_t *value) {
  PROB_CALL({
    if (!name || !value) throw Error(OCFFM_E_ARG, "null argument");
    const auto it = prob->p->counters.find(name);
    *value = it == prob->p->counters.end() ? 0 : it->second;
  });
}
int ocffm_problem_sync(ocffm_problem *prob) { PROB_CALL(prob->p->sync()); }
int ocffm_problem_layout_digest(ocffm_problem *prob, char *names, uint64_t *digests, int cap, int *count) {
  return guarded([&] {
    if (!prob || !prob->p || !count) throw Error(OCFFM_E_ARG, "null argument");
    const auto d = prob->p->layout_digest();
    *count = (int)d.size();
    for (int i = 0; i < cap && i < (int)d.size(); i++) {
      if (names) std::snprintf(names + 48 * (size_t)i, 48, "%s", d[i].first.c_str());
      if (digests) digests[i] = d[i].second;
    }
  });
}
void ocffm_problem_destroy(ocffm_problem *prob) { delete prob; }

}  // extern "C"
