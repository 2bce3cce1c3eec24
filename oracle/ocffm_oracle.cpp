// ocffm_oracle.cpp — TEST INFRASTRUCTURE ONLY.
//
// A clean-room CPU restatement (fp64, OpenMP) of the one-class FFM block
// Newton-CG solver of johncreed/one-class-ffm.  It is the checker for the
// product's HIP path: only tests/, __graft_entry__.smoke() and bench.py's
// cpu_baseline leg may load it.  The product library never links or calls it.
//
// Parity status: the reference needs a CBLAS header (OpenBLAS/MKL) that this
// image does not ship, so it cannot be built here.  This
// restatement is pinned by the reference's only known-answer test (the nDCG
// debug tool, script/nDCG_degub_tool/gen_ans.py, fixtures under tests/golden/)
// and by math identities checked in tests/ (gradient and Hessian-vector
// products against finite differences of the reference's objective
// ffm.cpp:1321-1351).  Training-path values are otherwise "parity unpinned"
// against a reference binary.
//
// Every function cites the reference lines it restates.  Data structures are
// our own (per-field CSR arrays instead of Node* vectors).
#include <omp.h>

#include <algorithm>
#include <cassert>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iomanip>
#include <iostream>
#include <memory>
#include <random>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

namespace orc {

// Per-function wall-time accumulators (seconds) for the CPU-baseline breakdown.
enum { T_GD_SIDE, T_GD_CROSS, T_HV, T_CG, T_UPD_SIDE, T_UPD_CROSS, T_SASB, T_N };
static double g_time[T_N];
struct Timer {
  int id;
  double t0;
  explicit Timer(int i) : id(i), t0(omp_get_wtime()) {}
  ~Timer() { g_time[id] += omp_get_wtime() - t0; }
};

using u64 = uint64_t;
using u32 = uint32_t;
using Vec = std::vector<double>;

// ffm.cpp:3-12 — fast inverse square root with magic 0x5fe6eb50c7b537a9 and
// one Newton step; the init bound is 0.1*qrsqrt(k), not 0.1/sqrt(k).
static double qrsqrt(double x) {
  double half = 0.5 * x;
  u64 bits;
  std::memcpy(&bits, &x, 8);
  bits = 0x5fe6eb50c7b537a9ULL - (bits >> 1);
  std::memcpy(&x, &bits, 8);
  return x * (1.5 - half * x * x);
}

// ffm.cpp:53-55 — packed index of block (f1,f2), f1<=f2, among f(f+1)/2.
static inline u32 block_index(u32 f1, u32 f2, u32 f) { return f2 + (f - 1) * f1 - f1 * (f1 - 1) / 2; }

// ffm.cpp:71-78 — one minstd_rand0 engine seeded by rand() per table,
// uniform_real_distribution<double>(-b, b), b = 0.1*qrsqrt(cols).
static void init_table(Vec &t, u64 rows, u64 cols) {
  std::minstd_rand0 eng(std::rand());
  const double b = 0.1 * qrsqrt((double)cols);
  std::uniform_real_distribution<double> dist(-b, b);
  t.assign(rows * cols, 0.0);
  for (auto &v : t) v = dist(eng);
}

// ---------------------------------------------------------------- data ---
// Restates ImpData (ffm.h:59-79): read (ffm.cpp:80-183), split_fields
// (185-257) and transY (259-294).
struct Data {
  std::string path;
  u64 m = 0, n = 0, f = 0;
  std::vector<u64> nnx;         // kept feature nodes per row
  std::vector<u64> yptr;        // labels / positives, CSR over rows
  std::vector<u64> ycol;        // item ids (user side) or user ids (item side)
  Vec yval;                     // y-tilde storage (ffm.cpp:393,400)
  std::vector<std::vector<u64>> xptr;  // per field CSR
  std::vector<std::vector<u64>> xidx;
  std::vector<Vec> xval;
  std::vector<u64> Ds;
  std::vector<std::vector<u64>> freq;
  Vec popular;
};

struct RawRows {
  std::vector<u64> xptr;
  std::vector<u32> fid;
  std::vector<u64> idx;
  Vec val;
  std::vector<u64> yptr, ycol;
  bool has_label = false;
  u64 f = 0;  // max fid + 1 over all tokens (also the dropped ones)
  u64 n = 0;  // max label + 1
};

// ffm.cpp:80-183.  Token grammar: optional label block "j1,j2,..." then
// "fid:idx:val" triples; with ds != nullptr a node with idx >= ds[fid] is
// dropped (test rows).  An empty line re-uses the previous label block.
static RawRows parse_file(const std::string &path, bool has_label, const u64 *ds, u64 nds) {
  std::ifstream fs(path);
  if (!fs) throw std::runtime_error("cannot open " + path);
  RawRows r;
  r.has_label = has_label;
  r.xptr.push_back(0);
  r.yptr.push_back(0);
  std::string line, label_block, tok;
  while (std::getline(fs, line)) {
    std::istringstream iss(line);
    if (has_label) {
      iss >> label_block;
      std::istringstream ls(label_block);
      while (std::getline(ls, tok, ',')) {
        u64 j = (u64)std::stoi(tok);
        r.ycol.push_back(j);
        r.n = std::max(r.n, j + 1);
      }
      r.yptr.push_back(r.ycol.size());
    }
    u64 fid, idx;
    double val;
    char c;
    while (iss >> fid >> c >> idx >> c >> val) {
      r.f = std::max(r.f, fid + 1);
      if (ds != nullptr && (fid >= nds || ds[fid] <= idx)) continue;
      r.fid.push_back((u32)fid);
      r.idx.push_back(idx);
      r.val.push_back(val);
    }
    r.xptr.push_back(r.fid.size());
  }
  return r;
}

// ffm.cpp:185-257 (split_fields) + popularity normalisation (172-176).
static void build_data(Data &d, const RawRows &r) {
  d.m = r.xptr.size() - 1;
  d.f = r.f;
  d.n = r.n;
  d.nnx.resize(d.m);
  for (u64 i = 0; i < d.m; i++) d.nnx[i] = r.xptr[i + 1] - r.xptr[i];
  if (r.has_label) {
    d.yptr = r.yptr;
    d.ycol = r.ycol;
    d.yval.assign(d.ycol.size(), 0.0);
    d.popular.assign(d.n, 0.0);
    for (u64 j : d.ycol) d.popular[j] += 1;
    double s = 0;
    for (double p : d.popular) s += p;
    for (double &p : d.popular) p /= s;
  } else {
    d.yptr.assign(d.m + 1, 0);
  }
  d.xptr.assign(d.f, std::vector<u64>(d.m + 1, 0));
  d.xidx.assign(d.f, {});
  d.xval.assign(d.f, {});
  d.Ds.assign(d.f, 0);
  for (u64 i = 0; i < d.m; i++)
    for (u64 p = r.xptr[i]; p < r.xptr[i + 1]; p++) d.xptr[r.fid[p]][i + 1]++;
  for (u64 fi = 0; fi < d.f; fi++) {
    for (u64 i = 0; i < d.m; i++) d.xptr[fi][i + 1] += d.xptr[fi][i];
    d.xidx[fi].resize(d.xptr[fi][d.m]);
    d.xval[fi].resize(d.xptr[fi][d.m]);
  }
  // Rows are visited in order, so a running cursor per field reproduces the
  // per-field node order of split_fields.
  std::vector<u64> cur(d.f, 0);
  for (u64 i = 0; i < d.m; i++)
    for (u64 p = r.xptr[i]; p < r.xptr[i + 1]; p++) {
      u32 fi = r.fid[p];
      u64 q = cur[fi]++;
      d.xidx[fi][q] = r.idx[p];
      d.xval[fi][q] = r.val[p];
      d.Ds[fi] = std::max(d.Ds[fi], r.idx[p] + 1);
    }
  d.freq.assign(d.f, {});
  for (u64 fi = 0; fi < d.f; fi++) {
    d.freq[fi].assign(d.Ds[fi], 0);
    for (u64 x : d.xidx[fi]) d.freq[fi][x]++;
  }
}

// ffm.cpp:259-294 — item-major positives built from the user-major labels,
// sorted by (item, user); labels >= #items are skipped.
static void trans_y(Data &V, const Data &U) {
  std::vector<u64> cnt(V.m + 1, 0);
  for (u64 i = 0; i < U.m; i++)
    for (u64 p = U.yptr[i]; p < U.yptr[i + 1]; p++)
      if (U.ycol[p] < V.m) cnt[U.ycol[p] + 1]++;
  for (u64 j = 0; j < V.m; j++) cnt[j + 1] += cnt[j];
  V.yptr = cnt;
  V.ycol.assign(cnt[V.m], 0);
  V.yval.assign(cnt[V.m], 0.0);
  std::vector<u64> cur(cnt.begin(), cnt.end() - 1);
  for (u64 i = 0; i < U.m; i++)  // users in increasing order => sorted by (item, user)
    for (u64 p = U.yptr[i]; p < U.yptr[i + 1]; p++) {
      u64 j = U.ycol[p];
      if (j >= V.m) continue;
      V.ycol[cur[j]++] = i;
    }
  V.n = U.m;
}

// ------------------------------------------------------------- problem ---
struct Param {
  double omega = 0.1, lambda = 1e-5, r = -1;
  u32 nr_pass = 20, k = 4, nr_threads = 1;
  bool self_side = true, freq = false;
};

struct Problem {
  Data *U, *Ut, *V;
  Param prm;
  double w, lam, r;
  u32 k, fu, fv, f;
  u64 m, n;
  std::vector<Vec> W, H, P, Q;
  Vec a, b, sa, sb;
  // validation (ffm.cpp:872-1016)
  std::vector<u32> top_k;
  Vec va_prec, va_ndcg;
  double loss = 0;
  std::vector<int> cg_log;  // CG iterations of every half, in solve order
  bool quiet = false;

  bool is_user(u32 fl) const { return fl < fu; }
  bool block_used(u32 f1, u32 f2) const { return prm.self_side || (f1 < fu && f2 >= fu); }

  // ffm.cpp:314-331 — C = X_field * A, row-wise gather-AXPY.
  void utx(const Data &d, u32 fi, const Vec &A, Vec &C) const {
    const u32 k = this->k;  // local copy: lets the compiler keep it in a register
    const u64 rows = d.m;
    C.assign(rows * k, 0.0);
    const auto &xp = d.xptr[fi];
    const auto &xi = d.xidx[fi];
    const auto &xv = d.xval[fi];
#pragma omp parallel for schedule(guided)
    for (u64 i = 0; i < rows; i++) {
      double *c = &C[i * k];
      for (u64 p = xp[i]; p < xp[i + 1]; p++) {
        const double v = xv[p];
        const double *ar = &A[xi[p] * k];
        for (u32 d2 = 0; d2 < k; d2++) c[d2] += v * ar[d2];
      }
    }
  }

  // inner() = cblas_ddot (ffm.cpp:57-60).  Its summation order is the BLAS
  // build's: serial here by default (dot_lanes = dot_chunks = 1).  For the
  // drift envelope (tools/fp64_drift.py) the order of an optimised build can
  // be restated: dot_chunks contiguous chunks (a threaded ddot) each summed in
  // dot_lanes interleaved accumulators (SIMD registers: element i into lane
  // i % lanes), the lanes reduced pairwise, the chunks added in order.
  u32 dot_lanes = 1, dot_chunks = 1;
  double dot(const double *x, const double *y, u64 len) const {
    if (dot_lanes <= 1 && dot_chunks <= 1) {
      double s = 0;
      for (u64 i = 0; i < len; i++) s += x[i] * y[i];
      return s;
    }
    const u32 L = std::max<u32>(1, std::min<u32>(dot_lanes, 64));
    const u64 nc = std::max<u64>(1, std::min<u64>(dot_chunks, len));
    double tot = 0;
    for (u64 c = 0; c < nc; c++) {
      const u64 b = len * c / nc, e = len * (c + 1) / nc;
      double acc[64] = {0};
      for (u64 i = b; i < e; i++) acc[(i - b) % L] += x[i] * y[i];
      for (u32 w = 1; w < L; w *= 2)
        for (u32 l = 0; l + w < L; l += 2 * w) acc[l] += acc[l + w];
      tot += acc[0];
    }
    return tot;
  }

  // ffm.cpp:334-350 + 467-512.
  void init() {
    lam = prm.lambda;
    w = prm.omega;
    r = prm.r;
    m = U->m;
    n = V->m;
    fu = (u32)U->f;
    fv = (u32)V->f;
    f = fu + fv;
    k = prm.k;
    a.assign(m, 0);
    b.assign(n, 0);
    sa.assign(m, 0);
    sb.assign(n, 0);
    const u32 nb = f * (f + 1) / 2;
    W.assign(nb, {});
    H.assign(nb, {});
    P.assign(nb, {});
    Q.assign(nb, {});
    for (u32 f1 = 0; f1 < f; f1++) {
      const Data &d1 = is_user(f1) ? *U : *V;
      const u32 fi = is_user(f1) ? f1 : f1 - fu;
      for (u32 f2 = f1; f2 < f; f2++) {
        const Data &d2 = is_user(f2) ? *U : *V;
        const u32 fj = is_user(f2) ? f2 : f2 - fu;
        if (!block_used(f1, f2)) continue;
        const u32 b12 = block_index(f1, f2, f);
        init_table(W[b12], d1.Ds[fi], k);
        init_table(H[b12], d2.Ds[fj], k);
        utx(d1, fi, W[b12], P[b12]);
        utx(d2, fj, H[b12], Q[b12]);
      }
    }
    cache_sasb();
    if (prm.self_side) calc_side();
    init_y_tilde();
  }

  // ffm.cpp:514-535.
  void cache_sasb() {
    const u32 k = this->k;  // local copy: lets the compiler keep it in a register
    Timer tm_(T_SASB);
    std::fill(sa.begin(), sa.end(), 0.0);
    std::fill(sb.begin(), sb.end(), 0.0);
    Vec t(k);
    for (u32 f1 = 0; f1 < fu; f1++)
      for (u32 f2 = fu; f2 < f; f2++) {
        const u32 b12 = block_index(f1, f2, f);
        const Vec &P1 = P[b12], &Q1 = Q[b12];
        std::fill(t.begin(), t.end(), 0.0);
        for (u64 j = 0; j < n; j++)
          for (u32 d = 0; d < k; d++) t[d] += Q1[j * k + d];
        for (u64 i = 0; i < m; i++) sa[i] += dot(&P1[i * k], t.data(), k);
        std::fill(t.begin(), t.end(), 0.0);
        for (u64 i = 0; i < m; i++)
          for (u32 d = 0; d < k; d++) t[d] += P1[i * k + d];
        for (u64 j = 0; j < n; j++) sb[j] += dot(&Q1[j * k], t.data(), k);
      }
  }

  // ffm.cpp:352-373.
  void calc_side() {
    const u32 k = this->k;  // local copy: lets the compiler keep it in a register
    for (u32 f1 = 0; f1 < f; f1++)
      for (u32 f2 = f1; f2 < f; f2++) {
        if (is_user(f1) != is_user(f2)) continue;
        const u32 b12 = block_index(f1, f2, f);
        Vec &t = is_user(f1) ? a : b;
        const u64 rows = is_user(f1) ? m : n;
        for (u64 i = 0; i < rows; i++) t[i] += dot(&P[b12][i * k], &Q[b12][i * k], k);
      }
  }

  // ffm.cpp:375-386.
  double cross(u64 i, u64 j) const {
    const u32 k = this->k;  // local copy: lets the compiler keep it in a register
    double s = 0;
    for (u32 f1 = 0; f1 < fu; f1++)
      for (u32 f2 = fu; f2 < f; f2++) {
        const u32 b12 = block_index(f1, f2, f);
        s += dot(&P[b12][i * k], &Q[b12][j * k], k);
      }
    return s;
  }

  // ffm.cpp:388-403 — both orientations hold the same value.
  void init_y_tilde() {
#pragma omp parallel for schedule(guided)
    for (u64 i = 0; i < m; i++)
      for (u64 p = U->yptr[i]; p < U->yptr[i + 1]; p++) {
        const u64 j = U->ycol[p];
        U->yval[p] = a[i] + b[j] + cross(i, j) - 1;
      }
#pragma omp parallel for schedule(guided)
    for (u64 j = 0; j < n; j++)
      for (u64 p = V->yptr[j]; p < V->yptr[j + 1]; p++) {
        const u64 i = V->ycol[p];
        V->yval[p] = a[i] + b[j] + cross(i, j) - 1;
      }
  }

  // Regulariser term of G/Hv: lambda*V or lambda*freq(d)*V (ffm.cpp:561-570,786-794).
  void add_reg(const Data &d, u32 fi, const Vec &X, Vec &out) const {
    const u32 k = this->k;  // local copy: lets the compiler keep it in a register
    const u64 D = d.Ds[fi];
    for (u64 row = 0; row < D; row++) {
      const double s = prm.freq ? lam * (double)d.freq[fi][row] : lam;
      for (u32 e = 0; e < k; e++) out[row * k + e] += s * X[row * k + e];
    }
  }

  struct Half {  // the solve-side view of a half block (rows R of side "own")
    Data *own, *oth;
    u32 fi;           // field index inside own side
    const Vec *a1, *b1, *sa1;
    u64 m1, n1;
    bool user;
  };
  Half half_for(u32 fl) {
    Half h;
    h.user = is_user(fl);
    h.own = h.user ? U : V;
    h.oth = h.user ? V : U;
    h.fi = h.user ? fl : fl - fu;
    h.a1 = h.user ? &a : &b;
    h.b1 = h.user ? &b : &a;
    h.sa1 = h.user ? &sa : &sb;
    h.m1 = h.user ? m : n;
    h.n1 = h.user ? n : m;
    return h;
  }

  // ffm.cpp:537-592 — G = lam*W1 + sum_i z_i x_i (x) q1_i.
  void gd_side(u32 fl, const Vec &W1, const Vec &Q1, Vec &G) {
    const u32 k = this->k;  // local copy: lets the compiler keep it in a register
    Timer tm_(T_GD_SIDE);
    Half h = half_for(fl);
    const auto &xp = h.own->xptr[h.fi];
    const auto &xi = h.own->xidx[h.fi];
    const auto &xv = h.own->xval[h.fi];
    double bsum = 0;
    for (double v : *h.b1) bsum += v;
    const u64 bs = G.size();
    const u32 T = prm.nr_threads;
    Vec Gt((u64)T * bs, 0.0);
    std::fill(G.begin(), G.end(), 0.0);
    add_reg(*h.own, h.fi, W1, G);
#pragma omp parallel for schedule(guided)
    for (u64 i = 0; i < h.m1; i++) {
      double *g = &Gt[(u64)omp_get_thread_num() * bs];
      double z = w * ((double)h.n1 * ((*h.a1)[i] - r) + bsum + (*h.sa1)[i]);
      for (u64 p = h.own->yptr[i]; p < h.own->yptr[i + 1]; p++) z += (1 - w) * h.own->yval[p] - w * (1 - r);
      const double *q = &Q1[i * k];
      for (u64 p = xp[i]; p < xp[i + 1]; p++) {
        double *gr = g + xi[p] * k;
        for (u32 d = 0; d < k; d++) gr[d] += q[d] * xv[p] * z;
      }
    }
    for (u32 t = 0; t < T; t++) {
#pragma omp parallel for schedule(static)
      for (u64 e = 0; e < bs; e++) G[e] += Gt[(u64)t * bs + e];
    }
  }

  // ffm.cpp:594-628 — Hv += sum_i d_i (x_i^T V q_i) x_i (x) q_i.
  void hs_side(u32 fl, const Vec &Vd, Vec &Hv, const Vec &Q1, Vec &Ht) {
    const u32 k = this->k;  // local copy: lets the compiler keep it in a register
    Half h = half_for(fl);
    const auto &xp = h.own->xptr[h.fi];
    const auto &xi = h.own->xidx[h.fi];
    const auto &xv = h.own->xval[h.fi];
    const u64 bs = Hv.size();
    const u32 T = prm.nr_threads;
#pragma omp parallel for schedule(guided)
    for (u64 i = 0; i < h.m1; i++) {
      double *hv = &Ht[(u64)omp_get_thread_num() * bs];
      const double *q = &Q1[i * k];
      const double dd = (1 - w) * (double)(u32)(h.own->yptr[i + 1] - h.own->yptr[i]) + w * (double)h.n1;
      double z = 0;
      for (u64 p = xp[i]; p < xp[i + 1]; p++) {
        const double *vr = &Vd[xi[p] * k];
        for (u32 d = 0; d < k; d++) z += q[d] * xv[p] * vr[d];
      }
      z *= dd;
      for (u64 p = xp[i]; p < xp[i + 1]; p++) {
        double *hr = hv + xi[p] * k;
        for (u32 d = 0; d < k; d++) hr[d] += q[d] * xv[p] * z;
      }
    }
    for (u32 t = 0; t < T; t++) {
#pragma omp parallel for schedule(static)
      for (u64 e = 0; e < bs; e++) Hv[e] += Ht[(u64)t * bs + e];
    }
  }

  // k x k Gram Acc = A^T B over `rows` rows (ffm.cpp:41-45, dgemm TN).
  // Threaded like the CBLAS dgemm it replaces: per-thread partials, then a
  // fixed-order sum.
  void gram(const Vec &A, const Vec &B, u64 rows, Vec &Acc) const {
    const u64 kk = (u64)k * k;
    const int NT = omp_get_max_threads();
    Vec part((u64)NT * kk, 0.0);
    const u32 K = k;
    const double *Ap = A.data(), *Bp = B.data();
#pragma omp parallel
    {
      double *acc = &part[(u64)omp_get_thread_num() * kk];
#pragma omp for schedule(static)
      for (u64 j = 0; j < rows; j++) {
        const double *aj = Ap + j * K, *bj = Bp + j * K;
        for (u32 e = 0; e < K; e++) {
          const double ae = aj[e];
          double *ar = acc + (u64)e * K;
          for (u32 d = 0; d < K; d++) ar[d] += ae * bj[d];
        }
      }
    }
    Acc.assign(kk, 0.0);
    for (int t = 0; t < NT; t++)
      for (u64 e = 0; e < kk; e++) Acc[e] += part[(u64)t * kk + e];
  }

  // ffm.cpp:630-703 — G = lam*W1 + sum_i x_i (x) [pk_i + w(T_i + (a_i-r)oQ + bQ)].
  void gd_cross(u32 fl, const Vec &Q1, const Vec &W1, Vec &G) {
    const u32 k = this->k;  // local copy: lets the compiler keep it in a register
    Timer tm_(T_GD_CROSS);
    Half h = half_for(fl);
    const std::vector<Vec> &Ps = h.user ? P : Q;
    const std::vector<Vec> &Qs = h.user ? Q : P;
    const auto &xp = h.own->xptr[h.fi];
    const auto &xi = h.own->xidx[h.fi];
    const auto &xv = h.own->xval[h.fi];
    std::fill(G.begin(), G.end(), 0.0);
    add_reg(*h.own, h.fi, W1, G);
    Vec oQ(k, 0.0), bQ(k, 0.0), T(h.m1 * k, 0.0), M;
    for (u64 j = 0; j < h.n1; j++)
      for (u32 d = 0; d < k; d++) {
        oQ[d] += Q1[j * k + d];
        bQ[d] += (*h.b1)[j] * Q1[j * k + d];
      }
    for (u32 al = 0; al < fu; al++)
      for (u32 be = fu; be < f; be++) {
        const u32 ab = block_index(al, be, f);
        gram(Qs[ab], Q1, h.n1, M);
        const double *Pa = Ps[ab].data(), *Mp = M.data();
        double *Tp = T.data();
        const u32 K = k;
#pragma omp parallel for schedule(static)
        for (u64 i = 0; i < h.m1; i++) {
          double *ti = Tp + i * K;
          for (u32 e = 0; e < K; e++) {
            const double pe = Pa[i * K + e];
            const double *me = Mp + (u64)e * K;
            for (u32 d = 0; d < K; d++) ti[d] += pe * me[d];
          }
        }
      }
    const u64 bs = G.size();
    const u32 NT = prm.nr_threads;
    Vec Gt((u64)NT * bs, 0.0);
#pragma omp parallel for schedule(guided)
    for (u64 i = 0; i < h.m1; i++) {
      double *g = &Gt[(u64)omp_get_thread_num() * bs];
      double pk[256];
      for (u32 d = 0; d < k; d++) pk[d] = 0;
      for (u64 p = h.own->yptr[i]; p < h.own->yptr[i + 1]; p++) {
        const double sc = (1 - w) * h.own->yval[p] - w * (1 - r);
        const double *q = &Q1[h.own->ycol[p] * k];
        for (u32 d = 0; d < k; d++) pk[d] += sc * q[d];
      }
      const double z = (*h.a1)[i] - r;
      const double *t = &T[i * k];
      for (u64 p = xp[i]; p < xp[i + 1]; p++) {
        double *gr = g + xi[p] * k;
        for (u32 d = 0; d < k; d++) gr[d] += (pk[d] + w * (t[d] + z * oQ[d] + bQ[d])) * xv[p];
      }
    }
    for (u32 t = 0; t < NT; t++) {
#pragma omp parallel for schedule(static)
      for (u64 e = 0; e < bs; e++) G[e] += Gt[(u64)t * bs + e];
    }
  }

  // ffm.cpp:706-742 — Hv += sum_i x_i (x) [(1-w) sum_j <phi_i,q_j> q_j + w tau_i].
  void hs_cross(u32 fl, const Vec &Vd, const Vec &VQTQ, Vec &Hv, const Vec &Q1, Vec &Ht) {
    const u32 k = this->k;  // local copy: lets the compiler keep it in a register
    Half h = half_for(fl);
    const auto &xp = h.own->xptr[h.fi];
    const auto &xi = h.own->xidx[h.fi];
    const auto &xv = h.own->xval[h.fi];
    const u64 bs = Hv.size();
    const u32 NT = prm.nr_threads;
#pragma omp parallel for schedule(guided)
    for (u64 i = 0; i < h.m1; i++) {
      double *hv = &Ht[(u64)omp_get_thread_num() * bs];
      double phi[256], tau[256], ka[256];
      for (u32 d = 0; d < k; d++) phi[d] = tau[d] = ka[d] = 0;
      for (u64 p = xp[i]; p < xp[i + 1]; p++) {
        const double *vr = &Vd[xi[p] * k];
        const double *tr = &VQTQ[xi[p] * k];
        for (u32 d = 0; d < k; d++) phi[d] += xv[p] * vr[d];
        for (u32 d = 0; d < k; d++) tau[d] += xv[p] * tr[d];
      }
      for (u64 p = h.own->yptr[i]; p < h.own->yptr[i + 1]; p++) {
        const double *q = &Q1[h.own->ycol[p] * k];
        const double s = dot(phi, q, k);
        for (u32 d = 0; d < k; d++) ka[d] += s * q[d];
      }
      for (u64 p = xp[i]; p < xp[i + 1]; p++) {
        double *hr = hv + xi[p] * k;
        for (u32 d = 0; d < k; d++) hr[d] += ((1 - w) * ka[d] + w * tau[d]) * xv[p];
      }
    }
    for (u32 t = 0; t < NT; t++) {
#pragma omp parallel for schedule(static)
      for (u64 e = 0; e < bs; e++) Hv[e] += Ht[(u64)t * bs + e];
    }
  }

  // lam*V + H(V) for one half (the Hessian-vector product used inside cg()).
  void hess_vec(u32 f1, u32 f2, const Vec &Vd, const Vec &Q1, const Vec &QTQ, Vec &Hv, Vec &Ht) {
    const u32 k = this->k;  // local copy: lets the compiler keep it in a register
    Timer tm_(T_HV);
    Half h = half_for(f1);
    std::fill(Hv.begin(), Hv.end(), 0.0);
    std::fill(Ht.begin(), Ht.end(), 0.0);
    add_reg(*h.own, h.fi, Vd, Hv);
    if (is_user(f1) == is_user(f2)) {
      hs_side(f1, Vd, Hv, Q1, Ht);
    } else {
      const u64 D = h.own->Ds[h.fi];
      Vec VQTQ(D * k, 0.0);
#pragma omp parallel for schedule(static)
      for (u64 row = 0; row < D; row++)
        for (u32 e = 0; e < k; e++) {
          const double ve = Vd[row * k + e];
          for (u32 d = 0; d < k; d++) VQTQ[row * k + d] += ve * QTQ[e * k + d];
        }
      hs_cross(f1, Vd, VQTQ, Hv, Q1, Ht);
    }
  }

  // ffm.cpp:744-813 — Newton-CG, eps 0.09 on |r|^2 vs |g|^2, at most 20 steps.
  void cg(u32 f1, u32 f2, Vec &S, const Vec &Q1, const Vec &G) {
    const u32 k = this->k;  // local copy: lets the compiler keep it in a register
    Timer tm_(T_CG);
    Half h = half_for(f1);
    const u64 Dk = h.own->Ds[h.fi] * k;
    Vec Ht((u64)prm.nr_threads * Dk), Vd(Dk), R(Dk), Hv(Dk), QTQ;
    if (is_user(f1) != is_user(f2)) gram(Q1, Q1, h.n1, QTQ);
    double g2 = 0;
    for (u64 e = 0; e < Dk; e++) {
      R[e] = -G[e];
      Vd[e] = R[e];
      g2 += G[e] * G[e];
    }
    double r2 = g2;
    int it = 0;
    while (g2 * 9e-2 < r2 && it < 20) {
      it++;
      hess_vec(f1, f2, Vd, Q1, QTQ, Hv, Ht);
      const double vHv = dot(Vd.data(), Hv.data(), Dk);
      const double gamma = r2;
      const double alpha = gamma / vHv;
      for (u64 e = 0; e < Dk; e++) S[e] += alpha * Vd[e];
      for (u64 e = 0; e < Dk; e++) R[e] -= alpha * Hv[e];
      r2 = dot(R.data(), R.data(), Dk);
      const double beta = r2 / gamma;
      for (u64 e = 0; e < Dk; e++) Vd[e] = beta * Vd[e] + R[e];
    }
    cg_log.push_back(it);
  }

  // ffm.cpp:405-437.
  void update_side(bool user, const Vec &S, const Vec &Q1, Vec &W1, u32 fi, Vec &P1) {
    const u32 k = this->k;  // local copy: lets the compiler keep it in a register
    Timer tm_(T_UPD_SIDE);
    Data &own = user ? *U : *V;
    Data &oth = user ? *V : *U;
    Vec &a1 = user ? a : b;
    for (u64 e = 0; e < S.size(); e++) W1[e] += S[e];
    Vec XS;
    utx(own, fi, S, XS);
    for (u64 e = 0; e < XS.size(); e++) P1[e] += XS[e];
    Vec gap(own.m);
    for (u64 i = 0; i < own.m; i++) gap[i] = dot(&XS[i * k], &Q1[i * k], k);
    for (u64 i = 0; i < own.m; i++) {
      a1[i] += gap[i];
      for (u64 p = own.yptr[i]; p < own.yptr[i + 1]; p++) own.yval[p] += gap[i];
    }
    for (u64 j = 0; j < oth.m; j++)
      for (u64 p = oth.yptr[j]; p < oth.yptr[j + 1]; p++) oth.yval[p] += gap[oth.ycol[p]];
  }

  // ffm.cpp:439-465.
  void update_cross(bool user, const Vec &S, const Vec &Q1, Vec &W1, u32 fi, Vec &P1) {
    const u32 k = this->k;  // local copy: lets the compiler keep it in a register
    Timer tm_(T_UPD_CROSS);
    Data &own = user ? *U : *V;
    Data &oth = user ? *V : *U;
    for (u64 e = 0; e < S.size(); e++) W1[e] += S[e];
    Vec XS;
    utx(own, fi, S, XS);
    for (u64 e = 0; e < XS.size(); e++) P1[e] += XS[e];
#pragma omp parallel for schedule(guided)
    for (u64 i = 0; i < own.m; i++)
      for (u64 p = own.yptr[i]; p < own.yptr[i + 1]; p++)
        own.yval[p] += dot(&XS[i * k], &Q1[own.ycol[p] * k], k);
#pragma omp parallel for schedule(guided)
    for (u64 j = 0; j < oth.m; j++)
      for (u64 p = oth.yptr[j]; p < oth.yptr[j + 1]; p++)
        oth.yval[p] += dot(&XS[oth.ycol[p] * k], &Q1[j * k], k);
  }

  // ffm.cpp:815-833.
  void solve_side(u32 f1, u32 f2) {
    const u32 b12 = block_index(f1, f2, f);
    const bool user = is_user(f1);
    const u32 base = user ? 0 : fu;
    Vec G1(W[b12].size()), G2(H[b12].size()), S1(W[b12].size(), 0.0), S2(H[b12].size(), 0.0);
    gd_side(f1, W[b12], Q[b12], G1);
    cg(f1, f2, S1, Q[b12], G1);
    update_side(user, S1, Q[b12], W[b12], f1 - base, P[b12]);
    gd_side(f2, H[b12], P[b12], G2);
    cg(f2, f1, S2, P[b12], G2);
    update_side(user, S2, P[b12], H[b12], f2 - base, Q[b12]);
  }

  // ffm.cpp:835-850.
  void solve_cross(u32 f1, u32 f2) {
    const u32 b12 = block_index(f1, f2, f);
    Vec GW(W[b12].size()), GH(H[b12].size()), SW(W[b12].size(), 0.0), SH(H[b12].size(), 0.0);
    gd_cross(f1, Q[b12], W[b12], GW);
    cg(f1, f2, SW, Q[b12], GW);
    update_cross(true, SW, Q[b12], W[b12], f1, P[b12]);
    gd_cross(f2, P[b12], H[b12], GH);
    cg(f2, f1, SH, P[b12], GH);
    update_cross(false, SH, P[b12], H[b12], f2 - fu, Q[b12]);
  }

  void solve_block(u32 f1, u32 f2) {
    if (is_user(f1) == is_user(f2)) solve_side(f1, f2);
    else solve_cross(f1, f2);
  }

  // ffm.cpp:852-870 — Gauss-Seidel block order.
  void one_epoch() {
    if (prm.self_side) {
      for (u32 f1 = 0; f1 < fu; f1++)
        for (u32 f2 = f1; f2 < fu; f2++) solve_side(f1, f2);
      for (u32 f1 = fu; f1 < f; f1++)
        for (u32 f2 = f1; f2 < f; f2++) solve_side(f1, f2);
    }
    for (u32 f1 = 0; f1 < fu; f1++)
      for (u32 f2 = fu; f2 < f; f2++) solve_cross(f1, f2);
    if (prm.self_side) cache_sasb();
  }

  // ------------------------------------------------------ evaluation ---
  // ffm.cpp:872-913.
  void init_va(u32 size) {
    if (Ut == nullptr) return;
    top_k.resize(size);
    va_prec.assign(size, 0);
    va_ndcg.assign(size, 0);
    u32 s = 5;
    if (!quiet) std::cout << "iter";
    for (u32 i = 0; i < size; i++) {
      top_k[i] = s;
      if (!quiet) {
        std::cout.width(9);
        std::cout << "( p@ " << s << ", ";
        std::cout.width(6);
        std::cout << "nDCG@" << s << " )";
      }
      s *= 2;
    }
    if (!quiet) {
      std::cout.width(12);
      std::cout << "ploss" << std::endl;
    }
  }

  // Repeated argmax with MIN_Z masking, first index wins ties
  // (ffm.cpp:1018-1128).  Returns per-cutoff hits and nDCG of one row.
  void rank_row(Vec &z, u64 max_z, const u64 *lab, u64 nlab, std::vector<u64> &hits, Vec &nd) const {
    const u32 nk = (u32)top_k.size();
    std::vector<u64> hit(nk, 0);
    Vec dcg(nk, 0), idcg(nk, 0);
    u64 cnt = 0;
    for (u32 s = 0; s < nk; s++)
      while (cnt < top_k[s]) {
        if (cnt >= max_z) break;
        u64 am = (u64)(std::max_element(z.begin(), z.begin() + max_z) - z.begin());
        z[am] = -1000;
        for (u64 t = 0; t < nlab; t++)
          if (lab[t] == am) {
            hit[s]++;
            dcg[s] += 1.0 / std::log2((double)cnt + 2);
            break;
          }
        if ((u32)nlab > cnt) idcg[s] += 1.0 / std::log2((double)cnt + 2);
        cnt++;
      }
    for (u32 s = 1; s < nk; s++) {
      hit[s] += hit[s - 1];
      dcg[s] += dcg[s - 1];
      idcg[s] += idcg[s - 1];
    }
    for (u32 s = 0; s < nk; s++) {
      hits[s] += hit[s];
      nd[s] += dcg[s] / idcg[s];
    }
  }

  // ffm.cpp:925-1016.  `forced` reproduces the EBUG_nDCG debug build
  // (scores z_j = n - j) used by the nDCG known-answer test.
  // per_row_ndcg (optional): nDCG@top_k[s] of test row i at [i * nk + s].
  void validate(bool forced = false, Vec *per_row_ndcg = nullptr) {
    if (Ut == nullptr) return;
    const u64 mt = Ut->m;
    const u32 nb = f * (f + 1) / 2;
    std::vector<Vec> Pva(nb), Qva(nb);
    for (u32 f1 = 0; f1 < f; f1++) {
      const Data &d1 = is_user(f1) ? *Ut : *V;
      const u32 fi = is_user(f1) ? f1 : f1 - fu;
      for (u32 f2 = f1; f2 < f; f2++) {
        const Data &d2 = is_user(f2) ? *Ut : *V;
        const u32 fj = is_user(f2) ? f2 : f2 - fu;
        if (!block_used(f1, f2)) continue;
        const u32 b12 = block_index(f1, f2, f);
        if (fi < d1.f) utx(d1, fi, W[b12], Pva[b12]); else Pva[b12].assign(d1.m * k, 0.0);
        if (fj < d2.f) utx(d2, fj, H[b12], Qva[b12]); else Qva[b12].assign(d2.m * k, 0.0);
      }
    }
    Vec at(mt, 0), bt(n, 0);
    if (prm.self_side)
      for (u32 f1 = 0; f1 < f; f1++)
        for (u32 f2 = f1; f2 < f; f2++) {
          if (is_user(f1) != is_user(f2)) continue;
          const u32 b12 = block_index(f1, f2, f);
          Vec &t = is_user(f1) ? at : bt;
          const u64 rows = is_user(f1) ? mt : n;
          for (u64 i = 0; i < rows; i++) t[i] += dot(&Pva[b12][i * k], &Qva[b12][i * k], k);
        }
    const u32 nk = (u32)top_k.size();
    const u64 max_z = U->popular.size();
    std::vector<u64> hits(nk, 0);
    Vec nd(nk, 0);
    double ploss = 0;
    if (per_row_ndcg) per_row_ndcg->assign(mt * nk, 0.0);
    for (u64 i = 0; i < mt; i++) {
      Vec z;
      if (Ut->nnx[i] == 0) {
        z = U->popular;
      } else {
        z = bt;
        for (u32 f1 = 0; f1 < fu; f1++)
          for (u32 f2 = fu; f2 < f; f2++) {
            const u32 b12 = block_index(f1, f2, f);
            const double *p = &Pva[b12][i * k];
            for (u64 j = 0; j < n; j++) z[j] += dot(&Qva[b12][j * k], p, k);
          }
      }
      for (u64 p = Ut->yptr[i]; p < Ut->yptr[i + 1]; p++) {
        const u64 j = Ut->ycol[p];
        if (j < z.size()) ploss += (1 - z[j] - at[i]) * (1 - z[j] - at[i]);
      }
      if (forced) {
        z.resize(n);
        for (u64 j = 0; j < n; j++) z[j] = (double)(n - j);
      }
      Vec nd_row(nk, 0);
      std::vector<u64> h_row(nk, 0);
      rank_row(z, std::min<u64>(max_z, z.size()), &Ut->ycol[Ut->yptr[i]], Ut->yptr[i + 1] - Ut->yptr[i], h_row, nd_row);
      for (u32 s = 0; s < nk; s++) {
        hits[s] += h_row[s];
        nd[s] += nd_row[s];
      }
      if (per_row_ndcg)
        for (u32 s = 0; s < nk; s++) (*per_row_ndcg)[i * nk + s] = nd_row[s];
    }
    loss = std::sqrt(ploss / (double)mt);
    for (u32 s = 0; s < nk; s++) {
      va_prec[s] = (double)hits[s] / (double)(mt * top_k[s]);
      va_ndcg[s] = nd[s] / (double)mt;
    }
  }

  // ffm.cpp:1130-1145.
  void print_epoch_info(u32 t) const {
    std::cout.width(2);
    std::cout << t + 1;
    if (Ut != nullptr) {
      for (u32 i = 0; i < top_k.size(); i++) {
        std::cout.width(9);
        std::cout << "( " << std::setprecision(3) << va_prec[i] * 100 << " ,";
        std::cout.width(6);
        std::cout << std::setprecision(3) << va_ndcg[i] * 100 << " )";
      }
      std::cout.width(13);
      std::cout << std::setprecision(3) << loss;
    }
    std::cout << std::endl;
  }

  // ffm.cpp:1147-1161.
  void solve() {
    init_va(5);
    for (u32 it = 0; it < prm.nr_pass; it++) {
      one_epoch();
      if (Ut != nullptr && it % 10 == 9) {
        validate();
        print_epoch_info(it);
      }
    }
  }

  // ffm.cpp:1303-1351 — brute-force objective over all m x n pairs.
  double func() const {
    double res = 0;
    for (u64 i = 0; i < m; i++) {
      for (u64 j = 0; j < n; j++) {
        double yh = 0;
        for (u32 f1 = 0; f1 < f; f1++)
          for (u32 f2 = f1; f2 < f; f2++) {
            if (!block_used(f1, f2)) continue;
            const u32 b12 = block_index(f1, f2, f);
            const u64 pi = is_user(f1) ? i : j;
            const u64 qj = is_user(f2) ? i : j;
            yh += dot(&Q[b12][qj * k], &P[b12][pi * k], k);
          }
        bool pos = false;
        for (u64 p = U->yptr[i]; p < U->yptr[i + 1]; p++)
          if (U->ycol[p] == j) {
            pos = true;
            break;
          }
        res += pos ? (1 - yh) * (1 - yh) : w * (r - yh) * (r - yh);
      }
    }
    for (u32 f1 = 0; f1 < f; f1++)
      for (u32 f2 = f1; f2 < f; f2++) {
        if (!block_used(f1, f2)) continue;
        const u32 b12 = block_index(f1, f2, f);
        res += lam * (dot(W[b12].data(), W[b12].data(), W[b12].size()) + dot(H[b12].data(), H[b12].data(), H[b12].size()));
      }
    return 0.5 * res;
  }

  // ffm.cpp:1163-1237 — text model, default 6 significant digits.
  void save_model(const std::string &path) const {
    std::ofstream o(path, std::ios::out | std::ios::trunc);
    o << f << "\n" << fu << "\n" << fv << "\n" << k << "\n";
    for (u32 i = 0; i < fu; i++) o << U->Ds[i] << "\n";
    for (u32 i = 0; i < fv; i++) o << V->Ds[i] << "\n";
    auto block = [&](const Vec &t, u64 rows, char c, u32 fi, u32 fj) {
      for (u64 row = 0; row < rows; row++) {
        o << c << ',' << fi << ',' << fj << ',' << row;
        for (u32 e = 0; e < k; e++) o << " " << t[row * k + e];
        o << "\n";
      }
    };
    for (u32 fi = 0; fi < f; fi++)
      for (u32 fj = fi; fj < f; fj++) {
        if (!block_used(fi, fj)) continue;
        const u32 b12 = block_index(fi, fj, f);
        const u64 r1 = is_user(fi) ? U->Ds[fi] : V->Ds[fi - fu];
        const u64 r2 = is_user(fj) ? U->Ds[fj] : V->Ds[fj - fu];
        block(W[b12], r1, 'W', fi, fj);
        block(H[b12], r2, 'H', fi, fj);
      }
  }

  // ffm.cpp:1239-1267 — binary model: u32 f, fu, fv, k; u64 user Ds, item
  // Ds; per used block u32 index_vec, u64 |W|, u64 |H|, W and H as doubles.
  void save_binary(const std::string &path) const {
    std::ofstream o(path, std::ios::binary | std::ios::trunc);
    const u32 hd[4] = {f, fu, fv, k};
    o.write(reinterpret_cast<const char *>(hd), sizeof(hd));
    o.write(reinterpret_cast<const char *>(U->Ds.data()), sizeof(u64) * fu);
    o.write(reinterpret_cast<const char *>(V->Ds.data()), sizeof(u64) * fv);
    for (u32 fi = 0; fi < f; fi++)
      for (u32 fj = fi; fj < f; fj++) {
        if (!block_used(fi, fj)) continue;
        const u32 b12 = block_index(fi, fj, f);
        const u64 nw = W[b12].size(), nh = H[b12].size();
        o.write(reinterpret_cast<const char *>(&b12), sizeof(b12));
        o.write(reinterpret_cast<const char *>(&nw), sizeof(nw));
        o.write(reinterpret_cast<const char *>(&nh), sizeof(nh));
        o.write(reinterpret_cast<const char *>(W[b12].data()), sizeof(double) * nw);
        o.write(reinterpret_cast<const char *>(H[b12].data()), sizeof(double) * nh);
      }
  }
};

}  // namespace orc

// ------------------------------------------------------------- C API ---
// Flat C entry points for the Python tests (ctypes).  Not a product API.
using namespace orc;

struct OrcCtx {
  std::unique_ptr<Data> U, Ut, V;
  Problem prob;
};

static thread_local std::string g_err;

extern "C" {

const char *orc_last_error() { return g_err.c_str(); }

// Build one data set from flat rows (same content as a parsed file).
void *orc_data_from_rows(uint64_t m, const uint64_t *xptr, const uint32_t *fid, const uint64_t *idx,
                         const double *val, const uint64_t *yptr, const uint64_t *ycol, const uint64_t *ds,
                         uint64_t nds) {
  RawRows r;
  r.has_label = yptr != nullptr;
  r.xptr.assign(1, 0);
  r.yptr.assign(1, 0);
  for (uint64_t i = 0; i < m; i++) {
    for (uint64_t p = xptr[i]; p < xptr[i + 1]; p++) {
      r.f = std::max<u64>(r.f, (u64)fid[p] + 1);
      if (ds != nullptr && (fid[p] >= nds || ds[fid[p]] <= idx[p])) continue;
      r.fid.push_back(fid[p]);
      r.idx.push_back(idx[p]);
      r.val.push_back(val[p]);
    }
    r.xptr.push_back(r.fid.size());
    if (r.has_label) {
      for (uint64_t p = yptr[i]; p < yptr[i + 1]; p++) {
        r.ycol.push_back(ycol[p]);
        r.n = std::max<u64>(r.n, ycol[p] + 1);
      }
      r.yptr.push_back(r.ycol.size());
    }
  }
  auto *d = new Data();
  build_data(*d, r);
  return d;
}

void *orc_data_read(const char *path, int has_label, const uint64_t *ds, uint64_t nds) {
  try {
    RawRows r = parse_file(path, has_label != 0, ds, nds);
    auto *d = new Data();
    d->path = path;
    build_data(*d, r);
    return d;
  } catch (std::exception &e) {
    g_err = e.what();
    return nullptr;
  }
}

uint64_t orc_data_m(void *d) { return ((Data *)d)->m; }
uint64_t orc_data_f(void *d) { return ((Data *)d)->f; }
void orc_data_ds(void *d, uint64_t *out) {
  auto *x = (Data *)d;
  for (u64 i = 0; i < x->f; i++) out[i] = x->Ds[i];
}

// Takes ownership of the three data sets (Ut may be null).
void *orc_problem_new(void *U, void *Ut, void *V, double omega, double lambda, double r, uint32_t nr_pass,
                      uint32_t k, uint32_t threads, int self_side, int freq) {
  auto *c = new OrcCtx();
  c->U.reset((Data *)U);
  c->Ut.reset((Data *)Ut);
  c->V.reset((Data *)V);
  trans_y(*c->V, *c->U);
  Problem &p = c->prob;
  p.U = c->U.get();
  p.Ut = c->Ut.get();
  p.V = c->V.get();
  p.prm.omega = omega;
  p.prm.lambda = lambda;
  p.prm.r = r;
  p.prm.nr_pass = nr_pass;
  p.prm.k = k;
  p.prm.nr_threads = threads;
  p.prm.self_side = self_side != 0;
  p.prm.freq = freq != 0;
  p.quiet = true;
  omp_set_num_threads((int)threads);
  return c;
}

void orc_problem_free(void *c) { delete (OrcCtx *)c; }
void orc_srand(uint32_t seed) { std::srand(seed); }
void orc_init(void *c) { ((OrcCtx *)c)->prob.init(); }
void orc_one_epoch(void *c) { ((OrcCtx *)c)->prob.one_epoch(); }
void orc_solve_block(void *c, uint32_t f1, uint32_t f2) { ((OrcCtx *)c)->prob.solve_block(f1, f2); }
void orc_cache_sasb(void *c) { ((OrcCtx *)c)->prob.cache_sasb(); }
double orc_func(void *c) { return ((OrcCtx *)c)->prob.func(); }
void orc_set_threads(void *c, uint32_t t) {
  ((OrcCtx *)c)->prob.prm.nr_threads = t;
  omp_set_num_threads((int)t);
}

// The ddot summation order of an optimised CBLAS (Problem::dot): lanes
// interleaved accumulators over `chunks` contiguous chunks.  1, 1 = serial.
void orc_set_dot_order(void *c, uint32_t lanes, uint32_t chunks) {
  ((OrcCtx *)c)->prob.dot_lanes = lanes;
  ((OrcCtx *)c)->prob.dot_chunks = chunks;
}

// out: [loss, prec@5..80, ndcg@5..80] (11 doubles).  per_row_ndcg
// (optional, cap doubles): nDCG@5,10,20,40,80 of each test row, row-major.
// Returns the number of doubles per_row_ndcg needs (5 x test rows).
uint64_t orc_validate(void *c, int forced, double *out, double *per_row_ndcg, uint64_t cap) {
  Problem &p = ((OrcCtx *)c)->prob;
  if (p.top_k.empty()) p.init_va(5);
  Vec rows;
  p.validate(forced != 0, per_row_ndcg ? &rows : nullptr);
  out[0] = p.loss;
  for (int s = 0; s < 5; s++) {
    out[1 + s] = p.va_prec[s];
    out[6 + s] = p.va_ndcg[s];
  }
  if (per_row_ndcg)
    for (u64 i = 0; i < rows.size() && i < cap; i++) per_row_ndcg[i] = rows[i];
  return p.Ut ? p.Ut->m * 5 : 0;
}

int orc_cg_log(void *c, int32_t *out, int cap) {
  auto &l = ((OrcCtx *)c)->prob.cg_log;
  int nn = (int)l.size();
  for (int i = 0; i < nn && i < cap; i++) out[i] = l[i];
  return nn;
}
void orc_cg_log_clear(void *c) { ((OrcCtx *)c)->prob.cg_log.clear(); }

// Access problem state.  what: 'W','H','P','Q' (block b12), 'a','b','s'(sa),
// 't'(sb), 'u' (user-major y-tilde), 'v' (item-major y-tilde).
// Returns the element count (copies at most cap values).
uint64_t orc_get(void *c, char what, uint32_t b12, double *out, uint64_t cap) {
  Problem &p = ((OrcCtx *)c)->prob;
  const Vec *src = nullptr;
  switch (what) {
    case 'W': src = &p.W[b12]; break;
    case 'H': src = &p.H[b12]; break;
    case 'P': src = &p.P[b12]; break;
    case 'Q': src = &p.Q[b12]; break;
    case 'a': src = &p.a; break;
    case 'b': src = &p.b; break;
    case 's': src = &p.sa; break;
    case 't': src = &p.sb; break;
    case 'u': src = &p.U->yval; break;
    case 'v': src = &p.V->yval; break;
    default: return 0;
  }
  if (out)
    for (u64 i = 0; i < src->size() && i < cap; i++) out[i] = (*src)[i];
  return src->size();
}

void orc_set(void *c, char what, uint32_t b12, const double *in, uint64_t len) {
  Problem &p = ((OrcCtx *)c)->prob;
  Vec *dst = nullptr;
  switch (what) {
    case 'W': dst = &p.W[b12]; break;
    case 'H': dst = &p.H[b12]; break;
    default: return;
  }
  dst->assign(in, in + len);
}

// Recompute every derived quantity (P, Q, a, b, sa, sb, y~) from W and H,
// as init() does after drawing them: lets tests perturb W/H and evaluate
// func() (finite-difference checks of gd_*/hs_*).
void orc_refresh(void *c) {
  Problem &p = ((OrcCtx *)c)->prob;
  for (u32 f1 = 0; f1 < p.f; f1++)
    for (u32 f2 = f1; f2 < p.f; f2++) {
      if (!p.block_used(f1, f2)) continue;
      const u32 b12 = block_index(f1, f2, p.f);
      p.utx(p.is_user(f1) ? *p.U : *p.V, p.is_user(f1) ? f1 : f1 - p.fu, p.W[b12], p.P[b12]);
      p.utx(p.is_user(f2) ? *p.U : *p.V, p.is_user(f2) ? f2 : f2 - p.fu, p.H[b12], p.Q[b12]);
    }
  std::fill(p.a.begin(), p.a.end(), 0.0);
  std::fill(p.b.begin(), p.b.end(), 0.0);
  p.cache_sasb();
  if (p.prm.self_side) p.calc_side();
  p.init_y_tilde();
}

// Gradient of one half without changing state: half 0 = W of block (f1,f2)
// (rows of f1's side), half 1 = H (rows of f2's side).
void orc_grad(void *c, uint32_t f1, uint32_t f2, int half, double *G) {
  Problem &p = ((OrcCtx *)c)->prob;
  const u32 b12 = block_index(f1, f2, p.f);
  const u32 fl = half == 0 ? f1 : f2;
  const Vec &Wt = half == 0 ? p.W[b12] : p.H[b12];
  const Vec &Q1 = half == 0 ? p.Q[b12] : p.P[b12];
  Vec Gv(Wt.size());
  if (p.is_user(f1) == p.is_user(f2)) p.gd_side(fl, Wt, Q1, Gv);
  else p.gd_cross(fl, Q1, Wt, Gv);
  std::copy(Gv.begin(), Gv.end(), G);
}

// lam*V + H(V) for one half (the product used inside cg()).
void orc_hv(void *c, uint32_t f1, uint32_t f2, int half, const double *Vin, double *Hv) {
  Problem &p = ((OrcCtx *)c)->prob;
  const u32 b12 = block_index(f1, f2, p.f);
  const u32 fl = half == 0 ? f1 : f2;
  const u32 fo = half == 0 ? f2 : f1;
  const Vec &Q1 = half == 0 ? p.Q[b12] : p.P[b12];
  const u64 sz = (half == 0 ? p.W[b12] : p.H[b12]).size();
  Vec Vd(Vin, Vin + sz), H(sz), Ht((u64)p.prm.nr_threads * sz), QTQ;
  Problem::Half h = p.half_for(fl);
  if (p.is_user(f1) != p.is_user(f2)) p.gram(Q1, Q1, h.n1, QTQ);
  p.hess_vec(fl, fo, Vd, Q1, QTQ, H, Ht);
  std::copy(H.begin(), H.end(), Hv);
}

// Accumulated per-function seconds: gd_side, gd_cross, hess_vec, cg (incl.
// hess_vec), update_side, update_cross, cache_sasb.
void orc_times(double *out, int reset) {
  for (int i = 0; i < T_N; i++) {
    out[i] = g_time[i];
    if (reset) g_time[i] = 0;
  }
}

void orc_save_model(void *c, const char *path) { ((OrcCtx *)c)->prob.save_model(path); }
void orc_save_binary(void *c, const char *path) { ((OrcCtx *)c)->prob.save_binary(path); }

// Wall-clock seconds of `epochs` calls to one_epoch (the CPU baseline).
double orc_time_epochs(void *c, uint32_t epochs) {
  Problem &p = ((OrcCtx *)c)->prob;
  double t0 = omp_get_wtime();
  for (u32 e = 0; e < epochs; e++) p.one_epoch();
  return omp_get_wtime() - t0;
}

}  // extern "C"

// ----------------------------------------------------------- CLI main ---
#ifdef ORC_MAIN
// Mirrors train.cpp:53-207 (argv grammar, defaults, exit codes) so the
// product binary's stdout and model file can be compared on tiny inputs.
static bool has_digit(const char *s) {
  for (; *s; s++)
    if (std::isdigit((unsigned char)*s)) return true;
  return false;
}

int main(int argc, char **argv) {
  try {
    if (argc == 1) throw std::invalid_argument("usage: oracle_train [options] item_file train_file");
    Param prm;
    std::string te, model;
    int i = 1;
    for (; i < argc; i++) {
      std::string s = argv[i];
      auto need = [&](bool numeric) {
        if (i + 1 >= argc) throw std::invalid_argument("missing value after " + s);
        i++;
        if (numeric && !has_digit(argv[i])) throw std::invalid_argument(s + " should be followed by a number");
        return argv[i];
      };
      if (s == "-l") prm.lambda = std::atof(need(true));
      else if (s == "-k") prm.k = (u32)std::atoi(need(true));
      else if (s == "-t") prm.nr_pass = (u32)std::atoi(need(true));
      else if (s == "-w") prm.omega = std::atof(need(true));
      else if (s == "-r") prm.r = std::atof(need(true));
      else if (s == "-c") prm.nr_threads = (u32)std::atof(need(true));
      else if (s == "-p") te = need(false);
      else if (s == "-o") model = need(false);
      else if (s == "--ns") prm.self_side = false;
      else if (s == "--freq") prm.freq = true;
      else break;
    }
    if (i + 1 >= argc) throw std::invalid_argument("training data not specified");
    std::string xt = argv[i], tr = argv[i + 1];
    omp_set_num_threads((int)prm.nr_threads);
    Data U, V, Ut;
    build_data(U, parse_file(tr, true, nullptr, 0));
    build_data(V, parse_file(xt, false, nullptr, 0));
    trans_y(V, U);
    if (!te.empty()) build_data(Ut, parse_file(te, true, U.Ds.data(), U.Ds.size()));
    Problem p;
    p.U = &U;
    p.V = &V;
    p.Ut = te.empty() ? nullptr : &Ut;
    p.prm = prm;
    p.init();
    p.solve();
    if (!model.empty()) p.save_model(model);
  } catch (std::invalid_argument &e) {
    std::cerr << e.what() << std::endl;
    return 1;
  }
  return 0;
}
#endif
