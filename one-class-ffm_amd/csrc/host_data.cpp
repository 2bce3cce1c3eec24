// host_data.cpp — parser and CSR builder (host).  See host_data.h.
#include "host_data.h"

#include <algorithm>
#include <cctype>
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <mutex>
#include <random>
#include <stdexcept>
#include <string>
#include <thread>

namespace ocffm {

namespace {

inline bool is_ws(char c) { return c == ' ' || c == '\t' || c == '\r' || c == '\v' || c == '\f'; }

// operator>> on an unsigned long (num_get): skip white space, optional sign,
// digits.  Returns false when no digit follows.
inline bool read_u64(const char *&p, const char *e, uint64_t &out) {
  while (p < e && is_ws(*p)) p++;
  bool neg = false;
  if (p < e && (*p == '+' || *p == '-')) {
    neg = *p == '-';
    p++;
  }
  if (p >= e || !std::isdigit((unsigned char)*p)) return false;
  uint64_t v = 0;
  while (p < e && std::isdigit((unsigned char)*p)) v = v * 10 + (uint64_t)(*p++ - '0');
  out = neg ? (uint64_t)(-(int64_t)v) : v;
  return true;
}

// `iss >> dummy` for a char: skip white space, take one character.
inline bool read_char(const char *&p, const char *e) {
  while (p < e && is_ws(*p)) p++;
  if (p >= e) return false;
  p++;
  return true;
}

inline bool read_f64(const char *&p, const char *e, double &out) {
  while (p < e && is_ws(*p)) p++;
  if (p >= e) return false;
  char buf[64];
  size_t len = 0;
  while (p + len < e && !is_ws(p[len]) && len < sizeof(buf) - 1) {
    buf[len] = p[len];
    len++;
  }
  buf[len] = 0;
  char *end = nullptr;
  out = std::strtod(buf, &end);
  if (end == buf) return false;
  p += (end - buf);
  return true;
}

// std::stoi on one comma-separated label piece.
inline uint64_t parse_label(const char *b, const char *e) {
  const char *p = b;
  while (p < e && std::isspace((unsigned char)*p)) p++;
  bool neg = false;
  if (p < e && (*p == '+' || *p == '-')) {
    neg = *p == '-';
    p++;
  }
  if (p >= e || !std::isdigit((unsigned char)*p)) throw std::invalid_argument("stoi");
  int64_t v = 0;
  while (p < e && std::isdigit((unsigned char)*p)) {
    v = v * 10 + (*p++ - '0');
    if (v > 2147483647LL + (neg ? 1 : 0)) throw std::out_of_range("stoi");
  }
  if (neg && v != 0) throw std::invalid_argument("negative label");
  return (uint64_t)v;
}

}  // namespace

// One chunk of a file (whole lines) parsed by one thread.  Blank lines at
// the chunk start re-use the label block of an earlier chunk: they are
// counted (lead_blank) and resolved when the chunks are joined in order.
struct Chunk {
  Rows r;
  uint64_t lead_blank = 0;
  bool any_label = false;   // a non-blank line set the label block
  std::string last_block;   // the label block in force at the chunk end
  std::exception_ptr err;
};

static void parse_labels(const std::string &block, std::vector<uint64_t> &ycol, uint64_t &n) {
  const char *lb = block.data(), *le = lb + block.size();
  while (lb < le) {
    const char *c = (const char *)std::memchr(lb, ',', (size_t)(le - lb));
    if (!c) c = le;
    const uint64_t j = parse_label(lb, c);
    ycol.push_back(j);
    n = std::max(n, j + 1);
    lb = c + 1;
  }
}

// ffm.cpp:80-183 on the lines [s, end): label block, then fid:idx:val
// triples until the first token that does not parse; an empty line re-uses
// the previous label block (the stale label_block of ffm.cpp:93).
static void parse_chunk(const char *s, const char *end, bool has_label, const uint64_t *ds, uint64_t nds, Chunk &ck,
                        bool reserve) {
  Rows &r = ck.r;
  r.has_label = has_label;
  // Parallel chunks reserve from the chunk size (a label takes >= 2 bytes, a
  // node >= 6): growing vectors in parallel threads re-map memory, and every
  // unmap in a threaded process stalls all of its threads (TLB shootdowns).
  if (reserve) {
    const size_t bytes = (size_t)(end - s);
    size_t lines = 1;
    for (const char *q = s; (q = (const char *)std::memchr(q, '\n', (size_t)(end - q))) != nullptr; q++) lines++;
    r.xptr.reserve(lines + 1);
    if (has_label) {
      r.yptr.reserve(lines + 1);
      r.ycol.reserve(bytes / 2 + 1);
    }
    r.fid.reserve(bytes / 6 + 1);
    r.idx.reserve(bytes / 6 + 1);
    r.val.reserve(bytes / 6 + 1);
  }
  std::string &label_block = ck.last_block;
  while (s < end) {
    const char *e = (const char *)std::memchr(s, '\n', (size_t)(end - s));
    if (!e) e = end;
    const char *p = s;
    if (has_label) {
      while (p < e && std::isspace((unsigned char)*p)) p++;
      if (p < e) {
        const char *q = p;
        while (q < e && !std::isspace((unsigned char)*q)) q++;
        label_block.assign(p, q);
        ck.any_label = true;
        p = q;
      }
      if (!ck.any_label) ck.lead_blank++;  // labels resolved at the join
      else parse_labels(label_block, r.ycol, r.n);
      r.yptr.push_back(r.ycol.size());
    }
    while (true) {
      uint64_t fid, idx;
      double val;
      if (!read_u64(p, e, fid) || !read_char(p, e) || !read_u64(p, e, idx) || !read_char(p, e) ||
          !read_f64(p, e, val))
        break;
      r.f = std::max(r.f, fid + 1);
      if (ds != nullptr && (fid >= nds || ds[fid] <= idx)) continue;
      r.fid.push_back((uint32_t)fid);
      r.idx.push_back(idx);
      r.val.push_back(val);
    }
    r.xptr.push_back(r.fid.size());
    s = e + 1;
  }
}

// The whole file in memory, cut into line-aligned chunks parsed by parallel
// threads (files under 4 MB: one), joined in file order.
Rows parse_rows(const std::string &path, bool has_label, const uint64_t *ds, uint64_t nds) {
  FILE *fp = std::fopen(path.c_str(), "rb");
  if (!fp) throw std::runtime_error("cannot open " + path);
  std::fseek(fp, 0, SEEK_END);
  long sz = std::ftell(fp);
  std::fseek(fp, 0, SEEK_SET);
  std::string buf((size_t)std::max(0L, sz), '\0');
  if (sz > 0 && std::fread(&buf[0], 1, (size_t)sz, fp) != (size_t)sz) {
    std::fclose(fp);
    throw std::runtime_error("read failed: " + path);
  }
  std::fclose(fp);

  const char *b = buf.data(), *end = b + buf.size();
  const unsigned hw = std::max(1u, std::min(32u, std::thread::hardware_concurrency()));
  unsigned nth = buf.size() < (4u << 20) ? 1u : hw;
  if (const char *e = std::getenv("OCFFM_PARSE_CHUNKS")) nth = (unsigned)std::max(1, std::atoi(e));  // tests
  std::vector<const char *> cut{b};
  for (unsigned t = 1; t < nth; t++) {
    const char *c = std::max(cut.back(), b + buf.size() * t / nth);
    const char *nl = c < end ? (const char *)std::memchr(c, '\n', (size_t)(end - c)) : nullptr;
    cut.push_back(nl ? nl + 1 : end);
  }
  cut.push_back(end);
  std::vector<Chunk> ck(nth);
  auto work = [&](unsigned t) {
    try {
      parse_chunk(cut[t], cut[t + 1], has_label, ds, nds, ck[t], nth > 1);
    } catch (...) {
      ck[t].err = std::current_exception();
    }
  };
  std::vector<std::thread> th;
  for (unsigned t = 1; t < nth; t++) th.emplace_back(work, t);
  work(0);
  for (auto &x : th) x.join();

  // join in file order; the first error in file order wins, as in a serial read
  Rows r;
  r.has_label = has_label;
  if (nth == 1 && !ck[0].err && !ck[0].lead_blank) return std::move(ck[0].r);
  size_t nx = 0, ny = 0, nr = 0;
  for (auto &c : ck) {
    nx += c.r.fid.size();
    ny += c.r.ycol.size();
    nr += c.r.xptr.size();
  }
  r.fid.reserve(nx);
  r.idx.reserve(nx);
  r.val.reserve(nx);
  r.xptr.reserve(nr);
  if (has_label) {
    r.yptr.reserve(nr);
    r.ycol.reserve(ny + 1024);
  }
  std::string carried;  // label block in force before the chunk
  for (unsigned t = 0; t < nth; t++) {
    Chunk &c = ck[t];
    std::vector<uint64_t> inherited;
    if (has_label && c.lead_blank) {
      try {
        parse_labels(carried, inherited, r.n);
      } catch (...) {
        std::rethrow_exception(std::current_exception());
      }
    }
    if (c.err) std::rethrow_exception(c.err);
    const uint64_t x0 = r.fid.size();
    r.fid.insert(r.fid.end(), c.r.fid.begin(), c.r.fid.end());
    r.idx.insert(r.idx.end(), c.r.idx.begin(), c.r.idx.end());
    r.val.insert(r.val.end(), c.r.val.begin(), c.r.val.end());
    for (size_t i = 1; i < c.r.xptr.size(); i++) r.xptr.push_back(x0 + c.r.xptr[i]);
    if (has_label) {
      uint64_t y0 = r.ycol.size();
      for (uint64_t i = 0; i < c.lead_blank; i++) {
        r.ycol.insert(r.ycol.end(), inherited.begin(), inherited.end());
        r.yptr.push_back(r.ycol.size());
      }
      y0 = r.ycol.size();
      r.ycol.insert(r.ycol.end(), c.r.ycol.begin(), c.r.ycol.end());
      for (size_t i = 1 + c.lead_blank; i < c.r.yptr.size(); i++) r.yptr.push_back(y0 + c.r.yptr[i]);
      if (c.any_label) carried = c.last_block;
    }
    r.f = std::max(r.f, c.r.f);
    r.n = std::max(r.n, c.r.n);
  }
  return r;
}

// The row-level part of ImpData::read / split_fields: m, f, n, nnx, the
// labels and Ds (ffm.cpp:126-181, 221), by one pass over the nodes cut
// among host threads.  The per-field split itself is deferred: the device
// build (devbuild.h) does it, or split_host when a host consumer asks.
void build(HostData &d, Rows &&r) {
  d.has_label = r.has_label;
  d.m = r.xptr.size() - 1;
  d.f = r.f;
  d.n = r.n;
  d.nnx.resize(d.m);
  for (uint64_t i = 0; i < d.m; i++) d.nnx[i] = r.xptr[i + 1] - r.xptr[i];
  if (r.has_label) {
    d.yptr = std::move(r.yptr);
    d.ycol = std::move(r.ycol);
  } else {
    d.yptr.assign(d.m + 1, 0);
    d.ycol.clear();
  }
  r.yptr.assign(1, 0);
  r.ycol.clear();
  const uint64_t nn = r.fid.size(), f = d.f;
  const unsigned hw = std::max(1u, std::min(32u, std::thread::hardware_concurrency()));
  const unsigned nth = nn < (1u << 20) ? 1u : hw;
  std::vector<std::vector<uint64_t>> ds(nth, std::vector<uint64_t>(f, 0));
  std::vector<char> bad(nth, 0);
  auto work = [&](unsigned t) {
    const uint64_t a = nn * t / nth, b = nn * (t + 1) / nth;
    std::vector<uint64_t> &m = ds[t];
    for (uint64_t p = a; p < b; p++) {
      const uint64_t x = r.idx[p];
      if (x >= (1ULL << 32) - 1) bad[t] = 1;
      m[r.fid[p]] = std::max<uint64_t>(m[r.fid[p]], x + 1);
    }
  };
  std::vector<std::thread> th;
  for (unsigned t = 1; t < nth; t++) th.emplace_back(work, t);
  work(0);
  for (auto &x : th) x.join();
  for (char b : bad)
    if (b) throw std::runtime_error("feature index exceeds 2^32-2");
  d.Ds.assign(f, 0);
  for (auto &m : ds)
    for (uint64_t fi = 0; fi < f; fi++) d.Ds[fi] = std::max(d.Ds[fi], m[fi]);
  d.raw = std::move(r);
}

// split_fields (ffm.cpp:185-257) + popularity (ffm.cpp:143,172-176) on the
// host: the checker of the device build and the input of the host consumers.
// Consumers on several threads may share one data set (per-GPU problems
// created concurrently): the lazy split runs under one lock, once.
const HostData &split_host(const HostData &d) {
  static std::mutex mu;
  std::lock_guard<std::mutex> lk(mu);
  if (d.split_done) return d;
  const Rows &r = d.raw;
  if (d.has_label) {
    d.popular.assign(d.n, 0.0);
    for (uint64_t j : d.ycol) d.popular[j] += 1;
    double s = 0;
    for (double v : d.popular) s += v;
    for (double &v : d.popular) v /= s;
  }
  d.xptr.assign(d.f, std::vector<int64_t>(d.m + 1, 0));
  d.xidx.assign(d.f, {});
  d.xval.assign(d.f, {});
  for (uint64_t i = 0; i < d.m; i++)
    for (uint64_t p = r.xptr[i]; p < r.xptr[i + 1]; p++) d.xptr[r.fid[p]][i + 1]++;
  for (uint64_t fi = 0; fi < d.f; fi++) {
    for (uint64_t i = 0; i < d.m; i++) d.xptr[fi][i + 1] += d.xptr[fi][i];
    d.xidx[fi].resize((size_t)d.xptr[fi][d.m]);
    d.xval[fi].resize((size_t)d.xptr[fi][d.m]);
  }
  std::vector<uint64_t> cur(d.f, 0);
  for (uint64_t i = 0; i < d.m; i++)
    for (uint64_t p = r.xptr[i]; p < r.xptr[i + 1]; p++) {
      const uint32_t fi = r.fid[p];
      const uint64_t q = cur[fi]++;
      d.xidx[fi][q] = (uint32_t)r.idx[p];
      d.xval[fi][q] = r.val[p];
    }
  d.split_done = true;
  return d;
}

// ffm.cpp:259-294.  The item-major positives themselves are built by the
// problem (solver.hip build_item_side: on the device, or on the host with
// OCFFM_HOST_BUILD=1), restricted to its rank's users; here only the
// pairing is recorded.  Labels >= #items: the reference skips them in
// transY and then reads out of bounds; the problem constructor rejects them.
void trans_y(HostData &V, const HostData &U) {
  (void)U;
  V.transposed = true;
}

// ffm.cpp:3-12.
static double qrsqrt(double x) {
  const double half = 0.5 * x;
  uint64_t bits;
  std::memcpy(&bits, &x, 8);
  bits = 0x5fe6eb50c7b537a9ULL - (bits >> 1);
  std::memcpy(&x, &bits, 8);
  return x * (1.5 - half * x * x);
}

// The table's one engine is consumed in order; every double takes exactly
// two engine steps (generate_canonical<double, 53> over minstd_rand0's
// 31-bit range), so the stream is cut into chunks whose start state is the
// seed state times a^(2*start) mod m (LCG jump-ahead) and the chunks are
// drawn by parallel threads through the same distribution object code: the
// values are those of one serial pass.
static uint64_t mulmod(uint64_t a, uint64_t b, uint64_t m) { return (uint64_t)((unsigned __int128)a * b % m); }
static uint64_t powmod(uint64_t a, uint64_t e, uint64_t m) {
  uint64_t r = 1;
  for (a %= m; e; e >>= 1, a = mulmod(a, a, m))
    if (e & 1) r = mulmod(r, a, m);
  return r;
}

TableDraw table_draw(uint32_t cols) {
  using E = std::minstd_rand0;
  const uint64_t seed = (uint64_t)(unsigned)std::rand();
  const double b = 0.1 * qrsqrt((double)cols);
  TableDraw t;
  t.x0 = seed % E::modulus;
  if (t.x0 == 0) t.x0 = 1;
  t.a = -b;
  t.width = b - t.a;  // uniform_real_distribution: a + (b - a) * canonical
  const long double r = (long double)E::max() - (long double)E::min() + 1.0L;
  t.r2 = (double)((long double)(double)r * r);  // generate_canonical's tmp after two rounds
  return t;
}

void init_table(double *out, uint64_t rows, uint32_t cols) {
  using E = std::minstd_rand0;
  const uint64_t seed = (uint64_t)(unsigned)std::rand();
  const double b = 0.1 * qrsqrt((double)cols);
  const uint64_t nn = rows * cols;
  uint64_t x0 = seed % E::modulus;
  if (x0 == 0) x0 = 1;  // linear_congruential_engine::seed
  const unsigned hw = std::max(1u, std::min(32u, std::thread::hardware_concurrency()));
  const unsigned nth = nn < (1u << 16) ? 1u : hw;
  auto work = [&](unsigned t) {
    const uint64_t i0 = nn * t / nth, i1 = nn * (t + 1) / nth;
    E eng((E::result_type)mulmod(x0, powmod(E::multiplier, 2 * i0, E::modulus), E::modulus));
    std::uniform_real_distribution<double> dist(-b, b);
    for (uint64_t i = i0; i < i1; i++) out[i] = dist(eng);
  };
  std::vector<std::thread> th;
  for (unsigned t = 1; t < nth; t++) th.emplace_back(work, t);
  work(0);
  for (auto &x : th) x.join();
}

}  // namespace ocffm
