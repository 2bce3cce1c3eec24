// host_data.cpp — parser and CSR builder (host).  See host_data.h.
#include "host_data.h"

#include <algorithm>
#include <cctype>
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <stdexcept>

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

// ffm.cpp:80-183 in one pass: label block, then fid:idx:val triples until the
// first token that does not parse; an empty line re-uses the previous label
// block (the stale label_block of ffm.cpp:93).
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

  Rows r;
  r.has_label = has_label;
  std::string label_block;
  const char *s = buf.data(), *end = s + buf.size();
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
        p = q;
      }
      const char *lb = label_block.data(), *le = lb + label_block.size();
      while (lb < le) {
        const char *c = (const char *)std::memchr(lb, ',', (size_t)(le - lb));
        if (!c) c = le;
        uint64_t j = parse_label(lb, c);
        r.ycol.push_back(j);
        r.n = std::max(r.n, j + 1);
        lb = c + 1;
      }
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
  return r;
}

// split_fields (ffm.cpp:185-257) + popularity (ffm.cpp:143,172-176).
void build(HostData &d, const Rows &r) {
  d.has_label = r.has_label;
  d.m = r.xptr.size() - 1;
  d.f = r.f;
  d.n = r.n;
  d.nnx.resize(d.m);
  for (uint64_t i = 0; i < d.m; i++) d.nnx[i] = r.xptr[i + 1] - r.xptr[i];
  if (r.has_label) {
    d.yptr = r.yptr;
    d.ycol = r.ycol;
    d.popular.assign(d.n, 0.0);
    for (uint64_t j : d.ycol) d.popular[j] += 1;
    double s = 0;
    for (double v : d.popular) s += v;
    for (double &v : d.popular) v /= s;
  } else {
    d.yptr.assign(d.m + 1, 0);
    d.ycol.clear();
  }
  d.xptr.assign(d.f, std::vector<int64_t>(d.m + 1, 0));
  d.xidx.assign(d.f, {});
  d.xval.assign(d.f, {});
  d.Ds.assign(d.f, 0);
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
      if (r.idx[p] >= (1ULL << 32) - 1) throw std::runtime_error("feature index exceeds 2^32-2");
      const uint64_t q = cur[fi]++;
      d.xidx[fi][q] = (uint32_t)r.idx[p];
      d.xval[fi][q] = r.val[p];
      d.Ds[fi] = std::max<uint64_t>(d.Ds[fi], r.idx[p] + 1);
    }
}

// ffm.cpp:259-294.  Labels >= #items are skipped here like the reference;
// the problem constructor rejects them (the reference reads out of bounds).
void trans_y(HostData &V, const HostData &U) {
  std::vector<uint64_t> cnt(V.m + 1, 0);
  for (uint64_t p = 0; p < U.ycol.size(); p++)
    if (U.ycol[p] < V.m) cnt[U.ycol[p] + 1]++;
  for (uint64_t j = 0; j < V.m; j++) cnt[j + 1] += cnt[j];
  V.tptr = cnt;
  V.tcol.assign(cnt[V.m], 0);
  std::vector<uint64_t> cur(cnt.begin(), cnt.end() - 1);
  for (uint64_t i = 0; i < U.m; i++)
    for (uint64_t p = U.yptr[i]; p < U.yptr[i + 1]; p++) {
      const uint64_t j = U.ycol[p];
      if (j < V.m) V.tcol[cur[j]++] = (uint32_t)i;
    }
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

void init_table(double *out, uint64_t rows, uint32_t cols) {
  std::minstd_rand0 eng(std::rand());
  const double b = 0.1 * qrsqrt((double)cols);
  std::uniform_real_distribution<double> dist(-b, b);
  const uint64_t nn = rows * cols;
  for (uint64_t i = 0; i < nn; i++) out[i] = dist(eng);
}

}  // namespace ocffm
