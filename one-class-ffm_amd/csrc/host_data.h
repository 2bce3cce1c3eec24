// host_data.h — host-side data layer of the product (parser, per-field CSR,
// label transpose).  Restates ImpData (ffm.h:51-79, ffm.cpp:80-294).
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace ocffm {

struct HostData {
  std::string path;
  bool has_label = false;
  uint64_t m = 0;  // rows
  uint64_t n = 0;  // max label + 1 (train/test)
  uint64_t f = 0;  // max fid + 1
  std::vector<uint64_t> nnx;         // kept feature nodes per row (ffm.cpp:126-181)
  std::vector<uint64_t> yptr, ycol;  // labels, user-major
  // per-field CSR (split_fields, ffm.cpp:185-257)
  std::vector<std::vector<int64_t>> xptr;
  std::vector<std::vector<uint32_t>> xidx;
  std::vector<std::vector<double>> xval;
  std::vector<uint64_t> Ds;
  std::vector<double> popular;  // normalised label counts (ffm.cpp:143,172-176)
  // item-major positives from transY (ffm.cpp:259-294): for item j, the
  // users that have j as a label, in increasing user order.
  bool transposed = false;
  std::vector<uint64_t> tptr;
  std::vector<uint32_t> tcol;
};

struct Rows {  // one file before split_fields
  std::vector<uint64_t> xptr{0};
  std::vector<uint32_t> fid;
  std::vector<uint64_t> idx;
  std::vector<double> val;
  std::vector<uint64_t> yptr{0}, ycol;
  bool has_label = false;
  uint64_t f = 0, n = 0;
};

// Throws std::runtime_error (I/O) or std::invalid_argument (malformed label,
// as stoi does in the reference, caught by train.cpp:201).
Rows parse_rows(const std::string &path, bool has_label, const uint64_t *ds, uint64_t nds);
void build(HostData &d, const Rows &r);
void trans_y(HostData &V, const HostData &U);

// ffm.cpp:71-78 + 3-12: one minstd_rand0 engine seeded from rand() per
// table, uniform_real_distribution<double>(-b, b), b = 0.1*qrsqrt(cols).
// Compiled with FMA contraction so the stream matches a -march=native build.
void init_table(double *out, uint64_t rows, uint32_t cols);

}  // namespace ocffm
