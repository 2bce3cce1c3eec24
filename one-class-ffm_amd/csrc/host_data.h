// host_data.h — host-side data layer of the product (parser, per-field CSR,
// label transpose).  Restates ImpData (ffm.h:51-79, ffm.cpp:80-294).
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace ocffm {

struct Rows {  // one file before split_fields
  std::vector<uint64_t> xptr{0};
  std::vector<uint32_t> fid;
  std::vector<uint64_t> idx;
  std::vector<double> val;
  std::vector<uint64_t> yptr{0}, ycol;
  bool has_label = false;
  uint64_t f = 0, n = 0;
};

struct HostData {
  std::string path;
  bool has_label = false;
  uint64_t m = 0;  // rows
  uint64_t n = 0;  // max label + 1 (train/test)
  uint64_t f = 0;  // max fid + 1
  std::vector<uint64_t> nnx;         // kept feature nodes per row (ffm.cpp:126-181)
  std::vector<uint64_t> yptr, ycol;  // labels, user-major
  std::vector<uint64_t> Ds;          // per-field max idx + 1 (ffm.cpp:221)
  // The parsed nodes in row order (raw.xptr / fid / idx / val; its label
  // arrays are moved to yptr / ycol): the input of the on-device build
  // (devbuild.h) and of split_host.
  Rows raw;
  // per-field CSR (split_fields, ffm.cpp:185-257) and the item popularity
  // (ffm.cpp:143,172-176), built on the host only when something asks for
  // them (split_host: the host build path, the SGD mode, the data getters)
  mutable bool split_done = false;
  mutable std::vector<std::vector<int64_t>> xptr;
  mutable std::vector<std::vector<uint32_t>> xidx;
  mutable std::vector<std::vector<double>> xval;
  mutable std::vector<double> popular;
  // transY (ffm.cpp:259-294) was applied: the item-major positives are
  // built by the problem (on the device, or by the host build path)
  bool transposed = false;
};

// Throws std::runtime_error (I/O) or std::invalid_argument (malformed label,
// as stoi does in the reference, caught by train.cpp:201).
Rows parse_rows(const std::string &path, bool has_label, const uint64_t *ds, uint64_t nds);
// m, f, n, nnx, labels and Ds from the parsed rows (one parallel pass over
// the nodes); the rows are kept in d.raw.
void build(HostData &d, Rows &&r);
// split_fields + popularity on the host (once; idempotent).
const HostData &split_host(const HostData &d);
void trans_y(HostData &V, const HostData &U);

// ffm.cpp:71-78 + 3-12: one minstd_rand0 engine seeded from rand() per
// table, uniform_real_distribution<double>(-b, b), b = 0.1*qrsqrt(cols).
// Compiled with FMA contraction so the stream matches a -march=native build.
void init_table(double *out, uint64_t rows, uint32_t cols);

// The same draw's parameters for the device (devbuild.h draw_table): one
// rand() call (the engine seed, reduced as linear_congruential_engine::seed
// does), the distribution's a = -b and b - a, and the divisor of
// generate_canonical<double, 53> (r^2 rounded to double, r = 2^31 - 2).
struct TableDraw {
  uint64_t x0;
  double a, width, r2;
};
TableDraw table_draw(uint32_t cols);

}  // namespace ocffm
