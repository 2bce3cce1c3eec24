// Sanitizer driver for the product's host data layer (test infrastructure).
// Built with -fsanitize=address,undefined by tests/sanitize/Makefile and run
// by tests/test_sanitize.py over the parser's edge-case inputs.  It drives
// the same calls as the C ABI (ocffm_data_read: parse_rows + build;
// ocffm_data_trans_y; the data getters: split_host), restating ImpData
// (/root/reference/ffm.cpp:80-294), and prints a digest of what was parsed.
//
//   parse_driver TRAIN ITEM [TEST]
// exit 0 ok, 3 invalid_argument (a malformed label, as stoi throws in the
// reference, train.cpp:201), 4 any other error (I/O).
#include <cstdio>
#include <stdexcept>
#include <string>

#include "host_data.h"

using namespace ocffm;

static uint64_t fnv(uint64_t h, const void *p, size_t n) {
  const unsigned char *c = static_cast<const unsigned char *>(p);
  for (size_t i = 0; i < n; i++) h = (h ^ c[i]) * 1099511628211ull;
  return h;
}

template <class T> static uint64_t digest(uint64_t h, const std::vector<T> &v) {
  return v.empty() ? h : fnv(h, v.data(), v.size() * sizeof(T));
}

static uint64_t describe(const char *what, const HostData &d) {
  const HostData &s = split_host(d);
  uint64_t h = 1469598103934665603ull;
  h = digest(h, s.nnx);
  h = digest(h, s.yptr);
  h = digest(h, s.ycol);
  h = digest(h, s.Ds);
  for (size_t f = 0; f < s.xptr.size(); f++) {
    h = digest(h, s.xptr[f]);
    h = digest(h, s.xidx[f]);
    h = digest(h, s.xval[f]);
  }
  h = digest(h, s.popular);
  std::printf("%s m=%llu n=%llu f=%llu nnz_x=%zu nnz_y=%zu digest=%016llx\n", what, (unsigned long long)s.m,
              (unsigned long long)s.n, (unsigned long long)s.f, s.raw.fid.size(), s.ycol.size(),
              (unsigned long long)h);
  return h;
}

int main(int argc, char **argv) {
  if (argc < 3) {
    std::fprintf(stderr, "usage: parse_driver TRAIN ITEM [TEST]\n");
    return 2;
  }
  try {
    HostData U, V, Ut;
    build(U, parse_rows(argv[1], true, nullptr, 0));
    build(V, parse_rows(argv[2], false, nullptr, 0));
    trans_y(V, U);
    describe("train", U);
    describe("item", V);
    if (argc > 3) {
      build(Ut, parse_rows(argv[3], true, U.Ds.data(), U.Ds.size()));
      describe("test", Ut);
    }
    // the init stream over a table of every field's shape
    for (uint64_t f = 0; f < U.Ds.size(); f++) {
      std::vector<double> w(U.Ds[f] * 5 + 1);
      init_table(w.data(), U.Ds[f], 5);
    }
  } catch (const std::invalid_argument &e) {
    std::printf("invalid_argument: %s\n", e.what());
    return 3;
  } catch (const std::exception &e) {
    std::printf("error: %s\n", e.what());
    return 4;
  }
  return 0;
}
