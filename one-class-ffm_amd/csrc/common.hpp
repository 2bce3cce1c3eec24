// common.hpp — host-side pieces shared by the library's translation units
// (solver.hip: the Newton-CG path; sgd.hip: the SGD/AdaGrad path): error
// codes through the C ABI, HIP/RCCL checks, device buffers.
#pragma once

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <new>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/ocffm.h"
#include "host_data.h"

namespace ocffm {

// ----------------------------------------------------------------- errors
struct Error : std::runtime_error {
  int code;
  Error(int c, const std::string &m) : std::runtime_error(m), code(c) {}
};
extern thread_local std::string g_last_error;  // solver.hip

#define HIPCHK(x)                                                                                 \
  do {                                                                                            \
    hipError_t e_ = (x);                                                                          \
    if (e_ != hipSuccess)                                                                         \
      throw Error(OCFFM_E_HIP, std::string("HIP: ") + hipGetErrorString(e_) + " at " #x);         \
  } while (0)
#define NCCLCHK(x)                                                                                \
  do {                                                                                            \
    ncclResult_t r_ = (x);                                                                        \
    if (r_ != ncclSuccess) throw Error(OCFFM_E_COMM, std::string("RCCL: ") + ncclGetErrorString(r_)); \
  } while (0)

template <typename T> struct DevBuf {
  T *p = nullptr;
  size_t n = 0;
  DevBuf() = default;
  DevBuf(const DevBuf &) = delete;
  DevBuf &operator=(const DevBuf &) = delete;
  DevBuf(DevBuf &&o) noexcept : p(o.p), n(o.n) {
    o.p = nullptr;
    o.n = 0;
  }
  DevBuf &operator=(DevBuf &&o) noexcept {
    if (this != &o) {
      release();
      p = o.p;
      n = o.n;
      o.p = nullptr;
      o.n = 0;
    }
    return *this;
  }
  ~DevBuf() { release(); }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
  }
  void alloc(size_t count, bool zero = true) {
    release();
    n = count;
    if (count == 0) return;
    HIPCHK(hipMalloc(&p, count * sizeof(T)));
    if (zero) {
      // The solver streams are non-blocking: they do not wait for the legacy
      // null stream, so the fill must have landed before any kernel runs.
      HIPCHK(hipMemset(p, 0, count * sizeof(T)));
      HIPCHK(hipStreamSynchronize(nullptr));
    }
  }
  void upload(const T *src, size_t count) {
    alloc(count, false);
    if (count) HIPCHK(hipMemcpy(p, src, count * sizeof(T), hipMemcpyHostToDevice));
  }
  void upload(const std::vector<T> &v) { upload(v.data(), v.size()); }
  uint64_t bytes() const { return (uint64_t)n * sizeof(T); }
};

}  // namespace ocffm

struct ocffm_data {
  ocffm::HostData d;
};

// Run an ABI body: exceptions become status codes + ocffm_last_error().
template <class F> inline int guarded(F &&f) {
  using ocffm::Error;
  using ocffm::g_last_error;
  try {
    f();
    return OCFFM_OK;
  } catch (Error &e) {
    g_last_error = e.what();
    return e.code;
  } catch (std::invalid_argument &e) {
    g_last_error = std::string("invalid argument: ") + e.what();
    return OCFFM_E_ARG;
  } catch (std::out_of_range &e) {
    g_last_error = std::string("out of range: ") + e.what();
    return OCFFM_E_DATA;
  } catch (std::bad_alloc &) {
    g_last_error = "host out of memory";
    return OCFFM_E_HIP;
  } catch (std::exception &e) {
    g_last_error = e.what();
    return OCFFM_E_IO;
  }
}

