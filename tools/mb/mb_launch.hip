// Microbenchmark: fixed costs on MI355X — an empty kernel, a kernel with the
// solver's grid reduction (fin_blocks: block sums + two-level last-block
// ticket), back to back on one stream.  Build:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I one-class-ffm_amd/csrc -o build/mb_launch tools/mb/mb_launch.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "kernels.hpp"

using namespace ocffm;
#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); \
      std::exit(1);                                                        \
    }                                                                      \
  } while (0)

__global__ __launch_bounds__(256) void k_empty(int *x) {
  if (threadIdx.x == 0 && blockIdx.x == 0 && x[0] == 12345) x[1] = 1;
}
__global__ __launch_bounds__(256) void k_red(Fin<float> f) {
  double ds[3] = {1.0 * threadIdx.x, 2.0, 3.0};
  fin_blocks<float, 1>(f, ds);
}

template <class F> float timeit(F &&f, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  f();
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a));
  for (int i = 0; i < reps; i++) f();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms * 1e3f / reps;
}

int main() {
  int *x;
  CK(hipMalloc(&x, 64));
  CK(hipMemset(x, 0, 64));
  double *part;
  unsigned *tick;
  CgState *st;
  CK(hipMalloc(&part, (1 << 20) * 8));
  CK(hipMalloc(&tick, TICK_WORDS * 4));
  CK(hipMemset(tick, 0, TICK_WORDS * 4));
  CK(hipMalloc(&st, sizeof(CgState)));
  CgState hs{};
  hs.r2 = 1;
  hs.g2 = 1;
  CK(hipMemcpy(st, &hs, sizeof hs, hipMemcpyHostToDevice));
  int *hostflag;
  CK(hipHostMalloc(&hostflag, 4096, hipHostMallocMapped));
  int *hostflag_dev;
  CK(hipHostGetDevicePointer((void **)&hostflag_dev, hostflag, 0));
  for (unsigned g : {1u, 64u, 256u, 1024u, 4096u}) {
    float us = timeit([&] { k_empty<<<g, 256>>>(x); }, 200);
    std::printf("empty kernel grid %5u: %6.2f us per launch (back to back)\n", g, us);
  }
  for (unsigned g : {64u, 256u, 1024u, 3125u}) {
    Fin<float> f{};
    f.lam = 1;
    f.st = st;
    f.part = part;
    f.tick = tick;
    f.it = 1;
    float us = timeit([&] { k_red<<<g, 256>>>(f); }, 200);
    f.run_host = hostflag_dev;
    float us2 = timeit([&] { k_red<<<g, 256>>>(f); }, 200);
    std::printf("grid reduction   grid %5u: %6.2f us per launch; with host-mapped flag %6.2f us\n", g, us, us2);
  }
  return 0;
}
