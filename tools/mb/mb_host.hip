// Microbenchmark: host-side costs around a CG verdict on MI355X.
//   1. host time per hipExtLaunchKernelGGL / hipLaunchKernelGGL (enqueue only)
//   2. round trip: a kernel publishes a host-mapped flag (system-scope store,
//      as cg_publish does), the host spins on it and launches the next kernel
//   3. the same with hipEventSynchronize instead of the spin
// Build (in-tree, CPU):
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/mb/mb_host tools/mb/mb_host.hip
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); \
      std::exit(1);                                                        \
    }                                                                      \
  } while (0)

struct Big {  // a kernel argument block of the solver's size (~200 B)
  void *p[20];
  double d[4];
};

__global__ __launch_bounds__(256) void k_empty(int *x, Big b) {
  if (threadIdx.x == 0 && blockIdx.x == 0 && x[0] == 12345) x[1] = (int)b.d[0];
}
__global__ __launch_bounds__(256) void k_flag(int *flag, int v) {
  if (threadIdx.x == 0 && blockIdx.x == gridDim.x - 1)
    __hip_atomic_store(flag, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
  int *x;
  CK(hipMalloc(&x, 64));
  CK(hipMemset(x, 0, 64));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  Big b{};
  const int N = 400;
  for (int rep = 0; rep < 2; rep++) {
    CK(hipStreamSynchronize(s));
    double t0 = now_us();
    for (int i = 0; i < N; i++) hipExtLaunchKernelGGL(k_empty, dim3(1024), dim3(256), 0, s, nullptr, nullptr, 0u, x, b);
    double t1 = now_us();
    CK(hipStreamSynchronize(s));
    double t2 = now_us();
    for (int i = 0; i < N; i++) hipLaunchKernelGGL(k_empty, dim3(1024), dim3(256), 0, s, x, b);
    double t3 = now_us();
    CK(hipStreamSynchronize(s));
    double t4 = now_us();
    std::printf("enqueue: hipExtLaunchKernelGGL %.2f us, hipLaunchKernelGGL %.2f us per launch; GPU drain %.2f / %.2f us per kernel\n",
                (t1 - t0) / N, (t3 - t2) / N, (t2 - t0) / N, (t4 - t2) / N);
  }
  int *hflag, *dflag;
  CK(hipHostMalloc((void **)&hflag, 4096, hipHostMallocMapped | hipHostMallocCoherent));
  CK(hipHostGetDevicePointer((void **)&dflag, hflag, 0));
  for (unsigned g : {1u, 1024u}) {
    *hflag = 0;
    CK(hipStreamSynchronize(s));
    double t0 = now_us();
    for (int i = 1; i <= N; i++) {
      hipExtLaunchKernelGGL(k_flag, dim3(g), dim3(256), 0, s, nullptr, nullptr, 0u, dflag, i);
      while (__atomic_load_n(hflag, __ATOMIC_ACQUIRE) != i) __builtin_ia32_pause();
    }
    double t1 = now_us();
    std::printf("round trip (launch, kernel publishes flag, host spin sees it), grid %u: %.2f us\n", g, (t1 - t0) / N);
    hipEvent_t e;
    CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    t0 = now_us();
    for (int i = 1; i <= N; i++) {
      hipExtLaunchKernelGGL(k_flag, dim3(g), dim3(256), 0, s, nullptr, nullptr, 0u, dflag, i);
      CK(hipEventRecord(e, s));
      CK(hipEventSynchronize(e));
    }
    t1 = now_us();
    std::printf("round trip with hipEventRecord + hipEventSynchronize, grid %u: %.2f us\n", g, (t1 - t0) / N);
    CK(hipEventDestroy(e));
  }
  // back to back: kernel with flag, host launches next one only after seeing
  // the flag but with one kernel of look-ahead already queued (the solver's scheme)
  {
    *hflag = 0;
    CK(hipStreamSynchronize(s));
    double t0 = now_us();
    hipExtLaunchKernelGGL(k_flag, dim3(1024), dim3(256), 0, s, nullptr, nullptr, 0u, dflag, 1);
    for (int i = 2; i <= N; i++) {
      hipExtLaunchKernelGGL(k_flag, dim3(1024), dim3(256), 0, s, nullptr, nullptr, 0u, dflag, i);
      while (__atomic_load_n(hflag, __ATOMIC_ACQUIRE) < i - 1) __builtin_ia32_pause();
    }
    CK(hipStreamSynchronize(s));
    double t1 = now_us();
    std::printf("look-ahead 1 chain of flag kernels: %.2f us per kernel\n", (t1 - t0) / N);
  }
  // a captured graph of K kernels: host cost of hipGraphLaunch and GPU time per kernel
  for (int K : {1, 4, 8, 16}) {
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    for (int k = 0; k < K; k++) hipLaunchKernelGGL(k_empty, dim3(1024), dim3(256), 0, s, x, b);
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CK(hipGraphLaunch(ge, s));
    CK(hipStreamSynchronize(s));
    const int M = 100;
    double t0 = now_us();
    for (int i = 0; i < M; i++) CK(hipGraphLaunch(ge, s));
    double t1 = now_us();
    CK(hipStreamSynchronize(s));
    double t2 = now_us();
    std::printf("graph of %2d kernels: hipGraphLaunch %.2f us host per launch (%.2f per kernel); GPU %.2f us per kernel\n",
                K, (t1 - t0) / M, (t1 - t0) / M / K, (t2 - t0) / M / K);
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
  }
  return 0;
}
