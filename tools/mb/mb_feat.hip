// Microbenchmark: the Hessian-vector feature pass (k_feat, MODE 1) on an
// id-like field (D columns of one entry each, kkbox item-id shape) against
// a pure streaming kernel moving the same bytes.  Build:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I one-class-ffm_amd/csrc -o build/mb_feat tools/mb/mb_feat.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <algorithm>
#include <cstdlib>
#include <vector>

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

// same traffic as MODE 1 finalisation with upd: read P,R,Hp,S,h; write P,R,S,Hp
__global__ __launch_bounds__(256) void k_stream(uint64_t nv, const float4 *h, float4 *P, float4 *R, float4 *Hp,
                                                float4 *S) {
  for (uint64_t v = (uint64_t)blockIdx.x * 256 + threadIdx.x; v < nv; v += (uint64_t)gridDim.x * 256) {
    float4 a = P[v], b = R[v], c = Hp[v], d = S[v], e = h[v];
    float4 rn = b - 0.5f * c, pe = rn + 0.25f * a;
    S[v] = d + 0.5f * a;
    R[v] = rn;
    P[v] = pe;
    Hp[v] = 2.f * pe + e;
  }
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

int main(int argc, char **argv) {
  const uint64_t D = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 100000;
  constexpr int KP = 32;
  using G = Geo<float, KP>;
  const uint64_t n = D * KP;
  float *P, *R, *Hp, *S, *W, *h, *acc, *wpart, *cval;
  uint32_t *crow;
  unsigned *cnt;
  double *part;
  CgState *st;
  Job *jobs;
  CK(hipMalloc(&P, n * 4));
  CK(hipMalloc(&R, n * 4));
  CK(hipMalloc(&Hp, n * 4));
  CK(hipMalloc(&S, n * 4));
  CK(hipMalloc(&W, n * 4));
  CK(hipMalloc(&h, n * 4));
  CK(hipMalloc(&acc, n * 4));
  CK(hipMalloc(&wpart, 1024 * 4));
  CK(hipMalloc(&crow, D * 4));
  CK(hipMalloc(&cval, D * 4));
  CK(hipMalloc(&cnt, D * 4));
  CK(hipMalloc(&part, (1 << 20) * 8));
  CK(hipMalloc(&st, sizeof(CgState)));
  std::vector<float> hv(n);
  for (uint64_t i = 0; i < n; i++) hv[i] = (float)((i * 2654435761u) % 1000) * 1e-3f;
  for (float *p : {P, R, Hp, S, W, h}) CK(hipMemcpy(p, hv.data(), n * 4, hipMemcpyHostToDevice));
  std::vector<uint32_t> cr(D);
  std::vector<float> cv(D, 1.f);
  for (uint64_t d = 0; d < D; d++) cr[d] = (uint32_t)d;
  CK(hipMemcpy(crow, cr.data(), D * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(cval, cv.data(), D * 4, hipMemcpyHostToDevice));
  CK(hipMemset(cnt, 0, D * 4));
  std::vector<Job> jb;
  for (uint64_t d = 0; d < D; d++) jb.push_back(Job{(uint32_t)d, 1u, 0u, 0u, (int64_t)d, (int64_t)d + 1});
  while (jb.size() % G::NSG) jb.push_back(Job{JOB_NONE, 1u, 0u, 0u, 0, 0});
  CK(hipMalloc(&jobs, jb.size() * sizeof(Job)));
  CK(hipMemcpy(jobs, jb.data(), jb.size() * sizeof(Job), hipMemcpyHostToDevice));
  unsigned *tick, *tick_;
  CK(hipMalloc(&tick, TICK_WORDS * 4));
  CK(hipMemset(tick, 0, TICK_WORDS * 4));
  tick_ = tick;
  CgState hs{};
  for (int i = 0; i < MAXCG + 2; i++) hs.run[i] = 1;
  hs.alpha = 1e-3;
  hs.beta = 0.5;
  hs.r2 = 1;
  hs.g2 = 1;
  CK(hipMemcpy(st, &hs, sizeof hs, hipMemcpyHostToDevice));

  Fin<float> f{nullptr, 1.0, W, nullptr, S, P, R, Hp, acc, cnt, st, part, tick, nullptr, 2};
  const uint64_t njw = jb.size() / G::NSG;
  {
    float us1 = 0;
    for (unsigned g : {512u, 1024u, 2048u, (unsigned)((njw + 3) / 4)}) {
      us1 = timeit([&] { k_feat<float, KP, 1, 1><<<std::min(g, (unsigned)((njw + 3) / 4)), 256>>>(njw, jobs, crow, cval, h, D * KP * 4, wpart, Fin<float>{nullptr, 1.0, W, nullptr, S, P, R, Hp, acc, cnt, st, part, tick_, nullptr, 2}, nullptr); }, 50);
      std::printf("k_feat JE=1 MODE1 grid %u: %8.2f us\n", g, us1);
    }
  }
  const double bytes = (double)n * 4 * 9 + D * (4 + 4 + sizeof(Job));
  float us = 0;
  for (unsigned g : {256u, 512u, 1024u, 2048u, (unsigned)((njw + 3) / 4)}) {
    us = timeit([&] { k_feat<float, KP, 1><<<std::min(g, (unsigned)((njw + 3) / 4)), 256>>>(njw, jobs, crow, cval, h, n * 4, wpart, f); }, 50);
    std::printf("k_feat  MODE1 D=%lu grid %u: %8.2f us  %7.1f GB/s\n", (unsigned long)D, g, us, bytes / us / 1e3);
  }
  f.it = 1;
  us = timeit([&] { k_feat<float, KP, 1><<<(unsigned)((njw + 3) / 4), 256>>>(njw, jobs, crow, cval, h, n * 4, wpart, f); }, 50);
  std::printf("k_feat  it=1     : %8.2f us\n", us);
  us = timeit([&] { k_feat<float, KP, 2><<<(unsigned)((njw + 3) / 4), 256>>>(njw, jobs, crow, cval, h, n * 4, wpart, f); }, 50);
  std::printf("k_feat  MODE2    : %8.2f us\n", us);
  const uint64_t nv = n / 4;
  for (unsigned g : {1024u, 2048u, 4096u, 8192u, (unsigned)((nv + 255) / 256)}) {
    us = timeit([&] { k_stream<<<g, 256>>>(nv, (float4 *)h, (float4 *)P, (float4 *)R, (float4 *)Hp, (float4 *)S); }, 50);
    std::printf("stream grid %6u : %8.2f us  %7.1f GB/s\n", g, us, (double)n * 4 * 9 / us / 1e3);
  }
  return 0;
}
