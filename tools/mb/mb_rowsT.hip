// Microbenchmark: k_rows_T<64> (config 5: T = sum_c P_c M_c over 39 tables
// of 2 M rows x 64 fp32) against variants with smaller LDS stages / more
// blocks per CU.  Build (repo root):
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I one-class-ffm_amd/csrc -o tools/mb/mb_rowsT tools/mb/mb_rowsT.hip
#include <hip/hip_runtime.h>

#include <cstdio>
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

namespace ocffm {
template <int KP, int TG_, int MINB>
__global__ __launch_bounds__(TBLOCK, MINB) void k_rows_Tv(uint64_t R, int C, const float *const *__restrict__ A,
                                                   const float *__restrict__ M, float *__restrict__ T) {
  using RT = RowsT<KP>;
  constexpr int NT = RT::NT, KH = RT::KH, TW = RT::TW, TG = TG_;
  typedef float f16x __attribute__((ext_vector_type(16)));
  typedef float v2f __attribute__((ext_vector_type(2)));
  __shared__ __align__(16) float Ms[TG * KP * KP];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int e = lane & 31, hf = lane >> 5;
  const uint32_t rowb = KP * 4;
  for (uint64_t base = (uint64_t)blockIdx.x * RT::ROWS; base < R; base += (uint64_t)gridDim.x * RT::ROWS) {
    f16x acc[TW][NT];
#pragma unroll
    for (int t = 0; t < TW; t++)
#pragma unroll
      for (int n = 0; n < NT; n++)
#pragma unroll
        for (int r = 0; r < 16; r++) acc[t][n][r] = 0.0f;
    // rows of this wave's tiles: row (base + (w TW + t) 32 + e); past R: zero (buffer range)
    for (int g0 = 0; g0 < C; g0 += TG) {
      const int ng = C - g0 < TG ? C - g0 : TG;
      __syncthreads();  // the previous stage's readers are done
      {
        // the stage in one round of independent 16-B loads (up to TG KP^2 / 4
        // / TBLOCK per thread), then the permuted LDS stores
        // (in two halves: the staging registers are not live beside the
        // operands' double buffer)
        constexpr int PER = (TG * KP * KP / 4 + TBLOCK - 1) / TBLOCK, PH = PER / 2 > 0 ? PER / 2 : 1;
        const BufView mb = buf_view(M + (size_t)g0 * KP * KP, (uint64_t)ng * KP * KP * 4);
#pragma unroll 1
        for (int u0 = 0; u0 < PER; u0 += PH) {
          f4v mv[PH];
#pragma unroll
          for (int u = 0; u < PH; u++) mv[u] = bld<float>(mb, (uint32_t)(threadIdx.x + (u0 + u) * TBLOCK) * 16u);
#pragma unroll
          for (int u = 0; u < PH; u++) {
            const int q = (threadIdx.x + (u0 + u) * TBLOCK) * 4;
            if (q < ng * KP * KP) {
              const int c = q / (KP * KP), rem = q % (KP * KP), k = rem / KP, col = rem % KP;
#pragma unroll
              for (int x = 0; x < 4; x++)
                Ms[((c * KP + k) * 32 + ((col + x) & 31)) * NT + ((col + x) >> 5)] = mv[u][x];
            }
          }
        }
      }
      __syncthreads();
      f4v a[2][TW][KH / 4];
      auto load = [&](auto SB, int c) {
        constexpr int sb = decltype(SB)::value;
        const BufView ab = buf_view(A[g0 + c], R * rowb);
#pragma unroll
        for (int t = 0; t < TW; t++) {
          const uint64_t row = base + (uint64_t)(w * TW + t) * 32 + e;
          const uint32_t off = row < R ? (uint32_t)(row * rowb + hf * KH * 4) : ab.oob;
#pragma unroll
          for (int q = 0; q < KH / 4; q++) a[sb][t][q] = bld<float>(ab, off + q * 16);
        }
      };
      // table c on register set c % 2 (compile-time: a runtime set index
      // would put the operands in scratch memory)
      auto compute = [&](auto SB, int c) {
        constexpr int sb = decltype(SB)::value;
        const float *mc = Ms + (size_t)c * KP * KP;
#pragma unroll
        for (int s = 0; s < KH; s++) {
          const int k = s + KH * hf;
          if constexpr (NT == 2) {
            const v2f b = *reinterpret_cast<const v2f *>(mc + (k * 32 + e) * 2);
#pragma unroll
            for (int t = 0; t < TW; t++) {
              const float av = a[sb][t][s >> 2][s & 3];
              acc[t][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, b[0], acc[t][0], 0, 0, 0);
              acc[t][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, b[1], acc[t][1], 0, 0, 0);
            }
          } else {
            const float b = mc[k * 32 + e];
#pragma unroll
            for (int t = 0; t < TW; t++)
              acc[t][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[sb][t][s >> 2][s & 3], b, acc[t][0], 0, 0, 0);
          }
        }
      };
      load(std::integral_constant<int, 0>(), 0);
      for (int c = 0; c < ng; c += 2) {
        if (c + 1 < ng) load(std::integral_constant<int, 1>(), c + 1);
        compute(std::integral_constant<int, 0>(), c);
        if (c + 1 >= ng) break;
        if (c + 2 < ng) load(std::integral_constant<int, 0>(), c + 2);
        compute(std::integral_constant<int, 1>(), c + 1);
      }
    }
    // D register r of lane l: row 8(r/4) + 4(l/32) + r%4 of the tile, column l%32 (+32 n)
#pragma unroll
    for (int t = 0; t < TW; t++)
#pragma unroll
      for (int n = 0; n < NT; n++)
#pragma unroll
        for (int r = 0; r < 16; r++) {
          const uint64_t m = base + (uint64_t)(w * TW + t) * 32 + 8 * (r >> 2) + 4 * hf + (r & 3);
          if (m < R) T[m * KP + n * 32 + e] = acc[t][n][r];
        }
  }
}

}  // namespace ocffm

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
  const uint64_t R = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 2000000;
  const int C = 39, KP = 64;
  std::vector<float *> tabs(C);
  for (int c = 0; c < C; c++) {
    CK(hipMalloc(&tabs[c], R * KP * 4));
    CK(hipMemset(tabs[c], 0, R * KP * 4));
  }
  float *M, *T;
  CK(hipMalloc(&M, (size_t)C * KP * KP * 4));
  CK(hipMemset(M, 0, (size_t)C * KP * KP * 4));
  CK(hipMalloc(&T, R * KP * 4));
  float **dA;
  CK(hipMalloc(&dA, C * sizeof(float *)));
  CK(hipMemcpy(dA, tabs.data(), C * sizeof(float *), hipMemcpyHostToDevice));
  const double flops = 2.0 * R * C * KP * KP, bytes = (double)R * (C + 1) * KP * 4;
  const uint64_t nb = (R + RowsT<64>::ROWS - 1) / RowsT<64>::ROWS;
  auto report = [&](const char *name, float us) {
    std::printf("%-34s %9.1f us  %6.1f TF/s (%.2f of 157.3)  %6.2f TB/s\n", name, us, flops / us / 1e6,
                flops / us / 1e6 / 157.3, bytes / us / 1e6);
  };
  for (unsigned g : {256u, 512u, 1024u}) {
    const unsigned grid = (unsigned)std::min<uint64_t>(nb, g);
    char name[64];
    std::snprintf(name, sizeof(name), "library TG8 grid %u", grid);
    report(name, timeit([&] { hipLaunchKernelGGL(k_rows_T<64>, grid, TBLOCK, 0, 0, R, C, (const float *const *)dA, M, T); }, 3));
    std::snprintf(name, sizeof(name), "TG4 minb2 grid %u", grid);
    report(name, timeit([&] { hipLaunchKernelGGL((k_rows_Tv<64, 4, 2>), grid, TBLOCK, 0, 0, R, C, (const float *const *)dA, M, T); }, 3));
    std::snprintf(name, sizeof(name), "TG4 minb1 grid %u", grid);
    report(name, timeit([&] { hipLaunchKernelGGL((k_rows_Tv<64, 4, 1>), grid, TBLOCK, 0, 0, R, C, (const float *const *)dA, M, T); }, 3));
    std::snprintf(name, sizeof(name), "TG2 minb2 grid %u", grid);
    report(name, timeit([&] { hipLaunchKernelGGL((k_rows_Tv<64, 2, 2>), grid, TBLOCK, 0, 0, R, C, (const float *const *)dA, M, T); }, 3));
  }
  return 0;
}
