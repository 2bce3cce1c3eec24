// Microbenchmark: the config-5 cross-half Grams (k_gram_mfma64: all C = 39
// Grams M_c = A_c^T B of 2 M rows x 64 fp32 in one launch) in variants of its
// load / MFMA schedule, against the dense f32 MFMA peak (157.3 TF/s).
// Build (from the repo root):
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I one-class-ffm_amd/csrc -o tools/mb/mb_gram64 tools/mb/mb_gram64.hip
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

// U row pairs per register set; SUMS: wave 0 of group 0 also sums B and
// wv*B; PIPE 1: the next set's loads are issued before the current set's
// MFMAs (software pipelined), 0: both sets loaded, then both consumed.
template <int U, bool SUMS, int PIPE, int OCC>
__global__ __launch_bounds__(256, OCC) void k_gram(uint64_t Rp, int C, const float *const *__restrict__ A,
                                                   const float *__restrict__ B, const float *__restrict__ wv,
                                                   float *__restrict__ part, uint64_t nout, uint64_t rows_per_block,
                                                   unsigned ngroups) {
  typedef float f16x __attribute__((ext_vector_type(16)));
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int e = lane & 31, hf = lane >> 5;
  const unsigned grp = blockIdx.x % ngroups, chunk = blockIdx.x / ngroups;
  const int c0 = (int)(grp * 4 + w);
  if (c0 >= C) return;
  const bool sums = SUMS && grp == 0 && w == 0;
  f16x acc[4];
#pragma unroll
  for (int t = 0; t < 4; t++)
#pragma unroll
    for (int r = 0; r < 16; r++) acc[t][r] = 0.0f;
  const BufView ab = buf_view(A[c0], Rp * 256);
  const BufView bb = buf_view(B, Rp * 256), wb = buf_view(wv, wv ? Rp * 4 : 0);
  const uint64_t r0 = (uint64_t)chunk * rows_per_block;
  const uint64_t r1 = r0 + rows_per_block < Rp ? r0 + rows_per_block : Rp;
  float cs[2] = {0, 0}, ws[2] = {0, 0}, wt = 0;
  float bv[2][U][2], av[2][U][2], wvv[2][U];
  auto load = [&](int sb, uint64_t j0) {
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint64_t jj = j0 + 2 * u + hf;
      const bool ok = jj < r1;
      const uint32_t off = ok ? (uint32_t)(jj * 256 + e * 4) : 0xffffff00u;
#pragma unroll
      for (int h = 0; h < 2; h++) {
        bv[sb][u][h] = bld1<float>(bb, off + h * 128);
        av[sb][u][h] = bld1<float>(ab, off + h * 128);
      }
      if (SUMS) wvv[sb][u] = bld1<float>(wb, ok ? (uint32_t)(jj * 4) : 0xffffff00u);
    }
  };
  auto step = [&](int sb) {
#pragma unroll
    for (int u = 0; u < U; u++) {
#pragma unroll
      for (int mt = 0; mt < 2; mt++)
#pragma unroll
        for (int nt = 0; nt < 2; nt++)
          acc[mt * 2 + nt] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[sb][u][mt], bv[sb][u][nt], acc[mt * 2 + nt], 0, 0, 0);
      if (sums) {
#pragma unroll
        for (int h = 0; h < 2; h++) {
          cs[h] += bv[sb][u][h];
          ws[h] += wvv[sb][u] * bv[sb][u][h];
        }
        if (e == 0) wt += wvv[sb][u];
      }
    }
  };
  if (PIPE == 0) {
    for (uint64_t j0 = r0; j0 < r1; j0 += 4 * U) {
      load(0, j0);
      load(1, j0 + 2 * U);
      step(0);
      step(1);
    }
  } else {
    load(0, r0);
    for (uint64_t j0 = r0; j0 < r1; j0 += 4 * U) {
      load(1, j0 + 2 * U);
      step(0);
      load(0, j0 + 4 * U);
      step(1);
    }
  }
  float *out = part + (size_t)chunk * nout;
#pragma unroll
  for (int t = 0; t < 4; t++)
#pragma unroll
    for (int r = 0; r < 16; r++) {
      const int m = (t >> 1) * 32 + 8 * (r >> 2) + 4 * hf + (r & 3), n = (t & 1) * 32 + e;
      out[(size_t)c0 * 4096 + m * 64 + n] = acc[t][r];
    }
  if (sums && hf == 0) {
    for (int h = 0; h < 2; h++) out[(size_t)C * 4096 + h * 32 + e] = cs[h] + ws[h] + wt;
  }
}

// NS register sets in a ring: set s is consumed NS - 1 sets after its loads
// were issued (deeper than PIPE 1), U row pairs per set.
template <int U, int NS, int OCC>
__global__ __launch_bounds__(256, OCC) void k_gram_deep(uint64_t Rp, int C, const float *const *__restrict__ A,
                                                        const float *__restrict__ B, const float *__restrict__ wv,
                                                        float *__restrict__ part, uint64_t nout, uint64_t rows_per_block,
                                                        unsigned ngroups) {
  typedef float f16x __attribute__((ext_vector_type(16)));
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int e = lane & 31, hf = lane >> 5;
  const unsigned grp = blockIdx.x % ngroups, chunk = blockIdx.x / ngroups;
  const int c0 = (int)(grp * 4 + w);
  if (c0 >= C) return;
  f16x acc[4];
#pragma unroll
  for (int t = 0; t < 4; t++)
#pragma unroll
    for (int r = 0; r < 16; r++) acc[t][r] = 0.0f;
  const BufView ab = buf_view(A[c0], Rp * 256);
  const BufView bb = buf_view(B, Rp * 256);
  const uint64_t r0 = (uint64_t)chunk * rows_per_block;
  const uint64_t r1 = r0 + rows_per_block < Rp ? r0 + rows_per_block : Rp;
  float bv[NS][U][2], av[NS][U][2];
  auto load = [&](auto SB, uint64_t j0) {
    constexpr int sb = decltype(SB)::value;
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint64_t jj = j0 + 2 * u + hf;
      const uint32_t off = jj < r1 ? (uint32_t)(jj * 256 + e * 4) : 0xffffff00u;
#pragma unroll
      for (int h = 0; h < 2; h++) {
        bv[sb][u][h] = bld1<float>(bb, off + h * 128);
        av[sb][u][h] = bld1<float>(ab, off + h * 128);
      }
    }
  };
  auto step = [&](auto SB) {
    constexpr int sb = decltype(SB)::value;
#pragma unroll
    for (int u = 0; u < U; u++)
#pragma unroll
      for (int mt = 0; mt < 2; mt++)
#pragma unroll
        for (int nt = 0; nt < 2; nt++)
          acc[mt * 2 + nt] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[sb][u][mt], bv[sb][u][nt], acc[mt * 2 + nt], 0, 0, 0);
  };
  sfor<NS>([&](auto S) { load(S, r0 + decltype(S)::value * 2 * U); });
  for (uint64_t j0 = r0; j0 < r1; j0 += NS * 2 * U) {
    sfor<NS>([&](auto S) {
      step(S);
      load(S, j0 + (decltype(S)::value + NS) * 2 * U);
    });
  }
  float *out = part + (size_t)chunk * nout;
#pragma unroll
  for (int t = 0; t < 4; t++)
#pragma unroll
    for (int r = 0; r < 16; r++) {
      const int m = (t >> 1) * 32 + 8 * (r >> 2) + 4 * hf + (r & 3), n = (t & 1) * 32 + e;
      out[(size_t)c0 * 4096 + m * 64 + n] = acc[t][r];
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
  const uint64_t Rp = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 2000000;
  const int C = 39;
  const unsigned blocks_cap = argc > 2 ? (unsigned)std::atoi(argv[2]) : 1024;
  std::vector<float *> tabs(C);
  for (int c = 0; c < C; c++) {
    CK(hipMalloc(&tabs[c], Rp * 256));
    CK(hipMemset(tabs[c], 0, Rp * 256));
  }
  float *B, *wv, *part;
  CK(hipMalloc(&B, Rp * 256));
  CK(hipMemset(B, 0, Rp * 256));
  CK(hipMalloc(&wv, Rp * 4));
  CK(hipMemset(wv, 0, Rp * 4));
  float **dA;
  CK(hipMalloc(&dA, C * sizeof(float *)));
  CK(hipMemcpy(dA, tabs.data(), C * sizeof(float *), hipMemcpyHostToDevice));
  const unsigned gy = (C + 3) / 4;
  const uint64_t nout = (uint64_t)C * 4096 + 129;
  uint64_t nbx = std::max<uint64_t>(1, std::min<uint64_t>((Rp + 63) / 64, blocks_cap / gy));
  const uint64_t rpb = ((Rp + nbx - 1) / nbx + 15) / 16 * 16;
  nbx = (Rp + rpb - 1) / rpb;
  CK(hipMalloc(&part, nbx * nout * 4));
  const double flops = 2.0 * Rp * C * 64 * 64, bytes = (double)Rp * (C + 1) * 256;
  auto run = [&](const char *name, auto kern) {
    const float us = timeit([&] { hipLaunchKernelGGL(kern, (unsigned)(nbx * gy), 256, 0, 0, Rp, C, (const float *const *)dA,
                                                      B, wv, part, nout, rpb, gy); }, 5);
    std::printf("%-28s %9.1f us  %6.1f TF/s (%.2f of 157.3)  %6.2f TB/s\n", name, us, flops / us / 1e6,
                flops / us / 1e6 / 157.3, bytes / us / 1e6);
  };
  std::printf("Rp %lu, C %d, blocks %lu (%lu chunks x %u groups), rows/block %lu\n", Rp, C, nbx * gy, nbx, gy, rpb);
  run("U4 nosums pipe0 occ3", k_gram<4, false, 0, 3>);
  run("U4 nosums pipe1 occ3", k_gram<4, false, 1, 3>);
  run("deep U4 NS3 occ3", k_gram_deep<4, 3, 3>);
  run("deep U4 NS4 occ3", k_gram_deep<4, 4, 3>);
  run("deep U2 NS4 occ3", k_gram_deep<2, 4, 3>);
  run("deep U2 NS6 occ3", k_gram_deep<2, 6, 3>);
  run("deep U4 NS3 occ2", k_gram_deep<4, 3, 2>);
  run("deep U2 NS4 occ4", k_gram_deep<2, 4, 4>);
  {  // the library kernel (sums on the matrix cores in the spare wave slot)
    const unsigned gy2 = (C + 1 + 3) / 4;
    const unsigned nw = (unsigned)(nbx * gy2), g8 = (nw + 7) / 8 * 8;  // the library's XCD-ordered grid
    const float us = timeit([&] { hipLaunchKernelGGL(k_gram_mfma64, g8, 256, 0, 0, Rp, C,
                                                      (const float *const *)dA, B, wv, part, nout, rpb, gy2, nw); }, 5);
    std::printf("%-28s %9.1f us  %6.1f TF/s (%.2f of 157.3)  %6.2f TB/s\n", "k_gram_mfma64 (library)", us,
                flops / us / 1e6, flops / us / 1e6 / 157.3, bytes / us / 1e6);
  }
  return 0;
}
