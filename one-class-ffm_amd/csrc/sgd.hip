// sgd.hip — field-aware FM trained by per-instance SGD / AdaGrad with
// HOGWILD writes and on-device negative sampling.
//
// BASELINE.json's north_star names this mode: the pairwise interaction
// phi(x) = sum_{a<b} <w[j_a][f_b], w[j_b][f_a]> x_a x_b with its SGD/AdaGrad
// step as HIP kernels, lock-free writes to W, negatives drawn on the device
// from an alias table, and model averaging over ranks with RCCL.  The
// reference (johncreed/one-class-ffm) has no such path — its solver is the
// block Newton-CG of ffm.cpp — so parity is pinned against
// oracle/sgd_oracle.cpp (a serial CPU statement of the same algorithm, whose
// header states it), not against the reference.
//
// Instances: every training positive (user i, item j) is an instance with
// label +1 and draws `nneg` negatives (user i, item ~ alias) with label -1.
// An instance's nodes are the user row's feature nodes followed by the item
// row's (global feature id = field offset + idx, fields 0..fu-1 then
// fu..fu+fv-1).  W and the AdaGrad sums G are NF x F x KP fp32 (KP = next
// power of two >= k, padding zero): the row w[j][f] is 16 B per lane over an
// LPR-lane subgroup, as in kernels.hpp.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <memory>
#include <type_traits>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/ocffm.h"
#include "common.hpp"
#include "host_data.h"
#include "kernels.hpp"

namespace ocffm {
namespace sgd {

constexpr int NMAX = 64;  // nodes per instance: one per lane
constexpr int SPG_MAX = 8;  // slots per subgroup held in registers (slots <= SPG * NSG); the
                            // launch picks the smallest of 2, 4, 8 that covers the widest instance

__host__ __device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

struct Args {
  uint64_t T, n_items;  // instances this epoch, item rows
  uint32_t nneg, F;
  const uint32_t *pu, *pv;  // positives (user row, item row)
  const float *prob;
  const uint32_t *alias;
  const uint64_t *uptr, *vptr;
  const uint32_t *unode, *ufld, *vnode, *vfld;
  const float *uval, *vval;
  float *W, *G;
  float eta, lam;
  int adagrad, norm;
  uint64_t seed, epoch, A, B;  // instance order qq = (A q + B) mod T
  double *loss;                // summed log-loss (one atomic per wave)
};

// Item of instance qq and its label: the positive's item, or an alias draw.
__device__ __forceinline__ uint32_t draw_item(const Args &d, uint64_t qq, uint64_t p, uint64_t r, float &y) {
  if (r == 0) {
    y = 1.0f;
    return d.pv[p];
  }
  y = -1.0f;
  const uint64_t h = mix64(d.seed + 0x9E3779B97F4A7C15ULL * (d.epoch * d.T + qq));
  const uint32_t idx = (uint32_t)(h >> 32) % (uint32_t)d.n_items;  // n_items < 2^32
  const float coin = (float)(uint32_t)(h & 0xffffffu) * (1.0f / 16777216.0f);
  return coin < d.prob[idx] ? (uint32_t)idx : d.alias[idx];
}

// Nodes of one instance, lane l < n holding node l (user row, then item row).
struct Nodes {
  uint32_t j, f;
  float x;
  int n;
};
__device__ __forceinline__ Nodes load_nodes(const Args &d, uint32_t u, uint32_t it, int lane) {
  const uint64_t ub = d.uptr[u], vb = d.vptr[it];
  const int nu = (int)(d.uptr[u + 1] - ub);
  Nodes o{0u, 0xffffffffu, 0.0f, nu + (int)(d.vptr[it + 1] - vb)};
  if (lane < nu) {
    o.j = d.unode[ub + lane];
    o.f = d.ufld[ub + lane];
    o.x = d.uval[ub + lane];
  } else if (lane < o.n) {
    o.j = d.vnode[vb + lane - nu];
    o.f = d.vfld[vb + lane - nu];
    o.x = d.vval[vb + lane - nu];
  }
  return o;
}

// One wave per instance (grid-stride).  Slot (a, f) = row w[j_a][f] of node
// a for field f; it takes part iff another node b != a sits in field f.  The
// wave's subgroups load their slots' W rows (and AdaGrad rows) in one round
// into registers and stage the W rows in this wave's LDS region; the
// forward pass (pair (a, b) = <slot(a, f_b), slot(b, f_a)>) and every slot's
// gradient sum_{b != a, f_b = f} x_b slot(b, f_a) then read LDS only, and the
// steps are stored (plain stores: HOGWILD).  LDS per wave: SMAX rows.
template <int KP, int SPG, int OCC>
__global__ __launch_bounds__(256, OCC) void k_sgd(Args d, int smax) {
  using Gm = Geo<float, KP>;
  constexpr int LPR = Gm::LPR, NG = Gm::NSG;
  extern __shared__ __align__(16) unsigned char smem_raw[];
  const int lane = threadIdx.x & 63, g = lane / LPR, li = lane % LPR;
  float *sl = reinterpret_cast<float *>(smem_raw) + (size_t)(threadIdx.x >> 6) * smax * KP;
  const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint64_t nwaves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
  const uint32_t F = d.F;
  double lsum = 0;
  // qq = (A q + B) mod T stepped incrementally over this wave's q (one
  // 64-bit modulo per wave, not per instance)
  const uint64_t step = (d.A * (nwaves % d.T)) % d.T;
  uint64_t qq = (d.A * (wave % d.T) + d.B) % d.T;
  const uint32_t m1 = 1 + d.nneg;
  for (uint64_t q = wave; q < d.T; q += nwaves) {
    uint64_t p, r;
    if (d.T < (1ull << 32)) {
      const uint32_t q32 = (uint32_t)qq, p32 = q32 / m1;
      p = p32;
      r = q32 - p32 * m1;
    } else {
      p = qq / m1;
      r = qq - p * m1;
    }
    float y;
    const uint32_t it = draw_item(d, qq, p, r, y);
    qq += step;
    if (qq >= d.T) qq -= d.T;
    const Nodes nd = load_nodes(d, d.pu[p], it, lane);
    const int n = nd.n, S = n * (int)F;
    // field populations (F <= 64): count of nodes per field, per lane f
    int fcnt = 0;
    for (int b = 0; b < n; b++) fcnt += (__builtin_amdgcn_readlane((int)nd.f, b) == lane) ? 1 : 0;
    float rn = 1.0f;
    if (d.norm) {
      float s2 = nd.x * nd.x;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) s2 += __shfl_xor(s2, o, 64);
      rn = s2 > 0 ? 1.0f / s2 : 1.0f;
    }
    // slot rows: one round of loads, W staged in LDS
    // (lane moves of node data happen here, with every lane active: a
    // ds_bpermute from a lane outside EXEC does not return its value)
    f4v gr[SPG];
    bool act[SPG];
    uint32_t sja[SPG], sfa[SPG];
    float sxa[SPG];
    {
      f4v wr[SPG];
#pragma unroll
      for (int t = 0; t < SPG; t++) {
        const int s = g + t * NG;
        const int a = min(s / (int)F, 63);
        const int fl = s % (int)F;
        sja[t] = __shfl(nd.j, a, 64);
        sfa[t] = __shfl(nd.f, a, 64);
        sxa[t] = __shfl(nd.x, a, 64);
        const int c = __shfl(fcnt, fl, 64) - (sfa[t] == (uint32_t)fl ? 1 : 0);
        act[t] = s < S && c > 0;
        if (act[t]) wr[t] = vld<float>(d.W + ((size_t)sja[t] * F + fl) * KP + li * 4);
      }
#pragma unroll
      for (int t = 0; t < SPG; t++)
        if (act[t]) {
          vst<float>(sl + (size_t)(g + t * NG) * KP + li * 4, wr[t]);
          if (d.adagrad) gr[t] = vld<float>(d.G + ((size_t)sja[t] * F + (g + t * NG) % (int)F) * KP + li * 4);
        }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    // forward over the pairs, from LDS
    const int npairs = n * (n - 1) / 2;
    float acc = 0;
    for (int base = 0; base < npairs; base += NG) {
      const int pq = min(base + g, npairs - 1);
      int a = 0, rem = pq;
      while (rem >= n - 1 - a) {
        rem -= n - 1 - a;
        a++;
      }
      const int b = a + 1 + rem;
      const uint32_t fa = __shfl(nd.f, a, 64), fb = __shfl(nd.f, b, 64);
      const float xab = __shfl(nd.x, a, 64) * __shfl(nd.x, b, 64);
      if (base + g < npairs) {
        const f4v wa = vld<float>(sl + ((size_t)a * F + fb) * KP + li * 4);
        const f4v wb = vld<float>(sl + ((size_t)b * F + fa) * KP + li * 4);
        acc += sg_sum<LPR>(hsum<float>(wa * wb)) * xab;
      }
    }
    const float phi = xsg_sum<LPR>(acc) * rn;
    const float ex = expf(-y * phi);
    const float kappa = -y * ex / (1.0f + ex);
    if (lane == 0) lsum += log1p((double)ex);
    // slot steps
#pragma unroll
    for (int t = 0; t < SPG; t++) {
      if (!act[t]) continue;
      const int s = g + t * NG;
      const int a = s / (int)F;
      const uint32_t fl = (uint32_t)(s % (int)F);
      const uint32_t ja = sja[t], fa = sfa[t];
      const float xa = sxa[t];
      f4v sacc = vzero<float>();
      for (int b = 0; b < n; b++) {  // wave-uniform trip count
        const uint32_t fb = (uint32_t)__builtin_amdgcn_readlane((int)nd.f, b);
        const float xb = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, nd.x), b));
        if (b != a && fb == fl) sacc += vsplat<float>(xb) * vld<float>(sl + ((size_t)b * F + fa) * KP + li * 4);
      }
      const size_t off = ((size_t)ja * F + fl) * KP + li * 4;
      const f4v w = vld<float>(sl + (size_t)s * KP + li * 4);
      const f4v gd = vsplat<float>(d.lam) * w + vsplat<float>(kappa * rn * xa) * sacc;
      if (d.adagrad) {
        const f4v gv = gr[t] + gd * gd;
        f4v st;
#pragma unroll
        for (int e = 0; e < 4; e++) st[e] = d.eta * gd[e] * __builtin_amdgcn_rsqf(gv[e]);  // 1-ulp rsq
        vst<float>(d.W + off, w - st);
        vst<float>(d.G + off, gv);
      } else {
        vst<float>(d.W + off, w - vsplat<float>(d.eta) * gd);
      }
    }
    __builtin_amdgcn_wave_barrier();  // LDS reads of this instance before the next one's writes
  }
  if (lane == 0 && lsum != 0) atomicAdd(d.loss, lsum);
}

// phi of given (user, item) pairs with the current W (evaluation / tests).
template <int KP>
__global__ __launch_bounds__(256) void k_phi(Args d, uint64_t npairs_in, const uint32_t *users,
                                             const uint32_t *items, float *out) {
  using Gm = Geo<float, KP>;
  constexpr int LPR = Gm::LPR, NG = Gm::NSG;
  const int lane = threadIdx.x & 63, g = lane / LPR, li = lane % LPR;
  const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint64_t nwaves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
  const uint32_t F = d.F;
  for (uint64_t q = wave; q < npairs_in; q += nwaves) {
    const uint32_t u = users[q], it = items[q];
    const uint64_t ub = d.uptr[u], vb = d.vptr[it];
    const int nu = (int)(d.uptr[u + 1] - ub), n = nu + (int)(d.vptr[it + 1] - vb);
    uint32_t nj = 0, nf = 0xffffffffu;
    float nx = 0;
    if (lane < nu) {
      nj = d.unode[ub + lane];
      nf = d.ufld[ub + lane];
      nx = d.uval[ub + lane];
    } else if (lane < n) {
      nj = d.vnode[vb + lane - nu];
      nf = d.vfld[vb + lane - nu];
      nx = d.vval[vb + lane - nu];
    }
    float rn = 1.0f;
    if (d.norm) {
      float s = nx * nx;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
      rn = s > 0 ? 1.0f / s : 1.0f;
    }
    const int npairs = n * (n - 1) / 2;
    float acc = 0;
    for (int base = 0; base < npairs; base += NG) {
      const int pq = min(base + g, npairs - 1);
      int a = 0, rem = pq;
      while (rem >= n - 1 - a) {
        rem -= n - 1 - a;
        a++;
      }
      const int b = a + 1 + rem;
      const uint32_t ja = __shfl(nj, a, 64), fa = __shfl(nf, a, 64), jb = __shfl(nj, b, 64), fb = __shfl(nf, b, 64);
      const float xab = __shfl(nx, a, 64) * __shfl(nx, b, 64);
      if (base + g < npairs) {
        const f4v wa = vld<float>(d.W + ((size_t)ja * F + fb) * KP + li * 4);
        const f4v wb = vld<float>(d.W + ((size_t)jb * F + fa) * KP + li * 4);
        acc += sg_sum<LPR>(hsum<float>(wa * wb)) * xab;
      }
    }
    const float phi = xsg_sum<LPR>(acc) * rn;
    if (lane == 0) out[q] = phi;
  }
}

// W (and G) /= ranks after the all-reduce (model averaging).
__global__ void k_scale(uint64_t n, float *x, float s) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    x[i] *= s;
}

}  // namespace sgd
}  // namespace ocffm

namespace ocffm {
namespace sgd {

// ---------------------------------------------------------------- host
class Trainer {
 public:
  Trainer(const HostData &U, const HostData &V, const ocffm_sgd_param &prm, int rank, int nranks, const void *cid,
          ocffm_allreduce_fn host_fn = nullptr, void *host_user = nullptr)
      : prm_(prm), rank_(rank), nranks_(nranks), host_fn_(host_fn), host_user_(host_user) {
    if (prm.k == 0 || prm.k > 128) throw Error(OCFFM_E_ARG, "k must be in 1..128");
    if (nranks < 1 || rank < 0 || rank >= nranks) throw Error(OCFFM_E_ARG, "bad rank / nranks");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
      throw Error(OCFFM_E_HIP, "no HIP device visible (this build has no CPU fallback)");
    HIPCHK(hipSetDevice(prm.device));
    HIPCHK(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
    kp_ = 4;
    while (kp_ < prm.k) kp_ *= 2;
    fu_ = (uint32_t)U.f;
    fv_ = (uint32_t)V.f;
    F_ = fu_ + fv_;
    if (F_ == 0) throw Error(OCFFM_E_DATA, "no fields");
    // global feature ids: user fields, then item fields
    std::vector<uint64_t> off(F_ + 1, 0);
    for (uint32_t f = 0; f < F_; f++) off[f + 1] = off[f] + (f < fu_ ? U.Ds[f] : V.Ds[f - fu_]);
    nf_ = off[F_];
    if (nf_ >= (1ull << 32)) throw Error(OCFFM_E_DATA, "more than 2^32 features");
    int umax = 0, vmax = 0;
    build_nodes(U, 0, off, uptr_, unode_, ufld_, uval_, umax);
    build_nodes(V, fu_, off, vptr_, vnode_, vfld_, vval_, vmax);
    const int nmax = umax + vmax;
    const int ng = 64 / std::max<int>(1, (int)(kp_ / 4));
    smax_ = std::max(1, nmax * (int)F_);
    if (F_ > 64) throw Error(OCFFM_E_ARG, "more than 64 fields in the SGD mode");
    if (nmax > NMAX || (uint64_t)nmax * F_ > (uint64_t)SPG_MAX * ng)
      throw Error(OCFFM_E_ARG, "instances too wide for the SGD kernel (nodes " + std::to_string(nmax) + " x fields " +
                                   std::to_string(F_) + " > " + std::to_string(SPG_MAX * ng) + " slots at this k)");
    spg_ = 2;
    while ((uint64_t)nmax * F_ > (uint64_t)spg_ * ng) spg_ *= 2;
    // positives of this rank's user shard
    for (uint64_t j : U.ycol)
      if (j >= V.m) throw Error(OCFFM_E_DATA, "train label >= number of item rows");
    const uint64_t u0 = U.m * (uint64_t)rank / nranks, u1 = U.m * (uint64_t)(rank + 1) / nranks;
    std::vector<uint32_t> pu, pv;
    for (uint64_t i = u0; i < u1; i++)
      for (uint64_t p = U.yptr[i]; p < U.yptr[i + 1]; p++) {
        pu.push_back((uint32_t)i);
        pv.push_back((uint32_t)U.ycol[p]);
      }
    P_ = pu.size();
    n_items_ = V.m;
    T_ = P_ * (1 + (uint64_t)prm.nneg);
    if (T_ >= (1ull << 40)) throw Error(OCFFM_E_ARG, "too many instances per epoch for one rank (2^40)");
    pu_.upload(pu);
    pv_.upload(pv);
    // alias table over item popularity^neg_power (all users' labels)
    std::vector<double> w(std::max<uint64_t>(V.m, 1), 0.0);
    for (uint64_t j : U.ycol) w[j] += 1.0;
    for (double &x : w) x = x > 0 ? std::pow(x, prm.neg_power) : 0.0;
    std::vector<float> prob(w.size(), 1.0f);
    std::vector<uint32_t> alias(w.size());
    build_alias(w, prob, alias);
    h_prob_ = prob;
    h_alias_ = alias;
    prob_.upload(prob);
    alias_.upload(alias);
    // W ~ U(0, 1/sqrt(k)) from a counter hash (libffm's init range), G = 1
    const size_t nw = (size_t)nf_ * F_ * kp_;
    std::vector<float> W(nw, 0.0f), G(nw, 1.0f);
    const float coef = 1.0f / std::sqrt((float)prm.k);
    for (size_t r = 0; r < (size_t)nf_ * F_; r++)
      for (uint32_t e = 0; e < prm.k; e++) {
        const uint64_t h = mix64(prm.seed * 0x2545F4914F6CDD1DULL + r * 131 + e);
        W[r * kp_ + e] = coef * ((float)(uint32_t)(h >> 40) * (1.0f / 16777216.0f));
      }
    W_.upload(W);
    G_.upload(G);
    loss_.alloc(1);
    if (cid && !host_fn_) {  // a one-rank communicator too (tests of the RCCL path)
      ncclUniqueId id;
      std::memcpy(&id, cid, sizeof(id));
      NCCLCHK(ncclCommInitRank(&nccl_, nranks, id, rank));
    }
  }
  ~Trainer() {
    if (nccl_) ncclCommDestroy(nccl_);
    if (stream_) (void)hipStreamDestroy(stream_);
  }

  // One pass over this rank's instances; returns the mean log-loss.
  double epoch() {
    Args a = args();
    a.epoch = epoch_;
    // instance order: qq = (A q + B) mod T with A coprime to T and A T < 2^64
    static const uint64_t primes[] = {1000003ull, 999983ull, 1000033ull, 999979ull, 1000037ull, 999961ull};
    a.A = 1;
    for (uint64_t c = 0; c < 6; c++) {
      const uint64_t cand = primes[(epoch_ + c) % 6];
      if (T_ % cand != 0 && cand < T_) {
        a.A = cand;
        break;
      }
    }
    a.B = T_ ? mix64(prm_.seed ^ (epoch_ * 0xD1B54A32D192ED03ULL)) % T_ : 0;
    last_A_ = a.A;
    last_B_ = a.B;
    HIPCHK(hipMemsetAsync(loss_.p, 0, sizeof(double), stream_));
    if (T_) {
      unsigned grid, block;
      if (prm_.serial) {
        grid = 1;
        block = 64;
      } else {
        block = 256;
        grid = (unsigned)std::min<uint64_t>((T_ + 3) / 4, grid_cap_);
      }
      const int smax = smax_;
      launch_kp([&](auto K) {
        constexpr int KPc = decltype(K)::value;
        const size_t smem = (size_t)(block / 64) * smax * KPc * sizeof(float);
        // occupancy bound: 4 waves/SIMD (a few VGPRs spill) or the compiler's choice (3 at k=32)
        if (occ4_) {
          if (spg_ == 2) hipLaunchKernelGGL((k_sgd<KPc, 2, 4>), grid, block, smem, stream_, a, smax);
          else if (spg_ == 4) hipLaunchKernelGGL((k_sgd<KPc, 4, 4>), grid, block, smem, stream_, a, smax);
          else hipLaunchKernelGGL((k_sgd<KPc, 8, 4>), grid, block, smem, stream_, a, smax);
        } else {
          if (spg_ == 2) hipLaunchKernelGGL((k_sgd<KPc, 2, 1>), grid, block, smem, stream_, a, smax);
          else if (spg_ == 4) hipLaunchKernelGGL((k_sgd<KPc, 4, 1>), grid, block, smem, stream_, a, smax);
          else hipLaunchKernelGGL((k_sgd<KPc, 8, 1>), grid, block, smem, stream_, a, smax);
        }
      });
      HIPCHK(hipGetLastError());
    }
    double loss = 0;
    HIPCHK(hipMemcpyAsync(&loss, loss_.p, sizeof(double), hipMemcpyDeviceToHost, stream_));
    HIPCHK(hipStreamSynchronize(stream_));
    epoch_++;
    return T_ ? loss / (double)T_ : 0.0;
  }

  // Model averaging over the ranks: W, G <- mean over ranks (RCCL).
  // With a host hook (tests on one GPU) the sums go through host memory.
  void average() {
    if (!nccl_ && !host_fn_) return;
    const size_t nw = (size_t)nf_ * F_ * kp_;
    if (host_fn_) {
      std::vector<float> hb(nw);
      for (float *dp : {W_.p, G_.p}) {
        HIPCHK(hipMemcpyAsync(hb.data(), dp, nw * sizeof(float), hipMemcpyDeviceToHost, stream_));
        HIPCHK(hipStreamSynchronize(stream_));
        if (host_fn_(hb.data(), nw, 0, host_user_) != 0) throw Error(OCFFM_E_HIP, "host all-reduce failed");
        HIPCHK(hipMemcpyAsync(dp, hb.data(), nw * sizeof(float), hipMemcpyHostToDevice, stream_));
      }
    } else {
      NCCLCHK(ncclAllReduce(W_.p, W_.p, nw, ncclFloat, ncclSum, nccl_, stream_));
      NCCLCHK(ncclAllReduce(G_.p, G_.p, nw, ncclFloat, ncclSum, nccl_, stream_));
    }
    const float s = 1.0f / (float)nranks_;
    hipLaunchKernelGGL(k_scale, 2048, 256, 0, stream_, (uint64_t)nw, W_.p, s);
    hipLaunchKernelGGL(k_scale, 2048, 256, 0, stream_, (uint64_t)nw, G_.p, s);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(stream_));
  }

  void phi(uint64_t n, const uint32_t *users, const uint32_t *items, float *out) {
    if (n == 0) return;
    for (uint64_t i = 0; i < n; i++)
      if (users[i] + 1 >= h_uptr_size_ || items[i] + 1 >= h_vptr_size_) throw Error(OCFFM_E_ARG, "row out of range");
    DevBuf<uint32_t> du, dv;
    DevBuf<float> dz;
    du.upload(users, n);
    dv.upload(items, n);
    dz.alloc(n, false);
    Args a = args();
    const unsigned grid = (unsigned)std::min<uint64_t>((n + 3) / 4, 2048);
    launch_kp([&](auto K) {
      hipLaunchKernelGGL(k_phi<decltype(K)::value>, grid, 256, 0, stream_, a, n, du.p, dv.p, dz.p);
    });
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(out, dz.p, n * sizeof(float), hipMemcpyDeviceToHost, stream_));
    HIPCHK(hipStreamSynchronize(stream_));
  }

  uint64_t get(char what, void *out, uint64_t cap) {
    HIPCHK(hipStreamSynchronize(stream_));
    const size_t nw = (size_t)nf_ * F_ * kp_;
    switch (what) {
      case 'W': case 'G': {
        if (out && cap) HIPCHK(hipMemcpy(out, (what == 'W' ? W_ : G_).p, std::min<uint64_t>(cap, nw) * 4, hipMemcpyDeviceToHost));
        return nw;
      }
      case 'p':
        if (out && cap) std::memcpy(out, h_prob_.data(), std::min<uint64_t>(cap, h_prob_.size()) * 4);
        return h_prob_.size();
      case 'a':
        if (out && cap) std::memcpy(out, h_alias_.data(), std::min<uint64_t>(cap, h_alias_.size()) * 4);
        return h_alias_.size();
      case 'o': {  // instance order of the last epoch: A, B, T
        if (out && cap >= 3) {
          uint64_t *o = (uint64_t *)out;
          o[0] = last_A_;
          o[1] = last_B_;
          o[2] = T_;
        }
        return 3;
      }
      default: throw Error(OCFFM_E_ARG, "unknown SGD state name");
    }
  }
  void set_w(const float *w, uint64_t n) {
    if (n != (uint64_t)nf_ * F_ * kp_) throw Error(OCFFM_E_ARG, "size mismatch");
    HIPCHK(hipMemcpy(W_.p, w, n * 4, hipMemcpyHostToDevice));
  }
  void info(ocffm_sgd_info *o) const {
    o->n_features = nf_;
    o->n_fields = F_;
    o->kp = kp_;
    o->positives = P_;
    o->instances = T_;
  }
  void sync() { HIPCHK(hipStreamSynchronize(stream_)); }

 private:
  template <class L> void launch_kp(L &&l) {
    switch (kp_) {
      case 4: l(std::integral_constant<int, 4>{}); break;
      case 8: l(std::integral_constant<int, 8>{}); break;
      case 16: l(std::integral_constant<int, 16>{}); break;
      case 32: l(std::integral_constant<int, 32>{}); break;
      case 64: l(std::integral_constant<int, 64>{}); break;
      default: l(std::integral_constant<int, 128>{}); break;
    }
  }
  Args args() {
    Args a{};
    a.T = T_;
    a.n_items = n_items_;
    a.nneg = prm_.nneg;
    a.F = F_;
    a.pu = pu_.p;
    a.pv = pv_.p;
    a.prob = prob_.p;
    a.alias = alias_.p;
    a.uptr = uptr_.p;
    a.vptr = vptr_.p;
    a.unode = unode_.p;
    a.ufld = ufld_.p;
    a.vnode = vnode_.p;
    a.vfld = vfld_.p;
    a.uval = uval_.p;
    a.vval = vval_.p;
    a.W = W_.p;
    a.G = G_.p;
    a.eta = prm_.eta;
    a.lam = prm_.lambda;
    a.adagrad = prm_.adagrad;
    a.norm = prm_.norm;
    a.seed = prm_.seed;
    a.epoch = epoch_;
    a.loss = loss_.p;
    return a;
  }
  // Row node lists (field-major within a row, file order within a field).
  void build_nodes(const HostData &Draw, uint32_t fbase, const std::vector<uint64_t> &off, DevBuf<uint64_t> &ptr,
                   DevBuf<uint32_t> &node, DevBuf<uint32_t> &fld, DevBuf<float> &val, int &nmax) {
    const HostData &D = split_host(Draw);
    std::vector<uint64_t> p(D.m + 1, 0);
    std::vector<uint32_t> nd, fd;
    std::vector<float> vl;
    nmax = 0;
    for (uint64_t i = 0; i < D.m; i++) {
      for (uint64_t f = 0; f < D.f; f++)
        for (int64_t t = D.xptr[f][i]; t < D.xptr[f][i + 1]; t++) {
          nd.push_back((uint32_t)(off[fbase + f] + D.xidx[f][t]));
          fd.push_back((uint32_t)(fbase + f));
          vl.push_back((float)D.xval[f][t]);
        }
      p[i + 1] = nd.size();
      nmax = std::max<int>(nmax, (int)(p[i + 1] - p[i]));
    }
    (fbase == 0 ? h_uptr_size_ : h_vptr_size_) = p.size();
    ptr.upload(p);
    node.upload(nd.empty() ? std::vector<uint32_t>{0} : nd);
    fld.upload(fd.empty() ? std::vector<uint32_t>{0} : fd);
    val.upload(vl.empty() ? std::vector<float>{0} : vl);
  }
  // Vose's alias method (the oracle states the same construction).
  static void build_alias(const std::vector<double> &w, std::vector<float> &prob, std::vector<uint32_t> &alias) {
    const uint64_t n = w.size();
    double tot = 0;
    for (double x : w) tot += x;
    std::vector<double> p(n);
    std::vector<uint64_t> small, large;
    for (uint64_t i = 0; i < n; i++) {
      p[i] = tot > 0 ? w[i] * (double)n / tot : 1.0;
      (p[i] < 1.0 ? small : large).push_back(i);
    }
    for (uint64_t i = 0; i < n; i++) alias[i] = (uint32_t)i;
    while (!small.empty() && !large.empty()) {
      const uint64_t sm = small.back(), lg = large.back();
      small.pop_back();
      large.pop_back();
      prob[sm] = (float)p[sm];
      alias[sm] = (uint32_t)lg;
      p[lg] = (p[lg] + p[sm]) - 1.0;
      (p[lg] < 1.0 ? small : large).push_back(lg);
    }
    for (uint64_t i : large) prob[i] = 1.0f;
    for (uint64_t i : small) prob[i] = 1.0f;
  }

  ocffm_sgd_param prm_;
  int rank_, nranks_;
  ocffm_allreduce_fn host_fn_ = nullptr;
  void *host_user_ = nullptr;
  hipStream_t stream_ = nullptr;
  ncclComm_t nccl_ = nullptr;
  uint32_t kp_ = 4, fu_ = 0, fv_ = 0, F_ = 0;
  int smax_ = 1;  // slot rows per wave in LDS: max nodes x fields
  int spg_ = 2;   // slots per subgroup of the k_sgd instantiation
  // blocks per epoch launch (grid-stride over the instances); OCFFM_SGD_GRID overrides.
  // Measured at kkbox shape, k=32 (tools/sgd_grid.sh, M instances/s): 512: 236, 1024: 395,
  // 2048: 398, 8192: 406, 32768: 411, 131072: 403, one block per 4 instances: 82
  uint64_t grid_cap_ = std::getenv("OCFFM_SGD_GRID") ? std::max<uint64_t>(1, std::strtoull(std::getenv("OCFFM_SGD_GRID"), nullptr, 10)) : 32768;
  bool occ4_ = std::getenv("OCFFM_SGD_OCC") == nullptr || std::atoi(std::getenv("OCFFM_SGD_OCC")) != 0;
  uint64_t nf_ = 0, P_ = 0, T_ = 0, n_items_ = 0, epoch_ = 0, last_A_ = 1, last_B_ = 0;
  uint64_t h_uptr_size_ = 0, h_vptr_size_ = 0;
  DevBuf<uint64_t> uptr_, vptr_;
  DevBuf<uint32_t> unode_, ufld_, vnode_, vfld_, pu_, pv_, alias_;
  DevBuf<float> uval_, vval_, prob_, W_, G_;
  DevBuf<double> loss_;
  std::vector<float> h_prob_;
  std::vector<uint32_t> h_alias_;
};

}  // namespace sgd
}  // namespace ocffm

// ====================================================================== ABI
struct ocffm_sgd {
  std::unique_ptr<ocffm::sgd::Trainer> t;
};

extern "C" {

void ocffm_sgd_param_default(ocffm_sgd_param *p) {
  p->k = 4;
  p->eta = 0.2f;      // libffm's defaults
  p->lambda = 2e-5f;
  p->nneg = 1;
  p->neg_power = 1.0;
  p->adagrad = 1;
  p->norm = 1;
  p->serial = 0;
  p->seed = 1;
  p->device = 0;
}

static int sgd_create(const ocffm_data *U, const ocffm_data *V, const ocffm_sgd_param *p, int rank, int nranks,
                      const void *cid, ocffm_sgd **out, ocffm_allreduce_fn fn = nullptr, void *user = nullptr) {
  return guarded([&] {
    if (!U || !V || !p || !out) throw ocffm::Error(OCFFM_E_ARG, "null argument");
    if (!U->d.has_label) throw ocffm::Error(OCFFM_E_ARG, "training data without labels");
    auto s = std::make_unique<ocffm_sgd>();
    s->t = std::make_unique<ocffm::sgd::Trainer>(U->d, V->d, *p, rank, nranks, cid, fn, user);
    *out = s.release();
  });
}

int ocffm_sgd_create(const ocffm_data *U, const ocffm_data *V, const ocffm_sgd_param *p, ocffm_sgd **out) {
  return sgd_create(U, V, p, 0, 1, nullptr, out);
}
int ocffm_sgd_create_dist(const ocffm_data *U, const ocffm_data *V, const ocffm_sgd_param *p, int rank, int nranks,
                          const void *comm_id, ocffm_sgd **out) {
  if (!comm_id && nranks > 1) return guarded([] { throw ocffm::Error(OCFFM_E_ARG, "comm_id required"); });
  return sgd_create(U, V, p, rank, nranks, comm_id, out);
}

int ocffm_sgd_create_dist_host(const ocffm_data *U, const ocffm_data *V, const ocffm_sgd_param *p, int rank,
                               int nranks, ocffm_allreduce_fn fn, void *user, ocffm_sgd **out) {
  if (!fn) return guarded([] { throw ocffm::Error(OCFFM_E_ARG, "all-reduce hook required"); });
  return sgd_create(U, V, p, rank, nranks, nullptr, out, fn, user);
}

#define SGD_CALL(body)                                                  \
  return guarded([&] {                                                  \
    if (!s || !s->t) throw ocffm::Error(OCFFM_E_ARG, "null SGD trainer"); \
    body;                                                               \
  })

int ocffm_sgd_epoch(ocffm_sgd *s, double *mean_loss) {
  SGD_CALL(const double l = s->t->epoch(); if (mean_loss) *mean_loss = l);
}
int ocffm_sgd_average(ocffm_sgd *s) { SGD_CALL(s->t->average()); }
int ocffm_sgd_phi(ocffm_sgd *s, uint64_t n, const uint32_t *users, const uint32_t *items, float *out) {
  SGD_CALL(s->t->phi(n, users, items, out));
}
int ocffm_sgd_get(ocffm_sgd *s, char what, void *out, uint64_t cap, uint64_t *len) {
  SGD_CALL(const uint64_t n = s->t->get(what, out, cap); if (len) *len = n);
}
int ocffm_sgd_set_w(ocffm_sgd *s, const float *w, uint64_t n) { SGD_CALL(s->t->set_w(w, n)); }
int ocffm_sgd_get_info(ocffm_sgd *s, ocffm_sgd_info *out) { SGD_CALL(s->t->info(out)); }
int ocffm_sgd_sync(ocffm_sgd *s) { SGD_CALL(s->t->sync()); }
void ocffm_sgd_destroy(ocffm_sgd *s) { delete s; }

}  // extern "C"
