// sgd_oracle.cpp — TEST INFRASTRUCTURE ONLY.
//
// CPU restatement of the product's field-aware FM SGD / AdaGrad trainer with
// sampled negatives (one-class-ffm_amd/csrc/sgd.hip).  BASELINE.json's
// north_star asks for this mode (per-instance pairwise interaction, SGD /
// AdaGrad, HOGWILD writes, negative sampling from an alias table); the
// reference (johncreed/one-class-ffm) has NO counterpart: its solver is the
// block Newton-CG of ffm.cpp.  This file is therefore "parity unpinned"
// against the reference.  It pins the GPU kernel against an independent
// serial statement of the same algorithm:
//
//   instance q of epoch e (positives P, nneg negatives per positive,
//   T = P (1 + nneg)):  qq = (A q + B) mod T  (A coprime with T),
//   p = qq / (1 + nneg), r = qq mod (1 + nneg); user = pu[p];
//   item = pv[p] (r == 0, label +1) or an alias draw (label -1) from
//   h = mix64(seed + 0x9E3779B97F4A7C15 (e T + qq)):
//   idx = (h >> 32) mod n, coin = (h & 0xffffff) 2^-24,
//   item = coin < prob[idx] ? idx : alias[idx].
//   nodes = user row nodes ++ item row nodes (global feature ids, fields).
//   phi = rn sum_{a<b} <W[j_a][f_b], W[j_b][f_a]> x_a x_b, rn = 1/sum x^2
//   (norm) or 1.  kappa = -y e^{-y phi} / (1 + e^{-y phi});
//   loss = log(1 + e^{-y phi}).  Every slot (a, f) with a partner b != a in
//   field f, from the pre-step W:
//   g = lam W[j_a][f] + kappa rn x_a sum_{b != a, f_b = f} x_b W[j_b][f_a];
//   AdaGrad: G += g^2, W -= eta g / sqrt(G); plain SGD: W -= eta g.
//
// Serial order and fp32 storage as the GPU's one-wave (serial) mode; the
// sums run in a different order there, so the tests compare with a tolerance.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

namespace {

inline uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

}  // namespace

extern "C" {

// Vose alias table over weights w[n].
void sgo_alias(uint64_t n, const double *w, float *prob, uint32_t *alias) {
  double tot = 0;
  for (uint64_t i = 0; i < n; i++) tot += w[i];
  std::vector<double> p(n);
  std::vector<uint64_t> small, large;
  for (uint64_t i = 0; i < n; i++) {
    p[i] = tot > 0 ? w[i] * (double)n / tot : 1.0;
    (p[i] < 1.0 ? small : large).push_back(i);
  }
  for (uint64_t i = 0; i < n; i++) alias[i] = (uint32_t)i;
  while (!small.empty() && !large.empty()) {
    const uint64_t s = small.back(), l = large.back();
    small.pop_back();
    large.pop_back();
    prob[s] = (float)p[s];
    alias[s] = (uint32_t)l;
    p[l] = (p[l] + p[s]) - 1.0;
    (p[l] < 1.0 ? small : large).push_back(l);
  }
  for (uint64_t i : large) prob[i] = 1.0f;
  for (uint64_t i : small) prob[i] = 1.0f;
}

// One serial epoch.  uptr/vptr: row offsets into node arrays (global feature
// id, field, value).  W, G: NF x F x KP floats, updated in place.  Returns
// the summed loss.
double sgo_epoch(uint64_t P, const uint32_t *pu, const uint32_t *pv, uint32_t nneg, uint64_t n_items,
                 const float *prob, const uint32_t *alias, const uint64_t *uptr, const uint32_t *unode,
                 const uint32_t *ufld, const float *uval, const uint64_t *vptr, const uint32_t *vnode,
                 const uint32_t *vfld, const float *vval, uint32_t F, uint32_t KP, float *W, float *G, float eta,
                 float lam, int adagrad, int norm, uint64_t seed, uint64_t epoch, uint64_t A, uint64_t B) {
  const uint64_t T = P * (1 + (uint64_t)nneg);
  double loss_sum = 0;
  std::vector<uint32_t> j, f;
  std::vector<float> x, acc(KP);
  std::vector<float *> wp, gp;
  std::vector<float> wn, gn;
  for (uint64_t q = 0; q < T; q++) {
    const uint64_t qq = (A * q + B) % T;
    const uint64_t p = qq / (1 + nneg), r = qq % (1 + nneg);
    const uint32_t u = pu[p];
    uint32_t it = pv[p];
    float y = 1.0f;
    if (r) {
      const uint64_t h = mix64(seed + 0x9E3779B97F4A7C15ULL * (epoch * T + qq));
      const uint64_t idx = (h >> 32) % n_items;
      const float coin = (float)(h & 0xffffffu) * (1.0f / 16777216.0f);
      it = coin < prob[idx] ? (uint32_t)idx : alias[idx];
      y = -1.0f;
    }
    j.clear();
    f.clear();
    x.clear();
    for (uint64_t t = uptr[u]; t < uptr[u + 1]; t++) {
      j.push_back(unode[t]);
      f.push_back(ufld[t]);
      x.push_back(uval[t]);
    }
    for (uint64_t t = vptr[it]; t < vptr[it + 1]; t++) {
      j.push_back(vnode[t]);
      f.push_back(vfld[t]);
      x.push_back(vval[t]);
    }
    const size_t n = j.size();
    float rn = 1.0f;
    if (norm) {
      float s = 0;
      for (float v : x) s += v * v;
      rn = s > 0 ? 1.0f / s : 1.0f;
    }
    auto row = [&](uint32_t feat, uint32_t fld) { return W + ((size_t)feat * F + fld) * KP; };
    float phi = 0;
    for (size_t a = 0; a < n; a++)
      for (size_t b = a + 1; b < n; b++) {
        const float *wa = row(j[a], f[b]), *wb = row(j[b], f[a]);
        float t = 0;
        for (uint32_t d = 0; d < KP; d++) t += wa[d] * wb[d];
        phi += t * x[a] * x[b];
      }
    phi *= rn;
    const float ex = std::exp(-y * phi);
    loss_sum += std::log1p((double)ex);
    const float kappa = -y * ex / (1.0f + ex);
    // every slot's step from the pre-step W, then the writes (slot order)
    wp.clear();
    gp.clear();
    wn.clear();
    gn.clear();
    for (size_t a = 0; a < n; a++)
      for (uint32_t fl = 0; fl < F; fl++) {
        bool any = false;
        std::fill(acc.begin(), acc.end(), 0.0f);
        for (size_t b = 0; b < n; b++) {
          if (b == a || f[b] != fl) continue;
          any = true;
          const float *wb = row(j[b], f[a]);
          for (uint32_t d = 0; d < KP; d++) acc[d] += x[b] * wb[d];
        }
        if (!any) continue;
        float *w = row(j[a], fl);
        float *g = G + (w - W);
        const float c = kappa * rn * x[a];
        for (uint32_t d = 0; d < KP; d++) {
          const float gr = lam * w[d] + c * acc[d];
          if (adagrad) {
            const float gv = g[d] + gr * gr;
            gn.push_back(gv);
            wn.push_back(w[d] - eta * gr / std::sqrt(gv));
          } else {
            gn.push_back(g[d]);
            wn.push_back(w[d] - eta * gr);
          }
        }
        wp.push_back(w);
        gp.push_back(g);
      }
    for (size_t s = 0; s < wp.size(); s++) {
      std::memcpy(wp[s], wn.data() + s * KP, KP * sizeof(float));
      std::memcpy(gp[s], gn.data() + s * KP, KP * sizeof(float));
    }
  }
  return loss_sum;
}

}  // extern "C"
