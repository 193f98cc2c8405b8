// Exact path-dependent TreeSHAP for the framework's flat forests (host runtime, multi-threaded).
//
// Reference: h2o-genmodel/src/main/java/hex/genmodel/algos/tree/TreeSHAP.java (Lundberg et al.,
// "Consistent Individualized Feature Attribution for Tree Ensembles", Algorithm 2). The recursion
// keeps the unique path of (feature, zero_fraction, one_fraction, pweight) elements; zero fractions
// come from node covers (weighted training rows). Rows are independent: worker threads take
// contiguous row ranges. Split semantics are the engine's: numeric x < thr goes left, NaN follows
// na_left, categorical levels go left when their bit is set (out-of-range -> NA direction).
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

namespace {

struct PathElement {
  int feature;
  double zero_fraction, one_fraction, pweight;
};

struct Forest {
  const int* feat;
  const float* thr;
  const int* left;
  const int* right;
  const int* na_left;
  const int* cat_off;
  const uint32_t* cat_bits;
  const int* cat_nbits;
  const float* value;
  const double* cover;
};

void extend_path(PathElement* p, int d, double zf, double of, int fi) {
  p[d].feature = fi;
  p[d].zero_fraction = zf;
  p[d].one_fraction = of;
  p[d].pweight = d == 0 ? 1.0 : 0.0;
  for (int i = d - 1; i >= 0; --i) {
    p[i + 1].pweight += of * p[i].pweight * (i + 1) / (double)(d + 1);
    p[i].pweight = zf * p[i].pweight * (d - i) / (double)(d + 1);
  }
}

void unwind_path(PathElement* p, int d, int pi) {
  const double of = p[pi].one_fraction, zf = p[pi].zero_fraction;
  double next = p[d].pweight;
  for (int i = d - 1; i >= 0; --i) {
    if (of != 0) {
      const double tmp = p[i].pweight;
      p[i].pweight = next * (d + 1) / ((i + 1) * of);
      next = tmp - p[i].pweight * zf * (d - i) / (double)(d + 1);
    } else {
      p[i].pweight = p[i].pweight * (d + 1) / (zf * (d - i));
    }
  }
  for (int i = pi; i < d; ++i) {
    p[i].feature = p[i + 1].feature;
    p[i].zero_fraction = p[i + 1].zero_fraction;
    p[i].one_fraction = p[i + 1].one_fraction;
  }
}

double unwound_sum(const PathElement* p, int d, int pi) {
  const double of = p[pi].one_fraction, zf = p[pi].zero_fraction;
  double next = p[d].pweight, total = 0;
  for (int i = d - 1; i >= 0; --i) {
    if (of != 0) {
      const double tmp = next * (d + 1) / ((i + 1) * of);
      total += tmp;
      next = p[i].pweight - tmp * zf * ((d - i) / (double)(d + 1));
    } else {
      total += (p[i].pweight / zf) / ((d - i) / (double)(d + 1));
    }
  }
  return total;
}

inline bool go_left(const Forest& t, int n, const float* x) {
  const float v = x[t.feat[n]];
  if (std::isnan(v)) return t.na_left[n] != 0;
  if (t.cat_off[n] >= 0) {
    const int code = (int)v;
    if (code < 0 || code >= t.cat_nbits[n]) return t.na_left[n] != 0;
    return (t.cat_bits[t.cat_off[n] + (code >> 5)] >> (code & 31)) & 1u;
  }
  return v < t.thr[n];
}

void recurse(const Forest& t, const float* x, double* phi, int node, int d, PathElement* parent, double pz, double po,
             int pf) {
  PathElement* p = parent + d + 1;
  if (d > 0) std::memcpy(p, parent, sizeof(PathElement) * d);
  extend_path(p, d, pz, po, pf);
  if (t.feat[node] < 0) {
    for (int i = 1; i <= d; ++i) {
      const double w = unwound_sum(p, d, i);
      phi[p[i].feature] += w * (p[i].one_fraction - p[i].zero_fraction) * t.value[node];
    }
    return;
  }
  const bool l = go_left(t, node, x);
  const int hot = l ? t.left[node] : t.right[node];
  const int cold = l ? t.right[node] : t.left[node];
  const double cn = t.cover[node] > 0 ? t.cover[node] : 1.0;
  const double hz = t.cover[hot] / cn, cz = t.cover[cold] / cn;
  double iz = 1, io = 1;
  const int sf = t.feat[node];
  int pi = 0;
  for (; pi <= d; ++pi)
    if (p[pi].feature == sf) break;
  if (pi != d + 1) {
    iz = p[pi].zero_fraction;
    io = p[pi].one_fraction;
    unwind_path(p, d, pi);
    d -= 1;
  }
  recurse(t, x, phi, hot, d + 1, p, hz * iz, io, sf);
  recurse(t, x, phi, cold, d + 1, p, cz * iz, 0, sf);
}

}  // namespace

extern "C" {

// X: float32 row-major [N, F]; roots/cls: per tree; out: float64 [N, K, F+1] (last = bias, accumulated).
int h2o_treeshap(const float* X, long long N, int F, int K, int n_trees, const int* roots, const int* cls,
                 const int* depth, const int* feat, const float* thr, const int* left, const int* right,
                 const int* na_left, const int* cat_off, const uint32_t* cat_bits, const int* cat_nbits,
                 const float* value, const double* cover, double* out, int nthreads) {
  Forest t{feat, thr, left, right, na_left, cat_off, cat_bits, cat_nbits, value, cover};
  int maxd = 0;
  for (int k = 0; k < n_trees; ++k) maxd = std::max(maxd, depth[k]);
  // expected value of every tree (cover-weighted mean of leaves) -> bias column
  std::vector<double> bias(n_trees, 0.0);
  for (int k = 0; k < n_trees; ++k) {
    std::vector<std::pair<int, double>> st{{roots[k], 1.0}};
    while (!st.empty()) {
      auto [n, w] = st.back();
      st.pop_back();
      if (feat[n] < 0) { bias[k] += w * value[n]; continue; }
      const double c = cover[n] > 0 ? cover[n] : 1.0;
      st.push_back({left[n], w * cover[left[n]] / c});
      st.push_back({right[n], w * cover[right[n]] / c});
    }
  }
  int nt = nthreads > 0 ? nthreads : (int)std::thread::hardware_concurrency();
  nt = (int)std::max<long long>(1, std::min<long long>(nt, std::max<long long>(1, N / 64)));
  std::vector<std::thread> th;
  for (int w = 0; w < nt; ++w) {
    th.emplace_back([&, w]() {
      std::vector<PathElement> buf((size_t)(maxd + 2) * (maxd + 3) / 2 + 8);
      std::vector<double> phi(F + 1);
      const long long lo = N * w / nt, hi = N * (w + 1) / nt;
      for (long long r = lo; r < hi; ++r) {
        const float* x = X + r * F;
        for (int k = 0; k < n_trees; ++k) {
          std::fill(phi.begin(), phi.end(), 0.0);
          recurse(t, x, phi.data(), roots[k], 0, buf.data(), 1, 1, -1);
          double* o = out + (r * K + cls[k]) * (F + 1);
          for (int f = 0; f < F; ++f) o[f] += phi[f];
          o[F] += bias[k];
        }
      }
    });
  }
  for (auto& x : th) x.join();
  return 0;
}

}  // extern "C"
