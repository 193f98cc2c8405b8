// Host harness for csrc/treeshap.cpp under ASan/UBSan or TSan: random complete trees (numeric splits, NA
// directions, one categorical split per tree), 8 threads; checks SHAP additivity (sum of contributions + bias ==
// the tree-sum prediction) for every row.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <random>
#include <vector>
extern "C" int h2o_treeshap(const float* X, long long N, int F, int K, int n_trees, const int* roots, const int* cls,
                            const int* depth, const int* feat, const float* thr, const int* left, const int* right,
                            const int* na_left, const int* cat_off, const uint32_t* cat_bits, const int* cat_nbits,
                            const float* value, const double* cover, double* out, int nthreads);
int main() {
  const int F = 6, T = 5, D = 4;
  const long long N = 3000;
  std::mt19937 rng(7);
  std::uniform_real_distribution<float> U(-1.f, 1.f);
  std::vector<int> feat, left, right, na_left, cat_off, cat_nbits, roots, cls, depth;
  std::vector<float> thr, value;
  std::vector<double> cover;
  std::vector<uint32_t> cat_bits;
  for (int t = 0; t < T; ++t) {
    const int base = (int)feat.size(), n = (1 << (D + 1)) - 1;
    roots.push_back(base); cls.push_back(0); depth.push_back(D);
    for (int i = 0; i < n; ++i) {
      const bool leaf = i >= (1 << D) - 1;
      const bool cat = !leaf && i == 1;                           // one categorical split (feature 5 codes 0..7)
      feat.push_back(leaf ? -1 : (cat ? 5 : (int)(rng() % 5)));
      thr.push_back(U(rng));
      left.push_back(leaf ? -1 : base + 2 * i + 1);
      right.push_back(leaf ? -1 : base + 2 * i + 2);
      na_left.push_back((int)(rng() % 2));
      cat_off.push_back(cat ? (int)cat_bits.size() : -1);
      cat_nbits.push_back(cat ? 8 : 0);
      if (cat) cat_bits.push_back(0x5Au);
      value.push_back(leaf ? U(rng) : 0.f);
      cover.push_back(0.0);
    }
    for (int i = n - 1; i >= 0; --i) {                            // covers: leaves random, parents = sum
      const int g = base + i;
      cover[g] = left[g] < 0 ? 1.0 + (rng() % 100) : cover[left[g]] + cover[right[g]];
    }
  }
  std::vector<float> X((size_t)N * F);
  for (long long r = 0; r < N; ++r)
    for (int f = 0; f < F; ++f) X[(size_t)r * F + f] = f == 5 ? (float)(rng() % 8) : (rng() % 50 == 0 ? NAN : U(rng));
  std::vector<double> out((size_t)N * (F + 1), 0.0);
  h2o_treeshap(X.data(), N, F, 1, T, roots.data(), cls.data(), depth.data(), feat.data(), thr.data(), left.data(),
               right.data(), na_left.data(), cat_off.data(), cat_bits.data(), cat_nbits.data(), value.data(),
               cover.data(), out.data(), 8);
  double worst = 0;
  for (long long r = 0; r < N; ++r) {
    double pred = 0, sum = 0;
    for (int t = 0; t < T; ++t) {                                 // the row's leaf, by the same split semantics
      int n = roots[t];
      while (left[n] >= 0) {
        const float x = X[(size_t)r * F + feat[n]];
        bool goleft;
        if (std::isnan(x)) goleft = na_left[n] != 0;
        else if (cat_off[n] >= 0) { const int c = (int)x; goleft = c < cat_nbits[n] && ((cat_bits[cat_off[n] + c / 32] >> (c % 32)) & 1u); }
        else goleft = x < thr[n];
        n = goleft ? left[n] : right[n];
      }
      pred += value[n];
    }
    for (int f = 0; f <= F; ++f) sum += out[(size_t)r * (F + 1) + f];
    worst = std::max(worst, std::fabs(sum - pred));
  }
  std::printf("rows %lld trees %d max |sum(phi) + bias - pred| = %.3g\n", N, T, worst);
  return worst < 1e-6 ? 0 : 1;
}
