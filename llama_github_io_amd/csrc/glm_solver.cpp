// GLM penalized solve on the (small, P x P) Gram, host side (reference: hex/glm/GLM.java COD /
// ComputationState: cyclic coordinate descent on the Gram after each GramTask).
//
// min_b  1/2 b'Gb - r'b + l2/2 |b_pen|^2 + l1 |b_pen|_1   (pen[j] = 0: unpenalized, e.g. the intercept)
// optional non-negativity of penalized coefficients and box constraints lb <= b <= ub (NaN = none).
// The gradient G b is kept up to date incrementally (one column axpy per changed coordinate).
#include <cmath>
#include <cstdint>
#include <vector>

extern "C" int h2o_gram_cd(const double* G, const double* r, int P, double l1, double l2, const double* pen,
                           int non_negative, const double* lb, const double* ub, double* b, int max_iter, double tol) {
  std::vector<double> grad(P, 0.0);
  for (int j = 0; j < P; ++j) {
    if (lb && !std::isnan(lb[j]) && b[j] < lb[j]) b[j] = lb[j];
    if (ub && !std::isnan(ub[j]) && b[j] > ub[j]) b[j] = ub[j];
  }
  for (int i = 0; i < P; ++i) {
    double s = 0.0;
    const double* gi = G + (int64_t)i * P;
    for (int j = 0; j < P; ++j) s += gi[j] * b[j];
    grad[i] = s;
  }
  int it = 0;
  for (; it < max_iter; ++it) {
    double mx = 0.0;
    for (int j = 0; j < P; ++j) {
      const double gjj = G[(int64_t)j * P + j];
      const double denom = gjj + l2 * pen[j];
      if (denom <= 0.0) continue;
      const double rho = r[j] - (grad[j] - gjj * b[j]);
      double nb;
      if (pen[j] == 0.0) {
        nb = rho / denom;
      } else {
        const double a = std::fabs(rho) - l1;
        nb = a > 0.0 ? std::copysign(a, rho) / denom : 0.0;
        if (non_negative && nb < 0.0) nb = 0.0;
      }
      if (lb && !std::isnan(lb[j]) && nb < lb[j]) nb = lb[j];
      if (ub && !std::isnan(ub[j]) && nb > ub[j]) nb = ub[j];
      const double d = nb - b[j];
      if (d != 0.0) {
        const double* gcol = G + (int64_t)j * P;   // G symmetric: row j == column j
        for (int i = 0; i < P; ++i) grad[i] += gcol[i] * d;
        b[j] = nb;
        if (std::fabs(d) > mx) mx = std::fabs(d);
      }
    }
    if (mx < tol) break;
  }
  return it;
}
