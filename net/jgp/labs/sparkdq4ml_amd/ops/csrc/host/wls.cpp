#include "wls.h"

#include <cmath>

#include "solvers.h"

namespace dq4ml {

WlsResult wls_fit(const double* flat, int nf, bool fit_intercept, double reg_param, double elastic_net,
                  bool standardize_features, bool standardize_label, int solver_type, int max_iter, double tol,
                  bool keep_system) {
  WlsResult res;
  const double count = flat[0], wSum = flat[1], bSum = flat[3], bbSum = flat[4];
  const double* aSum = flat + 5;
  const double* abSum = flat + 5 + nf;
  const double* aaSum = flat + 5 + 2 * (int64_t)nf;
  res.w_sum = wSum;
  if (wSum <= 0.0) {
    res.status = count > 0 ? WLS_ZERO_WEIGHT : WLS_EMPTY;
    return res;
  }
  const int k = fit_intercept ? nf + 1 : nf;
  const double rawBBar = bSum / wSum;
  const double rawBStd = std::sqrt(std::fmax(bbSum / wSum - rawBBar * rawBBar, 0.0));
  const double bStd = rawBStd == 0.0 ? std::fabs(rawBBar) : rawBStd;
  if (rawBStd == 0.0) {
    if (fit_intercept || rawBBar == 0.0) {
      res.status = rawBBar == 0.0 ? WLS_ZERO_LABEL : WLS_CONST_LABEL;
      res.solver = "none";
      res.coefficients.assign(nf, 0.0);
      res.intercept = rawBBar;
      res.objective_history.assign(1, 0.0);
      return res;
    }
    if (reg_param > 0.0 && standardize_label) {
      res.status = WLS_CONST_LABEL_REG_STD;
      return res;
    }
    res.status = WLS_CONST_LABEL_NO_ICPT;  // warning only
  }
  const double bBar = rawBBar / bStd;
  const double bbBar = bbSum / wSum / (bStd * bStd);
  std::vector<double> aStd(nf), aBar(nf), abBar(nf);
  for (int j = 0; j < nf; ++j) {
    const double m = aSum[j] / wSum;
    aStd[j] = std::sqrt(std::fmax(aaSum[pk(j, j)] / wSum - m * m, 0.0));
    aBar[j] = aStd[j] == 0.0 ? 0.0 : m / aStd[j];
    abBar[j] = aStd[j] == 0.0 ? 0.0 : abSum[j] / wSum / (aStd[j] * bStd);
  }
  // standardized packed A^T W A (+ intercept column [aBar, 1])
  std::vector<double> ata((size_t)k * (k + 1) / 2);
  for (int j = 0; j < nf; ++j)
    for (int i = 0; i <= j; ++i) {
      const double den = aStd[i] * aStd[j];
      ata[pk(i, j)] = den == 0.0 ? 0.0 : aaSum[pk(i, j)] / wSum / den;
    }
  const double eff_reg = reg_param / bStd;
  const double eff_l1 = elastic_net * eff_reg, eff_l2 = (1.0 - elastic_net) * eff_reg;
  for (int j = 0; j < nf; ++j) {
    double lam = eff_l2;
    if (!standardize_features) lam = aStd[j] != 0.0 ? lam / (aStd[j] * aStd[j]) : 0.0;
    if (!standardize_label) lam *= bStd;
    ata[pk(j, j)] += lam;
  }
  if (fit_intercept) {
    for (int i = 0; i < nf; ++i) ata[pk(i, nf)] = aBar[i];
    ata[pk(nf, nf)] = 1.0;
  }
  std::vector<double> atb(abBar);
  if (fit_intercept) atb.push_back(bBar);

  const bool use_qn = (solver_type == 0 && elastic_net != 0.0 && reg_param != 0.0) || solver_type == 2;
  std::vector<double> x;
  if (use_qn) {
    std::vector<double> l1;
    if (eff_l1 != 0.0) {
      l1.assign(k, eff_l1);
      if (!standardize_features)
        for (int j = 0; j < nf; ++j) l1[j] = aStd[j] != 0.0 ? eff_l1 / aStd[j] : 0.0;
      if (fit_intercept) l1[nf] = 0.0;
    }
    QNResult q = quasi_newton(bBar, bbBar, atb, ata, aBar, fit_intercept, max_iter, tol, l1);
    x = std::move(q.x);
    res.objective_history = std::move(q.objective_history);
    res.converged_reason = std::move(q.converged_reason);
    res.solver = l1.empty() ? "l-bfgs" : "owlqn";
  } else {
    try {
      x = cholesky_solve(k, ata, atb);
      res.solver = "cholesky";
      res.objective_history.assign(1, 0.0);
    } catch (const SingularMatrixError&) {
      if (solver_type != 0) throw;
      res.singular_fallback = true;
      QNResult q = quasi_newton(bBar, bbBar, atb, ata, aBar, fit_intercept, max_iter, tol, {});
      x = std::move(q.x);
      res.objective_history = std::move(q.objective_history);
      res.converged_reason = std::move(q.converged_reason);
      res.solver = "l-bfgs";
    }
  }
  res.coefficients.resize(nf);
  for (int j = 0; j < nf; ++j) res.coefficients[j] = aStd[j] != 0.0 ? x[j] * bStd / aStd[j] : 0.0;
  res.intercept = fit_intercept ? x[nf] * bStd : 0.0;
  if (keep_system && res.solver == "cholesky") {
    res.ata = std::move(ata);
    res.a_std = std::move(aStd);
  }
  return res;
}

}  // namespace dq4ml
