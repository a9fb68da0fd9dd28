// WeightedLeastSquares.fit driver on aggregated statistics: the whole
// standardize -> solve -> un-standardize sequence of Spark 2.4.4 WeightedLeastSquares in native
// code, so a normal-equation fit costs one D2H of the flat statistics plus microseconds of host
// work (the per-step host overhead that dominates the 8-GPU d=32 headline otherwise).
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace dq4ml {

enum WlsStatus {
  WLS_OK = 0,
  WLS_ZERO_WEIGHT = 1,         // Sum of weights cannot be zero (count > 0)
  WLS_EMPTY = 2,               // Training dataset is empty
  WLS_CONST_LABEL = 3,         // constant label short-circuit (coefficients 0, intercept = mean)
  WLS_ZERO_LABEL = 4,          // label mean and std both zero
  WLS_CONST_LABEL_REG_STD = 5, // constant label + regParam > 0 + standardizeLabel: error
  WLS_CONST_LABEL_NO_ICPT = 6, // constant label, no intercept: warning, continue
};

struct WlsResult {
  int status = WLS_OK;
  bool singular_fallback = false;   // Cholesky failed, retried with L-BFGS
  std::string solver;               // "cholesky" | "owlqn" | "l-bfgs" | "none"
  std::vector<double> coefficients; // original space
  double intercept = 0.0;
  std::vector<double> objective_history;
  std::string converged_reason;
  // lazily needed by diagInvAtWA: the standardized system and the feature stds
  std::vector<double> ata;  // packed upper (k(k+1)/2), k = nf (+1 with intercept)
  std::vector<double> a_std;
  double w_sum = 0.0;
};

// flat = [count, wSum, wwSum, bSum, bbSum, aSum(nf), abSum(nf), aaSum packed-upper(nf)]
// solver_type: 0 auto, 1 cholesky, 2 quasi-newton
WlsResult wls_fit(const double* flat, int nf, bool fit_intercept, double reg_param, double elastic_net,
                  bool standardize_features, bool standardize_label, int solver_type, int max_iter, double tol,
                  bool keep_system);

}  // namespace dq4ml
