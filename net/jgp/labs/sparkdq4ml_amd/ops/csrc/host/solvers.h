// Normal-equation solvers for the WeightedLeastSquares path of LinearRegression.fit.
//
// Behavioural spec: Spark 2.4.4 WeightedLeastSquares hands the standardized,
// packed (upper, column-major) A^T W A plus A^T W b to either a Cholesky solver (no L1) or a
// quasi-Newton solver (Breeze OWLQN when L1 > 0, L-BFGS otherwise) over the quadratic
// NormalEquationCostFun.  The reference lab triggers the OWLQN branch at
// DataQuality4MachineLearningApp.java:120-126 (maxIter 40, regParam 1, elasticNetParam 1).
//
// All arithmetic is IEEE f64 on the host: the systems are (d+1)x(d+1) with d <= a few hundred on
// this path (larger d goes to the device solver in models/optim/device_solver.py).
#pragma once
#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

namespace dq4ml {

struct SingularMatrixError : std::runtime_error {
  explicit SingularMatrixError(const std::string& m) : std::runtime_error(m) {}
};

// index of (i, j), i <= j, in a packed upper column-major matrix
inline int64_t pk(int64_t i, int64_t j) { return i + j * (j + 1) / 2; }

// y = A x for packed-upper symmetric A (BLAS dspmv, alpha=1, beta=0)
void dspmv(int k, const double* ap, const double* x, double* y);

// Solve A x = b (A packed upper SPD) via Cholesky (LAPACK dppsv semantics). Throws
// SingularMatrixError when A is not positive definite.
std::vector<double> cholesky_solve(int k, const std::vector<double>& ap, const std::vector<double>& b);

// Inverse of SPD packed-upper A, returned packed-upper (LAPACK dpptrf + dpptri).
std::vector<double> cholesky_inverse(int k, const std::vector<double>& ap);

struct QNResult {
  std::vector<double> x;
  std::vector<double> objective_history;
  std::string converged_reason;
};

// Breeze-compatible quasi-Newton over NormalEquationCostFun.
//   l1 : per-coordinate L1 strengths (empty => plain L-BFGS with strong-Wolfe line search)
QNResult quasi_newton(double bBar, double bbBar, const std::vector<double>& ab,
                      const std::vector<double>& aa_packed, const std::vector<double>& aBar,
                      bool fit_intercept, int max_iter, double tol, const std::vector<double>& l1,
                      int memory = 10);

}  // namespace dq4ml
