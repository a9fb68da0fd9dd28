// K6-small: device WLS Cholesky for <= 64 features (see wls_small.hip).
#pragma once
#include <hip/hip_runtime.h>

namespace dq4ml {

constexpr int kWlsSmallMaxFeatures = 64;

// out: [coef(nf), intercept, status, count, wSum, wwSum, bSum, bbSum]; status 0 = solved,
// 1 zero weight, 2 empty, 3 constant label, 7 not positive definite (host re-solves 1/2/3/7)
void wls_small(const double* flat, int nf, int fit_intercept, double reg, double enet, int std_f, int std_l,
               double* out, hipStream_t st);

constexpr int kWlsQnMaxK = 128;
// OWLQN branch (L1 > 0) for k <= 128, one wave: out = [coef(nf), intercept, status, count, wSum,
// wwSum, bSum, bbSum, H, reason, history(hist_cap)]; status 0 solved, 1/2/3 as wls_small,
// 8 history capacity exceeded, 9 no L1 term (host re-solves every non-zero status)
void wls_qn_small(const double* flat, int nf, int fit_intercept, double reg, double enet, int std_f, int std_l,
                  int max_iter, double tol, int hist_cap, double* out, hipStream_t st);

}  // namespace dq4ml
