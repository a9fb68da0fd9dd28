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

// OWLQN branch for 128 < k <= kWlsQnGridMaxK (wls_qn_grid.hip): one cooperative launch of
// wls_qn_grid_blocks(k) blocks, same out layout as wls_qn_small; work = wls_qn_grid_work(k, blocks)
// doubles of device scratch (the dense standardized system, vectors, history, partial sums)
constexpr int kWlsQnGridMaxK = 4608;
struct WlsQnWork {
  double *A, *ab, *l1, *bar, *sstd, *x, *g, *ag, *d, *cx, *cg, *cag, *S, *Y, *part, *scal;
  unsigned* gbar;  // grid barrier [arrivals, abandoned] (common.h grid_barrier)
};
int64_t wls_qn_grid_work(int k, int blocks);
int wls_qn_grid_blocks(int k);
void wls_qn_grid(const double* flat, int nf, int fit_intercept, double reg, double enet, int std_f, int std_l,
                 int max_iter, double tol, int hist_cap, double* work, int blocks, double* out, hipStream_t st);

}  // namespace dq4ml
