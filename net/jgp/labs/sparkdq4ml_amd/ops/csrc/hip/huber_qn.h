// Device L-BFGS-B for LinearRegression(loss="huber") (see huber_qn.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace dq4ml {

// the control word the passes and the host poll read (HCtl.act, the first int of the work block)
constexpr int kHuberEval = 0;
constexpr int kHuberDone = 3;

// f64 elements of the state block (control word first) and of the output
// [coef (d) | intercept | scale | status | why | states | iterations | evaluations | (pad) | history]
int64_t huber_qn_work(int d, bool fit_icpt);
int huber_qn_out(int d, int hist_cap);

// x0 = all ones (Spark's initial point) and the first trial
void huber_qn_init(int d, bool fit_icpt, int max_iter, double tol, int hist_cap, const double* sx, const double* lam,
                   const double* scale, const double* shift, double* work, double* trial, double* out, hipStream_t st);
// consume one (all-reduced) evaluation red = [loss, W, g_b, g_sigma, g_x (d)], write the next trial
void huber_qn_ctl(int d, bool fit_icpt, int max_iter, double tol, int hist_cap, const double* sx, const double* lam,
                  const double* scale, const double* shift, double* work, double* trial, const double* red,
                  double* out, hipStream_t st);

}  // namespace dq4ml
