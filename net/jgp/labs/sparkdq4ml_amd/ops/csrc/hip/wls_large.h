// K6-large: device WLS assembly + Jacobi-PCG for k > 1024 (see wls_large.hip).
#pragma once
#include <hip/hip_runtime.h>

namespace dq4ml {

// state words of the PCG control block (f64), followed in the same buffer by x(k) and coef(nf)
enum WlsPcgState : int {
  PCG_RZ = 0, PCG_THR = 1, PCG_RR = 2, PCG_CONV = 3, PCG_BAD = 4, PCG_OK = 5,
  PCG_ITERS = 6,    // PCG iterations run (converged ones excluded)
  PCG_STATUS = 7,   // 1: wSum <= 0 or a constant label -- the host driver owns the case
  PCG_WSUM = 8, PCG_BSTD = 9, PCG_BBAR = 10, PCG_EFFL2 = 11,
  PCG_HEAD = 12,    // [count, wSum, wwSum, bSum, bbSum] as the solve read them (5 words)
  PCG_STATE_WORDS = 24
};

// flat statistics -> (on the device, no host read) the head scalars + status, the standardized
// dense system A (k x k, row-major), right-hand side b, Jacobi preconditioner minv, per-feature
// aStd; BAD set in `o` when a diagonal entry is not > 0.
void wls_assemble(const double* flat, int nf, int fit_intercept, double reg, double enet, int std_f, int std_l,
                  double* A, double* b, double* minv, double* aStd, double* aBar, double* lam, double* o,
                  hipStream_t st);

// x = 0, r = b, p = minv r, rz, thr = rtol^2 |b|^2, rr, CONV (also set for a STATUS / BAD system)
void wls_pcg_init(const double* b, const double* minv, int k, double rtol, double* o, double* r, double* p,
                  hipStream_t st);

// `iters` PCG iterations (two kernels each: A p, then the vector update), then the true residual
// check of x (OK) and coef(j) = x_j bStd / aStd_j for the live features
void wls_pcg_chunk(const double* A, const double* b, const double* minv, const double* aStd, int k, int nf, int iters,
                   double* o, double* r, double* p, double* Ap, hipStream_t st);

}  // namespace dq4ml
