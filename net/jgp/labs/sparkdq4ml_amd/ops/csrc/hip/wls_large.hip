// K6-large: the WeightedLeastSquares normal-equation solve for k > 1024 (BASELINE config 5:
// k = 4097) on the device, straight from the all-reduced flat statistics (the
// solve behind DataQuality4MachineLearningApp.java:126 when numFeatures <= 4096).
//
// Why kernels and not torch ops.  The Gram of a 1e7 x 4096 fit is ~78 ms of MFMA work; the solve
// that follows was ~200 small torch launches (an 8.4 M-entry index scatter to build the dense
// system, then ~12 elementwise / dot / gemv ops per CG iteration) and took ~5 ms, almost all of
// it host issue and launch gaps (kernel trace: 1.65 ms of kernel time in a 5.0 ms tail).  Here:
//  * wls_head_kernel      one thread: the label / weight statistics of the head -> wSum, bStd, the
//                         label mean, the effective L2 and the short-circuit status (no weight,
//                         constant label: the host driver's cases), into the control block -- no
//                         launch of the solve needs a host read, so a fit enqueues it whole;
//  * wls_prep_kernel      one thread per feature: population std, standardized means, the L2
//                         diagonal, the right-hand side (same algebra and operation order as
//                         csrc/host/wls.cpp and models/optim.py);
//  * wls_dense_kernel     one 32 x 32 tile pair per block: reads the packed-upper statistics
//                         row-contiguously (lower tile), writes the tile and — through an LDS
//                         transpose — its mirror, both coalesced; the Jacobi preconditioner and
//                         the "diagonal not > 0" flag fall out of the diagonal tiles;
//  * PCG                  per iteration ONE memory-bound GEMV (one wave per row, 4 independent
//                         accumulator chains) and ONE one-wave vector update (all dots and axpys
//                         of the iteration, shuffle reductions, no LDS).  Converged
//                         iterations exit at their first instruction, so a fixed chunk of
//                         iterations needs no host check; the host reads one control block per
//                         chunk (state + x + coefficients) -- or, for an asynchronous fit, once,
//                         when the model is first read (models/regression.py _PendingWLS).
// Everything is fixed-order (no atomics): bitwise deterministic run to run.
#include <hip/hip_runtime.h>

#include "common.h"
#include "wls_large.h"

namespace dq4ml {

namespace {

constexpr int kUpdThreads = 64;  // the PCG vector kernels: one wave, no LDS

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int s = 32; s > 0; s >>= 1) v += __shfl_xor(v, s);
  return v;
}

// same algebra as models/optim.py _wls_device / csrc/host/wls.cpp: population label std, the
// elastic-net L2 part of the standardized regularization
__global__ void wls_head_kernel(const double* __restrict__ flat, double reg, double enet, double* __restrict__ o) {
  const double wSum = flat[1], bSum = flat[3], bbSum = flat[4];
  const double bBar = wSum > 0.0 ? bSum / wSum : 0.0;
  const double bStd = wSum > 0.0 ? sqrt(fmax(bbSum / wSum - bBar * bBar, 0.0)) : 0.0;
  const bool sc = !(wSum > 0.0) || bStd == 0.0;  // the native driver owns these cases' semantics
  for (int i = 0; i < 5; ++i) o[PCG_HEAD + i] = flat[i];
  o[PCG_WSUM] = wSum;
  o[PCG_BSTD] = sc ? 1.0 : bStd;
  o[PCG_BBAR] = bBar;
  o[PCG_EFFL2] = sc ? 0.0 : (1.0 - enet) * reg / bStd;
  o[PCG_STATUS] = sc ? 1.0 : 0.0;
  o[PCG_BAD] = 0.0;
  o[PCG_ITERS] = 0.0;
}

__global__ __launch_bounds__(256) void wls_prep_kernel(const double* __restrict__ flat, int nf, int fit_intercept,
                                                       int std_f, int std_l, double* __restrict__ aStd,
                                                       double* __restrict__ aBar, double* __restrict__ lam,
                                                       double* __restrict__ b, double* __restrict__ o) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  const double wSum = o[PCG_WSUM], bStd = o[PCG_BSTD], eff_l2 = o[PCG_EFFL2];
  if (j == 0 && fit_intercept) b[nf] = o[PCG_BBAR] / bStd;
  if (j >= nf) return;
  const double* aSum = flat + 5;
  const double* abSum = flat + 5 + nf;
  const double* aaP = flat + 5 + 2 * nf;
  const double m = aSum[j] / wSum;
  const double s = sqrt(fmax(aaP[(int64_t)j * (j + 1) / 2 + j] / wSum - m * m, 0.0));
  const bool nz = s != 0.0;
  const double safe = nz ? s : 1.0;
  aStd[j] = s;
  aBar[j] = nz ? m / safe : 0.0;
  b[j] = nz ? abSum[j] / wSum / (safe * bStd) : 0.0;
  double l = eff_l2;
  if (!std_f) l = nz ? l / (safe * safe) : 0.0;
  if (!std_l) l = l * bStd;
  lam[j] = l;
}

__device__ __forceinline__ double dense_val(const double* __restrict__ aaP, const double* __restrict__ aStd,
                                            const double* __restrict__ aBar, const double* __restrict__ lam,
                                            int nf, double wSum, int r, int c) {
  if (r < nf && c < nf) {
    const int i = r < c ? r : c, j = r < c ? c : r;
    const double s = aaP[(int64_t)j * (j + 1) / 2 + i] / wSum;
    const double den = aStd[r] * aStd[c];
    double v = den != 0.0 ? s / den : 0.0;
    if (r == c) v += lam[r];
    return v;
  }
  if (r == nf && c == nf) return 1.0;  // intercept column [aBar, 1]
  return r == nf ? aBar[c] : aBar[r];
}

// block t = one lower tile (tr >= tc) of the T x T tile grid; writes tile (tr, tc) and its mirror
__global__ __launch_bounds__(256) void wls_dense_kernel(const double* __restrict__ flat, int nf, int k,
                                                        const double* __restrict__ aStd,
                                                        const double* __restrict__ aBar,
                                                        const double* __restrict__ lam, double* __restrict__ A,
                                                        double* __restrict__ minv, double* __restrict__ o) {
  __shared__ double tile[32][33];
  const int64_t t = blockIdx.x;
  int tr = (int)((sqrt(8.0 * (double)t + 1.0) - 1.0) * 0.5);
  while ((int64_t)(tr + 1) * (tr + 2) / 2 <= t) ++tr;
  while ((int64_t)tr * (tr + 1) / 2 > t) --tr;
  const int tc = (int)(t - (int64_t)tr * (tr + 1) / 2);
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  const double* aaP = flat + 5 + 2 * nf;
  const double wSum = o[PCG_WSUM];
  const int c = tc * 32 + tx;
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    const int rr = ty + 8 * m, r = tr * 32 + rr;
    if (r < k && c < k) {
      const double v = dense_val(aaP, aStd, aBar, lam, nf, wSum, r, c);
      A[(int64_t)r * k + c] = v;
      tile[rr][tx] = v;
      if (r == c) {
        minv[r] = 1.0 / v;
        if (!(v > 0.0)) o[PCG_BAD] = 1.0;  // (a short-circuit head leaves BAD alone: STATUS rules)
      }
    }
  }
  if (tr == tc) return;  // block-uniform
  __syncthreads();
  const int r = tr * 32 + tx;  // the mirror: row c' of tile tc, column r
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    const int cc = ty + 8 * m, c2 = tc * 32 + cc;
    if (r < k && c2 < k) A[(int64_t)c2 * k + r] = tile[tx][cc];
  }
}

// The PCG vector kernels are ONE wave with no LDS (wave_sum over shuffles): in an asynchronous
// wide fit they run beside the next fit's SYRK, whose one block per CU holds the whole LDS --
// a kernel needing any LDS would wait for that SYRK to end (profiles/r6_wide_async.md).
__global__ __launch_bounds__(kUpdThreads) void pcg_init_kernel(const double* __restrict__ b,
                                                               const double* __restrict__ minv, int k, double rtol,
                                                               double* __restrict__ o, double* __restrict__ r,
                                                               double* __restrict__ p) {
  double* x = o + PCG_STATE_WORDS;
  double rz = 0.0, bb = 0.0;
  for (int e = threadIdx.x; e < k; e += kUpdThreads) {
    const double be = b[e], z = minv[e] * be;
    x[e] = 0.0;
    r[e] = be;
    p[e] = z;
    rz += be * z;
    bb += be * be;
  }
  rz = wave_sum(rz);
  bb = wave_sum(bb);
  if (threadIdx.x == 0) {
    const double thr = (rtol * rtol) * bb;
    o[PCG_RZ] = rz;
    o[PCG_THR] = thr;
    o[PCG_RR] = bb;
    // a short-circuit head or a non-positive diagonal: nothing to iterate (every later kernel of
    // the solve exits at once; the host reads STATUS / BAD and takes the exact fallback)
    o[PCG_CONV] = (bb <= thr || o[PCG_STATUS] != 0.0 || o[PCG_BAD] != 0.0) ? 1.0 : 0.0;
    o[PCG_OK] = 0.0;
  }
}

// out = A v, one wave per row (A row-major k x k); `skip`: nothing to do once CG has converged
__global__ __launch_bounds__(256) void pcg_matvec_kernel(const double* __restrict__ A, const double* __restrict__ v,
                                                         double* __restrict__ out, int k,
                                                         const double* __restrict__ o, int skip) {
  if (skip && o[PCG_CONV] != 0.0) return;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= k) return;  // wave-uniform
  const double* a = A + (int64_t)row * k;
  double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
  int c = lane;
  for (; c + 192 < k; c += 256) {
    s0 += a[c] * v[c];
    s1 += a[c + 64] * v[c + 64];
    s2 += a[c + 128] * v[c + 128];
    s3 += a[c + 192] * v[c + 192];
  }
  for (; c < k; c += 64) s0 += a[c] * v[c];
  const double s = wave_sum((s0 + s1) + (s2 + s3));
  if (lane == 0) out[row] = s;
}

// one PCG iteration's vector work (Jacobi preconditioner), Ap = A p already computed
__global__ __launch_bounds__(kUpdThreads) void pcg_update_kernel(const double* __restrict__ minv,
                                                                 const double* __restrict__ Ap, int k,
                                                                 double* __restrict__ o, double* __restrict__ r,
                                                                 double* __restrict__ p) {
  const double rr = o[PCG_RR], thr = o[PCG_THR], rz = o[PCG_RZ];
  if (!(rr > thr)) return;  // converged (or NaN): the iteration is a no-op, wave-uniform
  double* x = o + PCG_STATE_WORDS;
  double s = 0.0;
  for (int e = threadIdx.x; e < k; e += kUpdThreads) s += p[e] * Ap[e];
  const double alpha = rz / wave_sum(s);
  double rzn = 0.0, rrn = 0.0;
  for (int e = threadIdx.x; e < k; e += kUpdThreads) {
    x[e] += alpha * p[e];
    const double re = r[e] - alpha * Ap[e];
    r[e] = re;
    rzn += re * (minv[e] * re);
    rrn += re * re;
  }
  rzn = wave_sum(rzn);
  rrn = wave_sum(rrn);
  const double beta = rzn / rz;
  for (int e = threadIdx.x; e < k; e += kUpdThreads) p[e] = minv[e] * r[e] + beta * p[e];
  if (threadIdx.x == 0) {
    o[PCG_RZ] = rzn;
    o[PCG_RR] = rrn;
    o[PCG_CONV] = rrn <= thr ? 1.0 : 0.0;
    o[PCG_ITERS] += 1.0;
  }
}

// true residual of x (Ax = A x already computed) and the un-standardized coefficients
__global__ __launch_bounds__(kUpdThreads) void pcg_residual_kernel(const double* __restrict__ b,
                                                                   const double* __restrict__ Ax,
                                                                   const double* __restrict__ aStd, int k, int nf,
                                                                   double* __restrict__ o) {
  if (o[PCG_STATUS] != 0.0 || o[PCG_BAD] != 0.0) return;  // wave-uniform
  const double bStd = o[PCG_BSTD];
  const double* x = o + PCG_STATE_WORDS;
  double* coef = o + PCG_STATE_WORDS + k;
  double s = 0.0;
  for (int e = threadIdx.x; e < k; e += kUpdThreads) {
    const double re = b[e] - Ax[e];
    s += re * re;
  }
  for (int j = threadIdx.x; j < nf; j += kUpdThreads) coef[j] = aStd[j] != 0.0 ? x[j] * bStd / aStd[j] : 0.0;
  s = wave_sum(s);
  if (threadIdx.x == 0) o[PCG_OK] = s <= 100.0 * o[PCG_THR] ? 1.0 : 0.0;
}

}  // namespace

void wls_assemble(const double* flat, int nf, int fit_intercept, double reg, double enet, int std_f, int std_l,
                  double* A, double* b, double* minv, double* aStd, double* aBar, double* lam, double* o,
                  hipStream_t st) {
  const int k = fit_intercept ? nf + 1 : nf;
  hipLaunchKernelGGL(wls_head_kernel, dim3(1), dim3(1), 0, st, flat, reg, enet, o);
  hipLaunchKernelGGL(wls_prep_kernel, dim3((nf + 255) / 256 > 0 ? (nf + 255) / 256 : 1), dim3(256), 0, st, flat, nf,
                     fit_intercept, std_f, std_l, aStd, aBar, lam, b, o);
  const int64_t T = (k + 31) / 32;
  hipLaunchKernelGGL(wls_dense_kernel, dim3((unsigned)(T * (T + 1) / 2)), dim3(256), 0, st, flat, nf, k, aStd,
                     aBar, lam, A, minv, o);
  DQ_HIP_CHECK(hipGetLastError());
}

void wls_pcg_init(const double* b, const double* minv, int k, double rtol, double* o, double* r, double* p,
                  hipStream_t st) {
  hipLaunchKernelGGL(pcg_init_kernel, dim3(1), dim3(kUpdThreads), 0, st, b, minv, k, rtol, o, r, p);
  DQ_HIP_CHECK(hipGetLastError());
}

void wls_pcg_chunk(const double* A, const double* b, const double* minv, const double* aStd, int k, int nf, int iters,
                   double* o, double* r, double* p, double* Ap, hipStream_t st) {
  const dim3 mv((k + 3) / 4);
  for (int i = 0; i < iters; ++i) {
    hipLaunchKernelGGL(pcg_matvec_kernel, mv, dim3(256), 0, st, A, p, Ap, k, o, 1);
    hipLaunchKernelGGL(pcg_update_kernel, dim3(1), dim3(kUpdThreads), 0, st, minv, Ap, k, o, r, p);
  }
  hipLaunchKernelGGL(pcg_matvec_kernel, mv, dim3(256), 0, st, A, o + PCG_STATE_WORDS, Ap, k, o, 0);
  hipLaunchKernelGGL(pcg_residual_kernel, dim3(1), dim3(kUpdThreads), 0, st, b, Ap, aStd, k, nf, o);
  DQ_HIP_CHECK(hipGetLastError());
}

}  // namespace dq4ml
