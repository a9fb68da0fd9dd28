// K6-small: the whole WeightedLeastSquares Cholesky branch for k <= 65 in ONE
// workgroup, on the device, straight from the all-reduced flat statistics — so a normal-equation
// fit enqueues gram -> all-reduce -> solve with no host round trip (asynchronous fits).  Same
// algebra as csrc/host/wls.cpp (standardize with population std, L2 on the standardized diagonal,
// intercept column [aBar, 1], Cholesky, un-standardize); anything but the plain SPD case is
// flagged in the status word and re-solved by the host driver (constant label, empty data,
// non-positive pivot).
#include <hip/hip_runtime.h>

#include "common.h"
#include "wls_small.h"

namespace dq4ml {

namespace {

constexpr int kMaxK = kWlsSmallMaxFeatures + 1;

__device__ __forceinline__ int64_t pku(int i, int j) { return i + (int64_t)j * (j + 1) / 2; }

__global__ __launch_bounds__(64) void wls_small_kernel(const double* __restrict__ flat, int nf, int fit_intercept,
                                                       double reg, double enet, int std_f, int std_l,
                                                       double* __restrict__ out) {
  __shared__ double A[kMaxK * kMaxK];
  __shared__ double b[kMaxK], x[kMaxK], aStd[kMaxK], aBar[kMaxK];
  __shared__ int bad;
  const int t = threadIdx.x;
  const int k = fit_intercept ? nf + 1 : nf;
  const double count = flat[0], wSum = flat[1], bSum = flat[3], bbSum = flat[4];
  const double* aSum = flat + 5;
  const double* abSum = flat + 5 + nf;
  const double* aa = flat + 5 + 2 * nf;
  // out = [coef(nf), intercept, status, count, wSum, wwSum, bSum, bbSum]
  if (t < 5) out[nf + 2 + t] = flat[t];
  const double rawBBar = wSum > 0.0 ? bSum / wSum : 0.0;
  const double rawBStd = wSum > 0.0 ? sqrt(fmax(bbSum / wSum - rawBBar * rawBBar, 0.0)) : 0.0;
  if (wSum <= 0.0 || rawBStd == 0.0) {  // host driver owns these semantics
    if (t == 0) out[nf + 1] = wSum <= 0.0 ? (count > 0 ? 1.0 : 2.0) : 3.0;
    return;
  }
  const double bStd = rawBStd;
  for (int j = t; j < nf; j += blockDim.x) {
    const double m = aSum[j] / wSum;
    const double s = sqrt(fmax(aa[pku(j, j)] / wSum - m * m, 0.0));
    aStd[j] = s;
    aBar[j] = s == 0.0 ? 0.0 : m / s;
    b[j] = s == 0.0 ? 0.0 : abSum[j] / wSum / (s * bStd);
  }
  if (t == 0) bad = 0;
  __syncthreads();
  const double eff_l2 = (1.0 - enet) * reg / bStd;
  for (int e = t; e < nf * nf; e += blockDim.x) {
    const int i = e / nf, j = e - (e / nf) * nf;
    const int lo = i < j ? i : j, hi = i < j ? j : i;
    const double den = aStd[i] * aStd[j];
    double v = den == 0.0 ? 0.0 : aa[pku(lo, hi)] / wSum / den;
    if (i == j) {
      double lam = eff_l2;
      if (!std_f) lam = aStd[j] != 0.0 ? lam / (aStd[j] * aStd[j]) : 0.0;
      if (!std_l) lam *= bStd;
      v += lam;
    }
    A[i * kMaxK + j] = v;
  }
  if (fit_intercept) {
    for (int i = t; i < nf; i += blockDim.x) {
      A[i * kMaxK + nf] = aBar[i];
      A[nf * kMaxK + i] = aBar[i];
    }
    if (t == 0) {
      A[nf * kMaxK + nf] = 1.0;
      b[nf] = rawBBar / bStd;
    }
  }
  __syncthreads();
  // right-looking Cholesky, lower factor in place
  for (int c = 0; c < k; ++c) {
    if (t == 0) {
      const double p = A[c * kMaxK + c];
      if (!(p > 0.0)) bad = 1;
      A[c * kMaxK + c] = sqrt(fmax(p, 1e-300));
    }
    __syncthreads();
    const double dc = A[c * kMaxK + c];
    for (int r = c + 1 + t; r < k; r += blockDim.x) A[r * kMaxK + c] /= dc;
    __syncthreads();
    const int m = k - c - 1;
    for (int e = t; e < m * m; e += blockDim.x) {
      const int r = c + 1 + e / m, s = c + 1 + e % m;
      if (s <= r) A[r * kMaxK + s] -= A[r * kMaxK + c] * A[s * kMaxK + c];
    }
    __syncthreads();
  }
  if (bad) {
    if (t == 0) out[nf + 1] = 7.0;  // not positive definite: host falls back (L-BFGS in auto mode)
    return;
  }
  // L y = b, then L^T x = y: wave 0 reduces each dot product, one barrier per row
  for (int r = 0; r < k; ++r) {
    if (t < 64) {
      double s = 0.0;
      for (int p = t; p < r; p += 64) s += A[r * kMaxK + p] * x[p];
      s = wave_sum_f64(s);
      if (t == 0) x[r] = (b[r] - s) / A[r * kMaxK + r];
    }
    __syncthreads();
  }
  for (int r = k - 1; r >= 0; --r) {
    if (t < 64) {
      double s = 0.0;
      for (int p = r + 1 + t; p < k; p += 64) s += A[p * kMaxK + r] * x[p];
      s = wave_sum_f64(s);
      if (t == 0) x[r] = (x[r] - s) / A[r * kMaxK + r];
    }
    __syncthreads();
  }
  for (int j = t; j < nf; j += blockDim.x) out[j] = aStd[j] != 0.0 ? x[j] * bStd / aStd[j] : 0.0;
  if (t == 0) {
    out[nf] = fit_intercept ? x[nf] * bStd : 0.0;
    out[nf + 1] = 0.0;
  }
}

__device__ __forceinline__ double rl(double v, int l) {  // v_readlane x2: lane l's double, wave-uniform
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), l);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
  return __hiloint2double(hi, lo);
}

// Register-resident variant for k <= KMAX <= 64 (one wave, no LDS, no barriers): lane r holds row r
// of the standardized system in a fully unrolled register array; the right-looking Cholesky, the
// forward substitution and the un-standardization exchange values with v_readlane (wave-uniform
// lane index = unrolled loop counter).  ~k^2 readlanes instead of ~3k barrier-separated LDS steps.
template <int KMAX>
__global__ __launch_bounds__(64) void wls_reg_kernel(const double* __restrict__ flat, int nf, int fit_intercept,
                                                    double reg, double enet, int std_f, int std_l,
                                                    double* __restrict__ out) {
  const int r = threadIdx.x;
  const int k = fit_intercept ? nf + 1 : nf;
  const double count = flat[0], wSum = flat[1], bSum = flat[3], bbSum = flat[4];
  const double* aSum = flat + 5;
  const double* abSum = flat + 5 + nf;
  const double* aa = flat + 5 + 2 * nf;
  if (r < 5) out[nf + 2 + r] = flat[r];
  const double rawBBar = wSum > 0.0 ? bSum / wSum : 0.0;
  const double rawBStd = wSum > 0.0 ? sqrt(fmax(bbSum / wSum - rawBBar * rawBBar, 0.0)) : 0.0;
  if (wSum <= 0.0 || rawBStd == 0.0) {
    if (r == 0) out[nf + 1] = wSum <= 0.0 ? (count > 0 ? 1.0 : 2.0) : 3.0;
    return;
  }
  const double bStd = rawBStd;
  // my feature's moments (lane r = feature r; the intercept lane r == nf has none)
  double myStd = 0.0, myBar = 0.0, myB = 0.0;
  if (r < nf) {
    const double m = aSum[r] / wSum;
    myStd = sqrt(fmax(aa[pku(r, r)] / wSum - m * m, 0.0));
    myBar = myStd == 0.0 ? 0.0 : m / myStd;
    myB = myStd == 0.0 ? 0.0 : abSum[r] / wSum / (myStd * bStd);
  } else if (r == nf && fit_intercept) {
    myB = rawBBar / bStd;
  }
  const double eff_l2 = (1.0 - enet) * reg / bStd;
  double a[KMAX];
#pragma unroll
  for (int s = 0; s < KMAX; ++s) {
    double v = 0.0;
    if (s < k && r < k) {
      const double sStd = rl(myStd, s), sBar = rl(myBar, s);
      if (r < nf && s < nf) {
        const int lo = r < s ? r : s, hi = r < s ? s : r;
        const double den = myStd * sStd;
        v = den == 0.0 ? 0.0 : aa[pku(lo, hi)] / wSum / den;
        if (r == s) {
          double lam = eff_l2;
          if (!std_f) lam = myStd != 0.0 ? lam / (myStd * myStd) : 0.0;
          if (!std_l) lam *= bStd;
          v += lam;
        }
      } else if (r < nf) {  // s == nf: intercept column
        v = myBar;
      } else if (s < nf) {  // r == nf: intercept row
        v = sBar;
      } else {
        v = 1.0;
      }
    }
    a[s] = v;
  }
  // Cholesky: column c of L lives in a[c] of lanes r >= c
  bool bad = false;
#pragma unroll
  for (int c = 0; c < KMAX; ++c) {
    if (c < k) {
      const double p = rl(a[c], c);
      bad |= !(p > 0.0);
      const double dc = sqrt(fmax(p, 1e-300));
      const double l = r == c ? dc : a[c] / dc;
      a[c] = l;
#pragma unroll
      for (int s = c + 1; s < KMAX; ++s)
        if (s < k) a[s] -= (r > c ? l : 0.0) * rl(l, s);
    }
  }
  if (bad) {
    if (r == 0) out[nf + 1] = 7.0;
    return;
  }
  // forward: L y = b (lane r keeps b_r, consumed column by column)
  double y = myB;
#pragma unroll
  for (int c = 0; c < KMAX; ++c) {
    if (c < k) {
      const double yc = rl(y, c) / rl(a[c], c);
      if (r == c) y = yc;
      else if (r > c) y -= a[c] * yc;
    }
  }
  // backward: L^T x = y; x_c = (y_c - sum_{r > c} L[r][c] x_r) / L[c][c]
  double x = 0.0;
#pragma unroll
  for (int c = KMAX - 1; c >= 0; --c) {
    if (c < k) {
      const double t = wave_sum_f64(r > c && r < k ? a[c] * x : 0.0);
      const double xc = (rl(y, c) - t) / rl(a[c], c);
      if (r == c) x = xc;
    }
  }
  if (r < nf) out[r] = myStd != 0.0 ? x * bStd / myStd : 0.0;
  const double xi = rl(x, nf < 64 ? nf : 63);
  if (r == 0) {
    out[nf] = fit_intercept ? xi * bStd : 0.0;
    out[nf + 1] = 0.0;
  }
}

}  // namespace

void wls_small(const double* flat, int nf, int fit_intercept, double reg, double enet, int std_f, int std_l,
               double* out, hipStream_t st) {
  if (nf < 1 || nf > kWlsSmallMaxFeatures) throw std::invalid_argument("wls_small: nf out of range");
  const int k = fit_intercept ? nf + 1 : nf;
  if (k <= 16) {
    hipLaunchKernelGGL(wls_reg_kernel<16>, dim3(1), dim3(64), 0, st, flat, nf, fit_intercept, reg, enet, std_f, std_l, out);
  } else if (k <= 40) {
    hipLaunchKernelGGL(wls_reg_kernel<40>, dim3(1), dim3(64), 0, st, flat, nf, fit_intercept, reg, enet, std_f, std_l, out);
  } else if (k <= 64) {
    hipLaunchKernelGGL(wls_reg_kernel<64>, dim3(1), dim3(64), 0, st, flat, nf, fit_intercept, reg, enet, std_f, std_l, out);
  } else {  // k == 65: LDS variant (one wave: every __syncthreads is a single-wave barrier)
    hipLaunchKernelGGL(wls_small_kernel, dim3(1), dim3(64), 0, st, flat, nf, fit_intercept, reg, enet, std_f, std_l,
                       out);
  }
  DQ_HIP_CHECK(hipGetLastError());
  return;
  hipLaunchKernelGGL(wls_small_kernel, dim3(1), dim3(64), 0, st, flat, nf, fit_intercept, reg, enet, std_f, std_l,
                     out);
  DQ_HIP_CHECK(hipGetLastError());
}

}  // namespace dq4ml
