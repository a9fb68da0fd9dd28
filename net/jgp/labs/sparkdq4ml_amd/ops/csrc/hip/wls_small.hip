// K6-small: the whole WeightedLeastSquares Cholesky branch for k <= 65 in ONE
// workgroup, on the device, straight from the all-reduced flat statistics — so a normal-equation
// fit enqueues gram -> all-reduce -> solve with no host round trip (asynchronous fits).  Same
// algebra as csrc/host/wls.cpp (standardize with population std, L2 on the standardized diagonal,
// intercept column [aBar, 1], solve, un-standardize); anything but the plain SPD case is flagged
// in the status word and re-solved by the host driver (constant label, empty data, non-positive
// pivot).
//
// Latency design.  The solve sits on the critical path of every small-shard fit, and with one
// wave per SIMD nothing hides latency: the cost is the instruction count per elimination step
// times the dependent-issue latency.  So:
//  * Gauss-Jordan on the full system [A | b] (no back substitution: x_r = b_r / D_r at the end,
//    fully parallel).  Without pivoting it meets the same pivots as LDLᵀ / Cholesky; a pivot
//    <= 0 = not SPD, the case in which dppsv fails too.
//  * 256 threads; thread t OWNS elements e = t + 256 i of the (k x (k+1)) system and keeps them in
//    registers for the whole solve; the slot count is a template parameter sized for the actual k.
//  * ONE barrier per step and no branches in it: two parity copies of the system in LDS; step c
//    reads the pivot, column c and row c of parity c & 1 and every slot writes its new value to
//    the other parity (distinct addresses, coalesced).  The matrix stores 0 on its diagonal (the
//    diagonal lives in a separate vector per parity), which makes the pivot row's update a no-op
//    without a select.  Dead columns (< c) are not zeroed, so only each step's pivot is kept.
//  History (k = 33): unrolled per-lane register rows + v_readlane: ~19k straight-line
//  instructions, I-cache bound, 51 us; LDS read-modify-write LDLᵀ + back substitution: 34 us;
//  register-owned LDLᵀ sized for k = 65 (9 slots / thread whatever k): 31 us; Gauss-Jordan with
//  exec-masked publication of the next column / row: 29 us (every skipped masked store is a taken
//  s_cbranch_execz).
#include <hip/hip_runtime.h>

#include "common.h"
#include "wls_small.h"

namespace dq4ml {

namespace {

constexpr int kMaxK = kWlsSmallMaxFeatures + 1;
constexpr int kThreads = 256;

// scripts/wls_probe.hip builds this file with DQ4ML_WLS_PROBE: per-phase s_memtime stamps
#ifdef DQ4ML_WLS_PROBE
__device__ long long* g_wls_probe;
#define WLS_STAMP(i) \
  if (threadIdx.x == 0) g_wls_probe[i] = (long long)__builtin_amdgcn_s_memtime()
#else
#define WLS_STAMP(i)
#endif

__device__ __forceinline__ int64_t pku(int i, int j) { return i + (int64_t)j * (j + 1) / 2; }

template <int KMAX>
__global__ __launch_bounds__(kThreads) void wls_gj_kernel(const double* __restrict__ flat, int nf, int fit_intercept,
                                                         double reg, double enet, int std_f, int std_l,
                                                         double* __restrict__ out) {
  constexpr int kW = KMAX + 1;                                 // row width incl. the RHS column
  constexpr int kPer = (KMAX * kW + kThreads - 1) / kThreads;  // owned slots per thread
  constexpr int kBuf = KMAX * kW + KMAX + kThreads;            // [matrix | diagonal | trash] per parity
  __shared__ double M[2 * kBuf];
  __shared__ double aStd[KMAX], aBar[KMAX], iStd[KMAX], pivots[KMAX];
  __shared__ int bad;
  WLS_STAMP(0);
  const int t = threadIdx.x;
  const int k = fit_intercept ? nf + 1 : nf;
  const double* aSum = flat + 5;
  const double* abSum = flat + 5 + nf;
  const double* aa = flat + 5 + 2 * nf;
  // owned slots (r, s) of the k x (k+1) system (row stride kW) and their raw statistics:
  // branch-free clamped addresses, so every global load is in flight at once
  int er[kPer], es[kPer], woff[kPer];
  double a[kPer];
  const int w = k + 1;
#pragma unroll
  for (int i = 0; i < kPer; ++i) {
    const int e = t + kThreads * i;
    const int r = e / w, s = e - (e / w) * w;
    const bool live = r < k;
    er[i] = live ? r : 0;
    es[i] = live ? (s == k ? KMAX : s) : 0;  // the RHS lives in column KMAX
    // write target: the diagonal goes to the parity's diagonal vector (the matrix keeps 0 there),
    // dead slots to the thread's private trash double
    woff[i] = !live ? KMAX * kW + KMAX + t : (r == s ? KMAX * kW + r : r * kW + es[i]);
    const bool feat = live && r < nf && s < nf;
    const int lo = s < r ? s : r, hi = s < r ? r : s;
    const bool rhs = live && r < nf && s == k;
    a[i] = feat ? aa[pku(lo, hi)] : (rhs ? abSum[r] : 0.0);
    if (!live) er[i] = -1;
  }
  const int tf = t < nf ? t : 0;
  const double my_sum = aSum[tf], my_diag = aa[pku(tf, tf)];
  const double count = flat[0], wSum = flat[1], bSum = flat[3], bbSum = flat[4];
  // out = [coef(nf), intercept, status, count, wSum, wwSum, bSum, bbSum]
  if (t < 5) out[nf + 2 + t] = flat[t];
  const double rawBBar = wSum > 0.0 ? bSum / wSum : 0.0;
  const double rawBStd = wSum > 0.0 ? sqrt(fmax(bbSum / wSum - rawBBar * rawBBar, 0.0)) : 0.0;
  if (wSum <= 0.0 || rawBStd == 0.0) {  // host driver owns these semantics
    if (t == 0) out[nf + 1] = wSum <= 0.0 ? (count > 0 ? 1.0 : 2.0) : 3.0;
    return;
  }
  const double bStd = rawBStd;
  // divisions (not reciprocal multiplies) exactly as wls.cpp / Spark: a constant feature must get
  // an exactly-zero std, so the zero-pivot / singular fallback triggers identically
  if (t < nf) {
    const double m = my_sum / wSum;
    const double sd = sqrt(fmax(my_diag / wSum - m * m, 0.0));
    aStd[t] = sd;
    aBar[t] = sd == 0.0 ? 0.0 : m / sd;
    iStd[t] = sd == 0.0 ? 0.0 : 1.0 / (sd * sqrt(wSum));  // A_rs = aa_rs * iStd_r * iStd_s
  }
  if (t == 0) bad = 0;
  __syncthreads();
  WLS_STAMP(1);
  // standardized system into parity 0; the matrix diagonal is 0 in both parities
  const double eff_l2 = (1.0 - enet) * reg / bStd;
#pragma unroll
  for (int i = 0; i < kPer; ++i) {
    const int r = er[i], s = es[i];
    if (r < 0) continue;
    double v;
    if (s == KMAX) {  // RHS
      v = r < nf ? (aStd[r] == 0.0 ? 0.0 : a[i] / wSum / (aStd[r] * bStd)) : rawBBar / bStd;
    } else if (r < nf && s < nf) {
      // aa / wSum / (std_r std_s) as two multiplies (within an ulp of wls.cpp; exact zeros kept)
      v = a[i] * iStd[r] * iStd[s];
      if (r == s) {
        double lam = eff_l2;
        if (!std_f) lam = aStd[s] != 0.0 ? lam / (aStd[s] * aStd[s]) : 0.0;
        if (!std_l) lam *= bStd;
        v += lam;
      }
    } else if (r == nf && s == nf) {  // intercept diagonal
      v = 1.0;
    } else {  // intercept row / column
      v = aBar[r < nf ? r : s];
    }
    a[i] = v;
    M[woff[i]] = v;
    if (r == s) {
      M[r * kW + r] = 0.0;
      M[kBuf + r * kW + r] = 0.0;
    }
  }
  __syncthreads();
  WLS_STAMP(2);
  // Gauss-Jordan: step c reads parity c & 1 (pivot = diagonal vector[c], column c, row c) and
  // writes every owned slot to the other parity.  With 0 stored on the matrix diagonal, the pivot
  // row's update (uses M[c][c]) and the dead column's (uses M[c][c]) are no-ops — no selects, no
  // branches, one barrier per step.
  auto step = [&](const int c, const double* __restrict__ R, double* __restrict__ Wb) {
    const double p = R[KMAX * kW + c];
    double cv[kPer], rv[kPer];
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      cv[i] = R[(er[i] < 0 ? 0 : er[i]) * kW + c];
      rv[i] = R[c * kW + es[i]];
    }
    // 1/p: v_rcp_f64 + two Newton steps (p is a normal positive number when it is used)
    double ip = __builtin_amdgcn_rcp(p);
    ip = ip * (2.0 - p * ip);
    ip = ip * (2.0 - p * ip);
    if (t == 0) {
      if (!(p > 0.0)) bad = 1;
      pivots[c] = p;  // the diagonal vector keeps drifting after its step (dead columns are not zeroed)
    }
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      a[i] -= cv[i] * ip * rv[i];
      Wb[woff[i]] = a[i];
    }
    __syncthreads();
  };
  // unrolled by two: the parity buffers are compile-time bases (immediate LDS offsets)
  int c = 0;
  for (; c + 1 < k; c += 2) {
    step(c, M, M + kBuf);
    step(c + 1, M + kBuf, M);
  }
  if (c < k) step(c, M, M + kBuf);
  WLS_STAMP(3);
  if (bad) {
    if (t == 0) out[nf + 1] = 7.0;  // not positive definite: host falls back (L-BFGS in auto mode)
    return;
  }
  // x_r = b_r / D_r (the RHS owners), un-standardized
#pragma unroll
  for (int i = 0; i < kPer; ++i) {
    const int r = er[i];
    if (r >= 0 && es[i] == KMAX) {
      const double x = a[i] / pivots[r];
      if (r < nf) out[r] = aStd[r] != 0.0 ? x * bStd / aStd[r] : 0.0;
      else out[nf] = x * bStd;  // intercept (r == nf only when fitting it)
    }
  }
  if (t == 0) {
    if (!fit_intercept) out[nf] = 0.0;
    out[nf + 1] = 0.0;
  }
  WLS_STAMP(4);
}

}  // namespace

void wls_small(const double* flat, int nf, int fit_intercept, double reg, double enet, int std_f, int std_l,
               double* out, hipStream_t st) {
  if (nf < 1 || nf > kWlsSmallMaxFeatures) throw std::invalid_argument("wls_small: nf out of range");
  const int k = fit_intercept ? nf + 1 : nf;
#define DQ_WLS_LAUNCH(KM)                                                                                     \
  hipLaunchKernelGGL(wls_gj_kernel<KM>, dim3(1), dim3(kThreads), 0, st, flat, nf, fit_intercept, reg, enet, std_f, \
                     std_l, out)
  if (k <= 16) DQ_WLS_LAUNCH(16);
  else if (k <= 33) DQ_WLS_LAUNCH(33);
  else if (k <= 48) DQ_WLS_LAUNCH(48);
  else DQ_WLS_LAUNCH(kMaxK);
#undef DQ_WLS_LAUNCH
  DQ_HIP_CHECK(hipGetLastError());
}

}  // namespace dq4ml
