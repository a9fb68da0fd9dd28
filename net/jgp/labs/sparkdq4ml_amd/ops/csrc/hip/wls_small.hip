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

// ---- K6-small, L1 branch: OWLQN in one wave ---------------------------------------------------
// The OWLQN branch of WeightedLeastSquares (regParam > 0, elasticNetParam > 0: the lab's own
// LinearRegression at DataQuality4MachineLearningApp.java:120-126) for k <= 64 * SLOTS, entirely
// on the device: standardize -> Breeze OWLQN (m = 10 two-loop on the pseudo-gradient, orthant
// projection, backtracking line search, FunctionValuesConverged over 20 values, one history reset
// on a failed search; csrc/host/solvers.cpp is the reference implementation) -> un-standardize.
// One wave: lane l owns vector elements l + 64 s; dot products are wave reductions, every scalar
// decision is computed redundantly by all lanes (uniform control flow, no barriers except around
// the dspmv broadcast of x); the packed standardized system and the m = 10 history live in LDS.
// out = [coef(nf), intercept, status, count, wSum, wwSum, bSum, bbSum, H, reason, history(H)]
// status: 0 ok | 1, 2, 3 label / weight short-circuits (host owns them) | 8 history capacity
// exceeded | 9 no L1 term (host: L-BFGS).  reason: 0 max iterations, 1 function values converged,
// 2 gradient converged, 3 search failed.
constexpr int kQnMem = 10;
constexpr int kQnFvals = 20;

template <int SLOTS>
__global__ __launch_bounds__(64) void wls_qn_kernel(const double* __restrict__ flat, int nf, int fit_intercept,
                                                    double reg, double enet, int std_f, int std_l, int max_iter,
                                                    double tol, int hist_cap, double* __restrict__ out) {
  constexpr int KMAX = 64 * SLOTS;
  __shared__ double Ap[KMAX * (KMAX + 1) / 2];
  __shared__ double xs[KMAX];
  __shared__ double Sh[kQnMem][KMAX], Yh[kQnMem][KMAX];
  __shared__ double sStd[KMAX], sBar[KMAX];
  const int lane = threadIdx.x;
  const int k = fit_intercept ? nf + 1 : nf;
  const double* aSum = flat + 5;
  const double* abSum = flat + 5 + nf;
  const double* aa = flat + 5 + 2 * nf;
  const double count = flat[0], wSum = flat[1], bSum = flat[3], bbSum = flat[4];
  if (lane < 5) out[nf + 2 + lane] = flat[lane];
  const double rawBBar = wSum > 0.0 ? bSum / wSum : 0.0;
  const double rawBStd = wSum > 0.0 ? sqrt(fmax(bbSum / wSum - rawBBar * rawBBar, 0.0)) : 0.0;
  if (wSum <= 0.0 || rawBStd == 0.0) {
    if (lane == 0) out[nf + 1] = wSum <= 0.0 ? (count > 0 ? 1.0 : 2.0) : 3.0;
    return;
  }
  const double bStd = rawBStd, bBar = rawBBar / bStd, bbBar = bbSum / wSum / (bStd * bStd);
  const double eff_reg = reg / bStd, eff_l1 = enet * eff_reg, eff_l2 = (1.0 - enet) * eff_reg;
  if (eff_l1 == 0.0) {
    if (lane == 0) out[nf + 1] = 9.0;
    return;
  }
  for (int i = lane; i < KMAX; i += 64) {
    double sd = 0.0, bar = 0.0;
    if (i < nf) {
      const double m = aSum[i] / wSum;
      sd = sqrt(fmax(aa[pku(i, i)] / wSum - m * m, 0.0));
      bar = sd == 0.0 ? 0.0 : m / sd;
    }
    sStd[i] = sd;
    sBar[i] = bar;
  }
  __syncthreads();
  for (int j = 0; j < k; ++j)
    for (int i = lane; i <= j; i += 64) {
      double v;
      if (j < nf) {
        const double den = sStd[i] * sStd[j];
        v = den == 0.0 ? 0.0 : aa[pku(i, j)] / wSum / den;
        if (i == j) {
          double lam = eff_l2;
          if (!std_f) lam = sStd[j] != 0.0 ? lam / (sStd[j] * sStd[j]) : 0.0;
          if (!std_l) lam *= bStd;
          v += lam;
        }
      } else {
        v = i < nf ? sBar[i] : 1.0;
      }
      Ap[pku(i, j)] = v;
    }
  double ab[SLOTS], l1[SLOTS], bar[SLOTS];
#pragma unroll
  for (int s = 0; s < SLOTS; ++s) {
    const int i = lane + 64 * s;
    const double sd = i < nf ? sStd[i] : 0.0;
    ab[s] = i < nf ? (sd == 0.0 ? 0.0 : abSum[i] / wSum / (sd * bStd)) : (i == nf && fit_intercept ? bBar : 0.0);
    l1[s] = i < k ? (std_f ? eff_l1 : (sd != 0.0 ? eff_l1 / sd : 0.0)) : 0.0;
    if (fit_intercept && i == nf) l1[s] = 0.0;
    bar[s] = i < nf ? sBar[i] : 0.0;
  }
  __syncthreads();

  auto dot = [&](const double* a, const double* b) {
    double v = 0.0;
#pragma unroll
    for (int s = 0; s < SLOTS; ++s) v += a[s] * b[s];
    return wave_sum_f64(v);
  };
  auto sgn = [](double v) { return v > 0.0 ? 1.0 : (v < 0.0 ? -1.0 : 0.0); };
  // f(x) = 1/2 bbBar - x.ab + 1/2 x^T A x, g = A x - ab; the intercept is re-set to
  // bBar - coef.aBar first (in place, as the host cost function writes into the optimizer's x)
  auto cost = [&](double* x, double* g) {
    if (fit_intercept) {
      double p = 0.0;
#pragma unroll
      for (int s = 0; s < SLOTS; ++s) p += x[s] * bar[s];
      const double dp = wave_sum_f64(p);
#pragma unroll
      for (int s = 0; s < SLOTS; ++s)
        if (lane + 64 * s == nf) x[s] = bBar - dp;
    }
#pragma unroll
    for (int s = 0; s < SLOTS; ++s) xs[lane + 64 * s] = x[s];
    __syncthreads();
    double aax[SLOTS];
#pragma unroll
    for (int s = 0; s < SLOTS; ++s) {
      const int i = lane + 64 * s;
      double acc = 0.0;
      if (i < k) {
        for (int j = 0; j < i; ++j) acc += Ap[pku(j, i)] * xs[j];
        for (int j = i; j < k; ++j) acc += Ap[pku(i, j)] * xs[j];
      }
      aax[s] = acc;
    }
    __syncthreads();
    const double v = 0.5 * bbBar - dot(ab, x) + 0.5 * dot(x, aax);
#pragma unroll
    for (int s = 0; s < SLOTS; ++s) g[s] = aax[s] - ab[s];
    return v;
  };
  auto adjust = [&](const double* x, const double* g, double v, double* ag) {
    double p = 0.0;
#pragma unroll
    for (int s = 0; s < SLOTS; ++s) {
      const double l = l1[s];
      ag[s] = g[s];
      if (l != 0.0) {
        p += fabs(l * x[s]);
        if (x[s] == 0.0) {
          const double dp = g[s] + l, dm = g[s] - l;
          ag[s] = dm > 0.0 ? dm : (dp < 0.0 ? dp : 0.0);
        } else {
          ag[s] = g[s] + sgn(x[s]) * l;
        }
      }
    }
    return v + wave_sum_f64(p);
  };
  double x[SLOTS], grad[SLOTS], agrad[SLOTS];
#pragma unroll
  for (int s = 0; s < SLOTS; ++s) x[s] = (fit_intercept && lane + 64 * s == k - 1) ? bBar : 0.0;
  double value = cost(x, grad);
  double adj = adjust(x, grad, value, agrad);
  const double init_adj = adj;
  double fv[kQnFvals];
#pragma unroll
  for (int i = 0; i < kQnFvals; ++i) fv[i] = 0.0;
  int nfv = 1;
  fv[kQnFvals - 1] = __builtin_inf();
  int iter = 0, hh = 0, head = 0, H = 0;
  bool search_failed = false, failed_once = false, overflow = false;
  auto record = [&](double v) {
    if (H >= hist_cap) {
      overflow = true;
      return;
    }
    if (lane == 0) out[nf + 9 + H] = v;
    ++H;
  };
  auto converged = [&]() -> int {
    if (max_iter >= 0 && iter >= max_iter) return 0;
    if (nfv >= 2) {
      double mx = -__builtin_inf();
#pragma unroll
      for (int i = 0; i < kQnFvals; ++i)
        if (i >= kQnFvals - nfv) mx = fmax(mx, fv[i]);
      if (fabs(adj - mx) <= tol * fabs(init_adj)) return 1;
    }
    if (sqrt(dot(agrad, agrad)) <= fmax(tol * fabs(value), 1e-8)) return 2;
    if (search_failed) return 3;
    return -1;
  };
  // projected step x + a d, then (adjusted value, adjusted directional derivative)
  auto take_step = [&](const double* d, double a, double* nx) {
#pragma unroll
    for (int s = 0; s < SLOTS; ++s) {
      nx[s] = x[s] + d[s] * a;
      const double orth = x[s] != 0.0 ? sgn(x[s]) : sgn(-agrad[s]);
      if (sgn(nx[s]) != orth) nx[s] = 0.0;
    }
  };
  auto phi = [&](const double* d, double a, double& dd) {
    double nx[SLOTS], g[SLOTS], ag[SLOTS];
    take_step(d, a, nx);
    const double v = cost(nx, g);
    const double av = adjust(nx, g, v, ag);
    dd = dot(ag, d);
    return av;
  };
  record(adj);
  int why = converged();
  while (why < 0 && !overflow) {
    bool fail = false;
    double d[SLOTS];
    // two-loop recursion on the pseudo-gradient (history in LDS, position i = (head + i) % m)
    {
      double diag = 1.0;
      if (hh > 0) {
        double sv[SLOTS], yv[SLOTS];
#pragma unroll
        for (int s = 0; s < SLOTS; ++s) sv[s] = Sh[head][lane + 64 * s], yv[s] = Yh[head][lane + 64 * s];
        const double sy = dot(sv, yv), yy = dot(yv, yv);
        if (sy < 0.0 || sy != sy) fail = true;
        diag = sy / yy;
      }
#pragma unroll
      for (int s = 0; s < SLOTS; ++s) d[s] = agrad[s];
      double as_[kQnMem], rho[kQnMem];
#pragma unroll
      for (int i = 0; i < kQnMem; ++i) {
        as_[i] = rho[i] = 0.0;
        if (i < hh) {
          const int p = (head + i) % kQnMem;
          double sv[SLOTS], yv[SLOTS];
#pragma unroll
          for (int s = 0; s < SLOTS; ++s) sv[s] = Sh[p][lane + 64 * s], yv[s] = Yh[p][lane + 64 * s];
          rho[i] = dot(sv, yv);
          as_[i] = dot(sv, d) / rho[i];
          if (as_[i] != as_[i]) fail = true;
#pragma unroll
          for (int s = 0; s < SLOTS; ++s) d[s] -= as_[i] * yv[s];
        }
      }
#pragma unroll
      for (int s = 0; s < SLOTS; ++s) d[s] *= diag;
#pragma unroll
      for (int i = kQnMem - 1; i >= 0; --i) {
        if (i < hh) {
          const int p = (head + i) % kQnMem;
          double sv[SLOTS], yv[SLOTS];
#pragma unroll
          for (int s = 0; s < SLOTS; ++s) sv[s] = Sh[p][lane + 64 * s], yv[s] = Yh[p][lane + 64 * s];
          const double beta = dot(yv, d) / rho[i];
#pragma unroll
          for (int s = 0; s < SLOTS; ++s) d[s] += (as_[i] - beta) * sv[s];
        }
      }
#pragma unroll
      for (int s = 0; s < SLOTS; ++s) {
        d[s] = -d[s];
        if (!(d[s] * agrad[s] < 0.0)) d[s] = 0.0;
      }
    }
    double alpha = 0.0;
    if (!fail) {  // backtracking line search (Breeze BacktrackingLineSearch as OWLQN configures it)
      const double initfval = adj;
      const double shrink = iter < 1 ? 0.1 : 0.5, grow = 2.1, c1 = 1e-4, c2 = 0.9;
      double initd, fd;
      phi(d, 0.0, initd);
      alpha = iter < 1 ? 0.5 / sqrt(dot(grad, grad)) : 1.0;
      double f = phi(d, alpha, fd);
      for (int it = 0;; ++it) {
        double mult;
        if (f > initfval + alpha * initd * c1) mult = shrink;
        else if (fd < c2 * initd) mult = grow;
        else if (fd > -c2 * initd) mult = shrink;
        else mult = 1.0;
        if (mult == 1.0) break;
        const double na = alpha * mult;
        if (it >= 20 || na < 1e-10 || na > 1e10) {
          fail = true;
          break;
        }
        alpha = na;
        f = phi(d, alpha, fd);
        if (it + 1 >= 20) break;
      }
    }
    if (!fail) {
      double nx[SLOTS], g[SLOTS], ag[SLOTS];
      take_step(d, alpha, nx);
      const double v = cost(nx, g);
      const double av = adjust(nx, g, v, ag);
      head = (head + kQnMem - 1) % kQnMem;
#pragma unroll
      for (int s = 0; s < SLOTS; ++s) {
        Sh[head][lane + 64 * s] = nx[s] - x[s];
        Yh[head][lane + 64 * s] = g[s] - grad[s];
        x[s] = nx[s], grad[s] = g[s], agrad[s] = ag[s];
      }
      hh = hh < kQnMem ? hh + 1 : kQnMem;
#pragma unroll
      for (int i = 0; i < kQnFvals - 1; ++i) fv[i] = fv[i + 1];
      fv[kQnFvals - 1] = v;
      nfv = nfv < kQnFvals ? nfv + 1 : kQnFvals;
      value = v;
      adj = av;
      ++iter;
      failed_once = false;
    } else if (!failed_once) {
      failed_once = true;
      hh = 0;
    } else {
      search_failed = true;
    }
    record(adj);
    why = converged();
  }
  if (overflow) {
    if (lane == 0) out[nf + 1] = 8.0;
    return;
  }
#pragma unroll
  for (int s = 0; s < SLOTS; ++s) {
    const int i = lane + 64 * s;
    if (i < nf) out[i] = sStd[i] != 0.0 ? x[s] * bStd / sStd[i] : 0.0;
    if (i == nf) out[nf] = fit_intercept ? x[s] * bStd : 0.0;
  }
  if (!fit_intercept && lane == 0) out[nf] = 0.0;
  if (lane == 0) {
    out[nf + 1] = 0.0;
    out[nf + 7] = (double)H;
    out[nf + 8] = (double)why;
  }
}

}  // namespace

void wls_qn_small(const double* flat, int nf, int fit_intercept, double reg, double enet, int std_f, int std_l,
                  int max_iter, double tol, int hist_cap, double* out, hipStream_t st) {
  const int k = fit_intercept ? nf + 1 : nf;
  if (nf < 1 || k > kWlsQnMaxK) throw std::invalid_argument("wls_qn_small: k out of range");
  if (hist_cap < 1) throw std::invalid_argument("wls_qn_small: hist_cap must be positive");
  if (k <= 64) hipLaunchKernelGGL(wls_qn_kernel<1>, dim3(1), dim3(64), 0, st, flat, nf, fit_intercept, reg, enet,
                                  std_f, std_l, max_iter, tol, hist_cap, out);
  else hipLaunchKernelGGL(wls_qn_kernel<2>, dim3(1), dim3(64), 0, st, flat, nf, fit_intercept, reg, enet, std_f,
                          std_l, max_iter, tol, hist_cap, out);
  DQ_HIP_CHECK(hipGetLastError());
}

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
