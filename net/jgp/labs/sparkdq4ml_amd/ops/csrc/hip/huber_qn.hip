// LinearRegression(loss="huber") on the device, data-parallel, with no host read per evaluation:
// Breeze 0.13's LBFGSB -- the optimizer Spark 2.4 runs for the Huber loss (maxIter, memory 10,
// tol; every coordinate in [Double.MinValue, Double.MaxValue], sigma >= Double.MinPositiveValue;
// the estimator surface DataQuality4MachineLearningApp.java:120-123 configures) -- as a one-block
// control kernel over a state in HBM, the same algorithm as models/lbfgsb.py:
//
//  * direction: the generalized Cauchy point along the projected steepest-descent path
//    (breakpoints taken in ascending order by repeated arg-min, the piecewise quadratic of the
//    compact model B = theta I - W M W^T minimized segment by segment), then -- after the first
//    iteration -- the direct primal subspace minimization over the free variables (Breeze's
//    findAlpha always returns 1), projected onto the box;
//  * step: Breeze's StrongWolfeLineSearch (64 bracket / 64 zoom steps, cubic interpolation) from
//    t = 1 on the UNPROJECTED ray; the accepted point is projected and, when the projection moved
//    it, evaluated once more (CachedDiffFunction otherwise returns the last trial's values);
//  * memory: a pair is kept when |s.y| > 2.2e-16 y.y; theta = y.y / s.y; M = inv([[-D, L^T],
//    [L, theta S^T S]]) by Gauss-Jordan with partial pivoting (2m x 2m <= 20 x 20);
//  * convergence: ||P(x - g) - x||_inf <= 1e-5, max iterations, |f - max(last 20 f)| <= tol |f0|,
//    ||g|| <= max(tol |f|, 1e-8), a search failed twice (the first failure resets the memory).
//
// One evaluation = the Huber row pass over THIS rank's rows (rowops.hip huber_pass_dev: the trial
// point is read from HBM), its fold into red = [loss, W, g_b, g_sigma, g_x(d)], the caller's
// all-reduce of red (RCCL on the stream), then this kernel.  Everything is fixed-order: every rank
// reads the same reduced bytes and takes the same decisions.
#include <hip/hip_runtime.h>

#include "common.h"
#include "huber_qn.h"

#pragma clang fp contract(off)  // the scalar algebra mirrors models/lbfgsb.py's numpy expressions

namespace dq4ml {

namespace {

constexpr int kT = 256;
constexpr int kW = kT / 64;
constexpr int kM = 10;  // Spark's LBFGSB memory
constexpr int kFv = 20;
constexpr double kProjEps = 1e-5, kCurvEps = 2.2e-16, kDmax = 1.7976931348623157e308;
enum { kLsBracket = 0, kLsZoom = 1 };
enum { kPhInit = 0, kPhSearch = 1, kPhAccept = 2 };

struct HCtl {
  int act, phase, ls, bi, zi, iter, H, hh, nfv, failed_once, search_failed, why, overflow, nev;
  double alpha, value, init_value, theta, f0, d0, lo_t, lo_d, lo_f, hi_t, hi_d, hi_f;
  double fv[kFv];
};

struct HArgs {
  int d, dim, fit_icpt, max_iter, hist_cap;
  double tol;
  const double* sx;     // [d] feature std (0: a constant feature)
  const double* lam;    // [d] L2 weights of the theta-space coefficients
  const double* scale;  // [d] fp8 storage scales (or null)
  const double* shift;  // [d] storage shift (or null)
  double* work;
  double* trial;        // [d + 2] scaled effective coefficients | intercept | sigma
  const double* red;    // [4 + d] the all-reduced evaluation
  double* out;
};

// work layout (f64): HCtl | x | g | dir | xe | ge | xc | tb | dd | done | S[kM] | Y[kM] | M[2kM x 2kM]
struct HV {
  HCtl* C;
  double *x, *g, *dir, *xe, *ge, *xc, *tb, *dd, *done, *S, *Y, *M;
  double* Ms;  // M in LDS (the control kernel loads it once)
};

constexpr int64_t kCtlDoubles = (int64_t)((sizeof(HCtl) + 7) / 8);

__device__ __forceinline__ HV views(const HArgs& a) {
  HV v;
  double* p = a.work;
  v.C = reinterpret_cast<HCtl*>(p);
  p += kCtlDoubles;
  const int n = a.dim;
  v.x = p, p += n;
  v.g = p, p += n;
  v.dir = p, p += n;
  v.xe = p, p += n;
  v.ge = p, p += n;
  v.xc = p, p += n;
  v.tb = p, p += n;
  v.dd = p, p += n;
  v.done = p, p += n;
  v.S = p, p += (int64_t)kM * n;
  v.Y = p, p += (int64_t)kM * n;
  v.M = p;
  return v;
}

__device__ __forceinline__ double wsum(double v) {
#pragma unroll
  for (int s = 32; s > 0; s >>= 1) v += __shfl_xor(v, s);
  return v;
}

// every thread gets the block-wide sum (fixed order)
__device__ __forceinline__ double bsum(double v, double* red) {
  v = wsum(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  double s = 0.0;
  for (int i = 0; i < kW; ++i) s += red[i];
  return s;
}

__device__ __forceinline__ double lower_of(const HArgs& a, int i) { return i == a.dim - 1 ? 4.9406564584124654e-324 : -kDmax; }
__device__ __forceinline__ double upper_of(const HArgs&, int) { return kDmax; }
__device__ __forceinline__ double clampb(const HArgs& a, int i, double v) {
  const double lo = lower_of(a, i), hi = upper_of(a, i);
  return v < lo ? lo : (v > hi ? hi : v);
}

// W row i (2h entries: Y history, then theta S history; oldest first, as Breeze horzcats them)
__device__ __forceinline__ double wrow(const HV& v, const HCtl& C, int n, int i, int k) {
  const int h = C.hh;
  return k < h ? v.Y[(int64_t)k * n + i] : C.theta * v.S[(int64_t)(k - h) * n + i];
}

// the trial point of the next pass: theta -> scaled effective coefficients, intercept, sigma
__device__ __forceinline__ void write_trial(const HArgs& a, const double* th, double* red) {
  const int d = a.d;
  double sd = 0.0;
  for (int j = threadIdx.x; j < d; j += kT) {
    const double ce = a.sx[j] != 0.0 ? th[j] / a.sx[j] : 0.0;
    if (a.shift) sd += a.shift[j] * ce;
    a.trial[j] = a.scale ? ce * a.scale[j] : ce;
  }
  sd = a.shift ? bsum(sd, red) : 0.0;
  if (threadIdx.x == 0) {
    a.trial[d] = (a.fit_icpt ? th[d] : 0.0) + sd;
    a.trial[d + 1] = th[a.dim - 1];
  }
}

// the evaluation in red at xe -> (f, ge)
__device__ __forceinline__ double eval_of(const HArgs& a, const HV& v, double* red) {
  const int d = a.d;
  const double W = a.red[1];
  double reg = 0.0;
  for (int j = threadIdx.x; j < d; j += kT) {
    const double c = v.xe[j];
    const double gx = a.sx[j] != 0.0 ? a.red[4 + j] / a.sx[j] : 0.0;
    v.ge[j] = gx / W + a.lam[j] * c;
    reg += a.lam[j] * c * c;
  }
  reg = bsum(reg, red);
  if (threadIdx.x == 0) {
    if (a.fit_icpt) v.ge[d] = a.red[2] / W;
    v.ge[a.dim - 1] = a.red[3] / W;
  }
  __syncthreads();
  return a.red[0] / W + 0.5 * reg;
}

__device__ __forceinline__ int converged(const HArgs& a, const HV& v, const HCtl& C, double* red) {
  double pm = 0.0, gg = 0.0;
  for (int i = threadIdx.x; i < a.dim; i += kT) {
    pm = fmax(pm, fabs(clampb(a, i, v.x[i] - v.g[i]) - v.x[i]));
    gg += v.g[i] * v.g[i];
  }
  // max over the block (|.| >= 0: a max of non-negatives by shuffles, then LDS)
#pragma unroll
  for (int s = 32; s > 0; s >>= 1) pm = fmax(pm, __shfl_xor(pm, s));
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[kW + (threadIdx.x >> 6)] = pm;
  gg = bsum(gg, red);
  double pmax = 0.0;
  for (int i = 0; i < kW; ++i) pmax = fmax(pmax, red[kW + i]);
  if (pmax <= kProjEps) return 0;                                  // projected step converged
  if (a.max_iter >= 0 && C.iter >= a.max_iter) return 1;          // max iterations
  if (C.nfv >= 2) {
    double mx = -__builtin_inf();
    for (int i = kFv - C.nfv; i < kFv; ++i) mx = fmax(mx, C.fv[i]);
    if (fabs(C.value - mx) <= a.tol * fabs(C.init_value)) return 2;  // function values converged
  }
  if (sqrt(gg) <= fmax(a.tol * fabs(C.value), 1e-8)) return 3;   // gradient converged
  if (C.search_failed) return 4;
  return -1;
}

// Partial pivot of column `col` of an m-row matrix (row stride ld) in LDS, computed by EVERY wave
// (lanes read the rows, shuffle arg-max: the first strict maximum, as the one-thread scan): no
// block barrier, no serial LDS walk.
__device__ __forceinline__ int wave_pivot(const double* M, int ld, int m, int col) {
  const int lane = threadIdx.x & 63;
  double bv = -1.0;
  int bi = 0x7fffffff;
  if (lane >= col && lane < m) bv = fabs(M[lane * ld + col]), bi = lane;
#pragma unroll
  for (int s = 32; s > 0; s >>= 1) {
    const double ov = __shfl_xor(bv, s);
    const int oi = __shfl_xor(bi, s);
    if (ov > bv || (ov == bv && oi < bi)) bv = ov, bi = oi;
  }
  return bi;
}

// One Gauss-Jordan / forward-elimination step on [M | aug] (m rows, w columns, stride ld) at column
// col with partial pivoting, staged through registers: every thread reads the (swapped) values of
// its elements from the old matrix, one barrier, writes the new values, one barrier.  Each element
// gets the same operations in the same order as the one-thread elimination (pivot row normalized by
// its pivot / rows below eliminated by f = M'[r][col] / M'[col][col]).
template <bool GJ>
__device__ __forceinline__ void elim_step(double* M, int ld, int m, int w, int col) {
  const int piv = wave_pivot(M, ld, m, col);
  constexpr int kE = (2 * kM) * (4 * kM + 1) / kT + 1;  // elements per thread
  double nv[kE];
  const double pv = M[piv * ld + col];  // M'[col][col]
#pragma unroll
  for (int k = 0; k < kE; ++k) {
    const int e = threadIdx.x + k * kT;
    nv[k] = 0.0;
    if (e >= m * w) continue;
    const int r = e / w, c = e % w;
    const int src = r == col ? piv : (r == piv ? col : r);  // row r after the swap
    const double x = M[src * ld + c];
    if constexpr (GJ) {
      const double prow = M[piv * ld + c] / pv;  // the normalized pivot row
      if (r == col) {
        nv[k] = prow;
      } else {
        const double f = M[src * ld + col];
        nv[k] = f != 0.0 ? x - f * prow : x;
      }
    } else {
      if (r > col && c >= col) {
        const double f = M[src * ld + col] / pv;
        nv[k] = x - f * M[piv * ld + c];
      } else {
        nv[k] = x;
      }
    }
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < kE; ++k) {
    const int e = threadIdx.x + k * kT;
    if (e < m * w) M[(e / w) * ld + e % w] = nv[k];
  }
  __syncthreads();
}

// Wave-parallel dot products: wave w takes pairs w, w + kW, ... (lanes stride the n coordinates,
// then a fixed-order wave sum); `put(pair, value)` runs on lane 0.  No block barrier inside.
template <class F, class P>
__device__ __forceinline__ void wave_dots(int npairs, int n, F term, P put) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int q = wave; q < npairs; q += kW) {
    double s = 0.0;
    for (int e = lane; e < n; e += 64) s += term(q, e);
    s = wsum(s);
    if (lane == 0) put(q, s);
  }
}

// The same dot products for a short vector (n <= kShortN: Huber's dim is d + 2): one thread per
// pair walks i in order -- its loads are independent, so they are all in flight at once, where the
// wave-per-pair form pays one memory round trip (plus a wave reduction) per pair, serially per wave
// (~1 us each: 100 pairs per wave at m = 20 made M's rebuild ~45 us and the direction ~90 us).
constexpr int kShortN = 128;
template <class F, class P>
__device__ __forceinline__ void dots(int npairs, int n, F term, P put) {
  if (n <= kShortN) {
    for (int q = threadIdx.x; q < npairs; q += kT) {
      double s = 0.0;
      for (int e = 0; e < n; ++e) s += term(q, e);
      put(q, s);
    }
  } else {
    wave_dots(npairs, n, term, put);
  }
}

// M = inv(MM) of the current history: S^T Y and S^T S by wave dot products, then Gauss-Jordan
// with partial pivoting on [MM | I] in LDS, row operations spread over the block (each element
// takes the same operations in the same order as the one-thread elimination)
__device__ __forceinline__ void rebuild_m(const HArgs& a, const HV& v, HCtl& C, double* sh) {
  const int n = a.dim, h = C.hh, m2 = 2 * h, w2 = 2 * m2;
  double* A = sh;            // [h][h] S^T Y
  double* SS = sh + kM * kM;  // [h][h] S^T S
  double* T = sh + 2 * kM * kM;  // [m2][2 m2] augmented [MM | I]
  dots(h * h, n,
            [&](int q, int e) {
              const int i = q / h, j = q % h;
              return v.S[(int64_t)i * n + e] * v.Y[(int64_t)j * n + e];
            },
            [&](int q, double s) { A[(q / h) * kM + q % h] = s; });
  dots(h * h, n,
            [&](int q, int e) {
              const int i = q / h, j = q % h;
              return v.S[(int64_t)i * n + e] * v.S[(int64_t)j * n + e];
            },
            [&](int q, double s) { SS[(q / h) * kM + q % h] = s; });
  __syncthreads();
  for (int e = threadIdx.x; e < m2 * w2; e += kT) {
    const int r = e / w2, c = e % w2;
    double val;
    if (c >= m2) {
      val = (c - m2 == r) ? 1.0 : 0.0;
    } else if (r < h && c < h) {
      val = r == c ? -A[r * kM + r] : 0.0;  // -D
    } else if (r < h) {
      const int cc = c - h;                 // L^T: (r, cc) = L[cc][r] = A[cc][r] if cc > r
      val = cc > r ? A[cc * kM + r] : 0.0;
    } else if (c < h) {
      const int rr = r - h;                 // L: A[rr][c] if rr > c
      val = rr > c ? A[rr * kM + c] : 0.0;
    } else {
      val = SS[(r - h) * kM + (c - h)] * C.theta;
    }
    T[e] = val;
  }
  __syncthreads();
  for (int col = 0; col < m2; ++col) elim_step<true>(T, w2, m2, w2, col);
  for (int e = threadIdx.x; e < m2 * m2; e += kT) {
    const int r = e / m2, c = e % m2;
    v.M[r * (2 * kM) + c] = v.Ms[r * (2 * kM) + c] = T[r * w2 + m2 + c];
  }
  __syncthreads();
}

__device__ __forceinline__ double mget(const HV& v, int r, int c) { return v.Ms[r * (2 * kM) + c]; }


// generalized Cauchy point (xc) and c; then the direction into v.dir.  Returns g . dir.
__device__ __forceinline__ double direction(const HArgs& a, const HV& v, HCtl& C, double* red, double* sh) {
  const int n = a.dim, m2 = 2 * C.hh;
  __shared__ double p[2 * kM], c[2 * kM], tmp[2 * kM], tmp2[2 * kM], wb[2 * kM], rc3[3][2 * kM];
  __shared__ double s_f1, s_f2, s_dtmin, s_oldt;
  __shared__ int s_b;
  for (int i = threadIdx.x; i < n; i += kT) {
    const double gi = v.g[i];
    double ti, di = 0.0;
    if (gi == 0.0) {
      ti = kDmax;
    } else {
      ti = gi < 0.0 ? (v.x[i] - upper_of(a, i)) / gi : (v.x[i] - lower_of(a, i)) / gi;
      di = ti == 0.0 ? 0.0 : -gi;
    }
    v.tb[i] = ti;
    v.dd[i] = di;
    v.done[i] = 0.0;
    v.xc[i] = v.x[i];
  }
  __syncthreads();
  dots(m2, n, [&](int k, int i) { return wrow(v, C, n, i, k) * v.dd[i]; },
            [&](int k, double s) { p[k] = s, c[k] = 0.0; });
  double f1 = 0.0;
  for (int i = threadIdx.x; i < n; i += kT) f1 += v.g[i] * v.dd[i];
  f1 = bsum(f1, red);  // (its barriers also publish p)
  if (threadIdx.x < m2) {
    double mp = 0.0;
    for (int q = 0; q < m2; ++q) mp += mget(v, threadIdx.x, q) * p[q];
    tmp[threadIdx.x] = mp;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double pmp = 0.0;
    for (int r = 0; r < m2; ++r) pmp += p[r] * tmp[r];
    s_f1 = f1;
    s_f2 = -C.theta * f1 - pmp;
    s_dtmin = -(s_f1 / s_f2);
    s_oldt = 0.0;
  }
  __syncthreads();
  // breakpoints in ascending (t, index) order, from the first t != 0 (Breeze: sortWith, indexWhere)
  auto next_b = [&]() {
    double bt = __builtin_inf();
    int bi = 0x7fffffff;
    for (int i = threadIdx.x; i < n; i += kT) {
      const double ti = v.tb[i];
      if (v.done[i] == 0.0 && ti != 0.0 && (ti < bt || (ti == bt && i < bi))) bt = ti, bi = i;
    }
    // arg-min over the block: (t, i) lexicographic by shuffles, then wave leaders
#pragma unroll
    for (int s = 32; s > 0; s >>= 1) {
      const double ot = __shfl_xor(bt, s);
      const int oi = __shfl_xor(bi, s);
      if (ot < bt || (ot == bt && oi < bi)) bt = ot, bi = oi;
    }
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = bt, red[kW + (threadIdx.x >> 6)] = (double)bi;
    __syncthreads();
    if (threadIdx.x == 0) {
      double t0 = red[0];
      int i0 = (int)red[kW];
      for (int w = 1; w < kW; ++w) {
        const int iw = (int)red[kW + w];
        if (red[w] < t0 || (red[w] == t0 && iw < i0)) t0 = red[w], i0 = iw;
      }
      s_b = i0 < n ? i0 : -1;
    }
    __syncthreads();
  };
  next_b();
  for (;;) {
    const int b = s_b;
    if (b < 0) break;
    const double min_t = v.tb[b], delta_t = min_t - s_oldt;
    const bool go = delta_t <= s_dtmin;
    __syncthreads();  // every thread has read s_oldt / s_dtmin before they move
    if (!go) break;
    if (threadIdx.x < m2) {
      c[threadIdx.x] += p[threadIdx.x] * delta_t;
      wb[threadIdx.x] = wrow(v, C, n, b, threadIdx.x);
    }
    __syncthreads();
    if (threadIdx.x < m2) {  // rows of M c, M p, M wb
      double mc = 0.0, mp = 0.0, mw = 0.0;
      for (int q = 0; q < m2; ++q) {
        const double mv = mget(v, threadIdx.x, q);
        mc += mv * c[q];
        mp += mv * p[q];
        mw += mv * wb[q];
      }
      rc3[0][threadIdx.x] = mc, rc3[1][threadIdx.x] = mp, rc3[2][threadIdx.x] = mw;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      const double xb = v.dd[b] > 0.0 ? upper_of(a, b) : lower_of(a, b);
      v.xc[b] = xb;
      const double zb = xb - v.x[b];
      const double gb = v.g[b];
      double wMc = 0.0, wMp = 0.0, wMw = 0.0;
      for (int r = 0; r < m2; ++r) wMc += wb[r] * rc3[0][r], wMp += wb[r] * rc3[1][r], wMw += wb[r] * rc3[2][r];
      s_f1 += delta_t * s_f2 + gb * gb + C.theta * gb * zb - gb * wMc;
      s_f2 += -1.0 * C.theta * gb * gb - 2.0 * (gb * wMp) - gb * gb * wMw;
      for (int k = 0; k < m2; ++k) p[k] += wb[k] * gb;
      v.dd[b] = 0.0;
      v.done[b] = 1.0;
      s_dtmin = -s_f1 / s_f2;
      s_oldt = min_t;
    }
    __syncthreads();
    next_b();
  }
  if (threadIdx.x == 0) {
    if (s_dtmin < 0.0) s_dtmin = 0.0;  // math.max(dtMin, 0): a NaN stays NaN
    s_oldt += s_dtmin;
    for (int k = 0; k < m2; ++k) c[k] += p[k] * s_dtmin;
  }
  __syncthreads();
  const double oldt = s_oldt;
  for (int i = threadIdx.x; i < n; i += kT)
    if (v.done[i] == 0.0) v.xc[i] = clampb(a, i, v.x[i] + oldt * v.dd[i]);
    else v.xc[i] = clampb(a, i, v.xc[i]);
  __syncthreads();
  if (C.iter == 0) {  // iteration 0: the step to the Cauchy point itself
    double gd = 0.0;
    for (int i = threadIdx.x; i < n; i += kT) {
      const double di = v.xc[i] - v.x[i];
      v.dir[i] = di;
      gd += v.g[i] * di;
    }
    return bsum(gd, red);
  }
  // subspace minimization over the free variables of the Cauchy point
  const double it = 1.0 / C.theta;
  // Mc, then r = g + theta (xc - x) - W (M c) on the free variables (kept in v.tb)
  if (threadIdx.x < m2) {
    double s = 0.0;
    for (int q = 0; q < m2; ++q) s += mget(v, threadIdx.x, q) * c[q];
    tmp[threadIdx.x] = s;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += kT) {
    const bool fr = v.xc[i] != upper_of(a, i) && v.xc[i] != lower_of(a, i);
    double wmc = 0.0;
    for (int k = 0; k < m2; ++k) wmc += wrow(v, C, n, i, k) * tmp[k];
    v.tb[i] = fr ? (v.g[i] + (v.xc[i] - v.x[i]) * C.theta - wmc) : 0.0;
    v.done[i] = fr ? 1.0 : 0.0;
  }
  __syncthreads();
  // WZ rc and WZ WZ^T over the free variables
  double* N = sh;             // [m2][2 kM]
  double* NN = sh + 4 * kM * kM;  // [m2][2 kM + 1]: the subspace system and its right-hand side
  dots(m2, n, [&](int k, int i) { return v.done[i] != 0.0 ? wrow(v, C, n, i, k) * v.tb[i] : 0.0; },
            [&](int k, double s) { tmp2[k] = s; });
  dots(m2 * m2, n,
            [&](int q, int i) {
              const int k = q / m2, l = q % m2;
              return (l >= k && v.done[i] != 0.0) ? wrow(v, C, n, i, k) * wrow(v, C, n, i, l) : 0.0;
            },
            [&](int q, double s) {
              const int k = q / m2, l = q % m2;
              if (l >= k) N[k * kM * 2 + l] = s, N[l * kM * 2 + k] = s;
            });
  __syncthreads();
  // v = M (WZ rc);  N = I - M (WZ WZ^T) / theta;  v = N \ v (partial pivoting) on [N | v]
  constexpr int LA = 2 * kM + 1;  // row stride of the augmented system (v is column m2)
  __shared__ double vv[2 * kM];
  if (threadIdx.x < m2) {
    double s = 0.0;
    for (int q = 0; q < m2; ++q) s += mget(v, threadIdx.x, q) * tmp2[q];
    NN[threadIdx.x * LA + m2] = s;
  }
  for (int e = threadIdx.x; e < m2 * m2; e += kT) {
    const int r = e / m2, q = e % m2;
    double z = 0.0;
    for (int k = 0; k < m2; ++k) z += mget(v, r, k) * (N[k * kM * 2 + q] * it);
    NN[r * LA + q] = (r == q ? 1.0 : 0.0) - z;
  }
  __syncthreads();
  for (int col = 0; col < m2; ++col) elim_step<false>(NN, LA, m2, m2 + 1, col);
  if (threadIdx.x == 0) {
    for (int r = m2 - 1; r >= 0; --r) {
      double s = NN[r * LA + m2];
      for (int q = r + 1; q < m2; ++q) s -= NN[r * LA + q] * vv[q];
      vv[r] = s / NN[r * LA + r];
    }
  }
  __syncthreads();
  double gd = 0.0;
  for (int i = threadIdx.x; i < n; i += kT) {
    double sub = v.xc[i];
    if (v.done[i] != 0.0) {
      double wv = 0.0;
      for (int k = 0; k < m2; ++k) wv += wrow(v, C, n, i, k) * vv[k];
      const double du = -(v.tb[i] * it + wv * (it * it));
      sub = v.xc[i] + du;  // findAlpha: 1.0
    }
    const double di = clampb(a, i, sub) - v.x[i];
    v.dir[i] = di;
    gd += v.g[i] * di;
  }
  return bsum(gd, red);
}

__device__ __forceinline__ void record(const HArgs& a, HCtl& C) {
  if (C.H >= a.hist_cap) {
    C.overflow = 1;
    return;
  }
  a.out[a.d + 8 + C.H] = C.value;
  ++C.H;
}

// the output [coef(d) | intercept | scale | status | why | H | iter | nev | hist(H)]
__device__ __forceinline__ void finalize(const HArgs& a, const HV& v, HCtl& C) {
  const int d = a.d;
  for (int j = threadIdx.x; j < d; j += kT) a.out[j] = a.sx[j] != 0.0 ? v.x[j] / a.sx[j] : 0.0;
  if (threadIdx.x == 0) {
    a.out[d] = a.fit_icpt ? v.x[d] : 0.0;
    a.out[d + 1] = v.x[a.dim - 1];
    a.out[d + 2] = C.overflow ? 2.0 : 0.0;
    a.out[d + 3] = (double)C.why;
    a.out[d + 4] = (double)C.H;
    a.out[d + 5] = (double)C.iter;
    a.out[d + 6] = (double)C.nev;
    C.act = kHuberDone;
  }
}

// the trial at x + t dir (the line search evaluates the UNPROJECTED ray)
__device__ __forceinline__ void set_trial(const HArgs& a, const HV& v, HCtl& C, double t, double* red) {
  for (int i = threadIdx.x; i < a.dim; i += kT) v.xe[i] = v.x[i] + v.dir[i] * t;
  __syncthreads();
  write_trial(a, v.xe, red);
  if (threadIdx.x == 0) {
    C.alpha = t;
    C.act = kHuberEval;
  }
}

// a FirstOrderException (line search failed / zoom failed / non-descent direction)
__device__ __forceinline__ bool fail(const HArgs& a, HCtl& C) {
  if (!C.failed_once) {
    C.failed_once = 1;
    C.hh = 0;
    C.theta = 1.0;
  } else {
    C.search_failed = 1;
  }
  return true;
}

__device__ __forceinline__ double interp(double at, double ad, double af, double bt, double bd, double bf) {
  const double d1 = ad + bd - 3.0 * (af - bf) / (at - bt);
  const double d2 = sqrt(d1 * d1 - ad * bd);
  const double mul = bt - at;
  const double x = bt - mul * (bd + d2 - d1) / (bd - ad + 2.0 * d2);
  const double lb = at + 0.1 * mul, ub = at + 0.9 * mul;
  return x < lb ? lb : (x > ub ? ub : x);
}

}  // namespace

// ---- kernels ---------------------------------------------------------------------------------

namespace {

// state -> (convergence) -> the next direction and the first trial of its search, repeated while
// the direction fails (memory reset, then search failed)
__device__ __forceinline__ void next_search(const HArgs& a, const HV& v, HCtl& C, double* red, double* sh) {
  for (;;) {
    __syncthreads();
    if (threadIdx.x == 0) record(a, C);
    __syncthreads();
    const int why = converged(a, v, C, red);
    if (why >= 0 || C.overflow) {
      if (threadIdx.x == 0) C.why = why;
      __syncthreads();
      finalize(a, v, C);
      return;
    }
    const double d0 = direction(a, v, C, red, sh);
    if (d0 > 0.0) {  // "Line search invoked with non-descent direction"
      if (threadIdx.x == 0) fail(a, C);
      continue;      // the failed state is a state of the iterator: recorded, checked
    }
    if (threadIdx.x == 0) {
      C.phase = kPhSearch;
      C.ls = kLsBracket;
      C.bi = 0;
      C.f0 = C.value, C.d0 = d0;
      C.lo_t = 0.0, C.lo_d = d0, C.lo_f = C.value;
    }
    __syncthreads();
    set_trial(a, v, C, 1.0, red);
    return;
  }
}

__global__ __launch_bounds__(kT) void huber_qn_init_kernel(HArgs a) {
  __shared__ double red[2 * kW];
  __shared__ HCtl C;
  HV v = views(a);
  v.Ms = nullptr;
  if (threadIdx.x == 0) {
    HCtl z = {};
    z.act = kHuberEval;
    z.phase = kPhInit;
    z.theta = 1.0;
    C = z;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < a.dim; i += kT) v.x[i] = 1.0, v.xe[i] = 1.0;  // Spark: every coordinate 1
  __syncthreads();
  write_trial(a, v.xe, red);
  __syncthreads();
  if (threadIdx.x == 0) *v.C = C;
}

// The control step (one evaluation consumed): everything between the kernel's state load and store.
__device__ __forceinline__ void ctl_body(const HArgs& a, const HV& v, HCtl& C, double* red, double* sh) {
  const double f = eval_of(a, v, red);
  double dd = 0.0;
  for (int i = threadIdx.x; i < a.dim; i += kT) dd += v.ge[i] * v.dir[i];
  dd = bsum(dd, red);
  if (threadIdx.x == 0) ++C.nev;
  __syncthreads();
  const double c1 = 1e-4, c2 = 0.9;
  if (C.phase == kPhInit) {
    for (int i = threadIdx.x; i < a.dim; i += kT) v.g[i] = v.ge[i];
    if (threadIdx.x == 0) {
      C.value = f, C.init_value = f;
      C.fv[kFv - 1] = __builtin_inf();  // FunctionValuesConverged's initial info
      C.nfv = 1;
    }
    next_search(a, v, C, red, sh);
    __syncthreads();
    if (threadIdx.x == 0) *v.C = C;
    return;
  }
  bool accept = false, failed = false, same = false;
  double tnext = 0.0;
  if (C.phase == kPhAccept) {
    accept = true;  // (f, ge) at the projected accepted point
  } else if (threadIdx.x == 0) {
    const double t = C.alpha;
    if (C.ls == kLsBracket) {
      const int i = C.bi;
      if (!(f - f == 0.0)) {  // not finite: halve, same bracket step count
        tnext = t / 2.0;
      } else if (f > C.f0 + c1 * t * C.d0 || (f >= C.lo_f && i > 0)) {
        C.hi_t = t, C.hi_d = dd, C.hi_f = f;
        C.ls = kLsZoom, C.zi = 0;
      } else if (fabs(dd) <= c2 * fabs(C.d0)) {
        accept = true;
      } else if (dd >= 0.0) {
        C.hi_t = C.lo_t, C.hi_d = C.lo_d, C.hi_f = C.lo_f;
        C.lo_t = t, C.lo_d = dd, C.lo_f = f;
        C.ls = kLsZoom, C.zi = 0;
      } else {
        C.lo_t = t, C.lo_d = dd, C.lo_f = f;
        tnext = t * 1.5;
      }
      if (!accept && C.ls == kLsBracket && ++C.bi >= 64) failed = true;  // "Line search failed"
      if (!accept && !failed && C.ls == kLsZoom) {
        tnext = C.lo_t > C.hi_t ? interp(C.hi_t, C.hi_d, C.hi_f, C.lo_t, C.lo_d, C.lo_f)
                                : interp(C.lo_t, C.lo_d, C.lo_f, C.hi_t, C.hi_d, C.hi_f);
      }
    } else {  // zoom: the trial just evaluated
      if (f > C.f0 + c1 * t * C.d0 || f >= C.lo_f) {
        C.hi_t = t, C.hi_d = dd, C.hi_f = f;
      } else if (fabs(dd) <= c2 * fabs(C.d0)) {
        accept = true;
      } else {
        if (dd * (C.hi_t - C.lo_t) >= 0.0) C.hi_t = C.lo_t, C.hi_d = C.lo_d, C.hi_f = C.lo_f;
        C.lo_t = t, C.lo_d = dd, C.lo_f = f;
      }
      if (!accept && ++C.zi >= 64) failed = true;  // "Line search zoom failed"
      if (!accept && !failed)
        tnext = C.lo_t > C.hi_t ? interp(C.hi_t, C.hi_d, C.hi_f, C.lo_t, C.lo_d, C.lo_f)
                                : interp(C.lo_t, C.lo_d, C.lo_f, C.hi_t, C.hi_d, C.hi_f);
    }
    red[0] = accept ? 1.0 : 0.0, red[1] = failed ? 1.0 : 0.0, red[2] = tnext;
  }
  __syncthreads();
  if (C.phase != kPhAccept) {
    accept = red[0] != 0.0, failed = red[1] != 0.0, tnext = red[2];
  }
  __syncthreads();
  if (failed) {
    if (threadIdx.x == 0) fail(a, C);
    next_search(a, v, C, red, sh);
    __syncthreads();
    if (threadIdx.x == 0) *v.C = C;
    return;
  }
  if (!accept) {
    set_trial(a, v, C, tnext, red);
    __syncthreads();
    if (threadIdx.x == 0) *v.C = C;
    return;
  }
  if (C.phase == kPhSearch) {
    // the search's step: the projected point; unmoved by the projection it IS the last trial
    // (CachedDiffFunction hands back its values), else it is evaluated once more
    double moved = 0.0;
    for (int i = threadIdx.x; i < a.dim; i += kT) {
      const double p = clampb(a, i, v.xe[i]);
      if (p != v.xe[i]) moved += 1.0;
      v.xe[i] = p;
    }
    moved = bsum(moved, red);
    same = moved == 0.0;
    if (!same) {
      write_trial(a, v.xe, red);
      __syncthreads();
      if (threadIdx.x == 0) {
        C.phase = kPhAccept;
        C.act = kHuberEval;
        *v.C = C;
      }
      return;
    }
  }
  // accept: s = xe - x, y = ge - g into the memory (oldest dropped at kM), theta, M
  double sy = 0.0, yy = 0.0;
  for (int i = threadIdx.x; i < a.dim; i += kT) {
    const double s = v.xe[i] - v.x[i], y = v.ge[i] - v.g[i];
    sy += s * y;
    yy += y * y;
  }
  sy = bsum(sy, red);
  yy = bsum(yy, red);
  const int n = a.dim;
  if (kCurvEps * yy < fabs(sy)) {
    const int h = C.hh;
    if (h == kM) {  // drop the oldest pair
      for (int k = 0; k + 1 < kM; ++k)
        for (int i = threadIdx.x; i < n; i += kT) {
          v.S[(int64_t)k * n + i] = v.S[(int64_t)(k + 1) * n + i];
          v.Y[(int64_t)k * n + i] = v.Y[(int64_t)(k + 1) * n + i];
        }
      __syncthreads();
    }
    const int slot = h == kM ? kM - 1 : h;
    for (int i = threadIdx.x; i < n; i += kT) {
      v.S[(int64_t)slot * n + i] = v.xe[i] - v.x[i];
      v.Y[(int64_t)slot * n + i] = v.ge[i] - v.g[i];
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      C.hh = h == kM ? kM : h + 1;
      C.theta = yy / sy;
    }
    __syncthreads();
    rebuild_m(a, v, C, sh);
  }
  for (int i = threadIdx.x; i < n; i += kT) v.x[i] = v.xe[i], v.g[i] = v.ge[i];
  if (threadIdx.x == 0) {
    for (int i = 0; i < kFv - 1; ++i) C.fv[i] = C.fv[i + 1];
    C.fv[kFv - 1] = f;
    C.nfv = C.nfv < kFv ? C.nfv + 1 : kFv;
    C.value = f;
    ++C.iter;
    C.failed_once = 0;
  }
  next_search(a, v, C, red, sh);
  __syncthreads();
  if (threadIdx.x == 0) *v.C = C;
}

// Huber's short vectors (dim <= kShortN): the per-coordinate state and the s / y memory live in LDS
// for the call (one copy in, one copy out): every wrow / dot product / vector loop of the step then
// reads LDS instead of paying a memory round trip per access.
constexpr int kLocalDoubles = (9 + 2 * kM) * kShortN;

__global__ __launch_bounds__(kT) void huber_qn_ctl_kernel(HArgs a) {
  __shared__ double red[2 * kW];
  __shared__ double sh[4 * kM * kM + 2 * kM * 4 * kM];
  __shared__ double Ms[4 * kM * kM];
  __shared__ double vl[kLocalDoubles];
  __shared__ HCtl C;
  HV v = views(a);
  v.Ms = Ms;
  if (threadIdx.x == 0) C = *v.C;
  __syncthreads();
  if (C.act != kHuberEval) return;  // done: evaluations enqueued past the end
  for (int e = threadIdx.x; e < 4 * kM * kM; e += kT) Ms[e] = v.M[e];
  const int n = a.dim;
  const bool local = n <= kShortN;
  const int64_t nv = (9 + 2 * kM) * (int64_t)n;  // x .. done, S, Y: contiguous after the control block
  double* gv = v.x;
  if (local) {
    for (int64_t e = threadIdx.x; e < nv; e += kT) vl[e] = gv[e];
    HV w = v;
    double* p = vl;
    w.x = p, p += n;
    w.g = p, p += n;
    w.dir = p, p += n;
    w.xe = p, p += n;
    w.ge = p, p += n;
    w.xc = p, p += n;
    w.tb = p, p += n;
    w.dd = p, p += n;
    w.done = p, p += n;
    w.S = p, p += (int64_t)kM * n;
    w.Y = p;
    v = w;
  }
  __syncthreads();
  ctl_body(a, v, C, red, sh);
  __syncthreads();
  if (local)
    for (int64_t e = threadIdx.x; e < nv; e += kT) gv[e] = vl[e];
}

HArgs make(int d, bool fit_icpt, int max_iter, double tol, int hist_cap, const double* sx, const double* lam,
           const double* scale, const double* shift, double* work, double* trial, const double* red, double* out) {
  HArgs a{};
  a.d = d;
  a.dim = d + (fit_icpt ? 2 : 1);
  a.fit_icpt = fit_icpt ? 1 : 0;
  a.max_iter = max_iter;
  a.hist_cap = hist_cap;
  a.tol = tol;
  a.sx = sx, a.lam = lam, a.scale = scale, a.shift = shift;
  a.work = work, a.trial = trial, a.red = red, a.out = out;
  return a;
}

}  // namespace

int64_t huber_qn_work(int d, bool fit_icpt) {
  const int64_t n = d + (fit_icpt ? 2 : 1);
  return kCtlDoubles + 9 * n + 2 * (int64_t)kM * n + 4 * kM * kM;
}

int huber_qn_out(int d, int hist_cap) { return d + 8 + hist_cap; }

void huber_qn_init(int d, bool fit_icpt, int max_iter, double tol, int hist_cap, const double* sx, const double* lam,
                   const double* scale, const double* shift, double* work, double* trial, double* out,
                   hipStream_t st) {
  if (d < 1) throw std::invalid_argument("huber_qn: d must be >= 1");
  HArgs a = make(d, fit_icpt, max_iter, tol, hist_cap, sx, lam, scale, shift, work, trial, nullptr, out);
  hipLaunchKernelGGL(huber_qn_init_kernel, dim3(1), dim3(kT), 0, st, a);
  DQ_HIP_CHECK(hipGetLastError());
}

void huber_qn_ctl(int d, bool fit_icpt, int max_iter, double tol, int hist_cap, const double* sx, const double* lam,
                  const double* scale, const double* shift, double* work, double* trial, const double* red,
                  double* out, hipStream_t st) {
  HArgs a = make(d, fit_icpt, max_iter, tol, hist_cap, sx, lam, scale, shift, work, trial, red, out);
  hipLaunchKernelGGL(huber_qn_ctl_kernel, dim3(1), dim3(kT), 0, st, a);
  DQ_HIP_CHECK(hipGetLastError());
}

}  // namespace dq4ml
