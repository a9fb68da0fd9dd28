// K6: the OWLQN branch of WeightedLeastSquares (regParam > 0, elasticNetParam > 0: the lab's own
// LinearRegression at DataQuality4MachineLearningApp.java:120-126) for
// 128 < k <= kWlsQnGridMaxK, entirely on the device: ONE grid launch runs standardize ->
// Breeze OWLQN -> un-standardize with no host round trip, so an L1 fit at any k the tall path
// reaches can be asynchronous.  Same algorithm and decisions as the one-wave wls_qn_kernel
// (wls_small.hip) and the host driver (csrc/host/solvers.cpp): m = 10 two-loop recursion on the
// pseudo-gradient, orthant projection, backtracking line search seeded with 0.5 / |g| on the first
// iteration, FunctionValuesConverged over 20 values, one history reset on a failed search.
//
// Work split (one block per CU, co-resident; grid-wide barriers by common.h grid_barrier):
//  * the dense standardized k x k system lives in HBM (134 MB at k = 4097 -- MALL resident);
//    block b owns rows [b R, b R + R) and computes their part of every A x (all threads stride
//    the columns of a row, several rows' loads in flight, the full trial point staged in LDS);
//  * every cost evaluation is ONE grid barrier: each block writes four partial sums (x.ab,
//    x.Ax, sum |l1 x|, adjusted-gradient . d, plus |ag|^2) to a parity-double-buffered slab, and
//    after the barrier EVERY block sums the slab in the same fixed order, so all blocks take
//    bitwise identical line-search decisions (uniform control flow across the grid: no block
//    can skip a barrier the others wait at);
//  * the two-loop recursion (31 dependent dot products over k) runs in block 0 alone, between
//    two barriers, from the history vectors in HBM (L2 resident), with its direction in
//    registers; the other blocks wait at the barrier.
// Loop passes are bounded by hist_cap (every pass records one objective value) and each line
// search by 21 evaluations, so the kernel terminates on any input (NaNs included).
// out = [coef(nf), intercept, status, count, wSum, wwSum, bSum, bbSum, H, reason, history(H)] --
// the wls_qn_small layout (ops/device.py, models/optim.py owlqn_result read both).
#include <hip/hip_runtime.h>

#include "common.h"
#include "wls_small.h"

namespace dq4ml {

namespace {

constexpr int kQT = 512;  // threads per block
constexpr int kQW = kQT / kWave;
constexpr int kMem = 10;
constexpr int kFvals = 20;
constexpr int kParts = 5;  // per-block partial sums of one evaluation

__device__ __forceinline__ int64_t pk(int i, int j) { return i + (int64_t)j * (j + 1) / 2; }

// every thread gets the block-wide sum (fixed order: waves 0..kQW-1)
__device__ __forceinline__ double block_sum(double v, double* red) {
  v = wave_sum_f64(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  double s = 0.0;
#pragma unroll
  for (int i = 0; i < kQW; ++i) s += red[i];
  return s;
}

__device__ __forceinline__ double sgn(double v) { return v > 0.0 ? 1.0 : (v < 0.0 ? -1.0 : 0.0); }

template <int SL>  // block 0's register slots: element t + kQT s, k <= kQT * SL
__global__ __launch_bounds__(kQT) void wls_qn_grid_kernel(const double* __restrict__ flat, int nf, int fit_intercept,
                                                          double reg, double enet, int std_f, int std_l, int max_iter,
                                                          double tol, int hist_cap, WlsQnWork w,
                                                          double* __restrict__ out) {
  unsigned gen = 0;
  auto grid_sync = [&]() { grid_barrier(w.gbar, gen, gridDim.x); };
  extern __shared__ double sm[];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int B = gridDim.x, b = blockIdx.x;
  const int k = fit_intercept ? nf + 1 : nf;
  const int R = (k + B - 1) / B, r0 = b * R < k ? b * R : k, r1 = r0 + R < k ? r0 + R : k;
  double* nxs = sm;            // [k] the evaluation's trial point
  double* red = sm + k;        // [kQW]
  double* rowp = red + kQW;    // [R][kQW] per-wave row sums
  const double* aSum = flat + 5;
  const double* abSum = flat + 5 + nf;
  const double* aa = flat + 5 + 2 * nf;
  const double count = flat[0], wSum = flat[1], bSum = flat[3], bbSum = flat[4];
  if (b == 0 && t < 5) out[nf + 2 + t] = flat[t];
  const double rawBBar = wSum > 0.0 ? bSum / wSum : 0.0;
  const double rawBStd = wSum > 0.0 ? sqrt(fmax(bbSum / wSum - rawBBar * rawBBar, 0.0)) : 0.0;
  if (wSum <= 0.0 || rawBStd == 0.0) {  // uniform across the grid: no barrier has been reached
    if (b == 0 && t == 0) out[nf + 1] = wSum <= 0.0 ? (count > 0 ? 1.0 : 2.0) : 3.0;
    return;
  }
  const double bStd = rawBStd, bBar = rawBBar / bStd, bbBar = bbSum / wSum / (bStd * bStd);
  const double eff_reg = reg / bStd, eff_l1 = enet * eff_reg, eff_l2 = (1.0 - enet) * eff_reg;
  if (eff_l1 == 0.0) {
    if (b == 0 && t == 0) out[nf + 1] = 9.0;
    return;
  }
  // ---- standardization: owners write the per-feature vectors, then their rows of A ----------
  for (int i = r0 + t; i < r1; i += kQT) {
    double sd = 0.0, bar = 0.0;
    if (i < nf) {
      const double m = aSum[i] / wSum;
      sd = sqrt(fmax(aa[pk(i, i)] / wSum - m * m, 0.0));
      bar = sd == 0.0 ? 0.0 : m / sd;
    }
    w.sstd[i] = sd;
    w.bar[i] = bar;
    w.ab[i] = i < nf ? (sd == 0.0 ? 0.0 : abSum[i] / wSum / (sd * bStd)) : bBar;  // i == nf: the intercept
    double l = std_f ? eff_l1 : (sd != 0.0 ? eff_l1 / sd : 0.0);
    if (i >= nf) l = 0.0;
    w.l1[i] = l;
  }
  __threadfence();
  grid_sync();
  for (int r = r0; r < r1; ++r)
    for (int j = t; j < k; j += kQT) {
      double v;
      if (r < nf && j < nf) {
        const double den = w.sstd[r] * w.sstd[j];
        v = den == 0.0 ? 0.0 : aa[r <= j ? pk(r, j) : pk(j, r)] / wSum / den;
        if (r == j) {
          double lam = eff_l2;
          if (!std_f) lam = w.sstd[j] != 0.0 ? lam / (w.sstd[j] * w.sstd[j]) : 0.0;
          if (!std_l) lam *= bStd;
          v += lam;
        }
      } else if (r == nf && j == nf) {
        v = 1.0;
      } else {
        v = w.bar[r < nf ? r : j];
      }
      w.A[(int64_t)r * k + j] = v;
    }
  __syncthreads();  // this block's rows of A are read by this block only

  // ---- one evaluation: trial point -> (value, adjusted value, ag . d, |ag|^2) ---------------
  // mode 0: the start point; 1: proj(x + alpha d).  Owners leave the trial point, gradient and
  // adjusted gradient of their rows in the candidate vectors (the accepted step's new state).
  int parity = 0;
  auto evaluate = [&](int mode, double alpha, double& value, double& adjv, double& dd, double& agag) {
    for (int j = t; j < k; j += kQT) {
      double v;
      if (mode == 0) {
        v = (fit_intercept && j == k - 1) ? bBar : 0.0;
      } else {
        const double xj = w.x[j];
        v = xj + w.d[j] * alpha;
        const double orth = xj != 0.0 ? sgn(xj) : sgn(-w.ag[j]);
        if (sgn(v) != orth) v = 0.0;
      }
      nxs[j] = v;
    }
    __syncthreads();
    if (fit_intercept) {  // intercept re-set to bBar - coef . aBar (in place, as the host cost does)
      double p = 0.0;
      for (int j = t; j < nf; j += kQT) p += nxs[j] * w.bar[j];
      const double dp = block_sum(p, red);
      if (t == 0) nxs[nf] = bBar - dp;
      __syncthreads();
    }
    // the block's rows of A x: all 512 threads stride the columns of one row (SL loads each,
    // rows unrolled so several rows' loads are in flight), per-wave sums to LDS, then thread rr
    // owns row r0 + rr
    const int nr = r1 - r0;
    for (int rr = 0; rr < nr; rr += 4) {  // four rows' loads in flight (rows past nr re-read row r0)
      const double* Ar[4];
      double acc[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int q = 0; q < 4; ++q) Ar[q] = w.A + (int64_t)(r0 + (rr + q < nr ? rr + q : 0)) * k;
#pragma unroll
      for (int s = 0; s < SL; ++s) {
        const int j = t + kQT * s;
        if (j < k) {
          const double xv = nxs[j];
#pragma unroll
          for (int q = 0; q < 4; ++q) acc[q] += Ar[q][j] * xv;
        }
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const double v = wave_sum_f64(acc[q]);
        if (lane == 0 && rr + q < nr) rowp[(rr + q) * kQW + wave] = v;
      }
    }
    __syncthreads();
    double part[kParts] = {0.0, 0.0, 0.0, 0.0, 0.0};  // x.ab, x.Ax, |l1 x|, ag.d, ag.ag
    if (t < nr) {
      const int r = r0 + t;
      double acc = 0.0;
#pragma unroll
      for (int i = 0; i < kQW; ++i) acc += rowp[t * kQW + i];
      const double xr = nxs[r], g = acc - w.ab[r], l = w.l1[r];
      double ag = g;
      if (l != 0.0) {
        if (xr == 0.0) {
          const double dp = g + l, dm = g - l;
          ag = dm > 0.0 ? dm : (dp < 0.0 ? dp : 0.0);
        } else {
          ag = g + sgn(xr) * l;
        }
      }
      part[0] = xr * w.ab[r];
      part[1] = xr * acc;
      part[2] = fabs(l * xr);
      part[3] = mode == 0 ? 0.0 : ag * w.d[r];
      part[4] = ag * ag;
      w.cx[r] = xr;
      w.cg[r] = g;
      w.cag[r] = ag;
    }
    // block partials (thread rr holds row r0 + rr's terms): fixed-order block sums
    double* slab = w.part + (int64_t)parity * B * kParts + (int64_t)b * kParts;
#pragma unroll
    for (int q = 0; q < kParts; ++q) {
      const double s = block_sum(part[q], red);
      if (t == 0) slab[q] = s;
    }
    __threadfence();
    grid_sync();
    const double* all = w.part + (int64_t)parity * B * kParts;
    double s[kParts] = {0.0, 0.0, 0.0, 0.0, 0.0};
    for (int i = 0; i < B; ++i)
#pragma unroll
      for (int q = 0; q < kParts; ++q) s[q] += all[(int64_t)i * kParts + q];
    parity ^= 1;
    value = 0.5 * bbBar - s[0] + 0.5 * s[1];
    adjv = value + s[2];
    dd = s[3];
    agag = s[4];
  };

  // block 0: accept the candidate (history pair, new state), all vectors in HBM
  int head = 0, hh = 0;
  auto accept = [&](bool push) {
    if (b != 0) return;
    if (push) head = (head + kMem - 1) % kMem;
    for (int j = t; j < k; j += kQT) {
      const double nx = w.cx[j], g = w.cg[j];
      if (push) {
        w.S[(int64_t)head * k + j] = nx - w.x[j];
        w.Y[(int64_t)head * k + j] = g - w.g[j];
      }
      w.x[j] = nx;
      w.g[j] = g;
      w.ag[j] = w.cag[j];
    }
    __threadfence();
    __syncthreads();
  };

  double value, adj, dd0, agag;
  evaluate(0, 0.0, value, adj, dd0, agag);
  accept(false);
  const double init_adj = adj;
  double fv[kFvals];
#pragma unroll
  for (int i = 0; i < kFvals; ++i) fv[i] = 0.0;
  int nfv = 1;
  fv[kFvals - 1] = __builtin_inf();
  int iter = 0, H = 0;
  bool search_failed = false, failed_once = false, overflow = false;
  auto record = [&](double v) {
    if (H >= hist_cap) {
      overflow = true;
      return;
    }
    if (b == 0 && t == 0) out[nf + 9 + H] = v;
    ++H;
  };
  auto converged = [&]() -> int {
    if (max_iter >= 0 && iter >= max_iter) return 0;
    if (nfv >= 2) {
      double mx = -__builtin_inf();
#pragma unroll
      for (int i = 0; i < kFvals; ++i)
        if (i >= kFvals - nfv) mx = fmax(mx, fv[i]);
      if (fabs(adj - mx) <= tol * fabs(init_adj)) return 1;
    }
    if (sqrt(agag) <= fmax(tol * fabs(value), 1e-8)) return 2;
    if (search_failed) return 3;
    return -1;
  };
  record(adj);
  int why = converged();
  int pass = 0;  // loop passes (uniform over the grid): w.scal is double-buffered by its parity
  while (why < 0 && !overflow) {
    // scal[4 * (pass & 1) ..]: block 0 writes this pass's direction scalars while a slow block may
    // still read the previous pass's -- a failed search runs no grid barrier between the read and
    // block 0's next write
    double* scal = w.scal + 4 * (pass & 1);
    ++pass;
    // ---- block 0: two-loop recursion -> direction d (HBM), ag . d, g . g ---------------------
    if (b == 0) {
      auto dot = [&](const double* p, const double* q) {
        double v = 0.0;
#pragma unroll
        for (int s = 0; s < SL; ++s) {
          const int j = t + kQT * s;
          if (j < k) v += p[j] * q[j];
        }
        return block_sum(v, red);
      };
      auto dotr = [&](const double* p, const double (&q)[SL]) {
        double v = 0.0;
#pragma unroll
        for (int s = 0; s < SL; ++s) {
          const int j = t + kQT * s;
          if (j < k) v += p[j] * q[s];
        }
        return block_sum(v, red);
      };
      bool fail = false;
      double diag = 1.0;
      if (hh > 0) {
        const double* sv = w.S + (int64_t)head * k;
        const double* yv = w.Y + (int64_t)head * k;
        const double sy = dot(sv, yv), yy = dot(yv, yv);
        if (sy < 0.0 || sy != sy) fail = true;
        diag = sy / yy;
      }
      double d[SL], agr[SL];
#pragma unroll
      for (int s = 0; s < SL; ++s) {
        const int j = t + kQT * s;
        agr[s] = j < k ? w.ag[j] : 0.0;
        d[s] = agr[s];
      }
      double as_[kMem], rho[kMem];  // static indices (unrolled, guarded): registers, not scratch
#pragma unroll
      for (int i = 0; i < kMem; ++i) {
        as_[i] = rho[i] = 0.0;
        if (i >= hh) continue;
        const int p = (head + i) % kMem;
        const double* sv = w.S + (int64_t)p * k;
        const double* yv = w.Y + (int64_t)p * k;
        rho[i] = dot(sv, yv);
        as_[i] = dotr(sv, d) / rho[i];
        if (as_[i] != as_[i]) fail = true;
#pragma unroll
        for (int s = 0; s < SL; ++s) {
          const int j = t + kQT * s;
          if (j < k) d[s] -= as_[i] * yv[j];
        }
      }
#pragma unroll
      for (int s = 0; s < SL; ++s) d[s] *= diag;
#pragma unroll
      for (int i = kMem - 1; i >= 0; --i) {
        if (i >= hh) continue;
        const int p = (head + i) % kMem;
        const double* sv = w.S + (int64_t)p * k;
        const double* yv = w.Y + (int64_t)p * k;
        const double beta = dotr(yv, d) / rho[i];
#pragma unroll
        for (int s = 0; s < SL; ++s) {
          const int j = t + kQT * s;
          if (j < k) d[s] += (as_[i] - beta) * sv[j];
        }
      }
      double pd = 0.0, pg = 0.0;
#pragma unroll
      for (int s = 0; s < SL; ++s) {
        const int j = t + kQT * s;
        d[s] = -d[s];
        if (!(d[s] * agr[s] < 0.0)) d[s] = 0.0;
        if (j < k) {
          w.d[j] = d[s];
          pd += agr[s] * d[s];
          const double g = w.g[j];
          pg += g * g;
        }
      }
      const double initd = block_sum(pd, red), gg = block_sum(pg, red);
      if (t == 0) {
        scal[0] = initd;
        scal[1] = gg;
        scal[2] = fail ? 1.0 : 0.0;
      }
    }
    __threadfence();
    grid_sync();
    const double initd = scal[0], gg = scal[1];
    bool fail = scal[2] != 0.0;
    double alpha = 0.0, nv = 0.0, nadj = 0.0, nagag = 0.0;
    if (!fail) {  // backtracking line search (Breeze BacktrackingLineSearch as OWLQN configures it)
      const double initfval = adj;
      const double shrink = iter < 1 ? 0.1 : 0.5, grow = 2.1, c1 = 1e-4, c2 = 0.9;
      alpha = iter < 1 ? 0.5 / sqrt(gg) : 1.0;
      double f, fd;
      evaluate(1, alpha, nv, f, fd, nagag);
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
        evaluate(1, alpha, nv, f, fd, nagag);
        if (it + 1 >= 20) break;
      }
      nadj = f;
    }
    if (!fail) {  // the last evaluation was at alpha: its candidates are the new state
      accept(true);
      hh = hh < kMem ? hh + 1 : kMem;
#pragma unroll
      for (int i = 0; i < kFvals - 1; ++i) fv[i] = fv[i + 1];
      fv[kFvals - 1] = nv;
      nfv = nfv < kFvals ? nfv + 1 : kFvals;
      value = nv;
      adj = nadj;
      agag = nagag;
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
  if (b != 0) return;
  if (overflow) {
    if (t == 0) out[nf + 1] = 8.0;
    return;
  }
  for (int i = t; i < k; i += kQT) {
    const double x = w.x[i];
    if (i < nf) out[i] = w.sstd[i] != 0.0 ? x * bStd / w.sstd[i] : 0.0;
    else out[nf] = x * bStd;  // intercept (i == nf only when fitting it)
  }
  if (t == 0) {
    if (!fit_intercept) out[nf] = 0.0;
    out[nf + 1] = grid_abandoned(w.gbar) ? 9.0 : 0.0;  // 9: not finished (the host path re-runs)
    out[nf + 7] = (double)H;
    out[nf + 8] = (double)why;
  }
}

// LDS bytes: trial point, block-sum scratch, per-wave row sums of the block's rows
size_t qn_lds(int k, int blocks) {
  const int R = (k + blocks - 1) / blocks;
  return (size_t)(k + kQW + (size_t)R * kQW) * sizeof(double);
}

}  // namespace

int64_t wls_qn_grid_work(int k, int blocks) {
  return (int64_t)k * k + (int64_t)k * (13 + 2 * kMem) + (int64_t)2 * blocks * kParts + 8 + 1;
}

int wls_qn_grid_blocks(int k) {
  int dev = 0, cus = 0, per = 0;
  DQ_HIP_CHECK(hipGetDevice(&dev));
  DQ_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  DQ_HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, wls_qn_grid_kernel<9>, kQT, qn_lds(k, cus)));
  if (per < 1) throw std::runtime_error("wls_qn_grid: the kernel does not fit a CU");
  const int nb = cus;        // one block per CU: co-resident (grid_barrier relies on it)
  const int rows_min = 4;    // at least a few rows per block
  const int want = (k + rows_min - 1) / rows_min;
  const int blocks = nb < want ? nb : (want < 1 ? 1 : want);
  // a thread owns one row of its block's A x: R = ceil(k / blocks) rows must fit kQT threads
  if ((k + blocks - 1) / blocks > kQT)
    throw std::runtime_error("wls_qn_grid: too few CUs for k (rows per block > threads per block)");
  return blocks;
}

void wls_qn_grid(const double* flat, int nf, int fit_intercept, double reg, double enet, int std_f, int std_l,
                 int max_iter, double tol, int hist_cap, double* work, int blocks, double* out, hipStream_t st) {
  const int k = fit_intercept ? nf + 1 : nf;
  if (nf < 1 || k > kWlsQnGridMaxK) throw std::invalid_argument("wls_qn_grid: k out of range");
  if (hist_cap < 1) throw std::invalid_argument("wls_qn_grid: hist_cap must be positive");
  // (the caller's block count comes from wls_qn_grid_blocks, cached per device and k: no occupancy
  // query on the launch path)
  if (blocks < 1 || (k + blocks - 1) / blocks > kQT)
    throw std::invalid_argument("wls_qn_grid: more rows per block than threads (each thread owns one row)");
  WlsQnWork w;
  double* p = work;
  auto take = [&](int64_t n) {
    double* q = p;
    p += n;
    return q;
  };
  w.A = take((int64_t)k * k);
  w.ab = take(k), w.l1 = take(k), w.bar = take(k), w.sstd = take(k);
  w.x = take(k), w.g = take(k), w.ag = take(k), w.d = take(k);
  w.cx = take(k), w.cg = take(k), w.cag = take(k);
  w.S = take((int64_t)kMem * k), w.Y = take((int64_t)kMem * k);
  w.part = take((int64_t)2 * blocks * kParts);
  w.scal = take(8);
  w.gbar = reinterpret_cast<unsigned*>(take(1));
  const size_t lds = qn_lds(k, blocks);
  void* args[] = {&flat, &nf, &fit_intercept, &reg, &enet, &std_f, &std_l, &max_iter, &tol, &hist_cap, &w, &out};
  const void* kern = k <= kQT       ? (const void*)wls_qn_grid_kernel<1>
                     : k <= 2 * kQT ? (const void*)wls_qn_grid_kernel<2>
                     : k <= 4 * kQT ? (const void*)wls_qn_grid_kernel<4>
                                    : (const void*)wls_qn_grid_kernel<9>;
  // a plain launch of a co-resident grid (at most one block per CU, wls_qn_grid_blocks) with its
  // own barrier
  DQ_HIP_CHECK(hipMemsetAsync(w.gbar, 0, 2 * sizeof(unsigned), st));
  DQ_HIP_CHECK(hipLaunchKernel(kern, dim3(blocks), dim3(kQT), args, (unsigned)lds, st));
}

}  // namespace dq4ml
