// K9 on the device end to end: the squared-loss l-bfgs / OWLQN fit of LinearRegression
// (solver="l-bfgs", or "auto" with numFeatures > 4096: DataQuality4MachineLearningApp.java:120-126,
// SURVEY.md S13/K9) as ONE grid launch over the HBM-resident wide tiles.  Round 3 ran every
// cost evaluation as two streaming kernels (margins, then column sums: X read twice) and steered
// the Breeze line search from the host (one D2H per evaluation), so an l-bfgs fit could never be
// asynchronous.  Here:
//
//  * the standardization constants come from the summarizer head ([count, W, W2, Σwy, Σwy²,
//    Σwx, Σwx²], all on the device), so nothing is read back before the optimizer starts;
//  * ONE fused pass per evaluation: block b takes the 16-row (bf16) / 32-row (fp8) fragment
//    units u = b, b + B, ...; its 8 waves split the unit's feature tiles (wave w: tiles w, w + 8,
//    ...), sum the rows' partial margins in LDS, form v_r = w_r diff_r, then re-read the SAME
//    tiles (last-read first, so the tail still sits in the XCD's L2 and the rest in the 256 MiB
//    MALL: 256 units of 512 KiB are in flight between the two reads) and add v_r x_rj into
//    per-lane f64 column accumulators that live in registers for the whole pass -- one HBM read
//    of X per evaluation instead of two;
//  * the Breeze control flow of models/qn_device.py (itself the native driver's line for line)
//    runs uniformly in every block: the two-loop recursion and the history push in block 0 between
//    grid barriers, every line-search decision from scalars each block sums from the same
//    per-block partial slabs in the same order (bitwise identical decisions, no block can skip a
//    barrier the others wait at);
//  * the result ([coef, intercept, status, reason, H, head, history]) is un-standardized in the
//    kernel: an asynchronous fit enqueues the summarizer pass plus this launch and returns.
//
// Per evaluation: 2 grid barriers, a redundant O(d) trial-point build per block (the f32
// effective coefficients go to LDS), a distributed fixed-order fold of the per-block column slabs.
// Loop passes are bounded by hist_cap and every line search by 21 (backtracking) or 20 (strong
// Wolfe) evaluations, so the kernel terminates on any input.
#include <hip/hip_runtime.h>

#include "common.h"
#include "lsq.h"

#pragma clang fp contract(off)  // the scalar algebra mirrors the host's numpy / torch expressions

namespace dq4ml {

namespace {

constexpr int kT = 512;
constexpr int kW = kT / kWave;
constexpr int kMem = 10;
constexpr int kFv = 20;
constexpr int kDParts = 4;  // per-block partials of an evaluation: x.(regw x), Σ|l1 x|, dir . g, g . g


__device__ __forceinline__ double block_sum(double v, double* red) {
  v = wave_sum_f64(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  double s = 0.0;
#pragma unroll
  for (int i = 0; i < kW; ++i) s += red[i];
  return s;
}

__device__ __forceinline__ double sgn(double v) { return v > 0.0 ? 1.0 : (v < 0.0 ? -1.0 : 0.0); }

template <int L>
__device__ __forceinline__ void unpack(const u32x4 q, float* x) {
  if constexpr (L == 3) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int v = (int)q[k];
      x[4 * k + 0] = __builtin_amdgcn_cvt_f32_fp8(v, 0);
      x[4 * k + 1] = __builtin_amdgcn_cvt_f32_fp8(v, 1);
      x[4 * k + 2] = __builtin_amdgcn_cvt_f32_fp8(v, 2);
      x[4 * k + 3] = __builtin_amdgcn_cvt_f32_fp8(v, 3);
    }
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      x[2 * j] = __uint_as_float(q[j] << 16);
      x[2 * j + 1] = __uint_as_float(q[j] & 0xffff0000u);
    }
  }
}

// row of element e of the 16-byte fragment of lane half h in unit `sub` of superstep s (lsq.hip)
template <int L>
__device__ __forceinline__ int64_t frag_row(int64_t s, int sub, int h, int e) {
  if constexpr (L == 2) return s * 64 + 16 * sub + 8 * h + e;
  else return s * 64 + 16 * (2 * sub + (e >> 3)) + 8 * h + (e & 7);
}

struct Eval {
  double v, adj, dd, gg;
};

// ---- optimizer control (thread 0 of each block; scalar code, state in LDS) ------------------
enum { kActEval = 0, kActAccept = 1, kActApply = 2, kActDone = 3 };
enum { kLsInit = 0, kLsBack = 1, kLsBracket = 2, kLsZoom = 3 };

struct Ctl {
  // next action and the trial it evaluates
  int act, mode, ls;
  double alpha;
  // optimizer state (models/qn_device.py: st.*, fvals, history, flags)
  double value, adj, gnorm, init_adj;
  double fv[kFv];
  int nfv, iter, H, head, hh, pass, search_failed, failed_once, overflow, why, nev;
  int first;  // L-BFGS: the next evaluation is the first of its line search (it forms dvec)
  double pend;  // data-parallel form: the accepted step not yet folded into mvec (the next
                // search's first pass adds pend * dvec: one grid pass fewer per iteration)
  double last_v, last_adj, last_gg;  // the last evaluation (the accepted step's values)
  // line search: backtracking (initfval, initd, shrink, it, force) / strong Wolfe (f0, d0, bracket
  // counter, lo / hi points, zoom counter), |g| of the state for the step checks
  double initfval, initd, shrink, gnrm, f0, d0, lo_t, lo_d, lo_f, hi_t, hi_d, hi_f;
  int it, force, bi, zi;
  // two-loop scratch (block 0)
  double as_[kMem], rho[kMem];
};

struct QnArgs {
  const unsigned char* X;
  int d, NT, ntl;
  int64_t n, nunits;
  const double* y;
  const double* w;
  const double* scale;  // fp8 per-feature scale (x = q * scale), or null
  const double* shift;  // per-feature storage shift (x = x' + s), or null
  const double* head;   // [count, W, W2, Σwy, Σwy², Σwx (d), Σwx² (d)]
  int fit_icpt, std_f, owlqn;
  double reg, enet, tol;
  int max_iter, hist_cap;
  // workspace (doubles): vectors of d, the history, the per-block slabs
  float* cs;  // [NC] the trial's f32 effective coefficients
  double *inv_sx, *sx, *mx, *regw, *l1, *x, *g, *ag, *dir, *cx, *cg, *cag, *S, *Y, *part, *lpart, *dpart, *scal;
  double* out;  // [coef(d), intercept, status, reason, H, iters, evaluations, head(5), history(hist_cap)]
  // L-BFGS (not OWLQN): per row, the margin of the accepted point (no offset) and X . dir of the
  // current line search -- a trial's margins are mvec + alpha dvec, so only the first trial of a
  // search reads X twice (it forms dvec); every other evaluation reads X once (the column pass)
  double *mvec, *dvec;
  // data-parallel form (lsq_qn_dp_*): the optimizer state in HBM between launches, and the
  // per-evaluation buffer all-reduced between the pass and the control kernel: [Σ v x_j (d),
  // Σ ½ w diff², Σ v]
  Ctl* ctl;
  double* red;
  unsigned* gbar;  // the one-launch form's grid barrier [arrivals, abandoned] (grid_barrier)
};

__device__ void ctl_record(Ctl& C, const QnArgs& a, double* hist) {
  if (C.H >= a.hist_cap) {
    C.overflow = 1;
    return;
  }
  if (hist) hist[C.H] = C.adj;
  ++C.H;
}

__device__ int ctl_converged(const Ctl& C, const QnArgs& a) {
  if (a.max_iter >= 0 && C.iter >= a.max_iter) return 0;
  if (C.nfv >= 2) {
    double mxv = -__builtin_inf();
    for (int i = kFv - C.nfv; i < kFv; ++i) mxv = fmax(mxv, C.fv[i]);
    if (fabs(C.adj - mxv) <= a.tol * fabs(C.init_adj)) return 1;
  }
  if (C.gnorm <= fmax(a.tol * fabs(C.value), 1e-8)) return 2;
  if (C.search_failed) return 3;
  return -1;
}

// the end of a loop pass (host: last.clear(); history.append(adj); why = converged())
__device__ void ctl_end_pass(Ctl& C, const QnArgs& a, double* hist) {
  ctl_record(C, a, hist);
  C.why = ctl_converged(C, a);
  C.act = (C.why >= 0 || C.overflow) ? kActDone : kActApply;
}

__device__ void ctl_fail(Ctl& C, const QnArgs& a, double* hist) {  // a FirstOrderException
  if (!C.failed_once) {
    C.failed_once = 1;
    C.hh = 0;
  } else {
    C.search_failed = 1;
  }
  ctl_end_pass(C, a, hist);
}

__device__ double ctl_interp(double at, double ad, double af, double bt, double bd, double bf) {
  const double d1 = ad + bd - 3.0 * (af - bf) / (at - bt);
  const double d2 = sqrt(d1 * d1 - ad * bd);
  const double mul = bt - at;
  const double x = bt - mul * (bd + d2 - d1) / (bd - ad + 2.0 * d2);
  const double lb = at + 0.1 * mul, ub = at + 0.9 * mul;
  return x < lb ? lb : (x > ub ? ub : x);
}

__device__ void ctl_zoom_next(Ctl& C) {  // the next zoom trial (interp(hi, lo) if lo.t > hi.t)
  C.alpha = C.lo_t > C.hi_t ? ctl_interp(C.hi_t, C.hi_d, C.hi_f, C.lo_t, C.lo_d, C.lo_f)
                            : ctl_interp(C.lo_t, C.lo_d, C.lo_f, C.hi_t, C.hi_d, C.hi_f);
  C.act = kActEval;
  C.mode = 1;
}

__device__ void ctl_found(Ctl& C, const QnArgs& a, double* hist) {
  // L-BFGS: StepSizeUnderflow when the accepted step is tiny relative to |g|
  if (C.ls != kLsBack && C.alpha * C.gnrm < 1e-10) {
    ctl_fail(C, a, hist);
    return;
  }
  C.act = kActAccept;
}

__device__ void ctl_after_eval(Ctl& C, const Eval& ev, const QnArgs& a, double* hist) {
  C.last_v = ev.v, C.last_adj = ev.adj, C.last_gg = ev.gg;
  if (C.ls == kLsInit) {
    C.act = kActAccept;
    return;
  }
  const double c1 = 1e-4, c2 = 0.9;
  if (C.ls == kLsBack) {  // Breeze BacktrackingLineSearch as OWLQN configures it
    if (C.force) {
      C.act = kActAccept;
      return;
    }
    double mult;
    if (ev.adj > C.initfval + C.alpha * C.initd * c1) mult = C.shrink;
    else if (ev.dd < c2 * C.initd) mult = 2.1;
    else if (ev.dd > -c2 * C.initd) mult = C.shrink;
    else mult = 1.0;
    if (mult == 1.0) {
      C.act = kActAccept;
      return;
    }
    const double na = C.alpha * mult;
    if (C.it >= 20 || na < 1e-10 || na > 1e10) {
      ctl_fail(C, a, hist);
      return;
    }
    C.alpha = na;
    if (C.it + 1 >= 20) C.force = 1;  // takeWhile(iter < maxIterations) keeps the last state
    else ++C.it;
    C.act = kActEval;
    return;
  }
  const double f = ev.v, dd = ev.dd, tt = C.alpha;
  if (C.ls == kLsBracket) {  // Breeze StrongWolfeLineSearch, bracketing phase
    const int i = C.bi;
    if (!(f - f == 0.0)) {  // not finite: halve and retry
      C.alpha = tt / 2.0;
    } else if (f > C.f0 + c1 * tt * C.d0 || (f >= C.lo_f && i > 0)) {
      C.hi_t = tt, C.hi_d = dd, C.hi_f = f;
      C.ls = kLsZoom, C.zi = 0;
      ctl_zoom_next(C);
      return;
    } else if (fabs(dd) <= c2 * fabs(C.d0)) {
      ctl_found(C, a, hist);
      return;
    } else if (dd >= 0.0) {
      C.hi_t = C.lo_t, C.hi_d = C.lo_d, C.hi_f = C.lo_f;
      C.lo_t = tt, C.lo_d = dd, C.lo_f = f;
      C.ls = kLsZoom, C.zi = 0;
      ctl_zoom_next(C);
      return;
    } else {
      C.lo_t = tt, C.lo_d = dd, C.lo_f = f;
      C.alpha = tt * 1.5;
    }
    if (++C.bi >= 10) {
      ctl_fail(C, a, hist);  // "Line search failed"
      return;
    }
    C.act = kActEval;
    return;
  }
  // zoom
  if (f > C.f0 + c1 * tt * C.d0 || f >= C.lo_f) {
    C.hi_t = tt, C.hi_d = dd, C.hi_f = f;
  } else {
    if (fabs(dd) <= c2 * fabs(C.d0)) {
      ctl_found(C, a, hist);
      return;
    }
    if (dd * (C.hi_t - C.lo_t) >= 0.0) C.hi_t = C.lo_t, C.hi_d = C.lo_d, C.hi_f = C.lo_f;
    C.lo_t = tt, C.lo_d = dd, C.lo_f = f;
  }
  if (++C.zi >= 10) {
    ctl_fail(C, a, hist);  // "Line search zoom failed"
    return;
  }
  ctl_zoom_next(C);
}

__device__ void ctl_after_accept(Ctl& C, const QnArgs& a, double* hist) {
  if (C.ls == kLsInit) {  // the start point
    C.value = C.last_v, C.adj = C.last_adj, C.gnorm = sqrt(C.last_gg);
    C.init_adj = C.adj;
    ctl_record(C, a, hist);
    C.why = ctl_converged(C, a);
    C.act = (C.why >= 0 || C.overflow) ? kActDone : kActApply;
    return;
  }
  C.head = (C.head + kMem - 1) % kMem;
  C.hh = C.hh < kMem ? C.hh + 1 : kMem;
  for (int i = 0; i < kFv - 1; ++i) C.fv[i] = C.fv[i + 1];
  C.fv[kFv - 1] = C.last_v;
  C.nfv = C.nfv < kFv ? C.nfv + 1 : kFv;
  C.value = C.last_v, C.adj = C.last_adj, C.gnorm = sqrt(C.last_gg);
  ++C.iter;
  C.failed_once = 0;
  ctl_end_pass(C, a, hist);
}

__device__ void ctl_start_search(Ctl& C, const double* scal, const QnArgs& a, double* hist) {
  ++C.pass;
  const double initd = scal[0], gnrm = sqrt(scal[1]), dnrm = sqrt(scal[2]);
  C.gnrm = gnrm;
  if (scal[3] != 0.0) {  // NaN / negative-curvature history
    ctl_fail(C, a, hist);
    return;
  }
  C.mode = 1;
  C.act = kActEval;
  if (a.owlqn) {
    C.ls = kLsBack;
    C.initfval = C.adj;
    C.initd = initd;
    C.shrink = C.iter < 1 ? 0.1 : 0.5;
    C.alpha = C.iter < 1 ? 0.5 / gnrm : 1.0;
    C.it = 0, C.force = 0;
    return;
  }
  C.ls = kLsBracket;
  C.first = 1;
  C.f0 = C.value, C.d0 = initd;
  if (initd > 0.0) {  // "Line search invoked with non-descent direction"
    ctl_fail(C, a, hist);
    return;
  }
  C.alpha = C.iter == 0 ? 1.0 / dnrm : 1.0;
  C.lo_t = 0.0, C.lo_d = initd, C.lo_f = C.value;
  C.bi = 0;
}

// block 0: two-loop recursion on the (pseudo-)gradient -> dir (HBM); scal = [g . dir, |g|^2,
// |dir|^2, history failed]
__device__ void apply_dir(const QnArgs& a, Ctl& C, double* scal, double* red, bool owlqn) {
  const int t = threadIdx.x, d = a.d;
  const double* gv = owlqn ? a.ag : a.g;
  auto dot = [&](const double* p, const double* q) {
    double v = 0.0;
    for (int j = t; j < d; j += kT) v += p[j] * q[j];
    return block_sum(v, red);
  };
  const int hh = C.hh, head = C.head;
  bool fail = false;
  double diag = 1.0;
  for (int j = t; j < d; j += kT) a.dir[j] = gv[j];
  __syncthreads();
  if (hh > 0) {
    const double* sv = a.S + (int64_t)head * d;
    const double* yv = a.Y + (int64_t)head * d;
    const double sy = dot(sv, yv), yy = dot(yv, yv);
    if (sy < 0.0 || sy != sy) fail = true;
    diag = sy / yy;
  }
  for (int i = 0; i < hh; ++i) {
    const int p = (head + i) % kMem;
    const double* sv = a.S + (int64_t)p * d;
    const double* yv = a.Y + (int64_t)p * d;
    const double rho = dot(sv, yv);
    const double as = dot(sv, a.dir) / rho;
    if (as != as) fail = true;
    if (t == 0) C.rho[i] = rho, C.as_[i] = as;
    for (int j = t; j < d; j += kT) a.dir[j] = a.dir[j] - as * yv[j];
  }
  if (hh > 0)
    for (int j = t; j < d; j += kT) a.dir[j] = a.dir[j] * diag;
  __syncthreads();
  for (int i = hh - 1; i >= 0; --i) {
    const int p = (head + i) % kMem;
    const double* sv = a.S + (int64_t)p * d;
    const double* yv = a.Y + (int64_t)p * d;
    const double beta = dot(yv, a.dir) / C.rho[i];
    const double coef = C.as_[i] - beta;
    for (int j = t; j < d; j += kT) a.dir[j] = a.dir[j] + coef * sv[j];
  }
  double pd = 0.0, pgg = 0.0, pdd = 0.0;
  for (int j = t; j < d; j += kT) {
    double dj = -a.dir[j];
    if (owlqn && !(dj * gv[j] < 0.0)) dj = 0.0;
    a.dir[j] = dj;
    pd += gv[j] * dj;
    pgg += a.g[j] * a.g[j];
    pdd += dj * dj;
  }
  const double initd = block_sum(pd, red), gg = block_sum(pgg, red), dn = block_sum(pdd, red);
  if (t == 0) {
    scal[0] = initd;
    scal[1] = gg;
    scal[2] = dn;
    scal[3] = fail ? 1.0 : 0.0;
  }
  __threadfence();
}

// ---- pieces shared by the one-launch kernel and the data-parallel kernels ------------------

// standardization constants from the summarizer head (lbfgs_path._train_passes' expression order)
struct Std {
  double W, my, denom, ys, l1c, l2, icpt0, inv_ys, inv_w;
  int status;  // 0 ok, 1 empty data, 2 constant label (the host path owns those)
};

__device__ __forceinline__ Std std_of(const QnArgs& a) {
  const double* hd = a.head;
  Std S;
  S.W = hd[1];
  const double W2 = hd[2], bsum = hd[3], bbsum = hd[4];
  S.denom = S.W - W2 / S.W;
  S.my = bsum / S.W;
  const double var_y = S.denom > 0.0 ? fmax(bbsum - S.W * S.my * S.my, 0.0) / S.denom : 0.0;
  S.ys = sqrt(var_y);
  S.status = !(S.W > 0.0) ? 1 : (S.ys == 0.0 ? 2 : 0);
  const double eff_reg = a.reg / S.ys;
  S.l1c = a.enet * eff_reg;
  S.l2 = (1.0 - a.enet) * eff_reg;
  S.icpt0 = a.fit_icpt ? S.my / S.ys : 0.0;
  S.inv_ys = 1.0 / S.ys;
  S.inv_w = 1.0 / S.W;
  return S;
}

// per-feature constants of features [j0, j1) (threads of one block stride the range)
__device__ __forceinline__ void feature_consts(const QnArgs& a, const Std& S, int j0, int j1) {
  const double* hd = a.head;
  const int d = a.d;
  const bool owlqn = a.owlqn != 0;
  for (int j = j0 + (int)threadIdx.x; j < j1; j += kT) {
    const double m = hd[5 + j] / S.W;
    const double vx = S.denom > 0.0 ? fmax(hd[5 + d + j] - S.W * m * m, 0.0) / S.denom : 0.0;
    const double sx = sqrt(vx);
    const bool nz = sx != 0.0;
    const double safe = nz ? sx : 1.0;
    a.mx[j] = m;
    a.sx[j] = safe;
    a.inv_sx[j] = nz ? 1.0 / safe : 0.0;
    a.regw[j] = S.l2 != 0.0 ? (a.std_f ? 1.0 : (nz ? 1.0 / (safe * safe) : 0.0)) : 0.0;
    a.l1[j] = owlqn ? (a.std_f ? S.l1c : (nz ? S.l1c / safe : 0.0)) : 0.0;
    a.x[j] = 0.0;
    a.dir[j] = 0.0;
    a.ag[j] = 0.0;
  }
}

__device__ __forceinline__ void ctl_init(Ctl& C) {
  C.act = kActEval;
  C.mode = 0;
  C.alpha = 0.0;
  C.ls = kLsInit;
  C.head = 0, C.hh = 0, C.H = 0, C.iter = 0, C.nfv = 1, C.pass = 0;
  C.search_failed = 0, C.failed_once = 0, C.overflow = 0, C.why = -1, C.nev = 0, C.first = 0;
  C.pend = 0.0;
  for (int i = 0; i < kFv; ++i) C.fv[i] = 0.0;
  C.fv[kFv - 1] = __builtin_inf();
}

// E1 (one block): the trial point x + alpha dir (mode 1, projected for OWLQN) or x0 = 0 (mode 0),
// kept for the acceptance; the f32 effective coefficients (every pass block reads them through
// its L2) over the nc coefficient slots; the margin offset -> scal[16]
__device__ void build_trial(const QnArgs& a, const Std& S, int mode, double alpha, int nc, double* red) {
  const int t = threadIdx.x, d = a.d;
  const bool owlqn = a.owlqn != 0;
  double pm = 0.0, ps = 0.0;
#pragma unroll 2
  for (int j = t; j < nc; j += kT) {
    float c32 = 0.0f;
    if (j < d) {
      double nx = 0.0;
      if (mode == 1) {
        const double xj = a.x[j];
        nx = xj + a.dir[j] * alpha;
        if (owlqn) {
          const double orth = xj != 0.0 ? sgn(xj) : sgn(-a.ag[j]);
          if (sgn(nx) != orth) nx = 0.0;
        }
      }
      a.cx[j] = nx;
      const double cf = nx * a.inv_sx[j];
      pm += cf * a.mx[j];
      if (a.shift) ps += a.shift[j] * cf;
      // L-BFGS: the margin loop forms X . dir (a trial is mvec + alpha dvec); OWLQN's projected
      // trial is not affine in alpha: its margins come from the trial's coefficients
      const double cm = owlqn ? cf : a.dir[j] * a.inv_sx[j];
      c32 = (float)(a.scale ? cm * a.scale[j] : cm);
    }
    a.cs[j] = c32;
  }
  const double cfmx = block_sum(pm, red);
  double off = a.fit_icpt ? S.icpt0 - cfmx : S.icpt0;
  if (a.shift) off = off + block_sum(ps, red);
  if (t == 0) a.scal[16] = off;
  __threadfence();
}

// E2: the fused pass of block b of B over its fragment units (margins, then the column sums of
// the same tiles) -> the block's column slab part[b] and (loss, Σv) in lpart[b].  L-BFGS: margins
// only on the first trial of a line search (X . dir -> dvec; with pend != 0 the accepted step is
// folded into mvec first); the other trials read X once.  colacc must be zeroed by the caller.
template <int L, int TPW>
__device__ __forceinline__ void qn_pass(const QnArgs& a, const Std& S, int mode, double alpha, bool first, double pend,
                                        double offset, double* colacc, double* mrow, float* vrow, double* red,
                                        int b, int B) {
  constexpr int E = L == 3 ? 16 : 8;
  constexpr int64_t CH = L == 3 ? 2048 : 4096;
  constexpr int UPS = L == 3 ? 2 : 4;
  constexpr int NC = 8 * TPW * 32;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6, fl = lane & 31, hf = lane >> 5;
  const bool owlqn = a.owlqn != 0;
  const float* __restrict__ gcs = a.cs;
  const bool skip = !owlqn && !first;
  double loss = 0.0, vsum = 0.0;
  for (int64_t u = b; u < a.nunits; u += B) {
    const int64_t s = u / UPS;
    const int sub = (int)(u % UPS);
    const unsigned char* p = a.X + s * a.NT * CH + ((sub * 64 + lane) << 4);
    double acc[E];
#pragma unroll
    for (int e = 0; e < E; ++e) acc[e] = 0.0;
#pragma unroll 1
    for (int i0 = 0; i0 < (skip ? 0 : TPW); i0 += 8) {
      u32x4 q[8];
      float c[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int tt = wave + 8 * (i0 + k);
        q[k] = tt < a.ntl ? *gptr<u32x4>(p + (int64_t)tt * CH) : u32x4{0u, 0u, 0u, 0u};
        c[k] = *gptr<float>(gcs + tt * 32 + fl);
      }
      float s8[E];
#pragma unroll
      for (int e = 0; e < E; ++e) s8[e] = 0.0f;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        float xv[E];
        unpack<L>(q[k], xv);
#pragma unroll
        for (int e = 0; e < E; ++e) s8[e] = fmaf(xv[e], c[k], s8[e]);
      }
#pragma unroll
      for (int e = 0; e < E; ++e) acc[e] += (double)s8[e];
    }
    // feature sum across the 32 lanes of each half, then the 8 waves' partials in LDS
#pragma unroll
    for (int e = 0; e < E; ++e) {
#pragma unroll
      for (int o = 1; o < 32; o <<= 1) acc[e] += __shfl_xor(acc[e], o, 64);
    }
    double m = acc[0];
#pragma unroll
    for (int e = 1; e < E; ++e) m = fl == e ? acc[e] : m;
    if (fl < E) mrow[wave * 2 * E + hf * E + fl] = m;
    __syncthreads();
    if (t < 2 * E) {
      double mm = 0.0;
      const int64_t r = frag_row<L>(s, sub, t / E, t % E);
      if (!skip)
#pragma unroll
        for (int i = 0; i < kW; ++i) mm += mrow[i * 2 * E + t];
      if (!owlqn && r < a.n) {  // mm: this unit's X . dir (first trial) -> the trial's margin
        double mv = a.mvec[r];
        if (first && pend != 0.0) {  // (data-parallel form) the accepted step's margins, folded now
          mv = mv + pend * a.dvec[r];
          a.mvec[r] = mv;
        }
        const double md = skip ? a.dvec[r] : mm;
        if (first) a.dvec[r] = mm;
        mm = mv + alpha * md;
      }
      double vv = 0.0;
      if (r < a.n) {
        const double wr = a.w[r];
        if (wr != 0.0) {
          const double diff = mm + offset - a.y[r] * S.inv_ys;
          vv = wr * diff;
          loss += 0.5 * vv * diff;
          vsum += vv;
        }
      }
      vrow[t] = (float)vv;
    }
    __syncthreads();
    float vr[E];
#pragma unroll
    for (int e = 0; e < E; ++e) vr[e] = vrow[hf * E + e];
    // column sums of the same tiles, most recently read first; the two lane halves (the
    // feature's other rows) combine, then one f64 LDS accumulator per feature (this wave's
    // tiles only: no other wave touches them)
#pragma unroll 1
    for (int i0 = TPW - 8; i0 >= 0; i0 -= 8) {
      u32x4 q[8];
#pragma unroll
      for (int k = 7; k >= 0; --k) {
        const int tt = wave + 8 * (i0 + k);
        q[k] = tt < a.ntl ? *gptr<u32x4>(p + (int64_t)tt * CH) : u32x4{0u, 0u, 0u, 0u};
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        float xv[E];
        unpack<L>(q[k], xv);
        float sa = 0.0f;
#pragma unroll
        for (int e = 0; e < E; ++e) sa += vr[e] * xv[e];
        sa += __shfl_xor(sa, 32, 64);
        if (hf == 0) colacc[(wave + 8 * (i0 + k)) * 32 + fl] += (double)sa;
      }
    }
  }
  __syncthreads();
  // the block's column slab
  double* slab = a.part + (int64_t)b * NC;
  for (int j = t; j < NC; j += kT) slab[j] = colacc[j];
  const double bl = block_sum(loss, red), bv = block_sum(vsum, red);
  if (t == 0) a.lpart[2 * b] = bl, a.lpart[2 * b + 1] = bv;
}

// a column sum of the STORED values (q = x / scale, x' = x - shift) -> Σ v x_j
__device__ __forceinline__ double unscale_col(const QnArgs& a, int j, double graw, double vs) {
  if (a.scale) graw = graw * a.scale[j];
  if (a.shift) graw = graw + a.shift[j] * vs;
  return graw;
}

// E3 per feature: the column sum Σ v x_j -> gradient / adjusted gradient (cg, cag) and the partial
// evaluation scalars x.(regw x), Σ|l1 x|, dir . ag, ag . ag
__device__ __forceinline__ void grad_j(const QnArgs& a, const Std& S, int j, double graw, double& pr, double& pl,
                                       double& pd, double& pg) {
  const double nx = a.cx[j];
  double gj = graw * a.inv_sx[j] * S.inv_w;
  if (S.l2 != 0.0) {
    const double rx = a.regw[j] * nx;
    pr += nx * rx;
    gj = gj + S.l2 * rx;
  }
  double agj = gj;
  const double l = a.l1[j];
  if (a.owlqn) {
    pl += fabs(l * nx);
    if (l != 0.0) {
      if (nx == 0.0) {
        const double dp = gj + l, dm = gj - l;
        agj = dm > 0.0 ? dm : (dp < 0.0 ? dp : 0.0);
      } else {
        agj = gj + sgn(nx) * l;
      }
    }
  }
  a.cg[j] = gj;
  a.cag[j] = agj;
  pd += agj * a.dir[j];
  pg += agj * agj;
}

__device__ __forceinline__ Eval eval_of(const QnArgs& a, const Std& S, double lsum, double sr, double sl, double sd,
                                        double sg) {
  Eval ev;
  ev.v = lsum * S.inv_w;
  if (S.l2 != 0.0) ev.v = ev.v + 0.5 * S.l2 * sr;
  ev.adj = a.owlqn ? ev.v + sl : ev.v;
  ev.dd = sd;
  ev.gg = sg;
  return ev;
}

// the last evaluated trial becomes the state (history pair pushed first): one block
__device__ void accept_block(const QnArgs& a, const Ctl& C) {
  const int t = threadIdx.x, d = a.d;
  const bool push = C.ls != kLsInit;
  int hd0 = C.head;
  if (push) hd0 = (hd0 + kMem - 1) % kMem;
  for (int j = t; j < d; j += kT) {
    const double nx = a.cx[j], gj = a.cg[j];
    if (push) {
      a.S[(int64_t)hd0 * d + j] = nx - a.x[j];
      a.Y[(int64_t)hd0 * d + j] = gj - a.g[j];
    }
    a.x[j] = nx;
    a.g[j] = gj;
    a.ag[j] = a.cag[j];
  }
  __threadfence();
}

// un-standardize into out: coef = x ys / sigma (0 for constant features), intercept = ȳ - coef . x̄
__device__ void finalize_block(const QnArgs& a, const Ctl& C, const Std& S, double* red) {
  const int t = threadIdx.x, d = a.d;
  if (C.overflow) {
    if (t == 0) a.out[d + 1] = 8.0;
    return;
  }
  double pc = 0.0;
  for (int j = t; j < d; j += kT) {
    const double c = a.inv_sx[j] != 0.0 ? a.x[j] * S.ys / a.sx[j] : 0.0;
    a.out[j] = c;
    pc += c * a.mx[j];
  }
  const double cm = block_sum(pc, red);
  if (t == 0) {
    a.out[d] = a.fit_icpt ? S.my - cm : 0.0;
    a.out[d + 1] = 0.0;
    a.out[d + 2] = (double)C.why;
    a.out[d + 3] = (double)C.H;
    a.out[d + 4] = (double)C.iter;
    a.out[d + 5] = (double)C.nev;  // cost evaluations (data passes)
  }
}

template <int L, int TPW>
__global__ __launch_bounds__(kT, 1) void lsq_qn_kernel(QnArgs a) {
  unsigned gen = 0;
  auto grid_sync = [&]() { grid_barrier(a.gbar, gen, gridDim.x); };
  constexpr int E = L == 3 ? 16 : 8;
  constexpr int NC = 8 * TPW * 32;  // coefficient slots (tiles padded to whole wave strides)
  __shared__ double colacc[NC];  // the block's f64 column sums (<= 128 KiB)
  __shared__ double red[kW];
  __shared__ double mrow[kW * 2 * E];
  __shared__ float vrow[2 * E];
  __shared__ double fold[kW][64];
  __shared__ double bcast[4];
  __shared__ Ctl C;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int B = gridDim.x, b = blockIdx.x;
  const int d = a.d;

  // ---- standardization constants (lbfgs_path._train_passes, in the same expression order) ----
  const Std S = std_of(a);
  if (b == 0 && t < 5) a.out[d + 6 + t] = a.head[t];
  if (S.status != 0) {  // empty data / constant label: the host path owns the semantics
    if (b == 0 && t == 0) a.out[d + 1] = (double)S.status;
    return;  // uniform across the grid: no barrier has been reached
  }
  const bool owlqn = a.owlqn != 0;
  {
    const int per = (d + B - 1) / B, j0 = b * per, j1 = min(d, j0 + per);
    feature_consts(a, S, j0, j1);
  }
  for (int64_t r = (int64_t)b * kT + t; r < a.n; r += (int64_t)B * kT) a.mvec[r] = 0.0, a.dvec[r] = 0.0;  // x0 = 0
  __threadfence();
  grid_sync();

  // ---- one cost evaluation at x + alpha dir (mode 1, projected for OWLQN) or at x0 = 0 -------
  auto evaluate = [&](int mode, double alpha) -> Eval {
    // E1: block 0 builds the trial point, the f32 effective coefficients and the margin offset
    if (b == 0) build_trial(a, S, mode, alpha, NC, red);
    for (int j = t; j < NC; j += kT) colacc[j] = 0.0;
    grid_sync();
    // E2: the fused pass
    qn_pass<L, TPW>(a, S, mode, alpha, !owlqn && mode == 1 && C.first, 0.0, a.scal[16], colacc, mrow, vrow, red,
                    b, B);
    __threadfence();
    grid_sync();

    // E3: fixed-order fold of the slabs over this block's features -> gradient, adjusted gradient
    // (grid totals: wave 0, lane l sums entries l, l + 64, ...; the same order in every block)
    if (wave == 0) {
      double l0 = 0.0, l1s = 0.0;
      for (int i = lane; i < B; i += kWave) l0 += a.lpart[2 * i], l1s += a.lpart[2 * i + 1];
      l0 = wave_sum_f64(l0);
      l1s = wave_sum_f64(l1s);
      if (lane == 0) bcast[0] = l0, bcast[1] = l1s;
    }
    __syncthreads();
    const double lsum = bcast[0], vs = bcast[1];
    const int per = (d + B - 1) / B, j0 = b * per, j1 = min(d, j0 + per);
    double pr = 0.0, pl = 0.0, pd = 0.0, pg = 0.0;
    for (int jb = j0; jb < j1; jb += 64) {
      {
        const int j = jb + lane;
        double sp = 0.0;
        if (j < j1)
#pragma unroll 4
          for (int i = wave; i < B; i += kW) sp += a.part[(int64_t)i * NC + j];
        fold[wave][lane] = sp;
      }
      __syncthreads();
      const int j = jb + t;
      if (t < 64 && j < j1) {
        double graw = 0.0;
#pragma unroll
        for (int i = 0; i < kW; ++i) graw += fold[i][t];
        grad_j(a, S, j, unscale_col(a, j, graw, vs), pr, pl, pd, pg);
      }
      __syncthreads();
    }
    {
      const double s0 = block_sum(pr, red), s1 = block_sum(pl, red), s2 = block_sum(pd, red),
                   s3 = block_sum(pg, red);
      if (t == 0) {
        double* dp = a.dpart + (int64_t)b * kDParts;
        dp[0] = s0, dp[1] = s1, dp[2] = s2, dp[3] = s3;
      }
    }
    __threadfence();
    grid_sync();
    if (wave == 0) {
      double q[kDParts] = {0.0, 0.0, 0.0, 0.0};
      for (int i = lane; i < B; i += kWave)
#pragma unroll
        for (int k = 0; k < kDParts; ++k) q[k] += a.dpart[(int64_t)i * kDParts + k];
#pragma unroll
      for (int k = 0; k < kDParts; ++k) {
        q[k] = wave_sum_f64(q[k]);
        if (lane == 0) bcast[k] = q[k];
      }
    }
    __syncthreads();
    const double sr = bcast[0], sl = bcast[1], sd = bcast[2], sg = bcast[3];
    __syncthreads();  // bcast is rewritten by the next evaluation
    return eval_of(a, S, lsum, sr, sl, sd, sg);
  };

  // ---- the optimizer as a state machine: thread 0 of every block runs the same scalar logic on
  // the same inputs (its block's LDS copy of the state), so every block takes the same next
  // action; ONE evaluate call site keeps the control state out of the pass's registers ----------
  if (t == 0) ctl_init(C);
  __syncthreads();
  for (;;) {
    const int act = C.act;
    if (act == kActDone) break;
    if (act == kActEval) {
      const Eval ev = evaluate(C.mode, C.alpha);
      if (t == 0) {
        ++C.nev;
        C.first = 0;
        ctl_after_eval(C, ev, a, b == 0 ? a.out + d + 11 : nullptr);
      }
    } else if (act == kActAccept) {
      if (b == 0) accept_block(a, C);
      if (!owlqn && C.ls != kLsInit) {  // the accepted trial's margins: mvec + alpha dvec
        const double al = C.alpha;
        for (int64_t r = (int64_t)b * kT + t; r < a.n; r += (int64_t)B * kT) a.mvec[r] = a.mvec[r] + al * a.dvec[r];
      }
      __syncthreads();
      if (t == 0) ctl_after_accept(C, a, b == 0 ? a.out + d + 11 : nullptr);
    } else {  // kActApply
      double* scal = a.scal + 8 * (C.pass & 1);  // parity: a pass with no evaluation has no barrier after the read
      if (b == 0) apply_dir(a, C, scal, red, owlqn);
      grid_sync();
      if (t == 0) ctl_start_search(C, scal, a, b == 0 ? a.out + d + 11 : nullptr);
    }
    __syncthreads();
  }
  if (b != 0) return;
  finalize_block(a, C, S, red);
  if (t == 0 && grid_abandoned(a.gbar)) a.out[d + 1] = 9.0;  // not finished: the host path re-runs
}

// ---- data-parallel form (X4): the same fit split at the reduction ---------------------------
// Spark's l-bfgs sums every evaluation's loss and gradient over the partitions (treeAggregate,
// DataQuality4MachineLearningApp.java:120-126); across ranks that is an RCCL all-reduce, which a
// single grid launch cannot contain.  Per evaluation the host enqueues, on one stream with no
// host read in between:
//   lsq_qn_dp_pass_kernel  (grid)    the fused E2 pass over this rank's rows -> per-block slabs
//   lsq_qn_dp_fold_kernel  (d / 64)  fixed-order slab fold -> red = [Σ v x_j (d), loss, Σ v]
//   RCCL all-reduce(red)             (d + 2) f64
//   lsq_qn_dp_ctl_kernel   (1 block) E3 on the summed red, the Breeze state machine (after_eval,
//                                    accept, two-loop recursion, next line-search step), the next
//                                    trial point -- or the un-standardized result when done
// The optimizer state (Ctl) lives in HBM between launches; every rank's control kernel reads the
// same all-reduced bytes, so the ranks take identical decisions.  Once the state is done every
// kernel returns at once: the host enqueues evaluations in batches ahead of the device and stops
// when a pinned copy of the state's action says so (models/lbfgs_path.py).  The accepted step's
// margin update (mvec += alpha dvec, a grid pass in the one-launch kernel) is folded into the
// next search's first pass (Ctl.pend).

__global__ __launch_bounds__(kT) void lsq_qn_dp_init_kernel(QnArgs a, int nc) {
  __shared__ double red[kW];
  __shared__ Ctl C;
  const int t = threadIdx.x, d = a.d;
  const Std S = std_of(a);
  if (t < 5) a.out[d + 6 + t] = a.head[t];
  if (t == 0) ctl_init(C);
  __syncthreads();
  if (S.status != 0) {
    if (t == 0) {
      a.out[d + 1] = (double)S.status;
      C.act = kActDone;
    }
  } else {
    feature_consts(a, S, 0, d);
    __syncthreads();
    build_trial(a, S, 0, 0.0, nc, red);
  }
  __syncthreads();
  if (t == 0) *a.ctl = C;
}

template <int L, int TPW>
__global__ __launch_bounds__(kT, 1) void lsq_qn_dp_pass_kernel(QnArgs a) {
  constexpr int E = L == 3 ? 16 : 8;
  constexpr int NC = 8 * TPW * 32;
  __shared__ double colacc[NC];
  __shared__ double red[kW];
  __shared__ double mrow[kW * 2 * E];
  __shared__ float vrow[2 * E];
  const Ctl* C = a.ctl;  // written by the previous kernel on this stream
  if (C->act != kActEval) return;
  const int mode = C->mode;
  const double alpha = C->alpha, pend = C->pend;
  const bool first = a.owlqn == 0 && mode == 1 && C->first;
  const Std S = std_of(a);
  for (int j = threadIdx.x; j < NC; j += kT) colacc[j] = 0.0;
  __syncthreads();
  qn_pass<L, TPW>(a, S, mode, alpha, first, pend, a.scal[16], colacc, mrow, vrow, red, blockIdx.x, gridDim.x);
}

// one block per 64 features (block 0 also sums the loss partials); the same summation order as
// the one-launch kernel's E3
//
// The per-rank storage scale / shift is applied HERE, before the all-reduce: ranks may hold
// different fp8 scales (each shard's amax) and the shift term needs this rank's Σ v.
__global__ __launch_bounds__(kT) void lsq_qn_dp_fold_kernel(QnArgs a, int B, int nc) {
  __shared__ double fold[kW][64];
  __shared__ double lv[2];
  if (a.ctl->act != kActEval) return;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6, d = a.d;
  const int jb = blockIdx.x * 64;
  if (wave == 0) {  // this rank's loss and Σ v (every block: the shift term needs Σ v)
    double l0 = 0.0, l1s = 0.0;
    for (int i = lane; i < B; i += kWave) l0 += a.lpart[2 * i], l1s += a.lpart[2 * i + 1];
    l0 = wave_sum_f64(l0);
    l1s = wave_sum_f64(l1s);
    if (lane == 0) lv[0] = l0, lv[1] = l1s;
  }
  {
    const int j = jb + lane;
    double sp = 0.0;
    if (j < d)
#pragma unroll 4
      for (int i = wave; i < B; i += kW) sp += a.part[(int64_t)i * nc + j];
    fold[wave][lane] = sp;
  }
  __syncthreads();
  if (t < 64 && jb + t < d) {
    double graw = 0.0;
#pragma unroll
    for (int i = 0; i < kW; ++i) graw += fold[i][t];
    a.red[jb + t] = unscale_col(a, jb + t, graw, lv[1]);
  }
  if (blockIdx.x == 0 && t == 0) a.red[d] = lv[0], a.red[d + 1] = lv[1];
}

__global__ __launch_bounds__(kT) void lsq_qn_dp_ctl_kernel(QnArgs a, int nc) {
  __shared__ double red[kW];
  __shared__ Ctl C;
  const int t = threadIdx.x, d = a.d;
  if (t == 0) C = *a.ctl;
  __syncthreads();
  if (C.act != kActEval) return;
  const Std S = std_of(a);
  const bool owlqn = a.owlqn != 0;
  double* hist = a.out + d + 11;
  // E3 on the all-reduced sums
  const double lsum = a.red[d];
  double pr = 0.0, pl = 0.0, pd = 0.0, pg = 0.0;
  for (int j = t; j < d; j += kT) grad_j(a, S, j, a.red[j], pr, pl, pd, pg);
  const double sr = block_sum(pr, red), sl = block_sum(pl, red), sd = block_sum(pd, red), sg = block_sum(pg, red);
  const Eval ev = eval_of(a, S, lsum, sr, sl, sd, sg);
  __threadfence();
  __syncthreads();
  if (t == 0) {
    ++C.nev;
    C.first = 0;
    C.pend = 0.0;  // the pass just run folded it (only a search's first pass sees pend != 0)
    ctl_after_eval(C, ev, a, hist);
  }
  __syncthreads();
  for (;;) {
    const int act = C.act;
    if (act == kActEval) {
      build_trial(a, S, C.mode, C.alpha, nc, red);
      break;
    }
    if (act == kActDone) {
      finalize_block(a, C, S, red);
      break;
    }
    if (act == kActAccept) {
      accept_block(a, C);
      __syncthreads();
      if (t == 0) {
        if (!owlqn && C.ls != kLsInit) C.pend = C.alpha;  // mvec += alpha dvec, in the next first pass
        ctl_after_accept(C, a, hist);
      }
    } else {  // kActApply
      apply_dir(a, C, a.scal, red, owlqn);
      __syncthreads();
      if (t == 0) ctl_start_search(C, a.scal, a, hist);
    }
    __syncthreads();
  }
  __syncthreads();
  if (t == 0) *a.ctl = C;
}

template <int L, int TPW>
const void* kernel_of() {
  return (const void*)lsq_qn_kernel<L, TPW>;
}

const void* pick(int layout, int tpw) {
  if (layout == 2) {
    switch (tpw) {
      case 8: return kernel_of<2, 8>();
      case 16: return kernel_of<2, 16>();
      case 32: return kernel_of<2, 32>();
      default: return kernel_of<2, 64>();
    }
  }
  switch (tpw) {
    case 8: return kernel_of<3, 8>();
    case 16: return kernel_of<3, 16>();
    case 32: return kernel_of<3, 32>();
    default: return kernel_of<3, 64>();
  }
}

int tpw_of(int d) {
  const int ntl = (d + 31) / 32;
  const int need = (ntl + 7) / 8;
  return need <= 8 ? 8 : need <= 16 ? 16 : need <= 32 ? 32 : 64;
}

}  // namespace

int lsq_qn_blocks(int layout, int d) {
  if (layout != 2 && layout != 3) throw std::invalid_argument("lsq_qn: wide tile layouts only");
  if (d < 1 || d > kLsqQnMaxD) throw std::invalid_argument("lsq_qn: d out of range");
  int dev = 0, cus = 0, per = 0;
  DQ_HIP_CHECK(hipGetDevice(&dev));
  DQ_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  DQ_HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, pick(layout, tpw_of(d)), kT, 0));
  if (per < 1) throw std::runtime_error("lsq_qn: the kernel does not fit a CU");
  return cus;  // one block per CU: the grid is co-resident (grid_barrier relies on it)
}

int64_t lsq_qn_work(int d, int blocks, int64_t n) {
  const int64_t slab = 8LL * tpw_of(d) * 32;
  return 12LL * d + 2LL * kMem * d + (int64_t)blocks * slab + 2LL * blocks + (int64_t)blocks * kDParts + 24 + 1 +
         (8LL * tpw_of(d) * 32 + 1) / 2 + 2 * n;
}

namespace {

constexpr int64_t kCtlDoubles = (int64_t)((sizeof(Ctl) + 7) / 8);

QnArgs make_args(const LsqX& x, const double* y, const double* w, const double* scale, const double* shift,
                 const double* head, bool fit_icpt, bool std_f, double reg, double enet, int max_iter, double tol,
                 int hist_cap, double* work, int blocks, double* out, bool dp) {
  if (x.layout != 2 && x.layout != 3) throw std::invalid_argument("lsq_qn: wide tile layouts only");
  if (x.d < 1 || x.d > kLsqQnMaxD) throw std::invalid_argument("lsq_qn: d out of range");
  if (hist_cap < 1 || blocks < 1) throw std::invalid_argument("lsq_qn: bad history capacity / grid");
  const int d = x.d, tpw = tpw_of(d);
  QnArgs a{};
  a.X = reinterpret_cast<const unsigned char*>(x.X);
  a.d = d;
  a.ntl = (d + 31) / 32;
  a.NT = ((d + 255) / 256) * 8;
  a.n = x.n;
  a.nunits = ((x.n + 63) / 64) * (x.layout == 3 ? 2 : 4);
  a.y = y, a.w = w, a.scale = scale, a.shift = shift, a.head = head;
  a.fit_icpt = fit_icpt, a.std_f = std_f, a.owlqn = enet != 0.0 && reg != 0.0;
  a.reg = reg, a.enet = enet, a.tol = tol, a.max_iter = max_iter, a.hist_cap = hist_cap;
  double* p = work;
  auto take = [&](int64_t n) {
    double* q = p;
    p += n;
    return q;
  };
  a.inv_sx = take(d), a.sx = take(d), a.mx = take(d), a.regw = take(d), a.l1 = take(d);
  a.x = take(d), a.g = take(d), a.ag = take(d), a.dir = take(d), a.cx = take(d), a.cg = take(d), a.cag = take(d);
  a.S = take((int64_t)kMem * d), a.Y = take((int64_t)kMem * d);
  a.part = take((int64_t)blocks * 8 * tpw * 32);
  a.lpart = take(2LL * blocks);
  a.dpart = take((int64_t)blocks * kDParts);
  a.scal = take(24);
  a.gbar = reinterpret_cast<unsigned*>(take(1));
  a.cs = reinterpret_cast<float*>(take((8LL * tpw * 32 + 1) / 2));
  a.mvec = take(x.n), a.dvec = take(x.n);
  if (dp) {
    a.red = take(d + 2);
    a.ctl = reinterpret_cast<Ctl*>(take(kCtlDoubles));
  }
  a.out = out;
  return a;
}

template <int L, int TPW>
const void* dp_pass_of() {
  return (const void*)lsq_qn_dp_pass_kernel<L, TPW>;
}

const void* pick_dp(int layout, int tpw) {
  if (layout == 2) {
    switch (tpw) {
      case 8: return dp_pass_of<2, 8>();
      case 16: return dp_pass_of<2, 16>();
      case 32: return dp_pass_of<2, 32>();
      default: return dp_pass_of<2, 64>();
    }
  }
  switch (tpw) {
    case 8: return dp_pass_of<3, 8>();
    case 16: return dp_pass_of<3, 16>();
    case 32: return dp_pass_of<3, 32>();
    default: return dp_pass_of<3, 64>();
  }
}

}  // namespace

void lsq_qn(const LsqX& x, const double* y, const double* w, const double* scale, const double* shift,
            const double* head, bool fit_icpt, bool std_f, double reg, double enet, int max_iter, double tol,
            int hist_cap, double* work, int blocks, double* out, hipStream_t st) {
  QnArgs a = make_args(x, y, w, scale, shift, head, fit_icpt, std_f, reg, enet, max_iter, tol, hist_cap, work, blocks,
                       out, false);
  void* args[] = {&a};
  // a plain launch of a co-resident grid (one block per CU, lsq_qn_blocks) with its own barrier
  DQ_HIP_CHECK(hipMemsetAsync(a.gbar, 0, 2 * sizeof(unsigned), st));
  DQ_HIP_CHECK(hipLaunchKernel(pick(x.layout, tpw_of(x.d)), dim3(blocks), dim3(kT), args, 0, st));
}

int64_t lsq_qn_dp_work(int d, int blocks, int64_t n) { return lsq_qn_work(d, blocks, n) + d + 2 + kCtlDoubles; }

int64_t lsq_qn_dp_red_offset(int d, int blocks, int64_t n) { return lsq_qn_work(d, blocks, n); }

int64_t lsq_qn_dp_ctl_offset(int d, int blocks, int64_t n) { return lsq_qn_work(d, blocks, n) + d + 2; }

void lsq_qn_dp(int phase, const LsqX& x, const double* y, const double* w, const double* scale, const double* shift,
               const double* head, bool fit_icpt, bool std_f, double reg, double enet, int max_iter, double tol,
               int hist_cap, double* work, int blocks, double* out, hipStream_t st) {
  QnArgs a = make_args(x, y, w, scale, shift, head, fit_icpt, std_f, reg, enet, max_iter, tol, hist_cap, work, blocks,
                       out, true);
  const int tpw = tpw_of(x.d), nc = 8 * tpw * 32;
  if (phase == 0) {  // start: mvec = dvec = 0 (x0), constants, the state, the first trial point
    DQ_HIP_CHECK(hipMemsetAsync(a.mvec, 0, 2 * (size_t)x.n * sizeof(double), st));
    hipLaunchKernelGGL(lsq_qn_dp_init_kernel, dim3(1), dim3(kT), 0, st, a, nc);
  } else if (phase == 1) {  // one evaluation's pass over this rank's rows + the slab fold -> red
    void* args[] = {&a};
    DQ_HIP_CHECK(hipLaunchKernel(pick_dp(x.layout, tpw), dim3(blocks), dim3(kT), args, 0, st));
    hipLaunchKernelGGL(lsq_qn_dp_fold_kernel, dim3((x.d + 63) / 64), dim3(kT), 0, st, a, blocks, nc);
  } else if (phase == 2) {  // the control step on the all-reduced red
    hipLaunchKernelGGL(lsq_qn_dp_ctl_kernel, dim3(1), dim3(kT), 0, st, a, nc);
  } else {
    throw std::invalid_argument("lsq_qn_dp: phase 0, 1 or 2");
  }
  DQ_HIP_CHECK(hipGetLastError());
}

}  // namespace dq4ml
