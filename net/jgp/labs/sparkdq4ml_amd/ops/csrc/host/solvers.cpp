// Host f64 normal-equation solvers — see solvers.h for the behavioural contract.
//
// Line-search / convergence semantics follow Breeze 0.13 (the optimizer library bundled with
// Spark 2.4.4, POM:14): OWLQN = L-BFGS two-loop on the pseudo-gradient + orthant projection +
// backtracking line search seeded with 0.5/|g| on the first iteration; L-BFGS = strong-Wolfe
// cubic-interpolation search.  Convergence = max iterations || |f - max(last 20 f)| <= tol*|f0|
// || |adjusted gradient| <= max(tol*|f|, 1e-8) || search failed twice.
#include "solvers.h"

#include <algorithm>
#include <cmath>
#include <deque>
#include <limits>

namespace dq4ml {

namespace {

double dot(const std::vector<double>& a, const std::vector<double>& b) {
  double s = 0.0;
  for (size_t i = 0; i < a.size(); ++i) s += a[i] * b[i];
  return s;
}
double norm2(const std::vector<double>& a) { return std::sqrt(dot(a, a)); }
double signum(double v) { return v > 0 ? 1.0 : (v < 0 ? -1.0 : 0.0); }

struct FirstOrderException : std::runtime_error {
  explicit FirstOrderException(const std::string& m) : std::runtime_error(m) {}
};

// NormalEquationCostFun: f(x) = 1/2 bb - x.ab + 1/2 x^T aa x, grad = aa x - ab.  With an
// intercept the last coordinate is overwritten by bBar - coef.aBar on every evaluation
// (the cost function writes into the optimizer's vector in place).
struct CostFun {
  double bBar, bbBar;
  const std::vector<double>& ab;
  const std::vector<double>& aa;
  const std::vector<double>& aBar;
  bool fit_intercept;
  int nf;
  int k;
  // cache of the last evaluation (Breeze CachedDiffFunction)
  std::vector<double> last_x;
  double last_v = 0.0;
  std::vector<double> last_g;
  bool has_last = false;

  double calculate(std::vector<double>& x, std::vector<double>& g) {
    if (has_last && x == last_x) {
      g = last_g;
      return last_v;
    }
    if (fit_intercept) {
      double dp = 0.0;
      for (int j = 0; j < nf; ++j) dp += x[j] * aBar[j];
      x[nf] = bBar - dp;
    }
    std::vector<double> aax(k, 0.0);
    dspmv(k, aa.data(), x.data(), aax.data());
    double loss = 0.5 * bbBar - dot(ab, x) + 0.5 * dot(x, aax);
    for (int i = 0; i < k; ++i) aax[i] -= ab[i];
    g = aax;
    last_x = x;
    last_v = loss;
    last_g = g;
    has_last = true;
    return loss;
  }
};

struct History {
  int m;
  std::deque<std::vector<double>> s, y;  // most recent first
  // H * grad (two-loop recursion); returns the descent direction -H g
  std::vector<double> apply(const std::vector<double>& grad) const {
    double diag = 1.0;
    if (!s.empty()) {
      double sy = dot(s.front(), y.front());
      double yy = dot(y.front(), y.front());
      if (sy < 0 || std::isnan(sy)) throw FirstOrderException("NaNHistory");
      diag = sy / yy;
    }
    std::vector<double> dir = grad;
    const size_t h = s.size();
    std::vector<double> as(h), rho(h);
    for (size_t i = 0; i < h; ++i) {
      rho[i] = dot(s[i], y[i]);
      as[i] = dot(s[i], dir) / rho[i];
      if (std::isnan(as[i])) throw FirstOrderException("NaNHistory");
      for (size_t t = 0; t < dir.size(); ++t) dir[t] -= as[i] * y[i][t];
    }
    for (auto& v : dir) v *= diag;
    for (int i = static_cast<int>(h) - 1; i >= 0; --i) {
      double beta = dot(y[i], dir) / rho[i];
      for (size_t t = 0; t < dir.size(); ++t) dir[t] += (as[i] - beta) * s[i][t];
    }
    for (auto& v : dir) v = -v;
    return dir;
  }
  void update(const std::vector<double>& step, const std::vector<double>& gdelta) {
    s.push_front(step);
    y.push_front(gdelta);
    while (static_cast<int>(s.size()) > m) {
      s.pop_back();
      y.pop_back();
    }
  }
};

struct State {
  std::vector<double> x, grad, adj_grad;
  double value = 0, adj_value = 0, initial_adj_val = 0;
  int iter = 0;
  History hist;
  std::deque<double> fvals;  // FunctionValuesConverged info (starts with +inf)
  bool search_failed = false;
};

}  // namespace

void dspmv(int k, const double* ap, const double* x, double* y) {
  for (int i = 0; i < k; ++i) y[i] = 0.0;
  for (int j = 0; j < k; ++j) {
    const double* col = ap + static_cast<int64_t>(j) * (j + 1) / 2;
    double xj = x[j], acc = 0.0;
    for (int i = 0; i < j; ++i) {
      y[i] += col[i] * xj;
      acc += col[i] * x[i];
    }
    y[j] += col[j] * xj + acc;
  }
}

static std::vector<double> cholesky_factor(int k, const std::vector<double>& ap) {
  // A = U^T U, U upper, stored dense column-major k x k
  std::vector<double> u(static_cast<size_t>(k) * k, 0.0);
  for (int j = 0; j < k; ++j) {
    for (int i = 0; i <= j; ++i) u[i + static_cast<size_t>(j) * k] = ap[pk(i, j)];
  }
  for (int j = 0; j < k; ++j) {
    double* cj = &u[static_cast<size_t>(j) * k];
    for (int i = 0; i < j; ++i) {
      const double* ci = &u[static_cast<size_t>(i) * k];
      double s = cj[i];
      for (int t = 0; t < i; ++t) s -= ci[t] * cj[t];
      cj[i] = s / ci[i];
    }
    double d = cj[j];
    for (int t = 0; t < j; ++t) d -= cj[t] * cj[t];
    if (!(d > 0.0) || !std::isfinite(d)) {
      throw SingularMatrixError("LAPACK.dppsv returned " + std::to_string(j + 1) +
                                " because A is not positive definite. Is A derived from a singular matrix "
                                "(e.g. collinear column values)?");
    }
    cj[j] = std::sqrt(d);
  }
  return u;
}

std::vector<double> cholesky_solve(int k, const std::vector<double>& ap, const std::vector<double>& b) {
  auto u = cholesky_factor(k, ap);
  std::vector<double> z(b);
  for (int i = 0; i < k; ++i) {  // U^T z = b
    double s = z[i];
    for (int t = 0; t < i; ++t) s -= u[t + static_cast<size_t>(i) * k] * z[t];
    z[i] = s / u[i + static_cast<size_t>(i) * k];
  }
  for (int i = k - 1; i >= 0; --i) {  // U x = z
    double s = z[i];
    for (int t = i + 1; t < k; ++t) s -= u[i + static_cast<size_t>(t) * k] * z[t];
    z[i] = s / u[i + static_cast<size_t>(i) * k];
  }
  return z;
}

std::vector<double> cholesky_inverse(int k, const std::vector<double>& ap) {
  auto u = cholesky_factor(k, ap);
  // inv(U) (upper) then inv(A) = inv(U) inv(U)^T
  std::vector<double> ui(static_cast<size_t>(k) * k, 0.0);
  for (int j = 0; j < k; ++j) {
    ui[j + static_cast<size_t>(j) * k] = 1.0 / u[j + static_cast<size_t>(j) * k];
    for (int i = j - 1; i >= 0; --i) {
      double s = 0.0;
      for (int t = i + 1; t <= j; ++t) s += u[i + static_cast<size_t>(t) * k] * ui[t + static_cast<size_t>(j) * k];
      ui[i + static_cast<size_t>(j) * k] = -s / u[i + static_cast<size_t>(i) * k];
    }
  }
  std::vector<double> out(static_cast<size_t>(k) * (k + 1) / 2, 0.0);
  for (int j = 0; j < k; ++j) {
    for (int i = 0; i <= j; ++i) {
      double s = 0.0;
      for (int t = j; t < k; ++t) s += ui[i + static_cast<size_t>(t) * k] * ui[j + static_cast<size_t>(t) * k];
      out[pk(i, j)] = s;
    }
  }
  return out;
}

QNResult quasi_newton(double bBar, double bbBar, const std::vector<double>& ab,
                      const std::vector<double>& aa_packed, const std::vector<double>& aBar,
                      bool fit_intercept, int max_iter, double tol, const std::vector<double>& l1,
                      int memory) {
  const int nf = static_cast<int>(aBar.size());
  const int k = fit_intercept ? nf + 1 : nf;
  if (static_cast<int>(ab.size()) != k) throw std::invalid_argument("ab has wrong length");
  const bool owlqn = !l1.empty();
  if (owlqn && static_cast<int>(l1.size()) != k) throw std::invalid_argument("l1 has wrong length");
  const int fval_memory = 20;

  CostFun cf{bBar, bbBar, ab, aa_packed, aBar, fit_intercept, nf, k};

  auto adjust = [&](const std::vector<double>& x, const std::vector<double>& g, double v,
                    std::vector<double>& ag) -> double {
    ag = g;
    if (!owlqn) return v;
    double av = v;
    for (int i = 0; i < k; ++i) {
      const double l = l1[i];
      if (l == 0.0) continue;
      av += std::fabs(l * x[i]);
      if (x[i] == 0.0) {
        const double dp = g[i] + l, dm = g[i] - l;
        ag[i] = dm > 0 ? dm : (dp < 0 ? dp : 0.0);
      } else {
        ag[i] = g[i] + signum(x[i]) * l;
      }
    }
    return av;
  };

  State st;
  st.hist.m = memory;
  st.x.assign(k, 0.0);
  if (fit_intercept) st.x[k - 1] = bBar;
  st.value = cf.calculate(st.x, st.grad);
  st.adj_value = adjust(st.x, st.grad, st.value, st.adj_grad);
  st.initial_adj_val = st.adj_value;
  st.fvals.push_back(std::numeric_limits<double>::infinity());

  QNResult res;
  auto converged = [&](const State& s) -> std::string {
    if (max_iter >= 0 && s.iter >= max_iter) return "max iterations";
    if (s.fvals.size() >= 2) {
      double mx = -std::numeric_limits<double>::infinity();
      for (double v : s.fvals) mx = std::max(mx, v);
      if (std::fabs(s.adj_value - mx) <= tol * std::fabs(s.initial_adj_val)) return "function values converged";
    }
    if (norm2(s.adj_grad) <= std::max(tol * std::fabs(s.value), 1e-8)) return "gradient converged";
    if (s.search_failed) return "search failed";
    return "";
  };

  auto take_step = [&](const State& s, const std::vector<double>& dir, double a) {
    std::vector<double> nx(k);
    for (int i = 0; i < k; ++i) nx[i] = s.x[i] + dir[i] * a;
    if (owlqn) {
      for (int i = 0; i < k; ++i) {
        const double orth = s.x[i] != 0 ? signum(s.x[i]) : signum(-s.adj_grad[i]);
        if (signum(nx[i]) != orth) nx[i] = 0.0;
      }
    }
    return nx;
  };

  // phi(alpha) -> (value, derivative along dir), adjusted for OWLQN
  auto phi = [&](const State& s, const std::vector<double>& dir, double a, double& dd) {
    std::vector<double> nx = take_step(s, dir, a), g, ag;
    double v = cf.calculate(nx, g);
    double av = adjust(nx, g, v, ag);
    dd = dot(owlqn ? ag : g, dir);
    return owlqn ? av : v;
  };

  auto backtracking = [&](const State& s, const std::vector<double>& dir) {
    // Armijo reference: the regularized (adjusted) objective, consistent with the adjusted
    // directional derivative used below
    const double initfval = s.adj_value;
    const double shrink = s.iter < 1 ? 0.1 : 0.5, grow = 2.1, c1 = 1e-4, c2 = 0.9;
    double initd;
    phi(s, dir, 0.0, initd);
    double alpha = s.iter < 1 ? 0.5 / norm2(s.grad) : 1.0;
    double fd;
    double fv = phi(s, dir, alpha, fd);
    for (int it = 0;; ++it) {
      double mult;
      if (fv > initfval + alpha * initd * c1) mult = shrink;
      else if (fd < c2 * initd) mult = grow;
      else if (fd > -c2 * initd) mult = shrink;
      else mult = 1.0;
      if (mult == 1.0) return alpha;
      const double na = alpha * mult;
      if (it >= 20) throw FirstOrderException("LineSearchFailed");
      if (na < 1e-10) throw FirstOrderException("StepSizeUnderflow");
      if (na > 1e10) throw FirstOrderException("StepSizeOverflow");
      alpha = na;
      fv = phi(s, dir, alpha, fd);
      if (it + 1 >= 20) return alpha;  // takeWhile(iter < maxIterations) keeps the last state
    }
  };

  auto strong_wolfe = [&](const State& s, const std::vector<double>& dir) {
    struct B { double t, dd, f; };
    auto ev = [&](double t) { double d; double f = phi(s, dir, t, d); return B{t, d, f}; };
    const double c1 = 1e-4, c2 = 0.9;
    double t = s.iter == 0 ? 1.0 / norm2(dir) : 1.0;
    B low = ev(0.0);
    const double f0 = low.f, d0 = low.dd;
    if (d0 > 0) throw FirstOrderException("Line search invoked with non-descent direction");
    auto interp = [](const B& l, const B& r) {
      double d1 = l.dd + r.dd - 3 * (l.f - r.f) / (l.t - r.t);
      double d2 = std::sqrt(d1 * d1 - l.dd * r.dd);
      double mul = r.t - l.t;
      double tt = r.t - mul * (r.dd + d2 - d1) / (r.dd - l.dd + 2 * d2);
      double lb = l.t + 0.1 * mul, ub = l.t + 0.9 * mul;
      if (tt < lb) return lb;
      if (tt > ub) return ub;
      return tt;
    };
    auto zoom = [&](B lo, B hi) {
      for (int i = 0; i < 10; ++i) {
        double tt = lo.t > hi.t ? interp(hi, lo) : interp(lo, hi);
        B c = ev(tt);
        if (c.f > f0 + c1 * c.t * d0 || c.f >= lo.f) {
          hi = c;
        } else {
          if (std::fabs(c.dd) <= c2 * std::fabs(d0)) return c.t;
          if (c.dd * (hi.t - lo.t) >= 0) hi = lo;
          lo = c;
        }
      }
      throw FirstOrderException("Line search zoom failed");
    };
    for (int i = 0; i < 10; ++i) {
      B c = ev(t);
      if (!std::isfinite(c.f)) {
        t /= 2.0;
        continue;
      }
      if (c.f > f0 + c1 * t * d0 || (c.f >= low.f && i > 0)) return zoom(low, c);
      if (std::fabs(c.dd) <= c2 * std::fabs(d0)) return c.t;
      if (c.dd >= 0) return zoom(c, low);
      low = c;
      t *= 1.5;
    }
    throw FirstOrderException("Line search failed");
  };

  res.objective_history.push_back(st.adj_value);
  std::string why = converged(st);
  bool failed_once = false;
  while (why.empty()) {
    try {
      std::vector<double> dir = st.hist.apply(owlqn ? st.adj_grad : st.grad);
      if (owlqn) {
        for (int i = 0; i < k; ++i)
          if (!(dir[i] * st.adj_grad[i] < 0)) dir[i] = 0.0;
      }
      double step;
      if (owlqn) {
        step = backtracking(st, dir);
      } else {
        step = strong_wolfe(st, dir);
        if (step * norm2(st.grad) < 1e-10) throw FirstOrderException("StepSizeUnderflow");
      }
      std::vector<double> x = take_step(st, dir, step), g, ag;
      double v = cf.calculate(x, g);
      double av = adjust(x, g, v, ag);
      std::vector<double> sdiff(k), gdiff(k);
      for (int i = 0; i < k; ++i) {
        sdiff[i] = x[i] - st.x[i];
        gdiff[i] = g[i] - st.grad[i];
      }
      st.hist.update(sdiff, gdiff);
      st.fvals.push_back(v);
      while (static_cast<int>(st.fvals.size()) > fval_memory) st.fvals.pop_front();
      st.x = x;
      st.value = v;
      st.grad = g;
      st.adj_value = av;
      st.adj_grad = ag;
      st.iter += 1;
      failed_once = false;
    } catch (const FirstOrderException&) {
      if (!failed_once) {
        failed_once = true;
        st.hist.s.clear();
        st.hist.y.clear();
      } else {
        st.search_failed = true;
      }
    }
    res.objective_history.push_back(st.adj_value);
    why = converged(st);
  }
  res.x = st.x;
  res.converged_reason = why;
  return res;
}

}  // namespace dq4ml
