"""``models/lbfgsb.py`` -- Breeze 0.13 ``LBFGSB`` semantics -- against scipy's L-BFGS-B (the
Fortran reference implementation of the same Byrd-Lu-Nocedal-Zhu algorithm) on bound-constrained
problems, and the Huber fit that runs it against an independent fp64 oracle of Spark's objective."""
import numpy as np
import pytest
from scipy.optimize import minimize

from net.jgp.labs.sparkdq4ml_amd.models.lbfgsb import LBFGSB, PROJ_GRADIENT_EPS


def test_box_quadratic_solution_is_the_clamp():
    rng = np.random.default_rng(0)
    a = rng.normal(size=12) * 3
    lo, hi = np.full(12, -1.0), np.full(12, 1.5)
    opt = LBFGSB(lo, hi, max_iter=100, m=10, tolerance=1e-10)
    st, hist, why = opt.minimize(lambda x: (0.5 * float((x - a) @ (x - a)), x - a), np.zeros(12))
    np.testing.assert_allclose(st.x, np.clip(a, lo, hi), atol=1e-9)
    assert why in ("projected step converged", "gradient converged", "function values converged")
    assert all(b <= h + 1e-12 for h, b in zip(hist, hist[1:]))  # monotone


def _rosen(x):
    f = float(np.sum(100.0 * (x[1:] - x[:-1] ** 2) ** 2 + (1 - x[:-1]) ** 2))
    g = np.zeros_like(x)
    g[:-1] = -400 * x[:-1] * (x[1:] - x[:-1] ** 2) - 2 * (1 - x[:-1])
    g[1:] += 200 * (x[1:] - x[:-1] ** 2)
    return f, g


@pytest.mark.parametrize("n", [2, 6])
def test_bounded_rosenbrock_matches_scipy(n):
    lo = np.full(n, -2.0)
    hi = np.full(n, 2.0)
    hi[0] = 0.7  # an active bound at the optimum
    x0 = np.full(n, -1.2)
    st, hist, why = LBFGSB(lo, hi, max_iter=500, m=10, tolerance=1e-12).minimize(_rosen, x0)
    ref = minimize(_rosen, x0, jac=True, method="L-BFGS-B", bounds=list(zip(lo, hi)),
                   options=dict(maxiter=2000, ftol=1e-15, gtol=1e-12, maxcor=10))
    np.testing.assert_allclose(st.x, ref.x, atol=2e-5)
    assert st.x[0] == pytest.approx(0.7)  # on the bound, exactly (projection)
    assert hist[0] == pytest.approx(_rosen(x0)[0])


def test_first_direction_is_the_cauchy_step_and_bounds_hold():
    """Iteration 0 moves to the (projected) Cauchy point; every accepted iterate is in the box."""
    lo, hi = np.array([0.5, -np.inf]), np.array([np.inf, np.inf])
    seen = []
    opt = LBFGSB(lo, hi, max_iter=50, m=10, tolerance=1e-12)
    fg = lambda x: (0.5 * float(x @ x), x.copy())  # noqa: E731
    st, _, _ = opt.minimize(fg, np.array([3.0, 2.0]), on_state=lambda s, h: seen.append(s.x.copy()))
    assert all((p >= lo).all() for p in seen)
    np.testing.assert_allclose(st.x, [0.5, 0.0], atol=1e-8)
    pg = np.clip(st.x - st.grad, lo, hi) - st.x
    assert np.max(np.abs(pg)) <= max(PROJ_GRADIENT_EPS, 1e-8) or np.linalg.norm(st.grad[1:]) < 1e-8


def _huber_oracle(X, y, eps, reg, fit_icpt=True):
    """Spark's Huber objective (HuberAggregator + L2 on the std-scaled coefficients) minimized by
    scipy's L-BFGS-B from Spark's start (all ones) -- an independent fp64 oracle."""
    d, n = X.shape
    sx = X.std(axis=1)
    Xs = X / sx[:, None]

    @np.errstate(over="ignore", divide="ignore", invalid="ignore")  # (scipy probes tiny sigma)
    def fg(t):
        c, b, s = t[:d], (t[d] if fit_icpt else 0.0), t[-1]
        r = y - c @ Xs - b
        a = np.abs(r) <= eps * s
        loss = np.where(a, s + r * r / s, s + 2 * eps * np.abs(r) - eps * eps * s)
        f = 0.5 * loss.mean() + 0.5 * reg * float(c @ c)
        m = np.where(a, -2 * r / s, -2 * eps * np.sign(r))
        gc = 0.5 * (Xs @ m) / n + reg * c
        gb = 0.5 * m.mean()
        gs = 0.5 * np.where(a, 1 - (r / s) ** 2, 1 - eps * eps).mean()
        return f, np.concatenate([gc, [gb] if fit_icpt else [], [gs]])
    dim = d + (2 if fit_icpt else 1)
    bounds = [(None, None)] * (dim - 1) + [(5e-324, None)]
    res = minimize(fg, np.ones(dim), jac=True, method="L-BFGS-B", bounds=bounds,
                   options=dict(maxiter=5000, ftol=1e-16, gtol=1e-11, maxcor=10))
    t = res.x
    return t[:d] / sx, (t[d] if fit_icpt else 0.0), t[-1]


def test_huber_fit_matches_scipy_oracle(cpu_session):
    from net.jgp.labs.sparkdq4ml_amd import LinearRegression

    rng = np.random.default_rng(4)
    d, n = 5, 4000
    X = rng.normal(size=(d, n)) * np.array([[1.0], [2.0], [0.5], [3.0], [1.5]])
    beta = np.array([1.0, -2.0, 0.5, 0.25, 3.0])
    y = beta @ X + 1.5 + rng.standard_t(2, size=n) * 0.3
    df = cpu_session.createDataFrame({"features": X, "label": y})
    m = LinearRegression(loss="huber", maxIter=400, tol=1e-12, regParam=0.01).fit(df)
    coef, icpt, scale = _huber_oracle(X, y, 1.35, 0.01)
    np.testing.assert_allclose(m.coefficients.toArray(), coef, rtol=1e-5, atol=1e-6)
    assert m.intercept == pytest.approx(icpt, rel=1e-5, abs=1e-6)
    assert m.scale == pytest.approx(scale, rel=1e-5)
    h = np.asarray(m.summary.objectiveHistory)
    assert h.size == m.summary.totalIterations and h.size <= 400 + 1
    assert np.all(np.diff(h) <= 1e-12)  # strong-Wolfe steps decrease the objective
