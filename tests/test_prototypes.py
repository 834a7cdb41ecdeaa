"""CPU ports of the MATLAB prototypes (the reference's only quantitative tests)."""
import math

import numpy as np
import pytest

from multigpu_advectiondiffusion_amd.models import prototypes as P

# Matlab_Prototipes/DiffusionNd/TestingAccuracy.log:49-72 (n, L1, OOA, Linf, OOA)
LOG = {
    1: [(10, 1.81e-01, 0.00, 4.97e-02, 0.00), (20, 4.87e-02, 1.89, 1.34e-02, 1.90),
        (40, 9.89e-03, 2.30, 2.62e-03, 2.35), (80, 1.50e-03, 2.72, 8.34e-04, 1.65)],
    2: [(10, 2.97e-01, 0.00, 2.65e-02, 0.00), (20, 3.42e-02, 3.12, 2.96e-03, 3.17),
        (40, 5.14e-03, 2.73, 3.59e-04, 3.04), (80, 2.99e-03, 0.78, 2.64e-04, 0.45)],
    3: [(10, 3.99e-01, 0.00, 7.31e-03, 0.00), (20, 2.75e-02, 3.86, 5.04e-04, 3.86),
        (40, 1.35e-02, 1.02, 3.29e-04, 0.61), (80, 4.70e-03, 1.52, 8.33e-05, 1.98)],
}


@pytest.mark.parametrize("dims", [1, 2, 3])
def test_testing_accuracy_reproduces_reference_log(dims):
    res = P.testing_accuracy(dims=(dims,))[dims]
    for got, exp in zip(res, LOG[dims]):
        assert got[0] == exp[0]
        for g, e, tol in ((got[1], exp[1], 0.006), (got[3], exp[3], 0.006)):
            assert abs(g - e) <= tol * e + 1e-300, (dims, got, exp)  # 3 significant digits
        assert abs(got[2] - exp[2]) < 0.006 and abs(got[4] - exp[4]) < 0.006, (dims, got, exp)


def test_accuracy_table_format():
    txt = P.format_accuracy_table({1: [(10, 0.181, 0.0, 0.0497, 0.0)]})
    assert " Heat solver 1 D" in txt and " 10 \t 1.81e-01 \t 0.00 \t\t 4.97e-02 \t 0.00 " in txt


def test_axisymmetric_heat_matches_exact():
    l1, l2, linf, u, uE, r = P.heat2d_axisymmetric(nr=64, ny=16)
    assert linf < 2e-2 and l1 < 0.5
    # the mirror BC keeps the solution y-independent
    assert np.allclose(u[2], u[-3])


def test_common_ic_cases():
    x = np.linspace(-1, 1, 201)
    for c in range(1, 11):
        u = P.common_ic(x, c)
        assert u.shape == x.shape and np.all(np.isfinite(u))
    assert P.common_ic(x, 6)[0] == 2.0 and P.common_ic(x, 6)[-1] == 1.0
    sq = P.common_ic(x, 8)
    assert sq.max() == 2.0 and sq.min() == 1.0
    with pytest.raises(ValueError):
        P.common_ic(x, 11)


@pytest.mark.parametrize("order,res", [(5, P.weno5_res), (7, P.weno7_res)])
def test_weno_residual_order_on_smooth_data(order, res):
    errs = []
    flux = P.Flux("linear")
    for n in (41, 81, 161):
        x = np.linspace(-1, 1, n)
        dx = x[1] - x[0]
        u = np.sin(np.pi * x) + 2.0
        r = res(u, flux, dx, global_lf=True)
        inner = slice(3 * n // 8, 5 * n // 8)  # away from the critical points x = ±1/2
        errs.append(np.abs(r[inner] - np.pi * np.cos(np.pi * x[inner])).max())
    o = math.log2(errs[0] / errs[1]), math.log2(errs[1] / errs[2])
    assert min(o) > order - 0.7, (order, errs, o)


def test_weno5_axis_invariance():
    x = np.linspace(-1, 1, 30)
    f = np.exp(-20 * x ** 2)
    fl = P.Flux("burgers")
    r1 = P.weno5_res(f, fl, x[1] - x[0])
    u2 = np.tile(f[:, None], (1, 7))
    r2 = P.weno5_res(u2, fl, x[1] - x[0], axis=0)
    assert np.allclose(r2[:, 3], r1)


@pytest.mark.parametrize("order", [5, 7])
def test_lf_weno_burgers_shock_is_nonoscillatory(order):
    x = np.linspace(-1, 1, 101)
    u0 = P.common_ic(x, 6)  # Riemann problem 2 -> 1 (shock moving right at speed 1.5)
    u, t, it = P.lf_weno_fdm(u0, (x[1] - x[0],), 0.3, 0.3, "burgers", order=order)
    assert abs(t - 0.3) < 1e-14
    # (the prototype's first face flux is zero, so the leftmost cells drain: skip them)
    inner = u[x > -0.2]
    assert inner.max() < 2.0 + 2e-3 and inner.min() > 1.0 - 2e-3
    xs = x[np.argmin(np.abs(u - 1.5))]
    assert abs(xs - 0.45) < 0.05  # Rankine-Hugoniot: x_s = 1.5 t


def test_lsrk45_is_fourth_order():
    # u' = -u with the 5-stage low-storage scheme
    def run(h):
        u, res = 1.0, 0.0
        for _ in range(int(round(1 / h))):
            for a, b in zip(P.LSRK45_A, P.LSRK45_B):
                res = a * res + h * u   # residual convention of the prototypes: dF = +u
                u = u - b * res
        return abs(u - math.exp(-1))
    e1, e2 = run(0.1), run(0.05)
    assert math.log2(e1 / e2) > 3.8


def test_lf_weno_2d_3d_run():
    x = np.linspace(-1, 1, 24)
    X, Y = np.meshgrid(x, x, indexing="ij")
    u0 = np.exp(-(X ** 2 + Y ** 2) / 0.1)
    u, t, it = P.lf_weno_fdm(u0, (x[1] - x[0],) * 2, 0.1, 0.4, "burgers", order=5)
    assert np.all(np.isfinite(u)) and it > 2
    z = np.linspace(-1, 1, 16)
    X3, Y3, Z3 = np.meshgrid(z, z, z, indexing="ij")
    u3 = 0.2 + 0.5 * np.exp(-(X3 ** 2 + Y3 ** 2 + Z3 ** 2) / 0.1)
    u, t, it = P.lf_weno_fdm(u3, (z[1] - z[0],) * 3, 0.5, 0.3, "buckley", order=7, max_steps=3)
    assert np.all(np.isfinite(u)) and it == 3
