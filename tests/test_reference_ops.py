"""CPU tests of the PyTorch reference ops (the oracle the HIP kernels are checked against)."""
import math

import numpy as np
import pytest
import torch

from multigpu_advectiondiffusion_amd.ops import reference as ref


def test_weno5_single_division_equals_textbook():
    g = torch.Generator().manual_seed(0)
    v = [torch.randn(20000, generator=g, dtype=torch.float64) for _ in range(5)]
    # include smooth and discontinuous stencils
    v[3][:5000] = v[2][:5000] + 1e-3
    v[4][5000:10000] = 5.0
    for z in (False, True):
        a = ref.weno5(*v, z=z)
        b = ref.weno5_textbook(*v, z=z)
        assert torch.allclose(a, b, rtol=1e-12, atol=1e-13), (a - b).abs().max()


def test_weno5_reproduces_polynomials_exactly():
    # on smooth data the nonlinear weights tend to the linear ones: exact for quadratics
    x = torch.arange(-2, 3, dtype=torch.float64)
    for c in (0.0, 1.0, -3.0):
        vals = [torch.tensor([1.0 + 2.0 * xi + c * 0.0]) for xi in x]  # linear function
        for z in (False, True):
            r = ref.weno5(*vals, z=z)
            assert math.isclose(r.item(), 1.0 + 2.0 * 0.5, rel_tol=1e-12)


def test_weno5_fifth_order_on_smooth_data():
    # cell-point values of sin; reconstruct at x_{i+1/2}; error must drop ~h^5
    errs = []
    for n in (40, 80, 160):
        h = 2 * math.pi / n
        xi = torch.arange(n, dtype=torch.float64) * h + 0.3
        f = torch.sin
        vs = [f(xi + k * h) for k in (-2, -1, 0, 1, 2)]
        # finite-difference WENO reconstructs the flux h such that (h_{i+1/2}-h_{i-1/2})/h = f'
        hp = ref.weno5(*vs, z=True)
        hm = ref.weno5(*[f(xi + (k - 1) * h) for k in (-2, -1, 0, 1, 2)], z=True)
        deriv = (hp - hm) / h
        errs.append((deriv - torch.cos(xi)).abs().max().item())
    o1 = math.log2(errs[0] / errs[1])
    o2 = math.log2(errs[1] / errs[2])
    assert o1 > 4.5 and o2 > 4.5, errs


def test_lf_split_sums_to_flux():
    u = torch.linspace(-2, 2, 101, dtype=torch.float64)
    fp, fm = ref.lf_split(u)
    assert torch.allclose(fp + fm, 0.5 * u * u)
    # f+ is non-decreasing and f- non-increasing in u (upwind splitting)
    assert torch.all(fp.diff() >= -1e-15) and torch.all(fm.diff() <= 1e-15)


def _np_fd4_lap3(u, B, k0, k1, cx, cy, cz):
    """Plain numpy loop-free FD4 Laplacian for cross-checking the torch reference."""
    out = np.zeros_like(u)
    nz, ny, nx = u.shape
    for k in range(k0, k1):
        for j in range(B, ny - B):
            row = u[k, j]
            i = np.arange(B, nx - B)
            d2x = (-row[i - 2] + 16 * row[i - 1] - 30 * row[i] + 16 * row[i + 1] - row[i + 2]) / 12
            d2y = (-u[k, j - 2, i] + 16 * u[k, j - 1, i] - 30 * u[k, j, i] + 16 * u[k, j + 1, i]
                   - u[k, j + 2, i]) / 12
            d2z = (-u[k - 2, j, i] + 16 * u[k - 1, j, i] - 30 * u[k, j, i] + 16 * u[k + 1, j, i]
                   - u[k + 2, j, i]) / 12
            out[k, j, i] = cx * d2x + cy * d2y + cz * d2z
    return out


def test_diffusion3d_reference_matches_numpy_loop():
    g = np.random.default_rng(1)
    u = g.random((12, 10, 11))
    u0 = g.random((12, 10, 11))
    out = torch.zeros((12, 10, 11), dtype=torch.float64)
    B, k0, k1 = 2, 2, 10
    ref.diffusion3d_stage(torch.from_numpy(u), torch.from_numpy(u0), out, 11, 10, k0, k1, B, 4,
                          0.5, 0.7, 0.9, 0.01, 0.75, 0.25)
    lap = _np_fd4_lap3(u, B, k0, k1, 0.5, 0.7, 0.9)
    exp = np.zeros_like(u)
    exp[k0:k1, B:-B, B:-B] = 0.75 * u0[k0:k1, B:-B, B:-B] + 0.25 * (
        u[k0:k1, B:-B, B:-B] + 0.01 * lap[k0:k1, B:-B, B:-B])
    assert np.allclose(out.numpy(), exp, rtol=1e-13, atol=1e-14)


def test_fd4_laplacian_is_fourth_order():
    errs = []
    for n in (16, 32, 64):
        h = 1.0 / n
        x = torch.arange(n + 1, dtype=torch.float64) * h
        u = torch.sin(2 * x).view(1, 1, -1).expand(5, 5, -1).contiguous()
        u = u.clone()
        out = torch.zeros_like(u)
        # stage with dt=1, a=0, b=1 and "in" = u -> out = u + L(u); L only along x here
        ref.diffusion3d_stage(u, None, out, n + 1, 5, 2, 3, 2, 4, 1.0 / h ** 2, 0.0, 0.0, 1.0,
                              0.0, 1.0)
        # rows restricted by border in y; take the middle row
        lap = (out - u)[2, 2, 2:n - 1]
        exact = -4 * torch.sin(2 * x[2:n - 1])
        errs.append((lap - exact).abs().max().item())
    assert math.log2(errs[0] / errs[1]) > 3.7 and math.log2(errs[1] / errs[2]) > 3.7, errs


def test_burgers_rhs_conservative_telescoping():
    # with zero border fluxes, Σ L = -(F_right - F_left)/dx ... check the discrete
    # conservation: sum of -dF over a row equals -(F_last - F_first)
    g = torch.Generator().manual_seed(3)
    u = 0.2 * torch.randn((1, 12, 40), generator=g, dtype=torch.float64)
    L = ref.burgers_rhs_2d(u[0], 40, 3, 9, 3, True, 1.0, 0.0, 0.0, 0.0)
    fp, fm = ref.lf_split(u[0])
    F = ref._faces_last_axis(fp[3:9], fm[3:9], 2, 37, True)
    assert torch.allclose(L.sum(-1), -(F[:, -1] - F[:, 0]), atol=1e-13)


@pytest.mark.parametrize("z", [False, True])
def test_burgers3d_reference_axis_symmetry(z):
    """A field that depends only on x must give the same RHS as the same field along y/z."""
    n = 20
    x = torch.linspace(-1, 1, n, dtype=torch.float64)
    f = torch.exp(-x ** 2 / 0.1) + 0.1
    ux = f.view(1, 1, n).expand(n, n, n).contiguous()
    uy = f.view(1, n, 1).expand(n, n, n).contiguous()
    uz = f.view(n, 1, 1).expand(n, n, n).contiguous()
    kw = dict(nx=n, ny=n, k0=3, k1=n - 3, border=3, weno_z=z, rdx=2.0, rdy=2.0, rdz=2.0,
              vx=0.0, vy=0.0, vz=0.0)
    Lx = ref.burgers_rhs_3d(ux, **kw)
    Ly = ref.burgers_rhs_3d(uy, **kw)
    Lz = ref.burgers_rhs_3d(uz, **kw)
    assert torch.allclose(Lx[5, 5, :], Ly[5, :, 5], atol=1e-14)
    assert torch.allclose(Lx[5, 5, :], Lz[:, 5, 5], atol=1e-14)


def test_two_step_fallback_and_solver_pairing(monkeypatch):
    """CPU semantics of the two-step FD2 launch (ops/stencil.py::diffusion3d_step2x: two
    reference steps through a scratch field) and the solver's step pairing (eager, odd
    counts, t_end runs): identical to one step per launch."""
    from multigpu_advectiondiffusion_amd.models.base import Grid
    from multigpu_advectiondiffusion_amd.models.diffusion import Diffusion
    from multigpu_advectiondiffusion_amd.ops import stencil
    from multigpu_advectiondiffusion_amd.solver import Solver

    g = torch.Generator().manual_seed(3)
    u = torch.rand((20, 17, 19), generator=g, dtype=torch.float64)
    c, dt = (0.2, 0.15, 0.1), 0.9 / (2 * 0.45)
    kw = dict(nx=19, ny=17, zlo=1, zhi=19, border=1, cx=c[0], cy=c[1], cz=c[2], dt=dt)
    got = u.clone()
    stencil.diffusion3d_step2x(u, got, k0=1, k1=19, **kw)
    mid, exp = u.clone(), u.clone()
    for a, b in ((u, mid), (mid, exp)):
        stencil.diffusion3d_step(a, b, k0=1, k1=19, order=2, **kw)
    assert torch.equal(got, exp)

    def run(flag, **rk):
        monkeypatch.setenv("ADVDIFF_STEP2", flag)
        s = Solver(Diffusion(order=2), Grid((19, 17, 20), (1.0, 1.0, 1.0)), device="cpu")
        assert s.step2_capable() == (flag == "1")
        s.run(**rk)
        return s.owned.clone(), s.it, s.t

    for rk in (dict(iters=5), dict(t_end=0.05)):
        a, ita, ta = run("1", **rk)
        b, itb, tb = run("0", **rk)
        assert (ita, ta) == (itb, tb)
        assert torch.equal(a, b)
