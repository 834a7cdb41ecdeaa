"""WENO7 reconstruction and the low-storage RK4(5) integrator (CPU).

Parity anchors: the MATLAB prototypes `Matlab_Prototipes/InviscidBurgersNd/WENO7resAdv*.m`
(WENO7-JS, local Lax–Friedrichs split per axis) and `LFWENO7FDM{1,2,3}d.m` (LSRK4(5)
time loop), ported in ``models/prototypes.py``.  Their boundary treatment (constant
extrapolation) differs from the solver's frozen Dirichlet layer, so comparisons are on
cells whose stencils never reach a boundary."""
import numpy as np
import pytest
import torch

from multigpu_advectiondiffusion_amd import Burgers, Diffusion, Grid, Solver
from multigpu_advectiondiffusion_amd.launch import spawn_local
from multigpu_advectiondiffusion_amd.models import prototypes as mp
from multigpu_advectiondiffusion_amd.ops import reference as ref


def _field2(ny, nx, seed=0):
    g = np.random.default_rng(seed)
    y, x = np.meshgrid(np.linspace(0, 2, ny), np.linspace(0, 2, nx), indexing="ij")
    u = np.exp(-((x - 1) ** 2 + (y - 0.9) ** 2) / 0.1) - 0.4 * np.tanh(8 * (x - 1.3))
    return u + 0.01 * g.standard_normal(u.shape)


def test_weno7_rhs_matches_matlab_port_2d():
    ny, nx = 40, 52
    dx, dy = 2.0 / (nx - 1), 2.0 / (ny - 1)
    u = _field2(ny, nx)
    fl = mp.Flux("burgers")
    res = mp.weno7_res(u, fl, dx, axis=1) + mp.weno7_res(u, fl, dy, axis=0)
    B = 4
    L = ref.burgers_rhs_2d(torch.from_numpy(u), nx, B, ny - B, B, "js7", 1 / dx, 1 / dy, 0.0, 0.0)
    m = 8  # cells whose 9-point stencils stay away from the padded MATLAB boundary
    got = -L.numpy()[m - B:ny - m - B, m - B:nx - m - B]  # L[r, c] is cell (B+r, B+c)
    exp = res[m:ny - m, m:nx - m]
    np.testing.assert_allclose(got, exp, rtol=1e-11, atol=1e-11 * np.abs(exp).max())


def test_weno7_converges_7th_order_1d_smooth():
    errs = []
    for n in (40, 80):
        x = np.linspace(0, 2 * np.pi, n + 1)[:-1]
        h = x[1] - x[0]
        # linear flux, periodic: compare the reconstructed derivative with cos
        w = np.sin(x)
        wp = np.concatenate([w[-4:], w, w[:4]])  # cell i at padded index i+4
        fl = mp.Flux("linear")
        V, U = mp._split(wp, fl, True)
        fp, fm = torch.from_numpy(V), torch.from_numpy(U)
        F = ref._faces_last_axis(fp, fm, 3, n + 4, "js7")  # faces right of padded 3..n+3
        d = ((F[1:] - F[:-1]) / h).numpy()
        away = np.abs(np.cos(x)) > 0.7  # JS weights lose order at critical points
        errs.append(np.abs(d - np.cos(x))[away].max())
    assert np.log2(errs[0] / errs[1]) > 6.0, errs


def test_lsrk45_weno7_solver_matches_matlab_time_loop():
    nx, ny = 44, 44  # dx = dy: the MATLAB loop's dt uses the first spacing
    g = Grid((nx, ny), (2.0, 2.0))
    model = Burgers(viscosity=0.0, weno="js7", cfl=0.4, cfl_mode="adaptive")
    s = Solver(model, g, dtype=torch.float64, device="cpu", ic="gaussian",
               integrator="lsrk45")
    u0 = s.gather().copy()
    steps = 4
    s.run(iters=steps)
    # MATLAB loop: dt = CFL*dx/max|u| (dx = min spacing here), LSRK4(5) stages
    u_ml, t_ml, it = mp.lf_weno_fdm(u0, (g.spacing[1], g.spacing[0]), 10.0, 0.4, "burgers",
                                    order=7, max_steps=steps)
    assert it == steps and abs(t_ml - s.t) < 1e-14
    m = 10
    np.testing.assert_allclose(s.gather()[m:-m, m:-m], u_ml[m:-m, m:-m], rtol=0, atol=1e-12)


def test_lsrk45_heat_is_4th_order_in_time():
    # exact sine-mode decay; time error dominates with a large dt and FD4 in space
    errs = []
    for nsteps in (8, 16):
        g = Grid((24, 24, 24), (1.0, 1.0, 1.0))
        model = Diffusion(K=1.0, order=4)
        s = Solver(model, g, dtype=torch.float64, device="cpu", ic="sine", integrator="lsrk45")
        T = 0.002  # dt = T/8 sits at the explicit stability limit
        s.run(iters=nsteps, dt=T / nsteps)
        s2 = Solver(model, g, dtype=torch.float64, device="cpu", ic="sine", integrator="lsrk45")
        s2.run(iters=nsteps * 8, dt=T / (nsteps * 8))  # temporal reference
        errs.append(np.abs(s.gather() - s2.gather()).max())
    assert np.log2(errs[0] / errs[1]) > 3.5, errs


def _run(comm, kind, steps, decomp):
    if kind == "burg3w7":
        model, grid, ic = Burgers(viscosity=1e-3, weno="js7", cfl=0.3), Grid((22, 19, 27), (2.0, 2.0, 2.0)), "gaussian"
    elif kind == "burg2w7":
        model, grid, ic = Burgers(viscosity=0.0, weno="js7", cfl=0.3), Grid((30, 33), (2.0, 2.0)), "gaussian"
    else:
        model, grid, ic = Diffusion(K=1.0, order=4), Grid((20, 18, 23), (1.0, 1.0, 1.0)), "sine"
    s = Solver(model, grid, comm, dtype=torch.float64, device="cpu", ic=ic,
               integrator="lsrk45", decomp=decomp)
    s.run(iters=steps)
    g = s.gather()
    return None if g is None else g.copy()


@pytest.mark.parametrize("kind,world,decomp", [
    ("burg3w7", 2, None), ("burg3w7", 4, (1, 2, 2)), ("burg2w7", 3, None),
    ("diff3ls", 3, None), ("diff3ls", 4, (2, 1, 2)),
])
def test_lsrk45_weno7_decomposition_bitwise(kind, world, decomp):
    serial = spawn_local(1, _run, kind, 3, None)[0]
    out = spawn_local(world, _run, kind, 3, decomp)[0]
    assert np.array_equal(out, serial), np.abs(out - serial).max()
