"""WENO7 and low-storage RK (LSRK4(5)) stage kernels vs the PyTorch fp64 reference, and
the GPU solver paths that use them (single rank and multi-rank on one GPU)."""
import numpy as np
import pytest
import torch

from multigpu_advectiondiffusion_amd import Burgers, Diffusion, Grid, Solver
from multigpu_advectiondiffusion_amd.launch import spawn_local
from multigpu_advectiondiffusion_amd.ops import reference as ref, stencil

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _smooth(shape, seed, dtype):
    g = torch.Generator().manual_seed(seed)
    base = torch.rand(shape, generator=g, dtype=torch.float64)
    idx = torch.meshgrid(*[torch.linspace(0, 3, n, dtype=torch.float64) for n in shape],
                         indexing="ij")
    s = sum(torch.sin((i + 1) * x) for i, x in enumerate(idx))
    return (0.6 * s + 0.3 * base).to(dtype)


def _tol(dtype, scale=None):
    """fp64: to rounding of the reference.  fp32: error-scaled — 64 rounding steps of at
    most one ulp of `scale`, the op's sum of absolute terms (see _scale), instead of the
    absolute 5e-4 of rounds 1-5 (~1e3 ulps on O(1) data)."""
    if dtype == torch.float64:
        return 1e-11
    return 64 * 2.0 ** -23 * scale


def _scale(inp, aux, a, b, dt, rd, vv, stencil_sum):
    """|a aux| + |b| (max|inp| + dt L_abs): L_abs = per axis 2 rd max|F| (Σ|candidate
    coefficients|) + vv Σ|w_FD4| max|u| (heat: stencil_sum=Σ|w| of the Laplacian and
    F = u)."""
    m = lambda t: t.double().abs().max().item()  # noqa: E731
    fmax = m(inp) ** 2 / 2 if stencil_sum is None else m(inp)
    w = 64.0 / 12.0 if stencil_sum is None else stencil_sum
    adv = sum(2 * r * fmax * (64.0 / 12.0) for r in rd) if stencil_sum is None else \
        sum(r * w * fmax for r in rd)
    visc = sum(v * (64.0 / 12.0) * m(inp) for v in vv)
    Lmax = dt * (adv + visc)
    return abs(a) * m(aux) + abs(b) * (m(inp) + Lmax) + Lmax + m(aux)


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
@pytest.mark.parametrize("visc", [0.0, 0.02])
@pytest.mark.parametrize("mode", ["ssp1", "ssp", "ls1", "ls"])
def test_burgers3d_weno7_stage(dtype, visc, mode):
    nz, ny, nx, sx = 26, 37, 70, 72
    inp, aux, out = (_smooth((nz, ny, sx), s, dtype) for s in (1, 2, 3))
    ls = mode.startswith("ls")
    a, b = {"ssp1": (0.0, 1.0), "ssp": (0.75, 0.25), "ls1": (0.0, 0.15), "ls": (-0.4, 0.37)}[mode]
    border, k0, k1 = 4, 4, nz - 4
    rd = (1 / 0.02, 1 / 0.03, 1 / 0.025)
    vv = tuple(visc * r * r for r in rd)
    exp_out, exp_aux = out.double().clone(), aux.double().clone()
    ref.burgers3d_stage(inp.double(), exp_aux, exp_out, nx, ny, k0, k1, border, "js7", *rd, *vv,
                        1e-3, a, b, ls)
    g_aux, g_out = aux.to(DEV), out.to(DEV)
    stencil.burgers3d_stage(inp.to(DEV), g_aux, g_out, nx=nx, ny=ny, k0=k0, k1=k1, border=border,
                            weno_z="js7", rdx=rd[0], rdy=rd[1], rdz=rd[2], vx=vv[0], vy=vv[1],
                            vz=vv[2], dt=1e-3, a=a, b=b, ls=ls)
    torch.cuda.synchronize()
    sc = _scale(inp, aux, a, b, 1e-3, rd, vv, None)
    assert (g_out.cpu().double() - exp_out).abs().max().item() < _tol(dtype, sc)
    assert (g_aux.cpu().double() - exp_aux).abs().max().item() < _tol(dtype, sc)


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
@pytest.mark.parametrize("weno", ["js", "z", "js7"])
@pytest.mark.parametrize("mode", ["ssp", "ls1", "ls"])
def test_burgers2d_stage_schemes(dtype, weno, mode):
    ny, nx, sx = 45, 300, 320
    inp, aux, out = (_smooth((ny, sx), s, dtype) for s in (4, 5, 6))
    ls = mode.startswith("ls")
    a, b = {"ssp": (0.75, 0.25), "ls1": (0.0, 0.15), "ls": (-0.4, 0.37)}[mode]
    R = 4 if weno == "js7" else 3
    rd = (1 / 0.01, 1 / 0.02)
    vv = (0.01 * rd[0] ** 2, 0.01 * rd[1] ** 2)
    exp_out, exp_aux = out.double().clone(), aux.double().clone()
    ref.burgers2d_stage(inp.double(), exp_aux, exp_out, nx, R, ny - R, R, weno, *rd, *vv, 1e-3,
                        a, b, ls)
    g_aux, g_out = aux.to(DEV), out.to(DEV)
    stencil.burgers2d_stage(inp.to(DEV), g_aux, g_out, nx=nx, j0=R, j1=ny - R, border=R,
                            weno_z=weno, rdx=rd[0], rdy=rd[1], vx=vv[0], vy=vv[1], dt=1e-3,
                            a=a, b=b, ls=ls)
    torch.cuda.synchronize()
    sc = _scale(inp, aux, a, b, 1e-3, rd, vv, None)
    assert (g_out.cpu().double() - exp_out).abs().max().item() < _tol(dtype, sc)
    assert (g_aux.cpu().double() - exp_aux).abs().max().item() < _tol(dtype, sc)


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
@pytest.mark.parametrize("order", [4, 2])
@pytest.mark.parametrize("mode", ["ls1", "ls"])
def test_diffusion_ls_stages(dtype, order, mode):
    a, b = {"ls1": (0.0, 0.15), "ls": (-0.4, 0.37)}[mode]
    R = order // 2
    # 3-D
    nz, ny, nx, sx = 30, 41, 70, 72
    inp, aux, out = (_smooth((nz, ny, sx), s, dtype) for s in (7, 8, 9))
    eo, ea = out.double().clone(), aux.double().clone()
    ref.diffusion3d_stage(inp.double(), ea, eo, nx, ny, R, nz - R, R, order, 3.0, 2.0, 1.0,
                          1e-3, a, b, True)
    ga, go = aux.to(DEV), out.to(DEV)
    stencil.diffusion3d_stage(inp.to(DEV), ga, go, nx=nx, ny=ny, k0=R, k1=nz - R, border=R,
                              order=order, cx=3.0, cy=2.0, cz=1.0, dt=1e-3, a=a, b=b, ls=True)
    torch.cuda.synchronize()
    W = 64.0 / 12.0 if order == 4 else 4.0
    sc = _scale(inp, aux, a, b, 1e-3, (3.0, 2.0, 1.0), (), W)
    assert (go.cpu().double() - eo).abs().max().item() < _tol(dtype, sc)
    assert (ga.cpu().double() - ea).abs().max().item() < _tol(dtype, sc)
    # 2-D
    ny, nx, sx = 50, 300, 320
    inp, aux, out = (_smooth((ny, sx), s, dtype) for s in (10, 11, 12))
    eo, ea = out.double().clone(), aux.double().clone()
    ref.diffusion2d_stage(inp.double(), ea, eo, nx, R, ny - R, R, order, 3.0, 2.0, 1e-3, a, b,
                          True)
    ga, go = aux.to(DEV), out.to(DEV)
    stencil.diffusion2d_stage(inp.to(DEV), ga, go, nx=nx, j0=R, j1=ny - R, border=R,
                              order=order, cx=3.0, cy=2.0, dt=1e-3, a=a, b=b, ls=True)
    torch.cuda.synchronize()
    sc = _scale(inp, aux, a, b, 1e-3, (3.0, 2.0), (), W)
    assert (go.cpu().double() - eo).abs().max().item() < _tol(dtype, sc)
    assert (ga.cpu().double() - ea).abs().max().item() < _tol(dtype, sc)


def _make(kind):
    if kind == "burg3w7":
        return Burgers(viscosity=1e-4, weno="js7", cfl=0.3), Grid((66, 35, 40), (2.0, 2.0, 2.0)), "gaussian"
    if kind == "burg2w7":
        return Burgers(viscosity=0.0, weno="js7", cfl=0.3), Grid((260, 57), (2.0, 2.0)), "gaussian"
    return Diffusion(K=1.0, order=4), Grid((70, 33, 41), (1.0, 1.0, 1.0)), "sine"


@pytest.mark.parametrize("kind", ["burg3w7", "burg2w7", "diff3"])
def test_gpu_lsrk45_solver_matches_cpu(kind):
    model, grid, ic = _make(kind)
    sg = Solver(model, grid, dtype=torch.float64, device="cuda", ic=ic, integrator="lsrk45")
    sg.run(iters=9)  # graph replay (8) + one eager step
    model, grid, ic = _make(kind)
    sc = Solver(model, grid, dtype=torch.float64, device="cpu", ic=ic, integrator="lsrk45")
    sc.run(iters=9)
    assert sg.it == sc.it == 9 and abs(sg.t - sc.t) < 1e-15
    np.testing.assert_allclose(sg.gather(), sc.gather(), rtol=0, atol=1e-11)


def _run(comm, kind, steps, decomp):
    model, grid, ic = _make(kind)
    s = Solver(model, grid, comm, dtype=torch.float64, ic=ic, integrator="lsrk45",
               decomp=decomp)
    s.run(iters=steps)
    g = s.gather()
    return None if g is None else g.copy()


@pytest.mark.parametrize("kind,world,decomp", [("burg3w7", 2, None), ("burg3w7", 4, (1, 2, 2)),
                                               ("burg2w7", 2, (1, 2)), ("diff3", 3, None)])
def test_gpu_lsrk45_multirank_bitwise(kind, world, decomp, monkeypatch):
    monkeypatch.setenv("ADVDIFF_SHARE_GPU", "1")
    model, grid, ic = _make(kind)
    s = Solver(model, grid, dtype=torch.float64, device="cuda", ic=ic, integrator="lsrk45")
    s.run(iters=4)
    ref_g = s.gather()
    out = spawn_local(world, _run, kind, 4, decomp, device="cuda", backend="gloo")[0]
    assert np.array_equal(out, ref_g), np.abs(out - ref_g).max()


def test_stage_aliasing_rules():
    """SSP stages may read u0 from the input buffer; LSRK stages must not alias du."""
    n = 24
    u = _smooth((n, n, n), 1, torch.float64).to(DEV)
    o = torch.zeros_like(u)
    kw = dict(nx=n, ny=n, k0=3, k1=n - 3, border=3, weno_z="z", rdx=10.0, rdy=10.0, rdz=10.0,
              dt=1e-3, a=0.75, b=0.25)
    stencil.burgers3d_stage(u, u, o, **kw)  # u0 == in: fine
    with pytest.raises(RuntimeError):
        stencil.burgers3d_stage(u, u, o, ls=True, **kw)  # du == in: rejected
    with pytest.raises(RuntimeError):
        stencil.diffusion3d_stage(u, o, o, nx=n, ny=n, k0=2, k1=n - 2, border=2, order=4,
                                  cx=1.0, cy=1.0, cz=1.0, dt=1e-3, a=0.5, b=0.5, ls=True)
