"""The reference's RHS-exchange scheme (`Solver(exchange="lu")`, `--exchange lu`;
`MultiGPU/Diffusion3d_Baseline/main.c:209-288,300`): ranks exchange the boundary planes of
L(u) and advance their ghost planes redundantly with the RK update.  On the CPU (gloo) a
P-rank "lu" run must equal the 1-rank run bit for bit, with and without overlap, for both
integrators and every model family; the default "u" mode is the comparison."""
import numpy as np
import pytest
import torch

from multigpu_advectiondiffusion_amd import Burgers, Diffusion, Grid, Solver
from multigpu_advectiondiffusion_amd.launch import spawn_local


def _make(kind):
    if kind == "diff3":
        return Diffusion(K=1.0, order=4), Grid((14, 13, 23), (1.0, 1.0, 1.0)), "sine"
    if kind == "diff3o2":
        return Diffusion(K=0.5, order=2), Grid((13, 12, 19), (1.0, 2.0, 1.5)), "square"
    if kind == "diff2":
        return Diffusion(K=1.0, order=4), Grid((24, 27), (1.0, 1.0)), "heat"
    if kind == "burg3":
        return (Burgers(viscosity=1e-3, weno="z", cfl=0.3), Grid((14, 13, 26), (2.0, 2.0, 2.0)),
                "gaussian")
    if kind == "burg2":
        return Burgers(viscosity=0.0, weno="js", cfl=0.3), Grid((22, 29), (2.0, 2.0)), "gaussian"
    raise KeyError(kind)


def _run(comm, kind, steps, overlap, exchange, integrator):
    model, grid, ic = _make(kind)
    s = Solver(model, grid, comm, dtype=torch.float64, ic=ic, overlap=overlap,
               exchange=exchange, integrator=integrator)
    s.run(iters=steps)
    g = s.gather()
    return None if g is None else g.copy()


def _serial(kind, steps, integrator="ssprk3"):
    model, grid, ic = _make(kind)
    s = Solver(model, grid, dtype=torch.float64, device="cpu", ic=ic, fused=False,
               integrator=integrator)
    s.run(iters=steps)
    return s.gather()


@pytest.mark.parametrize("kind", ["diff3", "diff3o2", "diff2", "burg3", "burg2"])
@pytest.mark.parametrize("world", [2, 3])
def test_lu_exchange_bitwise(kind, world):
    ref = _serial(kind, 4)
    for overlap in (True, False):
        out = spawn_local(world, _run, kind, 4, overlap, "lu", "ssprk3")[0]
        assert out.shape == ref.shape
        assert np.array_equal(out, ref), (kind, world, overlap, np.abs(out - ref).max())


def test_lu_exchange_lsrk45():
    ref = _serial("diff3", 3, "lsrk45")
    out = spawn_local(3, _run, "diff3", 3, True, "lu", "lsrk45")[0]
    assert np.array_equal(out, ref), np.abs(out - ref).max()


def test_lu_exchange_single_rank_and_options():
    model, grid, ic = _make("diff3")
    s = Solver(model, grid, dtype=torch.float64, device="cpu", ic=ic, exchange="lu")
    assert not s.fused and s.L is not None and s.ghost == model.radius
    s.run(iters=3)
    assert np.array_equal(s.gather(), _serial("diff3", 3))
    with pytest.raises(ValueError):
        Solver(model, grid, dtype=torch.float64, device="cpu", ic=ic, exchange="rhs")


def _cart_lu(comm):
    model, grid, ic = _make("diff3")
    try:
        Solver(model, grid, comm, dtype=torch.float64, ic=ic, exchange="lu", decomp="1x2x1")
    except ValueError as e:
        return str(e)
    return None


def test_lu_exchange_rejects_cartesian():
    msgs = spawn_local(2, _cart_lu)
    assert all(m and "slab" in m for m in msgs)


def test_cli_exchange_flag():
    from multigpu_advectiondiffusion_amd.cli import parse
    ns = parse(["diffusion3d", "1", "1", "1", "1", "8", "8", "8", "2", "--exchange", "lu"])
    assert ns.exchange == "lu"
    assert parse(["diffusion3d", "1", "1", "1", "1", "8", "8", "8", "2"]).exchange == "u"


def _gpu_serial(kind, steps):
    model, grid, ic = _make(kind)
    s = Solver(model, grid, dtype=torch.float64, device="cuda", ic=ic, fused=False,
               kernel="torch")
    s.run(iters=steps)
    return s.gather()


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["diff3", "burg3"])
def test_lu_exchange_gpu_single(kind):
    model, grid, ic = _make(kind)
    s = Solver(model, grid, dtype=torch.float64, device="cuda", ic=ic, exchange="lu")
    s.run(iters=4)
    assert np.array_equal(s.gather(), _gpu_serial(kind, 4))


@pytest.mark.gpu
@pytest.mark.parametrize("transport", ["ipc", "host"])
def test_lu_exchange_gpu_two_ranks(transport, monkeypatch):
    """Two ranks on one GPU: L's boundary planes over device puts (ipc) or host-staged
    gloo; equal to the 1-rank PyTorch-ops run bit for bit."""
    monkeypatch.setenv("ADVDIFF_SHARE_GPU", "1")
    ref = _gpu_serial("diff3", 4)
    for overlap in (True, False):
        out = spawn_local(2, _run, "diff3", 4, overlap, "lu", "ssprk3", device="cuda",
                          backend="gloo", transport=transport, timeout=240)[0]
        assert np.array_equal(out, ref), (transport, overlap, np.abs(out - ref).max())
