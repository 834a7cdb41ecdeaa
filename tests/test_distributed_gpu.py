"""Multi-process runs of the GPU solver on ONE MI355X (the box has a single GPU and RCCL
refuses two ranks per device): ranks share the GPU and exchange halos host-staged over
gloo.  This exercises every device-side piece of the distributed path — per-rank slabs,
interior/boundary split launches, comm stream + events, overlap — against the 1-rank
run, bitwise.  Only the transport call differs from the production RCCL path."""
import os

import numpy as np
import pytest
import torch

from multigpu_advectiondiffusion_amd import Burgers, Diffusion, Grid, Solver
from multigpu_advectiondiffusion_amd.launch import spawn_local

pytestmark = pytest.mark.gpu


def _make(kind):
    if kind == "diff3":
        return Diffusion(K=1.0, order=4), Grid((70, 33, 41), (1.0, 1.0, 1.0)), "sine"
    if kind == "burg3":
        return Burgers(viscosity=1e-4, weno="z", cfl=0.3), Grid((66, 35, 40), (2.0, 2.0, 2.0)), "gaussian"
    if kind == "diff2":
        return Diffusion(K=1.0, order=4), Grid((300, 61), (1.0, 1.0)), "heat"
    if kind == "burg2":
        return Burgers(viscosity=0.0, weno="js", cfl=0.3), Grid((260, 57), (2.0, 2.0)), "gaussian"
    raise KeyError(kind)


def _run(comm, kind, steps, overlap):
    """overlap: True / False, or "bcomm" (boundary launch on the comm stream: the schedule
    the RCCL transport opts into with ADVDIFF_BCOMM=1 — here with the host-staged exchange,
    whose handle carries works like RCCL's)."""
    model, grid, ic = _make(kind)
    bc = overlap == "bcomm"
    s = Solver(model, grid, comm, dtype=torch.float64, ic=ic, overlap=bool(overlap),
               boundary_on_comm=bc)
    assert s.bcomm == bc
    s.run(iters=steps)
    g = s.gather()
    return None if g is None else g.copy()


@pytest.mark.parametrize("kind", ["diff3", "burg3", "diff2", "burg2"])
def test_gpu_multirank_bitwise(kind, monkeypatch):
    monkeypatch.setenv("ADVDIFF_SHARE_GPU", "1")
    model, grid, ic = _make(kind)
    s = Solver(model, grid, dtype=torch.float64, device="cuda", ic=ic)
    s.run(iters=5)
    ref = s.gather()
    for world, overlap in ((2, True), (3, True), (2, False), (3, "bcomm")):
        out = spawn_local(world, _run, kind, 5, overlap, device="cuda", backend="gloo")[0]
        assert np.array_equal(out, ref), (kind, world, overlap, np.abs(out - ref).max())


def _run_cart(comm, kind, steps, decomp, bcomm=False):
    model, grid, ic = _make(kind)
    s = Solver(model, grid, comm, dtype=torch.float64, ic=ic, decomp=decomp,
               boundary_on_comm=bcomm)
    assert s.cart
    s.run(iters=steps)
    g = s.gather()
    return None if g is None else g.copy()


@pytest.mark.parametrize("kind,world,decomp", [
    ("diff3", 4, (1, 2, 2)), ("diff3", 2, (1, 1, 2)), ("burg3", 4, (2, 1, 2)),
    ("diff2", 2, (1, 2)), ("burg2", 4, (2, 2)),
])
def test_gpu_cartesian_bitwise(kind, world, decomp, monkeypatch):
    """x/y-split blocks: strided face pack/unpack (copy_box), sub-box kernel views,
    device IC of a box — bitwise equal to the 1-rank run."""
    monkeypatch.setenv("ADVDIFF_SHARE_GPU", "1")
    model, grid, ic = _make(kind)
    s = Solver(model, grid, dtype=torch.float64, device="cuda", ic=ic)
    s.run(iters=4)
    ref = s.gather()
    for bc in (False, True):  # plain schedule, boundary boxes on the comm stream
        out = spawn_local(world, _run_cart, kind, 4, decomp, bc, device="cuda",
                          backend="gloo")[0]
        assert np.array_equal(out, ref), (kind, decomp, bc, np.abs(out - ref).max())


def test_gpu_init_ic_box_matches_torch():
    from multigpu_advectiondiffusion_amd.ops import stencil
    from multigpu_advectiondiffusion_amd.utils import ics
    shape, lengths = (37, 29, 23), (1.0, 2.0, 1.5)
    g = Grid(shape, lengths)
    offs, ext, sx = (5, -2, 30), (9, 12, 11), 16
    for name in ("sine", "heat", "gaussian", "square", "plates"):
        p = ics.IC_DEFAULT_PARAMS.get(name, (0.0, 0.0))
        u = torch.zeros(ext[:2] + (sx,), dtype=torch.float64, device="cuda")
        stencil.init_ic_box_device(u, ics.ic_code(name), nx=ext[2], ny=ext[1], nzl=ext[0],
                                   ig0=offs[2], jg0=offs[1], kg0=offs[0], NX=shape[0],
                                   NY=shape[1], NZ=shape[2], dx=g.spacing[0], dy=g.spacing[1],
                                   dz=g.spacing[2], p0=p[0], p1=p[1])
        ref = ics.evaluate_box(name, shape, g.spacing, offs, ext, sx)
        torch.testing.assert_close(u.cpu()[..., :ext[2]], ref[..., :ext[2]], rtol=1e-14, atol=1e-15)


def _nccl_world1(_comm):
    """init_process_group with the framework's RCCL options (eager device_id,
    high-priority stream) on a 1-rank group, then a collective and a barrier."""
    import datetime
    import os

    import torch.distributed as dist

    from multigpu_advectiondiffusion_amd.parallel.comm import pg_kwargs
    os.environ["MASTER_PORT"] = str(int(os.environ["MASTER_PORT"]) + 1)
    dev = torch.device("cuda", 0)
    dist.init_process_group(backend="nccl", rank=0, world_size=1,
                            timeout=datetime.timedelta(seconds=120), **pg_kwargs("nccl", dev))
    t = torch.ones(4, device=dev)
    dist.all_reduce(t)
    dist.barrier(device_ids=[0])
    ok = float(t.sum()) == 4.0
    dist.destroy_process_group()
    return ok


def test_rccl_init_options_world1():
    assert spawn_local(1, _nccl_world1, device="cuda", backend="gloo")[0]


@pytest.mark.parametrize("kind,world,decomp", [("diff3", 4, (1, 2, 2)), ("diff2", 4, (2, 2))])
def test_gpu_cartesian_fused_bitwise(kind, world, decomp, monkeypatch):
    """Fused full-step kernel on Cartesian blocks (3R ghosts incl. edges/corners)."""
    monkeypatch.setenv("ADVDIFF_SHARE_GPU", "1")
    model, grid, ic = _make(kind)
    s = Solver(model, grid, dtype=torch.float64, device="cuda", ic=ic)
    s.run(iters=5)
    ref_g = s.gather()
    out = spawn_local(world, _run_cart, kind, 5, decomp, device="cuda", backend="gloo")[0]
    assert np.array_equal(out, ref_g), np.abs(out - ref_g).max()
