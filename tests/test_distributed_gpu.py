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
    model, grid, ic = _make(kind)
    s = Solver(model, grid, comm, dtype=torch.float64, ic=ic, overlap=overlap)
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
    for world, overlap in ((2, True), (3, True), (2, False)):
        out = spawn_local(world, _run, kind, 5, overlap, device="cuda", backend="gloo")[0]
        assert np.array_equal(out, ref), (kind, world, overlap, np.abs(out - ref).max())
