"""Multi-rank FD2 with two RK3 steps per launch (6R ghost planes, one exchange every second
step): a P-rank run is BITWISE the 1-rank run, even and odd step counts, overlapped or
not (CPU, gloo; the kernels' torch reference path).  GPU versions (ipc ranks sharing the
box's GPU, eager and graph-replayed, both overlap schedules): tests/test_ipc_gpu.py."""
import numpy as np
import pytest
import torch

from multigpu_advectiondiffusion_amd import Diffusion, Grid, Solver
from multigpu_advectiondiffusion_amd.launch import spawn_local

GRID = ((17, 16, 40), (1.0, 2.0, 1.5))


def _solve(comm, steps, overlap, flag):
    import os
    os.environ["ADVDIFF_STEP2"] = flag
    try:
        s = Solver(Diffusion(K=0.5, order=2), Grid(*GRID), comm, dtype=torch.float64,
                   ic="square", overlap=overlap)
        info = (s._mr2, s.ghost, s.step2_capable())
        s.run(iters=steps)
        g = s.gather()
        return info, (None if g is None else g.copy()), s.it, s.t
    finally:
        os.environ.pop("ADVDIFF_STEP2", None)


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("steps", [4, 5])
def test_multirank_two_step_bitwise(world, steps):
    from multigpu_advectiondiffusion_amd.parallel import Comm
    (_, ref, it1, t1) = _solve(Comm(device="cpu"), steps, True, "0")
    for overlap in (True, False):
        out = spawn_local(world, _solve, steps, overlap, "1")
        (mr2, ghost, cap), g, it, t = out[0]
        assert mr2 and ghost == 6 and cap, (mr2, ghost, cap)
        assert (it, t) == (it1, t1)
        assert np.array_equal(g, ref), (world, steps, overlap, np.abs(g - ref).max())


def test_multirank_two_step_off_keeps_3r_halo():
    out = spawn_local(2, _solve, 2, True, "0")
    (mr2, ghost, cap), _, _, _ = out[0]
    assert not mr2 and ghost == 3 and not cap


def _thin(comm):
    import os
    os.environ["ADVDIFF_STEP2"] = "1"
    try:
        s = Solver(Diffusion(K=0.5, order=2), Grid((12, 12, 20), (1.0, 1.0, 1.0)), comm,
                   dtype=torch.float64, ic="sine")
        return s._mr2, s.ghost
    finally:
        os.environ.pop("ADVDIFF_STEP2", None)


def test_multirank_two_step_needs_6r_planes():
    """Slabs thinner than 6R planes keep one step per launch even when forced."""
    assert spawn_local(4, _thin)[0] == (False, 3)  # 5 planes per rank < 6
