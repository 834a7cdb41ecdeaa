"""hipGraph replay of the step loop (single process) must give bitwise the same result
as eager launches, for the fused and per-stage paths, iteration- and time-driven runs."""
import numpy as np
import pytest
import torch

from multigpu_advectiondiffusion_amd import Burgers, Diffusion, Grid, Solver

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("make", [
    lambda: (Diffusion(K=1.0, order=4), Grid((70, 60, 50), (1.0, 1.0, 1.0)), "sine", {"iters": 21}),
    lambda: (Diffusion(K=1.0, order=4, fused=False), Grid((70, 60, 50), (1.0, 1.0, 1.0)), "sine", {"iters": 13}),
    lambda: (Diffusion(K=1.0, order=4), Grid((300, 200), (1.0, 1.0)), "heat", {"iters": 19}),
    lambda: (Burgers(viscosity=1e-5, weno="z", cfl=0.3), Grid((48, 40, 36), (2.0, 2.0, 2.0)), "gaussian", {"t_end": 0.05}),
    lambda: (Burgers(viscosity=0.0, weno="js", cfl=0.4), Grid((200, 150), (2.0, 2.0)), "gaussian", {"t_end": 0.1}),
])
def test_graph_replay_bitwise(make):
    outs = []
    for graph in (False, True):
        model, grid, ic, run = make()
        s = Solver(model, grid, dtype=torch.float64, device="cuda", ic=ic)
        st = s.run(graph=graph, **run)
        outs.append((s.gather(), st.steps, s.t))
    (a, na, ta), (b, nb, tb) = outs
    assert na == nb and abs(ta - tb) < 1e-12
    assert np.array_equal(a, b)
