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


@pytest.mark.parametrize("fused", [True, False])
def test_graph_replay_after_odd_eager_steps(fused):
    """run(5) then run(20) (the bench's warm-up + timed pattern: the graph is captured in
    the first call, replayed in the second at the other u/un parity) == 25 eager steps."""
    g = Grid((40, 36, 34), (1.0, 1.0, 1.0))
    outs = []
    for graph in (False, True):
        m = Diffusion(K=1.0, order=4, fused=fused)
        s = Solver(m, g, dtype=torch.float64, device="cuda", ic="sine")
        dt = m.stable_dt()
        s.run(iters=5, dt=dt, graph=graph)
        s.run(iters=20, dt=dt, graph=graph)
        outs.append(s.gather())
    assert np.array_equal(outs[0], outs[1])


def test_torch_reference_kernel_path_on_gpu():
    """Solver(kernel="torch") runs the PyTorch reference ops on the GPU (naive A/B path)
    and agrees with the HIP kernels to rounding."""
    import numpy as np
    from multigpu_advectiondiffusion_amd import Burgers, Diffusion, Grid, Solver
    for mk, ic in ((lambda: Diffusion(K=1.0, order=4), "sine"),
                   (lambda: Burgers(viscosity=1e-4, weno="z", cfl=0.3), "gaussian")):
        g = Grid((40, 36, 34), (1.0, 1.0, 1.0))
        a = Solver(mk(), g, dtype=torch.float64, device="cuda", ic=ic, kernel="torch")
        b = Solver(mk(), g, dtype=torch.float64, device="cuda", ic=ic)
        a.run(iters=9)
        b.run(iters=9)
        np.testing.assert_allclose(a.gather(), b.gather(), rtol=0, atol=1e-12)
