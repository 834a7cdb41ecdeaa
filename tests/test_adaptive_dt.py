"""Adaptive CFL (true global max|u| every step) with dt computed on the DEVICE
(solver.py _advance_device_dt: reducer -> MAX allreduce -> advdiff_adaptive_dt -> stage
kernels read dt from memory; steps past t_end are exact no-ops): the step sequence, the
final time and the solution are bitwise those of the host-driven loop.  The CPU tests run
the same logic through the torch reference ops (ops/stencil.py adaptive_dt CPU branch)."""
import os

import numpy as np
import pytest
import torch

from multigpu_advectiondiffusion_amd import Burgers, Grid, Solver
from multigpu_advectiondiffusion_amd.launch import spawn_local


def _mk(kind):
    if kind == "b3":
        return (lambda: Burgers(viscosity=1e-3, weno="z", cfl=0.4, cfl_mode="adaptive"),
                Grid((30, 26, 22), (2.0, 2.0, 2.0)), "gaussian", "ssprk3")
    if kind == "b2":
        return (lambda: Burgers(viscosity=0.0, weno="js", cfl=0.5, cfl_mode="adaptive"),
                Grid((70, 50), (2.0, 2.0)), "gaussian", "ssprk3")
    if kind == "b3w7":
        return (lambda: Burgers(viscosity=1e-4, weno="js7", cfl=0.3, cfl_mode="adaptive"),
                Grid((28, 24, 26), (2.0, 2.0, 2.0)), "gaussian", "lsrk45")
    raise KeyError(kind)


def _solve(comm, kind, device, device_dt, t_end=0.07, iters=None):
    mk, g, ic, integ = _mk(kind)
    s = Solver(mk(), g, comm, dtype=torch.float64, device=device, ic=ic, integrator=integ,
               device_dt=device_dt)
    st = s.run(t_end=t_end) if iters is None else s.run(iters=iters)
    out = s.gather()
    return None if out is None else (out.copy(), s.t, st.steps)


@pytest.mark.parametrize("kind", ["b3", "b2", "b3w7"])
def test_device_dt_matches_host_loop_cpu(kind):
    a = _solve(None, kind, "cpu", False)
    b = _solve(None, kind, "cpu", True)
    assert a[2] == b[2] and a[1] == b[1], (a[1:], b[1:])
    assert np.array_equal(a[0], b[0])
    assert abs(a[1] - 0.07) < 1e-12
    c = _solve(None, kind, "cpu", False, iters=5)
    d = _solve(None, kind, "cpu", True, iters=5)
    assert c[2] == d[2] == 5 and c[1] == d[1] and np.array_equal(c[0], d[0])


def test_device_dt_multirank_gloo_cpu():
    ref = _solve(None, "b3", "cpu", False)
    got = spawn_local(2, _solve, "b3", "cpu", True, device="cpu", backend="gloo")[0]
    assert got[2] == ref[2] and got[1] == ref[1] and np.array_equal(got[0], ref[0])


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["b3", "b2", "b3w7"])
def test_device_dt_matches_host_loop_gpu(kind):
    """GPU: device dt with hipGraph replay (the default) == the host-driven loop."""
    a = _solve(None, kind, "cuda", False, t_end=0.2)
    b = _solve(None, kind, "cuda", True, t_end=0.2)
    assert a[2] == b[2] and a[1] == b[1], (a[1:], b[1:])
    assert np.array_equal(a[0], b[0])
    c = _solve(None, kind, "cuda", False, iters=19)
    d = _solve(None, kind, "cuda", True, iters=19)
    assert c[2] == d[2] == 19 and c[1] == d[1] and np.array_equal(c[0], d[0])


@pytest.mark.gpu
def test_device_dt_multirank_gpu_gloo(monkeypatch):
    monkeypatch.setenv("ADVDIFF_SHARE_GPU", "1")
    ref = _solve(None, "b3", "cuda", False)
    got = spawn_local(2, _solve, "b3", "cuda", True, device="cuda", backend="gloo")[0]
    assert got[2] == ref[2] and got[1] == ref[1] and np.array_equal(got[0], ref[0])


def _solve_ipc(comm, kind, bcomm, decomp):
    mk, g, ic, integ = _mk(kind)
    s = Solver(mk(), g, comm, dtype=torch.float64, ic=ic, integrator=integ, device_dt=True,
               transport="ipc", boundary_on_comm=bcomm, decomp=decomp)
    assert s.bcomm == bcomm
    st = s.run(t_end=0.07)
    assert comm.ipc().errors() == 0
    out = s.gather()
    return None if out is None else (out.copy(), s.t, st.steps)


@pytest.mark.gpu
@pytest.mark.parametrize("world,decomp", [(2, None), (4, (2, 2, 1))])
@pytest.mark.parametrize("bcomm", [True, False])
def test_device_dt_multirank_gpu_ipc(world, decomp, bcomm, monkeypatch):
    """Device dt over the peer-mapped transport, with the boundary launch on the comm
    stream (the ipc default: it reads the dt the compute stream's reduction wrote) and
    with the plain schedule: the same steps, time and field as the 1-rank host loop.
    Ranks share the one GPU: the hardware-queue cap and short wait timeout of
    tests/test_ipc_gpu.py::_shared_gpu_env apply."""
    monkeypatch.setenv("ADVDIFF_SHARE_GPU", "1")
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", os.environ.get("ADVDIFF_TEST_HW_QUEUES", "2"))
    monkeypatch.setenv("ADVDIFF_IPC_TIMEOUT_S", os.environ.get("ADVDIFF_IPC_TIMEOUT_S", "10"))
    ref = _solve(None, "b3", "cuda", False)
    got = spawn_local(world, _solve_ipc, "b3", bcomm, decomp, device="cuda", transport="ipc",
                      timeout=100)[0]
    assert got[2] == ref[2] and got[1] == ref[1] and np.array_equal(got[0], ref[0])
