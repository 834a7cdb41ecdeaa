"""Pitched allocation of device fields (Solver(pitch=(px, py)): rows of align256(nx) + px
elements, 3-D planes of ny + py rows — the reference's *_PitchedMem variants,
SingleGPU/Burgers3d_WENO5_PitchedMem): the padding is never read or written, so every
model, integrator, decomposition and transport gives the unpadded solution bit for bit."""
import os

import numpy as np
import pytest
import torch

from multigpu_advectiondiffusion_amd import Burgers, Diffusion, Grid, Solver
from multigpu_advectiondiffusion_amd.launch import spawn_local
from multigpu_advectiondiffusion_amd.solver import _pitch_pads


def test_pitch_pads_parsing(monkeypatch):
    monkeypatch.delenv("ADVDIFF_PITCH", raising=False)
    assert _pitch_pads((8, 1), 3, "cpu") == (0, 0)  # host fields: never padded
    assert _pitch_pads((8, 1), 3, "cuda") == (8, 1)
    assert _pitch_pads((8, 1), 2, "cuda") == (8, 0)  # 2-D: rows only
    monkeypatch.setenv("ADVDIFF_PITCH", "4,2")
    assert _pitch_pads(None, 3, "cuda") == (4, 2)
    with pytest.raises(ValueError):
        _pitch_pads((-1, 0), 3, "cuda")


def _case(kind):
    if kind == "fd4":
        return Diffusion(K=1.0, order=4), Grid((70, 45, 38), (1.0,) * 3), "sine", "ssprk3"
    if kind == "fd2":
        return Diffusion(K=1.0, order=2), Grid((67, 40, 44), (1.0,) * 3), "sine", "ssprk3"
    if kind == "b3":
        return (Burgers(viscosity=1e-4, weno="z", cfl=0.3), Grid((66, 35, 40), (2.0,) * 3),
                "gaussian", "ssprk3")
    if kind == "b3w7":
        return (Burgers(viscosity=1e-4, weno="js7", cfl=0.3), Grid((40, 36, 30), (2.0,) * 3),
                "gaussian", "lsrk45")
    if kind == "d2":
        return Diffusion(K=1.0, order=4), Grid((300, 61), (1.0, 1.0)), "heat", "ssprk3"
    raise KeyError(kind)


def _run(comm, kind, pitch, steps, decomp=None, graph=None):
    m, g, ic, integ = _case(kind)
    s = Solver(m, g, comm, dtype=torch.float64, ic=ic, integrator=integ, pitch=pitch,
               decomp=decomp)
    s.run(iters=steps, dt=m.stable_dt() if isinstance(m, Diffusion) else s.dt(), graph=graph)
    out = s.gather()
    return None if out is None else (out.copy(), s.sx, tuple(s.u.shape))


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["fd4", "fd2", "b3", "b3w7", "d2"])
def test_pitched_fields_bitwise_single_gpu(kind):
    ref = _run(None, kind, (0, 0), 9)
    for pitch in ((8, 1), (3, 2)):
        got = _run(None, kind, pitch, 9)
        assert np.array_equal(got[0], ref[0]), (kind, pitch)
        assert got[1] == ref[1] + pitch[0]
        if kind != "d2":
            assert got[2][1] == ref[2][1] + pitch[1]


@pytest.mark.gpu
def test_pitched_fields_error_norms():
    m, g, ic, _ = _case("fd4")
    a = Solver(m, g, dtype=torch.float64, ic=ic, pitch=(0, 0))
    b = Solver(m, g, dtype=torch.float64, ic=ic, pitch=(8, 1))
    for s in (a, b):
        s.run(iters=5, dt=m.stable_dt())
    assert a.error_norms() == b.error_norms()
    assert a.bit_hash() == b.bit_hash()


@pytest.fixture
def _shared_gpu(monkeypatch):
    monkeypatch.setenv("ADVDIFF_SHARE_GPU", "1")
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", os.environ.get("ADVDIFF_TEST_HW_QUEUES", "2"))
    monkeypatch.setenv("ADVDIFF_IPC_TIMEOUT_S", os.environ.get("ADVDIFF_IPC_TIMEOUT_S", "10"))


@pytest.mark.gpu
@pytest.mark.parametrize("kind,world,decomp", [("fd4", 2, None), ("b3", 3, None),
                                               ("fd4", 4, (2, 2, 1)), ("b3", 4, (1, 2, 2))])
def test_pitched_fields_ipc_bitwise(kind, world, decomp, _shared_gpu):
    """ipc puts into pitched ghost planes / boxes (eager and graph-replayed)."""
    ref = _run(None, kind, (0, 0), 16)
    for graph in (False, True):
        got = spawn_local(world, _run, kind, (8, 1), 16, decomp, graph, device="cuda",
                          transport="ipc", timeout=100)[0]
        assert np.array_equal(got[0], ref[0]), (kind, world, decomp, graph)


@pytest.mark.gpu
@pytest.mark.parametrize("decomp", [None, (1, 2, 1)])
def test_pitched_fields_host_staged_bitwise(decomp, _shared_gpu):
    ref = _run(None, "fd4", (0, 0), 8)
    got = spawn_local(2, _run, "fd4", (8, 1), 8, decomp, False, device="cuda",
                      backend="gloo", timeout=100)[0]
    assert np.array_equal(got[0], ref[0])


@pytest.mark.gpu
def test_cli_pitch_flag(tmp_path, capsys):
    """The Python front end's --pitch PX,PY: same result.bin, the padded row pitch and
    field bytes in the --json line."""
    import json
    from multigpu_advectiondiffusion_amd import cli
    args = ["diffusion3d", "1", "1", "1", "1", "50", "44", "46", "9", "--ic", "sine", "--json"]
    recs = []
    for pitch in ("0,0", "4,1"):
        assert cli.main(args + ["--write", str(tmp_path / f"{pitch}.bin"), "--pitch", pitch]) == 0
        out = capsys.readouterr().out
        recs.append(json.loads([ln for ln in out.splitlines() if ln.startswith("{")][-1]))
    a = np.fromfile(tmp_path / "0,0.bin", dtype=np.float32)
    b = np.fromfile(tmp_path / "4,1.bin", dtype=np.float32)
    assert np.array_equal(a, b)
    assert recs[1]["row_pitch"] == recs[0]["row_pitch"] + 4
    assert recs[1]["device_field_bytes"] > recs[0]["device_field_bytes"]


@pytest.mark.gpu
def test_pitched_fields_gather_with_ghosts():
    """The multi-GPU result.bin layout (every slab with its ghost planes) crops the plane
    padding rows: the same array as the dense layout."""
    m, g, ic, _ = _case("fd4")
    a = Solver(m, g, dtype=torch.float64, ic=ic, pitch=(0, 0))
    b = Solver(m, g, dtype=torch.float64, ic=ic, pitch=(4, 1))
    for s in (a, b):
        s.run(iters=3, dt=m.stable_dt())
    ga, gb = a.gather_with_ghosts(), b.gather_with_ghosts()
    assert ga.shape == gb.shape and np.array_equal(ga, gb)


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(256, 256, 256), (257, 256, 256), (256, 256, 257)])
def test_sizing_matches_solver_memory_at_the_pitch_threshold(shape):
    """utils/sizing.solver_bytes applies the pitch rule to the same quantity the Solver
    does (global cells per rank, ghosts excluded): equal to Solver.memory_bytes() at,
    and just above, the 128 MiB field threshold (round-5 advisor finding)."""
    from multigpu_advectiondiffusion_amd.utils.sizing import solver_bytes
    grid = Grid(shape, (1.0,) * 3)
    s = Solver(Diffusion(K=1.0, order=4), grid, dtype=torch.float64, device="cuda",
               ic="sine")
    alloc = (s.d.alloc, grid.ny, grid.nx)
    assert s.memory_bytes() == solver_bytes(alloc, 8, 2, cells_per_rank=grid.cells)
