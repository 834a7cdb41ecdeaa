"""Real multi-GPU runs: one process per GPU over RCCL (torch.distributed "nccl"), the
production halo path (zero-copy grouped send/recv on the high-priority comm stream,
overlapped with the interior launch) — bitwise equal to the 1-rank run.

The GPU tests switch themselves on when >= 2 GPUs are visible (the driver's 8-GPU node)
and skip on the 1-GPU box (RCCL refuses two ranks on one device).  The same case bodies
run with world=2 over gloo on the CPU (`test_harness_gloo_cpu`), so the harness itself is
exercised every round.

Reference being replaced: the MPI halo choreography between real ranks,
`MultiGPU/Diffusion3d_Baseline/main.c:201-302`, launched by `run.sh:2` (`mpirun -np 2`).
"""
import os
import subprocess
from pathlib import Path

import numpy as np
import pytest
import torch

from multigpu_advectiondiffusion_amd import Burgers, Diffusion, Grid, Solver
from multigpu_advectiondiffusion_amd.launch import free_port_block, spawn_local

ROOT = Path(__file__).resolve().parent.parent


def _ngpu() -> int:
    try:
        return torch.cuda.device_count()  # counting devices does not initialise HIP
    except Exception:  # pragma: no cover
        return 0


# (name, model kind, decomposition, overlap)
CASES = [
    ("heat3d_fused_slab", "diff3", None, True),
    ("heat3d_fused_slab_nooverlap", "diff3", None, False),
    ("heat3d_stage_slab", "diff3s", None, True),
    ("burgers3d_slab", "burg3", None, True),
    ("heat2d_fused_slab", "diff2", None, True),
    ("burgers2d_slab", "burg2", None, True),
    ("heat3d_fused_cart", "diff3", "cart", True),
    ("heat3d_stage_cart", "diff3s", "cart", True),
    ("burgers3d_cart", "burg3", "cart", True),
]
STEPS = 6


def _make(kind):
    if kind == "diff3":
        return Diffusion(K=1.0, order=4), Grid((70, 33, 41), (1.0, 1.0, 1.0)), "sine"
    if kind == "diff3s":
        return Diffusion(K=1.0, order=4, fused=False), Grid((70, 33, 41), (1.0, 1.0, 1.0)), "sine"
    if kind == "burg3":
        return Burgers(viscosity=1e-4, weno="z", cfl=0.3), Grid((66, 35, 40), (2.0, 2.0, 2.0)), "gaussian"
    if kind == "diff2":
        return Diffusion(K=1.0, order=4), Grid((300, 61), (1.0, 1.0)), "heat"
    if kind == "burg2":
        return Burgers(viscosity=0.0, weno="js", cfl=0.3), Grid((260, 57), (2.0, 2.0)), "gaussian"
    raise KeyError(kind)


def _cart_grid(world: int, dims: int):
    """A process grid that splits x and/or y (array order)."""
    if dims == 2:
        return {2: (1, 2), 4: (2, 2), 8: (2, 4)}[world]
    return {2: (1, 1, 2), 4: (1, 2, 2), 8: (2, 2, 2)}[world]


def _solve(comm, kind, decomp, overlap):
    model, grid, ic = _make(kind)
    if decomp == "cart":
        decomp = _cart_grid(comm.size, grid.dims) if comm.size > 1 else None
    s = Solver(model, grid, comm, dtype=torch.float64, ic=ic, overlap=overlap, decomp=decomp)
    if decomp is not None:
        assert s.cart
    s.run(iters=STEPS)
    g = s.gather()
    return None if g is None else g.copy()


def _rank_all_cases(comm):
    """Every case in ONE set of rank processes (one RCCL communicator for all)."""
    out = {"backend": comm.backend, "world": comm.size, "device_ids": comm.device_ids()}
    for name, kind, decomp, overlap in CASES:
        out[name] = _solve(comm, kind, decomp, overlap)
    return out


def _reference(device):
    from multigpu_advectiondiffusion_amd.parallel.comm import Comm
    comm = Comm(device=device)
    return {name: _solve(comm, kind, None, True) for name, kind, _, _ in CASES}


def _compare(ref, got):
    bad = []
    for name, *_ in CASES:
        a, b = ref[name], got[name]
        if a.shape != b.shape or not np.array_equal(a, b):
            bad.append((name, float(np.abs(a - b).max()) if a.shape == b.shape else "shape"))
    assert not bad, bad


def test_harness_gloo_cpu():
    """The RCCL test body, world=2 over gloo on the CPU: proves the harness each round."""
    ref = _reference("cpu")
    got = spawn_local(2, _rank_all_cases, device="cpu", backend="gloo")[0]
    assert got["backend"] == "gloo" and got["world"] == 2 and got["device_ids"] == [-1, -1]
    _compare(ref, got)


@pytest.mark.gpu
@pytest.mark.skipif(_ngpu() < 2, reason="needs >= 2 GPUs (RCCL refuses two ranks per GPU)")
@pytest.mark.parametrize("world", [2, 4, 8])
def test_rccl_multirank_bitwise(world):
    if _ngpu() < world:
        pytest.skip(f"needs {world} GPUs")
    ref = _reference("cuda")
    torch.cuda.synchronize()
    got = spawn_local(world, _rank_all_cases, device="cuda", backend="nccl", timeout=900)[0]
    assert got["backend"] == "nccl" and got["world"] == world
    assert got["device_ids"] == list(range(world)), got["device_ids"]
    _compare(ref, got)


# ---- native executables with --transport rccl ------------------------------------------
def _native(app, args, out, world, transport):
    exe = ROOT / "bin" / app
    assert exe.exists(), f"{exe} not built (make -C csrc apps)"
    port = free_port_block(world + 1)
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(world),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), ADVDIFF_PORT=str(port))
        cmd = [str(exe)] + [str(a) for a in args] + ["--write", str(out), "--transport",
                                                     transport]
        procs.append(subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT, text=True))
    outs = []
    for p in procs:
        so, _ = p.communicate(timeout=300)
        outs.append(so)
        assert p.returncode == 0, so
    return outs[0]


@pytest.mark.gpu
@pytest.mark.skipif(_ngpu() < 2, reason="needs >= 2 GPUs (RCCL refuses two ranks per GPU)")
@pytest.mark.parametrize("world", [2, 4, 8])
@pytest.mark.parametrize("app,args,shape,extra", [
    ("diffusion3d", [1.0, 1.0, 1.0, 1.0, 66, 40, 64, 12], (64, 40, 66), ["--ic", "sine"]),
    ("diffusion3d", [1.0, 1.0, 1.0, 1.0, 66, 40, 64, 12], (64, 40, 66), ["--ic", "sine", "--no-fused"]),
    ("burgers3d", [0.03, 0.3, 2.0, 2.0, 2.0, 40, 36, 64], (64, 36, 40), []),
    ("diffusion3d", [1.0, 1.0, 1.0, 1.0, 66, 64, 64, 12], (64, 64, 66), ["--ic", "sine", "--decomp", "cart"]),
    ("burgers3d", [0.03, 0.3, 2.0, 2.0, 2.0, 40, 64, 64], (64, 64, 40), ["--decomp", "cart"]),
])
def test_native_rccl_multirank_bitwise(tmp_path, world, app, args, shape, extra):
    if _ngpu() < world:
        pytest.skip(f"needs {world} GPUs")
    one, many = tmp_path / "one.bin", tmp_path / "many.bin"
    if "cart" in extra:  # Cartesian blocks of the native engine (y and z split)
        i = extra.index("cart")
        extra = extra[:i] + [{2: "1x2x1", 4: "2x2x1", 8: "2x4x1"}[world]] + extra[i + 1:]
        _native(app, args + [e for e in extra if e not in ("--decomp",) and "x" not in e],
                one, 1, "rccl")
    else:
        _native(app, args + extra, one, 1, "rccl")
    txt = _native(app, args + extra, many, world, "rccl")
    assert "transport=rccl" in txt
    a = np.fromfile(one, dtype=np.float32).reshape(shape)
    b = np.fromfile(many, dtype=np.float32).reshape(shape)
    assert np.array_equal(a, b), np.abs(a - b).max()
