"""The peer-mapped device transport (ipc: csrc/kernels/ipc.hip, parallel/ipc.py, native
IpcTransport) with several ranks sharing the one GPU of the box: every halo is a put
kernel straight into the neighbour's ghost cells + a device flag, no host staging, no
host synchronisation inside a step — the production multi-GPU data path (xGMI puts)
minus the link.  Results must equal the 1-rank run bitwise, eager and graph-replayed,
slab and Cartesian, with and without overlap.  Reference being replaced: the host-staged
MPI choreography of MultiGPU/Diffusion3d_Baseline/main.c:209-288."""
import os
import subprocess
from pathlib import Path

import numpy as np
import pytest
import torch

from multigpu_advectiondiffusion_amd import Burgers, Diffusion, Grid, Solver
from multigpu_advectiondiffusion_amd.launch import free_port_block, spawn_local

pytestmark = pytest.mark.gpu

ROOT = Path(__file__).resolve().parent.parent


def _make(kind):
    if kind == "diff3":
        return Diffusion(K=1.0, order=4), Grid((70, 33, 41), (1.0, 1.0, 1.0)), "sine"
    if kind == "diff3o2":
        return Diffusion(K=1.0, order=2), Grid((67, 36, 44), (1.0, 1.0, 1.0)), "sine"
    if kind == "burg3":
        return Burgers(viscosity=1e-4, weno="z", cfl=0.3), Grid((66, 35, 40), (2.0, 2.0, 2.0)), "gaussian"
    if kind == "diff2":
        return Diffusion(K=1.0, order=4), Grid((300, 61), (1.0, 1.0)), "heat"
    if kind == "burg2":
        return Burgers(viscosity=0.0, weno="js", cfl=0.3), Grid((260, 57), (2.0, 2.0)), "gaussian"
    raise KeyError(kind)


def _reference(kind, steps):
    model, grid, ic = _make(kind)
    s = Solver(model, grid, dtype=torch.float64, device="cuda", ic=ic)
    s.run(iters=steps, graph=False)
    return s.gather()


def _run(comm, kind, steps, overlap, decomp, graph):
    """overlap: True (the default schedule: boundary launch on the comm stream), "plain"
    (boundary launch on the compute stream after the halo wait) or False."""
    assert comm.transport == "ipc"
    model, grid, ic = _make(kind)
    bc = None
    if overlap == "plain":
        overlap, bc = True, False
    s = Solver(model, grid, comm, dtype=torch.float64, ic=ic, overlap=overlap, decomp=decomp,
               boundary_on_comm=bc)
    assert s.bcomm == (overlap and bc is None)
    assert s.graph_capable()
    s.run(iters=steps, graph=graph)
    g = s.gather()
    nerr = comm.ipc().errors()
    assert nerr == 0, f"{nerr} ipc wait timeouts"
    return None if g is None else g.copy()


def _spawn(world, *args):
    return spawn_local(world, _run, *args, device="cuda", transport="ipc", timeout=240)[0]


@pytest.fixture(autouse=True)
def _shared_gpu_env(monkeypatch):
    """All ranks share the box's one GPU: few hardware queues per rank keep every rank's
    queue mapped by the hardware scheduler (with 4 per rank, 8 ranks + the test process
    oversubscribe it, and a spinning device wait can starve a producer whose queue is
    unmapped).  Real runs have one rank per GPU and are not affected."""
    monkeypatch.setenv("ADVDIFF_SHARE_GPU", "1")
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", os.environ.get("ADVDIFF_TEST_HW_QUEUES", "2"))
    monkeypatch.setenv("ADVDIFF_IPC_TIMEOUT_S", os.environ.get("ADVDIFF_IPC_TIMEOUT_S", "10"))


@pytest.mark.parametrize("kind", ["diff3", "burg3", "diff2", "burg2", "diff3o2"])
def test_ipc_slab_bitwise(kind, monkeypatch):
    """z/y slabs, per-stage (Burgers) and fused-step (heat) exchanges, 2 and 3 ranks,
    overlap on (boundary on the comm stream, the default; and the plain schedule) / off,
    eager and hipGraph replay (16 steps = 2 graphs of 8) — all bitwise equal to the 1-rank
    run."""
    monkeypatch.setenv("ADVDIFF_SHARE_GPU", "1")
    ref = _reference(kind, 16)
    for world, overlap, graph in ((2, True, False), (3, True, True), (2, False, True),
                                  (3, "plain", True)):
        out = _spawn(world, kind, 16, overlap, None, graph)
        assert np.array_equal(out, ref), (kind, world, overlap, graph, np.abs(out - ref).max())


# (2, 2, 2) with 8 Python ranks ran here until round 3: 8 torch processes + the pytest process
# sharing one GPU oversubscribe its hardware scheduler, and once in a full-suite run a
# spinning device wait starved past its timeout (a test-rig artefact: one rank per GPU in
# production).  The 8-rank 2x2x2 device exchange is covered by the native executables
# below (lighter processes, both corner modes) and by the gloo tests on the CPU.
@pytest.mark.parametrize("kind,world,decomp,corners", [
    ("diff3", 4, (1, 2, 2), "direct"), ("diff3", 4, (2, 2, 1), "direct"),
    ("diff3", 4, (2, 2, 1), "phased"), ("burg3", 4, (2, 1, 2), "direct"),
    ("diff2", 4, (2, 2), "direct"), ("diff2", 4, (2, 2), "phased"), ("burg2", 2, (1, 2), "direct"),
])
def test_ipc_cartesian_bitwise(kind, world, decomp, corners, monkeypatch):
    """Cartesian blocks: strided boxes put straight into the neighbours' ghost boxes (no
    pack/unpack); the fused step's corner exchange one phase over all 3^d - 1 neighbour
    offsets (direct) or axis by axis ordered on the device by the flags (phased) — eager
    and graph-replayed, bitwise equal to the 1-rank run."""
    monkeypatch.setenv("ADVDIFF_SHARE_GPU", "1")
    monkeypatch.setenv("ADVDIFF_CORNERS", corners)
    ref = _reference(kind, 16)
    for overlap, graph in ((True, True), (False, False)):
        out = _spawn(world, kind, 16, overlap, decomp, graph)
        assert np.array_equal(out, ref), (kind, decomp, overlap, graph, np.abs(out - ref).max())


def _run_rebuilt(comm, kind, steps, decomps, final, empty=True):
    """bench.py's decomposition tuning: solvers of several grids alive and stepping
    interleaved, all freed (allocator cache emptied), then a new solver of `final`: its
    fields may come back at addresses the first solvers' exchanges were keyed on."""
    model, grid, ic = _make(kind)
    tries = [Solver(model, grid, comm, dtype=torch.float64, ic=ic, decomp=d) for d in decomps]
    for _ in range(2):
        for s in tries:
            s.run(iters=3)
    for s in tries:
        s.run(iters=steps)  # graphs of the trial solvers too
    del tries, s
    torch.cuda.synchronize()
    if empty:  # fresh allocations; else the new fields reuse the cached (exported) blocks
        torch.cuda.empty_cache()
    s = Solver(model, grid, comm, dtype=torch.float64, ic=ic, decomp=final)
    s.run(iters=steps)
    g = s.gather()
    assert comm.ipc().errors() == 0
    return None if g is None else g.copy()


@pytest.mark.parametrize("kind,world,decomps,final,empty", [
    ("diff3", 4, [None, (2, 2, 1)], (2, 2, 1), True), ("diff3", 4, [(2, 2, 1), None], None, True),
    ("burg3", 4, [None, (2, 2, 1)], (2, 2, 1), True), ("diff3", 2, [None], None, False),
    ("diff3o2", 4, [None, (2, 2, 1)], None, False),
])
def test_ipc_solver_rebuilt_after_free(kind, world, decomps, final, empty, monkeypatch):
    """Regression (round-3 bench rehearsal, 4 ipc ranks: L_inf 4.9e-5 after tuning): the
    peers' receive addresses learned by freed solvers must not be reused by a new one
    (IpcPeers.reset at solver construction, graphs keyed by its epoch)."""
    monkeypatch.setenv("ADVDIFF_SHARE_GPU", "1")
    ref = _reference(kind, 16)
    out = spawn_local(world, _run_rebuilt, kind, 16, decomps, final, empty, device="cuda",
                      transport="ipc", timeout=240)[0]
    assert np.array_equal(out, ref), np.abs(out - ref).max()


# ------------------------------------------------------------------------------------
# native executables (csrc/runtime/transport.cpp IpcTransport)
# ------------------------------------------------------------------------------------
def _native(app, args, out, world=1, extra=(), env_extra=None):
    exe = ROOT / "bin" / app
    assert exe.exists(), f"{exe} not built (make -C csrc apps)"
    port = free_port_block(world + 1)
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(world),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), ADVDIFF_PORT=str(port),
                   **(env_extra or {}))
        cmd = [str(exe)] + [str(a) for a in args] + ["--write", str(out)] + list(extra)
        procs.append(subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT, text=True))
    outs = [p.communicate(timeout=240)[0] for p in procs]
    bad = [(r, p.returncode, o) for r, (p, o) in enumerate(zip(procs, outs)) if p.returncode]
    assert not bad, "\n".join(f"rank {r} exit {c}:\n{o[-1500:]}" for r, c, o in bad)
    return outs[0]


NATIVE_CASES = [
    ("diffusion3d", [1.0, 1.0, 1.0, 1.0, 50, 44, 46, 9], (46, 44, 50), 8, "2x2x2",
     ["--ic", "sine", "--no-overlap"]),              # the round-2 intermittent case
    ("diffusion3d", [1.0, 1.0, 1.0, 1.0, 50, 44, 46, 9], (46, 44, 50), 8, "2x2x2",
     ["--ic", "sine"]),
    ("diffusion3d", [1.0, 1.0, 1.0, 1.0, 50, 44, 46, 9], (46, 44, 50), 8, "2x2x2",
     ["--ic", "sine", "ADVDIFF_CORNERS=phased"]),  # the axis-by-axis corner exchange
    ("diffusion3d", [1.0, 1.0, 1.0, 1.0, 66, 40, 45, 12], (45, 40, 66), 3, "slab",
     ["--ic", "sine"]),
    ("diffusion3d", [1.0, 1.0, 1.0, 1.0, 66, 40, 45, 12], (45, 40, 66), 4, "2x2x1",
     ["--ic", "sine", "--no-fused"]),
    ("burgers3d", [0.03, 0.3, 2.0, 2.0, 2.0, 40, 36, 41], (41, 36, 40), 4, "2x1x2", []),
    ("burgers3d", [0.03, 0.3, 2.0, 2.0, 2.0, 40, 36, 41], (41, 36, 40), 2, "slab", []),
    ("diffusion2d", [1.0, 1.0, 1.0, 130, 90, 30], (90, 130), 4, "2x2", ["--ic", "disc"]),
]


@pytest.mark.parametrize("app,args,shape,world,decomp,extra", NATIVE_CASES)
@pytest.mark.parametrize("transport", ["ipc", "socket"])
def test_native_poisoned_multirank_bitwise(tmp_path, app, args, shape, world, decomp, extra,
                                           transport):
    """ADVDIFF_POISON=1: every device allocation (fields with row padding and ghost
    shells, staging buffers) starts as NaN instead of zero, so a cell read before anybody
    wrote it shows up in the result.  The P-rank run over the ipc (device puts) and the
    socket (host-staged) transports must still equal the 1-rank run bitwise."""
    one, many = tmp_path / "one.bin", tmp_path / "many.bin"
    poison = {"ADVDIFF_POISON": "1"}
    poison.update(e.split("=", 1) for e in extra if e.startswith("ADVDIFF_"))
    extra = [e for e in extra if not e.startswith("ADVDIFF_")]
    _native(app, args, one, extra=extra, env_extra=poison)
    dec = [] if decomp == "slab" else ["--decomp", decomp]
    txt = _native(app, args, many, world=world, extra=extra + ["--transport", transport] + dec,
                  env_extra=poison)
    assert f"transport={transport}" in txt, txt
    a = np.fromfile(one, dtype=np.float32).reshape(shape)
    b = np.fromfile(many, dtype=np.float32).reshape(shape)
    assert np.isfinite(a).all()
    if not np.array_equal(a, b):
        bad = np.argwhere(a != b)
        pytest.fail(f"{len(bad)} cells differ, max {np.nanmax(np.abs(a - b))}, box "
                    f"{bad.min(axis=0)}..{bad.max(axis=0)} of {shape}\n{txt[-2000:]}")


@pytest.mark.parametrize("app,args,shape,world,decomp,extra", [
    NATIVE_CASES[1], NATIVE_CASES[3], NATIVE_CASES[4], NATIVE_CASES[5], NATIVE_CASES[6],
    NATIVE_CASES[7]])
def test_native_plain_overlap_bitwise(tmp_path, app, args, shape, world, decomp, extra):
    """Native engine, ipc transport, --no-boundary-on-comm: the plain overlap schedule
    (boundary launch on the compute stream after the halo wait; the ipc default since
    round 5 is the boundary launch on the comm stream, which the poisoned test above
    runs) — fused heat slab and 2x2x2, per-stage heat and Burgers, slab and Cartesian,
    2-D, graph-replayed, poisoned allocations: bitwise equal to one rank."""
    one, many = tmp_path / "one.bin", tmp_path / "many.bin"
    env = {"ADVDIFF_POISON": "1"}
    env.update(e.split("=", 1) for e in extra if e.startswith("ADVDIFF_"))
    extra = [e for e in extra if not e.startswith("ADVDIFF_")]
    _native(app, args, one, extra=extra, env_extra=env)
    dec = [] if decomp == "slab" else ["--decomp", decomp]
    txt = _native(app, args, many, world=world,
                  extra=extra + ["--transport", "ipc", "--no-boundary-on-comm"] + dec,
                  env_extra=env)
    a = np.fromfile(one, dtype=np.float32).reshape(shape)
    b = np.fromfile(many, dtype=np.float32).reshape(shape)
    assert np.isfinite(a).all() and np.array_equal(a, b), txt[-2000:]


def _preflight_then_run(comm, kind, steps):
    rec = comm.ipc().preflight(rounds=3)
    model, grid, ic = _make(kind)
    s = Solver(model, grid, comm, dtype=torch.float64, ic=ic, transport="ipc")
    s.run(iters=steps, graph=True)
    h = s.bit_hash()
    assert comm.ipc().errors() == 0
    return rec, h


@pytest.mark.parametrize("world", [2, 4])
def test_ipc_preflight_all_pairs_then_solver(world):
    """The preflight (every ordered pair of ranks, stale-cache pattern round trips) passes
    and leaves the flag counters consistent: a graph-replayed solver afterwards matches the
    1-rank run's bit hash."""
    model, grid, ic = _make("diff3")
    ref = Solver(model, grid, dtype=torch.float64, device="cuda", ic=ic)
    ref.run(iters=16, graph=False)
    h1 = ref.bit_hash()
    out = spawn_local(world, _preflight_then_run, "diff3", 16, device="cuda", transport="ipc",
                      timeout=240)
    for rec, h in out:
        assert rec["pairs"] == world * (world - 1) and not rec["cross_device"]
        assert h == h1


def _run_striped(comm, kind, steps, graph):
    model, grid, ic = _make(kind)
    s = Solver(model, grid, comm, dtype=torch.float64, ic=ic, transport="ipc", stripe=2)
    assert s.halo.striped
    s.run(iters=steps, graph=graph)
    g = s.gather()
    assert comm.ipc().errors() == 0
    return None if g is None else g.copy()


@pytest.mark.parametrize("kind", ["diff3", "burg3"])
@pytest.mark.parametrize("world", [4, 5])
def test_ipc_striped_slab_bitwise(kind, world, monkeypatch):
    """Striped slab exchange (part of every face message relayed through helper ranks:
    channel-1 puts into the helpers' parity buffers, channel-2 forwards into the ghost
    rows) — fused heat (1 exchange per step) and Burgers (3 per step), eager and
    graph-replayed (both relay buffer sets inside one graph), bitwise equal to 1 rank.
    ADVDIFF_STRIPE_SHARED=1 lets routes share links so 4-5 ranks have helpers."""
    monkeypatch.setenv("ADVDIFF_STRIPE_SHARED", "1")
    ref = _reference(kind, 17)
    for graph in (False, True):
        out = spawn_local(world, _run_striped, kind, 17, graph, device="cuda",
                          transport="ipc", timeout=240)[0]
        assert np.array_equal(out, ref), (kind, world, graph, np.abs(out - ref).max())


def _run_bcomm(comm, kind, steps, decomp, graph):  # noqa: D103
    model, grid, ic = _make(kind)
    s = Solver(model, grid, comm, dtype=torch.float64, ic=ic, transport="ipc", decomp=decomp,
               boundary_on_comm=True)
    assert s.bcomm
    s.run(iters=steps, graph=graph)
    g = s.gather()
    assert comm.ipc().errors() == 0
    return None if g is None else g.copy()


@pytest.mark.parametrize("kind,world,decomp", [("diff3", 2, None), ("diff3", 3, None),
                                               ("diff3", 4, (2, 2, 1)), ("burg3", 3, None),
                                               ("burg3", 4, (2, 2, 1)), ("diff2", 2, None)])
def test_ipc_boundary_on_comm_bitwise(kind, world, decomp):
    """Boundary launch on the comm stream (between the wait for its input's halo and the
    puts of its output) beside the interior launch on the compute stream — fused heat step
    and per-stage Burgers, eager and graph-replayed, slab and Cartesian: bitwise equal to
    one rank.  Round 4's three-stream version crashed in hipStreamEndCapture (event waits
    between two side streams of a capture, profiles/r5/diag_bstream.md)."""
    ref = _reference(kind, 17)
    for graph in (False, True):
        out = spawn_local(world, _run_bcomm, kind, 17, decomp, graph, device="cuda",
                          transport="ipc", timeout=240)[0]
        assert np.array_equal(out, ref), (kind, world, decomp, graph, np.abs(out - ref).max())


def _run_step2(comm, steps, overlap, graph, flag):  # noqa: D103
    if flag is None:
        os.environ.pop("ADVDIFF_STEP2", None)
    else:
        os.environ["ADVDIFF_STEP2"] = flag
    model, grid, ic = _make("diff3o2")
    bc = None
    if overlap == "plain":
        overlap, bc = True, False
    s = Solver(model, grid, comm, dtype=torch.float64, ic=ic, overlap=overlap,
               boundary_on_comm=bc)
    if flag == "1":
        assert s._mr2 and s.ghost == 6 and s.step2_capable()
    s.run(iters=steps, graph=graph)
    g = s.gather()
    assert comm.ipc().errors() == 0
    return s._mr2, (None if g is None else g.copy())


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("overlap", [True, "plain", False])
def test_ipc_multirank_two_step_bitwise(world, overlap):
    """Multi-rank FD2 with two steps per launch (v6_march on the interior and on each
    boundary slab, 6R ghost planes exchanged every second step): bitwise the one-rank run,
    odd step count (a one-step launch in the 6R layout at the end), eager and graph-
    replayed, all three schedules; and the measured choice (ADVDIFF_STEP2 unset) agrees on
    every rank."""
    ref = _reference("diff3o2", 17)
    for graph in (False, True):
        for flag in ("1", None):
            out = spawn_local(world, _run_step2, 17, overlap, graph, flag, device="cuda",
                              transport="ipc", timeout=240)
            assert len({o[0] for o in out}) == 1
            g = out[0][1]
            assert np.array_equal(g, ref), (world, overlap, graph, flag, np.abs(g - ref).max())


def _run_fused_put(comm, kind, steps, graph, dtype):  # noqa: D103
    model, grid, ic = _make(kind)
    s = Solver(model, grid, comm, dtype=dtype, ic=ic, transport="ipc", fused_put=True)
    assert s.fput and not s.bcomm and not s._mr2
    assert s.ghost == (3 if s.fused else 1) * model.radius
    s.run(iters=steps, graph=graph)
    g = s.gather()
    assert comm.ipc().errors() == 0
    return None if g is None else g.copy()


@pytest.mark.parametrize("kind,dtype", [("diff3", torch.float64), ("diff3o2", torch.float64),
                                        ("diff3", torch.float32), ("burg3", torch.float64)])
@pytest.mark.parametrize("world", [2, 3, 4])
def test_ipc_fused_put_bitwise(kind, dtype, world):
    """Fused halo puts (transport "ipc+fused"): ONE launch per step (heat) or per stage
    (WENO5-Z + viscous, adaptive device dt) over every owned plane that stores its boundary
    output planes straight into the neighbours' ghost planes (advdiff_diffusion3d_step_put
    / advdiff_burgers3d_stage_put), then signal + wait — uneven slabs (41 / 40 planes over
    2-4 ranks), FD4 and FD2, fp64 and fp32, eager and graph-replayed, odd step count:
    bitwise equal to the one-rank run."""
    model, grid, ic = _make(kind)
    r = Solver(model, grid, dtype=dtype, device="cuda", ic=ic)
    r.run(iters=17, graph=False)
    ref = r.gather()
    for graph in (False, True):
        out = spawn_local(world, _run_fused_put, kind, 17, graph, dtype, device="cuda",
                          transport="ipc", timeout=240)[0]
        assert np.array_equal(out, ref), (kind, dtype, world, graph, np.abs(out - ref).max())


def test_fused_put_needs_direct_ipc_slab():
    """fused_put is ignored where it does not apply (one rank)."""
    for kind in ("diff3", "burg3"):
        model, grid, ic = _make(kind)
        assert not Solver(model, grid, dtype=torch.float64, device="cuda", ic=ic,
                          fused_put=True).fput


def _run_fused_put_fp32_burgers(comm, steps):  # noqa: D103
    model, grid, ic = _make("burg3")
    s = Solver(model, grid, comm, dtype=torch.float32, ic=ic, transport="ipc", fused_put=True)
    assert not s.fput  # fp32 WENO5 runs packed pairs: the ordinary ipc exchange
    s.run(iters=steps)
    g = s.gather()
    return None if g is None else g.copy()


def test_fused_put_falls_back_for_fp32_burgers():
    """Where the stage cannot carry the puts (fp32 WENO5: packed pairs), "ipc+fused" is the
    plain ipc exchange — still bitwise equal to one rank."""
    model, grid, ic = _make("burg3")
    r = Solver(model, grid, dtype=torch.float32, device="cuda", ic=ic)
    r.run(iters=5)
    ref = r.gather()
    out = spawn_local(2, _run_fused_put_fp32_burgers, 5, device="cuda", transport="ipc",
                      timeout=240)[0]
    assert np.array_equal(out, ref)


@pytest.mark.parametrize("app,args,shape,world,extra", [
    NATIVE_CASES[3][:4] + (["--ic", "sine"],),
    NATIVE_CASES[3][:4] + (["--ic", "sine", "--order", "2"],),
    ("diffusion3d", [1.0, 1.0, 1.0, 1.0, 66, 40, 45, 12], (45, 40, 66), 4, ["--ic", "sine"]),
    NATIVE_CASES[6][:4] + ([],),
    ("burgers3d", [0.03, 0.3, 2.0, 2.0, 2.0, 40, 36, 41], (41, 36, 40), 3, ["--weno", "js"]),
])
def test_native_fused_put_bitwise(tmp_path, app, args, shape, world, extra):
    """Native engine, --transport ipc --fused-put: ONE launch per step (fused heat) or per
    stage (fp64 WENO5) storing its boundary planes into the neighbours' ghost planes, then
    signal + wait (engine.cpp step_fused / stage) — uneven slabs, graph-replayed, poisoned
    allocations: bitwise equal to one rank."""
    one, many = tmp_path / "one.bin", tmp_path / "many.bin"
    env = {"ADVDIFF_POISON": "1"}
    _native(app, args, one, extra=extra, env_extra=env)
    txt = _native(app, args, many, world=world,
                  extra=extra + ["--transport", "ipc", "--fused-put"], env_extra=env)
    assert "halo puts in the launch" in txt, txt[-2000:]
    a = np.fromfile(one, dtype=np.float32).reshape(shape)
    b = np.fromfile(many, dtype=np.float32).reshape(shape)
    assert np.isfinite(a).all() and np.array_equal(a, b), txt[-2000:]


def _run_fused_striped(comm, kind, steps, graph):  # noqa: D103
    model, grid, ic = _make(kind)
    s = Solver(model, grid, comm, dtype=torch.float64, ic=ic, transport="ipc", stripe=2,
               fused_put=True)
    assert s.fput and s.halo.striped
    s.run(iters=steps, graph=graph)
    g = s.gather()
    assert comm.ipc().errors() == 0
    return None if g is None else g.copy()


@pytest.mark.parametrize("kind", ["diff3", "diff3o2"])
@pytest.mark.parametrize("world", [4, 5])
def test_ipc_fused_put_striped_bitwise(kind, world, monkeypatch):
    """Fused puts over the striped exchange ("ipc+fused+stripe"): the step kernel stores
    its send rows' output cells straight into the neighbour's ghost rows (direct part) and
    into the helpers' relay buffers (relayed parts; their frozen cells primed by one
    ordinary exchange per relay set), the helpers forward as usual — eager and graph-
    replayed, bitwise equal to one rank.  ADVDIFF_STRIPE_SHARED=1 gives 4-5 ranks
    helpers."""
    monkeypatch.setenv("ADVDIFF_STRIPE_SHARED", "1")
    ref = _reference(kind, 17)
    for graph in (False, True):
        out = spawn_local(world, _run_fused_striped, kind, 17, graph, device="cuda",
                          transport="ipc", timeout=240)[0]
        assert np.array_equal(out, ref), (kind, world, graph, np.abs(out - ref).max())
