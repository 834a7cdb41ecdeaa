"""The native C++ executables (bin/*, reference CLIs) on the GPU: results must be bitwise
identical to the Python solver (same kernels, same launch geometry, same dt), and a
2-rank run (host-staged socket transport, both ranks on the one GPU) must equal the
1-rank run bitwise."""
import os
import subprocess
from pathlib import Path

import numpy as np
import pytest
import torch

from multigpu_advectiondiffusion_amd import Burgers, Diffusion, Grid, Solver
from multigpu_advectiondiffusion_amd.launch import free_port_block

pytestmark = pytest.mark.gpu

ROOT = Path(__file__).resolve().parent.parent
BIN = ROOT / "bin"


def _run(app, args, out, world=1, extra=()):
    exe = BIN / app
    assert exe.exists(), f"{exe} not built (make -C csrc apps)"
    port = free_port_block(world + 1)
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(world),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), ADVDIFF_PORT=str(port))
        cmd = [str(exe)] + [str(a) for a in args] + ["--write", str(out)] + list(extra)
        procs.append(subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT, text=True))
    outs = []
    for p in procs:
        so, _ = p.communicate(timeout=240)
        outs.append(so)
        assert p.returncode == 0, so
    _check_banner(outs[0])
    return outs[0]


def _check_banner(txt):
    """The executable was built from this tree's runtime and kernel sources."""
    from multigpu_advectiondiffusion_amd.ops import _lib
    from tests.test_native_host import runtime_tree_hash
    line = [l for l in txt.splitlines() if l.startswith("advdiff native build:")]
    assert line, txt[-1000:]
    assert f"runtime {runtime_tree_hash()}" in line[0], (line[0], runtime_tree_hash())
    assert f"kernels {_lib.source_hash()}" in line[0], (line[0], _lib.source_hash())


def _py(model, grid, ic, integrator="ssprk3", **run):
    s = Solver(model, grid, dtype=torch.float64, device="cuda", ic=ic, integrator=integrator)
    s.run(**run)
    return s.gather().astype(np.float32)


def test_diffusion3d_native_matches_python(tmp_path):
    out = tmp_path / "d3.bin"
    txt = _run("diffusion3d", [1.0, 1.0, 1.0, 1.0, 70, 60, 56, 20, 64, 4, 1], out,
               extra=["--ic", "sine"])
    assert "Total effective GFLOPs" in txt and "3D Grid Size                                 :  70 x 60 x 56" in txt
    got = np.fromfile(out, dtype=np.float32).reshape(56, 60, 70)
    exp = _py(Diffusion(K=1.0, order=4), Grid((70, 60, 56), (1.0, 1.0, 1.0)), "sine", iters=20)
    assert np.array_equal(got, exp), np.abs(got - exp).max()


def test_burgers3d_native_matches_python(tmp_path):
    out = tmp_path / "b3.bin"
    _run("burgers3d", [0.05, 0.3, 2.0, 2.0, 2.0, 48, 44, 40], out)
    got = np.fromfile(out, dtype=np.float32).reshape(40, 44, 48)
    exp = _py(Burgers(viscosity=1e-5, weno="z", cfl=0.3), Grid((48, 44, 40), (2.0, 2.0, 2.0)),
              "gaussian", t_end=0.05)
    assert np.array_equal(got, exp), np.abs(got - exp).max()


def test_diffusion2d_and_burgers2d_native(tmp_path):
    out = tmp_path / "d2.bin"
    _run("diffusion2d", [1.0, 1.0, 1.0, 130, 90, 30], out, extra=["--ic", "disc", "--order", "2"])
    got = np.fromfile(out, dtype=np.float32).reshape(90, 130)
    exp = _py(Diffusion(K=1.0, order=2), Grid((130, 90), (1.0, 1.0)), "disc", iters=30)
    assert np.array_equal(got, exp)
    out = tmp_path / "b2.bin"
    _run("burgers2d", [0.1, 0.4, 2.0, 2.0, 140, 100], out, extra=["--weno", "js", "--visc", "0"])
    got = np.fromfile(out, dtype=np.float32).reshape(100, 140)
    exp = _py(Burgers(viscosity=0.0, weno="js", cfl=0.4), Grid((140, 100), (2.0, 2.0)),
              "gaussian", t_end=0.1)
    assert np.array_equal(got, exp)


@pytest.mark.parametrize("app,args,shape", [
    ("diffusion3d", [1.0, 1.0, 1.0, 1.0, 66, 40, 45, 12], (45, 40, 66)),
    ("burgers3d", [0.03, 0.3, 2.0, 2.0, 2.0, 40, 36, 41], (41, 36, 40)),
])
def test_native_multirank_socket_bitwise(tmp_path, app, args, shape):
    one = tmp_path / "one.bin"
    two = tmp_path / "two.bin"
    _run(app, args, one)
    txt = _run(app, args, two, world=2, extra=["--transport", "socket"])
    assert "transport=socket" in txt
    a = np.fromfile(one, dtype=np.float32).reshape(shape)
    b = np.fromfile(two, dtype=np.float32).reshape(shape)
    assert np.array_equal(a, b), np.abs(a - b).max()


def test_native_error_norms_heat(tmp_path):
    txt = _run("diffusion3d", [1.0, 10.0, 10.0, 10.0, 41, 41, 41, 30], tmp_path / "h.bin",
               extra=["--error-norms"])
    line = [l for l in txt.splitlines() if l.startswith("Linf norm")][0]
    assert float(line.split(":")[1]) < 5e-2


def test_native_weno7_lsrk45_matches_python(tmp_path):
    out = tmp_path / "b7.bin"
    _run("burgers3d", [0.04, 0.3, 2.0, 2.0, 2.0, 46, 40, 38], out,
         extra=["--weno", "js7", "--integrator", "lsrk45"])
    got = np.fromfile(out, dtype=np.float32).reshape(38, 40, 46)
    exp = _py(Burgers(viscosity=1e-5, weno="js7", cfl=0.3), Grid((46, 40, 38), (2.0, 2.0, 2.0)),
              "gaussian", integrator="lsrk45", t_end=0.04)
    assert np.array_equal(got, exp), np.abs(got - exp).max()
    out = tmp_path / "d2ls.bin"
    _run("diffusion2d", [1.0, 1.0, 1.0, 130, 90, 25], out, extra=["--ic", "disc",
                                                                  "--integrator", "lsrk45"])
    got = np.fromfile(out, dtype=np.float32).reshape(90, 130)
    exp = _py(Diffusion(K=1.0, order=4), Grid((130, 90), (1.0, 1.0)), "disc",
              integrator="lsrk45", iters=25)
    assert np.array_equal(got, exp)


def test_native_fused_equals_per_stage_and_multirank(tmp_path):
    args = [1.0, 1.0, 1.0, 1.0, 66, 40, 45, 12]
    a, b, c = tmp_path / "f.bin", tmp_path / "s.bin", tmp_path / "f2.bin"
    _run("diffusion3d", args, a, extra=["--ic", "sine"])
    _run("diffusion3d", args, b, extra=["--ic", "sine", "--no-fused"])
    _run("diffusion3d", args, c, world=3, extra=["--ic", "sine", "--transport", "socket"])
    fa, fb, fc = (np.fromfile(p, dtype=np.float32) for p in (a, b, c))
    assert np.array_equal(fa, fb) and np.array_equal(fa, fc)


@pytest.mark.parametrize("app,args,shape,world,decomp,extra", [
    ("diffusion3d", [1.0, 1.0, 1.0, 1.0, 66, 40, 45, 12], (45, 40, 66), 4, "1x2x2",
     ["--ic", "sine"]),                                   # fused step, x and y split
    ("diffusion3d", [1.0, 1.0, 1.0, 1.0, 66, 40, 45, 12], (45, 40, 66), 4, "2x2x1",
     ["--ic", "sine", "--no-fused"]),                     # per-stage kernels on views
    ("diffusion3d", [1.0, 1.0, 1.0, 1.0, 50, 44, 46, 9], (46, 44, 50), 8, "2x2x2",
     ["--ic", "sine", "--no-overlap"]),
    ("burgers3d", [0.03, 0.3, 2.0, 2.0, 2.0, 40, 36, 41], (41, 36, 40), 4, "2x1x2", []),
    ("diffusion2d", [1.0, 1.0, 1.0, 130, 90, 30], (90, 130), 4, "2x2", ["--ic", "disc"]),
    ("burgers2d", [0.1, 0.4, 2.0, 2.0, 140, 100], (100, 140), 2, "1x2",
     ["--weno", "js", "--visc", "0"]),
])
def test_native_cartesian_socket_bitwise(tmp_path, app, args, shape, world, decomp, extra):
    """Native Cartesian blocks (csrc/runtime/cart.cpp: kernels on views, face / phased
    corner exchange over the socket full mesh, ranks sharing the GPU) == the 1-rank run."""
    one, many = tmp_path / "one.bin", tmp_path / "many.bin"
    _run(app, args, one, extra=extra)
    txt = _run(app, args, many, world=world,
               extra=extra + ["--transport", "socket", "--decomp", decomp])
    assert f"decomp={decomp}" in txt, txt
    a = np.fromfile(one, dtype=np.float32).reshape(shape)
    b = np.fromfile(many, dtype=np.float32).reshape(shape)
    if not np.array_equal(a, b):
        # locate the wrong region (which block / face / corner) for the failure report
        bad = np.argwhere(a != b)
        lo, hi = bad.min(axis=0), bad.max(axis=0)
        pytest.fail(f"{len(bad)} cells differ, max {np.abs(a - b).max()}, box {lo}..{hi} "
                    f"of {shape}; zero cells in the {world}-rank run: {int((b == 0).sum())} "
                    f"vs {int((a == 0).sum())}\n{txt[-2000:]}")


def test_native_cartesian_error_norms(tmp_path):
    """--error-norms on Cartesian blocks == the slab run's norms."""
    base = [1.0, 10.0, 10.0, 10.0, 41, 41, 41, 30]
    t1 = _run("diffusion3d", base, tmp_path / "a.bin", extra=["--error-norms"])
    t4 = _run("diffusion3d", base, tmp_path / "b.bin", world=4,
              extra=["--error-norms", "--transport", "socket", "--decomp", "1x2x2"])
    pick = lambda t, k: float([l for l in t.splitlines() if l.startswith(k)][0].split(":")[1])  # noqa
    for k in ("L1 norm", "L2 norm", "Linf norm"):
        assert abs(pick(t1, k) - pick(t4, k)) <= 1e-12 * max(abs(pick(t1, k)), 1e-30), k


def test_native_write_ghosts(tmp_path):
    """--write-ghosts (native): every rank's slab with its ghost planes, rank after rank —
    the reference's multi-GPU result.bin (MultiGPU/Diffusion3d_Baseline/main.c:341); the
    owned planes equal --write's, the inner ghosts equal the neighbour's boundary planes;
    the summary's HtD/DtH lines are timed (non-zero)."""
    nx, ny, nz = 40, 36, 30
    res, gh = tmp_path / "r.bin", tmp_path / "g.bin"
    txt = _run("diffusion3d", [1.0, 1.0, 1.0, 1.0, nx, ny, nz, 5], res, world=2,
               extra=["--ic", "sine", "--transport", "socket", "--write-ghosts", str(gh)])
    glob = np.fromfile(res, dtype=np.float32).reshape(nz, ny, nx)
    raw = np.fromfile(gh, dtype=np.float32)
    G, c = 6, nz // 2
    assert raw.size == 2 * (c + 2 * G) * ny * nx
    b0, b1 = (x.reshape(c + 2 * G, ny, nx) for x in np.split(raw, 2))
    assert np.array_equal(b0[G:G + c], glob[:c]) and np.array_equal(b1[G:G + c], glob[c:])
    assert np.array_equal(b0[G + c:], glob[c:c + G]) and np.array_equal(b1[:G], glob[c - G:c])
    for key in ("Data transfer(s) HtD", "Data transfer(s) DtH"):
        v = float([l for l in txt.splitlines() if key in l][0].split(":")[1].split()[0])
        assert v > 0.0, key


@pytest.mark.parametrize("app,args,shape,extra", [
    ("diffusion3d", [1.0, 1.0, 1.0, 1.0, 70, 60, 56, 21], (56, 60, 70), ["--ic", "sine"]),
    ("diffusion3d", [1.0, 1.0, 1.0, 1.0, 70, 60, 56, 19], (56, 60, 70),
     ["--ic", "sine", "--no-fused"]),
    ("burgers3d", [0.05, 0.3, 2.0, 2.0, 2.0, 48, 44, 40], (40, 44, 48),
     ["--weno", "js7", "--integrator", "lsrk45"]),
    ("diffusion2d", [1.0, 1.0, 1.0, 130, 90, 30], (90, 130), ["--ic", "disc"]),
    ("burgers2d", [0.1, 0.4, 2.0, 2.0, 140, 100], (100, 140), ["--weno", "js"]),
])
def test_native_graph_steps_bitwise(tmp_path, app, args, shape, extra):
    """hipGraph stepping of the native engine (Engine::steps: 2 eager steps, then graphs of
    8 steps, eager remainder) == eager stepping, bitwise; the banner says which ran."""
    a, b = tmp_path / "graph.bin", tmp_path / "eager.bin"
    txt = _run(app, args, a, extra=extra + ["--graph"])
    assert "hipGraph steps" in txt, txt[-800:]
    txt = _run(app, args, b, extra=extra + ["--no-graph"])
    assert "hipGraph steps" not in txt
    ga = np.fromfile(a, dtype=np.float32).reshape(shape)
    gb = np.fromfile(b, dtype=np.float32).reshape(shape)
    assert np.isfinite(ga).all() and np.array_equal(ga, gb), np.abs(ga - gb).max()


@pytest.mark.parametrize("world,decomp,extra", [
    (2, "slab", []), (4, "2x2x1", []), (8, "2x2x2", []), (4, "2x1x2", ["--no-fused"]),
])
def test_native_ipc_graph_steps_bitwise(tmp_path, world, decomp, extra):
    """Multi-rank hipGraph replay over the ipc transport (puts, signal and wait kernels
    captured with the stencil launches; ranks share the one GPU) == the 1-rank eager run."""
    args = [1.0, 1.0, 1.0, 1.0, 50, 44, 46, 21]
    one, many = tmp_path / "one.bin", tmp_path / "many.bin"
    _run("diffusion3d", args, one, extra=["--ic", "sine", "--no-graph"] + extra)
    dec = [] if decomp == "slab" else ["--decomp", decomp]
    env = dict(os.environ)
    os.environ.update(ADVDIFF_SHARE_GPU="1", GPU_MAX_HW_QUEUES="2", ADVDIFF_IPC_TIMEOUT_S="60")
    try:
        txt = _run("diffusion3d", args, many, world=world,
                   extra=["--ic", "sine", "--transport", "ipc"] + dec + extra)
    finally:
        os.environ.clear()
        os.environ.update(env)
    assert "hipGraph steps" in txt, txt[-800:]
    a = np.fromfile(one, dtype=np.float32).reshape(46, 44, 50)
    b = np.fromfile(many, dtype=np.float32).reshape(46, 44, 50)
    assert np.array_equal(a, b), np.abs(a - b).max()


# ---- checkpoint / restart of the native engine (csrc/runtime/checkpoint.cpp) ----------
def _ckpt(prefix, shape):
    """(fp64 global array, header) of a shard set, read with the Python loader."""
    from multigpu_advectiondiffusion_amd.utils import io as aio
    arr, meta = aio.load_checkpoint_box(prefix, [0] * len(shape), list(shape))
    return arr, meta


@pytest.mark.parametrize("world,extra", [
    (1, []),
    (2, ["--transport", "socket"]),                         # slab restart on 2 ranks
    (2, ["--transport", "socket", "--decomp", "1x2x1"]),    # Cartesian blocks
])
def test_native_checkpoint_restart_bitwise(tmp_path, world, extra):
    """20 steps in one run == 10 steps, fp64 shards, restart (any layout) + 10 steps, bit
    for bit (the shards are fp64: the comparison is on the solver's own precision)."""
    nx, ny, nz = 54, 46, 40
    args = lambda it: [1.0, 1.0, 1.0, 1.0, nx, ny, nz, it]
    ic = ["--ic", "sine"]
    _run("diffusion3d", args(20), tmp_path / "a.bin", extra=ic + ["--checkpoint", str(tmp_path / "a")])
    _run("diffusion3d", args(10), tmp_path / "b.bin", extra=ic + ["--checkpoint", str(tmp_path / "b")])
    txt = _run("diffusion3d", args(10), tmp_path / "c.bin", world=world,
               extra=ic + ["--restart", str(tmp_path / "b"), "--checkpoint", str(tmp_path / "c")] + extra)
    a, ma = _ckpt(tmp_path / "a", (nz, ny, nx))
    c, mc = _ckpt(tmp_path / "c", (nz, ny, nx))
    assert np.array_equal(a, c), np.abs(a - c).max()
    assert (ma["it"], mc["it"]) == (20, 20) and ma["t"] == mc["t"], (ma, mc)
    assert mc["world"] == world and mc["model"]["writer"] == "native"
    assert np.array_equal(np.fromfile(tmp_path / "a.bin", dtype=np.float32),
                          np.fromfile(tmp_path / "c.bin", dtype=np.float32)), txt[-500:]


def test_native_python_checkpoint_interop(tmp_path):
    """Python shards restart the native engine and native shards restart the Python solver:
    Python 8 steps -> native 6 -> Python 6 equals 20 Python steps bit for bit (3-D heat,
    and 2-D heat restarted on 2 ranks)."""
    for dims in (3, 2):
        if dims == 3:
            shape, lens, app = (50, 44, 38), (1.0, 1.0, 1.0), "diffusion3d"
            args = lambda it: [1.0, *lens, *shape, it]
            ic, extra = "sine", ["--ic", "sine"]
        else:
            shape, lens, app = (120, 84), (1.0, 1.0), "diffusion2d"
            args = lambda it: [1.0, *lens, *shape, it]
            ic, extra = "disc", ["--ic", "disc", "--decomp", "2x1"]
        mk = lambda: Solver(Diffusion(K=1.0, order=4), Grid(shape, lens), dtype=torch.float64,
                            device="cuda", ic=ic)
        ref = mk()
        ref.run(iters=20)
        full = ref.gather()
        s = mk()
        s.run(iters=8)
        s.save_checkpoint(tmp_path / f"p{dims}")
        world = 2 if dims == 2 else 1
        _run(app, args(6), tmp_path / f"n{dims}.bin", world=world,
             extra=extra + (["--transport", "socket"] if world > 1 else [])
             + ["--restart", str(tmp_path / f"p{dims}"), "--checkpoint", str(tmp_path / f"n{dims}")])
        s2 = mk()
        meta = s2.load_checkpoint(tmp_path / f"n{dims}")
        assert meta["it"] == 14 and meta["model"]["writer"] == "native", meta
        s2.run(iters=6)
        got = s2.gather()
        assert s2.it == 20 and s2.t == ref.t
        assert np.array_equal(got, full), (dims, np.abs(got - full).max())


def test_native_burgers_restart_continues(tmp_path):
    """A Burgers restart continues from the checkpoint's t to tEnd (3-D, WENO5-Z)."""
    base = [0.3, 2.0, 2.0, 2.0, 40, 36, 32]
    _run("burgers3d", [0.02] + base, tmp_path / "a.bin", extra=["--checkpoint", str(tmp_path / "a")])
    _run("burgers3d", [0.04] + base, tmp_path / "b.bin",
         extra=["--restart", str(tmp_path / "a"), "--checkpoint", str(tmp_path / "b")])
    a, ma = _ckpt(tmp_path / "a", (32, 36, 40))
    b, mb = _ckpt(tmp_path / "b", (32, 36, 40))
    assert abs(ma["t"] - 0.02) < 1e-12 and abs(mb["t"] - 0.04) < 1e-12, (ma["t"], mb["t"])
    assert mb["it"] > ma["it"] and np.isfinite(b).all() and not np.array_equal(a, b)


# ---- failure detection of the native engine ------------------------------------------
def _run_expect_fail(app, args, world, extra=(), env_extra=None):
    exe = BIN / app
    port = free_port_block(world + 1)
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(world),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), ADVDIFF_PORT=str(port),
                   **(env_extra or {}))
        procs.append(subprocess.Popen([str(exe)] + [str(a) for a in args] + list(extra),
                                      env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT, text=True))
    return [(p.communicate(timeout=240)[0], p.returncode) for p in procs]


@pytest.mark.parametrize("world", [1, 2])
def test_native_watchdog_stops_unstable_run(world):
    """--check-every: a run made unstable (dt 4x the FD4 limit) stops on EVERY rank with a
    'non-finite solution' error instead of running on (SURVEY §5 failure detection)."""
    res = _run_expect_fail("diffusion3d", [1.0, 1.0, 1.0, 1.0, 40, 36, 34, 600], world,
                           extra=["--ic", "sine", "--safety", "4", "--check-every", "10"]
                           + (["--transport", "socket"] if world > 1 else []))
    for out, rc in res:
        assert rc != 0 and "non-finite solution at step" in out, out[-800:]


def test_native_watchdog_and_sync_debug_keep_results(tmp_path):
    """A stable run with the watchdog, and one with ADVDIFF_SYNC_DEBUG=1 (device sync +
    error check after every launch), give the same bits as the plain run."""
    args = [1.0, 1.0, 1.0, 1.0, 44, 40, 36, 12]
    _run("diffusion3d", args, tmp_path / "a.bin", extra=["--ic", "sine"])
    _run("diffusion3d", args, tmp_path / "b.bin", extra=["--ic", "sine", "--check-every", "3"])
    os.environ["ADVDIFF_SYNC_DEBUG"] = "1"
    try:
        _run("diffusion3d", args, tmp_path / "c.bin", world=2,
             extra=["--ic", "sine", "--transport", "socket"])
    finally:
        del os.environ["ADVDIFF_SYNC_DEBUG"]
    a = np.fromfile(tmp_path / "a.bin", dtype=np.float32)
    for f in ("b.bin", "c.bin"):
        assert np.array_equal(a, np.fromfile(tmp_path / f, dtype=np.float32)), f


def test_native_launcher_fail_fast_on_injected_fault():
    """ADVDIFF_FAULT=1:3 makes native rank 1 fail after step 3; the launcher stops rank 0
    (blocked in its next halo exchange) instead of letting it hang, and reports the error."""
    import time
    from multigpu_advectiondiffusion_amd.launch import launch
    os.environ["ADVDIFF_FAULT"] = "1:3"
    try:
        t0 = time.monotonic()
        rc = launch(2, ["diffusion3d", "1", "1", "1", "1", "48", "40", "36", "200", "--ic", "sine",
                        "--transport", "socket"], native=True, timeout=120)
    finally:
        del os.environ["ADVDIFF_FAULT"]
    assert rc not in (0, 124), rc
    assert time.monotonic() - t0 < 100


def test_native_ascii_and_print_match_python(tmp_path):
    """--ascii (one %g per line, fp64) and --print (rows of %8.2f) of the native apps give
    the same text as the Python front end (the reference's Save3D / Print3D)."""
    import sys
    args = ["1", "1", "1", "1", "12", "10", "8", "5", "--ic", "sine"]
    py = subprocess.run([sys.executable, "-m", "multigpu_advectiondiffusion_amd", "diffusion3d",
                         *args, "--ascii", str(tmp_path / "py.txt"), "--print"],
                        capture_output=True, text=True, check=True, cwd=ROOT).stdout
    nat = _run("diffusion3d", args, tmp_path / "n.bin",
               extra=["--ascii", str(tmp_path / "n.txt"), "--print"])
    a, b = (tmp_path / "py.txt").read_text(), (tmp_path / "n.txt").read_text()
    assert a == b and len(a.splitlines()) == 12 * 10 * 8
    block = py[:py.index("\n\n\n") + 3]  # Python prints the field before its summary
    assert block.count("\n") > 80 and block in nat


def test_native_config_file(tmp_path):
    """--config FILE.json (positional "args" + options, overriding the command line) runs
    the same problem as the equivalent command line, bit for bit."""
    import json
    cfg = tmp_path / "run.json"
    cfg.write_text(json.dumps({"args": [1.0, 1.0, 1.0, 1.0, 30, 28, 26, 6], "ic": "sine",
                               "order": 2, "no_fused": True, "error-norms": False}))
    _run("diffusion3d", [1.0, 1.0, 1.0, 1.0, 30, 28, 26, 6], tmp_path / "a.bin",
         extra=["--ic", "sine", "--order", "2", "--no-fused"])
    txt = _run("diffusion3d", [], tmp_path / "b.bin",
               extra=["--config", str(cfg), "--ic", "heat", "--error-norms"])
    assert "L1 norm" not in txt  # "error-norms": false in the file wins
    assert np.array_equal(np.fromfile(tmp_path / "a.bin", dtype=np.float32),
                          np.fromfile(tmp_path / "b.bin", dtype=np.float32))


def test_native_singlegpu_summary_style(tmp_path):
    """--style singlegpu prints the single-GPU apps' block (Final Time, no HtD/DtH lines,
    norms inside it) with the labels of the Python front end's."""
    txt = _run("diffusion3d", [1.0, 1.0, 1.0, 1.0, 24, 22, 20, 4], tmp_path / "a.bin",
               extra=["--ic", "sine", "--style", "singlegpu", "--error-norms"])
    assert "Final Time                                   :  " in txt
    assert "Data transfer(s) HtD" not in txt
    assert "3D Grid Size                                 :  24 x 22 x 20 \n" in txt
    assert "Linf norm                                    :  " in txt


def test_native_initial_and_json(tmp_path):
    """--initial writes the starting field (as the Python front end's --initial) and
    --json prints one metrics line with the Python front end's keys."""
    import json
    import sys
    args = ["1", "1", "1", "1", "20", "18", "16", "4", "--ic", "sine"]
    subprocess.run([sys.executable, "-m", "multigpu_advectiondiffusion_amd", "diffusion3d", *args,
                    "--initial", str(tmp_path / "py0.bin")], check=True, cwd=ROOT,
                   capture_output=True)
    txt = _run("diffusion3d", args, tmp_path / "n.bin",
               extra=["--initial", str(tmp_path / "n0.bin"), "--json"])
    a = np.fromfile(tmp_path / "py0.bin", dtype=np.float32)
    assert np.array_equal(a, np.fromfile(tmp_path / "n0.bin", dtype=np.float32)) and a.size == 20 * 18 * 16
    line = json.loads([l for l in txt.splitlines() if l.startswith("{")][-1])
    assert line["app"] == "diffusion3d" and line["grid"] == [20, 18, 16] and line["steps"] == 4
    assert line["n_procs"] == 1 and line["dtype"] == "fp64" and line["mlups"] > 0


@pytest.mark.parametrize("app,args,world,extra", [
    ("diffusion3d", [1.0, 1.0, 1.0, 1.0, 40, 36, 34, 10], 1, ["--ic", "sine"]),
    ("diffusion3d", [1.0, 1.0, 1.0, 1.0, 40, 36, 34, 10], 2, ["--ic", "sine", "--transport", "ipc"]),
    ("burgers3d", [0.02, 0.3, 2.0, 2.0, 2.0, 36, 32, 30], 1, []),
])
def test_native_warmup_keeps_the_result(tmp_path, app, args, world, extra):
    """--warmup N runs N untimed steps (graphs, handshakes and clocks warm) and restores the
    state: the result equals the run without warm-up bit for bit."""
    env = dict(os.environ)
    if world > 1:
        os.environ.update(ADVDIFF_SHARE_GPU="1", GPU_MAX_HW_QUEUES="2", ADVDIFF_IPC_TIMEOUT_S="60")
    try:
        _run(app, args, tmp_path / "a.bin", world=world, extra=extra)
        txt = _run(app, args, tmp_path / "b.bin", world=world, extra=extra + ["--warmup", "9"])
    finally:
        os.environ.clear()
        os.environ.update(env)
    assert np.array_equal(np.fromfile(tmp_path / "a.bin", dtype=np.float32),
                          np.fromfile(tmp_path / "b.bin", dtype=np.float32)), txt[-400:]


def test_native_watchdog_ends_survivor_without_launcher():
    """Comm watchdog (SURVEY §5 failure detection): two native socket ranks started as
    plain processes (NO fail-fast launcher); rank 1 is stopped (SIGSTOP: alive, sockets
    open, silent) mid-run.  Rank 0, blocked in its next exchange, must end on its own with
    the watchdog's exit code 6 within ADVDIFF_COMM_TIMEOUT (+ margin), not hang."""
    import signal
    import sys
    import time
    from multigpu_advectiondiffusion_amd.launch import _child_env
    exe = ROOT / "bin" / "diffusion3d"
    port = free_port_block(2 + 18)
    cmd = [str(exe), "1", "1", "1", "1", "64", "60", "56", "200000", "--ic", "sine",
           "--transport", "socket"]
    procs = []
    for r in range(2):
        env = _child_env(r, 2, port, cpu=False)
        env.update(ADVDIFF_SHARE_GPU="1", ADVDIFF_COMM_TIMEOUT="10")
        procs.append(subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    try:
        time.sleep(8.0)  # both ranks are stepping (200000 steps take minutes)
        assert procs[0].poll() is None and procs[1].poll() is None, [p.poll() for p in procs]
        os.kill(procs[1].pid, signal.SIGSTOP)
        t0 = time.monotonic()
        try:
            _, err = procs[0].communicate(timeout=60)
        except subprocess.TimeoutExpired:
            pytest.fail("rank 0 still blocked 60 s after its peer stopped")
        waited = time.monotonic() - t0
        assert procs[0].returncode == 6, (procs[0].returncode, err[-1500:])
        assert "[watchdog] rank 0" in err and "no progress" in err, err[-1500:]
        assert waited < 40, waited
        print(f"survivor exited {procs[0].returncode} after {waited:.1f} s", file=sys.stderr)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
            p.wait(timeout=30)


@pytest.mark.parametrize("app,args,model", [
    ("diffusion3d", [1, 1, 1, 1, 60, 44, 36, 4], lambda: Diffusion(K=1.0, order=4)),
    ("burgers3d", [0.01, 0.3, 2, 2, 2, 40, 36, 32], lambda: Burgers(viscosity=1e-5, weno="z", cfl=0.3)),
])
def test_native_field_memory_matches_python(tmp_path, app, args, model):
    """--json reports the device bytes of the resident fields: the fused heat step keeps
    u and its ping-pong partner only (2 fields, as solver.py and utils/sizing.py), the
    per-stage Burgers step 3 — the same bytes as the Python solver's layout."""
    import json
    txt = _run(app, args, tmp_path / "r.bin", extra=["--json"])
    rec = json.loads([ln for ln in txt.splitlines() if ln.startswith("{")][-1])
    m = model()
    shape = tuple(int(a) for a in args[4:7]) if app == "diffusion3d" else tuple(int(a) for a in args[5:8])
    lengths = (1.0, 1.0, 1.0) if app == "diffusion3d" else (2.0, 2.0, 2.0)
    s = Solver(m, Grid(shape, lengths), dtype=torch.float64, device="cuda",
               ic="sine" if app == "diffusion3d" else "gaussian")
    assert rec["device_field_bytes"] == s.memory_bytes(), (rec, s.memory_bytes())
    assert rec["device_field_bytes"] == (2 if app == "diffusion3d" else 3) * s.u.numel() * 8


@pytest.mark.parametrize("app,args,shape", [
    ("diffusion3d", [1.0, 1.0, 1.0, 1.0, 50, 44, 46, 21], (46, 44, 50)),
    ("burgers3d", [0.03, 0.3, 2.0, 2.0, 2.0, 40, 36, 41], (41, 36, 40)),
])
def test_native_pitched_fields_bitwise(tmp_path, app, args, shape):
    """--pitch PX,PY (extra elements per row, extra rows per plane; engine.cpp pitch_pads):
    one rank, 2 socket ranks and 4 ipc ranks on a 2x2x1 grid all give the unpadded 1-rank
    result, and --json reports the padded field bytes the Python solver allocates."""
    import json
    ref = tmp_path / "ref.bin"
    _run(app, args, ref, extra=["--pitch", "0,0"])
    a = np.fromfile(ref, dtype=np.float32).reshape(shape)
    out = tmp_path / "p.bin"
    txt = _run(app, args, out, extra=["--pitch", "8,1", "--json"])
    assert np.array_equal(np.fromfile(out, dtype=np.float32).reshape(shape), a)
    rec = json.loads([ln for ln in txt.splitlines() if ln.startswith("{")][-1])
    if app == "diffusion3d":
        m, grid, ic = Diffusion(K=1.0, order=4), Grid(tuple(args[4:7]), (1.0,) * 3), "sine"
    else:
        m = Burgers(viscosity=1e-5, weno="z", cfl=0.3)
        grid, ic = Grid(tuple(args[5:8]), (2.0,) * 3), "gaussian"
    s = Solver(m, grid, dtype=torch.float64, device="cuda", ic=ic, pitch=(8, 1))
    assert s.sx == 72 and s.u.shape[1] == shape[1] + 1
    assert rec["device_field_bytes"] == s.memory_bytes(), (rec, s.memory_bytes())
    del s
    _run(app, args, out, world=2, extra=["--pitch", "8,1", "--transport", "socket"])
    assert np.array_equal(np.fromfile(out, dtype=np.float32).reshape(shape), a)
    env = dict(os.environ)
    os.environ.update(ADVDIFF_SHARE_GPU="1", GPU_MAX_HW_QUEUES="2", ADVDIFF_IPC_TIMEOUT_S="60")
    try:
        _run(app, args, out, world=4, extra=["--pitch", "8,1", "--transport", "ipc",
                                             "--decomp", "1x2x2"])
    finally:
        os.environ.clear()
        os.environ.update(env)
    assert np.array_equal(np.fromfile(out, dtype=np.float32).reshape(shape), a)


def test_native_default_pitch_matches_python(tmp_path, monkeypatch):
    """Past 128 MiB per field both front ends pad by the same rule (engine.cpp pitch_pads,
    solver.py pitch_default): equal device bytes, and equal results."""
    import json
    monkeypatch.delenv("ADVDIFF_PITCH", raising=False)
    args = [1.0, 1.0, 1.0, 1.0, 260, 256, 262, 2]
    txt = _run("diffusion3d", args, tmp_path / "big.bin", extra=["--ic", "sine", "--json"])
    rec = json.loads([ln for ln in txt.splitlines() if ln.startswith("{")][-1])
    s = Solver(Diffusion(K=1.0, order=4), Grid((260, 256, 262), (1.0,) * 3),
               dtype=torch.float64, device="cuda", ic="sine")
    assert s.ypad == 1 and s.sx == 288 + 4
    assert rec["device_field_bytes"] == s.memory_bytes(), (rec, s.memory_bytes())
    s.run(iters=2)
    got = np.fromfile(tmp_path / "big.bin", dtype=np.float32).reshape(262, 256, 260)
    assert np.array_equal(got, s.gather().astype(np.float32))


@pytest.mark.parametrize("graph", ["--graph", "--no-graph"])
def test_native_fd2_two_step_launch_bitwise(tmp_path, monkeypatch, graph):
    """Single-rank FD2 heat: the engine pairs its steps into two-step launches
    (Engine::step2, advdiff_diffusion3d_step2x) — bitwise equal to one step per launch
    (ADVDIFF_STEP2=0) and to the Python solver (which pairs the same way); odd step count."""
    args = [1.0, 1.0, 1.0, 1.0, 70, 60, 56, 21]
    outs = {}
    for flag in ("1", "0"):
        monkeypatch.setenv("ADVDIFF_STEP2", flag)
        out = tmp_path / f"s{flag}.bin"
        _run("diffusion3d", args, out, extra=["--ic", "sine", "--order", "2", graph])
        outs[flag] = np.fromfile(out, dtype=np.float32).reshape(56, 60, 70)
    assert np.array_equal(outs["1"], outs["0"]), np.abs(outs["1"] - outs["0"]).max()
    monkeypatch.setenv("ADVDIFF_STEP2", "1")
    exp = _py(Diffusion(K=1.0, order=2), Grid((70, 60, 56), (1.0, 1.0, 1.0)), "sine", iters=21)
    assert np.array_equal(outs["1"], exp), np.abs(outs["1"] - exp).max()
