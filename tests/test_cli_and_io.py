"""CPU tests: CLI (reference positional layouts, config files), summaries, I/O,
checkpoints, local launcher, device scan, run-all orchestrator."""
import json
import subprocess
import sys

import numpy as np
import pytest
import torch

from multigpu_advectiondiffusion_amd import Burgers, Diffusion, Grid, Solver, cli
from multigpu_advectiondiffusion_amd.utils import io as aio
from multigpu_advectiondiffusion_amd.utils import metrics


def test_cli_positional_layouts():
    ns = cli.parse(["diffusion3d", "1.0", "10", "10", "10", "21", "19", "20", "5", "32", "4", "4"])
    assert ns.pos["Nx"] == 21 and ns.pos["iters"] == 5 and ns.blocks == ["32", "4", "4"]
    ns = cli.parse(["burgers2d", "0.4", "0.4", "2", "2", "40", "40"])
    assert ns.pos["tEnd"] == 0.4 and ns.pos["Ny"] == 40
    with pytest.raises(SystemExit):
        cli.parse(["diffusion2d", "1.0", "2"])


def test_cli_config_file(tmp_path):
    cfg = tmp_path / "c.json"
    cfg.write_text(json.dumps({"args": [1.0, 1, 1, 16, 16, 3], "ic": "sine", "order": 2}))
    ns = cli.parse(["diffusion2d", "--config", str(cfg)])
    assert ns.order == 2 and ns.ic == "sine" and ns.pos["iters"] == 3
    toml = tmp_path / "c.toml"
    toml.write_text('args = [0.05, 0.3, 2.0, 2.0, 2.0, 16, 16, 16]\nweno = "js"\n')
    ns = cli.parse(["burgers3d", "--config", str(toml)])
    assert ns.weno == "js" and ns.pos["Nz"] == 16


def test_cli_end_to_end_cpu(tmp_path, capsys):
    out = tmp_path / "r.bin"
    rc = cli.main(["diffusion3d", "1.0", "10", "10", "10", "21", "19", "20", "4", "--device", "cpu",
                   "--write", str(out), "--error-norms", "--json"])
    assert rc == 0
    txt = capsys.readouterr().out
    assert "Total effective GFLOPs" in txt and "L1 norm" in txt
    assert "3D Grid Size                                 :  21 x 19 x 20" in txt
    line = [l for l in txt.splitlines() if l.startswith("{")][-1]
    assert json.loads(line)["steps"] == 4
    arr = aio.load_binary(out, (20, 19, 21))
    assert arr.dtype == np.float32 and np.isfinite(arr).all()


def test_summary_labels_byte_compatible():
    txt = metrics.summary_multigpu("Diffusion-3D MPI-GPU-FD4", "Pitched Memory", 1.0, 0.1, 0.2,
                                   5.0, 101, (400, 200, 206))
    lines = txt.splitlines()
    assert lines[1] == "Optimization                                 :  Pitched Memory"
    assert lines[2] == "Kernel time ex. data transfers               :  1.000000 seconds"
    assert lines[8] == "3D Grid Size                                 :  400 x 200 x 206"
    assert lines[9] == "Iterations                                   :  101 x 3 RK steps"
    assert metrics.gflops_reference(6.802646, 101, 400 * 200 * 206) == pytest.approx(5.872, rel=1e-3)


def test_checkpoint_roundtrip_single(tmp_path):
    s = Solver(Burgers(viscosity=1e-3, weno="js"), Grid((16, 14, 18), (2.0, 2.0, 2.0)),
               device="cpu", ic="gaussian")
    s.run(iters=2)
    s.save_checkpoint(tmp_path / "ck")
    s2 = Solver(Burgers(viscosity=1e-3, weno="js"), Grid((16, 14, 18), (2.0, 2.0, 2.0)),
                device="cpu", ic="zero")
    meta = s2.load_checkpoint(tmp_path / "ck")
    assert meta["it"] == 2 and s2.it == 2 and s2.t == s.t
    s.run(iters=2)
    s2.run(iters=2)
    assert np.array_equal(s.gather(), s2.gather())
    with pytest.raises(ValueError):
        Solver(Burgers(), Grid((16, 14, 19), (2.0, 2.0, 2.0)), device="cpu").load_checkpoint(tmp_path / "ck")


def test_checkpoint_rejects_mixed_shards(tmp_path):
    """Stale shards of another checkpoint under the same prefix (an earlier run on more
    ranks) are refused instead of being mixed into the restart."""
    from multigpu_advectiondiffusion_amd.utils import io as aio
    s = Solver(Diffusion(K=1.0), Grid((12, 10, 9), (1.0, 1.0, 1.0)), device="cpu", ic="sine")
    s.run(iters=2)
    s.save_checkpoint(tmp_path / "ck")
    stale = dict(s.meta(), it=7)
    aio.save_checkpoint(tmp_path / "ck", 1, np.zeros((1, 10, 12)), 8, stale)
    with pytest.raises(ValueError, match="another checkpoint"):
        s.load_checkpoint(tmp_path / "ck")


def test_nan_watchdog():
    s = Solver(Diffusion(K=1.0, safety=50.0, fused=False), Grid((16, 16, 16), (1.0, 1.0, 1.0)),
               device="cpu", ic="square", check_every=5)
    with pytest.raises(FloatingPointError):
        s.run(iters=400)


def test_watchdog_catches_an_isolated_nan():
    """One NaN cell among finite ones (max|u| alone can miss it) stops the run."""
    s = Solver(Diffusion(K=1.0), Grid((14, 12, 10), (1.0, 1.0, 1.0)), device="cpu", ic="sine")
    s.check_finite()
    s.owned[3, 4, 5] = float("nan")
    with pytest.raises(FloatingPointError):
        s.check_finite()


def test_cli_geometry_and_graph_flags():
    """--geometry prints every rank's decomposition as JSON and runs no steps (2 gloo ranks,
    Cartesian blocks: the halo phases too); --no-graph runs eagerly with the same result."""
    from multigpu_advectiondiffusion_amd.launch import free_port
    import os
    port = free_port()
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE="2",
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen(
            [sys.executable, "-m", "multigpu_advectiondiffusion_amd", "diffusion3d", "1", "1", "1",
             "1", "20", "18", "16", "5", "--device", "cpu", "--decomp", "1x2x1", "--geometry"],
            env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    outs = [p.communicate(timeout=120)[0] for p in procs]
    assert all(p.returncode == 0 for p in procs), outs
    lines = [json.loads(l) for l in outs[0].splitlines() if l.startswith("{")]
    assert [g["rank"] for g in lines] == [0, 1] and lines[0]["pgrid"] == [1, 2, 1]
    assert lines[0]["halo_phases"] and lines[0]["halo_phases"][0][0]["peer"] == 1
    assert "Total effective GFLOPs" not in outs[0]
    assert cli.main(["diffusion3d", "1", "1", "1", "1", "12", "10", "8", "3", "--device", "cpu",
                     "--no-graph"]) == 0


def test_fp32_cpu_path():
    s = Solver(Diffusion(K=1.0), Grid((20, 20, 20), (1.0, 1.0, 1.0)), device="cpu",
               dtype=torch.float32, ic="sine")
    s.run(iters=3)
    assert s.u.dtype == torch.float32
    l1, l2, linf = s.error_norms()
    assert linf < 5e-2


def test_adaptive_cfl_uses_true_max():
    m = Burgers(viscosity=0.0, cfl=0.3, cfl_mode="adaptive")
    s = Solver(m, Grid((16, 16, 16), (2.0, 2.0, 2.0)), device="cpu", ic="gaussian")
    dt = s.dt()
    assert dt == pytest.approx(0.3 * (2.0 / 15) / s.global_max_abs())


def test_launch_cli_cpu_two_ranks(tmp_path):
    out = tmp_path / "two.bin"
    rc = subprocess.run([sys.executable, "-m", "multigpu_advectiondiffusion_amd.launch", "-np", "2",
                         "--cpu", "--timeout", "200", "diffusion3d", "1", "1", "1", "1", "16", "16",
                         "20", "3", "--ic", "sine", "--write", str(out)],
                        capture_output=True, text=True, timeout=300)
    assert rc.returncode == 0, rc.stderr[-2000:]
    s = Solver(Diffusion(K=1.0), Grid((16, 16, 20), (1.0, 1.0, 1.0)), device="cpu", ic="sine")
    s.run(iters=3)
    two = aio.load_binary(out, (20, 16, 16))
    assert np.array_equal(two, s.gather().astype(np.float32))


def test_devices_scan_runs():
    from multigpu_advectiondiffusion_amd import devices
    d = devices.scan()
    assert "devices" in d


def test_runall_quick_subset(capsys):
    from multigpu_advectiondiffusion_amd import runall
    rc = runall.main(["--quick", "--only", "MG Diffusion2d", "--device", "cpu"])
    assert rc == 0
    assert "2D Grid Size" in capsys.readouterr().out


def test_ascii_dump_and_print(tmp_path, capsys):
    from multigpu_advectiondiffusion_amd.cli import main
    from multigpu_advectiondiffusion_amd.utils import io as aio
    out = tmp_path / "r.txt"
    assert main(["diffusion2d", "1", "1", "1", "9", "7", "3", "--device", "cpu", "--ascii",
                 str(out), "--print"]) == 0
    vals = np.loadtxt(out)
    assert vals.shape == (63,)
    txt = capsys.readouterr().out
    assert txt.count("\n") > 7
    block = aio.format_field(np.arange(6.0).reshape(2, 3))
    assert block.splitlines()[0] == "    0.00    1.00    2.00"


def test_torch_kernel_switch_cpu_equivalence():
    """kernel="torch" is the explicit A/B path; on the CPU both settings run the reference."""
    m, g = Diffusion(K=1.0, order=4), Grid((12, 12, 12), (1.0, 1.0, 1.0))
    a = Solver(m, g, dtype=torch.float64, device="cpu", ic="sine", kernel="torch")
    b = Solver(Diffusion(K=1.0, order=4), g, dtype=torch.float64, device="cpu", ic="sine")
    a.run(iters=2)
    b.run(iters=2)
    assert np.array_equal(a.gather(), b.gather())
    with pytest.raises(ValueError):
        Solver(m, g, dtype=torch.float64, device="cpu", kernel="triton")


def test_write_ghosts_layout(tmp_path):
    """--write-ghosts: the reference's multi-GPU result.bin (every rank's slab WITH its
    ghost planes, rank after rank: SaveBinary3D(h_u, Nx, Ny, _Nz + 6),
    MultiGPU/Diffusion3d_Baseline/main.c:341).  Each block's owned planes equal the
    global result, its inner ghost planes equal the neighbour's boundary planes, and the
    summary block carries timed HtD/DtH lines."""
    out, gh = tmp_path / "res.bin", tmp_path / "ghosts.bin"
    nx, ny, nz, iters = 16, 14, 20, 3
    rc = subprocess.run([sys.executable, "-m", "multigpu_advectiondiffusion_amd.launch", "-np", "2",
                         "--cpu", "--timeout", "200", "diffusion3d", "1", "1", "1", "1", str(nx),
                         str(ny), str(nz), str(iters), "--ic", "sine", "--write", str(out),
                         "--write-ghosts", str(gh)],
                        capture_output=True, text=True, timeout=300)
    assert rc.returncode == 0, rc.stderr[-2000:]
    glob = aio.load_binary(out, (nz, ny, nx))
    raw = np.fromfile(gh, dtype=np.float32)
    G = 6  # fused FD4 step: 3R ghost planes
    counts = [10, 10]
    assert raw.size == sum(c + 2 * G for c in counts) * ny * nx
    blocks = np.split(raw, [(counts[0] + 2 * G) * ny * nx])
    b0 = blocks[0].reshape(counts[0] + 2 * G, ny, nx)
    b1 = blocks[1].reshape(counts[1] + 2 * G, ny, nx)
    assert np.array_equal(b0[G:G + 10], glob[0:10]) and np.array_equal(b1[G:G + 10], glob[10:20])
    assert np.array_equal(b0[G + 10:], glob[10:10 + G])   # rank 0's upper ghosts
    assert np.array_equal(b1[:G], glob[10 - G:10])         # rank 1's lower ghosts
    txt = rc.stdout
    htod = float([l for l in txt.splitlines() if "Data transfer(s) HtD" in l][0].split(":")[1].split()[0])
    dtoh = float([l for l in txt.splitlines() if "Data transfer(s) DtH" in l][0].split(":")[1].split()[0])
    assert htod > 0.0 and dtoh > 0.0
