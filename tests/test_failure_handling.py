"""Failure detection (absent in the reference, which only exits on MPI
errors): fail-fast launcher, fault injection, launcher timeout, NaN/Inf watchdog."""
import time

import pytest

from multigpu_advectiondiffusion_amd.launch import launch

ARGS = ["diffusion3d", "1", "1", "1", "1", "20", "20", "24", "400"]


def test_launcher_fail_fast_on_injected_fault(monkeypatch):
    monkeypatch.setenv("ADVDIFF_FAULT", "1:3")  # rank 1 raises after step 3
    monkeypatch.setenv("ADVDIFF_COMM_TIMEOUT", "300")
    t0 = time.monotonic()
    rc = launch(2, ARGS, cpu=True, timeout=240)
    # rank 0 is left blocked in a halo receive; the launcher must kill it right away
    assert rc not in (0, 124)
    assert time.monotonic() - t0 < 120


def test_launcher_timeout(monkeypatch):
    monkeypatch.setenv("ADVDIFF_COMM_TIMEOUT", "300")
    rc = launch(2, ["diffusion3d", "1", "1", "1", "1", "40", "40", "40", "100000"], cpu=True,
                timeout=20)
    assert rc == 124


def test_launcher_success():
    assert launch(2, ARGS[:-1] + ["3"], cpu=True, timeout=240) == 0

# NaN/Inf watchdog: tests/test_cli_and_io.py::test_nan_watchdog*


def test_launcher_profile_wraps_each_rank(monkeypatch, tmp_path):
    """--profile DIR: every rank's command is its own rocprofv3 kernel trace into
    DIR/rank<r>, the program right after `--` (no shell / env hop)."""
    from multigpu_advectiondiffusion_amd import launch as L
    seen = []

    class P:
        def __init__(self, cmd, env):
            seen.append((cmd, env["RANK"]))

        def poll(self):
            return 0

        def wait(self, timeout=None):
            return 0

    monkeypatch.setattr(L.subprocess, "Popen", P)
    assert L.launch(2, ["diffusion3d", "1", "1", "1", "1", "8", "8", "8", "2"], cpu=True,
                    profile_dir=str(tmp_path)) == 0
    for cmd, rank in seen:
        i = cmd.index("--")
        assert cmd[0].endswith("rocprofv3") and "--kernel-trace" in cmd[:i]
        assert cmd[cmd.index("-d") + 1] == str(tmp_path / f"rank{rank}")
        assert cmd[i + 1] == __import__("sys").executable


def _die_on_rank1(comm):
    import os
    if comm.rank == 1:
        os._exit(7)  # no report, no traceback: like a segfault inside a HIP call
    comm.barrier()  # rank 0 blocks in a collective its peer never joins
    return comm.rank


def test_spawn_local_reports_a_dead_rank_fast():
    """A rank that dies without reporting (the round-4 graph-capture crash looked like a
    240 s hang) fails spawn_local within seconds, naming the rank and its exit code."""
    import time

    from multigpu_advectiondiffusion_amd.launch import spawn_local
    t0 = time.monotonic()
    with pytest.raises(RuntimeError, match=r"\(1, 7\)"):
        spawn_local(2, _die_on_rank1, timeout=120)
    assert time.monotonic() - t0 < 60
