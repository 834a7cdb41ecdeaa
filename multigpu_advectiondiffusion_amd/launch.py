"""Local multi-process launcher (the reference's ``mpirun -np P``, `MultiGPU/*/run.sh`).

Two entry points:

* CLI: ``python -m multigpu_advectiondiffusion_amd.launch -np 8 diffusion3d 1 2 2 2 512 512 512 100``
  starts P child processes of ``python -m multigpu_advectiondiffusion_amd`` (``--native``:
  of the C++ executable ``bin/<app>``) with the
  torchrun environment (RANK, LOCAL_RANK, WORLD_SIZE, MASTER_ADDR=127.0.0.1,
  MASTER_PORT) — one process per GPU; ``--cpu`` runs P gloo ranks on the CPU (the
  oversubscription / no-cluster test mode of SURVEY.md §4, done properly).
* ``--profile DIR``: every rank runs under its own profiler, ``rocprofv3 --kernel-trace
  --output-format csv -d DIR/rank<r> -- <rank command>`` (the reference profiles each MPI
  rank into its own file: ``nvprof -o X.%q{OMPI_COMM_WORLD_RANK}.nvprof``,
  `MultiGPU/Diffusion3d_Baseline/run.sh:2`, `profile.sh:1-2`); bench/trace_overlap.py
  reads the per-rank directories.
* ``launch_cmd(P, cmd)``: the same fail-fast supervision for any command (bench.py
  self-launches its ranks with it).
* API: ``spawn_local(world, fn, *args)`` runs ``fn(comm, *args)`` in `world` fresh
  processes with an initialised process group and returns the per-rank results — used
  by the multi-rank tests.

Children are started as subprocesses (never exec'd from a process that touched the GPU).
"""
from __future__ import annotations

import argparse
import os
import socket
import subprocess
import sys
import traceback


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def free_port_block(n: int, tries: int = 64) -> int:
    """A base port b with b .. b+n all bindable right now: the native socket transport
    listens on ADVDIFF_PORT (rendezvous) and ADVDIFF_PORT+1+i (rank i of the full mesh),
    so a lone free port is not enough on a busy host."""
    import random
    for _ in range(tries):
        # below Linux's ephemeral range (32768+): an outgoing connection of another
        # process (or of an earlier rank) cannot take a port of the block meanwhile
        b = random.randint(20000, 32000 - n - 1)
        socks = []
        try:
            for q in range(b, b + n + 1):
                s = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
                socks.append(s)
                s.bind(("0.0.0.0", q))
            return b
        except OSError:
            continue
        finally:
            for s in socks:
                s.close()
    return free_port()


def _child_env(rank: int, world: int, port: int, cpu: bool) -> dict:
    env = dict(os.environ)
    env.update({"RANK": str(rank), "LOCAL_RANK": str(rank), "WORLD_SIZE": str(world),
                "LOCAL_WORLD_SIZE": str(world), "MASTER_ADDR": "127.0.0.1",
                "MASTER_PORT": str(port)})
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    if cpu:
        env["ADVDIFF_DEVICE"] = "cpu"
    return env


def profiled(cmd: list, profile_dir: str, rank: int) -> list:
    """`cmd` under its own rocprofv3 kernel trace in profile_dir/rank<r> (the program
    itself right after `--`: no env/shell hop the profiler's preload would exec through)."""
    import shutil
    prof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    return [prof, "--kernel-trace", "--output-format", "csv", "-d",
            os.path.join(profile_dir, f"rank{rank}"), "--"] + list(cmd)


def launch_cmd(np_: int, cmd, cpu: bool = False, timeout: float | None = None,
               poll_s: float = 0.2, port: int | None = None,
               profile_dir: str | None = None, extra_env: dict | None = None,
               dump_signal: int | None = None) -> int:
    """Run `cmd` (a list, or a callable rank -> list) as P ranks with the torchrun
    environment; fail fast: the first rank that exits non-zero (or the wall-clock
    `timeout`, rc 124) terminates the others, so a crashed rank never leaves its peers
    blocked in a halo exchange until the collective timeout.  dump_signal (e.g.
    signal.SIGUSR1 for ranks that registered faulthandler on it, as bench.py's do): sent
    to the ranks still alive before they are terminated, so their stacks — where each
    one was stuck — reach the shared stderr.  Returns the first non-zero exit code (0 if
    all succeed).  The ranks are fresh subprocesses (never an exec)."""
    import time
    port = port or free_port()
    procs = []
    for r in range(np_):
        c = cmd(r) if callable(cmd) else list(cmd)
        if profile_dir:
            c = profiled(c, profile_dir, r)
        env = _child_env(r, np_, port, cpu)
        if extra_env:
            env.update(extra_env)
        procs.append(subprocess.Popen(c, env=env))
    deadline = None if timeout is None else time.monotonic() + timeout
    rc = 0
    try:
        while True:
            codes = [p.poll() for p in procs]
            bad = [(r, c) for r, c in enumerate(codes) if c not in (None, 0)]
            if bad:
                r, rc = bad[0]
                print(f"[launch] rank {r} exited with {rc}; terminating the other ranks",
                      file=sys.stderr, flush=True)
                break
            if all(c == 0 for c in codes):
                break
            if deadline is not None and time.monotonic() > deadline:
                print(f"[launch] timeout after {timeout:g} s", file=sys.stderr, flush=True)
                rc = 124
                break
            time.sleep(poll_s)
    finally:
        alive = [p for p in procs if p.poll() is None]
        if alive and dump_signal is not None:
            for p in alive:
                try:
                    p.send_signal(dump_signal)
                except OSError:
                    pass
            time.sleep(2.0)  # the stack dumps are written by a C-level handler
        for p in procs:
            if p.poll() is None:
                p.terminate()
        for p in procs:
            try:
                p.wait(timeout=10)
            except subprocess.TimeoutExpired:
                p.kill()
    return rc


def launch(np_: int, argv: list[str], cpu: bool = False, timeout: float | None = None,
           poll_s: float = 0.2, native: bool = False, profile_dir: str | None = None) -> int:
    """Run P ranks of the Python front end (or, native=True, of bin/<app>); see
    launch_cmd.  Returns the first non-zero exit code (0 if all succeed)."""
    # native ranks listen on MASTER_PORT+17 (rendezvous) and MASTER_PORT+18+i (socket mesh)
    port = free_port_block(np_ + 18) if native else free_port()
    if native:  # the C++ executables: bin/<app> <args...> (RCCL or --transport socket)
        from pathlib import Path
        exe = Path(__file__).resolve().parent.parent / "bin" / argv[0]
        if not exe.exists():
            raise FileNotFoundError(f"{exe} not built (make -C csrc apps)")
        cmd = [str(exe)] + argv[1:]
    else:
        cmd = [sys.executable, "-m", "multigpu_advectiondiffusion_amd"] + argv
    if cpu and not native and "--device" not in argv:
        cmd += ["--device", "cpu"]
    return launch_cmd(np_, cmd, cpu=cpu, timeout=timeout, poll_s=poll_s, port=port,
                      profile_dir=profile_dir)


# ----------------------------------------------------------------------------------
# in-process API for tests
# ----------------------------------------------------------------------------------
def _spawn_entry(rank, world, port, device, backend, fn, args, queue, transport=None,
                 dump_after=None):
    os.environ.update({"RANK": str(rank), "LOCAL_RANK": str(rank), "WORLD_SIZE": str(world),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    import faulthandler
    faulthandler.enable()  # a crashing rank (SIGSEGV / SIGABRT) prints its Python stack
    if dump_after:
        # a rank still running shortly before the parent gives up prints every thread's
        # stack (captured with the test's stderr): a deadlock names its call site
        faulthandler.dump_traceback_later(dump_after, exit=False)
    try:
        import torch
        torch.set_num_threads(1)
        from .parallel.comm import Comm
        comm = Comm.from_env(device=device, backend=backend, transport=transport)
        try:
            res = fn(comm, *args)
        finally:
            comm.finalize()
        queue.put((rank, "ok", res))
    except BaseException as e:  # report instead of hanging the parent
        queue.put((rank, "err", f"{type(e).__name__}: {e}\n{traceback.format_exc()}"))


def spawn_local(world: int, fn, *args, device: str = "cpu", backend: str | None = None,
                timeout: float = 300.0, transport: str | None = None):
    """Run fn(comm, *args) on `world` local ranks; return [result_rank0, ...].
    transport: the halo transport of device fields (Comm.transport; "ipc" with
    ADVDIFF_SHARE_GPU=1 runs all ranks on one GPU with device-side exchanges)."""
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    import queue as _queue
    import time
    dump_after = max(timeout - 20.0, timeout * 0.75)
    procs = [ctx.Process(target=_spawn_entry,
                         args=(r, world, port, device, backend, fn, args, q, transport,
                               dump_after))
             for r in range(world)]
    for p in procs:
        p.start()
    results = [None] * world
    errors = []
    done = set()
    deadline = time.monotonic() + timeout
    dead_since = None
    try:
        while len(done) < world:
            try:
                rank, status, payload = q.get(timeout=1.0)
            except _queue.Empty:
                late = [r for r in range(world) if r not in done]
                # a rank that died (signal / non-zero exit) without reporting: give the
                # queue a short grace, then fail now instead of at the deadline (its
                # faulthandler stack is in the captured stderr)
                dead = [(r, procs[r].exitcode) for r in late
                        if procs[r].exitcode not in (None, 0)]
                if dead:
                    dead_since = dead_since or time.monotonic()
                    if time.monotonic() - dead_since > 3.0:
                        raise RuntimeError(f"spawn_local: ranks {dead} (rank, exit code) died "
                                           "without reporting; their stacks are in stderr")
                if time.monotonic() > deadline:
                    gone = [(r, procs[r].exitcode) for r in late if not procs[r].is_alive()]
                    raise TimeoutError(f"spawn_local: ranks {late} did not finish within "
                                       f"{timeout:g} s (exited without reporting: {gone}); "
                                       "their stacks were dumped to stderr") from None
                continue
            done.add(rank)
            if status == "ok":
                results[rank] = payload
            else:
                errors.append(f"rank {rank}: {payload}")
    finally:
        for p in procs:
            p.join(timeout=10)
            if p.is_alive():
                p.kill()
    if errors:
        raise RuntimeError("\n".join(errors))
    return results


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="launch P local ranks (one per GPU)")
    ap.add_argument("-np", "--nproc", type=int, required=True)
    ap.add_argument("--cpu", action="store_true", help="gloo ranks on the CPU")
    ap.add_argument("--timeout", type=float, default=None)
    ap.add_argument("--native", action="store_true",
                    help="run the native executable bin/<app> instead of the Python front end")
    ap.add_argument("--profile", default=None, metavar="DIR",
                    help="run every rank under its own rocprofv3 kernel trace in DIR/rank<r>")
    ap.add_argument("rest", nargs=argparse.REMAINDER)
    ns = ap.parse_args(argv)
    return launch(ns.nproc, ns.rest, cpu=ns.cpu, timeout=ns.timeout, native=ns.native,
                  profile_dir=ns.profile)


if __name__ == "__main__":
    sys.exit(main())
