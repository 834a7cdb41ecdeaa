"""Hang-isolated preflight of (process grid, halo transport) candidates.

The reference fails fast on a communication error: every MPI call returns its error code
(`MPI_ERRORS_RETURN`) and `MPI_CHECK` exits (`MultiGPU/Diffusion3d_Baseline/Tools.c:228-234`).
A device-side transport cannot report a deadlock that way: a grouped RCCL send/recv whose
peer never posts the matching call spins on the GPU and blocks the host in the next wait
— in the process that would then have to report it.  So every candidate a run may use
is first exercised in CHILD processes, where a hang costs a kill and not the run:

* each rank of the caller starts one child (``python -m ...parallel.preflight``; a fresh
  subprocess, never an exec, started before the caller touches the GPU).  The children
  form their own process group — nccl for the rccl candidates, gloo for the host / ipc
  ones — plus a gloo control group;
* per candidate the children build the real Solver (real global grid, process grid,
  transport, schedule) and run `steps` steps, then agree over the control group: ``ok``
  only if every rank finished and all bit hashes equal the one-rank solution of the same
  grid (rank 0 computes it in the child) — a transport that delivers wrong ghosts fails
  here too, not only one that hangs;
* the parent reads the children's progress lines with a deadline per candidate; a child
  silent past it is sent SIGUSR1 (its faulthandler prints every thread's stack to the
  shared stderr), then killed.  Its open candidate is marked failed, and a new session
  with a new port continues with the candidates after it.  A child that dies is treated
  the same way, so the ranks' records agree;
* the last session's children all-gather the failure records over the control group, so
  every rank returns the same verdicts.

Fault injection (``tests/test_bench_deadline.py``): ``ADVDIFF_FAULT=hang:<candidate key>``
makes the last rank's child sleep instead of running that candidate (its peers block in
the exchange, as in a real deadlock); ``corrupt:<candidate key>`` flips one bit of its
solution after the steps.  The children's rendezvous port is
chosen by rank 0's caller and shared through a file keyed by the launcher's pid, the
master port and the world size (all ranks run on one node: bench.py's contract).
"""
from __future__ import annotations

import glob
import json
import os
import queue
import signal
import socket
import subprocess
import sys
import tempfile
import threading
import time

STRIPE = 2  # relay helpers per face message of the striped ipc slab exchange


def transport_kwargs(t) -> dict:
    """Solver keyword arguments of a candidate transport name: "ipc+stripe" = ipc with
    relayed parts, "ipc+fused" = ipc with the halo puts inside the step launch (fused heat
    step, slabs), "ipc+fused+stripe" = both (the heat step's kernel stores the direct and
    the relayed row parts), "rccl+bc" = rccl with the boundary launch on the comm stream,
    "rccl-plain" = rccl with the boundary launch after the interior on the compute
    stream (the pre-round-6 rccl default)."""
    if t is None:
        return {}
    if t == "ipc+stripe":
        return {"transport": "ipc", "stripe": STRIPE}
    if t == "ipc+fused":
        return {"transport": "ipc", "fused_put": True}
    if t == "ipc+fused+stripe":
        return {"transport": "ipc", "fused_put": True, "stripe": STRIPE}
    if t == "rccl+bc":
        return {"transport": "rccl", "boundary_on_comm": True}
    if t == "rccl-plain":
        return {"transport": "rccl", "boundary_on_comm": False}
    return {"transport": t}


def cand_key(model: str, pgrid, transport: str) -> str:
    p = "slab" if pgrid is None else "x".join(str(x) for x in pgrid)
    return f"{model}:{p}/{transport}"


def family(transport: str) -> str:
    """Process-group backend the children of a transport need."""
    return "nccl" if transport.startswith("rccl") else "gloo"


# ---------------------------------------------------------------------------------------
# child side
# ---------------------------------------------------------------------------------------
def _emit(*parts):
    sys.stdout.write("PF " + json.dumps(list(parts)) + "\n")
    sys.stdout.flush()


def _make_model(spec):
    from ..models import Burgers, Diffusion
    kind, kw = spec["model"]
    return Diffusion(**kw) if kind == "diffusion" else Burgers(**kw)


def _solver(spec, comm, pgrid, transport):
    import torch

    from ..models.base import Grid
    from ..solver import Solver
    grid = Grid(tuple(spec["shape"]), tuple(spec["spacing"]))
    return Solver(_make_model(spec), grid, comm, dtype=getattr(torch, spec["dtype"]),
                  ic=spec["ic"], decomp=None if pgrid is None else tuple(pgrid),
                  **transport_kwargs(transport))


def _hang_requested(key: str, rank: int, world: int) -> bool:
    v = os.environ.get("ADVDIFF_FAULT", "")
    return v == f"hang:{key}" and rank == world - 1


def _child_main(spec_path: str) -> int:
    import faulthandler
    faulthandler.enable()
    faulthandler.register(signal.SIGUSR1, all_threads=True)
    with open(spec_path) as f:
        spec = json.load(f)
    import datetime

    import torch
    import torch.distributed as dist

    from .comm import Comm
    torch.set_num_threads(1)
    comm = Comm.from_env(device=spec["device"], backend=spec["backend"],
                         timeout_s=spec["op_timeout"])
    ctl = (dist.new_group(backend="gloo", timeout=datetime.timedelta(seconds=spec["op_timeout"]))
           if comm.backend == "nccl" else None)
    rank, world = comm.rank, comm.size
    _emit("ready", rank)

    def agree(obj):
        out = [None] * world
        dist.all_gather_object(out, obj, group=ctl)
        return out

    failed = dict(spec["failed"])
    ref_hash = {}
    ipc_state = None  # None: not needed / not run; "" ok; else the failure
    for c in spec["cands"]:
        key, mkey = c["key"], c["mkey"]
        _emit("begin", key)
        if _hang_requested(key, rank, world):
            while True:
                time.sleep(3600)
        status = None
        if c["transport"].startswith("ipc") and comm.device.type == "cuda":
            if ipc_state is None:
                try:
                    comm.ipc().preflight()
                    ipc_state = ""
                except Exception as e:  # noqa: BLE001
                    ipc_state = f"ipc pair preflight: {type(e).__name__}: {e}"
            if ipc_state:
                status = ("fail", ipc_state)
        if status is None:
            try:
                s = _solver(spec["models"][mkey], comm, c["pgrid"], c["transport"])
                s.run(iters=spec["steps"], dt=s.model.stable_dt())
                if os.environ.get("ADVDIFF_FAULT", "") == f"corrupt:{key}" and rank == world - 1:
                    o = s.owned  # a wrong ghost plane's effect: one cell off by one ulp
                    i = (0,) * o.dim()
                    o[i] = (o[i].clone().view(1).view(torch.int64) ^ 1).view(o.dtype)[0]
                h = s.bit_hash()
                multi_ipc = s._ipc_multi()
                del s
                if comm.device.type == "cuda":
                    torch.cuda.empty_cache()
                if multi_ipc:
                    comm.ipc().reset()
                status = ("ok", int(h))
            except Exception as e:  # noqa: BLE001 - any failure rejects the candidate
                status = ("fail", f"{type(e).__name__}: {e}"[:400])
        if mkey not in ref_hash and spec["check"]:
            # one-rank solution of the same grid (rank 0, single-process solver)
            h1 = None
            if rank == 0:
                try:
                    single = Comm(device=str(comm.device))
                    s1 = _solver(spec["models"][mkey], single, None, None)
                    s1.run(iters=spec["steps"], dt=s1.model.stable_dt())
                    h1 = int(s1.bit_hash())
                    del s1
                except Exception as e:  # noqa: BLE001 - e.g. the whole grid does not fit
                    print(f"preflight: no one-rank reference for {mkey} "
                          f"({type(e).__name__}: {e}); ranks are still compared with each "
                          "other", file=sys.stderr, flush=True)
                if comm.device.type == "cuda":
                    torch.cuda.empty_cache()
            ref_hash[mkey] = agree(h1)[0]
        every = agree(status)
        bad = [f"rank {r}: {m}" for r, (st, m) in enumerate(every) if st != "ok"]
        if not bad:
            hs = {m for _, m in every}
            if len(hs) != 1:
                bad = [f"ranks disagree on the solution hash ({sorted(hs)})"]
            elif spec["check"] and ref_hash.get(mkey) is not None and hs != {ref_hash[mkey]}:
                bad = [f"{world}-rank solution differs from the one-rank solution "
                       f"(hash {next(iter(hs)) & (2**64 - 1):016x} vs "
                       f"{ref_hash[mkey] & (2**64 - 1):016x})"]
        if bad:
            failed[key] = "; ".join(bad)[:600]
            _emit("fail", key, failed[key])
        else:
            _emit("ok", key)
    # the verdicts every rank will use: union of every rank's failure records
    merged = {}
    for rec in agree(failed):
        for k, v in rec.items():
            merged.setdefault(k, v)
    _emit("agreed", merged)
    sys.stderr.flush()
    os._exit(0)  # no communicator teardown: the verdicts are out, nothing else can hang


# ---------------------------------------------------------------------------------------
# parent side
# ---------------------------------------------------------------------------------------
def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _port_file(session: int) -> str:
    tag = "_".join([str(os.getppid()), os.environ.get("MASTER_PORT", "0"),
                    os.environ.get("WORLD_SIZE", "1"), str(session)])
    return os.path.join(tempfile.gettempdir(), f"advdiff_preflight_{os.getuid()}_{tag}.port")


def _shared_port(rank: int, session: int, wait_s: float = 180.0) -> int:
    """Rendezvous port of a child session: rank 0 picks a free one and publishes it in a
    file (atomic rename) that the other ranks of this launch poll."""
    path = _port_file(session)
    if rank == 0:
        port = _free_port()
        tmp = f"{path}.{os.getpid()}.tmp"
        with open(tmp, "w") as f:
            f.write(str(port))
        os.replace(tmp, path)
        return port
    t0 = time.monotonic()
    while time.monotonic() - t0 < wait_s:
        try:
            with open(path) as f:
                txt = f.read().strip()
            if txt:
                return int(txt)
        except (OSError, ValueError):
            pass
        time.sleep(0.05)
    raise TimeoutError(f"preflight: no session port from rank 0 within {wait_s:g} s ({path})")


def _reader(stream, q):
    for line in stream:
        if line.startswith("PF "):
            try:
                q.put(json.loads(line[3:]))
            except ValueError:
                pass
    q.put(None)


def _run_session(spec, rank, world, session, init_s, cand_s, log):
    """One child session.  Returns (closed: {key: verdict} of the candidates it finished,
    agreed: the children's merged failure records, or None if the session did not end
    cleanly, dead_at_start: it ended before any candidate began)."""
    port = _shared_port(rank, session)
    fd, path = tempfile.mkstemp(prefix="advdiff_pf_", suffix=".json")
    with os.fdopen(fd, "w") as f:
        json.dump(spec, f)
    # the children's process group is their own: drop torchrun's agent-store setting
    # (TORCHELASTIC_USE_AGENT_STORE=True makes rank 0 connect to MASTER_PORT as a client
    # instead of serving the store) and the rest of the elastic agent's variables
    env = {k: v for k, v in os.environ.items() if not k.startswith(("TORCHELASTIC_", "TORCH_ELASTIC"))}
    env.update({"RANK": str(rank), "LOCAL_RANK": os.environ.get("LOCAL_RANK", str(rank)),
                "WORLD_SIZE": str(world), "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    pkg_root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    env["PYTHONPATH"] = os.pathsep.join([pkg_root] + [x for x in [env.get("PYTHONPATH")] if x])
    if spec["backend"] == "gloo":
        env["ADVDIFF_BACKEND"] = "gloo"
    p = subprocess.Popen([sys.executable, "-u", "-m", __name__, path], env=env,
                         stdout=subprocess.PIPE, text=True, bufsize=1)
    q = queue.Queue()
    threading.Thread(target=_reader, args=(p.stdout, q), daemon=True).start()
    closed, agreed, open_key = {}, None, None
    limit = time.monotonic() + init_s
    why = None
    ready = False
    # a child that dies before its process group is up leaves a marker next to the port
    # file, so the other ranks' children (blocked in the rendezvous) are ended at once
    # instead of after init_s
    dead_mark = f"{_port_file(session)}.dead"
    try:
        while True:
            try:
                msg = q.get(timeout=max(0.05, min(1.0, limit - time.monotonic())))
            except queue.Empty:
                if not ready and glob.glob(dead_mark + ".*"):
                    why = "another rank's preflight child died starting the process group"
                    break
                if time.monotonic() > limit:
                    why = (f"no progress within {cand_s if open_key else init_s:g} s "
                           f"({'in the exchange' if open_key else 'starting the process group'})")
                    break
                continue
            if msg is None:  # the child's stdout closed: it exited
                rc = p.wait()
                if agreed is None:
                    why = f"preflight child exited with {rc}"
                    if not ready:
                        with open(f"{dead_mark}.{rank}", "w") as f:
                            f.write(str(rc))
                break
            kind = msg[0]
            if kind == "ready":
                ready = True
                limit = time.monotonic() + cand_s
            elif kind == "begin":
                open_key = msg[1]
                limit = time.monotonic() + cand_s
            elif kind in ("ok", "fail"):
                closed[msg[1]] = "ok" if kind == "ok" else msg[2]
                open_key = None
                limit = time.monotonic() + cand_s
            elif kind == "agreed":
                agreed = msg[1]
                limit = time.monotonic() + 20.0  # the child exits right after
    finally:
        if p.poll() is None and agreed is None:
            try:  # stacks of every thread of the stuck child -> the shared stderr
                p.send_signal(signal.SIGUSR1)
                p.wait(timeout=2.0)
            except (subprocess.TimeoutExpired, OSError):
                pass
        if p.poll() is None:
            p.kill()
            p.wait()
        os.unlink(path)
        if rank == 0:
            for f in [_port_file(session)] + glob.glob(dead_mark + ".*"):
                try:
                    os.unlink(f)
                except OSError:
                    pass
    if agreed is None:
        if open_key is not None:
            closed[open_key] = f"hang or crash: {why}"
            log(f"preflight: candidate {open_key} failed ({why})")
        else:
            log(f"preflight: session {session} failed before a candidate ({why})")
    return closed, agreed, (open_key is None and agreed is None)


def run_preflight(cands, models, *, device: str, backend: str, steps: int = 2,
                  cand_s: float = 60.0, init_s: float = 90.0, total_s: float = 300.0,
                  op_timeout: float = 120.0, check: bool = True, log=None,
                  max_hangs: int = 2) -> dict:
    """Exercise every candidate in hang-isolated child sessions (module doc).

    cands: [(mkey, pgrid, transport)] — mkey names an entry of `models`:
    {mkey: {"model": (kind, kwargs), "shape", "spacing", "ic", "dtype"}}; backend: the
    children's process-group backend ("nccl" for rccl candidates, "gloo" otherwise).
    Returns {key: "ok" | failure text} for every candidate, the same on every rank (the
    children agree over their control group; a candidate that hung is failed on every
    rank, because every rank's session ends at it).  After `max_hangs` hangs the family's
    remaining candidates are not run (a transport that deadlocks twice is not trusted,
    and each hang costs cand_s of the run's budget).  Call it on every rank, before the
    caller touches the GPU."""
    log = log or (lambda m: print(m, file=sys.stderr, flush=True))
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    try:
        return _preflight(cands, models, device, backend, steps, cand_s, init_s, total_s,
                          op_timeout, check, log, max_hangs, rank, world)
    except (OSError, TimeoutError) as e:
        # the preflight machinery itself failed (no rendezvous file from rank 0, no port):
        # nothing was learnt about the candidates — the caller keeps them all, as before
        # the preflight existed, and records why
        log(f"preflight: unavailable ({type(e).__name__}: {e}); candidates kept unverified")
        return {cand_key(m, p, t): "ok (unverified: preflight unavailable)" for m, p, t in cands}


def _preflight(cands, models, device, backend, steps, cand_s, init_s, total_s, op_timeout,
               check, log, max_hangs, rank, world) -> dict:
    todo = [{"key": cand_key(m, p, t), "mkey": m, "pgrid": p, "transport": t}
            for m, p, t in cands]
    verdict, failed = {}, {}
    t_end = time.monotonic() + total_s
    session = 0
    while True:
        spec = {"cands": todo, "models": models, "device": device, "backend": backend,
                "steps": steps, "op_timeout": op_timeout, "failed": failed, "check": check}
        left = t_end - time.monotonic()
        closed, agreed, dead_at_start = _run_session(
            spec, rank, world, session, min(init_s, max(left, 5.0)),
            min(cand_s, max(left, 5.0)), log)
        session += 1
        if agreed is not None:
            for c in todo:
                verdict[c["key"]] = agreed.get(c["key"], "ok")
            for k, v in agreed.items():
                verdict.setdefault(k, v)
            return verdict
        for k, v in closed.items():
            verdict[k] = v
            if v != "ok":
                failed[k] = v
        hangs = sum(v.startswith("hang") for v in verdict.values())
        if dead_at_start or time.monotonic() > t_end or hangs >= max_hangs:
            why = ("the preflight process group did not start" if dead_at_start
                   else f"preflight budget of {total_s:g} s spent" if hangs < max_hangs
                   else f"{hangs} candidates of this transport family hung")
            for c in todo:
                if c["key"] not in verdict:
                    verdict[c["key"]] = f"not run: {why}"
            return verdict
        todo = [c for c in todo if c["key"] not in verdict]
        # a session that hung at its last candidate: one more (empty) session only agrees


if __name__ == "__main__":
    sys.exit(_child_main(sys.argv[1]))
