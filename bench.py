#!/usr/bin/env python3
"""Headline benchmark (BASELINE.json): whole-node MLUPS of the fp64 3-D heat solver
(FD4 13-point + SSP-RK3, synthetic sinusoidal IC) with per-GPU work fixed at 512³ cells
(weak scaling: 1 GPU -> 512³, 8 GPUs -> 1024³), plus the 3-D WENO5-Z viscous Burgers
solver at 256³ per GPU reported alongside.

    python bench.py --gpus N --steps K --warmup W
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

One RK3 step of the heat solver = ONE temporally blocked launch that computes all three
SSP-RK3 stages (diffusion_fused.hip; bit-identical to three per-stage launches) + ONE halo
exchange of 3R ghost planes per step when N > 1 (no work skipped).  Burgers steps are three
fused WENO stage launches + three exchanges.  K steps are timed between a barrier + device
sync on both sides; the max over ranks is reported.  MLUPS = global cells x K / seconds /
1e6.  Rank 0 prints ONE JSON line.

Self-validation (outside the timed region): after the timed steps the heat solution is
compared with the exact decaying sine mode exp(-3 pi^2 K t) sin sin sin (L_inf, relative to
the initial amplitude) and the run fails if it exceeds linf_bound().  The 7-point (FD2)
Laplacian named by BASELINE.json is measured on the same grid and reported as `fd2_7pt`.

Clock settling: the fp64 stencil load runs the chip at its power limit, and the clock
controller dips for tens of ms after a load starts (per-launch times rise from 676 to 862
us and decay over ~20 launches: profiles/archive/launch_times_r2s5.txt), so a 20-step
window right behind a few warm-up steps times the dip.  After the W warm-up steps the
bench therefore runs --settle-ms (default 300 ms) more untimed steps of the same solver,
then times exactly K steps; the count is reported as `settle`.  `sustained`
(informational, AFTER the K timed steps): --sustained-steps more steps timed the same way.

Failure handling (N > 1 has never run on distinct GPUs before the driver's node): every
(process grid, transport) candidate first runs 2 real steps in hang-isolated child
process groups (parallel/preflight.py: a candidate that hangs, crashes or differs from
the one-rank solution is dropped and recorded in `preflight`); the whole run has one
deadline below the driver's limit (--deadline, default 540 s from the launcher's start):
every rank dumps its stacks 15 s before it, and at it rank 0 prints the JSON line with
whatever finished (`status` says where it stopped) and every rank exits 124.

FD2 on one GPU runs one RK3 step per launch or two (diffusion_fused.hip v6_march;
bit-identical), whichever the solver measured faster for the shape at construction
(advdiff_diffusion3d_step2_pick; at 512^3 fp64 one step per launch wins by 3 %):
`fd2_7pt.steps_per_launch`.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
# (the package is imported inside run(): a self-launching parent, --gpus N without
# WORLD_SIZE, never touches the GPU)

METRIC = "MLUPS (whole node), 3D diffusion 512^3 + Burgers3D WENO5, 1/2/4/8 MI355X"
BASE_DIFFUSION = 927.2   # best published 3-D heat MLUPS (SingleGPU/Diffusion3d_Blocking/Run.m:3-12)
BASE_BURGERS = 344.4     # best published 3-D Burgers MLUPS (SingleGPU/Burgers3d_WENO5_PitchedMem/Run.m:15-25)
# L_inf bound of the timed Burgers solution vs the same steps through the PyTorch fp64
# reference ops (ops/reference.py): both are fp64 WENO5-Z with different operation orders,
# so they agree to accumulated rounding (measured: profiles/r5/bench_burgers_ref.log); a
# wrong face, halo or stage gives O(dt |u|) ~ 1e-3 and fails it
BURGERS_REF_BOUND = 1e-9


def linf_bound(grid, K: float, t: float, order: int) -> float:
    """Bound of L_inf(u - exact) for the sine mode after time t (unit amplitude).

    The scheme's truncation error is O(h^4) (FD4) / O(h^2) (FD2) ~ 1e-10 here; what
    dominates is the reference's Dirichlet treatment: FD4 freezes the 2-cell border
    (`MultiGPU/Diffusion3d_Baseline/Kernels.cu` updates [2, n-2)), so the cell at distance
    h from a wall keeps its initial value sin(pi h) while the exact mode decays by
    exp(-lam t): |error| <= sin(pi h)(1 - exp(-lam t)) there, less inside.  Twice that plus
    the truncation allowance is the bound; a wrong stencil, halo plane or schedule gives
    errors of O(dt/h^2 * |u|) ~ 1e-1 and fails it."""
    import math
    Ls = [(n - 1) * d for n, d in zip(grid.shape, grid.spacing)]
    lam = K * math.pi ** 2 * sum(1.0 / L ** 2 for L in Ls)
    h = max(d / L for d, L in zip(grid.spacing, Ls))
    frozen = math.sin(math.pi * h) * (1.0 - math.exp(-lam * t)) if order == 4 else 0.0
    trunc = 1e-9 if order == 4 else 10.0 * (math.pi * h) ** 2 * lam * t
    return 2.0 * frozen + trunc


SETTLE = {}  # model -> settle record of its last timed() call (reported in the JSON)


def timed(solver, steps: int, warmup: int, dt: float, settle_ms: float = 0.0,
          key: str = "heat") -> float:
    """W warm-up steps, then settle_ms of further untimed steps of the same solver (the
    power controller's clock dip after a load starts lasts tens of ms: a short window
    right behind a few warm-up steps times the dip, not the solver), then exactly K timed
    steps between a barrier + device sync on both sides (max over ranks)."""
    per = None
    if warmup:
        per = solver.run(iters=warmup, dt=dt).compute_s / warmup
    n_settle = 0
    if settle_ms > 0:
        if per is None:
            per = solver.run(iters=2, dt=dt).compute_s / 2
            n_settle += 2
        # compute_s is the max over ranks, so every rank takes the same count; even keeps
        # the u/un parity of the timed run
        n = int(settle_ms * 1e-3 / max(per, 1e-6)) + 1
        n += n % 2
        solver.run(iters=n, dt=dt)
        n_settle += n
    SETTLE[key] = {"steps": n_settle, "target_ms": settle_ms}
    st = solver.run(iters=steps, dt=dt)  # barrier + sync on both sides, max over ranks
    return st.compute_s


def sustained(solver, steps: int, dt: float, cells: int) -> dict | None:
    """Informational settled-clock rate: `steps` more steps right after the headline
    window, timed the same way (barrier + sync both sides, max over ranks)."""
    if steps <= 0:
        return None
    st = solver.run(iters=steps, dt=dt)
    return {"steps": steps, "value": round(cells * steps / st.compute_s / 1e6, 1),
            "ms_per_step": round(st.compute_s / steps * 1e3, 4)}


def _free(dev):
    if dev.type == "cuda":
        torch.cuda.empty_cache()


def _fingerprint(s):
    """(Σ|u|, Σu², max|u|) over the global owned cells: identical to rounding for every
    decomposition (the kernels are bitwise decomposition-invariant; only the order of
    the cross-rank sum differs)."""
    s.sync_halos()
    a, b, c = s.reducer()(s.u, None, s._owned_xyz_box())
    return (s.comm.allreduce_sum(a), s.comm.allreduce_sum(b), s.comm.allreduce_max(c))


_T0 = time.perf_counter()


def progress(comm, msg):
    """One stderr line per bench phase (rank 0): long multi-rank runs show they are alive."""
    if comm.rank == 0:
        print(f"bench [{time.perf_counter() - _T0:7.1f} s] {msg}", file=sys.stderr, flush=True)


def tune(make, cands, dt, dev, trial_steps=8, rounds=3):
    """Autotuning of the (process grid, halo transport) pair, N > 1, outside the timed
    region.  cands = [(pgrid, transport)]: the slab + grids of
    parallel.decomposition.candidate_proc_grids (fewer bytes over the busiest xGMI link)
    times the transports that passed their preflight (rccl: grouped RCCL send/recv,
    stepped eagerly; ipc: device puts, hipGraph-replayed).  Every candidate is built,
    warmed up by 2 steps, then timed over `rounds` interleaved rounds of `trial_steps`
    steps (A B C A B C ..., so the chip's power-management clock dip cannot favour
    whichever runs first; trial_steps = one graph's worth, so graph-replayed candidates
    are timed as the run will use them); a candidate's time is its best round (max over
    ranks, so every rank picks the same).  The fastest candidate whose solution matches
    the first's (global Σ|u|, Σu², max|u| to 1e-10 relative) wins.
    Returns ((pgrid, transport), {"ZxYxX/transport": ms/step or a rejection note})."""
    if len(cands) == 1:
        return cands[0], {}
    solvers = []
    for p, t in cands:
        s = make(p, t)
        s.run(iters=2, dt=dt)
        solvers.append(s)
    best_ms = [float("inf")] * len(cands)
    for _ in range(rounds):
        for i, s in enumerate(solvers):
            ms = s.run(iters=trial_steps, dt=dt).compute_s / trial_steps * 1e3
            best_ms[i] = min(best_ms[i], ms)
    trials, best, ref = {}, None, None
    for (p, t), s, ms in zip(cands, solvers, best_ms):
        fp = _fingerprint(s)
        key = "x".join(map(str, p)) + "/" + t
        if ref is None:
            ref = fp
        elif any(abs(x - y) > 1e-10 * max(abs(y), 1e-300) for x, y in zip(fp, ref)):
            trials[key] = f"rejected: solution differs from the first candidate's ({fp} vs {ref})"
            continue
        trials[key] = round(ms, 4)
        if best is None or ms < best[0]:
            best = (ms, (p, t))
    del solvers, s
    _free(dev)
    return best[1], trials


from multigpu_advectiondiffusion_amd.parallel.preflight import (  # noqa: E402
    cand_key, family, run_preflight, transport_kwargs as solver_transport)


def planned_transports(world: int, on_gpu: bool, want: str) -> list:
    """Halo transports the run may use (before any process group exists): with the nccl
    backend rccl (boundary launch on the comm stream, the default schedule), rccl-plain
    (boundary launch after the interior), ipc, ipc+fused (the heat step's halo puts inside
    its one launch; slabs) and, at 7-8 ranks, ipc+stripe and ipc+fused+stripe; with ranks
    sharing one GPU (ADVDIFF_SHARE_GPU=1, gloo) host, ipc and ipc+fused (+ the striped
    pair); on the CPU host only."""
    if world == 1:
        return [None]
    if not on_gpu:
        return ["host"]
    if want != "tune":
        return [want]
    if os.environ.get("ADVDIFF_SHARE_GPU", "0") == "1" or os.environ.get("ADVDIFF_BACKEND") == "gloo":
        names = ["host", "ipc", "ipc+fused"]
    else:
        names = ["rccl", "rccl-plain", "ipc", "ipc+fused"]
    from multigpu_advectiondiffusion_amd.parallel.ipc import stripe_plan
    if any(stripe_plan(world, STRIPE).values()):  # 7-8 ranks: idle links exist
        names += ["ipc+stripe", "ipc+fused+stripe"]
    return names


STRIPE = 2


def ipc_pair_check(comm, names):
    """The main process's own ipc pair preflight (its fields are new mappings): a failure
    drops ipc from the candidates.  Returns (names, record)."""
    if not any(t.startswith("ipc") for t in names) or comm.size == 1:
        return names, None
    try:
        pre = comm.ipc().preflight()
    except Exception as e:  # noqa: BLE001 - any failure rejects the transport
        pre = f"failed: {type(e).__name__}: {e}"
        if comm.rank == 0:
            print(f"bench: ipc transport rejected ({pre})", file=sys.stderr, flush=True)
        names = [t for t in names if not t.startswith("ipc")]
    return names, pre


def bitwise_vs_1gpu(make_n, make_1, steps, dt, comm, dev):
    """N > 1: the timed configuration (fresh solver, same process grid and transport —
    graph replay included for ipc) and ONE GPU (rank 0's, a single-process solver of the
    same global grid) run the same `steps` steps; their bit_hash()es (order-independent
    64-bit hash of every cell's bit pattern with its global index) must agree.  The
    kernels are bitwise decomposition-invariant, so any difference is a halo or transport
    error (a stale ghost plane, a lost put) — which a tolerance check against the exact
    solution could miss.  Returns (equal, {"hash_n", "hash_1"})."""
    s = make_n()
    s.run(iters=steps, dt=dt)
    hn = s.bit_hash()
    ipc = s._ipc_multi()
    del s
    _free(dev)
    if ipc:
        comm.ipc().reset()  # the peers unmap the freed fields before rank 0 reallocates
    h1 = None
    if comm.rank == 0:
        s1 = make_1()
        s1.run(iters=steps, dt=dt)
        h1 = s1.bit_hash()
        del s1
        _free(dev)
    h1 = comm.broadcast_object(h1)
    return hn == h1, {"steps": steps, "hash_n": f"{hn & (2**64 - 1):016x}",
                      "hash_1": f"{h1 & (2**64 - 1):016x}"}


def halo_diag(s, reps=5, dt=None):
    """Exchange-only timing of the timed configuration (N > 1): ms per full exchange
    (all phases, stream-ordered, max over ranks) and the implied rate of the busiest
    link — the xGMI bandwidth this run actually saw."""
    import time as _t
    if s.comm.size == 1:
        return {}
    from multigpu_advectiondiffusion_amd.parallel.decomposition import halo_link_bytes
    s.sync_halos()
    s.halo.exchange(s.u)
    s._sync()
    s.comm.barrier()
    t0 = _t.perf_counter()
    for _ in range(reps):
        s.halo.exchange(s.u)
    s._sync()
    s.comm.barrier()
    ms = s.comm.allreduce_max((_t.perf_counter() - t0) / reps * 1e3)
    parts = 1
    if getattr(s.halo, "striped", False):
        parts = 1 + min(len(h) for h in s.halo._plan.values())
    link = halo_link_bytes(s.cd.shape, s.pgrid, s.ghost, s.u.element_size(),
                           corners=s.cart and s.fused,
                           direct=getattr(s.halo, "direct", True), stripe_parts=parts)
    # the same steps with the exchange switched off (ghosts go stale — run LAST, after
    # the validation): the compute-only step time; the timed ms/step minus this is the
    # part of the exchange the overlap did not hide
    dt = s.model.stable_dt() if dt is None else dt
    s.sync_halos()
    start = s.halo.start
    s.halo.start = lambda *a, **k: None
    try:  # eager: a cached hipGraph (ipc transport) would replay the exchange anyway
        s.run(iters=2, dt=dt, graph=False)
        nohalo = s.run(iters=reps, dt=dt, graph=False).compute_s / reps * 1e3
    finally:
        s.halo.start = start
    return {"halo_exchange_ms": round(ms, 4), "halo_link_MB": round(link / 1e6, 2),
            "halo_link_GBps": round(link / (ms * 1e-3) / 1e9, 1) if ms > 0 else None,
            "step_ms_without_exchange": round(nohalo, 4)}


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--base", type=int, default=512, help="diffusion cells per GPU = base^3")
    ap.add_argument("--burgers-base", type=int, default=256, help="Burgers cells per GPU = base^3")
    ap.add_argument("--burgers-steps", type=int, default=None)
    ap.add_argument("--no-burgers", action="store_true")
    ap.add_argument("--no-fd2", action="store_true")
    ap.add_argument("--burgers-ref-bound", type=float, default=BURGERS_REF_BOUND,
                    help="fail if the timed Burgers solution differs from the fp64 torch "
                         "reference ops by more than this (L_inf); <= 0 skips the check")
    ap.add_argument("--no-overlap", action="store_true")
    ap.add_argument("--decomp", default="tune",
                    help="process grid: 'tune' (default: the fastest of the candidate grids "
                         "measured over a few steps; the slab on 1 GPU), 'slab', 'auto' or "
                         "PZxPYxPX")
    ap.add_argument("--transport", default="tune",
                    help="halo transport for N > 1: 'tune' (default: every transport that "
                         "passes its preflight, the fastest measured), 'rccl', 'rccl-plain', "
                         "'ipc', 'ipc+stripe' or 'host'")
    ap.add_argument("--scaling", choices=["weak", "strong"], default="weak",
                    help="weak: base^3 cells per GPU (default); strong: the 8-GPU grid "
                         "(2*base)^3 on any N")
    ap.add_argument("--device", default=None)
    ap.add_argument("--settle-ms", type=float, default=300.0,
                    help="untimed steps after the W warm-up steps, in ms of stepping, so the "
                         "timed window sees the settled clock, not the power controller's "
                         "dip after the load starts (reported as 'settle'; 0 = off)")
    ap.add_argument("--sustained-steps", type=int, default=200,
                    help="extra steps timed after the headline window (informational "
                         "'sustained' fields; 0 = off)")
    ap.add_argument("--check-steps", type=int, default=10,
                    help="N > 1: steps of the bitwise N-rank vs 1-GPU check (0 = off)")
    ap.add_argument("--deadline", type=float, default=540.0,
                    help="seconds from the launcher's start (below the driver's 600 s): the "
                         "ranks dump their stacks 15 s before; at the deadline rank 0 prints "
                         "the JSON line with what finished and every rank exits 124")
    ap.add_argument("--preflight", choices=["on", "off"], default="on",
                    help="N > 1: run every (grid, transport) candidate for 2 steps in "
                         "hang-isolated child process groups first (parallel/preflight.py)")
    ap.add_argument("--preflight-cand-s", type=float, default=60.0,
                    help="preflight: seconds without progress after which a candidate is "
                         "taken to hang")
    ap.add_argument("--preflight-total-s", type=float, default=240.0)
    return ap.parse_args(argv)


def self_launch(args, deadline) -> int:
    """--gpus N > 1 without a launcher: start N ranks of this script ourselves (fresh
    subprocesses with the torchrun environment, before this process touches the GPU;
    never an exec) and return the first failing rank's exit code.  Rank 0 prints the
    JSON line.  The ranks keep their own deadline (this process is their launcher, so
    they count from its start); 20 s after it the ranks still alive get SIGUSR1 (stack
    dump) and are terminated."""
    import signal

    from multigpu_advectiondiffusion_amd.launch import launch_cmd
    cmd = [sys.executable, "-u", os.path.abspath(__file__)] + sys.argv[1:]
    rc = launch_cmd(args.gpus, cmd, timeout=max(deadline.remaining() + 20.0, 30.0),
                    dump_signal=signal.SIGUSR1)
    if rc != 0:
        print(f"bench: {args.gpus}-rank run failed (exit {rc})", file=sys.stderr, flush=True)
    return rc


def main(argv=None) -> int:
    from multigpu_advectiondiffusion_amd.utils.deadline import Deadline
    args = parse_args(argv)
    # a dead peer must end an ipc wait well before the driver's clock does
    os.environ.setdefault("ADVDIFF_IPC_TIMEOUT_S", "60")
    world = int(os.environ.get("WORLD_SIZE", "0") or 0)
    dl = Deadline(args.deadline)
    if world == 0 and args.gpus > 1:
        return self_launch(args, dl)
    if world and world != args.gpus:
        print(f"bench: --gpus {args.gpus} but WORLD_SIZE={world}: refusing to report a "
              f"{world}-rank run as {args.gpus} GPUs", file=sys.stderr, flush=True)
        return 2
    # the process group's own timeout must not fire before the deadline does (with nccl a
    # timed-out collective aborts the process: no JSON line)
    os.environ.setdefault("ADVDIFF_COMM_TIMEOUT", str(int(max(dl.remaining(), 0) + 120)))
    rank = int(os.environ.get("RANK", "0") or 0)
    dl.on_expire = (lambda d: report_partial(d)) if rank == 0 else None
    dl.heartbeat_s = 60.0 if rank == 0 else 0.0
    dl.arm()
    STATE["deadline"] = dl
    try:
        return run(args)
    finally:
        dl.cancel()


# ---- what a run has finished so far (printed by rank 0 if the deadline cuts it short) --
STATE = {"result": None, "deadline": None}


def report_partial(dl):
    res = dict(STATE["result"] or {"metric": METRIC, "value": None, "unit": "MLUPS"})
    res["status"] = (f"incomplete: the {dl.seconds:g} s bench deadline was reached in phase "
                     f"'{dl.phase}' (every rank's stack is in stderr)")
    print(json.dumps(res), flush=True)


def time_left() -> float:
    """Seconds until the bench deadline (inf without one)."""
    dl = STATE["deadline"]
    return float("inf") if dl is None else dl.remaining()


def skip_note(comm, what, need_s):
    """Optional phases (FD2, Burgers, the Burgers torch self-check) give way to the
    deadline: the headline line is worth more than a phase that cannot finish.  Ranks
    agree (max over ranks of the remaining time is not enough: the slowest decides)."""
    left = comm.allreduce_min(time_left()) if comm.size > 1 else time_left()
    if left >= need_s:
        return None
    note = f"skipped: {left:.0f} s left before the bench deadline, {what} needs ~{need_s:.0f} s"
    progress(comm, note)
    return note


def phase(comm, name):
    """Enter a bench phase: progress line, deadline bookkeeping, fault injection
    (ADVDIFF_FAULT=hang:phase:<prefix> makes the last rank sleep in the first phase whose
    name starts with <prefix>: tests)."""
    dl = STATE["deadline"]
    if dl is not None:
        dl.phase = name
    progress(comm, name)
    f = os.environ.get("ADVDIFF_FAULT", "")
    if (f.startswith("hang:phase:") and name.startswith(f[len("hang:phase:"):])
            and comm.rank == comm.size - 1):
        while True:
            time.sleep(3600)


def preflight_candidates(args, n, on_gpu, transports, heat_spec, burgers_spec):
    """Run every (model, grid, transport) candidate in child process groups (N > 1) and
    return ({mkey: [(pgrid, transport) that passed]}, record)."""
    from multigpu_advectiondiffusion_amd.parallel.decomposition import candidate_proc_grids
    grids = {}
    for mkey, spec, ghost, corners in heat_spec + burgers_spec:
        ashape = tuple(reversed(spec["shape"]))
        if args.decomp == "tune":
            grids[mkey] = candidate_proc_grids(n, ashape, ghost, 8, corners=corners)
        else:
            grids[mkey] = [None if args.decomp == "slab" else args.decomp]
    models = {mkey: spec for mkey, spec, _, _ in heat_spec + burgers_spec}

    def ok_for(m, p, t):  # striping and fused puts: slabs only; both: the heat step only
        slab = p in (None, "slab") or tuple(p)[1:] == (1, 1)
        if t == "ipc+fused+stripe":
            return slab and m == "heat"
        return t not in ("ipc+stripe", "ipc+fused") or slab
    allc = [(m, p, t) for m in models for p in grids[m] for t in transports
            if ok_for(m, p, t)]
    if n == 1 or args.preflight == "off":
        return {m: [(p, t) for mm, p, t in allc if mm == m] for m in models}, None
    verdict = {}
    dev = "cuda" if on_gpu else "cpu"
    for fam in ("gloo", "nccl"):  # ipc first: its pair preflight bounds itself
        # the newest transports last in their family: a family stops after two hangs, and
        # those then cost only the candidates behind them
        cs = sorted((c for c in allc if family(c[2]) == fam),
                    key=lambda c: {"ipc+stripe": 1, "ipc+fused": 2,
                                   "ipc+fused+stripe": 3}.get(c[2], 0))
        if not cs:
            continue
        dl = STATE["deadline"]
        budget = min(args.preflight_total_s, max(dl.remaining() - 200.0, 30.0)) if dl else \
            args.preflight_total_s
        t0 = time.perf_counter()
        verdict.update(run_preflight(cs, models, device=dev, backend=fam,
                                     cand_s=args.preflight_cand_s, total_s=budget,
                                     init_s=max(args.preflight_cand_s, 90.0),
                                     log=lambda m: print(m, file=sys.stderr, flush=True)))
        if int(os.environ.get("RANK", "0")) == 0:
            print(f"bench [{time.perf_counter() - _T0:7.1f} s] preflight ({fam}): "
                  f"{sum(v.startswith('ok') for v in verdict.values())} ok of {len(verdict)} "
                  f"in {time.perf_counter() - t0:.1f} s", file=sys.stderr, flush=True)
    passed = {m: [(p, t) for mm, p, t in allc
                  if mm == m and str(verdict.get(cand_key(m, p, t))).startswith("ok")]
              for m in models}
    return passed, verdict


def run(args) -> int:
    from multigpu_advectiondiffusion_amd import Burgers, Diffusion, Grid, Solver
    from multigpu_advectiondiffusion_amd.parallel import Comm, weak_scaling_grid

    n = args.gpus
    on_gpu = (args.device or ("cuda" if torch.cuda.device_count() > 0 else "cpu")).startswith("cuda")
    grid_of = ((lambda b: weak_scaling_grid(b, n)) if args.scaling == "weak"
               else (lambda b: weak_scaling_grid(b, 8)))
    shape = grid_of(args.base)
    bshape = grid_of(args.burgers_base)
    heat_kw = {"K": 1.0, "order": 4}
    burg_kw = {"viscosity": 1e-5, "weno": "z", "cfl": 0.3}
    heat_spec = [("heat", {"model": ("diffusion", heat_kw), "shape": list(shape),
                           "spacing": [1.0, 1.0, 1.0], "ic": "sine", "dtype": "float64"},
                  3 * 2, True)]
    burgers_spec = [] if args.no_burgers else [
        ("burgers", {"model": ("burgers", burg_kw), "shape": list(bshape),
                     "spacing": [2.0, 2.0, 2.0], "ic": "gaussian", "dtype": "float64"}, 3, False)]

    # ---- N > 1: exercise every candidate in hang-isolated child process groups first ----
    transports = planned_transports(n, on_gpu, args.transport)
    passed, pf = preflight_candidates(args, n, on_gpu, transports, heat_spec, burgers_spec)
    backend = None
    if n > 1 and on_gpu and pf is not None:
        ok_t = {t for c in passed.values() for _, t in c}
        if (any(family(t) == "nccl" for t in transports)
                and not any(family(t) == "nccl" for t in ok_t)):
            backend = "gloo"  # RCCL failed everywhere: gloo control plane + ipc puts
    if n > 1 and not passed.get("heat"):
        # nothing passed: last resort, the unexercised host-staged exchange (gloo)
        if on_gpu:
            backend = "gloo"
        passed = {m: [(None, "host")] for m in passed}

    comm = Comm.from_env(device=args.device, backend=backend)
    if comm.size != n:
        raise SystemExit(f"bench: world {comm.size} != --gpus {n}")
    dev = comm.device
    single = Comm(device=str(dev)) if dev.type == "cuda" else Comm(device="cpu")
    phase(comm, f"{n} rank(s) on {comm.device_ids()}, backend {comm.backend}")
    names, ipc_pre = ipc_pair_check(comm, sorted({t for c in passed.values() for _, t in c
                                                  if t is not None}))
    passed = {m: [(p, t) for p, t in c if t is None or t in names] for m, c in passed.items()}

    # ---- headline: 3-D heat, FD4, fp64, sine IC -------------------------------------
    grid = Grid(shape, (1.0, 1.0, 1.0))
    model = Diffusion(**heat_kw)
    model.bind(grid)
    dt = model.stable_dt()

    def make_heat(p, t, m=model, c=comm):
        return Solver(m, grid, c, dtype=torch.float64, ic="sine",
                      overlap=not args.no_overlap, decomp=p, **solver_transport(t))

    result = {"metric": METRIC, "value": None, "unit": "MLUPS", "n_gpus": n,
              "steps": args.steps, "warmup": args.warmup, "higher_is_better": True,
              "scaling": args.scaling, "dtype": "fp64",
              "data": "synthetic (sinusoidal IC sin(pi x)sin(pi y)sin(pi z), random-free "
                      "analytic init)",
              "config": {"model": "diffusion3d FD4 13-point + SSP-RK3", "global_batch": 1,
                         "seq_len": grid.cells, "grid": list(shape),
                         "cells_per_gpu": grid.cells // n}}
    if pf is not None:
        result["preflight"] = pf
    STATE["result"] = result
    phase(comm, f"heat: tuning {len(passed['heat'])} (grid, transport) candidates")
    (decomp, transport), trials = tune(make_heat, passed["heat"], dt, dev)
    phase(comm, f"heat: timed run ({decomp}, {transport})")
    solver = make_heat(decomp, transport)
    secs = timed(solver, args.steps, args.warmup, dt, args.settle_ms, "heat")
    mlups = grid.cells * args.steps / secs / 1e6
    pg = solver.pgrid
    link = {"ipc": "ipc device puts", "ipc+fused": "ipc puts inside the step launches",
            "ipc+fused+stripe": "ipc puts inside the step launches, striped over idle links",
            "rccl": "RCCL, boundary launch on the comm stream",
            "host": "host-staged", "rccl-plain": "RCCL, boundary launch after the interior",
            "ipc+stripe": "ipc device puts striped over idle links"}.get(transport, transport)
    result.update({
        "value": round(mlups, 1), "settle": SETTLE.get("heat"),
        "ms_per_step": round(secs / args.steps * 1e3, 4),
        "vs_baseline": round(mlups / BASE_DIFFUSION, 2)})
    result["config"]["parallelism"] = (
        "single GPU" if n == 1 else
        f"z-slab{n} ({link} halo, overlapped)" if pg[1:] == (1, 1) else
        f"cartesian {'x'.join(map(str, pg))} (z,y,x; {link} halo)")
    result["status"] = "running"
    phase(comm, "heat: sustained window and validation")
    sust = sustained(solver, args.sustained_steps, dt, grid.cells)
    # self-validation against the exact solution (outside the timed region)
    finite = solver.check_finite()
    _, _, linf = solver.error_norms()
    t_end = solver.t
    diag = halo_diag(solver, dt=dt)
    del solver
    _free(dev)
    bound = linf_bound(grid, model.K, t_end, 4)
    result.update({
        "max_abs_u": finite, **({"sustained": sust} if sust else {}),
        "linf_vs_exact": float(f"{linf:.3e}"), "linf_bound": float(f"{bound:.3e}"),
        "t_end": t_end, "halo_transport": transport if n > 1 else None,
        "rccl_world": comm.rccl_world, "transport_trials_ms_per_step": trials,
        **({"ipc_preflight": ipc_pre} if ipc_pre is not None else {}), **diag,
        "comm_backend": comm.backend or "none (single process)",
        "device_ids": comm.device_ids()})
    if not linf <= bound:
        return fail(comm, result, f"bench validation failed: L_inf vs exact = {linf:.3e} > "
                                  f"{bound:.3e}")
    if n > 1:
        result["bitwise_vs_1gpu"] = {}
    if n > 1 and args.check_steps > 0:
        phase(comm, "heat: bitwise check against one GPU")
        ok, rec = bitwise_vs_1gpu(lambda: make_heat(decomp, transport),
                                  lambda: make_heat(None, None, c=single),
                                  args.check_steps, dt, comm, dev)
        result["bitwise_vs_1gpu"]["heat"] = ok
        result["bitwise_check"] = rec
        if not ok:
            return fail(comm, result, f"bench validation failed: {n}-rank heat solution "
                                      f"differs from the 1-GPU solution ({rec})")

    # ---- the 7-point (FD2) Laplacian named by BASELINE.json, same grid ----------------
    if not args.no_fd2 and (note := skip_note(comm, "the FD2 run", 120.0)):
        result["fd2_7pt"] = {"skipped": note}
    elif not args.no_fd2:
        phase(comm, "fd2: FD2 7-point run")
        m2 = Diffusion(K=1.0, order=2)
        s2 = make_heat(decomp, transport, m=m2)
        secs2 = timed(s2, args.steps, args.warmup, m2.stable_dt(), args.settle_ms, "fd2")
        per_launch = 2 if s2.step2_capable() else 1
        _, _, linf2 = s2.error_norms()
        bound2 = linf_bound(grid, m2.K, s2.t, 2)
        del s2
        _free(dev)
        ml2 = grid.cells * args.steps / secs2 / 1e6
        result["fd2_7pt"] = {"value": round(ml2, 1), "unit": "MLUPS",
                             "ms_per_step": round(secs2 / args.steps * 1e3, 4),
                             "vs_baseline": round(ml2 / BASE_DIFFUSION, 2),
                             "linf_vs_exact": float(f"{linf2:.3e}"),
                             "settle": SETTLE.get("fd2"),
                             "steps_per_launch": per_launch,
                             "model": "diffusion3d FD2 7-point + SSP-RK3"}
        if not linf2 <= bound2:
            return fail(comm, result, f"bench validation failed: FD2 L_inf vs exact = "
                                      f"{linf2:.3e} > {bound2:.3e}")

    # ---- secondary: 3-D Burgers WENO5-Z + C∇²u, fp64 ----------------------------------
    if not args.no_burgers and not passed.get("burgers"):
        result["burgers3d"] = {"skipped": "no (grid, transport) candidate passed the preflight"}
    elif not args.no_burgers and (note := skip_note(comm, "the Burgers run", 150.0)):
        result["burgers3d"] = {"skipped": note}
    elif not args.no_burgers:
        bgrid = Grid(bshape, (2.0, 2.0, 2.0))
        bmodel = Burgers(**burg_kw)
        bmodel.bind(bgrid)
        bdt = bmodel.stable_dt()

        def make_burgers(p, t, c=comm):
            return Solver(bmodel, bgrid, c, dtype=torch.float64, ic="gaussian",
                          overlap=not args.no_overlap, decomp=p, **solver_transport(t))
        phase(comm, f"burgers: tuning {len(passed['burgers'])} candidates")
        (bdecomp, btransport), btrials = tune(make_burgers, passed["burgers"], bdt, dev)
        phase(comm, f"burgers: timed run ({bdecomp}, {btransport})")
        bsolver = make_burgers(bdecomp, btransport)
        bsteps = args.burgers_steps or args.steps
        bsecs = timed(bsolver, bsteps, args.warmup, bdt, args.settle_ms, "burgers")
        bml = bgrid.cells * bsteps / bsecs / 1e6
        brec = result["burgers3d"] = {
            "value": round(bml, 1), "unit": "MLUPS", "grid": list(bshape), "steps": bsteps,
            "ms_per_step": round(bsecs / bsteps * 1e3, 4), "settle": SETTLE.get("burgers"),
            "vs_baseline": round(bml / BASE_BURGERS, 2),
            "model": "burgers3d WENO5-Z + FD4 viscous (C=1e-5) + SSP-RK3",
            "pgrid": list(bsolver.pgrid), "halo_transport": btransport if n > 1 else None,
            "transport_trials_ms_per_step": btrials}
        bsust = sustained(bsolver, args.sustained_steps, bdt, bgrid.cells)
        if bsust:
            brec["sustained"] = bsust
        bsolver.check_finite()
        # the torch ops take ~5 ns per cell and step on one MI355X (699 steps of 256^3:
        # 57.5 s, profiles/r6/bench_pruned.log); x2 margin + the bitwise check after it
        est = 2 * 5e-9 * bsolver.it * bgrid.cells / n + 60.0
        rnote = skip_note(comm, "the Burgers torch self-check", est) \
            if args.burgers_ref_bound > 0 else None
        if rnote:
            brec["reference_check"] = {"skipped": rnote}
        elif args.burgers_ref_bound > 0:
            # self-check (outside the timed region): every step the timed solver took,
            # again through the fp64 PyTorch reference ops on the same decomposition
            phase(comm, f"burgers: {bsolver.it} reference steps (torch ops)")
            ref = Solver(bmodel, bgrid, comm, dtype=torch.float64, ic="gaussian",
                         overlap=not args.no_overlap, decomp=bdecomp, kernel="torch",
                         **solver_transport(btransport))
            t_ref = time.perf_counter()
            ref.run(iters=bsolver.it, dt=bdt, graph=False)
            ref.sync_halos()
            _, _, blinf = bsolver.error_norms(exact=ref.u)
            bref = {"linf_vs_torch": float(f"{blinf:.3e}"), "bound": args.burgers_ref_bound,
                    "steps": bsolver.it, "t": bsolver.t,
                    "torch_s": round(time.perf_counter() - t_ref, 1)}
            del ref
            brec["linf_vs_torch"] = bref["linf_vs_torch"]
            brec["reference_check"] = bref
        del bsolver
        _free(dev)
        if "linf_vs_torch" in brec and not brec["linf_vs_torch"] <= args.burgers_ref_bound:
            return fail(comm, result, f"bench validation failed: Burgers L_inf vs the torch "
                                      f"reference = {brec['linf_vs_torch']:.3e} > "
                                      f"{args.burgers_ref_bound:.1e}")
        if n > 1 and args.check_steps > 0:
            phase(comm, "burgers: bitwise check against one GPU")
            ok, rec = bitwise_vs_1gpu(lambda: make_burgers(bdecomp, btransport),
                                      lambda: make_burgers(None, None, c=single),
                                      args.check_steps, bdt, comm, dev)
            brec["bitwise_check"] = rec
            result["bitwise_vs_1gpu"]["burgers3d"] = ok
            if not ok:
                return fail(comm, result, f"bench validation failed: {n}-rank Burgers "
                                          f"solution differs from the 1-GPU solution ({rec})")

    result["status"] = "ok"
    if STATE["deadline"] is not None:
        STATE["deadline"].cancel()
    if comm.rank == 0:
        print(json.dumps(result), flush=True)
    comm.finalize()
    return 0


def fail(comm, result, msg) -> int:
    """A validation failure: no result line (the numbers are not valid), the reason on
    stderr, exit 1 on every rank."""
    STATE["result"] = None
    if STATE["deadline"] is not None:
        STATE["deadline"].cancel()
    if comm.rank == 0:
        print(msg, file=sys.stderr, flush=True)
    comm.finalize()
    return 1


if __name__ == "__main__":
    sys.exit(main())
