"""Command-line front end with the reference's positional argument layouts.

Reference CLIs:

    diffusion2d  C|K L W Nx Ny iters [bx by]            (SingleGPU/Diffusion2d/main.cpp:32-47,
                                                         MultiGPU/Diffusion2d_Baseline/main.c:36-51)
    diffusion3d  C|K L W H Nx Ny Nz iters [bx by bz]    (SingleGPU/Diffusion3d_*/main.cpp:32-50,
                                                         MultiGPU/Diffusion3d_Baseline/main.c:36-54)
    burgers2d    tEnd CFL L W Nx Ny [bx by]             (MultiGPU/Burgers2d_Baseline/main.c:36-51)
    burgers3d    tEnd CFL L W H Nx Ny Nz [bx by bz]     (SingleGPU/Burgers3d_WENO5/main.cpp:32-50,
                                                         MultiGPU/Burgers3d_Baseline/main.c:36-54)

Block sizes are accepted for compatibility and ignored (the gfx950 tiles are fixed:
64-wide wave rows).  Everything the reference hard-codes at compile time is a runtime
flag here: --ic, --order, --weno, --viscosity, --dtype, --overlap,
--write, --checkpoint/--restart, --config (JSON/TOML/YAML file of the same keys).

Multi-GPU: run under torchrun (one process per GPU), e.g.
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \
        -m multigpu_advectiondiffusion_amd diffusion3d 1 2 2 2 1024 1024 1024 100
or with the bundled launcher:  python -m multigpu_advectiondiffusion_amd.launch -np 8 diffusion3d ...
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

APPS = {
    "diffusion2d": ["K", "L", "W", "Nx", "Ny", "iters"],
    "diffusion3d": ["K", "L", "W", "H", "Nx", "Ny", "Nz", "iters"],
    "burgers2d": ["tEnd", "CFL", "L", "W", "Nx", "Ny"],
    "burgers3d": ["tEnd", "CFL", "L", "W", "H", "Nx", "Ny", "Nz"],
}
_INT = {"Nx", "Ny", "Nz", "iters"}


def _load_config(path):
    p = Path(path)
    text = p.read_text()
    if p.suffix in (".toml",):
        try:
            import tomllib
        except ImportError:  # py3.10
            import tomli as tomllib
        return tomllib.loads(text)
    if p.suffix in (".yaml", ".yml"):
        import yaml
        return yaml.safe_load(text)
    return json.loads(text)


def build_parser():
    ap = argparse.ArgumentParser(prog="multigpu_advectiondiffusion_amd",
                                 description="MI355X-native advection-diffusion stencil solvers")
    ap.add_argument("app", choices=sorted(APPS))
    ap.add_argument("args", nargs="*", help="reference positional arguments (see module doc)")
    ap.add_argument("--config", help="JSON/TOML/YAML file with any of the named options")
    ap.add_argument("--ic", help="initial condition: zero|square|sine|heat|gaussian|plates|disc")
    ap.add_argument("--order", type=int, default=4, help="diffusion FD order: 4 (13-pt) or 2 (7-pt)")
    ap.add_argument("--safety", type=float, default=0.9, help="diffusion dt safety factor (MG used 0.8)")
    ap.add_argument("--weno", choices=["js", "z", "js7"], default="z",
                    help="WENO5-JS, WENO5-Z (default) or WENO7-JS")
    ap.add_argument("--integrator", choices=["ssprk3", "lsrk45"], default="ssprk3",
                    help="SSP-RK3 (reference apps) or low-storage RK4(5) (MATLAB WENO7)")
    ap.add_argument("--viscosity", type=float, default=1e-5, help="Burgers C (0 = inviscid)")
    ap.add_argument("--cfl-mode", choices=["fixed", "adaptive"], default="fixed")
    ap.add_argument("--dtype", choices=["fp64", "fp32"], default="fp64")
    ap.add_argument("--device", choices=["cuda", "cpu"], default=None)
    ap.add_argument("--no-overlap", action="store_true", help="disable halo/compute overlap")
    ap.add_argument("--kernel", choices=["native", "torch"], default="native",
                    help="stencil implementation: gfx950 HIP kernels or the PyTorch reference ops")
    ap.add_argument("--exchange", choices=["u", "lu"], default="u",
                    help="halo payload: u (stage output) or lu (the reference's RHS exchange "
                         "with redundant ghost-plane updates; slab, PyTorch ops)")
    ap.add_argument("--boundary-on-comm", dest="bcomm", action="store_true", default=None,
                    help="overlap: boundary launch on the comm stream between the halo wait "
                         "and the puts (default on for --transport rccl and ipc; ADVDIFF_BCOMM)")
    ap.add_argument("--no-boundary-on-comm", dest="bcomm", action="store_false")
    ap.add_argument("--pitch", default=None, metavar="PX,PY",
                    help="pitched device fields: PX extra elements per row, PY extra rows "
                         "per 3-D plane (default ADVDIFF_PITCH, else 4 fp64 / 16 fp32 "
                         "elements + 1 row on 3-D fields past 128 MiB per rank; 0,0 = the "
                         "256-B row pitch only)")
    ap.add_argument("--stripe", type=int, default=None,
                    help="ipc slab halos: relay part of every face message through up to N "
                         "helper ranks over idle xGMI links (default: ADVDIFF_STRIPE or 0)")
    ap.add_argument("--fused-put", action="store_true", default=None,
                    help="ipc slab halos of the fused 3-D heat step: the step launch stores "
                         "its boundary planes into the neighbours' ghost planes itself "
                         "(default: ADVDIFF_FUSED_PUT)")
    ap.add_argument("--decomp", default=None,
                    help="process grid: slab (default), auto, or PZxPYxPX / PYxPX")
    ap.add_argument("--transport", choices=["rccl", "ipc", "host"], default=None,
                    help="halo transport: rccl (nccl backend), ipc (peer-mapped device puts "
                         "+ device flags) or host (gloo, host-staged)")
    ap.add_argument("--write", default=None, help="write float32 result.bin to this path")
    ap.add_argument("--write-ghosts", default=None,
                    help="write the multi-GPU result.bin layout: every rank's slab WITH its "
                         "ghost planes, rank after rank (MultiGPU/Diffusion3d_Baseline/main.c:341)")
    ap.add_argument("--initial", default=None, help="write float32 initial.bin to this path")
    ap.add_argument("--ascii", default=None, help="write the result as ASCII (one %%g per line)")
    ap.add_argument("--print", dest="print_field", action="store_true",
                    help="print the final field (small grids; the reference's Print3D)")
    ap.add_argument("--checkpoint", default=None, help="write fp64 checkpoint shards to PREFIX")
    ap.add_argument("--restart", default=None, help="restart from checkpoint PREFIX")
    ap.add_argument("--style", choices=["multigpu", "singlegpu"], default="multigpu",
                    help="summary block layout / GFLOPs formula of the reference")
    ap.add_argument("--error-norms", action="store_true",
                    help="print L1/L2/Linf vs the exact solution (sine/heat ICs)")
    ap.add_argument("--check-every", type=int, default=0, help="NaN/Inf watchdog period (steps)")
    ap.add_argument("--json", action="store_true", help="also print one JSON metrics line")
    ap.add_argument("--warmup", type=int, default=0, help="untimed warm-up steps")
    g = ap.add_mutually_exclusive_group()
    g.add_argument("--graph", dest="graph", action="store_const", const=True, default=None,
                   help="replay hipGraphs of the steps (default: wherever they are safe)")
    g.add_argument("--no-graph", dest="graph", action="store_const", const=False,
                   help="launch every step eagerly (the native apps' --no-graph)")
    ap.add_argument("--geometry", action="store_true",
                    help="print this rank's decomposition (owned box, halo messages) as "
                         "JSON and exit, like the native apps' --geometry")
    return ap


def parse(argv=None):
    ap = build_parser()
    ns = ap.parse_args(argv)
    if ns.config:
        cfg = _load_config(ns.config)
        for k, v in cfg.items():
            k2 = k.replace("-", "_")
            if k2 == "args":
                ns.args = [str(x) for x in v]
            elif hasattr(ns, k2):
                setattr(ns, k2, v)
            else:
                ap.error(f"unknown config key {k!r}")
    names = APPS[ns.app]
    if len(ns.args) < len(names):
        ap.error(f"{ns.app} needs positional args: {' '.join(names)} [block sizes]")
    pos = {}
    for n, v in zip(names, ns.args):
        pos[n] = int(v) if n in _INT else float(v)
    ns.pos = pos
    ns.blocks = ns.args[len(names):]
    return ns


def make_problem(ns):
    """Return (model, grid, ic, run_kwargs) from parsed args."""
    from .models import Burgers, Diffusion, Grid
    p = ns.pos
    if ns.app.startswith("diffusion"):
        model = Diffusion(K=p["K"], order=ns.order, safety=ns.safety)
        if ns.app == "diffusion3d":
            grid = Grid((p["Nx"], p["Ny"], p["Nz"]), (p["L"], p["W"], p["H"]))
        else:
            grid = Grid((p["Nx"], p["Ny"]), (p["L"], p["W"]))
        ic = ns.ic or "heat"
        run = {"iters": p["iters"]}
    else:
        model = Burgers(viscosity=ns.viscosity, weno=ns.weno, cfl=p["CFL"], cfl_mode=ns.cfl_mode)
        if ns.app == "burgers3d":
            grid = Grid((p["Nx"], p["Ny"], p["Nz"]), (p["L"], p["W"], p["H"]))
        else:
            grid = Grid((p["Nx"], p["Ny"]), (p["L"], p["W"]))
        ic = ns.ic or "gaussian"
        run = {"t_end": p["tEnd"]}
    return model, grid, ic, run


def main(argv=None) -> int:
    import torch

    from .parallel.comm import Comm
    from .solver import Solver
    from .utils import metrics

    ns = parse(argv)
    model, grid, ic, run = make_problem(ns)
    import os
    import time
    comm = Comm.from_env(device=ns.device or os.environ.get("ADVDIFF_DEVICE"),
                         transport=ns.transport)
    dtype = torch.float64 if ns.dtype == "fp64" else torch.float32
    t0 = 0.1 if (ic == "heat") else 0.0  # heat kernel IC is the exact solution at t0

    def fenced(fn):
        """fn() timed between barriers + device syncs, max over ranks (the reference's
        MPI_Barrier-fenced HtD / DtH timers, MultiGPU/Diffusion3d_Baseline/main.c:137-148,
        313-323)."""
        sync = (lambda: torch.cuda.synchronize(comm.device)) if comm.device.type == "cuda" \
            else (lambda: None)
        sync()
        comm.barrier()
        t = time.perf_counter()
        out = fn()
        sync()
        comm.barrier()
        return out, comm.allreduce_max(time.perf_counter() - t)

    # HtD: building the device fields — the IC is generated on the device (no host array
    # is copied), so this line times the allocation + IC kernels + stage-buffer copies
    solver, htod_s = fenced(lambda: Solver(
        model, grid, comm, dtype=dtype, ic=ic, overlap=not ns.no_overlap, t0=t0,
        check_every=ns.check_every, decomp=ns.decomp, integrator=ns.integrator,
        kernel=ns.kernel, exchange=ns.exchange, stripe=ns.stripe, boundary_on_comm=ns.bcomm,
        pitch=None if ns.pitch is None else tuple(int(v) for v in ns.pitch.split(",")),
        fused_put=ns.fused_put))
    # the shape-dependent launch picks (GPU measurements) after the fenced HtD, as the
    # native engine does after init_s_
    solver.tune_launches()
    if ns.geometry:  # decomposition only (no steps), one JSON line per rank in rank order
        geo = {"rank": comm.rank, "world": comm.size, "pgrid": list(solver.pgrid),
               "global_box": [list(b) for b in solver.cd.global_box()],
               "owned_box": [list(b) for b in solver.cd.owned_box()],
               "ghost": solver.cd.ghost, "row_pitch": solver.sx,
               "rows_per_plane": int(solver.u.shape[-2]) if solver.u.dim() == 3 else None}
        if solver.cart:
            geo["halo_phases"] = [
                [{"peer": p, "send": [list(b) for b in sb], "recv": [list(b) for b in rb],
                  "offset": list(off)} for p, sb, rb, off in solver.halo.boxes(axes)]
                for axes in solver.halo._phases()]
        allg = [geo]
        if comm.size > 1:
            import torch.distributed as dist
            allg = [None] * comm.size
            dist.all_gather_object(allg, geo)
        if comm.rank == 0:
            for g in allg:
                print(json.dumps(g), flush=True)
        comm.finalize()
        return 0
    if ns.restart:
        solver.load_checkpoint(ns.restart)
    if ns.initial:
        solver.save_result(ns.initial)
    if ns.warmup:
        wt, wi = solver.t, solver.it
        saved = [f.clone() for f in solver.fields()]
        solver.run(iters=ns.warmup, graph=ns.graph)
        for f, s in zip(solver.fields(), saved):
            f.copy_(s)
        solver.t, solver.it = wt, wi
    if "t_end" in run:
        run = {"t_end": run["t_end"] + (t0 if ic == "heat" else 0.0)}
    stats = solver.run(**run, graph=ns.graph)
    extra = {}
    if ns.error_norms and ic in ("sine", "heat"):
        l1, l2, li = solver.error_norms()
        extra = {"L1 norm": f"{l1:e}", "L2 norm": f"{l2:e}", "Linf norm": f"{li:e}"}
    # DtH: the final field to the host and — when an output needs the global field — its
    # gather on rank 0 (the reference's timed DtH + Merge_domains).  Without one, each rank
    # times the copy of its own block only (no full-field copy on rank 0's host)
    if ns.write or ns.ascii or ns.print_field:
        g, dtoh_s = fenced(solver.gather)
    else:
        g, dtoh_s = fenced(solver.copy_to_host)
    stats.htod_s, stats.dtoh_s = htod_s, dtoh_s
    text = solver.summary(stats, style=ns.style, extra=extra)
    from .utils import io as aio
    if comm.rank == 0:
        if ns.write:
            aio.save_binary(ns.write, g)
        if ns.ascii:
            aio.save_ascii(ns.ascii, g)
        if ns.print_field:
            print(aio.format_field(g))
    if ns.write_ghosts:
        gg = solver.gather_with_ghosts()
        if comm.rank == 0:
            aio.save_binary(ns.write_ghosts, gg)
    if ns.checkpoint:
        solver.save_checkpoint(ns.checkpoint)
    if comm.rank == 0:
        if ns.blocks:
            print(f"(block sizes {' '.join(ns.blocks)} ignored: gfx950 tiles are fixed)")
        print(text)
        if ns.json:
            print(json.dumps({
                "app": ns.app, "grid": list(grid.shape), "steps": stats.steps,
                "seconds": stats.compute_s,
                "mlups": metrics.mlups(stats.compute_s, stats.steps, grid.cells),
                "n_procs": comm.size, "dtype": ns.dtype, "t": stats.t,
                "device_field_bytes": solver.memory_bytes(), "row_pitch": solver.sx}))
    sys.stdout.flush()
    comm.finalize()
    return 0
