#!/usr/bin/env python3
"""Headline benchmark (BASELINE.json): whole-node MLUPS of the fp64 3-D heat solver
(FD4 13-point + SSP-RK3, synthetic sinusoidal IC) with per-GPU work fixed at 512³ cells
(weak scaling: 1 GPU -> 512³, 8 GPUs -> 1024³), plus the 3-D WENO5-Z viscous Burgers
solver at 256³ per GPU reported alongside.

    python bench.py --gpus N --steps K --warmup W
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

One RK3 step = 3 fused stage kernels + 3 halo exchanges (no work skipped).  K steps are
timed between a barrier + device sync on both sides; the max over ranks is reported.
MLUPS = global cells x K / seconds / 1e6.  Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from multigpu_advectiondiffusion_amd import Burgers, Diffusion, Grid, Solver  # noqa: E402
from multigpu_advectiondiffusion_amd.parallel import Comm, weak_scaling_grid  # noqa: E402

METRIC = "MLUPS (whole node), 3D diffusion 512^3 + Burgers3D WENO5, 1/2/4/8 MI355X"
BASE_DIFFUSION = 927.2   # best published 3-D heat MLUPS (SingleGPU/Diffusion3d_Blocking/Run.m:3-12)
BASE_BURGERS = 344.4     # best published 3-D Burgers MLUPS (SingleGPU/Burgers3d_WENO5_PitchedMem/Run.m:15-25)


def timed(solver: Solver, steps: int, warmup: int, dt: float) -> float:
    if warmup:
        solver.run(iters=warmup, dt=dt)
    st = solver.run(iters=steps, dt=dt)  # barrier + sync on both sides, max over ranks
    return st.compute_s


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--base", type=int, default=512, help="diffusion cells per GPU = base^3")
    ap.add_argument("--burgers-base", type=int, default=256, help="Burgers cells per GPU = base^3")
    ap.add_argument("--burgers-steps", type=int, default=None)
    ap.add_argument("--no-burgers", action="store_true")
    ap.add_argument("--no-overlap", action="store_true")
    ap.add_argument("--decomp", default=None, help="process grid (default: z-slabs)")
    ap.add_argument("--scaling", choices=["weak", "strong"], default="weak",
                    help="weak: base^3 cells per GPU (default); strong: the 8-GPU grid "
                         "(2*base)^3 on any N")
    ap.add_argument("--device", default=None)
    args = ap.parse_args()

    comm = Comm.from_env(device=args.device)
    n = comm.size
    if args.gpus != n and comm.rank == 0:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={n}; using {n}", file=sys.stderr)
    dev = comm.device

    # ---- headline: 3-D heat, FD4, fp64, sine IC -------------------------------------
    grid_of = ((lambda b: weak_scaling_grid(b, n)) if args.scaling == "weak"
               else (lambda b: weak_scaling_grid(b, 8)))
    shape = grid_of(args.base)
    grid = Grid(shape, (1.0, 1.0, 1.0))
    model = Diffusion(K=1.0, order=4)
    solver = Solver(model, grid, comm, dtype=torch.float64, ic="sine",
                    overlap=not args.no_overlap, decomp=args.decomp)
    dt = model.stable_dt()
    secs = timed(solver, args.steps, args.warmup, dt)
    mlups = grid.cells * args.steps / secs / 1e6
    # sanity: the solution must stay finite and decay (sine mode)
    finite = solver.check_finite()
    pg = solver.pgrid
    del solver
    if dev.type == "cuda":
        torch.cuda.empty_cache()

    result = {
        "metric": METRIC,
        "value": round(mlups, 1),
        "unit": "MLUPS",
        "n_gpus": n,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(secs / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": args.scaling,
        "vs_baseline": round(mlups / BASE_DIFFUSION, 2),
        "dtype": "fp64",
        "data": "synthetic (sinusoidal IC sin(pi x)sin(pi y)sin(pi z), random-free analytic init)",
        "config": {"model": "diffusion3d FD4 13-point + SSP-RK3", "global_batch": 1,
                   "seq_len": grid.cells, "grid": list(shape),
                   "parallelism": ("single GPU" if n == 1 else
                                   f"z-slab{n} (RCCL halo, overlapped)" if pg[1:] == (1, 1) else
                                   f"cartesian {'x'.join(map(str, pg))} (z,y,x; RCCL halo)"),
                   "cells_per_gpu": grid.cells // n},
        "max_abs_u": finite,
    }

    # ---- secondary: 3-D Burgers WENO5-Z + C∇²u, fp64 ----------------------------------
    if not args.no_burgers:
        bshape = grid_of(args.burgers_base)
        bgrid = Grid(bshape, (2.0, 2.0, 2.0))
        bmodel = Burgers(viscosity=1e-5, weno="z", cfl=0.3)
        bsolver = Solver(bmodel, bgrid, comm, dtype=torch.float64, ic="gaussian",
                         overlap=not args.no_overlap, decomp=args.decomp)
        bsteps = args.burgers_steps or args.steps
        bsecs = timed(bsolver, bsteps, args.warmup, bmodel.stable_dt())
        bml = bgrid.cells * bsteps / bsecs / 1e6
        bsolver.check_finite()
        result["burgers3d"] = {"value": round(bml, 1), "unit": "MLUPS", "grid": list(bshape),
                               "steps": bsteps, "ms_per_step": round(bsecs / bsteps * 1e3, 4),
                               "vs_baseline": round(bml / BASE_BURGERS, 2),
                               "model": "burgers3d WENO5-Z + FD4 viscous (C=1e-5) + SSP-RK3"}
        del bsolver

    if comm.rank == 0:
        print(json.dumps(result), flush=True)
    comm.finalize()


if __name__ == "__main__":
    main()
