#!/usr/bin/env python3
"""Pitched allocation in the solver (Solver(pitch=(px, py)): rows of align256(nx) + px
elements, planes of ny + py rows): the bench's three cases — heat FD4 / FD2 at 512^3 and
Burgers WENO5-Z at 256^3 — plus Burgers 512^3, every candidate pitch built side by side
and timed in interleaved rounds of hipGraph-replayed steps after a settling run; the
solutions must agree bitwise (bit_hash).  One JSON line per (case, pitch).

    python bench/pitch_solver_ab.py [--pitches 0,0 8,0 8,1] [--cases fd4 fd2 b256 b512]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multigpu_advectiondiffusion_amd import Burgers, Diffusion, Grid, Solver  # noqa: E402


def make(case, pitch):
    if case in ("fd4", "fd2"):
        m = Diffusion(K=1.0, order=4 if case == "fd4" else 2)
        return Solver(m, Grid((512,) * 3, (1.0,) * 3), dtype=torch.float64, ic="sine",
                      pitch=pitch), m.stable_dt()
    n = 256 if case == "b256" else 512
    s = Solver(Burgers(viscosity=1e-5, weno="z", cfl=0.3), Grid((n,) * 3, (2.0,) * 3),
               dtype=torch.float64, ic="gaussian", pitch=pitch)
    return s, s.dt()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pitches", nargs="+", default=["0,0", "8,0", "8,1", "4,1", "32,1"])
    ap.add_argument("--cases", nargs="+", default=["fd4", "fd2", "b256", "b512"])
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--target-ms", type=float, default=40.0)
    a = ap.parse_args()
    pitches = [tuple(int(v) for v in p.split(",")) for p in a.pitches]
    for case in a.cases:
        solvers = {}
        for p in pitches:
            s, dt = make(case, p)
            s.run(iters=8, dt=dt)
            solvers[p] = s
        s0 = solvers[pitches[0]]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        s0.run(iters=16, dt=dt)
        per = (time.perf_counter() - t0) / 16
        steps = max(16, int(a.target_ms * 1e-3 / per) // 8 * 8)
        for s in solvers.values():  # settle at the measured load
            s.run(iters=steps, dt=dt)
        best = {p: float("inf") for p in pitches}
        for _ in range(a.rounds):
            for p, s in solvers.items():
                st = s.run(iters=steps, dt=dt)
                best[p] = min(best[p], st.compute_s / st.steps * 1e3)
        # same step count everywhere: the solutions must agree bitwise
        its = {p: s.it for p, s in solvers.items()}
        top = max(its.values())
        for p, s in solvers.items():
            if s.it < top:
                s.run(iters=top - s.it, dt=dt)
        hashes = {p: s.bit_hash() for p, s in solvers.items()}
        cells = s0.grid.cells
        for p in pitches:
            s = solvers[p]
            print(json.dumps({"case": case, "pitch": list(p), "row_pitch": s.sx,
                              "rows_per_plane": s.u.shape[1], "steps": steps,
                              "ms_per_step": round(best[p], 4),
                              "mlups": round(cells / (best[p] * 1e3), 1),
                              "vs_first": round(best[pitches[0]] / best[p], 4),
                              "bitwise_equal": hashes[p] == hashes[pitches[0]]}), flush=True)
        del solvers, s0, s
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
