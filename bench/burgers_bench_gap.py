#!/usr/bin/env python3
"""Why the bench's Burgers window (0.578-0.582 ms/step at 256^3) sits ~6 % above
bench/burgers3d_rate.py (0.542-0.545 ms): the same solver built the two ways — the rate
tool's (default comm) and the bench's (Comm.from_env, overlap=True, decomp=None) — timed
in one process in interleaved rounds, cold, and again after a heat-FD4 load of the
bench's length (thermal / power state).

    python bench/burgers_bench_gap.py [--n 256] [--heat-s 20]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multigpu_advectiondiffusion_amd import Burgers, Diffusion, Grid, Solver  # noqa: E402
from multigpu_advectiondiffusion_amd.parallel import Comm  # noqa: E402


def rates(solvers, dt, rounds=3, iters=100):
    out = {k: [] for k in solvers}
    for _ in range(rounds):
        for k, s in solvers.items():
            out[k].append(round(s.run(iters=iters, dt=dt).compute_s / iters * 1e3, 4))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=256)
    ap.add_argument("--heat-s", type=float, default=20.0)
    a = ap.parse_args()
    m = Burgers(viscosity=1e-5, weno="z", cfl=0.3)
    g = Grid((a.n,) * 3, (2.0, 2.0, 2.0))
    m.bind(g)
    dt = m.stable_dt()
    comm = Comm.from_env(device="cuda")
    solvers = {"rate_tool": Solver(m, g, dtype=torch.float64, ic="gaussian"),
               "bench": Solver(m, g, comm, dtype=torch.float64, ic="gaussian", overlap=True,
                               decomp=None)}
    for s in solvers.values():
        s.run(iters=200, dt=dt)
    cold = rates(solvers, dt)
    # a heat FD4 512^3 load of the bench's length, then the same rounds
    hg = Grid((512,) * 3, (1.0, 1.0, 1.0))
    hm = Diffusion(K=1.0, order=4)
    hm.bind(hg)
    hs = Solver(hm, hg, comm, dtype=torch.float64, ic="sine", overlap=True, decomp=None)
    hdt = hm.stable_dt()
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < a.heat_s:
        hs.run(iters=200, dt=hdt)
    del hs
    torch.cuda.empty_cache()
    hot = rates(solvers, dt)
    print(json.dumps({"n": a.n, "cold_ms": cold, "after_heat_ms": hot}), flush=True)


if __name__ == "__main__":
    main()
