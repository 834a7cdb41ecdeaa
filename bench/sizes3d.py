#!/usr/bin/env python3
"""One-GPU rate of the 3-D solvers against grid size: heat FD4 / FD2 (fused step) on cubes
64^3 .. 1024^3 and viscous Burgers WENO5-Z on 64^3 .. 512^3, fp64, in the solver
(hipGraph-replayed steps), each timed for ~50 ms after a ~50 ms warm-up so the clock has
settled.  One line per case: size, ms per step, MLUPS.

    python bench/sizes3d.py [--max 1024] [--burgers-max 512]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multigpu_advectiondiffusion_amd import Burgers, Diffusion, Grid, Solver  # noqa: E402


def rate(model, n, ic):
    g = Grid((n, n, n), (1.0, 1.0, 1.0) if isinstance(model, Diffusion) else (2.0, 2.0, 2.0))
    s = Solver(model, g, dtype=torch.float64, ic=ic)
    dt = model.stable_dt() if isinstance(model, Diffusion) else s.dt()
    # size the runs from one step's time
    s.run(iters=8, dt=dt)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    s.run(iters=8, dt=dt)
    torch.cuda.synchronize()
    per = max((time.perf_counter() - t0) / 8, 1e-6)
    steps = max(16, int(0.05 / per) // 8 * 8)
    s.run(iters=steps, dt=dt)  # warm-up at the measured load
    st = s.run(iters=steps, dt=dt)
    ms = st.compute_s / st.steps * 1e3
    del s
    torch.cuda.empty_cache()
    return {"n": n, "steps": steps, "ms_per_step": round(ms, 4),
            "mlups": round(n ** 3 / (ms * 1e3), 1)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--max", type=int, default=1024)
    ap.add_argument("--burgers-max", type=int, default=512)
    a = ap.parse_args()
    sizes = [n for n in (64, 96, 128, 192, 256, 384, 512, 768, 1024) if n <= a.max]
    for order in (4, 2):
        for n in sizes:
            r = rate(Diffusion(K=1.0, order=order), n, "sine")
            print(json.dumps({"case": f"heat FD{order}", **r}), flush=True)
    for n in [n for n in sizes if n <= a.burgers_max]:
        r = rate(Burgers(viscosity=1e-5, weno="z", cfl=0.3), n, "gaussian")
        print(json.dumps({"case": "burgers WENO5-Z", **r}), flush=True)


if __name__ == "__main__":
    main()
