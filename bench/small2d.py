#!/usr/bin/env python3
"""Small 2-D grids (the reference's MultiGPU 2-D rows, 400x406, and 1001^2): MLUPS of the
2-D Burgers (WENO5-JS inviscid) and 2-D heat (FD4) solvers, one MI355X, fp64.  These
grids hold 0.16-1 M cells, so a stage is a few microseconds and latency-bound (the
Burgers stage walks one row per wave in sequence at these sizes: the chunk floor of 1
row measured best, profiles/archive/small2d_r2.log).

    python bench/small2d.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multigpu_advectiondiffusion_amd import Burgers, Diffusion, Grid, Solver  # noqa: E402

CASES = [
    ("burgers2d_js_400x406", lambda: Burgers(viscosity=0.0, weno="js", cfl=0.4), (400, 406), "gaussian", 400),
    ("burgers2d_js_1001x1001", lambda: Burgers(viscosity=0.0, weno="js", cfl=0.4), (1001, 1001), "gaussian", 200),
    ("burgers2d_z_visc_2048x2048", lambda: Burgers(viscosity=1e-5, weno="z", cfl=0.3), (2048, 2048), "gaussian", 100),
    ("burgers2d_js_4096x4096", lambda: Burgers(viscosity=0.0, weno="js", cfl=0.4), (4096, 4096), "gaussian", 50),
    ("burgers2d_js_16384x16384", lambda: Burgers(viscosity=0.0, weno="js", cfl=0.4), (16384, 16384), "gaussian", 10),
    ("heat2d_fd4_400x406", lambda: Diffusion(K=1.0, order=4, safety=0.8), (400, 406), "disc", 2000),
    ("heat2d_fd4_1001x1001", lambda: Diffusion(K=1.0, order=4), (1001, 1001), "heat", 2000),
]


def main():
    out = {"knobs": {k: v for k, v in os.environ.items() if k.startswith("ADVDIFF_")}}
    only = sys.argv[1:]  # optional name filters
    for name, mk, shape, ic, steps in CASES:
        if only and not any(o in name for o in only):
            continue
        m = mk()
        g = Grid(shape, (2.0,) * len(shape))
        m.bind(g)
        s = Solver(m, g, dtype=torch.float64, ic=ic)
        dt = m.stable_dt()
        s.run(iters=20, dt=dt)
        best = min(s.run(iters=steps, dt=dt).compute_s for _ in range(3))
        out[name] = {"mlups": round(g.cells * steps / best / 1e6, 1),
                     "us_per_step": round(best / steps * 1e6, 2),
                     "max_abs_u": s.check_finite()}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
