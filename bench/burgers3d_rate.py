#!/usr/bin/env python3
"""In-solver rate of the bench's 3-D Burgers case (WENO5-Z + FD4 viscous, 256^3, fp64,
SSP-RK3) — one JSON line per process, for interleaved A/B runs of two builds or
settings (ADVDIFF_B3_PACK / B3_TX / B3_VER; knobs are read once per process):

    python bench/burgers3d_rate.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multigpu_advectiondiffusion_amd import Burgers, Grid, Solver  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    m = Burgers(viscosity=1e-5, weno="z", cfl=0.3)
    g = Grid((n, n, n), (2.0, 2.0, 2.0))
    m.bind(g)
    s = Solver(m, g, dtype=torch.float64, ic="gaussian")
    dt = m.stable_dt()
    s.run(iters=200, dt=dt)  # past the clock dip
    times = [s.run(iters=100, dt=dt).compute_s / 100 for _ in range(5)]
    knobs = {k: v for k, v in os.environ.items() if k.startswith("ADVDIFF_")}
    print(json.dumps({"knobs": knobs, "n": n, "ms_per_step": [round(t * 1e3, 4) for t in times],
                      "best_mlups": round(g.cells / min(times) / 1e6, 1),
                      "max_abs_u": s.check_finite()}), flush=True)


if __name__ == "__main__":
    main()
