#!/usr/bin/env python3
"""In-solver rate of the fused 3-D FD4 heat step on the reference's 3-D heat grids and the
bench grid — one JSON line per process, for interleaved A/B runs of two builds or of
ADVDIFF_STEP_BANDED=0/1 (knobs are read once per process):

    python bench/heat3d_rate.py [order: 4 (default) | 2]
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multigpu_advectiondiffusion_amd import Diffusion, Grid, Solver  # noqa: E402

SHAPES = [(201, 199, 200), (400, 200, 206), (512, 512, 512)]


def main():
    order = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    out = {"knobs": {k: v for k, v in os.environ.items() if k.startswith("ADVDIFF_")},
           "order": order}
    for shape in SHAPES:
        m = Diffusion(K=1.0, order=order)
        g = Grid(shape, (1.0, 1.0, 1.0))
        m.bind(g)
        s = Solver(m, g, dtype=torch.float64, ic="sine")
        dt = m.stable_dt()
        steps = max(30, int(4e9 / g.cells))  # ~20-30 ms per timed run
        s.run(iters=steps, dt=dt)
        best = min(s.run(iters=steps, dt=dt).compute_s for _ in range(3))
        out["x".join(map(str, shape))] = {"mlups": round(g.cells * steps / best / 1e6, 1),
                                          "us_per_step": round(best / steps * 1e6, 2),
                                          "max_abs_u": s.check_finite()}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
