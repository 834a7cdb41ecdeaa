#!/usr/bin/env python3
"""2-D heat (FD4, fused step) throughput across grid sizes on one GPU.

    python bench/heat2d_sizes.py [--sizes 400 1001 2048 4096 8192]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multigpu_advectiondiffusion_amd import Diffusion, Grid, Solver  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--sizes", type=int, nargs="+", default=[400, 1001, 2048, 4096, 8192, 16384])
ap.add_argument("--steps", type=int, default=64)
a = ap.parse_args()
out = {}
for n in a.sizes:
    s = Solver(Diffusion(K=1.0, order=4), Grid((n, n), (1.0, 1.0)), dtype=torch.float64,
               device="cuda", ic="sine")
    s.run(iters=16)
    st = s.run(iters=a.steps)
    out[n] = {"MLUPS": round(n * n * a.steps / st.compute_s / 1e6, 1),
              "us_per_step": round(st.compute_s / a.steps * 1e6, 1)}
    del s
    torch.cuda.empty_cache()
print(json.dumps(out))
