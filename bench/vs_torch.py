#!/usr/bin/env python3
"""A/B of the hand-written gfx950 kernels against the PyTorch reference ops running on
the SAME GPU through the same solver schedule (Solver(kernel="torch") — the "naive
kernel" baseline of SURVEY.md §7.1).  fp64, per-step time and speed-up.

    python bench/vs_torch.py [--n 256] [--nb 192] [--steps 10]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multigpu_advectiondiffusion_amd import Burgers, Diffusion, Grid, Solver  # noqa: E402


def run(model_fn, n, ic, kernel, steps):
    model = model_fn()
    s = Solver(model, Grid((n, n, n), (1.0, 1.0, 1.0)), dtype=torch.float64, device="cuda",
               ic=ic, kernel=kernel)
    dt = model.stable_dt()
    s.run(iters=2, dt=dt, graph=False)
    st = s.run(iters=steps, dt=dt, graph=False)
    return st.compute_s / steps * 1e3, s.gather()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=256)
    ap.add_argument("--nb", type=int, default=192)
    ap.add_argument("--steps", type=int, default=10)
    a = ap.parse_args()
    out = {}
    for name, fn, n, ic in (("heat3d_fd4", lambda: Diffusion(K=1.0, order=4), a.n, "sine"),
                            ("burgers3d_weno5z_visc",
                             lambda: Burgers(viscosity=1e-5, weno="z", cfl=0.3), a.nb,
                             "gaussian")):
        tn, un = run(fn, n, ic, "native", a.steps)
        tt, ut = run(fn, n, ic, "torch", a.steps)
        out[name] = {"grid": n, "native_ms_per_step": round(tn, 3),
                     "torch_ms_per_step": round(tt, 3), "speedup": round(tt / tn, 1),
                     "max_abs_diff": float(np.abs(un - ut).max())}
        torch.cuda.empty_cache()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
