#!/usr/bin/env python3
"""Grids sized for one MI355X's 288 GB of HBM3E: 2048³ fp64 heat (fused step, 2 fields,
137 GB) and 1536³ fp64 viscous Burgers (3 fields, 87 GB), timed like bench.py.

    python bench/large_grid.py [--heat 2048] [--burgers 1536] [--steps 10]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multigpu_advectiondiffusion_amd import Burgers, Diffusion, Grid, Solver  # noqa: E402


def run(model, n, ic, steps, warmup):
    s = Solver(model, Grid((n, n, n), (1.0, 1.0, 1.0)), dtype=torch.float64, device="cuda",
               ic=ic)
    mem = s.memory_bytes()
    dt = model.stable_dt()
    s.run(iters=warmup, dt=dt)
    st = s.run(iters=steps, dt=dt)
    mx = s.check_finite()
    out = {"grid": [n, n, n], "cells": n ** 3, "fields_GB": round(mem / 1e9, 1),
           "peak_alloc_GB": round(torch.cuda.max_memory_allocated() / 1e9, 1),
           "steps": steps, "ms_per_step": round(st.compute_s / steps * 1e3, 2),
           "MLUPS": round(n ** 3 * steps / st.compute_s / 1e6, 1), "max_abs_u": mx,
           "fused": s.fused}
    del s
    torch.cuda.empty_cache()
    torch.cuda.reset_peak_memory_stats()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--heat", type=int, default=2048)
    ap.add_argument("--burgers", type=int, default=1536)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    a = ap.parse_args()
    t0 = time.time()
    res = {"device": torch.cuda.get_device_name(0),
           "hbm_GB": round(torch.cuda.get_device_properties(0).total_memory / 1e9, 1)}
    res["heat3d_fd4_fused"] = run(Diffusion(K=1.0, order=4), a.heat, "sine", a.steps, a.warmup)
    print(json.dumps(res), flush=True)
    res["burgers3d_weno5z_visc"] = run(Burgers(viscosity=1e-5, weno="z", cfl=0.3), a.burgers,
                                       "gaussian", max(a.steps // 3, 2), 1)
    res["wall_s"] = round(time.time() - t0, 1)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
