#!/usr/bin/env python3
"""BASELINE.json config 1: "Diffusion2d 256×256 on CPU (Matlab_Prototipes serial path)".

Runs the same problem three ways on the CPU and prints one JSON line:
* the MATLAB prototype port (`Matlab_Prototipes/DiffusionNd/diffusion2dTest.m` ->
  models/prototypes.heat_test, numpy),
* the framework's Solver on the CPU (PyTorch reference ops, 1 process),
* the Solver on P gloo ranks (y-slabs) — bitwise equal to 1 rank.
Accuracy (L1/L2/Linf vs the exact heat kernel) is the target here, not speed.

    python bench/cpu_diffusion2d.py [--n 256] [--t-final 0.2] [--ranks 2]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multigpu_advectiondiffusion_amd import Diffusion, Grid, Solver  # noqa: E402
from multigpu_advectiondiffusion_amd.launch import spawn_local  # noqa: E402
from multigpu_advectiondiffusion_amd.models import prototypes as mp  # noqa: E402


def _solver_run(comm, n, t_final):
    g = Grid((n, n), (10.0, 10.0))
    s = Solver(Diffusion(K=1.0, order=4), g, comm, dtype=torch.float64, device="cpu",
               ic="heat", t0=0.1)
    st = s.run(t_end=t_final)
    l1, l2, li = s.error_norms()
    u = s.gather()
    return None if u is None else (st.steps, st.compute_s, (l1, l2, li), u)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=256)
    ap.add_argument("--t-final", type=float, default=0.2)
    ap.add_argument("--ranks", type=int, default=2)
    a = ap.parse_args()
    n = a.n
    t0 = time.perf_counter()
    l1, l2, li, it, _ = mp.heat_test(2, n, a.t_final)
    tp = time.perf_counter() - t0
    steps, ts, norms, u1 = spawn_local(1, _solver_run, n, a.t_final)[0]
    stepsP, tsP, normsP, uP = spawn_local(a.ranks, _solver_run, n, a.t_final)[0]
    out = {
        "config": f"Diffusion2d {n}x{n} FD4 + SSP-RK3 on CPU (heat kernel t0=0.1 -> {a.t_final})",
        "matlab_port": {"steps": it, "s": round(tp, 3), "MLUPS": round(n * n * it / tp / 1e6, 2),
                        "L1": l1, "L2": l2, "Linf": li},
        "solver_1rank": {"steps": steps, "s": round(ts, 3),
                         "MLUPS": round(n * n * steps / ts / 1e6, 2), "L1": norms[0],
                         "L2": norms[1], "Linf": norms[2]},
        f"solver_{a.ranks}ranks_gloo": {"steps": stepsP, "s": round(tsP, 3),
                                        "bitwise_equal_to_1rank": bool(np.array_equal(u1, uP))},
    }
    print(json.dumps(out))


if __name__ == "__main__":
    main()
