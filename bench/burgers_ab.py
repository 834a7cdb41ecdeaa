#!/usr/bin/env python3
"""Interleaved A/B of the 3-D WENO5 v9 stage (advdiff_set_b3_prio 0 / 1) at 256^3 fp64,
WENO5-Z + viscous, SSP stage 2 epilogue; medians of rounds x reps launches (HIP events),
outputs compared bit for bit.

    python bench/burgers_ab.py [--n 256] [--rounds 7] [--reps 10]
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multigpu_advectiondiffusion_amd.ops import _lib, stencil  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=256)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    lib = _lib.require()
    n = a.n
    g = torch.Generator(device="cuda").manual_seed(4)
    u = torch.rand((n, n, n), dtype=torch.float64, device="cuda", generator=g) * 0.5 + 0.1
    u0 = torch.rand_like(u)
    kw = dict(nx=n, ny=n, k0=3, k1=n - 3, border=3, weno_z=True, rdx=n / 2.0, rdy=n / 2.0,
              rdz=n / 2.0, vx=1e-5 * n * n / 4, vy=1e-5 * n * n / 4, vz=1e-5 * n * n / 4,
              dt=1e-4, a=0.75, b=0.25)
    variants = (0, 1)
    times = {v: [] for v in variants}
    ref = None
    for rnd in range(a.rounds):
        for v in variants:
            lib.advdiff_set_b3_prio(v)
            o = u0.clone()
            stencil.burgers3d_stage(u, u0, o, **kw)
            torch.cuda.synchronize()
            if ref is None:
                ref = o.clone()
            elif rnd == 0 and not torch.equal(o, ref):
                raise SystemExit(f"b3_prio {v} differs: {(o - ref).abs().max().item()}")
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.reps):
                stencil.burgers3d_stage(u, u0, o, **kw)
            e1.record()
            e1.synchronize()
            times[v].append(e0.elapsed_time(e1) / a.reps * 1e3)
    lib.advdiff_set_b3_prio(0)
    print(json.dumps({"n": n, **{str(v): {"median_us": round(statistics.median(t), 1),
                                          "min_us": round(min(t), 1)} for v, t in times.items()}}))


if __name__ == "__main__":
    main()
