#!/usr/bin/env python3
"""Interleaved A/B of the fused 3-D heat step's built variants (advdiff_set_step_var: 0 the
plain kernel, -1 the order's phase-overlap default — FD4 graded wave priority (VAR 3), FD2
adjacent rows + deferred stage 3 + priority (VAR 23); a new VAR needs its instance in
csrc/kernels/diffusion_fused.hip), 512^3 fp64, FD4 and FD2.  Rounds x variants x reps
launches timed with HIP events, medians per variant; every variant's output must equal the
first one's bit for bit.

    python bench/step_ab.py [--n 512] [--rounds 5] [--reps 10] [--vars 0,-1]
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
    ap.add_argument("--n", type=int, default=512)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--vars", default="0,-1")
    ap.add_argument("--orders", default="4,2")
    a = ap.parse_args()
    lib = _lib.require()
    variants = [int(v) for v in a.vars.split(",")]
    n = a.n
    g = torch.Generator(device="cuda").manual_seed(3)
    u = torch.rand((n, n, n), dtype=torch.float64, device="cuda", generator=g)
    out = {}
    for order in [int(o) for o in a.orders.split(",")]:
        R = order // 2
        kw = dict(nx=n, ny=n, k0=R, k1=n - R, zlo=R, zhi=n - R, border=R, order=order,
                  cx=0.21, cy=0.17, cz=0.13, dt=0.9 / (2 * 0.51) if order == 2 else 0.5 / 0.51)
        ref = None
        times = {v: [] for v in variants}
        for rnd in range(a.rounds):
            for v in variants:
                lib.advdiff_set_step_var(v)
                o = u.clone()  # cells the step does not write keep u
                stencil.diffusion3d_step(u, o, **kw)
                torch.cuda.synchronize()
                if rnd == 0:
                    if ref is None:
                        ref = o.clone()
                    elif not torch.equal(o, ref):
                        raise SystemExit(f"variant {v} (order {order}) differs from variant "
                                         f"{variants[0]}: {(o - ref).abs().max().item()}")
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.reps):
                    stencil.diffusion3d_step(u, o, **kw)
                e1.record()
                e1.synchronize()
                times[v].append(e0.elapsed_time(e1) / a.reps * 1e3)
        lib.advdiff_set_step_var(-1)
        res = {str(v): {"median_us": round(statistics.median(t), 1), "min_us": round(min(t), 1),
                        "mlups_median": round(n ** 3 / statistics.median(t), 0)}
               for v, t in times.items()}
        out[f"fd{order}"] = res
        print(json.dumps({"order": order, "n": n, **res}), flush=True)


if __name__ == "__main__":
    main()
