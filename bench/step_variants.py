#!/usr/bin/env python3
"""A/B timing of the 3-D fused-step kernel variants (diffusion_fused.hip dispatch_step)
at production size: median HIP-event time per launch, persistent (exclusive) and grid
schedules, FD4 and FD2, fp64.

    python bench/step_variants.py [--n 512] [--reps 20] [--cfgs 0,16,20,21,22,23]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multigpu_advectiondiffusion_amd.ops import _lib, stencil  # noqa: E402


def timeit(fn, reps):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(reps):
        e0.record()
        fn()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e-3)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=512)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--cfgs", default="0,21,23,24,25,27")
    ap.add_argument("--orders", default="4,2")
    ap.add_argument("--edges", default="1", help="v3 edge tiles on/off values to A/B (1,0)")
    ap.add_argument("--schedules", default="persist,grid")
    ap.add_argument("--rounds", type=int, default=1,
                    help="interleave the configs over this many rounds (median): clock drift "
                         "between configs cancels")
    args = ap.parse_args()
    lib = _lib.require()
    n = args.n
    u = torch.rand((n, n, n), dtype=torch.float64, device="cuda")
    v = torch.empty_like(u)
    ref = {}
    out = {}
    import statistics
    for order in [int(o) for o in args.orders.split(",")]:
        R = order // 2
        kw = dict(nx=n, ny=n, k0=R, k1=n - R, zlo=R, zhi=n - R, border=R, order=order,
                  cx=1.0, cy=1.0, cz=1.0, dt=0.01)
        cfgs = [int(c) for c in args.cfgs.split(",")]
        times = {}
        for _ in range(args.rounds):
            for cfg, edge in [(c, e) for c in cfgs for e in map(int, args.edges.split(","))]:
                lib.advdiff_set_step_cfg(cfg)
                lib.advdiff_set_step_edge(edge)
                for excl in [s == "persist" for s in args.schedules.split(",")]:
                    lib.advdiff_set_step_persist(1 if excl else 0)
                    t = timeit(lambda: stencil.diffusion3d_step(u, v, exclusive=excl, **kw),
                               args.reps)
                    torch.cuda.synchronize()
                    key = (order, excl)
                    tag = (f"fd{order}_cfg{cfg}{'' if edge else '_noedge'}_"
                           f"{'persist' if excl else 'grid'}")
                    if key not in ref:
                        ref[key] = v.clone()
                        same = True
                    else:
                        same = bool(torch.equal(ref[key], v))
                    times.setdefault(tag, []).append(t)
                    out[tag] = {"us": round(statistics.median(times[tag]) * 1e6, 1),
                                "mlups": round(n ** 3 / statistics.median(times[tag]) / 1e6, 1),
                                "bitwise_vs_first": same and out.get(tag, {}).get(
                                    "bitwise_vs_first", True)}
        for tag in [t for t in out if t.startswith(f"fd{order}_")]:
            print(tag, out[tag], flush=True)
    lib.advdiff_set_step_cfg(0)
    lib.advdiff_set_step_persist(0)
    lib.advdiff_set_step_edge(1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
