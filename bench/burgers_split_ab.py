#!/usr/bin/env python3
"""Slab-rank WENO5-Z + viscous stage: the split launches of the overlapped schedule (the
interior launch + ONE launch of both R-plane boundary slabs) against one launch over every
owned plane, and against that launch with its boundary planes also stored into a "peer"
field (the fused halo puts, advdiff_burgers3d_stage_put; the peer in this GPU's HBM, so
the kernel side only) (round 6).  One
process, the per-rank blocks of the weak-scaling Burgers bench (base 256, fp64, R = 3
ghost planes per side); interleaved rounds of 3-stage sequences (HIP events, min).

    python bench/burgers_split_ab.py [--shapes 8,4,2] [--rounds 5] [--steps 10]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multigpu_advectiondiffusion_amd.ops import stencil  # noqa: E402

# ranks -> (nx, ny, owned planes) of one slab rank of weak_scaling_grid(256, ranks)
SHAPES = {8: (512, 512, 64), 4: (256, 512, 128), 2: (256, 256, 256), 1: (256, 256, 256)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="8,4,2")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=10)
    a = ap.parse_args()
    R = 3
    for n in (int(v) for v in a.shapes.split(",")):
        nx, ny, own = SHAPES[n]
        nz = own + 2 * R
        h = 2.0 / 256
        kw = dict(nx=nx, ny=ny, border=3, weno_z=True, rdx=1 / h, rdy=1 / h, rdz=1 / h,
                  vx=1e-5 / h ** 2, vy=1e-5 / h ** 2, vz=1e-5 / h ** 2, dt=1e-4)
        u = (torch.rand((nz, ny, nx), dtype=torch.float64, device="cuda") - 0.5)
        A, B = u.clone(), u.clone()
        stages = ((u, None, A, 0.0, 1.0), (A, u, B, 0.75, 0.25), (B, u, u, 1.0 / 3, 2.0 / 3))

        def split():
            for _ in range(a.steps):
                for i, u0, o, aa, bb in stages:
                    stencil.burgers3d_stage(i, u0 if u0 is not None else i, o, k0=2 * R,
                                            k1=own, a=aa, b=bb, **kw)
                    stencil.burgers3d_stage(i, u0 if u0 is not None else i, o, k0=R, k1=2 * R,
                                            k0b=own, k1b=own + R, a=aa, b=bb, **kw)

        def whole():
            for _ in range(a.steps):
                for i, u0, o, aa, bb in stages:
                    stencil.burgers3d_stage(i, u0 if u0 is not None else i, o, k0=R,
                                            k1=own + R, a=aa, b=bb, **kw)

        peer = torch.zeros_like(u)
        szb = u.stride(0) * 8
        put = ((peer.data_ptr() + (R + own) * szb, R, 2 * R), (peer.data_ptr(), own, own + R))

        def fused():
            for _ in range(a.steps):
                for i, u0, o, aa, bb in stages:
                    stencil.burgers3d_stage(i, u0 if u0 is not None else i, o, k0=R,
                                            k1=own + R, a=aa, b=bb, put=put, **kw)

        def timed(run):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            run()
            e1.record()
            e1.synchronize()
            return e0.elapsed_time(e1) * 1e3 / a.steps

        runs = {"split": split, "whole": whole, "put": fused}
        for _ in range(2):
            for r in runs.values():
                r()
        best = {k: 1e30 for k in runs}
        for _ in range(a.rounds):
            for k, r in runs.items():
                best[k] = min(best[k], timed(r))
        cells = nx * ny * own
        print(json.dumps({"ranks": n, "rank_block": [nx, ny, own],
                          **{f"{k}_us_per_step": round(t, 1) for k, t in best.items()},
                          **{f"{k}_mlups": round(cells / t, 1) for k, t in best.items()},
                          "whole_vs_split": round(best["split"] / best["whole"], 4),
                          "put_vs_split": round(best["split"] / best["put"], 4)}),
              flush=True)
        del u, A, B, peer
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
