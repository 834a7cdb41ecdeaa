#!/usr/bin/env python3
"""Banded z schedule of the fused heat step (advdiff_set_step_banded: one long z band per
column, then short bands that fill the last round of resident workgroups) against uniform
z chunks, at the bench's shape and the per-rank blocks of multi-GPU runs: 512^3, the
8-GPU z-slab rank (1024 x 1024 x 128 owned + 2 x 3R ghosts, interior launch), the 4 x 2
rank (1024 x 512 x 256) and 1024^3; pitched fields as the solver allocates them.
Interleaved rounds of back-to-back launches after a settling burst; the two schedules'
outputs must agree bitwise.

    python bench/banded_ab.py [--cases 512,slab8,r4x2,1024] [--rounds 5]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multigpu_advectiondiffusion_amd.ops import _lib, stencil  # noqa: E402


def case(name, order):
    R = order // 2
    G = 3 * R
    if name in ("512", "1024"):
        n = int(name)
        return (n, n, n), dict(k0=R, k1=n - R, zlo=R, zhi=n - R)
    if name == "slab8":
        nz = 128 + 2 * G
        return (nz, 1024, 1024), dict(k0=2 * G, k1=nz - 2 * G, zlo=0, zhi=nz)
    if name == "r4x2":
        nz = 256 + 2 * G
        return (nz, 512 + G, 1024), dict(k0=2 * G, k1=nz - 2 * G, zlo=0, zhi=nz)
    raise KeyError(name)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", default="512,slab8,r4x2,1024")
    ap.add_argument("--orders", default="4,2")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--pitch", default="4,1")
    a = ap.parse_args()
    lib = _lib.require()
    px, py = (int(v) for v in a.pitch.split(","))
    for name in a.cases.split(","):
        for order in map(int, a.orders.split(",")):
            (nz, ny, nx), rng = case(name, order)
            u = torch.rand((nz, ny + py, nx + px), dtype=torch.float64, device="cuda")
            kw = dict(nx=nx, ny=ny, border=order // 2, order=order, cx=1.0, cy=1.0, cz=1.0,
                      dt=0.01, **rng)
            outs = {}
            for m in (0, 1):
                old = lib.advdiff_set_step_banded(m)
                o = u.clone()
                stencil.diffusion3d_step(u, o, **kw)
                torch.cuda.synchronize()
                lib.advdiff_set_step_banded(old)
                outs[m] = o
            same = torch.equal(outs[0], outs[1])
            del outs
            pair = [u, u.clone()]

            def run(k):
                for _ in range(k):
                    stencil.diffusion3d_step(pair[0], pair[1], **kw)
                    pair.reverse()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            run(60)
            best = {0: float("inf"), 1: float("inf")}
            for _ in range(a.rounds):
                for m in (0, 1):
                    old = lib.advdiff_set_step_banded(m)
                    run(3)
                    s.record()
                    run(12)
                    e.record()
                    torch.cuda.synchronize()
                    lib.advdiff_set_step_banded(old)
                    best[m] = min(best[m], s.elapsed_time(e) * 1e3 / 12)
            cells = (nx - 2 * (order // 2)) * (ny - 2 * (order // 2)) * (rng["k1"] - rng["k0"])
            print(json.dumps({"case": name, "order": order, "shape": [nz, ny, nx],
                              "uniform_us": round(best[0], 1), "banded_us": round(best[1], 1),
                              "speedup": round(best[0] / best[1], 4),
                              "banded_mlups": round(cells / best[1], 1),
                              "bitwise_equal": same}), flush=True)
            del u, pair
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
