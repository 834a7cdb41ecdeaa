#!/usr/bin/env python3
"""Pitched-allocation A/B of the fused heat step (the reference's *_PitchedMem variants,
SingleGPU/Burgers3d_WENO5_PitchedMem): the same n^3 launch on fields allocated as
(n, n + py, n + px) — row pitch n + px elements, plane pitch (n + py) rows — so that
power-of-two row / plane strides do not map every row of a tile onto the same HBM channels.
Interleaved rounds of back-to-back launches after a settling run; one JSON line per
(order, px, py) with the best round's us per step and MLUPS, and whether the solution
equals the unpadded one bitwise.

    python bench/pitch_ab.py [--n 512] [--dtype fp64] [--pads 0,0 8,0 64,0 0,1 8,1]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multigpu_advectiondiffusion_amd.ops import stencil  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, nargs="+", default=[512])
    ap.add_argument("--dtype", default="fp64", choices=["fp64", "fp32"])
    ap.add_argument("--pads", nargs="+", default=["0,0", "8,0", "64,0", "0,1", "8,1", "0,4"])
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--orders", type=int, nargs="+", default=[4, 2])
    ap.add_argument("--dims", type=int, default=3, choices=[2, 3],
                    help="2: the fused 2-D step on (n, n + px) fields (py ignored)")
    a = ap.parse_args()
    if a.dims == 2:
        return main2d(a)
    dt_ = torch.float64 if a.dtype == "fp64" else torch.float32
    pads = [tuple(int(v) for v in p.split(",")) for p in a.pads]
    for n in a.n:
        for order in a.orders:
            R = order // 2
            kw = dict(nx=n, ny=n, k0=R, k1=n - R, zlo=R, zhi=n - R, border=R, order=order,
                      cx=0.1, cy=0.1, cz=0.1, dt=0.5, exclusive=True)
            g = torch.Generator(device="cuda").manual_seed(3)
            base = torch.rand((n, n, n), dtype=dt_, device="cuda", generator=g)
            fields, ref = {}, None
            for px, py in pads:
                u = torch.zeros((n, n + py, n + px), dtype=dt_, device="cuda")
                v = torch.zeros_like(u)
                u[:, :n, :n] = base
                v[:, :n, :n] = base
                stencil.diffusion3d_step(u, v, **kw)
                out = v[:, :n, :n].clone()
                if ref is None:
                    ref = out
                fields[(px, py)] = ([u, v], torch.equal(out, ref))
                del out
            del base
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            best = {p: float("inf") for p in pads}

            def run(pair, k):
                for _ in range(k):
                    stencil.diffusion3d_step(pair[0], pair[1], **kw)
                    pair.reverse()
            run(fields[pads[0]][0], 200)  # settle the clock
            for _ in range(a.rounds):
                for p in pads:
                    pair = fields[p][0]
                    run(pair, 4)
                    s.record()
                    run(pair, 16)
                    e.record()
                    torch.cuda.synchronize()
                    best[p] = min(best[p], s.elapsed_time(e) * 1e3 / 16)
            cells = (n - 2 * R) ** 3
            for p in pads:
                print(json.dumps({"n": n, "order": order, "dtype": a.dtype, "px": p[0],
                                  "py": p[1], "row_pitch": n + p[0], "rows_per_plane": n + p[1],
                                  "us": round(best[p], 1),
                                  "mlups": round(cells / best[p], 1),
                                  "vs_unpadded": round(best[pads[0]] / best[p], 4),
                                  "bitwise_equal": fields[p][1]}), flush=True)
            del fields, ref
            torch.cuda.empty_cache()


def main2d(a):
    dt_ = torch.float64 if a.dtype == "fp64" else torch.float32
    pads = sorted({int(p.split(",")[0]) for p in a.pads}, key=[int(p.split(",")[0]) for p in a.pads].index)
    for n in a.n:
        for order in a.orders:
            R = order // 2
            kw = dict(nx=n, j0=R, j1=n - R, ylo=R, yhi=n - R, border=R, order=order, cx=0.1,
                      cy=0.1, dt=0.5)
            g = torch.Generator(device="cuda").manual_seed(3)
            base = torch.rand((n, n), dtype=dt_, device="cuda", generator=g)
            fields, ref = {}, None
            for px in pads:
                u = torch.zeros((n, n + px), dtype=dt_, device="cuda")
                v = torch.zeros_like(u)
                u[:, :n] = base
                v[:, :n] = base
                stencil.diffusion2d_step(u, v, **kw)
                out = v[:, :n].clone()
                ref = out if ref is None else ref
                fields[px] = ([u, v], torch.equal(out, ref))
            del base
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            best = {p: float("inf") for p in pads}

            def run(pair, k):
                for _ in range(k):
                    stencil.diffusion2d_step(pair[0], pair[1], **kw)
                    pair.reverse()
            run(fields[pads[0]][0], 200)
            for _ in range(a.rounds):
                for p in pads:
                    run(fields[p][0], 4)
                    s.record()
                    run(fields[p][0], 16)
                    e.record()
                    torch.cuda.synchronize()
                    best[p] = min(best[p], s.elapsed_time(e) * 1e3 / 16)
            cells = (n - 2 * R) ** 2
            for p in pads:
                print(json.dumps({"dims": 2, "n": n, "order": order, "dtype": a.dtype, "px": p,
                                  "us": round(best[p], 2), "mlups": round(cells / best[p], 1),
                                  "vs_unpadded": round(best[pads[0]] / best[p], 4),
                                  "bitwise_equal": fields[p][1]}), flush=True)
            del fields, ref
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
