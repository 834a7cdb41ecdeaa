#!/usr/bin/env python3
"""Fused FD2 heat step: tile A/B (advdiff_set_step_fd2_tile: 0 = 12 waves x 3 rows, one
workgroup per CU; --alt 1 = 8 waves x 3 rows, two per CU; --alt 2 = 12 waves x 4 rows,
48-row tiles), fp64, per size; interleaved rounds
of back-to-back launches after a settling burst, min over rounds; bitwise comparison of
one step across the tiles.  (An FD4 8 x 2 / 8 x 3 / 12 x 2 counterpart was not built:
8 x 3 and 12 x 2 spill 86 / 102 VGPRs at two workgroups per CU, and 8 x 2 carries 29 %
more stage work than 16 x 2 — after FD2 8 x 3 lost 5-13 %, profiles/r5/ab/step_tile_ab.log.)

    python bench/step_tile_ab.py [--sizes 384,512,640,768,1024] [--rounds 4]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multigpu_advectiondiffusion_amd.ops import _lib, stencil  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="384,512,640,768,1024")
    ap.add_argument("--dtype", default="float64")
    ap.add_argument("--alt", type=int, default=1, help="tile to compare with 12 x 3: 1 = 8 x 3, "
                    "2 = 12 x 4")
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--reps", type=int, default=8)
    ap.add_argument("--pitch", default="0,0", help="fields of (n, n + PY, n + PX)")
    a = ap.parse_args()
    px, py = (int(v) for v in a.pitch.split(","))
    lib = _lib.require()
    dtype = getattr(torch, a.dtype)
    setter = lib.advdiff_set_step_fd2_tile
    R = 1
    names = ("tile12x3", {1: "tile8x3", 2: "tile12x4"}[a.alt])
    for n in (int(v) for v in a.sizes.split(",")):
        u = torch.rand((n, n + py, n + px), dtype=dtype, device="cuda")
        pair = [u, u.clone()]
        kw = dict(nx=n, ny=n, k0=R, k1=n - R, zlo=R, zhi=n - R, border=R, cx=1.0, cy=1.0,
                  cz=1.0, dt=0.05, order=2, exclusive=True)
        outs = {}
        for t, tv in ((0, 0), (1, a.alt)):
            old = setter(tv)
            o = u.clone()
            stencil.diffusion3d_step(u, o, **kw)
            torch.cuda.synchronize()
            setter(old)
            outs[t] = o
        same = torch.equal(outs[0], outs[1])
        del outs

        def step():
            stencil.diffusion3d_step(pair[0], pair[1], **kw)
            pair.reverse()
        best = {0: float("inf"), 1: float("inf")}
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for _ in range(30):
            step()
        for _ in range(a.rounds):
            for t, tv in ((0, 0), (1, a.alt)):
                old = setter(tv)
                try:
                    for _ in range(2):
                        step()
                    s.record()
                    for _ in range(a.reps):
                        step()
                    e.record()
                    torch.cuda.synchronize()
                finally:
                    setter(old)
                best[t] = min(best[t], s.elapsed_time(e) * 1e3 / a.reps)
        cells = (n - 2 * R) ** 3
        print(json.dumps({"n": n, "dtype": a.dtype, "bitwise_equal": same,
                          f"{names[0]}_us": round(best[0], 1), f"{names[1]}_us": round(best[1], 1),
                          f"{names[0]}_mlups": round(cells / best[0], 1),
                          f"{names[1]}_mlups": round(cells / best[1], 1),
                          f"speedup_{names[1]}": round(best[0] / best[1], 3)}), flush=True)
        del u, pair
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
