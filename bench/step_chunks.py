#!/usr/bin/env python3
"""Fused heat step (fp64) against its z-chunk length, at the shapes that matter: 512^3,
1024^3 and the 8-GPU slab rank's block (1024 x 1024 x 128 owned planes + 2 x 6 ghosts; its
interior launch [12, 128)).  Each case times the automatic chunk (pick_chunk_rounds) and
forced chunks, interleaved over rounds (clock drift), by HIP events over a run of
back-to-back launches after a settling run.  Per case: us per launch and MLUPS per chunk.

    python bench/step_chunks.py [--rounds 3] [--cases 512,1024,slab8] [--pitch PX,PY]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multigpu_advectiondiffusion_amd.ops import _lib, stencil  # noqa: E402


def case_args(name, order):
    R = order // 2
    if name == "512":
        n = 512
        return (n, n, n), dict(k0=R, k1=n - R, zlo=R, zhi=n - R), (n - 2 * R) ** 2 * (n - 2 * R)
    if name == "1024":
        n = 1024
        return (n, n, n), dict(k0=R, k1=n - R, zlo=R, zhi=n - R), (n - 2 * R) ** 2 * (n - 2 * R)
    if name == "slab8":  # interior launch of a middle rank: ghosts 3R, owned 128
        G = 3 * R
        nz = 128 + 2 * G
        return (nz, 1024, 1024), dict(k0=2 * G, k1=nz - 2 * G, zlo=0, zhi=nz), \
            (1024 - 2 * R) ** 2 * (nz - 4 * G)
    raise KeyError(name)


def time_launches(fn, n):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--cases", default="512,1024,slab8")
    ap.add_argument("--orders", default="4,2")
    ap.add_argument("--pitch", default="0,0",
                    help="fields of (nz, ny + PY, nx + PX): the solver's pitched layout")
    a = ap.parse_args()
    px, py = (int(v) for v in a.pitch.split(","))
    lib = _lib.require()
    for name in a.cases.split(","):
        for order in map(int, a.orders.split(",")):
            shape, rng, cells = case_args(name, order)
            nz, ny, nx = shape
            u = torch.rand((nz, ny + py, nx + px), dtype=torch.float64, device="cuda")
            v = u.clone()
            kw = dict(nx=nx, ny=ny, border=order // 2, order=order, cx=1.0, cy=1.0, cz=1.0,
                      dt=0.01, **rng)
            span = rng["k1"] - rng["k0"]
            chunks = [0] + sorted({c for c in (8, 12, 16, 20, 24, 29, 32, 40, 48, 58, 64, 96,
                                               128, 256) if c <= span})
            best = {c: float("inf") for c in chunks}
            pair = [u, v]

            def fn():
                stencil.diffusion3d_step(pair[0], pair[1], **kw)
                pair.reverse()
            lib.advdiff_set_step_zchunk(0)
            time_launches(fn, 40)  # settle the clock at this load
            for _ in range(a.rounds):
                for c in chunks:
                    lib.advdiff_set_step_zchunk(c)
                    time_launches(fn, 4)
                    best[c] = min(best[c], time_launches(fn, 12))
            lib.advdiff_set_step_zchunk(0)
            rec = {"case": name, "order": order, "shape": list(shape), "pitch": [px, py],
                   "auto_us": round(best[0], 1),
                   "auto_mlups": round(cells / best[0], 1),
                   "by_chunk_us": {str(c): round(best[c], 1) for c in chunks if c}}
            bc = min((c for c in chunks if c), key=lambda c: best[c])
            rec["best_chunk"] = bc
            rec["best_mlups"] = round(cells / best[bc], 1)
            print(json.dumps(rec), flush=True)
            del u, v, pair
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
