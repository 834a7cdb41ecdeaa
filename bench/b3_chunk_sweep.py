#!/usr/bin/env python3
"""3-D WENO5-Z viscous stage (v9, fp64): stage time against the forced z-chunk length
(advdiff_set_b3_zchunk; 0 = the rounds model) and the tile row (64 / 32), per grid —
where the 512^3 stage loses its ~10 % against 256^3.  Interleaved rounds of back-to-back
stage launches after a settling burst; min over rounds.

    python bench/b3_chunk_sweep.py [--sizes 256,512] [--chunks 0,32,64,...] [--rounds 3]
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
    ap.add_argument("--sizes", default="256,512")
    ap.add_argument("--chunks", default="0,16,32,48,64,85,102,128,170,253,506")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    lib = _lib.require()
    for n in (int(s) for s in a.sizes.split(",")):
        x = torch.linspace(0, 1, n, dtype=torch.float64, device="cuda")
        u = (torch.sin(5 * x.view(1, 1, -1) + 2 * x.view(1, -1, 1)) * torch.cos(3 * x.view(-1, 1, 1))
             + 0.5 * torch.tanh(30 * (x.view(1, 1, -1) - 0.4)))
        i, u0, o = u.clone(), u.clone(), u.clone()
        del u
        rd = n / 2.0
        v = 1e-5 * rd * rd
        kw = dict(nx=n, ny=n, k0=3, k1=n - 3, border=3, weno_z=True, rdx=rd, rdy=rd, rdz=rd,
                  vx=v, vy=v, vz=v, dt=1e-4, a=0.75, b=0.25)
        chunks = [int(c) for c in a.chunks.split(",") if int(c) <= n - 6]
        cfgs = [(tx, zc) for tx in (64, 32) for zc in chunks]
        best = {c: float("inf") for c in cfgs}
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for _ in range(40):  # settle the clock
            stencil.burgers3d_stage(i, u0, o, **kw)
        for _ in range(a.rounds):
            for tx, zc in cfgs:
                ot, oz = lib.advdiff_set_b3_tx(tx), lib.advdiff_set_b3_zchunk(zc)
                try:
                    for _ in range(3):
                        stencil.burgers3d_stage(i, u0, o, **kw)
                    s.record()
                    for _ in range(a.reps):
                        stencil.burgers3d_stage(i, u0, o, **kw)
                    e.record()
                    torch.cuda.synchronize()
                finally:
                    lib.advdiff_set_b3_tx(ot)
                    lib.advdiff_set_b3_zchunk(oz)
                best[(tx, zc)] = min(best[(tx, zc)], s.elapsed_time(e) * 1e3 / a.reps)
        cells = (n - 6) ** 3
        for (tx, zc), t in sorted(best.items(), key=lambda kv: kv[1]):
            print(json.dumps({"n": n, "tx": tx, "zchunk": zc, "us": round(t, 1),
                              "stage_mlups": round(cells / t, 1),
                              "step_mlups": round(cells / t / 3, 1)}), flush=True)
        del i, u0, o
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
