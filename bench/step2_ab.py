#!/usr/bin/env python3
"""Two steps per launch (FD2 v6_march) vs one step per launch (v3_march), interleaved
rounds of back-to-back launches after a settling run; bitwise comparison of one pair of
steps.  MLUPS counts cell updates per step (a two-step launch updates every cell twice).

    python bench/step2_ab.py [--sizes 512,1024] [--rounds 4]
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
    ap.add_argument("--sizes", default="512,1024")
    ap.add_argument("--dtypes", default="float64,float32")
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--reps", type=int, default=8, help="two-step pairs per timed window")
    a = ap.parse_args()
    for dname in a.dtypes.split(","):
        dtype = getattr(torch, dname)
        for n in (int(s) for s in a.sizes.split(",")):
            u = torch.rand((n, n, n), dtype=dtype, device="cuda")
            v = u.clone()
            w = u.clone()
            kw = dict(nx=n, ny=n, k0=1, k1=n - 1, zlo=1, zhi=n - 1, border=1, cx=1.0, cy=1.0,
                      cz=1.0, dt=0.1)
            stencil.diffusion3d_step(u, v, order=2, **kw)
            stencil.diffusion3d_step(v, w, order=2, **kw)
            x = u.clone()
            stencil.diffusion3d_step2x(u, x, **kw)
            torch.cuda.synchronize()
            same = torch.equal(w, x)
            diff = 0.0 if same else (w - x).abs().max().item()
            del w, x
            pair = [u, v]

            def one():  # two one-step launches
                stencil.diffusion3d_step(pair[0], pair[1], order=2, **kw)
                stencil.diffusion3d_step(pair[1], pair[0], order=2, **kw)

            def two():  # one two-step launch
                stencil.diffusion3d_step2x(pair[0], pair[1], **kw)
                pair.reverse()
            fns = {"one_step": one, "two_step": two}
            best = {k: float("inf") for k in fns}
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            for _ in range(30):
                one()
            for _ in range(a.rounds):
                for k, fn in fns.items():
                    for _ in range(3):
                        fn()
                    s.record()
                    for _ in range(a.reps):
                        fn()
                    e.record()
                    torch.cuda.synchronize()
                    best[k] = min(best[k], s.elapsed_time(e) * 1e3 / (2 * a.reps))
            cells = (n - 2) ** 3
            print(json.dumps({"dtype": dname, "n": n, "bitwise_equal": same, "max_diff": diff,
                              **{f"{k}_us_per_step": round(t, 1) for k, t in best.items()},
                              **{f"{k}_mlups": round(cells / t, 1) for k, t in best.items()},
                              "speedup": round(best["one_step"] / best["two_step"], 3)}),
                  flush=True)
            del u, v, pair
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
