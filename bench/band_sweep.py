#!/usr/bin/env python3
"""Measured landscape of the banded z schedule for one fused-step launch: forced splits
(advdiff_set_step_bands first, rest) against uniform chunks and the model's split, at
512^3 fp64 on the pitched layout; interleaved rounds after a settling burst.

    python bench/band_sweep.py [--order 4] [--first 254,300,340,387,420,460]
        [--rest 64,84,100,121,127]
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
    ap.add_argument("--n", type=int, default=512)
    ap.add_argument("--order", type=int, default=4)
    ap.add_argument("--first", default="254,300,340,387,420,460")
    ap.add_argument("--rest", default="64,84,100,121,127")
    ap.add_argument("--rounds", type=int, default=4)
    a = ap.parse_args()
    lib = _lib.require()
    n, R = a.n, a.order // 2
    u = torch.rand((n, n + 1, n + 4), dtype=torch.float64, device="cuda")
    pair = [u, u.clone()]
    kw = dict(nx=n, ny=n, k0=R, k1=n - R, zlo=R, zhi=n - R, border=R, order=a.order, cx=1.0,
              cy=1.0, cz=1.0, dt=0.01)
    cfgs = [("uniform", 0, 0, 0), ("model", 1, 0, 0)]
    for f in (int(v) for v in a.first.split(",")):
        for r in (int(v) for v in a.rest.split(",")):
            if f < n - 2 * R:
                cfgs.append((f"{f}+{r}", 1, f, r))

    def run(k):
        for _ in range(k):
            stencil.diffusion3d_step(pair[0], pair[1], **kw)
            pair.reverse()

    def setc(c):
        lib.advdiff_set_step_banded(c[1])
        lib.advdiff_set_step_bands(c[2], c[3])
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    setc(cfgs[0])
    run(60)
    best = {c[0]: float("inf") for c in cfgs}
    for _ in range(a.rounds):
        for c in cfgs:
            setc(c)
            run(2)
            s.record()
            run(8)
            e.record()
            torch.cuda.synchronize()
            best[c[0]] = min(best[c[0]], s.elapsed_time(e) * 1e3 / 8)
    lib.advdiff_set_step_banded(-1)
    lib.advdiff_set_step_bands(0, 0)
    ref = best["uniform"]
    for name, us in sorted(best.items(), key=lambda kv: kv[1]):
        print(json.dumps({"order": a.order, "n": n, "split": name, "us": round(us, 1),
                          "vs_uniform": round(ref / us, 4)}), flush=True)


if __name__ == "__main__":
    main()
