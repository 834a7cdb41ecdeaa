#!/usr/bin/env python3
"""FD2 heat: one-step and two-step launches against the forced z-chunk length
(advdiff_set_step_zchunk; 0 = the rounds model) — why the two-step launch loses at 512^3
fp64 while it wins at 384-1024 (profiles/r5/ab/step2_ab.log, step2_sizes.log).
Interleaved rounds after a settling burst, min over rounds, us per STEP.

    python bench/step2_chunks.py [--n 512] [--chunks 0,32,...] [--rounds 4]
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
    ap.add_argument("--dtype", default="float64")
    ap.add_argument("--chunks", default="0,32,51,64,73,85,102,128,170,255,510")
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--reps", type=int, default=6)
    a = ap.parse_args()
    lib = _lib.require()
    n = a.n
    dtype = getattr(torch, a.dtype)
    u = torch.rand((n, n, n), dtype=dtype, device="cuda")
    pair = [u, u.clone()]
    kw = dict(nx=n, ny=n, k0=1, k1=n - 1, zlo=1, zhi=n - 1, border=1, cx=1.0, cy=1.0, cz=1.0,
              dt=0.1)

    def one():
        stencil.diffusion3d_step(pair[0], pair[1], order=2, **kw)
        stencil.diffusion3d_step(pair[1], pair[0], order=2, **kw)

    def two():
        stencil.diffusion3d_step2x(pair[0], pair[1], **kw)
        pair.reverse()
    chunks = [int(c) for c in a.chunks.split(",")]
    cfgs = [(k, zc) for zc in chunks for k in ("one", "two")]
    fns = {"one": one, "two": two}
    best = {c: float("inf") for c in cfgs}
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(30):
        one()
    for _ in range(a.rounds):
        for k, zc in cfgs:
            old = lib.advdiff_set_step_zchunk(zc)
            try:
                for _ in range(2):
                    fns[k]()
                s.record()
                for _ in range(a.reps):
                    fns[k]()
                e.record()
                torch.cuda.synchronize()
            finally:
                lib.advdiff_set_step_zchunk(old)
            best[(k, zc)] = min(best[(k, zc)], s.elapsed_time(e) * 1e3 / (2 * a.reps))
    cells = (n - 2) ** 3
    for (k, zc), t in sorted(best.items(), key=lambda kv: kv[1]):
        print(json.dumps({"n": n, "dtype": a.dtype, "launch": k, "zchunk": zc,
                          "us_per_step": round(t, 1), "mlups": round(cells / t, 1)}), flush=True)


if __name__ == "__main__":
    main()
