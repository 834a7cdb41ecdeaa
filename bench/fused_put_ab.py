#!/usr/bin/env python3
"""Slab-rank FD4 step: split launches vs one launch with the halo puts inside it (round 6,
transport "ipc+fused").  One process, the per-rank blocks of the weak-scaling bench
(pitched fp64 fields with 3R = 6 ghost planes per side):

* split   : the interior launch (owned planes >= 6 from a face) + ONE launch of both
            6-plane boundary slabs (the ipc / rccl schedule; the puts are a third launch,
            not timed here);
* whole   : one launch over every owned plane (no halo at all: the lower bound);
* put     : the same launch storing its 2 x 6 boundary planes also into a "peer" field —
            here a second field in this GPU's HBM, so what is timed is the kernel side of
            the fused puts (the extra stores and their system scope), not xGMI.

Interleaved rounds of back-to-back launch sequences (HIP events, min per round).

    python bench/fused_put_ab.py [--shapes 8,4,2] [--rounds 5] [--steps 20]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multigpu_advectiondiffusion_amd.ops import _lib, stencil  # noqa: E402

# ranks -> (nx, ny, owned planes) of one slab rank of the weak-scaling grid (base 512)
SHAPES = {8: (1024, 1024, 128), 4: (512, 1024, 256), 2: (512, 512, 512)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="8,4,2")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    G = 6
    for n in (int(v) for v in a.shapes.split(",")):
        nx, ny, own = SHAPES[n]
        nz = own + 2 * G
        c = (1.0, 1.0, 1.0)
        kw = dict(nx=nx, ny=ny, border=2, order=4, cx=c[0], cy=c[1], cz=c[2],
                  dt=0.9 / (2 * sum(c) * 16 / 12), zlo=0, zhi=nz)
        u = torch.rand((nz, ny + 1, nx + 4), dtype=torch.float64, device="cuda")
        v = u.clone()
        peer = torch.zeros_like(u)
        szb = u.stride(0) * 8
        # lower peer: my planes [G, 2G) -> its top ghosts (+own); upper peer: my planes
        # [own, own + G) -> its bottom ghosts (-own); one "peer" field serves both
        put = ((peer.data_ptr() + (G + own) * szb, G, 2 * G),
               (peer.data_ptr() + 0 * szb, own, own + G))

        def split(x, y):
            stencil.diffusion3d_step(x, y, k0=2 * G, k1=own, **kw)
            stencil.diffusion3d_step(x, y, k0=G, k1=2 * G, k0b=own, k1b=own + G, **kw)

        def whole(x, y):
            stencil.diffusion3d_step(x, y, k0=G, k1=own + G, **kw)

        def fused(x, y):
            stencil.diffusion3d_step(x, y, k0=G, k1=own + G, put=put, **kw)

        def seq(fn):
            def run():
                x, y = u, v
                for _ in range(a.steps):
                    fn(x, y)
                    x, y = y, x
            return run

        def timed(run):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            run()
            e1.record()
            e1.synchronize()
            return e0.elapsed_time(e1) * 1e3 / a.steps

        lib = _lib.require()

        def banded(fn):  # the same sequence with the banded z schedule forced
            def run():
                old = lib.advdiff_set_step_banded(1)
                try:
                    fn()
                finally:
                    lib.advdiff_set_step_banded(old)
            return run
        runs = {"split": seq(split), "whole": seq(whole), "put": seq(fused),
                "whole_banded": banded(seq(whole)), "put_banded": banded(seq(fused))}
        for _ in range(3):
            for r in runs.values():
                r()
        best = {k: 1e30 for k in runs}
        for _ in range(a.rounds):
            for k, r in runs.items():
                best[k] = min(best[k], timed(r))
        # the puts landed: the peer planes equal my boundary output planes (both schedules)
        w = torch.empty_like(u)
        stencil.diffusion3d_step(u, w, k0=G, k1=own + G, **kw)
        ok = True
        for m in (0, 1):
            peer.zero_()
            old = lib.advdiff_set_step_banded(m)
            stencil.diffusion3d_step(u, v, k0=G, k1=own + G, put=put, **kw)
            lib.advdiff_set_step_banded(old)
            torch.cuda.synchronize()
            i = (slice(None), slice(2, ny - 2), slice(2, nx - 2))  # the interior of a plane
            ok = (ok and torch.equal(v[G:own + G][i], w[G:own + G][i])
                  and torch.equal(peer[G + own:2 * G + own][i], w[G:2 * G][i])
                  and torch.equal(peer[0:G][i], w[own:own + G][i]))
        cells = nx * ny * own
        print(json.dumps({"ranks": n, "rank_block": [nx, ny, own],
                          **{f"{k}_us": round(t, 1) for k, t in best.items()},
                          **{f"{k}_mlups": round(cells / t, 1) for k, t in best.items()},
                          "put_vs_split": round(best["split"] / best["put"], 4),
                          "put_banded_vs_split": round(best["split"] / best["put_banded"], 4),
                          "puts_exact": bool(ok)}), flush=True)
        del u, v, peer, w
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
