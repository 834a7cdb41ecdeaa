#!/usr/bin/env python3
"""Compute-side cost of the multi-GPU overlap split for the fused heat step, measured on
one GPU (no communication): a rank's slab of the 8-GPU weak-scaling run (1024² x 128
planes + 3R ghosts each side) stepped as
  (a) one launch over all owned planes (what 1 GPU would do),
  (b) interior launch + two boundary launches (3R planes each),
  (c) interior launch + ONE launch for both boundary slabs (advdiff_diffusion3d_step2).
(b)/(c) minus (a) is the price of hiding the halo exchange behind the interior.

    python bench/split_overhead.py [--n 1024] [--planes 128] [--reps 20]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multigpu_advectiondiffusion_amd.ops import stencil  # noqa: E402


def timeit(fn, reps):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3  # µs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1024)
    ap.add_argument("--planes", type=int, default=128)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    R = 2
    G = 3 * R
    nz = a.planes + 2 * G
    u = torch.rand((nz, a.n, a.n), dtype=torch.float64, device="cuda")
    v = torch.empty_like(u)
    kw = dict(nx=a.n, ny=a.n, zlo=0, zhi=nz, border=R, order=4, cx=1.0, cy=1.0, cz=1.0,
              dt=0.01)
    o0, o1 = G, G + a.planes

    def full():
        stencil.diffusion3d_step(u, v, k0=o0, k1=o1, **kw)

    def split2():
        stencil.diffusion3d_step(u, v, k0=o0 + G, k1=o1 - G, **kw)
        stencil.diffusion3d_step(u, v, k0=o0, k1=o0 + G, **kw)
        stencil.diffusion3d_step(u, v, k0=o1 - G, k1=o1, **kw)

    def split1():
        stencil.diffusion3d_step(u, v, k0=o0 + G, k1=o1 - G, **kw)
        stencil.diffusion3d_step(u, v, k0=o0, k1=o0 + G, k0b=o1 - G, k1b=o1, **kw)

    def interior():
        stencil.diffusion3d_step(u, v, k0=o0 + G, k1=o1 - G, **kw)

    lo_pri, hi_pri = torch.cuda.Stream.priority_range()
    side = torch.cuda.Stream(priority=hi_pri)

    def split_conc():  # (d) the boundary launch on a high-priority stream BESIDE the interior
        cur = torch.cuda.current_stream()
        side.wait_stream(cur)
        stencil.diffusion3d_step(u, v, k0=o0 + G, k1=o1 - G, **kw)
        with torch.cuda.stream(side):
            stencil.diffusion3d_step(u, v, k0=o0, k1=o0 + G, k0b=o1 - G, k1b=o1, **kw)
        cur.wait_stream(side)

    def split_conc_first():  # (e) boundary first (on the side stream), interior behind it
        cur = torch.cuda.current_stream()
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            stencil.diffusion3d_step(u, v, k0=o0, k1=o0 + G, k0b=o1 - G, k1b=o1, **kw)
        stencil.diffusion3d_step(u, v, k0=o0 + G, k1=o1 - G, **kw)
        cur.wait_stream(side)

    def boundary1():
        stencil.diffusion3d_step(u, v, k0=o0, k1=o0 + G, k0b=o1 - G, k1b=o1, **kw)

    res = {"slab": [a.n, a.n, a.planes], "ghost": G}
    for name, fn in (("full_us", full), ("interior_us", interior),
                     ("boundary_merged_us", boundary1), ("split_3_launches_us", split2),
                     ("split_2_launches_us", split1), ("split_concurrent_us", split_conc),
                     ("split_concurrent_bfirst_us", split_conc_first)):
        res[name] = round(timeit(fn, a.reps), 1)
    res["overhead_3_launches_pct"] = round(100 * (res["split_3_launches_us"] / res["full_us"] - 1), 1)
    res["overhead_2_launches_pct"] = round(100 * (res["split_2_launches_us"] / res["full_us"] - 1), 1)
    res["overhead_concurrent_pct"] = round(100 * (res["split_concurrent_us"] / res["full_us"] - 1), 1)
    res["overhead_concurrent_bfirst_pct"] = round(
        100 * (res["split_concurrent_bfirst_us"] / res["full_us"] - 1), 1)
    print(json.dumps(res))




def cartesian(pgrid=(4, 2, 1), n=1024, reps=10, rank=None):
    """Same measurement for one block of a Cartesian 8-GPU decomposition of n^3 (fused
    kernel on views, 3R ghosts on split axes): full block launch vs interior + boundary
    boxes.  No communication (a stand-in Comm with the block's rank)."""
    from multigpu_advectiondiffusion_amd import Diffusion, Grid, Solver
    from multigpu_advectiondiffusion_amd.parallel.comm import Comm
    size = pgrid[0] * pgrid[1] * pgrid[2]
    rank = size // 2 if rank is None else rank  # an interior-ish block
    comm = Comm(rank=rank, size=size, device="cuda:0")
    s = Solver(Diffusion(K=1.0, order=4), Grid((n, n, n), (1.0, 1.0, 1.0)), comm,
               dtype=torch.float64, ic="sine", decomp=pgrid)
    assert s.cart and s.fused
    dt = s.model.stable_dt()
    res = {"pgrid": list(pgrid), "block": [c for _, c in s.cd.global_box()],
           "boundary_boxes": len(s.boundary)}
    res["full_us"] = round(timeit(lambda: s._launch_fused_box(s.full, dt), reps), 1)
    res["interior_us"] = round(timeit(lambda: s._launch_fused_box(s.interior, dt), reps), 1)

    def bnd():
        for b in s.boundary:
            s._launch_fused_box(b, dt)
    res["boundary_us"] = round(timeit(bnd, reps), 1)
    res["overhead_pct"] = round(100 * ((res["interior_us"] + res["boundary_us"]) / res["full_us"] - 1), 1)
    print(json.dumps(res))


if __name__ == "__main__":
    if "--cart" in sys.argv:
        for pg in ((4, 2, 1), (2, 2, 2), (2, 4, 1)):
            cartesian(pg)
    else:
        main()
