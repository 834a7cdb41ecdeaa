#!/usr/bin/env python3
"""Per-kernel timing of the fused stage kernels (HIP events, interleaved repetitions).

    python bench/kernels.py [--n 512] [--reps 20]

Prints time per stage kernel and the effective HBM bandwidth implied by the minimum
traffic (stage 1: read in + write out = 16 B/cell; stages 2/3: + read u0 = 24 B/cell).
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multigpu_advectiondiffusion_amd.ops import stencil  # noqa: E402


def timeit(fn, reps):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(reps):
        e0.record()
        fn()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e-3)
    ts.sort()
    return ts[len(ts) // 2], ts[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=512)
    ap.add_argument("--nb", type=int, default=256)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--dtype", default="fp64")
    args = ap.parse_args()
    dt = torch.float64 if args.dtype == "fp64" else torch.float32
    es = torch.empty((), dtype=dt).element_size()
    n = args.n
    res = {}
    u = torch.rand((n, n, n), dtype=dt, device="cuda")
    A = torch.rand_like(u)
    B = torch.rand_like(u)
    cells = n ** 3
    for order in (4, 2):
        R = order // 2
        kw = dict(nx=n, ny=n, k0=R, k1=n - R, border=R, order=order, cx=1.0, cy=1.0, cz=1.0,
                  dt=0.01)
        t1, t1m = timeit(lambda: stencil.diffusion3d_stage(u, None, A, a=0.0, b=1.0, **kw), args.reps)
        t2, t2m = timeit(lambda: stencil.diffusion3d_stage(A, u, B, a=0.75, b=0.25, **kw), args.reps)
        res[f"diffusion3d_fd{order}_stage1_us"] = round(t1 * 1e6, 1)
        res[f"diffusion3d_fd{order}_stage23_us"] = round(t2 * 1e6, 1)
        res[f"diffusion3d_fd{order}_stage1_TBps"] = round(2 * es * cells / t1 / 1e12, 2)
        res[f"diffusion3d_fd{order}_stage23_TBps"] = round(3 * es * cells / t2 / 1e12, 2)
        res[f"diffusion3d_fd{order}_step_mlups"] = round(cells / (t1 + 2 * t2) / 1e6, 1)
    for order in (4, 2):
        R = order // 2
        kw = dict(nx=n, ny=n, k0=R, k1=n - R, zlo=R, zhi=n - R, border=R, order=order,
                  cx=1.0, cy=1.0, cz=1.0, dt=0.01)
        tf, _ = timeit(lambda: stencil.diffusion3d_step(u, A, **kw), args.reps)
        res[f"diffusion3d_fd{order}_fused_step_us"] = round(tf * 1e6, 1)
        res[f"diffusion3d_fd{order}_fused_step_mlups"] = round(cells / tf / 1e6, 1)
        res[f"diffusion3d_fd{order}_fused_TBps_eff"] = round(2 * es * cells / tf / 1e12, 2)
        # exclusive launch: one round of persistent groups (single-rank production path)
        tp, _ = timeit(lambda: stencil.diffusion3d_step(u, A, exclusive=True, **kw), args.reps)
        res[f"diffusion3d_fd{order}_fused_persist_us"] = round(tp * 1e6, 1)
        res[f"diffusion3d_fd{order}_fused_persist_mlups"] = round(cells / tp / 1e6, 1)
    # copy roofline for reference: B <- A (16 B/cell)
    tc, _ = timeit(lambda: B.copy_(A), args.reps)
    res["copy_TBps"] = round(2 * es * cells / tc / 1e12, 2)
    del u, A, B
    nb = args.nb
    u = torch.rand((nb, nb, nb), dtype=dt, device="cuda") * 0.5 + 0.1
    A = torch.rand_like(u)
    B = torch.rand_like(u)
    for wz in ("z", "js", "js7"):
        for visc in (1e-5, 0.0):
            R = 4 if wz == "js7" else 3
            kw = dict(nx=nb, ny=nb, k0=R, k1=nb - R, border=R, weno_z=wz, rdx=nb / 2.0,
                      rdy=nb / 2.0, rdz=nb / 2.0, vx=visc * (nb / 2.0) ** 2,
                      vy=visc * (nb / 2.0) ** 2, vz=visc * (nb / 2.0) ** 2, dt=1e-4)
            t2, _ = timeit(lambda: stencil.burgers3d_stage(A, u, B, a=0.75, b=0.25, **kw), args.reps)
            tag = f"burgers3d_{wz}_{'visc' if visc else 'inv'}"
            res[tag + "_stage_us"] = round(t2 * 1e6, 1)
            res[tag + "_step_mlups"] = round(nb ** 3 / (3 * t2) / 1e6, 1)
            if wz == "js7":  # low-storage RK4(5) stage (5 per step)
                tl, _ = timeit(lambda: stencil.burgers3d_stage(A, u, B, a=-0.4, b=0.3, ls=True,
                                                               **kw), args.reps)
                res[tag + "_ls_stage_us"] = round(tl * 1e6, 1)
                res[tag + "_lsrk45_step_mlups"] = round(nb ** 3 / (5 * tl) / 1e6, 1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
