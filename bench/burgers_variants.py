#!/usr/bin/env python3
"""A/B of the 3-D WENO5 stage kernel variants (burgers.hip: advdiff_set_b3_ver / _ty) at
production size, interleaved round by round so clock/thermal drift hits all alike:
median HIP-event time per launch, and the max deviation of each variant's output from
the fp64 PyTorch reference of the same stage (ops/reference.py) on a smaller grid.

    python bench/burgers_variants.py [--n 256] [--reps 20] [--rounds 5]
        [--variants 1:8,2:8,2:16,3:8,3:16]
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multigpu_advectiondiffusion_amd.ops import _lib, reference, stencil  # noqa: E402


def stage_kw(n, wz, visc):
    v = visc * (n / 2.0) ** 2
    return dict(nx=n, ny=n, k0=3, k1=n - 3, border=3, weno_z=wz, rdx=n / 2.0, rdy=n / 2.0,
                rdz=n / 2.0, vx=v, vy=v, vz=v, dt=1e-4, a=0.75, b=0.25)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=256)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--variants", default="1:8,2:8,2:16,3:8,3:16")
    ap.add_argument("--check-n", type=int, default=72)
    a = ap.parse_args()
    lib = _lib.require()
    variants = [tuple(int(x) for x in v.split(":")) for v in a.variants.split(",")]

    def select(ver, ty):
        lib.advdiff_set_b3_ver(ver)
        lib.advdiff_set_b3_ty(ty)

    out = {}
    # ---- numerics vs the fp64 reference (smaller grid, shock-like data) -------------
    m = a.check_n
    g = torch.Generator().manual_seed(0)
    x = torch.linspace(0, 1, m, dtype=torch.float64)
    base = (torch.sin(6 * x.view(1, 1, -1) + 3 * x.view(1, -1, 1)) * torch.cos(4 * x.view(-1, 1, 1))
            + 0.5 * torch.tanh(40 * (x.view(1, 1, -1) - 0.5)))
    uin = base + 0.05 * torch.rand((m, m, m), generator=g, dtype=torch.float64)
    u0 = torch.rand((m, m, m), generator=g, dtype=torch.float64)
    for wz in (True, False):
        kw = stage_kw(m, wz, 1e-3)
        exp = u0.clone()
        reference.burgers3d_stage(uin, u0, exp, m, m, 3, m - 3, 3, wz, kw["rdx"], kw["rdy"],
                                  kw["rdz"], kw["vx"], kw["vy"], kw["vz"], kw["dt"], kw["a"],
                                  kw["b"])
        for ver, ty in variants:
            select(ver, ty)
            gi, g0 = uin.cuda(), u0.cuda()
            go = g0.clone()
            stencil.burgers3d_stage(gi, g0, go, **kw)
            torch.cuda.synchronize()
            err = (go.cpu() - exp).abs().max().item()
            out[f"err_v{ver}_ty{ty}_wz{int(wz)}"] = err
            print(f"v{ver} ty{ty} wz{int(wz)} max|err| vs fp64 ref = {err:.3e}", flush=True)

    # ---- timing -----------------------------------------------------------------------
    n = a.n
    u = torch.rand((n, n, n), dtype=torch.float64, device="cuda") * 0.5 + 0.1
    o = torch.rand_like(u)
    for wz, visc in ((True, 1e-5), (False, 1e-5), (True, 0.0)):
        kw = stage_kw(n, wz, visc)
        ts = {v: [] for v in variants}
        for _ in range(a.rounds):
            for v in variants:
                select(*v)
                for _ in range(2):
                    stencil.burgers3d_stage(u, u, o, **kw)
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.reps):
                    stencil.burgers3d_stage(u, u, o, **kw)
                e1.record()
                e1.synchronize()
                ts[v].append(e0.elapsed_time(e1) * 1e3 / a.reps)
        for v in variants:
            us = statistics.median(ts[v])
            tag = f"v{v[0]}_ty{v[1]}_wz{int(wz)}_visc{visc:g}"
            out[tag] = {"us": round(us, 1), "stage_mlups": round(n ** 3 / us, 1),
                        "min_us": round(min(ts[v]), 1)}
            print(tag, out[tag], flush=True)
    select(2, 8)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
