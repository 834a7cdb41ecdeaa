#!/usr/bin/env python3
"""Every hot kernel once per rep, at production size, with known analytic HBM traffic —
the target of the roofline PMC passes (scripts/roofline.sh) and of a kernel-trace run.

    python bench/roofline_targets.py [--reps 3] [--n 512] [--nb 256]

Kernels (fp64) and their compulsory traffic per cell:
  copy_box   (aux.hip)              read 8 + write 8          = 16 B
  stage1     (diffusion.hip, a = 0)  read u 8 + write 8        = 16 B
  stage2     (diffusion.hip, a > 0)  read u, u0 16 + write 8   = 24 B
  fused_fd4 / fused_fd2 (diffusion_fused.hip, one RK3 step)    = 16 B
  weno5_stage (burgers.hip, a > 0, 256^3)                      = 24 B
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
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--n", type=int, default=512)
    ap.add_argument("--nb", type=int, default=256)
    ap.add_argument("--only", default=None)
    a = ap.parse_args()
    n, nb = a.n, a.nb
    u = torch.rand((n, n, n), dtype=torch.float64, device="cuda") * 0.5 + 0.1
    v = torch.rand_like(u)
    w = torch.rand_like(u)
    kw = dict(nx=n, ny=n, border=2, order=4, cx=1.0, cy=1.0, cz=1.0, dt=0.01)
    ub = u[:nb, :nb, :nb].contiguous()
    vb = torch.rand_like(ub)
    wb = torch.rand_like(ub)
    targets = {
        "copy_box": (lambda: stencil.copy_box(v, u, n, n, n), n ** 3, 16),
        "stage1": (lambda: stencil.diffusion3d_stage(u, u, v, k0=2, k1=n - 2, a=0.0, b=1.0,
                                                     **kw), (n - 4) ** 3, 16),
        "stage2": (lambda: stencil.diffusion3d_stage(u, w, v, k0=2, k1=n - 2, a=0.75, b=0.25,
                                                     **kw), (n - 4) ** 3, 24),
        "fused_fd4": (lambda: stencil.diffusion3d_step(u, v, k0=2, k1=n - 2, zlo=2, zhi=n - 2,
                                                       **kw), (n - 4) ** 3, 16),
        "fused_fd2": (lambda: stencil.diffusion3d_step(u, v, k0=1, k1=n - 1, zlo=1, zhi=n - 1,
                                                       **dict(kw, border=1, order=2)),
                      (n - 2) ** 3, 16),
        "weno5_stage": (lambda: stencil.burgers3d_stage(
            ub, wb, vb, nx=nb, ny=nb, k0=3, k1=nb - 3, border=3, weno_z=True, rdx=nb / 2.0,
            rdy=nb / 2.0, rdz=nb / 2.0, vx=1e-5 * nb * nb / 4, vy=1e-5 * nb * nb / 4,
            vz=1e-5 * nb * nb / 4, dt=1e-4, a=0.75, b=0.25), (nb - 6) ** 3, 24),
    }
    meta = {}
    for name, (fn, cells, bpc) in targets.items():
        if a.only and name not in a.only.split(","):
            continue
        for _ in range(a.reps):
            fn()
        torch.cuda.synchronize()
        meta[name] = {"cells": cells, "bytes_per_cell": bpc}
    print(json.dumps(meta))


if __name__ == "__main__":
    main()
