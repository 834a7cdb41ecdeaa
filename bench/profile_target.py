#!/usr/bin/env python3
"""Run ONE stencil kernel repeatedly (for rocprofv3 --pmc / --kernel-trace).

    python bench/profile_target.py {fused,fused2,step2x,stage,burgers,burgers512,copy} [--n 512]
        [--reps 5]
        [--pitch PX,PY]   (fields of (n, n + PY, n + PX): the solver's pitched layout)

Per-rank shapes of the 8-GPU weak-scaling run (FD4 fused step, round 6):
  slab8_int / slab8_bnd  the z-slab rank (1024 x 1024 x 128 owned + 2 x 6 ghost planes):
                         its interior launch (116 planes) / its two 6-plane boundary slabs
                         in one launch
  r4x2_int               the 4 x 2 x 1 Cartesian rank's interior launch (1024 x 512 x 256
                         owned, ghosts on z and y)
  cube1024               one launch over 1024^3
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multigpu_advectiondiffusion_amd.ops import stencil  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("which", choices=["fused", "fused2", "step2x", "stage", "burgers", "burgers_js",
                                  "burgers512",
                                  "copy", "slab8_int", "slab8_bnd", "r4x2_int", "cube1024"])
ap.add_argument("--n", type=int, default=512)
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--pitch", default="0,0")
a = ap.parse_args()
n = (a.n if a.which in ("fused", "fused2", "step2x", "stage", "copy") else
     512 if a.which == "burgers512" else min(a.n, 256))
px, py = (int(v) for v in a.pitch.split(","))
RANK = {"slab8_int": ((140, 1024, 1024), dict(k0=12, k1=128, zlo=0, zhi=140)),
        "slab8_bnd": ((140, 1024, 1024), dict(k0=6, k1=12, k0b=128, k1b=134, zlo=0, zhi=140)),
        "r4x2_int": ((268, 518, 1024), dict(k0=12, k1=256, zlo=0, zhi=268)),
        "cube1024": ((1024, 1024, 1024), dict(k0=2, k1=1022, zlo=2, zhi=1022))}
shape = RANK[a.which][0] if a.which in RANK else (n, n, n)
u = torch.rand((shape[0], shape[1] + py, shape[2] + px), dtype=torch.float64,
               device="cuda") * 0.5 + 0.1
o = torch.rand_like(u)
for _ in range(a.reps):
    if a.which in RANK:
        stencil.diffusion3d_step(u, o, nx=shape[2], ny=shape[1], border=2, order=4, cx=1.0,
                                 cy=1.0, cz=1.0, dt=0.01, **RANK[a.which][1])
    elif a.which == "copy":  # calibration: exactly n^3 x 8 B read and written
        stencil.copy_box(o, u, n, n, n)
    elif a.which in ("fused", "fused2"):
        R = 2 if a.which == "fused" else 1
        stencil.diffusion3d_step(u, o, nx=n, ny=n, k0=R, k1=n - R, zlo=R, zhi=n - R, border=R,
                                 order=2 * R, cx=1.0, cy=1.0, cz=1.0, dt=0.01)
    elif a.which == "step2x":  # two FD2 steps per launch (the bench's 512^3 shape)
        stencil.diffusion3d_step2x(u, o, nx=n, ny=n, k0=1, k1=n - 1, zlo=1, zhi=n - 1, border=1,
                                   cx=1.0, cy=1.0, cz=1.0, dt=0.01)
    elif a.which == "stage":
        stencil.diffusion3d_stage(u, u, o, nx=n, ny=n, k0=2, k1=n - 2, border=2, order=4, cx=1.0,
                                  cy=1.0, cz=1.0, dt=0.01, a=0.75, b=0.25)
    else:
        stencil.burgers3d_stage(u, u, o, nx=n, ny=n, k0=3, k1=n - 3, border=3,
                                weno_z=a.which != "burgers_js", rdx=n / 2.0, rdy=n / 2.0,
                                rdz=n / 2.0, vx=1e-5 * n * n / 4, vy=1e-5 * n * n / 4,
                                vz=1e-5 * n * n / 4, dt=1e-4, a=0.75, b=0.25)
torch.cuda.synchronize()
print("done", a.which)
