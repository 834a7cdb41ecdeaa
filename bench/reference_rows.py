#!/usr/bin/env python3
"""Re-measure every published reference row on this framework, same grid and
physics, one MI355X, fp64.  MLUPS = cells x RK3 steps / s (the reference's GFLOPs were
converted to MLUPS in BASELINE.md the same way).  Steps are capped so the whole table runs
in about a minute; throughput does not depend on the step count once warm.

    python bench/reference_rows.py [--md profiles/reference_rows.md]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multigpu_advectiondiffusion_amd import Burgers, Diffusion, Grid, Solver  # noqa: E402

# (label, reference MLUPS, reference source, model factory, grid, lengths, ic, steps)
ROWS = [
    ("SG Diffusion-2D FD4 1001^2", 893.8, "SingleGPU/Diffusion2d_PitchedMem/Run.m:3-12",
     lambda: Diffusion(K=1.0, order=4), (1001, 1001), (10.0, 10.0), "heat", 2000),
    ("SG Diffusion-3D FD4 201x199x200", 927.2, "SingleGPU/Diffusion3d_Blocking/Run.m:3-12",
     lambda: Diffusion(K=1.0, order=4), (201, 199, 200), (10.0, 10.0, 10.0), "heat", 605),
    ("MG Diffusion-3D FD4 400x200x206 (ref: 2 GPUs)", 244.7, "MultiGPU/Diffusion3d_Baseline/Run.m:4-14",
     lambda: Diffusion(K=1.0, order=4, safety=0.8), (400, 200, 206), (2.0, 2.0, 2.0), "square", 300),
    ("MG Diffusion-2D FD4 400x406 (ref: 2 GPUs)", 255.5, "MultiGPU/Diffusion2d_Baseline/Run.m:4-14",
     lambda: Diffusion(K=1.0, order=4, safety=0.8), (400, 406), (2.0, 2.0), "disc", 1001),
    ("SG Burgers-3D WENO5-Z visc 512^3", 344.4, "SingleGPU/Burgers3d_WENO5_PitchedMem/Run.m:15-25",
     lambda: Burgers(viscosity=1e-5, weno="z", cfl=0.3), (512, 512, 512), (2.0, 2.0, 2.0), "gaussian", 20),
    ("SG Burgers-3D WENO5-Z visc 1000x1000x200", 139.1, "SingleGPU/Burgers3d_WENO5_PitchedMem/Run.m:27-37",
     lambda: Burgers(viscosity=1e-5, weno="z", cfl=0.3), (1000, 1000, 200), (2.0, 2.0, 2.0), "gaussian", 20),
    ("SG Burgers-3D WENO5-Z visc 1601x986x35", 107.2, "SingleGPU/Burgers3d_WENO5_PitchedMem/Run.m:3-13",
     lambda: Burgers(viscosity=1e-5, weno="z", cfl=0.3), (1601, 986, 35), (2.0, 2.0, 2.0), "gaussian", 40),
    ("MG Burgers-3D WENO5-JS 400x400x406 (ref: 2 GPUs)", 12.6, "MultiGPU/Burgers3d_Baseline/Run.m:4-14",
     lambda: Burgers(viscosity=0.0, weno="js", cfl=0.3), (400, 400, 406), (2.0, 2.0, 4.0), "gaussian", 30),
    ("MG Burgers-2D WENO5-JS 400x406 (ref: 2 GPUs)", 5.2, "MultiGPU/Burgers2d_Baseline/Run.m:4-14",
     lambda: Burgers(viscosity=0.0, weno="js", cfl=0.4), (400, 406), (2.0, 2.0), "gaussian", 200),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--md", default=None)
    ap.add_argument("--scale", type=float, default=1.0, help="step-count multiplier")
    ap.add_argument("--only", default=None, help="substring filter on the case label")
    a = ap.parse_args()
    out = []
    for label, ref, src, mk, shape, lengths, ic, steps in ROWS:
        if a.only and a.only not in label:
            continue
        model = mk()
        s = Solver(model, Grid(shape, lengths), dtype=torch.float64, device="cuda", ic=ic)
        n = max(int(steps * a.scale), 8)
        s.run(iters=min(n, 16))  # warm-up (+ graph capture)
        st = s.run(iters=n)
        cells = s.grid.cells
        ml = cells * n / st.compute_s / 1e6
        row = {"case": label, "ref_mlups": ref, "mlups": round(ml, 1),
               "speedup": round(ml / ref, 1), "steps": n, "s": round(st.compute_s, 4),
               "fused": bool(getattr(s, "fused", False)), "source": src}
        out.append(row)
        print(json.dumps(row), flush=True)
        del s
        torch.cuda.empty_cache()
    if a.md:
        with open(a.md, "w") as f:
            f.write("| case | reference MLUPS | this framework MLUPS (1 MI355X, fp64) | speed-up | reference source |\n")
            f.write("|---|---|---|---|---|\n")
            for r in out:
                f.write(f"| {r['case']} | {r['ref_mlups']} | {r['mlups']} | {r['speedup']}x | `{r['source']}` |\n")
        print("wrote", a.md)


if __name__ == "__main__":
    main()
