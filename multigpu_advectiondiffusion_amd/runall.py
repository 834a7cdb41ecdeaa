"""Run the reference's canonical invocations (`*/run.sh`, `SingleGPU/RunAll.m`,
SURVEY.md Appendix A) through this framework and print their summary blocks — the
orchestration layer L6 (`Run.m` parameter files) as one command:

    python -m multigpu_advectiondiffusion_amd.runall [--quick] [--only diffusion3d] [--plot DIR]

`--quick` shrinks every grid/iteration count 8x for a smoke pass.
"""
from __future__ import annotations

import argparse
import os
import sys

# (label, app, positional args, extra flags) — reference file:line in the comment
CANONICAL = [
    # SingleGPU/Diffusion2d/run.sh:2  (C L W Nx Ny iters bx by)
    ("SG Diffusion2d", "diffusion2d", [1.0, 10.0, 10.0, 1001, 1001, 10000], ["--style", "singlegpu"]),
    # SingleGPU/Diffusion3d_*/run.sh:2
    ("SG Diffusion3d", "diffusion3d", [1.0, 10.0, 10.0, 10.0, 201, 199, 200, 605],
     ["--style", "singlegpu", "--error-norms"]),
    # SingleGPU/Burgers3d_WENO5/run.sh:2 (grid C of BASELINE.md) and grid B (512^3)
    ("SG Burgers3d 1000x1000x200", "burgers3d", [0.10, 0.30, 2.0, 2.0, 2.0, 1000, 1000, 200], []),
    ("SG Burgers3d 512^3", "burgers3d", [0.10, 0.30, 2.0, 2.0, 2.0, 512, 512, 512], []),
    # MultiGPU/*/run.sh (run here with as many ranks as launched)
    ("MG Diffusion3d", "diffusion3d", [1.0, 2.0, 2.0, 2.0, 400, 200, 200, 1000],
     ["--ic", "square", "--safety", "0.8"]),
    ("MG Burgers3d", "burgers3d", [0.40, 0.30, 2.0, 2.0, 4.0, 200, 200, 200],
     ["--weno", "js", "--viscosity", "0"]),
    ("MG Diffusion2d", "diffusion2d", [1.0, 2.0, 2.0, 400, 400, 1000], ["--ic", "disc", "--safety", "0.8"]),
    ("MG Burgers2d", "burgers2d", [0.40, 0.40, 2.0, 2.0, 400, 400], ["--weno", "js", "--viscosity", "0"]),
    # Matlab_Prototipes/InviscidBurgersNd/LFWENO7FDM{2,3}d.m: WENO7 + LSRK4(5), dt from max|u|
    ("MP Burgers2d WENO7", "burgers2d", [0.40, 0.40, 2.0, 2.0, 400, 400],
     ["--weno", "js7", "--integrator", "lsrk45", "--cfl-mode", "adaptive", "--viscosity", "0"]),
    ("MP Burgers3d WENO7", "burgers3d", [0.20, 0.40, 2.0, 2.0, 2.0, 160, 160, 160],
     ["--weno", "js7", "--integrator", "lsrk45", "--cfl-mode", "adaptive", "--viscosity", "0"]),
]


def _shrink(app, args):
    a = list(args)
    if app.startswith("diffusion"):
        ng = 2 if app == "diffusion2d" else 3
        for i in range(3 if app == "diffusion2d" else 4, 3 + ng + (1 if app == "diffusion3d" else 0)):
            a[i] = max(int(a[i]) // 8, 16)
        a[-1] = max(int(a[-1]) // 8, 4)
    else:
        ng = 2 if app == "burgers2d" else 3
        first = 4 if app == "burgers2d" else 5
        for i in range(first, first + ng):
            a[i] = max(int(a[i]) // 8, 16)
        a[0] = a[0] / 8
    return a


def main(argv=None) -> int:
    from . import cli
    ap = argparse.ArgumentParser()
    ap.add_argument("--quick", action="store_true")
    ap.add_argument("--only", default=None)
    ap.add_argument("--plot", default=None, help="directory for result PNGs")
    ap.add_argument("--device", default=None)
    ns = ap.parse_args(argv)
    rc = 0
    for label, app, args, extra in CANONICAL:
        if ns.only and ns.only not in (app, label):
            continue
        a = _shrink(app, args) if ns.quick else args
        argv2 = [app] + [str(x) for x in a] + list(extra)
        if ns.device:
            argv2 += ["--device", ns.device]
        out = None
        if ns.plot:
            os.makedirs(ns.plot, exist_ok=True)
            out = os.path.join(ns.plot, label.replace(" ", "_").replace("^", "") + ".bin")
            argv2 += ["--write", out]
        print(f"### {label}: {' '.join(argv2)}", flush=True)
        rc |= cli.main(argv2)
        if out and os.path.exists(out):
            from .utils.plot import plot_slices
            import numpy as np
            shape = [int(x) for x in (a[4:7] if app == "diffusion3d" else a[3:5] if app == "diffusion2d"
                                       else a[5:8] if app == "burgers3d" else a[4:6])]
            arr = np.fromfile(out, dtype=np.float32).reshape(tuple(reversed(shape)))
            plot_slices(arr, out[:-4] + ".png", label)
    return rc


if __name__ == "__main__":
    sys.exit(main())
