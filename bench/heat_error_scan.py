#!/usr/bin/env python3
"""Error of the 3-D heat solver vs the exact decaying sine mode, per grid size and
execution path (fused step / per-stage kernels / PyTorch reference ops), with the
location of the max error — the bench's self-validation check, dissected.

    python bench/heat_error_scan.py [--sizes 128,256,512] [--steps 25]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multigpu_advectiondiffusion_amd import Diffusion, Grid, Solver  # noqa: E402
from multigpu_advectiondiffusion_amd.utils import ics  # noqa: E402
import bench as B  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="128,256,512")
    ap.add_argument("--steps", type=int, default=25)
    ap.add_argument("--paths", default="fused,stage,torch")
    ap.add_argument("--order", type=int, default=4)
    ap.add_argument("--graph", type=int, default=-1)
    args = ap.parse_args()
    dev = "cuda" if torch.cuda.is_available() else "cpu"
    for n in [int(s) for s in args.sizes.split(",")]:
        g = Grid((n, n, n), (1.0, 1.0, 1.0))
        for path in args.paths.split(","):
            m = Diffusion(K=1.0, order=args.order)
            kw = dict(fused=(path == "fused"), kernel=("torch" if path == "torch" else "native"))
            s = Solver(m, g, dtype=torch.float64, device=dev, ic="sine", **kw)
            dt = m.stable_dt()
            s.run(iters=args.steps, dt=dt, graph=None if args.graph < 0 else bool(args.graph))
            _, _, li = s.error_norms()
            u = s.owned
            ex = ics.exact_solution_box("sine", g.shape, g.spacing, s.t, 1.0, None, [0, 0, 0],
                                        [n, n, n], n, torch.float64, dev)
            e = (u - ex).abs()
            idx = int(e.argmax())
            loc = (idx // (n * n), (idx // n) % n, idx % n)
            print(json.dumps({"n": n, "path": path, "order": args.order, "t": s.t,
                              "linf": li, "linf_direct": float(e.max()), "argmax_zyx": loc,
                              "bound": B.linf_bound(g, 1.0, s.t, args.order)}), flush=True)
            del s, u, ex, e
            if dev == "cuda":
                torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
