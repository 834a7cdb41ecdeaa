#!/usr/bin/env python3
"""Bitwise reproducibility of the 3-D Burgers solver: the solution hash after 8 steps
(fp64 WENO5-Z + viscous, gaussian IC) for repeated runs of each v9 tile shape and a
forced z chunk, in one process.  Every hash of a shape must be the same.

    python bench/burgers_determinism.py [--reps 3]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multigpu_advectiondiffusion_amd import Burgers, Grid, Solver  # noqa: E402
from multigpu_advectiondiffusion_amd.ops import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--shapes", default="256x256x256,512x512x64,96x80x70")
    a = ap.parse_args()
    lib = _lib.require()
    for sh in a.shapes.split(","):
        shape = tuple(int(v) for v in sh.split("x"))
        rec = {}
        for tx in (64, 32):
            for graph in (True, False):
                hs = []
                for _ in range(a.reps):
                    old = lib.advdiff_set_b3_tx(tx)
                    try:
                        m = Burgers(viscosity=1e-5, weno="z", cfl=0.3)
                        s = Solver(m, Grid(shape, (2.0, 2.0, 2.0)), dtype=torch.float64,
                                   ic="gaussian")
                        dt = m.stable_dt()
                        s.run(iters=8, dt=dt, graph=graph)
                        hs.append(s.bit_hash())
                        del s
                        torch.cuda.empty_cache()
                    finally:
                        lib.advdiff_set_b3_tx(old)
                rec[f"tx{tx}_{'graph' if graph else 'eager'}"] = sorted(set(hs))
        allh = set(h for v in rec.values() for h in v)
        print(json.dumps({"shape": shape, "distinct_hashes": len(allh), **rec}), flush=True)


if __name__ == "__main__":
    main()
