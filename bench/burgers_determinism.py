#!/usr/bin/env python3
"""Bitwise reproducibility of the 3-D Burgers solver: the solution hash after 8 steps
(fp64 WENO5-Z + viscous, gaussian IC) for every (v9 tile row, forced z chunk, graph /
eager) combination, each repeated, in one process.  Separates the two ways a hash can
differ: run-to-run (the repeats of ONE configuration disagree: a race) and between
configurations (tile or chunk boundaries move the arithmetic).  Every hash of a shape
must be the same.

    python bench/burgers_determinism.py [--reps 2] [--shapes 256x256x256,...]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multigpu_advectiondiffusion_amd import Burgers, Grid, Solver  # noqa: E402
from multigpu_advectiondiffusion_amd.ops import _lib  # noqa: E402


def run_hash(shape, graph, dtype=torch.float64, steps=8):
    m = Burgers(viscosity=1e-5, weno="z", cfl=0.3)
    s = Solver(m, Grid(shape, (2.0, 2.0, 2.0)), dtype=dtype, ic="gaussian")
    s.run(iters=steps, dt=m.stable_dt(), graph=graph)
    h = s.bit_hash()
    del s
    torch.cuda.empty_cache()
    return h


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--shapes", default="256x256x256,512x512x64,96x80x70")
    ap.add_argument("--chunks", default="0,7,32")
    ap.add_argument("--dtype", default="float64")
    a = ap.parse_args()
    lib = _lib.require()
    dtype = getattr(torch, a.dtype)
    ok = True
    for sh in a.shapes.split(","):
        shape = tuple(int(v) for v in sh.split("x"))
        rec, racy = {}, []
        for tx in (64, 32):
            for zc in (int(c) for c in a.chunks.split(",")):
                for graph in (True, False):
                    old_tx, old_zc = lib.advdiff_set_b3_tx(tx), lib.advdiff_set_b3_zchunk(zc)
                    try:
                        hs = {run_hash(shape, graph, dtype) for _ in range(a.reps)}
                    finally:
                        lib.advdiff_set_b3_tx(old_tx)
                        lib.advdiff_set_b3_zchunk(old_zc)
                    key = f"tx{tx}_z{zc}_{'graph' if graph else 'eager'}"
                    rec[key] = sorted(hs)
                    if len(hs) > 1:
                        racy.append(key)
        allh = sorted({h for v in rec.values() for h in v})
        groups = {h: [k for k, v in rec.items() if h in v] for h in allh}
        ok &= len(allh) == 1
        print(json.dumps({"shape": shape, "dtype": a.dtype, "distinct_hashes": len(allh),
                          "run_to_run_differs": racy, "groups": groups}), flush=True)
    print("BITWISE_OK" if ok else "BITWISE_MISMATCH", flush=True)
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
