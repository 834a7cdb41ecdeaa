#!/usr/bin/env python3
"""A/B of WENO5 v9 launch variants on the 3-D viscous Burgers stage, fp64, in the solver
(hipGraph-replayed steps): cubes and the per-rank blocks of the multi-GPU Burgers configs.
Variants are environment knobs (read once per process), so every variant runs in its own
child process; rounds alternate the variants (clock drift).  Bitwise: the solution after
a fixed 8 steps must be the same for every variant.

    python bench/burgers_tile_ab.py [--rounds 3] [--variants "B3_TX=64 B3_TX=32 B3_TX=0"]
"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHAPES = [(256, 256, 256), (384, 384, 384), (512, 512, 512), (512, 512, 64),
          (1024, 1024, 64), (1000, 1000, 200)]

CHILD = r'''
import json, sys, time, torch
sys.path.insert(0, %r)
from multigpu_advectiondiffusion_amd import Burgers, Grid, Solver
out = []
for shape in %r:
    m = Burgers(viscosity=1e-5, weno="z", cfl=0.3)
    s = Solver(m, Grid(shape, (2.0, 2.0, 2.0)), dtype=torch.float64, ic="gaussian")
    dt = m.stable_dt()
    s.run(iters=8, dt=dt)
    h = s.bit_hash()
    t0 = time.perf_counter(); s.run(iters=8, dt=dt); per = (time.perf_counter() - t0) / 8
    steps = max(16, int(0.06 / per) // 8 * 8)
    s.run(iters=steps, dt=dt)
    st = s.run(iters=steps, dt=dt)
    ms = st.compute_s / steps * 1e3
    cells = shape[0] * shape[1] * shape[2]
    out.append({"shape": list(shape), "ms": round(ms, 4), "mlups": round(cells / ms / 1e3, 1),
                "hash": h})
    del s; torch.cuda.empty_cache()
print(json.dumps(out))
'''


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--variants", default="B3_TX=64 B3_TX=32 B3_TX=0")
    a = ap.parse_args()
    variants = a.variants.split()
    best = {}
    hashes = {}
    for r in range(a.rounds):
        for var in variants:
            env = dict(os.environ)
            for kv in var.split(","):
                k, v = kv.split("=")
                env["ADVDIFF_" + k] = v
            res = subprocess.run([sys.executable, "-c", CHILD % (ROOT, SHAPES)], env=env,
                                 capture_output=True, text=True, check=True, timeout=600)
            for rec in json.loads(res.stdout.strip().splitlines()[-1]):
                key = (tuple(rec["shape"]), var)
                best[key] = max(best.get(key, 0.0), rec["mlups"])
                hashes.setdefault(tuple(rec["shape"]), {}).setdefault(var, []).append(rec["hash"])
            print(f"round {r} variant {var} done", flush=True)
    for shape in SHAPES:
        per = hashes[tuple(shape)]  # variant -> hash of every round (one process each)
        allh = {h for hs in per.values() for h in hs}
        print(json.dumps({"shape": shape, **{f"mlups[{v}]": best[(tuple(shape), v)]
                                             for v in variants},
                          "bitwise_equal": len(allh) == 1,
                          "hashes_per_variant": {v: hs for v, hs in per.items()}}), flush=True)


if __name__ == "__main__":
    main()
