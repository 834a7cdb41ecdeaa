#!/usr/bin/env python3
"""fp32 vs fp64 3-D WENO5-Z viscous stage (v9): fp64, fp32 one cell per lane and fp32
packed z pairs (v_pk_* arithmetic, the default), interleaved rounds of back-to-back stage
launches; bitwise comparison of the two fp32 variants.

    python bench/burgers_fp32_ab.py [--sizes 256,512] [--rounds 4]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multigpu_advectiondiffusion_amd.ops import _lib, stencil  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="256,512")
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    lib = _lib.require()
    for n in (int(s) for s in a.sizes.split(",")):
        x = torch.linspace(0, 1, n, dtype=torch.float64, device="cuda")
        f64 = (torch.sin(5 * x.view(1, 1, -1) + 2 * x.view(1, -1, 1)) * torch.cos(3 * x.view(-1, 1, 1))
               + 0.5 * torch.tanh(30 * (x.view(1, 1, -1) - 0.4)))
        rd = n / 2.0
        v = 1e-5 * rd * rd
        kw = dict(nx=n, ny=n, k0=3, k1=n - 3, border=3, weno_z=True, rdx=rd, rdy=rd, rdz=rd,
                  vx=v, vy=v, vz=v, dt=1e-4, a=0.75, b=0.25)
        bufs = {"f64": [f64.clone(), f64.clone(), f64.clone()],
                "f32": [f64.float(), f64.float(), f64.float()]}
        variants = {"fp64": ("f64", 1), "fp32_scalar": ("f32", 0), "fp32_packed": ("f32", 1)}
        outs = {}
        for name, (key, pk) in variants.items():
            lib.advdiff_set_b3_pack(pk)
            i, u0, o = bufs[key]
            stencil.burgers3d_stage(i, u0, o, **kw)
            torch.cuda.synchronize()
            outs[name] = o.clone()
        same = torch.equal(outs["fp32_scalar"], outs["fp32_packed"])
        dev = (outs["fp32_packed"].double() - outs["fp64"]).abs().max().item()
        del outs
        best = {k: float("inf") for k in variants}
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for _ in range(a.rounds):
            for name, (key, pk) in variants.items():
                lib.advdiff_set_b3_pack(pk)
                i, u0, o = bufs[key]
                for _ in range(3):
                    stencil.burgers3d_stage(i, u0, o, **kw)
                s.record()
                for _ in range(a.reps):
                    stencil.burgers3d_stage(i, u0, o, **kw)
                e.record()
                torch.cuda.synchronize()
                best[name] = min(best[name], s.elapsed_time(e) * 1e3 / a.reps)
        lib.advdiff_set_b3_pack(1)
        cells = (n - 6) ** 3
        print(json.dumps({"n": n, "packed_bitwise_equal_scalar": same,
                          "fp32_vs_fp64_max_abs": dev,
                          **{f"{k}_us": round(t, 1) for k, t in best.items()},
                          **{f"{k}_mlups": round(cells / t, 1) for k, t in best.items()},
                          "packed_over_fp64": round(best["fp32_packed"] / best["fp64"], 3),
                          "scalar_over_fp64": round(best["fp32_scalar"] / best["fp64"], 3)}),
              flush=True)
        del bufs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
