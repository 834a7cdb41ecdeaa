#!/usr/bin/env python3
"""fp32 fused heat step: tile A/B (advdiff_set_step_f32_tile 0 = the fp64 shapes, 3 / 4 =
16 waves x 3 / 4 rows; default 0) at each --n, interleaved rounds of back-to-back launches after a
settling run, bitwise comparison of one step across the tiles.  Effective TB/s = the
step's compulsory 8 B/cell (read u^n + write u^{n+1}, fp32) / time.

    python bench/step_fp32_ab.py [--n 512 384 ...] [--rounds 4]
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
    ap.add_argument("--n", type=int, nargs="+", default=[512])
    ap.add_argument("--rounds", type=int, default=4)
    a = ap.parse_args()
    lib = _lib.require()
    default = lib.advdiff_set_step_f32_tile(0)
    for n, order in [(n, o) for n in a.n for o in (4, 2)]:
        R = order // 2
        u = torch.rand((n, n, n), dtype=torch.float32, device="cuda")
        v = torch.zeros_like(u)
        kw = dict(nx=n, ny=n, k0=R, k1=n - R, zlo=R, zhi=n - R, border=R, order=order,
                  cx=1.0, cy=1.0, cz=1.0, dt=0.01)
        outs = {}
        for t in (0, 3, 4):
            lib.advdiff_set_step_f32_tile(t)
            v.zero_()
            stencil.diffusion3d_step(u, v, **kw)
            torch.cuda.synchronize()
            outs[t] = v.clone()
        same = all(torch.equal(outs[0], outs[t]) for t in (3, 4))
        del outs
        best = {t: float("inf") for t in (0, 3, 4)}
        pair = [u, v]

        def fn():
            stencil.diffusion3d_step(pair[0], pair[1], **kw)
            pair.reverse()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        lib.advdiff_set_step_f32_tile(default)
        for _ in range(60):
            fn()
        for _ in range(a.rounds):
            for t in (0, 3, 4):
                lib.advdiff_set_step_f32_tile(t)
                for _ in range(4):
                    fn()
                s.record()
                for _ in range(16):
                    fn()
                e.record()
                torch.cuda.synchronize()
                best[t] = min(best[t], s.elapsed_time(e) * 1e3 / 16)
        lib.advdiff_set_step_f32_tile(default)
        cells = (n - 2 * R) ** 3
        print(json.dumps({"order": order, "n": n, "bitwise_equal_across_tiles": same,
                          **{f"tile{t}_us": round(best[t], 1) for t in best},
                          **{f"tile{t}_TBps_eff": round(cells * 8 / (best[t] * 1e-6) / 1e12, 2)
                             for t in best},
                          **{f"tile{t}_mlups": round(cells / best[t], 1) for t in best}}),
              flush=True)
        del u, v, pair
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
