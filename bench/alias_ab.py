#!/usr/bin/env python3
"""Where two fields sit relative to each other: the fused heat step u -> v at n^3 with u
and v carved out of ONE allocation at a chosen distance (v = u + field bytes + gap), for
the dense layout and a pitched one, next to two separately allocated fields.  Distances of
exactly 2^k bytes put u[i] and v[i] on the same HBM channel / bank for every i.  Interleaved
rounds after a settling run, best round per configuration.

    python bench/alias_ab.py [--n 512] [--gaps-kib 0 4 64 2052]
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
    ap.add_argument("--n", type=int, default=512)
    ap.add_argument("--gaps-kib", type=int, nargs="+", default=[0, 4, 64, 2052])
    ap.add_argument("--pitches", nargs="+", default=["0,0", "8,1"])
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--orders", type=int, nargs="+", default=[4, 2])
    a = ap.parse_args()
    n = a.n
    g = torch.Generator(device="cuda").manual_seed(3)
    base = torch.rand((n, n, n), dtype=torch.float64, device="cuda", generator=g)
    cfgs = {}
    keep = []
    for p in a.pitches:
        px, py = (int(v) for v in p.split(","))
        shape = (n, n + py, n + px)
        numel = shape[0] * shape[1] * shape[2]
        for gap in ["sep"] + a.gaps_kib:
            if gap == "sep":
                u = torch.zeros(shape, dtype=torch.float64, device="cuda")
                v = torch.zeros_like(u)
            else:
                ge = gap * 1024 // 8
                buf = torch.zeros(2 * numel + ge, dtype=torch.float64, device="cuda")
                keep.append(buf)
                u = buf[:numel].view(shape)
                v = buf[numel + ge:2 * numel + ge].view(shape)
            u[:, :n, :n] = base
            v[:, :n, :n] = base
            dist = v.data_ptr() - u.data_ptr()
            cfgs[(p, gap)] = ([u, v], dist)
    del base
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for order in a.orders:
        R = order // 2
        kw = dict(nx=n, ny=n, k0=R, k1=n - R, zlo=R, zhi=n - R, border=R, order=order,
                  cx=0.1, cy=0.1, cz=0.1, dt=0.5, exclusive=True)

        def run(pair, k):
            for _ in range(k):
                stencil.diffusion3d_step(pair[0], pair[1], **kw)
                pair.reverse()
        first = next(iter(cfgs.values()))[0]
        run(first, 200)
        best = {c: float("inf") for c in cfgs}
        for _ in range(a.rounds):
            for c, (pair, _) in cfgs.items():
                run(pair, 4)
                s.record()
                run(pair, 16)
                e.record()
                torch.cuda.synchronize()
                best[c] = min(best[c], s.elapsed_time(e) * 1e3 / 16)
        ref = best[(a.pitches[0], "sep")]
        for c, (_, dist) in cfgs.items():
            print(json.dumps({"order": order, "pitch": c[0], "gap_kib": c[1],
                              "distance_bytes": dist, "distance_mod_1MiB": dist % (1 << 20),
                              "us": round(best[c], 1), "vs_first": round(ref / best[c], 4)}),
                  flush=True)


if __name__ == "__main__":
    main()
