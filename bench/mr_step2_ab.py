#!/usr/bin/env python3
"""FD2 slab-rank step, one RK3 step per launch vs two (round 6, multi-rank two-step).

A middle rank of the 8-GPU z-slab run (1024 x 1024 x 128 owned planes, fp64, pitched
fields as the solver allocates them) issues per step, without the exchange itself:

* one step per launch (3R = 3 ghost planes, 134 planes allocated): the interior launch
  (owned planes >= 3 from a face) + ONE launch of both 3-plane boundary slabs;
* two steps per launch (6R = 6 ghost planes, 140 planes): every second step the two-step
  interior launch (owned planes >= 6 from a face) + one two-step launch per 6-plane
  boundary slab (diffusion_fused.hip v6_march).

Both move the same halo bytes per step.  Interleaved rounds of back-to-back launch
sequences (HIP events, min per round over the settled clock); the rate is owned cells per
step time.  Also the one-GPU 512^3 step for reference, and the solver's own choice for
the rank shape (advdiff_diffusion3d_step2_pick on the interior, the rule
Solver._choose_multirank_step2 applies).

    python bench/mr_step2_ab.py [--owned 128] [--nx 1024] [--rounds 5] [--steps 20]
    python bench/mr_step2_ab.py --order 4   # the FD4 slab rank's step (one per launch,
                                            # 3R = 6 ghost planes): interior + boundary
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
    ap.add_argument("--nx", type=int, default=1024)
    ap.add_argument("--owned", type=int, default=128)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--pitch", default="4,1")
    ap.add_argument("--order", type=int, default=2, choices=[2, 4])
    a = ap.parse_args()
    if a.order == 4:
        return fd4_rank(a)
    px, py = (int(v) for v in a.pitch.split(","))
    n, own = a.nx, a.owned
    c = (1.0, 1.0, 1.0)
    dt = 0.9 / (2 * sum(c))
    kw = dict(nx=n, ny=n, border=1, cx=c[0], cy=c[1], cz=c[2], dt=dt)

    def fields(G):
        u = torch.rand((own + 2 * G, n + py, n + px), dtype=torch.float64, device="cuda")
        return u, u.clone()

    u1, v1 = fields(3)
    u2, v2 = fields(6)
    nz1, nz2 = own + 6, own + 12

    def one_step(uin, uout):
        stencil.diffusion3d_step(uin, uout, k0=6, k1=nz1 - 6, zlo=0, zhi=nz1, order=2, **kw)
        stencil.diffusion3d_step(uin, uout, k0=3, k1=6, k0b=nz1 - 6, k1b=nz1 - 3, zlo=0,
                                 zhi=nz1, order=2, **kw)

    def two_steps(uin, uout):
        stencil.diffusion3d_step2x(uin, uout, k0=12, k1=nz2 - 12, zlo=0, zhi=nz2, **kw)
        stencil.diffusion3d_step2x(uin, uout, k0=6, k1=12, zlo=0, zhi=nz2, **kw)
        stencil.diffusion3d_step2x(uin, uout, k0=nz2 - 12, k1=nz2 - 6, zlo=0, zhi=nz2, **kw)

    def seq1():
        nonlocal u1, v1
        for _ in range(a.steps):
            one_step(u1, v1)
            u1, v1 = v1, u1

    def seq2():
        nonlocal u2, v2
        for _ in range(a.steps // 2):
            two_steps(u2, v2)
            u2, v2 = v2, u2

    def timed(fn):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        e1.synchronize()
        return e0.elapsed_time(e1) * 1e3 / a.steps  # us per step

    for _ in range(3):  # settle the clock
        seq1()
        seq2()
    best = {"one": 1e30, "two": 1e30}
    for _ in range(a.rounds):
        best["one"] = min(best["one"], timed(seq1))
        best["two"] = min(best["two"], timed(seq2))
    cells = own * n * n
    # the solver's rule for this rank shape: the interior launch timed both ways
    inter = stencil.diffusion3d_step2_pick(u2, v2, k0=12, k1=nz2 - 12, zlo=0, zhi=nz2, **kw)
    # one-GPU 512^3 (the bench's N = 1 shape) for reference
    m = 512
    w = torch.rand((m, m + py, m + px), dtype=torch.float64, device="cuda")
    wo = w.clone()
    kw5 = dict(kw, nx=m, ny=m)

    def seq5():
        nonlocal w, wo
        for _ in range(a.steps):
            stencil.diffusion3d_step(w, wo, k0=1, k1=m - 1, zlo=1, zhi=m - 1, order=2, **kw5)
            w, wo = wo, w
    for _ in range(3):
        seq5()
    t5 = min(timed(seq5) for _ in range(a.rounds))
    out = {"rank_block": [n, n, own], "one_step_us": round(best["one"], 1),
           "two_step_us": round(best["two"], 1),
           "one_step_mlups": round(cells / best["one"], 1),
           "two_step_mlups": round(cells / best["two"], 1),
           "speedup_two": round(best["one"] / best["two"], 4),
           "solver_pick_two_step": bool(inter),
           "one_gpu_512_us": round(t5, 1), "one_gpu_512_mlups": round(m ** 3 / t5, 1)}
    print(json.dumps(out), flush=True)


def fd4_rank(a):
    """FD4 slab rank per step: interior launch + one launch of both 3R-plane boundary
    slabs, vs the same cells in one launch (what the rank would cost without the overlap
    split) and the one-GPU 512^3 step."""
    px, py = (int(v) for v in a.pitch.split(","))
    n, own, G = a.nx, a.owned, 6
    nz = own + 2 * G
    kw = dict(nx=n, ny=n, border=2, order=4, cx=1.0, cy=1.0, cz=1.0, dt=0.01)
    pair = [torch.rand((nz, n + py, n + px), dtype=torch.float64, device="cuda")]
    pair.append(pair[0].clone())

    def split(k):
        for _ in range(k):
            stencil.diffusion3d_step(pair[0], pair[1], k0=2 * G, k1=nz - 2 * G, zlo=0, zhi=nz, **kw)
            stencil.diffusion3d_step(pair[0], pair[1], k0=G, k1=2 * G, k0b=nz - 2 * G,
                                     k1b=nz - G, zlo=0, zhi=nz, **kw)
            pair.reverse()

    def whole(k):
        for _ in range(k):
            stencil.diffusion3d_step(pair[0], pair[1], k0=G, k1=nz - G, zlo=0, zhi=nz, **kw)
            pair.reverse()

    def inter(k):
        for _ in range(k):
            stencil.diffusion3d_step(pair[0], pair[1], k0=2 * G, k1=nz - 2 * G, zlo=0, zhi=nz, **kw)
            pair.reverse()

    def bnd(k):
        for _ in range(k):
            stencil.diffusion3d_step(pair[0], pair[1], k0=G, k1=2 * G, k0b=nz - 2 * G,
                                     k1b=nz - G, zlo=0, zhi=nz, **kw)
            pair.reverse()

    lo, hi = torch.cuda.Stream.priority_range()
    cs = torch.cuda.Stream(priority=hi)

    def two_streams(k):
        """The solver's comm-stream schedule minus the exchange: per step the interior on
        the compute stream beside the boundary launch on the (high-priority) comm stream,
        joined before the next step (Solver._step_fused_bcomm)."""
        cur = torch.cuda.current_stream()
        for _ in range(k):
            cs.wait_stream(cur)
            stencil.diffusion3d_step(pair[0], pair[1], k0=2 * G, k1=nz - 2 * G, zlo=0, zhi=nz, **kw)
            with torch.cuda.stream(cs):
                stencil.diffusion3d_step(pair[0], pair[1], k0=G, k1=2 * G, k0b=nz - 2 * G,
                                         k1b=nz - G, zlo=0, zhi=nz, **kw)
            cur.wait_stream(cs)
            pair.reverse()

    def timed(fn):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn(a.steps)
        e1.record()
        e1.synchronize()
        return e0.elapsed_time(e1) * 1e3 / a.steps

    fns = {"split": split, "two_streams": two_streams, "whole": whole, "interior": inter,
           "boundary": bnd}
    for f in fns.values():
        f(10)
    best = {k: 1e30 for k in fns}
    for _ in range(a.rounds):
        for k, f in fns.items():
            best[k] = min(best[k], timed(f))
    cells = own * n * n
    print(json.dumps({"order": 4, "rank_block": [n, n, own],
                      **{f"{k}_us": round(v, 1) for k, v in best.items()},
                      "split_mlups": round(cells / best["split"], 1),
                      "two_streams_mlups": round(cells / best["two_streams"], 1),
                      "whole_mlups": round(cells / best["whole"], 1)}), flush=True)


if __name__ == "__main__":
    main()
