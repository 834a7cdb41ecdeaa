#!/usr/bin/env python3
"""A/B of the fused 3-D heat step between two builds of libadvdiff.so in ONE process,
alternating launch by launch, so clock and thermal drift hit both builds alike (separate
runs on this pool differ by ±5 % from the clock alone).

    python bench/ab_step.py LIB_A LIB_B [--n 512] [--reps 20] [--rounds 8] [--orders 4,2]
        [--pitch PX,PY]   (fields of (n, n + PY, n + PX): the solver's pitched layout)
"""
import argparse
import ctypes
import json
import statistics

import torch


def load(path):
    lib = ctypes.CDLL(path)
    f = lib.advdiff_diffusion3d_step_box_ex
    ci, c64, cd, cv = ctypes.c_int, ctypes.c_int64, ctypes.c_double, ctypes.c_void_p
    f.argtypes = [ci, cv, cv, ci, ci, c64, c64, ci, ci, ci, ci, ci, ci, ci,
                  ctypes.POINTER(ci), ci, cd, cd, cd, cd, ci, cv]
    f.restype = ci
    return f


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs=2)
    ap.add_argument("--n", type=int, default=512)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--orders", default="4,2")
    ap.add_argument("--pitch", default="0,0")
    a = ap.parse_args()
    n = a.n
    px, py = (int(v) for v in a.pitch.split(","))
    u = torch.rand((n, n + py, n + px), dtype=torch.float64, device="cuda")
    sy, sz = u.stride(1), u.stride(0)
    outs = [torch.empty_like(u), torch.empty_like(u)]
    st = torch.cuda.current_stream().cuda_stream
    fns = [load(p) for p in a.libs]
    res = {}
    for order in [int(o) for o in a.orders.split(",")]:
        R = order // 2
        box = (ctypes.c_int * 8)(R, n - R, R, n - R, 0, n, 0, n)
        args = lambda o: (1, u.data_ptr(), o.data_ptr(), n, n, sy, sz, n, R, n - R, 0, 0,  # noqa
                          R, n - R, box, order, 1.0, 1.0, 1.0, 0.01, 1, st)
        ts = [[], []]
        for _ in range(a.rounds):
            for i, f in enumerate(fns):
                assert f(*args(outs[i])) == 0
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.reps):
                    f(*args(outs[i]))
                e1.record()
                e1.synchronize()
                ts[i].append(e0.elapsed_time(e1) * 1e3 / a.reps)
        torch.cuda.synchronize()
        same = bool(torch.equal(outs[0], outs[1]))
        res[f"fd{order}"] = {"A_us": round(statistics.median(ts[0]), 1),
                             "B_us": round(statistics.median(ts[1]), 1),
                             "B_vs_A": round(statistics.median(ts[1]) / statistics.median(ts[0]), 4),
                             "bitwise_equal": same}
        print(f"fd{order}", res[f"fd{order}"], flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
