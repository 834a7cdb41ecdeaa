#!/usr/bin/env python3
"""A/B the WENO5 Burgers stage kernel of two builds of libadvdiff.so in one process
(alternating, so clock/thermal drift hits both alike); both builds must give the same
bits (checked on the same inputs after the timing).

    python bench/ab_burgers.py LIB_A LIB_B [--n 256] [--reps 50] [--rounds 5] [--fp32]
"""
import argparse
import ctypes
import json

import torch


def load(path):
    lib = ctypes.CDLL(path)
    f = lib.advdiff_burgers3d_stage
    c_int, c_i64, c_dbl, c_vp = ctypes.c_int, ctypes.c_int64, ctypes.c_double, ctypes.c_void_p
    f.argtypes = [c_int, c_vp, c_vp, c_vp, c_int, c_int, c_i64, c_i64, c_int, c_int, c_int,
                  c_int, c_dbl, c_dbl, c_dbl, c_dbl, c_dbl, c_dbl, c_dbl, c_dbl, c_dbl, c_vp]
    f.restype = c_int
    return f


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs=2)
    ap.add_argument("--n", type=int, default=256)
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--fp32", action="store_true")
    a = ap.parse_args()
    n = a.n
    dt = torch.float32 if a.fp32 else torch.float64
    u = (torch.rand((n, n, n), dtype=torch.float64, device="cuda") * 0.5 + 0.1).to(dt)
    A, B = torch.rand_like(u), torch.rand_like(u)
    st = torch.cuda.current_stream().cuda_stream
    fns = [load(p) for p in a.libs]
    res = {}
    for wz, visc in ((1, 1e-5), (1, 0.0), (0, 1e-5)):
        v = visc * (n / 2.0) ** 2
        code = 0 if a.fp32 else 1  # ADVDIFF_F32 / ADVDIFF_F64
        args = (code, A.data_ptr(), u.data_ptr(), B.data_ptr(), n, n, n, n * n, 3, n - 3, 3, wz,
                n / 2.0, n / 2.0, n / 2.0, v, v, v, 1e-4, 0.75, 0.25, st)
        best = [1e9, 1e9]
        for _ in range(a.rounds):
            for i, f in enumerate(fns):
                for _ in range(3):
                    assert f(*args) == 0
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.reps):
                    f(*args)
                e1.record()
                torch.cuda.synchronize()
                best[i] = min(best[i], e0.elapsed_time(e1) * 1e3 / a.reps)
        outs = []
        for f in fns:
            A.copy_(u)
            B.zero_()
            assert f(*args) == 0
            torch.cuda.synchronize()
            outs.append(B.clone())
        res[f"wz{wz}_visc{visc}"] = {"A_us": round(best[0], 1), "B_us": round(best[1], 1),
                                     "B_over_A": round(best[1] / best[0], 4),
                                     "bitwise_equal": bool(torch.equal(outs[0], outs[1]))}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
