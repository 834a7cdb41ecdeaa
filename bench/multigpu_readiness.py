#!/usr/bin/env python3
"""Multi-GPU readiness measured on ONE MI355X (the 8-GPU node is not ours to launch):

1. per-rank compute split — for every candidate decomposition of the weak-scaling grids
   (N = 2, 4, 8; 512^3 cells per rank) the fused heat step of ONE rank's block as a full
   launch vs interior + boundary launches (the overlap schedule), the halo bytes that
   rank sends per step and neighbour, and the host time to issue one overlapped step;
2. interference — the interior launch of the N=8 slab rank (1024 x 1024 x 128) running
   while a 50 MB transfer executes on a high-priority stream: a plain device copy, and a
   REAL RCCL send/recv pair (a world-1 group sending to itself: the copy kernels RCCL
   runs for a peer, minus the xGMI link);
3. host cost of one grouped RCCL call (batch_isend_irecv, 2 ops) from Python.

    python bench/multigpu_readiness.py [--reps 10] [--skip-rccl]

Prints one JSON object per measurement; profiles/multigpu_readiness.md is written from
the output.  Reference choreography being replaced:
`MultiGPU/Diffusion3d_Baseline/main.c:201-302`.
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multigpu_advectiondiffusion_amd import Burgers, Diffusion, Grid, Solver  # noqa: E402
from multigpu_advectiondiffusion_amd.parallel import weak_scaling_grid  # noqa: E402
from multigpu_advectiondiffusion_amd.parallel.comm import Comm  # noqa: E402


def gpu_time(fn, reps):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3  # us


def host_time(fn, reps):
    """Host time to ISSUE one call (the GPU runs behind; nothing here blocks)."""
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    return (t1 - t0) / reps * 1e6  # us


def halo_bytes(s):
    """Bytes one rank sends per step, per neighbour message (all phases)."""
    elem = s.u.element_size()
    out = []
    if s.cart:
        for axes in s.halo._phases():
            for peer, sv, rv, key in s.halo._regions(s.u, axes):
                out.append({"axis": key[0], "side": key[1], "peer": peer,
                            "MB": round(sv.numel() * elem / 1e6, 2)})
    else:
        d = s.d
        for side, peer, rng in ((-1, d.lower, d.send_lower() if d.lower is not None else None),
                                (1, d.upper, d.send_upper() if d.upper is not None else None)):
            if peer is None:
                continue
            v = s.u[rng[0]:rng[1]]
            out.append({"axis": 0, "side": side, "peer": peer,
                        "MB": round(v.numel() * elem / 1e6, 2)})
    return out


def split_case(kind, n_ranks, pgrid, reps):
    base = 512 if kind == "heat" else 256
    shape = weak_scaling_grid(base, n_ranks)
    size = n_ranks
    # a rank in the middle of the process grid (most neighbours)
    rank = {1: 0, 2: 1, 4: 1, 8: 3}.get(size, size // 2)
    if pgrid is not None and all(p > 1 for p in pgrid):
        rank = size - 1
    comm = Comm(rank=rank, size=size, device="cuda:0")
    if kind == "heat":
        model = Diffusion(K=1.0, order=4)
        s = Solver(model, Grid(shape, (1.0,) * 3), comm, dtype=torch.float64, ic="sine",
                   decomp=pgrid)
    else:
        model = Burgers(viscosity=1e-5, weno="z", cfl=0.3)
        s = Solver(model, Grid(shape, (2.0,) * 3), comm, dtype=torch.float64, ic="gaussian",
                   decomp=pgrid)
    dt = model.stable_dt()
    res = {"case": "split", "kind": kind, "N": n_ranks, "grid": list(shape),
           "pgrid": list(s.pgrid), "rank": rank,
           "block_zyx": [c for _, c in s.cd.global_box()], "fused": s.fused}
    if s.fused:
        full = (lambda: s._launch_fused_box(s.full, dt, True)) if s.cart else \
            (lambda: s._launch_fused(s.full, dt, exclusive=True))
        inner = (lambda: s._launch_fused_box(s.interior, dt)) if s.cart else \
            (lambda: s._launch_fused(s.interior, dt))

        def bnd():
            if s.cart:
                for b in s.boundary:
                    s._launch_fused_box(b, dt)
            else:
                s._launch_fused(s.boundary[0], dt, s.boundary[1])
    else:  # Burgers: one RK stage (u -> A)
        full = lambda: s._launch(s.u, None, s.A, s.full, dt, 0.0, 1.0)  # noqa: E731
        inner = lambda: s._launch(s.u, None, s.A, s.interior, dt, 0.0, 1.0)  # noqa: E731

        def bnd():
            if s.cart:
                for r in s.boundary:
                    s._launch(s.u, None, s.A, r, dt, 0.0, 1.0)
            else:  # both slabs in one launch, as Solver._stage issues them
                s._launch(s.u, None, s.A, s.boundary[0], dt, 0.0, 1.0, rng2=s.boundary[1])
    res["full_us"] = round(gpu_time(full, reps), 1)
    res["interior_us"] = round(gpu_time(inner, reps), 1)
    res["boundary_us"] = round(gpu_time(bnd, reps), 1)
    res["split_overhead_pct"] = round(
        100 * ((res["interior_us"] + res["boundary_us"]) / res["full_us"] - 1), 1)

    def issue():
        inner()
        bnd()
    res["host_issue_us_per_launch_set"] = round(host_time(issue, reps), 1)
    msgs = halo_bytes(s)
    res["halo_msgs"] = msgs
    res["halo_MB_per_step"] = round(sum(m["MB"] for m in msgs), 2)
    res["halo_max_link_MB"] = round(max((m["MB"] for m in msgs), default=0.0), 2)
    res["halo_phases"] = len(s.halo._phases()) if s.cart else 1
    print(json.dumps(res), flush=True)
    del s
    torch.cuda.empty_cache()
    return res


def interference(reps, use_rccl):
    """Interior launch of the N=8 slab rank with a concurrent 50 MB transfer."""
    comm = Comm(rank=3, size=8, device="cuda:0")
    model = Diffusion(K=1.0, order=4)
    s = Solver(model, Grid(weak_scaling_grid(512, 8), (1.0,) * 3), comm, dtype=torch.float64,
               ic="sine")
    dt = model.stable_dt()
    G = s.ghost
    plane = s.u[0].numel()
    nbytes = G * plane * s.u.element_size()
    src = torch.rand(G * plane, dtype=torch.float64, device="cuda")
    dst = torch.empty_like(src)
    lo, hi = torch.cuda.Stream.priority_range()
    hp = torch.cuda.Stream(priority=hi)
    main = torch.cuda.current_stream()

    def interior():
        s._launch_fused(s.interior, dt)

    xfers = {"copy": lambda: dst.copy_(src)}
    if use_rccl:
        import torch.distributed as dist
        if not dist.is_initialized():
            from multigpu_advectiondiffusion_amd.launch import free_port
            from multigpu_advectiondiffusion_amd.parallel.comm import pg_kwargs
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ["MASTER_PORT"] = str(free_port())
            dist.init_process_group("nccl", rank=0, world_size=1,
                                    **pg_kwargs("nccl", torch.device("cuda", 0)))

        def rccl_self():
            ops = [dist.P2POp(dist.isend, src, 0), dist.P2POp(dist.irecv, dst, 0)]
            for w in dist.batch_isend_irecv(ops):
                w.wait()
        xfers["rccl_self_sendrecv"] = rccl_self
        # host cost of one grouped call
        with torch.cuda.stream(hp):
            hc = host_time(rccl_self, reps)
        print(json.dumps({"case": "rccl_host_cost", "ops": 2, "MB": round(nbytes / 1e6, 1),
                          "host_us_per_grouped_call": round(hc, 1)}), flush=True)

    t_int = gpu_time(interior, reps)
    for name, fn in xfers.items():
        with torch.cuda.stream(hp):
            t_x = gpu_time(fn, reps)
        # concurrent: interior on the main stream, transfer on the high-priority stream
        # started right after the interior launch; per-stream events
        ti, tx = [], []
        for _ in range(reps):
            torch.cuda.synchronize()
            a0, a1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            b0, b1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a0.record(main)
            interior()
            a1.record(main)
            b0.record(hp)
            with torch.cuda.stream(hp):
                fn()
            b1.record(hp)
            torch.cuda.synchronize()
            ti.append(a0.elapsed_time(a1) * 1e3)
            tx.append(a0.elapsed_time(b1) * 1e3)
        ti.sort()
        tx.sort()
        res = {"case": "interference", "transfer": name, "MB": round(nbytes / 1e6, 1),
               "interior_alone_us": round(t_int, 1), "transfer_alone_us": round(t_x, 1),
               "transfer_alone_GBps": round(nbytes / t_x / 1e3, 1),
               "interior_concurrent_us": round(ti[len(ti) // 2], 1),
               "transfer_done_after_us": round(tx[len(tx) // 2], 1),
               "interior_slowdown_pct": round(100 * (ti[len(ti) // 2] / t_int - 1), 1)}
        print(json.dumps(res), flush=True)
    del s
    torch.cuda.empty_cache()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--skip-rccl", action="store_true")
    ap.add_argument("--skip-split", action="store_true")
    a = ap.parse_args()
    if not a.skip_split:
        cands = {2: [None], 4: [None, (2, 2, 1)], 8: [None, (4, 2, 1), (2, 4, 1), (2, 2, 2)]}
        for kind in ("heat", "burgers"):
            for n, pgs in cands.items():
                for pg in pgs:
                    try:
                        split_case(kind, n, pg, a.reps)
                    except Exception as e:  # report and go on
                        print(json.dumps({"case": "split", "kind": kind, "N": n,
                                          "pgrid": pg, "error": str(e)}), flush=True)
    interference(a.reps, not a.skip_rccl)


if __name__ == "__main__":
    main()
