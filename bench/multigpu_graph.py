#!/usr/bin/env python3
"""Host issue cost vs GPU time of a multi-rank step, eager and hipGraph-replayed.

Two ranks share the box's one GPU over the ipc transport (device puts + flags), each with
the per-rank block of the 8-GPU weak-scaling runs: heat 1024x1024x128 (global z = 256
here) and Burgers WENO5-Z 512x512x64 (global z = 128).  Per configuration it reports

  * host_issue_ms_per_step: wall time the host spends ISSUING one step (eager: the
    Python solver's launches + exchange kernels; graph: one replay of 8 steps / 8), with
    the GPU still busy — what must stay below the GPU time for the host to keep ahead;
  * gpu_ms_per_step: synchronised wall time per step with both ranks on the one GPU
    (so about twice one rank's GPU time).

    python bench/multigpu_graph.py [--steps 16]
Output: one JSON line per (model, mode).
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _rank(comm, kind, steps):
    import torch

    from multigpu_advectiondiffusion_amd import Burgers, Diffusion, Grid, Solver
    if kind == "heat":
        model, grid, ic = Diffusion(K=1.0, order=4), Grid((1024, 1024, 256), (1.0, 1.0, 1.0)), "sine"
    else:
        model, grid, ic = (Burgers(viscosity=1e-5, weno="z", cfl=0.3),
                           Grid((512, 512, 128), (2.0, 2.0, 2.0)), "gaussian")
    s = Solver(model, grid, comm, dtype=torch.float64, ic=ic)
    dt = s.dt()
    out = {}
    for mode in ("eager", "graph"):
        s.run(iters=8, dt=dt, graph=(mode == "graph"))  # warm-up (+ capture)
        torch.cuda.synchronize()
        comm.barrier()
        # host issue: time the issuing of `steps` steps, then wait for the GPU
        t0 = time.perf_counter()
        if mode == "graph":
            g = s._graph_for(dt)
            s.sync_halos()
            for _ in range(steps // s.GRAPH_STEPS):
                g.replay()
        else:
            for _ in range(steps):
                s.step(dt)
            s.sync_halos()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        comm.barrier()
        issue = comm.allreduce_max(t1 - t0) / steps
        wall = comm.allreduce_max(t2 - t0) / steps
        out[mode] = (issue, wall)
    assert comm.ipc().errors() == 0
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=32)
    a = ap.parse_args()
    os.environ.setdefault("ADVDIFF_SHARE_GPU", "1")
    os.environ.setdefault("GPU_MAX_HW_QUEUES", "1")
    from multigpu_advectiondiffusion_amd.launch import spawn_local
    for kind in ("heat", "burgers"):
        res = spawn_local(2, _rank, kind, a.steps, device="cuda", transport="ipc", timeout=600)[0]
        for mode, (issue, wall) in res.items():
            print(json.dumps({"model": kind, "per_rank_block": "1024x1024x128" if kind == "heat"
                              else "512x512x64", "ranks_on_one_gpu": 2, "transport": "ipc",
                              "mode": mode, "host_issue_ms_per_step": round(issue * 1e3, 4),
                              "gpu_ms_per_step_two_ranks": round(wall * 1e3, 4)}), flush=True)


if __name__ == "__main__":
    main()
