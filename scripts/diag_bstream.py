"""Diagnose the round-4 boundary-stream hang (tests/test_ipc_gpu.py
test_ipc_boundary_stream_bitwise[diff3-2-None]): 2 ipc ranks sharing one GPU, one step at
a time with a device sync after each, a short ipc wait timeout (ADVDIFF_IPC_TIMEOUT_S) so a
missing signal shows up as a counted timeout instead of a hang, and per-step progress
lines on stderr.

    python scripts/diag_bstream.py MODE [eager|graph] [steps]

MODE: comm (boundary launch on the comm stream), plain (the default overlapped path).
(Round 4's "bstream" mode, a third stream, is gone: its graph capture crashed in
hipStreamEndCapture, see profiles/r5/diag_bstream.md.)  GPU_MAX_HW_QUEUES is taken from the
environment (the tests pin 2)."""
import faulthandler
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _run(comm, mode, graph, steps):
    import torch

    from multigpu_advectiondiffusion_amd import Diffusion, Grid, Solver
    faulthandler.dump_traceback_later(60, exit=False)
    model, grid = Diffusion(K=1.0, order=4), Grid((70, 33, 41), (1.0, 1.0, 1.0))
    kw = {}
    if mode == "comm":
        kw["boundary_on_comm"] = True
    s = Solver(model, grid, comm, dtype=torch.float64, ic="sine", transport="ipc", **kw)
    dt = s.dt()
    t0 = time.perf_counter()
    if graph:
        s.run(iters=steps, graph=True)
        torch.cuda.synchronize()
        print(f"rank {comm.rank}: graph run of {steps} steps done "
              f"{time.perf_counter() - t0:.2f} s, ipc errors {comm.ipc().errors()}",
              file=sys.stderr, flush=True)
    else:
        for i in range(steps):
            s.step(dt)
            torch.cuda.synchronize()
            print(f"rank {comm.rank}: step {i} done {time.perf_counter() - t0:.2f} s, "
                  f"ipc errors {comm.ipc().errors()}", file=sys.stderr, flush=True)
        s.sync_halos()
        torch.cuda.synchronize()
    h = s.bit_hash()
    faulthandler.cancel_dump_traceback_later()
    return h, comm.ipc().errors()


def main():
    from multigpu_advectiondiffusion_amd.launch import spawn_local
    mode = sys.argv[1] if len(sys.argv) > 1 else "comm"
    graph = len(sys.argv) > 2 and sys.argv[2] == "graph"
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 17
    os.environ["ADVDIFF_SHARE_GPU"] = "1"
    os.environ.setdefault("ADVDIFF_IPC_TIMEOUT_S", "5")
    print(f"diag_bstream mode={mode} graph={graph} steps={steps} "
          f"GPU_MAX_HW_QUEUES={os.environ.get('GPU_MAX_HW_QUEUES')}", flush=True)
    out = spawn_local(2, _run, mode, graph, steps, device="cuda", transport="ipc", timeout=100)
    print("result", out, flush=True)
    hs = {h for h, _ in out}
    errs = sum(e for _, e in out)
    print("OK" if len(hs) == 1 and errs == 0 else "BAD", flush=True)
    return 0 if len(hs) == 1 and errs == 0 else 1


if __name__ == "__main__":
    sys.exit(main())
