#!/usr/bin/env python3
"""Probe: IPC export of device buffers across free + reallocation (2 ranks sharing one
GPU).  Each trial allocates a buffer, exports it (advdiff_ipc_describe: hipIpcGetMemHandle),
the peer maps it (advdiff_ipc_map: hipIpcOpenMemHandle); then the buffer is freed (the
allocator cache emptied: hipFree) and the collective reset (the peer closes its mappings)
runs either BEFORE the next allocation (the order Solver construction now enforces) or
AFTER it.  The second order is what the bench did when a solver was built right after
another was freed: the new field's export failed with "invalid argument" (4 ipc ranks,
1.04 GB fields), and in this probe the 8 MiB case of that order hung until the box's
watchdog killed it (profiles/ipc_realloc_probe_r3.log) — so it runs only on request.

    python bench/ipc_realloc_probe.py [--after]
"""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _rank(comm, mb, reset_before_alloc):
    import torch

    from multigpu_advectiondiffusion_amd.ops import _lib
    ipc = comm.ipc()
    lib = ipc.lib
    out = []
    peer = 1 - comm.rank
    for trial in range(3):
        t = torch.empty(int(mb * 2 ** 20) // 8, dtype=torch.float64, device=comm.device)
        if trial and not reset_before_alloc:
            ipc.reset()  # the peer closes its mapping of the freed buffer only now
        a = _lib.IpcAddr()
        e = lib.advdiff_ipc_describe(ipc.ctx, t.data_ptr(), ctypes.byref(a))
        ok = comm.allreduce_max(float(e))  # both ranks agree whether to swap
        rec = {"trial": trial, "ptr": hex(t.data_ptr()), "describe": e}
        if ok == 0:
            b = _lib.IpcAddr.from_buffer_copy(ipc._swap([peer], [bytes(a)])[0])
            p = ctypes.c_void_p()
            rec["map"] = lib.advdiff_ipc_map(ipc.ctx, ctypes.byref(b), ctypes.byref(p))
        torch.cuda.synchronize()
        comm.barrier()
        del t
        torch.cuda.empty_cache()
        if reset_before_alloc:
            ipc.reset()
        out.append(rec)
    return out


def main():
    os.environ.setdefault("ADVDIFF_SHARE_GPU", "1")
    os.environ.setdefault("GPU_MAX_HW_QUEUES", "2")
    from multigpu_advectiondiffusion_amd.launch import spawn_local
    orders = (True, False) if "--after" in sys.argv else (True,)
    for mb in (8, 1036):
        for before in orders:
            res = spawn_local(2, _rank, mb, before, device="cuda", transport="ipc", timeout=300)
            print(json.dumps({"MiB": mb, "reset": "before the new allocation" if before else
                              "after the new allocation", "rank0": res[0], "rank1": res[1]}),
                  flush=True)


if __name__ == "__main__":
    main()
