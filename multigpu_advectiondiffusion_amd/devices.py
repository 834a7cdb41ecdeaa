"""Device scan — the reference's `DeviceScan` / `ECCCheck` / `AssignDevices`
(`MultiGPU/Diffusion3d_Baseline/Util.cu:32-101`): list the visible MI355X devices, their
memory, CU count, architecture and the rank->device binding a launch would use.

    python -m multigpu_advectiondiffusion_amd.devices
"""
from __future__ import annotations

import json
import os


def scan() -> dict:
    import torch
    out = {"torch": torch.__version__, "hip": getattr(torch.version, "hip", None),
           "devices": []}
    if not torch.cuda.is_available():
        out["note"] = "no HIP device visible"
        return out
    for i in range(torch.cuda.device_count()):
        p = torch.cuda.get_device_properties(i)
        out["devices"].append({
            "index": i, "name": p.name, "arch": getattr(p, "gcnArchName", ""),
            "total_memory_GiB": round(p.total_memory / 2 ** 30, 1),
            "compute_units": p.multi_processor_count,
            "warp_size": getattr(p, "warp_size", 64),
        })
    world = int(os.environ.get("WORLD_SIZE", "1"))
    n = len(out["devices"])
    out["binding"] = {r: (r % n if n else None) for r in range(world)}
    try:
        from .ops import _lib
        out["libadvdiff"] = _lib.build_info() if _lib.available() else _lib.load_error()
    except Exception as e:  # pragma: no cover
        out["libadvdiff"] = str(e)
    return out


if __name__ == "__main__":
    print(json.dumps(scan(), indent=1))
