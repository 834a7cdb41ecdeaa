"""Device scan — the reference's `DeviceScan` / `ECCCheck` / `AssignDevices`
(`MultiGPU/Diffusion3d_Baseline/Util.cu:32-101`): list the visible MI355X devices, their
memory, CU count, architecture, ECC state, L2/LDS sizes, the xGMI peer topology (link
type and hop count for every device pair, via the native library) and the rank->device
binding a launch would use.

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
    _native_details(out)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    n = len(out["devices"])
    out["binding"] = {r: (r % n if n else None) for r in range(world)}
    try:
        from .ops import _lib
        out["libadvdiff"] = _lib.build_info() if _lib.available() else _lib.load_error()
    except Exception as e:  # pragma: no cover
        out["libadvdiff"] = str(e)
    return out


def _native_details(out: dict) -> None:
    import ctypes
    try:
        from .ops import _lib
        if not _lib.available():
            return
        lib = _lib.require()
    except Exception:  # pragma: no cover
        return
    keys = ("compute_units", "ecc_enabled", "l2_bytes", "lds_per_workgroup", "clock_khz",
            "mem_clock_khz", "mem_bus_bits", "wavefront")
    for d in out["devices"]:
        buf = (ctypes.c_int64 * len(keys))()
        if lib.advdiff_device_info(d["index"], buf, len(keys)) == 0:
            d.update({k: int(v) for k, v in zip(keys, buf)})
    n = len(out["devices"])
    names = {0: "hypertransport", 1: "qpi", 2: "pcie", 3: "infiniband", 4: "xgmi"}
    topo = []
    for a in range(n):
        for b in range(n):
            if a == b:
                continue
            ca, lt, hc = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
            if lib.advdiff_peer_info(a, b, ctypes.byref(ca), ctypes.byref(lt),
                                     ctypes.byref(hc)) == 0:
                topo.append({"a": a, "b": b, "peer_access": bool(ca.value),
                             "link": names.get(lt.value, lt.value), "hops": hc.value})
    if topo:
        out["peer_topology"] = topo


def main(argv=None) -> int:
    print(json.dumps(scan(), indent=1))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
