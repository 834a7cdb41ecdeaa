"""Tracing hooks: roctx ranges (visible in rocprofv3 --marker-trace / rocprof timelines)
and a sync-debug mode.

Reference: the only tracing is the external ``nvprof`` wrapper
(`MultiGPU/Diffusion3d_Baseline/run.sh:2`, `profile.sh:2`) and MPI_Wtime/clock() timers;
error checking is the always-on ``checkCuda``/``CudaCheckError`` (device sync after each
launch, `MultiGPU/Diffusion2d_Baseline/Kernels.cu:12-57`).  Here:

* ``ADVDIFF_TRACE=1`` wraps every stage/halo phase in a named roctx range;
* ``ADVDIFF_SYNC_DEBUG=1`` synchronises the device after every launch and re-raises the
  first asynchronous fault at the op that caused it (off by default: it serialises
  streams and kills the compute/comm overlap).
"""
from __future__ import annotations

import contextlib
import os

import torch

TRACE = os.environ.get("ADVDIFF_TRACE", "0") not in ("", "0")
SYNC_DEBUG = os.environ.get("ADVDIFF_SYNC_DEBUG", "0") not in ("", "0")


def _nvtx():
    try:
        return torch.cuda.nvtx  # roctx-backed on ROCm builds
    except Exception:  # pragma: no cover
        return None


@contextlib.contextmanager
def range_(name: str, enabled: bool | None = None):
    on = TRACE if enabled is None else enabled
    nv = _nvtx() if on and torch.cuda.is_available() else None
    if nv is not None:
        nv.range_push(name)
    try:
        yield
    finally:
        if nv is not None:
            nv.range_pop()


def sync_check(what: str, device) -> None:
    if SYNC_DEBUG and torch.device(device).type == "cuda":
        try:
            torch.cuda.synchronize(device)
        except RuntimeError as e:  # pragma: no cover - needs a faulting kernel
            raise RuntimeError(f"asynchronous device fault detected after {what}: {e}") from e
