"""ctypes binding of ``lib/libadvdiff.so`` (the hand-written gfx950 HIP kernels).

The library exposes a plain C ABI (``csrc/include/advdiff/kernels.h``) so the very same
kernels serve the Python/PyTorch path (device tensors' ``data_ptr()`` + the current HIP
stream handle) and the native C++ apps.  Loading is lazy; on a machine with a GPU the
ops refuse to silently fall back to PyTorch (``require()`` raises), so a test that passes
on a GPU box has provably run the native kernels.
"""
from __future__ import annotations

import ctypes
import hashlib
import os
import threading
from pathlib import Path

_LIB_DIR = Path(__file__).resolve().parent.parent / "lib"
LIB_PATH = Path(os.environ.get("ADVDIFF_LIB", _LIB_DIR / "libadvdiff.so"))
CSRC = Path(__file__).resolve().parents[2] / "csrc"

_lock = threading.Lock()
_lib = None
_err: str | None = None

c_int, c_i64, c_dbl, c_vp, c_sz = (ctypes.c_int, ctypes.c_int64, ctypes.c_double,
                                   ctypes.c_void_p, ctypes.c_size_t)

_SIGS = {
    "advdiff_diffusion3d_stage": [c_int, c_vp, c_vp, c_vp, c_int, c_int, c_i64, c_i64, c_int,
                                  c_int, c_int, c_int, c_dbl, c_dbl, c_dbl, c_dbl, c_dbl,
                                  c_dbl, c_vp],
    "advdiff_diffusion3d_step": [c_int, c_vp, c_vp, c_int, c_int, c_i64, c_i64, c_int, c_int,
                                 c_int, c_int, c_int, c_int, c_int, c_dbl, c_dbl, c_dbl, c_dbl,
                                 c_vp],
    "advdiff_diffusion3d_step2": [c_int, c_vp, c_vp, c_int, c_int, c_i64, c_i64, c_int, c_int,
                                  c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_dbl, c_dbl,
                                  c_dbl, c_dbl, c_vp],
    "advdiff_diffusion2d_step": [c_int, c_vp, c_vp, c_int, c_i64, c_int, c_int, c_int, c_int,
                                 c_int, c_int, c_int, c_dbl, c_dbl, c_dbl, c_vp],
    "advdiff_diffusion3d_step2x": [c_int, c_vp, c_vp, c_int, c_int, c_i64, c_i64, c_int, c_int,
                                   c_int, c_int, c_int, ctypes.POINTER(c_int), c_dbl, c_dbl,
                                   c_dbl, c_dbl, c_vp],
    "advdiff_diffusion3d_step2_pick": [c_int, c_vp, c_vp, c_int, c_int, c_i64, c_i64, c_int,
                                       c_int, c_int, c_int, c_int, ctypes.POINTER(c_int), c_dbl,
                                       c_dbl, c_dbl, c_dbl, c_vp, ctypes.POINTER(c_int)],
    "advdiff_diffusion3d_step_sched_pick": [c_int, c_vp, c_vp, c_int, c_int, c_i64, c_i64,
                                            c_int, c_int, c_int, c_int, c_int,
                                            ctypes.POINTER(c_int), c_int, c_dbl, c_dbl, c_dbl,
                                            c_dbl, c_vp, ctypes.POINTER(c_int)],
    "advdiff_diffusion3d_step_box": [c_int, c_vp, c_vp, c_int, c_int, c_i64, c_i64, c_int,
                                     c_int, c_int, c_int, c_int, c_int, c_int,
                                     ctypes.POINTER(c_int), c_int, c_dbl, c_dbl, c_dbl, c_dbl,
                                     c_vp],
    "advdiff_diffusion3d_step_box_ex": [c_int, c_vp, c_vp, c_int, c_int, c_i64, c_i64, c_int,
                                        c_int, c_int, c_int, c_int, c_int, c_int,
                                        ctypes.POINTER(c_int), c_int, c_dbl, c_dbl, c_dbl,
                                        c_dbl, c_int, c_vp],
    "advdiff_diffusion3d_step_putv": [c_int, c_vp, c_vp, c_int, c_int, c_i64, c_i64, c_int,
                                      c_int, c_int, c_int, c_int, c_int, c_int, c_dbl, c_dbl,
                                      c_dbl, c_dbl, c_int, ctypes.POINTER(c_vp),
                                      ctypes.POINTER(c_int), ctypes.POINTER(c_int),
                                      ctypes.POINTER(c_int), ctypes.POINTER(c_int),
                                      ctypes.POINTER(c_i64), c_vp],
    "advdiff_diffusion3d_step_put": [c_int, c_vp, c_vp, c_int, c_int, c_i64, c_i64, c_int,
                                     c_int, c_int, c_int, c_int, c_int, c_int, c_dbl, c_dbl,
                                     c_dbl, c_dbl, c_vp, c_int, c_int, c_vp, c_int, c_int,
                                     c_vp],
    "advdiff_diffusion2d_step_box": [c_int, c_vp, c_vp, c_int, c_i64, c_int, c_int, c_int,
                                     c_int, c_int, ctypes.POINTER(c_int), c_int, c_dbl, c_dbl,
                                     c_dbl, c_vp],
    "advdiff_diffusion2d_stage": [c_int, c_vp, c_vp, c_vp, c_int, c_i64, c_int, c_int, c_int,
                                  c_int, c_dbl, c_dbl, c_dbl, c_dbl, c_dbl, c_vp],
    "advdiff_burgers3d_stage": [c_int, c_vp, c_vp, c_vp, c_int, c_int, c_i64, c_i64, c_int,
                                c_int, c_int, c_int, c_dbl, c_dbl, c_dbl, c_dbl, c_dbl, c_dbl,
                                c_dbl, c_dbl, c_dbl, c_vp],
    "advdiff_burgers2d_stage": [c_int, c_vp, c_vp, c_vp, c_int, c_i64, c_int, c_int, c_int,
                                c_int, c_dbl, c_dbl, c_dbl, c_dbl, c_dbl, c_dbl, c_dbl, c_vp],
    "advdiff_burgers3d_stage_dt": [c_int, c_vp, c_vp, c_vp, c_int, c_int, c_i64, c_i64, c_int,
                                   c_int, c_int, c_int, c_dbl, c_dbl, c_dbl, c_dbl, c_dbl,
                                   c_dbl, c_dbl, c_dbl, c_dbl, c_int, c_vp, c_vp],
    "advdiff_burgers3d_stage2_dt": [c_int, c_vp, c_vp, c_vp, c_int, c_int, c_i64, c_i64, c_int,
                                    c_int, c_int, c_int, c_int, c_int, c_dbl, c_dbl, c_dbl,
                                    c_dbl, c_dbl, c_dbl, c_dbl, c_dbl, c_dbl, c_int, c_vp,
                                    c_vp],
    "advdiff_burgers3d_stage_put": [c_int, c_vp, c_vp, c_vp, c_int, c_int, c_i64, c_i64, c_int,
                                    c_int, c_int, c_int, c_dbl, c_dbl, c_dbl, c_dbl, c_dbl,
                                    c_dbl, c_dbl, c_dbl, c_dbl, c_vp, c_vp, c_int, c_int, c_vp,
                                    c_int, c_int, c_vp],
    "advdiff_burgers2d_stage_dt": [c_int, c_vp, c_vp, c_vp, c_int, c_i64, c_int, c_int, c_int,
                                   c_int, c_dbl, c_dbl, c_dbl, c_dbl, c_dbl, c_dbl, c_dbl, c_int,
                                   c_vp, c_vp],
    "advdiff_preload": [],
    "advdiff_adaptive_dt": [c_vp, c_vp, c_dbl, c_dbl, c_dbl, c_int, c_vp],
    "advdiff_reduce_norms": [c_int, c_vp, c_vp, c_i64, c_i64, c_int, c_int, c_int, c_int,
                             c_int, c_int, c_vp, c_vp, c_vp],
    "advdiff_init_ic": [c_int, c_int, c_vp, c_int, c_int, c_int, c_i64, c_i64, c_int, c_int,
                        c_int, c_int, c_dbl, c_dbl, c_dbl, c_dbl, c_dbl, c_vp],
    "advdiff_init_ic_box": [c_int, c_int, c_vp, c_int, c_int, c_int, c_i64, c_i64, c_int,
                            c_int, c_int, c_int, c_int, c_int, c_dbl, c_dbl, c_dbl, c_dbl,
                            c_dbl, c_vp],
    "advdiff_debug_print": [c_int, c_vp, c_i64, c_i64, c_int, c_int, c_int, c_int, c_int,
                            c_int, c_vp],
    "advdiff_copy_box": [c_int, c_vp, c_i64, c_i64, c_vp, c_i64, c_i64, c_int, c_int, c_int,
                         c_vp],
}


class IpcAddr(ctypes.Structure):
    """advdiff_ipc_addr (kernels.h): IPC handle of an allocation + byte offset."""
    _fields_ = [("handle", ctypes.c_ubyte * 64), ("offset", ctypes.c_uint64),
                ("bytes", ctypes.c_uint64)]


_IPC_SIGS = {
    "advdiff_ipc_create": [c_int, c_int, ctypes.POINTER(c_vp)],
    "advdiff_ipc_destroy": [c_vp],
    "advdiff_ipc_describe": [c_vp, c_vp, ctypes.POINTER(IpcAddr)],
    "advdiff_ipc_flags_addr": [c_vp, ctypes.POINTER(IpcAddr)],
    "advdiff_ipc_map": [c_vp, ctypes.POINTER(IpcAddr), ctypes.POINTER(c_vp)],
    "advdiff_ipc_set_peer": [c_vp, c_int, ctypes.POINTER(IpcAddr)],
    "advdiff_ipc_put": [c_int, c_vp, c_i64, c_i64, c_vp, c_i64, c_i64, c_int, c_int, c_int,
                        c_vp],
    "advdiff_ipc_signal": [c_vp, ctypes.POINTER(c_int), c_int, c_vp],
    "advdiff_ipc_signal_ch": [c_vp, c_int, ctypes.POINTER(c_int), c_int, c_vp],
    "advdiff_ipc_wait_ch": [c_vp, c_int, ctypes.POINTER(c_int), c_int, c_vp],
    "advdiff_ipc_wait": [c_vp, ctypes.POINTER(c_int), c_int, c_vp],
    "advdiff_ipc_errors": [c_vp, ctypes.POINTER(ctypes.c_longlong)],
    "advdiff_ipc_reset": [c_vp],
}

# low-storage RK variants share the signature of the SSP stage entries
for _k in ("advdiff_diffusion3d_stage", "advdiff_diffusion2d_stage", "advdiff_burgers3d_stage",
           "advdiff_burgers2d_stage"):
    _SIGS[_k + "_ls"] = _SIGS[_k]


def source_hash() -> str | None:
    """Hash of the library sources in this tree, exactly as ``csrc/Makefile`` computes
    SRC_HASH (sha256 of the contents of kernels/*.hip, kernels/*.hpp and
    include/advdiff/kernels.h concatenated in sorted relative-path order; 16 hex digits).
    None when the tree carries no csrc/ (an installed copy)."""
    kdir = CSRC / "kernels"
    if not kdir.is_dir():
        return None
    rel = sorted([f"kernels/{p.name}" for p in kdir.iterdir() if p.suffix in (".hip", ".hpp")]
                 + ["include/advdiff/kernels.h"])
    h = hashlib.sha256()
    for r in rel:
        h.update((CSRC / r).read_bytes())
    return h.hexdigest()[:16]


def _load():
    global _lib, _err
    with _lock:
        if _lib is not None or _err is not None:
            return _lib
        if not LIB_PATH.exists():
            _err = f"{LIB_PATH} not built (run `python -c 'import __graft_entry__ as g; g.build()'` or `make -C csrc`)"
            return None
        try:
            lib = ctypes.CDLL(str(LIB_PATH))
        except OSError as e:  # missing HIP runtime etc.
            _err = f"failed to load {LIB_PATH}: {e}"
            return None
        # A library built from other sources than this tree's is refused: every GPU result
        # must come from code that is in the tree (ADVDIFF_ALLOW_STALE=1 overrides, for A/B).
        try:
            lib.advdiff_source_hash.restype = ctypes.c_char_p
            built = lib.advdiff_source_hash().decode()
        except AttributeError:  # built before the hash existed
            built = "unknown"
        tree = source_hash()
        if tree is not None and built != tree and os.environ.get("ADVDIFF_ALLOW_STALE") != "1":
            _err = (f"{LIB_PATH} is stale: built from sources {built}, tree is {tree} "
                    f"(rebuild with `make -C csrc`)")
            return None
        for name, args in _SIGS.items():
            fn = getattr(lib, name)
            fn.argtypes = args
            fn.restype = c_int
        lib.advdiff_set_b3_ver.argtypes = [c_int]
        lib.advdiff_set_b3_ver.restype = c_int
        lib.advdiff_step_bands_plan.argtypes = [c_int, ctypes.c_longlong, ctypes.c_longlong,
                                                c_int, c_int, ctypes.POINTER(ctypes.c_longlong)]
        lib.advdiff_step_bands_plan.restype = c_int
        lib.advdiff_set_step_banded.argtypes = [c_int]
        lib.advdiff_set_step_banded.restype = c_int
        lib.advdiff_set_b3_pack.argtypes = [c_int]
        lib.advdiff_set_b3_pack.restype = c_int
        lib.advdiff_set_b3_tx.argtypes = [c_int]
        lib.advdiff_set_b3_tx.restype = c_int
        lib.advdiff_set_b3_zchunk.argtypes = [c_int]
        lib.advdiff_set_b3_zchunk.restype = c_int
        lib.advdiff_set_b2_ver.argtypes = [c_int]
        lib.advdiff_set_b2_ver.restype = c_int
        for name, args in _IPC_SIGS.items():
            fn = getattr(lib, name)
            fn.argtypes = args
            fn.restype = c_int
        lib.advdiff_reduce_workspace_bytes.restype = c_sz
        lib.advdiff_reduce_workspace_bytes.argtypes = []
        lib.advdiff_build_info.restype = ctypes.c_char_p
        lib.advdiff_device_info.argtypes = [c_int, ctypes.POINTER(c_i64), c_int]
        lib.advdiff_device_info.restype = c_int
        lib.advdiff_peer_info.argtypes = [c_int, c_int] + [ctypes.POINTER(c_int)] * 3
        lib.advdiff_peer_info.restype = c_int
        _lib = lib
        return _lib


def available() -> bool:
    return _load() is not None


def load_error() -> str | None:
    _load()
    return _err


def require():
    lib = _load()
    if lib is None:
        raise RuntimeError(f"advdiff native kernels unavailable: {_err}")
    return lib


_preloaded = set()


def preload(device_index: int) -> None:
    """Load every kernel file's code object on `device_index` now (advdiff_preload): the
    HIP runtime otherwise loads each at its first launch (~20 ms for the WENO5 file),
    inside whatever the caller is timing.  Once per device and process."""
    if device_index in _preloaded:
        return
    import torch
    lib = require()
    with torch.cuda.device(device_index):
        check(lib.advdiff_preload(), "advdiff_preload")
    _preloaded.add(device_index)


def check(code: int, what: str) -> None:
    if code != 0:
        raise RuntimeError(f"{what} failed with hipError_t {code}")


def build_info() -> str:
    lib = require()
    return f"{lib.advdiff_build_info().decode()} [src {lib.advdiff_source_hash().decode()}]"


def library_hash() -> str:
    return require().advdiff_source_hash().decode()
