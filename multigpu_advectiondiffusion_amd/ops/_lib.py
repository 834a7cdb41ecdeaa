"""ctypes binding of ``lib/libadvdiff.so`` (the hand-written gfx950 HIP kernels).

The library exposes a plain C ABI (``csrc/include/advdiff/kernels.h``) so the very same
kernels serve the Python/PyTorch path (device tensors' ``data_ptr()`` + the current HIP
stream handle) and the native C++ apps.  Loading is lazy; on a machine with a GPU the
ops refuse to silently fall back to PyTorch (``require()`` raises), so a test that passes
on a GPU box has provably run the native kernels.
"""
from __future__ import annotations

import ctypes
import os
import threading
from pathlib import Path

_LIB_DIR = Path(__file__).resolve().parent.parent / "lib"
LIB_PATH = Path(os.environ.get("ADVDIFF_LIB", _LIB_DIR / "libadvdiff.so"))

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
    "advdiff_diffusion3d_step_box": [c_int, c_vp, c_vp, c_int, c_int, c_i64, c_i64, c_int,
                                     c_int, c_int, c_int, c_int, c_int, c_int,
                                     ctypes.POINTER(c_int), c_int, c_dbl, c_dbl, c_dbl, c_dbl,
                                     c_vp],
    "advdiff_diffusion3d_step_box_ex": [c_int, c_vp, c_vp, c_int, c_int, c_i64, c_i64, c_int,
                                        c_int, c_int, c_int, c_int, c_int, c_int,
                                        ctypes.POINTER(c_int), c_int, c_dbl, c_dbl, c_dbl,
                                        c_dbl, c_int, c_vp],
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

# low-storage RK variants share the signature of the SSP stage entries
for _k in ("advdiff_diffusion3d_stage", "advdiff_diffusion2d_stage", "advdiff_burgers3d_stage",
           "advdiff_burgers2d_stage"):
    _SIGS[_k + "_ls"] = _SIGS[_k]


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
        for name, args in _SIGS.items():
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


def check(code: int, what: str) -> None:
    if code != 0:
        raise RuntimeError(f"{what} failed with hipError_t {code}")


def build_info() -> str:
    return require().advdiff_build_info().decode()
