"""Stencil ops: hand-written gfx950 HIP kernels (``libadvdiff.so`` via ctypes) for device
tensors, PyTorch reference implementations for CPU tensors."""
from . import reference
from ._lib import available as native_available
from ._lib import build_info, load_error
from .stencil import (NormReducer, burgers2d_stage, burgers3d_stage, copy_box,
                      diffusion2d_stage, diffusion3d_stage, diffusion3d_step,
                      diffusion3d_step2x,
                      init_ic_device)

__all__ = ["reference", "native_available", "build_info", "load_error", "NormReducer",
           "burgers2d_stage", "burgers3d_stage", "copy_box", "diffusion2d_stage",
           "diffusion3d_stage", "diffusion3d_step", "diffusion3d_step2x", "init_ic_device"]
