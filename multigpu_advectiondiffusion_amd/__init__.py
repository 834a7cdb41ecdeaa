"""multigpu_advectiondiffusion_amd — an MI355X-native (gfx950 / CDNA4) advection-diffusion
stencil framework with the capabilities of cfd-learner/MultiGPU_AdvectionDiffusion.

Layers (SURVEY.md §1 mapping):
  L1/L2  csrc/kernels/*.hip -> lib/libadvdiff.so (C ABI)   -> ops/ (ctypes + torch reference)
  L3     parallel/ (torch.distributed RCCL/gloo, slab decomposition, halo exchange)
  L4     solver.Solver (SSP-RK3 engine, overlap scheduler), models/ (physics)
  L5/L6  cli.py / launch.py / bench.py, csrc/apps (native C++ executables)
"""
__version__ = "0.1.0"

from .models import Burgers, Diffusion, Grid  # noqa: E402
from .solver import Solver  # noqa: E402

__all__ = ["Burgers", "Diffusion", "Grid", "Solver", "__version__"]
