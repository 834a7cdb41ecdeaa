"""Heat equation u_t = K ∇²u (2-D / 3-D), FD4 (13-point in 3-D, 9-point in 2-D) or FD2.

Reference apps: MultiGPU Diffusion2d/3d_Baseline, SingleGPU
Diffusion2d{,_PitchedMem,_TextureMem}, Diffusion3d_{baselineCode,PitchedMem,Blocking},
Matlab_Prototipes/DiffusionNd.  All memory variants collapse into one fused kernel
(``csrc/kernels/diffusion.hip``).

Deliberate deltas from the reference:
* every axis uses its own coefficient K/(12 d²) (the MultiGPU 3-D kernel used
  ``diff_x/12`` for all axes, an effective K/12 — quirk #2);
* the fixed time step is ``safety / (2K Σ 1/d²)`` with safety 0.9 (SingleGPU,
  `SingleGPU/Diffusion3d_baselineCode/main.cpp:58`) by default; ``safety=0.8``
  reproduces the MultiGPU choice (`MultiGPU/Diffusion3d_Baseline/main.c:64`);
* iteration counts are exact (the MultiGPU ``while t < dt*iters`` loop ran iters+1).
"""
from __future__ import annotations

import os

from ..ops import stencil
from .base import Model


class Diffusion(Model):
    name = "diffusion"

    def __init__(self, K: float = 1.0, order: int = 4, safety: float = 0.9, border=None,
                 fused: bool = True):
        if order not in (2, 4):
            raise ValueError("order must be 2 (7-pt) or 4 (13-pt)")
        self.K = float(K)
        self.order = order
        self.safety = float(safety)
        self.radius = order // 2
        self.border = self.radius if border is None else int(border)
        if self.border < self.radius:
            raise ValueError("frozen border must be >= stencil radius")
        self.fused = bool(fused)

    def bind(self, grid):
        super().bind(grid)
        d = grid.spacing
        self.coef = tuple(self.K / (h * h) for h in d)
        self.dims = grid.dims
        self.title = f"Diffusion-{grid.dims}D MI355X-FD{self.order}"

    @property
    def supports_fused(self) -> bool:
        """One temporally blocked launch per RK3 step (diffusion_fused.hip in 3-D,
        diffusion2d_fused.hip in 2-D)."""
        return self.fused

    @property
    def bytes_per_cell_step(self):
        # fused step: read u^n + write u^{n+1}; per-stage: 16 + 24 + 24 B
        return 16.0 if self.supports_fused else 64.0

    @property
    def supports_step2(self) -> bool:
        """Two RK3 steps per launch (3-D FD2, one rank: diffusion_fused.hip v6_march, half
        the HBM traffic per step).  ADVDIFF_STEP2=0 keeps one step per launch."""
        return (self.fused and self.dims == 3 and self.order == 2
                and os.environ.get("ADVDIFF_STEP2", "1") != "0")

    def step2_preferred(self, uin, uout, lo, hi, zlo, zhi, dt) -> bool:
        """Two steps per launch faster than one for this shape (measured on the GPU,
        stencil.diffusion3d_step2_pick; uout is scratch)."""
        g = self.grid
        return stencil.diffusion3d_step2_pick(uin, uout, nx=g.nx, ny=g.ny, k0=lo, k1=hi,
                                              zlo=zlo, zhi=zhi, border=self.border,
                                              cx=self.coef[0], cy=self.coef[1], cz=self.coef[2],
                                              dt=dt)

    def sched_pick(self, uin, uout, lo, hi, zlo, zhi, dt, nx=None, ny=None, box=None) -> bool:
        """Banded or uniform z chunks for this 3-D fused launch, measured on the GPU
        (stencil.diffusion3d_step_sched_pick; uout is scratch).  2-D: nothing to pick."""
        if self.dims != 3:
            return False
        g = self.grid
        return stencil.diffusion3d_step_sched_pick(
            uin, uout, nx=g.nx if nx is None else nx, ny=g.ny if ny is None else ny, k0=lo,
            k1=hi, zlo=zlo, zhi=zhi, border=self.border, order=self.order, cx=self.coef[0],
            cy=self.coef[1], cz=self.coef[2], dt=dt, box=box)

    def step2(self, uin, uout, lo, hi, zlo, zhi, dt, stream=None):
        """Two fused RK3 steps on planes [lo, hi) of a whole (one-rank) field."""
        g = self.grid
        stencil.diffusion3d_step2x(uin, uout, nx=g.nx, ny=g.ny, k0=lo, k1=hi, zlo=zlo, zhi=zhi,
                                   border=self.border, cx=self.coef[0], cy=self.coef[1],
                                   cz=self.coef[2], dt=dt, stream=stream)

    def step(self, uin, uout, lo, hi, zlo, zhi, dt, stream=None, lo2=0, hi2=0, nx=None,
             ny=None, box=None, exclusive=False, put=None):
        """Fused RK3 step on planes [lo, hi) (and [lo2, hi2) in the same launch).
        nx/ny/box: extents and explicit active/output bounds of a view (Cartesian blocks).
        exclusive: the launch has the GPU to itself (3-D: persistent schedule; the 2-D
        step has one grid schedule — its y-march waves are independent — and ignores it).
        put: fused halo puts of a 3-D slab rank (stencil.diffusion3d_step)."""
        g = self.grid
        nx = g.nx if nx is None else nx
        ny = g.ny if ny is None else ny
        if self.dims == 2:
            for a, b in ((lo, hi), (lo2, hi2)):
                if b > a:
                    stencil.diffusion2d_step(uin, uout, nx=nx, j0=a, j1=b, ylo=zlo, yhi=zhi,
                                             border=self.border, order=self.order,
                                             cx=self.coef[0], cy=self.coef[1], dt=dt,
                                             stream=stream, box=box)
            return
        stencil.diffusion3d_step(uin, uout, nx=nx, ny=ny, k0=lo, k1=hi, zlo=zlo, zhi=zhi,
                                 border=self.border, order=self.order, cx=self.coef[0],
                                 cy=self.coef[1], cz=self.coef[2], dt=dt, stream=stream,
                                 k0b=lo2, k1b=hi2, box=box, exclusive=exclusive, put=put)

    def stable_dt(self, umax=None) -> float:
        return self.safety / (2.0 * sum(self.coef))

    def stage(self, inp, u0, out, lo, hi, dt, a, b, stream=None, nx=None, ny=None,
              border=None, ls=False):
        """nx/ny/border override the grid's for launches on a sub-box view (Cartesian)."""
        g = self.grid
        nx = g.nx if nx is None else nx
        ny = g.ny if ny is None else ny
        border = self.border if border is None else border
        if self.dims == 3:
            stencil.diffusion3d_stage(inp, u0, out, nx=nx, ny=ny, k0=lo, k1=hi,
                                      border=border, order=self.order, cx=self.coef[0],
                                      cy=self.coef[1], cz=self.coef[2], dt=dt, a=a, b=b,
                                      stream=stream, ls=ls)
        else:
            stencil.diffusion2d_stage(inp, u0, out, nx=nx, j0=lo, j1=hi, border=border,
                                      order=self.order, cx=self.coef[0], cy=self.coef[1],
                                      dt=dt, a=a, b=b, stream=stream, ls=ls)

    def rhs(self, inp, L, lo, hi):
        if hi <= lo:
            return
        from ..ops import reference as ref
        g = self.grid
        if self.dims == 3:
            lap = ref.diffusion3d_rhs(inp, g.nx, g.ny, lo, hi, self.border, self.order,
                                      *self.coef)
        else:
            lap = ref.diffusion2d_rhs(inp, g.nx, lo, hi, self.border, self.order, *self.coef)
        self._active(L, lo, hi).copy_(lap)

    def describe(self):
        d = super().describe()
        d.update({"K": self.K, "order": self.order, "safety": self.safety,
                  "fused_step": self.supports_fused})
        return d
