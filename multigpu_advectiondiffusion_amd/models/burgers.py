"""Burgers u_t + Σ_d ∂_d(u²/2) = C ∇²u (2-D / 3-D) with WENO5 flux splitting.

Reference apps: MultiGPU Burgers2d/3d_Baseline (inviscid, WENO5-JS), SingleGPU
Burgers3d_WENO5{,_PitchedMem,_SharedMem,_TextureMem,_Hybrid,_Hybrid2} (viscous C=1e-5,
WENO5-Z), Matlab_Prototipes/InviscidBurgersNd (WENO5-JS).  One fused HIP kernel per
dimensionality (``csrc/kernels/burgers.hip``) covers all of them: ``weno="js"|"z"``,
``viscosity=0`` compiles the viscous term out.

Time step (`SingleGPU/Burgers3d_WENO5/main.cpp:130-133`, `MultiGPU/Burgers3d_Baseline/main.c:193`):
    dt = min(CFL·min(d)/umax, 0.9 / (2C Σ 1/d²))
The reference hard-codes umax = 1 (no reduction).  ``cfl_mode="fixed"``
keeps that (default: matches the reference step count); ``"adaptive"`` uses the true
global max|u| (as the MATLAB prototype `LFWENO5FDM3d.m:71`) computed ON THE DEVICE every
step — norm reducer -> RCCL MAX allreduce on the stream -> ``advdiff_adaptive_dt`` ->
the stage kernels read dt from device memory — so the step loop never waits for the
host and single-process runs replay it as hipGraphs (solver.py ``_run_device_dt``).

Deltas by design: each face flux is computed once (the reference's MultiGPU x-sweep
starts at i=2 with a zero "old" flux — quirk #8 — and the SingleGPU y-sweep covers
i < Ny only — quirk #6); frozen Dirichlet border of 3 cells on every face.
"""
from __future__ import annotations

import torch

from ..ops import stencil
from .base import Model


class Burgers(Model):
    name = "burgers"

    def __init__(self, viscosity: float = 0.0, weno: str = "z", cfl: float = 0.3,
                 cfl_mode: str = "fixed", umax: float = 1.0, border: int | None = None):
        if weno not in ("js", "z", "js7"):
            raise ValueError("weno must be 'js' (WENO5 Jiang-Shu), 'z' (WENO5 Borges-Z) or "
                             "'js7' (WENO7 Jiang-Shu, the MATLAB LFWENO7 prototype)")
        if cfl_mode not in ("fixed", "adaptive"):
            raise ValueError("cfl_mode must be 'fixed' or 'adaptive'")
        self.C = float(viscosity)
        self.weno = weno
        self.cfl = float(cfl)
        self.cfl_mode = cfl_mode
        self.umax = float(umax)
        self.radius = 4 if weno == "js7" else 3
        self.border = self.radius if border is None else int(border)
        if self.border < self.radius:
            raise ValueError(f"WENO needs a frozen border >= {self.radius}")
        self.needs_umax = cfl_mode == "adaptive"

    def bind(self, grid):
        super().bind(grid)
        d = grid.spacing
        self.dims = grid.dims
        self.rd = tuple(1.0 / h for h in d)
        self.visc = tuple(self.C / (h * h) for h in d)
        kind = {"z": "WENO5-Z", "js": "WENO5-JS", "js7": "WENO7-JS"}[self.weno]
        self.title = f"Burgers-{grid.dims}D MI355X-{kind}"

    @property
    def bytes_per_cell_step(self):
        return 64.0

    def stable_dt(self, umax=None) -> float:
        u = self.umax if (umax is None or self.cfl_mode == "fixed") else max(umax, 1e-300)
        dt = self.cfl * min(self.grid.spacing) / u
        if self.C > 0:
            dt = min(dt, 0.9 / (2.0 * sum(self.visc)))
        return dt

    def cfl_terms(self):
        """(cfl * min(d), viscous dt limit or 0): stable_dt(umax) = min(cfl_h / umax, dv),
        the two constants of the device-side adaptive step (ops/stencil.py adaptive_dt)."""
        dv = 0.9 / (2.0 * sum(self.visc)) if self.C > 0 else 0.0
        return self.cfl * min(self.grid.spacing), dv

    # stage() takes a second plane range (lo2, hi2): the 3-D kernel serves both boundary
    # slabs of a slab rank in one launch
    two_range_stage = True

    def stage_put_ok(self, dtype) -> bool:
        """The stage can carry fused halo puts (advdiff_burgers3d_stage_put)."""
        return self.dims == 3 and self.weno in ("js", "z") and dtype == torch.float64

    def stage(self, inp, u0, out, lo, hi, dt, a, b, stream=None, nx=None, ny=None,
              border=None, ls=False, dt_dev=None, lo2=0, hi2=0, put=None):
        g = self.grid
        nx = g.nx if nx is None else nx
        ny = g.ny if ny is None else ny
        border = self.border if border is None else border
        z = self.weno
        if self.dims == 3:
            stencil.burgers3d_stage(inp, u0, out, nx=nx, ny=ny, k0=lo, k1=hi,
                                    border=border, weno_z=z, rdx=self.rd[0],
                                    rdy=self.rd[1], rdz=self.rd[2], vx=self.visc[0],
                                    vy=self.visc[1], vz=self.visc[2], dt=dt, a=a, b=b,
                                    stream=stream, ls=ls, dt_dev=dt_dev, k0b=lo2, k1b=hi2,
                                    put=put)
        else:
            for j0, j1 in ((lo, hi), (lo2, hi2)):
                if j1 > j0:
                    stencil.burgers2d_stage(inp, u0, out, nx=nx, j0=j0, j1=j1, border=border,
                                            weno_z=z, rdx=self.rd[0], rdy=self.rd[1],
                                            vx=self.visc[0], vy=self.visc[1], dt=dt, a=a, b=b,
                                            stream=stream, ls=ls, dt_dev=dt_dev)

    def rhs(self, inp, L, lo, hi):
        if hi <= lo:
            return
        from ..ops import reference as ref
        g = self.grid
        if self.dims == 3:
            f = ref.burgers_rhs_3d(inp, g.nx, g.ny, lo, hi, self.border, self.weno, *self.rd,
                                   *self.visc)
        else:
            f = ref.burgers_rhs_2d(inp, g.nx, lo, hi, self.border, self.weno, *self.rd,
                                   *self.visc)
        self._active(L, lo, hi).copy_(f)

    def describe(self):
        d = super().describe()
        d.update({"viscosity": self.C, "weno": self.weno, "cfl": self.cfl,
                  "cfl_mode": self.cfl_mode})
        return d
