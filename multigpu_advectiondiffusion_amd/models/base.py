"""Model interface: a PDE right-hand side that knows how to run one fused SSP-RK3 stage.

A *model* is the analogue of one reference application's physics (`Diffusion2d/3d`,
`Burgers2d/3d`): it owns the constants (diffusivity, viscosity, scheme options), the
stencil radius (= ghost width) and frozen-border width, the time-step rule, and the
launch of the fused stage kernel on a range of local planes.  Everything about
parallelism, buffers, streams and time looping lives in ``solver.Solver``.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field


@dataclass(frozen=True)
class Grid:
    """Vertex-centred uniform grid: x_i = i*dx on [0, L], dx = L/(n-1)
    (`MultiGPU/Diffusion3d_Baseline/main.c:61-63`).  shape = (nx, ny[, nz])."""
    shape: tuple
    lengths: tuple

    def __post_init__(self):
        if len(self.shape) not in (2, 3) or len(self.lengths) != len(self.shape):
            raise ValueError("Grid needs 2 or 3 extents and matching lengths")
        if any(n < 2 for n in self.shape):
            raise ValueError("every extent must be >= 2")

    @property
    def dims(self) -> int:
        return len(self.shape)

    @property
    def spacing(self) -> tuple:
        return tuple(L / (n - 1) for n, L in zip(self.shape, self.lengths))

    @property
    def cells(self) -> int:
        return math.prod(self.shape)

    @property
    def nx(self):
        return self.shape[0]

    @property
    def ny(self):
        return self.shape[1]

    @property
    def nz(self):
        return self.shape[2] if self.dims == 3 else 1

    @property
    def n_decomposed(self) -> int:
        """Extent of the slowest (decomposed, marched) axis: z in 3-D, y in 2-D."""
        return self.shape[-1]


class Model:
    """Base class. Subclasses set ``name``, ``radius``, ``border`` and implement
    ``stage`` and ``stable_dt``."""
    name = "model"
    title = "Model"          # for the summary banner
    radius = 2               # stencil radius = ghost width
    border = 2               # frozen Dirichlet layer width
    flops_per_cell = 8.0     # reference's FLOPS constant (metric only)
    bytes_per_cell_step = 64.0  # HBM traffic estimate of the fused path (metric only)
    needs_umax = False
    supports_fused = False   # one launch per full RK3 step (ghost width 3R)

    def stage_put_ok(self, dtype) -> bool:
        """The per-stage launch can carry fused halo puts (slab ranks, ipc)."""
        return False
    supports_step2 = False   # one launch per TWO RK3 steps (single rank)

    def bind(self, grid: Grid) -> None:
        self.grid = grid

    def stage(self, inp, u0, out, lo, hi, dt, a, b, stream=None, nx=None, ny=None,
              border=None, ls=False):  # pragma: no cover
        raise NotImplementedError

    def stable_dt(self, umax: float | None = None) -> float:  # pragma: no cover
        raise NotImplementedError

    # -- RHS-exchange stages (Solver(exchange="lu"), the reference's MultiGPU scheme) --
    def rhs(self, inp, L, lo, hi) -> None:  # pragma: no cover
        """L[lo:hi] = the spatial operator of `inp` on planes [lo, hi) (active x/y cells;
        PyTorch ops)."""
        raise NotImplementedError

    def _active(self, t, lo, hi):
        """View of planes [lo, hi), x/y cells inside the frozen border."""
        B = self.border
        if self.grid.dims == 3:
            return t[lo:hi, B:self.grid.ny - B, B:self.grid.nx - B]
        return t[lo:hi, B:self.grid.nx - B]

    def rk_update(self, inp, u0, out, L, lo, hi, dt, a, b, ls=False) -> None:
        """out = a·u0 + b·(inp + dt·L) on planes [lo, hi) — the combine of the fused stage
        (ops/reference.py::_combine), bit for bit."""
        if hi <= lo:
            return
        from ..ops import reference as ref
        v = self._active
        ref._combine(v(out, lo, hi), v(u0, lo, hi) if (a != 0 or ls) else None,
                     v(inp, lo, hi), v(L, lo, hi), dt, a, b, ls)

    def describe(self) -> dict:
        return {"model": self.name, "radius": self.radius, "border": self.border}


@dataclass
class RunStats:
    steps: int = 0
    t: float = 0.0
    compute_s: float = 0.0
    htod_s: float = 0.0
    dtoh_s: float = 0.0
    extra: dict = field(default_factory=dict)
