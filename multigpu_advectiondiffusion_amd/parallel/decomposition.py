"""Slab domain decomposition along the slowest axis (z in 3-D, y in 2-D).

Reference: `MultiGPU/Diffusion3d_Baseline/main.c:69-71` (``_Nz = Nz/P``, ``_NZ = _Nz+6``)
and the diagram in `DiffusionMPICUDA.h:31-43`.  Differences by design:

* remainders are allowed (the reference requires ``Nz % P == 0``): the first ``Nz % P``
  ranks own one extra plane;
* the ghost width G equals the stencil radius R of the model (2 for FD4, 1 for FD2,
  3 for WENO5) instead of a fixed 3;
* with x fastest and the decomposition along the slowest axis every halo is a
  contiguous block of G planes, so halo exchange needs no pack/unpack — RCCL sends
  straight out of, and receives straight into, the field buffers.

Local array layout along axis 0:  [ G ghost | n_own owned | G ghost ]
local index ``l`` <-> global plane ``start - G + l``.
"""
from __future__ import annotations

from dataclasses import dataclass


@dataclass(frozen=True)
class SlabDecomposition:
    n: int        # global extent of the decomposed axis
    size: int     # number of ranks
    rank: int
    ghost: int    # ghost width G (= stencil radius)

    def __post_init__(self):
        if self.size < 1 or not 0 <= self.rank < self.size:
            raise ValueError(f"bad rank {self.rank}/{self.size}")
        if self.n < self.size * max(self.ghost, 1):
            raise ValueError(
                f"{self.n} planes cannot be split over {self.size} ranks with ghost width "
                f"{self.ghost}: every rank needs >= {max(self.ghost, 1)} planes")

    # ---- ownership -------------------------------------------------------------
    def count_of(self, r: int) -> int:
        q, rem = divmod(self.n, self.size)
        return q + (1 if r < rem else 0)

    def start_of(self, r: int) -> int:
        q, rem = divmod(self.n, self.size)
        return r * q + min(r, rem)

    @property
    def count(self) -> int:
        return self.count_of(self.rank)

    @property
    def start(self) -> int:
        return self.start_of(self.rank)

    @property
    def stop(self) -> int:
        return self.start + self.count

    @property
    def alloc(self) -> int:
        return self.count + 2 * self.ghost

    @property
    def lower(self):
        return self.rank - 1 if self.rank > 0 else None

    @property
    def upper(self):
        return self.rank + 1 if self.rank < self.size - 1 else None

    # ---- local index helpers ------------------------------------------------------
    def to_local(self, g: int) -> int:
        return g - self.start + self.ghost

    @property
    def owned(self) -> tuple[int, int]:
        """Local index range of the owned planes."""
        return self.ghost, self.ghost + self.count

    def compute_range(self, border: int) -> tuple[int, int]:
        """Local range of owned planes that are updated (global planes in
        [border, n-border) are interior; the rest are frozen Dirichlet layers)."""
        lo = max(self.start, border)
        hi = min(self.stop, self.n - border)
        if hi <= lo:
            return self.ghost, self.ghost
        return self.to_local(lo), self.to_local(hi)

    def split_ranges(self, border: int, radius: int):
        """Split the compute range into (interior, boundary_lo, boundary_hi).

        * boundary_lo: planes whose stencil reads the LOWER ghost planes (only if a lower
          neighbour exists), boundary_hi likewise for the upper side;
        * interior: everything else — computable while the halo is in flight.
        Ranges are half-open local (lo, hi) tuples and may be empty (lo == hi).
        """
        lo, hi = self.compute_range(border)
        o0, o1 = self.owned
        if hi <= lo:
            e = (lo, lo)
            return e, e, e
        blo_end = min(hi, o0 + radius) if self.lower is not None else lo
        bhi_start = max(lo, o1 - radius) if self.upper is not None else hi
        blo = (lo, max(lo, blo_end))
        if bhi_start < blo[1]:  # slab thinner than 2R: one boundary launch, no interior
            return (blo[1], blo[1]), (lo, hi), (hi, hi)
        bhi = (bhi_start, hi)
        interior = (blo[1], bhi_start)
        return interior, blo, bhi

    # ---- halo geometry (local index ranges) -------------------------------------
    def send_lower(self):
        o0, _ = self.owned
        return o0, o0 + self.ghost

    def send_upper(self):
        _, o1 = self.owned
        return o1 - self.ghost, o1

    def recv_lower(self):
        return 0, self.ghost

    def recv_upper(self):
        _, o1 = self.owned
        return o1, o1 + self.ghost


def weak_scaling_grid(base: int, nranks: int, dims: int = 3) -> tuple:
    """Global grid for weak scaling with `base`^dims cells per rank: the factors of
    nranks (a power of two) are spread over the axes, z first, so 1 -> base³,
    2 -> (base, base, 2base), 4 -> (base, 2base, 2base), 8 -> (2base)³."""
    f = [1] * dims
    n = nranks
    ax = dims - 1
    while n > 1:
        if n % 2:
            f[dims - 1] *= n
            break
        f[ax] *= 2
        n //= 2
        ax = (ax - 1) % dims
    return tuple(base * x for x in f)
