"""Per-GPU problem sizing for 288 GB of HBM3E (MI355X).

Device memory of a solver = number of resident fields × local cells (ghost planes, the
256-B row padding and the pitch pads of solver.pitch_default included) × element size; everything else (reduction workspace, halo
pack buffers of a Cartesian grid) is negligible.  Resident fields:

=============================  =======  =======================================
path                           fields   buffers
=============================  =======  =======================================
3-D heat, fused SSP-RK3 step   2        u, u' (ping-pong)
SSP-RK3 per stage              3        u, A, B (stage 3 writes u in place)
low-storage RK4(5)             3        u, u' (ping-pong), du
=============================  =======  =======================================

So one MI355X holds a 2048³ fp64 heat problem (2 × 68.7 GB) or a 2048³ fp64 Burgers
problem (3 × 68.7 GB = 206 GB) — and an 8-GPU node 4096³ heat cells.

    python -m multigpu_advectiondiffusion_amd.utils.sizing [--mem-gb 288] [--gpus 8]
"""
from __future__ import annotations

import argparse
import math

HBM_BYTES_MI355X = 288 * 10 ** 9


def fields_resident(fused: bool, integrator: str = "ssprk3") -> int:
    if integrator == "lsrk45":
        return 3
    return 2 if fused else 3


def row_pitch(nx: int, elem: int, align: int = 256) -> int:
    per = max(align // elem, 1)
    return (nx + per - 1) // per * per


def solver_bytes(shape_local_alloc, elem: int, fields: int, pitch=None,
                 cells_per_rank: int | None = None) -> int:
    """Bytes of the resident fields for a local allocation (array order, last axis x);
    pitch = (extra elements per row, extra rows per 3-D plane), None = the solver's
    default rule (solver.pitch_default), which the Solver applies to the GLOBAL cells per
    rank (grid.cells // world, ghosts excluded): pass that as cells_per_rank.  Without
    it the owned cells are taken as the allocation minus nothing — callers that size a
    ghost-inclusive block should pass cells_per_rank, or the rule can flip near its
    threshold."""
    *outer, nx = shape_local_alloc
    if pitch is None:
        from ..solver import pitch_default
        n = math.prod(shape_local_alloc) if cells_per_rank is None else int(cells_per_rank)
        pitch = pitch_default(len(shape_local_alloc), elem, n)
    if len(outer) == 2:
        outer = [outer[0], outer[1] + pitch[1]]
    return fields * math.prod(outer) * (row_pitch(nx, elem) + pitch[0]) * elem


def max_cube(mem_bytes: int = HBM_BYTES_MI355X, elem: int = 8, fields: int = 2,
             ghost: int = 6, headroom: float = 0.92, multiple: int = 64) -> int:
    """Largest n (a multiple of `multiple`) with an n³ slab (+2·ghost planes) fitting in
    `headroom` × mem_bytes."""
    budget = headroom * mem_bytes
    n = multiple
    while solver_bytes((n + multiple + 2 * ghost, n + multiple, n + multiple), elem,
                       fields, cells_per_rank=(n + multiple) ** 3) <= budget:
        n += multiple
    return n


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--mem-gb", type=float, default=HBM_BYTES_MI355X / 1e9)
    ap.add_argument("--gpus", type=int, default=1)
    a = ap.parse_args(argv)
    mem = int(a.mem_gb * 1e9)
    for label, fields, ghost in (("heat 3-D fused step (fp64)", 2, 6),
                                 ("heat / Burgers SSP-RK3 per stage (fp64)", 3, 3),
                                 ("Burgers WENO7 + LSRK4(5) (fp64)", 3, 4)):
        n = max_cube(mem, 8, fields, ghost)
        print(f"{label:42s}: {n}^3 per GPU ({fields} fields, "
              f"{solver_bytes((n + 2 * ghost, n, n), 8, fields, cells_per_rank=n ** 3) / 1e9:.0f} GB); "
              f"{a.gpus} GPUs (z-slabs): {n}x{n}x{n * a.gpus}")


if __name__ == "__main__":
    main()
