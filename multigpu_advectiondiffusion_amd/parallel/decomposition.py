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


# ---------------------------------------------------------------------------------------
# Cartesian (2-D / 3-D) process grids
# ---------------------------------------------------------------------------------------
def _prod(xs):
    p = 1
    for x in xs:
        p *= x
    return p


def parse_proc_grid(spec, world: int, shape_array: tuple, ghost: int) -> tuple:
    """Process grid in ARRAY axis order (3-D: (pz, py, px); 2-D: (py, px)).

    spec: None / "slab" -> (world, 1, 1) (the reference's layout);
          "auto"        -> the factorisation of `world` with the smallest halo surface
                            (ties: more ranks on the slower axes, which keeps the
                            contiguous z faces);
          "PZxPYxPX" / "PYxPX" string or a tuple -> explicit.
    """
    dims = len(shape_array)
    if spec is None or spec == "slab":
        return (world,) + (1,) * (dims - 1)
    if isinstance(spec, str) and spec != "auto":
        spec = tuple(int(v) for v in spec.lower().split("x"))
    if spec == "auto":
        best = None
        for p in _factorisations(world, dims):
            if any(n < q * max(ghost, 1) for n, q in zip(shape_array, p)):
                continue
            local = [n / q for n, q in zip(shape_array, p)]
            # halo cells moved per rank: 2 faces per decomposed axis
            surf = sum(2 * _prod(local) / local[a] for a in range(dims) if p[a] > 1)
            key = (surf, tuple(-q for q in p))
            if best is None or key < best[0]:
                best = (key, p)
        if best is None:
            raise ValueError(f"no process grid of {world} ranks fits {shape_array}")
        return best[1]
    p = tuple(int(v) for v in spec)
    if len(p) != dims or _prod(p) != world:
        raise ValueError(f"process grid {p} does not match {dims}-D and world size {world}")
    return p


def halo_link_bytes(shape_array: tuple, pgrid: tuple, ghost: int, elem: int,
                    corners: bool, direct: bool = True, stripe_parts: int = 1) -> float:
    """Bytes one rank moves over its busiest xGMI link per exchange (upper bound over
    ranks).  Every GPU pair of an 8-GPU node has its own point-to-point link, so messages
    to different neighbours overlap.  corners (the fused step) with direct = True: one
    phase, edges and corners straight from the diagonal neighbours, so the busiest link
    carries the largest face; direct = False (the phased exchange: axis by axis, fastest
    first, each phase carrying the ghosts of the axes before it): the phases run one after
    another, so their per-phase maxima add up.
    stripe_parts (slabs, parallel/ipc.py stripe_rows): each face in that many parts, the
    direct one 2/(k+1) of the bytes and each relayed one 1/(k+1) crossing two links one
    after the other — the critical path carries 2/(k+1) of the face (k = 2: 2/3)."""
    dims = len(shape_array)
    if stripe_parts > 1 and all(p == 1 for p in pgrid[1:]):
        return halo_link_bytes(shape_array, pgrid, ghost, elem, corners, direct) * \
            2.0 / (stripe_parts + 1)
    local = [-(-n // p) for n, p in zip(shape_array, pgrid)]  # largest block
    split = [a for a in range(dims) if pgrid[a] > 1]
    if corners and direct:
        faces = [0.0]
        for a in split:
            face = ghost
            for b in range(dims):
                if b != a:
                    face *= local[b]
            faces.append(face * elem)
        return float(max(faces))
    done = set()
    per_phase = []
    for a in sorted(split, reverse=True):
        face = ghost
        for b in range(dims):
            if b == a:
                continue
            face *= (local[b] + 2 * ghost) if (corners and b in done) else local[b]
        per_phase.append(face * elem)
        done.add(a)
    if not per_phase:
        return 0.0
    return float(sum(per_phase) if corners else max(per_phase))


def candidate_proc_grids(world: int, shape_array: tuple, ghost: int, elem: int = 8,
                         corners: bool = False, keep: int = 3, direct: bool = True) -> list:
    """Process grids worth trying on an xGMI node, best first by `halo_link_bytes`: the
    slab, plus grids that split only the two slowest axes (a split of the contiguous x
    axis makes the strided x faces AND boundary boxes a few cells wide, which waste
    most of a 64-lane x tile: +16 % compute at (2,2,2), profiles/multigpu_readiness.md)
    that move fewer bytes per link than the slab."""
    dims = len(shape_array)
    slab = (world,) + (1,) * (dims - 1)
    out = [slab]
    if dims < 2 or world == 1:
        return out
    scored = []
    for p in _factorisations(world, dims):
        if p == slab or p[-1] > 1:
            continue
        if any(n // q < max(ghost, 1) for n, q in zip(shape_array, p)):
            continue
        scored.append((halo_link_bytes(shape_array, p, ghost, elem, corners, direct), p))
    base = halo_link_bytes(shape_array, slab, ghost, elem, corners, direct)
    for b, p in sorted(scored):
        if b < 0.9 * base and len(out) < keep:
            out.append(p)
    return out


def _factorisations(n: int, dims: int):
    if dims == 1:
        yield (n,)
        return
    for a in range(1, n + 1):
        if n % a == 0:
            for rest in _factorisations(n // a, dims - 1):
                yield (a,) + rest


@dataclass(frozen=True)
class CartesianDecomposition:
    """Block decomposition over a process grid (row-major ranks, axis 0 slowest).

    Every array axis is a 1-D :class:`SlabDecomposition`; axis 0 (the marched z / y axis)
    always carries G ghost layers (as the slab layout does), the other axes carry G
    ghosts only when they are split.  With ``pgrid = (P, 1, 1)`` this is exactly the slab
    layout.  Star stencils (FD Laplacians, dimension-split WENO) need face ghosts only, so
    edges/corners of the ghost shell are never exchanged.
    """
    shape: tuple   # global extents in array order
    pgrid: tuple   # processes per array axis
    rank: int
    ghost: int

    def __post_init__(self):
        if len(self.shape) != len(self.pgrid):
            raise ValueError("shape / process grid rank mismatch")
        if not 0 <= self.rank < self.size:
            raise ValueError(f"bad rank {self.rank}/{self.size}")
        for a in range(self.dims):
            self.axis(a)  # validates extents

    @property
    def dims(self) -> int:
        return len(self.shape)

    @property
    def size(self) -> int:
        return _prod(self.pgrid)

    def coords_of(self, r: int) -> tuple:
        c = []
        for p in reversed(self.pgrid):
            c.append(r % p)
            r //= p
        return tuple(reversed(c))

    def rank_of(self, coords) -> int:
        r = 0
        for c, p in zip(coords, self.pgrid):
            r = r * p + c
        return r

    @property
    def coords(self) -> tuple:
        return self.coords_of(self.rank)

    @property
    def is_slab(self) -> bool:
        return all(p == 1 for p in self.pgrid[1:])

    def ghost_of_axis(self, a: int) -> int:
        return self.ghost if (a == 0 or self.pgrid[a] > 1) else 0

    def axis(self, a: int, rank: int | None = None) -> SlabDecomposition:
        c = self.coords_of(self.rank if rank is None else rank)
        return SlabDecomposition(self.shape[a], self.pgrid[a], c[a], self.ghost_of_axis(a))

    def neighbor(self, a: int, side: int):
        """Rank of the neighbour along axis a on side -1 / +1 (None at the domain edge)."""
        c = list(self.coords)
        c[a] += side
        if not 0 <= c[a] < self.pgrid[a]:
            return None
        return self.rank_of(c)

    @property
    def alloc(self) -> tuple:
        return tuple(self.axis(a).alloc for a in range(self.dims))

    def owned_box(self) -> tuple:
        """Local (lo, hi) per axis of the owned cells."""
        return tuple(self.axis(a).owned for a in range(self.dims))

    def global_box(self, rank: int | None = None) -> tuple:
        """Global (start, count) per axis of the cells owned by `rank`."""
        out = []
        for a in range(self.dims):
            ax = self.axis(a, rank)
            out.append((ax.start, ax.count))
        return tuple(out)

    def compute_box(self, border: int) -> tuple:
        return tuple(self.axis(a).compute_range(border) for a in range(self.dims))

    def split_boxes(self, border: int, width: int):
        """Partition the compute box into (interior, [boundary boxes]).

        Interior = cells >= `width` away from every face that has a neighbour (computable
        while the halo is in flight).  The boundary shell is cut into at most 2*dims
        disjoint boxes: axis-0 slabs over the full extent of the other axes, then axis-1
        bands inside the axis-0 interior, and so on.  Empty boxes are dropped."""
        full, inner, sides = [], [], []
        for a in range(self.dims):
            inter, blo, bhi = self.axis(a).split_ranges(border, width)
            full.append(self.axis(a).compute_range(border))
            inner.append(inter)
            sides.append((blo, bhi))
        boundary = []
        for a in range(self.dims):
            for rng in sides[a]:
                box = tuple(inner[b] if b < a else (rng if b == a else full[b])
                            for b in range(self.dims))
                if all(hi > lo for lo, hi in box):
                    boundary.append(box)
        interior = tuple(inner)
        return interior, boundary


def fused_view(cd: CartesianDecomposition, radius: int, border: int, a: int, lo: int, hi: int):
    """View window, active and output bounds (view coordinates) along array axis a of a
    fused-step launch on local cells [lo, hi) of a Cartesian block: the window reaches 3R
    beyond the box (ghosts on split axes), the active range is the global interior
    (mirror: csrc/runtime/cart.cpp fused_view)."""
    R3 = 3 * radius
    ax = cd.axis(a)
    v0, v1 = max(0, lo - R3), min(ax.alloc, hi + R3)
    origin = ax.start - ax.ghost + v0  # global index of view cell 0
    N = cd.shape[a]
    return (v0, v1), (max(0, border - origin), min(v1 - v0, N - border - origin)), (lo - v0, hi - v0)
