"""Property-based checks of the halo geometry (hypothesis): for random grids, process grids
and ghost widths, simulate every rank's exchange in one process — each message's send box
copied into the peer's matching receive box, phase by phase — and check that

* every message has exactly one partner message of the same shape (the peer's message
  back, offset negated), so the grouped send/recv of a phase always matches;
* after the exchange every ghost cell the mode promises holds the owner's value: the face
  ghosts for star stencils, the whole ghost shell (edges and corners too) for the fused
  step, in both corner modes (direct: one phase over 3^d - 1 neighbours; phased: axis by
  axis), and nothing outside the domain is written;
* `halo_link_bytes` bounds the largest message any rank sends (direct corners / faces);
* the compute box splits into interior + boundary boxes that tile it exactly.

The reference only splits z (`MultiGPU/Diffusion3d_Baseline/main.c:209-288`): these are the
invariants the Cartesian generalisation (parallel/halo.py, csrc/runtime/cart.cpp) must keep.
"""
import math

import numpy as np
import pytest

hyp = pytest.importorskip("hypothesis")
from hypothesis import given, settings  # noqa: E402
from hypothesis import strategies as st  # noqa: E402

from multigpu_advectiondiffusion_amd.parallel.decomposition import (  # noqa: E402
    CartesianDecomposition, halo_link_bytes)
from multigpu_advectiondiffusion_amd.parallel.halo import CartesianHalo  # noqa: E402


@st.composite
def layouts(draw):
    dims = draw(st.sampled_from([2, 3]))
    pgrid = tuple(draw(st.integers(1, 3)) for _ in range(dims))
    if math.prod(pgrid) == 1:
        pgrid = (2,) + pgrid[1:]
    G = draw(st.integers(1, 6))
    shape = tuple(p * G + draw(st.integers(0, 9)) for p in pgrid)
    mode = draw(st.sampled_from(["faces", "phased", "direct"]))
    return shape, pgrid, G, mode


def _halo(cd, mode):
    return CartesianHalo(None, cd, corners=mode != "faces", direct=mode == "direct")


def _global_index(cd, a, i):
    return cd.axis(a).start - cd.ghost_of_axis(a) + i


def _simulate(shape, pgrid, G, mode):
    world = math.prod(pgrid)
    glob = np.arange(math.prod(shape), dtype=np.float64).reshape(shape)
    cds = [CartesianDecomposition(shape, pgrid, r, G) for r in range(world)]
    halos = [_halo(cd, mode) for cd in cds]
    loc = []
    for cd in cds:
        f = np.full(cd.alloc, -1.0)
        own = cd.owned_box()
        gb = cd.global_box()
        f[tuple(slice(lo, hi) for lo, hi in own)] = glob[tuple(slice(s, s + n) for s, n in gb)]
        loc.append(f)
    for ph in halos[0]._phases():
        msgs = [h.boxes(ph) for h in halos]
        snap = [f.copy() for f in loc]  # a phase's messages travel simultaneously
        for r in range(world):
            for peer, _, rb, off in msgs[r]:
                back = [(sb2, o2) for q2, sb2, _, o2 in msgs[peer] if q2 == r
                        and tuple(-x for x in o2) == tuple(off)]
                assert len(back) == 1, (r, peer, off)
                sb2 = back[0][0]
                src = snap[peer][tuple(slice(lo, hi) for lo, hi in sb2)]
                dst = tuple(slice(lo, hi) for lo, hi in rb)
                assert loc[r][dst].shape == src.shape, (r, peer, off)
                loc[r][dst] = src
    return glob, cds, halos, loc


@settings(max_examples=150, deadline=None, derandomize=True)
@given(layouts())
def test_exchange_fills_promised_ghosts(layout):
    shape, pgrid, G, mode = layout
    glob, cds, _, loc = _simulate(shape, pgrid, G, mode)
    for cd, f in zip(cds, loc):
        own = cd.owned_box()
        grids = np.meshgrid(*[np.arange(n) for n in cd.alloc], indexing="ij")
        gidx = [_global_index(cd, a, grids[a]) for a in range(cd.dims)]
        inside = np.ones(cd.alloc, dtype=bool)
        outside_owned = np.zeros(cd.alloc, dtype=np.int64)
        for a in range(cd.dims):
            inside &= (gidx[a] >= 0) & (gidx[a] < shape[a])
            outside_owned += (grids[a] < own[a][0]) | (grids[a] >= own[a][1])
        promised = inside & ((outside_owned <= 1) if mode == "faces" else True)
        want = glob[tuple(np.clip(gidx[a], 0, shape[a] - 1) for a in range(cd.dims))]
        assert np.array_equal(f[promised], want[promised]), (shape, pgrid, G, mode, cd.rank)
        # nothing outside the domain (and, for faces, no edge / corner ghost) is written
        assert np.all(f[~promised] == -1.0), (shape, pgrid, G, mode, cd.rank)


@settings(max_examples=150, deadline=None, derandomize=True)
@given(layouts())
def test_link_bytes_bound_the_largest_message(layout):
    shape, pgrid, G, mode = layout
    if mode == "phased":
        return  # phased: the bound adds per-phase maxima (checked in test_distributed)
    cds = [CartesianDecomposition(shape, pgrid, r, G) for r in range(math.prod(pgrid))]
    biggest = 0
    for cd in cds:
        h = _halo(cd, mode)
        for ph in h._phases():
            for _, sb, _, _ in h.boxes(ph):
                biggest = max(biggest, math.prod(hi - lo for lo, hi in sb) * 8)
    bound = halo_link_bytes(shape, pgrid, G, 8, corners=mode != "faces", direct=True)
    assert biggest <= bound
    assert biggest == bound  # the first rank's blocks are the largest (remainders go first)


@settings(max_examples=150, deadline=None, derandomize=True)
@given(layouts(), st.integers(0, 4))
def test_interior_and_boundary_tile_the_compute_box(layout, extra_border):
    shape, pgrid, G, _ = layout
    border = min(G, 2) + extra_border
    for r in range(math.prod(pgrid)):
        cd = CartesianDecomposition(shape, pgrid, r, G)
        full = cd.compute_box(border)
        interior, boundary = cd.split_boxes(border, G)
        cover = np.zeros(cd.alloc, dtype=np.int64)
        for box in [interior] + list(boundary):
            if all(hi > lo for lo, hi in box):
                cover[tuple(slice(lo, hi) for lo, hi in box)] += 1
        want = np.zeros(cd.alloc, dtype=np.int64)
        if all(hi > lo for lo, hi in full):
            want[tuple(slice(lo, hi) for lo, hi in full)] = 1
        assert np.array_equal(cover, want), (shape, pgrid, G, border, r)
