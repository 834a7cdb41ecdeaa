"""Initial conditions, evaluated for a local slab directly on its device.

Every rank builds only the planes it owns (+ ghosts) from global coordinates, so there
is no host-side global array and no scatter (the reference builds the full global array
on EVERY rank and slices it: `MultiGPU/Diffusion3d_Baseline/main.c:76-103`,
`Tools.c:124-199`).

Grid convention: vertex-centred, x_i = i*dx on [0, L] with dx = L/(nx-1)
(`MultiGPU/Diffusion3d_Baseline/main.c:61-63`).

Registry (name -> device-kernel code in ``csrc/kernels/aux.hip``):

=========  ====  ==========================================================================
name       code  formula / reference
=========  ====  ==========================================================================
zero       0     u = 0 (`MultiGPU/Diffusion3d_Baseline/Tools.c:145-156`, IC 2)
square     1     1 inside the middle half of every axis (square jump, `Tools.c:129-143`)
sine       2     sin(πx/Lx)·sin(πy/Ly)·sin(πz/Lz), zero faces; exact decay
                 exp(-Kπ²(1/Lx²+1/Ly²+1/Lz²)t) (`SingleGPU/Diffusion3d_baselineCode/tools.cpp:115-127`)
heat       3     heat kernel exp(-|x-c|²/(4 d t0)) at t0 (d=p0=1, t0=p1=0.1), zero faces
                 (`SingleGPU/Diffusion3d_baselineCode/tools.cpp:128-139`)
gaussian   4     Burgers pulse exp(-|x-c|²/w), w = p0 = 0.1 (`SingleGPU/Burgers3d_WENO5/Burgers.h:41`)
plates     5     two bottom/top planes at 1 (`SingleGPU/Diffusion3d_baselineCode/tools.cpp:100-114`)
disc       6     1 inside a centred disc of radius p0·min(Lx,Ly), p0 = 0.2 (2-D heat,
                 `MultiGPU/Diffusion2d_Baseline/Tools.c:108-122`)
=========  ====  ==========================================================================
"""
from __future__ import annotations

import math

import torch

IC_CODES = {"zero": 0, "square": 1, "sine": 2, "heat": 3, "gaussian": 4, "plates": 5,
            "disc": 6}
IC_DEFAULT_PARAMS = {"heat": (1.0, 0.1), "gaussian": (0.1, 0.0), "disc": (0.2, 0.0)}


def ic_code(name: str) -> int:
    try:
        return IC_CODES[name]
    except KeyError:
        raise ValueError(f"unknown IC {name!r}; choose from {sorted(IC_CODES)}") from None


def evaluate(name: str, shape_global, spacing, axis0_offset: int, n_local: int, sx: int,
             dtype=torch.float64, device="cpu", params=None) -> torch.Tensor:
    """Return the local slab (n_local along axis 0) of the IC as a tensor.

    3-D: shape_global = (NX, NY, NZ), result (n_local, NY, sx), axis 0 = global planes
    axis0_offset .. axis0_offset+n_local-1 (may extend beyond [0,NZ): those are zero).
    2-D: shape_global = (NX, NY), result (n_local, sx), axis 0 = global rows.
    Columns >= NX (row padding) are zero.
    """
    p0, p1 = params if params is not None else IC_DEFAULT_PARAMS.get(name, (0.0, 0.0))
    twod = len(shape_global) == 2
    dev = torch.device(device)
    f64 = torch.float64
    NX, NY = shape_global[0], shape_global[1]
    NZ = 1 if twod else shape_global[2]
    dx, dy = spacing[0], spacing[1]
    dz = 0.0 if twod else spacing[2]
    i = torch.arange(sx, device=dev)
    a0 = torch.arange(axis0_offset, axis0_offset + n_local, device=dev)
    if twod:
        jg = a0.view(-1, 1)
        ii = i.view(1, -1)
        kk = torch.zeros(1, 1, dtype=torch.long, device=dev)
        jj = jg
    else:
        kk = a0.view(-1, 1, 1)
        jj = torch.arange(NY, device=dev).view(1, -1, 1)
        ii = i.view(1, 1, -1)
    x, y, z = ii.to(f64) * dx, jj.to(f64) * dy, kk.to(f64) * dz
    cx, cy, cz = 0.5 * (NX - 1) * dx, 0.5 * (NY - 1) * dy, 0.5 * (NZ - 1) * dz
    face = (ii == 0) | (ii == NX - 1) | (jj == 0) | (jj == NY - 1)
    if not twod:
        face = face | (kk == 0) | (kk == NZ - 1)
    if twod:
        outside = (jj < 0) | (jj >= NY)
    else:
        outside = (kk < 0) | (kk >= NZ)
    outside = outside | (ii >= NX)

    def r2(with_z=True):
        r = (x - cx) ** 2 + (y - cy) ** 2
        if not twod and with_z:
            r = r + (z - cz) ** 2
        return r

    if name == "zero":
        v = torch.zeros_like(x + y + z)
    elif name == "square":
        m = (ii >= NX // 4) & (ii < 3 * NX // 4) & (jj >= NY // 4) & (jj < 3 * NY // 4)
        if not twod:
            m = m & (kk >= NZ // 4) & (kk < 3 * NZ // 4)
        v = m.to(f64)
    elif name == "sine":
        Lx, Ly = (NX - 1) * dx, (NY - 1) * dy
        v = torch.sin(math.pi * x / Lx) * torch.sin(math.pi * y / Ly)
        if not twod:
            Lz = (NZ - 1) * dz
            v = v * torch.sin(math.pi * z / Lz)
        v = torch.where(face, torch.zeros_like(v), v)
    elif name == "heat":
        v = torch.exp(-r2() / (4.0 * p0 * p1))
        v = torch.where(face, torch.zeros_like(v), v)
    elif name == "gaussian":
        v = torch.exp(-r2() / p0)
    elif name == "plates":
        a = jj if twod else kk
        n = NY if twod else NZ
        v = ((a < 2) | (a >= n - 2)).to(f64) + 0.0 * x
    elif name == "disc":
        R = p0 * min((NX - 1) * dx, (NY - 1) * dy)
        v = (r2(with_z=False) < R * R).to(f64)
    else:
        raise ValueError(f"unknown IC {name!r}")
    shape = (n_local, sx) if twod else (n_local, NY, sx)
    v = v.expand(shape)
    v = torch.where(outside.expand(shape), torch.zeros((), dtype=f64, device=dev), v)
    return v.to(dtype).contiguous()


def _window(full: torch.Tensor, offsets, extents, pad_last: int) -> torch.Tensor:
    """Cut the box [offsets, offsets+extents) (array axis order) out of a global-extent
    tensor; cells outside the global array are zero; the last axis is padded to
    `pad_last` columns."""
    shape = tuple(extents[:-1]) + (pad_last,)
    out = torch.zeros(shape, dtype=full.dtype, device=full.device)
    src, dst = [], []
    for a, (o, n) in enumerate(zip(offsets, extents)):
        lo, hi = max(o, 0), min(o + n, full.shape[a])
        if hi <= lo:
            return out
        src.append(slice(lo, hi))
        dst.append(slice(lo - o, hi - o))
    out[tuple(dst)] = full[tuple(src)]
    return out


def evaluate_box(name: str, shape_global, spacing, offsets, extents, sx: int,
                 dtype=torch.float64, device="cpu", params=None) -> torch.Tensor:
    """IC on a local box of a Cartesian decomposition (array axis order: 3-D (z, y, x),
    2-D (y, x)); offsets are global indices of local index 0 (may be negative: ghost
    cells beyond the domain are zero).  Evaluated as a global slab, then cut."""
    NX = shape_global[0]
    full = evaluate(name, shape_global, spacing, offsets[0], extents[0], NX, dtype, device,
                    params)
    offs = (0,) + tuple(offsets[1:])
    return _window(full, offs, extents, sx)


def exact_solution_box(name: str, shape_global, spacing, t: float, K, params, offsets,
                       extents, sx: int, dtype=torch.float64, device="cpu"):
    NX = shape_global[0]
    full = exact_solution(name, shape_global, spacing, t, K, params, offsets[0], extents[0],
                          NX, dtype, device)
    return _window(full, (0,) + tuple(offsets[1:]), extents, sx)


def exact_solution(name: str, shape_global, spacing, t: float, K: float = 1.0,
                   params=None, axis0_offset=0, n_local=None, sx=None, dtype=torch.float64,
                   device="cpu"):
    """Exact heat-equation solution for the ``sine`` and ``heat`` ICs at time t.

    sine: u0 · exp(-Kπ²Σ1/L_d² · t) (`SingleGPU/Diffusion3d_baselineCode/tools.cpp:167`).
    heat: (t0/t)^(dims/2) · exp(-|x-c|²/(4 K t)) where the IC is taken at t0
          (`Matlab_Prototipes/DiffusionNd/heat3d.m:36`); free-space kernel, so only
          accurate while the solution is negligible on the (zero) boundary.
    """
    twod = len(shape_global) == 2
    NX, NY = shape_global[0], shape_global[1]
    NZ = 1 if twod else shape_global[2]
    n_local = (NY if twod else NZ) if n_local is None else n_local
    sx = NX if sx is None else sx
    u0 = evaluate(name, shape_global, spacing, axis0_offset, n_local, sx, torch.float64,
                  device, params)
    if name == "sine":
        Ls = [(n - 1) * d for n, d in zip(shape_global, spacing)]
        lam = K * math.pi ** 2 * sum(1.0 / L ** 2 for L in Ls)
        return (u0 * math.exp(-lam * t)).to(dtype)
    if name == "heat":
        p0, p1 = params if params is not None else IC_DEFAULT_PARAMS["heat"]
        dims = len(shape_global)
        # evaluate the kernel at time t with the same diffusivity
        ut = evaluate("heat", shape_global, spacing, axis0_offset, n_local, sx, torch.float64,
                      device, params=(K, t))
        return ((p1 / t) ** (dims / 2.0) * ut).to(dtype)
    raise ValueError(f"no exact solution for IC {name!r}")
