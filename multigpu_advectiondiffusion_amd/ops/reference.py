"""PyTorch reference implementations of the stencil stages (CPU or GPU tensors).

These are the numerics oracle for the HIP kernels (tests compare the two in fp64) and the
compute path of the CPU backend (``gloo`` multi-process runs, laptops).  They mirror the
kernels' semantics exactly — same index ranges, same frozen Dirichlet border, same RK
combination ``out = a*u0 + b*(in + dt*L(in))`` — but use whole-array slicing instead of
tiles.

Array convention: axis 0 is the marching/decomposed axis (z in 3-D, y in 2-D); x is the
last (contiguous) axis.  3-D tensors are ``(nz_alloc, ny, sx)``, 2-D ``(ny_alloc, sx)``
with ``sx >= nx`` (padded row pitch).

Reference numerics: SURVEY.md §2.10 (FD4 `MultiGPU/Diffusion3d_Baseline/Kernels.cu:207-261`,
WENO5 `MultiGPU/Burgers3d_Baseline/Kernels.cu:112-220`, WENO5-Z
`SingleGPU/Burgers3d_WENO5/kernels.cu:142-192`, SSP-RK3 `Kernels.cu:290-297`).
"""
from __future__ import annotations

import torch

EPS = 1e-6
C1312 = 13.0 / 12.0


# ---------------------------------------------------------------------------------
# building blocks
# ---------------------------------------------------------------------------------
def d2_fd4(m2, m1, c, p1, p2):
    """Unscaled FD4 second difference (divide by 12 dx² outside)."""
    return 16.0 * (m1 + p1) - (m2 + p2) - 30.0 * c


def d2_fd2(m1, c, p1):
    return (m1 + p1) - 2.0 * c


def lf_split(u):
    """Local Lax-Friedrichs split of the Burgers flux: f± = ½(u²/2 ± |u|u)."""
    q = 0.25 * u * u
    s = (0.5 * u.abs()) * u
    return q + s, q - s


def weno5(v0, v1, v2, v3, v4, z: bool):
    """Left-biased WENO5 value at the right face of v2 (single-division form, as the
    HIP kernel: csrc/kernels/common.hpp)."""
    t0a = v0 - 2.0 * v1 + v2
    t0b = v0 - 4.0 * v1 + 3.0 * v2
    t1a = v1 - 2.0 * v2 + v3
    t1b = v1 - v3
    t2a = v2 - 2.0 * v3 + v4
    t2b = 3.0 * v2 - 4.0 * v3 + v4
    b0 = C1312 * t0a * t0a + 0.25 * t0b * t0b
    b1 = C1312 * t1a * t1a + 0.25 * t1b * t1b
    b2 = C1312 * t2a * t2a + 0.25 * t2b * t2b
    q0 = 2.0 * v0 - 7.0 * v1 + 11.0 * v2
    q1 = -v1 + 5.0 * v2 + 2.0 * v3
    q2 = 2.0 * v2 + 5.0 * v3 - v4
    if z:
        tau = (b0 - b2).abs()
        e0, e1, e2 = b0 + EPS, b1 + EPS, b2 + EPS
        w0 = 0.1 * (e0 + tau) * (e1 * e2)
        w1 = 0.6 * (e1 + tau) * (e0 * e2)
        w2 = 0.3 * (e2 + tau) * (e0 * e1)
    else:
        s0 = (EPS + b0) * (EPS + b0)
        s1 = (EPS + b1) * (EPS + b1)
        s2 = (EPS + b2) * (EPS + b2)
        w0 = 0.1 * (s1 * s2)
        w1 = 0.6 * (s0 * s2)
        w2 = 0.3 * (s0 * s1)
    return (w0 * q0 + w1 * q1 + w2 * q2) / (6.0 * (w0 + w1 + w2))


def weno5_textbook(v0, v1, v2, v3, v4, z: bool):
    """Textbook WENO5 (alpha_k / sum alpha), written as in the reference
    (`MultiGPU/Burgers3d_Baseline/Kernels.cu:176-215`, `SingleGPU/.../kernels.cu:142-192`).
    Used only to verify that the single-division rewrite is the same scheme."""
    b0 = C1312 * (v0 - 2 * v1 + v2) ** 2 + 0.25 * (v0 - 4 * v1 + 3 * v2) ** 2
    b1 = C1312 * (v1 - 2 * v2 + v3) ** 2 + 0.25 * (v1 - v3) ** 2
    b2 = C1312 * (v2 - 2 * v3 + v4) ** 2 + 0.25 * (3 * v2 - 4 * v3 + v4) ** 2
    if z:
        tau = (b0 - b2).abs()
        a0 = 0.1 * (1 + tau / (b0 + EPS))
        a1 = 0.6 * (1 + tau / (b1 + EPS))
        a2 = 0.3 * (1 + tau / (b2 + EPS))
    else:
        a0 = 0.1 / (EPS + b0) ** 2
        a1 = 0.6 / (EPS + b1) ** 2
        a2 = 0.3 / (EPS + b2) ** 2
    s = a0 + a1 + a2
    return (a0 / s * (2 * v0 - 7 * v1 + 11 * v2) + a1 / s * (-v1 + 5 * v2 + 2 * v3)
            + a2 / s * (2 * v2 + 5 * v3 - v4)) / 6.0


def weno5_face(fp, fm, sl, z: bool):
    """Face fluxes F_{i+½} along the LAST axis for i in the index list `sl(off)`.
    `sl(o)` returns the shifted view fp[..., i+o]."""
    return weno5(sl(fp, -2), sl(fp, -1), sl(fp, 0), sl(fp, 1), sl(fp, 2), z) + \
        weno5(sl(fm, 3), sl(fm, 2), sl(fm, 1), sl(fm, 0), sl(fm, -1), z)


def _combine(out_view, u0_view, c, L, dt, a, b):
    v = b * (c + dt * L)
    if a != 0.0:
        v = a * u0_view + v
    out_view.copy_(v)


# ---------------------------------------------------------------------------------
# heat equation stages
# ---------------------------------------------------------------------------------
def diffusion3d_stage(inp, u0, out, nx, ny, k0, k1, border, order, cx, cy, cz, dt, a, b):
    if k1 <= k0 or nx - 2 * border <= 0 or ny - 2 * border <= 0:
        return
    B = border
    s = 1.0 / 12.0 if order == 4 else 1.0
    cx, cy, cz = cx * s, cy * s, cz * s

    def sh(dk, dj, di):
        return inp[k0 + dk:k1 + dk, B + dj:ny - B + dj, B + di:nx - B + di]

    c = sh(0, 0, 0)
    if order == 4:
        lap = (cx * d2_fd4(sh(0, 0, -2), sh(0, 0, -1), c, sh(0, 0, 1), sh(0, 0, 2))
               + cy * d2_fd4(sh(0, -2, 0), sh(0, -1, 0), c, sh(0, 1, 0), sh(0, 2, 0))
               + cz * d2_fd4(sh(-2, 0, 0), sh(-1, 0, 0), c, sh(1, 0, 0), sh(2, 0, 0)))
    elif order == 2:
        lap = (cx * d2_fd2(sh(0, 0, -1), c, sh(0, 0, 1)) + cy * d2_fd2(sh(0, -1, 0), c, sh(0, 1, 0))
               + cz * d2_fd2(sh(-1, 0, 0), c, sh(1, 0, 0)))
    else:
        raise ValueError(f"order {order}")
    _combine(out[k0:k1, B:ny - B, B:nx - B], u0[k0:k1, B:ny - B, B:nx - B] if a != 0 else None,
             c, lap, dt, a, b)


def diffusion3d_step(uin, uout, nx, ny, k0, k1, zlo, zhi, border, order, cx, cy, cz, dt):
    """One full SSP-RK3 step (semantics of advdiff_diffusion3d_step): intermediate stages
    on the active planes [zlo, zhi) that the outputs [k0, k1) depend on, frozen cells
    carry A = B = u."""
    R = order // 2
    nz = uin.shape[0]
    A = uin.clone()
    B = uin.clone()
    lo1, hi1 = max(zlo, k0 - 2 * R, R), min(zhi, k1 + 2 * R, nz - R)
    lo2, hi2 = max(zlo, k0 - R, R), min(zhi, k1 + R, nz - R)
    diffusion3d_stage(uin, None, A, nx, ny, lo1, hi1, border, order, cx, cy, cz, dt, 0.0, 1.0)
    diffusion3d_stage(A, uin, B, nx, ny, lo2, hi2, border, order, cx, cy, cz, dt, 0.75, 0.25)
    diffusion3d_stage(B, uin, uout, nx, ny, k0, k1, border, order, cx, cy, cz, dt, 1.0 / 3.0,
                      2.0 / 3.0)


def diffusion2d_stage(inp, u0, out, nx, j0, j1, border, order, cx, cy, dt, a, b):
    if j1 <= j0 or nx - 2 * border <= 0:
        return
    B = border
    s = 1.0 / 12.0 if order == 4 else 1.0
    cx, cy = cx * s, cy * s

    def sh(dj, di):
        return inp[j0 + dj:j1 + dj, B + di:nx - B + di]

    c = sh(0, 0)
    if order == 4:
        lap = (cx * d2_fd4(sh(0, -2), sh(0, -1), c, sh(0, 1), sh(0, 2))
               + cy * d2_fd4(sh(-2, 0), sh(-1, 0), c, sh(1, 0), sh(2, 0)))
    else:
        lap = cx * d2_fd2(sh(0, -1), c, sh(0, 1)) + cy * d2_fd2(sh(-1, 0), c, sh(1, 0))
    _combine(out[j0:j1, B:nx - B], u0[j0:j1, B:nx - B] if a != 0 else None, c, lap, dt, a, b)


# ---------------------------------------------------------------------------------
# Burgers stages
# ---------------------------------------------------------------------------------
def _faces_last_axis(fp, fm, lo, hi, z):
    """F_{i+½} for i in [lo, hi) along the last axis."""
    def sl(t, o):
        return t[..., lo + o:hi + o]
    return weno5_face(fp, fm, sl, z)


def burgers_rhs_3d(inp, nx, ny, k0, k1, border, weno_z, rdx, rdy, rdz, vx, vy, vz):
    """L(u) on the box k in [k0,k1), j,i in [border, n-border). Requires border >= 3."""
    B = border
    fp, fm = lf_split(inp)
    # x faces i+½ for i in [B-1, nx-B): rows restricted to the box
    box_x_p = fp[k0:k1, B:ny - B, :]
    box_x_m = fm[k0:k1, B:ny - B, :]
    Fx = _faces_last_axis(box_x_p, box_x_m, B - 1, nx - B, weno_z)
    dFx = Fx[..., 1:] - Fx[..., :-1]
    # y faces: move y to the last axis
    py = fp[k0:k1, :, B:nx - B].transpose(1, 2)
    my = fm[k0:k1, :, B:nx - B].transpose(1, 2)
    Fy = _faces_last_axis(py, my, B - 1, ny - B, weno_z)
    dFy = (Fy[..., 1:] - Fy[..., :-1]).transpose(1, 2)
    # z faces
    pz = fp[:, B:ny - B, B:nx - B].permute(1, 2, 0)
    mz = fm[:, B:ny - B, B:nx - B].permute(1, 2, 0)
    Fz = _faces_last_axis(pz, mz, k0 - 1, k1, weno_z)
    dFz = (Fz[..., 1:] - Fz[..., :-1]).permute(2, 0, 1)
    L = -(dFx * rdx + dFy * rdy + dFz * rdz)
    if vx != 0.0 or vy != 0.0 or vz != 0.0:
        s = 1.0 / 12.0

        def sh(dk, dj, di):
            return inp[k0 + dk:k1 + dk, B + dj:ny - B + dj, B + di:nx - B + di]
        c = sh(0, 0, 0)
        L = L + ((vx * s) * d2_fd4(sh(0, 0, -2), sh(0, 0, -1), c, sh(0, 0, 1), sh(0, 0, 2))
                 + (vy * s) * d2_fd4(sh(0, -2, 0), sh(0, -1, 0), c, sh(0, 1, 0), sh(0, 2, 0))
                 + (vz * s) * d2_fd4(sh(-2, 0, 0), sh(-1, 0, 0), c, sh(1, 0, 0), sh(2, 0, 0)))
    return L


def burgers3d_stage(inp, u0, out, nx, ny, k0, k1, border, weno_z, rdx, rdy, rdz, vx, vy, vz,
                    dt, a, b):
    if k1 <= k0 or nx - 2 * border <= 0 or ny - 2 * border <= 0:
        return
    if border < 3:
        raise ValueError("WENO5 needs a frozen border of at least 3 cells")
    B = border
    L = burgers_rhs_3d(inp, nx, ny, k0, k1, B, weno_z, rdx, rdy, rdz, vx, vy, vz)
    c = inp[k0:k1, B:ny - B, B:nx - B]
    _combine(out[k0:k1, B:ny - B, B:nx - B], u0[k0:k1, B:ny - B, B:nx - B] if a != 0 else None,
             c, L, dt, a, b)


def burgers_rhs_2d(inp, nx, j0, j1, border, weno_z, rdx, rdy, vx, vy):
    B = border
    fp, fm = lf_split(inp)
    Fx = _faces_last_axis(fp[j0:j1, :], fm[j0:j1, :], B - 1, nx - B, weno_z)
    dFx = Fx[..., 1:] - Fx[..., :-1]
    py = fp[:, B:nx - B].transpose(0, 1)
    my = fm[:, B:nx - B].transpose(0, 1)
    Fy = _faces_last_axis(py, my, j0 - 1, j1, weno_z)
    dFy = (Fy[..., 1:] - Fy[..., :-1]).transpose(0, 1)
    L = -(dFx * rdx + dFy * rdy)
    if vx != 0.0 or vy != 0.0:
        s = 1.0 / 12.0

        def sh(dj, di):
            return inp[j0 + dj:j1 + dj, B + di:nx - B + di]
        c = sh(0, 0)
        L = L + ((vx * s) * d2_fd4(sh(0, -2), sh(0, -1), c, sh(0, 1), sh(0, 2))
                 + (vy * s) * d2_fd4(sh(-2, 0), sh(-1, 0), c, sh(1, 0), sh(2, 0)))
    return L


def burgers2d_stage(inp, u0, out, nx, j0, j1, border, weno_z, rdx, rdy, vx, vy, dt, a, b):
    if j1 <= j0 or nx - 2 * border <= 0:
        return
    if border < 3:
        raise ValueError("WENO5 needs a frozen border of at least 3 cells")
    B = border
    L = burgers_rhs_2d(inp, nx, j0, j1, B, weno_z, rdx, rdy, vx, vy)
    c = inp[j0:j1, B:nx - B]
    _combine(out[j0:j1, B:nx - B], u0[j0:j1, B:nx - B] if a != 0 else None, c, L, dt, a, b)


def norms(x, y=None):
    """(Σ|x-y|, Σ(x-y)², max|x-y|) in float64."""
    d = x.double() if y is None else x.double() - y.double()
    ad = d.abs()
    if ad.numel() == 0:
        return 0.0, 0.0, 0.0
    return float(ad.sum()), float((d * d).sum()), float(ad.max())
