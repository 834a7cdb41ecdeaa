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


def weno7(m3, m2, m1, o, p1, p2, p3):
    """Left-biased WENO7-JS value at the right face of `o`, written as the MATLAB prototype
    (`Matlab_Prototipes/InviscidBurgersNd/WENO7resAdv1d.m`): alpha_k = g_k/(eps+beta_k)²,
    w_k = alpha_k/Σalpha — the textbook form the HIP kernel's common-denominator rewrite
    (csrc/kernels/common.hpp::weno7_nd) is checked against."""
    B0 = (m1 * (134241 * m1 - 114894 * o) + m3 * (56694 * m1 - 47214 * m2 + 6649 * m3 - 22778 * o)
          + 25729 * o * o + m2 * (-210282 * m1 + 85641 * m2 + 86214 * o))
    B1 = (o * (41001 * o - 30414 * p1) + m2 * (-19374 * m1 + 3169 * m2 + 19014 * o - 5978 * p1)
          + 6649 * p1 * p1 + m1 * (33441 * m1 - 70602 * o + 23094 * p1))
    B2 = (p1 * (33441 * p1 - 19374 * p2) + m1 * (6649 * m1 - 30414 * o + 23094 * p1 - 5978 * p2)
          + 3169 * p2 * p2 + o * (41001 * o - 70602 * p1 + 19014 * p2))
    B3 = (p2 * (85641 * p2 - 47214 * p3) + o * (25729 * o - 114894 * p1 + 86214 * p2 - 22778 * p3)
          + 6649 * p3 * p3 + p1 * (134241 * p1 - 210282 * p2 + 56694 * p3))
    g = (1 / 35, 12 / 35, 18 / 35, 4 / 35)
    al = [gk / (EPS + Bk) ** 2 for gk, Bk in zip(g, (B0, B1, B2, B3))]
    sm = al[0] + al[1] + al[2] + al[3]
    q0 = -3 * m3 + 13 * m2 - 23 * m1 + 25 * o
    q1 = m2 - 5 * m1 + 13 * o + 3 * p1
    q2 = -m1 + 7 * o + 7 * p1 - p2
    q3 = 3 * o + 13 * p1 - 5 * p2 + p3
    return (al[0] * q0 + al[1] * q1 + al[2] * q2 + al[3] * q3) / (12.0 * sm)


def weno7_face(fp, fm, sl):
    """WENO7 face fluxes along the last axis: f⁺ from i-3..i+3, f⁻ mirrored from i+4..i-2."""
    return (weno7(*(sl(fp, o) for o in range(-3, 4)))
            + weno7(*(sl(fm, o) for o in range(4, -3, -1))))


SCHEMES = {"js": 0, "z": 1, "js7": 2}


def scheme_code(weno) -> int:
    """bool (legacy weno_z flag) | "js" | "z" | "js7" | int code -> kernel scheme code."""
    if isinstance(weno, bool):
        return int(weno)
    if isinstance(weno, str):
        return SCHEMES[weno]
    return int(weno)


def scheme_radius(weno) -> int:
    return 4 if scheme_code(weno) == 2 else 3


def _combine(out_view, u0_view, c, L, dt, a, b, ls=False):
    if ls:  # low-storage RK: u0_view is du (read/written)
        d = dt * L if a == 0.0 else a * u0_view + dt * L
        u0_view.copy_(d)
        out_view.copy_(c + b * d)
        return
    v = b * (c + dt * L)
    if a != 0.0:
        v = a * u0_view + v
    out_view.copy_(v)


# ---------------------------------------------------------------------------------
# heat equation stages
# ---------------------------------------------------------------------------------
def diffusion3d_rhs(inp, nx, ny, k0, k1, border, order, cx, cy, cz):
    """K∇²u on the box k in [k0,k1), j,i in [border, n-border) (cx = K/dx² ...)."""
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
    return lap


def diffusion3d_stage(inp, u0, out, nx, ny, k0, k1, border, order, cx, cy, cz, dt, a, b,
                      ls=False):
    if k1 <= k0 or nx - 2 * border <= 0 or ny - 2 * border <= 0:
        return
    B = border
    lap = diffusion3d_rhs(inp, nx, ny, k0, k1, B, order, cx, cy, cz)
    _combine(out[k0:k1, B:ny - B, B:nx - B],
             u0[k0:k1, B:ny - B, B:nx - B] if (a != 0 or ls) else None,
             inp[k0:k1, B:ny - B, B:nx - B], lap, dt, a, b, ls)


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


def _sub3(t, ys, ye, xs, xe, R):
    return None if t is None else t[:, ys - R:ye + R, xs - R:xe + R]


def diffusion3d_step_box(uin, uout, nx, ny, k0, k1, zlo, zhi, box, order, cx, cy, cz, dt):
    """Semantics of advdiff_diffusion3d_step_box: box = (xa0, xa1, ya0, ya1, xo0, xo1,
    yo0, yo1); cells outside the active box are frozen (A = B = u), u^{n+1} is written on
    active cells inside the output box."""
    xa0, xa1, ya0, ya1, xo0, xo1, yo0, yo1 = box
    R = order // 2
    nz = uin.shape[0]
    A = uin.clone()
    B = uin.clone()
    xs, xe = max(xa0, R), min(xa1, nx - R)
    ys, ye = max(ya0, R), min(ya1, ny - R)
    if xe <= xs or ye <= ys:
        return
    lo1, hi1 = max(zlo, k0 - 2 * R, R), min(zhi, k1 + 2 * R, nz - R)
    lo2, hi2 = max(zlo, k0 - R, R), min(zhi, k1 + R, nz - R)
    kw = dict(nx=xe - xs + 2 * R, ny=ye - ys + 2 * R, border=R, order=order, cx=cx, cy=cy,
              cz=cz, dt=dt)
    diffusion3d_stage(_sub3(uin, ys, ye, xs, xe, R), None, _sub3(A, ys, ye, xs, xe, R),
                      k0=lo1, k1=hi1, a=0.0, b=1.0, **kw)
    diffusion3d_stage(_sub3(A, ys, ye, xs, xe, R), _sub3(uin, ys, ye, xs, xe, R),
                      _sub3(B, ys, ye, xs, xe, R), k0=lo2, k1=hi2, a=0.75, b=0.25, **kw)
    oxs, oxe = max(xo0, xs), min(xo1, xe)
    oys, oye = max(yo0, ys), min(yo1, ye)
    if oxe <= oxs or oye <= oys:
        return
    kw.update(nx=oxe - oxs + 2 * R, ny=oye - oys + 2 * R)
    diffusion3d_stage(_sub3(B, oys, oye, oxs, oxe, R), _sub3(uin, oys, oye, oxs, oxe, R),
                      _sub3(uout, oys, oye, oxs, oxe, R), k0=k0, k1=k1, a=1.0 / 3.0,
                      b=2.0 / 3.0, **kw)


def diffusion2d_step_box(uin, uout, nx, j0, j1, ylo, yhi, box, order, cx, cy, dt):
    """Semantics of advdiff_diffusion2d_step_box: box = (xa0, xa1, xo0, xo1)."""
    xa0, xa1, xo0, xo1 = box
    R = order // 2
    ny = uin.shape[0]
    A = uin.clone()
    B = uin.clone()
    xs, xe = max(xa0, R), min(xa1, nx - R)
    if xe <= xs:
        return
    lo1, hi1 = max(ylo, j0 - 2 * R, R), min(yhi, j1 + 2 * R, ny - R)
    lo2, hi2 = max(ylo, j0 - R, R), min(yhi, j1 + R, ny - R)

    def sub(t, a, b):
        return None if t is None else t[:, a - R:b + R]
    kw = dict(nx=xe - xs + 2 * R, border=R, order=order, cx=cx, cy=cy, dt=dt)
    diffusion2d_stage(sub(uin, xs, xe), None, sub(A, xs, xe), j0=lo1, j1=hi1, a=0.0, b=1.0,
                      **kw)
    diffusion2d_stage(sub(A, xs, xe), sub(uin, xs, xe), sub(B, xs, xe), j0=lo2, j1=hi2,
                      a=0.75, b=0.25, **kw)
    oxs, oxe = max(xo0, xs), min(xo1, xe)
    if oxe <= oxs:
        return
    kw.update(nx=oxe - oxs + 2 * R)
    diffusion2d_stage(sub(B, oxs, oxe), sub(uin, oxs, oxe), sub(uout, oxs, oxe), j0=j0, j1=j1,
                      a=1.0 / 3.0, b=2.0 / 3.0, **kw)


def diffusion2d_step(uin, uout, nx, j0, j1, ylo, yhi, border, order, cx, cy, dt):
    """2-D counterpart of diffusion3d_step (semantics of advdiff_diffusion2d_step)."""
    R = order // 2
    ny = uin.shape[0]
    A = uin.clone()
    B = uin.clone()
    lo1, hi1 = max(ylo, j0 - 2 * R, R), min(yhi, j1 + 2 * R, ny - R)
    lo2, hi2 = max(ylo, j0 - R, R), min(yhi, j1 + R, ny - R)
    diffusion2d_stage(uin, None, A, nx, lo1, hi1, border, order, cx, cy, dt, 0.0, 1.0)
    diffusion2d_stage(A, uin, B, nx, lo2, hi2, border, order, cx, cy, dt, 0.75, 0.25)
    diffusion2d_stage(B, uin, uout, nx, j0, j1, border, order, cx, cy, dt, 1.0 / 3.0, 2.0 / 3.0)


def diffusion2d_rhs(inp, nx, j0, j1, border, order, cx, cy):
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
    return lap


def diffusion2d_stage(inp, u0, out, nx, j0, j1, border, order, cx, cy, dt, a, b, ls=False):
    if j1 <= j0 or nx - 2 * border <= 0:
        return
    B = border
    lap = diffusion2d_rhs(inp, nx, j0, j1, B, order, cx, cy)
    _combine(out[j0:j1, B:nx - B], u0[j0:j1, B:nx - B] if (a != 0 or ls) else None,
             inp[j0:j1, B:nx - B], lap, dt, a, b, ls)


# ---------------------------------------------------------------------------------
# Burgers stages
# ---------------------------------------------------------------------------------
def _faces_last_axis(fp, fm, lo, hi, z):
    """F_{i+½} for i in [lo, hi) along the last axis (z: scheme, see scheme_code)."""
    def sl(t, o):
        return t[..., lo + o:hi + o]
    code = scheme_code(z)
    if code == 2:
        return weno7_face(fp, fm, sl)
    return weno5_face(fp, fm, sl, bool(code))


def burgers_rhs_3d(inp, nx, ny, k0, k1, border, weno_z, rdx, rdy, rdz, vx, vy, vz):
    """L(u) on the box k in [k0,k1), j,i in [border, n-border). Requires border >= R."""
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
                    dt, a, b, ls=False):
    if k1 <= k0 or nx - 2 * border <= 0 or ny - 2 * border <= 0:
        return
    if border < scheme_radius(weno_z):
        raise ValueError("WENO needs a frozen border of at least R cells")
    B = border
    L = burgers_rhs_3d(inp, nx, ny, k0, k1, B, weno_z, rdx, rdy, rdz, vx, vy, vz)
    c = inp[k0:k1, B:ny - B, B:nx - B]
    _combine(out[k0:k1, B:ny - B, B:nx - B],
             u0[k0:k1, B:ny - B, B:nx - B] if (a != 0 or ls) else None, c, L, dt, a, b, ls)


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


def burgers2d_stage(inp, u0, out, nx, j0, j1, border, weno_z, rdx, rdy, vx, vy, dt, a, b,
                    ls=False):
    if j1 <= j0 or nx - 2 * border <= 0:
        return
    if border < scheme_radius(weno_z):
        raise ValueError("WENO needs a frozen border of at least R cells")
    B = border
    L = burgers_rhs_2d(inp, nx, j0, j1, B, weno_z, rdx, rdy, vx, vy)
    c = inp[j0:j1, B:nx - B]
    _combine(out[j0:j1, B:nx - B], u0[j0:j1, B:nx - B] if (a != 0 or ls) else None, c, L, dt,
             a, b, ls)


def norms(x, y=None):
    """(Σ|x-y|, Σ(x-y)², max|x-y|) in float64."""
    d = x.double() if y is None else x.double() - y.double()
    ad = d.abs()
    if ad.numel() == 0:
        return 0.0, 0.0, 0.0
    return float(ad.sum()), float((d * d).sum()), float(ad.max())
