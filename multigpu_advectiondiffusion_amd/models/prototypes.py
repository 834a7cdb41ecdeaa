"""Serial CPU ports of the reference's MATLAB prototypes (`Matlab_Prototipes/`), the
numerical specification and accuracy oracle of the reference.

These are re-implemented in vectorised numpy with the prototypes' exact semantics —
including their boundary treatments and the time-loop quirk of the heat tests (the
step that overshoots tFinal is taken with the full dt, and only the clock is clamped;
`Matlab_Prototipes/DiffusionNd/diffusion3dTest.m:56-82`) — so their recorded output
(`TestingAccuracy.log`) can be reproduced.  Contents:

* heat equation, FD4 + SSP-RK3, 1-D/2-D/3-D, exact heat-kernel solutions and L1/L2/Linf
  norms (`heat{1,2,3}d.m`, `diffusion{1,2,3}dTest.m`, `Laplace{1,2,3}d.m`);
* axisymmetric r–y heat with the FD4 (1/r)∂u/∂r correction, mirror BC in y, Dirichlet
  in r (`heat2d_axisymmetric.m`, `Laplace2d_axisymmetric.m`, `RadCorr2d.m`);
* the order-of-accuracy harness (`TestingAccuracy.m`);
* 10 one-dimensional ICs (`InviscidBurgersNd/CommonIC.m`);
* WENO5-JS and WENO7 flux-split residuals along any axis with constant-extrapolation
  ghost cells, local (N-d) or global (1-d) Lax-Friedrichs splitting
  (`WENO5resAdv{1d,_X,_Y,_Z}.m`, `WENO7resAdv{1d,_X,_Y,_Z}.m`);
* linear / Burgers / Buckley-Leverett fluxes; SSP-RK3 (WENO5) and the Carpenter–Kennedy
  low-storage RK4(5) (WENO7) drivers `LFWENO{5,7}FDM{1,2,3}d.m` with dt = CFL·dx/max|u|.

The GPU solvers (``models.diffusion`` / ``models.burgers``) implement the reference's
*GPU* semantics (frozen Dirichlet border); these ports are the CPU path of BASELINE.json's
"Diffusion2d 256x256 on CPU" config and the accuracy tests.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np

# ==================================================================================
# heat equation
# ==================================================================================


def laplace_fd4(u: np.ndarray, D: tuple) -> np.ndarray:
    """FD4 Laplacian with Lu = 0 on the two outermost layers of every axis
    (`Laplace1d.m`, `Laplace2d.m`, `Laplace3d.m`: i>2 && i<nx-1 in 1-based indexing).
    D[d] = K/d_d² (the prototypes' Dx, Dy, Dz; the 1/12 is applied here)."""
    Lu = np.zeros_like(u)
    core = tuple(slice(2, n - 2) for n in u.shape)
    acc = np.zeros(tuple(max(n - 4, 0) for n in u.shape))
    for ax, Dd in enumerate(D):
        def sh(o, ax=ax):
            s = list(core)
            n = u.shape[ax]
            s[ax] = slice(2 + o, n - 2 + o)
            return u[tuple(s)]
        acc += Dd / 12.0 * (-sh(2) + 16 * sh(1) - 30 * sh(0) + 16 * sh(-1) - sh(-2))
    Lu[core] = acc
    return Lu


def _heat_grid(n: int, L: float = 10.0):
    dx = L / (n - 1)
    x = np.arange(n) * dx - L / 2
    return x, dx


def heat_test(dims: int, n: int, t_final: float, param: float = 0.9, K: float = 1.0,
              t0: float = 0.1, L: float = 10.0):
    """Port of `diffusion{1,2,3}dTest(n[,n,n], tFinal, param)`: Gaussian heat kernel at t0
    on [-L/2, L/2]^dims, zero Dirichlet faces, FD4 + SSP-RK3 with dt = param/(2KΣ1/d²).
    Returns (L1, L2, Linf, iterations, u)."""
    x, dx = _heat_grid(n, L)
    grids = np.meshgrid(*([x] * dims), indexing="ij")
    r2 = sum(g * g for g in grids)
    u = np.exp(-r2 / (4 * 1.0 * t0))
    uE = (t0 / t_final) ** (dims / 2.0) * np.exp(-r2 / (4 * 1.0 * t_final))
    Dd = tuple(K / dx ** 2 for _ in range(dims))
    dt = 1.0 / (2 * K * dims / dx ** 2) * param
    t, it = t0, 0
    while t < t_final:
        uo = u
        u = uo + dt * laplace_fd4(u, Dd)
        u = 0.75 * uo + 0.25 * (u + dt * laplace_fd4(u, Dd))
        u = (uo + 2 * (u + dt * laplace_fd4(u, Dd))) / 3
        for ax in range(dims):  # set BCs
            idx = [slice(None)] * dims
            idx[ax] = 0
            u[tuple(idx)] = 0
            idx[ax] = n - 1
            u[tuple(idx)] = 0
        if t + dt > t_final:  # the MATLAB quirk: clamps the clock, not the step taken
            dt = t_final - t
        it += 1
        t += dt
    err = np.abs(uE - u).ravel()
    vol = dx ** dims
    return vol * err.sum(), math.sqrt(vol * (err ** 2).sum()), err.max(), it, u


def testing_accuracy(ncells=(10, 20, 40, 80), t_end: float = 1.0, factor: float = 0.9,
                     dims=(1, 2, 3)):
    """Port of `TestingAccuracy.m`: L1/Linf norms and observed orders (log2 ratios).
    Returns {dims: [(n, L1, OOA1, Linf, OOAinf), ...]}.

    The defaults are the parameters that produced the recorded `TestingAccuracy.log`
    (nc = 10,20,40,80 and tEnd = 1.0 reproduce all 24 logged norms and orders; the
    script as committed says nc = [9,17,33,65], tEnd = 0.5)."""
    out = {}
    for d in dims:
        rows = []
        prev = None
        for n in ncells:
            l1, _, linf, _, _ = heat_test(d, n, t_end, factor)
            o1 = oi = 0.0
            if prev is not None:
                o1 = math.log2(prev[0] / l1)
                oi = math.log2(prev[1] / linf)
            rows.append((n, l1, o1, linf, oi))
            prev = (l1, linf)
        out[d] = rows
    return out


def format_accuracy_table(res) -> str:
    """Same layout as the MATLAB printout (`TestingAccuracy.m:60-69`)."""
    lines = []
    for d, rows in res.items():
        lines.append("*" * 63)
        lines.append(f" Heat solver {d} D")
        lines.append("*" * 63)
        lines.append(" nE \t L1-Norm \t Degree \t Linf-Norm \t Degree")
        for nE, l1, o1, li, oi in rows:
            lines.append(f"{nE:3.0f} \t {l1:1.2e} \t {o1:2.2f} \t\t {li:1.2e} \t {oi:2.2f} ")
    return "\n".join(lines)


def heat2d_axisymmetric(nr: int = 128, ny: int = 32, D: float = 0.27, t0: float = 1.0,
                        t_final: float = 2.5, L: float = 10.0, W: float = 10.0,
                        param: float = 0.9):
    """Port of `heat2d_axisymmetric.m`: u_t = D(u_rr + (1/r)u_r + u_yy) on
    [-L/2,L/2]x[-W/2,W/2] with mirror (Neumann) BC in y and zero Dirichlet in r.
    Returns (L1, L2, Linf, u, uE, r)."""
    dr, dy = L / (nr - 1), W / (ny - 1)
    r = np.arange(nr) * dr - L / 2
    y = np.arange(ny) * dy - W / 2
    with np.errstate(divide="ignore"):
        inv_r = 1.0 / r
    inv_r[~np.isfinite(inv_r)] = 0.0
    Dr, Dy = D / (12 * dr ** 2), D / (12 * dy ** 2)
    R, _ = np.meshgrid(r, y)  # [y][r]
    u = np.exp(-(R ** 2) / (4 * D * t0))
    uE = 1.0 / t_final * np.exp(-(R ** 2) / (4 * D * t_final))
    dt = 1.0 / (2 * D * (1 / dr ** 2 + 1 / dy ** 2)) * param

    def lap(u):
        Lu = np.zeros_like(u)
        c = u[2:-2, 2:-2]
        Lu[2:-2, 2:-2] = (Dr * (-u[2:-2, 4:] + 16 * u[2:-2, 3:-1] - 30 * c + 16 * u[2:-2, 1:-3]
                                - u[2:-2, :-4])
                          + Dy * (-u[4:, 2:-2] + 16 * u[3:-1, 2:-2] - 30 * c + 16 * u[1:-3, 2:-2]
                                  - u[:-4, 2:-2])
                          + Dr * dr * inv_r[2:-2] * (u[2:-2, :-4] - 8 * u[2:-2, 1:-3]
                                                     + 8 * u[2:-2, 3:-1] - u[2:-2, 4:]))
        return Lu

    def bcs(u):
        u[0, :] = u[2, :]
        u[-1, :] = u[-3, :]
        u[1, :] = u[2, :]
        u[-2, :] = u[-3, :]
        u[:, 0] = 0
        u[:, -1] = 0
        return u

    t = t0
    while t < t_final:
        uo = u
        u = bcs(uo + dt * lap(u))
        u = bcs(0.75 * uo + 0.25 * (u + dt * lap(u)))
        u = bcs((uo + 2 * (u + dt * lap(u))) / 3)
        if t + dt > t_final:
            dt = t_final - t
        t += dt
    err = np.abs(uE - u).ravel()
    return dr * dy * err.sum(), math.sqrt(dr * dy * (err ** 2).sum()), err.max(), u, uE, r


# ==================================================================================
# hyperbolic prototypes (WENO5 / WENO7)
# ==================================================================================


@dataclass(frozen=True)
class Flux:
    name: str

    def f(self, w):
        if self.name == "linear":
            return 1.0 * w
        if self.name == "burgers":
            return 0.5 * w * w
        if self.name == "buckley":
            return 4 * w ** 2 / (4 * w ** 2 + (1 - w) ** 2)
        raise ValueError(self.name)

    def df(self, w):
        if self.name == "linear":
            return np.ones_like(w)
        if self.name == "burgers":
            return w
        if self.name == "buckley":
            return 8 * w * (1 - w) / (5 * w ** 2 - 2 * w + 1) ** 2
        raise ValueError(self.name)


def _rect(a, b, x):
    """MATLAB rectangularPulse(a, b, x): 1 inside, 1/2 on the edges, 0 outside."""
    return np.where((x > a) & (x < b), 1.0, np.where((x == a) | (x == b), 0.5, 0.0))


def common_ic(x: np.ndarray, case: int) -> np.ndarray:
    """`CommonIC.m` cases 1-10."""
    Lx = x[-1] - x[0]
    xmid = 0.5 * (x[-1] + x[0])
    if case == 1:
        return np.exp(-20 * (x - xmid) ** 2)
    if case == 2:
        return np.exp(-(x - xmid) ** 2 / (4 * 0.01))
    if case == 3:
        return np.sin(np.pi * x)
    if case == 4:
        return 0.5 - np.sin(np.pi * x)
    if case == 5:
        return 0.5 * (1 - np.tanh(x / (4 * 0.02)))
    if case == 6:
        u = np.ones_like(x)
        u[x <= xmid] = 2.0
        return u
    if case == 7:
        a, b = x[0], x[-1]
        xi = 8.0 / (b - a) * (x - a) - 4
        return 0.5 * (np.tanh(-4 * xi) + 1)
    if case == 8:
        return _rect(xmid - 0.1 * Lx, xmid + 0.1 * Lx, x) + 1
    if case == 9:
        xm = -0.25
        return _rect(xm - 0.125 * Lx, xm + 0.125 * Lx, x) + 1
    if case == 10:
        return np.exp(-x) * _rect(xmid - 0.1 * Lx, xmid + 0.1 * Lx, x) * np.exp(0.1)
    raise ValueError("case not in the list")


def _pad_axis(w, axis, left, right):
    """Constant-extrapolation ghost cells (`WENO5resAdv_X.m:53`)."""
    n = w.shape[axis]
    idx = np.concatenate([np.zeros(left, int), np.arange(n), np.full(right, n - 1)])
    return np.take(w, idx, axis=axis)


def _split(W, flux: Flux, global_lf: bool):
    a = np.abs(flux.df(W))
    if global_lf:
        a = a.max()
    return 0.5 * (flux.f(W) + a * W), 0.5 * (flux.f(W) - a * W)


def _w5(v0, v1, v2, v3, v4, d):
    eps = 1e-6
    b0 = 13 / 12 * (v0 - 2 * v1 + v2) ** 2 + 1 / 4 * (v0 - 4 * v1 + 3 * v2) ** 2
    b1 = 13 / 12 * (v1 - 2 * v2 + v3) ** 2 + 1 / 4 * (v1 - v3) ** 2
    b2 = 13 / 12 * (v2 - 2 * v3 + v4) ** 2 + 1 / 4 * (3 * v2 - 4 * v3 + v4) ** 2
    a0, a1, a2 = d[0] / (eps + b0) ** 2, d[1] / (eps + b1) ** 2, d[2] / (eps + b2) ** 2
    s = a0 + a1 + a2
    return a0, a1, a2, s


def weno5_res(w: np.ndarray, flux: Flux, dx: float, axis: int = -1,
              global_lf: bool = False) -> np.ndarray:
    """df/dx along `axis` (`WENO5resAdv1d.m` with global_lf=True, `_X/_Y/_Z` otherwise).
    Faces: h_{i+½} for i in ghost-padded 1..N; the face left of cell 1 is zero as in the
    prototype (hn/hp are initialised to zero there)."""
    axis = axis % w.ndim
    N = w.shape[axis]
    W = _pad_axis(w, axis, 2, 3)
    V, U = _split(W, flux, global_lf)

    def s(T, o):  # T[..., I+o] for I = 2..N+1 (0-based; MATLAB I = 3..N+2)
        return np.take(T, np.arange(2 + o, N + 2 + o), axis=axis)

    vmm, vm, v, vp, vpp = s(V, -2), s(V, -1), s(V, 0), s(V, 1), s(V, 2)
    a0, a1, a2, sm = _w5(vmm, vm, v, vp, vpp, (0.1, 0.6, 0.3))
    hn = (a0 / sm * (2 * vmm - 7 * vm + 11 * v) + a1 / sm * (-vm + 5 * v + 2 * vp)
          + a2 / sm * (2 * v + 5 * vp - vpp)) / 6
    umm, um, uu, up, upp = s(U, -1), s(U, 0), s(U, 1), s(U, 2), s(U, 3)
    # B0p uses (umm, um, u) etc. with weights (0.3, 0.6, 0.1): the mirror of _w5
    b0 = 13 / 12 * (umm - 2 * um + uu) ** 2 + 1 / 4 * (umm - 4 * um + 3 * uu) ** 2
    b1 = 13 / 12 * (um - 2 * uu + up) ** 2 + 1 / 4 * (um - up) ** 2
    b2 = 13 / 12 * (uu - 2 * up + upp) ** 2 + 1 / 4 * (3 * uu - 4 * up + upp) ** 2
    eps = 1e-6
    p0, p1, p2 = 0.3 / (eps + b0) ** 2, 0.6 / (eps + b1) ** 2, 0.1 / (eps + b2) ** 2
    ps = p0 + p1 + p2
    hp = (p0 / ps * (-umm + 5 * um + 2 * uu) + p1 / ps * (2 * um + 5 * uu - up)
          + p2 / ps * (11 * uu - 7 * up + 2 * upp)) / 6
    h = hn + hp
    hl = np.concatenate([np.zeros_like(np.take(h, [0], axis=axis)),
                         np.take(h, np.arange(N - 1), axis=axis)], axis=axis)
    return (h - hl) / dx


def _b7(m3, m2, m1, o, p1, p2, p3):
    """WENO7 smoothness indicators (`WENO7resAdv1d.m`) for the 4 sub-stencils."""
    B0 = (m1 * (134241 * m1 - 114894 * o) + m3 * (56694 * m1 - 47214 * m2 + 6649 * m3 - 22778 * o)
          + 25729 * o ** 2 + m2 * (-210282 * m1 + 85641 * m2 + 86214 * o))
    B1 = (o * (41001 * o - 30414 * p1) + m2 * (-19374 * m1 + 3169 * m2 + 19014 * o - 5978 * p1)
          + 6649 * p1 ** 2 + m1 * (33441 * m1 - 70602 * o + 23094 * p1))
    B2 = (p1 * (33441 * p1 - 19374 * p2) + m1 * (6649 * m1 - 30414 * o + 23094 * p1 - 5978 * p2)
          + 3169 * p2 ** 2 + o * (41001 * o - 70602 * p1 + 19014 * p2))
    B3 = (p2 * (85641 * p2 - 47214 * p3) + o * (25729 * o - 114894 * p1 + 86214 * p2 - 22778 * p3)
          + 6649 * p3 ** 2 + p1 * (134241 * p1 - 210282 * p2 + 56694 * p3))
    return B0, B1, B2, B3


def weno7_res(w: np.ndarray, flux: Flux, dx: float, axis: int = -1,
              global_lf: bool = False) -> np.ndarray:
    """df/dx along `axis` with 7th-order WENO (`WENO7resAdv1d.m`, `_X/_Y/_Z`)."""
    axis = axis % w.ndim
    N = w.shape[axis]
    W = _pad_axis(w, axis, 3, 4)
    V, U = _split(W, flux, global_lf)

    def s(T, o):  # MATLAB I = 4..N+3 -> 0-based 3..N+2
        return np.take(T, np.arange(3 + o, N + 3 + o), axis=axis)

    eps = 1e-6
    v = [s(V, o) for o in (-3, -2, -1, 0, 1, 2, 3)]
    B = _b7(*v)
    g = (1 / 35, 12 / 35, 18 / 35, 4 / 35)
    al = [gk / (eps + Bk) ** 2 for gk, Bk in zip(g, B)]
    sm = sum(al)
    vmmm, vmm, vm, vo, vp, vpp, vppp = v
    hn = (al[0] / sm * (-3 * vmmm + 13 * vmm - 23 * vm + 25 * vo)
          + al[1] / sm * (vmm - 5 * vm + 13 * vo + 3 * vp)
          + al[2] / sm * (-vm + 7 * vo + 7 * vp - vpp)
          + al[3] / sm * (3 * vo + 13 * vp - 5 * vpp + vppp)) / 12
    u = [s(U, o) for o in (-2, -1, 0, 1, 2, 3, 4)]
    B = _b7(*u)
    g = (4 / 35, 18 / 35, 12 / 35, 1 / 35)
    al = [gk / (eps + Bk) ** 2 for gk, Bk in zip(g, B)]
    sm = sum(al)
    ummm, umm, um, uo, up, upp, uppp = u
    hp = (al[0] / sm * (ummm - 5 * umm + 13 * um + 3 * uo)
          + al[1] / sm * (-umm + 7 * um + 7 * uo - up)
          + al[2] / sm * (3 * um + 13 * uo - 5 * up + upp)
          + al[3] / sm * (25 * uo - 23 * up + 13 * upp - 3 * uppp)) / 12
    h = hn + hp
    hl = np.concatenate([np.zeros_like(np.take(h, [0], axis=axis)),
                         np.take(h, np.arange(N - 1), axis=axis)], axis=axis)
    return (h - hl) / dx


# Carpenter–Kennedy low-storage RK4(5) (`LFWENO7FDM1d.m:60-75`)
LSRK45_A = (0.0, -567301805773.0 / 1357537059087.0, -2404267990393.0 / 2016746695238.0,
            -3550918686646.0 / 2091501179385.0, -1275806237668.0 / 842570457699.0)
LSRK45_B = (1432997174477.0 / 9575080441755.0, 5161836677717.0 / 13612068292357.0,
            1720146321549.0 / 2090206949498.0, 3134564353537.0 / 4481467310338.0,
            2277821191437.0 / 14882151754819.0)
LSRK45_C = (0.0, 1432997174477.0 / 9575080441755.0, 2526269341429.0 / 6820363962896.0,
            2006345519317.0 / 3224310063776.0, 2802321613138.0 / 2924317926251.0)


def lf_weno_fdm(u0: np.ndarray, spacing, t_end: float, cfl: float, flux: Flux | str = "burgers",
                order: int = 5, max_steps: int | None = None):
    """`LFWENO{5,7}FDM{1,2,3}d.m`: dt = CFL·dx/max|u| each step; WENO5 + SSP-RK3 or
    WENO7 + LSRK4(5).  1-D uses global LF splitting (WENO5resAdv1d / WENO7resAdv1d);
    N-d uses local LF per axis (_X/_Y/_Z).  Returns (u, t, iterations)."""
    if isinstance(flux, str):
        flux = Flux(flux)
    u = np.array(u0, dtype=np.float64)
    dims = u.ndim
    res = weno5_res if order == 5 else weno7_res
    glob = dims == 1

    def rhs(u):  # = Σ df/dx (the prototypes' dF + dG + dH)
        return sum(res(u, flux, spacing[ax], axis=ax, global_lf=glob) for ax in range(dims))

    t, it = 0.0, 0
    res_u = np.zeros_like(u)
    while t < t_end and (max_steps is None or it < max_steps):
        dt = cfl * spacing[0] / np.abs(u).max()
        if t + dt > t_end:
            dt = t_end - t
        t += dt
        it += 1
        if order == 5:
            uo = u
            u = uo - dt * rhs(u)
            u = 0.75 * uo + 0.25 * (u - dt * rhs(u))
            u = (uo + 2 * (u - dt * rhs(u))) / 3
        else:
            for a, b in zip(LSRK45_A, LSRK45_B):
                res_u = a * res_u + dt * rhs(u)
                u = u - b * res_u
    return u, t, it
