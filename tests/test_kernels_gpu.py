"""Numerics of the hand-written HIP kernels vs the PyTorch fp64 reference of the same op.

Every test runs the native gfx950 kernel (libadvdiff.so; no fallback on device tensors)
and the CPU reference on identical random data, then compares the whole output array
(untouched cells included, so out-of-range writes are caught too)."""
import math

import pytest
import torch

from multigpu_advectiondiffusion_amd.ops import _lib, reference as ref, stencil

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _rand3(nz, ny, sx, dtype=torch.float64, seed=0):
    g = torch.Generator().manual_seed(seed)
    return torch.rand((nz, ny, sx), generator=g, dtype=torch.float64).to(dtype)


def _tol(dtype):
    return 1e-12 if dtype == torch.float64 else 2e-5


EPS32 = 2.0 ** -23  # fp32 machine epsilon (ulp of 1)


def _fp32_bound(scale: float, nops: int) -> float:
    """Error bound of an fp32 kernel against the fp64 reference of the same op on the same
    (fp32-exact) inputs: every rounding step (an fp32 op, or an fp32-rounded coefficient)
    adds at most ε/2 relative to the magnitude it works on, and no intermediate exceeds
    `scale` — the op's sum of absolute terms (the 'condition' of the stencil sum:
    |a u0| + |b inp| + b dt Σ|coefficients| max|inp|).  nops = the rounding steps a cell
    goes through, counted from the kernel (c = nops/2 · 2 for a 2x margin: nops · ε)."""
    return nops * EPS32 * scale


def _diff_scale(inp, u0, a, b, dt, cs, order):
    W = 64.0 / 12.0 if order == 4 else 4.0  # Σ|w| of the second-difference stencil
    m = lambda t: t.double().abs().max().item()  # noqa: E731
    return abs(a) * m(u0) + abs(b) * m(inp) * (1.0 + dt * sum(cs) * W)


def _burgers_scale(inp, u0, a, b, dt, rd, vv):
    """Per axis the face fluxes (|f| <= max u²/2, WENO candidates: Σ|coef|/6 = 20/6) are
    differenced and scaled by rd, the viscous term by vv Σ|w_FD4| max|u|."""
    m = lambda t: t.double().abs().max().item()  # noqa: E731
    fmax = m(inp) ** 2 / 2
    adv = sum(2 * r * fmax * (20.0 / 6.0) for r in rd)
    visc = sum(v * (64.0 / 12.0) * m(inp) for v in vv)
    return abs(a) * m(u0) + abs(b) * (m(inp) + dt * (adv + visc))


def test_library_loaded():
    assert _lib.available(), _lib.load_error()
    assert "gfx950" in _lib.build_info()


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
@pytest.mark.parametrize("order", [4, 2])
@pytest.mark.parametrize("shape", [(37, 45, 70, 72), (20, 9, 130, 192), (70, 64, 64, 64)])
@pytest.mark.parametrize("stage", [0, 1, 2])
def test_diffusion3d_stage(dtype, order, shape, stage):
    nz, ny, nx, sx = shape
    R = order // 2
    border = R + (1 if stage == 1 else 0)
    a, b = [(0.0, 1.0), (0.75, 0.25), (1 / 3, 2 / 3)][stage]
    inp = _rand3(nz, ny, sx, dtype, 1)
    u0 = _rand3(nz, ny, sx, dtype, 2)
    out = _rand3(nz, ny, sx, dtype, 3)
    k0, k1 = R + 1, nz - R - 2
    kw = dict(nx=nx, ny=ny, k0=k0, k1=k1, border=border, order=order, cx=0.7, cy=1.3, cz=0.9,
              dt=0.05, a=a, b=b)
    target = u0 if stage == 2 else out  # third stage runs in place (out aliases u0)
    exp = target.double().clone()
    ref.diffusion3d_stage(inp.double(), u0.double(), exp, nx, ny, k0, k1, border, order, 0.7,
                          1.3, 0.9, 0.05, a, b)
    gin, gu0 = inp.to(DEV), u0.to(DEV)
    gout = gu0 if stage == 2 else out.to(DEV)
    stencil.diffusion3d_stage(gin, gu0, gout, **kw)
    torch.cuda.synchronize()
    err = (gout.cpu().double() - exp).abs().max().item()
    if dtype == torch.float64:
        assert err < _tol(dtype) * 50, err
    else:  # 3 axes x (4 stencil adds + 1 fma) + the RK combination + 4 fp32 coefficients
        scale = _diff_scale(inp, u0, a, b, 0.05, (0.7, 1.3, 0.9), order)
        assert err <= _fp32_bound(scale, 24), (err, scale)


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
@pytest.mark.parametrize("order", [4, 2])
@pytest.mark.parametrize("shape", [(41, 300, 320), (300, 57, 64)])
def test_diffusion2d_stage(dtype, order, shape):
    ny, nx, sx = shape
    R = order // 2
    g = torch.Generator().manual_seed(5)
    inp = torch.rand((ny, sx), generator=g, dtype=torch.float64).to(dtype)
    u0 = torch.rand((ny, sx), generator=g, dtype=torch.float64).to(dtype)
    out = torch.rand((ny, sx), generator=g, dtype=torch.float64).to(dtype)
    j0, j1 = R, ny - R
    exp = out.double().clone()
    ref.diffusion2d_stage(inp.double(), u0.double(), exp, nx, j0, j1, R, order, 0.3, 0.6, 0.1,
                          0.75, 0.25)
    gout = out.to(DEV)
    stencil.diffusion2d_stage(inp.to(DEV), u0.to(DEV), gout, nx=nx, j0=j0, j1=j1, border=R,
                              order=order, cx=0.3, cy=0.6, dt=0.1, a=0.75, b=0.25)
    torch.cuda.synchronize()
    err = (gout.cpu().double() - exp).abs().max().item()
    if dtype == torch.float64:
        assert err < _tol(dtype) * 50, err
    else:  # 2 axes x (4 stencil adds + 1 fma) + the RK combination + 3 fp32 coefficients
        scale = _diff_scale(inp, u0, 0.75, 0.25, 0.1, (0.3, 0.6), order)
        assert err <= _fp32_bound(scale, 18), (err, scale)


def _smooth3(nz, ny, sx, seed, dtype):
    """Smooth-ish field with a shock-like feature (exercises nonlinear weights)."""
    g = torch.Generator().manual_seed(seed)
    z = torch.linspace(0, 1, nz, dtype=torch.float64).view(-1, 1, 1)
    y = torch.linspace(0, 1, ny, dtype=torch.float64).view(1, -1, 1)
    x = torch.linspace(0, 1, sx, dtype=torch.float64).view(1, 1, -1)
    f = torch.sin(6 * x + 3 * y) * torch.cos(4 * z) + 0.5 * torch.tanh(40 * (x - 0.5))
    f = f + 0.05 * torch.rand((nz, ny, sx), generator=g, dtype=torch.float64)
    return f.to(dtype)


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
@pytest.mark.parametrize("weno_z", [False, True])
@pytest.mark.parametrize("visc", [0.0, 0.02])
@pytest.mark.parametrize("shape", [(30, 21, 70, 72), (16, 40, 130, 160)])
@pytest.mark.parametrize("stage", [0, 2])
def test_burgers3d_stage(dtype, weno_z, visc, shape, stage):
    nz, ny, nx, sx = shape
    a, b = [(0.0, 1.0), (0.75, 0.25), (1 / 3, 2 / 3)][stage]
    inp = _smooth3(nz, ny, sx, 1, dtype)
    u0 = _smooth3(nz, ny, sx, 2, dtype)
    out = _smooth3(nz, ny, sx, 3, dtype)
    border = 3
    k0, k1 = 3, nz - 3
    rd = (1 / 0.02, 1 / 0.03, 1 / 0.025)
    vv = tuple(visc * r * r for r in rd)
    kw = dict(nx=nx, ny=ny, k0=k0, k1=k1, border=border, weno_z=weno_z, rdx=rd[0], rdy=rd[1],
              rdz=rd[2], vx=vv[0], vy=vv[1], vz=vv[2], dt=1e-3, a=a, b=b)
    target = u0 if stage == 2 else out
    exp = target.double().clone()
    ref.burgers3d_stage(inp.double(), u0.double(), exp, nx, ny, k0, k1, border, weno_z, *rd,
                        *vv, 1e-3, a, b)
    gin, gu0 = inp.to(DEV), u0.to(DEV)
    gout = gu0 if stage == 2 else out.to(DEV)
    stencil.burgers3d_stage(gin, gu0, gout, **kw)
    torch.cuda.synchronize()
    err = (gout.cpu().double() - exp).abs().max().item()
    if dtype == torch.float64:
        assert err < 1e-11, err
    else:  # a face: split (4) + one side (~37) + combine (~7) rounding steps, x2 faces,
        # x3 axes, the viscous sums and the RK combination: ~64 on the largest term
        scale = _burgers_scale(inp, u0, a, b, 1e-3, rd, vv)
        assert err <= _fp32_bound(scale, 64), (err, scale)


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
@pytest.mark.parametrize("weno_z", [False, True])
@pytest.mark.parametrize("visc", [0.0, 0.01])
def test_burgers2d_stage(dtype, weno_z, visc):
    ny, nx, sx = 45, 300, 320
    f = _smooth3(1, ny, sx, 4, dtype)[0]
    u0 = _smooth3(1, ny, sx, 5, dtype)[0]
    out = _smooth3(1, ny, sx, 6, dtype)[0]
    rd = (1 / 0.01, 1 / 0.02)
    vv = tuple(visc * r * r for r in rd)
    exp = out.double().clone()
    ref.burgers2d_stage(f.double(), u0.double(), exp, nx, 3, ny - 3, 3, weno_z, *rd, *vv, 1e-3,
                        0.75, 0.25)
    gout = out.to(DEV)
    stencil.burgers2d_stage(f.to(DEV), u0.to(DEV), gout, nx=nx, j0=3, j1=ny - 3, border=3,
                            weno_z=weno_z, rdx=rd[0], rdy=rd[1], vx=vv[0], vy=vv[1], dt=1e-3,
                            a=0.75, b=0.25)
    torch.cuda.synchronize()
    err = (gout.cpu().double() - exp).abs().max().item()
    if dtype == torch.float64:
        assert err < 1e-11, err
    else:  # as test_burgers3d_stage, two axes
        scale = _burgers_scale(f, u0, 0.75, 0.25, 1e-3, rd, vv)
        assert err <= _fp32_bound(scale, 64), (err, scale)


@pytest.mark.parametrize("ver", [2, 1])
@pytest.mark.parametrize("mode", ["ssp1", "ssp", "ls"])
@pytest.mark.parametrize("weno_z,visc", [(False, 0.0), (True, 0.01)])
@pytest.mark.parametrize("rows", [(3, 4), (3, 9), (5, 44), (3, 130)])
def test_burgers2d_stage_versions(ver, mode, weno_z, visc, rows):
    """Both 2-D WENO5 kernels (v2: barrier-free wave strips, the default; v1: the generic
    row tile) in every stage epilogue, on row ranges shorter than, equal to and not a
    multiple of v2's 5-row unroll, a width with a partial last strip and an idle wave
    (nx = 203: 197 active columns = 3 strips + 8), against the fp64 reference; cells
    outside the updated box must be untouched."""
    from multigpu_advectiondiffusion_amd.ops import _lib
    lib = _lib.require()
    j0, j1 = rows
    ny, nx, sx = 136, 203, 208
    f = _smooth3(1, ny, sx, 14, torch.float64)[0]
    u0 = _smooth3(1, ny, sx, 15, torch.float64)[0]
    aux = _smooth3(1, ny, sx, 16, torch.float64)[0]
    rd = (1 / 0.01, 1 / 0.02)
    vv = tuple(visc * r * r for r in rd)
    a, b = {"ssp1": (0.0, 1.0), "ssp": (0.75, 0.25), "ls": (-0.4, 0.3)}[mode]
    ls = mode == "ls"
    exp_out, exp_aux = u0.clone(), aux.clone()
    if ls:
        ref.burgers2d_stage(f, exp_aux, exp_out, nx, j0, j1, 3, weno_z, *rd, *vv, 1e-3, a, b,
                            ls=True)
    else:
        ref.burgers2d_stage(f, u0, exp_out, nx, j0, j1, 3, weno_z, *rd, *vv, 1e-3, a, b)
    old = lib.advdiff_set_b2_ver(ver)
    try:
        gout, gaux = u0.to(DEV), aux.to(DEV)
        kw = dict(nx=nx, j0=j0, j1=j1, border=3, weno_z=weno_z, rdx=rd[0], rdy=rd[1],
                  vx=vv[0], vy=vv[1], dt=1e-3, a=a, b=b)
        if ls:
            stencil.burgers2d_stage(f.to(DEV), gaux, gout, ls=True, **kw)
        else:
            stencil.burgers2d_stage(f.to(DEV), gout.clone(), gout, **kw)
        torch.cuda.synchronize()
    finally:
        lib.advdiff_set_b2_ver(old)
    assert (gout.cpu() - exp_out).abs().max().item() < 1e-11
    if ls:
        assert (gaux.cpu() - exp_aux).abs().max().item() < 1e-11


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_norms(dtype):
    x = _rand3(13, 17, 40, dtype, 7) - 0.5
    y = _rand3(13, 17, 40, dtype, 8) - 0.5
    box = ((2, 35), (1, 16), (3, 12))
    r = stencil.NormReducer(DEV)
    got = r(x.to(DEV), y.to(DEV), box)
    sub = (x.double() - y.double())[3:12, 1:16, 2:35]
    exp = (sub.abs().sum().item(), (sub * sub).sum().item(), sub.abs().max().item())
    for gv, ev in zip(got, exp):
        assert math.isclose(gv, ev, rel_tol=1e-10), (got, exp)
    got1 = r(x.to(DEV), None, box)
    assert math.isclose(got1[2], x.double()[3:12, 1:16, 2:35].abs().max().item(), rel_tol=1e-12)


@pytest.mark.parametrize("ic", ["zero", "square", "sine", "heat", "gaussian", "plates"])
def test_init_ic_device_matches_torch(ic):
    from multigpu_advectiondiffusion_amd.utils import ics
    shape = (33, 29, 41)
    sp = (1 / 32, 1 / 28, 1 / 40)
    params = ics.IC_DEFAULT_PARAMS.get(ic, (0.0, 0.0))
    exp = ics.evaluate(ic, shape, sp, -2, 20, 64, torch.float64, "cpu", params)
    got = torch.full((20, 29, 64), 7.0, dtype=torch.float64, device=DEV)
    stencil.init_ic_device(got, ics.ic_code(ic), nx=33, ny=29, nzl=20, kg0=-2, NX=33, NY=29,
                           NZ=41, dx=sp[0], dy=sp[1], dz=sp[2], p0=params[0], p1=params[1])
    torch.cuda.synchronize()
    err = (got.cpu()[..., :33] - exp[..., :33]).abs().max().item()
    assert err < 1e-12, err


def test_copy_box():
    src = _rand3(6, 10, 40, torch.float64, 9).to(DEV)
    dst = torch.zeros((6, 12, 48), dtype=torch.float64, device=DEV)
    stencil.copy_box(dst, src, 33, 9, 5)
    torch.cuda.synchronize()
    assert torch.equal(dst[:5, :9, :33].cpu(), src[:5, :9, :33].cpu())
    assert dst[5].abs().sum().item() == 0.0


def test_debug_print_kernel(capfd):
    u = torch.arange(24, dtype=torch.float64, device=DEV).reshape(2, 3, 4)
    stencil.debug_print(u, ((1, 3), (0, 2), (1, 2)))
    torch.cuda.synchronize()
    out = capfd.readouterr().out
    assert "[k=1]" in out and "13.0000" in out and "18.0000" in out


@pytest.mark.parametrize("ver", [3, 9])
@pytest.mark.parametrize("weno_z", [False, True])
def test_burgers3d_stage_variants(ver, weno_z):
    """Both 3-D WENO5 kernels (v9 default, v3 = the fallback for planes of 2 GiB and more)
    against the fp64 reference, on a shape that leaves partial tiles in x and y and a
    remainder z chunk."""
    from multigpu_advectiondiffusion_amd.ops import _lib
    lib = _lib.require()
    nz, ny, nx, sx = 37, 45, 131, 136
    inp = _smooth3(nz, ny, sx, 4, torch.float64)
    u0 = _smooth3(nz, ny, sx, 5, torch.float64)
    rd = (1 / 0.02, 1 / 0.03, 1 / 0.025)
    vv = tuple(0.01 * r * r for r in rd)
    kw = dict(nx=nx, ny=ny, k0=3, k1=nz - 3, border=3, weno_z=weno_z, rdx=rd[0], rdy=rd[1],
              rdz=rd[2], vx=vv[0], vy=vv[1], vz=vv[2], dt=1e-3, a=0.75, b=0.25)
    exp = u0.clone()
    ref.burgers3d_stage(inp, u0, exp, nx, ny, 3, nz - 3, 3, weno_z, *rd, *vv, 1e-3, 0.75, 0.25)
    old_v = lib.advdiff_set_b3_ver(ver)
    try:
        g0 = u0.to(DEV)
        gout = g0.clone()
        stencil.burgers3d_stage(inp.to(DEV), g0, gout, **kw)
        torch.cuda.synchronize()
    finally:
        lib.advdiff_set_b3_ver(old_v)
    err = (gout.cpu() - exp).abs().max().item()
    assert err < 1e-11, err


@pytest.mark.parametrize("k0,k1", [(3, 4), (3, 5), (7, 18), (3, 58)])
@pytest.mark.parametrize("mode", ["ssp1", "ssp", "ls"])
def test_burgers3d_v9_plane_ranges(k0, k1, mode):
    """The default 3-D WENO5 kernel (v9: 10-plane unroll, clamped unconditional
    prefetches) on plane ranges of 1, 2, 11 and 55 planes — chunks shorter than, equal to
    and not a multiple of the unroll — in every stage epilogue, against the fp64
    reference; cells outside [k0, k1) must be untouched."""
    nz, ny, nx, sx = 61, 21, 70, 72
    inp = _smooth3(nz, ny, sx, 7, torch.float64)
    u0 = _smooth3(nz, ny, sx, 8, torch.float64)
    aux = _smooth3(nz, ny, sx, 9, torch.float64)
    rd = (1 / 0.02, 1 / 0.03, 1 / 0.025)
    vv = tuple(0.01 * r * r for r in rd)
    a, b = {"ssp1": (0.0, 1.0), "ssp": (0.75, 0.25), "ls": (-0.4, 0.3)}[mode]
    ls = mode == "ls"
    exp_out, exp_aux = u0.clone(), aux.clone()
    if ls:
        ref.burgers3d_stage(inp, exp_aux, exp_out, nx, ny, k0, k1, 3, True, *rd, *vv, 1e-3, a, b,
                            ls=True)
    else:
        ref.burgers3d_stage(inp, u0, exp_out, nx, ny, k0, k1, 3, True, *rd, *vv, 1e-3, a, b)
    lib = _lib.require()
    old = lib.advdiff_set_b3_ver(9)
    try:
        gout, gaux = u0.to(DEV), aux.to(DEV)
        kw = dict(nx=nx, ny=ny, k0=k0, k1=k1, border=3, weno_z=True, rdx=rd[0], rdy=rd[1],
                  rdz=rd[2], vx=vv[0], vy=vv[1], vz=vv[2], dt=1e-3, a=a, b=b)
        if ls:
            stencil.burgers3d_stage(inp.to(DEV), gaux, gout, ls=True, **kw)
        else:
            stencil.burgers3d_stage(inp.to(DEV), gout.clone(), gout, **kw)
        torch.cuda.synchronize()
    finally:
        lib.advdiff_set_b3_ver(old)
    assert (gout.cpu() - exp_out).abs().max().item() < 1e-11
    if ls:
        assert (gaux.cpu() - exp_aux).abs().max().item() < 1e-11


@pytest.mark.parametrize("ver", [9, 3])
@pytest.mark.parametrize("r1,r2", [((3, 6), (40, 43)), ((3, 20), (21, 58)), ((0, 0), (9, 12)),
                                   ((5, 9), (0, 0))])
def test_burgers3d_two_range_launch(ver, r1, r2):
    """advdiff_burgers3d_stage2_dt (a slab rank's two boundary slabs): one launch with v9,
    two launches with the other kernels — bitwise equal to two single-range launches."""
    nz, ny, nx, sx = 61, 21, 70, 72
    inp = _smooth3(nz, ny, sx, 11, torch.float64).to(DEV)
    u0 = _smooth3(nz, ny, sx, 12, torch.float64).to(DEV)
    rd = (1 / 0.02, 1 / 0.03, 1 / 0.025)
    vv = tuple(0.01 * r * r for r in rd)
    kw = dict(nx=nx, ny=ny, border=3, weno_z=True, rdx=rd[0], rdy=rd[1], rdz=rd[2], vx=vv[0],
              vy=vv[1], vz=vv[2], dt=1e-3, a=0.75, b=0.25)
    lib = _lib.require()
    old = lib.advdiff_set_b3_ver(ver)
    try:
        one = u0.clone()
        stencil.burgers3d_stage(inp, u0, one, k0=r1[0], k1=r1[1], k0b=r2[0], k1b=r2[1], **kw)
        two = u0.clone()
        for lo, hi in (r1, r2):
            if hi > lo:
                stencil.burgers3d_stage(inp, u0, two, k0=lo, k1=hi, **kw)
        torch.cuda.synchronize()
    finally:
        lib.advdiff_set_b3_ver(old)
    assert torch.equal(one, two)
    assert not torch.equal(one, u0)


def test_burgers3d_production_size_vs_reference():
    """The bench's Burgers launch at production size (256³, fp64, WENO5-Z + viscous, the
    default v9 kernel, SSP stage with u^n) against the fp64 PyTorch reference of the same
    stage evaluated on the GPU: exercises the launch math (z chunking, tile counts, 32-bit
    plane offsets) at the size that is timed."""
    n = 256
    g = torch.Generator(device=DEV).manual_seed(3)
    x = torch.linspace(0, 1, n, dtype=torch.float64, device=DEV)
    inp = (torch.sin(5 * x.view(1, 1, -1) + 2 * x.view(1, -1, 1)) * torch.cos(3 * x.view(-1, 1, 1))
           + 0.5 * torch.tanh(30 * (x.view(1, 1, -1) - 0.4)))
    inp = inp + 0.01 * torch.rand((n, n, n), generator=g, dtype=torch.float64, device=DEV)
    u0 = torch.rand((n, n, n), generator=g, dtype=torch.float64, device=DEV)
    rd = n / 2.0
    v = 1e-5 * rd * rd
    kw = dict(nx=n, ny=n, k0=3, k1=n - 3, border=3, weno_z=True, rdx=rd, rdy=rd, rdz=rd,
              vx=v, vy=v, vz=v, dt=1e-4, a=0.75, b=0.25)
    out = u0.clone()
    stencil.burgers3d_stage(inp, u0, out, **kw)
    exp = u0.clone()
    ref.burgers3d_stage(inp, u0, exp, n, n, 3, n - 3, 3, True, rd, rd, rd, v, v, v, 1e-4, 0.75,
                        0.25)
    torch.cuda.synchronize()
    assert (out - exp).abs().max().item() < 1e-11


def test_watchdog_catches_an_isolated_nan_gpu():
    """The device reduction's max uses fmax (drops NaN): the watchdog also checks the sum,
    so one NaN cell among finite ones stops the run on the GPU path too."""
    from multigpu_advectiondiffusion_amd import Diffusion, Grid, Solver
    s = Solver(Diffusion(K=1.0), Grid((70, 33, 41), (1.0, 1.0, 1.0)), dtype=torch.float64,
               device="cuda", ic="sine")
    s.check_finite()
    s.owned[7, 9, 11] = float("nan")
    with pytest.raises(FloatingPointError):
        s.check_finite()


@pytest.mark.parametrize("tx", [32, 64])
@pytest.mark.parametrize("shape", [(37, 45, 131), (40, 38, 70), (23, 70, 33)])
def test_burgers3d_v9_tile_rows_vs_reference(tx, shape):
    """Both v9 tile shapes (64-cell rows x 8, 32-cell rows x 16 — two rows per wave) against
    the fp64 reference on odd sizes (partial x and y tiles), and bitwise equal to each
    other."""
    nz, ny, nx = shape
    sx = (nx + 31) // 32 * 32
    inp = _smooth3(nz, ny, sx, 21, torch.float64)
    u0 = _smooth3(nz, ny, sx, 22, torch.float64)
    rd = (1 / 0.02, 1 / 0.03, 1 / 0.025)
    vv = tuple(0.01 * r * r for r in rd)
    exp = u0.clone()
    ref.burgers3d_stage(inp, u0, exp, nx, ny, 3, nz - 3, 3, True, *rd, *vv, 1e-3, 0.75, 0.25)
    lib = _lib.require()
    kw = dict(nx=nx, ny=ny, k0=3, k1=nz - 3, border=3, weno_z=True, rdx=rd[0], rdy=rd[1],
              rdz=rd[2], vx=vv[0], vy=vv[1], vz=vv[2], dt=1e-3, a=0.75, b=0.25)
    outs = {}
    old_v, old_t = lib.advdiff_set_b3_ver(9), lib.advdiff_set_b3_tx(tx)
    try:
        for t in (tx, 96 - tx):
            lib.advdiff_set_b3_tx(t)
            g0 = u0.to(DEV)
            gout = g0.clone()
            stencil.burgers3d_stage(inp.to(DEV), g0, gout, **kw)
            torch.cuda.synchronize()
            outs[t] = gout.cpu()
    finally:
        lib.advdiff_set_b3_ver(old_v)
        lib.advdiff_set_b3_tx(old_t)
    assert (outs[tx] - exp).abs().max().item() < 1e-11
    assert torch.equal(outs[32], outs[64])


@pytest.mark.parametrize("tx", [64, 32])
@pytest.mark.parametrize("weno_z,visc", [(True, 0.01), (False, 0.0)])
@pytest.mark.parametrize("mode", ["ssp1", "ssp", "ls"])
@pytest.mark.parametrize("ranges", [((3, 58), (0, 0)), ((3, 4), (0, 0)), ((3, 6), (7, 18)),
                                    ((5, 30), (31, 58))])
def test_burgers3d_fp32_packed_pairs(tx, weno_z, visc, mode, ranges):
    """fp32 3-D WENO5 (v9): packed z pairs (two half chunks per lane, v_pk_* arithmetic —
    the default) bitwise equal to one cell per lane, on odd / one-plane / two-range
    launches (a dummy last pair iteration) in every stage epilogue, both tile shapes; and
    against the fp64 reference to fp32 rounding."""
    lib = _lib.require()
    (k0, k1), (k0b, k1b) = ranges
    nz, ny, nx, sx = 61, 37, 131, 136
    inp = _smooth3(nz, ny, sx, 31, torch.float32)
    u0 = _smooth3(nz, ny, sx, 32, torch.float32)
    aux = _smooth3(nz, ny, sx, 33, torch.float32)
    rd = (1 / 0.02, 1 / 0.03, 1 / 0.025)
    vv = tuple(visc * r * r for r in rd)
    a, b = {"ssp1": (0.0, 1.0), "ssp": (0.75, 0.25), "ls": (-0.4, 0.3)}[mode]
    ls = mode == "ls"
    kw = dict(nx=nx, ny=ny, k0=k0, k1=k1, k0b=k0b, k1b=k1b, border=3, weno_z=weno_z,
              rdx=rd[0], rdy=rd[1], rdz=rd[2], vx=vv[0], vy=vv[1], vz=vv[2], dt=1e-3, a=a, b=b)
    outs = {}
    old_v, old_t, old_p = (lib.advdiff_set_b3_ver(9), lib.advdiff_set_b3_tx(tx),
                           lib.advdiff_set_b3_pack(1))
    try:
        for pk in (1, 0):
            lib.advdiff_set_b3_pack(pk)
            gout, gaux = u0.to(DEV), aux.to(DEV)
            if ls:
                stencil.burgers3d_stage(inp.to(DEV), gaux, gout, ls=True, **kw)
            else:
                stencil.burgers3d_stage(inp.to(DEV), gout.clone(), gout, **kw)
            torch.cuda.synchronize()
            outs[pk] = (gout.cpu(), gaux.cpu())
    finally:
        lib.advdiff_set_b3_ver(old_v)
        lib.advdiff_set_b3_tx(old_t)
        lib.advdiff_set_b3_pack(old_p)
    assert torch.equal(outs[1][0], outs[0][0]), (outs[1][0] - outs[0][0]).abs().max().item()
    assert torch.equal(outs[1][1], outs[0][1])
    exp_out, exp_aux = u0.double(), aux.double()
    for lo, hi in ((k0, k1), (k0b, k1b)):
        if hi <= lo:
            continue
        if ls:
            ref.burgers3d_stage(inp.double(), exp_aux, exp_out, nx, ny, lo, hi, 3, weno_z, *rd,
                                *vv, 1e-3, a, b, ls=True)
        else:
            ref.burgers3d_stage(inp.double(), u0.double(), exp_out, nx, ny, lo, hi, 3, weno_z,
                                *rd, *vv, 1e-3, a, b)
    # fp32 arithmetic on inputs that are exact in fp64: error-scaled bound (round 4 had an
    # absolute 5e-4, ~1e4 ulps)
    err = (outs[1][0].double() - exp_out).abs().max().item()
    assert err <= 1e-5 * exp_out.abs().max().item(), err
    if not ls:
        scale = _burgers_scale(inp, u0, a, b, 1e-3, rd, vv)
        assert err <= _fp32_bound(scale, 64), (err, scale)
