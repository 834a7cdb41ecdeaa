"""The temporally blocked full-step kernel (diffusion_fused.hip) must be BIT-IDENTICAL to
three per-stage launches (same fma helpers), for sub-ranges, frozen planes, odd sizes,
fp32/fp64 and FD2/FD4, and match the CPU reference to rounding."""
import pytest
import torch

from multigpu_advectiondiffusion_amd.ops import reference as ref, stencil

pytestmark = pytest.mark.gpu


def _per_stage(u, nx, ny, k0, k1, zlo, zhi, border, order, c, dt):
    R = order // 2
    nz = u.shape[0]
    A, B, out = u.clone(), u.clone(), u.clone()
    lo1, hi1 = max(zlo, k0 - 2 * R, R), min(zhi, k1 + 2 * R, nz - R)
    lo2, hi2 = max(zlo, k0 - R, R), min(zhi, k1 + R, nz - R)
    kw = dict(nx=nx, ny=ny, border=border, order=order, cx=c[0], cy=c[1], cz=c[2], dt=dt)
    stencil.diffusion3d_stage(u, None, A, k0=lo1, k1=hi1, a=0.0, b=1.0, **kw)
    stencil.diffusion3d_stage(A, u, B, k0=lo2, k1=hi2, a=0.75, b=0.25, **kw)
    stencil.diffusion3d_stage(B, u, out, k0=k0, k1=k1, a=1.0 / 3.0, b=2.0 / 3.0, **kw)
    return out


CASES = [
    # (nz, ny, nx, sx, k0, k1, zlo, zhi, border)
    (40, 37, 70, 72, 2, 38, 2, 38, 2),        # whole interior, frozen faces
    (64, 64, 128, 128, 9, 50, 2, 62, 2),      # sub-range inside a larger active box
    (30, 20, 56, 64, 6, 24, 0, 30, 2),        # "middle rank": every plane active
    (33, 45, 61, 64, 3, 30, 3, 30, 3),        # wider frozen border
    (130, 19, 200, 256, 2, 128, 2, 128, 2),   # several z chunks
]


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
@pytest.mark.parametrize("order", [4, 2])
@pytest.mark.parametrize("case", CASES)
def test_fused_step_bitwise_equals_per_stage(dtype, order, case):
    nz, ny, nx, sx, k0, k1, zlo, zhi, border = case
    g = torch.Generator().manual_seed(11)
    u = torch.rand((nz, ny, sx), generator=g, dtype=torch.float64).to(dtype).cuda()
    c = (0.21, 0.17, 0.13)
    dt = 0.9 / (2 * sum(c)) if order == 2 else 0.5 / sum(c)
    exp = _per_stage(u, nx, ny, k0, k1, zlo, zhi, border, order, c, dt)
    got = u.clone()
    stencil.diffusion3d_step(u, got, nx=nx, ny=ny, k0=k0, k1=k1, zlo=zlo, zhi=zhi,
                             border=border, order=order, cx=c[0], cy=c[1], cz=c[2], dt=dt)
    torch.cuda.synchronize()
    assert torch.equal(got, exp), (got - exp).abs().max().item()
    # and the CPU reference to rounding
    cpu = u.cpu().double()
    out = cpu.clone()
    ref.diffusion3d_step(cpu, out, nx, ny, k0, k1, zlo, zhi, border, order, *c, dt)
    tol = 1e-12 if dtype == torch.float64 else 1e-5
    assert (got.cpu().double() - out).abs().max().item() < tol


@pytest.mark.parametrize("order", [4, 2])
@pytest.mark.parametrize("case", CASES + [
    (200, 70, 130, 136, 3, 197, 3, 197, 3),   # many z chunks
    (140, 200, 300, 304, 12, 128, 0, 140, 2),  # a slab rank's interior launch
])
def test_fused_step_banded_schedule_bitwise(order, case):
    """The banded z schedule (one long band, short bands after it: advdiff_set_step_banded,
    the default) is bitwise the uniform z chunks and the per-stage path."""
    from multigpu_advectiondiffusion_amd.ops import _lib
    lib = _lib.require()
    nz, ny, nx, sx, k0, k1, zlo, zhi, border = case
    g = torch.Generator().manual_seed(17)
    u = torch.rand((nz, ny, sx), generator=g, dtype=torch.float64).cuda()
    c = (0.21, 0.17, 0.13)
    dt = 0.9 / (2 * sum(c)) if order == 2 else 0.5 / sum(c)
    exp = _per_stage(u, nx, ny, k0, k1, zlo, zhi, border, order, c, dt)
    got = {}
    for m in (0, 1):
        old = lib.advdiff_set_step_banded(m)
        try:
            o = u.clone()
            stencil.diffusion3d_step(u, o, nx=nx, ny=ny, k0=k0, k1=k1, zlo=zlo, zhi=zhi,
                                     border=border, order=order, cx=c[0], cy=c[1], cz=c[2],
                                     dt=dt)
            torch.cuda.synchronize()
            got[m] = o
        finally:
            lib.advdiff_set_step_banded(old)
    assert torch.equal(got[0], exp) and torch.equal(got[1], exp)


@pytest.mark.parametrize("order", [4, 2])
@pytest.mark.parametrize("case", CASES + [
    (200, 70, 130, 136, 3, 197, 3, 197, 3),   # many z chunks
])
def test_fused_step_two_ranges_bitwise(order, case):
    """Two plane ranges in one launch (a slab rank's two boundary slabs) == two launches,
    bitwise; the placement flag (exclusive) never changes a result."""
    nz, ny, nx, sx, k0, k1, zlo, zhi, border = case
    g = torch.Generator().manual_seed(7)
    u = torch.rand((nz, ny, sx), generator=g, dtype=torch.float64).cuda()
    c = (0.21, 0.17, 0.13)
    dt = 0.5 / sum(c)
    kw = dict(nx=nx, ny=ny, zlo=zlo, zhi=zhi, border=border, order=order, cx=c[0], cy=c[1],
              cz=c[2], dt=dt)
    mid = (k0 + k1) // 2
    one, two, excl = u.clone(), u.clone(), u.clone()
    stencil.diffusion3d_step(u, one, k0=k0, k1=k0 + 3, k0b=mid, k1b=k1, **kw)
    stencil.diffusion3d_step(u, two, k0=k0, k1=k0 + 3, **kw)
    stencil.diffusion3d_step(u, two, k0=mid, k1=k1, **kw)
    stencil.diffusion3d_step(u, excl, k0=k0, k1=k0 + 3, k0b=mid, k1b=k1, exclusive=True, **kw)
    torch.cuda.synchronize()
    assert torch.equal(one, two), (one - two).abs().max().item()
    assert torch.equal(one, excl)


def _per_stage_2d(u, nx, j0, j1, ylo, yhi, border, order, c, dt):
    R = order // 2
    ny = u.shape[0]
    A, B, out = u.clone(), u.clone(), u.clone()
    lo1, hi1 = max(ylo, j0 - 2 * R, R), min(yhi, j1 + 2 * R, ny - R)
    lo2, hi2 = max(ylo, j0 - R, R), min(yhi, j1 + R, ny - R)
    kw = dict(nx=nx, border=border, order=order, cx=c[0], cy=c[1], dt=dt)
    stencil.diffusion2d_stage(u, None, A, j0=lo1, j1=hi1, a=0.0, b=1.0, **kw)
    stencil.diffusion2d_stage(A, u, B, j0=lo2, j1=hi2, a=0.75, b=0.25, **kw)
    stencil.diffusion2d_stage(B, u, out, j0=j0, j1=j1, a=1.0 / 3.0, b=2.0 / 3.0, **kw)
    return out


CASES_2D = [
    # (ny, nx, sx, j0, j1, ylo, yhi, border)
    (60, 130, 192, 2, 58, 2, 58, 2),
    (300, 1001, 1024, 2, 298, 2, 298, 2),     # many tiles, several y chunks
    (90, 57, 64, 20, 70, 0, 90, 2),           # middle-rank rows, all active
    (45, 61, 64, 3, 42, 3, 42, 3),            # wider frozen border
]


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
@pytest.mark.parametrize("order", [4, 2])
@pytest.mark.parametrize("case", CASES_2D)
def test_fused_step_2d_bitwise_equals_per_stage(dtype, order, case):
    ny, nx, sx, j0, j1, ylo, yhi, border = case
    g = torch.Generator().manual_seed(5)
    u = torch.rand((ny, sx), generator=g, dtype=torch.float64).to(dtype).cuda()
    c = (0.23, 0.19)
    dt = 0.9 / (2 * sum(c)) if order == 2 else 0.5 / sum(c)
    exp = _per_stage_2d(u, nx, j0, j1, ylo, yhi, border, order, c, dt)
    got = u.clone()
    stencil.diffusion2d_step(u, got, nx=nx, j0=j0, j1=j1, ylo=ylo, yhi=yhi, border=border,
                             order=order, cx=c[0], cy=c[1], dt=dt)
    torch.cuda.synchronize()
    assert torch.equal(got, exp), (got - exp).abs().max().item()


def test_fused_step_box_bounds_match_reference():
    """Explicit active/output boxes (Cartesian views) vs the CPU reference."""
    nz, ny, nx = 40, 44, 70
    g = torch.Generator().manual_seed(3)
    u = torch.rand((nz, ny, nx), generator=g, dtype=torch.float64).cuda()
    c = (0.21, 0.17, 0.13)
    dt = 0.5 / sum(c)
    for box in ((2, 68, 2, 42, 0, 70, 0, 44),      # slab-like
                (0, 70, 0, 44, 6, 64, 6, 38),      # interior block: everything active
                (0, 63, 4, 44, 6, 60, 9, 38)):     # global edge on the high x side
        got = u.clone()
        stencil.diffusion3d_step(u, got, nx=nx, ny=ny, k0=6, k1=34, zlo=0, zhi=nz, border=2,
                                 order=4, cx=c[0], cy=c[1], cz=c[2], dt=dt, box=box)
        cpu = u.cpu()
        out = cpu.clone()
        ref.diffusion3d_step_box(cpu, out, nx, ny, 6, 34, 0, nz, box, 4, *c, dt)
        torch.cuda.synchronize()
        assert (got.cpu() - out).abs().max().item() < 1e-12, box


@pytest.mark.parametrize("order", [4, 2])
@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_fused_step_odd_subrange_bitwise(order, dtype):
    """The step kernel of each order (FD4: 16 waves x 2 rows, FD2: 12 x 3) is bit-identical
    to the per-stage path on a sub-range with frozen planes, odd sizes and chunk lengths
    that are not a multiple of the march unroll."""
    nz, ny, nx, sx, k0, k1, zlo, zhi, border = (77, 53, 133, 136, 5, 70, 2, 74, 2)
    g = torch.Generator().manual_seed(5)
    u = torch.rand((nz, ny, sx), generator=g, dtype=torch.float64).to(dtype).cuda()
    c = (0.21, 0.17, 0.13)
    dt = 0.9 / (2 * sum(c)) if order == 2 else 0.5 / sum(c)
    exp = _per_stage(u, nx, ny, k0, k1, zlo, zhi, border, order, c, dt)
    for kk in ((k0, k1), (k0, k0 + 1), (k0, k0 + 11), (k0 + 3, k1)):
        got = u.clone()
        stencil.diffusion3d_step(u, got, nx=nx, ny=ny, k0=kk[0], k1=kk[1], zlo=zlo, zhi=zhi,
                                 border=border, order=order, cx=c[0], cy=c[1], cz=c[2], dt=dt)
        torch.cuda.synchronize()
        want = u.clone()
        want[kk[0]:kk[1]] = exp[kk[0]:kk[1]]
        assert torch.equal(got, want), (kk, (got - want).abs().max().item())


@pytest.mark.parametrize("order", [4, 2])
def test_fused_step_production_size_bitwise(order):
    """The bench's launch at production size (512^3, fp64) is bitwise equal to three
    per-stage launches over the whole grid."""
    n, R = 512, order // 2
    g = torch.Generator(device="cuda").manual_seed(5)
    u = torch.rand((n, n, n), generator=g, dtype=torch.float64, device="cuda")
    c = (0.21, 0.17, 0.13)
    dt = 0.9 / (2 * sum(c)) if order == 2 else 0.5 / sum(c)
    kw = dict(nx=n, ny=n, k0=R, k1=n - R, zlo=R, zhi=n - R, border=R, order=order, cx=c[0],
              cy=c[1], cz=c[2], dt=dt)
    exp = _per_stage(u, n, n, R, n - R, R, n - R, R, order, c, dt)
    got = u.clone()
    stencil.diffusion3d_step(u, got, exclusive=True, **kw)
    torch.cuda.synchronize()
    assert torch.equal(got, exp), (got - exp).abs().max().item()


@pytest.mark.parametrize("order", [4, 2])
@pytest.mark.parametrize("boxkind", ["slab", "interior", "edge_hi_x_lo_y", "edge_lo_x_hi_y"])
@pytest.mark.parametrize("shape", [(40, 44, 70, 72), (24, 130, 300, 320), (20, 37, 61, 64)])
def test_fused_step_edge_tiles_bitwise(order, boxkind, shape):
    """Boundary-anchored edge tiles (axis_tile): every cell of the output box written
    exactly once with the reference value (output initialised with a sentinel), for slab
    and Cartesian-view boxes (output >= 3R inside view edges that are not global
    boundaries, as the solver's boxes are).  (Round 6 removed the plain-partition switch
    this test used to compare against: the CPU reference box step is the oracle.)"""
    nz, ny, nx, sx = shape
    box = {"slab": None,
           "interior": (0, nx, 0, ny, 6, nx - 6, 6, ny - 6),
           "edge_hi_x_lo_y": (0, nx - 3, 3, ny, 6, nx, 3, ny - 6),
           "edge_lo_x_hi_y": (3, nx, 0, ny - 3, 3, nx - 6, 6, ny)}[boxkind]
    g = torch.Generator().manual_seed(13)
    u = torch.rand((nz, ny, sx), generator=g, dtype=torch.float64).cuda()
    c = (0.21, 0.17, 0.13)
    dt = 0.9 / (2 * sum(c)) if order == 2 else 0.5 / sum(c)
    kw = dict(nx=nx, ny=ny, k0=3, k1=nz - 3, zlo=2, zhi=nz - 2, border=3, order=order,
              cx=c[0], cy=c[1], cz=c[2], dt=dt, box=box)
    got = torch.full_like(u, float("nan"))
    stencil.diffusion3d_step(u, got, **kw)
    torch.cuda.synchronize()
    cpu = u.cpu()
    ref_out = torch.full_like(cpu, float("nan"))
    rbox = box if box is not None else (3, nx - 3, 3, ny - 3, 0, nx, 0, ny)
    ref.diffusion3d_step_box(cpu, ref_out, nx, ny, 3, nz - 3, 2, nz - 2, rbox, order, *c, dt)
    written = ~got.isnan().cpu()
    assert torch.equal(written, ~ref_out.isnan())
    assert (got.cpu()[written] - ref_out[written]).abs().max().item() < 1e-12


# ---- two steps per launch (v6_march, FD2): == two one-step launches, bit for bit ----
STEP2_CASES = CASES + [
    (24, 33, 50, 64, 1, 23, 1, 23, 1),        # border 1 (the solver's FD2 default), thin
    (150, 90, 300, 320, 1, 149, 1, 149, 1),   # several tiles and z chunks per axis
]


def _two_steps(u, nx, ny, k0, k1, zlo, zhi, border, c, dt, box=None):
    kw = dict(nx=nx, ny=ny, zlo=zlo, zhi=zhi, border=border, order=2, cx=c[0], cy=c[1],
              cz=c[2], dt=dt)
    # u^{n+1} on the whole active box (the two-step launch's intermediate), u^{n+2} on
    # the output box
    box1 = None if box is None else tuple(box[:4]) + (0, nx, 0, ny)
    # the first step on the active planes the outputs depend on (a one-step launch asked
    # for a frozen plane would overwrite it: the solver never does)
    mid, out = u.clone(), u.clone()
    stencil.diffusion3d_step(u, mid, k0=max(k0 - 5, zlo), k1=min(k1 + 5, zhi), box=box1, **kw)
    stencil.diffusion3d_step(mid, out, k0=k0, k1=k1, box=box, **kw)
    return out


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
@pytest.mark.parametrize("case", STEP2_CASES)
def test_two_step_kernel_bitwise_equals_two_steps(dtype, case):
    nz, ny, nx, sx, k0, k1, zlo, zhi, border = case
    g = torch.Generator().manual_seed(5)
    u = torch.rand((nz, ny, sx), generator=g, dtype=torch.float64).to(dtype).cuda()
    c = (0.21, 0.17, 0.13)
    dt = 0.9 / (2 * sum(c))
    exp = _two_steps(u, nx, ny, k0, k1, zlo, zhi, border, c, dt)
    got = u.clone()
    stencil.diffusion3d_step2x(u, got, nx=nx, ny=ny, k0=k0, k1=k1, zlo=zlo, zhi=zhi,
                               border=border, cx=c[0], cy=c[1], cz=c[2], dt=dt)
    torch.cuda.synchronize()
    assert torch.equal(got, exp), (got - exp).abs().max().item()


def test_two_step_kernel_box_and_tiles():
    """An explicit active / output box (a Cartesian block's view), edge tiles."""
    nz, ny, nx, sx = 60, 70, 150, 160
    g = torch.Generator().manual_seed(9)
    u = torch.rand((nz, ny, sx), generator=g, dtype=torch.float64).cuda()
    c = (0.21, 0.17, 0.13)
    dt = 0.9 / (2 * sum(c))
    box = (3, 140, 2, 66, 10, 120, 7, 60)
    exp = _two_steps(u, nx, ny, 6, 54, 1, 59, 1, c, dt, box=box)
    got = u.clone()
    stencil.diffusion3d_step2x(u, got, nx=nx, ny=ny, k0=6, k1=54, zlo=1, zhi=59, border=1,
                               cx=c[0], cy=c[1], cz=c[2], dt=dt, box=box)
    torch.cuda.synchronize()
    assert torch.equal(got, exp), (got - exp).abs().max().item()


def test_solver_two_step_path_bitwise(monkeypatch):
    """A single-rank FD2 heat run pairs its steps into two-step launches (eager and graph
    replay, odd step counts too) with results identical to one step per launch."""
    from multigpu_advectiondiffusion_amd.models.base import Grid
    from multigpu_advectiondiffusion_amd.models.diffusion import Diffusion
    from multigpu_advectiondiffusion_amd.solver import Solver

    def run(flag, iters, graph):
        monkeypatch.setenv("ADVDIFF_STEP2", flag)
        s = Solver(Diffusion(order=2), Grid((67, 45, 38), (1.0, 1.0, 1.0)), device="cuda")
        assert s.step2_capable() == (flag == "1")
        s.run(iters=iters, graph=graph)
        return s.owned.clone(), s.it, s.t

    for iters, graph in ((5, False), (19, True)):
        a, ita, ta = run("1", iters, graph)
        b, itb, tb = run("0", iters, graph)
        assert (ita, ta) == (itb, tb)
        assert torch.equal(a, b), (a - b).abs().max().item()


def test_step2_pick_measured_leaves_u_and_results(monkeypatch):
    """ADVDIFF_STEP2 unset: the solver measures one step vs two per launch for its shape
    at construction (advdiff_diffusion3d_step2_pick, u -> un only).  u must come out of
    the measurement untouched, the pick must be cached per shape, and the run must equal
    the one-step-per-launch run bitwise whichever launch the pick chose."""
    from multigpu_advectiondiffusion_amd.models.base import Grid
    from multigpu_advectiondiffusion_amd.models.diffusion import Diffusion
    from multigpu_advectiondiffusion_amd.ops import stencil
    from multigpu_advectiondiffusion_amd.solver import Solver

    g = Grid((67, 45, 38), (1.0, 1.0, 1.0))
    monkeypatch.delenv("ADVDIFF_STEP2", raising=False)
    s = Solver(Diffusion(order=2), g, device="cuda")
    picked = s.step2_capable()
    assert isinstance(picked, bool)
    u_after_pick = s.u.clone()
    m = s.model
    again = stencil.diffusion3d_step2_pick(s.u, s.un, nx=g.nx, ny=g.ny, k0=s.full[0],
                                           k1=s.full[1], zlo=s.zact[0], zhi=s.zact[1],
                                           border=m.border, cx=m.coef[0], cy=m.coef[1],
                                           cz=m.coef[2], dt=m.stable_dt())
    assert again == picked  # cached
    s.run(iters=9, graph=True)
    monkeypatch.setenv("ADVDIFF_STEP2", "0")
    s0 = Solver(Diffusion(order=2), g, device="cuda")
    assert not s0.step2_capable()
    assert torch.equal(u_after_pick, s0.u)
    s0.run(iters=9, graph=True)
    assert (s.it, s.t) == (s0.it, s0.t)
    assert torch.equal(s.owned, s0.owned), (s.owned - s0.owned).abs().max().item()


@pytest.mark.parametrize("order", [4, 2])
def test_sched_pick_measured_and_bitwise(order):
    """The solver measures banded vs uniform z chunks for its fused launch at construction
    (advdiff_diffusion3d_step_sched_pick, u -> un only; cached per launch); whichever it
    keeps, the run equals the uniform-chunk run bitwise, and u is untouched by the pick."""
    from multigpu_advectiondiffusion_amd.models.base import Grid
    from multigpu_advectiondiffusion_amd.models.diffusion import Diffusion
    from multigpu_advectiondiffusion_amd.ops import _lib
    from multigpu_advectiondiffusion_amd.solver import Solver
    lib = _lib.require()
    g = Grid((131, 97, 140), (1.0, 1.0, 1.0))
    ref = Solver(Diffusion(order=order), g, device="cuda", ic="sine")
    u0 = ref.u.clone()
    old = lib.advdiff_set_step_banded(0)
    try:
        ref.run(iters=7, graph=False)
    finally:
        lib.advdiff_set_step_banded(old)
    s = Solver(Diffusion(order=order), g, device="cuda", ic="sine")
    assert torch.equal(s.u, u0)  # the pick wrote un only
    m = s.model
    again = m.sched_pick(s.u, s.un, s.full[0], s.full[1], s.zact[0], s.zact[1], m.stable_dt())
    assert isinstance(again, bool)
    s.run(iters=7, graph=False)
    assert torch.equal(s.owned, ref.owned)
