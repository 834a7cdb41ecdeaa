"""The time-stepping engine: device-resident blocks, SSP-RK3 (or low-storage RK4(5)) with
fused stage kernels — or ONE temporally blocked launch per step for the heat equation —
and halo exchange overlapped with interior compute.

Reference call stack being replaced (`MultiGPU/Diffusion3d_Baseline/main.c:30-385`):
host builds the global array on every rank -> host scatter -> HtD -> per step: memcpy
uo <- u, 3 x {boundary Laplacian on 2 send streams, pack, D2H, host-blocking
stream sync, MPI_Isend; interior Laplacian; MPI_Irecv/Wait; H2D; unpack; RK kernel;
cudaDeviceSynchronize} -> DtH -> host gather.

Here, per exchange (per stage: buffers u -> A -> B -> u, no Lu array, no uo copy; or per
step in the fused path: u <-> u' with 3R ghosts):

    compute stream : [interior(in -> out)] --wait(halo of in)--> [boundary(in -> out)] --event-->
    comm stream    :                                   grouped RCCL send/recv of out's ghosts
                                                       (overlaps the NEXT interior)

Decompositions: z-slabs (default) or 2-D/3-D Cartesian blocks (boxes launched on kernel
views).  The host never blocks inside a step; the only host/device syncs are the
optional adaptive-CFL reduction and the timers around ``run``.  Single-process runs
replay the step loop as hipGraphs.
"""
from __future__ import annotations

import contextlib
import time

import numpy as np
import torch

from .models.base import Grid, Model, RunStats
from .models.prototypes import LSRK45_A, LSRK45_B
from .ops import stencil
from .parallel.comm import Comm
from .parallel.decomposition import CartesianDecomposition, fused_view, parse_proc_grid
from .parallel.halo import CartesianHalo, SlabHalo
from .utils import ics
from .utils import io as aio
from .utils import metrics, trace

# Shu–Osher SSP-RK3: out = a*u^n + b*(in + dt*L(in))
RK3 = ((0.0, 1.0), (0.75, 0.25), (1.0 / 3.0, 2.0 / 3.0))
# Carpenter–Kennedy low-storage RK4(5) (2N storage): du = A*du + dt*L(u); u += B*du
# (`Matlab_Prototipes/InviscidBurgersNd/LFWENO7FDM1d.m`, models/prototypes.py LSRK45_*)
INTEGRATORS = ("ssprk3", "lsrk45")


def _fault_from_env():
    """Fault injection for failure-handling tests: ADVDIFF_FAULT="RANK:STEP" raises on
    that rank right after that step (eager stepping path).  (The "hang:..." forms belong
    to bench.py and parallel/preflight.py.)"""
    import os
    import re
    v = os.environ.get("ADVDIFF_FAULT")
    if not v or not re.fullmatch(r"\d+:\d+", v):
        return None
    r, st = v.split(":")
    return int(r), int(st)


_FAULT = _fault_from_env()


def _row_pitch(nx: int, elem: int, align_bytes: int = 256) -> int:
    per = max(align_bytes // elem, 1)
    return ((nx + per - 1) // per) * per


def _pitch_pads(pitch, dims: int, device, elem: int = 8, cells_per_rank: int = 0) -> tuple:
    """(extra elements per row after the 256-B alignment, extra rows per plane) of a
    device field: `pitch` = (px, py), else ADVDIFF_PITCH="px,py", else the default rule
    (pitch_default).  The extra rows are real rows of the tensor that no kernel reads or
    writes (like the row padding columns), so every plane range stays one dense block
    (zero-copy halo sends) and `clone()` keeps the layout.  2-D fields take px only; CPU
    fields none.  The result depends on global quantities only, so every slab rank gets
    the same plane layout (RCCL sends whole plane ranges between equal layouts)."""
    import os
    if torch.device(device).type != "cuda":
        return 0, 0
    if pitch is None:
        env = os.environ.get("ADVDIFF_PITCH")
        pitch = (tuple(int(v) for v in env.split(",")) if env
                 else pitch_default(dims, elem, cells_per_rank))
    px, py = (int(pitch[0]), int(pitch[1]) if len(pitch) > 1 else 0)
    if px < 0 or py < 0:
        raise ValueError(f"pitch pads must be >= 0, got {pitch}")
    return px, (py if dims == 3 else 0)


# Pitched allocation of 3-D device fields.  Rows of 2^k elements put every row of a tile,
# and every plane of the z march, on the same HBM channels; a few more elements per row and
# one more row per plane spread them.  Solver-level A/B at 512^3 fp64, two processes
# (bench/pitch_solver_ab.py, profiles/r5/ab/pitch_solver_c_*.log): FD4 640.5 -> 617.2 us
# (+3.8 %), FD2 540.4 -> 511.6 us (+5.6 %) with 4 elements + 1 row, bitwise the same
# solution; every pad from 2 to 24 elements lands within 1 % for FD4.  384^3-768^3 FD2
# gains 14-22 % (pitch_sweep_sizes.log).  fp32: 16 elements + 1 row (FD4 +4.8 %, FD2
# +10.6 %, pitch_ab_fp32.log).  Not at or below MALL_FIELD_BYTES per field: at 256^3
# (128 MiB fields) the two heat fields share the 256 MB Infinity Cache and the padding
# that pushes them past it costs FD2 10 %.  Burgers: neutral (+-0.6 %).
PITCH_PAD_ELEMS = {8: 4, 4: 16}
MALL_FIELD_BYTES = 128 << 20


def pitch_default(dims: int, elem: int, cells_per_rank: int) -> tuple:
    if dims != 3 or cells_per_rank * elem <= MALL_FIELD_BYTES:
        return 0, 0
    return PITCH_PAD_ELEMS.get(elem, max(32 // elem, 1)), 1


class Solver:
    def __init__(self, model: Model, grid: Grid, comm: Comm | None = None, *,
                 dtype=torch.float64, device=None, ic: str = "sine", ic_params=None,
                 overlap: bool = True, pad_rows: bool = True, t0: float = 0.0,
                 check_every: int = 0, fused: bool | None = None, decomp=None,
                 integrator: str = "ssprk3", kernel: str = "native",
                 device_dt: bool | None = None, exchange: str = "u",
                 transport: str | None = None, stripe: int | None = None,
                 boundary_stream: bool | None = None, boundary_on_comm: bool | None = None,
                 pitch=None, fused_put: bool | None = None):
        """decomp: process grid — None/"slab" (split the slowest axis only, the
        reference's layout), "auto" (smallest halo surface) or "PZxPYxPX" / a tuple in
        array axis order ((pz, py, px) in 3-D, (py, px) in 2-D).
        integrator: "ssprk3" (3 stages, the C++/CUDA apps) or "lsrk45" (low-storage
        RK4(5), 5 stages, the MATLAB WENO7 prototypes).
        kernel: "native" (the gfx950 HIP kernels) or "torch" (the PyTorch reference ops on
        the same device — the naive A/B baseline; same launch ranges and schedule).
        device_dt: adaptive-CFL models compute dt on the device (no per-step host sync;
        graph-replayable); None = on for the native GPU path, False = the host-driven
        loop (bitwise the same step sequence, tests/test_adaptive_dt.py).
        transport: halo transport of this solver ("ipc", "rccl", "host"; None = the
        Comm's, Comm.transport) — solvers with different transports can coexist on one
        Comm (bench.py tunes the transport this way).
        boundary_on_comm (N > 1 device ranks, overlap): the boundary launch on the COMM
        stream, right after the wait for the halo of its input and right before the puts
        of its output — two streams per rank, the interior launch beside the whole
        exchange (None = ADVDIFF_BCOMM, else on for the ipc and rccl transports and off
        for host).  boundary_stream is its round-4 name (that version used a third stream;
        see _step_fused_bcomm).
        pitch: (px, py) — device fields get rows of align256(nx) + px elements and, in
        3-D, planes of ny + py rows (the extra rows and columns are never read or written;
        the reference's pitched-memory variants, SingleGPU/*_PitchedMem); None =
        ADVDIFF_PITCH="px,py", else pitch_default() (4 fp64 / 16 fp32 elements and one row
        on 3-D fields past 128 MiB per rank).  pad_rows=False: no padding at all.
        stripe: ipc slab exchanges of 3-D fields relay part of every face message through
        up to this many helper ranks over otherwise idle xGMI links (parallel/halo.py
        SlabHalo; None = ADVDIFF_STRIPE, default 0 = direct only).
        exchange: "u" (default: exchange the stage OUTPUT's ghost planes) or "lu" (the
        reference's MultiGPU scheme, `MultiGPU/Diffusion3d_Baseline/main.c:209-288,300`:
        exchange the boundary planes of the RHS L(u) and advance the ghost planes
        redundantly with the RK update).  "lu" is a slab, per-stage, PyTorch-ops mode kept
        for semantic parity; its results equal the "u" mode's bit for bit
        (tests/test_lu_exchange.py).
        fused_put (3-D slab ranks, direct ipc transport): ONE launch per step (fused heat
        step) or per stage (WENO5 fp64, SSP-RK3) over all owned planes that also stores its
        boundary output planes straight into the neighbours' ghost planes over xGMI
        (advdiff_diffusion3d_step_put / advdiff_burgers3d_stage_put), then signal + wait —
        no boundary launch and no put launch (_step_fused_put, _stage_put).  None =
        ADVDIFF_FUSED_PUT=1; ignored where it does not apply (other models / dtypes /
        integrators, Cartesian grids, striped or non-ipc transports, the multi-rank FD2
        two-step launch)."""
        if kernel not in ("native", "torch"):
            raise ValueError("kernel must be 'native' or 'torch'")
        if exchange not in ("u", "lu"):
            raise ValueError("exchange must be 'u' or 'lu'")
        self.kernel = kernel
        self.exchange = exchange
        if integrator not in INTEGRATORS:
            raise ValueError(f"integrator must be one of {INTEGRATORS}")
        self.integrator = integrator
        if comm is None:
            comm = Comm(device=device or ("cuda" if torch.cuda.is_available() else "cpu"))
            if comm.device.type == "cuda" and comm.device.index is None:
                comm.device = torch.device("cuda", torch.cuda.current_device())
        self.comm = comm
        if transport not in (None, "ipc", "rccl", "host"):
            raise ValueError("transport must be ipc, rccl or host")
        self.transport = transport or comm.transport
        self.device = comm.device
        if self.device.type == "cuda" and kernel != "torch":
            from .ops import _lib
            if _lib.available():
                _lib.preload(self.device.index)  # code objects loaded outside any timing
        self.model = model
        self.grid = grid
        self.dtype = dtype
        self.overlap = overlap
        self.check_every = int(check_every)
        model.bind(grid)
        # fused: one temporally blocked launch per step -> ghost width 3R, ONE halo
        # exchange per step; otherwise one fused launch + one exchange per RK stage.
        ashape = tuple(reversed(grid.shape))  # array axis order: (z, y, x) / (y, x)
        self.pgrid = parse_proc_grid(decomp, comm.size, ashape, model.radius)
        self.cart = any(p > 1 for p in self.pgrid[1:])
        if exchange == "lu" and self.cart:
            raise ValueError("exchange='lu' is the reference's slab scheme: use a slab "
                             "decomposition")
        self.fused = model.supports_fused if fused is None else (fused and model.supports_fused)
        if exchange == "lu":
            self.fused = False  # the RHS exchange is a per-stage scheme
        thin = any(n // p < 3 * model.radius for n, p in zip(ashape, self.pgrid) if p > 1)
        if self.fused and (integrator != "ssprk3" or thin):
            self.fused = False  # LSRK, or blocks thinner than the wide (3R) halo
        elem = torch.empty((), dtype=dtype).element_size()
        if fused_put is None:
            import os
            fused_put = os.environ.get("ADVDIFF_FUSED_PUT") == "1"
        self._want_put = bool(fused_put)
        # multi-rank FD2 slabs: two RK3 steps per launch with a 6R-plane halo every second
        # step (the same bytes per step as 3R every step, half the messages and launches);
        # decided before the fields exist, since it sets the ghost width
        self._mr2 = self._choose_multirank_step2(ashape, elem, pitch, pad_rows, exchange)
        G = (6 if self._mr2 else 3) * model.radius if self.fused else model.radius
        self.ghost = G
        self.cd = CartesianDecomposition(ashape, self.pgrid, comm.rank, G)
        self.d = self.cd.axis(0)
        ax = self.cd.alloc[-1]
        px, self.ypad = (_pitch_pads(pitch, grid.dims, self.device, elem,
                                     grid.cells // comm.size) if pad_rows else (0, 0))
        self.sx = _row_pitch(ax, elem) + px if pad_rows else ax
        self.ic_name, self.ic_params = ic, ic_params
        if self._ipc_multi():
            # BEFORE allocating: the peers close their mappings of any field freed since
            # (a new allocation made while a peer still maps freed memory cannot be
            # exported: bench/ipc_realloc_probe.py), and no cached address survives
            comm.ipc().reset()
        self.u = self._initial_field(ic, ic_params)
        self.du = None
        if self.fused:
            self.un = self.u.clone()  # ping-pong partner; frozen cells keep the IC
            self.A = self.B = None
        elif integrator == "lsrk45":
            self.un = self.u.clone()  # stage ping-pong partner
            self.du = torch.zeros_like(self.u)
            self.A = self.B = None
        else:
            self.A = self.u.clone()
            self.B = self.u.clone()
        # exchange="lu": the RHS of a stage (ghost planes = the neighbours' L).  Two buffers
        # alternate: the ipc transport's puts carry no receiver acknowledgement, so a buffer
        # may only be written again by a peer after an exchange that orders this rank's
        # reads of it (as u/A/B rotate in the default mode) — with ONE buffer a peer's
        # next-stage put can land before this rank's ghost update has read the last one
        self.L = torch.zeros_like(self.u) if exchange == "lu" else None
        self._L2 = torch.zeros_like(self.u) if exchange == "lu" else None
        self.t = float(t0)
        self.it = 0
        self.comm_stream = None
        self.bcomm = False
        if self.device.type == "cuda" and comm.size > 1:
            lo, hi = torch.cuda.Stream.priority_range()
            self.comm_stream = torch.cuda.Stream(device=self.device, priority=hi)
            if boundary_on_comm is None:
                boundary_on_comm = boundary_stream
            if boundary_on_comm is None:
                import os
                # default: on for the ipc transport (every exchange step is a kernel on
                # the comm stream; 2 ranks on one GPU: 90-100 % of the put time beside the
                # interior launch instead of 8-33 %, profiles/r5/overlap.md) and for rccl
                # (the grouped send/recv is issued from the comm stream, so RCCL's stream
                # waits for the boundary launch and the next boundary launch waits for
                # RCCL — the same two-stream order; the reference's boundary-on-send-stream
                # concurrency, MultiGPU/Diffusion3d_Baseline/main.c:118-122,209-260);
                # off for the host-staged exchange, which blocks the host inside start
                env = os.environ.get("ADVDIFF_BCOMM")
                boundary_on_comm = ((env == "1") if env
                                    else self.transport in ("ipc", "rccl"))
            # the boundary launch on the (high-priority) comm stream, between the wait for
            # the halo of its input and the puts of its output: _step_fused_bcomm (with the
            # host-staged transport, gloo device tests only, the host blocks on the comm
            # stream inside the exchange: allowed, eager only, for testing the schedule
            # with an exchange handle that carries works like RCCL's)
            self.bcomm = bool(boundary_on_comm and overlap and exchange == "u")
        if self.cart:
            # the fused step stacks three star stencils: it needs edge/corner ghosts too
            self.halo = CartesianHalo(comm, self.cd, self.comm_stream, corners=self.fused,
                                      transport=self.transport)
            self.full = self.cd.compute_box(model.border)
            self.interior, self.boundary = self.cd.split_boxes(model.border, G)
        else:
            if stripe is None:
                import os
                stripe = int(os.environ.get("ADVDIFF_STRIPE", "0") or 0)
            self.halo = SlabHalo(comm, self.d, self.comm_stream, transport=self.transport,
                                 stripe=stripe if grid.dims == 3 else 0)
            self.full = self.d.compute_range(model.border)
            self.interior, blo, bhi = self.d.split_ranges(model.border, G)
            self.boundary = [blo, bhi]
        # fused halo puts: the step launch (fused heat step) or every stage launch (3-D
        # WENO5 fp64 SSP-RK3) stores the send planes into the peers itself
        # (striped exchanges: the fused heat step only — its kernel stores the direct and
        # the relayed row parts, the helpers forward as usual)
        striped = getattr(self.halo, "striped", False)  # SlabHalo only
        puts_fit = self.fused or (integrator == "ssprk3" and model.stage_put_ok(dtype)
                                  and not striped)
        self.fput = bool(self._want_put and puts_fit and not self.cart and grid.dims == 3
                         and comm.size > 1 and self.transport == "ipc"
                         and self.device.type == "cuda" and kernel == "native"
                         and exchange == "u" and not self._mr2)
        self._primed = None  # striped fused puts: the ipc epoch whose relay sets are primed
        self._put_cache = {}
        if self.fput:
            self.bcomm = False
        # planes (local, ghosts included) whose intermediate stages are updated
        off = self.d.start - G
        self.zact = (max(0, model.border - off), min(self.d.alloc, grid.n_decomposed - model.border - off))
        self._pending = {}
        self._reducer = None
        self._dt_dev = None  # device dt of the step being issued (adaptive CFL)
        self._dts = None     # device [t, dt, steps] of the adaptive loop
        if device_dt is None:
            device_dt = self.device.type == "cuda" and kernel == "native"
        self.device_dt = bool(device_dt) and model.needs_umax and exchange == "u"
        # launch-shape measurements (FD2 steps per launch, z schedule): tune_launches(),
        # on the first run() or explicitly — not here, so building the solver (the CLI's
        # barrier-fenced HtD time) does not include them (the native engine also picks
        # after its init timer)
        self._step2_on = False
        self._picked = False

    def _pick2(self) -> bool:
        self.tune_launches()
        return self._step2_on

    def tune_launches(self) -> None:
        """Measure the launch choices that depend on the shape once (before any graph
        capture): one FD2 step per launch or two (_pick_step2), banded or uniform z chunks
        (_pick_sched).  Idempotent; run() calls it first."""
        if self._picked:
            return
        self._picked = True
        self._step2_on = self._pick_step2()
        self._pick_sched()

    def _choose_multirank_step2(self, ashape, elem, pitch, pad_rows, exchange) -> bool:
        """Several slab ranks, 3-D FD2 fused step: one step per launch (3R ghost planes,
        one exchange per step) or two (diffusion_fused.hip v6_march on the interior and on
        each boundary slab, 6R ghost planes, one exchange per two steps — bit-identical).
        ADVDIFF_STEP2=0/1 forces; otherwise, on the GPU, the rank's interior launch is
        timed both ways once per shape on scratch fields (advdiff_diffusion3d_step2_pick,
        two per launch only if >= 3 % faster) and rank 0's answer is every rank's (the
        ghost width must agree).  CPU runs default to one per launch."""
        import os
        m, comm = self.model, self.comm
        if not (self.fused and comm.size > 1 and not self.cart and m.supports_step2
                and self.integrator == "ssprk3" and exchange == "u" and not self._want_put):
            return False
        G2 = 6 * m.radius
        if ashape[0] // comm.size < G2:
            return False  # a neighbour must own the 6R planes it sends
        env = os.environ.get("ADVDIFF_STEP2")
        if env in ("0", "1"):
            return env == "1"
        on = False
        if self.device.type == "cuda" and self.kernel == "native" and comm.rank == 0:
            cd = CartesianDecomposition(ashape, self.pgrid, 0, G2)
            d = cd.axis(0)
            inter, _, _ = d.split_ranges(m.border, G2)
            if inter[1] > inter[0]:
                px, ypad = (_pitch_pads(pitch, self.grid.dims, self.device, elem,
                                        self.grid.cells // comm.size) if pad_rows else (0, 0))
                sx = _row_pitch(cd.alloc[-1], elem) + px if pad_rows else cd.alloc[-1]
                a = torch.zeros((d.alloc, self.grid.ny + ypad, sx), dtype=self.dtype,
                                device=self.device)
                b = torch.zeros_like(a)
                off = d.start - G2
                zlo = max(0, m.border - off)
                zhi = min(d.alloc, self.grid.n_decomposed - m.border - off)
                on = m.step2_preferred(a, b, inter[0], inter[1], zlo, zhi, m.stable_dt())
                del a, b
                torch.cuda.empty_cache()
        return comm.allreduce_max(1.0 if on else 0.0) > 0.5

    def _ipc_multi(self) -> bool:
        return (self.device.type == "cuda" and self.comm.size > 1
                and self.transport == "ipc")

    def _ipc_epoch(self) -> int:
        return self.comm.ipc().epoch if self._ipc_multi() else 0

    def _initial_field(self, ic, params):
        """IC of the local slab incl. ghosts (ghosts = the neighbours' planes at t0).
        On the GPU the native init kernel fills it in place (no host array, no torch
        temporaries); on the CPU the torch formulas of utils/ics.py."""
        g, G = self.grid, self.ghost
        if self.cart:
            return self._initial_box(ic, params)
        if self.device.type == "cuda":
            p = params if params is not None else ics.IC_DEFAULT_PARAMS.get(ic, (0.0, 0.0))
            if g.dims == 3:
                u = torch.zeros((self.d.alloc, g.ny + self.ypad, self.sx), dtype=self.dtype,
                                device=self.device)
                stencil.init_ic_device(u, ics.ic_code(ic), nx=g.nx, ny=g.ny, nzl=self.d.alloc,
                                       kg0=self.d.start - G, NX=g.nx, NY=g.ny, NZ=g.nz,
                                       dx=g.spacing[0], dy=g.spacing[1], dz=g.spacing[2],
                                       p0=p[0], p1=p[1])
            else:
                u = torch.zeros((self.d.alloc, self.sx), dtype=self.dtype, device=self.device)
                stencil.init_ic_device(u, ics.ic_code(ic), nx=g.nx, ny=self.d.alloc, nzl=1,
                                       kg0=self.d.start - G, NX=g.nx, NY=g.ny, NZ=1,
                                       dx=g.spacing[0], dy=g.spacing[1], dz=0.0, p0=p[0], p1=p[1])
            return u
        return ics.evaluate(ic, g.shape, g.spacing, self.d.start - G, self.d.alloc, self.sx,
                            self.dtype, self.device, params)

    def _initial_box(self, ic, params):
        """Cartesian block (ghost shell included) of the IC."""
        g, cd = self.grid, self.cd
        offs = [cd.axis(a).start - cd.ghost_of_axis(a) for a in range(cd.dims)]
        ext = list(cd.alloc)
        if self.device.type == "cuda":
            p = params if params is not None else ics.IC_DEFAULT_PARAMS.get(ic, (0.0, 0.0))
            pad = (0, self.ypad, 0) if g.dims == 3 else (0, 0)
            u = torch.zeros(tuple(e + p for e, p in zip(ext[:-1], pad)) + (self.sx,),
                            dtype=self.dtype, device=self.device)
            if g.dims == 3:
                stencil.init_ic_box_device(u, ics.ic_code(ic), nx=ext[2], ny=ext[1], nzl=ext[0],
                                           ig0=offs[2], jg0=offs[1], kg0=offs[0], NX=g.nx,
                                           NY=g.ny, NZ=g.nz, dx=g.spacing[0], dy=g.spacing[1],
                                           dz=g.spacing[2], p0=p[0], p1=p[1])
            else:
                stencil.init_ic_box_device(u, ics.ic_code(ic), nx=ext[1], ny=ext[0], nzl=1,
                                           ig0=offs[1], jg0=offs[0], kg0=0, NX=g.nx, NY=g.ny,
                                           NZ=1, dx=g.spacing[0], dy=g.spacing[1], dz=0.0,
                                           p0=p[0], p1=p[1])
            return u
        return ics.evaluate_box(ic, g.shape, g.spacing, offs, ext, self.sx, self.dtype,
                                self.device, params)

    # ------------------------------------------------------------------------------
    # geometry helpers
    # ------------------------------------------------------------------------------
    @property
    def owned(self) -> torch.Tensor:
        """View of the owned cells (no ghosts, row padding cropped)."""
        return self.u[tuple(slice(lo, hi) for lo, hi in self.cd.owned_box())]

    def _owned_xyz_box(self):
        """Owned box in the reducer's (x, y, z) order of local indices."""
        return tuple(reversed(self.cd.owned_box()))

    def memory_bytes(self) -> int:
        """Device bytes of the resident fields (see utils/sizing.py)."""
        n = sum(f.numel() for f in self.fields()) + sum(
            t.numel() for t in (self.du, self.L, self._L2) if t is not None)
        return n * self.u.element_size()

    def fields(self):
        if self.fused:
            return (self.u, self.un)
        if self.du is not None:
            return (self.u, self.un)  # du is scratch (never read at stage 1)
        return (self.u, self.A, self.B)

    # ------------------------------------------------------------------------------
    # stepping
    # ------------------------------------------------------------------------------
    def _launch(self, inp, u0, out, rng, dt, a, b, ls=False, rng2=(0, 0)):
        if self.cart:
            self._launch_box(inp, u0, out, rng, dt, a, b, ls)
            return
        (lo, hi), (lo2, hi2) = rng, rng2
        if hi > lo or hi2 > lo2:
            kw = {} if self._dt_dev is None else {"dt_dev": self._dt_dev}
            if hi2 > lo2:
                kw.update(lo2=lo2, hi2=hi2)
            self.model.stage(inp, u0, out, lo, hi, dt, a, b, ls=ls, **kw)
            trace.sync_check(f"{self.model.name} stage [{lo},{hi}) [{lo2},{hi2})", self.device)

    def _launch_box(self, inp, u0, out, box, dt, a, b, ls=False):
        """Stage on a local box (array order).  The kernels update [border, n-border) of
        the x/y extent they are given, so a box is launched on a VIEW widened by R on
        each side with border R (the views never leave the allocation: every box lies
        >= R inside it, see CartesianDecomposition)."""
        if any(hi <= lo for lo, hi in box):
            return
        R = self.model.radius
        if self.grid.dims == 3:
            (z0, z1), (y0, y1), (x0, x1) = box
            sl = (slice(None), slice(y0 - R, y1 + R), slice(x0 - R, x1 + R))
            kw = dict(nx=x1 - x0 + 2 * R, ny=y1 - y0 + 2 * R, border=R)
        else:
            (z0, z1), (x0, x1) = box
            sl = (slice(None), slice(x0 - R, x1 + R))
            kw = dict(nx=x1 - x0 + 2 * R, border=R)
        v = (lambda t: None if t is None else t[sl])
        if self._dt_dev is not None:
            kw["dt_dev"] = self._dt_dev
        self.model.stage(v(inp), v(u0), v(out), z0, z1, dt, a, b, ls=ls, **kw)
        trace.sync_check(f"{self.model.name} stage box {box}", self.device)

    def _launch_boundary(self, inp, u0, out, a, b, dt, ls):
        if not self.cart and getattr(self.model, "two_range_stage", False):
            self._launch(inp, u0, out, self.boundary[0], dt, a, b, ls, self.boundary[1])
        else:
            for rng in self.boundary:
                self._launch(inp, u0, out, rng, dt, a, b, ls)

    def _stage_bcomm(self, inp, u0, out, a, b, dt, ls, pend):
        """Per-stage counterpart of _step_fused_bcomm."""
        cur = torch.cuda.current_stream(self.device)
        cs = self.comm_stream
        cs.wait_stream(cur)  # the previous stage's interior launch has read / written
        with trace.range_("interior"):
            self._launch(inp, u0, out, self.interior, dt, a, b, ls)
        with torch.cuda.stream(cs):
            if pend is not None:
                pend.wait()  # ipc: stream order on cs already (no event); rccl: joins RCCL
            with trace.range_("boundary"):
                self._launch_boundary(inp, u0, out, a, b, dt, ls)
            bdone = torch.cuda.Event()
            bdone.record(cs)
            with trace.range_("halo_start"):
                self._pending[id(out)] = self.halo.start(out, after_event=False)
        cur.wait_event(bdone)

    def _stage_put(self, inp, u0, out, a, b, dt, ls, pend):
        """Per-stage counterpart of _step_fused_put: one launch over every owned plane that
        also stores the boundary planes of `out` into the neighbours' ghost planes, then
        signal + wait.  Ordering (SSP-RK3, out = A, B, u): the peer last read the ghosts of
        its A in its stage 2 of the previous step, of its B in its stage 3, of its u in its
        stage 1 of this step — each before the signal this stage's wait follows — and none
        of the peer's concurrent stage reads its own output's ghosts (stage 3 reads u as
        the aux operand on owned cells only)."""
        if pend is not None:
            pend.wait()
        put = self._put_targets(out)
        lo, hi = self.full
        if hi > lo:
            kw = {} if self._dt_dev is None else {"dt_dev": self._dt_dev}
            with trace.range_("stage+puts"):
                self.model.stage(inp, u0, out, lo, hi, dt, a, b, ls=ls, put=put, **kw)
                trace.sync_check(f"{self.model.name} stage + puts [{lo},{hi})", self.device)
        with trace.range_("halo_signal"):
            self._pending[id(out)] = self.halo.start(out, puts=False)

    def _stage(self, inp, u0, out, a, b, dt, ls=False):
        pend = self._pending.pop(id(inp), None)
        if self.fput:
            self._stage_put(inp, u0, out, a, b, dt, ls, pend)
            return
        if self.bcomm and self.comm.size > 1:
            self._stage_bcomm(inp, u0, out, a, b, dt, ls, pend)
            return
        if self.comm.size == 1:
            self._launch(inp, u0, out, self.full, dt, a, b, ls)
            return
        if self.overlap:
            with trace.range_("interior"):
                self._launch(inp, u0, out, self.interior, dt, a, b, ls)
            with trace.range_("halo_wait"):
                if pend is not None:
                    pend.wait()
            with trace.range_("boundary"):
                if not self.cart and getattr(self.model, "two_range_stage", False):
                    # both boundary slabs in ONE launch
                    self._launch(inp, u0, out, self.boundary[0], dt, a, b, ls, self.boundary[1])
                else:
                    for rng in self.boundary:
                        self._launch(inp, u0, out, rng, dt, a, b, ls)
        else:
            if pend is not None:
                pend.wait()
            self._launch(inp, u0, out, self.full, dt, a, b, ls)
        with trace.range_("halo_start"):
            self._pending[id(out)] = self.halo.start(out)

    def _stage_lu(self, inp, u0, out, a, b, dt, ls=False):
        """One RK stage with the reference's RHS exchange (main.c:209-288, 300): L(inp) on
        the owned planes, L's boundary planes to the neighbours' ghost planes, then the RK
        update of every active plane, the ghost planes included — each rank advances its
        ghost planes with the same formula as their owner, so no u exchange is needed.
        Overlapped like the reference: boundary L first, its exchange beside the interior
        L and the owned-plane update."""
        m, L = self.model, self.L
        self.L, self._L2 = self._L2, self.L
        lo, hi = self.full
        z0, z1 = self.zact
        if self.comm.size == 1:
            m.rhs(inp, L, lo, hi)
        elif self.overlap:
            with trace.range_("boundary"):
                for rng in self.boundary:
                    m.rhs(inp, L, *rng)
            with trace.range_("halo_start"):
                pend = self.halo.start(L)
            with trace.range_("interior"):
                m.rhs(inp, L, *self.interior)
                m.rk_update(inp, u0, out, L, lo, hi, dt, a, b, ls)
            with trace.range_("halo_wait"):
                if pend is not None:
                    pend.wait()
            m.rk_update(inp, u0, out, L, z0, lo, dt, a, b, ls)
            m.rk_update(inp, u0, out, L, hi, z1, dt, a, b, ls)
            return
        else:
            m.rhs(inp, L, lo, hi)
            with trace.range_("halo"):
                self.halo.exchange(L)
        m.rk_update(inp, u0, out, L, z0, z1, dt, a, b, ls)

    def _launch_fused(self, rng, dt, rng2=(0, 0), exclusive=False):
        """exclusive: nothing else (RCCL copy kernels) runs beside this launch — a single
        rank, or a full-range launch after the halo wait — so the 3-D step may run as one
        round of persistent workgroups (ops/stencil.py::diffusion3d_step)."""
        if self.cart:  # boundary boxes are launched one by one by the caller
            self._launch_fused_box(rng, dt, exclusive)
            return
        (lo, hi), (lo2, hi2) = rng, rng2
        if hi > lo or hi2 > lo2:
            self.model.step(self.u, self.un, lo, hi, self.zact[0], self.zact[1], dt, lo2=lo2,
                            hi2=hi2, exclusive=exclusive)
            trace.sync_check(f"{self.model.name} fused step [{lo},{hi}) [{lo2},{hi2})",
                             self.device)

    def _fused_view(self, a: int, lo: int, hi: int):
        """View window, active and output bounds along array axis a (decomposition.fused_view)."""
        return fused_view(self.cd, self.model.radius, self.model.border, a, lo, hi)

    def _launch_fused_box(self, box, dt, exclusive=False, pick=False):
        """Fused step of a Cartesian block box (array order) on a kernel VIEW.  pick: measure
        the launch's z schedule instead of stepping (3-D; _pick_sched)."""
        if any(hi <= lo for lo, hi in box):
            return
        if self.grid.dims == 3:
            (z0, z1), (y0, y1), (x0, x1) = box
            (vy0, vy1), (ya0, ya1), (yo0, yo1) = self._fused_view(1, y0, y1)
            (vx0, vx1), (xa0, xa1), (xo0, xo1) = self._fused_view(2, x0, x1)
            sl = (slice(None), slice(vy0, vy1), slice(vx0, vx1))
            vbox = (xa0, xa1, ya0, ya1, xo0, xo1, yo0, yo1)
            if pick:
                self.model.sched_pick(self.u[sl], self.un[sl], z0, z1, self.zact[0],
                                      self.zact[1], dt, nx=vx1 - vx0, ny=vy1 - vy0, box=vbox)
                return
            self.model.step(self.u[sl], self.un[sl], z0, z1, self.zact[0], self.zact[1], dt,
                            nx=vx1 - vx0, ny=vy1 - vy0, box=vbox, exclusive=exclusive)
        else:
            (y0, y1), (x0, x1) = box
            (vx0, vx1), (xa0, xa1), (xo0, xo1) = self._fused_view(1, x0, x1)
            sl = (slice(None), slice(vx0, vx1))
            self.model.step(self.u[sl], self.un[sl], y0, y1, self.zact[0], self.zact[1], dt,
                            nx=vx1 - vx0, box=(xa0, xa1, xo0, xo1), exclusive=exclusive)
        trace.sync_check(f"{self.model.name} fused step box {box}", self.device)

    def _put_targets(self, field):
        """(cached per field and ipc epoch) the peer addresses of the fused step's halo
        puts into `field`'s counterparts.  First use: the device drains first, so every
        rank's fields are initialised (the IC, the partner clone) before a peer's store can
        land in them — the handshake in put_targets is pairwise, so the peer has drained
        too.  Never called for the first time inside a graph capture (_prepare_graph_halos
        resolves both fields before it)."""
        striped = self.halo.striped
        key = (field.data_ptr(), self._ipc_epoch(), self.halo.parity if striped else None)
        t = self._put_cache.get(key)
        if t is None:
            torch.cuda.synchronize(self.device)
            t = self.halo.put_parts(field) if striped else self.halo.put_targets(field)
            self._put_cache[key] = t
        return t

    def _prime_relays(self):
        """Striped fused puts: the kernel stores only the OUTPUT cells of its send rows, and
        the helpers forward whole rows, so every relay buffer must first hold the frozen
        cells (Dirichlet borders, padding) of its rows: one ordinary striped exchange of u
        per relay set, once per ipc epoch (collective; the ghost planes it writes already
        hold those values).  Outside any graph capture (_prepare_graph_halos / first step)."""
        if not (self.fput and self.halo.striped) or self._primed == self._ipc_epoch():
            return
        self.sync_halos()
        for _ in range(2):  # both relay sets (the exchange parity alternates)
            self.halo.start(self.u).wait()
        self._primed = self._ipc_epoch()

    def _step_fused_put(self, dt: float, pend) -> None:
        """One launch over every owned plane whose boundary output planes also go straight
        into the neighbours' ghost planes (the peers' output fields, IPC-mapped), then
        signal + wait on the comm stream:

            compute : [wait halo n-1 (join)][step n + puts] ------------> [step n+1 ...
            comm    :                                    [signal n, wait halo n]

        The wait for halo n-1 also orders this step's stores into a peer's field after the
        peer's step n-1, the last reader of that buffer (ping-pong: the peer's output of
        step n is its input of step n-1), so no acknowledgement is needed.  No boundary
        launch (its 4R-plane z warm-up per slab) and no put launch; the puts run beside
        the compute of every other workgroup."""
        if pend is not None:
            pend.wait()
        if self.halo.striped and self._primed != self._ipc_epoch():
            self._prime_relays()
        put = self._put_targets(self.un)
        with trace.range_("step+puts"):
            lo, hi = self.full
            if hi > lo:
                self.model.step(self.u, self.un, lo, hi, self.zact[0], self.zact[1], dt,
                                put=put)
                trace.sync_check(f"{self.model.name} fused step + puts [{lo},{hi})",
                                 self.device)
        self.u, self.un = self.un, self.u
        with trace.range_("halo_signal"):
            self._pending[id(self.u)] = self.halo.start(self.u, puts=False)
        self.t += dt
        self.it += 1

    def _step_fused(self, dt: float) -> None:
        pend = self._pending.pop(id(self.u), None)
        if self.fput:
            self._step_fused_put(dt, pend)
            return
        if self.bcomm and self.comm.size > 1:
            self._step_fused_bcomm(dt, pend)
            return
        if self.comm.size == 1:
            self._launch_fused(self.full, dt, exclusive=True)
        elif self.overlap:
            with trace.range_("interior"):
                self._launch_fused(self.interior, dt)
            with trace.range_("halo_wait"):
                if pend is not None:
                    pend.wait()
            with trace.range_("boundary"):  # both boundary slabs in ONE launch
                if self.cart:
                    for box in self.boundary:
                        self._launch_fused_box(box, dt)
                else:
                    self._launch_fused(self.boundary[0], dt, self.boundary[1])
        else:  # the launch starts after the exchange has completed: nothing runs beside it
            if pend is not None:
                pend.wait()
            self._launch_fused(self.full, dt, exclusive=True)
        self.u, self.un = self.un, self.u
        if self.comm.size > 1:
            with trace.range_("halo_start"):
                self._pending[id(self.u)] = self.halo.start(self.u)
        self.t += dt
        self.it += 1

    def _step_fused_bcomm(self, dt: float, pend) -> None:
        """Overlapped fused step, boundary launch on the comm stream: per rank two streams,

            compute : [interior n] ---------------------wait(bdone n)--> [interior n+1] ...
            comm    : [wait halo n-1][boundary n] bdone [puts n, signal, wait halo n] ...

        so the boundary launch starts as soon as the halo of u has arrived (not after the
        interior launch, as on the default path), the puts of its planes start right after
        it, and the interior launch runs beside the whole exchange.  The compute stream
        joins the comm stream at bdone only (the next interior launch reads the new
        boundary planes and overwrites the buffer the boundary launch read), never at the
        wait for the peers, so a spinning device wait never blocks a compute launch; the
        comm stream joins the compute stream before each boundary launch (the interior
        launch of the previous step read the buffer it overwrites).  No third stream."""
        cur = torch.cuda.current_stream(self.device)
        cs = self.comm_stream
        cs.wait_stream(cur)
        with trace.range_("interior"):
            self._launch_fused(self.interior, dt)
        with torch.cuda.stream(cs):
            if pend is not None:
                pend.wait()  # ipc: stream order on cs already (no event); rccl: joins RCCL
            with trace.range_("boundary"):
                if self.cart:
                    for box in self.boundary:
                        self._launch_fused_box(box, dt)
                else:
                    self._launch_fused(self.boundary[0], dt, self.boundary[1])
            bdone = torch.cuda.Event()
            bdone.record(cs)
            self.u, self.un = self.un, self.u
            with trace.range_("halo_start"):
                self._pending[id(self.u)] = self.halo.start(self.u, after_event=False)
        cur.wait_event(bdone)
        self.t += dt
        self.it += 1

    def step2_capable(self) -> bool:
        """Two fixed-dt steps in one launch (3-D FD2 heat: the model's step2, bit-identical
        to two steps) — where that is the faster launch for this shape (one rank: measured
        once per shape on the GPU before the first run, _pick_step2; several slab ranks:
        decided at construction, _choose_multirank_step2)."""
        if self.comm.size > 1:
            return self._mr2 and self._dt_dev is None
        return (self.fused and not self.cart and self.du is None
                and self.model.supports_step2 and self._dt_dev is None and self._pick2())

    def _pick_sched(self) -> None:
        """Banded or uniform z chunks for the fused 3-D launch that carries most planes (one
        rank: the full range; several: the interior range or box), measured once per launch
        shape on the GPU before any graph capture (diffusion_fused.hip step_bands; the
        kernel library caches the choice; ADVDIFF_STEP_BANDED=0/1 forces)."""
        if not (self.fused and self.grid.dims == 3 and self.kernel == "native"
                and self.device.type == "cuda" and hasattr(self.model, "sched_pick")):
            return
        dt = self.model.stable_dt() if not self.model.needs_umax else 0.0
        # fused puts: the one launch over every owned plane (timed without its puts: the
        # same geometry, the same cached choice)
        rng = self.full if self.comm.size == 1 or self.fput else self.interior
        if self.cart:
            self._launch_fused_box(rng, dt, pick=True)
        elif rng[1] > rng[0]:
            self.model.sched_pick(self.u, self.un, rng[0], rng[1], self.zact[0], self.zact[1],
                                  dt)

    def _pick_step2(self) -> bool:
        """One FD2 step or two per launch, decided before any graph capture: two per
        launch halves the HBM traffic but wins or loses by shape (+9-25 % at 384^3 and
        640^3-1024^3 fp64, -3 % at 512^3: profiles/r5/ab/step2_*.log).  The pick times
        both launches u -> un (u untouched; un is the step's scratch partner)."""
        if not (self.fused and self.comm.size == 1 and not self.cart and self.du is None
                and self.model.supports_step2):
            return False
        if self.kernel == "torch" or self.device.type != "cuda":
            return True
        lo, hi = self.full
        dt = self.model.stable_dt() if not self.model.needs_umax else 0.0
        return self.model.step2_preferred(self.u, self.un, lo, hi, self.zact[0], self.zact[1],
                                          dt)

    def step2(self, dt: float) -> None:
        """Two steps at the same dt (one launch when step2_capable)."""
        if not self.step2_capable():
            self.step(dt)
            self.step(dt)
            return
        ctx = stencil.use_torch_reference() if self.kernel == "torch" else contextlib.nullcontext()
        if self.comm.size > 1:
            with ctx:
                self._step2_multi(dt)
            return
        with ctx:
            self._pending.pop(id(self.u), None)
            lo, hi = self.full
            self.model.step2(self.u, self.un, lo, hi, self.zact[0], self.zact[1], dt)
            trace.sync_check(f"{self.model.name} fused 2-step [{lo},{hi})", self.device)
        self.u, self.un = self.un, self.u
        for _ in range(2):  # same rounding as two steps
            self.t += dt
        self.it += 2

    def _step2_multi(self, dt: float) -> None:
        """Two steps of a slab rank in two-step launches (6R ghost planes): the interior
        (owned planes >= 6R from a rank face: no ghost in their dependency cone) beside the
        halo, then each boundary slab, then ONE exchange of 6R planes — the schedule of
        _step_fused / _step_fused_bcomm with v6_march launches."""
        pend = self._pending.pop(id(self.u), None)
        z0, z1 = self.zact

        def launch(rng):
            lo, hi = rng
            if hi > lo:
                self.model.step2(self.u, self.un, lo, hi, z0, z1, dt)
                trace.sync_check(f"{self.model.name} fused 2-step [{lo},{hi})", self.device)

        if self.bcomm:
            cur = torch.cuda.current_stream(self.device)
            cs = self.comm_stream
            cs.wait_stream(cur)
            with trace.range_("interior"):
                launch(self.interior)
            with torch.cuda.stream(cs):
                if pend is not None:
                    pend.wait()
                with trace.range_("boundary"):
                    for rng in self.boundary:
                        launch(rng)
                bdone = torch.cuda.Event()
                bdone.record(cs)
                self.u, self.un = self.un, self.u
                with trace.range_("halo_start"):
                    self._pending[id(self.u)] = self.halo.start(self.u, after_event=False)
            cur.wait_event(bdone)
        else:
            if self.overlap:
                with trace.range_("interior"):
                    launch(self.interior)
                with trace.range_("halo_wait"):
                    if pend is not None:
                        pend.wait()
                with trace.range_("boundary"):
                    for rng in self.boundary:
                        launch(rng)
            else:
                if pend is not None:
                    pend.wait()
                launch(self.full)
            self.u, self.un = self.un, self.u
            with trace.range_("halo_start"):
                self._pending[id(self.u)] = self.halo.start(self.u)
        for _ in range(2):  # same rounding as two steps
            self.t += dt
        self.it += 2

    def _steps(self, n: int, dt: float) -> None:
        """n steps at a fixed dt: pairs in one launch where possible."""
        if self.step2_capable():
            for _ in range(n // 2):
                self.step2(dt)
            n %= 2
        for _ in range(n):
            self.step(dt)

    def step(self, dt: float) -> None:
        if self.kernel == "torch":
            with stencil.use_torch_reference():
                self._step(dt)
        else:
            self._step(dt)

    def _step(self, dt: float) -> None:
        if self.fused:
            self._step_fused(dt)
            return
        stage = self._stage_lu if self.exchange == "lu" else self._stage
        if self.du is not None:
            for A, Bc in zip(LSRK45_A, LSRK45_B):
                stage(self.u, self.du, self.un, A, Bc, dt, ls=True)
                self.u, self.un = self.un, self.u
        else:
            u, A, B = self.u, self.A, self.B
            (a1, b1), (a2, b2), (a3, b3) = RK3
            stage(u, None, A, a1, b1, dt)
            stage(A, u, B, a2, b2, dt)
            stage(B, u, u, a3, b3, dt)
        if self._dt_dev is None:  # device-dt steps keep t / it on the device
            self.t += dt
            self.it += 1

    def sync_halos(self):
        """Complete every in-flight exchange (stream-ordered)."""
        for p in list(self._pending.values()):
            if p is not None:
                p.wait()
        self._pending.clear()

    def _sync(self):
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)

    # ------------------------------------------------------------------------------
    def reducer(self):
        if self._reducer is None:
            self._reducer = stencil.NormReducer(self.device)
        return self._reducer

    def global_max_abs(self) -> float:
        r = self.reducer()
        _, _, mx = r(self.u, None, self._owned_xyz_box())
        return self.comm.allreduce_max(mx)

    def dt(self) -> float:
        umax = self.global_max_abs() if self.model.needs_umax else None
        return self.model.stable_dt(umax)

    # ------------------------------------------------------------------------------
    # hipGraph replay (single process): one graph = GRAPH_STEPS steps at a fixed dt.
    # Small grids are launch-bound (a 1001² heat stage is ~5 µs of HBM time); replaying
    # a captured graph removes the per-launch host cost (ctypes + hipLaunchKernel).
    # ------------------------------------------------------------------------------
    GRAPH_STEPS = 8  # even: fused / LSRK paths ping-pong u/un, so buffers line up on replay

    def graph_capable(self) -> bool:
        """Single process, or several ranks whose halos are device puts (ipc transport:
        every exchange step is a stream-ordered kernel, so a whole multi-rank step —
        interior, puts, flags, waits, boundary — replays as one graph)."""
        multi_ok = self.comm.size == 1 or self.transport == "ipc"
        return (self.device.type == "cuda" and multi_ok and self.exchange == "u"
                and not trace.SYNC_DEBUG
                and not trace.TRACE)

    def _prepare_graph_halos(self):
        """Multi-rank capture: join every in-flight exchange into the current stream (an
        event recorded outside a capture cannot be waited on inside it) and learn the
        peers' receive addresses of every field now (the one-time handshake is host
        communication, which a capture must not contain)."""
        if self.comm.size > 1:
            self.sync_halos()
            for f in self.fields():
                self.halo.prepare(f)
            if self.fput:
                self._prime_relays()
                for f in self.fields():
                    for _ in range(2 if self.halo.striped else 1):  # both relay sets
                        self._put_targets(f)
                        if self.halo.striped:
                            self.halo.parity ^= 1

    def _graph_for(self, dt: float | None, t_end: float | None = None):
        """dt=None: a graph of device-dt (adaptive CFL) steps towards t_end."""
        self.tune_launches()  # never inside the capture
        # A graph bakes in the buffer addresses: the fused / LSRK paths ping-pong u <-> un,
        # so after an odd number of eager steps the other parity needs its own graph.
        # multi-rank ipc: the graph also bakes in the peers' receive addresses, valid for the
        # IpcPeers epoch it was captured in
        ep = self._ipc_epoch()
        # striped halos: the relay buffer set of the first exchange is baked in as well
        key = (None if dt is None else float(dt), t_end, self.GRAPH_STEPS, self.u.data_ptr(),
               getattr(self.halo, "parity", 0), ep)
        g = getattr(self, "_graphs", {}).get(key)
        if g is not None:
            return g
        if not hasattr(self, "_graphs"):
            self._graphs = {}
        self._graphs = {k: v for k, v in self._graphs.items() if k[-1] == ep}
        # state snapshot: capture executes nothing, but keep t/it bookkeeping exact
        t, it = self.t, self.it
        self._prepare_graph_halos()
        side = torch.cuda.Stream(device=self.device)
        side.wait_stream(torch.cuda.current_stream())
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.stream(side):
            with torch.cuda.graph(graph, stream=side):
                if dt is None:
                    for _ in range(self.GRAPH_STEPS):
                        self._step_device_dt(t_end)
                else:
                    self._steps(self.GRAPH_STEPS, dt)
                if self.comm.size > 1:
                    self.sync_halos()  # every comm-stream fork joins back into the capture
        torch.cuda.current_stream().wait_stream(side)
        self.t, self.it = t, it
        self._graphs[key] = graph
        return graph

    def _advance(self, n: int, dt: float, use_graph: bool):
        if use_graph and n >= self.GRAPH_STEPS:
            g = self._graph_for(dt)
            if self.comm.size > 1:
                self.sync_halos()  # halos of eager steps: joined before the replay
            for _ in range(n // self.GRAPH_STEPS):
                g.replay()
                for _ in range(self.GRAPH_STEPS):  # same rounding as eager stepping
                    self.t += dt
                self.it += self.GRAPH_STEPS
            n %= self.GRAPH_STEPS
        self._steps(n, dt)

    # ------------------------------------------------------------------------------
    # adaptive CFL on the device: max|u| (norm reducer) -> RCCL MAX allreduce on the
    # stream -> advdiff_adaptive_dt -> stage kernels read dt from device memory.  The
    # host learns t only at chunk ends; steps issued past t_end get dt = 0 and are exact
    # no-ops.  Same step sequence as the host-driven loop (bitwise; tests).
    # ------------------------------------------------------------------------------
    def _allreduce_max_device(self, red):
        import torch.distributed as dist
        v = red[2:3]
        if self.comm.backend == "nccl":
            dist.all_reduce(v, op=dist.ReduceOp.MAX)  # on-stream, no host sync
        else:  # gloo (CPU / one-GPU tests): host round trip
            h = v.cpu()
            dist.all_reduce(h, op=dist.ReduceOp.MAX)
            v.copy_(h)

    def _step_device_dt(self, t_end):
        red = self.reducer()(self.u, None, self._owned_xyz_box(), sync=False)
        if self.comm.size > 1:
            self._allreduce_max_device(red)
        cfl_h, dv = self.model.cfl_terms()
        stencil.adaptive_dt(red, self._dts, cfl_h=cfl_h, dt_visc=dv, t_end=t_end)
        self._dt_dev = self._dts[1:2]
        try:
            self.step(0.0)  # the kernels take dt from _dt_dev
        finally:
            self._dt_dev = None

    def _issue_device_dt(self, n, t_end, use_graph):
        if use_graph and n >= self.GRAPH_STEPS:
            g = self._graph_for(None, t_end)
            for _ in range(n // self.GRAPH_STEPS):
                g.replay()
            n %= self.GRAPH_STEPS
        for _ in range(n):
            self._step_device_dt(t_end)

    def _advance_device_dt(self, iters, t_end, use_graph):
        import math
        if self._dts is None:
            self._dts = torch.zeros(3, dtype=torch.float64, device=self.device)
        self._dts.copy_(torch.tensor([self.t, 0.0, 0.0], dtype=torch.float64))
        it0 = self.it
        if iters is not None:
            self._issue_device_dt(iters, None, use_graph)
            t, _, steps = self._dts.tolist()
        else:
            n = 1
            while True:
                self._issue_device_dt(n, t_end, use_graph)
                t, dt_last, steps = self._dts.tolist()  # the chunk's only host sync
                if t >= t_end * (1 - 1e-14) or dt_last == 0.0:
                    break
                n = int(min(max(math.ceil((t_end - t) / dt_last), 1), 64))
        self.t, self.it = t, it0 + int(steps)

    def run(self, iters: int | None = None, t_end: float | None = None, dt: float | None = None,
            callback=None, graph: bool | None = None) -> RunStats:
        """Advance `iters` steps (fixed dt) or until `t_end`. Times the loop with a
        barrier + device sync on both sides (reference: MPI_Barrier-fenced MPI_Wtime,
        `main.c:184-186,305-307`).  graph=None: replay hipGraphs when possible (single
        process, fixed dt, no per-step callback/watchdog)."""
        if iters is None and t_end is None:
            raise ValueError("give iters or t_end")
        self.tune_launches()  # outside the timed region, before any capture
        fixed_dt = dt if dt is not None else (None if self.model.needs_umax else self.dt())
        dev_dt = (fixed_dt is None and self.device_dt and callback is None
                  and not self.check_every and _FAULT is None)
        use_graph = (self.graph_capable() and (fixed_dt is not None or dev_dt)
                     and callback is None and not self.check_every) if graph is None else graph
        if self.comm.size > 1 and fixed_dt is None:
            use_graph = False  # the device-dt chunk's max|u| allreduce is not captured
        if use_graph:  # capture outside the timed region (like a warm-up)
            if fixed_dt is not None:
                self._graph_for(fixed_dt)
            elif dev_dt:
                if self._dts is None:
                    self._dts = torch.zeros(3, dtype=torch.float64, device=self.device)
                self._graph_for(None, t_end if iters is None else None)
        self._sync()
        self.comm.barrier()
        t_start = time.perf_counter()
        steps0 = self.it
        if dev_dt:
            self._advance_device_dt(iters, t_end, use_graph)
        elif use_graph:
            if iters is not None:
                n = iters
            else:  # full steps that fit before t_end, then a short last step
                n = max(int((t_end - self.t) / fixed_dt * (1 + 1e-12)), 0)
                while n > 0 and self.t + n * fixed_dt > t_end:
                    n -= 1
            self._advance(n, fixed_dt, True)
        # two steps per launch where the model has it and nothing runs between steps
        pair_ok = (fixed_dt is not None and callback is None and not self.check_every
                   and _FAULT is None and self.step2_capable())
        while not dev_dt:
            if iters is not None and self.it - steps0 >= iters:
                break
            if t_end is not None and self.t >= t_end * (1 - 1e-14):
                break
            h = fixed_dt if fixed_dt is not None else self.dt()
            if t_end is not None and self.t + h > t_end:
                h = t_end - self.t
            if pair_ok and h == fixed_dt:
                if iters is not None:
                    pair = iters - (self.it - steps0) >= 2
                else:  # the second step is a full one as well (same test as the loop's)
                    t1 = self.t + h
                    pair = t1 < t_end * (1 - 1e-14) and t1 + h <= t_end
                if pair:
                    with trace.range_(f"steps {self.it}-{self.it + 1}"):
                        self.step2(h)
                    continue
            with trace.range_(f"step {self.it}"):
                self.step(h)
            if _FAULT is not None and _FAULT == (self.comm.rank, self.it):
                raise RuntimeError(f"injected fault on rank {self.comm.rank} at step {self.it}")
            if self.check_every and self.it % self.check_every == 0:
                self.check_finite()
            if callback is not None:
                callback(self)
        self.sync_halos()
        self._sync()
        self.comm.barrier()
        elapsed = time.perf_counter() - t_start
        elapsed = self.comm.allreduce_max(elapsed)
        st = RunStats(steps=self.it - steps0, t=self.t, compute_s=elapsed)
        return st

    # ------------------------------------------------------------------------------
    # diagnostics
    # ------------------------------------------------------------------------------
    def check_finite(self):
        """NaN/Inf watchdog (absent in the reference).  Σ|u| as well as
        max|u|: the device reduction takes its max with fmax, which drops NaN operands, so
        an isolated NaN cell shows only in the sum; the ranks agree on a flag (NaN
        comparisons inside a MAX allreduce are not reliable either)."""
        s1, _, mx = self.reducer()(self.u, None, self._owned_xyz_box())
        bad = 0.0 if (np.isfinite(s1) and np.isfinite(mx)) else 1.0
        if self.comm.allreduce_max(bad) > 0.0:
            raise FloatingPointError(f"non-finite solution at step {self.it}, t={self.t:g}")
        return self.comm.allreduce_max(mx)

    def bit_hash(self, chunk_cells: int = 1 << 26) -> int:
        """Order-independent 64-bit hash of the global solution's BIT PATTERNS: the sum
        (mod 2^64) over the owned cells of mix(global linear index, raw bits).  Equal for
        every decomposition, transport and rank count exactly when the solutions agree
        bit for bit (up to a 2^-64 collision chance) — the N-rank-vs-1-GPU check of
        bench.py compares it without gathering the field.  Collective (all ranks)."""
        self.sync_halos()
        own = self.owned
        gb = self.cd.global_box()
        gshape = self.cd.shape
        dev = own.device
        ibits = torch.int64 if own.element_size() == 8 else torch.int32
        # strides of the global linear index, array order
        gstr = [1] * len(gshape)
        for a in range(len(gshape) - 2, -1, -1):
            gstr[a] = gstr[a + 1] * gshape[a + 1]
        rest = [torch.arange(s, s + c, dtype=torch.int64, device=dev) * st
                for (s, c), st in zip(gb[1:], gstr[1:])]
        inner = rest[0]
        for r in rest[1:]:
            inner = inner[..., None] + r
        per = max(1, chunk_cells // max(inner.numel(), 1))
        K1, K2 = -7046029254386353131, -4658895280553007687  # odd 64-bit mixers
        h = torch.zeros((), dtype=torch.int64, device=dev)
        n0 = own.shape[0]
        for z0 in range(0, n0, per):
            z1 = min(n0, z0 + per)
            bits = own[z0:z1].contiguous().view(ibits).to(torch.int64)
            zi = torch.arange(gb[0][0] + z0, gb[0][0] + z1, dtype=torch.int64, device=dev)
            idx = zi.view((-1,) + (1,) * inner.dim()) * gstr[0] + inner
            x = (bits ^ (idx * K1)) * K2
            x = x ^ ((x >> 31) & 0x1FFFFFFFF)  # logical shift of the high half
            h = h + (x * K1).sum()
        tot = self.comm.allreduce_tensor(h.view(1), "sum") if self.comm.size > 1 else h.view(1)
        return int(tot.item())

    def error_norms(self, exact: torch.Tensor | None = None, K: float | None = None,
                    t_exact: float | None = None):
        """Global (L1, L2, Linf) of u - exact, with the reference's cell-volume weights
        (`Matlab_Prototipes/DiffusionNd/heat3d.m`, fixed `CalcError` indexing)."""
        cd = self.cd
        if exact is None:
            K = K if K is not None else getattr(self.model, "K", 1.0)
            tt = self.t if t_exact is None else t_exact
            # same (ghost-inclusive, padded) layout as u, so both share the strides
            offs = [cd.axis(a).start - cd.ghost_of_axis(a) for a in range(cd.dims)]
            exact = ics.exact_solution_box(self.ic_name, self.grid.shape, self.grid.spacing,
                                           tt, K, self.ic_params, offs, list(cd.alloc),
                                           self.sx, self.dtype, self.device)
            if self.ypad:  # the plane padding rows (never read)
                e = torch.zeros_like(self.u)
                e[:, :exact.shape[1]] = exact
                exact = e
        elif tuple(exact.shape) != tuple(self.u.shape):
            raise ValueError(f"exact must have the local layout {tuple(self.u.shape)}")
        r = self.reducer()
        s1, s2, mx = r(self.u, exact, self._owned_xyz_box())
        s1 = self.comm.allreduce_sum(s1)
        s2 = self.comm.allreduce_sum(s2)
        mx = self.comm.allreduce_max(mx)
        vol = float(np.prod(self.grid.spacing))
        return vol * s1, (vol * s2) ** 0.5, mx

    # ------------------------------------------------------------------------------
    # I/O
    # ------------------------------------------------------------------------------
    def gather(self) -> np.ndarray | None:
        """Global solution (no ghosts) on rank 0 as numpy [z][y][x] ([y][x] in 2-D)."""
        self.sync_halos()
        self._sync()
        if self.cart:
            boxes = [self.cd.global_box(r) for r in range(self.comm.size)]
            g = self.comm.gather_boxes(self.owned.contiguous(), boxes, self.cd.shape)
        else:
            counts = [self.d.count_of(r) for r in range(self.comm.size)]
            g = self.comm.gather_planes(self.owned.contiguous(), counts)
        return None if g is None else g.numpy()

    def copy_to_host(self) -> None:
        """Per-rank device-to-host copy of the owned block through one reused pinned
        buffer of a few planes (the reference's timed DtH without the rank-0 merge; host
        memory O(planes) at any grid size).  Returns None."""
        self.sync_halos()
        self._sync()
        own = self.owned
        if own.device.type != "cuda":
            return None
        n0 = own.shape[0]
        per = max(1, (64 << 20) // max(own[0].numel() * own.element_size(), 1))
        buf = torch.empty((min(per, n0),) + tuple(own.shape[1:]), dtype=own.dtype,
                          pin_memory=True)
        for z0 in range(0, n0, per):
            z1 = min(n0, z0 + per)
            buf[:z1 - z0].copy_(own[z0:z1], non_blocking=True)
            torch.cuda.current_stream(self.device).synchronize()
        return None

    def gather_with_ghosts(self) -> np.ndarray | None:
        """Rank 0: every rank's slab INCLUDING its ghost planes, concatenated in rank
        order — the reference's multi-GPU result.bin layout (each rank's Nx*Ny*(_Nz+6)
        block, SaveBinary3D(h_u, Nx, Ny, NZ), MultiGPU/Diffusion3d_Baseline/main.c:341,
        Tools.c:91-119).  Slab decompositions only."""
        if self.cart:
            raise ValueError("gather_with_ghosts: slab decompositions only")
        self.sync_halos()
        self._sync()
        nx = self.grid.shape[0]
        # crop the row padding and, in 3-D, the plane padding rows (pitched fields)
        local = (self.u[:, :self.grid.shape[1], :nx] if self.grid.dims == 3
                 else self.u[..., :nx]).contiguous()
        counts = [self.cd.axis(0, r).alloc for r in range(self.comm.size)]
        g = self.comm.gather_planes(local, counts)
        return None if g is None else g.numpy()

    def save_result(self, path) -> None:
        g = self.gather()
        if self.comm.rank == 0:
            aio.save_binary(path, g)

    def meta(self) -> dict:
        return {"grid": list(self.grid.shape), "lengths": list(self.grid.lengths),
                "t": self.t, "it": self.it, "model": self.model.describe(),
                "ic": self.ic_name, "world": self.comm.size, "pgrid": list(self.pgrid),
                "integrator": self.integrator}

    def save_checkpoint(self, prefix):
        self.sync_halos()
        self._sync()
        local = self.owned.detach().to(torch.float64).cpu().numpy()
        box0 = [s for s, _ in self.cd.global_box()]
        path = aio.save_checkpoint(prefix, self.comm.rank, local, self.d.start, self.meta(),
                                   box0=box0)
        self.comm.barrier()  # every shard written before stale ones are removed
        if self.comm.rank == 0:
            aio.remove_stale_shards(prefix, self.comm.size)
        self.comm.barrier()
        return path

    def load_checkpoint(self, prefix):
        """Restart from shards written by ANY decomposition of the same grid."""
        gb = self.cd.global_box()
        arr, meta = aio.load_checkpoint_box(prefix, [s for s, _ in gb], [c for _, c in gb])
        if list(meta["grid"]) != list(self.grid.shape):
            raise ValueError(f"checkpoint grid {meta['grid']} != {list(self.grid.shape)}")
        src = torch.from_numpy(arr).to(self.device, self.dtype)
        self.owned.copy_(src)
        self.t = float(meta["t"])
        self.it = int(meta["it"])
        self._pending.clear()
        self.halo.exchange(self.u)
        for f in self.fields()[1:]:
            f.copy_(self.u)
        return meta

    # ------------------------------------------------------------------------------
    def summary(self, stats: RunStats, style: str = "multigpu", extra=None) -> str:
        g = self.grid
        cells = g.cells
        gf = metrics.gflops_reference(stats.compute_s, stats.steps, cells,
                                      times3=(style == "multigpu" or self.model.name == "burgers"))
        ml = metrics.mlups(stats.compute_s, stats.steps, cells)
        # LSRK stage: read u, du; write du, u (stage 1 skips the du read)
        # (per-stage launches of a fusable model — LSRK, thin slabs, --exchange lu — move
        # the per-stage 64 B, not the fused step's 16 B)
        bpc = (5 * 32.0 - 8.0 if self.du is not None
               else self.model.bytes_per_cell_step if self.fused else 64.0)
        if self.step2_capable():  # two steps per launch: u^n read and u^{n+2} written once
            bpc /= 2.0
        bw = bpc * cells * stats.steps / max(stats.compute_s, 1e-30)
        ex = {("MLUPS (cells x RK steps / s)" if self.du is not None
               else "MLUPS (cells x RK3 steps / s)"): f"{ml:.1f}",
              "Stage-MLUPS": f"{(5 if self.du is not None else 3) * ml:.1f}",
              "Effective HBM bandwidth (GB/s, est.)": f"{bw / 1e9:.1f}",
              "Processes / devices": f"{self.comm.size} x {self.device.type}"}
        if self.exchange == "lu":
            ex["Halo payload"] = "RHS L(u) boundary planes, redundant ghost update"
        if extra:
            ex.update(extra)
        opt = "Fused LDS z-march + RK3 (gfx950)" if self.device.type == "cuda" else "PyTorch CPU"
        if self.device.type == "cuda" and (self.kernel == "torch" or self.exchange == "lu"):
            opt = "PyTorch reference ops (GPU)"
        if style == "multigpu":
            return metrics.summary_multigpu(self.model.title, opt, stats.compute_s, stats.htod_s,
                                            stats.dtoh_s, gf, stats.steps, g.shape, ex,
                                            stages=5 if self.du is not None else 3)
        return metrics.summary_singlegpu(self.model.title, opt, stats.compute_s, gf, stats.steps,
                                         g.shape, stats.t, ex)
