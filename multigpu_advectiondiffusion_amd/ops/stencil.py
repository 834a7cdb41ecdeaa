"""Device-dispatching stencil ops.

``cuda`` (HIP) tensors run the hand-written gfx950 kernels of ``libadvdiff.so``; CPU
tensors run the PyTorch reference (``ops/reference.py``).  There is deliberately NO silent
fallback for device tensors: if the native library is missing on a GPU box the op raises.

All ops enqueue on the current HIP stream (``torch.cuda.current_stream()``) unless a
``stream`` is given, and never synchronise, so they can be captured into a hipGraph.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib
from . import reference as ref

_DT = {torch.float32: 0, torch.float64: 1}

# Explicit A/B switch: run the PyTorch reference ops (ops/reference.py) on device tensors
# instead of the HIP kernels — the "naive kernel" baseline of SURVEY.md §7.1.  Off by
# default and never a silent fallback: it must be requested (use_torch_reference() or
# Solver(kernel="torch")).
_TORCH_REF = False


class use_torch_reference:
    """Context manager (or call .enable()/.disable()) selecting the PyTorch stencil ops."""

    def __init__(self, on: bool = True):
        self.on = on

    def __enter__(self):
        global _TORCH_REF
        self.prev, _TORCH_REF = _TORCH_REF, self.on
        return self

    def __exit__(self, *exc):
        global _TORCH_REF
        _TORCH_REF = self.prev


def _native(t) -> bool:
    return t.is_cuda and not _TORCH_REF


def _dtype_code(t: torch.Tensor) -> int:
    try:
        return _DT[t.dtype]
    except KeyError:
        raise TypeError(f"unsupported dtype {t.dtype} (float32/float64 only)") from None


def _stream_ptr(stream) -> int:
    s = stream if stream is not None else torch.cuda.current_stream()
    return s.cuda_stream


def _check_layout(*ts):
    for t in ts:
        if t is None:
            continue
        if t.stride(-1) != 1:
            raise ValueError("x (last axis) must be contiguous")


def _ptr(t):
    return None if t is None else t.data_ptr()


def _aux_ptr(u0, a, ls):
    if ls:
        if u0 is None:
            raise ValueError("low-storage RK stage needs the du buffer")
        return u0.data_ptr()
    return _ptr(u0) if a != 0 else None


def diffusion3d_stage(inp, u0, out, *, nx, ny, k0, k1, border, order, cx, cy, cz, dt, a, b,
                      stream=None, ls=False):
    """out[k0:k1] = a*u0 + b*(inp + dt*K∇²inp) on the interior box (see kernels.h).
    ls=True: low-storage RK stage, u0 is du: du = a*du + dt*L; out = inp + b*du."""
    _check_layout(inp, u0, out)
    if _native(inp):
        lib = _lib.require()
        R = order // 2
        assert k0 >= R and k1 + R <= inp.shape[0], "stencil planes out of bounds"
        assert nx <= inp.shape[2] and ny <= inp.shape[1]
        fn = lib.advdiff_diffusion3d_stage_ls if ls else lib.advdiff_diffusion3d_stage
        code = fn(_dtype_code(inp), _ptr(inp), _aux_ptr(u0, a, ls), _ptr(out), nx, ny,
                  inp.stride(1), inp.stride(0), k0, k1, border, order, cx, cy, cz, dt, a, b,
                  _stream_ptr(stream))
        _lib.check(code, "diffusion3d_stage")
    else:
        ref.diffusion3d_stage(inp, u0, out, nx, ny, k0, k1, border, order, cx, cy, cz, dt, a, b,
                              ls)


def _int_array(vals):
    import ctypes
    return (ctypes.c_int * len(vals))(*[int(v) for v in vals])


EXCLUSIVE = 1  # ADVDIFF_EXCLUSIVE (kernels.h)


def diffusion3d_step(uin, uout, *, nx, ny, k0, k1, zlo, zhi, border, order, cx, cy, cz, dt,
                     stream=None, k0b=0, k1b=0, box=None, exclusive=False, put=None):
    """A FULL SSP-RK3 step in one launch (temporal blocking): uout[k0:k1] = RK3(uin), and
    uout[k0b:k1b] too when a second range is given (one launch for both).
    box = (xa0, xa1, ya0, ya1, xo0, xo1, yo0, yo1): explicit active / output x-y bounds
    (Cartesian blocks launched on a view); default from `border`.
    exclusive=True: nothing else runs on the GPU meanwhile (single rank / full-range
    launch) -> one round of persistent workgroups; False (an interior launch overlapping
    RCCL) keeps the dynamically balanced grid of z chunks.  Results are bit-identical.
    put: the ipc transport's fused halo puts (one plane range, default box, native device
    fields) — ((dst_lo, lo_k0, lo_k1), (dst_hi, hi_k0, hi_k1)): the output planes
    [lo_k0, lo_k1) / [hi_k0, hi_k1) also go to the peer addresses dst_lo / dst_hi (the peer
    plane of local plane lo_k0 / hi_k0; 0 = no peer; advdiff_diffusion3d_step_put); or a
    list of parts (dst, k0, k1, y0, y1, plane_bytes): planes [k0, k1), rows [y0, y1) to
    dst + (k - k0) plane_bytes + the own in-plane offset (striped exchanges;
    advdiff_diffusion3d_step_putv, up to 6 parts)."""
    _check_layout(uin, uout)
    if uin.data_ptr() == uout.data_ptr():
        raise ValueError("the fused step needs distinct input/output buffers")
    if put is not None:
        if not _native(uin) or box is not None or k1b > k0b:
            raise ValueError("fused halo puts: native device fields, one range, default box")
        lib = _lib.require()
        nz = uin.shape[0]
        assert 0 <= k0 and k1 <= nz and 0 <= zlo and zhi <= nz
        assert nx <= uin.shape[2] and ny <= uin.shape[1]
        if len(put) == 2 and len(put[0]) == 3:  # the two-face form
            (dlo, lo0, lo1), (dhi, hi0, hi1) = put
            code = lib.advdiff_diffusion3d_step_put(
                _dtype_code(uin), _ptr(uin), _ptr(uout), nx, ny, uin.stride(1), uin.stride(0),
                nz, k0, k1, zlo, zhi, border, order, cx, cy, cz, dt, dlo or None, lo0, lo1,
                dhi or None, hi0, hi1, _stream_ptr(stream))
        else:
            n = len(put)
            if n > 6:
                raise ValueError("fused halo puts: at most 6 parts")
            arr = [list(col) for col in zip(*put)] if n else [[]] * 6
            code = lib.advdiff_diffusion3d_step_putv(
                _dtype_code(uin), _ptr(uin), _ptr(uout), nx, ny, uin.stride(1), uin.stride(0),
                nz, k0, k1, zlo, zhi, border, order, cx, cy, cz, dt, n,
                (ctypes.c_void_p * max(n, 1))(*arr[0]), _int_array(arr[1]),
                _int_array(arr[2]), _int_array(arr[3]), _int_array(arr[4]),
                (ctypes.c_int64 * max(n, 1))(*arr[5]), _stream_ptr(stream))
        _lib.check(code, "diffusion3d_step_put")
        return
    if box is None:
        box = (border, nx - border, border, ny - border, 0, nx, 0, ny)
    if _native(uin):
        lib = _lib.require()
        nz = uin.shape[0]
        assert 0 <= k0 and k1 <= nz and 0 <= zlo and zhi <= nz and 0 <= k0b and k1b <= nz
        assert nx <= uin.shape[2] and ny <= uin.shape[1]
        code = lib.advdiff_diffusion3d_step_box_ex(
            _dtype_code(uin), _ptr(uin), _ptr(uout), nx, ny, uin.stride(1), uin.stride(0), nz,
            k0, k1, k0b, k1b, zlo, zhi, _int_array(box), order, cx, cy, cz, dt,
            EXCLUSIVE if exclusive else 0, _stream_ptr(stream))
        _lib.check(code, "diffusion3d_step")
    else:
        for a, b in ((k0, k1), (k0b, k1b)):
            if b > a:
                ref.diffusion3d_step_box(uin, uout, nx, ny, a, b, zlo, zhi, box, order, cx, cy,
                                         cz, dt)


def diffusion3d_step2_pick(uin, uout, *, nx, ny, k0, k1, zlo, zhi, border, cx, cy, cz, dt,
                           stream=None, box=None) -> bool:
    """True if two FD2 steps per launch beat one step per launch for this shape on this
    GPU (advdiff_diffusion3d_step2_pick: measured once per shape and process; uin is not
    modified, uout is used as scratch; ADVDIFF_STEP2=0/1 forces).  Synchronous: call it
    outside a graph capture.  Not a native device field: True (the CPU path pairs)."""
    import os
    if not _native(uin):
        return os.environ.get("ADVDIFF_STEP2", "1") != "0"
    _check_layout(uin, uout)
    if box is None:
        box = (border, nx - border, border, ny - border, 0, nx, 0, ny)
    lib = _lib.require()
    use2 = ctypes.c_int(0)
    code = lib.advdiff_diffusion3d_step2_pick(
        _dtype_code(uin), _ptr(uin), _ptr(uout), nx, ny, uin.stride(1), uin.stride(0),
        uin.shape[0], k0, k1, zlo, zhi, _int_array(box), cx, cy, cz, dt, _stream_ptr(stream),
        ctypes.byref(use2))
    _lib.check(code, "diffusion3d_step2_pick")
    return bool(use2.value)


def diffusion3d_step_sched_pick(uin, uout, *, nx, ny, k0, k1, zlo, zhi, border, order, cx,
                                cy, cz, dt, stream=None, box=None) -> bool:
    """Measure the banded against the uniform z schedule of this fused-step launch
    (advdiff_diffusion3d_step_sched_pick: uin -> uout, uout is scratch; synchronous, call
    it outside a graph capture) and keep the faster for every later launch of it.  True
    if banded.  Not a native device field: False (nothing to pick)."""
    if not _native(uin):
        return False
    _check_layout(uin, uout)
    if box is None:
        box = (border, nx - border, border, ny - border, 0, nx, 0, ny)
    lib = _lib.require()
    out = ctypes.c_int(0)
    code = lib.advdiff_diffusion3d_step_sched_pick(
        _dtype_code(uin), _ptr(uin), _ptr(uout), nx, ny, uin.stride(1), uin.stride(0),
        uin.shape[0], k0, k1, zlo, zhi, _int_array(box), order, cx, cy, cz, dt,
        _stream_ptr(stream), ctypes.byref(out))
    _lib.check(code, "diffusion3d_step_sched_pick")
    return bool(out.value)


def diffusion3d_step2x(uin, uout, *, nx, ny, k0, k1, zlo, zhi, border, cx, cy, cz, dt,
                       stream=None, box=None):
    """TWO FD2 SSP-RK3 steps in one launch (diffusion_fused.hip v6_march): uout[k0:k1] =
    RK3(RK3(uin)), bit-identical to two diffusion3d_step calls through a scratch field
    (the first on the whole active box, the second on the output box).
    u^n is read once and u^{n+2} written once: half the HBM traffic per step.  The planes
    within 5 of [k0, k1) must hold u^n (one rank: the whole field)."""
    _check_layout(uin, uout)
    if uin.data_ptr() == uout.data_ptr():
        raise ValueError("the fused step needs distinct input/output buffers")
    if box is None:
        box = (border, nx - border, border, ny - border, 0, nx, 0, ny)
    if _native(uin):
        lib = _lib.require()
        nz = uin.shape[0]
        assert 0 <= k0 and k1 <= nz and 0 <= zlo and zhi <= nz
        assert nx <= uin.shape[2] and ny <= uin.shape[1]
        code = lib.advdiff_diffusion3d_step2x(
            _dtype_code(uin), _ptr(uin), _ptr(uout), nx, ny, uin.stride(1), uin.stride(0), nz,
            k0, k1, zlo, zhi, _int_array(box), cx, cy, cz, dt, _stream_ptr(stream))
        _lib.check(code, "diffusion3d_step2x")
    elif k1 > k0:
        # the kernel's dependency cone: U1 on [k0-5, k1+5) from u^n, then u^{n+2}
        # (u^{n+1} on the whole active box: the output box applies to u^{n+2})
        nz = uin.shape[0]
        mid = uin.clone()
        box1 = tuple(box[:4]) + (0, nx, 0, ny)
        ref.diffusion3d_step_box(uin, mid, nx, ny, max(k0 - 5, zlo, 1), min(k1 + 5, zhi, nz - 1),
                                 zlo, zhi, box1, 2, cx, cy, cz, dt)
        ref.diffusion3d_step_box(mid, uout, nx, ny, k0, k1, zlo, zhi, box, 2, cx, cy, cz, dt)


def diffusion2d_step(uin, uout, *, nx, j0, j1, ylo, yhi, border, order, cx, cy, dt,
                     stream=None, box=None):
    """A FULL 2-D SSP-RK3 step in one launch: uout[j0:j1] = RK3(uin) (rows).
    box = (xa0, xa1, xo0, xo1): explicit active / output columns (Cartesian blocks)."""
    _check_layout(uin, uout)
    if uin.data_ptr() == uout.data_ptr():
        raise ValueError("the fused step needs distinct input/output buffers")
    if box is None:
        box = (border, nx - border, 0, nx)
    if _native(uin):
        lib = _lib.require()
        ny = uin.shape[0]
        assert 0 <= j0 and j1 <= ny and 0 <= ylo and yhi <= ny and nx <= uin.shape[1]
        code = lib.advdiff_diffusion2d_step_box(
            _dtype_code(uin), _ptr(uin), _ptr(uout), nx, uin.stride(0), ny, j0, j1, ylo, yhi,
            _int_array(box), order, cx, cy, dt, _stream_ptr(stream))
        _lib.check(code, "diffusion2d_step")
    else:
        ref.diffusion2d_step_box(uin, uout, nx, j0, j1, ylo, yhi, box, order, cx, cy, dt)


def diffusion2d_stage(inp, u0, out, *, nx, j0, j1, border, order, cx, cy, dt, a, b,
                      stream=None, ls=False):
    _check_layout(inp, u0, out)
    if _native(inp):
        lib = _lib.require()
        R = order // 2
        assert j0 >= R and j1 + R <= inp.shape[0], "stencil rows out of bounds"
        fn = lib.advdiff_diffusion2d_stage_ls if ls else lib.advdiff_diffusion2d_stage
        code = fn(_dtype_code(inp), _ptr(inp), _aux_ptr(u0, a, ls), _ptr(out), nx,
                  inp.stride(0), j0, j1, border, order, cx, cy, dt, a, b, _stream_ptr(stream))
        _lib.check(code, "diffusion2d_stage")
    else:
        ref.diffusion2d_stage(inp, u0, out, nx, j0, j1, border, order, cx, cy, dt, a, b, ls)


def _dt_of(dt, dt_dev):
    """Host value of a device dt (torch/CPU paths only; the HIP kernels read it on device)."""
    if dt_dev is None:
        return dt, False
    d = float(dt_dev.reshape(-1)[0])
    return d, d == 0.0


def burgers3d_stage(inp, u0, out, *, nx, ny, k0, k1, border, weno_z, rdx, rdy, rdz,
                    vx=0.0, vy=0.0, vz=0.0, dt, a, b, stream=None, ls=False, dt_dev=None,
                    k0b=0, k1b=0, put=None):
    """weno_z: scheme — bool (WENO5 Z / JS) or "js" | "z" | "js7" (WENO7).
    dt_dev: float64 device scalar holding dt (adaptive CFL: written on the device by
    adaptive_dt, read by the kernel — no host sync); 0 there makes the stage out = in.
    [k0b, k1b): an optional second plane range (a slab rank's other boundary slab),
    served by the same launch (advdiff_burgers3d_stage2_dt).
    put = ((dst_lo, lo_k0, lo_k1), (dst_hi, hi_k0, hi_k1)): fused halo puts of a slab rank
    (advdiff_burgers3d_stage_put: native fp64 fields, WENO5, SSP-RK3, one range)."""
    _check_layout(inp, u0, out)
    code_s, R = ref.scheme_code(weno_z), ref.scheme_radius(weno_z)
    if border < R:
        raise ValueError(f"WENO needs a frozen border of at least {R} cells")
    if put is not None:
        if (not _native(inp) or inp.dtype != torch.float64 or code_s not in (0, 1) or ls
                or k1b > k0b):
            raise ValueError("fused halo puts: native fp64 WENO5 SSP-RK3 stages, one range")
        lib = _lib.require()
        assert k0 >= R and k1 + R <= inp.shape[0], "stencil planes out of bounds"
        (dlo, lo0, lo1), (dhi, hi0, hi1) = put
        code = lib.advdiff_burgers3d_stage_put(
            _dtype_code(inp), _ptr(inp), _aux_ptr(u0, a, ls), _ptr(out), nx, ny,
            inp.stride(1), inp.stride(0), k0, k1, border, code_s, rdx, rdy, rdz, vx, vy, vz,
            dt, a, b, None if dt_dev is None else dt_dev.data_ptr(), dlo or None, lo0, lo1,
            dhi or None, hi0, hi1, _stream_ptr(stream))
        _lib.check(code, "burgers3d_stage_put")
        return
    ranges = [(lo, hi) for lo, hi in ((k0, k1), (k0b, k1b)) if hi > lo]
    if _native(inp):
        lib = _lib.require()
        for lo, hi in ranges:
            assert lo >= R and hi + R <= inp.shape[0], "stencil planes out of bounds"
        code = lib.advdiff_burgers3d_stage2_dt(
            _dtype_code(inp), _ptr(inp), _aux_ptr(u0, a, ls), _ptr(out), nx, ny,
            inp.stride(1), inp.stride(0), k0, k1, k0b, k1b, border, code_s, rdx, rdy, rdz, vx,
            vy, vz, dt, a, b, 1 if ls else 0, None if dt_dev is None else dt_dev.data_ptr(),
            _stream_ptr(stream))
        _lib.check(code, "burgers3d_stage")
    else:
        dt, noop = _dt_of(dt, dt_dev)
        for lo, hi in ranges:
            if noop:
                sl = (slice(lo, hi), slice(border, ny - border), slice(border, nx - border))
                out[sl] = inp[sl]
            else:
                ref.burgers3d_stage(inp, u0, out, nx, ny, lo, hi, border, code_s, rdx, rdy,
                                    rdz, vx, vy, vz, dt, a, b, ls)


def burgers2d_stage(inp, u0, out, *, nx, j0, j1, border, weno_z, rdx, rdy, vx=0.0, vy=0.0,
                    dt, a, b, stream=None, ls=False, dt_dev=None):
    _check_layout(inp, u0, out)
    code_s, R = ref.scheme_code(weno_z), ref.scheme_radius(weno_z)
    if border < R:
        raise ValueError(f"WENO needs a frozen border of at least {R} cells")
    if _native(inp):
        lib = _lib.require()
        assert j0 >= R and j1 + R <= inp.shape[0], "stencil rows out of bounds"
        code = lib.advdiff_burgers2d_stage_dt(
            _dtype_code(inp), _ptr(inp), _aux_ptr(u0, a, ls), _ptr(out), nx, inp.stride(0),
            j0, j1, border, code_s, rdx, rdy, vx, vy, dt, a, b, 1 if ls else 0,
            None if dt_dev is None else dt_dev.data_ptr(), _stream_ptr(stream))
        _lib.check(code, "burgers2d_stage")
    else:
        dt, noop = _dt_of(dt, dt_dev)
        if noop:
            if j1 > j0:
                out[j0:j1, border:nx - border] = inp[j0:j1, border:nx - border]
            return
        ref.burgers2d_stage(inp, u0, out, nx, j0, j1, border, code_s, rdx, rdy, vx, vy,
                            dt, a, b, ls)


def adaptive_dt(red, state, *, cfl_h, dt_visc, t_end=None, stream=None):
    """Device-side adaptive CFL step (see kernels.h advdiff_adaptive_dt): red = the norm
    reducer's result tensor (max|u| at [2]), state = float64[3] device tensor [t, dt,
    steps], updated in place."""
    if state.is_cuda:
        lib = _lib.require()
        code = lib.advdiff_adaptive_dt(red.data_ptr(), state.data_ptr(), cfl_h, dt_visc,
                                       0.0 if t_end is None else t_end,
                                       0 if t_end is None else 1, _stream_ptr(stream))
        _lib.check(code, "adaptive_dt")
        return
    t = float(state[0])
    dt = 0.0
    if not (t_end is not None and t >= t_end * (1 - 1e-14)):
        u = max(float(red[2]), 1e-300)
        dt = cfl_h / u
        if dt_visc > 0.0 and dt_visc < dt:
            dt = dt_visc
        if t_end is not None and t + dt > t_end:
            dt = t_end - t
    state[1] = dt
    if dt != 0.0:
        state[0] = t + dt
        state[2] = float(state[2]) + 1.0


class NormReducer:
    """Σ|x-y|, Σ(x-y)², max|x-y| over a box, on device (two-pass deterministic tree)."""

    def __init__(self, device):
        self.device = torch.device(device)
        if self.device.type == "cuda":
            lib = _lib.require()
            nbytes = lib.advdiff_reduce_workspace_bytes()
            self.ws = torch.empty(nbytes, dtype=torch.uint8, device=self.device)
            self.res = torch.empty(3, dtype=torch.float64, device=self.device)

    def __call__(self, x, y=None, box=None, stream=None, sync=True):
        """box = ((i0,i1),(j0,j1),(k0,k1)) in array coordinates (3-D) or
        ((i0,i1),(j0,j1)) (2-D).  Returns a float64 tensor [3] (device) or tuple."""
        if x.dim() == 2:
            xs = x.unsqueeze(0)
            ys = None if y is None else y.unsqueeze(0)
            if box is None:
                box = ((0, x.shape[1]), (0, x.shape[0]))
            box = (box[0], box[1], (0, 1))
        else:
            xs, ys = x, y
            if box is None:
                box = ((0, x.shape[2]), (0, x.shape[1]), (0, x.shape[0]))
        (i0, i1), (j0, j1), (k0, k1) = box
        if not x.is_cuda:
            sub = xs[k0:k1, j0:j1, i0:i1]
            suby = None if ys is None else ys[k0:k1, j0:j1, i0:i1]
            r = ref.norms(sub, suby)
            return torch.tensor(r, dtype=torch.float64) if not sync else r
        lib = _lib.require()
        code = lib.advdiff_reduce_norms(
            _dtype_code(x), xs.data_ptr(), None if ys is None else ys.data_ptr(),
            xs.stride(1), xs.stride(0), i0, i1, j0, j1, k0, k1, self.ws.data_ptr(),
            self.res.data_ptr(), _stream_ptr(stream))
        _lib.check(code, "reduce_norms")
        if sync:
            return tuple(float(v) for v in self.res.cpu())
        return self.res


def copy_box(dst, src, ni, nj, nk, stream=None):
    """Strided 3-D box copy dst[k, j, i] = src[k, j, i] (halo pack/unpack)."""
    if dst.is_cuda:
        lib = _lib.require()
        d3 = dst if dst.dim() == 3 else dst.unsqueeze(0)
        s3 = src if src.dim() == 3 else src.unsqueeze(0)
        code = lib.advdiff_copy_box(_dtype_code(dst), d3.data_ptr(), d3.stride(1),
                                    d3.stride(0), s3.data_ptr(), s3.stride(1), s3.stride(0),
                                    ni, nj, nk, _stream_ptr(stream))
        _lib.check(code, "copy_box")
    else:
        if dst.dim() == 3:
            dst[:nk, :nj, :ni].copy_(src[:nk, :nj, :ni])
        else:
            dst[:nj, :ni].copy_(src[:nj, :ni])


def init_ic_device(u, ic_code, *, nx, ny, nzl, kg0, NX, NY, NZ, dx, dy, dz, p0=0.0, p1=0.0,
                   stream=None):
    """Fill a local slab with a built-in IC on the device (see kernels.h codes)."""
    lib = _lib.require()
    u3 = u if u.dim() == 3 else u.unsqueeze(0)
    code = lib.advdiff_init_ic(_dtype_code(u), ic_code, u3.data_ptr(), nx, ny, nzl,
                               u3.stride(1), u3.stride(0), kg0, NX, NY, NZ, dx, dy, dz, p0,
                               p1, _stream_ptr(stream))
    _lib.check(code, "init_ic")


def init_ic_box_device(u, ic_code, *, nx, ny, nzl, ig0, jg0, kg0, NX, NY, NZ, dx, dy, dz,
                       p0=0.0, p1=0.0, stream=None):
    """Fill a local box of a Cartesian decomposition: local (i, j, k) is global
    (ig0+i, jg0+j, kg0+k); 2-D arrays use (i, j) with nzl = 1 and NZ = 1."""
    lib = _lib.require()
    u3 = u if u.dim() == 3 else u.unsqueeze(0)
    code = lib.advdiff_init_ic_box(_dtype_code(u), ic_code, u3.data_ptr(), nx, ny, nzl,
                                   u3.stride(1), u3.stride(0), ig0, jg0, kg0, NX, NY, NZ, dx,
                                   dy, dz, p0, p1, _stream_ptr(stream))
    _lib.check(code, "init_ic_box")


def debug_print(u, box, stream=None):
    """Device-side printf of a small box ((i0,i1),(j0,j1),(k0,k1)) of a 3-D (or 2-D) field —
    the reference's PrintGPUmemory.  CPU tensors are printed from the host."""
    (i0, i1), (j0, j1), (k0, k1) = box if len(box) == 3 else (box[0], box[1], (0, 1))
    u3 = u if u.dim() == 3 else u.unsqueeze(0)
    if not u.is_cuda:
        for k in range(k0, k1):
            print(f"[k={k}]")
            for j in range(j0, j1):
                print(" ".join(f"{float(v):8.4f}" for v in u3[k, j, i0:i1]))
        return
    lib = _lib.require()
    code = lib.advdiff_debug_print(_dtype_code(u), u3.data_ptr(), u3.stride(1), u3.stride(0),
                                   i0, i1, j0, j1, k0, k1, _stream_ptr(stream))
    _lib.check(code, "debug_print")
