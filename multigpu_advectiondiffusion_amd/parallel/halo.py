"""Halo (ghost-plane) exchange for slab decompositions.

Reference: the host-staged per-stage choreography inline in
`MultiGPU/Diffusion3d_Baseline/main.c:201-302` (pack kernel -> cudaMemcpy2DAsync D2H ->
cudaStreamSynchronize -> MPI_Isend/Irecv -> MPI_Wait -> H2D -> unpack kernel, exchanging
the RHS ``Lu`` of 3 boundary planes, 6 exchanges per step).

Here:
* the payload is the stage INPUT ``u`` itself (G = stencil-radius planes), so ghosts are
  exact copies of the neighbour's owned planes and a P-rank run is bitwise identical to
  a 1-rank run (tests/test_distributed.py);
* planes are contiguous, so RCCL reads/writes the field buffers directly (zero copy,
  no pack/unpack kernels, no host staging);
* all four transfers of a rank go out as ONE grouped RCCL call
  (``batch_isend_irecv`` -> ncclGroupStart/Send/Recv/GroupEnd) on a dedicated comm
  stream, ordered after the producing kernel by a HIP event and joined back into the
  compute stream by ``wait()`` — the host never blocks;
* on CPU/gloo the same code path runs synchronously (tests).
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from .decomposition import SlabDecomposition


class PendingExchange:
    """Handle of an in-flight halo exchange."""

    def __init__(self, works, stream=None, finish=None):
        self.works = works
        self.stream = stream
        self.finish = finish

    def wait(self):
        """Make the CURRENT stream wait for completion (device); block on CPU/gloo."""
        for w in self.works:
            w.wait()
        self.works = []
        if self.finish is not None:
            self.finish()
            self.finish = None


def _joinable(cs) -> PendingExchange:
    """Handle whose wait() joins the comm stream `cs` (at this point) into the current
    stream — nothing to do when the current stream IS `cs` (stream order)."""
    done = torch.cuda.Event()
    done.record(cs)

    def join():
        s = torch.cuda.current_stream()
        if s != cs:
            s.wait_event(done)
    return PendingExchange([], cs, join)


def _order_after(cs, cur, after_event) -> None:
    """Order the comm stream `cs` after the producer of the field: after `after_event`,
    or (None) after everything queued on the current stream `cur` so far.  False: the
    producer ran on `cs` itself (the boundary launch on the comm stream), so stream order
    already holds — no event, and no same-stream event wait inside a graph capture
    (hipStreamEndCapture crashed on those, profiles/r5/diag_bstream.md)."""
    if after_event is False or (after_event is None and cs == cur):
        return
    if after_event is None:
        after_event = torch.cuda.Event()
        after_event.record(cur)
    cs.wait_event(after_event)


def _start_ipc_routed(comm, comm_stream, phases, after_event=None, tag=None,
                      puts=None) -> PendingExchange:
    """Like _start_ipc for phases of one-way-capable routes: phases = [(channel, {peer:
    (send_view | None, recv_view | None)})], run in order on the comm stream; `tag`
    keys the handshake cache (IpcPeers._resolve_pairs); puts: per phase, whether its
    sends are put here (False: the producing kernel stored them — fused puts)."""
    cur = torch.cuda.current_stream()
    cs = comm_stream or cur
    _order_after(cs, cur, after_event)
    ipc = comm.ipc()
    for q, (ch, pairs) in enumerate(phases):
        ipc.route(pairs, cs, ch, tag, puts=True if puts is None else puts[q])
    return _joinable(cs)


def _start_ipc(comm, comm_stream, phases, after_event=None, puts=True) -> PendingExchange:
    """Device puts into the peers' ghost cells (parallel/ipc.py) on the comm stream after
    `after_event`, phases in order; the returned handle joins the current stream.
    puts=False: the producing kernel stored the boxes itself — signal and wait only."""
    cur = torch.cuda.current_stream()
    cs = comm_stream or cur
    _order_after(cs, cur, after_event)
    ipc = comm.ipc()
    for msgs in phases:
        ipc.exchange(msgs, cs, puts=puts)
    return _joinable(cs)


def _ipc_on(halo, field) -> bool:
    return field.is_cuda and halo.comm.size > 1 and halo.transport == "ipc"


class SlabHalo:
    def __init__(self, comm, decomp: SlabDecomposition, comm_stream=None,
                 transport: str | None = None, stripe: int = 0):
        """transport: "ipc", "rccl" or "host" (None: the Comm's default, Comm.transport).
        stripe (ipc, 3-D fields): up to this many relay helpers per face message — part
        of every message goes source -> helper -> destination over the node's otherwise
        idle xGMI links (parallel/ipc.py stripe_plan; 8 ranks: 1 helper each, the face
        then crosses the busiest link as 2/3 of its bytes).  0: direct messages only."""
        self.comm = comm
        self.d = decomp
        self.comm_stream = comm_stream
        self.transport = transport or (comm.transport if comm is not None else None)
        self.parity = 0  # striped: which of the two relay buffer sets the next exchange uses
        self._plan = None
        self._fwd = {}
        self._fid = {}  # field address -> ordinal (the same on every rank: same call order)
        if stripe and self.transport == "ipc" and comm is not None and comm.size > 1:
            import os
            from .ipc import stripe_plan
            # ADVDIFF_STRIPE_SHARED=1 (tests): helpers may share links, so the relay
            # mechanism runs on fewer ranks than the 7-8 that have idle links for it
            plan = stripe_plan(comm.size, stripe,
                               exclusive_links=os.environ.get("ADVDIFF_STRIPE_SHARED") != "1")
            if any(plan.values()):
                self._plan = plan
        # striped handshake tags carry the ipc epoch this halo was made in (every Solver on
        # ipc resets the peers at construction, collectively): two striped solvers alive
        # at once (bench.py tunes ipc+stripe and ipc+fused+stripe side by side) must not
        # share a (field ordinal, parity) tag in the peers' address cache
        ipc = getattr(comm, "ipc", None) if self._plan is not None else None
        self._hid = getattr(ipc(), "epoch", 0) if ipc is not None else 0

    @property
    def striped(self) -> bool:
        return self._plan is not None

    def _fwd_buf(self, key, like, shape):
        b = self._fwd.get(key)
        if b is None or tuple(b.shape) != tuple(shape) or b.dtype != like.dtype:
            # no fill: an (asynchronous) fill kernel could land after a peer's first put
            b = torch.empty(shape, dtype=like.dtype, device=like.device)
            self._fwd[key] = b
        return b

    def _stripe_phases(self, field, parity):
        """The two phases of a striped exchange for this rank: channel 1 = the direct
        parts to / from the neighbours and the relayed parts into the helpers' buffers,
        channel 2 = the helpers' forwards into the destinations' ghost rows.  Parts are
        row ranges of the G ghost planes (parallel/ipc.py stripe_rows).  The relay buffers
        alternate between two sets by exchange parity: a source's next put into a set
        comes only after the destination consumed that set's previous forward (it needed
        it for the step whose output the source now sends), so no acknowledgement is
        needed — the same argument as the direct puts'."""
        from .ipc import stripe_rows
        d, me = self.d, self.comm.rank
        p1, p2 = {}, {}

        def add(ph, peer, send=None, recv=None):
            s0, r0 = ph.get(peer, (None, None))
            ph[peer] = (send if send is not None else s0, recv if recv is not None else r0)
        rows = field.shape[1]
        for (src, dst), hs in self._plan.items():
            if me != src and me != dst and me not in hs:
                continue
            parts = stripe_rows(rows, 1 + len(hs))
            up = dst == src + 1  # the message goes to the upper neighbour
            if me == src:
                s0, s1 = d.send_upper() if up else d.send_lower()
                (a, b) = parts[0]
                add(p1, dst, send=field[s0:s1, a:b])
                for h, (a, b) in zip(hs, parts[1:]):
                    add(p1, h, send=field[s0:s1, a:b])
            if me == dst:
                r0, r1 = d.recv_lower() if up else d.recv_upper()
                (a, b) = parts[0]
                add(p1, src, recv=field[r0:r1, a:b])
                for h, (a, b) in zip(hs, parts[1:]):
                    add(p2, h, recv=field[r0:r1, a:b])
            if me in hs:
                (a, b) = parts[1 + hs.index(me)]
                buf = self._fwd_buf((src, dst, parity), field,
                                    (d.ghost, b - a, field.shape[2]))
                add(p1, src, recv=buf)
                add(p2, dst, send=buf)
        return p1, p2

    def _use_stripes(self, field) -> bool:
        return self._plan is not None and field.is_cuda and field.dim() == 3

    def _tag(self, field, parity):
        """Handshake key of a striped exchange that every rank derives alike: the field's
        ordinal (fields reach the halo in the same order on every rank) and the parity."""
        return (self._hid, self._fid.setdefault(field.data_ptr(), len(self._fid)), parity)

    def _ops(self, field: torch.Tensor):
        d = self.d
        ops = []
        if d.lower is not None:
            s0, s1 = d.send_lower()
            r0, r1 = d.recv_lower()
            ops.append(dist.P2POp(dist.irecv, field[r0:r1], d.lower))
            ops.append(dist.P2POp(dist.isend, field[s0:s1], d.lower))
        if d.upper is not None:
            s0, s1 = d.send_upper()
            r0, r1 = d.recv_upper()
            ops.append(dist.P2POp(dist.isend, field[s0:s1], d.upper))
            ops.append(dist.P2POp(dist.irecv, field[r0:r1], d.upper))
        return ops

    def _start_host_staged(self, field: torch.Tensor, after_event=None) -> PendingExchange:
        """Device tensors over a CPU-only backend (gloo): stage the G-plane slabs through
        pinned host buffers on the comm stream — the reference's scheme
        (`MultiGPU/Diffusion3d_Baseline/main.c:209-288`).  Used to run multi-process
        tests on ONE GPU (RCCL refuses two ranks per device) and as a fallback transport;
        the production path is RCCL (zero copy)."""
        d = self.d
        cur = torch.cuda.current_stream()
        cs = self.comm_stream or cur
        _order_after(cs, cur, after_event)
        sends, recvs, ops = [], [], []
        with torch.cuda.stream(cs):
            for peer, (s0, s1), (r0, r1) in ((d.lower, d.send_lower(), d.recv_lower()),
                                              (d.upper, d.send_upper(), d.recv_upper())):
                if peer is None:
                    continue
                hs = torch.empty(field[s0:s1].shape, dtype=field.dtype, pin_memory=True)
                hs.copy_(field[s0:s1], non_blocking=True)
                hr = torch.empty_like(hs, pin_memory=True)
                sends.append((peer, hs))
                recvs.append((peer, hr, (r0, r1)))
        cs.synchronize()  # host buffers filled before gloo reads them
        for peer, hs in sends:
            ops.append(dist.P2POp(dist.isend, hs, peer))
        for peer, hr, _ in recvs:
            ops.append(dist.P2POp(dist.irecv, hr, peer))
        works = dist.batch_isend_irecv(ops)

        def finish():
            with torch.cuda.stream(cs):
                for _, hr, (r0, r1) in recvs:
                    field[r0:r1].copy_(hr, non_blocking=True)
                done = torch.cuda.Event()
                done.record(cs)
            if torch.cuda.current_stream() != cs:
                torch.cuda.current_stream().wait_event(done)
            # keep the pinned buffers alive until the copies have run
            cs.synchronize()

        return PendingExchange(works, cs, finish)

    def _ipc_msgs(self, field):
        d = self.d
        msgs = []
        for peer, s, r in ((d.lower, d.send_lower(), d.recv_lower()),
                           (d.upper, d.send_upper(), d.recv_upper())):
            if peer is not None:
                msgs.append((peer, field[s[0]:s[1]], field[r[0]:r[1]]))
        return msgs

    def prepare(self, field: torch.Tensor) -> None:
        """Collective, outside any graph capture: learn the peers' receive addresses of
        this field's exchange (ipc transport; a no-op otherwise) — for both relay buffer
        sets when striped (a graph replays exchanges of both parities)."""
        if _ipc_on(self, field) and self._use_stripes(field):
            ipc = self.comm.ipc()
            for par in (0, 1):
                p1, p2 = self._stripe_phases(field, par)
                ipc._resolve_pairs(1, p1, self._tag(field, par))
                ipc._resolve_pairs(2, p2, self._tag(field, par))
        elif _ipc_on(self, field):
            self.comm.ipc()._resolve(self._ipc_msgs(field))

    def put_parts(self, field: torch.Tensor) -> list:
        """Fused halo puts of a striped exchange (ipc, 3-D; the next exchange's relay set,
        self.parity): [(dst, k0, k1, y0, y1, plane_bytes)] — every channel-1 send box of
        `field` (planes [k0, k1), rows [y0, y1): the direct part to a neighbour's ghost rows
        and the relayed parts to the helpers' row buffers) with dst offset so that row y of
        plane k lands at dst + (k - k0) plane_bytes + the own in-plane offset (each receive
        box has this field's row pitch).  start(field, puts=False) then runs channel 1
        without its puts and the helpers' forwards (channel 2) as usual."""
        if not (_ipc_on(self, field) and self._use_stripes(field)):
            raise ValueError("put_parts: the striped ipc exchange of a 3-D slab")
        par = self.parity
        p1, _ = self._stripe_phases(field, par)
        dests = self.comm.ipc()._resolve_pairs(1, p1, self._tag(field, par))
        e = field.element_size()
        out = []
        for peer, (send, _) in sorted(p1.items()):
            if send is None:
                continue
            ptr, rsy, rsz = dests[peer]
            if rsy != field.stride(1):
                raise ValueError(f"fused halo puts: peer {peer} row pitch {rsy} != "
                                 f"{field.stride(1)}")
            off = send.storage_offset() - field.storage_offset()
            k0, a = off // field.stride(0), (off % field.stride(0)) // field.stride(1)
            out.append((ptr - a * rsy * e, k0, k0 + send.shape[0], a, a + send.shape[1],
                        rsz * e))
        return out

    def put_targets(self, field: torch.Tensor):
        """Fused halo puts (ipc, direct, 3-D): ((dst_lo, k0, k1), (dst_hi, k0, k1)) — the
        peer address of my send planes [k0, k1) of `field` towards the lower / upper
        neighbour (dst 0: no neighbour), for a step kernel that stores its output planes
        there itself (stencil.diffusion3d_step put=).  The peers' receive boxes must have
        this field's strides (slab ranks of one grid); start(field, puts=False) then only
        signals and waits.  Striped exchanges: put_parts."""
        if not _ipc_on(self, field) or self._use_stripes(field) or field.dim() != 3:
            raise ValueError("fused halo puts: the direct ipc transport of a 3-D slab")
        msgs = self._ipc_msgs(field)
        dests = self.comm.ipc().targets(msgs)
        d = self.d
        out = [(0, 0, 0), (0, 0, 0)]
        for (peer, send, _), (ptr, rsy, rsz) in zip(msgs, dests):
            if (rsy, rsz) != (field.stride(1), field.stride(0)):
                raise ValueError(f"fused halo puts: peer {peer} field strides {(rsy, rsz)} "
                                 f"!= {(field.stride(1), field.stride(0))}")
            s0, s1 = d.send_lower() if peer == d.lower else d.send_upper()
            out[0 if peer == d.lower else 1] = (ptr, s0, s1)
        return tuple(out)

    def start(self, field: torch.Tensor, after_event=None,
              puts: bool = True) -> PendingExchange | None:
        """Begin exchanging the ghost planes of `field` (axis 0).

        On device: the transfers are issued on the comm stream after `after_event`
        (None: after all work currently queued on the current stream; False: the field's
        producer ran on the comm stream itself).  puts=False (ipc, direct): the producer
        already stored the send planes into the peers (put_targets) — signal and wait."""
        if self.comm.size == 1:
            return None
        if not puts:
            if not _ipc_on(self, field):
                raise ValueError("puts=False: the ipc transport only")
            if self._use_stripes(field):  # channel 1 stored by the kernel, forwards as usual
                par = self.parity
                p1, p2 = self._stripe_phases(field, par)
                self.parity ^= 1
                return _start_ipc_routed(self.comm, self.comm_stream, [(1, p1), (2, p2)],
                                         after_event, tag=self._tag(field, par),
                                         puts=(False, True))
            return _start_ipc(self.comm, self.comm_stream, [self._ipc_msgs(field)],
                              after_event, puts=False)
        if _ipc_on(self, field) and self._use_stripes(field):
            par = self.parity
            p1, p2 = self._stripe_phases(field, par)
            self.parity ^= 1
            return _start_ipc_routed(self.comm, self.comm_stream, [(1, p1), (2, p2)],
                                     after_event, tag=self._tag(field, par))
        if _ipc_on(self, field):
            return _start_ipc(self.comm, self.comm_stream, [self._ipc_msgs(field)], after_event)
        ops = self._ops(field)
        if not ops:
            return None
        if field.is_cuda and self.comm.backend != "nccl":
            return self._start_host_staged(field, after_event)
        if field.is_cuda and self.comm_stream is not None:
            _order_after(self.comm_stream, torch.cuda.current_stream(), after_event)
            with torch.cuda.stream(self.comm_stream):
                works = dist.batch_isend_irecv(ops)
            return PendingExchange(works, self.comm_stream)
        works = dist.batch_isend_irecv(ops)
        return PendingExchange(works)

    def exchange(self, field: torch.Tensor) -> None:
        """Blocking (stream-ordered) exchange."""
        p = self.start(field)
        if p is not None:
            p.wait()


class CartesianHalo:
    """Ghost exchange for a 2-D/3-D process grid (``CartesianDecomposition``).

    faces (default, star stencils applied once per exchange): per split axis and side one
    message of G layers over the owned extent of the other axes; all messages of a rank
    form ONE grouped RCCL call.
    corners=True (the fused full-step kernel: three stacked star stencils reach diagonal
    neighbours), two ways to fill the edge and corner ghosts:
      direct (default, ADVDIFF_CORNERS=direct): ONE phase with a message to every
        neighbour in the 3^d - 1 offsets of the process grid — faces to the face
        neighbours, edges and corners straight from the diagonal neighbours.  An 8-GPU
        MI355X node is fully connected by xGMI (7 links per GPU), so a diagonal neighbour
        is one hop away and every message of the phase has a link of its own: a 2x2x2
        grid uses all 7 links at once, and no phase waits for another;
      phased (ADVDIFF_CORNERS=phased): axis by axis, fastest first (x, then y, then z);
        each phase's message spans the FULL allocated extent of the axes already
        exchanged, so edge and corner ghosts arrive with the faces — three dependent
        phases, ordered on the comm stream (no host blocking).
    Both fill every ghost cell with the owner's value: bitwise the same results.
    Axis-0 messages with full x/y extent are whole planes (contiguous, zero-copy); other
    messages are strided and go through pack/unpack with the native ``advdiff_copy_box``
    kernel on the comm stream.  Reference: none (the reference only splits z, §2.5).
    """

    def __init__(self, comm, decomp, comm_stream=None, corners: bool = False,
                 direct: bool | None = None, transport: str | None = None):
        import os
        self.comm = comm
        self.transport = transport or (comm.transport if comm is not None else None)
        self.cd = decomp
        self.comm_stream = comm_stream
        self.corners = corners
        if direct is None:
            direct = os.environ.get("ADVDIFF_CORNERS", "direct") != "phased"
        self.direct = bool(corners and direct)
        self._bufs = {}

    def _phases(self):
        """Axis groups exchanged together: all at once (faces), fastest axis first
        (phased corners), or None = one phase over every neighbour offset (direct)."""
        split = [a for a in range(self.cd.dims) if self.cd.pgrid[a] > 1]
        if not split:
            return []
        if self.direct:
            return [None]
        return [sorted(split, reverse=True)] if not self.corners else \
            [[a] for a in sorted(split, reverse=True)]

    def _offsets(self):
        """Neighbour offsets of the direct exchange (fastest axis varying fastest, as the
        native halo_plan): every d in {-1,0,1}^dims, d != 0, zero on unsplit axes."""
        import itertools
        cd = self.cd
        rng = [(-1, 0, 1) if cd.pgrid[a] > 1 else (0,) for a in range(cd.dims)]
        return [d for d in itertools.product(*rng) if any(d)]

    def boxes(self, axes):
        """[(peer, send_box, recv_box, offset)] of one phase as local index ranges
        ((lo, hi) per array axis; offset = the neighbour's coordinate offset) — the
        geometry the native runtime must reproduce (csrc/runtime/cart.cpp halo_plan,
        tests/test_native_host.py)."""
        cd = self.cd
        own = cd.owned_box()
        out = []
        if axes is None:  # direct: one message per neighbour offset
            G = cd.ghost
            coords = cd.coords
            for d in self._offsets():
                c = [x + dx for x, dx in zip(coords, d)]
                if not all(0 <= c[a] < cd.pgrid[a] for a in range(cd.dims)):
                    continue
                sb, rb = [], []
                for a, (lo, hi) in enumerate(own):
                    if d[a] < 0:
                        sb.append((lo, lo + G))
                        rb.append((0, G))
                    elif d[a] > 0:
                        sb.append((hi - G, hi))
                        rb.append((hi, hi + G))
                    else:
                        sb.append((lo, hi))
                        rb.append((lo, hi))
                out.append((cd.rank_of(c), tuple(sb), tuple(rb), tuple(d)))
            return out
        for a in axes:
            ax = cd.axis(a)
            for side, peer in ((-1, cd.neighbor(a, -1)), (1, cd.neighbor(a, 1))):
                if peer is None:
                    continue
                s = ax.send_lower() if side < 0 else ax.send_upper()
                r = ax.recv_lower() if side < 0 else ax.recv_upper()
                sb = []
                for b, (lo, hi) in enumerate(own):
                    if self.corners and b > a:  # already exchanged: carry its ghosts
                        sb.append((0, cd.axis(b).alloc))
                    else:
                        sb.append((lo, hi))
                rb = list(sb)
                sb[a] = tuple(s)
                rb[a] = tuple(r)
                off = tuple(side if b == a else 0 for b in range(cd.dims))
                out.append((peer, tuple(sb), tuple(rb), off))
        return out

    def _regions(self, field, axes):
        """[(peer, send_view, recv_view, key)] for the given axes, fixed order."""
        out = []
        for peer, sb, rb, key in self.boxes(axes):
            sv = field[tuple(slice(lo, hi) for lo, hi in sb)]
            rv = field[tuple(slice(lo, hi) for lo, hi in rb)]
            out.append((peer, sv, rv, key))
        return out

    def _buf(self, key, like):
        b = self._bufs.get(key)
        if b is None or b.shape != like.shape or b.dtype != like.dtype or b.device != like.device:
            b = torch.empty(like.shape, dtype=like.dtype, device=like.device)
            self._bufs[key] = b
        return b

    @staticmethod
    def _copy(dst, src):
        if dst.is_cuda:
            from ..ops import stencil
            d3 = dst if dst.dim() == 3 else dst.unsqueeze(0)
            s3 = src if src.dim() == 3 else src.unsqueeze(0)
            stencil.copy_box(d3, s3, d3.shape[2], d3.shape[1], d3.shape[0])
        else:
            dst.copy_(src)

    def _plan(self, field, axes):
        """Contiguous send/recv tensors + the unpack list of one phase."""
        sends, recvs, unpack = [], [], []
        for peer, sv, rv, key in self._regions(field, axes):
            if sv.is_contiguous():
                st = sv
            else:
                st = self._buf(("s",) + key, sv)
                self._copy(st, sv)
            if rv.is_contiguous():
                rt = rv
            else:
                rt = self._buf(("r",) + key, rv)
                unpack.append((rv, rt))
            sends.append((peer, st))
            recvs.append((peer, rt))
        return sends, recvs, unpack

    @staticmethod
    def _ops(sends, recvs):
        ops = [dist.P2POp(dist.isend, t, p) for p, t in sends]
        ops += [dist.P2POp(dist.irecv, t, p) for p, t in recvs]
        return ops

    def _ipc_phases(self, field):
        return [[(p, sv, rv) for p, sv, rv, _ in self._regions(field, axes)]
                for axes in self._phases()]

    def prepare(self, field: torch.Tensor) -> None:
        """Collective, outside any graph capture: learn the peers' receive addresses of
        this field's exchange (ipc transport; a no-op otherwise)."""
        if _ipc_on(self, field):
            ipc = self.comm.ipc()
            for msgs in self._ipc_phases(field):
                ipc._resolve(msgs)

    def start(self, field: torch.Tensor, after_event=None) -> PendingExchange | None:
        if self.comm.size == 1:
            return None
        if _ipc_on(self, field):
            return _start_ipc(self.comm, self.comm_stream, self._ipc_phases(field), after_event)
        phases = self._phases()
        if not field.is_cuda:  # gloo on the CPU: phases run to completion here
            for axes in phases:
                sends, recvs, unpack = self._plan(field, axes)
                ops = self._ops(sends, recvs)
                for w in (dist.batch_isend_irecv(ops) if ops else []):
                    w.wait()
                for dst, src in unpack:
                    dst.copy_(src)
            return None
        cur = torch.cuda.current_stream()
        cs = self.comm_stream or cur
        _order_after(cs, cur, after_event)
        if self.comm.backend != "nccl":
            # device tensors over gloo (one-GPU multi-process tests): host-staged, blocking
            for axes in phases:
                with torch.cuda.stream(cs):
                    sends, recvs, unpack = self._plan(field, axes)
                    hs = [(p, t.cpu()) for p, t in sends]
                    hr = [(p, torch.empty(t.shape, dtype=t.dtype)) for p, t in recvs]
                ops = self._ops(hs, hr)
                for w in (dist.batch_isend_irecv(ops) if ops else []):
                    w.wait()
                with torch.cuda.stream(cs):
                    for (_, dev), (_, host) in zip(recvs, hr):
                        dev.copy_(host)
                    for dst, src in unpack:
                        self._copy(dst, src)
                cs.synchronize()
            return _joinable(cs)
        with torch.cuda.stream(cs):
            for axes in phases:  # stream-ordered phases: pack -> RCCL -> unpack
                sends, recvs, unpack = self._plan(field, axes)
                ops = self._ops(sends, recvs)
                for w in (dist.batch_isend_irecv(ops) if ops else []):
                    w.wait()  # comm stream waits for RCCL (no host block)
                for dst, src in unpack:
                    self._copy(dst, src)
        return _joinable(cs)

    def exchange(self, field: torch.Tensor) -> None:
        p = self.start(field)
        if p is not None:
            p.wait()
