"""Peer-mapped device transport of one node (the P2PComm of SURVEY.md §7.1).

A rank writes its boundary cells STRAIGHT INTO the neighbour's ghost cells: the neighbour's
field allocation is mapped into this process with ``hipIpcOpenMemHandle`` and a copy
kernel (``advdiff_copy_box``) stores into it — over xGMI between GPUs, through the same
HBM when several ranks share one GPU (the multi-process test setup of a 1-GPU box, where
RCCL refuses two ranks per device).  After its puts the rank raises the neighbour's device
flag with a release store (``advdiff_ipc_signal``) and makes its own comm stream wait for
its flags with an acquire spin (``advdiff_ipc_wait``).  Every step of an exchange is a
kernel on the comm stream: no host synchronisation, no staging buffer, no pack / unpack
kernels, and the exchange can be captured into a hipGraph (counters live on the device).

The only host communication is a one-time handshake per message pattern (the first time a
(peer, send buffer, receive buffer, shape) combination is exchanged, the two ranks swap the
IPC address and strides of their receive boxes over the process group).

Replaces the reference's host-staged choreography (`MultiGPU/Diffusion3d_Baseline/
main.c:209-288`: pack -> D2H -> host-blocking sync -> MPI_Isend/Irecv -> MPI_Wait -> H2D ->
unpack).  Native counterpart: ``csrc/runtime/transport.cpp`` IpcTransport.
"""
from __future__ import annotations

import ctypes
import struct

import torch
import torch.distributed as dist

from ..ops import _lib
from ..ops.stencil import _dtype_code

# IpcAddr (80 B) | rsy, rsz (i64) | ni, nj, nk, dtype (i32) | call (u64) | has_recv, has_send
_ANN = struct.Struct("<80sqqiiiiQii")


def _box_geom(t: torch.Tensor):
    """(ni, nj, nk, sy, sz) of a 1-3-D tensor view with a contiguous last axis."""
    if t.stride(-1) != 1:
        raise ValueError("ipc halo boxes need a contiguous last axis")
    if t.dim() == 3:
        return t.shape[2], t.shape[1], t.shape[0], t.stride(1), t.stride(0)
    if t.dim() == 2:
        return t.shape[1], t.shape[0], 1, t.stride(0), 0
    return t.shape[0], 1, 1, t.shape[0], t.shape[0]


class IpcPeers:
    """One process's IPC context: its flag block mapped by every peer, the peers' flag
    blocks mapped here, and the receive addresses learned per message pattern."""

    def __init__(self, comm):
        self.comm = comm
        self.lib = _lib.require()
        ctx = ctypes.c_void_p()
        _lib.check(self.lib.advdiff_ipc_create(comm.size, comm.rank, ctypes.byref(ctx)),
                   "advdiff_ipc_create")
        self.ctx = ctx
        mine = _lib.IpcAddr()
        _lib.check(self.lib.advdiff_ipc_flags_addr(self.ctx, ctypes.byref(mine)),
                   "advdiff_ipc_flags_addr")
        allf = [None] * comm.size
        dist.all_gather_object(allf, bytes(mine))
        for q in range(comm.size):
            if q != comm.rank:
                a = _lib.IpcAddr.from_buffer_copy(allf[q])
                _lib.check(self.lib.advdiff_ipc_set_peer(self.ctx, q, ctypes.byref(a)),
                           "advdiff_ipc_set_peer")
        comm.barrier()  # every flag block mapped before anyone signals
        self._dest = {}
        self._calls = {}
        self.epoch = 0  # bumped by reset(): graphs captured before it hold stale pointers

    def reset(self) -> None:
        """Collective: forget every learned receive address and peer mapping (the flag
        blocks and their counters stay).  Called when a solver allocates
        its fields: a field freed and reallocated (another solver, the allocator's cache
        emptied) can come back at an address the cache still keys, while the peer's new
        receive box lives elsewhere — puts through the stale entry would miss it."""
        torch.cuda.synchronize(self.comm.device)
        self.comm.barrier()  # nobody has a put in flight into a mapping being closed
        _lib.check(self.lib.advdiff_ipc_reset(self.ctx), "advdiff_ipc_reset")
        self._dest.clear()
        self._calls.clear()
        self.epoch += 1
        self.comm.barrier()

    # ------------------------------------------------------------------------------
    def _swap(self, peers, payloads):
        """Pairwise swap of equal-size byte strings with each peer (handshake only)."""
        dev = self.comm.device if self.comm.backend == "nccl" else torch.device("cpu")
        n = len(payloads[0])
        sends = [torch.frombuffer(bytearray(p), dtype=torch.uint8).to(dev) for p in payloads]
        recvs = [torch.empty(n, dtype=torch.uint8, device=dev) for _ in peers]
        ops = [dist.P2POp(dist.isend, s, p) for s, p in zip(sends, peers)]
        ops += [dist.P2POp(dist.irecv, r, p) for r, p in zip(recvs, peers)]
        for w in dist.batch_isend_irecv(ops):
            w.wait()
        return [bytes(r.cpu().numpy().tobytes()) for r in recvs]

    def _resolve(self, msgs):
        """Peer receive (pointer, sy, sz) of every message of a symmetric exchange
        (channel 0); handshake on first use."""
        pairs = {peer: (send, recv) for peer, send, recv in msgs}
        dests = self._resolve_pairs(0, pairs)
        return [dests[peer] for peer, _, _ in msgs]

    def _resolve_pairs(self, ch, pairs, tag=None):
        """pairs = {peer: (send_view | None, recv_view | None)} of one exchange phase on
        flag channel `ch` (at most one message each way per peer; a phase may be one-way
        for a pair, as the striped exchange's relay hops are).  Returns {peer: (pointer,
        sy, sz) of the peer's receive box for my send, or None}.  First use of a pattern:
        both ranks of the pair swap announcements of their receive boxes.  Both must agree
        on "first use", so the cache key may only hold what both sides know: tag=None (a
        symmetric exchange, both boxes of a pair cut from the same field on each side):
        the own boxes' addresses; otherwise the caller's `tag` (the striped exchange: the
        field's ordinal and the relay-set parity), the own boxes being checked against the
        cached pattern instead (a changed box under a known tag is an error, not a silent
        hang)."""
        out, miss = {}, []
        for peer, (send, recv) in sorted(pairs.items(), key=lambda kv: kv[0]):
            ck = (ch, peer)
            self._calls[ck] = self._calls.get(ck, 0) + 1
            mine = (0 if send is None else send.data_ptr(),
                    () if send is None else tuple(send.shape),
                    0 if recv is None else recv.data_ptr(),
                    () if recv is None else tuple(recv.shape))
            key = (ch, None, peer) + mine if tag is None else (ch, tag, peer)
            if key in self._dest:
                d, was = self._dest[key]
                if was != mine:
                    raise RuntimeError(f"ipc: rank {self.comm.rank}: halo pattern {tag} with "
                                       f"peer {peer} changed its boxes (reset() missing?)")
                out[peer] = d
            else:
                miss.append((peer, key))
        if not miss:
            return out
        anns, peers = [], []
        for peer, _ in miss:
            send, recv = pairs[peer]
            a = _lib.IpcAddr()
            geo = (0, 0, 0, 0, 0, 0)
            if recv is not None:
                _lib.check(self.lib.advdiff_ipc_describe(self.ctx, recv.data_ptr(),
                                                         ctypes.byref(a)), "advdiff_ipc_describe")
                ni, nj, nk, sy, sz = _box_geom(recv)
                geo = (sy, sz, ni, nj, nk, _dtype_code(recv))
            anns.append(_ANN.pack(bytes(a), geo[0], geo[1], geo[2], geo[3], geo[4], geo[5],
                                  self._calls[(ch, peer)], int(recv is not None),
                                  int(send is not None)))
            peers.append(peer)
        theirs = self._swap(peers, anns)
        for (peer, key), raw in zip(miss, theirs):
            send, recv = pairs[peer]
            addr, rsy, rsz, ni, nj, nk, dt, call, has_recv, has_send = _ANN.unpack(raw)
            bad = call != self._calls[(ch, peer)] or bool(has_recv) != (send is not None) \
                or bool(has_send) != (recv is not None)
            if send is not None and not bad:
                gi, gj, gk, _, _ = _box_geom(send)
                bad = (ni, nj, nk, dt) != (gi, gj, gk, _dtype_code(send))
            if bad:
                raise RuntimeError(
                    f"ipc: rank {self.comm.rank} and peer {peer} disagree on a halo message "
                    f"(channel {ch}: calls {self._calls[(ch, peer)]} vs {call}, mine send/recv "
                    f"{send is not None}/{recv is not None}, theirs {bool(has_send)}/"
                    f"{bool(has_recv)}, box {(ni, nj, nk, dt)})")
            d = None
            if send is not None:
                a = _lib.IpcAddr.from_buffer_copy(addr)
                ptr = ctypes.c_void_p()
                _lib.check(self.lib.advdiff_ipc_map(self.ctx, ctypes.byref(a),
                                                    ctypes.byref(ptr)), "advdiff_ipc_map")
                d = (ptr.value, rsy, rsz)
            send, recv = pairs[peer]
            self._dest[key] = (d, (0 if send is None else send.data_ptr(),
                                   () if send is None else tuple(send.shape),
                                   0 if recv is None else recv.data_ptr(),
                                   () if recv is None else tuple(recv.shape)))
            out[peer] = d
        return out

    def exchange(self, msgs, stream, puts: bool = True) -> None:
        """Enqueue on `stream`: put every send box into its peer's matching receive box,
        signal the peers, wait for their puts into ours.  msgs = [(peer, send_view,
        recv_view)] with distinct peers.  puts=False: the boxes were already stored by a
        kernel earlier on `stream` (the fused step's halo puts, targets()): signal + wait."""
        if not msgs:
            return
        peers = [m[0] for m in msgs]
        if len(set(peers)) != len(peers):
            raise ValueError("ipc: one message per peer and exchange")
        self.route({peer: (send, recv) for peer, send, recv in msgs}, stream, 0, puts=puts)

    def targets(self, msgs) -> list:
        """Peer receive (pointer, sy, sz) of every message of a symmetric exchange — for a
        kernel that stores the send boxes itself (then exchange(..., puts=False)).  The
        same handshake and cache as exchange()."""
        return self._resolve(msgs)

    def route(self, pairs, stream, ch: int, tag=None, puts: bool = True) -> None:
        """One exchange phase on flag channel `ch`: pairs = {peer: (send_view | None,
        recv_view | None)}.  Enqueues the puts of every send box into the peer's receive
        box, the signal of the peers I sent to, and the wait for the peers that send to
        me (channel ch counts only this phase kind, so a pair that meets in several
        phases of one exchange never mixes its counts)."""
        if not pairs:
            return
        dests = self._resolve_pairs(ch, pairs, tag)
        sp = stream.cuda_stream
        to = sorted(p for p, (snd, _) in pairs.items() if snd is not None)
        frm = sorted(p for p, (_, rcv) in pairs.items() if rcv is not None)
        for peer in (to if puts else ()):
            send = pairs[peer][0]
            dptr, dsy, dsz = dests[peer]
            ni, nj, nk, ssy, ssz = _box_geom(send)
            _lib.check(self.lib.advdiff_ipc_put(_dtype_code(send), dptr, dsy, dsz,
                                                send.data_ptr(), ssy, ssz, ni, nj, nk, sp),
                       "ipc put")
        if to:
            arr = (ctypes.c_int * len(to))(*to)
            _lib.check(self.lib.advdiff_ipc_signal_ch(self.ctx, ch, arr, len(to), sp),
                       "advdiff_ipc_signal")
        if frm:
            arr = (ctypes.c_int * len(frm))(*frm)
            _lib.check(self.lib.advdiff_ipc_wait_ch(self.ctx, ch, arr, len(frm), sp),
                       "advdiff_ipc_wait")

    def preflight(self, rounds: int = 3, box=(3, 24, 200)) -> dict:
        """Collective validation of the transport between EVERY pair of ranks, before a
        run relies on it (the first multi-GPU run must not trust an unexercised path):

        * ranks on different GPUs: ``hipDeviceCanAccessPeer`` for each pair;
        * `rounds` round trips of a distinct pattern per (sender, receiver, round) through
          strided boxes (the shape of a halo face), each preceded by a read of the
          receive boxes — so a receiver whose caches still hold the previous round's
          lines after the wait (a broken link 3 of ipc.hip's ordering chain), or a put
          whose stores are not visible when the flag is (link 1/2), shows up as a
          mismatch; the receiver checks every box on the device.
        Raises RuntimeError (on every rank) on any mismatch, wait timeout or missing peer
        access; returns {"pairs", "rounds", "cross_device"}."""
        comm, dev = self.comm, self.comm.device
        peers = [q for q in range(comm.size) if q != comm.rank]
        ids = comm.device_ids()
        mine = dev.index
        cross = sorted({ids[q] for q in peers} - {mine})
        noacc = [d for d in cross if not torch.cuda.can_device_access_peer(mine, d)]
        bad_access = comm.allreduce_max(float(len(noacc)))
        if bad_access:
            raise RuntimeError(f"ipc preflight: rank {comm.rank} (device {mine}) has no peer "
                               f"access to devices {noacc}")
        nk, nj, ni = box
        pitch = ni + 56  # strided rows, like a face of a padded field
        send = torch.zeros((len(peers), nk, nj, pitch), dtype=torch.float64, device=dev)
        recv = torch.zeros_like(send)
        msgs = [(p, send[i, :, :, :ni], recv[i, :, :, :ni]) for i, p in enumerate(peers)]
        base = torch.arange(nk * nj * ni, dtype=torch.float64, device=dev).view(nk, nj, ni)

        def pattern(src, dst, r):  # exact in fp64: distinct for every (src, dst, r, cell)
            return base + (src * 64 + dst) * 1e6 + r * 1e9 + 0.5

        stream = torch.cuda.Stream(device=dev)
        cur = torch.cuda.current_stream(dev)
        mism = []
        for r in range(rounds):
            for i, p in enumerate(peers):
                send[i, :, :, :ni].copy_(pattern(comm.rank, p, r))
            float(recv.sum())  # the stale boxes pass through this GPU's caches
            comm.barrier()
            ev = torch.cuda.Event()
            ev.record(cur)
            stream.wait_event(ev)
            self.exchange(msgs, stream)
            cur.wait_stream(stream)
            for i, p in enumerate(peers):
                if not torch.equal(recv[i, :, :, :ni], pattern(p, comm.rank, r)):
                    mism.append((p, r))
            # every rank knows after each round (a broken path costs one wait timeout,
            # not one per round); also: nobody starts the next round's puts before all
            # have compared
            if comm.allreduce_max(float(len(mism) + self.errors())) > 0:
                break
        torch.cuda.synchronize(dev)
        timeouts = self.errors()
        del send, recv, msgs
        self.reset()  # the peers' preflight boxes are freed: close their mappings
        bad = comm.allreduce_max(float(len(mism) + timeouts))
        if bad:
            raise RuntimeError(f"ipc preflight failed: rank {comm.rank}: mismatching "
                               f"(peer, round) {mism[:8]}, wait timeouts {timeouts}")
        return {"pairs": comm.size * (comm.size - 1), "rounds": rounds,
                "cross_device": comm.allreduce_max(float(len(cross))) > 0}

    def errors(self) -> int:
        n = ctypes.c_longlong(0)
        _lib.check(self.lib.advdiff_ipc_errors(self.ctx, ctypes.byref(n)), "advdiff_ipc_errors")
        return int(n.value)

    def close(self):
        if self.ctx:
            torch.cuda.synchronize(self.comm.device)
            self.comm.barrier()  # nobody unmaps while a peer may still put into it
            self.lib.advdiff_ipc_destroy(self.ctx)
            self.ctx = None


# ----------------------------------------------------------------------------------
# Striped slab exchange: a face message also travels over the node's idle links
# ----------------------------------------------------------------------------------
def stripe_plan(world: int, max_helpers: int, exclusive_links: bool = True) -> dict:
    """Relay helpers of every slab halo message {(src, dst): [helper, ...]}, the same on
    every rank.  A slab rank uses 2 of the 7 xGMI links of a fully connected 8-GPU node
    (its neighbours'); part of each face message instead goes src -> helper -> dst over
    two links no other route uses: (src, h) and (h, dst) must be neither a neighbour link
    (those carry the direct parts) nor a link of another route.  Every message gets the
    same number of helpers t (the exchange waits for its slowest message, so an extra
    helper for some messages only would buy nothing): the largest t <= max_helpers for
    which a depth-first search finds such an assignment (8 ranks: t = 1; 42 spare
    directed links, two per route).
    exclusive_links=False (tests: the mechanism on fewer ranks): any helper other than
    the pair itself, links shared."""
    msgs = [(r, r + 1) for r in range(world - 1)] + [(r + 1, r) for r in range(world - 1)]
    direct = {(a, b) for a, b in msgs}
    if not exclusive_links:
        # per phase, each directed link at most once (one message per peer, direction and
        # phase — what SlabHalo's phases need); greedy, helper counts may differ
        p1, p2 = set(direct), set()
        plan = {m: [] for m in msgs}
        for _ in range(max(0, max_helpers)):
            for s, d in msgs:
                for h in range(world):
                    if h in (s, d) or h in plan[(s, d)] or (s, h) in p1 or (h, d) in p2:
                        continue
                    p1.add((s, h))
                    p2.add((h, d))
                    plan[(s, d)].append(h)
                    break
        return plan
    def cands(s, d):  # farthest from the pair first: deterministic
        return sorted((h for h in range(world) if h not in (s, d)),
                      key=lambda h: (-min(abs(h - s), abs(h - d)), h))

    def solve(t):
        order = [m for _ in range(t) for m in msgs]  # round-robin slots
        helpers = {m: [] for m in msgs}
        used = set(direct)
        budget = [20000]  # search steps: give up (a smaller t) rather than search long

        def dfs(i):
            if i == len(order):
                return True
            budget[0] -= 1
            if budget[0] < 0:
                return False
            s, d = order[i]
            for h in cands(s, d):
                if h in helpers[(s, d)] or (s, h) in used or (h, d) in used:
                    continue
                used.update(((s, h), (h, d)))
                helpers[(s, d)].append(h)
                if dfs(i + 1):
                    return True
                helpers[(s, d)].pop()
                used.difference_update(((s, h), (h, d)))
            return False
        return helpers if dfs(0) else None

    for t in range(max(0, max_helpers), 0, -1):
        plan = solve(t)
        if plan is not None:
            return plan
    return {m: [] for m in msgs}


def stripe_rows(rows: int, k: int) -> list:
    """Row ranges of the k parts of a message: the direct part 2/(k+1) of the rows, the
    k-1 relayed parts (two hops each) 1/(k+1) each — every part then spends the same time
    on the links (a relayed part crosses two links one after the other)."""
    if k <= 1:
        return [(0, rows)]
    w = [2.0] + [1.0] * (k - 1)
    tot = sum(w)
    cuts, acc = [0], 0.0
    for x in w[:-1]:
        acc += x
        cuts.append(int(round(rows * acc / tot)))
    cuts.append(rows)
    return [(a, b) for a, b in zip(cuts[:-1], cuts[1:])]
