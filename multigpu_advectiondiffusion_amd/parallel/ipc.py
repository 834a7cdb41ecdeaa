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

# IpcAddr (80 B) | rsy, rsz (i64) | ni, nj, nk, dtype (i32) | call (u64)
_ANN = struct.Struct("<80sqqiiiiQ")


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
        """Peer receive (pointer, sy, sz) of every message; handshake on first use."""
        out, miss = [None] * len(msgs), []
        for q, (peer, send, recv) in enumerate(msgs):
            self._calls[peer] = self._calls.get(peer, 0) + 1
            key = (peer, send.data_ptr(), recv.data_ptr(), tuple(send.shape))
            d = self._dest.get(key)
            if d is None:
                miss.append(q)
            else:
                out[q] = d
        if not miss:
            return out
        anns, peers = [], []
        for q in miss:
            peer, send, recv = msgs[q]
            a = _lib.IpcAddr()
            _lib.check(self.lib.advdiff_ipc_describe(self.ctx, recv.data_ptr(), ctypes.byref(a)),
                       "advdiff_ipc_describe")
            ni, nj, nk, sy, sz = _box_geom(recv)
            anns.append(_ANN.pack(bytes(a), sy, sz, ni, nj, nk, _dtype_code(recv),
                                  self._calls[peer]))
            peers.append(peer)
        theirs = self._swap(peers, anns)
        for q, raw in zip(miss, theirs):
            peer, send, recv = msgs[q]
            addr, rsy, rsz, ni, nj, nk, dt, call = _ANN.unpack(raw)
            gi, gj, gk, _, _ = _box_geom(send)
            if (ni, nj, nk, dt) != (gi, gj, gk, _dtype_code(send)) or call != self._calls[peer]:
                raise RuntimeError(f"ipc: rank {self.comm.rank} and peer {peer} disagree on a "
                                   f"halo message ({(gi, gj, gk)} vs {(ni, nj, nk)})")
            a = _lib.IpcAddr.from_buffer_copy(addr)
            ptr = ctypes.c_void_p()
            _lib.check(self.lib.advdiff_ipc_map(self.ctx, ctypes.byref(a), ctypes.byref(ptr)),
                       "advdiff_ipc_map")
            d = (ptr.value, rsy, rsz)
            self._dest[(peer, send.data_ptr(), recv.data_ptr(), tuple(send.shape))] = d
            out[q] = d
        return out

    def exchange(self, msgs, stream) -> None:
        """Enqueue on `stream`: put every send box into its peer's matching receive box,
        signal the peers, wait for their puts into ours.  msgs = [(peer, send_view,
        recv_view)] with distinct peers."""
        if not msgs:
            return
        peers = [m[0] for m in msgs]
        if len(set(peers)) != len(peers):
            raise ValueError("ipc: one message per peer and exchange")
        dests = self._resolve(msgs)
        sp = stream.cuda_stream
        for (peer, send, _), (dptr, dsy, dsz) in zip(msgs, dests):
            ni, nj, nk, ssy, ssz = _box_geom(send)
            _lib.check(self.lib.advdiff_ipc_put(_dtype_code(send), dptr, dsy, dsz,
                                                send.data_ptr(), ssy, ssz, ni, nj, nk, sp),
                       "ipc put")
        arr = (ctypes.c_int * len(peers))(*peers)
        _lib.check(self.lib.advdiff_ipc_signal(self.ctx, arr, len(peers), sp), "advdiff_ipc_signal")
        _lib.check(self.lib.advdiff_ipc_wait(self.ctx, arr, len(peers), sp), "advdiff_ipc_wait")

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
            comm.barrier()  # nobody starts the next round's puts before all have compared
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
