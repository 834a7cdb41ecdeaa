"""Striped slab exchange (parallel/ipc.py stripe_plan / stripe_rows, parallel/halo.py
SlabHalo._stripe_phases) on the CPU: the routing uses only idle links, one route per
link, the same helper count for every message; and the phases of ALL ranks, simulated
together, deliver every ghost row of every rank exactly once with matching shapes — the
geometry the ipc puts rely on (the device path itself: tests/test_ipc_gpu.py)."""
import pytest
import torch

from multigpu_advectiondiffusion_amd.parallel.decomposition import (SlabDecomposition,
                                                                    halo_link_bytes)
from multigpu_advectiondiffusion_amd.parallel.halo import SlabHalo
from multigpu_advectiondiffusion_amd.parallel.ipc import stripe_plan, stripe_rows


def test_plan_eight_ranks_uses_idle_links_once():
    plan = stripe_plan(8, 3)
    msgs = [(r, r + 1) for r in range(7)] + [(r + 1, r) for r in range(7)]
    assert sorted(plan) == sorted(msgs)
    counts = {len(h) for h in plan.values()}
    assert counts == {1}  # 42 spare directed links, 2 per route: one helper each
    used = set(msgs)
    for (s, d), hs in plan.items():
        for h in hs:
            assert h not in (s, d)
            for link in ((s, h), (h, d)):
                assert link not in used, link
                used.add(link)
    assert stripe_plan(8, 3) == plan  # deterministic: every rank computes the same


@pytest.mark.parametrize("world", [2, 3, 4, 6])
def test_plan_small_worlds_have_no_idle_links(world):
    assert all(not h for h in stripe_plan(world, 2).values())


def test_rows_split_weights():
    assert stripe_rows(1024, 1) == [(0, 1024)]
    parts = stripe_rows(1024, 2)
    assert parts == [(0, 683), (683, 1024)]
    assert stripe_rows(10, 4) == [(0, 4), (4, 6), (6, 8), (8, 10)]


class _C:
    def __init__(self, rank, size):
        self.rank, self.size, self.transport = rank, size, "ipc"


@pytest.mark.parametrize("world,helpers,shared", [(8, 2, False), (3, 1, True), (4, 2, True),
                                                  (5, 1, True), (5, 3, True)])
def test_phases_deliver_every_ghost_row_once(world, helpers, shared, monkeypatch):
    if shared:
        monkeypatch.setenv("ADVDIFF_STRIPE_SHARED", "1")
    nz, ny, sx, G = 6 * world, 9, 5, 3
    halos, fields = [], []
    for r in range(world):
        d = SlabDecomposition(nz, world, r, G)
        h = SlabHalo(_C(r, world), d, transport="ipc", stripe=helpers)
        assert h.striped
        for (src, dst), hs in h._plan.items():  # one message per peer, direction, phase
            assert len(set(hs)) == len(hs)
        halos.append(h)
        # owned cells carry their global (z, y) identity; ghosts start at -1
        f = torch.full((d.alloc, ny, sx), -1.0, dtype=torch.float64)
        for lz in range(d.ghost, d.ghost + d.count):
            f[lz] = (d.start + lz - d.ghost) * 1000.0 + torch.arange(ny, dtype=torch.float64)[:, None]
        fields.append(f)
    for parity in (0, 1):
        phases = [h._stripe_phases(f, parity) for h, f in zip(halos, fields)]
        for ph in (0, 1):  # simulate the puts of every phase, in order
            for r in range(world):
                for peer, (send, _) in phases[r][ph].items():
                    if send is None:
                        continue
                    recv = phases[peer][ph][r][1]
                    assert recv is not None and recv.shape == send.shape, (r, peer, ph)
                    recv.copy_(send)
            for r in range(world):  # one-way pairs: a receiver always has a sender
                for peer, (_, recv) in phases[r][ph].items():
                    if recv is not None:
                        assert phases[peer][ph][r][0] is not None
        for r, (h, f) in enumerate(zip(halos, fields)):
            d = h.d
            for lo, hi, g0 in ((0, d.ghost, d.start - d.ghost),
                               (d.ghost + d.count, d.alloc, d.start + d.count)):
                if (lo == 0 and d.lower is None) or (lo > 0 and d.upper is None):
                    continue
                for lz in range(lo, hi):
                    want = (g0 + lz - lo) * 1000.0 + torch.arange(ny, dtype=torch.float64)[:, None]
                    assert torch.equal(f[lz], want.expand(ny, sx)), (r, lz)
            for lz in list(range(0, d.ghost)) + list(range(d.ghost + d.count, d.alloc)):
                f[lz] = -1.0  # next parity starts from stale ghosts again


def test_link_model_striped():
    base = halo_link_bytes((1024, 1024, 1024), (8, 1, 1), 6, 8, True)
    assert halo_link_bytes((1024, 1024, 1024), (8, 1, 1), 6, 8, True, stripe_parts=2) == \
        pytest.approx(base * 2 / 3)


def _mock_striped(comm, world, exchanges):
    """Every rank runs the striped phases through IpcPeers.route with the native calls
    replaced by recorders: returns the (signal / wait, channel, peer) counts."""
    import collections
    import os
    os.environ["ADVDIFF_STRIPE_SHARED"] = "1"
    from multigpu_advectiondiffusion_amd.parallel import ipc as ipcmod
    log = collections.Counter()

    class FakeLib:
        def advdiff_ipc_describe(self, ctx, ptr, out):
            return 0

        def advdiff_ipc_map(self, ctx, a, p):
            return 0

        def advdiff_ipc_put(self, *a):
            return 0

        def advdiff_ipc_signal_ch(self, ctx, ch, arr, n, sp):
            for i in range(n):
                log[("sig", ch, arr[i])] += 1
            return 0

        def advdiff_ipc_wait_ch(self, ctx, ch, arr, n, sp):
            for i in range(n):
                log[("wait", ch, arr[i])] += 1
            return 0
    ip = object.__new__(ipcmod.IpcPeers)
    ip.comm, ip.lib, ip.ctx, ip._dest, ip._calls, ip.epoch = comm, FakeLib(), None, {}, {}, 0
    ipcmod._lib.check = lambda code, what: None
    ipcmod._dtype_code = lambda t: 1
    comm._ipc = ip

    class S:
        cuda_stream = None
    d = SlabDecomposition(6 * world, world, comm.rank, 3)
    h = SlabHalo(comm, d, transport="ipc", stripe=2)
    f = torch.zeros((d.alloc, 9, 8), dtype=torch.float64)
    g = torch.zeros_like(f)
    for e in range(exchanges):  # two fields in an irregular order, both parities
        fld = f if e % 3 else g
        par = h.parity
        p1, p2 = h._stripe_phases(fld, par)
        h.parity ^= 1
        ip.route(p1, S, 1, h._tag(fld, par))
        ip.route(p2, S, 2, h._tag(fld, par))
    comm._ipc = None
    return dict(log)


@pytest.mark.parametrize("world", [3, 5, 8])
def test_striped_handshakes_and_counts_match(world):
    """All ranks' striped exchanges: every pair agrees on each handshake (no rank waits in
    a swap its peer skips — the one-way relay hops key their cache by a tag both sides
    derive alike) and every signal on a channel meets exactly one wait."""
    from multigpu_advectiondiffusion_amd.launch import spawn_local
    logs = spawn_local(world, _mock_striped, world, 12, device="cpu", backend="gloo",
                       timeout=120)
    n = 0
    for r in range(world):
        for (kind, ch, p), k in logs[r].items():
            if kind == "sig":
                assert logs[p].get(("wait", ch, r), 0) == k, (r, p, ch)
                n += k
        for (kind, ch, p), k in logs[r].items():
            if kind == "wait":
                assert logs[p].get(("sig", ch, r), 0) == k, (r, p, ch)
    assert n > 0
